"""VideoPainterID LoRA adapters on the attention projections, applied UNFUSED as PEFT does.

The reference loads the ID-resample adapter unfused through PEFT (`pipe.load_lora_weights(path,
weight_name="pytorch_lora_weights.safetensors", adapter_name=..., target_modules=["transformer"])`,
infer/inpaint.py:310-315, `fuse_lora` commented out at :316; `CogVideoXLoraLoaderMixin.load_lora_into_transformer`,
diffusers/loaders/lora_pipeline.py:2632-2705).  Its forward on to_q / to_k / to_v / to_out.0 (the training script's
`LoraConfig(target_modules=["to_q", "to_k", "to_v", "to_out.0"])`, train/train_cogvideox_inpainting_i2v_video_resample
.py:1520-1525) is

    y = x W0^T + b + s (x A^T) B^T,    s = lora_alpha / r * lora_scale * adapter weight

where the loader passes no network alphas, so `get_peft_kwargs` sets lora_alpha = r (utils/peft_utils.py:153): s =
lora_scale (attention_kwargs["scale"], default 1.0, cogvideox_transformer_3d.py:490-499) for PEFT files; kohya files
(`lora_down` / `lora_up` + `.alpha`) keep alpha / r.

Here every adapted projection runs ONE GEMM on K-augmented operands (`AugmentedProjection`):
    x_aug = [x | T],   T = x [A_0; A_1; ...]^T   (one small GEMM; rank block i belongs to projection i),
    W_aug_i = [W0_i | s_i B_i]                  (bf16, per projection, cached on the factors' versions and s),
and the GEMM's per-segment A tail (include/vp_hip.h vp_gemm_desc.a_tail_k / a_tail_off) lets segment i of the fused
QKV read only its own rank block: the extra work is PEFT's (2 r (K + N) per row and projection), the delta enters
in the fp32 accumulator before the fused epilogues (qk-norm + RoPE, the gated residual), and W0 is never modified —
the reference's arithmetic up to PEFT's extra bf16 roundings of x A^T and of the delta.

Loaded adapters (`attach_lora_`, `load_lora_weights`) and trainable ones (`add_trainable_adapter_`, PEFT's
`add_adapter`) take the same path.  `fuse_lora` is the explicit fold (W = W0 + s B A in fp32, rounded once; the base
weights are kept so `unfuse_lora` and a re-fold at another scale are exact).  An adapter on a Linear outside the
attention projections (which only the GEMMs of to_q/k/v/out.0 augment) is folded at load time, with its base kept, so
the per-call scale stays exact there too; a TRAINABLE adapter there raises (it would get no gradient).

Parity: PEFT is not installed here; `tests/test_lora_cpu.py` checks the augmented operands against the unmerged
LoRA formula, and the GPU tests run the model with an unfused adapter against the oracle's restatement of PEFT's
unmerged forward (`oracle/cogvideox_oracle.py` lora hooks) — "parity unpinned" against PEFT itself.
"""
from __future__ import annotations

import math
import os
import re
import weakref
from typing import Dict, List, Optional, Tuple

import torch

TARGETS = ("to_q", "to_k", "to_v", "to_out.0")
_PEFT = re.compile(r"^(?:(?P<prefix>transformer)\.)?(?P<mod>.+)\.lora_(?P<ab>[AB])(?:\.[^.]+)?\.weight$")
_KOHYA = re.compile(r"^(?:(?P<prefix>transformer)\.)?(?P<mod>.+)\.lora_(?P<ab>down|up)\.weight$")
# the Linears the augmented GEMMs cover: the attention projections of every block (transformer and branch)
_COVERED = re.compile(r"(^|\.)attn1\.(to_q|to_k|to_v|to_out\.0)$")
AUG_ALIGN = 64  # the per-projection tail width is padded to whole 64-wide K-tiles of the GEMM (zero columns / rows)
_AUG_BUFFERS: Dict[int, "weakref.ref"] = {}  # id -> weakref of the live x_aug buffers from augmented_rows()


def covered(module_name: str) -> bool:
    return _COVERED.search(module_name) is not None


def load_lora_state_dict(path: str, weight_name: str = "pytorch_lora_weights.safetensors") -> Dict[str, torch.Tensor]:
    """The adapter file (safetensors only: nothing in it is executed)."""
    from safetensors.torch import load_file
    f = os.path.join(path, weight_name) if os.path.isdir(path) else path
    return load_file(f)


def lora_pairs(sd: Dict[str, torch.Tensor]) -> Dict[str, dict]:
    """{module path: {"A": [r, in], "B": [out, r], "alpha": float or None}} from a PEFT or kohya state dict."""
    pairs: Dict[str, dict] = {}
    for k, v in sd.items():
        m = _PEFT.match(k) or _KOHYA.match(k)
        if m is None:
            if k.endswith(".alpha"):
                mod = k[:-len(".alpha")]
                mod = mod[len("transformer."):] if mod.startswith("transformer.") else mod
                pairs.setdefault(mod, {})["alpha"] = float(v)
            continue
        ab = {"A": "A", "down": "A", "B": "B", "up": "B"}[m.group("ab")]
        pairs.setdefault(m.group("mod"), {})[ab] = v
    for mod, p in pairs.items():
        if "A" not in p or "B" not in p:
            raise ValueError(f"LoRA module {mod} has only {sorted(k for k in p if k in 'AB')}")
        if p["B"].shape[1] != p["A"].shape[0]:
            raise ValueError(f"LoRA module {mod}: B {tuple(p['B'].shape)} and A {tuple(p['A'].shape)} disagree")
    return pairs


def _scale(p: dict, scale: float, weight: float) -> float:
    r = p["A"].shape[0]
    return scale * weight * (p["alpha"] / r if p.get("alpha") is not None else 1.0)


@torch.no_grad()
def fold_lora_(model: torch.nn.Module, sd: Dict[str, torch.Tensor], lora_scale: float = 1.0,
               strict: bool = True) -> int:
    """W += s * B @ A for every adapted Linear of `model` (in place, fp32 then one bf16 rounding); returns the number
    of folded layers.  The stateless fold (tests and the fused path use it); `attach_lora_` is the stateful loader."""
    mods = dict(model.named_modules())
    n = 0
    for mod, p in lora_pairs(sd).items():
        lin = mods.get(mod)
        if lin is None or not hasattr(lin, "weight"):
            if strict:
                raise KeyError(f"LoRA targets {mod}, which the model does not have")
            continue
        W = lin.weight
        if tuple(W.shape) != (p["B"].shape[0], p["A"].shape[1]):
            raise ValueError(f"LoRA {mod}: B@A is {(p['B'].shape[0], p['A'].shape[1])}, weight is {tuple(W.shape)}")
        delta = p["B"].to(W.device, torch.float32) @ p["A"].to(W.device, torch.float32)
        W.copy_((W.float() + _scale(p, lora_scale, 1.0) * delta).to(W.dtype))
        n += 1
    return n


def load_lora_into_transformer(transformer: torch.nn.Module, path: str,
                               weight_name: str = "pytorch_lora_weights.safetensors", lora_scale: float = 1.0,
                               strict: bool = True) -> int:
    """The adapter file folded once into the weights (the stateless form of `fuse_lora`)."""
    sd = load_lora_state_dict(path, weight_name)
    if any(k.startswith("transformer.") for k in sd):  # the pipeline-level file (lora_pipeline.py:2653-2656)
        sd = {k: v for k, v in sd.items() if k.startswith("transformer.")}
    return fold_lora_(transformer, sd, lora_scale, strict)


def unfold_lora_(model: torch.nn.Module, sd: Dict[str, torch.Tensor], lora_scale: float = 1.0) -> int:
    """Remove a folded adapter (W -= s B A; exact only up to the weight dtype's rounding)."""
    return fold_lora_(model, sd, -lora_scale)


class LoraState:
    """The adapters of one model (kept in its __dict__: the state dict stays the reference's)."""

    def __init__(self):
        self.adapters: list = []      # [(name, {module: {"A", "B", "alpha"}})]
        self.scale: float = 1.0       # the per-call scale (attention_kwargs["scale"])
        self.weights: Dict[str, float] = {}   # set_adapters() weights per adapter (1.0 when loaded, 0 = inactive)
        self.trainable: set = set()   # adapters added by add_trainable_adapter_ (factors are Parameters)
        self.fused = False            # fuse_lora(): loaded adapters folded into W0, per-call scale no longer applied
        self.fused_scale = 1.0
        self.base: Dict[str, torch.Tensor] = {}   # W0 of every module whose weight holds a fold (fused / uncovered)


def lora_state(model: torch.nn.Module) -> Optional[LoraState]:
    return model.__dict__.get("_vp_lora")


def _state(model) -> LoraState:
    st = lora_state(model)
    if st is None:
        st = model.__dict__["_vp_lora"] = LoraState()
    return st


def _folded_here(st: LoraState, mod: str) -> bool:
    """Do the loaded adapters of this module live in its weight (fused, or a module the GEMMs do not augment)?"""
    return (st.fused and covered(mod)) or not covered(mod)


@torch.no_grad()
def _refold_module(st: LoraState, mod: str, W: torch.Tensor) -> None:
    """W = W0 + sum over active LOADED adapters of s B A (fp32, one rounding): the fold's exact expression."""
    acc = st.base[mod].to(W.device, torch.float32)
    sc = st.fused_scale if (st.fused and covered(mod)) else st.scale
    for name, pairs in st.adapters:
        p = pairs.get(mod)
        w = st.weights.get(name, 1.0)
        if p is None or w == 0.0 or name in st.trainable:
            continue
        acc = acc + _scale(p, sc, w) * (p["B"].to(W.device, torch.float32) @ p["A"].to(W.device, torch.float32))
    W.copy_(acc.to(W.dtype))


def _requant_fp8(model) -> None:
    for blk in getattr(model, "transformer_blocks", []):
        if getattr(blk, "qkv_mx", None) is not None:
            blk.enable_fp8_qkv(True)
        if getattr(blk, "out_mx", None) is not None:
            blk.enable_fp8_out(True)


@torch.no_grad()
def refold_lora_(model: torch.nn.Module, scale: Optional[float] = None) -> int:
    """Set the per-call scale and rebuild every weight that holds a fold from its kept base (exact).  Unfused
    projections need nothing: their augmented operands follow the scale.  Re-quantises an enabled fp8 QKV."""
    st = lora_state(model)
    if st is None:
        return 0
    if scale is not None:
        st.scale = float(scale)
    mods = dict(model.named_modules())
    for mod in st.base:
        _refold_module(st, mod, mods[mod].weight)
    if st.base:
        _requant_fp8(model)
    return len(st.base)


def _mark(lin, st: LoraState, mod: str) -> None:
    lin.__dict__["_vp_lora_mod"] = (st, mod)


def _check_fp8_free(model, mods_of_blocks) -> None:
    """Unfused adapters cannot ride the MX-FP8 QKV / output-projection GEMMs: raise BEFORE anything is attached
    (fuse_lora folds them)."""
    mods = dict(model.named_modules())
    for name, _ in mods_of_blocks:
        blk = name.rsplit(".attn1.", 1)[0]
        b = mods.get(blk)
        if b is not None and getattr(b, "qkv_mx", None) is not None and re.search(r"\.to_[qkv]$", name):
            raise NotImplementedError(f"{name}: the fp8 QKV projection is enabled; unfused LoRA runs on the bf16 "
                                      "GEMM (disable fp8 QKV, or fuse_lora())")
        if b is not None and getattr(b, "out_mx", None) is not None and re.search(r"\.to_out\.0$", name):
            raise NotImplementedError(f"{name}: the fp8 output projection is enabled; unfused LoRA runs on the bf16 "
                                      "GEMM (disable it, or fuse_lora())")


@torch.no_grad()
def attach_lora_(model: torch.nn.Module, sd: Dict[str, torch.Tensor], lora_scale: Optional[float] = None,
                 adapter_name: Optional[str] = None, strict: bool = True) -> int:
    """Register a loaded adapter (PEFT's load_lora_weights): unfused on the attention projections, folded (base kept)
    on any other Linear.  `lora_scale` sets the per-call scale (None keeps it)."""
    mods = dict(model.named_modules())
    pairs = {}
    for mod, p in lora_pairs(sd).items():
        lin = mods.get(mod)
        if lin is None or not hasattr(lin, "weight"):
            if strict:
                raise KeyError(f"LoRA targets {mod}, which the model does not have")
            continue
        W = lin.weight
        if tuple(W.shape) != (p["B"].shape[0], p["A"].shape[1]):
            raise ValueError(f"LoRA {mod}: B@A is {(p['B'].shape[0], p['A'].shape[1])}, weight is {tuple(W.shape)}")
        pairs[mod] = {"A": p["A"].to(W.device, W.dtype), "B": p["B"].to(W.device, W.dtype), "alpha": p.get("alpha")}
    st = _state(model)
    name = adapter_name or f"default_{len(st.adapters)}"
    if any(n == name for n, _ in st.adapters):
        raise ValueError(f"adapter {name!r} is already loaded")
    if not st.fused:
        _check_fp8_free(model, [(m, mods[m]) for m in pairs if covered(m)])
    for mod in pairs:
        if _folded_here(st, mod) and mod not in st.base:
            st.base[mod] = mods[mod].weight.detach().clone()
        if covered(mod):
            _mark(mods[mod], st, mod)
    st.adapters.append((name, pairs))
    st.weights[name] = 1.0
    refold_lora_(model, lora_scale)
    return len(pairs)


@torch.no_grad()
def set_adapter_weights_(model: torch.nn.Module, names, weights=None) -> None:
    """PEFT's `set_adapters(names, weights)`: the listed adapters active with their weights, the others off."""
    st = lora_state(model)
    if st is None:
        raise ValueError("no LoRA adapter is loaded")
    names = [names] if isinstance(names, str) else list(names)
    known = [n for n, _ in st.adapters]
    for n in names:
        if n not in known:
            raise ValueError(f"adapter {n!r} is not loaded (loaded: {known})")
    ws = [1.0] * len(names) if weights is None else (
        [float(weights)] * len(names) if not isinstance(weights, (list, tuple)) else [float(w) for w in weights])
    if len(ws) != len(names):
        raise ValueError("one weight per adapter name")
    st.weights = {n: 0.0 for n in known}
    st.weights.update(dict(zip(names, ws)))
    refold_lora_(model)


@torch.no_grad()
def fuse_lora_(model: torch.nn.Module, lora_scale: float = 1.0) -> None:
    """The pipeline's `fuse_lora(lora_scale=...)`: the loaded adapters of the attention projections folded into
    W (base kept), at `lora_scale` x their adapter weights; later per-call scales no longer reach them (PEFT's merged
    layers).  Trainable adapters stay unfused."""
    st = lora_state(model)
    if st is None:
        return
    mods = dict(model.named_modules())
    for _, pairs in st.adapters:
        for mod in pairs:
            if covered(mod) and mod not in st.base:
                st.base[mod] = mods[mod].weight.detach().clone()
    st.fused, st.fused_scale = True, float(lora_scale)
    refold_lora_(model)


@torch.no_grad()
def unfuse_lora_(model: torch.nn.Module) -> None:
    """Undo `fuse_lora_`: the attention projections back to W0 (exact: the kept base) and unfused again."""
    st = lora_state(model)
    if st is None or not st.fused:
        return
    mods = dict(model.named_modules())
    # (unfused adapters cannot ride an enabled fp8 QKV — raise before anything changes, not half-way)
    _check_fp8_free(model, [(m, mods[m]) for m in st.base if covered(m)])
    for mod in [m for m in st.base if covered(m)]:
        mods[mod].weight.copy_(st.base.pop(mod))
    st.fused = False
    _requant_fp8(model)


class LoraFactor(torch.nn.Module):
    """One trainable LoRA factor as PEFT names it: `<module>.lora_A.weight` [r, in] / `<module>.lora_B.weight`
    [out, r] (the keys `get_peft_model_state_dict` saves and `load_lora_weights` reads)."""

    def __init__(self, rows: int, cols: int, device=None, dtype=None):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.empty(rows, cols, device=device, dtype=dtype))


@torch.no_grad()
def add_trainable_adapter_(model: torch.nn.Module, r: int, lora_alpha: float, target_modules=TARGETS,
                           adapter_name: str = "default", init_lora_weights: bool = True,
                           dtype: Optional[torch.dtype] = None) -> int:
    """PEFT's `model.add_adapter(LoraConfig(r, lora_alpha, init_lora_weights, target_modules))` (the resample
    training script, train/train_cogvideox_inpainting_i2v_video_resample.py:1520-1526): a trainable (lora_A, lora_B)
    pair on every Linear whose name ends in one of `target_modules`, PEFT's default init (A kaiming-uniform
    a = sqrt(5), B = 0, so the adapted model starts equal to the base), scaling lora_alpha / r.  The factors are
    registered as `<module>.lora_A.weight` / `.lora_B.weight` parameters; every other parameter of the model is
    frozen, as PEFT does.  The adapter runs UNFUSED (AugmentedProjection), so only the attention projections can
    carry it: any other matched module raises before anything is changed."""
    if r <= 0:
        raise ValueError("LoRA rank must be positive")
    targets = tuple(target_modules)
    st = _state(model)
    if any(n == adapter_name for n, _ in st.adapters):
        raise ValueError(f"adapter {adapter_name!r} is already loaded")
    matched = [(name, lin) for name, lin in model.named_modules()
               if any(name == t or name.endswith("." + t) for t in targets) and hasattr(lin, "weight")]
    if not matched:
        raise ValueError(f"no module matches target_modules {targets}")
    bad = [name for name, _ in matched if not covered(name)]
    if bad:
        raise ValueError(f"trainable LoRA runs unfused on the attention projections (to_q / to_k / to_v / to_out.0) "
                         f"only; {bad[:4]} would get no forward delta and no gradient")
    for name, lin in matched:
        if hasattr(lin, "lora_A"):
            raise ValueError(f"{name} already carries a trainable adapter (one trainable adapter per model)")
    _check_fp8_free(model, matched)
    model.requires_grad_(False)
    pairs = {}
    for name, lin in matched:
        W = lin.weight
        out_f, in_f = W.shape
        dt = dtype or W.dtype
        lin.lora_A = LoraFactor(r, in_f, W.device, dt)
        lin.lora_B = LoraFactor(out_f, r, W.device, dt)
        if init_lora_weights:
            a = torch.empty(r, in_f, device=W.device, dtype=torch.float32)
            torch.nn.init.kaiming_uniform_(a, a=math.sqrt(5))
            lin.lora_A.weight.copy_(a)
            lin.lora_B.weight.zero_()
        lin.lora_A.weight.requires_grad_(True)
        lin.lora_B.weight.requires_grad_(True)
        pairs[name] = {"A": lin.lora_A.weight, "B": lin.lora_B.weight, "alpha": float(lora_alpha)}
        _mark(lin, st, name)
    st.adapters.append((adapter_name, pairs))
    st.weights[adapter_name] = 1.0
    st.trainable.add(adapter_name)
    return len(pairs)


def trainable_lora_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """`get_peft_model_state_dict(transformer)`: the trainable factors under PEFT's saved names."""
    return {k: v.detach() for k, v in model.state_dict().items() if ".lora_A.weight" in k or ".lora_B.weight" in k}


# ------------------------------------------------------------------------------------------------------------------
# Unfused adapters: K-augmented projection operands
# ------------------------------------------------------------------------------------------------------------------

def module_pairs(lin) -> List[Tuple[torch.Tensor, torch.Tensor, float]]:
    """[(A [r, in], B [out, r], s)] of the adapters this Linear applies unfused (trainable ones: the Parameters
    themselves), s = call scale x adapter weight x alpha / r (PEFT's scaling)."""
    t = lin.__dict__.get("_vp_lora_mod")
    if t is None:
        return []
    st, mod = t
    out = []
    for name, pairs in st.adapters:
        p = pairs.get(mod)
        w = st.weights.get(name, 1.0)
        if p is None or w == 0.0:
            continue
        if name not in st.trainable and _folded_here(st, mod):
            continue
        out.append((p["A"], p["B"], _scale(p, st.scale, w)))
    return out


def trainable_pair(lin):
    """(A, B, s) of the trainable adapter on the Linear `lin`, or None."""
    for A, B, s in module_pairs(lin):
        if isinstance(A, torch.nn.Parameter):
            return A, B, s
    return None


class AugmentedProjection:
    """One GEMM over several projections (the fused QKV, the prev-clip K/V, to_out) whose Linears carry unfused
    adapters: y_i = x W0_i^T + b_i + sum_j s_ij (x A_ij^T) B_ij^T as
        x_aug = [x | T],  T = x [A_0; A_1; ...]^T   (bf16; projection i's rank block at columns K + i r),
        W_aug_i = [W0_i | s_i0 B_i0 | s_i1 B_i1 | 0]  (bf16 [out_i, K + r], r = the largest rank sum, 64-padded),
    with the GEMM's per-segment A tail (a_tail_k = K, a_tail_off[i] = i r) so segment i reads only its own block.
    W_aug_i depends on its own Linear only (cached per Linear on the factors' versions, s and r), so the fused QKV
    and the prev-clip K/V share the cache.  Projections narrower than a 256-column GEMM tile (tiny test models,
    where a tile would straddle two segments) take the block-diagonal form instead: W_aug_i = [W0_i | 0 .. s B_i ..
    0] over the whole T, no A tail (`full`)."""

    def __init__(self, lins):
        self.lins = list(lins)
        self.pairs = [module_pairs(l) for l in self.lins]
        self.ranks = [sum(A.shape[0] for A, _, _ in ps) for ps in self.pairs]
        self.r = (max(self.ranks) + AUG_ALIGN - 1) // AUG_ALIGN * AUG_ALIGN
        self.R = self.r * len(self.lins)
        self.K = self.lins[0].weight.shape[1]
        # the tail form needs whole 256-column tiles per segment and >= 8 K-tiles (the GEMM's default loop); one
        # projection needs no tail at all (its rank block starts right after x)
        self.full = len(self.lins) > 1 and (any(l.weight.shape[0] % 256 for l in self.lins) or self.K + self.r < 512)
        self.tail = None if self.full or len(self.lins) == 1 else (self.K, [i * self.r for i in range(len(self.lins))])

    def block_col(self, i: int) -> int:
        """First column of projection i's rank block in W_aug_i."""
        return self.K + (i * self.r if self.full else 0)

    @staticmethod
    def of(lins):
        """The augmentation of these projections, or None when none carries an unfused adapter."""
        if not any(module_pairs(l) for l in lins):
            return None
        return AugmentedProjection(lins)

    @staticmethod
    def _pkey(ps):
        return tuple((A._version, B._version, A.data_ptr(), B.data_ptr(), s) for A, B, s in ps)

    def _key(self):
        return tuple(self._pkey(ps) for ps in self.pairs) + tuple((l.weight._version, l.weight.data_ptr())
                                                                  for l in self.lins) + (self.r, self.full)

    def a_cat(self) -> torch.Tensor:
        """[R, K] bf16: projection i's A factors stacked in rows i r .. (zero rows for the padding)."""
        owner = self.lins[0]
        key = ("A", tuple(id(l) for l in self.lins)) + self._key()
        c = owner.__dict__.get("_vp_aug_A")
        if c is None or c[0] != key:
            W = self.lins[0].weight
            a = torch.zeros(self.R, self.K, device=W.device, dtype=torch.bfloat16)
            for i, ps in enumerate(self.pairs):
                o = i * self.r
                for A, _, _ in ps:
                    a[o:o + A.shape[0]].copy_(A.detach())
                    o += A.shape[0]
            c = (key, a)
            owner.__dict__["_vp_aug_A"] = c
        return c[1]

    def a_cat_t(self) -> torch.Tensor:
        """[K, R] bf16 = a_cat()^T (the dgrad operand of T = x A_cat^T)."""
        from . import kernels as K
        owner = self.lins[0]
        key = ("At", tuple(id(l) for l in self.lins)) + self._key()
        c = owner.__dict__.get("_vp_aug_At")
        if c is None or c[0] != key:
            c = (key, K.transpose(self.a_cat()))
            owner.__dict__["_vp_aug_At"] = c
        return c[1]

    def weights(self):
        """[W_aug_i] bf16 [out_i, K + r] (one per Linear, cached on the Linear; [out_i, K + R] when `full`)."""
        out = []
        for i, (l, ps) in enumerate(zip(self.lins, self.pairs)):
            k = (self._pkey(ps), l.weight._version, l.weight.data_ptr(), self.r, self.full,
                 self.block_col(i) if self.full else 0, self.R if self.full else 0)
            c = l.__dict__.get("_vp_aug_W")
            if c is None or c[0] != k:
                W = l.weight.detach()
                w = torch.zeros(W.shape[0], self.K + (self.R if self.full else self.r), device=W.device,
                                dtype=torch.bfloat16)
                w[:, :self.K].copy_(W)
                o = self.block_col(i)
                for A, B, s in ps:
                    w[:, o:o + A.shape[0]].copy_(B.detach().float() * s)
                    o += A.shape[0]
                c = (k, w)
                l.__dict__["_vp_aug_W"] = c
            out.append(c[1])
        return out

    def input(self, x2d: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x_aug [M, K + R] = [x | x A_cat^T] (one GEMM for T).  `out`: a buffer whose first K columns already
        hold x (the producer wrote them in place: no copy); x2d itself when it is the first K columns of a buffer
        from augmented_rows() for these projections."""
        from . import kernels as K
        M = x2d.shape[0]
        if out is None:
            out = _augmented_base(x2d, M, self.K + self.R)
        if out is None:
            out = torch.empty(M, self.K + self.R, device=x2d.device, dtype=torch.bfloat16)
            out[:, :self.K].copy_(x2d)
        K.gemm(out[:, :self.K], [self.a_cat()], [None], out[:, self.K:])
        return out

    def gemm(self, x_aug: torch.Tensor, biases, out2d: torch.Tensor, **kw) -> torch.Tensor:
        """The projections' GEMM on the augmented operands (any epilogue of the bf16 GEMM's tail form)."""
        from . import kernels as K
        if self.tail is None:  # block-diagonal form, or one projection: x_aug's first K + width columns
            return K.gemm(x_aug, self.weights(), biases, out2d, **kw)
        return K.gemm(x_aug, self.weights(), biases, out2d, a_tail=self.tail, **kw)


def _augmented_base(x2d: torch.Tensor, M: int, width: int) -> Optional[torch.Tensor]:
    """The augmented_rows() buffer whose first columns x2d is, when it is one of width `width`."""
    base = x2d._base
    ref = _AUG_BUFFERS.get(id(base)) if base is not None else None
    if (ref is None or ref() is not base or tuple(base.shape) != (M, width)
            or x2d.data_ptr() != base.data_ptr() or x2d.stride() != (width, 1)):
        return None
    return base


def augmented_rows(lins, B: int, Ntok: int, K: int, device) -> torch.Tensor:
    """A bf16 [B, Ntok, K] tensor for the input of the projections `lins`: when they carry unfused adapters, the
    first K columns of a fresh x_aug buffer [B*Ntok, K + R] (the producer — AdaLN, attention — writes x in place and
    AugmentedProjection.input only adds T: no copy of x), else a plain tensor."""
    aug = AugmentedProjection.of(lins)
    if aug is None or aug.K != K:
        return torch.empty(B, Ntok, K, device=device, dtype=torch.bfloat16)
    buf = torch.empty(B * Ntok, K + aug.R, device=device, dtype=torch.bfloat16)
    key = id(buf)
    _AUG_BUFFERS[key] = weakref.ref(buf, lambda _r, k=key: _AUG_BUFFERS.pop(k, None) if _AUG_BUFFERS.get(k) is _r
                                    else None)
    return buf[:, :K].view(B, Ntok, K)
