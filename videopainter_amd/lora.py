"""VideoPainterID LoRA adapters, folded into the base weights at load time.

The reference loads the ID-resample adapter unfused through PEFT (`pipe.load_lora_weights(path,
weight_name="pytorch_lora_weights.safetensors", adapter_name=..., target_modules=["transformer"])`,
infer/inpaint.py:310-315; `CogVideoXLoraLoaderMixin.load_lora_into_transformer`,
diffusers/loaders/lora_pipeline.py:2632-2705).  Its forward is `W x + s * B (A x)` on to_q / to_k / to_v /
to_out.0 (the training script's `LoraConfig(target_modules=["to_q", "to_k", "to_v", "to_out.0"])`,
train/train_cogvideox_inpainting_i2v_video_resample.py:1520-1525) with

    s = lora_alpha / r * lora_scale

where the loader passes no network alphas, so `get_peft_kwargs` sets lora_alpha = r (utils/peft_utils.py:153) —
s = lora_scale (attention_kwargs["scale"], default 1.0) whatever alpha the adapter was trained with.  Folding that
product into W once (`W + s B A`, accumulated in fp32, rounded to the weight dtype) gives every kernel of the HIP
path the adapted weights with no per-step cost.  Kohya-style files (`lora_down` / `lora_up` + `.alpha`) are
accepted too; their alpha is honoured (alpha / r), as the generic diffusers conversion does.

Runtime scale: the reference scales the adapters per call (`attention_kwargs["scale"]`, default 1.0,
cogvideox_transformer_3d.py:490-499 -> `scale_lora_layers`).  `attach_lora_` keeps the base weights of the adapted
layers (a device copy, 4 x 3072^2 bf16 per block) and the adapter factors, so `refold_lora_` can rebuild
`W0 + s * B A` exactly (the same fp32 expression as the first fold, bit-identical to folding s from scratch)
whenever a call passes a different scale; the transformer's forward does that before its first launch.

Parity: PEFT is not installed here, so the reference's unfused LoRA forward cannot run; `tests/test_lora_cpu.py`
checks the fold against the LoRA formula on the module level and the round trip (fold, unfold) — "parity unpinned"
against PEFT itself.
"""
from __future__ import annotations

import os
import re
from typing import Dict, Optional

import torch

TARGETS = ("to_q", "to_k", "to_v", "to_out.0")
_PEFT = re.compile(r"^(?:(?P<prefix>transformer)\.)?(?P<mod>.+)\.lora_(?P<ab>[AB])(?:\.[^.]+)?\.weight$")
_KOHYA = re.compile(r"^(?:(?P<prefix>transformer)\.)?(?P<mod>.+)\.lora_(?P<ab>down|up)\.weight$")


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


@torch.no_grad()
def fold_lora_(model: torch.nn.Module, sd: Dict[str, torch.Tensor], lora_scale: float = 1.0,
               strict: bool = True) -> int:
    """W += s * B @ A for every adapted Linear of `model` (in place); returns the number of folded layers.
    s = lora_scale for PEFT-format adapters (the reference loader's alpha = r), alpha / r * lora_scale for kohya
    files that carry an alpha.  Fold BEFORE `enable_fp8*` (those quantise the weights they find)."""
    mods = dict(model.named_modules())
    n = 0
    for mod, p in lora_pairs(sd).items():
        lin = mods.get(mod)
        if lin is None or not hasattr(lin, "weight"):
            if strict:
                raise KeyError(f"LoRA targets {mod}, which the model does not have")
            continue
        A, B = p["A"], p["B"]
        r = A.shape[0]
        s = lora_scale * (p["alpha"] / r if p.get("alpha") is not None else 1.0)
        W = lin.weight
        if tuple(W.shape) != (B.shape[0], A.shape[1]):
            raise ValueError(f"LoRA {mod}: B@A is {(B.shape[0], A.shape[1])}, weight is {tuple(W.shape)}")
        delta = B.to(W.device, torch.float32) @ A.to(W.device, torch.float32)
        W.copy_((W.float() + s * delta).to(W.dtype))
        n += 1
    return n


def load_lora_into_transformer(transformer: torch.nn.Module, path: str,
                               weight_name: str = "pytorch_lora_weights.safetensors", lora_scale: float = 1.0,
                               strict: bool = True) -> int:
    """What `pipe.load_lora_weights(path, weight_name=...)` + `attention_kwargs={"scale": lora_scale}` do to the
    transformer's forward, as a one-time weight fold."""
    sd = load_lora_state_dict(path, weight_name)
    keys = [k for k in sd if k.startswith("transformer.")]
    if keys:  # the pipeline-level file: only the transformer's entries (lora_pipeline.py:2653-2656)
        sd = {k: v for k, v in sd.items() if k.startswith("transformer.")}
    return fold_lora_(transformer, sd, lora_scale, strict)


def unfold_lora_(model: torch.nn.Module, sd: Dict[str, torch.Tensor], lora_scale: float = 1.0) -> int:
    """Remove a folded adapter (W -= s B A; exact only up to the weight dtype's rounding)."""
    return fold_lora_(model, sd, -lora_scale)


class LoraState:
    """What the model needs to re-fold at another scale: base weights of the adapted layers, the adapters, the scale
    currently folded.  Kept in the module's __dict__ (not buffers: the state dict stays the reference's)."""

    def __init__(self):
        self.base: Dict[str, torch.Tensor] = {}
        self.adapters: list = []      # [(name, {module: {"A", "B", "alpha"}})]
        self.scale: Optional[float] = None
        self.weights: Dict[str, float] = {}   # set_adapters() weights per adapter (1.0 when loaded, 0 = inactive)
        self.fused = False            # fuse_lora(): the folded scale no longer follows the per-call scale
        self.trainable: set = set()   # adapters added by add_trainable_adapter_: applied unfused, never folded


def lora_state(model: torch.nn.Module) -> Optional[LoraState]:
    return model.__dict__.get("_vp_lora")


def _fold_module(st: LoraState, mod: str, W: torch.Tensor, scale: float) -> None:
    acc = st.base[mod].to(W.device, torch.float32)
    for name, pairs in st.adapters:
        p = pairs.get(mod)
        if p is None or st.weights.get(name, 1.0) == 0.0 or name in st.trainable:
            continue
        r = p["A"].shape[0]
        s = scale * st.weights.get(name, 1.0) * (p["alpha"] / r if p.get("alpha") is not None else 1.0)
        acc = acc + s * (p["B"].detach().to(W.device, torch.float32) @ p["A"].detach().to(W.device, torch.float32))
    W.copy_(acc.to(W.dtype))


def _requant_fp8(model) -> None:
    for blk in getattr(model, "transformer_blocks", []):
        if getattr(blk, "qkv_mx", None) is not None:
            blk.enable_fp8_qkv(True)


@torch.no_grad()
def refold_lora_(model: torch.nn.Module, scale: float) -> int:
    """W = W0 + scale * sum over adapters of (alpha / r) B A, from the kept base weights (exact: the first fold's
    expression).  Re-quantises an enabled fp8 QKV projection of the blocks whose weights changed."""
    st = lora_state(model)
    if st is None:
        return 0
    mods = dict(model.named_modules())
    for mod in st.base:
        _fold_module(st, mod, mods[mod].weight, scale)
    st.scale = float(scale)
    _requant_fp8(model)
    return len(st.base)


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
    frozen, as PEFT does.  The adapter runs UNFUSED like PEFT's (y = x W0^T + s (x A^T) B^T, the delta added in
    output space, so updates far below a bf16 ulp of W0 still reach the forward): the projection GEMM runs on the
    K-augmented operands [x | x A^T] and [W0 | s B] (`AugmentedProjection`) with its fused epilogue unchanged; the
    backward splits the augmented gradients into the factors' (autograd.py)."""
    import math
    if r <= 0:
        raise ValueError("LoRA rank must be positive")
    targets = tuple(target_modules)
    model.requires_grad_(False)
    st = lora_state(model)
    if st is None:
        st = model.__dict__["_vp_lora"] = LoraState()
    if any(n == adapter_name for n, _ in st.adapters):
        raise ValueError(f"adapter {adapter_name!r} is already loaded")
    pairs = {}
    for name, lin in list(model.named_modules()):
        if not any(name == t or name.endswith("." + t) for t in targets) or not hasattr(lin, "weight"):
            continue
        if hasattr(lin, "lora_A"):
            raise ValueError(f"{name} already carries a trainable adapter (one trainable adapter per model)")
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
        lin.__dict__["_vp_lora_train"] = (st, adapter_name, float(lora_alpha))
        if name not in st.base:
            st.base[name] = W.detach().clone()
    if not pairs:
        raise ValueError(f"no module matches target_modules {targets}")
    st.adapters.append((adapter_name, pairs))
    st.weights[adapter_name] = 1.0
    st.trainable.add(adapter_name)
    refold_lora_(model, st.scale if st.scale is not None else 1.0)
    return len(pairs)


def trainable_lora_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """`get_peft_model_state_dict(transformer)`: the trainable factors under PEFT's saved names."""
    return {k: v.detach() for k, v in model.state_dict().items() if ".lora_A.weight" in k or ".lora_B.weight" in k}


@torch.no_grad()
def attach_lora_(model: torch.nn.Module, sd: Dict[str, torch.Tensor], lora_scale: float = 1.0,
                 adapter_name: Optional[str] = None, strict: bool = True) -> int:
    """Register an adapter on `model` and fold it (with every adapter attached before) at `lora_scale`."""
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
        pairs[mod] = {"A": p["A"].to(W.device), "B": p["B"].to(W.device), "alpha": p.get("alpha")}
    st = lora_state(model)
    if st is None:
        st = model.__dict__["_vp_lora"] = LoraState()
    if st.scale is not None and st.scale != lora_scale:
        refold_lora_(model, lora_scale)
    for mod in pairs:
        if mod not in st.base:
            st.base[mod] = mods[mod].weight.detach().clone()
    name = adapter_name or f"default_{len(st.adapters)}"
    if any(n == name for n, _ in st.adapters):
        raise ValueError(f"adapter {name!r} is already loaded")
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
    refold_lora_(model, st.scale if st.scale is not None else 1.0)


# ------------------------------------------------------------------------------------------------------------------
# Trainable adapters, unfused: K-augmented projection operands
# ------------------------------------------------------------------------------------------------------------------

def trainable_pair(lin):
    """(A, B, s) of the trainable (unfused) adapter on the Linear `lin`, or None: A [r, in], B [out, r] (the
    parameters themselves), s = call scale x adapter weight x alpha / r (PEFT's scaling)."""
    t = lin.__dict__.get("_vp_lora_train")
    if t is None or getattr(lin, "lora_A", None) is None:
        return None
    st, name, alpha = t
    w = st.weights.get(name, 1.0)
    if w == 0.0:
        return None
    A, B = lin.lora_A.weight, lin.lora_B.weight
    s = (st.scale if st.scale is not None else 1.0) * w * alpha / A.shape[0]
    return A, B, s


AUG_ALIGN = 64  # the augmented K is padded to whole 64-wide K-tiles of the GEMM (zero columns / rows)


class AugmentedProjection:
    """One GEMM over several projections (the fused QKV, the prev-clip K/V, to_out) whose Linears carry trainable
    adapters, as PEFT computes them unfused: y_i = x W_i^T + b_i + s_i (x A_i^T) B_i^T, as ONE GEMM on
    K-augmented operands
        x_aug = [x | T],  T = x [A_1; A_2; ...]^T  (bf16, zero-padded to a multiple of 64 columns),
        W_aug_i = [W_i | 0 .. s_i B_i .. 0]        (bf16, s_i B_i in projection i's rank block),
    so the fused epilogues (qk-norm + RoPE, gated residual) see the adapted projection, and the delta enters in the
    fp32 accumulator (a factor update far below a bf16 ulp of W still changes the output, which folding it into a
    bf16 weight loses).  Built per forward from the live factors (cached on their versions and the scale)."""

    def __init__(self, lins):
        self.lins = list(lins)
        self.pairs = [trainable_pair(l) for l in self.lins]
        self.offs = []
        off = 0
        for p in self.pairs:
            self.offs.append(off)
            off += p[0].shape[0] if p is not None else 0
        self.R = off
        self.Rp = (off + AUG_ALIGN - 1) // AUG_ALIGN * AUG_ALIGN
        self.K = self.lins[0].weight.shape[1]

    @staticmethod
    def of(lins):
        """The augmentation of these projections, or None when none carries a trainable adapter."""
        if not any(trainable_pair(l) is not None for l in lins):
            return None
        return AugmentedProjection(lins)

    def _key(self):
        return tuple((p[0]._version, p[1]._version, p[0].data_ptr(), p[1].data_ptr(), p[2]) if p is not None
                     else None for p in self.pairs) + tuple((l.weight._version, l.weight.data_ptr())
                                                            for l in self.lins)

    def a_cat(self) -> torch.Tensor:
        """[Rp, K] bf16: the A factors stacked (zero rows for the padding)."""
        owner = self.lins[0]
        key = ("A", tuple(id(l) for l in self.lins)) + self._key()
        c = owner.__dict__.get("_vp_aug_A")
        if c is None or c[0] != key:
            W = self.lins[0].weight
            a = torch.zeros(self.Rp, self.K, device=W.device, dtype=torch.bfloat16)
            for p, o in zip(self.pairs, self.offs):
                if p is not None:
                    a[o:o + p[0].shape[0]].copy_(p[0].detach())
            c = (key, a)
            owner.__dict__["_vp_aug_A"] = c
        return c[1]

    def a_cat_t(self) -> torch.Tensor:
        """[K, Rp] bf16 = a_cat()^T (the dgrad operand of T = x A_cat^T)."""
        from . import kernels as K
        owner = self.lins[0]
        key = ("At", tuple(id(l) for l in self.lins)) + self._key()
        c = owner.__dict__.get("_vp_aug_At")
        if c is None or c[0] != key:
            c = (key, K.transpose(self.a_cat()))
            owner.__dict__["_vp_aug_At"] = c
        return c[1]

    def weights(self):
        """[W_aug_i] bf16 [out_i, K + Rp] (one per Linear)."""
        out = []
        key = self._key()
        for i, (l, p) in enumerate(zip(self.lins, self.pairs)):
            k = ("W", tuple(id(x) for x in self.lins), i) + key
            c = l.__dict__.get("_vp_aug_W")
            if c is None or c[0] != k:
                W = l.weight.detach()
                w = torch.zeros(W.shape[0], self.K + self.Rp, device=W.device, dtype=torch.bfloat16)
                w[:, :self.K].copy_(W)
                if p is not None:
                    o = self.offs[i]
                    w[:, self.K + o:self.K + o + p[0].shape[0]].copy_((p[1].detach().float() * p[2]))
                c = (k, w)
                l.__dict__["_vp_aug_W"] = c
            out.append(c[1])
        return out

    def input(self, x2d: torch.Tensor) -> torch.Tensor:
        """x_aug [M, K + Rp] = [x | x A_cat^T] (one GEMM for T)."""
        from . import kernels as K
        M = x2d.shape[0]
        xa = torch.empty(M, self.K + self.Rp, device=x2d.device, dtype=torch.bfloat16)
        xa[:, :self.K].copy_(x2d)
        K.gemm(x2d, [self.a_cat()], [None], xa[:, self.K:])
        return xa
