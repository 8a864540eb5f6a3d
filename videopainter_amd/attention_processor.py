"""The attention module and the two CogVideoX attention processors, on the HIP kernels.

Secondary drop-in boundary: `Attention.set_processor` / `set_attn_processor` and the processor
call signature `(attn, hidden_states, encoder_hidden_states, attention_mask=None, resample_mask=None,
image_rotary_emb=None, prev_hidden_states=None, prev_clip_weight=None, prev_resample_mask=None)
-> (hidden_states, encoder_hidden_states)` of DF/models/attention_processor.py:2107-2118 / :2223-2234.
The processors work on any `attn` object exposing to_q/to_k/to_v/to_out[0]/norm_q/norm_k/heads (ours, or a
reference `Attention` holding bf16 device weights).

`attend()` is the fused core (QKV projection -> qk-LN + RoPE -> flash attention, everything before to_out); the
block calls it directly so that to_out runs as one GEMM with the gated residual fused in its epilogue.
"""
from __future__ import annotations

import inspect
import os
from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import _native as NAT
from . import kernels as K
from .lora import AugmentedProjection, augmented_rows
from .modules import Dropout, LayerNorm, Linear

BF16 = torch.bfloat16


# Python-side A/B switches, read from the environment once at import (as the library's knob table is at load) and
# changed only through set_switch (tests/conftest.py `knobs`): VP_NO_QKV_FUSION=1 (separate qk-norm launches),
# VP_ATTN_BOUNDED=0 (no score-bound flag), VP_RESAMPLE_PARTITION / _NULLMASS / _K2_STRIDED=0 (resample-processor forms)
SWITCHES = {k: os.environ.get(k) for k in ("VP_NO_QKV_FUSION", "VP_ATTN_BOUNDED", "VP_RESAMPLE_PARTITION",
                                           "VP_RESAMPLE_NULLMASS", "VP_RESAMPLE_K2_STRIDED")}


def set_switch(name: str, value: Optional[str]) -> Optional[str]:
    """Set (value None: unset) one of SWITCHES; returns the previous value."""
    if name not in SWITCHES:
        raise KeyError(f"unknown switch {name}")
    prev = SWITCHES[name]
    SWITCHES[name] = value
    return prev


def _sw(name: str, default: str) -> str:
    v = SWITCHES[name]
    return default if v is None else v


class RopeTables(tuple):
    """(cos, sin) fp32 [F*Hh*Ww, 64] on the device, plus the video grid (F, Hh, Ww) they were built for when the
    transformer's forward knows it (None otherwise): the resample processor needs the grid to sum its null keys in
    closed form (kernels.null_key_mass)."""
    grid = None


def _rope_dev(rope, device, grid=None):
    if rope is None:
        return None
    cos, sin = rope
    if cos.device != device or cos.dtype != torch.float32 or not cos.is_contiguous():
        cos = cos.to(device=device, dtype=torch.float32).contiguous()
    if sin.device != device or sin.dtype != torch.float32 or not sin.is_contiguous():
        sin = sin.to(device=device, dtype=torch.float32).contiguous()
    out = RopeTables((cos, sin))
    out.grid = tuple(grid) if grid is not None else getattr(rope, "grid", None)
    return out


def _u8(mask: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """A token mask as contiguous uint8 (the kernels test a byte for non-zero).  An already contiguous uint8 mask is
    returned as is — the same tensor — so the per-forward mask plan (_mask_plan, keyed on the tensor) is built once
    and found by every layer."""
    if mask is None:
        return None
    if mask.dtype == torch.uint8 and mask.is_contiguous():
        return mask
    if mask.dtype == torch.bool:
        return mask.contiguous().view(torch.uint8)
    return (mask != 0).to(torch.uint8).contiguous()


class Attention(nn.Module):
    """Parameter layout of the reference `Attention` as CogVideoXBlock builds it (attention_processor.py:96-264:
    qk_norm="layer_norm" eps 1e-6, bias=True, out_bias=True, scale = dim_head**-0.5)."""

    def __init__(self, query_dim: int, dim_head: int = 64, heads: int = 8, bias: bool = True, out_bias: bool = True,
                 eps: float = 1e-6, processor=None):
        super().__init__()
        self.inner_dim = dim_head * heads
        self.heads = heads
        self.dim_head = dim_head
        self.scale = dim_head ** -0.5
        self.is_cross_attention = False
        self.norm_q = LayerNorm(dim_head, eps=eps)
        self.norm_k = LayerNorm(dim_head, eps=eps)
        self.to_q = Linear(query_dim, self.inner_dim, bias=bias)
        self.to_k = Linear(query_dim, self.inner_dim, bias=bias)
        self.to_v = Linear(query_dim, self.inner_dim, bias=bias)
        self.to_out = nn.ModuleList([Linear(self.inner_dim, query_dim, bias=out_bias), Dropout()])
        self.set_processor(processor if processor is not None else CogVideoXAttnProcessor2_0())

    def set_processor(self, processor) -> None:
        self.processor = processor

    def get_processor(self, return_deprecated_lora: bool = False):
        return self.processor

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **cross_attention_kwargs):
        # kwargs the processor does not declare are dropped, as in the reference (:479-488)
        params = set(inspect.signature(self.processor.__call__).parameters.keys())
        kw = {k: v for k, v in cross_attention_kwargs.items() if k in params}
        return self.processor(self, hidden_states, encoder_hidden_states=encoder_hidden_states,
                              attention_mask=attention_mask, **kw)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """bf16 [B, N, D] rows with a contiguous last dim, at any row stride (the first columns of an x_aug buffer,
    lora.augmented_rows, stay in place)."""
    t = t.to(BF16)
    return t if t.stride(-1) == 1 else t.contiguous()


def _qkv(attn, x: torch.Tensor, norm_rope=None) -> torch.Tensor:
    """The fused QKV projection; with norm_rope = (text_len, rope) q and k leave the GEMM already through norm_q /
    norm_k and RoPE (the epilogue EPI_BIAS_QKNORM_ROPE: bit-equal to the GEMM + vp_head_norm_rope_bf16 on each)."""
    B, Ntok, D = x.shape
    out = torch.empty(B, Ntok, 3 * attn.inner_dim if hasattr(attn, "inner_dim") else 3 * D, device=x.device,
                      dtype=BF16)
    ws = [attn.to_q.weight, attn.to_k.weight, attn.to_v.weight]
    bs = [attn.to_q.bias, attn.to_k.bias, attn.to_v.bias]
    a = x.reshape(-1, D)
    aug = AugmentedProjection.of((attn.to_q, attn.to_k, attn.to_v))
    kw = {}
    if norm_rope is not None:
        text_len, rope = norm_rope
        kw = dict(epilogue=NAT.EPI_BIAS_QKNORM_ROPE, qk_norm=(attn.norm_q, attn.norm_k), rope=rope,
                  tokens_per_batch=Ntok, text_len=text_len)
    if aug is not None:  # LoRA adapters, unfused (lora.AugmentedProjection)
        aug.gemm(aug.input(a), bs, out.view(B * Ntok, -1), **kw)
    else:
        K.gemm(a, ws, bs, out.view(B * Ntok, -1), **kw)
    return out


def _kv(attn, x: torch.Tensor) -> torch.Tensor:
    B, Ntok, D = x.shape
    out = torch.empty(B, Ntok, 2 * D, device=x.device, dtype=BF16)
    a, ws = x.reshape(-1, D), [attn.to_k.weight, attn.to_v.weight]
    aug = AugmentedProjection.of((attn.to_k, attn.to_v))
    if aug is not None:
        aug.gemm(aug.input(a), [attn.to_k.bias, attn.to_v.bias], out.view(B * Ntok, -1))
    else:
        K.gemm(a, ws, [attn.to_k.bias, attn.to_v.bias], out.view(B * Ntok, -1))
    return out


def project_out(lin, o2d: torch.Tensor, out2d: torch.Tensor, **gemm_kw) -> torch.Tensor:
    """to_out.0 on [M, D] rows with any GEMM epilogue (the block's gated residual), its LoRA adapters applied
    unfused (lora.AugmentedProjection) when it carries any."""
    aug = AugmentedProjection.of((lin,))
    if aug is not None:
        return aug.gemm(aug.input(o2d), [lin.bias], out2d, **gemm_kw)
    return K.gemm(o2d, [lin.weight], [lin.bias], out2d, **gemm_kw)


def _fusable_norms(attn) -> bool:
    """norm_q / norm_k are LayerNorm(64) with bf16 affine parameters (CogVideoX's qk_norm, the fused epilogue's
    contract); env VP_NO_QKV_FUSION=1 keeps the separate vp_head_norm_rope_bf16 launches (A/B)."""
    if _sw("VP_NO_QKV_FUSION", "0") == "1":
        return False
    for ln in (getattr(attn, "norm_q", None), getattr(attn, "norm_k", None)):
        if ln is None or getattr(ln, "weight", None) is None or getattr(ln, "bias", None) is None:
            return False
        if ln.weight.numel() != 64 or ln.weight.dtype != BF16 or ln.bias.dtype != BF16:
            return False
    return True


def bounded_scores(attn) -> bool:
    """True when the qk-LayerNorm weights bound every attention score of `attn` within the kernel's exact
    no-running-max range (kernels.score_bound_log2 <= SCORE_BOUND_LOG2).  Cached per layer on the weights' storage and
    version (one host sync per weight update); env VP_ATTN_BOUNDED=0 forces the running-max kernel (A/B)."""
    if _sw("VP_ATTN_BOUNDED", "1") == "0":
        return False
    nq, nk = attn.norm_q, attn.norm_k
    key = tuple((t.data_ptr(), t._version) for t in (nq.weight, nq.bias, nk.weight, nk.bias)) + (float(attn.scale),)
    cached = getattr(attn, "_vp_score_bound", None)
    if cached is None or cached[0] != key:
        cached = (key, K.score_bound_log2(nq, nk, float(attn.scale)) <= K.SCORE_BOUND_LOG2)
        attn._vp_score_bound = cached
    return cached[1]


class CogVideoXAttnProcessor2_0:
    """HIP restatement of `CogVideoXAttnProcessor2_0.__call__` (attention_processor.py:2107-2209)."""

    def attend(self, attn, x: torch.Tensor, text_len: int, image_rotary_emb=None, prev_hidden_states=None,
               prev_clip_weight=None, resample_mask=None, prev_resample_mask=None,
               qkv: Optional[torch.Tensor] = None, lse_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """lse_out: optional fp32 [B, H, N] receiving the softmax statistics of the (single-segment, bf16) attention
        — a training forward keeps them with the output for the backward (autograd.SAVE_ATTENTION)."""
        B, Ntok, D = x.shape
        H = attn.heads
        rope = _rope_dev(image_rotary_emb, x.device)
        fp8 = getattr(attn, "fp8_qk_exp", None)
        if lse_out is not None and (fp8 is not None or prev_hidden_states is not None):
            raise ValueError("lse_out: the single-segment bf16 attention only")
        fused = qkv is None and fp8 is None and _fusable_norms(attn)
        if qkv is None:  # (the block may hand over an fp8 projection)
            qkv = _qkv(attn, x, (text_len, rope) if fused else None)
        q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
        eps_k = attn.norm_k.eps
        if fp8 is not None:
            return self._attend_fp8(attn, q, k, v, text_len, rope, fp8, prev_hidden_states, prev_clip_weight)
        if not fused:
            K.head_norm_rope(q, q, H, text_len, attn.norm_q.weight, attn.norm_q.bias, attn.norm_q.eps, rope)
            K.head_norm_rope(k, k, H, text_len, attn.norm_k.weight, attn.norm_k.bias, eps_k, rope)
        o = augmented_rows((attn.to_out[0],), B, Ntok, D, x.device)
        if prev_hidden_states is not None and prev_clip_weight is not None and prev_clip_weight > 0.0:
            pkv = _kv(attn, _rows(prev_hidden_states))
            pk, pv = pkv[..., :D], pkv[..., D:]
            K.head_norm_rope(pk, pk, H, text_len, attn.norm_k.weight, attn.norm_k.bias, eps_k, rope)
            w = float(prev_clip_weight)
            bs = bounded_scores(attn)
            K.attention(q, k, v, o, H, scale=attn.scale, out_scale=1.0 - w, bounded_scores=bs)
            K.attention(q, pk, pv, o, H, scale=attn.scale, out_scale=w, accumulate=True, bounded_scores=bs)
        else:
            K.attention(q, k, v, o, H, scale=attn.scale, bounded_scores=bounded_scores(attn), lse=lse_out)
        return o

    @staticmethod
    def _attend_fp8(attn, q, k, v, text_len, rope, exps, prev_hidden_states, prev_clip_weight) -> torch.Tensor:
        """fp8 attention (BASELINE config 5): qk-norm + RoPE written as e4m3 with the static power-of-two factors
        chosen by `CogVideoXBlock.enable_fp8_attention` (Q's includes scale * log2 e), V packed to e4m3 V^T with
        per-(d, 32 keys) scales, the block-scaled MFMA kernel; the prev-clip blend as in the bf16 path."""
        B, Ntok, D = q.shape
        H = attn.heads
        q_exp, k_exp = exps
        qmul = attn.scale * K.LOG2E * 2.0 ** q_exp
        q8 = K.head_norm_rope_fp8(q, H, text_len, attn.norm_q.weight, attn.norm_q.bias, attn.norm_q.eps, rope, qmul)
        k8 = K.head_norm_rope_fp8(k, H, text_len, attn.norm_k.weight, attn.norm_k.bias, attn.norm_k.eps, rope,
                                  2.0 ** k_exp)
        vp = K.v_pack_fp8(v, H)
        o = augmented_rows((attn.to_out[0],), B, Ntok, D, q.device)
        if prev_hidden_states is not None and prev_clip_weight is not None and prev_clip_weight > 0.0:
            pkv = _kv(attn, _rows(prev_hidden_states))
            pk8 = K.head_norm_rope_fp8(pkv[..., :D], H, text_len, attn.norm_k.weight, attn.norm_k.bias,
                                       attn.norm_k.eps, rope, 2.0 ** k_exp)
            pvp = K.v_pack_fp8(pkv[..., D:], H)
            del pkv
            w = float(prev_clip_weight)
            K.attention_fp8(q8, k8, vp, o, H, q_exp, k_exp, out_scale=1.0 - w)
            K.attention_fp8(q8, pk8, pvp, o, H, q_exp, k_exp, out_scale=w, accumulate=True)
        else:
            K.attention_fp8(q8, k8, vp, o, H, q_exp, k_exp)
        return o

    def __call__(self, attn, hidden_states: torch.Tensor, encoder_hidden_states: torch.Tensor,
                 attention_mask: Optional[torch.Tensor] = None, resample_mask: Optional[torch.Tensor] = None,
                 image_rotary_emb=None, prev_hidden_states: Optional[torch.Tensor] = None,
                 prev_clip_weight: Optional[float] = None, prev_resample_mask: Optional[torch.Tensor] = None
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is never set on the CogVideoX path (SURVEY.md §3.2)")
        t = encoder_hidden_states.size(1)
        x = torch.cat([encoder_hidden_states, hidden_states], dim=1).to(BF16).contiguous()
        o = self.attend(attn, x, t, image_rotary_emb, prev_hidden_states, prev_clip_weight, resample_mask,
                        prev_resample_mask)
        out = torch.empty_like(o)
        project_out(attn.to_out[0], o.view(-1, o.shape[-1]), out.view(-1, o.shape[-1]))
        return out[:, t:], out[:, :t]


class CogVideoXAttnProcessor2_0_wo_text(CogVideoXAttnProcessor2_0):
    """HIP restatement of `CogVideoXAttnProcessor2_0_wo_text.__call__` (attention_processor.py:2306-2366): the
    branch's text-free mode, self-attention over the video tokens alone with RoPE on every token — `attend` with
    text_len = 0.  Without RoPE the reference never runs its attention (the call sits inside its
    `if image_rotary_emb is not None:`, :2349-2356): its head merge (:2358, `transpose(1, 2).reshape(B, -1, D)`)
    then scrambles the processor's INPUT, which goes on to to_out — restated as that exact permutation (attend)."""

    def attend(self, attn, x: torch.Tensor, text_len: int, image_rotary_emb=None, *args, **kwargs) -> torch.Tensor:
        if image_rotary_emb is not None:
            return super().attend(attn, x, text_len, image_rotary_emb, *args, **kwargs)
        # no RoPE: o[b] = x[b]^T read back as [N, D] rows (the reference's transpose + reshape of a [B, N, D] tensor);
        # the Q / K / V it computes and drops are skipped
        B, N, D = x.shape
        o = torch.empty(B, N, D, device=x.device, dtype=BF16)
        for b in range(B):
            K.transpose(x[b], out=o[b].view(D, N))
        return o

    def __call__(self, attn, hidden_states: torch.Tensor, encoder_hidden_states: Optional[torch.Tensor] = None,
                 attention_mask: Optional[torch.Tensor] = None, image_rotary_emb=None) -> torch.Tensor:
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is never set on the CogVideoX path (SURVEY.md §3.2)")
        x = hidden_states.to(BF16).contiguous()
        o = self.attend(attn, x, 0, image_rotary_emb)
        out = torch.empty_like(o)
        project_out(attn.to_out[0], o.view(-1, o.shape[-1]), out.view(-1, o.shape[-1]))
        return out


_MASK_PLANS: dict = {}


def _mask_plan(m: torch.Tensor, text_len: int, grid):
    """(dst_rows, counts, segments) of a resample mask — the stable partition (masked rows first) and, with a grid,
    the null-key segments (kernels.mask_null_segments) — computed once per mask and reused by every layer of the
    forward (the transformer hands all blocks the same mask tensor).  Keyed on the mask's storage and version; the
    entry holds the mask, so its address is not reused while cached; an event orders a reuse on another stream."""
    key = (m.data_ptr(), m._version, tuple(m.shape), text_len, grid)
    hit = _MASK_PLANS.get(key)
    if hit is not None and hit[0] is m:
        torch.cuda.current_stream(m.device).wait_event(hit[4])
        return hit[1], hit[2], hit[3]
    dst, cnt = K.partition_rows_index(m)
    segments = None
    if grid is not None:
        segments = K.mask_null_segments(m, text_len, grid)
        # only the masked rows are segment 2 now: the null rows' copies are skipped (dst -1)
        dst = torch.where(m.bool(), dst, torch.full_like(dst, -1))
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(m.device))
    if len(_MASK_PLANS) >= 8:
        _MASK_PLANS.pop(next(iter(_MASK_PLANS)))
    _MASK_PLANS[key] = (m, dst, cnt, segments, ev)
    return dst, cnt, segments


class CogVideoXAttnProcessor2_0_resample(CogVideoXAttnProcessor2_0):
    """HIP restatement of `CogVideoXAttnProcessor2_0_resample.__call__` (attention_processor.py:2223-2304).

    The doubled K/V (cat along the sequence, :2283-2284) is not materialised: the masked copy is built once
    (LN of the zero-masked projection -> the LN bias "null key", then RoPE) and passed to the flash kernel as a
    second K/V segment."""

    def attend(self, attn, x: torch.Tensor, text_len: int, image_rotary_emb=None, prev_hidden_states=None,
               prev_clip_weight=None, resample_mask=None, prev_resample_mask=None,
               qkv: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, Ntok, D = x.shape
        rope = _rope_dev(image_rotary_emb, x.device)
        prev = prev_hidden_states is not None and prev_clip_weight is not None and prev_clip_weight > 0.0
        if not prev and resample_mask is None:
            raise ValueError("the resample processor needs resample_mask (id_pool_resample needs masks)")
        m = _u8(prev_resample_mask if prev else resample_mask)
        plan = self.plan(attn, m, text_len, rope)
        # with the null keys in closed form segment 2 holds masked rows only, and those of window 0 are rows of the
        # normed + rotated K itself: q / k then leave the QKV GEMM through the fused norm + RoPE epilogue
        fused = plan[3] is not None and qkv is None and _fusable_norms(attn)
        if qkv is None:  # (the block may hand over an fp8 projection)
            qkv = _qkv(attn, x, (text_len, rope) if fused else None)
        pk = pv = None
        if prev:
            pkv = _kv(attn, _rows(prev_hidden_states))
            pk, pv = pkv[..., :D], pkv[..., D:]
        o = augmented_rows((attn.to_out[0],), B, Ntok, D, x.device)
        return self.attend_heads(attn, qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:], text_len, rope, m, plan,
                                 fused, pk, pv, float(prev_clip_weight) if prev else 0.0, o)

    @staticmethod
    def plan(attn, m: torch.Tensor, text_len: int, rope):
        """(dst_rows, counts, segments, axes) of the token mask m [B, N] (uint8).  The second segment in partitioned
        row order: the masked rows' keys / values first, then the null keys (LN of a zeroed row = the norm_k bias,
        rotated) whose values are zero — they only add to the row sums.  The order of keys does not change
        attention.  With the video grid known and the RoPE table separable, the null keys leave the segment (k2_len
        = the masked-row count) and their row mass is summed in closed form over the grid (null_key_mass ->
        l_extra, DESIGN_LOG.md §3.0; axes = the per-axis RoPE tables); otherwise they stay as row-sum-only keys
        (k2_full).  VP_RESAMPLE_NULLMASS=0: keep them as keys; VP_RESAMPLE_PARTITION=0: original order (A/B)."""
        dst = cnt = segments = axes = None
        grid = getattr(rope, "grid", None)
        if _sw("VP_RESAMPLE_PARTITION", "1") != "0":
            if (grid is not None and _sw("VP_RESAMPLE_NULLMASS", "1") != "0"
                    and attn.norm_k.bias is not None and attn.norm_k.bias.dtype == BF16
                    and K.null_key_mass_supported(grid)):
                axes = K.rope_axis_tables(rope, grid)
            dst, cnt, segments = _mask_plan(m, text_len, grid if axes is not None else None)
        return dst, cnt, segments, axes

    def attend_heads(self, attn, q, k, v, text_len: int, rope, m, plan, fused: bool, pk=None, pv=None,
                     w: float = 0.0, o=None) -> torch.Tensor:
        """The processor's attention on [B, N, h*64] views of every head (or of one head group: the Ulysses split,
        videopainter_amd/ulysses.py) — q / k normed + rotated already when `fused`, pre-norm otherwise; pk / pv: the
        previous window's pre-norm K / V projections (prev-clip blend with weight w), or None."""
        B, Ntok, D = q.shape
        H = D // 64
        dst, cnt, segments, axes = plan
        grid = getattr(rope, "grid", None)
        # segment 2 with the row stride of the fused QKV output (3 D): the attention kernel then streams its full tiles
        # on the same precomputed lane offsets as segment 1 (DESIGN_LOG.md §3.R4)
        # (VP_RESAMPLE_K2_STRIDED=0: contiguous k2 / v2, the general per-lane DMA path; A/B)
        if _sw("VP_RESAMPLE_K2_STRIDED", "1") != "0":
            kv2 = torch.empty(B, Ntok, 3 * D, device=q.device, dtype=BF16)
            k2, v2 = kv2[..., :D], kv2[..., D:2 * D]
        else:
            k2 = torch.empty(B, Ntok, D, device=q.device, dtype=BF16)
            v2 = torch.empty(B, Ntok, D, device=q.device, dtype=BF16)
        if pk is not None:
            K.head_norm_rope(pk, k2, H, text_len, attn.norm_k.weight, attn.norm_k.bias, attn.norm_k.eps,
                             rope, tok_mask=m, pre_scale=w, dst_rows=dst)
            K.mask_scale_rows(pv, v2, m, w, dst_rows=dst)
        elif fused:  # LN(1 . k) + RoPE of a masked row is K's row (bit-equal: the epilogue's arithmetic)
            K.mask_scale_rows(k, k2, m, 1.0, dst_rows=dst)
            K.mask_scale_rows(v, v2, m, 1.0, dst_rows=dst)
        else:
            K.head_norm_rope(k, k2, H, text_len, attn.norm_k.weight, attn.norm_k.bias, attn.norm_k.eps, rope,
                             tok_mask=m, pre_scale=1.0, dst_rows=dst)
            K.mask_scale_rows(v, v2, m, 1.0, dst_rows=dst)
        if not fused:
            K.head_norm_rope(q, q, H, text_len, attn.norm_q.weight, attn.norm_q.bias, attn.norm_q.eps, rope)
            K.head_norm_rope(k, k, H, text_len, attn.norm_k.weight, attn.norm_k.bias, attn.norm_k.eps, rope)
        if o is None:
            o = torch.empty(B, Ntok, D, device=q.device, dtype=BF16)
        if axes is not None:
            lx = K.null_key_mass(q, H, text_len, grid, attn.norm_k.bias, axes, m, segments, attn.scale)
            K.attention(q, k, v, o, H, k2=k2, v2=v2, scale=attn.scale, bounded_scores=bounded_scores(attn),
                        k2_len=cnt, l_extra=lx)
        else:
            K.attention(q, k, v, o, H, k2=k2, v2=v2, scale=attn.scale, bounded_scores=bounded_scores(attn),
                        k2_full=cnt)
        return o
