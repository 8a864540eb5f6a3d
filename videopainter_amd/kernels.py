"""Torch-tensor front end of the HIP kernels (thin: validate, take pointers + current stream, call the C ABI).

Tensors are plumbing here — device memory and streams.  Every arithmetic op on the hot path runs in libvp_hip.so.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import torch

from . import _native as N

BF16 = torch.bfloat16


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


# Optional per-launch timing (bench.py's roofline): name -> list of (start, end) HIP events on the launch stream.
_TIMED: dict = {}


class timed_launches:
    """Context manager recording HIP events around every launch of the named kernels (on their stream)."""

    def __init__(self, *names):
        self.names = names

    def __enter__(self):
        for n in self.names:
            _TIMED[n] = []
        return self

    def __exit__(self, *exc):
        self.events = {n: _TIMED.pop(n, []) for n in self.names}

    def mean_ms(self, name: str) -> float:
        ev = self.events.get(name, [])
        torch.cuda.synchronize()
        return sum(s.elapsed_time(e) for s, e in ev) / max(1, len(ev))

    def count(self, name: str) -> int:
        return len(self.events.get(name, []))


def _t0(name):
    if name in _TIMED:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        return ev
    return None


def _t1(name, ev):
    if ev is not None:
        ev[1].record()
        _TIMED[name].append(ev)


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _chk(t: torch.Tensor, name: str, dtype=BF16):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA/HIP device tensor")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")


def _rowmajor(t: torch.Tensor, name: str) -> int:
    """Return the row stride of a 2-D (or last-dim-contiguous) tensor viewed as rows."""
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dimension")
    return t.stride(-2) if t.dim() >= 2 else t.shape[-1]


# ------------------------------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------------------------------

def gemm(a: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[Optional[torch.Tensor]],
         out: torch.Tensor, *, epilogue: int = N.EPI_BIAS, M: Optional[int] = None, lda: Optional[int] = None,
         ldc: Optional[int] = None, rows_per_group: Optional[int] = None, group_stride: int = 0, row_offset: int = 0,
         alpha: float = 1.0, resid: Optional[torch.Tensor] = None, ldr: Optional[int] = None,
         mod: Optional[torch.Tensor] = None, gate_chunk: int = 2, gate_text_chunk: int = 5,
         tokens_per_batch: int = 1, text_len: int = 0, inject: Optional[torch.Tensor] = None,
         inject_ld: int = 0, inject_bstride: int = 0, inject_mask: Optional[torch.Tensor] = None,
         addrows: Optional[torch.Tensor] = None, addrows_offset: int = 0, qk_norm=None, rope=None,
         a_tail: Optional[Tuple[int, Sequence[int]]] = None, aux: Optional[torch.Tensor] = None,
         z: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = epilogue(a @ cat(weights).T).  `a` rows: M rows of length K at stride lda.
    EPI_BIAS_QKNORM_ROPE: qk_norm = (norm_q, norm_k) LayerNorm(64) modules, rope = (cos, sin) fp32 [N - text_len, 64]
    or None; rows are (batch, token) with `tokens_per_batch` / `text_len`.
    a_tail = (k0, offsets): the per-segment A tail (vp_gemm_desc.a_tail_k / a_tail_off; unfused LoRA): for K columns
    k >= k0, weight segment s reads column k + offsets[s] of `a`.
    aux (ABI 17, the training forward): a bf16 [M, *] row-major second output — EPI_BIAS_GELU stores the
    pre-activation there, EPI_BIAS_QKNORM_ROPE the pre-norm q | k (its first 2 n_seg columns).
    z: EPI_GELU_BWD's GELU input, bf16 [M, N] row-major: out = bf16(bf16(a @ W^T + b) * gelu'(z))."""
    _chk(a, "a")
    _chk(out, "out")
    K = weights[0].shape[1]
    nseg = weights[0].shape[0]
    for w in weights:
        _chk(w, "weight")
        if w.shape != weights[0].shape or not w.is_contiguous():
            raise ValueError("weight segments must be contiguous and of equal shape")
    Ntot = nseg * len(weights)
    M = a.numel() // a.shape[-1] if M is None else M
    lda = _rowmajor(a, "a") if lda is None else lda
    if a.shape[-1] < K:
        raise ValueError(f"a has K={a.shape[-1]} < weight K={K}")
    d = N.GemmDesc()
    d.M, d.N, d.K, d.epilogue = M, Ntot, K, epilogue
    d.A, d.lda = _p(a), lda
    for i, w in enumerate(weights):
        d.W[i] = _p(w)
        b = biases[i] if biases is not None and i < len(biases) else None
        if b is not None:
            _chk(b, "bias")
        d.bias[i] = _p(b)
    d.n_seg = nseg
    d.C = _p(out)
    d.ldc = _rowmajor(out, "out") if ldc is None else ldc
    d.rows_per_group = M if rows_per_group is None else rows_per_group
    d.group_stride, d.row_offset = group_stride, row_offset
    d.alpha = alpha
    if epilogue == N.EPI_GATED:
        _chk(resid, "resid")
        _chk(mod, "mod")
        D = Ntot
        d.R = _p(resid)
        d.ldr = _rowmajor(resid, "resid") if ldr is None else ldr
        d.gate = mod.data_ptr() + gate_chunk * D * mod.element_size()
        d.gate_text = mod.data_ptr() + gate_text_chunk * D * mod.element_size()
        d.gate_bstride = mod.stride(0)
        d.tokens_per_batch, d.text_len = tokens_per_batch, text_len
        if inject is not None:
            _chk(inject, "inject")
            d.inject, d.inject_ld, d.inject_bstride = _p(inject), inject_ld, inject_bstride
            if inject_mask is not None:
                _chk(inject_mask, "inject_mask", torch.uint8)
                d.inject_mask = _p(inject_mask)
                d.inject_mask_bstride = inject_mask.stride(0)
    if epilogue == N.EPI_BIAS_QKNORM_ROPE:
        for i, ln in enumerate(qk_norm):
            _chk(ln.weight, "ln weight")
            _chk(ln.bias, "ln bias")
            if ln.weight.numel() != 64:
                raise ValueError("the fused qk-norm epilogue is LayerNorm over head_dim 64")
            d.qk_ln_w[i], d.qk_ln_b[i], d.qk_eps[i] = _p(ln.weight), _p(ln.bias), float(ln.eps)
        d.tokens_per_batch, d.text_len = tokens_per_batch, text_len
        if rope is not None:
            cos, sin = rope
            _chk(cos, "cos", torch.float32)
            _chk(sin, "sin", torch.float32)
            if (cos.shape != (tokens_per_batch - text_len, 64) or sin.shape != cos.shape or not cos.is_contiguous()
                    or not sin.is_contiguous()):
                raise ValueError(f"rope tables must be fp32 [{tokens_per_batch - text_len}, 64], "
                                 f"got {tuple(cos.shape)}")
            d.rope_cos, d.rope_sin = _p(cos), _p(sin)
            # a separable 3D table (the transformer's RopeTables carry their grid): the epilogue reads the per-axis
            # rows instead (the same values; ROPE_SEPARABLE = False keeps the full-table reads, A/B).  The division
            # magics ceil(2^32 / d) are exact for token indices v with v * d < 2^32.
            grid = getattr(rope, "grid", None)
            axes = rope_axis_tables(rope, grid) if grid is not None and ROPE_SEPARABLE else None
            if axes is not None and cos.shape[0] * int(grid[1]) * int(grid[2]) < (1 << 32):
                hw, w = int(grid[1]) * int(grid[2]), int(grid[2])
                for i, t in enumerate(axes):
                    d.rope_ax[i] = _p(t)
                d.rope_hw, d.rope_w = hw, w
                d.rope_mhw, d.rope_mw = ((1 << 32) + hw - 1) // hw, ((1 << 32) + w - 1) // w
    if aux is not None:
        _chk(aux, "aux")
        if epilogue not in (N.EPI_BIAS_GELU, N.EPI_BIAS_QKNORM_ROPE):
            raise ValueError("aux output: EPI_BIAS_GELU or EPI_BIAS_QKNORM_ROPE only")
        width = Ntot if epilogue == N.EPI_BIAS_GELU else 2 * nseg
        if aux.numel() // aux.shape[-1] != M or aux.shape[-1] < width:
            raise ValueError(f"aux must hold {M} rows of >= {width} columns, got {tuple(aux.shape)}")
        d.aux, d.ld_aux = _p(aux), _rowmajor(aux, "aux")
    if epilogue == N.EPI_GELU_BWD:
        _chk(z, "z")
        if z.numel() // z.shape[-1] != M or z.shape[-1] != Ntot:
            raise ValueError(f"z must be [{M}, {Ntot}], got {tuple(z.shape)}")
        d.R, d.ldr = _p(z), _rowmajor(z, "z")
    if epilogue == N.EPI_BIAS_ADDROWS:
        _chk(addrows, "addrows")
        d.addrows, d.addrows_ld, d.addrows_offset = _p(addrows), _rowmajor(addrows, "addrows"), addrows_offset
    if a_tail is not None:
        k0, offs = a_tail
        if len(offs) != len(weights) or not 0 < k0 < K or a.shape[-1] < K + max(offs):
            raise ValueError(f"a_tail {a_tail} does not fit a of width {a.shape[-1]} and K={K}")
        d.a_tail_k = int(k0)
        for i, o in enumerate(offs):
            d.a_tail_off[i] = int(o)
    L = N.lib()
    # split-K for GEMMs too small to fill the chip (e.g. T5 at 2 x 226 rows): fp32 partials from the caching
    # allocator, so they are ordered on the launch stream
    nb = L.vp_gemm_bf16_workspace_bytes(C.byref(d))
    ev = _t0("gemm")
    if nb > 0:
        ws = torch.empty(nb, device=out.device, dtype=torch.uint8)
        N.check(L.vp_gemm_bf16_ws(C.byref(d), _p(ws), nb, _stream()), "vp_gemm_bf16_ws")
    else:
        N.check(L.vp_gemm_bf16(C.byref(d), _stream()), "vp_gemm_bf16")
    _t1("gemm", ev)
    return out


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], out: Optional[torch.Tensor] = None,
           gelu: bool = False, scale: Optional[float] = None) -> torch.Tensor:
    """nn.Linear (+ GELU-tanh, + output scale) on the last dim of a contiguous activation."""
    x2 = x.reshape(-1, x.shape[-1])
    if out is None:
        out = torch.empty(*x.shape[:-1], weight.shape[0], device=x.device, dtype=BF16)
    epi = N.EPI_BIAS_GELU if gelu else (N.EPI_BIAS_SCALE if scale is not None and scale != 1.0 else N.EPI_BIAS)
    gemm(x2, [weight], [bias], out.view(-1, weight.shape[0]), epilogue=epi, alpha=1.0 if scale is None else scale)
    return out


# ------------------------------------------------------------------------------------------------------------------
# MX-FP8 (BASELINE config 5): e4m3 elements + one E8M0 scale per 32 K-elements, scale layout of include/vp_hip.h
# ------------------------------------------------------------------------------------------------------------------

class MXTensor:
    """rows x K MX-FP8 matrix on the device: `q` uint8 e4m3 [rows padded to a multiple of 256, K] (the GEMM streams
    whole 256-row tiles) and `scales` uint8 in the 1-KiB tile layout."""

    def __init__(self, rows: int, K: int, device, q: Optional[torch.Tensor] = None,
                 scales: Optional[torch.Tensor] = None, zero: bool = True):
        """zero=False leaves the padding rows uninitialised (they only feed GEMM rows that are never stored)."""
        if K % 128:
            raise ValueError(f"MX-FP8 needs K % 128 == 0, got {K}")
        self.rows, self.K = rows, K
        pad = (rows + 255) // 256 * 256
        alloc = torch.zeros if zero else torch.empty
        self.q = alloc(pad, K, device=device, dtype=torch.uint8) if q is None else q
        nb = N.lib().vp_mx_scale_bytes(rows, K)
        self.scales = alloc(nb, device=device, dtype=torch.uint8) if scales is None else scales

    def __repr__(self):
        return f"MXTensor(rows={self.rows}, K={self.K})"


def mx_quantize(x: torch.Tensor, out: Optional["MXTensor"] = None) -> "MXTensor":
    """bf16 [..., K] (last dim contiguous) -> MXTensor [rows, K]."""
    _chk(x, "x")
    x2 = x.reshape(-1, x.shape[-1])
    rows, Kk = x2.shape
    out = MXTensor(rows, Kk, x.device) if out is None else out
    N.check(N.lib().vp_mx_quantize_bf16(_p(x2), _rowmajor(x2, "x"), _p(out.q), out.q.stride(0), _p(out.scales), rows,
                                        Kk, _stream()), "vp_mx_quantize_bf16")
    return out


def gemm_mx(a: "MXTensor", weights: Sequence["MXTensor"], biases: Sequence[Optional[torch.Tensor]], out, *,
            epilogue: int = N.EPI_BIAS, alpha: float = 1.0, resid: Optional[torch.Tensor] = None,
            mod: Optional[torch.Tensor] = None, gate_chunk: int = 2, gate_text_chunk: int = 5,
            tokens_per_batch: int = 1, text_len: int = 0, inject: Optional[torch.Tensor] = None,
            inject_mask: Optional[torch.Tensor] = None):
    """out = epilogue(a @ cat(weights).T) on the block-scaled fp8 MFMA.  `out` is a bf16 [M, N] tensor, or an
    MXTensor for EPI_BIAS_GELU_MXFP8 (the FF1 -> FF2 hand-off stays in fp8)."""
    Kk = a.K
    for w in weights:
        if w.K != Kk or w.rows != weights[0].rows:
            raise ValueError("weight segments must share K and rows")
    nseg = weights[0].rows
    Ntot = nseg * len(weights)
    x = N.GemmMxDesc()
    d = x.base
    d.M, d.N, d.K, d.epilogue = a.rows, Ntot, Kk, epilogue
    d.A, d.lda = _p(a.q), a.q.stride(0)
    x.a_scale = _p(a.scales)
    for i, w in enumerate(weights):
        d.W[i] = _p(w.q)
        x.w_scale[i] = _p(w.scales)
        b = biases[i] if biases is not None and i < len(biases) else None
        if b is not None:
            _chk(b, "bias")
        d.bias[i] = _p(b)
    d.n_seg = nseg
    d.rows_per_group = a.rows
    d.alpha = alpha
    if epilogue == N.EPI_BIAS_GELU_MXFP8:
        if not isinstance(out, MXTensor) or out.K != Ntot or out.rows != a.rows:
            raise ValueError("EPI_BIAS_GELU_MXFP8 writes an MXTensor [M, N]")
        d.C, d.ldc = _p(out.q), out.q.stride(0)
        x.c_scale = _p(out.scales)
    else:
        _chk(out, "out")
        d.C, d.ldc = _p(out), _rowmajor(out, "out")
    if epilogue == N.EPI_GATED:
        _chk(resid, "resid")
        _chk(mod, "mod")
        d.R, d.ldr = _p(resid), _rowmajor(resid, "resid")
        d.gate = mod.data_ptr() + gate_chunk * Ntot * mod.element_size()
        d.gate_text = mod.data_ptr() + gate_text_chunk * Ntot * mod.element_size()
        d.gate_bstride = mod.stride(0)
        d.tokens_per_batch, d.text_len = tokens_per_batch, text_len
        if inject is not None:
            _chk(inject, "inject")
            d.inject, d.inject_ld, d.inject_bstride = _p(inject), inject.stride(1), inject.stride(0)
            if inject_mask is not None:
                _chk(inject_mask, "inject_mask", torch.uint8)
                d.inject_mask = _p(inject_mask)
                d.inject_mask_bstride = inject_mask.stride(0)
    ev = _t0("gemm_mx")
    N.check(N.lib().vp_gemm_mx_fp8(C.byref(x), _stream()), "vp_gemm_mx_fp8")
    _t1("gemm_mx", ev)
    return out


def adaln_modulate_mx(x: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, mod: torch.Tensor, text_len: int,
                      eps: float, out: Optional["MXTensor"] = None) -> "MXTensor":
    """AdaLN-Zero modulate writing MX-FP8 rows (the fp8 FeedForward's input)."""
    _chk(x, "x")
    if not x.is_contiguous():
        raise ValueError("x must be contiguous [B, N, D]")
    B, Ntok, D = x.shape
    out = MXTensor(B * Ntok, D, x.device, zero=False) if out is None else out
    N.check(N.lib().vp_adaln_modulate_mx_fp8(_p(x), _p(out.q), _p(out.scales), B, Ntok, D, text_len, _p(ln_w),
                                             _p(ln_b), eps, _p(mod), mod.stride(0), _stream()),
            "vp_adaln_modulate_mx_fp8")
    return out


def mx_mfma_probe(A: torch.Tensor, B: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """One block-scaled MFMA (layout self-test): A, B uint8 e4m3 [16, 128]; sa, sb uint8 [64] (lane scales)."""
    Cm = torch.empty(16, 16, device=A.device, dtype=torch.float32)
    N.check(N.lib().vp_mx_mfma_probe(_p(A), _p(B), _p(sa), _p(sb), _p(Cm), _stream()), "vp_mx_mfma_probe")
    return Cm


# ------------------------------------------------------------------------------------------------------------------
# attention
# ------------------------------------------------------------------------------------------------------------------

def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: torch.Tensor, heads: int, *,
              k2: Optional[torch.Tensor] = None, v2: Optional[torch.Tensor] = None, scale: float = 0.125,
              out_scale: float = 1.0, accumulate: bool = False, bounded_scores: bool = False,
              lse: Optional[torch.Tensor] = None, k2_full: Optional[torch.Tensor] = None,
              k2_len: Optional[torch.Tensor] = None, l_extra: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q, k, v, out: [B, N, heads*64] views (last dim contiguous, any row/batch stride); k2 / v2: an optional second
    K/V segment of the same form.  The native side sees only pointers and strides, so every extent is checked here.
    lse: optional fp32 [B, heads, Nq] receiving the softmax statistics the backward needs.  k2_full: optional int32
    [B] (device): segment-2 keys at or past k2_full[b] have zero values (v2 rows there must be zero) and enter only the
    row sums (include/vp_hip.h vp_attn_desc.k2_full).  k2_len: optional int32 [B] (device): only the first
    min(k2_len[b], Nk2) keys of segment 2 exist for batch row b.  l_extra: optional fp32 [B, heads, Nq]: log2 of
    extra row-sum mass per query in score units (scale * log2 e * q.k), keys with zero values outside the segments
    (the resample processor's null keys, null_key_mass)."""
    segs = [(q, "q"), (k, "k"), (v, "v"), (out, "out")]
    if (k2 is None) != (v2 is None):
        raise ValueError("k2 and v2 must be given together")
    if k2 is not None:
        segs += [(k2, "k2"), (v2, "v2")]
    for t, n in segs:
        _chk(t, n)
        if t.dim() != 3 or t.stride(-1) != 1 or t.shape[-1] != heads * 64:
            raise ValueError(f"{n} must be [B, N, heads*64] with a contiguous last dim, got {tuple(t.shape)}")
        if t.shape[0] != q.shape[0]:
            raise ValueError(f"{n} batch {t.shape[0]} != q batch {q.shape[0]}")
    if out.shape[1] != q.shape[1]:
        raise ValueError(f"out length {out.shape[1]} != q length {q.shape[1]}")
    if k.shape[1] != v.shape[1] or k.shape[1] == 0:
        raise ValueError("k and v lengths differ (or are empty)")
    if k2 is not None and (k2.shape[1] != v2.shape[1] or k2.shape[1] == 0):
        raise ValueError("k2 and v2 lengths differ (or are empty)")
    d = N.AttnDesc()
    d.B, d.H, d.Nq, d.head_dim = q.shape[0], heads, q.shape[1], 64
    d.Q, d.q_sb, d.q_sn = _p(q), q.stride(0), q.stride(1)
    d.K, d.V = _p(k), _p(v)
    d.k_sb, d.k_sn, d.v_sb, d.v_sn = k.stride(0), k.stride(1), v.stride(0), v.stride(1)
    d.Nk = k.shape[1]
    if k2 is not None:
        d.K2, d.V2 = _p(k2), _p(v2)
        d.k2_sb, d.k2_sn, d.v2_sb, d.v2_sn = k2.stride(0), k2.stride(1), v2.stride(0), v2.stride(1)
        d.Nk2 = k2.shape[1]
    if k2_full is not None:
        if k2 is None:
            raise ValueError("k2_full needs a second segment")
        _chk(k2_full, "k2_full", torch.int32)
        if tuple(k2_full.shape) != (q.shape[0],) or not k2_full.is_contiguous():
            raise ValueError(f"k2_full must be contiguous int32 [{q.shape[0]}]")
        d.k2_full = _p(k2_full)
    if k2_len is not None:
        if k2 is None:
            raise ValueError("k2_len needs a second segment")
        _chk(k2_len, "k2_len", torch.int32)
        if tuple(k2_len.shape) != (q.shape[0],) or not k2_len.is_contiguous():
            raise ValueError(f"k2_len must be contiguous int32 [{q.shape[0]}]")
        d.k2_len = _p(k2_len)
    if l_extra is not None:
        _chk(l_extra, "l_extra", torch.float32)
        if tuple(l_extra.shape) != (q.shape[0], heads, q.shape[1]) or not l_extra.is_contiguous():
            raise ValueError(f"l_extra must be contiguous fp32 [{q.shape[0]}, {heads}, {q.shape[1]}]")
        d.l_extra = _p(l_extra)
    d.O, d.o_sb, d.o_sn = _p(out), out.stride(0), out.stride(1)
    d.scale, d.out_scale, d.accumulate = scale, out_scale, int(accumulate)
    if lse is not None:
        _chk(lse, "lse", torch.float32)
        if lse.shape != (q.shape[0], heads, q.shape[1]) or not lse.is_contiguous():
            raise ValueError("lse must be contiguous fp32 [B, heads, Nq]")
        d.lse = _p(lse)
    # bounded_scores: the caller guarantees |scale * q.k| * log2 e <= SCORE_BOUND_LOG2 (score_bound_log2)
    d.flags = ATTN_BOUNDED_SCORES if bounded_scores else 0
    L = N.lib()
    nb = L.vp_attention_workspace_bytes(C.byref(d))
    if nb < 0:
        raise ValueError("invalid attention descriptor")
    # tail-split partials: taken from the caching allocator per call, so they are ordered on the launch stream
    # (a caller may run attention on several streams at once)
    ws = torch.empty(nb, device=q.device, dtype=torch.uint8) if nb > 0 else None
    ev = _t0("attention")
    N.check(L.vp_attention_fwd_bf16_ws(C.byref(d), _p(ws), nb, _stream()), "vp_attention_fwd_bf16_ws")
    _t1("attention", ev)
    return out


def attention_variant_built(name: str) -> bool:
    """Is the attention kernel variant `name` (a value of VP_ATTN_BOUNDED_MODE / VP_ATTN_UNBOUNDED_MODE) in the
    library (host-only query)?  The rejected A/B variants of rounds 1-5 were pruned in round 6."""
    return bool(N.lib().vp_attention_variant_built(name.encode()))


def set_knob(name: str, value: Optional[str]) -> Optional[str]:
    """Switch one of the library's A/B knobs (include/vp_hip.h vp_set_knob: kernel-variant selection, read from the
    environment once when the library loads) for the launches that follow; value None = unset.  Returns the previous
    value, so a caller can restore it."""
    if name not in N.KNOBS:
        raise ValueError(f"unknown knob {name!r} (one of {N.KNOBS})")
    L = N.lib()
    prev = N.knob_values.get(name)
    N.check(L.vp_set_knob(name.encode(), None if value is None else str(value).encode()), f"vp_set_knob({name})")
    N.knob_values[name] = None if value is None else str(value)
    return prev


class knob:
    """Context manager form of `set_knob`: `with kernels.knob("VP_GEMM_VARIANT", 11): ...`."""

    def __init__(self, name: str, value: Optional[str]):
        self.name, self.value = name, value

    def __enter__(self):
        self.prev = set_knob(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_knob(self.name, self.prev)


def gemm_variant_built(variant) -> bool:
    """Is the GEMM main loop VP_GEMM_VARIANT = variant in this library build (1, 5, 11, 13; the rejected 12 / 20 / 30
    were pruned in round 6)?"""
    return bool(N.lib().vp_gemm_variant_built(int(variant)))


def attention_bwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, o: torch.Tensor, do: torch.Tensor,
                  lse: torch.Tensor, heads: int, scale: float = 0.125, dq: Optional[torch.Tensor] = None,
                  dk: Optional[torch.Tensor] = None, dv: Optional[torch.Tensor] = None):
    """Flash-attention backward (vp_attention_bwd_bf16) of `attention(q, k, v, o, heads, lse=lse)`: returns
    (dq, dk, dv), each [B, N, heads*64] bf16 (new contiguous tensors unless given)."""
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (o, "o"), (do, "do")):
        _chk(t, n)
        if t.dim() != 3 or t.stride(-1) != 1 or t.shape[-1] != heads * 64 or t.shape[0] != q.shape[0]:
            raise ValueError(f"{n} must be [B, N, heads*64] with a contiguous last dim")
    if o.shape[1] != q.shape[1] or do.shape[1] != q.shape[1] or k.shape[1] != v.shape[1]:
        raise ValueError("attention_bwd: length mismatch")
    _chk(lse, "lse", torch.float32)
    B, Nq, Nk = q.shape[0], q.shape[1], k.shape[1]
    if lse.shape != (B, heads, Nq) or not lse.is_contiguous():
        raise ValueError("lse must be contiguous fp32 [B, heads, Nq]")
    dq = torch.empty(B, Nq, heads * 64, device=q.device, dtype=BF16) if dq is None else dq
    dk = torch.empty(B, Nk, heads * 64, device=q.device, dtype=BF16) if dk is None else dk
    dv = torch.empty(B, Nk, heads * 64, device=q.device, dtype=BF16) if dv is None else dv
    for t, n, L in ((dq, "dq", Nq), (dk, "dk", Nk), (dv, "dv", Nk)):
        _chk(t, n)
        if t.shape != (B, L, heads * 64) or t.stride(-1) != 1:
            raise ValueError(f"{n} must be [B, {L}, heads*64]")
    delta = torch.empty(B, heads, Nq, device=q.device, dtype=torch.float32)
    d = N.AttnBwdDesc()
    d.B, d.H, d.Nq, d.Nk, d.head_dim = B, heads, Nq, Nk, 64
    for name, t in (("q", q), ("k", k), ("v", v), ("o", o), ("do", do), ("dq", dq), ("dk", dk), ("dv", dv)):
        setattr(d, {"q": "Q", "k": "K", "v": "V", "o": "O", "do": "dO", "dq": "dQ", "dk": "dK", "dv": "dV"}[name],
                _p(t))
        setattr(d, f"{name}_sb", t.stride(0))
        setattr(d, f"{name}_sn", t.stride(1))
    d.lse, d.delta, d.scale = _p(lse), _p(delta), scale
    L = N.lib()
    nb = L.vp_attention_bwd_workspace_bytes(C.byref(d))
    if nb < 0:
        raise ValueError("invalid attention backward descriptor")
    # the grid-tail pieces' fp32 sums (caching allocator, ordered on the launch stream like the forward's)
    ws = torch.empty(nb, device=q.device, dtype=torch.uint8) if nb > 0 else None
    ev = _t0("attention_bwd")
    N.check(L.vp_attention_bwd_bf16_ws(C.byref(d), _p(ws), nb, _stream()), "vp_attention_bwd_bf16_ws")
    _t1("attention_bwd", ev)
    return dq, dk, dv


# ---- fp8 attention (BASELINE config 5; formats in include/vp_hip.h) ----

LOG2E = 1.4426950408889634
ATTN_BOUNDED_SCORES = 1      # include/vp_hip.h VP_ATTN_BOUNDED_SCORES
SCORE_BOUND_LOG2 = 60.0      # include/vp_hip.h VP_ATTN_SCORE_BOUND


def ln_output_norm_bound(ln) -> float:
    """Upper bound of the L2 norm of any output row of LayerNorm(64) `ln` (then rotated by RoPE, which preserves
    it): x_hat has sum(x_hat^2) = 64 var / (var + eps) < 64, so |gamma * x_hat + beta| <= 8 max|gamma| + |beta|_2."""
    w = ln.weight.detach().float()
    b = ln.bias.detach().float()
    return float(8.0 * w.abs().max() + b.norm())


def score_bound_log2(norm_q, norm_k, scale: float) -> float:
    """Bound of |scale * q.k| * log2 e over every query / key pair of a CogVideoX attention (q, k the outputs of
    norm_q / norm_k + RoPE, attention_processor.py:2143-2154), with 3 % for the bf16 roundings of q, k and of the
    pre-scaled Q fragments."""
    return ln_output_norm_bound(norm_q) * ln_output_norm_bound(norm_k) * scale * LOG2E * 1.03


def mx_mfma_probe32(A: torch.Tensor, B: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """One v_mfma_scale_f32_32x32x64_f8f6f4 (layout self-test): A, B uint8 e4m3 [32, 64]; sa, sb uint8 [64]."""
    Cm = torch.empty(32, 32, device=A.device, dtype=torch.float32)
    N.check(N.lib().vp_mx_mfma_probe32(_p(A), _p(B), _p(sa), _p(sb), _p(Cm), _stream()), "vp_mx_mfma_probe32")
    return Cm


def qk_fp8_exponent(ln_w: torch.Tensor, ln_b: torch.Tensor, mul: float = 1.0) -> int:
    """Largest a with |x| * mul * 2^a <= 448 for every output x of LN(64) + RoPE with this affine: after the
    LayerNorm |x_hat| <= sqrt(63), so |x| <= sqrt(63) max|gamma| + max|beta|, and RoPE mixes pairs (x sqrt 2)."""
    import math
    bound = math.sqrt(2.0) * (math.sqrt(63.0) * float(ln_w.float().abs().max()) + float(ln_b.float().abs().max()))
    bound = max(bound * mul, 1e-30)
    return int(math.floor(math.log2(448.0 / bound)))


def head_norm_rope_fp8(x_in: torch.Tensor, heads: int, text_len: int, ln_w, ln_b, eps: float, rope, out_mul: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LN(64) + RoPE as `head_norm_rope`, written as e4m3 (x * out_mul) into uint8 [B, N, heads*64]."""
    _chk(x_in, "x_in")
    B, Ntok, _ = x_in.shape
    if out is None:
        out = torch.empty(B, Ntok, heads * 64, device=x_in.device, dtype=torch.uint8)
    cos = sin = None
    if rope is not None:
        cos, sin = rope
        _chk(cos, "cos", torch.float32)
        _chk(sin, "sin", torch.float32)
        if cos.shape[0] != Ntok - text_len or cos.shape[1] != 64 or not cos.is_contiguous() or not sin.is_contiguous():
            raise ValueError(f"rope tables must be fp32 [{Ntok - text_len}, 64], got {tuple(cos.shape)}")
    N.check(N.lib().vp_head_norm_rope_fp8(_p(x_in), x_in.stride(1), x_in.stride(0), _p(out), out.stride(1),
                                          out.stride(0), B, Ntok, heads, text_len, _p(ln_w), _p(ln_b), eps, _p(cos),
                                          _p(sin), out_mul, _stream()), "vp_head_norm_rope_fp8")
    return out


class VPacked:
    """V^T in e4m3 with the fp8 attention's tile K-slot order and per-(d, 32 keys) E8M0 scales."""

    def __init__(self, vt: torch.Tensor, vs: torch.Tensor, npad: int, n: int):
        self.vt, self.vs, self.npad, self.n = vt, vs, npad, n


def v_pack_fp8(v: torch.Tensor, heads: int) -> VPacked:
    _chk(v, "v")
    B, Nk, _ = v.shape
    npad, sbytes = C.c_int64(), C.c_int64()
    nb = N.lib().vp_v_pack_fp8_bytes(B, heads, Nk, C.byref(npad), C.byref(sbytes))
    if nb <= 0:
        raise ValueError("bad V shape")
    vt = torch.empty(nb, device=v.device, dtype=torch.uint8)
    vs = torch.empty(sbytes.value, device=v.device, dtype=torch.uint8)
    N.check(N.lib().vp_v_pack_fp8(_p(v), v.stride(0), v.stride(1), B, Nk, heads, _p(vt), _p(vs), _stream()),
            "vp_v_pack_fp8")
    return VPacked(vt, vs, npad.value, Nk)


def attention_fp8(q8: torch.Tensor, k8: torch.Tensor, vp: VPacked, out: torch.Tensor, heads: int, q_exp: int,
                  k_exp: int, out_scale: float = 1.0, accumulate: bool = False) -> torch.Tensor:
    """q8 = e4m3(q * scale * log2 e * 2^q_exp), k8 = e4m3(k * 2^k_exp): uint8 [B, N, heads*64]; out bf16."""
    for t, n in ((q8, "q8"), (k8, "k8")):
        _chk(t, n, torch.uint8)
        if t.dim() != 3 or t.stride(-1) != 1 or t.shape[-1] != heads * 64:
            raise ValueError(f"{n} must be [B, N, heads*64] uint8")
    _chk(out, "out")
    if k8.shape[1] != vp.n:
        raise ValueError("k and packed v lengths differ")
    if not (-127 <= q_exp <= 127 and -127 <= k_exp <= 127):
        raise ValueError("scale exponents out of the E8M0 range")
    dd = N.AttnFp8Desc()
    d = dd.base
    d.B, d.H, d.Nq, d.head_dim = q8.shape[0], heads, q8.shape[1], 64
    d.Q, d.q_sb, d.q_sn = _p(q8), q8.stride(0), q8.stride(1)
    d.K, d.k_sb, d.k_sn = _p(k8), k8.stride(0), k8.stride(1)
    d.V = _p(vp.vt)
    d.Nk = k8.shape[1]
    d.O, d.o_sb, d.o_sn = _p(out), out.stride(0), out.stride(1)
    d.scale, d.out_scale, d.accumulate = 1.0, out_scale, int(accumulate)
    dd.vs, dd.npad = _p(vp.vs), vp.npad
    dd.qk_scale = (127 - q_exp) | ((127 - k_exp) << 8)
    L = N.lib()
    nb = L.vp_attention_fp8_workspace_bytes(C.byref(dd))
    # the persistent kernel's ticket counters (caching allocator, ordered on the launch stream)
    ws = torch.empty(nb, device=q8.device, dtype=torch.uint8) if nb > 0 else None
    ev = _t0("attention_fp8")
    N.check(L.vp_attention_fwd_fp8_ws(C.byref(dd), _p(ws), nb, _stream()), "vp_attention_fwd_fp8_ws")
    _t1("attention_fp8", ev)
    return out


# ------------------------------------------------------------------------------------------------------------------
# norms
# ------------------------------------------------------------------------------------------------------------------

def adaln_modulate(x: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, mod: torch.Tensor, text_len: int,
                   eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _chk(x, "x")
    if not x.is_contiguous():
        raise ValueError("x must be contiguous [B, N, D]")
    B, Ntok, D = x.shape
    out = torch.empty_like(x) if out is None else out
    _chk(out, "out")
    ldy = out.stride(-2)  # [B, Ntok, D] rows (or [B*Ntok, D]) at any row stride, rows packed across the batch
    if (out.shape[-1] != D or out.stride(-1) != 1 or out.numel() != B * Ntok * D
            or (out.dim() == 3 and out.stride(0) != Ntok * ldy)):
        raise ValueError("adaln out must be [B, N, D] / [B*N, D] rows with a contiguous last dim")
    N.check(N.lib().vp_adaln_modulate_bf16(_p(x), _p(out), ldy, B, Ntok, D, text_len, _p(ln_w), _p(ln_b), eps,
                                           _p(mod), mod.stride(0), _stream()), "vp_adaln_modulate_bf16")
    return out


def head_norm_rope(x_in: torch.Tensor, x_out: torch.Tensor, heads: int, text_len: int, ln_w, ln_b, eps: float,
                   rope=None, tok_mask: Optional[torch.Tensor] = None, pre_scale: float = 1.0,
                   dst_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x_in / x_out: [B, N, heads*64] views with contiguous last dim.  dst_rows: int32 [B, N] output row of each input
    row (partition_rows_index), or None."""
    _chk(x_in, "x_in")
    _chk(x_out, "x_out")
    B, Ntok, _ = x_in.shape
    cos = sin = None
    if rope is not None:
        cos, sin = rope
        _chk(cos, "cos", torch.float32)
        _chk(sin, "sin", torch.float32)
        if cos.shape[0] != Ntok - text_len or cos.shape[1] != 64 or not cos.is_contiguous() or not sin.is_contiguous():
            raise ValueError(f"rope tables must be fp32 [{Ntok - text_len}, 64], got {tuple(cos.shape)}")
    mb = 0
    if tok_mask is not None:
        _chk(tok_mask, "tok_mask", torch.uint8)
        mb = tok_mask.stride(0)
    _chk_rows(dst_rows, B, Ntok)
    N.check(N.lib().vp_head_norm_rope_bf16(_p(x_in), x_in.stride(1), x_in.stride(0), _p(x_out), x_out.stride(1),
                                           x_out.stride(0), B, Ntok, heads, text_len, _p(ln_w), _p(ln_b), eps,
                                           _p(cos), _p(sin), _p(tok_mask), mb, pre_scale, _p(dst_rows), _stream()),
            "vp_head_norm_rope_bf16")
    return x_out


def _chk_rows(dst_rows: Optional[torch.Tensor], B: int, Ntok: int) -> None:
    if dst_rows is not None:
        _chk(dst_rows, "dst_rows", torch.int32)
        if tuple(dst_rows.shape) != (B, Ntok) or not dst_rows.is_contiguous():
            raise ValueError(f"dst_rows must be contiguous int32 [{B}, {Ntok}], got {tuple(dst_rows.shape)}")


def partition_rows_index(tok_mask: torch.Tensor):
    """Stable partition of the token mask [B, N] (uint8): (dst_rows int32 [B, N], counts int32 [B]) — set rows
    first.  Device-side counts: no host sync."""
    _chk(tok_mask, "tok_mask", torch.uint8)
    B, Ntok = tok_mask.shape
    dst = torch.empty(B, Ntok, device=tok_mask.device, dtype=torch.int32)
    cnt = torch.empty(B, device=tok_mask.device, dtype=torch.int32)
    N.check(N.lib().vp_partition_rows_index(_p(tok_mask), tok_mask.stride(0), B, Ntok, _p(dst), _p(cnt), _stream()),
            "vp_partition_rows_index")
    return dst, cnt


ROPE_SEPARABLE = True  # the fused QKV epilogue reads a separable RoPE table per axis (gemm, VP_EPI_BIAS_QKNORM_ROPE)


def rope_axis_tables(rope, grid):
    """The per-axis factors of CogVideoX's separable 3D RoPE table (embeddings.py:457-530: dims 0-15 rotate by the
    frame, 16-39 by the row, 40-63 by the column): (cos_t, sin_t [F, 16], cos_y, sin_y [Hh, 24], cos_x, sin_x
    [Ww, 24]) fp32, or None when the [F*Hh*Ww, 64] table is not exactly that product (checked element-wise on the
    device; one host sync per new table — the result is cached while the table is alive and unmodified)."""
    cos, sin = rope[0], rope[1]
    F_, Hh, Ww = (int(g) for g in grid)
    key = (cos.data_ptr(), cos._version, sin.data_ptr(), sin._version, F_, Hh, Ww)
    hit = _AXIS_CACHE.get(key)
    if hit is not None:
        return hit[2]
    res = None
    if (cos.dim() == 2 and tuple(cos.shape) == (F_ * Hh * Ww, 64) and tuple(sin.shape) == tuple(cos.shape)
            and cos.dtype == torch.float32 and sin.dtype == torch.float32):
        parts = []
        ok = True
        for tab in (cos, sin):
            g = tab.view(F_, Hh, Ww, 64)
            t_, y_, x_ = g[:, 0, 0, 0:16], g[0, :, 0, 16:40], g[0, 0, :, 40:64]
            ok = ok and torch.equal(g[..., 0:16], t_[:, None, None, :].expand(F_, Hh, Ww, 16))
            ok = ok and torch.equal(g[..., 16:40], y_[None, :, None, :].expand(F_, Hh, Ww, 24))
            ok = ok and torch.equal(g[..., 40:64], x_[None, None, :, :].expand(F_, Hh, Ww, 24))
            parts.append((t_.contiguous(), y_.contiguous(), x_.contiguous()))
        if ok:
            (ct, cy, cx), (st, sy, sx) = parts
            res = (ct, st, cy, sy, cx, sx)
    if len(_AXIS_CACHE) >= 4:
        _AXIS_CACHE.pop(next(iter(_AXIS_CACHE)))
    _AXIS_CACHE[key] = (cos, sin, res)  # (holding the tables keeps their addresses from being reused)
    return res


_AXIS_CACHE: dict = {}


def mask_null_segments(tok_mask: torch.Tensor, text_len: int, grid):
    """The null pattern of tok_mask [B, text_len + F*Hh*Ww] (uint8) for null_key_mass: (segs uint8 [B*F*Hh, 16],
    meta int32 [B*F + B]) — per (b, frame) the runs of equal consecutive rows holding null keys, and the text rows with
    mask 0 per b (resample.hip mask_null_segments_kernel).  Computed once per mask (the processor caches it)."""
    _chk(tok_mask, "tok_mask", torch.uint8)
    F_, Hh, Ww = (int(g) for g in grid)
    B, Ntok = tok_mask.shape
    if Ntok != text_len + F_ * Hh * Ww:
        raise ValueError(f"tok_mask length {Ntok} != {text_len} + {F_}*{Hh}*{Ww}")
    if tok_mask.stride(1) != 1:
        raise ValueError("tok_mask rows must be contiguous")
    segs = torch.empty(B * F_ * Hh, 16, device=tok_mask.device, dtype=torch.uint8)
    meta = torch.empty(B * F_ + B, device=tok_mask.device, dtype=torch.int32)
    N.check(N.lib().vp_mask_null_segments(_p(tok_mask), tok_mask.stride(0), B, text_len, F_, Hh, Ww, _p(segs),
                                          _p(meta), _stream()), "vp_mask_null_segments")
    return segs, meta


def null_key_mass_supported(grid) -> bool:
    F_, Hh, Ww = (int(g) for g in grid)
    return (0 < F_ <= 16 and 0 < Hh <= 64 and 0 < Ww <= 255
            and N.lib().vp_null_key_mass_lds_bytes(F_, Hh, Ww) <= 160 * 1024)


def null_key_mass(q: torch.Tensor, heads: int, text_len: int, grid, beta: torch.Tensor, axis_tables,
                  tok_mask: torch.Tensor, segments, scale: float) -> torch.Tensor:
    """log2 of the resample processor's null-key row mass per query, fp32 [B, heads, N] (the attention kernel's
    l_extra): the keys LN(0) = beta (rotated by the RoPE on video rows) of every mask-0 row, in score units
    scale * log2 e * q.k (include/vp_hip.h vp_null_key_mass).  q: the normed and rotated queries [B, N, heads*64];
    segments: mask_null_segments(tok_mask, ...)."""
    _chk(q, "q")
    _chk(beta, "beta")
    _chk(tok_mask, "tok_mask", torch.uint8)
    segs, meta = segments
    _chk(segs, "segs", torch.uint8)
    _chk(meta, "meta", torch.int32)
    F_, Hh, Ww = (int(g) for g in grid)
    B, Ntok, D = q.shape
    if D != heads * 64 or q.stride(-1) != 1 or Ntok != text_len + F_ * Hh * Ww:
        raise ValueError(f"q must be [B, {text_len} + {F_}*{Hh}*{Ww}, heads*64], got {tuple(q.shape)}")
    if tuple(beta.shape) != (64,) or not beta.is_contiguous():
        raise ValueError("beta must be contiguous bf16 [64]")
    if (tuple(tok_mask.shape) != (B, Ntok) or tok_mask.stride(1) != 1 or tuple(segs.shape) != (B * F_ * Hh, 16)
            or tuple(meta.shape) != (B * F_ + B,) or not segs.is_contiguous() or not meta.is_contiguous()):
        raise ValueError("tok_mask / segments do not match q")
    tabs = list(axis_tables)
    for t, shp in zip(tabs, ((F_, 16), (F_, 16), (Hh, 24), (Hh, 24), (Ww, 24), (Ww, 24))):
        _chk(t, "rope axis table", torch.float32)
        if tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"rope axis table must be contiguous fp32 {shp}, got {tuple(t.shape)}")
    out = torch.empty(B, heads, Ntok, device=q.device, dtype=torch.float32)
    N.check(N.lib().vp_null_key_mass(_p(q), q.stride(0), q.stride(1), B, heads, Ntok, text_len, F_, Hh, Ww, _p(beta),
                                     *[_p(t) for t in tabs], _p(tok_mask), tok_mask.stride(0), _p(segs), _p(meta),
                                     scale, _p(out), _stream()), "vp_null_key_mass")
    return out


def mask_scale_rows(x_in: torch.Tensor, out: torch.Tensor, tok_mask: torch.Tensor, scale: float,
                    dst_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    _chk(x_in, "x_in")
    _chk(out, "out")
    _chk(tok_mask, "tok_mask", torch.uint8)
    B, Ntok, D = x_in.shape
    _chk_rows(dst_rows, B, Ntok)
    N.check(N.lib().vp_mask_scale_rows_bf16(_p(x_in), x_in.stride(1), x_in.stride(0), _p(out), out.stride(1),
                                            out.stride(0), B, Ntok, D, _p(tok_mask), tok_mask.stride(0), scale,
                                            _p(dst_rows), _stream()), "vp_mask_scale_rows_bf16")
    return out


def final_norm(x: torch.Tensor, text_len: int, ln1_w, ln1_b, ln2_w, ln2_b, eps: float, mod: torch.Tensor,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _chk(x, "x")
    B, Ntok, D = x.shape
    out = torch.empty(B, Ntok - text_len, D, device=x.device, dtype=BF16) if out is None else out
    N.check(N.lib().vp_final_norm_bf16(_p(x), _p(out), B, Ntok, D, text_len, _p(ln1_w), _p(ln1_b), _p(ln2_w),
                                       _p(ln2_b), eps, _p(mod), mod.stride(0), _stream()), "vp_final_norm_bf16")
    return out


# ------------------------------------------------------------------------------------------------------------------
# conditioning path / data movement / step glue
# ------------------------------------------------------------------------------------------------------------------

ACT_NONE, ACT_SILU = 0, 1


def linear_small(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], act_in: int = ACT_NONE,
                 act_out: int = ACT_NONE, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _chk(x, "x")
    _chk(weight, "weight")
    M, K = x.shape
    Nn = weight.shape[0]
    out = torch.empty(M, Nn, device=x.device, dtype=BF16) if out is None else out
    N.check(N.lib().vp_linear_small_bf16(_p(x), x.stride(0), _p(weight), _p(bias), _p(out), out.stride(0), M, Nn, K,
                                         act_in, act_out, _stream()), "vp_linear_small_bf16")
    return out


def timestep_embedding(timesteps: torch.Tensor, dim: int, freq_shift: float = 0.0) -> torch.Tensor:
    ts = timesteps.to(dtype=torch.float32).contiguous()
    _chk(ts, "timesteps", torch.float32)
    out = torch.empty(ts.shape[0], dim, device=ts.device, dtype=BF16)
    N.check(N.lib().vp_timestep_embedding_bf16(_p(ts), _p(out), ts.shape[0], dim, freq_shift, _stream()),
            "vp_timestep_embedding_bf16")
    return out


def patchify(src1: torch.Tensor, src2: Optional[torch.Tensor], p: int, kpad: int) -> torch.Tensor:
    _chk(src1, "src1")
    B, F, C1, H, W = src1.shape
    C2 = 0
    if src2 is not None:
        _chk(src2, "src2")
        C2 = src2.shape[2]
        if src2.shape[:2] != src1.shape[:2] or src2.shape[3:] != src1.shape[3:]:
            raise ValueError("branch_cond must match hidden_states in batch/frames/height/width")
    out = torch.empty(B * F * (H // p) * (W // p), kpad, device=src1.device, dtype=BF16)
    N.check(N.lib().vp_patchify_bf16(_p(src1), C1, _p(src2), C2, _p(out), kpad, B, F, H, W, p, _stream()),
            "vp_patchify_bf16")
    return out


def patch_mask(mask: torch.Tensor, p: int) -> torch.Tensor:
    if mask.dtype not in (torch.float32, BF16):
        mask = mask.to(torch.float32)
    mask = mask.contiguous()
    B, F, _, H, W = mask.shape
    out = torch.empty(B, F * (H // p) * (W // p), device=mask.device, dtype=torch.uint8)
    N.check(N.lib().vp_patch_mask(_p(mask), int(mask.dtype == torch.float32), _p(out), B, F, H, W, p, _stream()),
            "vp_patch_mask")
    return out


def guide_rows(x: torch.Tensor, guide: torch.Tensor, tok_mask: torch.Tensor, inject: Optional[torch.Tensor] = None,
               inject_all: bool = False) -> torch.Tensor:
    """Self-guidance after a block (vp_guide_rows_bf16), in place on the video rows x [B, rows, D]: rows whose
    tok_mask is 0 take `guide`, then `inject` is added on those rows (on every row with inject_all)."""
    for t, n in ((x, "x"), (guide, "guide")) + (((inject, "inject"),) if inject is not None else ()):
        _chk(t, n)
        if t.dim() != 3 or t.stride(-1) != 1 or tuple(t.shape) != tuple(x.shape):
            raise ValueError(f"{n} must be [B, rows, D] with a contiguous last dim, shaped like x")
    _chk(tok_mask, "tok_mask", torch.uint8)
    B, R, D = x.shape
    if tok_mask.dim() != 2 or tuple(tok_mask.shape) != (B, R) or tok_mask.stride(-1) != 1:
        raise ValueError(f"tok_mask must be uint8 [{B}, {R}]")
    ld_i, bs_i = (inject.stride(1), inject.stride(0)) if inject is not None else (0, 0)
    N.check(N.lib().vp_guide_rows_bf16(_p(x), x.stride(1), x.stride(0), _p(guide), guide.stride(1), guide.stride(0),
                                       _p(inject), ld_i, bs_i, int(bool(inject_all)), _p(tok_mask), tok_mask.stride(0),
                                       B, R, D, _stream()), "vp_guide_rows_bf16")
    return x


def unpatchify(proj: torch.Tensor, B: int, F: int, Cout: int, H: int, W: int, p: int) -> torch.Tensor:
    _chk(proj, "proj")
    out = torch.empty(B, F, Cout, H, W, device=proj.device, dtype=BF16)
    N.check(N.lib().vp_unpatchify_bf16(_p(proj), proj.stride(0), _p(out), B, F, Cout, H, W, p, _stream()),
            "vp_unpatchify_bf16")
    return out


def dpm_step(desc: "N.DpmDesc") -> None:
    N.check(N.lib().vp_dpm_step_bf16(C.byref(desc), _stream()), "vp_dpm_step_bf16")


def fill_normal_(t: torch.Tensor, seed: int, mean: float = 0.0, std: float = 1.0) -> torch.Tensor:
    _chk(t, "t")
    if not t.is_contiguous():
        raise ValueError("fill target must be contiguous")
    N.check(N.lib().vp_fill_normal_bf16(_p(t), t.numel(), seed & 0xFFFFFFFFFFFFFFFF, mean, std, _stream()),
            "vp_fill_normal_bf16")
    return t


# ------------------------------------------------------------------------------------------------------------------
# CogVideoX 3D causal VAE (channels-last bf16 activations [B, T, H, W, C])
# ------------------------------------------------------------------------------------------------------------------

def conv3d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], *, Tout: int, Hout: int, Wout: int,
           tmap: Sequence[int], hist: Optional[torch.Tensor] = None, stride: int = 1, pad: int = 0, up: int = 1,
           resid: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           ldy: Optional[int] = None) -> torch.Tensor:
    """Implicit-GEMM conv (vp_conv3d_bf16): x / hist [B, T, Hin, Win, Cin] channels-last, w [Cout, kt, kh, kw, Cin];
    tmap[t + dt] = x frame (>= 0) or -1 - hist frame for output frame t and temporal tap dt."""
    _chk(x, "x")
    _chk(w, "w")
    if not x.is_contiguous() or not w.is_contiguous() or x.dim() != 5 or w.dim() != 5:
        raise ValueError("conv3d: x [B,T,H,W,C] and w [Cout,kt,kh,kw,Cin] must be contiguous")
    B, xf, Hin, Win, Cin = x.shape
    Cout, kt, kh, kw, wc = w.shape
    if wc != Cin:
        raise ValueError(f"conv3d: weight Cin {wc} != activation channels {Cin}")
    if len(tmap) != Tout + kt - 1 or len(tmap) > N.CONV_MAX_T:
        raise ValueError("conv3d: tmap must have Tout + kt - 1 <= CONV_MAX_T entries")
    ldy = ldy if ldy is not None else (Cout + 7) // 8 * 8
    if out is None:
        out = torch.empty(B, Tout, Hout, Wout, ldy, device=x.device, dtype=BF16)
    elif out.shape != (B, Tout, Hout, Wout, ldy) or not out.is_contiguous():
        raise ValueError("conv3d: out has the wrong shape")
    d = N.Conv3dDesc()
    d.B, d.Cin, d.Cout, d.Tout, d.Hout, d.Wout, d.Hin, d.Win = B, Cin, Cout, Tout, Hout, Wout, Hin, Win
    d.kt, d.kh, d.kw, d.sh, d.sw, d.ph, d.pw, d.uh, d.uw = kt, kh, kw, stride, stride, pad, pad, up, up
    d.x_frames = xf
    if hist is not None:
        _chk(hist, "hist")
        if not hist.is_contiguous() or hist.shape[0] != B or hist.shape[2:] != x.shape[2:]:
            raise ValueError("conv3d: hist must be [B, Th, Hin, Win, Cin] contiguous")
        d.hist, d.hist_frames = _p(hist), hist.shape[1]
    for i, v in enumerate(tmap):
        d.tmap[i] = int(v)
    d.x, d.w, d.y, d.ldy = _p(x), _p(w), _p(out), ldy
    if bias is not None:
        _chk(bias, "bias")
        d.bias = _p(bias)
    if resid is not None:
        _chk(resid, "resid")
        if resid.shape[:4] != out.shape[:4] or not resid.is_contiguous():
            raise ValueError("conv3d: resid must be [B, Tout, Hout, Wout, ldr] contiguous")
        d.resid, d.ldr = _p(resid), resid.shape[4]
    ev = _t0("conv3d")
    N.check(N.lib().vp_conv3d_bf16(C.byref(d), _stream()), "vp_conv3d_bf16")
    _t1("conv3d", ev)
    return out


def group_norm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int, eps: float, *,
               silu: bool = False, mod: Optional[torch.Tensor] = None, tzmap: Optional[Sequence[int]] = None,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(GroupNorm(x) [* mod_y + mod_b]) over channels-last x [B, T, H, W, C] (vp_group_norm_stats + _apply);
    mod [B, Tz, Hz, Wz, 2C] = conv_y(z) | conv_b(z) at latent resolution, tzmap[t] = its frame for frame t."""
    _chk(x, "x")
    _chk(gamma, "gamma")
    _chk(beta, "beta")
    if not x.is_contiguous() or x.dim() != 5:
        raise ValueError("group_norm: x must be contiguous [B, T, H, W, C]")
    B, T, H, W, Cc = x.shape
    L = N.lib()
    part = torch.empty(L.vp_group_norm_workspace_floats(B, groups), device=x.device, dtype=torch.float32)
    stats = torch.empty(B, groups, 2, device=x.device, dtype=torch.float32)
    N.check(L.vp_group_norm_stats(_p(x), B, T * H * W, Cc, groups, eps, _p(part), _p(stats), _stream()),
            "vp_group_norm_stats")
    out = torch.empty_like(x) if out is None else out
    tz = None
    Tz = Hz = Wz = 0
    if mod is not None:
        _chk(mod, "mod")
        if not mod.is_contiguous() or mod.shape[0] != B or mod.shape[4] != 2 * Cc or tzmap is None or len(tzmap) != T:
            raise ValueError("group_norm: mod must be [B, Tz, Hz, Wz, 2C] with a tzmap of T entries")
        Tz, Hz, Wz = mod.shape[1:4]
        tz = (N.i32 * T)(*[int(v) for v in tzmap])
    N.check(L.vp_group_norm_apply_bf16(_p(x), _p(out), B, T, H, W, Cc, groups, _p(stats), _p(gamma), _p(beta),
                                       _p(mod), Tz, Hz, Wz, tz, int(silu), _stream()), "vp_group_norm_apply_bf16")
    return out


def time_pool2(x: torch.Tensor) -> torch.Tensor:
    _chk(x, "x")
    B, T, H, W, Cc = x.shape
    T2 = (T + 1) // 2 if T % 2 else T // 2
    out = torch.empty(B, T2, H, W, Cc, device=x.device, dtype=BF16)
    N.check(N.lib().vp_time_pool2_bf16(_p(x.contiguous()), _p(out), B, T, H * W, Cc, _stream()), "vp_time_pool2_bf16")
    return out


def ncdhw_to_ndhwc(x: torch.Tensor, cpad: int) -> torch.Tensor:
    if not x.is_cuda or x.dtype not in (torch.float32, BF16):
        raise TypeError("ncdhw_to_ndhwc: x must be a float32 / bfloat16 device tensor")
    x = x.contiguous()
    B, Cc, T, H, W = x.shape
    out = torch.empty(B, T, H, W, cpad, device=x.device, dtype=BF16)
    N.check(N.lib().vp_ncdhw_to_ndhwc_bf16(_p(x), int(x.dtype == torch.float32), _p(out), B, Cc, T, H, W, cpad,
                                           _stream()), "vp_ncdhw_to_ndhwc_bf16")
    return out


def ndhwc_to_ncdhw(x: torch.Tensor, channels: int, c0: int = 0) -> torch.Tensor:
    _chk(x, "x")
    B, T, H, W, ld = x.shape
    out = torch.empty(B, channels, T, H, W, device=x.device, dtype=BF16)
    N.check(N.lib().vp_ndhwc_to_ncdhw_bf16(_p(x.contiguous()), ld, _p(out), B, channels, T, H, W, c0, _stream()),
            "vp_ndhwc_to_ncdhw_bf16")
    return out


def latent_dist(params: torch.Tensor, latent_channels: int, noise: Optional[torch.Tensor] = None):
    """(mean, logvar[, sample]) NCDHW bf16 from the encoder output rows [B, T, H, W, >= 2L]."""
    _chk(params, "params")
    B, T, H, W, ld = params.shape
    L = latent_channels
    mean = torch.empty(B, L, T, H, W, device=params.device, dtype=BF16)
    logvar = torch.empty_like(mean)
    sample = None
    if noise is not None:
        _chk(noise, "noise")
        if tuple(noise.shape) != tuple(mean.shape):
            raise ValueError("latent_dist: noise must be [B, L, T, H, W]")
        noise = noise.contiguous()
        sample = torch.empty_like(mean)
    N.check(N.lib().vp_latent_dist_bf16(_p(params.contiguous()), ld, _p(mean), _p(logvar), _p(noise), _p(sample), B, L,
                                        T, H, W, _stream()), "vp_latent_dist_bf16")
    return (mean, logvar) if noise is None else (mean, logvar, sample)


def tile_blend_(a: torch.Tensor, b: torch.Tensor, axis: int, extent: int) -> torch.Tensor:
    """In place on b (channels-last [B, T, H, W, C]): the reference's blend_v (axis 0) / blend_h (axis 1)."""
    _chk(a, "a")
    _chk(b, "b")
    if not a.is_contiguous() or not b.is_contiguous():
        raise ValueError("tile_blend_: tiles must be contiguous")
    B, T, Ha, Wa, Cc = a.shape
    Hb, Wb = b.shape[2], b.shape[3]
    if b.shape[0] != B or b.shape[1] != T or b.shape[4] != Cc:
        raise ValueError("tile_blend_: tiles differ in batch / frames / channels")
    N.check(N.lib().vp_tile_blend_bf16(_p(a), _p(b), B, T, Ha, Wa, Hb, Wb, Cc, axis, extent, _stream()),
            "vp_tile_blend_bf16")
    return b


# ------------------------------------------------------------------------------------------------------------------
# T5 encoder pieces
# ------------------------------------------------------------------------------------------------------------------

def embedding_gather(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    _chk(table, "table")
    if not ids.is_cuda or ids.dtype != torch.int64:
        raise TypeError("ids must be an int64 device tensor")
    ids = ids.contiguous()
    vocab, D = table.shape
    out = torch.empty(ids.numel(), D, device=table.device, dtype=BF16)
    N.check(N.lib().vp_embedding_gather_bf16(_p(table), _p(ids), _p(out), ids.numel(), D, vocab, _stream()),
            "vp_embedding_gather_bf16")
    return out


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _chk(x, "x")
    _chk(w, "w")
    D = x.shape[-1]
    if not x.is_contiguous() or w.numel() != D:
        raise ValueError("rms_norm: x must be contiguous with the weight's width")
    out = torch.empty_like(x) if out is None else out
    N.check(N.lib().vp_rms_norm_bf16(_p(x), _p(w), _p(out), x.numel() // D, D, eps, _stream()), "vp_rms_norm_bf16")
    return out


def mul(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _chk(a, "a")
    _chk(b, "b")
    if a.shape != b.shape or not a.is_contiguous() or not b.is_contiguous():
        raise ValueError("mul: contiguous operands of one shape")
    out = torch.empty_like(a) if out is None else out
    N.check(N.lib().vp_mul_bf16(_p(a), _p(b), _p(out), a.numel(), _stream()), "vp_mul_bf16")
    return out


def t5_attention(qkv: torch.Tensor, B: int, L: int, H: int, bias_table: torch.Tensor, buckets: torch.Tensor,
                 mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qkv [B * L, 3 * H * 64] (q | k | v) -> [B * L, H * 64]."""
    _chk(qkv, "qkv")
    _chk(bias_table, "bias_table")
    _chk(buckets, "buckets", torch.int32)
    inner = H * 64
    if qkv.shape != (B * L, 3 * inner) or buckets.shape != (L, L) or bias_table.shape[1] != H:
        raise ValueError("t5_attention: shape mismatch")
    if mask is not None:
        _chk(mask, "mask", torch.int64)
        if mask.shape != (B, L):
            raise ValueError("t5_attention: mask must be [B, L]")
        mask = mask.contiguous()
    out = torch.empty(B * L, inner, device=qkv.device, dtype=BF16)
    N.check(N.lib().vp_t5_attention_bf16(_p(qkv), qkv.stride(0), inner, B, L, H, _p(bias_table.contiguous()),
                                         _p(buckets.contiguous()), _p(mask), _p(out), out.stride(0), _stream()),
            "vp_t5_attention_bf16")
    return out


# ------------------------------------------------------------------------------------------------------------------
# pixel-space glue of the pipeline's VAE stage
# ------------------------------------------------------------------------------------------------------------------

def scale_bf16(x: torch.Tensor, s: float) -> torch.Tensor:
    _chk(x, "x")
    x = x.contiguous()
    out = torch.empty_like(x)
    N.check(N.lib().vp_scale_bf16(_p(x), _p(out), x.numel(), s, _stream()), "vp_scale_bf16")
    return out


def mask_video(video: torch.Tensor, mask: torch.Tensor, keep_above: bool = False) -> torch.Tensor:
    """bf16(video * (mask < 0.5)) — or (mask >= 0.5) for keep_above — video [B, C, F, H, W] fp32/bf16, mask
    [B, 1, F, H, W] fp32."""
    if not video.is_cuda or video.dtype not in (torch.float32, BF16):
        raise TypeError("mask_video: video must be a float32 / bfloat16 device tensor")
    _chk(mask, "mask", torch.float32)
    video, mask = video.contiguous(), mask.contiguous()
    B, Cc = video.shape[:2]
    P = video[0, 0].numel()
    if mask.shape[0] != B or mask.shape[1] != 1 or mask[0, 0].numel() != P:
        raise ValueError("mask_video: mask must be [B, 1, F, H, W] matching the video")
    out = torch.empty(video.shape, device=video.device, dtype=BF16)
    N.check(N.lib().vp_mask_video_bf16(_p(video), int(video.dtype == torch.float32), _p(mask), int(keep_above),
                                       _p(out), B, Cc, P, _stream()), "vp_mask_video_bf16")
    return out


def nearest_resize_3d(x: torch.Tensor, size) -> torch.Tensor:
    _chk(x, "x", torch.float32)
    x = x.contiguous()
    B, Cc, T, H, W = x.shape
    t, h, w = size
    out = torch.empty(B, Cc, t, h, w, device=x.device, dtype=BF16)
    N.check(N.lib().vp_nearest_resize3d_bf16(_p(x), _p(out), B * Cc, T, H, W, t, h, w, _stream()),
            "vp_nearest_resize3d_bf16")
    return out


def denormalize_bf16(x: torch.Tensor) -> torch.Tensor:
    _chk(x, "x")
    x = x.contiguous()
    out = torch.empty_like(x)
    N.check(N.lib().vp_denormalize_bf16(_p(x), _p(out), x.numel(), _stream()), "vp_denormalize_bf16")
    return out


# ------------------------------------------------------------------------------------------------------------------
# training backward (csrc/backward.hip)
# ------------------------------------------------------------------------------------------------------------------

def transpose(x: torch.Tensor, out: Optional[torch.Tensor] = None, pad_to: int = 1) -> torch.Tensor:
    """x: [R, C] or [nb, R, C] (contiguous last dim, any row / batch stride) -> [C, nb*R rounded up to pad_to]
    (batch b in columns b*R ..); the pad columns are zero."""
    _chk(x, "x")
    x3 = x if x.dim() == 3 else x.unsqueeze(0)
    nb, R, Cc = x3.shape
    if x3.stride(-1) != 1:
        raise ValueError("x must have a contiguous last dimension")
    cols = nb * R
    colp = (cols + pad_to - 1) // pad_to * pad_to
    if out is None:
        out = torch.empty(Cc, colp, device=x.device, dtype=BF16)
    _chk(out, "out")
    if out.shape[0] != Cc or out.shape[1] < cols or out.stride(1) != 1:
        raise ValueError(f"transpose out must be [{Cc}, >= {cols}]")
    if out.shape[1] > cols:
        out[:, cols:].zero_()
    N.check(N.lib().vp_transpose_bf16(_p(x3), x3.stride(1), x3.stride(0) if nb > 1 else 0, _p(out), out.stride(0), R,
                                      R, Cc, nb, _stream()), "vp_transpose_bf16")
    return out


def colsum(a: torch.Tensor, b: Optional[torch.Tensor] = None, *, tokens_per_batch: Optional[int] = None,
           text_len: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Column sums of a (* b) over rows, split per (batch, text/video): fp32 [rows / tokens_per_batch, 2, cols]
    (index 1 = the text rows).  tokens_per_batch=None sums every row into [1, 2, cols][0, 0]."""
    _chk(a, "a")
    rows, cols = a.shape[0], a.shape[-1]
    if a.dim() != 2:
        a = a.reshape(-1, cols)
        rows = a.shape[0]
    ntok = rows if tokens_per_batch is None else tokens_per_batch
    nb = rows // ntok
    if out is None:
        out = torch.zeros(nb, 2, cols, device=a.device, dtype=torch.float32)
    _chk(out, "out", torch.float32)
    ldb = 0
    if b is not None:
        _chk(b, "b")
        b = b.reshape(-1, cols) if b.dim() != 2 else b
        if b.shape[0] != rows:
            raise ValueError("colsum: a and b row counts differ")
        ldb = _rowmajor(b, "b")
    N.check(N.lib().vp_colsum_bf16(_p(a), _rowmajor(a, "a"), _p(b), ldb, rows, cols, ntok, text_len, _p(out),
                                   _stream()), "vp_colsum_bf16")
    return out


def adaln_bwd(x: torch.Tensor, dy: torch.Tensor, dx: torch.Tensor, text_len: int, ln_w, ln_b, eps: float,
              mod: torch.Tensor, chunks=(0, 1, 3, 4), n_out=None, dn_out=None, xhat_out=None) -> torch.Tensor:
    """dx += LN'(dy (1 + scale) w) for y = bf16(bf16(LN(x) w + b) (1 + scale) + shift); x, dy, dx contiguous
    [B, Ntok, D]; chunks = (shift_v, scale_v, shift_t, scale_t) of mod [B, *]."""
    for t, n in ((x, "x"), (dy, "dy"), (dx, "dx")):
        _chk(t, n)
        if not t.is_contiguous() or t.shape != x.shape:
            raise ValueError(f"{n} must be contiguous {tuple(x.shape)}")
    B, Ntok, D = x.shape
    for t in (n_out, dn_out, xhat_out):
        if t is not None and (t.shape != x.shape or not t.is_contiguous()):
            raise ValueError("adaln_bwd outputs must be contiguous like x")
    if mod.shape[0] != B or mod.stride(-1) != 1:
        raise ValueError("mod must be [B, *] with a contiguous last dim")
    N.check(N.lib().vp_adaln_bwd_bf16(_p(x), _p(dy), _p(dx), B, Ntok, D, text_len, _p(ln_w), _p(ln_b), eps, _p(mod),
                                      mod.stride(0), *chunks, _p(n_out), _p(dn_out), _p(xhat_out), _stream()),
            "vp_adaln_bwd_bf16")
    return dx


def rowscale(x: torch.Tensor, out: torch.Tensor, tokens_per_batch: int, text_len: int, mod: torch.Tensor,
             chunk_v: int, chunk_t: int) -> torch.Tensor:
    """out = bf16(x * mod[b, chunk]) per row (video / text chunk); x, out 2-D [rows, D] row-major views."""
    _chk(x, "x")
    _chk(out, "out")
    rows, D = x.shape
    if out.shape != x.shape:
        raise ValueError("rowscale: shape mismatch")
    N.check(N.lib().vp_rowscale_bf16(_p(x), _rowmajor(x, "x"), _p(out), _rowmajor(out, "out"), rows,
                                     tokens_per_batch, D, text_len, _p(mod), mod.stride(0), chunk_v, chunk_t,
                                     _stream()), "vp_rowscale_bf16")
    return out


def _flat(t: torch.Tensor, name: str) -> None:
    _chk(t, name)
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def gelu(z: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _flat(z, "z")
    out = torch.empty_like(z) if out is None else out
    _flat(out, "out")
    N.check(N.lib().vp_gelu_bf16(_p(z), _p(out), z.numel(), _stream()), "vp_gelu_bf16")
    return out


def gelu_bwd(dh: torch.Tensor, z: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _flat(dh, "dh")
    _flat(z, "z")
    out = torch.empty_like(z) if out is None else out
    _flat(out, "out")
    if dh.numel() != z.numel() or out.numel() != z.numel():
        raise ValueError("gelu_bwd: size mismatch")
    N.check(N.lib().vp_gelu_bwd_bf16(_p(dh), _p(z), _p(out), z.numel(), _stream()), "vp_gelu_bwd_bf16")
    return out


def axpy(a: torch.Tensor, b: torch.Tensor, alpha: float = 1.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _flat(a, "a")
    _flat(b, "b")
    out = torch.empty_like(a) if out is None else out
    _flat(out, "out")
    if a.numel() != b.numel() or out.numel() != a.numel():
        raise ValueError("axpy: size mismatch")
    N.check(N.lib().vp_axpy_bf16(_p(a), _p(b), alpha, _p(out), a.numel(), _stream()), "vp_axpy_bf16")
    return out


def silu(x: torch.Tensor) -> torch.Tensor:
    _flat(x, "x")
    out = torch.empty_like(x)
    N.check(N.lib().vp_silu_bf16(_p(x), _p(out), x.numel(), _stream()), "vp_silu_bf16")
    return out


def silu_bwd(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    _flat(dy, "dy")
    _flat(x, "x")
    if dy.numel() != x.numel():
        raise ValueError("silu_bwd: size mismatch")
    out = torch.empty_like(x)
    N.check(N.lib().vp_silu_bwd_bf16(_p(dy), _p(x), _p(out), x.numel(), _stream()), "vp_silu_bwd_bf16")
    return out


def head_norm_rope_bwd(x_in: torch.Tensor, dy: torch.Tensor, dx: torch.Tensor, heads: int, text_len: int, ln,
                       rope=None, dln: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """Backward of head_norm_rope (LayerNorm(64) module `ln`, RoPE on rows >= text_len): [B, N, heads*64] views with
    contiguous last dim (dx may alias dy); dln = fp32 ([64], [64]) accumulators for the affine grads, or None."""
    for t, n in ((x_in, "x_in"), (dy, "dy"), (dx, "dx")):
        _chk(t, n)
        if t.dim() != 3 or t.stride(-1) != 1 or t.shape != x_in.shape or t.shape[-1] != heads * 64:
            raise ValueError(f"{n} must be [B, N, heads*64] with a contiguous last dim")
    B, Ntok, _ = x_in.shape
    cos = sin = None
    if rope is not None:
        cos, sin = rope
        if cos.shape != (Ntok - text_len, 64) or not cos.is_contiguous() or not sin.is_contiguous():
            raise ValueError(f"rope tables must be fp32 [{Ntok - text_len}, 64]")
    dw = db = None
    if dln is not None:
        dw, db = dln
        _chk(dw, "dln_w", torch.float32)
        _chk(db, "dln_b", torch.float32)
    N.check(N.lib().vp_head_norm_rope_bwd_bf16(_p(x_in), x_in.stride(1), x_in.stride(0), _p(dy), dy.stride(1),
                                               dy.stride(0), _p(dx), dx.stride(1), dx.stride(0), B, Ntok, heads,
                                               text_len, _p(ln.weight), _p(ln.bias), float(ln.eps), _p(cos), _p(sin),
                                               _p(dw), _p(db), _stream()), "vp_head_norm_rope_bwd_bf16")
    return dx


WGRAD_PAD = 64  # the GEMM's fast path wants whole 64-wide K tiles


def wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW = dy^T x for a linear y = x W^T (+ b): dy [M, N], x [M, K] (or [nb, R, *] batched row views) -> bf16 [N, K]
    by one GEMM over the token dimension (both operands transposed, M zero-padded to whole K tiles)."""
    dyt = transpose(dy, pad_to=WGRAD_PAD)
    xt = transpose(x, pad_to=WGRAD_PAD)
    out = torch.empty(dyt.shape[0], xt.shape[0], device=dy.device, dtype=BF16)
    gemm(dyt, [xt], [None], out)
    return out
