"""Training backward of the CogVideoX transformer + VideoPainter branch on the HIP kernels.

The caller is the reference's training step (train/train_cogvideox_inpainting_i2v_video.py:1857-1892): the branch
(trainable) runs on the noisy latents + masked-video condition, its per-block samples are injected into the frozen
42-layer transformer, the v-prediction loss is backpropagated (`accelerator.backward(loss)`) through the frozen
transformer into the branch's parameters.  Each piece is a `torch.autograd.Function` whose forward is the inference
path itself (same launches, same rounding points) and whose backward runs only native kernels:

  * `_BlockFn` — one CogVideoXBlock (cogvideox_transformer_3d.py:125-184), gradient-checkpointed: only the block
    input is saved; the backward recomputes mod1/mod2, the AdaLN outputs, the pre-norm q/k/v, the normed q/k, the
    attention output + softmax statistics, the gated residual and the FF1 pre-activation, then runs
      FF2 dgrad -> GELU' -> FF1 dgrad -> AdaLN2' (+ residual) -> gate1 row-scale -> to_out dgrad
      -> flash-attention backward -> (LayerNorm(64) + RoPE)' for q, k -> fused QKV dgrad -> AdaLN1' (+ residual)
    with the dgrad GEMMs against cached transposed weights.  Trainable blocks add the weight gradients (one GEMM over
    the token dimension per weight, `kernels.wgrad`), bias / LayerNorm-affine / modulation sums (`kernels.colsum`)
    and the modulation linear's backward into the time embedding.
  * `_HeadFn` — norm_final + norm_out (AdaLN, shift|scale) + proj_out + unpatchify (:613-637), input gradient only
    (the transformer is frozen in the reference's training; trainable head parameters raise).
  * `_PatchEmbedFn` (embeddings.py:400-454), `_TimeEmbedFn` (embeddings.py:729-774), `_RowLinearFn` (the branch's
    zero-initialised output linears, branch_cogvideox.py:418-426): parameter gradients (inputs are data).

Grad tensors are bf16 like the parameters (fp32 accumulation inside every kernel; the per-column sums are fp32 until
the final cast).

VideoPainterID training (train/train_cogvideox_inpainting_i2v_video_resample.py:1520-1526, 1951-1961): the blocks'
resample processor (window 0: attention over [K; LN(mask . k) + RoPE] and [V; mask . v],
attention_processor.py:2223-2304) is differentiable — the backward recomputes both segments explicitly, runs the
flash backward over all 2N keys and routes the second segment's gradients back through the masked copy (masked rows
to k / v, the null keys' to the norm_k affine) — and trainable LoRA factors on to_q / to_k / to_v / to_out.0
(`transformer.add_adapter`, lora.py) run unfused like PEFT's, on K-augmented operands (lora.AugmentedProjection):
dA = dT^T x and dB = s dy^T T from the augmented projection's gradients (dT = s dy B, T = x A^T).
Out of scope for the backward (NotImplementedError): the fp8 modes, the previous-clip blend (windows > 0) and
`return_hidden_states` — inference-only in the reference.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from . import _native as NAT
from . import kernels as K
from .attention_processor import bounded_scores
from .attention_processor import project_out
from .lora import AugmentedProjection, augmented_rows

BF16 = torch.bfloat16
F32 = torch.float32


# ------------------------------------------------------------------------------------------------------------------
# transposed weights for the dgrad GEMMs (cached on the parameter, keyed on storage + version)
# ------------------------------------------------------------------------------------------------------------------

def _wt(w: torch.Tensor) -> torch.Tensor:
    key = (w.data_ptr(), w._version, tuple(w.shape))
    c = getattr(w, "_vp_wt", None)
    if c is None or c[0] != key:
        c = (key, K.transpose(w.detach()))
        w._vp_wt = c
    return c[1]


def _qkv_t(attn) -> torch.Tensor:
    """[D, 3D] = cat(W_q, W_k, W_v)^T: the fused QKV dgrad's weight."""
    ws = (attn.to_q.weight, attn.to_k.weight, attn.to_v.weight)
    key = tuple((w.data_ptr(), w._version) for w in ws)
    c = getattr(attn, "_vp_qkv_t", None)
    if c is None or c[0] != key:
        D = ws[0].shape[1]
        n = ws[0].shape[0]
        wt = torch.empty(D, 3 * n, device=ws[0].device, dtype=BF16)
        for s, w in enumerate(ws):
            K.transpose(w.detach(), out=wt[:, s * n:(s + 1) * n])
        c = (key, wt)
        attn._vp_qkv_t = c
    return c[1]


def _aug_tail_t(aug: AugmentedProjection) -> torch.Tensor:
    """[R, sum out_i]: the transposed block-diagonal tail of the augmented weights — rows i r .. of projection i's
    columns hold W_aug_i[:, K:]^T = (s B_i)^T, zero elsewhere (cached on the first Linear, keyed like them)."""
    ws = aug.weights()
    key = tuple(id(l) for l in aug.lins) + aug._key()
    owner = aug.lins[0]
    c = owner.__dict__.get("_vp_aug_tail_t")
    if c is None or c[0] != key:
        n = sum(w.shape[0] for w in ws)
        wt = torch.zeros(aug.R, n, device=ws[0].device, dtype=BF16)
        off = 0
        for i, w in enumerate(ws):
            c0 = aug.block_col(i)
            K.transpose(w[:, c0:c0 + aug.r], out=wt[i * aug.r:(i + 1) * aug.r, off:off + w.shape[0]])
            off += w.shape[0]
        c = (key, wt)
        owner.__dict__["_vp_aug_tail_t"] = c
    return c[1]


def _aug_dgrad(aug: AugmentedProjection, dy2: torch.Tensor, x2: Optional[torch.Tensor], out2: torch.Tensor, train: bool,
               G: "_Grads", x_aug: Optional[torch.Tensor] = None) -> None:
    """Backward of the unfused-LoRA projections y_i = x_aug W_aug_i^T (lora.AugmentedProjection; segment i reads
    rank block i of T = x A_cat^T), given out2 = dy W0 (the base dgrad): out2 += dT A_cat with dT = dy W_tail
    (block i = s dy_i B_i).  With train: W0_i's gradient only when it trains (dy_i^T x), dB = s (dy_i^T T_i) from
    the GEMM over rank block i of x_aug alone, dA = dT^T x — no full [N, K + R] weight gradient for frozen bases."""
    Kd, r = aug.K, aug.r
    M = dy2.shape[0]
    dT = torch.empty(M, aug.R, device=dy2.device, dtype=BF16)
    K.gemm(dy2, [_aug_tail_t(aug)], [None], dT)
    dxl = torch.empty(M, Kd, device=dy2.device, dtype=BF16)
    K.gemm(dT, [aug.a_cat_t()], [None], dxl)  # dT A_cat
    K.axpy(out2, dxl, out=out2)
    if not train:
        return
    dA = None
    row = 0
    for i, (lin, ps) in enumerate(zip(aug.lins, aug.pairs)):
        n = lin.weight.shape[0]
        dyi = dy2[:, row:row + n]
        if lin.weight.requires_grad:
            G.put(lin.weight, K.wgrad(dyi, x2))
        if any(B.requires_grad for _, B, _ in ps):
            dbt = K.wgrad(dyi, x_aug[:, Kd + i * r:Kd + (i + 1) * r])  # [n, r] = dy_i^T T_i
        o = 0
        for A, B, sc in ps:
            ra = A.shape[0]
            if B.requires_grad:
                G.put(B, dbt[:, o:o + ra].float() * sc)
            if A.requires_grad:
                if dA is None:
                    dA = K.wgrad(dT, x2)  # [R, K]
                G.put(A, dA[i * r + o:i * r + o + ra])
            o += ra
        row += n


def _dgrad(dy2: torch.Tensor, w: torch.Tensor, out2: torch.Tensor) -> torch.Tensor:
    """out = dy W for y = x W^T: the GEMM C = A B^T with B = W^T."""
    return K.gemm(dy2, [_wt(w)], [None], out2)


def _total(a: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 column sum over every row of a 2-D view (of a * b)."""
    return K.colsum(a, b)[0, 0]


class _Grads:
    """Collects parameter gradients (bf16, the parameter's shape) for parameters that require them."""

    def __init__(self):
        self.g: Dict[int, torch.Tensor] = {}

    def put(self, p: Optional[torch.Tensor], g: torch.Tensor) -> None:
        if p is None or not p.requires_grad:
            return
        g = g.reshape(p.shape).to(p.dtype)
        if id(p) in self.g:
            self.g[id(p)] = self.g[id(p)] + g
        else:
            self.g[id(p)] = g

    def out(self, params: Sequence[torch.Tensor]) -> List[Optional[torch.Tensor]]:
        return [self.g.get(id(p)) for p in params]


def _mod_grad(shift: torch.Tensor, scale: torch.Tensor, gate: torch.Tensor) -> torch.Tensor:
    """[B, 6D] bf16 gradient of the CogVideoXLayerNormZero modulation (shift|scale|gate|enc_shift|enc_scale|enc_gate)
    from the per-(batch, video/text) column sums [B, 2, D]."""
    B, _, D = shift.shape
    return torch.stack((shift[:, 0], scale[:, 0], gate[:, 0], shift[:, 1], scale[:, 1], gate[:, 1]), 1) \
        .reshape(B, 6 * D).to(BF16)


def _small_linear_bwd(G: _Grads, lin, x_in: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """Backward of y = x_in W^T + b on a few rows (the modulation / time-embedding linears): parameter grads into G,
    returns d x_in (bf16 [rows, in])."""
    G.put(lin.weight, K.wgrad(dy, x_in))
    if lin.bias is not None:
        G.put(lin.bias, _total(dy))
    return K.linear_small(dy, _wt(lin.weight), None)


# ------------------------------------------------------------------------------------------------------------------
# the block
# ------------------------------------------------------------------------------------------------------------------

def _check_block_trainable_path(block, resample_mask=None) -> None:
    a = block.attn1
    if (block.ff_mx is not None or block.qkv_mx is not None or getattr(block, "out_mx", None) is not None
            or getattr(a, "fp8_qk_exp", None) is not None):
        raise NotImplementedError("the backward runs the bf16 path: disable the fp8 modes for training")
    from .attention_processor import CogVideoXAttnProcessor2_0_resample
    if isinstance(a.processor, CogVideoXAttnProcessor2_0_resample) and resample_mask is None:
        raise ValueError("the resample processor needs resample_mask (id_pool_resample needs masks)")


def _put_linear_grads(G: _Grads, lin, dw: torch.Tensor) -> None:
    """The weight gradient of one projection without a trainable adapter (those go through _aug_dgrad)."""
    G.put(lin.weight, dw)


def _block_front(block, x: torch.Tensor, T: int, temb: torch.Tensor, rope, resample_mask, attn_saved=None,
                 with_h: bool = False) -> dict:
    """forward_joint's launches up to the FF1 pre-activation, with its rounding points, keeping what the backward
    reads: the recompute of the checkpointed backward, and the front of the training forward (block_forward_saving).
    The QKV projection runs forward_joint's fused qk-norm + RoPE epilogue and also stores the pre-norm q | k (the
    GEMM's aux output, ABI 17) for the LayerNorm backward; with_h: FF1 runs its GELU epilogue and stores the
    pre-activation z as the aux output (h and z from one pass: the same bits as FF1 + vp_gelu_bf16)."""
    B, Ntok, D = x.shape
    M = B * Ntok
    a = block.attn1
    H = a.heads
    n1, n2 = block.norm1, block.norm2
    ff0, to_out = block.ff.net[0].proj, block.attn1.to_out[0]
    F4 = ff0.weight.shape[0]
    dev = x.device
    mod1 = n1.modulation(temb)
    mod2 = n2.modulation(temb)
    # trainable LoRA factors run unfused: the projections on K-augmented operands (lora.AugmentedProjection),
    # which AdaLN and the attention write in place (lora.augmented_rows)
    xn = K.adaln_modulate(x, n1.norm.weight, n1.norm.bias, mod1, T, n1.norm.eps,
                          out=augmented_rows((a.to_q, a.to_k, a.to_v), B, Ntok, D, dev))
    qkv = torch.empty(B, Ntok, 3 * D, device=dev, dtype=BF16)
    qaug = AugmentedProjection.of((a.to_q, a.to_k, a.to_v))
    oaug = AugmentedProjection.of((to_out,))
    xq = xn.view(M, D) if qaug is None else qaug.input(xn.view(M, D))
    resample = resample_mask is not None
    qkp = None
    kw = {}
    if not resample:
        # qkv = [norm_q(q) + RoPE | norm_k(k) + RoPE | v] and qkp = the pre-norm [q | k], one GEMM
        qkp = torch.empty(B, Ntok, 2 * D, device=dev, dtype=BF16)
        kw = dict(epilogue=NAT.EPI_BIAS_QKNORM_ROPE, qk_norm=(a.norm_q, a.norm_k), rope=rope, tokens_per_batch=Ntok,
                  text_len=T, aux=qkp.view(M, 2 * D))
    if qaug is None:
        K.gemm(xq, [a.to_q.weight, a.to_k.weight, a.to_v.weight], [a.to_q.bias, a.to_k.bias, a.to_v.bias],
               qkv.view(M, 3 * D), **kw)
    else:
        qaug.gemm(xq, [a.to_q.bias, a.to_k.bias, a.to_v.bias], qkv.view(M, 3 * D), **kw)
    v = qkv[..., 2 * D:]
    if resample:
        # the resample processor's keys / values as one explicit 2N-key sequence: [K; K2], [V; V2] with
        # K2 = LN(mask . k) + RoPE (masked rows: = K's rows; null rows: the norm_k bias, rotated), V2 = mask . v
        qn = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
        kc = torch.empty(B, 2 * Ntok, D, device=dev, dtype=BF16)
        vc = torch.empty(B, 2 * Ntok, D, device=dev, dtype=BF16)
        kn = kc[:, :Ntok]
        K.head_norm_rope(qkv[..., D:2 * D], kc[:, Ntok:], H, T, a.norm_k.weight, a.norm_k.bias, a.norm_k.eps, rope,
                         tok_mask=resample_mask, pre_scale=1.0)
        vc[:, :Ntok].copy_(v)
        K.mask_scale_rows(v, vc[:, Ntok:], resample_mask, 1.0)
        katt, vatt = kc, vc
        K.head_norm_rope(qkv[..., :D], qn, H, T, a.norm_q.weight, a.norm_q.bias, a.norm_q.eps, rope)
        K.head_norm_rope(qkv[..., D:2 * D], kn, H, T, a.norm_k.weight, a.norm_k.bias, a.norm_k.eps, rope)
    else:
        qn, katt, vatt = qkv[..., :D], qkv[..., D:2 * D], v
    if attn_saved is not None and not resample:
        o, lse = attn_saved
    else:
        o = augmented_rows((to_out,), B, Ntok, D, dev)
        lse = torch.empty(B, H, Ntok, device=dev, dtype=F32)
        K.attention(qn, katt, vatt, o, H, scale=a.scale, bounded_scores=bounded_scores(a), lse=lse)
    x_mid = torch.empty_like(x)
    project_out(to_out, o.view(M, D), x_mid.view(M, D), epilogue=NAT.EPI_GATED, resid=x.view(M, D), mod=mod1,
                gate_chunk=2, gate_text_chunk=5, tokens_per_batch=Ntok, text_len=T)
    xn2 = K.adaln_modulate(x_mid, n2.norm.weight, n2.norm.bias, mod2, T, n2.norm.eps)
    z = torch.empty(M, F4, device=dev, dtype=BF16)
    st = dict(mod1=mod1, mod2=mod2, xn=xn, xq=xq, qkv=qkv, o=o, lse=lse, x_mid=x_mid, xn2=xn2, z=z)
    if with_h:
        st["h"] = torch.empty(M, F4, device=dev, dtype=BF16)
        K.gemm(xn2.view(M, D), [ff0.weight], [ff0.bias], st["h"], epilogue=NAT.EPI_BIAS_GELU, aux=z)
    else:
        K.gemm(xn2.view(M, D), [ff0.weight], [ff0.bias], z)
    if resample:
        st.update(qn=qn, kc=kc, vc=vc)
    else:
        st["qkp"] = qkp
    return st


def block_forward_saving(block, x: torch.Tensor, T: int, temb: torch.Tensor, rope, inject=None, inject_mask=None,
                         keep_train: bool = False):
    """The block's forward for a training step, keeping its intermediates for the backward (SAVE_ACTIVATIONS): the
    launches of _block_front (the fused QKV epilogue also storing the pre-norm q | k, FF1's GELU epilogue also storing
    its pre-activation z), then FF2 with the gated residual + injection exactly as forward_joint: the same output
    bits.  Kept: mod1 / mod2, the normed q | k + v and the pre-norm q | k, the attention output + lse, x_mid, z (and,
    for a block with trainable parameters or a temb that needs its gradient, the AdaLN outputs and h)."""
    B, Ntok, D = x.shape
    M = B * Ntok
    ff2 = block.ff.net[2]
    st = _block_front(block, x, T, temb, rope, None, with_h=True)
    h = st.pop("h")
    out = torch.empty_like(x)
    kw = {}
    if inject is not None:
        kw = dict(inject=inject, inject_ld=inject.stride(1), inject_bstride=inject.stride(0), inject_mask=inject_mask)
    K.gemm(h.view(M, -1), [ff2.weight], [ff2.bias], out.view(M, D), epilogue=NAT.EPI_GATED,
           resid=st["x_mid"].view(M, D), mod=st["mod2"], gate_chunk=2, gate_text_chunk=5, tokens_per_batch=Ntok,
           text_len=T, **kw)
    if keep_train:
        st["h"] = h
    else:
        del h
        for k in ("xn", "xq", "xn2"):
            st.pop(k)
    return out, st


def block_backward(block, x: torch.Tensor, T: int, temb: torch.Tensor, rope, inject_mask: Optional[torch.Tensor],
                   dout: torch.Tensor, want_dtemb: bool, want_dinject: bool, train: bool,
                   resample_mask: Optional[torch.Tensor] = None, attn_saved=None, front: Optional[dict] = None):
    """Gradient-checkpointed backward of `block.forward_joint(x, T, temb, rope, resample_mask=.., inject=..,
    inject_mask=..)`.  Returns (dx [B, Ntok, D], dtemb or None, dinject [B, Nv, D] or None, _Grads).  attn_saved:
    the forward's (attention output, lse) — then the attention is not recomputed (SAVE_ATTENTION); front: the
    training forward's kept intermediates (block_forward_saving) — then nothing is recomputed."""
    B, Ntok, D = x.shape
    M = B * Ntok
    a = block.attn1
    H = a.heads
    n1, n2 = block.norm1, block.norm2
    ff0, ff2, to_out = block.ff.net[0].proj, block.ff.net[2], a.to_out[0]
    F4 = ff0.weight.shape[0]
    dev = x.device
    need_dmod = train or want_dtemb
    G = _Grads()

    # ---- the forward's intermediates: kept by the training forward (SAVE_ACTIVATIONS = "all", block_forward_saving)
    # or recomputed here with forward_joint's launches and rounding points ----
    if front is None:
        front = _block_front(block, x, T, temb, rope, resample_mask, attn_saved, with_h=need_dmod)
    f = front
    mod1, mod2, qkv, o, lse, x_mid, z = (f.pop(k) for k in ("mod1", "mod2", "qkv", "o", "lse", "x_mid", "z"))
    xn, xq, xn2, h_saved = f.pop("xn", None), f.pop("xq", None), f.pop("xn2", None), f.pop("h", None)
    qaug = AugmentedProjection.of((a.to_q, a.to_k, a.to_v))
    oaug = AugmentedProjection.of((to_out,))
    resample = resample_mask is not None
    v = qkv[..., 2 * D:]
    kc = vc = None
    if resample:  # qkv: the pre-norm projections
        qn, kc, vc = f.pop("qn"), f.pop("kc"), f.pop("vc")
        qpre, kpre = qkv[..., :D], qkv[..., D:2 * D]
    else:  # qkv: the normed q | k and v; qkp: the pre-norm q | k
        qkp = f.pop("qkp")
        qn, kn = qkv[..., :D], qkv[..., D:2 * D]
        qpre, kpre = qkp[..., :D], qkp[..., D:]
    del front, f

    dout = dout.contiguous()
    dout2 = dout.view(M, D)
    dinj = None
    if want_dinject:
        if inject_mask is None:
            dinj = dout[:, T:].clone()
        else:
            dinj = torch.empty(B, Ntok - T, D, device=dev, dtype=BF16)
            K.mask_scale_rows(dout[:, T:], dinj, (inject_mask == 0).to(torch.uint8), 1.0)

    # ---- FeedForward + gated residual 2 ----
    g = dout.clone()  # d x_mid, then d x
    df = torch.empty(M, D, device=dev, dtype=BF16)
    K.rowscale(dout2, df, Ntok, T, mod2, 2, 5)
    dz = torch.empty(M, F4, device=dev, dtype=BF16)
    K.gemm(df, [_wt(ff2.weight)], [None], dz, epilogue=NAT.EPI_GELU_BWD, z=z)  # (df W2) * GELU'(z), one pass
    dxn2 = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
    _dgrad(dz, ff0.weight, dxn2.view(M, D))
    n2o = dn2 = xh2 = None
    if need_dmod:
        n2o, dn2, xh2 = (torch.empty_like(x) for _ in range(3))
    K.adaln_bwd(x_mid, dxn2, g, T, n2.norm.weight, n2.norm.bias, n2.norm.eps, mod2, n_out=n2o, dn_out=dn2,
                xhat_out=xh2)
    if need_dmod:
        # h exactly as the forward made it: GELU applied in the FF1 GEMM epilogue on the fp32 accumulator (a GELU
        # of the bf16-rounded z would differ by one rounding, and so would ff2's weight and gate-2 gradients)
        h = h_saved if h_saved is not None else K.linear(xn2.view(M, D), ff0.weight, ff0.bias, gelu=True)
        f = torch.empty(M, D, device=dev, dtype=BF16)
        K.gemm(h, [ff2.weight], [ff2.bias], f)
        dmod2 = _mod_grad(K.colsum(dxn2.view(M, D), tokens_per_batch=Ntok, text_len=T),
                          K.colsum(dxn2.view(M, D), n2o.view(M, D), tokens_per_batch=Ntok, text_len=T),
                          K.colsum(dout2, f, tokens_per_batch=Ntok, text_len=T))
        del f
        if train:
            G.put(ff2.weight, K.wgrad(df, h))
            G.put(ff2.bias, _total(df))
            G.put(ff0.weight, K.wgrad(dz, xn2.view(M, D)))
            G.put(ff0.bias, _total(dz))
            G.put(n2.norm.weight, _total(dn2.view(M, D), xh2.view(M, D)))
            G.put(n2.norm.bias, _total(dn2.view(M, D)))
        del h
    del z, dz, df, xn2, n2o, dn2, xh2, dxn2, h_saved

    # ---- attention + gated residual 1 ----
    dao = torch.empty(M, D, device=dev, dtype=BF16)
    K.rowscale(g.view(M, D), dao, Ntok, T, mod1, 2, 5)
    o_aug = None
    if need_dmod:
        ao = torch.empty(M, D, device=dev, dtype=BF16)
        project_out(to_out, o.view(M, D), ao)
        gate1 = K.colsum(g.view(M, D), ao, tokens_per_batch=Ntok, text_len=T)
        del ao
        if train:
            if oaug is None:
                if to_out.weight.requires_grad:
                    _put_linear_grads(G, to_out, K.wgrad(dao, o.view(M, D)))
            else:
                o_aug = oaug.input(o.view(M, D))
            G.put(to_out.bias, _total(dao))
    do = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
    _dgrad(dao, to_out.weight, do.view(M, D))
    if oaug is not None:
        _aug_dgrad(oaug, dao, o.view(M, D), do.view(M, D), train and need_dmod, G, o_aug)
    del dao, o_aug
    dqkv = torch.empty(B, Ntok, 3 * D, device=dev, dtype=BF16)
    dk2 = None
    if resample:
        dkc = torch.empty(B, 2 * Ntok, D, device=dev, dtype=BF16)
        dvc = torch.empty(B, 2 * Ntok, D, device=dev, dtype=BF16)
        K.attention_bwd(qn, kc, vc, o, do, lse, H, scale=a.scale, dq=dqkv[..., :D], dk=dkc, dv=dvc)
        dqkv[..., D:2 * D].copy_(dkc[:, :Ntok])
        dv2 = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
        K.mask_scale_rows(dvc[:, Ntok:], dv2, resample_mask, 1.0)  # V2 = mask . v
        torch.add(dvc[:, :Ntok], dv2, out=dv2)
        dqkv[..., 2 * D:].copy_(dv2)
        dk2 = dkc[:, Ntok:]
        del dvc, dv2, kc, vc
    else:
        K.attention_bwd(qn, kn, v, o, do, lse, H, scale=a.scale, dq=dqkv[..., :D], dk=dqkv[..., D:2 * D],
                        dv=dqkv[..., 2 * D:])
        del qn, kn, v, qkv
    del do, o, lse
    dlnq = dlnk = None
    if train and (a.norm_q.weight.requires_grad or a.norm_k.weight.requires_grad):
        dlnq = (torch.zeros(64, device=dev, dtype=F32), torch.zeros(64, device=dev, dtype=F32))
        dlnk = (torch.zeros(64, device=dev, dtype=F32), torch.zeros(64, device=dev, dtype=F32))
    K.head_norm_rope_bwd(qpre, dqkv[..., :D], dqkv[..., :D], H, T, a.norm_q, rope, dlnq)
    K.head_norm_rope_bwd(kpre, dqkv[..., D:2 * D], dqkv[..., D:2 * D], H, T, a.norm_k, rope, dlnk)
    if dk2 is not None:
        # K2 = LN(mask . k) + RoPE: (LN + RoPE)' at the masked input, then x mask (null rows: LN of a zero row,
        # whose input gradient the mask cancels; their d beta stays in dlnk)
        km = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
        K.mask_scale_rows(kpre, km, resample_mask, 1.0)
        dkm = K.head_norm_rope_bwd(km, dk2, torch.empty(B, Ntok, D, device=dev, dtype=BF16), H, T, a.norm_k, rope,
                                   dlnk)
        K.mask_scale_rows(dkm, km, resample_mask, 1.0)
        dqkv[..., D:2 * D].add_(km)
        del km, dkm, dk2, dkc
    del qpre, kpre
    if dlnq is not None:
        G.put(a.norm_q.weight, dlnq[0])
        G.put(a.norm_q.bias, dlnq[1])
        G.put(a.norm_k.weight, dlnk[0])
        G.put(a.norm_k.bias, dlnk[1])
    dxn = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
    K.gemm(dqkv.view(M, 3 * D), [_qkv_t(a)], [None], dxn.view(M, D))
    if train:
        db = _total(dqkv.view(M, 3 * D))
        if qaug is None and any(l.weight.requires_grad for l in (a.to_q, a.to_k, a.to_v)):
            dw = K.wgrad(dqkv.view(M, 3 * D), xq)
            for s, lin in enumerate((a.to_q, a.to_k, a.to_v)):
                _put_linear_grads(G, lin, dw[s * D:(s + 1) * D])
            del dw
        for s, lin in enumerate((a.to_q, a.to_k, a.to_v)):
            G.put(lin.bias, db[s * D:(s + 1) * D])
        if qaug is not None:
            _aug_dgrad(qaug, dqkv.view(M, 3 * D), xn.view(M, D), dxn.view(M, D), True, G, xq)
    elif qaug is not None:
        # (no parameter gradients: x2 is not read — and a frozen block's saving forward keeps no xn)
        _aug_dgrad(qaug, dqkv.view(M, 3 * D), None, dxn.view(M, D), False, G)
    del dqkv, xn, xq
    n1o = dn1 = xh1 = None
    if need_dmod:
        n1o, dn1, xh1 = (torch.empty_like(x) for _ in range(3))
    K.adaln_bwd(x, dxn, g, T, n1.norm.weight, n1.norm.bias, n1.norm.eps, mod1, n_out=n1o, dn_out=dn1, xhat_out=xh1)

    dtemb = None
    if need_dmod:
        dmod1 = _mod_grad(K.colsum(dxn.view(M, D), tokens_per_batch=Ntok, text_len=T),
                          K.colsum(dxn.view(M, D), n1o.view(M, D), tokens_per_batch=Ntok, text_len=T), gate1)
        if train:
            G.put(n1.norm.weight, _total(dn1.view(M, D), xh1.view(M, D)))
            G.put(n1.norm.bias, _total(dn1.view(M, D)))
        s = K.silu(temb.contiguous())
        ds = K.axpy(_small_linear_bwd(G, n1.linear, s, dmod1), _small_linear_bwd(G, n2.linear, s, dmod2))
        if want_dtemb:
            dtemb = K.silu_bwd(ds, temb.contiguous())
    return g, dtemb, dinj, G


# The block forward keeps its attention output and softmax statistics for the backward (~113 MB per block at B = 1,
# N = 17 776: 5 GB for the 44 blocks of a training step, against 288 GB of HBM), so the backward recomputes the
# projections and norms but not the attention — the checkpointing otherwise stays as the reference's
# --gradient_checkpointing has it.  The same kernel call produces both (bit-identical to the recompute: the fused QKV
# epilogue equals the separate norm launches).  False: recompute the attention too.
SAVE_ATTENTION = True
# Beyond that, while the device has room (SAVE_ACTIVATIONS = True; the budget below), the training forward runs the
# backward's front itself (block_forward_saving) and keeps every intermediate the backward reads, so the backward
# recomputes nothing: ~1.2 GB per frozen 5b block at B = 1, N = 17 776 (q | k | v, the normed q | k, O, x_mid, the FF1
# pre-activation z).
# A block whose kept set would leave less than SAVE_RESERVE_BYTES free (or four times its own size) falls back to
# the attention-only form, so a larger batch degrades to recompute instead of running out of memory.
SAVE_ACTIVATIONS = True
SAVE_RESERVE_BYTES = 16 << 30


def _room_for(x: torch.Tensor, F4: int, keep_train: bool = False, R: int = 0) -> bool:
    B, Ntok, D = x.shape
    per_row = 5 * D + D + D + F4  # q | k | v, normed q | k, O, x_mid, z (bf16)
    if keep_train:  # + h [F4], the AdaLN outputs xn / xn2 and xq (with the adapters' rank tail R)
        per_row += F4 + 3 * D + R
    need = B * Ntok * per_row * 2
    free, _ = torch.cuda.mem_get_info(x.device)
    return free - need > max(SAVE_RESERVE_BYTES, 4 * need)


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, block, T, rope, inject_mask, resample_mask, x, temb, inject, *params):
        ctx.front = ctx.attn_saved = None
        keep_train = any(p.requires_grad for p in params) or temb.requires_grad
        qaug = AugmentedProjection.of((block.attn1.to_q, block.attn1.to_k, block.attn1.to_v)) if keep_train else None
        if SAVE_ACTIVATIONS and resample_mask is None and _room_for(
                x, block.ff.net[0].proj.weight.shape[0], keep_train, qaug.R if qaug is not None else 0):
            out, ctx.front = block_forward_saving(block, x, T, temb, rope, inject,
                                                  inject_mask if inject is not None else None, keep_train)
        else:
            save = {} if SAVE_ATTENTION and resample_mask is None else None
            out = block.forward_joint(x, T, temb, rope, resample_mask=resample_mask, inject=inject,
                                      inject_mask=inject_mask if inject is not None else None, attn_save=save)
            ctx.attn_saved = (save["o"], save["lse"]) if save else None
        ctx.block, ctx.T, ctx.rope, ctx.inject_mask, ctx.resample_mask = block, T, rope, inject_mask, resample_mask
        ctx.has_inject = inject is not None
        ctx.params = params
        ctx.save_for_backward(x, temb)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, temb = ctx.saved_tensors
        need = ctx.needs_input_grad
        train = any(need[8:])
        front, ctx.front = ctx.front, None  # (the backward pops it: each intermediate is freed as it is used)
        attn_saved, ctx.attn_saved = ctx.attn_saved, None
        dx, dtemb, dinj, G = block_backward(ctx.block, x, ctx.T, temb, ctx.rope,
                                            ctx.inject_mask if ctx.has_inject else None, dout, need[6],
                                            need[7] and ctx.has_inject, train, ctx.resample_mask, attn_saved, front)
        return (None, None, None, None, None, dx if need[5] else None, dtemb, dinj, *G.out(ctx.params))


def block_apply(block, x: torch.Tensor, T: int, temb: torch.Tensor, rope, inject: Optional[torch.Tensor] = None,
                inject_mask: Optional[torch.Tensor] = None,
                resample_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Differentiable `block.forward_joint` (gradient-checkpointed).  resample_mask: the uint8 token mask of the
    blocks' resample processor (window 0 of VideoPainterID training)."""
    _check_block_trainable_path(block, resample_mask)
    params = [p for p in block.parameters()]
    return _BlockFn.apply(block, T, rope, inject_mask, resample_mask, x, temb, inject, *params)


# ------------------------------------------------------------------------------------------------------------------
# head, embeddings, branch output linears
# ------------------------------------------------------------------------------------------------------------------

class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, dims, x, emb):
        B, F, H, W, T = dims
        cfg = model.config
        p = cfg.patch_size
        D = x.shape[-1]
        Nv = x.shape[1] - T
        mod = K.linear_small(emb, model.norm_out.linear.weight, model.norm_out.linear.bias, act_in=K.ACT_SILU)
        y = K.final_norm(x, T, model.norm_final.weight, model.norm_final.bias, model.norm_out.norm.weight,
                         model.norm_out.norm.bias, model.norm_out.norm.eps, mod)
        proj = K.linear(y.view(B * Nv, D), model.proj_out.weight, model.proj_out.bias)
        ctx.model, ctx.dims = model, dims
        ctx.save_for_backward(x, emb)
        return K.unpatchify(proj, B, F, cfg.out_channels, H, W, p)

    @staticmethod
    def backward(ctx, dout):
        x, emb = ctx.saved_tensors
        m = ctx.model
        B, F, H, W, T = ctx.dims
        cfg = m.config
        p = cfg.patch_size
        _, Ntok, D = x.shape
        Nv = Ntok - T
        if ctx.needs_input_grad[3]:
            raise NotImplementedError("the head's time-embedding gradient (a trainable transformer time embedding) "
                                      "is not implemented: the reference trains the branch only")
        mod = K.linear_small(emb, m.norm_out.linear.weight, m.norm_out.linear.bias, act_in=K.ACT_SILU)
        dproj = K.patchify(dout.to(BF16).contiguous(), None, p, p * p * cfg.out_channels)
        dy = torch.empty(B * Nv, D, device=x.device, dtype=BF16)
        _dgrad(dproj, m.proj_out.weight, dy)
        zero_mod = torch.zeros(B, 6 * D, device=x.device, dtype=BF16)
        n1 = K.adaln_modulate(x, m.norm_final.weight, m.norm_final.bias, zero_mod, T, m.norm_final.eps)
        dx = torch.zeros_like(x)
        dn1 = torch.empty(1, Nv, D, device=x.device, dtype=BF16)
        for b in range(B):
            dn1.zero_()
            K.adaln_bwd(n1[b:b + 1, T:], dy[b * Nv:(b + 1) * Nv].view(1, Nv, D), dn1, 0, m.norm_out.norm.weight,
                        m.norm_out.norm.bias, m.norm_out.norm.eps, mod[b:b + 1], chunks=(0, 1, 0, 1))
            K.adaln_bwd(x[b:b + 1, T:], dn1, dx[b:b + 1, T:], 0, m.norm_final.weight, m.norm_final.bias,
                        m.norm_final.eps, zero_mod[b:b + 1], chunks=(0, 1, 0, 1))
        return None, None, dx, None


def head_apply(model, x: torch.Tensor, emb: torch.Tensor, dims) -> torch.Tensor:
    head = [model.norm_final.weight, model.norm_final.bias, model.norm_out.linear.weight, model.norm_out.linear.bias,
            model.norm_out.norm.weight, model.norm_out.norm.bias, model.proj_out.weight, model.proj_out.bias]
    if any(t is not None and t.requires_grad for t in head):
        raise NotImplementedError("trainable transformer head parameters: the reference trains the branch only")
    return _HeadFn.apply(model, dims, x, emb)


class _PatchEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pe, text, video, video2, *params):
        ctx.pe = pe
        ctx.params = params
        ctx.save_for_backward(text, video, video2)
        return pe.embed(text, video, video2)

    @staticmethod
    def backward(ctx, dx):
        text, video, video2 = ctx.saved_tensors
        pe = ctx.pe
        G = _Grads()
        dx = dx.contiguous()
        B, Ntok, D = dx.shape
        T = text.shape[1]
        G.put(pe.text_proj.weight, K.wgrad(dx[:, :T], text))
        wp, kpad = pe._padded_conv_weight()
        cols = K.patchify(video, video2, pe.patch_size, kpad)
        w = pe.proj.weight
        kk = w.shape[1] * w.shape[2] * w.shape[3]
        dwp = K.wgrad(dx[:, T:], cols)
        G.put(w, dwp[:, :kk].contiguous())
        if pe.text_proj.bias is not None or pe.proj.bias is not None:
            st = torch.zeros(1, 2, D, device=dx.device, dtype=F32)
            sv = torch.zeros(1, 2, D, device=dx.device, dtype=F32)
            for b in range(B):
                K.colsum(dx[b, :T], out=st)
                K.colsum(dx[b, T:], out=sv)
            G.put(pe.text_proj.bias, st[0, 0])
            G.put(pe.proj.bias, sv[0, 0])
        return (None, None, None, None, *G.out(ctx.params))


def patch_embed_apply(pe, text: torch.Tensor, video: torch.Tensor, video2: Optional[torch.Tensor] = None):
    if any(t is not None and t.requires_grad for t in (text, video, video2)):
        raise NotImplementedError("gradients w.r.t. the latents / prompt embeddings are not implemented (the "
                                  "reference's training feeds them as data)")
    params = [pe.text_proj.weight, pe.text_proj.bias, pe.proj.weight, pe.proj.bias]
    if not any(p is not None and p.requires_grad for p in params):
        return pe.embed(text, video, video2)
    return _PatchEmbedFn.apply(pe, text, video, video2, *[p for p in params if p is not None])


class _TimeEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, te, t0, *params):
        h = K.linear_small(t0, te.linear_1.weight, te.linear_1.bias, act_out=K.ACT_SILU)
        ctx.te, ctx.params = te, params
        ctx.save_for_backward(t0)
        return K.linear_small(h, te.linear_2.weight, te.linear_2.bias)

    @staticmethod
    def backward(ctx, demb):
        (t0,) = ctx.saved_tensors
        te = ctx.te
        G = _Grads()
        a1 = K.linear_small(t0, te.linear_1.weight, te.linear_1.bias)
        h = K.silu(a1)
        dh = _small_linear_bwd(G, te.linear_2, h, demb.to(BF16).contiguous())
        _small_linear_bwd(G, te.linear_1, t0, K.silu_bwd(dh, a1))
        return (None, None, *G.out(ctx.params))


def time_embed_apply(te, t0: torch.Tensor) -> torch.Tensor:
    params = [p for p in te.parameters()]
    if not any(p.requires_grad for p in params):
        h = K.linear_small(t0, te.linear_1.weight, te.linear_1.bias, act_out=K.ACT_SILU)
        return K.linear_small(h, te.linear_2.weight, te.linear_2.bias)
    return _TimeEmbedFn.apply(te, t0, *params)


class _RowLinearFn(torch.autograd.Function):
    """y = (x W^T + b) * scale over every row of the joint buffer (the branch's output linears)."""

    @staticmethod
    def forward(ctx, x, w, b, scale):
        B, Ntok, D = x.shape
        o = torch.empty(B, Ntok, w.shape[0], device=x.device, dtype=BF16)
        epi = NAT.EPI_BIAS if scale == 1.0 else NAT.EPI_BIAS_SCALE
        K.gemm(x.reshape(B * Ntok, D), [w], [b], o.view(B * Ntok, -1), epilogue=epi, alpha=scale)
        ctx.scale = scale
        ctx.save_for_backward(x, w, b)
        return o

    @staticmethod
    def backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        B, Ntok, D = x.shape
        dy = dy.to(BF16).contiguous()
        if ctx.scale != 1.0:
            dy = K.scale_bf16(dy, ctx.scale)
        dy2 = dy.view(B * Ntok, -1)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _dgrad(dy2, w, dx.view(B * Ntok, D))
        if ctx.needs_input_grad[1]:
            dw = K.wgrad(dy2, x.reshape(B * Ntok, D)).to(w.dtype)
        if b is not None and ctx.needs_input_grad[2]:
            db = _total(dy2).to(b.dtype)
        return dx, dw, db, None


def row_linear_apply(x: torch.Tensor, lin, scale: float) -> torch.Tensor:
    return _RowLinearFn.apply(x, lin.weight, lin.bias, float(scale))


def needs_grad(module, *tensors) -> bool:
    """The training path is taken when autograd is on and a parameter or an input requires grad."""
    if not torch.is_grad_enabled():
        return False
    if any(p.requires_grad for p in module.parameters()):
        return True
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.requires_grad:
            return True
        if isinstance(t, (list, tuple)) and any(isinstance(s, torch.Tensor) and s.requires_grad for s in t):
            return True
    return False
