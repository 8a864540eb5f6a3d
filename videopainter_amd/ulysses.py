"""Ulysses head-parallel split of ONE clip's denoising forward over P ranks (the optional
"within one forward" row; not in the reference, whose multi-GPU story is data parallel only).

Every rank holds a contiguous shard of n = ceil(N / P) rows of the joint [B, N, D] buffer (text first, like the
single-GPU layout; the last shard zero-padded to n rows) for the whole forward: AdaLN, the fused QKV projection with
qk-norm + RoPE, to_out, the FeedForward, the gated residuals and the branch injection are row-local, so they run
unchanged on the shard (a shard's text rows are always a prefix of it: `text_len` becomes the shard's own count, the
RoPE table / injection / mask are sliced at the shard's first video row).  Only attention mixes rows:

    qkv [B, n, 3D] --all-to-all--> [B, N_pad, 3 * D/P]   (rank r receives every row of head group r)
    flash attention over the N real keys for H/P heads
    o [B, N_pad, D/P] --all-to-all--> [B, n, D]

two RCCL all-to-alls per block of 3 / 1 x n*D*2 B * (P-1)/P per rank.  The head gathers the proj_out rows
(all-gather of [B, n, 64]) and every rank unpatchifies the whole noise prediction, so the CFG / DPM step that follows
runs replicated exactly as on one GPU.  The branch runs sharded the same way and its samples stay local (the
injection of a shard's rows reads only the branch's same rows).

Communicators: `DistComm` (torch.distributed; backend "nccl" = RCCL over xGMI) and `ThreadComm`, which runs the P
ranks as P threads of one process on one GPU (same launches in the same order per rank; the exchanges are local
copies) — the single-GPU rehearsal the GPU tests use to check the split against the unsplit forward.

Scope: the bf16 path with both processors of the any-length pipeline — the standard one (config 2, the headline;
with the previous-clip blend) and the ID-resample one (config 4: window 0's masked second K / V segment, later
windows' masked previous-window K / V): the projections stay row-local, the masks and the RoPE table of the
head-group attention are the full ones.  The fp8 modes raise NotImplementedError under the split.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _native as NAT
from . import kernels as K
from .attention_processor import (CogVideoXAttnProcessor2_0, CogVideoXAttnProcessor2_0_resample, _fusable_norms,
                                  _kv, _qkv, _rope_dev, _u8, bounded_scores)
from .transformer import BF16, Transformer2DModelOutput, _bf

# ------------------------------------------------------------------------------------------------------------------
# communicators
# ------------------------------------------------------------------------------------------------------------------


class DistComm:
    """RCCL over a torch.distributed group (one process per GPU)."""

    def __init__(self, group=None):
        self.group = group
        self.P = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_to_all(self, rank: int, send: torch.Tensor) -> torch.Tensor:
        """send [P, ...] contiguous, chunk j for rank j -> [P, ...], chunk j from rank j."""
        out = torch.empty_like(send)
        dist.all_to_all_single(out, send, group=self.group)
        return out

    def all_gather(self, rank: int, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        out = torch.empty((self.P * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        dist.all_gather_into_tensor(out, x, group=self.group)  # (concatenated along dim 0, as gloo requires)
        return out.view((self.P,) + tuple(x.shape))


class ThreadComm:
    """P ranks emulated by P threads of one process sharing one GPU stream (tests / single-GPU rehearsal).  An
    exchange publishes each thread's buffer, waits for all P, copies its chunks, and waits again before the slots
    are reused; every copy is launched after the producers' launches, so stream order makes it correct."""

    def __init__(self, P: int):
        self.P = P
        self._slots: List[Optional[torch.Tensor]] = [None] * P
        self._bar = threading.Barrier(P)

    def all_to_all(self, rank: int, send: torch.Tensor) -> torch.Tensor:
        self._slots[rank] = send
        self._bar.wait()
        out = torch.stack([self._slots[j][rank] for j in range(self.P)])
        self._bar.wait()
        return out

    def all_gather(self, rank: int, x: torch.Tensor) -> torch.Tensor:
        self._slots[rank] = x.contiguous()
        self._bar.wait()
        out = torch.stack(list(self._slots))
        self._bar.wait()
        return out

    def run(self, fn, *args, **kw):
        """fn(rank, *args, **kw) on P threads; returns the P results (the first exception re-raised)."""
        res: List = [None] * self.P
        err: List = []

        def body(r):
            try:
                with torch.no_grad():  # (grad mode is thread-local)
                    res[r] = fn(r, *args, **kw)
            except BaseException as e:  # noqa: BLE001 - re-raised below after every thread ended
                err.append(e)
                self._bar.abort()

        ts = [threading.Thread(target=body, args=(r,)) for r in range(self.P)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if err:
            self._bar.reset()
            raise err[0]
        return res


# ------------------------------------------------------------------------------------------------------------------
# shard geometry
# ------------------------------------------------------------------------------------------------------------------

@dataclass
class Shard:
    N: int       # real joint rows
    T: int       # text rows
    P: int
    rank: int

    def __post_init__(self):
        self.n = -(-self.N // self.P)
        self.r0 = self.rank * self.n
        self.Npad = self.n * self.P
        self.valid = max(0, min(self.n, self.N - self.r0))    # real rows in this shard
        self.tl = max(0, min(self.n, self.T - self.r0))       # local text rows (a prefix of the shard)
        self.v0 = max(0, self.r0 - self.T)                    # video index of the first local video row
        self.nv = self.n - self.tl                            # local video rows (padding included)
        if self.nv == 0:
            # the whole shard is text (T >= ceil(N / P) with a small clip or a large P): the row-local kernels would
            # get zero video rows and proj_out an empty launch
            raise ValueError(f"Ulysses split: shard {self.rank} of {self.P} holds only text rows (N = {self.N}, "
                             f"T = {self.T}, {self.n} rows per shard); use fewer ranks for this clip size")

    def rows(self, x: torch.Tensor) -> torch.Tensor:
        """This shard's rows of a full [B, N, ...] tensor (zero-padded)."""
        out = torch.zeros((x.shape[0], self.n) + tuple(x.shape[2:]), device=x.device, dtype=x.dtype)
        if self.valid > 0:
            out[:, :self.valid] = x[:, self.r0:self.r0 + self.valid]
        return out

    def video_rows(self, v: torch.Tensor) -> torch.Tensor:
        """This shard's video rows of a [B, Nv, ...] tensor (zero-padded)."""
        out = torch.zeros((v.shape[0], self.nv) + tuple(v.shape[2:]), device=v.device, dtype=v.dtype)
        k = max(0, min(self.nv, v.shape[1] - self.v0))
        if k > 0:
            out[:, :k] = v[:, self.v0:self.v0 + k]
        return out

    def rope(self, rope):
        if rope is None:
            return None
        cos, sin = rope
        return tuple(self.video_rows(t.unsqueeze(0))[0].contiguous() for t in (cos, sin))


class _Ctx:
    """One rank's attention of the split forward.  rope_full: the whole RoPE table (with its grid) for the head-group
    rows; mask / prev_mask: the resample processor's full token masks [B, N] (this window's, the previous one's)."""

    def __init__(self, comm, rank: int, shard: Shard, rope_full=None, mask=None, prev_mask=None):
        self.comm, self.rank, self.sh = comm, rank, shard
        self.rope_full, self.mask, self.prev_mask = rope_full, mask, prev_mask

    def attend(self, attn, xn: torch.Tensor, text_len: int, rope, pn: Optional[torch.Tensor] = None,
               prev_clip_weight=None, resample_mask=None, prev_resample_mask=None) -> torch.Tensor:
        """Head-parallel attention of the shard's rows with the semantics of the block's processor:
        CogVideoXAttnProcessor2_0 (with the previous-clip blend when pn, the previous window's normed shard rows,
        is given) or CogVideoXAttnProcessor2_0_resample (window 0's masked second segment, or the previous window's
        masked K / V).  The row-local projections run on the shard; the masks and the RoPE table of the head-group
        attention are the full ones of the context (resample_mask / prev_resample_mask, the shard-level arguments
        of forward_joint, are not used)."""
        B, n, D = xn.shape
        P = self.comm.P
        H = attn.heads
        if H % P:
            raise ValueError(f"{H} heads do not split {P} ways")
        Hp = H // P
        Dp = Hp * 64
        N, T = self.sh.N, self.sh.T
        prev = pn is not None and prev_clip_weight is not None and prev_clip_weight > 0.0
        resample = isinstance(attn.processor, CogVideoXAttnProcessor2_0_resample)
        m = plan = None
        if resample:
            m = _u8(self.prev_mask if prev else self.mask)
            if m is None:
                raise ValueError("the resample processor needs resample_mask (id_pool_resample needs masks)")
            plan = attn.processor.plan(attn, m, T, self.rope_full)
            fused = plan[3] is not None and _fusable_norms(attn)
        else:
            fused = _fusable_norms(attn)
        qkv = _qkv(attn, xn, (text_len, rope) if fused else None)
        if not fused and not resample:
            K.head_norm_rope(qkv[..., :D], qkv[..., :D], H, text_len, attn.norm_q.weight, attn.norm_q.bias,
                             attn.norm_q.eps, rope)
            K.head_norm_rope(qkv[..., D:2 * D], qkv[..., D:2 * D], H, text_len, attn.norm_k.weight, attn.norm_k.bias,
                             attn.norm_k.eps, rope)
        full = qkv_to_heads(self.comm, self.rank, qkv)
        del qkv
        pk = pv = None
        if prev:  # the previous window's K / V of this shard's rows (pre-norm) -> every row of the head group
            pkv = qkv_to_heads(self.comm, self.rank, _kv(attn, pn), parts=2)
            pk, pv = pkv[:, :N, :Dp], pkv[:, :N, Dp:]
        o_full = torch.zeros(B, P * n, Dp, device=xn.device, dtype=BF16)
        if resample:
            q, k, v = full[:, :N, :Dp], full[:, :N, Dp:2 * Dp], full[:, :N, 2 * Dp:]
            attn.processor.attend_heads(attn, q, k, v, T, self.rope_full, m, plan, fused, pk, pv,
                                        float(prev_clip_weight) if prev else 0.0, o_full[:, :N])
        else:
            q, k, v = full[..., :Dp], full[:, :N, Dp:2 * Dp], full[:, :N, 2 * Dp:]
            bs = bounded_scores(attn)
            if prev:  # (attention_processor.py:2156-2189: (1 - w) self + w previous clip, one blended output)
                w = float(prev_clip_weight)
                K.head_norm_rope(pk, pk, Hp, T, attn.norm_k.weight, attn.norm_k.bias, attn.norm_k.eps,
                                 self.rope_full)
                K.attention(q, k, v, o_full, Hp, scale=attn.scale, out_scale=1.0 - w, bounded_scores=bs)
                K.attention(q, pk, pv, o_full, Hp, scale=attn.scale, out_scale=w, accumulate=True, bounded_scores=bs)
            else:
                K.attention(q, k, v, o_full, Hp, scale=attn.scale, bounded_scores=bs)
        del full
        return heads_to_rows(self.comm, self.rank, o_full)


def qkv_to_heads(comm, rank: int, qkv: torch.Tensor, parts: int = 3) -> torch.Tensor:
    """This shard's rows of q|k|v [B, n, 3D] (parts = 3; k|v: 2) -> every row of head group `rank`:
    [B, P n, parts * Dp]."""
    B, n, Dn = qkv.shape
    P = comm.P
    Dp = Dn // parts // P
    send = qkv.reshape(B, n, parts, P, Dp).permute(3, 0, 1, 2, 4).contiguous()  # [P(head group), B, n, parts, Dp]
    recv = comm.all_to_all(rank, send)                                            # [P(row shard), B, n, parts, Dp]
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * n, parts * Dp)


def heads_to_rows(comm, rank: int, o_full: torch.Tensor) -> torch.Tensor:
    """Head group `rank` of every row [B, P n, Dp] -> this shard's rows of all heads [B, n, P Dp]."""
    B, Npad, Dp = o_full.shape
    P = comm.P
    n = Npad // P
    send = o_full.view(B, P, n, Dp).permute(1, 0, 2, 3).contiguous()          # [P(row shard), B, n, Dp]
    recv = comm.all_to_all(rank, send)                                          # [P(head group), B, n, Dp]
    return recv.permute(1, 2, 0, 3).reshape(B, n, P * Dp)


def _check(model, fp8_attrs=("ff_mx", "qkv_mx", "out_mx")):
    for blk in model.transformer_blocks:
        if any(getattr(blk, a, None) is not None for a in fp8_attrs) or \
                getattr(blk.attn1, "fp8_qk_exp", None) is not None:
            raise NotImplementedError("the head-parallel split runs the bf16 path (disable the fp8 modes)")
        if type(blk.attn1.processor) not in (CogVideoXAttnProcessor2_0, CogVideoXAttnProcessor2_0_resample):
            raise NotImplementedError("the head-parallel split runs the standard and ID-resample processors")


# ------------------------------------------------------------------------------------------------------------------
# sharded forwards (the models' forward semantics, one rank's shard)
# ------------------------------------------------------------------------------------------------------------------

def branch_forward(branch, comm, rank: int, hidden_states, encoder_hidden_states, branch_cond, timestep,
                   image_rotary_emb=None, conditioning_scale: float = 1.0) -> List[torch.Tensor]:
    """CogvideoXBranchModel.forward on one shard: returns the samples as this shard's video rows [B, nv, D]."""
    _check(branch)
    dev = branch.proj_out.weight.device
    B = hidden_states.shape[0]
    hs, bc, enc = (_bf(t.to(dev)) for t in (hidden_states, branch_cond, encoder_hidden_states))
    T = enc.shape[1]
    emb = branch._time_embed(timestep, B, dev)
    x_full = branch.patch_embed.embed(enc, hs, bc)
    sh = Shard(x_full.shape[1], T, comm.P, rank)
    x = sh.rows(x_full)
    del x_full
    ctx = _Ctx(comm, rank, sh)
    rope = sh.rope(_rope_dev(image_rotary_emb, dev))
    D = x.shape[-1]
    outs = []
    scale = float(conditioning_scale)
    for block, lin in zip(branch.transformer_blocks, branch.branch_blocks):
        x = block.forward_joint(x, sh.tl, emb, rope, attend=ctx.attend)
        o = torch.empty(B, sh.n, D, device=dev, dtype=BF16)
        epi = NAT.EPI_BIAS if scale == 1.0 else NAT.EPI_BIAS_SCALE
        K.gemm(x.view(B * sh.n, D), [lin.weight], [lin.bias], o.view(B * sh.n, D), epilogue=epi, alpha=scale)
        outs.append(o[:, sh.tl:])
    return outs


def transformer_forward(model, comm, rank: int, hidden_states, encoder_hidden_states, timestep,
                        image_rotary_emb=None, branch_block_samples=None, branch_block_masks=None,
                        add_first: bool = False, return_hidden_states: bool = False,
                        id_pool_resample_learnable: bool = False, prev_hidden_states=None,
                        prev_clip_weight: Optional[float] = None, prev_resample_mask=None):
    """CogVideoXTransformer3DModel.forward on one shard.  `branch_block_samples` are the branch's shard samples
    (`branch_forward` on the same rank).  Returns the full noise prediction on every rank (and this shard's hidden
    states when asked: [B, n, D] each).  The any-length pipeline's window hand-off (anyl.py:962-988):
    prev_hidden_states = the previous window's shard hidden states ({layer: [B, n, D]}, what this function returned
    for it), prev_clip_weight, and prev_resample_mask = the full [B, N] mask the previous window returned."""
    _check(model)
    dev = model.proj_out.weight.device
    cfg = model.config
    B, F, C, H, W = hidden_states.shape
    p = cfg.patch_size
    hs, enc = _bf(hidden_states.to(dev)), _bf(encoder_hidden_states.to(dev))
    T = enc.shape[1]
    Nv = F * (H // p) * (W // p)
    emb = model._time_embed(timestep, B, dev)
    x_full = model.patch_embed.embed(enc, hs)
    sh = Shard(x_full.shape[1], T, comm.P, rank)
    x = sh.rows(x_full)
    del x_full
    rope_full = _rope_dev(image_rotary_emb, dev, grid=(F, H // p, W // p))
    rope = sh.rope(rope_full)
    tok_mask = full_mask = None
    if branch_block_masks is not None:
        tm = K.patch_mask(branch_block_masks.to(dev), p)
        tok_mask = sh.video_rows(tm).contiguous()
        if id_pool_resample_learnable:
            full_mask = torch.zeros(B, T + tm.shape[1], device=dev, dtype=torch.bool)
            full_mask[:, T:] = tm.bool()
    if id_pool_resample_learnable and full_mask is None:
        raise ValueError("id_pool_resample needs masks")
    ctx = _Ctx(comm, rank, sh, rope_full, _u8(full_mask), _u8(prev_resample_mask))
    bs = list(branch_block_samples) if branch_block_samples is not None else None
    nl = len(model.transformer_blocks)
    interval = int(np.ceil(nl / len(bs))) if bs else 1
    hs_list = []
    for i, block in enumerate(model.transformer_blocks):
        inj = None
        if bs is not None:
            if not add_first:
                inj = bs[i // interval]
            elif i < len(bs):
                inj = bs[i]
        pj = None
        if prev_hidden_states is not None:
            pj = prev_hidden_states.get(i) if isinstance(prev_hidden_states, dict) else prev_hidden_states
        x = block.forward_joint(x, sh.tl, emb, rope, prev_joint=pj,
                                prev_clip_weight=prev_clip_weight if pj is not None else None,
                                inject=inj, inject_mask=tok_mask if inj is not None else None, attend=ctx.attend)
        if return_hidden_states:
            hs_list.append(x)
    D = x.shape[-1]
    mod = K.linear_small(emb, model.norm_out.linear.weight, model.norm_out.linear.bias, act_in=K.ACT_SILU)
    y = K.final_norm(x, sh.tl, model.norm_final.weight, model.norm_final.bias, model.norm_out.norm.weight,
                     model.norm_out.norm.bias, model.norm_out.norm.eps, mod)
    pc = model.proj_out.weight.shape[0]
    proj = torch.zeros(B, sh.n, pc, device=dev, dtype=BF16)
    proj[:, :sh.nv] = K.linear(y.view(B * sh.nv, D), model.proj_out.weight, model.proj_out.bias).view(B, sh.nv, pc)
    allp = comm.all_gather(rank, proj)                                            # [P, B, n, pc]
    rows = []
    for j in range(comm.P):
        sj = Shard(sh.N, T, comm.P, j)
        rows.append(allp[j, :, :sj.nv])
    full = torch.cat(rows, 1)[:, :Nv].reshape(B * Nv, pc).contiguous()
    out = K.unpatchify(full, B, F, cfg.out_channels, H, W, p)
    return (out, hs_list) if return_hidden_states else (out,)


class UlyssesModels:
    """The pair (transformer, branch) behind the harness's call forms, split head-parallel over `comm` (this process
    = rank `rank`).  Pass `.transformer` / `.branch` to `CogVideoXI2VDualInpaintAnyLHarness` in place of the models."""

    def __init__(self, transformer, branch, comm, rank: Optional[int] = None):
        self.comm = comm
        self.rank = comm.rank if rank is None else rank
        self.transformer = _TransformerView(transformer, self)
        self.branch = _BranchView(branch, self)


class _BranchView:
    def __init__(self, model, owner):
        self.model, self.o = model, owner
        self.config = model.config

    def __call__(self, hidden_states, encoder_hidden_states, branch_cond, timestep, image_rotary_emb=None,
                 conditioning_scale=1.0, attention_kwargs=None, return_dict=True, **_):
        outs = branch_forward(self.model, self.o.comm, self.o.rank, hidden_states, encoder_hidden_states,
                              branch_cond, timestep, image_rotary_emb, conditioning_scale)
        return (outs,)


class _TransformerView:
    def __init__(self, model, owner):
        self.model, self.o = model, owner
        self.config = model.config
        self.proj_out = model.proj_out

    def __call__(self, hidden_states, encoder_hidden_states, timestep, image_rotary_emb=None, attention_kwargs=None,
                 branch_block_samples=None, branch_block_masks=None, add_first=False,
                 id_pool_resample_learnable=False, return_hidden_states=False, return_resample_mask=False,
                 return_dict=True, **_):
        # the per-call LoRA scale (attention_kwargs["scale"], default 1.0): unfused adapters take it in their
        # augmented operands (rebuilt from the live factors, so an optimizer step's updates reach them too), exactly as
        # the single-GPU forward does (transformer.py, lora.AugmentedProjection)
        self.model._call_lora_scale(attention_kwargs)
        akw = attention_kwargs or {}
        res = transformer_forward(self.model, self.o.comm, self.o.rank, hidden_states, encoder_hidden_states,
                                  timestep, image_rotary_emb, branch_block_samples, branch_block_masks, add_first,
                                  return_hidden_states, id_pool_resample_learnable, akw.get("prev_hidden_states"),
                                  akw.get("prev_clip_weight"), akw.get("prev_resample_mask"))
        out = res[0]
        if not return_hidden_states:
            return (out,) if not return_dict else Transformer2DModelOutput(sample=out)
        rm = None
        if return_resample_mask:
            if branch_block_masks is None:
                raise ValueError("id_pool_resample needs masks")
            p = self.config.patch_size
            tm = K.patch_mask(branch_block_masks.to(out.device), p)
            T = encoder_hidden_states.shape[1]
            rm = torch.zeros(tm.shape[0], T + tm.shape[1], device=out.device, dtype=torch.bool)
            rm[:, T:] = tm.bool()
            return (out, res[1], rm)
        return (out, res[1])
