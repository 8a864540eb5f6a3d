"""CogVideoX-5b-I2V DiT on the HIP kernels — drop-in for the reference `CogVideoXTransformer3DModel` /
`CogVideoXBlock` (DF/models/transformers/cogvideox_transformer_3d.py:38-646): same constructor kwargs, same
state-dict keys, same `forward` signature and return forms.

MI355X data layout: the text and video token streams live in ONE resident bf16 buffer [B, T + Nv, D] (text first),
which is exactly the reference's `cat([encoder_hidden_states, hidden_states], dim=1)`, so every per-block
`cat`/`split` of the reference disappears; per-segment behaviour (text vs video modulation, gates, RoPE only on
video tokens, injection only on video tokens) is selected per row inside the kernels.  Each block is 10 launches:

  norm1 linear (small-M) -> AdaLN modulate -> fused QKV GEMM -> qk-LN+RoPE (q, k) -> flash attention
  -> to_out GEMM (+ gate * . + residual) -> norm2 linear -> AdaLN modulate -> FF1 GEMM (+GELU-tanh)
  -> FF2 GEMM (+ gate * . + residual + masked branch injection)

With `return_hidden_states=True` every block writes its output into a fresh buffer that IS the returned
`hidden_states_list[i]` (no copies).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn as nn

from . import kernels as K
from . import _native as NAT
from .attention_processor import (Attention, CogVideoXAttnProcessor2_0, CogVideoXAttnProcessor2_0_resample,
                                  CogVideoXAttnProcessor2_0_wo_text,
                                  _rope_dev, _u8, project_out)
from .embeddings import joint_sincos_pos_embedding
from .lora import augmented_rows
from .modules import Conv2dPatch, Dropout, LayerNorm, Linear, ModelMixin, _empty

BF16 = torch.bfloat16


@dataclass
class Transformer2DModelOutput:
    sample: torch.Tensor


def _bf(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.dtype != BF16:
        t = t.to(BF16)
    return t.contiguous()


# ------------------------------------------------------------------------------------------------------------------
# sub-modules with the reference's parameter names
# ------------------------------------------------------------------------------------------------------------------

class CogVideoXLayerNormZero(nn.Module):
    """DF/models/normalization.py:358-386 — linear: 6*D x temb, norm: LayerNorm(D)."""

    def __init__(self, conditioning_dim: int, embedding_dim: int, elementwise_affine: bool = True, eps: float = 1e-5,
                 bias: bool = True):
        super().__init__()
        self.linear = Linear(conditioning_dim, 6 * embedding_dim, bias=bias)
        self.norm = LayerNorm(embedding_dim, eps=eps, elementwise_affine=elementwise_affine)

    def modulation(self, temb: torch.Tensor) -> torch.Tensor:
        """silu(temb) @ W + b -> bf16 [B, 6D] = shift|scale|gate|enc_shift|enc_scale|enc_gate."""
        return K.linear_small(temb, self.linear.weight, self.linear.bias, act_in=K.ACT_SILU)


class GELUProj(nn.Module):
    def __init__(self, dim_in, dim_out, bias=True):
        super().__init__()
        self.proj = Linear(dim_in, dim_out, bias=bias)
        self.approximate = "tanh"


class FeedForward(nn.Module):
    """DF/models/attention.py:1144-1202 with activation_fn="gelu-approximate": net = [GELU(proj), Dropout, Linear,
    Dropout] (non-gated; SURVEY.md finding 1)."""

    def __init__(self, dim: int, inner_dim: Optional[int] = None, bias: bool = True, final_dropout: bool = True):
        super().__init__()
        inner_dim = inner_dim or 4 * dim
        mods = [GELUProj(dim, inner_dim, bias=bias), Dropout(), Linear(inner_dim, dim, bias=bias)]
        if final_dropout:
            mods.append(Dropout())
        self.net = nn.ModuleList(mods)


class TimestepEmbedding(nn.Module):
    """DF/models/embeddings.py:729-774 (linear_1 -> SiLU -> linear_2)."""

    def __init__(self, in_channels: int, time_embed_dim: int):
        super().__init__()
        self.linear_1 = Linear(in_channels, time_embed_dim)
        self.linear_2 = Linear(time_embed_dim, time_embed_dim)


class CogVideoXPatchEmbed(nn.Module):
    """DF/models/embeddings.py:337-454 — parameters only; `embed()` runs im2col + two GEMMs with fused bias and
    positional-embedding add, writing text rows then video rows of the joint buffer."""

    def __init__(self, patch_size: int, in_channels: int, embed_dim: int, text_embed_dim: int, sample_width: int,
                 sample_height: int, sample_frames: int, temporal_compression_ratio: int, max_text_seq_length: int,
                 spatial_interpolation_scale: float, temporal_interpolation_scale: float,
                 use_positional_embeddings: bool, use_learned_positional_embeddings: bool):
        super().__init__()
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.sample_height, self.sample_width, self.sample_frames = sample_height, sample_width, sample_frames
        self.temporal_compression_ratio = temporal_compression_ratio
        self.max_text_seq_length = max_text_seq_length
        self.spatial_interpolation_scale = spatial_interpolation_scale
        self.temporal_interpolation_scale = temporal_interpolation_scale
        self.use_positional_embeddings = use_positional_embeddings
        self.use_learned_positional_embeddings = use_learned_positional_embeddings
        self.proj = Conv2dPatch(in_channels, embed_dim, patch_size)
        self.text_proj = Linear(text_embed_dim, embed_dim)
        self._pos_cache = {}
        self._wpad = None
        if use_positional_embeddings or use_learned_positional_embeddings:
            pe = self._sincos(sample_height, sample_width, sample_frames)
            if use_learned_positional_embeddings:
                self.register_buffer("pos_embedding", _empty(*pe.shape).data, persistent=True)
                with torch.no_grad():
                    self.pos_embedding.copy_(pe)
            else:
                self.register_buffer("pos_embedding", pe.to(self.proj.weight.device, BF16), persistent=False)

    def _sincos(self, h, w, frames):
        return joint_sincos_pos_embedding(self.embed_dim, self.patch_size, self.max_text_seq_length, h, w, frames,
                                          self.temporal_compression_ratio, self.spatial_interpolation_scale,
                                          self.temporal_interpolation_scale)

    def _padded_conv_weight(self) -> Tuple[torch.Tensor, int]:
        w = self.proj.weight
        kk = w.shape[1] * w.shape[2] * w.shape[3]
        kpad = (kk + 63) // 64 * 64
        key = (w.data_ptr(), w._version, kpad)
        if self._wpad is None or self._wpad[0] != key:
            wp = torch.zeros(w.shape[0], kpad, device=w.device, dtype=BF16)
            wp[:, :kk] = w.reshape(w.shape[0], kk)
            self._wpad = (key, wp)
        return self._wpad[1], kpad

    def _pos_for(self, h: int, w: int, frames_latent: int, device) -> Optional[torch.Tensor]:
        """Reference :431-450: learned buffer at the sample resolution / frame count; 3D sin-cos recomputed for
        other frame counts; ValueError for another resolution with learned embeddings."""
        if not (self.use_positional_embeddings or self.use_learned_positional_embeddings):
            return None
        if self.use_learned_positional_embeddings and (self.sample_width != w or self.sample_height != h):
            raise ValueError(
                "It is currently not possible to generate videos at a different resolution that the defaults. This "
                "should only be the case with 'THUDM/CogVideoX-5b-I2V'.If you think this is incorrect, please open "
                "an issue at https://github.com/huggingface/diffusers/issues.")
        pre = (frames_latent - 1) * self.temporal_compression_ratio + 1
        if self.sample_height != h or self.sample_width != w or self.sample_frames != pre:
            key = (h, w, pre, str(device))
            if key not in self._pos_cache:
                self._pos_cache[key] = self._sincos(h, w, pre)[0].to(device=device, dtype=BF16).contiguous()
            return self._pos_cache[key]
        return self.pos_embedding[0]

    def embed(self, text: torch.Tensor, video: torch.Tensor, video2: Optional[torch.Tensor] = None) -> torch.Tensor:
        """text [B, T, Ct], video [B, F, C1, H, W] (+ video2 [B, F, C2, H, W] concatenated on channels)
        -> joint bf16 [B, T + F*(H/p)*(W/p), D]."""
        B, T, _ = text.shape
        _, F, _, H, W = video.shape
        p = self.patch_size
        Nv = F * (H // p) * (W // p)
        Ntok = T + Nv
        D = self.embed_dim
        if T != self.max_text_seq_length and (self.use_learned_positional_embeddings or self.use_positional_embeddings):
            raise ValueError(f"text length {T} != max_text_seq_length {self.max_text_seq_length}")
        pos = self._pos_for(H, W, F, video.device)
        x = torch.empty(B, Ntok, D, device=video.device, dtype=BF16)
        xf = x.view(B * Ntok, D)
        epi = NAT.EPI_BIAS_ADDROWS if pos is not None else NAT.EPI_BIAS
        K.gemm(text.reshape(B * T, -1), [self.text_proj.weight], [self.text_proj.bias], xf, epilogue=epi,
               rows_per_group=T, group_stride=Ntok, row_offset=0, addrows=pos, addrows_offset=0)
        wp, kpad = self._padded_conv_weight()
        cols = K.patchify(video, video2, p, kpad)
        K.gemm(cols, [wp], [self.proj.bias], xf, epilogue=epi, rows_per_group=Nv, group_stride=Ntok, row_offset=T,
               addrows=pos, addrows_offset=T)
        return x


class CogVideoXBlock(nn.Module):
    """DF/models/transformers/cogvideox_transformer_3d.py:38-216."""

    def __init__(self, dim: int, num_attention_heads: int, attention_head_dim: int, time_embed_dim: int,
                 dropout: float = 0.0, activation_fn: str = "gelu-approximate", attention_bias: bool = False,
                 qk_norm: bool = True, norm_elementwise_affine: bool = True, norm_eps: float = 1e-5,
                 final_dropout: bool = True, ff_inner_dim: Optional[int] = None, ff_bias: bool = True,
                 attention_out_bias: bool = True, wo_text: bool = False, id_pool_resample_learnable: bool = False):
        super().__init__()
        if activation_fn != "gelu-approximate":
            raise NotImplementedError(f"activation_fn={activation_fn!r}: CogVideoX uses gelu-approximate")
        if not qk_norm:
            raise NotImplementedError("CogVideoX uses qk_norm=True")
        self.norm1 = CogVideoXLayerNormZero(time_embed_dim, dim, norm_elementwise_affine, norm_eps, bias=True)
        # wo_text (the branch's text-free mode, :96-97): the blocks run `forward_joint` with no text rows
        self.wo_text = bool(wo_text)
        self.processor = CogVideoXAttnProcessor2_0_wo_text() if wo_text else \
            CogVideoXAttnProcessor2_0_resample() if id_pool_resample_learnable else CogVideoXAttnProcessor2_0()
        self.attn1 = Attention(query_dim=dim, dim_head=attention_head_dim, heads=num_attention_heads, eps=1e-6,
                               bias=attention_bias, out_bias=attention_out_bias, processor=self.processor)
        self.norm2 = CogVideoXLayerNormZero(time_embed_dim, dim, norm_elementwise_affine, norm_eps, bias=True)
        self.ff = FeedForward(dim, inner_dim=ff_inner_dim, bias=ff_bias, final_dropout=final_dropout)
        self.dim = dim
        self.ff_mx = None  # (W1, W2) as MX-FP8 when the fp8 FeedForward is enabled (BASELINE config 5)
        self.qkv_mx = None  # (Wq, Wk, Wv) as MX-FP8 when the fp8 QKV projection is enabled
        self.out_mx = None  # W_out as MX-FP8 when the fp8 attention output projection is enabled

    def enable_fp8_ffn(self, enabled: bool = True) -> None:
        """Run the FeedForward on the block-scaled fp8 MFMA: both weights quantised once to MX-FP8 (e4m3 + one
        E8M0 scale per 32 inputs), the norm2 AdaLN output written in MX-FP8, FF1's GELU output re-quantised in its
        epilogue, FF2 accumulating in fp32 into the bf16 gated residual.  The state dict is unchanged."""
        if not enabled:
            self.ff_mx = None
            return
        w1, w2 = self.ff.net[0].proj.weight, self.ff.net[2].weight
        if w1.shape[0] % 256 or w2.shape[0] % 256 or w1.shape[1] % 128 or w2.shape[1] % 128:
            raise ValueError(f"fp8 FeedForward needs widths that are multiples of 256, got {tuple(w1.shape)}")
        self.ff_mx = (K.mx_quantize(w1), K.mx_quantize(w2))

    def enable_fp8_qkv(self, enabled: bool = True) -> None:
        """Fused QKV projection on the block-scaled fp8 MFMA: the three weights quantised once to MX-FP8, the norm1
        AdaLN writing MX-FP8 directly, bf16 q/k/v out (the prev-clip K/V projection stays bf16)."""
        if not enabled:
            self.qkv_mx = None
            return
        a = self.attn1
        from .lora import module_pairs
        if any(module_pairs(l) for l in (a.to_q, a.to_k, a.to_v)):
            raise NotImplementedError("fp8 QKV with unfused LoRA adapters on q / k / v: fuse_lora() (loaded adapters) "
                                      "or drop the adapter first")
        ws = (a.to_q.weight, a.to_k.weight, a.to_v.weight)
        if any(w.shape[0] % 256 or w.shape[1] % 128 for w in ws):
            raise ValueError("fp8 QKV needs widths that are multiples of 256")
        self.qkv_mx = tuple(K.mx_quantize(w) for w in ws)

    def enable_fp8_out(self, enabled: bool = True) -> None:
        """The attention's output projection (to_out[0], attention_processor.py:2202) on the block-scaled fp8 MFMA:
        the weight quantised once to MX-FP8, the attention output quantised per call (vp_mx_quantize_bf16), the gated
        residual in the fp8 GEMM's epilogue as in the bf16 path."""
        if not enabled:
            self.out_mx = None
            return
        lin = self.attn1.to_out[0]
        from .lora import module_pairs
        if module_pairs(lin):
            raise NotImplementedError("fp8 output projection with an unfused LoRA adapter on to_out: fuse_lora() "
                                      "(loaded adapters) or drop the adapter first")
        if lin.weight.shape[0] % 256 or lin.weight.shape[1] % 128:
            raise ValueError("fp8 output projection needs widths that are multiples of 256")
        self.out_mx = K.mx_quantize(lin.weight)

    def enable_fp8_attention(self, enabled: bool = True) -> None:
        """Run self-attention on the block-scaled fp8 MFMA (vp_attention_fwd_fp8): Q and K leave the qk-norm + RoPE
        kernel as e4m3 with one static power-of-two factor each, chosen from the LayerNorm's bound on its outputs
        (kernels.qk_fp8_exponent: nothing can saturate), V is packed to e4m3 with per-(channel, 32 keys) scales,
        and P is rounded to e4m3 inside the kernel.  The resample processor (two K/V segments) stays bf16."""
        attn = self.attn1
        if not enabled:
            attn.fp8_qk_exp = None
            return
        attn.fp8_qk_exp = (K.qk_fp8_exponent(attn.norm_q.weight, attn.norm_q.bias, attn.scale * K.LOG2E),
                           K.qk_fp8_exponent(attn.norm_k.weight, attn.norm_k.bias))

    # -- joint-buffer fast path used by the models --
    def forward_joint(self, x: torch.Tensor, text_len: int, temb: torch.Tensor, rope=None,
                      resample_mask: Optional[torch.Tensor] = None, prev_joint: Optional[torch.Tensor] = None,
                      prev_clip_weight: Optional[float] = None, prev_resample_mask: Optional[torch.Tensor] = None,
                      inject: Optional[torch.Tensor] = None, inject_mask: Optional[torch.Tensor] = None,
                      out: Optional[torch.Tensor] = None, attend=None, attn_save: Optional[dict] = None) -> torch.Tensor:
        """attend: optional replacement of the processor's attention, `attend(attn, xn, text_len, rope) -> o`
        [B, N, D] (the Ulysses head-parallel split, videopainter_amd/ulysses.py).  attn_save: a dict that receives the
        attention output "o" and its softmax statistics "lse" (a training forward keeps them for the backward,
        autograd.SAVE_ATTENTION); left empty where the attention is not the single-segment bf16 one."""
        B, Ntok, D = x.shape
        xf = x.view(B * Ntok, D)
        processor = self.attn1.processor
        if not isinstance(processor, CogVideoXAttnProcessor2_0):
            raise ValueError(f"Unsupported processor type: {type(processor)}")
        mod1 = self.norm1.modulation(temb)
        qkv = None
        if attend is not None and (self.qkv_mx is not None or self.out_mx is not None):
            raise NotImplementedError("the head-parallel split runs the bf16 path")
        if self.qkv_mx is not None:
            a = self.attn1
            xq = K.adaln_modulate_mx(x, self.norm1.norm.weight, self.norm1.norm.bias, mod1, text_len,
                                     self.norm1.norm.eps)
            qkv = torch.empty(B, Ntok, 3 * D, device=x.device, dtype=x.dtype)
            K.gemm_mx(xq, list(self.qkv_mx), [a.to_q.bias, a.to_k.bias, a.to_v.bias], qkv.view(B * Ntok, 3 * D))
            del xq
            xn = None
        else:
            a = self.attn1  # (unfused LoRA: AdaLN writes straight into the projection's K-augmented operand)
            xn = K.adaln_modulate(x, self.norm1.norm.weight, self.norm1.norm.bias, mod1, text_len,
                                  self.norm1.norm.eps,
                                  out=None if attend is not None else
                                  augmented_rows((a.to_q, a.to_k, a.to_v), B, Ntok, D, x.device))
        pn = None
        if prev_joint is not None:
            # the block normalises the previous window's states with its own norm1 (reference :141-146)
            a = self.attn1
            pout = augmented_rows((a.to_k, a.to_v), prev_joint.shape[0], prev_joint.shape[1], D, x.device)
            pn = K.adaln_modulate(_bf(prev_joint), self.norm1.norm.weight, self.norm1.norm.bias, mod1, text_len,
                                  self.norm1.norm.eps, out=pout)
        lse = None
        if (attn_save is not None and attend is None and type(processor) is CogVideoXAttnProcessor2_0 and pn is None
                and qkv is None and getattr(self.attn1, "fp8_qk_exp", None) is None):
            lse = torch.empty(B, self.attn1.heads, Ntok, device=x.device, dtype=torch.float32)
        if attend is not None:
            o = attend(self.attn1, xn, text_len, rope, pn, prev_clip_weight, resample_mask, prev_resample_mask)
        elif lse is not None:
            o = processor.attend(self.attn1, xn, text_len, rope, lse_out=lse)
            attn_save["o"], attn_save["lse"] = o, lse
        else:
            o = processor.attend(self.attn1, xn if xn is not None else x, text_len, rope, pn, prev_clip_weight,
                                 resample_mask, prev_resample_mask, qkv=qkv)
        del qkv
        del xn, pn
        x_mid = torch.empty_like(x)
        if self.out_mx is not None:
            om = K.mx_quantize(o.view(B * Ntok, D), out=K.MXTensor(B * Ntok, D, x.device, zero=False))
            del o
            K.gemm_mx(om, [self.out_mx], [self.attn1.to_out[0].bias], x_mid.view(B * Ntok, D),
                      epilogue=NAT.EPI_GATED, resid=xf, mod=mod1, tokens_per_batch=Ntok, text_len=text_len)
            del om
        else:
            project_out(self.attn1.to_out[0], o.view(B * Ntok, D), x_mid.view(B * Ntok, D), epilogue=NAT.EPI_GATED,
                        resid=xf, mod=mod1, gate_chunk=2, gate_text_chunk=5, tokens_per_batch=Ntok,
                        text_len=text_len)
            del o
        mod2 = self.norm2.modulation(temb)
        ff0 = self.ff.net[0].proj
        ff2 = self.ff.net[2]
        if out is None:
            out = torch.empty_like(x)
        if self.ff_mx is not None:
            w1, w2 = self.ff_mx
            xq = K.adaln_modulate_mx(x_mid, self.norm2.norm.weight, self.norm2.norm.bias, mod2, text_len,
                                     self.norm2.norm.eps)
            h1 = K.MXTensor(B * Ntok, w1.rows, x.device, zero=False)
            K.gemm_mx(xq, [w1], [ff0.bias], h1, epilogue=NAT.EPI_BIAS_GELU_MXFP8)
            del xq
            K.gemm_mx(h1, [w2], [ff2.bias], out.view(B * Ntok, D), epilogue=NAT.EPI_GATED,
                      resid=x_mid.view(B * Ntok, D), mod=mod2, tokens_per_batch=Ntok, text_len=text_len,
                      inject=inject, inject_mask=inject_mask)
            return out
        xn2 = K.adaln_modulate(x_mid, self.norm2.norm.weight, self.norm2.norm.bias, mod2, text_len,
                               self.norm2.norm.eps)
        h1 = K.linear(xn2, ff0.weight, ff0.bias, gelu=True)
        del xn2
        kw = {}
        if inject is not None:
            kw = dict(inject=inject, inject_ld=inject.stride(1), inject_bstride=inject.stride(0),
                      inject_mask=inject_mask)
        K.gemm(h1.view(B * Ntok, -1), [ff2.weight], [ff2.bias], out.view(B * Ntok, D), epilogue=NAT.EPI_GATED,
               resid=x_mid.view(B * Ntok, D), mod=mod2, gate_chunk=2, gate_text_chunk=5, tokens_per_batch=Ntok,
               text_len=text_len, **kw)
        return out

    def forward(self, hidden_states: torch.Tensor, encoder_hidden_states: torch.Tensor, temb: torch.Tensor,
                image_rotary_emb=None, attention_mask=None, resample_mask=None,
                attention_kwargs: Optional[Dict[str, Any]] = None):
        """Reference signature (:125-134); returns (hidden_states, encoder_hidden_states)."""
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is never set on the CogVideoX path")
        t = encoder_hidden_states.size(1)
        x = torch.cat([_bf(encoder_hidden_states), _bf(hidden_states)], dim=1).contiguous()
        kw = attention_kwargs or {}
        prev = kw.get("prev_hidden_states")
        prev = prev if isinstance(prev, torch.Tensor) else None
        out = self.forward_joint(x, t, _bf(temb), _rope_dev(image_rotary_emb, x.device), _u8(resample_mask), prev,
                                 kw.get("prev_clip_weight"), _u8(kw.get("prev_resample_mask")))
        return out[:, t:], out[:, :t]


class CogVideoXTransformer3DModel(ModelMixin):
    """Drop-in for DF/models/transformers/cogvideox_transformer_3d.py:218-646."""

    _is_branch = False

    def __init__(self, num_attention_heads: int = 30, attention_head_dim: int = 64, in_channels: int = 16,
                 out_channels: Optional[int] = 16, flip_sin_to_cos: bool = True, freq_shift: int = 0,
                 time_embed_dim: int = 512, text_embed_dim: int = 4096, num_layers: int = 30, dropout: float = 0.0,
                 attention_bias: bool = True, sample_width: int = 90, sample_height: int = 60,
                 sample_frames: int = 49, patch_size: int = 2, temporal_compression_ratio: int = 4,
                 max_text_seq_length: int = 226, activation_fn: str = "gelu-approximate",
                 timestep_activation_fn: str = "silu", norm_elementwise_affine: bool = True, norm_eps: float = 1e-5,
                 spatial_interpolation_scale: float = 1.875, temporal_interpolation_scale: float = 1.0,
                 use_rotary_positional_embeddings: bool = False, use_learned_positional_embeddings: bool = False,
                 id_pool_resample_learnable: Optional[bool] = False):
        super().__init__()
        self._init_config(dict(locals_without_self(locals())))
        inner_dim = num_attention_heads * attention_head_dim
        if not use_rotary_positional_embeddings and use_learned_positional_embeddings:
            raise ValueError(
                "There are no CogVideoX checkpoints available with disable rotary embeddings and learned positional "
                "embeddings. If you're using a custom model and/or believe this should be supported, please open an "
                "issue at https://github.com/huggingface/diffusers/issues.")
        if timestep_activation_fn != "silu" or not flip_sin_to_cos:
            raise NotImplementedError("CogVideoX uses silu time embedding with flip_sin_to_cos=True")
        self.patch_embed = CogVideoXPatchEmbed(
            patch_size, self._patch_channels(), inner_dim, text_embed_dim, sample_width, sample_height,
            sample_frames, temporal_compression_ratio, max_text_seq_length, spatial_interpolation_scale,
            temporal_interpolation_scale, not use_rotary_positional_embeddings, use_learned_positional_embeddings)
        self.embedding_dropout = Dropout()
        self.time_embedding = TimestepEmbedding(inner_dim, time_embed_dim)
        self.transformer_blocks = nn.ModuleList([
            CogVideoXBlock(dim=inner_dim, num_attention_heads=num_attention_heads,
                           attention_head_dim=attention_head_dim, time_embed_dim=time_embed_dim, dropout=dropout,
                           activation_fn=activation_fn, attention_bias=attention_bias,
                           norm_elementwise_affine=norm_elementwise_affine, norm_eps=norm_eps,
                           id_pool_resample_learnable=self._block_resample())
            for _ in range(num_layers)])
        self.norm_final = LayerNorm(inner_dim, norm_eps, norm_elementwise_affine)
        self._build_head(inner_dim, time_embed_dim, norm_elementwise_affine, norm_eps, patch_size, out_channels)

    def load_lora_weights(self, path: str, weight_name: str = "pytorch_lora_weights.safetensors",
                          adapter_name: Optional[str] = None, lora_scale: Optional[float] = None, **_):
        """The VideoPainterID adapter (PEFT safetensors) on to_q/to_k/to_v/to_out.0, applied UNFUSED as the
        reference's PEFT does (infer/inpaint.py:310-316; videopainter_amd/lora.py): the projections run on K-augmented
        operands, W0 untouched.  Every forward applies its own `attention_kwargs["scale"]` (default 1.0);
        `lora_scale` sets it now.  `fuse_lora` folds explicitly."""
        from .lora import attach_lora_, load_lora_state_dict
        sd = load_lora_state_dict(path, weight_name)
        if any(k.startswith("transformer.") for k in sd):  # the pipeline-level file (lora_pipeline.py:2653-2656)
            sd = {k: v for k, v in sd.items() if k.startswith("transformer.")}
        attach_lora_(self, sd, lora_scale, adapter_name)
        return self

    def get_list_adapters(self):
        from .lora import lora_state
        st = lora_state(self)
        return [n for n, _ in st.adapters] if st is not None else []

    def set_lora_scale(self, scale: float):
        """The per-call LoRA scale (what a call with attention_kwargs={"scale": scale} does): unfused adapters take
        it in their augmented operands; weights holding a fold are rebuilt exactly from their kept base."""
        from .lora import lora_state, refold_lora_
        st = lora_state(self)
        if st is not None and st.scale != float(scale):
            refold_lora_(self, float(scale))
        return self

    def set_adapters(self, adapter_names, weights=None):
        """PEFT's set_adapters on the folded adapters: the listed ones active with these weights, the rest off."""
        from .lora import set_adapter_weights_
        set_adapter_weights_(self, adapter_names, weights)
        return self

    def fuse_lora(self, lora_scale: float = 1.0):
        """The pipeline's `fuse_lora(lora_scale=...)`: the loaded adapters folded into W0 + s B A at `lora_scale`
        (base kept), no longer following per-call scales (PEFT's merged layers no longer see `scale_lora_layers`)."""
        from .lora import fuse_lora_
        fuse_lora_(self, lora_scale)
        return self

    def unfuse_lora(self):
        """PEFT's `unfuse_lora`: back to W0 (exact, from the kept base) with the adapters applied unfused."""
        from .lora import unfuse_lora_
        unfuse_lora_(self)
        return self

    def add_adapter(self, adapter_config, adapter_name: str = "default"):
        """PEFT's `transformer.add_adapter(LoraConfig(r=..., lora_alpha=..., init_lora_weights=True,
        target_modules=["to_q", "to_k", "to_v", "to_out.0"]))` (train/train_cogvideox_inpainting_i2v_video_resample.py
        :1520-1526): trainable lora_A / lora_B factors on the target Linears, everything else frozen
        (videopainter_amd/lora.py add_trainable_adapter_).  `adapter_config`: any object (or dict) with r,
        lora_alpha and optionally target_modules / init_lora_weights — peft's LoraConfig itself qualifies."""
        from .lora import TARGETS, add_trainable_adapter_
        get = (lambda k, d=None: adapter_config.get(k, d)) if isinstance(adapter_config, dict) else (
            lambda k, d=None: getattr(adapter_config, k, d))
        tm = get("target_modules") or TARGETS
        if isinstance(tm, str):
            tm = [tm]
        add_trainable_adapter_(self, int(get("r")), float(get("lora_alpha", get("r"))), tuple(tm), adapter_name,
                               bool(get("init_lora_weights", True)))
        return self

    def get_lora_state_dict(self):
        """The trainable factors under PEFT's saved names (`get_peft_model_state_dict(transformer)`), for
        `save_lora_weights(transformer_lora_layers=...)`."""
        from .lora import trainable_lora_state_dict
        return trainable_lora_state_dict(self)

    def _call_lora_scale(self, attention_kwargs):
        from .lora import lora_state
        st = lora_state(self)
        if st is None:
            return
        s = attention_kwargs.get("scale", 1.0) if attention_kwargs else 1.0
        self.set_lora_scale(1.0 if s is None else s)

    def enable_fp8_ffn(self, enabled: bool = True):
        """fp8 FeedForward in every block (BASELINE config 5; see CogVideoXBlock.enable_fp8_ffn).  Call after the
        weights are loaded; re-call after changing them."""
        for blk in self.transformer_blocks:
            blk.enable_fp8_ffn(enabled)
        return self

    def enable_fp8_attention(self, enabled: bool = True):
        """fp8 self-attention in every block (BASELINE config 5; see CogVideoXBlock.enable_fp8_attention).  Call
        after the weights are loaded (the Q/K factors come from the qk-norm affine)."""
        for blk in self.transformer_blocks:
            blk.enable_fp8_attention(enabled)
        return self

    def enable_fp8_qkv(self, enabled: bool = True):
        """fp8 fused QKV projection in every block (see CogVideoXBlock.enable_fp8_qkv)."""
        for blk in self.transformer_blocks:
            blk.enable_fp8_qkv(enabled)
        return self

    def enable_fp8_out(self, enabled: bool = True):
        """fp8 attention output projection in every block (see CogVideoXBlock.enable_fp8_out)."""
        for blk in self.transformer_blocks:
            blk.enable_fp8_out(enabled)
        return self

    def enable_fp8(self, ffn: bool = True, attention: bool = True, qkv: bool = True, out: bool = True):
        """BASELINE config 5: "attn + FFN in fp8" (the QKV projection, the attention products, the attention's output
        projection, the FeedForward)."""
        self.enable_fp8_ffn(ffn)
        self.enable_fp8_qkv(qkv)
        self.enable_fp8_out(out)
        return self.enable_fp8_attention(attention)

    def _patch_channels(self):
        return self.config.in_channels

    def _block_resample(self):
        return bool(self.config.id_pool_resample_learnable)

    def _build_head(self, inner_dim, time_embed_dim, affine, eps, patch_size, out_channels):
        self.norm_out = AdaLayerNorm(time_embed_dim, 2 * inner_dim, affine, eps)
        self.proj_out = Linear(inner_dim, patch_size * patch_size * out_channels)

    # -- processor plumbing (reference :372-430) --
    @property
    def attn_processors(self):
        procs = {}
        for name, m in self.named_modules():
            if hasattr(m, "get_processor"):
                procs[f"{name}.processor"] = m.get_processor()
        return procs

    def set_attn_processor(self, processor):
        count = len(self.attn_processors)
        if isinstance(processor, dict) and len(processor) != count:
            raise ValueError(f"A dict of processors was passed, but the number of processors {len(processor)} does "
                             f"not match the number of attention layers: {count}.")
        processor = dict(processor) if isinstance(processor, dict) else processor
        for name, m in self.named_modules():
            if hasattr(m, "set_processor"):
                m.set_processor(processor.pop(f"{name}.processor") if isinstance(processor, dict) else processor)

    # -- QKV fusion switches (reference :431-470) --
    def fuse_qkv_projections(self):
        """Reference :432-456 fuses to_q / to_k / to_v of every Attention into one projection and installs
        FusedCogVideoXAttnProcessor2_0.  Here Q, K and V always run as ONE GEMM over the three weight segments with
        the qk-norm + RoPE epilogue (CogVideoXBlock.forward_joint), so there is nothing to fuse: the call records
        the processors like the reference (for unfuse) and leaves weights, state-dict keys and outputs unchanged."""
        for _, proc in self.attn_processors.items():
            if "Added" in type(proc).__name__:
                raise ValueError("`fuse_qkv_projections()` is not supported for models having added KV projections.")
        self.original_attn_processors = self.attn_processors
        self._qkv_fused = True

    def unfuse_qkv_projections(self):
        """Reference :459-470: restores the processors recorded by fuse_qkv_projections (a no-op for the math, as
        fusing is)."""
        if getattr(self, "original_attn_processors", None) is not None:
            self.set_attn_processor(self.original_attn_processors)
        self._qkv_fused = False

    # -- shared pieces --
    def _time_embed(self, timestep, batch: int, device) -> torch.Tensor:
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep] * batch, device=device)
        timestep = timestep.to(device)
        if timestep.dim() == 0:
            timestep = timestep.expand(batch)
        temb0 = K.timestep_embedding(timestep, self.config.num_attention_heads * self.config.attention_head_dim,
                                     float(self.config.freq_shift))
        from .autograd import time_embed_apply
        return time_embed_apply(self.time_embedding, temb0)

    def forward(self, hidden_states: torch.Tensor, encoder_hidden_states: torch.Tensor,
                timestep: Union[int, float, torch.LongTensor], timestep_cond: Optional[torch.Tensor] = None,
                image_rotary_emb: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                attention_kwargs: Optional[Dict[str, Any]] = None, branch_block_samples=None,
                branch_block_masks: Optional[torch.Tensor] = None, add_first: Optional[bool] = False,
                self_guidance_hidden_states=None, self_guidance_masks=None,
                return_hidden_states: Optional[bool] = False, return_resample_mask: Optional[bool] = False,
                id_pool_resample_learnable: Optional[bool] = False, return_dict: bool = True):
        """Reference :472-646.  With autograd on and a parameter or input requiring grad, the differentiable path
        (videopainter_amd/autograd.py: gradient-checkpointed blocks on the HIP backward kernels) runs instead."""
        from . import autograd as AG
        if AG.needs_grad(self, hidden_states, encoder_hidden_states, branch_block_samples):
            if self_guidance_hidden_states is not None or self_guidance_masks is not None:
                raise NotImplementedError("self-guidance is inference-only (no training script passes it)")
            return self._forward_train(hidden_states, encoder_hidden_states, timestep, image_rotary_emb,
                                       attention_kwargs, branch_block_samples, branch_block_masks, add_first,
                                       self_guidance_hidden_states, return_hidden_states, return_resample_mask,
                                       id_pool_resample_learnable, timestep_cond, return_dict)
        if timestep_cond is not None:
            raise ValueError("timestep_cond requires a cond_proj, which CogVideoX's TimestepEmbedding does not have")
        attention_kwargs = dict(attention_kwargs) if attention_kwargs is not None else None
        # LoRA scale per call, default 1.0 (reference :490-499): the folded adapters are re-folded when it changes
        self._call_lora_scale(attention_kwargs)
        if attention_kwargs is not None:
            attention_kwargs.pop("scale", None)
        dev = self.proj_out.weight.device
        B, F, C, H, W = hidden_states.shape
        cfg = self.config
        p = cfg.patch_size
        hs = _bf(hidden_states.to(dev))
        enc = _bf(encoder_hidden_states.to(dev))
        T = enc.shape[1]
        Nv = F * (H // p) * (W // p)
        Ntok = T + Nv
        D = cfg.num_attention_heads * cfg.attention_head_dim

        emb = self._time_embed(timestep, B, dev)
        x = self.patch_embed.embed(enc, hs)
        # the token mask: from self_guidance_masks when given, else from branch_block_masks (reference :518-523); it
        # is the injection mask (when branch_block_masks is given), the resample mask and the self-guidance mask
        tok_mask = None
        mask_src = self_guidance_masks if self_guidance_masks is not None else branch_block_masks
        if mask_src is not None:
            tok_mask = K.patch_mask(mask_src.to(dev), p)
        if self_guidance_hidden_states is not None and tok_mask is None:
            # the reference reads an unbound `masks` here; we fail explicitly
            raise ValueError("self_guidance_hidden_states need self_guidance_masks or branch_block_masks")
        resample_mask = None
        if id_pool_resample_learnable or return_resample_mask:
            if tok_mask is None:
                # the reference reads an unbound `masks` here (UnboundLocalError); we fail explicitly
                raise ValueError("id_pool_resample needs masks")
            resample_mask = torch.zeros(B, Ntok, device=dev, dtype=torch.bool)
            resample_mask[:, T:] = tok_mask.bool()
        rope = _rope_dev(image_rotary_emb, dev, grid=(F, H // p, W // p))
        rm_u8 = _u8(resample_mask)

        prev_states = None
        prev_w = None
        prev_mask = None
        if attention_kwargs and "prev_hidden_states" in attention_kwargs:
            prev_states = attention_kwargs["prev_hidden_states"]
            prev_w = attention_kwargs.get("prev_clip_weight")
            prev_mask = _u8(attention_kwargs.get("prev_resample_mask"))

        bs = None
        if branch_block_samples is not None:
            bs = [_bf(s.to(dev)) for s in branch_block_samples]
        nl = len(self.transformer_blocks)
        interval = int(np.ceil(nl / len(bs))) if bs else 1
        hidden_states_list: List[torch.Tensor] = []
        ping = None
        for i, block in enumerate(self.transformer_blocks):
            inj = None
            if bs is not None:
                if not add_first:
                    inj = bs[i // interval]
                elif i < len(bs):
                    inj = bs[i]
            pj = None
            if prev_states is not None:
                pj = prev_states.get(i) if isinstance(prev_states, dict) else prev_states
            if return_hidden_states:
                out = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
            else:
                out = ping if (ping is not None and ping.data_ptr() != x.data_ptr()) else torch.empty_like(x)
                ping = x
            guide = None
            if self_guidance_hidden_states is not None:
                guide = _bf(self_guidance_hidden_states[i].to(dev))
            # (self-guidance replaces the unmasked video rows BEFORE the injection, reference :593-608: the block then
            # runs without its fused injection, and vp_guide_rows_bf16 applies both)
            x = block.forward_joint(x, T, emb, rope, rm_u8, pj, prev_w if pj is not None else None,
                                    prev_mask if pj is not None else None, inj if guide is None else None,
                                    tok_mask if (inj is not None and branch_block_masks is not None) else None, out)
            if guide is not None:
                xv = x[:, T:]
                K.guide_rows(xv, guide.expand_as(xv), tok_mask, inj, inject_all=branch_block_masks is None)
            if return_hidden_states:
                hidden_states_list.append(x)

        mod = K.linear_small(emb, self.norm_out.linear.weight, self.norm_out.linear.bias, act_in=K.ACT_SILU)
        if not cfg.use_rotary_positional_embeddings:
            raise NotImplementedError("CogVideoX-2B head (norm_final on video rows only) is not on the 5B-I2V path")
        y = K.final_norm(x, T, self.norm_final.weight, self.norm_final.bias, self.norm_out.norm.weight,
                         self.norm_out.norm.bias, self.norm_out.norm.eps, mod)
        proj = K.linear(y.view(B * Nv, D), self.proj_out.weight, self.proj_out.bias)
        output = K.unpatchify(proj, B, F, cfg.out_channels, H, W, p)

        if not return_dict:
            if return_hidden_states:
                if return_resample_mask:
                    return (output, hidden_states_list, resample_mask)
                return (output, hidden_states_list)
            return (output,)
        return Transformer2DModelOutput(sample=output)


    def _forward_train(self, hidden_states, encoder_hidden_states, timestep, image_rotary_emb, attention_kwargs,
                       branch_block_samples, branch_block_masks, add_first, self_guidance_hidden_states,
                       return_hidden_states, return_resample_mask, id_pool_resample_learnable, timestep_cond,
                       return_dict):
        """The training step's transformer call (train_cogvideox_inpainting_i2v_video.py:1867-1876): the same
        forward launches, every block a gradient-checkpointed autograd node."""
        from . import autograd as AG
        if timestep_cond is not None or self_guidance_hidden_states is not None:
            raise NotImplementedError("timestep_cond / self-guidance are not on the training path")
        if attention_kwargs and attention_kwargs.get("prev_hidden_states") is not None:
            raise NotImplementedError("the previous-clip blend is inference-only (no backward)")
        if return_hidden_states:
            raise NotImplementedError("return_hidden_states is inference-only (no backward)")
        self._call_lora_scale(attention_kwargs)
        dev = self.proj_out.weight.device
        B, F, C, H, W = hidden_states.shape
        cfg = self.config
        p = cfg.patch_size
        if not cfg.use_rotary_positional_embeddings:
            raise NotImplementedError("CogVideoX-2B head (norm_final on video rows only) is not on the 5B-I2V path")
        hs = _bf(hidden_states.to(dev))
        enc = _bf(encoder_hidden_states.to(dev))
        T = enc.shape[1]
        emb = self._time_embed(timestep, B, dev)
        x = AG.patch_embed_apply(self.patch_embed, enc, hs)
        tok_mask = None
        if branch_block_masks is not None:
            tok_mask = K.patch_mask(branch_block_masks.detach().to(dev), p)
        resample_mask = rm_u8 = None
        if id_pool_resample_learnable or return_resample_mask:
            # the VideoPainterID training step (train_cogvideox_inpainting_i2v_video_resample.py:1951-1961): window
            # 0's resample processor, differentiable (autograd.block_backward)
            if tok_mask is None:
                raise ValueError("id_pool_resample needs masks")
            resample_mask = torch.zeros(B, T + tok_mask.shape[1], device=dev, dtype=torch.bool)
            resample_mask[:, T:] = tok_mask.bool()
            rm_u8 = _u8(resample_mask)
        rope = _rope_dev(image_rotary_emb, dev, grid=(F, H // p, W // p))
        bs = None
        if branch_block_samples is not None:
            bs = [s.to(dev, BF16) for s in branch_block_samples]
        nl = len(self.transformer_blocks)
        interval = int(np.ceil(nl / len(bs))) if bs else 1
        for i, block in enumerate(self.transformer_blocks):
            inj = None
            if bs is not None:
                if not add_first:
                    inj = bs[i // interval]
                elif i < len(bs):
                    inj = bs[i]
            x = AG.block_apply(block, x, T, emb, rope, inj, tok_mask if inj is not None else None, rm_u8)
        output = AG.head_apply(self, x, emb, (B, F, H, W, T))
        if not return_dict:
            return (output,)  # (the reference returns the mask only together with the hidden states)
        return Transformer2DModelOutput(sample=output)


class AdaLayerNorm(nn.Module):
    """DF/models/normalization.py:31-85 with chunk_dim=1 (shift, scale order)."""

    def __init__(self, embedding_dim: int, output_dim: int, norm_elementwise_affine: bool, norm_eps: float):
        super().__init__()
        self.linear = Linear(embedding_dim, output_dim)
        self.norm = LayerNorm(output_dim // 2, norm_eps, norm_elementwise_affine)


def locals_without_self(loc: dict) -> dict:
    return {k: v for k, v in loc.items() if k not in ("self", "__class__")}
