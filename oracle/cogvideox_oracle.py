"""CPU ORACLE for the VideoPainter denoising hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module, and only as the
checker / the timed CPU baseline.  The product path (`videopainter_amd`) never imports it and fails loudly when its
HIP library is missing.

What it is: a functional, plain-PyTorch (CPU) restatement of the reference's per-step forward — the CogVideoX-5b-I2V
DiT (`CogVideoXTransformer3DModel.forward`), the 2-layer context-encoder branch (`CogvideoXBranchModel.forward`),
both attention processors (standard + ID-resample), the DPM-Solver scheduler step and the any-length pipeline's step
glue.  It consumes diffusers state-dict keys (a dict name -> tensor) and a config dict with the reference's
constructor kwargs.  Every function cites the reference file:line it restates; paths are relative to
`/root/reference/diffusers/src/diffusers/` (abbreviated DF/).

Pinning: `tests/golden/make_golden.py` imports the reference (vendored diffusers 0.31.0.dev0 fork, run in the survey
container) and records its outputs on deterministic weights; `tests/test_oracle_golden.py` checks this restatement
against those fixtures (fp32, rel err <= 1e-5).  The heavy arithmetic lives in torch itself (SDPA, Linear,
LayerNorm, GELU), exactly as in the reference (SURVEY.md §8c "Third-party arithmetic").

`dtype` selects the arithmetic dtype: float32 (the parity oracle) or bfloat16 (mimics the reference's bf16 rounding
points — used to state tolerance bands).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


# ------------------------------------------------------------------------------------------------------------------
# embeddings / tables
# ------------------------------------------------------------------------------------------------------------------

def timestep_embedding(timesteps: torch.Tensor, dim: int, flip_sin_to_cos: bool = True,
                       downscale_freq_shift: float = 0.0, max_period: int = 10000) -> torch.Tensor:
    """DF/models/embeddings.py:27-78 (`get_timestep_embedding`), as used by `Timesteps` (:777-793). fp32 out."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32)
    exponent = exponent / (half - downscale_freq_shift)
    emb = torch.exp(exponent)
    emb = timesteps[:, None].float() * emb[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def get_resize_crop_region_for_grid(src, tgt_width, tgt_height):
    """DF/pipelines/cogvideo/pipeline_cogvideox_inpainting_i2v_branch_anyl.py:68-83."""
    tw = tgt_width
    th = tgt_height
    h, w = src
    r = h / w
    if r > (th / tw):
        resize_height = th
        resize_width = int(round(th / h * w))
    else:
        resize_width = tw
        resize_height = int(round(tw / w * h))
    crop_top = int(round((th - resize_height) / 2.0))
    crop_left = int(round((tw - resize_width) / 2.0))
    return (crop_top, crop_left), (crop_top + resize_height, crop_left + resize_width)


def get_1d_rotary_pos_embed(dim: int, pos: np.ndarray, theta: float = 10000.0):
    """DF/models/embeddings.py:589-652 with use_real=True, repeat_interleave_real=True (CogVideoX form)."""
    pos_t = torch.from_numpy(pos)
    freqs = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float32)[: (dim // 2)] / dim))
    freqs = torch.outer(pos_t, freqs)
    return freqs.cos().repeat_interleave(2, dim=1).float(), freqs.sin().repeat_interleave(2, dim=1).float()


def get_3d_rotary_pos_embed(embed_dim, crops_coords, grid_size, temporal_size, theta: int = 10000):
    """DF/models/embeddings.py:457-522.  Returns (cos, sin) fp32 [T*H*W, embed_dim]; token order t, h, w."""
    start, stop = crops_coords
    gh, gw = grid_size
    grid_h = np.linspace(start[0], stop[0], gh, endpoint=False, dtype=np.float32)
    grid_w = np.linspace(start[1], stop[1], gw, endpoint=False, dtype=np.float32)
    grid_t = np.linspace(0, temporal_size, temporal_size, endpoint=False, dtype=np.float32)
    dim_t = embed_dim // 4
    dim_h = embed_dim // 8 * 3
    dim_w = embed_dim // 8 * 3
    ft = get_1d_rotary_pos_embed(dim_t, grid_t, theta)
    fh = get_1d_rotary_pos_embed(dim_h, grid_h, theta)
    fw = get_1d_rotary_pos_embed(dim_w, grid_w, theta)

    def combine(t, h, w):
        t = t[:, None, None, :].expand(-1, gh, gw, -1)
        h = h[None, :, None, :].expand(temporal_size, -1, gw, -1)
        w = w[None, None, :, :].expand(temporal_size, gh, -1, -1)
        return torch.cat([t, h, w], dim=-1).reshape(temporal_size * gh * gw, -1)

    return combine(ft[0], fh[0], fw[0]), combine(ft[1], fh[1], fw[1])


def prepare_rotary_positional_embeddings(height: int, width: int, num_frames: int, attention_head_dim: int = 64,
                                         vae_scale_factor_spatial: int = 8, patch_size: int = 2):
    """DF/pipelines/cogvideo/pipeline_cogvideox_inpainting_i2v_branch_anyl.py:589-613 (pixel height/width)."""
    grid_height = height // (vae_scale_factor_spatial * patch_size)
    grid_width = width // (vae_scale_factor_spatial * patch_size)
    base_w = 720 // (vae_scale_factor_spatial * patch_size)
    base_h = 480 // (vae_scale_factor_spatial * patch_size)
    crops = get_resize_crop_region_for_grid((grid_height, grid_width), base_w, base_h)
    return get_3d_rotary_pos_embed(attention_head_dim, crops, (grid_height, grid_width), num_frames)


def apply_rotary_emb(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """DF/models/embeddings.py:655-701 (use_real_unbind_dim=-1): interleaved pairs, fp32 math, cast back."""
    cos = cos[None, None]
    sin = sin[None, None]
    x_real, x_imag = x.reshape(*x.shape[:-1], -1, 2).unbind(-1)
    x_rot = torch.stack([-x_imag, x_real], dim=-1).flatten(3)
    return (x.float() * cos + x_rot.float() * sin).to(x.dtype)


# ------------------------------------------------------------------------------------------------------------------
# layers
# ------------------------------------------------------------------------------------------------------------------

def linear(x, sd: SD, p: str):
    """nn.Linear; with LoRA factors in the state dict (`<p>.lora_A.weight` [r, in], `<p>.lora_B.weight` [out, r] and
    the scaling `<p>.lora_scaling`), PEFT's UNMERGED LoRA Linear forward, which the reference runs for the
    VideoPainterID adapter (infer/inpaint.py:310-316: load_lora_weights, fuse_lora commented out; peft is an unpinned
    requirement, requirements.txt:21, not installed here — its published `lora.Linear.forward`:
    result = base_layer(x); result = result + lora_B(lora_A(dropout(x))) * scaling, dropout 0 at inference)."""
    y = F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))
    A = sd.get(p + ".lora_A.weight")
    if A is not None:
        y = y + F.linear(F.linear(x, A), sd[p + ".lora_B.weight"]) * float(sd[p + ".lora_scaling"])
    return y


def layer_norm(x, sd: SD, p: str, eps: float):
    return F.layer_norm(x, (x.shape[-1],), sd.get(p + ".weight"), sd.get(p + ".bias"), eps)


def time_embed(sd: SD, timestep: torch.Tensor, inner_dim: int, dtype) -> torch.Tensor:
    """`Timesteps` + `TimestepEmbedding` (DF/models/embeddings.py:729-793); transformer :508-515."""
    t_emb = timestep_embedding(timestep, inner_dim, True, 0).to(dtype)
    h = linear(t_emb, sd, "time_embedding.linear_1")
    h = F.silu(h)
    return linear(h, sd, "time_embedding.linear_2")


def patch_embed(sd: SD, cfg: dict, text_embeds, image_embeds, masks=None):
    """`CogVideoXPatchEmbed.forward` DF/models/embeddings.py:400-454 (learned pos-emb path)."""
    p = cfg["patch_size"]
    text = linear(text_embeds, sd, "patch_embed.text_proj")
    b, f, c, h, w = image_embeds.shape
    x = image_embeds.reshape(-1, c, h, w)
    x = F.conv2d(x, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=p)
    x = x.view(b, f, *x.shape[1:]).flatten(3).transpose(2, 3).flatten(1, 2)
    tok_mask = None
    if masks is not None:
        m = masks.reshape(-1, 1, h, w)
        m = F.avg_pool2d(m, kernel_size=p, stride=p)
        m = m.view(b, f, *m.shape[1:]).flatten(3).transpose(2, 3).flatten(1, 2)
        tok_mask = (m > 0.0).bool()  # [B, Nv, 1]
    embeds = torch.cat([text, x], dim=1).contiguous()
    if cfg.get("use_learned_positional_embeddings", False) or not cfg.get("use_rotary_positional_embeddings", False):
        if cfg.get("use_learned_positional_embeddings", False) and (cfg["sample_width"] != w or cfg["sample_height"] != h):
            raise ValueError("It is currently not possible to generate videos at a different resolution that the "
                             "defaults. This should only be the case with 'THUDM/CogVideoX-5b-I2V'.")
        pre_frames = (f - 1) * cfg.get("temporal_compression_ratio", 4) + 1
        if cfg["sample_frames"] != pre_frames or cfg["sample_height"] != h or cfg["sample_width"] != w:
            pos = sincos_joint_pos_embedding(cfg, h, w, pre_frames).to(embeds.dtype)
        else:
            pos = sd["patch_embed.pos_embedding"]
        embeds = embeds + pos
    return embeds, tok_mask


def sincos_joint_pos_embedding(cfg: dict, sample_height: int, sample_width: int, sample_frames: int):
    """`CogVideoXPatchEmbed._get_positional_embeddings` DF/models/embeddings.py:371-390 (+ get_3d_sincos :81-125)."""
    p = cfg["patch_size"]
    d = cfg["num_attention_heads"] * cfg["attention_head_dim"]
    ph, pw = sample_height // p, sample_width // p
    tf = (sample_frames - 1) // cfg.get("temporal_compression_ratio", 4) + 1
    si = cfg.get("spatial_interpolation_scale", 1.875)
    ti = cfg.get("temporal_interpolation_scale", 1.0)
    ds, dt = 3 * d // 4, d // 4

    def one_d(dim, pos):
        omega = np.arange(dim // 2, dtype=np.float64) / (dim / 2.0)
        omega = 1.0 / 10000 ** omega
        out = np.einsum("m,d->md", pos.reshape(-1), omega)
        return np.concatenate([np.sin(out), np.cos(out)], axis=1)

    grid_h = np.arange(ph, dtype=np.float32) / si
    grid_w = np.arange(pw, dtype=np.float32) / si
    grid = np.stack(np.meshgrid(grid_w, grid_h), axis=0).reshape([2, 1, ph, pw])
    emb_h = one_d(ds // 2, grid[0])
    emb_w = one_d(ds // 2, grid[1])
    spatial = np.concatenate([emb_h, emb_w], axis=1)
    temporal = one_d(dt, np.arange(tf, dtype=np.float32) / ti)
    spatial = np.repeat(spatial[None], tf, axis=0)
    temporal = np.repeat(temporal[:, None, :], ph * pw, axis=1)
    pe = np.concatenate([temporal, spatial], axis=-1).reshape(tf * ph * pw, d)
    joint = torch.zeros(1, cfg["max_text_seq_length"] + tf * ph * pw, d)
    joint[:, cfg["max_text_seq_length"]:] = torch.from_numpy(pe).float()
    return joint


def layer_norm_zero(sd: SD, p: str, h, e, temb, eps):
    """`CogVideoXLayerNormZero.forward` DF/models/normalization.py:373-379."""
    shift, scale, gate, enc_shift, enc_scale, enc_gate = linear(F.silu(temb), sd, p + ".linear").chunk(6, dim=1)
    h = layer_norm(h, sd, p + ".norm", eps) * (1 + scale)[:, None, :] + shift[:, None, :]
    e = layer_norm(e, sd, p + ".norm", eps) * (1 + enc_scale)[:, None, :] + enc_shift[:, None, :]
    return h, e, gate[:, None, :], enc_gate[:, None, :]


def _heads(x, b, heads):
    return x.view(b, -1, heads, x.shape[-1] // heads).transpose(1, 2)


def attn_standard(sd: SD, p: str, heads: int, h, e, rope, prev_hidden_states=None, prev_clip_weight=None):
    """`CogVideoXAttnProcessor2_0.__call__` DF/models/attention_processor.py:2107-2209 (incl. prev-clip :2156-2189)."""
    t = e.size(1)
    x = torch.cat([e, h], dim=1)
    b = x.shape[0]
    q = _heads(linear(x, sd, p + ".to_q"), b, heads)
    k = _heads(linear(x, sd, p + ".to_k"), b, heads)
    v = _heads(linear(x, sd, p + ".to_v"), b, heads)
    q = layer_norm(q, sd, p + ".norm_q", 1e-6)
    k = layer_norm(k, sd, p + ".norm_k", 1e-6)
    if rope is not None:
        q[:, :, t:] = apply_rotary_emb(q[:, :, t:], *rope)
        k[:, :, t:] = apply_rotary_emb(k[:, :, t:], *rope)
    if prev_hidden_states is not None and prev_clip_weight is not None and prev_clip_weight > 0.0:
        pk = _heads(linear(prev_hidden_states, sd, p + ".to_k"), b, heads)
        pv = _heads(linear(prev_hidden_states, sd, p + ".to_v"), b, heads)
        pk = layer_norm(pk, sd, p + ".norm_k", 1e-6)
        if rope is not None:
            pk[:, :, t:] = apply_rotary_emb(pk[:, :, t:], *rope)
        o = F.scaled_dot_product_attention(q, k, v) * (1 - prev_clip_weight)
        o = o + F.scaled_dot_product_attention(q, pk, pv) * prev_clip_weight
    else:
        o = F.scaled_dot_product_attention(q, k, v)
    o = o.transpose(1, 2).reshape(b, -1, q.shape[1] * q.shape[3])
    o = linear(o, sd, p + ".to_out.0")
    return o[:, t:], o[:, :t]


def attn_resample(sd: SD, p: str, heads: int, h, e, rope, resample_mask, prev_hidden_states=None,
                  prev_clip_weight=None, prev_resample_mask=None):
    """`CogVideoXAttnProcessor2_0_resample.__call__` DF/models/attention_processor.py:2223-2304.

    K/V are doubled along the sequence with masked copies; masking happens before norm_k, so masked tokens get
    key = RoPE(beta_k) and value 0 (SURVEY.md finding 5)."""
    t = e.size(1)
    x = torch.cat([e, h], dim=1)
    b = x.shape[0]
    q = linear(x, sd, p + ".to_q")
    k = linear(x, sd, p + ".to_k")
    v = linear(x, sd, p + ".to_v")
    if prev_hidden_states is not None and prev_clip_weight is not None and prev_clip_weight > 0.0:
        pk = linear(prev_hidden_states, sd, p + ".to_k")
        pv = linear(prev_hidden_states, sd, p + ".to_v")
        km = pk * prev_resample_mask.unsqueeze(-1) * prev_clip_weight
        vm = pv * prev_resample_mask.unsqueeze(-1) * prev_clip_weight
    else:
        km = k * resample_mask.unsqueeze(-1)
        vm = v * resample_mask.unsqueeze(-1)
    q, k, v, km, vm = (_heads(z, b, heads) for z in (q, k, v, km, vm))
    q = layer_norm(q, sd, p + ".norm_q", 1e-6)
    k = layer_norm(k, sd, p + ".norm_k", 1e-6)
    km = layer_norm(km, sd, p + ".norm_k", 1e-6)
    if rope is not None:
        q[:, :, t:] = apply_rotary_emb(q[:, :, t:], *rope)
        k[:, :, t:] = apply_rotary_emb(k[:, :, t:], *rope)
        km[:, :, t:] = apply_rotary_emb(km[:, :, t:], *rope)
    k = torch.cat([k, km], dim=-2)
    v = torch.cat([v, vm], dim=-2)
    o = F.scaled_dot_product_attention(q, k, v)
    o = o.transpose(1, 2).reshape(b, -1, q.shape[1] * q.shape[3])
    o = linear(o, sd, p + ".to_out.0")
    return o[:, t:], o[:, :t]


def feed_forward(sd: SD, p: str, x):
    """`FeedForward` DF/models/attention.py:1144-1202 with GELU(approximate='tanh') DF/models/activations.py:65-90."""
    x = linear(x, sd, p + ".net.0.proj")
    x = F.gelu(x, approximate="tanh")
    return linear(x, sd, p + ".net.2")


def block_forward(sd: SD, p: str, cfg: dict, h, e, temb, rope, resample_mask=None, attention_kwargs=None,
                  resample: bool = False):
    """`CogVideoXBlock.forward` DF/models/transformers/cogvideox_transformer_3d.py:125-184."""
    eps = cfg.get("norm_eps", 1e-5)
    heads = cfg["num_attention_heads"]
    t = e.size(1)
    nh, ne, gate, enc_gate = layer_norm_zero(sd, p + ".norm1", h, e, temb, eps)
    kw = dict(attention_kwargs or {})
    if "prev_hidden_states" in kw and kw["prev_hidden_states"] is not None:
        prev = kw["prev_hidden_states"]
        pe_, ph_ = prev[:, :t], prev[:, t:]
        nph, npe, _, _ = layer_norm_zero(sd, p + ".norm1", ph_, pe_, temb, eps)
        kw["prev_hidden_states"] = torch.cat([npe, nph], dim=1)
    if resample:
        ah, ae = attn_resample(sd, p + ".attn1", heads, nh, ne, rope, resample_mask,
                               kw.get("prev_hidden_states"), kw.get("prev_clip_weight"), kw.get("prev_resample_mask"))
    else:
        ah, ae = attn_standard(sd, p + ".attn1", heads, nh, ne, rope, kw.get("prev_hidden_states"),
                               kw.get("prev_clip_weight"))
    h = h + gate * ah
    e = e + enc_gate * ae
    nh, ne, gate_ff, enc_gate_ff = layer_norm_zero(sd, p + ".norm2", h, e, temb, eps)
    ff = feed_forward(sd, p + ".ff", torch.cat([ne, nh], dim=1))
    h = h + gate_ff * ff[:, t:]
    e = e + enc_gate_ff * ff[:, :t]
    return h, e


def transformer_forward(sd: SD, cfg: dict, hidden_states, encoder_hidden_states, timestep, image_rotary_emb=None,
                        attention_kwargs=None, branch_block_samples=None, branch_block_masks=None, add_first=False,
                        return_hidden_states=False, return_resample_mask=False, id_pool_resample_learnable=False,
                        self_guidance_hidden_states=None, self_guidance_masks=None):
    """`CogVideoXTransformer3DModel.forward` DF/models/transformers/cogvideox_transformer_3d.py:472-646.
    self_guidance_masks replace branch_block_masks as the token mask (:518-523); the guidance states take the
    unmasked video rows after every block, before the injection (:593-594).

    Returns the tuple form (`return_dict=False`, :638-645)."""
    dtype = hidden_states.dtype
    inner = cfg["num_attention_heads"] * cfg["attention_head_dim"]
    attention_kwargs = dict(attention_kwargs) if attention_kwargs else None
    if attention_kwargs is not None:
        attention_kwargs.pop("scale", None)
    b, f, c, hh, ww = hidden_states.shape
    emb = time_embed(sd, timestep, inner, dtype)
    masks = None
    x, tok_mask = patch_embed(sd, cfg, encoder_hidden_states, hidden_states,
                              self_guidance_masks if self_guidance_masks is not None else branch_block_masks)
    if tok_mask is not None:
        masks = tok_mask.repeat(1, 1, x.shape[-1] // tok_mask.shape[-1])
    t = encoder_hidden_states.shape[1]
    e, h = x[:, :t], x[:, t:]
    resample = bool(cfg.get("id_pool_resample_learnable", False))
    resample_mask = None
    if id_pool_resample_learnable or return_resample_mask:
        if masks is None:
            raise ValueError("id_pool_resample needs masks")
        resample_mask = torch.zeros((b, t + h.shape[1]), dtype=torch.bool)
        resample_mask[:, t:] = masks[:, :, 0].bool()
    hs_list = []
    nl = len([k for k in sd if k.endswith(".norm1.linear.weight") and k.startswith("transformer_blocks.")])
    for i in range(nl):
        kw = {}
        if attention_kwargs:
            kw = dict(attention_kwargs)
            if "prev_hidden_states" in attention_kwargs:
                ls = attention_kwargs["prev_hidden_states"].get(i)
                if ls is not None:
                    kw["prev_hidden_states"] = ls
                    kw["prev_clip_weight"] = attention_kwargs["prev_clip_weight"]
                else:
                    kw.pop("prev_hidden_states")
                prm = attention_kwargs.get("prev_resample_mask")
                if prm is not None:
                    kw["prev_resample_mask"] = prm
        h, e = block_forward(sd, f"transformer_blocks.{i}", cfg, h, e, emb, image_rotary_emb, resample_mask, kw,
                             resample)
        if self_guidance_hidden_states is not None:
            h = torch.where(masks == False, self_guidance_hidden_states[i], h)  # noqa: E712
        if branch_block_samples is not None:
            if not add_first:
                interval = int(np.ceil(nl / len(branch_block_samples)))
                if branch_block_masks is None:
                    h = h + branch_block_samples[i // interval]
                else:
                    h = torch.where(masks == False, h + branch_block_samples[i // interval], h)  # noqa: E712
            elif i < len(branch_block_samples):
                if branch_block_masks is None:
                    h = h + branch_block_samples[i]
                else:
                    h = torch.where(masks == False, h + branch_block_samples[i], h)  # noqa: E712
        if return_hidden_states:
            hs_list.append(torch.cat([e, h], dim=1))
    eps = cfg.get("norm_eps", 1e-5)
    if not cfg.get("use_rotary_positional_embeddings", False):
        h = layer_norm(h, sd, "norm_final", eps)
    else:
        h = layer_norm(torch.cat([e, h], dim=1), sd, "norm_final", eps)[:, t:]
    mod = linear(F.silu(emb), sd, "norm_out.linear")
    shift, scale = mod.chunk(2, dim=1)
    h = layer_norm(h, sd, "norm_out.norm", eps) * (1 + scale[:, None, :]) + shift[:, None, :]
    h = linear(h, sd, "proj_out")
    p = cfg["patch_size"]
    out = h.reshape(b, f, hh // p, ww // p, -1, p, p).permute(0, 1, 4, 2, 5, 3, 6).flatten(5, 6).flatten(3, 4)
    if return_hidden_states:
        if return_resample_mask:
            return out, hs_list, resample_mask
        return out, hs_list
    return (out,)


def layer_norm_zero_wo_text(sd: SD, p: str, h, temb, eps):
    """`CogVideoXLayerNormZero.forward_wo_text` DF/models/normalization.py:381-386 (the video chunks only)."""
    shift, scale, gate, _, _, _ = linear(F.silu(temb), sd, p + ".linear").chunk(6, dim=1)
    h = layer_norm(h, sd, p + ".norm", eps) * (1 + scale)[:, None, :] + shift[:, None, :]
    return h, gate[:, None, :]


def attn_wo_text(sd: SD, p: str, heads: int, h, rope):
    """`CogVideoXAttnProcessor2_0_wo_text.__call__` DF/models/attention_processor.py:2306-2366: self-attention over
    the video tokens alone, RoPE on every token."""
    b = h.shape[0]
    q = _heads(linear(h, sd, p + ".to_q"), b, heads)
    k = _heads(linear(h, sd, p + ".to_k"), b, heads)
    v = _heads(linear(h, sd, p + ".to_v"), b, heads)
    q = layer_norm(q, sd, p + ".norm_q", 1e-6)
    k = layer_norm(k, sd, p + ".norm_k", 1e-6)
    if rope is None:
        # the reference computes the attention inside its `if image_rotary_emb is not None:` (:2349-2356): without
        # RoPE its input goes on to the head merge (:2358, transpose(1, 2) of a [B, N, D] tensor) and to_out
        return linear(h.transpose(1, 2).reshape(b, -1, h.shape[-1]), sd, p + ".to_out.0")
    q = apply_rotary_emb(q, *rope)
    k = apply_rotary_emb(k, *rope)
    o = F.scaled_dot_product_attention(q, k, v)
    o = o.transpose(1, 2).reshape(b, -1, q.shape[1] * q.shape[3])
    return linear(o, sd, p + ".to_out.0")


def block_forward_wo_text(sd: SD, p: str, cfg: dict, h, temb, rope):
    """`CogVideoXBlock.forward_wo_text` DF/models/transformers/cogvideox_transformer_3d.py:186-216."""
    eps = cfg.get("norm_eps", 1e-5)
    nh, gate = layer_norm_zero_wo_text(sd, p + ".norm1", h, temb, eps)
    h = h + gate * attn_wo_text(sd, p + ".attn1", cfg["num_attention_heads"], nh, rope)
    nh, gate_ff = layer_norm_zero_wo_text(sd, p + ".norm2", h, temb, eps)
    return h + gate_ff * feed_forward(sd, p + ".ff", nh)


def branch_forward(sd: SD, cfg: dict, hidden_states, encoder_hidden_states, branch_cond, timestep,
                   image_rotary_emb=None, conditioning_scale=1.0, wo_text=False):
    """`CogvideoXBranchModel.forward` DF/models/branch_cogvideox.py:295-434 (wo_text: the blocks' forward_wo_text on
    the video tokens, :400-412; the text embedding is computed and left unused, :362-366).  Returns the list."""
    dtype = hidden_states.dtype
    inner = cfg["num_attention_heads"] * cfg["attention_head_dim"]
    emb = time_embed(sd, timestep, inner, dtype)
    x, _ = patch_embed(sd, cfg, encoder_hidden_states, torch.concat([hidden_states, branch_cond], dim=-3))
    t = encoder_hidden_states.shape[1]
    e, h = x[:, :t], x[:, t:]
    nl = len([k for k in sd if k.endswith(".norm1.linear.weight") and k.startswith("transformer_blocks.")])
    samples = []
    for i in range(nl):
        if wo_text:
            h = block_forward_wo_text(sd, f"transformer_blocks.{i}", cfg, h, emb, image_rotary_emb)
        else:
            h, e = block_forward(sd, f"transformer_blocks.{i}", cfg, h, e, emb, image_rotary_emb)
        samples.append(h)
    outs = [linear(s, sd, f"branch_blocks.{j}") for j, s in enumerate(samples)]
    return [(o * conditioning_scale).to(dtype) for o in outs]


# ------------------------------------------------------------------------------------------------------------------
# scheduler + step glue
# ------------------------------------------------------------------------------------------------------------------

class DPMSchedulerOracle:
    """`CogVideoXDPMScheduler` DF/schedulers/scheduling_dpm_cogvideox.py:181-486 (scaled_linear, v_prediction)."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012, snr_shift_scale=1.0,
                 rescale_betas_zero_snr=True, set_alpha_to_one=True, timestep_spacing="trailing"):
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float64) ** 2
        ac = torch.cumprod(1.0 - betas, dim=0)
        ac = ac / (snr_shift_scale + (1 - snr_shift_scale) * ac)
        if rescale_betas_zero_snr:
            s = ac.sqrt()
            s0, sT = s[0].clone(), s[-1].clone()
            s -= sT
            s *= s0 / (s0 - sT)
            ac = s ** 2
        self.alphas_cumprod = ac
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else ac[0]
        self.num_train_timesteps = num_train_timesteps
        self.timestep_spacing = timestep_spacing
        self.num_inference_steps = None

    def set_timesteps(self, n):
        """:261-304 (trailing)."""
        self.num_inference_steps = n
        ratio = self.num_train_timesteps / n
        ts = np.round(np.arange(self.num_train_timesteps, 0, -ratio)).astype(np.int64) - 1
        self.timesteps = torch.from_numpy(ts)
        return self.timesteps

    def coefficients(self, timestep: int, timestep_back: Optional[int]):
        """:306-328 + :386-406.  fp64 scalars (0-dim tensors, as in the reference)."""
        prev_t = timestep - self.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[timestep]
        a_prev = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.final_alpha_cumprod
        a_back = self.alphas_cumprod[timestep_back] if timestep_back is not None else None
        lamb = ((a_t / (1 - a_t)) ** 0.5).log()
        lamb_next = ((a_prev / (1 - a_prev)) ** 0.5).log()
        h = lamb_next - lamb
        mult1 = ((1 - a_prev) / (1 - a_t)) ** 0.5 * (-h).exp()
        mult2 = (-2 * h).expm1() * a_prev ** 0.5
        mult3 = mult4 = None
        if a_back is not None:
            lamb_prev = ((a_back / (1 - a_back)) ** 0.5).log()
            r = (lamb - lamb_prev) / h
            mult3 = 1 + 1 / (2 * r)
            mult4 = 1 / (2 * r)
        mult_noise = (1 - a_prev) ** 0.5 * (1 - (-2 * h).exp()) ** 0.5
        return dict(prev_t=prev_t, a_t=a_t, a_prev=a_prev, mult1=mult1, mult2=mult2, mult3=mult3, mult4=mult4,
                    mult_noise=mult_noise)

    def step(self, model_output, old_pred_original_sample, timestep, timestep_back, sample, noise1, noise2):
        """:330-439 with the stochastic noises passed in (the reference draws them from the CPU generator)."""
        c = self.coefficients(int(timestep), None if timestep_back is None else int(timestep_back))
        beta_t = 1 - c["a_t"]
        pred = (c["a_t"] ** 0.5) * sample - (beta_t ** 0.5) * model_output
        prev_sample = c["mult1"] * sample - c["mult2"] * pred + c["mult_noise"] * noise1
        if old_pred_original_sample is None or c["prev_t"] < 0:
            return prev_sample, pred
        denoised_d = c["mult3"] * pred - c["mult4"] * old_pred_original_sample
        x_adv = c["mult1"] * sample - c["mult2"] * denoised_d + c["mult_noise"] * noise2
        return x_adv, pred

    def add_noise(self, original, noise, timesteps):
        """:442-466 (alphas cast to the sample dtype first)."""
        ac = self.alphas_cumprod.to(dtype=original.dtype)
        sa = ac[timesteps] ** 0.5
        sb = (1 - ac[timesteps]) ** 0.5
        while sa.dim() < original.dim():
            sa = sa.unsqueeze(-1)
            sb = sb.unsqueeze(-1)
        return sa * original + sb * noise


def dynamic_cfg_scale(guidance_scale: float, num_inference_steps: int, t: int) -> float:
    """anyl.py:991-994 (uses the raw timestep t, a reference quirk)."""
    return 1 + guidance_scale * ((1 - math.cos(math.pi * ((num_inference_steps - t) / num_inference_steps) ** 5.0)) / 2)
