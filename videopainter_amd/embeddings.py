"""Host-side position tables (computed once per window, like the reference, then kept resident in HBM).

  get_resize_crop_region_for_grid  DF/pipelines/cogvideo/pipeline_cogvideox_inpainting_i2v_branch_anyl.py:68-83
  get_3d_rotary_pos_embed          DF/models/embeddings.py:457-522 (+ get_1d_rotary_pos_embed :589-652)
  CogVideoX joint sin-cos pos-emb  DF/models/embeddings.py:371-390, get_3d_sincos_pos_embed :81-125

The RoPE tables are (cos, sin) fp32 [F*Hp*Wp, head_dim] in the reference's token order (t, h, w) with the
repeat_interleave(2) pair layout that `vp_head_norm_rope_bf16` consumes.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch


def get_resize_crop_region_for_grid(src, tgt_width, tgt_height):
    h, w = src
    r = h / w
    if r > (tgt_height / tgt_width):
        resize_height = tgt_height
        resize_width = int(round(tgt_height / h * w))
    else:
        resize_width = tgt_width
        resize_height = int(round(tgt_width / w * h))
    crop_top = int(round((tgt_height - resize_height) / 2.0))
    crop_left = int(round((tgt_width - resize_width) / 2.0))
    return (crop_top, crop_left), (crop_top + resize_height, crop_left + resize_width)


def _rope_1d(dim: int, pos: np.ndarray, theta: float = 10000.0):
    # fp32 like the reference: freqs = 1 / theta^(arange(0, dim, 2)/dim); outer(pos, freqs); cos/sin; interleave
    idx = torch.arange(0, dim, 2, dtype=torch.float32)[: dim // 2]
    freqs = 1.0 / (theta ** (idx / dim))
    f = torch.outer(torch.from_numpy(pos), freqs)
    return f.cos().repeat_interleave(2, dim=1), f.sin().repeat_interleave(2, dim=1)


def get_3d_rotary_pos_embed(embed_dim: int, crops_coords, grid_size, temporal_size: int, theta: int = 10000):
    (s0, s1), (e0, e1) = crops_coords
    gh, gw = grid_size
    grid_h = np.linspace(s0, e0, gh, endpoint=False, dtype=np.float32)
    grid_w = np.linspace(s1, e1, gw, endpoint=False, dtype=np.float32)
    grid_t = np.linspace(0, temporal_size, temporal_size, endpoint=False, dtype=np.float32)
    dt, dh, dw = embed_dim // 4, embed_dim // 8 * 3, embed_dim // 8 * 3
    tc, ts = _rope_1d(dt, grid_t, theta)
    hc, hs = _rope_1d(dh, grid_h, theta)
    wc, ws = _rope_1d(dw, grid_w, theta)

    def comb(t, h, w):
        t = t[:, None, None, :].expand(-1, gh, gw, -1)
        h = h[None, :, None, :].expand(temporal_size, -1, gw, -1)
        w = w[None, None, :, :].expand(temporal_size, gh, -1, -1)
        return torch.cat([t, h, w], dim=-1).reshape(temporal_size * gh * gw, -1).contiguous()

    return comb(tc, hc, wc), comb(ts, hs, ws)


def prepare_rotary_positional_embeddings(height: int, width: int, num_frames: int, attention_head_dim: int = 64,
                                         vae_scale_factor_spatial: int = 8, patch_size: int = 2,
                                         device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """`CogVideoXI2VDualInpaintAnyLPipeline._prepare_rotary_positional_embeddings` (pixel height/width, latent
    frames)."""
    gh = height // (vae_scale_factor_spatial * patch_size)
    gw = width // (vae_scale_factor_spatial * patch_size)
    base_w = 720 // (vae_scale_factor_spatial * patch_size)
    base_h = 480 // (vae_scale_factor_spatial * patch_size)
    crops = get_resize_crop_region_for_grid((gh, gw), base_w, base_h)
    cos, sin = get_3d_rotary_pos_embed(attention_head_dim, crops, (gh, gw), num_frames)
    if device is not None:
        cos, sin = cos.to(device), sin.to(device)
    return cos, sin


def _sincos_1d(dim: int, pos: np.ndarray) -> np.ndarray:
    omega = np.arange(dim // 2, dtype=np.float64) / (dim / 2.0)
    omega = 1.0 / 10000 ** omega
    out = np.einsum("m,d->md", pos.reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


def joint_sincos_pos_embedding(embed_dim: int, patch_size: int, max_text_seq_length: int, sample_height: int,
                               sample_width: int, sample_frames: int, temporal_compression_ratio: int = 4,
                               spatial_interpolation_scale: float = 1.875,
                               temporal_interpolation_scale: float = 1.0) -> torch.Tensor:
    """[1, T + F*Hp*Wp, D] fp32; text rows zero."""
    ph, pw = sample_height // patch_size, sample_width // patch_size
    tf = (sample_frames - 1) // temporal_compression_ratio + 1
    ds, dt = 3 * embed_dim // 4, embed_dim // 4
    grid_h = np.arange(ph, dtype=np.float32) / spatial_interpolation_scale
    grid_w = np.arange(pw, dtype=np.float32) / spatial_interpolation_scale
    grid = np.stack(np.meshgrid(grid_w, grid_h), axis=0).reshape([2, 1, ph, pw])
    spatial = np.concatenate([_sincos_1d(ds // 2, grid[0]), _sincos_1d(ds // 2, grid[1])], axis=1)
    temporal = _sincos_1d(dt, np.arange(tf, dtype=np.float32) / temporal_interpolation_scale)
    spatial = np.repeat(spatial[None], tf, axis=0)
    temporal = np.repeat(temporal[:, None, :], ph * pw, axis=1)
    pe = np.concatenate([temporal, spatial], axis=-1).reshape(tf * ph * pw, embed_dim)
    joint = torch.zeros(1, max_text_seq_length + tf * ph * pw, embed_dim)
    joint[:, max_text_seq_length:] = torch.from_numpy(pe).float()
    return joint
