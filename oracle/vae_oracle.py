"""CPU ORACLE for the CogVideoX 3D causal VAE — TEST INFRASTRUCTURE ONLY (same rules as cogvideox_oracle.py: only
tests/ and the bench's CPU baseline may import it; the product path `videopainter_amd.vae` never does).

A functional plain-PyTorch restatement of `AutoencoderKLCogVideoX` (DF/models/autoencoders/autoencoder_kl_cogvideox.py)
on diffusers state-dict keys: causal conv3d with the fake-context-parallel frame cache (:67-145), spatial norm (:148-188),
resnet blocks (:191-309), down / mid / up blocks (:312-608, DF/models/downsampling.py:288-353,
DF/models/upsampling.py:351-412), encoder / decoder (:611-883) and the frame-batched encode / decode (:1085-1190).
Pinned to the reference's own outputs by tests/golden/vae.safetensors (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


class Caches(dict):
    """conv prefix -> the last (kt - 1) input frames of the previous frame batch (CogVideoXCausalConv3d.conv_cache)."""


def causal_conv3d(sd: SD, p: str, x: torch.Tensor, caches: Caches, kt: int) -> torch.Tensor:
    """`CogVideoXCausalConv3d.forward` :133-145: prepend the cached frames (or kt-1 copies of the first frame),
    remember the last kt-1 input frames, zero-pad H/W by k//2, conv3d stride 1 (the SafeConv3d chunking :43-64 is a
    memory split with identical results)."""
    w = sd[p + ".conv.weight"]
    if kt > 1:
        prev = caches.get(p)
        head = [prev] if prev is not None else [x[:, :, :1]] * (kt - 1)
        x = torch.cat(head + [x], dim=2)
    caches[p] = x[:, :, -kt + 1:].clone() if kt > 1 else None
    kh, kw = w.shape[3], w.shape[4]
    x = F.pad(x, (kw // 2, kw // 2, kh // 2, kh // 2))
    return F.conv3d(x, w, sd[p + ".conv.bias"])


def group_norm(sd: SD, p: str, x, groups: int, eps: float):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], eps)


def spatial_norm(sd: SD, p: str, f, zq, groups: int, caches: Caches):
    """`CogVideoXSpatialNorm3D.forward` :175-188 (GroupNorm eps 1e-6; zq nearest-resized, first frame apart when f has an
    odd frame count > 1)."""
    if f.shape[2] > 1 and f.shape[2] % 2 == 1:
        z_first = F.interpolate(zq[:, :, :1], size=f[:, :, :1].shape[-3:])
        z_rest = F.interpolate(zq[:, :, 1:], size=f[:, :, 1:].shape[-3:])
        zq = torch.cat([z_first, z_rest], dim=2)
    else:
        zq = F.interpolate(zq, size=f.shape[-3:])
    n = F.group_norm(f, groups, sd[p + ".norm_layer.weight"], sd[p + ".norm_layer.bias"], 1e-6)
    return n * causal_conv3d(sd, p + ".conv_y", zq, caches, 1) + causal_conv3d(sd, p + ".conv_b", zq, caches, 1)


def resnet(sd: SD, p: str, x, caches: Caches, groups: int, eps: float, zq=None):
    """`CogVideoXResnetBlock3D.forward` :277-309 (temb_channels = 0 in the VAE; conv_shortcut = 1x1x1 SafeConv3d)."""
    h = spatial_norm(sd, p + ".norm1", x, zq, groups, caches) if zq is not None else group_norm(sd, p + ".norm1", x,
                                                                                                  groups, eps)
    h = causal_conv3d(sd, p + ".conv1", F.silu(h), caches, 3)
    h = spatial_norm(sd, p + ".norm2", h, zq, groups, caches) if zq is not None else group_norm(sd, p + ".norm2", h,
                                                                                                  groups, eps)
    h = causal_conv3d(sd, p + ".conv2", F.silu(h), caches, 3)
    if p + ".conv_shortcut.weight" in sd:
        x = F.conv3d(x, sd[p + ".conv_shortcut.weight"], sd[p + ".conv_shortcut.bias"])
    return h + x


def downsample(sd: SD, p: str, x, compress_time: bool):
    """`CogVideoXDownsample3D.forward` DF/models/downsampling.py:322-353."""
    if compress_time:
        b, c, t, h, w = x.shape
        x = x.permute(0, 3, 4, 1, 2).reshape(b * h * w, c, t)
        if x.shape[-1] % 2 == 1:
            first, rest = x[..., 0], x[..., 1:]
            if rest.shape[-1] > 0:
                rest = F.avg_pool1d(rest, kernel_size=2, stride=2)
            x = torch.cat([first[..., None], rest], dim=-1)
        else:
            x = F.avg_pool1d(x, kernel_size=2, stride=2)
        x = x.reshape(b, h, w, c, x.shape[-1]).permute(0, 3, 4, 1, 2)
    x = F.pad(x, (0, 1, 0, 1))
    b, c, t, h, w = x.shape
    x = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    x = F.conv2d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], stride=2)
    return x.reshape(b, t, x.shape[1], x.shape[2], x.shape[3]).permute(0, 2, 1, 3, 4)


def upsample(sd: SD, p: str, x, compress_time: bool):
    """`CogVideoXUpsample3D.forward` DF/models/upsampling.py:384-412."""
    if compress_time:
        if x.shape[2] > 1 and x.shape[2] % 2 == 1:
            first, rest = x[:, :, 0], x[:, :, 1:]
            first = F.interpolate(first, scale_factor=2.0)
            rest = F.interpolate(rest, scale_factor=2.0)
            x = torch.cat([first[:, :, None], rest], dim=2)
        elif x.shape[2] > 1:
            x = F.interpolate(x, scale_factor=2.0)
        else:
            x = F.interpolate(x.squeeze(2), scale_factor=2.0)[:, :, None]
    else:
        b, c, t, h, w = x.shape
        x = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
        x = F.interpolate(x, scale_factor=2.0)
        x = x.reshape(b, t, c, *x.shape[2:]).permute(0, 2, 1, 3, 4)
    b, c, t, h, w = x.shape
    x = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    x = F.conv2d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], padding=1)
    return x.reshape(b, t, *x.shape[1:]).permute(0, 2, 1, 3, 4)


def encoder(sd: SD, cfg: dict, x, caches: Caches):
    """`CogVideoXEncoder3D.forward` :708-742."""
    groups, eps = cfg["norm_num_groups"], cfg["norm_eps"]
    nb = len(cfg["block_out_channels"])
    tcl = int(math.log2(cfg["temporal_compression_ratio"]))
    h = causal_conv3d(sd, "encoder.conv_in", x, caches, 3)
    for i in range(nb):
        for j in range(cfg["layers_per_block"]):
            h = resnet(sd, f"encoder.down_blocks.{i}.resnets.{j}", h, caches, groups, eps)
        if i < nb - 1:
            h = downsample(sd, f"encoder.down_blocks.{i}.downsamplers.0", h, compress_time=i < tcl)
    for j in range(2):
        h = resnet(sd, f"encoder.mid_block.resnets.{j}", h, caches, groups, eps)
    h = F.silu(group_norm(sd, "encoder.norm_out", h, groups, 1e-6))
    return causal_conv3d(sd, "encoder.conv_out", h, caches, 3)


def decoder(sd: SD, cfg: dict, z, caches: Caches):
    """`CogVideoXDecoder3D.forward` :849-883 (spatial norms conditioned on the decoder's own input latent)."""
    groups, eps = cfg["norm_num_groups"], cfg["norm_eps"]
    nb = len(cfg["block_out_channels"])
    tcl = int(math.log2(cfg["temporal_compression_ratio"]))
    h = causal_conv3d(sd, "decoder.conv_in", z, caches, 3)
    for j in range(2):
        h = resnet(sd, f"decoder.mid_block.resnets.{j}", h, caches, groups, eps, zq=z)
    for i in range(nb):
        for j in range(cfg["layers_per_block"] + 1):
            h = resnet(sd, f"decoder.up_blocks.{i}.resnets.{j}", h, caches, groups, eps, zq=z)
        if i < nb - 1:
            h = upsample(sd, f"decoder.up_blocks.{i}.upsamplers.0", h, compress_time=i < tcl)
    h = F.silu(spatial_norm(sd, "decoder.norm_out", h, z, groups, caches))
    return causal_conv3d(sd, "decoder.conv_out", h, caches, 3)


def frame_batches(n: int, size: int, min_one: bool):
    """The reference's frame batching (:1091-1099 encode with size 8, :1144-1151 decode with size 2): batch 0 takes
    the remainder too."""
    nb = n // size if (n > 1 or not min_one) else 1
    if min_one and n <= 1:
        nb = 1
    out = []
    for i in range(nb):
        rem = n % size
        out.append((size * i + (0 if i == 0 else rem), size * (i + 1) + rem))
    return out


def _pointwise(sd: SD, p: str, x):
    """A 1x1x1 `CogVideoXSafeConv3d` (quant_conv / post_quant_conv, :979-980)."""
    return F.conv3d(x, sd[p + ".weight"], sd[p + ".bias"])


def encode(sd: SD, cfg: dict, x) -> torch.Tensor:
    """`AutoencoderKLCogVideoX._encode` :1085-1108 -> the latent_dist parameters (mean ++ logvar on channels);
    quant_conv after the encoder per frame batch when the config has it (:1101-1102)."""
    caches = Caches()
    parts = []
    for a, b in frame_batches(x.shape[2], 8, True):
        h = encoder(sd, cfg, x[:, :, a:b], caches)
        parts.append(_pointwise(sd, "quant_conv", h) if cfg.get("use_quant_conv") else h)
    return torch.cat(parts, dim=2)


def decode(sd: SD, cfg: dict, z) -> torch.Tensor:
    """`AutoencoderKLCogVideoX.decode` / `_decode` :1138-1190 (post_quant_conv before the decoder per frame batch when
    the config has it, :1152-1153)."""
    if z.shape[2] == 1:
        z = torch.cat([z, z], dim=2)
    caches = Caches()
    parts = []
    for a, b in frame_batches(z.shape[2], 2, False):
        zi = z[:, :, a:b]
        if cfg.get("use_post_quant_conv"):
            zi = _pointwise(sd, "post_quant_conv", zi)
        parts.append(decoder(sd, cfg, zi, caches))
    return torch.cat(parts, dim=2)


def latent_dist(params: torch.Tensor):
    """`DiagonalGaussianDistribution.__init__` DF/models/autoencoders/vae.py:768-778: (mean, logvar clamped to
    [-30, 20], std)."""
    mean, logvar = torch.chunk(params, 2, dim=1)
    logvar = torch.clamp(logvar, -30.0, 20.0)
    return mean, logvar, torch.exp(0.5 * logvar)


VAE_DEFAULTS = dict(in_channels=3, out_channels=3, block_out_channels=(128, 256, 256, 512), latent_channels=16,
                    layers_per_block=3, act_fn="silu", norm_eps=1e-6, norm_num_groups=32,
                    temporal_compression_ratio=4, sample_height=480, sample_width=720, scaling_factor=1.15258426)


def full_vae_config(kw: Optional[dict] = None) -> dict:
    c = dict(VAE_DEFAULTS)
    c.update(kw or {})
    return c


def _blend(a, b, extent, dim):
    """`blend_v` (dim 3) / `blend_h` (dim 4) :1192-1206, in place on b."""
    e = min(a.shape[dim], b.shape[dim], extent)
    for y in range(e):
        if dim == 3:
            b[:, :, :, y, :] = a[:, :, :, -e + y, :] * (1 - y / e) + b[:, :, :, y, :] * (y / e)
        else:
            b[:, :, :, :, y] = a[:, :, :, :, -e + y] * (1 - y / e) + b[:, :, :, :, y] * (y / e)
    return b


def tiled(sd: SD, cfg: dict, x, encode_: bool):
    """`tiled_encode` :1208-1277 / `tiled_decode` :1279-1358 with the default tile sizes of the config
    (sample_height // 2 x sample_width // 2, latent / 2^(levels - 1), overlap factors 1/6, 1/5)."""
    nb = len(cfg["block_out_channels"])
    ts_h, ts_w = cfg["sample_height"] // 2, cfg["sample_width"] // 2
    tl_h, tl_w = int(ts_h / (2 ** (nb - 1))), int(ts_w / (2 ** (nb - 1)))
    fh, fw = 1 / 6, 1 / 5
    tin_h, tin_w, tout_h, tout_w = (ts_h, ts_w, tl_h, tl_w) if encode_ else (tl_h, tl_w, ts_h, ts_w)
    ov_h, ov_w = int(tin_h * (1 - fh)), int(tin_w * (1 - fw))
    be_h, be_w = int(tout_h * fh), int(tout_w * fw)
    lim_h, lim_w = tout_h - be_h, tout_w - be_w
    run = (lambda t: encode(sd, cfg, t)) if encode_ else (lambda t: decode(sd, cfg, t))
    rows = [[run(x[:, :, :, i:i + tin_h, j:j + tin_w]) for j in range(0, x.shape[4], ov_w)]
            for i in range(0, x.shape[3], ov_h)]
    out = []
    for i, row in enumerate(rows):
        res = []
        for j, tile in enumerate(row):
            if i > 0:
                tile = _blend(rows[i - 1][j], tile, be_h, 3)
            if j > 0:
                tile = _blend(row[j - 1], tile, be_w, 4)
            res.append(tile[:, :, :, :lim_h, :lim_w])
        out.append(torch.cat(res, dim=4))
    return torch.cat(out, dim=3)
