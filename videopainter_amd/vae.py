"""`AutoencoderKLCogVideoX` on the HIP kernels: the CogVideoX 3D causal VAE encode / decode the
any-length pipeline calls per window (prepare_latents / decode_latents, anyl.py:366-372, 423-430, 479-483).

Reference: DF/models/autoencoders/autoencoder_kl_cogvideox.py (class :886-1376, encoder :611-742, decoder :745-883,
resnet :191-309, spatial norm :148-188, causal conv :67-145), DF/models/downsampling.py:288-353,
DF/models/upsampling.py:351-412, DiagonalGaussianDistribution DF/models/autoencoders/vae.py:767-830.

Same constructor kwargs, state-dict keys, `encode` / `decode` / `forward` return forms, frame batching (8 sample
frames / 2 latent frames per encoder / decoder call, with the causal-conv frame caches carried across calls), slicing
and tiling (tiles blended in place in the reference's order) as the reference.  Every arithmetic op runs in
libvp_hip.so on channels-last bf16 activations:

  CausalConv3d / conv_shortcut / Downsample3D conv / Upsample3D (nearest x2 + conv)  -> vp_conv3d_bf16 (one
      implicit-GEMM MFMA kernel; the causal frame cache is the conv's second frame source, the nearest upsampling
      and the temporal frame repeat are folded into its gather, the resnet residual into its epilogue)
  GroupNorm (+ SiLU), SpatialNorm3D (GroupNorm * conv_y(zq) + conv_b(zq), zq nearest-resized)
      -> vp_group_norm_stats + vp_group_norm_apply_bf16 (conv_y | conv_b run once at latent resolution: a 1x1x1
         conv commutes with nearest resizing, so the apply kernel gathers the modulation at the nearest source)
  Downsample3D temporal avg-pool -> vp_time_pool2_bf16;  DiagonalGaussianDistribution -> vp_latent_dist_bf16;
  blend_v / blend_h -> vp_tile_blend_bf16;  NCDHW <-> channels-last -> vp_ncdhw_to_ndhwc / vp_ndhwc_to_ncdhw.

Torch only allocates, slices, concatenates and copies (frame caches, tile crops).  Outputs are bfloat16 (the
pipeline runs the VAE in bf16); inputs may be float32 or bfloat16.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import kernels as K
from . import weights as W
from .config import full_vae_config, vae_state_dict_shapes
from .modules import FrozenConfig, device_scope  # noqa: F401  (device_scope: same construction idiom)
from . import modules as _M


def _on(t: torch.Tensor):
    return torch.cuda.device(t.device) if t.is_cuda else contextlib.nullcontext()


def _cpad(c: int) -> int:
    """Channel count of the channels-last activation holding c channels: a power of two >= 8."""
    p = 8
    while p < c:
        p *= 2
    return p


def _nearest_map(n_out: int, n_in: int) -> List[int]:
    """torch's nearest rule (upsample_nearest: float scale in / out, floor, clamp) for an explicit output size."""
    if n_out == n_in:
        return list(range(n_out))
    scale = np.float32(n_in) / np.float32(n_out)
    return [min(int(np.floor(np.float32(i) * scale)), n_in - 1) for i in range(n_out)]


def _spatial_norm_tmap(tf: int, tz: int) -> List[int]:
    """`CogVideoXSpatialNorm3D.forward` :176-184: the zq frame of each f frame (first frame apart when f has an odd
    frame count > 1)."""
    if tf > 1 and tf % 2 == 1:
        return [0] + [1 + v for v in _nearest_map(tf - 1, tz - 1)]
    return _nearest_map(tf, tz)


class DiagonalGaussianDistribution:
    """DF/models/autoencoders/vae.py:767-830 on the encoder output (mean / clamped logvar made by vp_latent_dist_bf16);
    `sample` draws the noise like the reference (randn_tensor on the caller's generator) and combines on the GPU."""

    def __init__(self, params_nhwc: torch.Tensor, latent_channels: int, deterministic: bool = False):
        self._p = params_nhwc
        self._L = latent_channels
        self.mean, self.logvar = K.latent_dist(params_nhwc, latent_channels)
        self.deterministic = deterministic

    @property
    def parameters(self) -> torch.Tensor:
        return K.ndhwc_to_ncdhw(self._p, 2 * self._L)

    def sample_from(self, noise: torch.Tensor) -> torch.Tensor:
        """mean + exp(0.5 logvar) * noise on the GPU (vp_latent_dist_bf16)."""
        return K.latent_dist(self._p, self._L, noise.to(device=self.mean.device, dtype=torch.bfloat16))[2]

    def sample(self, generator: Optional[torch.Generator] = None) -> torch.Tensor:
        if self.deterministic:
            return self.mean
        gdev = generator.device if generator is not None else self.mean.device
        noise = torch.randn(self.mean.shape, generator=generator, device=gdev, dtype=torch.bfloat16)
        return self.sample_from(noise)

    def mode(self) -> torch.Tensor:
        return self.mean


@dataclass
class AutoencoderKLOutput:
    latent_dist: DiagonalGaussianDistribution


@dataclass
class DecoderOutput:
    sample: torch.Tensor
    commit_loss: Optional[torch.Tensor] = None


class _Node(nn.Module):
    """A level of the reference's module tree (only holds parameters: state-dict keys load unchanged)."""


class AutoencoderKLCogVideoX(nn.Module):
    """Drop-in for `AutoencoderKLCogVideoX` (autoencoder_kl_cogvideox.py:886-1376), inference only."""

    config_name = W.CONFIG_NAME
    _supports_gradient_checkpointing = True

    def __init__(self, in_channels: int = 3, out_channels: int = 3,
                 down_block_types: Tuple[str, ...] = ("CogVideoXDownBlock3D",) * 4,
                 up_block_types: Tuple[str, ...] = ("CogVideoXUpBlock3D",) * 4,
                 block_out_channels: Tuple[int, ...] = (128, 256, 256, 512), latent_channels: int = 16,
                 layers_per_block: int = 3, act_fn: str = "silu", norm_eps: float = 1e-6, norm_num_groups: int = 32,
                 temporal_compression_ratio: float = 4, sample_height: int = 480, sample_width: int = 720,
                 scaling_factor: float = 1.15258426, shift_factor: Optional[float] = None,
                 latents_mean: Optional[Tuple[float]] = None, latents_std: Optional[Tuple[float]] = None,
                 force_upcast: float = True, use_quant_conv: bool = False, use_post_quant_conv: bool = False):
        nn.Module.__init__(self)  # never a re-based library base's __init__ (integration.install)
        cfg = full_vae_config(dict(
            in_channels=in_channels, out_channels=out_channels, down_block_types=tuple(down_block_types),
            up_block_types=tuple(up_block_types), block_out_channels=tuple(block_out_channels),
            latent_channels=latent_channels, layers_per_block=layers_per_block, act_fn=act_fn, norm_eps=norm_eps,
            norm_num_groups=norm_num_groups, temporal_compression_ratio=temporal_compression_ratio,
            sample_height=sample_height, sample_width=sample_width, scaling_factor=scaling_factor,
            shift_factor=shift_factor, latents_mean=latents_mean, latents_std=latents_std,
            force_upcast=force_upcast, use_quant_conv=use_quant_conv, use_post_quant_conv=use_post_quant_conv))
        if (use_quant_conv or use_post_quant_conv) and out_channels != latent_channels:
            # the reference builds them with 2*out_channels / out_channels (pixel) channels (:979-980) and applies them
            # to the 2*latent_channels encoder output / the latents (:1101-1102, :1152-1153): only a config with
            # out_channels == latent_channels runs (no CogVideoX checkpoint enables them); the reference fails at its
            # first encode / decode, the drop-in at construction
            raise ValueError("use_quant_conv / use_post_quant_conv need out_channels == latent_channels "
                             f"(got {out_channels} / {latent_channels})")
        if any(t != "CogVideoXDownBlock3D" for t in down_block_types) or \
                any(t != "CogVideoXUpBlock3D" for t in up_block_types):
            raise ValueError("Invalid block type: must be CogVideoXDownBlock3D / CogVideoXUpBlock3D")
        if act_fn not in ("silu", "swish"):
            raise NotImplementedError(f"act_fn {act_fn!r} (CogVideoX uses silu)")
        for c in block_out_channels:
            if c != _cpad(c) or c % norm_num_groups:
                raise NotImplementedError("block_out_channels must be powers of two >= 8 divisible by the groups")
        object.__setattr__(self, "_internal_config", FrozenConfig(cfg))
        for key, shape in vae_state_dict_shapes(cfg).items():
            parts = key.split(".")
            mod = self
            for p in parts[:-1]:
                if p not in mod._modules:
                    mod.add_module(p, _Node())
                mod = mod._modules[p]
            mod.register_parameter(parts[-1], _M._empty(*shape))
        self.use_slicing = False
        self.use_tiling = False
        self.gradient_checkpointing = False
        self.num_latent_frames_batch_size = 2
        self.num_sample_frames_batch_size = 8
        self.tile_sample_min_height = sample_height // 2
        self.tile_sample_min_width = sample_width // 2
        nb = len(block_out_channels)
        self.tile_latent_min_height = int(self.tile_sample_min_height / (2 ** (nb - 1)))
        self.tile_latent_min_width = int(self.tile_sample_min_width / (2 ** (nb - 1)))
        self.tile_overlap_factor_height = 1 / 6
        self.tile_overlap_factor_width = 1 / 5
        self._prepared: Dict[str, Tuple[torch.Tensor, Optional[torch.Tensor]]] = {}
        self._caches: Dict[str, torch.Tensor] = {}
        self.flop_counter: Optional[list] = None

    # ---------------------------------------------------------------------------------------------------------
    # config / weights
    # ---------------------------------------------------------------------------------------------------------
    @property
    def config(self) -> FrozenConfig:
        return self._internal_config

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device

    @classmethod
    def from_config(cls, config: dict, device=None, dtype=torch.bfloat16, **overrides):
        cfg = {k: v for k, v in dict(config).items() if not k.startswith("_")}
        cfg.update(overrides)
        with _M.device_scope(device or _M._DEFAULT_DEVICE, dtype):
            return cls(**cfg)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, subfolder: Optional[str] = None,
                        torch_dtype=torch.bfloat16, device=None, **kwargs):
        """config.json + diffusion_pytorch_model*.safetensors of a diffusers VAE folder (e.g. subfolder="vae")."""
        from safetensors.torch import load_file
        if not os.path.isdir(pretrained_model_name_or_path):
            raise FileNotFoundError(f"{pretrained_model_name_or_path} is not a local directory (no hub access)")
        cfg = W.load_config(pretrained_model_name_or_path, subfolder)
        cfg.update({k: v for k, v in kwargs.items() if k in full_vae_config({})})
        dev = device or "cpu"
        model = cls.from_config(cfg, device=dev, dtype=torch_dtype or torch.bfloat16)
        sd = {}
        for f in W.weight_files(pretrained_model_name_or_path, subfolder):
            sd.update(load_file(f, device=str(dev)))
        model.load_diffusers_state_dict(sd)
        return model

    def load_diffusers_state_dict(self, sd: dict, strict: bool = True):
        own = self.state_dict()
        missing = [k for k in own if k not in sd]
        unexpected = [k for k in sd if k not in own]
        if strict and (missing or unexpected):
            raise RuntimeError(f"state dict mismatch: missing={missing[:8]} unexpected={unexpected[:8]}")
        with torch.no_grad():
            for k, t in own.items():
                if k in sd:
                    if tuple(sd[k].shape) != tuple(t.shape):
                        raise RuntimeError(f"{k}: shape {tuple(sd[k].shape)} != {tuple(t.shape)}")
                    t.copy_(sd[k].to(device=t.device, dtype=t.dtype))
        self._prepared.clear()
        return self

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._prepared.clear()
        return out

    def save_pretrained(self, save_directory: str, **_):
        from safetensors.torch import save_file
        W.save_config(save_directory, dict(self.config), type(self).__name__)
        save_file({k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()},
                  os.path.join(save_directory, W.WEIGHTS_NAME))

    def init_synthetic_weights_(self, seed: int = 0, host_exact: bool = False):
        """The deterministic synthetic weights of `weights.param_std` (host_exact: numpy, bit-reproducible)."""
        with torch.no_grad():
            for name, p in self.state_dict().items():
                if host_exact or not p.is_cuda:
                    p.copy_(torch.from_numpy(W.synth_param(name, tuple(p.shape), seed)).to(p.device, p.dtype))
                else:
                    mean, std = W.param_std(name, tuple(p.shape))
                    K.fill_normal_(p, W.counter_seed(name, seed), mean, std)
        self._prepared.clear()
        return self

    def _apply(self, fn, *args, **kwargs):  # .to() / .cuda(): the kernel-layout weights follow the parameters
        self._prepared = {}
        return super()._apply(fn, *args, **kwargs)

    # -- training-compat toggles (inference only: no backward kernels) --
    def enable_gradient_checkpointing(self):
        self.gradient_checkpointing = True

    def disable_gradient_checkpointing(self):
        self.gradient_checkpointing = False

    def enable_tiling(self, tile_sample_min_height: Optional[int] = None, tile_sample_min_width: Optional[int] = None,
                      tile_overlap_factor_height: Optional[float] = None,
                      tile_overlap_factor_width: Optional[float] = None) -> None:
        """:1028-1062"""
        nb = len(self.config.block_out_channels)
        self.use_tiling = True
        self.tile_sample_min_height = tile_sample_min_height or self.tile_sample_min_height
        self.tile_sample_min_width = tile_sample_min_width or self.tile_sample_min_width
        self.tile_latent_min_height = int(self.tile_sample_min_height / (2 ** (nb - 1)))
        self.tile_latent_min_width = int(self.tile_sample_min_width / (2 ** (nb - 1)))
        self.tile_overlap_factor_height = tile_overlap_factor_height or self.tile_overlap_factor_height
        self.tile_overlap_factor_width = tile_overlap_factor_width or self.tile_overlap_factor_width

    def disable_tiling(self) -> None:
        self.use_tiling = False

    def enable_slicing(self) -> None:
        self.use_slicing = True

    def disable_slicing(self) -> None:
        self.use_slicing = False

    def _clear_fake_context_parallel_cache(self):
        self._caches.clear()

    # ---------------------------------------------------------------------------------------------------------
    # kernel-layout weights (once per load): conv weights [Cout, kt, kh, kw, Cin_pad]; spatial-norm conv_y | conv_b
    # concatenated into one 1x1x1 conv [2C, 1, 1, 1, L_pad]
    # ---------------------------------------------------------------------------------------------------------
    def _param(self, name: str) -> torch.Tensor:
        mod = self
        parts = name.split(".")
        for p in parts[:-1]:
            mod = mod._modules[p]
        return getattr(mod, parts[-1])

    @staticmethod
    def _relayout(w: torch.Tensor) -> torch.Tensor:
        if w.dim() == 4:  # nn.Conv2d [Cout, Cin, kh, kw]
            w = w.unsqueeze(2)
        cout, cin = w.shape[:2]
        w = w.permute(0, 2, 3, 4, 1).to(torch.bfloat16)
        cp = _cpad(cin)
        if cp != cin:
            w = torch.nn.functional.pad(w, (0, cp - cin))
        return w.contiguous()

    def _conv_w(self, prefix: str):
        """prefix = the module holding weight / bias ('...conv' of a causal conv, '...conv_shortcut', ...)."""
        got = self._prepared.get(prefix)
        if got is None:
            w = self._param(prefix + ".weight").detach()
            got = (self._relayout(w), self._param(prefix + ".bias").detach().to(torch.bfloat16).contiguous(),
                   w.shape[1])
            self._prepared[prefix] = got
        return got

    def _mod_w(self, prefix: str):
        got = self._prepared.get(prefix + "#yb")
        if got is None:
            w = torch.cat([self._param(f"{prefix}.conv_y.conv.weight"), self._param(f"{prefix}.conv_b.conv.weight")])
            b = torch.cat([self._param(f"{prefix}.conv_y.conv.bias"), self._param(f"{prefix}.conv_b.conv.bias")])
            got = (self._relayout(w.detach()), b.detach().to(torch.bfloat16).contiguous(), w.shape[1])
            self._prepared[prefix + "#yb"] = got
        return got

    def _affine(self, prefix: str):
        got = self._prepared.get(prefix + "#gn")
        if got is None:
            got = tuple(self._param(f"{prefix}.{n}").detach().to(torch.bfloat16).contiguous()
                        for n in ("weight", "bias"))
            self._prepared[prefix + "#gn"] = got
        return got

    # ---------------------------------------------------------------------------------------------------------
    # layers (channels-last bf16 activations [B, T, H, W, C])
    # ---------------------------------------------------------------------------------------------------------
    def _conv(self, x: torch.Tensor, wbc, **kw) -> torch.Tensor:
        """vp_conv3d_bf16 + the algorithmic FLOP count (2 * output pixels * Cout * taps * logical Cin) when
        `self.flop_counter` is a list (bench / roofline)."""
        w, b, cin = wbc
        y = K.conv3d(x, w, b, **kw)
        if self.flop_counter is not None:
            self.flop_counter.append(2.0 * x.shape[0] * kw["Tout"] * kw["Hout"] * kw["Wout"] * w.shape[0] *
                                     w.shape[1] * w.shape[2] * w.shape[3] * cin)
        return y

    def _causal_conv(self, name: str, x: torch.Tensor, resid: Optional[torch.Tensor] = None) -> torch.Tensor:
        """`CogVideoXCausalConv3d.forward` :133-145: the previous frame batch's last kt-1 input frames (or kt-1
        copies of the first frame) in front, zero padding k//2 in H / W, stride 1; the frame cache is the conv's
        second frame source (nothing is concatenated)."""
        wbc = self._conv_w(name + ".conv")
        kt, kh = wbc[0].shape[1], wbc[0].shape[2]
        B, T, H, Wd, _ = x.shape
        hist = None
        tmap = list(range(T))
        if kt > 1:
            hist = self._caches.get(name)
            head = [-1 - i for i in range(kt - 1)] if hist is not None else [0] * (kt - 1)
            tmap = head + tmap
            last = tmap[-(kt - 1):]
            new = torch.stack([x[:, f] if f >= 0 else hist[:, -1 - f] for f in last], dim=1).contiguous()
        y = self._conv(x, wbc, Tout=T, Hout=H, Wout=Wd, tmap=tmap, hist=hist, pad=kh // 2, resid=resid)
        if kt > 1:
            self._caches[name] = new
        return y

    def _pointwise(self, name: str, x: torch.Tensor) -> torch.Tensor:
        """The 1x1x1 SafeConv3d conv_shortcut (:273)."""
        B, T, H, Wd, _ = x.shape
        return self._conv(x, self._conv_w(name), Tout=T, Hout=H, Wout=Wd, tmap=list(range(T)))

    def _norm(self, prefix: str, x: torch.Tensor, eps: float, zq: Optional[torch.Tensor]) -> torch.Tensor:
        """GroupNorm + SiLU (encoder), or CogVideoXSpatialNorm3D + SiLU (decoder, conditioned on zq) — the SiLU is the
        resnet's nonlinearity / the norm_out conv_act that always follows."""
        g = self.config.norm_num_groups
        if zq is None:
            gamma, beta = self._affine(prefix)
            return K.group_norm(x, gamma, beta, g, eps, silu=True)
        gamma, beta = self._affine(prefix + ".norm_layer")
        Bz, Tz, Hz, Wz, _ = zq.shape
        mod = self._conv(zq, self._mod_w(prefix), Tout=Tz, Hout=Hz, Wout=Wz, tmap=list(range(Tz)))
        return K.group_norm(x, gamma, beta, g, 1e-6, silu=True, mod=mod, tzmap=_spatial_norm_tmap(x.shape[1], Tz))

    def _resnet(self, prefix: str, x: torch.Tensor, zq: Optional[torch.Tensor] = None) -> torch.Tensor:
        """`CogVideoXResnetBlock3D.forward` :277-309 (temb None, dropout 0); the residual add is conv2's epilogue."""
        eps = self.config.norm_eps
        h = self._norm(prefix + ".norm1", x, eps, zq)
        h = self._causal_conv(prefix + ".conv1", h)
        h = self._norm(prefix + ".norm2", h, eps, zq)
        sc = self._pointwise(prefix + ".conv_shortcut", x) if (prefix + ".conv_shortcut") in self._shortcuts() else x
        return self._causal_conv(prefix + ".conv2", h, resid=sc)

    def _shortcuts(self):
        s = self._prepared.get("#shortcuts")
        if s is None:
            s = {k[:-len(".weight")] for k in self.state_dict() if k.endswith("conv_shortcut.weight")}
            self._prepared["#shortcuts"] = s
        return s

    def _downsample(self, prefix: str, x: torch.Tensor, compress_time: bool) -> torch.Tensor:
        """`CogVideoXDownsample3D.forward` downsampling.py:322-353: temporal 2:1 average (first frame kept when the
        count is odd), zero pad right / bottom by 1, 3x3 conv stride 2 per frame."""
        if compress_time:
            x = K.time_pool2(x)
        B, T, H, Wd, _ = x.shape
        return self._conv(x, self._conv_w(prefix + ".conv"), Tout=T, Hout=(H - 2) // 2 + 1, Wout=(Wd - 2) // 2 + 1,
                          tmap=list(range(T)), stride=2)

    def _upsample(self, prefix: str, x: torch.Tensor, compress_time: bool) -> torch.Tensor:
        """`CogVideoXUpsample3D.forward` upsampling.py:384-412: nearest x2 in H / W (and in time for compress_time,
        the first frame kept single when the count is odd > 1), 3x3 conv padding 1 — the resize is the conv's
        gather (uh = uw = 2, tmap repeats frames)."""
        B, T, H, Wd, _ = x.shape
        if compress_time and T > 1 and T % 2 == 1:
            tmap = [0] + [1 + k // 2 for k in range(2 * (T - 1))]
        elif compress_time and T > 1:
            tmap = [k // 2 for k in range(2 * T)]
        else:
            tmap = list(range(T))
        return self._conv(x, self._conv_w(prefix + ".conv"), Tout=len(tmap), Hout=2 * H, Wout=2 * Wd, tmap=tmap,
                          pad=1, up=2)

    def _encoder(self, x: torch.Tensor) -> torch.Tensor:
        """`CogVideoXEncoder3D.forward` :708-742 on one frame batch -> [B, T', h, w, 2L] channels-last."""
        cfg = self.config
        nb = len(cfg.block_out_channels)
        tcl = int(np.log2(cfg.temporal_compression_ratio))
        h = self._causal_conv("encoder.conv_in", x)
        for i in range(nb):
            for j in range(cfg.layers_per_block):
                h = self._resnet(f"encoder.down_blocks.{i}.resnets.{j}", h)
            if i < nb - 1:
                h = self._downsample(f"encoder.down_blocks.{i}.downsamplers.0", h, compress_time=i < tcl)
        for j in range(2):
            h = self._resnet(f"encoder.mid_block.resnets.{j}", h)
        gamma, beta = self._affine("encoder.norm_out")
        h = K.group_norm(h, gamma, beta, cfg.norm_num_groups, 1e-6, silu=True)
        h = self._causal_conv("encoder.conv_out", h)
        if cfg.use_quant_conv:  # (:1101-1102, per frame batch / tile)
            h = self._pointwise("quant_conv", h)
        return h

    def _decoder(self, z: torch.Tensor) -> torch.Tensor:
        """`CogVideoXDecoder3D.forward` :849-883 on one latent frame batch (channels-last, L padded) -> [B, T, H, W, 8]
        (channels 3..7 zero)."""
        cfg = self.config
        nb = len(cfg.block_out_channels)
        tcl = int(np.log2(cfg.temporal_compression_ratio))
        if cfg.use_post_quant_conv:  # (:1152-1153: before the decoder, whose spatial norms then see its output)
            z = self._pointwise("post_quant_conv", z)
        h = self._causal_conv("decoder.conv_in", z)
        for j in range(2):
            h = self._resnet(f"decoder.mid_block.resnets.{j}", h, zq=z)
        for i in range(nb):
            for j in range(cfg.layers_per_block + 1):
                h = self._resnet(f"decoder.up_blocks.{i}.resnets.{j}", h, zq=z)
            if i < nb - 1:
                h = self._upsample(f"decoder.up_blocks.{i}.upsamplers.0", h, compress_time=i < tcl)
        h = self._norm("decoder.norm_out", h, 1e-6, z)
        return self._causal_conv("decoder.conv_out", h)

    # ---------------------------------------------------------------------------------------------------------
    # encode / decode (reference frame batching, slicing, tiling)
    # ---------------------------------------------------------------------------------------------------------
    def _check(self, t: torch.Tensor, what: str):
        if not t.is_cuda:
            raise ValueError(f"{what} must be a device tensor (the VAE runs on the HIP kernels only)")
        if t.dim() != 5:
            raise ValueError(f"{what} must be [B, C, F, H, W]")
        if torch.is_grad_enabled() and t.requires_grad:
            raise NotImplementedError("videopainter_amd's VAE is inference only; call under torch.no_grad()")

    @staticmethod
    def _frame_batches(num_frames: int, size: int, min_one: bool):
        """:1091-1099 (encode, min_one) / :1144-1151 (decode): batch 0 absorbs the remainder."""
        nb = num_frames // size if (num_frames > 1 or not min_one) else 1
        rem = num_frames % size
        return [(size * i + (0 if i == 0 else rem), size * (i + 1) + rem) for i in range(nb)]

    def _encode_nhwc(self, x_cl: torch.Tensor) -> torch.Tensor:
        """Frame-batched encoder over a channels-last video [B, F, H, W, 8] -> params [B, T, h, w, 2L]."""
        self._clear_fake_context_parallel_cache()
        parts = [self._encoder(x_cl[:, a:b].contiguous())
                 for a, b in self._frame_batches(x_cl.shape[1], self.num_sample_frames_batch_size, True)]
        self._clear_fake_context_parallel_cache()
        return parts[0] if len(parts) == 1 else torch.cat(parts, dim=1)

    def _decode_nhwc(self, z_cl: torch.Tensor) -> torch.Tensor:
        self._clear_fake_context_parallel_cache()
        parts = [self._decoder(z_cl[:, a:b].contiguous())
                 for a, b in self._frame_batches(z_cl.shape[1], self.num_latent_frames_batch_size, False)]
        self._clear_fake_context_parallel_cache()
        return parts[0] if len(parts) == 1 else torch.cat(parts, dim=1)

    def _encode(self, x: torch.Tensor) -> torch.Tensor:
        """:1085-1108 -> channels-last latent-distribution parameters [B, T, h, w, 2L]."""
        B, C, F, H, Wd = x.shape
        with _on(x):
            x_cl = K.ncdhw_to_ndhwc(x, _cpad(C))
            if self.use_tiling and (Wd > self.tile_sample_min_width or H > self.tile_sample_min_height):
                return self._tiled(x_cl, encode=True)
            return self._encode_nhwc(x_cl)

    def encode(self, x: torch.Tensor, return_dict: bool = True):
        """:1110-1136"""
        self._check(x, "x")
        if self.use_slicing and x.shape[0] > 1:
            p = torch.cat([self._encode(s) for s in x.split(1)])
        else:
            p = self._encode(x)
        post = DiagonalGaussianDistribution(p, self.config.latent_channels)
        return AutoencoderKLOutput(latent_dist=post) if return_dict else (post,)

    def _decode(self, z: torch.Tensor) -> torch.Tensor:
        B, C, T, h, w = z.shape
        with _on(z):
            z_cl = K.ncdhw_to_ndhwc(z, _cpad(C))
            if self.use_tiling and (w > self.tile_latent_min_width or h > self.tile_latent_min_height):
                out = self._tiled(z_cl, encode=False)
            else:
                out = self._decode_nhwc(z_cl)
            return K.ndhwc_to_ncdhw(out, self.config.out_channels)

    def decode(self, z: torch.Tensor, return_dict: bool = True):
        """:1165-1190 (a single latent frame is duplicated first)."""
        self._check(z, "z")
        if z.shape[2] == 1:
            z = torch.cat([z, z], dim=2)
        if self.use_slicing and z.shape[0] > 1:
            dec = torch.cat([self._decode(s) for s in z.split(1)])
        else:
            dec = self._decode(z)
        return DecoderOutput(sample=dec) if return_dict else (dec,)

    def _tiled(self, x_cl: torch.Tensor, encode: bool) -> torch.Tensor:
        """`tiled_encode` :1208-1277 / `tiled_decode` :1279-1358 on channels-last tiles: overlapping spatial tiles run
        through the frame-batched encoder / decoder separately, then each tile is blended in place with the tile above
        and the tile to its left (in the reference's order, so already-blended neighbours feed later blends) and
        cropped; the crops are concatenated."""
        H, Wd = x_cl.shape[2], x_cl.shape[3]
        if encode:
            tmin_h, tmin_w = self.tile_sample_min_height, self.tile_sample_min_width
            omin_h, omin_w = self.tile_latent_min_height, self.tile_latent_min_width
        else:
            tmin_h, tmin_w = self.tile_latent_min_height, self.tile_latent_min_width
            omin_h, omin_w = self.tile_sample_min_height, self.tile_sample_min_width
        overlap_h = int(tmin_h * (1 - self.tile_overlap_factor_height))
        overlap_w = int(tmin_w * (1 - self.tile_overlap_factor_width))
        blend_h = int(omin_h * self.tile_overlap_factor_height)
        blend_w = int(omin_w * self.tile_overlap_factor_width)
        limit_h, limit_w = omin_h - blend_h, omin_w - blend_w
        run = self._encode_nhwc if encode else self._decode_nhwc
        rows = []
        for i in range(0, H, overlap_h):
            rows.append([run(x_cl[:, :, i:i + tmin_h, j:j + tmin_w].contiguous()) for j in range(0, Wd, overlap_w)])
        out_rows = []
        for i, row in enumerate(rows):
            crops = []
            for j, tile in enumerate(row):
                if i > 0:
                    K.tile_blend_(rows[i - 1][j], tile, 0, blend_h)
                if j > 0:
                    K.tile_blend_(row[j - 1], tile, 1, blend_w)
                crops.append(tile[:, :, :limit_h, :limit_w])
            out_rows.append(torch.cat(crops, dim=3))
        return torch.cat(out_rows, dim=2).contiguous()

    def forward(self, sample: torch.Tensor, sample_posterior: bool = False, return_dict: bool = True,
                generator: Optional[torch.Generator] = None):
        """:1360-1376"""
        post = self.encode(sample).latent_dist
        z = post.sample(generator=generator) if sample_posterior else post.mode()
        dec = self.decode(z)
        return dec if return_dict else (dec,)

