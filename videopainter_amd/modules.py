"""Parameter containers with the reference's module tree (so diffusers state-dict keys load unchanged) and a small
ModelMixin/ConfigMixin stand-in (`config`, `from_pretrained`, `save_pretrained`, `from_config`).

Reference: DF/models/modeling_utils.py:266 (save_pretrained), :412 (from_pretrained), :160
(enable_gradient_checkpointing); DF/configuration_utils.py:608 (register_to_config).  The containers hold bf16
device tensors; their forward is never called — the model classes drive the HIP kernels directly.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn as nn

from . import weights as W
from .config import full_config, state_dict_shapes

_DEFAULT_DEVICE = "cpu"
_DEFAULT_DTYPE = torch.bfloat16


@contextlib.contextmanager
def device_scope(device, dtype=torch.bfloat16):
    """Allocate parameters of models constructed inside this scope directly on `device` (no host staging)."""
    global _DEFAULT_DEVICE, _DEFAULT_DTYPE
    old = (_DEFAULT_DEVICE, _DEFAULT_DTYPE)
    _DEFAULT_DEVICE, _DEFAULT_DTYPE = device, dtype
    try:
        yield
    finally:
        _DEFAULT_DEVICE, _DEFAULT_DTYPE = old


def _empty(*shape):
    return nn.Parameter(torch.empty(*shape, device=_DEFAULT_DEVICE, dtype=_DEFAULT_DTYPE), requires_grad=False)


class FrozenConfig(dict):
    """dict with attribute access, like diffusers' FrozenDict config."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        raise AttributeError("config is frozen; use register_to_config-style construction")


class Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = _empty(out_features, in_features)
        self.bias = _empty(out_features) if bias else None


class LayerNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5, elementwise_affine: bool = True):
        super().__init__()
        self.eps = eps
        self.normalized_shape = (dim,)
        if not elementwise_affine:
            raise NotImplementedError("CogVideoX uses affine LayerNorms (norm_elementwise_affine=True)")
        self.weight = _empty(dim)
        self.bias = _empty(dim)


class Conv2dPatch(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, patch: int):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, (patch, patch)
        self.weight = _empty(out_channels, in_channels, patch, patch)
        self.bias = _empty(out_channels)


class Dropout(nn.Module):
    """p = 0 in every CogVideoX config (dropout=0.0); inference never drops."""


class ModelMixin(nn.Module):
    _is_branch = False
    config_name = W.CONFIG_NAME
    _supports_gradient_checkpointing = True

    def __init__(self):
        nn.Module.__init__(self)  # never a re-based library base's __init__ (integration.install)

    def _init_config(self, kwargs: dict):
        cfg = full_config(kwargs, branch=self._is_branch)
        object.__setattr__(self, "_internal_config", FrozenConfig(cfg))
        self.gradient_checkpointing = False

    @property
    def config(self) -> FrozenConfig:
        return self._internal_config

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device

    # -- training toggles (modeling_utils.py:160).  The block backward always recomputes from the block input
    # (autograd._BlockFn, DESIGN_LOG.md §3.5), i.e. it is checkpointed whether or not the flag is set --
    def enable_gradient_checkpointing(self):
        self.gradient_checkpointing = True

    def disable_gradient_checkpointing(self):
        self.gradient_checkpointing = False

    # -- construction / weights --
    @classmethod
    def from_config(cls, config: dict, device=None, dtype=torch.bfloat16, **overrides):
        cfg = {k: v for k, v in dict(config).items() if not k.startswith("_")}
        cfg.update(overrides)
        with device_scope(device or _DEFAULT_DEVICE, dtype):
            return cls(**cfg)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, subfolder: Optional[str] = None,
                        torch_dtype=torch.bfloat16, device=None, **kwargs):
        """Load `config.json` + `diffusion_pytorch_model*.safetensors` (diffusers layout).  Extra kwargs override
        config entries (e.g. id_pool_resample_learnable=True, as infer/inpaint.py:296-300 does)."""
        from safetensors.torch import load_file
        if not os.path.isdir(pretrained_model_name_or_path):
            raise FileNotFoundError(f"{pretrained_model_name_or_path} is not a local directory (no hub access)")
        cfg = W.load_config(pretrained_model_name_or_path, subfolder)
        cfg.update({k: v for k, v in kwargs.items() if k in full_config({}, branch=cls._is_branch)})
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
                    src = sd[k]
                    if tuple(src.shape) != tuple(t.shape):
                        raise RuntimeError(f"{k}: shape {tuple(src.shape)} != {tuple(t.shape)}")
                    t.copy_(src.to(device=t.device, dtype=t.dtype))
        return self

    def save_pretrained(self, save_directory: str, safe_serialization: bool = True, **_):
        from safetensors.torch import save_file
        W.save_config(save_directory, dict(self.config), type(self).__name__)
        sd = {k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()}
        save_file(sd, os.path.join(save_directory, W.WEIGHTS_NAME))

    def expected_state_dict_shapes(self):
        return state_dict_shapes(dict(self.config), branch=self._is_branch)

    def reset_parameters_(self, seed: int = 0):
        """PyTorch's default module initialisation, as the reference modules get it in `__init__`: nn.Linear /
        nn.Conv2d weight and bias U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (kaiming_uniform with a = sqrt 5), LayerNorm
        weight 1 / bias 0; the positional-embedding buffer keeps its sin-cos initialisation.  Drawn on the host from a
        seeded torch.Generator (the reference draws from the global RNG), then copied to the parameters' device."""
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for mod in self.modules():
                if isinstance(mod, (Linear, Conv2dPatch)):
                    fan_in = mod.weight[0].numel()
                    bound = 1.0 / fan_in ** 0.5
                    for t in (mod.weight, mod.bias):
                        if t is not None:
                            t.copy_((torch.rand(t.shape, generator=g) * 2 - 1) * bound)
                elif isinstance(mod, LayerNorm):
                    mod.weight.fill_(1.0)
                    mod.bias.zero_()
        return self

    def init_synthetic_weights_(self, seed: int = 0, host_exact: bool = False):
        """Fill every parameter with the deterministic synthetic distribution of `weights.param_std`.

        host_exact=True: generate with numpy on the host (bit-reproducible parity fixtures; slow for 5B params).
        host_exact=False: generate on the device with `vp_fill_normal_bf16` (same splitmix64/Box-Muller stream)."""
        with torch.no_grad():
            for name, p in self.state_dict().items():
                if host_exact or not p.is_cuda:
                    p.copy_(torch.from_numpy(W.synth_param(name, tuple(p.shape), seed)).to(p.device, p.dtype))
                else:
                    from . import kernels as K
                    mean, std = W.param_std(name, tuple(p.shape))
                    K.fill_normal_(p, W.counter_seed(name, seed), mean, std)
        return self
