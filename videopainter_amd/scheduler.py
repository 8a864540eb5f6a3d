"""CogVideoX DPM-Solver++ scheduler — drop-in for the reference `CogVideoXDPMScheduler`
(DF/schedulers/scheduling_dpm_cogvideox.py:127-491).

Host side: the fp64 noise-schedule scalars (betas, SNR shift, zero-terminal-SNR rescale, λ multipliers) exactly as
the reference computes them with 0-dim fp64 tensors.  Device side: one fused HIP launch per step
(`vp_dpm_step_bf16`), with each scalar rounded to the dtype the reference's torch type promotion gives it (a 0-dim
fp64 tensor times a bf16 tensor is computed with the scalar rounded to bf16; times an fp32 tensor, to fp32).
The stochastic noise is drawn exactly like the reference (`randn_tensor`: the CPU generator, in the sample's dtype)
so seeded runs match.
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import kernels as K
from . import _native as NAT
from .modules import FrozenConfig

BF16 = torch.bfloat16

SCHEDULER_DEFAULTS = dict(num_train_timesteps=1000, beta_start=0.00085, beta_end=0.0120, beta_schedule="scaled_linear",
                          trained_betas=None, clip_sample=True, set_alpha_to_one=True, steps_offset=0,
                          prediction_type="epsilon", clip_sample_range=1.0, sample_max_value=1.0,
                          timestep_spacing="leading", rescale_betas_zero_snr=False, snr_shift_scale=3.0)


def randn_tensor(shape, generator=None, device=None, dtype=None):
    """DF/utils/torch_utils.py:38-83 for a single (CPU) generator: draw on the generator's device, then move."""
    rand_device = generator.device if generator is not None else (device or "cpu")
    out = torch.randn(shape, generator=generator, device=rand_device, dtype=dtype)
    if device is None or torch.device(device) == out.device:
        return out
    if out.device.type == "cpu" and torch.device(device).type == "cuda":
        # same values, but the host->device copy is queued on the stream from pinned memory instead of a pageable
        # copy that blocks the host until the GPU has drained the step's forward (the CPU draw then ran while the GPU
        # idled: ~15 ms per second-order step at config 2, profiles/r01_bench_kernel_trace gap analysis)
        return out.pin_memory().to(device, non_blocking=True)
    return out.to(device)


def _rbf(x: float) -> float:
    return float(torch.tensor(float(x), dtype=torch.float64).to(BF16).float())


def _f32(x: float) -> float:
    return float(np.float32(float(x)))


class CogVideoXDPMScheduler:
    order = 1

    def __init__(self, **kwargs):
        unknown = set(kwargs) - set(SCHEDULER_DEFAULTS) - {"_class_name", "_diffusers_version"}
        if unknown:
            raise TypeError(f"unexpected scheduler config keys {sorted(unknown)}")
        cfg = dict(SCHEDULER_DEFAULTS)
        cfg.update({k: v for k, v in kwargs.items() if not k.startswith("_")})
        self.config = FrozenConfig(cfg)
        if cfg["trained_betas"] is not None:
            betas = torch.tensor(cfg["trained_betas"], dtype=torch.float32)
        elif cfg["beta_schedule"] == "linear":
            betas = torch.linspace(cfg["beta_start"], cfg["beta_end"], cfg["num_train_timesteps"], dtype=torch.float32)
        elif cfg["beta_schedule"] == "scaled_linear":
            betas = torch.linspace(cfg["beta_start"] ** 0.5, cfg["beta_end"] ** 0.5, cfg["num_train_timesteps"],
                                   dtype=torch.float64) ** 2
        else:
            raise NotImplementedError(f"{cfg['beta_schedule']} is not implemented for {self.__class__}")
        self.betas = betas
        self.alphas = 1.0 - betas
        ac = torch.cumprod(self.alphas, dim=0)
        s = cfg["snr_shift_scale"]
        ac = ac / (s + (1 - s) * ac)
        if cfg["rescale_betas_zero_snr"]:
            sq = ac.sqrt()
            s0, sT = sq[0].clone(), sq[-1].clone()
            sq -= sT
            sq *= s0 / (s0 - sT)
            ac = sq ** 2
        self.alphas_cumprod = ac
        self.final_alpha_cumprod = torch.tensor(1.0) if cfg["set_alpha_to_one"] else ac[0]
        self.init_noise_sigma = 1.0
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, cfg["num_train_timesteps"])[::-1].copy().astype(np.int64))

    @classmethod
    def from_config(cls, config, **kwargs):
        cfg = {k: v for k, v in dict(config).items() if not k.startswith("_")}
        cfg.update(kwargs)
        return cls(**cfg)

    def scale_model_input(self, sample, timestep=None):
        return sample

    def set_timesteps(self, num_inference_steps: int, device=None):
        """:261-304."""
        c = self.config
        if num_inference_steps > c.num_train_timesteps:
            raise ValueError(f"`num_inference_steps`: {num_inference_steps} cannot be larger than "
                             f"`self.config.train_timesteps`: {c.num_train_timesteps}")
        self.num_inference_steps = num_inference_steps
        if c.timestep_spacing == "linspace":
            ts = np.linspace(0, c.num_train_timesteps - 1, num_inference_steps).round()[::-1].copy().astype(np.int64)
        elif c.timestep_spacing == "leading":
            r = c.num_train_timesteps // num_inference_steps
            ts = (np.arange(0, num_inference_steps) * r).round()[::-1].copy().astype(np.int64) + c.steps_offset
        elif c.timestep_spacing == "trailing":
            r = c.num_train_timesteps / num_inference_steps
            ts = np.round(np.arange(c.num_train_timesteps, 0, -r)).astype(np.int64) - 1
        else:
            raise ValueError(f"{c.timestep_spacing} is not supported.")
        self.timesteps = torch.from_numpy(ts).to(device)

    def coefficients(self, timestep: int, timestep_back: Optional[int]):
        """fp64 scalars of :362-406, computed with the reference's own 0-dim-tensor expressions."""
        prev_t = timestep - self.config.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[timestep]
        a_prev = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.final_alpha_cumprod
        a_back = self.alphas_cumprod[timestep_back] if timestep_back is not None else None
        beta_t = 1 - a_t
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
        return dict(prev_t=prev_t, sa=float(a_t ** 0.5), sb=float(beta_t ** 0.5), m1=float(mult1), m2=float(mult2),
                    m3=None if mult3 is None else float(mult3), m4=None if mult4 is None else float(mult4),
                    mn=float(mult_noise))

    def fill_desc(self, d: "NAT.DpmDesc", timestep: int, timestep_back: Optional[int], has_old: bool,
                  sample_dtype=BF16, mo_dtype=torch.float32) -> bool:
        """Fill the scalar fields of a step descriptor; returns whether the 2nd-order branch runs."""
        c = self.coefficients(int(timestep), None if timestep_back is None else int(timestep_back))
        rs = _rbf if sample_dtype == BF16 else _f32
        rm = _rbf if mo_dtype == BF16 else _f32
        d.sa, d.sb = rs(c["sa"]), rm(c["sb"])
        d.m1, d.m2, d.mn = rs(c["m1"]), _f32(c["m2"]), rs(c["mn"])
        second = has_old and c["prev_t"] >= 0
        d.second_order = int(second)
        d.m3 = _f32(c["m3"]) if second else 0.0
        d.m4 = _f32(c["m4"]) if second else 0.0
        return second

    def step(self, model_output: torch.Tensor, old_pred_original_sample: Optional[torch.Tensor], timestep: int,
             timestep_back: Optional[int], sample: torch.Tensor, eta: float = 0.0,
             use_clipped_model_output: bool = False, generator=None, variance_noise=None, return_dict: bool = False):
        """:330-439 (v_prediction).  Returns (prev_sample fp32, pred_original_sample fp32)."""
        if self.num_inference_steps is None:
            raise ValueError("Number of inference steps is 'None', you need to run 'set_timesteps' after creating "
                             "the scheduler")
        if self.config.prediction_type != "v_prediction":
            raise NotImplementedError("CogVideoX-5b uses prediction_type='v_prediction'")
        if sample.dtype != BF16:
            raise NotImplementedError("the HIP step kernel takes bf16 latents (the pipeline's dtype)")
        dev = sample.device
        n = sample.numel()
        mo = model_output.to(device=dev, dtype=torch.float32).contiguous()
        smp = sample.contiguous()
        d = NAT.DpmDesc()
        second = self.fill_desc(d, int(timestep), timestep_back, old_pred_original_sample is not None)
        noise1 = randn_tensor(sample.shape, generator=generator, device=dev, dtype=sample.dtype)
        noise2 = randn_tensor(sample.shape, generator=generator, device=dev, dtype=sample.dtype) if second else None
        pred = torch.empty(sample.shape, device=dev, dtype=torch.float32)
        prev = torch.empty(sample.shape, device=dev, dtype=torch.float32)
        old = old_pred_original_sample.to(device=dev, dtype=torch.float32).contiguous() if second else None
        d.n = n
        d.model_output = mo.data_ptr()
        d.sample = smp.data_ptr()
        d.old_pred = old.data_ptr() if old is not None else None
        d.pred_out = pred.data_ptr()
        d.noise1 = noise1.data_ptr()
        d.noise2 = noise2.data_ptr() if noise2 is not None else None
        d.prev_out = prev.data_ptr()
        K.dpm_step(d)
        return (prev, pred)

    def add_noise_scalars(self, timestep: int, dtype=BF16) -> Tuple[float, float]:
        """:442-466: alphas cast to the sample dtype first, then sqrt in that dtype."""
        ac = self.alphas_cumprod.to(dtype=dtype)
        t = torch.tensor([int(timestep)])
        return float((ac[t] ** 0.5).float()), float(((1 - ac[t]) ** 0.5).float())

    def add_noise(self, original_samples: torch.Tensor, noise: torch.Tensor, timesteps: torch.IntTensor):
        """:442-466 (host formula; the pipeline fuses it into the step kernel)."""
        ac = self.alphas_cumprod.to(device=original_samples.device, dtype=original_samples.dtype)
        timesteps = timesteps.to(original_samples.device)
        sa = ac[timesteps] ** 0.5
        sb = (1 - ac[timesteps]) ** 0.5
        while sa.dim() < original_samples.dim():
            sa = sa.unsqueeze(-1)
            sb = sb.unsqueeze(-1)
        return sa * original_samples + sb * noise

    def get_velocity(self, sample, noise, timesteps):
        ac = self.alphas_cumprod.to(device=sample.device, dtype=sample.dtype)
        timesteps = timesteps.to(sample.device)
        sa = ac[timesteps] ** 0.5
        sb = (1 - ac[timesteps]) ** 0.5
        while sa.dim() < sample.dim():
            sa = sa.unsqueeze(-1)
            sb = sb.unsqueeze(-1)
        return sa * noise - sb * sample

    def __len__(self):
        return self.config.num_train_timesteps
