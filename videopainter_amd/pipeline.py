"""Harness of the any-length VideoPainter pipeline on the HIP models.

Restates the step loop of `CogVideoXI2VDualInpaintAnyLPipeline.__call__`
(DF/pipelines/cogvideo/pipeline_cogvideox_inpainting_i2v_branch_anyl.py:932-1050) and its window loop
(:759, 828-872, 962-988, 1052-1069).  `__call__` starts from the per-window latents the VAE stage produced;
`generate` starts from the preprocessed pixels (the video / mask processors' outputs) and runs the VAE stage on the HIP
VAE too — per window prepare_latents (:339-412: first-frame encode, video encode, initial noise) and
prepare_mask_latents (:434-477: nearest mask resize, masked-video encode), drawing from the caller's generator in
the reference's order — then decodes the overlap-averaged latents (decode_latents :479-484, :1071-1073).  One
denoising step = branch forward + transformer forward at B=2 (CFG) + one fused CFG/DPM/replace-gt kernel.

Reference quirks reproduced on purpose:
  * dynamic CFG uses the raw timestep t (anyl.py:991-994);
  * `prev_resample_mask` is re-bound to the transformer's output EVERY step (anyl.py:967), so from the second step
    of a window k>0 the "previous" mask is the current window's own mask;
  * window k>0 conditions on the previous window's last latent frame (anyl.py:866-872).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from . import kernels as K
from . import _native as NAT
from .embeddings import prepare_rotary_positional_embeddings
from .scheduler import randn_tensor

BF16 = torch.bfloat16


@dataclass
class WindowState:
    latents: torch.Tensor            # bf16 [1, F, C, h, w]
    image_in: torch.Tensor           # bf16 [2, F, C, h, w]   (cat([image_latents]*2))
    branch_in: torch.Tensor          # bf16 [2, F, C+1, h, w] (masked latents ++ mask)
    mask1: torch.Tensor              # bf16 [2, F, 1, h, w]   branch_block_masks
    init_mask: torch.Tensor          # bf16 [1, F, C, h, w]   replace-gt blend mask
    video_latents: Optional[torch.Tensor]
    noise: Optional[torch.Tensor]
    old_pred: Optional[torch.Tensor] = None
    last_states: Optional[Dict[int, torch.Tensor]] = None
    extra: dict = field(default_factory=dict)


class CogVideoXI2VDualInpaintAnyLHarness:
    def __init__(self, transformer, branch, scheduler, vae_scale_factor_spatial: int = 8,
                 vae_scale_factor_temporal: int = 4, cfg_pair=None, vae=None, noise_dtype=BF16):
        """cfg_pair: optional `distributed.CFGPair`.  The two CFG halves of every step then run on the pair's two
        ranks at B=1 and their noise predictions are all-gathered (latency mode); both ranks apply the
        same CFG combine + DPM step with the same generator stream, so their latents stay bit-identical."""
        self.transformer = transformer
        self.branch = branch
        self.scheduler = scheduler
        self.vae_scale_factor_spatial = vae_scale_factor_spatial
        self.vae_scale_factor_temporal = vae_scale_factor_temporal
        self.prev_resample_mask = None
        self.cfg_pair = cfg_pair
        self.vae = vae
        # dtype of every generator draw (posterior samples, initial noise, scheduler noise): the reference draws in the
        # pipeline's dtype (bf16 in the inference scripts); torch's CPU generator gives different values for a bf16
        # and an fp32 draw of the same shape, so replaying an fp32 reference run needs float32 here
        self.noise_dtype = noise_dtype

    @property
    def device(self):
        return self.transformer.proj_out.weight.device

    # ------------------------------------------------------------------------------------------------------------
    def make_window(self, latents, image_latents, masked_video_latents, mask, video_latents=None, noise=None
                    ) -> WindowState:
        """mask: [2, 1, F, h, w] (prepare_mask_latents output, CFG-duplicated); masked_video_latents [2, F, C, h, w];
        image_latents [1, F, C, h, w] (frame 0 = conditioning latent, rest zero)."""
        dev = self.device
        lat = latents.to(dev, BF16).contiguous()
        C = lat.shape[2]
        m = mask.to(dev, BF16).permute(0, 2, 1, 3, 4).repeat(1, 1, C, 1, 1)  # anyl.py:920
        image_in = torch.cat([image_latents.to(dev, BF16)] * 2).contiguous()
        branch_in = torch.cat([masked_video_latents.to(dev, BF16), m[:, :, :1]], dim=-3).contiguous()
        mask1 = m[:, :, :1].contiguous()
        init_mask = m.chunk(2)[0].contiguous()
        return WindowState(latents=lat, image_in=image_in, branch_in=branch_in, mask1=mask1, init_mask=init_mask,
                           video_latents=None if video_latents is None else video_latents.to(dev, BF16).contiguous(),
                           noise=None if noise is None else noise.to(dev, BF16).contiguous())

    def rope_for(self, latent_frames: int, height_lat: int, width_lat: int):
        return prepare_rotary_positional_embeddings(height_lat * self.vae_scale_factor_spatial,
                                                    width_lat * self.vae_scale_factor_spatial, latent_frames,
                                                    self.transformer.config.attention_head_dim,
                                                    self.vae_scale_factor_spatial, self.transformer.config.patch_size,
                                                    device=self.device)

    # ------------------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, st: WindowState, i: int, timesteps: torch.Tensor, prompt_embeds: torch.Tensor, rope, *,
             guidance_scale: float = 6.0, use_dynamic_cfg: bool = True, conditioning_scale: float = 1.0,
             replace_gt: bool = True, mask_add: bool = True, mask_background: bool = False, add_first: bool = False,
             id_pool_resample_learnable: bool = False, attention_kwargs: Optional[dict] = None,
             prev_window_states: Optional[Dict[int, torch.Tensor]] = None, prev_clip_weight: float = 0.0,
             capture_last_states: bool = False, step_noise: Optional[Callable[[], torch.Tensor]] = None,
             generator=None) -> None:
        """One denoising step (anyl.py:933-1034); updates `st` in place."""
        t = timesteps[i]
        t_int = int(t)
        dev = self.device
        lat = st.latents
        # CFG batch (anyl.py:937-945); with a CFG pair this rank runs only its own half at B=1
        if self.cfg_pair is None:
            nb, sl = 2, slice(0, 2)
        else:
            c = self.cfg_pair.cfg_index
            nb, sl = 1, slice(c, c + 1)
        lvi = torch.cat([lat] * nb)
        lmi = torch.cat([lvi, st.image_in[sl]], dim=2)
        pe = prompt_embeds[sl]
        ts = torch.full((nb,), t_int, device=dev, dtype=torch.int64)
        bs = self.branch(hidden_states=lvi, encoder_hidden_states=pe, branch_cond=st.branch_in[sl],
                         conditioning_scale=conditioning_scale, timestep=ts, image_rotary_emb=rope,
                         attention_kwargs=attention_kwargs, return_dict=False)[0]
        akw = dict(attention_kwargs) if attention_kwargs else {}
        if prev_window_states is not None:
            akw["prev_hidden_states"] = prev_window_states
            akw["prev_clip_weight"] = prev_clip_weight
            akw["prev_resample_mask"] = self.prev_resample_mask
        noise_pred, hs_list, self.prev_resample_mask = self.transformer(
            hidden_states=lmi, encoder_hidden_states=pe, branch_block_samples=bs, timestep=ts,
            image_rotary_emb=rope, attention_kwargs=akw, add_first=add_first,
            branch_block_masks=st.mask1[sl] if mask_add else None,
            id_pool_resample_learnable=id_pool_resample_learnable,
            return_hidden_states=True, return_resample_mask=True, return_dict=False)
        if capture_last_states and t_int == int(timesteps[-1]):
            st.last_states = {k: h for k, h in enumerate(hs_list)}
        del hs_list, bs
        if self.cfg_pair is not None:
            noise_pred = self.cfg_pair.allgather(noise_pred.contiguous())  # [2, F, C, h, w] = (uncond, text)
        n_steps = len(timesteps)
        g = guidance_scale
        if use_dynamic_cfg:
            g = 1 + guidance_scale * ((1 - math.cos(math.pi * ((n_steps - t_int) / n_steps) ** 5.0)) / 2)
        d = NAT.DpmDesc()
        second = self.scheduler.fill_desc(d, t_int, int(timesteps[i - 1]) if i > 0 else None, st.old_pred is not None)

        def draw():
            if step_noise is not None:
                return step_noise().to(dev, BF16).contiguous()
            n = randn_tensor(lat.shape, generator=generator, device=dev, dtype=self.noise_dtype)
            return n.to(BF16).contiguous()

        noise1 = draw()
        noise2 = draw() if second else None
        n = lat.numel()
        pred = torch.empty(lat.shape, device=dev, dtype=torch.float32)
        new_lat = torch.empty_like(lat)
        d.n = n
        d.noise_pred = noise_pred.data_ptr()
        d.do_cfg = 1
        d.guidance = g
        d.sample = lat.data_ptr()
        d.old_pred = st.old_pred.data_ptr() if second else None
        d.pred_out = pred.data_ptr()
        d.noise1 = noise1.data_ptr()
        d.noise2 = noise2.data_ptr() if noise2 is not None else None
        d.latents_out = new_lat.data_ptr()
        if replace_gt:
            if st.video_latents is None:
                raise ValueError("replace_gt needs the window's video latents")
            d.replace_gt = 1
            d.mask_background = int(mask_background)
            d.gt = st.video_latents.data_ptr()
            d.mask = st.init_mask.data_ptr()
            if i < n_steps - 1:
                d.gt_add_noise = 1
                d.gt_noise = st.noise.data_ptr()
                d.gsa, d.gsb = self.scheduler.add_noise_scalars(int(timesteps[i + 1]), BF16)
        if not noise_pred.is_contiguous() or noise_pred.dtype != BF16:
            raise RuntimeError("transformer output must be contiguous bf16")
        K.dpm_step(d)
        st.extra["keep"] = (noise_pred, noise1, noise2)  # keep sources alive until the kernel is ordered
        st.latents = new_lat
        st.old_pred = pred

    # ------------------------------------------------------------------------------------------------------------
    def frame_layout(self, n_windows: int, num_frames: int, stride: int, latent_frames: int):
        """Latent-frame count of the whole clip and the first latent frame of each window (anyl.py:828-842,
        1052-1064)."""
        vt = self.vae_scale_factor_temporal
        if stride < num_frames:
            nfl = ((num_frames - 1) // vt + 1) * n_windows - (n_windows - 1) * ((num_frames - stride) // vt + 1)
        elif stride == num_frames:
            nfl = ((num_frames - 1) // vt) * n_windows + 1
        else:
            raise ValueError(f"stride: {stride}, num_frames: {num_frames}")
        starts = []
        for w in range(n_windows):
            start = w * latent_frames
            if w > 0 and stride < num_frames:
                start -= (int((num_frames - stride) // vt) + 1) * w
            elif w > 0 and stride == num_frames:
                start -= w
            starts.append(start)
        return nfl, starts

    def window_image_latents(self, w: int, win: dict, prev_latents: Optional[torch.Tensor], num_frames: int,
                             stride: int) -> torch.Tensor:
        """Window 0 conditions on the encoded first frame; window k>0 on the previous window's latent frame at the
        overlap boundary (anyl.py:862-872)."""
        if w == 0:
            return win["image_latents"]
        back = int((num_frames - stride) // self.vae_scale_factor_temporal)
        img = prev_latents[:, -back - 1:-back + 1 - 1] if -back < 0 else prev_latents[:, -1:]
        C, hh, ww = prev_latents.shape[2:]
        pad = torch.zeros(1, prev_latents.shape[1] - 1, C, hh, ww, device=self.device, dtype=BF16)
        return torch.cat([img, pad], dim=1)

    @torch.no_grad()
    def run_window(self, w: int, win: dict, image_latents: torch.Tensor, prompt_embeds_cfg: torch.Tensor,
                   timesteps: torch.Tensor, *, prev_states=None, prev_mask=None, capture: bool = False,
                   guidance_scale: float = 6.0, use_dynamic_cfg: bool = True, conditioning_scale: float = 1.0,
                   replace_gt: bool = True, mask_add: bool = True, prev_clip_weight: float = 0.0,
                   id_pool_resample_learnable: bool = False, add_first: bool = False,
                   step_noise: Optional[Callable[[], torch.Tensor]] = None, generator=None):
        """All denoising steps of one window (anyl.py:933-1050).  Returns (latents, last-step hidden states or
        None, the transformer's last resample mask) — the hand-off the next window needs."""
        st = self.make_window(win["latents"], image_latents, win["masked_video_latents"], win["mask"],
                              win.get("video_latents"), win.get("noise"))
        hh, ww = st.latents.shape[3], st.latents.shape[4]
        rope = self.rope_for(st.latents.shape[1], hh, ww)
        self.prev_resample_mask = prev_mask
        for i in range(len(timesteps)):
            self.step(st, i, timesteps, prompt_embeds_cfg, rope, guidance_scale=guidance_scale,
                      use_dynamic_cfg=use_dynamic_cfg, conditioning_scale=conditioning_scale, replace_gt=replace_gt,
                      mask_add=mask_add, add_first=add_first, id_pool_resample_learnable=id_pool_resample_learnable,
                      prev_window_states=prev_states if w > 0 else None, prev_clip_weight=prev_clip_weight,
                      capture_last_states=capture, step_noise=step_noise, generator=generator)
        return st.latents, (st.last_states if capture else None), self.prev_resample_mask

    def assemble(self, window_latents: List[torch.Tensor], num_frames: int, stride: int) -> torch.Tensor:
        """Overlap-averaged latent video [1, F_total, C, h, w] (anyl.py:1052-1069)."""
        lat0 = window_latents[0]
        Fw, C, hh, ww = lat0.shape[1:]
        nfl, starts = self.frame_layout(len(window_latents), num_frames, stride, Fw)
        acc = torch.zeros(1, nfl, C, hh, ww, device=lat0.device, dtype=BF16)
        counts = torch.zeros(nfl)
        for latents, start in zip(window_latents, starts):
            for i in range(Fw):
                acc[:, start + i] += latents[:, i]
                counts[start + i] += 1
        for i in range(nfl):
            if counts[i] > 0:
                acc[:, i] /= counts[i]
        return acc

    def prepare_call(self, prompt_embeds, negative_prompt_embeds, num_inference_steps: int):
        pe = torch.cat([negative_prompt_embeds, prompt_embeds], dim=0).to(self.device, BF16).contiguous()
        self.scheduler.set_timesteps(num_inference_steps)
        return pe, self.scheduler.timesteps.cpu()

    @torch.no_grad()
    def __call__(self, windows: List[dict], prompt_embeds: torch.Tensor, negative_prompt_embeds: torch.Tensor, *,
                 num_inference_steps: int = 50, num_frames: int = 49, stride: Optional[int] = None,
                 guidance_scale: float = 6.0, use_dynamic_cfg: bool = True, conditioning_scale: float = 1.0,
                 replace_gt: bool = True, mask_add: bool = True, prev_clip_weight: float = 0.0,
                 id_pool_resample_learnable: bool = False, add_first: bool = False,
                 step_noise: Optional[Callable[[], torch.Tensor]] = None, generator=None) -> torch.Tensor:
        """Window loop (anyl.py:759-1069) with output_type="latent".  windows[k] holds what prepare_latents /
        prepare_mask_latents produced for window k: latents, noise, video_latents, mask, masked_video_latents, and
        (window 0 only) image_latents.  Returns the overlap-averaged latent video [1, F_total, C, h, w]."""
        stride = num_frames if stride is None else stride
        pe, timesteps = self.prepare_call(prompt_embeds, negative_prompt_embeds, num_inference_steps)
        n_windows = len(windows)
        self.frame_layout(n_windows, num_frames, stride, windows[0]["latents"].shape[1])  # validates stride
        kw = dict(guidance_scale=guidance_scale, use_dynamic_cfg=use_dynamic_cfg, conditioning_scale=conditioning_scale,
                  replace_gt=replace_gt, mask_add=mask_add, prev_clip_weight=prev_clip_weight,
                  id_pool_resample_learnable=id_pool_resample_learnable, add_first=add_first, step_noise=step_noise,
                  generator=generator)
        outs = []
        latents, states, mask = None, None, None
        for w, win in enumerate(windows):
            img = self.window_image_latents(w, win, latents, num_frames, stride)
            latents, states, mask = self.run_window(w, win, img, pe, timesteps, prev_states=states, prev_mask=mask,
                                                    capture=w < n_windows - 1, **kw)
            outs.append(latents)
        return self.assemble(outs, num_frames, stride)


    # ------------------------------------------------------------------------------------------------------------
    # pixel-space entry: the VAE stage of each window on the HIP VAE
    # ------------------------------------------------------------------------------------------------------------
    def _vae_sample(self, x: torch.Tensor, generator) -> torch.Tensor:
        """retrieve_latents(vae.encode(x), generator) * scaling_factor, as [B, F, C, h, w] (anyl.py:145-152,
        412-423); the posterior noise is drawn from the caller's generator in `noise_dtype`."""
        post = self.vae.encode(x).latent_dist
        noise = randn_tensor(post.mean.shape, generator=generator, dtype=self.noise_dtype)
        z = post.sample_from(noise)
        return K.scale_bf16(z, float(self.vae.config.scaling_factor)).permute(0, 2, 1, 3, 4)

    def encode_window(self, w: int, window_video: torch.Tensor, mask_condition: torch.Tensor,
                      image: Optional[torch.Tensor], generator, prev_latents: Optional[torch.Tensor], num_frames: int,
                      stride: int, mask_background: bool = False) -> dict:
        """prepare_latents + prepare_mask_latents of window w (anyl.py:339-477, 852-908) from the preprocessed window
        video [1, 3, F, H, W] in [-1, 1], mask [1, 1, F, H, W] in [0, 1] and (window 0) the first frame [1, 3, H, W].
        Generator order as the reference: first-frame posterior (window 0), video posterior, initial noise,
        masked-video posterior."""
        dev = self.device
        vt = self.vae_scale_factor_temporal
        F, H, W = window_video.shape[2:]
        lf, hh, ww = (F - 1) // vt + 1, H // self.vae_scale_factor_spatial, W // self.vae_scale_factor_spatial
        C = self.transformer.config.in_channels // 2
        video = window_video.to(dev)
        if w == 0:
            img_lat = self._vae_sample(image.to(dev).unsqueeze(2), generator)  # [1, 1, C, h, w]
            image_latents = torch.cat([img_lat, torch.zeros(1, lf - 1, C, hh, ww, device=dev, dtype=BF16)], dim=1)
        else:
            image_latents = self.window_image_latents(w, {}, prev_latents, num_frames, stride)
        video_latents = self._vae_sample(video, generator)
        noise = randn_tensor((1, lf, C, hh, ww), generator=generator, device=dev, dtype=self.noise_dtype).to(BF16)
        mcond = mask_condition.to(dev, torch.float32)
        masked = K.mask_video(video, mcond, keep_above=mask_background)
        mask = K.nearest_resize_3d(mcond, (lf, hh, ww))
        masked_latents = self._vae_sample(masked, generator)
        return dict(latents=noise, noise=noise, image_latents=image_latents, video_latents=video_latents,
                    mask=torch.cat([mask] * 2), masked_video_latents=torch.cat([masked_latents] * 2))

    def decode(self, latents: torch.Tensor, output_type: str = "pt") -> torch.Tensor:
        """decode_latents (anyl.py:479-484) + the video processor's denormalisation for output_type "pt"
        ([B, F, 3, H, W] in [0, 1]); "raw" returns the VAE output [B, 3, F, H, W] in [-1, 1]."""
        z = K.scale_bf16(latents.permute(0, 2, 1, 3, 4).contiguous(), 1.0 / float(self.vae.config.scaling_factor))
        video = self.vae.decode(z).sample
        if output_type == "raw":
            return video
        return K.denormalize_bf16(video).permute(0, 2, 1, 3, 4)

    @torch.no_grad()
    def generate(self, video: torch.Tensor, masks: torch.Tensor, image: torch.Tensor, prompt_embeds: torch.Tensor,
                 negative_prompt_embeds: torch.Tensor, *, generator=None, num_inference_steps: int = 50,
                 num_frames: int = 49, stride: Optional[int] = None, output_type: str = "pt",
                 mask_background: bool = False, **kw) -> torch.Tensor:
        """The whole any-length call from preprocessed pixels: video [1, 3, T, H, W] in [-1, 1] (preprocess_video),
        masks [1, 1, T, H, W] in [0, 1] (the masked-video processor), image [1, 3, H, W] (the first frame, window 0).
        Returns the latent video ("latent") or the decoded frames ("pt": [1, F, 3, H, W] in [0, 1])."""
        if self.vae is None:
            raise ValueError("generate() needs the harness built with vae=")
        stride = num_frames if stride is None else stride
        pe, timesteps = self.prepare_call(prompt_embeds, negative_prompt_embeds, num_inference_steps)
        total = video.shape[2]
        n_windows = (total - num_frames) // stride + 1
        outs = []
        latents, states, mask = None, None, None
        for w in range(n_windows):
            s0 = w * stride
            win = self.encode_window(w, video[:, :, s0:s0 + num_frames], masks[:, :, s0:s0 + num_frames],
                                     image if w == 0 else None, generator, latents, num_frames, stride,
                                     mask_background=mask_background)
            latents, states, mask = self.run_window(w, win, win["image_latents"], pe, timesteps, prev_states=states,
                                                    prev_mask=mask, capture=w < n_windows - 1, generator=generator,
                                                    **kw)
            outs.append(latents)
        lat = self.assemble(outs, num_frames, stride)
        return lat if output_type == "latent" else self.decode(lat, output_type)


@torch.no_grad()
def run_any_length_pipelined(harness: CogVideoXI2VDualInpaintAnyLHarness, stages, clips: List[dict],
                             prompt_embeds: torch.Tensor, negative_prompt_embeds: torch.Tensor, *,
                             num_inference_steps: int = 50, num_frames: int = 49, stride: Optional[int] = None,
                             **kw) -> List[torch.Tensor]:
    """The any-length loop of `CogVideoXI2VDualInpaintAnyLHarness.__call__` for several clips on a multi-rank
    stage pipeline (`distributed.WindowStages`): window w of every clip runs on stage w % S;
    consecutive stages hand off (final latents, last-step hidden states, resample mask, generator state); with
    `WindowStages(cfg_split=True)` each stage is a CFG pair exchanging one noise prediction per step.  Same result
    as running the clips one after another through `harness(...)` with clip j's generator."""
    from .distributed import run_window_chain
    stride = num_frames if stride is None else stride
    harness.cfg_pair = stages.pair
    pe, timesteps = harness.prepare_call(prompt_embeds, negative_prompt_embeds, num_inference_steps)
    first = clips[0]["windows"][0]["latents"]
    cfg = harness.transformer.config
    p = cfg.patch_size
    _, F, C, hh, ww = first.shape
    ntok = pe.shape[1] + F * (hh // p) * (ww // p)
    rows = 1 if stages.pair is not None else 2
    lat_like = torch.empty(tuple(first.shape), device=harness.device, dtype=BF16)
    state_shape = (rows, ntok, cfg.num_attention_heads * cfg.attention_head_dim)
    mask_shape = (rows, ntok)

    def rw(j, w, win, img, prev_states, prev_mask, capture):
        return harness.run_window(w, win, img, pe, timesteps, prev_states=prev_states, prev_mask=prev_mask,
                                  capture=capture, generator=clips[j].get("generator"), **kw)

    return run_window_chain(stages, clips, rw,
                            lambda w, win, prev: harness.window_image_latents(w, win, prev, num_frames, stride),
                            lambda lats: harness.assemble(lats, num_frames, stride), lat_like, state_shape,
                            mask_shape)


@torch.no_grad()
def run_any_length_concurrent(harness: CogVideoXI2VDualInpaintAnyLHarness, windows: List[dict],
                              prompt_embeds: torch.Tensor, negative_prompt_embeds: torch.Tensor, *,
                              num_inference_steps: int = 50, num_frames: int = 49, stride: Optional[int] = None,
                              seed: int = 0, **kw) -> torch.Tensor:
    """NON-PARITY multi-GPU any-length mode (the north-star's "clip segments sharded across the GPUs with an
    all-gather of the overlapping-region latents"; distributed.run_windows_concurrent): every window needs its own
    `image_latents` (its first frame, encoded) and runs without the previous window's conditioning latent or
    hidden states (prev_clip_weight is forced to 0); window w draws its scheduler noise from a generator seeded
    seed + w.  The reference's chained semantics are `harness(...)` / `run_any_length_pipelined`."""
    from .distributed import run_windows_concurrent
    stride = num_frames if stride is None else stride
    pe, timesteps = harness.prepare_call(prompt_embeds, negative_prompt_embeds, num_inference_steps)
    kw = dict(kw, prev_clip_weight=0.0)
    for w, win in enumerate(windows):
        if "image_latents" not in win:
            raise ValueError(f"window {w} has no image_latents (the concurrent mode conditions every window on its "
                             "own first frame)")

    def rw(w, win):
        lat, _, _ = harness.run_window(w, win, win["image_latents"], pe, timesteps, prev_states=None, prev_mask=None,
                                       capture=False, generator=torch.Generator().manual_seed(seed + w), **kw)
        return lat

    like = torch.empty(tuple(windows[0]["latents"].shape), device=harness.device, dtype=BF16)
    return run_windows_concurrent(windows, rw, lambda outs: harness.assemble(outs, num_frames, stride), like)
