"""Denoising steps/s of the VideoPainter hot path on MI355X (BASELINE.json config 2, data-parallel clips for N>1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--cpu-baseline-only]
    (N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

One step = one iteration of the any-length pipeline's denoising loop (anyl.py:933-1034): 2-layer branch forward +
42-layer CogVideoX-5b-I2V transformer forward at B=2 (CFG) with return_hidden_states / resample mask as the pipeline
requests them, then the fused CFG + DPM-Solver + replace-gt kernel.  Random-init weights of the 5b-I2V architecture
(no checkpoints offline), synthetic latents of the 49f 480x720 shape (latent 13x60x90, N = 226 + 17550 tokens).
N GPUs: each rank runs its own clip (weak scaling, no per-step collective); weights are initialised on rank 0 and
broadcast over RCCL (config 3).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "denoising steps/sec, CogVideoX-5b+branch 49f 480×720, 1→8 MI355X; MFMA util%"
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA peak, MI355X_MICROARCH.md
PEAK_FP8_TFLOPS = 5000.0   # dense fp8 (block-scaled MFMA) peak
B, T, F, D, H, L, LB = 2, 226, 13, 3072, 48, 42, 2
# BASELINE config 2 (the headline): 49f 480x720 -> latent 60x90; config 5: 49f 720x1280 -> latent 90x160, fp8 FFN
HL, WL = 60, 90
NV = F * (HL // 2) * (WL // 2)
NTOK = T + NV


def set_config(cfg: int) -> None:
    global HL, WL, NV, NTOK
    HL, WL = (90, 160) if cfg == 5 else (60, 90)
    NV = F * (HL // 2) * (WL // 2)
    NTOK = T + NV


def step_flops(split: bool = False):
    """Algorithmic FLOP per denoising step: transformer + branch at B=2.  split=True returns
    (total, FeedForward part) — the FeedForward GEMMs are the fp8 part of config 5."""
    blk = 24 * NTOK * D * D + 4 * NTOK * NTOK * D
    tr = B * (L * blk + 2 * NV * 128 * D + 2 * T * 4096 * D + 2 * NV * D * 64)
    br = B * (LB * blk + 2 * NV * 132 * D + 2 * T * 4096 * D + LB * 2 * NTOK * D * D)
    ffn = B * (L + LB) * 16 * NTOK * D * D
    return (float(tr + br), float(ffn)) if split else float(tr + br)


def attn_flops_per_launch() -> float:
    return 4.0 * B * H * NTOK * NTOK * 64


def profiled_traffic():
    """Latest committed PMC-derived HBM traffic per attention launch (profiles/<round>_attention_traffic.json,
    written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_attention_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(seconds_budget: float = 30.0) -> dict:
    """The oracle (plain PyTorch CPU restatement of the reference) on this host's cores: one full-size
    CogVideoXBlock forward at B=2, N=17776 in bf16 (the reference's inference dtype), extrapolated to a step as
    (42 + 2) block-forwards (blocks are >99% of the step's FLOPs)."""
    from oracle import cogvideox_oracle as O
    from videopainter_amd.config import block_shapes
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    sd = {}
    for k, shp in block_shapes(D, 512).items():
        std = 0.02 if len(shp) == 1 else (1.0 / math.sqrt(shp[1]))
        sd["b." + k] = (torch.randn(shp, generator=g) * std + (1.0 if (len(shp) == 1 and ".norm" in k and
                                                                        k.endswith("weight")) else 0.0)).bfloat16()
    for n in ("norm_q", "norm_k"):
        sd[f"b.attn1.{n}.weight"] = torch.ones(64, dtype=torch.bfloat16)
        sd[f"b.attn1.{n}.bias"] = torch.zeros(64, dtype=torch.bfloat16)
    h = torch.randn(B, NV, D, generator=g).bfloat16()
    e = torch.randn(B, T, D, generator=g).bfloat16()
    temb = torch.randn(B, 512, generator=g).bfloat16()
    rope = O.prepare_rotary_positional_embeddings(480, 720, F, 64)
    t0 = time.time()
    with torch.no_grad():
        O.block_forward(sd, "b", dict(num_attention_heads=H, norm_eps=1e-5), h, e, temb, rope)
    dt = time.time() - t0
    step_s = (L + LB) * dt
    return {"value": 1.0 / step_s, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle (plain PyTorch CPU restatement) bf16: 1 full CogVideoXBlock fwd at B=2, N={NTOK} took "
                      f"{dt:.1f}s on {threads} threads; step = (42+2) block-forwards = {step_s:.0f}s"}


def build_models(device, seed: int, rank: int, world: int):
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    from videopainter_amd.config import COGVIDEOX_5B_I2V
    # config 5 (720x1280): random-init 5b-shaped model whose learned positional embedding is sized for the latent
    # 90x160 grid (SURVEY.md finding 2: the real 5b-I2V checkpoint is locked to 60x90)
    cfg = dict(COGVIDEOX_5B_I2V, sample_height=HL, sample_width=WL)
    with device_scope(device):
        tr = CogVideoXTransformer3DModel(**cfg)
        br = CogvideoXBranchModel(**dict(cfg, num_layers=LB))
    if rank == 0 or world == 1:
        tr.init_synthetic_weights_(seed)
        br.init_synthetic_weights_(seed + 1)
    if world > 1:
        from videopainter_amd.distributed import broadcast_module
        for m in (tr, br):
            broadcast_module(m, src=0)
    torch.cuda.synchronize()
    return tr, br


def make_state(harness, device, seed: int):
    """Synthetic config-2 window inputs: N(0,1) latents, image latent frame 0 only, centred
    50% x 50% mask with frame 0 unmasked (first_frame_gt), masked latents zeroed inside the mask."""
    g = torch.Generator().manual_seed(seed)
    lat = torch.randn(1, F, 16, HL, WL, generator=g)
    img = torch.zeros(1, F, 16, HL, WL)
    img[:, 0] = torch.randn(1, 16, HL, WL, generator=g) * 0.7
    mask = torch.zeros(1, 1, F, HL, WL)
    mask[:, :, 1:, HL // 4:HL // 4 + HL // 2, WL // 4:WL // 4 + WL // 2] = 1.0
    vid = torch.randn(1, F, 16, HL, WL, generator=g)
    masked = vid * (1 - mask.permute(0, 2, 1, 3, 4))
    st = harness.make_window(lat, img, torch.cat([masked] * 2), torch.cat([mask] * 2), vid, lat.clone())
    pe = torch.randn(2, T, 4096, generator=g).to(device, torch.bfloat16)
    return st, pe


def config4_step_flops(window: int) -> float:
    """Algorithmic FLOP of one config-4 denoising step (1.024e15 window 0, 1.080e15 windows 1-3):
    the ID-resample processor doubles every transformer attention's keys (the masked / previous-window K/V
    segment, Nk = 2N); windows > 0 also project the previous window's states to K/V (4 N D^2 per block)."""
    attn = 4 * NTOK * (2 * NTOK) * D
    kv = 4 * NTOK * D * D if window > 0 else 0
    blk = 24 * NTOK * D * D + attn + kv
    tr = B * (L * blk + 2 * NV * 128 * D + 2 * T * 4096 * D + 2 * NV * D * 64)
    br_blk = 24 * NTOK * D * D + 4 * NTOK * NTOK * D
    br = B * (LB * br_blk + 2 * NV * 132 * D + 2 * T * 4096 * D + LB * 2 * NTOK * D * D)
    return float(tr + br)


def run_config4(args, world: int, local: int) -> None:
    """BASELINE config 4 on one GPU: the VideoPainterID any-length chain — 196 frames as 4 windows of 49 at
    stride 49, ID-resample processor, prev_clip_weight 0.5, each window conditioned on the previous one's last
    latent and last-step hidden states — with --steps denoising steps per window (the reference runs 50; the
    per-step work is the same).  value = denoising steps/s over the whole chain.  The chain is serial; its
    multi-GPU form is the window-stage pipeline (distributed.run_window_chain, tests/test_distributed_cpu.py)."""
    if world != 1:
        raise SystemExit("bench --config 4 runs the serial chain on one GPU (multi-GPU: window-stage pipeline tests)")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    from videopainter_amd import kernels as K
    from videopainter_amd.config import COGVIDEOX_5B_I2V
    from videopainter_amd.pipeline import CogVideoXI2VDualInpaintAnyLHarness
    from videopainter_amd.scheduler import CogVideoXDPMScheduler
    t_setup = time.time()
    cfg = dict(COGVIDEOX_5B_I2V, sample_height=HL, sample_width=WL)
    with device_scope(device):
        tr = CogVideoXTransformer3DModel(**dict(cfg, id_pool_resample_learnable=True))
        br = CogvideoXBranchModel(**dict(cfg, num_layers=LB))
    tr.init_synthetic_weights_(1234)
    br.init_synthetic_weights_(1235)
    sch = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                                clip_sample=False, set_alpha_to_one=True, timestep_spacing="trailing")
    harness = CogVideoXI2VDualInpaintAnyLHarness(tr, br, sch)
    n_windows = 4
    g = torch.Generator().manual_seed(42)
    windows = []
    for w in range(n_windows):
        lat = torch.randn(1, F, 16, HL, WL, generator=g)
        vid = torch.randn(1, F, 16, HL, WL, generator=g)
        mask = torch.zeros(1, 1, F, HL, WL)
        mask[:, :, 1:, HL // 4:HL // 4 + HL // 2, WL // 4:WL // 4 + WL // 2] = 1.0
        masked = vid * (1 - mask.permute(0, 2, 1, 3, 4))
        win = dict(latents=lat, noise=lat.clone(), video_latents=vid, mask=torch.cat([mask] * 2),
                   masked_video_latents=torch.cat([masked] * 2))
        if w == 0:
            img = torch.zeros(1, F, 16, HL, WL)
            img[:, 0] = torch.randn(1, 16, HL, WL, generator=g) * 0.7
            win["image_latents"] = img
        windows.append({k: v.to(device, torch.bfloat16) for k, v in win.items()})
    pe = torch.randn(1, T, 4096, generator=g).to(device, torch.bfloat16)
    npe = torch.randn(1, T, 4096, generator=g).to(device, torch.bfloat16)
    kw = dict(num_frames=49, stride=49, guidance_scale=6.0, use_dynamic_cfg=True, replace_gt=True, mask_add=True,
              prev_clip_weight=0.5, id_pool_resample_learnable=True)
    log(f"[bench] config 4 setup {time.time() - t_setup:.1f}s")
    with torch.no_grad():
        harness(windows[:2], pe, npe, num_inference_steps=max(1, args.warmup), generator=torch.Generator().manual_seed(0),
                **kw)  # warm-up: both window kinds (resample w0, prev-clip w>0)
        torch.cuda.synchronize()
        with K.timed_launches("attention", "gemm") as tl:
            t0 = time.perf_counter()
            out = harness(windows, pe, npe, num_inference_steps=args.steps,
                          generator=torch.Generator().manual_seed(0), **kw)
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
    n_steps = n_windows * args.steps
    steps_per_s = n_steps / elapsed
    fl = sum(config4_step_flops(w) for w in range(n_windows)) * args.steps
    attn_ms = tl.mean_ms("attention")
    line = {
        "metric": METRIC, "value": steps_per_s, "unit": "steps/s", "n_gpus": 1, "steps": n_steps,
        "warmup": args.warmup, "ms_per_step": elapsed / n_steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic latents/prompt embeds of the 4 x 49f 480x720 windows; random-init CogVideoX-5b-I2V "
                "(ID-resample processor) + 2-layer branch weights (no checkpoints offline)",
        "config": {"workload": f"BASELINE config 4: any-length 196 frames = 4 windows x 49f 480x720 at stride 49, "
                               f"ID-resample + prev_clip_weight 0.5, {args.steps} denoising steps per window "
                               "(value = denoising steps/s over the chain)",
                   "windows": n_windows, "tokens": NTOK, "keys_per_attention": 2 * NTOK, "layers": L,
                   "branch_layers": LB, "parallelism": "serial window chain on 1 GPU"},
        "step_flop_mean": fl / n_steps,
        "step_mfma_frac": fl / elapsed / (PEAK_BF16_TFLOPS * 1e12),
        "attention_ms_per_launch": attn_ms, "attention_launches": tl.count("attention"),
        "attention_ms_per_step": attn_ms * tl.count("attention") / n_steps,
        "output_latents": list(out.shape),
    }
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-only", action="store_true")
    ap.add_argument("--config", type=int, default=2, choices=(2, 4, 5),
                    help="BASELINE config: 2 = 49f 480x720 bf16 (headline), 4 = the any-length ID-resample chain "
                         "(4 windows, --steps denoising steps each), 5 = 49f 720x1280 with attention + FeedForward in fp8")
    args = ap.parse_args()
    set_config(args.config)

    if args.cpu_baseline_only:
        print(json.dumps({"cpu_baseline": cpu_baseline()}))
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config == 4:
        run_config4(args, world, local)
        return
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        from videopainter_amd.distributed import init as dist_init
        dist_init("nccl", device)

    from videopainter_amd import kernels as K
    from videopainter_amd.pipeline import CogVideoXI2VDualInpaintAnyLHarness
    from videopainter_amd.scheduler import CogVideoXDPMScheduler

    t_setup = time.time()
    tr, br = build_models(device, 1234, rank, world)
    sch = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                                clip_sample=False, set_alpha_to_one=True, timestep_spacing="trailing")
    sch.set_timesteps(50)
    timesteps = sch.timesteps.cpu()
    harness = CogVideoXI2VDualInpaintAnyLHarness(tr, br, sch)
    st, pe = make_state(harness, device, 42 + rank)
    rope = harness.rope_for(F, HL, WL)
    gen = torch.Generator().manual_seed(42 + rank)
    fp8_drift = None
    if args.config == 5:
        # the fp8 path's drift from this same model in bf16, one full forward on the step's inputs
        # (re-stated tolerance of config 5; block level vs the reference: tests/test_model_gpu.py)
        with torch.no_grad():
            lmi = torch.cat([torch.cat([st.latents] * 2), st.image_in], dim=2)
            ts = torch.full((2,), 999, device=device, dtype=torch.int64)

            def fwd():
                bs = br(hidden_states=torch.cat([st.latents] * 2), encoder_hidden_states=pe, branch_cond=st.branch_in,
                        timestep=ts, image_rotary_emb=rope, return_dict=False)[0]
                return tr(hidden_states=lmi, encoder_hidden_states=pe, branch_block_samples=bs, timestep=ts,
                          image_rotary_emb=rope, branch_block_masks=st.mask1, return_dict=False)[0].float()
            ref16 = fwd()
            tr.enable_fp8()
            br.enable_fp8()
            out8 = fwd()
            fp8_drift = float((out8 - ref16).norm() / ref16.norm())
            del ref16, out8, lmi
        log(f"[bench] config 5: fp8 QKV+attention+FFN noise_pred vs bf16 rel-L2 {fp8_drift:.3e}")
    log(f"[bench] setup {time.time() - t_setup:.1f}s; rank {rank}/{world}")

    def one(i):
        k = i % len(timesteps)
        if k == 0:
            st.old_pred = None
        harness.step(st, k, timesteps, pe, rope, guidance_scale=6.0, use_dynamic_cfg=True, replace_gt=True,
                     mask_add=True, generator=gen)

    with torch.no_grad():
        for i in range(args.warmup):
            one(i)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        with K.timed_launches("attention", "attention_fp8", "gemm", "gemm_mx") as tl:
            t0 = time.perf_counter()
            for i in range(args.warmup, args.warmup + args.steps):
                one(i)
            torch.cuda.synchronize()
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
    if dist is not None:
        from videopainter_amd.distributed import max_over_ranks
        elapsed = max_over_ranks(elapsed, device)
    steps_per_s = world * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    attn_name = "attention_fp8" if args.config == 5 else "attention"
    attn_ms = tl.mean_ms(attn_name)
    attn_peak = PEAK_FP8_TFLOPS if args.config == 5 else PEAK_BF16_TFLOPS
    attn_tf = attn_flops_per_launch() / (attn_ms * 1e-3) / 1e12
    gemm_ev = tl.events.get("gemm", []) + tl.events.get("gemm_mx", [])
    torch.cuda.synchronize()
    gemm_ms_total = sum(s.elapsed_time(e) for s, e in gemm_ev)
    traffic, traffic_src = profiled_traffic() if args.config == 2 else (None, None)  # PMC file is per config
    total_fl, ffn_fl = step_flops(split=True)
    if args.config == 5:  # time the step would take at the dense peaks of the dtypes its MFMAs use
        f8_fl = ffn_fl + (L + LB) * (attn_flops_per_launch() + B * 6 * NTOK * D * D)  # + attention, QKV per block
        t_ideal = (total_fl - f8_fl) / (PEAK_BF16_TFLOPS * 1e12) + f8_fl / (PEAK_FP8_TFLOPS * 1e12)
    else:
        t_ideal = total_fl / (PEAK_BF16_TFLOPS * 1e12)
    step_frac = t_ideal * (steps_per_s / world)
    if not math.isfinite(steps_per_s):
        raise RuntimeError("non-finite timing")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == 2:
        del st
        cpu = cpu_baseline()
    if rank == 0:
        out = {
            "metric": METRIC, "value": steps_per_s, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.config == 2 else "bf16 + fp8 (e4m3, block-scaled MFMA) QKV, attention, FeedForward",
            "data": f"synthetic latents/prompt embeds of the 49f {HL * 8}x{WL * 8} shape; random-init "
                    "CogVideoX-5b-I2V (42 layers) + 2-layer branch weights (no checkpoints offline)",
            "config": {"workload": (f"BASELINE config {args.config}: CogVideoX-5b-I2V + 2-layer branch, 49f "
                                    f"{HL * 8}x{WL * 8} (latent 13x{HL}x{WL}), CFG batch 2, {T}+{NV}={NTOK} tokens, "
                                    "1 denoising step = branch + transformer + CFG/DPM/replace-gt"
                                    + (", QKV projection + attention + FeedForward in fp8" if args.config == 5
                                       else "")),
                       "clips_per_gpu": 1, "cfg_batch": B,
                       "tokens": NTOK, "layers": L, "branch_layers": LB,
                       "parallelism": f"dp{world} (independent clips, weights broadcast over RCCL)"},
            "roofline": {"kernel": "attention (vp_attention_fwd_%s, dominant by time)"
                                   % ("fp8" if args.config == 5 else "bf16"),
                         "bound": "mfma", "achieved": attn_tf, "peak": attn_peak, "unit": "TFLOP/s",
                         "frac": attn_tf / attn_peak, "traffic": traffic, "traffic_unit": "bytes/launch",
                         "traffic_source": traffic_src,
                         "per_launch_ms": attn_ms, "launches": tl.count(attn_name),
                         "algorithmic_flop_per_launch": attn_flops_per_launch()},
            "step_mfma_frac": step_frac,
            "fp8_rel_l2_vs_bf16": fp8_drift,
            "step_flop": step_flops(),
            "gemm_ms_per_step": gemm_ms_total / args.steps,
            "attention_ms_per_step": attn_ms * tl.count(attn_name) / args.steps,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
