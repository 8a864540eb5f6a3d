"""Denoising steps/s of the VideoPainter hot path on MI355X (BASELINE.json config 2, data-parallel clips for N>1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|4|5] [--mode dp|cfgpair|ulysses|stages]
                    [--no-cpu-baseline] [--cpu-baseline-only [--cpu-full-step]]
    (N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

One step = one iteration of the any-length pipeline's denoising loop (anyl.py:933-1034): 2-layer branch forward +
42-layer CogVideoX-5b-I2V transformer forward at B=2 (CFG) with return_hidden_states / resample mask as the pipeline
requests them, then the fused CFG + DPM-Solver + replace-gt kernel.  Random-init weights of the 5b-I2V architecture
(no checkpoints offline), synthetic latents of the 49f 480x720 shape (latent 13x60x90, N = 226 + 17550 tokens).
N GPUs, --mode dp (default): each rank runs its own clip (weak scaling, no per-step collective); weights are
initialised on rank 0 and broadcast over RCCL (config 3).  --mode cfgpair: one clip per rank PAIR, each rank runs one
CFG half at B=1 and the pair exchanges the noise prediction with one all-gather per step (SURVEY.md §8e latency
mode); value = clips' denoising steps/s summed over pairs.  The timed steps run without instrumentation; a separate
pass afterwards records HIP events around every GEMM / attention launch for the per-kernel roofline.  Rank 0 prints
ONE JSON line.
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


def profiled_traffic(kind: str):
    """Latest committed PMC-derived HBM traffic per launch of kernel class `kind` ("attention" | "attention_fp8" |
    "gemm"):
    profiles/<round>_<kind>_traffic.json, written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes (MI355X_MICROARCH.md §HBM correction)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{kind}_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores(capped: bool = True) -> int:
    """The thread count the CPU baseline runs at (the reference CPU path on the node's own host
    cores): the physical cores of this process's affinity mask (SMT siblings counted once), capped by the CPU share
    the host allots this job when it states one in OMP_NUM_THREADS (the GPU boxes set it to 16 per GPU and ask jobs
    to keep to it; the CPU is shared with the other GPUs' jobs).  VP_CPU_BASELINE_THREADS overrides both."""
    env = int(os.environ.get("VP_CPU_BASELINE_THREADS", "0") or 0)
    if env > 0 and capped:
        return env
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    seen = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            seen.add((pkg, core))
        except OSError:
            seen.add(("cpu", c))
    return max(1, min(len(seen), share) if share > 0 and capped else len(seen))


def _oracle_block_weights(g, dtype):
    from videopainter_amd.config import block_shapes
    sd = {}
    for k, shp in block_shapes(D, 512).items():
        std = 0.02 if len(shp) == 1 else (1.0 / math.sqrt(shp[1]))
        sd["b." + k] = (torch.randn(shp, generator=g) * std + (1.0 if (len(shp) == 1 and ".norm" in k and
                                                                        k.endswith("weight")) else 0.0)).to(dtype)
    for n in ("norm_q", "norm_k"):
        sd[f"b.attn1.{n}.weight"] = torch.ones(64, dtype=dtype)
        sd[f"b.attn1.{n}.bias"] = torch.zeros(64, dtype=dtype)
    return sd


def block_flop() -> float:
    """Algorithmic FLOP of one CogVideoXBlock forward at B=2."""
    return float(B * (24 * NTOK * D * D + 4 * NTOK * NTOK * D + 2 * 2 * 512 * 18432))


def cpu_baseline() -> dict:
    """The oracle (plain PyTorch CPU restatement of the reference, parity-locked to it: tests/test_oracle_golden.py)
    on this host's cores, a BOUNDED sample of the config-2 step: a warm-up block at N/8, then one full-size
    CogVideoXBlock forward at B=2, N=17776 in bf16 (the reference's inference dtype) and one in fp32, each timed;
    the step (branch + transformer, 6.974e14 FLOP) is extrapolated by FLOP from the block (7.9e12 x 2 = 99 % of the
    step is the 44 blocks).  `--cpu-baseline-only --cpu-full-step` times a whole step instead
    (profiles/r02_cpu_full_step.json)."""
    from oracle import cogvideox_oracle as O
    threads = physical_cores()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    rope = O.prepare_rotary_positional_embeddings(480, 720, F, 64)
    out = {}
    with torch.no_grad():
        sdw = _oracle_block_weights(g, torch.bfloat16)  # warm-up block: allocator, thread pool, kernels
        n8 = NV // 8
        O.block_forward(sdw, "b", dict(num_attention_heads=H, norm_eps=1e-5),
                        torch.randn(B, n8, D, generator=g).bfloat16(), torch.randn(B, T, D, generator=g).bfloat16(),
                        torch.randn(B, 512, generator=g).bfloat16(), (rope[0][:n8], rope[1][:n8]))
        for dt, name in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
            sd = _oracle_block_weights(g, dt)
            h = torch.randn(B, NV, D, generator=g).to(dt)
            e = torch.randn(B, T, D, generator=g).to(dt)
            temb = torch.randn(B, 512, generator=g).to(dt)
            t0 = time.time()
            O.block_forward(sd, "b", dict(num_attention_heads=H, norm_eps=1e-5), h, e, temb, rope)
            out[name] = time.time() - t0
            del sd, h, e
    step_s = {k: v * step_flops() / block_flop() for k, v in out.items()}
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"value": 1.0 / step_s["bf16"], "unit": "steps/s", "cores": threads, "kind": "port",
            "threads": torch.get_num_threads(), "host_physical_cores": physical_cores(capped=False),
            "affinity_cpus": aff, "host_cpus": os.cpu_count(),
            "value_fp32": 1.0 / step_s["fp32"], "cpu_model": _cpu_model(),
            "sample": f"EXTRAPOLATED, not a timed step: oracle (plain PyTorch CPU restatement) after a warm-up "
                      f"block, 1 full-size CogVideoXBlock "
                      f"forward at B=2, N={NTOK} took {out['bf16']:.1f} s in bf16 and {out['fp32']:.1f} s in fp32 on "
                      f"{threads} threads = the physical cores of the process affinity mask capped by the job's "
                      f"CPU share OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')} ({aff} of the host's "
                      f"{os.cpu_count()} logical CPUs in the mask; "
                      f"{_cpu_model()}); step = step FLOP / block FLOP x block time = "
                      f"{step_s['bf16']:.0f} s bf16 / {step_s['fp32']:.0f} s fp32"}


def cpu_full_step(dtype=torch.bfloat16) -> dict:
    """One complete config-2 denoising step on the CPU through the oracle: branch (2 blocks) + transformer (42
    blocks) forward at B=2 with the full 5b-I2V weights (random, std 1/sqrt(fan_in)), CFG + DPM step + replace-gt;
    timed after a warm-up block, on the physical cores of the affinity mask (~7 min in bf16 on 16 threads)."""
    from oracle import cogvideox_oracle as O
    from videopainter_amd.config import COGVIDEOX_5B_I2V, full_config, state_dict_shapes
    torch.set_num_threads(physical_cores())
    g = torch.Generator().manual_seed(0)
    tcfg = full_config(dict(COGVIDEOX_5B_I2V))
    bcfg = full_config(dict(COGVIDEOX_5B_I2V, num_layers=LB), True)

    def weights(cfg, branch):
        sd = {}
        for k, shp in state_dict_shapes(cfg, branch).items():
            t = torch.empty(shp, dtype=dtype)
            if len(shp) == 1:
                t.fill_(1.0 if (k.endswith("norm.weight") or ".norm_" in k and k.endswith("weight") or
                                k.startswith("norm_final.weight")) else 0.0)
            else:
                t.normal_(0.0, 1.0 / math.sqrt(math.prod(shp[1:])), generator=g)
            sd[k] = t
        return sd
    t_w = time.time()
    tsd, bsd = weights(tcfg, False), weights(bcfg, True)
    t_w = time.time() - t_w
    rope = O.prepare_rotary_positional_embeddings(480, 720, F, 64)
    lat = torch.randn(1, F, 16, HL, WL, generator=g)
    img = torch.zeros(1, F, 16, HL, WL)
    img[:, 0] = torch.randn(1, 16, HL, WL, generator=g) * 0.7
    mask = torch.zeros(2, F, 1, HL, WL)
    mask[:, 1:, :, HL // 4:HL // 4 + HL // 2, WL // 4:WL // 4 + WL // 2] = 1.0
    masked = torch.randn(2, F, 16, HL, WL, generator=g) * (1 - mask)
    pe = torch.randn(2, T, 4096, generator=g)
    sch = O.DPMSchedulerOracle()
    sch.set_timesteps(50)
    ts = [int(x) for x in sch.timesteps]
    with torch.no_grad():
        warm = {"b." + k[len("transformer_blocks.0."):]: v for k, v in tsd.items()
                if k.startswith("transformer_blocks.0.")}
        O.block_forward(warm, "b", dict(num_attention_heads=H, norm_eps=1e-5),
                        torch.randn(B, NV // 8, D, generator=g).to(dtype), torch.randn(B, T, D, generator=g).to(dtype),
                        torch.randn(B, 512, generator=g).to(dtype), (rope[0][:NV // 8], rope[1][:NV // 8]))
        t0 = time.time()
        c = lambda x: x.to(dtype)  # noqa: E731
        lmi = torch.cat([torch.cat([lat] * 2), torch.cat([img] * 2)], dim=2)
        tt = torch.full((2,), ts[0], dtype=torch.int64)
        bs = O.branch_forward(bsd, bcfg, c(torch.cat([lat] * 2)), c(pe), c(torch.cat([masked, mask], 2)), tt, rope)
        out = O.transformer_forward(tsd, tcfg, c(lmi), c(pe), tt, rope, branch_block_samples=bs,
                                    branch_block_masks=c(mask))[0].float()
        u, cnd = out.chunk(2)
        gsc = O.dynamic_cfg_scale(6.0, 50, ts[0])
        mo = u + gsc * (cnd - u)
        n1 = torch.randn(lat.shape, generator=g)
        n2 = torch.randn(lat.shape, generator=g)
        prev, _ = sch.step(mo, None, ts[0], None, lat.to(torch.bfloat16), n1, n2)
        gt = sch.add_noise(lat.to(torch.bfloat16), n1.to(torch.bfloat16), torch.tensor([ts[1]]))
        m1 = mask[:1]
        _ = (1 - m1) * gt + m1 * prev.to(torch.bfloat16)
        step = time.time() - t0
    return {"step_seconds": step, "steps_per_s": 1.0 / step, "dtype": str(dtype).replace("torch.", ""),
            "threads": torch.get_num_threads(), "cpu_model": _cpu_model(), "weight_init_seconds": t_w,
            "what": "oracle: branch (2 blocks) + transformer (42 blocks) forward at B=2, N=17776, full 5b-I2V "
                    "weights, + CFG + DPM step + replace-gt; after a warm-up block"}


def build_models(device, seed: int, rank: int, world: int, bcast: str = "scatter_allgather", always: bool = False):
    """Random-init 5b-I2V transformer + 2-layer branch; for N>1 initialised on rank 0 and broadcast over RCCL.
    Returns (transformer, branch, replication record or None): {"seconds": the chosen method's time (float),
    "method", "per_method": {method: seconds}, "verified_buckets": {method: count}}.  always: replicate and verify
    at world size 1 too (--rccl-world1: the RCCL path on one GPU, identities there)."""
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
    t_b = None
    if world > 1 or always:
        # replicate with the chosen method (timed), check every rank's bytes against rank 0's (per-bucket digests:
        # the first hardware run of the RCCL-only code paths validates itself), then time the other method too
        from videopainter_amd.distributed import barrier, broadcast_module, verify_replicas
        t_b = {"method": bcast, "per_method": {}, "verified_buckets": {}}
        for method in (bcast, "broadcast" if bcast == "scatter_allgather" else "scatter_allgather"):
            torch.cuda.synchronize()
            barrier(device)
            t0 = time.perf_counter()
            for m in (tr, br):
                broadcast_module(m, src=0, method=method, always=always)
            torch.cuda.synchronize()
            barrier(device)
            t_b["per_method"][method] = time.perf_counter() - t0
            checks = [verify_replicas(m, always=always) for m in (tr, br)]
            if not all(ok for ok, _ in checks):
                raise RuntimeError(f"weight replication ({method}) left ranks with different weights")
            t_b["verified_buckets"][method] = sum(n for _, n in checks)
        t_b["seconds"] = t_b["per_method"][bcast]
    torch.cuda.synchronize()
    return tr, br, t_b


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


def config4_step_flops_executed(window: int, n_masked: int) -> float:
    """The MFMA FLOP the HIP path executes per config-4 step: the ID-resample attention streams segment 1 (N keys)
    and only the n_masked masked video rows of segment 2 (the null keys are summed in closed form by
    vp_null_key_mass: 88 short dot products per query, not counted); everything else as config4_step_flops."""
    attn = 4 * NTOK * (NTOK + n_masked) * D
    kv = 4 * NTOK * D * D if window > 0 else 0
    blk = 24 * NTOK * D * D + attn + kv
    tr = B * (L * blk + 2 * NV * 128 * D + 2 * T * 4096 * D + 2 * NV * D * 64)
    br_blk = 24 * NTOK * D * D + 4 * NTOK * NTOK * D
    br = B * (LB * br_blk + 2 * NV * 132 * D + 2 * T * 4096 * D + LB * 2 * NTOK * D * D)
    return float(tr + br)


def _window_inputs(g, device, first: bool):
    lat = torch.randn(1, F, 16, HL, WL, generator=g)
    vid = torch.randn(1, F, 16, HL, WL, generator=g)
    mask = torch.zeros(1, 1, F, HL, WL)
    mask[:, :, 1:, HL // 4:HL // 4 + HL // 2, WL // 4:WL // 4 + WL // 2] = 1.0
    masked = vid * (1 - mask.permute(0, 2, 1, 3, 4))
    win = dict(latents=lat, noise=lat.clone(), video_latents=vid, mask=torch.cat([mask] * 2),
               masked_video_latents=torch.cat([masked] * 2))
    if first:
        img = torch.zeros(1, F, 16, HL, WL)
        img[:, 0] = torch.randn(1, 16, HL, WL, generator=g) * 0.7
        win["image_latents"] = img
    return {k: v.to(device, torch.bfloat16) for k, v in win.items()}


def run_config4(args, world: int, rank: int, local: int) -> None:
    """BASELINE config 4: the VideoPainterID any-length chain — 196 frames as 4 windows of 49 at stride 49,
    ID-resample processor, prev_clip_weight 0.5, each window conditioned on the previous one's last latent and
    last-step hidden states — with --steps denoising steps per window (the reference runs 50; the per-step work is
    the same).  The chain is serial, so N GPUs run it as a window-stage pipeline
    (distributed.WindowStages: window w on stage w % N, point-to-point hand-off of latents + 42 hidden states + mask
    + generator state) over N clips, so every stage is busy once the pipeline is full.  value = denoising steps/s
    over all clips' windows; 1 GPU = the serial chain of one clip."""
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    from videopainter_amd import kernels as K
    from videopainter_amd.config import COGVIDEOX_5B_I2V
    from videopainter_amd.pipeline import CogVideoXI2VDualInpaintAnyLHarness, run_any_length_pipelined
    from videopainter_amd.scheduler import CogVideoXDPMScheduler
    stages = None
    if world > 1:
        import torch.distributed as dist
        from videopainter_amd.distributed import WindowStages, init as dist_init
        dist_init(os.environ.get("VP_BENCH_DIST_BACKEND", "nccl"), device)
        stages = WindowStages()
    t_setup = time.time()
    cfg = dict(COGVIDEOX_5B_I2V, sample_height=HL, sample_width=WL)
    with device_scope(device):
        tr = CogVideoXTransformer3DModel(**dict(cfg, id_pool_resample_learnable=True))
        br = CogvideoXBranchModel(**dict(cfg, num_layers=LB))
    tr.init_synthetic_weights_(1234)  # every rank fills the same counter-generated weights (no broadcast needed)
    br.init_synthetic_weights_(1235)
    mk_sched = lambda: CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction",  # noqa: E731
                                             rescale_betas_zero_snr=True, clip_sample=False, set_alpha_to_one=True,
                                             timestep_spacing="trailing")
    harness = CogVideoXI2VDualInpaintAnyLHarness(tr, br, mk_sched())
    n_windows = 4
    n_clips = max(1, world)
    g = torch.Generator().manual_seed(42)
    clips = []
    for j in range(n_clips):
        clips.append([_window_inputs(g, device, w == 0) for w in range(n_windows)])
    pe = torch.randn(1, T, 4096, generator=g).to(device, torch.bfloat16)
    npe = torch.randn(1, T, 4096, generator=g).to(device, torch.bfloat16)
    kw = dict(num_frames=49, stride=49, guidance_scale=6.0, use_dynamic_cfg=True, replace_gt=True, mask_add=True,
              prev_clip_weight=0.5, id_pool_resample_learnable=True)

    def run(n_steps, wins_per_clip=None):
        if stages is None:
            return [harness(clips[0][:wins_per_clip or n_windows], pe, npe, num_inference_steps=n_steps,
                            generator=torch.Generator().manual_seed(0), **kw)]
        return run_any_length_pipelined(
            harness, stages, [{"windows": c[:wins_per_clip or n_windows],
                               "generator": torch.Generator().manual_seed(j)} for j, c in enumerate(clips)],
            pe, npe, num_inference_steps=n_steps, **kw)
    log(f"[bench] config 4 setup {time.time() - t_setup:.1f}s; rank {rank}/{world}")
    with torch.no_grad():
        run(max(1, args.warmup), 2)  # warm-up: both window kinds (resample w0, prev-clip w>0)
        torch.cuda.synchronize()
        if stages is not None:
            from videopainter_amd.distributed import barrier
            barrier(device)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = run(args.steps)
        torch.cuda.synchronize()
        if stages is not None:
            barrier(device)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if stages is not None:
            from videopainter_amd.distributed import max_over_ranks
            elapsed = max_over_ranks(elapsed, device)
        with K.timed_launches("attention", "gemm") as tl:  # instrumented pass (not timed): per-kernel breakdown
            run(1, 1)
            torch.cuda.synchronize()
    n_steps = n_clips * n_windows * args.steps
    steps_per_s = n_steps / elapsed
    fl = sum(config4_step_flops(w) for w in range(n_windows)) * args.steps * n_clips
    # masked video rows of each window's resample mask (the rows segment 2 streams), counted as the transformer does
    n_masked = [int(K.patch_mask(clips[0][w]["mask"][:1].permute(0, 2, 1, 3, 4).contiguous(), 2).sum())
                for w in range(n_windows)]
    fl_exec = sum(config4_step_flops_executed(w, n_masked[w - 1 if w > 0 else 0])
                  for w in range(n_windows)) * args.steps * n_clips
    attn_ms = tl.mean_ms("attention")
    if rank == 0:
        line = {
            "metric": METRIC, "value": steps_per_s, "unit": "steps/s", "n_gpus": world, "steps": n_steps,
            "warmup": args.warmup, "ms_per_step": elapsed / n_steps * 1e3 * world, "higher_is_better": True,
            "scaling": "strong" if args.mode == "ulysses" else "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic latents/prompt embeds of the 4 x 49f 480x720 windows; random-init CogVideoX-5b-I2V "
                    "(ID-resample processor) + 2-layer branch weights (no checkpoints offline)",
            "config": {"workload": f"BASELINE config 4: any-length 196 frames = 4 windows x 49f 480x720 at stride 49, "
                                   f"ID-resample + prev_clip_weight 0.5, {args.steps} denoising steps per window, "
                                   f"{n_clips} clip(s) (value = denoising steps/s over all windows)",
                       "windows": n_windows, "clips": n_clips, "tokens": NTOK, "keys_per_attention": 2 * NTOK,
                       "layers": L, "branch_layers": LB,
                       "parallelism": "serial window chain on 1 GPU" if world == 1 else
                                      f"{world}-stage window pipeline (P2P hand-off), {n_clips} clips"},
            "step_flop_mean": fl / n_steps,
            "step_mfma_frac": fl / elapsed / world / (PEAK_BF16_TFLOPS * 1e12),
            "flop_basis": "the reference's work: attention over all 2N keys (K and its masked copy); the HIP path sums "
                          "the masked copy's null keys in closed form and streams only the masked rows, so it executes "
                          "fewer MFMA FLOPs than counted here",
            "step_flop_executed_mean": fl_exec / n_steps,
            "step_mfma_frac_executed": fl_exec / elapsed / world / (PEAK_BF16_TFLOPS * 1e12),
            "executed_basis": f"the MFMA FLOP the HIP path runs: attention over N + the masked rows of segment 2 "
                              f"({n_masked[0]} of {NV} video rows per window), null keys in closed form not counted",
            "attention_ms_per_launch": attn_ms, "output_latents": list(out[0].shape),
        }
        print(json.dumps(line), flush=True)
    if stages is not None:
        dist.destroy_process_group()


def clip_of(rank: int, mode: str) -> int:
    """The clip a rank works on: its own (dp) or its CFG pair's (cfgpair: ranks 2p, 2p + 1 share clip p)."""
    return rank // 2 if mode == "cfgpair" else (0 if mode == "ulysses" else rank)


def timed_steps(one, sync_all, warmup: int, steps: int) -> float:
    """The timing contract: `warmup` untimed steps, then exactly `steps` steps bracketed by a barrier +
    synchronize on both sides (sync_all); returns this rank's elapsed seconds."""
    for i in range(warmup):
        one(i)
    sync_all()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        one(i)
    sync_all()
    return time.perf_counter() - t0


def job_value(elapsed_max: float, steps: int, world: int, mode: str):
    """Whole-job denoising steps/s from the slowest rank's time: every clip advances `steps` steps."""
    clips = world // 2 if mode == "cfgpair" else (1 if mode == "ulysses" else world)
    return clips, clips * steps / elapsed_max


def fp8_proj_flops(fp8_out: bool) -> float:
    """Config 5's fp8 projection FLOP per step besides the FeedForward: the fused QKV (6 N D^2 per block and CFG
    half) and, unless kept in bf16, the attention's output projection (2 N D^2)."""
    return (L + LB) * B * (6 + (2 if fp8_out else 0)) * NTOK * D * D


def kernel_classes(tl, n_steps: int, fp8: bool, share: float = 1.0, fp8_out: bool = True):
    """Per-kernel-class roofline from the instrumented pass: algorithmic FLOP per step of the class / its summed
    launch time per step.  attention: 4 B H N^2 64 per launch (one call = main grid + tail split + merge); gemm: every
    projection GEMM of the step (step FLOP - attention FLOP), bf16 (and the MX-FP8 FeedForward GEMMs for config 5).
    share: the fraction of the step's work one rank does (1/P under the head-parallel split)."""
    torch.cuda.synchronize()
    attn_name = "attention_fp8" if fp8 else "attention"
    attn_ev = tl.events.get(attn_name, [])
    attn_ms_total = sum(a.elapsed_time(b) for a, b in attn_ev)
    gemm_ev = tl.events.get("gemm", []) + tl.events.get("gemm_mx", [])
    gemm_ms_total = sum(a.elapsed_time(b) for a, b in gemm_ev)
    attn_fl_step = (L + LB) * attn_flops_per_launch() * share
    total_fl, ffn_fl = step_flops(split=True)
    gemm_fl_step = total_fl * share - attn_fl_step
    attn_ms = attn_ms_total / n_steps
    gemm_ms = gemm_ms_total / n_steps
    out = {}
    peak_a = PEAK_FP8_TFLOPS if fp8 else PEAK_BF16_TFLOPS
    a_tf = attn_fl_step / (attn_ms * 1e-3) / 1e12
    traffic, src = profiled_traffic("attention_fp8" if fp8 else "attention")
    out["attention"] = {"kernel": "vp_attention_fwd_%s" % ("fp8" if fp8 else "bf16"), "bound": "mfma",
                        "achieved": a_tf, "peak": peak_a, "unit": "TFLOP/s", "frac": a_tf / peak_a,
                        "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": src,
                        "per_launch_ms": attn_ms_total / max(1, len(attn_ev)), "launches_per_step": len(attn_ev) / n_steps,
                        "ms_per_step": attn_ms, "algorithmic_flop_per_launch": attn_flops_per_launch() * share}
    if fp8:  # the MX-FP8 GEMMs (5 PF peak), the rest bf16: the peak of the class is the FLOP-weighted mix
        f8 = ffn_fl + fp8_proj_flops(fp8_out)
        t_ideal = (gemm_fl_step - f8) / (PEAK_BF16_TFLOPS * 1e12) + f8 / (PEAK_FP8_TFLOPS * 1e12)
        peak_g = gemm_fl_step / t_ideal / 1e12
    else:
        peak_g = PEAK_BF16_TFLOPS
    g_tf = gemm_fl_step / (gemm_ms * 1e-3) / 1e12
    traffic, src = profiled_traffic("gemm") if not fp8 else (None, None)
    out["gemm"] = {"kernel": "vp_gemm_bf16" + (" + vp_gemm_mx_fp8" if fp8 else ""), "bound": "mfma",
                   "achieved": g_tf, "peak": peak_g, "unit": "TFLOP/s", "frac": g_tf / peak_g,
                   "traffic": traffic, "traffic_unit": "bytes/launch (QKV-shape launch)", "traffic_source": src,
                   "launches_per_step": len(gemm_ev) / n_steps, "ms_per_step": gemm_ms,
                   "algorithmic_flop_per_step": gemm_fl_step}
    dominant = max(out, key=lambda k: out[k]["ms_per_step"])
    return out, dominant


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fp8-out-bf16", action="store_true",
                    help="config 5 A/B: keep the attention output projection in bf16 (the round-6 form before)")
    ap.add_argument("--cpu-baseline-only", action="store_true")
    ap.add_argument("--cpu-full-step", action="store_true",
                    help="with --cpu-baseline-only: time one whole config-2 step on the CPU (bf16, ~7 min)")
    ap.add_argument("--config", type=int, default=2, choices=(2, 4, 5),
                    help="BASELINE config: 2 = 49f 480x720 bf16 (headline), 4 = the any-length ID-resample chain "
                         "(4 windows, --steps denoising steps each), 5 = 49f 720x1280 with attention + FeedForward in fp8")
    ap.add_argument("--mode", default="dp", choices=("dp", "cfgpair", "ulysses", "stages"),
                    help="multi-GPU layout of configs 2/5: dp = one clip per rank, cfgpair = one clip per rank pair "
                         "(CFG halves, one all-gather per step), ulysses = ONE clip split head-parallel over all "
                         "ranks (two all-to-alls per block; strong scaling); stages = the any-length window chain "
                         "as a window-stage pipeline (point-to-point hand-offs; = --config 4)")
    ap.add_argument("--bcast", default="scatter_allgather", choices=("scatter_allgather", "broadcast"),
                    help="weight replication for N > 1 (distributed.broadcast_module)")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="at N=1: initialise torch.distributed on RCCL anyway and run the weight replication + replica "
                         "check through it (identities at world size 1; the untimed setup, not the steps)")
    ap.add_argument("--lora-rank", type=int, default=0,
                    help="> 0: a synthetic VideoPainterID-style adapter of this rank on every transformer block's "
                         "to_q / to_k / to_v / to_out.0, loaded as the reference loads it (unfused, PEFT's forward)")
    ap.add_argument("--qk-gamma", type=float, default=0.0,
                    help="> 0: every norm_q / norm_k gain drawn U(0.1, G) per channel (trained-like qk-LayerNorm "
                         "weights; past the static score bound the attention runs the anchored kernel)")
    args = ap.parse_args()
    set_config(args.config)

    if args.cpu_baseline_only:
        res = cpu_full_step() if args.cpu_full_step else cpu_baseline()
        print(json.dumps({"cpu_full_step" if args.cpu_full_step else "cpu_baseline": res}))
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VP_BENCH_DIST_BACKEND=gloo: a functional rehearsal of the multi-rank path with several ranks on the GPUs there
    # are (ranks share a device; the timing then says nothing about scaling); the driver's runs use RCCL, one rank
    # per GPU
    backend = os.environ.get("VP_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if args.config == 4 or args.mode == "stages":
        set_config(2)  # the any-length chain runs 49f 480x720 windows
        run_config4(args, world, rank, local)
        return
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    pair = None
    if world > 1 or args.rccl_world1:
        if world == 1:  # a one-rank job started without a launcher: its own env:// rendezvous on the loopback
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(port)), ("RANK", "0"),
                         ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
                os.environ.setdefault(k, v)
        import torch.distributed as dist
        from videopainter_amd.distributed import init as dist_init
        dist_init(backend, device)
    if args.mode == "cfgpair":
        if world % 2:
            raise SystemExit("--mode cfgpair needs an even number of ranks")
        from videopainter_amd.distributed import CFGPair
        pair = CFGPair()

    from videopainter_amd import kernels as K
    from videopainter_amd.pipeline import CogVideoXI2VDualInpaintAnyLHarness
    from videopainter_amd.scheduler import CogVideoXDPMScheduler

    t_setup = time.time()
    tr, br, t_bcast = build_models(device, 1234, rank, world, args.bcast, args.rccl_world1)
    if args.lora_rank > 0:
        from videopainter_amd.lora import attach_lora_
        gl = torch.Generator(device=device).manual_seed(91)
        lsd = {}
        for i, blk in enumerate(tr.transformer_blocks):
            for t, lin in (("to_q", blk.attn1.to_q), ("to_k", blk.attn1.to_k), ("to_v", blk.attn1.to_v),
                           ("to_out.0", blk.attn1.to_out[0])):
                o_f, i_f = lin.weight.shape
                lsd[f"transformer_blocks.{i}.attn1.{t}.lora_A.weight"] = (
                    torch.randn(args.lora_rank, i_f, device=device, generator=gl) * i_f ** -0.5).to(torch.bfloat16)
                lsd[f"transformer_blocks.{i}.attn1.{t}.lora_B.weight"] = (
                    torch.randn(o_f, args.lora_rank, device=device, generator=gl) * 0.01).to(torch.bfloat16)
        attach_lora_(tr, lsd, 1.0, "vpid")
        del lsd
        log(f"[bench] rank-{args.lora_rank} LoRA on {4 * len(tr.transformer_blocks)} projections, unfused")
    bounded_layers = None
    if args.qk_gamma > 0:
        from videopainter_amd.attention_processor import bounded_scores
        gq = torch.Generator().manual_seed(77)
        with torch.no_grad():
            for m in (tr, br):
                for blk in m.transformer_blocks:
                    for ln in (blk.attn1.norm_q, blk.attn1.norm_k):
                        ln.weight.copy_((0.1 + (args.qk_gamma - 0.1) * torch.rand(64, generator=gq)).to(ln.weight))
        bounded_layers = sum(bounded_scores(blk.attn1) for m in (tr, br) for blk in m.transformer_blocks)
        log(f"[bench] qk-norm gains U(0.1, {args.qk_gamma}): {bounded_layers} of "
            f"{len(tr.transformer_blocks) + len(br.transformer_blocks)} layers within the static score bound")
    sch = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                                clip_sample=False, set_alpha_to_one=True, timestep_spacing="trailing")
    sch.set_timesteps(50)
    timesteps = sch.timesteps.cpu()
    if args.mode == "ulysses":
        from videopainter_amd import ulysses as U
        views = U.UlyssesModels(tr, br, U.DistComm() if world > 1 else U.ThreadComm(1), rank=rank)
        harness = CogVideoXI2VDualInpaintAnyLHarness(views.transformer, views.branch, sch)
    else:
        harness = CogVideoXI2VDualInpaintAnyLHarness(tr, br, sch, cfg_pair=pair)
    clip = clip_of(rank, args.mode)
    st, pe = make_state(harness, device, 42 + clip)
    rope = harness.rope_for(F, HL, WL)
    gen = torch.Generator().manual_seed(42 + clip)
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
            tr.enable_fp8(out=not args.fp8_out_bf16)
            br.enable_fp8(out=not args.fp8_out_bf16)
            out8 = fwd()
            fp8_drift = float((out8 - ref16).norm() / ref16.norm())
            del ref16, out8, lmi
        log(f"[bench] config 5: fp8 QKV+attention+{'' if args.fp8_out_bf16 else 'out+'}FFN noise_pred vs bf16 "
            f"rel-L2 {fp8_drift:.3e}")
    log(f"[bench] setup {time.time() - t_setup:.1f}s; rank {rank}/{world}"
        + (f"; weight replication {t_bcast}" if t_bcast is not None else ""))

    def one(i):
        k = i % len(timesteps)
        if k == 0:
            st.old_pred = None
        harness.step(st, k, timesteps, pe, rope, guidance_scale=6.0, use_dynamic_cfg=True, replace_gt=True,
                     mask_add=True, generator=gen)

    def sync_all():
        torch.cuda.synchronize()
        if dist is not None:
            from videopainter_amd.distributed import barrier
            barrier(device)
        torch.cuda.synchronize()

    with torch.no_grad():
        elapsed = timed_steps(one, sync_all, args.warmup, args.steps)  # uninstrumented
        # separate instrumented pass (HIP events around every GEMM / attention launch on its stream), NOT timed
        n_prof = min(2, args.steps)
        with K.timed_launches("attention", "attention_fp8", "gemm", "gemm_mx") as tl:
            for i in range(args.warmup + args.steps, args.warmup + args.steps + n_prof):
                one(i)
            torch.cuda.synchronize()
    if dist is not None:
        from videopainter_amd.distributed import max_over_ranks
        elapsed = max_over_ranks(elapsed, device)
    clips, steps_per_s = job_value(elapsed, args.steps, world, args.mode)
    ms_per_step = elapsed / args.steps * 1e3
    classes, dominant = kernel_classes(tl, n_prof, args.config == 5, 1.0 / world if args.mode == "ulysses" else 1.0,
                                       fp8_out=not args.fp8_out_bf16)
    total_fl, ffn_fl = step_flops(split=True)
    if args.config == 5:  # time the step would take at the dense peaks of the dtypes its MFMAs use
        f8_fl = ffn_fl + (L + LB) * attn_flops_per_launch() + fp8_proj_flops(not args.fp8_out_bf16)
        t_ideal = (total_fl - f8_fl) / (PEAK_BF16_TFLOPS * 1e12) + f8_fl / (PEAK_FP8_TFLOPS * 1e12)
    else:
        t_ideal = total_fl / (PEAK_BF16_TFLOPS * 1e12)
    # a CFG pair computes one step on 2 GPUs: per-GPU MFMA fraction of the step
    step_frac = t_ideal * steps_per_s / world
    if not math.isfinite(steps_per_s):
        raise RuntimeError("non-finite timing")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == 2:
        del st
        cpu = cpu_baseline()
    if rank == 0:
        rf = dict(classes[dominant])
        rf["kernel"] = f"{rf['kernel']} ({dominant}: dominant by time in this run)"
        par = (f"cfgpair x{clips} (CFG halves on rank pairs, one noise-prediction all-gather per step)" if pair
               else f"ulysses{world} (one clip, head-parallel: 2 all-to-alls per block)" if args.mode == "ulysses"
               else f"dp{world} (independent clips, weights replicated over RCCL: {args.bcast})")
        out = {
            "metric": METRIC, "value": steps_per_s, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if args.mode == "ulysses" else "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.config == 2 else ("bf16 + fp8 (e4m3, block-scaled MFMA) QKV, attention, "
                                                      + ("" if args.fp8_out_bf16 else "output projection, ")
                                                      + "FeedForward"),
            "data": f"synthetic latents/prompt embeds of the 49f {HL * 8}x{WL * 8} shape; random-init "
                    "CogVideoX-5b-I2V (42 layers) + 2-layer branch weights (no checkpoints offline)",
            "config": {"workload": (f"BASELINE config {args.config}: CogVideoX-5b-I2V + 2-layer branch, 49f "
                                    f"{HL * 8}x{WL * 8} (latent 13x{HL}x{WL}), CFG batch 2, {T}+{NV}={NTOK} tokens, "
                                    "1 denoising step = branch + transformer + CFG/DPM/replace-gt"
                                    + ((", QKV projection + attention + "
                                        + ("" if args.fp8_out_bf16 else "output projection + ")
                                        + "FeedForward in fp8") if args.config == 5 else "")),
                       "clips": clips, "cfg_batch": B, "tokens": NTOK, "layers": L, "branch_layers": LB,
                       "parallelism": par,
                       **({"qk_norm_gain_max": args.qk_gamma, "layers_within_static_score_bound": bounded_layers}
                          if args.qk_gamma > 0 else {}),
                       **({"lora_rank": args.lora_rank, "lora": "unfused (PEFT's forward), not in step_flop"}
                          if args.lora_rank > 0 else {})},
            "roofline": rf,
            "roofline_kernels": classes,
            "step_mfma_frac": step_frac,
            "fp8_rel_l2_vs_bf16": fp8_drift,
            "step_flop": step_flops(),
            "gemm_ms_per_step": classes["gemm"]["ms_per_step"],
            "attention_ms_per_step": classes["attention"]["ms_per_step"],
            "weight_broadcast_s": t_bcast["seconds"] if t_bcast else None,
            "weight_replication": t_bcast,
            "timing": "timed steps uninstrumented; per-kernel numbers from a separate instrumented pass of "
                      f"{n_prof} steps (HIP events on the launch stream)",
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
