"""Training-step throughput of the VideoPainter training path on one MI355X.

    python tools/bench_train.py [--steps K] [--warmup W] [--height 60 --width 90] [--optimizer]

One step = the reference's training iteration (train/train_cogvideox_inpainting_i2v_video.py:1856-1892 with the
launch script train/VideoPainter.sh: 49 frames 480x720 -> latent 13x60x90, batch 1, bf16, branch_layer_num 2,
--mask_add, --gradient_checkpointing): 2-layer branch forward (trainable) -> 42-layer 5b-I2V transformer forward
(frozen) with the samples injected under the mask -> backward of a synthetic loss gradient into every branch
parameter.  --optimizer adds torch's AdamW (foreach) on the branch parameters (PyTorch's kernels, not ours; off by
default).  Random-init weights, synthetic latents.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

T, F, D, L, LB = 226, 13, 3072, 42, 2


def flops(ntok: int, nv: int) -> dict:
    """Algorithmic FLOP of one training step at B=1: forward of both models, input-gradient (dgrad) backward of
    every block and of the injection path, weight-gradient backward of the branch.  Recompute (checkpointing) and
    the attention backward's score recompute are overhead, not counted."""
    gemm_f = 24 * ntok * D * D
    attn_f = 4 * ntok * ntok * D
    fwd = (L + LB) * (gemm_f + attn_f) + LB * 2 * ntok * D * D
    dgrad = (L + LB) * (gemm_f + 2 * attn_f) + LB * 2 * ntok * D * D
    wgrad = LB * (gemm_f + 2 * ntok * D * D)
    return dict(forward=float(fwd), backward=float(dgrad + wgrad), total=float(fwd + dgrad + wgrad))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--height", type=int, default=60)
    ap.add_argument("--width", type=int, default=90)
    ap.add_argument("--optimizer", action="store_true")
    ap.add_argument("--classes", action="store_true", help="per-class HIP-event timing pass afterwards")
    args = ap.parse_args()
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    from videopainter_amd import kernels as K
    from videopainter_amd.config import COGVIDEOX_5B_I2V
    from videopainter_amd.embeddings import prepare_rotary_positional_embeddings

    dev = "cuda"
    HL, WL = args.height, args.width
    cfg = dict(COGVIDEOX_5B_I2V, sample_height=HL, sample_width=WL)
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**cfg)
        br = CogvideoXBranchModel(**dict(cfg, num_layers=LB))
    tr.init_synthetic_weights_(1234)
    br.init_synthetic_weights_(1235)
    br.requires_grad_(True)
    params = [p for p in br.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-5, betas=(0.9, 0.95), foreach=True) if args.optimizer else None

    g = torch.Generator().manual_seed(7)
    lat = torch.randn(1, F, 16, HL, WL, generator=g).to(dev, torch.bfloat16)
    img = torch.zeros(1, F, 16, HL, WL)
    img[:, 0] = torch.randn(1, 16, HL, WL, generator=g)
    img = img.to(dev, torch.bfloat16)
    mask = torch.zeros(1, F, 1, HL, WL)
    mask[:, 1:, :, HL // 4:HL // 4 + HL // 2, WL // 4:WL // 4 + WL // 2] = 1.0
    mask = mask.to(dev, torch.bfloat16)
    cond = torch.cat([lat * (1 - mask), mask], 2)
    hidden = torch.cat([lat, img], 2)
    enc = torch.randn(1, T, 4096, generator=g).to(dev, torch.bfloat16)
    ts = torch.tensor([500], device=dev)
    rope = tuple(t.to(dev) for t in prepare_rotary_positional_embeddings(HL * 8, WL * 8, F, 64))
    dout = torch.randn(1, F, 16, HL, WL, generator=g).to(dev, torch.bfloat16)
    nv = F * (HL // 2) * (WL // 2)
    ntok = T + nv

    def step():
        samples = br(hidden_states=lat, encoder_hidden_states=enc, branch_cond=cond, timestep=ts,
                     image_rotary_emb=rope, return_dict=False)[0]
        out = tr(hidden_states=hidden, encoder_hidden_states=enc, timestep=ts, image_rotary_emb=rope,
                 branch_block_samples=samples, branch_block_masks=mask, return_dict=False)[0]
        out.backward(dout)
        if opt is not None:
            opt.step()
        for p in params:
            p.grad = None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        torch.cuda.synchronize()
        print(f"step {i}: {time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)
    el = (time.perf_counter() - t0) / args.steps
    fl = flops(ntok, nv)
    res = dict(metric="training steps/sec (VideoPainter branch, 5b-I2V frozen, 49f 480x720, B=1)",
               value=1.0 / el, unit="steps/s", ms_per_step=el * 1e3, steps=args.steps, warmup=args.warmup,
               optimizer="torch AdamW foreach" if opt is not None else None,
               tflops_per_s=fl["total"] / el / 1e12, flop_per_step=fl, ntok=ntok,
               peak_mem_gib=torch.cuda.max_memory_allocated() / 2 ** 30)
    if args.classes:
        with K.timed_launches("gemm", "attention", "attention_bwd") as tl:
            step()
        torch.cuda.synchronize()
        res["classes_ms"] = {n: tl.mean_ms(n) * tl.count(n) for n in ("gemm", "attention", "attention_bwd")}
        res["counts"] = {n: tl.count(n) for n in ("gemm", "attention", "attention_bwd")}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
