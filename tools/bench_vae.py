"""CogVideoX-5b VAE (random-init weights of the real architecture) on one MI355X: decode of the config-2 latent
(13 frames 60x90 -> 49 frames 480x720, the pipeline's decode_latents, anyl.py:479-483) and encode of a 49-frame
480x720 video (prepare_latents, anyl.py:423-430), untiled (frame-batched) and with the any-length inference's
tiling + slicing (infer/inpaint.py:413-415).

    python tools/bench_vae.py [--iters 2] [--tiled] [--frames 49]

Prints one JSON line: seconds per call, the conv kernel's algorithmic TFLOP/s (2 * output pixels * Cout * taps *
logical Cin, summed over every conv of the call) over the HIP-event time of its launches, and the share of the
call spent in the conv kernel.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from videopainter_amd.vae import AutoencoderKLCogVideoX  # noqa: E402


def run(vae, fn, iters):
    fn()
    torch.cuda.synchronize()
    vae.flop_counter = []
    with K.timed_launches("conv3d") as tl:
        fn()
        torch.cuda.synchronize()
    flops = sum(vae.flop_counter)
    vae.flop_counter = None
    conv_ms = tl.mean_ms("conv3d") * tl.count("conv3d")
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / iters
    return dict(seconds=sec, conv_launches=tl.count("conv3d"), conv_tflop=flops / 1e12,
                conv_ms=conv_ms, conv_tflops=flops / (conv_ms / 1e3) / 1e12, conv_share=conv_ms / 1e3 / sec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--frames", type=int, default=49)
    ap.add_argument("--tiled", action="store_true")
    args = ap.parse_args()
    torch.manual_seed(0)
    vae = AutoencoderKLCogVideoX.from_config(dict(scaling_factor=0.7), device="cuda").init_synthetic_weights_(2002)
    if args.tiled:
        vae.enable_tiling()
        vae.enable_slicing()
    lf = (args.frames - 1) // 4 + 1
    z = torch.randn(1, 16, lf, 60, 90, device="cuda").bfloat16()
    x = (torch.rand(1, 3, args.frames, 480, 720, device="cuda") * 2 - 1).bfloat16()
    out = {"config": f"CogVideoX-5b VAE, {args.frames}f 480x720 ({lf} latent frames), bf16, "
                     f"{'tiled+sliced' if args.tiled else 'frame-batched, untiled'}", "peak_tflops": 2500.0}
    with torch.no_grad():
        out["decode"] = run(vae, lambda: vae.decode(z), args.iters)
        out["encode"] = run(vae, lambda: vae.encode(x), args.iters)
    for k in ("decode", "encode"):
        out[k]["conv_mfma_frac"] = out[k]["conv_tflops"] / out["peak_tflops"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
