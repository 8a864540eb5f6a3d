"""Per-tile fixed cost of vp_gemm_bf16: time vs K at fixed M, N (and whole-round M) on random data.

    python tools/gemm_kscan.py [--iters 10]

A linear fit t(K) = rounds * (m * K / 3072 + e) separates the main-loop time per 3072 of K (m) from the per-tile
fixed cost (e: pipeline fill, epilogue, write burst), rounds = ceil(tiles / 256).
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from videopainter_amd import _native as N  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--epi", default="bias", choices=("bias", "gelu"))
    args = ap.parse_args()
    dev = "cuda"
    epi = N.EPI_BIAS if args.epi == "bias" else N.EPI_BIAS_GELU
    res = {}
    for Mrows, Ncols in ((35552, 3072), (32768, 3072), (35552, 12288)):
        for Kd in (768, 1536, 3072, 6144, 12288):
            a = (torch.rand(Mrows, Kd, device=dev) * 2 - 1).bfloat16()
            w = ((torch.rand(Ncols, Kd, device=dev) * 2 - 1) / math.sqrt(Kd)).bfloat16()
            b = torch.zeros(Ncols, device=dev).bfloat16()
            out = torch.empty(Mrows, Ncols, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: K.gemm(a, [w], [b], out, epilogue=epi), args.iters)
            tiles = math.ceil(Mrows / 256) * math.ceil(Ncols / 256)
            rounds = math.ceil(tiles / 256)
            key = f"M{Mrows}_N{Ncols}_K{Kd}"
            res[key] = dict(ms=t * 1e3, tflops=2 * Mrows * Ncols * Kd / t / 1e12, tiles=tiles, rounds=rounds,
                            us_per_round=t * 1e6 / rounds)
            print(key, res[key], flush=True)
            del a, w, b, out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
