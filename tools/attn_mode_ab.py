"""Interleaved A/B of the bf16 attention kernel's bounded-score forms at config 2 (B 2, H 48, N 17776), one process.

    python tools/attn_mode_ab.py [--modes bounded,dot] [--rounds 3] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="bounded,dot")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    B, N, H = 2, 17776, 48
    qkv = torch.randn(B, N, 3 * H * 64, device="cuda").bfloat16()
    q, k, v = qkv[..., :H * 64], qkv[..., H * 64:2 * H * 64], qkv[..., 2 * H * 64:]
    o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * H * N * N * 64
    for r in range(a.rounds):
        for m in a.modes.split(","):
            K.set_knob("VP_ATTN_BOUNDED_MODE", m)
            t = timeit(lambda: K.attention(q, k, v, o, H, bounded_scores=True), a.iters)
            print(f"round {r} {m}: {t * 1e3:.3f} ms {fl / t / 1e12:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
