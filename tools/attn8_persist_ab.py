"""Interleaved A/B of the persistent fp8 attention (default, ABI 20 workspace) against one workgroup per block
(VP_ATTN_PERSIST=0) at config 5's shape (B 2, H 48, N 47 026), random e4m3 operands.

    python tools/attn8_persist_ab.py [--rounds 5] [--iters 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--n", type=int, default=47026)
    a = ap.parse_args()
    B, H, N = 2, 48, a.n
    torch.manual_seed(0)
    q = torch.randn(B, N, H * 64, device="cuda")
    k = torch.randn(B, N, H * 64, device="cuda")
    v = torch.randn(B, N, H * 64, device="cuda").bfloat16()
    q8 = (q * 0.125 * K.LOG2E * 4).to(torch.float8_e4m3fn).view(torch.uint8)
    k8 = (k * 4).to(torch.float8_e4m3fn).view(torch.uint8)
    vp = K.v_pack_fp8(v, H)
    o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * H * N * N * 64
    res = {"persistent": [], "grid": []}
    for _ in range(a.rounds):
        for arm in res:
            K.set_knob("VP_ATTN_PERSIST", None if arm == "persistent" else "0")
            res[arm].append(timeit(lambda: K.attention_fp8(q8, k8, vp, o, H, 2, 2), a.iters) * 1e3)
    K.set_knob("VP_ATTN_PERSIST", None)
    summ = {arm: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                  "median_pflops": round(fl / (statistics.median(v) / 1e3) / 1e15, 4)} for arm, v in res.items()}
    print(json.dumps({"n": N, "results": summ}))


if __name__ == "__main__":
    main()
