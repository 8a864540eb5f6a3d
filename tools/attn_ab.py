"""Interleaved A/B of bf16 attention kernel variants at config 2 (B 2, H 48, N 17 776), one process, random data;
median and min per variant over the rounds (cdna_hip_programming.md §5.4 rule 24).

    python tools/attn_ab.py --modes p2,s16 [--rounds 5] [--iters 20] [--unbounded p2a,a16]
Modes are VP_ATTN_BOUNDED_MODE values (bounded-score launches); --unbounded adds VP_ATTN_UNBOUNDED_MODE values run
without the bounded flag.
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
    ap.add_argument("--modes", default="p2,s16")
    ap.add_argument("--unbounded", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=17776)
    a = ap.parse_args()
    B, N, H = 2, a.n, 48
    torch.manual_seed(0)
    qkv = torch.randn(B, N, 3 * H * 64, device="cuda").bfloat16()
    q, k, v = qkv[..., :H * 64], qkv[..., H * 64:2 * H * 64], qkv[..., 2 * H * 64:]
    o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * H * N * N * 64
    arms = [("b", m) for m in a.modes.split(",") if m] + [("u", m) for m in a.unbounded.split(",") if m]
    res = {f"{kind}:{m}": [] for kind, m in arms}
    for r in range(a.rounds):
        for kind, m in arms:
            if kind == "b":
                K.set_knob("VP_ATTN_BOUNDED_MODE", m)
                K.set_knob("VP_ATTN_UNBOUNDED_MODE", None)
            else:
                K.set_knob("VP_ATTN_UNBOUNDED_MODE", m)
                K.set_knob("VP_ATTN_BOUNDED_MODE", None)
            t = timeit(lambda: K.attention(q, k, v, o, H, bounded_scores=kind == "b"), a.iters)
            res[f"{kind}:{m}"].append(t * 1e3)
            print(f"round {r} {kind}:{m}: {t * 1e3:.3f} ms {fl / t / 1e12:.0f} TF/s", flush=True)
    summ = {k: {"median_ms": statistics.median(v), "min_ms": min(v),
                "median_tflops": fl / (statistics.median(v) / 1e3) / 1e12} for k, v in res.items()}
    for k, s in summ.items():
        print(f"{k}: median {s['median_ms']:.3f} ms ({s['median_tflops']:.0f} TF/s), min {s['min_ms']:.3f} ms")
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
