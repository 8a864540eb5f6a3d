"""Interleaved A/B of the attention grid-tail handling (VP_ATTN_TAIL) at the step's own launch: bounded p2a, one
process, random data; median and min per setting over the rounds.

    python tools/attn_tail_ab.py --tails legacy,0:8,1:4,2:2 [--batch 2] [--rounds 5] [--iters 20]
    python tools/attn_tail_ab.py --tails p1,p0       # VP_ATTN_PERSIST 1 / 0 (default tail)
"legacy" = the two-launch remainder split (main grid, then the remainder's key-range pieces); "R:S" = one launch
whose last workgroups are S key-range pieces of each remainder block and of R whole rounds before them.
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
    ap.add_argument("--tails", default="legacy,0:8,1:4,2:2")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=17776)
    ap.add_argument("--unbounded", action="store_true")
    a = ap.parse_args()
    B, N, H = a.batch, a.n, 48
    torch.manual_seed(0)
    qkv = (torch.randn(B, N, 3 * H * 64, device="cuda") * 0.5).bfloat16()
    q, k, v = qkv[..., :H * 64], qkv[..., H * 64:2 * H * 64], qkv[..., 2 * H * 64:]
    o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * H * N * N * 64
    arms = [t for t in a.tails.split(",") if t]
    res = {t: [] for t in arms}
    for r in range(a.rounds):
        for t in arms:
            if t in ("p1", "p0"):
                K.set_knob("VP_ATTN_TAIL", None)
                K.set_knob("VP_ATTN_PERSIST", t[1])
            else:
                K.set_knob("VP_ATTN_PERSIST", None)
                K.set_knob("VP_ATTN_TAIL", None if t == "legacy" else t)
            ms = timeit(lambda: K.attention(q, k, v, o, H, bounded_scores=not a.unbounded), a.iters) * 1e3
            res[t].append(ms)
            print(f"round {r} {t}: {ms:.3f} ms {fl / ms / 1e9:.0f} TF/s", flush=True)
    K.set_knob("VP_ATTN_TAIL", None)
    K.set_knob("VP_ATTN_PERSIST", None)
    summ = {t: {"median_ms": statistics.median(v), "min_ms": min(v),
                "median_tflops": fl / (statistics.median(v) / 1e3) / 1e12} for t, v in res.items()}
    for t, s in summ.items():
        print(f"{t}: median {s['median_ms']:.3f} ms ({s['median_tflops']:.0f} TF/s), min {s['min_ms']:.3f} ms")
    print(json.dumps({"batch": B, "n": N, "unbounded": a.unbounded, "results": summ}))


if __name__ == "__main__":
    main()
