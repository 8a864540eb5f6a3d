"""Config-4 resample attention, the two ways of handling the null keys, interleaved A/B (median / min per arm):
  keys:  segment 2 = all N rows (masked rows first, then the null keys: row sums only, k2_full)
  null:  segment 2 = the masked rows only (k2_len) + the null keys' mass in closed form (null_key_mass -> l_extra;
         the mask's segments computed once, as the processor caches them)
plus the null_key_mass kernel alone.  Shapes: B 2 (CFG), H 48, N = 226 + 13x30x45, the bench's config-4 mask (frames
1-12, the centred half-height x half-width rectangle).

    python tools/null_ab.py [--rounds 5] [--iters 20]
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
from oracle.cogvideox_oracle import prepare_rotary_positional_embeddings  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, H, T = 2, 48, 226
    grid = (13, 30, 45)
    F_, Hh, Ww = grid
    N = T + F_ * Hh * Ww
    D = H * 64
    torch.manual_seed(0)
    qkv = torch.randn(B, N, 3 * D, device="cuda").bfloat16()
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    m = torch.zeros(B, N, dtype=torch.bool)
    vid = m[:, T:].view(B, F_, Hh, Ww)
    vid[:, 1:, Hh // 4:Hh // 4 + Hh // 2, Ww // 4:Ww // 4 + Ww // 2] = True
    m8 = m.to(torch.uint8).cuda()
    dst, cnt = K.partition_rows_index(m8)
    k2 = torch.randn(B, N, D, device="cuda").bfloat16()
    v2 = torch.randn(B, N, D, device="cuda").bfloat16()
    nm = int(cnt[0])
    v2[:, nm:] = 0
    cos, sin = prepare_rotary_positional_embeddings(Hh * 16, Ww * 16, F_, 64)
    axes = K.rope_axis_tables((cos.float().cuda(), sin.float().cuda()), grid)
    assert axes is not None
    beta = (torch.randn(64) * 0.5).bfloat16().cuda()
    o = torch.empty(B, N, D, device="cuda", dtype=torch.bfloat16)
    segs0 = K.mask_null_segments(m8, T, grid)  # (once per mask in the processor)

    def keys():
        K.attention(q, k, v, o, H, k2=k2, v2=v2, bounded_scores=True, k2_full=cnt)

    def null():
        lx = K.null_key_mass(q, H, T, grid, beta, axes, m8, segs0, 0.125)
        K.attention(q, k, v, o, H, k2=k2, v2=v2, bounded_scores=True, k2_len=cnt, l_extra=lx)

    def mass():
        K.null_key_mass(q, H, T, grid, beta, axes, m8, segs0, 0.125)

    arms = {"keys": keys, "null": null, "null_key_mass": mass}
    res = {n: [] for n in arms}
    print(f"N {N}, masked rows {nm} ({nm / N:.1%})", flush=True)
    for r in range(a.rounds):
        for n, fn in arms.items():
            t = timeit(fn, a.iters)
            res[n].append(t * 1e3)
            print(f"round {r} {n}: {t * 1e3:.3f} ms", flush=True)
    summ = {n: {"median_ms": statistics.median(v), "min_ms": min(v)} for n, v in res.items()}
    for n, s in summ.items():
        print(f"{n}: median {s['median_ms']:.3f} ms, min {s['min_ms']:.3f} ms")
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
