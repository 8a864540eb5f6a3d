"""Calibration only: hipBLASLt (torch.matmul) against gemm.hip at the config-2 GEMM shapes, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24), random operands.  gemm.hip is timed with the plain bias epilogue
and with the epilogue each projection has in the step (FF1: GELU; QKV: qk-norm + RoPE; out / FF2: gated residual).

    python tools/blas_calibration.py [--rounds 3] [--iters 10]
"""
import argparse
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import _native as NN  # noqa: E402
from videopainter_amd import kernels as K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = "cuda"
    B, T, Ntok, D = 2, 226, 17776, 3072
    M = B * Ntok
    cos = torch.randn(Ntok - T, 64, device=dev)
    sin = torch.randn(Ntok - T, 64, device=dev)
    ln = SimpleNamespace(weight=torch.ones(64, device=dev, dtype=torch.bfloat16),
                         bias=torch.zeros(64, device=dev, dtype=torch.bfloat16), eps=1e-6)
    mod = torch.randn(B, 6 * D, device=dev).bfloat16()
    shapes = {"qkv": (3 * D, D), "out": (D, D), "ff1": (4 * D, D), "ff2": (D, 4 * D)}
    for rnd in range(args.rounds):
        for name, (N, Kk) in shapes.items():
            a = torch.randn(M, Kk, device=dev).bfloat16()
            w = (torch.randn(N, Kk, device=dev) * Kk ** -0.5).bfloat16()
            b = torch.zeros(N, device=dev, dtype=torch.bfloat16)
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2 * M * N * Kk
            res = {"hipblaslt": timeit(lambda: torch.matmul(a, w.t(), out=c), args.iters)}
            res["vp_bias"] = timeit(lambda: K.gemm(a, [w], [b], c), args.iters)
            if name == "ff1":
                res["vp_step_epi"] = timeit(lambda: K.gemm(a, [w], [b], c, epilogue=NN.EPI_BIAS_GELU), args.iters)
            elif name == "qkv":
                ws = list(w.view(3, D, Kk).unbind(0))
                bs = list(b.view(3, D).unbind(0))
                res["vp_step_epi"] = timeit(lambda: K.gemm(a, ws, bs, c, epilogue=NN.EPI_BIAS_QKNORM_ROPE,
                                                           qk_norm=(ln, ln), rope=(cos, sin), tokens_per_batch=Ntok,
                                                           text_len=T), args.iters)
            else:
                r = torch.randn(M, N, device=dev).bfloat16()
                res["vp_step_epi"] = timeit(lambda: K.gemm(a, [w], [b], c, epilogue=NN.EPI_GATED, resid=r, mod=mod,
                                                           tokens_per_batch=Ntok, text_len=T), args.iters)
            print(f"r{rnd} {name:4s} {M}x{N}x{Kk}: " + "  ".join(f"{k} {fl / t / 1e12:.0f} TF ({t * 1e3:.3f} ms)"
                                                           for k, t in res.items()), flush=True)
            del a, w, c


if __name__ == "__main__":
    main()
