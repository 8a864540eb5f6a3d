"""The CogVideoX block's four projection GEMMs at config-2 shapes WITH their fused epilogues (random data):
QKV (bias + qk-LayerNorm + RoPE), to_out (gated residual), FF1 (bias + GELU-tanh), FF2 (gated residual + masked
branch injection).  Prints ms and TFLOP/s per shape (2 rounds in one process).

    python tools/gemm_block_shapes.py [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from videopainter_amd import _native as N  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

B, T, NV, D = 2, 226, 17550, 3072
NTOK = T + NV
M = B * NTOK


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev).bfloat16()  # noqa: E731
    w = lambda n, k: (torch.randn(n, k, device=dev) * k ** -0.5).bfloat16()  # noqa: E731
    x = r(M, D)
    h = r(M, 4 * D)
    wq, wk, wv, wo = w(D, D), w(D, D), w(D, D), w(D, D)
    w1, w2 = w(4 * D, D), w(D, 4 * D)
    bias = [r(D) * 0.1 for _ in range(4)]
    b1 = r(4 * D) * 0.1
    nq, nk = torch.nn.LayerNorm(64).to(dev).bfloat16(), torch.nn.LayerNorm(64).to(dev).bfloat16()
    cos, sin = torch.rand(NV, 64, device=dev), torch.rand(NV, 64, device=dev)
    mod = r(B, 6 * D) * 0.1
    inject = r(B, NV, D)
    mask = (torch.rand(B, NV, device=dev) > 0.75).to(torch.uint8)
    qkv = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    o1 = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
    calls = {
        "qkv": (2 * M * 3 * D * D, lambda: K.gemm(x, [wq, wk, wv], bias[:3], qkv, epilogue=N.EPI_BIAS_QKNORM_ROPE,
                                                   tokens_per_batch=NTOK, text_len=T, qk_norm=(nq, nk), rope=(cos, sin))),
        "out": (2 * M * D * D, lambda: K.gemm(x, [wo], [bias[3]], o1, epilogue=N.EPI_GATED, resid=x, mod=mod,
                                               tokens_per_batch=NTOK, text_len=T)),
        "ff1": (2 * M * 4 * D * D, lambda: K.gemm(x, [w1], [b1], o2, epilogue=N.EPI_BIAS_GELU)),
        "ff2": (2 * M * 4 * D * D, lambda: K.gemm(h, [w2], [bias[0]], o1, epilogue=N.EPI_GATED, resid=x, mod=mod,
                                                   tokens_per_batch=NTOK, text_len=T, inject=inject,
                                                   inject_ld=inject.stride(1), inject_bstride=inject.stride(0),
                                                   inject_mask=mask)),
    }
    res = {}
    for rnd in range(2):
        for name, (fl, fn) in calls.items():
            t = timeit(fn, args.iters)
            res[f"{name}_r{rnd}"] = dict(ms=t * 1e3, tflops=fl / t / 1e12)
            print(name, res[f"{name}_r{rnd}"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
