"""Per-head LN(64) + RoPE kernels at config 5's shape (B = 2, 226 + 46 800 tokens, 48 heads; q read in place from
the [B, N, 3D] QKV buffer): the fp8 form the config-5 step runs and the bf16 form, with a bit-identity digest of each
output, so two library builds (VP_HIP_LIB) can be compared for speed and bits in interleaved processes.

    python tools/bench_head_norm.py [--iters 20] [--video-tokens 46800]
"""
import argparse
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--video-tokens", type=int, default=46800)
    a = ap.parse_args()
    B, T, H, D = 2, 226, 48, 3072
    Ntok = T + a.video_tokens
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, Ntok, 3 * D, device="cuda", generator=g).bfloat16()
    q = qkv[..., :D]
    lw = (1 + 0.1 * torch.randn(64, device="cuda", generator=g)).bfloat16()
    lb = (0.1 * torch.randn(64, device="cuda", generator=g)).bfloat16()
    cos = torch.randn(a.video_tokens, 64, device="cuda", generator=g)
    sin = torch.randn(a.video_tokens, 64, device="cuda", generator=g)
    out8 = torch.empty(B, Ntok, D, device="cuda", dtype=torch.uint8)
    out16 = torch.empty(B, Ntok, D, device="cuda", dtype=torch.bfloat16)
    f8 = lambda: K.head_norm_rope_fp8(q, H, T, lw, lb, 1e-6, (cos, sin), 4.0, out=out8)  # noqa: E731
    f16 = lambda: K.head_norm_rope(q, out16, H, T, lw, lb, 1e-6, (cos, sin))  # noqa: E731
    res = {}
    nbytes16 = B * Ntok * D * 2
    for name, fn, wbytes in (("fp8", f8, nbytes16 // 2), ("bf16", f16, nbytes16)):
        t = timeit(fn, a.iters)
        res[name] = {"us": t * 1e6, "tb_per_s": (nbytes16 + wbytes) / t / 1e12}
    torch.cuda.synchronize()
    res["digest_fp8"] = hashlib.sha256(out8.cpu().numpy().tobytes()).hexdigest()[:16]
    res["digest_bf16"] = hashlib.sha256(out16.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
    res["lib"] = os.environ.get("VP_HIP_LIB", "default")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
