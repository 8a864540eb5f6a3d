"""Micro-benchmark of the hot kernels at config-2 shapes (B=2 CFG, N=17776, D=3072) on one MI355X.

    python tools/bench_kernels.py [--iters 10]

Prints TFLOP/s (algorithmic flops) per kernel and shape.  Random data (cdna_hip_programming.md §5.4 rule 25).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from videopainter_amd import _native as N  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--gemm-variants", default="5,11", help="VP_GEMM_VARIANT values, interleaved over 2 rounds")
    ap.add_argument("--variant", default="", help="attention kernel(s): p2a, a16, p2w, p2w2, p2, s16, bounded (default: p2a, bounded)")
    ap.add_argument("--variant8", default="", help="fp8 attention kernel variant(s) (VP_ATTN8_VARIANT), e.g. 1,2")
    ap.add_argument("--only", default="", help="attention | attn8 | gemm | mx | norms: run just that kernel (for rocprofv3 "
                    "--pmc passes; attn8 = the fp8 attention only)")
    ap.add_argument("--video-tokens", type=int, default=17550,
                    help="video tokens per clip (17550 = config 2's 49f 480x720; 46800 = config 5's 49f 720x1280)")
    args = ap.parse_args()
    dev = "cuda"
    B, T, Nv, D, H = 2, 226, args.video_tokens, 3072, 48
    Ntok = T + Nv
    M = B * Ntok
    res = {}
    x = torch.randn(M, 4 * D, device=dev).to(torch.bfloat16)
    shapes = [("qkv", 3 * D, D), ("out", D, D), ("ff1", 4 * D, D), ("ff2", D, 4 * D)]
    if args.only in ("attention", "attn8", "norms"):
        shapes = []
    if args.only == "mx":
        # MX-FP8 FeedForward GEMMs (BASELINE config 5 path) next to their bf16 versions, interleaved
        from videopainter_amd import _native as NN
        for rnd in range(2):
            for name, Nn, Kk in (("ff1", 4 * D, D), ("ff2", D, 4 * D)):
                a16 = torch.randn(M, Kk, device=dev).to(torch.bfloat16)
                w16 = (torch.randn(Nn, Kk, device=dev) * Kk ** -0.5).to(torch.bfloat16)
                b = torch.randn(Nn, device=dev).to(torch.bfloat16) * 0.1
                A, W = K.mx_quantize(a16), K.mx_quantize(w16)
                out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
                t = timeit(lambda: K.gemm_mx(A, [W], [b], out), args.iters)
                res[f"mx_{name}_r{rnd}"] = dict(ms=t * 1e3, tflops=2 * M * Nn * Kk / t / 1e12)
                print("gemm mxfp8", name, res[f"mx_{name}_r{rnd}"], flush=True)
                if name == "ff1":
                    H = K.MXTensor(M, Nn, dev)
                    t = timeit(lambda: K.gemm_mx(A, [W], [b], H, epilogue=NN.EPI_BIAS_GELU_MXFP8), args.iters)
                    res[f"mx_ff1_gelu_mx_r{rnd}"] = dict(ms=t * 1e3, tflops=2 * M * Nn * Kk / t / 1e12)
                    print("gemm mxfp8 ff1+gelu->mx", res[f"mx_ff1_gelu_mx_r{rnd}"], flush=True)
                t = timeit(lambda: K.gemm(a16, [w16], [b], out), args.iters)
                res[f"bf16_{name}_r{rnd}"] = dict(ms=t * 1e3, tflops=2 * M * Nn * Kk / t / 1e12)
                print("gemm bf16", name, res[f"bf16_{name}_r{rnd}"], flush=True)
                del a16, w16, A, W, out
        print(json.dumps(res))
        return
    for rnd in range(2):  # interleaved A/B rounds in one process (cdna_hip_programming.md §5.4 rule 24)
        for name, Nn, Kk in shapes:
            w = (torch.randn(Nn, Kk, device=dev) * Kk ** -0.5).to(torch.bfloat16)
            b = torch.randn(Nn, device=dev).to(torch.bfloat16) * 0.1
            out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
            a = x[:, :Kk]
            for gv in args.gemm_variants.split(","):
                K.set_knob("VP_GEMM_VARIANT", gv)
                t = timeit(lambda: K.gemm(a, [w], [b], out, lda=x.stride(0)), args.iters)
                res[f"gemm{gv}_{name}_r{rnd}"] = dict(ms=t * 1e3, tflops=2 * M * Nn * Kk / t / 1e12)
                print(f"gemm v{gv}", name, res[f"gemm{gv}_{name}_r{rnd}"], flush=True)
            del w, b, out
        K.set_knob("VP_GEMM_VARIANT", None)
    del x
    qkv = torch.randn(B, Ntok, 3 * D, device=dev).to(torch.bfloat16)
    o = torch.empty(B, Ntok, D, device=dev, dtype=torch.bfloat16)
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    fl = 4 * B * H * Ntok * Ntok * 64
    if args.only == "gemm":
        print(json.dumps(res))
        return
    # p2a = the default (no bound needed); bounded = the launch with VP_ATTN_BOUNDED_SCORES (these random q, k:
    # |q.k| * 0.125 * log2 e stays far below the bound of 60), p2a there too unless VP_ATTN_BOUNDED_MODE names p2 / s16
    variants = tuple(args.variant.split(",")) if args.variant else ("p2a", "bounded")
    if args.only in ("attn8", "norms"):
        variants = ()
    for rnd in range(2):  # interleaved A/B rounds in one process (cdna_hip_programming.md §5.4 rule 24)
        for var in variants:
            # unbounded-score kernels (p2a = the default without a proven bound, a16, p2w, p2w2) vs bounded ones
            unb = var in ("a16", "p2a", "p2w", "p2w2", "p2s")
            K.set_knob("VP_ATTN_BOUNDED_MODE", None)
            K.set_knob("VP_ATTN_UNBOUNDED_MODE", None)
            if var != "bounded":
                K.set_knob("VP_ATTN_UNBOUNDED_MODE" if unb else "VP_ATTN_BOUNDED_MODE", var)
            t = timeit(lambda: K.attention(q, k, v, o, H, bounded_scores=not unb), max(2, args.iters // 2))
            res[f"attention_{var}_r{rnd}"] = dict(ms=t * 1e3, tflops=fl / t / 1e12)
            print("attention", var, res[f"attention_{var}_r{rnd}"], flush=True)
    if args.only == "attention":  # bf16 attention only (rocprofv3 --pmc passes filter on the kernel name)
        print(json.dumps(res))
        return
    if args.only == "attn8":
        # fp8 attention (config 5 path) on the same operands: producers once, then the kernel, interleaved with bf16
        q_exp, k_exp = 5, 4
        q8 = (q.float() * 0.125 * K.LOG2E * 2.0 ** q_exp).to(torch.float8_e4m3fn).view(torch.uint8)
        k8 = (k.float() * 2.0 ** k_exp).to(torch.float8_e4m3fn).view(torch.uint8)
        t = timeit(lambda: K.v_pack_fp8(v, H), args.iters)
        res["v_pack_fp8"] = dict(ms=t * 1e3, gbps=(B * Ntok * D * 3) / t / 1e9)
        print("v_pack_fp8", res["v_pack_fp8"], flush=True)
        vp = K.v_pack_fp8(v, H)
        for rnd in range(2):
            for var in (args.variant8.split(",") if args.variant8 else [""]):
                if var:
                    K.set_knob("VP_ATTN8_VARIANT", var)
                t = timeit(lambda: K.attention_fp8(q8, k8, vp, o, H, q_exp, k_exp), max(2, args.iters // 2))
                res[f"attention_fp8_v{var}_r{rnd}"] = dict(ms=t * 1e3, tflops=fl / t / 1e12)
                print("attention fp8", var, res[f"attention_fp8_v{var}_r{rnd}"], flush=True)
        K.set_knob("VP_ATTN8_VARIANT", None)
        print(json.dumps(res))
        return
    xin = torch.randn(B, Ntok, D, device=dev).to(torch.bfloat16)
    mod = torch.randn(B, 6 * D, device=dev).to(torch.bfloat16)
    lw = torch.ones(D, device=dev, dtype=torch.bfloat16)
    lb = torch.zeros(D, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(xin)
    t = timeit(lambda: K.adaln_modulate(xin, lw, lb, mod, T, 1e-5, out=y), args.iters)
    res["adaln"] = dict(ms=t * 1e3, gbps=2 * xin.numel() * 2 / t / 1e9)
    print("adaln", res["adaln"], flush=True)
    # the read+write ceiling these one-pass kernels are held to: a plain device-to-device copy of the same bytes
    # (same dtype and layout, so torch hands it to the runtime's copy), the same 1:1 read:write mix as AdaLN / qk-norm
    t = timeit(lambda: y.copy_(xin), args.iters)
    res["copy_d2d"] = dict(ms=t * 1e3, gbps=2 * xin.numel() * 2 / t / 1e9)
    print("copy roofline", res["copy_d2d"], flush=True)
    cos = torch.randn(Nv, 64, device=dev)
    sin = torch.randn(Nv, 64, device=dev)
    lw64 = torch.ones(64, device=dev, dtype=torch.bfloat16)
    lb64 = torch.zeros(64, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: K.head_norm_rope(q, q, H, T, lw64, lb64, 1e-6, (cos, sin)), args.iters)
    res["qk_norm_rope(q)"] = dict(ms=t * 1e3, gbps=2 * B * Ntok * D * 2 / t / 1e9)
    print("qknorm", res["qk_norm_rope(q)"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
