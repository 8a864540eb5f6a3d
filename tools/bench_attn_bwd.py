"""Flash-attention backward timing at the training shape (B=1, 48 heads, N = 226 + 17550): dQ and dK/dV kernels
via rocprof or this script's HIP events around the whole vp_attention_bwd_bf16 call.
    python tools/bench_attn_bwd.py [--n 17776] [--heads 48] [--iters 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=17776)
    ap.add_argument("--heads", type=int, default=48)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--variants", default="", help="comma-separated VP_ATTN_BWD_VARIANT values, timed interleaved")
    ap.add_argument("--split-ab", action="store_true", help="grid-tail split (default) vs VP_ATTN_NO_SPLIT=1, interleaved")
    a = ap.parse_args()
    from videopainter_amd import kernels as K
    torch.manual_seed(0)
    B, H, N = 1, a.heads, a.n
    q, k, v, do = (torch.randn(B, N, H * 64, device="cuda").bfloat16() for _ in range(4))
    o = torch.empty_like(q)
    lse = torch.empty(B, H, N, device="cuda", dtype=torch.float32)
    K.attention(q, k, v, o, H, lse=lse)
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    for _ in range(2):
        K.attention_bwd(q, k, v, o, do, lse, H, dq=dq, dk=dk, dv=dv)
    torch.cuda.synchronize()
    fl = 8.0 * B * H * N * N * 64  # dV, dP, dQ, dK (the S recompute not counted)
    if a.variants:  # interleaved A/B of the library's backward variants, 3 rounds
        res = {v: [] for v in a.variants.split(",")}
        for _ in range(3):
            for var in res:
                K.set_knob("VP_ATTN_BWD_VARIANT", var)
                K.attention_bwd(q, k, v, o, do, lse, H, dq=dq, dk=dk, dv=dv)
                with K.timed_launches("attention_bwd") as tl:
                    for _ in range(a.iters):
                        K.attention_bwd(q, k, v, o, do, lse, H, dq=dq, dk=dk, dv=dv)
                res[var].append(round(tl.mean_ms("attention_bwd"), 4))
        K.set_knob("VP_ATTN_BWD_VARIANT", None)
        print(json.dumps({"n": N, "heads": H, "bwd_ms_by_variant": res}))
        return
    if a.split_ab:  # interleaved: the backward's grid-tail split against the unsplit grids (5 rounds)
        res = {"split": [], "whole": []}
        for _ in range(5):
            for arm in res:
                K.set_knob("VP_ATTN_NO_SPLIT", "1" if arm == "whole" else None)
                K.attention_bwd(q, k, v, o, do, lse, H, dq=dq, dk=dk, dv=dv)
                with K.timed_launches("attention_bwd") as tl:
                    for _ in range(a.iters):
                        K.attention_bwd(q, k, v, o, do, lse, H, dq=dq, dk=dk, dv=dv)
                res[arm].append(round(tl.mean_ms("attention_bwd"), 4))
        K.set_knob("VP_ATTN_NO_SPLIT", None)
        print(json.dumps({"n": N, "heads": H, "bwd_ms": res}))
        return
    with K.timed_launches("attention_bwd", "attention") as tl:
        for _ in range(a.iters):
            K.attention(q, k, v, o, H, lse=lse)
            K.attention_bwd(q, k, v, o, do, lse, H, dq=dq, dk=dk, dv=dv)
    ms = tl.mean_ms("attention_bwd")
    print(json.dumps({"n": N, "heads": H, "bwd_ms": ms, "fwd_ms": tl.mean_ms("attention"),
                      "bwd_useful_tflops": fl / ms / 1e9, "fwd_tflops": 4.0 * B * H * N * N * 64 / tl.mean_ms("attention") / 1e9}))


if __name__ == "__main__":
    main()
