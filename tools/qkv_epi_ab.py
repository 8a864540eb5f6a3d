"""The fused QKV GEMM's epilogue cost at config 2's shape (M = 2 x 17776, N = 3 x 3072, K = 3072), interleaved in one
process: the bias epilogue, the qk-norm + RoPE epilogue with the [Nv, 64] fp32 RoPE tables, the same epilogue
with no RoPE table (no table loads: what the table traffic costs), and with the separable table's per-axis rows.
    python tools/qkv_epi_ab.py [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    from videopainter_amd.modules import LayerNorm
    dev = "cuda"
    B, T, Nv, D = 2, 226, 17550, 3072
    Ntok = T + Nv
    M = B * Ntok
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    ws = [(torch.randn(D, D, device=dev, generator=g) * D ** -0.5).to(torch.bfloat16) for _ in range(3)]
    bs = [(torch.randn(D, device=dev, generator=g) * 0.1).to(torch.bfloat16) for _ in range(3)]
    nq, nk = LayerNorm(64, eps=1e-6).to(dev, torch.bfloat16), LayerNorm(64, eps=1e-6).to(dev, torch.bfloat16)
    from videopainter_amd.attention_processor import RopeTables
    from videopainter_amd.embeddings import prepare_rotary_positional_embeddings
    cos, sin = prepare_rotary_positional_embeddings(480, 720, 13, 64, device=dev)  # config 2's table (13 x 30 x 45)
    rope_sep = RopeTables((cos.float().contiguous(), sin.float().contiguous()))
    rope_sep.grid = (13, 30, 45)
    cos, sin = rope_sep
    out = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    runs = {
        "bias": lambda: K.gemm(x, ws, bs, out),
        "qknorm_rope": lambda: K.gemm(x, ws, bs, out, epilogue=N.EPI_BIAS_QKNORM_ROPE, qk_norm=(nq, nk),
                                      rope=(cos, sin), tokens_per_batch=Ntok, text_len=T),
        "qknorm_norope": lambda: K.gemm(x, ws, bs, out, epilogue=N.EPI_BIAS_QKNORM_ROPE, qk_norm=(nq, nk),
                                        rope=None, tokens_per_batch=Ntok, text_len=T),
        "qknorm_rope_sep": lambda: K.gemm(x, ws, bs, out, epilogue=N.EPI_BIAS_QKNORM_ROPE, qk_norm=(nq, nk),
                                          rope=rope_sep, tokens_per_batch=Ntok, text_len=T),
    }
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, f in runs.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(round(e0.elapsed_time(e1) / a.iters, 4))
    print(json.dumps({"qkv_ms": res}))


if __name__ == "__main__":
    main()
