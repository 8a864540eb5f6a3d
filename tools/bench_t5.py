"""T5-XXL text encoder (CogVideoX's, google t5-v1_1-xxl: 24 layers, d_model 4096, 64 heads, d_ff 10240) on one
MI355X: the prompt + negative prompt (batch 2 x 226 tokens, the pipeline's _get_t5_prompt_embeds, anyl.py:216-256)
through the HIP encoder, random-init weights of the real shapes.

    python tools/bench_t5.py [--iters 5] [--batch 2]

At M = 452 token rows every projection streams its weights once (4.76e9 parameters = 9.5 GB bf16 per forward), so
the weights are read once (9.3 GB: an HBM floor of 1.5 ms at 6.3 TB/s) against 4.2 TFLOP (1.7 ms at the bf16 MFMA
peak): both roofs are close, the MFMA one slightly higher.  Times the eager forward and the HIP-graph replay
(T5EncoderModel.enable_hip_graphs) and checks they agree bit for bit.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402
from videopainter_amd.t5 import T5EncoderModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--tokens", type=int, default=226)
    args = ap.parse_args()
    m = T5EncoderModel.from_config({}, device="cuda")
    nparam = 0
    wbytes = 0
    flop_tok = 0
    for i, (name, p) in enumerate(m.named_parameters()):
        if p.dim() == 1:
            p.data.fill_(1.0)
        else:
            K.fill_normal_(p.data, 1000 + i, 0.0, p.shape[1] ** -0.5)
        nparam += p.numel()
        if "embed" in name or "shared" in name:
            continue  # the token table is gathered (452 rows), not streamed
        wbytes += p.numel() * p.element_size()
        if p.dim() == 2 and "relative_attention_bias" not in name:
            flop_tok += 2 * p.numel()
    cfg = m.config
    L, B = args.tokens, args.batch
    attn_flop = cfg.num_layers * 4 * B * L * L * cfg.num_heads * cfg.d_kv
    flop = flop_tok * B * L + attn_flop
    ids = torch.randint(0, cfg.vocab_size, (B, L), device="cuda")
    with torch.no_grad():
        out = m(input_ids=ids)[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            out = m(input_ids=ids)[0]
        torch.cuda.synchronize()
        sec = (time.perf_counter() - t0) / args.iters
        eager = out.float()
        m.enable_hip_graphs()
        out = m(input_ids=ids)[0]  # capture
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            out = m(input_ids=ids)[0]
        torch.cuda.synchronize()
        sec_graph = (time.perf_counter() - t0) / args.iters
        same = bool(torch.equal(out.float(), eager))
    finite = bool(torch.isfinite(out.float()).all())
    print(json.dumps({"config": f"T5-XXL encoder (t5-v1_1-xxl shapes), batch {B} x {L} tokens, bf16, random weights",
                      "seconds_eager": sec, "seconds": sec_graph, "graph_equals_eager": same,
                      "params": nparam, "weight_bytes": wbytes, "hbm_gbps": wbytes / sec_graph / 1e9,
                      "hbm_frac_of_8tbs": wbytes / sec_graph / 8e12, "tflop": flop / 1e12,
                      "tflops": flop / sec_graph / 1e12, "mfma_frac": flop / sec_graph / 2.5e15,
                      "output": list(out.shape), "finite": finite}))


if __name__ == "__main__":
    main()
