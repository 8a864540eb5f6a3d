"""A/B of the p2 / p2a attention with kept LDS addresses (default) against the per-tile slot-base form (VP_P2_KEPT=0)
at config 2's shape, in one process: bit identity of the outputs first, then interleaved timings."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402


def main():
    B, H, N = 2, 48, 17776
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn(B, N, H * 64, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(B, N, H * 64, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(B, N, H * 64, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty_like(q)
    for bounded in (True, False):
        outs = {}
        for kept in ("1", "0"):
            os.environ["VP_P2_KEPT"] = kept
            if bounded:
                K.set_knob("VP_ATTN_BOUNDED_MODE", "p2")
            K.attention(q, k, v, o, H, bounded_scores=bounded)
            torch.cuda.synchronize()
            outs[kept] = o.clone()
            K.set_knob("VP_ATTN_BOUNDED_MODE", None)
        same = torch.equal(outs["1"].view(torch.int16), outs["0"].view(torch.int16))
        print(f"{'p2 (bounded)' if bounded else 'p2a'}: kept vs slot-base outputs bit-identical: {same}", flush=True)
        if not same:
            raise SystemExit(1)
    fl = 4 * B * H * N * N * 64
    for rnd in range(3):
        for kept in ("1", "0"):
            os.environ["VP_P2_KEPT"] = kept
            K.attention(q, k, v, o, H)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                K.attention(q, k, v, o, H)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            print(f"round {rnd} p2a kept={kept}: {dt * 1e3:.3f} ms {fl / dt / 1e12:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
