"""Diagnose the operand/scale layout of v_mfma_scale_f32_32x32x64_f8f6f4 (vp_mx_mfma_probe32): with unit data in
one 32-column K-block at a time and one lane's scale doubled, print which rows / columns of C change.

    python tools/mx_probe32.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402


def e4m3(x):
    return x.to(torch.float8_e4m3fn).view(torch.uint8)


def main():
    dev = "cuda"
    s127 = torch.full((64,), 127, dtype=torch.uint8)
    for which in ("A", "B"):
        print(f"--- scale of operand {which} ---", flush=True)
        for L in list(range(0, 64, 1)):
            hits = []
            for kb in range(2):
                A = torch.zeros(32, 64)
                A[:, 32 * kb:32 * kb + 32] = 1.0
                Bm = torch.ones(32, 64)
                Aq, Bq = e4m3(A).to(dev), e4m3(Bm).to(dev)
                base = K.mx_mfma_probe32(Aq, Bq, s127.to(dev), s127.to(dev)).cpu()
                s = s127.clone()
                s[L] = 128
                if which == "A":
                    C = K.mx_mfma_probe32(Aq, Bq, s.to(dev), s127.to(dev)).cpu()
                else:
                    C = K.mx_mfma_probe32(Aq, Bq, s127.to(dev), s.to(dev)).cpu()
                nz = ((C - base) != 0).nonzero()
                if len(nz):
                    rows = sorted(set(nz[:, 0].tolist()))
                    cols = sorted(set(nz[:, 1].tolist()))
                    hits.append(f"kb{kb}: rows {rows[:3]}..({len(rows)}) cols {cols[:3]}..({len(cols)}) "
                                f"delta {float((C - base)[nz[0, 0], nz[0, 1]]):g}")
            print(f"lane {L:2d}: " + ("; ".join(hits) if hits else "no effect"), flush=True)
    # data layout: one nonzero byte at A[r][k] -> which C entries
    print("--- data: A[0][k] = 1, B = ones: C row 0 should be 1 for every k ---", flush=True)
    for k in range(0, 64, 4):
        A = torch.zeros(32, 64)
        A[0, k] = 1.0
        C = K.mx_mfma_probe32(e4m3(A).to(dev), e4m3(torch.ones(32, 64)).to(dev), s127.to(dev), s127.to(dev)).cpu()
        print(f"k {k:2d}: C row0 sum {float(C[0].sum()):g} total {float(C.sum()):g}", flush=True)


if __name__ == "__main__":
    main()
