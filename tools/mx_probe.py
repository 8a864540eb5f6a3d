"""Diagnose the scale layout of v_mfma_scale_f32_16x16x128_f8f6f4 on the GPU (one MFMA per probe).

    python tools/mx_probe.py

The probe kernel (vp_mx_mfma_probe) loads lane l's 32 operand bytes from row l % 16, bytes 32*(l // 16) .. +31 of
a [16][128] e4m3 matrix and lane l's scale byte from sa[l] / sb[l].  With unit data restricted to the bytes of lane
group b (= stored columns 32b .. 32b+31) and one lane's A scale doubled, the change in C shows which rows and which
lane group's data that lane's scale multiplies.
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
    ones = torch.ones(16, 128)
    Bq = e4m3(ones).to(dev)
    s127 = torch.full((64,), 127, dtype=torch.uint8)
    for which in ("A", "B"):
        print(f"--- scale of operand {which} ---", flush=True)
        for L in range(64):
            hits = []
            for b in range(4):
                A = torch.zeros(16, 128)
                A[:, 32 * b:32 * b + 32] = 1.0
                Aq = e4m3(A).to(dev)
                base = K.mx_mfma_probe(Aq, Bq, s127.to(dev), s127.to(dev)).cpu()
                s = s127.clone()
                s[L] = 128
                if which == "A":
                    C = K.mx_mfma_probe(Aq, Bq, s.to(dev), s127.to(dev)).cpu()
                else:
                    C = K.mx_mfma_probe(Aq, Bq, s127.to(dev), s.to(dev)).cpu()
                d = C - base
                nz = (d != 0).nonzero()
                if len(nz):
                    rows = sorted(set(nz[:, 0].tolist()))
                    cols = sorted(set(nz[:, 1].tolist()))
                    hits.append(f"b{b}: rows {rows[:4]}{'...' if len(rows) > 4 else ''} cols {cols[:4]}"
                                f"{'...' if len(cols) > 4 else ''} delta {float(d[nz[0, 0], nz[0, 1]]):g}")
            print(f"lane {L:2d}: " + ("; ".join(hits) if hits else "no effect"), flush=True)


if __name__ == "__main__":
    main()
