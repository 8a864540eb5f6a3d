"""Debug helper for the p1 attention kernel: error pattern by query / dim against fp32 SDPA."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videopainter_amd import kernels as K  # noqa: E402


def run(Nq, Nk, mode, split):
    K.set_knob("VP_ATTN_BOUNDED_MODE", mode)
    if split:
        K.set_knob("VP_ATTN_NO_SPLIT", None)
    else:
        K.set_knob("VP_ATTN_NO_SPLIT", "1")
    g = torch.Generator().manual_seed(0)
    B, H = 1, 1
    q = (torch.randn(B, Nq, 64, generator=g) * 0.5).bfloat16()
    k = (torch.randn(B, Nk, 64, generator=g) * 0.5).bfloat16()
    v = torch.randn(B, Nk, 64, generator=g).bfloat16()
    o = torch.empty(B, Nq, 64, device="cuda", dtype=torch.bfloat16)
    K.attention(q.cuda(), k.cuda(), v.cuda(), o, H, bounded_scores=True)
    torch.cuda.synchronize()
    ref = F.scaled_dot_product_attention(q.float()[:, None], k.float()[:, None], v.float()[:, None])[:, 0]
    err = (o.float().cpu() - ref)[0]
    rel = float(err.norm() / ref.norm())
    rq = err.norm(dim=1) / ref[0].norm(dim=1)
    bad = (rq > 2e-2).nonzero().flatten().tolist()
    print(f"{mode} Nq={Nq} Nk={Nk} split={split}: rel {rel:.3e}  bad rows {len(bad)}/{Nq}", bad[:12])
    if bad:
        q0 = bad[0]
        print("   dims err row", q0, [round(x, 3) for x in err[q0, :16].tolist()])
        print("   by (q%64)//32:", [float(rq[[i for i in range(Nq) if (i % 64) // 32 == b]].mean()) for b in (0, 1)])
        print("   ratio o/ref row", q0, [round(x, 3) for x in (o.float().cpu()[0, q0, :8] / ref[0, q0, :8]).tolist()])


for mode in ("p1", "p2"):
    for Nq, Nk, split in ((256, 128, False), (256, 256, False), (256, 640, False), (256, 300, False),
                          (300, 300, True), (512, 1024, False)):
        run(Nq, Nk, mode, split)
