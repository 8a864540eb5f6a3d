"""Workgroup timeline of the default bf16 attention launch (p2a with its one-launch grid tail) at config 2's shape,
from a diagnostic build with -DVP_CLOCK_STAMPS=1 -DVP_CLOCK_WG=1 (realtime at workgroup entry, loop start, loop end
and exit, 100 MHz):

    python tools/attn_wg_timeline.py --build                 # CPU host: videopainter_amd/_lib/libvp_hip_clkwg.so
    VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_clkwg.so python tools/attn_wg_timeline.py [--batch 2]

Prints the prologue / loop / epilogue split per workgroup, the slot concurrency over time and the idle slot-time
at the end of the launch.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--tail", default="", help="VP_ATTN_TAIL value (default: the library default)")
    ap.add_argument("--items", action="store_true",
                    help="per work item of the persistent launch (the -DVP_CLOCK_WG=2 build, libvp_hip_clkitem.so)")
    a = ap.parse_args()
    if a.build:
        from videopainter_amd.build import build
        build(out=os.path.join(ROOT, "videopainter_amd", "_lib", "libvp_hip_clkwg.so"),
              extra_flags={"attention.hip": ["-DVP_CLOCK_STAMPS=1", "-DVP_CLOCK_WG=1"]})
        build(out=os.path.join(ROOT, "videopainter_amd", "_lib", "libvp_hip_clkitem.so"),
              extra_flags={"attention.hip": ["-DVP_CLOCK_STAMPS=1", "-DVP_CLOCK_WG=2"]})
        return
    import numpy as np
    import torch
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    L = N.lib()
    L.vp_diag_clock_read.restype = C.c_int
    L.vp_diag_clock_read.argtypes = [C.c_void_p, C.c_int64]
    if a.tail:
        K.set_knob("VP_ATTN_TAIL", a.tail)
    B, H, Nt = a.batch, 48, 17776
    qkv = (torch.randn(B, Nt, 3 * H * 64, device="cuda") * 0.5).bfloat16()
    q, k, v = qkv[..., :H * 64], qkv[..., H * 64:2 * H * 64], qkv[..., 2 * H * 64:]
    o = torch.empty(B, Nt, H * 64, device="cuda", dtype=torch.bfloat16)
    run = lambda: K.attention(q, k, v, o, H, bounded_scores=True)  # noqa: E731
    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    run()
    e.record()
    torch.cuda.synchronize()
    one = s.elapsed_time(e)
    for _ in range(max(3, int(a.seconds * 1e3 / one))):
        run()
    s.record()
    run()
    e.record()
    torch.cuda.synchronize()
    wall = s.elapsed_time(e) * 1e3
    n = 32768
    buf = (C.c_uint64 * (4 * n))()
    N.check(L.vp_diag_clock_read(buf, n), "vp_diag_clock_read")
    if a.items:
        raw = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4)
        wgs = (raw[:, 0] >> np.uint64(48)).astype(np.int64)
        st = (raw[:, 0] & np.uint64((1 << 48) - 1)).astype(np.float64)
        r0, r1, ex = (raw[:, i].astype(np.float64) for i in (1, 2, 3))
        ok = st > 0
        last = ex[ok].max()
        ok &= st > last - wall * 100 * 1.5
        st, r0, r1, ex, wgs = st[ok], r0[ok], r1[ok], ex[ok], wgs[ok]
        t0 = st.min()
        pro, loop, epi = (r0 - st) / 100, (r1 - r0) / 100, (ex - r1) / 100
        gaps = []
        for w in np.unique(wgs):
            m = wgs == w
            o = np.argsort(st[m])
            s_, e_ = st[m][o], ex[m][o]
            gaps += list((s_[1:] - e_[:-1]) / 100)
        gaps = np.array(gaps)
        pc = lambda v: [round(float(np.percentile(v, p)), 2) for p in (10, 50, 90)]  # noqa: E731
        slots = len(np.unique(wgs))
        print(json.dumps(dict(items=int(ok.sum()), workgroups=slots, wall_us=round(wall, 1),
                              span_us=round(float(ex.max() - t0) / 100, 1),
                              loop_over_span=round(float(loop.sum()) / (slots * float(ex.max() - t0) / 100), 4),
                              prologue_us=pc(pro), loop_us=pc(loop), epilogue_us=pc(epi), gap_us=pc(gaps),
                              mean_us=dict(prologue=round(float(pro.mean()), 2), epilogue=round(float(epi.mean()), 2),
                                           gap=round(float(gaps.mean()), 2), loop=round(float(loop.mean()), 1)))))
        return
    x = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.float64)
    wid = np.arange(n)
    keep = x[:, 0] > 0
    x, wid = x[keep], wid[keep]
    last = x[:, 3].max()
    keep = x[:, 0] > last - wall * 100 * 1.5  # this launch's workgroups (every launch writes the same slots)
    x, wid = x[keep], wid[keep]
    # per XCD (workgroup id % 8: the dispatcher's round robin), in that XCD's own realtime stamps
    xcd = []
    for c in range(8):
        m = wid % 8 == c
        if not m.any():
            continue
        xs = x[m]
        xcd.append(dict(xcd=c, n=int(m.sum()), first_entry_us=round(float(xs[:, 0].min() - x[:, 0].min()) / 100, 1),
                        last_exit_us=round(float(xs[:, 3].max() - x[:, 0].min()) / 100, 1),
                        loop_us_median=round(float(np.median(xs[:, 2] - xs[:, 1])) / 100, 1),
                        busy_over_64_span=round(float(np.sum(xs[:, 3] - xs[:, 0])) /
                                                (64 * float(xs[:, 3].max() - xs[:, 0].min())), 4)))
    t0 = x[:, 0].min()
    e0, r0, r1, ex = ((x[:, i] - t0) / 100.0 for i in range(4))  # us
    span = ex.max()
    pro, loop, epi = r0 - e0, r1 - r0, ex - r1
    ev = np.concatenate([np.stack([e0, np.ones_like(e0)], 1), np.stack([ex, -np.ones_like(ex)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    conc = np.cumsum(ev[:, 1])
    tt = ev[:, 0]
    bins = []
    nb = 16
    for w in range(nb):
        w0, w1 = span * w / nb, span * (w + 1) / nb
        m = (tt >= w0) & (tt < w1)
        idx = np.where(m)[0]
        if len(idx) == 0:
            continue
        t2 = np.append(tt[idx], w1)
        bins.append(round(float(np.sum(np.diff(t2) * conc[idx]) / (w1 - w0)), 1))
    busy = float(np.sum(ex - e0))
    slots = int(conc.max())
    pct = lambda v: [round(float(np.percentile(v, p)), 1) for p in (10, 50, 90)]  # noqa: E731
    res = dict(batch=B, tail=a.tail or "default", workgroups=len(x), wall_us=round(wall, 1), span_us=round(span, 1),
               slots_max=slots, busy_over_span=round(busy / (slots * span), 4),
               loop_over_span=round(float(np.sum(loop)) / (slots * span), 4),
               prologue_us_p10_50_90=pct(pro), loop_us_p10_50_90=pct(loop), epilogue_us_p10_50_90=pct(epi),
               concurrency_by_sixteenth=bins, per_xcd=xcd)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
