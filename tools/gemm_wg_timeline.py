"""Per-XCD workgroup timeline of one GEMM launch (FF1 / out / QKV / FF2 at config 2's M), from a diagnostic build
with -DVP_CLOCK_STAMPS=1 on gemm.hip (realtime at workgroup entry and exit per blockIdx):

    python tools/gemm_wg_timeline.py --build            # CPU host: videopainter_amd/_lib/libvp_hip_gemmclk.so
    VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_gemmclk.so python tools/gemm_wg_timeline.py [--shape ff1]

The dispatcher gives every XCD (workgroup id % 8) the same number of workgroups; this shows when each XCD finished
its share (the tail split is off: VP_GEMM_NO_TAIL, so one launch holds every tile).
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
    ap.add_argument("--shape", default="ff1")
    ap.add_argument("--m", type=int, default=35552)
    a = ap.parse_args()
    if a.build:
        from videopainter_amd.build import build
        build(out=os.path.join(ROOT, "videopainter_amd", "_lib", "libvp_hip_gemmclk.so"),
              extra_flags={"gemm.hip": ["-DVP_CLOCK_STAMPS=1"]})
        return
    import numpy as np
    import torch
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    L = N.lib()
    L.vp_diag_gemm_clock_read.restype = C.c_int
    L.vp_diag_gemm_clock_read.argtypes = [C.c_void_p, C.c_int64]
    K.set_knob("VP_GEMM_NO_TAIL", "1")
    M, D, F = a.m, 3072, 12288
    Kk, Nn = {"ff1": (D, F), "out": (D, D), "qkv": (D, 3 * D), "ff2": (F, D)}[a.shape]
    x = torch.randn(M, Kk, device="cuda").bfloat16()
    w = (torch.randn(Nn, Kk, device="cuda") * Kk ** -0.5).bfloat16()
    b = torch.zeros(Nn, device="cuda").bfloat16()
    out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    run = lambda: K.gemm(x, [w], [b], out)  # noqa: E731
    for _ in range(max(3, int(2000 / 2))):  # ~2 s back to back: the clock the chip holds
        run()
        if _ > 20:
            break
    torch.cuda.synchronize()
    for _ in range(200):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    run()
    e.record()
    torch.cuda.synchronize()
    wall = s.elapsed_time(e) * 1e3
    tiles = ((M + 255) // 256) * ((Nn + 255) // 256)
    buf = (C.c_uint64 * (2 * tiles))()
    N.check(L.vp_diag_gemm_clock_read(buf, tiles), "vp_diag_gemm_clock_read")
    x_ = np.frombuffer(buf, dtype=np.uint64).reshape(tiles, 2).astype(np.float64)
    t0 = x_[:, 0].min()
    e0, ex = (x_[:, 0] - t0) / 100.0, (x_[:, 1] - t0) / 100.0
    dur = ex - e0
    wid = np.arange(tiles)
    per = []
    for c in range(8):
        m = wid % 8 == c
        per.append(dict(xcd=c, n=int(m.sum()), last_exit_us=round(float(ex[m].max()), 1),
                        tile_us_median=round(float(np.median(dur[m])), 1),
                        busy_over_32_span=round(float(dur[m].sum()) / (32 * float(ex[m].max() - e0[m].min())), 4)))
    fin = [p["last_exit_us"] for p in per]
    print(json.dumps(dict(shape=a.shape, m=M, tiles=tiles, wall_us=round(wall, 1), span_us=round(float(ex.max()), 1),
                          xcd_finish_mean_us=round(sum(fin) / 8, 1), xcd_finish_max_us=max(fin), per_xcd=per)))
    K.set_knob("VP_GEMM_NO_TAIL", None)


if __name__ == "__main__":
    main()
