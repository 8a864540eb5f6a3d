"""In-kernel clock of the bf16 attention kernels (MI355X_MICROARCH.md 'DVFS give-back' item 6).

    python tools/attn_clock.py --build            # on the CPU host: the diagnostic libraries (in-tree, they travel)
    VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_clk.so python tools/attn_clock.py --variants p2a,s16

Each diagnostic library is the default one built with -DVP_CLOCK_STAMPS=1 (every p2 / p2a / s16 / a16 workgroup
stamps s_memtime and s_memrealtime around its key loop into a buffer of its own) and optionally -DVP_P1_ABL=<bits>
(p2 / p2a ablations, outputs invalid: 1 = no K/V DMA after the prologue, 2 = v_exp_f32 -> v_mov_b32).  At config 2's
attention shape on random data: >= 2 s of back-to-back launches per variant, then the wall time per call (HIP events)
and the clock = median over main-grid workgroups of delta memtime / delta realtime x 100 MHz.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIBS = {"clk": {}, "clk_nodma": {"attention.hip": ["-DVP_P1_ABL=1"]}, "clk_noexp": {"attention.hip": ["-DVP_P1_ABL=2"]},
        "clk_noboth": {"attention.hip": ["-DVP_P1_ABL=3"]}, "clk_l2": {"attention.hip": ["-DVP_P1_ABL=4"]}}


def build_all():
    from videopainter_amd.build import build
    for name, extra in LIBS.items():
        fl = {"attention.hip": ["-DVP_CLOCK_STAMPS=1"] + extra.get("attention.hip", [])}
        build(out=os.path.join(ROOT, "videopainter_amd", "_lib", f"libvp_hip_{name}.so"), extra_flags=fl)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default="p2a,s16")
    ap.add_argument("--seconds", type=float, default=2.5)
    ap.add_argument("--label", default="")
    ap.add_argument("--video-tokens", type=int, default=17550)
    ap.add_argument("--dump", default="", help="path prefix: per-workgroup stamps (t0 r0 t1 r1) + per-head phase stats")
    args = ap.parse_args()
    if args.build:
        build_all()
        return
    import torch
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    L = N.lib()
    L.vp_diag_clock_read.restype = C.c_int
    L.vp_diag_clock_read.argtypes = [C.c_void_p, C.c_int64]
    B, T, H, D = 2, 226, 48, 3072
    Ntok = T + args.video_tokens
    qkv = torch.randn(B, Ntok, 3 * D, device="cuda").to(torch.bfloat16)
    o = torch.empty(B, Ntok, D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    fl = 4 * B * H * Ntok * Ntok * 64
    res = {}
    for var in args.variants.split(","):
        nblk = B * H * ((Ntok + 511) // 512 if var.startswith("p2w") else (Ntok + 255) // 256)
        unb = var in ("a16", "p2a", "p2w", "p2w2", "p2s")
        K.set_knob("VP_ATTN_BOUNDED_MODE", None)
        K.set_knob("VP_ATTN_UNBOUNDED_MODE", None)
        K.set_knob("VP_ATTN_UNBOUNDED_MODE" if unb else "VP_ATTN_BOUNDED_MODE", var)
        # no grid-tail split: every block is a main-grid workgroup with its own stamp slot
        K.set_knob("VP_ATTN_NO_SPLIT", "1")
        run = lambda: K.attention(q, k, v, o, H, bounded_scores=not unb)  # noqa: E731
        run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e.record()
        torch.cuda.synchronize()
        one = s.elapsed_time(e) / 1e3
        warm = max(3, int(args.seconds / one))
        for _ in range(warm):  # >= 2 s back to back: the clock the chip holds under this load
            run()
        n = 5
        s.record()
        for _ in range(n):
            run()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / n / 1e3
        buf = (C.c_uint64 * (4 * nblk))()
        N.check(L.vp_diag_clock_read(buf, nblk), "vp_diag_clock_read")
        ghz = []
        for i in range(nblk):
            t0, r0, t1, r1 = buf[4 * i:4 * i + 4]
            if r1 > r0 and t1 > t0:
                ghz.append((t1 - t0) / (r1 - r0) * 0.1)
        ghz.sort()
        q10 = ghz[len(ghz) // 10] if ghz else float("nan")
        q90 = ghz[9 * len(ghz) // 10] if ghz else float("nan")
        loop_us = statistics.median([(buf[4 * i + 3] - buf[4 * i + 1]) / 100.0 for i in range(nblk)])
        # per-head phase: blocks t = xcd_remap(blockIdx) of one (b, h) are t // nqb; sorted start times of a head's
        # blocks, the span of its first 64 (one XCD's worth of slots) and the lag of the rest, in loop times
        phase = {}
        if not var.startswith("p2w") and args.dump:
            nqb = (Ntok + 255) // 256
            qq, rr = divmod(nblk, 8)
            starts = {}
            for i in range(nblk):
                x, idx = i % 8, i // 8
                tq = (x * (qq + 1) if x < rr else rr * (qq + 1) + (x - rr) * qq) + idx
                starts.setdefault(tq // nqb, []).append(buf[4 * i + 1])
            loop_t = loop_us * 100.0
            sp64, lag = [], []
            for bh, st in starts.items():
                st.sort()
                sp64.append((st[min(63, len(st) - 1)] - st[0]) / loop_t)
                if len(st) > 64:
                    lag.append((st[-1] - st[0]) / loop_t)
            sp64.sort()
            lag.sort()
            phase = dict(heads=len(starts), span64_median=round(statistics.median(sp64), 3),
                         span64_p90=round(sp64[9 * len(sp64) // 10], 3),
                         span_all_median=round(statistics.median(lag), 3) if lag else None)
            with open(args.dump + f".{var}.txt", "w") as f:
                for i in range(nblk):
                    f.write(" ".join(str(v) for v in buf[4 * i:4 * i + 4]) + "\n")
        res[var] = dict(ms=round(t * 1e3, 4), tflops=round(fl / t / 1e12, 1), clock_ghz_median=round(statistics.median(ghz), 4),
                        clock_ghz_p10=round(q10, 4), clock_ghz_p90=round(q90, 4), loop_us_median=round(loop_us, 1),
                        workgroups=len(ghz), warm_launches=warm, **phase)
        print(args.label, var, json.dumps(res[var]), flush=True)
    K.set_knob("VP_ATTN_NO_SPLIT", None)
    print(json.dumps({"label": args.label, "lib": N.LIB_PATH, "results": res}))


if __name__ == "__main__":
    main()
