"""Per-wave-tile view of the attention PMC passes (tools/pmc_attn.sh): python tools/pmc_attn_summary.py 3 17 ...

Counters are summed over all XCDs; SQ_*_CYCLES/ACTIVE/WAIT are quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES (cycles).
A "wave-tile" is one wave's 32 queries x one 64-key tile at config-2 shapes.
"""
import csv
import glob
import sys

B, H, N = 2, 48, 17776


def load(v):
    d = {}
    for f in glob.glob(f"gpurun_out/pmc_attn_v{v}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "attn" in r["Kernel_Name"]:
                d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(x) / len(x) for k, x in d.items()}


for v in sys.argv[1:]:
    c = load(v)
    nw = 8 if v in ("1", "2", "5", "6", "9", "10", "17") else 4
    qb = nw * 32
    wave_tiles = B * H * ((N + qb - 1) // qb) * nw * ((N + 63) // 64)
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
    simd_cycles = cyc * 1024
    print(f"variant {v}: kernel {cyc / 2.4e3:.0f} us-ish  wave-tiles {wave_tiles:.3e}")
    for k in sorted(c):
        per = c[k] / wave_tiles
        extra = ""
        if k.startswith(("SQ_ACTIVE", "SQ_WAIT", "SQ_WAVE_CYCLES", "SQ_BUSY")):
            extra = f"  ({4 * c[k] / simd_cycles:.1%} of SIMD-cycles as x4)"
        if k == "SQ_VALU_MFMA_BUSY_CYCLES":
            extra = f"  ({c[k] / simd_cycles:.1%} MFMA busy)"
        print(f"  {k:32s} {c[k]:.4e}  per wave-tile {per:9.1f}{extra}")
