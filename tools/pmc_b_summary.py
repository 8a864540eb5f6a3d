"""Summary of tools/pmc_attn_p1.sh passes: python tools/pmc_b_summary.py w64 p1 (main attention grid only)."""
import csv
import glob
import sys


def load(v):
    d = {}
    for f in glob.glob(f"gpurun_out/pmc_b_{v}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "attn_fwd" in n and "Lb1E" not in n.split("attn_fwd")[1][:12]:
                d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(x) / len(x) for k, x in d.items()}


for v in sys.argv[1:]:
    c = load(v)
    gui = c.get("GRBM_GUI_ACTIVE", 0)
    simd = gui / 8 * 1024  # SIMD-cycles (gui counts per XCD ... summed over 8 XCDs)
    mf = c.get("SQ_INSTS_MFMA", 1)
    print(f"== {v}: GRBM_GUI_ACTIVE {gui:.4e}")
    for k in sorted(c):
        extra = ""
        if k.startswith(("SQ_ACTIVE", "SQ_WAIT", "SQ_WAVE_CYCLES", "SQ_BUSY")):
            extra = f"  x4/SIMD-cycles {4 * c[k] / simd:.3f}"
        if k == "SQ_VALU_MFMA_BUSY_CYCLES":
            extra = f"  /SIMD-cycles {c[k] / simd:.3f}"
        if k.startswith("SQ_INSTS"):
            extra = f"  per MFMA {c[k] / mf:.3f}"
        print(f"  {k:30s} {c[k]:.4e}{extra}")
