"""Effective clock and MFMA-busy share per kernel from tools/pmc_clock.sh: clock = GRBM_GUI_ACTIVE / 8 (the counter
sums the 8 XCDs) / dispatch wall time (MI355X_MICROARCH.md 'DVFS give-back'); the kernel's bf16 / fp8 dense peak AT
that clock = peak x clock / 2.4 GHz.  Writes profiles/<round>_kernel_clocks.json.

    python tools/pmc_clock_summary.py --round r02
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = ("gemm_bf16_kernel", "attn_fwd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r02")
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out", "pmc_clock"))
    a = ap.parse_args()
    res = {"source": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace on tools/bench_kernels.py "
                     "(random data; config-2 shapes, fp8 attention at config-5 shape); profiled passes run a few % "
                     "below the un-profiled clock", "formula": "clock_ghz = GRBM_GUI_ACTIVE / 8 / wall_ns",
           "kernels": {}}
    for sub in ("gemm", "attn", "attn8"):
        per = collections.defaultdict(list)
        for f in glob.glob(os.path.join(a.dir, sub, "**", "*counter_collection.csv"), recursive=True):
            rows = list(csv.DictReader(open(f)))
            by = collections.defaultdict(dict)
            for r in rows:
                if not any(k in r["Kernel_Name"] for k in KEEP):
                    continue
                key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0],
                       int(r.get("Grid_Size") or 0), r["Dispatch_Id"])
                by[key][r["Counter_Name"]] = float(r["Counter_Value"])
                by[key]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) \
                    if "End_Timestamp" in r else by[key].get("_ns")
            for (name, grid, _), c in by.items():
                per[(name, grid)].append(c)
        for (name, grid), cs in per.items():
            clk = [c["GRBM_GUI_ACTIVE"] / 8 / c["_ns"] for c in cs if c.get("_ns")]
            busy = [c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024) for c in cs]
            res["kernels"][f"{name} grid {grid}"] = {
                "dispatches": len(cs), "clock_ghz_median": statistics.median(clk) if clk else None,
                "wall_ms_median": statistics.median(c["_ns"] for c in cs) / 1e6 if clk else None,
                "mfma_busy_frac_median": statistics.median(busy)}
    path = os.path.join(ROOT, "profiles", f"{a.round}_kernel_clocks.json")
    json.dump(res, open(path, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(k, v)


if __name__ == "__main__":
    main()
