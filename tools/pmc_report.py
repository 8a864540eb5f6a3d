"""One kernel's PMC passes as a text report: every counter averaged over the kernel's dispatches, the clock the chip
held (GRBM_GUI_ACTIVE / 8 / dispatch wall time, MI355X_MICROARCH.md 'DVFS give-back'), per-MFMA instruction mixes
and the wave-cycle shares (SQ_WAIT_ANY = parked in s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stalls,
SQ_ACTIVE_INST_ANY = issuing; the three add up to SQ_WAVE_CYCLES).

    python tools/pmc_report.py --dir gpurun_out/pmc_b_p2 --kernel attn_fwd_p1 --exclude Lb1E [--out profiles/x.txt]
"""
import argparse
import collections
import csv
import glob
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--exclude", default="", help="comma-separated substrings that drop a dispatch")
    ap.add_argument("--out", default="")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    excl = [e for e in a.exclude.split(",") if e]
    vals = collections.defaultdict(list)
    ns = []
    names = set()
    for f in sorted(glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True)):
        seen = set()
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if a.kernel not in n or any(e in n for e in excl):
                continue
            names.add(n.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", ""))
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "End_Timestamp" in r and r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                ns.append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"]), float(r["Counter_Value"])))
    c = {k: statistics.mean(v) for k, v in vals.items()}
    lines = [a.title or f"PMC report: {a.dir} kernel~{a.kernel}", "kernels: " + "; ".join(sorted(names))]
    gui = c.get("GRBM_GUI_ACTIVE")
    if ns:
        clk = [g / 8 / t for t, g in ns if t > 0]
        lines.append(f"dispatch wall time mean {statistics.mean(t for t, _ in ns) / 1e6:.3f} ms over {len(ns)} dispatches; "
                     f"clock = GRBM_GUI_ACTIVE / 8 / wall = {statistics.mean(clk):.3f} GHz (min {min(clk):.3f}, "
                     f"max {max(clk):.3f})")
    simd = gui / 8 * 1024 if gui else None  # SIMD-cycles: 256 CUs x 4 SIMDs, GUI summed over the 8 XCDs
    mf = c.get("SQ_INSTS_MFMA")
    wave = c.get("SQ_WAVE_CYCLES")
    for k in sorted(c):
        extra = ""
        if wave and k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            extra = f"  share of wave-cycles {c[k] / wave:.3f}"
        if simd and k == "SQ_VALU_MFMA_BUSY_CYCLES":
            extra = f"  MFMA busy = /SIMD-cycles {c[k] / simd:.3f}"
        if simd and k == "SQ_VALU_MFMA_COEXEC_CYCLES":
            extra = f"  /SIMD-cycles {c[k] / simd:.3f}"
        if simd and k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_BUSY_CYCLES"):
            extra = f"  x4/SIMD-cycles {4 * c[k] / simd:.3f}"
        if mf and k.startswith("SQ_INSTS") and k != "SQ_INSTS_MFMA":
            extra = f"  per MFMA {c[k] / mf:.3f}"
        lines.append(f"  {k:30s} {c[k]:.4e}{extra}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
