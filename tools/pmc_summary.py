"""Summarise rocprofv3 outputs into profiles/<round>_*.{csv,json,md}.

    python tools/pmc_summary.py --round r01 --prof gpurun_out/prof --fetch gpurun_out/pmc_fetch \
        --write gpurun_out/pmc_write

HBM traffic per attention launch, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced stream, so
    traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(WRITE_SIZE is exact for 16 B/lane stores).  Infinity-Cache hits are counted in FETCH_SIZE.
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, counter, kernel_substr):
    """Per attention CALL: one call = the main grid + (when the grid-tail split is active) the split grid and the
    merge kernel, so the counter is summed over every dispatch of the call and divided by the number of main-grid
    dispatches (the largest grid)."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and
            (kernel_substr in r["Kernel_Name"] or "attn_combine" in r["Kernel_Name"])]
    if not rows:
        return 0.0, 0
    grid = lambda r: int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)  # noqa: E731
    gmax = max(grid(r) for r in rows if kernel_substr in r["Kernel_Name"])
    calls = sum(1 for r in rows if kernel_substr in r["Kernel_Name"] and grid(r) == gmax)
    return sum(float(r["Counter_Value"]) for r in rows) / max(1, calls), calls


def dispatch_breakdown(trace, kernel_substr):
    """Mean duration (ms) per call of each dispatch kind from a kernel trace: main grid, tail split, merge."""
    rows = [r for r in csv.DictReader(open(trace)) if kernel_substr in r["Kernel_Name"] or
            "attn_combine" in r["Kernel_Name"]]
    if not rows:
        return {}
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
    grid = lambda r: int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)  # noqa: E731
    att = [r for r in rows if kernel_substr in r["Kernel_Name"]]
    gmax = max(grid(r) for r in att)
    main = [dur(r) for r in att if grid(r) == gmax]
    split = [dur(r) for r in att if grid(r) != gmax]
    comb = [dur(r) for r in rows if "attn_combine" in r["Kernel_Name"]]
    mean = lambda v: sum(v) / len(v) if v else 0.0  # noqa: E731
    n = max(1, len(main))
    return {"calls": len(main), "main_ms": mean(main), "split_ms": sum(split) / n, "merge_ms": sum(comb) / n,
            "per_call_ms": (sum(main) + sum(split) + sum(comb)) / n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--prof", default="gpurun_out/prof")
    ap.add_argument("--fetch", default="gpurun_out/pmc_fetch")
    ap.add_argument("--write", default="gpurun_out/pmc_write")
    ap.add_argument("--kernel", default="attn_fwd_dma")
    ap.add_argument("--algorithmic-bytes", type=float, default=4 * 2 * 17776 * 3072 * 2.0,
                    help="Q+K+V+O bytes per config-2 attention launch")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(a.prof, "bench_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out, f"{a.round}_bench_kernel_stats.csv"))
        shutil.copy(os.path.join(a.prof, "bench_domain_stats.csv"), os.path.join(out, f"{a.round}_bench_domain_stats.csv"))
    res = {}
    f = os.path.join(a.fetch, "attn_counter_collection.csv")
    w = os.path.join(a.write, "attn_counter_collection.csv")
    if os.path.exists(f) and os.path.exists(w):
        fk, nf = counters(f, "FETCH_SIZE", a.kernel)
        wk, nw = counters(w, "WRITE_SIZE", a.kernel)
        traffic = (2 * fk + wk) * 1024
        res = {"kernel": a.kernel, "calls_fetch": nf, "calls_write": nw,
               "FETCH_SIZE_KiB_raw": fk, "WRITE_SIZE_KiB": wk, "traffic_bytes_per_launch": traffic,
               "algorithmic_bytes_per_launch": a.algorithmic_bytes,
               "traffic_over_algorithmic": traffic / a.algorithmic_bytes,
               "correction": "traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE reads 1/2 of 16B/lane "
                             "streams; MI355X_MICROARCH.md §HBM)"}
        trace = os.path.join(a.prof, "bench_kernel_trace.csv")
        if os.path.exists(trace):
            res["step_dispatches"] = dispatch_breakdown(trace, a.kernel)
        for src, name in ((f, "fetch"), (w, "write")):
            rows = [r for r in csv.DictReader(open(src)) if a.kernel in r["Kernel_Name"] or
                    "attn_combine" in r["Kernel_Name"]]
            with open(os.path.join(out, f"{a.round}_attn_pmc_{name}.csv"), "w", newline="") as fo:
                wr = csv.DictWriter(fo, fieldnames=list(rows[0].keys()))
                wr.writeheader()
                wr.writerows(rows)
        with open(os.path.join(out, f"{a.round}_attention_traffic.json"), "w") as fo:
            json.dump(res, fo, indent=2)
    print(json.dumps(res, indent=2))


if __name__ == "__main__":
    main()
