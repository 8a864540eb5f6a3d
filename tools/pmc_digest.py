"""Digest rocprofv3 --pmc passes (tools/pmc_gemm.sh / tools/pmc_attn.sh outputs) into profiles/<round>_pmc_summary.json:
per-dispatch counter means for the GEMM / attention kernels and the derived figures DESIGN.md quotes.

    python tools/pmc_digest.py --round r02 --gemm gpurun_out/pmc_gemm_v11 --attn gpurun_out/pmc_attn_vbounded
    python tools/pmc_digest.py --round r02 --merge --attn8 gpurun_out/pmc_attn8   (tools/pmc_attn8.sh, config-5 shape)

mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): GRBM_GUI_ACTIVE sums the 8 XCDs, so
GRBM_GUI_ACTIVE / 8 is the kernel's cycle count at the clock the chip held (MI355X_MICROARCH.md, DVFS give-back)."""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEMM_GRIDS = {5004 * 512: "qkv 35552x9216x3072", 1668 * 512: "out 35552x3072x3072 / ff2 35552x3072x12288",
              6672 * 512: "ff1 35552x12288x3072"}


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(collections.Counter)
    for p in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            k = (name, int(r.get("Grid_Size") or 0))
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    return {k: {c: v / cnt[k][c] for c, v in dd.items()} for k, dd in agg.items()}


def derived(c, mfma_per_unit=None):
    clk = c["GRBM_GUI_ACTIVE"] / 8
    out = {"mfma_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * 1024),
           "wait_any_share_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
           "wait_inst_any_share_of_wave_cycles": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]}
    if "SQ_INSTS_MFMA" in c:
        m = c["SQ_INSTS_MFMA"]
        out["non_mfma_valu_per_mfma"] = (c["SQ_INSTS_VALU"] - m) / m
        if "SQ_INSTS_SALU" in c:
            out["salu_per_mfma"] = c["SQ_INSTS_SALU"] / m
        out["lds_insts_per_mfma"] = c["SQ_INSTS_LDS"] / m
        out["lds_bank_conflict_share"] = c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_LDS_IDX_ACTIVE"])
        if "SQ_INSTS_VALU_TRANS_F32" in c:
            out["exp_per_mfma"] = c["SQ_INSTS_VALU_TRANS_F32"] / m
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in c:
            out["valu_mfma_coexec_share_of_mfma_busy"] = c["SQ_VALU_MFMA_COEXEC_CYCLES"] / c["SQ_VALU_MFMA_BUSY_CYCLES"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r02")
    ap.add_argument("--gemm", default="")
    ap.add_argument("--attn", default="")
    ap.add_argument("--attn8", default="", help="fp8 attention passes (tools/pmc_attn8.sh: config-5 shape)")
    ap.add_argument("--merge", action="store_true", help="add to the round's existing summary instead of replacing it")
    a = ap.parse_args()
    path = os.path.join(ROOT, "profiles", f"{a.round}_pmc_summary.json")
    res = {"source": "rocprofv3 --pmc passes on tools/bench_kernels.py (config-2 shapes, random data; the fp8 "
                     "attention at config-5 shape), separate runs per counter set; per-dispatch means", "kernels": {}}
    if a.merge and os.path.exists(path):
        res["kernels"] = json.load(open(path))["kernels"]
    for d, kind in ((a.gemm, "gemm"), (a.attn, "attention"), (a.attn8, "attention")):
        if not d:
            continue
        for (name, grid), c in load(d).items():
            if kind == "gemm" and "gemm_bf16_kernel" not in name:
                continue
            if kind == "attention" and not name.startswith("attn_fwd"):
                continue
            label = f"{name} grid {grid}" + (f" ({GEMM_GRIDS[grid]})" if kind == "gemm" and grid in GEMM_GRIDS else "")
            res["kernels"][label] = {"derived": derived(c), "counters": {k: round(v) for k, v in c.items()}}
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["kernels"].items():
        print(k, {x: round(y, 3) for x, y in v["derived"].items()})


if __name__ == "__main__":
    main()
