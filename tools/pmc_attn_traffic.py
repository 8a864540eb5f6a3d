"""HBM traffic per attention CALL from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes: the sum over every
dispatch of the call's kernels (bf16: main grid + grid-tail split + merge + the redo launch of p2a; fp8: the one
kernel) divided by the number of calls (= dispatches of the main kernel).

    python tools/pmc_attn_traffic.py --fetch D1 --write D2 --kernels attn_fwd_p1,attn_combine,attn_fwd_s16 \
        --main attn_fwd_p1 --algorithmic 873725952 --what "..." --out profiles/r04_attention_traffic.json

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE in KiB, FETCH_SIZE counts half the bytes of a wide coalesced
stream on gfx950: traffic = (2 FETCH_SIZE + WRITE_SIZE) x 1024 (Infinity-Cache hits included in FETCH_SIZE)."""
import argparse
import csv
import glob
import json
import os


def collect(d, counter, kernels, main):
    tot, calls, per = 0.0, 0, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if r["Counter_Name"] != counter or not any(k in n for k in kernels):
                continue
            v = float(r["Counter_Value"])
            tot += v
            key = n.split("(")[0][-60:]
            per[key] = per.get(key, 0.0) + v
            if main in n:
                calls += 1
    return tot, calls, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernels", required=True)
    ap.add_argument("--main", required=True)
    ap.add_argument("--algorithmic", type=float, required=True)
    ap.add_argument("--what", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ks = a.kernels.split(",")
    f, nf, pf = collect(a.fetch, "FETCH_SIZE", ks, a.main)
    w, nw, pw = collect(a.write, "WRITE_SIZE", ks, a.main)
    if nf == 0 or nw == 0:
        raise SystemExit("no dispatches of the main kernel found")
    t = (2 * f / nf + w / nw) * 1024
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on {a.kernels}",
           "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 per call (MI355X_MICROARCH.md HBM correction)",
           "calls": [nf, nw], "fetch_kib_per_kernel": pf, "write_kib_per_kernel": pw, "what": a.what,
           "traffic_bytes_per_launch": t, "algorithmic_bytes_per_launch": a.algorithmic,
           "traffic_over_algorithmic": t / a.algorithmic}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
