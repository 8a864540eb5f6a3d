"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace (host-side stalls: syncs, CPU work while the
GPU waits).  usage: python tools/trace_gaps.py <kernel_trace.csv> [min_gap_us]"""
import csv
import sys


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    gaps = []
    for a, b in zip(rows, rows[1:]):
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if g >= min_us:
            gaps.append((g, a["Kernel_Name"][:70], b["Kernel_Name"][:70]))
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows) / 1e6
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
    print(f"{len(rows)} dispatches, busy {busy:.1f} ms over a span of {span:.1f} ms; {len(gaps)} gaps >= {min_us} us")
    for g, a, b in sorted(gaps, reverse=True)[:30]:
        print(f"{g:10.1f} us  {a}  ->  {b}")


if __name__ == "__main__":
    main()
