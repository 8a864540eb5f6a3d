"""Per-shape GEMM durations in a rocprofv3 kernel trace of bench.py (config 2): dispatches of gemm_bf16_kernel are
told apart by grid size (256 x 256 tiles: QKV 139 x 36, out / FF2 139 x 12, FF1 139 x 48; the branch / patch /
proj_out GEMMs are listed by their own grids).  usage: python tools/gemm_shapes.py <kernel_trace.csv> [...]"""
import collections
import csv
import sys

M = 2 * 17776
SHAPES = {139 * 36: ("qkv", M * 9216 * 3072 * 2), 139 * 48: ("ff1", M * 12288 * 3072 * 2)}


def main():
    for path in sys.argv[1:]:
        rows = [r for r in csv.DictReader(open(path)) if "gemm_bf16_kernel" in r["Kernel_Name"]]
        by = collections.defaultdict(list)
        for r in rows:
            grid = int(r.get("Grid_Size") or r.get("Grid_Size_X")) // int(r.get("Workgroup_Size") or
                                                                          r.get("Workgroup_Size_X"))
            by[(r["Kernel_Name"].split("(")[0][-40:], grid)].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        print(path)
        tot = 0.0
        for (name, grid), d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            ms = sum(d) / len(d)
            tot += sum(d)
            lab, fl = SHAPES.get(grid, (f"grid {grid}", None))
            extra = f"  {fl / ms / 1e9:.0f} TF/s" if fl else ""
            print(f"  {name:40s} {lab:12s} n={len(d):4d} mean {ms:.3f} ms  total {sum(d):.1f} ms{extra}")
        print(f"  all GEMM dispatches: {tot:.1f} ms")


if __name__ == "__main__":
    main()
