"""Compare the device ISA of every kernel two assembly dumps have in common (hipcc --cuda-device-only -S):
a source refactor that must not change the shipped kernels is checked by 'identical' here (kernels renamed by the
refactor are matched to a kernel of the first dump with the identical body).

    python tools/isa_diff.py before.s after.s
"""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):\s*(;.*)?$", line)
        if m and cur is None and not line.startswith(".L"):
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                out[cur] = [l for l in body if not l.strip().startswith(";") and ".loc" not in l
                            and not l.strip().startswith((".section", ".amdhsa_kernel"))]  # (names only)
                cur = None
            else:
                body.append(re.sub(r"\s*;.*$", "", re.sub(r"\.LBB\d+_", ".LBB_", line)))  # (comments: block numbers)
    return out


a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
common = sorted(set(a) & set(b))
same = [k for k in common if a[k] == b[k]]
diff = [k for k in common if a[k] != b[k]]
print(f"{len(a)} / {len(b)} functions, {len(common)} common: {len(same)} identical, {len(diff)} differ; "
      f"only before: {len(set(a) - set(b))}, only after: {len(set(b) - set(a))}")
for k in diff:
    print("DIFFERS", k[:160])
# renamed kernels (a template parameter dropped): matched by identical bodies
bodies = {tuple(v): k for k, v in a.items()}
unmatched = 0
for k in sorted(set(b) - set(a)):
    twin = bodies.get(tuple(b[k]))
    print("NEW", k[:110], "== body of", twin[:110] if twin else "NOTHING (new code)")
    unmatched += twin is None
sys.exit(1 if diff or unmatched else 0)
