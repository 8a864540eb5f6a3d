"""Build libvp_hip.so (gfx950) in-tree with hipcc — no JIT cache, so the .so travels with the repo snapshot.

    python -m videopainter_amd.build [--force]
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libvp_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# attention: no NaN semantics needed (masked scores are -inf, never NaN); without this hipcc inserts a
# canonicalising v_max before every fmaxf of an MFMA result (cdna_hip_programming.md, attention pitfalls)
# attention: -fno-slp-vectorize keeps the softmax row sums as single f32 adds — the SLP pass packs them into
# v_pk_add_f32, which costs more issue cycles beside MFMAs (MI355X_MICROARCH.md cycle constants): measured
# 1.07 -> 1.13 PF/s at config 2 (an interleaved bench A/B, tools/gpu.sh).  The GEMM keeps SLP (no gain there: the epilogue is not under MFMA).
# attention: -amdgpu-mfma-vgpr-form keeps the MFMA accumulators of the one-wave-per-SIMD kernel (p1, 512 registers
# available) in arch VGPRs; by default the compiler picks the AGPR form there and shuttles every S tile through
# v_accvgpr_read for the softmax (the other attention kernels compile to identical code with or without it).
PER_FILE_FLAGS = {"attention.hip": ["-fno-honor-nans", "-Wno-inline-asm", "-fno-slp-vectorize", "-mllvm",
                                    "-amdgpu-mfma-vgpr-form"],
                  "gemm.hip": ["-Wno-inline-asm"],
                  # attention backward: without SLP the dS products stay single v_mul_f32 (the pairing into
                  # v_pk_mul_f32 cost a v_mov per operand pair beside the MFMAs): 12.50 -> 12.01 ms per training-shape
                  # call, bit-identical arithmetic (profiles/r06_attn_bwd_noslp_ab.log)
                  "attention_bwd.hip": ["-fno-slp-vectorize"]}
CFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-result",
          "-Wno-unused-function", "-munsafe-fp-atomics"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def source_digest() -> str:
    """sha256 of the sources, headers and flags (repo-relative paths: the GPU box's checkout path differs)."""
    h = hashlib.sha256()
    for p in _sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "vp_hip.h"),
                                                                          os.path.join(ROOT, "include",
                                                                                       "vp_hip_diag.h")]:
        with open(p, "rb") as f:
            h.update(os.path.relpath(p, ROOT).encode())  # relative: the GPU box's checkout path differs
            h.update(f.read())
    h.update(" ".join(CFLAGS).encode())
    h.update(repr(sorted(PER_FILE_FLAGS.items())).encode())
    return h.hexdigest()


def compiler_digest() -> str:
    r = subprocess.run([HIPCC, "--version"], capture_output=True, text=True)
    return hashlib.sha256((r.stdout + r.stderr).encode()).hexdigest()[:16]


def _digest() -> str:
    return source_digest() + ":" + compiler_digest()


def build(force: bool = False, verbose: bool = True, out: str = LIB, extra_flags=None) -> str:
    """out / extra_flags ({file: [flags]}) build an A/B copy of the library (VP_HIP_LIB selects it at load time)."""
    libdir = os.path.dirname(out)
    os.makedirs(libdir, exist_ok=True)
    # the stamp is a local cache (git-ignored): a checkout that changes csrc/ changes source_digest() and rebuilds;
    # _native.lib() also compares the digest compiled INTO the library with the sources at load time
    stamp = os.path.join(libdir, os.path.basename(out).replace(".so", ".sha256"))
    dg = _digest()
    if extra_flags:
        dg += ":" + hashlib.sha256(repr(sorted(extra_flags.items())).encode()).hexdigest()[:16]
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read().strip() == dg:
        return out
    objs = []
    # objects in a private directory per build: two builds into one libdir (e.g. an A/B copy with extra flags next
    # to the default library) must not link each other's objects
    objdir = tempfile.mkdtemp(dir=libdir, prefix=".obj-" + os.path.basename(out) + "-")

    def cc(src):
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        extra = PER_FILE_FLAGS.get(os.path.basename(src), []) + (extra_flags or {}).get(os.path.basename(src), [])
        cmd = [HIPCC, *CFLAGS, *extra, f'-DVP_BUILD_DIGEST="{dg}"', "-I", os.path.join(ROOT, "include"), "-c", src,
               "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        return obj

    jobs = max(1, min(len(_sources()), int(os.environ.get("MAX_JOBS", "8"))))
    try:
        with cf.ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(cc, _sources()))
        tmp = os.path.join(objdir, os.path.basename(out))
        r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    with open(stamp, "w") as f:
        f.write(dg)
    if verbose:
        print(f"[videopainter_amd] built {out}")
    return out


if __name__ == "__main__":
    # python -m videopainter_amd.build [--force] [--diag] [--out PATH] [--extra FILE:FLAG ...]
    args = sys.argv[1:]
    o, ex = LIB, {}
    for i, a in enumerate(args):
        if a == "--out":
            o = os.path.abspath(args[i + 1])
        if a == "--extra":
            f, fl = args[i + 1].split(":", 1)
            ex.setdefault(f, []).append(fl)
    if "--diag" in args:  # the diagnostic entry points (include/vp_hip_diag.h) in a library of their own
        o = o if "--out" in args else os.path.join(LIBDIR, "libvp_hip_diag.so")
        for f in ("attention.hip", "gemm.hip"):
            ex.setdefault(f, []).append("-DVP_DIAG=1")
    build(force="--force" in args, out=o, extra_flags=ex)
