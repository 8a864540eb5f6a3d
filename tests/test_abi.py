"""The C-ABI library builds, loads and exports every symbol include/vp_hip.h declares (CPU-only: no compute)."""
import os
import re

from videopainter_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "vp_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|void|int64_t|const char\*)\s+(vp_\w+)\(", src, flags=re.M)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(N.EXPORTS)


def test_library_loads_and_exports_everything():
    from videopainter_amd.build import build
    build(verbose=False)
    L = N.lib()  # checks ABI version and descriptor struct sizes against ctypes
    for name in header_functions():
        assert hasattr(L, name), name
    assert L.vp_abi_version() == N.ABI_VERSION


def test_default_library_exports_no_diagnostic_symbols():
    """include/vp_hip_diag.h's entry points (MFMA layout probes) exist only in the --diag build: the default library
    exports exactly the header's functions, and the diagnostic header declares exactly the diagnostic bindings."""
    import subprocess
    L = N.lib()
    if os.environ.get("VP_HIP_LIB"):
        return  # (an A/B or diagnostic library was selected explicitly)
    for name in N.DIAG_SIGS:
        assert not hasattr(L, name), name
    src = open(os.path.join(ROOT, "include", "vp_hip_diag.h")).read()
    assert sorted(re.findall(r"^int\s+(vp_\w+)\(", src, flags=re.M)) == sorted(N.DIAG_SIGS)
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (vp_\w+)$", out, flags=re.M)))
    assert exported == header_functions()


def test_descriptor_argument_errors_are_reported_without_a_gpu():
    import ctypes as C
    L = N.lib()
    d = N.GemmDesc()  # all-zero descriptor: rejected on the host before any launch
    assert L.vp_gemm_bf16(C.byref(d), None) == 1000
    a = N.AttnDesc()
    a.head_dim = 128
    a.Q = a.K = a.V = a.O = 1
    assert L.vp_attention_fwd_bf16(C.byref(a), None) == 1001
