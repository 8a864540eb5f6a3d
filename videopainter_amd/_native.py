"""ctypes binding of libvp_hip.so (the C ABI declared in include/vp_hip.h).

This is the only place Python touches the native library.  There is no fallback: if the library is missing or was
built against a different ABI, `lib()` raises — the product path never silently runs a non-HIP implementation.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VP_HIP_LIB", os.path.join(_HERE, "_lib", "libvp_hip.so"))
ABI_VERSION = 20

vp = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
f32 = C.c_float


class GemmDesc(C.Structure):
    _fields_ = [("M", i32), ("N", i32), ("K", i32), ("epilogue", i32),
                ("A", vp), ("lda", i64),
                ("W", vp * 3), ("bias", vp * 3),
                ("n_seg", i32), ("pad0", i32),
                ("C", vp), ("ldc", i64),
                ("rows_per_group", i32), ("pad1", i32),
                ("group_stride", i64), ("row_offset", i64),
                ("alpha", f32), ("pad2", i32),
                ("R", vp), ("ldr", i64), ("gate", vp), ("gate_text", vp), ("gate_bstride", i64),
                ("tokens_per_batch", i32), ("text_len", i32),
                ("inject", vp), ("inject_ld", i64), ("inject_bstride", i64), ("inject_mask", vp),
                ("inject_mask_bstride", i64),
                ("addrows", vp), ("addrows_ld", i64), ("addrows_offset", i64),
                ("qk_ln_w", vp * 2), ("qk_ln_b", vp * 2), ("qk_eps", f32 * 2), ("rope_cos", vp), ("rope_sin", vp),
                ("a_tail_k", i32), ("pad3", i32), ("a_tail_off", i64 * 3), ("rope_ax", vp * 6), ("rope_hw", i32),
                ("rope_w", i32), ("rope_mhw", C.c_uint32), ("rope_mw", C.c_uint32), ("aux", vp), ("ld_aux", i64)]


class AttnDesc(C.Structure):
    _fields_ = [("B", i32), ("H", i32), ("Nq", i32), ("head_dim", i32),
                ("Q", vp), ("q_sb", i64), ("q_sn", i64),
                ("K", vp), ("V", vp), ("k_sb", i64), ("k_sn", i64), ("v_sb", i64), ("v_sn", i64),
                ("Nk", i32), ("Nk2", i32),
                ("K2", vp), ("V2", vp), ("k2_sb", i64), ("k2_sn", i64), ("v2_sb", i64), ("v2_sn", i64),
                ("O", vp), ("o_sb", i64), ("o_sn", i64),
                ("scale", f32), ("out_scale", f32), ("accumulate", i32), ("flags", i32), ("lse", vp),
                ("k2_full", vp), ("k2_len", vp), ("l_extra", vp)]


class GemmMxDesc(C.Structure):
    _fields_ = [("base", GemmDesc), ("a_scale", vp), ("w_scale", vp * 3), ("c_scale", vp)]


class AttnFp8Desc(C.Structure):
    _fields_ = [("base", AttnDesc), ("vs", vp), ("npad", i32), ("qk_scale", i32)]


class DpmDesc(C.Structure):
    _fields_ = [("n", i64), ("noise_pred", vp), ("do_cfg", i32), ("guidance", f32), ("model_output", vp),
                ("sample", vp), ("old_pred", vp), ("pred_out", vp), ("noise1", vp), ("noise2", vp),
                ("second_order", i32), ("replace_gt", i32),
                ("sa", f32), ("sb", f32), ("m1", f32), ("m2", f32), ("mn", f32), ("m3", f32), ("m4", f32),
                ("gt_add_noise", i32), ("mask_background", i32),
                ("gt", vp), ("gt_noise", vp), ("mask", vp), ("gsa", f32), ("gsb", f32), ("latents_out", vp),
                ("prev_out", vp)]


CONV_MAX_T = 128


class Conv3dDesc(C.Structure):
    _fields_ = [("B", i32), ("Cin", i32), ("Cout", i32), ("Tout", i32), ("Hout", i32), ("Wout", i32),
                ("Hin", i32), ("Win", i32), ("kt", i32), ("kh", i32), ("kw", i32), ("sh", i32), ("sw", i32),
                ("ph", i32), ("pw", i32), ("uh", i32), ("uw", i32), ("x_frames", i32), ("hist_frames", i32),
                ("ldy", i32), ("ldr", i32), ("tmap", i32 * CONV_MAX_T),
                ("x", vp), ("hist", vp), ("w", vp), ("bias", vp), ("resid", vp), ("y", vp)]


class AttnBwdDesc(C.Structure):
    _fields_ = [("B", i32), ("H", i32), ("Nq", i32), ("Nk", i32), ("head_dim", i32), ("pad0", i32),
                ("Q", vp), ("q_sb", i64), ("q_sn", i64), ("K", vp), ("k_sb", i64), ("k_sn", i64),
                ("V", vp), ("v_sb", i64), ("v_sn", i64), ("O", vp), ("o_sb", i64), ("o_sn", i64),
                ("dO", vp), ("do_sb", i64), ("do_sn", i64), ("lse", vp), ("delta", vp),
                ("dQ", vp), ("dq_sb", i64), ("dq_sn", i64), ("dK", vp), ("dk_sb", i64), ("dk_sn", i64),
                ("dV", vp), ("dv_sb", i64), ("dv_sn", i64), ("scale", f32), ("pad1", i32)]


(EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_SCALE, EPI_GATED, EPI_BIAS_ADDROWS, EPI_BIAS_GELU_MXFP8, EPI_BIAS_QKNORM_ROPE,
 EPI_GELU_BWD) = range(8)

# name -> (restype, argtypes)
_SIGS = {
    "vp_abi_version": (i32, []),
    "vp_build_digest": (C.c_char_p, []),
    "vp_set_knob": (i32, [C.c_char_p, C.c_char_p]),
    "vp_struct_sizes": (None, [C.POINTER(i64)]),
    "vp_gemm_bf16": (i32, [C.POINTER(GemmDesc), vp]),
    "vp_gemm_bf16_workspace_bytes": (i64, [C.POINTER(GemmDesc)]),
    "vp_gemm_bf16_ws": (i32, [C.POINTER(GemmDesc), vp, i64, vp]),
    "vp_gemm_mx_fp8": (i32, [C.POINTER(GemmMxDesc), vp]),
    "vp_mx_scale_bytes": (i64, [i64, i64]),
    "vp_mx_quantize_bf16": (i32, [vp, i64, vp, i64, vp, i32, i32, vp]),
    "vp_adaln_modulate_mx_fp8": (i32, [vp, vp, vp, i32, i32, i32, i32, vp, vp, f32, vp, i64, vp]),
    "vp_attention_fwd_bf16": (i32, [C.POINTER(AttnDesc), vp]),
    "vp_attention_fwd_fp8": (i32, [C.POINTER(AttnFp8Desc), vp]),
    "vp_attention_fp8_workspace_bytes": (i64, [C.POINTER(AttnFp8Desc)]),
    "vp_attention_fwd_fp8_ws": (i32, [C.POINTER(AttnFp8Desc), vp, i64, vp]),
    "vp_attention_workspace_bytes": (i64, [C.POINTER(AttnDesc)]),
    "vp_attention_fwd_bf16_ws": (i32, [C.POINTER(AttnDesc), vp, i64, vp]),
    "vp_attention_variant_built": (i32, [C.c_char_p]),
    "vp_gemm_variant_built": (i32, [i32]),
    "vp_v_pack_fp8_bytes": (i64, [i32, i32, i32, C.POINTER(i64), C.POINTER(i64)]),
    "vp_v_pack_fp8": (i32, [vp, i64, i64, i32, i32, i32, vp, vp, vp]),
    "vp_head_norm_rope_fp8": (i32, [vp, i64, i64, vp, i64, i64, i32, i32, i32, i32, vp, vp, f32, vp, vp, f32, vp]),
    "vp_adaln_modulate_bf16": (i32, [vp, vp, i64, i32, i32, i32, i32, vp, vp, f32, vp, i64, vp]),
    "vp_head_norm_rope_bf16": (i32, [vp, i64, i64, vp, i64, i64, i32, i32, i32, i32, vp, vp, f32, vp, vp, vp, i64,
                                     f32, vp, vp]),
    "vp_mask_scale_rows_bf16": (i32, [vp, i64, i64, vp, i64, i64, i32, i32, i32, vp, i64, f32, vp, vp]),
    "vp_partition_rows_index": (i32, [vp, i64, i32, i32, vp, vp, vp]),
    "vp_mask_null_segments": (i32, [vp, i64, i32, i32, i32, i32, i32, vp, vp, vp]),
    "vp_null_key_mass_lds_bytes": (i64, [i32, i32, i32]),
    "vp_null_key_mass": (i32, [vp, i64, i64, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i64,
                               vp, vp, f32, vp, vp]),
    "vp_final_norm_bf16": (i32, [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, f32, vp, i64, vp]),
    "vp_linear_small_bf16": (i32, [vp, i64, vp, vp, vp, i64, i32, i32, i32, i32, i32, vp]),
    "vp_timestep_embedding_bf16": (i32, [vp, vp, i32, i32, f32, vp]),
    "vp_patchify_bf16": (i32, [vp, i32, vp, i32, vp, i32, i32, i32, i32, i32, i32, vp]),
    "vp_patch_mask": (i32, [vp, i32, vp, i32, i32, i32, i32, i32, vp]),
    "vp_unpatchify_bf16": (i32, [vp, i64, vp, i32, i32, i32, i32, i32, i32, vp]),
    "vp_guide_rows_bf16": (i32, [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, vp, i64, i32, i32, i32, vp]),
    "vp_dpm_step_bf16": (i32, [C.POINTER(DpmDesc), vp]),
    "vp_fill_normal_bf16": (i32, [vp, i64, C.c_uint64, f32, f32, vp]),
    "vp_conv3d_bf16": (i32, [C.POINTER(Conv3dDesc), vp]),
    "vp_group_norm_workspace_floats": (i64, [i32, i32]),
    "vp_group_norm_stats": (i32, [vp, i32, i64, i32, i32, f32, vp, vp, vp]),
    "vp_group_norm_apply_bf16": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, i32, i32,
                                       C.POINTER(i32), i32, vp]),
    "vp_time_pool2_bf16": (i32, [vp, vp, i32, i32, i64, i32, vp]),
    "vp_ncdhw_to_ndhwc_bf16": (i32, [vp, i32, vp, i32, i32, i32, i32, i32, i32, vp]),
    "vp_ndhwc_to_ncdhw_bf16": (i32, [vp, i32, vp, i32, i32, i32, i32, i32, i32, vp]),
    "vp_latent_dist_bf16": (i32, [vp, i32, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "vp_tile_blend_bf16": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
    "vp_embedding_gather_bf16": (i32, [vp, vp, vp, i32, i32, i32, vp]),
    "vp_rms_norm_bf16": (i32, [vp, vp, vp, i32, i32, f32, vp]),
    "vp_mul_bf16": (i32, [vp, vp, vp, i64, vp]),
    "vp_t5_attention_bf16": (i32, [vp, i64, i32, i32, i32, i32, vp, vp, vp, vp, i64, vp]),
    "vp_scale_bf16": (i32, [vp, vp, i64, f32, vp]),
    "vp_mask_video_bf16": (i32, [vp, i32, vp, i32, vp, i32, i32, i64, vp]),
    "vp_nearest_resize3d_bf16": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
    "vp_denormalize_bf16": (i32, [vp, vp, i64, vp]),
    "vp_attention_bwd_bf16": (i32, [C.POINTER(AttnBwdDesc), vp]),
    "vp_attention_bwd_workspace_bytes": (i64, [C.POINTER(AttnBwdDesc)]),
    "vp_attention_bwd_bf16_ws": (i32, [C.POINTER(AttnBwdDesc), vp, i64, vp]),
    "vp_transpose_bf16": (i32, [vp, i64, i64, vp, i64, i64, i32, i32, i32, vp]),
    "vp_colsum_bf16": (i32, [vp, i64, vp, i64, i32, i32, i32, i32, vp, vp]),
    "vp_adaln_bwd_bf16": (i32, [vp, vp, vp, i32, i32, i32, i32, vp, vp, f32, vp, i64, i32, i32, i32, i32, vp, vp, vp,
                                vp]),
    "vp_rowscale_bf16": (i32, [vp, i64, vp, i64, i32, i32, i32, i32, vp, i64, i32, i32, vp]),
    "vp_gelu_bf16": (i32, [vp, vp, i64, vp]),
    "vp_gelu_bwd_bf16": (i32, [vp, vp, vp, i64, vp]),
    "vp_axpy_bf16": (i32, [vp, vp, f32, vp, i64, vp]),
    "vp_silu_bf16": (i32, [vp, vp, i64, vp]),
    "vp_silu_bwd_bf16": (i32, [vp, vp, vp, i64, vp]),
    "vp_head_norm_rope_bwd_bf16": (i32, [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, i32, i32, i32, vp, vp, f32, vp,
                                         vp, vp, vp, vp]),
}

EXPORTS = tuple(_SIGS)
# include/vp_hip_diag.h: only in a library built with -DVP_DIAG=1 (python -m videopainter_amd.build --diag)
DIAG_SIGS = {
    "vp_mx_mfma_probe": (i32, [vp, vp, vp, vp, vp, vp]),
    "vp_mx_mfma_probe32": (i32, [vp, vp, vp, vp, vp, vp]),
}

# the library's A/B knobs (vp_set_knob): read from the environment once at load; knob_values mirrors them
KNOBS = ("VP_GEMM_VARIANT", "VP_GEMM_NO_TAIL", "VP_GEMM_GROUP", "VP_GEMM8_VARIANT", "VP_ATTN_BOUNDED_MODE",
         "VP_ATTN_UNBOUNDED_MODE", "VP_ATTN_NO_SPLIT", "VP_ATTN8_VARIANT", "VP_T5_ATTN", "VP_CONV_HOIST", "VP_CONV_PIPE",
         "VP_ATTN_BWD_VARIANT", "VP_ATTN_TAIL", "VP_ATTN_PERSIST")
knob_values: dict = {}

_lib = None
_lock = threading.Lock()


class HipLibraryError(RuntimeError):
    pass


def lib():
    """Load (once) and return the native library; raise if it is missing or ABI-incompatible."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HipLibraryError(f"{LIB_PATH} not found: build it with `python -m videopainter_amd.build` "
                                  "(the HIP path has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in DIAG_SIGS.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
        if L.vp_abi_version() != ABI_VERSION:
            raise HipLibraryError(f"libvp_hip ABI {L.vp_abi_version()} != {ABI_VERSION}; rebuild")
        built = (L.vp_build_digest() or b"").decode()
        src = _source_digest()
        if src is not None and built.split(":")[0] != src:
            raise HipLibraryError(f"{LIB_PATH} was built from other sources (digest {built[:12]}.. != "
                                  f"{src[:12]}..); rebuild with `python -m videopainter_amd.build`")
        sizes = (i64 * 7)()
        L.vp_struct_sizes(sizes)
        want = (C.sizeof(GemmDesc), C.sizeof(AttnDesc), C.sizeof(DpmDesc), C.sizeof(GemmMxDesc),
                C.sizeof(AttnFp8Desc), C.sizeof(Conv3dDesc), C.sizeof(AttnBwdDesc))
        if tuple(sizes) != want:
            raise HipLibraryError(f"descriptor size mismatch lib={tuple(sizes)} python={want}; rebuild")
        knob_values.update({k: os.environ.get(k) for k in KNOBS})  # what the library read at load
        _lib = L
        return L


def has_diag() -> bool:
    """True when the loaded library is the diagnostic build (include/vp_hip_diag.h entry points present)."""
    return all(hasattr(lib(), n) for n in DIAG_SIGS)


def _source_digest():
    """Digest of the csrc/ sources next to this package (None when they are absent, e.g. a binary-only install)."""
    from . import build as _b
    if not _b._sources():
        return None
    return _b.source_digest()


_ERRS = {1000: "VP_ERR_ARG (invalid size/stride/pointer)", 1001: "VP_ERR_UNSUPPORTED"}


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {_ERRS.get(rc, f'hipError {rc}')}")
