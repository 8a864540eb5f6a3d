/* Diagnostic entry points of libvp_hip — built only with -DVP_DIAG=1 (python -m videopainter_amd.build --diag,
 * which writes videopainter_amd/_lib/libvp_hip_diag.so; select it with VP_HIP_LIB).  The default library exports
 * none of them.  Not part of the drop-in boundary: hardware layout self-tests behind the fp8 kernels' operand
 * formats (tests/test_mx_gpu.py, tests/test_attention_fp8_gpu.py run them when the diagnostic library is loaded). */
#ifndef VP_HIP_DIAG_H
#define VP_HIP_DIAG_H
#include "vp_hip.h"
#ifdef __cplusplus
extern "C" {
#endif

/* layout self-test of one block-scaled MFMA (one wave): A, B e4m3 [16][128] row-major, per-lane scale bytes sa/sb
 * [64]: lane l feeds K-chunks l/16 and l/16+4 (16 bytes each) of row l%16 and the scale of row l%16, K-block l/16;
 * C fp32 [16][16] = Σ_k A[i][k]·2^(sa[i+16(k/32)]-127) · B[j][k]·2^(sb[j+16(k/32)]-127) */
int vp_mx_mfma_probe(const void* A, const void* B, const void* sa, const void* sb, float* C, void* stream);

/* One v_mfma_scale_f32_32x32x64_f8f6f4 with the layout the fp8 attention assumes (lane l: row l % 32, 16-byte
 * K-chunks l/32 and l/32 + 2 of A[32][64] / B[32][64], scale bytes sa[l] / sb[l] for (row l % 32, K-block l/32));
 * C[32][32] row-major fp32 = A_deq . B_deq^T.  Layout self-test. */
int vp_mx_mfma_probe32(const void* A, const void* B, const void* sa, const void* sb, float* C, void* stream);

#ifdef __cplusplus
}
#endif
#endif
