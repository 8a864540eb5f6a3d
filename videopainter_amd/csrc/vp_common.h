// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of the VideoPainter denoising hot path.
// Wave = 64 lanes.  bf16 is the storage type everywhere; arithmetic accumulates in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vp_hip.h"
#ifndef VP_DIAG
#define VP_DIAG 0  // 1: the diagnostic entry points of include/vp_hip_diag.h (python -m videopainter_amd.build --diag)
#endif
#if VP_DIAG
#include "../../include/vp_hip_diag.h"
#endif

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define VP_WAVE 64
#define VP_DEV __device__ __forceinline__

VP_DEV float bf2f(bf16 x) { return (float)x; }
VP_DEV bf16 f2bf(float x) { return (bf16)x; }
// round-trip through bf16 (emulates the reference's bf16 storage points)
VP_DEV float rbf(float x) { return (float)(bf16)x; }

VP_DEV float gelu_tanh(float x) {
  // torch F.gelu(approximate="tanh"): 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))
  // = x / (1 + exp(-2u)) = x / (1 + 2^(x (c0 + c1 x^2))) with c0 = -2 k0 log2(e), c1 = c0 k1: 5 VALU + v_exp_f32 +
  // v_rcp_f32 (1 ulp).  The IEEE division of the textbook form costs ~10 VALU per element, and in the FF1 GEMM's
  // epilogue (256 x 256 outputs per workgroup, not overlapped with MFMA) that was ~20 % of the tile time.  Large
  // |x| saturates correctly: 2^(+big) = inf -> rcp = 0 -> -0; 2^(-big) = 0 -> x.
  const float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f, c1 = c0 * 0.044715f;
  const float a = x * __builtin_fmaf(c1, x * x, c0);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(a));
}

// d/dx of the tanh-form GELU (torch's gelu_backward, approximate="tanh"), fp32 from the bf16 pre-activation.
// tanh(u) = 1 - 2 / (1 + 2^(2 u log2 e)) on v_exp_f32 + v_rcp_f32 (absolute error ~1e-7, far below the bf16 output's
// ulp; saturates to +-1 through inf / 0): the libm tanhf it replaces cost ~10x the VALU, which in the FF2 dgrad GEMM's
// epilogue (VP_EPI_GELU_BWD, not overlapped with MFMA) was as slow as the separate elementwise pass.
// Every fused multiply-add is explicit and contraction is off, so the standalone pass and the GEMM epilogue compile
// to the same arithmetic whatever the surrounding code (they are compared bit for bit).
VP_DEV float gelu_grad(float x) {
#pragma clang fp contract(off)
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * __builtin_fmaf(k1 * x2, x, x);  // k0 (x + k1 x^3)
  const float t = __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * (2.f * 1.4426950408889634f))),
                                 1.f);
  const float dt = __builtin_fmaf(-t, t, 1.f);                 // 1 - t^2
  const float pd = k0 * __builtin_fmaf(3.f * k1, x2, 1.f);     // k0 (1 + 3 k1 x^2)
  return __builtin_fmaf(0.5f, 1.f + t, (0.5f * x) * dt * pd);
}

VP_DEV float silu(float x) { return x / (1.f + __expf(-x)); }

// norm_q / norm_k + apply_rotary_emb on one 64-wide head spread over 4 lanes (g = the lane's quarter, partners at
// lane xor X1 and xor X2; the 4 lanes are active together), 16 values each: x[4 j + r] is column 16 j + 4 g + r —
// the layout of a 16x16 MFMA accumulator row (4 consecutive columns per lane, 4 fragments per head), so the QKV
// GEMM applies it to its accumulators (X1, X2 = 16, 32) and vp_head_norm_rope_* to loaded rows (X1, X2 = 1, 2)
// with the same arithmetic in the same order: bit-equal.  LayerNorm(64) in fp32 from the bf16 inputs (two-pass mean
// / centred variance, rstd = rsqrt(var + eps)), bf16 output (torch LayerNorm on bf16,
// attention_processor.py:2143-2154), then when cr / sr are given (video tokens) the interleaved-pair rotation in
// fp32 of the bf16 values, x * cos + rot(x) * sin (embeddings.py:655-701, apply_rotary_emb).
// s + (s of the lane xor X): 16 / 32 by a permlane swap (VALU: the pair {own, partner} in either order, and the
// f32 add is commutative, so the sum is the same bits as with the shuffle), other distances by __shfl_xor
template <int X>
VP_DEV float add_partner(float v) {
  if constexpr (X == 16 || X == 32) {
    const unsigned u = __float_as_uint(v);
    const auto sw = X == 16 ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                            : __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  } else {
    return v + __shfl_xor(v, X, 64);
  }
}

// the arithmetic of ln64_rope16 on operands already in registers (w / bb: the LayerNorm weight / bias quads of
// columns 16 j + 4 g, cs / sn: the RoPE cos / sin quads; rot: apply the rotation)
template <int X1, int X2>
VP_DEV void ln64_rope16_regs(float (&x)[16], const bf16x4 (&w)[4], const bf16x4 (&bb)[4], float eps,
                             const f32x4 (&cs)[4], const f32x4 (&sn)[4], bool rot) {
  // every multiply-add spelled out (fma or not) and no contraction: otherwise hipcc fuses differently in different
  // surroundings (SLP-packed v_pk_mul + v_add in one kernel, v_fmac in another) and the two users drift by an ulp
#pragma clang fp contract(off)
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += x[e];
  s = add_partner<X2>(add_partner<X1>(s));
  const float mean = s * (1.f / 64.f);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float t = x[e] - mean;
    q = __builtin_fmaf(t, t, q);
  }
  q = add_partner<X2>(add_partner<X1>(q));
  const float rstd = rsqrtf(__builtin_fmaf(q, 1.f / 64.f, eps));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      x[4 * j + r] = rbf(__builtin_fmaf((x[4 * j + r] - mean) * rstd, bf2f(w[j][r]), bf2f(bb[j][r])));
    const float x0 = x[4 * j], x1 = x[4 * j + 1], x2 = x[4 * j + 2], x3 = x[4 * j + 3];
    const float y0 = __builtin_fmaf(x0, cs[j][0], -(x1 * sn[j][0]));
    const float y1 = __builtin_fmaf(x1, cs[j][1], x0 * sn[j][1]);
    const float y2 = __builtin_fmaf(x2, cs[j][2], -(x3 * sn[j][2]));
    const float y3 = __builtin_fmaf(x3, cs[j][3], x2 * sn[j][3]);
    x[4 * j] = rot ? y0 : x0;
    x[4 * j + 1] = rot ? y1 : x1;
    x[4 * j + 2] = rot ? y2 : x2;
    x[4 * j + 3] = rot ? y3 : x3;
  }
}

// norm_q / norm_k + apply_rotary_emb on one 64-wide head spread over 4 lanes (g = the lane's quarter, partners at
// lane xor X1 and xor X2; the 4 lanes are active together), 16 values each: x[4 j + r] is column 16 j + 4 g + r —
// the layout of a 16x16 MFMA accumulator row (4 consecutive columns per lane, 4 fragments per head), so the QKV
// GEMM applies it to its accumulators (X1, X2 = 16, 32) and vp_head_norm_rope_* to loaded rows (X1, X2 = 1, 2)
// with the same arithmetic in the same order (ln64_rope16_regs): bit-equal.  LayerNorm(64) in fp32 from the bf16
// inputs (two-pass mean / centred variance, rstd = rsqrt(var + eps)), bf16 output (torch LayerNorm on bf16,
// attention_processor.py:2143-2154), then when cr / sr are given (video tokens) the interleaved-pair rotation in
// fp32 of the bf16 values, x * cos + rot(x) * sin (embeddings.py:655-701, apply_rotary_emb).  Every operand is
// loaded before the reductions, so their latency overlaps them.
template <int X1, int X2>
VP_DEV void ln64_rope16(float (&x)[16], int g, const bf16* __restrict__ lw, const bf16* __restrict__ lb, float eps,
                        const float* __restrict__ cr, const float* __restrict__ sr) {
  bf16x4 w[4], bb[4];
  f32x4 cs[4], sn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 16 * j + 4 * g;
    w[j] = *(const bf16x4*)(lw + c);
    bb[j] = *(const bf16x4*)(lb + c);
    cs[j] = cr != nullptr ? *(const f32x4*)(cr + c) : (f32x4){1.f, 1.f, 1.f, 1.f};
    sn[j] = cr != nullptr ? *(const f32x4*)(sr + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  ln64_rope16_regs<X1, X2>(x, w, bb, eps, cs, sn, cr != nullptr);
}

VP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

VP_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// sum over the 16 lanes of a 16-lane row group (lanes sharing lane>>4)
VP_DEV float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// bijective XCD-aware remap of a 1-D workgroup id: blocks that share an XCD (id % 8) get a contiguous range of
// logical tile ids (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
VP_DEV int xcd_remap(int wg, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = wg % 8, idx = wg / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// persistent launches (p2 / p2a attention): the next of n work items for a workgroup on XCD x (-1: none left).  Item ranges are
// xcd_remap's (XCD y owns a contiguous range, counted by tickets[y]); an XCD whose range is done takes from the
// others'.  tickets: 8 ints, zero at launch.  (The dispatcher hands each XCD the same number of workgroups while the
// XCDs run at different clocks: per-XCD attention loop times 419-464 us at config 2, tools/attn_wg_timeline.py.)
VP_DEV int xcd_ticket(int* tickets, int n, int x) {
  const int q = n >> 3, r = n & 7;
#pragma unroll 1
  for (int k = 0; k < 8; ++k) {
    const int y = (x + k) & 7;
    const int size = q + (y < r ? 1 : 0);
    const int lo = y < r ? y * (q + 1) : r * (q + 1) + (y - r) * q;
    if (__hip_atomic_load(tickets + y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= size) continue;
    const int c = __hip_atomic_fetch_add(tickets + y, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c < size) return lo + c;
  }
  return -1;
}

// ---- MX-FP8 (e4m3 + E8M0 per 32 elements; layout and rounding rule in include/vp_hip.h) ----
// byte offset of the scale of (row r, K-block kb) in an MX scale array of a tensor with K columns
VP_DEV int64_t mx_scale_off(int64_t r, int kb, int K) {
  return ((r >> 8) * (K >> 7) + (kb >> 2)) * 1024 + (kb & 3) * 256 + (r & 15) * 16 + ((r >> 4) & 15);
}

// scale exponent s = ceil(log2(amax / 448)) in [-127, 127]; -127 (byte 0) for an all-zero block
VP_DEV int mx_exponent(float amax) {
  if (!(amax > 0.f)) return -127;
  const uint32_t u = __float_as_uint(amax * (1.f / 448.f));
  int e = (int)((u >> 23) & 0xff) - 127;  // floor(log2) for normal values
  if ((u & 0x7fffff) != 0) ++e;           // not a power of two -> round up
  if (((u >> 23) & 0xff) == 0) e = -126;  // subnormal ratio: below 2^-126
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// 2^-s as a float, s in [-127, 127] (2^-127 is subnormal)
VP_DEV float mx_inv_scale(int s) {
  const int e = 127 - s;  // biased exponent of 2^-s, in [0, 254]
  return e == 0 ? __uint_as_float(0x00400000u) : __uint_as_float((uint32_t)e << 23);
}

// 8 floats -> 8 e4m3 bytes (RNE, |x| clamped to 448 first)
VP_DEV u32x2 mx_pack8(const float (&v)[8], float mul) {
  u32x2 r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int w = 0;
    const float a = __builtin_amdgcn_fmed3f(v[4 * h + 0] * mul, 448.f, -448.f);
    const float b = __builtin_amdgcn_fmed3f(v[4 * h + 1] * mul, 448.f, -448.f);
    const float c = __builtin_amdgcn_fmed3f(v[4 * h + 2] * mul, 448.f, -448.f);
    const float d = __builtin_amdgcn_fmed3f(v[4 * h + 3] * mul, 448.f, -448.f);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
    r[h] = (uint32_t)w;
  }
  return r;
}

// one 32-element MX block held as 8 values by each of 4 consecutive lanes (lane & 3 = block quarter): block
// exponent via two xor-shuffles; returns the 8 packed bytes of this lane and the block's scale byte
VP_DEV u32x2 mx_quantize_quarter(const float (&v)[8], uint8_t& scale_byte) {
  float am = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[e]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  const int s = mx_exponent(am);
  scale_byte = (uint8_t)(s + 127);
  return mx_pack8(v, mx_inv_scale(s));
}

// A/B knobs (include/vp_hip.h vp_set_knob): the environment read once at library load (misc.hip), then only
// vp_set_knob.  vp_knob(k) = the value, or nullptr when unset — what getenv of the same name returned.
enum VpKnob {
  VPK_GEMM_VARIANT,
  VPK_GEMM_NO_TAIL,
  VPK_GEMM_GROUP,
  VPK_GEMM8_VARIANT,
  VPK_ATTN_BOUNDED_MODE,
  VPK_ATTN_UNBOUNDED_MODE,
  VPK_ATTN_NO_SPLIT,
  VPK_ATTN8_VARIANT,
  VPK_T5_ATTN,
  VPK_CONV_HOIST,
  VPK_CONV_PIPE,
  VPK_ATTN_BWD_VARIANT,
  VPK_ATTN_TAIL,
  VPK_ATTN_PERSIST,
  VPK_COUNT
};
const char* vp_knob(int k);

#define VP_CHECK_LAUNCH()                               \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return (int)_e;                   \
  } while (0)
