// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of the VideoPainter denoising hot path.
// Wave = 64 lanes.  bf16 is the storage type everywhere; arithmetic accumulates in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vp_hip.h"

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

VP_DEV float silu(float x) { return x / (1.f + __expf(-x)); }

// norm_q / norm_k + apply_rotary_emb on one 64-wide head held as 8 consecutive values by each of 8 consecutive lanes
// (sub = the lane's eighth; the 8 lanes are active together): LayerNorm(64) in fp32 from the bf16 inputs (two-pass
// mean / centred variance, rstd = rsqrt(var + eps)), bf16 output (torch LayerNorm on bf16,
// attention_processor.py:2143-2154), then when cr / sr are given (video tokens) the interleaved-pair rotation in
// fp32 of the bf16 values, x * cos + rot(x) * sin (embeddings.py:655-701, apply_rotary_emb).  Shared by
// vp_head_norm_rope_* and the QKV GEMM's fused epilogue so the two are bit-equal.
VP_DEV void ln64_rope8(float (&x)[8], int sub, const bf16* __restrict__ lw, const bf16* __restrict__ lb, float eps,
                       const float* __restrict__ cr, const float* __restrict__ sr) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s += x[e];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  const float mean = s * (1.f / 64.f);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t = x[e] - mean;
    q += t * t;
  }
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  q += __shfl_xor(q, 4, 64);
  const float rstd = rsqrtf(q * (1.f / 64.f) + eps);
  const bf16x8 w = *(const bf16x8*)(lw + sub * 8);
  const bf16x8 bb = *(const bf16x8*)(lb + sub * 8);
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = rbf((x[e] - mean) * rstd * bf2f(w[e]) + bf2f(bb[e]));
  if (cr != nullptr) {
    const f32x4 c0 = *(const f32x4*)(cr + sub * 8), c1 = *(const f32x4*)(cr + sub * 8 + 4);
    const f32x4 s0 = *(const f32x4*)(sr + sub * 8), s1 = *(const f32x4*)(sr + sub * 8 + 4);
    const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    float y[8];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      y[e] = x[e] * cs[e] + (-x[e + 1]) * sn[e];
      y[e + 1] = x[e + 1] * cs[e + 1] + x[e] * sn[e + 1];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = y[e];
  }
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

#define VP_CHECK_LAUNCH()                                 \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return (int)_e;                   \
  } while (0)
