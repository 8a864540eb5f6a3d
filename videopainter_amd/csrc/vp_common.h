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
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  // tanh(u) = 1 - 2 / (exp(2u) + 1), stable for large |u|
  float e = __expf(2.f * u);
  float t = 1.f - 2.f / (e + 1.f);
  return 0.5f * x * (1.f + t);
}

VP_DEV float silu(float x) { return x / (1.f + __expf(-x)); }

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

#define VP_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return (int)_e;                   \
  } while (0)
