// Conditioning-path and data-movement kernels of the denoising step (gfx950): small-M linears (time embedding,
// AdaLN modulation vectors), sinusoidal timestep embedding, patchify / token mask / unpatchify, the fused
// CFG + DPM-Solver + replace-gt step glue, and a device-side synthetic-weight generator.
#include <stdlib.h>
#include <string.h>

#include "vp_common.h"

namespace {

// ---- small-M linear: y[m, n] = act_out(Σ_k act_in(x[m, k]) W[n, k] + b[n]) ----
constexpr int LS_THREADS = 256;
constexpr int LS_COLS_PER_WAVE = 4;

__global__ __launch_bounds__(LS_THREADS) void linear_small_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                                 const bf16* __restrict__ W,
                                                                 const bf16* __restrict__ bias, bf16* __restrict__ y,
                                                                 int64_t ldy, int M, int N, int K, int act_in,
                                                                 int act_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xs = (bf16*)smem;  // [M][K] act_in(x), bf16
  if ((K % 8) == 0 && (ldx % 8) == 0 && ((uintptr_t)x & 15) == 0) {  // 16-byte chunks (one load per thread)
    const int kc = K / 8;
    for (int i = threadIdx.x; i < M * kc; i += LS_THREADS) {
      const int m = i / kc, c = i - m * kc;
      bf16x8 v8 = *(const bf16x8*)(x + (int64_t)m * ldx + c * 8);
      if (act_in == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = f2bf(rbf(silu(bf2f(v8[e]))));
      }
      *(bf16x8*)(xs + m * K + c * 8) = v8;
    }
  } else {
    for (int i = threadIdx.x; i < M * K; i += LS_THREADS) {
      const int m = i / K, k = i - m * K;
      float v = bf2f(x[(int64_t)m * ldx + k]);
      if (act_in == 1) v = rbf(silu(v));
      xs[i] = f2bf(v);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nch = K / 8;
  for (int cc = 0; cc < LS_COLS_PER_WAVE; ++cc) {
    const int n = (blockIdx.x * (LS_THREADS / 64) + wave) * LS_COLS_PER_WAVE + cc;
    if (n >= N) break;
    float acc[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m] = 0.f;
    for (int c = lane; c < nch; c += 64) {
      const bf16x8 w = *(const bf16x8*)(W + (int64_t)n * K + c * 8);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (m < M) {
          const bf16x8 xv = *(const bf16x8*)(xs + m * K + c * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[m] = fmaf(bf2f(w[e]), bf2f(xv[e]), acc[m]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (m < M) {
        float s = wave_sum(acc[m]);
        if (lane == 0) {
          float v = rbf(s + (bias ? bf2f(bias[n]) : 0.f));
          if (act_out == 1) v = rbf(silu(v));
          y[(int64_t)m * ldy + n] = f2bf(v);
        }
      }
    }
  }
}

// ---- get_timestep_embedding (embeddings.py:27-78), flip_sin_to_cos = True ----
__global__ void timestep_embedding_kernel(const float* __restrict__ ts, bf16* __restrict__ out, int B, int dim,
                                          float shift) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int half = dim / 2;
  if (i >= B * half) return;
  const int b = i / half, j = i - b * half;
  const float expo = -9.210340371976184f * (float)j / ((float)half - shift);  // -ln(10000) * j / (half - shift)
  const float freq = expf(expo);
  const float arg = ts[b] * freq;
  out[(int64_t)b * dim + j] = f2bf(cosf(arg));
  out[(int64_t)b * dim + half + j] = f2bf(sinf(arg));
}

// ---- patchify: rows (b, f, y, x), cols c*p*p + dy*p + dx ----
__global__ void patchify_kernel(const bf16* __restrict__ s1, int C1, const bf16* __restrict__ s2, int C2,
                                bf16* __restrict__ out, int Kpad, int B, int F, int H, int W, int p) {
  const int Hp = H / p, Wp = W / p;
  const int C = C1 + C2;
  const int64_t total = (int64_t)B * F * Hp * Wp * (Kpad / (p * p));
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int cslots = Kpad / (p * p);
  const int c = (int)(i % cslots);
  const int64_t row = i / cslots;
  const int x = (int)(row % Wp);
  const int yy = (int)((row / Wp) % Hp);
  const int f = (int)((row / ((int64_t)Wp * Hp)) % F);
  const int b = (int)(row / ((int64_t)Wp * Hp * F));
  bf16* o = out + row * Kpad + c * p * p;
  if (c >= C) {
    for (int k = 0; k < p * p; ++k) o[k] = f2bf(0.f);
    return;
  }
  const bf16* src = c < C1 ? s1 + (((int64_t)b * F + f) * C1 + c) * H * W
                           : s2 + (((int64_t)b * F + f) * C2 + (c - C1)) * H * W;
  for (int dy = 0; dy < p; ++dy)
    for (int dx = 0; dx < p; ++dx) o[dy * p + dx] = src[(int64_t)(yy * p + dy) * W + x * p + dx];
}

__global__ void patch_mask_kernel(const void* __restrict__ mask, int is_f32, uint8_t* __restrict__ out, int B, int F,
                                  int H, int W, int p) {
  const int Hp = H / p, Wp = W / p;
  const int64_t total = (int64_t)B * F * Hp * Wp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % Wp);
  const int yy = (int)((i / Wp) % Hp);
  const int64_t bf = i / ((int64_t)Wp * Hp);
  float s = 0.f;
  for (int dy = 0; dy < p; ++dy)
    for (int dx = 0; dx < p; ++dx) {
      const int64_t off = bf * H * W + (int64_t)(yy * p + dy) * W + x * p + dx;
      s += is_f32 ? ((const float*)mask)[off] : bf2f(((const bf16*)mask)[off]);
    }
  out[i] = (s / (float)(p * p)) > 0.f ? 1 : 0;
}

// one thread per 8 columns of one row (self-guidance + injection after a block, vp_guide_rows_bf16)
__global__ void guide_rows_kernel(bf16* __restrict__ x, int64_t ld_x, int64_t bs_x, const bf16* __restrict__ g,
                                  int64_t ld_g, int64_t bs_g, const bf16* __restrict__ inj, int64_t ld_i, int64_t bs_i,
                                  int inject_all, const uint8_t* __restrict__ mask, int64_t mask_bs, int rows, int D,
                                  int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c8 = D / 8;
  const int c = (int)(i % c8) * 8;
  const int64_t br = i / c8;
  const int r = (int)(br % rows), b = (int)(br / rows);
  const bool keep = mask[(int64_t)b * mask_bs + r] != 0;
  if (keep && !(inj != nullptr && inject_all)) return;  // a masked row without injection: unchanged
  bf16* xp = x + (int64_t)b * bs_x + (int64_t)r * ld_x + c;
  bf16x8 v = keep ? *(const bf16x8*)xp : *(const bf16x8*)(g + (int64_t)b * bs_g + (int64_t)r * ld_g + c);
  if (inj != nullptr) {
    const bf16x8 a = *(const bf16x8*)(inj + (int64_t)b * bs_i + (int64_t)r * ld_i + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(a[e]));
  }
  *(bf16x8*)xp = v;
}

__global__ void unpatchify_kernel(const bf16* __restrict__ proj, int64_t ld, bf16* __restrict__ out, int B, int F,
                                  int C, int H, int W, int p) {
  const int64_t total = (int64_t)B * F * C * H * W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int xx = (int)(i % W);
  const int yy = (int)((i / W) % H);
  const int c = (int)((i / ((int64_t)W * H)) % C);
  const int64_t bf = i / ((int64_t)W * H * C);
  const int Hp = H / p, Wp = W / p;
  const int64_t row = bf * Hp * Wp + (int64_t)(yy / p) * Wp + (xx / p);
  out[i] = proj[row * ld + c * p * p + (yy % p) * p + (xx % p)];
}

// ---- fused CFG + DPM step + replace-gt (see vp_hip.h) ----
__global__ void dpm_step_kernel(const vp_dpm_desc d) {
#pragma clang fp contract(off)  // the reference evaluates every product / sum as a separate rounded torch op
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.n) return;
  const bf16* np = (const bf16*)d.noise_pred;
  float mo;
  if (d.model_output != nullptr) {
    mo = d.model_output[i];
  } else if (d.do_cfg) {
    const float u = bf2f(np[i]), t = bf2f(np[d.n + i]);
    mo = u + d.guidance * (t - u);
  } else {
    mo = bf2f(np[i]);
  }
  const float x = bf2f(((const bf16*)d.sample)[i]);
  // pred_original_sample = sqrt(a_t) * sample (bf16 op) - sqrt(1 - a_t) * model_output (fp32 op)
  const float pred = rbf(d.sa * x) - d.sb * mo;
  d.pred_out[i] = pred;
  const float x1 = rbf(d.m1 * x);
  float prev;
  if (d.second_order) {
    const float old = d.old_pred[i];
    const float den = d.m3 * pred - d.m4 * old;
    prev = (x1 - d.m2 * den) + rbf(d.mn * bf2f(((const bf16*)d.noise2)[i]));
  } else {
    prev = (x1 - d.m2 * pred) + rbf(d.mn * bf2f(((const bf16*)d.noise1)[i]));
  }
  if (d.prev_out != nullptr) d.prev_out[i] = prev;
  if (d.latents_out == nullptr) return;
  float lat = rbf(prev);
  if (d.replace_gt) {
    const float g = bf2f(((const bf16*)d.gt)[i]);
    float init = g;
    if (d.gt_add_noise) init = rbf(rbf(d.gsa * g) + rbf(d.gsb * bf2f(((const bf16*)d.gt_noise)[i])));
    const float m = bf2f(((const bf16*)d.mask)[i]);
    if (d.mask_background) lat = rbf(rbf(m * init) + rbf(rbf(1.f - m) * lat));
    else lat = rbf(rbf(rbf(1.f - m) * init) + rbf(m * lat));
  }
  ((bf16*)d.latents_out)[i] = f2bf(lat);
}

VP_DEV uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_normal_kernel(bf16* __restrict__ out, int64_t n, uint64_t seed, float mean, float std) {
#pragma clang fp contract(off)  // z * std + mean rounded like the numpy generator (weights.synth_param)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t r1 = splitmix64(seed + 2ull * (uint64_t)i);
  const uint64_t r2 = splitmix64(seed + 2ull * (uint64_t)i + 1ull);
  const double u1 = ((double)(r1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
  const double u2 = (double)(r2 >> 11) * (1.0 / 9007199254740992.0);
  const float z = (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
  out[i] = f2bf(z * std + mean);
}

}  // namespace

extern "C" int vp_abi_version(void) { return VP_ABI_VERSION; }

// digest of the sources + flags this library was compiled from (set by videopainter_amd/build.py), checked at load
// time against the sources next to it so a stale library never runs silently
#ifndef VP_BUILD_DIGEST
#define VP_BUILD_DIGEST "unknown"
#endif
extern "C" const char* vp_build_digest(void) { return VP_BUILD_DIGEST; }

// ---- A/B knobs: the environment read ONCE (the first vp_knob / vp_set_knob call, from the load-time constructor
// below), kept in a table; launches read the table, never the environment ----
namespace {
const char* const knob_names[VPK_COUNT] = {"VP_GEMM_VARIANT",        "VP_GEMM_NO_TAIL",   "VP_GEMM_GROUP",
                                           "VP_GEMM8_VARIANT",       "VP_ATTN_BOUNDED_MODE",
                                           "VP_ATTN_UNBOUNDED_MODE", "VP_ATTN_NO_SPLIT",  "VP_ATTN8_VARIANT",
                                           "VP_T5_ATTN",             "VP_CONV_HOIST",     "VP_CONV_PIPE",
                                           "VP_ATTN_BWD_VARIANT",    "VP_ATTN_TAIL",
                                           "VP_ATTN_PERSIST"};
struct KnobTable {
  char val[VPK_COUNT][32];
  bool set[VPK_COUNT];
  KnobTable() {
    for (int k = 0; k < VPK_COUNT; ++k) {
      const char* e = getenv(knob_names[k]);
      set[k] = e != nullptr && strlen(e) < sizeof(val[k]);
      val[k][0] = 0;
      if (set[k]) strcpy(val[k], e);
    }
  }
};
KnobTable& knobs() {
  static KnobTable t;  // initialised once (thread-safe static), at library load by the constructor below
  return t;
}
__attribute__((constructor)) void knobs_at_load() { (void)knobs(); }
}  // namespace

const char* vp_knob(int k) {
  KnobTable& t = knobs();
  return k >= 0 && k < VPK_COUNT && t.set[k] ? t.val[k] : nullptr;
}

extern "C" int vp_set_knob(const char* name, const char* value) {
  if (name == nullptr || (value != nullptr && strlen(value) >= 32)) return VP_ERR_ARG;
  KnobTable& t = knobs();
  for (int k = 0; k < VPK_COUNT; ++k) {
    if (strcmp(name, knob_names[k]) != 0) continue;
    t.set[k] = value != nullptr;
    t.val[k][0] = 0;
    if (value != nullptr) strcpy(t.val[k], value);
    return VP_OK;
  }
  return VP_ERR_ARG;
}

extern "C" void vp_struct_sizes(int64_t* out) {
  out[0] = (int64_t)sizeof(vp_gemm_desc);
  out[1] = (int64_t)sizeof(vp_attn_desc);
  out[2] = (int64_t)sizeof(vp_dpm_desc);
  out[3] = (int64_t)sizeof(vp_gemm_mx_desc);
  out[4] = (int64_t)sizeof(vp_attn_fp8_desc);
  out[5] = (int64_t)sizeof(vp_conv3d_desc);
  out[6] = (int64_t)sizeof(vp_attn_bwd_desc);
}

// M <= 2 rows (the CFG pair's AdaLN / time-embedding vectors), K <= 512: a weight-streaming kernel.  Each wave owns
// LSF_COLS columns and each lane one 16-byte K-chunk of every column, so a wave has LSF_COLS x 1 KiB of weights in
// flight at once (the general kernel above has one column's 1 KiB per round trip); x comes straight from global
// memory (2 x 16 bytes per lane), no LDS and no barrier.  Same per-lane products and wave sums as the general
// kernel: bit-identical results.
constexpr int LSF_COLS = 8;
__global__ __launch_bounds__(LS_THREADS) void linear_small_fast_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                                      const bf16* __restrict__ W,
                                                                      const bf16* __restrict__ bias,
                                                                      bf16* __restrict__ y, int64_t ldy, int M, int N,
                                                                      int K, int act_in, int act_out) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nbase = (blockIdx.x * (LS_THREADS / 64) + wave) * LSF_COLS;
  const bool on = lane < K / 8;
  bf16x8 w[LSF_COLS];
#pragma unroll
  for (int cc = 0; cc < LSF_COLS; ++cc)
    w[cc] = (on && nbase + cc < N) ? *(const bf16x8*)(W + (int64_t)(nbase + cc) * K + lane * 8) : bf16x8{};
  bf16x8 xv[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    xv[m] = (on && m < M) ? *(const bf16x8*)(x + (int64_t)m * ldx + lane * 8) : bf16x8{};
    if (act_in == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[m][e] = f2bf(rbf(silu(bf2f(xv[m][e]))));
    }
  }
#pragma unroll
  for (int cc = 0; cc < LSF_COLS; ++cc) {
    const int n = nbase + cc;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (m >= M) continue;
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(bf2f(w[cc][e]), bf2f(xv[m][e]), acc);
      const float sum = wave_sum(acc);
      if (lane == 0 && n < N) {
        float v = rbf(sum + (bias ? bf2f(bias[n]) : 0.f));
        if (act_out == 1) v = rbf(silu(v));
        y[(int64_t)m * ldy + n] = f2bf(v);
      }
    }
  }
}

extern "C" int vp_linear_small_bf16(const void* x, int64_t ldx, const void* W, const void* bias, void* y,
                                    int64_t ldy, int32_t M, int32_t N, int32_t K, int32_t act_in, int32_t act_out,
                                    void* stream) {
  if (!x || !W || !y || M <= 0 || M > 16 || N <= 0 || K <= 0 || (K % 8) || ldx < K || ldy < N) return VP_ERR_ARG;
  if (M <= 2 && K <= 512 && (ldx % 8) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)W & 15) == 0) {
    const int cpb = (LS_THREADS / 64) * LSF_COLS;
    hipLaunchKernelGGL(linear_small_fast_kernel, dim3((N + cpb - 1) / cpb), dim3(LS_THREADS), 0, (hipStream_t)stream,
                       (const bf16*)x, ldx, (const bf16*)W, (const bf16*)bias, (bf16*)y, ldy, M, N, K, act_in,
                       act_out);
    VP_CHECK_LAUNCH();
    return VP_OK;
  }
  const size_t lds = (size_t)M * K * 2;
  if (lds > 160 * 1024) return VP_ERR_ARG;
  const int cols_per_block = (LS_THREADS / 64) * LS_COLS_PER_WAVE;
  const int grid = (N + cols_per_block - 1) / cols_per_block;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)linear_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(linear_small_kernel, dim3(grid), dim3(LS_THREADS), lds, (hipStream_t)stream, (const bf16*)x, ldx,
                     (const bf16*)W, (const bf16*)bias, (bf16*)y, ldy, M, N, K, act_in, act_out);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_timestep_embedding_bf16(const float* timesteps, void* out, int32_t B, int32_t dim,
                                          float freq_shift, void* stream) {
  if (!timesteps || !out || B <= 0 || dim <= 0 || (dim % 2)) return VP_ERR_ARG;
  const int total = B * (dim / 2);
  hipLaunchKernelGGL(timestep_embedding_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     timesteps, (bf16*)out, B, dim, freq_shift);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_patchify_bf16(const void* src1, int32_t C1, const void* src2, int32_t C2, void* out, int32_t Kpad,
                                int32_t B, int32_t F, int32_t H, int32_t W, int32_t p, void* stream) {
  if (!src1 || !out || C1 <= 0 || C2 < 0 || (C2 > 0 && !src2) || p <= 0 || (H % p) || (W % p)) return VP_ERR_ARG;
  if (Kpad < (C1 + C2) * p * p || (Kpad % (p * p))) return VP_ERR_ARG;
  const int64_t total = (int64_t)B * F * (H / p) * (W / p) * (Kpad / (p * p));
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)src1, C1, (const bf16*)src2, C2, (bf16*)out, Kpad, B, F, H, W, p);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_patch_mask(const void* mask, int32_t mask_is_f32, uint8_t* out, int32_t B, int32_t F, int32_t H,
                             int32_t W, int32_t p, void* stream) {
  if (!mask || !out || p <= 0 || (H % p) || (W % p)) return VP_ERR_ARG;
  const int64_t total = (int64_t)B * F * (H / p) * (W / p);
  hipLaunchKernelGGL(patch_mask_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mask,
                     mask_is_f32, out, B, F, H, W, p);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_guide_rows_bf16(void* x, int64_t ld_x, int64_t bs_x, const void* guide, int64_t ld_g, int64_t bs_g,
                                  const void* inject, int64_t ld_i, int64_t bs_i, int32_t inject_all,
                                  const uint8_t* tok_mask, int64_t mask_bstride, int32_t B, int32_t rows, int32_t D,
                                  void* stream) {
  if (!x || !guide || !tok_mask || B <= 0 || rows <= 0 || D <= 0 || (D % 8)) return VP_ERR_ARG;
  if ((ld_x % 8) || (bs_x % 8) || (ld_g % 8) || (bs_g % 8) || ld_x < D || ld_g < D) return VP_ERR_ARG;
  if (inject && ((ld_i % 8) || (bs_i % 8) || ld_i < D)) return VP_ERR_ARG;
  const int64_t total = (int64_t)B * rows * (D / 8);
  hipLaunchKernelGGL(guide_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (bf16*)x, ld_x, bs_x, (const bf16*)guide, ld_g, bs_g, (const bf16*)inject, ld_i, bs_i, inject_all,
                     tok_mask, mask_bstride, rows, D, total);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_unpatchify_bf16(const void* proj, int64_t ld, void* out, int32_t B, int32_t F, int32_t C, int32_t H,
                                  int32_t W, int32_t p, void* stream) {
  if (!proj || !out || p <= 0 || (H % p) || (W % p) || ld < C * p * p) return VP_ERR_ARG;
  const int64_t total = (int64_t)B * F * C * H * W;
  hipLaunchKernelGGL(unpatchify_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)proj, ld, (bf16*)out, B, F, C, H, W, p);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_dpm_step_bf16(const vp_dpm_desc* d, void* stream) {
  if (!d || d->n <= 0 || (!d->noise_pred && !d->model_output) || !d->sample || !d->pred_out || !d->noise1)
    return VP_ERR_ARG;
  if (!d->latents_out && !d->prev_out) return VP_ERR_ARG;
  if (d->second_order && (!d->old_pred || !d->noise2)) return VP_ERR_ARG;
  if (d->replace_gt && (!d->gt || !d->mask || (d->gt_add_noise && !d->gt_noise))) return VP_ERR_ARG;
  hipLaunchKernelGGL(dpm_step_kernel, dim3((unsigned)((d->n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *d);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_fill_normal_bf16(void* out, int64_t n, uint64_t seed, float mean, float std, void* stream) {
  if (!out || n <= 0) return VP_ERR_ARG;
  hipLaunchKernelGGL(fill_normal_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (bf16*)out, n, seed, mean, std);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
