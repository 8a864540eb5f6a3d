// T5 v1.1 encoder pieces for gfx950 (CogVideoX's text encoder, T5-XXL, 226 tokens, once per
// prompt).  The projections run on vp_gemm_bf16; this file holds what is T5-specific: the token-embedding gather,
// T5LayerNorm (RMS norm, no mean, no bias), the gated-GELU product and the self-attention with the bucketed
// relative-position bias and no 1/sqrt(d) scaling.
// Reference algorithm: transformers `modeling_t5.py` (pinned transformers==4.42.2 in the reference's
// requirements.txt): T5LayerNorm, T5DenseGatedActDense, T5Attention (compute_bias / _relative_position_bucket),
// called by the pipeline's `_get_t5_prompt_embeds` (…_anyl.py:216-256).
#include <stdlib.h>
#include <string.h>

#include "vp_common.h"

namespace {

__global__ __launch_bounds__(256) void embed_gather_kernel(const bf16* __restrict__ table, const int64_t* __restrict__ ids,
                                                           bf16* __restrict__ out, int rows, int D, int vocab) {
  const int C8 = D >> 3;
  const int64_t total = (int64_t)rows * C8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int r = (int)(i / C8), c = (int)(i - (int64_t)r * C8);
    int64_t id = ids[r];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // the host checks the range; never read out of bounds
    *(bf16x8*)(out + (int64_t)r * D + c * 8) = *(const bf16x8*)(table + id * D + c * 8);
  }
}

// T5LayerNorm: y = w * bf16(x * rsqrt(mean(x^2) + eps)) — fp32 statistics from the bf16 row, bf16 rounding of the
// normalised row before the weight, like the reference module on bf16 weights.  One wave per row.
__global__ __launch_bounds__(256) void rms_norm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                       bf16* __restrict__ y, int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* xr = x + (int64_t)row * D;
  const int C8 = D >> 3;
  float ss = 0.f;
  for (int c = lane; c < C8; c += 64) {
    const bf16x8 v = *(const bf16x8*)(xr + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss = __builtin_fmaf(bf2f(v[e]), bf2f(v[e]), ss);
  }
  const float r = rsqrtf(wave_sum(ss) / (float)D + eps);
  for (int c = lane; c < C8; c += 64) {
    const bf16x8 v = *(const bf16x8*)(xr + c * 8);
    const bf16x8 wv = *(const bf16x8*)(w + c * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(wv[e]) * rbf(bf2f(v[e]) * r));
    *(bf16x8*)(y + (int64_t)row * D + c * 8) = o;
  }
}

__global__ __launch_bounds__(256) void mul_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                  bf16* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const bf16x8 u = *(const bf16x8*)(a + i * 8), v = *(const bf16x8*)(b + i * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(u[e]) * bf2f(v[e]));
    *(bf16x8*)(y + i * 8) = o;
  }
}

// Self-attention of one (batch, head) over L <= T5_MAX_L tokens (d_kv = 64): K and V of the head in LDS (K rows
// padded to 66 elements: the score pass reads one key row per lane), 4 waves x QW queries per block.
// scores = bf16(q.k) (the reference's bf16 matmul output) + bias (bf16 add), softmax in fp32 -> bf16 weights,
// out = bf16(sum_j w_j v_j) with fp32 accumulation; masked keys (mask[b, j] == 0) get the dtype minimum added.
constexpr int T5_MAX_L = 384;  // LDS: K + V + QW weight rows per wave <= 160 KB
constexpr int QW = 8;  // queries per wave
constexpr int KROW = 66;

__global__ __launch_bounds__(256) void t5_attention_kernel(const bf16* __restrict__ qkv, int64_t ld, int inner,
                                                           int L, int H, const bf16* __restrict__ bias_table,
                                                           const int32_t* __restrict__ buckets,
                                                           const int64_t* __restrict__ mask, bf16* __restrict__ out,
                                                           int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lp = (L + 7) & ~7;                 // 16-byte aligned sub-arrays
  bf16* Ks = (bf16*)smem;                       // [Lp][KROW]
  bf16* Vs = Ks + Lp * KROW;                    // [Lp][64]
  float* Bs = (float*)(Vs + Lp * 64);           // [2 Lp]: the head's bias by relative position j - q + L - 1
  float* Ms = Bs + 2 * Lp;                      // [Lp]: 1 where the key is masked
  bf16* Ps = (bf16*)(Ms + Lp);                  // [4 waves][QW][Lp]: softmax weights (bf16-rounded values)
  const int nqb = (L + 4 * QW - 1) / (4 * QW);
  const int bh = blockIdx.x / nqb, qb = blockIdx.x - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* base = qkv + (int64_t)b * L * ld;
  for (int i = tid; i < L * 8; i += 256) {
    const int j = i >> 3, c = i & 7;
    const bf16x8 kv = *(const bf16x8*)(base + (int64_t)j * ld + inner + h * 64 + c * 8);
    const bf16x8 vv = *(const bf16x8*)(base + (int64_t)j * ld + 2 * inner + h * 64 + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) Ks[j * KROW + c * 8 + e] = kv[e];
    *(bf16x8*)(Vs + j * 64 + c * 8) = vv;
  }
  // the bucket of (q, j) depends only on j - q (bidirectional T5 buckets): row 0 of the bucket matrix holds
  // j - q >= 0, column 0 holds j - q <= 0
  for (int r = tid; r < 2 * L - 1; r += 256) {
    const int rel = r - (L - 1);
    const int bk = rel >= 0 ? buckets[rel] : buckets[(int64_t)(-rel) * L];
    Bs[r] = bf2f(bias_table[bk * H + h]);
  }
  for (int j = tid; j < L; j += 256) Ms[j] = (mask != nullptr && mask[(int64_t)b * L + j] == 0) ? 1.f : 0.f;
  __syncthreads();
  // phase 1, per query of this wave: scores, softmax, the bf16-rounded weights into P[qi][:]; phase 2: one pass over
  // the keys accumulates all QW queries at once (V row read once per key, QW independent FMA chains; the per-query
  // serial chain over L keys was latency-bound), in the same key order as before
  bf16* P = Ps + wave * QW * Lp;
  int nq = 0;
  for (int qi = 0; qi < QW; ++qi) {
    const int q = (qb * 4 + wave) * QW + qi;
    if (q >= L) break;  // wave-uniform
    ++nq;
    bf16* Pq = P + qi * Lp;
    const bf16* qrow = base + (int64_t)q * ld + h * 64;
    float qv[64];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bf16x8 v = *(const bf16x8*)(qrow + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) qv[c * 8 + e] = bf2f(v[e]);
    }
    float mx = -INFINITY;
    float sv[T5_MAX_L / 64];  // this lane's scores (register-resident: fully unrolled indices)
#pragma unroll
    for (int i = 0; i < T5_MAX_L / 64; ++i) sv[i] = -INFINITY;
#pragma unroll
    for (int i = 0; i < T5_MAX_L / 64; ++i) {
      const int j = lane + 64 * i;
      if (j >= L) break;
      float s = 0.f;
      const bf16* kr = Ks + j * KROW;
#pragma unroll
      for (int e = 0; e < 64; e += 2) {
        const bf16x2 k2 = *(const bf16x2*)(kr + e);
        s = __builtin_fmaf(qv[e], bf2f(k2[0]), s);
        s = __builtin_fmaf(qv[e + 1], bf2f(k2[1]), s);
      }
      float sc = rbf(rbf(s) + Bs[j - q + L - 1]);
      if (Ms[j] != 0.f) sc = rbf(sc + -3.3895313892515355e38f);
      sv[i] = sc;  // this lane's keys j = lane + 64 i
      mx = fmaxf(mx, sc);
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < T5_MAX_L / 64; ++i) {
      const int j = lane + 64 * i;
      if (j < L) {
        sv[i] = __expf(sv[i] - mx);
        sum += sv[i];
      }
    }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
#pragma unroll
    for (int i = 0; i < T5_MAX_L / 64; ++i) {
      const int j = lane + 64 * i;
      if (j < L) Pq[j] = f2bf(sv[i] * inv);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  // out[q][d = lane] = sum_j w_qj v_j[d]
  float acc[QW];
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) acc[qi] = 0.f;
  for (int j = 0; j < L; ++j) {
    const float v = bf2f(Vs[j * 64 + lane]);
#pragma unroll
    for (int qi = 0; qi < QW; ++qi) acc[qi] = __builtin_fmaf(bf2f(P[qi * Lp + j]), v, acc[qi]);
  }
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) {
    const int q = (qb * 4 + wave) * QW + qi;
    if (qi < nq) out[(int64_t)(b * L + q) * ldo + h * 64 + lane] = f2bf(acc[qi]);
  }
}

// MFMA form (default; the scalar kernel above stays as the A/B, VP_T5_ATTN=scalar).  One workgroup per (batch, head,
// 64 queries), 4 waves x 16 queries.  K [Lp][64] (16-byte chunk c of row r at c ^ (r & 7)) and V^T [64][Lp + 4] of
// the head in LDS, keys padded to whole 32-key chunks (zero rows).  S^T = K Q^T on v_mfma_f32_16x16x32_bf16 (A = 16
// key rows from LDS, B = this wave's 16 queries from global, two MFMAs per 16 keys over d = 64): lane (ql, g) holds
// the scores of query ql for keys 16 kb + 4 g + r.  The same roundings as the scalar kernel: bf16(q.k) + bias (bf16
// add), the dtype minimum on masked keys, fp32 softmax (max / sum across the 4 lane groups), bf16 weights; then
// O^T = V^T P^T on the same MFMA, 32 keys per step: the B operand's K-slots 8 g .. 8 g + 7 hold this lane's keys
// {4 g .. 4 g + 3} and {16 + 4 g .. 16 + 4 g + 3} of the chunk straight from the score layout, and the A operand
// reads V^T at the same keys (two 8-byte reads per row).  fp32 accumulation, one bf16 rounding at the store.
constexpr int T5M_MAXKB = T5_MAX_L / 16;

__global__ __launch_bounds__(256, 2) void t5_attention_mfma_kernel(const bf16* __restrict__ qkv, int64_t ld, int inner,
                                                                int L, int H, const bf16* __restrict__ bias_table,
                                                                const int32_t* __restrict__ buckets,
                                                                const int64_t* __restrict__ mask, bf16* __restrict__ out,
                                                                int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lp = (L + 31) & ~31;
  const int VS = Lp + 4;
  bf16* Ks = (bf16*)smem;              // [Lp][64]
  bf16* Vt = Ks + Lp * 64;             // [64][VS]
  float* Bs = (float*)(Vt + 64 * VS);  // [2 Lp]: bias by relative position j - q + L - 1
  float* Ms = Bs + 2 * Lp;             // [Lp]: 1 where the key is masked
  const int nqb = (L + 63) / 64;
  const int bh = blockIdx.x / nqb, qb = blockIdx.x - bh * nqb;
  const int b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* base = qkv + (int64_t)b * L * ld;
  for (int i = tid; i < Lp * 8; i += 256) {
    const int j = i >> 3, c = i & 7;
    bf16x8 kv, vv;
    if (j < L) {
      kv = *(const bf16x8*)(base + (int64_t)j * ld + inner + h * 64 + c * 8);
      vv = *(const bf16x8*)(base + (int64_t)j * ld + 2 * inner + h * 64 + c * 8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) kv[e] = vv[e] = (bf16)0.f;
    }
    *(bf16x8*)(Ks + j * 64 + ((c ^ (j & 7)) << 3)) = kv;
#pragma unroll
    for (int e = 0; e < 8; ++e) Vt[(c * 8 + e) * VS + j] = vv[e];
  }
  for (int r = tid; r < 2 * L - 1; r += 256) {
    const int rel = r - (L - 1);
    const int bk = rel >= 0 ? buckets[rel] : buckets[(int64_t)(-rel) * L];
    Bs[r] = bf2f(bias_table[bk * H + h]);
  }
  for (int j = tid; j < L; j += 256) Ms[j] = (mask != nullptr && mask[(int64_t)b * L + j] == 0) ? 1.f : 0.f;
  __syncthreads();

  const int ql = lane & 15, g = lane >> 4;
  const int q = qb * 64 + wave * 16 + ql;
  const int qc = q < L ? q : L - 1;  // rows past L compute on the last query and are not stored
  const bf16* qrow = base + (int64_t)qc * ld + h * 64;
  const bf16x8 qf0 = *(const bf16x8*)(qrow + 8 * g), qf1 = *(const bf16x8*)(qrow + 32 + 8 * g);
  const int nkb = Lp >> 4;
  f32x4 s[T5M_MAXKB];
#pragma unroll
  for (int kb = 0; kb < T5M_MAXKB; ++kb) {
    if (kb < nkb) {  // wave-uniform (no break: the loop must unroll for s[] to stay in registers)
      const int r = kb * 16 + ql;
      const bf16x8 a0 = *(const bf16x8*)(Ks + r * 64 + ((g ^ (r & 7)) << 3));
      const bf16x8 a1 = *(const bf16x8*)(Ks + r * 64 + (((4 + g) ^ (r & 7)) << 3));
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
      z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, qf0, z, 0, 0, 0);
      s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, qf1, z, 0, 0, 0);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < T5M_MAXKB; ++kb) {
    if (kb < nkb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = kb * 16 + 4 * g + r;
        float t = -INFINITY;
        if (k < L) {
          t = rbf(rbf(s[kb][r]) + Bs[k - qc + L - 1]);
          if (Ms[k] != 0.f) t = rbf(t + -3.3895313892515355e38f);
        }
        s[kb][r] = t;
        mx = fmaxf(mx, t);
      }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < T5M_MAXKB; ++kb) {
    if (kb < nkb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = kb * 16 + 4 * g + r < L ? __expf(s[kb][r] - mx) : 0.f;
        s[kb][r] = p;
        sum += p;
      }
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  f32x4 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < T5M_MAXKB / 2; ++c) {
    if (2 * c < nkb) {
      bf16x8 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pb[r] = f2bf(s[2 * c][r] * inv);
        pb[4 + r] = f2bf(s[2 * c + 1][r] * inv);
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16* vr = Vt + (db * 16 + ql) * VS + 32 * c + 4 * g;
        const bf16x4 lo = *(const bf16x4*)vr, hi = *(const bf16x4*)(vr + 16);
        const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb, o[db], 0, 0, 0);
      }
    }
  }
  if (q < L) {
    bf16* orow = out + (int64_t)(b * L + q) * ldo + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[db][r]);
      *(bf16x4*)(orow + db * 16 + 4 * g) = v;
    }
  }
}

int grid_for(int64_t work) {
  const int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > (1 << 20) ? (1 << 20) : g));
}

}  // namespace

extern "C" int vp_embedding_gather_bf16(const void* table, const int64_t* ids, void* out, int32_t rows, int32_t D,
                                        int32_t vocab, void* stream) {
  if (table == nullptr || ids == nullptr || out == nullptr || rows <= 0 || D <= 0 || (D % 8) || vocab <= 0)
    return VP_ERR_ARG;
  hipLaunchKernelGGL(embed_gather_kernel, dim3(grid_for((int64_t)rows * (D / 8))), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)table, ids, (bf16*)out, rows, D, vocab);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_rms_norm_bf16(const void* x, const void* w, void* y, int32_t rows, int32_t D, float eps,
                                void* stream) {
  if (x == nullptr || w == nullptr || y == nullptr || rows <= 0 || D <= 0 || (D % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(rms_norm_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (const bf16*)w, (bf16*)y, rows, D, eps);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_mul_bf16(const void* a, const void* b, void* y, int64_t n, void* stream) {
  if (a == nullptr || b == nullptr || y == nullptr || n <= 0 || (n % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(mul_kernel, dim3(grid_for(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)a,
                     (const bf16*)b, (bf16*)y, n / 8);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_t5_attention_bf16(const void* qkv, int64_t ld, int32_t inner, int32_t B, int32_t L, int32_t H,
                                    const void* bias_table, const int32_t* buckets, const int64_t* mask, void* out,
                                    int64_t ldo, void* stream) {
  if (qkv == nullptr || bias_table == nullptr || buckets == nullptr || out == nullptr) return VP_ERR_ARG;
  if (B <= 0 || L <= 0 || H <= 0 || inner != H * 64 || ld < 3 * inner || (ld % 8) || ldo < inner) return VP_ERR_ARG;
  if (L > T5_MAX_L) return VP_ERR_UNSUPPORTED;
  const char* ev = vp_knob(VPK_T5_ATTN);
  if (ev == nullptr || strcmp(ev, "scalar") != 0) {  // the MFMA kernel (default)
    if ((ldo % 4) != 0) return VP_ERR_ARG;
    const size_t Lp32 = (size_t)((L + 31) & ~31);
    const size_t lds_m = Lp32 * 64 * 2 + 64 * (Lp32 + 4) * 2 + 3 * Lp32 * 4;
    static bool attr_m = false;
    if (!attr_m) {
      const size_t mx = (size_t)T5_MAX_L * 64 * 2 + 64 * (T5_MAX_L + 4) * 2 + 3 * T5_MAX_L * 4;
      (void)hipFuncSetAttribute((const void*)t5_attention_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)mx);
      attr_m = true;
    }
    const int nqb_m = (L + 63) / 64;
    hipLaunchKernelGGL(t5_attention_mfma_kernel, dim3(B * H * nqb_m), dim3(256), lds_m, (hipStream_t)stream,
                       (const bf16*)qkv, ld, inner, L, H, (const bf16*)bias_table, buckets, mask, (bf16*)out, ldo);
    VP_CHECK_LAUNCH();
    return 0;
  }
  const size_t Lp = (size_t)((L + 7) & ~7);
  const size_t lds = Lp * KROW * 2 + Lp * 64 * 2 + 3 * Lp * 4 + 4 * QW * Lp * 2;
  static bool attr = false;
  if (!attr) {
    const size_t mx = (size_t)T5_MAX_L * (KROW * 2 + 64 * 2 + 12 + 8 * QW);
    (void)hipFuncSetAttribute((const void*)t5_attention_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mx);
    attr = true;
  }
  const int nqb = (L + 4 * QW - 1) / (4 * QW);
  hipLaunchKernelGGL(t5_attention_kernel, dim3(B * H * nqb), dim3(256), lds, (hipStream_t)stream,
                     (const bf16*)qkv, ld, inner, L, H, (const bf16*)bias_table, buckets, mask, (bf16*)out, ldo);
  VP_CHECK_LAUNCH();
  return 0;
}
