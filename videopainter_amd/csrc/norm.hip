// Row normalisations on the CogVideoX block path (gfx950).  All HBM-bound: one pass over bf16 rows, 16-byte
// vector loads/stores, fp32 statistics (two-pass mean/variance from registers, like torch's LayerNorm), bf16
// rounding at the same points as the reference's bf16 module chain.
#include "vp_common.h"

namespace {

constexpr int ROW_THREADS = 256;   // 4 waves, one row per wave
constexpr int MAXC = 8;            // up to 8 x 16-byte chunks per lane  ->  D <= 4096

// Load one row of D bf16 (D % 8 == 0) into per-lane registers, chunk c of the row handled by lane c % 64.
struct RowRegs {
  float v[MAXC][8];
};

VP_DEV void load_row(const bf16* row, int nch, int lane, RowRegs& r) {
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      const bf16x8 x = *(const bf16x8*)(row + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) r.v[i][e] = bf2f(x[e]);
    }
  }
}

VP_DEV void row_stats(const RowRegs& r, int nch, int lane, int D, float& mean, float& rstd, float eps) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i)
    if (lane + i * 64 < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += r.v[i][e];
  mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i)
    if (lane + i * 64 < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = r.v[i][e] - mean;
        q += t * t;
      }
  rstd = rsqrtf(wave_sum(q) / (float)D + eps);
}

// AdaLN row body: x (this wave's row as NCH bf16 chunks per lane) -> normalised, modulated row (same arithmetic,
// in the same order, as the reference chain: LayerNorm in fp32 from bf16, bf16 rounding after the affine, after
// (1 + scale), after the product and after + shift)
template <bool MX, int NCH>
VP_DEV void adaln_row(bf16x8 (&xr)[NCH], int row, int lane, int Ntok, int D, int text_len, const bf16* __restrict__ lw,
                      const bf16* __restrict__ lb, float eps, const bf16* __restrict__ mod, int64_t mod_bs,
                      void* __restrict__ y, uint8_t* __restrict__ yscale, int64_t ldy) {
  const int b = row / Ntok;
  const int tok = row - b * Ntok;
  const int nch = D / 8;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i)
    if (lane + i * 64 < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += bf2f(xr[i][e]);
  const float mean = wave_sum(s) / (float)D;
  // opaque: keep the row as bf16 (re-widened per use, 1 VALU) instead of 8 floats per chunk across the reductions
#pragma unroll
  for (int i = 0; i < NCH; ++i) asm volatile("" : "+v"(xr[i]));
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i)
    if (lane + i * 64 < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = bf2f(xr[i][e]) - mean;
        q += t * t;
      }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < NCH; ++i) asm volatile("" : "+v"(xr[i]));
  const bool text = tok < text_len;
  const bf16* shift = mod + (int64_t)b * mod_bs + (text ? 3 : 0) * D;
  const bf16* scale = mod + (int64_t)b * mod_bs + (text ? 4 : 1) * D;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      const bf16x8 w = *(const bf16x8*)(lw + c * 8);
      const bf16x8 bb = *(const bf16x8*)(lb + c * 8);
      const bf16x8 sh = *(const bf16x8*)(shift + c * 8);
      const bf16x8 sc = *(const bf16x8*)(scale + c * 8);
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float n = rbf((bf2f(xr[i][e]) - mean) * rstd * bf2f(w[e]) + bf2f(bb[e]));
        const float s1 = rbf(1.f + bf2f(sc[e]));
        f[e] = rbf(rbf(n * s1) + bf2f(sh[e]));
      }
      if constexpr (MX) {
        uint8_t sb;
        const u32x2 qq = mx_quantize_quarter(f, sb);
        *(u32x2*)((uint8_t*)y + (int64_t)row * D + c * 8) = qq;
        if ((c & 3) == 0) yscale[mx_scale_off(row, c >> 2, D)] = sb;
      } else {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(f[e]);
        *(bf16x8*)((bf16*)y + (int64_t)row * ldy + c * 8) = o;
      }
    }
    // one chunk's parameter loads live at a time (hoisting all 4 x NCH of them costs 96 VGPRs and half the
    // occupancy; the other resident rows cover their L2 latency)
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NCH>
VP_DEV void load_row_bf16(bf16x8 (&xr)[NCH], const bf16* __restrict__ xrow, int lane, int nch) {
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * 64;
    if (c < nch) xr[i] = *(const bf16x8*)(xrow + c * 8);
  }
}

// ---- AdaLN-Zero modulate (DF/models/normalization.py:373-379) ----
// MX = true: the modulated row is written as MX-FP8 (e4m3 + E8M0 per 32 columns, include/vp_hip.h) for the fp8
// FeedForward — a 32-column block is 4 consecutive 8-column chunks = 4 consecutive lanes of the row's wave.
// HBM-latency bound: one row's load -> reduce -> store chain leaves the memory pipe idle unless many rows overlap.
// The row stays in registers as bf16 (NCH 16-byte chunks per lane, 4 VGPRs each: 24 VGPRs at D = 3072).
// One row per wave, 6-7 waves per SIMD (70-76 VGPRs): 4.4-4.5 TB/s at config 2 (3.8 with the row held as floats, 116
// VGPRs).  Measured and dropped (tools/gpu_ab_norms.sh): persistent waves prefetching the next row (126 VGPRs,
// 3.7 TB/s); 512-thread blocks staging the affine + shift / scale in LDS (3.4-3.5 TB/s); 8 waves/SIMD with 10
// spilled VGPRs (3.1 TB/s).
template <bool MX, int NCH>
__global__ __launch_bounds__(ROW_THREADS) void adaln_modulate_kernel(const bf16* __restrict__ x, void* __restrict__ y,
                                                                        uint8_t* __restrict__ yscale,
                                                                        int rows, int Ntok, int D, int text_len,
                                                                        const bf16* __restrict__ lw,
                                                                        const bf16* __restrict__ lb, float eps,
                                                                        const bf16* __restrict__ mod, int64_t mod_bs,
                                                                        int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  bf16x8 xr[NCH];
  load_row_bf16<NCH>(xr, x + (int64_t)row * D, lane, D / 8);
  adaln_row<MX, NCH>(xr, row, lane, Ntok, D, text_len, lw, lb, eps, mod, mod_bs, y, yscale, ldy);
}

template <bool MX>
void launch_adaln(int rows, hipStream_t s, const bf16* x, void* y, uint8_t* ys, int Ntok, int D,
                  int text_len, const bf16* lw, const bf16* lb, float eps, const bf16* mod, int64_t mod_bs,
                  int64_t ldy) {
  const int nch = (D / 8 + 63) / 64;  // 16-byte chunks per lane
  const int grid = (rows + 3) / 4;
#define VP_ADALN(N) hipLaunchKernelGGL((adaln_modulate_kernel<MX, N>), dim3(grid), dim3(ROW_THREADS), 0, s, x, y, ys, \
                                       rows, Ntok, D, text_len, lw, lb, eps, mod, mod_bs, ldy)
  if (nch <= 1) VP_ADALN(1);
  else if (nch <= 2) VP_ADALN(2);
  else if (nch <= 4) VP_ADALN(4);
  else if (nch <= 6) VP_ADALN(6);
  else VP_ADALN(8);
#undef VP_ADALN
}

// ---- final norm_final + norm_out (cogvideox_transformer_3d.py:617-624; normalization.py:73-85) ----
__global__ __launch_bounds__(ROW_THREADS) void final_norm_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                                 int rows, int Nv, int Ntok, int D, int text_len,
                                                                 const bf16* __restrict__ w1,
                                                                 const bf16* __restrict__ b1,
                                                                 const bf16* __restrict__ w2,
                                                                 const bf16* __restrict__ b2, float eps,
                                                                 const bf16* __restrict__ mod, int64_t mod_bs) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int b = row / Nv;
  const int v = row - b * Nv;
  const int nch = D / 8;
  RowRegs r;
  load_row(x + ((int64_t)b * Ntok + text_len + v) * D, nch, lane, r);
  float mean, rstd;
  row_stats(r, nch, lane, D, mean, rstd, eps);
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      const bf16x8 w = *(const bf16x8*)(w1 + c * 8);
      const bf16x8 bb = *(const bf16x8*)(b1 + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) r.v[i][e] = rbf((r.v[i][e] - mean) * rstd * bf2f(w[e]) + bf2f(bb[e]));
    }
  }
  row_stats(r, nch, lane, D, mean, rstd, eps);
  const bf16* shift = mod + (int64_t)b * mod_bs;
  const bf16* scale = shift + D;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      const bf16x8 w = *(const bf16x8*)(w2 + c * 8);
      const bf16x8 bb = *(const bf16x8*)(b2 + c * 8);
      const bf16x8 sh = *(const bf16x8*)(shift + c * 8);
      const bf16x8 sc = *(const bf16x8*)(scale + c * 8);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float n = rbf((r.v[i][e] - mean) * rstd * bf2f(w[e]) + bf2f(bb[e]));
        o[e] = f2bf(rbf(n * rbf(1.f + bf2f(sc[e]))) + bf2f(sh[e]));
      }
      *(bf16x8*)(y + (int64_t)row * D + c * 8) = o;
    }
  }
}

// ---- per-head LN(64) + RoPE (attention_processor.py:2143-2154; embeddings.py:655-701) ----
// 4 lanes per 64-wide head vector, 16 elements each in the MFMA-accumulator column order of ln64_rope16 (lane g
// holds columns 16 j + 4 g + r: four 8-byte pieces) — the arithmetic of the QKV GEMM's fused epilogue.  Each 4-lane
// group takes HPG heads of one token (h = hg + k H / HPG: at step k the groups of a token read consecutive heads):
// the LayerNorm affine and the token's cos / sin quads, the same for every head, are loaded once per group, and the
// HPG vectors' loads are in flight together (one vector per group: 16 of the 20 loads were the shared operands, and
// one HBM load chain per thread left the stream at 3 TB/s).  64 groups per 256-thread block.  FP8: the bf16 value
// the bf16 kernel writes, times out_mul, as e4m3 (strides then in bytes)
template <bool FP8, int HPG>
__global__ __launch_bounds__(256) void head_norm_rope_kernel(const bf16* __restrict__ xin, int64_t ld_in,
                                                            int64_t bs_in, void* __restrict__ xout, int64_t ld_out,
                                                            int64_t bs_out, int64_t ngroups, int Ntok, int H,
                                                            int text_len, const bf16* __restrict__ lw,
                                                            const bf16* __restrict__ lb, float eps,
                                                            const float* __restrict__ cosp,
                                                            const float* __restrict__ sinp,
                                                            const uint8_t* __restrict__ tok_mask, int64_t mask_bs,
                                                            float pre_scale, float out_mul,
                                                            const int32_t* __restrict__ dst_rows) {
  const int64_t grp = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
  const int g = threadIdx.x & 3;
  const bool valid = grp < ngroups;
  const int64_t gg = valid ? grp : ngroups - 1;
  const int Hg = H / HPG;
  const int hg = (int)(gg % Hg);
  const int64_t bn = gg / Hg;
  const int n = (int)(bn % Ntok);
  const int b = (int)(bn / Ntok);
  const int nd = dst_rows != nullptr ? dst_rows[(int64_t)b * Ntok + n] : n;
  if (nd < 0) return;  // a row the caller does not need (uniform over the group's 4 lanes; no block barrier here)
  const bf16* src = xin + (int64_t)b * bs_in + (int64_t)n * ld_in + hg * 64 + g * 4;
  bf16x4 xr[HPG][4];
#pragma unroll
  for (int k = 0; k < HPG; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) xr[k][j] = *(const bf16x4*)(src + k * Hg * 64 + 16 * j);
  const bool rot = cosp != nullptr && n >= text_len;
  const float* cr = rot ? cosp + (int64_t)(n - text_len) * 64 : nullptr;
  const float* sr = rot ? sinp + (int64_t)(n - text_len) * 64 : nullptr;
  bf16x4 w[4], bb[4];
  f32x4 cs[4], sn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 16 * j + 4 * g;
    w[j] = *(const bf16x4*)(lw + c);
    bb[j] = *(const bf16x4*)(lb + c);
    cs[j] = rot ? *(const f32x4*)(cr + c) : (f32x4){1.f, 1.f, 1.f, 1.f};
    sn[j] = rot ? *(const f32x4*)(sr + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  float m = 1.f;
  if (tok_mask != nullptr) m = tok_mask[(int64_t)b * mask_bs + n] ? 1.f : 0.f;
  const int64_t o0 = (int64_t)b * bs_out + (int64_t)nd * ld_out + hg * 64 + g * 4;
#pragma unroll
  for (int k = 0; k < HPG; ++k) {
    float x[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = bf2f(xr[k][j][r]);
        if (tok_mask != nullptr) t = rbf(rbf(t * m) * pre_scale);
        x[4 * j + r] = t;
      }
    ln64_rope16_regs<1, 2>(x, w, bb, eps, cs, sn, rot);
    if (valid) {
      const int64_t o = o0 + k * Hg * 64;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (FP8) {
          int wd = 0;
          float y[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = __builtin_amdgcn_fmed3f(rbf(x[4 * j + r]) * out_mul, 448.f, -448.f);
          wd = __builtin_amdgcn_cvt_pk_fp8_f32(y[0], y[1], wd, false);
          wd = __builtin_amdgcn_cvt_pk_fp8_f32(y[2], y[3], wd, true);
          *(uint32_t*)((uint8_t*)xout + o + 16 * j) = (uint32_t)wd;
        } else {
          bf16x4 ov;
#pragma unroll
          for (int r = 0; r < 4; ++r) ov[r] = f2bf(x[4 * j + r]);
          *(bf16x4*)((bf16*)xout + o + 16 * j) = ov;
        }
      }
    }
  }
}

#ifndef VP_HNR_HPG
#define VP_HNR_HPG 4  // A/B build: 1 = one head per lane group (round 6 before)
#endif
// the launch: VP_HNR_HPG heads per lane group when H is a multiple of it, else 1
template <bool FP8>
void launch_head_norm_rope(hipStream_t s, const bf16* xin, int64_t ld_in, int64_t bs_in, void* xout, int64_t ld_out,
                           int64_t bs_out, int B, int Ntok, int H, int text_len, const bf16* lw, const bf16* lb,
                           float eps, const float* cosp, const float* sinp, const uint8_t* tok_mask, int64_t mask_bs,
                           float pre_scale, float out_mul, const int32_t* dst_rows) {
  const int hpg = H % VP_HNR_HPG == 0 ? VP_HNR_HPG : 1;
  const int64_t ngroups = (int64_t)B * Ntok * (H / hpg);
  const dim3 grid((unsigned)((ngroups + 63) / 64));
  if (hpg == 4)  // (VP_HNR_HPG is 1 or 4)
    hipLaunchKernelGGL((head_norm_rope_kernel<FP8, 4>), grid, dim3(256), 0, s, xin, ld_in, bs_in, xout, ld_out,
                       bs_out, ngroups, Ntok, H, text_len, lw, lb, eps, cosp, sinp, tok_mask, mask_bs, pre_scale,
                       out_mul, dst_rows);
  else
    hipLaunchKernelGGL((head_norm_rope_kernel<FP8, 1>), grid, dim3(256), 0, s, xin, ld_in, bs_in, xout, ld_out,
                       bs_out, ngroups, Ntok, H, text_len, lw, lb, eps, cosp, sinp, tok_mask, mask_bs, pre_scale,
                       out_mul, dst_rows);
}

__global__ __launch_bounds__(256) void mask_scale_rows_kernel(const bf16* __restrict__ xin, int64_t ld_in,
                                                             int64_t bs_in, bf16* __restrict__ y, int64_t ld_out,
                                                             int64_t bs_out, int64_t nchunks, int Ntok, int D,
                                                             const uint8_t* __restrict__ tok_mask, int64_t mask_bs,
                                                             float scale, const int32_t* __restrict__ dst_rows) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nchunks) return;
  const int cpr = D / 8;
  const int c = (int)(i % cpr);
  const int64_t bn = i / cpr;
  const int n = (int)(bn % Ntok);
  const int b = (int)(bn / Ntok);
  const int nd = dst_rows != nullptr ? dst_rows[(int64_t)b * Ntok + n] : n;
  if (nd < 0) return;  // a row the caller does not need
  const float m = tok_mask[(int64_t)b * mask_bs + n] ? 1.f : 0.f;
  const bf16x8 x = *(const bf16x8*)(xin + (int64_t)b * bs_in + (int64_t)n * ld_in + c * 8);
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(rbf(rbf(bf2f(x[e]) * m) * scale));
  *(bf16x8*)(y + (int64_t)b * bs_out + (int64_t)nd * ld_out + c * 8) = o;
}

// ---- stable partition index of the resample processor's token mask (vp_partition_rows_index): one workgroup per
// batch row; rows with mask != 0 go first in order, the others after them in order ----
__global__ __launch_bounds__(1024) void partition_index_kernel(const uint8_t* __restrict__ mask, int64_t mask_bs, int N,
                                                              int32_t* __restrict__ dst, int32_t* __restrict__ counts) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint8_t* m = mask + (int64_t)b * mask_bs;
  // pass 1: the number of set rows
  int cnt = 0;
  for (int n = tid; n < N; n += 1024) cnt += m[n] != 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane == 0) wsum[wv] = cnt;
  __syncthreads();
  int total = 0;
  for (int w = 0; w < 16; ++w) total += wsum[w];
  if (tid == 0) {
    counts[b] = total;
    carry = 0;
  }
  __syncthreads();
  // pass 2: 1024-row chunks, exclusive scan of the set flags
  for (int base = 0; base < N; base += 1024) {
    const int n = base + tid;
    const int f = (n < N && m[n] != 0) ? 1 : 0;
    const unsigned long long bal = __ballot(f);
    const int below = __popcll(bal & ((1ull << lane) - 1ull));
    __syncthreads();  // wsum reuse
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < wv; ++w) pre += wsum[w];
    pre += below;  // set rows before n
    if (n < N) dst[(int64_t)b * N + n] = f ? pre : total + (n - pre);
    __syncthreads();
    if (tid == 0) {
      int add = 0;
      for (int w = 0; w < 16; ++w) add += wsum[w];
      carry += add;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int vp_adaln_modulate_bf16(const void* x, void* y, int64_t ldy, int32_t B, int32_t Ntok, int32_t D,
                                      int32_t text_len, const void* ln_w, const void* ln_b, float eps,
                                      const void* mod, int64_t mod_bstride, void* stream) {
  if (!x || !y || !ln_w || !ln_b || !mod || B <= 0 || Ntok <= 0 || D <= 0 || (D % 8) || D > MAXC * 512)
    return VP_ERR_ARG;
  if ((mod_bstride % 8) || ldy < D || (ldy % 8)) return VP_ERR_ARG;
  const int rows = B * Ntok;
  launch_adaln<false>(rows, (hipStream_t)stream, (const bf16*)x, y, nullptr, Ntok, D, text_len,
                      (const bf16*)ln_w, (const bf16*)ln_b, eps, (const bf16*)mod, mod_bstride, ldy);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_adaln_modulate_mx_fp8(const void* x, void* q, void* scales, int32_t B, int32_t Ntok, int32_t D,
                                        int32_t text_len, const void* ln_w, const void* ln_b, float eps,
                                        const void* mod, int64_t mod_bstride, void* stream) {
  if (!x || !q || !scales || !ln_w || !ln_b || !mod || B <= 0 || Ntok <= 0 || D <= 0 || (D % 128) || D > MAXC * 512)
    return VP_ERR_ARG;
  if (mod_bstride % 8) return VP_ERR_ARG;
  const int rows = B * Ntok;
  launch_adaln<true>(rows, (hipStream_t)stream, (const bf16*)x, q, (uint8_t*)scales, Ntok, D, text_len,
                     (const bf16*)ln_w, (const bf16*)ln_b, eps, (const bf16*)mod, mod_bstride, D);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_final_norm_bf16(const void* x, void* y, int32_t B, int32_t Ntok, int32_t D, int32_t text_len,
                                  const void* ln1_w, const void* ln1_b, const void* ln2_w, const void* ln2_b,
                                  float eps, const void* mod, int64_t mod_bstride, void* stream) {
  if (!x || !y || !ln1_w || !ln1_b || !ln2_w || !ln2_b || !mod) return VP_ERR_ARG;
  if (B <= 0 || Ntok <= text_len || D <= 0 || (D % 8) || D > MAXC * 512 || (mod_bstride % 8)) return VP_ERR_ARG;
  const int Nv = Ntok - text_len;
  const int rows = B * Nv;
  hipLaunchKernelGGL(final_norm_kernel, dim3((rows + 3) / 4), dim3(ROW_THREADS), 0, (hipStream_t)stream,
                     (const bf16*)x, (bf16*)y, rows, Nv, Ntok, D, text_len, (const bf16*)ln1_w, (const bf16*)ln1_b,
                     (const bf16*)ln2_w, (const bf16*)ln2_b, eps, (const bf16*)mod, mod_bstride);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_head_norm_rope_bf16(const void* x_in, int64_t ld_in, int64_t bs_in, void* x_out, int64_t ld_out,
                                      int64_t bs_out, int32_t B, int32_t Ntok, int32_t H, int32_t text_len,
                                      const void* ln_w, const void* ln_b, float eps, const float* cos,
                                      const float* sin, const uint8_t* tok_mask, int64_t mask_bstride,
                                      float pre_scale, const int32_t* dst_rows, void* stream) {
  if (!x_in || !x_out || !ln_w || !ln_b || B <= 0 || Ntok <= 0 || H <= 0) return VP_ERR_ARG;
  if (dst_rows != nullptr && x_in == x_out) return VP_ERR_ARG;  // a permuted write must not alias its input
  if ((ld_in % 8) || (ld_out % 8) || (bs_in % 8) || (bs_out % 8)) return VP_ERR_ARG;
  if ((cos == nullptr) != (sin == nullptr)) return VP_ERR_ARG;
  launch_head_norm_rope<false>((hipStream_t)stream, (const bf16*)x_in, ld_in, bs_in, x_out, ld_out, bs_out, B, Ntok, H,
                               text_len, (const bf16*)ln_w, (const bf16*)ln_b, eps, cos, sin, tok_mask, mask_bstride,
                               pre_scale, 1.f, dst_rows);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_head_norm_rope_fp8(const void* x_in, int64_t ld_in, int64_t bs_in, void* q_out, int64_t ld_out,
                                     int64_t bs_out, int32_t B, int32_t Ntok, int32_t H, int32_t text_len,
                                     const void* ln_w, const void* ln_b, float eps, const float* cos,
                                     const float* sin, float out_mul, void* stream) {
  if (!x_in || !q_out || !ln_w || !ln_b || B <= 0 || Ntok <= 0 || H <= 0) return VP_ERR_ARG;
  if ((ld_in % 8) || (bs_in % 8) || (ld_out % 8) || (bs_out % 8)) return VP_ERR_ARG;
  if ((cos == nullptr) != (sin == nullptr) || !(out_mul > 0.f)) return VP_ERR_ARG;
  launch_head_norm_rope<true>((hipStream_t)stream, (const bf16*)x_in, ld_in, bs_in, q_out, ld_out, bs_out, B, Ntok, H,
                              text_len, (const bf16*)ln_w, (const bf16*)ln_b, eps, cos, sin, nullptr, 0, 1.f, out_mul,
                              nullptr);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_mask_scale_rows_bf16(const void* x_in, int64_t ld_in, int64_t bs_in, void* y, int64_t ld_out,
                                       int64_t bs_out, int32_t B, int32_t Ntok, int32_t D, const uint8_t* tok_mask,
                                       int64_t mask_bstride, float scale, const int32_t* dst_rows, void* stream) {
  if (!x_in || !y || !tok_mask || B <= 0 || Ntok <= 0 || D <= 0 || (D % 8)) return VP_ERR_ARG;
  if (dst_rows != nullptr && x_in == y) return VP_ERR_ARG;
  if ((ld_in % 8) || (ld_out % 8) || (bs_in % 8) || (bs_out % 8)) return VP_ERR_ARG;
  const int64_t nchunks = (int64_t)B * Ntok * (D / 8);
  hipLaunchKernelGGL(mask_scale_rows_kernel, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)x_in, ld_in, bs_in, (bf16*)y, ld_out, bs_out, nchunks, Ntok,
                     D, tok_mask, mask_bstride, scale, dst_rows);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_partition_rows_index(const uint8_t* mask, int64_t mask_bstride, int32_t B, int32_t N,
                                       int32_t* dst_rows, int32_t* counts, void* stream) {
  if (!mask || !dst_rows || !counts || B <= 0 || N <= 0 || mask_bstride < N) return VP_ERR_ARG;
  hipLaunchKernelGGL(partition_index_kernel, dim3((unsigned)B), dim3(1024), 0, (hipStream_t)stream, mask,
                     mask_bstride, N, dst_rows, counts);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
