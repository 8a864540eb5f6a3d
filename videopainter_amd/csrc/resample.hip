// The ID-resample processor's null keys in closed form on gfx950 (MI355X): vp_mask_null_segments and
// vp_null_key_mass (include/vp_hip.h).  Reference: DF/models/attention_processor.py:2223-2304 (the masked K/V copy;
// LN of a zeroed row = the norm_k bias), DF/models/embeddings.py:457-530 (get_3d_rotary_pos_embed: the separable 3D
// RoPE) and :655-701 (apply_rotary_emb, interleaved pairs).
//
// A null key is LN(0) = beta (the norm_k bias), rotated by its video position's RoPE (text rows: beta itself); its
// value is zero, so it only adds exp2(score) to its query's row sum.  Each dim of a rotated key depends on one axis
// of the position only: dims 0-15 on the frame t, 16-39 on the row y, 40-63 on the column x (the host verifies the
// table, kernels.rope_axis_tables), so with the per-axis key pieces K_t(t) [16], K_y(y) [24], K_x(x) [24] (each
// rounded to bf16 exactly like the rotated key the reference builds)
//   score(q, null key at (t, y, x)) = S_t(t) + S_y(y) + S_x(x),  S_a(p) = c q_a . K_a(p)  (c = scale * log2 e)
//   sum over null (t, y, x) of 2^score = 2^(mt + my + mx) sum_t E_t(t) sum_y E_y(y) sum_{x null in (t, y)} E_x(x)
// with E_a = 2^(S_a - max S_a).  A frame's null pattern is a list of segments — runs of consecutive rows with the
// same null columns, themselves a few runs (vp_mask_null_segments, once per mask) — so per query the triple sum is
// a few prefix-sum differences per segment: 88 short dot products, 88 exp2 and a few hundred LDS reads, instead of a
// 64-wide dot product and an exp2 for each of the ~N null keys in the attention kernel.
#include "vp_common.h"

namespace {

constexpr int NM_R = 6;     // runs per segment record; rows with more are their own segment, scanned per column
constexpr int NM_NT = 128;  // threads (queries) per block of the mass kernel
constexpr int NM_MAXF = 16;
constexpr int NM_MAXH = 64;  // rows per frame: one lane each in the segment kernel
// the mass kernel's p loops unrolled by VP_NM_UNROLL: independent dot-product chains (and prefix-sum reads) in flight
// together instead of one 24-deep dependent FMA chain at a time; every chain keeps its own order (same results)
#ifndef VP_NM_UNROLL
#define VP_NM_UNROLL 4
#endif
// query chunks of NM_NT per block: the block's prologue (the key-piece tables and segment records into LDS, a chain of
// dependent global loads) is paid once per NM_CH chunks
constexpr int NM_CH = 4;
// (Measured and dropped, profiles/r05_null_key_mass_ab.log: the per-axis scores of a wave's 64 queries as 32x32x16
// MFMAs written to LDS for the same per-query pass — 0.79 against 0.47 ms at config 4: the dot products are not what
// the kernel waits on, the extra LDS pass of the scores is.)

// one wave per (b, t): lane y finds the null runs of row y, equal neighbouring rows merge into segments.
// segs[((b F + t) Hh + i)] (16 bytes): byte 0 = y0, 1 = y1 (exclusive), 2 = run count (255: scan the row),
// bytes 4 + 2k, 5 + 2k = run k's [start, end) columns.  meta[b F + t] = segment count, meta[B F + b] = text rows with
// mask 0.  Rows without a null key make no segment.
__global__ __launch_bounds__(64) void mask_null_segments_kernel(const uint8_t* __restrict__ mask, int64_t mask_bs,
                                                                int B, int T, int F, int Hh, int Ww,
                                                                uint4* __restrict__ segs, int* __restrict__ meta) {
  const int bt = blockIdx.x;
  const int b = bt / F, t = bt - b * F;
  const int lane = threadIdx.x;
  const uint8_t* mb = mask + (int64_t)b * mask_bs;
  uint32_t w1 = 0, w2 = 0, w3 = 0;
  int n = 0;
  if (lane < Hh) {
    const uint8_t* mrow = mb + T + ((int64_t)t * Hh + lane) * Ww;
    int s = -1;
    for (int x = 0; x <= Ww; ++x) {
      const bool z = x < Ww && mrow[x] == 0;
      if (z && s < 0) s = x;
      if (!z && s >= 0) {  // run [s, x) ends: its (start, end) bytes go to slot n of w1..w3
        const uint32_t pr = (uint32_t)s | ((uint32_t)x << 8);
        const uint32_t sh = (n & 1) ? pr << 16 : pr;
        w1 |= n < 2 ? sh : 0u;
        w2 |= (n >> 1) == 1 ? sh : 0u;
        w3 |= (n >> 1) == 2 ? sh : 0u;
        ++n;
        s = -1;
      }
    }
  }
  const int nf = n > NM_R ? 255 : n;
  const uint32_t pn = __shfl_up((uint32_t)nf, 1, 64), p1 = __shfl_up(w1, 1, 64), p2 = __shfl_up(w2, 1, 64),
                 p3 = __shfl_up(w3, 1, 64);
  const bool same = lane > 0 && nf != 255 && (uint32_t)nf == pn && w1 == p1 && w2 == p2 && w3 == p3;
  const bool start = lane < Hh && !same;
  const uint64_t starts = __ballot(start);
  const uint64_t later = lane < 63 ? starts >> (lane + 1) : 0ull;
  const int y1 = later ? lane + 1 + __builtin_ctzll(later) : Hh;
  const bool keep = start && nf != 0;
  const uint64_t kept = __ballot(keep);
  if (keep) {
    const int idx = __builtin_popcountll(kept & ((1ull << lane) - 1ull));
    segs[((int64_t)b * F + t) * Hh + idx] = make_uint4((uint32_t)lane | ((uint32_t)y1 << 8) | ((uint32_t)nf << 16),
                                                       w1, w2, w3);
  }
  if (lane == 0) meta[b * F + t] = __builtin_popcountll(kept);
  if (t == 0) {
    int tn = 0;
    for (int i0 = 0; i0 < T; i0 += 64) {
      const int i = i0 + lane;
      tn += __builtin_popcountll(__ballot(i < T && mb[i] == 0));
    }
    if (lane == 0) meta[B * F + b] = tn;
  }
}

VP_DEV float rbf16(float v) { return bf2f(f2bf(v)); }

// one thread per (b, h, query), NM_NT queries of one (b, h) per block.  Dynamic LDS:
//   kt [F][16], ky [Hh][24], kx [Ww][24] (the rotated-beta pieces), seg [F][Hh] records, nseg [F] + text count,
//   py [Hh + 1][NM_NT], px [Ww + 1][NM_NT] (this thread's E_y / E_x prefix sums in column tid)
__global__ __launch_bounds__(NM_NT) void null_key_mass_kernel(
    const bf16* __restrict__ q, int64_t q_sb, int64_t q_sn, int H, int N, int T, int F, int Hh, int Ww,
    const bf16* __restrict__ beta, const float* __restrict__ ct, const float* __restrict__ st,
    const float* __restrict__ cy, const float* __restrict__ sy, const float* __restrict__ cx,
    const float* __restrict__ sx, const uint8_t* __restrict__ mask, int64_t mask_bs, const uint4* __restrict__ segs,
    const int* __restrict__ meta, int B, float c, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float nm_smem[];
  float* kt = nm_smem;
  float* ky = kt + F * 16;
  float* kx = ky + Hh * 24;
  uint4* sg = (uint4*)(kx + Ww * 24);  // (F*16 + (Hh + Ww)*24) floats: a multiple of 4
  int* nseg = (int*)(sg + F * Hh);
  float* py = (float*)(nseg + ((F + 1 + 3) & ~3));
  float* px = py + (Hh + 1) * NM_NT;
  const int tid = threadIdx.x;
  const int nqb = (N + NM_NT * NM_CH - 1) / (NM_NT * NM_CH);
  const int bh = blockIdx.x / nqb, qb = blockIdx.x - bh * nqb;
  const int b = bh / H, h = bh - b * H;

  // the rotated null key's dims, as head_norm_rope writes them: y0 = b0 c0 - b1 s0, y1 = b1 c1 + b0 s1, to bf16
  auto rot = [&](int d, float cs, float sn) {
    const float b0 = bf2f(beta[d & ~1]), b1 = bf2f(beta[d | 1]);
    return (d & 1) ? rbf16(b1 * cs + b0 * sn) : rbf16(b0 * cs - b1 * sn);
  };
  // (independent loads, unrolled so they are in flight together; every segment record slot is copied, used or not,
  // so no copy waits for the record counts)
#pragma unroll 4
  for (int i = tid; i < F * 16; i += NM_NT) kt[i] = rot(i & 15, ct[i], st[i]);
#pragma unroll 4
  for (int i = tid; i < Hh * 24; i += NM_NT) ky[i] = rot(16 + i % 24, cy[i], sy[i]);
#pragma unroll 4
  for (int i = tid; i < Ww * 24; i += NM_NT) kx[i] = rot(40 + i % 24, cx[i], sx[i]);
#pragma unroll 4
  for (int i = tid; i < F * Hh; i += NM_NT) sg[i] = segs[(int64_t)b * F * Hh + i];
  if (tid < F) nseg[tid] = meta[b * F + tid];
  if (tid == 0) nseg[F] = meta[B * F + b];
  __syncthreads();

#pragma unroll 1
  for (int ch = 0; ch < NM_CH; ++ch) {
    const int q0 = (qb * NM_CH + ch) * NM_NT;
    if (q0 >= N) break;  // (block-uniform)
    const int qi = q0 + tid;
    const int qc = qi < N ? qi : N - 1;
    const bf16* qrow = q + (int64_t)b * q_sb + (int64_t)qc * q_sn + h * 64;
    float qs[64];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x8 qv = *(const bf16x8*)(qrow + 8 * j);
#pragma unroll
      for (int e = 0; e < 8; ++e) qs[8 * j + e] = bf2f(qv[e]);
    }
    float s_text = 0.f;  // text rows: their null keys are beta itself (no rotation)
#pragma unroll
    for (int d = 0; d < 64; ++d) s_text += qs[d] * bf2f(beta[d]);
    s_text *= c;

    float et[NM_MAXF];
    float mt = -INFINITY, my = -INFINITY, mx = -INFINITY;
#pragma unroll
    for (int p = 0; p < NM_MAXF; ++p) {
      float sv = -INFINITY;
      if (p < F) {
        sv = 0.f;
#pragma unroll
        for (int dd = 0; dd < 16; ++dd) sv += qs[dd] * kt[p * 16 + dd];
        sv *= c;
      }
      et[p] = sv;
      mt = fmaxf(mt, sv);
    }
#pragma unroll VP_NM_UNROLL
    for (int p = 0; p < Hh; ++p) {
      float sv = 0.f;
#pragma unroll
      for (int dd = 0; dd < 24; ++dd) sv += qs[16 + dd] * ky[p * 24 + dd];
      sv *= c;
      py[(p + 1) * NM_NT + tid] = sv;
      my = fmaxf(my, sv);
    }
#pragma unroll VP_NM_UNROLL
    for (int p = 0; p < Ww; ++p) {
      float sv = 0.f;
#pragma unroll
      for (int dd = 0; dd < 24; ++dd) sv += qs[40 + dd] * kx[p * 24 + dd];
      sv *= c;
      px[(p + 1) * NM_NT + tid] = sv;
      mx = fmaxf(mx, sv);
    }
    float acc = 0.f;
    px[tid] = 0.f;
#pragma unroll VP_NM_UNROLL
    for (int p = 0; p < Ww; ++p) {
      acc += __builtin_amdgcn_exp2f(px[(p + 1) * NM_NT + tid] - mx);
      px[(p + 1) * NM_NT + tid] = acc;
    }
    acc = 0.f;
    py[tid] = 0.f;
#pragma unroll VP_NM_UNROLL
    for (int p = 0; p < Hh; ++p) {
      acc += __builtin_amdgcn_exp2f(py[(p + 1) * NM_NT + tid] - my);
      py[(p + 1) * NM_NT + tid] = acc;
    }
#pragma unroll
    for (int p = 0; p < NM_MAXF; ++p) et[p] = p < F ? __builtin_amdgcn_exp2f(et[p] - mt) : 0.f;

    const uint8_t* mv = mask + (int64_t)b * mask_bs + T;
    float zv = 0.f;
#pragma unroll
    for (int t = 0; t < NM_MAXF; ++t) {
      if (t >= F) break;
      const int ns = nseg[t];
      float zt = 0.f;
      for (int i = 0; i < ns; ++i) {
        const uint4 r = sg[t * Hh + i];
        const int y0 = r.x & 255, y1 = (r.x >> 8) & 255, n = (r.x >> 16) & 255;
        const float ey = py[y1 * NM_NT + tid] - py[y0 * NM_NT + tid];
        float zx = 0.f;
        if (n != 255) {
          const uint32_t w[3] = {r.y, r.z, r.w};
#pragma unroll
          for (int k = 0; k < NM_R; ++k) {
            if (k >= n) break;
            const uint32_t pr = w[k >> 1] >> (16 * (k & 1));
            zx += px[((pr >> 8) & 255) * NM_NT + tid] - px[(pr & 255) * NM_NT + tid];
          }
        } else {  // many runs: per column
          const uint8_t* mr = mv + ((int64_t)t * Hh + y0) * Ww;
          for (int x = 0; x < Ww; ++x)
            if (mr[x] == 0) zx += px[(x + 1) * NM_NT + tid] - px[x * NM_NT + tid];
        }
        zt += ey * zx;
      }
      zv += et[t] * zt;
    }
    if (qi < N) {
      // log2(text_null 2^s_text + zv 2^(mt + my + mx)), stably
      const int tn = nseg[F];
      const float lt = tn > 0 ? s_text + __log2f((float)tn) : -INFINITY;
      const float lv = zv > 0.f ? mt + my + mx + __log2f(zv) : -INFINITY;
      const float mm = fmaxf(lt, lv);
      float res = -INFINITY;
      if (mm > -INFINITY) res = mm + __log2f(__builtin_amdgcn_exp2f(lt - mm) + __builtin_amdgcn_exp2f(lv - mm));
      out[((int64_t)b * H + h) * N + qi] = res;
    }
  }
}

}  // namespace

extern "C" int vp_mask_null_segments(const uint8_t* mask, int64_t mask_bstride, int32_t B, int32_t T, int32_t F,
                                     int32_t Hh, int32_t Ww, void* segs, int32_t* meta, void* stream) {
  if (!mask || !segs || !meta || B <= 0 || T < 0 || F <= 0 || F > NM_MAXF || Hh <= 0 || Hh > NM_MAXH || Ww <= 0 ||
      Ww > 255)
    return VP_ERR_ARG;
  if (mask_bstride < (int64_t)T + (int64_t)F * Hh * Ww) return VP_ERR_ARG;
  hipLaunchKernelGGL(mask_null_segments_kernel, dim3((unsigned)(B * F)), dim3(64), 0, (hipStream_t)stream, mask,
                     mask_bstride, B, T, F, Hh, Ww, (uint4*)segs, meta);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int64_t vp_null_key_mass_lds_bytes(int32_t F, int32_t Hh, int32_t Ww) {
  return ((int64_t)F * 16 + (int64_t)(Hh + Ww) * 24) * 4 + (int64_t)F * Hh * 16 + (int64_t)((F + 1 + 3) & ~3) * 4 +
         ((int64_t)Hh + 1 + Ww + 1) * NM_NT * 4;
}

extern "C" int vp_null_key_mass(const void* q, int64_t q_sb, int64_t q_sn, int32_t B, int32_t H, int32_t N,
                                int32_t T, int32_t F, int32_t Hh, int32_t Ww, const void* beta, const float* cos_t,
                                const float* sin_t, const float* cos_y, const float* sin_y, const float* cos_x,
                                const float* sin_x, const uint8_t* mask, int64_t mask_bstride, const void* segs,
                                const int32_t* meta, float scale, float* out, void* stream) {
  if (!q || !beta || !cos_t || !sin_t || !cos_y || !sin_y || !cos_x || !sin_x || !mask || !segs || !meta || !out)
    return VP_ERR_ARG;
  if (B <= 0 || H <= 0 || N <= 0 || T < 0 || F <= 0 || F > NM_MAXF || Hh <= 0 || Hh > NM_MAXH || Ww <= 0 || Ww > 255)
    return VP_ERR_ARG;
  if ((int64_t)T + (int64_t)F * Hh * Ww != N || (q_sn % 8) || (q_sb % 8)) return VP_ERR_ARG;
  const int64_t lds = vp_null_key_mass_lds_bytes(F, Hh, Ww);
  if (lds > 160 * 1024) return VP_ERR_UNSUPPORTED;
  const void* kern = (const void*)null_key_mass_kernel;
  static int64_t attr = 64 * 1024;  // dynamic LDS the kernel may take (raised on demand)
  if (lds > attr) {
    const hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr = lds;
  }
  const int64_t nblk = (int64_t)B * H * ((N + NM_NT * NM_CH - 1) / (NM_NT * NM_CH));  // = B * H * nqb (kernels)
  if (nblk > 0x7fffffff) return VP_ERR_ARG;
  hipLaunchKernelGGL(null_key_mass_kernel, dim3((unsigned)nblk), dim3(NM_NT), (size_t)lds, (hipStream_t)stream,
                     (const bf16*)q, q_sb, q_sn, H, N, T, F, Hh, Ww, (const bf16*)beta, cos_t, sin_t, cos_y, sin_y,
                     cos_x, sin_x, mask, mask_bstride, (const uint4*)segs, (const int*)meta, B,
                     scale * 1.4426950408889634f, out);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
