// Flash-attention forward for CogVideoX joint 3D attention on gfx950 (MI355X): head_dim 64, non-causal, no mask,
// N up to ~47k tokens, optional second K/V segment (the ID-resample processor's doubled K/V, reference
// DF/models/attention_processor.py:2283-2290) and an output blend (the prev-clip path :2177-2189).
//
// Layout of the math (one wave = 32 queries, one workgroup = 8 waves = 256 queries of one (batch, head)):
//   S^T[key][q] = K · Q^T        v_mfma_f32_32x32x16_bf16, A = K rows from LDS (ds_read_b128, XOR-swizzled),
//                                B = Q^T held in registers for the whole key loop.
//   The accumulator has the query on the lane, so the online-softmax state (running max m, sum l) is per lane and
//   the row max is 31 in-register fmax + one cross-half shuffle.
//   O^T[d][q] += V^T · P^T      A = V^T read with ds_read_b64_tr_b16 (hardware transpose) from a padded V image,
//                                B = P^T taken straight from the S^T accumulator registers (bf16-packed, with the
//                                k-order permutation of cdna_hip_programming.md §3 "accumulator tile as operand").
//   O^T keeps the query on the lane too, so the rescale by exp(m_old - m_new) is a per-lane scalar.
// K/V tiles of 64 keys are double-buffered in LDS with register staging (global loads issued before the tile's
// MFMAs, LDS writes after them; one barrier per tile).
// Roofline: MFMA-bound in principle (4·N²·64 flop per (b,h)); at d=64 the softmax VALU (one exp per 256 MFMA
// flops) is the co-bottleneck.
#include <stdlib.h>

#include "vp_common.h"

namespace {

constexpr int NWAVES = 8;
constexpr int NTHREADS = NWAVES * 64;
constexpr int QBLK = NWAVES * 32;   // 256 queries per workgroup
constexpr int KBLK = 64;            // keys per tile
constexpr int K_TILE_BYTES = KBLK * 128;
constexpr int V_STRIDE = 192;       // bytes per V row in LDS (128 data + 64 pad: conflict-free transposed reads)
constexpr int V_TILE_BYTES = KBLK * V_STRIDE;
constexpr int STAGE_BYTES = K_TILE_BYTES + V_TILE_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

VP_DEV int swz(int row) { return (row >> 1) & 7; }

struct Seg {
  const bf16* k;
  const bf16* v;
  int64_t k_sn, v_sn;
  int n;
  int key0;
};

VP_DEV Seg tile_seg(const vp_attn_desc& d, int ti, int tiles1, int b, int h) {
  Seg s;
  if (ti < tiles1) {
    s.k = (const bf16*)d.K + (int64_t)b * d.k_sb + h * 64;
    s.v = (const bf16*)d.V + (int64_t)b * d.v_sb + h * 64;
    s.k_sn = d.k_sn;
    s.v_sn = d.v_sn;
    s.n = d.Nk;
    s.key0 = ti * KBLK;
  } else {
    s.k = (const bf16*)d.K2 + (int64_t)b * d.k2_sb + h * 64;
    s.v = (const bf16*)d.V2 + (int64_t)b * d.v2_sb + h * 64;
    s.k_sn = d.k2_sn;
    s.v_sn = d.v2_sn;
    s.n = d.Nk2;
    s.key0 = (ti - tiles1) * KBLK;
  }
  return s;
}

// ------------------------------------------------------------------------------------------------------------
// v2: software-pipelined tile loop.  Within one wave the next tile's S^T = K Q^T MFMAs are issued ahead of the
// current tile's softmax VALU work (they are independent), so the matrix pipe and the VALU overlap inside each
// wave instead of alternating at every barrier; 3-slot LDS ring (tile t: V in use, t+1: K in use, t+2: landing),
// register staging one tile ahead; the O rescale is skipped when no query's running max moved.
// ------------------------------------------------------------------------------------------------------------
constexpr int RING = 3;
constexpr int LDS_BYTES_V2 = RING * STAGE_BYTES;

VP_DEV void qk_tile(const char* Kl, const bf16x8 (&qf)[4], f32x16 (&s)[2], int lane) {
  const int hl = lane >> 5;
  bf16x8 kf[2][4];  // all 8 fragment reads in flight before the first MFMA
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const int row = kh * 32 + (lane & 31);
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      const int ch = ds * 2 + hl;
      kf[kh][ds] = *(const bf16x8*)(Kl + row * 128 + ((ch ^ swz(row)) << 4));
    }
  }
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[kh][i] = 0.f;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kh][ds], qf[ds], s[kh], 0, 0, 0);
  }
}

VP_DEV void mask_tail(f32x16 (&s)[2], int lim, int hl) {
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kh * 32 + (i & 3) + 8 * (i >> 2) + 4 * hl;
      if (key >= lim) s[kh][i] = -INFINITY;
    }
}

VP_DEV void softmax_tile(f32x16 (&s)[2], float& m_run, float& l_run, f32x16 (&o)[2], bf16x8 (&pf)[4], float c) {
  // max over the lane's 32 scores as 4 independent v_max3_f32 chains (short dependency chains: the wave has
  // little other work to hide latency behind); the file is built with -fno-honor-nans so no canonicalising v_max
  // is inserted on the MFMA results
  float m4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x16& v = s[j >> 1];
    const int o = (j & 1) * 8;
    m4[j] = fmaxf(fmaxf(fmaxf(v[o], v[o + 1]), v[o + 2]), fmaxf(fmaxf(v[o + 3], v[o + 4]), v[o + 5]));
    m4[j] = fmaxf(fmaxf(m4[j], v[o + 6]), v[o + 7]);
  }
  float mx = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float m_new = fmaxf(m_run, mx);
  if (__ballot(m_new > m_run) != 0ull) {  // wave-uniform: some query's max moved -> rescale O and l
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * c);
    l_run *= alpha;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[0][i] *= alpha;
      o[1][i] *= alpha;
    }
    m_run = m_new;
  }
  const float mc = m_run * c;
  float ps[4] = {0.f, 0.f, 0.f, 0.f};  // 4 independent partial sums (8-deep chains instead of one 32-deep)
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __builtin_amdgcn_exp2f(fmaf(s[kh][i], c, -mc));
      ps[i & 3] += p;
      pf[kh * 2 + (i >> 3)][i & 7] = f2bf(p);
    }
  l_run += (ps[0] + ps[1]) + (ps[2] + ps[3]);
}

VP_DEV void pv_tile(const char* Vl, const bf16x8 (&pf)[4], f32x16 (&o)[2], int trow, int tcol) {
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const char* base = Vl + (ks * 16 + trow) * V_STRIDE + (dh * 32 + tcol) * 2;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)base);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + 8 * V_STRIDE));
      const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[ks], o[dh], 0, 0, 0);
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// Main kernel: NW waves x 32 queries per workgroup, one barrier per 64-key tile, 2-slot LDS ring with register
// staging (global loads for tile t+1 issued before tile t's MFMAs, written to LDS after them).  With NW = 4 two
// workgroups share a CU, so their waves are not barrier-locked to each other and one workgroup's softmax VALU runs
// beside the other's MFMAs.
// ------------------------------------------------------------------------------------------------------------
template <int NW>
__global__ __launch_bounds__(NW * 64, 2) void attn_fwd_t(const vp_attn_desc d) {
  constexpr int NT = NW * 64;
  constexpr int QB = NW * 32;
  constexpr int CH_PER_THREAD = (KBLK * 8) / NT;  // 16-byte chunks of a K (and of a V) tile per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane >> 5;

  const int nqb = (d.Nq + QB - 1) / QB;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;
  const int tiles1 = (d.Nk + KBLK - 1) / KBLK;
  const int tiles2 = d.Nk2 > 0 ? (d.Nk2 + KBLK - 1) / KBLK : 0;
  const int ntiles = tiles1 + tiles2;

  const int q = qb * QB + wave * 32 + (lane & 31);
  const int qc = q < d.Nq ? q : d.Nq - 1;
  const bf16* qrow = (const bf16*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
  bf16x8 qf[4];
#pragma unroll
  for (int ds = 0; ds < 4; ++ds) qf[ds] = *(const bf16x8*)(qrow + ds * 16 + hl * 8);

  int k_off[CH_PER_THREAD], v_off[CH_PER_THREAD], srow[CH_PER_THREAD], sch[CH_PER_THREAD];
#pragma unroll
  for (int i = 0; i < CH_PER_THREAD; ++i) {
    const int cidx = tid + i * NT;
    srow[i] = cidx >> 3;
    sch[i] = cidx & 7;
    k_off[i] = srow[i] * 128 + ((sch[i] ^ swz(srow[i])) << 4);
    v_off[i] = K_TILE_BYTES + srow[i] * V_STRIDE + sch[i] * 16;
  }
  bf16x8 kreg[CH_PER_THREAD], vreg[CH_PER_THREAD];
  // Per-chunk source pointers advance by one tile per call; recomputed (with the row clamp) only at a segment start
  // or for a segment's partial last tile, so the steady-state address math is one 64-bit add per chunk.
  const bf16* kp[CH_PER_THREAD];
  const bf16* vp[CH_PER_THREAD];
  auto gload = [&](int ti) {
    Seg sg = tile_seg(d, ti, tiles1, b, h);
    const bool fresh = (ti == 0) || (ti == tiles1) || (sg.key0 + KBLK > sg.n);
#pragma unroll
    for (int i = 0; i < CH_PER_THREAD; ++i) {
      if (fresh) {
        const int key = min(sg.key0 + srow[i], sg.n - 1);
        kp[i] = sg.k + (int64_t)key * sg.k_sn + sch[i] * 8;
        vp[i] = sg.v + (int64_t)key * sg.v_sn + sch[i] * 8;
      } else {
        kp[i] += KBLK * sg.k_sn;
        vp[i] += KBLK * sg.v_sn;
      }
      kreg[i] = *(const bf16x8*)kp[i];
      vreg[i] = *(const bf16x8*)vp[i];
    }
  };
  auto lstore = [&](char* slotp) {
#pragma unroll
    for (int i = 0; i < CH_PER_THREAD; ++i) {
      *(bf16x8*)(slotp + k_off[i]) = kreg[i];
      *(bf16x8*)(slotp + v_off[i]) = vreg[i];
    }
  };

  gload(0);
  lstore(smem);
  __syncthreads();

  const float c = d.scale * 1.4426950408889634f;
  float m_run = -1e30f, l_run = 0.f;
  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.f;
    o[1][i] = 0.f;
  }
  const int g = lane >> 4;
  const int trow = 4 * (g >> 1) + ((lane & 15) >> 2);
  const int tcol = 16 * (g & 1) + 4 * (lane & 3);

  for (int ti = 0; ti < ntiles; ++ti) {
    const char* Kl = smem + (ti & 1) * STAGE_BYTES;
    const bool has_next = ti + 1 < ntiles;
    if (has_next) gload(ti + 1);
    f32x16 s[2];
    qk_tile(Kl, qf, s, lane);
    {
      Seg sg = tile_seg(d, ti, tiles1, b, h);
      const int lim = sg.n - sg.key0;
      if (lim < KBLK) mask_tail(s, lim, hl);
    }
    bf16x8 pf[4];
    softmax_tile(s, m_run, l_run, o, pf, c);
    pv_tile(Kl + K_TILE_BYTES, pf, o, trow, tcol);
    if (has_next) lstore(smem + ((ti + 1) & 1) * STAGE_BYTES);
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / l_tot;
  if (q < d.Nq) {
    bf16* orow = (bf16*)d.O + (int64_t)b * d.o_sb + (int64_t)q * d.o_sn + h * 64;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int dd = dh * 32 + 8 * gq + 4 * hl;
        bf16x4 ov;
        bf16x4 old;
        if (d.accumulate) old = *(const bf16x4*)(orow + dd);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = rbf(o[dh][4 * gq + r] * inv);
          if (d.out_scale != 1.f) v = rbf(v * d.out_scale);
          if (d.accumulate) v = bf2f(old[r]) + v;
          ov[r] = f2bf(v);
        }
        *(bf16x4*)(orow + dd) = ov;
      }
  }
}

__global__ __launch_bounds__(NTHREADS, 2) void attn_fwd_kernel_v2(const vp_attn_desc d) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane >> 5;

  const int nqb = (d.Nq + QBLK - 1) / QBLK;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;

  const int tiles1 = (d.Nk + KBLK - 1) / KBLK;
  const int tiles2 = d.Nk2 > 0 ? (d.Nk2 + KBLK - 1) / KBLK : 0;
  const int ntiles = tiles1 + tiles2;

  const int q = qb * QBLK + wave * 32 + (lane & 31);
  const int qc = q < d.Nq ? q : d.Nq - 1;
  const bf16* qrow = (const bf16*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
  bf16x8 qf[4];
#pragma unroll
  for (int ds = 0; ds < 4; ++ds) qf[ds] = *(const bf16x8*)(qrow + ds * 16 + hl * 8);

  const int srow = tid >> 3;
  const int schunk = tid & 7;
  const int k_lds_off = srow * 128 + ((schunk ^ swz(srow)) << 4);
  const int v_lds_off = K_TILE_BYTES + srow * V_STRIDE + schunk * 16;
  auto slot = [&](int ti) -> char* { return smem + (ti % RING) * STAGE_BYTES; };
  auto gload = [&](int ti, bf16x8& kr, bf16x8& vr) {
    Seg s = tile_seg(d, ti, tiles1, b, h);
    int key = s.key0 + srow;
    key = key < s.n ? key : s.n - 1;
    kr = *(const bf16x8*)(s.k + (int64_t)key * s.k_sn + schunk * 8);
    vr = *(const bf16x8*)(s.v + (int64_t)key * s.v_sn + schunk * 8);
  };
  auto tile_limit = [&](int ti) -> int {  // valid keys in tile ti (64 unless it is a segment's partial tail)
    Seg s = tile_seg(d, ti, tiles1, b, h);
    return min(KBLK, s.n - s.key0);
  };

  bf16x8 kreg, vreg;
  gload(0, kreg, vreg);
  *(bf16x8*)(slot(0) + k_lds_off) = kreg;
  *(bf16x8*)(slot(0) + v_lds_off) = vreg;
  if (ntiles > 1) {
    gload(1, kreg, vreg);
    *(bf16x8*)(slot(1) + k_lds_off) = kreg;
    *(bf16x8*)(slot(1) + v_lds_off) = vreg;
  }
  __syncthreads();
  if (ntiles > 2) gload(2, kreg, vreg);

  const float c = d.scale * 1.4426950408889634f;
  float m_run = -1e30f, l_run = 0.f;
  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.f;
    o[1][i] = 0.f;
  }
  const int g = lane >> 4;
  const int trow = 4 * (g >> 1) + ((lane & 15) >> 2);
  const int tcol = 16 * (g & 1) + 4 * (lane & 3);

  f32x16 sa[2], sb[2];
  qk_tile(slot(0), qf, sa, lane);

  auto body = [&](f32x16 (&scur)[2], f32x16 (&snxt)[2], int ti) {
    if (ti + 1 < ntiles) qk_tile(slot(ti + 1), qf, snxt, lane);
    const int lim = tile_limit(ti);
    if (lim < KBLK) mask_tail(scur, lim, hl);
    bf16x8 pf[4];
    softmax_tile(scur, m_run, l_run, o, pf, c);
    pv_tile(slot(ti) + K_TILE_BYTES, pf, o, trow, tcol);
    if (ti + 2 < ntiles) {
      *(bf16x8*)(slot(ti + 2) + k_lds_off) = kreg;
      *(bf16x8*)(slot(ti + 2) + v_lds_off) = vreg;
    }
    __syncthreads();
    if (ti + 3 < ntiles) gload(ti + 3, kreg, vreg);
  };
  for (int ti = 0; ti < ntiles; ti += 2) {
    body(sa, sb, ti);
    if (ti + 1 < ntiles) body(sb, sa, ti + 1);
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / l_tot;
  if (q < d.Nq) {
    bf16* orow = (bf16*)d.O + (int64_t)b * d.o_sb + (int64_t)q * d.o_sn + h * 64;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int dd = dh * 32 + 8 * gq + 4 * hl;
        bf16x4 ov;
        bf16x4 old;
        if (d.accumulate) old = *(const bf16x4*)(orow + dd);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = rbf(o[dh][4 * gq + r] * inv);
          if (d.out_scale != 1.f) v = rbf(v * d.out_scale);
          if (d.accumulate) v = bf2f(old[r]) + v;
          ov[r] = f2bf(v);
        }
        *(bf16x4*)(orow + dd) = ov;
      }
  }
}

}  // namespace

extern "C" int vp_attention_fwd_bf16(const vp_attn_desc* d, void* stream) {
  if (d == nullptr || d->Q == nullptr || d->K == nullptr || d->V == nullptr || d->O == nullptr) return VP_ERR_ARG;
  if (d->head_dim != 64) return VP_ERR_UNSUPPORTED;
  if (d->B <= 0 || d->H <= 0 || d->Nq <= 0 || d->Nk <= 0 || d->Nk2 < 0) return VP_ERR_ARG;
  if (d->Nk2 > 0 && (d->K2 == nullptr || d->V2 == nullptr)) return VP_ERR_ARG;
  if ((d->q_sn % 8) || (d->k_sn % 8) || (d->v_sn % 8) || (d->o_sn % 4) || (d->q_sb % 8) || (d->k_sb % 8) ||
      (d->v_sb % 8) || (d->o_sb % 4))
    return VP_ERR_ARG;
  if (d->Nk2 > 0 && ((d->k2_sn % 8) || (d->v2_sn % 8) || (d->k2_sb % 8) || (d->v2_sb % 8))) return VP_ERR_ARG;
  static bool attr_set = false;
  const char* e = getenv("VP_ATTN_VARIANT");  // A/B switch for benchmarking kernel variants
  const int variant = (e != nullptr && e[0] >= '1' && e[0] <= '9') ? e[0] - '0' : 1;
  if (!attr_set) {
    attr_set = true;
    (void)hipFuncSetAttribute((const void*)attn_fwd_t<8>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)attn_fwd_t<4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)attn_fwd_kernel_v2, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES_V2);
  }
  const int nw = (variant == 3) ? 4 : 8;
  const int nqb = (d->Nq + nw * 32 - 1) / (nw * 32);
  const int64_t grid = (int64_t)d->B * d->H * nqb;
  if (grid > 0x7fffffff) return VP_ERR_ARG;
  if (variant == 2)
    hipLaunchKernelGGL(attn_fwd_kernel_v2, dim3((unsigned)grid), dim3(NTHREADS), LDS_BYTES_V2, (hipStream_t)stream,
                       *d);
  else if (variant == 3)
    hipLaunchKernelGGL(attn_fwd_t<4>, dim3((unsigned)grid), dim3(256), LDS_BYTES, (hipStream_t)stream, *d);
  else
    hipLaunchKernelGGL(attn_fwd_t<8>, dim3((unsigned)grid), dim3(512), LDS_BYTES, (hipStream_t)stream, *d);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
