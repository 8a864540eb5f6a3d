// Flash-attention backward for CogVideoX joint attention on gfx950 (the training caller's
// `accelerator.backward(loss)`, train/train_cogvideox_inpainting_i2v_video.py:1892, through
// F.scaled_dot_product_attention at DF/models/attention_processor.py:2192).  head_dim 64, non-causal, no mask.
//
// Given Q, K, V, the forward output O, the output gradient dO and the forward's softmax statistics
// lse = m + log2(l) (vp_attn_desc.lse, log2 units of c * q.k with c = scale * log2 e):
//   P = exp2(c q.k - lse),  dP = dO . V^T,  D = rowsum(dO * O),  dS = P * (dP - D)
//   dQ = scale * dS . K,   dK = scale * dS^T . Q,   dV = P^T . dO
// Three launches: the D rows; dQ with a workgroup per 128 queries looping over 64-key tiles (S^T = K Q^T with Q^T in
// registers, exactly the forward's layout, so P^T and dS^T leave the accumulator as the B operand of
// dQ^T += K^T dS^T, K^T read with ds_read_b64_tr_b16); dK / dV with a workgroup per 128 keys looping over 64-query
// tiles (S = Q K^T with K^T in registers: P and dS are the B operands of dV^T += dO^T P and dK^T += Q^T dS).  Every
// product on v_mfma_f32_32x32x16_bf16; tiles stream through a 2-slot LDS ring by LDS-DMA (global_load_lds_dwordx4,
// bank swizzle on the source address).  Roofline: MFMA (2.5 x the forward's 4 N^2 d FLOP per head: S twice, dP
// twice, dQ, dK, dV), VALU exp2 per score twice.
#include <stdlib.h>

#include "vp_common.h"

namespace {

constexpr int BW = 4;                 // waves per workgroup
constexpr int BT = 64;                // rows per streamed tile
constexpr int TILE = BT * 128;        // bytes of one 64 x 64 bf16 tile
constexpr int STAGE = 2 * TILE + 512; // two tiles + 64 fp32 lse + 64 fp32 D (dK/dV kernel)
constexpr int LDS_BWD = 2 * STAGE;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) void lds_void_t;

// bank swizzle of a staged tile: 16-B chunk c of row r sits at chunk c ^ swz(r).  V = 0 (round 2): (r >> 1) & 7,
// conflict-free for ds_read_b128 but 2-way for the transposing ds_read_b64_tr_b16 (rows 4m and 4m + 2 of one lane
// group land on the same banks).  V = 1: the same bijection of (r >> 1) & 7 with its low bit moved to bit 2, so rows
// 4m and 4m + 2 differ in chunk bit 2 — conflict-free for both reads (checked by enumerating the lane groups of
// MI355X_MICROARCH.md's LDS table); bits 1-3 of r only, so every 16-row slab has the same pattern.
template <int V>
VP_DEV int swz(int row) {
  return V ? (((row >> 2) & 3) | (((row >> 1) & 1) << 2)) : ((row >> 1) & 7);
}

VP_DEV void glds16(const char* sbase, int voff, char* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t*)lds;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(la), "v"(voff), "s"(sbase)
               : "memory", "m0");
}

// stage 64 rows of a [N, ld] bf16 head slice (64 columns from `base`) into a swizzled [64][128 B] LDS tile: 2 DMA
// pieces of 8 rows per wave (rows past `nrows` re-read the last row; the caller masks them)
template <int V>
VP_DEV void stage_tile(const bf16* base, int64_t ld, int row0, int nrows, char* tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pc = wave + i * BW;               // piece: tile rows pc*8 .. pc*8+7
    const int r = pc * 8 + (lane >> 3);
    const int rs = min(row0 + r, nrows - 1) - row0;
    const int ch = (lane & 7) ^ swz<V>(r);
    glds16((const char*)(base + (int64_t)row0 * ld), (int)((rs * ld + ch * 8) * 2), tile + pc * 1024);
  }
}

// V = 1: the two DMA source offsets of a full tile, computed once per kernel (kept VGPRs); only a partial last tile
// recomputes them with the row clamp.  (Per-tile 64-bit offset math let the compiler pair a dead high half with an
// unrelated register, whose pending load the loop then waited for before the DMA issue.)
struct TileOffs {
  int o[2];
};
VP_DEV TileOffs tile_offs(int64_t ld, int wave, int lane) {
  TileOffs t;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave + i * BW) * 8 + (lane >> 3);
    t.o[i] = (r * (int)ld + (((lane & 7) ^ swz<1>(r)) * 8)) * 2;
  }
  return t;
}
VP_DEV void stage_tile_fast(const bf16* base, int64_t ld, int row0, int nrows, char* tile, int wave, int lane,
                            const TileOffs& to) {
  if (row0 + BT <= nrows) {  // wave-uniform
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16((const char*)(base + (int64_t)row0 * ld), to.o[i], tile + (wave + i * BW) * 1024);
  } else {
    stage_tile<1>(base, ld, row0, nrows, tile, wave, lane);
  }
}

#ifndef VP_DKDV_OPQ
#define VP_DKDV_OPQ 1  // A/B: 0 = the dK / dV tile body on the kernel-wide lane offsets (spilled, round 6 before)
#endif
// the lane id from v_mbcnt in volatile asm: values derived from it are recomputed where they are used instead of being
// kept live (and spilled) across a loop
VP_DEV int lane_id_opaque() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// A-operand rows (ds_read_b128) of a 32-row half of a swizzled tile: chunk (2c + hl) ^ swz(row) = dims 16c + 8hl
template <int V>
VP_DEV void read_rows(const char* tile, int half, int lane, bf16x8 (&f)[4]) {
  const int hl = lane >> 5;
  const int row = half * 32 + (lane & 31);
  const char* rp = tile + row * 128;
  const int sw = swz<V>(row);
#pragma unroll
  for (int c = 0; c < 4; ++c) f[c] = *(const bf16x8*)(rp + (((2 * c + hl) ^ sw) << 4));
}

// A-operand of X^T (rows = the 64 columns in two 32-halves dh, k = 16 tile rows of slab `slab`) by transposing
// reads of the swizzled tile, in the k order of a 32x32 accumulator used as the B operand (lane group hl supplies
// rows {4hl..4hl+3, 8+4hl..8+4hl+3} of the slab): the forward's V^T read (attention.hip pv_half)
struct TrAddr {
  int lo[2], hi[2];
};
template <int V>
VP_DEV TrAddr tr_addr(int lane) {
  const int g = lane >> 4;
  const int trow = 4 * (g >> 1) + ((lane & 15) >> 2);
  const int tcol = 16 * (g & 1) + 4 * (lane & 3);
  TrAddr a;
#pragma unroll
  for (int dh = 0; dh < 2; ++dh) {
    const int chunk = dh * 4 + (tcol >> 3);
    a.lo[dh] = trow * 128 + ((chunk ^ swz<V>(trow)) << 4) + (tcol & 7) * 2;
    a.hi[dh] = (trow + 8) * 128 + ((chunk ^ swz<V>(trow + 8)) << 4) + (tcol & 7) * 2;
  }
  return a;
}
VP_DEV bf16x8 read_tr(const char* tile, int slab, const TrAddr& a, int dh) {
  const char* base = tile + slab * 16 * 128;  // swz depends on row bits 1-3: the same for every 16-row slab
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + a.lo[dh]));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + a.hi[dh]));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

VP_DEV f32x16 splat16(float v) {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = v;
  return z;
}

VP_DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// 8 fp32 -> bf16x8 as 4 pair conversions (v_cvt_pk_bf16_f32 each): element-wise inserts made the compiler add
// v_alignbit / v_perm shuffles and duplicate conversions (V = 1 only; the same RNE roundings)
typedef float f32v2 __attribute__((ext_vector_type(2)));
VP_DEV bf16x8 pack8(const float (&v)[8]) {
  u32x4 w;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16x2 h = __builtin_convertvector((f32v2){v[2 * e], v[2 * e + 1]}, bf16x2);
    w[e] = __builtin_bit_cast(uint32_t, h);
  }
  return __builtin_bit_cast(bf16x8, w);
}

// 32x32 accumulator element i of lane group hl sits in row 8 (i / 4) + 4 hl + i % 4
VP_DEV int acc_row(int i, int hl) { return 8 * (i >> 2) + 4 * hl + (i & 3); }

// store a transposed accumulator pair X^T (rows = 64 columns in halves dh, col = lane % 32 = this lane's row) as
// bf16 row `row` of a [N, ld] tensor, times `mul`
VP_DEV void store_rowT(bf16* rowp, const f32x16 (&x)[2], int hl, float mul) {
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(x[dh][4 * j + r] * mul);
      *(bf16x4*)(rowp + dh * 32 + 8 * j + 4 * hl) = v;
    }
}

// Grid tail (V = 1): the blocks of the last partial round run as nsplit pieces each over a range of the loop's tiles
// (keys for dQ, queries for dK / dV), dispatched after the whole blocks in the same launch; each piece leaves its fp32
// sums in `ws` ([piece][128 rows][64 dQ | 64 dK + 64 dV]) and bwd_tail_reduce_kernel adds them up.  Without it the
// last round ran 16 of 512 dQ workgroups (training shape: 6 672 blocks) and 528 of 768 dK / dV workgroups alone.
struct BwdSplit {
  int main_blocks;  // whole blocks (logical ids 0 .. main_blocks - 1, XCD-remapped); the tail blocks follow
  int nsplit;       // 1: no tail split
  float* ws;
};

// fp32 partial of a transposed accumulator pair in store_rowT's column order, row `row` of a [rows][ld] record
VP_DEV void store_partT(float* rowp, const f32x16 (&x)[2], int hl) {
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *(f32x4*)(rowp + dh * 32 + 8 * j + 4 * hl) = (f32x4){x[dh][4 * j], x[dh][4 * j + 1], x[dh][4 * j + 2], x[dh][4 * j + 3]};
}

// ---- D = rowsum(dO * O): one thread per (b, q, h), fp32 ----
__global__ __launch_bounds__(256) void bwd_delta_kernel(const vp_attn_bwd_desc d) {
  const int64_t total = (int64_t)d.B * d.Nq * d.H;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int h = (int)(i % d.H);
    const int64_t bq = i / d.H;
    const int q = (int)(bq % d.Nq), b = (int)(bq / d.Nq);
    const bf16* o = (const bf16*)d.O + (int64_t)b * d.o_sb + (int64_t)q * d.o_sn + h * 64;
    const bf16* g = (const bf16*)d.dO + (int64_t)b * d.do_sb + (int64_t)q * d.do_sn + h * 64;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bf16x8 a = *(const bf16x8*)(o + c * 8), bb = *(const bf16x8*)(g + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s = __builtin_fmaf(bf2f(a[e]), bf2f(bb[e]), s);
    }
    d.delta[((int64_t)b * d.H + h) * d.Nq + q] = s;
  }
}

// ---- dQ: a workgroup per (b, h, 128 queries), 64-key tiles ----
// V = 1 (default): conflict-free swizzle (swz<1>), the last partial key tile peeled out of the loop (the full-tile body
// is straight-line code without the per-score mask), inactive waves skip the compute as one block.  V = 0: round 2.
#ifndef VP_DQ_WAVES
#define VP_DQ_WAVES 2  // waves per SIMD the dQ kernel is register-budgeted for (A/B: -DVP_DQ_WAVES=3)
#endif
template <int V>
__global__ __launch_bounds__(BW * 64, VP_DQ_WAVES) void bwd_dq_kernel(const vp_attn_bwd_desc d, const BwdSplit sp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqb = (d.Nq + BW * 32 - 1) / (BW * 32);
  const int pj = (int)blockIdx.x - sp.main_blocks;
  const bool piece = sp.nsplit > 1 && pj >= 0;  // (V = 1 only: V = 0 launches unsplit)
  const int split = piece ? pj % sp.nsplit : 0;
  const int t = piece ? sp.main_blocks + pj / sp.nsplit : xcd_remap(blockIdx.x, sp.nsplit > 1 ? sp.main_blocks : gridDim.x);
  const int bh = t / nqb, qb = t - bh * nqb;
  const int b = bh / d.H, h = bh - b * d.H;
  const int q = qb * BW * 32 + wave * 32 + (lane & 31);
  const int qc = min(q, d.Nq - 1);
  const float c = d.scale * 1.4426950408889634f;
  // B operands: Q^T pre-scaled by c (the forward's rounding) and dO^T, from this lane's query row
  bf16x8 qf[4], gf[4];
  {
    const bf16* qr = (const bf16*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
    const bf16* gr = (const bf16*)d.dO + (int64_t)b * d.do_sb + (int64_t)qc * d.do_sn + h * 64;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      qf[ds] = *(const bf16x8*)(qr + ds * 16 + hl * 8);
      gf[ds] = *(const bf16x8*)(gr + ds * 16 + hl * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[ds][e] = f2bf(bf2f(qf[ds][e]) * c);
    }
  }
  const int64_t so = ((int64_t)b * d.H + h) * d.Nq + qc;
  const f32x16 negl = splat16(-d.lse[so]), negd = splat16(-d.delta[so]);
  const bf16* kb = (const bf16*)d.K + (int64_t)b * d.k_sb + h * 64;
  const bf16* vb = (const bf16*)d.V + (int64_t)b * d.v_sb + h * 64;
  const TrAddr ta = tr_addr<V>(lane);
  f32x16 dqt[2] = {zero16(), zero16()};
  const bool active = qb * BW * 32 + wave * 32 < d.Nq;  // wave-uniform
  const int ntiles = (d.Nk + BT - 1) / BT;
  const int tbeg = piece ? ntiles * split / sp.nsplit : 0, tend = piece ? ntiles * (split + 1) / sp.nsplit : ntiles;
  const TileOffs ko = tile_offs(d.k_sn, wave, lane), vo = tile_offs(d.v_sn, wave, lane);
  auto issue = [&](int ti) {
    char* st = smem + (ti & 1) * STAGE;
    if (V) {
      stage_tile_fast(kb, d.k_sn, ti * BT, d.Nk, st, wave, lane, ko);
      stage_tile_fast(vb, d.v_sn, ti * BT, d.Nk, st + TILE, wave, lane, vo);
    } else {
      stage_tile<V>(kb, d.k_sn, ti * BT, d.Nk, st, wave, lane);
      stage_tile<V>(vb, d.v_sn, ti * BT, d.Nk, st + TILE, wave, lane);
    }
  };
  // one 32-key half of a staged tile.  The accumulators start at -lse / -D (C-init), so P = exp2(S) and dS = P * dP
  // come straight off the matrix pipe: one exp and one multiply per score; with `lim` < BT (last tile only) keys past
  // Nk start at -inf instead
  auto half = [&](const char* Kt, const char* Vt, int kh, bool masked, int lim) {
    bf16x8 a[4];
    read_rows<V>(Kt, kh, lane, a);
    // first MFMA of each chain in asm with the loop-invariant C (dst != srcC: the -lse / -D registers are never
    // copied)
    f32x16 s, dp;
    if (!masked) {
      asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(s) : "v"(a[0]), "v"(qf[0]), "v"(negl));
    } else {
      f32x16 cm = negl;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (kh * 32 + acc_row(i, hl) >= lim) cm[i] = -INFINITY;
      // (builtin here: the compiler places the VALU-write -> MFMA-srcC wait states, which it does not for asm)
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], qf[0], cm, 0, 0, 0);
    }
#pragma unroll
    for (int ds = 1; ds < 4; ++ds) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ds], qf[ds], s, 0, 0, 0);
    read_rows<V>(Vt, kh, lane, a);
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(dp) : "v"(a[0]), "v"(gf[0]), "v"(negd));
#pragma unroll
    for (int ds = 1; ds < 4; ++ds) dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ds], gf[ds], dp, 0, 0, 0);
    bf16x8 pf[2];
    if (V) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float a[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] = __builtin_amdgcn_exp2f(s[8 * j + e]) * dp[8 * j + e];
        pf[j] = pack8(a);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) pf[i >> 3][i & 7] = f2bf(__builtin_amdgcn_exp2f(s[i]) * dp[i]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
        dqt[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Kt, kh * 2 + j, ta, dh), pf[j], dqt[dh], 0, 0, 0);
  };
  issue(tbeg);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (V == 0) {
    for (int ti = 0; ti < ntiles; ++ti) {
      if (ti + 1 < ntiles) issue(ti + 1);
      const char* Kt = smem + (ti & 1) * STAGE;
      const int lim = d.Nk - ti * BT;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        if (!active) break;
        half(Kt, Kt + TILE, kh, lim < BT, lim);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    const int nfull = d.Nk / BT;
    const int fend = min(tend, nfull);
    for (int ti = tbeg; ti < fend; ++ti) {
      if (ti + 1 < tend) issue(ti + 1);
      const char* Kt = smem + (ti & 1) * STAGE;
      if (active) {
        half(Kt, Kt + TILE, 0, false, BT);
        half(Kt, Kt + TILE, 1, false, BT);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (nfull < tend && active) {  // the partial last tile (staged by the last loop iteration, or the prologue)
      const char* Kt = smem + (nfull & 1) * STAGE;
      const int lim = d.Nk - nfull * BT;
      half(Kt, Kt + TILE, 0, true, lim);
      if (lim > 32) half(Kt, Kt + TILE, 1, true, lim);
    }
  }
  if (piece)
    store_partT(sp.ws + ((int64_t)pj * (BW * 32) + wave * 32 + (lane & 31)) * 64, dqt, hl);
  else if (q < d.Nq)
    store_rowT((bf16*)d.dQ + (int64_t)b * d.dq_sb + (int64_t)q * d.dq_sn + h * 64, dqt, hl, d.scale);
}

// ---- dK, dV: a workgroup per (b, h, 128 keys), 64-query tiles ----
// V = 1 (default): conflict-free swizzle; the next tile's per-query statistics loaded as raw values with no
// dependent instruction until they are stored to LDS after the compute (V = 0 negated them at once, which put an
// s_waitcnt vmcnt(0) — a wait for the whole next-tile DMA just issued — at the top of every tile); inactive waves
// skip the compute as one block.
// (round 6, measured and dropped: 2 waves per SIMD, +4-7 %; the four A fragments of a chain read before its first
// MFMA and kept live together, +14 % — the extra registers spill at 3 waves per SIMD; profiles/r06_attn_bwd_variants_ab.log)
template <int V>
__global__ __launch_bounds__(BW * 64, V ? 3 : 2) void bwd_dkdv_kernel(const vp_attn_bwd_desc d, const BwdSplit sp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkb = (d.Nk + BW * 32 - 1) / (BW * 32);
  const int pj = (int)blockIdx.x - sp.main_blocks;
  const bool piece = sp.nsplit > 1 && pj >= 0;
  const int split = piece ? pj % sp.nsplit : 0;
  const int t = piece ? sp.main_blocks + pj / sp.nsplit : xcd_remap(blockIdx.x, sp.nsplit > 1 ? sp.main_blocks : gridDim.x);
  const int bh = t / nkb, kb = t - bh * nkb;
  const int b = bh / d.H, h = bh - b * d.H;
  const int key = kb * BW * 32 + wave * 32 + (lane & 31);
  const int kc = min(key, d.Nk - 1);
  const float c = d.scale * 1.4426950408889634f;
  // B operands: K^T pre-scaled by c (so S comes out in log2 units) and V^T, from this lane's key row
  bf16x8 kf[4], vf[4];
  {
    const bf16* kr = (const bf16*)d.K + (int64_t)b * d.k_sb + (int64_t)kc * d.k_sn + h * 64;
    const bf16* vr = (const bf16*)d.V + (int64_t)b * d.v_sb + (int64_t)kc * d.v_sn + h * 64;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      kf[ds] = *(const bf16x8*)(kr + ds * 16 + hl * 8);
      vf[ds] = *(const bf16x8*)(vr + ds * 16 + hl * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) kf[ds][e] = f2bf(bf2f(kf[ds][e]) * c);
      // V = 1: consume V^T here (an empty asm use), so its load is complete before the loop; otherwise the wait
      // analysis cannot see the prologue's asm wait and places counted waits on it inside the loop, where the
      // in-order counter also holds the next tile's DMA
      if (V) asm volatile("" : "+v"(vf[ds]));
    }
  }
  const bf16* qb = (const bf16*)d.Q + (int64_t)b * d.q_sb + h * 64;
  const bf16* gb = (const bf16*)d.dO + (int64_t)b * d.do_sb + h * 64;
  const float* lse_row = d.lse + ((int64_t)b * d.H + h) * d.Nq;
  const float* d_row = d.delta + ((int64_t)b * d.H + h) * d.Nq;
  const float* stat_row = wave == 0 ? lse_row : d_row;  // (BT = 64: wave 0 holds the lse, wave 1 the D; scalar)
  const TrAddr ta = tr_addr<V>(lane);
  f32x16 dkt[2] = {zero16(), zero16()}, dvt[2] = {zero16(), zero16()};
  const bool active = kb * BW * 32 + wave * 32 < d.Nk;  // wave-uniform
  const int ntiles = (d.Nq + BT - 1) / BT;
  const int tbeg = piece ? ntiles * split / sp.nsplit : 0, tend = piece ? ntiles * (split + 1) / sp.nsplit : ntiles;
  // per-query statistics of a tile: thread tid < 64 holds lse, 64 <= tid < 128 D (plain loads, written to LDS after
  // the tile's compute, before the barrier that publishes the stage).  Rows past Nq: lse = +inf, so their S
  // accumulators start at -inf and P = 0 there (no per-score mask); stored negated: they are the C-init of the S / dP
  // accumulators
  float stat = 0.f;
  auto load_stat = [&](int ti) {
    const int qq = ti * BT + (tid & 63);
    if (V == 0) {
      if (tid < 2 * BT) stat = qq < d.Nq ? -(tid < BT ? lse_row[qq] : d_row[qq]) : (tid < BT ? -INFINITY : 0.f);
    } else {
      stat = stat_row[min(ti * BT + lane, d.Nq - 1)];  // every thread, in bounds; nothing uses it until put_stat
    }
  };
  auto put_stat = [&](int ti) {
    float v = stat;
    if (V != 0) {  // (every thread: the load's wait is then on every path, none is left to the next tile's DMA)
      const int qq = ti * BT + (tid & 63);
      v = qq < d.Nq ? -stat : (tid < BT ? -INFINITY : 0.f);
      v = __builtin_amdgcn_fmed3f(v, -INFINITY, INFINITY);
    }
    if (tid < 2 * BT) ((float*)(smem + (ti & 1) * STAGE + 2 * TILE))[tid] = v;
  };
  const TileOffs qo = tile_offs(d.q_sn, wave, lane), go = tile_offs(d.do_sn, wave, lane);
  auto issue = [&](int ti) {
    char* st = smem + (ti & 1) * STAGE;
    if (V) {
      stage_tile_fast(qb, d.q_sn, ti * BT, d.Nq, st, wave, lane, qo);
      stage_tile_fast(gb, d.do_sn, ti * BT, d.Nq, st + TILE, wave, lane, go);
    } else {
      stage_tile<V>(qb, d.q_sn, ti * BT, d.Nq, st, wave, lane);
      stage_tile<V>(gb, d.do_sn, ti * BT, d.Nq, st + TILE, wave, lane);
    }
  };
  auto half = [&](const char* Qt, const char* Gt, const float* st, int qh) {
    // S and dP accumulators start at -lse / -D of their query rows (C-init from the staged, negated statistics): P =
    // exp2(S), dS = P * dP, one exp and one multiply per score.  (V = 1: the lane's LDS offsets are recomputed here
    // from an opaque lane id; kept live across the tile loop they were spilled at this kernel's 168-register budget,
    // and each reload's vmcnt(0) also waited for the next tile's DMA.)
    const int ln = V && VP_DKDV_OPQ ? lane_id_opaque() : lane;
    const int hlq = ln >> 5;
    f32x16 s, dp;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r0 = qh * 32 + 8 * j + 4 * hlq;
      const f32x4 l4 = *(const f32x4*)(st + r0), d4 = *(const f32x4*)(st + BT + r0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[4 * j + r] = l4[r];
        dp[4 * j + r] = d4[r];
      }
    }
    bf16x8 a[4];
    read_rows<V>(Qt, qh, ln, a);
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ds], kf[ds], s, 0, 0, 0);
    read_rows<V>(Gt, qh, ln, a);
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ds], vf[ds], dp, 0, 0, 0);
    bf16x8 pp[2], pd[2];
    // (element-wise inserts here: the pair-packed form of the dQ kernel spills at this kernel's 168-register budget)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __builtin_amdgcn_exp2f(s[i]);
      pp[i >> 3][i & 7] = f2bf(p);
      pd[i >> 3][i & 7] = f2bf(p * dp[i]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        dvt[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Gt, qh * 2 + j, ta, dh), pp[j], dvt[dh], 0, 0, 0);
        dkt[dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(read_tr(Qt, qh * 2 + j, ta, dh), pd[j], dkt[dh], 0, 0, 0);
      }
  };
  issue(tbeg);
  load_stat(tbeg);
  put_stat(tbeg);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ti = tbeg; ti < tend; ++ti) {
    if (ti + 1 < tend) {
      issue(ti + 1);
      load_stat(ti + 1);
    }
    const char* Qt = smem + (ti & 1) * STAGE;
    const char* Gt = Qt + TILE;
    const float* st = (const float*)(Qt + 2 * TILE);
    if (V == 0) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        if (!active) break;
        half(Qt, Gt, st, qh);
      }
    } else if (active) {
      half(Qt, Gt, st, 0);
      half(Qt, Gt, st, 1);
    }
    if (ti + 1 < tend) put_stat(ti + 1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (piece) {
    float* rec = sp.ws + ((int64_t)pj * (BW * 32) + wave * 32 + (lane & 31)) * 128;
    store_partT(rec, dkt, hl);
    store_partT(rec + 64, dvt, hl);
  } else if (key < d.Nk) {
    store_rowT((bf16*)d.dK + (int64_t)b * d.dk_sb + (int64_t)key * d.dk_sn + h * 64, dkt, hl, d.scale);
    store_rowT((bf16*)d.dV + (int64_t)b * d.dv_sb + (int64_t)key * d.dv_sn + h * 64, dvt, hl, 1.f);
  }
}

// the tail pieces' sums, 4 columns per thread: dQ (64 columns, scale x sum) or dK | dV (128 columns: scale x sum |
// sum); rows past the length skipped
__global__ __launch_bounds__(256) void bwd_tail_reduce_kernel(const vp_attn_bwd_desc d, const BwdSplit sp, int ntail,
                                                              int kv) {
  const int cols = kv ? 128 : 64;
  const int per_row = cols / 4;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / per_row;
  const int c4 = (int)(gid - row * per_row) * 4;
  if (row >= (int64_t)ntail * (BW * 32)) return;
  const int j = (int)(row / (BW * 32)), r = (int)(row - (int64_t)j * (BW * 32));
  const int t = sp.main_blocks + j;
  const int nb = ((kv ? d.Nk : d.Nq) + BW * 32 - 1) / (BW * 32);
  const int bh = t / nb, blk = t - bh * nb;
  const int b = bh / d.H, h = bh - b * d.H;
  const int n = blk * BW * 32 + r;
  if (n >= (kv ? d.Nk : d.Nq)) return;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < sp.nsplit; ++s) {
    const f32x4 v = *(const f32x4*)(sp.ws + (((int64_t)j * sp.nsplit + s) * (BW * 32) + r) * cols + c4);
    acc[0] += v[0];
    acc[1] += v[1];
    acc[2] += v[2];
    acc[3] += v[3];
  }
  bf16* dst;
  float mul = d.scale;
  if (!kv) {
    dst = (bf16*)d.dQ + (int64_t)b * d.dq_sb + (int64_t)n * d.dq_sn + h * 64 + c4;
  } else if (c4 < 64) {
    dst = (bf16*)d.dK + (int64_t)b * d.dk_sb + (int64_t)n * d.dk_sn + h * 64 + c4;
  } else {
    dst = (bf16*)d.dV + (int64_t)b * d.dv_sb + (int64_t)n * d.dv_sn + h * 64 + c4 - 64;
    mul = 1.f;
  }
  bf16x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[e] * mul);
  *(bf16x4*)dst = o;
}

struct BwdPlan {
  int64_t nq = 0, nk = 0;          // dQ / dK-dV blocks
  int tq = 0, sq = 1, tk = 0, sk = 1;  // tail blocks and pieces per tail block of each kernel
  int64_t wq = 0, wk = 0;          // workspace bytes of each
};

int bwd_check(const vp_attn_bwd_desc* d) {
  if (d == nullptr || !d->Q || !d->K || !d->V || !d->O || !d->dO || !d->lse || !d->delta || !d->dQ || !d->dK ||
      !d->dV)
    return VP_ERR_ARG;
  if (d->head_dim != 64) return VP_ERR_UNSUPPORTED;
  if (d->B <= 0 || d->H <= 0 || d->Nq <= 0 || d->Nk <= 0) return VP_ERR_ARG;
  const int64_t strides[] = {d->q_sn, d->k_sn, d->v_sn, d->o_sn, d->do_sn, d->dq_sn, d->dk_sn, d->dv_sn,
                             d->q_sb, d->k_sb, d->v_sb, d->o_sb, d->do_sb, d->dq_sb, d->dk_sb, d->dv_sb};
  for (int64_t s : strides)
    if (s % 8) return VP_ERR_ARG;
  // the LDS-DMA source offsets are 32-bit: a tile's rows lie within 2^31 bytes of its first row
  if ((int64_t)BT * d->q_sn * 2 >= ((int64_t)1 << 31) || (int64_t)BT * d->k_sn * 2 >= ((int64_t)1 << 31) ||
      (int64_t)BT * d->v_sn * 2 >= ((int64_t)1 << 31) || (int64_t)BT * d->do_sn * 2 >= ((int64_t)1 << 31))
    return VP_ERR_ARG;
  return VP_OK;
}

// the tail split of one kernel: `slots` concurrent workgroups, nblk blocks, ntile loop tiles; the remainder blocks
// of the last partial round in S = min(8, ceil(2 slots / remainder), ntile) pieces (about two rounds of pieces, the
// forward's rule) when at least one whole round stays unsplit
void bwd_tail(int slots, int64_t nblk, int ntile, int& tail, int& S) {
  tail = 0;
  S = 1;
  if (slots <= 0) return;
  const int rem = (int)(nblk % slots);
  if (rem == 0 || rem + slots > nblk) return;
  const int s = min(min(8, (2 * slots + rem - 1) / rem), ntile);
  if (s < 2) return;
  tail = rem;
  S = s;
}

void bwd_attr() {
  static bool attr = false;
  if (attr) return;
  attr = true;
  for (const void* f : {(const void*)bwd_dq_kernel<0>, (const void*)bwd_dkdv_kernel<0>, (const void*)bwd_dq_kernel<1>,
                        (const void*)bwd_dkdv_kernel<1>})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BWD);
}

BwdPlan bwd_plan(const vp_attn_bwd_desc* d, bool split) {
  BwdPlan pl;
  pl.nq = (int64_t)d->B * d->H * ((d->Nq + BW * 32 - 1) / (BW * 32));
  pl.nk = (int64_t)d->B * d->H * ((d->Nk + BW * 32 - 1) / (BW * 32));
  const char* ns = vp_knob(VPK_ATTN_NO_SPLIT);
  if (!split || (ns != nullptr && ns[0] != '0')) return pl;
  static int slots_q = -1, slots_k = -1;
  if (slots_q < 0) {
    bwd_attr();
    int dev = 0, cus = 0, pq = 0, pk = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pq, (const void*)bwd_dq_kernel<1>, BW * 64, LDS_BWD) != hipSuccess)
      pq = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pk, (const void*)bwd_dkdv_kernel<1>, BW * 64, LDS_BWD) !=
        hipSuccess)
      pk = 0;
    slots_q = pq * cus;
    slots_k = pk * cus;
  }
  bwd_tail(slots_q, pl.nq, (d->Nk + BT - 1) / BT, pl.tq, pl.sq);
  bwd_tail(slots_k, pl.nk, (d->Nq + BT - 1) / BT, pl.tk, pl.sk);
  pl.wq = (int64_t)pl.tq * pl.sq * (BW * 32) * 64 * 4;
  pl.wk = (int64_t)pl.tk * pl.sk * (BW * 32) * 128 * 4;
  return pl;
}
}  // namespace

extern "C" int64_t vp_attention_bwd_workspace_bytes(const vp_attn_bwd_desc* d) {
  if (bwd_check(d) != VP_OK) return -1;
  const char* kv = vp_knob(VPK_ATTN_BWD_VARIANT);
  if (kv != nullptr && atoi(kv) != 1) return 0;  // the round-2 kernels run unsplit
  const BwdPlan pl = bwd_plan(d, true);
  return pl.wq + pl.wk;
}

extern "C" int vp_attention_bwd_bf16(const vp_attn_bwd_desc* d, void* stream) {
  return vp_attention_bwd_bf16_ws(d, nullptr, 0, stream);
}

extern "C" int vp_attention_bwd_bf16_ws(const vp_attn_bwd_desc* d, void* workspace, int64_t workspace_bytes,
                                        void* stream) {
  const int rc = bwd_check(d);
  if (rc != VP_OK) return rc;
  // VP_ATTN_BWD_VARIANT: 1 (default) or 0 (round 2's kernels); A/B only — same arithmetic, same results.  Measured and
  // dropped in round 5 (profiles/r05_attn_bwd_ab.log): variant 1 with the dK / dV kernel at 2 waves per SIMD (+7 %),
  // with dQ at 3 (60 B of scratch, +8 %; with the pair packing 24 B, equal), and an in-wave software pipeline of
  // both kernels (+4 %)
  const char* kv = vp_knob(VPK_ATTN_BWD_VARIANT);
  const int var = kv ? atoi(kv) : 1;
  if (var != 0 && var != 1) return VP_ERR_UNSUPPORTED;
  bwd_attr();
  // the tail split needs the workspace (vp_attention_bwd_workspace_bytes) and the default kernels
  BwdPlan pl = bwd_plan(d, var == 1);
  if (pl.wq + pl.wk > 0 &&
      (workspace == nullptr || workspace_bytes < pl.wq + pl.wk || ((uintptr_t)workspace & 15) != 0))
    pl = bwd_plan(d, false);
  if (pl.nq > 0x7fffffff || pl.nk > 0x7fffffff) return VP_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nd = (int64_t)d->B * d->Nq * d->H;
  const int64_t gd = (nd + 255) / 256;
  hipLaunchKernelGGL(bwd_delta_kernel, dim3((unsigned)(gd < (1 << 20) ? gd : (1 << 20))), dim3(256), 0, s, *d);
  VP_CHECK_LAUNCH();
  // whole blocks first, then the tail pieces, in one grid per kernel; then the pieces' sums
  const BwdSplit spq = {(int)(pl.nq - pl.tq), pl.sq, (float*)workspace};
  const BwdSplit spk = {(int)(pl.nk - pl.tk), pl.sk, (float*)((char*)workspace + pl.wq)};
  void (*dq)(const vp_attn_bwd_desc, const BwdSplit) = var ? bwd_dq_kernel<1> : bwd_dq_kernel<0>;
  hipLaunchKernelGGL(dq, dim3((unsigned)(pl.nq - pl.tq + (int64_t)pl.tq * pl.sq)), dim3(BW * 64), LDS_BWD, s, *d, spq);
  VP_CHECK_LAUNCH();
  void (*dkdv)(const vp_attn_bwd_desc, const BwdSplit) = var ? bwd_dkdv_kernel<1> : bwd_dkdv_kernel<0>;
  hipLaunchKernelGGL(dkdv, dim3((unsigned)(pl.nk - pl.tk + (int64_t)pl.tk * pl.sk)), dim3(BW * 64), LDS_BWD, s, *d,
                     spk);
  VP_CHECK_LAUNCH();
  if (pl.tq > 0) {
    const int64_t n = (int64_t)pl.tq * (BW * 32) * 16;
    hipLaunchKernelGGL(bwd_tail_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *d, spq, pl.tq, 0);
    VP_CHECK_LAUNCH();
  }
  if (pl.tk > 0) {
    const int64_t n = (int64_t)pl.tk * (BW * 32) * 32;
    hipLaunchKernelGGL(bwd_tail_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *d, spk, pl.tk, 1);
    VP_CHECK_LAUNCH();
  }
  return VP_OK;
}
