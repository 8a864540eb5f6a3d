// Flash-attention forward for CogVideoX joint 3D attention on gfx950 (MI355X): head_dim 64, non-causal, no mask,
// N up to ~47k tokens, optional second K/V segment (the ID-resample processor's doubled K/V, reference
// DF/models/attention_processor.py:2283-2290) and an output blend (the prev-clip path :2177-2189).
//
// Layout of the math (one wave = 32 queries, one workgroup = 8 waves = 256 queries of one (batch, head)):
//   S^T[key][q] = K · Q^T        v_mfma_f32_32x32x16_bf16, A = K rows from LDS (ds_read_b128, XOR-swizzled),
//                                B = Q^T held in registers for the whole key loop (pre-scaled by scale·log2 e, so
//                                the scores leave the matrix pipe in log2 units and the softmax is a bare v_exp_f32).
//   The accumulator has the query on the lane, so the online-softmax state (running max m, sum l) is per lane.
//   O^T[d][q] += V^T · P^T      A = V^T read with ds_read_b64_tr_b16 (hardware transpose) from the V tile,
//                                B = P^T taken straight from the S^T accumulator registers (bf16-packed, with the
//                                k-order permutation of cdna_hip_programming.md §3 "accumulator tile as operand").
// 128-key K/V tiles stream into a 2-slot LDS ring by LDS-DMA (global_load_lds_dwordx4) and are consumed as 32-key
// halves (16 score + 8 packed-P registers live: 128 VGPRs, 4 waves per SIMD = two 8-wave workgroups per CU).
// Roofline: MFMA-bound in principle (4·N²·64 flop per (b,h)); at d = 64 every score costs one v_exp_f32, a bf16 pack
// and a row-sum add against 256 MFMA flops, so the softmax VALU issue is the co-bottleneck (DESIGN_LOG.md §3).
//
// Softmax modes (template MODE):
//   LAZY   (default for unbounded scores): C-init QK^T (the running max enters the first MFMA as C = -m, so S - m
//          leaves the matrix pipe), then exp2 straight off the accumulator; the max path runs only when a lane's
//          half-sum shows an exponent above the threshold.
//   BOUNDED (the host proves |score| <= VP_ATTN_SCORE_BOUND in log2 units, flag VP_ATTN_BOUNDED_SCORES): no
//          running max at all — p = exp2(s) is exact in bf16 and fp32 over [2^-60, 2^60] and O / l is invariant to
//          the reference point.  CogVideoX's qk-LayerNorm bounds every score: |q|, |k| <= 8 max|gamma| + |beta|_2
//          (attention_processor.py:2143-2146), so the processors set the flag per layer from the norm weights.
//          The row sums run on the matrix pipe: one v_mfma_f32_16x16x32_bf16 per 16 keys with a 0/1 selector as A
//          and the P^T operand as B gives all 32 queries' sums, so the VALU does only exp2 + pack per score.
//          (Measured at config 2: 1.15 PF/s against 1.13 for LAZY; the same no-max kernel with the sums on the VALU
//          needs a second score tile live and spills at 128 VGPRs: 0.97.)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>


#include "vp_common.h"

namespace {

constexpr int NW = 8;               // waves per workgroup
constexpr int QB = NW * 32;         // 256 queries per workgroup
constexpr int KB = 128;             // keys per LDS tile
constexpr int KT = KB * 128;        // bytes per K (or V) tile
constexpr int ST = 2 * KT;          // one ring slot = K + V
constexpr int LDS_BYTES = 2 * ST;   // 2-slot ring
constexpr int NP = KB / 8;          // 1-KiB DMA pieces (8 rows) per operand per tile
constexpr int PPW = NP / NW;        // pieces per wave
constexpr int HALVES = KB / 32;
static_assert(NP % NW == 0, "pieces per wave");

// ---- diagnostic builds only (tools/attn_clock.py builds them into their own library; the default library has
// none of this).  VP_CLOCK_STAMPS: every workgroup of p2 / p2a / s16 / a16 stamps s_memtime and s_memrealtime before
// and after its key loop into vp_clock_buf (MI355X_MICROARCH.md 'DVFS give-back' item 6: in-kernel clock =
// delta memtime / delta realtime x 100 MHz); the stamps go to that buffer only, never into an output.
// VP_P1_ABL (p2 / p2a only, outputs invalid): bit 0 = no K / V DMA after the prologue (the loop re-reads stale
// tiles), bit 1 = the softmax's v_exp_f32 replaced by v_mov_b32 — which part of the loop's power holds the clock;
// bit 2 = every full K / V tile streamed from the head's first 8 tiles (same DMA instructions, all L2 hits): what
// the K / V fetches from beyond L2 cost.
#ifndef VP_CLOCK_STAMPS
#define VP_CLOCK_STAMPS 0
#endif
#ifndef VP_P1_ABL
#define VP_P1_ABL 0
#endif
#ifndef VP_CLOCK_WG
#define VP_CLOCK_WG 0  // 1 (p2 / p2a): realtime at workgroup entry, loop start, loop end, exit instead; 2: per work item
#endif
#if VP_CLOCK_STAMPS
constexpr int CLOCK_SLOTS = 1 << 15;
__device__ unsigned long long vp_clock_buf[CLOCK_SLOTS * 4];
struct ClockStamp {
  unsigned long long t0, r0, e0 = 0, r1 = 0;
  __device__ __forceinline__ void entry() { e0 = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ void start() {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ void stop(int tid) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
    if (!VP_CLOCK_WG && tid == 0 && blockIdx.x < CLOCK_SLOTS) {  // one lane, plain vector stores
      unsigned long long* p = vp_clock_buf + (size_t)blockIdx.x * 4;
      p[0] = t0;
      p[1] = r0;
      p[2] = t1;
      p[3] = r1;
    }
  }
  __device__ __forceinline__ void exit(int tid) {
    if (VP_CLOCK_WG == 1 && tid == 0 && blockIdx.x < CLOCK_SLOTS) {
      unsigned long long* p = vp_clock_buf + (size_t)blockIdx.x * 4;
      p[0] = e0;
      p[1] = r0;
      p[2] = r1;
      p[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
  // VP_CLOCK_WG = 2 (persistent p2 / p2a): one record per work item (its ticket value), the workgroup id in the top
  // 16 bits of the entry stamp
  __device__ __forceinline__ void item(int tid, int slot) {
    if (VP_CLOCK_WG == 2 && tid == 0 && slot >= 0 && slot < CLOCK_SLOTS) {
      unsigned long long* p = vp_clock_buf + (size_t)slot * 4;
      p[0] = e0 | ((unsigned long long)blockIdx.x << 48);
      p[1] = r0;
      p[2] = r1;
      p[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
};
#else
struct ClockStamp {
  __device__ __forceinline__ void entry() {}
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void stop(int) {}
  __device__ __forceinline__ void exit(int) {}
  __device__ __forceinline__ void item(int, int) {}
};
#endif

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

VP_DEV int swz(int row) { return (row >> 1) & 7; }

// inf / NaN by the exponent bits.  This file builds with -fno-honor-nans, under which the compiler may fold any NaN
// class test of a float to false — the bit test included (it recognises it as one): the empty asm makes the bits
// opaque.  (Without it p2a stored NaN rows of an overflowing block instead of flagging it for the a16 redo: the
// NaN half of the test had been folded away; tests/test_kernels_gpu.py::test_attention_anchored_late_jump_whole_blocks.)
VP_DEV bool nonfinite(float x) {
  uint32_t u = __float_as_uint(x);
  asm volatile("" : "+v"(u));
  return (u & 0x7f800000u) == 0x7f800000u;
}

struct Seg {
  const bf16* k;
  const bf16* v;
  int64_t k_sn, v_sn;
  int n;
  int key0;
};

// n2: the keys of segment 2 for this batch row (Nk2, or min(k2_len[b], Nk2) in the 16x16x32 kernels)
VP_DEV Seg tile_seg(const vp_attn_desc& d, int ti, int tiles1, int b, int h, int n2) {
  Seg s;
  if (ti < tiles1) {
    s.k = (const bf16*)d.K + (int64_t)b * d.k_sb + h * 64;
    s.v = (const bf16*)d.V + (int64_t)b * d.v_sb + h * 64;
    s.k_sn = d.k_sn;
    s.v_sn = d.v_sn;
    s.n = d.Nk;
    s.key0 = ti * KB;
  } else {
    s.k = (const bf16*)d.K2 + (int64_t)b * d.k2_sb + h * 64;
    s.v = (const bf16*)d.V2 + (int64_t)b * d.v2_sb + h * 64;
    s.k_sn = d.k2_sn;
    s.v_sn = d.v2_sn;
    s.n = n2;
    s.key0 = (ti - tiles1) * KB;
  }
  return s;
}
VP_DEV Seg tile_seg(const vp_attn_desc& d, int ti, int tiles1, int b, int h) {
  return tile_seg(d, ti, tiles1, b, h, d.Nk2);
}

// keys past the segment end (the DMA re-read the last key there) get score -inf
VP_DEV void mask_half(f32x16& s, int lim, int kh, int hl) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int key = kh * 32 + (i & 3) + 8 * (i >> 2) + 4 * hl;
    if (key >= lim) s[i] = -INFINITY;
  }
}

// ---- LDS-DMA staging (global_load_lds_dwordx4, saddr + 32-bit voffset): the LDS destination is lane-linear, so
// both images are unpadded [rows][128 B] and their bank swizzles are applied on the SOURCE address
// (cdna_hip_programming.md §5.4 rule 21).  K: chunk ^ swz(row) (conflict-free ds_read_b128).  V: chunk ^
// vswz(row) with vswz(r) = 4*((r>>1)&1): the 4-row x 16-column blocks a 32-lane half reads with
// ds_read_b64_tr_b16 (rows r..r+3, 64 contiguous bytes) then land on 4 disjoint 16-bank groups. ----
VP_DEV int vswz(int row) { return ((row >> 1) & 1) << 2; }

typedef __attribute__((address_space(3))) void lds_void_t;

// the lane id computed in place (a hoisted copy would be one more long-lived VGPR)
VP_DEV int lane_id_opaque() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// the same with the LDS destination given as a 32-bit LDS byte address (wave-uniform, e.g. a precomputed base of
// the dynamic LDS plus a constant): no generic -> LDS pointer conversion (and its null check) per instruction
VP_DEV void glds16_lds(const char* sbase, int voff, unsigned la) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(la), "v"(voff), "s"(sbase)
               : "memory", "m0");
}

VP_DEV void glds16(const char* sbase, int voff, char* lds) {
  // (the LDS address is wave-uniform; readfirstlane keeps it an SGPR where the compiler loses track of that)
  // (the low 32 bits of a generic LDS address are the LDS offset: no address-space cast, whose null check the
  // compiler mis-selects inside the persistent p2a loop)
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(la), "v"(voff), "s"(sbase)
               : "memory", "m0");
}

// O = O^T accumulator / l, rounded to bf16 like the reference's SDPA output, then the optional prev-clip blend.
// split_sum: l_run holds this lane's half of the row sum (the partner lane l ^ 32 has the other half).
VP_DEV void store_out(const vp_attn_desc& d, const f32x16 (&o)[2], float l_run, int q, int b, int h, int hl,
                      bool split_sum = true, float m_lse = NAN) {
  const float l_tot = split_sum ? l_run + __shfl_xor(l_run, 32, 64) : l_run;
  const float inv = 1.f / l_tot;
  if (q >= d.Nq) return;
  // softmax statistics for the backward (both lanes of a pair hold the same query, m and l: one writes)
  if (d.lse != nullptr && hl == 0 && !nonfinite(m_lse))  // (NaN: no statistics from this kernel; an opaque test, see nonfinite)
    d.lse[((int64_t)b * d.H + h) * d.Nq + q] = m_lse + __log2f(l_tot);
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

// ---- grid-tail split: the last partial round of workgroups (nblk mod resident slots) is re-launched as
// nsplit workgroups per block, each over a contiguous range of key tiles, writing an unnormalised partial
// (O relative to its own running max, row sum, max) to a workspace; attn_combine_kernel merges them.  Without it the
// last round runs a few workgroups on an otherwise idle chip (at config 2: 6720 blocks on 512 slots -> 64 blocks
// alone for a whole block time). ----
struct AttnSplit {
  int t_base;   // first block index of this launch
  int nsplit;   // 1: normal launch; > 1: key-range split of blocks t_base + blockIdx.x / nsplit
  float* ws;    // partials: [block - t_base][split][query in block (QB)][66] = O[64], m, l
  // anchored p2 (p2a) redo flags, one int per main-grid block then one per (tail block, split): written 0 / 1 by every
  // p2a workgroup (1 = a non-finite or underflowing row: nothing stored), read by the combine pass (skips a flagged
  // tail block) and by the redo launch of the anchored 16x16x32 kernel (runs only the flagged blocks); NULL: none
  int* flags;
  int flag_main;     // main-grid blocks (the tail's flags follow them)
  int flag_nsplit;   // splits per tail block
  int redo;          // a16 redo launch: a workgroup whose block is not flagged returns at once
  int flag_shift;    // redo of p2w: flags are per 512-query block (two of a16's 256-query blocks): shift 1
  // one-launch tail (p2 / p2a): workgroups blockIdx < main_blocks run whole blocks (XCD-remapped over main_blocks),
  // the rest are the key-range pieces of blocks t_base + (blockIdx - main_blocks) / nsplit, dispatched last
  int main_blocks;
  // persistent launch (p2 / p2a; NULL: one workgroup per block): 9 zeroed counters — the whole blocks of XCD x's
  // xcd_remap range are handed out by tickets[x], to that XCD's workgroups first and then to any XCD's that ran out;
  // then the npieces tail pieces by tickets[8]
  int* tickets;
  int npieces;
};

// the next work item of a persistent p2 / p2a workgroup on XCD x: a whole block (logical id < main_blocks), a tail
// piece (main_blocks + piece index) or -1.  The dispatcher gives every XCD the same number of workgroups while the
// XCDs run at different clocks (per-XCD loop time 419-464 us at config 2, tools/attn_wg_timeline.py): with one
// workgroup per block the slowest XCD finished its static share 5 % after the mean.
VP_DEV int p1_ticket(const AttnSplit& sp, int x) {
  const int c = xcd_ticket(sp.tickets, sp.main_blocks, x);
  if (c >= 0) return c;
  if (sp.npieces > 0 && __hip_atomic_load(sp.tickets + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sp.npieces) {
    const int c2 = __hip_atomic_fetch_add(sp.tickets + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c2 < sp.npieces) return sp.main_blocks + c2;
  }
  return -1;
}

// is block t flagged by its p2a workgroup(s)?
VP_DEV bool block_flagged(const AttnSplit& sp, int t, int Nq) {
  if (sp.flag_shift) {  // t: a 256-query block; the flags are per (256 << flag_shift)-query block of the same head
    const int nqb = (Nq + 255) / 256, nqbw = (Nq + (256 << sp.flag_shift) - 1) / (256 << sp.flag_shift);
    const int bh = t / nqb;
    t = bh * nqbw + ((t - bh * nqb) >> sp.flag_shift);
  }
  if (t < sp.flag_main) return sp.flags[t] != 0;
  const int* f = sp.flags + sp.flag_main + (int64_t)(t - sp.flag_main) * sp.flag_nsplit;
  int any = 0;
  for (int s = 0; s < sp.flag_nsplit; ++s) any |= f[s];
  return any != 0;
}

// O^T accumulator layout of one lane (store_out): dim d = dh*32 + 8*gq + 4*hl + r  <->  o[dh][4*gq + r]
VP_DEV void store_partial(float* rec, const f32x16 (&o)[2], float m_run, float l_tot, int hl) {
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int dd = dh * 32 + 8 * gq + 4 * hl;
      *(f32x4*)(rec + dd) = (f32x4){o[dh][4 * gq], o[dh][4 * gq + 1], o[dh][4 * gq + 2], o[dh][4 * gq + 3]};
    }
  if (hl == 0) {
    rec[64] = m_run;
    rec[65] = l_tot;
  }
}

// 16 threads per (tail block, query), 4 output dims each: merge the nsplit partials and store like store_out (per
// element the same operations in the same order as one thread per query: the split count is the only loop)
__global__ __launch_bounds__(256) void attn_combine_kernel(const vp_attn_desc d, int t_base, int ntail, int nsplit,
                                                           int qb_size, const float* __restrict__ ws,
                                                           const int* __restrict__ flags) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int quad = gid & 15;
  const int row = gid >> 4;
  if (row >= ntail * qb_size) return;
  const int j = row / qb_size, qi = row - j * qb_size;
  if (flags != nullptr) {  // p2a: a flagged tail block is left to the redo launch (nothing stored here)
    int any = 0;
    for (int s = 0; s < nsplit; ++s) any |= flags[t_base + j * nsplit + s];
    if (any) return;
  }
  const int t = t_base + j;
  const int nqb = (d.Nq + qb_size - 1) / qb_size;
  const int bh = t / nqb, qb = t - bh * nqb;
  const int b = bh / d.H, h = bh - b * d.H;
  const int q = qb * qb_size + qi;
  if (q >= d.Nq) return;
  const float* rec0 = ws + ((int64_t)j * nsplit * qb_size + qi) * 66;
  float mx = -INFINITY;
  for (int s = 0; s < nsplit; ++s) mx = fmaxf(mx, rec0[(int64_t)s * qb_size * 66 + 64]);
  // the extra mass enters the reference point too, so no weight below exceeds 1 (a mass far above every partial's
  // reference would otherwise overflow the denominator)
  const float lx = d.l_extra != nullptr ? d.l_extra[((int64_t)b * d.H + h) * d.Nq + q] : -INFINITY;
  mx = fmaxf(mx, lx);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float l = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float* rec = rec0 + (int64_t)s * qb_size * 66;
    const float w = __builtin_amdgcn_exp2f(rec[64] - mx);
    l += rec[65] * w;
    const f32x4 v = *(const f32x4*)(rec + 4 * quad);
    acc[0] += v[0] * w;
    acc[1] += v[1] * w;
    acc[2] += v[2] * w;
    acc[3] += v[3] * w;
  }
  if (d.l_extra != nullptr) l += __builtin_amdgcn_exp2f(lx - mx);
  const float inv = 1.f / l;
  if (d.lse != nullptr && quad == 0) d.lse[((int64_t)b * d.H + h) * d.Nq + q] = mx + __log2f(l);
  bf16* orow = (bf16*)d.O + (int64_t)b * d.o_sb + (int64_t)q * d.o_sn + h * 64 + 4 * quad;
  bf16x4 ov;
  bf16x4 old;
  if (d.accumulate) old = *(const bf16x4*)orow;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = rbf(acc[r] * inv);
    if (d.out_scale != 1.f) v = rbf(v * d.out_scale);
    if (d.accumulate) v = bf2f(old[r]) + v;
    ov[r] = f2bf(v);
  }
  *(bf16x4*)orow = ov;
}

// ------------------------------------------------------------------------------------------------------------
// 4-wave workgroups of 256 queries, each wave TWO 32-query blocks (the round-2 W64 structure, pruned in round 6 with
// the 8-wave LAZY / W32 kernel: DESIGN_LOG.md): the K and V^T fragments of a 32-key half are read from LDS once and
// feed both blocks' MFMAs, 2 waves/SIMD (256 VGPRs), two workgroups per CU with independent barriers.
// ------------------------------------------------------------------------------------------------------------
constexpr int NW4 = 4;
constexpr int PPW4 = NP / NW4;
static_assert(NW4 * 64 == QB, "same query block as the 8-wave kernel");

// ------------------------------------------------------------------------------------------------------------
// P2 (the software-pipelined "p1 step" form, two workgroups per CU): 4 waves x 64 queries = two 32-query blocks per
// wave, 32x32x16 MFMA, row sums on the matrix pipe, and the work of a wave software-pipelined over "jobs" j =
// (32-key half, query block): step j runs the QK^T of job j + 1 and the PV (+ row sum) of job j - 1 on the matrix
// pipe while the VALU does job j's exp2 + bf16 packs, so every MFMA gap holds two v_exp_f32 and one pack.  The K
// fragments of a half are read one step ahead (double-buffered by half parity); the pipeline runs across tile
// boundaries.  (The round-1 one-workgroup-per-CU form "p1" on a 4-slot ring was pruned in round 6: DESIGN_LOG.md.)
// ------------------------------------------------------------------------------------------------------------
struct P1Regs {
  bf16x8 qf[2][4];  // Q^T of the two query blocks (pre-scaled)
  f32x16 o[2][2];   // O^T[block][dim half]
  f32x16 s[2];      // S^T of the job in flight per block
  u32x4 pf[2][2];   // packed bf16 P^T per block, 16-key slabs
  bf16x8 kf[2][4];  // K fragments by half parity
  bf16x8 vf[1][4];  // V^T fragments of the current half: [slab j * 2 + dim half]
  f32x4 lsum[2];
  f32x16 negm;      // anchored (p2a): C operand of every QK^T chain = -anchor (wave-uniform), unused otherwise
  float anc;        // the wave's anchor (log2 score units)
};

VP_DEV void p1_read_k(const char* Kl, int kh, int lane, bf16x8 (&kf)[4]) {
  const int hl = lane >> 5;
  const int row = kh * 32 + (lane & 31);
  const char* kr = Kl + row * 128;
  const int sw = swz(row);
#pragma unroll
  for (int c = 0; c < 4; ++c) kf[c] = *(const bf16x8*)(kr + (((2 * c + hl) ^ sw) << 4));
}

VP_DEV void p1_read_v(const char* Vl, int kh, const int (&vo)[2], bf16x8 (&vf)[4]) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const char* base = Vl + (kh * 2 + j) * 16 * 128 + vo[dh];
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)base);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + 8 * 128));
      vf[j * 2 + dh] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
}

// The schedule is pinned by hand: every MFMA (a builtin, so the compiler still sees its hazards, e.g. when it copies
// an accumulator) sits alone between two sched_barrier(0), and the gap's fillers (2 v_exp_f32 + 1 pack, volatile asm:
// kept in program order) follow it.  The compiler allocates registers and places the lgkmcnt waits of the LDS reads,
// which stay where the step puts them.  Filler hazards it cannot see inside asm, and why none needs a wait state: the
// exps read S at least a whole 4-MFMA group after the MFMA chain that wrote it; each pack reads exps issued one gap
// earlier (the transcendental -> VALU distance).
VP_DEV void p1_fence() { __builtin_amdgcn_sched_barrier(0); }
VP_DEV void p1_exp(float& p0, float& p1, float s0, float s1) {
#if VP_P1_ABL & 2
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=&v"(p0), "=&v"(p1) : "v"(s0), "v"(s1));
#else
  asm volatile("v_exp_f32 %0, %2\n\tv_exp_f32 %1, %3" : "=&v"(p0), "=&v"(p1) : "v"(s0), "v"(s1));
#endif
}
VP_DEV uint32_t p1_pack(float a, float b) {
  uint32_t w;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(w) : "v"(a), "v"(b));
  return w;
}
VP_DEV bf16x8 as_bf16x8(const u32x4& w) { return __builtin_bit_cast(bf16x8, w); }

#ifndef VP_P1_RS_SPREAD
#define VP_P1_RS_SPREAD 0
#endif
#ifndef VP_P1_SEAM
#define VP_P1_SEAM 0
#endif
#ifndef VP_F8_GENERIC_DMA
#define VP_F8_GENERIC_DMA 0
#endif
// one pipeline step: the QK^T chain of block QB_ (K buffer KB_; skipped when !QK) interleaved with the PV MFMAs of
// block PB (V buffer VB_) so that no MFMA waits on the one before it, then the two row-sum MFMAs; every gap holds the
// next exp pair of block EB's 16 scores and the pack of the pair before:
//   g0 QK c0 | g1 PV (slab 0, d 0-31) | g2 QK c1 | g3 PV (0, 32-63) | g4 QK c2 | g5 PV (1, 0-31) | g6 QK c3 |
//   g7 PV (1, 32-63) | row sum slab 0 | row sum slab 1
// SEAM (the tile-seam step, VP_P1_SEAM A/B): MFMA order PV0 PV1 QK0 PV2 QK1 PV3 QK2 QK3, so the K fragments read
// right after the seam barrier get two MFMAs of cover; the QK^T chain then ends one gap later, and an s_nop pads the
// distance to the next step's first (asm) exp of its result
template <int EB, int QB_, int PB, int KB_, int VB_, bool QK, bool SEAM = false, bool ANCH = false>
VP_DEV void p1_step(P1Regs& r, const bf16x8& sel) {
  float p[16];
  const f32x16 z = {};
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    constexpr int seam_kind[8] = {1, 1, 0, 1, 0, 1, 0, 0};  // 0 = QK, 1 = PV
    constexpr int seam_idx[8] = {0, 1, 0, 2, 1, 3, 2, 3};
    const int c = SEAM ? seam_idx[g] : g >> 1;
    if ((SEAM ? seam_kind[g] : (g & 1)) == 0) {
      if constexpr (QK) {
        p1_fence();
        // anchored: the chain starts from C = -anchor, so S - anchor leaves the matrix pipe (no VALU).  Its first MFMA
        // is inline asm with an early-clobber destination: with the builtin the compiler coalesces the
        // rescale branch's update of s[0] with -anchor and copies the tuple (8 v_mov_b64) before the chain
        if (ANCH && c == 0)
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3"
                       : "=&v"(r.s[QB_]) : "v"(r.kf[KB_][0]), "v"(r.qf[QB_][0]), "v"(r.negm));
        else
          r.s[QB_] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r.kf[KB_][c], r.qf[QB_][c], c == 0 ? z : r.s[QB_], 0,
                                                             0, 0);
        p1_fence();
      }
    } else {
      p1_fence();
      r.o[PB][c & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r.vf[VB_][c], as_bf16x8(r.pf[PB][c >> 1]),
                                                                r.o[PB][c & 1], 0, 0, 0);
      p1_fence();
    }
    p1_exp(p[2 * g], p[2 * g + 1], r.s[EB][2 * g], r.s[EB][2 * g + 1]);
    if (g > 0) r.pf[EB][(g - 1) >> 2][(g - 1) & 3] = p1_pack(p[2 * g - 2], p[2 * g - 1]);
#if VP_P1_RS_SPREAD
    if (g == 3) {  // slab 0's row sum as soon as slab 0's PV MFMAs are issued (the two sums are not back to back)
      p1_fence();
      r.lsum[PB] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, as_bf16x8(r.pf[PB][0]), r.lsum[PB], 0, 0, 0);
      p1_fence();
    }
#endif
  }
#if !VP_P1_RS_SPREAD
  p1_fence();
  r.lsum[PB] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, as_bf16x8(r.pf[PB][0]), r.lsum[PB], 0, 0, 0);
#endif
  p1_fence();
  r.pf[EB][1][3] = p1_pack(p[14], p[15]);
  p1_fence();
  r.lsum[PB] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, as_bf16x8(r.pf[PB][1]), r.lsum[PB], 0, 0, 0);
  p1_fence();
  if constexpr (SEAM) asm volatile("s_nop 7" ::: "memory");
}

// keys past the segment end (lane key (i & 3) + 8 (i >> 2) + 4 hl of the half >= rem = lim - 32 h): score -inf.  In
// asm so that the compiler cannot hoist the compares out of the (rare, uniform) masked branch into every step.
VP_DEV void p1_mask(f32x16& s, int rem, int hl4) {
  const float ninf = -INFINITY;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float x = s[i];
    int t;
    asm volatile(
        "v_add_u32 %1, %3, %4\n\t"
        "v_cmp_le_i32 vcc, %2, %1\n\t"
        "v_cndmask_b32 %0, %0, %5, vcc"
        : "+v"(x), "=&v"(t)
        : "s"(rem), "v"(hl4), "i"((i & 3) + 8 * (i >> 2)), "v"(ninf)
        : "vcc");
    s[i] = x;
  }
}

// one 128-key tile = 8 steps (halves h = 0..3 x blocks 0, 1).  Step (h, b) exps job (h, b)'s scores while the
// matrix pipe runs the QK^T of the next job and the PV of the previous one:
//   even step (h, 0): read K(h+1) | QK (h, 1) [K(h)] + PV (h-1, 1) [V(h-1)], then read V(h)
//   odd  step (h, 1):               QK (h+1, 0) [K(h+1)] + PV (h, 0) [V(h)]
// K fragments double-buffered by half parity, each read a whole step ahead of its first use; V^T single-buffered
// (read after the even step's PV, a 4-MFMA group before the odd step's).  On entry s[0] holds job (0, 0)'s scores,
// kf[0] K(0) of this tile, vf[0] / pf[1] the previous tile's V(3) / last P (zeros before the first tile).  The next
// tile's DMA is issued at the top of the tile into the slot this tile's predecessor used, so every read of a slot
// comes before the seam barrier; the seam is at the end of step (3, 0), after V(3) is read: wait for the next tile
// (vmcnt), pass the barrier, read its K(0); last: no next tile (the last tile's step (3, 1) runs its QK^T on stale K
// fragments, result unused: one code path, so the accumulators keep their registers through the tile).
// masked: keys >= lim get score -inf (a segment's partial last tile; a uniform branch before the step).
// VMC: the seam's vmcnt when the tile after next is already in flight (p2w: a 4-slot ring, tile t + 2 issued at the
// top of tile t, VMC = this tile's DMA instructions per wave; 0 for the 2-slot ring)
// sync: the seam waits for the DMA and passes the barrier (false: the next tile was published by an earlier barrier —
// p2w2's one barrier per two tiles)
template <bool ANCH = false, int VMC = 0>
VP_DEV void p1_tile(P1Regs& r, const bf16x8& sel, const char* Kl, const char* Kn, int lim, bool masked, bool last,
                    bool wait_all, int lane, const int (&vo)[2], bool sync = true) {
  const int hl = lane >> 5;
  const char* Vl = Kl + KT;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    // even step (h, 0)
    if (h < 3) p1_read_k(Kl, h + 1, lane, r.kf[(h + 1) & 1]);
    if (masked) p1_mask(r.s[0], lim - 32 * h, 4 * hl);
    if (h & 1)
      p1_step<0, 1, 1, 1, 0, true, false, ANCH>(r, sel);
    else
      p1_step<0, 1, 1, 0, 0, true, false, ANCH>(r, sel);
    p1_read_v(Vl, h, vo, r.vf[0]);
    if (h == 3 && !last) {
      if (sync) {
        if (VMC == 0 || wait_all)
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VMC) : "memory");
        __builtin_amdgcn_s_barrier();
      }
      asm volatile("" ::: "memory");
      p1_read_k(Kn, 0, lane, r.kf[0]);
    }
    // odd step (h, 1)
    if (masked) p1_mask(r.s[1], lim - 32 * h, 4 * hl);
    if (VP_P1_SEAM && h == 3)
      p1_step<1, 0, 0, 0, 0, true, true, ANCH>(r, sel);
    else if (h & 1)
      p1_step<1, 0, 0, 0, 0, true, false, ANCH>(r, sel);
    else
      p1_step<1, 0, 0, 1, 0, true, false, ANCH>(r, sel);
  }
  if constexpr (ANCH) {
    // Anchored: a wave whose partial row sums passed 2^62 (a rare, wave-uniform branch) moves its anchor up by 64.
    // State after step (3, 1): o / lsum of block 0 through job (3, 0) and of block 1 through job (2, 1); pf[1] = the
    // packed P of job (3, 1) (its PV and row sum run in the next step); s[0] = the next tile's job (0, 0) scores —
    // all relative to the old anchor, so all of them are scaled by 2^-64 (P, O, l) or moved by -64 (S).
    float big = 0.f;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int j = 0; j < 4; ++j) big = fmaxf(big, r.lsum[qi][j]);
    if (__ballot(!(big <= 0x1p62f)) != 0ull) {
      const float f = 0x1p-64f;
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        r.lsum[qi] *= f;
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) r.o[qi][dh] *= f;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t w = r.pf[1][j][e];
          const float lo = __uint_as_float(w << 16) * f, hi = __uint_as_float(w & 0xffff0000u) * f;
          r.pf[1][j][e] = (uint32_t)__builtin_bit_cast(uint16_t, f2bf(lo)) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, f2bf(hi)) << 16);
        }
#pragma unroll
      for (int i = 0; i < 16; ++i) r.s[0][i] -= 64.f;
      r.anc += 64.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) r.negm[i] = -r.anc;
    }
  }
}

// ANCH (p2a): the anchored softmax on the p2 pipeline, for scores with no proven bound.  The wave's
// reference point (anchor) is an actual score: the max over its 64 queries and the first 32 keys it visits; it enters
// every QK^T chain as the C operand (C = -anchor: no VALU), and moves up by 64 when a partial row sum passes 2^62
// (p1_tile).  At the end a workgroup with a non-finite output or row sum (a score more than ~127 log2 units above
// the anchor inside one tile), or a row sum under 2^-96 (a query whose scores sit far below the wave's anchor, where
// small terms would underflow) stores nothing and raises its flag in sp.flags; the launcher then re-runs exactly
// those blocks with the anchored 16x16x32 kernel (per-query anchors and its exact two-pass re-run).
// NWV = 8 (p2w): the same per-wave pipeline in 8-wave workgroups of 512 queries, one per CU, on a 4-slot
// ring (tile t + 2 issued at the top of tile t): a K / V tile loaded once serves twice the queries, so each wave
// issues half the LDS-DMA instructions per tile (4 instead of 8) — the DMA issue is ~7 % of p2a's time
// (tools/attn_clock.py ablation, DESIGN_LOG.md §3.R5) — and the L2 -> LDS bytes per FLOP halve.
// TPB = 2 (p2w only): one barrier per two tiles — tiles t + 2 and t + 3 issued together at the top of every even tile
// of the range, both waited for and published by the barrier at the seam of the odd tile before them.
// one block (logical id t; a key-range piece `split` of it when `piece`) of attn_fwd_p1
template <bool TAIL, bool ANCH, int NWV, int TPB>
VP_DEV __attribute__((always_inline)) void p1_block(const vp_attn_desc& d, const AttnSplit& sp, const int t,
                                                    const bool piece, const int split, ClockStamp& ck) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int QBV = NWV * 64;               // queries per workgroup
  constexpr int PPWV = NP / NWV;              // DMA pieces per operand, wave and tile
  constexpr int RING = NWV == 8 ? 4 : 2;      // LDS ring slots
  constexpr int AHEAD = RING / 2;             // tiles issued ahead
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane >> 5;

  const int nqb = (d.Nq + QBV - 1) / QBV;
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;
  const int tiles1 = (d.Nk + KB - 1) / KB;
  // segment 2 of this batch row: its first k2_len[b] keys (the resample processor's masked rows), or all Nk2
  const int n2 = d.k2_len != nullptr ? max(0, min(__builtin_amdgcn_readfirstlane(d.k2_len[b]), d.Nk2)) : d.Nk2;
  const int tiles2 = n2 > 0 ? (n2 + KB - 1) / KB : 0;
  const int ntiles_all = tiles1 + tiles2;
  const int tbeg = piece ? (int)((int64_t)ntiles_all * split / sp.nsplit) : 0;
  const int tend = piece ? (int)((int64_t)ntiles_all * (split + 1) / sp.nsplit) : ntiles_all;
  const int qw0 = qb * QBV + wave * 64;
#ifdef VP_P1_PRIO
  if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);  // A/B: static priority for every other workgroup
#endif

  P1Regs r;
  {
    const float cq = d.scale * 1.4426950408889634f;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      const int q = qw0 + qi * 32 + (lane & 31);
      const int qc = q < d.Nq ? q : d.Nq - 1;
      const bf16* qrow = (const bf16*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
#pragma unroll
      for (int ds = 0; ds < 4; ++ds) {
        r.qf[qi][ds] = *(const bf16x8*)(qrow + ds * 16 + hl * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) r.qf[qi][ds][j] = f2bf(bf2f(r.qf[qi][ds][j]) * cq);
      }
    }
  }
  auto slot_of = [&](int ti) { return smem + (ti & (RING - 1)) * ST; };
  // full tiles of segment 1 (all but possibly its last): one scalar base per operand and tile, the lane offsets fixed
  // (voff_*), the LDS destination from a precomputed base; segment 2 and partial tiles take the general path with the
  // lane's rows recomputed from the lane id (rows past the end re-read the last key)
  int voff_k[PPWV], voff_v[PPWV];
#pragma unroll
  for (int i = 0; i < PPWV; ++i) {
    const int prow = (wave + i * NWV) * 8 + (lane >> 3);
    voff_k[i] = (prow * (int)d.k_sn + (((lane & 7) ^ swz(prow)) * 8)) * 2;
    voff_v[i] = (prow * (int)d.v_sn + (((lane & 7) ^ vswz(prow)) * 8)) * 2;
  }
  const char* kseg1 = (const char*)((const bf16*)d.K + (int64_t)b * d.k_sb + h * 64);
  const char* vseg1 = (const char*)((const bf16*)d.V + (int64_t)b * d.v_sb + h * 64);
  const int full1 = d.Nk / KB;
  // segment 2 (the resample processor's masked keys) takes the same fast path for its full tiles when its rows have
  // segment 1's strides (the processor allocates them so): the same lane offsets, its own base
  const bool seg2fast = d.K2 != nullptr && d.k2_sn == d.k_sn && d.v2_sn == d.v_sn;
  const int full2 = seg2fast ? n2 / KB : 0;
  const char* kseg2 = seg2fast ? (const char*)((const bf16*)d.K2 + (int64_t)b * d.k2_sb + h * 64) : nullptr;
  const char* vseg2 = seg2fast ? (const char*)((const bf16*)d.V2 + (int64_t)b * d.v2_sb + h * 64) : nullptr;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)smem) + wave * 1024;
  auto issue = [&](int ti) {
    const bool s1 = ti < full1;
    if (s1 || (ti >= tiles1 && ti - tiles1 < full2)) {
      const unsigned la = lds0 + (ti & (RING - 1)) * ST;
#if VP_P1_ABL & 4
      const int tt = (s1 ? ti : ti - tiles1) & 7;  // ablation: every full tile from the head's first 8 (L2-resident)
#else
      const int tt = s1 ? ti : ti - tiles1;
#endif
      const char* kb = (s1 ? kseg1 : kseg2) + (int64_t)tt * KB * d.k_sn * 2;
      const char* vb = (s1 ? vseg1 : vseg2) + (int64_t)tt * KB * d.v_sn * 2;
#pragma unroll
      for (int i = 0; i < PPWV; ++i) {
        glds16_lds(kb, voff_k[i], la + i * NWV * 1024);
        glds16_lds(vb, voff_v[i], la + KT + i * NWV * 1024);
      }
      return;
    }
    const int ln = lane_id_opaque();
    const Seg sg = tile_seg(d, ti, tiles1, b, h, n2);
    char* slot = slot_of(ti);
    const int last = sg.n - 1 - sg.key0;
    const char* kb = (const char*)(sg.k + (int64_t)sg.key0 * sg.k_sn);
    const char* vb = (const char*)(sg.v + (int64_t)sg.key0 * sg.v_sn);
    const int ksn = (int)sg.k_sn, vsn = (int)sg.v_sn;
#pragma unroll
    for (int i = 0; i < PPWV; ++i) {
      const int pc = wave + i * NWV;
      const int prow = pc * 8 + (ln >> 3);
      const int rr = min(prow, last);
      glds16(kb, (rr * ksn + (((ln & 7) ^ swz(prow)) * 8)) * 2, slot + pc * 1024);
      glds16(vb, (rr * vsn + (((ln & 7) ^ vswz(prow)) * 8)) * 2, slot + KT + pc * 1024);
    }
  };
  static_assert(2 * PPW4 == 8, "vmcnt(8) in p1_tile = one tile of DMA per wave");

  const int g = lane >> 4;
  const int trow = 4 * (g >> 1) + ((lane & 15) >> 2);
  const int tcol = 16 * (g & 1) + 4 * (lane & 3);
  int vo[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh) vo[dh] = trow * 128 + (((dh * 4 + (tcol >> 3)) ^ vswz(trow)) << 4) + (tcol & 7) * 2;

#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      r.o[qi][0][i] = 0.f;
      r.o[qi][1][i] = 0.f;
    }
    r.lsum[qi] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) r.pf[qi][j] = (u32x4){0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) r.vf[0][c] = (bf16x8){};  // job -1: 0 x 0
  bf16x8 sel;
  {
    const bf16 one = f2bf((((lane >> 4) & 1) == 0) == ((lane & 15) < 8) ? 1.f : 0.f);
#pragma unroll
    for (int e = 0; e < 8; ++e) sel[e] = one;
  }

  // (a tail-split range is empty when k2_len leaves this row fewer tiles than splits: its record is O = 0, l = 0)
  const bool any = tbeg < tend;  // workgroup-uniform
  if (any) issue(tbeg);
  if (TPB == 2 && tbeg + 1 < tend) {  // both tiles of the first pair, published by the prologue barrier
    issue(tbeg + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (AHEAD == 2 && tbeg + 1 < tend) {
    issue(tbeg + 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPWV) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (any) p1_read_k(slot_of(tbeg), 0, lane, r.kf[0]);
  {
    const f32x16 z = {};
#pragma unroll
    for (int c = 0; c < 4; ++c)
      r.s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r.kf[0][c], r.qf[0][c], c == 0 ? z : r.s[0], 0, 0, 0);
    r.anc = 0.f;
    if constexpr (ANCH) {
      // the anchor: max over both blocks' scores of the first 32 keys (rows past a segment end re-read its last key,
      // queries past Nq re-read the last query: every value is a real score).  Block 1's job (0, 1) is recomputed by
      // the first step with C = -anchor.
#pragma unroll
      for (int c = 0; c < 4; ++c)
        r.s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r.kf[0][c], r.qf[1][c], c == 0 ? z : r.s[1], 0, 0, 0);
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fmaxf(r.s[0][i], r.s[1][i]));
#pragma unroll
      for (int sh = 1; sh < 64; sh <<= 1) mx = fmaxf(mx, __shfl_xor(mx, sh, 64));
      // rounded up to an integer: P = 2^(S - anchor) is then 2^S with an exact exponent shift (its bf16 rounding and
      // so every output are those of the unanchored p2 up to the fp32 rounding of S - anchor), independent of which
      // queries share the wave
      mx = __builtin_ceilf(mx);
      r.anc = any ? __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(mx))) : -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        r.s[0][i] -= r.anc;
        r.negm[i] = -r.anc;
      }
    }
  }
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // S -> the first (asm) exp
  ck.start();
  for (int ti = tbeg; ti < tend; ++ti) {
    bool sync = true;
    if constexpr (TPB == 2) {
      const bool even = ((ti - tbeg) & 1) == 0;
      if (even) {
        if (ti + 2 < tend) issue(ti + 2);
        if (ti + 3 < tend) issue(ti + 3);
      }
      sync = !even;
    } else if (ti + AHEAD < tend && (!(VP_P1_ABL & 1) || ti == tbeg)) {
      issue(ti + AHEAD);
    }
    int lim = KB;
    if (ti >= full1) {
      const Seg sg = tile_seg(d, ti, tiles1, b, h, n2);
      lim = sg.n - sg.key0;
    }
    p1_tile<ANCH, RING == 4 && TPB == 1 ? 2 * PPWV : 0>(r, sel, slot_of(ti), slot_of(ti + 1),
                                                        __builtin_amdgcn_readfirstlane(lim), lim < KB,
                                                        ti + 1 >= tend, TPB == 2 || ti + 2 >= tend, lane, vo, sync);
  }
  // drain: PV + row sums of the last job (3, 1)
#pragma unroll
  for (int c = 0; c < 4; ++c)
    r.o[1][c & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r.vf[0][c], as_bf16x8(r.pf[1][c >> 1]),
                                                            r.o[1][c & 1], 0, 0, 0);
  r.lsum[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, as_bf16x8(r.pf[1][0]), r.lsum[1], 0, 0, 0);
  r.lsum[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, as_bf16x8(r.pf[1][1]), r.lsum[1], 0, 0, 0);
  ck.stop(tid);

  const int qq = lane & 31;
  float l_tot[2];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    l_tot[qi] = __shfl(r.lsum[qi][0], qq < 16 ? qq : qq + 16, 64);
    const int q = qw0 + qi * 32 + qq;
    // l_extra: row-sum mass of keys outside the segments (the resample processor's null keys, log2 score units,
    // relative to the reference point: 0 when bounded, the anchor when anchored); a tail-split partial leaves it to
    // attn_combine_kernel
    if (!TAIL && !piece && d.l_extra != nullptr)
      l_tot[qi] += __builtin_amdgcn_exp2f(d.l_extra[((int64_t)b * d.H + h) * d.Nq + min(q, d.Nq - 1)] - r.anc);
  }
  if constexpr (ANCH) {
    // any non-finite row sum or output, or a row sum under 2^-96 (its terms would underflow), in the workgroup ->
    // store nothing, flag the block for the exact re-run (workgroup-uniform decision through 16 bytes of LDS past
    // the ring; the barrier also retires every wave's last reads of the ring)
    bool bad = false;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      // (a tail-split partial of an empty key range holds no mass: only its non-finite values count.  A non-empty
      // partial whose row sum underflowed is flagged too — its anchor, shared by the wave, sits far above that
      // query's scores, and the combine's weights relative to it would underflow as well.)
      bad |= nonfinite(l_tot[qi]) || (any && !(l_tot[qi] >= 0x1p-96f));
      const float inv = 1.f / l_tot[qi];
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int i = 0; i < 16; ++i) bad |= nonfinite(!piece ? r.o[qi][dh][i] * inv : r.o[qi][dh][i]);
    }
    int* wflag = (int*)(smem + RING * ST);
    const int mine = __ballot(bad) != 0ull;
    if (lane == 0) wflag[wave] = mine;
    __syncthreads();
    int redo = 0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) redo |= wflag[w];
    if (tid == 0 && sp.flags != nullptr)
      sp.flags[piece ? sp.flag_main + (t - sp.t_base) * sp.nsplit + split : t] = redo;
    if (redo) return;
  }
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int q = qw0 + qi * 32 + qq;
    if (piece) {
      const int qin = wave * 64 + qi * 32 + qq;
      store_partial(sp.ws + (((int64_t)(t - sp.t_base) * sp.nsplit + split) * QBV + qin) * 66, r.o[qi], r.anc,
                    l_tot[qi], hl);
    } else {
      store_out(d, r.o[qi], l_tot[qi], q, b, h, hl, false, r.anc);
    }
  }
}

// PERS: the persistent instance (p2 / p2a; AttnSplit.tickets)
template <bool TAIL = false, bool ANCH = false, int NWV = 4, int TPB = 1, bool PERS = false>
__global__ __launch_bounds__(NWV * 64, NWV == 8 ? 1 : 2) void attn_fwd_p1(const vp_attn_desc d, const AttnSplit sp) {
  static_assert(NWV == 4 || NWV == 8, "4-wave (p2 / p2a) or 8-wave (p2w) workgroups");
  static_assert(TPB == 1 || NWV == 8, "one barrier per two tiles needs the 4-slot ring");
  static_assert(!PERS || (!TAIL && NWV == 4), "persistent: p2 / p2a main instances");
  ClockStamp ck;
  ck.entry();
  if constexpr (!PERS) {
    // a key-range piece of a tail block (the TAIL instance of a two-launch tail, or blockIdx >= main_blocks of a
    // one-launch tail), or a whole block
    const int pj = (int)blockIdx.x - sp.main_blocks;
    const bool piece = sp.nsplit > 1 && pj >= 0;
    const int split = piece ? pj % sp.nsplit : 0;
    const int t = piece ? sp.t_base + pj / sp.nsplit : xcd_remap(blockIdx.x, sp.nsplit > 1 ? sp.main_blocks : gridDim.x);
    p1_block<TAIL, ANCH, NWV, TPB>(d, sp, t, piece, split, ck);
  } else {
    // persistent (p2 / p2a): work items by ticket until none is left; the two barriers around the broadcast also
    // retire every wave's reads of the ring and the flag words before the next item's DMA and flags
    __shared__ int tk[1];
    const int x = (int)(blockIdx.x & 7);  // the dispatcher's XCD of this workgroup
#pragma unroll 1
    for (;;) {
      if (threadIdx.x == 0) tk[0] = p1_ticket(sp, x);
      __syncthreads();
      const int c = tk[0];
      __syncthreads();
      if (c < 0) break;
      const bool piece = c >= sp.main_blocks;
      const int pj = c - sp.main_blocks;
      if (VP_CLOCK_WG == 2) ck.entry();
      p1_block<TAIL, ANCH, NWV, TPB>(d, sp, piece ? sp.t_base + pj / sp.nsplit : c, piece, piece ? pj % sp.nsplit : 0,
                                     ck);
      ck.item(threadIdx.x, c);
    }
  }
  ck.exit(threadIdx.x);
}

// ------------------------------------------------------------------------------------------------------------
// P2S ("build the pipelined 16x16x32 form and decide by wall"): p2a's software pipeline — the same
// jobs (32-key half x 32-query block), the same step order, ring, seam, anchor, rescale, flags and redo — on
// v_mfma_f32_16x16x32_bf16, the shape the chip holds a higher clock on under load (MI355X_MICROARCH.md 'DVFS
// give-back' item 7).  A job is 2 query tiles (16 queries) x 2 key tiles (16 keys):
//   QK^T  S^T[kt][qt] = K[kt] . Q^T[qt]      2 chains of 2 per (qt, kt): 8 MFMAs; lane l: query 16 qt + l % 16,
//                                             keys 16 kt + 4 (l / 16) + i (the s16 layout, the query on the lane)
//   PV    O^T[dt][qt] += V^T[dt] . P^T[qt]   8 MFMAs; P^T straight from the lane's own 8 scores (k-slot 8 (l / 16) + j
//                                             <-> key 4 (l / 16) + j, then 16 + 4 (l / 16) + j - 4), V^T by two
//                                             ds_read_b64_tr_b16 per 16-dim tile from the vswz16 image
//   rows  l[qt] += ones . P^T[qt]            2 MFMAs (every accumulator row is the query's sum)
// = 18 MFMAs of 16 cycles per job: the same 288 matrix cycles as p2a's 10, at twice the instructions; each gap holds
// one v_exp_f32 and every other one a pack.  Registers as p2a (o 64, S 32, K 32 by half parity, V^T 16, Q^T 32, P
// 16), the anchor's C operand 4 instead of 16.
// ------------------------------------------------------------------------------------------------------------
struct P2SRegs {
  bf16x8 qf[4][2];     // Q^T B operands [qt][c]: query 16 qt + l % 16, dims 32 c + 8 (l / 16) + j (pre-scaled)
  f32x4 o[4][4];       // O^T[dt][qt]: dims 16 dt + 4 (l / 16) + i of query 16 qt + l % 16
  f32x4 s[2][2][2];    // S^T of the job in flight per block qi: [qt' (query tile 2 qi + qt')][kt]
  u32x4 pf[2][2];      // packed P^T per block [qt']: words = key pairs (4g, 4g+1) (4g+2, 4g+3) (16+4g, ..) (16+4g+2, ..)
  bf16x8 kf[2][2][2];  // K A operands by half parity [kt][c]: key 16 kt + l % 16, dims 32 c + 8 (l / 16) + j
  bf16x8 vf[4];        // V^T A operands of the current half [dt]
  f32x4 lsum[4];       // row sums per query tile (the four entries equal)
  f32x4 negm;          // C operand of every QK^T chain: -anchor
  float anc;
};

// the job's score p (0..15) = query tile qt' = p / 8, key tile kt = (p / 4) % 2, element p % 4: the pairs (2m, 2m + 1)
// are the P^T words pf[m / 4][m % 4] (p2a's flat order)
VP_DEV void p2s_read_k(const char* Kl, int kh, int lane, bf16x8 (&kf)[2][2]) {
  const int g = lane >> 4;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int row = kh * 32 + kt * 16 + (lane & 15);
    const char* kr = Kl + row * 128;
    const int sw = swz(row);
#pragma unroll
    for (int c = 0; c < 2; ++c) kf[kt][c] = *(const bf16x8*)(kr + (((4 * c + g) ^ sw) << 4));
  }
}

VP_DEV void p2s_read_v(const char* Vl, int kh, const int (&vo)[4], bf16x8 (&vf)[4]) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const char* base = Vl + kh * 32 * 128 + vo[dt];
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)base);
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + 16 * 128));
    vf[dt] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

VP_DEV void p2s_exp(float& p0, float s0) {
#if VP_P1_ABL & 2
  asm volatile("v_mov_b32 %0, %1" : "=&v"(p0) : "v"(s0));
#else
  asm volatile("v_exp_f32 %0, %1" : "=&v"(p0) : "v"(s0));
#endif
}

// one step (the p1_step roles): QK^T of block QB_ on K buffer KB_ interleaved with the PV of block PB, then the two
// row-sum MFMAs; gap g holds exp g of block EB's 16 scores and, every other gap, the pack of an earlier pair:
//   g even: QK op g / 2 = chain (qt' = g / 8, kt = (g / 4) % 2), d-half c = (g / 2) % 2   (c = 0 from C = -anchor)
//   g odd:  PV op (dt = g / 4, qt' = (g / 2) % 2)
template <int EB, int QB_, int PB, int KB_>
VP_DEV void p2s_step(P2SRegs& r, const bf16x8& ones) {
  float p[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int n = g >> 1;
    if ((g & 1) == 0) {
      const int qt = n >> 2, kt = (n >> 1) & 1, c = n & 1;
      p1_fence();
      if (c == 0)  // (asm, early-clobber: -anchor stays in its own registers, never copied into the chain)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %3"
                     : "=&v"(r.s[QB_][qt][kt]) : "v"(r.kf[KB_][kt][0]), "v"(r.qf[2 * QB_ + qt][0]), "v"(r.negm));
      else
        r.s[QB_][qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.kf[KB_][kt][1], r.qf[2 * QB_ + qt][1],
                                                                    r.s[QB_][qt][kt], 0, 0, 0);
      p1_fence();
    } else {
      const int dt = n >> 1, qt = n & 1;
      p1_fence();
      r.o[dt][2 * PB + qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.vf[dt], as_bf16x8(r.pf[PB][qt]),
                                                                      r.o[dt][2 * PB + qt], 0, 0, 0);
      p1_fence();
    }
    p2s_exp(p[g], r.s[EB][g >> 3][(g >> 2) & 1][g & 3]);
    // the pair exp'd two and three gaps back: two transcendentals sit between, so no wait state before the pack
    if (g >= 3 && (g & 1) == 1) {
      const int m = (g - 3) >> 1;
      r.pf[EB][m >> 2][m & 3] = p1_pack(p[g - 3], p[g - 2]);
    }
  }
  p1_fence();
  r.lsum[2 * PB] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, as_bf16x8(r.pf[PB][0]), r.lsum[2 * PB], 0, 0, 0);
  p1_fence();
  r.pf[EB][1][3] = p1_pack(p[14], p[15]);
  p1_fence();
  r.lsum[2 * PB + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, as_bf16x8(r.pf[PB][1]), r.lsum[2 * PB + 1], 0,
                                                                0, 0);
  p1_fence();
}

// keys at or past rem = lim - 32 h of a block's scores: -inf (asm, as p1_mask)
VP_DEV void p2s_mask(f32x4 (&s)[2][2], int rem, int g4) {
  const float ninf = -INFINITY;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = s[qt][kt][i];
        int t;
        asm volatile(
            "v_add_u32 %1, %3, %4\n\t"
            "v_cmp_le_i32 vcc, %2, %1\n\t"
            "v_cndmask_b32 %0, %0, %5, vcc"
            : "+v"(x), "=&v"(t)
            : "s"(rem), "v"(g4), "i"(16 * kt + i), "v"(ninf)
            : "vcc");
        s[qt][kt][i] = x;
      }
}

// one 128-key tile, p1_tile's schedule (the even step reads K(h + 1), then V(h) after its PV; the seam at the end of
// step (3, 0)), then the anchored rescale check
VP_DEV void p2s_tile(P2SRegs& r, bf16x8& ones, const char* Kl, const char* Kn, int lim, bool masked, bool last,
                     int lane, const int (&vo)[4]) {
  const int g4 = 4 * (lane >> 4);
  const char* Vl = Kl + KT;
  // the all-ones row-sum operand is wave-uniform: opaque here, so the compiler keeps it in VGPRs instead of
  // re-materialising it from SGPRs before every row-sum MFMA (2 v_mov_b64 + s_nop per step)
  asm volatile("" : "+v"(ones));
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    if (h < 3) p2s_read_k(Kl, h + 1, lane, r.kf[(h + 1) & 1]);
    if (masked) p2s_mask(r.s[0], lim - 32 * h, g4);
    if (h & 1)
      p2s_step<0, 1, 1, 1>(r, ones);
    else
      p2s_step<0, 1, 1, 0>(r, ones);
    p2s_read_v(Vl, h, vo, r.vf);
    if (h == 3 && !last) {  // the seam (2-slot ring: the next tile is the only DMA in flight)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      p2s_read_k(Kn, 0, lane, r.kf[0]);
    }
    if (masked) p2s_mask(r.s[1], lim - 32 * h, g4);
    if (h & 1)
      p2s_step<1, 0, 0, 0>(r, ones);
    else
      p2s_step<1, 0, 0, 1>(r, ones);
  }
  // anchored rescale (p1_tile): a wave whose partial row sums passed 2^62 scales O, l and the packed P of job (3, 1)
  // by 2^-64, moves the next tile's job (0, 0) scores by -64 and its anchor up by 64
  float big = 0.f;
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) big = fmaxf(big, r.lsum[qt][0]);
  if (__ballot(!(big <= 0x1p62f)) != 0ull) {
    const float f = 0x1p-64f;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      r.lsum[qt] *= f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) r.o[dt][qt] *= f;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t w = r.pf[1][j][e];
        const float lo = __uint_as_float(w << 16) * f, hi = __uint_as_float(w & 0xffff0000u) * f;
        r.pf[1][j][e] = (uint32_t)__builtin_bit_cast(uint16_t, f2bf(lo)) |
                        ((uint32_t)__builtin_bit_cast(uint16_t, f2bf(hi)) << 16);
      }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) r.s[0][qt][kt] -= 64.f;
    r.anc += 64.f;
    r.negm = (f32x4){-r.anc, -r.anc, -r.anc, -r.anc};
  }
}

VP_DEV int vswz16(int row) { return ((row >> 1) & 3) << 1; }

template <bool TAIL = false>
__global__ __launch_bounds__(NW4 * 64, 2) void attn_fwd_p2s(const vp_attn_desc d, const AttnSplit sp) {
  constexpr int QBV = NW4 * 64;
  constexpr int PPWV = NP / NW4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int c16 = lane & 15;

  const int nqb = (d.Nq + QBV - 1) / QBV;
  const int split = sp.nsplit > 1 ? (int)(blockIdx.x % sp.nsplit) : 0;
  const int t = sp.nsplit > 1 ? sp.t_base + (int)(blockIdx.x / sp.nsplit) : xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;
  const int tiles1 = (d.Nk + KB - 1) / KB;
  const int n2 = d.k2_len != nullptr ? max(0, min(__builtin_amdgcn_readfirstlane(d.k2_len[b]), d.Nk2)) : d.Nk2;
  const int tiles2 = n2 > 0 ? (n2 + KB - 1) / KB : 0;
  const int ntiles_all = tiles1 + tiles2;
  const int tbeg = sp.nsplit > 1 ? (int)((int64_t)ntiles_all * split / sp.nsplit) : 0;
  const int tend = sp.nsplit > 1 ? (int)((int64_t)ntiles_all * (split + 1) / sp.nsplit) : ntiles_all;
  const int qw0 = qb * QBV + wave * 64;

  P2SRegs r;
  {
    const float cq = d.scale * 1.4426950408889634f;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const int q = qw0 + qt * 16 + c16;
      const int qc = q < d.Nq ? q : d.Nq - 1;
      const bf16* qrow = (const bf16*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        r.qf[qt][c] = *(const bf16x8*)(qrow + c * 32 + g * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) r.qf[qt][c][j] = f2bf(bf2f(r.qf[qt][c][j]) * cq);
      }
    }
  }
  auto slot_of = [&](int ti) { return smem + (ti & 1) * ST; };
  // DMA as attn_fwd_p1 (2-slot ring), the V image in the vswz16 swizzle of the 16x16x32 transposed reads
  int voff_k[PPWV], voff_v[PPWV];
#pragma unroll
  for (int i = 0; i < PPWV; ++i) {
    const int prow = (wave + i * NW4) * 8 + (lane >> 3);
    voff_k[i] = (prow * (int)d.k_sn + (((lane & 7) ^ swz(prow)) * 8)) * 2;
    voff_v[i] = (prow * (int)d.v_sn + (((lane & 7) ^ vswz16(prow)) * 8)) * 2;
  }
  const char* kseg1 = (const char*)((const bf16*)d.K + (int64_t)b * d.k_sb + h * 64);
  const char* vseg1 = (const char*)((const bf16*)d.V + (int64_t)b * d.v_sb + h * 64);
  const int full1 = d.Nk / KB;
  const bool seg2fast = d.K2 != nullptr && d.k2_sn == d.k_sn && d.v2_sn == d.v_sn;
  const int full2 = seg2fast ? n2 / KB : 0;
  const char* kseg2 = seg2fast ? (const char*)((const bf16*)d.K2 + (int64_t)b * d.k2_sb + h * 64) : nullptr;
  const char* vseg2 = seg2fast ? (const char*)((const bf16*)d.V2 + (int64_t)b * d.v2_sb + h * 64) : nullptr;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void_t*)smem) + wave * 1024;
  auto issue = [&](int ti) {
    const bool s1 = ti < full1;
    if (s1 || (ti >= tiles1 && ti - tiles1 < full2)) {
      const unsigned la = lds0 + (ti & 1) * ST;
      const int tt = s1 ? ti : ti - tiles1;
      const char* kb = (s1 ? kseg1 : kseg2) + (int64_t)tt * KB * d.k_sn * 2;
      const char* vb = (s1 ? vseg1 : vseg2) + (int64_t)tt * KB * d.v_sn * 2;
#pragma unroll
      for (int i = 0; i < PPWV; ++i) {
        glds16_lds(kb, voff_k[i], la + i * NW4 * 1024);
        glds16_lds(vb, voff_v[i], la + KT + i * NW4 * 1024);
      }
      return;
    }
    const int ln = lane_id_opaque();
    const Seg sg = tile_seg(d, ti, tiles1, b, h, n2);
    char* slot = slot_of(ti);
    const int last = sg.n - 1 - sg.key0;
    const char* kb = (const char*)(sg.k + (int64_t)sg.key0 * sg.k_sn);
    const char* vb = (const char*)(sg.v + (int64_t)sg.key0 * sg.v_sn);
    const int ksn = (int)sg.k_sn, vsn = (int)sg.v_sn;
#pragma unroll
    for (int i = 0; i < PPWV; ++i) {
      const int pc = wave + i * NW4;
      const int prow = pc * 8 + (ln >> 3);
      const int rr = min(prow, last);
      glds16(kb, (rr * ksn + (((ln & 7) ^ swz(prow)) * 8)) * 2, slot + pc * 1024);
      glds16(vb, (rr * vsn + (((ln & 7) ^ vswz16(prow)) * 8)) * 2, slot + KT + pc * 1024);
    }
  };
  // transposed V^T reads (the s16 kernel's): lane 4 tq + tp of its 16-lane group addresses key row 4 g + tq (second
  // read: + 16), columns 16 dt + 4 tp .. + 3
  int vo[4];
  {
    const int vrow = 4 * g + ((lane & 15) >> 2);
    const int tp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vo[dt] = vrow * 128 + (((2 * dt + (tp >> 1)) ^ vswz16(vrow)) << 4) + (tp & 1) * 8;
  }
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    r.lsum[qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) r.o[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int j = 0; j < 2; ++j) r.pf[qi][j] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) r.vf[dt] = (bf16x8){};  // job -1: 0 x 0
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = f2bf(1.f);

  const bool any = tbeg < tend;  // workgroup-uniform
  if (any) issue(tbeg);
  if (tbeg + 1 < tend) {
    issue(tbeg + 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPWV) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (any) p2s_read_k(slot_of(tbeg), 0, lane, r.kf[0]);
  {
    // job (0, 0) and, for the anchor, job (0, 1) from C = 0; the anchor = ceil(max over the wave's 64 queries x the
    // first 32 keys), as p2a's; job (0, 1) is recomputed by the first step with C = -anchor
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          r.s[qi][qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.kf[0][kt][0], r.qf[2 * qi + qt][0], z, 0, 0, 0);
          r.s[qi][qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.kf[0][kt][1], r.qf[2 * qi + qt][1],
                                                                     r.s[qi][qt][kt], 0, 0, 0);
        }
    float mx = -INFINITY;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = fmaxf(mx, r.s[qi][qt][kt][i]);
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) mx = fmaxf(mx, __shfl_xor(mx, sh, 64));
    mx = __builtin_ceilf(mx);
    r.anc = any ? __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(mx))) : -INFINITY;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) r.s[0][qt][kt] -= r.anc;
    r.negm = (f32x4){-r.anc, -r.anc, -r.anc, -r.anc};
  }
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // S -> the first (asm) exp
  ClockStamp ck;
  ck.start();
  for (int ti = tbeg; ti < tend; ++ti) {
    if (ti + 1 < tend && (!(VP_P1_ABL & 1) || ti == tbeg)) issue(ti + 1);
    int lim = KB;
    if (ti >= full1) {
      const Seg sg = tile_seg(d, ti, tiles1, b, h, n2);
      lim = sg.n - sg.key0;
    }
    p2s_tile(r, ones, slot_of(ti), slot_of(ti + 1), __builtin_amdgcn_readfirstlane(lim), lim < KB, ti + 1 >= tend,
             lane, vo);
  }
  // drain: PV + row sums of the last job (3, 1)
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      r.o[dt][2 + qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r.vf[dt], as_bf16x8(r.pf[1][qt]), r.o[dt][2 + qt], 0,
                                                                 0, 0);
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
    r.lsum[2 + qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, as_bf16x8(r.pf[1][qt]), r.lsum[2 + qt], 0, 0, 0);
  ck.stop(tid);

  float l_tot[4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    l_tot[qt] = r.lsum[qt][0];
    const int q = qw0 + qt * 16 + c16;
    if (!TAIL && d.l_extra != nullptr)
      l_tot[qt] += __builtin_amdgcn_exp2f(d.l_extra[((int64_t)b * d.H + h) * d.Nq + min(q, d.Nq - 1)] - r.anc);
  }
  {
    // p2a's flags: a non-finite row sum or output, or a row sum under 2^-96, anywhere in the workgroup -> store
    // nothing, flag the block for the a16 redo
    bool bad = false;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      bad |= nonfinite(l_tot[qt]) || (any && !(l_tot[qt] >= 0x1p-96f));
      const float inv = 1.f / l_tot[qt];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) bad |= nonfinite(sp.nsplit == 1 ? r.o[dt][qt][i] * inv : r.o[dt][qt][i]);
    }
    int* wflag = (int*)(smem + 2 * ST);
    const int mine = __ballot(bad) != 0ull;
    if (lane == 0) wflag[wave] = mine;
    __syncthreads();
    int redo = 0;
#pragma unroll
    for (int w = 0; w < NW4; ++w) redo |= wflag[w];
    if (tid == 0 && sp.flags != nullptr)
      sp.flags[sp.nsplit > 1 ? sp.flag_main + (t - sp.t_base) * sp.nsplit + split : t] = redo;
    if (redo) return;
  }
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const int q = qw0 + qt * 16 + c16;
    if (sp.nsplit > 1) {
      float* rec = sp.ws + (((int64_t)(t - sp.t_base) * sp.nsplit + split) * QBV + wave * 64 + qt * 16 + c16) * 66;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) *(f32x4*)(rec + dt * 16 + 4 * g) = r.o[dt][qt];
      if (g == 0) {
        rec[64] = r.anc;
        rec[65] = l_tot[qt];
      }
      continue;
    }
    if (q >= d.Nq) continue;
    const float inv = 1.f / l_tot[qt];
    if (d.lse != nullptr && g == 0) d.lse[((int64_t)b * d.H + h) * d.Nq + q] = r.anc + __log2f(l_tot[qt]);
    bf16* orow = (bf16*)d.O + (int64_t)b * d.o_sb + (int64_t)q * d.o_sn + h * 64 + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 ov;
      bf16x4 old;
      if (d.accumulate) old = *(const bf16x4*)(orow + dt * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = rbf(r.o[dt][qt][i] * inv);
        if (d.out_scale != 1.f) v = rbf(v * d.out_scale);
        if (d.accumulate) v = bf2f(old[i]) + v;
        ov[i] = f2bf(v);
      }
      *(bf16x4*)(orow + dt * 16) = ov;
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// S16: the W64 structure (4-wave workgroups of 256 queries, 64 queries per wave, 128-key tiles through the same
// 2-slot LDS-DMA ring) on the 16x16x32 bf16 MFMA instead of 32x32x16.  Same FLOPs, same LDS bytes and the same VALU
// per score; the chip holds a higher clock on the 16x16x32 shape under load (MI355X_MICROARCH.md 'DVFS give-back'
// item 7: 1.12-1.15x the FLOP/s of the 32x32x16 loop at equal cycles per FLOP).
// Per 32-key half and wave (4 query tiles qt of 16, 2 key tiles kt of 16, 4 head-dim tiles dt of 16):
//   S^T[kt][qt] = K[kt] . Q^T[qt]   2 MFMAs each (d = 0..31, 32..63): 16 MFMAs; lane l holds queries l % 16 and keys
//                                   16 kt + 4 (l / 16) + i (i = 0..3): the query on the lane, as before.
//   P^T[qt] (B operand, k-slot 8 (l / 16) + j  <->  key 4 (l / 16) + j for j < 4, 16 + 4 (l / 16) + j - 4 after):
//                                   the lane's own 8 scores, exp2 + pack, no cross-lane move.
//   O^T[dt][qt] += V^T[dt] . P^T[qt]  16 MFMAs; V^T[dt] (A operand, row d = 16 dt + l % 16, the same k-slots) by two
//                                   ds_read_b64_tr_b16 (keys 4 (l / 16) + 0..3 and 16 + 4 (l / 16) + 0..3).
//   l[qt] += ones . P^T[qt]         4 MFMAs: every accumulator row is the query's sum over the half's 32 keys.
// V image swizzle vswz16 (row r: chunk ^ 2 ((r >> 1) & 3)): the 32 lanes of a transposed read take keys r0 .. r0 + 7
// of one 16-column block, conflict-free only if rows 4 apart land in different chunk pairs.
// ------------------------------------------------------------------------------------------------------------


VP_DEV float xmax16(float x) {  // max over the 4 lanes c16 + 16 g (one query's lanes)
  x = fmaxf(x, __shfl_xor(x, 16, 64));
  return fmaxf(x, __shfl_xor(x, 32, 64));
}

// ANCH (anchored softmax, no bound on the scores needed): every query's exponent reference m is an actual score of
// its row — the max over the first 32 keys its workgroup visits — so the row sum is >= 1 (nothing underflows), and
// p = exp2(s - m) leaves the QK^T MFMA through its C operand (C = -m, free).  m then stays fixed: no running max.
// After each tile a wave whose row sums passed 2^64 (a rare, wave-uniform branch) rescales those queries' O and l
// by 2^-64 and raises m by 64.  A row whose scores jump more than ~120 log2 units above m inside one tile would
// overflow: the kernel checks every output and row sum at the end, and a workgroup that saw a non-finite value re-runs
// its block exactly (pass 1: the row maxima over all keys; pass 2: p = exp2(s - max) <= 1).  Without ANCH (the host
// proved |score| <= VP_ATTN_SCORE_BOUND) m = 0 and nothing is checked.
template <bool TAIL = false, bool ANCH = false>
__global__ __launch_bounds__(NW4 * 64, 2) void attn_fwd_s16(const vp_attn_desc d, const AttnSplit sp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int c16 = lane & 15;

  const int nqb = (d.Nq + QB - 1) / QB;
  const int split = sp.nsplit > 1 ? (int)(blockIdx.x % sp.nsplit) : 0;
  const int t = sp.nsplit > 1 ? sp.t_base + (int)(blockIdx.x / sp.nsplit) : xcd_remap(blockIdx.x, gridDim.x);
  // redo launch after the anchored p2: only the blocks p2a flagged (workgroup-uniform: one block per workgroup)
  if (sp.redo && !block_flagged(sp, t, d.Nq)) return;
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;
  const int tiles1 = (d.Nk + KB - 1) / KB;
  // segment 2 of this batch row: its first k2_len[b] keys (the resample processor's masked rows), or all Nk2
  const int n2 = d.k2_len != nullptr ? max(0, min(__builtin_amdgcn_readfirstlane(d.k2_len[b]), d.Nk2)) : d.Nk2;
  const int tiles2 = n2 > 0 ? (n2 + KB - 1) / KB : 0;
  const int ntiles_all = tiles1 + tiles2;
  // (a split range may be empty when k2_len shortens this row: its record is O = 0, l = 0, m = 0)
  const int tbeg = sp.nsplit > 1 ? (int)((int64_t)ntiles_all * split / sp.nsplit) : 0;
  const int tend = sp.nsplit > 1 ? (int)((int64_t)ntiles_all * (split + 1) / sp.nsplit) : ntiles_all;
  // segment-2 keys past k2_full[b] have zero values: their whole tiles skip the V^T DMA, reads and PV MFMAs
  const int k2f = d.k2_full != nullptr ? __builtin_amdgcn_readfirstlane(d.k2_full[b]) : 0x7fffffff;
  auto tile_full = [&](int ti) { return ti < tiles1 || (ti - tiles1) * KB < k2f; };

  const int qw0 = qb * QB + wave * 64;  // first query of this wave
  bf16x8 qf[4][2];                      // Q^T B operands: query 16 qt + l % 16, dims 32 c + 8 (l / 16) + j
  {
    const float cq = d.scale * 1.4426950408889634f;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const int q = qw0 + qt * 16 + c16;
      const int qc = q < d.Nq ? q : d.Nq - 1;
      const bf16* qrow = (const bf16*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        qf[qt][c] = *(const bf16x8*)(qrow + c * 32 + g * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qt][c][j] = f2bf(bf2f(qf[qt][c][j]) * cq);
      }
    }
  }

  int prow[PPW4], kch[PPW4], vch[PPW4];
#pragma unroll
  for (int i = 0; i < PPW4; ++i) {
    prow[i] = (wave + i * NW4) * 8 + (lane >> 3);
    kch[i] = (lane & 7) ^ swz(prow[i]);
    vch[i] = (lane & 7) ^ vswz16(prow[i]);
  }
  auto slot_of = [&](int ti) { return smem + (ti & 1) * ST; };
  auto issue = [&](int ti) {
    const Seg sg = tile_seg(d, ti, tiles1, b, h, n2);
    char* slot = slot_of(ti);
    const int last = sg.n - 1 - sg.key0;
    const char* kb = (const char*)(sg.k + (int64_t)sg.key0 * sg.k_sn);
    const char* vb = (const char*)(sg.v + (int64_t)sg.key0 * sg.v_sn);
    const int ksn = (int)sg.k_sn, vsn = (int)sg.v_sn;
    if (tile_full(ti)) {
#pragma unroll
      for (int i = 0; i < PPW4; ++i) {
        const int pc = wave + i * NW4;
        const int r = min(prow[i], last);
        glds16(kb, (r * ksn + kch[i] * 8) * 2, slot + pc * 1024);
        glds16(vb, (r * vsn + vch[i] * 8) * 2, slot + KT + pc * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PPW4; ++i) {
        const int pc = wave + i * NW4;
        const int r = min(prow[i], last);
        glds16(kb, (r * ksn + kch[i] * 8) * 2, slot + pc * 1024);
      }
    }
  };

  // transposed V^T reads: lane 4 tq + tp of its 16-lane group addresses key row 4 g + tq (second read: + 16),
  // columns 16 dt + 4 tp .. + 3; vswz16 depends on row bits 1-2 only, so one offset serves every half and both reads
  int vo[4];
  {
    const int vrow = 4 * g + ((lane & 15) >> 2);
    const int tp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vo[dt] = vrow * 128 + (((2 * dt + (tp >> 1)) ^ vswz16(vrow)) << 4) + (tp & 1) * 8;
  }

  f32x4 o[4][4];  // O^T[dt][qt]: dims 16 dt + 4 (l / 16) + i of query 16 qt + l % 16
  f32x4 lsum[4];
  f32x4 negm[4];  // C operand of the QK^T chains: -m of the lane's query (ANCH), else 0
  float m[4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    m[qt] = 0.f;
    negm[qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = f2bf(1.f);

  const bool active = qw0 < d.Nq;  // wave-uniform

  // one pass over this workgroup's key tiles through the LDS ring; body(Kl, Vl, lim, first_tile, full) per tile
  auto tile_loop = [&](auto&& body) {
    if (tbeg >= tend) return;
    issue(tbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int ti = tbeg; ti < tend; ++ti) {
      if (ti + 1 < tend) issue(ti + 1);
      const char* Kl = slot_of(ti);
      const Seg sg = tile_seg(d, ti, tiles1, b, h, n2);
      if (active) body(Kl, Kl + KT, sg.n - sg.key0, ti == tbeg, tile_full(ti));
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  };
  // S^T of one 32-key half: key 32 kh + 16 kt + 4 (l / 16) + i, C-initialised with negm (-m, or 0)
  auto qk_half = [&](const char* Kl, int kh, int lim, f32x4 (&sc)[4][2], auto mask_c) {
    bf16x8 kf[2][2];  // K A operands: key 32 kh + 16 kt + l % 16, dims 32 c + 8 (l / 16) + j
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int row = kh * 32 + kt * 16 + c16;
      const char* kr = Kl + row * 128;
      const int sw = swz(row);
#pragma unroll
      for (int c = 0; c < 2; ++c) kf[kt][c] = *(const bf16x8*)(kr + (((4 * c + g) ^ sw) << 4));
    }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        sc[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][0], qf[qt][0], negm[qt], 0, 0, 0);
        sc[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][1], qf[qt][1], sc[qt][kt], 0, 0, 0);
      }
    if constexpr (decltype(mask_c)::value) {
      if (lim < KB) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool dead = kh * 32 + kt * 16 + 4 * g + i >= lim;
#pragma unroll
            for (int qt = 0; qt < 4; ++qt)
              if (dead) sc[qt][kt][i] = -INFINITY;
          }
      }
    }
  };
  using MaskT = std::integral_constant<bool, true>;
  using MaskF = std::integral_constant<bool, false>;
  // P = exp2(S) packed as the P^T B operand, then O^T += V^T P^T and the row sums
  auto pv_half = [&](const char* Vl, int kh, const f32x4 (&sc)[4][2]) {
    bf16x8 pf[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pf[qt][i] = f2bf(__builtin_amdgcn_exp2f(sc[qt][0][i]));
        pf[qt][4 + i] = f2bf(__builtin_amdgcn_exp2f(sc[qt][1][i]));
      }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const char* base = Vl + kh * 32 * 128 + vo[dt];
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)base);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + 16 * 128));
      const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt], o[dt][qt], 0, 0, 0);
    }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) lsum[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qt], lsum[qt], 0, 0, 0);
  };
  // keys with zero values: exp2 + pack and the row sums only
  auto rs_half = [&](const f32x4 (&sc)[4][2]) {
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      bf16x8 pq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pq[i] = f2bf(__builtin_amdgcn_exp2f(sc[qt][0][i]));
        pq[4 + i] = f2bf(__builtin_amdgcn_exp2f(sc[qt][1][i]));
      }
      lsum[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pq, lsum[qt], 0, 0, 0);
    }
  };
  auto zero_acc = [&]() {
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      lsum[qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  };
  auto set_ref = [&](int qt, float mq) {
    m[qt] = mq;
    negm[qt] = (f32x4){-mq, -mq, -mq, -mq};
  };

  // ---- main pass ----
  zero_acc();
  ClockStamp ck;
  ck.start();
  tile_loop([&](const char* Kl, const char* Vl, int lim, bool first_tile, bool full) {
#pragma unroll
    for (int kh = 0; kh < HALVES; ++kh) {
      f32x4 sc[4][2];
      qk_half(Kl, kh, lim, sc, MaskT{});
      if constexpr (ANCH) {
        if (first_tile && kh == 0) {  // the anchor: max over the first 32 keys (all valid: key0 < n)
#pragma unroll
          for (int qt = 0; qt < 4; ++qt) {
            float mx = fmaxf(fmaxf(fmaxf(sc[qt][0][0], sc[qt][0][1]), fmaxf(sc[qt][0][2], sc[qt][0][3])),
                             fmaxf(fmaxf(sc[qt][1][0], sc[qt][1][1]), fmaxf(sc[qt][1][2], sc[qt][1][3])));
            mx = __builtin_ceilf(xmax16(mx));  // an integer reference: exact exponent shifts of 2^S (as p2a's)
            set_ref(qt, mx);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              sc[qt][0][i] -= mx;
              sc[qt][1][i] -= mx;
            }
          }
        }
      }
      if (full) pv_half(Vl, kh, sc);
      else rs_half(sc);
    }
    if constexpr (ANCH) {
      bool big = false;
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) big |= lsum[qt][0] > 0x1p64f;
      if (__ballot(big) != 0ull) {  // rare: shift the reference of those queries by 64
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) {
          const bool bq = lsum[qt][0] > 0x1p64f;
          const float f = bq ? 0x1p-64f : 1.f;
          if (bq) set_ref(qt, m[qt] + 64.f);
          lsum[qt] *= f;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= f;
        }
      }
    }
  });
  ck.stop(tid);

  // l_extra: row-sum mass of keys that are not in the segments (log2, score units; the null keys of the resample
  // processor), added relative to the query's reference m; a tail-split partial leaves it to attn_combine_kernel
  float lx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if constexpr (!TAIL) {
    if (d.l_extra != nullptr) {
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        const int q = min(qw0 + qt * 16 + c16, d.Nq - 1);
        lx[qt] = d.l_extra[((int64_t)b * d.H + h) * d.Nq + q];
      }
    }
  }
  auto add_extra = [&]() {
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) lsum[qt][0] += __builtin_amdgcn_exp2f(lx[qt] - m[qt]);
  };
  add_extra();

  if constexpr (ANCH) {
    // any non-finite row sum or output of the block -> the exact two-pass re-run (workgroup-uniform decision)
    bool bad = false;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const float inv = 1.f / lsum[qt][0];
      bad |= nonfinite(lsum[qt][0]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) bad |= nonfinite(o[dt][qt][r] * inv);
    }
    int* flag = (int*)smem;  // the ring is idle after the loop's last barrier
    const int mine = __ballot(bad && active) != 0ull;
    if (lane == 0) flag[wave] = mine;
    __syncthreads();  // (waits for the LDS stores before the barrier)
    const bool redo = (flag[0] | flag[1] | flag[2] | flag[3]) != 0;
    __syncthreads();  // flags read before the ring is refilled
    if (redo) {
      // pass 1: exact row maxima
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) set_ref(qt, 0.f);
      float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      tile_loop([&](const char* Kl, const char*, int lim, bool, bool) {
#pragma unroll
        for (int kh = 0; kh < HALVES; ++kh) {
          f32x4 sc[4][2];
          qk_half(Kl, kh, lim, sc, MaskT{});
#pragma unroll
          for (int qt = 0; qt < 4; ++qt)
#pragma unroll
            for (int i = 0; i < 4; ++i) mx[qt] = fmaxf(mx[qt], fmaxf(sc[qt][0][i], sc[qt][1][i]));
        }
      });
      // pass 2: p = exp2(s - max) <= 1 (the max includes l_extra's log mass)
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) set_ref(qt, __builtin_ceilf(fmaxf(xmax16(mx[qt]), lx[qt])));
      zero_acc();
      tile_loop([&](const char* Kl, const char* Vl, int lim, bool, bool full) {
#pragma unroll
        for (int kh = 0; kh < HALVES; ++kh) {
          f32x4 sc[4][2];
          qk_half(Kl, kh, lim, sc, MaskT{});
          if (full) pv_half(Vl, kh, sc);
          else rs_half(sc);
        }
      });
      add_extra();
    }
  }

#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const float l_tot = lsum[qt][0];
    const int q = qw0 + qt * 16 + c16;
    if (sp.nsplit > 1) {
      float* rec = sp.ws + (((int64_t)(t - sp.t_base) * sp.nsplit + split) * QB + wave * 64 + qt * 16 + c16) * 66;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) *(f32x4*)(rec + dt * 16 + 4 * g) = o[dt][qt];
      if (g == 0) {
        rec[64] = m[qt];
        rec[65] = l_tot;
      }
      continue;
    }
    if (q >= d.Nq) continue;
    const float inv = 1.f / l_tot;
    if (d.lse != nullptr && g == 0) d.lse[((int64_t)b * d.H + h) * d.Nq + q] = m[qt] + __log2f(l_tot);
    bf16* orow = (bf16*)d.O + (int64_t)b * d.o_sb + (int64_t)q * d.o_sn + h * 64 + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 ov;
      bf16x4 old;
      if (d.accumulate) old = *(const bf16x4*)(orow + dt * 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = rbf(o[dt][qt][r] * inv);
        if (d.out_scale != 1.f) v = rbf(v * d.out_scale);
        if (d.accumulate) v = bf2f(old[r]) + v;
        ov[r] = f2bf(v);
      }
      *(bf16x4*)(orow + dt * 16) = ov;
    }
  }
}

// ============================================================================================================
// fp8 attention (BASELINE config 5: "attn + FFN in fp8").  Both products on the block-scaled e4m3 MFMA
// v_mfma_scale_f32_32x32x64_f8f6f4 (K = 64 per instruction: QK^T over the whole head in ONE MFMA per 32 keys, PV
// over a 64-key tile in one MFMA per 32 output dims).
//
// Operand layout of the 32x32x64 MFMA (measured by vp_mx_mfma_probe32, tests/test_attention_fp8_gpu.py): lane l
// supplies row l % 32 and the 16-byte K-chunks g = l / 32 and g + 2 (VGPRs 0-3 and 4-7), and the E8M0 scale of
// (row l % 32, K-block g), a K-block being 32 consecutive K-slots.  C/D as the bf16 32x32 MFMA.
//
// Data formats (written by vp_head_norm_rope_fp8 and vp_v_pack_fp8):
//  * Q, K: e4m3 [B, N, H*64] with ONE power-of-two factor each (Q also carries scale * log2 e), undone by the
//    MFMA's constant scale bytes.  Their magnitude is bounded by the LayerNorm (|x| <= sqrt(63)|gamma| + |beta|,
//    RoPE at most sqrt 2 more), so a static factor leaves the whole e4m3 range to the data.
//  * V^T: e4m3 [B, H, 64 (d), Npad] — keys contiguous per d so the PV A-operand is two 16-byte row reads — with
//    the keys of every 64-key tile stored in MFMA K-slot order: slot k holds key tile_key(k), the key whose score
//    the S^T accumulator gives the lane that feeds slot k of the P^T B-operand (so P needs no cross-lane move),
//    and one E8M0 scale per (d, 32-slot K-block) = per (d, 32 keys): [B, H, Npad/64, 64 lanes][2 (d-half)].
// ============================================================================================================
typedef int i32x8 __attribute__((ext_vector_type(8)));

// K-slot -> key within a 64-key tile: slot k = 32 hh + 16 g + e  <->  S^T accumulator element e of half hh held
// by lane group g (row 8 (e/4) + 4 g + e % 4 of the 32x32 C layout)
VP_DEV int tile_key(int k) {
  const int hh = k >> 5, g = (k >> 4) & 1, e = k & 15;
  return 32 * hh + 8 * (e >> 2) + 4 * g + (e & 3);
}
// 64-byte fp8 tile rows in LDS: physical 16-byte chunk = logical ^ swz8(row) (rows 4 apart land 16 banks apart)
VP_DEV int swz8(int row) { return (row >> 2) & 3; }

#if VP_DIAG  // diagnostic build only (include/vp_hip_diag.h)
// probe: one 32x32x64 scaled MFMA with the layout above; C row-major [32][32] fp32
__global__ void mx_probe32_kernel(const uint8_t* A, const uint8_t* B, const uint8_t* sa, const uint8_t* sb,
                                  float* C) {
  const int l = threadIdx.x;
  const int r = l & 31, g = l >> 5;
  i32x8 a, b;
  u32x4* ah = (u32x4*)&a;
  u32x4* bh = (u32x4*)&b;
  ah[0] = *(const u32x4*)(A + r * 64 + g * 16);
  ah[1] = *(const u32x4*)(A + r * 64 + (g + 2) * 16);
  bh[0] = *(const u32x4*)(B + r * 64 + g * 16);
  bh[1] = *(const u32x4*)(B + r * 64 + (g + 2) * 16);
  f32x16 c;
  for (int i = 0; i < 16; ++i) c[i] = 0.f;
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, (int)sa[l], 0, (int)sb[l]);
  for (int i = 0; i < 16; ++i) C[(8 * (i >> 2) + 4 * g + (i & 3)) * 32 + r] = c[i];
}
#endif

// V [B, N, ld] bf16 (head h at column h*64) -> V^T fp8 in tile K-slot order + per-(d, 32 keys) E8M0 scales.
// One 256-thread block per (b, h, 64-key tile); thread t: d = t / 4, slots 16 (t % 4) .. +15.
__global__ __launch_bounds__(256) void v_pack_fp8_kernel(const bf16* __restrict__ V, int64_t v_sb, int64_t v_sn,
                                                         int N, int H, int ntiles, uint8_t* __restrict__ vt,
                                                         uint8_t* __restrict__ vs) {
  __shared__ bf16 tile[64][64 + 8];
  const int blk = blockIdx.x;
  const int t = blk % ntiles;
  const int bh = blk / ntiles;
  const int h = bh % H, b = bh / H;
  const int tid = threadIdx.x;
  const bf16* src = V + (int64_t)b * v_sb + h * 64;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int key = pass * 32 + (tid >> 3);
    const int n = t * 64 + key;
    bf16x8 x = {};
    if (n < N) x = *(const bf16x8*)(src + (int64_t)n * v_sn + (tid & 7) * 8);
    *(bf16x8*)&tile[key][(tid & 7) * 8] = x;
  }
  __syncthreads();
  const int d = tid >> 2, qq = tid & 3;
  float v[16];
  float am = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    v[e] = bf2f(tile[tile_key(16 * qq + e)][d]);
    am = fmaxf(am, fabsf(v[e]));
  }
  am = fmaxf(am, __shfl_xor(am, 1, 64));  // the 32 slots of one K-block = two threads
  const int sx = mx_exponent(am);
  const float mul = mx_inv_scale(sx);
  float lo[8], hi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    lo[e] = v[e];
    hi[e] = v[8 + e];
  }
  const u32x2 p0 = mx_pack8(lo, mul), p1 = mx_pack8(hi, mul);
  const int64_t npad = (int64_t)ntiles * 64;
  *(u32x4*)(vt + ((int64_t)bh * 64 + d) * npad + t * 64 + 16 * qq) = (u32x4){p0[0], p0[1], p1[0], p1[1]};
  if ((qq & 1) == 0) {
    const int lane = (d & 31) + 32 * (qq >> 1);  // the MFMA lane that supplies (row d % 32, K-block qq / 2)
    vs[((int64_t)bh * ntiles + t) * 128 + lane * 2 + (d >> 5)] = (uint8_t)(sx + 127);
  }
}

constexpr int F8_TILE = 64 * 64;                   // bytes of a K or V^T tile
constexpr int F8_STAGE = 2 * F8_TILE + 128;        // + the V^T scales

// fp8 attention: NW waves x 32 queries per workgroup, 64-key tiles through a 2-slot LDS ring by LDS-DMA (waves
// 0-3: the 4 K pieces, 4-7: the 4 V^T pieces, wave 0 lanes 0-7 also the V^T scales).  Per tile: S^T for the two
// 32-key halves (C-init: S = s - m + F8_OFF), one max over both, thresholded rescale, exp2 -> P in e4m3 straight
// into the PV B-operand registers, PV as two MFMAs over all 64 keys.
// P = exp2(S) in e4m3, 4 per VGPR: VGPRs 0-3 = half 0 (K-slots 16g..), 4-7 = half 1 (32+16g..); returns this
// lane's sum of the 32 values (dead code, removed by the compiler, when the sums run on the matrix pipe)
VP_DEV float f8_exp_pack(const f32x16 (&s)[2], i32x8& pf) {
  float ps[4];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float p0 = __builtin_amdgcn_exp2f(s[hh][4 * w + 0]);
      const float p1 = __builtin_amdgcn_exp2f(s[hh][4 * w + 1]);
      const float p2 = __builtin_amdgcn_exp2f(s[hh][4 * w + 2]);
      const float p3 = __builtin_amdgcn_exp2f(s[hh][4 * w + 3]);
      // the low-word pack's "old" operand is p0's own bits (dead after this, so its register becomes the result
      // in place): its high word is overwritten by the second pack, and a literal 0 there costs a v_mov per VGPR
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(p0, p1, __float_as_int(p0), false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(p2, p3, pk, true);
      pf[hh * 4 + w] = pk;
      const float a = (p0 + p1) + (p2 + p3);
      ps[w] = hh == 0 ? a : ps[w] + a;
    }
  return (ps[0] + ps[1]) + (ps[2] + ps[3]);
}

// LIN: P in e4m3 by linear mantissa interpolation, one VALU op per score instead of v_exp_f32 (8 issue cycles) plus
// half a v_cvt_pk_fp8_f32.  The e4m3 code of a positive value 2^x is I = 8 (x + 7) at every power of two (exponent
// field E = floor(x) + 7, mantissa field M = 8 (2^frac(x) - 1) ~ 8 frac(x)), so with the scores pre-scaled by 8
// (Q's MFMA scale byte + 3) and C-initialised to LIN_C0 - 8 m, the accumulator holds 8 (s - m + OFF) + 56 - delta
// and v_cvt_pk_u8_f32 (round to nearest, clamp to [0, 255]) writes the code straight into the packed P^T operand.
// Interpolating 2^frac linearly instead of rounding 2^frac to 3 bits: relative error of P 3.2 % rms against
// 2.7 % for exp2 + RNE (delta = 0.45 centres it; 8.3 % vs 5.9 % worst case), and the row sums are taken over the
// same codes, so O = sum P V / sum P keeps the bias out.  Codes stay <= 8 (OFF + THR) + 56 = 124 < 0x7F (NaN)
// because the max path still runs every tile; masked (-inf) scores and anything below code 0 clamp to P = 0.
constexpr float LIN_DELTA = 0.45f;

// LIN 2: the same linear codes, two per v_cvt_pknorm_u16_f32 (the accumulator holds code / 2^16: the Q scale byte
// takes 2^-13 instead of 2^3 and C0 / LS are scaled alike; round(code (1 - 2^-16)) equals round(code) up to a 2e-3
// shift of the rounding boundary for codes <= 124) and a v_perm_b32 that gathers the 4 low bytes of two packed
// u16 pairs: 3 VALU per 4 scores instead of 4.  The u16 codes must stay below 256 for the byte gather, which the
// max path (every tile) guarantees: codes <= 8 (OFF + THR) + 56; masked (-inf) and negative values clamp to 0.
VP_DEV void f8_lin2_pack(const f32x16 (&s)[2], i32x8& pf) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const u16x2 lo = __builtin_amdgcn_cvt_pknorm_u16(s[hh][4 * w + 0], s[hh][4 * w + 1]);
      const u16x2 hi = __builtin_amdgcn_cvt_pknorm_u16(s[hh][4 * w + 2], s[hh][4 * w + 3]);
      pf[hh * 4 + w] = (int)__builtin_amdgcn_perm(__builtin_bit_cast(unsigned, hi), __builtin_bit_cast(unsigned, lo),
                                                  0x06040200u);
    }
}

VP_DEV void f8_lin_pack(const f32x16 (&s)[2], i32x8& pf) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unsigned pk = __builtin_amdgcn_cvt_pk_u8_f32(s[hh][4 * w + 0], 0, 0u);
      pk = __builtin_amdgcn_cvt_pk_u8_f32(s[hh][4 * w + 1], 1, pk);
      pk = __builtin_amdgcn_cvt_pk_u8_f32(s[hh][4 * w + 2], 2, pk);
      pk = __builtin_amdgcn_cvt_pk_u8_f32(s[hh][4 * w + 3], 3, pk);
      pf[hh * 4 + w] = (int)pk;
    }
}

// The kernel.  P is stored as p * 2^7 with the max path every tile and rescale threshold 1.5 (P <= 2^8.5 < 448).
// RS: the row sums on the matrix pipe instead of 28 VALU adds per lane and tile — the packed P^T operand read as the
// B operand of ONE v_mfma_scale_f32_16x16x128_f8f6f4 (lane l: column l % 16, K-chunks l / 16 and l / 16 + 4), whose
// column n then holds query n's 64 keys in K-chunks {0, 2, 4, 6} and query n + 16's in {1, 3, 5, 7}; a 0/1 e4m3
// selector as A (row 0 = the first set, row 1 = the second) leaves sum(query n) in accumulator row 0 and
// sum(query n + 16) in row 1, i.e. in lane n's registers 0 and 1.  (The sum is then over the e4m3-ROUNDED P the PV
// product uses, in fp32.)  At d = 64 the softmax VALU (32 exp2 at 8 cycles + max + pack) outweighs the tile's 4
// MFMAs (256 cycles), so moving 112 VALU cycles onto a 32-cycle MFMA is the lever.
template <int NW, int OCC, int SUB, bool RS, int LIN>
__global__ __launch_bounds__(NW * 64, OCC) void attn_fwd_fp8(const vp_attn_fp8_desc dd) {
  static_assert(NW == 8, "the DMA split assumes 8 waves");
  static_assert(RS || !LIN, "the linear codes are summed on the matrix pipe");
  constexpr int OFF = 7;        // P is stored as p * 2^OFF
  constexpr float THR = 1.5f;   // max path: P <= 2^(OFF + THR) < 448
  // accumulator units: S = LS (s - m) + C0 (log2 units + OFF for the exp2 form, e4m3 codes for LIN, codes / 2^16
  // for LIN 2)
  constexpr float USC = LIN == 2 ? 0x1p-16f : 1.f;
  constexpr float LS = LIN ? 8.f * USC : 1.f;
  constexpr float C0 = LIN ? (8.f * OFF + 56.f - LIN_DELTA) * USC : (float)OFF;
  const vp_attn_desc& d = dd.base;
  constexpr int QB = NW * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 5;

  const int nqb = (d.Nq + QB - 1) / QB;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;
  const int ntiles = dd.npad >> 6;

  const int q = qb * QB + wave * 32 + (lane & 31);
  const int qc = q < d.Nq ? q : d.Nq - 1;
  i32x8 qf;
  {
    const uint8_t* qrow = (const uint8_t*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
    u32x4* hq = (u32x4*)&qf;
    hq[0] = *(const u32x4*)(qrow + g * 16);
    hq[1] = *(const u32x4*)(qrow + (g + 2) * 16);
  }
  // LIN: scores x 8 (LIN 2: x 8 / 2^16)
  const int sq = (dd.qk_scale & 0xff) + (LIN == 2 ? 3 - 16 : LIN ? 3 : 0), sk = (dd.qk_scale >> 8) & 0xff;

  // DMA: this lane's row of its wave's piece (16 rows x 64 B) and the logical source chunk of its physical chunk,
  // held as ONE byte offset per lane (waves 0-3 stage K, 4-7 stage V^T) from a wave-uniform base that advances by
  // whole tiles; only the last K tile (rows past Nk re-read the last key) recomputes the row from the lane id.  More
  // long-lived address VGPRs get spilled at 128, and the spill reload's vmcnt(0) sits in front of the DMA issue.
  const int ksn = (int)d.k_sn;
  auto dma_off = [&](int ln) {
    const int prow = (wave & 3) * 16 + (ln >> 2);
    const int pch = (ln & 3) ^ swz8(prow);
    return wave < 4 ? prow * ksn + pch * 16 : prow * dd.npad + pch * 16;
  };
  // LIN: recomputed from the lane id at each issue (a few VALU per tile): held across the loop it is spilled
  const int dma_kept = LIN ? 0 : dma_off(lane);
  const char* kbase = (const char*)d.K + (int64_t)b * d.k_sb + h * 64;
  const char* vtbase = (const char*)d.V + (int64_t)bh * 64 * dd.npad;
  const char* vsbase = (const char*)dd.vs + (int64_t)bh * ntiles * 128;
  // ring slot ti holds SUB consecutive 64-key tiles (one barrier per SUB tiles)
  const int nsup = (ntiles + SUB - 1) / SUB;
  // LDS destinations as 32-bit LDS addresses from one wave-uniform base (no generic-pointer conversion and null
  // check per DMA instruction)
  const unsigned lds_smem = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void_t*)smem);
  const unsigned lds_base = lds_smem + (wave < 4 ? wave * 1024 : F8_TILE + (wave - 4) * 1024);
#if VP_F8_GENERIC_DMA  // A/B: the generic-pointer destination (conversion + null check per instruction)
  auto glds16_lds = [&](const char* sbase, int voff, unsigned la) { glds16(sbase, voff, smem + (la - lds_smem)); };
#endif
  auto issue = [&](int ti) {
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int kt = ti * SUB + sb;
      if (SUB > 1 && kt >= ntiles) break;  // wave-uniform
      const unsigned st = lds_base + ((ti & 1) * SUB + sb) * F8_STAGE;
      if (wave < 4) {
        if (kt * 64 + 64 <= d.Nk) {
          glds16_lds(kbase + (int64_t)kt * 64 * ksn, LIN ? dma_off(lane_id_opaque()) : dma_kept, st);
        } else {  // rows past the end re-read the last key (masked later)
          const int ln = lane_id_opaque();
          const int prow = (wave & 3) * 16 + (ln >> 2);
          const int r = min(kt * 64 + prow, d.Nk - 1);
          glds16_lds(kbase, r * ksn + (((ln & 3) ^ swz8(prow)) << 4), st);
        }
      } else {
        glds16_lds(vtbase + kt * 64, LIN ? dma_off(lane_id_opaque()) : dma_kept, st);
      }
      if (wave == 0 && lane < 8) glds16_lds(vsbase + kt * 128, lane * 16, st + 2 * F8_TILE);  // wave 0: st = slot + 0
    }
  };

  // LDS read offsets (within a stage) of this lane's two 16-byte chunks of row r: r*64 + ((c ^ swz8(r)) << 4)
  const int r0 = lane & 31;
  const int ca = (g ^ swz8(r0)) << 4, cb = ((g + 2) ^ swz8(r0)) << 4;  // swz8(r0 + 32) == swz8(r0)

  float m_run = 0.f, l_run = 0.f, thr = -INFINITY;
  f32x16 o[2], negm;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.f;
    o[1][i] = 0.f;
    negm[i] = C0;
  }
  // RS: this lane's selector word (e4m3 1.0 = 0x38) and the 16x16 accumulator of the row sums.  The 8-VGPR
  // selector tuple is re-materialised from the word next to each row-sum MFMA (after the scores died), not kept
  // live through the softmax: at 128 VGPRs that is the difference between 13 spilled registers and none.
  int selw = 0;
  f32x4 lsum = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RS) {
    const int col = lane & 15, c = lane >> 4;
    selw = ((col == 0 && (c & 1) == 0) || (col == 1 && (c & 1) == 1)) ? 0x38383838 : 0;
  }
  const bool active = qb * QB + wave * 32 < d.Nq;  // wave-uniform
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int ti = 0; ti < nsup; ++ti) {
    if (ti + 1 < nsup) issue(ti + 1);
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int kt = ti * SUB + sb;
      if (SUB > 1 && kt >= ntiles) break;
      const char* st = smem + ((ti & 1) * SUB + sb) * F8_STAGE;
      if (active) {
        f32x16 s[2];
        const int lim = d.Nk - kt * 64;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const char* kr = st + (hh * 32 + r0) * 64;
          i32x8 kf;
          u32x4* hk = (u32x4*)&kf;
          hk[0] = *(const u32x4*)(kr + ca);
          hk[1] = *(const u32x4*)(kr + cb);
          if (hh == 0) {
            s[0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, negm, 0, 0, 0, sk, 0, sq);
          } else {
            // asm: a fresh (early-clobber) destination with C = -m + OFF kept in its own registers (the builtin
            // form makes the compiler refill a copy of it with 8 v_mov_b64 per tile), then the 19 wait states a
            // VALU read of a 16-pass XDL result needs (the hazard recognizer cannot see into asm)
            asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %3, %4, %5 op_sel_hi:[0,0,0]\n\t"
                         "s_nop 15\n\ts_nop 2"
                         : "=&v"(s[1])
                         : "v"(kf), "v"(qf), "v"(negm), "v"(sk), "v"(sq));
          }
        }
        if (lim < 64) {
          mask_half(s[0], lim, 0, g);
          mask_half(s[1], lim, 1, g);
        }
        // the tile max over both halves and the lane pair, thresholded rescale of O, l, S and -m
        float mx = s[0][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s[0][i]);
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[1][i]);
        // the threshold in accumulator units (thr = -inf, then C0 + LS THR), tested on each lane's half-row max: a
        // query's max (its two lanes, l and l ^ 32) passes iff one of them does, so the ballot decides the same and
        // the pair max and its log2-unit form are computed only on the (rare) rescale path
        if (__ballot(mx > thr) != 0ull) {
          {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
            mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
          }
          float ml = mx - C0;
          if constexpr (LIN) ml *= 1.f / LS;
          const float dm = mx > thr ? ml : 0.f;
          const float alpha = __builtin_amdgcn_exp2f(-dm);
          if constexpr (RS) {
            // lane n < 16 holds the sums of queries n (this lane's) and n + 16 (lane n + 16's)
            const float a16 = __shfl(alpha, (lane_id_opaque() + 16) & 63, 64);
            lsum[0] *= alpha;
            lsum[1] *= a16;
          } else {
            l_run *= alpha;
          }
          m_run += dm;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            o[0][i] *= alpha;
            o[1][i] *= alpha;
            s[0][i] -= LS * dm;
            s[1][i] -= LS * dm;
            negm[i] = C0 - LS * m_run;
          }
          thr = C0 + LS * THR;
        }
        i32x8 pf;
        float ls = 0.f;
        if constexpr (LIN == 2) {
          f8_lin2_pack(s, pf);
        } else if constexpr (LIN) {
          f8_lin_pack(s, pf);
        } else
          ls = f8_exp_pack(s, pf);
        if constexpr (RS) {
          // opaque copy keeps the tuple inside the loop; built as 64-bit halves so the copies are v_mov_b64
          uint32_t wlo, whi;
          asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %2" : "=v"(wlo), "=v"(whi) : "v"(selw));
          const uint64_t w2 = ((uint64_t)whi << 32) | wlo;
          uint64_t w3, w4, w5;
          asm volatile("v_mov_b64 %0, %3\n\tv_mov_b64 %1, %3\n\tv_mov_b64 %2, %3" : "=v"(w3), "=v"(w4), "=v"(w5)
                       : "v"(w2));
          typedef uint64_t u64x4 __attribute__((ext_vector_type(4)));
          const i32x8 sel = __builtin_bit_cast(i32x8, (u64x4){w2, w3, w4, w5});
          lsum = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(sel, pf, lsum, 0, 0, 0, 127, 0, 127);
        }
        else
          l_run += ls;
        const int vsw = *(const unsigned short*)(st + 2 * F8_TILE + lane * 2);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const char* vr = st + F8_TILE + (dh * 32 + r0) * 64;
          i32x8 vf;
          u32x4* hv = (u32x4*)&vf;
          hv[0] = *(const u32x4*)(vr + ca);
          hv[1] = *(const u32x4*)(vr + cb);
          if (dh == 0)
            o[0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, o[0], 0, 0, 0, vsw, 0, 127);
          else
            o[1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, o[1], 0, 0, 1, vsw, 0, 127);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  if constexpr (RS) {
    const int qq = lane & 31;
    const float v0 = __shfl(lsum[0], qq & 15, 64), v1 = __shfl(lsum[1], qq & 15, 64);
    store_out(d, o, qq < 16 ? v0 : v1, q, b, h, g, false);
  } else {
    store_out(d, o, l_run, q, b, h, g);
  }
}

// Skewed fp8 attention (variants 5 / 6): the lin-2 kernel above with the wave's tile loop turned by one tile —
// QK^T of tile t is issued first, then PV and the row sums of tile t - 1, then the softmax of tile t — so the three
// MFMAs of t - 1 (160 matrix cycles) cover the QK^T result latency that the unskewed loop waits out in s_nops (two
// 17-state pads per tile).  The PV of t - 1 reads its V^T after the ring moved on by one tile, so the ring has 3
// slots (SUB tiles each): the DMA into slot (i + 1) % 3 at superstep i cannot race a skewed read of slot (i - 1) % 3.
// Each wave has ONE DMA source (waves 0-3: 16 K rows, 4-7: 16 V^T rows) as a wave-uniform base + tile stride and
// one kept per-lane offset, so a tile's issue is an address add and the LDS-DMA (the last K tile, whose rows past
// Nk re-read the last key, takes the clamped form).  Same arithmetic, same order of accumulation as variant 3
// (bit-identical results, tests/test_attention_fp8_gpu.py).  The first skewed PV is a zero P against tile 0.
constexpr int F8S_SLOTS = 3;
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) const unsigned short lds_u16;
// one 256-query block (logical id t) of attn_fwd_fp8s
template <int SUB>
VP_DEV __attribute__((always_inline)) void fp8s_block(const vp_attn_fp8_desc& dd, const int t) {
  constexpr int NW = 8;
  constexpr int OFF = 7;
  constexpr float THR = 1.5f;
  constexpr float USC = 0x1p-16f;
  constexpr float LS = 8.f * USC;
  constexpr float C0 = (8.f * OFF + 56.f - LIN_DELTA) * USC;
  const vp_attn_desc& d = dd.base;
  constexpr int QB = NW * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 5;

  const int nqb = (d.Nq + QB - 1) / QB;
  const int bh = t / nqb;
  const int qb = t - bh * nqb;
  const int b = bh / d.H;
  const int h = bh - b * d.H;
  const int ntiles = dd.npad >> 6;

  const int q = qb * QB + wave * 32 + (lane & 31);
  const int qc = q < d.Nq ? q : d.Nq - 1;
  i32x8 qf;
  {
    const uint8_t* qrow = (const uint8_t*)d.Q + (int64_t)b * d.q_sb + (int64_t)qc * d.q_sn + h * 64;
    u32x4* hq = (u32x4*)&qf;
    hq[0] = *(const u32x4*)(qrow + g * 16);
    hq[1] = *(const u32x4*)(qrow + (g + 2) * 16);
  }
  // Q's loads complete here, before the first LDS-DMA: the compiler cannot see the asm DMAs, so a vmcnt wait for Q
  // left to the first MFMA inside the loop would also wait for the DMA that superstep has just issued
  asm volatile("" ::"v"(qf));
  const int sq = (dd.qk_scale & 0xff) + 3 - 16, sk = (dd.qk_scale >> 8) & 0xff;

  // DMA source of this wave: rows (wave & 3) * 16 + lane / 4 of each 64-row tile, physical chunk lane % 4 holding
  // logical chunk (lane % 4) ^ swz8(row) (swz8(row) = (lane / 16) % 4 here)
  const bool kw = wave < 4;
  const int ksn = (int)d.k_sn;
  const int pch = (lane & 3) ^ ((lane >> 4) & 3);
  const int rstride = kw ? ksn : (int)dd.npad;
  const int voff = (lane >> 2) * rstride + pch * 16;
  const char* kbase = (const char*)d.K + (int64_t)b * d.k_sb + h * 64;
  const char* src0 = kw ? kbase + (int64_t)(wave & 3) * 16 * ksn
                        : (const char*)d.V + ((int64_t)bh * 64 + (wave & 3) * 16) * dd.npad;
  const int64_t tstride = kw ? (int64_t)64 * ksn : 64;
  const int nfull = kw ? d.Nk >> 6 : ntiles;  // tiles whose rows all lie below Nk
  const char* vsbase = (const char*)dd.vs + (int64_t)bh * ntiles * 128;
  // (the low 32 bits of a generic LDS address are the LDS offset: no address-space cast inside the persistent loop)
  const unsigned lds_smem = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)smem);
  const unsigned lds_w = lds_smem + (kw ? wave * 1024 : F8_TILE + (wave - 4) * 1024);
  const int nsup = (ntiles + SUB - 1) / SUB;
  auto issue = [&](int ti, int slot) {
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int kt = ti * SUB + sb;
      if (SUB > 1 && kt >= ntiles) break;  // wave-uniform
      const unsigned st = lds_w + (slot * SUB + sb) * F8_STAGE;
      if (kt < nfull) {
        glds16_lds(src0 + kt * tstride, voff, st);
      } else {  // the last K tile: rows past Nk re-read the last key (masked later)
        const int ln = lane_id_opaque();
        const int r = min(kt * 64 + (wave & 3) * 16 + (ln >> 2), d.Nk - 1);
        glds16_lds(kbase, r * ksn + pch * 16, st);
      }
      if (wave == 0 && lane < 8) glds16_lds(vsbase + kt * 128, lane * 16, st + 2 * F8_TILE);
    }
  };

  const int r0 = lane & 31;
  // per-lane LDS addresses of the two 16-byte chunks of row r0 (K at +0, V^T at +F8_TILE, row + 32 at +2048) and
  // of this lane's V^T scale pair, LDS base included: opaque, so each stays one VGPR and every tile's read is that
  // VGPR + an immediate (the compiler re-derives base + lane offset per tile otherwise)
  unsigned la = lds_smem + r0 * 64 + ((g ^ swz8(r0)) << 4), lb = lds_smem + r0 * 64 + (((g + 2) ^ swz8(r0)) << 4);
  unsigned lsv = lds_smem + 2 * F8_TILE + lane * 2;
  asm volatile("" : "+v"(la), "+v"(lb), "+v"(lsv));
  // the QK^T scale operands held in VGPRs (2 registers; re-materialised from SGPRs they cost 2 v_mov per tile)
  int skv = sk, sqv = sq;
  asm volatile("" : "+v"(skv), "+v"(sqv));
  float m_run = 0.f, thr = -INFINITY;
  f32x16 o[2], negm;
  // the initial C operand from an opaque copy of C0: otherwise the compiler ties the rescale path's C0 to the initial
  // splat and keeps a 16-register tuple of it in scratch (68 B per lane, stored by every wave: +0.5 GB of writes)
  float c0v = C0;
  asm volatile("" : "+v"(c0v));
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.f;
    o[1][i] = 0.f;
    negm[i] = c0v;
  }
  const int col = lane & 15, cq = lane >> 4;
  const int selw = ((col == 0 && (cq & 1) == 0) || (col == 1 && (cq & 1) == 1)) ? 0x38383838 : 0;
  const uint64_t selp = ((uint64_t)(uint32_t)selw << 32) | (uint32_t)selw;
  f32x4 lsum = {0.f, 0.f, 0.f, 0.f};
  // (no inactive waves: the last query block's waves past Nq run on clamped duplicate queries, store_out drops them)
  i32x8 pf = {0, 0, 0, 0, 0, 0, 0, 0};
  // the skewed PV + row sums of the previous tile (P in pf, its stage at byte offset pst: a constant at every call
  // site inside the unrolled ring, so all LDS addresses are a kept lane base + an immediate offset)
  auto load_v = [&](i32x8& vf, int pst, int dh) {
    u32x4* hv = (u32x4*)&vf;
    hv[0] = *(const lds_u32x4*)(uintptr_t)(la + pst + F8_TILE + dh * 2048);
    hv[1] = *(const lds_u32x4*)(uintptr_t)(lb + pst + F8_TILE + dh * 2048);
  };
  auto pv_prev = [&](int pst) {
    const int vsw = *(const lds_u16*)(uintptr_t)(lsv + pst);
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      i32x8 vf;
      load_v(vf, pst, dh);
      if (dh == 0)
        o[0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, o[0], 0, 0, 0, vsw, 0, 127);
      else
        o[1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, o[1], 0, 0, 1, vsw, 0, 127);
      // one V^T half live at a time (the scores of the next tile are live through this phase)
      __builtin_amdgcn_sched_barrier(0);
    }
    // the 8-VGPR selector tuple from the resident (selw, selw) pair: 4 v_mov_b64 (opaque, so the tuple is rebuilt
    // here rather than kept live through the softmax)
    uint64_t w2, w3, w4, w5;
    asm volatile("v_mov_b64 %0, %4\n\tv_mov_b64 %1, %4\n\tv_mov_b64 %2, %4\n\tv_mov_b64 %3, %4"
                 : "=v"(w2), "=v"(w3), "=v"(w4), "=v"(w5) : "v"(selp));
    typedef uint64_t u64x4 __attribute__((ext_vector_type(4)));
    const i32x8 sel = __builtin_bit_cast(i32x8, (u64x4){w2, w3, w4, w5});
    lsum = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(sel, pf, lsum, 0, 0, 0, 127, 0, 127);
    __builtin_amdgcn_sched_barrier(0);
  };

  // one tile: QK^T of tile kt, the skewed PV + row sums of the previous tile, then the softmax of kt into pf.
  // Keys past Nk (last tile) duplicate key Nk - 1 (the DMA clamp), so they leave the tile max as it is and only
  // their P codes are zeroed, after the pack: the result equals variant 3's -inf scores bit for bit.
  i32x8 kq[2];  // the K^T fragments of the tile
  auto load_k = [&](int stoff) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      u32x4* hk = (u32x4*)&kq[hh];
      hk[0] = *(const lds_u32x4*)(uintptr_t)(la + stoff + hh * 2048);
      hk[1] = *(const lds_u32x4*)(uintptr_t)(lb + stoff + hh * 2048);
    }
  };
  auto step = [&](int kt, int stoff, int pst) {
    f32x16 s[2];
    load_k(stoff);

#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
      s[hh] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kq[hh], qf, negm, 0, 0, 0, skv, 0, sqv);
    // phases pinned in program order: the K fragments die at the QK^T issue, before the V^T reads of pv_prev
    __builtin_amdgcn_sched_barrier(0);
    pv_prev(pst);
    float mx = s[0][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s[0][i]);
#pragma unroll
    for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[1][i]);
    if (__ballot(mx > thr) != 0ull) {  // per-lane half-row max against thr in accumulator units, as in attn_fwd_fp8
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      const float dm = mx > thr ? (mx - C0) * (1.f / LS) : 0.f;
      const float alpha = __builtin_amdgcn_exp2f(-dm);
      const float a16 = __shfl(alpha, (lane_id_opaque() + 16) & 63, 64);
      lsum[0] *= alpha;
      lsum[1] *= a16;
      m_run += dm;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o[0][i] *= alpha;
        o[1][i] *= alpha;
        s[0][i] -= LS * dm;
        s[1][i] -= LS * dm;
        negm[i] = C0 - LS * m_run;
      }
      thr = C0 + LS * THR;
    }
    f8_lin2_pack(s, pf);
    const int lim = d.Nk - kt * 64;
    if (lim < 64) {  // byte j of pf[4 hh + w] is key 32 hh + 8 w + 4 g + j (lane id opaque: nothing hoisted)
      const int kb = 4 * (lane_id_opaque() >> 5);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = lim - (32 * (i >> 2) + 8 * (i & 3) + kb);
        const unsigned mk = n >= 4 ? ~0u : n <= 0 ? 0u : (1u << (8 * n)) - 1u;
        pf[i] &= (int)mk;
      }
    }
  };
  // the first skewed PV (superstep 0, sub-tile 0) reads the stage ring slot 2's last sub-tile would hold: zeroed
  // V^T and scales there, against P = 0, add exactly 0
  constexpr int ZST = ((F8S_SLOTS - 1) * SUB + SUB - 1) * F8_STAGE + F8_TILE;
  if (tid < (F8_TILE + 128) / 16) *(u32x4*)(smem + ZST + tid * 16) = (u32x4){0u, 0u, 0u, 0u};
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // one superstep on ring slot SL (a constant): DMA of the next superstep into slot SL + 1, SUB tiles, barrier
  auto superstep = [&](int ti, auto SLC) {
    constexpr int SL = decltype(SLC)::value;
    constexpr int NSL = SL == F8S_SLOTS - 1 ? 0 : SL + 1;
    constexpr int PSL = SL == 0 ? F8S_SLOTS - 1 : SL - 1;
    if (ti + 1 < nsup) issue(ti + 1, NSL);
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int kt = ti * SUB + sb;
      if (SUB > 1 && kt >= ntiles) break;
      step(kt, (SL * SUB + sb) * F8_STAGE, sb == 0 ? (PSL * SUB + SUB - 1) * F8_STAGE : (SL * SUB + sb - 1) * F8_STAGE);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  for (int ti = 0; ti < nsup; ti += F8S_SLOTS) {
    superstep(ti, std::integral_constant<int, 0>{});
    if (ti + 1 < nsup) superstep(ti + 1, std::integral_constant<int, 1>{});
    if (ti + 2 < nsup) superstep(ti + 2, std::integral_constant<int, 2>{});
  }
  {  // the last tile's PV
    const int lt = ntiles - 1, lti = lt / SUB;
    pv_prev(((lti % F8S_SLOTS) * SUB + lt - lti * SUB) * F8_STAGE);
  }
  const int qq = lane & 31;
  const float v0 = __shfl(lsum[0], qq & 15, 64), v1 = __shfl(lsum[1], qq & 15, 64);
  store_out(d, o, qq < 16 ? v0 : v1, q, b, h, g, false);
}

// PERS: persistent (tickets: 8 zeroed counters) — resident workgroups take the blocks by per-XCD ticket (xcd_ticket):
// the XCDs run at different clocks
template <int SUB, bool PERS = false>
__global__ __launch_bounds__(512, 4) void attn_fwd_fp8s(const vp_attn_fp8_desc dd, int* tickets) {
  if constexpr (!PERS) {
    fp8s_block<SUB>(dd, xcd_remap(blockIdx.x, gridDim.x));
  } else {
    __shared__ int tk[1];
    const int n = dd.base.B * dd.base.H * ((dd.base.Nq + 255) / 256);
    const int x = (int)(blockIdx.x & 7);  // the dispatcher's XCD of this workgroup
#pragma unroll 1
    for (;;) {
      // (the two barriers also retire every wave's reads of the previous block's ring before the next DMA)
      if (threadIdx.x == 0) tk[0] = xcd_ticket(tickets, n, x);
      __syncthreads();
      const int c = tk[0];
      __syncthreads();
      if (c < 0) break;
      fp8s_block<SUB>(dd, c);
    }
  }
}

}  // namespace

namespace {
// The attention kernels of the library: the default p2a, its redo kernel a16, and the challengers kept for A/B
// (p2 = p2a without the anchor for proven score bounds, s16 = the 16x16x32 form, p2w / p2w2 = p2a in 8-wave
// workgroups).  The rejected variants of rounds 1-5 (lazy / w32 / w64 / w64f / s16i / p1 / p2wf, fp8 variants 1 and
// 4) were pruned in round 6; their measurements stay in DESIGN_LOG.md and profiles/.
struct AttnVar {
  const char* name;
  const void* fn;
  const void* fn_tail;  // the grid-tail split instance
  int threads;
  int lds;  // dynamic LDS bytes
  int qb = QB;  // queries per workgroup
  const void* fn_pers = nullptr;  // the persistent instance (p2 / p2a)
};
enum { V_S16, V_A16, V_P2, V_P2A, V_P2W, V_P2W2, V_P2S, V_NVAR };
static const AttnVar attn_vars[] = {
    {"s16", (const void*)attn_fwd_s16<false>, (const void*)attn_fwd_s16<true>, NW4 * 64, LDS_BYTES},
    {"a16", (const void*)attn_fwd_s16<false, true>, (const void*)attn_fwd_s16<true, true>, NW4 * 64, LDS_BYTES},
    {"p2", (const void*)attn_fwd_p1<false>, (const void*)attn_fwd_p1<true>, NW4 * 64, 2 * ST + 32, QB,
     (const void*)attn_fwd_p1<false, false, 4, 1, true>},
    {"p2a", (const void*)attn_fwd_p1<false, true>, (const void*)attn_fwd_p1<true, true>, NW4 * 64, 2 * ST + 32, QB,
     (const void*)attn_fwd_p1<false, true, 4, 1, true>},
    // p2a in 8-wave workgroups of 512 queries on a 4-slot ring (attn_fwd_p1 NWV = 8)
    {"p2w", (const void*)attn_fwd_p1<false, true, 8>, (const void*)attn_fwd_p1<true, true, 8>, 8 * 64, 4 * ST + 32,
     512},
    // p2w with one barrier per two tiles
    {"p2w2", (const void*)attn_fwd_p1<false, true, 8, 2>, (const void*)attn_fwd_p1<true, true, 8, 2>, 8 * 64,
     4 * ST + 32, 512},
    // p2a's pipeline on the 16x16x32 MFMA (anchored)
    {"p2s", (const void*)attn_fwd_p2s<false>, (const void*)attn_fwd_p2s<true>, NW4 * 64, 2 * ST + 16},
};
static_assert(sizeof(attn_vars) / sizeof(attn_vars[0]) == V_NVAR, "variant table");
// the anchored p2 family (a flag per block, the a16 redo)
static bool anchored_var(int v) { return v == V_P2A || v == V_P2W || v == V_P2W2 || v == V_P2S; }

struct AttnPlan {
  const AttnVar* v;
  int var;
  int64_t nblk;
  int ntail = 0, nsplit = 1;  // tail split: the last ntail blocks as ntail * nsplit key-range workgroups
  bool one_launch = false;    // the pieces ride at the end of the main grid (p2 / p2a) instead of a launch after it
  bool persist = false;       // p2 / p2a persistent instance: grid_pers workgroups take blocks and pieces by ticket
  int grid_pers = 0;
  int64_t tk_off = 0;         // the 9 ticket counters (zeroed per launch) in the workspace
  int64_t ws_bytes = 0;       // tail partials, then (p2a) the redo flags
  int64_t part_bytes = 0;     // the tail partials' part of it
};

int attn_check(const vp_attn_desc* d) {
  if (d == nullptr || d->Q == nullptr || d->K == nullptr || d->V == nullptr || d->O == nullptr) return VP_ERR_ARG;
  if (d->head_dim != 64) return VP_ERR_UNSUPPORTED;
  if (d->B <= 0 || d->H <= 0 || d->Nq <= 0 || d->Nk <= 0 || d->Nk2 < 0) return VP_ERR_ARG;
  if (d->Nk2 > 0 && (d->K2 == nullptr || d->V2 == nullptr)) return VP_ERR_ARG;
  if ((d->q_sn % 8) || (d->k_sn % 8) || (d->v_sn % 8) || (d->o_sn % 4) || (d->q_sb % 8) || (d->k_sb % 8) ||
      (d->v_sb % 8) || (d->o_sb % 4))
    return VP_ERR_ARG;
  if (d->Nk2 > 0 && ((d->k2_sn % 8) || (d->v2_sn % 8) || (d->k2_sb % 8) || (d->v2_sb % 8))) return VP_ERR_ARG;
  if (d->flags & ~VP_ATTN_BOUNDED_SCORES) return VP_ERR_ARG;
  // the LDS-DMA source offsets are 32-bit: a tile's rows must lie within 2^31 bytes of its first row
  if ((int64_t)KB * d->k_sn * 2 >= ((int64_t)1 << 31) || (int64_t)KB * d->v_sn * 2 >= ((int64_t)1 << 31))
    return VP_ERR_ARG;
  return VP_OK;
}

int variant_by_name(const char* e) {
  if (e == nullptr || e[0] == 0) return -1;
  for (int i = 0; i < V_NVAR; ++i)
    if (strcmp(e, attn_vars[i].name) == 0) return i;
  return -2;
}

int attn_plan(const vp_attn_desc* d, AttnPlan& pl) {
  static bool attr_set = false;
  static int slots_v[V_NVAR] = {};  // resident workgroups chip-wide per variant
  static int slots_p[V_NVAR] = {};  // the same for the persistent instances
  if (!attr_set) {
    attr_set = true;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    for (int i = 0; i < V_NVAR; ++i) {
      if (attn_vars[i].fn == nullptr) continue;
      (void)hipFuncSetAttribute(attn_vars[i].fn, hipFuncAttributeMaxDynamicSharedMemorySize, attn_vars[i].lds);
      (void)hipFuncSetAttribute(attn_vars[i].fn_tail, hipFuncAttributeMaxDynamicSharedMemorySize, attn_vars[i].lds);
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, attn_vars[i].fn, attn_vars[i].threads, attn_vars[i].lds) !=
          hipSuccess)
        per_cu = 0;
      slots_v[i] = per_cu * cus;
      if (attn_vars[i].fn_pers != nullptr) {
        (void)hipFuncSetAttribute(attn_vars[i].fn_pers, hipFuncAttributeMaxDynamicSharedMemorySize, attn_vars[i].lds);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, attn_vars[i].fn_pers, attn_vars[i].threads,
                                                         attn_vars[i].lds) != hipSuccess)
          per_cu = 0;
        slots_p[i] = per_cu * cus;
      }
    }
  }
  // p2a for every launch: the p2 pipeline (the software-pipelined p1 steps at two workgroups per CU, 6.04 vs 6.49 ms
  // per config-2 call for w64f, profiles/r03_attn_p2_ab.log) with the anchored softmax and a redo launch of a16 for
  // the blocks it flags (needs the workspace for its flags; without one: a16).  With VP_ATTN_BOUNDED_SCORES (the host
  // proved |score| <= VP_ATTN_SCORE_BOUND) VP_ATTN_BOUNDED_MODE may name p2 (no anchor) or s16; without it
  // VP_ATTN_UNBOUNDED_MODE may name a16 (A/B; a variant outside this build is VP_ERR_UNSUPPORTED).
  const bool bounded = (d->flags & VP_ATTN_BOUNDED_SCORES) != 0;
  int variant = variant_by_name(vp_knob(bounded ? VPK_ATTN_BOUNDED_MODE : VPK_ATTN_UNBOUNDED_MODE));
  if (variant == -2) return VP_ERR_UNSUPPORTED;
  // default: p2a for every launch (6.13 ms per config-2 call against 6.15-6.30 for p2 interleaved,
  // profiles/r04_attn_p2a_ab.log: the anchor costs nothing and no bound has to hold); p2 stays the bounded challenger
  if (variant < 0) variant = V_P2A;
  // an unbounded launch needs a kernel that does not assume the bound: lazy, a16, p2a or p2w
  const bool anchored = anchored_var(variant);
  if (!bounded && variant != V_A16 && !anchored) return VP_ERR_UNSUPPORTED;
  if (attn_vars[variant].fn == nullptr) return VP_ERR_UNSUPPORTED;
  // the resample processor's segment hints: k2_len / l_extra (the closed-form null keys, the default) are taken by
  // s16 / a16 and p1 / p2 / p2a; k2_full (null keys as zero-value keys) by the 16x16x32 kernels only (config 4 ran
  // s16 + k2_full at 11.3 ms per call against 13.8 for a w64 instance with the hint, profiles/r03_bench_config4_*),
  // so a k2_full launch, and any hinted launch of another kernel, takes s16 (bounded) / a16 (unbounded)
  if (d->k2_full != nullptr || d->k2_len != nullptr || d->l_extra != nullptr) {
    const bool takes = variant == V_S16 || variant == V_A16 ||
                       ((variant == V_P2 || anchored) && d->k2_full == nullptr);
    if (!takes) variant = bounded ? V_S16 : V_A16;
  }
  pl.var = variant;
  pl.v = &attn_vars[variant];
  const int slots = slots_v[variant];
  const int nqb = (d->Nq + pl.v->qb - 1) / pl.v->qb;
  pl.nblk = (int64_t)d->B * d->H * nqb;
  if (pl.nblk > 0x7fffffff) return VP_ERR_ARG;
  const char* ns = vp_knob(VPK_ATTN_NO_SPLIT);
  if (slots > 0 && (ns == nullptr || ns[0] == '0')) {
    const int tail = (int)(pl.nblk % slots);
    const int ntile = (d->Nk + KB - 1) / KB + (d->Nk2 > 0 ? (d->Nk2 + KB - 1) / KB : 0);
    // p2 / p2a: one launch whose last workgroups are the key-range pieces (S per block) of the remainder blocks —
    // dispatched last, they fill the slots the main blocks' uneven finish leaves idle, where the two-launch split
    // below first waits for the slowest main block.  S = min(8, ceil(2 slots / remainder)): about two rounds of
    // pieces.  Config 2 (64 remainder blocks, S = 8) 6.22 vs 6.26 ms; B = 1 (288 remainder blocks, no two-launch
    // split: 2 x 288 > 512 slots; S = 4) 3.15 vs 3.26 ms; splitting whole rounds as well (R > 0) is slower
    // (profiles/r06_attn_one_launch_tail_ab.log).  VP_ATTN_TAIL = "R:S" sets R extra whole rounds and S (A/B),
    // "legacy" the two-launch split.
    const char* tk = vp_knob(VPK_ATTN_TAIL);
    int R = 0, S1 = tail > 0 ? min(8, (2 * slots + tail - 1) / tail) : 0;
    if (tk != nullptr && (sscanf(tk, "%d:%d", &R, &S1) != 2 || R < 0 || R > 4 || S1 < 2 || S1 > 8)) R = -1;
    const bool p1v = pl.var == V_P2 || pl.var == V_P2A;
    const int64_t nt = tail + (int64_t)max(R, 0) * slots;
    if (p1v && R >= 0 && nt > 0 && nt + slots <= pl.nblk && min(S1, ntile) >= 2) {
      // (at least one whole round stays unsplit; a grid under two rounds keeps the two-launch rule below)
      pl.ntail = (int)nt;
      pl.nsplit = min(S1, ntile);
      pl.one_launch = true;
      pl.part_bytes = nt * pl.nsplit * pl.v->qb * 66 * 4;
    } else if (tail > 0 && 2 * tail <= slots) {
      const int S = min(min(8, slots / tail), ntile);
      if (S >= 2) {
        pl.ntail = tail;
        pl.nsplit = S;
        pl.part_bytes = (int64_t)tail * S * pl.v->qb * 66 * 4;
      }
    }
  }
  pl.ws_bytes = pl.part_bytes;
  if (anchored_var(pl.var)) pl.ws_bytes += ((pl.nblk - pl.ntail) + (int64_t)pl.ntail * pl.nsplit) * 4;
  // persistent p2 / p2a (VP_ATTN_PERSIST=0: one workgroup per block): XCD-balanced by tickets, for grids of at least
  // two rounds (with the remainder's pieces, if split, handed out last)
  const char* pk = vp_knob(VPK_ATTN_PERSIST);
  const int sp_ = slots_p[pl.var];
  if (pl.v->fn_pers != nullptr && sp_ > 0 && (pk == nullptr || pk[0] != '0') && (pl.ntail == 0 || pl.one_launch) &&
      pl.nblk >= 2 * (int64_t)sp_) {
    pl.persist = true;
    const int64_t items = pl.nblk - pl.ntail + (int64_t)pl.ntail * pl.nsplit;
    pl.grid_pers = (int)min((int64_t)sp_, items);
    pl.tk_off = (pl.ws_bytes + 15) & ~(int64_t)15;
    pl.ws_bytes = pl.tk_off + 64;
  }
  return VP_OK;
}
}  // namespace

extern "C" int vp_attention_variant_built(const char* name) {
  if (name != nullptr && strncmp(name, "fp8:", 4) == 0) {  // the fp8 kernel's VP_ATTN8_VARIANT values
    const int f = atoi(name + 4);
    return f == 2 || f == 3 || f == 5 ? 1 : 0;
  }
  const int v = variant_by_name(name);
  return v >= 0 && attn_vars[v].fn != nullptr ? 1 : 0;
}

extern "C" int64_t vp_attention_workspace_bytes(const vp_attn_desc* d) {
  if (attn_check(d) != VP_OK) return -1;
  AttnPlan pl;
  if (attn_plan(d, pl) != VP_OK) return -1;
  return pl.ws_bytes;
}

extern "C" int vp_attention_fwd_bf16_ws(const vp_attn_desc* d, void* workspace, int64_t workspace_bytes,
                                        void* stream) {
  int rc = attn_check(d);
  if (rc != VP_OK) return rc;
  AttnPlan pl;
  rc = attn_plan(d, pl);
  if (rc != VP_OK) return rc;
  const bool have_ws = workspace != nullptr && workspace_bytes >= pl.ws_bytes && ((uintptr_t)workspace & 15) == 0;
  if (anchored_var(pl.var) && !have_ws) {
    // p2a / p2w need their redo flags: without the workspace, the anchored 16x16x32 kernel alone (unsplit)
    pl.nblk = (int64_t)d->B * d->H * ((d->Nq + QB - 1) / QB);  // a16's 256-query blocks
    pl.var = V_A16;
    pl.v = &attn_vars[V_A16];
    pl.ntail = 0;
    pl.nsplit = 1;
    pl.persist = false;
  }
  const AttnVar& v = *pl.v;
  const bool split = pl.ntail > 0 && have_ws;
  const int64_t main_blocks = split ? pl.nblk - pl.ntail : pl.nblk;
  int* flags = anchored_var(pl.var) ? (int*)((char*)workspace + pl.part_bytes) : nullptr;
  hipError_t le = hipSuccess;
  if (pl.persist && have_ws) {
    // persistent: grid_pers workgroups take the whole blocks (each XCD its xcd_remap range, then the others') and
    // then the pieces by ticket
    int* tickets = (int*)((char*)workspace + pl.tk_off);
    le = hipMemsetAsync(tickets, 0, 64, (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
    const AttnSplit sp = {(int)main_blocks, split ? pl.nsplit : 1, (float*)workspace, flags, (int)main_blocks,
                          split ? pl.nsplit : 1, 0, 0, (int)main_blocks, tickets,
                          split ? pl.ntail * pl.nsplit : 0};
    void* args[] = {(void*)d, (void*)&sp};
    le = hipLaunchKernel(v.fn_pers, dim3((unsigned)pl.grid_pers), dim3(v.threads), args, v.lds, (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
  } else if (split && pl.one_launch) {
    // whole blocks first, then the pieces: one grid, dispatched in blockIdx order
    const AttnSplit sp = {(int)main_blocks, pl.nsplit, (float*)workspace, flags, (int)main_blocks, pl.nsplit, 0, 0,
                          (int)main_blocks};
    void* args[] = {(void*)d, (void*)&sp};
    le = hipLaunchKernel(v.fn, dim3((unsigned)(main_blocks + (int64_t)pl.ntail * pl.nsplit)), dim3(v.threads), args,
                         v.lds, (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
  } else if (main_blocks > 0) {
    const AttnSplit none = {0, 1, nullptr, flags, (int)main_blocks, pl.nsplit, 0};
    void* args[] = {(void*)d, (void*)&none};
    le = hipLaunchKernel(v.fn, dim3((unsigned)main_blocks), dim3(v.threads), args, v.lds, (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
  }
  if (split) {
    if (!pl.one_launch && !(pl.persist && have_ws)) {
      const AttnSplit sp = {(int)main_blocks, pl.nsplit, (float*)workspace, flags, (int)main_blocks, pl.nsplit, 0};
      void* args[] = {(void*)d, (void*)&sp};
      le = hipLaunchKernel(v.fn_tail, dim3((unsigned)(pl.ntail * pl.nsplit)), dim3(v.threads), args, v.lds,
                           (hipStream_t)stream);
      if (le != hipSuccess) return (int)le;
    }
    const int nthreads = pl.ntail * v.qb * 16;
    hipLaunchKernelGGL(attn_combine_kernel, dim3((nthreads + 255) / 256), dim3(256), 0, (hipStream_t)stream, *d,
                       (int)main_blocks, pl.ntail, pl.nsplit, v.qb, (const float*)workspace, (const int*)flags);
  }
  if (flags != nullptr) {
    // the blocks p2a / p2w flagged, exactly, with the anchored 16x16x32 kernel (every other workgroup returns at
    // once); its blocks are 256 queries, p2w's flags per 512 (flag_shift)
    const AttnVar& r = attn_vars[V_A16];
    const int shift = v.qb == 512 ? 1 : 0;
    const AttnSplit rs = {0, 1, nullptr, flags, (int)main_blocks, split ? pl.nsplit : 1, 1, shift};
    const int64_t rblk = (int64_t)d->B * d->H * ((d->Nq + QB - 1) / QB);
    void* args[] = {(void*)d, (void*)&rs};
    le = hipLaunchKernel(r.fn, dim3((unsigned)rblk), dim3(r.threads), args, r.lds, (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
  }
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_attention_fwd_bf16(const vp_attn_desc* d, void* stream) {
  return vp_attention_fwd_bf16_ws(d, nullptr, 0, stream);
}

#if VP_CLOCK_STAMPS
// diagnostic builds only (not in include/vp_hip.h): the stamps of the last launches, 4 x u64 per workgroup slot
extern "C" int vp_diag_clock_read(void* host, int64_t slots) {
  if (host == nullptr || slots <= 0 || slots > CLOCK_SLOTS) return VP_ERR_ARG;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vp_clock_buf), (size_t)slots * 32, 0, hipMemcpyDeviceToHost);
}
#endif

#if VP_DIAG
extern "C" int vp_mx_mfma_probe32(const void* A, const void* B, const void* sa, const void* sb, float* C,
                                  void* stream) {
  if (!A || !B || !sa || !sb || !C) return VP_ERR_ARG;
  hipLaunchKernelGGL(mx_probe32_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t*)A,
                     (const uint8_t*)B, (const uint8_t*)sa, (const uint8_t*)sb, C);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
#endif

extern "C" int64_t vp_v_pack_fp8_bytes(int32_t B, int32_t H, int32_t N, int64_t* npad, int64_t* scale_bytes) {
  if (B <= 0 || H <= 0 || N <= 0) return -1;
  const int64_t np = ((int64_t)N + 63) / 64 * 64;
  if (npad) *npad = np;
  if (scale_bytes) *scale_bytes = (int64_t)B * H * (np / 64) * 128;
  return (int64_t)B * H * 64 * np;
}

extern "C" int vp_v_pack_fp8(const void* V, int64_t v_sb, int64_t v_sn, int32_t B, int32_t N, int32_t H, void* vt,
                             void* vs, void* stream) {
  if (!V || !vt || !vs || B <= 0 || N <= 0 || H <= 0 || (v_sn % 8) || (v_sb % 8)) return VP_ERR_ARG;
  const int ntiles = (N + 63) / 64;
  const int64_t grid = (int64_t)B * H * ntiles;
  if (grid > 0x7fffffff) return VP_ERR_ARG;
  hipLaunchKernelGGL(v_pack_fp8_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, (const bf16*)V,
                     v_sb, v_sn, N, H, ntiles, (uint8_t*)vt, (uint8_t*)vs);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

namespace {
// resident workgroups of the persistent fp8 kernel chip-wide (0: none)
int fp8_pers_slots() {
  static int slots = -1;
  if (slots < 0) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_fp8s<2, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              F8S_SLOTS * 2 * F8_STAGE);
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)attn_fwd_fp8s<2, true>, 512,
                                                     F8S_SLOTS * 2 * F8_STAGE) != hipSuccess)
      per_cu = 0;
    slots = per_cu * cus;
  }
  return slots;
}
}  // namespace

// the persistent default kernel's ticket counters (VP_ATTN_PERSIST=0 or VP_ATTN8_VARIANT != 5: none)
extern "C" int64_t vp_attention_fp8_workspace_bytes(const vp_attn_fp8_desc* dd) {
  if (dd == nullptr) return -1;
  const char* e = vp_knob(VPK_ATTN8_VARIANT);
  const char* pk = vp_knob(VPK_ATTN_PERSIST);
  if ((e != nullptr && atoi(e) != 5 && atoi(e) >= 1 && atoi(e) <= 5) || (pk != nullptr && pk[0] == '0')) return 0;
  const int slots = fp8_pers_slots();
  const int64_t grid = (int64_t)dd->base.B * dd->base.H * ((dd->base.Nq + 255) / 256);
  return slots > 0 && grid >= 2 * (int64_t)slots ? 64 : 0;
}

extern "C" int vp_attention_fwd_fp8(const vp_attn_fp8_desc* dd, void* stream) {
  return vp_attention_fwd_fp8_ws(dd, nullptr, 0, stream);
}

extern "C" int vp_attention_fwd_fp8_ws(const vp_attn_fp8_desc* dd, void* ws, int64_t ws_bytes, void* stream) {
  if (dd == nullptr) return VP_ERR_ARG;
  int* workspace = ws != nullptr && ws_bytes >= 64 && ((uintptr_t)ws & 15) == 0 &&
                           vp_attention_fp8_workspace_bytes(dd) > 0
                       ? (int*)ws
                       : nullptr;
  const vp_attn_desc& d = dd->base;
  if (!d.Q || !d.K || !d.V || !d.O || !dd->vs) return VP_ERR_ARG;
  if (d.head_dim != 64 || d.Nk2 != 0) return VP_ERR_UNSUPPORTED;
  if (d.B <= 0 || d.H <= 0 || d.Nq <= 0 || d.Nk <= 0) return VP_ERR_ARG;
  if (dd->npad != (d.Nk + 63) / 64 * 64) return VP_ERR_ARG;
  if ((d.q_sn % 16) || (d.k_sn % 16) || (d.q_sb % 16) || (d.k_sb % 16) || (d.o_sn % 4) || (d.o_sb % 4))
    return VP_ERR_ARG;
  if ((int64_t)d.Nk * d.k_sn > 0x7fffffff || (int64_t)64 * dd->npad > 0x7fffffff) return VP_ERR_ARG;
  constexpr int NW = 8;
  // VP_ATTN8_VARIANT (A/B): 1 = P by v_exp_f32 + RNE pack, 2 = P by linear mantissa interpolation (LIN),
  // 3 = the same codes packed two per v_cvt_pknorm_u16_f32 + a byte gather (LIN 2, default: 2.11-2.15 against
  // 2.04-2.11 PF/s for 2, interleaved at config 5's length, profiles/r03_fp8_lin2_ab.log);
  // both with the row sums on the matrix pipe, 128 keys per barrier at 4 waves/SIMD.  Dropped after A/B: row sums on
  // the VALU (1.40 against 1.50 PF/s), lazy max (159 VGPRs, spills: 0.21 PF/s), 3 waves/SIMD (1.01), 64 keys per
  // barrier (1.43 against 1.46); 4 = f8p, the lin2 codes in a p1-style software pipeline at 2 waves/SIMD: parity
  // identical to 3, but 0.93-0.94x its speed (profiles/r03_f8p_ab_rejected.log: at two waves per SIMD the wave's own
  // instruction issue, ~13 VALU + ~6 SALU per MFMA, not the matrix pipe, sets the step), kept for A/B.
  // 5 = the lin-2 kernel with its tile loop skewed by one tile (attn_fwd_fp8s; default since round 4: bit-identical
  // to 3, 2.28-2.30 against 2.22-2.24 PF/s interleaved at config 5's length, profiles/r04_fp8_skew_ab.log; a 3-tile
  // ring slot (1.26-1.71), K^T read one tile ahead (spills) and the first V^T half read beside K^T (-1.2 %) were
  // measured and dropped; so was its MFMA issue at raised wave priority, within noise, profiles/r04_fp8_prio_ab_rejected.log).
  // variants 1 (exp2 + RNE) and 4 (f8p) were rejected A/B forms, pruned in round 6 (DESIGN_LOG.md)
  static const void* const fns[] = {nullptr, (const void*)attn_fwd_fp8<NW, 4, 2, true, 1>,
                                    (const void*)attn_fwd_fp8<NW, 4, 2, true, 2>};
  static bool attr_set = false;
  if (!attr_set) {
    attr_set = true;
    for (int i = 0; i < 3; ++i)
      if (fns[i] != nullptr)
        (void)hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 2 * F8_STAGE);
    (void)hipFuncSetAttribute((const void*)attn_fwd_fp8s<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              F8S_SLOTS * 2 * F8_STAGE);
    (void)hipFuncSetAttribute((const void*)attn_fwd_fp8s<2, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              F8S_SLOTS * 2 * F8_STAGE);
  }
  const char* e = vp_knob(VPK_ATTN8_VARIANT);
  int variant = e != nullptr ? atoi(e) : 0;
  if (variant < 1 || variant > 5) variant = 5;
  if (variant == 5) {  // the skewed loop (default)
    constexpr int sub = 2;
    const int nqb5 = (d.Nq + NW * 32 - 1) / (NW * 32);
    const int64_t grid5 = (int64_t)d.B * d.H * nqb5;
    if (grid5 > 0x7fffffff) return VP_ERR_ARG;
    const int slots = fp8_pers_slots();
    int* tickets = workspace;
    if (tickets != nullptr && slots > 0 && grid5 >= 2 * (int64_t)slots) {
      // persistent (vp_attention_fp8_workspace_bytes > 0)
      hipError_t le = hipMemsetAsync(tickets, 0, 32, (hipStream_t)stream);
      if (le != hipSuccess) return (int)le;
      void* args5[] = {(void*)dd, (void*)&tickets};
      le = hipLaunchKernel((const void*)attn_fwd_fp8s<sub, true>, dim3((unsigned)slots), dim3(NW * 64), args5,
                           F8S_SLOTS * sub * F8_STAGE, (hipStream_t)stream);
      if (le != hipSuccess) return (int)le;
      VP_CHECK_LAUNCH();
      return VP_OK;
    }
    int* none = nullptr;
    void* args5[] = {(void*)dd, (void*)&none};
    const hipError_t le5 =
        hipLaunchKernel((const void*)attn_fwd_fp8s<sub>, dim3((unsigned)grid5),
                        dim3(NW * 64), args5, F8S_SLOTS * sub * F8_STAGE, (hipStream_t)stream);
    if (le5 != hipSuccess) return (int)le5;
    VP_CHECK_LAUNCH();
    return VP_OK;
  }
  if (variant == 1 || variant == 4) return VP_ERR_UNSUPPORTED;
  const int nqb = (d.Nq + NW * 32 - 1) / (NW * 32);
  const int64_t grid = (int64_t)d.B * d.H * nqb;
  if (grid > 0x7fffffff) return VP_ERR_ARG;
  void* args[] = {(void*)dd};
  const hipError_t le = hipLaunchKernel(fns[variant - 1], dim3((unsigned)grid), dim3(NW * 64), args, 2 * 2 * F8_STAGE,
                                        (hipStream_t)stream);
  if (le != hipSuccess) return (int)le;
  VP_CHECK_LAUNCH();
  return VP_OK;
}
