// CogVideoX 3D causal VAE kernels for gfx950 (MI355X): implicit-GEMM conv3d on MFMA, GroupNorm (+ the decoder's
// spatial-norm modulation and SiLU), temporal 2:1 pooling, NCDHW <-> channels-last layout, latent distribution.
// Reference: DF/models/autoencoders/autoencoder_kl_cogvideox.py; the ABI is include/vp_hip.h.
//
// conv3d as an implicit GEMM: rows = output pixels (b, t, y, x), columns = output channels, K = (tap, input channel)
// with the channels contiguous in the channels-last activation, so every 16-byte K-chunk of an A row is one
// 16-byte read of one input pixel (or of a zero chunk where the tap falls into the padding).  Tile 128 pixels x BN
// channels x 64 K, 4 waves, 16x16x32 bf16 MFMA with the weight fragment as the first operand (each lane's
// accumulator = 4 consecutive output channels of one pixel), operand tiles staged by LDS-DMA
// (global_load_lds_dwordx4: per-lane gather source, lane-linear LDS destination, bank swizzle on the source address
// and undone on the read), 2-stage ring.  Roofline: MFMA-bound for Cin >= 64 (AI = 2*128*BN*64 / 16+BN/8 KB).
#include <stdlib.h>

#include "vp_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

__device__ __attribute__((aligned(16))) bf16 g_zero16[8];  // 16 zero bytes: the source of padding taps / K tail

constexpr int CBM = 128, CBK = 64, CNT = 256;

VP_DEV int cswz(int row) { return (row >> 1) & 7; }

template <int BN>
struct ConvGeom {
  static constexpr int WAVES_M = BN >= 128 ? 2 : 4;
  static constexpr int WAVES_N = 4 / WAVES_M;
  static constexpr int WM = CBM / WAVES_M, WN = BN / WAVES_N;
  static constexpr int FM = WM / 16, FN = WN / 16;
  static constexpr int A_BYTES = CBM * CBK * 2;  // 16 KB
  static constexpr int B_BYTES = BN * CBK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int B_INSTR = BN * 8 / CNT;  // 16-byte weight chunks per thread per K-tile
  static constexpr int LDS = 2 * STAGE + VP_CONV_MAX_T * 4;
};

VP_DEV void glds16(const bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)lds, 16, 0, 0);
}

// HOIST (Cin >= 64): a 64-channel K-tile never straddles a tap, so the tap of K-tile kt is wave-uniform and each of
// this lane's 4 A rows needs its gather address only once per tap (then + the tile's channel offset): 3 VALU per
// row and K-tile instead of the full tap decode + bounds + 64-bit pixel arithmetic (~25 VALU), which on the
// 128-channel high-resolution convs issued as many VALU cycles as the tile's 32 MFMAs.  The weight rows are one
// 64-bit pointer per instruction plus a uniform K offset.
template <int BN, bool HOIST>
__global__ __launch_bounds__(CNT, 2) void conv3d_kernel(const vp_conv3d_desc d, int c8s) {
  using G = ConvGeom<BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tmapl = (int*)(smem + 2 * G::STAGE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / G::WAVES_N, wc = wave % G::WAVES_N;

  const int HWo = d.Hout * d.Wout;
  const int64_t THWo = (int64_t)d.Tout * HWo;
  const int64_t M = (int64_t)d.B * THWo;
  const int tiles_n = (d.Cout + BN - 1) / BN;
  const int tl = xcd_remap(blockIdx.x, gridDim.x);  // consecutive logical tiles (same pixels, all N) share an XCD
  const int n0 = (tl % tiles_n) * BN;
  const int64_t m0 = (int64_t)(tl / tiles_n) * CBM;

  const int nv = d.Tout + d.kt - 1;
  for (int v = tid; v < nv; v += CNT) tmapl[v] = d.tmap[v];

  // this lane's 4 A rows (one per LDS-DMA instruction): validity, batch, output frame, top-left input position
  const int C8 = d.Cin >> 3;
  const int khw = d.kh * d.kw;
  const int kc_total = d.kt * khw * C8;  // 16-byte K-chunks
  const int64_t Ktot = (int64_t)kc_total * 8;
  const int Hu = d.Hin * d.uh, Wu = d.Win * d.uw;
  const int ush = d.uh >> 1, usw = d.uw >> 1;
  const int64_t HWi = (int64_t)d.Hin * d.Win;
  int rb[4], rt[4], ry[4], rx[4];
  bool rv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (i * 4 + wave) * 8 + (lane >> 3);
    const int64_t m = m0 + r;
    rv[i] = m < M;
    const int64_t mm = rv[i] ? m : 0;
    const int b = (int)(mm / THWo);
    const int rem = (int)(mm - (int64_t)b * THWo);
    const int t = rem / HWo;
    const int rem2 = rem - t * HWo;
    const int yo = rem2 / d.Wout;
    const int xo = rem2 - yo * d.Wout;
    rb[i] = b;
    rt[i] = t;
    ry[i] = yo * d.sh - d.ph;
    rx[i] = xo * d.sw - d.pw;
  }
  const bf16* X = (const bf16*)d.x;
  const bf16* Hs = (const bf16*)d.hist;
  const bf16* Wt = (const bf16*)d.w;

  // source pixel (element offset of its channel 0, from X or the history) of row i at tap (dt, dy, dx), or null
  auto row_src = [&](int i, int dt, int dy, int dx) -> const bf16* {
    const int yu = ry[i] + dy, xu = rx[i] + dx;
    if (!rv[i] || yu < 0 || yu >= Hu || xu < 0 || xu >= Wu) return nullptr;
    const int f = tmapl[rt[i] + dt];
    const int64_t pix = (f >= 0 ? (int64_t)rb[i] * d.x_frames + f : (int64_t)rb[i] * d.hist_frames + (-1 - f)) *
                            HWi + (int64_t)(yu >> ush) * d.Win + (xu >> usw);
    return (f >= 0 ? X : Hs) + pix * d.Cin;
  };

  // HOIST state: per row the tap's source address (+ this lane's swizzled chunk) and a keep-offset mask
  const char* abase[4];
  int amask[4];
  const char* wbase[G::B_INSTR];
  const int tpt = HOIST ? (C8 >> 3) : 1;  // K-tiles per tap (power of two)
  if constexpr (HOIST) {
#pragma unroll
    for (int j = 0; j < G::B_INSTR; ++j) {
      const int r = (j * 4 + wave) * 8 + (lane >> 3);
      const int n = min(n0 + r, d.Cout - 1);
      wbase[j] = (const char*)(Wt + (int64_t)n * Ktot + (((lane & 7) ^ cswz(r)) << 3));
    }
  }
  auto set_tap = [&](int tap) {  // HOIST: wave-uniform tap
    const int dt = khw == 1 ? tap : tap / khw;
    const int rem = tap - dt * khw;
    const int dy = d.kw == 1 ? rem : rem / 3;
    const int dx = rem - dy * d.kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (i * 4 + wave) * 8 + (lane >> 3);
      const bf16* p = row_src(i, dt, dy, dx);
      amask[i] = p != nullptr ? -1 : 0;
      abase[i] = p != nullptr ? (const char*)(p + (((lane & 7) ^ cswz(r)) << 3)) : (const char*)g_zero16;
    }
  };

  auto stage = [&](int kt, char* buf) {
    if constexpr (HOIST) {
      if ((kt & (tpt - 1)) == 0) set_tap(kt / tpt);
      const int cb = (kt & (tpt - 1)) * 128;  // byte offset of the tile's 64 channels within the tap
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16((const bf16*)(abase[i] + (cb & amask[i])), buf + (i * 4 + wave) * 1024);
#pragma unroll
      for (int j = 0; j < G::B_INSTR; ++j)
        glds16((const bf16*)(wbase[j] + (int64_t)kt * 128), buf + G::A_BYTES + (j * 4 + wave) * 1024);
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rbase = (i * 4 + wave) * 8;
      const int r = rbase + (lane >> 3);
      const int kc = kt * 8 + ((lane & 7) ^ cswz(r));
      const bf16* src = g_zero16;
      if (rv[i] && kc < kc_total) {
        const int tap = kc >> c8s;
        const int cin = (kc & (C8 - 1)) << 3;
        const int dt = khw == 1 ? tap : (tap * 57) >> 9;  // tap / 9 for tap < 64
        const int rem = tap - dt * khw;
        const int dy = d.kw == 1 ? rem : (rem * 11) >> 5;  // rem / 3 for rem < 9
        const int dx = rem - dy * d.kw;
        const bf16* p = row_src(i, dt, dy, dx);
        if (p != nullptr) src = p + cin;
      }
      glds16(src, buf + rbase * 128);
    }
#pragma unroll
    for (int j = 0; j < G::B_INSTR; ++j) {
      const int rbase = (j * 4 + wave) * 8;
      const int r = rbase + (lane >> 3);
      const int kc = kt * 8 + ((lane & 7) ^ cswz(r));
      const int n = min(n0 + r, d.Cout - 1);
      const bf16* src = kc < kc_total ? Wt + (int64_t)n * Ktot + (int64_t)kc * 8 : g_zero16;
      glds16(src, buf + G::A_BYTES + rbase * 128);
    }
  };

  f32x4 acc[G::FN][G::FM];
#pragma unroll
  for (int j = 0; j < G::FN; ++j)
#pragma unroll
    for (int i = 0; i < G::FM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // tmap in LDS
  const int nk = (kc_total + 7) / 8;
  stage(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int lrow = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * G::STAGE;
    if (kt + 1 < nk) stage(kt + 1, smem + ((kt + 1) & 1) * G::STAGE);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[G::FM], wf[G::FN];
#pragma unroll
      for (int i = 0; i < G::FM; ++i) {
        const int row = wr * G::WM + i * 16 + lrow;
        af[i] = *(const bf16x8*)(cur + row * 128 + ((ch ^ cswz(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < G::FN; ++j) {
        const int row = wc * G::WN + j * 16 + lrow;
        wf[j] = *(const bf16x8*)(cur + G::A_BYTES + row * 128 + ((ch ^ cswz(row)) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < G::FN; ++j)
#pragma unroll
        for (int i = 0; i < G::FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds channels n..n+3 of pixel m per fragment; bias, bf16 rounding (the reference's conv output),
  // residual add (the resnet's `hidden_states + inputs`), 8-byte stores; channels [Cout, ldy) are written as 0
  const bf16* bias = (const bf16*)d.bias;
  const bf16* R = (const bf16*)d.resid;
  bf16* Y = (bf16*)d.y;
#pragma unroll
  for (int j = 0; j < G::FN; ++j) {
    const int n = n0 + wc * G::WN + j * 16 + (lane >> 4) * 4;
    if (n >= d.ldy) continue;
    float bv[4];
    if (bias != nullptr && n + 3 < d.Cout) {  // one 8-byte load (per-element loads came out as serial round trips)
      const bf16x4 b4 = *(const bf16x4*)(bias + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bf2f(b4[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (bias != nullptr && n + r < d.Cout) ? bf2f(bias[n + r]) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < G::FM; ++i) {
      const int64_t m = m0 + wr * G::WM + i * 16 + lrow;
      if (m >= M) continue;
      bf16x4 rv4;
      if (R != nullptr && n < d.Cout) rv4 = *(const bf16x4*)(R + m * d.ldr + n);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = rbf(acc[j][i][r] + bv[r]);
        if (R != nullptr && n < d.Cout) v += bf2f(rv4[r]);
        o[r] = f2bf(n + r < d.Cout ? v : 0.f);
      }
      *(bf16x4*)(Y + m * d.ldy + n) = o;
    }
  }
}

// ---- PIPE: the counted-vmcnt pipeline for the wide convolutions (Cin >= 64, Cout > 64) ----
// 8 waves, 256 pixels x 128 channels per workgroup (4 x 2 waves of 64 x 64, the same per-wave fragment code as above),
// 64-K tiles through a 3-slot LDS ring (48 KB per slot, one workgroup per CU, 2 waves per SIMD).  The DMA of tile
// kt + 2 is issued right after the barrier that opens tile kt, so two tiles' loads stay in flight across every
// barrier and the wait before it is counted (vmcnt(6): the next tile's 6 loads per thread may still be pending),
// never a drain — the GEMM's pipelining rule (cdna_hip_programming.md §5 "Pipelining across barriers").  The DMA is
// inline asm: with the builtin the compiler would wait for every LDS-DMA write before each LDS read.
constexpr int PBM = 256, PBN = 128, PNT = 512, PSLOTS = 3;
constexpr int P_A = PBM * CBK * 2;                           // 32 KB
constexpr int P_B = PBN * CBK * 2;                           // 16 KB
constexpr int P_STAGE = P_A + P_B;                           // 48 KB
constexpr int P_LDS = PSLOTS * P_STAGE + VP_CONV_MAX_T * 4;  // 144.5 KB
constexpr int P_AI = PBM * 8 / PNT;                          // A chunks (DMA instructions) per thread and K-tile
constexpr int P_BI = PBN * 8 / PNT;                          // B chunks
static_assert(P_AI == 4 && P_BI == 2, "vmcnt(6) below = one K-tile of DMA per thread");

VP_DEV void glds16_asm(const void* src, char* lds) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(la), "v"(src) : "memory", "m0");
}

// V2 (default, VP_CONV_PIPE=2; 1 = the round-3 form): the tap's 4 frame-map reads issued together (each was a
// branch with its own lgkmcnt(0) wait, run by all 8 waves at once right after the barrier with the matrix pipe idle),
// both half-steps' fragments read before the first MFMA, and the next DMA + tap math issued between the two groups of
// 16 MFMAs, so that address work runs beside the matrix pipe.
template <bool V2>
__global__ __launch_bounds__(PNT, 1) void conv3d_pipe_kernel(const vp_conv3d_desc d) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tmapl = (int*)(smem + PSLOTS * P_STAGE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  constexpr int FM = 4, FN = 4, WM = 64, WN = 64;

  const int HWo = d.Hout * d.Wout;
  const int64_t THWo = (int64_t)d.Tout * HWo;
  const int64_t M = (int64_t)d.B * THWo;
  const int tiles_n = (d.Cout + PBN - 1) / PBN;
  const int tl = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = (tl % tiles_n) * PBN;
  const int64_t m0 = (int64_t)(tl / tiles_n) * PBM;

  const int nv = d.Tout + d.kt - 1;
  for (int v = tid; v < nv; v += PNT) tmapl[v] = d.tmap[v];

  const int C8 = d.Cin >> 3;
  const int khw = d.kh * d.kw;
  const int kc_total = d.kt * khw * C8;
  const int64_t Ktot = (int64_t)kc_total * 8;
  const int Hu = d.Hin * d.uh, Wu = d.Win * d.uw;
  const int ush = d.uh >> 1, usw = d.uw >> 1;
  const int64_t HWi = (int64_t)d.Hin * d.Win;
  int rb[P_AI], rt[P_AI], ry[P_AI], rx[P_AI];
  bool rv[P_AI];
#pragma unroll
  for (int i = 0; i < P_AI; ++i) {
    const int r = (i * 8 + wave) * 8 + (lane >> 3);
    const int64_t m = m0 + r;
    rv[i] = m < M;
    const int64_t mm = rv[i] ? m : 0;
    const int b = (int)(mm / THWo);
    const int rem = (int)(mm - (int64_t)b * THWo);
    const int t = rem / HWo;
    const int rem2 = rem - t * HWo;
    const int yo = rem2 / d.Wout;
    const int xo = rem2 - yo * d.Wout;
    rb[i] = b;
    rt[i] = t;
    ry[i] = yo * d.sh - d.ph;
    rx[i] = xo * d.sw - d.pw;
  }
  const bf16* X = (const bf16*)d.x;
  const bf16* Hs = (const bf16*)d.hist;
  const bf16* Wt = (const bf16*)d.w;
  const char* abase[P_AI];
  int amask[P_AI];
  const char* wbase[P_BI];
#pragma unroll
  for (int j = 0; j < P_BI; ++j) {
    const int r = (j * 8 + wave) * 8 + (lane >> 3);
    const int n = min(n0 + r, d.Cout - 1);
    wbase[j] = (const char*)(Wt + (int64_t)n * Ktot + (((lane & 7) ^ cswz(r)) << 3));
  }
  const int tpt = C8 >> 3;  // K-tiles per tap
  auto set_tap = [&](int tap) {
    const int dt = khw == 1 ? tap : tap / khw;
    const int rem = tap - dt * khw;
    const int dy = d.kw == 1 ? rem : rem / 3;
    const int dx = rem - dy * d.kw;
    int fm[P_AI];  // V2: the frame maps of the 4 rows read together (rt + dt <= Tout + kt - 2 for every row)
    if constexpr (V2) {
#pragma unroll
      for (int i = 0; i < P_AI; ++i) fm[i] = tmapl[rt[i] + dt];
    }
#pragma unroll
    for (int i = 0; i < P_AI; ++i) {
      const int r = (i * 8 + wave) * 8 + (lane >> 3);
      const int yu = ry[i] + dy, xu = rx[i] + dx;
      const bf16* p = nullptr;
      if (rv[i] && yu >= 0 && yu < Hu && xu >= 0 && xu < Wu) {
        const int f = V2 ? fm[i] : tmapl[rt[i] + dt];
        const int64_t pix = (f >= 0 ? (int64_t)rb[i] * d.x_frames + f : (int64_t)rb[i] * d.hist_frames + (-1 - f)) *
                                HWi + (int64_t)(yu >> ush) * d.Win + (xu >> usw);
        p = (f >= 0 ? X : Hs) + pix * d.Cin;
      }
      amask[i] = p != nullptr ? -1 : 0;
      abase[i] = p != nullptr ? (const char*)(p + (((lane & 7) ^ cswz(r)) << 3)) : (const char*)g_zero16;
    }
  };
  auto stage = [&](int kt, char* buf) {
    if ((kt & (tpt - 1)) == 0) set_tap(kt / tpt);
    const int cb = (kt & (tpt - 1)) * 128;
#pragma unroll
    for (int i = 0; i < P_AI; ++i) glds16_asm(abase[i] + (cb & amask[i]), buf + (i * 8 + wave) * 1024);
#pragma unroll
    for (int j = 0; j < P_BI; ++j) glds16_asm(wbase[j] + (int64_t)kt * 128, buf + P_A + (j * 8 + wave) * 1024);
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // tmap in LDS
  const int nk = kc_total / 8;  // Cin >= 64: whole 64-channel K-tiles
  stage(0, smem);
  if (nk > 1) stage(1, smem + P_STAGE);
  const int lrow = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* cur = smem + (kt % PSLOTS) * P_STAGE;
    if constexpr (V2) {
      bf16x8 af[2][FM], wf[2][FN];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = ks * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wr * WM + i * 16 + lrow;
          af[ks][i] = *(const bf16x8*)(cur + row * 128 + ((ch ^ cswz(row)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wc * WN + j * 16 + lrow;
          wf[ks][j] = *(const bf16x8*)(cur + P_A + row * 128 + ((ch ^ cswz(row)) << 4));
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][j], af[ks][i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (ks == 0) {  // the next DMA (and, on a tap change, its gather addresses) beside the first 16 MFMAs
          __builtin_amdgcn_sched_barrier(0);
          if (kt + 2 < nk) stage(kt + 2, smem + ((kt + 2) % PSLOTS) * P_STAGE);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      continue;
    }
    if (kt + 2 < nk) stage(kt + 2, smem + ((kt + 2) % PSLOTS) * P_STAGE);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[FM], wf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wr * WM + i * 16 + lrow;
        af[i] = *(const bf16x8*)(cur + row * 128 + ((ch ^ cswz(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wc * WN + j * 16 + lrow;
        wf[j] = *(const bf16x8*)(cur + P_A + row * 128 + ((ch ^ cswz(row)) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  const bf16* bias = (const bf16*)d.bias;
  const bf16* R = (const bf16*)d.resid;
  bf16* Y = (bf16*)d.y;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wc * WN + j * 16 + (lane >> 4) * 4;
    if (n >= d.ldy) continue;
    float bv[4];
    if (bias != nullptr && n + 3 < d.Cout) {  // one 8-byte load (per-element loads came out as serial round trips)
      const bf16x4 b4 = *(const bf16x4*)(bias + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bf2f(b4[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (bias != nullptr && n + r < d.Cout) ? bf2f(bias[n + r]) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int64_t m = m0 + wr * WM + i * 16 + lrow;
      if (m >= M) continue;
      bf16x4 rv4;
      if (R != nullptr && n < d.Cout) rv4 = *(const bf16x4*)(R + m * d.ldr + n);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = rbf(acc[j][i][r] + bv[r]);
        if (R != nullptr && n < d.Cout) v += bf2f(rv4[r]);
        o[r] = f2bf(n + r < d.Cout ? v : 0.f);
      }
      *(bf16x4*)(Y + m * d.ldy + n) = o;
    }
  }
}

// ---- GroupNorm ----
constexpr int GN_MAX_BLOCKS = 1024;

// per-block shifted sums of each group over a pixel range: partials[((b*G + g)*nblk + blk)*2 + {0,1}] =
// (sum(x - s_g), sum((x - s_g)^2)) with s_g = x[b, pixel 0, first channel of g] (the shift keeps the fp32 sums free of
// cancellation when |mean| >> std; the same shift in every block keeps the partials additive)
__global__ __launch_bounds__(256) void gn_partial_kernel(const bf16* __restrict__ x, int64_t P, int C, int G,
                                                         int nblk, float* __restrict__ partials) {
  __shared__ float red[2 * 2048];
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int C8 = C >> 3;
  const int rows = 256 / C8;
  const int chunk = tid % C8, prow = tid / C8;
  const int cg = C / G;
  const bf16* xb = x + (int64_t)b * P * C;
  float sh[8], s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = chunk * 8 + e;
    sh[e] = bf2f(xb[(c / cg) * cg]);
    s[e] = 0.f;
    q[e] = 0.f;
  }
  const int64_t p0 = P * blockIdx.x / nblk, p1 = P * (blockIdx.x + 1) / nblk;
  for (int64_t p = p0 + prow; p < p1; p += rows) {
    const bf16x8 v = *(const bf16x8*)(xb + p * C + chunk * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = bf2f(v[e]) - sh[e];
      s[e] += f;
      q[e] = __builtin_fmaf(f, f, q[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[prow * C + chunk * 8 + e] = s[e];
    red[2048 + prow * C + chunk * 8 + e] = q[e];
  }
  __syncthreads();
  // channel totals over the block's pixel rows, kept in row 0 of each half
  float cs[8], cq[8];
  const int nch = (C + 255) / 256;
  for (int k = 0; k < nch && k < 8; ++k) {
    const int c = tid + k * 256;
    cs[k] = 0.f;
    cq[k] = 0.f;
    if (c < C)
      for (int r = 0; r < rows; ++r) {
        cs[k] += red[r * C + c];
        cq[k] += red[2048 + r * C + c];
      }
  }
  __syncthreads();
  for (int k = 0; k < nch && k < 8; ++k) {
    const int c = tid + k * 256;
    if (c < C) {
      red[c] = cs[k];
      red[2048 + c] = cq[k];
    }
  }
  __syncthreads();
  for (int g = tid; g < G; g += 256) {
    float ss = 0.f, qq = 0.f;
    for (int c = g * cg; c < (g + 1) * cg; ++c) {
      ss += red[c];
      qq += red[2048 + c];
    }
    float* o = partials + (((int64_t)b * G + g) * nblk + blockIdx.x) * 2;
    o[0] = ss;
    o[1] = qq;
  }
}

__global__ __launch_bounds__(64) void gn_finalize_kernel(const float* __restrict__ partials, int nblk,
                                                         const bf16* __restrict__ x, int64_t P, int C, int G,
                                                         float eps, float* __restrict__ stats) {
  const int bg = blockIdx.x;
  const int b = bg / G, g = bg % G;
  const int lane = threadIdx.x;
  double s = 0.0, q = 0.0;
  for (int k = lane; k < nblk; k += 64) {
    s += (double)partials[((int64_t)bg * nblk + k) * 2];
    q += (double)partials[((int64_t)bg * nblk + k) * 2 + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if (lane == 0) {
    const int cg = C / G;
    const double n = (double)P * cg;
    const double ms = s / n;
    double var = q / n - ms * ms;
    if (var < 0.0) var = 0.0;
    const float shift = bf2f(x[(int64_t)b * P * C + g * cg]);
    stats[bg * 2] = (float)(shift + ms);
    stats[bg * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

struct GnApplyArgs {
  const bf16* x;
  bf16* y;
  const float* stats;
  const bf16* gamma;
  const bf16* beta;
  const bf16* mod;
  int B, T, H, W, C, G, Tz, Hz, Wz, silu;
  float shs, sws;  // torch nearest scale factors Hz / H, Wz / W (float)
  int tzmap[VP_CONV_MAX_T];
};

__global__ __launch_bounds__(256) void gn_apply_kernel(const GnApplyArgs a) {
  const int C8 = a.C >> 3;
  const int cg = a.C / a.G;
  const int64_t HW = (int64_t)a.H * a.W;
  const int64_t total = (int64_t)a.B * a.T * HW * C8;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int chunk = (int)(idx % C8);
    const int64_t pix = idx / C8;
    const int c0 = chunk * 8;
    const int b = (int)(pix / ((int64_t)a.T * HW));
    const bf16x8 xv = *(const bf16x8*)(a.x + pix * a.C + c0);
    const bf16x8 gv = *(const bf16x8*)(a.gamma + c0);
    const bf16x8 bv = *(const bf16x8*)(a.beta + c0);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int g = (c0 + e) / cg;
      const float mean = a.stats[(b * a.G + g) * 2], rstd = a.stats[(b * a.G + g) * 2 + 1];
      v[e] = __builtin_fmaf((bf2f(xv[e]) - mean) * rstd, bf2f(gv[e]), bf2f(bv[e]));
    }
    if (a.mod != nullptr) {
      const int64_t thw = pix - (int64_t)b * a.T * HW;
      const int t = (int)(thw / HW);
      const int hw = (int)(thw - (int64_t)t * HW);
      const int h = hw / a.W, w = hw - (hw / a.W) * a.W;
      const int zh = min((int)floorf((float)h * a.shs), a.Hz - 1);
      const int zw = min((int)floorf((float)w * a.sws), a.Wz - 1);
      const int64_t mp = (((int64_t)b * a.Tz + a.tzmap[t]) * a.Hz + zh) * a.Wz + zw;
      const bf16x8 my = *(const bf16x8*)(a.mod + mp * 2 * a.C + c0);
      const bf16x8 mb = *(const bf16x8*)(a.mod + mp * 2 * a.C + a.C + c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = __builtin_fmaf(v[e], bf2f(my[e]), bf2f(mb[e]));
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(a.silu ? v[e] * __builtin_amdgcn_rcpf(1.f + __expf(-v[e])) : v[e]);
    *(bf16x8*)(a.y + pix * a.C + c0) = o;
  }
}

__global__ __launch_bounds__(256) void time_pool2_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B,
                                                         int T, int T2, int64_t P, int C) {
  const int C8 = C >> 3;
  const int64_t per_frame = P * C8;
  const int64_t total = (int64_t)B * T2 * per_frame;
  const bool odd = (T & 1) != 0;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t within = idx % per_frame;
    const int64_t bt = idx / per_frame;
    const int t2 = (int)(bt % T2);
    const int b = (int)(bt / T2);
    const bf16* xb = x + (int64_t)b * T * P * C + within * 8;
    bf16x8 o;
    if (odd && t2 == 0) {
      o = *(const bf16x8*)xb;
    } else {
      const int ta = odd ? 2 * t2 - 1 : 2 * t2;
      const bf16x8 u = *(const bf16x8*)(xb + (int64_t)ta * P * C);
      const bf16x8 v = *(const bf16x8*)(xb + (int64_t)(ta + 1) * P * C);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf((bf2f(u[e]) + bf2f(v[e])) * 0.5f);
    }
    *(bf16x8*)(y + idx * 8) = o;
  }
}

__global__ __launch_bounds__(256) void ncdhw_to_ndhwc_kernel(const void* __restrict__ x, int is_f32,
                                                             bf16* __restrict__ y, int B, int C, int64_t THW,
                                                             int Cpad) {
  const int64_t total = (int64_t)B * THW;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int b = (int)(idx / THW);
    const int64_t p = idx - (int64_t)b * THW;
    for (int c0 = 0; c0 < Cpad; c0 += 8) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        float v = 0.f;
        if (c < C) {
          const int64_t src = ((int64_t)b * C + c) * THW + p;
          v = is_f32 ? ((const float*)x)[src] : bf2f(((const bf16*)x)[src]);
        }
        o[e] = f2bf(v);
      }
      *(bf16x8*)(y + idx * Cpad + c0) = o;
    }
  }
}

__global__ __launch_bounds__(256) void ndhwc_to_ncdhw_kernel(const bf16* __restrict__ x, int ldx,
                                                             bf16* __restrict__ y, int B, int C, int64_t THW,
                                                             int c0) {
  const int64_t total = (int64_t)B * C * THW;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t p = idx % THW;
    const int64_t bc = idx / THW;
    const int c = (int)(bc % C);
    const int b = (int)(bc / C);
    y[idx] = x[((int64_t)b * THW + p) * ldx + c0 + c];
  }
}

__global__ __launch_bounds__(256) void latent_dist_kernel(const bf16* __restrict__ prm, int ldp,
                                                          bf16* __restrict__ mean, bf16* __restrict__ logvar,
                                                          const bf16* __restrict__ noise, bf16* __restrict__ sample,
                                                          int B, int L, int64_t THW) {
  const int64_t total = (int64_t)B * L * THW;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t p = idx % THW;
    const int64_t bl = idx / THW;
    const int l = (int)(bl % L);
    const int b = (int)(bl / L);
    const bf16* row = prm + ((int64_t)b * THW + p) * ldp;
    const float mu = bf2f(row[l]);
    const float lv = fminf(fmaxf(bf2f(row[L + l]), -30.f), 20.f);
    mean[idx] = f2bf(mu);
    logvar[idx] = f2bf(lv);
    if (noise != nullptr) sample[idx] = f2bf(__builtin_fmaf(__expf(0.5f * lv), bf2f(noise[idx]), mu));
  }
}


__global__ __launch_bounds__(256) void tile_blend_kernel(const bf16* __restrict__ a, bf16* __restrict__ b, int BT,
                                                         int Ha, int Wa, int Hb, int Wb, int C, int axis, int e) {
  // one 16-byte chunk of b's first e rows (axis 0) / columns (axis 1) per thread
  const int C8 = C >> 3;
  const int64_t inner = axis == 0 ? (int64_t)Wb * C8 : (int64_t)C8;
  const int64_t per_bt = axis == 0 ? (int64_t)e * inner : (int64_t)Hb * e * C8;
  const int64_t total = (int64_t)BT * per_bt;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int bt = (int)(idx / per_bt);
    int64_t r = idx - (int64_t)bt * per_bt;
    int y, x, c8, k;
    if (axis == 0) {
      y = (int)(r / inner);
      r -= (int64_t)y * inner;
      x = (int)(r / C8);
      c8 = (int)(r - (int64_t)x * C8);
      k = y;
    } else {
      y = (int)(r / ((int64_t)e * C8));
      r -= (int64_t)y * e * C8;
      x = (int)(r / C8);
      c8 = (int)(r - (int64_t)x * C8);
      k = x;
    }
    const int ya = axis == 0 ? Ha - e + y : y;
    const int xa = axis == 0 ? x : Wa - e + x;
    const float wb = (float)k / (float)e, wa = 1.f - wb;
    bf16* pb = b + (((int64_t)bt * Hb + y) * Wb + x) * C + c8 * 8;
    const bf16x8 va = *(const bf16x8*)(a + (((int64_t)bt * Ha + ya) * Wa + xa) * C + c8 * 8);
    const bf16x8 vb = *(const bf16x8*)pb;
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(__builtin_fmaf(bf2f(va[q]), wa, bf2f(vb[q]) * wb));
    *(bf16x8*)pb = o;
  }
}

int grid_for(int64_t work, int per_block = 256) {
  const int64_t g = (work + per_block - 1) / per_block;
  return (int)(g < 1 ? 1 : (g > (1 << 20) ? (1 << 20) : g));
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int BN>
int launch_conv(const vp_conv3d_desc& d, int c8s, int64_t tiles, hipStream_t s) {
  using G = ConvGeom<BN>;
  static bool attr = false;  // > 64 KB of dynamic LDS needs the opt-in (once per instance)
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3d_kernel<BN, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              G::LDS);
    (void)hipFuncSetAttribute((const void*)conv3d_kernel<BN, true>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    attr = true;
  }
  // VP_CONV_HOIST=0 keeps the per-K-tile tap decode (A/B)
  const char* he = vp_knob(VPK_CONV_HOIST);
  if (d.Cin >= 64 && (he == nullptr || atoi(he) != 0))
    hipLaunchKernelGGL((conv3d_kernel<BN, true>), dim3((unsigned)tiles), dim3(CNT), G::LDS, s, d, c8s);
  else
    hipLaunchKernelGGL((conv3d_kernel<BN, false>), dim3((unsigned)tiles), dim3(CNT), G::LDS, s, d, c8s);
  VP_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int vp_conv3d_bf16(const vp_conv3d_desc* d, void* stream) {
  if (d == nullptr || d->x == nullptr || d->w == nullptr || d->y == nullptr) return VP_ERR_ARG;
  if (d->B <= 0 || d->Cin <= 0 || d->Cout <= 0 || d->Tout <= 0 || d->Hout <= 0 || d->Wout <= 0 || d->Hin <= 0 ||
      d->Win <= 0)
    return VP_ERR_ARG;
  if (d->Cin < 8 || d->Cin > 4096 || (d->Cin & (d->Cin - 1)) != 0) return VP_ERR_UNSUPPORTED;
  if (!((d->kt == 1 || d->kt == 3) && ((d->kh == 1 && d->kw == 1) || (d->kh == 3 && d->kw == 3))))
    return VP_ERR_UNSUPPORTED;
  if ((d->sh != 1 && d->sh != 2) || (d->sw != 1 && d->sw != 2) || (d->uh != 1 && d->uh != 2) ||
      (d->uw != 1 && d->uw != 2))
    return VP_ERR_UNSUPPORTED;
  if (d->ldy < d->Cout || (d->ldy % 8) != 0) return VP_ERR_ARG;
  if (d->resid != nullptr && (d->ldr < d->Cout || (d->ldr % 4) != 0)) return VP_ERR_ARG;
  if (!aligned16(d->x) || !aligned16(d->w) || (d->hist != nullptr && !aligned16(d->hist)) || !aligned16(d->y))
    return VP_ERR_ARG;
  const int nv = d->Tout + d->kt - 1;
  if (nv > VP_CONV_MAX_T) return VP_ERR_UNSUPPORTED;
  for (int v = 0; v < nv; ++v) {
    const int f = d->tmap[v];
    if (f >= 0 ? f >= d->x_frames : (d->hist == nullptr || -1 - f >= d->hist_frames)) return VP_ERR_ARG;
  }
  int c8s = 0;
  while ((8 << c8s) < d->Cin) ++c8s;
  const int64_t M = (int64_t)d->B * d->Tout * d->Hout * d->Wout;
  const int64_t tiles_m = (M + CBM - 1) / CBM;
  hipStream_t s = (hipStream_t)stream;
  if (d->Cout <= 32) {
    const int64_t t = tiles_m * ((d->Cout + 31) / 32);
    if (t >= (1ll << 31)) return VP_ERR_UNSUPPORTED;
    return launch_conv<32>(*d, c8s, t, s);
  }
  if (d->Cout <= 64) {
    const int64_t t = tiles_m * ((d->Cout + 63) / 64);
    if (t >= (1ll << 31)) return VP_ERR_UNSUPPORTED;
    return launch_conv<64>(*d, c8s, t, s);
  }
  // wide convolutions (Cin >= 64): the counted-vmcnt pipeline (VP_CONV_PIPE: 2 = V2, default; 1 = its round-3 form;
  // 0 = the 2-stage ring; A/B)
  const char* pe = vp_knob(VPK_CONV_PIPE);
  const int pipe = pe != nullptr ? atoi(pe) : 2;
  if (d->Cin >= 64 && pipe != 0) {
    const int64_t t = ((M + PBM - 1) / PBM) * ((d->Cout + PBN - 1) / PBN);
    if (t >= (1ll << 31)) return VP_ERR_UNSUPPORTED;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)conv3d_pipe_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                P_LDS);
      (void)hipFuncSetAttribute((const void*)conv3d_pipe_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                P_LDS);
      attr = true;
    }
    if (pipe == 1)
      hipLaunchKernelGGL(conv3d_pipe_kernel<false>, dim3((unsigned)t), dim3(PNT), P_LDS, s, *d);
    else
      hipLaunchKernelGGL(conv3d_pipe_kernel<true>, dim3((unsigned)t), dim3(PNT), P_LDS, s, *d);
    VP_CHECK_LAUNCH();
    return VP_OK;
  }
  const int64_t t = tiles_m * ((d->Cout + 127) / 128);
  if (t >= (1ll << 31)) return VP_ERR_UNSUPPORTED;
  return launch_conv<128>(*d, c8s, t, s);
}

extern "C" int64_t vp_group_norm_workspace_floats(int32_t B, int32_t G) {
  return (int64_t)B * G * GN_MAX_BLOCKS * 2;
}

extern "C" int vp_group_norm_stats(const void* x, int32_t B, int64_t P, int32_t C, int32_t G, float eps,
                                   float* partials, float* stats, void* stream) {
  if (x == nullptr || partials == nullptr || stats == nullptr || B <= 0 || P <= 0 || C <= 0 || G <= 0)
    return VP_ERR_ARG;
  if ((C % 8) != 0 || C > 2048 || (C % G) != 0 || ((C / 8) & (C / 8 - 1)) != 0 || !aligned16(x))
    return VP_ERR_UNSUPPORTED;
  const int rows = 256 / (C / 8);
  int64_t nb = (P + rows * 16 - 1) / (rows * 16);  // >= 16 pixel rows per thread
  const int nblk = (int)(nb < 1 ? 1 : (nb > GN_MAX_BLOCKS ? GN_MAX_BLOCKS : nb));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_partial_kernel, dim3(nblk, B), dim3(256), 0, s, (const bf16*)x, P, C, G, nblk, partials);
  VP_CHECK_LAUNCH();
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(B * G), dim3(64), 0, s, (const float*)partials, nblk, (const bf16*)x,
                     P, C, G, eps, stats);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_group_norm_apply_bf16(const void* x, void* y, int32_t B, int32_t T, int32_t H, int32_t W, int32_t C,
                                        int32_t G, const float* stats, const void* gamma, const void* beta,
                                        const void* mod, int32_t Tz, int32_t Hz, int32_t Wz,
                                        const int32_t* tzmap_host, int32_t silu, void* stream) {
  if (x == nullptr || y == nullptr || stats == nullptr || gamma == nullptr || beta == nullptr) return VP_ERR_ARG;
  if (B <= 0 || T <= 0 || H <= 0 || W <= 0 || C <= 0 || G <= 0 || (C % 8) != 0 || (C % G) != 0) return VP_ERR_ARG;
  if (!aligned16(x) || !aligned16(y) || !aligned16(gamma) || !aligned16(beta)) return VP_ERR_ARG;
  GnApplyArgs a;
  a.x = (const bf16*)x;
  a.y = (bf16*)y;
  a.stats = stats;
  a.gamma = (const bf16*)gamma;
  a.beta = (const bf16*)beta;
  a.mod = (const bf16*)mod;
  a.B = B, a.T = T, a.H = H, a.W = W, a.C = C, a.G = G, a.silu = silu ? 1 : 0;
  a.Tz = Tz, a.Hz = Hz, a.Wz = Wz;
  a.shs = 0.f, a.sws = 0.f;
  for (int i = 0; i < VP_CONV_MAX_T; ++i) a.tzmap[i] = 0;
  if (mod != nullptr) {
    if (tzmap_host == nullptr || Tz <= 0 || Hz <= 0 || Wz <= 0 || T > VP_CONV_MAX_T || !aligned16(mod))
      return VP_ERR_ARG;
    for (int t = 0; t < T; ++t) {
      if (tzmap_host[t] < 0 || tzmap_host[t] >= Tz) return VP_ERR_ARG;
      a.tzmap[t] = tzmap_host[t];
    }
    a.shs = (float)Hz / (float)H;
    a.sws = (float)Wz / (float)W;
  }
  const int64_t work = (int64_t)B * T * H * W * (C / 8);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, a);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_time_pool2_bf16(const void* x, void* y, int32_t B, int32_t T, int64_t P, int32_t C, void* stream) {
  if (x == nullptr || y == nullptr || B <= 0 || T <= 0 || P <= 0 || C <= 0 || (C % 8) != 0) return VP_ERR_ARG;
  if (!aligned16(x) || !aligned16(y)) return VP_ERR_ARG;
  const int T2 = (T & 1) ? (T + 1) / 2 : T / 2;
  const int64_t work = (int64_t)B * T2 * P * (C / 8);
  hipLaunchKernelGGL(time_pool2_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (bf16*)y, B, T, T2, P, C);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_ncdhw_to_ndhwc_bf16(const void* x, int32_t x_is_f32, void* y, int32_t B, int32_t C, int32_t T,
                                      int32_t H, int32_t W, int32_t Cpad, void* stream) {
  if (x == nullptr || y == nullptr || B <= 0 || C <= 0 || T <= 0 || H <= 0 || W <= 0) return VP_ERR_ARG;
  if (Cpad < C || (Cpad % 8) != 0 || !aligned16(y)) return VP_ERR_ARG;
  const int64_t THW = (int64_t)T * H * W;
  hipLaunchKernelGGL(ncdhw_to_ndhwc_kernel, dim3(grid_for((int64_t)B * THW)), dim3(256), 0, (hipStream_t)stream, x,
                     x_is_f32 ? 1 : 0, (bf16*)y, B, C, THW, Cpad);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_ndhwc_to_ncdhw_bf16(const void* x, int32_t ldx, void* y, int32_t B, int32_t C, int32_t T,
                                      int32_t H, int32_t W, int32_t c0, void* stream) {
  if (x == nullptr || y == nullptr || B <= 0 || C <= 0 || T <= 0 || H <= 0 || W <= 0 || c0 < 0 || c0 + C > ldx)
    return VP_ERR_ARG;
  const int64_t THW = (int64_t)T * H * W;
  hipLaunchKernelGGL(ndhwc_to_ncdhw_kernel, dim3(grid_for((int64_t)B * C * THW)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, (bf16*)y, B, C, THW, c0);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_latent_dist_bf16(const void* params, int32_t ldp, void* mean, void* logvar, const void* noise,
                                   void* sample, int32_t B, int32_t L, int32_t T, int32_t H, int32_t W, void* stream) {
  if (params == nullptr || mean == nullptr || logvar == nullptr || B <= 0 || L <= 0 || T <= 0 || H <= 0 || W <= 0)
    return VP_ERR_ARG;
  if (ldp < 2 * L || (noise != nullptr && sample == nullptr)) return VP_ERR_ARG;
  const int64_t THW = (int64_t)T * H * W;
  hipLaunchKernelGGL(latent_dist_kernel, dim3(grid_for((int64_t)B * L * THW)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)params, ldp, (bf16*)mean, (bf16*)logvar, (const bf16*)noise, (bf16*)sample, B, L,
                     THW);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_tile_blend_bf16(const void* a, void* b, int32_t B, int32_t T, int32_t Ha, int32_t Wa, int32_t Hb,
                                  int32_t Wb, int32_t C, int32_t axis, int32_t extent, void* stream) {
  if (a == nullptr || b == nullptr || B <= 0 || T <= 0 || Ha <= 0 || Wa <= 0 || Hb <= 0 || Wb <= 0 || C <= 0 ||
      (C % 8) != 0 || (axis != 0 && axis != 1))
    return VP_ERR_ARG;
  if ((axis == 0 && Wa != Wb) || (axis == 1 && Ha != Hb) || !aligned16(a) || !aligned16(b)) return VP_ERR_ARG;
  const int e = axis == 0 ? min(min(Ha, Hb), extent) : min(min(Wa, Wb), extent);
  if (e <= 0) return 0;
  const int64_t work = (int64_t)B * T * (axis == 0 ? (int64_t)e * Wb : (int64_t)Hb * e) * (C / 8);
  hipLaunchKernelGGL(tile_blend_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, (const bf16*)a,
                     (bf16*)b, B * T, Ha, Wa, Hb, Wb, C, axis, e);
  VP_CHECK_LAUNCH();
  return 0;
}
