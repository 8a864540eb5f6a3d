// bf16 MFMA GEMM with fused epilogues for every projection on the CogVideoX block path (gfx950 / MI355X).
//
//   C[m, n] = epilogue( Σ_k A[m, k] · W[n, k] )          A: activations [M, K], W: nn.Linear weight [N, K]
//
// Both operands are K-contiguous, so both MFMA fragments are 16-byte row reads.  The MFMA is issued with W as the
// A-operand and the activation as the B-operand, so each lane's accumulator holds 4 *consecutive output columns*
// of one output row (C/D map of v_mfma_f32_16x16x32_bf16: col = lane&15 -> m, row = 4*(lane>>4)+r -> n); the
// epilogue packs them into 8-byte LDS writes and streams the tile out as full 16-byte rows.
//
// Tile 256x256x64, 512 threads (8 waves = 2 (M) x 4 (N), 128x64 per wave, 8x4 16x16 fragments), 2-stage LDS ring
// filled by global_load_lds_dwordx4 (LDS-DMA, lane-linear destination; the bank swizzle is applied on the SOURCE
// address and undone on the read, cdna_hip_programming.md §5.4 rule 21), XCD-aware grouped tile order.
// Roofline: MFMA-bound (AI = 2*256*256*64 flop / 64 KB staged per k-step).
#include <stdlib.h>

#include "vp_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int WM = 128, WN = 64;
constexpr int FM = WM / 16, FN = WN / 16;
constexpr int TILE_BYTES = BM * BK * 2;       // 32 KB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;   // A + B
constexpr int CT_STRIDE = BN * 2 + 8;         // bytes per C row in the epilogue LDS image (bank-conflict pad)
constexpr int LDS_BYTES = (2 * STAGE_BYTES > BM * CT_STRIDE) ? 2 * STAGE_BYTES : BM * CT_STRIDE;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void g_void;

VP_DEV int swz(int row) { return (row >> 1) & 7; }

__device__ __attribute__((aligned(16))) bf16 g_zero_chunk[8];  // 16 zero bytes: source of the K tail

// Tile rows each lane stages (4 LDS-DMA wave-instructions per operand per k-step): instruction i, lane l ->
// tile row r = (i*8 + wave)*8 + l/8, physical 16-byte chunk p = l%8, logical chunk c = p ^ swz(r).
VP_DEV int stage_row(int i, int wave, int lane) { return (i * 8 + wave) * 8 + (lane >> 3); }

// Stage one 256x64 bf16 operand tile into `tile` as [256][8 chunks of 16 B], physical chunk = logical ^ swz(row).
// rows[i] = this lane's source row pointer for instruction i (clamped to a valid row, hoisted out of the k-loop);
// chunks past K read a zero chunk.
VP_DEV void stage_tile(const bf16* const (&rows)[4], int K, int k0, char* tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rb = i * 8 + wave;
    const int r = stage_row(i, wave, lane);
    const int c = (lane & 7) ^ swz(r);
    const int kc = k0 + c * 8;
    const bf16* src = kc < K ? rows[i] + kc : g_zero_chunk;
    __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(tile + rb * 1024), 16, 0, 0);
  }
}

VP_DEV bf16x8 lds_frag(const char* tile, int row, int chunk) {
  return *(const bf16x8*)(tile + row * 128 + ((chunk ^ swz(row)) << 4));
}

// ---- variant 2 main-loop pieces: BK = 32 half-steps, 4-slot LDS ring (128 KB), 3 half-steps of LDS-DMA in flight
// across raw barriers (counted vmcnt, never 0 in the loop: cdna_hip_programming.md §5 "Pipelining across barriers").
constexpr int HK = 32;                      // k per half-step
constexpr int HTILE = BM * HK * 2;          // 16 KB per operand half-tile
constexpr int HSLOT = 2 * HTILE;            // A + B
VP_DEV int swz64(int row) { return ((row >> 2) & 1) << 1; }  // conflict-free ds_read_b128 on 64-byte rows

VP_DEV void stage_half(const bf16* const (&rows)[2], int K, int k0, char* tile, int wave, int lane) {
  // wave-instruction i covers 16 rows x 64 B: lane l -> row (i*8 + wave)*16 + l/4, physical chunk l%4
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rb = i * 8 + wave;
    const int r = rb * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz64(r);
    const int kc = k0 + c * 8;
    const bf16* src = kc < K ? rows[i] + kc : g_zero_chunk;
    __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)(tile + rb * 1024), 16, 0, 0);
  }
}

VP_DEV bf16x8 lds_frag64(const char* tile, int row, int chunk) {
  return *(const bf16x8*)(tile + row * 64 + ((chunk ^ swz64(row)) << 4));
}

template <int VAR>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_bf16_kernel(const vp_gemm_desc d) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2;  // 0..1  (M)
  const int wc = wave & 3;   // 0..3  (N)

  const int tiles_m = (d.M + BM - 1) / BM;
  const int tiles_n = (d.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int group_id = t / per_group;
  const int first_m = group_id * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + ((t % per_group) % gsz);
  const int tn = (t % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // per-lane source rows of the two operand tiles (the weight rows may come from up to 3 segments: fused QKV)
  const bf16* arow[4];
  const bf16* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = stage_row(i, wave, lane);
    const int m = min(m0 + r, d.M - 1);
    arow[i] = (const bf16*)d.A + (int64_t)m * d.lda;
    const int n = min(n0 + r, d.N - 1);
    const int sg = n / d.n_seg;
    wrow[i] = (const bf16*)d.W[sg] + (int64_t)(n - sg * d.n_seg) * d.K;
  }

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if constexpr (VAR == 1) {
    const int nk = (d.K + BK - 1) / BK;
    stage_tile(arow, d.K, 0, smem, wave, lane);
    stage_tile(wrow, d.K, 0, smem + TILE_BYTES, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
      char* cur = smem + (kt & 1) * STAGE_BYTES;
      if (kt + 1 < nk) {
        char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
        stage_tile(arow, d.K, (kt + 1) * BK, nxt, wave, lane);
        stage_tile(wrow, d.K, (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
      }
      const char* As = cur;
      const char* Bs = cur + TILE_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[FM], wf[FN];
        const int ch = ks * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = lds_frag(As, wr * WM + i * 16 + (lane & 15), ch);
#pragma unroll
        for (int j = 0; j < FN; ++j) wf[j] = lds_frag(Bs, wc * WN + j * 16 + (lane & 15), ch);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // per-lane half-tile source rows (2 LDS-DMA instructions per operand per half-step)
    const bf16* ah[2];
    const bf16* wh[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (i * 8 + wave) * 16 + (lane >> 2);
      ah[i] = (const bf16*)d.A + (int64_t)min(m0 + r, d.M - 1) * d.lda;
      const int n = min(n0 + r, d.N - 1);
      const int sg = n / d.n_seg;
      wh[i] = (const bf16*)d.W[sg] + (int64_t)(n - sg * d.n_seg) * d.K;
    }
    const int nh = (d.K + HK - 1) / HK;
    auto issue = [&](int t) {
      char* slot = smem + (t & 3) * HSLOT;
      stage_half(ah, d.K, t * HK, slot, wave, lane);
      stage_half(wh, d.K, t * HK, slot + HTILE, wave, lane);
    };
    issue(0);
    if (nh > 1) issue(1);
    if (nh > 2) issue(2);
    for (int t = 0; t < nh; ++t) {
      // retire half-step t (4 LDS-DMA per half-step per lane); keep the later ones in flight
      if (t + 2 < nh) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (t + 1 < nh) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + 3 < nh) issue(t + 3);
      const char* As = smem + (t & 3) * HSLOT;
      const char* Bs = As + HTILE;
      bf16x8 af[FM], wf[FN];
      const int ch = lane >> 4;
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = lds_frag64(As, wr * WM + i * 16 + (lane & 15), ch);
#pragma unroll
      for (int j = 0; j < FN; ++j) wf[j] = lds_frag64(Bs, wc * WN + j * 16 + (lane & 15), ch);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();  // all waves done with the ring before the epilogue reuses the LDS
  }

  // ---- epilogue phase 1: per-fragment bias / activation, bf16 into the LDS C image ----
  const int epi = d.epilogue;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nloc = wc * WN + j * 16 + (lane >> 4) * 4;  // 4 consecutive columns
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + nloc + r;
      if (n < d.N) {
        const int sg = n / d.n_seg;
        const bf16* bp = (const bf16*)d.bias[sg];
        if (bp != nullptr) bv[r] = bf2f(bp[n - sg * d.n_seg]);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int mloc = wr * WM + i * 16 + (lane & 15);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = rbf(acc[j][i][r] + bv[r]);
        if (epi == VP_EPI_BIAS_GELU) v = gelu_tanh(v);
        else if (epi == VP_EPI_BIAS_SCALE) v = v * d.alpha;
        o[r] = f2bf(v);
      }
      *(bf16x4*)(smem + mloc * CT_STRIDE + nloc * 2) = o;
    }
  }
  __syncthreads();

  // ---- epilogue phase 2: coalesced 16-byte row stores (+ residual / gate / injection / pos-emb) ----
  bf16* C = (bf16*)d.C;
  const int chunk = tid & 31;         // 16-byte chunk within the 512-byte tile row
  const int ncol = n0 + chunk * 8;
#pragma unroll 1
  for (int it = 0; it < BM / 16; ++it) {
    const int mloc = it * 16 + (tid >> 5);
    const int m = m0 + mloc;
    if (m >= d.M || ncol >= d.N) continue;
    bf16x8 v = *(const bf16x8*)(smem + mloc * CT_STRIDE + chunk * 16);
    const int64_t orow = (int64_t)(m / d.rows_per_group) * d.group_stride + d.row_offset + (m % d.rows_per_group);
    if (epi == VP_EPI_GATED) {
      const int b = m / d.tokens_per_batch;
      const int tok = m - b * d.tokens_per_batch;
      const bf16* g = (const bf16*)(tok < d.text_len ? d.gate_text : d.gate) + (int64_t)b * d.gate_bstride + ncol;
      const bf16x8 gv = *(const bf16x8*)g;
      const bf16x8 rv = *(const bf16x8*)((const bf16*)d.R + orow * d.ldr + ncol);
      bool inj = false;
      bf16x8 iv;
      if (d.inject != nullptr && tok >= d.text_len) {
        const int vtok = tok - d.text_len;
        inj = (d.inject_mask == nullptr) || (d.inject_mask[(int64_t)b * d.inject_mask_bstride + vtok] == 0);
        if (inj) iv = *(const bf16x8*)((const bf16*)d.inject + (int64_t)b * d.inject_bstride +
                                       (int64_t)vtok * d.inject_ld + ncol);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o = rbf(bf2f(rv[e]) + rbf(bf2f(gv[e]) * bf2f(v[e])));
        if (inj) o = rbf(o + bf2f(iv[e]));
        v[e] = f2bf(o);
      }
    } else if (epi == VP_EPI_BIAS_ADDROWS) {
      const bf16x8 pv = *(const bf16x8*)((const bf16*)d.addrows +
                                         (int64_t)((m % d.rows_per_group) + d.addrows_offset) * d.addrows_ld + ncol);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(pv[e]));
    }
    *(bf16x8*)(C + orow * d.ldc + ncol) = v;
  }
}

}  // namespace

extern "C" int vp_gemm_bf16(const vp_gemm_desc* d, void* stream) {
  if (d == nullptr || d->A == nullptr || d->W[0] == nullptr || d->C == nullptr) return VP_ERR_ARG;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || (d->K % 8) != 0 || (d->N % 8) != 0) return VP_ERR_ARG;
  if (d->lda < d->K || d->ldc < d->N || (d->lda % 8) != 0 || (d->ldc % 8) != 0) return VP_ERR_ARG;
  if (d->rows_per_group <= 0) return VP_ERR_ARG;
  const int nsegs = d->W[2] ? 3 : (d->W[1] ? 2 : 1);
  if (d->n_seg <= 0 || d->n_seg * nsegs != d->N) return VP_ERR_ARG;
  if (d->epilogue < VP_EPI_BIAS || d->epilogue > VP_EPI_BIAS_ADDROWS) return VP_ERR_ARG;
  if (d->epilogue == VP_EPI_GATED) {
    if (d->R == nullptr || d->gate == nullptr || d->gate_text == nullptr || d->tokens_per_batch <= 0) return VP_ERR_ARG;
    if ((d->ldr % 8) != 0 || (d->gate_bstride % 8) != 0) return VP_ERR_ARG;
    if (d->inject != nullptr && ((d->inject_ld % 8) != 0 || (d->inject_bstride % 8) != 0)) return VP_ERR_ARG;
  }
  if (d->epilogue == VP_EPI_BIAS_ADDROWS && (d->addrows == nullptr || (d->addrows_ld % 8) != 0)) return VP_ERR_ARG;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    attr_set = true;
  }
  const char* e = getenv("VP_GEMM_VARIANT");  // A/B switch for benchmarking main-loop variants
  const int variant = (e != nullptr && e[0] == '2') ? 2 : 1;
  const int tiles = ((d->M + BM - 1) / BM) * ((d->N + BN - 1) / BN);
  if (variant == 2)
    hipLaunchKernelGGL(gemm_bf16_kernel<2>, dim3(tiles), dim3(NTHREADS), LDS_BYTES, (hipStream_t)stream, *d);
  else
    hipLaunchKernelGGL(gemm_bf16_kernel<1>, dim3(tiles), dim3(NTHREADS), LDS_BYTES, (hipStream_t)stream, *d);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
