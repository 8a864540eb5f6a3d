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
#include <string.h>

#include <type_traits>

#include "vp_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int WM = 128, WN = 64;
constexpr int FM = WM / 16, FN = WN / 16;
constexpr int TILE_BYTES = BM * BK * 2;       // 32 KB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;   // A + B
constexpr int CT_STRIDE = BN * 2 + 8;         // bytes per C row in the epilogue LDS image (bank-conflict pad)
// the gated epilogue's per-row injection flags (one byte per tile row) sit past the C image
constexpr int EPI_FLAG_OFF = BM * CT_STRIDE;
constexpr int LDS_BYTES = (2 * STAGE_BYTES > EPI_FLAG_OFF + BM) ? 2 * STAGE_BYTES : EPI_FLAG_OFF + BM;

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

// LDS-DMA of 16 bytes per lane with saddr + 32-bit voffset addressing: global [sbase + voff] -> LDS [m0 + 16*lane]
// (inline asm: the builtin form makes the compiler keep a 64-bit address per lane and instruction)
VP_DEV void glds16(const char* sbase, int voff, char* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void*)lds;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(la), "v"(voff), "s"(sbase)
               : "memory", "m0");
}

VP_DEV bf16x8 lds_frag(const char* tile, int row, int chunk) {
  return *(const bf16x8*)(tile + row * 128 + ((chunk ^ swz(row)) << 4));
}

// MX-FP8 extension of the descriptor (zero for the bf16 path)
struct MxExt {
  const uint8_t* a_scale;
  const uint8_t* w_scale[3];
  uint8_t* c_scale;
  // split-K (vp_gemm_bf16_ws): workgroup = (tile, K-chunk); fp32 partial tiles [nsplit][M][N] in ws, or (tail mode:
  // the last partial round of a large GEMM) tiles t_base.. with compact partials [tile - t_base][nsplit][BM][BN]
  float* ws;
  int kchunk, nsplit;
  int t_base, tail;
  int group;  // M-tiles per tile group of the grouped order (0: the kernel's GROUP)
};

// scale ring of the fp8 path: 4 K-tiles x (A, W) x 1 KiB after the two operand stages (the ring slot of tile t is
// refilled 3 tiles after its last read, so the LDS-DMA never races a reader)
constexpr int SCALE_OFF = 2 * STAGE_BYTES;
constexpr int LDS_BYTES_FP8 = (SCALE_OFF + 8 * 1024 > LDS_BYTES) ? SCALE_OFF + 8 * 1024 : LDS_BYTES;

typedef int i32x8 __attribute__((ext_vector_type(8)));



// One block-scaled e4m3 MFMA, D = C in place.  Inline asm because the builtin form makes hipcc (ROCm 7.2) allocate
// a fresh destination tuple per accumulator (dst != srcC), which does not fit the 256-VGPR budget of this tile and
// spills.  The scale of the first operand (W) is byte BW of sw, of the second (A) byte BA of sa (op_sel /
// op_sel_hi = low / high bit of the byte index).  Hazards the compiler does not see inside asm: the operands come
// from ds_read (the compiler's lgkmcnt waits cover asm inputs), the same accumulator is reused only >= 8 MFMAs
// later, and the kernel pads with s_nop before the epilogue reads the accumulators.
template <int BW, int BA>
VP_DEV void mfma_mx(f32x4& acc, const i32x8& w, const i32x8& a, int sw, int sa) {
  if constexpr (BW == 0 && BA == 0)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[0,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 0 && BA == 1)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,1,0] op_sel_hi:[0,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 0 && BA == 2)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[0,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 0 && BA == 3)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,1,0] op_sel_hi:[0,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 1 && BA == 0)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,0,0] op_sel_hi:[0,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 1 && BA == 1)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,1,0] op_sel_hi:[0,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 1 && BA == 2)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,0,0] op_sel_hi:[0,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 1 && BA == 3)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,1,0] op_sel_hi:[0,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 2 && BA == 0)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[1,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 2 && BA == 1)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,1,0] op_sel_hi:[1,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 2 && BA == 2)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[1,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 2 && BA == 3)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,1,0] op_sel_hi:[1,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 3 && BA == 0)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 3 && BA == 1)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,1,0] op_sel_hi:[1,0,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 3 && BA == 2)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,0,0] op_sel_hi:[1,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
  if constexpr (BW == 3 && BA == 3)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,1,0] op_sel_hi:[1,1,0]"
                 : "+v"(acc) : "v"(w), "v"(a), "v"(sw), "v"(sa));
}

// the gated epilogue loads its residual rows before the LDS image (default; 0 = inside the row loop, A/B:
// profiles/r04_gemm_epi_ab.log, out-projection 0.574-0.582 vs 0.630 ms)
#ifndef VP_GEMM_EPI_RPRE
#define VP_GEMM_EPI_RPRE 1
#endif
// the gated row pass's branch-free form (epi_rows_gated; 0 = the per-row form for every tile, A/B)
#ifndef VP_GEMM_GATED_FAST
#define VP_GEMM_GATED_FAST 1
#endif
// ---- fused epilogue shared by the GEMM kernels: acc[j][i] = the 16x16 fragment (W rows j, A rows i) of a wave
// whose C block is rows wr*WM.., cols wc*WN.. of the BM x BN tile.  Three pieces: epi_values (per-fragment bias /
// activation / qk-norm in registers -> bf16), epi_to_lds (a wave's values into the LDS C image), epi_rows_out (NT
// threads stream image rows out as 16-byte row stores, with the row-wise epilogues: residual / gate / injection /
// pos-emb / MX).  The persistent kernel runs the last two per half tile so the next tile's first K-tile can load
// into the other half of the LDS meanwhile. ----
// Internal instance kinds (not ABI values): an epilogue with the aux output (vp_gemm_desc.aux) is its own instance,
// so the inference instances carry none of its code or registers.
constexpr int EPI_QKNORM_AUX = 8, EPI_GELU_AUX = 9;
// the ABI epilogue of an instance kind, and whether the instance writes aux (EPI = -1: both from the descriptor)
template <int EPI>
VP_DEV int epi_kind(const vp_gemm_desc& d) {
  if constexpr (EPI < 0) return d.epilogue;
  return EPI == EPI_QKNORM_AUX ? VP_EPI_BIAS_QKNORM_ROPE : EPI == EPI_GELU_AUX ? VP_EPI_BIAS_GELU : EPI;
}
template <int EPI>
VP_DEV bool epi_aux(const vp_gemm_desc& d) {
  if constexpr (EPI < 0) return d.aux != nullptr;
  return EPI == EPI_QKNORM_AUX || EPI == EPI_GELU_AUX;
}

// EPI >= 0: the epilogue kind as a compile-time constant (the persistent kernel is instantiated per kind; with the
// runtime switch its register allocation spills), FULL_N: N % 256 == 0 (no column guard)
template <int FN, int FM, int WN, int WM, int EPI = -1, bool FULL_N = false, class Sink>
VP_DEV void epi_values(const vp_gemm_desc& d, const f32x4 (&acc)[FN][FM], Sink&& sink, int m0, int n0, int wr, int wc,
                       int lane) {
  const int epi = epi_kind<EPI>(d);
  const bool aux = epi_aux<EPI>(d);
  // head by head (4 fragments = 64 columns; WN % 64 == 0 and n0 % 256 == 0), so a head's accumulators die as its
  // values go to the sink.  Fused QKV (VP_EPI_BIAS_QKNORM_ROPE): q / k heads go through norm + RoPE in registers
  // (ln64_rope16: lane xor 16 / 32 are the other column quarters of the same row); v heads take the plain path.
  static_assert(FN % 4 == 0 && WN % 64 == 0, "whole heads per wave");
  const int g = lane >> 4;
  // no integer division per element: the segment of a column by compares (at most 3 segments), the token of a row
  // from the tile's first token (one division per tile)
  auto seg_of = [&](int c) { return (int)(c >= d.n_seg) + (int)(c >= 2 * d.n_seg); };
  const int tok0 = epi == VP_EPI_BIAS_QKNORM_ROPE ? m0 % d.tokens_per_batch : 0;
#pragma unroll
  for (int hh = 0; hh < FN / 4; ++hh) {
    const int nh = n0 + wc * WN + hh * 64;  // first column of the head
    const int sgh = seg_of(nh);
    if (epi == VP_EPI_BIAS_QKNORM_ROPE && nh < d.N && sgh < 2) {
      const bf16* bp = (const bf16*)d.bias[sgh];
      const int hc = nh - sgh * d.n_seg;  // column within the segment
      // one 8-byte load per 4 columns, all issued before any use (16 scalar bf16 loads came out of the compiler as
      // 16 serialised round trips, each behind its own vmcnt(0))
      float bv[16];
      bf16x4 b4[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        b4[jj] = bp != nullptr ? *(const bf16x4*)(bp + hc + 16 * jj + 4 * g) : bf16x4{};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[4 * jj + r] = bp != nullptr ? bf2f(b4[jj][r]) : 0.f;
      // the LayerNorm weight / bias quads once per head; per row fragment the RoPE quads are loaded (from row 0 for
      // text tokens, then not applied) before the reductions, so no load sits on the fragment's critical path
      bf16x4 lw4[4], lb4[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        lw4[jj] = *(const bf16x4*)((const bf16*)d.qk_ln_w[sgh] + 16 * jj + 4 * g);
        lb4[jj] = *(const bf16x4*)((const bf16*)d.qk_ln_b[sgh] + 16 * jj + 4 * g);
      }
      const bool has_rope = d.rope_cos != nullptr;
      // the RoPE quads of row fragment i + 1 are loaded before fragment i's reductions (double-buffered), so their
      // latency runs under the previous fragment's work instead of in front of each fragment
      f32x4 csb[2][4], snb[2][4];
      bool rotb[2];
      const bool sep = has_rope && d.rope_ax[0] != nullptr;  // separable table: per-axis rows (vp_gemm_desc)
      auto load_rope = [&](int i, f32x4 (&cs)[4], f32x4 (&sn)[4], bool& rot) {
        int tok = tok0 + wr * WM + i * 16 + (lane & 15);
        while (tok >= d.tokens_per_batch) tok -= d.tokens_per_batch;
        rot = has_rope && tok >= d.text_len;
        if (sep) {
          // token v -> (frame t, row y, column x) by the host's division magics; lane group g's quad of dims
          // 16 jj + 4 g .. + 3 lies in one axis (the axis boundaries 16 and 40 are multiples of 4)
          const unsigned v = rot ? (unsigned)(tok - d.text_len) : 0u;
          const unsigned t = __umulhi(v, d.rope_mhw);
          const unsigned rr = v - t * (unsigned)d.rope_hw;
          const unsigned y = __umulhi(rr, d.rope_mw);
          const unsigned x = rr - y * (unsigned)d.rope_w;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int dim0 = 16 * jj + 4 * g;
            int ax, off;
            if (jj == 0) {
              ax = 0, off = (int)t * 16 + dim0;
            } else if (jj == 1 || (jj == 2 && g < 2)) {
              ax = 2, off = (int)y * 24 + dim0 - 16;
            } else {
              ax = 4, off = (int)x * 24 + dim0 - 40;
            }
            cs[jj] = *(const f32x4*)(d.rope_ax[ax] + off);
            sn[jj] = *(const f32x4*)(d.rope_ax[ax + 1] + off);
          }
          return;
        }
        const int64_t ro = rot ? (int64_t)(tok - d.text_len) * 64 : 0;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          cs[jj] = has_rope ? *(const f32x4*)(d.rope_cos + ro + 16 * jj + 4 * g) : (f32x4){1.f, 1.f, 1.f, 1.f};
          sn[jj] = has_rope ? *(const f32x4*)(d.rope_sin + ro + 16 * jj + 4 * g) : (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      };
      load_rope(0, csb[0], snb[0], rotb[0]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if (i + 1 < FM) load_rope(i + 1, csb[(i + 1) & 1], snb[(i + 1) & 1], rotb[(i + 1) & 1]);
        const f32x4(&cs)[4] = csb[i & 1];
        const f32x4(&sn)[4] = snb[i & 1];
        const bool rot = rotb[i & 1];
        float x[16];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) x[4 * jj + r] = rbf(acc[hh * 4 + jj][i][r] + bv[4 * jj + r]);
        if (aux) {  // the pre-norm q | k for the training backward (vp_gemm_desc.aux)
          const int m = m0 + wr * WM + i * 16 + (lane & 15);
          if (m < d.M) {
            bf16* ap = (bf16*)d.aux + (int64_t)m * d.ld_aux + nh + 4 * g;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              bf16x4 o;
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = f2bf(x[4 * jj + r]);
              *(bf16x4*)(ap + 16 * jj) = o;
            }
          }
        }
        ln64_rope16_regs<16, 32>(x, lw4, lb4, d.qk_eps[sgh], cs, sn, rot);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(x[4 * jj + r]);
          sink(hh * 4 + jj, i, o);
        }
      }
      continue;
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = hh * 4 + jj;
      const int nloc = wc * WN + j * 16 + g * 4;  // 4 consecutive columns
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      {
        // the 4 columns share a segment (n_seg % 8 == 0) and are all in range or all out (N % 8 == 0, the first
        // column a multiple of 4): one 8-byte load
        const int sg = seg_of(n0 + nloc);
        const bf16* bp = (const bf16*)d.bias[sg];
        const int n = n0 + nloc;
        if (bp != nullptr && (FULL_N || n < d.N)) {
          const bf16x4 b4 = *(const bf16x4*)(bp + n - sg * d.n_seg);
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[r] = bf2f(b4[r]);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = rbf(acc[j][i][r] + bv[r]);
          // (with an aux output the GELU runs in the row pass, on the bf16 pre-activation it stores: the same bits)
          if ((epi == VP_EPI_BIAS_GELU && !aux) || epi == VP_EPI_BIAS_GELU_MXFP8) v = gelu_tanh(v);
          else if (epi == VP_EPI_BIAS_SCALE) v = v * d.alpha;
          o[r] = f2bf(v);
        }
        sink(j, i, o);
      }
    }
  }
}

// the LDS C image address of fragment (j, i)'s 4 values for this lane (image row = tile row - row0); CTS: bytes per
// image row (tile columns x 2 + a bank-conflict pad)
template <int WN, int WM, int CTS = CT_STRIDE>
VP_DEV char* epi_lds_addr(char* img, int j, int i, int row0, int wr, int wc, int lane) {
  return img + (wr * WM + i * 16 + (lane & 15) - row0) * CTS + (wc * WN + j * 16 + (lane >> 4) * 4) * 2;
}

// image rows [0, nrows) = tile rows row0.. out to C (coalesced 16-byte row stores + the row-wise epilogues); BNC:
// the tile's columns (256, or 128 for the two-workgroups-per-CU kernel)
template <int NT, bool FP8, int EPI = -1, int BNC = BN, int NPRE = 0>
VP_DEV void epi_rows_out(const vp_gemm_desc& d, const MxExt& mx, const char* smem, int row0, int nrows, int m0,
                         int n0, int tid, const bf16x8* rpre = nullptr) {
  constexpr int CPR = BNC / 8;        // 16-byte chunks per tile row
  constexpr int CTS = BNC * 2 + 8;
  const int epi = epi_kind<EPI>(d);
  const bool aux = epi_aux<EPI>(d);
  bf16* C = (bf16*)d.C;
  const int chunk = tid & (CPR - 1);  // 16-byte chunk within the tile row
  const int ncol = n0 + chunk * 8;
  // row bookkeeping without an integer division per row: the image rows are consecutive matrix rows, so the output
  // group (rows_per_group) and the batch (tokens_per_batch) of the image's first row are computed once and the
  // rows of this thread step forward from there (at most one boundary per few rows unless a group is tiny)
  const int mbase = m0 + row0;
  const int rpg = d.rows_per_group;
  const int grp0 = mbase / rpg, gin0 = mbase - grp0 * rpg;
  const int tpb = d.tokens_per_batch;
  const bool need_b = epi == VP_EPI_GATED;
  const int b0 = need_b ? mbase / tpb : 0, tk0 = need_b ? mbase - b0 * tpb : 0;
  // NPRE > 0: the gated epilogue's residual rows were loaded before the LDS image (rpre[it]); the loop is unrolled
  // so they stay in registers
#pragma unroll(NPRE > 0 ? NPRE : 1)
  for (int it = 0; it < nrows / (NT / CPR); ++it) {
    const int mloc = it * (NT / CPR) + tid / CPR;
    const int m = mbase + mloc;
    if (m >= d.M || ncol >= d.N) continue;
    bf16x8 v = *(const bf16x8*)(smem + mloc * CTS + chunk * 16);
    int grp = grp0, gin = gin0 + mloc;
    while (gin >= rpg) {
      gin -= rpg;
      ++grp;
    }
    const int64_t orow = (int64_t)grp * d.group_stride + d.row_offset + gin;
    if (FP8 && epi == VP_EPI_BIAS_GELU_MXFP8) {
      // MX-quantise the GELU output: the 4 lanes holding one 32-column block agree on its scale (N % 256 == 0, so
      // a block's lanes are all in or all out of range)
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = bf2f(v[e]);
      uint8_t sb;
      const u32x2 q = mx_quantize_quarter(f, sb);
      *(u32x2*)((uint8_t*)d.C + orow * d.ldc + ncol) = q;
      if ((tid & 3) == 0) mx.c_scale[mx_scale_off(orow, ncol >> 5, d.N)] = sb;
      continue;
    }
    if (epi == VP_EPI_BIAS_GELU && aux) {
      // the training forward's FF1: the pre-activation z to aux, GELU(z) to C
      *(bf16x8*)((bf16*)d.aux + (int64_t)m * d.ld_aux + ncol) = v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(gelu_tanh(bf2f(v[e])));
    } else if (epi == VP_EPI_GELU_BWD) {
      const bf16x8 z = *(const bf16x8*)((const bf16*)d.R + (int64_t)m * d.ldr + ncol);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) * gelu_grad(bf2f(z[e])));
    } else if (epi == VP_EPI_GATED) {
      int b = b0, tok = tk0 + mloc;
      while (tok >= tpb) {
        tok -= tpb;
        ++b;
      }
      const bf16* g = (const bf16*)(tok < d.text_len ? d.gate_text : d.gate) + (int64_t)b * d.gate_bstride + ncol;
      const bf16x8 gv = *(const bf16x8*)g;
      const bf16x8 rv = NPRE > 0 ? rpre[it] : *(const bf16x8*)((const bf16*)d.R + orow * d.ldr + ncol);
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
      const bf16x8 pv = *(const bf16x8*)((const bf16*)d.addrows + (int64_t)(gin + d.addrows_offset) * d.addrows_ld + ncol);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(pv[e]));
    }
#ifdef VP_GEMM_ABL_NOSTORE  // ablation build (tools/gemm_kscan.py): everything but the global store
    asm volatile("" ::"v"(v));
#else
    *(bf16x8*)(C + orow * d.ldc + ncol) = v;
#endif
  }
}


// The gated row pass with the residual rows preloaded (rpre), for tiles whose rows cross at most one batch and one
// output-group boundary (tokens_per_batch, rows_per_group >= BM): every load of the pass is issued up front and
// branch-free — the <= 4 gate vectors the tile's rows use (text / video x 2 batches), the 16 rows' injection-mask bytes,
// then their injection rows — so the pass waits for memory twice instead of three times per row (the per-row form
// with its data-dependent branches came out of the compiler fully serialised).  Same arithmetic per element as
// epi_rows_out: bit-identical.
template <int NT, int NPRE>
VP_DEV void epi_rows_gated(const vp_gemm_desc& d, const char* smem, int m0, int n0, int tid,
                           const bf16x8 (&rpre)[NPRE]) {
  constexpr int CPR = BN / 8, CTS = BN * 2 + 8, RS = NT / CPR;
  const int chunk = tid & (CPR - 1);
  const int ncol = n0 + chunk * 8;
  const bool col_ok = ncol < d.N;
  const int r0 = tid / CPR;
  const int rpg = d.rows_per_group, tpb = d.tokens_per_batch, T = d.text_len;
  const int grp0 = m0 / rpg, gin0 = m0 - grp0 * rpg;
  const int b0 = m0 / tpb, tk0 = m0 - b0 * tpb;
  // the tile's gate vectors: batch b0, and b0 + 1 when the tile reaches it (uniform)
  const bool two_b = tk0 + BM > tpb && (int64_t)(b0 + 1) * tpb < d.M;
  const bf16* gvid = (const bf16*)d.gate + ncol;
  const bf16* gtxt = (const bf16*)d.gate_text + ncol;
  const bf16x8 gv0 = col_ok ? *(const bf16x8*)(gvid + (int64_t)b0 * d.gate_bstride) : bf16x8{};
  const bf16x8 gt0 = col_ok ? *(const bf16x8*)(gtxt + (int64_t)b0 * d.gate_bstride) : bf16x8{};
  const bf16x8 gv1 = (col_ok && two_b) ? *(const bf16x8*)(gvid + (int64_t)(b0 + 1) * d.gate_bstride) : bf16x8{};
  const bf16x8 gt1 = (col_ok && two_b) ? *(const bf16x8*)(gtxt + (int64_t)(b0 + 1) * d.gate_bstride) : bf16x8{};
  const bool has_inj = d.inject != nullptr;
  uint32_t injbits = 0;  // bit it: row it takes the injection (flags staged in LDS by gemm_epilogue, one per row)
  if (has_inj) {
    // the flags of rows r0 + 16 it are bytes it of one 16-byte LDS word (stored transposed by gemm_epilogue)
    static_assert(NPRE == 16 && RS == 16, "the flag layout assumes 16 rows per step and 16 steps");
    const u32x4 fw = *(const u32x4*)(smem + EPI_FLAG_OFF + r0 * 16);
#pragma unroll
    for (int it = 0; it < NPRE; ++it)
      injbits |= (col_ok && ((fw[it >> 2] >> (8 * (it & 3))) & 0xffu) != 0 ? 1u : 0u) << it;
  }
  bf16x8 iv[NPRE];
#pragma unroll
  for (int it = 0; it < NPRE; ++it) {
    const int mloc = it * RS + r0;
    int tok = tk0 + mloc, b = b0;
    if (tok >= tpb) {
      tok -= tpb;
      ++b;
    }
    iv[it] = ((injbits >> it) & 1u) ? *(const bf16x8*)((const bf16*)d.inject + (int64_t)b * d.inject_bstride +
                                                       (int64_t)(tok - T) * d.inject_ld + ncol)
                                    : bf16x8{};
  }
  bf16* C = (bf16*)d.C;
#pragma unroll
  for (int it = 0; it < NPRE; ++it) {
    const int mloc = it * RS + r0;
    if (m0 + mloc >= d.M || !col_ok) continue;
    bf16x8 v = *(const bf16x8*)(smem + mloc * CTS + chunk * 16);
    int gin = gin0 + mloc, grp = grp0;
    if (gin >= rpg) {
      gin -= rpg;
      ++grp;
    }
    int tok = tk0 + mloc;
    const bool hi = tok >= tpb;
    if (hi) tok -= tpb;
    const bf16x8 gv = tok < T ? (hi ? gt1 : gt0) : (hi ? gv1 : gv0);
    const bf16x8 rv = rpre[it];
    const bool inj = (injbits >> it) & 1u;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float o = rbf(bf2f(rv[e]) + rbf(bf2f(gv[e]) * bf2f(v[e])));
      if (inj) o = rbf(o + bf2f(iv[it][e]));
      v[e] = f2bf(o);
    }
    const int64_t orow = (int64_t)grp * d.group_stride + d.row_offset + gin;
    *(bf16x8*)(C + orow * d.ldc + ncol) = v;
  }
}

template <int NT, int FN, int FM, int WN, int WM, bool FP8, int EPI = -1>
VP_DEV void gemm_epilogue(const vp_gemm_desc& d, const MxExt& mx, const f32x4 (&acc)[FN][FM], char* smem, int m0,
                          int n0, int wr, int wc, int lane, int tid) {
#if VP_GEMM_EPI_RPRE
  if constexpr (EPI == VP_EPI_GATED && !FP8 && NT == NTHREADS) {
    // the residual rows of this thread's row pass, loaded before the LDS image is written (their latency and the
    // round's residual burst run under epi_values and the barrier instead of inside the row loop)
    constexpr int CPR = BN / 8, NPRE = BM / (NT / CPR);
    bf16x8 rpre[NPRE];
    const int chunk = tid & (CPR - 1);
    const int ncol = n0 + chunk * 8;
    const int rpg = d.rows_per_group;
    const int grp0 = m0 / rpg, gin0 = m0 - grp0 * rpg;
    if (d.inject != nullptr && tid < BM) {
      // the injection flag of tile row tid: a video row whose mask byte is 0 (or no mask); one byte load per row
      // for the whole tile, read back from LDS by the row pass (flags area past the C image: no overlap with the
      // ring or the image)
      const int m = m0 + tid;
      const int tpb = d.tokens_per_batch;
      const int b = m / tpb, tok = m - b * tpb;
      const bool vid = m < d.M && tok >= d.text_len;
      const bool f = vid && (d.inject_mask == nullptr ||
                             d.inject_mask[(int64_t)b * d.inject_mask_bstride + (tok - d.text_len)] == 0);
      smem[EPI_FLAG_OFF + (tid & 15) * 16 + (tid >> 4)] = f ? 1 : 0;  // row tid -> word tid % 16, byte tid / 16
    }
#pragma unroll
    for (int it = 0; it < NPRE; ++it) {
      const int mloc = it * (NT / CPR) + tid / CPR;
      int grp = grp0, gin = gin0 + mloc;
      while (gin >= rpg) {
        gin -= rpg;
        ++grp;
      }
      const int64_t orow = (int64_t)grp * d.group_stride + d.row_offset + gin;
      rpre[it] = (m0 + mloc < d.M && ncol < d.N) ? *(const bf16x8*)((const bf16*)d.R + orow * d.ldr + ncol)
                                                  : bf16x8{};
    }
    epi_values<FN, FM, WN, WM, EPI>(
        d, acc,
        [&](int j, int i, const bf16x4& o) { *(bf16x4*)epi_lds_addr<WN, WM>(smem, j, i, 0, wr, wc, lane) = o; },
        m0, n0, wr, wc, lane);
    __syncthreads();
    if (VP_GEMM_GATED_FAST && d.tokens_per_batch >= BM && d.rows_per_group >= BM)
      epi_rows_gated<NT, NPRE>(d, smem, m0, n0, tid, rpre);
    else
      epi_rows_out<NT, FP8, EPI, BN, NPRE>(d, mx, smem, 0, BM, m0, n0, tid, rpre);
    return;
  }
#endif
  epi_values<FN, FM, WN, WM, EPI>(
      d, acc,
      [&](int j, int i, const bf16x4& o) { *(bf16x4*)epi_lds_addr<WN, WM>(smem, j, i, 0, wr, wc, lane) = o; }, m0,
      n0, wr, wc, lane);
  __syncthreads();
  // (the row loop stays rolled for the epilogues without row-wise inputs: an unrolled, branch-free form issued the
  // 16 image reads together but was 1-1.5 % slower on QKV / FF1, profiles/r04_gemm_plain_rowpass_ab_rejected.log —
  // the pass is store-issue bound, as round 2's unroll A/B found)
  epi_rows_out<NT, FP8, EPI>(d, mx, smem, 0, BM, m0, n0, tid);
}

// EPI >= 0: the epilogue kind as a compile-time constant (the default main loop is instantiated per kind: the dead
// kinds' code and branches leave the epilogue), -1: runtime switch
// SPLIT: the split-K instance (fp32 partial tiles to mx.ws, the epilogue runs in gemm_splitk_reduce_kernel)
// ATAIL: the per-segment A tail of vp_gemm_desc (unfused LoRA): A K-tiles from a_tail_k on are read a_tail_off[seg]
// columns further right (one scalar add per A DMA of those tiles)
#ifndef VP_CLOCK_STAMPS
#define VP_CLOCK_STAMPS 0
#endif
#if VP_CLOCK_STAMPS
// diagnostic builds only (tools/gemm_wg_timeline.py): realtime at workgroup entry and exit per blockIdx
constexpr int GEMM_CLOCK_SLOTS = 1 << 15;
__device__ unsigned long long vp_gemm_clock_buf[GEMM_CLOCK_SLOTS * 2];
struct GemmStamp {
  unsigned long long e0;
  __device__ __forceinline__ GemmStamp() : e0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ __forceinline__ ~GemmStamp() {
    if (threadIdx.x == 0 && blockIdx.x < GEMM_CLOCK_SLOTS) {
      vp_gemm_clock_buf[blockIdx.x * 2] = e0;
      vp_gemm_clock_buf[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
};
#else
struct GemmStamp {};
#endif

template <int VAR, bool FP8 = false, int GROUP = 4, int EPI = -1, bool SPLIT = false, bool ATAIL = false>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_bf16_kernel(const vp_gemm_desc d, const MxExt mx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  [[maybe_unused]] GemmStamp stamp;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2;  // 0..1  (M)
  const int wc = wave & 3;   // 0..3  (N)

  const int tiles_m = (d.M + BM - 1) / BM;
  const int tiles_n = (d.N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int t = SPLIT ? mx.t_base + lin / mx.nsplit : lin;
  const int kc = SPLIT ? lin % mx.nsplit : 0;  // K-chunk of this workgroup
  // this workgroup's K range: [kbeg, kbeg + Kloop) (the whole K unless split)
  const int kbeg = SPLIT ? kc * mx.kchunk : 0;
  const int Kloop = SPLIT ? min(mx.kchunk, d.K - kbeg) : d.K;
  const int G = mx.group > 0 ? mx.group : GROUP;
  const int per_group = G * tiles_n;
  const int group_id = t / per_group;
  const int first_m = group_id * G;
  const int gsz = min(tiles_m - first_m, G);
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

  if constexpr (VAR == 5 || VAR == 11 || VAR == 13) {
    // Quadrant-phase pipeline.  Each wave's 128x64 C block is split into 4 quadrants (64 rows x 32 cols); a K-tile
    // (BK = 64) runs as 4 phases of 16 MFMAs, in the quadrant order (A0,B0) (A0,B1) (A1,B1) (A1,B0) so each phase
    // needs ONE new operand subtile, which is read from LDS into registers during the previous phase.  The LDS
    // holds two K-tiles as 4 "units" each (A rows of quadrant-row 0 / 1, W rows of quadrant-col 0 / 1, 16 KB = two
    // LDS-DMA instructions per thread).  Phase slot s issues one unit (B0 and B1 and A1 of tile k+2 in phases 0-2
    // of tile k, A0 of tile k+3 in phase 3), so every unit is in flight for 7 phases before it is read; at the top of
    // each slot a wave waits for the unit issued 7 slots earlier (vmcnt(12): 6 units stay in flight) and for its
    // own LDS reads, then ONE barrier both publishes that unit and retires the reads of the region the slot's DMA
    // overwrites (each unit's region is last read in the slot just before the one that refills it).
    // bf16: a K-tile is 64 elements; fp8: 128 (the same 128 bytes per row, so the LDS images are identical)
    constexpr int EB = FP8 ? 1 : 2;                 // bytes per element
    constexpr int TK = FP8 ? 128 : BK;              // K elements per tile
    const int nk = (Kloop + TK - 1) / TK;
    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, 1>;
    // Per-lane 32-bit byte offsets of the 4 units' source rows (2 LDS-DMA instructions each) from a wave-uniform
    // base (the activation, or the weight segment that holds the 8-row block: blocks never straddle a segment since
    // n_seg % 8 == 0), so the DMA uses saddr + voffset addressing and the per-tile advance is a scalar add.
    int uoff[4][2];
    const char* ubase[4][2];
    // fp8 (the caller pads A to whole 256-row tiles and N % 256 == 0, so no row is clamped): every unit's
    // per-lane offset is one of two lane values (the swizzle depends only on row bits 1-3, which the unit and
    // instruction offsets do not touch) plus a wave-uniform base — 2 VGPRs instead of 8
    int uoffA = 0, uoffW = 0;
    int sgW = 0;
    if constexpr (FP8) {
      const int ra = wave * 8 + (lane >> 3);
      uoffA = ra * (int)d.lda + (((lane & 7) ^ swz(ra)) << 4);
      const int rw = (wave >> 2) * 64 + (wave & 3) * 8 + (lane >> 3);
      uoffW = rw * d.K + (((lane & 7) ^ swz(rw)) << 4);
      sgW = __builtin_amdgcn_readfirstlane(n0 / d.n_seg);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int g = i * 8 + wave;
          const int rb = (u < 2) ? (g >> 3) * 128 + u * 64 + (g & 7) * 8 : (g >> 2) * 64 + (u - 2) * 32 + (g & 3) * 8;
          const int r = rb + (lane >> 3);
          const int c = (lane & 7) ^ swz(r);
          if (u < 2) {
            // 64-bit tile base + 32-bit in-tile offset (M * lda can pass 2^31 bytes: FF2 at config 5)
            ubase[u][i] = (const char*)d.A + ((int64_t)m0 * d.lda + kbeg) * EB;
            uoff[u][i] = (min(m0 + r, d.M - 1) - m0) * (int)d.lda * EB + c * 16;
          } else {
            const int sg = __builtin_amdgcn_readfirstlane(min(n0 + rb, d.N - 1) / d.n_seg);
            ubase[u][i] = (const char*)d.W[sg] + (int64_t)kbeg * EB;
            uoff[u][i] = ((min(n0 + r, d.N - 1) - sg * d.n_seg) * d.K) * EB + c * 16;
          }
        }
    }
    // unit u: 0 = A quadrant-row 0, 1 = A quadrant-row 1, 2 = W quadrant-col 0, 3 = W quadrant-col 1
    // (this variant runs only for K % 64 == 0, so there is no K tail here)
    [[maybe_unused]] int tail_tile0 = 0;
    [[maybe_unused]] int64_t tail_skip = 0;
    if constexpr (ATAIL) {
      tail_tile0 = d.a_tail_k / BK;
      const int sg = __builtin_amdgcn_readfirstlane(n0 / d.n_seg);  // n_seg % BN == 0: one segment per tile
      tail_skip = (sg == 0 ? d.a_tail_off[0] : sg == 1 ? d.a_tail_off[1] : d.a_tail_off[2]) * 2;
    }
    auto issue_unit = [&](int u, int tile) {
      char* base = smem + (tile & 1) * STAGE_BYTES + (u >= 2 ? TILE_BYTES : 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int g = i * 8 + wave;
        const int rb = (u < 2) ? (g >> 3) * 128 + u * 64 + (g & 7) * 8 : (g >> 2) * 64 + (u - 2) * 32 + (g & 3) * 8;
        if constexpr (FP8) {
          if (u < 2)
            glds16((const char*)d.A + (int64_t)(m0 + i * 128 + u * 64) * d.lda + tile * 128, uoffA, base + rb * 128);
          else
            glds16((const char*)d.W[sgW] + (int64_t)(n0 - sgW * d.n_seg + i * 128 + (u - 2) * 32) * d.K + tile * 128,
                   uoffW, base + rb * 128);
        } else if constexpr (ATAIL) {
          glds16(ubase[u][i] + tile * 128 + (u < 2 && tile >= tail_tile0 ? tail_skip : 0), uoff[u][i], base + rb * 128);
        } else {
          glds16(ubase[u][i] + tile * 128, uoff[u][i], base + rb * 128);
        }
      }
    };
    // fp8: the scales of tile T (1 KiB per operand, MX tile layout) ride with tile T's first unit (slot 4T-9):
    // wave 0 fetches the A scales, wave 1 the W scales, into ring slot T & 3 — issued before that unit's DMA, so
    // the wait that publishes the unit publishes them too
    const char* sA = nullptr;
    const char* sW = nullptr;
    if constexpr (FP8) {
      const int sgw = __builtin_amdgcn_readfirstlane(min(n0, d.N - 1) / d.n_seg);
      sA = (const char*)mx.a_scale + (int64_t)(m0 >> 8) * nk * 1024;
      sW = (const char*)mx.w_scale[sgw] + (int64_t)((n0 - sgw * d.n_seg) >> 8) * nk * 1024;
    }
    auto issue_scales = [&](int tile) {
      if constexpr (FP8) {
        char* dst = smem + SCALE_OFF + (tile & 3) * 2048;
        if (wave < 2) {
          // lane * 16 materialised in place (a hoisted copy would be one more long-lived VGPR, and its spill reload
          // would drain the DMA queue with vmcnt(0))
          int off;
          asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshlrev_b32 %0, 4, %0"
                       : "=v"(off));
          glds16(wave == 0 ? sA + tile * 1024 : sW + tile * 1024, off, wave == 0 ? dst : dst + 1024);
        }
      }
    };
    auto slot_tile = [&](int sl, int& u) -> int {  // unit and tile issued by slot sl (sl >= -9)
      const int k = (sl + 12) / 4 - 3;
      const int p = sl - 4 * k;
      u = p == 0 ? 2 : p == 1 ? 3 : p == 2 ? 1 : 0;
      return p < 3 ? k + 2 : k + 3;
    };
    auto exists = [&](int sl) {
      int u;
      return slot_tile(sl, u) < nk;
    };
    auto issue_slot = [&](int sl) {
      int u;
      const int tile = slot_tile(sl, u);
      if (tile < nk) {
        if (u == 0) issue_scales(tile);
        issue_unit(u, tile);
      }
    };
    auto top = [&](int sl) {
      if (exists(sl - 1)) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    // LDS fragment addresses: swz(row) depends only on lane&15 here (rows step by 16), so every read is one of two
    // lane bases (k-halves) plus a compile-time offset (buffer parity, quadrant, fragment)
    const int lrow = lane & 15;
    int lbase[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // bf16: k-step ks of a 16x16x32 fragment is chunk ks*4 + lane/16.  fp8 (measured, tools/mx_probe.py): the
      // 32 bytes lane l feeds a 16x16x128 MFMA are K-chunks lane/16 and lane/16 + 4 of its row — the same two
      // chunks, so the same conflict-free reads; K-block b = chunks 2b, 2b+1 takes lane (row, b)'s scale
      const int ch = ks * 4 + (lane >> 4);
      lbase[ks] = lrow * 128 + ((ch ^ swz(lrow)) << 4);
    }
    // fp8 scales of one K-tile, read once per tile: this lane's (row lane%16, K-block lane/16) byte of the A
    // fragments (8 rows-groups: byte i of word qm = quadrant-row qm, fragment i) and of the W fragments (byte
    // qn*2 + j).  Tile k+1's scales are read in tile k's phase 2, next to its first A fragments.
    struct TileScales {
      int a0, a1, w;
    };
    const int sbase = (lane >> 4) * 256 + lrow * 16;
    auto readS = [&](TileScales& ts, int tile) {
      if constexpr (FP8) {
        const char* sp = smem + SCALE_OFF + (tile & 3) * 2048 + sbase;
        const u32x2 a = *(const u32x2*)(sp + wr * 8);
        ts.a0 = (int)a[0];
        ts.a1 = (int)a[1];
        ts.w = *(const int*)(sp + 1024 + wc * 4);
      }
    };
    // register fragments of one quadrant: bf16 = 4 (A) / 2 (W) 16x16x32 fragments x 2 k-steps; fp8 = 4 / 2
    // 16x16x128 fragments of 8 VGPRs each (both halves read straight into one register tuple)
    using FragA = std::conditional_t<FP8, i32x8[4], bf16x8[8]>;
    using FragB = std::conditional_t<FP8, i32x8[2], bf16x8[4]>;
    auto read8 = [&](const char* p) -> i32x8 {
      i32x8 f;
      u32x4* h = (u32x4*)&f;  // both 16-byte halves land in one 8-VGPR tuple (no copy into the MFMA operand)
      h[0] = *(const u32x4*)(p + lbase[0]);
      h[1] = *(const u32x4*)(p + lbase[1]);
      return f;
    };
    auto readA = [&](FragA& a, auto par_c, auto qm_c) {
      constexpr int par = decltype(par_c)::value, qm = decltype(qm_c)::value;
      const char* As = smem + par * STAGE_BYTES + (wr * WM + qm * 64) * 128;
      if constexpr (FP8) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = read8(As + i * 16 * 128);
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) a[ks * 4 + i] = *(const bf16x8*)(As + lbase[ks] + i * 16 * 128);
      }
    };
    auto readB = [&](FragB& bb, auto par_c, auto qn_c) {
      constexpr int par = decltype(par_c)::value, qn = decltype(qn_c)::value;
      const char* Bs = smem + par * STAGE_BYTES + TILE_BYTES + (wc * WN + qn * 32) * 128;
      if constexpr (FP8) {
#pragma unroll
        for (int j = 0; j < 2; ++j) bb[j] = read8(Bs + j * 16 * 128);
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 2; ++j) bb[ks * 2 + j] = *(const bf16x8*)(Bs + lbase[ks] + j * 16 * 128);
      }
    };
    auto mma = [&](const FragA& a, const FragB& bb, auto qm_c, auto qn_c, int sa, int sb) {
      constexpr int qm = decltype(qm_c)::value, qn = decltype(qn_c)::value;
      __builtin_amdgcn_sched_barrier(0);  // keep the next subtile's reads above this phase's MFMAs
      __builtin_amdgcn_s_setprio(1);
      if constexpr (FP8) {
        // 16x16x128 e4m3 x e4m3 with per-lane E8M0 scales, W (quadrant-col qn) as the first operand like the bf16
        // path; the byte opsel picks each fragment's scale out of the tile's scale words
#define VP_MX_MMA(J, I) mfma_mx<qn * 2 + J, I>(acc[qn * 2 + J][qm * 4 + I], bb[J], a[I], sb, sa)
        VP_MX_MMA(0, 0); VP_MX_MMA(0, 1); VP_MX_MMA(0, 2); VP_MX_MMA(0, 3);
        VP_MX_MMA(1, 0); VP_MX_MMA(1, 1); VP_MX_MMA(1, 2); VP_MX_MMA(1, 3);
#undef VP_MX_MMA
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[qn * 2 + j][qm * 4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  bb[ks * 2 + j], a[ks * 4 + i], acc[qn * 2 + j][qm * 4 + i], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    };
    {  // (the round-4 VAR 12 loop, one barrier per K-tile, was pruned in round 6: DESIGN_LOG.md)
    // VAR 11 = VAR 5 with the two wave groups STAGGERED (cdna_hip_programming.md §5 "256² 8-phase template",
    // MI355X_MICROARCH.md "Two waves per SIMD" item 9): every slot is [memory part] barrier [16 MFMAs] barrier and
    // waves 4-7 (quadrant-row 1, one wave on each SIMD) run one barrier behind waves 0-3, so on every SIMD one
    // wave's MFMA cluster overlaps its partner's LDS-DMA issue + ds_reads instead of both contending for the matrix
    // pipe and then both stalling at the same barrier.  With the stagger a staged unit must be waited for one slot
    // BEFORE the slot that reads it (the reader group may be a barrier ahead of the issuer group), so a slot waits
    // for the unit issued 6 slots earlier (vmcnt(10)) and reads the one issued 7 earlier; a slot's own reads retire
    // (lgkmcnt(0)) before its first barrier, so the v5 refill distance (one slot after the last read) still holds.
    // VAR 13 = VAR 11 with each slot's fragment reads issued BEFORE its vmcnt wait and LDS-DMA issue, so the read
    // latency runs under the DMA issue instead of after it (the reads of slot s are of units published at slot s - 1)
    constexpr bool STAGGER = VAR == 11 || VAR == 13;
    constexpr bool RFIRST = VAR == 13;
    FragA a0, a1;
    FragB bx, by;
    // prologue: slots -9..-2 (tiles 0 and 1, and nothing that overwrites tile 0's quadrant-row-0 A before it is
    // read), then the first subtiles, then slot -1 (A quadrant-row 0 of tile 2 into tile 0's region)
    for (int sl = -9; sl < -1; ++sl) issue_slot(sl);
    if constexpr (STAGGER) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // slots -9..-7 landed (nk >= 8)
    else if (exists(-2)) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // units of slots -9, -8 landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    TileScales scx = {0, 0, 0}, scy = {0, 0, 0};
    readA(a0, Z{}, Z{});
    readB(bx, Z{}, Z{});
    readS(scx, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_slot(-1);
    if constexpr (STAGGER) {
      if (wr == 1) __builtin_amdgcn_s_barrier();  // wave-uniform: waves 4-7 start one barrier behind
    }
    // one K-tile; PAR = k & 1 selects the LDS buffer and which of bx/by holds quadrant-col 0.  STEADY: every slot
    // of this tile issues a unit and 6 later units exist (k + 3 < nk), so the waits are the fixed vmcnt(12).
    auto tile_body = [&](int k, auto par_c, auto steady_c, FragB& b0, FragB& b1, const TileScales& sc,
                         TileScales& scn) {
      using P = decltype(par_c);
      using NP = std::integral_constant<int, 1 - P::value>;
      constexpr bool STEADY = decltype(steady_c)::value;
      const int s0 = 4 * k;
      auto slot = [&](int sl) {
        if constexpr (STAGGER) {
          // memory part, first half: wait for the unit the NEXT slot reads, then issue this slot's unit
          if (STEADY || exists(sl - 1)) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          issue_slot(sl);
        } else if constexpr (STEADY) {
          asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          int u;
          const int tile = slot_tile(sl, u);
          if (u == 0) issue_scales(tile);
          issue_unit(u, tile);
        } else {
          top(sl);
          issue_slot(sl);
        }
      };
      const bool more = STEADY || k + 1 < nk;
      auto cluster = [&]() {  // stagger: this slot's reads retire, then the MFMA cluster between two barriers
        if constexpr (STAGGER) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
      };
      auto cluster_end = [&]() {
        if constexpr (STAGGER) __builtin_amdgcn_s_barrier();
      };
      if constexpr (!RFIRST) slot(s0);
      readB(b1, P{}, O{});
      if constexpr (RFIRST) slot(s0);
      cluster();
      mma(a0, b0, Z{}, Z{}, sc.a0, sc.w);
      cluster_end();
      if constexpr (!RFIRST) slot(s0 + 1);
      readA(a1, P{}, O{});
      if constexpr (RFIRST) slot(s0 + 1);
      cluster();
      mma(a0, b1, Z{}, O{}, sc.a0, sc.w);
      cluster_end();
      if constexpr (!RFIRST) slot(s0 + 2);
      if (more) {
        readA(a0, NP{}, Z{});
        readS(scn, k + 1);
      }
      if constexpr (RFIRST) slot(s0 + 2);
      cluster();
      mma(a1, b1, O{}, O{}, sc.a1, sc.w);
      cluster_end();
      if constexpr (!RFIRST) slot(s0 + 3);
      if (more) readB(b1, NP{}, Z{});  // b1's registers carry the next tile's quadrant-col 0
      if constexpr (RFIRST) slot(s0 + 3);
      cluster();
      mma(a1, b0, O{}, Z{}, sc.a1, sc.w);
      cluster_end();
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    int k = 0;
    for (; k + 4 < nk; k += 2) {
      tile_body(k, Z{}, T_{}, bx, by, scx, scy);
      tile_body(k + 1, O{}, T_{}, by, bx, scy, scx);
    }
    // tail (at most 4 tiles; k is even here, so the parities are static)
    if (k < nk) tile_body(k, Z{}, F_{}, bx, by, scx, scy);
    if (k + 1 < nk) tile_body(k + 1, O{}, F_{}, by, bx, scy, scx);
    if (k + 2 < nk) tile_body(k + 2, Z{}, F_{}, bx, by, scx, scy);
    if (k + 3 < nk) tile_body(k + 3, O{}, F_{}, by, bx, scy, scx);
    if constexpr (STAGGER) {
      if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups (equal barrier counts)
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (FP8) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // asm MFMA results
    __syncthreads();
    }  // VAR 5 / 11
  } else if constexpr (VAR == 1) {
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
  }

  if constexpr (SPLIT) {
    // fp32 partial tile: lane (j, i) holds 4 consecutive columns of one row (16-byte stores)
    if (mx.tail) {  // compact: this workgroup's BM x BN slab
      float* P = mx.ws + ((int64_t)(t - mx.t_base) * mx.nsplit + kc) * (BM * BN);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int ml = wr * WM + i * 16 + (lane & 15);
          const int nl = wc * WN + j * 16 + (lane >> 4) * 4;
          *(f32x4*)(P + ml * BN + nl) = acc[j][i];
        }
      return;
    }
    float* P = mx.ws + (int64_t)kc * d.M * d.N;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wr * WM + i * 16 + (lane & 15);
        const int n = n0 + wc * WN + j * 16 + (lane >> 4) * 4;
        if (m < d.M && n < d.N) *(f32x4*)(P + (int64_t)m * d.N + n) = acc[j][i];
      }
    return;
  }
#ifdef VP_GEMM_ABL_NOEPI  // ablation build (tools/gemm_kscan.py): main loop only, accumulators kept live
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(acc[j][i]));
#else
  gemm_epilogue<NTHREADS, FN, FM, WN, WM, FP8, EPI>(d, mx, acc, smem, m0, n0, wr, wc, lane, tid);
#endif
}


// split-K reduce + epilogue: one thread per 8 consecutive output columns of one row; the chunks are summed in a fixed
// order, then the same roundings as the fused epilogues (epi_values + epi_rows_out)
VP_DEV void splitk_epilogue(const vp_gemm_desc& d, int m, int n, const float (&a)[8]);
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const vp_gemm_desc d, const float* __restrict__ ws,
                                                                 int nsplit) {
  const int c8 = d.N >> 3;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)d.M * c8) return;
  const int m = (int)(idx / c8);
  const int n = (int)(idx - (int64_t)m * c8) * 8;
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  const int64_t MN = (int64_t)d.M * d.N;
  for (int s = 0; s < nsplit; ++s) {
    const float* p = ws + s * MN + (int64_t)m * d.N + n;
    const f32x4 lo = *(const f32x4*)p, hi = *(const f32x4*)(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] += lo[e];
      a[4 + e] += hi[e];
    }
  }
  splitk_epilogue(d, m, n, a);
}

// tail mode: the last partial round's tiles (t_base..) from their compact partial slabs; 32 blocks of 256 threads
// per tile (8 rows x 32 eight-column chunks each); the tile coordinates as the GEMM kernel's grouped order (GROUP 4)
__global__ __launch_bounds__(256) void gemm_tail_reduce_kernel(const vp_gemm_desc d, const float* __restrict__ ws,
                                                               int t_base, int nsplit, int GROUP) {
  const int j = blockIdx.x >> 5;
  const int r = (blockIdx.x & 31) * 8 + (threadIdx.x >> 5);
  const int c = threadIdx.x & 31;
  const int t = t_base + j;
  const int tiles_m = (d.M + BM - 1) / BM, tiles_n = (d.N + BN - 1) / BN;
  const int per_group = GROUP * tiles_n;
  const int first_m = (t / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + ((t % per_group) % gsz), tn = (t % per_group) / gsz;
  const int m = tm * BM + r, n = tn * BN + c * 8;
  if (m >= d.M || n >= d.N) return;
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float* p = ws + ((int64_t)j * nsplit + s) * (BM * BN) + r * BN + c * 8;
    const f32x4 lo = *(const f32x4*)p, hi = *(const f32x4*)(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] += lo[e];
      a[4 + e] += hi[e];
    }
  }
  splitk_epilogue(d, m, n, a);
}

VP_DEV void splitk_epilogue(const vp_gemm_desc& d, int m, int n, const float (&a)[8]) {
  const int sg = (int)(n >= d.n_seg) + (int)(n >= 2 * d.n_seg);
  const bf16* bp = (const bf16*)d.bias[sg];
  const int grp = m / d.rows_per_group, gin = m - grp * d.rows_per_group;
  const int64_t orow = (int64_t)grp * d.group_stride + d.row_offset + gin;
  bf16x8 o, av;
  bf16x8 pv, gv, iv;
  bool inj = false;
  if (d.epilogue == VP_EPI_BIAS_ADDROWS) {
    pv = *(const bf16x8*)((const bf16*)d.addrows + (int64_t)(gin + d.addrows_offset) * d.addrows_ld + n);
  } else if (d.epilogue == VP_EPI_GELU_BWD) {
    pv = *(const bf16x8*)((const bf16*)d.R + (int64_t)m * d.ldr + n);
  } else if (d.epilogue == VP_EPI_GATED) {
    // epi_rows_out's gated row: residual (R, output row), the batch's text / video gate, the optional injection
    const int b = m / d.tokens_per_batch, tok = m - b * d.tokens_per_batch;
    gv = *(const bf16x8*)((const bf16*)(tok < d.text_len ? d.gate_text : d.gate) + (int64_t)b * d.gate_bstride + n);
    pv = *(const bf16x8*)((const bf16*)d.R + orow * d.ldr + n);
    if (d.inject != nullptr && tok >= d.text_len) {
      const int vtok = tok - d.text_len;
      inj = d.inject_mask == nullptr || d.inject_mask[(int64_t)b * d.inject_mask_bstride + vtok] == 0;
      if (inj)
        iv = *(const bf16x8*)((const bf16*)d.inject + (int64_t)b * d.inject_bstride + (int64_t)vtok * d.inject_ld + n);
    }
  }
  const bf16x8 b8 = bp != nullptr ? *(const bf16x8*)(bp + n - sg * d.n_seg) : bf16x8{};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float v = rbf(a[e] + (bp != nullptr ? bf2f(b8[e]) : 0.f));
    av[e] = f2bf(v);
    if (d.epilogue == VP_EPI_BIAS_GELU) v = rbf(gelu_tanh(v));
    else if (d.epilogue == VP_EPI_BIAS_SCALE) v = rbf(v * d.alpha);
    else if (d.epilogue == VP_EPI_BIAS_ADDROWS) v = bf2f(f2bf(v)) + bf2f(pv[e]);
    else if (d.epilogue == VP_EPI_GELU_BWD) v = rbf(v * gelu_grad(bf2f(pv[e])));
    else if (d.epilogue == VP_EPI_GATED) {
      v = rbf(bf2f(pv[e]) + rbf(bf2f(gv[e]) * v));
      if (inj) v = rbf(v + bf2f(iv[e]));
    }
    o[e] = f2bf(v);
  }
  if (d.epilogue == VP_EPI_BIAS_GELU && d.aux != nullptr) *(bf16x8*)((bf16*)d.aux + (int64_t)m * d.ld_aux + n) = av;
  *(bf16x8*)((bf16*)d.C + orow * d.ldc + n) = o;
}

// split-K plan: only when fewer than half the CUs would get a tile, whole 512-K chunks (the staggered main loop's
// minimum), at most one round of workgroups
struct SplitPlan {
  int nsplit = 1, kchunk = 0;
  int64_t ws_bytes = 0;
  int tail = 0;  // > 0: tail mode (the last `tail` tiles split, the others one main launch)
};
int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}
// Tail mode: a large GEMM whose last round of tiles (one 8-wave workgroup per CU) is at most a quarter full runs that
// round as split-K workgroups over whole 512-K chunks (one round, compact fp32 partials) plus a reduce that applies
// the epilogue, instead of a round of whole tiles on a mostly idle chip (config 2's FF1: 6 672 tiles = 26 rounds +
// 16).  The default main loop only (VP_GEMM_VARIANT unset or 13), and the epilogues the reduce implements.
SplitPlan tail_plan(const vp_gemm_desc* d, int tiles) {
  SplitPlan p;
  const char* e = vp_knob(VPK_GEMM_VARIANT);
  const char* nt = vp_knob(VPK_GEMM_NO_TAIL);
  if ((e != nullptr && atoi(e) != 13) || (nt != nullptr && strcmp(nt, "q") != 0)) return p;
  const int cus = device_cus();
  const int tail = tiles % cus;
  // up to half a round (the pieces then fit one round: tail x nsplit <= CUs).  Round 6 widened it from a quarter
  // (VP_GEMM_NO_TAIL=q keeps that rule, A/B): the training shape's N = 3072 GEMMs (M = 17 776: 840 tiles = 3 rounds
  // + 72) and the gated epilogue in the reduce
  if (tiles <= cus || tail == 0 || (nt != nullptr ? 4 : 2) * tail > cus) return p;
  if ((d->N % BN) != 0 || (d->K % BK) != 0) return p;
  const int nk = d->K / BK;
  const int ns = min(cus / tail, nk / 8);
  if (ns < 2) return p;
  const int chunk_t = (nk + ns - 1) / ns;
  p.kchunk = chunk_t * BK;
  p.nsplit = (nk + chunk_t - 1) / chunk_t;
  if (p.nsplit < 2 || d->K - (p.nsplit - 1) * p.kchunk < 8 * BK) return SplitPlan{};
  p.tail = tail;
  p.ws_bytes = (int64_t)tail * p.nsplit * BM * BN * 4;
  return p;
}
SplitPlan split_plan(const vp_gemm_desc* d) {
  SplitPlan p;
  const int tiles = ((d->M + BM - 1) / BM) * ((d->N + BN - 1) / BN);
  const bool epi_ok = d->epilogue == VP_EPI_BIAS || d->epilogue == VP_EPI_BIAS_GELU ||
                      d->epilogue == VP_EPI_BIAS_SCALE || d->epilogue == VP_EPI_BIAS_ADDROWS ||
                      d->epilogue == VP_EPI_GELU_BWD || d->epilogue == VP_EPI_GATED;
  if (!epi_ok || (d->K % BK) != 0 || d->a_tail_k > 0) return p;
  const int64_t tile_a0 = (int64_t)BM * d->lda * 2, wseg0 = (int64_t)d->n_seg * d->K * 2;
  if (tiles >= 128) return (tile_a0 < ((int64_t)1 << 31) && wseg0 < ((int64_t)1 << 31)) ? tail_plan(d, tiles) : p;
  if (d->K < 1024) return p;
  const int64_t tile_a = (int64_t)BM * d->lda * 2, wseg = (int64_t)d->n_seg * d->K * 2;
  if (tile_a >= ((int64_t)1 << 31) || wseg >= ((int64_t)1 << 31)) return p;
  // the fp32 partials (nsplit x M x N x 4 B, written and read back) should not outweigh the weights (N x K x 2 B)
  int ns = min(min(256 / tiles, d->K / 512), max(2, d->K / (2 * d->M)));
  if (ns < 2) return p;
  const int kt = d->K / BK;
  const int chunk_t = (kt + ns - 1) / ns;
  p.kchunk = chunk_t * BK;
  p.nsplit = (kt + chunk_t - 1) / chunk_t;
  if (p.nsplit < 2 || d->K - (p.nsplit - 1) * p.kchunk < 8 * BK) return SplitPlan{};  // last chunk >= 8 K-tiles
  p.ws_bytes = (int64_t)p.nsplit * d->M * d->N * 4;
  return p;
}

}  // namespace

#if VP_CLOCK_STAMPS
extern "C" int vp_diag_gemm_clock_read(void* host, int64_t slots) {
  if (host == nullptr || slots <= 0 || slots > GEMM_CLOCK_SLOTS) return VP_ERR_ARG;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vp_gemm_clock_buf), (size_t)slots * 16, 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" int vp_gemm_variant_built(int variant) {
  if (variant == 1 || variant == 5 || variant == 11 || variant == 13) return 1;
  return 0;  // (the rejected loops 12, 20, 30 were pruned in round 6: DESIGN_LOG.md)
}

// M-tiles per group of the grouped tile order (the VP_GEMM_GROUP knob overrides, A/B)
static int gemm_group(const vp_gemm_desc* d) {
  (void)d;
  const char* g = vp_knob(VPK_GEMM_GROUP);
  const int v = g != nullptr ? atoi(g) : 0;
  return v > 0 && v <= 64 ? v : 4;
}

// the ABI-17 fields: the aux output (VP_EPI_BIAS_GELU / _QKNORM_ROPE only) and VP_EPI_GELU_BWD's Z operand
static int check_aux(const vp_gemm_desc* d) {
  if (d->aux != nullptr) {
    if (d->epilogue == VP_EPI_BIAS_GELU) {
      if (d->ld_aux < d->N || (d->ld_aux % 8) != 0) return VP_ERR_ARG;
    } else if (d->epilogue == VP_EPI_BIAS_QKNORM_ROPE) {
      if (d->ld_aux < 2 * (int64_t)d->n_seg || (d->ld_aux % 8) != 0) return VP_ERR_ARG;
    } else {
      return VP_ERR_ARG;
    }
  }
  if (d->epilogue == VP_EPI_GELU_BWD && (d->R == nullptr || d->ldr < d->N || (d->ldr % 8) != 0)) return VP_ERR_ARG;
  return VP_OK;
}

// the instance-table slot of a descriptor: the ABI epilogue, or the aux instance of its kind
static int kernel_index(const vp_gemm_desc* d) {
  if (d->aux == nullptr) return d->epilogue;
  return d->epilogue == VP_EPI_BIAS_QKNORM_ROPE ? EPI_QKNORM_AUX : EPI_GELU_AUX;
}

// main_tiles > 0: launch only the first main_tiles tiles of the grouped order (tail mode's main launch)
static int gemm_bf16_launch(const vp_gemm_desc* d, void* stream, int main_tiles) {
  if (d == nullptr || d->A == nullptr || d->W[0] == nullptr || d->C == nullptr) return VP_ERR_ARG;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || (d->K % 8) != 0 || (d->N % 8) != 0) return VP_ERR_ARG;
  if (d->lda < d->K || d->ldc < d->N || (d->lda % 8) != 0 || (d->ldc % 8) != 0) return VP_ERR_ARG;
  if (d->rows_per_group <= 0) return VP_ERR_ARG;
  const int nsegs = d->W[2] ? 3 : (d->W[1] ? 2 : 1);
  if (d->n_seg <= 0 || d->n_seg * nsegs != d->N) return VP_ERR_ARG;
  if (d->epilogue < VP_EPI_BIAS || d->epilogue > VP_EPI_GELU_BWD || d->epilogue == VP_EPI_BIAS_GELU_MXFP8)
    return VP_ERR_ARG;
  if (check_aux(d) != VP_OK) return VP_ERR_ARG;
  if (d->epilogue == VP_EPI_BIAS_QKNORM_ROPE) {
    if (nsegs != 3 || (d->n_seg % 64) != 0 || d->rows_per_group != d->M || d->tokens_per_batch <= 0) return VP_ERR_ARG;
    for (int s = 0; s < 2; ++s)
      if (d->qk_ln_w[s] == nullptr || d->qk_ln_b[s] == nullptr) return VP_ERR_ARG;
    if ((d->rope_cos == nullptr) != (d->rope_sin == nullptr)) return VP_ERR_ARG;
  }
  if (d->epilogue == VP_EPI_GATED) {
    if (d->R == nullptr || d->gate == nullptr || d->gate_text == nullptr || d->tokens_per_batch <= 0) return VP_ERR_ARG;
    if ((d->ldr % 8) != 0 || (d->gate_bstride % 8) != 0) return VP_ERR_ARG;
    if (d->inject != nullptr && ((d->inject_ld % 8) != 0 || (d->inject_bstride % 8) != 0)) return VP_ERR_ARG;
  }
  if (d->epilogue == VP_EPI_BIAS_ADDROWS && (d->addrows == nullptr || (d->addrows_ld % 8) != 0)) return VP_ERR_ARG;
  MxExt mx = {};
  mx.group = gemm_group(d);
  if (d->a_tail_k != 0) {
    // the per-segment A tail (unfused LoRA): the default main loop only, on whole K-tiles and whole-tile segments
    static const void* const k13t[10] = {(const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS, false, true>,
                                        nullptr, nullptr,
                                        (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_GATED, false, true>,
                                        nullptr, nullptr,
                                        (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS_QKNORM_ROPE, false, true>,
                                        nullptr,
                                        (const void*)gemm_bf16_kernel<13, false, 4, EPI_QKNORM_AUX, false, true>,
                                        nullptr};
    static bool attr_t = false;
    if (!attr_t) {
      for (const void* f : k13t)
        if (f != nullptr) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      attr_t = true;
    }
    if (d->a_tail_k < 0 || d->a_tail_k >= d->K || (d->a_tail_k % BK) != 0) return VP_ERR_ARG;
    const int ki = kernel_index(d);
    int64_t amax = 0;
    for (int s = 0; s < nsegs; ++s) {
      if (d->a_tail_off[s] < 0 || (d->a_tail_off[s] % 8) != 0) return VP_ERR_ARG;
      amax = d->a_tail_off[s] > amax ? d->a_tail_off[s] : amax;
    }
    if (d->lda < d->K + amax) return VP_ERR_ARG;  // every segment's tail columns inside the rows
    const char* e = vp_knob(VPK_GEMM_VARIANT);
    if ((e != nullptr && atoi(e) != 13) || (d->K % BK) != 0 || d->K < 8 * BK || (nsegs > 1 && (d->n_seg % BN) != 0) ||
        k13t[ki] == nullptr || (int64_t)BM * d->lda * 2 >= ((int64_t)1 << 31) ||
        (int64_t)d->n_seg * d->K * 2 >= ((int64_t)1 << 31))
      return VP_ERR_UNSUPPORTED;
    const int ttiles = ((d->M + BM - 1) / BM) * (d->N / BN);
    void* args[] = {(void*)d, (void*)&mx};
    const hipError_t le = hipLaunchKernel(k13t[ki], dim3(main_tiles > 0 ? min(main_tiles, ttiles) : ttiles),
                                          dim3(NTHREADS), args, LDS_BYTES, (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
    VP_CHECK_LAUNCH();
    return VP_OK;
  }
  // main loops: 13 = the quadrant-phase pipeline with the two wave groups staggered and each slot's fragment reads
  // issued before its DMA, instantiated per epilogue kind (default: +3.6-5.2 % over 11 on every config-2 shape and
  // 283.7 against 295.4 ms of GEMM per step, profiles/r04_gemm13_ab.log), 11 = the same with the reads after the DMA
  // (VP_GEMM_VARIANT=11, A/B), 5 = the unstaggered pipeline (A/B; also K < 512), 1 = the 2-stage ring (K % 64 != 0,
  // e.g. the patch-embed im2col K = 132)
  static const void* const k11[10] = {
      (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_BIAS>, (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_BIAS_GELU>,
      (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_BIAS_SCALE>, (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_GATED>,
      (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_BIAS_ADDROWS>, nullptr,
      (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_BIAS_QKNORM_ROPE>,
      (const void*)gemm_bf16_kernel<11, false, 4, VP_EPI_GELU_BWD>,
      nullptr, nullptr};
  static const void* const k13[10] = {
      (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS>, (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS_GELU>,
      (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS_SCALE>, (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_GATED>,
      (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS_ADDROWS>, nullptr,
      (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS_QKNORM_ROPE>,
      (const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_GELU_BWD>,
      (const void*)gemm_bf16_kernel<13, false, 4, EPI_QKNORM_AUX>,
      (const void*)gemm_bf16_kernel<13, false, 4, EPI_GELU_AUX>};
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* f : k13)
      if (f != nullptr) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<5>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    for (const void* f : k11)
      if (f != nullptr) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_set = true;
  }
  const char* e = vp_knob(VPK_GEMM_VARIANT);  // the knob table (vp_set_knob): tests switch it between launches
  int variant = e != nullptr ? atoi(e) : 13;
  if (variant != 1 && variant != 5 && variant != 11 && variant != 12 && variant != 13 && variant != 20 && variant != 30)
    variant = 13;
  // the rejected A/B loops 12, 20, 30 (profiles/r04_gemm_v12_ab_rejected.log, r04_gemm_v30_ab_rejected.log) were
  // pruned in round 6: naming one is VP_ERR_UNSUPPORTED
  if (!vp_gemm_variant_built(variant)) return VP_ERR_UNSUPPORTED;
  // the quadrant pipeline adds 32-bit in-tile source offsets to a 64-bit tile base (A) / segment base (W)
  const bool w32 = (int64_t)d->n_seg * d->K * 2 < ((int64_t)1 << 31);
  const bool tile32 = (int64_t)BM * d->lda * 2 < ((int64_t)1 << 31) && w32;
  if (variant != 1 && ((d->K % BK) != 0 || !tile32)) variant = 1;  // needs whole K-tiles
  if ((variant == 11 || variant == 13) && d->K < 8 * BK) variant = 5;  // the staggered prologue assumes >= 8 K-tiles
  const int all_tiles = ((d->M + BM - 1) / BM) * ((d->N + BN - 1) / BN);
  const int tiles = main_tiles > 0 ? min(main_tiles, all_tiles) : all_tiles;
  const int ki = kernel_index(d);
  if (variant == 11 && k11[ki] == nullptr) return VP_ERR_UNSUPPORTED;
  if (variant == 13) {
    void* args[] = {(void*)d, (void*)&mx};
    const void* const* kt = k13;
    const hipError_t le = hipLaunchKernel(kt[ki], dim3(tiles), dim3(NTHREADS), args, LDS_BYTES,
                                          (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
  } else if (variant == 11) {
    void* args[] = {(void*)d, (void*)&mx};
    const hipError_t le = hipLaunchKernel(k11[ki], dim3(tiles), dim3(NTHREADS), args, LDS_BYTES,
                                          (hipStream_t)stream);
    if (le != hipSuccess) return (int)le;
  } else if (variant == 5) {
    hipLaunchKernelGGL(gemm_bf16_kernel<5>, dim3(tiles), dim3(NTHREADS), LDS_BYTES, (hipStream_t)stream, *d, mx);
  } else {
    hipLaunchKernelGGL(gemm_bf16_kernel<1>, dim3(tiles), dim3(NTHREADS), LDS_BYTES, (hipStream_t)stream, *d, mx);
  }
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_gemm_bf16(const vp_gemm_desc* d, void* stream) { return gemm_bf16_launch(d, stream, 0); }

extern "C" int64_t vp_gemm_bf16_workspace_bytes(const vp_gemm_desc* d) {
  if (d == nullptr) return -1;
  return split_plan(d).ws_bytes;
}

extern "C" int vp_gemm_bf16_ws(const vp_gemm_desc* d, void* workspace, int64_t workspace_bytes, void* stream) {
  if (d == nullptr) return VP_ERR_ARG;
  const SplitPlan p = split_plan(d);
  if (p.nsplit < 2) return vp_gemm_bf16(d, stream);
  if (workspace == nullptr || workspace_bytes < p.ws_bytes || ((uintptr_t)workspace & 15) != 0) return VP_ERR_ARG;
  // the same argument checks as the unsplit launch (a zero-tile dry run is not possible: validate by hand)
  if (d->A == nullptr || d->W[0] == nullptr || d->C == nullptr || d->M <= 0 || d->N <= 0 || (d->N % 8) != 0 ||
      d->lda < d->K || d->ldc < d->N || (d->lda % 8) != 0 || (d->ldc % 8) != 0 || d->rows_per_group <= 0)
    return VP_ERR_ARG;
  const int nsegs = d->W[2] ? 3 : (d->W[1] ? 2 : 1);
  if (d->n_seg <= 0 || d->n_seg * nsegs != d->N) return VP_ERR_ARG;
  if (d->epilogue == VP_EPI_BIAS_ADDROWS && (d->addrows == nullptr || (d->addrows_ld % 8) != 0)) return VP_ERR_ARG;
  if (check_aux(d) != VP_OK) return VP_ERR_ARG;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_set = true;
  }
  MxExt mx = {};
  mx.ws = (float*)workspace;
  mx.kchunk = p.kchunk;
  mx.nsplit = p.nsplit;
  const int tiles = ((d->M + BM - 1) / BM) * ((d->N + BN - 1) / BN);
  if (p.tail > 0) {
    // tail mode: every tile but the last p.tail as one main launch (the validation and main loop of vp_gemm_bf16),
    // the tail tiles as split-K workgroups into compact partials, then their reduce + epilogue
    const int rc = gemm_bf16_launch(d, stream, tiles - p.tail);
    if (rc != VP_OK) return rc;
    mx.t_base = tiles - p.tail;
    mx.tail = 1;
    mx.group = gemm_group(d);
    hipLaunchKernelGGL((gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS, true>), dim3(p.tail * p.nsplit),
                       dim3(NTHREADS), LDS_BYTES, (hipStream_t)stream, *d, mx);
    VP_CHECK_LAUNCH();
    hipLaunchKernelGGL(gemm_tail_reduce_kernel, dim3(p.tail * 32), dim3(256), 0, (hipStream_t)stream, *d,
                       (const float*)workspace, tiles - p.tail, p.nsplit, mx.group);
    VP_CHECK_LAUNCH();
    return VP_OK;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<13, false, 4, VP_EPI_BIAS, true>), dim3(tiles * p.nsplit), dim3(NTHREADS),
                     LDS_BYTES, (hipStream_t)stream, *d, mx);
  VP_CHECK_LAUNCH();
  const int64_t work = (int64_t)d->M * (d->N / 8);
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *d, (const float*)workspace, p.nsplit);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

extern "C" int vp_gemm_mx_fp8(const vp_gemm_mx_desc* x, void* stream) {
  if (x == nullptr) return VP_ERR_ARG;
  const vp_gemm_desc* d = &x->base;
  if (d->A == nullptr || d->W[0] == nullptr || d->C == nullptr || x->a_scale == nullptr || x->w_scale[0] == nullptr)
    return VP_ERR_ARG;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || (d->K % 128) != 0 || (d->N % 256) != 0) return VP_ERR_ARG;
  if (d->lda < d->K || (d->lda % 16) != 0 || d->rows_per_group <= 0) return VP_ERR_ARG;
  const int nsegs = d->W[2] ? 3 : (d->W[1] ? 2 : 1);
  if (d->n_seg <= 0 || d->n_seg * nsegs != d->N || (d->n_seg % 256) != 0) return VP_ERR_ARG;
  for (int s = 0; s < nsegs; ++s)
    if (x->w_scale[s] == nullptr) return VP_ERR_ARG;
  if (d->epilogue < VP_EPI_BIAS || d->epilogue > VP_EPI_BIAS_GELU_MXFP8 || d->aux != nullptr) return VP_ERR_ARG;
  if (d->epilogue == VP_EPI_BIAS_GELU_MXFP8) {
    if (x->c_scale == nullptr || (d->ldc % 16) != 0 || d->ldc < d->N || d->rows_per_group != d->M) return VP_ERR_ARG;
  } else if (d->ldc < d->N || (d->ldc % 8) != 0) {
    return VP_ERR_ARG;
  }
  if (d->epilogue == VP_EPI_GATED) {
    if (d->R == nullptr || d->gate == nullptr || d->gate_text == nullptr || d->tokens_per_batch <= 0) return VP_ERR_ARG;
    if ((d->ldr % 8) != 0 || (d->gate_bstride % 8) != 0) return VP_ERR_ARG;
    if (d->inject != nullptr && ((d->inject_ld % 8) != 0 || (d->inject_bstride % 8) != 0)) return VP_ERR_ARG;
  }
  if (d->epilogue == VP_EPI_BIAS_ADDROWS && (d->addrows == nullptr || (d->addrows_ld % 8) != 0)) return VP_ERR_ARG;
  // 32-bit DMA source offsets
  if ((int64_t)d->M * d->lda >= ((int64_t)1 << 31) || (int64_t)d->n_seg * d->K >= ((int64_t)1 << 31)) return VP_ERR_ARG;
  // instantiated per epilogue kind for the block's fp8 GEMMs (QKV: BIAS, FF1: GELU_MXFP8, FF2: GATED); the others
  // take the runtime switch of variant 5
  static const void* const kf[6] = {(const void*)gemm_bf16_kernel<5, true, 4, VP_EPI_BIAS>, nullptr, nullptr,
                                    (const void*)gemm_bf16_kernel<5, true, 4, VP_EPI_GATED>, nullptr,
                                    (const void*)gemm_bf16_kernel<5, true, 4, VP_EPI_BIAS_GELU_MXFP8>};
  // 13 (default, nk >= 8): the staggered read-first pipeline of the bf16 default on the e4m3 operands — config 5's
  // fp8 GEMMs 446.7 against 466.3 ms per step with 5 (profiles/r04_c5_gemm8_ab.log); VP_GEMM8_VARIANT=5: the
  // unstaggered loop (A/B; also nk < 8)
  static const void* const kf13[6] = {(const void*)gemm_bf16_kernel<13, true, 4, VP_EPI_BIAS>, nullptr, nullptr,
                                      (const void*)gemm_bf16_kernel<13, true, 4, VP_EPI_GATED>, nullptr,
                                      (const void*)gemm_bf16_kernel<13, true, 4, VP_EPI_BIAS_GELU_MXFP8>};
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<5, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES_FP8);
    for (const void* f : kf)
      if (f != nullptr) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES_FP8);
    for (const void* f : kf13)
      if (f != nullptr) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES_FP8);
    attr_set = true;
  }
  const char* e8 = vp_knob(VPK_GEMM8_VARIANT);  // (A/B knob)
  const bool use13 = (e8 == nullptr || atoi(e8) != 5) && d->K / 128 >= 8 && kf13[d->epilogue] != nullptr;
  MxExt mx = {};  // no split; the grouped tile order of the bf16 path (VP_GEMM_GROUP, default 4)
  mx.group = gemm_group(d);
  mx.a_scale = (const uint8_t*)x->a_scale;
  for (int s = 0; s < 3; ++s) mx.w_scale[s] = (const uint8_t*)x->w_scale[s];
  mx.c_scale = (uint8_t*)x->c_scale;
  const int tiles = ((d->M + BM - 1) / BM) * (d->N / BN);
  const void* fn = use13 ? kf13[d->epilogue]
                   : kf[d->epilogue] != nullptr ? kf[d->epilogue] : (const void*)gemm_bf16_kernel<5, true>;
  void* args[] = {(void*)d, (void*)&mx};
  const hipError_t le = hipLaunchKernel(fn, dim3(tiles), dim3(NTHREADS), args, LDS_BYTES_FP8, (hipStream_t)stream);
  if (le != hipSuccess) return (int)le;
  VP_CHECK_LAUNCH();
  return VP_OK;
}

// ---- MX quantiser: 8 elements per thread, 4 threads per 32-element block ----
__global__ __launch_bounds__(256) void mx_quantize_kernel(const bf16* __restrict__ x, int64_t ld_in,
                                                          uint8_t* __restrict__ q, int64_t ld_out,
                                                          uint8_t* __restrict__ scales, int rows, int K) {
  const int cpr = K / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = i / cpr;
  const int c = (int)(i - r * cpr);
  if (r >= rows) return;  // whole 4-lane groups leave together (cpr % 4 == 0)
  const bf16x8 v = *(const bf16x8*)(x + r * ld_in + c * 8);
  float f[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = bf2f(v[e]);
  uint8_t sb;
  const u32x2 pk = mx_quantize_quarter(f, sb);
  *(u32x2*)(q + r * ld_out + c * 8) = pk;
  if ((c & 3) == 0) scales[mx_scale_off(r, c >> 2, K)] = sb;
}

extern "C" int64_t vp_mx_scale_bytes(int64_t rows, int64_t K) { return ((rows + 255) / 256) * (K / 128) * 1024; }

extern "C" int vp_mx_quantize_bf16(const void* x, int64_t ld_in, void* q, int64_t ld_out, void* scales, int32_t rows,
                                   int32_t K, void* stream) {
  if (!x || !q || !scales || rows <= 0 || K <= 0 || (K % 128) || ld_in < K || ld_out < K || (ld_in % 8) ||
      (ld_out % 8))
    return VP_ERR_ARG;
  const int64_t n = (int64_t)rows * (K / 8);
  hipLaunchKernelGGL(mx_quantize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ld_in, (uint8_t*)q, ld_out, (uint8_t*)scales, rows, K);
  VP_CHECK_LAUNCH();
  return VP_OK;
}

#if VP_DIAG  // diagnostic build only (include/vp_hip_diag.h)
// ---- layout self-test: one wave, one block-scaled MFMA ----
__global__ __launch_bounds__(64) void mx_probe_kernel(const uint8_t* A, const uint8_t* B, const uint8_t* sa,
                                                      const uint8_t* sb, float* C) {
  const int l = threadIdx.x;
  // lane l feeds K-chunks l/16 and l/16 + 4 (16 bytes each) of row l % 16
  i32x8 a, b;
  u32x4* ha = (u32x4*)&a;
  u32x4* hb = (u32x4*)&b;
  ha[0] = *(const u32x4*)(A + (l & 15) * 128 + (l >> 4) * 16);
  ha[1] = *(const u32x4*)(A + (l & 15) * 128 + ((l >> 4) + 4) * 16);
  hb[0] = *(const u32x4*)(B + (l & 15) * 128 + (l >> 4) * 16);
  hb[1] = *(const u32x4*)(B + (l & 15) * 128 + ((l >> 4) + 4) * 16);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, (int)sa[l], 0, (int)sb[l]);
#pragma unroll
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

extern "C" int vp_mx_mfma_probe(const void* A, const void* B, const void* sa, const void* sb, float* C, void* stream) {
  if (!A || !B || !sa || !sb || !C) return VP_ERR_ARG;
  hipLaunchKernelGGL(mx_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t*)A,
                     (const uint8_t*)B, (const uint8_t*)sa, (const uint8_t*)sb, C);
  VP_CHECK_LAUNCH();
  return VP_OK;
}
#endif
