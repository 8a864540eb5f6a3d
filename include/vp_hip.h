/* vp_hip.h — C ABI of the MI355X (gfx950) VideoPainter denoising hot path (libvp_hip.so).
 *
 * Every entry point takes plain device pointers, sizes and element strides, plus the HIP stream to launch on
 * (`void* stream` = hipStream_t; NULL = default stream).  No torch types cross this boundary.
 *   - Ownership: the caller allocates every output and workspace; no entry point allocates or frees.
 *   - Errors: return 0 on success, VP_ERR_* (>= 1000) for an argument error detected on the host, or the
 *     hipError_t of the failed launch.  Nothing is printed.
 *   - Threading: stateless and re-entrant; each call is asynchronous on `stream` and may be captured in a graph.
 *   - Storage dtype: bf16 (`__bf16` / torch.bfloat16) unless stated; accumulation is fp32.
 *
 * Each entry point cites the reference interface it replaces (paths relative to
 * /root/reference/diffusers/src/diffusers/, abbreviated DF/).  The Python host mirror that binds them by ctypes is
 * videopainter_amd/_native.py; the reference-side binding a maintainer would add is shown in INTEGRATION.md.
 */
#ifndef VP_HIP_H
#define VP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP_OK 0
#define VP_ERR_ARG 1000      /* invalid size / stride / pointer combination */
#define VP_ERR_UNSUPPORTED 1001

/* ABI version: bump when any struct layout or signature below changes. */
#define VP_ABI_VERSION 20
int vp_abi_version(void);
/* "<sha256 of sources + flags>:<sha256 of the compiler version>" of the build (no reference counterpart) */
const char* vp_build_digest(void);
/* A/B switches of the library (kernel-variant selection only, never numerics of the default path; DESIGN_LOG.md §5):
 * VP_GEMM_VARIANT, VP_GEMM_NO_TAIL, VP_GEMM_GROUP, VP_GEMM8_VARIANT, VP_ATTN_BOUNDED_MODE, VP_ATTN_UNBOUNDED_MODE,
 * VP_ATTN_NO_SPLIT, VP_ATTN8_VARIANT, VP_T5_ATTN, VP_CONV_HOIST, VP_CONV_PIPE,
 * VP_ATTN_BWD_VARIANT, VP_ATTN_TAIL, VP_ATTN_PERSIST.  Each is read from the environment
 * once, when the library is loaded; afterwards only vp_set_knob changes it (value NULL = unset), e.g. a test that
 * runs two variants on the same operands.  Returns VP_ERR_ARG for an unknown name or a value over 31 bytes.  Host
 * only; not thread-safe against launches in flight on other host threads.  (ABI 14.) */
int vp_set_knob(const char* name, const char* value);
/* sizeof of the descriptor structs as compiled into the library: out[0..6] = gemm, attn, dpm, gemm_mx, attn_fp8,
 * conv3d, attn_bwd (ABI check) */
void vp_struct_sizes(int64_t* out);

/* ---------------------------------------------------------------------------------------------------------------
 * GEMM  C = epilogue(A · Wᵀ)   — replaces every nn.Linear / patch-embed conv on the path:
 *   attn.to_q/to_k/to_v/to_out.0 (DF/models/attention_processor.py:2132-2134,2202), FeedForward net.0.proj + GELU
 *   and net.2 (DF/models/attention.py:1177,1191; activations.py:65-90), the gated residuals
 *   (DF/models/transformers/cogvideox_transformer_3d.py:169-170,181-182), the branch injection (:596-609), the
 *   patch-embed conv + text_proj + pos-emb (DF/models/embeddings.py:400-454), the branch zero-linears
 *   (DF/models/branch_cogvideox.py:415-421) and proj_out (cogvideox_transformer_3d.py:624).
 * A: bf16 [M, K] (row stride lda); W: up to 3 weight segments, each bf16 [n_seg, K] (nn.Linear layout), columns
 * [s*n_seg, (s+1)*n_seg) of C come from segment s (fused QKV without packing the weights).  K % 8 == 0
 * (a K tail is zero-filled on the device).
 * Output row remap: C row of GEMM row m = (m / rows_per_group) * group_stride + row_offset + (m % rows_per_group).
 * ------------------------------------------------------------------------------------------------------------- */
enum {
  VP_EPI_BIAS = 0,        /* C = rnd(acc + bias)                                                            */
  VP_EPI_BIAS_GELU = 1,   /* C = rnd(gelu_tanh(rnd(acc + bias)))                                             */
  VP_EPI_BIAS_SCALE = 2,  /* C = rnd(rnd(acc + bias) * alpha)            (branch conditioning_scale)         */
  VP_EPI_GATED = 3,       /* C = rnd(R + rnd(gate * rnd(acc + bias))) [then rnd(C + inject) on video rows]   */
  VP_EPI_BIAS_ADDROWS = 4, /* C = rnd(rnd(acc + bias) + addrows[(m % rows_per_group) + addrows_offset, n])  */
  /* 5 = VP_EPI_BIAS_GELU_MXFP8 (vp_gemm_mx_fp8 only, below) */
  VP_EPI_BIAS_QKNORM_ROPE = 6, /* fused QKV projection: segments 0 / 1 (q / k): every 64-column head of
                               * y = rnd(acc + bias) -> rnd(LayerNorm64(y; qk_ln_w[s], qk_ln_b[s], qk_eps[s])), then on
                               * video rows (m % tokens_per_batch >= text_len) the interleaved-pair RoPE from
                               * rope_cos / rope_sin (fp32 [tokens_per_batch - text_len][64]) -> rnd; segment 2 (v) as
                               * VP_EPI_BIAS.  = vp_gemm_bf16 + vp_head_norm_rope_bf16 on q and k, bit for bit. */
  VP_EPI_GELU_BWD = 7     /* C = rnd(rnd(acc + bias) * gelu_tanh'(Z[m, n])), Z = R (bf16 [M][N], row m at ldr; no
                           * row remap): the FeedForward's dgrad through its GELU — the dgrad GEMM of net.2 followed
                           * by vp_gelu_bwd_bf16, bit for bit, in one pass (ABI 17) */
};

typedef struct vp_gemm_desc {
  int32_t M, N, K, epilogue;
  const void* A;
  int64_t lda;
  const void* W[3];
  const void* bias[3]; /* bf16 [n_seg] per segment, or NULL */
  int32_t n_seg, pad0;
  void* C;
  int64_t ldc;
  int32_t rows_per_group, pad1;
  int64_t group_stride, row_offset;
  float alpha;
  int32_t pad2;
  /* VP_EPI_GATED: rows are (batch, token) of a [B, tokens_per_batch, N] stream; text tokens (token < text_len)
   * take gate_text[b], video tokens gate[b]; gate vectors bf16 [N] at batch stride gate_bstride.  R may alias C. */
  const void* R;
  int64_t ldr;
  const void* gate;
  const void* gate_text;
  int64_t gate_bstride;
  int32_t tokens_per_batch, text_len;
  /* optional branch injection on video rows: C += inject[b, token - text_len, :] where inject_mask[b, v] == 0
   * (or always when inject_mask == NULL) */
  const void* inject;
  int64_t inject_ld, inject_bstride;
  const uint8_t* inject_mask;
  int64_t inject_mask_bstride;
  /* VP_EPI_BIAS_ADDROWS */
  const void* addrows;
  int64_t addrows_ld, addrows_offset;
  /* VP_EPI_BIAS_QKNORM_ROPE (norm_q / norm_k are LayerNorm(64) with affine bf16 weights; rows_per_group == M) */
  const void* qk_ln_w[2];
  const void* qk_ln_b[2];
  float qk_eps[2];
  const float* rope_cos; /* NULL: no RoPE (image_rotary_emb None) */
  const float* rope_sin;
  /* Per-segment A tail (unfused LoRA, PEFT's y = x W^T + s (x A^T) B^T as ONE GEMM on K-augmented operands;
   * DF/loaders/lora_pipeline.py:2632-2705 load_lora_into_transformer, infer/inpaint.py:310-316): a_tail_k > 0 splits
   * K at a_tail_k; for k >= a_tail_k, segment s reads A column k + a_tail_off[s] (its own rank block of
   * T = x [A_0; A_1; ...]^T stored after x in the same rows), so every weight segment carries only its own rank
   * (W_s = [W0_s | s B_s], K = a_tail_k + r).  Needs K % 64 == a_tail_k % 64 == 0, n_seg % 256 == 0 with more than one
   * segment, the default
   * main loop (VP_ERR_UNSUPPORTED otherwise) and epilogue BIAS, GATED or BIAS_QKNORM_ROPE.  0: no tail.  (ABI 14.) */
  int32_t a_tail_k, pad3;
  int64_t a_tail_off[3];
  /* VP_EPI_BIAS_QKNORM_ROPE with a separable 3D RoPE table (ABI 16; NULL rope_ax[0]: the full table): rope_ax = the
   * per-axis factors of rope_cos / rope_sin — cos_t, sin_t [F][16], cos_y, sin_y [Hh][24], cos_x, sin_x [Ww][24] fp32,
   * exact slices of the full table (CogVideoX's 3D RoPE, DF/models/embeddings.py:457-530: dims 0-15 by frame, 16-39 by
   * row, 40-63 by column) — with rope_hw = Hh * Ww, rope_w = Ww and their division magics rope_mhw / rope_mw
   * (ceil(2^32 / d)); the epilogue reads those rows (a few KB, cache-resident) instead of the token's row of the
   * [F*Hh*Ww][64] table: the same values, bit-identical output.  rope_cos / rope_sin stay set. */
  const float* rope_ax[6];
  int32_t rope_hw, rope_w;
  uint32_t rope_mhw, rope_mw;
  /* Optional second output for the training forward (ABI 17; NULL: none), bf16, row m of the GEMM at aux + m * ld_aux
   * (no row remap): VP_EPI_BIAS_GELU writes the pre-activation rnd(acc + bias) there (the GELU's backward input, so
   * no separate vp_gelu_bf16 pass); VP_EPI_BIAS_QKNORM_ROPE writes the pre-norm rnd(acc + bias) of segments 0 / 1
   * (q | k, columns [0, 2 n_seg)) there (the LayerNorm backward's input).  Other epilogues: VP_ERR_ARG. */
  void* aux;
  int64_t ld_aux;
} vp_gemm_desc;

int vp_gemm_bf16(const vp_gemm_desc* d, void* stream);

/* 1 when the GEMM main loop VP_GEMM_VARIANT = variant (1, 5, 11, 13 = the default; 12, 20, 30 only in a
 * VP_GEMM_EXTRA_VARIANTS build: the rejected A/B loops) is in this library, else 0.  Host-only.  vp_gemm_bf16 returns
 * VP_ERR_UNSUPPORTED for a variant outside the build.  (ABI 13.) */
int vp_gemm_variant_built(int variant);

/* Split-K form for GEMMs too small to fill the chip (fewer than 128 output tiles of 256 x 256, e.g. the T5 encoder's
 * projections at M = 2 x 226 token rows; reference callers: transformers T5EncoderModel, anyl.py:216-256): the K
 * range is cut into chunks of >= 512, each (tile, chunk) workgroup writes its fp32 partial tile to `workspace`, and a
 * reduce pass sums the chunks in a fixed order (deterministic) and applies the epilogue (VP_EPI_BIAS, _GELU, _SCALE,
 * _BIAS_ADDROWS; others never split).  vp_gemm_bf16_workspace_bytes: bytes this descriptor needs (0: no split, and
 * vp_gemm_bf16_ws then runs vp_gemm_bf16).  vp_gemm_bf16 never splits. */
int64_t vp_gemm_bf16_workspace_bytes(const vp_gemm_desc* d);
int vp_gemm_bf16_ws(const vp_gemm_desc* d, void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * MX-FP8 (OCP e4m3 elements, one E8M0 power-of-two scale per 32 consecutive K elements) — the fp8 path of
 * BASELINE config 5.  The same projections as vp_gemm_bf16 (FeedForward net.0.proj / net.2,
 * DF/models/attention.py:1177,1191), on gfx950's block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4: 2x the
 * bf16 MFMA rate; the hardware applies the scales, so the accumulator is the dequantised dot product).
 *
 * Data layout of an MX tensor with R rows and K columns (K % 128 == 0):
 *   elements: uint8 e4m3 [R][K] at row stride ld (bytes);
 *   scales:   uint8 E8M0 (value 2^(s-127)) in 256-row x 128-column tiles of 1 KiB, tile (R/256, K/128) at
 *             byte ((r >> 8) * (K / 128) + (k >> 7)) * 1024, and inside it block b = (k >> 5) & 3 of row r at
 *             b * 256 + (r & 15) * 16 + ((r >> 4) & 15) — one GEMM K-step's scales are one contiguous 1 KiB
 *             LDS-DMA, and a lane's scales for 4 consecutive 16-row fragments are one aligned dword.
 *             Size: ceil(R / 256) * (K / 128) * 1024 bytes.
 * Quantisation of a 32-element block x: s = ceil(log2(amax|x| / 448)) (clamped to [-127, 127]),
 * q = RNE_e4m3(x * 2^-s) (|q| <= 448, no clipping), scale byte s + 127 (0 for an all-zero block).
 * ------------------------------------------------------------------------------------------------------------- */
#define VP_MX_BLOCK 32
int64_t vp_mx_scale_bytes(int64_t rows, int64_t K);

/* rows x K bf16 (row stride ld_in elements) -> MX e4m3 (row stride ld_out bytes) + scales (layout above) */
int vp_mx_quantize_bf16(const void* x, int64_t ld_in, void* q, int64_t ld_out, void* scales, int32_t rows, int32_t K,
                        void* stream);

/* out = epilogue(A · Wᵀ) with A and W in MX-FP8.  base: as vp_gemm_desc with A / W[] pointing at the e4m3
 * elements (lda in BYTES; W rows are K bytes), epilogues VP_EPI_BIAS .. VP_EPI_BIAS_ADDROWS writing bf16 C, or
 * VP_EPI_BIAS_GELU_MXFP8: C = MX-quantise(rnd(gelu_tanh(rnd(acc + bias)))) written as e4m3 [M][N] (ldc in bytes)
 * plus c_scale (the FF1 -> FF2 hand-off stays in fp8).  K % 128 == 0, N % 256 == 0. */
#define VP_EPI_BIAS_GELU_MXFP8 5
typedef struct vp_gemm_mx_desc {
  vp_gemm_desc base;
  const void* a_scale;
  const void* w_scale[3];
  void* c_scale;
} vp_gemm_mx_desc;

int vp_gemm_mx_fp8(const vp_gemm_mx_desc* d, void* stream);


/* ---------------------------------------------------------------------------------------------------------------
 * Flash attention forward, head_dim 64, non-causal, no mask — replaces F.scaled_dot_product_attention in
 * CogVideoXAttnProcessor2_0 (DF/models/attention_processor.py:2177-2197) and CogVideoXAttnProcessor2_0_resample
 * (:2283-2290; the doubled K/V is passed as two segments instead of being concatenated).
 * Element (b, h, n, d) of Q is Q[b*q_sb + n*q_sn + h*64 + d]; likewise K, V, K2, V2, O.
 * O = rnd(out_scale * rnd(softmax(scale Q Kᵀ) V)) (+ O_old when accumulate) — the prev-clip blend.
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct vp_attn_desc {
  int32_t B, H, Nq, head_dim;
  const void* Q;
  int64_t q_sb, q_sn;
  const void* K;
  const void* V;
  int64_t k_sb, k_sn, v_sb, v_sn;
  int32_t Nk, Nk2;
  const void* K2; /* optional second key/value segment (Nk2 == 0: none) */
  const void* V2;
  int64_t k2_sb, k2_sn, v2_sb, v2_sn;
  void* O;
  int64_t o_sb, o_sn;
  float scale, out_scale;
  int32_t accumulate;
  int32_t flags; /* VP_ATTN_BOUNDED_SCORES: the caller guarantees |scale * q.k| * log2(e) <= VP_ATTN_SCORE_BOUND for
                    every (query, key) pair, so the kernel runs without a reference point (p2: exact, bf16/fp32 hold
                    2^+-60 and O / l is invariant to the reference point).  CogVideoX's qk-LayerNorm gives the bound
                    from the norm weights: videopainter_amd.kernels.score_bound_log2.  Without the flag (any
                    scores): p2a, the same pipeline with an anchored reference point, plus a re-run of the blocks it
                    flags by the exact anchored 16x16x32 kernel — which needs the workspace of
                    vp_attention_fwd_bf16_ws (without one the 16x16x32 kernel runs alone). */
  float* lse;     /* optional fp32 [B, H, Nq]: per query log2-sum-exp2 of the scaled log2-unit scores (m + log2 l), the
                     softmax statistics vp_attention_bwd_bf16 recomputes P from (bf16 kernel only; NULL: not written) */
  const int32_t* k2_full; /* optional int32 [B] (device), a hint: segment-2 rows n >= k2_full[b] of V2 are zero
                             (the caller guarantees it), so those keys enter only the row sums — the resample
                             processor's null keys, partitioned behind its masked keys by vp_partition_rows_index.
                             The 16x16x32 kernels skip their V^T DMA, reads and PV products for whole tiles past
                             k2_full[b]; the other kernels read the zeros.  NULL: no hint. */
  const int32_t* k2_len;  /* optional int32 [B] (device): segment 2 holds only its first min(k2_len[b], Nk2) keys for
                             batch row b (the rest are not read) — the resample processor's masked rows when its null
                             keys are summed in closed form (vp_null_key_mass).  NULL: Nk2 keys for every row. */
  const float* l_extra;   /* optional fp32 [B, H, Nq] (device): log2 of extra row-sum mass per query, in the kernel's
                             score units (scale * log2 e * q.k), added to the softmax denominator — the null keys'
                             total exp2(score) (their values are zero).  -inf: none.  NULL: nothing added.
                             k2_len / l_extra are taken by the s16 / a16 and the p2 / p2a kernels, k2_full by the
                             16x16x32 kernels only (a k2_full launch runs s16 / a16). */
} vp_attn_desc;
#define VP_ATTN_BOUNDED_SCORES 1
#define VP_ATTN_SCORE_BOUND 60.0f

int vp_attention_fwd_bf16(const vp_attn_desc* d, void* stream);

/* The same with a caller-provided workspace for the grid-tail split: when the last round of workgroups would run
 * on a mostly idle chip (blocks mod resident slots <= half the slots), those blocks run as several key-range
 * workgroups each plus a merge pass.  vp_attention_workspace_bytes: bytes needed for this descriptor (0: no split;
 * -1: invalid descriptor).  A null or too small workspace runs the unsplit grid. */
int64_t vp_attention_workspace_bytes(const vp_attn_desc* d);
int vp_attention_fwd_bf16_ws(const vp_attn_desc* d, void* workspace, int64_t workspace_bytes, void* stream);

/* 1 when the attention kernel variant `name` (the values of the A/B environment switches VP_ATTN_BOUNDED_MODE /
 * VP_ATTN_UNBOUNDED_MODE: "p2", "p2a", "s16", "a16", and with a VP_ATTN_EXTRA_VARIANTS build "lazy", "w32", "w64",
 * "w64f", "s16i", "p1"; "fp8:N" for the fp8 kernel's VP_ATTN8_VARIANT = N: 2 and 3, and 1 and 4 with that build) is
 * in this library, else 0.  Host-only.  A launch that names a variant outside the build returns VP_ERR_UNSUPPORTED. */
int vp_attention_variant_built(const char* name);

/* fp8 attention (BASELINE config 5 "attn + FFN in fp8"; same math as vp_attention_fwd_bf16, single K/V segment).
 * base.Q / base.K: e4m3 [B, N, H*64] written by vp_head_norm_rope_fp8 (strides in bytes, multiples of 16), each
 * carrying one power-of-two factor undone by the E8M0 bytes in qk_scale (bits 0-7: Q, bits 8-15: K; Q's factor
 * also includes scale * log2 e, so base.scale is ignored).  base.V: V^T e4m3 [B, H, 64, npad] and vs: its scales,
 * both from vp_v_pack_fp8.  base.O / out_scale / accumulate as in the bf16 kernel.  The probabilities P enter the
 * PV product (and the row sums) as e4m3 codes of p * 2^7 made by linear mantissa interpolation of exp2 (relative
 * error 3.2 % rms; env VP_ATTN8_VARIANT=1: exp2 + round-to-nearest e4m3, 2.7 %) — DESIGN_LOG.md §3.1. */
typedef struct vp_attn_fp8_desc {
  vp_attn_desc base;
  const void* vs;
  int32_t npad;     /* ceil(Nk / 64) * 64 */
  int32_t qk_scale; /* E8M0 bytes: Q | K << 8 */
} vp_attn_fp8_desc;

int vp_attention_fwd_fp8(const vp_attn_fp8_desc* d, void* stream);
/* The same with a workspace (ABI 20): the default kernel runs persistent — resident workgroups take the query blocks
 * by per-XCD ticket — when vp_attention_fp8_workspace_bytes (0: none needed, -1: invalid) bytes are given; a smaller
 * or NULL workspace runs one workgroup per block (same results, bit for bit). */
int64_t vp_attention_fp8_workspace_bytes(const vp_attn_fp8_desc* d);
int vp_attention_fwd_fp8_ws(const vp_attn_fp8_desc* d, void* workspace, int64_t workspace_bytes, void* stream);

/* V [B, N, H*64] bf16 (row stride v_sn, batch stride v_sb, elements) -> V^T e4m3 [B, H, 64, npad] with the keys of
 * every 64-key tile in MFMA K-slot order, plus one E8M0 scale per (d, 32 keys) (MX rule of vp_mx_quantize_bf16).
 * Padded keys are zero.  vp_v_pack_fp8_bytes returns the V^T bytes and reports npad and the scale bytes. */
int64_t vp_v_pack_fp8_bytes(int32_t B, int32_t H, int32_t N, int64_t* npad, int64_t* scale_bytes);
int vp_v_pack_fp8(const void* V, int64_t v_sb, int64_t v_sn, int32_t B, int32_t N, int32_t H, void* vt, void* vs,
                  void* stream);


/* ---------------------------------------------------------------------------------------------------------------
 * AdaLN-Zero modulate — CogVideoXLayerNormZero.forward (DF/models/normalization.py:373-379):
 * y = rnd(rnd(rnd(LN(x)) * rnd(1 + scale)) + shift) over rows of x [B, Ntok, D] (contiguous).  mod is the bf16
 * output of the block's norm linear, [B, 6D] = shift | scale | gate | enc_shift | enc_scale | enc_gate at batch
 * stride mod_bstride; text rows (token < text_len) use the enc_* chunks.  LN affine (ln_w, ln_b), eps.  y rows at
 * stride ldy (>= D, % 8 == 0: e.g. the first D columns of an unfused-LoRA projection's K-augmented operand; ABI 15).
 * ------------------------------------------------------------------------------------------------------------- */
int vp_adaln_modulate_bf16(const void* x, void* y, int64_t ldy, int32_t B, int32_t Ntok, int32_t D, int32_t text_len,
                           const void* ln_w, const void* ln_b, float eps, const void* mod, int64_t mod_bstride,
                           void* stream);
/* the same, writing the modulated rows as MX-FP8 (q: e4m3 [B*Ntok][D], scales: MX layout with R = B*Ntok, K = D)
 * — the input of the fp8 FeedForward (BASELINE config 5).  D % 128 == 0. */
int vp_adaln_modulate_mx_fp8(const void* x, void* q, void* scales, int32_t B, int32_t Ntok, int32_t D,
                             int32_t text_len, const void* ln_w, const void* ln_b, float eps, const void* mod,
                             int64_t mod_bstride, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Per-head LayerNorm(64) + interleaved-pair RoPE — attn.norm_q / norm_k (attention_processor.py:2143-2146) and
 * apply_rotary_emb on tokens >= text_len (:2149-2154; DF/models/embeddings.py:655-701).
 * x_in/x_out: [B, Ntok, H*64] with row stride ld_* and batch stride bs_*; may alias.  cos/sin fp32 [Ntok-text_len,
 * 64] (NULL: no RoPE).  Optional pre-mask (resample processor, attention_processor.py:2251-2256): if tok_mask !=
 * NULL the input row is first replaced by rnd(rnd(x * tok_mask[b, n]) * pre_scale) — LN of a zeroed row gives the
 * LN bias (the "null key").
 * ------------------------------------------------------------------------------------------------------------- */
int vp_head_norm_rope_bf16(const void* x_in, int64_t ld_in, int64_t bs_in, void* x_out, int64_t ld_out,
                           int64_t bs_out, int32_t B, int32_t Ntok, int32_t H, int32_t text_len, const void* ln_w,
                           const void* ln_b, float eps, const float* cos, const float* sin, const uint8_t* tok_mask,
                           int64_t mask_bstride, float pre_scale, const int32_t* dst_rows, void* stream);

/* The same LN(64) + RoPE, output e4m3 (x_bf16 * out_mul, clamped to +-448, RNE) for the fp8 attention; ld_out /
 * bs_out in bytes. */
int vp_head_norm_rope_fp8(const void* x_in, int64_t ld_in, int64_t bs_in, void* q_out, int64_t ld_out,
                          int64_t bs_out, int32_t B, int32_t Ntok, int32_t H, int32_t text_len, const void* ln_w,
                          const void* ln_b, float eps, const float* cos, const float* sin, float out_mul,
                          void* stream);

/* y[b, n, :] = rnd(rnd(x[b, n, :] * tok_mask[b, n]) * scale) — the masked value copy of the resample processor. */
/* (vp_head_norm_rope_bf16 and vp_mask_scale_rows_bf16 with dst_rows != NULL: output row n of batch b is written to
 * row dst_rows[b * Ntok + n] — the partition permutation of vp_partition_rows_index; a negative entry skips the row
 * (neither read nor written: the null rows when their keys are summed in closed form); the output must not alias the
 * input.) */

/* Stable partition of the resample processor's token mask (attention_processor.py:2244-2252): per batch row b,
 * counts[b] = #{n : mask[b, n] != 0}, dst_rows[b * N + n] = the rank of n among the set rows, or counts[b] + its
 * rank among the clear rows.  Written once per window (the mask is the same for every layer and step); the masked
 * keys / values then form the first counts[b] rows of the attention's second segment and the null keys (zero
 * values) the rest (vp_attn_desc.k2_full). */
int vp_partition_rows_index(const uint8_t* mask, int64_t mask_bstride, int32_t B, int32_t N, int32_t* dst_rows,
                            int32_t* counts, void* stream);

/* The resample processor's null keys in closed form (attention_processor.py:2244-2290 with mask 0: key LN(0) = the
 * norm_k bias beta, rotated by the position's RoPE on video rows; value 0).  With CogVideoX's separable 3D RoPE
 * (dims 0-15 by frame, 16-39 by row, 40-63 by column) a null key's score is S_t(t) + S_y(y) + S_x(x), so the
 * per-query sum of exp2(score) over all null keys factorises over the grid (DESIGN_LOG.md §3.0).
 * vp_mask_null_segments: the null pattern of the token mask [B, T + F*Hh*Ww] (text rows first), once per mask:
 *   segs (16-byte records, capacity B*F*Hh): per (b, t) the runs of equal consecutive rows that hold null keys —
 *   byte 0 = first row, 1 = end row, 2 = run count (<= 6, or 255: the row is scanned instead), bytes 4+2k / 5+2k =
 *   run k's [start, end) columns; meta int32 [B*F + B]: segments per (b, t), then the text rows with mask 0 per b.
 * vp_null_key_mass: out[b, h, n] = log2 of sum over the null keys of exp2(scale * log2 e * q[b, n, h] . k_null),
 *   -inf when there is none.  q: the normed + rotated queries [B, N, H*64] bf16 (strides in elements),
 *   N = T + F*Hh*Ww; beta bf16 [64]; the per-axis RoPE tables fp32: cos_t / sin_t [F][16], cos_y / sin_y [Hh][24],
 *   cos_x / sin_x [Ww][24].  segs / meta as vp_mask_null_segments wrote them (all B*F*Hh record slots are read,
 *   used or not).  F <= 16, Hh <= 64, Ww <= 255, vp_null_key_mass_lds_bytes <= 160 KiB. */
int vp_mask_null_segments(const uint8_t* mask, int64_t mask_bstride, int32_t B, int32_t T, int32_t F, int32_t Hh,
                          int32_t Ww, void* segs, int32_t* meta, void* stream);
int64_t vp_null_key_mass_lds_bytes(int32_t F, int32_t Hh, int32_t Ww);
int vp_null_key_mass(const void* q, int64_t q_sb, int64_t q_sn, int32_t B, int32_t H, int32_t N, int32_t T, int32_t F,
                     int32_t Hh, int32_t Ww, const void* beta, const float* cos_t, const float* sin_t,
                     const float* cos_y, const float* sin_y, const float* cos_x, const float* sin_x,
                     const uint8_t* mask, int64_t mask_bstride, const void* segs, const int32_t* meta, float scale,
                     float* out, void* stream);
int vp_mask_scale_rows_bf16(const void* x_in, int64_t ld_in, int64_t bs_in, void* y, int64_t ld_out, int64_t bs_out,
                            int32_t B, int32_t Ntok, int32_t D, const uint8_t* tok_mask, int64_t mask_bstride,
                            float scale, const int32_t* dst_rows, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Output head norms — norm_final (cogvideox_transformer_3d.py:617-620) then AdaLayerNorm(chunk_dim=1)
 * (DF/models/normalization.py:73-85, shift|scale order): for video rows only,
 * y[b, v] = rnd(rnd(rnd(LN2(rnd(LN1(x[b, text_len + v])))) * rnd(1 + scale)) + shift);  mod bf16 [B, 2D].
 * ------------------------------------------------------------------------------------------------------------- */
int vp_final_norm_bf16(const void* x, void* y, int32_t B, int32_t Ntok, int32_t D, int32_t text_len,
                       const void* ln1_w, const void* ln1_b, const void* ln2_w, const void* ln2_b, float eps,
                       const void* mod, int64_t mod_bstride, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Small-M linear for the conditioning path: y[m, n] = act_out(Σ_k act_in(x[m, k]) W[n, k] + bias[n]), M <= 16.
 * act: 0 none, 1 SiLU (rounded to bf16 like the reference's bf16 nn.SiLU).  Replaces TimestepEmbedding
 * (DF/models/embeddings.py:729-774) and the AdaLN linears (normalization.py:64,370).
 * ------------------------------------------------------------------------------------------------------------- */
int vp_linear_small_bf16(const void* x, int64_t ldx, const void* W, const void* bias, void* y, int64_t ldy, int32_t M,
                         int32_t N, int32_t K, int32_t act_in, int32_t act_out, void* stream);

/* sinusoidal timestep embedding, flip_sin_to_cos: out bf16 [B, dim] — get_timestep_embedding
 * (DF/models/embeddings.py:27-78); timesteps: device fp32 [B] (the reference casts to float). */
int vp_timestep_embedding_bf16(const float* timesteps, void* out, int32_t B, int32_t dim, float freq_shift,
                               void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Patch embedding data movement (DF/models/embeddings.py:413-430; branch concat branch_cogvideox.py:359):
 * im2col of src1 [B,F,C1,H,W] ⊕ src2 [B,F,C2,H,W] (channel concat) into rows (b, f, y, x) of out [B*F*(H/p)*(W/p),
 * Kpad], column c*p*p + dy*p + dx, zero-padded to Kpad.
 * ------------------------------------------------------------------------------------------------------------- */
int vp_patchify_bf16(const void* src1, int32_t C1, const void* src2, int32_t C2, void* out, int32_t Kpad, int32_t B,
                     int32_t F, int32_t H, int32_t W, int32_t p, void* stream);

/* token mask: out[b, v] = (Σ of mask[b, f, 0, patch(v)] > 0) — avg_pool2d(p) > 0 (embeddings.py:421-428).
 * mask_is_f32: 1 if mask is fp32, 0 if bf16. */
int vp_patch_mask(const void* mask, int32_t mask_is_f32, uint8_t* out, int32_t B, int32_t F, int32_t H, int32_t W,
                  int32_t p, void* stream);

/* Self-guidance after block i (cogvideox_transformer_3d.py:593-608): the unmasked video rows take the guidance
 * states, then the branch injection is added — per row r of batch b (tok_mask[b, r] from vp_patch_mask):
 *   tok_mask == 0:  x = guide                       (+ inject: rnd(guide + inject))
 *   tok_mask != 0:  x unchanged                     (+ inject when inject_all: rnd(x + inject))
 * x, guide, inject: bf16 [B, rows, D] at row stride ld_* and batch stride bs_*; inject NULL: none; inject_all: the
 * reference's unmasked injection (no branch_block_masks).  D % 8 == 0, strides % 8 == 0.  (ABI 18.) */
int vp_guide_rows_bf16(void* x, int64_t ld_x, int64_t bs_x, const void* guide, int64_t ld_g, int64_t bs_g,
                       const void* inject, int64_t ld_i, int64_t bs_i, int32_t inject_all, const uint8_t* tok_mask,
                       int64_t mask_bstride, int32_t B, int32_t rows, int32_t D, void* stream);

/* unpatchify (cogvideox_transformer_3d.py:630-632): out[b,f,c,y*p+py,x*p+px] = proj[b, (f,y,x), c*p*p+py*p+px] */
int vp_unpatchify_bf16(const void* proj, int64_t ld, void* out, int32_t B, int32_t F, int32_t C, int32_t H, int32_t W,
                       int32_t p, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * One denoising-step glue, fused: CFG combine (anyl.py:995-997), CogVideoXDPMScheduler.step
 * (DF/schedulers/scheduling_dpm_cogvideox.py:330-439, v-prediction, incl. the 2nd-order branch) and the replace-gt
 * blend with add_noise (anyl.py:1017-1034; scheduler :442-466).  Scalars are precomputed on the host in the
 * reference's dtypes (bf16-rounded where the reference multiplies a bf16 tensor by a 0-dim fp64 tensor).
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct vp_dpm_desc {
  int64_t n;
  const void* noise_pred; /* bf16 [2, n] when do_cfg (uncond, text), else [n]                               */
  int32_t do_cfg;
  float guidance;
  const float* model_output; /* fp32 [n]: used instead of noise_pred when non-NULL (scheduler.step API)     */
  const void* sample;     /* bf16 [n] */
  const float* old_pred;  /* fp32 [n] or NULL */
  float* pred_out;        /* fp32 [n] */
  const void* noise1;     /* bf16 [n] */
  const void* noise2;     /* bf16 [n] (second-order step only) */
  int32_t second_order, replace_gt;
  float sa, sb, m1, m2, mn, m3, m4; /* sqrt(a_t) (bf16-rounded), sqrt(1-a_t), mult1 (bf16), mult2, mult_noise
                                       (bf16), mult3, mult4 */
  int32_t gt_add_noise, mask_background;
  const void* gt;         /* bf16 [n] video latents */
  const void* gt_noise;   /* bf16 [n] */
  const void* mask;       /* bf16 [n] */
  float gsa, gsb;         /* add_noise scalars, bf16-rounded */
  void* latents_out;      /* bf16 [n] (cast + replace-gt) or NULL */
  float* prev_out;        /* fp32 [n] pre-cast prev_sample (scheduler.step API) or NULL */
} vp_dpm_desc;

int vp_dpm_step_bf16(const vp_dpm_desc* d, void* stream);

/* deterministic N(mean, std²) fill (splitmix64 + Box-Muller) for synthetic weights on the device */
int vp_fill_normal_bf16(void* out, int64_t n, uint64_t seed, float mean, float std, void* stream);

/* ---- CogVideoX 3D causal VAE (DF/models/autoencoders/autoencoder_kl_cogvideox.py) ----
 * Activations are channels-last bf16 [B, T, H, W, C] ("NDHWC"); a channel count that is not a power of two >= 8
 * (the 3 pixel channels, ...) is zero-padded to one.  Conv weights are re-laid-out once at load time as
 * [Cout, kt, kh, kw, Cin] (Cin padded like the activation) so every conv is an implicit GEMM whose K runs over
 * (tap, channel) with channels contiguous. */
#define VP_CONV_MAX_T 128
typedef struct vp_conv3d_desc {
  int32_t B, Cin, Cout;            /* Cin = the (padded, power of two >= 8) channel count of x / hist / weight rows */
  int32_t Tout, Hout, Wout;        /* output grid */
  int32_t Hin, Win;                /* physical input grid (before the nearest upsampling below) */
  int32_t kt, kh, kw;              /* kernel (each 1 or 3); temporal stride 1 */
  int32_t sh, sw;                  /* spatial stride (1 or 2) */
  int32_t ph, pw;                  /* top / left zero padding in the upsampled grid (bottom / right: the bounds) */
  int32_t uh, uw;                  /* nearest upsampling of the input grid (1 or 2), folded into the gather */
  int32_t x_frames, hist_frames;   /* frames per batch element of x / hist */
  int32_t ldy, ldr;                /* row (pixel) strides of y / resid in elements: multiples of 8, >= Cout */
  int32_t tmap[VP_CONV_MAX_T];     /* virtual input frame v = t + dt (t: output frame, dt: temporal tap) ->
                                      >= 0: frame of x, < 0: frame (-1 - value) of hist (the causal cache) */
  const void* x;                   /* bf16 [B, x_frames, Hin, Win, Cin] */
  const void* hist;                /* bf16 [B, hist_frames, Hin, Win, Cin] or NULL */
  const void* w;                   /* bf16 [Cout, kt, kh, kw, Cin] */
  const void* bias;                /* bf16 [Cout] or NULL */
  const void* resid;               /* bf16 [B, Tout, Hout, Wout] rows of stride ldr, added after the bias, or NULL */
  void* y;                         /* bf16 [B, Tout, Hout, Wout] rows of stride ldy; channels [Cout, ldy) get 0 */
} vp_conv3d_desc;

/* CogVideoXCausalConv3d.forward (:133-145; kt = 3, 1x1x1), the resnet conv_shortcut (:273), CogVideoXDownsample3D's
 * stride-2 conv2d (DF/models/downsampling.py:344-353) and CogVideoXUpsample3D's nearest-upsample + conv2d
 * (DF/models/upsampling.py:384-412) as one implicit-GEMM MFMA kernel. */
int vp_conv3d_bf16(const vp_conv3d_desc* d, void* stream);

/* nn.GroupNorm over [B, P, C] channels-last (groups of C / G consecutive channels), fp32 statistics (per-thread sums
 * shifted by the group's first element, combined in fp64): stats = float [B, G, 2] (mean, rstd); partials: float
 * workspace of vp_group_norm_workspace_floats(B, G) floats. */
int64_t vp_group_norm_workspace_floats(int32_t B, int32_t G);
int vp_group_norm_stats(const void* x, int32_t B, int64_t P, int32_t C, int32_t G, float eps, float* partials,
                        float* stats, void* stream);

/* y = act(GroupNorm(x) [* Ymod + Bmod]) over [B, T, H, W, C]: GroupNorm affine (gamma, beta bf16 [C]); with
 * mod != NULL the CogVideoXSpatialNorm3D modulation (:175-188): mod = bf16 [B, Tz, Hz, Wz, 2C] holding
 * conv_y(z) | conv_b(z) at the LATENT resolution (a 1x1x1 conv commutes with nearest resizing), gathered at the
 * nearest source position: frame tzmap[t] (host array of T entries), row floor(h * (Hz / H)), column
 * floor(w * (Wz / W)) (torch's nearest rule, float scale); act = SiLU if silu. */
int vp_group_norm_apply_bf16(const void* x, void* y, int32_t B, int32_t T, int32_t H, int32_t W, int32_t C,
                             int32_t G, const float* stats, const void* gamma, const void* beta, const void* mod,
                             int32_t Tz, int32_t Hz, int32_t Wz, const int32_t* tzmap_host, int32_t silu,
                             void* stream);

/* CogVideoXDownsample3D's temporal compression (DF/models/downsampling.py:323-342): x [B, T, P, C] ->
 * [B, T', P, C] with frame 0 kept when T is odd and every following pair averaged. */
int vp_time_pool2_bf16(const void* x, void* y, int32_t B, int32_t T, int64_t P, int32_t C, void* stream);

/* layout: NCDHW (fp32 or bf16) [B, C, T, H, W] <-> channels-last bf16 [B, T, H, W, Cpad] (zero padding channels);
 * the reverse takes channels [c0, c0 + C) of rows of stride ldx and writes bf16 NCDHW */
int vp_ncdhw_to_ndhwc_bf16(const void* x, int32_t x_is_f32, void* y, int32_t B, int32_t C, int32_t T, int32_t H,
                           int32_t W, int32_t Cpad, void* stream);
int vp_ndhwc_to_ncdhw_bf16(const void* x, int32_t ldx, void* y, int32_t B, int32_t C, int32_t T, int32_t H,
                           int32_t W, int32_t c0, void* stream);

/* DiagonalGaussianDistribution (DF/models/autoencoders/vae.py:768-789) on the encoder output [B, T, H, W] rows of
 * stride ldp holding mean | logvar (2L channels): mean, logvar clamped to [-30, 20] as bf16 NCDHW [B, L, T, H, W];
 * with noise != NULL (bf16 NCDHW) sample = mean + exp(0.5 logvar) * noise is written to `sample`. */
int vp_latent_dist_bf16(const void* params, int32_t ldp, void* mean, void* logvar, const void* noise, void* sample,
                        int32_t B, int32_t L, int32_t T, int32_t H, int32_t W, void* stream);

/* AutoencoderKLCogVideoX.blend_v / blend_h (:1192-1206) on channels-last tiles, in place on b: with e = min(Ha, Hb,
 * extent) (axis 0) rows y < e of b become a[row Ha - e + y] * (1 - y / e) + b[row y] * (y / e); axis 1 the same over
 * columns (e = min(Wa, Wb, extent)).  a [B, T, Ha, Wa, C], b [B, T, Hb, Wb, C], both contiguous; axis 0 needs
 * Wa == Wb, axis 1 Ha == Hb. */
int vp_tile_blend_bf16(const void* a, void* b, int32_t B, int32_t T, int32_t Ha, int32_t Wa, int32_t Hb, int32_t Wb,
                       int32_t C, int32_t axis, int32_t extent, void* stream);


/* ---- T5 v1.1 encoder (transformers modeling_t5.py, pinned transformers==4.42.2) ----
 * The projections (q|k|v fused, o, wi_0 + GELU-tanh, wi_1, wo) run on vp_gemm_bf16 (no bias; the residual adds are
 * its VP_EPI_BIAS_ADDROWS epilogue).  T5Stack.embed_tokens: out[r] = table[ids[r]] (bf16 [vocab, D]). */
int vp_embedding_gather_bf16(const void* table, const int64_t* ids, void* out, int32_t rows, int32_t D, int32_t vocab,
                             void* stream);
/* T5LayerNorm: y = w * bf16(x * rsqrt(mean(x^2) + eps)) over rows of D (bf16 in / out, fp32 statistics) */
int vp_rms_norm_bf16(const void* x, const void* w, void* y, int32_t rows, int32_t D, float eps, void* stream);
/* T5DenseGatedActDense's product: y = bf16(a * b) elementwise (n % 8 == 0) */
int vp_mul_bf16(const void* a, const void* b, void* y, int64_t n, void* stream);
/* T5Attention (encoder, bidirectional): qkv [B, L, ld] bf16 holding q | k | v (inner = H * 64 columns each);
 * scores = bf16(q . k) + bias_table[buckets[q * L + k], h] (no 1/sqrt(d) scaling), masked keys (mask[b, k] == 0,
 * int64 [B, L], or mask NULL) get the bf16 minimum added, softmax in fp32, out [B, L] rows of stride ldo, head h at
 * column h * 64.  buckets: int32 [L, L] from T5Attention._relative_position_bucket (host-computed); L <= 512. */
int vp_t5_attention_bf16(const void* qkv, int64_t ld, int32_t inner, int32_t B, int32_t L, int32_t H,
                         const void* bias_table, const int32_t* buckets, const int64_t* mask, void* out, int64_t ldo,
                         void* stream);


/* ---- pixel-space glue of the any-length pipeline's VAE stage (…_anyl.py:339-484) ---- */
/* y = bf16(x * s) (the latents' scaling_factor and its inverse, :372 / :430 / :481) */
int vp_scale_bf16(const void* x, void* y, int64_t n, float s, void* stream);
/* out = video * (mask < 0.5) (keep_above: >= 0.5, mask_background) over [B, C, P] with mask [B, 1, P] fp32
 * (:890-893); video fp32 or bf16, out bf16 */
int vp_mask_video_bf16(const void* video, int32_t video_is_f32, const float* mask, int32_t keep_above, void* out,
                       int32_t B, int32_t C, int64_t P, void* stream);
/* F.interpolate(mode="nearest", size=(t, h, w)) of fp32 [BC, T, H, W] -> bf16 (:437-439) */
int vp_nearest_resize3d_bf16(const float* x, void* y, int32_t BC, int32_t T, int32_t H, int32_t W, int32_t t,
                             int32_t h, int32_t w, void* stream);
/* VaeImageProcessor.denormalize on bf16: (x / 2 + 0.5).clamp(0, 1) */
int vp_denormalize_bf16(const void* x, void* y, int64_t n, void* stream);


/* ---- backward (train/train_cogvideox_inpainting_i2v_video.py:1892 accelerator.backward) ---- */
/* Flash-attention backward of vp_attention_fwd_bf16 (one K/V segment, no blend): with P = exp2(c q.k - lse),
 * c = scale * log2 e, lse from the forward's vp_attn_desc.lse: dQ = scale dS K, dK = scale dS^T Q, dV = P^T dO with
 * dS = P (dO V^T - rowsum(dO O)).  delta: fp32 workspace [B, H, Nq].  All tensors [B, N, H*64]-strided bf16. */
typedef struct vp_attn_bwd_desc {
  int32_t B, H, Nq, Nk, head_dim, pad0;
  const void* Q;
  int64_t q_sb, q_sn;
  const void* K;
  int64_t k_sb, k_sn;
  const void* V;
  int64_t v_sb, v_sn;
  const void* O;
  int64_t o_sb, o_sn;
  const void* dO;
  int64_t do_sb, do_sn;
  const float* lse;
  float* delta;
  void* dQ;
  int64_t dq_sb, dq_sn;
  void* dK;
  int64_t dk_sb, dk_sn;
  void* dV;
  int64_t dv_sb, dv_sn;
  float scale;
  int32_t pad1;
} vp_attn_bwd_desc;
int vp_attention_bwd_bf16(const vp_attn_bwd_desc* d, void* stream);
/* The same with a workspace for the grid-tail split (ABI 19): the blocks of each kernel's last partial round run as
 * key- / query-range pieces at the end of its grid, their fp32 sums merged by a small pass.
 * vp_attention_bwd_workspace_bytes: bytes needed for this descriptor (0: no split; -1: invalid descriptor); a smaller
 * or NULL workspace runs unsplit.  VP_ATTN_NO_SPLIT disables the split (A/B). */
int64_t vp_attention_bwd_workspace_bytes(const vp_attn_bwd_desc* d);
int vp_attention_bwd_bf16_ws(const vp_attn_bwd_desc* d, void* workspace, int64_t workspace_bytes, void* stream);


/* The other backward passes (row / elementwise / column reductions; the backward's matrix products run on
 * vp_gemm_bf16 against transposed operands).  y[c][r] = x[r][c] for nbatch R x C bf16 matrices: */
int vp_transpose_bf16(const void* x, int64_t ldx, int64_t x_bs, void* y, int64_t ldy, int64_t y_bs, int32_t R,
                      int32_t Cc, int32_t nbatch, void* stream);
/* out[(batch * 2 + type) * cols + n] += sum over rows m of that (batch = m / Ntok, type = text (1) if m % Ntok <
 * text_len) of a[m, n] (* b[m, n] when b != NULL): bias / gate / shift / scale / LayerNorm-affine gradients (fp32
 * atomics; cols % 8 == 0) */
int vp_colsum_bf16(const void* a, int64_t lda, const void* b, int64_t ldb, int32_t rows, int32_t cols, int32_t Ntok,
                   int32_t text_len, float* out, void* stream);
/* CogVideoXLayerNormZero backward (normalization.py:373-379): with n = bf16(LN(x) w + b) and the forward's
 * y = bf16(bf16(n (1 + scale)) + shift) (scale / shift = chunks scale_v / shift_v of mod for video rows, _t for
 * text rows), dx += LN'(dy (1 + scale) w) (bf16 in place); optionally writes n, dn = dy (1 + scale) and LN(x) (bf16
 * [rows, D]) for the parameter column sums. */
int vp_adaln_bwd_bf16(const void* x, const void* dy, void* dx, int32_t B, int32_t Ntok, int32_t D, int32_t text_len,
                      const void* ln_w, const void* ln_b, float eps, const void* mod, int64_t mod_bstride,
                      int32_t shift_v, int32_t scale_v, int32_t shift_t, int32_t scale_t, void* n_out, void* dn_out,
                      void* xhat_out, void* stream);
/* y = bf16(x * gate) with gate = chunk chunk_v (video rows) / chunk_t (text rows) of mod [B, *] (the gated
 * residual's gradient into its branch, cogvideox_transformer_3d.py:161-162, 179-180) */
int vp_rowscale_bf16(const void* x, int64_t ldx, void* y, int64_t ldy, int32_t rows, int32_t Ntok, int32_t D,
                     int32_t text_len, const void* mod, int64_t mod_bstride, int32_t chunk_v, int32_t chunk_t,
                     void* stream);
/* GELU(tanh) forward h = gelu(z) and backward dz = dh * gelu'(z) (activations.py:65-90), elementwise bf16 */
int vp_gelu_bf16(const void* z, void* h, int64_t n, void* stream);
int vp_gelu_bwd_bf16(const void* dh, const void* z, void* dz, int64_t n, void* stream);
/* y = bf16(a + alpha b) (gradient accumulation), n % 8 == 0 */
int vp_axpy_bf16(const void* a, const void* b, float alpha, void* y, int64_t n, void* stream);
/* y = silu(x) and y = dy * silu'(x) (the AdaLN / time-embedding SiLU) */
int vp_silu_bf16(const void* x, void* y, int64_t n, void* stream);
int vp_silu_bwd_bf16(const void* dy, const void* x, void* y, int64_t n, void* stream);
/* backward of vp_head_norm_rope_bf16 (LayerNorm(64) + RoPE on rows >= text_len; no token mask): x_in = the
 * pre-norm q or k, dy = the gradient of the normed + rotated output, dx = the gradient of x_in; dln_w / dln_b: fp32
 * [64] accumulated (atomics) or both NULL */
int vp_head_norm_rope_bwd_bf16(const void* x_in, int64_t ld_in, int64_t bs_in, const void* dy, int64_t ld_dy,
                               int64_t bs_dy, void* dx, int64_t ld_dx, int64_t bs_dx, int32_t B, int32_t Ntok,
                               int32_t H, int32_t text_len, const void* ln_w, const void* ln_b, float eps,
                               const float* cos, const float* sin, float* dln_w, float* dln_b, void* stream);


#ifdef __cplusplus
}
#endif
#endif /* VP_HIP_H */
