// Backward kernels of the CogVideoX block path other than attention and the GEMMs (the training
// caller, train/train_cogvideox_inpainting_i2v_video.py:1857-1892, backpropagates through the frozen transformer into
// the trainable branch).  Every one is a row / elementwise / column-reduction pass (HBM-bound); the matrix products
// of the backward run on vp_gemm_bf16 (dgrad against transposed weights, wgrad against transposed activations) and
// vp_attention_bwd_bf16.
// Reference forward: CogVideoXLayerNormZero (DF/models/normalization.py:358-386), the gated residuals and the
// FeedForward of CogVideoXBlock (cogvideox_transformer_3d.py:125-184, attention.py:1144-1202 with GELU(tanh)), the
// q/k LayerNorm + RoPE of CogVideoXAttnProcessor2_0 (attention_processor.py:2143-2160, embeddings.py:655-701).
#include "vp_common.h"

namespace {

int grid_for(int64_t work) {
  const int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > (1 << 20) ? (1 << 20) : g));
}

// y[c][r] = x[r][c] for a batch of R x C bf16 matrices, 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void transpose_kernel(const bf16* __restrict__ x, int64_t ldx, int64_t xbs,
                                                        bf16* __restrict__ y, int64_t ldy, int64_t ybs, int R, int C) {
  __shared__ bf16 tile[64][66];
  const int tc = blockIdx.x, tr = blockIdx.y, b = blockIdx.z;
  const bf16* xb = x + (int64_t)b * xbs;
  bf16* yb = y + (int64_t)b * ybs;
  const int tid = threadIdx.x;
  for (int i = tid; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    const int gr = tr * 64 + r, gc = tc * 64 + c;
    tile[r][c] = (gr < R && gc < C) ? xb[(int64_t)gr * ldx + gc] : f2bf(0.f);
  }
  __syncthreads();
  for (int i = tid; i < 64 * 64; i += 256) {
    const int c = i >> 6, r = i & 63;
    const int gr = tr * 64 + r, gc = tc * 64 + c;
    if (gr < R && gc < C) yb[(int64_t)gc * ldy + gr] = tile[r][c];
  }
}

// out[(batch * 2 + type) * cols + n] += sum over the rows of that (batch, type) of a[m, n] (* b[m, n]); type 1 =
// text rows (token < text_len).  Each thread sums 8 columns over a 256-row stripe, then one fp32 atomic per column.
constexpr int CS_ROWS = 256;
__global__ __launch_bounds__(256) void colsum_kernel(const bf16* __restrict__ a, int64_t lda,
                                                     const bf16* __restrict__ bm, int64_t ldb, int rows, int cols,
                                                     int Ntok, int text_len, float* __restrict__ out) {
  const int c8 = blockIdx.x * 256 + threadIdx.x;  // column chunk
  if (c8 * 8 >= cols) return;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(rows, r0 + CS_ROWS);
  float acc[8], acc_t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = acc_t[e] = 0.f;
  int cur_b = r0 / Ntok;
  auto flush = [&](int b) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (acc[e] != 0.f) atomicAdd(out + ((int64_t)b * 2) * cols + c8 * 8 + e, acc[e]);
      if (acc_t[e] != 0.f) atomicAdd(out + ((int64_t)b * 2 + 1) * cols + c8 * 8 + e, acc_t[e]);
      acc[e] = acc_t[e] = 0.f;
    }
  };
  for (int m = r0; m < r1; ++m) {
    const int b = m / Ntok;
    if (b != cur_b) {
      flush(cur_b);
      cur_b = b;
    }
    const bool text = (m - b * Ntok) < text_len;
    const bf16x8 va = *(const bf16x8*)(a + (int64_t)m * lda + c8 * 8);
    bf16x8 vb;
    if (bm != nullptr) vb = *(const bf16x8*)(bm + (int64_t)m * ldb + c8 * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = bm != nullptr ? bf2f(va[e]) * bf2f(vb[e]) : bf2f(va[e]);
      if (text) acc_t[e] += v;
      else acc[e] += v;
    }
  }
  flush(cur_b);
}

// AdaLN-Zero backward (forward: n = bf16(LN(x) w + b), y = bf16(bf16(n (1 + scale)) + shift), scale / shift the
// video or text chunks of mod): dx += LN'(dy (1 + scale) w); optionally writes n, dn = dy (1 + scale) and xhat (bf16)
// for the parameter column sums.  One wave per row, the row in registers.
template <int NCH>
__global__ __launch_bounds__(256) void adaln_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        bf16* __restrict__ dx, int rows, int Ntok, int D,
                                                        int text_len, const bf16* __restrict__ lw,
                                                        const bf16* __restrict__ lb, float eps,
                                                        const bf16* __restrict__ mod, int64_t mod_bs, int sh_v,
                                                        int sc_v, int sh_t, int sc_t, bf16* __restrict__ n_out,
                                                        bf16* __restrict__ dn_out, bf16* __restrict__ xh_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int b = row / Ntok;
  const bool text = (row - b * Ntok) < text_len;
  const int nch = D / 8;
  const bf16* xr = x + (int64_t)row * D;
  float s = 0.f;
  bf16x8 xv[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      xv[i] = *(const bf16x8*)(xr + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += bf2f(xv[i][e]);
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i)
    if (lane + i * 64 < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = bf2f(xv[i][e]) - mean;
        q += t * t;
      }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  const bf16* scale = mod + (int64_t)b * mod_bs + (text ? sc_t : sc_v) * D;
  const bf16* shift = mod + (int64_t)b * mod_bs + (text ? sh_t : sh_v) * D;
  (void)shift;
  // dxhat = dy (1 + scale) w;  sums of dxhat and dxhat * xhat over the row
  float g1 = 0.f, g2 = 0.f;
  float dxh[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      const bf16x8 dv = *(const bf16x8*)(dy + (int64_t)row * D + c * 8);
      const bf16x8 sc = *(const bf16x8*)(scale + c * 8);
      const bf16x8 w = *(const bf16x8*)(lw + c * 8);
      const bf16x8 bb = *(const bf16x8*)(lb + c * 8);
      bf16x8 nv, dnv, xhv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (bf2f(xv[i][e]) - mean) * rstd;
        const float dn = bf2f(dv[e]) * rbf(1.f + bf2f(sc[e]));
        dxh[i][e] = dn * bf2f(w[e]);
        g1 += dxh[i][e];
        g2 += dxh[i][e] * xh;
        nv[e] = f2bf(__builtin_fmaf(xh, bf2f(w[e]), bf2f(bb[e])));
        dnv[e] = f2bf(dn);
        xhv[e] = f2bf(xh);
      }
      if (n_out != nullptr) *(bf16x8*)(n_out + (int64_t)row * D + c * 8) = nv;
      if (dn_out != nullptr) *(bf16x8*)(dn_out + (int64_t)row * D + c * 8) = dnv;
      if (xh_out != nullptr) *(bf16x8*)(xh_out + (int64_t)row * D + c * 8) = xhv;
    }
  }
  g1 = wave_sum(g1) / (float)D;
  g2 = wave_sum(g2) / (float)D;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      bf16* dp = dx + (int64_t)row * D + c * 8;
      const bf16x8 old = *(const bf16x8*)dp;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (bf2f(xv[i][e]) - mean) * rstd;
        o[e] = f2bf(bf2f(old[e]) + rstd * (dxh[i][e] - g1 - xh * g2));
      }
      *(bf16x8*)dp = o;
    }
  }
}

// y = bf16(x * gate[b, video / text chunk, :])  (the gated residual's branch gradient)
__global__ __launch_bounds__(256) void rowscale_kernel(const bf16* __restrict__ x, int64_t ldx, bf16* __restrict__ y,
                                                       int64_t ldy, int rows, int Ntok, int D, int text_len,
                                                       const bf16* __restrict__ mod, int64_t mod_bs, int ch_v,
                                                       int ch_t) {
  const int C8 = D >> 3;
  const int64_t total = (int64_t)rows * C8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / C8), c = (int)(i - (int64_t)m * C8);
    const int b = m / Ntok;
    const bool text = (m - b * Ntok) < text_len;
    const bf16x8 g = *(const bf16x8*)(mod + (int64_t)b * mod_bs + (text ? ch_t : ch_v) * D + c * 8);
    const bf16x8 v = *(const bf16x8*)(x + (int64_t)m * ldx + c * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(v[e]) * bf2f(g[e]));
    *(bf16x8*)(y + (int64_t)m * ldy + c * 8) = o;
  }
}

// GELU (tanh form) and its derivative (gelu_grad, vp_common.h: shared with the GEMM's VP_EPI_GELU_BWD), elementwise

__global__ __launch_bounds__(256) void gelu_kernel(const bf16* __restrict__ z, bf16* __restrict__ h, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const bf16x8 v = *(const bf16x8*)(z + i * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(gelu_tanh(bf2f(v[e])));
    *(bf16x8*)(h + i * 8) = o;
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const bf16* __restrict__ dh, const bf16* __restrict__ z,
                                                       bf16* __restrict__ dz, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const bf16x8 g = *(const bf16x8*)(dh + i * 8), v = *(const bf16x8*)(z + i * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(g[e]) * gelu_grad(bf2f(v[e])));
    *(bf16x8*)(dz + i * 8) = o;
  }
}

// y = bf16(a + alpha * b)
__global__ __launch_bounds__(256) void axpy_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, float alpha,
                                                   bf16* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const bf16x8 u = *(const bf16x8*)(a + i * 8), v = *(const bf16x8*)(b + i * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(__builtin_fmaf(alpha, bf2f(v[e]), bf2f(u[e])));
    *(bf16x8*)(y + i * 8) = o;
  }
}

// y = silu(x) (the input of the AdaLN / time-embedding linears, for their weight gradients)
__global__ __launch_bounds__(256) void silu_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = bf2f(x[i]);
    y[i] = f2bf(v / (1.f + __expf(-v)));
  }
}

// y = dy * silu'(x) = dy * sigmoid(x) (1 + x (1 - sigmoid(x)))  (the AdaLN / time-embedding SiLU)
__global__ __launch_bounds__(256) void silu_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                       bf16* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = bf2f(x[i]);
    const float sg = 1.f / (1.f + __expf(-v));
    y[i] = f2bf(bf2f(dy[i]) * sg * (1.f + v * (1.f - sg)));
  }
}

// backward of LayerNorm(64) (+ RoPE on video rows) per head vector: 4 lanes x 16 elements (lane g holds columns
// 16 j + 4 g + r, like ln64_rope16); parameter grads reduced over the block's 64 vectors, one atomic per column
__global__ __launch_bounds__(256) void head_norm_rope_bwd_kernel(const bf16* __restrict__ xin, int64_t ld_in,
                                                                 int64_t bs_in, const bf16* __restrict__ dyin,
                                                                 int64_t ld_dy, int64_t bs_dy, bf16* __restrict__ dx,
                                                                 int64_t ld_dx, int64_t bs_dx, int64_t nvec, int Ntok,
                                                                 int H, int text_len, const bf16* __restrict__ lw,
                                                                 const bf16* __restrict__ lb, float eps,
                                                                 const float* __restrict__ cosp,
                                                                 const float* __restrict__ sinp,
                                                                 float* __restrict__ dlw, float* __restrict__ dlb) {
  __shared__ float red[2][64][64 + 1];
  const int64_t vec = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
  const int vl = threadIdx.x >> 2;
  const int g = threadIdx.x & 3;
  const bool valid = vec < nvec;
  const int64_t vv = valid ? vec : nvec - 1;
  const int h = (int)(vv % H);
  const int64_t bn = vv / H;
  const int n = (int)(bn % Ntok);
  const int b = (int)(bn / Ntok);
  const bf16* src = xin + (int64_t)b * bs_in + (int64_t)n * ld_in + h * 64 + g * 4;
  const bf16* dsrc = dyin + (int64_t)b * bs_dy + (int64_t)n * ld_dy + h * 64 + g * 4;
  float x[16], dy[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x4 xr = *(const bf16x4*)(src + 16 * j);
    const bf16x4 dr = *(const bf16x4*)(dsrc + 16 * j);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[4 * j + r] = bf2f(xr[r]);
      dy[4 * j + r] = bf2f(dr[r]);
    }
  }
  // RoPE^T on video rows: y0 = n0 c0 - n1 s0, y1 = n1 c1 + n0 s1  ->  dn0 = dy0 c0 + dy1 s1, dn1 = dy1 c1 - dy0 s0
  if (cosp != nullptr && n >= text_len) {
    const float* cr = cosp + (int64_t)(n - text_len) * 64;
    const float* sr = sinp + (int64_t)(n - text_len) * 64;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 16 * j + 4 * g;
      const f32x4 cs = *(const f32x4*)(cr + c), sn = *(const f32x4*)(sr + c);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float d0 = dy[4 * j + 2 * p], d1 = dy[4 * j + 2 * p + 1];
        dy[4 * j + 2 * p] = d0 * cs[2 * p] + d1 * sn[2 * p + 1];
        dy[4 * j + 2 * p + 1] = d1 * cs[2 * p + 1] - d0 * sn[2 * p];
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += x[e];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  const float mean = s * (1.f / 64.f);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float t = x[e] - mean;
    q = __builtin_fmaf(t, t, q);
  }
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  const float rstd = rsqrtf(__builtin_fmaf(q, 1.f / 64.f, eps));
  float g1 = 0.f, g2 = 0.f, xh[16], dxh[16];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * j + r, c = 16 * j + 4 * g + r;
      xh[e] = (x[e] - mean) * rstd;
      dxh[e] = dy[e] * bf2f(lw[c]);
      g1 += dxh[e];
      g2 += dxh[e] * xh[e];
      if (dlw != nullptr) {
        red[0][vl][c] = valid ? dy[e] * xh[e] : 0.f;
        red[1][vl][c] = valid ? dy[e] : 0.f;
      }
    }
  g1 += __shfl_xor(g1, 1, 64);
  g1 += __shfl_xor(g1, 2, 64);
  g2 += __shfl_xor(g2, 1, 64);
  g2 += __shfl_xor(g2, 2, 64);
  g1 *= 1.f / 64.f;
  g2 *= 1.f / 64.f;
  if (valid) {
    bf16* dst = dx + (int64_t)b * bs_dx + (int64_t)n * ld_dx + h * 64 + g * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(rstd * (dxh[4 * j + r] - g1 - xh[4 * j + r] * g2));
      *(bf16x4*)(dst + 16 * j) = o;
    }
  }
  if (dlw != nullptr) {
    __syncthreads();
    if (threadIdx.x < 128) {
      const int which = threadIdx.x >> 6, c = threadIdx.x & 63;
      float acc = 0.f;
      for (int v2 = 0; v2 < 64; ++v2) acc += red[which][v2][c];
      atomicAdd((which ? dlb : dlw) + c, acc);
    }
  }
}

}  // namespace

extern "C" int vp_transpose_bf16(const void* x, int64_t ldx, int64_t x_bs, void* y, int64_t ldy, int64_t y_bs,
                                 int32_t R, int32_t Cc, int32_t nbatch, void* stream) {
  if (x == nullptr || y == nullptr || R <= 0 || Cc <= 0 || nbatch <= 0 || ldx < Cc || ldy < R) return VP_ERR_ARG;
  if ((R + 63) / 64 > 65535 || nbatch > 65535) return VP_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(transpose_kernel, dim3((Cc + 63) / 64, (R + 63) / 64, nbatch), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, x_bs, (bf16*)y, ldy, y_bs, R, Cc);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_colsum_bf16(const void* a, int64_t lda, const void* b, int64_t ldb, int32_t rows, int32_t cols,
                              int32_t Ntok, int32_t text_len, float* out, void* stream) {
  if (a == nullptr || out == nullptr || rows <= 0 || cols <= 0 || (cols % 8) || (lda % 8) || Ntok <= 0) return VP_ERR_ARG;
  if (b != nullptr && (ldb % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(colsum_kernel, dim3((cols / 8 + 255) / 256, (rows + CS_ROWS - 1) / CS_ROWS), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)a, lda, (const bf16*)b, ldb, rows, cols, Ntok, text_len, out);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_adaln_bwd_bf16(const void* x, const void* dy, void* dx, int32_t B, int32_t Ntok, int32_t D,
                                 int32_t text_len, const void* ln_w, const void* ln_b, float eps, const void* mod,
                                 int64_t mod_bstride, int32_t shift_v, int32_t scale_v, int32_t shift_t,
                                 int32_t scale_t, void* n_out, void* dn_out, void* xhat_out, void* stream) {
  if (!x || !dy || !dx || !ln_w || !ln_b || !mod || B <= 0 || Ntok <= 0 || D <= 0 || (D % 8) || D > 4096)
    return VP_ERR_ARG;
  const int rows = B * Ntok;
  const int nch = (D / 8 + 63) / 64;
  hipStream_t s = (hipStream_t)stream;
#define VP_ADB(N)                                                                                                  \
  hipLaunchKernelGGL(adaln_bwd_kernel<N>, dim3((rows + 3) / 4), dim3(256), 0, s, (const bf16*)x, (const bf16*)dy,   \
                     (bf16*)dx, rows, Ntok, D, text_len, (const bf16*)ln_w, (const bf16*)ln_b, eps, (const bf16*)mod, \
                     mod_bstride, shift_v, scale_v, shift_t, scale_t, (bf16*)n_out, (bf16*)dn_out, (bf16*)xhat_out)
  if (nch <= 1) VP_ADB(1);
  else if (nch <= 2) VP_ADB(2);
  else if (nch <= 4) VP_ADB(4);
  else if (nch <= 6) VP_ADB(6);
  else VP_ADB(8);
#undef VP_ADB
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_rowscale_bf16(const void* x, int64_t ldx, void* y, int64_t ldy, int32_t rows, int32_t Ntok,
                                int32_t D, int32_t text_len, const void* mod, int64_t mod_bstride, int32_t chunk_v,
                                int32_t chunk_t, void* stream) {
  if (!x || !y || !mod || rows <= 0 || Ntok <= 0 || D <= 0 || (D % 8) || (ldx % 8) || (ldy % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(rowscale_kernel, dim3(grid_for((int64_t)rows * (D / 8))), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, (bf16*)y, ldy, rows, Ntok, D, text_len, (const bf16*)mod, mod_bstride,
                     chunk_v, chunk_t);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_gelu_bf16(const void* z, void* h, int64_t n, void* stream) {
  if (!z || !h || n <= 0 || (n % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)z, (bf16*)h,
                     n / 8);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_gelu_bwd_bf16(const void* dh, const void* z, void* dz, int64_t n, void* stream) {
  if (!dh || !z || !dz || n <= 0 || (n % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)dh,
                     (const bf16*)z, (bf16*)dz, n / 8);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_axpy_bf16(const void* a, const void* b, float alpha, void* y, int64_t n, void* stream) {
  if (!a || !b || !y || n <= 0 || (n % 8)) return VP_ERR_ARG;
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)a,
                     (const bf16*)b, alpha, (bf16*)y, n / 8);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_silu_bf16(const void* x, void* y, int64_t n, void* stream) {
  if (!x || !y || n <= 0) return VP_ERR_ARG;
  hipLaunchKernelGGL(silu_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y, n);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_silu_bwd_bf16(const void* dy, const void* x, void* y, int64_t n, void* stream) {
  if (!dy || !x || !y || n <= 0) return VP_ERR_ARG;
  hipLaunchKernelGGL(silu_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16*)dy,
                     (const bf16*)x, (bf16*)y, n);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_head_norm_rope_bwd_bf16(const void* x_in, int64_t ld_in, int64_t bs_in, const void* dy,
                                          int64_t ld_dy, int64_t bs_dy, void* dx, int64_t ld_dx, int64_t bs_dx,
                                          int32_t B, int32_t Ntok, int32_t H, int32_t text_len, const void* ln_w,
                                          const void* ln_b, float eps, const float* cos, const float* sin,
                                          float* dln_w, float* dln_b, void* stream) {
  if (!x_in || !dy || !dx || !ln_w || !ln_b || B <= 0 || Ntok <= 0 || H <= 0) return VP_ERR_ARG;
  if ((dln_w == nullptr) != (dln_b == nullptr)) return VP_ERR_ARG;
  if ((ld_in % 4) || (ld_dy % 4) || (ld_dx % 4)) return VP_ERR_ARG;
  const int64_t nvec = (int64_t)B * Ntok * H;
  const int64_t grid = (nvec + 63) / 64;
  if (grid > 0x7fffffff) return VP_ERR_ARG;
  hipLaunchKernelGGL(head_norm_rope_bwd_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x_in, ld_in, bs_in, (const bf16*)dy, ld_dy, bs_dy, (bf16*)dx, ld_dx, bs_dx, nvec,
                     Ntok, H, text_len, (const bf16*)ln_w, (const bf16*)ln_b, eps, cos, sin, dln_w, dln_b);
  VP_CHECK_LAUNCH();
  return 0;
}
