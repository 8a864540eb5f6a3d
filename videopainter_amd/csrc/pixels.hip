// Pixel-space glue of the any-length pipeline's VAE stage (gfx950): the latent scaling by the VAE's scaling_factor,
// the masked-video product, the nearest resize of the mask to the latent grid and the video processor's
// denormalisation — elementwise, HBM-bound, run once per window.
// Reference: DF/pipelines/cogvideo/pipeline_cogvideox_inpainting_i2v_branch_anyl.py:372,430 (scaling), :890-893
// (masked video), :437-439 (mask resize), :481 (1 / scaling), DF/image_processor.py VaeImageProcessor.denormalize.
#include "vp_common.h"

namespace {

int grid_for(int64_t work) {
  const int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > (1 << 20) ? (1 << 20) : g));
}

__global__ __launch_bounds__(256) void scale_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int64_t n,
                                                    float s) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = f2bf(bf2f(x[i]) * s);
}

// out[b, c, f, h, w] = video[b, c, f, h, w] * (mask[b, 0, f, h, w] < 0.5)   (or >= 0.5 with keep_above)
__global__ __launch_bounds__(256) void mask_video_kernel(const void* __restrict__ v, int v_f32,
                                                         const float* __restrict__ m, int keep_above,
                                                         bf16* __restrict__ out, int B, int C, int64_t P) {
  const int64_t total = (int64_t)B * C * P;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t p = i % P;
    const int b = (int)(i / ((int64_t)C * P));
    const float x = v_f32 ? ((const float*)v)[i] : bf2f(((const bf16*)v)[i]);
    const float mk = m[(int64_t)b * P + p];
    const bool keep = keep_above ? (mk >= 0.5f) : (mk < 0.5f);
    out[i] = f2bf(keep ? x : 0.f);
  }
}

// torch nearest (explicit size): src = min(floor(dst * (in / out)), in - 1), float scale
VP_DEV int nearest_src(int dst, int n_in, int n_out) {
  if (n_in == n_out) return dst;
  const float sc = (float)n_in / (float)n_out;
  return min((int)floorf((float)dst * sc), n_in - 1);
}

__global__ __launch_bounds__(256) void nearest3d_kernel(const float* __restrict__ x, bf16* __restrict__ y, int BC,
                                                        int T, int H, int W, int t, int h, int w) {
  const int64_t total = (int64_t)BC * t * h * w;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int ow = (int)(i % w);
    const int oh = (int)((i / w) % h);
    const int ot = (int)((i / ((int64_t)w * h)) % t);
    const int bc = (int)(i / ((int64_t)w * h * t));
    const int st = nearest_src(ot, T, t), sh = nearest_src(oh, H, h), sw = nearest_src(ow, W, w);
    y[i] = f2bf(x[(((int64_t)bc * T + st) * H + sh) * W + sw]);
  }
}

// VaeImageProcessor.denormalize on bf16: (x / 2 + 0.5).clamp(0, 1), rounded after each bf16 op
__global__ __launch_bounds__(256) void denorm_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = rbf(rbf(bf2f(x[i]) * 0.5f) + 0.5f);
    y[i] = f2bf(fminf(fmaxf(v, 0.f), 1.f));
  }
}

}  // namespace

extern "C" int vp_scale_bf16(const void* x, void* y, int64_t n, float s, void* stream) {
  if (x == nullptr || y == nullptr || n <= 0) return VP_ERR_ARG;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y, n,
                     s);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_mask_video_bf16(const void* video, int32_t video_is_f32, const float* mask, int32_t keep_above,
                                  void* out, int32_t B, int32_t C, int64_t P, void* stream) {
  if (video == nullptr || mask == nullptr || out == nullptr || B <= 0 || C <= 0 || P <= 0) return VP_ERR_ARG;
  hipLaunchKernelGGL(mask_video_kernel, dim3(grid_for((int64_t)B * C * P)), dim3(256), 0, (hipStream_t)stream, video,
                     video_is_f32 ? 1 : 0, mask, keep_above ? 1 : 0, (bf16*)out, B, C, P);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_nearest_resize3d_bf16(const float* x, void* y, int32_t BC, int32_t T, int32_t H, int32_t W,
                                        int32_t t, int32_t h, int32_t w, void* stream) {
  if (x == nullptr || y == nullptr || BC <= 0 || T <= 0 || H <= 0 || W <= 0 || t <= 0 || h <= 0 || w <= 0)
    return VP_ERR_ARG;
  hipLaunchKernelGGL(nearest3d_kernel, dim3(grid_for((int64_t)BC * t * h * w)), dim3(256), 0, (hipStream_t)stream, x,
                     (bf16*)y, BC, T, H, W, t, h, w);
  VP_CHECK_LAUNCH();
  return 0;
}

extern "C" int vp_denormalize_bf16(const void* x, void* y, int64_t n, void* stream) {
  if (x == nullptr || y == nullptr || n <= 0) return VP_ERR_ARG;
  hipLaunchKernelGGL(denorm_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y, n);
  VP_CHECK_LAUNCH();
  return 0;
}
