// Bandwidth-bound kernels of the DiffusionDrive hot path: layout conversion, pooling, bilinear
// resize, LayerNorm, softmax and activations. All HBM-bound: one pass, coalesced along the
// contiguous NHWC channel axis, wave64 shuffles for row reductions.
#include "common.h"

namespace ddmi {

static inline int grid_for(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  if (g > 65535 * 8) g = 65535 * 8;
  return (int)g;
}

// ---------------------------------------------------------------- NCHW -> NHWC (channel pad)
// Input camera (B,3,256,1024) / LiDAR (B,1,256,256) as the feature builder produces them
// (transfuser_features.py:57-138); padded to 4 channels so the stem's implicit GEMM reads float4.
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ in, float* __restrict__ out, int B, int C,
                                    int H, int W, int Cp) {
  const int64_t npix = (int64_t)B * H * W;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = p / ((int64_t)H * W);
    const int64_t hw = p - b * H * W;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = (c < C) ? in[(b * C + c) * H * W + hw] : 0.f;
    float* o = out + p * Cp;
    if (Cp == 4) {
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int c = 0; c < Cp; ++c) o[c] = c < 8 ? v[c] : 0.f;
    }
  }
}

void launch_nchw_to_nhwc(const float* in, float* out, int B, int C, int H, int W, int Cp, hipStream_t st) {
  if (C > 8 || Cp < C) throw std::runtime_error("nchw_to_nhwc: unsupported channel count");
  const int64_t n = (int64_t)B * H * W;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, out, B, C, H, W, Cp);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- maxpool 3x3 s2 p1 (timm stem)
__global__ void maxpool_kernel(const float4* __restrict__ in, float4* __restrict__ out, int B, int H, int W,
                               int C4, int Ho, int Wo) {
  const int64_t n = (int64_t)B * Ho * Wo * C4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = i % C4;
    int64_t t = i / C4;
    const int ox = t % Wo;
    t /= Wo;
    const int oy = t % Ho;
    const int64_t b = t / Ho;
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    for (int dy = 0; dy < 3; ++dy) {
      const int y = oy * 2 - 1 + dy;
      if ((unsigned)y >= (unsigned)H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int x = ox * 2 - 1 + dx;
        if ((unsigned)x >= (unsigned)W) continue;
        const float4 v = in[((b * H + y) * W + x) * C4 + c];
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    out[i] = m;
  }
}

void launch_maxpool3x3s2(const float* in, float* out, int B, int H, int W, int C, int Ho, int Wo,
                         hipStream_t st) {
  if (C % 4) throw std::runtime_error("maxpool: C % 4 != 0");
  const int64_t n = (int64_t)B * Ho * Wo * (C / 4);
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid_for(n)), dim3(256), 0, st, reinterpret_cast<const float4*>(in),
                     reinterpret_cast<float4*>(out), B, H, W, C / 4, Ho, Wo);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- adaptive avg pool (exact windows)
// transfuser_backbone.py:47-58,249-250: windows divide exactly at every scale.
__global__ void avgpool_kernel(const float* __restrict__ in, int B, int H, int W, int C, int oh, int ow,
                               View4 out, const float* __restrict__ add) {
  const int kh = H / oh, kw = W / ow;
  const float inv = 1.0f / (float)(kh * kw);
  const int64_t n = (int64_t)B * oh * ow * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = i % C;
    int64_t t = i / C;
    const int x = t % ow;
    t /= ow;
    const int y = t % oh;
    const int64_t b = t / oh;
    float s = 0.f;
    for (int dy = 0; dy < kh; ++dy) {
      const float* row = in + ((b * H + (int64_t)y * kh + dy) * W + (int64_t)x * kw) * C + c;
      for (int dx = 0; dx < kw; ++dx) s += row[(int64_t)dx * C];
    }
    float v = s * inv;
    if (add) v += add[((int64_t)y * ow + x) * C + c];
    out.p[b * out.sn + y * out.sh + x * out.sw + c * out.sc] = v;
  }
}

void launch_avgpool(const float* in, int B, int H, int W, int C, int oh, int ow, View4 out, const float* add,
                    hipStream_t st) {
  if (H % oh || W % ow) throw std::runtime_error("avgpool: non-integer window");
  const int64_t n = (int64_t)B * oh * ow * C;
  hipLaunchKernelGGL(avgpool_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, B, H, W, C, oh, ow, out, add);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- bilinear, align_corners=False
// PyTorch upsample_bilinear2d: src = max(ratio * (dst + 0.5) - 0.5, 0); i0 = floor(src);
// i1 = i0 + (i0 < in - 1); l1 = src - i0; l0 = 1 - l1.
__device__ inline void bl_index(int dst, float ratio, int in_size, int& i0, int& i1, float& l0, float& l1) {
  float src = ratio * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  i0 = (int)src;
  i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
}

__global__ void bilinear_kernel(View4 in, int B, int Hi, int Wi, int C, View4 out, int Ho, int Wo, float rh,
                                float rw, int accumulate) {
  const int64_t n = (int64_t)B * Ho * Wo * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = i % C;
    int64_t t = i / C;
    const int x = t % Wo;
    t /= Wo;
    const int y = t % Ho;
    const int64_t b = t / Ho;
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    bl_index(y, rh, Hi, y0, y1, ly0, ly1);
    bl_index(x, rw, Wi, x0, x1, lx0, lx1);
    const float* base = in.p + b * in.sn + (int64_t)c * in.sc;
    const float v00 = base[y0 * in.sh + x0 * in.sw];
    const float v01 = base[y0 * in.sh + x1 * in.sw];
    const float v10 = base[y1 * in.sh + x0 * in.sw];
    const float v11 = base[y1 * in.sh + x1 * in.sw];
    const float v = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
    float* o = out.p + b * out.sn + (int64_t)y * out.sh + (int64_t)x * out.sw + (int64_t)c * out.sc;
    *o = accumulate ? (*o + v) : v;
  }
}

void launch_bilinear(View4 in, int B, int Hi, int Wi, int C, View4 out, int Ho, int Wo, float ratio_h,
                     float ratio_w, int accumulate, hipStream_t st) {
  const int64_t n = (int64_t)B * Ho * Wo * C;
  hipLaunchKernelGGL(bilinear_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, B, Hi, Wi, C, out, Ho, Wo,
                     ratio_h, ratio_w, accumulate);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- LayerNorm (+ residual, + FiLM)
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ inline float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// One wave64 per row; up to 32 values per lane kept in registers (C <= 2048); two-pass variance.
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ res, int64_t ldres, int res_div,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        const float* __restrict__ fs, const float* __restrict__ fb,
                                                        float* y, int64_t ldy, int rows, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[32];
  const float* xr = x + (int64_t)row * ldx;
  const float* rr = res ? res + (int64_t)(row / res_div) * ldres : nullptr;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int c = lane + 64 * i;
    float t = 0.f;
    if (c < C) {
      t = xr[c];
      if (rr) t += rr[c];
    }
    v[i] = t;
    s += t;
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int c = lane + 64 * i;
    const float d = (c < C) ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + 1e-5f);
  float* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      float o = (v[i] - mean) * rstd * g[c] + b[c];
      if (fs) o = o * (1.f + fs[c]) + fb[c];
      yr[c] = o;
    }
  }
}

void launch_layernorm(const float* x, int64_t ldx, const float* res, int64_t ldres, int res_div, const float* g,
                      const float* b, const float* film_scale, const float* film_shift, float* y, int64_t ldy,
                      int rows, int C, hipStream_t st) {
  if (C > 2048) throw std::runtime_error("layernorm: C > 2048");
  if (rows == 0) return;
  hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, ldx, res, ldres,
                     res_div < 1 ? 1 : res_div, g, b, film_scale, film_shift, y, ldy, rows, C);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- row softmax (scaled)
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* x, int64_t ld, int rows, int L, float scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float* r = x + (int64_t)row * ld;
  float v[16];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < L) ? r[c] * scale : -INFINITY;
    m = fmaxf(m, v[i]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < L) ? expf(v[i] - m) : 0.f;
    s += v[i];
  }
  const float inv = 1.f / wave_sum(s);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    if (c < L) r[c] = v[i] * inv;
  }
}

void launch_softmax_rows(float* x, int64_t ld, int rows, int L, float scale, hipStream_t st) {
  if (L > 1024) throw std::runtime_error("softmax: L > 1024");
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, ld, rows, L, scale);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- row broadcast
__global__ void broadcast_rows_kernel(const float* __restrict__ src, int nsrc, float* __restrict__ dst, int rows, int C) {
  const int64_t n = (int64_t)rows * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / C;
    const int c = i - r * C;
    dst[i] = src[(r % nsrc) * C + c];
  }
}

void launch_broadcast_rows(const float* src, int nsrc, float* dst, int rows, int C, hipStream_t st) {
  const int64_t n = (int64_t)rows * C;
  hipLaunchKernelGGL(broadcast_rows_kernel, dim3(grid_for(n)), dim3(256), 0, st, src, nsrc, dst, rows, C);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- activations
__device__ inline float mish_f(float x) {
  // x * tanh(softplus(x)); softplus with PyTorch's threshold 20 (F.softplus default).
  const float sp = x > 20.f ? x : log1pf(expf(x));
  return x * tanhf(sp);
}

__global__ void activation_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int act) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    y[i] = act == 0 ? mish_f(v) : fmaxf(v, 0.f);
  }
}

void launch_activation(const float* x, float* y, int64_t n, int act, hipStream_t st) {
  hipLaunchKernelGGL(activation_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n, act);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
