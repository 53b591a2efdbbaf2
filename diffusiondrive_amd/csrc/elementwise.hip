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

__global__ void set_ptrs_kernel(const float** tab, const float* a, const float* b) {
  if (threadIdx.x == 0) {
    tab[0] = a;
    tab[1] = b;
  }
}

void launch_set_ptrs(const float** tab, const float* a, const float* b, hipStream_t st) {
  hipLaunchKernelGGL(set_ptrs_kernel, dim3(1), dim3(64), 0, st, tab, a, b);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_nchw_to_nhwc(const float* in, float* out, int B, int C, int H, int W, int Cp, hipStream_t st) {
  if (C > 8 || Cp < C) throw std::runtime_error("nchw_to_nhwc: unsupported channel count");
  const int64_t n = (int64_t)B * H * W;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, out, B, C, H, W, Cp);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- maxpool 3x3 s2 p1 (timm stem)
// One block row per output row (blockIdx.z = b, blockIdx.y = oy): 32-bit index math, float4 channel vectors along x.
__global__ void maxpool_kernel(const float4* __restrict__ in, float4* __restrict__ out, int H, int W, int C4,
                               int Ho, int Wo) {
  const int b = blockIdx.z, oy = blockIdx.y;
  const int row = b * Ho + oy;
  const int n = Wo * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int ox = i / C4, c = i - ox * C4;
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int y = oy * 2 - 1 + dy;
      if ((unsigned)y >= (unsigned)H) continue;
      const float4* rowp = in + ((size_t)b * H + y) * W * C4 + c;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int x = ox * 2 - 1 + dx;
        if ((unsigned)x >= (unsigned)W) continue;
        const float4 v = rowp[(size_t)x * C4];
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    out[(size_t)row * n + i] = m;
  }
}

void launch_maxpool3x3s2(const float* in, float* out, int B, int H, int W, int C, int Ho, int Wo,
                         hipStream_t st) {
  if (C % 4) throw std::runtime_error("maxpool: C % 4 != 0");
  const int n = Wo * (C / 4);
  dim3 grid((n + 255) / 256, Ho, B);
  hipLaunchKernelGGL(maxpool_kernel, grid, dim3(256), 0, st, reinterpret_cast<const float4*>(in),
                     reinterpret_cast<float4*>(out), H, W, C / 4, Ho, Wo);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- adaptive avg pool (exact windows)
// transfuser_backbone.py:47-58,249-250: windows divide exactly at every scale. One block row per
// output row (b, y), threads over (x, c); the window sum runs in the reference's (dy, dx) order.
__global__ void avgpool_kernel(const float* __restrict__ in, int H, int W, int C, int oh, int ow, View4 out,
                               const float* __restrict__ add) {
  const int kh = H / oh, kw = W / ow;
  const float inv = 1.0f / (float)(kh * kw);
  const int b = blockIdx.z, y = blockIdx.y;
  const int n = ow * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int x = i / C, c = i - x * C;
    float s = 0.f;
    for (int dy = 0; dy < kh; ++dy) {
      const float* r = in + (((size_t)b * H + (size_t)y * kh + dy) * W + (size_t)x * kw) * C + c;
      for (int dx = 0; dx < kw; ++dx) s += r[(size_t)dx * C];
    }
    float v = s * inv;
    if (add) v += add[((size_t)y * ow + x) * C + c];
    out.p[(int64_t)b * out.sn + (int64_t)y * out.sh + (int64_t)x * out.sw + (int64_t)c * out.sc] = v;
  }
}

void launch_avgpool(const float* in, int B, int H, int W, int C, int oh, int ow, View4 out, const float* add,
                    hipStream_t st) {
  if (H % oh || W % ow) throw std::runtime_error("avgpool: non-integer window");
  const int n = ow * C;
  dim3 grid((n + 255) / 256, oh, B);
  hipLaunchKernelGGL(avgpool_kernel, grid, dim3(256), 0, st, in, H, W, C, oh, ow, out, add);
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

// One block row per output row (b, y) (the y taps are block-uniform); threads over (x, channel
// vector). VEC = 4: float4 channel vectors (unit channel stride, 16-B aligned rows); VEC = 1: any
// strides. Same arithmetic order as the scalar form (fp-contract off for this file).
template <int VEC>
__global__ void bilinear_kernel(View4 in, int Hi, int Wi, int C, View4 out, int Ho, int Wo, float rh, float rw,
                                int accumulate) {
  const int b = blockIdx.z, y = blockIdx.y;
  int y0, y1;
  float ly0, ly1;
  bl_index(y, rh, Hi, y0, y1, ly0, ly1);
  const int CV = C / VEC;
  const int n = Wo * CV;
  const float* base = in.p + (int64_t)b * in.sn;
  float* obase = out.p + (int64_t)b * out.sn + (int64_t)y * out.sh;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int x = i / CV, cv = i - x * CV;
    int x0, x1;
    float lx0, lx1;
    bl_index(x, rw, Wi, x0, x1, lx0, lx1);
    if constexpr (VEC == 4) {
      const int c = cv * 4;
      const float4 v00 = *reinterpret_cast<const float4*>(base + y0 * in.sh + x0 * in.sw + c);
      const float4 v01 = *reinterpret_cast<const float4*>(base + y0 * in.sh + x1 * in.sw + c);
      const float4 v10 = *reinterpret_cast<const float4*>(base + y1 * in.sh + x0 * in.sw + c);
      const float4 v11 = *reinterpret_cast<const float4*>(base + y1 * in.sh + x1 * in.sw + c);
      float4 v;
      v.x = ly0 * (lx0 * v00.x + lx1 * v01.x) + ly1 * (lx0 * v10.x + lx1 * v11.x);
      v.y = ly0 * (lx0 * v00.y + lx1 * v01.y) + ly1 * (lx0 * v10.y + lx1 * v11.y);
      v.z = ly0 * (lx0 * v00.z + lx1 * v01.z) + ly1 * (lx0 * v10.z + lx1 * v11.z);
      v.w = ly0 * (lx0 * v00.w + lx1 * v01.w) + ly1 * (lx0 * v10.w + lx1 * v11.w);
      float4* o = reinterpret_cast<float4*>(obase + (int64_t)x * out.sw + c);
      if (accumulate) {
        const float4 p = *o;
        v.x = p.x + v.x;
        v.y = p.y + v.y;
        v.z = p.z + v.z;
        v.w = p.w + v.w;
      }
      *o = v;
    } else {
      const int c = cv;
      const float* cb = base + (int64_t)c * in.sc;
      const float v00 = cb[y0 * in.sh + x0 * in.sw];
      const float v01 = cb[y0 * in.sh + x1 * in.sw];
      const float v10 = cb[y1 * in.sh + x0 * in.sw];
      const float v11 = cb[y1 * in.sh + x1 * in.sw];
      const float v = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
      float* o = obase + (int64_t)x * out.sw + (int64_t)c * out.sc;
      *o = accumulate ? (*o + v) : v;
    }
  }
}

// VEC = 4 upsample-add over HBM-sized maps: kBlU channel vectors per thread (block-strided), every destination
// load issued before the first is used (kBlU x the bytes in flight of bilinear_kernel<4>'s one per thread); the
// per-element arithmetic is bilinear_kernel<4>'s, so the result is bit-identical.
constexpr int kBlU = 2;  // vectors per thread (same-box bench A/B: 2 -5 % against 4, 8 +4 %)
__global__ __launch_bounds__(256) void bilinear_add4_kernel(View4 in, int Hi, int Wi, int C, View4 out, int Ho,
                                                            int Wo, float rh, float rw) {
  const int b = blockIdx.z, y = blockIdx.y;
  int y0, y1;
  float ly0, ly1;
  bl_index(y, rh, Hi, y0, y1, ly0, ly1);
  const int CV = C / 4;
  const int n = Wo * CV;
  const float* __restrict__ base = in.p + (int64_t)b * in.sn;
  float* __restrict__ obase = out.p + (int64_t)b * out.sn + (int64_t)y * out.sh;
  const int i0 = blockIdx.x * (256 * kBlU) + threadIdx.x;
  float4 p[kBlU];
#pragma unroll
  for (int u = 0; u < kBlU; ++u) {
    const int i = i0 + u * 256;
    const int x = i / CV, c = (i - x * CV) * 4;
    p[u] = i < n ? *reinterpret_cast<const float4*>(obase + (int64_t)x * out.sw + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < kBlU; ++u) {
    const int i = i0 + u * 256;
    if (i >= n) break;
    const int x = i / CV, c = (i - x * CV) * 4;
    int x0, x1;
    float lx0, lx1;
    bl_index(x, rw, Wi, x0, x1, lx0, lx1);
    const float4 v00 = *reinterpret_cast<const float4*>(base + y0 * in.sh + x0 * in.sw + c);
    const float4 v01 = *reinterpret_cast<const float4*>(base + y0 * in.sh + x1 * in.sw + c);
    const float4 v10 = *reinterpret_cast<const float4*>(base + y1 * in.sh + x0 * in.sw + c);
    const float4 v11 = *reinterpret_cast<const float4*>(base + y1 * in.sh + x1 * in.sw + c);
    float4 v;
    v.x = ly0 * (lx0 * v00.x + lx1 * v01.x) + ly1 * (lx0 * v10.x + lx1 * v11.x);
    v.y = ly0 * (lx0 * v00.y + lx1 * v01.y) + ly1 * (lx0 * v10.y + lx1 * v11.y);
    v.z = ly0 * (lx0 * v00.z + lx1 * v01.z) + ly1 * (lx0 * v10.z + lx1 * v11.z);
    v.w = ly0 * (lx0 * v00.w + lx1 * v01.w) + ly1 * (lx0 * v10.w + lx1 * v11.w);
    v.x = p[u].x + v.x;
    v.y = p[u].y + v.y;
    v.z = p[u].z + v.z;
    v.w = p[u].w + v.w;
    // nontemporal output store (common.h epi_quads: +0.5 % scenes/s with all three sites)
    typedef float ntf4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store((ntf4){v.x, v.y, v.z, v.w}, reinterpret_cast<ntf4*>(obase + (int64_t)x * out.sw + c));
  }
}

void launch_bilinear(View4 in, int B, int Hi, int Wi, int C, View4 out, int Ho, int Wo, float ratio_h,
                     float ratio_w, int accumulate, hipStream_t st) {
  if (Ho > 65535 || B > 65535) throw std::runtime_error("bilinear: Ho / B > 65535");
  if ((int64_t)Hi * in.sh >= (int64_t(1) << 31) || (int64_t)Wo * out.sw >= (int64_t(1) << 31))
    throw std::runtime_error("bilinear: per-image extent too large");
  const bool vec = C % 4 == 0 && in.sc == 1 && out.sc == 1 && in.sh % 4 == 0 && in.sw % 4 == 0 &&
                   in.sn % 4 == 0 && out.sh % 4 == 0 && out.sw % 4 == 0 && out.sn % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(in.p) % 16 == 0 && reinterpret_cast<uintptr_t>(out.p) % 16 == 0;
  const int n = Wo * (vec ? C / 4 : C);
  // the in-place upsample-add onto a separate map (GPT fusion back into the trunks): the wide-issue form
  const bool sep = in.p + (int64_t)B * in.sn <= out.p || out.p + (int64_t)B * out.sn <= in.p;
  if (vec && accumulate && sep) {
    dim3 g4((n + 256 * kBlU - 1) / (256 * kBlU), Ho, B);
    hipLaunchKernelGGL(bilinear_add4_kernel, g4, dim3(256), 0, st, in, Hi, Wi, C, out, Ho, Wo, ratio_h, ratio_w);
    DD_HIP_CHECK(hipGetLastError());
    return;
  }
  dim3 grid((n + 255) / 256, Ho, B);
  if (vec)
    hipLaunchKernelGGL(bilinear_kernel<4>, grid, dim3(256), 0, st, in, Hi, Wi, C, out, Ho, Wo, ratio_h, ratio_w,
                       accumulate);
  else
    hipLaunchKernelGGL(bilinear_kernel<1>, grid, dim3(256), 0, st, in, Hi, Wi, C, out, Ho, Wo, ratio_h, ratio_w,
                       accumulate);
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
                                                        int film_div, int64_t film_ld,
                                                        float* y, int64_t ldy, int rows, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  if (fs && film_div > 0) {  // per-group FiLM rows (training head: one time embedding per scene)
    fs += (int64_t)(row / film_div) * film_ld;
    fb += (int64_t)(row / film_div) * film_ld;
  }
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

// Vectorised variant for power-of-two C >= 64 with 16-B aligned rows: a row is spread over LPR lanes
// (min(64, C/4)), each holding VPL float4 channel quads, so a wave normalises 64/LPR rows at once
// with 16-B loads / stores and a log2(LPR)-step reduction. Same two-pass arithmetic as above.
template <int LPR, int VPL>
__global__ __launch_bounds__(256) void layernorm_v4_kernel(const float* __restrict__ x, int64_t ldx,
                                                           const float* __restrict__ res, int64_t ldres, int res_div,
                                                           const float* __restrict__ g, const float* __restrict__ b,
                                                           const float* __restrict__ fs, const float* __restrict__ fb,
                                                           int film_div, int64_t film_ld,
                                                           float* y, int64_t ldy, int rows) {
  constexpr int C = LPR * 4 * VPL;
  const int sub = threadIdx.x % LPR;
  const int row = (blockIdx.x * 256 + threadIdx.x) / LPR;
  const bool live = row < rows;
  const int r = live ? row : rows - 1;  // dead lanes still join the xor reductions
  if (fs && film_div > 0) {  // per-group FiLM rows (training head: one time embedding per scene)
    fs += (int64_t)(r / film_div) * film_ld;
    fb += (int64_t)(r / film_div) * film_ld;
  }
  const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)r * ldx);
  const float4* rr = res ? reinterpret_cast<const float4*>(res + (int64_t)(r / res_div) * ldres) : nullptr;
  float4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    float4 t = xr[sub + LPR * i];
    if (rr) {
      const float4 u = rr[sub + LPR * i];
      t.x += u.x;
      t.y += u.y;
      t.z += u.z;
      t.w += u.w;
    }
    v[i] = t;
    s += (t.x + t.y) + (t.z + t.w);
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
    q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / (float)C + 1e-5f);
  if (!live) return;
  float4* yr = reinterpret_cast<float4*>(y + (int64_t)row * ldy);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c4 = sub + LPR * i;
    const float4 gg = reinterpret_cast<const float4*>(g)[c4], bb = reinterpret_cast<const float4*>(b)[c4];
    float4 o;
    o.x = (v[i].x - mean) * rstd * gg.x + bb.x;
    o.y = (v[i].y - mean) * rstd * gg.y + bb.y;
    o.z = (v[i].z - mean) * rstd * gg.z + bb.z;
    o.w = (v[i].w - mean) * rstd * gg.w + bb.w;
    if (fs) {
      const float4 a = reinterpret_cast<const float4*>(fs)[c4], c = reinterpret_cast<const float4*>(fb)[c4];
      o.x = o.x * (1.f + a.x) + c.x;
      o.y = o.y * (1.f + a.y) + c.y;
      o.z = o.z * (1.f + a.z) + c.z;
      o.w = o.w * (1.f + a.w) + c.w;
    }
#ifdef DDMI_NT2  // experiment build (DDMI_BUILD_VARIANT=nt2): nontemporal LayerNorm output stores
    typedef float ntf4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store((ntf4){o.x, o.y, o.z, o.w}, reinterpret_cast<ntf4*>(yr + c4));
#else
    yr[c4] = o;
#endif
  }
}

void launch_layernorm(const float* x, int64_t ldx, const float* res, int64_t ldres, int res_div, const float* g,
                      const float* b, const float* film_scale, const float* film_shift, float* y, int64_t ldy,
                      int rows, int C, hipStream_t st, int film_div, int64_t film_ld) {
  if (C > 2048) throw std::runtime_error("layernorm: C > 2048");
  if (rows == 0) return;
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool vec = C >= 64 && (C & (C - 1)) == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (!res || ldres % 4 == 0) &&
                   al(x) && al(y) && al(res) && al(g) && al(b) && al(film_scale) && al(film_shift);
  if (vec) {
    const int lpr = C / 4 < 64 ? C / 4 : 64;
    const dim3 grid((unsigned)(((int64_t)rows * lpr + 255) / 256));
    const int rd = res_div < 1 ? 1 : res_div;
#define LNV(L, V)                                                                                                  \
  hipLaunchKernelGGL((layernorm_v4_kernel<L, V>), grid, dim3(256), 0, st, x, ldx, res, ldres, rd, g, b, film_scale, \
                     film_shift, film_div, film_ld, y, ldy, rows)
    switch (C) {
      case 64: LNV(16, 1); break;
      case 128: LNV(32, 1); break;
      case 256: LNV(64, 1); break;
      case 512: LNV(64, 2); break;
      case 1024: LNV(64, 4); break;
      default: LNV(64, 8); break;
    }
#undef LNV
    DD_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, ldx, res, ldres,
                     res_div < 1 ? 1 : res_div, g, b, film_scale, film_shift, film_div, film_ld, y, ldy, rows, C);
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

// ---------------------------------------------------------------- device normal draw (noise == NULL)
// Philox4x32-10 (Salmon et al., SC'11) keyed by the 64-bit seed; counter (j, 0, 0, 0) for the j-th group of
// four normals, j = first / 4 + thread. Box-Muller on u = ((x >> 8) + 1) 2^-24 in (0, 1] and v = (y >> 8) 2^-24:
// r = sqrt(-2 ln u), normals r cos(2 pi v), r sin(2 pi v) from (x0, x1) and from (x2, x3).
__device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
    c[0] = n0;
    c[1] = n1;
    c[2] = n2;
    c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__global__ void normal_philox_kernel(float* __restrict__ out, int64_t n4, uint32_t k0, uint32_t k1, uint64_t group0) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const uint64_t g = group0 + (uint64_t)i;
  uint32_t c[4] = {(uint32_t)g, (uint32_t)(g >> 32), 0u, 0u};
  philox4x32_10(c, k0, k1);
  float4 o;
  float* po = &o.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float u = (float)((c[2 * h] >> 8) + 1u) * 5.9604644775390625e-8f;  // 2^-24
    const float v = (float)(c[2 * h + 1] >> 8) * 5.9604644775390625e-8f;
    const float r = sqrtf(-2.0f * logf(u));
    float s, co;
    sincospif(2.0f * v, &s, &co);
    po[2 * h] = r * co;
    po[2 * h + 1] = r * s;
  }
  reinterpret_cast<float4*>(out)[i] = o;
}

void launch_normal_philox(float* out, int64_t n, uint64_t seed, uint64_t first, hipStream_t st) {
  if (n % 4 || first % 4 || (reinterpret_cast<uintptr_t>(out) & 15))
    throw std::runtime_error("normal_philox: n and first must be multiples of 4, out 16-B aligned");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  hipLaunchKernelGGL(normal_philox_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, out, n4,
                     (uint32_t)seed, (uint32_t)(seed >> 32), first / 4);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
