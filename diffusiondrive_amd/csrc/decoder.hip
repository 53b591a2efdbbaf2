// Truncated-diffusion trajectory decoder kernels (TrajectoryHead.forward_test,
// transfuser_model_v2.py:578-641) plus the small attention used by both decoders.
// The dense Linear layers of the decoder run on the MFMA conv_gemm kernel; these kernels carry
// the per-query glue: DDIM arithmetic, sine embeddings, the BEV grid-sample attention gather,
// multi-head attention over <= 128 keys, and mode selection.
#include "common.h"

namespace ddmi {

static inline int blocks_for(int64_t n, int block = 256) { return (int)((n + block - 1) / block); }

// norm_odo / denorm_odo on (x, y) (transfuser_model_v2.py:480-500)
__device__ inline float norm_x(float x) { return 2.f * (x + 1.2f) / 56.9f - 1.f; }
__device__ inline float norm_y(float y) { return 2.f * (y + 20.f) / 46.f - 1.f; }
__device__ inline float denorm_x(float x) { return (x + 1.f) / 2.f * 56.9f - 1.2f; }
__device__ inline float denorm_y(float y) { return (y + 1.f) / 2.f * 46.f - 20.f; }

// ---------------------------------------------------------------- DDIM add_noise at t_trunc (:591-597)
__global__ void ddim_init_kernel(const float* __restrict__ anchor, const float* __restrict__ noise,
                                 float* __restrict__ img, int B, int QP, float sa, float s1a) {
  const int64_t n = (int64_t)B * QP;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int qp = i % QP;
  const float ax = anchor[qp * 2 + 0], ay = anchor[qp * 2 + 1];
  img[i * 2 + 0] = sa * norm_x(ax) + s1a * noise[i * 2 + 0];
  img[i * 2 + 1] = sa * norm_y(ay) + s1a * noise[i * 2 + 1];
}

void launch_ddim_init(const float* anchor, const float* noise, float* img, int B, int QP, float sa, float s1a,
                      hipStream_t st) {
  const int64_t n = (int64_t)B * QP;
  hipLaunchKernelGGL(ddim_init_kernel, dim3(blocks_for(n)), dim3(256), 0, st, anchor, noise, img, B, QP, sa, s1a);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- clamp + denorm + sine embed
// gen_sineembed_for_position(pos, 64) (blocks.py:22-40): per coordinate v,
// e[i] = (v * 2pi) / 10000^(2*(i//2)/32); even i -> sin, odd i -> cos; output cat(y-part, x-part).
// dim_t values are correctly rounded constants (10000^(j/16), j = 0..15).
__constant__ float c_dim_t[16];

__global__ void traj_embed_kernel(const float* __restrict__ img, float* __restrict__ pts, float* __restrict__ emb,
                                  int rows, int P) {
  // one thread per (row, point, 64-dim slot)
  const int64_t n = (int64_t)rows * P * 64;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int d = i & 63;
  const int64_t rp = i >> 6;  // row * P + p
  const float cx = fminf(fmaxf(img[rp * 2 + 0], -1.f), 1.f);
  const float cy = fminf(fmaxf(img[rp * 2 + 1], -1.f), 1.f);
  const float px = denorm_x(cx), py = denorm_y(cy);
  if (d == 0) {
    pts[rp * 2 + 0] = px;
    pts[rp * 2 + 1] = py;
  }
  const float scale = 6.283185307179586f;
  const int j = d & 31;
  const float v = (d < 32 ? py : px) * scale;
  const float a = v / c_dim_t[j >> 1];
  emb[rp * 64 + d] = (j & 1) ? cosf(a) : sinf(a);
}

void decoder_init_constants() {
  float t[16];
  for (int j = 0; j < 16; ++j) t[j] = (float)std::pow(10000.0, (double)j / 16.0);
  DD_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_dim_t), t, sizeof(t)));
}

void launch_traj_embed(const float* img, float* pts, float* emb, int rows, int P, hipStream_t st) {
  const int64_t n = (int64_t)rows * P * 64;
  hipLaunchKernelGGL(traj_embed_kernel, dim3(blocks_for(n)), dim3(256), 0, st, img, pts, emb, rows, P);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- SinusoidalPosEmb (conditional_unet1d.py:53-66)
__global__ void timestep_embed_kernel(float t, float* out, int dim) {
  const int half = dim / 2;
  const int i = threadIdx.x + blockIdx.x * blockDim.x;
  if (i >= half) return;
  const float e = (float)(-9.210340371976184 / (double)(half - 1));  // -ln(10000)/(half-1)
  const float f = expf((float)i * e);
  const float a = t * f;
  out[i] = sinf(a);
  out[half + i] = cosf(a);
}

void launch_timestep_embed(float t, float* out, int dim, hipStream_t st) {
  hipLaunchKernelGGL(timestep_embed_kernel, dim3(blocks_for(dim / 2)), dim3(256), 0, st, t, out, dim);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- BEV grid-sample attention (blocks.py:88-129)
// One wave64 per (scene, query); each lane owns 4 contiguous channels (C = 256 -> 1 KB NHWC rows,
// one coalesced float4 load per lane per bilinear tap). Zero padding, align_corners=False.
__global__ __launch_bounds__(256) void bev_sample_attn_kernel(const float* __restrict__ logits,
                                                              const float* __restrict__ pts,
                                                              const float* __restrict__ value,
                                                              float* __restrict__ out, int B, int Q, int P, int Hv,
                                                              int Wv, int C, float inv_max_x, float inv_max_y) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= B * Q) return;
  const int b = item / Q;
  const float* lg = logits + (int64_t)item * P;
  float mx = -INFINITY;
  for (int p = 0; p < P; ++p) mx = fmaxf(mx, lg[p]);
  float w[16];
  float s = 0.f;
  for (int p = 0; p < P; ++p) {
    w[p] = expf(lg[p] - mx);
    s += w[p];
  }
  const float inv = 1.f / s;
  const float* vb = value + (int64_t)b * Hv * Wv * C;
  for (int c4 = lane * 4; c4 < C; c4 += 256) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < P; ++p) {
      const float tx = pts[((int64_t)item * P + p) * 2 + 0];
      const float ty = pts[((int64_t)item * P + p) * 2 + 1];
      const float gx = ty * inv_max_x;  // grid x (width) <- trajectory y  (blocks.py:101-108)
      const float gy = tx * inv_max_y;  // grid y (height) <- trajectory x
      const float ix = ((gx + 1.f) * (float)Wv - 1.f) / 2.f;
      const float iy = ((gy + 1.f) * (float)Hv - 1.f) / 2.f;
      const float fx = floorf(ix), fy = floorf(iy);
      const int x0 = (int)fx, y0 = (int)fy;
      const int x1 = x0 + 1, y1 = y0 + 1;
      const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
      const float wne = (ix - (float)x0) * ((float)y1 - iy);
      const float wsw = ((float)x1 - ix) * (iy - (float)y0);
      const float wse = (ix - (float)x0) * (iy - (float)y0);
      float4 sp = make_float4(0.f, 0.f, 0.f, 0.f);
      auto tap = [&](int yy, int xx, float wt) {
        if ((unsigned)yy < (unsigned)Hv && (unsigned)xx < (unsigned)Wv) {
          const float4 v = *reinterpret_cast<const float4*>(vb + ((int64_t)yy * Wv + xx) * C + c4);
          sp.x += v.x * wt;
          sp.y += v.y * wt;
          sp.z += v.z * wt;
          sp.w += v.w * wt;
        }
      };
      tap(y0, x0, wnw);
      tap(y0, x1, wne);
      tap(y1, x0, wsw);
      tap(y1, x1, wse);
      const float wp = w[p] * inv;
      acc.x += wp * sp.x;
      acc.y += wp * sp.y;
      acc.z += wp * sp.z;
      acc.w += wp * sp.w;
    }
    *reinterpret_cast<float4*>(out + (int64_t)item * C + c4) = acc;
  }
}

void launch_bev_sample_attn(const float* logits, const float* pts, const float* value, float* out, int B, int Q,
                            int P, int Hv, int Wv, int C, float inv_max_x, float inv_max_y, hipStream_t st) {
  if (P > 16 || C % 4) throw std::runtime_error("bev_sample_attn: P <= 16 and C % 4 == 0 required");
  const int items = B * Q;
  hipLaunchKernelGGL(bev_sample_attn_kernel, dim3((items + 3) / 4), dim3(256), 0, st, logits, pts, value, out, B, Q,
                     P, Hv, Wv, C, inv_max_x, inv_max_y);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- gathered value rows for the BEV sampling
// value_proj is a 3x3 conv over the whole 64x64 BEV map (blocks.py:68-76,114), but grid_sample reads it
// at only B x Q x P x 4 bilinear taps (:115-122). The gathered form evaluates the conv at those taps:
// bev_tap_rows writes, per (scene, query, point, tap), the map pixel the tap reads (same ix / iy
// arithmetic as bev_sample_attn) or -1 when zero padding applies; conv_x3 evaluates the conv at those
// rows (ConvArgs::rowmap) into a compact (B*Q*P*4, C) array; bev_sample_attn_gathered then reads
// tap t of point p of item from row (item * P + p) * 4 + t. Tap order: nw, ne, sw, se.
__device__ inline void bev_tap_geometry(const float* pts, int64_t ip, int Hv, int Wv, float inv_max_x,
                                        float inv_max_y, int& x0, int& y0, float wt[4]) {
  const float tx = pts[ip * 2 + 0];
  const float ty = pts[ip * 2 + 1];
  const float gx = ty * inv_max_x;  // grid x (width) <- trajectory y  (blocks.py:101-108)
  const float gy = tx * inv_max_y;  // grid y (height) <- trajectory x
  const float ix = ((gx + 1.f) * (float)Wv - 1.f) / 2.f;
  const float iy = ((gy + 1.f) * (float)Hv - 1.f) / 2.f;
  const float fx = floorf(ix), fy = floorf(iy);
  x0 = (int)fx;
  y0 = (int)fy;
  const int x1 = x0 + 1, y1 = y0 + 1;
  wt[0] = ((float)x1 - ix) * ((float)y1 - iy);
  wt[1] = (ix - (float)x0) * ((float)y1 - iy);
  wt[2] = ((float)x1 - ix) * (iy - (float)y0);
  wt[3] = (ix - (float)x0) * (iy - (float)y0);
}

__global__ __launch_bounds__(256) void bev_tap_rows_kernel(const float* __restrict__ pts, int* __restrict__ rows,
                                                           int B, int Q, int P, int Hv, int Wv, float inv_max_x,
                                                           float inv_max_y) {
  const int64_t ip = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ip >= (int64_t)B * Q * P) return;
  const int b = (int)(ip / ((int64_t)Q * P));
  int x0, y0;
  float wt[4];
  bev_tap_geometry(pts, ip, Hv, Wv, inv_max_x, inv_max_y, x0, y0, wt);
  int4 r;
  auto px = [&](int yy, int xx) {
    return ((unsigned)yy < (unsigned)Hv && (unsigned)xx < (unsigned)Wv) ? (b * Hv + yy) * Wv + xx : -1;
  };
  r.x = px(y0, x0);
  r.y = px(y0, x0 + 1);
  r.z = px(y0 + 1, x0);
  r.w = px(y0 + 1, x0 + 1);
  *reinterpret_cast<int4*>(rows + ip * 4) = r;
}

// Deduplicated form: one workgroup per scene marks the map pixels its Q x P x 4 taps read in an
// LDS table, compacts them in pixel order into rows[b * cap .. b * cap + count) (the rest -1, so
// the conv's tiles past a scene's count exit at once; cap = Q * P * 4 keeps scene blocks at fixed
// offsets) and writes each tap's compact row (or -1 for a zero-padded tap) to slots.
__global__ __launch_bounds__(256) void bev_tap_dedup_kernel(const float* __restrict__ pts, int* __restrict__ rows,
                                                            int* __restrict__ slots, int Q, int P, int Hv, int Wv,
                                                            float inv_max_x, float inv_max_y) {
  __shared__ int table[4096];
  __shared__ int scan[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int HW = Hv * Wv, QP = Q * P, cap = QP * 4;
  const int64_t base = (int64_t)b * cap;
  for (int e = tid; e < HW; e += 256) table[e] = 0;
  __syncthreads();
  for (int u = tid; u < QP; u += 256) {
    int x0, y0;
    float wt[4];
    bev_tap_geometry(pts, (int64_t)b * QP + u, Hv, Wv, inv_max_x, inv_max_y, x0, y0, wt);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int yy = y0 + (t >> 1), xx = x0 + (t & 1);
      if ((unsigned)yy < (unsigned)Hv && (unsigned)xx < (unsigned)Wv) table[yy * Wv + xx] = 1;
    }
  }
  __syncthreads();
  // exclusive scan of the marks: thread t owns entries [t * E, t * E + E)
  const int E = (HW + 255) / 256;
  int cnt = 0;
  for (int e = tid * E; e < min(HW, tid * E + E); ++e) cnt += table[e];
  scan[tid] = cnt;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int v = tid >= off ? scan[tid - off] : 0;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  int r = scan[tid] - cnt;
  const int total = scan[255];
  for (int e = tid * E; e < min(HW, tid * E + E); ++e)
    if (table[e]) {
      table[e] = r;
      rows[base + r] = b * HW + e;
      ++r;
    }
  for (int j = total + tid; j < cap; j += 256) rows[base + j] = -1;
  __syncthreads();
  for (int u = tid; u < QP; u += 256) {
    int x0, y0;
    float wt[4];
    bev_tap_geometry(pts, (int64_t)b * QP + u, Hv, Wv, inv_max_x, inv_max_y, x0, y0, wt);
    int4 sl;
    auto slot = [&](int yy, int xx) {
      return ((unsigned)yy < (unsigned)Hv && (unsigned)xx < (unsigned)Wv) ? (int)(base + table[yy * Wv + xx]) : -1;
    };
    sl.x = slot(y0, x0);
    sl.y = slot(y0, x0 + 1);
    sl.z = slot(y0 + 1, x0);
    sl.w = slot(y0 + 1, x0 + 1);
    *reinterpret_cast<int4*>(slots + ((int64_t)b * QP + u) * 4) = sl;
  }
}

__global__ __launch_bounds__(256) void bev_sample_attn_gathered_kernel(
    const float* __restrict__ logits, const float* __restrict__ pts, const float* __restrict__ vrows,
    const int* __restrict__ slots, float* __restrict__ out, int B, int Q, int P, int Hv, int Wv, int C,
    float inv_max_x, float inv_max_y) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= B * Q) return;
  const float* lg = logits + (int64_t)item * P;
  float mx = -INFINITY;
  for (int p = 0; p < P; ++p) mx = fmaxf(mx, lg[p]);
  float w[16];
  float s = 0.f;
  for (int p = 0; p < P; ++p) {
    w[p] = expf(lg[p] - mx);
    s += w[p];
  }
  const float inv = 1.f / s;
  for (int c4 = lane * 4; c4 < C; c4 += 256) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < P; ++p) {
      const int64_t ip = (int64_t)item * P + p;
      int x0, y0;
      float wt[4];
      bev_tap_geometry(pts, ip, Hv, Wv, inv_max_x, inv_max_y, x0, y0, wt);
      float4 sp = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int yy = y0 + (t >> 1), xx = x0 + (t & 1);
        if ((unsigned)yy < (unsigned)Hv && (unsigned)xx < (unsigned)Wv) {
          // compact row of this tap: its own (ip * 4 + t) without dedup, else the scene's pixel slot
          const int64_t row = slots ? (int64_t)slots[ip * 4 + t] : ip * 4 + t;
          const float4 v = *reinterpret_cast<const float4*>(vrows + row * C + c4);
          sp.x += v.x * wt[t];
          sp.y += v.y * wt[t];
          sp.z += v.z * wt[t];
          sp.w += v.w * wt[t];
        }
      }
      const float wp = w[p] * inv;
      acc.x += wp * sp.x;
      acc.y += wp * sp.y;
      acc.z += wp * sp.z;
      acc.w += wp * sp.w;
    }
    *reinterpret_cast<float4*>(out + (int64_t)item * C + c4) = acc;
  }
}

void launch_bev_tap_rows(const float* pts, int* rows, int B, int Q, int P, int Hv, int Wv, float inv_max_x,
                         float inv_max_y, hipStream_t st) {
  const int64_t n = (int64_t)B * Q * P;
  if (n == 0) return;
  if ((int64_t)B * Hv * Wv >= (int64_t(1) << 31)) throw std::runtime_error("bev_tap_rows: map too large");
  hipLaunchKernelGGL(bev_tap_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pts, rows, B, Q, P,
                     Hv, Wv, inv_max_x, inv_max_y);
  DD_HIP_CHECK(hipGetLastError());
}

bool launch_bev_tap_dedup(const float* pts, int* rows, int* slots, int B, int Q, int P, int Hv, int Wv,
                          float inv_max_x, float inv_max_y, hipStream_t st) {
  if (Hv * Wv > 4096 || (int64_t)B * Q * P * 4 >= (int64_t(1) << 31) || (int64_t)B * Hv * Wv >= (int64_t(1) << 31))
    return false;
  if (B == 0) return true;
  hipLaunchKernelGGL(bev_tap_dedup_kernel, dim3(B), dim3(256), 0, st, pts, rows, slots, Q, P, Hv, Wv, inv_max_x,
                     inv_max_y);
  DD_HIP_CHECK(hipGetLastError());
  return true;
}

void launch_bev_sample_attn_gathered(const float* logits, const float* pts, const float* vrows, const int* slots,
                                     float* out, int B, int Q, int P, int Hv, int Wv, int C, float inv_max_x,
                                     float inv_max_y, hipStream_t st) {
  if (P > 16 || C % 4) throw std::runtime_error("bev_sample_attn: P <= 16 and C % 4 == 0 required");
  const int items = B * Q;
  if (items == 0) return;
  hipLaunchKernelGGL(bev_sample_attn_gathered_kernel, dim3((items + 3) / 4), dim3(256), 0, st, logits, pts, vrows,
                     slots, out, B, Q, P, Hv, Wv, C, inv_max_x, inv_max_y);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- small MHA (nn.MultiheadAttention core)
// One wave64 per (scene, head, query row): lanes own keys j and j+64 for the scores, softmax via
// wave shuffles, then lanes (d, half) accumulate the P.V product over half the keys each.
__global__ __launch_bounds__(256) void mha_small_kernel(const float* __restrict__ q, int64_t ldq,
                                                        const float* __restrict__ k, const float* __restrict__ v,
                                                        int64_t ldkv, float* __restrict__ out, int64_t ldo, int B,
                                                        int Lq, int Lk, int nh, int hd, int64_t qbs, int64_t kvbs,
                                                        int64_t obs) {
  __shared__ float pbuf[4][128];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wv;
  const bool active = item < B * nh * Lq;
  const int it = active ? item : 0;
  const int i = it % Lq;
  const int h = (it / Lq) % nh;
  const int b = it / (Lq * nh);
  const float* qr = q + b * qbs + (int64_t)i * ldq + h * hd;
  const float* kb = k + b * kvbs + h * hd;
  const float* vb = v + b * kvbs + h * hd;
  const float scale = 1.0f / sqrtf((float)hd);
  float s0 = -INFINITY, s1 = -INFINITY;
  if (lane < Lk) {
    float d = 0.f;
    for (int e = 0; e < hd; ++e) d += qr[e] * kb[(int64_t)lane * ldkv + e];
    s0 = d * scale;
  }
  if (lane + 64 < Lk) {
    float d = 0.f;
    for (int e = 0; e < hd; ++e) d += qr[e] * kb[(int64_t)(lane + 64) * ldkv + e];
    s1 = d * scale;
  }
  float m = fmaxf(s0, s1);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const float e0 = lane < Lk ? expf(s0 - m) : 0.f;
  const float e1 = lane + 64 < Lk ? expf(s1 - m) : 0.f;
  float sum = e0 + e1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  const float inv = 1.f / sum;
  pbuf[wv][lane] = e0 * inv;
  pbuf[wv][lane + 64] = e1 * inv;
  __syncthreads();
  const int halfsz = (Lk + 1) / 2;
  for (int d0 = 0; d0 < hd; d0 += 32) {
    const int d = d0 + (lane & 31);
    const int part = lane >> 5;
    float acc = 0.f;
    if (d < hd) {
      const int j0 = part * halfsz, j1 = min(Lk, j0 + halfsz);
      for (int j = j0; j < j1; ++j) acc += pbuf[wv][j] * vb[(int64_t)j * ldkv + d];
    }
    acc += __shfl_xor(acc, 32, 64);
    if (active && part == 0 && d < hd) out[b * obs + (int64_t)i * ldo + h * hd + d] = acc;
  }
}

// One workgroup per (scene, head): the head's Lq x hd queries and Lk x hd keys / values are staged in
// LDS with coalesced row loads (one global round trip instead of a dependent load chain per query
// row), then all Lq x Lk scores, the row softmaxes and the P.V product run out of LDS. Same
// arithmetic as mha_small_kernel (k-ordered dot, * scale, max / exp / sum / * 1/sum, j-ordered P.V).
__global__ __launch_bounds__(256) void mha_head_kernel(const float* __restrict__ q, int64_t ldq,
                                                       const float* __restrict__ k, const float* __restrict__ v,
                                                       int64_t ldkv, float* __restrict__ out, int64_t ldo, int Lq,
                                                       int Lk, int nh, int hd, int64_t qbs, int64_t kvbs, int64_t obs) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int hp = hd + 1;  // padded row pitch (conflict-free column walks)
  float* Qs = sm;                  // [Lq][hp]
  float* Ks = Qs + Lq * hp;        // [Lk][hp]
  float* Vs = Ks + Lk * hp;        // [Lk][hd]
  float* Ps = Vs + Lk * hd;        // [Lq][Lk + 1]
  const int pp = Lk + 1;
  const int h = blockIdx.x % nh, b = blockIdx.x / nh;
  const float* qb = q + b * qbs + h * hd;
  const float* kb = k + b * kvbs + h * hd;
  const float* vb = v + b * kvbs + h * hd;
  for (int t = threadIdx.x; t < Lq * hd; t += 256) {
    const int i = t / hd, e = t - i * hd;
    Qs[i * hp + e] = qb[(int64_t)i * ldq + e];
  }
  for (int t = threadIdx.x; t < Lk * hd; t += 256) {
    const int j = t / hd, e = t - j * hd;
    Ks[j * hp + e] = kb[(int64_t)j * ldkv + e];
    Vs[j * hd + e] = vb[(int64_t)j * ldkv + e];
  }
  __syncthreads();
  const float scale = 1.0f / sqrtf((float)hd);
  for (int t = threadIdx.x; t < Lq * Lk; t += 256) {
    const int i = t / Lk, j = t - i * Lk;
    float d = 0.f;
    for (int e = 0; e < hd; ++e) d += Qs[i * hp + e] * Ks[j * hp + e];
    Ps[i * pp + j] = d * scale;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = wv; i < Lq; i += 4) {
    float* pr = Ps + i * pp;
    const float s0 = lane < Lk ? pr[lane] : -INFINITY;
    const float s1 = lane + 64 < Lk ? pr[lane + 64] : -INFINITY;
    float m = fmaxf(s0, s1);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const float e0 = lane < Lk ? expf(s0 - m) : 0.f;
    const float e1 = lane + 64 < Lk ? expf(s1 - m) : 0.f;
    float sum = e0 + e1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    const float inv = 1.f / sum;
    if (lane < Lk) pr[lane] = e0 * inv;
    if (lane + 64 < Lk) pr[lane + 64] = e1 * inv;
  }
  __syncthreads();
  float* ob = out + b * obs + h * hd;
  for (int t = threadIdx.x; t < Lq * hd; t += 256) {
    const int i = t / hd, e = t - i * hd;
    const float* pr = Ps + i * pp;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc += pr[j] * Vs[j * hd + e];
    ob[(int64_t)i * ldo + e] = acc;
  }
}

void launch_mha_small(const float* q, int64_t ldq, const float* k, const float* v, int64_t ldkv, float* out,
                      int64_t ldo, int B, int Lq, int Lk, int nh, int hd, int64_t q_bstride, int64_t kv_bstride,
                      int64_t o_bstride, hipStream_t st) {
  if (Lk > 128 || Lk < 1) throw std::runtime_error("mha_small: 1 <= Lk <= 128 required");
  const size_t lds = sizeof(float) * ((size_t)Lq * (hd + 1) + (size_t)Lk * (hd + 1) + (size_t)Lk * hd +
                                      (size_t)Lq * (Lk + 1));
  if (lds <= 64 * 1024) {
    hipLaunchKernelGGL(mha_head_kernel, dim3(B * nh), dim3(256), lds, st, q, ldq, k, v, ldkv, out, ldo, Lq, Lk, nh,
                       hd, q_bstride, kv_bstride, o_bstride);
    DD_HIP_CHECK(hipGetLastError());
    return;
  }
  const int items = B * nh * Lq;

  hipLaunchKernelGGL(mha_small_kernel, dim3((items + 3) / 4), dim3(256), 0, st, q, ldq, k, v, ldkv, out, ldo, B, Lq,
                     Lk, nh, hd, q_bstride, kv_bstride, o_bstride);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- reg finalize (transfuser_model_v2.py:376-380)
__global__ void reg_finalize_kernel(const float* __restrict__ r, const float* __restrict__ pts, float* __restrict__ reg,
                                    float* __restrict__ pts_next, int rows, int P) {
  const int64_t n = (int64_t)rows * P;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = r[i * 3 + 0] + pts[i * 2 + 0];
  const float y = r[i * 3 + 1] + pts[i * 2 + 1];
  reg[i * 3 + 0] = x;
  reg[i * 3 + 1] = y;
  reg[i * 3 + 2] = tanhf(r[i * 3 + 2]) * 3.14159265358979323846f;
  if (pts_next) {
    pts_next[i * 2 + 0] = x;
    pts_next[i * 2 + 1] = y;
  }
}

void launch_reg_finalize(const float* r, const float* pts, float* reg, float* pts_next, int rows, int P,
                         hipStream_t st) {
  const int64_t n = (int64_t)rows * P;
  hipLaunchKernelGGL(reg_finalize_kernel, dim3(blocks_for(n)), dim3(256), 0, st, r, pts, reg, pts_next, rows, P);
  DD_HIP_CHECK(hipGetLastError());
}


// ---------------------------------------------------------------- DDIM step (eta = 0), diffusers semantics
struct StepCoef {
  float sa_t, sb_t, sa_p, sdir;
};

__global__ void ddim_step_kernel(const float* __restrict__ reg, float* __restrict__ img, int64_t n, StepCoef c) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x0x = norm_x(reg[i * 3 + 0]);
  const float x0y = norm_y(reg[i * 3 + 1]);
  const float sx = img[i * 2 + 0], sy = img[i * 2 + 1];
  const float ex = (sx - c.sa_t * x0x) / c.sb_t;
  const float ey = (sy - c.sa_t * x0y) / c.sb_t;
  const float cx = fminf(fmaxf(x0x, -1.f), 1.f);
  const float cy = fminf(fmaxf(x0y, -1.f), 1.f);
  img[i * 2 + 0] = c.sa_p * cx + c.sdir * ex;
  img[i * 2 + 1] = c.sa_p * cy + c.sdir * ey;
}

void launch_ddim_step(const float* reg, float* img, int rows, int P, float a_t, float a_prev, hipStream_t st) {
  StepCoef c;
  c.sa_t = std::sqrt(a_t);
  c.sb_t = std::sqrt(1.0f - a_t);
  c.sa_p = std::sqrt(a_prev);
  c.sdir = std::sqrt(1.0f - a_prev);
  const int64_t n = (int64_t)rows * P;
  hipLaunchKernelGGL(ddim_step_kernel, dim3(blocks_for(n)), dim3(256), 0, st, reg, img, n, c);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- argmax mode selection (:637-641)
__global__ void select_mode_kernel(const float* __restrict__ cls, const float* __restrict__ reg, float* __restrict__ traj,
                                   int* __restrict__ idx, int B, int Q, int P) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int best = 0;
  float bv = cls[(int64_t)b * Q];
  for (int q = 1; q < Q; ++q) {
    const float v = cls[(int64_t)b * Q + q];
    if (v > bv || (v != v && bv == bv)) {  // first maximal index; NaN propagates like torch.argmax
      bv = v;
      best = q;
    }
  }
  if (idx) idx[b] = best;
  const float* src = reg + ((int64_t)b * Q + best) * P * 3;
  for (int e = 0; e < P * 3; ++e) traj[(int64_t)b * P * 3 + e] = src[e];
}

void launch_select_mode(const float* cls, const float* reg, float* traj, int* idx, int B, int Q, int P,
                        hipStream_t st) {
  hipLaunchKernelGGL(select_mode_kernel, dim3(blocks_for(B, 64)), dim3(64), 0, st, cls, reg, traj, idx, B, Q, P);
  DD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- agent head post (:194-205)
__global__ void agent_post_kernel(float* s, int rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  float* r = s + (int64_t)i * 5;
  r[0] = tanhf(r[0]) * 32.f;
  r[1] = tanhf(r[1]) * 32.f;
  r[2] = tanhf(r[2]) * 3.14159265358979323846f;
}

void launch_agent_post(float* states, int rows, hipStream_t st) {
  hipLaunchKernelGGL(agent_post_kernel, dim3(blocks_for(rows)), dim3(256), 0, st, states, rows);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
