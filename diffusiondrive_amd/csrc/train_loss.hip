// Loss evaluator of the training-mode trajectory head: the per-scene pieces of
// TrajectoryHead.forward_train (transfuser_model_v2.py:520-576) that differ from forward_test - per-scene DDIM
// coefficients and time embeddings - and the losses: LossComputer (modules/multimodal_loss.py:119-168: nearest-anchor
// mode, sigmoid focal loss over the 20 logits, L1 of the selected mode against the target) and the BEV-semantic
// cross entropy of transfuser_loss (transfuser_loss.py:28-29).
//
// Reductions are deterministic: per-scene (or per-workgroup) partial sums in a fixed order, then one workgroup sums
// the partials in index order. Built with -ffp-contract=off: every mul / add rounds like PyTorch-CPU's separate ops.
#include "common.h"

namespace ddmi {

namespace {

__device__ inline float norm_xt(float x) { return 2.f * (x + 1.2f) / 56.9f - 1.f; }
__device__ inline float norm_yt(float y) { return 2.f * (y + 20.f) / 46.f - 1.f; }

// tree sum over the 256 threads of a block (fixed order)
__device__ inline float block_sum256(float v, float* sh) {
  const int tid = threadIdx.x;
  sh[tid] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) sh[tid] = sh[tid] + sh[tid + s];
    __syncthreads();
  }
  const float r = sh[0];
  __syncthreads();
  return r;
}

// torch.binary_cross_entropy_with_logits (no weight, no pos_weight) as ATen's CPU kernel evaluates it:
// (1 - t) * x + max_val + log(exp(-max_val) + exp(-x - max_val)), max_val = max(-x, 0)
__device__ inline float bce_logits(float x, float t) {
  const float mv = fmaxf(-x, 0.f);
  return (1.f - t) * x + mv + logf(expf(-mv) + expf(-x - mv));
}

}  // namespace

// diffusers add_noise coefficients per scene: sa = alphas_cumprod[t] ** 0.5, s1a = (1 - alphas_cumprod[t]) ** 0.5
__global__ void train_coeffs_kernel(const int* __restrict__ t, const float* __restrict__ ac, float* sa, float* s1a,
                                    int B, int tmax) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int k = t[b];
  k = k < 0 ? 0 : (k >= tmax ? tmax - 1 : k);
  const float a = ac[k];
  sa[b] = sqrtf(a);
  s1a[b] = sqrtf(1.f - a);
}

// img = sa[b] * norm_odo(anchor) + s1a[b] * noise (forward_train :536-540, before the clamp)
__global__ void train_noisy_kernel(const float* __restrict__ anchor, const float* __restrict__ noise,
                                   const float* __restrict__ sa, const float* __restrict__ s1a, float* img, int B,
                                   int QP) {
  const int64_t n = (int64_t)B * QP;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int b = (int)(i / QP), qp = (int)(i % QP);
  const float ax = anchor[qp * 2 + 0], ay = anchor[qp * 2 + 1];
  img[i * 2 + 0] = sa[b] * norm_xt(ax) + s1a[b] * noise[i * 2 + 0];
  img[i * 2 + 1] = sa[b] * norm_yt(ay) + s1a[b] * noise[i * 2 + 1];
}

// SinusoidalPosEmb(dim) of every scene's timestep (conditional_unet1d.py:53-66): out[b][dim]
__global__ void timestep_embed_rows_kernel(const int* __restrict__ t, float* out, int B, int dim) {
  const int half = dim / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * half) return;
  const int b = i / half, j = i % half;
  const float e = (float)(-9.210340371976184 / (double)(half - 1));  // -ln(10000)/(half-1)
  const float f = expf((float)j * e);
  const float a = (float)t[b] * f;
  out[(int64_t)b * dim + j] = sinf(a);
  out[(int64_t)b * dim + half + j] = cosf(a);
}

// LossComputer per scene (multimodal_loss.py:131-168): mode = argmin_m mean_p ||target_p[:2] - anchor_{m,p}||;
// part[b] = (sum_m focal(cls[b, m], onehot(mode)), sum_{p,c} |reg[b, mode, p, c] - target[b, p, c]|)
__global__ __launch_bounds__(64) void traj_loss_scene_kernel(const float* __restrict__ reg, const float* __restrict__ cls,
                                                             const float* __restrict__ target,
                                                             const float* __restrict__ anchor, float* part, int Q,
                                                             int P, float alpha, float gamma) {
  const int b = blockIdx.x, lane = threadIdx.x;
  __shared__ float dist[64];
  __shared__ int mode_s;
  __shared__ float foc[64];
  const float* tg = target + (int64_t)b * P * 3;
  if (lane < Q) {
    float s = 0.f;
    for (int p = 0; p < P; ++p) {
      const float dx = tg[p * 3 + 0] - anchor[(lane * P + p) * 2 + 0];
      const float dy = tg[p * 3 + 1] - anchor[(lane * P + p) * 2 + 1];
      s = s + sqrtf(dx * dx + dy * dy);
    }
    dist[lane] = s / (float)P;
  }
  __syncthreads();
  if (lane == 0) {
    int m = 0;
    for (int q = 1; q < Q; ++q)
      if (dist[q] < dist[m]) m = q;  // torch.argmin: the first minimum
    mode_s = m;
  }
  __syncthreads();
  const int mode = mode_s;
  float f = 0.f;
  if (lane < Q) {
    const float x = cls[(int64_t)b * Q + lane];
    const float t = lane == mode ? 1.f : 0.f;
    const float ps = 1.f / (1.f + expf(-x));
    const float pt = (1.f - ps) * t + ps * (1.f - t);
    const float fw = (alpha * t + (1.f - alpha) * (1.f - t)) * (gamma == 2.f ? pt * pt : powf(pt, gamma));
    f = bce_logits(x, t) * fw;
  }
  foc[lane] = f;
  __syncthreads();
  if (lane == 0) {
    float fs = 0.f, ls = 0.f;
    for (int q = 0; q < Q; ++q) fs = fs + foc[q];
    const float* rg = reg + ((int64_t)b * Q + mode) * P * 3;
    for (int e = 0; e < P * 3; ++e) ls = ls + fabsf(rg[e] - tg[e]);
    part[2 * b + 0] = fs;
    part[2 * b + 1] = ls;
  }
}

// loss = cls_w * (sum_b focal_b) / (B Q) + reg_w * (sum_b l1_b) / (B P 3), sums over b in index order (one block)
__global__ __launch_bounds__(256) void traj_loss_reduce_kernel(const float* __restrict__ part, float* out, int B, int Q,
                                                               int P, float cls_w, float reg_w) {
  __shared__ float sh[256];
  float fs = 0.f, ls = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    fs = fs + part[2 * b + 0];
    ls = ls + part[2 * b + 1];
  }
  fs = block_sum256(fs, sh);
  ls = block_sum256(ls, sh);
  if (threadIdx.x == 0) {
    const float fm = fs / (float)((int64_t)B * Q);
    const float lm = ls / (float)((int64_t)B * P * 3);
    out[0] = cls_w * fm + reg_w * lm;
  }
}

// BEV-semantic cross entropy partials: logits (B, C, H, W) NCHW (the reference's layout of bev_semantic_map), target
// ids (B, H, W) uint8; each block sums -log softmax(logits)[target] over its pixels in a fixed order
__global__ __launch_bounds__(256) void bev_ce_partial_kernel(const float* __restrict__ logits,
                                                             const uint8_t* __restrict__ target, float* part, int B,
                                                             int C, int HW) {
  __shared__ float sh[256];
  const int64_t n = (int64_t)B * HW;
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  float v = 0.f;
  if (i < n) {
    const int64_t b = i / HW, px = i % HW;
    const float* l = logits + b * C * HW + px;
    float mx = l[0];
    for (int c = 1; c < C; ++c) mx = fmaxf(mx, l[(int64_t)c * HW]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s = s + expf(l[(int64_t)c * HW] - mx);
    const int t = target[i];
    // an id outside [0, C) (F.cross_entropy raises on it) poisons the loss instead of reading past the logits
    v = t < C ? (logf(s) + mx) - l[(int64_t)t * HW] : __builtin_nanf("");
  }
  v = block_sum256(v, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}

__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part, int n, float denom,
                                                           float* out) {
  __shared__ float sh[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s = s + part[i];
  s = block_sum256(s, sh);
  if (threadIdx.x == 0) out[0] = s / denom;
}

__global__ void add2_kernel(float* o) { o[2] = o[0] + o[1]; }

void launch_add2(float* o, hipStream_t st) {
  hipLaunchKernelGGL(add2_kernel, dim3(1), dim3(1), 0, st, o);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_train_coeffs(const int* t, const float* ac, float* sa, float* s1a, int B, int tmax, hipStream_t st) {
  hipLaunchKernelGGL(train_coeffs_kernel, dim3((B + 255) / 256), dim3(256), 0, st, t, ac, sa, s1a, B, tmax);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_train_noisy(const float* anchor, const float* noise, const float* sa, const float* s1a, float* img, int B,
                        int QP, hipStream_t st) {
  const int64_t n = (int64_t)B * QP;
  hipLaunchKernelGGL(train_noisy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, anchor, noise, sa, s1a,
                     img, B, QP);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_timestep_embed_rows(const int* t, float* out, int B, int dim, hipStream_t st) {
  const int n = B * (dim / 2);
  hipLaunchKernelGGL(timestep_embed_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, t, out, B, dim);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_traj_loss_scene(const float* reg, const float* cls, const float* target, const float* anchor, float* part,
                            int B, int Q, int P, hipStream_t st) {
  if (Q > 64) throw std::runtime_error("traj_loss: Q > 64");
  hipLaunchKernelGGL(traj_loss_scene_kernel, dim3(B), dim3(64), 0, st, reg, cls, target, anchor, part, Q, P, 0.25f,
                     2.0f);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_traj_loss_reduce(const float* part, float* out, int B, int Q, int P, float cls_w, float reg_w,
                             hipStream_t st) {
  hipLaunchKernelGGL(traj_loss_reduce_kernel, dim3(1), dim3(256), 0, st, part, out, B, Q, P, cls_w, reg_w);
  DD_HIP_CHECK(hipGetLastError());
}

size_t bev_ce_partials(int B, int HW) { return (size_t)(((int64_t)B * HW + 255) / 256); }

void launch_bev_ce(const float* logits, const uint8_t* target, float* part, float* out, int B, int C, int HW,
                   hipStream_t st) {
  const int nb = (int)bev_ce_partials(B, HW);
  hipLaunchKernelGGL(bev_ce_partial_kernel, dim3(nb), dim3(256), 0, st, logits, target, part, B, C, HW);
  DD_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, st, part, nb, (float)((int64_t)B * HW), out);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
