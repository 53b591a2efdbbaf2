// Latency-bound small GEMMs / 1x1 convs on fp32 MFMA (v_mfma_f32_16x16x4_f32): the decoder's
// per-mode Linear layers (M = B x 20 rows: plan_anchor_encoder, cross-attention projections, FFN,
// cls / reg branches; transfuser_model_v2.py:208-256,297-382,459-468), the tf decoder's (M = B x 31,
// :73-82), the time MLP and FiLM (M = 1) and the agent / status heads.
//
// Those GEMMs have M x N of 1e3 - 1e6 and K = 256 .. 1024: a tiled implicit GEMM walks K in 32-wide
// chunks, each paying a global-load round trip, so a 5-GFLOP decoder GEMM took 12-15 us at 11 TF/s.
// Here the whole K of a 16 x 64 output tile is in flight at once:
//  * 4 waves split K in quarters; inside a wave, lane group g = lane >> 4 takes every 4th 16-B
//    quad of the quarter (k = 16 j + 4 g + 0..3: the MFMA k index is permuted per lane - same sum,
//    different fp32 order), so every operand load is a 16-B vector load of the lane's own A / W
//    row and the 4 lane groups of one row read 64 contiguous bytes; 16 floats per operand row per
//    chunk, the next chunk prefetched under the current chunk's 64 MFMAs.
//  * The four K-quarter partial tiles meet in LDS (fixed order w = 0..3), then 256 threads run
//    the conv_gemm epilogue (alpha, bias, residual, ReLU, strided NHWC store).
// Arithmetic: exact fp32 products (f32 MFMA), fp32 sums - at least as accurate as conv_gemm / f16x3.
#include "common.h"

namespace ddmi {

namespace {

typedef float gl_f4 __attribute__((ext_vector_type(4)));

constexpr int kTM = 16, kTN = 64, kKC = 16;  // tile rows, tile cols, k floats per lane per chunk

__global__ __launch_bounds__(256) void gemm_lat_kernel(ConvArgs a, int M, int K) {
  __shared__ float red[4][kTM * kTN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * kTM, n0 = blockIdx.y * kTN;
  const int HW = a.Ho * a.Wo;
  // A row of this lane (clamped: rows past M compute garbage that is never stored)
  const float* arow;
  {
    const int m = min(m0 + r, M - 1);
    const int n = m / HW, rem = m - n * HW;
    const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
    arow = a.in + (int64_t)n * a.in_sn + (int64_t)oh * a.stride * a.in_sh + (int64_t)ow * a.stride * a.in_sw;
  }
  const float* brow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) brow[j] = a.wgt + (int64_t)min(n0 + 16 * j + r, a.Cout - 1) * a.ldb;
  const int k0 = wave * (K / 4) + 4 * g;       // this lane's first float; quads every 16 floats
  const int nch = K / 16 / kKC;

  gl_f4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = (gl_f4){0.f, 0.f, 0.f, 0.f};
  gl_f4 ac[kKC / 4], bc[4][kKC / 4], an[kKC / 4], bn[4][kKC / 4];
  auto load = [&](gl_f4* av, gl_f4 (*bv)[kKC / 4], int c) {
    const int k = k0 + c * 4 * kKC;
#pragma unroll
    for (int i = 0; i < kKC / 4; ++i) av[i] = *reinterpret_cast<const gl_f4*>(arow + k + 16 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < kKC / 4; ++i) bv[j][i] = *reinterpret_cast<const gl_f4*>(brow[j] + k + 16 * i);
  };
  load(ac, bc, 0);
  for (int c = 0; c < nch; ++c) {
    // next chunk (clamped to the last one: an unconditional load keeps the waitcnt exact; with one
    // chunk the prefetch is skipped uniformly)
    if (nch > 1) load(an, bn, min(c + 1, nch - 1));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kKC / 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[i].x, bc[j][i].x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[i].y, bc[j][i].y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[i].z, bc[j][i].z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[i].w, bc[j][i].w, acc[j], 0, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kKC / 4; ++i) {
      ac[i] = an[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bc[j][i] = bn[j][i];
    }
  }
  // partial tile of this K quarter: D row 4 g + e (tile row), column r of N-subtile j
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave][(4 * g + e) * kTN + 16 * j + r] = acc[j][e];
  __syncthreads();
  // epilogue: thread t -> tile row t / 16, 4 consecutive columns
  const int tr = threadIdx.x >> 4, tc = (threadIdx.x & 15) * 4;
  const int m = m0 + tr;
  if (m >= M) return;
  const int n = m / HW, rem = m - n * HW;
  const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
  float* orow = a.out + (int64_t)n * a.out_sn + (int64_t)oh * a.out_sh + (int64_t)ow * a.out_sw;
  const float* rrow = a.res ? a.res + (int64_t)n * a.res_sn + (int64_t)oh * a.res_sh + (int64_t)ow * a.res_sw : nullptr;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int col = n0 + tc + e;
    if (col >= a.Cout) break;
    const int o = tr * kTN + tc + e;
    const float s = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
    float v = s * a.alpha + (a.bias ? a.bias[col] : 0.f);
    if (rrow) v += rrow[col];
    if (a.relu) v = fmaxf(v, 0.f);
    orow[col] = v;
  }
}

}  // namespace

// Returns false when the GEMM is not a small 1x1 / linear shape this kernel covers (the caller then
// takes the tiled kernels). Off by default (DDMI_GEMM_LAT=1 enables it): measured in the B = 64 bench
// graph it LOSES to conv_x3's 64 x 64 f16x3 tiles (18.32 vs 17.98 ms per forward; rocprof: 9.3 us vs
// 12.7 us for conv_gemm-fp32 at 1280 x 256 x 256, but 70 vs 31 us at 4096 x 512 x 512) - kept as the
// exact-fp32 option and for the record.
bool launch_gemm_lat(const ConvArgs& a, hipStream_t st) {
  static const int on = getenv("DDMI_GEMM_LAT") ? atoi(getenv("DDMI_GEMM_LAT")) : 0;
  if (!on) return false;
  if (a.KH != 1 || a.KW != 1 || a.pad != 0 || a.batch != 1 || a.b_kn || !a.wgt) return false;
  const int K = a.Cin;
  if (K % (16 * kKC) != 0 || K > 4096 || a.ldb % 4 || a.in_sw % 4 || a.in_sh % 4 || a.in_sn % 4) return false;
  if ((reinterpret_cast<uintptr_t>(a.in) & 15) || (reinterpret_cast<uintptr_t>(a.wgt) & 15)) return false;
  const int64_t M64 = (int64_t)a.Nimg * a.Ho * a.Wo;
  if (M64 == 0 || a.Cout == 0) return false;
  const int64_t tiles = ((M64 + kTM - 1) / kTM) * ((a.Cout + kTN - 1) / kTN);
  // small problems only: the tiled kernels win once there are thousands of tiles of work
  static const int64_t max_m = getenv("DDMI_GEMM_LAT_MAXM") ? atoll(getenv("DDMI_GEMM_LAT_MAXM")) : 4160;
  if (M64 > max_m || tiles > 2048) return false;
  const dim3 grid((unsigned)((M64 + kTM - 1) / kTM), (unsigned)((a.Cout + kTN - 1) / kTN));
  hipLaunchKernelGGL(gemm_lat_kernel, grid, dim3(256), 0, st, a, (int)M64, K);
  DD_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace ddmi
