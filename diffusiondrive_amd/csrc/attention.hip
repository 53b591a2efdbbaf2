// Fused GPT self-attention core of the Transfuser fusion transformer (transfuser_backbone.py
// :386-410, SelfAttention.forward): per (scene, head)
//     att = softmax((q @ k^T) * 1/sqrt(hs));  y = att @ v          (attn / resid dropout: eval no-ops)
// on fp32 MFMA (v_mfma_f32_16x16x4_f32), one launch instead of score GEMM + softmax + value GEMM.
//
// Input qkv [B][T][3C] (the fused q | k | v projection, heads h*hs .. (h+1)*hs inside each third),
// output y [B][T][C] (heads re-interleaved, i.e. `y.transpose(1, 2).view(B, T, C)`).
//
// Workgroup = (scene, head, block of 64 query rows), 4 waves, the 64 x T score block in LDS:
//  1. S[64][T] = Q K^T: wave w takes every 4th 16-key tile against all four 16-row query tiles, so
//     each k fragment feeds 4 MFMA chains. The dot product's k index is permuted per lane: lane group
//     g = lane >> 4 owns the contiguous slice k in [g hs/4, (g+1) hs/4), so each lane feeds the MFMA
//     from 16-B loads of its own q / k row (the sum over k is the same; only fp32 summation order
//     differs from a GEMM library). The next key tile's fragment is loaded during this one's MFMAs.
//  2. S rows -> softmax(scale * s) in LDS (max, exp, sum, * 1/sum: the arithmetic of
//     softmax_rows_kernel, which this replaces), four threads per row.
//  3. Y[64][hs] = P V: same k permutation over the T keys (lane group g owns keys [g T/4, (g+1) T/4));
//     wave = (16-column tile, group of query tiles); P from LDS as 16-B reads, V as 64-B row segments
//     per 16 lanes, prefetched 8 keys ahead (L2-resident: a head's V is read by every query block).
// Bound: fp32 MFMA (2 * 2 T^2 hs FLOP per (scene, head)); operands stay in L2 (qkv of one scene
// 0.3-2.4 MB).
#include <cmath>
#include <cstdlib>

#include "common.h"

namespace ddmi {

namespace {

typedef float at_f4 __attribute__((ext_vector_type(4)));

__device__ inline float at_wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ inline float at_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

constexpr int kQB = 64;  // query rows per workgroup (4 tiles of 16)

template <int HS>
__global__ __launch_bounds__(256) void gpt_attn_kernel(const float* __restrict__ qkv, float* __restrict__ y, int T,
                                                       int C, int heads, int nqb, float scale) {
  constexpr int KQ = HS / 4;                // k slice per lane group in phase 1
  constexpr int KC = KQ <= 32 ? KQ : 16;    // k floats per lane per register chunk
  constexpr int NCH = KQ / KC;              // chunks (1 for hs <= 128: q stays in registers)
  static_assert(HS % 16 == 0 && KQ % KC == 0, "head size");
  // S [kQB][T] with the 16-B column block XOR-swizzled by (row & 15) inside its aligned group of
  // 16 blocks (T % 64 == 0): conflict-free phase-1 stores and phase-3 reads at pitch T, and
  // 64 x 320 x 4 B = 80 KB, so two workgroups share a CU's 160 KB
  extern __shared__ float S[];
  const int ldS = T;
  auto sidx = [&](int row, int col) { return row * ldS + ((((col >> 2) ^ (row & 15))) << 2) + (col & 3); };
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  int bid = blockIdx.x;
  const int qb = bid % nqb;
  bid /= nqb;
  const int h = bid % heads;
  const int b = bid / heads;
  const int64_t ld = 3 * (int64_t)C;
  const float* base = qkv + (int64_t)b * T * ld + (int64_t)h * HS;
  const int q0 = qb * kQB;

  // ---- phase 1: scores
  {
    const float* qp = base + (int64_t)(q0 + r) * ld + g * KQ;  // + 16 mt ld
    at_f4 qf[4][KC / 4];
    auto load_q = [&](int ch) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < KC / 4; ++j)
          qf[mt][j] = *reinterpret_cast<const at_f4*>(qp + (int64_t)mt * 16 * ld + ch * KC + 4 * j);
    };
    if constexpr (NCH == 1) load_q(0);
    const int ntiles = T / 16;
    at_f4 kf[KC / 4], kn[KC / 4];
    auto load_k = [&](at_f4* dst, int n, int ch) {
      const float* kp = base + C + (int64_t)(n * 16 + r) * ld + g * KQ + ch * KC;
#pragma unroll
      for (int j = 0; j < KC / 4; ++j) dst[j] = *reinterpret_cast<const at_f4*>(kp + 4 * j);
    };
    if (wave < ntiles) load_k(kf, wave, 0);
    for (int n = wave; n < ntiles; n += 4) {
      at_f4 acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = (at_f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int ch = 0; ch < NCH; ++ch) {
        if constexpr (NCH > 1) load_q(ch);
        // prefetch the next (tile, chunk) fragment under this one's MFMAs; issued unconditionally
        // (clamped to the last tile) so the waitcnt for kf below never has to drain it
        const int nn = ch + 1 < NCH ? n : min(n + 4, ntiles - 1);
        const int nc = ch + 1 < NCH ? ch + 1 : 0;
        load_k(kn, nn, nc);
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch above the MFMAs it hides under
#pragma unroll
        for (int j = 0; j < KC / 4; ++j)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[mt][j].x, kf[j].x, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[mt][j].y, kf[j].y, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[mt][j].z, kf[j].z, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[mt][j].w, kf[j].w, acc[mt], 0, 0, 0);
          }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < KC / 4; ++j) kf[j] = kn[j];
      }
      // D: row 4 g + i of query tile mt, column r of key tile n
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) S[sidx(mt * 16 + 4 * g + i, n * 16 + r)] = acc[mt][i];
    }
  }
  __syncthreads();

  // ---- phase 2: row softmax of scale * s. Four threads per row, each holding a quarter of it in
  // registers (16-B LDS reads / writes), the row max / sum combined over the 4 lanes by 2 xor steps:
  // no dependent wave-wide reduction chains (what a row-per-wave softmax is bound by here).
  {
    constexpr int QMAX = 512 / 16;  // float4 per thread at T <= 512
    const int row = threadIdx.x >> 2, seg = threadIdx.x & 3;
    const int nq = T / 16;          // float4 per thread
    float* sr = S + row * ldS;
    const int blk0 = seg * (T / 16);  // first 16-B block of this thread's quarter
    at_f4 v[QMAX];
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < QMAX; ++i)
      if (i < nq) {
        v[i] = *reinterpret_cast<const at_f4*>(sr + (((blk0 + i) ^ (row & 15)) << 2)) * scale;
        m = fmaxf(m, fmaxf(fmaxf(v[i].x, v[i].y), fmaxf(v[i].z, v[i].w)));
      }
    m = fmaxf(m, __shfl_xor(m, 1));
    m = fmaxf(m, __shfl_xor(m, 2));
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < QMAX; ++i)
      if (i < nq) {
        v[i].x = expf(v[i].x - m);
        v[i].y = expf(v[i].y - m);
        v[i].z = expf(v[i].z - m);
        v[i].w = expf(v[i].w - m);
        sum += (v[i].x + v[i].y) + (v[i].z + v[i].w);
      }
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    const float inv = 1.f / sum;
#pragma unroll
    for (int i = 0; i < QMAX; ++i)
      if (i < nq) *reinterpret_cast<at_f4*>(sr + (((blk0 + i) ^ (row & 15)) << 2)) = v[i] * inv;
  }
  __syncthreads();

  // ---- phase 3: y = P V. Work unit = (column tile ct, group of MG query tiles); 4 units per wave
  // round when hs >= 64, otherwise the 4 query tiles are split so every wave has a unit.
  constexpr int NN = HS / 16;
  constexpr int MG = NN >= 4 ? 4 : NN;  // query tiles per unit
  constexpr int NU = NN * (4 / MG);     // units
  const int KT = T / 4;                 // keys per lane group
  for (int u = wave; u < NU; u += 4) {
    const int ct = u % NN, m0 = (u / NN) * MG;
    const float* pr = S + (m0 * 16 + r) * ldS;  // row & 15 == r for every query tile
    const int pb = g * (KT / 4);                 // first 16-B block of this lane group's keys
    const float* vp = base + 2 * C + (int64_t)(g * KT) * ld + ct * 16 + r;
    at_f4 acc[MG];
#pragma unroll
    for (int mt = 0; mt < MG; ++mt) acc[mt] = (at_f4){0.f, 0.f, 0.f, 0.f};
    float vc[8], vn[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vc[j] = vp[(int64_t)j * ld];
    for (int j0 = 0; j0 < KT; j0 += 8) {
      const int jn = min(j0 + 8, KT - 8);  // unconditional prefetch (see phase 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) vn[j] = vp[(int64_t)(jn + j) * ld];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 0; jj < 8; jj += 4) {
#pragma unroll
        for (int mt = 0; mt < MG; ++mt) {
          const at_f4 p = *reinterpret_cast<const at_f4*>(pr + mt * 16 * ldS + (((pb + (j0 + jj) / 4) ^ r) << 2));
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.x, vc[jj + 0], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.y, vc[jj + 1], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.z, vc[jj + 2], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.w, vc[jj + 3], acc[mt], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) vc[j] = vn[j];
    }
#pragma unroll
    for (int mt = 0; mt < MG; ++mt) {
      float* yp = y + ((int64_t)b * T + q0 + (m0 + mt) * 16 + 4 * g) * C + h * HS + ct * 16 + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) yp[(int64_t)i * C] = acc[mt][i];
    }
  }
}

}  // namespace

void launch_gpt_attention(const float* qkv, int B, int T, int C, int heads, float* y, hipStream_t st) {
  if (heads <= 0 || C % heads) throw std::runtime_error("gpt_attention: C % heads != 0");
  const int hs = C / heads;
  // phase 3 splits the keys into 4 contiguous lane-group slices read as 16-B LDS vectors
  if (T % 64 || (T / 4) % 8 || T > 512 || (T / 4) % 4)
    throw std::runtime_error("gpt_attention: T must be a multiple of 64 with T/4 % 8 == 0, and <= 512");
  if ((reinterpret_cast<uintptr_t>(qkv) & 15) || (C % 4))
    throw std::runtime_error("gpt_attention: qkv must be 16-byte aligned with C % 4 == 0");
  const int nqb = T / kQB;
  const size_t lds = (size_t)kQB * T * sizeof(float);
  const float scale = (float)(1.0 / std::sqrt((double)hs));  // math.sqrt in the reference
  const dim3 grid((unsigned)((int64_t)B * heads * nqb)), block(256);
  switch (hs) {
#define AT(HS)                                                                                          \
  case HS:                                                                                              \
    hipLaunchKernelGGL((gpt_attn_kernel<HS>), grid, block, lds, st, qkv, y, T, C, heads, nqb, scale); \
    break;
    AT(16) AT(32) AT(64) AT(128) AT(256) AT(512)
#undef AT
    default:
      throw std::runtime_error("gpt_attention: head size " + std::to_string(hs) + " not in {16..512}");
  }
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
