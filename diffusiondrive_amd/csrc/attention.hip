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
#include <type_traits>
#include <cstdlib>

#include "common.h"

// f16x3 GPT attention, waves per workgroup (the largest divisor of T / 32 up to): 10 for head sizes <= 64 - one
// workgroup per (scene, head) at T = 320, so each K / V tile is split and staged once, not twice (hs 64:
// 59 -> 42 us, hs 16 / 32: -11 %; tools/micro/attn_bench.py, same box); 5 at hs = 128, whose 10-wave form spills
#define DDMI_ATTN_NW 10
#define DDMI_ATTN_NW128 5
// score operand splits: 2 = f16x3's three products (default), 3 = six products on three-way splits. The two agree
// to fp32 rounding (attention output vs a float64 reference: 4-10e-7 relative for both, tools/micro/attn_bench.py);
// the three-way form spends 2x the score MFMAs, a third K image and 32 more registers (hs 128: 118 -> 81 us,
// hs 64: 40 -> 34 us, same box, profiles/round3_i_attn_ss.txt). prec 2 (the bf16 backbone mode) keeps SS = 3: that
// mode's C4 bar statistic (max over 1280 trajectories of the bf16 forward) sits at the edge of its 0.1 m bar and
// moved 0.081 -> 0.105 m under this fp32-rounding-level change
#define DDMI_ATTN_SS_DEFAULT 2
#include "mk_core.h"

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


// ---------------------------------------------------------------------------------------------------
// f16x3 form (the f16x3 / bf16 modes): NW waves per workgroup, one per 32-query block (T / 32 NW
// workgroups per (scene, head); at T = 320 NW = 10 for hs <= 64, 5 for hs = 128, whose 10-wave form spills),
// flash-style over 32-key
// tiles staged in LDS already split (K two (SS = 3: three) ways as key rows, V two ways transposed to dimension rows;
// double-buffered at hs <= 32, single at 64 / 128 so 2-3 workgroups share a CU), so no wave splits an
// operand element more than once:
//  * S^T = K Q^T on v_mfma_f32_32x32x16_f16 with both operands split two ways (f16x3's 3 products; SS = 3
//    keeps the earlier six-product form on three-way splits for precision studies) - keys on the accumulator
//    rows, queries on the lanes, so each lane owns one query's online-softmax state (with lane ^ 32);
//  * O = P V with P taken straight from the S^T accumulators as the A operand: an MFMA step's k order
//    is free, so it is the C layout's key order (lane half hh, element e <-> key 16 s + 4 hh + (e & 3)
//    + 8 (e >> 2)), and V's B fragment gathers the same keys from the staged rows;
//    P and V split two ways (f16x3, as every other contraction of the path); O's C layout (lane = dimension, rows = queries) makes the final stores 128-B row segments; the
//    per-query rescale / 1/l reach it through a 32-float LDS slot per wave.
struct Split3 {
  mk_h8 h, m, l;
};
__device__ inline Split3 split3(const float a[8]) {
  Split3 s;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s.h[e] = (_Float16)a[e];
    const float r = a[e] - (float)s.h[e];
    s.m[e] = (_Float16)r;
    s.l[e] = (_Float16)(r - (float)s.m[e]);
  }
  return s;
}
__device__ inline void mfma6s(mk_f16& acc, const Split3& a, const Split3& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.h, b.h, acc, 0, 0, 0);
}

typedef _Float16 at_h2 __attribute__((ext_vector_type(2)));
typedef float at_f2 __attribute__((ext_vector_type(2)));
// pairs through v_cvt_pk_f16_f32: hi = f16(x), lo = f16(x - hi) [, lo2 = f16(x - hi - lo)]
__device__ inline void split2x2(float a, float b, at_h2& hi, at_h2& lo) {
  hi = __builtin_convertvector((at_f2){a, b}, at_h2);
  const at_f2 f = __builtin_convertvector(hi, at_f2);
  lo = __builtin_convertvector((at_f2){a - f.x, b - f.y}, at_h2);
}
__device__ inline void split3x2(float a, float b, at_h2& hi, at_h2& mi, at_h2& lo) {
  hi = __builtin_convertvector((at_f2){a, b}, at_h2);
  const at_f2 f = __builtin_convertvector(hi, at_f2);
  const at_f2 r = (at_f2){a - f.x, b - f.y};
  mi = __builtin_convertvector(r, at_h2);
  const at_f2 g = __builtin_convertvector(mi, at_f2);
  lo = __builtin_convertvector((at_f2){r.x - g.x, r.y - g.y}, at_h2);
}

// LDS images per stage of 32 keys (halfs): K split three ways [3][32 keys][HS + 8] (16-B rows 4 banks apart),
// V^T split two ways [2][HS dims][36] (8-B reads of 4 consecutive keys, 18-dword rows -> conflict-free)
template <int HS, int SS>
struct AttnLds {
  static constexpr int KPH = HS + 8;               // K image row pitch (halfs)
  static constexpr int VPH = 36;                   // V^T image row pitch (halfs)
  static constexpr int KIMG = 32 * KPH;            // halfs per K image
  static constexpr int VIMG = HS * VPH;            // halfs per V^T image
  static constexpr int STAGE = SS * KIMG + 2 * VIMG;  // halfs per stage
};

template <int HS, int NW, int SS>
__global__ __launch_bounds__(64 * NW) void gpt_attn_x3_kernel(const float* __restrict__ qkv, float* __restrict__ y, int T,
                                                              int C, int heads, float scale) {
  static_assert(SS == 2 || SS == 3, "score operand splits");
  using LY = AttnLds<HS, SS>;
  constexpr int NB = HS >= 64 ? 1 : 2;  // LDS stages (one for the large heads: 2-3 workgroups per CU)
  constexpr int NKS = HS / 16;           // k16 steps of the score product
  constexpr int NDT = (HS + 31) / 32;    // 32-wide dimension tiles of O
  constexpr int NT = 64 * NW;
  constexpr int NKE = 32 * HS / 4;       // K float4 per tile
  constexpr int NVE = 8 * HS;            // V (4 keys, 1 dim) groups per tile
  constexpr int NPK = (NKE + NT - 1) / NT, NPV = (NVE + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) _Float16 LH[];
  float* AL = reinterpret_cast<float*>(LH + NB * LY::STAGE) + (threadIdx.x >> 6) * 32;  // per-wave 32 floats
  const int G = T / (32 * NW);  // workgroups per (scene, head)
  const int bh = blockIdx.x / G, grp = blockIdx.x - bh * G;
  const int b = bh / heads, h = bh - (bh / heads) * heads;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, hh = lane >> 5;
  const int ld = 3 * C;
  const float* base = qkv + (int64_t)b * T * ld;
  const float* Qg = base + h * HS;
  const float* Kg = base + C + h * HS;
  const float* Vg = base + 2 * C + h * HS;
  const int q0 = (grp * NW + wave) * 32;

  // Q^T B fragments: k = head dimension, n = query q0 + li (SS = 2: only .h / .m are used)
  Split3 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    float q8[8];
    ld8(Qg + (int64_t)(q0 + li) * ld + 16 * ks + 8 * hh, q8);
    if constexpr (SS == 3) {
      qf[ks] = split3(q8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        qf[ks].h[e] = (_Float16)q8[e];
        qf[ks].m[e] = (_Float16)(q8[e] - (float)qf[ks].h[e]);
      }
    }
  }
  // staging: K float4 e -> (row e / (HS/4), quad e % (HS/4)); V group e -> (dim e % HS, keys 4 (e / HS) ..)
  float4 kr[NPK], vr[NPV];
  auto fetch = [&](int t) {
#pragma unroll
    for (int i = 0; i < NPK; ++i) {
      const int e = tid + NT * i;
      if (e < NKE) {
        const int row = e / (HS / 4), c4 = e - row * (HS / 4);
        kr[i] = *reinterpret_cast<const float4*>(Kg + (int64_t)(32 * t + row) * ld + c4 * 4);
      }
    }
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int e = tid + NT * i;
      if (e < NVE) {
        const int d = e % HS, k4 = e / HS;
        const float* p = Vg + (int64_t)(32 * t + 4 * k4) * ld + d;
        vr[i] = make_float4(p[0], p[ld], p[2 * ld], p[3 * ld]);
      }
    }
  };
  auto stage = [&](int buf) {
    _Float16* S0 = LH + buf * LY::STAGE;
#pragma unroll
    for (int i = 0; i < NPK; ++i) {
      const int e = tid + NT * i;
      if (e < NKE) {
        const int row = e / (HS / 4), c4 = e - row * (HS / 4);
        at_h2 hv[2], mv[2], lv[2];
        if constexpr (SS == 3) {
          split3x2(kr[i].x, kr[i].y, hv[0], mv[0], lv[0]);
          split3x2(kr[i].z, kr[i].w, hv[1], mv[1], lv[1]);
        } else {
          split2x2(kr[i].x, kr[i].y, hv[0], mv[0]);
          split2x2(kr[i].z, kr[i].w, hv[1], mv[1]);
        }
        const int o = row * LY::KPH + c4 * 4;
        uint2 u;
        __builtin_memcpy(&u, hv, 8);
        *reinterpret_cast<uint2*>(S0 + o) = u;
        __builtin_memcpy(&u, mv, 8);
        *reinterpret_cast<uint2*>(S0 + LY::KIMG + o) = u;
        if constexpr (SS == 3) {
          __builtin_memcpy(&u, lv, 8);
          *reinterpret_cast<uint2*>(S0 + 2 * LY::KIMG + o) = u;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int e = tid + NT * i;
      if (e < NVE) {
        const int d = e % HS, k4 = e / HS;
        at_h2 hv[2], lv[2];
        split2x2(vr[i].x, vr[i].y, hv[0], lv[0]);
        split2x2(vr[i].z, vr[i].w, hv[1], lv[1]);
        const int o = SS * LY::KIMG + d * LY::VPH + 4 * k4;
        uint2 u;
        __builtin_memcpy(&u, hv, 8);
        *reinterpret_cast<uint2*>(S0 + o) = u;
        __builtin_memcpy(&u, lv, 8);
        *reinterpret_cast<uint2*>(S0 + LY::VIMG + o) = u;
      }
    }
  };

  float m_run = -INFINITY, l_run = 0.f;
  mk_f16 o[NDT];
#pragma unroll
  for (int d = 0; d < NDT; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  const int nt = T / 32;
  fetch(0);
  stage(0);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) fetch(t + 1);
    const _Float16* K0 = LH + (NB == 2 ? (t & 1) : 0) * LY::STAGE;
    const _Float16* V0 = K0 + SS * LY::KIMG;
    // S^T = K Q^T on pre-split images: six products (SS = 3) or f16x3's three (SS = 2)
    mk_f16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int o = li * LY::KPH + 16 * ks + 8 * hh;
      Split3 kf;
      kf.h = *reinterpret_cast<const mk_h8*>(K0 + o);
      kf.m = *reinterpret_cast<const mk_h8*>(K0 + LY::KIMG + o);
      if constexpr (SS == 3) {
        kf.l = *reinterpret_cast<const mk_h8*>(K0 + 2 * LY::KIMG + o);
        mfma6s(s, kf, qf[ks]);
      } else {
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf.m, qf[ks].h, s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf.h, qf[ks].m, s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf.h, qf[ks].h, s, 0, 0, 0);
      }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] *= scale;
      mt = fmaxf(mt, s[r]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = __expf(m_run - m_new);  // 0 on the first tile (v_exp_f32 path: ~2 ulp)
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = __expf(s[r] - m_new);
      ls += s[r];
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
    if (hh == 0) AL[li] = alpha;
    // (one wave's LDS accesses complete in order: the reads below see this wave's writes); skipped when no
    // query's running max moved (alpha == 1 in every lane), the common case after the first tiles
    if (__any(alpha != 1.f))
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 a4 = *reinterpret_cast<const float4*>(AL + 8 * i + 4 * hh);  // queries 8i + 4hh + 0..3
#pragma unroll
      for (int d = 0; d < NDT; ++d) {
        o[d][4 * i] *= a4.x;
        o[d][4 * i + 1] *= a4.y;
        o[d][4 * i + 2] *= a4.z;
        o[d][4 * i + 3] *= a4.w;
      }
    }
    // O += P V: P (A) from the accumulators and V (B), both split two ways: f16x3
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      mk_h8 ph, pl;  // P split two ways (hi, lo)
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        at_h2 a, c;
        split2x2(s[8 * s2 + e], s[8 * s2 + e + 1], a, c);
        ph[e] = a.x;
        ph[e + 1] = a.y;
        pl[e] = c.x;
        pl[e + 1] = c.y;
      }
      const int kb = 16 * s2 + 4 * hh;  // keys kb .. kb+3 and kb+8 .. kb+11
#pragma unroll
      for (int d = 0; d < NDT; ++d) {
        const int dim = 32 * d + li;
        mk_h8 vh, vl;
        if (HS % 32 == 0 || dim < HS) {
          const _Float16* vp = V0 + dim * LY::VPH + kb;
          const uint2 a0 = *reinterpret_cast<const uint2*>(vp), a1 = *reinterpret_cast<const uint2*>(vp + 8);
          const uint2 b0 = *reinterpret_cast<const uint2*>(vp + LY::VIMG), b1 = *reinterpret_cast<const uint2*>(vp + LY::VIMG + 8);
          vh = __builtin_bit_cast(mk_h8, make_uint4(a0.x, a0.y, a1.x, a1.y));
          vl = __builtin_bit_cast(mk_h8, make_uint4(b0.x, b0.y, b1.x, b1.y));
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) vh[e] = vl[e] = (_Float16)0.f;
        }
        o[d] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pl, vh, o[d], 0, 0, 0);
        o[d] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ph, vl, o[d], 0, 0, 0);
        o[d] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ph, vh, o[d], 0, 0, 0);
      }
    }
    if (t + 1 < nt) {
      if constexpr (NB == 1) __syncthreads();  // every wave is done with the stage before it is refilled
      stage(NB == 2 ? (t + 1) & 1 : 0);
    }
    __syncthreads();
  }
  if (hh == 0) AL[li] = 1.f / l_run;
  float* yb = y + ((int64_t)b * T + q0) * C + h * HS;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 inv = *reinterpret_cast<const float4*>(AL + 8 * i + 4 * hh);
    const float iv[4] = {inv.x, inv.y, inv.z, inv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * i + 4 * hh + j;
#pragma unroll
      for (int d = 0; d < NDT; ++d) {
        const int dim = 32 * d + li;
        if (HS % 32 == 0 || dim < HS) yb[(int64_t)row * C + dim] = o[d][4 * i + j] * iv[j];
      }
    }
  }
}

}  // namespace

void launch_gpt_attention(const float* qkv, int B, int T, int C, int heads, float* y, int prec, hipStream_t st) {
  if (heads <= 0 || C % heads) throw std::runtime_error("gpt_attention: C % heads != 0");
  const int hs = C / heads;
  if (prec != 0) {
    // f16x3 form: T % 32 == 0, NW (waves per workgroup) = the largest divisor of T / 32 that is <= DDMI_ATTN_NW
    // (DDMI_ATTN_NW128 at hs = 128; compile-time constants, profiles/round3_i_attn_ss.txt)
    if (T % 32 || T > 1024 || (reinterpret_cast<uintptr_t>(qkv) & 15) || C % 4)
      throw std::runtime_error("gpt_attention(f16x3): T % 32 == 0, T <= 1024, 16-B aligned qkv, C % 4 == 0");
    const int nq = T / 32;
    // the largest instantiated wave count (10, 5, 4, 3, 2, 1) <= the cap that divides T / 32
    int nw = hs >= 128 ? DDMI_ATTN_NW128 : DDMI_ATTN_NW;
    while (nw > 1 && (nq % nw || (nw > 5 && nw != 10))) --nw;
    const float scale = (float)(1.0 / std::sqrt((double)hs));
    const dim3 grid((unsigned)((int64_t)B * heads * (nq / nw))), block((unsigned)(64 * nw));
    // score operand splits: three-way (six products) for prec 2 (the bf16 mode's attention), else
    // DDMI_ATTN_SS_DEFAULT (two-way, f16x3's three products)
    const int ss = prec == 2 ? 3 : DDMI_ATTN_SS_DEFAULT;
    const size_t lds = (size_t)(hs >= 64 ? 1 : 2) * (ss * 32 * (hs + 8) + 2 * hs * 36) * 2 + (size_t)nw * 32 * sizeof(float);
    auto go = [&](auto HSC) {
      constexpr int HS = decltype(HSC)::value;
      auto go2 = [&](auto SSC) {
        constexpr int SS = decltype(SSC)::value;
        switch (nw) {
          case 10: hipLaunchKernelGGL((gpt_attn_x3_kernel<HS, 10, SS>), grid, block, lds, st, qkv, y, T, C, heads, scale); break;
          case 5: hipLaunchKernelGGL((gpt_attn_x3_kernel<HS, 5, SS>), grid, block, lds, st, qkv, y, T, C, heads, scale); break;
          case 4: hipLaunchKernelGGL((gpt_attn_x3_kernel<HS, 4, SS>), grid, block, lds, st, qkv, y, T, C, heads, scale); break;
          case 3: hipLaunchKernelGGL((gpt_attn_x3_kernel<HS, 3, SS>), grid, block, lds, st, qkv, y, T, C, heads, scale); break;
          case 2: hipLaunchKernelGGL((gpt_attn_x3_kernel<HS, 2, SS>), grid, block, lds, st, qkv, y, T, C, heads, scale); break;
          case 1: hipLaunchKernelGGL((gpt_attn_x3_kernel<HS, 1, SS>), grid, block, lds, st, qkv, y, T, C, heads, scale); break;
          default: throw std::runtime_error("gpt_attention(f16x3): no kernel for " + std::to_string(nw) + " waves");
        }
      };
      if (ss == 3) go2(std::integral_constant<int, 3>()); else go2(std::integral_constant<int, 2>());
    };
    switch (hs) {
      case 16: go(std::integral_constant<int, 16>()); break;
      case 32: go(std::integral_constant<int, 32>()); break;
      case 64: go(std::integral_constant<int, 64>()); break;
      case 128: go(std::integral_constant<int, 128>()); break;
      default:
        throw std::runtime_error("gpt_attention(f16x3): head size " + std::to_string(hs) + " not in {16..128}");
    }
    DD_HIP_CHECK(hipGetLastError());
    return;
  }
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
