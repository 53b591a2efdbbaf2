// The decoder's cross-BEV attention contraction - value_proj, a 3x3 conv 256 -> 256 + ReLU over the 64 x 64
// cross-BEV map (modules/blocks.py:68-76,114) - evaluated only at the map pixels the grid-sample taps read
// (blocks.py:101-122): the scenes' distinct tap pixels, counted and listed by the decoder megakernel's dedup,
// compacted into full 256-row tiles.
//
// Two kernels. The union-staged form (vproj_union_kernel, below: the default) stages each tile's union of 3 x 3
// neighbourhoods in LDS once per channel group. The gathered form here (vproj_kernel<2>) computes the tiles whose
// union does not fit (fb_only, right after the union launch) and every tile under DDMI_VPROJ_UNION=0.
//
// Gathered form, per workgroup: 8 waves (4 x 2, wave tile 64 x 64), a row tile's 128-channel half (the two halves
// are two workgroups on one XCD); A = the tile's gathered rows by LDS-DMA (per-lane 16-B buffer loads at each row's
// own pixel offset; out-of-map taps read zero through the out-of-range offset), B = the pre-split fp16 hi / lo
// weight images, 2-3 LDS stages (chunks in flight under the current one's MFMAs), f16x3 products (conv_x3.hip's
// arithmetic), A split at fragment-read time. Epilogue from the accumulators (no LDS park): C layout of 32x32
// MFMA - lanes 0-31 of a register hold 32 consecutive channels of one row, so every store below is a 128-B row
// segment per half-wave: bias, ReLU, the value row out where the megakernel's slots point (row b * cap + l of scene
// b's l-th pixel). (A 256-channel form with the K split over three workgroups and a partial combine measured slower
// than the halves - profiles/round3_f_vproj_splitk_ab.txt, round4 - and was removed in round 6, git history.)
#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 vp_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 vp_h2 __attribute__((ext_vector_type(2)));
typedef float vp_f2 __attribute__((ext_vector_type(2)));
typedef float vp_f16 __attribute__((ext_vector_type(16)));
typedef int vp_i4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kOOBv = 0x80000000u;
constexpr int kC = 256, kHW = 64;          // channels in / out, BEV map side
constexpr int VP_WM = 4, VP_WN = 2, VP_TM = 2;
constexpr int VP_NW = VP_WM * VP_WN, VP_NT = 64 * VP_NW;
constexpr int VP_BM = VP_WM * VP_TM * 32;  // 256 rows
constexpr int VP_KC = 32;                  // K chunk
constexpr int VP_NK = 9 * kC / VP_KC;      // 72 chunks
constexpr int VP_AB = VP_BM * VP_KC * 4;   // A stage bytes: fp32 rows of 128 B
constexpr int VP_A_IN = VP_BM / 8 / VP_NW;   // A DMA instructions per wave per chunk
static_assert(VP_A_IN >= 1, "DMA split over the waves");
static_assert(VP_BM == 256, "the compacted row table holds 256 rows");
// Tile width: TN = 2 -> 128 output channels (the two N halves of a row tile are two workgroups on one XCD)
template <int TN>
struct VpTile {
  static constexpr int BN = VP_WN * TN * 32;
  static constexpr int BB = BN * VP_KC * 2;  // one B image: fp16 rows of 64 B
  static constexpr int STAGE = VP_AB + 2 * BB;
  static constexpr int B_IN = BN / 16 / VP_NW;  // B DMA instructions per wave per chunk and image
  // LDS stages of the A / B ring: two chunks in flight under the current one's MFMAs where three fit
  static constexpr int NSTAGE = 3 * STAGE <= 160 * 1024 - 4096 ? 3 : 2;
  static_assert(2 * STAGE <= 160 * 1024 - 4096, "stages");
  static_assert(B_IN >= 1, "DMA split over the waves");
};

template <int N>
__device__ inline void vp_barrier_n() {  // at most N of this wave's DMAs outstanding, LDS ops retired, barrier
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ inline vp_i4 vp_rsrc(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  vp_i4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r.z = (int)kOOBv;  // num_records: offsets >= 2^31 read as zero
  r.w = 0x00020000;
  return r;
}

// 16 B per lane from global into LDS at m0 + 16 * lane (inline asm: invisible to the compiler's vmcnt pass)
__device__ inline void vp_dma(vp_i4 rsrc, uint32_t lds_wave, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds_wave), "v"(voff), "s"(rsrc)
               : "memory");
}

// every DMA of this wave has landed, LDS ops retired, then the workgroup barrier
__device__ inline void vp_barrier0() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ inline void vp_split8(const float4& p, const float4& q, vp_h8& hi, vp_h8& lo) {
  const float x[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const vp_h2 h = __builtin_convertvector((vp_f2){x[e], x[e + 1]}, vp_h2);
    const vp_f2 f = __builtin_convertvector(h, vp_f2);
    const vp_h2 l = __builtin_convertvector((vp_f2){x[e] - f.x, x[e + 1] - f.y}, vp_h2);
    hi[e] = h.x;
    hi[e + 1] = h.y;
    lo[e] = l.x;
    lo[e + 1] = l.y;
  }
}

// cache-policy bits of the raw buffer intrinsics: sc1 (write-through stores, L1-bypassing loads)
constexpr int kSC1 = 16;

}  // namespace

template <int VP_TN>
__global__ __launch_bounds__(VP_NT) void vproj_kernel(VprojArgs a) {
  constexpr int VP_BN = VpTile<VP_TN>::BN, VP_BB = VpTile<VP_TN>::BB, VP_STAGE = VpTile<VP_TN>::STAGE;
  constexpr int VP_B_IN = VpTile<VP_TN>::B_IN;
  constexpr int NH = kC / VP_BN;  // N parts of a row tile
  static_assert(NH == 2, "the two 128-channel halves of a row tile");
  constexpr int NST = VpTile<VP_TN>::NSTAGE;
  __shared__ __attribute__((aligned(1024))) char lds[NST * VP_STAGE];
  __shared__ int g_rows[VP_BM];
  __shared__ int g_pre[257];
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // after the union-staged kernel: only the (tile, half) pairs it handed over (their flags cleared here)
  if (a.fb_only) {
    const int bq = blockIdx.x / (8 * NH), rq = blockIdx.x % (8 * NH);
    const int f = (bq * 8 + rq % 8) * NH + rq / 8;
    if (__hip_atomic_load(a.fb + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
    __syncthreads();  // every thread read the flag before it is cleared
    if (threadIdx.x == 0) a.fb[f] = 0u;
  }
  // ---- compacted rows: launch row m = the m-th live row over the scenes in order
  rowcount_prefix(a.counts, a.B, g_pre);
  const int total = g_pre[a.B];
  const int tiles = (total + VP_BM - 1) / VP_BM;
  // the NH halves of row tile m take blocks with equal blockIdx % 8 (one XCD under round-robin placement: the
  // second half finds the gathered A rows in that XCD's L2; speed only)
  const int nh = (blockIdx.x % (8 * NH)) / 8;
  const int mt = blockIdx.x / (8 * NH) * 8 + blockIdx.x % 8;
  if (mt >= tiles) return;  // workgroup-uniform
  const int m0 = mt * VP_BM;
  const int n0 = nh * VP_BN;
  constexpr int kbeg = 0, kend = VP_NK;
  for (int r = tid; r < VP_BM; r += VP_NT) {
    const int g = m0 + r;
    int idx = -1;
    if (g < total) {
      int lo = 0, hi = a.B - 1;  // the last scene whose prefix is <= g
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (g_pre[mid] <= g) lo = mid; else hi = mid - 1;
      }
      idx = lo * a.cap + (g - g_pre[lo]);
    }
    g_rows[r] = idx;
  }
  __syncthreads();

  const vp_i4 rin = vp_rsrc(a.map);
  const vp_i4 rwh = vp_rsrc(a.wh);
  const vp_i4 rwl = vp_rsrc(a.wl);

  // ---- A DMA lanes: instruction q of this wave fills rows a_rbase + 8 q .. + 7 (128 B each); per row the
  // element offset of tap (0, 0) at the lane's channel slot and the validity bits of the 9 taps
  const int a_rbase = wave * VP_A_IN * 8;
  int abase[VP_A_IN];
  uint32_t amask[VP_A_IN];
#pragma unroll
  for (int q = 0; q < VP_A_IN; ++q) {
    const int r = a_rbase + q * 8 + (lane >> 3);
    const int akq = (lane & 7) ^ ((r >> 1) & 7);  // logical 16-B slot (4 channels) this lane fetches
    const int ri = g_rows[r];
    const int px = ri >= 0 ? a.rows[ri] : -1;
    const int pp = px >= 0 ? px : 0;
    const int n = pp / (kHW * kHW), y = (pp / kHW) % kHW, x = pp % kHW;
    abase[q] = ((n * kHW + y - 1) * kHW + (x - 1)) * kC + akq * 4;
    uint32_t mk = 0;
    if (px >= 0)
      for (int kh = 0; kh < 3; ++kh)
        for (int kw = 0; kw < 3; ++kw)
          if ((unsigned)(y - 1 + kh) < (unsigned)kHW && (unsigned)(x - 1 + kw) < (unsigned)kHW)
            mk |= 1u << (kh * 3 + kw);
    amask[q] = mk;
  }
  // ---- B DMA lanes: instruction q fills rows b_rbase + 16 q .. + 15 of each image
  const int b_rbase = wave * VP_B_IN * 16;
  uint32_t boff[VP_B_IN];
#pragma unroll
  for (int q = 0; q < VP_B_IN; ++q) {
    const int c = b_rbase + q * 16 + (lane >> 2);
    const int slot = (lane & 3) ^ ((c >> 2) & 3);
    boff[q] = (uint32_t)((n0 + c) * a.ldh + slot * 8) * 2u;
  }
  // chunk ck: tap ck / 8 (kh, kw), channels (ck % 8) * 32 ..
  auto issue = [&](int buf, int ck) {
    const uint32_t st = lds_u32 + buf * VP_STAGE;
    const int tap = ck >> 3, ci0 = (ck & 7) * VP_KC;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = (kh * kHW + kw) * kC + ci0;
#pragma unroll
    for (int q = 0; q < VP_A_IN; ++q) {
      const bool ok = (amask[q] >> tap) & 1u;
      vp_dma(rin, __builtin_amdgcn_readfirstlane(st + (a_rbase + q * 8) * 128),
             ok ? (uint32_t)(abase[q] + toff) * 4u : kOOBv);
    }
    const uint32_t kb = (uint32_t)(tap * kC + ci0) * 2u;
#pragma unroll
    for (int q = 0; q < VP_B_IN; ++q) {
      vp_dma(rwh, __builtin_amdgcn_readfirstlane(st + VP_AB + (b_rbase + q * 16) * 64), boff[q] + kb);
      vp_dma(rwl, __builtin_amdgcn_readfirstlane(st + VP_AB + VP_BB + (b_rbase + q * 16) * 64), boff[q] + kb);
    }
  };

  const int wm = wave / VP_WN, wn = wave % VP_WN;
  const int li = lane & 31, hh = lane >> 5;
  vp_f16 acc[VP_TM][VP_TN];
#pragma unroll
  for (int i = 0; i < VP_TM; ++i)
#pragma unroll
    for (int j = 0; j < VP_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int a_ro[2][VP_TM][2], b_ro[2][VP_TN];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int i = 0; i < VP_TM; ++i) {
      const int r = (wm * VP_TM + i) * 32 + li;
#pragma unroll
      for (int u = 0; u < 2; ++u) a_ro[s2][i][u] = r * 128 + (((4 * s2 + 2 * hh + u) ^ ((r >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < VP_TN; ++j) {
      const int c = (wn * VP_TN + j) * 32 + li;
      b_ro[s2][j] = VP_AB + c * 64 + (((2 * s2 + hh) ^ ((c >> 2) & 3)) << 4);
    }
  }

  // every chunk issues the same DMA count per wave (out-of-range taps read zero through the offset, not skipped)
  constexpr int DPC = VP_A_IN + 2 * VP_B_IN;
  issue(0, kbeg);
  if (NST == 3 && kbeg + 1 < kend) issue(1, kbeg + 1);
  int cur = 0;
  for (int kc = kbeg; kc < kend; ++kc) {
    // this wave's chunk kc has landed (the younger chunk kc + 1 may stay in flight), every wave's has (barrier),
    // and every wave finished reading chunk kc - 1, whose stage is refilled below
    if (NST == 3 && kc + 1 < kend)
      vp_barrier_n<DPC>();
    else
      vp_barrier0();
    const int nxt = kc + NST - 1;
    if (nxt < kend) issue(cur == 0 ? NST - 1 : cur - 1, nxt);
    const char* st = lds + cur * VP_STAGE;
    cur = cur + 1 == NST ? 0 : cur + 1;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      vp_h8 ah[VP_TM], al[VP_TM], bh[VP_TN], bl[VP_TN];
#pragma unroll
      for (int j = 0; j < VP_TN; ++j) {
        bh[j] = *reinterpret_cast<const vp_h8*>(st + b_ro[s2][j]);
        bl[j] = *reinterpret_cast<const vp_h8*>(st + b_ro[s2][j] + VP_BB);
      }
#pragma unroll
      for (int i = 0; i < VP_TM; ++i)
        vp_split8(*reinterpret_cast<const float4*>(st + a_ro[s2][i][0]),
                  *reinterpret_cast<const float4*>(st + a_ro[s2][i][1]), ah[i], al[i]);
#pragma unroll
      for (int i = 0; i < VP_TM; ++i)
#pragma unroll
        for (int j = 0; j < VP_TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < VP_TM; ++i)
#pragma unroll
        for (int j = 0; j < VP_TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < VP_TM; ++i)
#pragma unroll
        for (int j = 0; j < VP_TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue from the accumulators: element (i, j, r) is row (wm TM + i) 32 + (r & 3) + 8 (r >> 2) + 4 hh of the
  // tile, channel (wn TN + j) 32 + li
  bool bad = false;
  float sc[VP_TN], bias[VP_TN];
#pragma unroll
  for (int j = 0; j < VP_TN; ++j) {
    const int col = n0 + (wn * VP_TN + j) * 32 + li;
    sc[j] = a.wsinv[col];
    bias[j] = a.bias[col];
  }
#pragma unroll
  for (int i = 0; i < VP_TM; ++i)
#pragma unroll
    for (int j = 0; j < VP_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        bad |= !__builtin_isfinite(acc[i][j][r]);
        acc[i][j][r] *= sc[j];
      }
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
  auto row_of = [&](int i, int r) { return (wm * VP_TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh; };
  auto finish = [&](int i, int j, int r, float v) {
    const int ri = g_rows[row_of(i, r)];
    if (ri >= 0) a.out[(int64_t)ri * kC + n0 + (wn * VP_TN + j) * 32 + li] = fmaxf(v + bias[j], 0.f);
  };
#pragma unroll
  for (int i = 0; i < VP_TM; ++i)
#pragma unroll
    for (int j = 0; j < VP_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) finish(i, j, r, acc[i][j][r]);
}

// ==================================================================================================================
// Union-staged form (the default of the two-half mode). The 256 rows of a row tile are distinct map pixels of one or
// two scenes, sorted by (scene, pixel); their 3 x 3 neighbourhoods overlap heavily (at B = 64, ~600 distinct pixels
// for the 2304 (row, tap) pairs of a tile). Instead of gathering every (row, tap) pair from L2 per K chunk, the
// workgroup stages the UNION of the neighbourhoods once per 16-channel group - register-staged 16-B loads issued
// one group ahead, split into fp16 hi / lo in registers, written as 64-B pixel rows [hi 16 | lo 16 halfs] into the
// other of two union buffers - and the 9 taps read their A fragments from it through a per-(row, tap) union-slot
// table (a neighbour outside the map reads a zero row). B (pre-split weights, K order (kh, kw, ci)) streams through a
// 4-slot LDS ring by LDS-DMA three steps ahead, every vector-memory op inline asm with an exact vmcnt per step (as
// conv_x6.hip). K walks (channel group g) x (tap t): 16 x 9 steps of k = 16, f16x3 products.
//
// The union: a bitmap over the tile's key range (key = scene * 4096 + pixel; rows sorted, so the neighbours of the
// tile lie in [first - 65, last + 65]), prefix popcounts, union slot = rank of the key (sorted, deterministic).
// A tile whose range or union exceeds the staging capacity raises its fallback flag and returns; the gathered
// kernel above (vproj_kernel<2>, launched right after with fb_only) computes exactly those tiles and clears the flags.
namespace {
constexpr int VU_BM = 256, VU_BN = 128, VU_WM = 4, VU_WN = 2, VU_TM = 2, VU_TN = 2;
constexpr int VU_NW = VU_WM * VU_WN, VU_NT = 64 * VU_NW;
constexpr int VU_UMAX = 704;                           // union rows per buffer; row VU_UMAX is a zero row
constexpr int VU_UBYTES = (VU_UMAX + 1) * 64;          // one union buffer: 45120 B
constexpr int VU_BIMG = VU_BN * 32;                    // one B image of a ring slot: 128 rows x 16 k x 2 B
constexpr int VU_BSLOT = 2 * VU_BIMG;                  // 8 KB
constexpr int VU_D = 3, VU_NSLOT = 5;                  // DMA lead (steps), ring slots (D + 2: see BAR2)
constexpr int VU_BQ = VU_BN / 32;                      // DMA instructions (32 rows of 32 B) per image per step
constexpr int VU_BPS = 2 * VU_BQ / VU_NW;              // per wave per step
constexpr int VU_ALD = ((VU_UMAX + 1) * 4 + VU_NT - 1) / VU_NT;  // union float4 loads per thread per group
constexpr int VU_RBITS = 3 * 4096;                     // key range the bitmap covers (3 scenes)
constexpr int VU_RW = VU_RBITS / 32;
constexpr int VU_TA = 1, VU_TS = 7;                    // taps at which the next group's union is issued / stored
constexpr int VU_NG = kC / 16;                         // channel groups
constexpr int VU_LDS = 2 * VU_UBYTES + VU_NSLOT * VU_BSLOT;
static_assert(VU_BPS >= 1 && (2 * VU_BQ) % VU_NW == 0 && VU_BQ % VU_BPS == 0, "B DMA split over the waves");
static_assert(VU_NSLOT >= VU_D + 1, "ring");
static_assert(VU_LDS <= 136 * 1024, "LDS (the other shared arrays add ~9 KB; 160 KB per workgroup)");

// 16-B slot swizzle of a 64-B union row: 16 consecutive rows at one logical slot hit 16 distinct bank groups
__device__ inline int vu_swz(int u) { return (u >> 2) & 3; }

// was a union load (issued at the open of tap VU_TA) issued after B(step t), i.e. at an open in [t - D, t - 1]?
// The first group's union was loaded in the prologue, before every B DMA.
constexpr bool vu_union_in_window(int t, bool first) {
  for (int j = 1; j <= VU_D; ++j) {
    const int u = t - j;
    if (first && u < 0) return false;
    if (((u % 9) + 9) % 9 == VU_TA) return true;
  }
  return false;
}
static_assert(VU_TA + VU_D < VU_TS, "the union loads leave every open window before their wait");
// union loads issued at the opens [t - D + e, t - 1] (e = 1: the barrier also covers the next step's B)
constexpr bool vu_union_in_window_e(int t, bool first, int e) {
  for (int j = 1; j <= VU_D - e; ++j) {
    const int u = t - j;
    if (first && u < 0) return false;
    if (((u % 9) + 9) % 9 == VU_TA) return true;
  }
  return false;
}
static_assert(VU_NSLOT >= VU_D + 2, "a step without a barrier may refill the slot of step s - 2");

template <int N>
__device__ inline void vu_step_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
template <int N>
__device__ inline void vu_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
typedef float vu_f4 __attribute__((ext_vector_type(4)));
__device__ inline vu_f4 vu_vload(vp_i4 rsrc, uint32_t voff) {
  vu_f4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rsrc) : "memory");
  return v;
}
__device__ inline void vu_split4(const vu_f4 v, uint2& hi, uint2& lo) {
  const vp_h2 h01 = __builtin_convertvector((vp_f2){v.x, v.y}, vp_h2);
  const vp_h2 h23 = __builtin_convertvector((vp_f2){v.z, v.w}, vp_h2);
  const vp_f2 f01 = __builtin_convertvector(h01, vp_f2);
  const vp_f2 f23 = __builtin_convertvector(h23, vp_f2);
  const vp_h2 l01 = __builtin_convertvector((vp_f2){v.x - f01.x, v.y - f01.y}, vp_h2);
  const vp_h2 l23 = __builtin_convertvector((vp_f2){v.z - f23.x, v.w - f23.y}, vp_h2);
  hi = make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
  lo = make_uint2(__builtin_bit_cast(uint32_t, l01), __builtin_bit_cast(uint32_t, l23));
}
}  // namespace

#ifdef DDMI_VU_STAMPS
// diagnostic build only (DDMI_BUILD_VARIANT=vust, tools/micro/vu_stamps.py): per workgroup s_memtime at start / K loop
// entry / K loop exit / end, and wave 0's cycles inside the step barriers and the union-store waits
__device__ unsigned long long g_vu_st[8192 * 6];
extern "C" int dd_vu_stamps_read(unsigned long long* h, int n) {
  void* d = nullptr;  // read, then clear for the next launch
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_vu_st)) != hipSuccess) return -1;
  if (hipMemcpy(h, d, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(d, 0, (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#define VU_STAMP(k) vust[k] = __builtin_amdgcn_s_memtime()
#else
#define VU_STAMP(k)
#endif

// BAR2: the step barrier only at every other step of a group pair's 18-step sequence and at every group's tap 0 (the
// union buffer it reads was stored since the last barrier): the barrier at step s waits for the B of steps s and
// s + 1 when s + 1 has none, and a ring slot refilled at a barrier-less step s (with B(s + D)) held step
// s + D - NSLOT <= s - 2, which every wave finished before the barrier at s - 1 (NSLOT = D + 2)
template <bool BAR2>
__global__ __launch_bounds__(VU_NT, 1) void vproj_union_kernel(VprojArgs a) {
  __shared__ __attribute__((aligned(1024))) char lds[VU_LDS];
  __shared__ int g_rows[VU_BM];   // output row (scene b's l-th pixel: b * cap + l) of each tile row, -1 = none
  __shared__ int g_key[VU_BM];    // its key (scene * 4096 + pixel), -1 = none
  __shared__ unsigned g_bm[VU_RW];
  __shared__ int g_wpre[VU_RW + 1];
  __shared__ int g_upix[VU_UMAX];  // key of each union slot
  __shared__ int g_pre[257];
  __shared__ int g_usize;
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef DDMI_VU_STAMPS
  unsigned long long vust[6] = {0, 0, 0, 0, 0, 0};
  auto vu_flush = [&]() {
    if (tid == 0 && blockIdx.x < 8192)
      for (int k = 0; k < 6; ++k) g_vu_st[blockIdx.x * 6 + k] = vust[k];
  };
#endif
  VU_STAMP(0);

  // ---- tile: the two 128-channel halves of row tile mt take blocks with equal (blockIdx / S) % 8 (one XCD); split sp
  // of S takes channel groups [16 sp / S, 16 (sp + 1) / S)
  const int S = a.usplit, sp = blockIdx.x % S, bq = blockIdx.x / S;
  const int gq = bq / 16, rq = bq % 16;
  const int nh = rq / 8, mt = gq * 8 + rq % 8;
  const int gbeg = sp * (VU_NG / S), gend = gbeg + VU_NG / S;
  rowcount_prefix(a.counts, a.B, g_pre);
  const int total = g_pre[a.B];
  const int tiles = (total + VU_BM - 1) / VU_BM;
  if (mt >= tiles) return;  // workgroup-uniform
  const int m0 = mt * VU_BM, n0 = nh * VU_BN;
  for (int r = tid; r < VU_BM; r += VU_NT) {
    const int g = m0 + r;
    int idx = -1, key = -1;
    if (g < total) {
      int lo = 0, hi = a.B - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (g_pre[mid] <= g) lo = mid; else hi = mid - 1;
      }
      idx = lo * a.cap + (g - g_pre[lo]);
      key = a.rows[idx];
    }
    g_rows[r] = idx;
    g_key[r] = key;
  }
  __syncthreads();
  // ---- the union of the rows' 3 x 3 neighbourhoods: bitmap over [key(first) - 65, key(last) + 65]
  const int nrow = min(VU_BM, total - m0);
  const int kbase = g_key[0] - 65;
  const int range = g_key[nrow - 1] + 66 - kbase;
  if (range > VU_RBITS) {
    if (tid == 0 && sp == 0) a.fb[mt * 2 + nh] = 1u;  // the gathered kernel computes this tile
    return;
  }
  const int nwords = (range + 31) >> 5;
  for (int w = tid; w < nwords; w += VU_NT) g_bm[w] = 0u;
  __syncthreads();
  if (tid < nrow) {
    const int key = g_key[tid], p = key & 4095, y = p >> 6, x = p & 63;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if ((unsigned)yy < (unsigned)kHW && (unsigned)xx < (unsigned)kHW) {
        const int k = key + (t / 3 - 1) * kHW + (t % 3 - 1) - kbase;
        atomicOr(&g_bm[k >> 5], 1u << (k & 31));
      }
    }
  }
  __syncthreads();
  if (tid < 64) {  // exclusive prefix of the words' popcounts (<= 384 words: 6 per lane)
    constexpr int PL = (VU_RW + 63) / 64;
    int c[PL], sum = 0;
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int w = PL * tid + j;
      c[j] = w < nwords ? __builtin_popcount(g_bm[w]) : 0;
      sum += c[j];
    }
    int inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (tid >= o) inc += v;
    }
    int run = inc - sum;
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int w = PL * tid + j;
      if (w <= VU_RW) g_wpre[w] = run;
      run += c[j];
    }
    if (tid == 63) g_usize = run;
  }
  __syncthreads();
  const int U = g_usize;
  if (U > VU_UMAX || U > a.umax) {
    if (tid == 0 && sp == 0) a.fb[mt * 2 + nh] = 1u;
    return;
  }
  for (int w = tid; w < nwords; w += VU_NT) {
    unsigned bits = g_bm[w];
    int slot = g_wpre[w];
    while (bits) {
      const int b = __builtin_ctz(bits);
      bits &= bits - 1;
      g_upix[slot++] = kbase + w * 32 + b;
    }
  }
  // the zero rows (neighbours outside the map) of both union buffers
  if (tid < 32) reinterpret_cast<uint32_t*>(lds + (tid >> 4) * VU_UBYTES + VU_UMAX * 64)[tid & 15] = 0u;
  __syncthreads();

  const vp_i4 rin = vp_rsrc(a.map);
  // ---- union staging: thread element e = tid + NT i -> union slot e >> 2, channels 4 (e & 3) .. of the group.
  // Offsets come from the slot table in LDS at each issue; the LDS write addresses are recomputed at the store.
  vu_f4 hr[VU_ALD];
  auto union_issue = [&](int g) {
    const bool gv = g < gend;
#pragma unroll
    for (int i = 0; i < VU_ALD; ++i) {
      const int e = tid + VU_NT * i, u = e >> 2;
      const bool ok = gv && u < U;
      const int o = ok ? g_upix[u] * kC + 4 * (e & 3) + g * 16 : 0;
      hr[i] = vu_vload(rin, ok ? (uint32_t)o * 4u : kOOBv);
    }
  };
  auto union_tie = [&]() {
#pragma unroll
    for (int i = 0; i < VU_ALD; ++i) asm volatile("" : "+v"(hr[i]));
  };
  auto union_store = [&](int buf) {
    char* base = lds + buf * VU_UBYTES;
#pragma unroll
    for (int i = 0; i < VU_ALD; ++i) {
      const int e = tid + VU_NT * i, u = e >> 2, q = e & 3;
      if (u >= U) continue;
      // hi: logical slot q >> 1, 8-B half q & 1; lo: logical slot + 2 (32 B further, before the swizzle)
      const int w = u * 64 + ((((q >> 1) ^ vu_swz(u)) & 3) << 4) + ((q & 1) << 3);
      uint2 hi, lo;
      vu_split4(hr[i], hi, lo);
      *reinterpret_cast<uint2*>(base + w) = hi;
      *reinterpret_cast<uint2*>(base + (w ^ 32)) = lo;
    }
  };

  // ---- B ring DMA: wave instruction j covers one image, rows rb .. rb+31 of the slot (32 B each, 16-B slot of
  // lane l = l & 1 ^ (row >> 3) & 1)
  uint32_t boff[VU_BPS];
  int brow[VU_BPS];
#pragma unroll
  for (int j = 0; j < VU_BPS; ++j) {
    const int qi = wave * VU_BPS + j;
    const int rb = (qi % VU_BQ) * 32;
    const int c = rb + (lane >> 1);
    const int ls = (lane & 1) ^ ((c >> 3) & 1);
    boff[j] = (uint32_t)((n0 + c) * a.ldh + ls * 8) * 2u;
    brow[j] = rb;
  }
  const bool bimg_lo = (wave * VU_BPS) / VU_BQ == 1;
  const vp_i4 rwb = vp_rsrc(bimg_lo ? (const void*)a.wl : (const void*)a.wh);
  auto b_issue = [&](int slot, int tap, int g) {
    const bool gv = g < gend;
    const uint32_t kb = (uint32_t)(tap * kC + g * 16) * 2u;
#pragma unroll
    for (int j = 0; j < VU_BPS; ++j) {
      const uint32_t dst = lds_u32 + 2 * VU_UBYTES + slot * VU_BSLOT + (bimg_lo ? VU_BIMG : 0) + brow[j] * 32;
      vp_dma(rwb, __builtin_amdgcn_readfirstlane(dst), gv ? boff[j] + kb : kOOBv);
    }
  };

  // ---- fragment addresses. A of (row tile i, tap t): the lane's row's union slot, 16-bit pairs per tap
  const int wm = wave / VU_WN, wn = wave % VU_WN;
  const int li = lane & 31, hh = lane >> 5;
  static_assert(VU_TM == 2, "slot pairs");
  uint32_t uslot[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) uslot[t] = 0u;
#pragma unroll
  for (int i = 0; i < VU_TM; ++i) {
    const int m = (wm * VU_TM + i) * 32 + li;
    const int key = g_key[m];
    const int p = key & 4095, y = p >> 6, x = p & 63;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      int u = VU_UMAX;
      if (key >= 0 && (unsigned)yy < (unsigned)kHW && (unsigned)xx < (unsigned)kHW) {
        const int k = key + (t / 3 - 1) * kHW + (t % 3 - 1) - kbase;
        u = g_wpre[k >> 5] + __builtin_popcount(g_bm[k >> 5] & ((1u << (k & 31)) - 1u));
      }
      uslot[t] |= (uint32_t)u << (16 * i);
    }
  }
  auto a_addr = [&](int i, int t) {  // hi 8 halfs of k 8 hh .. of the group (lo: ^ 32)
    const int u = (int)((uslot[t] >> (16 * i)) & 0xffffu);
    return u * 64 + (((hh ^ vu_swz(u)) & 3) << 4);
  };
  int bad_[VU_TN];
#pragma unroll
  for (int j = 0; j < VU_TN; ++j) {
    const int c = (wn * VU_TN + j) * 32 + li;
    bad_[j] = c * 32 + ((hh ^ ((c >> 3) & 1)) << 4);
  }

  vp_f16 acc[VU_TM][VU_TN];
#pragma unroll
  for (int i = 0; i < VU_TM; ++i)
#pragma unroll
    for (int j = 0; j < VU_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  struct Frag {
    vp_h8 ah[VU_TM], al[VU_TM], bh[VU_TN], bl[VU_TN];
  };
  Frag F0, F1;
  auto load_frag = [&](Frag& F, int slot, int g, auto TAP) {
    constexpr int t = decltype(TAP)::value;
    const char* ubuf = lds + (g & 1) * VU_UBYTES;
    const char* bbuf = lds + 2 * VU_UBYTES + slot * VU_BSLOT;
#pragma unroll
    for (int j = 0; j < VU_TN; ++j) {
      F.bh[j] = *reinterpret_cast<const vp_h8*>(bbuf + bad_[j]);
      F.bl[j] = *reinterpret_cast<const vp_h8*>(bbuf + VU_BIMG + bad_[j]);
    }
#pragma unroll
    for (int i = 0; i < VU_TM; ++i) {
      const int o = a_addr(i, t);
      F.ah[i] = *reinterpret_cast<const vp_h8*>(ubuf + o);
      F.al[i] = *reinterpret_cast<const vp_h8*>(ubuf + (o ^ 32));
    }
  };
  // small terms first, the hi x hi term last: the cross terms (part 0) go ahead of the next step's barrier, the
  // hi x hi term (part 1) after it, under the next step's fragment reads
  auto mfma_part = [&](const Frag& F, auto PART) {
    if constexpr (decltype(PART)::value == 0) {
#pragma unroll
      for (int i = 0; i < VU_TM; ++i)
#pragma unroll
        for (int j = 0; j < VU_TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[i], F.bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < VU_TM; ++i)
#pragma unroll
        for (int j = 0; j < VU_TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bl[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < VU_TM; ++i)
#pragma unroll
        for (int j = 0; j < VU_TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bh[j], acc[i][j], 0, 0, 0);
    }
  };

  // Barrier opening step (g, t): this wave's B(g, t) DMAs have landed (vmcnt = memory ops issued after them: B of
  // the next D - 1 steps, plus the union loads if they were issued in the D opens since), every wave's have, every
  // wave's LDS reads and union stores retired (lgkmcnt(0)). Then B(s + D) into the slot of step s - 1 (all its reads
  // retired), and at t == TA the next group's union loads.
  int slot = 0;
  auto open_step = [&](int g, auto TAP, auto FIRST, auto PAR) {
    constexpr int t = decltype(TAP)::value;
    constexpr bool first = decltype(FIRST)::value;
    constexpr int par = decltype(PAR)::value;  // the group's place in its pair: step parity (t + 9 par) & 1
    constexpr bool bar = !BAR2 || t == 0 || ((t + par) & 1) == 0;
    constexpr bool next_bar = !BAR2 || t == 8 || ((t + 1 + par) & 1) == 0;
    constexpr int e = next_bar ? 0 : 1;
    constexpr int N = (VU_D - 1 - e) * VU_BPS + (vu_union_in_window_e(t, first, e) ? VU_ALD : 0);
    if constexpr (bar) {
#ifdef DDMI_VU_STAMPS
      const unsigned long long b0 = __builtin_amdgcn_s_memtime();
      vu_step_barrier<N>();
      vust[4] += __builtin_amdgcn_s_memtime() - b0;
#else
      vu_step_barrier<N>();
#endif
    }
    constexpr int tn = (t + VU_D) % 9;
    int ns = slot + VU_D;
    if (ns >= VU_NSLOT) ns -= VU_NSLOT;
    b_issue(ns, tn, t + VU_D >= 9 ? g + 1 : g);
    if constexpr (t == VU_TA) union_issue(g + 1);
  };

  // ---- prologue: union of the first group -> its buffer, B of its steps 0 .. D-1, open step 0, its fragments
  union_issue(gbeg);
#pragma unroll
  for (int u = 0; u < VU_D; ++u) b_issue(u % VU_NSLOT, u, gbeg);
  vu_wait_vm<VU_D * VU_BPS>();
  union_tie();
  union_store(gbeg & 1);
  open_step(gbeg, std::integral_constant<int, 0>(), std::true_type(), std::integral_constant<int, 0>());
  load_frag(F0, 0, gbeg, std::integral_constant<int, 0>());

  // step s = (g, t), software pipelined: [open step s+1] [its fragment reads into the other set] [MFMAs of step s];
  // at t == TS the next group's union (loaded since the open of tap TA) goes to the other buffer, whose last reads
  // (group g - 1) retired long before
  auto step = [&](int g, auto TAP, auto FIRST, auto PAR, Frag& Fc, Frag& Fn) {
    constexpr int t = decltype(TAP)::value;
    constexpr bool first = decltype(FIRST)::value;
    constexpr int par = decltype(PAR)::value;
    constexpr int t1 = (t + 1) % 9;
    const int g1 = t == 8 ? g + 1 : g;
    if (++slot == VU_NSLOT) slot = 0;
    mfma_part(Fc, std::integral_constant<int, 0>());
    __builtin_amdgcn_sched_barrier(0);
    // (t < 8: g1 = g < gend, known at compile time - a runtime test here would merge two paths before the MFMAs,
    // and the compiler's wait count at the merge would make them wait for the fragment reads issued just above)
    if (t != 8 || g1 < gend) {
      open_step(g1, std::integral_constant<int, t1>(), std::integral_constant<bool, first && t != 8>(),
                std::integral_constant<int, t == 8 ? 1 - par : par>());
      load_frag(Fn, slot, g1, std::integral_constant<int, t1>());
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_part(Fc, std::integral_constant<int, 1>());
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (t == VU_TS) {
      // the union of group g + 1 was issued when step TA opened; younger: B issued at the opens of taps TA+1 .. TS+1
#ifdef DDMI_VU_STAMPS
      const unsigned long long w0 = __builtin_amdgcn_s_memtime();
      vu_wait_vm<(VU_TS + 1 - VU_TA) * VU_BPS>();
      union_tie();
      vust[5] += __builtin_amdgcn_s_memtime() - w0;
#else
      vu_wait_vm<(VU_TS + 1 - VU_TA) * VU_BPS>();
      union_tie();
#endif
      union_store((g + 1) & 1);
    }
  };
  // 9 steps of a group; the fragment sets alternate per step, so a group starting from set A leaves the next
  // group's tap 0 in set Bf (9 is odd): groups run in pairs (A, Bf), (Bf, A)
  auto group = [&](int g, auto FIRST, auto PAR, Frag& A, Frag& Bf) {
    step(g, std::integral_constant<int, 0>(), FIRST, PAR, A, Bf);
    step(g, std::integral_constant<int, 1>(), FIRST, PAR, Bf, A);
    step(g, std::integral_constant<int, 2>(), FIRST, PAR, A, Bf);
    step(g, std::integral_constant<int, 3>(), FIRST, PAR, Bf, A);
    step(g, std::integral_constant<int, 4>(), FIRST, PAR, A, Bf);
    step(g, std::integral_constant<int, 5>(), FIRST, PAR, Bf, A);
    step(g, std::integral_constant<int, 6>(), FIRST, PAR, A, Bf);
    step(g, std::integral_constant<int, 7>(), FIRST, PAR, Bf, A);
    step(g, std::integral_constant<int, 8>(), FIRST, PAR, A, Bf);
  };
  const std::integral_constant<int, 0> P0;
  const std::integral_constant<int, 1> P1;
  VU_STAMP(1);
  group(gbeg, std::true_type(), P0, F0, F1);
  if (gbeg + 1 < gend) group(gbeg + 1, std::false_type(), P1, F1, F0);
  for (int g = gbeg + 2; g < gend; g += 2) {
    group(g, std::false_type(), P0, F0, F1);
    group(g + 1, std::false_type(), P1, F1, F0);
  }
  vu_step_barrier<0>();  // drain the trailing (all-OOB) DMAs and LDS reads
  VU_STAMP(2);

  // ---- epilogue from the accumulators: scale, bias, ReLU, the value rows out. With S splits each stores its scaled
  // partial write-through, adds to the (tile, half) counter, and the last to arrive sums the partials in split order
  // (its own from registers: deterministic whichever arrives last), as vproj_kernel<4>
  bool bad = false;
  float sc[VU_TN], bias[VU_TN];
#pragma unroll
  for (int j = 0; j < VU_TN; ++j) {
    const int col = n0 + (wn * VU_TN + j) * 32 + li;
    sc[j] = a.wsinv[col];
    bias[j] = a.bias[col];
  }
  auto row_of = [&](int i, int r) { return (wm * VU_TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh; };
#pragma unroll
  for (int i = 0; i < VU_TM; ++i)
#pragma unroll
    for (int j = 0; j < VU_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        bad |= g_rows[row_of(i, r)] >= 0 && !__builtin_isfinite(acc[i][j][r]);
        acc[i][j][r] *= sc[j];
      }
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
  auto finish = [&](int i, int j, int r, float v) {
    const int ri = g_rows[row_of(i, r)];
    if (ri >= 0) a.out[(int64_t)ri * kC + n0 + (wn * VU_TN + j) * 32 + li] = fmaxf(v + bias[j], 0.f);
  };
  if (S == 1) {
#pragma unroll
    for (int i = 0; i < VU_TM; ++i)
#pragma unroll
      for (int j = 0; j < VU_TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) finish(i, j, r, acc[i][j][r]);
#ifdef DDMI_VU_STAMPS
    VU_STAMP(3);
    vu_flush();
#endif
    return;
  }
  const int64_t MR = (int64_t)a.B * a.cap;
  const __amdgpu_buffer_rsrc_t rpart = __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, (int)kOOBv, 0x00020000);
  auto part_off = [&](int s_, int i, int j, int r) {
    return (int)((((int64_t)s_ * MR + m0 + row_of(i, r)) * kC + n0 + (wn * VU_TN + j) * 32 + li) * 4);
  };
#pragma unroll
  for (int i = 0; i < VU_TM; ++i)
#pragma unroll
    for (int j = 0; j < VU_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (m0 + row_of(i, r) < total) {
          const float v = acc[i][j][r];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rpart, part_off(sp, i, j, r), 0, kSC1);
        }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned* cnt = a.ucnt + mt * 2 + nh;
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a count at or past S: this launch did not start the counter from zero (the sum would run twice or never)
    if (old >= (unsigned)S && a.flags) atomicOr(a.flags, DD_NUM_SYNC_STATE);
    g_usize = old == (unsigned)(S - 1);
    if (old == (unsigned)(S - 1)) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!g_usize) return;
  // the sum in split order, from the partials (this split's too: its stores are behind the vmcnt wait above), over
  // 16-B quads of the tile's rows: a thread's loads of up to 8 splits x 2 quads go out together (a split past S
  // reads nothing: OOB offset)
  constexpr int QR = VU_BN / 4;  // quads per row
  typedef unsigned vu_u4 __attribute__((ext_vector_type(4)));
  for (int e0 = tid; e0 < VU_BM * QR; e0 += 2 * VU_NT) {
    vu_f4 x[8][2];
    int ri[2], col[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = e0 + k * VU_NT, row = e / QR;
      col[k] = n0 + 4 * (e % QR);
      ri[k] = m0 + row < total ? g_rows[row] : -1;
#pragma unroll
      for (int s_ = 0; s_ < 8; ++s_) {
        const int off = (int)((((int64_t)s_ * MR + m0 + row) * kC + col[k]) * 4);
        x[s_][k] = __builtin_bit_cast(vu_f4, __builtin_amdgcn_raw_buffer_load_b128(rpart, (s_ < S && ri[k] >= 0) ? off : (int)kOOBv, 0, kSC1));
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (ri[k] < 0) continue;
      vu_f4 v = x[0][k];
#pragma unroll
      for (int s_ = 1; s_ < 8; ++s_) v = s_ < S ? v + x[s_][k] : v;
      const vu_f4 bq = *reinterpret_cast<const vu_f4*>(a.bias + col[k]);
      vu_f4 o = v + bq;
      o.x = fmaxf(o.x, 0.f);
      o.y = fmaxf(o.y, 0.f);
      o.z = fmaxf(o.z, 0.f);
      o.w = fmaxf(o.w, 0.f);
      *reinterpret_cast<vu_f4*>(a.out + (int64_t)ri[k] * kC + col[k]) = o;
    }
  }
}

bool vproj_supported(int C, int Cout, int H, int W) { return C == kC && Cout == kC && H == kHW && W == kHW; }

size_t vproj_tiles(int B, int cap) { return ((size_t)B * cap + VP_BM - 1) / VP_BM; }

void launch_vproj(const VprojArgs& a, hipStream_t st) {
  if (!a.map || !a.wh || !a.wl || !a.wsinv || !a.bias || !a.rows || !a.counts || !a.out)
    throw std::runtime_error("vproj: missing operand");
  if (a.B < 1 || a.B > 256 || a.cap < 1 || a.ldh < 9 * kC || a.ldh % 8)
    throw std::runtime_error("vproj: B in [1, 256], ldh >= 2304 and a multiple of 8");
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al16(a.map) || !al16(a.wh) || !al16(a.wl) || !al16(a.wsinv) || !al16(a.bias) || !al16(a.out) ||
      (a.part && !al16(a.part)))
    throw std::runtime_error("vproj: operands must be 16-byte aligned");
  // buffer offsets are 32-bit byte offsets below 2^31: the map, the weight images and the union split's partials
  // (usplit slabs of B * cap rows)
  if ((int64_t)a.B * kHW * kHW * kC * 4 >= (int64_t)kOOBv || (int64_t)kC * a.ldh * 2 >= (int64_t)kOOBv ||
      (a.union_stage && (int64_t)a.usplit * a.B * a.cap * kC * 4 >= (int64_t)kOOBv))
    throw std::runtime_error("vproj: operand extent >= 2 GiB");
  // two 128-channel halves per row tile: grid in groups of 8 tiles x 2 halves
  const size_t t8 = (vproj_tiles(a.B, a.cap) + 7) / 8 * 8;
  if (a.union_stage) {
    if (!a.fb || (a.usplit > 1 && (!a.ucnt || !a.part)) || a.usplit < 1 || (a.usplit & (a.usplit - 1)) ||
        a.usplit > 8)
      throw std::runtime_error("vproj: the union-staged form needs fallback flags, a power-of-two split <= 8 "
                               "and, split, its counters and partials");
    hipLaunchKernelGGL(vproj_union_kernel<true>, dim3((unsigned)(t8 * 2 * a.usplit)), dim3(VU_NT), 0, st, a);
    DD_HIP_CHECK(hipGetLastError());
    VprojArgs f = a;
    f.fb_only = 1;  // tiles whose union did not fit: the gathered form
    hipLaunchKernelGGL(vproj_kernel<2>, dim3((unsigned)(t8 * 2)), dim3(VP_NT), 0, st, f);
  } else {
    hipLaunchKernelGGL(vproj_kernel<2>, dim3((unsigned)(t8 * 2)), dim3(VP_NT), 0, st, a);
  }
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
