// The decoder's cross-BEV attention contraction - value_proj, a 3x3 conv 256 -> 256 + ReLU over the 64 x 64
// cross-BEV map (modules/blocks.py:68-76,114) - evaluated only at the map pixels the grid-sample taps read
// (blocks.py:101-122): the scenes' distinct tap pixels, counted and listed by the decoder megakernel's dedup,
// compacted into full 256-row tiles, K split over up to three workgroups so the launch is one wave of the chip.
//
// Why this shape: a (step, layer) has ~21 K live rows at B = 64 (M 21 K, N 256, K 2304). conv_x3's 128 x 128 tiles
// (332 of them: 1.3 waves) stream 32 KB of operands per 32-deep K chunk for 3 MFLOP - about the ~30 B/clk a CU
// takes in from L2 at the MFMA rate (PMC MFMA busy 0.27). A 256 x 256 tile halves the bytes per FLOP (A 32 KB + B
// 32 KB per chunk for 4x the work: ~15 B/clk) but there are only ~83 of them; split three ways over K they are
// ~249 workgroups - one wave. (An earlier 128 x 256 form with the same split ran 498 workgroups, 1.95 waves, and
// was 20 % slower than conv_x3: profiles/round3_f_vproj_splitk_ab.txt.)
//
// Splits: S = the largest of 3, 2, 1 with (live tiles) x S <= the CU budget (256, or 192 while the tf-decoder
// megakernel holds 64 CUs beside the first launch), decided in the kernel from the live-row count (known only on the
// device); split s of S takes K chunks [72 s / S, 72 (s + 1) / S) of the 72 (9 taps x 8 channel chunks of 32).
//
// Per workgroup: 8 waves (4 x 2, wave tile 64 x 128), A = the tile's gathered rows by LDS-DMA (per-lane 16-B
// buffer loads at each row's own pixel offset; out-of-map taps read zero through the out-of-range offset), B = the
// pre-split fp16 hi / lo weight images, 2 LDS stages (one chunk in flight under the current one's MFMAs: a chunk
// is ~2 us of MFMAs), f16x3 products (conv_x3.hip's arithmetic), A split at fragment-read time.
// Epilogue from the accumulators (no LDS park): C layout of 32x32 MFMA - lanes 0-31 of a register hold 32
// consecutive channels of one row, so every store / load below is a 128-B row segment per half-wave.
//  * S = 1: bias, ReLU, the value row out.
//  * S > 1: every split stores its scaled partial write-through (sc1), drains, and adds to the tile's counter
//    (agent scope); the workgroup whose add returns S - 1 - the last - loads the others' partials (sc1), sums
//    p0 + p1 [+ p2] in that fixed order (its own from registers: deterministic whichever split arrives last), adds
//    the bias, applies ReLU, writes the value rows where the megakernel's slots point (row b * cap + l of scene b's
//    l-th pixel) and zeroes the counter for the next launch (MI355X_MICROARCH.md, inter-workgroup visibility:
//    sc1 stores, one agent add per storing workgroup, the last adder told by the returned value, sc1 loads).
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
// Tile width: TN = 4 -> 256 output channels (every one; the K split fills the chip), TN = 2 -> 128 (the two N halves
// of a row tile are two workgroups on one XCD, no K split and no partials)
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

// splits for a launch with `tiles` live 256-row tiles: the most (<= 3) that keep the grid within one wave of the
// `budget` CUs this launch has (the whole chip, or what a concurrent kernel leaves: one workgroup per CU here)
__device__ inline int vp_splits(int tiles, int cap, int budget) {
  const int s = tiles * 3 <= budget ? 3 : (tiles * 2 <= budget ? 2 : 1);
  return s < cap ? s : cap;
}

}  // namespace

template <int VP_TN>
__global__ __launch_bounds__(VP_NT) void vproj_kernel(VprojArgs a) {
  constexpr int VP_BN = VpTile<VP_TN>::BN, VP_BB = VpTile<VP_TN>::BB, VP_STAGE = VpTile<VP_TN>::STAGE;
  constexpr int VP_B_IN = VpTile<VP_TN>::B_IN;
  constexpr int NH = kC / VP_BN;  // N parts of a row tile
  constexpr int NST = VpTile<VP_TN>::NSTAGE;
  __shared__ __attribute__((aligned(1024))) char lds[NST * VP_STAGE];
  __shared__ int g_rows[VP_BM];
  __shared__ int g_pre[257];
  __shared__ int g_last;
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // ---- compacted rows: launch row m = the m-th live row over the scenes in order
  rowcount_prefix(a.counts, a.B, g_pre);
  const int total = g_pre[a.B];
  const int tiles = (total + VP_BM - 1) / VP_BM;
  const int S = NH > 1 ? 1 : vp_splits(tiles, a.max_splits, a.max_wgs);
  int bid = blockIdx.x;
  int nh = 0;
  if constexpr (NH > 1) {
    // the NH halves of row tile m take blocks with equal blockIdx % 8 (one XCD under round-robin placement: the
    // second half finds the gathered A rows in that XCD's L2; speed only)
    const int g = bid / (8 * NH), r = bid % (8 * NH);
    nh = r / 8;
    bid = g * 8 + r % 8;
  }
  if (bid >= tiles * S) return;  // workgroup-uniform; touches no counter
  const int mt = bid / S, sp = bid - mt * S;
  const int m0 = mt * VP_BM;
  const int n0 = nh * VP_BN;
  const int kbeg = sp * VP_NK / S, kend = (sp + 1) * VP_NK / S;
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
        acc[i][j][r] *= sc[j];  // the scaled partial
      }
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
  auto row_of = [&](int i, int r) { return (wm * VP_TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh; };
  auto finish = [&](int i, int j, int r, float v) {
    const int ri = g_rows[row_of(i, r)];
    if (ri >= 0) a.out[(int64_t)ri * kC + n0 + (wn * VP_TN + j) * 32 + li] = fmaxf(v + bias[j], 0.f);
  };
  if (NH > 1 || S == 1) {
#pragma unroll
    for (int i = 0; i < VP_TM; ++i)
#pragma unroll
      for (int j = 0; j < VP_TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) finish(i, j, r, acc[i][j][r]);
    return;
  }
  if constexpr (NH > 1) return;
  // ---- this split's partial out, write-through; every storing wave drains before the counter add
  const int64_t MR = (int64_t)a.B * a.cap;
  const __amdgpu_buffer_rsrc_t rpart = __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, (int)kOOBv, 0x00020000);
  auto part_off = [&](int s, int i, int j, int r) {
    return (int)((((int64_t)s * MR + m0 + row_of(i, r)) * VP_BN + (wn * VP_TN + j) * 32 + li) * 4);
  };
#pragma unroll
  for (int i = 0; i < VP_TM; ++i)
#pragma unroll
    for (int j = 0; j < VP_TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (m0 + row_of(i, r) < total) {
          const float v = acc[i][j][r];  // (a bit_cast of the vector-element lvalue itself reads element 0)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rpart, part_off(sp, i, j, r), 0, kSC1);
        }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    // the sc1 / drained / one-adder / sc1-load form above is the measured hand-off of MI355X_MICROARCH.md's table
    // (row 1); the agent-scope release before the add and the acquire after it make the ordering the memory
    // model's, not the cache-policy bits' (one each per workgroup; the compiler-hazard wait after the release)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(a.tile_cnt + mt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g_last = old == (unsigned)(S - 1);
    if (old == (unsigned)(S - 1)) {
      __hip_atomic_store(a.tile_cnt + mt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!g_last) return;
  // ---- the last split: p0 + p1 [+ p2] in split order (its own from registers, the others by sc1 loads)
#pragma unroll
  for (int i = 0; i < VP_TM; ++i)
#pragma unroll
    for (int j = 0; j < VP_TN; ++j) {
      float p[3][16];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        if (s >= S) break;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          p[s][r] = (s == sp || m0 + row_of(i, r) >= total)
                        ? acc[i][j][r]
                        : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rpart, part_off(s, i, j, r), 0, kSC1));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = p[0][r] + p[1][r];
        if (S == 3) v = v + p[2][r];
        finish(i, j, r, v);
      }
    }
}

bool vproj_supported(int C, int Cout, int H, int W) { return C == kC && Cout == kC && H == kHW && W == kHW; }

size_t vproj_tiles(int B, int cap) { return ((size_t)B * cap + VP_BM - 1) / VP_BM; }

void launch_vproj(const VprojArgs& a, hipStream_t st) {
  if (!a.map || !a.wh || !a.wl || !a.wsinv || !a.bias || !a.rows || !a.counts || !a.part || !a.tile_cnt || !a.out)
    throw std::runtime_error("vproj: missing operand");
  if (a.B < 1 || a.B > 256 || a.cap < 1 || a.ldh < 9 * kC || a.ldh % 8 || a.max_splits < 1 || a.max_splits > 3 ||
      a.max_wgs < 1)
    throw std::runtime_error("vproj: B in [1, 256], ldh >= 2304 and a multiple of 8, max_splits in [1, 3]");
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al16(a.map) || !al16(a.wh) || !al16(a.wl) || !al16(a.wsinv) || !al16(a.bias) || !al16(a.part) || !al16(a.out))
    throw std::runtime_error("vproj: operands must be 16-byte aligned");
  // buffer offsets are 32-bit byte offsets below 2^31
  if ((int64_t)a.B * kHW * kHW * kC * 4 >= (int64_t)kOOBv || (int64_t)3 * a.B * a.cap * kC * 4 >= (int64_t)kOOBv ||
      (int64_t)kC * a.ldh * 2 >= (int64_t)kOOBv)
    throw std::runtime_error("vproj: operand extent >= 2 GiB");
  if (a.nsplit == 2) {
    // two 128-channel halves per row tile, no K split: grid in groups of 8 tiles x 2 halves
    const size_t t8 = (vproj_tiles(a.B, a.cap) + 7) / 8 * 8;
    hipLaunchKernelGGL(vproj_kernel<2>, dim3((unsigned)(t8 * 2)), dim3(VP_NT), 0, st, a);
  } else {
    // every (tile, split) the kernel may pick: up to 3 splits of every possible tile
    const dim3 grid((unsigned)(vproj_tiles(a.B, a.cap) * 3));
    hipLaunchKernelGGL(vproj_kernel<4>, grid, dim3(VP_NT), 0, st, a);
  }
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
