// The decoder's cross-BEV attention contraction - value_proj, a 3x3 conv 256 -> 256 + ReLU over the 64 x 64
// cross-BEV map (modules/blocks.py:68-76,114) - evaluated only at the map pixels the grid-sample taps read
// (blocks.py:101-122): the scenes' distinct tap pixels, counted and listed by the decoder megakernel's dedup,
// compacted into full 128-row tiles, K split three ways by filter row so the launch fills the chip.
//
// Why split K: a (step, layer) has ~21 K live rows at B = 64. As one implicit GEMM (M 21 K, N 256, K 2304) that is
// 166 tiles of 128 x 256 - 0.65 of a 256-CU wave - or 332 tiles of 128 x 128, whose 48 KB of operand traffic per
// 32-deep K chunk is above what a CU takes in from L2 at MFMA rate (conv_x3's form: 0.27 MFMA busy). Split by the
// filter row kh (K = 3 taps x 256 channels = 768 per split) the 128 x 256 tiles become ~500 workgroups (1.95 waves)
// of 16 B/clk each.
//
// Per workgroup (M tile mt, split kh): 8 waves (2 x 4, wave tile 64 x 64), A = the tile's gathered rows' tap-row
// kh channels by LDS-DMA (per-lane 16-B buffer loads at each row's own pixel offset; out-of-map taps read zero
// through the out-of-range offset), B = the pre-split fp16 hi / lo weight images, 3 LDS stages, one barrier per
// 32-deep chunk with the exact vmcnt (conv_x5.hip's scheme), f16x3 products (conv_x3.hip's arithmetic).
// Combine: every split stores its scaled partial tile write-through (sc1), drains, and adds to the tile's
// counter (agent scope); the workgroup whose add returns 2 - the last of the three - loads the other two partials
// (sc1 loads), sums p0 + p1 + p2 in that fixed order (deterministic whichever split arrives last), adds the bias,
// applies ReLU and writes the value rows where the megakernel's slots point (row b * cap + l of scene b's l-th
// pixel), then zeroes the counter for the next launch (MI355X_MICROARCH.md, inter-workgroup visibility table,
// first row: sc1 stores, one agent add per storing workgroup, the last adder told by the returned value, sc1 loads).
#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 vp_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 vp_h2 __attribute__((ext_vector_type(2)));
typedef float vp_f2 __attribute__((ext_vector_type(2)));
typedef float vp_f4 __attribute__((ext_vector_type(4)));
typedef float vp_f16 __attribute__((ext_vector_type(16)));
typedef int vp_i4 __attribute__((ext_vector_type(4)));
typedef unsigned vp_u4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kOOBv = 0x80000000u;
constexpr int kC = 256, kHW = 64;          // channels in / out, BEV map side
constexpr int VP_WM = 2, VP_WN = 4, VP_TM = 2, VP_TN = 2;
constexpr int VP_NW = VP_WM * VP_WN, VP_NT = 64 * VP_NW;
constexpr int VP_BM = VP_WM * VP_TM * 32;  // 128 rows
constexpr int VP_BN = VP_WN * VP_TN * 32;  // 256 = every output channel
constexpr int VP_KC = 32;                  // K chunk
constexpr int VP_NS = 3;                   // LDS stages
constexpr int VP_AB = VP_BM * VP_KC * 4;   // A stage bytes: fp32 rows of 128 B
constexpr int VP_BB = VP_BN * VP_KC * 2;   // one B image: fp16 rows of 64 B
constexpr int VP_STAGE = VP_AB + 2 * VP_BB;
constexpr int VP_A_IN = VP_BM / 8 / VP_NW;   // A DMA instructions per wave per chunk
constexpr int VP_B_IN = VP_BN / 16 / VP_NW;  // B DMA instructions per wave per chunk and image
constexpr int VP_DPC = VP_A_IN + 2 * VP_B_IN;
constexpr int VP_NK = 3 * kC / VP_KC;        // chunks per split: 3 taps x 256 channels
static_assert(VP_NS * VP_STAGE <= 160 * 1024, "stages");
static_assert(VP_BM * VP_BN * 4 <= VP_NS * VP_STAGE, "parked tile fits the stage LDS");
static_assert(VP_A_IN >= 1 && VP_B_IN >= 1, "DMA split over the waves");

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

template <int N>
__device__ inline void vp_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

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

__global__ __launch_bounds__(VP_NT) void vproj_kernel(VprojArgs a) {
  __shared__ __attribute__((aligned(1024))) char lds[VP_NS * VP_STAGE];
  __shared__ int g_rows[VP_BM];
  __shared__ int g_pre[257];
  __shared__ int g_last;
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int mt = blockIdx.x, kh = blockIdx.y;
  const int m0 = mt * VP_BM;

  // ---- compacted rows: launch row m = the m-th live row over the scenes in order
  rowcount_prefix(a.counts, a.B, g_pre);
  const int total = g_pre[a.B];
  if (m0 >= total) return;  // past every live row (workgroup-uniform; touches no counter)
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
  // element offset of (tap row kh, kw = 0, channel slot) and the validity bits of kw = 0, 1, 2
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
    const int iy = y - 1 + kh;
    abase[q] = ((n * kHW + iy) * kHW + (x - 1)) * kC + akq * 4;
    uint32_t mk = 0;
    if (px >= 0 && (unsigned)iy < (unsigned)kHW)
      for (int kw = 0; kw < 3; ++kw)
        if ((unsigned)(x - 1 + kw) < (unsigned)kHW) mk |= 1u << kw;
    amask[q] = mk;
  }
  // ---- B DMA lanes: instruction q fills rows b_rbase + 16 q .. + 15 of each image
  const int b_rbase = wave * VP_B_IN * 16;
  uint32_t boff[VP_B_IN];
#pragma unroll
  for (int q = 0; q < VP_B_IN; ++q) {
    const int c = b_rbase + q * 16 + (lane >> 2);
    const int slot = (lane & 3) ^ ((c >> 2) & 3);
    boff[q] = (uint32_t)(c * a.ldh + kh * 3 * kC + slot * 8) * 2u;
  }
  // chunk ck (0 .. 23): tap kw = ck / 8, channels (ck % 8) * 32 ..; chunks past the split read zero
  auto issue = [&](int buf, int ck) {
    const uint32_t st = lds_u32 + buf * VP_STAGE;
    const bool cv = ck < VP_NK;
    const int kw = ck >> 3, ci0 = (ck & 7) * VP_KC;
#pragma unroll
    for (int q = 0; q < VP_A_IN; ++q) {
      const bool ok = cv && ((amask[q] >> kw) & 1u);
      vp_dma(rin, __builtin_amdgcn_readfirstlane(st + (a_rbase + q * 8) * 128),
             ok ? (uint32_t)(abase[q] + kw * kC + ci0) * 4u : kOOBv);
    }
    const uint32_t kb = (uint32_t)(kw * kC + ci0) * 2u;
#pragma unroll
    for (int q = 0; q < VP_B_IN; ++q) {
      const uint32_t off = cv ? boff[q] + kb : kOOBv;
      vp_dma(rwh, __builtin_amdgcn_readfirstlane(st + VP_AB + (b_rbase + q * 16) * 64), off);
      vp_dma(rwl, __builtin_amdgcn_readfirstlane(st + VP_AB + VP_BB + (b_rbase + q * 16) * 64), off);
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

#pragma unroll
  for (int u = 0; u < VP_NS - 1; ++u) issue(u, u);
  int cur = 0;
  for (int kc = 0; kc < VP_NK; ++kc) {
    // this wave's chunk kc has landed (NS - 2 younger chunks may fly), every wave's has (barrier), and every
    // wave finished reading chunk kc - 1, whose stage is refilled below
    vp_barrier<(VP_NS - 2) * VP_DPC>();
    int nxt = cur + VP_NS - 1;
    if (nxt >= VP_NS) nxt -= VP_NS;
    issue(nxt, kc + VP_NS - 1);
    const char* st = lds + cur * VP_STAGE;
    if (++cur == VP_NS) cur = 0;
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
  vp_barrier<0>();  // the trailing (all-OOB) DMAs have landed; every wave is past its last fragment read

  // ---- park the scaled partial tile as [128 rows][256] fp32 (16-B slot XOR-swizzled by bit 2 of the row)
  float* ct = reinterpret_cast<float*>(lds);
  bool bad = false;
#pragma unroll
  for (int j = 0; j < VP_TN; ++j) {
    const int col = (wn * VP_TN + j) * 32 + li;
    const float sc = a.wsinv[col];
#pragma unroll
    for (int i = 0; i < VP_TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[i][j][r];
        bad |= !__builtin_isfinite(v);
        const int pr = (wm * VP_TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        ct[pr * VP_BN + ((((col >> 2) ^ (((pr >> 2) & 1) << 3))) << 2) + (col & 3)] = v * sc;
      }
  }
  __syncthreads();
  // ---- this split's partial rows out, write-through; every storing wave drains before the counter add
  constexpr int QN = VP_BN / 4, RPP = VP_NT / QN, IT = VP_BM / RPP;
  const int qn = tid % QN;
  const int64_t MR = (int64_t)a.B * a.cap;
  const __amdgpu_buffer_rsrc_t rpart = __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, (int)kOOBv, 0x00020000);
  auto part_off = [&](int s, int g) { return (uint32_t)((((int64_t)s * MR + g) * VP_BN + 4 * qn) * 4); };
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int pr = tid / QN + k * RPP;
    if (m0 + pr >= total) continue;
    const vp_f4 v = *reinterpret_cast<const vp_f4*>(ct + pr * VP_BN + ((qn ^ (((pr >> 2) & 1) << 3)) << 2));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vp_u4, v), rpart, (int)part_off(kh, m0 + pr), 0, kSC1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.tile_cnt + mt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g_last = old == 2u;
    if (old == 2u) __hip_atomic_store(a.tile_cnt + mt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
  if (!g_last) return;
  // ---- the last split: p0 + p1 + p2 (own partial from LDS, the others by sc1 loads), bias, ReLU
  const vp_f4 bias = *reinterpret_cast<const vp_f4*>(a.bias + 4 * qn);
#pragma unroll 4
  for (int k = 0; k < IT; ++k) {
    const int pr = tid / QN + k * RPP;
    if (m0 + pr >= total) continue;
    vp_f4 p[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      if (s == kh) {
        p[s] = *reinterpret_cast<const vp_f4*>(ct + pr * VP_BN + ((qn ^ (((pr >> 2) & 1) << 3)) << 2));
      } else {
        p[s] = __builtin_bit_cast(vp_f4, __builtin_amdgcn_raw_buffer_load_b128(rpart, (int)part_off(s, m0 + pr), 0, kSC1));
      }
    }
    vp_f4 v = (p[0] + p[1]) + p[2] + bias;
    v.x = fmaxf(v.x, 0.f);
    v.y = fmaxf(v.y, 0.f);
    v.z = fmaxf(v.z, 0.f);
    v.w = fmaxf(v.w, 0.f);
    *reinterpret_cast<vp_f4*>(a.out + (int64_t)g_rows[pr] * VP_BN + 4 * qn) = v;
  }
}

bool vproj_supported(int C, int Cout, int H, int W) { return C == kC && Cout == kC && H == kHW && W == kHW; }

size_t vproj_tiles(int B, int cap) { return ((size_t)B * cap + VP_BM - 1) / VP_BM; }

void launch_vproj(const VprojArgs& a, hipStream_t st) {
  if (!a.map || !a.wh || !a.wl || !a.wsinv || !a.bias || !a.rows || !a.counts || !a.part || !a.tile_cnt || !a.out)
    throw std::runtime_error("vproj: missing operand");
  if (a.B < 1 || a.B > 256 || a.cap < 1 || a.ldh < 9 * kC || a.ldh % 8)
    throw std::runtime_error("vproj: B in [1, 256], ldh >= 2304 and a multiple of 8");
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al16(a.map) || !al16(a.wh) || !al16(a.wl) || !al16(a.wsinv) || !al16(a.bias) || !al16(a.part) || !al16(a.out))
    throw std::runtime_error("vproj: operands must be 16-byte aligned");
  // buffer offsets are 32-bit byte offsets below 2^31
  if ((int64_t)a.B * kHW * kHW * kC * 4 >= (int64_t)kOOBv || (int64_t)3 * a.B * a.cap * VP_BN * 4 >= (int64_t)kOOBv ||
      (int64_t)kC * a.ldh * 2 >= (int64_t)kOOBv)
    throw std::runtime_error("vproj: operand extent >= 2 GiB");
  const dim3 grid((unsigned)vproj_tiles(a.B, a.cap), 3);
  hipLaunchKernelGGL(vproj_kernel, grid, dim3(VP_NT), 0, st, a);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
