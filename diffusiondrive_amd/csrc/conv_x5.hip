// f16x3 / bf16 implicit-GEMM conv / GEMM, LDS-DMA edition (the default kernel for grids that fill the
// chip; conv_x3.hip keeps the register-staged variant for the rest).
//
// Same arithmetic as conv_x3.hip (fp32 operands split into fp16 hi + lo, products ah*bh + ah*bl +
// al*bh on v_mfma_f32_32x32x16_f16, fp32 accumulation; numerics in that file's header), different
// staging. conv_x3's measured bound is its register-staged operand pipeline: global loads into
// VGPRs, the split, and ds_writes through the ~80 B/clk VGPR->LDS store path, serialised with the
// MFMAs. Here both operands go HBM/L2 -> LDS by LDS-DMA (`buffer_load_dwordx4 ... lds`), which
// bypasses VGPRs and the store path:
//  * A (fp32 NHWC activations) lands in LDS unsplit as [BM][32] fp32 rows (128 B) whose 16-B slots
//    are XOR-swizzled by (row >> 1) & 7: the DMA writes lane-linearly, so each lane fetches the
//    global piece that belongs at its LDS position, and a 16-lane ds_read_b128 group (16 rows, one
//    logical slot) hits 16 distinct slots of the 256-B bank row - conflict-free.
//  * The split moves to fragment-read time: each wave converts the 8 fp32 of its A fragment into
//    half8 hi / lo in registers (v_cvt_pk_f16_f32), ~2 VALU per MFMA, hidden under the MFMAs.
//  * B (pre-split fp16 hi / lo weight images [N][ldh]) lands as [BN][32] fp16 rows (64 B) per
//    image, slot swizzle (row >> 2) & 3, read with ds_read_b128 as in conv_x3.
//  * Conv zero padding and ragged M / N / K edges: out-of-range buffer offsets (>= num_records)
//    make the DMA deposit zeros; no per-element branches.
//  * NS LDS stages, chunks issued NS-1 ahead; one barrier per 32-wide K chunk. Every DMA is inline
//    asm, so the compiler's waitcnt pass (which cannot tell an LDS-DMA target from the stage being
//    read and otherwise drains vmcnt(0) before the first ds_read after an issue - the serialisation
//    that held this kernel at conv_x3's speed) never sees them; the kernel waits itself with the exact
//    count: at chunk kc, vmcnt((NS-2) * DMAs per chunk) = this wave's chunk kc has landed, then the
//    barrier (every wave's has, and every wave finished reading the stage chunk kc+NS-1 refills).
//  * 256 x 256 / 256 x 128 / 256 x 64 tiles (8 / 8 / 4 waves): 64 KB of operands per 32-deep K chunk
//    feed 384 MFMAs at 256 x 256 - half the L2 bytes per MFMA of conv_x3's 128 x 128.
//  * XCD-aware bijective tile remap; fused epilogue (per-channel weight scale, alpha, bias,
//    residual, ReLU, strided NHWC store, non-finite flag) as conv_x3.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half2_v __attribute__((ext_vector_type(2)));
typedef float float2_v __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));

constexpr int KC = 32;                 // K chunk (KCT = 16: the deep-ring form, below)
constexpr uint32_t kOOB5 = 0x80000000u;

typedef int x5i4 __attribute__((ext_vector_type(4)));

__device__ inline x5i4 rsrc5a(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  x5i4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xffffu);  // stride 0
  r.z = (int)kOOB5;                             // num_records: offsets >= 2^31 read as zero
  r.w = 0x00020000;
  // wave-uniform by construction; readfirstlane keeps it in SGPRs for the "s" asm operands
  r.x = __builtin_amdgcn_readfirstlane(r.x);
  r.y = __builtin_amdgcn_readfirstlane(r.y);
  return r;
}

// 16 B per lane from global (buffer offset voff) into LDS at m0 + 16 * lane (m0 = wave base),
// invisible to the compiler's vmcnt bookkeeping (see the header)
__device__ inline void dma16(x5i4 rsrc, uint32_t lds_wave, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds_wave), "v"(voff), "s"(rsrc)
               : "memory");
}

template <int N>
__device__ inline void chunk_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt");
#ifdef DDMI_X5_NOBAR  // timing diagnostic only: races by construction
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#else
  // lgkmcnt(0) as well: every fragment read of the stage refilled after this barrier has returned even if the
  // compiler moved the MFMA that consumes it (and with it the wait) below this asm
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
#endif
}

// 8 fp32 -> hi / lo fp16 fragments (RNE twice)
__device__ inline void split8(const float4& p, const float4& q, half8_t& hi, half8_t& lo) {
  const float x[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const half2_v h = __builtin_convertvector((float2_v){x[e], x[e + 1]}, half2_v);
    const float2_v f = __builtin_convertvector(h, float2_v);
    const half2_v l = __builtin_convertvector((float2_v){x[e] - f.x, x[e + 1] - f.y}, half2_v);
    hi[e] = h.x;
    hi[e + 1] = h.y;
    lo[e] = l.x;
    lo[e + 1] = l.y;
  }
}

// 8 fp32 -> bf16 fragment (RNE)
__device__ inline bf16x8_t to_bf16x8(const float4& p, const float4& q) {
  const float x[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
  bf16x8_t r;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const bf16x2_v b = __builtin_convertvector((float2_v){x[e], x[e + 1]}, bf16x2_v);
    r[e] = b.x;
    r[e + 1] = b.y;
  }
  return r;
}

}  // namespace

#ifdef DDMI_X5_STAMPS
// diagnostic build only (DDMI_BUILD_VARIANT=x5st, tools/micro/conv_bench -DX5_STAMPS): per-workgroup
// s_memtime at start / K loop entry / K loop exit / end
__device__ unsigned long long g_x5_st[4096 * 4];
extern "C" int dd_x5_stamps_read(unsigned long long* h, int n) {
  void* d = nullptr;  // read, then clear for the next launch
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_x5_st)) != hipSuccess) return -1;
  if (hipMemcpy(h, d, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(d, 0, (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#define X5_STAMP(k) x5st[k] = __builtin_amdgcn_s_memtime()
#else
#define X5_STAMP(k)
#endif

// PREC 0: f16x3; PREC 1: the bf16 mode (A converted to bf16 at fragment-read time, B = the bf16 weight
// image, one v_mfma_f32_32x32x16_bf16 per MAC; the stage's second B image is not filled).
// KCT: K chunk depth. 32 = two k16 steps per chunk; 16 = the deep-ring form: half the stage bytes, so twice
// the stages fit (256 x 256: 4 stages of 32 KB, three chunks in flight instead of one), one k16 step and one
// barrier per chunk. The MFMA sequence (k16 order, al*bh / ah*bl / ah*bh per step) is the same: bit-identical.
template <int WM, int WN, int TM, int TN, int MODE, int NS, int PREC, int KCT = KC>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 8 && TM * TN == 2) ? 4 : 1) void conv_x5_kernel(ConvArgs a, int M, int K, int n_tiles_m,
                                                               int n_tiles_n) {
  // MODE 1: Cin % KCT == 0 and KH*KW <= 32 (scalar tap walk, per-row tap masks); MODE 0: generic K.
  static_assert(KCT == 16 || KCT == 32, "K chunk");
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int ARB = KCT * 4;        // A row bytes (fp32): 128 / 64
  constexpr int AS = KCT / 4;         // 16-B slots per A row: 8 / 4
  constexpr int ARPI = 64 / AS;       // A rows per DMA instruction: 8 / 16
  constexpr int ASW = 256 / ARB;      // A rows per 256-B bank row: the swizzle key is r / ASW
  constexpr int BRB = KCT * 2;        // B row bytes per image (fp16): 64 / 32
  constexpr int BS = KCT / 8;         // 16-B slots per B row: 4 / 2
  constexpr int BRPI = 64 / BS;       // B rows per DMA instruction: 16 / 32
  constexpr int BSW = 256 / BRB;      // B rows per 256-B bank row
  constexpr int AB = BM * ARB;        // A stage bytes
  constexpr int BB = BN * BRB;        // one B image
  constexpr int STAGE = AB + (PREC ? 1 : 2) * BB;  // bf16: one B image (so one more stage fits)
  constexpr int A_IN = BM / ARPI / NW;   // A DMA instructions per wave per chunk
  constexpr int B_IN = BN / BRPI / NW;   // B DMA instructions per wave per chunk and image
  static_assert(A_IN >= 1 && BM % (ARPI * NW) == 0, "A rows per wave");
  static_assert(B_IN >= 1 && BN % (BRPI * NW) == 0, "B rows per wave");
  static_assert(NS >= 2 && NS * STAGE <= 160 * 1024, "stages");
  constexpr int DPC = A_IN + (PREC ? 1 : 2) * B_IN;  // DMA instructions per wave per chunk
  constexpr int LDS_EPI = epi_quads_lds<WM, WN, TM, TN>();
  __shared__ __attribute__((aligned(1024))) char lds[NS * STAGE > LDS_EPI ? NS * STAGE : LDS_EPI];
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
#ifdef DDMI_X5_STAMPS
  unsigned long long x5st[4];
#endif
  X5_STAMP(0);
  const int nblk = n_tiles_m * n_tiles_n;
  const int bid = blockIdx.x;
  int tile = bid;
  if (nblk >= 16) {
    const int q = nblk / 8, r = nblk % 8, x = bid % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int mt_idx = tile / n_tiles_n;
  const int nt_idx = tile - mt_idx * n_tiles_n;
  const int m0 = mt_idx * BM;
  const int n0 = nt_idx * BN;

  const x5i4 rin = rsrc5a(a.in);
  const x5i4 rwh = rsrc5a(a.wh);
  const x5i4 rwl = rsrc5a(a.wl);
  const int in_sh = (int)a.in_sh, in_sw = (int)a.in_sw;
  const int ldh = (int)a.ldh;
  const int Kp = (K + 7) & ~7;

  // ---- A DMA lanes: instruction q of this wave fills rows a_rbase + q*ARPI ..; lane -> (row, LDS slot)
  const int a_rbase = wave * A_IN * ARPI;
  int abase[A_IN], aih0[A_IN], aiw0[A_IN], akq[A_IN];
  uint32_t amask[A_IN];
#pragma unroll
  for (int q = 0; q < A_IN; ++q) {
    const int r = a_rbase + q * ARPI + lane / AS;
    akq[q] = (lane % AS) ^ ((r / ASW) % AS);  // logical 16-B slot (4 channels) this lane fetches
    const int m = m0 + r;
    const bool v = m < M;
    const int mm = v ? m : 0;
    const int ow = mm % a.Wo;
    const int t2 = mm / a.Wo;
    const int oh = t2 % a.Ho;
    const int n = t2 / a.Ho;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    if constexpr (MODE == 1) {
      abase[q] = n * (int)a.in_sn + ih0 * in_sh + iw0 * in_sw + akq[q] * 4;
      uint32_t mk = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
            mk |= 1u << (kh * a.KW + kw);
      amask[q] = v ? mk : 0u;
    } else {
      abase[q] = n * (int)a.in_sn;
      aih0[q] = v ? ih0 : -(1 << 28);
      aiw0[q] = iw0;
    }
  }
  // ---- B DMA lanes: instruction q fills rows b_rbase + q*BRPI .. of each image
  const int b_rbase = wave * B_IN * BRPI;
  uint32_t boff[B_IN];
  bool bok[B_IN];
  int bkb[B_IN];
#pragma unroll
  for (int q = 0; q < B_IN; ++q) {
    const int c = b_rbase + q * BRPI + lane / BS;
    const int slot = (lane % BS) ^ ((c / BSW) % BS);
    const int n = n0 + c;
    bok[q] = n < a.Cout;
    bkb[q] = slot * 8;
    boff[q] = (uint32_t)(n * ldh + slot * 8) * 2u;
  }

  int t_tap = 0, t_ci = 0, t_kw = 0, t_off = 0;  // MODE 1 scalar tap walk (chunk order)
  auto issue = [&](int buf, int k0) {
    const uint32_t st = lds_u32 + buf * STAGE;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int q = 0; q < A_IN; ++q) {
        const bool ok = t_tap < 32 && ((amask[q] >> (t_tap & 31)) & 1u);
        dma16(rin, __builtin_amdgcn_readfirstlane(st + (a_rbase + q * ARPI) * ARB), ok ? (uint32_t)(abase[q] + t_off) * 4u : kOOB5);
      }
      t_ci += KCT;
      t_off += KCT;
      if (t_ci == a.Cin) {
        t_ci = 0;
        ++t_tap;
        t_off += in_sw - a.Cin;
        if (++t_kw == a.KW) {
          t_kw = 0;
          t_off += in_sh - a.KW * in_sw;
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < A_IN; ++q) {
        const int kk = k0 + akq[q] * 4;
        const int tap = kk / a.Cin;
        const int ci = kk - tap * a.Cin;
        const int kh = tap / a.KW;
        const int kw = tap - kh * a.KW;
        const int ih = aih0[q] + kh, iw = aiw0[q] + kw;
        const bool ok = kk < K && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        dma16(rin, __builtin_amdgcn_readfirstlane(st + (a_rbase + q * ARPI) * ARB),
              ok ? (uint32_t)(abase[q] + ih * in_sh + iw * in_sw + ci) * 4u : kOOB5);
      }
    }
#pragma unroll
    for (int q = 0; q < B_IN; ++q) {
      const uint32_t off = (bok[q] && k0 + bkb[q] < Kp) ? boff[q] + (uint32_t)k0 * 2u : kOOB5;
      dma16(rwh, __builtin_amdgcn_readfirstlane(st + AB + (b_rbase + q * BRPI) * BRB), off);
      if constexpr (PREC == 0) dma16(rwl, __builtin_amdgcn_readfirstlane(st + AB + BB + (b_rbase + q * BRPI) * BRB), off);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, hh = lane >> 5;
  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fragment read offsets per k16 step s2: A fp32 logical slots 4*s2 + 2*hh, +1; B slot 2*s2 + hh
  constexpr int NS2 = KCT / 16;
  int a_ro[NS2][TM][2], b_ro[NS2][TN];
#pragma unroll
  for (int s2 = 0; s2 < NS2; ++s2) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = (wm * TM + i) * 32 + li;
#pragma unroll
      for (int u = 0; u < 2; ++u) a_ro[s2][i][u] = r * ARB + (((4 * s2 + 2 * hh + u) ^ ((r / ASW) % AS)) << 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = (wn * TN + j) * 32 + li;
      b_ro[s2][j] = AB + c * BRB + (((2 * s2 + hh) ^ ((c / BSW) % BS)) << 4);
    }
  }

  const int nk = (K + KCT - 1) / KCT;
  // prologue: chunks 0 .. NS-2 (the MODE 1 tap walk advances in chunk order: issue order = k order)
#pragma unroll
  for (int u = 0; u < NS - 1; ++u) issue(u, u * KCT);
  int cur = 0;  // stage of chunk kc
  X5_STAMP(1);
  for (int kc = 0; kc < nk; ++kc) {
    // this wave's DMAs of chunk kc have landed (NS-2 younger chunks may fly), every wave's have
    // (barrier), and every wave finished reading chunk kc-1, whose stage is refilled below
    chunk_barrier<(NS - 2) * DPC>();
    int nxt = cur + NS - 1;
    if (nxt >= NS) nxt -= NS;
    issue(nxt, (kc + NS - 1) * KCT);
    const char* st = lds + cur * STAGE;
    if (++cur == NS) cur = 0;
    if constexpr (PREC == 1) {
#pragma unroll
      for (int s2 = 0; s2 < NS2; ++s2) {
        bf16x8_t ab[TM], bb[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bb[j] = *reinterpret_cast<const bf16x8_t*>(st + b_ro[s2][j]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
          ab[i] = to_bf16x8(*reinterpret_cast<const float4*>(st + a_ro[s2][i][0]),
                            *reinterpret_cast<const float4*>(st + a_ro[s2][i][1]));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab[i], bb[j], acc[i][j], 0, 0, 0);
      }
      continue;
    }
#pragma unroll
    for (int s2 = 0; s2 < NS2; ++s2) {
      half8_t ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const half8_t*>(st + b_ro[s2][j]);
        bl[j] = *reinterpret_cast<const half8_t*>(st + b_ro[s2][j] + BB);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float4 p = *reinterpret_cast<const float4*>(st + a_ro[s2][i][0]);
        const float4 q = *reinterpret_cast<const float4*>(st + a_ro[s2][i][1]);
        split8(p, q, ah[i], al[i]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    }
  }
  chunk_barrier<0>();  // drain the trailing (all-OOB) DMAs before the block retires
  X5_STAMP(2);

  // ---- epilogue: 16-B quads through LDS when every row is 16-B aligned, else per accumulator element
  bool bad = false;
  if (epi_quads_ok(a)) {
    bad = epi_quads<WM, WN, TM, TN>(a, acc, lds, m0, n0, M, tid);
  } else {
    float scl_v[TN], bias_v[TN];
    int ncol[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      ncol[j] = n0 + (wn * TN + j) * 32 + li;
      const bool nv = ncol[j] < a.Cout;
      bias_v[j] = (a.bias && nv) ? a.bias[ncol[j]] : 0.f;
      scl_v[j] = nv ? a.wsinv[ncol[j]] * a.alpha : 0.f;
    }
    float* out = a.out;
    const float* res = a.res;
    // row offsets once per row (the stage LDS is free: every wave is past its last fragment read)
    const long long* tab = reinterpret_cast<const long long*>(lds);
    epi_row_table<BM, 64 * WM * WN>(a, m0, M, tid, reinterpret_cast<long long*>(lds));
    __syncthreads();
    auto row_at = [&](int i, int q, int e) { return ((wm * TM + i) * 32 + 8 * q + 4 * hh + e) * 2; };
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // this 32-row slab's residuals are all loaded before its first store: out may alias res (in
      // place x += f(x)), so loads interleaved with stores would serialise on memory latency
      float rv[4][4][TN];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r2 = row_at(i, q, e);
          const float* rrow = (res && tab[r2] >= 0) ? res + tab[r2 + 1] : nullptr;
#pragma unroll
          for (int j = 0; j < TN; ++j) rv[q][e][j] = (rrow && ncol[j] < a.Cout) ? rrow[ncol[j]] : 0.f;
        }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long long oo = tab[row_at(i, q, e)];
          if (oo < 0) continue;
          float* orow = out + oo;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (ncol[j] < a.Cout) {
              const float acc_v = acc[i][j][q * 4 + e];
              bad |= !__builtin_isfinite(acc_v);
              float v = acc_v * scl_v[j] + bias_v[j] + rv[q][e][j];
              if (a.relu) v = fmaxf(v, 0.f);
              orow[ncol[j]] = v;
            }
          }
        }
    }
  }
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
#ifdef DDMI_X5_STAMPS
  __syncthreads();
  X5_STAMP(3);
  if (tid == 0 && blockIdx.x < 4096)
    for (int k = 0; k < 4; ++k) g_x5_st[blockIdx.x * 4 + k] = x5st[k];
#endif
}

template <int WM, int WN, int TM, int TN, int NS, int PREC, int KCT>
static void launch_x5_one(const ConvArgs& a, int M, int K, hipStream_t st) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const int ntm = (M + BM - 1) / BM;
  const int ntn = (a.Cout + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, 1);
  static const std::string name = "conv_x5<" + std::to_string(BM) + "," + std::to_string(BN) +
                                  (KCT == 16 ? ",k16" : "") + (PREC ? ",bf16>" : ">");
  set_last_conv_config(name.c_str());
  if (a.Cin % KCT == 0 && a.KH * a.KW <= 32)
    hipLaunchKernelGGL((conv_x5_kernel<WM, WN, TM, TN, 1, NS, PREC, KCT>), grid, dim3(64 * WM * WN), 0, st, a, M, K,
                       ntm, ntn);
  else
    hipLaunchKernelGGL((conv_x5_kernel<WM, WN, TM, TN, 0, NS, PREC, KCT>), grid, dim3(64 * WM * WN), 0, st, a, M, K,
                       ntm, ntn);
  DD_HIP_CHECK(hipGetLastError());
}
// NS: stages of the 32-deep ring. (A 16-deep ring with twice the stages, bit-identical, measured slower on every GPT
// shape: 123.6 -> 130.7 us per 256 x 256 launch; removed in round 6, git history.)
template <int WM, int WN, int TM, int TN, int NS>
static void launch_x5_cfg(const ConvArgs& a, int M, int K, hipStream_t st) {
  if (a.prec == 1)
    launch_x5_one<WM, WN, TM, TN, NS + 1, 1, KC>(a, M, K, st);  // the freed B image buys a stage
  else
    launch_x5_one<WM, WN, TM, TN, NS, 0, KC>(a, M, K, st);
}

// Returns false when the shape is better served by conv_x3 (grids too small to fill the chip).
// Tiles: 256 x 256 with 2 stages (128 KB), 256 x 128 / 256 x 64 with 3 (144 / 96 KB). The Cout > 128
// grids that fill the chip only at 256 x 128, and 128 x 128 tiles for the mid-size GEMMs, measured
// slower than conv_x3 on the GPT shapes (tools/micro/gemm_x3_bench.py) and are not routed here.
bool launch_conv_x5(const ConvArgs& a, int M, int K, hipStream_t st) {
  if (a.prec != 0 && a.prec != 1) return false;
  const int64_t m256 = (M + 255) / 256;
  const int64_t n256 = (a.Cout + 255) / 256, n128 = (a.Cout + 127) / 128;
  // 1x1 stride-1 GEMMs (the GPT M = 20480 token GEMMs): 256 x 256 tiles already pay at half a chip of
  // tiles when Cout is a multiple of 256 from 512 up (MLP-down K = 2048: 172 -> 161 us, qkv C = 256:
  // 52 -> 43 us, MLP-up C = 128: 34 -> 31 us), 256 x 128 for Cout = 256 k + 128 (qkv C = 128: 25 -> 23 us);
  // Cout = 256 GEMMs with 80 tiles stay on conv_x3 (tools/micro/conv_bench; the round-3 tile sweep)
  const bool gemm = a.KH * a.KW == 1 && a.stride == 1;
  // short-K GEMMs with Cout = 512 / 1024 fill more of the chip with 192 x 256 tiles (proj C = 512: 61 -> 57 us,
  // MLP-up C = 256: 72 -> 65 us, C = 128: 30 -> 27 us); K = 2048 and the qkv shapes lose with the 3 x 2 wave
  // fragment layout (MLP-down 160 -> 162 us, qkv C = 512: 116 -> 145 us)
  // 128 x 128 tiles at two workgroups per CU (8 waves of 32 x 64, 84 VGPRs, 66 KB LDS): one workgroup's epilogue
  // and prologue run beside the other's K loop, and the grid is 4x finer than 256 x 256. Taken where it measured
  // faster than the 256-wide tiles (tools/gpu_r6v.sh, profiles/round6/x5_t128_ab.md): the GPT MLP-up / MLP-down
  // GEMMs (C = 256 / 512: -4 to -21 %) and the C = 512 proj, and the stride-2 3x3 convs except where the 256 x 256
  // grid fills the chip in whole rounds (image layer 3 entry: +18 % there), and the 1x1 stride-2 residual downsamples
  // (tools/gpu_r6y.sh); the qkv GEMMs (Cout = 3 K) keep 256 x 256.
  // bf16 (config C4's trunk mode): the short-K 1x1 GEMMs - the ResNet-50 bottleneck expands, HBM-bound on their
  // outputs - on the same two-per-CU tiles (C4 forward -0.35 ms; the compute-heavy GEMMs and the strided downsamples
  // lost there, tools/gpu_r6aa.sh, profiles/round6/x5_t128_ab.md)
  if (M >= 16384 && a.prec == 1 && gemm && K <= 256 && a.Cin % KC == 0 && a.Cout % 128 == 0) {
    launch_x5_cfg<4, 2, 1, 2, 2>(a, M, K, st);
    return true;
  }
  if (M >= 16384 && a.prec == 0 && a.Cin % KC == 0 && a.Cout % 128 == 0) {
    const bool mlp = gemm && ((a.Cout >= 1024 && a.Cout % 1024 == 0 && K <= 512) || (K >= 1024 && a.Cout >= 256) ||
                              (a.Cout == K && K >= 512));
    const bool s2 = a.stride == 2 && a.KH == 3 && a.KW == 3 &&
                    !(a.Cout >= 256 && (m256 * n256) % 256 == 0);
    const bool ds = a.stride == 2 && a.KH == 1 && a.KW == 1;  // the residual downsamples: -6 to -24 %
    if (mlp || s2 || ds) {
      launch_x5_cfg<4, 2, 1, 2, 2>(a, M, K, st);
      return true;
    }
  }
  if (gemm && K <= 512 && (a.Cout == 512 || a.Cout == 1024) && M >= 16384) {
    launch_x5_cfg<2, 4, 3, 2, 2>(a, M, K, st);  // 192 x 256, 8 waves
    return true;
  }
  if (a.Cout <= 64) {
    if (m256 < 256) return false;
    launch_x5_cfg<4, 1, 2, 2, 3>(a, M, K, st);  // 256 x 64, 4 waves
  } else if (a.Cout > 128 && m256 * n256 >= 256) {
    // (4 waves of 128 x 128 at one wave per SIMD, 512 VGPRs: 2.8x slower on the C = 512 qkv / MLP-up shapes, round 6)
    launch_x5_cfg<4, 2, 2, 4, 2>(a, M, K, st);  // 256 x 256, 8 waves
  } else if (a.Cout <= 128 && m256 * n128 >= 256) {
    launch_x5_cfg<4, 2, 2, 2, 3>(a, M, K, st);  // 256 x 128, 8 waves
  } else if (gemm && a.Cout >= 512 && a.Cout % 256 == 0 && m256 * n256 >= 128) {
    launch_x5_cfg<4, 2, 2, 4, 2>(a, M, K, st);
  } else if (gemm && a.Cout % 256 == 128 && m256 * n128 >= 192) {
    launch_x5_cfg<4, 2, 2, 2, 3>(a, M, K, st);
  } else {
    return false;
  }
  return true;
}

}  // namespace ddmi
