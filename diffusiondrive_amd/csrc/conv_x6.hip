// f16x3 direct 3x3 convolution (stride 1, pad 1) with halo reuse - the default kernel for every
// 3x3 stride-1 conv of the path: the ResNet-34 BasicBlocks of both trunks (transfuser_backbone.py
// :23-33, timm BasicBlock conv1/conv2), the FPN up-convs (:124-159) and the decoder's value_proj
// (modules/blocks.py:68-76,114).
//
// Arithmetic: exactly conv_x3.hip's f16x3 (fp32 operand = fp16 hi + lo, products ah*bh + ah*bl +
// al*bh on v_mfma_f32_32x32x16_f16, fp32 accumulation; numerics and range in that file's header;
// non-finite accumulators raise DD_NUM_F16_OVERFLOW), or the bf16 mode's one bf16 product per MAC
// (v_mfma_f32_32x32x16_bf16; PREC 1 below: 64-channel K chunks in the same LDS bytes).
//
// Why a direct kernel: the implicit GEMM (conv_x3 / conv_x5) fetches every input pixel once per
// filter tap, 9x; with f16x3's 4 B per operand element that needs 21-53 B/clk per CU at full MFMA
// rate - above what a CU takes in from L2 (~30 B/clk, MI355X_MICROARCH.md "Indexed rows"). Here a
// workgroup owns a TH x TW output tile (256 pixels of one image) x BN output channels and walks
// K as (32-channel chunk c) x (9 taps):
//  * A: the (TH+2) x (TW+2) input halo of chunk c is fetched ONCE (register-staged 16-B buffer
//    loads, OOB offsets give the zero padding), split into hi / lo fp16 in registers, and written
//    to LDS as 128-B pixel rows [hi 32 | lo 32 halfs]. The 9 taps then read their A fragments from
//    the same halo at a (kh, kw) shift. Halo double buffered: chunk c+1's halo is loaded during
//    chunk c's taps and written into the other buffer at its last tap.
//  * B: pre-split weight images [Cout][ldh] (K order kh, kw, ci) stream through a 3-slot LDS ring,
//    one slot per (chunk, tap) step, by LDS-DMA (`buffer_load_dwordx4 ... lds`), two steps ahead.
//  * Per step: one s_waitcnt vmcnt(N) with the exact count of younger memory ops, one barrier.
//    Every vector-memory op of the main loop is inline asm, so the compiler's waitcnt pass (which
//    cannot tell an LDS-DMA target from the buffer being read and drains vmcnt(0) before every
//    ds_read - what serialised conv_x5) never sees them; the counts are derived in the kernel.
//  * LDS banking: A rows are 128 B; the 16-B slot is XOR-swizzled by (hx >> 1) & 7 of the halo
//    column, so each 16-lane ds_read_b128 group (output pixels x..x+15 of one or two tile rows,
//    shifted by kw) hits 16 distinct (row parity, slot) pairs: conflict-free for every tap. B rows
//    are 64 B per image, slot ^ (n >> 2) & 3 as in conv_x3.
//  * Traffic per step (BN = 128): B 16 KB + A 41.5 KB / 9 = 21 KB per 1536 MFMA cycles = 13.5
//    B/clk per CU (implicit GEMM at 256 x 128: 32 B/clk).
//  * 8 waves (4 x 2), wave tile 64 x (BN / 2); one workgroup per CU (132-136 KB LDS).
//  * Fused epilogue as conv_x3 (per-channel weight scale, alpha, bias, residual, ReLU, strided NHWC).
#include <type_traits>

#include "common.h"


namespace ddmi {

namespace {

typedef _Float16 x6h8 __attribute__((ext_vector_type(8)));
typedef _Float16 x6h2 __attribute__((ext_vector_type(2)));
typedef float x6f2 __attribute__((ext_vector_type(2)));
typedef float x6f4 __attribute__((ext_vector_type(4)));
typedef float x6f16 __attribute__((ext_vector_type(16)));
typedef int x6i4 __attribute__((ext_vector_type(4)));
typedef __bf16 x6b8 __attribute__((ext_vector_type(8)));
typedef __bf16 x6b2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kOOB6 = 0x80000000u;

__device__ inline x6i4 rsrc6(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  x6i4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xffffu);  // stride 0
  r.z = (int)kOOB6;                             // num_records: offsets >= 2^31 read as zero
  r.w = 0x00020000;
  // wave-uniform by construction; readfirstlane keeps it in SGPRs for the "s" asm operands
  r.x = __builtin_amdgcn_readfirstlane(r.x);
  r.y = __builtin_amdgcn_readfirstlane(r.y);
  return r;
}

// 16 B per lane from global (buffer offset voff) into LDS at m0 + 16 * lane (m0 = wave base).
__device__ inline void dma6(x6i4 rsrc, uint32_t lds_wave, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds_wave), "v"(voff), "s"(rsrc)
               : "memory");
}

__device__ inline x6f4 vload6(x6i4 rsrc, uint32_t voff) {
  x6f4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rsrc) : "memory");
  return v;
}

// wait until at most N vector-memory ops of this wave are outstanding, then LDS ops, then barrier
template <int N>
__device__ inline void step_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt");
#ifdef DDMI_X6_NOBAR  // timing diagnostic only (variant build x6nb): races by construction
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
#else
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
#endif
}

template <int N>
__device__ inline void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ inline void split4(const x6f4 v, uint2& hi, uint2& lo) {
  const x6h2 h01 = __builtin_convertvector((x6f2){v.x, v.y}, x6h2);
  const x6h2 h23 = __builtin_convertvector((x6f2){v.z, v.w}, x6h2);
  const x6f2 f01 = __builtin_convertvector(h01, x6f2);
  const x6f2 f23 = __builtin_convertvector(h23, x6f2);
  const x6h2 l01 = __builtin_convertvector((x6f2){v.x - f01.x, v.y - f01.y}, x6h2);
  const x6h2 l23 = __builtin_convertvector((x6f2){v.z - f23.x, v.w - f23.y}, x6h2);
  hi = make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
  lo = make_uint2(__builtin_bit_cast(uint32_t, l01), __builtin_bit_cast(uint32_t, l23));
}

__device__ inline uint2 to_bf16x4(const x6f4 v) {  // RNE (v_cvt_pk_bf16_f32)
  const x6b2 b01 = __builtin_convertvector((x6f2){v.x, v.y}, x6b2);
  const x6b2 b23 = __builtin_convertvector((x6f2){v.z, v.w}, x6b2);
  return make_uint2(__builtin_bit_cast(uint32_t, b01), __builtin_bit_cast(uint32_t, b23));
}

// Does a halo issue (at tap TA of some chunk) fall in the D steps before step t, i.e. after the B
// DMAs of step t were issued (D steps earlier, ahead of that step's halo)? For the first chunk the
// window stops at step 0 (the prologue issued chunk 0's halo before every B DMA).
constexpr bool halo_in_window(int t, int D, int TA, bool first) {
  for (int j = 1; j <= D; ++j) {
    const int u = t - j;
    if (first && u < 0) return false;
    if (((u % 9) + 9) % 9 == TA) return true;
  }
  return false;
}

}  // namespace

#ifdef DDMI_X6_STAMPS
// diagnostic build only (DDMI_BUILD_VARIANT=x6st, tools/micro/build_conv_bench.sh x6st): per-workgroup
// s_memtime at start / K loop entry / K loop exit / end
__device__ unsigned long long g_x6_st[8192 * 4];
extern "C" int dd_x6_stamps_read(unsigned long long* h, int n) {
  void* d = nullptr;  // read, then clear for the next launch
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_x6_st)) != hipSuccess) return -1;
  if (hipMemcpy(h, d, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(d, 0, (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#define X6_STAMP(k) x6st[k] = __builtin_amdgcn_s_memtime()
#else
#define X6_STAMP(k)
#endif

// TH x TW output pixels x BN channels per workgroup of WM x WN waves; B ring of NSLOT slots filled
// D steps ahead (NSLOT >= D + 1). SH = 1: ONE halo buffer (the next chunk's halo is written after a
// barrier that retires every wave's last read of the current one), so a 4-wave BN = 64 workgroup
// fits twice per CU (66 KB of LDS) and one workgroup's prologue / epilogue runs beside the other's
// MFMAs.
// PREC 0: f16x3 (32-channel chunks; a halo pixel row / B slot holds the hi and lo fp16 images of them);
// PREC 1: bf16 (64-channel chunks; the same bytes hold channels 0-31 and 32-63 of the chunk in bf16, and
// each fragment set feeds two bf16 MFMAs, ah*bh + al*bl, instead of three f16 ones - one product per MAC).
template <int TH, int TW, int BN, int WM, int WN, int D, int NSLOT, int SH, int PREC>
__global__ __launch_bounds__(64 * WM * WN, SH >= 2 ? SH + 1 : (SH ? (WM * WN == 8 ? 4 : 2) : 1)) void conv_x6_kernel(ConvArgs a, int tiles_x, int tiles_y, int n_sp,
                                                               int ntn, int nchunks) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int BM = TH * TW;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && TM * WM * 32 == BM && TN * WN * 32 == BN, "wave tiling");
  static_assert(NSLOT >= D + 1 && D >= 1 && D <= 8, "ring");
  constexpr int P = TW + 2;                 // halo row pitch (pixels); even
  constexpr int HP = (TH + 2) * P;          // halo pixels
  constexpr int ABYTES = HP * 128;          // one split halo buffer
  constexpr int BIMG = BN * 64;             // one B image of one ring slot
  constexpr int BSLOT = 2 * BIMG;
  constexpr int BQ = BN / 16;               // DMA instructions per image per step
  constexpr int BPS = 2 * BQ / NW;          // per wave per step
  static_assert(BPS >= 1 && (2 * BQ) % NW == 0 && BQ % BPS == 0, "B DMA split over the waves");
  constexpr int CH = PREC ? 64 : 32;           // input channels per K chunk
  constexpr int QP = CH / 4;                   // float4 quads per halo pixel per chunk
  constexpr int ALD = (HP * QP + NT - 1) / NT;  // halo float4 loads per thread per chunk
  constexpr int TA = 1;                        // tap step at which the next chunk's halo is issued
  constexpr int NHB = SH ? 1 : 2;          // halo buffers
  constexpr int B_OFF = NHB * ABYTES;
  constexpr int LDS_MAIN = NHB * ABYTES + NSLOT * BSLOT, LDS_EPI = BM * BN * 4;
  __shared__ __attribute__((aligned(1024))) char lds[LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI];
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef DDMI_X6_STAMPS
  unsigned long long x6st[4];
#endif
  X6_STAMP(0);

  // ---- tile (XCD-aware bijective remap: each XCD takes a contiguous run of tiles, N-tile major)
  const int nblk = n_sp * ntn;
  int tile = blockIdx.x;
  if (nblk >= 16) {
    const int q = nblk / 8, r = nblk % 8, x = tile % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
  }
  const int nt_idx = tile / n_sp;
  const int sp = tile - nt_idx * n_sp;
  const int txi = sp % tiles_x;
  const int t2 = sp / tiles_x;
  const int tyi = t2 % tiles_y;
  const int nimg = t2 / tiles_y;
  const int oy0 = tyi * TH, ox0 = txi * TW;
  const int n0 = nt_idx * BN;
  const int Cin = a.Cin;

  const x6i4 rin = rsrc6(a.in);

  // ---- halo staging: thread element e = tid + NT i -> halo pixel e >> 3, channels 4 (e & 7) ..
  // hofs: element offset of (pixel, 4q) at chunk 0, or -1 (zero fill); hwad: LDS byte offset (in a
  // halo buffer) of the hi 8 bytes (bf16: of the quad's 8 bytes), -1 = no write. Kept in registers for
  // 8-wave workgroups, recomputed per use by 4-wave ones (ALD = 11), whose register file is the limit.
  constexpr bool HKEEP = NW == 8 && ALD <= 12 && !SH;
  auto hofs_of = [&](int i) {
    const int e = tid + NT * i;
    const int px = e / QP, q = e % QP;
    const int hy = px / P, hx = px - (px / P) * P;
    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
    const bool in = px < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    return in ? (int)(nimg * a.in_sn + iy * a.in_sh + ix * a.in_sw) + 4 * q : -1;
  };
  auto hwad_of = [&](int i) {
    const int e = tid + NT * i;
    const int px = e / QP, q = e % QP;
    const int q7 = q & 7, half = q >> 3;  // bf16: quads 8..15 (channels 32..63) fill the second 64 B
    const int hx = px - (px / P) * P;
    return px < HP ? (px * 128 + ((((q7 >> 1) ^ (hx >> 1)) & 7) << 4) + ((q7 & 1) << 3)) ^ (half << 6) : -1;
  };
  int hofs[HKEEP ? ALD : 1], hwad[HKEEP ? ALD : 1];
  if constexpr (HKEEP) {
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      hofs[i] = hofs_of(i);
      hwad[i] = hwad_of(i);
    }
  }
  x6f4 hr[ALD];
  auto halo_issue = [&](int c) {
    const bool cv = c < nchunks;
    const int co = c * CH;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      const int ho = HKEEP ? hofs[HKEEP ? i : 0] : hofs_of(i);
      hr[i] = vload6(rin, (cv && ho >= 0) ? (uint32_t)(ho + co) * 4u : kOOB6);
    }
  };
  auto halo_tie = [&]() {  // after a wait: no use of the staged registers may move above it
#pragma unroll
    for (int i = 0; i < ALD; ++i) asm volatile("" : "+v"(hr[i]));
  };
  auto halo_store = [&](int buf) {
    char* base = lds + buf * ABYTES;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      const int hw = HKEEP ? hwad[HKEEP ? i : 0] : hwad_of(i);
      if (hw < 0) continue;
      if constexpr (PREC == 1) {
        *reinterpret_cast<uint2*>(base + hw) = to_bf16x4(hr[i]);
      } else {
        uint2 hi, lo;
        split4(hr[i], hi, lo);
        *reinterpret_cast<uint2*>(base + hw) = hi;
        *reinterpret_cast<uint2*>(base + (hw ^ 64)) = lo;
      }
    }
  };

  // ---- B ring DMA: wave instruction j covers one image, rows rb .. rb+15 of the slot
  uint32_t boff[BPS];
  bool bok[BPS];
  int brow[BPS];
#pragma unroll
  for (int j = 0; j < BPS; ++j) {
    const int qi = wave * BPS + j;
    const int rb = (qi % BQ) * 16;
    const int c = rb + (lane >> 2);
    const int ls = (lane & 3) ^ ((c >> 2) & 3);
    const int n = n0 + c;
    bok[j] = n < a.Cout;
    boff[j] = (uint32_t)(n * (int)a.ldh + ls * 8) * 2u;
    brow[j] = rb;
  }
  const bool bimg_lo = (wave * BPS) / BQ == 1;
  // f16x3: the second image of a slot is the lo split image; bf16: channels 32..63 of the same image
  const x6i4 rwb = rsrc6((bimg_lo && !PREC) ? (const void*)a.wl : (const void*)a.wh);
  const uint32_t kb_lo = (PREC && bimg_lo) ? 64u : 0u;
  auto b_issue = [&](int slot, int tap, int c) {
    const bool cv = c < nchunks;
    const uint32_t kb = (uint32_t)(tap * Cin + c * CH) * 2u + kb_lo;
#pragma unroll
    for (int j = 0; j < BPS; ++j) {
      const uint32_t dst = lds_u32 + B_OFF + slot * BSLOT + (bimg_lo ? BIMG : 0) + brow[j] * 64;
      dma6(rwb, __builtin_amdgcn_readfirstlane(dst), (cv && bok[j]) ? boff[j] + kb : kOOB6);
    }
  };

  // ---- fragment addresses
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, hh = lane >> 5;
  int aad[TM][3];  // A (hi, k16 step 0) byte offset in a halo buffer for tap (0, kw)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = (wm * TM + i) * 32 + li;
    const int y = m / TW, x = m % TW;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) aad[i][kw] = (y * P + x + kw) * 128 + (((hh ^ ((x + kw) >> 1)) & 7) << 4);
  }
  int bad_[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c = (wn * TN + j) * 32 + li;
    bad_[j] = c * 64 + (((hh ^ (c >> 2)) & 3) << 4);
  }

  x6f16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // PIPE: each half-step's fragment reads are issued under the previous half-step's MFMAs (two fragment sets in
  // registers). The two-per-CU 8-wave form (128 VGPRs) keeps one set: reads, then their MFMAs - the other three
  // waves of its SIMD cover the LDS latency. (Every step barrier drains lgkmcnt: the compiler may sink a step's
  // MFMAs below the barrier asm, and with them the wait on its fragment reads, while another wave's DMA for step
  // s + D already targets that slot.)
  constexpr bool PIPE = !(SH && NW == 8);
  // fragments of one k16 half-step: F0 = (step, s2 = 0), F1 = (step, s2 = 1)
  struct Frag {
    x6h8 ah[TM], al[TM], bh[TN], bl[TN];
  };
  Frag F0, F1;
  auto load_frag = [&](Frag& F, int slot, int c, auto TAP, auto S2) {
    constexpr int t = decltype(TAP)::value, s2 = decltype(S2)::value;
    constexpr int kh = t / 3, kw = t % 3;
    const char* abuf = lds + (SH ? 0 : (c & 1)) * ABYTES + kh * P * 128;
    const char* bbuf = lds + B_OFF + slot * BSLOT;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = bad_[j] ^ (32 * s2);
      F.bh[j] = *reinterpret_cast<const x6h8*>(bbuf + o);
      F.bl[j] = *reinterpret_cast<const x6h8*>(bbuf + BIMG + o);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int o = aad[i][kw] ^ (32 * s2);
      F.ah[i] = *reinterpret_cast<const x6h8*>(abuf + o);
      F.al[i] = *reinterpret_cast<const x6h8*>(abuf + (o ^ 64));
    }
  };
  auto mfma_frag = [&](const Frag& F) {
    if constexpr (PREC == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(x6b8, F.ah[i]),
                                                             __builtin_bit_cast(x6b8, F.bh[j]), acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(x6b8, F.al[i]),
                                                             __builtin_bit_cast(x6b8, F.bl[j]), acc[i][j], 0, 0, 0);
      return;
    }
    // small terms first, the hi x hi term last (independent accumulators interleaved)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[i], F.bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bh[j], acc[i][j], 0, 0, 0);
  };

  // Barrier opening step (c, t): this wave's B(c, t) DMAs have landed (vmcnt = memory ops issued
  // after them: B of the next D-1 steps, plus the halo loads if they were issued in the D steps
  // before), every wave's have (barrier), and every wave finished reading step (c, t) - 1.
  // Then: issue B(s + D); at t == TA the halo of chunk c + 1.
  int slot = 0;  // ring slot of the current step
  auto open_step = [&](int c, auto TAP, auto FIRST) {
    constexpr int t = decltype(TAP)::value;
    constexpr bool first = decltype(FIRST)::value;
    constexpr int N = (D - 1) * BPS + (halo_in_window(t, D, TA, first) ? ALD : 0);
    step_barrier<N>();
    constexpr int tn = (t + D) % 9;
    int ns = slot + D;
    if (ns >= NSLOT) ns -= NSLOT;
    b_issue(ns, tn, t + D >= 9 ? c + 1 : c);
    if constexpr (t == TA) halo_issue(c + 1);
  };

  // ---- prologue: halo of chunk 0, B of steps 0 .. D-1, open step 0, its first fragments
  halo_issue(0);
#pragma unroll
  for (int u = 0; u < D; ++u) b_issue(u % NSLOT, u, 0);
  wait_vm<D * BPS>();
  halo_tie();
  halo_store(0);
  open_step(0, std::integral_constant<int, 0>(), std::true_type());
  if constexpr (PIPE) load_frag(F0, 0, 0, std::integral_constant<int, 0>(), std::integral_constant<int, 0>());

  // step (c, t), software pipelined: [F1 reads] [MFMAs F0] [(t == 8) halo c+1 -> other buffer]
  // [open step s+1] [F0 reads of s+1] [MFMAs F1]: every fragment read is in flight under the
  // previous half-step's MFMAs, and the MFMAs after the barrier need no LDS wait.
  auto step = [&](int c, auto TAP, auto FIRST) {
    constexpr int t = decltype(TAP)::value;
    constexpr bool first = decltype(FIRST)::value;
    if constexpr (!PIPE) {
      load_frag(F0, slot, c, TAP, std::integral_constant<int, 0>());
      mfma_frag(F0);
      load_frag(F0, slot, c, TAP, std::integral_constant<int, 1>());
      mfma_frag(F0);
      if constexpr (t == 8) {
        wait_vm<(8 - TA) * BPS>();
        halo_tie();
        // every wave's fragment reads of this chunk's halo have returned
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        halo_store(0);
      }
      if (++slot == NSLOT) slot = 0;
      open_step(t == 8 ? c + 1 : c, std::integral_constant<int, (t + 1) % 9>(),
                std::integral_constant<bool, first && t != 8>());
      return;
    }
    load_frag(F1, slot, c, TAP, std::integral_constant<int, 1>());
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs they overlap
    mfma_frag(F0);
    if constexpr (t == 8) {
      // the halo of chunk c+1 was issued when step TA opened; younger: B issued at steps TA+1 .. 8
      wait_vm<(8 - TA) * BPS>();
      halo_tie();
      if constexpr (SH) {
        // every wave's fragment reads of this chunk's halo (the F1 reads above) have returned
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        halo_store(0);
      } else {
        halo_store((c + 1) & 1);
      }
    }
    constexpr int t1 = (t + 1) % 9;
    const int c1 = t == 8 ? c + 1 : c;
    if (++slot == NSLOT) slot = 0;
    open_step(c1, std::integral_constant<int, t1>(), std::integral_constant<bool, first && t != 8>());
    load_frag(F0, slot, c1, std::integral_constant<int, t1>(), std::integral_constant<int, 0>());
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(F1);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto chunk = [&](int c, auto FIRST) {
    step(c, std::integral_constant<int, 0>(), FIRST);
    step(c, std::integral_constant<int, 1>(), FIRST);
    step(c, std::integral_constant<int, 2>(), FIRST);
    step(c, std::integral_constant<int, 3>(), FIRST);
    step(c, std::integral_constant<int, 4>(), FIRST);
    step(c, std::integral_constant<int, 5>(), FIRST);
    step(c, std::integral_constant<int, 6>(), FIRST);
    step(c, std::integral_constant<int, 7>(), FIRST);
    step(c, std::integral_constant<int, 8>(), FIRST);
  };
  X6_STAMP(1);
  chunk(0, std::true_type());
  for (int c = 1; c < nchunks; ++c) chunk(c, std::false_type());
  // drain the trailing (all-OOB) DMAs and LDS reads; every wave done with the ring and the halo
  step_barrier<0>();
  X6_STAMP(2);

  // ---- epilogue through LDS: the 256 x BN fp32 tile is parked as [pixel][BN], then every lane
  // finishes 16-B channel quads: weight scale, alpha, bias, residual, ReLU, one 16-B store.
  // C/D map of 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5).
  constexpr int QN = BN / 4;  // channel quads per pixel
  static_assert(NT % QN == 0, "epilogue quads");
  const int qn = tid % QN;    // fixed per thread (NT % QN == 0)
  const int nq = n0 + 4 * qn;
  const bool nv = nq < a.Cout;
  float* out = a.out + (int64_t)nimg * a.out_sn + nq;
  const float* res = a.res ? a.res + (int64_t)nimg * a.res_sn + nq : nullptr;
  const int osh = (int)a.out_sh, osw = (int)a.out_sw;
  const int rsh = (int)a.res_sh, rsw = (int)a.res_sw;
  // the residual / scale / bias loads go out before the accumulators are parked, so their latency
  // hides under the LDS staging and its barrier (when the per-thread residual fits beside the
  // accumulators; 4-wave workgroups load it after the barrier)
  constexpr int IT = BM / (NT / QN);  // pixels per thread
  // (8-wave workgroups: up to 16 quads - the fragment / halo registers are dead by now; ~1 % on the BN = 128
  // layers, same-box A/B)
  constexpr bool EARLY = IT <= (NW == 8 && !SH ? 16 : 8);
  x6f4 rv[IT];
  int ooff[IT];
  auto load_res = [&]() {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int p = tid / QN + k * (NT / QN);
      const int oy = oy0 + p / TW, ox = ox0 + p % TW;
      const bool ok = nv && oy < a.Ho && ox < a.Wo;
      ooff[k] = ok ? oy * osh + ox * osw : -1;
      rv[k] = (res && ok) ? *reinterpret_cast<const x6f4*>(res + (oy * rsh + ox * rsw)) : (x6f4){0.f, 0.f, 0.f, 0.f};
    }
  };
  if constexpr (EARLY) load_res();
  x6f4 scl = {0.f, 0.f, 0.f, 0.f}, bia = {0.f, 0.f, 0.f, 0.f};
  if (nv) {
    scl = *reinterpret_cast<const x6f4*>(a.wsinv + nq) * a.alpha;
    if (a.bias) bia = *reinterpret_cast<const x6f4*>(a.bias + nq);
  }
  float* ct = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        ct[m * BN + (wn * TN + j) * 32 + li] = acc[i][j][r];
      }
  __syncthreads();
  if constexpr (!EARLY) load_res();
  bool bad = false;
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    if (ooff[k] < 0) continue;
    const int p = tid / QN + k * (NT / QN);
    const x6f4 acc_v = *reinterpret_cast<const x6f4*>(ct + p * BN + 4 * qn);
    bad |= !(__builtin_isfinite(acc_v.x) && __builtin_isfinite(acc_v.y) && __builtin_isfinite(acc_v.z) &&
             __builtin_isfinite(acc_v.w));
    x6f4 v = acc_v * scl + bia + rv[k];
    if (a.relu) {
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
    }
    // nontemporal output stores (common.h epi_quads: +0.5 % scenes/s with all three sites)
    __builtin_nontemporal_store(v, reinterpret_cast<x6f4*>(out + ooff[k]));
    if (a.pool_out) *reinterpret_cast<x6f4*>(ct + p * BN + 4 * qn) = v;  // the finished value, for the pool
  }
  if (a.pool_out) {
    // fused GPT token pooling: every P x P window of the tile (the launcher checked that windows never
    // straddle tiles and that tiles lie inside the map), summed dy-outer / dx-inner as avgpool_kernel
    __syncthreads();
    const int P = a.pool_p, WX = TW / P, NWIN = (TH / P) * WX;
    const float inv = 1.0f / (float)(P * P);
    for (int w = tid; w < NWIN * QN; w += NT) {
      const int win = w / QN, q = w - win * QN;
      const int nc = n0 + 4 * q;
      if (nc >= a.Cout) continue;
      const int wy = win / WX, wx = win - wy * WX;
      x6f4 sum = {0.f, 0.f, 0.f, 0.f};
      for (int dy = 0; dy < P; ++dy)
        for (int dx = 0; dx < P; ++dx)
          sum += *reinterpret_cast<const x6f4*>(ct + ((wy * P + dy) * TW + wx * P + dx) * BN + 4 * q);
      x6f4 v = sum * inv;
      const int py = oy0 / P + wy, px = ox0 / P + wx;
      if (a.pool_add) v += *reinterpret_cast<const x6f4*>(a.pool_add + py * a.pool_add_sh + px * a.pool_add_sw + nc);
      *reinterpret_cast<x6f4*>(a.pool_out + nimg * a.pool_sn + py * a.pool_sh + px * a.pool_sw + nc) = v;
    }
  }
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
#ifdef DDMI_X6_STAMPS
  __syncthreads();
  X6_STAMP(3);
  if (tid == 0 && blockIdx.x < 8192)
    for (int k = 0; k < 4; ++k) g_x6_st[blockIdx.x * 4 + k] = x6st[k];
#endif
}

template <int TH, int TW, int BN, int WM, int WN, int D, int NSLOT, int SH, int PREC>
static void launch_x6_one(const ConvArgs& a_in, hipStream_t st) {
  ConvArgs a = a_in;
  // fused token pooling: whole tiles only, windows inside tiles, 16-B aligned channel quads
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool pool = a.pool_out && a.pool_p >= 1 && TH % a.pool_p == 0 && TW % a.pool_p == 0 && a.Ho % TH == 0 &&
                    a.Wo % TW == 0 && al16(a.pool_out) && a.pool_sn % 4 == 0 && a.pool_sh % 4 == 0 &&
                    a.pool_sw % 4 == 0 && (!a.pool_add || (al16(a.pool_add) && a.pool_add_sh % 4 == 0 &&
                                                           a.pool_add_sw % 4 == 0));
  if (!pool) a.pool_out = nullptr;
  set_last_conv_pooled(pool);
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  const int n_sp = a.Nimg * tiles_x * tiles_y;
  const int ntn = (a.Cout + BN - 1) / BN;
  static const std::string name = "conv_x6<" + std::to_string(TH) + "," + std::to_string(TW) + "," +
                                  std::to_string(BN) + "," + std::to_string(WM) + "," + std::to_string(WN) +
                                  (PREC ? ",bf16>" : ">");
  set_last_conv_config(name.c_str());
  hipLaunchKernelGGL((conv_x6_kernel<TH, TW, BN, WM, WN, D, NSLOT, SH, PREC>), dim3(n_sp * ntn), dim3(64 * WM * WN), 0,
                     st, a, tiles_x, tiles_y, n_sp, ntn, a.Cin / (PREC ? 64 : 32));
  DD_HIP_CHECK(hipGetLastError());
}
template <int TH, int TW, int BN, int WM, int WN, int D, int NSLOT, int SH>
static void launch_x6_cfg(const ConvArgs& a, hipStream_t st) {
  if constexpr (SH == 0) {
    if (a.prec == 1) {
      launch_x6_one<TH, TW, BN, WM, WN, D, NSLOT, SH, 1>(a, st);
      return;
    }
  } else {
    if (a.prec == 1) throw std::runtime_error("conv_x6: bf16 takes the 8-wave configurations");
  }
  launch_x6_one<TH, TW, BN, WM, WN, D, NSLOT, SH, 0>(a, st);
}

// Returns false when the conv is not a 3x3 / stride 1 / pad 1 f16x3 / bf16 conv this kernel covers (the
// caller then takes conv_x5 / conv_x3).
bool launch_conv_x6(const ConvArgs& a, hipStream_t st) {
  if ((a.prec != 0 && a.prec != 1) || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 ||
      a.Cin % (a.prec ? 64 : 32) != 0 || a.batch != 1 || a.b_kn)
    return false;
  if (a.Ho != a.H || a.Wo != a.W || a.Ho < 8) return false;
  // the epilogue moves 16-B channel quads
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (a.Cout % 4 || a.out_sw % 4 || a.out_sh % 4 || a.out_sn % 4 || !al16(a.out) || !al16(a.wsinv) ||
      (a.bias && !al16(a.bias)))
    return false;
  if (a.res && (a.res_sw % 4 || a.res_sh % 4 || a.res_sn % 4 || !al16(a.res))) return false;
  // int32 offsets inside the kernel (the launcher checks the 2 GiB buffer-offset bound)
  if ((int64_t)a.Nimg * a.in_sn >= (int64_t(1) << 29) || (int64_t)a.Cout * a.ldh >= (int64_t(1) << 30)) return false;
  // 8 x 8 maps (LiDAR layer 4): one 8 x 8 tile per image, 8 waves of 32 x 32 (wave tile 32 rows x 32
  // channels: 4 fragment reads per 3 MFMAs, the LDS keeps up at this layer's 144 K steps); 102 -> 68 us per
  // launch against conv_x3. (The same tile on the 16 x 16 LiDAR layer-3 maps, whose 16 x 16 tiles leave half
  // the CUs idle, measured 72 us against 61: the 10 x 10 halo per 64 pixels costs more than the idle CUs.)
  if (a.Ho == 8 && a.Wo == 8 && a.Cout % 128 == 0) {
    if ((int64_t)a.Nimg * (a.Cout / 128) < 128) return false;
    launch_x6_cfg<8, 8, 128, 2, 4, 3, 4, 0>(a, st);
    return true;
  }
  const bool wide = a.Ho < 16;  // 8 x 32 tiles for the 8-row maps (layer4 of the image trunk)
  if (wide && a.Wo < 32) return false;
  const int64_t n_sp = (int64_t)a.Nimg * (wide ? ((a.Ho + 7) / 8) * ((a.Wo + 31) / 32)
                                               : ((a.Ho + 15) / 16) * ((a.Wo + 15) / 16));
  const bool bn128 = a.Cout > 64 && n_sp * ((a.Cout + 127) / 128) >= 256;
  // BN = 64 with Cin <= 64 (2 K chunks per tile: prologue / epilogue-heavy): 4-wave workgroups
  // (wave tile 64 x 64) with one halo buffer, two per CU - 12 % faster on the 64-channel layers,
  // 11 % slower at Cin = 256 (tools/micro/conv_bench). bf16 keeps the 8-wave form (its 64-channel halo
  // chunk would double the 4-wave form's staging registers)
  // (measured and removed in round 6, git history: a two-per-CU BN = 128 form on 8 x 16 tiles, +-4 %, and a
  // three-per-CU BN = 64 layer-1 form, 0.3 % slower at 3 lanes in flight)
  const bool sh4 = a.prec == 0 && a.Cin <= 64;
  const bool b128 = bn128;
#define X6(TH, TW, BN, WM, WN, D, NS, SH) launch_x6_cfg<TH, TW, BN, WM, WN, D, NS, SH>(a, st)
  // small grids (batches of a few scenes): the routed form would run fewer than 128 workgroups, each through the
  // whole K loop; 8 x 8 pixel tiles x 64 channels (4 waves of 32 x 32) give 4-8x the workgroups at a quarter of the
  // work per K step. The K order (32-channel chunk, tap, k16 half) is every form's: bit-identical results.
  // DDMI_X6_SMALL=0 keeps the routed form, 2 forces the small-grid form (A/B).
  {
    const int64_t wgs = b128 ? n_sp * ((a.Cout + 127) / 128) : n_sp * ((a.Cout + 63) / 64);
    const char* se = getenv("DDMI_X6_SMALL");
    const int sm = se ? atoi(se) : 1;
    if (sm == 2 || (wgs < 128 && sm != 0)) {
      X6(8, 8, 64, 2, 2, 2, 3, 0);
      return true;
    }
  }
  if (wide) {
    if (b128) {
      X6(8, 32, 128, 4, 2, 3, 4, 0);
    } else {
      if (sh4) X6(8, 32, 64, 4, 1, 2, 3, 1); else X6(8, 32, 64, 4, 2, 2, 3, 0);
    }
  } else {
    if (b128) {
      X6(16, 16, 128, 4, 2, 3, 4, 0);
    } else {
      if (sh4) X6(16, 16, 64, 4, 1, 2, 3, 1); else X6(16, 16, 64, 4, 2, 2, 3, 0);
    }
  }
#undef X6
  return true;
}

}  // namespace ddmi
