// Implicit-GEMM convolution / GEMM on CDNA4 f16 MFMA with a 3-product fp16 split
// ("f16x3": fp32-class accuracy at 5.3x the fp32-MFMA issue rate).
//
// Same contract as conv_gemm.hip (ConvArgs; the reference ops it carries are listed there). Every
// fp32 operand x is split into two fp16 values, hi = f16(x) and lo = f16(x - hi), so
// x = hi + lo + r with |r| <= 2^-22 |x| (RNE twice). The product a*b is taken as
//     ah*bh + ah*bl + al*bh          (the al*bl term is <= 2^-22 |a b| and dropped)
// on v_mfma_f32_32x32x16_f16 with fp32 accumulation: each f16 x f16 product is exact in fp32, so
// the only error beyond the fp32 path's summation-order difference is the <= ~3*2^-22 relative
// per-product split residue. Measured end to end: waypoint L2 vs the fp64
// restatement 1.2e-5, vs 9.5e-6 for plain fp32 - the same class; the bar is 1e-4.
//
// Range: weights are pre-split on the host with a per-output-channel power-of-two scale that puts
// max|w| at 2^15 (exact; undone in the epilogue), so no weight lo part is lost to fp16 subnormals.
// Activations are split unscaled: an |x| >= 65504 overflows its fp16 hi part, which makes every
// output it feeds non-finite; the epilogue ORs DD_NUM_F16_OVERFLOW into *flags for any non-finite
// accumulator (the runtime reports it via dd_numerics_flags; the host raises / re-runs in fp32). Activations below 2^-3 have a subnormal lo part: absolute error
// <= 2^-25, negligible against the row sums it feeds.
//
// Tiling (MI355X-first):
//  * WM x WN waves (64*WM*WN threads), each wave TM x TN 32x32 MFMA tiles; BK = 32.
//  * A (fp32 NHWC activations) is loaded as 16-B float4 channel slices with raw buffer loads (OOB
//    offset -> hardware zero for conv padding and ragged edges, no per-load branches), split in
//    registers, and written to LDS as separate hi / lo images. B (pre-split fp16 weights, [N][Kp])
//    is loaded as 16-B pieces straight into its hi / lo images. LDS rows are 64 B (32 halfs) with
//    the 16-B slot XOR-swizzled by (row >> 2) & 3 so that a 16-lane ds_read_b128 group (16
//    consecutive rows, one slot) covers all 16 slots of a 256-B bank row: conflict-free.
//  * Double-buffered LDS; chunk k+1's global loads are in flight during chunk k's MFMAs.
//  * XCD-aware bijective tile remap (blocks b, b+8, ... share an XCD's L2 -> consecutive tiles).
//  * Fused epilogue: per-channel weight scale, alpha, bias, residual, ReLU, strided NHWC store.
#include <type_traits>

#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr uint32_t kOOB = 0x80000000u;

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kOOB, 0x00020000);
}

__device__ inline uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0);
  return *reinterpret_cast<uint4*>(&v);
}

}  // namespace

// SPLIT: blockIdx.y = split sp of gridDim.y takes K chunks [nk sp / S, nk (sp + 1) / S) and stores its raw
// accumulators into ConvArgs::split_part[sp][M][Cout] (x3_split_reduce applies the epilogue)
template <int WM, int WN, int TM, int TN, int MODE, int PREC = 0, int GATHER = 0, int SPLIT = 0>
__global__ __launch_bounds__(64 * WM * WN) void conv_x3_kernel(ConvArgs a, int M, int K, int n_tiles_m,
                                                               int n_tiles_n) {
  // MODE 1: Cin % 32 == 0 and KH*KW <= 32 - a 32-wide K chunk lies inside one filter tap, the
  //         tap walk is scalar and each A row carries a precomputed base offset + tap-valid mask;
  // MODE 0: generic K (stem 7x7 on 4 padded channels, small Cin): per-lane tap decode.
  // PREC 0: f16x3 (hi / lo images of both operands, 3 MFMA products);
  // PREC 1: bf16 (one bf16 image per operand, 1 MFMA product) - the reduced-precision mode.
  // GATHER 1: gathered output rows (ConvArgs::rowmap, MODE 1 only), compacted over the images when
  //           ConvArgs::rowcount is set (the decoder's value_proj at the grid-sample taps).
  constexpr int NT = 64 * WM * WN;
  static_assert(!GATHER || MODE == 1, "gathered rows take the MODE-1 tap walk");
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int A_LD = BM * (BK / 4) / NT;  // float4 A pieces per thread per chunk
  constexpr int B_LD = BN * 4 / NT;         // 16-B B pieces per thread per chunk, per image (hi / lo)
  static_assert(A_LD >= 1 && BM * (BK / 4) % NT == 0, "A tile / threads");
  static_assert(B_LD >= 1 && BN * 4 % NT == 0, "B tile / threads");
  constexpr int ROWB = BK * 2;                       // 64-B LDS rows (32 halfs)
  constexpr int NIMG = PREC == 0 ? 2 : 1;             // images per operand
  constexpr int STAGE = NIMG * (BM + BN) * ROWB;      // Ah, [Al], Bh, [Bl]
  constexpr int LDS_EPI = epi_quads_lds<WM, WN, TM, TN>();
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE > LDS_EPI ? 2 * STAGE : LDS_EPI];

  const int tid = threadIdx.x;
  // GATHER: g_rows[r] = the row-map index (= output row) of tile row r, -1 = none
  __shared__ int g_rows[GATHER ? BM : 1];
  __shared__ int g_pre[GATHER ? 257 : 1];
  const int nblk = n_tiles_m * n_tiles_n;
  const int bid = blockIdx.x;
  int tile = bid;
  // (gathered rows: the live tiles are a prefix of the grid whose length only the kernel knows - the XCD remap
  // would hand that prefix to the first XCDs alone, so consecutive tiles go round-robin over the XCDs instead)
  if (!GATHER && nblk >= 16) {
    const int q = nblk / 8, r = nblk % 8, x = bid % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int mt_idx = tile / n_tiles_n;
  const int nt_idx = tile - mt_idx * n_tiles_n;
  const int m0 = mt_idx * BM;
  const int n0 = nt_idx * BN;
  if constexpr (GATHER) {
    if (a.rowcount) {
      // exclusive prefix of the images' live-row counts; launch row m = the m-th live row in image order
      const int nimg = a.rowmap_nimg;
      rowcount_prefix(a.rowcount, nimg, g_pre);
      const int total = g_pre[nimg];
      if (m0 >= total) return;  // past every live row (workgroup-uniform)
      for (int r = tid; r < BM; r += NT) {
        const int g = m0 + r;
        int idx = -1;
        if (g < total) {
          int lo = 0, hi = nimg - 1;  // the last image whose prefix is <= g
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (g_pre[mid] <= g) lo = mid; else hi = mid - 1;
          }
          idx = lo * a.rowcap + (g - g_pre[lo]);
        }
        g_rows[r] = idx;
      }
    } else {
      for (int r = tid; r < BM; r += NT) g_rows[r] = m0 + r < M ? m0 + r : -1;
    }
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in);
  const __amdgpu_buffer_rsrc_t rwh = make_rsrc(a.wh);
  const __amdgpu_buffer_rsrc_t rwl = make_rsrc(a.wl);
  const int in_sh = (int)a.in_sh, in_sw = (int)a.in_sw;
  const int ldh = (int)a.ldh;
  const int Kp = (K + 7) & ~7;
  // this workgroup's K range (chunks of BK): the whole K, or split sp's slice
  const int nk_all = (K + BK - 1) / BK;
  const int sp = SPLIT ? (int)blockIdx.y : 0, S = SPLIT ? (int)gridDim.y : 1;
  const int c_beg = SPLIT ? nk_all * sp / S : 0, c_end = SPLIT ? nk_all * (sp + 1) / S : nk_all;
  const int kbeg = c_beg * BK;
  const int kend = SPLIT ? min(K, c_end * BK) : K;     // A reads stop here
  const int kbend = SPLIT ? min(Kp, c_end * BK) : Kp;  // B reads stop here

  // ---- per-thread A rows (fixed across K chunks)
  const int kq = tid & 7;  // float4 index inside the 32-wide K chunk
  int abase[A_LD], aih0[A_LD], aiw0[A_LD];
  uint32_t amask[A_LD];
  int any_row = 0;  // gathered rows: some row of this tile is live
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + (tid >> 3) + (NT / 8) * i;
    const bool v = m < M;
    const int mm = v ? m : 0;
    int ow = mm % a.Wo;
    const int t2 = mm / a.Wo;
    int oh = t2 % a.Ho;
    int n = t2 / a.Ho;
    bool rv = v;
    if constexpr (GATHER) {
      // gathered rows: the pixel comes from the row map (stride 1: output geometry = input's)
      const int ri = g_rows[(tid >> 3) + (NT / 8) * i];
      const int px = ri >= 0 ? a.rowmap[ri] : -1;
      rv = px >= 0;
      any_row |= (int)rv;
      const int pp = rv ? px : 0;
      ow = pp % a.W;
      oh = (pp / a.W) % a.H;
      n = pp / (a.W * a.H);
    }
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    if constexpr (MODE == 1) {
      // element offset of tap (0, 0) channel kq*4, and bit t set iff tap t reads inside the image
      abase[i] = n * (int)a.in_sn + ih0 * in_sh + iw0 * in_sw + kq * 4;
      uint32_t mk = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
            mk |= 1u << (kh * a.KW + kw);
      amask[i] = rv ? mk : 0u;
    } else {
      abase[i] = n * (int)a.in_sn;
      aih0[i] = v ? ih0 : -(1 << 28);
      aiw0[i] = iw0;
    }
  }
  // gathered rows: a tile whose rows are all don't-care (-1: the unused tail of a scene's
  // deduplicated pixel list) does no work; the predicate is workgroup-uniform
  if (GATHER && !__syncthreads_or(any_row)) return;
  // B rows: constant part of the byte offset and validity
  uint32_t boff[B_LD];
  bool bok[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int u = tid + NT * j;
    const int n = n0 + (u >> 2);
    bok[j] = n < a.Cout;
    boff[j] = (uint32_t)(n * ldh + (u & 3) * 8) * 2u;
  }

  // two register staging sets: chunk c lives in set c % 2 (global loads run two chunks ahead)
  float4 ra[2][A_LD];
  uint4 rbh[2][B_LD], rbl[2][B_LD];
  // scalar tap walk (MODE 1): the chunk at k0 reads channels ci0 .. ci0+31 of tap (kh, kw)
  int t_tap = 0, t_ci = 0, t_kw = 0, t_off = 0;
  if (SPLIT && MODE == 1) {  // the walk's state at this slice's first chunk (slices start on chunk boundaries)
    t_tap = kbeg / a.Cin;
    t_ci = kbeg - t_tap * a.Cin;
    t_kw = t_tap % a.KW;
    t_off = (t_tap / a.KW) * in_sh + t_kw * in_sw + t_ci;
  }

  auto load_chunk = [&](auto SET, int k0) {
    constexpr int S = decltype(SET)::value;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const bool ok = t_tap < 32 && ((amask[i] >> (t_tap & 31)) & 1u) && (!SPLIT || k0 < kend);
        const uint32_t off = ok ? (uint32_t)(abase[i] + t_off) * 4u : kOOB;
        uint4 u = bload16(rin, off);
        ra[S][i] = *reinterpret_cast<float4*>(&u);
      }
      // advance the walk by 32 channels (wave-uniform: SALU)
      t_ci += BK;
      t_off += BK;
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
      const int kk = k0 + kq * 4;
      const bool kv = kk < kend;
      const int tap = kk / a.Cin;
      const int ci = kk - tap * a.Cin;
      const int kh = tap / a.KW;
      const int kw = tap - kh * a.KW;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const int ih = aih0[i] + kh, iw = aiw0[i] + kw;
        const bool ok = kv && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const uint32_t off = ok ? (uint32_t)(abase[i] + ih * in_sh + iw * in_sw + ci) * 4u : kOOB;
        uint4 u = bload16(rin, off);
        ra[S][i] = *reinterpret_cast<float4*>(&u);
      }
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int kb = k0 + ((tid + NT * j) & 3) * 8;
      const uint32_t off = (bok[j] && kb < kbend) ? boff[j] + (uint32_t)k0 * 2u : kOOB;
      rbh[S][j] = bload16(rwh, off);
      if constexpr (PREC == 0) rbl[S][j] = bload16(rwl, off);
    }
  };

  // LDS byte offsets of this thread's A / B writes (fixed across chunks)
  int a_woff[A_LD], b_woff[B_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int r = (tid >> 3) + (NT / 8) * i;
    a_woff[i] = r * ROWB + (((kq >> 1) ^ ((r >> 2) & 3)) << 4) + ((kq & 1) << 3);
  }
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int u = tid + NT * j;
    const int r = u >> 2;
    b_woff[j] = r * ROWB + (((u & 3) ^ ((r >> 2) & 3)) << 4);
  }

  auto store_chunk = [&](int buf, auto SET) {
    constexpr int S = decltype(SET)::value;
    char* st = lds + buf * STAGE;
    char* sah = st;
    char* sal = st + BM * ROWB;
    char* sbh = st + NIMG * BM * ROWB;
    char* sbl = st + (NIMG * BM + BN) * ROWB;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const float4 v = ra[S][i];
      if constexpr (PREC == 1) {
        const bf16x2 b01 = __builtin_convertvector((float2_t){v.x, v.y}, bf16x2);
        const bf16x2 b23 = __builtin_convertvector((float2_t){v.z, v.w}, bf16x2);
        *reinterpret_cast<uint2*>(sah + a_woff[i]) =
            make_uint2(__builtin_bit_cast(uint32_t, b01), __builtin_bit_cast(uint32_t, b23));
        continue;
      }
      const half2_t h01 = __builtin_convertvector((float2_t){v.x, v.y}, half2_t);
      const half2_t h23 = __builtin_convertvector((float2_t){v.z, v.w}, half2_t);
      const float2_t f01 = __builtin_convertvector(h01, float2_t);
      const float2_t f23 = __builtin_convertvector(h23, float2_t);
      const half2_t l01 = __builtin_convertvector((float2_t){v.x - f01.x, v.y - f01.y}, half2_t);
      const half2_t l23 = __builtin_convertvector((float2_t){v.z - f23.x, v.w - f23.y}, half2_t);
      *reinterpret_cast<uint2*>(sah + a_woff[i]) =
          make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
      *reinterpret_cast<uint2*>(sal + a_woff[i]) =
          make_uint2(__builtin_bit_cast(uint32_t, l01), __builtin_bit_cast(uint32_t, l23));
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      *reinterpret_cast<uint4*>(sbh + b_woff[j]) = rbh[S][j];
      if constexpr (PREC == 0) *reinterpret_cast<uint4*>(sbl + b_woff[j]) = rbl[S][j];
    }
  };

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, hh = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fragment read offsets: step s of a chunk reads 16-B slot (2s + hh) of its row (swizzled)
  int a_roff[2][TM], b_roff[2][TN];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = (wm * TM + i) * 32 + li;
      a_roff[s2][i] = r * ROWB + (((2 * s2 + hh) ^ ((r >> 2) & 3)) << 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = (wn * TN + j) * 32 + li;
      b_roff[s2][j] = r * ROWB + (((2 * s2 + hh) ^ ((r >> 2) & 3)) << 4);
    }
  }

  const int nk = c_end - c_beg;
  const std::integral_constant<int, 0> I0;
  const std::integral_constant<int, 1> I1;

  auto compute = [&](int cur) {
    const char* st = lds + cur * STAGE;
    const char* sah = st;
    const char* sal = st + BM * ROWB;
    const char* sbh = st + NIMG * BM * ROWB;
    const char* sbl = st + (NIMG * BM + BN) * ROWB;
    half8 ah[2][TM], al[2][TM], bh[2][TN], bl[2][TN];
    if constexpr (PREC == 1) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bh[s2][j] = *reinterpret_cast<const half8*>(sbh + b_roff[s2][j]);
#pragma unroll
        for (int i = 0; i < TM; ++i) ah[s2][i] = *reinterpret_cast<const half8*>(sah + a_roff[s2][i]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ah[s2][i]),
                                                               __builtin_bit_cast(bf16x8, bh[s2][j]), acc[i][j], 0,
                                                               0, 0);
      return;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[s2][j] = *reinterpret_cast<const half8*>(sbh + b_roff[s2][j]);
        bl[s2][j] = *reinterpret_cast<const half8*>(sbl + b_roff[s2][j]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[s2][i] = *reinterpret_cast<const half8*>(sah + a_roff[s2][i]);
        al[s2][i] = *reinterpret_cast<const half8*>(sal + a_roff[s2][i]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      // small terms first, the hi x hi term last (independent accumulators interleaved)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s2][i], bh[s2][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s2][i], bl[s2][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s2][i], bh[s2][j], acc[i][j], 0, 0, 0);
    }
  };
  // iteration kc: MFMAs on LDS buffer kc&1, then chunk kc+1 (register set NEXT) -> LDS buffer
  // (kc+1)&1 and chunk kc+3's loads into the freed set; chunk kc+2 stays in flight meanwhile.
  // Every load / store is unconditional (chunks past K read as zeros through the OOB offset, and the
  // K loop runs to an even count): a conditional load would make hipcc's vmcnt bookkeeping fall
  // back to vmcnt(0) and drain the chunk kept in flight.
  auto iteration = [&](int kc, auto NEXT) {
    compute(kc & 1);
    store_chunk((kc + 1) & 1, NEXT);
    load_chunk(NEXT, kbeg + (kc + 3) * BK);
    __syncthreads();
  };

  load_chunk(I0, kbeg);
  load_chunk(I1, kbeg + BK);
  store_chunk(0, I0);
  load_chunk(I0, kbeg + 2 * BK);
  __syncthreads();
  for (int kc = 0; kc < nk; kc += 2) {
    iteration(kc, I1);
    iteration(kc + 1, I0);
  }

  if constexpr (SPLIT) {
    // raw partial accumulators, C layout: lanes 0-31 of a register hold 32 consecutive channels of one row
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + (wn * TN + j) * 32 + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (m < M && n < a.Cout) a.split_part[((int64_t)sp * M + m) * a.Cout + n] = acc[i][j][r];
        }
      }
    return;
  }
  // ---- epilogue: 16-B quads through LDS when every row is 16-B aligned, else per accumulator element
  bool bad = false;
  if (epi_quads_ok(a)) {
    bad = epi_quads<WM, WN, TM, TN>(a, acc, lds, m0, n0, M, tid, GATHER ? g_rows : nullptr);
  } else {
    // ---- fused epilogue. C/D map of 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5).
    // An activation beyond the fp16 range (|x| >= 65504) makes its hi part infinite, so every output
    // it feeds becomes inf / NaN: a non-finite result raises DD_NUM_F16_OVERFLOW.
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
    epi_row_table<BM, 64 * WM * WN>(a, m0, M, tid, reinterpret_cast<long long*>(lds), GATHER ? g_rows : nullptr);
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
}

template <int WM, int WN, int TM, int TN, int GATHER = 0>
static void launch_x3_cfg(const ConvArgs& a, int M, int K, hipStream_t st) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const int ntm = (M + BM - 1) / BM;
  const int ntn = (a.Cout + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, 1);
  const bool walk = a.Cin % BK == 0 && a.KH * a.KW <= 32;
  static const std::string name[2] = {
      "conv_x3<" + std::to_string(BM) + "," + std::to_string(BN) + ",f16x3>",
      "conv_x3<" + std::to_string(BM) + "," + std::to_string(BN) + ",bf16>"};
  set_last_conv_config(name[a.prec == 1].c_str());
  if constexpr (GATHER) {
    hipLaunchKernelGGL((conv_x3_kernel<WM, WN, TM, TN, 1, 0, 1>), grid, dim3(64 * WM * WN), 0, st, a, M, K, ntm, ntn);
    DD_HIP_CHECK(hipGetLastError());
    return;
  }
  if (a.prec == 1) {
    if (walk)
      hipLaunchKernelGGL((conv_x3_kernel<WM, WN, TM, TN, 1, 1>), grid, dim3(64 * WM * WN), 0, st, a, M, K, ntm, ntn);
    else
      hipLaunchKernelGGL((conv_x3_kernel<WM, WN, TM, TN, 0, 1>), grid, dim3(64 * WM * WN), 0, st, a, M, K, ntm, ntn);
  } else if (walk) {
    hipLaunchKernelGGL((conv_x3_kernel<WM, WN, TM, TN, 1>), grid, dim3(64 * WM * WN), 0, st, a, M, K, ntm, ntn);
  } else {
    hipLaunchKernelGGL((conv_x3_kernel<WM, WN, TM, TN, 0>), grid, dim3(64 * WM * WN), 0, st, a, M, K, ntm, ntn);
  }
  DD_HIP_CHECK(hipGetLastError());
}

// the K-split partials summed in split order, then conv_x3's epilogue (scale, bias, residual, ReLU, strided NHWC out)
// (SS = S as a template parameter: every split's load is issued before the ordered sum)
template <int SS>
__global__ __launch_bounds__(256) void x3_split_reduce(ConvArgs a, int M) {
  const int QN = a.Cout / 4;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * QN) return;
  const int m = (int)(e / QN), nq = 4 * (int)(e - (int64_t)m * QN);
  float4 p[SS];
#pragma unroll
  for (int sp = 0; sp < SS; ++sp)
    p[sp] = *reinterpret_cast<const float4*>(a.split_part + ((int64_t)sp * M + m) * a.Cout + nq);
  float4 s = p[0];
#pragma unroll
  for (int sp = 1; sp < SS; ++sp) {
    s.x += p[sp].x;
    s.y += p[sp].y;
    s.z += p[sp].z;
    s.w += p[sp].w;
  }
  const bool bad = !(__builtin_isfinite(s.x) && __builtin_isfinite(s.y) && __builtin_isfinite(s.z) &&
                     __builtin_isfinite(s.w));
  const int ow = m % a.Wo, t2 = m / a.Wo, oh = t2 % a.Ho, n = t2 / a.Ho;
  const float sc[4] = {a.wsinv[nq] * a.alpha, a.wsinv[nq + 1] * a.alpha, a.wsinv[nq + 2] * a.alpha,
                       a.wsinv[nq + 3] * a.alpha};
  float b[4] = {0.f, 0.f, 0.f, 0.f}, r[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.bias)
    for (int k = 0; k < 4; ++k) b[k] = a.bias[nq + k];
  if (a.res) {
    const float* rr = a.res + n * a.res_sn + oh * a.res_sh + ow * a.res_sw + nq;
    for (int k = 0; k < 4; ++k) r[k] = rr[k];
  }
  const float sv[4] = {s.x, s.y, s.z, s.w};
  float* o = a.out + n * a.out_sn + oh * a.out_sh + ow * a.out_sw + nq;
  for (int k = 0; k < 4; ++k) {
    float v = sv[k] * sc[k] + b[k] + r[k];
    if (a.relu) v = fmaxf(v, 0.f);
    o[k] = v;
  }
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
}

// K-split conv_x3 (64 x 64 tiles, f16x3, the MODE-1 tap walk) for grids far below the chip: S splits of the K chunks,
// then the reduce launch. The latency of one workgroup's whole K loop (LiDAR layer 4 at batch 1: 8 workgroups,
// K = 4608, 61-75 us) becomes S shorter loops side by side.
static int x3_split_mode() {
  // read per dispatch; 2 (default): the split ahead of conv_x6 with up to 256 workgroups, 1: only where conv_x6 /
  // conv_x5 decline (up to 128), 0: off
  const char* se = getenv("DDMI_X3_SPLIT");
  return se ? atoi(se) : 2;
}
static bool launch_x3_split(const ConvArgs& a, int M, int K, hipStream_t st, int wg_target = 128) {
  if (!x3_split_mode()) return false;
  if (!a.split_part || a.prec != 0 || a.rowmap || a.Cin % BK || a.KH * a.KW > 32 || a.Cout % 4) return false;
  const int64_t tiles = (int64_t)((M + 63) / 64) * ((a.Cout + 63) / 64);
  const int nk = (K + BK - 1) / BK;
  if (tiles >= 64 || nk < 32) return false;
  int S = 1;
  while (S < 8 && tiles * S * 2 <= wg_target && nk / (S * 2) >= 8) S *= 2;
  if (S < 2 || (int64_t)S * M * a.Cout > a.split_cap) return false;
  const int ntm = (M + 63) / 64, ntn = (a.Cout + 63) / 64;
  static const std::string name = "conv_x3<64,64,f16x3,ksplit>";
  set_last_conv_config(name.c_str());
  hipLaunchKernelGGL((conv_x3_kernel<2, 2, 1, 1, 1, 0, 0, 1>), dim3(ntm * ntn, S), dim3(256), 0, st, a, M, K, ntm,
                     ntn);
  DD_HIP_CHECK(hipGetLastError());
  const int64_t quads = (int64_t)M * (a.Cout / 4);
  const dim3 rg((unsigned)((quads + 255) / 256));
  if (S == 2)
    hipLaunchKernelGGL(x3_split_reduce<2>, rg, dim3(256), 0, st, a, M);
  else if (S == 4)
    hipLaunchKernelGGL(x3_split_reduce<4>, rg, dim3(256), 0, st, a, M);
  else
    hipLaunchKernelGGL(x3_split_reduce<8>, rg, dim3(256), 0, st, a, M);
  DD_HIP_CHECK(hipGetLastError());
  return true;
}

bool launch_conv_x5(const ConvArgs& a, int M, int K, hipStream_t st);  // conv_x5.hip
bool launch_conv_x6(const ConvArgs& a, hipStream_t st);                 // conv_x6.hip

static thread_local const char* g_last_conv = "conv_gemm";
const char* last_conv_kernel() { return g_last_conv; }
void set_last_conv_kernel(const char* k) { g_last_conv = k; }
static thread_local bool g_last_pooled = false;
bool last_conv_pooled() { return g_last_pooled; }
void set_last_conv_pooled(bool p) { g_last_pooled = p; }
static thread_local bool g_last_ln = false;
bool last_conv_ln() { return g_last_ln; }
void set_last_conv_ln(bool p) { g_last_ln = p; }
static thread_local const char* g_last_cfg = "";
const char* last_conv_config() { return g_last_cfg; }
void set_last_conv_config(const char* c) { g_last_cfg = c; }

void launch_conv_x3(const ConvArgs& a, hipStream_t st) {
  if (a.Cin % 4 != 0) throw std::runtime_error("conv_x3: Cin must be a multiple of 4");
  if ((a.in_sw % 4) || (a.in_sh % 4) || (a.in_sn % 4) || (reinterpret_cast<uintptr_t>(a.in) % 16))
    throw std::runtime_error("conv_x3: input strides / base must be 16-byte aligned");
  if (!a.wh || (a.prec == 0 && !a.wl) || !a.wsinv) throw std::runtime_error("conv_x3: missing split weights");
  if ((a.ldh % 8) || (reinterpret_cast<uintptr_t>(a.wh) % 16) || (reinterpret_cast<uintptr_t>(a.wl) % 16))
    throw std::runtime_error("conv_x3: split weight rows must be 16-byte aligned");
  if (a.batch != 1 || a.b_kn) throw std::runtime_error("conv_x3: batched / KN operands are not supported");
  const int64_t M64 = (int64_t)a.Nimg * a.Ho * a.Wo;
  if (M64 >= (int64_t(1) << 31)) throw std::runtime_error("conv_x3: M too large");
  const int M = (int)M64;
  const int K = a.KH * a.KW * a.Cin;
  if (a.ldh < K) throw std::runtime_error("conv_x3: ldh < K");
  if (M == 0 || a.Cout == 0) return;
  if (a.rowmap && (a.stride != 1 || a.Cin % BK != 0 || a.KH * a.KW > 32 || a.Nimg != 1 || a.Wo != 1 ||
                   a.rowmap_nimg < 1 || a.prec != 0))
    throw std::runtime_error("conv_x3: gathered rows need a stride-1 f16x3 MODE-1 conv into Nimg=1, Wo=1");
  if (a.rowcount && (!a.rowmap || a.rowmap_nimg > 256 || a.rowcap < 1 || (int64_t)a.rowmap_nimg * a.rowcap > M))
    throw std::runtime_error("conv_x3: compacted rows need a row map of <= 256 images x rowcap rows");
  const int64_t in_extent = (int64_t)((a.rowmap ? a.rowmap_nimg : a.Nimg) - 1) * a.in_sn + (int64_t)(a.H - 1) * a.in_sh +
                            (int64_t)(a.W - 1) * a.in_sw + a.Cin;
  if (in_extent * 4 >= (int64_t)kOOB || (int64_t)a.Cout * a.ldh * 2 >= (int64_t)kOOB)
    throw std::runtime_error("conv_x3: operand extent >= 2 GiB (split the batch)");
  if ((int64_t)a.Ho * a.out_sh >= (int64_t(1) << 31) || (int64_t)a.Ho * a.res_sh >= (int64_t(1) << 31))
    throw std::runtime_error("conv_x3: per-image output extent too large");
  set_last_conv_ln(false);
  // a fused LayerNorm of the output rows (ConvArgs::ln_out) needs one N tile spanning the row in the quad epilogue:
  // 64 x 64 tiles at Cout 64, 64 x 128 at Cout 128 (the same K order per output as every other tile: the GEMM output
  // is unchanged); otherwise the request is ignored and the caller runs its LayerNorm launch
  if (a.ln_out && a.ln_g && a.ln_b && !a.rowmap && a.KH == 1 && a.KW == 1 && (a.Cout == 64 || a.Cout == 128) &&
      epi_quads_ok(a)) {
    g_last_conv = "conv_x3";
    set_last_conv_ln(true);
    if (a.Cout == 64)
      launch_x3_cfg<2, 2, 1, 1>(a, M, K, st);  // 64 x 64
    else
      launch_x3_cfg<2, 2, 1, 2>(a, M, K, st);  // 64 x 128
    return;
  }
  ConvArgs b = a;
  b.ln_out = nullptr;  // every other route ignores it
  const ConvArgs& a0 = b;
  // default f16x3 path: 3x3 stride-1 convs on the halo-reuse direct kernel (conv_x6.hip), other
  // grids that fill the chip on the LDS-DMA implicit GEMM (conv_x5.hip), the rest here
  if (a0.rowmap) {
    g_last_conv = "conv_x3";
    launch_x3_cfg<2, 2, 2, 2, 1>(a0, M, K, st);  // gathered rows: 128 x 128
    return;
  }
  if (x3_split_mode() == 2 && launch_x3_split(a0, M, K, st, 256)) {
    g_last_conv = "conv_x3";
    return;
  }
  if (launch_conv_x6(a0, st)) {
    g_last_conv = "conv_x6";
    return;
  }
  if (launch_conv_x5(a0, M, K, st)) {
    g_last_conv = "conv_x5";
    return;
  }
  g_last_conv = "conv_x3";
  if (launch_x3_split(a0, M, K, st)) return;
  const int64_t t128 = ((M + 127) / 128) * (int64_t)((a0.Cout + 127) / 128);
  const bool generic = !(a0.Cin % BK == 0 && a0.KH * a0.KW <= 32);
  if (a0.Cout <= 64) {
    if (!generic && (M + 255) / 256 >= 256)
      launch_x3_cfg<4, 1, 2, 2>(a0, M, K, st);  // 256 x 64
    else
      launch_x3_cfg<2, 2, 1, 1>(a0, M, K, st);  // 64 x 64
  } else if (t128 >= 512) {
    launch_x3_cfg<2, 2, 2, 2>(a0, M, K, st);    // 128 x 128
  } else {
    launch_x3_cfg<2, 2, 1, 1>(a0, M, K, st);    // 64 x 64
  }
}

}  // namespace ddmi
