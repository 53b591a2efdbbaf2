// Fused timm BasicBlock of ResNet-34 layer 1 (both trunks): conv1 3x3 + bn1 + ReLU, conv2 3x3 + bn2, + identity,
// ReLU (transfuser_backbone.py:23-33,188-192; timm BasicBlock, stride 1, 64 -> 64 channels, no downsample) as ONE
// launch per block instead of two conv_x6 launches.
//
// Why: layer 1 is the least efficient stage of the trunks (0.32-0.36 of the f16x3 MFMA ceiling over 12 launches per
// forward, 2.1 ms at B = 64): with K = 576 per output a 64-channel conv is short on MFMA work per byte, and each
// conv_x6 tile alternates an MFMA phase with an HBM burst (halo in, output + residual). Here a workgroup owns a
// 16 x 16 output tile x 64 channels and keeps conv1's output for the 18 x 18 pixels conv2 reads in LDS: the
// 64-channel intermediate map never reaches HBM (per block 1.48 -> 0.96 GB at B = 64 on the image trunk) for 13 %
// more MFMA work (conv1 over 18 x 18 instead of 16 x 16 pixels).
//
// Per workgroup (8 waves, one per CU: 155 KB of LDS):
//  * conv1: M = the 18 x 18 region (324 rows in 11 tiles of 32), N = 64 (2 tiles), K = 2 chunks of 32 channels x
//    9 taps. A from the 20 x 20 input halo of the chunk (register-staged 16-B loads, split into fp16 hi / lo in
//    registers, 128-B swizzled LDS pixel rows: conv_x6.hip's halo layout); chunk 1's halo is loaded under chunk 0.
//    Wave w takes N tile w % 2 and M tiles w / 2, w / 2 + 4, w / 2 + 8 (the third for w < 6).
//  * conv1 epilogue, per N tile: the accumulators parked as fp32 [row][32] (over the dead input halo), then every
//    (pixel, channel quad): scale, bias, ReLU - conv_x6's epilogue expression - zero outside the map (conv2's zero
//    padding), split into hi / lo, into the intermediate: 2 chunk images of 18 x 18 swizzled 128-B pixel rows.
//  * conv2: conv_x6's 16 x 16 x 64 form reading the intermediate as its halo (no loads), K = 2 chunks x 9 taps.
//  * B: the two convs' pre-split weight images stream through one 3-slot LDS ring by LDS-DMA, two steps ahead, as
//    36 consecutive steps (conv1's 18, then conv2's); every vector-memory op of the loop is inline asm with an exact
//    vmcnt per step (conv_x6.hip).
//  * conv2 epilogue: conv_x6's (park, residual = the block input, bias, ReLU, nontemporal 16-B stores, optional
//    fused GPT token pooling of the stage's last block).
// The arithmetic of every output is that of the two conv_x6 launches (same products, same K order, same epilogue
// expressions, the intermediate split the same way conv_x6 splits its halo): bit-identical (tests/test_ops_gpu.py).
#include <type_traits>

#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 bb_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 bb_h2 __attribute__((ext_vector_type(2)));
typedef float bb_f2 __attribute__((ext_vector_type(2)));
typedef float bb_f4 __attribute__((ext_vector_type(4)));
typedef float bb_f16 __attribute__((ext_vector_type(16)));
typedef int bb_i4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kOOBb = 0x80000000u;
constexpr int C = 64, CH = 32, NCH = 2;   // channels, K chunk, chunks per conv
constexpr int TH = 16, TW = 16;           // conv2 output tile
constexpr int RH = TH + 2, RW = TW + 2;   // conv1 output region 18 x 18
constexpr int H1 = TH + 4, P1 = TW + 4;   // input halo 20 x 20 (pitch P1)
constexpr int HP1 = H1 * P1;              // 400 halo pixels
constexpr int M1 = RH * RW;               // 324 conv1 rows
constexpr int MT1 = (M1 + 31) / 32;       // 11 M tiles
constexpr int P2 = RW;                    // intermediate pitch
constexpr int NT = 512, NW = 8;
constexpr int ABYTES1 = HP1 * 128;        // 51200: input halo of one chunk (hi | lo)
constexpr int IBYTES = M1 * 128;          // 41472: one intermediate chunk image
constexpr int OFF_I = ABYTES1;
constexpr int OFF_B = OFF_I + NCH * IBYTES;  // 134144
constexpr int BIMG = C * 64;              // one B image of a ring slot: 64 rows x 32 k x 2 B
constexpr int BSLOT = 2 * BIMG;
constexpr int D = 2, NSLOT = 3;           // DMA lead, ring slots
constexpr int LDS_BYTES = OFF_B + NSLOT * BSLOT;  // 158720
constexpr int BQ = C / 16;                // DMA instructions per image per step
constexpr int BPS = 2 * BQ / NW;          // per wave per step
constexpr int ALD = (HP1 * 8 + NT - 1) / NT;  // halo float4 loads per thread per chunk (7)
constexpr int NS1 = NCH * 9;              // steps per conv (18)
constexpr int TA = 1;                     // step at which chunk 1's input halo is issued
static_assert(BPS == 1 && (2 * BQ) % NW == 0, "B DMA split over the waves");
static_assert(NSLOT >= D + 1, "ring");
static_assert(M1 * 32 * 4 <= ABYTES1, "conv1 park over the input halo");
static_assert(TH * TW * C * 4 <= OFF_B, "conv2 park over the halo and the intermediate");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

__device__ inline bb_i4 bb_rsrc(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  bb_i4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r.z = (int)kOOBb;
  r.w = 0x00020000;
  return r;
}
__device__ inline void bb_dma(bb_i4 rsrc, uint32_t lds_wave, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds_wave), "v"(voff), "s"(rsrc)
               : "memory");
}
__device__ inline bb_f4 bb_vload(bb_i4 rsrc, uint32_t voff) {
  bb_f4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rsrc) : "memory");
  return v;
}
template <int N>
__device__ inline void bb_step_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
template <int N>
__device__ inline void bb_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// conv_x6.hip's split4 (fp32 -> fp16 hi + fp16 lo of the remainder, RNE twice)
__device__ inline void bb_split4(const bb_f4 v, uint2& hi, uint2& lo) {
  const bb_h2 h01 = __builtin_convertvector((bb_f2){v.x, v.y}, bb_h2);
  const bb_h2 h23 = __builtin_convertvector((bb_f2){v.z, v.w}, bb_h2);
  const bb_f2 f01 = __builtin_convertvector(h01, bb_f2);
  const bb_f2 f23 = __builtin_convertvector(h23, bb_f2);
  const bb_h2 l01 = __builtin_convertvector((bb_f2){v.x - f01.x, v.y - f01.y}, bb_h2);
  const bb_h2 l23 = __builtin_convertvector((bb_f2){v.z - f23.x, v.w - f23.y}, bb_h2);
  hi = make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
  lo = make_uint2(__builtin_bit_cast(uint32_t, l01), __builtin_bit_cast(uint32_t, l23));
}
// LDS byte offset of channel quad q of pixel px (halo column hx) in a 128-B swizzled pixel-row image (conv_x6.hip)
__device__ inline int bb_hwad(int px, int hx, int q) {
  return px * 128 + ((((q >> 1) ^ (hx >> 1)) & 7) << 4) + ((q & 1) << 3);
}

// f(integral_constant<I>) for I in [I0, N), unrolled
template <int I, int N, class F>
__device__ inline void bb_unroll(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    bb_unroll<I + 1, N>(f);
  }
}

// halo load of global step s' window (issued at the open of step TA): was it issued after B(s) (s in [TA+1, TA+D])?
constexpr bool bb_halo_in_window(int s) { return s > TA && s <= TA + D; }

}  // namespace

__global__ __launch_bounds__(NT, 1) void basicblock_kernel(ConvArgs c1, ConvArgs c2, int tiles_x, int tiles_y,
                                                           int ntiles) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, hh = lane >> 5;

  // ---- tile (XCD-aware bijective remap as conv_x6)
  int tile = blockIdx.x;
  if (ntiles >= 16) {
    const int q = ntiles / 8, r = ntiles % 8, x = tile % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
  }
  const int txi = tile % tiles_x, t2 = tile / tiles_x;
  const int tyi = t2 % tiles_y, nimg = t2 / tiles_y;
  const int oy0 = tyi * TH, ox0 = txi * TW;
  const int H = c1.H, W = c1.W;

  // ---- input halo staging (conv1's A): element e = tid + NT i -> halo pixel e >> 3, channels 4 (e & 7) ..
  const bb_i4 rin = bb_rsrc(c1.in);
  bb_f4 hr[ALD];
  auto halo_ofs = [&](int i) {
    const int e = tid + NT * i, px = e >> 3, q = e & 7;
    const int hy = px / P1, hx = px - (px / P1) * P1;
    const int iy = oy0 - 2 + hy, ix = ox0 - 2 + hx;
    const bool in = px < HP1 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    return in ? (int)(nimg * c1.in_sn + iy * c1.in_sh + ix * c1.in_sw) + 4 * q : -1;
  };
  auto halo_issue = [&](int c) {
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      const int ho = halo_ofs(i);
      hr[i] = bb_vload(rin, ho >= 0 ? (uint32_t)(ho + c * CH) * 4u : kOOBb);
    }
  };
  auto halo_tie = [&]() {
#pragma unroll
    for (int i = 0; i < ALD; ++i) asm volatile("" : "+v"(hr[i]));
  };
  auto halo_store = [&]() {
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      const int e = tid + NT * i, px = e >> 3, q = e & 7;
      if (px >= HP1) continue;
      const int w = bb_hwad(px, px % P1, q);
      uint2 hi, lo;
      bb_split4(hr[i], hi, lo);
      *reinterpret_cast<uint2*>(lds + w) = hi;
      *reinterpret_cast<uint2*>(lds + (w ^ 64)) = lo;
    }
  };

  // ---- B ring: global step s = conv * 18 + chunk * 9 + tap; wave w fills rows 16 (w % 4) .. of the hi (w < 4) or
  // lo image of the slot
  const bool bimg_lo = wave >= NW / 2;
  const int brow = (wave % BQ) * 16;
  const int bc = brow + (lane >> 2);
  const int bls = (lane & 3) ^ ((bc >> 2) & 3);
  const bb_i4 rw1 = bb_rsrc(bimg_lo ? (const void*)c1.wl : (const void*)c1.wh);
  const bb_i4 rw2 = bb_rsrc(bimg_lo ? (const void*)c2.wl : (const void*)c2.wh);
  const uint32_t boff1 = (uint32_t)(bc * (int)c1.ldh + bls * 8) * 2u;
  const uint32_t boff2 = (uint32_t)(bc * (int)c2.ldh + bls * 8) * 2u;
  auto b_issue = [&](int slot, int s) {  // s >= 36: past the end (reads zero)
    const uint32_t dst = lds_u32 + OFF_B + slot * BSLOT + (bimg_lo ? BIMG : 0) + brow * 64;
    const int sc = s % NS1, ck = sc / 9, tp = sc % 9;
    const uint32_t kb = (uint32_t)(tp * C + ck * CH) * 2u;
    if (s < NS1)
      bb_dma(rw1, __builtin_amdgcn_readfirstlane(dst), boff1 + kb);
    else
      bb_dma(rw2, __builtin_amdgcn_readfirstlane(dst), s < 2 * NS1 ? boff2 + kb : kOOBb);
  };

  // ---- fragment addresses
  const int wn = wave & 1, wq = wave >> 1;  // N tile; conv1 M tiles wq, wq + 4, wq + 8; conv2 M tiles 2 wq, 2 wq + 1
  const bool has3 = wq + 8 < MT1;
  int aad1[3][3];  // conv1: A (hi, k16 step 0) offset in the input halo of tap (0, kw), per M tile
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    int m = (wq + 4 * i) * 32 + li;
    m = m < M1 ? m : M1 - 1;  // padding rows read a real pixel; their outputs are never stored
    const int y = m / RW, x = m % RW;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) aad1[i][kw] = (y * P1 + x + kw) * 128 + (((hh ^ ((x + kw) >> 1)) & 7) << 4);
  }
  int aad2[2][3];  // conv2: in an intermediate chunk image
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = (2 * wq + i) * 32 + li;
    const int y = m / TW, x = m % TW;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) aad2[i][kw] = (y * P2 + x + kw) * 128 + (((hh ^ ((x + kw) >> 1)) & 7) << 4);
  }
  const int bcol = wn * 32 + li;
  const int bad = bcol * 64 + (((hh ^ (bcol >> 2)) & 3) << 4);

  bb_f16 acc1[3], acc2[2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[i][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[i][r] = 0.f;

  struct Frag {
    bb_h8 ah[3], al[3], bh, bl;
  };
  Frag F0, F1;
  // fragments of half-step S2 of global step S into F
  auto load_frag = [&](Frag& F, int slot, auto S, auto S2) {
    constexpr int s = decltype(S)::value, s2 = decltype(S2)::value;
    constexpr int sc = s % NS1, ck = sc / 9, tp = sc % 9, kh = tp / 3, kw = tp % 3;
    const char* bbuf = lds + OFF_B + slot * BSLOT;
    F.bh = *reinterpret_cast<const bb_h8*>(bbuf + (bad ^ (32 * s2)));
    F.bl = *reinterpret_cast<const bb_h8*>(bbuf + BIMG + (bad ^ (32 * s2)));
    if constexpr (s < NS1) {
      const char* abuf = lds + kh * P1 * 128;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (i == 2 && !has3) break;
        const int o = aad1[i][kw] ^ (32 * s2);
        F.ah[i] = *reinterpret_cast<const bb_h8*>(abuf + o);
        F.al[i] = *reinterpret_cast<const bb_h8*>(abuf + (o ^ 64));
      }
    } else {
      const char* abuf = lds + OFF_I + ck * IBYTES + kh * P2 * 128;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = aad2[i][kw] ^ (32 * s2);
        F.ah[i] = *reinterpret_cast<const bb_h8*>(abuf + o);
        F.al[i] = *reinterpret_cast<const bb_h8*>(abuf + (o ^ 64));
      }
    }
  };
  // conv_x6's product order: small terms first, the hi x hi term last (independent accumulators interleaved)
  auto mfma_frag = [&](const Frag& F, auto S) {
    constexpr int s = decltype(S)::value;
    if constexpr (s < NS1) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i < 2 || has3) acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[i], F.bh, acc1[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i < 2 || has3) acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bl, acc1[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i < 2 || has3) acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bh, acc1[i], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[i], F.bh, acc2[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bl, acc2[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[i], F.bh, acc2[i], 0, 0, 0);
    }
  };

  // Barrier opening step s: this wave's B(s) DMAs have landed (younger: B(s + 1 .. s + D - 1) and the chunk-1 halo
  // loads when they went out after B(s)), every wave's have, every wave's LDS reads of the steps before retired.
  // Then B(s + D) into the slot of step s - 1, and at s == TA chunk 1's input halo.
  int slot = 0;
  auto open_step = [&](auto S) {
    constexpr int s = decltype(S)::value;
    constexpr int N = (D - 1) * BPS + (bb_halo_in_window(s) ? ALD : 0);
    bb_step_barrier<N>();
    int ns = slot + D;
    if (ns >= NSLOT) ns -= NSLOT;
    b_issue(ns, s + D);
    if constexpr (s == TA) halo_issue(1);
  };

  // ---- conv1 epilogue: per N tile r, the waves holding it park their accumulators as fp32 [row][32] over the dead
  // input halo; then every (region pixel, quad): scale, bias, ReLU (conv_x6's expression), zero outside the map,
  // split into the intermediate chunk image r
  float* park1 = reinterpret_cast<float*>(lds);
  auto conv1_epilogue = [&]() {
    bool bad1 = false;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (wn == r) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (i == 2 && !has3) break;
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const int m = (wq + 4 * i) * 32 + (k & 3) + 8 * (k >> 2) + 4 * hh;
            if (m < M1) park1[m * 32 + li] = acc1[i][k];
          }
        }
      }
      __syncthreads();
      for (int e = tid; e < M1 * 8; e += NT) {
        const int m = e >> 3, q = e & 7;
        const int nq = r * CH + 4 * q;
        const bb_f4 acc_v = *reinterpret_cast<const bb_f4*>(park1 + m * 32 + 4 * q);
        bad1 |= !(__builtin_isfinite(acc_v.x) && __builtin_isfinite(acc_v.y) && __builtin_isfinite(acc_v.z) &&
                  __builtin_isfinite(acc_v.w));
        const bb_f4 scl = *reinterpret_cast<const bb_f4*>(c1.wsinv + nq) * c1.alpha;
        const bb_f4 bia = *reinterpret_cast<const bb_f4*>(c1.bias + nq);
        const bb_f4 rv = {0.f, 0.f, 0.f, 0.f};
        bb_f4 v = acc_v * scl + bia + rv;
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
        const int y = m / RW, x = m % RW;
        const int iy = oy0 - 1 + y, ix = ox0 - 1 + x;
        if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) v = (bb_f4){0.f, 0.f, 0.f, 0.f};
        uint2 hi, lo;
        bb_split4(v, hi, lo);
        const int w = OFF_I + r * IBYTES + bb_hwad(m, x, q);
        *reinterpret_cast<uint2*>(lds + w) = hi;
        *reinterpret_cast<uint2*>(lds + (w ^ 64)) = lo;
      }
      __syncthreads();  // the park is read before the next N tile overwrites it
    }
    if (bad1 && c1.flags) atomicOr(c1.flags, (unsigned)DD_NUM_F16_OVERFLOW);
  };

  // step s, software pipelined as conv_x6: [F1 reads of s] [MFMAs F0] [(s == 8) chunk 1's halo -> LDS after a
  // barrier] [open s + 1] [F0 reads of s + 1] [MFMAs F1]. s = 17 (conv1's last) instead finishes both halves, runs
  // the conv1 epilogue, then opens conv2's first step.
  auto step = [&](auto S) {
    constexpr int s = decltype(S)::value;
    load_frag(F1, slot, S, std::integral_constant<int, 1>());
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(F0, S);
    if constexpr (s == 8) {
      // chunk 1's halo was issued when step TA opened; younger: B issued at the opens of steps TA+1 .. 8
      bb_wait_vm<(8 - TA) * BPS>();
      halo_tie();
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave's reads of chunk 0 retired
      halo_store();
    }
    if constexpr (s == NS1 - 1) {
      __builtin_amdgcn_sched_barrier(0);
      mfma_frag(F1, S);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave's reads of the halo retired
      conv1_epilogue();
      if (++slot == NSLOT) slot = 0;
      open_step(std::integral_constant<int, s + 1>());
      load_frag(F0, slot, std::integral_constant<int, s + 1>(), std::integral_constant<int, 0>());
      return;
    }
    if (++slot == NSLOT) slot = 0;
    if constexpr (s + 1 < 2 * NS1) {
      open_step(std::integral_constant<int, s + 1>());
      load_frag(F0, slot, std::integral_constant<int, s + 1>(), std::integral_constant<int, 0>());
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(F1, S);
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: chunk 0's halo, B of steps 0 .. D-1, open step 0, its first fragments
  halo_issue(0);
#pragma unroll
  for (int u = 0; u < D; ++u) b_issue(u % NSLOT, u);
  bb_wait_vm<D * BPS>();
  halo_tie();
  halo_store();
  open_step(std::integral_constant<int, 0>());
  load_frag(F0, 0, std::integral_constant<int, 0>(), std::integral_constant<int, 0>());
  bb_unroll<0, 2 * NS1>(step);
  bb_step_barrier<0>();  // drain the trailing (past-the-end) DMAs and LDS reads

  // ---- conv2 epilogue: conv_x6's (BM 256, BN 64, 8 waves: wave tile rows 2 wq .. 2 wq + 1, columns wn)
  constexpr int BM = TH * TW, BN = C, QN = BN / 4;
  constexpr int IT = BM / (NT / QN);
  const ConvArgs& a = c2;
  const int qn = tid % QN;
  const int nq = 4 * qn;
  float* out = a.out + (int64_t)nimg * a.out_sn + nq;
  const float* res = a.res ? a.res + (int64_t)nimg * a.res_sn + nq : nullptr;
  const int osh = (int)a.out_sh, osw = (int)a.out_sw;
  const int rsh = (int)a.res_sh, rsw = (int)a.res_sw;
  bb_f4 rv[IT];
  int ooff[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int p = tid / QN + k * (NT / QN);
    const int oy = oy0 + p / TW, ox = ox0 + p % TW;
    const bool ok = oy < a.Ho && ox < a.Wo;
    ooff[k] = ok ? oy * osh + ox * osw : -1;
    rv[k] = (res && ok) ? *reinterpret_cast<const bb_f4*>(res + (oy * rsh + ox * rsw)) : (bb_f4){0.f, 0.f, 0.f, 0.f};
  }
  const bb_f4 scl = *reinterpret_cast<const bb_f4*>(a.wsinv + nq) * a.alpha;
  const bb_f4 bia = a.bias ? *reinterpret_cast<const bb_f4*>(a.bias + nq) : (bb_f4){0.f, 0.f, 0.f, 0.f};
  float* ct = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = (2 * wq + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      ct[m * BN + wn * 32 + li] = acc2[i][r];
    }
  __syncthreads();
  bool bad2 = false;
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    if (ooff[k] < 0) continue;
    const int p = tid / QN + k * (NT / QN);
    const bb_f4 acc_v = *reinterpret_cast<const bb_f4*>(ct + p * BN + 4 * qn);
    bad2 |= !(__builtin_isfinite(acc_v.x) && __builtin_isfinite(acc_v.y) && __builtin_isfinite(acc_v.z) &&
              __builtin_isfinite(acc_v.w));
    bb_f4 v = acc_v * scl + bia + rv[k];
    if (a.relu) {
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
    }
    __builtin_nontemporal_store(v, reinterpret_cast<bb_f4*>(out + ooff[k]));
    if (a.pool_out) *reinterpret_cast<bb_f4*>(ct + p * BN + 4 * qn) = v;  // the finished value, for the pool
  }
  if (a.pool_out) {
    // fused GPT token pooling (conv_x6's): every P x P window of the tile, summed dy-outer / dx-inner
    __syncthreads();
    const int P = a.pool_p, WX = TW / P, NWIN = (TH / P) * WX;
    const float inv = 1.0f / (float)(P * P);
    for (int w = tid; w < NWIN * QN; w += NT) {
      const int win = w / QN, q = w - win * QN;
      const int nc = 4 * q;
      const int wy = win / WX, wx = win - wy * WX;
      bb_f4 sum = {0.f, 0.f, 0.f, 0.f};
      for (int dy = 0; dy < P; ++dy)
        for (int dx = 0; dx < P; ++dx)
          sum += *reinterpret_cast<const bb_f4*>(ct + ((wy * P + dy) * TW + wx * P + dx) * BN + 4 * q);
      bb_f4 v = sum * inv;
      const int py = oy0 / P + wy, px = ox0 / P + wx;
      if (a.pool_add) v += *reinterpret_cast<const bb_f4*>(a.pool_add + py * a.pool_add_sh + px * a.pool_add_sw + nc);
      *reinterpret_cast<bb_f4*>(a.pool_out + nimg * a.pool_sn + py * a.pool_sh + px * a.pool_sw + nc) = v;
    }
  }
  if (bad2 && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
}

// c1 / c2: the block's two convs as launch_conv_gemm would take them (c1: x -> the intermediate, ReLU; c2: the
// intermediate -> y with residual x, ReLU, optional pool_out). Returns false (nothing launched) unless both are
// f16x3 3 x 3 / stride 1 / pad 1 convs 64 -> 64 on one contiguous NHWC map whose sides are multiples of 16.
bool launch_basicblock(const ConvArgs& c1, const ConvArgs& c2, hipStream_t st) {
  auto is33 = [](const ConvArgs& a) {
    return a.prec == 0 && a.wh && a.wl && a.wsinv && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 &&
           a.Cin == C && a.Cout == C && a.batch == 1 && !a.b_kn && !a.rowmap && a.Ho == a.H && a.Wo == a.W;
  };
  if (!is33(c1) || !is33(c2) || c1.H != c2.H || c1.W != c2.W || c1.Nimg != c2.Nimg || !c1.relu || !c2.relu || !c1.bias ||
      !c2.bias)
    return false;
  if (c1.H % TH || c1.W % TW) return false;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int64_t hw = (int64_t)c1.H * c1.W * C;
  auto dense = [&](int64_t sn, int64_t sh, int64_t sw) { return sn == hw && sh == (int64_t)c1.W * C && sw == C; };
  if (!dense(c1.in_sn, c1.in_sh, c1.in_sw) || !dense(c2.out_sn, c2.out_sh, c2.out_sw) || !al16(c1.in) || !al16(c2.out) ||
      !al16(c1.wsinv) || !al16(c2.wsinv) || !al16(c1.bias) || !al16(c2.bias))
    return false;
  if (c2.res && (!dense(c2.res_sn, c2.res_sh, c2.res_sw) || !al16(c2.res))) return false;
  if (c1.ldh % 8 || c2.ldh % 8 || c1.ldh < 9 * C || c2.ldh < 9 * C) return false;
  if ((int64_t)c1.Nimg * hw >= (int64_t(1) << 29)) return false;  // int32 element offsets
  const bool pool = c2.pool_out && c2.pool_p >= 1 && TH % c2.pool_p == 0 && TW % c2.pool_p == 0 &&
                    al16(c2.pool_out) && c2.pool_sn % 4 == 0 && c2.pool_sh % 4 == 0 && c2.pool_sw % 4 == 0 &&
                    (!c2.pool_add || (al16(c2.pool_add) && c2.pool_add_sh % 4 == 0 && c2.pool_add_sw % 4 == 0));
  ConvArgs b2 = c2;
  if (!pool) b2.pool_out = nullptr;
  set_last_conv_pooled(pool);
  const int tiles_x = c1.W / TW, tiles_y = c1.H / TH;
  const int64_t nt = (int64_t)c1.Nimg * tiles_x * tiles_y;
  if (nt >= (int64_t(1) << 31)) return false;
  hipLaunchKernelGGL(basicblock_kernel, dim3((unsigned)nt), dim3(NT), 0, st, c1, b2, tiles_x, tiles_y, (int)nt);
  DD_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace ddmi
