// Fused ResNet stem: conv 7x7 / stride 2 / pad 3 (Cin 4: the camera's RGB or the LiDAR histogram,
// zero-padded to 4 channels; Cout 64) + folded BatchNorm + ReLU + maxpool 3x3 / stride 2 / pad 1
// (timm conv1 / bn1 / act1 / maxpool of both trunks, transfuser_backbone.py:23-33,50-55,175-192).
//
// The unfused path writes the 64-channel stem map (1.07 GB at B = 64 for the camera) and reads it
// back for the pool; here a workgroup owns a PH x PW tile of POOLED outputs, computes the
// (2PH+1) x (2PW+1) stem pixels under it (the pool windows overlap by one stem row / column, which
// is recomputed: 17 % at the 5 x 8 tile), keeps them in LDS and writes only the pooled map.
//
// Arithmetic: f16x3 as conv_x3.hip (fp32 operands split into fp16 hi + lo, products al*bh + ah*bl +
// ah*bh on v_mfma_f32_32x32x16_f16, fp32 accumulation, per-channel power-of-two weight scale undone
// in the epilogue, non-finite accumulators raise DD_NUM_F16_OVERFLOW), or (PREC 1, the bf16 mode) one
// bf16 product per MAC on v_mfma_f32_32x32x16_bf16 from the bf16 weight image.
//  * GEMM view per tile: M = stem pixels (187 -> 6 tiles of 32), N = 64 channels (2 tiles),
//    K = 7 kh x 8 kw x 4 ch = 224 (kw = 7 is a zero tap): 14 k16 steps, each = one kernel row kh and
//    four consecutive taps = 4 consecutive input pixels of that row.
//  * A: the (4PH+7) x (4PW+8) input patch is split once into fp16 hi / lo images in LDS (8 B per
//    pixel); a lane's 8-half fragment is the 2 input pixels (2sx - 3 + kw, kw = 4g + 2h, +1) of one
//    row - one 16-B ds_read_b128 per image (the patch starts at an odd input column so every such
//    pair is 16-B aligned).
//  * B: the 64 x 224 weight images are loop-invariant: each wave keeps its 32-channel half as 14
//    hi + 14 lo fragments in registers for the whole persistent loop over tiles.
//  * Epilogue: scale, bias, ReLU into an LDS [pixel][64] fp32 stem tile (stem pixels outside the map
//    are written as 0: every pool window holds at least one real pixel, all >= 0 after the ReLU, so
//    0 stands in for the pool's -inf padding), then the 3 x 3 / 2 max over float4 channel quads and
//    one 16-B store per pooled pixel quad.
//  * Persistent grid (two 4-wave workgroups per CU, 66 KB LDS each); the next tile's input patch is
//    loaded into registers while the current tile's MFMAs run.
// Bound: MFMA (f16x3 ceiling 833 TF): 49 x 4 x 64 x 2 = 25 KFLOP per stem pixel, 1.17 x recompute,
// 224 / 196 K padding; HBM traffic = the input once (+ halo re-reads) + the pooled map.
#include <type_traits>
#include <utility>

#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 sp_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 sp_h4 __attribute__((ext_vector_type(4)));
typedef float sp_f4 __attribute__((ext_vector_type(4)));
typedef float sp_f16 __attribute__((ext_vector_type(16)));
typedef __bf16 sp_b8 __attribute__((ext_vector_type(8)));
typedef __bf16 sp_b4 __attribute__((ext_vector_type(4)));

// 5 x 8 pooled outputs per tile: 11 x 17 = 187 stem pixels = 6 M tiles of 32, so the 12 (M, N) tiles split
// evenly over 4 waves (3 each). 4-wave workgroups with 66 KB of LDS run two per CU, whose phases drift apart, so
// one's stem-tile epilogue and pool overlap the other's MFMAs: 0.73 -> 0.70 ms per forward against the 8-wave
// 7 x 8 tile (255 stem pixels, one workgroup per CU; same-box bench A/B). (A 4 x 16 tile's 297 pixels made 10 M
// tiles: 3 for half the waves, 2 for the rest.)
constexpr int PH = 5, PW = 8;                      // pooled outputs per tile
constexpr int SH = 2 * PH + 1, SW = 2 * PW + 1;    // stem pixels per tile (11 x 17)
constexpr int NSP = SH * SW;                       // 187
constexpr int NMT = (NSP + 31) / 32;               // 6 M tiles
constexpr int IH = 4 * PH + 7, IW = 4 * PW + 8;    // input pixels per tile (27 x 40; the last column feeds
                                                   // only the zero kw = 7 tap, but must be finite)
// LDS pitch in pixels: even (a k-step's 2-pixel fragment is 16-B aligned at every kernel row) and = 2 (mod 16): a
// lane's fragment slot is then p + ly (mod 16) for stem pixel p = 17 ly + lx, so a 16-lane ds_read_b128 group
// crossing a stem row collides on at most one slot pair (IP = 40: shift 7 per row); -1.5 % stem time, same-box A/B.
// (The kernel's PMC bank-conflict share stays 0.38: a 16-lane group still spans two stem rows. A rotated layout that
// removes the conflicts entirely measured 6 % slower - the per-read address arithmetic costs more than the LDS
// cycles it saves)
constexpr int IP = 50;
constexpr int KS = 14;                             // k16 steps
constexpr int SOP = 64;                            // stem tile pitch (floats): a 16-lane ds_read_b128 group of
                                                   // the pool (quads of pixels 2k apart) then hits 64 distinct
                                                   // banks; the epilogue's 32-lane ds_write_b32 groups are
                                                   // consecutive channels either way
constexpr int NT = 256;                            // threads (4 waves; two workgroups per CU)
constexpr int MSTEP = NT / 128;                    // M-tile stride of a wave (waves = 2 N halves x MSTEP)
constexpr int MPW = NMT / MSTEP;                   // M tiles per wave (3)
static_assert(MPW * MSTEP == NMT, "the M tiles split evenly over the waves");
constexpr int ILD = (IH * IW + NT - 1) / NT;       // input pixels per thread per tile
constexpr int IMG_BYTES = IH * IP * 8;             // one fp16 input image
constexpr int LDS_BYTES = 2 * IMG_BYTES + NMT * 32 * SOP * 4;

// One input channel (the LiDAR histogram, SRC_C = 1; opt-in, DDMI_STEM1=1, read per dispatch): K = 7 kh x 8 kw = 56 real taps (kw = 7 and kh = 7 zero) in 4 k16 steps instead of 14 over the
// 4-channel pixels. A lane's 8 halves are 8 consecutive input columns of one row, which start at an even column 2 lx:
// the patch is held as 4 copies shifted by 0, 2, 4, 6 columns, so the read for stem column lx comes from copy lx & 3
// at the 16-B aligned column 8 (lx >> 2). Copies 2368 B apart (= 64 mod 256): the 16 lanes of a ds_read_b128 group in
// one stem row fall on 16 distinct 4-bank groups.
// The f16x3 cross products (al bh, ah bl) accumulate apart from ah bh and are added once at the end. With all three
// in one accumulator (rounds 4-5) the B = 64 golden's per-mode headings of one scene moved to 1.1e-4 against the 1e-4
// bar although the pooled stem map was within 2e-7 of the 4-channel form's and 1.6e-7 of fp64 (as accurate as it);
// apart, every per-mode pose is within 1.4e-5 of the golden, as with the 4-channel form (profiles/round6_stem1.md,
// tools/debug/stem1_diag.py, tools/micro/stem_prec.py). The reference's own per-mode response to a summation-order
// change of the LiDAR stem (the oracle with that conv in fp64) is 0.7-1.3e-5 (tests/test_conditioning.py). Still
// opt-in: the tf decoder's query_out tap then reads 2.03e-5 against its 2e-5 bar at B = 64 (4.7-9.5e-6 with the
// 4-channel form), and the LiDAR stem runs on the side stream beside the camera stem, off the critical path.
constexpr int KS1 = 4;
constexpr int IH1 = IH + 1;                        // + a zero row for the kh = 7 padding tap
constexpr int IP1 = 40;                            // halves per copy row (80 B: 16-B aligned rows)
constexpr int CB1 = 2368;                          // bytes per copy (>= IH1 * IP1 * 2)
static_assert(IH1 * IP1 * 2 <= CB1 && CB1 % 256 == 64 && IW <= IP1, "one-channel copies");
constexpr int IMG1_BYTES = 4 * CB1;                // the 4 copies of one fp16 image
constexpr int ILD1 = (IH * IW + NT - 1) / NT;      // input pixels per thread per tile
constexpr int LDS1_BYTES = 2 * IMG1_BYTES + NMT * 32 * SOP * 4;

// f(integral_constant<U>) for U in the sequence, in order (a compile-time unrolled loop)
template <class F, int... U>
__device__ inline void sp_for_each(F&& f, std::integer_sequence<int, U...>) {
  (f(std::integral_constant<int, U>()), ...);
}

__device__ inline void sp_split4(const sp_f4 v, sp_h4& hi, sp_h4& lo) {
  hi = __builtin_convertvector(v, sp_h4);
  const sp_f4 r = v - __builtin_convertvector(hi, sp_f4);
  lo = __builtin_convertvector(r, sp_h4);
}

// SRC_C = 0: the input is the NHWC image padded to 4 channels at `in`; SRC_C = 1..3: the reference's NCHW feature
// tensor with SRC_C channels, whose address the kernel reads from *src (a device word the runtime sets per call
// outside the captured graph), the missing channels zero - the same 4-channel pixels, without the transpose pass.
template <int PREC, int SRC_C, int ONE = 0>
__global__ __launch_bounds__(NT, 2) void stem_pool_kernel(const float* __restrict__ in, const float* const* src, int H,
                                                       int W, int Hs, int Ws,
                                                       int Hp, int Wp, const uint16_t* __restrict__ wh,
                                                       const uint16_t* __restrict__ wl, int ldh,
                                                       const float* __restrict__ wsinv,
                                                       const float* __restrict__ bias, float alpha,
                                                       float* __restrict__ out, unsigned* flags, int tiles_x,
                                                       int tiles_y, int ntiles) {
  static_assert(!ONE || SRC_C == 1, "the one-channel form reads a one-channel NCHW input");
  constexpr bool C1 = ONE;
  constexpr int KSN = C1 ? KS1 : KS;
  constexpr int IMGB = C1 ? IMG1_BYTES : IMG_BYTES;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* in_hi = lds;
  char* in_lo = lds + IMGB;
  float* so = reinterpret_cast<float*>(lds + 2 * IMGB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, hl = lane >> 5;
  const int nt = wave & 1, mg = wave >> 1;
  const int co = nt * 32 + li;

  // ---- loop-invariant B fragments of this wave's 32 channels (k = kh*28 + kw*4 + ci; one channel: k = kh*8 + kw)
  sp_h8 bh[KSN], bl[KSN];
  if constexpr (C1) {
#pragma unroll
    for (int s = 0; s < KS1; ++s) {
      const int kh = 2 * s + hl;
      _Float16 h8[8], l8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool live = kh < 7 && e < 7;
        const int64_t o = (int64_t)co * ldh + kh * 28 + e * 4;
        h8[e] = live ? __builtin_bit_cast(_Float16, wh[o]) : (_Float16)0.f;
        l8[e] = (live && !PREC) ? __builtin_bit_cast(_Float16, wl[o]) : (_Float16)0.f;
      }
      bh[s] = (sp_h8){h8[0], h8[1], h8[2], h8[3], h8[4], h8[5], h8[6], h8[7]};
      bl[s] = (sp_h8){l8[0], l8[1], l8[2], l8[3], l8[4], l8[5], l8[6], l8[7]};
    }
    // the zero row under every copy (the kh = 7 padding tap reads it against zero weights)
    for (int i = tid; i < 8 * IP1 / 2; i += NT) {
      const int cp = i / (IP1 / 2), w = i % (IP1 / 2);
      *reinterpret_cast<uint32_t*>(lds + cp * CB1 + IH * IP1 * 2 + 4 * w) = 0u;
    }
  } else {
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int kh = s >> 1, kw0 = 4 * (s & 1) + 2 * hl;
    const int64_t o = (int64_t)co * ldh + kh * 28 + kw0 * 4;
    const uint2 h0 = *reinterpret_cast<const uint2*>(wh + o);
    const uint2 l0 = PREC ? make_uint2(0u, 0u) : *reinterpret_cast<const uint2*>(wl + o);
    uint2 h1 = make_uint2(0u, 0u), l1 = make_uint2(0u, 0u);
    if (kw0 + 1 < 7) {
      h1 = *reinterpret_cast<const uint2*>(wh + o + 4);
      if (!PREC) l1 = *reinterpret_cast<const uint2*>(wl + o + 4);
    }
    const uint4 hv = make_uint4(h0.x, h0.y, h1.x, h1.y), lv = make_uint4(l0.x, l0.y, l1.x, l1.y);
    bh[s] = __builtin_bit_cast(sp_h8, hv);
    bl[s] = __builtin_bit_cast(sp_h8, lv);
  }
  }
  const float scl = wsinv[co] * alpha;
  const float bia = bias ? bias[co] : 0.f;
  float nf = 0.f;  // NaN once any accumulator was non-finite

  auto tile_origin = [&](int t, int& b, int& py0, int& px0) {
    const int tx = t % tiles_x, t2 = t / tiles_x;
    px0 = tx * PW;
    py0 = (t2 % tiles_y) * PH;
    b = t2 / tiles_y;
  };
  sp_f4 pre[C1 ? 1 : ILD];
  float pre1[C1 ? ILD1 : 1];
  const float* __restrict__ img = SRC_C ? *src : in;
  const int64_t plane = (int64_t)H * W;
  auto load_patch = [&](int t) {
    int b, py0, px0;
    tile_origin(t, b, py0, px0);
    const int iy0 = 4 * py0 - 5, ix0 = 4 * px0 - 5;
    if constexpr (C1) {
#pragma unroll
      for (int i = 0; i < ILD1; ++i) {
        const int e = tid + NT * i;
        const int r = e / IW, c = e - (e / IW) * IW;
        const int iy = iy0 + r, ix = ix0 + c;
        const bool ok = e < IH * IW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        pre1[i] = ok ? img[(int64_t)b * plane + (int64_t)iy * W + ix] : 0.f;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < ILD; ++i) {
      const int e = tid + NT * i;
      const int r = e / IW, c = e - (e / IW) * IW;
      const int iy = iy0 + r, ix = ix0 + c;
      const bool ok = e < IH * IW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      if constexpr (SRC_C == 0) {
        pre[i] = ok ? *reinterpret_cast<const sp_f4*>(img + (((int64_t)b * H + iy) * W + ix) * 4)
                    : (sp_f4){0.f, 0.f, 0.f, 0.f};
      } else {
        // consecutive threads take consecutive columns: each plane's loads coalesce
        const float* p = img + (int64_t)b * SRC_C * plane + (int64_t)iy * W + ix;
        sp_f4 v = {0.f, 0.f, 0.f, 0.f};
        if (ok) {
          v.x = p[0];
          if constexpr (SRC_C > 1) v.y = p[plane];
          if constexpr (SRC_C > 2) v.z = p[2 * plane];
        }
        pre[i] = v;
      }
    }
  };
  auto store_patch = [&]() {
    if constexpr (C1) {
      // column c of the patch -> column c - 2 cp of copy cp (cp = 0..3; the columns a read never reaches are left)
#pragma unroll
      for (int i = 0; i < ILD1; ++i) {
        const int e = tid + NT * i;
        if (e < IH * IW) {
          const int r = e / IW, c = e - (e / IW) * IW;
          _Float16 h, l;
          if constexpr (PREC == 1) {
            h = __builtin_bit_cast(_Float16, __builtin_bit_cast(uint16_t, (__bf16)pre1[i]));
            l = (_Float16)0.f;
          } else {
            h = (_Float16)pre1[i];
            l = (_Float16)(pre1[i] - (float)h);
          }
#pragma unroll
          for (int cp = 0; cp < 4; ++cp) {
            const int cc = c - 2 * cp;
            if (cc >= 0) {
              const int o = cp * CB1 + (r * IP1 + cc) * 2;
              *reinterpret_cast<_Float16*>(in_hi + o) = h;
              if constexpr (PREC == 0) *reinterpret_cast<_Float16*>(in_lo + o) = l;
            }
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < ILD; ++i) {
      const int e = tid + NT * i;
      if (e < IH * IW) {
        const int r = e / IW, c = e - (e / IW) * IW;
        if constexpr (PREC == 1) {
          *reinterpret_cast<sp_b4*>(in_hi + (r * IP + c) * 8) = __builtin_convertvector(pre[i], sp_b4);
        } else {
          sp_h4 hi, lo;
          sp_split4(pre[i], hi, lo);
          *reinterpret_cast<sp_h4*>(in_hi + (r * IP + c) * 8) = hi;
          *reinterpret_cast<sp_h4*>(in_lo + (r * IP + c) * 8) = lo;
        }
      }
    }
  };

  // XCD-aware tile walk: the workgroups of one XCD (blockIdx % 8) take one contiguous eighth of the tiles, 64 (grid / 8)
  // consecutive tiles at a time, so the input halos that neighbouring tiles share are read into the same L2. (A grid
  // that is not a multiple of 8 walks the tiles with the grid stride.)
  const int G = gridDim.x;
  const bool xcd = G % 8 == 0;
  const int xq = (ntiles + 7) / 8, xb = xcd ? (int)(blockIdx.x % 8) * xq : 0, xe = xcd ? min(xb + xq, ntiles) : ntiles;
  const int xs = xcd ? G / 8 : G;
  int t = xb + (xcd ? (int)blockIdx.x / 8 : (int)blockIdx.x);
  if (t < xe) load_patch(t);
  for (; t < xe; t += xs) {
    store_patch();
    __syncthreads();

    int b, py0, px0;
    tile_origin(t, b, py0, px0);
    const int sy0 = 2 * py0 - 1, sx0 = 2 * px0 - 1;
    // ---- stem GEMM: wave (nt, mg) takes M tiles mg, mg + 2, mg + 4, one after the other (one accumulator), each
    // tile's 14 k16 steps then its epilogue into the LDS stem tile. The 42 (tile, step) units run as one unrolled
    // sequence whose fragment reads are issued two units ahead (a ring of three fragment sets), across tile
    // boundaries too, so every read lands under earlier MFMAs (or a tile's epilogue) instead of being waited for
    // right before its own MFMAs. Per accumulator: the steps in order, the three products in the same order.
    int abase[MPW];
#pragma unroll
    for (int i = 0; i < MPW; ++i) {
      const int p = min((mg + MSTEP * i) * 32 + li, NSP - 1);
      const int ly = p / SW, lx = p - (p / SW) * SW;
      // 4 channels: input pixel of (kh 0, kw 2h); one channel: copy lx & 3, row 2 ly + hl (+ 2 s), 16-B aligned column
      // 8 (lx >> 2)
      abase[i] = C1 ? (lx & 3) * CB1 + ((2 * ly + hl) * IP1 + 8 * (lx >> 2)) * 2
                    : ((2 * ly) * IP + 2 * lx + 2 * hl) * 8;
    }
    constexpr int NU = MPW * KSN, PD = 2;  // units, prefetch distance
    sp_h8 fh[PD + 1], fl[PD + 1];
    auto issue = [&](auto U) {
      constexpr int u = decltype(U)::value;
      if constexpr (u < NU) {
        constexpr int i = u / KSN, st = u % KSN;
        constexpr int so_ = C1 ? st * 2 * IP1 * 2 : ((st >> 1) * IP + 4 * (st & 1)) * 8;
        fh[u % (PD + 1)] = *reinterpret_cast<const sp_h8*>(in_hi + abase[i] + so_);
        if constexpr (PREC == 0) fl[u % (PD + 1)] = *reinterpret_cast<const sp_h8*>(in_lo + abase[i] + so_);
      }
    };
    sp_f16 acc, acc2;
    auto unit = [&](auto U) {
      constexpr int u = decltype(U)::value;
      constexpr int i = u / KSN, st = u % KSN, f = u % (PD + 1);
      if constexpr (st == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
      }
      issue(std::integral_constant<int, u + PD>());
      __builtin_amdgcn_sched_barrier(0);  // the reads of unit u + PD go out ahead of this unit's MFMAs
      if constexpr (PREC == 1) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(sp_b8, fh[f]), __builtin_bit_cast(sp_b8, bh[st]),
                                                      acc, 0, 0, 0);
      } else if constexpr (C1) {  // the cross products in an accumulator of their own (header: one channel)
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fl[f], bh[st], acc2, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[f], bl[st], acc2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[f], bh[st], acc, 0, 0, 0);
      } else {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fl[f], bh[st], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[f], bl[st], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[f], bh[st], acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (st == KSN - 1) {
        if constexpr (C1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] += acc2[r];
        }
        // epilogue of tile i into the LDS stem tile. C/D layout: column (channel) li, row (pixel) (r & 3) + 8 (r >> 2) +
        // 4 hl. A non-finite accumulator turns the running fma(acc, 0, nf) into NaN (one fma per value instead of a class
        // test; the padding rows of the last M tile are clamped to pixel NSP - 1, so finite). Rows NSP..191 of the last
        // M tile are written and never read.
        float* sob = so + ((mg + MSTEP * i) * 32 + 4 * hl) * SOP + co;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          nf = __builtin_fmaf(acc[r], 0.f, nf);
          sob[((r & 3) + 8 * (r >> 2)) * SOP] = fmaxf(acc[r] * scl + bia, 0.f);
        }
      }
    };
    issue(std::integral_constant<int, 0>());
    issue(std::integral_constant<int, 1>());
    sp_for_each(unit, std::make_integer_sequence<int, NU>());
    // the next tile's input patch: lands under this tile's pool (issued after the MFMAs, so its registers are not live
    // beside the fragments)
    if (t + xs < xe) load_patch(t + xs);
    __syncthreads();
    // tiles at the map's edge: the stem pixels outside the map become 0 (every pool window holds at least one real
    // pixel, all >= 0 after the ReLU, so 0 stands in for the pool's -inf padding)
    if (sy0 < 0 || sx0 < 0 || sy0 + SH > Hs || sx0 + SW > Ws) {
      for (int i = tid; i < NSP * 16; i += NT) {
        const int pr = i >> 4, q = i & 15;
        const int sy = sy0 + pr / SW, sx = sx0 + pr % SW;
        if ((unsigned)sy >= (unsigned)Hs || (unsigned)sx >= (unsigned)Ws)
          *reinterpret_cast<sp_f4*>(so + pr * SOP + 4 * q) = (sp_f4){0.f, 0.f, 0.f, 0.f};
      }
      __syncthreads();
    }
    // ---- 3 x 3 / 2 max pool over the stem tile: (pooled pixel, channel quad) items
    for (int i = tid; i < PH * PW * 16; i += NT) {
      const int q = i & 15, pp = i >> 4;
      const int py = pp / PW, px = pp - (pp / PW) * PW;
      const int gy = py0 + py, gx = px0 + px;
      sp_f4 mx = *reinterpret_cast<const sp_f4*>(so + ((2 * py) * SW + 2 * px) * SOP + 4 * q);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const sp_f4 v = *reinterpret_cast<const sp_f4*>(so + ((2 * py + dy) * SW + 2 * px + dx) * SOP + 4 * q);
          mx.x = fmaxf(mx.x, v.x);
          mx.y = fmaxf(mx.y, v.y);
          mx.z = fmaxf(mx.z, v.z);
          mx.w = fmaxf(mx.w, v.w);
        }
      if (gy < Hp && gx < Wp) *reinterpret_cast<sp_f4*>(out + (((int64_t)b * Hp + gy) * Wp + gx) * 64 + 4 * q) = mx;
    }
    __syncthreads();  // the next tile overwrites the patch and the stem tile
  }
  if (!__builtin_isfinite(nf) && flags) atomicOr(flags, (unsigned)DD_NUM_F16_OVERFLOW);
}

}  // namespace

// Returns false when the conv is not a 7x7 / s2 / p3, Cin 4, Cout 64 f16x3 / bf16 stem on a contiguous
// NHWC4 input (src == nullptr) or on the NCHW tensor of src_c channels whose address is the device word *src
// (the caller then runs the conv and the pool separately).
bool launch_stem_pool(const ConvArgs& a, float* pool_out, int Hp, int Wp, hipStream_t st, const float* const* src,
                      int src_c) {
  if (!a.wh || (a.prec == 0 && !a.wl) || (a.prec != 0 && a.prec != 1) || !a.wsinv) return false;
  if (a.KH != 7 || a.KW != 7 || a.stride != 2 || a.pad != 3 || a.Cin != 4 || a.Cout != 64 || a.batch != 1 || a.res ||
      !a.relu)
    return false;
  if (src) {
    if (src_c < 1 || src_c > 3 || (int64_t)a.Nimg * src_c * a.H * a.W >= (int64_t(1) << 31)) return false;
  } else if (a.in_sw != 4 || a.in_sh != (int64_t)a.W * 4 || a.in_sn != (int64_t)a.H * a.W * 4) {
    return false;
  }
  if (a.ldh < 196 || a.ldh % 4) return false;
  const int Hs = a.Ho, Ws = a.Wo;
  if (Hp != (Hs + 2 - 3) / 2 + 1 || Wp != (Ws + 2 - 3) / 2 + 1) return false;
  if ((!src && (reinterpret_cast<uintptr_t>(a.in) & 15)) || (reinterpret_cast<uintptr_t>(pool_out) & 15) ||
      (reinterpret_cast<uintptr_t>(a.wh) & 7) || (a.prec == 0 && (reinterpret_cast<uintptr_t>(a.wl) & 7)))
    return false;
  const int tiles_x = (Wp + PW - 1) / PW, tiles_y = (Hp + PH - 1) / PH;
  const int64_t nt64 = (int64_t)a.Nimg * tiles_x * tiles_y;
  if (nt64 >= (int64_t(1) << 31)) return false;
  const int ntiles = (int)nt64;
  int dev = 0, cus = 256;
  DD_HIP_CHECK(hipGetDevice(&dev));
  DD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int per_cu = NT == 512 ? 1 : 2;
  const int grid = ntiles < per_cu * cus ? ntiles : per_cu * cus;
  const int c = src ? src_c : 0;
  const char* oe = getenv("DDMI_STEM1");
  const bool one = c == 1 && oe && atoi(oe) != 0;
  static std::atomic<uint64_t> attr[2][5];
  auto go = [&](auto kern, int c) {
    const int lds = (c == 1 && one) ? LDS1_BYTES : LDS_BYTES;
    set_max_lds_once(attr[a.prec][c == 1 && one ? 4 : c], reinterpret_cast<const void*>(kern), lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, st, a.in, src, a.H, a.W, Hs, Ws, Hp, Wp, a.wh, a.wl,
                       (int)a.ldh, a.wsinv, a.bias, a.alpha, pool_out, a.flags, tiles_x, tiles_y, ntiles);
  };
  auto pick = [&](auto PR) {
    constexpr int P = decltype(PR)::value;
    switch (c) {
      case 1:
        if (one) go(stem_pool_kernel<P, 1, 1>, 1); else go(stem_pool_kernel<P, 1, 0>, 1);
        break;
      case 2: go(stem_pool_kernel<P, 2>, 2); break;
      case 3: go(stem_pool_kernel<P, 3>, 3); break;
      default: go(stem_pool_kernel<P, 0>, 0); break;
    }
  };
  if (a.prec == 1)
    pick(std::integral_constant<int, 1>());
  else
    pick(std::integral_constant<int, 0>());
  set_last_conv_config(a.prec == 1 ? "stem_pool<bf16>" : "stem_pool<f16x3>");
  DD_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace ddmi
