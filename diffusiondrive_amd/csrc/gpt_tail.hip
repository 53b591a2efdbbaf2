// Fused tail of a GPT block at C = 64 / 128 (transfuser_backbone.py:327-361 Block.forward: x = x + proj(attn(ln1 x));
// x = x + mlp(ln2 x), mlp = Linear(C, 4C) -> ReLU -> Linear(4C, C); then the next block's ln1 or ln_f), one launch
// instead of three (proj + ln2 fold, MLP-up, MLP-down + next-LN fold on conv_x3 / conv_x5):
//   Y (attention output) -> proj + bias + residual -> x (written) -> LayerNorm ln2 -> MLP-up in four C-wide hidden
//   chunks, ReLU, each chunk fed at once to its K-slice of MLP-down (accumulating in registers, chunk by chunk) ->
//   + bias + residual -> x (written) -> the next LayerNorm -> Hb (written).
// The 4C hidden activations never leave LDS (the unfused chain wrote and re-read M x 4C fp32), and the ln2 output
// is not written at all.
//
// Arithmetic: every product, its K order and every epilogue are those of the unfused kernels, so the result is
// bit-identical to them (test_gpt_tail_fusion_is_bit_identical):
//  * f16x3 on v_mfma_f32_32x32x16_f16: A split into fp16 hi / lo (RNE twice) from the fp32 value, the pre-split
//    weight images [N][ldh] (hi / lo, per-channel scale wsinv), per k16 step al*bh, ah*bl, ah*bh, k ascending (the
//    lane <-> k map of conv_x3 / conv_x5: lane half hh holds k 8 hh .. 8 hh + 7 of the step);
//  * epilogue v = acc * (wsinv * alpha) + bias (+ residual), ReLU, as epi_quads (same expression, same contraction:
//    this file takes the default flags, as conv_x3 / conv_x5);
//  * LayerNorm with layernorm_v4's / epi_quads' arithmetic: a row is C / 4 consecutive lanes holding float4
//    quads, sums (x + y) + (z + w), xor tree, no contraction.
// Tiling: BM rows x C columns per workgroup of 4 waves, BM x C = 4 tiles of 32 x 32, one per wave (C = 64: BM 64;
// C = 128: BM 32); A operands (Y, ln2 x, a hidden chunk) as split images in LDS (row pitch 2C + 16 B: 16-lane
// b128 reads of consecutive rows are conflict-free), weights as 16-B fragment loads from L2.
#include "common.h"

namespace ddmi {

namespace {

typedef _Float16 gt_h8 __attribute__((ext_vector_type(8)));
typedef float gt_f16 __attribute__((ext_vector_type(16)));
typedef float gt_f4 __attribute__((ext_vector_type(4)));

constexpr int GT_NT = 256;

// split 4 consecutive fp32 into the hi / lo images at (row, c4) (pitch P halfs)
__device__ inline void gt_st_split4(_Float16* hi, _Float16* lo, int P, int row, int c4, gt_f4 v) {
  _Float16 h[4], l[4];
  const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (_Float16)x[e];
    l[e] = (_Float16)(x[e] - (float)h[e]);
  }
  uint2 hv, lv;
  __builtin_memcpy(&hv, h, 8);
  __builtin_memcpy(&lv, l, 8);
  *reinterpret_cast<uint2*>(hi + row * P + c4) = hv;
  *reinterpret_cast<uint2*>(lo + row * P + c4) = lv;
}

// the B fragments of one 32-column x K GEMM (weights W[n][kw0 ..], columns nb*32 ..): issued together, ahead of
// the GEMM that consumes them (the caller keeps two sets in flight)
template <int K>
struct GtFrag {
  gt_h8 h[K / 16], l[K / 16];
};
template <int K>
__device__ inline void gt_load(GtFrag<K>& f, const GptTailW& w, int nb, int kw0) {
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  const int64_t wo = (int64_t)(nb * 32 + li) * w.ldh + kw0 + 8 * hh;
  const gt_h8* bh_p = reinterpret_cast<const gt_h8*>(w.wh + wo);
  const gt_h8* bl_p = reinterpret_cast<const gt_h8*>(w.wl + wo);
#pragma unroll
  for (int s = 0; s < K / 16; ++s) {
    f.h[s] = bh_p[2 * s];
    f.l[s] = bl_p[2 * s];
  }
}
// acc += A[rows rb*32 .. +31][0 .. K) (split images, pitch P) x the fragments' columns
template <int K>
__device__ inline void gt_gemm(gt_f16& acc, const _Float16* ahi, const _Float16* alo, int P, int rb,
                               const GtFrag<K>& f) {
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  const _Float16* ah_p = ahi + (rb * 32 + li) * P + 8 * hh;
  const _Float16* al_p = alo + (rb * 32 + li) * P + 8 * hh;
#pragma unroll
  for (int s = 0; s < K / 16; ++s) {
    const gt_h8 ah = *reinterpret_cast<const gt_h8*>(ah_p + 16 * s);
    const gt_h8 al = *reinterpret_cast<const gt_h8*>(al_p + 16 * s);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, f.h[s], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, f.l[s], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, f.h[s], acc, 0, 0, 0);
  }
}

// LayerNorm of the finished rows of xf (fp32, pitch XP) with layernorm_v4's arithmetic; f(row, c4, x4, ln4)
template <int C, int BM, class F>
__device__ inline void gt_ln_rows(const float* xf, int XP, const float* g, const float* b, F&& f) {
  constexpr int QN = C / 4, RPP = GT_NT / QN;
  const int tid = threadIdx.x, qn = tid % QN;
  const gt_f4 lg = *reinterpret_cast<const gt_f4*>(g + 4 * qn), lb = *reinterpret_cast<const gt_f4*>(b + 4 * qn);
#pragma unroll
  for (int k = 0; k < BM / RPP; ++k) {
    const int row = tid / QN + k * RPP;
    const gt_f4 v = *reinterpret_cast<const gt_f4*>(xf + row * XP + 4 * qn);
    gt_f4 o4;
    {
#pragma clang fp contract(off)
    float s = 0.f;
    s += (v.x + v.y) + (v.z + v.w);
#pragma unroll
    for (int o = QN / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)C;
    const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
    float q = 0.f;
    q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
#pragma unroll
    for (int o = QN / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q / (float)C + 1e-5f);
    o4.x = (v.x - mean) * rstd * lg.x + lb.x;
    o4.y = (v.y - mean) * rstd * lg.y + lb.y;
    o4.z = (v.z - mean) * rstd * lg.z + lb.z;
    o4.w = (v.w - mean) * rstd * lg.w + lb.w;
    }
    f(row, 4 * qn, v, o4);
  }
}

template <int C, int BM>
__global__ __launch_bounds__(GT_NT) void gpt_tail_kernel(GptTailArgs a) {
  constexpr int RB = BM / 32, NB = C / 32;
  static_assert(RB * NB == 4, "one 32 x 32 tile per wave");
  constexpr int P = C + 8;     // split image pitch (halfs): 2C + 16 B
  constexpr int XP = C + 4;    // fp32 row pitch (floats)
  constexpr int IMG = BM * P;  // halfs per image
  extern __shared__ __attribute__((aligned(16))) char gt_lds[];
  _Float16* a_hi = reinterpret_cast<_Float16*>(gt_lds);  // Y, then the hidden chunk
  _Float16* a_lo = a_hi + IMG;
  _Float16* h_hi = a_lo + IMG;                           // ln2(x)
  _Float16* h_lo = h_hi + IMG;
  float* xf = reinterpret_cast<float*>(h_lo + IMG);      // x after proj, then after the MLP
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, hh = lane >> 5;
  const int m0 = blockIdx.x * BM;
  const int rb = wave % RB, nb = wave / RB;
  const int col = nb * 32 + li;
  bool bad = false;
  // two fragment sets in flight: proj's and MLP-up chunk 0's before the Y staging
  GtFrag<C> fa, fb;
  gt_load(fa, a.proj, nb, 0);
  gt_load(fb, a.up, nb, 0);

  // ---- Y -> split image (rows >= M zero)
  constexpr int QC = C / 4;
  for (int e = tid; e < BM * QC; e += GT_NT) {
    const int row = e / QC, c4 = (e % QC) * 4;
    const int m = m0 + row;
    const gt_f4 v = m < a.M ? *reinterpret_cast<const gt_f4*>(a.y + (int64_t)m * C + c4) : (gt_f4){0.f, 0.f, 0.f, 0.f};
    gt_st_split4(a_hi, a_lo, P, row, c4, v);
  }
  __syncthreads();

  // ---- proj + bias + residual -> xf
  auto epi_row = [&](int r) { return rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh; };
  {
    gt_f16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    gt_gemm<C>(acc, a_hi, a_lo, P, rb, fa);
    gt_load(fa, a.down, nb, 0);  // MLP-down chunk 0
    const float scl = a.proj.sinv[col] * a.proj.alpha, bia = a.proj.bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = epi_row(r), m = m0 + row;
      if (m < a.M) bad |= !__builtin_isfinite(acc[r]);
      const float res = m < a.M ? a.x[(int64_t)m * C + col] : 0.f;
      xf[row * XP + col] = acc[r] * scl + bia + res;
    }
  }
  __syncthreads();
  // ---- x out, ln2(x) -> split image
  gt_ln_rows<C, BM>(xf, XP, a.ln2_g, a.ln2_b, [&](int row, int c4, gt_f4 v, gt_f4 o) {
    const int m = m0 + row;
    if (m < a.M) *reinterpret_cast<gt_f4*>(a.x + (int64_t)m * C + c4) = v;
    gt_st_split4(h_hi, h_lo, P, row, c4, m < a.M ? o : (gt_f4){0.f, 0.f, 0.f, 0.f});
  });
  __syncthreads();

  // ---- MLP: hidden chunk c (columns c C ..) = ReLU(ln2 x W0_c^T + b0_c) -> split image, then its K-slice of MLP-down
  gt_f16 acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
#pragma unroll 1
  for (int c = 0; c < 4; ++c) {
    gt_f16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    gt_gemm<C>(acc, h_hi, h_lo, P, rb, fb);
    if (c < 3) gt_load(fb, a.up, (c + 1) * NB + nb, 0);
    const int hc = c * C + col;
    const float scl = a.up.sinv[hc] * a.up.alpha, bia = a.up.bias[hc];
    float hv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (m0 + epi_row(r) < a.M) bad |= !__builtin_isfinite(acc[r]);
      hv[r] = fmaxf(acc[r] * scl + bia + 0.f, 0.f);
    }
    if (c) __syncthreads();  // every wave is done with the previous chunk's image
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = m0 + epi_row(r) < a.M ? hv[r] : 0.f;
      const _Float16 h = (_Float16)v;
      a_hi[epi_row(r) * P + col] = h;
      a_lo[epi_row(r) * P + col] = (_Float16)(v - (float)h);
    }
    __syncthreads();
    gt_gemm<C>(acc2, a_hi, a_lo, P, rb, fa);
    if (c < 3) gt_load(fa, a.down, nb, (c + 1) * C);
  }
  // ---- MLP-down + bias + residual -> xf (each lane its own elements), then x out and the next LayerNorm
  {
    const float scl = a.down.sinv[col] * a.down.alpha, bia = a.down.bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = epi_row(r);
      if (m0 + row < a.M) bad |= !__builtin_isfinite(acc2[r]);
      xf[row * XP + col] = acc2[r] * scl + bia + xf[row * XP + col];
    }
  }
  __syncthreads();
  gt_ln_rows<C, BM>(xf, XP, a.lnn_g, a.lnn_b, [&](int row, int c4, gt_f4 v, gt_f4 o) {
    const int m = m0 + row;
    if (m < a.M) {
      *reinterpret_cast<gt_f4*>(a.x + (int64_t)m * C + c4) = v;
      *reinterpret_cast<gt_f4*>(a.hb + (int64_t)m * C + c4) = o;
    }
  });
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
}

template <int C, int BM>
void launch_gt(const GptTailArgs& a, hipStream_t st) {
  constexpr int LDS = 4 * BM * (C + 8) * 2 + BM * (C + 4) * 4;
  static std::atomic<uint64_t> attr;
  set_max_lds_once(attr, reinterpret_cast<const void*>(gpt_tail_kernel<C, BM>), LDS);
  hipLaunchKernelGGL((gpt_tail_kernel<C, BM>), dim3((a.M + BM - 1) / BM), dim3(GT_NT), LDS, st, a);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace

bool gpt_tail_supported(int C) { return C == 64 || C == 128; }

void launch_gpt_tail(const GptTailArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const GptTailW* ws[3] = {&a.proj, &a.up, &a.down};
  for (const GptTailW* w : ws)
    if (!w->wh || !w->wl || !w->sinv || !w->bias || w->ldh % 8 || !al16(w->wh) || !al16(w->wl))
      throw std::runtime_error("gpt_tail: weight image missing or misaligned");
  if (!a.y || !a.x || !a.hb || !al16(a.y) || !al16(a.x) || !al16(a.hb) || !a.ln2_g || !a.ln2_b || !a.lnn_g || !a.lnn_b)
    throw std::runtime_error("gpt_tail: operand missing or misaligned");
  if (a.proj.ldh < a.C || a.up.ldh < a.C || a.down.ldh < 4 * a.C)
    throw std::runtime_error("gpt_tail: weight image pitch below K");
  if (a.C == 64) launch_gt<64, 64>(a, st);
  else if (a.C == 128) launch_gt<128, 32>(a, st);
  else throw std::runtime_error("gpt_tail: C must be 64 or 128");
}

}  // namespace ddmi
