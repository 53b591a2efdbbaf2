// Implicit-GEMM convolution / GEMM on CDNA4 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One kernel family carries every contraction of the DiffusionDrive hot path: the ResNet-34
// trunk convs (timm BasicBlock 3x3 / 1x1 downsample / 7x7 stem, transfuser_backbone.py:24-55),
// the GPT projections and attention matmuls (:365-431), the FPN convs (:153-159), value_proj
// (blocks.py:68-76), bev_proj and every nn.Linear of the decoders (transfuser_model_v2.py).
//
// Numerics: f32-input MFMA is an exact k-ordered f32 fma chain (no xf32 on gfx950), so results
// differ from the reference's CPU fp32 only by summation order.
//
// Tiling (MI355X-first):
//  * 256-thread workgroups = 4 wave64 as 2x2; each wave owns WTM x WTN 32x32 MFMA tiles.
//  * K staged in BK = 32 chunks; HBM/L2 -> registers (16-B buffer loads of NHWC channel slices)
//    -> LDS, double-buffered: chunk k+1's loads are in flight while chunk k's MFMAs run.
//  * Operand loads are raw buffer loads with 32-bit offsets. Conv zero padding and ragged
//    M/N/K edges use an out-of-range offset (>= num_records) so the hardware returns zeros:
//    no branch, no select on data, every load unconditional (a predicated `ok ? load : 0` makes
//    hipcc branch per load and wait vmcnt(0) after each, serialising the prefetch).
//  * LDS rows padded to 36 floats (144 B): the 16-lane groups of ds_read_b128 hit 16 distinct
//    16-B slots (row stride 9 slots, coprime with 16) -> conflict-free fragment reads.
//  * k-permutation: within each 8-k group, MFMA step s consumes k = {s, 4+s} (lane halves), so one
//    ds_read_b128 per operand feeds 4 consecutive MFMAs (A[i][4h..4h+3], B[j][4h..4h+3]).
//  * XCD-aware tile order: blocks b, b+8, b+16, ... share one XCD's L2 under round-robin dispatch,
//    so they get consecutive tiles (same A rows / neighbouring conv halos) — speed only.
//  * Epilogue fused: alpha, bias (BN folded at load time), residual, ReLU, strided NHWC store
//    (channel offsets / strides let convs write straight into concat buffers and token slabs).
#include "common.h"

namespace ddmi {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDSK = BK + 4;
constexpr uint32_t kOOB = 0x80000000u;  // byte offset >= num_records -> buffer load returns 0

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const float* base) {
  // raw buffer, stride 0, num_records = 2 GiB (every in-range offset of a launch is < 2^31 B)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)kOOB, 0x00020000);
}

__device__ inline float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0);
  return *reinterpret_cast<float4*>(&v);
}

template <int WTM, int WTN, int BKN>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvArgs a, int M, int K, int n_tiles_m,
                                                           int n_tiles_n) {
  constexpr int BM = 2 * WTM * 32;
  constexpr int BN = 2 * WTN * 32;
  constexpr int A_LD = BM * BK / 4 / 256;
  constexpr int B_LD = BN * BK / 4 / 256;
  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * LDSK];

  const int tid = threadIdx.x;
  // XCD-aware bijective remap of the linear block id (MI355X: 8 XCDs, round-robin dispatch).
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

  // batched pointer offsets
  const int z = blockIdx.z;
  const int z1 = z / a.zdiv, z2 = z - z1 * a.zdiv;
  const float* in = a.in + z1 * a.in_z1 + z2 * a.in_z2;
  const float* wgt = a.wgt + z1 * a.w_z1 + z2 * a.w_z2;
  float* out = a.out + z1 * a.out_z1 + z2 * a.out_z2;
  const float* res = a.res ? a.res + z1 * a.res_z1 + z2 * a.res_z2 : nullptr;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(in);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(wgt);

  const int in_sh = (int)a.in_sh, in_sw = (int)a.in_sw;
  const int ldb = (int)a.ldb;

  // ---- per-thread A-row decode (fixed across K chunks); element offsets in int32
  const int k4 = (tid & 7) * 4;
  int arow[A_LD], aih0[A_LD], aiw0[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    const bool v = m < M;
    const int mm = v ? m : 0;
    const int ow = mm % a.Wo;
    const int t2 = mm / a.Wo;
    const int oh = t2 % a.Ho;
    const int n = t2 / a.Ho;
    arow[i] = n * (int)a.in_sn;
    // invalid rows get an origin far outside the image so every tap fails the bounds test
    aih0[i] = v ? oh * a.stride - a.pad : -(1 << 28);
    aiw0[i] = ow * a.stride - a.pad;
  }

  float4 ra[A_LD], rb[B_LD];

#define DD_LOAD_CHUNK(K0)                                                                            \
  {                                                                                                  \
    const int kk = (K0) + k4;                                                                        \
    const bool kv = kk < K;                                                                          \
    const int tap = kk / a.Cin;                                                                      \
    const int ci = kk - tap * a.Cin;                                                                 \
    const int kh = tap / a.KW;                                                                       \
    const int kw = tap - kh * a.KW;                                                                  \
    _Pragma("unroll") for (int i = 0; i < A_LD; ++i) {                                               \
      const int ih = aih0[i] + kh, iw = aiw0[i] + kw;                                                \
      const bool ok = kv && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;            \
      const uint32_t off = ok ? (uint32_t)(arow[i] + ih * in_sh + iw * in_sw + ci) * 4u : kOOB;      \
      ra[i] = bload4(rin, off);                                                                      \
    }                                                                                                \
    if constexpr (!BKN) {                                                                            \
      _Pragma("unroll") for (int i = 0; i < B_LD; ++i) {                                             \
        const int n = n0 + (tid >> 3) + 32 * i;                                                      \
        const bool ok = kv && n < a.Cout;                                                            \
        rb[i] = bload4(rw, ok ? (uint32_t)(n * ldb + kk) * 4u : kOOB);                               \
      }                                                                                              \
    } else {                                                                                         \
      constexpr int NF4 = BN / 4;                                                                    \
      constexpr int RPP = 256 / NF4;                                                                 \
      _Pragma("unroll") for (int i = 0; i < B_LD; ++i) {                                             \
        const int kr = (K0) + tid / NF4 + RPP * i;                                                   \
        const int n = n0 + (tid % NF4) * 4;                                                          \
        const bool ok = kr < K && n < a.Cout;                                                        \
        rb[i] = bload4(rw, ok ? (uint32_t)(kr * ldb + n) * 4u : kOOB);                               \
      }                                                                                              \
    }                                                                                                \
  }

#define DD_STORE_CHUNK(BUF)                                                                          \
  {                                                                                                  \
    float* as = lds + (BUF) * BM * LDSK;                                                             \
    float* bs = lds + 2 * BM * LDSK + (BUF) * BN * LDSK;                                             \
    _Pragma("unroll") for (int i = 0; i < A_LD; ++i)                                                 \
      *reinterpret_cast<float4*>(as + ((tid >> 3) + 32 * i) * LDSK + k4) = ra[i];                     \
    if constexpr (!BKN) {                                                                            \
      _Pragma("unroll") for (int i = 0; i < B_LD; ++i)                                               \
        *reinterpret_cast<float4*>(bs + ((tid >> 3) + 32 * i) * LDSK + k4) = rb[i];                   \
    } else {                                                                                         \
      constexpr int NF4 = BN / 4;                                                                    \
      constexpr int RPP = 256 / NF4;                                                                 \
      _Pragma("unroll") for (int i = 0; i < B_LD; ++i) {                                             \
        const int kr = tid / NF4 + RPP * i;                                                          \
        const int n = (tid % NF4) * 4;                                                               \
        bs[(n + 0) * LDSK + kr] = rb[i].x;                                                           \
        bs[(n + 1) * LDSK + kr] = rb[i].y;                                                           \
        bs[(n + 2) * LDSK + kr] = rb[i].z;                                                           \
        bs[(n + 3) * LDSK + kr] = rb[i].w;                                                           \
      }                                                                                              \
    }                                                                                                \
  }

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, hh = lane >> 5;

  f32x16 acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  DD_LOAD_CHUNK(0);
  DD_STORE_CHUNK(0);
  __syncthreads();

  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) DD_LOAD_CHUNK((kc + 1) * BK);
    const float* as = lds + cur * BM * LDSK;
    const float* bs = lds + 2 * BM * LDSK + cur * BN * LDSK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      float4 av[WTM], bv[WTN];
#pragma unroll
      for (int i = 0; i < WTM; ++i)
        av[i] = *reinterpret_cast<const float4*>(as + ((wm * WTM + i) * 32 + li) * LDSK + g * 8 + 4 * hh);
#pragma unroll
      for (int j = 0; j < WTN; ++j)
        bv[j] = *reinterpret_cast<const float4*>(bs + ((wn * WTN + j) * 32 + li) * LDSK + g * 8 + 4 * hh);
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].z, bv[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].w, bv[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (more) DD_STORE_CHUNK(cur ^ 1);
    __syncthreads();
  }
#undef DD_LOAD_CHUNK
#undef DD_STORE_CHUNK

  // ---- fused epilogue. C/D map of 32x32 f32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5).
  float bias_v[WTN];
  int ncol[WTN];
#pragma unroll
  for (int j = 0; j < WTN; ++j) {
    ncol[j] = n0 + (wn * WTN + j) * 32 + li;
    bias_v[j] = (a.bias && ncol[j] < a.Cout) ? a.bias[ncol[j]] : 0.f;
  }
  const int osh = (int)a.out_sh, osw = (int)a.out_sw;
  const int rsh = (int)a.res_sh, rsw = (int)a.res_sw;
#pragma unroll
  for (int i = 0; i < WTM; ++i) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mbase = m0 + (wm * WTM + i) * 32 + 8 * q + 4 * hh;
      int ow = mbase % a.Wo;
      int t2 = mbase / a.Wo;
      int oh = t2 % a.Ho;
      int n = t2 / a.Ho;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = mbase + e;
        if (m < M) {
          float* orow = out + (int64_t)n * a.out_sn + (oh * osh + ow * osw);
          const float* rrow = res ? res + (int64_t)n * a.res_sn + (oh * rsh + ow * rsw) : nullptr;
#pragma unroll
          for (int j = 0; j < WTN; ++j) {
            if (ncol[j] < a.Cout) {
              float v = acc[i][j][q * 4 + e] * a.alpha + bias_v[j];
              if (rrow) v += rrow[ncol[j]];
              if (a.relu) v = fmaxf(v, 0.f);
              orow[ncol[j]] = v;
            }
          }
        }
        if (++ow == a.Wo) {
          ow = 0;
          if (++oh == a.Ho) {
            oh = 0;
            ++n;
          }
        }
      }
    }
  }
}

template <int WTM, int WTN>
static void launch_cfg(const ConvArgs& a, int M, int K, hipStream_t st) {
  constexpr int BM = 2 * WTM * 32, BN = 2 * WTN * 32;
  const int ntm = (M + BM - 1) / BM;
  const int ntn = (a.Cout + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, a.batch);
  if (a.b_kn)
    hipLaunchKernelGGL((conv_gemm_kernel<WTM, WTN, 1>), grid, dim3(256), 0, st, a, M, K, ntm, ntn);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<WTM, WTN, 0>), grid, dim3(256), 0, st, a, M, K, ntm, ntn);
  DD_HIP_CHECK(hipGetLastError());
}

void set_last_conv_kernel(const char* k);  // conv_x3.hip

void launch_conv_gemm(const ConvArgs& a, hipStream_t st) {
  set_last_conv_pooled(false);
  set_last_conv_ln(false);
  if (a.rowmap && !a.wh) throw std::runtime_error("conv_gemm: gathered rows need the f16x3 kernel (conv_x3)");
  if (a.wh) {
    launch_conv_x3(a, st);
    return;
  }
  set_last_conv_kernel("conv_gemm");
  set_last_conv_config("conv_gemm");
  if (a.Cin % 4 != 0) throw std::runtime_error("conv_gemm: Cin must be a multiple of 4");
  if ((a.in_sw % 4) || (a.in_sh % 4) || (a.in_sn % 4) || (reinterpret_cast<uintptr_t>(a.in) % 16))
    throw std::runtime_error("conv_gemm: input strides / base must be 16-byte aligned");
  if ((a.ldb % 4) || (reinterpret_cast<uintptr_t>(a.wgt) % 16))
    throw std::runtime_error("conv_gemm: weight ldb / base must be 16-byte aligned");
  if (a.b_kn && (a.Cout % 4)) throw std::runtime_error("conv_gemm: KN weights need Cout % 4 == 0");
  if (a.batch > 1 && ((a.in_z1 % 4) || (a.in_z2 % 4) || (a.w_z1 % 4) || (a.w_z2 % 4)))
    throw std::runtime_error("conv_gemm: batch strides must keep 16-byte alignment");
  const int64_t M64 = (int64_t)a.Nimg * a.Ho * a.Wo;
  if (M64 >= (int64_t(1) << 31)) throw std::runtime_error("conv_gemm: M too large");
  const int M = (int)M64;
  const int K = a.KH * a.KW * a.Cin;
  if (M == 0 || a.Cout == 0) return;
  // 32-bit buffer offsets: the furthest element a launch touches must stay below 2^31 bytes.
  const int64_t in_extent = (int64_t)(a.Nimg - 1) * a.in_sn + (int64_t)(a.H - 1) * a.in_sh +
                            (int64_t)(a.W - 1) * a.in_sw + a.Cin;
  const int64_t w_extent = a.b_kn ? (int64_t)K * a.ldb : (int64_t)a.Cout * a.ldb;
  if (in_extent * 4 >= (int64_t)kOOB || w_extent * 4 >= (int64_t)kOOB)
    throw std::runtime_error("conv_gemm: operand extent >= 2 GiB (split the batch)");
  if ((int64_t)a.Ho * a.out_sh >= (int64_t(1) << 31) || (int64_t)a.Ho * a.res_sh >= (int64_t(1) << 31))
    throw std::runtime_error("conv_gemm: per-image output extent too large");
  const int64_t tiles_big = ((M + 127) / 128) * (int64_t)((a.Cout + 127) / 128) * a.batch;
  if (a.Cout <= 64) {
    if (((M + 127) / 128) * (int64_t)a.batch >= 512)
      launch_cfg<2, 1>(a, M, K, st);
    else
      launch_cfg<1, 1>(a, M, K, st);
  } else if (tiles_big >= 512) {
    launch_cfg<2, 2>(a, M, K, st);
  } else {
    launch_cfg<1, 1>(a, M, K, st);
  }
}

}  // namespace ddmi
