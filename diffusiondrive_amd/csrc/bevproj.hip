// Fused bev_proj: cross_bev = LayerNorm(ReLU(Linear_320->256(cat(bilinear(keyval 8x8 -> 64x64), p3))))
// (transfuser_model_v2.py:123-140, the concat_cross_bev / bev_proj of V2TransfuserModel.forward) in one pass
// over the 64 x 64 BEV map.
//
// By linearity, W[:, :256] bilinear(keyval) = bilinear(W[:, :256] keyval): the keyval half is projected
// at 8 x 8 beforehand (`kvp`, one small GEMM) and interpolated here per pixel, so this kernel reads p3
// (64 channels) and writes cross_bev (256 channels) - 1.25 KB per pixel, nothing else touches HBM. The
// unfused chain (bilinear into cross_bev, the K = 64 GEMM with a residual read of it, an in-place
// LayerNorm) moves ~4.25 KB per pixel.
//
// Workgroups of 8 waves (LDS: one per CU) each step over a chunk of 8 consecutive 32-pixel tiles:
//  * XCD-aware chunk order (each XCD walks a contiguous eighth of the map: its L2 keeps only those
//    scenes' kvp maps); cross_bev written non-temporally (streamed once);
//  * a 4-stage LDS ring filled by LDS-DMA (buffer_load ... lds, no VGPRs) 3 tiles ahead: the p3 tile
//    (32 x 64 fp32 in 256-B rows whose 16-B slots are XOR-swizzled by row, so a 16-row ds_read_b128
//    group is conflict-free) and the tile's kvp footprint (it lies in one BEV row: 2 rows x 8 columns
//    x 256); zero-fill DMAs past the last tile keep every wave's vmcnt arithmetic exact;
//  * wave w owns output columns 32w..32w+31; its W_p3 fragments (4 k16 steps x hi / lo, the
//    decoder megakernel's MkLin image) stay in VGPRs for the whole kernel; f16x3 MFMA
//    (a_lo b_hi + a_hi b_lo + a_hi b_hi) on v_mfma_f32_32x32x16_f16, A split at fragment-read time;
//  * acc * scale + bias -> LDS [32][260]; then each wave takes 4 pixel rows at once (16 lanes per row):
//    + bilinear(kvp) from the staged taps, ReLU, two-pass LayerNorm (eps 1e-5; 16-lane DPP sums),
//    coalesced 256-B row-segment stores.
// Arithmetic order matches the unfused chain: ((acc * s + b) + bilinear) -> ReLU -> LayerNorm.
#include "common.h"
#include "decoder_mk.h"

namespace ddmi {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half2_v __attribute__((ext_vector_type(2)));
typedef float float2_v __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int NT = 512;
constexpr int TP = 32;   // pixels per tile
constexpr int CIN = 64;  // p3 channels
constexpr int VP = 260;  // LDS pitch of the projected tile
constexpr int KC = 8;    // kvp columns staged per tile (a 32-pixel tile spans <= 6 at the 8x upsample)

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

template <int CTRL>
__device__ inline float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over each 16-lane row (every lane gets it): quad xor 1, quad xor 2, row half-mirror, row mirror
__device__ inline float sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}

// as elementwise.hip's bl_index (PyTorch upsample_bilinear2d, align_corners = False)
__device__ inline void bl_idx(int dst, float ratio, int in_size, int& i0, int& i1, float& l0, float& l1) {
  float src = ratio * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  i0 = (int)src;
  i1 = i0 + ((i0 < in_size - 1) ? 1 : 0);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;  // buffer offsets >= num_records read as zero
constexpr int NS = 4;                   // LDS stages (tiles in flight)
constexpr int TPW = 8;                  // tiles per workgroup
constexpr int A_BYTES = TP * CIN * 4;   // p3 tile, 256-B rows, 16-B slots XOR-swizzled by row
constexpr int K_BYTES = 2 * KC * 1024;  // kvp footprint [row][column][256]
constexpr int STAGE = A_BYTES + K_BYTES;
constexpr int V_OFF = NS * STAGE;

__device__ inline i32x4 rsrc(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r.z = (int)kOOB;
  r.w = 0x00020000;
  return r;
}
// 16 B per lane from global (buffer offset voff) into LDS at m0 + 16 * lane; hidden from the compiler's
// vmcnt bookkeeping, so the kernel waits itself (wait_stage)
__device__ inline void dma16(i32x4 r, uint32_t lds_wave, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(__builtin_amdgcn_readfirstlane(lds_wave)),
               "v"(voff), "s"(r)
               : "memory");
}
template <int N>
__device__ inline void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One workgroup per CU, NS-stage LDS ring fed by LDS-DMA: per tile each wave issues 3 DMAs (4 p3 rows,
// two 1-KB kvp pieces) NS - 1 tiles ahead, so ~3 tiles of loads are in flight per CU with no VGPR cost.
__global__ __launch_bounds__(NT) void bevproj_kernel(BevProjArgs a, int ntiles) {
  __shared__ __attribute__((aligned(1024))) char lds[V_OFF + TP * VP * 4];
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds);
  float* Vs = reinterpret_cast<float*>(lds + V_OFF);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, hh = lane >> 5;
  const int HW = a.H * a.W;
  const float rh = (float)a.Hk / (float)a.H, rw = (float)a.Wk / (float)a.W;

  uint4 wh[4], wl[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const uint4* p = a.w + ((size_t)(wave * 4 + ks) * 64 + lane) * 2;
    wh[ks] = p[0];
    wl[ks] = p[1];
  }
  const int col = wave * 32 + li;
  const float sc = a.s[col], bs = a.bias[col];
  bool bad = false;

  // XCD-aware tile order: the workgroups of XCD x (blockIdx % 8, round-robin dispatch) take consecutive
  // TPW-tile chunks of the x-th contiguous eighth of the tiles, so each XCD's L2 holds the kvp maps of
  // B / 8 scenes. Chunks rather than a persistent grid: when another kernel holds some CUs (the tf
  // decoder beside this one), the hardware hands the remaining chunks to the free CUs.
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int t_beg = (int)(((int64_t)ntiles * xcd) >> 3) + slot * TPW;
  const int t_end = (int)(((int64_t)ntiles * (xcd + 1)) >> 3);
  const int n = t_beg < t_end ? min(TPW, t_end - t_beg) : 0;
  constexpr int nper = 1;

  // tile geometry: a tile lies in one BEV row y (W % 32 == 0) and reads kvp rows y0, y1 at columns
  // xs .. xs + KC - 1 (clamped)
  struct Geo {
    int b, y0, y1, xs;
    float ly0, ly1;
  };
  auto geo = [&](int t) {
    Geo g;
    const int m0 = t * TP;  // < 2^31 (launch_bevproj checks)
    g.b = m0 / HW;
    const int rem = m0 - g.b * HW;
    const int y = rem / a.W, x = rem - y * a.W;
    bl_idx(y, rh, a.Hk, g.y0, g.y1, g.ly0, g.ly1);
    int x1;
    float l0, l1;
    bl_idx(x, rw, a.Wk, g.xs, x1, l0, l1);
    return g;
  };
  // DMAs of the k-th tile of this workgroup into stage k % NS (zero-filling past the end, so every
  // wave issues the same 3 per tile and the vmcnt arithmetic below holds to the last tile)
  const int arow = 4 * wave + (lane >> 4);
  const int aslot = (lane & 15) ^ (arow & 15);  // logical 16-B slot this lane fetches
  auto issue = [&](int k) {
    const bool ok = k < n;
    const int t = ok ? t_beg + k * nper : t_beg;
    const uint32_t st = lds_u32 + (uint32_t)((k % NS) * STAGE);
    dma16(rsrc(a.p3 + (int64_t)t * TP * a.p3_ld), st + wave * 1024,
          ok ? (uint32_t)(arow * a.p3_ld * 4 + aslot * 16) : kOOB);
    const Geo g = geo(t);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = 2 * wave + u, r = j / KC, c = j % KC;
      const int xc = min(g.xs + c, a.Wk - 1);
      const float* src = a.kvp + ((int64_t)(g.b * a.Hk + (r ? g.y1 : g.y0)) * a.Wk + xc) * 256;
      dma16(rsrc(src), st + A_BYTES + j * 1024, ok ? (uint32_t)(lane * 16) : kOOB);
    }
  };

#pragma unroll
  for (int k = 0; k < NS - 1; ++k) issue(k);
  for (int k = 0; k < n; ++k) {
    // tile k's DMAs have landed: VMEM ops issued after them = the DMAs of tiles k+1 .. k+NS-2 (3 each)
    // and the row stores (4 per wave) of the tiles since - 18 in the steady state
    if (k >= 3) wait_barrier<18>();
    else if (k == 2) wait_barrier<14>();
    else if (k == 1) wait_barrier<10>();
    else wait_barrier<6>();
    static_assert(NS == 4, "the vmcnt counts above assume 4 stages");
    issue(k + NS - 1);
    const char* st = lds + (k % NS) * STAGE;
    f32x16_t acc, acc1, acc2;  // one accumulator per product: three 4-deep MFMA chains instead of one 12-deep
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc1[r] = acc2[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int s0 = 4 * ks + 2 * hh;  // logical slots s0, s0 + 1 of row li
      const float4 p = *reinterpret_cast<const float4*>(st + li * 256 + ((s0 ^ (li & 15)) << 4));
      const float4 q = *reinterpret_cast<const float4*>(st + li * 256 + (((s0 + 1) ^ (li & 15)) << 4));
      half8_t ah, al;
      split8(p, q, ah, al);
      const half8_t bh = __builtin_bit_cast(half8_t, wh[ks]);
      const half8_t bl = __builtin_bit_cast(half8_t, wl[ks]);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc2, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float x = (acc1[r] + acc2[r]) + acc[r];
      bad |= !__builtin_isfinite(x);
      Vs[row * VP + col] = x * sc + bs;
    }
    lds_barrier();
    // LayerNorm rows: wave w takes pixel rows 4w..4w+3 at once, 16 lanes per row; lane sub holds channel
    // quads sub + 16 j (j = 0..3), so each store instruction writes 4 contiguous 256-B row segments and
    // the row sums are 16-lane DPP reductions
    const int t = t_beg + k * nper;
    const Geo g = geo(t);
    const float* K0 = reinterpret_cast<const float*>(st + A_BYTES);
    const float* K1 = K0 + KC * 256;
    const int row = wave * 4 + (lane >> 4), sub = lane & 15;
    int x0, x1;
    float lx0, lx1;
    bl_idx((t * TP) % a.W + row, rw, a.Wk, x0, x1, lx0, lx1);
    const int c0 = (x0 - g.xs) * 256, c1 = (x1 - g.xs) * 256;
    const float ly0 = g.ly0, ly1 = g.ly1;
    float4 v[4];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = (sub + 16 * j) * 4;
      const float4 v00 = *reinterpret_cast<const float4*>(K0 + c0 + c), v01 = *reinterpret_cast<const float4*>(K0 + c1 + c);
      const float4 v10 = *reinterpret_cast<const float4*>(K1 + c0 + c), v11 = *reinterpret_cast<const float4*>(K1 + c1 + c);
      const float4 tv = *reinterpret_cast<const float4*>(&Vs[row * VP + c]);
      v[j].x = fmaxf(tv.x + (ly0 * (lx0 * v00.x + lx1 * v01.x) + ly1 * (lx0 * v10.x + lx1 * v11.x)), 0.f);
      v[j].y = fmaxf(tv.y + (ly0 * (lx0 * v00.y + lx1 * v01.y) + ly1 * (lx0 * v10.y + lx1 * v11.y)), 0.f);
      v[j].z = fmaxf(tv.z + (ly0 * (lx0 * v00.z + lx1 * v01.z) + ly1 * (lx0 * v10.z + lx1 * v11.z)), 0.f);
      v[j].w = fmaxf(tv.w + (ly0 * (lx0 * v00.w + lx1 * v01.w) + ly1 * (lx0 * v10.w + lx1 * v11.w)), 0.f);
      sum += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
    const float mean = sum16(sum) / 256.f;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j].x -= mean;
      v[j].y -= mean;
      v[j].z -= mean;
      v[j].w -= mean;
      q += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
    }
    const float rstd = rsqrtf(sum16(q) / 256.f + 1e-5f);
    float* orow = a.out + (int64_t)(t * TP + row) * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c4 = sub + 16 * j;
      const float4 gg = reinterpret_cast<const float4*>(a.g)[c4], bb = reinterpret_cast<const float4*>(a.beta)[c4];
      const f32x4_t o = {v[j].x * rstd * gg.x + bb.x, v[j].y * rstd * gg.y + bb.y, v[j].z * rstd * gg.z + bb.z,
                         v[j].w * rstd * gg.w + bb.w};
      __builtin_nontemporal_store(o, reinterpret_cast<f32x4_t*>(orow) + c4);
    }
  }
  wait_barrier<0>();  // drain the trailing zero-fill DMAs before the workgroup retires
  if (bad && a.flags) atomicOr(a.flags, (unsigned)DD_NUM_F16_OVERFLOW);
}

}  // namespace

// a tile must lie in one BEV row and span <= KC - 2 kvp columns (the 8x upsample: 32 pixels -> 5)
bool bevproj_supported(int C, int cin, int H, int W, int Hk, int Wk) {
  return C == 256 && cin == CIN && W % TP == 0 && Hk >= 1 && Wk >= 1 && (int64_t)TP * Wk <= (int64_t)(KC - 2) * W;
}

void launch_bevproj(const BevProjArgs& a, hipStream_t st) {
  if (!bevproj_supported(256, CIN, a.H, a.W, a.Hk, a.Wk) || a.B <= 0 || a.w == nullptr ||
      (int64_t)a.B * a.H * a.W >= (1ll << 31))
    throw std::runtime_error("launch_bevproj: needs 256 outputs, 64 p3 channels, W % 32 == 0, Wk <= 6 W / 32");
  const int ntiles = a.B * a.H * a.W / TP;
  // 8 x the chunks of the largest XCD eighth
  const int per_xcd = (ntiles + 7) / 8;
  const int grid = 8 * ((per_xcd + TPW - 1) / TPW);
  hipLaunchKernelGGL(bevproj_kernel, dim3(grid), dim3(NT), 0, st, a, ntiles);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
