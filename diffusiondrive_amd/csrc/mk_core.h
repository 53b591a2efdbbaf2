// Shared device core of the megakernels (decoder_mk.hip, tfdec_mk.hip): one 512-thread workgroup holds a
// 32-row activation tile in LDS and runs 256-wide f16x3 Linears on v_mfma_f32_32x32x16_f16 with the weights
// streamed from L2 in MFMA-fragment order (decoder_mk.h MkLin) through a per-wave register ring.
#pragma once
#include "decoder_mk.h"

namespace ddmi {
namespace {

typedef _Float16 mk_h8 __attribute__((ext_vector_type(8)));
typedef float mk_f16 __attribute__((ext_vector_type(16)));
typedef unsigned mk_u4 __attribute__((ext_vector_type(4)));
typedef float mk_f4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;
constexpr int FP = 260;   // fp32 row pitch (floats)
constexpr int HP = 264;   // split row pitch (halfs), K = 256: 528 B, 16 mod 256 -> conflict-free b128 reads
constexpr int HP2 = 520;  // split row pitch (halfs), K = 512: 1040 B

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The B (weight) fragments stream through a ring of PF fragment pairs per wave (PF x 32 B per lane). A GEMM
// starts with its first PF steps already in the ring and, as its last PF steps free their slots, loads the
// first PF steps of the NEXT GEMM (`nx`, tile nnt, k-step nwks), so those loads fly under this GEMM's tail,
// its epilogue, the barrier and whatever LDS / VALU phase separates the two GEMMs.
constexpr int PF = 8;
struct Ring {
  mk_u4 h[PF], l[PF];
};

// Weights and parameters are read through global-address-space pointers: a pointer the compiler cannot
// prove global (one loaded from memory, e.g. tfdec_mk's per-layer table) becomes a FLAT load, which also
// counts in lgkmcnt - every LDS wait (lgkmcnt(0)) would then drain the whole weight ring.
template <class T>
__device__ inline const __attribute__((address_space(1))) T* gptr(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
typedef const __attribute__((address_space(1))) mk_u4* gu4p;

__device__ inline gu4p mk_wbase(const MkLin& L, int nt, int wks) {
  return (gu4p)L.w + ((size_t)(nt * L.nks + wks) * 64 + (threadIdx.x & 63)) * 2;
}

__device__ inline void ring_fill(Ring& R, const MkLin& L, int nt, int wks) {
  gu4p wb = mk_wbase(L, nt, wks);
#pragma unroll
  for (int s = 0; s < PF; ++s) {
    R.h[s] = wb[s * 128];
    R.l[s] = wb[s * 128 + 1];
  }
}

// acc += A[32][aks*16 .. (aks+NKS)*16) (split LDS images, row pitch hp halfs) x W[:, wks*16 ..]^T for the 32
// output columns of tile nt, 3 f16 MFMAs per k16 step (small terms first, as conv_x3); R holds this GEMM's
// first PF steps on entry and the next GEMM's (nx) on exit (nx.w == nullptr: nothing next)
template <int NKS>
__device__ inline void mk_gemm(const char* ahi, const char* alo, int hp, const MkLin& L, int nt, int wks, mk_f16& acc,
                               int aks, Ring& R, const MkLin& nx, int nnt, int nwks) {
  static_assert(NKS % PF == 0 && NKS >= PF, "ring");
  __builtin_amdgcn_sched_barrier(0);
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  gu4p wb = mk_wbase(L, nt, wks);
  // nothing next: re-read this GEMM's first fragments (cache hits) rather than branch per step - a
  // conditional load makes the waitcnt pass fall back to vmcnt(0) for every later ring slot
  gu4p nb = nx.w ? mk_wbase(nx, nnt, nwks) : wb;
  const int aoff = li * hp * 2 + hh * 16 + aks * 32;
  // A fragments double-buffered one step ahead, and the issue order pinned per step (the scheduler
  // otherwise waits out each LDS read right before its MFMA): the next step's 2 LDS reads, this step's
  // 3 MFMAs, the ring refill's 2 global loads
  mk_h8 ah[2], al[2];
  ah[0] = *reinterpret_cast<const mk_h8*>(ahi + aoff);
  al[0] = *reinterpret_cast<const mk_h8*>(alo + aoff);
  __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // step 0's reads first
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int c = s & 1;
    if (s + 1 < NKS) {
      ah[c ^ 1] = *reinterpret_cast<const mk_h8*>(ahi + aoff + (s + 1) * 32);
      al[c ^ 1] = *reinterpret_cast<const mk_h8*>(alo + aoff + (s + 1) * 32);
    }
    const mk_h8 wh = __builtin_bit_cast(mk_h8, R.h[s % PF]), wl = __builtin_bit_cast(mk_h8, R.l[s % PF]);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[c], wh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], wl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], wh, acc, 0, 0, 0);
    if (s + PF < NKS) {
      R.h[s % PF] = wb[(s + PF) * 128];
      R.l[s % PF] = wb[(s + PF) * 128 + 1];
    } else {
      const int t = s + PF - NKS;
      R.h[s % PF] = nb[t * 128];
      R.l[s % PF] = nb[t * 128 + 1];
    }
    if (s + 1 < NKS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);                   // MFMA
    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);                   // VMEM read
  }
  __builtin_amdgcn_sched_barrier(0);
}

__device__ inline void zero_acc(mk_f16& acc) {
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
}

// epilogue: f(row, col, acc * s + b) for this lane's 16 accumulator rows (C/D map of the 32x32 MFMA:
// column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)); non-finite accumulators of live rows
// (< LIVE; an activation beyond the fp16 range met the split) raise the numerics flag
template <int LIVE, class F>
__device__ inline void mk_epi(const mk_f16& acc, const MkLin& L, int nt, unsigned* flags, F&& f) {
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  const int col = nt * 32 + li;
  const float s = gptr(L.s)[col], bias = L.b ? gptr(L.b)[col] : 0.f;
  bool bad = false;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
    if (row < LIVE) bad |= !__builtin_isfinite(acc[r]);
    f(row, col, acc[r] * s + bias);
  }
  if (bad && flags) atomicOr(flags, (unsigned)DD_NUM_F16_OVERFLOW);
}

__device__ inline void st_split(char* hi, int hp, int row, int col, float v) {
  const _Float16 h = (_Float16)v;
  const _Float16 l = (_Float16)(v - (float)h);
  reinterpret_cast<_Float16*>(hi)[row * hp + col] = h;
  reinterpret_cast<_Float16*>(hi + 32 * hp * 2)[row * hp + col] = l;
}

// 4 consecutive columns of a row into a split buffer (8 B hi, 8 B lo)
__device__ inline void st_split4(char* hi, int hp, int row, int c4, float4 v) {
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
  *reinterpret_cast<uint2*>(hi + (row * hp + c4) * 2) = hv;
  *reinterpret_cast<uint2*>(hi + 32 * hp * 2 + (row * hp + c4) * 2) = lv;
}

// LayerNorm(256) of one row held as one float4 per lane (layernorm_v4's arithmetic, eps 1e-5)
__device__ inline float4 ln256(float4 v, const float* g, const float* b, int lane) {
  float s = (v.x + v.y) + (v.z + v.w);
  s = wave_sum(s);
  const float mean = s / 256.f;
  const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
  float q = (dx * dx + dy * dy) + (dz * dz + dw * dw);
  q = wave_sum(q);
  const float rstd = rsqrtf(q / 256.f + 1e-5f);
  const mk_f4 g4 = gptr(reinterpret_cast<const mk_f4*>(g))[lane], b4 = gptr(reinterpret_cast<const mk_f4*>(b))[lane];
  const float4 gg = make_float4(g4.x, g4.y, g4.z, g4.w), bb = make_float4(b4.x, b4.y, b4.z, b4.w);
  float4 o;
  o.x = (v.x - mean) * rstd * gg.x + bb.x;
  o.y = (v.y - mean) * rstd * gg.y + bb.y;
  o.z = (v.z - mean) * rstd * gg.z + bb.z;
  o.w = (v.w - mean) * rstd * gg.w + bb.w;
  return o;
}

__device__ inline float4 relu4(float4 v) {
  return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
}

// 8 consecutive floats
__device__ inline void ld8(const float* p, float a[8]) {
  const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
  a[0] = x.x;
  a[1] = x.y;
  a[2] = x.z;
  a[3] = x.w;
  a[4] = y.x;
  a[5] = y.y;
  a[6] = y.z;
  a[7] = y.w;
}

// acc += A B for fp32 fragments split at use into fp16 hi / lo (al bh + ah bl + ah bh)
__device__ inline void mfma3(mk_f16& acc, const float a[8], const float b[8]) {
  mk_h8 ah, al, bh, bl;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ah[e] = (_Float16)a[e];
    al[e] = (_Float16)(a[e] - (float)ah[e]);
    bh[e] = (_Float16)b[e];
    bl[e] = (_Float16)(b[e] - (float)bh[e]);
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
}

// acc += A B with both fragments split three ways (x = h + m + l, each fp16) and the six products down to
// the 2^-22 terms (h h, h m, m h, h l, m m, l h): ~fp32-accurate. For the attention scores, whose error the
// softmax turns into a relative probability error (scores reach |100|: 3-product f16x3 left ~5e-5 in the
// decoded queries at B = 64, this ~4e-6)
__device__ inline void mfma6(mk_f16& acc, const float a[8], const float b[8]) {
  mk_h8 ah, am, al, bh, bm, bl;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ah[e] = (_Float16)a[e];
    const float ra = a[e] - (float)ah[e];
    am[e] = (_Float16)ra;
    al[e] = (_Float16)(ra - (float)am[e]);
    bh[e] = (_Float16)b[e];
    const float rb = b[e] - (float)bh[e];
    bm[e] = (_Float16)rb;
    bl[e] = (_Float16)(rb - (float)bm[e]);
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
}

}  // namespace
}  // namespace ddmi
