// Transformer-decoder megakernel: V2TransfuserModel._tf_decoder (transfuser_model_v2.py:141-142: 3 x
// nn.TransformerDecoderLayer(d 256, 8 heads, ffn 1024, ReLU, post-norm), query = the 31 learned query
// embeddings, memory = the scene's 65 keyval tokens) in ONE launch, one 512-thread workgroup per scene,
// followed by the trajectory head's step-invariant hoists of the decoded queries (the agent K / V
// projections and the ego cross-attention over one key, out_proj(v_proj(ego)), of both diffusion layers).
// The unfused chain is ~40 launches of 5-50 us (12 GEMMs, 6 attentions, 9 LayerNorms, 6 projections).
//
// Per layer, with x the scene's [31 (+1 zero pad) = 32][256] rows:
//   self-attention: q | k | v = x W_in^T + b (three 256-column units) -> fp32 LDS; 8 heads x 31 keys,
//     a wave per head on MFMA; out_proj + residual; norm1
//   cross-attention: q = x W_q^T + b; K / V of the memory come precomputed (one GEMM over every scene and
//     layer before the launch, `kvx`) and are read as MFMA fragments straight from L2; out_proj +
//     residual; norm2
//   attention per head (wave): S^T = K Q^T on MFMA with a three-way fp16 split (6 products; the softmax
//     amplifies score errors), keys on the accumulator rows, queries on the lanes; the softmax over each lane's own keys (+ one lane ^ 32 exchange), then O^T = V^T P^T whose
//     B operand is the S^T accumulator registers themselves (the k order of an MFMA step is free, so it
//     is chosen as the C layout's key order): no transpose, no LDS round trip for P
//   FFN 256 -> 1024 (ReLU) -> 256 in four hidden chunks, the second GEMM accumulating in registers;
//     residual; norm3
// Residuals read x back from its split LDS image (hi + lo: within 2^-22 relative of the fp32 value).
//
// Arithmetic as decoder_mk.hip (mk_core.h): f16x3 on v_mfma_f32_32x32x16_f16 with fragment-order weights
// streamed from L2 through a register ring chained across GEMMs; softmax / LayerNorm / attention in
// fp32 VALU. LDS: four 33 KB regions - XS (x as split hi / lo, the A operand), R1 (fp32 rows), R2 and R3
// (fp32 q / k / v, split operands).
#include <cmath>

#include "decoder_mk.h"
#include "mk_core.h"

namespace ddmi {

namespace {

constexpr int tQ = 31;   // queries: ego + 30 agents
constexpr int tM = 65;   // memory tokens: 8 x 8 BEV + status
constexpr int tD = 256, tNH = 8, tHD = 32, tFF = 1024, tL = 3;
constexpr int REG = 32 * HP * 2 * 2;  // one LDS region: a split [32][HP] hi + lo pair = 33792 B
constexpr int SPB = 32 * HP * 2;      // one split image
constexpr int LDS_T = 4 * REG;
static_assert(32 * FP * 4 <= REG, "fp32 rows fit a region");
static_assert(tQ <= 32 && tM <= 96, "one / three key tiles");

// x[row][col] from its split image
__device__ inline float xres(const char* xs, int row, int col) {
  const _Float16* h = reinterpret_cast<const _Float16*>(xs);
  return (float)h[row * HP + col] + (float)h[32 * HP + row * HP + col];
}

// LayerNorm of the fp32 rows of src into the split image dst (rows >= 31 zero); optionally also the fp32
// result of the live rows to gout [31][256]
__device__ inline void ln_rows(const float* src, const float* g, const float* b, char* dst, float* gout) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int q = wave + 8 * k;
    const float4 o = ln256(reinterpret_cast<const float4*>(src + q * FP)[lane], g, b, lane);
    st_split4(dst, HP, q, lane * 4, q < tQ ? o : make_float4(0.f, 0.f, 0.f, 0.f));
    if (gout && q < tQ) reinterpret_cast<float4*>(gout + q * tD)[lane] = o;
  }
}

// a MkLin read from the constant address space (scalar loads)
__device__ inline MkLin ld_lin(const __attribute__((address_space(4))) MkLin& x) {
  MkLin m;
  m.w = x.w;
  m.s = x.s;
  m.b = x.b;
  m.nks = x.nks;
  return m;
}

// B fragments of Q_h^T (k = head dimension, n = query = lane % 32) for the two k16 steps
__device__ inline void load_q_frags(const float* q, int h, float qf[2][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ld8(q + (lane & 31) * FP + h * tHD + 16 * ks + 8 * (lane >> 5), qf[ks]);
}

// Softmax over the keys of S^T tiles (C layout: key = 32 t + (r & 3) + 8 (r >> 2) + 4 (lane >> 5), query =
// lane % 32): each lane holds half of its query's keys, the other half sits in lane ^ 32. Keys >= nkeys masked.
template <int NTL>
__device__ inline void softmax_keys(mk_f16 st[NTL], int nkeys, float scale) {
  const int hh = (threadIdx.x & 63) >> 5;
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float v = key < nkeys ? st[t][r] * scale : -INFINITY;
      st[t][r] = v;
      m = fmaxf(m, v);
    }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = expf(st[t][r] - m);  // exp(-inf) = 0 for the masked keys
      st[t][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) st[t][r] *= inv;
}

// o += V_h^T P^T (o: C layout, row = head dimension, column = query = lane % 32). The k16 step (t, s) takes
// accumulator registers 8 s .. 8 s + 7 of tile t as the B fragment unchanged; the contraction order of its
// 16 keys is the one the C layout implies - lane half hh, element e <-> key 32 t + 16 s + 4 hh + (e & 3) +
// 8 (e >> 2) - and the A fragment (V^T) gathers the same keys: lane reads V[key][dim = lane % 32]
template <int NTL, class VROW>
__device__ inline void attn_pv_t(const mk_f16 st[NTL], mk_f16& o, VROW&& vrow, int nkeys) {
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float a8[8], b8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int key = 32 * t + 16 * s + 4 * hh + (e & 3) + 8 * (e >> 2);
        a8[e] = key < nkeys ? vrow(key)[li] : 0.f;
        b8[e] = st[t][8 * s + e];
      }
      mfma3(o, a8, b8);
    }
}

// the head's output O[query][h * 32 + dim] from o (C layout) into the split image dst; rows >= 31 zero
__device__ inline void store_head_out(char* dst, int h, const mk_f16& o) {
  const int lane = threadIdx.x & 63, q = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int dim = (r & 3) + 8 * (r >> 2) + 4 * hh;
    st_split(dst, HP, q, h * tHD + dim, q < tQ ? o[r] : 0.f);
  }
}

__global__ __launch_bounds__(NT, 1) void tfdec_mk_kernel(TfMkArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* XS = lds;
  float* R1 = reinterpret_cast<float*>(lds + REG);
  char* R2 = lds + 2 * REG;
  char* R3 = lds + 3 * REG;
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const MkLin none{};
  const float scale = 1.0f / sqrtf((float)tHD);
#ifdef DDMI_MK_STAMPS
  __shared__ unsigned long long st_lds[40];
  if (tid < 40) st_lds[tid] = 0ull;
  auto stamp = [&](int k) {
    if (tid == 0) st_lds[k] = __builtin_amdgcn_s_memtime();
  };
#else
  auto stamp = [](int) {};
#endif
  stamp(0);
  Ring R;
  // the per-layer table through the constant address space: scalar loads into SGPRs
  const __attribute__((address_space(4))) TfMkLayer* lay = (const __attribute__((address_space(4))) TfMkLayer*)a.layers;
  ring_fill(R, ld_lin(lay[0].sa_in), wave, 0);

  // x = the query embedding (transfuser_model_v2.py:141: query_embedding.weight[None].repeat(B, 1, 1))
  for (int e = tid; e < 32 * 64; e += NT) {
    const int q = e >> 6, c4 = (e & 63) * 4;
    const float4 v = q < tQ ? *reinterpret_cast<const float4*>(a.qemb + q * tD + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    st_split4(XS, HP, q, c4, v);
  }
  __syncthreads();

  mk_f16 acc, acc2;
#pragma unroll 1
  for (int l = 0; l < tL; ++l) {
    TfMkLayer L;
    {
      const __attribute__((address_space(4))) TfMkLayer& c = lay[l];
      L.sa_in = ld_lin(c.sa_in);
      L.sa_out = ld_lin(c.sa_out);
      L.ca_q = ld_lin(c.ca_q);
      L.ca_out = ld_lin(c.ca_out);
      L.l1 = ld_lin(c.l1);
      L.l2 = ld_lin(c.l2);
      L.n1g = c.n1g;
      L.n1b = c.n1b;
      L.n2g = c.n2g;
      L.n2b = c.n2b;
      L.n3g = c.n3g;
      L.n3b = c.n3b;
    }
    // ============================================================ self-attention
    float* Qf = R1;
    float* Kf = reinterpret_cast<float*>(R2);
    float* Vf = reinterpret_cast<float*>(R3);
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int nt = u * 8 + wave;
      zero_acc(acc);
      // (the ring is not carried through the attention phases, which need the registers: refilled there)
      mk_gemm<16>(XS, XS + SPB, HP, L.sa_in, nt, 0, acc, 0, R, u < 2 ? L.sa_in : none, u < 2 ? nt + 8 : 0, 0);
      float* dst = u == 0 ? Qf : (u == 1 ? Kf : Vf);
      mk_epi<tQ>(acc, L.sa_in, nt, a.flags, [&](int row, int col, float v) { dst[row * FP + col - u * tD] = v; });
    }
    __syncthreads();
    stamp(1 + 10 * l);
    {
      // wave = head h on MFMA (f16x3): S^T = K Q^T (keys on the C rows, queries on the lanes), softmax over
      // each lane's keys, then O^T = V^T P^T with P^T taken straight from the S^T accumulators (attn_pv_t)
      const int h = wave;
      float qf[2][8];
      load_q_frags(Qf, h, qf);
      mk_f16 sc;
      zero_acc(sc);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const float* kr = Kf + (lane & 31) * FP + h * tHD + 16 * ks + 8 * (lane >> 5);
        float a8[8];
        ld8(kr, a8);
        mfma6(sc, a8, qf[ks]);
      }
      mk_f16 st[3];
      st[0] = sc;
      softmax_keys<1>(st, tQ, scale);
      mk_f16 o;
      zero_acc(o);
      attn_pv_t<1>(st, o, [&](int key) { return Vf + key * FP + h * tHD; }, tQ);
      ring_fill(R, L.sa_out, wave, 0);
      __syncthreads();  // every wave is done with Q / K / V: R2 takes the attention output (split)
      store_head_out(R2, h, o);
    }
    __syncthreads();
    stamp(2 + 10 * l);
    // out_proj + residual -> R1; norm1 -> XS
    zero_acc(acc);
    mk_gemm<16>(R2, R2 + SPB, HP, L.sa_out, wave, 0, acc, 0, R, L.ca_q, wave, 0);
    mk_epi<tQ>(acc, L.sa_out, wave, a.flags,
               [&](int row, int col, float v) { R1[row * FP + col] = v + xres(XS, row, col); });
    __syncthreads();
    stamp(3 + 10 * l);
    ln_rows(R1, L.n1g, L.n1b, XS, nullptr);
    __syncthreads();
    stamp(4 + 10 * l);

    // ============================================================ cross-attention over the 65 memory tokens
    zero_acc(acc);
    mk_gemm<16>(XS, XS + SPB, HP, L.ca_q, wave, 0, acc, 0, R, none, 0, 0);
    float* Qc = reinterpret_cast<float*>(R2);
    mk_epi<tQ>(acc, L.ca_q, wave, a.flags, [&](int row, int col, float v) { Qc[row * FP + col] = v; });
    __syncthreads();
    stamp(5 + 10 * l);
    {
      // wave = head h on MFMA (f16x3), K / V fragments straight from the precomputed memory projections (L2):
      // S^T = K Q^T over 3 key tiles (65 keys, the rest masked), softmax, O^T = V^T P^T
      const int h = wave, li = lane & 31, hh = lane >> 5;
      const float* kvx = a.kvx + (int64_t)b * tM * 1536 + l * 512;
      float qf[2][8];
      load_q_frags(Qc, h, qf);
      mk_f16 st[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        zero_acc(st[t]);
        const int key = 32 * t + li;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          float a8[8];
          if (key < tM) {
            ld8(kvx + (int64_t)key * 1536 + h * tHD + 16 * ks + 8 * hh, a8);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) a8[e] = 0.f;
          }
          mfma6(st[t], a8, qf[ks]);
        }
      }
      softmax_keys<3>(st, tM, scale);
      mk_f16 o;
      zero_acc(o);
      attn_pv_t<3>(st, o, [&](int key) { return kvx + (int64_t)key * 1536 + tD + h * tHD; }, tM);
      ring_fill(R, L.ca_out, wave, 0);
      __syncthreads();  // every wave has read its q slice of R2
      store_head_out(R2, h, o);
    }
    __syncthreads();
    stamp(6 + 10 * l);
    zero_acc(acc);
    mk_gemm<16>(R2, R2 + SPB, HP, L.ca_out, wave, 0, acc, 0, R, L.l1, wave, 0);
    mk_epi<tQ>(acc, L.ca_out, wave, a.flags,
               [&](int row, int col, float v) { R1[row * FP + col] = v + xres(XS, row, col); });
    __syncthreads();
    stamp(7 + 10 * l);
    ln_rows(R1, L.n2g, L.n2b, XS, nullptr);
    __syncthreads();
    stamp(8 + 10 * l);

    // ============================================================ FFN, residual, norm3
    zero_acc(acc2);
#pragma unroll 1
    for (int c = 0; c < tFF / tD; ++c) {
      zero_acc(acc);
      mk_gemm<16>(XS, XS + SPB, HP, L.l1, c * 8 + wave, 0, acc, 0, R, L.l2, wave, c * 16);
      mk_epi<tQ>(acc, L.l1, c * 8 + wave, a.flags,
                 [&](int row, int col, float v) { st_split(R2, HP, row, col - c * tD, row < tQ ? fmaxf(v, 0.f) : 0.f); });
      __syncthreads();
      const bool more = c + 1 < tFF / tD;
      const MkLin nx = more ? L.l1 : (l + 1 < tL ? ld_lin(lay[l + 1].sa_in) : a.ag_kv[0]);
      mk_gemm<16>(R2, R2 + SPB, HP, L.l2, wave, c * 16, acc2, 0, R, nx, more ? (c + 1) * 8 + wave : wave, 0);
      __syncthreads();
    }
    mk_epi<tQ>(acc2, L.l2, wave, a.flags,
               [&](int row, int col, float v) { R1[row * FP + col] = v + xres(XS, row, col); });
    __syncthreads();
    stamp(9 + 10 * l);
    ln_rows(R1, L.n3g, L.n3b, XS, l + 1 == tL ? a.query_out + (int64_t)b * tQ * tD : nullptr);
    __syncthreads();
    stamp(10 + 10 * l);
  }

  // ============================================================ hoists of the trajectory head
  // agent K | V of both diffusion layers (rows 1..30 = the agent queries)
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int nt = u * 8 + wave;
      zero_acc(acc);
      const MkLin& nx = u == 0 ? a.ag_kv[d] : (d == 0 ? a.ag_kv[1] : a.eg_v[0]);
      mk_gemm<16>(XS, XS + SPB, HP, a.ag_kv[d], nt, 0, acc, 0, R, nx, u == 0 ? nt + 8 : wave, 0);
      float* out = a.akv[d] + (int64_t)b * 30 * 512;
      mk_epi<tQ>(acc, a.ag_kv[d], nt, a.flags, [&](int row, int col, float v) {
        if (row >= 1 && row < tQ) out[(row - 1) * 512 + col] = v;
      });
    }
  stamp(31);
  // ego: v_proj of query row 0 (split into R2 / R3, other rows zero), then out_proj
  zero_acc(acc);
  mk_gemm<16>(XS, XS + SPB, HP, a.eg_v[0], wave, 0, acc, 0, R, a.eg_v[1], wave, 0);
  mk_epi<1>(acc, a.eg_v[0], wave, a.flags, [&](int row, int col, float v) { st_split(R2, HP, row, col, row == 0 ? v : 0.f); });
  zero_acc(acc);
  mk_gemm<16>(XS, XS + SPB, HP, a.eg_v[1], wave, 0, acc, 0, R, a.eg_out[0], wave, 0);
  mk_epi<1>(acc, a.eg_v[1], wave, a.flags, [&](int row, int col, float v) { st_split(R3, HP, row, col, row == 0 ? v : 0.f); });
  __syncthreads();
  zero_acc(acc);
  mk_gemm<16>(R2, R2 + SPB, HP, a.eg_out[0], wave, 0, acc, 0, R, a.eg_out[1], wave, 0);
  mk_epi<1>(acc, a.eg_out[0], wave, a.flags, [&](int row, int col, float v) {
    if (row == 0) a.ego[0][(int64_t)b * tD + col] = v;
  });
  zero_acc(acc);
  mk_gemm<16>(R3, R3 + SPB, HP, a.eg_out[1], wave, 0, acc, 0, R, none, 0, 0);
  mk_epi<1>(acc, a.eg_out[1], wave, a.flags, [&](int row, int col, float v) {
    if (row == 0) a.ego[1][(int64_t)b * tD + col] = v;
  });
#ifdef DDMI_MK_STAMPS
  __syncthreads();
  stamp(32);
  if (a.stamps && tid < 40) a.stamps[(int64_t)b * 40 + tid] = st_lds[tid];
#endif
}

// ================================================================================================
// Four workgroups per scene (TfMkArgs::groups = 4). One workgroup streams every weight of the layer stack
// through its 8 waves' rings at the latency of its in-flight loads (~12.5 MB at ~45 GB/s: 0.3 ms, batch 1);
// here workgroup g of a scene takes
//   * heads 2g, 2g+1 of both attentions (their q | k | v / q column tiles: 6 and 2 waves),
//   * hidden chunk g (columns 256 g ..) of FFN linear1 and that K-slice of linear2 as a partial sum,
//   * one quarter of the trajectory-head hoists (g 0, 1: agent K | V of diffusion layer g; g 2, 3: the ego
//     chain of layer g - 2),
// and every workgroup runs the out_projs, residuals and LayerNorms on the full rows itself (identical inputs,
// identical arithmetic: identical results), so a layer exchanges three times through L2: the two attention
// outputs (each workgroup's 64 columns) and the four linear2 partials, summed in slab order 0..3 by every
// workgroup. Per wave a layer is 6 weight-streaming GEMM units instead of 14. The linear2 sum order differs
// from the one-workgroup kernel's single accumulation chain (fp32 rounding level; checked against the unfused
// chain and the goldens like it).
constexpr int tG = 4;
constexpr int XSLAB = 32 * tD;   // one [32][256] fp32 slab
constexpr int XBUF = tG * XSLAB;  // one exchange buffer (the linear2 partials take all four slabs)
constexpr int tNX = 3 * tL;       // exchanges per launch, each with a buffer of its own: a workgroup never reads
                                  // a line it (or its XCD's L2) read earlier in the launch, whose stale copy the
                                  // per-XCD L2 could serve after another XCD rewrote it

// Barrier of the scene's tG workgroups (MI355X_MICROARCH.md, inter-workgroup visibility): every wave's (sc1)
// stores drained, workgroup barrier, lane 0: agent release + vmcnt(0), relaxed arrival add, relaxed poll until
// the counter reaches target (monotonic within a launch: the n-th barrier waits for n * tG arrivals), agent
// acquire + vmcnt(0); workgroup barrier; then sc1 loads. A wait that outlives any healthy schedule raises a flag
// and goes on rather than hang the device. The arrival checks the count its add returned: at the n-th barrier a
// workgroup finds between (n - 1) tG (it is the first to arrive) and n tG - 1 (the last) earlier arrivals - no
// workgroup passes barrier n before every one has arrived at it - so anything else is a counter this launch did not
// start from zero (a stale or clobbered counter would let the wait pass early, silently): DD_NUM_SYNC_STATE.
__device__ inline void scene_sync(unsigned* cnt, unsigned target, unsigned* flags, unsigned spin_limit) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old >= target || old + tG < target) && flags) atomicOr(flags, DD_NUM_SYNC_STATE);
    unsigned n = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++n >= spin_limit) {
        if (flags) atomicOr(flags, DD_NUM_SYNC_TIMEOUT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// Exchange data moves with sc1 (write-through) stores and sc1 loads through a buffer resource over the scene's
// exchange area, as value_proj's split partials (MI355X_MICROARCH.md hand-off table)
constexpr int kXSC1 = 16;
__device__ inline __amdgpu_buffer_rsrc_t xrsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// head h's output O[query][h * 32 + dim] from o (C layout) into an fp32 exchange slab (float offset so); rows >= 31 zero
__device__ inline void put_head_out(__amdgpu_buffer_rsrc_t rx, int so, int h, const mk_f16& o) {
  const int lane = threadIdx.x & 63, q = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int dim = (r & 3) + 8 * (r >> 2) + 4 * hh;
    const float v = q < tQ ? o[r] : 0.f;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rx, (so + q * tD + h * tHD + dim) * 4, 0,
                                          kXSC1);
  }
}

// a [32][256] fp32 exchange slab (float offset so) into a split image
__device__ inline void get_rows_split(__amdgpu_buffer_rsrc_t rx, int so, char* dst) {
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = threadIdx.x + NT * k;
    const int row = e >> 6, c4 = (e & 63) * 4;
    v[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, (so + row * tD + c4) * 4, 0, kXSC1));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = threadIdx.x + NT * k;
    st_split4(dst, HP, e >> 6, (e & 63) * 4, v[k]);
  }
}

__global__ __launch_bounds__(NT, 1) void tfdec_mk4_kernel(TfMkArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* XS = lds;
  float* R1 = reinterpret_cast<float*>(lds + REG);
  char* R2 = lds + 2 * REG;
  char* R3 = lds + 3 * REG;
  const int b = blockIdx.x / tG, g = blockIdx.x - (blockIdx.x / tG) * tG;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 31, hh = lane >> 5;
  const MkLin none{};
  const float scale = 1.0f / sqrtf((float)tHD);
  unsigned* cnt = a.sync_cnt + b;
  const __amdgpu_buffer_rsrc_t rx = xrsrc(a.xbuf + (int64_t)b * tNX * XBUF);
  unsigned nsync = 0;
  auto sync = [&]() {
    ++nsync;
    scene_sync(cnt, nsync * tG, a.flags, a.spin_limit);
  };
  auto xbuf_next = [&]() { return (int)nsync * XBUF; };  // exchange n writes buffer n (float offset)
  const __attribute__((address_space(4))) TfMkLayer* lay = (const __attribute__((address_space(4))) TfMkLayer*)a.layers;
  // this wave's tiles: self-attention q | k | v unit wave / 2 of head 2g + (wave & 1) (waves 0..5), cross q of
  // head 2g + wave (waves 0, 1), FFN hidden tile wave of chunk g
  const int qkv_nt = (wave >> 1) * 8 + 2 * g + (wave & 1);
  const int caq_nt = 2 * g + wave;
  const int l1_nt = 8 * g + wave;
  Ring R;
  if (wave < 6) ring_fill(R, ld_lin(lay[0].sa_in), qkv_nt, 0);

  for (int e = tid; e < 32 * 64; e += NT) {
    const int q = e >> 6, c4 = (e & 63) * 4;
    const float4 v = q < tQ ? *reinterpret_cast<const float4*>(a.qemb + q * tD + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    st_split4(XS, HP, q, c4, v);
  }
  __syncthreads();

  mk_f16 acc, acc2;
#pragma unroll 1
  for (int l = 0; l < tL; ++l) {
    TfMkLayer L;
    {
      const __attribute__((address_space(4))) TfMkLayer& c = lay[l];
      L.sa_in = ld_lin(c.sa_in);
      L.sa_out = ld_lin(c.sa_out);
      L.ca_q = ld_lin(c.ca_q);
      L.ca_out = ld_lin(c.ca_out);
      L.l1 = ld_lin(c.l1);
      L.l2 = ld_lin(c.l2);
      L.n1g = c.n1g;
      L.n1b = c.n1b;
      L.n2g = c.n2g;
      L.n2b = c.n2b;
      L.n3g = c.n3g;
      L.n3b = c.n3b;
    }
    // ============================================================ self-attention, heads 2g, 2g+1
    float* Qf = R1;
    float* Kf = reinterpret_cast<float*>(R2);
    float* Vf = reinterpret_cast<float*>(R3);
    if (wave < 6) {
      const int u = wave >> 1;
      zero_acc(acc);
      mk_gemm<16>(XS, XS + SPB, HP, L.sa_in, qkv_nt, 0, acc, 0, R, none, 0, 0);
      float* dst = u == 0 ? Qf : (u == 1 ? Kf : Vf);
      mk_epi<tQ>(acc, L.sa_in, qkv_nt, a.flags, [&](int row, int col, float v) { dst[row * FP + col - u * tD] = v; });
    }
    __syncthreads();
    int xo = xbuf_next();
    if (wave < 2) {
      const int h = 2 * g + wave;
      float qf[2][8];
      load_q_frags(Qf, h, qf);
      mk_f16 sc;
      zero_acc(sc);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float a8[8];
        ld8(Kf + li * FP + h * tHD + 16 * ks + 8 * hh, a8);
        mfma6(sc, a8, qf[ks]);
      }
      mk_f16 st[3];
      st[0] = sc;
      softmax_keys<1>(st, tQ, scale);
      mk_f16 o;
      zero_acc(o);
      attn_pv_t<1>(st, o, [&](int key) { return Vf + key * FP + h * tHD; }, tQ);
      put_head_out(rx, xo, h, o);
    }
    ring_fill(R, L.sa_out, wave, 0);
    sync();
    get_rows_split(rx, xo, R2);
    __syncthreads();
    // out_proj + residual -> R1; norm1 -> XS (every workgroup, full rows)
    zero_acc(acc);
    mk_gemm<16>(R2, R2 + SPB, HP, L.sa_out, wave, 0, acc, 0, R, wave < 2 ? L.ca_q : none, wave < 2 ? caq_nt : 0, 0);
    mk_epi<tQ>(acc, L.sa_out, wave, a.flags,
               [&](int row, int col, float v) { R1[row * FP + col] = v + xres(XS, row, col); });
    __syncthreads();
    ln_rows(R1, L.n1g, L.n1b, XS, nullptr);
    __syncthreads();

    // ============================================================ cross-attention, heads 2g, 2g+1
    float* Qc = reinterpret_cast<float*>(R2);
    if (wave < 2) {
      zero_acc(acc);
      mk_gemm<16>(XS, XS + SPB, HP, L.ca_q, caq_nt, 0, acc, 0, R, none, 0, 0);
      mk_epi<tQ>(acc, L.ca_q, caq_nt, a.flags, [&](int row, int col, float v) { Qc[row * FP + col] = v; });
    }
    __syncthreads();
    xo = xbuf_next();
    if (wave < 2) {
      const int h = 2 * g + wave;
      const float* kvx = a.kvx + (int64_t)b * tM * 1536 + l * 512;
      float qf[2][8];
      load_q_frags(Qc, h, qf);
      mk_f16 st[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        zero_acc(st[t]);
        const int key = 32 * t + li;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          float a8[8];
          if (key < tM) {
            ld8(kvx + (int64_t)key * 1536 + h * tHD + 16 * ks + 8 * hh, a8);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) a8[e] = 0.f;
          }
          mfma6(st[t], a8, qf[ks]);
        }
      }
      softmax_keys<3>(st, tM, scale);
      mk_f16 o;
      zero_acc(o);
      attn_pv_t<3>(st, o, [&](int key) { return kvx + (int64_t)key * 1536 + tD + h * tHD; }, tM);
      put_head_out(rx, xo, h, o);
    }
    ring_fill(R, L.ca_out, wave, 0);
    sync();
    get_rows_split(rx, xo, R2);
    __syncthreads();
    zero_acc(acc);
    mk_gemm<16>(R2, R2 + SPB, HP, L.ca_out, wave, 0, acc, 0, R, L.l1, l1_nt, 0);
    mk_epi<tQ>(acc, L.ca_out, wave, a.flags,
               [&](int row, int col, float v) { R1[row * FP + col] = v + xres(XS, row, col); });
    __syncthreads();
    ln_rows(R1, L.n2g, L.n2b, XS, nullptr);
    __syncthreads();

    // ============================================================ FFN: hidden chunk g, its linear2 partial
    zero_acc(acc);
    mk_gemm<16>(XS, XS + SPB, HP, L.l1, l1_nt, 0, acc, 0, R, L.l2, wave, g * 16);
    mk_epi<tQ>(acc, L.l1, l1_nt, a.flags,
               [&](int row, int col, float v) { st_split(R2, HP, row, col - g * tD, row < tQ ? fmaxf(v, 0.f) : 0.f); });
    __syncthreads();
    zero_acc(acc2);
    {
      MkLin nx = none;
      int nnt = 0;
      if (l + 1 < tL) {
        if (wave < 6) {
          nx = ld_lin(lay[l + 1].sa_in);
          nnt = qkv_nt;
        }
      } else {
        nx = g < 2 ? a.ag_kv[g] : a.eg_v[g - 2];
        nnt = wave;
      }
      mk_gemm<16>(R2, R2 + SPB, HP, L.l2, wave, g * 16, acc2, 0, R, nx, nnt, 0);
    }
    const int xp = xbuf_next();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned u = __builtin_bit_cast(unsigned, (float)acc2[r]);
      __builtin_amdgcn_raw_buffer_store_b32(u, rx, (xp + g * XSLAB + ((r & 3) + 8 * (r >> 2) + 4 * hh) * tD + wave * 32 + li) * 4,
                                            0, kXSC1);
    }
    sync();
    // every workgroup: x = LN3(x + (p0 + p1 + p2 + p3) s + b), its waves summing their own tiles' partials
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = (xp + ((r & 3) + 8 * (r >> 2) + 4 * hh) * tD + wave * 32 + li) * 4;
      float p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        p[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, o + j * XSLAB * 4, 0, kXSC1));
      acc2[r] = ((p[0] + p[1]) + p[2]) + p[3];
    }
    mk_epi<tQ>(acc2, L.l2, wave, a.flags,
               [&](int row, int col, float v) { R1[row * FP + col] = v + xres(XS, row, col); });
    __syncthreads();
    ln_rows(R1, L.n3g, L.n3b, XS, (l + 1 == tL && g == 0) ? a.query_out + (int64_t)b * tQ * tD : nullptr);
    __syncthreads();
  }

  // every workgroup of the scene is past its last wait: the last to get here resets the scene's counters
  if (tid == 0) {
    unsigned* done = a.sync_cnt + a.B + b;
    const unsigned old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old >= tG && a.flags) atomicOr(a.flags, DD_NUM_SYNC_STATE);
    if (old == tG - 1 && !a.no_reset) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // ============================================================ hoists of the trajectory head, a quarter each
  if (g < 2) {
    // agent K | V of diffusion layer d = g (rows 1..30 = the agent queries)
    const int d = g;
    float* out = a.akv[d] + (int64_t)b * 30 * 512;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int nt = u * 8 + wave;
      zero_acc(acc);
      mk_gemm<16>(XS, XS + SPB, HP, a.ag_kv[d], nt, 0, acc, 0, R, u == 0 ? a.ag_kv[d] : none, u == 0 ? nt + 8 : 0, 0);
      mk_epi<tQ>(acc, a.ag_kv[d], nt, a.flags, [&](int row, int col, float v) {
        if (row >= 1 && row < tQ) out[(row - 1) * 512 + col] = v;
      });
    }
  } else {
    // ego of diffusion layer d = g - 2: out_proj(v_proj(query row 0))
    const int d = g - 2;
    zero_acc(acc);
    mk_gemm<16>(XS, XS + SPB, HP, a.eg_v[d], wave, 0, acc, 0, R, a.eg_out[d], wave, 0);
    mk_epi<1>(acc, a.eg_v[d], wave, a.flags, [&](int row, int col, float v) { st_split(R2, HP, row, col, row == 0 ? v : 0.f); });
    __syncthreads();
    zero_acc(acc);
    mk_gemm<16>(R2, R2 + SPB, HP, a.eg_out[d], wave, 0, acc, 0, R, none, 0, 0);
    mk_epi<1>(acc, a.eg_out[d], wave, a.flags, [&](int row, int col, float v) {
      if (row == 0) a.ego[d][(int64_t)b * tD + col] = v;
    });
  }
}

}  // namespace

bool tfdec_mk_layer_ok(const TfMkLayer& L) {
  return L.sa_in.nks == 16 && L.sa_out.nks == 16 && L.ca_q.nks == 16 && L.ca_out.nks == 16 && L.l1.nks == 16 &&
         L.l2.nks == 64 && L.sa_in.w && L.l2.w && L.n3b;
}

size_t tfdec_mk_xbuf_floats(int B) { return (size_t)B * tNX * XBUF; }

bool tfdec_mk_supported(int nq, int nmem, int d, int heads, int ffn, int layers) {
  return nq == tQ && nmem == tM && d == tD && heads == tNH && ffn == tFF && layers == tL;
}

void launch_tfdec_mk(const TfMkArgs& a, hipStream_t st) {
  if (a.B <= 0) return;
  if (!a.layers || !a.qemb || !a.kvx || !a.query_out || !a.akv[0] || !a.akv[1] || !a.ego[0] || !a.ego[1])
    throw std::runtime_error("tfdec_mk: missing operand");
  if (a.groups == tG) {
    if (!a.xbuf || !a.sync_cnt) throw std::runtime_error("tfdec_mk: groups = 4 needs xbuf / sync_cnt");
    if (a.xbuf_floats < tfdec_mk_xbuf_floats(a.B))
      throw std::runtime_error("tfdec_mk: xbuf holds " + std::to_string(a.xbuf_floats) + " floats, groups = 4 needs " +
                               std::to_string(tfdec_mk_xbuf_floats(a.B)));
    if (a.sync_cnt_n < (size_t)2 * a.B) throw std::runtime_error("tfdec_mk: sync_cnt needs 2 B counters");
    static std::atomic<uint64_t> attr4;
    // the scene counters start at zero (zeroed at allocation) and the last workgroup of a scene to finish resets
    // them: only agent-scope atomics ever write them. (A memset node zeroing them ahead of the kernel was not seen by
    // the kernel's memory-side atomic arrivals in graph replays: profiles/round6_memset_node.md.)
    TfMkArgs aa = a;
    // tests/test_sync_gpu.py, read per dispatch (eager forwards): DDMI_TF_NORESET=1 leaves the counters as they are
    // (the next launch starts dirty), DDMI_TF_SPIN=n gives every wait up after n polls (forced timeouts)
    if (const char* e = getenv("DDMI_TF_NORESET")) aa.no_reset = atoi(e) != 0;
    if (const char* e = getenv("DDMI_TF_SPIN")) aa.spin_limit = (unsigned)std::max(1, atoi(e));
    set_max_lds_once(attr4, reinterpret_cast<const void*>(tfdec_mk4_kernel), LDS_T);
    hipLaunchKernelGGL(tfdec_mk4_kernel, dim3(a.B * tG), dim3(NT), LDS_T, st, aa);
    DD_HIP_CHECK(hipGetLastError());
    return;
  }
  if (a.groups != 1) throw std::runtime_error("tfdec_mk: groups must be 1 or 4");
  static std::atomic<uint64_t> attr;
  set_max_lds_once(attr, reinterpret_cast<const void*>(tfdec_mk_kernel), LDS_T);
  hipLaunchKernelGGL(tfdec_mk_kernel, dim3(a.B), dim3(NT), LDS_T, st, a);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
