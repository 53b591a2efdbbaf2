// ddmi — internal declarations shared by the HIP kernel TUs and the runtime.
// All feature maps live in HBM as fp32 NHWC ("channels-last"): a pixel's channel vector is
// contiguous, so implicit-GEMM convs read 16-B float4 channel slices and the BEV gathers of
// the decoder read whole 1 KB rows (see DESIGN.md §Data layout).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>
#include <stdexcept>
#include <string>

#define DD_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " __FILE__ ":" + std::to_string(__LINE__) + ": " #expr); \
  } while (0)

namespace ddmi {

// Raise a kernel's dynamic-LDS limit to `bytes` once per device (the attribute is per device; the
// bit of a device is claimed atomically, so two threads driving two handles each set their own).
// `mask` is the caller's function-local static.
inline void set_max_lds_once(std::atomic<uint64_t>& mask, const void* kernel, int bytes) {
  int dev = 0;
  DD_HIP_CHECK(hipGetDevice(&dev));
  const uint64_t bit = uint64_t(1) << (dev & 63);
  if (mask.load(std::memory_order_acquire) & bit) return;
  DD_HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  mask.fetch_or(bit, std::memory_order_acq_rel);
}

// Strided 4-D view (n, h, w, c) with element strides; c stride is sc.
struct View4 {
  float* p = nullptr;
  int64_t sn = 0, sh = 0, sw = 0, sc = 1;
};

// ----------------------------------------------------------------------------------------
// Implicit-GEMM convolution / GEMM on fp32 MFMA (conv_gemm.hip).
//   out[n,oh,ow,co] = act( sum_{kh,kw,ci} in[n, oh*s-p+kh, ow*s-p+kw, ci] * W(co; kh,kw,ci)
//                          + bias[co] + res[n,oh,ow,co] )
// GEMM view: M = Nimg*Ho*Wo, N = Cout, K = KH*KW*Cin (k order kh, kw, ci).
// Input channel stride must be 1 and Cin % 4 == 0; in_sw/in_sh/in_sn are element strides.
// W(co; k) = wgt[co*ldb + k] (b_kn = 0, "nn.Linear / OHWI" layout) or wgt[k*ldb + co] (b_kn = 1).
// Batched launches (gridDim.z = batch): every pointer is offset by z1*?_z1 + z2*?_z2 with
// z1 = z / zdiv, z2 = z % zdiv (used for per-(scene, head) attention GEMMs).
struct ConvArgs {
  const float* in = nullptr;
  int64_t in_sn = 0, in_sh = 0, in_sw = 0;
  int H = 1, W = 1, Cin = 0;
  const float* wgt = nullptr;
  int64_t ldb = 0;
  int b_kn = 0;
  const float* bias = nullptr;
  const float* res = nullptr;
  int64_t res_sn = 0, res_sh = 0, res_sw = 0;
  float* out = nullptr;
  int64_t out_sn = 0, out_sh = 0, out_sw = 0;
  int Nimg = 1, Ho = 1, Wo = 1, Cout = 0;
  int KH = 1, KW = 1, stride = 1, pad = 0;
  int relu = 0;
  float alpha = 1.0f;  // scale applied to the accumulator before bias/res
  // K-split scratch for conv_x3 at small grids (runtime-owned, one per stream of the forward): S x M x Cout fp32
  // partials, summed in split order by a reduce launch that applies the epilogue; null: no split
  float* split_part = nullptr;
  int64_t split_cap = 0;  // floats
  int batch = 1, zdiv = 1;
  int64_t in_z1 = 0, in_z2 = 0, w_z1 = 0, w_z2 = 0, out_z1 = 0, out_z2 = 0, res_z1 = 0, res_z2 = 0;
  int64_t flops_K = -1;  // algorithmic K per output (excluding channel padding); -1 = KH*KW*Cin
  // f16x3 split path (conv_x3.hip): pre-split weights hi / lo [Cout][ldh] fp16 (K order as wgt,
  // zero padded to ldh % 8 == 0) with per-channel inverse power-of-two scales; flags receives
  // DD_NUM_* bits. When wh is set, launch_conv_gemm dispatches to the f16x3 kernel.
  const uint16_t* wh = nullptr;
  const uint16_t* wl = nullptr;
  const float* wsinv = nullptr;
  int64_t ldh = 0;
  unsigned* flags = nullptr;
  int prec = 0;  // 0 = f16x3 (wh / wl fp16 hi / lo), 1 = bf16 (wh = bf16 image, one product)
  // Gathered output rows (conv_x3 MODE 1 only): output row m (launch geometry Nimg = 1, Ho = M,
  // Wo = 1, compact rows out + m * out_sh) is the conv at input-geometry pixel rowmap[m] =
  // n * H * W + oh * W + ow (stride 1, Ho = H, Wo = W), or a don't-care row when rowmap[m] < 0.
  // rowmap_nimg = images in the input (operand-extent check).
  const int* rowmap = nullptr;
  int rowmap_nimg = 0;
  // Compacted gathered rows: rowcount[n] live rows of image n sit at rowmap[n * rowcap + l], l < rowcount[n];
  // launch row m is the m-th live row over the images in order (rows past the total are don't-care), and
  // its output goes to row n * rowcap + l - so every tile is full except the last, and the output layout
  // stays the per-image one the consumer indexes.
  const int* rowcount = nullptr;
  int rowcap = 0;
  // Fused GPT token pooling (conv_x6 only; launch_conv_gemm reports it through last_conv_pooled()):
  // when pool_out is set, the mean of every pool_p x pool_p output window (after bias / residual / ReLU)
  // plus pool_add[wy * pool_add_sh + wx * pool_add_sw + c] (if set) is also written to
  // pool_out[n * pool_sn + wy * pool_sh + wx * pool_sw + c] - the avgpool_kernel arithmetic, same order.
  float* pool_out = nullptr;
  int pool_p = 0;
  int64_t pool_sn = 0, pool_sh = 0, pool_sw = 0;
  const float* pool_add = nullptr;
  int64_t pool_add_sh = 0, pool_add_sw = 0;
  // Fused LayerNorm of the finished output rows (conv_x3's quad epilogue with one N tile spanning the row, Cout 64
  // or 128; launch_conv_gemm reports it through last_conv_ln()): ln_out (the same row layout as out) receives
  // LayerNorm(out row) * ln_g + ln_b with layernorm_v4's arithmetic and lane order (bit-identical to the separate
  // launch). Not fused: ln_out untouched, last_conv_ln() false.
  float* ln_out = nullptr;
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
};
constexpr unsigned DD_NUM_F16_OVERFLOW = 1u;  // an activation |x| >= 65504 met the f16x3 split
constexpr unsigned DD_NUM_SYNC_TIMEOUT = 2u;  // a megakernel's inter-workgroup wait gave up (tfdec_mk groups)
// a megakernel's inter-workgroup counter held a value no healthy launch leaves there (an arrival saw more or fewer
// earlier arrivals than its barrier allows): the waits it guards cannot be trusted; dd_numerics_flags' clear re-zeroes
// the counters
constexpr unsigned DD_NUM_SYNC_STATE = 4u;

#ifdef __HIPCC__
// Implicit-GEMM epilogue row table: element offsets of output / residual row m0 + r (r < BM) of a tile,
// written to LDS as [BM][2] int64 (-1 output offset = row past M). One runtime-divisor (n, oh, ow)
// decomposition per row and thread, instead of one per fragment row and pass - the division sequences
// cost conv_x5 as many cycles as its K loop on the GPT GEMMs (K = 256 - 512).
// rowidx (optional, per tile row): the output row of tile row r (< 0: none) instead of m0 + r.
template <int BM, int NT>
__device__ inline void epi_row_table(const ConvArgs& a, int m0, int M, int tid, long long* tab,
                                     const int* rowidx = nullptr) {
  for (int r = tid; r < BM; r += NT) {
    const int m = rowidx ? rowidx[r] : m0 + r;
    long long oo = -1, ro = 0;
    if (m >= 0 && m < M) {
      const int ow = m % a.Wo, t2 = m / a.Wo;
      const int oh = t2 % a.Ho, n = t2 / a.Ho;
      oo = (long long)n * a.out_sn + (long long)oh * a.out_sh + (long long)ow * a.out_sw;
      ro = (long long)n * a.res_sn + (long long)oh * a.res_sh + (long long)ow * a.res_sw;
    }
    tab[2 * r] = oo;
    tab[2 * r + 1] = ro;
  }
}

// Exclusive prefix of n <= 256 per-image row counts into pre[0..n] (pre[n] = total), by the first wave of the
// workgroup: 4 counts per lane, a 64-lane shuffle scan (a serial loop by one thread cost ~4 us per workgroup).
// Every thread must call it; it ends with a workgroup barrier.
__device__ inline void rowcount_prefix(const int* counts, int n, int* pre) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    int c[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * tid + j;
      c[j] = i < n ? counts[i] : 0;
      s += c[j];
    }
    int inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (tid >= o) inc += v;
    }
    int run = inc - s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * tid + j;
      if (i <= n) pre[i] = run;
      run += c[j];
    }
    if (tid == 63 && n == 256) pre[256] = run;
  }
  __syncthreads();
}

// Can epi_quads serve this launch? Every output / residual row starts 16-B aligned and Cout % 4 == 0.
__host__ __device__ inline bool epi_quads_ok(const ConvArgs& a) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  auto st4 = [](int64_t s, int n) { return n == 1 || s % 4 == 0; };
  return a.Cout % 4 == 0 && al(a.out) && al(a.wsinv) && (!a.bias || al(a.bias)) && st4(a.out_sn, a.Nimg) &&
         st4(a.out_sh, a.Ho) && st4(a.out_sw, a.Wo) &&
         (!a.res || (al(a.res) && st4(a.res_sn, a.Nimg) && st4(a.res_sh, a.Ho) && st4(a.res_sw, a.Wo)));
}
template <int WM, int WN, int TM, int TN>
constexpr int epi_quads_lds() {  // bytes: one parked slab of every wave + the row table
  return WM * 32 * WN * TN * 32 * 4 + WM * TM * 32 * 16;
}

// Implicit-GEMM epilogue through LDS (after the K loop, with the stage LDS free): slab i (32 rows per
// wave row) of the WM x WN waves' 32x32 accumulators is parked as [WM*32 rows][BN] fp32, then every
// thread finishes 16-B channel quads of whole rows - weight scale, alpha, bias, residual, ReLU - with
// one 16-B store each. The accumulator layout's own stores (4 B per lane, 128 B per half-wave) are
// store-issue bound: the 256 x 256 tile's 1024 of them per workgroup took as long as a K = 512 loop.
// Parked 16-B slots are XOR-ed with bit 2 of the row (<< 3): a park store's two half-waves write rows
// 4 apart, which then fall on opposite 32-bank halves. Returns true if an accumulator was non-finite.
// C/D map of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
template <int WM, int WN, int TM, int TN, typename Acc>
__device__ inline bool epi_quads(const ConvArgs& a, const Acc (&acc)[TM][TN], char* lds, int m0, int n0, int M,
                                 int tid, const int* rowidx = nullptr) {
  typedef float f4_t __attribute__((ext_vector_type(4)));
  constexpr int NT = 64 * WM * WN, BN = WN * TN * 32, QN = BN / 4, PR = WM * 32;
  constexpr int RPP = NT / QN, IT = PR / RPP;  // rows per pass, quads per thread per slab
  static_assert(NT % QN == 0 && PR % RPP == 0 && BN >= 64, "quad epilogue tiling");
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN, li = lane & 31, hh = lane >> 5;
  float* ct = reinterpret_cast<float*>(lds);
  long long* tab = reinterpret_cast<long long*>(lds + PR * BN * 4);
  epi_row_table<WM * TM * 32, NT>(a, m0, M, tid, tab, rowidx);
  const int qn = tid % QN, nq = n0 + 4 * qn;
  const bool nv = nq < a.Cout;
  f4_t scl = {0.f, 0.f, 0.f, 0.f}, bia = {0.f, 0.f, 0.f, 0.f};
  if (nv) {
    scl = *reinterpret_cast<const f4_t*>(a.wsinv + nq) * a.alpha;
    if (a.bias) bia = *reinterpret_cast<const f4_t*>(a.bias + nq);
  }
  // fused LayerNorm (ConvArgs::ln_out): only when this tile spans the whole row
  const bool ln = a.ln_out && BN == a.Cout && (QN == 16 || QN == 32 || QN == 64);
  f4_t lg = {0.f, 0.f, 0.f, 0.f}, lb = {0.f, 0.f, 0.f, 0.f};
  if (ln) {
    lg = *reinterpret_cast<const f4_t*>(a.ln_g + nq);
    lb = *reinterpret_cast<const f4_t*>(a.ln_b + nq);
  }
  bool bad = false;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if (i) __syncthreads();  // every thread has read the previous slab
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int col = (wn * TN + j) * 32 + li;
        ct[pr * BN + ((((col >> 2) ^ (((pr >> 2) & 1) << 3))) << 2) + (col & 3)] = acc[i][j][r];
      }
    __syncthreads();
    // the slab's residuals are all loaded before its first store (out may alias res)
    f4_t rv[IT];
    long long oo[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int pr = tid / QN + k * RPP;
      const int tr = ((pr >> 5) * TM + i) * 32 + (pr & 31);
      oo[k] = nv ? tab[2 * tr] : -1;
      rv[k] = (a.res && oo[k] >= 0) ? *reinterpret_cast<const f4_t*>(a.res + tab[2 * tr + 1] + nq)
                                    : (f4_t){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      if (oo[k] < 0) continue;
      const int pr = tid / QN + k * RPP;
      const f4_t c = *reinterpret_cast<const f4_t*>(ct + pr * BN + ((qn ^ (((pr >> 2) & 1) << 3)) << 2));
      bad |= !(__builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z) &&
               __builtin_isfinite(c.w));
      f4_t v = c * scl + bia + rv[k];
      if (a.relu) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      // nontemporal: with conv_x6's and the upsample-add's output stores the same, +0.5 % scenes/s same-box in both
      // the in-flight and the one-at-a-time bench (profiles/round3_o_nt_stores_ab.txt); conv_x5 / conv_x3 shapes
      // alone 1-10 % faster on the conv micro-benchmark
      __builtin_nontemporal_store(v, reinterpret_cast<f4_t*>(a.out + oo[k] + nq));
      if (ln) {
        // LayerNorm of the finished row: the row is the QN consecutive lanes of this pass (QN = BN / 4 = Cout / 4 =
        // layernorm_v4's LPR, VPL 1, lane sub = quad), so the sums, the xor tree and the rounding (no contraction)
        // are layernorm_v4's: bit-identical to the separate launch. Dead rows are dead for the whole lane group.
#pragma clang fp contract(off)
        float s = 0.f;
        s += (v.x + v.y) + (v.z + v.w);
#pragma unroll
        for (int o = QN / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        const float mean = s / (float)BN;
        const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
        float q = 0.f;
        q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
#pragma unroll
        for (int o = QN / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        const float rstd = rsqrtf(q / (float)BN + 1e-5f);
        f4_t o4;
        o4.x = (v.x - mean) * rstd * lg.x + lb.x;
        o4.y = (v.y - mean) * rstd * lg.y + lb.y;
        o4.z = (v.z - mean) * rstd * lg.z + lb.z;
        o4.w = (v.w - mean) * rstd * lg.w + lb.w;
        *reinterpret_cast<f4_t*>(a.ln_out + oo[k] + nq) = o4;
      }
    }
  }
  return bad;
}
#endif
void launch_conv_gemm(const ConvArgs& a, hipStream_t st);
void launch_conv_x3(const ConvArgs& a, hipStream_t st);
// Fused stem conv 7x7/2 (Cin 4, Cout 64, f16x3) + bias + ReLU + maxpool 3x3/2 into pool_out (B,Hp,Wp,64)
// (stem_pool.hip); false when `a` is not such a stem (then nothing is launched).
// src (optional): the device word holding the address of the reference's NCHW input of src_c channels (read by the
// kernel; the NHWC4 a.in is then unused).
bool launch_stem_pool(const ConvArgs& a, float* pool_out, int Hp, int Wp, hipStream_t st,
                      const float* const* src = nullptr, int src_c = 0);
// Device-side input table: tab[0] = a, tab[1] = b (one thread; launched per forward outside the captured graph).
void launch_set_ptrs(const float** tab, const float* a, const float* b, hipStream_t st);
// name of the kernel the last conv / GEMM dispatch on this thread went to ("conv_gemm", "conv_x3",
// "conv_x5", "conv_x6"); the runtime's profiler attributes launch time per kernel with it
const char* last_conv_kernel();
bool last_conv_pooled();           // did the last launch_conv_gemm also write ConvArgs::pool_out?
void set_last_conv_pooled(bool p);
bool last_conv_ln();               // did the last launch_conv_gemm also write ConvArgs::ln_out?
void set_last_conv_ln(bool p);
// the kernel + tile configuration of the calling thread's last conv / GEMM launch, e.g.
// "conv_x6<8,32,128,4,2>" (TH, TW, BN, wave grid), "conv_x5<256,256>", "conv_x3<128,128,f16x3>"
const char* last_conv_config();
void set_last_conv_config(const char* cfg);

// ----------------------------------------------------------------------------------------
// The gathered value_proj (value_proj.hip): value rows = ReLU(conv3x3(map) + bias) at the scenes' distinct tap
// pixels, rows[b * cap + l] (l < counts[b]) = pixel b * 4096 + y * 64 + x of the (B, 64, 64, 256) NHWC map; row
// b * cap + l of `out` receives it. wh / wl: the f16x3 weight images [256][ldh] (K order kh, kw, ci) with
// per-column inverse scales wsinv; part: [3][B * cap][256] fp32 scratch; tile_cnt: vproj_tiles(B, cap) zeroed
// words (left zeroed by every launch).
struct VprojArgs {
  const float* map = nullptr;
  const uint16_t* wh = nullptr;
  const uint16_t* wl = nullptr;
  const float* wsinv = nullptr;
  int ldh = 0;
  const float* bias = nullptr;
  const int* rows = nullptr;
  const int* counts = nullptr;
  int B = 0, cap = 0;
  float* part = nullptr;  // the union form's split partials (usplit > 1): [usplit][B * cap][256]
  float* out = nullptr;
  unsigned* flags = nullptr;
  // the union-staged kernel, then the gathered one for the tiles it flagged (fb: [tiles][2] words, zero between
  // launches); union 0 = the gathered kernel for every tile (DDMI_VPROJ_UNION=0)
  int union_stage = 1;
  int umax = 1 << 30;  // union size above which a tile falls back (tests: DDMI_VPROJ_UMAX; the kernel's capacity rules)
  unsigned* fb = nullptr;
  int fb_only = 0;     // (set by launch_vproj) the gathered kernel computes only the flagged (tile, half) pairs
  int usplit = 1;      // union form: K split over the 16 channel groups (1, 2, 4, 8, 16); partials in `part`
  unsigned* ucnt = nullptr;  // union form with usplit > 1: [tiles][2] arrival counters, zero between launches
};
bool vproj_supported(int C, int Cout, int H, int W);
size_t vproj_tiles(int B, int cap);
void launch_vproj(const VprojArgs& a, hipStream_t st);

// ----------------------------------------------------------------------------------------
// Bandwidth / small kernels (elementwise.hip)
// NCHW fp32 (B, C, H, W) -> NHWC padded to Cp channels (zero fill).
void launch_nchw_to_nhwc(const float* in, float* out, int B, int C, int H, int W, int Cp, hipStream_t st);
// 3x3 / stride 2 / pad 1 max pool, NHWC contiguous.
void launch_maxpool3x3s2(const float* in, float* out, int B, int H, int W, int C, int Ho, int Wo,
                         hipStream_t st);
// Adaptive average pool with exact integer windows (H % oh == 0, W % ow == 0), NHWC contiguous in;
// out (n, y, x, c) strided; optional add[y*ow + x][c] (broadcast over n).
void launch_avgpool(const float* in, int B, int H, int W, int C, int oh, int ow, View4 out,
                    const float* add, hipStream_t st);
// Bilinear resize, align_corners=False (PyTorch upsample_bilinear2d semantics):
// out[n,y,x,c] (= or +=) bilinear(in)[n,y,x,c]. ratio_h/ratio_w = in/out unless a scale factor is given.
void launch_bilinear(View4 in, int B, int Hi, int Wi, int C, View4 out, int Ho, int Wo, float ratio_h,
                     float ratio_w, int accumulate, hipStream_t st);
// Row LayerNorm (eps 1e-5): y[r] = LN(x[r] + res[r / res_div]) * g + b, then optional FiLM
// y = y * (1 + film_scale) + film_shift - one FiLM vector for every row, or (film_div > 0) the FiLM vectors of row
// group r / film_div at film_ld floats apart. C <= 2048. In-place allowed (y == x).
void launch_layernorm(const float* x, int64_t ldx, const float* res, int64_t ldres, int res_div,
                      const float* g, const float* b, const float* film_scale, const float* film_shift,
                      float* y, int64_t ldy, int rows, int C, hipStream_t st, int film_div = 0,
                      int64_t film_ld = 0);
// Fused GPT self-attention (attention.hip): y[b,t,h*hs..] = softmax(q.k^T / sqrt(hs)) v per
// (scene, head) from the packed projection qkv [B][T][3C]; y is [B][T][C]. T % 64 == 0, (T/4) % 8 == 0,
// T <= 512, hs in {16, ..., 512}.
// prec 0: fp32 MFMA; 1: f16x3 MFMA (three-way split scores), the f16x3 / bf16 modes
void launch_gpt_attention(const float* qkv, int B, int T, int C, int heads, float* y, int prec, hipStream_t st);
// Fused GPT block tail at C = 64 / 128 (gpt_tail.hip): x += proj(y); h = ln2(x); x += mlp(h); hb = lnn(x) in one
// launch over M token rows, f16x3 products bit-identical to the unfused conv_x3 / conv_x5 chain.
struct GptTailW {
  const uint16_t* wh = nullptr;  // pre-split fp16 hi / lo images [N][ldh] (weights.cpp prep_split)
  const uint16_t* wl = nullptr;
  const float* sinv = nullptr;   // per-output-channel inverse weight scale
  const float* bias = nullptr;
  int ldh = 0;
  float alpha = 1.0f;
};
struct GptTailArgs {
  const float* y = nullptr;  // [M][C] attention output
  float* x = nullptr;        // [M][C] residual stream, updated in place
  float* hb = nullptr;       // [M][C] lnn(x) out
  int M = 0, C = 0;
  GptTailW proj, up, down;   // [C][C], [4C][C], [C][4C]
  const float *ln2_g = nullptr, *ln2_b = nullptr, *lnn_g = nullptr, *lnn_b = nullptr;
  unsigned* flags = nullptr;
};
bool gpt_tail_supported(int C);
void launch_gpt_tail(const GptTailArgs& a, hipStream_t st);
// Row softmax of (scale * x), in place, rows of length L (<= 1024), row stride ld.
void launch_softmax_rows(float* x, int64_t ld, int rows, int L, float scale, hipStream_t st);
// dst[r][:] = src[r % nsrc][:] for r < rows (row length C, contiguous).
void launch_broadcast_rows(const float* src, int nsrc, float* dst, int rows, int C, hipStream_t st);
// y = act(x) elementwise, n elements; act 0 = mish, 1 = relu.
void launch_activation(const float* x, float* y, int64_t n, int act, hipStream_t st);
// out[i] = N(0, 1) draw number first + i of the Philox4x32-10 / Box-Muller stream keyed by seed (n, first % 4 == 0)
void launch_normal_philox(float* out, int64_t n, uint64_t seed, uint64_t first, hipStream_t st);

// ----------------------------------------------------------------------------------------
// Feature builder (features.hip): cams = B x 3 (l0, f0, r0) x H x W x 3 uint8 HWC -> out
// (B, 3, oh, ow) float NCHW; LiDAR planar xyz per scene at 3 * offs[b] -> (B, C, nb, nb) float.
void launch_camera_feature(const uint8_t* cams, int B, int H, int W, float* out, int oh, int ow, hipStream_t st);
void launch_lidar_feature(const float* xyz, const int64_t* offs, int B, int C, float* out, int nb, float lo,
                          float hi, int ppm, float max_h, float split_h, int hist_max, int64_t max_points,
                          hipStream_t st);

// ----------------------------------------------------------------------------------------
// Decoder kernels (decoder.hip)
// img = sqrt(a)*norm_odo(anchor) + sqrt(1-a)*noise; (B, Q, P, 2)
void launch_ddim_init(const float* anchor, const float* noise, float* img, int B, int QP, float sa,
                      float s1a, hipStream_t st);
// Uploads the sine-embedding frequency table (call once per device before launch_traj_embed).
void decoder_init_constants();
// pts = denorm_odo(clamp(img, -1, 1)); emb = gen_sineembed_for_position(pts, 64).flatten(-2)
void launch_traj_embed(const float* img, float* pts, float* emb, int rows, int P, hipStream_t st);
// SinusoidalPosEmb(dim) of a scalar timestep, written to out[dim].
void launch_timestep_embed(float t, float* out, int dim, hipStream_t st);
// GridSampleCrossBEVAttention core: per (scene, query): softmax over P logits, bilinear gather of
// value (NHWC, Hv x Wv x C, zero padding, align_corners=False) at P points, weighted sum -> out[C].
void launch_bev_sample_attn(const float* logits, const float* pts, const float* value, float* out,
                            int B, int Q, int P, int Hv, int Wv, int C, float inv_max_x,
                            float inv_max_y, hipStream_t st);
// Gathered form (decoder.hip): the (B*Q*P*4) tap pixels (or -1) of the points, and the sampling
// attention over a compact (B*Q*P*4, C) value array holding the conv at those taps.
void launch_bev_tap_rows(const float* pts, int* rows, int B, int Q, int P, int Hv, int Wv, float inv_max_x,
                         float inv_max_y, hipStream_t st);
// Deduplicated taps (one workgroup per scene, Hv * Wv <= 4096, else false and nothing launched):
// rows[b * Q*P*4 + j] = the scene's j-th distinct tap pixel (pixel order; -1 past its count),
// slots[tap] = the compact row holding the tap's pixel (-1 for zero padding).
bool launch_bev_tap_dedup(const float* pts, int* rows, int* slots, int B, int Q, int P, int Hv, int Wv,
                          float inv_max_x, float inv_max_y, hipStream_t st);
// slots == nullptr: row of tap t of point ip is ip * 4 + t (launch_bev_tap_rows layout)
void launch_bev_sample_attn_gathered(const float* logits, const float* pts, const float* vrows, const int* slots,
                                     float* out, int B, int Q, int P, int Hv, int Wv, int C, float inv_max_x,
                                     float inv_max_y, hipStream_t st);
// Small multi-head attention: out[b,i,h*hd+d] = sum_j softmax_j(q.k / sqrt(hd)) v. Lk <= 128, hd <= 64.
void launch_mha_small(const float* q, int64_t ldq, const float* k, const float* v, int64_t ldkv,
                      float* out, int64_t ldo, int B, int Lq, int Lk, int nh, int hd,
                      int64_t q_bstride, int64_t kv_bstride, int64_t o_bstride, hipStream_t st);
// reg (rows, P, 3) from the raw branch output r (rows, P*3): xy += pts, heading = tanh * pi;
// optionally also writes the cascade's next points (rows, P, 2).
void launch_reg_finalize(const float* r, const float* pts, float* reg, float* pts_next, int rows, int P,
                         hipStream_t st);
// img = DDIM.step(norm_odo(reg[..., :2]), t -> t-1, img), eta = 0, prediction 'sample', clip.
void launch_ddim_step(const float* reg, float* img, int rows, int P, float a_t, float a_prev,
                      hipStream_t st);
// argmax over Q cls logits per scene, gather reg[b, argmax] -> traj (B, P, 3); also writes index.
void launch_select_mode(const float* cls, const float* reg, float* traj, int* idx, int B, int Q, int P,
                        hipStream_t st);
// Agent head post-processing: states (rows, 5) in place: [0:2] = tanh*32, [2] = tanh*pi.
void launch_agent_post(float* states, int rows, hipStream_t st);

// ----------------------------------------------------------------------------------------
// Training-mode trajectory head / loss evaluator (train_loss.hip; transfuser_model_v2.py:520-576,
// multimodal_loss.py:119-168, transfuser_loss.py:28-29)
// per scene: sa = sqrt(ac[t]), s1a = sqrt(1 - ac[t]) (t clamped to [0, tmax))
void launch_train_coeffs(const int* t, const float* ac, float* sa, float* s1a, int B, int tmax, hipStream_t st);
// img = sa[b] * norm_odo(anchor) + s1a[b] * noise, (B, QP, 2)
void launch_train_noisy(const float* anchor, const float* noise, const float* sa, const float* s1a, float* img, int B,
                        int QP, hipStream_t st);
// SinusoidalPosEmb(dim) of every scene's integer timestep: out[B][dim]
void launch_timestep_embed_rows(const int* t, float* out, int B, int dim, hipStream_t st);
// LossComputer partials per scene: part[b] = (focal sum over the Q logits, L1 sum of the nearest-anchor mode)
void launch_traj_loss_scene(const float* reg, const float* cls, const float* target, const float* anchor, float* part,
                            int B, int Q, int P, hipStream_t st);
// out[0] = cls_w * mean focal + reg_w * mean L1 over the B scenes' partials (index order)
void launch_traj_loss_reduce(const float* part, float* out, int B, int Q, int P, float cls_w, float reg_w,
                             hipStream_t st);
// o[2] = o[0] + o[1] (the summed trajectory loss of the two decoder layers, forward_train :563-565)
void launch_add2(float* o, hipStream_t st);
// BEV-semantic cross entropy (mean over B x HW pixels) of NCHW logits against uint8 class ids; part holds
// bev_ce_partials(B, HW) floats
size_t bev_ce_partials(int B, int HW);
void launch_bev_ce(const float* logits, const uint8_t* target, float* part, float* out, int B, int C, int HW,
                   hipStream_t st);

}  // namespace ddmi
