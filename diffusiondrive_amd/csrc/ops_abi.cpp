// Single-kernel C-ABI entry points (include/ddmi.h, "single-op entry points"): used by the GPU
// parity tests to check each kernel in isolation against PyTorch-CPU fp32 on the same inputs.
#include <cmath>
#include <string>

#include "../../include/ddmi.h"
#include "common.h"
#include "decoder_mk.h"
#include "weights.h"
#include <vector>

namespace {
thread_local std::string g_op_err;

template <class F>
int op_guard(F&& f) {
  try {
    f();
    return DD_OK;
  } catch (const std::invalid_argument& e) {
    g_op_err = e.what();
    return DD_ERR_INVALID;
  } catch (const std::exception& e) {
    g_op_err = e.what();
    return DD_ERR_RUNTIME;
  }
}
hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }
}  // namespace

using namespace ddmi;

extern "C" {

const char* dd_op_last_error(void) { return g_op_err.c_str(); }

const char* dd_op_last_kernel(void) { return last_conv_config(); }

int dd_op_mk_linear(const float* A, int K, const float* wgt, const float* bias, float* out, int N, void* stream) {
  return op_guard([&] {
    std::vector<float> hw((size_t)N * K);
    DD_HIP_CHECK(hipStreamSynchronize(S(stream)));
    DD_HIP_CHECK(hipMemcpy(hw.data(), wgt, hw.size() * sizeof(float), hipMemcpyDeviceToHost));
    std::vector<_Float16> pk;
    std::vector<float> sinv;
    pack_mk_weights(hw.data(), N, K, pk, sinv);
    Arena ar;
    const size_t wo = ar.add(reinterpret_cast<const float*>(pk.data()), pk.size() / 2);
    const size_t so = ar.add(sinv);
    ar.upload();
    MkLin m;
    m.w = reinterpret_cast<const uint4*>(ar.ptr(wo));
    m.s = ar.ptr(so);
    m.b = bias;
    m.nks = K / 16;
    launch_mk_linear_test(A, K, m, N, out, S(stream));
    DD_HIP_CHECK(hipStreamSynchronize(S(stream)));
  });
}

int dd_op_bevproj(const float* p3, int64_t p3_ld, const float* kvp, const float* wgt, const float* bias,
                  const float* ln_g, const float* ln_b, float* out, int B, int H, int W, int Hk, int Wk, void* stream) {
  return op_guard([&] {
    if (!bevproj_supported(256, 64, H, W, Hk, Wk)) throw std::invalid_argument("dd_op_bevproj: unsupported shape");
    std::vector<float> hw((size_t)256 * 64);
    DD_HIP_CHECK(hipStreamSynchronize(S(stream)));
    DD_HIP_CHECK(hipMemcpy(hw.data(), wgt, hw.size() * sizeof(float), hipMemcpyDeviceToHost));
    std::vector<_Float16> pk;
    std::vector<float> sinv;
    pack_mk_weights(hw.data(), 256, 64, pk, sinv);
    Arena ar;
    const size_t wo = ar.add(reinterpret_cast<const float*>(pk.data()), pk.size() / 2);
    const size_t so = ar.add(sinv);
    ar.upload();
    BevProjArgs a;
    a.p3 = p3;
    a.p3_ld = p3_ld;
    a.kvp = kvp;
    a.w = reinterpret_cast<const uint4*>(ar.ptr(wo));
    a.s = ar.ptr(so);
    a.bias = bias;
    a.g = ln_g;
    a.beta = ln_b;
    a.out = out;
    a.B = B;
    a.H = H;
    a.W = W;
    a.Hk = Hk;
    a.Wk = Wk;
    launch_bevproj(a, S(stream));
    DD_HIP_CHECK(hipStreamSynchronize(S(stream)));
  });
}

int dd_op_conv2d(const float* in, int B, int H, int W, int Cin, const float* wgt, const float* bias, const float* res,
                 float* out, int Cout, int KH, int KW, int stride, int pad, int relu, void* stream) {
  return op_guard([&] {
    ConvArgs a;
    a.in = in;
    a.in_sw = Cin;
    a.in_sh = (int64_t)W * Cin;
    a.in_sn = (int64_t)H * W * Cin;
    a.H = H;
    a.W = W;
    a.Cin = Cin;
    a.wgt = wgt;
    a.ldb = (int64_t)KH * KW * Cin;
    a.bias = bias;
    a.Nimg = B;
    a.Ho = (H + 2 * pad - KH) / stride + 1;
    a.Wo = (W + 2 * pad - KW) / stride + 1;
    a.Cout = Cout;
    a.out = out;
    a.out_sw = Cout;
    a.out_sh = (int64_t)a.Wo * Cout;
    a.out_sn = (int64_t)a.Ho * a.Wo * Cout;
    a.res = res;
    a.res_sw = a.out_sw;
    a.res_sh = a.out_sh;
    a.res_sn = a.out_sn;
    a.KH = KH;
    a.KW = KW;
    a.stride = stride;
    a.pad = pad;
    a.relu = relu;
    launch_conv_gemm(a, S(stream));
  });
}

int dd_op_conv2d_x3(const float* in, int B, int H, int W, int Cin, const float* wgt, const float* bias,
                    const float* res, float* out, int Cout, int KH, int KW, int stride, int pad, int relu, int prec,
                    unsigned* flags, void* stream) {
  return op_guard([&] {
    // split the (device) fp32 weights on the host exactly as dd_create does (weights.cpp:prep_split)
    const int K = KH * KW * Cin;
    std::vector<float> hw((size_t)Cout * K);
    DD_HIP_CHECK(hipStreamSynchronize(S(stream)));
    DD_HIP_CHECK(hipMemcpy(hw.data(), wgt, hw.size() * sizeof(float), hipMemcpyDeviceToHost));
    Arena ar;
    const SplitW x = prep_split(ar, hw.data(), Cout, K);
    ar.upload();
    ConvArgs a;
    a.in = in;
    a.in_sw = Cin;
    a.in_sh = (int64_t)W * Cin;
    a.in_sn = (int64_t)H * W * Cin;
    a.H = H;
    a.W = W;
    a.Cin = Cin;
    a.wgt = wgt;
    a.ldb = K;
    a.bias = bias;
    a.Nimg = B;
    a.Ho = (H + 2 * pad - KH) / stride + 1;
    a.Wo = (W + 2 * pad - KW) / stride + 1;
    a.Cout = Cout;
    a.out = out;
    a.out_sw = Cout;
    a.out_sh = (int64_t)a.Wo * Cout;
    a.out_sn = (int64_t)a.Ho * a.Wo * Cout;
    a.res = res;
    a.res_sw = a.out_sw;
    a.res_sh = a.out_sh;
    a.res_sn = a.out_sn;
    a.KH = KH;
    a.KW = KW;
    a.stride = stride;
    a.pad = pad;
    a.relu = relu;
    if (prec != 0 && prec != 1) throw std::invalid_argument("prec must be 0 (f16x3) or 1 (bf16)");
    a.prec = prec;
    a.wh = reinterpret_cast<const uint16_t*>(ar.ptr(prec ? x.b16 : x.hi));
    a.wl = reinterpret_cast<const uint16_t*>(ar.ptr(x.lo));
    a.wsinv = ar.ptr(x.sinv);
    a.ldh = x.ldh;
    a.flags = flags;
    // K-split scratch, as the forward provides it (runtime.cpp: conv): small grids may take conv_x3's split form
    const int64_t mo = (int64_t)B * a.Ho * a.Wo * Cout;
    float* part = nullptr;
    if (prec == 0 && mo <= (1 << 20)) {
      DD_HIP_CHECK(hipMalloc(&part, (size_t)(8 * mo) * sizeof(float)));
      a.split_part = part;
      a.split_cap = 8 * mo;
    }
    launch_conv_gemm(a, S(stream));
    const hipError_t e = hipStreamSynchronize(S(stream));  // the split images die with `ar`
    if (part) DD_HIP_CHECK(hipFree(part));
    DD_HIP_CHECK(e);
  });
}

static int dd_op_stem_pool_impl(const float* in, int src_c, int B, int H, int W, const float* wgt, const float* bias,
                                float* out, int prec, unsigned* flags, void* stream);

int dd_op_stem_pool_x3(const float* in, int B, int H, int W, const float* wgt, const float* bias, float* out,
                       unsigned* flags, void* stream) {
  return dd_op_stem_pool(in, B, H, W, wgt, bias, out, 0, flags, stream);
}

int dd_op_stem_pool_nchw(const float* in, int B, int C, int H, int W, const float* wgt, const float* bias, float* out,
                         int prec, unsigned* flags, void* stream) {
  if (C < 1 || C > 3) return op_guard([&] { throw std::invalid_argument("stem_pool_nchw: C must be 1..3"); });
  return dd_op_stem_pool_impl(in, C, B, H, W, wgt, bias, out, prec, flags, stream);
}

int dd_op_stem_pool(const float* in, int B, int H, int W, const float* wgt, const float* bias, float* out, int prec,
                    unsigned* flags, void* stream) {
  return dd_op_stem_pool_impl(in, 0, B, H, W, wgt, bias, out, prec, flags, stream);
}

static int dd_op_stem_pool_impl(const float* in, int src_c, int B, int H, int W, const float* wgt, const float* bias,
                                float* out, int prec, unsigned* flags, void* stream) {
  return op_guard([&] {
    if (prec != 0 && prec != 1) throw std::invalid_argument("stem_pool: prec must be 0 (f16x3) or 1 (bf16)");
    const int Cin = 4, Cout = 64, K = 7 * 7 * Cin;
    std::vector<float> hw((size_t)Cout * K);
    DD_HIP_CHECK(hipStreamSynchronize(S(stream)));
    DD_HIP_CHECK(hipMemcpy(hw.data(), wgt, hw.size() * sizeof(float), hipMemcpyDeviceToHost));
    Arena ar;
    const SplitW x = prep_split(ar, hw.data(), Cout, K);
    ar.upload();
    ConvArgs a;
    a.in = in;
    a.in_sw = Cin;
    a.in_sh = (int64_t)W * Cin;
    a.in_sn = (int64_t)H * W * Cin;
    a.H = H;
    a.W = W;
    a.Cin = Cin;
    a.wgt = wgt;
    a.ldb = K;
    a.bias = bias;
    a.Nimg = B;
    a.Ho = (H + 6 - 7) / 2 + 1;
    a.Wo = (W + 6 - 7) / 2 + 1;
    a.Cout = Cout;
    a.KH = a.KW = 7;
    a.stride = 2;
    a.pad = 3;
    a.relu = 1;
    a.prec = prec;
    a.wh = reinterpret_cast<const uint16_t*>(ar.ptr(prec ? x.b16 : x.hi));
    a.wl = reinterpret_cast<const uint16_t*>(ar.ptr(x.lo));
    a.wsinv = ar.ptr(x.sinv);
    a.ldh = x.ldh;
    a.flags = flags;
    const int hp = (a.Ho + 2 - 3) / 2 + 1, wp = (a.Wo + 2 - 3) / 2 + 1;
    // NCHW input of src_c channels: the kernel reads its address from a device word
    const float** word = nullptr;
    if (src_c) {
      DD_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&word), sizeof(const float*)));
      DD_HIP_CHECK(hipMemcpy(word, &in, sizeof(const float*), hipMemcpyHostToDevice));
    }
    bool ok = false;
    try {
      ok = launch_stem_pool(a, out, hp, wp, S(stream), src_c ? word : nullptr, src_c);
      DD_HIP_CHECK(hipStreamSynchronize(S(stream)));  // the split images die with `ar`
    } catch (...) {
      if (word) (void)hipFree(word);
      throw;
    }
    if (word) DD_HIP_CHECK(hipFree(word));
    if (!ok) throw std::invalid_argument("stem_pool: shape not supported");
  });
}

int dd_build_camera(const uint8_t* cams, int B, int src_h, int src_w, float* out, int out_h, int out_w,
                    void* stream) {
  return op_guard([&] {
    if (!cams || !out) throw std::invalid_argument("null pointer");
    launch_camera_feature(cams, B, src_h, src_w, out, out_h, out_w, S(stream));
  });
}

int dd_build_lidar(const float* xyz, const int64_t* offsets, int B, int channels, float* out, int resolution,
                   float range_lo, float range_hi, int pixels_per_meter, float max_height, float split_height,
                   int hist_max, long long max_points, void* stream) {
  return op_guard([&] {
    if (!offsets || !out || (!xyz && max_points > 0)) throw std::invalid_argument("null pointer");
    launch_lidar_feature(xyz, offsets, B, channels, out, resolution, range_lo, range_hi, pixels_per_meter,
                         max_height, split_height, hist_max, max_points, S(stream));
  });
}

int dd_op_gemm(const float* A, int M, int K, const float* W, const float* bias, const float* res, float* C, int N,
               int relu, void* stream) {
  return op_guard([&] {
    ConvArgs a;
    a.in = A;
    a.in_sn = K;
    a.Cin = K;
    a.wgt = W;
    a.ldb = K;
    a.bias = bias;
    a.res = res;
    a.res_sn = N;
    a.out = C;
    a.out_sn = N;
    a.Nimg = M;
    a.Cout = N;
    a.relu = relu;
    launch_conv_gemm(a, S(stream));
  });
}

int dd_op_gemm_batched(const float* A, const float* Bm, float* C, int batch, int M, int N, int K, int kn,
                       void* stream) {
  return op_guard([&] {
    ConvArgs a;
    a.in = A;
    a.in_sn = K;
    a.Cin = K;
    a.wgt = Bm;
    a.ldb = kn ? N : K;
    a.b_kn = kn;
    a.out = C;
    a.out_sn = N;
    a.Nimg = M;
    a.Cout = N;
    a.batch = batch;
    a.zdiv = 1;
    a.in_z1 = (int64_t)M * K;
    a.w_z1 = (int64_t)K * N;
    a.out_z1 = (int64_t)M * N;
    launch_conv_gemm(a, S(stream));
  });
}

int dd_op_layernorm(const float* x, const float* res, int res_div, const float* g, const float* b,
                    const float* film_scale, const float* film_shift, float* y, int rows, int C, void* stream) {
  return op_guard([&] {
    launch_layernorm(x, C, res, C, res_div, g, b, film_scale, film_shift, y, C, rows, C, S(stream));
  });
}

int dd_bev_semantic_loss(const float* logits, const unsigned char* target, int B, int C, int H, int W, float* work,
                         float* loss, void* stream) {
  return op_guard([&] {
    if (!logits || !target || !work || !loss || B < 1 || C < 1 || C > 255 || H < 1 || W < 1)
      throw std::invalid_argument("dd_bev_semantic_loss: null pointer or bad shape");
    launch_bev_ce(logits, target, work, loss, B, C, H * W, S(stream));
  });
}

size_t dd_bev_semantic_loss_work(int B, int H, int W) { return bev_ce_partials(B, H * W); }

int dd_op_softmax_rows(float* x, int rows, int L, float scale, void* stream) {
  return op_guard([&] { launch_softmax_rows(x, L, rows, L, scale, S(stream)); });
}

int dd_op_bilinear(const float* in, int B, int Hi, int Wi, int C, float* out, int Ho, int Wo, void* stream) {
  return op_guard([&] {
    View4 a{const_cast<float*>(in), (int64_t)Hi * Wi * C, (int64_t)Wi * C, C, 1};
    View4 o{out, (int64_t)Ho * Wo * C, (int64_t)Wo * C, C, 1};
    launch_bilinear(a, B, Hi, Wi, C, o, Ho, Wo, (float)Hi / (float)Ho, (float)Wi / (float)Wo, 0, S(stream));
  });
}

int dd_op_bilinear_add(const float* in, int B, int Hi, int Wi, int C, float* out, int Ho, int Wo, void* stream) {
  return op_guard([&] {
    View4 a{const_cast<float*>(in), (int64_t)Hi * Wi * C, (int64_t)Wi * C, C, 1};
    View4 o{out, (int64_t)Ho * Wo * C, (int64_t)Wo * C, C, 1};
    launch_bilinear(a, B, Hi, Wi, C, o, Ho, Wo, (float)Hi / (float)Ho, (float)Wi / (float)Wo, 1, S(stream));
  });
}

int dd_op_maxpool3x3s2(const float* in, int B, int H, int W, int C, float* out, void* stream) {
  return op_guard([&] {
    const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
    launch_maxpool3x3s2(in, out, B, H, W, C, Ho, Wo, S(stream));
  });
}

int dd_op_avgpool(const float* in, int B, int H, int W, int C, int oh, int ow, float* out, void* stream) {
  return op_guard([&] {
    View4 o{out, (int64_t)oh * ow * C, (int64_t)ow * C, C, 1};
    launch_avgpool(in, B, H, W, C, oh, ow, o, nullptr, S(stream));
  });
}

int dd_op_bev_sample_attn(const float* logits, const float* pts, const float* value, float* out, int B, int Q, int P,
                          int Hv, int Wv, int C, void* stream) {
  return op_guard([&] {
    launch_bev_sample_attn(logits, pts, value, out, B, Q, P, Hv, Wv, C, 1.0f / 32.0f, 1.0f / 32.0f, S(stream));
  });
}

int dd_op_mha_small(const float* q, const float* k, const float* v, float* out, int B, int Lq, int Lk, int nh, int hd,
                    void* stream) {
  return op_guard([&] {
    const int d = nh * hd;
    launch_mha_small(q, d, k, v, d, out, d, B, Lq, Lk, nh, hd, (int64_t)Lq * d, (int64_t)Lk * d, (int64_t)Lq * d,
                     S(stream));
  });
}

int dd_op_gpt_attention(const float* qkv, float* y, int B, int T, int C, int heads, int prec, void* stream) {
  return op_guard([&] { launch_gpt_attention(qkv, B, T, C, heads, y, prec, S(stream)); });
}

}  // extern "C"
