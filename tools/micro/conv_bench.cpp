// Conv microbenchmark: the path's dominant conv shapes (B = 64 scenes, NHWC fp32) through
// ddmi::launch_conv_gemm in f16x3 mode (the kernel the runtime would pick; DDMI_X6 / DDMI_X5 env
// switches select variants) against the fp32-MFMA kernel on the same inputs.
// Prints one line per shape: device ms per launch (HIP events, median of reps), algorithmic TF/s,
// and max |f16x3 - fp32| / max |fp32|.
//   build: tools/micro/build_conv_bench.sh     run: tools/micro/conv_bench [reps] [shape-substring]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "common.h"
#include "weights.h"
#if defined(X5_STAMPS) || defined(X6_STAMPS)
#include <string>
extern "C" int dd_x5_stamps_read(unsigned long long* h, int n);
extern "C" int dd_x6_stamps_read(unsigned long long* h, int n);
#endif

using namespace ddmi;

struct Shape {
  const char* name;
  int B, H, W, Cin, Cout, k, s, res;
};

static const Shape kShapes[] = {
    {"img.l1.3x3", 64, 64, 256, 64, 64, 3, 1, 1},
    {"img.l2.3x3", 64, 32, 128, 128, 128, 3, 1, 1},
    {"img.l3.3x3", 64, 16, 64, 256, 256, 3, 1, 1},
    {"img.l4.3x3", 64, 8, 32, 512, 512, 3, 1, 1},
    {"lid.l1.3x3", 64, 64, 64, 64, 64, 3, 1, 1},
    {"lid.l2.3x3", 64, 32, 32, 128, 128, 3, 1, 1},
    {"lid.l3.3x3", 64, 16, 16, 256, 256, 3, 1, 1},
    {"value_proj", 64, 64, 64, 256, 256, 3, 1, 0},
    {"img.l2.s2", 64, 64, 256, 64, 128, 3, 2, 0},
    {"img.stem7", 64, 256, 1024, 4, 64, 7, 2, 0},
    {"gpt.mlp0", 64 * 320, 1, 1, 512, 2048, 1, 1, 0},
    {"gpt.mlp0.h", 16 * 256, 1, 1, 512, 2048, 1, 1, 0},   // 128 tiles: half the chip (shared-bandwidth probe)
    {"gpt.mlp0.q", 8 * 256, 1, 1, 512, 2048, 1, 1, 0},    // 64 tiles: a quarter
    {"gpt.qkv4", 64 * 320, 1, 1, 512, 1536, 1, 1, 0},
    {"gpt.mlp2", 64 * 320, 1, 1, 2048, 512, 1, 1, 1},
    {"gpt.proj4", 64 * 320, 1, 1, 512, 512, 1, 1, 1},
    {"gpt.mlp0s3", 64 * 320, 1, 1, 256, 1024, 1, 1, 0},
    {"gpt.mlp2s3", 64 * 320, 1, 1, 1024, 256, 1, 1, 1},
    {"gpt.qkv3", 64 * 320, 1, 1, 256, 768, 1, 1, 0},
    {"gpt.mlp0s2", 64 * 320, 1, 1, 128, 512, 1, 1, 0},
    {"gpt.qkv2", 64 * 320, 1, 1, 128, 384, 1, 1, 0},
    {"gpt.proj3", 64 * 320, 1, 1, 256, 256, 1, 1, 1},
    {"img.l4.s2", 64, 16, 64, 256, 512, 3, 2, 0},
    {"img.l4.ds", 64, 16, 64, 256, 512, 1, 2, 0},
    {"img.l2.ds", 64, 64, 256, 64, 128, 1, 2, 0},
    {"img.l3.s2", 64, 32, 128, 128, 256, 3, 2, 0},
    {"img.l3.ds", 64, 32, 128, 128, 256, 1, 2, 0},
    {"lid.l4.3x3", 64, 8, 8, 512, 512, 3, 1, 1},
    {"lid.l2.s2", 64, 64, 64, 64, 128, 3, 2, 0},
    {"lid.l3.s2", 64, 32, 32, 128, 256, 3, 2, 0},
    {"lid.l4.s2", 64, 16, 16, 256, 512, 3, 2, 0},
    {"lid.l3.ds", 64, 32, 32, 128, 256, 1, 2, 0},
    {"lid.l4.ds", 64, 16, 16, 256, 512, 1, 2, 0},
    // fixed-cost probes: the img.l2 / img.l3 tiles with the K walk halved / doubled
    {"fx.l3.c128", 64, 16, 64, 128, 256, 3, 1, 1},
    {"fx.l3.c512", 64, 16, 64, 512, 256, 3, 1, 1},
    {"fx.l2.c64", 64, 32, 128, 64, 128, 3, 1, 1},
    {"fx.l2.c256", 64, 32, 128, 256, 128, 3, 1, 1},
    {"fx.l2.nores", 64, 32, 128, 128, 128, 3, 1, 0},
    {"fx.l3.nores", 64, 16, 64, 256, 256, 3, 1, 0},
};

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const char* filt = argc > 2 ? argv[2] : nullptr;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  unsigned* flags;
  CK(hipMalloc(&flags, 4));
  printf("%-12s %9s %9s %8s %10s\n", "shape", "ms", "TF/s", "fp32_ms", "rel_err");
  for (const Shape& sh : kShapes) {
    if (filt && !strstr(sh.name, filt)) continue;
    const int pad = sh.k / 2;
    const int Ho = (sh.H + 2 * pad - sh.k) / sh.s + 1, Wo = (sh.W + 2 * pad - sh.k) / sh.s + 1;
    const size_t nin = (size_t)sh.B * sh.H * sh.W * sh.Cin, nout = (size_t)sh.B * Ho * Wo * sh.Cout;
    const int K = sh.k * sh.k * sh.Cin;
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> u01(0.f, 1.f);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> hin(nin), hw((size_t)sh.Cout * K), hb(sh.Cout), hres(sh.res ? nout : 0);
    for (auto& v : hin) v = u01(rng) * 2.f;  // post-ReLU-like activations
    const float ws = std::sqrt(2.f / K);
    for (auto& v : hw) v = nd(rng) * ws;
    for (auto& v : hb) v = nd(rng) * 0.1f;
    for (auto& v : hres) v = u01(rng);
    float *din, *dw, *db, *dres = nullptr, *dout, *dref;
    CK(hipMalloc(&din, nin * 4));
    CK(hipMalloc(&dw, hw.size() * 4));
    CK(hipMalloc(&db, hb.size() * 4));
    CK(hipMalloc(&dout, nout * 4));
    CK(hipMalloc(&dref, nout * 4));
    CK(hipMemcpy(din, hin.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    if (sh.res) {
      CK(hipMalloc(&dres, nout * 4));
      CK(hipMemcpy(dres, hres.data(), nout * 4, hipMemcpyHostToDevice));
    }
    Arena ar;
    const SplitW x = prep_split(ar, hw.data(), sh.Cout, K);
    ar.upload();
    ConvArgs a;
    a.in = din;
    a.in_sw = sh.Cin;
    a.in_sh = (int64_t)sh.W * sh.Cin;
    a.in_sn = (int64_t)sh.H * sh.W * sh.Cin;
    a.H = sh.H;
    a.W = sh.W;
    a.Cin = sh.Cin;
    a.wgt = dw;
    a.ldb = K;
    a.bias = db;
    a.Nimg = sh.B;
    a.Ho = Ho;
    a.Wo = Wo;
    a.Cout = sh.Cout;
    a.out = dref;
    a.out_sw = sh.Cout;
    a.out_sh = (int64_t)Wo * sh.Cout;
    a.out_sn = (int64_t)Ho * Wo * sh.Cout;
    a.res = dres;
    a.res_sw = a.out_sw;
    a.res_sh = a.out_sh;
    a.res_sn = a.out_sn;
    a.KH = a.KW = sh.k;
    a.stride = sh.s;
    a.pad = pad;
    a.relu = 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const ConvArgs& c) {
      for (int i = 0; i < 3; ++i) launch_conv_gemm(c, st);
      std::vector<float> ts;
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0, st));
        launch_conv_gemm(c, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      return ts[ts.size() / 2];
    };
    const float ms32 = timed(a);  // fp32 MFMA reference
    ConvArgs b = a;
    b.out = dout;
    b.wh = reinterpret_cast<const uint16_t*>(ar.ptr(x.hi));
    b.wl = reinterpret_cast<const uint16_t*>(ar.ptr(x.lo));
    b.wsinv = ar.ptr(x.sinv);
    b.ldh = x.ldh;
    b.flags = flags;
    CK(hipMemset(dout, 0xff, nout * 4));  // NaN fill: a skipped output shows up
    const float ms = timed(b);
    CK(hipStreamSynchronize(st));
#if defined(X5_STAMPS) || defined(X6_STAMPS)
    {  // per-workgroup phase stamps of the last launch (diagnostic library, DDMI_BUILD_VARIANT=x5st / x6st)
#ifdef X5_STAMPS
      const char* kname = "conv_x5";
      auto rd = dd_x5_stamps_read;
      const int NWG = 4096;  // g_x5_st
#else
      const char* kname = "conv_x6";
      auto rd = dd_x6_stamps_read;
      const int NWG = 8192;  // g_x6_st
#endif
      std::vector<unsigned long long> t(NWG * 4);
      if (rd(t.data(), NWG * 4) == 0 && std::string(last_conv_kernel()) == kname) {
        int n = 0;
        double pro = 0, mainl = 0, epi = 0;
        for (int w = 0; w < NWG; ++w) {
          if (!t[w * 4 + 3] || t[w * 4 + 3] < t[w * 4]) continue;
          ++n;
          pro += t[w * 4 + 1] - t[w * 4];
          mainl += t[w * 4 + 2] - t[w * 4 + 1];
          epi += t[w * 4 + 3] - t[w * 4 + 2];
        }
        if (n)
          printf("  stamps: %d WGs  per WG: prologue %.0f  main %.0f  epilogue %.0f (s_memtime ticks)\n", n, pro / n,
                 mainl / n, epi / n);
      }
    }
#endif
    std::vector<float> ho(nout), hr(nout);
    CK(hipMemcpy(ho.data(), dout, nout * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), dref, nout * 4, hipMemcpyDeviceToHost));
    double mx = 0, md = 0;
    for (size_t i = 0; i < nout; ++i) {
      mx = std::max(mx, (double)std::fabs(hr[i]));
      const double d = std::fabs((double)ho[i] - hr[i]);
      md = std::isfinite(d) ? std::max(md, d) : INFINITY;
    }
    const double fl = 2.0 * sh.B * Ho * Wo * (double)sh.Cout * K * (sh.Cin == 4 ? 3.0 / 4.0 : 1.0);
    printf("%-12s %9.4f %9.1f %8.4f %10.3e\n", sh.name, ms, fl / ms * 1e-9, ms32, md / mx);
    fflush(stdout);
    (void)hipFree(din);
    (void)hipFree(dw);
    (void)hipFree(db);
    (void)hipFree(dout);
    (void)hipFree(dref);
    if (dres) (void)hipFree(dres);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  return 0;
}
