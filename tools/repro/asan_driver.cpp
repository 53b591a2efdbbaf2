// Host-AddressSanitizer driver of the C ABI (Handle lifetime): the library's sources compiled
// into this executable with -Xarch_host -fsanitize=address (device code untouched), driven through a handle history
// like the GPU test suite's - handles created and destroyed in every gemm mode, batch sizes 1 / 4 / 8, heads on and
// off, single-stream graphs on a caller stream, the training forward, taps and numerics flags - beside one long-lived
// handle replayed every iteration. A heap overflow or use-after-free in the host code is reported by ASan and ends
// the run; a clean run prints "asan_driver: ... no error".
//
//   asan_driver <weights.ddw1> <iterations>      (weights: python -c 'pack_blob(seeded_state_dict(...))' > file)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <vector>

#include "ddmi.h"

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(3);                                                                           \
    }                                                                                         \
  } while (0)
#define DD(x)                                                                        \
  do {                                                                               \
    int r_ = (x);                                                                    \
    if (r_ != 0) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, r_, dd_last_error()); \
      std::exit(4);                                                                  \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: asan_driver <weights.ddw1> <iterations>\n");
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (blob.size() < 8) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  const int iters = std::atoi(argv[2]);
  dd_config cfg;
  dd_default_config(&cfg);
  const int BM = 8, Q = cfg.num_modes, P = cfg.num_poses;
  const size_t ncam = (size_t)BM * 3 * cfg.cam_h * cfg.cam_w, nlid = (size_t)BM * cfg.lidar_channels * cfg.lidar_h * cfg.lidar_w;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::normal_distribution<float> nrm(0.f, 1.f);
  auto up = [&](size_t n, bool normal) {
    std::vector<float> h(n);
    for (auto& v : h) v = normal ? nrm(rng) : u(rng);
    float* d = nullptr;
    CK(hipMalloc(&d, n * sizeof(float)));
    CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    return d;
  };
  float* cam = up(ncam, false);
  float* lid = up(nlid, false);
  float* st = up((size_t)BM * 8, true);
  float* nz = up((size_t)BM * Q * P * 2, true);
  float* tgt = up((size_t)BM * P * 3, true);
  int* tt = nullptr;
  {
    std::vector<int> h(BM);
    for (int b = 0; b < BM; ++b) h[b] = (b * 7) % 50;
    CK(hipMalloc(&tt, BM * sizeof(int)));
    CK(hipMemcpy(tt, h.data(), BM * sizeof(int), hipMemcpyHostToDevice));
  }
  float *traj = nullptr, *modes = nullptr, *cls = nullptr, *sem = nullptr, *ags = nullptr, *agl = nullptr, *loss = nullptr;
  float *reg2[2] = {nullptr, nullptr}, *cls2[2] = {nullptr, nullptr};
  CK(hipMalloc(&traj, (size_t)BM * P * 3 * 4));
  CK(hipMalloc(&modes, (size_t)BM * Q * P * 3 * 4));
  CK(hipMalloc(&cls, (size_t)BM * Q * 4));
  CK(hipMalloc(&sem, (size_t)BM * 7 * (cfg.lidar_h / 2) * cfg.lidar_w * 4));
  CK(hipMalloc(&ags, (size_t)BM * 30 * 5 * 4));
  CK(hipMalloc(&agl, (size_t)BM * 30 * 4));
  CK(hipMalloc(&loss, 3 * 4));
  for (int l = 0; l < 2; ++l) {
    CK(hipMalloc(&reg2[l], (size_t)BM * Q * P * 3 * 4));
    CK(hipMalloc(&cls2[l], (size_t)BM * Q * 4));
  }
  hipStream_t caller;
  CK(hipStreamCreateWithFlags(&caller, hipStreamNonBlocking));

  dd_handle* keep = nullptr;
  DD(dd_create(&cfg, blob.data(), blob.size(), 0, &keep));
  DD(dd_set_gemm_mode(keep, DD_GEMM_F16X3));
  std::vector<float> host((size_t)BM * P * 3);
  for (int i = 0; i < iters; ++i) {
    const int B = (int[]){1, 4, 8}[i % 3];
    const int mode = (int[]){DD_GEMM_F16X3, DD_GEMM_FP32, DD_GEMM_BF16}[(i / 3) % 3];
    dd_outputs o{};
    o.trajectory = traj;
    o.poses_reg = modes;
    o.poses_cls = cls;
    if (i % 2) {
      o.bev_semantic_map = sem;
      o.agent_states = ags;
      o.agent_labels = agl;
    }
    dd_handle* h = nullptr;
    DD(dd_create(&cfg, blob.data(), blob.size(), 0, &h));
    DD(dd_set_gemm_mode(h, mode));
    for (int r = 0; r < 3; ++r) DD(dd_forward_ex(h, cam, lid, st, (r & 1) ? nullptr : nz, B, 2, &o, nullptr));
    if (i % 4 == 0) {  // a batches-in-flight lane: single-stream graphs replayed on the caller's stream
      DD(dd_set_streams(h, 1));
      for (int r = 0; r < 3; ++r) DD(dd_forward_ex(h, cam, lid, st, nz, B, 2, &o, caller));
      CK(hipStreamSynchronize(caller));
      DD(dd_set_streams(h, 2));
      DD(dd_forward_ex(h, cam, lid, st, nz, B, 2, &o, nullptr));
    }
    if (i % 5 == 0) {  // the loss evaluator
      dd_train_outputs t{};
      t.trajectory = traj;
      t.poses_reg[0] = reg2[0];
      t.poses_reg[1] = reg2[1];
      t.poses_cls[0] = cls2[0];
      t.poses_cls[1] = cls2[1];
      t.loss = loss;
      for (int r = 0; r < 2; ++r) DD(dd_forward_train(h, cam, lid, st, nz, tt, tgt, B, 10.f, 8.f, &t, nullptr));
    }
    unsigned flags = 0;
    DD(dd_numerics_flags(h, &flags, 1));
    size_t got = 0;
    DD(dd_tap(h, "trajectory", nullptr, 0, &got, nullptr));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(host.data(), traj, (size_t)B * P * 3 * 4, hipMemcpyDeviceToHost));
    DD(dd_forward_ex(keep, cam, lid, st, nz, 4, 2, &o, nullptr));  // the long-lived handle between the others
    DD(dd_destroy(h));
    CK(hipDeviceSynchronize());
    std::printf("iter %d ok (B %d, mode %d, heads %d, flags %u, traj[0] %.4f)\n", i, B, mode, i % 2, flags, host[0]);
    std::fflush(stdout);
  }
  DD(dd_destroy(keep));
  CK(hipStreamDestroy(caller));
  std::printf("asan_driver: %d iterations, no error\n", iters);
  return 0;
}
