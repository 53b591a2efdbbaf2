// Minimal reproducer for the round-3 host segfault inside hipGraphLaunch (Handle lifetime):
// the ddmi handle lifecycle with trivial kernels and nothing else - per handle two non-blocking streams, events, one
// buffer; the forward captured once per handle (two-stream fork / join on the handle's own streams after an event
// hand-off from the caller's stream, or single-stream directly on a long-lived caller stream), replayed, then the
// handle torn down in runtime.cpp ~Model's order (sync, exec destroy, events, streams, buffer).
//
//   graph_churn <iterations> <pool 0|1> <kernels per branch> [all 0|1] [forks] [memset 0|1]
//
// pool 1 keeps destroyed handles' streams for the next handles (runtime.cpp's process-wide pool), pool 0 destroys
// them. all 1: no stream outlives an iteration (the caller streams and the long-lived handle are re-created every
// iteration too), so the runtime's hardware queues - GPU_MAX_HW_QUEUES, shared round-robin by streams - can be
// released and re-created between handles. forks: fork / join pairs to the side stream per captured body (the
// forward's LiDAR-trunk, time-MLP, tf-decoder and heads branches all fork to one side stream); memset 1: a
// hipMemsetAsync node on each branch. Prints one line per 25 iterations; a segfault ends the process (the
// driving script reports the exit code).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(3);                                                                 \
    }                                                                               \
  } while (0)

__global__ void k_add(float* p, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + v;
}

static bool g_pool = true;
static int g_forks = 1;
static bool g_memset = false;
static std::vector<hipStream_t> g_streams;

static hipStream_t take_stream() {
  if (g_pool && !g_streams.empty()) {
    hipStream_t s = g_streams.back();
    g_streams.pop_back();
    return s;
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}

static void give_stream(hipStream_t s) {
  CK(hipStreamSynchronize(s));
  if (g_pool) g_streams.push_back(s);
  else CK(hipStreamDestroy(s));
}

struct Handle {
  hipStream_t s_main = nullptr, s_side = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  std::vector<hipEvent_t> fj;
  hipGraphExec_t ex = nullptr;
  float* buf = nullptr;
  int n = 1 << 16, K = 64, calls = 0;
  bool single = false;

  Handle(bool single_, int K_) : K(K_), single(single_) {
    s_main = take_stream();
    s_side = take_stream();
    CK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_out, hipEventDisableTiming));
    fj.resize(2 * g_forks);
    for (auto& e : fj) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipMalloc(&buf, 2 * n * sizeof(float)));
    CK(hipMemsetAsync(buf, 0, 2 * n * sizeof(float), s_main));
    CK(hipStreamSynchronize(s_main));
  }
  void body(hipStream_t st) {
    const dim3 g((n + 255) / 256), b(256);
    if (single) {
      for (int k = 0; k < 2 * K; ++k) hipLaunchKernelGGL(k_add, g, b, 0, st, buf + (k & 1) * n, n, 1.0f);
      return;
    }
    for (int f = 0; f < g_forks; ++f) {
      CK(hipEventRecord(fj[2 * f], st));
      CK(hipStreamWaitEvent(s_side, fj[2 * f], 0));
      if (g_memset) {
        CK(hipMemsetAsync(buf + n, 0, 1024, s_side));
        CK(hipMemsetAsync(buf, 0, 1024, st));
      }
      for (int k = 0; k < K / g_forks; ++k) {
        hipLaunchKernelGGL(k_add, g, b, 0, st, buf, n, 1.0f);
        hipLaunchKernelGGL(k_add, g, b, 0, s_side, buf + n, n, 2.0f);
      }
      CK(hipEventRecord(fj[2 * f + 1], s_side));
      CK(hipStreamWaitEvent(st, fj[2 * f + 1], 0));
    }
  }
  void forward(hipStream_t caller) {
    const bool direct = single && caller != nullptr;
    hipStream_t st = direct ? caller : s_main;
    if (!direct) {
      CK(hipEventRecord(ev_in, caller));
      CK(hipStreamWaitEvent(s_main, ev_in, 0));
    }
    if (calls++ == 0) {
      body(st);  // eager first call
    } else {
      if (!ex) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        body(st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      CK(hipGraphLaunch(ex, st));
    }
    CK(hipEventRecord(ev_out, st));
    if (!direct) CK(hipStreamWaitEvent(caller, ev_out, 0));
  }
  ~Handle() {
    (void)hipEventSynchronize(ev_out);
    (void)hipStreamSynchronize(s_main);
    (void)hipStreamSynchronize(s_side);
    if (ex) CK(hipGraphExecDestroy(ex));
    CK(hipEventDestroy(ev_in));
    CK(hipEventDestroy(ev_out));
    for (auto& e : fj) CK(hipEventDestroy(e));
    give_stream(s_main);
    give_stream(s_side);
    CK(hipFree(buf));
  }
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  g_pool = argc > 2 ? atoi(argv[2]) != 0 : true;
  const int K = argc > 3 ? atoi(argv[3]) : 64;
  const bool all = argc > 4 && atoi(argv[4]) != 0;
  g_forks = argc > 5 ? atoi(argv[5]) : 1;
  g_memset = argc > 6 && atoi(argv[6]) != 0;
  if (g_forks < 1 || g_forks > K) {
    std::fprintf(stderr, "forks must be in [1, kernels per branch]\n");
    return 2;
  }
  CK(hipSetDevice(0));
  hipStream_t callers[3];
  for (auto& s : callers) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));  // torch's pooled streams
  Handle* keep = new Handle(false, K);  // a long-lived two-stream handle (the tests' module-scoped model)
  for (int i = 0; i < iters; ++i) {
    if (all && i > 0) {  // nothing outlives the iteration: every stream of the process is re-created
      delete keep;
      for (auto& s : callers) CK(hipStreamDestroy(s));
      CK(hipDeviceSynchronize());
      for (auto& s : callers) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      keep = new Handle(false, K);
    }
    {  // three lanes in flight: the first a two-stream handle on the null stream, two single-stream clones
      Handle a(false, K), b(true, K), c(true, K);
      for (int r = 0; r < 4; ++r) {
        a.forward(nullptr);
        b.forward(callers[(i + 1) % 3]);
        c.forward(callers[(i + 2) % 3]);
      }
      CK(hipDeviceSynchronize());
    }
    {  // then a fresh two-stream handle, and the long-lived one replayed
      Handle d(false, K);
      for (int r = 0; r < 3; ++r) d.forward(nullptr);
      keep->forward(nullptr);
      CK(hipDeviceSynchronize());
    }
    if (i % 25 == 0) {
      std::printf("iter %d ok (pool %d, live pooled streams %zu)\n", i, (int)g_pool, g_streams.size());
      std::fflush(stdout);
    }
  }
  // the long-lived handle destroyed, then a fresh two-stream handle (which takes its streams' recycled objects):
  // eager, captured (instantiate + first launch), replayed - the shape of the faulting test order
  delete keep;
  {
    Handle e(false, K);
    for (int r = 0; r < 3; ++r) e.forward(nullptr);
    CK(hipDeviceSynchronize());
  }
  std::printf("final fresh handle after the long-lived one: ok\n");
  for (auto& s : callers) CK(hipStreamDestroy(s));
  std::printf("graph_churn: %d iterations, pool %d, %d kernels per branch, all %d, forks %d, memset %d: no fault\n", iters,
              (int)g_pool, K, (int)all, g_forks, (int)g_memset);
  return 0;
}
