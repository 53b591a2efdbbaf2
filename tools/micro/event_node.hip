// Does an external event-record node inside a captured single-stream graph order a later hipStreamWaitEvent on
// another stream? Graph M (stream m): spin ~spin_us, write gen into flag, [record e], spin again. Stream s:
// hipStreamWaitEvent(s, e) issued after hipGraphLaunch(M), then a kernel that copies flag into out[i].
// out[i] == i + 1 for every launch i means the wait saw the in-graph record of the same launch.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/event_node.hip -o /tmp/event_node && /tmp/event_node
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP %s at line %d\n", hipGetErrorString(e_), __LINE__);       \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

__global__ void spin_then_bump(unsigned* flag, long long cycles, int bump) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (bump && threadIdx.x == 0) flag[0] = flag[0] + 1u;
}
__global__ void copy_flag(const unsigned* flag, unsigned* out, int i) {
  if (threadIdx.x == 0) out[i] = flag[0];
}

int main() {
  const int N = 200;
  unsigned *flag, *out;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&out, N * 4));
  CK(hipMemset(flag, 0, 4));
  CK(hipMemset(out, 0, N * 4));
  hipStream_t m, s, cap;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  hipEvent_t e;
  CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const long long spin = 200000;  // ~0.1 ms at 2 GHz
  hipGraph_t g;
  CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(spin_then_bump, dim3(1), dim3(64), 0, cap, flag, spin, 1);
  CK(hipEventRecordWithFlags(e, cap, hipEventRecordExternal));
  hipLaunchKernelGGL(spin_then_bump, dim3(1), dim3(64), 0, cap, flag, spin, 0);
  CK(hipStreamEndCapture(cap, &g));
  size_t n = 0;
  CK(hipGraphGetNodes(g, nullptr, &n));
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  for (int i = 0; i < N; ++i) {
    CK(hipGraphLaunch(ex, m));
    CK(hipStreamWaitEvent(s, e, 0));
    hipLaunchKernelGGL(copy_flag, dim3(1), dim3(64), 0, s, flag, out, i);
    // the next launch of M must not start before this copy: order m behind s
    hipEvent_t j;
    CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    CK(hipEventRecord(j, s));
    CK(hipStreamWaitEvent(m, j, 0));
    CK(hipEventDestroy(j));
  }
  CK(hipDeviceSynchronize());
  unsigned h[N];
  CK(hipMemcpy(h, out, N * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < N; ++i) bad += h[i] != (unsigned)(i + 1);
  printf("graph nodes %zu; launches %d; wrong %d (first values %u %u %u)\n", n, N, bad, h[0], h[1], h[2]);
  return bad ? 1 : 0;
}
