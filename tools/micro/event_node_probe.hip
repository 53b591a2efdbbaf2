#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* f) { if (threadIdx.x == 0) f[0] += 1; }
static void tryit(const char* name, hipStream_t cap, hipEvent_t e, bool memset_first, unsigned* f, int info = 0) {
  hipError_t r = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
  if (memset_first) (void)hipMemsetAsync(f, 0, 4, cap);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, cap, f);
  if (info == 1) {
    hipStreamCaptureStatus cs; size_t nd = 0;
    hipStreamGetCaptureInfo_v2(cap, &cs, nullptr, nullptr, nullptr, &nd);
  }
  if (info == 2) { hipMemcpyAsync(f, f + 1, 4, hipMemcpyDeviceToDevice, cap); }
  if (info == 3) { (void)hipMemsetAsync(f, 0, 4, cap); }
  hipError_t rr = hipEventRecordWithFlags(e, cap, hipEventRecordExternal);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, cap, f);
  hipGraph_t g = nullptr;
  hipError_t re = hipStreamEndCapture(cap, &g);
  printf("%-32s begin %d record %d (%s) end %d\n", name, r, rr, hipGetErrorString(rr), re);
  if (g) hipGraphDestroy(g);
  (void)hipGetLastError();
}
int main() {
  unsigned* f; hipMalloc(&f, 4);
  hipStream_t s0, sp, sd; hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
  int lo, hi; hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, 0);
  hipStreamCreateWithPriority(&sd, hipStreamNonBlocking, hi);
  hipEvent_t e1, e2, e3, e4; 
  hipEventCreateWithFlags(&e1, hipEventDisableTiming); hipEventCreateWithFlags(&e2, hipEventDisableTiming);
  hipEventCreateWithFlags(&e3, hipEventDisableTiming); hipEventCreateWithFlags(&e4, hipEventDisableTiming);
  tryit("plain", s0, e1, false, f);
  tryit("priority0 stream", sp, e2, false, f);
  tryit("priority hi stream", sd, e3, false, f);
  hipEventRecord(e4, s0); hipStreamSynchronize(s0);
  tryit("event recorded before", s0, e4, false, f);
  tryit("memset first", s0, e1, true, f);
  hipEvent_t e5; hipEventCreate(&e5);
  tryit("timing event", s0, e5, false, f);
  hipFree(f); hipMalloc(&f, 64);
  tryit("after GetCaptureInfo_v2", s0, e1, false, f, 1);
  tryit("after memcpy node", s0, e1, false, f, 2);
  tryit("after memset node", s0, e1, false, f, 3);
  return 0;
}
