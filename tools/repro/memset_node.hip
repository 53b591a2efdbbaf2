// Reproducer for the round-5 tfdec_mk4 replay failure (profiles/round5_ab.md, "Two more found by the in-flight
// lanes test"): with a hipMemsetAsync node zeroing the scene counters ahead of tfdec_mk4, replays of the TWO-stream
// program went wrong (flags 0, query_out off by up to 0.35) while the single-stream program stayed right
// (gpurun_out/tfr_memset.log). In the two-stream program the tf decoder is a side segment of its own: a graph whose
// ROOT node is that memset, launched on the side stream right after hipStreamWaitEvent(side, fork event).
//
// Each case below replays one small graph `reps` times. A "writer" kernel W first sleeps ~sleep_us on the device,
// then stores a nonzero tag (agent-scope atomic stores) into n counters; the graph under test zeroes the counters and
// a checker kernel C reads them (agent-scope atomic loads) and counts every replay in which it saw a nonzero word.
// W is ordered before the graph by the stream (same stream) or by an event (other stream): a nonzero count means the
// zeroing did not run after W, or C did not run after the zeroing.
//
//   case 0  W on main, event, wait on side, graph [memset, C] on side          (the product's side segment)
//   case 1  as 0, graph [noop kernel, memset, C]                                (memset not the root)
//   case 2  W on side, graph [memset, C] on side                                (same stream, no event)
//   case 3  as 0, graph [zero kernel, C]                                        (zeroing by a kernel node)
//   case 4  as 0, graph [memsetD32, C]
//   case 5  as 0, no graph: hipMemsetAsync + C launched on side directly        (stream semantics, eager)
//   case 6  as 0, graph [C] only                                                (control: C must see the tag)
//   case 7  as 0, graph [memset, A]: A = 256 workgroups (all XCDs), each adds 1 to counter (wg % n) with an
//           agent-scope atomic (memory-side), writes back its XCD's L2 (agent release fence), sleeps, adds 1 again:
//           the adds must return 0 | 1 | 2 | 3 for the two phases (4 workgroups per counter); anything else = the
//           memset's zeros and the atomics disagree (the tfdec_mk4 counter pattern)
//   case 8  as 7, the counters zeroed by a kernel node with agent-scope atomic stores
//   case 9  as 7 with the memset in the middle of the graph: [noop, memset, A] (in the product a K / V GEMM precedes
//           the counters' memset in the same segment)
//   case 10 as 9 with a kernel between the memset and A: [noop, memset, noop, A]
//
//   memset_node <reps> <sleep_us> [dot-dir|-] [words]
// words (1..64, default 64): counters zeroed and used by cases 7 / 8 (the product zeroes 2 B words: 64 B at B = 8).
// Prints one line per case: replays, replays in which C saw a nonzero counter, and the first bad value.
// With dot-dir, each case's graph is written as <dot-dir>/case<k>.dot (hipGraphDebugDotPrint) to show its edges.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(3);                                                                            \
    }                                                                                          \
  } while (0)

constexpr int kN = 64;  // counters (the product zeroes 2 * B words)

// W: spin ~sleep_ticks of the 100 MHz constant clock, then tag every counter (vector atomic stores)
__global__ void k_writer(unsigned* cnt, unsigned long long sleep_ticks, const unsigned* tag) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < sleep_ticks) __builtin_amdgcn_s_sleep(8);
  }
  __syncthreads();
  const unsigned v = __hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kN) __hip_atomic_store(cnt + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// C: count a replay whose counters are not all zero; bump the tag for the next replay
__global__ void k_check(const unsigned* cnt, unsigned* bad, unsigned* first, unsigned* tag) {
  const unsigned v = threadIdx.x < kN ? __hip_atomic_load(cnt + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  const bool nz = __any(v != 0);
  if (v != 0) atomicCAS(first, 0u, v);
  if (threadIdx.x == 0) {
    if (nz) atomicAdd(bad, 1u);
    atomicAdd(tag, 1u);
  }
}

// A: 4 workgroups per counter, two arrival phases separated by an agent release (buffer_wbl2) + acquire
__global__ void k_arrive(unsigned* cnt, unsigned* bad, unsigned* first, int nw) {
  if (threadIdx.x != 0) return;
  unsigned* c = cnt + (blockIdx.x % nw);
  const unsigned o1 = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < 300) __builtin_amdgcn_s_sleep(4);  // ~3 us
  const unsigned o2 = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (o1 > 7 || o2 > 7 || o2 == 0) {
    atomicAdd(bad, 1u);
    atomicCAS(first, 0u, 0x10000u | (o1 << 8) | o2);
  }
}

__global__ void k_zero(unsigned* cnt) {
  if (threadIdx.x < kN) __hip_atomic_store(cnt + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_noop(unsigned* p) {
  if (threadIdx.x == 0 && p == nullptr) p[0] = 0;  // never taken
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 500;
  const int sleep_us = argc > 2 ? atoi(argv[2]) : 50;
  const char* dot = argc > 3 && std::string(argv[3]) != "-" ? argv[3] : nullptr;
  const int nw = argc > 4 ? std::max(1, std::min(kN, atoi(argv[4]))) : kN;
  CK(hipSetDevice(0));
  hipStream_t sm, ss;
  CK(hipStreamCreateWithFlags(&sm, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned *cnt, *bad, *first, *tag;
  CK(hipMalloc(&cnt, kN * sizeof(unsigned)));
  CK(hipMalloc(&bad, sizeof(unsigned)));
  CK(hipMalloc(&first, sizeof(unsigned)));
  CK(hipMalloc(&tag, sizeof(unsigned)));
  const unsigned long long ticks = (unsigned long long)sleep_us * 100ull;  // wall_clock64: 100 MHz
  int fails = 0;
  for (int c = 0; c <= 10; ++c) {
    const unsigned one = 1, zero = 0;
    CK(hipMemcpy(tag, &one, sizeof(unsigned), hipMemcpyHostToDevice));
    CK(hipMemcpy(bad, &zero, sizeof(unsigned), hipMemcpyHostToDevice));
    CK(hipMemcpy(first, &zero, sizeof(unsigned), hipMemcpyHostToDevice));
    CK(hipMemset(cnt, 0, kN * sizeof(unsigned)));
    CK(hipDeviceSynchronize());
    const hipStream_t gs = c == 2 ? ss : ss;  // every graph runs on the side stream
    hipGraphExec_t ex = nullptr;
    if (c != 5) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(gs, hipStreamCaptureModeThreadLocal));
      if (c == 1 || c >= 9) hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, gs, cnt);
      if (c == 0 || c == 1 || c == 2) CK(hipMemsetAsync(cnt, 0, kN * sizeof(unsigned), gs));
      if (c == 7 || c >= 9) CK(hipMemsetAsync(cnt, 0, nw * sizeof(unsigned), gs));
      if (c == 10) hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, gs, cnt);
      if (c == 3 || c == 8) hipLaunchKernelGGL(k_zero, dim3(1), dim3(kN), 0, gs, cnt);
      if (c == 4) CK(hipMemsetD32Async((hipDeviceptr_t)cnt, 0, kN, gs));
      if (c >= 7)
        hipLaunchKernelGGL(k_arrive, dim3(4 * nw), dim3(64), 0, gs, cnt, bad, first, nw);
      else
        hipLaunchKernelGGL(k_check, dim3(1), dim3(kN), 0, gs, cnt, bad, first, tag);
      CK(hipStreamEndCapture(gs, &g));
      if (dot) CK(hipGraphDebugDotPrint(g, (std::string(dot) + "/case" + std::to_string(c) + ".dot").c_str(), 0));
      CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      CK(hipGraphDestroy(g));
    }
    for (int r = 0; r < reps; ++r) {
      if (c >= 7) {  // the counters hold the last replay's final counts (8) when the graph starts
        CK(hipEventRecord(ev, sm));
        CK(hipStreamWaitEvent(ss, ev, 0));
      } else if (c == 2) {
        hipLaunchKernelGGL(k_writer, dim3(1), dim3(kN), 0, ss, cnt, ticks, tag);
      } else {
        hipLaunchKernelGGL(k_writer, dim3(1), dim3(kN), 0, sm, cnt, ticks, tag);
        CK(hipEventRecord(ev, sm));
        CK(hipStreamWaitEvent(ss, ev, 0));
      }
      if (c == 5) {
        CK(hipMemsetAsync(cnt, 0, kN * sizeof(unsigned), ss));
        hipLaunchKernelGGL(k_check, dim3(1), dim3(kN), 0, ss, cnt, bad, first, tag);
      } else {
        CK(hipGraphLaunch(ex, ss));
      }
      // the next replay's writer waits for this replay's checker (the writer runs on main)
      CK(hipEventRecord(ev, ss));
      CK(hipStreamWaitEvent(sm, ev, 0));
    }
    CK(hipDeviceSynchronize());
    unsigned nb = 0, fv = 0;
    CK(hipMemcpy(&nb, bad, sizeof(unsigned), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&fv, first, sizeof(unsigned), hipMemcpyDeviceToHost));
    const bool expect_bad = c == 6;
    const bool ok = expect_bad ? nb == (unsigned)reps : nb == 0;
    if (!ok) ++fails;
    std::printf("case %d: %d replays, %u %s (first value 0x%x) -> %s\n", c, reps, nb,
                c >= 7 ? "arrivals out of range" : "saw a nonzero counter", fv,
                ok ? "as expected" : "ORDER VIOLATED");
    std::fflush(stdout);
    if (ex) CK(hipGraphExecDestroy(ex));
  }
  CK(hipFree(cnt));
  CK(hipFree(bad));
  CK(hipFree(first));
  CK(hipFree(tag));
  CK(hipEventDestroy(ev));
  CK(hipStreamDestroy(sm));
  CK(hipStreamDestroy(ss));
  std::printf("memset_node: %d case(s) violated the expected order\n", fails);
  return 0;
}
