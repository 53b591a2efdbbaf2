// Microbenchmark: sustained f16 MFMA rate on the whole chip, 32x32x16 vs 16x16x32, with operands that
// change every instruction (four register sets of pseudo-random fp16), ~2 s of back-to-back launches per
// arm so the clock settles. Calibrates whether the 16x16x32 shape holds a higher clock under DVFS.
//   hipcc -O3 --offload-arch=gfx950 mfma_shape.hip -o mfma_shape && ./mfma_shape
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k32(const half8* seed, float* out, int iters) {
  half8 a[4], b[4];
  for (int i = 0; i < 4; ++i) a[i] = seed[(threadIdx.x * 5 + i * 17) % 256], b[i] = seed[(threadIdx.x * 3 + i * 29 + 7) % 256];
  f32x16 acc[4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(s + i) & 3], b[s], acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// same FLOPs per iteration: 4 x (4 16x16x32 per 32x32x16 output block pair) -> 2x instructions of half length
__global__ __launch_bounds__(256) void k16(const half8* seed, float* out, int iters) {
  half8 a[4], b[4];
  for (int i = 0; i < 4; ++i) a[i] = seed[(threadIdx.x * 5 + i * 17) % 256], b[i] = seed[(threadIdx.x * 3 + i * 29 + 7) % 256];
  f32x4 acc[16] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        acc[(s * 8 + i) & 15] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(s + i) & 3], b[(s + (i >> 2)) & 3], acc[(s * 8 + i) & 15], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 16; ++i)
    for (int r = 0; r < 4; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  std::vector<_Float16> hs(256 * 8);
  uint32_t x = 12345;
  for (auto& h : hs) {
    x = x * 1664525u + 1013904223u;
    h = (_Float16)(((x >> 8) & 0xffff) / 65536.0f - 0.5f);
  }
  half8* dh;
  float* dout;
  hipMalloc(&dh, hs.size() * 2);
  hipMalloc(&dout, 512 * 256 * 4);
  hipMemcpy(dh, hs.data(), hs.size() * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000, reps = 1200;
  for (int round = 0; round < 2; ++round)
    for (int shape : {32, 16}) {
      const int grid = 512;  // 2 WG/CU = 2 waves/SIMD
      for (int r = 0; r < 3; ++r) (shape == 32 ? k32 : k16)<<<grid, 256>>>(dh, dout, iters);
      hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) (shape == 32 ? k32 : k16)<<<grid, 256>>>(dh, dout, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flops = (double)reps * grid * 4 * iters * 16 * 32 * 32 * 16 * 2;
      printf("f16 %dx%d: %.1f TFLOP/s (%.1f ms)\n", shape, shape, flops / ms / 1e9, ms);
    }
  return 0;
}
