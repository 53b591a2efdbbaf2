// Microbenchmark: sustained v_mfma_f32_32x32x16_f16 / _f32_32x32x2_f32 rate on the whole chip
// (no memory traffic). Used to calibrate the practical MFMA ceiling under DVFS on random data.
//   hipcc -O3 --offload-arch=gfx950 mfma_peak.hip -o mfma_peak && ./mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_f16(const half8* seed, float* out, int iters) {
  half8 a = seed[threadIdx.x % 64], b = seed[(threadIdx.x + 7) % 64];
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma_f32(const float* seed, float* out, int iters) {
  float a = seed[threadIdx.x % 64], b = seed[(threadIdx.x + 7) % 64];
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  std::vector<_Float16> hs(64 * 8);
  std::vector<float> fs(64);
  for (int i = 0; i < 64 * 8; ++i) hs[i] = (_Float16)((i * 37 % 101) / 101.0f - 0.5f);
  for (int i = 0; i < 64; ++i) fs[i] = (i * 53 % 97) / 97.0f - 0.5f;
  half8* dh;
  float *df, *dout;
  hipMalloc(&dh, hs.size() * 2);
  hipMalloc(&df, fs.size() * 4);
  hipMalloc(&dout, 256 * 2048 * 4);
  hipMemcpy(dh, hs.data(), hs.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(df, fs.data(), fs.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int wgs_per_cu : {1, 2}) {
    const int grid = 256 * wgs_per_cu;
    mfma_f16<4><<<grid, 256>>>(dh, dout, 100);
    hipEventRecord(e0);
    mfma_f16<4><<<grid, 256>>>(dh, dout, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)grid * 4 /*waves*/ * iters * 4 /*acc*/ * 32 * 32 * 16 * 2;
    printf("f16 32x32x16: %d WG/CU (%d waves/SIMD): %.1f TFLOP/s (%.3f ms)\n", wgs_per_cu, wgs_per_cu,
           flops / ms / 1e9, ms);
  }
  {
    const int grid = 512;
    mfma_f32<<<grid, 256>>>(df, dout, 100);
    hipEventRecord(e0);
    mfma_f32<<<grid, 256>>>(df, dout, iters / 4);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)grid * 4 * (iters / 4) * 4 * 32 * 32 * 2 * 2;
    printf("f32 32x32x2: 2 WG/CU: %.1f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
  }
  return 0;
}
