// GPU feature builder: the input side of the boundary, replacing the CPU
// numpy/cv2 work of TransfuserFeatureBuilder.compute_features (transfuser_features.py:39-138).
//
//  * camera: crop + stitch (l0[28:-28, 416:-416] | f0[28:-28] | r0[28:-28, 416:-416]), cv2
//    INTER_LINEAR resize to out_w x out_h, ToTensor (uint8 HWC -> float CHW / 255), fused in one
//    pass: each output pixel reads its 2x2 source block straight from the camera it falls in (the
//    stitched image is never materialised). At the NAVSIM geometry (4096x1024 -> 1024x256, exact
//    factor f = 4) OpenCV's fixed-point bilinear weighs the taps at rows / columns f*d + f/2 - 1 and
//    f*d + f/2 by 0.5 each, which rounds to (p00 + p01 + p10 + p11 + 2) >> 2 (oracle/features.py).
//    Memory-bound: 6 B read per output pixel and channel-row pair, 12 B written per pixel.
//  * LiDAR: np.histogramdd splat (:111-138) as one atomic-add pass over the points into a uint32
//    count image that aliases the float output, then an in-place finalize min(c, hist_max) /
//    hist_max (double, rounded to float like numpy's float64 -> float32). Binning is done in double
//    ((x + 32) * 4 is exact there), so bin edges, the inclusive upper range end and NaN / out-of-
//    range drops match histogramdd bit for bit (pinned by tests/golden/lidar_feat_*.npz).
#include <algorithm>
#include <cstdint>
#include <string>

#include "common.h"

namespace ddmi {

__global__ void camera_feature_kernel(const uint8_t* __restrict__ cams, int H, int W, float* __restrict__ out,
                                      int oh, int ow, int f, int crop_top, int crop_side) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  const int b = blockIdx.z;
  if (x >= ow) return;
  const int wl = W - 2 * crop_side;  // cropped width of l0 / r0
  const int o = f / 2 - 1;
  const int sx = f * x + o;          // stitched column of the left tap (the right tap is sx + 1)
  int cam, cx;
  if (sx < wl) {
    cam = 0;
    cx = sx + crop_side;
  } else if (sx < wl + W) {
    cam = 1;
    cx = sx - wl;
  } else {
    cam = 2;
    cx = sx - wl - W + crop_side;
  }
  const int sy = crop_top + f * y + o;
  const uint8_t* img = cams + ((size_t)b * 3 + cam) * (size_t)H * W * 3;
  const uint8_t* r0 = img + ((size_t)sy * W + cx) * 3;
  const uint8_t* r1 = r0 + (size_t)W * 3;
  const size_t plane = (size_t)oh * ow;
  float* o0 = out + (size_t)b * 3 * plane + (size_t)y * ow + x;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int s = (int)r0[c] + (int)r0[3 + c] + (int)r1[c] + (int)r1[3 + c];
    o0[c * plane] = (float)((s + 2) >> 2) / 255.0f;
  }
}

__device__ inline int hist_bin(float v, double lo, double hi, double ppm, int nb) {
  const double d = (double)v;
  if (!(d >= lo && d <= hi)) return -1;  // out of range or NaN: dropped by histogramdd
  int i = (int)floor((d - lo) * ppm);
  return i >= nb ? nb - 1 : i;            // v == hi belongs to the last bin
}

// xyz: per scene b, planar rows x[N_b], y[N_b], z[N_b] starting at 3 * offs[b] (NAVSIM lidar_pc[:3]).
__global__ void lidar_splat_kernel(const float* __restrict__ xyz, const int64_t* __restrict__ offs, int C,
                                   unsigned* __restrict__ counts, int nb, double lo, double hi, double ppm,
                                   float max_h, float split_h) {
  const int b = blockIdx.y;
  const int64_t p0 = offs[b], n = offs[b + 1] - p0;
  const float* px = xyz + 3 * p0;
  const float* py = px + n;
  const float* pz = py + n;
  unsigned* cb = counts + (size_t)b * C * nb * nb;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float z = pz[i];
    if (!(z < max_h)) continue;  // transfuser_features.py:131 (NaN z dropped too)
    const bool above = z > split_h;
    int ch;
    if (C == 2)
      ch = above ? 1 : 0;        // use_ground_plane: [below, above]
    else if (above)
      ch = 0;
    else
      continue;
    const int ix = hist_bin(px[i], lo, hi, ppm, nb);
    const int iy = hist_bin(py[i], lo, hi, ppm, nb);
    if (ix < 0 || iy < 0) continue;
    atomicAdd(cb + ((size_t)ch * nb + ix) * nb + iy, 1u);
  }
}

__global__ void lidar_finalize_kernel(float* __restrict__ out, size_t n, int hist_max) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned c = reinterpret_cast<const unsigned*>(out)[i];
  const unsigned cl = c > (unsigned)hist_max ? (unsigned)hist_max : c;
  out[i] = (float)((double)cl / (double)hist_max);
}

void launch_camera_feature(const uint8_t* cams, int B, int H, int W, float* out, int oh, int ow, hipStream_t st) {
  constexpr int crop_top = 28, crop_side = 416;  // transfuser_features.py:68-70
  const int wl = W - 2 * crop_side;
  const int sw = 2 * wl + W, sh = H - 2 * crop_top;
  if (B <= 0 || oh <= 0 || ow <= 0 || wl <= 0 || sh <= 0)
    throw std::invalid_argument("camera feature: bad sizes");
  const int f = sh / oh;
  if (sh != f * oh || sw != f * ow || f < 2 || (f % 2) || (wl % f) || (W % f))
    throw std::invalid_argument("camera feature: the stitched " + std::to_string(sw) + "x" + std::to_string(sh) +
                                " image must down-scale to " + std::to_string(ow) + "x" + std::to_string(oh) +
                                " by one even integer factor with camera seams on factor boundaries");
  dim3 grid((ow + 255) / 256, oh, B);
  hipLaunchKernelGGL(camera_feature_kernel, grid, dim3(256), 0, st, cams, H, W, out, oh, ow, f, crop_top, crop_side);
  DD_HIP_CHECK(hipGetLastError());
}

void launch_lidar_feature(const float* xyz, const int64_t* offs, int B, int C, float* out, int nb, float lo,
                          float hi, int ppm, float max_h, float split_h, int hist_max, int64_t max_points,
                          hipStream_t st) {
  if (B <= 0 || (C != 1 && C != 2) || nb <= 0 || hist_max <= 0)
    throw std::invalid_argument("lidar feature: bad arguments");
  if ((int64_t)((hi - lo) * ppm) != nb) throw std::invalid_argument("lidar feature: (hi - lo) * ppm != resolution");
  const size_t n = (size_t)B * C * nb * nb;
  DD_HIP_CHECK(hipMemsetAsync(out, 0, n * sizeof(float), st));
  const int64_t per = max_points > 0 ? max_points : 1;
  const int bx = (int)std::min<int64_t>((per + 255) / 256, 1024);
  hipLaunchKernelGGL(lidar_splat_kernel, dim3(bx, B), dim3(256), 0, st, xyz, offs, C,
                     reinterpret_cast<unsigned*>(out), nb, (double)lo, (double)hi, (double)ppm, max_h, split_h);
  DD_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(lidar_finalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n, hist_max);
  DD_HIP_CHECK(hipGetLastError());
}

}  // namespace ddmi
