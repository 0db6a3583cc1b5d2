// Device-side CIFAR-style data augmentation (reference: `data/cifar10/data_loader.py:58-103`,
// torchvision RandomCrop(32, padding=4) + RandomHorizontalFlip + Cutout(16) + Normalize on the CPU).
//
// One fused pass over a [B, C, H, W] fp32 batch already in HBM: every output pixel gathers its
// source pixel through the sample's random crop offset and flip, is zeroed inside the sample's
// cutout square, and is normalised per channel. Per-sample randomness comes from Philox4x32 keyed
// by (seed, sample id), so a batch is reproducible and independent of launch geometry.
#include "common.h"

__global__ __launch_bounds__(256) void augment_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                      const int64_t* __restrict__ sample_ids, int B, int C, int H,
                                                      int W, int pad, int cutout, int flip, const float* __restrict__ mean,
                                                      const float* __restrict__ inv_std, uint32_t seed) {
  const int b = blockIdx.y;
  const int64_t sid = sample_ids ? sample_ids[b] : b;
  const Philox4 r = philox4x32((uint32_t)sid, (uint32_t)(sid >> 32), 0x41554721u, 0u, seed, 0x9E3779B9u);
  const int dy = pad ? (int)(r.v[0] % (uint32_t)(2 * pad + 1)) - pad : 0;
  const int dx = pad ? (int)(r.v[1] % (uint32_t)(2 * pad + 1)) - pad : 0;
  const bool fl = flip && (r.v[2] & 1u);
  const int cy = cutout ? (int)(r.v[3] % (uint32_t)H) : -1000000;
  const int cx = cutout ? (int)((r.v[3] >> 16) % (uint32_t)W) : -1000000;
  const int half = cutout / 2;
  const int n = C * H * W;
  const float* xs = x + (int64_t)b * n;
  float* ys = y + (int64_t)b * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c = i / (H * W), rem = i % (H * W);
    const int oh = rem / W, ow = rem % W;
    const int sw0 = fl ? (W - 1 - ow) : ow;  // flip is applied after the crop (torchvision order)
    const int sh = oh + dy, sw = sw0 + dx;
    float v = (sh >= 0 && sh < H && sw >= 0 && sw < W) ? xs[(int64_t)c * H * W + sh * W + sw] : 0.f;
    if (oh >= cy - half && oh < cy + half && ow >= cx - half && ow < cx + half) v = 0.f;
    ys[i] = mean ? (v - mean[c]) * inv_std[c] : v;
  }
}

FA_EXPORT int fa_augment(const float* x, float* y, const int64_t* sample_ids, int B, int C, int H, int W, int pad,
                         int cutout, int flip, const float* mean, const float* inv_std, uint32_t seed,
                         hipStream_t stream) {
  const int n = C * H * W;
  dim3 grid((unsigned)fa_grid(n, 256, 64), (unsigned)B);
  hipLaunchKernelGGL(augment_kernel, grid, dim3(256), 0, stream, x, y, sample_ids, B, C, H, W, pad, cutout, flip, mean,
                     inv_std, seed);
  return (int)hipGetLastError();
}
