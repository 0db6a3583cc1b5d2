// Channels-last (NHWC) training-mode BatchNorm with fused residual add + ReLU, for the per-client
// (wide-CNN, e.g. ResNet-18) path of the virtual-client engine. Replaces MIOpen's six batch-norm
// kernels per layer (mean/var, final mean/var, norm; dscale/dbias, final, dx) plus the separate
// ReLU / residual-add elementwise kernels with four launches:
//
//   fwd: bnc_stats  (per-channel Σx, Σx² → fp32 atomics)      bnc_apply (scale/shift → y = act(x·s + t [+ r]))
//   bwd: bnc_reduce (g = dy·[y>0]; Σg, Σg·(x−μ); dres = g)    bnc_dx   (dx = A·g + B·x + D; dγ, dβ)
//
// Layout: x is [M = N·H·W, C] bf16 rows (NCHW tensors with channels-last strides). Each lane owns 8
// consecutive channels of one row (one 16-B load); C/8 lanes cover a row, 256/(C/8) rows per block
// pass, so C ∈ {8, 16, …, 2048}. The statistics pass reduces its rows in registers, then across the
// block's rows in LDS, then issues one device-scope fp32 atomic per channel per block into a zeroed
// [2C] accumulator; the consumer pass reads it after the kernel boundary (no in-launch hand-off, so
// no cross-XCD visibility protocol is needed). Reference semantics: `torch.nn.BatchNorm2d` training
// forward (biased variance for normalisation, unbiased for the running estimate; the reference's
// CIFAR ResNets, `model/cv/resnet.py:38-120`, put one after every convolution).
#include "common.h"

namespace bnc {

constexpr int kThreads = 256;

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f32_to_bf16(f[2 * i]) | ((uint32_t)f32_to_bf16(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// block-level reduction of per-lane [8] partials a and b over the rows a block pass covers, then one
// atomic per channel: acc[ch] += Σa, acc[C + ch] += Σb
__device__ __forceinline__ void reduce_to_acc(const float* a, const float* b, int cg, float* acc, float* red) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[k * kThreads + tid] = a[k];
    red[(8 + k) * kThreads + tid] = b[k];
  }
  __syncthreads();
  const int rpb = kThreads / cg, C = cg * 8;
  for (int t = tid; t < cg * 16; t += kThreads) {
    const int j = t % cg, k = t / cg;
    float s = 0.f;
    for (int r = 0; r < rpb; ++r) s += red[k * kThreads + r * cg + j];
    atomicAdd(&acc[(k < 8 ? 0 : C) + j * 8 + (k & 7)], s);
  }
}

// Shifted sums: every block accumulates Σ(x − k), Σ(x − k)² with the per-channel pivot k = x[row 0]
// (read by every block, so all partial sums share it): the variance then has no E[x²] − mean²
// cancellation when |mean| ≫ std.
__global__ __launch_bounds__(kThreads) void stats_kernel(const uint4* __restrict__ x, int64_t M, int cg,
                                                         float* __restrict__ acc) {
  __shared__ float red[16 * kThreads];
  const int j = threadIdx.x % cg, rpb = kThreads / cg;
  float piv[8];
  unpack8(x[j], piv);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t r = (int64_t)blockIdx.x * rpb + threadIdx.x / cg; r < M; r += (int64_t)gridDim.x * rpb) {
    float f[8];
    unpack8(x[r * cg + j], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = f[k] - piv[k];
      s[k] += d;
      q[k] = fmaf(d, d, q[k]);
    }
  }
  reduce_to_acc(s, q, cg, acc, red);
}

// per-channel coefficients (block 0 also publishes mean / invstd and the running estimates)
__global__ __launch_bounds__(kThreads) void apply_kernel(const uint4* __restrict__ x, const uint4* __restrict__ res,
                                                         uint4* __restrict__ y, int64_t M, int cg,
                                                         const float* __restrict__ acc, const float* __restrict__ w,
                                                         const float* __restrict__ b, float eps, float momentum,
                                                         float* __restrict__ rmean, float* __restrict__ rvar,
                                                         float* __restrict__ save, int relu) {
  __shared__ float4 coef[2 * 2048 / 4];  // scale[C], shift[C]
  float* sc = reinterpret_cast<float*>(coef);
  const int C = cg * 8;
  float* sh = sc + C;
  const float inv_m = 1.f / (float)M;
  const float unbias = M > 1 ? (float)M / (float)(M - 1) : 1.f;
  const uint16_t* x16 = reinterpret_cast<const uint16_t*>(x);   // row 0 = the statistics pivot
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float dm = acc[c] * inv_m;                              // mean of (x − k)
    const float mean = bf16_to_f32(x16[c]) + dm;
    const float var = fmaxf(acc[C + c] * inv_m - dm * dm, 0.f);
    const float inv = rsqrtf(var + eps);
    const float s = w ? w[c] * inv : inv;
    sc[c] = s;
    sh[c] = (b ? b[c] : 0.f) - mean * s;
    if (blockIdx.x == 0) {
      save[c] = mean;
      save[C + c] = inv;
      if (rmean) {
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * unbias;
      }
    }
  }
  __syncthreads();
  const int64_t nvec = M * cg;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * kThreads) {
    const int j = (int)(i % cg);
    float f[8], r[8];
    unpack8(x[i], f);
    if (res) unpack8(res[i], r);
    const float4 s0 = coef[2 * j], s1 = coef[2 * j + 1];
    const float4 t0 = coef[cg * 2 + 2 * j], t1 = coef[cg * 2 + 2 * j + 1];
    const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float tv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = fmaf(f[k], sv[k], tv[k]);
      if (res) v += r[k];
      f[k] = relu ? fmaxf(v, 0.f) : v;
    }
    y[i] = pack8(f);
  }
}

// g = dy · [y > 0] (relu) ; Σg, Σg·(x − μ) ; dres = g
__global__ __launch_bounds__(kThreads) void reduce_kernel(const uint4* __restrict__ dy, const uint4* __restrict__ x,
                                                          const uint4* __restrict__ y, uint4* __restrict__ dres,
                                                          int64_t M, int cg, const float* __restrict__ save,
                                                          float* __restrict__ acc) {
  __shared__ float red[16 * kThreads];
  const int j = threadIdx.x % cg, rpb = kThreads / cg;
  float mu[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) mu[k] = save[j * 8 + k];
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t r = (int64_t)blockIdx.x * rpb + threadIdx.x / cg; r < M; r += (int64_t)gridDim.x * rpb) {
    const int64_t i = r * cg + j;
    float g[8], f[8];
    unpack8(dy[i], g);
    unpack8(x[i], f);
    if (y) {
      float o[8];
      unpack8(y[i], o);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = o[k] > 0.f ? g[k] : 0.f;
      if (dres) dres[i] = pack8(g);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[k] += g[k];
      q[k] = fmaf(g[k], f[k] - mu[k], q[k]);
    }
  }
  reduce_to_acc(s, q, cg, acc, red);
}

// dx = γ·inv·(g − mean(g) − x̂·mean(g·x̂)) = A·g + B·x + D per channel; block 0 writes dγ, dβ
__global__ __launch_bounds__(kThreads) void dx_kernel(const uint4* __restrict__ dy, const uint4* __restrict__ x,
                                                      const uint4* __restrict__ y, uint4* __restrict__ dx, int64_t M,
                                                      int cg, const float* __restrict__ save,
                                                      const float* __restrict__ acc, const float* __restrict__ w,
                                                      float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float4 coef[3 * 2048 / 4];
  float* A = reinterpret_cast<float*>(coef);
  const int C = cg * 8;
  float* B = A + C;
  float* D = B + C;
  const float inv_m = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float mean = save[c], inv = save[C + c];
    const float sg = acc[c], sgx = acc[C + c] * inv;  // Σg, Σg·x̂
    const float k1 = (w ? w[c] : 1.f) * inv;
    const float mg = sg * inv_m, mgx = sgx * inv_m;
    A[c] = k1;
    B[c] = -k1 * inv * mgx;
    D[c] = -k1 * mg + k1 * inv * mgx * mean;
    if (blockIdx.x == 0) {
      if (dw) dw[c] = sgx;
      if (db) db[c] = sg;
    }
  }
  __syncthreads();
  const int64_t nvec = M * cg;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * kThreads) {
    const int j = (int)(i % cg);
    float g[8], f[8];
    unpack8(dy[i], g);
    unpack8(x[i], f);
    if (y) {
      float o[8];
      unpack8(y[i], o);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = o[k] > 0.f ? g[k] : 0.f;
    }
    const float4 a0 = coef[2 * j], a1 = coef[2 * j + 1];
    const float4 b0 = coef[cg * 2 + 2 * j], b1 = coef[cg * 2 + 2 * j + 1];
    const float4 d0 = coef[cg * 4 + 2 * j], d1 = coef[cg * 4 + 2 * j + 1];
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = fmaf(av[k], g[k], fmaf(bv[k], f[k], dv[k]));
    dx[i] = pack8(g);
  }
}

static inline bool shape_ok(int64_t M, int C) {
  return M > 0 && C >= 8 && C <= 2048 && C % 8 == 0 && (kThreads % (C / 8)) == 0;
}

// statistics grid: ≥8 rows per lane, at most 1024 blocks (bounded atomic traffic)
static inline int stats_grid(int64_t M, int cg) {
  const int64_t rows_per_block = (int64_t)(kThreads / cg) * 8;
  int64_t g = (M + rows_per_block - 1) / rows_per_block;
  if (g > 1024) g = 1024;
  return g < 1 ? 1 : (int)g;
}

}  // namespace bnc

FA_EXPORT int fa_bnc_fwd(const void* x, const void* res, void* y, int64_t M, int C, float* acc, const float* w,
                         const float* b, float eps, float momentum, float* rmean, float* rvar, float* save, int relu,
                         hipStream_t stream) {
  if (!bnc::shape_ok(M, C)) return (int)hipErrorInvalidValue;
  const int cg = C / 8;
  hipLaunchKernelGGL(bnc::stats_kernel, dim3(bnc::stats_grid(M, cg)), dim3(bnc::kThreads), 0, stream,
                     (const uint4*)x, M, cg, acc);
  hipLaunchKernelGGL(bnc::apply_kernel, dim3(fa_grid(M * cg, bnc::kThreads, 2048)), dim3(bnc::kThreads), 0, stream,
                     (const uint4*)x, (const uint4*)res, (uint4*)y, M, cg, acc, w, b, eps, momentum, rmean, rvar, save,
                     relu);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_bnc_bwd(const void* dy, const void* x, const void* y, void* dres, void* dx, int64_t M, int C,
                         const float* save, float* acc, const float* w, float* dw, float* db, hipStream_t stream) {
  if (!bnc::shape_ok(M, C)) return (int)hipErrorInvalidValue;
  const int cg = C / 8;
  hipLaunchKernelGGL(bnc::reduce_kernel, dim3(bnc::stats_grid(M, cg)), dim3(bnc::kThreads), 0, stream,
                     (const uint4*)dy, (const uint4*)x, (const uint4*)y, (uint4*)dres, M, cg, save, acc);
  hipLaunchKernelGGL(bnc::dx_kernel, dim3(fa_grid(M * cg, bnc::kThreads, 2048)), dim3(bnc::kThreads), 0, stream,
                     (const uint4*)dy, (const uint4*)x, (const uint4*)y, (uint4*)dx, M, cg, save, acc, w, dw, db);
  return (int)hipGetLastError();
}
