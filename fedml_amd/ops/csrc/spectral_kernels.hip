// K12 — Fourier amplitude mixing of HS-FedAvg (FedDG style; reference hs_fedavg/hs_fft.py:8-84, numpy per
// image on the host). Three launches per batch, all on device, fp32 throughout, deterministic:
//
//   spec_fft2_kernel        one workgroup per (image, channel) plane: the plane is staged in LDS and its 2-D DFT
//                           runs as two passes of twiddle-table dot products (rows, then columns) —
//                           F[u][v] = Σ_h e^{-2πi·hu/H} Σ_w x[h][w]·e^{-2πi·wv/W}. Writes F (complex) and |F|.
//   spec_amp_update_kernel  the batch-mean amplitude per (channel, u, v) in a fixed order (no atomics) and the
//                           running-amplitude EMA (reference `process`: amp ← (1−m)·amp + m·mean, or mean on the
//                           first call), in place.
//   spec_mix_ifft2_kernel   per plane: inside the low-frequency band (|f_u| ≤ b, |f_v| ≤ b in unshifted
//                           coordinates ≡ the reference's centred (2b+1)² box after fftshift) the amplitude becomes
//                           the running one with the phase kept, F' = F·(A/|F|) (F = 0: phase 0, as torch.polar of
//                           angle(0)); then the inverse 2-D DFT, real part, ÷ HW.
//
// Images are ≤ 64×64 (CIFAR 32², MNIST 28², any size, not only powers of two): an O(H·W·(H+W)) DFT per plane
// is a few hundred k FMAs, far below the launch cost, so no butterfly network is needed. Twiddles come from a
// per-plane table built in double precision (index (k·n) mod N, incremented, no multiply), so the transform is
// as accurate as rocFFT's fp32 plan.
#include "common.h"

namespace spec {

constexpr int kMaxHW = 64;

// tw[k] = e^{sign·2πi·k/n}, k < n
__device__ __forceinline__ void twiddles(float2* tw, int n, float sign) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    double s, c;
    sincospi(2.0 * k / n, &s, &c);
    tw[k] = make_float2((float)c, (float)(sign * s));
  }
}

__global__ __launch_bounds__(256) void spec_fft2_kernel(const float* __restrict__ x, float2* __restrict__ F,
                                                        float* __restrict__ amp, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // twH[H] twW[W] Y[HW] X[HW]
  const int HW = H * W;
  float2* twH = reinterpret_cast<float2*>(smem);
  float2* twW = twH + kMaxHW;
  float2* Y = twW + kMaxHW;
  float* X = reinterpret_cast<float*>(Y + HW);
  const int64_t plane = blockIdx.x;
  const float* xp = x + plane * HW;
  for (int i = threadIdx.x; i < HW; i += blockDim.x) X[i] = xp[i];
  twiddles(twH, H, -1.f);
  twiddles(twW, W, -1.f);
  __syncthreads();
  // rows: Y[h][v] = Σ_w X[h][w]·e^{-2πi·wv/W}
  for (int i = threadIdx.x; i < HW; i += blockDim.x) {
    const int h = i / W, v = i - h * W;
    float2 acc = make_float2(0.f, 0.f);
    int k = 0;
    for (int w = 0; w < W; ++w) {
      const float xv = X[h * W + w];
      const float2 t = twW[k];
      acc.x = fmaf(xv, t.x, acc.x);
      acc.y = fmaf(xv, t.y, acc.y);
      k += v;
      if (k >= W) k -= W;
    }
    Y[i] = acc;
  }
  __syncthreads();
  // columns: F[u][v] = Σ_h Y[h][v]·e^{-2πi·hu/H}
  float2* Fp = F + plane * HW;
  float* ap = amp + plane * HW;
  for (int i = threadIdx.x; i < HW; i += blockDim.x) {
    const int u = i / W, v = i - u * W;
    float2 acc = make_float2(0.f, 0.f);
    int k = 0;
    for (int h = 0; h < H; ++h) {
      const float2 y = Y[h * W + v], t = twH[k];
      acc.x = fmaf(y.x, t.x, fmaf(-y.y, t.y, acc.x));
      acc.y = fmaf(y.x, t.y, fmaf(y.y, t.x, acc.y));
      k += u;
      if (k >= H) k -= H;
    }
    Fp[i] = acc;
    ap[i] = sqrtf(acc.x * acc.x + acc.y * acc.y);
  }
}

// running[c][i] (CHW elements): mean over the B planes of channel c, then the EMA (mode 0: keep, 1: EMA,
// 2: replace — the reference's first call, when the running amplitude is still all zeros)
__global__ __launch_bounds__(256) void spec_amp_update_kernel(const float* __restrict__ amp, float* __restrict__ run,
                                                              int B, int C, int HW, float momentum, int mode) {
  const int64_t n = (int64_t)C * HW;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += amp[(int64_t)b * n + e];
    const float mean = s / (float)B;
    if (mode == 1) run[e] = run[e] * (1.f - momentum) + mean * momentum;
    else if (mode == 2) run[e] = mean;
  }
}

__global__ __launch_bounds__(256) void spec_mix_ifft2_kernel(const float2* __restrict__ F, const float* __restrict__ amp,
                                                             const float* __restrict__ trg, float* __restrict__ out,
                                                             int C, int H, int W, int band) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // twH[H] twW[W] Y[HW] Z[HW]
  const int HW = H * W;
  float2* twH = reinterpret_cast<float2*>(smem);
  float2* twW = twH + kMaxHW;
  float2* Y = twW + kMaxHW;
  float2* Z = Y + HW;
  const int64_t plane = blockIdx.x;
  const int c = (int)(plane % C);
  const float2* Fp = F + plane * HW;
  const float* ap = amp + plane * HW;
  const float* tp = trg + (int64_t)c * HW;
  for (int i = threadIdx.x; i < HW; i += blockDim.x) {
    const int u = i / W, v = i - u * W;
    float2 f = Fp[i];
    if (min(u, H - u) <= band && min(v, W - v) <= band) {
      const float a = ap[i], A = tp[i];
      f = a > 0.f ? make_float2(f.x * (A / a), f.y * (A / a)) : make_float2(A, 0.f);
    }
    Z[i] = f;
  }
  twiddles(twH, H, 1.f);
  twiddles(twW, W, 1.f);
  __syncthreads();
  // Y[u][w] = Σ_v Z[u][v]·e^{+2πi·vw/W}
  for (int i = threadIdx.x; i < HW; i += blockDim.x) {
    const int u = i / W, w = i - u * W;
    float2 acc = make_float2(0.f, 0.f);
    int k = 0;
    for (int v = 0; v < W; ++v) {
      const float2 z = Z[u * W + v], t = twW[k];
      acc.x = fmaf(z.x, t.x, fmaf(-z.y, t.y, acc.x));
      acc.y = fmaf(z.x, t.y, fmaf(z.y, t.x, acc.y));
      k += w;
      if (k >= W) k -= W;
    }
    Y[i] = acc;
  }
  __syncthreads();
  // out[h][w] = Re Σ_u Y[u][w]·e^{+2πi·uh/H} / HW
  float* op = out + plane * HW;
  const float inv = 1.f / (float)HW;
  for (int i = threadIdx.x; i < HW; i += blockDim.x) {
    const int h = i / W, w = i - h * W;
    float acc = 0.f;
    int k = 0;
    for (int u = 0; u < H; ++u) {
      const float2 y = Y[u * W + w], t = twH[k];
      acc = fmaf(y.x, t.x, fmaf(-y.y, t.y, acc));
      k += h;
      if (k >= H) k -= H;
    }
    op[i] = acc * inv;
  }
}

}  // namespace spec

// x [B][C][H][W] fp32 → F [B][C][H][W] complex (float2), amp = |F|. H, W ≤ 64.
FA_EXPORT int fa_spec_fft2(const float* x, void* F, float* amp, int64_t planes, int H, int W, hipStream_t stream) {
  if (H < 1 || W < 1 || H > spec::kMaxHW || W > spec::kMaxHW || planes < 1) return -2;
  const size_t smem = (size_t)2 * spec::kMaxHW * 8 + (size_t)H * W * 12;
  hipLaunchKernelGGL(spec::spec_fft2_kernel, dim3((unsigned)planes), dim3(256), smem, stream, x,
                     reinterpret_cast<float2*>(F), amp, H, W);
  return (int)hipGetLastError();
}

// running [C][H][W] ← EMA of the batch-mean amplitude (mode 0 keep | 1 EMA | 2 replace)
FA_EXPORT int fa_spec_amp_update(const float* amp, float* running, int B, int C, int HW, float momentum, int mode,
                                 hipStream_t stream) {
  if (mode == 0) return 0;
  hipLaunchKernelGGL(spec::spec_amp_update_kernel, dim3(fa_grid((int64_t)C * HW, 256, 1024)), dim3(256), 0, stream,
                     amp, running, B, C, HW, momentum, mode);
  return (int)hipGetLastError();
}

// out [B][C][H][W] = Re ifft2(F with amplitude ← trg inside the band |f| ≤ band)
FA_EXPORT int fa_spec_mix_ifft2(const void* F, const float* amp, const float* trg, float* out, int64_t planes, int C,
                                int H, int W, int band, hipStream_t stream) {
  if (H < 1 || W < 1 || H > spec::kMaxHW || W > spec::kMaxHW || planes < 1) return -2;
  const size_t smem = (size_t)2 * spec::kMaxHW * 8 + (size_t)H * W * 16;
  (void)hipFuncSetAttribute((const void*)spec::spec_mix_ifft2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)smem);
  hipLaunchKernelGGL(spec::spec_mix_ifft2_kernel, dim3((unsigned)planes), dim3(256), smem, stream,
                     reinterpret_cast<const float2*>(F), amp, trg, out, C, H, W, band);
  return (int)hipGetLastError();
}
