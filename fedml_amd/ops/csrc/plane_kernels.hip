// Client-batched depthwise convolution and BatchNorm(+ReLU) on the batched interpreter's client-stacked NCHW
// activations [B][CC = C·Ch][H][W] (parallel/batched_nn.py) — the MobileNet family's depthwise-separable blocks
// (reference `model/cv/mobilenet.py:58-150`, `mobilenet_v3.py:148-316`). In this layout every (image, client,
// channel) is one contiguous H×W plane and a depthwise filter touches exactly one plane, so the kernels work on
// planes directly: no layout bridge, no grouped-GEMM lowering (a depthwise conv has 9 MACs per output — it is
// a streaming op, not an MFMA one).
//
//   dw_fwd        y = x ⋆ w_cc                 one thread per output element (taps from L1/L2)
//   dw_bwd_data   dx = dy ⋆ flip(w_cc)          one thread per input element (stride-2 parity aware)
//   dw_wgrad      dw_cc = Σ_{b,p} dy·x_tap     one workgroup per channel, fixed-order tree (deterministic)
//   pbn_stats     μ, σ² per channel (shifted sums, one workgroup per channel)
//   pbn_apply     y = act(x·s + t)             s = γ/σ, t = β − μ·s
//   pbn_bwd_red   Σg', Σg'·(x − μ)  with g' = g·[x·s + t > 0] (ReLU mask recomputed from x)
//   pbn_dx        dx = s·(g' − Σg'/n − x̂·Σg'x̂/n)
// Weights / BN parameters are read from the client-stacked fp32 arena views (client stride given), the
// storage type T of the activations is fp32 (the reference's precision) or bf16; statistics are fp32.
#include "common.h"

namespace pk {

template <typename T>
__device__ __forceinline__ float ld(const T* p);
template <>
__device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <typename T>
__device__ __forceinline__ void st(T* p, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

// weight of stacked channel cc = c·Ch + ch: w + c·wcs + ch·K·K
__device__ __forceinline__ const float* wrow(const float* w, int64_t wcs, int Ch, int cc, int KK) {
  return w + (int64_t)(cc / Ch) * wcs + (int64_t)(cc % Ch) * KK;
}

template <typename T, int K, int S>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w, int64_t wcs,
                                                     T* __restrict__ y, int B, int CC, int Ch, int H, int W, int Ho,
                                                     int Wo) {
  constexpr int P = K / 2;
  const int64_t n = (int64_t)B * CC * Ho * Wo;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int ox = (int)(e % Wo);
    const int64_t r = e / Wo;
    const int oy = (int)(r % Ho);
    const int64_t pl = r / Ho;                       // plane = b·CC + cc
    const int cc = (int)(pl % CC);
    const float* wk = wrow(w, wcs, Ch, cc, K * K);
    const T* xp = x + pl * H * W;
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - P + ky;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int ix = ox * S - P + kx;
        if (ix < 0 || ix >= W) continue;
        acc = fmaf(ld<T>(xp + iy * W + ix), wk[ky * K + kx], acc);
      }
    }
    st<T>(y + e, acc);
  }
}

template <typename T, int K, int S>
__global__ __launch_bounds__(256) void dw_bwd_data_kernel(const T* __restrict__ dy, const float* __restrict__ w,
                                                          int64_t wcs, T* __restrict__ dx, int B, int CC, int Ch, int H,
                                                          int W, int Ho, int Wo) {
  constexpr int P = K / 2;
  const int64_t n = (int64_t)B * CC * H * W;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int ix = (int)(e % W);
    const int64_t r = e / W;
    const int iy = (int)(r % H);
    const int64_t pl = r / H;
    const int cc = (int)(pl % CC);
    const float* wk = wrow(w, wcs, Ch, cc, K * K);
    const T* gp = dy + pl * Ho * Wo;
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ty = iy + P - ky;                    // = oy·S
      if (ty < 0 || ty % S) continue;
      const int oy = ty / S;
      if (oy >= Ho) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int tx = ix + P - kx;
        if (tx < 0 || tx % S) continue;
        const int ox = tx / S;
        if (ox >= Wo) continue;
        acc = fmaf(ld<T>(gp + oy * Wo + ox), wk[ky * K + kx], acc);
      }
    }
    st<T>(dx + e, acc);
  }
}

// one workgroup per stacked channel: dw[cc][tap] = Σ_b Σ_(oy,ox) dy·x (fixed per-thread order + fixed tree)
template <typename T, int K, int S>
// dw: dense [CC][K·K] (ocs = 0) or, ocs > 0, accumulated (+=) into client c = cc / Ch's gradient-arena rows
// [Ch][K·K] at dw + c·ocs (single writer per element: no atomics, deterministic)
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       float* __restrict__ dw, int B, int CC, int H, int W, int Ho,
                                                       int Wo, int Ch, int64_t ocs) {
  constexpr int P = K / 2, KK = K * K;
  __shared__ float red[4][KK];
  const int cc = blockIdx.x;
  float acc[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) acc[t] = 0.f;
  const int per = Ho * Wo;
  for (int64_t i = threadIdx.x; i < (int64_t)B * per; i += 256) {
    const int b = (int)(i / per), q = (int)(i - (int64_t)b * per);
    const int oy = q / Wo, ox = q - oy * Wo;
    const int64_t pl = (int64_t)b * CC + cc;
    const float g = ld<T>(dy + pl * per + q);
    const T* xp = x + pl * H * W;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - P + ky;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int ix = ox * S - P + kx;
        const bool in = iy >= 0 && iy < H && ix >= 0 && ix < W;
        acc[ky * K + kx] = fmaf(g, in ? ld<T>(xp + iy * W + ix) : 0.f, acc[ky * K + kx]);
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    const float s = wave_sum(acc[t]);
    if (lane == 0) red[wv][t] = s;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < KK; t += 256) {
    const float v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    if (ocs > 0)
      dw[(int64_t)(cc / Ch) * ocs + (int64_t)(cc % Ch) * KK + t] += v;
    else
      dw[(int64_t)cc * KK + t] = v;
  }
}

// ---- BatchNorm over planes: channel cc's elements are B planes of HW at stride CC·HW ----
__device__ __forceinline__ float block_sum4(float v, float* sh) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// running statistics of the BN's arena rows (client stride rcs), updated like torch's training-mode BN
// (momentum, unbiased variance, num_batches_tracked) for active clients; null rm: no update
struct PbnRun {
  float* rm;
  float* rv;
  float* nbt;
  int64_t rcs;
  float momentum;
  const float* active;
  int Ch;
};

template <typename T>
__global__ __launch_bounds__(256) void pbn_stats_kernel(const T* __restrict__ x, float* __restrict__ mean,
                                                        float* __restrict__ var, int B, int CC, int HW, PbnRun run) {
  __shared__ float sh[4];
  const int cc = blockIdx.x;
  const float k = ld<T>(x + (int64_t)cc * HW);      // shift: the channel's first element (cancellation guard)
  float s = 0.f, s2 = 0.f;
  for (int64_t i = threadIdx.x; i < (int64_t)B * HW; i += 256) {
    const int b = (int)(i / HW), q = (int)(i - (int64_t)b * HW);
    const float v = ld<T>(x + ((int64_t)b * CC + cc) * HW + q) - k;
    s += v;
    s2 = fmaf(v, v, s2);
  }
  const float n = (float)B * HW;
  const float S = block_sum4(s, sh);
  const float S2 = block_sum4(s2, sh);
  if (threadIdx.x == 0) {
    const float m = S / n;
    const float mu = k + m, v = fmaxf(S2 / n - m * m, 0.f);
    mean[cc] = mu;
    var[cc] = v;
    if (run.rm) {
      const int c = cc / run.Ch, ch = cc - c * run.Ch;
      if (!run.active || run.active[c] > 0.f) {
        const int64_t o = (int64_t)c * run.rcs + ch;
        const float mom = run.momentum;
        run.rm[o] = (1.f - mom) * run.rm[o] + mom * mu;
        run.rv[o] = (1.f - mom) * run.rv[o] + mom * (v * (n / fmaxf(n - 1.f, 1.f)));
        if (run.nbt && ch == 0) run.nbt[(int64_t)c * run.rcs] += 1.f;
      }
    }
  }
}

// s/t from (γ, β) of the arena rows (client stride pcs; null γ/β: no affine) and the batch statistics
__device__ __forceinline__ void pbn_affine(int cc, int Ch, const float* g, const float* b, int64_t pcs,
                                           const float* mean, const float* var, float eps, float& s, float& t) {
  const int64_t o = (int64_t)(cc / Ch) * pcs + cc % Ch;
  const float rs = rsqrtf(var[cc] + eps);
  s = (g ? g[o] : 1.f) * rs;
  t = (b ? b[o] : 0.f) - mean[cc] * s;
}

template <typename T>
__global__ __launch_bounds__(256) void pbn_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                        const float* __restrict__ g, const float* __restrict__ bb,
                                                        int64_t pcs, const float* __restrict__ mean,
                                                        const float* __restrict__ var, float eps, int relu, int B,
                                                        int CC, int Ch, int HW) {
  const int64_t n = (int64_t)B * CC * HW;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int cc = (int)((e / HW) % CC);
    float s, t;
    pbn_affine(cc, Ch, g, bb, pcs, mean, var, eps, s, t);
    float v = fmaf(ld<T>(x + e), s, t);
    if (relu) v = fmaxf(v, 0.f);
    st<T>(y + e, v);
  }
}

// red[cc] = (Σg', Σg'·(x − μ)), g' = g·[relu ⇒ x·s + t > 0]
template <typename T>
__global__ __launch_bounds__(256) void pbn_bwd_red_kernel(const T* __restrict__ gy, const T* __restrict__ x,
                                                          const float* __restrict__ g, const float* __restrict__ bb,
                                                          int64_t pcs, const float* __restrict__ mean,
                                                          const float* __restrict__ var, float eps, int relu,
                                                          float* __restrict__ red, int B, int CC, int Ch, int HW,
                                                          float* __restrict__ dg, float* __restrict__ db, int64_t dcs) {
  __shared__ float sh[4];
  const int cc = blockIdx.x;
  float s, t;
  pbn_affine(cc, Ch, g, bb, pcs, mean, var, eps, s, t);
  const float m = mean[cc];
  float a = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < (int64_t)B * HW; i += 256) {
    const int b = (int)(i / HW), q = (int)(i - (int64_t)b * HW);
    const int64_t o = ((int64_t)b * CC + cc) * HW + q;
    const float xv = ld<T>(x + o);
    float gv = ld<T>(gy + o);
    if (relu && !(fmaf(xv, s, t) > 0.f)) gv = 0.f;
    a += gv;
    c = fmaf(gv, xv - m, c);
  }
  const float A = block_sum4(a, sh);
  const float Cs = block_sum4(c, sh);
  if (threadIdx.x == 0) {
    red[2 * cc] = A;
    red[2 * cc + 1] = Cs;
    // dγ = Σg'·x̂ = rs·Σg'(x − μ), dβ = Σg' straight into the gradient arena rows (single writer per element)
    const int64_t o = (int64_t)(cc / Ch) * dcs + cc % Ch;
    if (dg) dg[o] += Cs * rsqrtf(var[cc] + eps);
    if (db) db[o] += A;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pbn_dx_kernel(const T* __restrict__ gy, const T* __restrict__ x,
                                                     T* __restrict__ dx, const float* __restrict__ g,
                                                     const float* __restrict__ bb, int64_t pcs,
                                                     const float* __restrict__ mean, const float* __restrict__ var,
                                                     float eps, int relu, const float* __restrict__ red, int B, int CC,
                                                     int Ch, int HW) {
  const int64_t n = (int64_t)B * CC * HW;
  const float inv_n = 1.f / ((float)B * HW);
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int cc = (int)((e / HW) % CC);
    float s, t;
    pbn_affine(cc, Ch, g, bb, pcs, mean, var, eps, s, t);
    const float rs = rsqrtf(var[cc] + eps);
    const float xv = ld<T>(x + e);
    float gv = ld<T>(gy + e);
    if (relu && !(fmaf(xv, s, t) > 0.f)) gv = 0.f;
    const float xh = (xv - mean[cc]) * rs;
    // Σg'·x̂ = rs·Σg'(x − μ)
    st<T>(dx + e, s * (gv - red[2 * cc] * inv_n - xh * (rs * red[2 * cc + 1]) * inv_n));
  }
}

template <typename T>
int dw_dispatch(int op, const void* a, const void* b, const float* w, int64_t wcs, void* out, int B, int CC, int Ch,
                int H, int W, int Ho, int Wo, int K, int S, hipStream_t st) {
  const int64_t no = (int64_t)B * CC * Ho * Wo, ni = (int64_t)B * CC * H * W;
#define DW_CASE(KK_, SS_)                                                                                          \
  if (K == KK_ && S == SS_) {                                                                                      \
    if (op == 0)                                                                                                   \
      hipLaunchKernelGGL((dw_fwd_kernel<T, KK_, SS_>), dim3(fa_grid(no, 256, 16384)), dim3(256), 0, st,            \
                         (const T*)a, w, wcs, (T*)out, B, CC, Ch, H, W, Ho, Wo);                                   \
    else if (op == 1)                                                                                              \
      hipLaunchKernelGGL((dw_bwd_data_kernel<T, KK_, SS_>), dim3(fa_grid(ni, 256, 16384)), dim3(256), 0, st,       \
                         (const T*)a, w, wcs, (T*)out, B, CC, Ch, H, W, Ho, Wo);                                   \
    else                                                                                                           \
      hipLaunchKernelGGL((dw_wgrad_kernel<T, KK_, SS_>), dim3(CC), dim3(256), 0, st, (const T*)a, (const T*)b,     \
                         (float*)out, B, CC, H, W, Ho, Wo, Ch, wcs);                                               \
    return (int)hipGetLastError();                                                                                 \
  }
  DW_CASE(3, 1) DW_CASE(3, 2) DW_CASE(5, 1) DW_CASE(5, 2) DW_CASE(7, 1) DW_CASE(7, 2)
#undef DW_CASE
  return -2;
}

}  // namespace pk

// op 0: y = dw_fwd(x=a); 1: dx = dw_bwd_data(dy=a); 2: dw [CC][K·K] = dw_wgrad(dy=a, x=b), or with wcs > 0
// dw += into client-strided gradient-arena rows (out = client 0's [Ch][1][K][K] grad rows, client stride wcs).
// w: fp32 arena view of client 0's [Ch][1][K][K] rows, client stride wcs. Pad = K/2 (the reference's depthwise
// layers). is_bf16: T.
FA_EXPORT int fa_dwconv(int op, int is_bf16, const void* a, const void* b, const float* w, int64_t wcs, void* out,
                        int B, int CC, int Ch, int H, int W, int Ho, int Wo, int K, int S, hipStream_t stream) {
  if (is_bf16) return pk::dw_dispatch<uint16_t>(op, a, b, w, wcs, out, B, CC, Ch, H, W, Ho, Wo, K, S, stream);
  return pk::dw_dispatch<float>(op, a, b, w, wcs, out, B, CC, Ch, H, W, Ho, Wo, K, S, stream);
}

// op 0: stats (mean, var) of x; 1: y = act(x·s + t); 2: bwd reduce of (gy, x) into red [CC][2]; 3: dx.
// ext (optional, may be null): op 0 — running-statistics update {rm, rv, nbt, rcs, momentum, active, Ch};
// op 2 — dγ / dβ accumulated into the gradient arena {dg, db, dcs}
struct PbnExt {
  float* rm;
  float* rv;
  float* nbt;
  int64_t rcs;
  float momentum;
  const float* active;
  float* dg;
  float* db;
  int64_t dcs;
};

FA_EXPORT int fa_plane_bn(int op, int is_bf16, const void* x, const void* gy, void* out, const float* g,
                          const float* bb, int64_t pcs, float* mean, float* var, float eps, int relu, float* red, int B,
                          int CC, int Ch, int HW, const PbnExt* ext, hipStream_t stream) {
  const int64_t n = (int64_t)B * CC * HW;
  const unsigned grid = (unsigned)fa_grid(n, 256, 16384);
  pk::PbnRun run = {nullptr, nullptr, nullptr, 0, 0.f, nullptr, Ch};
  float* dg = nullptr;
  float* db = nullptr;
  int64_t dcs = 0;
  if (ext) {
    run.rm = ext->rm; run.rv = ext->rv; run.nbt = ext->nbt; run.rcs = ext->rcs; run.momentum = ext->momentum;
    run.active = ext->active;
    dg = ext->dg; db = ext->db; dcs = ext->dcs;
  }
#define PBN(T)                                                                                                     \
  switch (op) {                                                                                                    \
    case 0: hipLaunchKernelGGL(pk::pbn_stats_kernel<T>, dim3(CC), dim3(256), 0, stream, (const T*)x, mean, var, B, \
                               CC, HW, run); break;                                                               \
    case 1: hipLaunchKernelGGL(pk::pbn_apply_kernel<T>, dim3(grid), dim3(256), 0, stream, (const T*)x, (T*)out, g, \
                               bb, pcs, mean, var, eps, relu, B, CC, Ch, HW); break;                              \
    case 2: hipLaunchKernelGGL(pk::pbn_bwd_red_kernel<T>, dim3(CC), dim3(256), 0, stream, (const T*)gy,           \
                               (const T*)x, g, bb, pcs, mean, var, eps, relu, red, B, CC, Ch, HW, dg, db, dcs);   \
      break;                                                                                                       \
    case 3: hipLaunchKernelGGL(pk::pbn_dx_kernel<T>, dim3(grid), dim3(256), 0, stream, (const T*)gy, (const T*)x,  \
                               (T*)out, g, bb, pcs, mean, var, eps, relu, red, B, CC, Ch, HW); break;             \
    default: return -2;                                                                                            \
  }
  if (is_bf16) { PBN(uint16_t) } else { PBN(float) }
#undef PBN
  return (int)hipGetLastError();
}
