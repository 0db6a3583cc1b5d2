// GroupNorm and max-pool for the client-batched NHWC activations of the native ResNet-GN step
// (parallel/native_resnet_gn.py; reference: model/cv/resnet_gn.py:187-239, model/cv/group_normalization.py:7-93,
// where GroupNorm is built from F.batch_norm on a reshaped [1, N·G, ...] copy).
//
// Layout: act [C][N][HW][Ch] (client-stacked NHWC, bf16 or fp32 storage per prec.h), per-client affine parameters
// read in place from the fp32 client arena (row stride ldw). One 256-thread workgroup per (image, client) holds the
// whole image in registers (≤ 16 quads of 4 channels per thread: HW·Ch ≤ 16384), so mean, variance and the
// normalised output need ONE read of the input. A thread's channels are the same in every quad it holds
// (Ch | 1024), so its group is fixed and group sums are fixed-order reductions (deterministic, no atomics):
//
//   gnh_fwd   mean / rstd per (client, image, group) → out = act(γ·x̂ + β [+ residual])  (act: ReLU or none)
//   gnh_bwd   g' = upstream ⊙ [out > 0] (ReLU'd GN) ; dx = rstd·(g'γ − mean(g'γ) − x̂·mean(g'γ·x̂)) per group;
//             per-image dγ / dβ partials (Σ g'·x̂, Σ g') → gnh_param_reduce adds them into the gradient arena
//             (images in order: deterministic)
//   maxpool   k×k / stride / pad forward with the arg-max tap per output (uint8) and the backward as a gather
//             over the ≤ ⌈k/s⌉² windows that cover an input pixel (fixed order, no atomics).
#include "prec.h"

namespace gnh {

constexpr int NT = 256;
constexpr int MAXQ = 16;

struct GnArgs {
  const void* x;        // GN input (pre-norm) [C][N][HW][Ch]
  const void* res;      // forward: residual added after the affine (or null)
  void* out;            // forward: output | backward: dx
  const void* go;       // backward: upstream gradient
  const void* act;      // backward: the forward's post-ReLU output (ReLU mask), or null
  float* ms;            // [C][N][G][2] mean, rstd (written by forward, read by backward)
  float* pscr;          // backward: [C][N][2][Ch] per-image Σ g'·x̂, Σ g'
  const float* arena;
  int64_t ldw, off_g, off_b;
  const int* nimg;
  int N, HW, Ch, G;
  float eps;
};

// Fixed-order sum over the threads of each group: members of group g are t = cyc·Qc + g·qg + j (Qc = Ch/4 threads
// per channel cycle, qg = cpg/4), wave w reduces groups w, w + 4, ...; gsum[g] = the group's total.
__device__ __forceinline__ void group_reduce(const float* part, float* gsum, int Ch, int G) {
  const int Qc = Ch / 4, qg = Qc / G, M = NT / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int g = w; g < G; g += NT / 64) {
    float s = 0.f;
    for (int m = lane; m < M; m += 64) s += part[(m / qg) * Qc + g * qg + (m % qg)];
    s = wave_sum(s);
    if (lane == 0) gsum[g] = s;
  }
}

template <class P, int RELU, int RES>
__global__ __launch_bounds__(NT) void gnh_fwd_kernel(GnArgs a) {
  using T = typename P::T;
  __shared__ float part[NT];
  __shared__ float gs[64];
  const int n = blockIdx.x, c = blockIdx.y;
  if (a.nimg && n >= a.nimg[c]) return;
  const int t = threadIdx.x;
  const int Q = a.HW * a.Ch / 4, cpg = a.Ch / a.G;
  const int ch0 = (t * 4) % a.Ch, g = ch0 / cpg;
  const int64_t base = ((int64_t)c * a.N + n) * a.HW * a.Ch;
  const T* x = reinterpret_cast<const T*>(a.x) + base;
  float v[MAXQ][4];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int i = t + q * NT;
    if (i < Q) {
      P::load4(x + 4 * i, v[q]);
      s += (v[q][0] + v[q][1]) + (v[q][2] + v[q][3]);
    } else {
      v[q][0] = v[q][1] = v[q][2] = v[q][3] = 0.f;
    }
  }
  part[t] = s;
  __syncthreads();
  group_reduce(part, gs, a.Ch, a.G);
  __syncthreads();
  const float inv = 1.f / (float)(a.HW * cpg);
  const float mean = gs[g] * inv;
  float q2 = 0.f;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q)
    if (t + q * NT < Q)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[q][j] - mean;
        q2 += d * d;
      }
  __syncthreads();
  part[t] = q2;
  __syncthreads();
  group_reduce(part, gs + 32, a.Ch, a.G);   // gs[32 + g]: Σ (x − mean)² (G ≤ 32)
  __syncthreads();
  const float rstd = rsqrtf(gs[32 + g] * inv + a.eps);
  if (t < a.G) {
    float* m = a.ms + (((int64_t)c * a.N + n) * a.G + t) * 2;
    m[0] = gs[t] * inv;
    m[1] = rsqrtf(gs[32 + t] * inv + a.eps);
  }
  const float* pa = a.arena + (int64_t)c * a.ldw;
  float sc[4], sh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sc[j] = (a.off_g >= 0 ? pa[a.off_g + ch0 + j] : 1.f) * rstd;
    sh[j] = (a.off_b >= 0 ? pa[a.off_b + ch0 + j] : 0.f) - mean * sc[j];
  }
  T* out = reinterpret_cast<T*>(a.out) + base;
  const T* res = RES ? reinterpret_cast<const T*>(a.res) + base : nullptr;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int i = t + q * NT;
    if (i < Q) {
      float o[4], r[4];
      if (RES) P::load4(res + 4 * i, r);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float y = v[q][j] * sc[j] + sh[j];
        if (RES) y += r[j];
        o[j] = RELU ? fmaxf(y, 0.f) : y;
      }
      P::store4(out + 4 * i, o);
    }
  }
}

template <class P, int RELU>
__global__ __launch_bounds__(NT) void gnh_bwd_kernel(GnArgs a) {
  using T = typename P::T;
  __shared__ float part[NT];
  __shared__ float gs[64];
  __shared__ float cpart[2][NT][4];
  const int n = blockIdx.x, c = blockIdx.y;
  if (a.nimg && n >= a.nimg[c]) return;
  const int t = threadIdx.x;
  const int Q = a.HW * a.Ch / 4, cpg = a.Ch / a.G;
  const int ch0 = (t * 4) % a.Ch, g = ch0 / cpg;
  const int64_t base = ((int64_t)c * a.N + n) * a.HW * a.Ch;
  const T* x = reinterpret_cast<const T*>(a.x) + base;
  const T* go = reinterpret_cast<const T*>(a.go) + base;
  const T* ac = RELU ? reinterpret_cast<const T*>(a.act) + base : nullptr;
  const float* m = a.ms + (((int64_t)c * a.N + n) * a.G + g) * 2;
  const float mean = m[0], rstd = m[1];
  const float* pa = a.arena + (int64_t)c * a.ldw;
  float gam[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) gam[j] = a.off_g >= 0 ? pa[a.off_g + ch0 + j] : 1.f;
  float xh[MAXQ][4], dh[MAXQ][4];
  float sA = 0.f, sB = 0.f, cg[4] = {0.f, 0.f, 0.f, 0.f}, cb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int i = t + q * NT;
    if (i < Q) {
      float xv[4], gv[4], av[4];
      P::load4(x + 4 * i, xv);
      P::load4(go + 4 * i, gv);
      if (RELU) P::load4(ac + 4 * i, av);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gm = (RELU && !(av[j] > 0.f)) ? 0.f : gv[j];
        xh[q][j] = (xv[j] - mean) * rstd;
        dh[q][j] = gm * gam[j];
        sA += dh[q][j];
        sB += dh[q][j] * xh[q][j];
        cg[j] += gm * xh[q][j];
        cb[j] += gm;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) xh[q][j] = dh[q][j] = 0.f;
    }
  }
  part[t] = sA;
  __syncthreads();
  group_reduce(part, gs, a.Ch, a.G);
  __syncthreads();
  part[t] = sB;
  __syncthreads();
  group_reduce(part, gs + 32, a.Ch, a.G);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cpart[0][t][j] = cg[j];
    cpart[1][t][j] = cb[j];
  }
  __syncthreads();
  const float inv = 1.f / (float)(a.HW * cpg);
  const float mA = gs[g] * inv, mB = gs[32 + g] * inv;
  T* dx = reinterpret_cast<T*>(a.out) + base;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int i = t + q * NT;
    if (i < Q) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rstd * (dh[q][j] - mA - xh[q][j] * mB);
      P::store4(dx + 4 * i, o);
    }
  }
  // per-image dγ / dβ of this thread's 4 channels: the threads holding them are t + cyc·Qc
  const int Qc = a.Ch / 4;
  if (t < Qc) {
    float sg[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
    for (int u = t; u < NT; u += Qc)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sg[j] += cpart[0][u][j];
        sb[j] += cpart[1][u][j];
      }
    float* ps = a.pscr + ((int64_t)c * a.N + n) * 2 * a.Ch;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ps[ch0 + j] = sg[j];
      ps[a.Ch + ch0 + j] = sb[j];
    }
  }
}

// garena[c][off_g + ch] += Σ_n<nimg pscr[c][n][0][ch]; [off_b + ch] += Σ pscr[c][n][1][ch]  (images in order)
__global__ __launch_bounds__(NT) void gnh_param_reduce_kernel(const float* __restrict__ pscr, float* __restrict__ garena,
                                                              int64_t ldw, int64_t off_g, int64_t off_b, int N, int Ch,
                                                              const int* __restrict__ nimg) {
  const int c = blockIdx.y;
  const int k = blockIdx.x * NT + threadIdx.x;     // 0 .. 2·Ch
  if (k >= 2 * Ch) return;
  const int Ne = nimg ? min(N, nimg[c]) : N;
  float s = 0.f;
  for (int n = 0; n < Ne; ++n) s += pscr[((int64_t)c * N + n) * 2 * Ch + k];
  const int64_t off = k < Ch ? off_g + k : off_b + (k - Ch);
  if ((k < Ch ? off_g : off_b) >= 0) garena[(int64_t)c * ldw + off] += s;
}

// ---- max-pool k×k / stride s / pad p (NHWC); one thread per output quad of 4 channels
template <class P>
__global__ __launch_bounds__(NT) void maxpool_fwd_kernel(const typename P::T* __restrict__ x,
                                                         typename P::T* __restrict__ y, uint8_t* __restrict__ idx,
                                                         int C, int N, int H, int W, int Ch, int Ho, int Wo, int k,
                                                         int s, int p, const int* __restrict__ nimg) {
  const int64_t qi = (int64_t)blockIdx.x * NT + threadIdx.x;
  const int Qc = Ch / 4;
  const int64_t total = (int64_t)N * Ho * Wo * Qc;
  const int c = blockIdx.y;
  if (qi >= total) return;
  const int q = (int)(qi % Qc);
  const int64_t pix = qi / Qc;
  const int n = (int)(pix / ((int64_t)Ho * Wo));
  if (nimg && n >= nimg[c]) return;
  const int r = (int)(pix % ((int64_t)Ho * Wo));
  const int oh = r / Wo, ow = r % Wo;
  float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int arg[4] = {0, 0, 0, 0};
  const typename P::T* xc = x + ((int64_t)c * N + n) * H * W * Ch + 4 * q;
  for (int kh = 0; kh < k; ++kh) {
    const int ih = oh * s - p + kh;
    if (ih < 0 || ih >= H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int iw = ow * s - p + kw;
      if (iw < 0 || iw >= W) continue;
      float v[4];
      P::load4(xc + ((int64_t)ih * W + iw) * Ch, v);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {   // NaN propagates, like torch
          best[j] = v[j];
          arg[j] = kh * k + kw;
        }
    }
  }
  const int64_t o = ((int64_t)c * N * Ho * Wo + pix) * Ch + 4 * q;
  P::store4(y + o, best);
#pragma unroll
  for (int j = 0; j < 4; ++j) idx[o + j] = (uint8_t)arg[j];
}

template <class P>
__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(const typename P::T* __restrict__ gy,
                                                         const uint8_t* __restrict__ idx,
                                                         typename P::T* __restrict__ gx, int C, int N, int H, int W,
                                                         int Ch, int Ho, int Wo, int k, int s, int p,
                                                         const int* __restrict__ nimg) {
  const int64_t qi = (int64_t)blockIdx.x * NT + threadIdx.x;
  const int Qc = Ch / 4;
  const int64_t total = (int64_t)N * H * W * Qc;
  const int c = blockIdx.y;
  if (qi >= total) return;
  const int q = (int)(qi % Qc);
  const int64_t pix = qi / Qc;
  const int n = (int)(pix / ((int64_t)H * W));
  if (nimg && n >= nimg[c]) return;
  const int r = (int)(pix % ((int64_t)H * W));
  const int ih = r / W, iw = r % W;
  const int oh_lo = max(0, (ih + p - k + s) / s), oh_hi = min(Ho - 1, (ih + p) / s);
  const int ow_lo = max(0, (iw + p - k + s) / s), ow_hi = min(Wo - 1, (iw + p) / s);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ob = (int64_t)c * N * Ho * Wo + (int64_t)n * Ho * Wo;
  for (int oh = oh_lo; oh <= oh_hi; ++oh)
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int tap = (ih + p - oh * s) * k + (iw + p - ow * s);
      const int64_t o = (ob + (int64_t)oh * Wo + ow) * Ch + 4 * q;
      float g[4];
      P::load4(gy + o, g);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (idx[o + j] == tap) acc[j] += g[j];
    }
  P::store4(gx + ((int64_t)c * N * H * W + pix) * Ch + 4 * q, acc);
}

template <class P>
static int gn_fwd(GnArgs a, int C, int relu, hipStream_t st) {
  if (a.Ch % 4 || 1024 % a.Ch || a.G < 1 || a.G > 32 || a.Ch % a.G || (a.Ch / a.G) % 4 ||
      (int64_t)a.HW * a.Ch > (int64_t)4 * MAXQ * NT)
    return -3;
  dim3 grid(a.N, C);
  if (relu && a.res) hipLaunchKernelGGL((gnh_fwd_kernel<P, 1, 1>), grid, dim3(NT), 0, st, a);
  else if (relu) hipLaunchKernelGGL((gnh_fwd_kernel<P, 1, 0>), grid, dim3(NT), 0, st, a);
  else if (a.res) hipLaunchKernelGGL((gnh_fwd_kernel<P, 0, 1>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((gnh_fwd_kernel<P, 0, 0>), grid, dim3(NT), 0, st, a);
  return (int)hipGetLastError();
}

template <class P>
static int gn_bwd(GnArgs a, int C, hipStream_t st) {
  if (a.Ch % 4 || 1024 % a.Ch || a.G < 1 || a.G > 32 || a.Ch % a.G || (a.Ch / a.G) % 4 ||
      (int64_t)a.HW * a.Ch > (int64_t)4 * MAXQ * NT)
    return -3;
  dim3 grid(a.N, C);
  if (a.act) hipLaunchKernelGGL((gnh_bwd_kernel<P, 1>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((gnh_bwd_kernel<P, 0>), grid, dim3(NT), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace gnh

using gnh::GnArgs;

static GnArgs gn_args(const void* x, const void* res, void* out, const void* go, const void* act, float* ms, float* pscr,
                      const float* arena, int64_t ldw, int64_t off_g, int64_t off_b, const int* nimg, int N, int HW,
                      int Ch, int G, float eps) {
  GnArgs a;
  a.x = x; a.res = res; a.out = out; a.go = go; a.act = act; a.ms = ms; a.pscr = pscr; a.arena = arena; a.ldw = ldw;
  a.off_g = off_g; a.off_b = off_b; a.nimg = nimg; a.N = N; a.HW = HW; a.Ch = Ch; a.G = G; a.eps = eps;
  return a;
}

FA_EXPORT int fa_gnh_fwd(int bf16, const void* x, const void* res, void* out, float* ms, const float* arena,
                         int64_t ldw, int64_t off_g, int64_t off_b, const int* nimg, int C, int N, int HW, int Ch,
                         int G, float eps, int relu, hipStream_t st) {
  GnArgs a = gn_args(x, res, out, nullptr, nullptr, ms, nullptr, arena, ldw, off_g, off_b, nimg, N, HW, Ch, G, eps);
  return bf16 ? gnh::gn_fwd<prec::BF16>(a, C, relu, st) : gnh::gn_fwd<prec::F32>(a, C, relu, st);
}

FA_EXPORT int fa_gnh_bwd(int bf16, const void* x, const void* go, const void* act, void* dx, const float* ms,
                         float* pscr, const float* arena, int64_t ldw, int64_t off_g, const int* nimg, int C, int N,
                         int HW, int Ch, int G, hipStream_t st) {
  GnArgs a = gn_args(x, nullptr, dx, go, act, const_cast<float*>(ms), pscr, arena, ldw, off_g, -1, nimg, N, HW, Ch,
                     G, 0.f);
  return bf16 ? gnh::gn_bwd<prec::BF16>(a, C, st) : gnh::gn_bwd<prec::F32>(a, C, st);
}

FA_EXPORT int fa_gnh_param_reduce(const float* pscr, float* garena, int64_t ldw, int64_t off_g, int64_t off_b, int C,
                                  int N, int Ch, const int* nimg, hipStream_t st) {
  hipLaunchKernelGGL(gnh::gnh_param_reduce_kernel, dim3((2 * Ch + gnh::NT - 1) / gnh::NT, C), dim3(gnh::NT), 0, st,
                     pscr, garena, ldw, off_g, off_b, N, Ch, nimg);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_maxpool_fwd(int bf16, const void* x, void* y, uint8_t* idx, int C, int N, int H, int W, int Ch, int Ho,
                             int Wo, int k, int s, int p, const int* nimg, hipStream_t st) {
  if (Ch % 4 || k * k > 255) return -3;
  const int64_t total = (int64_t)N * Ho * Wo * (Ch / 4);
  dim3 grid((unsigned)((total + gnh::NT - 1) / gnh::NT), C);
  if (bf16)
    hipLaunchKernelGGL(gnh::maxpool_fwd_kernel<prec::BF16>, grid, dim3(gnh::NT), 0, st, (const uint16_t*)x,
                       (uint16_t*)y, idx, C, N, H, W, Ch, Ho, Wo, k, s, p, nimg);
  else
    hipLaunchKernelGGL(gnh::maxpool_fwd_kernel<prec::F32>, grid, dim3(gnh::NT), 0, st, (const float*)x, (float*)y, idx,
                       C, N, H, W, Ch, Ho, Wo, k, s, p, nimg);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_maxpool_bwd(int bf16, const void* gy, const uint8_t* idx, void* gx, int C, int N, int H, int W,
                             int Ch, int Ho, int Wo, int k, int s, int p, const int* nimg, hipStream_t st) {
  if (Ch % 4 || k * k > 255) return -3;
  const int64_t total = (int64_t)N * H * W * (Ch / 4);
  dim3 grid((unsigned)((total + gnh::NT - 1) / gnh::NT), C);
  if (bf16)
    hipLaunchKernelGGL(gnh::maxpool_bwd_kernel<prec::BF16>, grid, dim3(gnh::NT), 0, st, (const uint16_t*)gy, idx,
                       (uint16_t*)gx, C, N, H, W, Ch, Ho, Wo, k, s, p, nimg);
  else
    hipLaunchKernelGGL(gnh::maxpool_bwd_kernel<prec::F32>, grid, dim3(gnh::NT), 0, st, (const float*)gy, idx,
                       (float*)gx, C, N, H, W, Ch, Ho, Wo, k, s, p, nimg);
  return (int)hipGetLastError();
}
