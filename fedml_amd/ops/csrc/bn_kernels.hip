// Per-(client, channel) BatchNorm finalisation, fused block epilogues and small layout kernels
// for the native client-batched ResNet executor. Layout as in conv_kernels.hip:
// activations [C][N][H][W][Ch] bf16 | fp32 (`_f32` entry points); vectors [C][Ch] fp32; parameters/grads in the client-stacked
// fp32 arenas [C][ldw] addressed by offset.
#include "prec.h"
#include "detacc.h"
#include "bnlazy.h"

FA_DET_EXPORT(bn)

using prec::BF16;
using prec::F32;

// ---- forward finalisation: statistics → folded scale/shift, running-stat update ----
// stats[c][ch][2] = (Σy, Σy²) over n = N·H·W elements of client c, of the STORED activation
// y = conv − K (K = pivot[c][ch], null → 0; the conv epilogue subtracted it). Everything downstream
// works on the stored values: scale = γ·rstd, shift = β − mean_s·scale with mean_s = mean(y), saved
// with rstd for the backward. The true mean (mean_s + K) feeds the running statistics and becomes the
// next step's pivot (written back into `pivot`), so the stored activations stay centred near 0.
// Running statistics (torch semantics: unbiased variance, momentum) and num_batches_tracked
// are updated in the parameter arena for ACTIVE clients only.
__global__ void bn_fwd_finalize_kernel(const float* __restrict__ stats, int Ch, float n, float* __restrict__ arena,
                                       int64_t ldw, int64_t off_gamma, int64_t off_beta, int64_t off_rm,
                                       int64_t off_rv, int64_t off_nbt, float momentum, float eps,
                                       const float* __restrict__ active, float* __restrict__ scale,
                                       float* __restrict__ shift, float* __restrict__ mean_out,
                                       float* __restrict__ rstd_out, int update_running, float* __restrict__ pivot,
                                       const int* __restrict__ nimg, int hw) {
  const int c = blockIdx.y;
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= Ch) return;
  if (nimg) n = (float)nimg[c] * (float)hw;   // heterogeneous batches: this client's valid elements
  if (n <= 0.f) return;                       // client without data this step: nothing to normalise
  float* pa = arena + (int64_t)c * ldw;
  const int64_t v = (int64_t)c * Ch + ch;
  const float g = off_gamma >= 0 ? pa[off_gamma + ch] : 1.f;
  const float b = off_beta >= 0 ? pa[off_beta + ch] : 0.f;
  const BnFwdFold f = bn_fold_fwd(stats[v * 2 + 0], stats[v * 2 + 1], n, eps, g, b);   // shared with bnlazy.h
  const float k = pivot ? pivot[v] : 0.f;
  const float true_mean = __fadd_rn(f.mean, k);
  scale[v] = f.scale;
  shift[v] = f.shift;
  mean_out[v] = f.mean;
  rstd_out[v] = f.rstd;
  const bool on = active ? active[c] > 0.f : true;
  if (pivot && on) pivot[v] = true_mean;
  if (update_running && on) {
    if (off_rm >= 0) pa[off_rm + ch] = bn_running_update(pa[off_rm + ch], momentum, true_mean);
    if (off_rv >= 0) pa[off_rv + ch] = bn_running_update(pa[off_rv + ch], momentum, bn_unbiased(f.var, n));
    if (off_nbt >= 0 && ch == 0) pa[off_nbt] += 1.f;
  }
}

FA_EXPORT int fa_bn_fwd_finalize(const float* stats, int C, int Ch, float n, float* arena, int64_t ldw,
                                 int64_t off_gamma, int64_t off_beta, int64_t off_rm, int64_t off_rv, int64_t off_nbt,
                                 float momentum, float eps, const float* active, float* scale, float* shift,
                                 float* mean_out, float* rstd_out, int update_running, float* pivot, const int* nimg,
                                 int hw, hipStream_t stream) {
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((Ch + 63) / 64, C), dim3(64), 0, stream, stats, Ch, n, arena, ldw,
                     off_gamma, off_beta, off_rm, off_rv, off_nbt, momentum, eps, active, scale, shift, mean_out,
                     rstd_out, update_running, pivot, nimg, hw);
  return (int)hipGetLastError();
}

// ---- inference folding (eval mode: the running statistics, no batch statistics): scale = γ·rsqrt(rv + ε),
// shift = β − rm·scale per (client, channel) — the vectors every consumer kernel's BN prologue / block-output pass
// reads. Used by the native batched inference of many models at once (coalition valuation, core/valuation.py).
__global__ void bn_eval_fold_kernel(int Ch, const float* __restrict__ arena, int64_t ldw, int64_t off_gamma,
                                    int64_t off_beta, int64_t off_rm, int64_t off_rv, float eps,
                                    float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.y;
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= Ch) return;
  const float* pa = arena + (int64_t)c * ldw;
  const float g = off_gamma >= 0 ? pa[off_gamma + ch] : 1.f;
  const float b = off_beta >= 0 ? pa[off_beta + ch] : 0.f;
  const float s = g * rsqrtf(pa[off_rv + ch] + eps);
  scale[(int64_t)c * Ch + ch] = s;
  shift[(int64_t)c * Ch + ch] = b - pa[off_rm + ch] * s;
}

FA_EXPORT int fa_bn_eval_fold(int C, int Ch, const float* arena, int64_t ldw, int64_t off_gamma, int64_t off_beta,
                              int64_t off_rm, int64_t off_rv, float eps, float* scale, float* shift,
                              hipStream_t stream) {
  if (off_rm < 0 || off_rv < 0) return -3;
  hipLaunchKernelGGL(bn_eval_fold_kernel, dim3((Ch + 63) / 64, C), dim3(64), 0, stream, Ch, arena, ldw, off_gamma,
                     off_beta, off_rm, off_rv, eps, scale, shift);
  return (int)hipGetLastError();
}

// ---- backward finalisation: (Σg, Σg·y) → dγ, dβ into the gradient arena and the folded
// coefficients of dy = α·g + β·y + γc consumed by the conv backward kernels.
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ bstats, int NS, int q_gy, int Ch, float n,
                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                       const float* __restrict__ arena, float* __restrict__ garena, int64_t ldw,
                                       int64_t off_gamma, int64_t off_beta, float* __restrict__ alpha,
                                       float* __restrict__ beta_c, float* __restrict__ gamma_c,
                                       const int* __restrict__ nimg, int hw) {
  const int c = blockIdx.y;
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= Ch) return;
  if (nimg) n = (float)nimg[c] * (float)hw;
  if (n <= 0.f) return;
  const int64_t v = (int64_t)c * Ch + ch;
  const float g = off_gamma >= 0 ? arena[(int64_t)c * ldw + off_gamma + ch] : 1.f;
  const BnBwdFold f = bn_fold_bwd(bstats[v * NS + 0], bstats[v * NS + q_gy], mean[v], rstd[v], g, n);
  if (off_gamma >= 0) garena[(int64_t)c * ldw + off_gamma + ch] += f.dgamma;
  if (off_beta >= 0) garena[(int64_t)c * ldw + off_beta + ch] += f.dbeta;
  alpha[v] = f.a;
  beta_c[v] = f.b;
  gamma_c[v] = f.c;
}

FA_EXPORT int fa_bn_bwd_finalize(const float* bstats, int NS, int q_gy, int C, int Ch, float n, const float* mean,
                                 const float* rstd, const float* arena, float* garena, int64_t ldw, int64_t off_gamma,
                                 int64_t off_beta, float* alpha, float* beta_c, float* gamma_c, const int* nimg, int hw,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((Ch + 63) / 64, C), dim3(64), 0, stream, bstats, NS, q_gy, Ch, n,
                     mean, rstd, arena, garena, ldw, off_gamma, off_beta, alpha, beta_c, gamma_c, nimg, hw);
  return (int)hipGetLastError();
}

// ---- fused block output: out = relu(y·s + t + R), R = yd·sd + td (downsample) | x (identity) | 0
// One 16-B vector (P::VEC channels) per thread (no grid-stride loop, no 64-bit modulo); the
// per-channel vectors are read as float4 (L1-resident). Streams 3 tensors: HBM-bound by construction.
// UNR 16-B vectors per thread, 256 apart (coalesced), all loads issued before any math: ≥ 3 streams × UNR
// outstanding 16-B requests per lane keep HBM busy (one vector per thread reached ~2.6 TB/s on MI355X).
constexpr int kEwUnr = 4;

template <class P, int RES>
__global__ __launch_bounds__(256) void block_out_kernel(const typename P::T* __restrict__ y, const float* __restrict__ s,
                                                        const float* __restrict__ t,
                                                        const typename P::T* __restrict__ r,
                                                        const float* __restrict__ rs, const float* __restrict__ rt,
                                                        typename P::T* __restrict__ out, int nvec, int cg,
                                                        const int* __restrict__ nimg, int vec_per_img) {
  constexpr int V = P::VEC;
  const int c = blockIdx.y;
  const int lim = nimg ? min(nvec, nimg[c] * vec_per_img) : nvec;   // valid images of client c only
  const int v0 = blockIdx.x * (256 * kEwUnr) + threadIdx.x;
  if (v0 >= lim) return;
  const int64_t cbase = (int64_t)c * nvec * V;
  uint4 yv[kEwUnr], rv[kEwUnr];
#pragma unroll
  for (int u = 0; u < kEwUnr; ++u) {
    const int v = v0 + u * 256;
    yv[u] = make_uint4(0, 0, 0, 0);
    rv[u] = make_uint4(0, 0, 0, 0);
    if (v < lim) {
      yv[u] = *reinterpret_cast<const uint4*>(y + cbase + (int64_t)v * V);
      if (RES) rv[u] = *reinterpret_cast<const uint4*>(r + cbase + (int64_t)v * V);
    }
  }
#pragma unroll
  for (int u = 0; u < kEwUnr; ++u) {
    const int v = v0 + u * 256;
    if (v >= lim) break;
    const int64_t co = (int64_t)c * cg * V + (v % cg) * V;
    float f[V], g[V];
    P::unpack(yv[u], f);
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = f[j] * s[co + j] + t[co + j];
    if (RES) {
      P::unpack(rv[u], g);
      if (RES == 2) {
#pragma unroll
        for (int j = 0; j < V; ++j) f[j] += g[j] * rs[co + j] + rt[co + j];
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) f[j] += g[j];
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = fmaxf(f[j], 0.f);
    *reinterpret_cast<uint4*>(out + cbase + (int64_t)v * V) = P::pack(f);
  }
}

template <class P>
static int block_out(const void* y, const float* s, const float* t, const void* r, const float* rs, const float* rt,
                     void* out, int C, int64_t per_client, int Ch, const int* nimg, int per_img,
                     hipStream_t stream) {
  using T = typename P::T;
  constexpr int V = P::VEC;
  if (Ch % V != 0 || per_client / V > INT32_MAX - 256 * kEwUnr) return -3;
  const int nvec = (int)(per_client / V);
  dim3 grid((nvec + 256 * kEwUnr - 1) / (256 * kEwUnr), C);
  const T* y_ = (const T*)y;
  const T* r_ = (const T*)r;
  T* o_ = (T*)out;
  if (!r)
    hipLaunchKernelGGL((block_out_kernel<P, 0>), grid, dim3(256), 0, stream, y_, s, t, r_, rs, rt, o_, nvec, Ch / V,
                       nimg, per_img / V);
  else if (!rs)
    hipLaunchKernelGGL((block_out_kernel<P, 1>), grid, dim3(256), 0, stream, y_, s, t, r_, rs, rt, o_, nvec, Ch / V,
                       nimg, per_img / V);
  else
    hipLaunchKernelGGL((block_out_kernel<P, 2>), grid, dim3(256), 0, stream, y_, s, t, r_, rs, rt, o_, nvec, Ch / V,
                       nimg, per_img / V);
  return (int)hipGetLastError();
}

// per_img: elements of one image (H·W·Ch); nimg: per-client valid images (null: all)
FA_EXPORT int fa_block_out(const uint16_t* y, const float* s, const float* t, const uint16_t* r, const float* rs,
                           const float* rt, uint16_t* out, int C, int64_t per_client, int Ch, const int* nimg,
                           int per_img, hipStream_t stream) {
  return block_out<BF16>(y, s, t, r, rs, rt, out, C, per_client, Ch, nimg, per_img, stream);
}
FA_EXPORT int fa_block_out_f32(const float* y, const float* s, const float* t, const float* r, const float* rs,
                               const float* rt, float* out, int C, int64_t per_client, int Ch, const int* nimg,
                               int per_img, hipStream_t stream) {
  return block_out<F32>(y, s, t, r, rs, rt, out, C, per_client, Ch, nimg, per_img, stream);
}

// ---- materialised BN backward operand: dy = α·g + β·y + γ (per client and channel), valid images only.
// The wide-layer backward kernels then stream ONE tensor instead of two (g, y) and skip the transform —
// the weight-gradient kernel re-reads dy once per K-tile (36× for a 512-channel 3×3 layer).
template <class P>
__global__ __launch_bounds__(256) void dy_apply_kernel(const typename P::T* __restrict__ g,
                                                       const typename P::T* __restrict__ y, const float* __restrict__ a,
                                                       const float* __restrict__ b, const float* __restrict__ cg_,
                                                       typename P::T* __restrict__ out, int nvec, int cg,
                                                       const int* __restrict__ nimg, int vec_per_img) {
  constexpr int V = P::VEC;
  const int c = blockIdx.y;
  const int lim = nimg ? min(nvec, nimg[c] * vec_per_img) : nvec;
  const int v0 = blockIdx.x * (256 * kEwUnr) + threadIdx.x;
  if (v0 >= lim) return;
  const int64_t cbase = (int64_t)c * nvec * V;
  uint4 gv[kEwUnr], yv[kEwUnr];
#pragma unroll
  for (int u = 0; u < kEwUnr; ++u) {
    const int v = v0 + u * 256;
    gv[u] = yv[u] = make_uint4(0, 0, 0, 0);
    if (v < lim) {
      gv[u] = *reinterpret_cast<const uint4*>(g + cbase + (int64_t)v * V);
      yv[u] = *reinterpret_cast<const uint4*>(y + cbase + (int64_t)v * V);
    }
  }
#pragma unroll
  for (int u = 0; u < kEwUnr; ++u) {
    const int v = v0 + u * 256;
    if (v >= lim) break;
    const int64_t co = (int64_t)c * cg * V + (v % cg) * V;
    float f[V], h[V];
    P::unpack(gv[u], f);
    P::unpack(yv[u], h);
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = a[co + j] * f[j] + b[co + j] * h[j] + cg_[co + j];
    *reinterpret_cast<uint4*>(out + cbase + (int64_t)v * V) = P::pack(f);
  }
}

template <class P>
static int dy_apply(const void* g, const void* y, const float* a, const float* b, const float* cc, void* out, int C,
                    int64_t per_client, int Ch, const int* nimg, int per_img, hipStream_t stream) {
  using T = typename P::T;
  constexpr int V = P::VEC;
  if (Ch % V != 0 || per_client / V > INT32_MAX - 256 * kEwUnr) return -3;
  const int nvec = (int)(per_client / V);
  hipLaunchKernelGGL(dy_apply_kernel<P>, dim3((nvec + 256 * kEwUnr - 1) / (256 * kEwUnr), C), dim3(256), 0, stream,
                     (const T*)g, (const T*)y, a, b, cc, (T*)out, nvec, Ch / V, nimg, per_img / V);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_dy_apply(const uint16_t* g, const uint16_t* y, const float* a, const float* b, const float* c,
                          uint16_t* out, int C, int64_t per_client, int Ch, const int* nimg, int per_img,
                          hipStream_t stream) {
  return dy_apply<BF16>(g, y, a, b, c, out, C, per_client, Ch, nimg, per_img, stream);
}
FA_EXPORT int fa_dy_apply_f32(const float* g, const float* y, const float* a, const float* b, const float* c,
                              float* out, int C, int64_t per_client, int Ch, const int* nimg, int per_img,
                              hipStream_t stream) {
  return dy_apply<F32>(g, y, a, b, c, out, C, per_client, Ch, nimg, per_img, stream);
}

// ---- global average pool (forward): pooled[c][n][ch] = mean_hw out[c][n][hw][ch] (fp32 out)
// Padding images (n ≥ nimg[c], N images per client) get zero rows: the head reads them (with zero loss
// weight) and must see finite values.
template <class P>
__global__ __launch_bounds__(256) void avgpool_kernel(const typename P::T* __restrict__ x, float* __restrict__ pooled,
                                                      int HW, int Ch, const int* __restrict__ nimg, int N) {
  const int cn = blockIdx.x;  // flattened (client, sample)
  const bool valid = !nimg || (cn % N) < nimg[cn / N];
  const typename P::T* xs = x + (int64_t)cn * HW * Ch;
  for (int ch = threadIdx.x; ch < Ch; ch += blockDim.x) {
    float s = 0.f;
    if (valid)
      for (int p = 0; p < HW; ++p) s += P::to_f(xs[(int64_t)p * Ch + ch]);
    pooled[(int64_t)cn * Ch + ch] = s / (float)HW;
  }
}

FA_EXPORT int fa_avgpool(const uint16_t* x, float* pooled, int CN, int HW, int Ch, const int* nimg, int N,
                         hipStream_t stream) {
  hipLaunchKernelGGL(avgpool_kernel<BF16>, dim3(CN), dim3(Ch < 256 ? 64 * ((Ch + 63) / 64) : 256), 0, stream, x,
                     pooled, HW, Ch, nimg, N);
  return (int)hipGetLastError();
}
FA_EXPORT int fa_avgpool_f32(const float* x, float* pooled, int CN, int HW, int Ch, const int* nimg, int N,
                             hipStream_t stream) {
  hipLaunchKernelGGL(avgpool_kernel<F32>, dim3(CN), dim3(Ch < 256 ? 64 * ((Ch + 63) / 64) : 256), 0, stream, x,
                     pooled, HW, Ch, nimg, N);
  return (int)hipGetLastError();
}

// ---- head backward: gpre = (dpool/HW)·[out > 0]; stats (Σg, Σg·y3, Σg·yd)
// one workgroup per (client, sample): channels across threads, spatial loop inside,
// per-channel partial sums atomically added once per workgroup.
template <class P>
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ dpool,
                                                       const typename P::T* __restrict__ out,
                                                       const typename P::T* __restrict__ y3,
                                                       const typename P::T* __restrict__ yd,
                                                       typename P::T* __restrict__ gpre, float* __restrict__ stats,
                                                       int N, int HW, int Ch, int NS, const int* __restrict__ nimg) {
  const int cn = blockIdx.x;
  const int c = cn / N;
  if (nimg && (cn % N) >= nimg[c]) return;   // padding image: its gradient is never read
  const int64_t base = (int64_t)cn * HW * Ch;
  const float inv = 1.f / (float)HW;
  for (int ch = threadIdx.x; ch < Ch; ch += blockDim.x) {
    const float d = dpool[(int64_t)cn * Ch + ch] * inv;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int p = 0; p < HW; ++p) {
      const int64_t i = base + (int64_t)p * Ch + ch;
      const float g = P::to_f(out[i]) > 0.f ? d : 0.f;
      const typename P::T gb = P::from_f(g);
      gpre[i] = gb;
      const float gr = P::to_f(gb);
      a0 += gr;
      if (y3) a1 += gr * P::to_f(y3[i]);   // null: a recomputed-y last conv gets Σg·y from its Gram pass
      if (yd) a2 += gr * P::to_f(yd[i]);
    }
    float* st = stats + ((int64_t)c * Ch + ch) * NS;
    fa_acc_add(st + 0, a0);
    fa_acc_add(st + 1, a1);
    if (yd && NS > 2) fa_acc_add(st + 2, a2);
  }
}

// Σ_p g·(y − K) of a recomputed-y 1×1 convolution's BN from the Gram product G = gᵀ·act(x) (its output y =
// act(x)·Wᵀ is never stored): stats[c][o][1] = Σ_i W[c][o][i]·G[c][o][i] − K[c][o]·stats[c][o][0]; the consumed
// G row is cleared for the next use. One wave per (output channel, client); CI ≤ 256.
__global__ __launch_bounds__(256) void gy_from_gram_kernel(const float* __restrict__ arena, int64_t ldw, int64_t woff,
                                                           float* __restrict__ G, int64_t ldg,
                                                           const float* __restrict__ pivot, float* __restrict__ stats,
                                                           int NS, int CO, int CI) {
  const int c = blockIdx.y;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= CO) return;
  const float* w = arena + (int64_t)c * ldw + woff + (int64_t)o * CI;
  float* gr = G + (int64_t)c * ldg + (int64_t)o * CI;
  float s = 0.f;
  for (int i = lane; i < CI; i += 64) {
    s += w[i] * gr[i];
    gr[i] = 0.f;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) {
    float* st = stats + ((int64_t)c * CO + o) * NS;
    st[1] = s - (pivot ? pivot[(int64_t)c * CO + o] : 0.f) * st[0];
  }
}

FA_EXPORT int fa_gy_from_gram(const float* arena, int64_t ldw, int64_t woff, float* G, int64_t ldg, const float* pivot,
                              float* stats, int NS, int C, int CO, int CI, hipStream_t stream) {
  if (CI > 4096 || NS < 2) return -3;
  hipLaunchKernelGGL(gy_from_gram_kernel, dim3((CO + 3) / 4, C), dim3(256), 0, stream, arena, ldw, woff, G, ldg, pivot,
                     stats, NS, CO, CI);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_head_bwd(const float* dpool, const uint16_t* out, const uint16_t* y3, const uint16_t* yd,
                          uint16_t* gpre, float* stats, int C, int N, int HW, int Ch, int NS, const int* nimg,
                          hipStream_t stream) {
  hipLaunchKernelGGL(head_bwd_kernel<BF16>, dim3(C * N), dim3(Ch < 256 ? 64 * ((Ch + 63) / 64) : 256), 0, stream,
                     dpool, out, y3, yd, gpre, stats, N, HW, Ch, NS, nimg);
  return (int)hipGetLastError();
}
FA_EXPORT int fa_head_bwd_f32(const float* dpool, const float* out, const float* y3, const float* yd, float* gpre,
                              float* stats, int C, int N, int HW, int Ch, int NS, const int* nimg, hipStream_t stream) {
  hipLaunchKernelGGL(head_bwd_kernel<F32>, dim3(C * N), dim3(Ch < 256 ? 64 * ((Ch + 63) / 64) : 256), 0, stream,
                     dpool, out, y3, yd, gpre, stats, N, HW, Ch, NS, nimg);
  return (int)hipGetLastError();
}

// ---- input conversion: x [C][N][Cin][H][W] fp32 (NCHW per client) → [C][N][H][W][Cpad] bf16 | fp32
template <class P>
__global__ __launch_bounds__(256) void nchw_to_nhwc_pad_kernel(const float* __restrict__ x,
                                                               typename P::T* __restrict__ y, int64_t CN, int Cin,
                                                               int HW, int Cpad) {
  const int64_t total = CN * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cn = i / HW;
    const int p = (int)(i % HW);
    const float* src = x + cn * Cin * HW + p;
    typename P::T* dst = y + i * Cpad;
    for (int ch = 0; ch < Cpad; ++ch) dst[ch] = ch < Cin ? P::from_f(src[(int64_t)ch * HW]) : P::from_f(0.f);
  }
}

FA_EXPORT int fa_nchw_to_nhwc_pad(const float* x, uint16_t* y, int64_t CN, int Cin, int HW, int Cpad,
                                  hipStream_t stream) {
  hipLaunchKernelGGL(nchw_to_nhwc_pad_kernel<BF16>, dim3(fa_grid(CN * HW, 256, 4096)), dim3(256), 0, stream, x, y, CN,
                     Cin, HW, Cpad);
  return (int)hipGetLastError();
}
FA_EXPORT int fa_nchw_to_nhwc_pad_f32(const float* x, float* y, int64_t CN, int Cin, int HW, int Cpad,
                                      hipStream_t stream) {
  hipLaunchKernelGGL(nchw_to_nhwc_pad_kernel<F32>, dim3(fa_grid(CN * HW, 256, 4096)), dim3(256), 0, stream, x, y, CN,
                     Cin, HW, Cpad);
  return (int)hipGetLastError();
}

// ---- bn_relu_apply: out = relu(y·s + t) (stem activation materialisation)
FA_EXPORT int fa_bn_relu_apply(const uint16_t* y, const float* s, const float* t, uint16_t* out, int C,
                               int64_t per_client, int Ch, hipStream_t stream) {
  return fa_block_out(y, s, t, nullptr, nullptr, nullptr, out, C, per_client, Ch, nullptr, 0, stream);
}
