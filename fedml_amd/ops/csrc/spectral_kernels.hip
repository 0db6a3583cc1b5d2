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
                                                              int B, int C, int HW, float momentum, int mode,
                                                              const unsigned char* __restrict__ first) {
  if (first) mode = *first ? 2 : 1;   // the reference's `np.sum(running_amp) == 0`, decided on the device
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


// ---------------------------------------------------------------------------------------------------------------
// Power-of-two planes up to 512 × 512 (HS-FedAvg's 3 × 512 × 512 amplitude, hs_fedavg/fedavg_api.py:135): a
// radix-8 Stockham FFT in LDS (in-register 8-point butterflies, in place through registers, bank-padded indices),
// applied separably — a row pass (whole rows in LDS, several per workgroup) and a column pass (a 16-column × H tile
// in LDS, coalesced 128-B row segments on both sides). Forward: rows (real in) → columns (F out, |F| fused). Inverse with the band mix:
// columns (mix applied while loading F) → rows (real part × 1/HW out). O(HW·log HW) per plane instead of the
// DFT's O(HW·(H+W)).
constexpr int kMaxN = 512;

// tw[k] = e^{sign·2πi·k/n}, k < n (double-precision table, as accurate as rocFFT's fp32 plan)
__device__ __forceinline__ void twiddles_full(float2* tw, int n, float sign) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    double sn, cs;
    sincospi(2.0 * k / n, &sn, &cs);
    tw[k] = make_float2((float)cs, (float)(sign * sn));
  }
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
// a · e^{sign·iπ/2}
__device__ __forceinline__ float2 cmul_i(float2 a, float sign) { return make_float2(-sign * a.y, sign * a.x); }

// In-register DFT of R ∈ {2, 4, 8} points: a[k] ← Σ_j a[j]·e^{sign·2πi·jk/R} (decimation in frequency)
template <int R>
__device__ __forceinline__ void dft_small(float2 (&a)[R], float sign) {
  if (R == 2) {
    const float2 t = a[0];
    a[0] = cadd(t, a[1]);
    a[1] = csub(t, a[1]);
  } else if (R == 4) {
    const float2 d0 = cadd(a[0], a[2]), d2 = csub(a[0], a[2]);
    const float2 d1 = cadd(a[1], a[3]), d3 = cmul_i(csub(a[1], a[3]), sign);
    a[0] = cadd(d0, d1);
    a[2] = csub(d0, d1);
    a[1] = cadd(d2, d3);
    a[3] = csub(d2, d3);
  } else {
    const float h = 0.70710678118654752f;
    float2 e[4] = {cadd(a[0], a[4]), cadd(a[1], a[5]), cadd(a[2], a[6]), cadd(a[3], a[7])};
    float2 o[4] = {csub(a[0], a[4]), cmul(csub(a[1], a[5]), make_float2(h, sign * h)),
                   cmul_i(csub(a[2], a[6]), sign), cmul(csub(a[3], a[7]), make_float2(-h, sign * h))};
    dft_small<4>(e, sign);
    dft_small<4>(o, sign);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[2 * k] = e[k];
      a[2 * k + 1] = o[k];
    }
  }
}

// Transform-local LDS index with one float2 of padding per 8: the radix-8 stages' strided accesses (output stride
// R·s) land on distinct banks (a 512-point stage 1 writes 8p + k → 9p + k: 18-float lane stride, 32 lanes on 64
// distinct banks) instead of 4-16-way conflicts.
__device__ __forceinline__ int lpad(int i) { return i + (i >> 3); }
// LDS leading dimension of one transform: N + N/8 padded to ≡ 2 (mod 32) float2, so the 16 transforms of a column
// tile written by one half-wave (consecutive columns) also fall on distinct banks
__host__ __device__ __forceinline__ int lds_ld(int n) { return ((n + n / 8 + 29) / 32) * 32 + 2; }

// One radix-R Stockham (autosort) stage of nfft length-N transforms IN PLACE in LDS (transform f at x + f·ld,
// padded indices): current stride s, sub-length n = N/s, m = n/R. Task (p, q): inputs x[q + s(p + jm)], j < R;
// outputs y[q + s(Rp + k)] = DFT_R(inputs)[k] · e^{sign·2πi·pk/n} — the twiddle is tw[p·k·s] of the length-N
// table. Every thread loads all its tasks' inputs into registers, the workgroup synchronises, then the outputs
// overwrite the same buffer: one LDS buffer instead of a ping-pong pair (twice the workgroups per CU).
// MAXT = the tasks a thread may own (nfft·N/R ≤ MAXT·blockDim).
template <int R, int MAXT>
__device__ __forceinline__ void stockham_stage_ip(float2* __restrict__ x, const float2* __restrict__ tw, int lgN,
                                                  int ls, int nfft, int ld, float sign) {
  const int N = 1 << lgN, s = 1 << ls;
  const int lgR = R == 8 ? 3 : R == 4 ? 2 : 1;
  const int m = N >> (ls + lgR);
  const int tasks = N >> lgR;
  const int total = nfft * tasks;
  float2 a[MAXT][R];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int i = threadIdx.x + t * blockDim.x;
    if (i < total) {
      const int f = i >> (lgN - lgR);
      const int r = i & (tasks - 1);
      const int p = r >> ls, q = r & (s - 1);
      const float2* xf = x + f * ld;
#pragma unroll
      for (int j = 0; j < R; ++j) a[t][j] = xf[lpad(q + s * (p + j * m))];
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int i = threadIdx.x + t * blockDim.x;
    if (i < total) {
      const int f = i >> (lgN - lgR);
      const int r = i & (tasks - 1);
      const int p = r >> ls, q = r & (s - 1);
      dft_small<R>(a[t], sign);
      float2* yf = x + f * ld;
      yf[lpad(q + s * R * p)] = a[t][0];
#pragma unroll
      for (int k = 1; k < R; ++k) yf[lpad(q + s * (R * p + k))] = cmul(a[t][k], tw[p * k * s]);
    }
  }
  __syncthreads();
}

// nfft independent length-2^lg transforms at x + f·ld (padded indices), in place, natural order out: radix-8 stages
// then one radix-4 or radix-2 stage for the remainder (a 512-point transform: 3 LDS passes). PPT = the points a
// thread holds in registers per stage: nfft·2^lg ≤ PPT·blockDim (sized per kernel — a 32-point worst case for every
// kernel cost 248 VGPRs, two waves per SIMD).
template <int PPT>
__device__ void stockham(float2* x, const float2* tw, int lg, int nfft, int ld, float sign) {
  int ls = 0;
  while (ls < lg) {
    const int left = lg - ls;
    if (left >= 3) {
      stockham_stage_ip<8, (PPT + 7) / 8>(x, tw, lg, ls, nfft, ld, sign);
      ls += 3;
    } else if (left == 2) {
      stockham_stage_ip<4, (PPT + 3) / 4>(x, tw, lg, ls, nfft, ld, sign);
      ls += 2;
    } else {
      stockham_stage_ip<2, (PPT + 1) / 2>(x, tw, lg, ls, nfft, ld, sign);
      ls += 1;
    }
  }
}

constexpr int kRowPoints = 2048;   // points per row-pass workgroup (R = 2048 / W rows)
constexpr int kColTile = 16;
// 512 threads: two column-tile workgroups fill a CU's LDS, so the waves that hide the strided global traffic come from
// a wider workgroup (16 per CU instead of 8)
constexpr int kColThreads = 512;

// R rows of length W = 2^lg per workgroup. In: real (xr) or complex (xc). Out: complex (out) or the real part
// (out_r), times `scale`.
__global__ __launch_bounds__(256) void fft_rows_kernel(const float* __restrict__ xr, const float2* __restrict__ xc,
                                                       float2* __restrict__ out, float* __restrict__ out_r,
                                                       int64_t rows, int lg, int R, float sign, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int W = 1 << lg, ld = lds_ld(W);
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* A = tw + kMaxN;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, rows - r0);
  for (int i = threadIdx.x; i < nr * W; i += blockDim.x) {
    const int64_t g = r0 * W + i;
    const int rr = i >> lg, w = i & (W - 1);
    A[rr * ld + lpad(w)] = xr ? make_float2(xr[g], 0.f) : xc[g];
  }
  twiddles_full(tw, W, sign);
  __syncthreads();
  stockham<kRowPoints / 256>(A, tw, lg, nr, ld, sign);
  for (int i = threadIdx.x; i < nr * W; i += blockDim.x) {
    const int64_t g = r0 * W + i;
    const int rr = i >> lg, w = i & (W - 1);
    const float2 v = A[rr * ld + lpad(w)];
    if (out_r) out_r[g] = v.x * scale;
    else out[g] = make_float2(v.x * scale, v.y * scale);
  }
}


// a kColTile-column tile of one plane [H = 2^lg][W]: column transforms in LDS (transform per column, padded). `trg`
// non-null: inverse pass of the band mix — inside the band the loaded F is rescaled to amplitude trg[c] (F = 0:
// trg + 0i). `amp_out` non-null: |F| of the result as well.
__global__ __launch_bounds__(kColThreads) void fft_cols_kernel(const float2* __restrict__ in, float2* __restrict__ out,
                                                       float* __restrict__ amp_out, const float* __restrict__ amp_in,
                                                       const float* __restrict__ trg, int C, int band, int lg, int W,
                                                       float sign) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = 1 << lg, ld = lds_ld(H);
  const int tc = min(kColTile, W);
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* A = tw + kMaxN;
  const int64_t plane = blockIdx.y;
  const int c0 = blockIdx.x * tc;
  const int64_t base = plane * (int64_t)H * W;
  const float* tp = trg ? trg + (int64_t)(plane % C) * H * W : nullptr;
  for (int i = threadIdx.x; i < tc * H; i += blockDim.x) {
    const int h = i / tc, cc = i - h * tc;
    const int64_t g = base + (int64_t)h * W + c0 + cc;
    float2 v = in[g];
    if (tp) {
      const int u = h, vv = c0 + cc;
      if (min(u, H - u) <= band && min(vv, W - vv) <= band) {
        const float a = amp_in[g], A_ = tp[(int64_t)h * W + c0 + cc];
        v = a > 0.f ? make_float2(v.x * (A_ / a), v.y * (A_ / a)) : make_float2(A_, 0.f);
      }
    }
    A[cc * ld + lpad(h)] = v;
  }
  twiddles_full(tw, H, sign);
  __syncthreads();
  stockham<kColTile * kMaxN / kColThreads>(A, tw, lg, tc, ld, sign);
  for (int i = threadIdx.x; i < tc * H; i += blockDim.x) {
    const int h = i / tc, cc = i - h * tc;
    const int64_t g = base + (int64_t)h * W + c0 + cc;
    const float2 v = A[cc * ld + lpad(h)];
    out[g] = v;
    if (amp_out) amp_out[g] = sqrtf(v.x * v.x + v.y * v.y);
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
                     amp, running, B, C, HW, momentum, mode, nullptr);
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

static int spec_lg(int n) {
  int lg = 0;
  while ((1 << lg) < n) ++lg;
  return (1 << lg) == n && n >= 2 && n <= spec::kMaxN ? lg : -1;
}

static int spec_rows(const float* xr, const float2* xc, float2* out, float* out_r, int64_t rows, int W, float sign,
                     float scale, hipStream_t stream) {
  const int lg = spec_lg(W);
  if (lg < 0) return -2;
  const int R = max(1, spec::kRowPoints / W);
  const size_t smem = (size_t)(spec::kMaxN + R * spec::lds_ld(W)) * sizeof(float2);
  if (smem > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)spec::fft_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(spec::fft_rows_kernel, dim3((unsigned)((rows + R - 1) / R)), dim3(256), smem, stream, xr, xc, out,
                     out_r, rows, lg, R, sign, scale);
  return (int)hipGetLastError();
}

static int spec_cols(const float2* in, float2* out, float* amp_out, const float* amp_in, const float* trg, int C,
                     int band, int64_t planes, int H, int W, float sign, hipStream_t stream) {
  const int lg = spec_lg(H);
  if (lg < 0 || spec_lg(W) < 0) return -2;
  const int tc = min(spec::kColTile, W);
  const size_t smem = (size_t)(spec::kMaxN + tc * spec::lds_ld(H)) * sizeof(float2);
  if (smem > 160 * 1024) return -5;
  (void)hipFuncSetAttribute((const void*)spec::fft_cols_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(spec::fft_cols_kernel, dim3((unsigned)(W / tc), (unsigned)planes), dim3(spec::kColThreads), smem,
                     stream, in,
                     out, amp_out, amp_in, trg, C, band, lg, W, sign);
  return (int)hipGetLastError();
}

// Power-of-two planes (2..512 per side): x [planes][H][W] fp32 → F complex + |F|; `tmp` complex scratch of the
// same size (the row pass's output).
FA_EXPORT int fa_spec_fft2_pow2(const float* x, void* F, float* amp, void* tmp, int64_t planes, int H, int W,
                                hipStream_t stream) {
  int rc = spec_rows(x, nullptr, reinterpret_cast<float2*>(tmp), nullptr, planes * H, W, -1.f, 1.f, stream);
  if (rc) return rc;
  return spec_cols(reinterpret_cast<const float2*>(tmp), reinterpret_cast<float2*>(F), amp, nullptr, nullptr, 1, 0,
                   planes, H, W, -1.f, stream);
}

// out = Re ifft2(F with amplitude ← trg inside the band), power-of-two planes; tmp: complex scratch
FA_EXPORT int fa_spec_mix_ifft2_pow2(const void* F, const float* amp, const float* trg, float* out, void* tmp,
                                     int64_t planes, int C, int H, int W, int band, hipStream_t stream) {
  int rc = spec_cols(reinterpret_cast<const float2*>(F), reinterpret_cast<float2*>(tmp), nullptr, amp, trg, C, band,
                     planes, H, W, 1.f, stream);
  if (rc) return rc;
  return spec_rows(nullptr, reinterpret_cast<const float2*>(tmp), nullptr, out, planes * H, W, 1.f,
                   1.f / ((float)H * (float)W), stream);
}

// mode 3: EMA, or replace when Σ running == 0 (`flag` = that test, evaluated on the device: no host sync)
FA_EXPORT int fa_spec_amp_update_auto(const float* amp, float* running, const unsigned char* first, int B, int C,
                                      int HW, float momentum, hipStream_t stream) {
  hipLaunchKernelGGL(spec::spec_amp_update_kernel, dim3(fa_grid((int64_t)C * HW, 256, 1024)), dim3(256), 0, stream,
                     amp, running, B, C, HW, momentum, 1, first);
  return (int)hipGetLastError();
}
