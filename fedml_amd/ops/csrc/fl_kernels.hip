// Federated-learning kernels for MI355X (gfx950): aggregation, fused multi-client
// optimizers, robust aggregation, compression, fused loss, on-device metrics.
//
// Every kernel works on the flat parameter arena: a client stack is a row-major
// [C, P] buffer (row stride ldx elements, 256-B aligned rows), the global model
// is [P]. All are launched on the caller's HIP stream (graph-capturable: no
// allocation, no sync, no host-side scalars that change between replays unless
// passed by device pointer).
#include <algorithm>

#include "common.h"

// =====================================================================================
// K1  FedAvg weighted sum: out[p] = beta*out[p] + Σ_c w[c] * X[c, p]
//     (reference hot loop: `simulation/single_process/fedavg/fedavg_api.py:206-221`,
//      `mpi_p2p_mp/fedavg/FedAVGAggregator.py:82-90` — a Python loop over keys × clients)
//     HBM-streaming: 16-B loads, C unrolled by 4, fp32 accumulation.
// =====================================================================================
template <typename T>
__device__ __forceinline__ f32x4 load4(const T* p);
template <>
__device__ __forceinline__ f32x4 load4<float>(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}
template <>
__device__ __forceinline__ f32x4 load4<uint16_t>(const uint16_t* p) {
  uint2 u = *reinterpret_cast<const uint2*>(p);
  f32x4 r;
  r.x = __uint_as_float(u.x << 16);
  r.y = __uint_as_float(u.x & 0xffff0000u);
  r.z = __uint_as_float(u.y << 16);
  r.w = __uint_as_float(u.y & 0xffff0000u);
  return r;
}
template <typename T>
__device__ __forceinline__ float load1(const T* p);
template <>
__device__ __forceinline__ float load1<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float load1<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }

template <typename T>
__global__ __launch_bounds__(256) void weighted_sum_kernel(const T* __restrict__ X, int64_t ldx, int C,
                                                           const float* __restrict__ w, float* __restrict__ out,
                                                           int64_t P, float beta) {
  const int64_t nvec = P >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v << 2;
    f32x4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
    int c = 0;
    for (; c + 1 < C; c += 2) {
      const f32x4 x0 = load4<T>(X + (int64_t)c * ldx + i);
      const f32x4 x1 = load4<T>(X + (int64_t)(c + 1) * ldx + i);
      const float w0 = w[c], w1 = w[c + 1];
      a0 += w0 * x0;
      a1 += w1 * x1;
    }
    if (c < C) a0 += w[c] * load4<T>(X + (int64_t)c * ldx + i);
    a0 += a1;
    f32x4* o = reinterpret_cast<f32x4*>(out + i);
    if (beta != 0.f) a0 += beta * (*o);
    *o = a0;
  }
  // tail (P % 4 elements) handled by the first threads of block 0
  if (blockIdx.x == 0) {
    const int64_t i = (nvec << 2) + threadIdx.x;
    if (i < P) {
      float a = 0.f;
      for (int c = 0; c < C; ++c) a += w[c] * load1<T>(X + (int64_t)c * ldx + i);
      out[i] = (beta != 0.f ? beta * out[i] : 0.f) + a;
    }
  }
}

FA_EXPORT int fa_weighted_sum(const void* X, int x_is_bf16, int64_t ldx, int C, const float* w, float* out,
                              int64_t P, float beta, hipStream_t stream) {
  const int block = 256;
  const int grid = fa_grid((P >> 2) + 1, block, 2048);
  if (x_is_bf16)
    hipLaunchKernelGGL(weighted_sum_kernel<uint16_t>, dim3(grid), dim3(block), 0, stream, (const uint16_t*)X, ldx, C,
                       w, out, P, beta);
  else
    hipLaunchKernelGGL(weighted_sum_kernel<float>, dim3(grid), dim3(block), 0, stream, (const float*)X, ldx, C, w,
                       out, P, beta);
  return (int)hipGetLastError();
}

// =====================================================================================
// K1/K3  Many aggregations at once on MFMA: OUT[S, P] = W[S, C] · X[C, P]
//     Shapley subset valuation needs 2^(K-1)·K weighted sums of the same client stack
//     (`s_fedavg/fedavg_api.py:258-325`). Exact-f32 MFMA (v_mfma_f32_32x32x2_f32):
//     a workgroup owns a 128-column P slab, keeps that slab's X fragments in registers
//     (C ≤ 64 → ≤ 32 VGPRs per lane), and sweeps every 32-row S tile, so X is read from
//     HBM exactly once and the kernel is bound by the OUT write stream.
//     A-operand map (32x32x2 f32): lane l holds A[i=l&31][k=l>>5]; B: B[k=l>>5][j=l&31];
//     C/D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
// =====================================================================================
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KSTEPS>
__global__ __launch_bounds__(256) void subset_agg_mfma_kernel(const float* __restrict__ W, int S, int C,
                                                              const float* __restrict__ X, int64_t ldx, int64_t P,
                                                              float* __restrict__ OUT, int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t p0 = (int64_t)blockIdx.x * 128 + wid * 32;
  const int col = lane & 31;
  const int khalf = lane >> 5;
  const int64_t p = p0 + col;
  const bool pin = p < P;
  float bfrag[KSTEPS];
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int k = ks * 2 + khalf;
    bfrag[ks] = (pin && k < C) ? X[(int64_t)k * ldx + p] : 0.f;
  }
  for (int s0 = blockIdx.y * 32; s0 < S; s0 += gridDim.y * 32) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const int srow = s0 + col;  // A row for this lane
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int k = ks * 2 + khalf;
      const float a = (srow < S && k < C) ? W[(int64_t)srow * C + k] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bfrag[ks], acc, 0, 0, 0);
    }
    if (pin) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * khalf;
        const int s = s0 + row;
        if (s < S) OUT[(int64_t)s * ldo + p] = acc[r];
      }
    }
  }
}

FA_EXPORT int fa_subset_aggregate(const float* W, int S, int C, const float* X, int64_t ldx, int64_t P, float* OUT,
                                  int64_t ldo, hipStream_t stream) {
  if (C > 64) return -1;  // caller chunks C
  const int gx = (int)((P + 127) / 128);
  int gy = (S + 31) / 32;
  // enough workgroups to fill 256 CUs several times over, but keep X register reuse
  while (gy > 1 && (int64_t)gx * gy > 8192) gy = (gy + 1) / 2;
  dim3 grid(gx, gy);
  const int ksteps = (C + 1) / 2;
#define LAUNCH_SA(KS)                                                                                         \
  hipLaunchKernelGGL(subset_agg_mfma_kernel<KS>, grid, dim3(256), 0, stream, W, S, C, X, ldx, P, OUT, ldo)
  if (ksteps <= 4) LAUNCH_SA(4);
  else if (ksteps <= 8) LAUNCH_SA(8);
  else if (ksteps <= 16) LAUNCH_SA(16);
  else LAUNCH_SA(32);
#undef LAUNCH_SA
  return (int)hipGetLastError();
}

// =====================================================================================
// K2  Fused multi-client SGD over a [C, P] stack (torch.optim.SGD semantics + FedProx).
//     g' = g + mu*(p - p_global) + wd*p;  buf = m*buf + (1-damp)*g' (buf=g' on first step);
//     d = nesterov ? g' + m*buf : buf;   p -= lr * active[c] * d
//     grid.y = client; `active` (nullable) masks clients whose data is exhausted.
// =====================================================================================
template <typename G>
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ param, const G* __restrict__ grad,
                                                  float* __restrict__ mom, const float* __restrict__ pref,
                                                  int64_t P, int64_t ld, float lr, float wd, float momentum,
                                                  float dampening, int nesterov, float mu, int first_step,
                                                  const float* __restrict__ active, const float* __restrict__ lr_scale) {
  const int c = blockIdx.y;
  float scale = active ? active[c] : 1.f;
  if (lr_scale) scale *= lr_scale[0];
  if (scale == 0.f) return;
  float* pc = param + (int64_t)c * ld;
  const G* gc = grad + (int64_t)c * ld;
  float* mc = mom ? mom + (int64_t)c * ld : nullptr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    float p = pc[i];
    float g = load1<G>(gc + i);
    if (mu != 0.f) g += mu * (p - pref[i]);
    if (wd != 0.f) g += wd * p;
    float d = g;
    if (mc) {
      float b = first_step ? g : momentum * mc[i] + (1.f - dampening) * g;
      mc[i] = b;
      d = nesterov ? g + momentum * b : b;
    }
    pc[i] = p - lr * scale * d;
  }
}

FA_EXPORT int fa_sgd_step(float* param, const void* grad, int grad_is_bf16, float* mom, const float* pref, int C,
                          int64_t P, int64_t ld, float lr, float wd, float momentum, float dampening, int nesterov,
                          float mu, int first_step, const float* active, const float* lr_scale, hipStream_t stream) {
  dim3 grid(fa_grid(P, 256, 1024), C);
  if (grad_is_bf16)
    hipLaunchKernelGGL(sgd_kernel<uint16_t>, grid, dim3(256), 0, stream, param, (const uint16_t*)grad, mom, pref, P,
                       ld, lr, wd, momentum, dampening, nesterov, mu, first_step, active, lr_scale);
  else
    hipLaunchKernelGGL(sgd_kernel<float>, grid, dim3(256), 0, stream, param, (const float*)grad, mom, pref, P, ld, lr,
                       wd, momentum, dampening, nesterov, mu, first_step, active, lr_scale);
  return (int)hipGetLastError();
}

// torch.optim.Adam(amsgrad=…, weight_decay=… as L2) over a [C, P] stack. The step count
// lives on the device (`step`, per client) so the launch is replayable from a hipGraph.
// A client's first step (t ≤ 1) starts from zero moments without reading them — torch's state at step 1 — so
// the per-round moment resets need no fill pass over the [C, P] buffers (and the first step reads 2–3 fewer
// streams).
template <typename G>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ param, const G* __restrict__ grad,
                                                   float* __restrict__ m1, float* __restrict__ m2,
                                                   float* __restrict__ vmax, const float* __restrict__ step, int64_t P,
                                                   int64_t ld, float lr, float beta1, float beta2, float eps, float wd,
                                                   int decoupled, const float* __restrict__ active,
                                                   uint16_t* __restrict__ shadow) {
  const int c = blockIdx.y;
  const float scale = active ? active[c] : 1.f;
  if (scale == 0.f) return;
  const float t = step[c];
  const float bc1 = 1.f - __powf(beta1, t);
  const float bc2 = 1.f - __powf(beta2, t);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const bool fresh = t <= 1.f;
  float* pc = param + (int64_t)c * ld;
  const G* gc = grad + (int64_t)c * ld;
  float* a = m1 + (int64_t)c * ld;
  float* b = m2 + (int64_t)c * ld;
  float* vm = vmax ? vmax + (int64_t)c * ld : nullptr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // 16-B vectors (4 elements a thread) when every row is 16-B aligned: ≈ 30 B of HBM traffic per element, so the
  // step is a pure stream
  const bool vec = (P & 3) == 0 && (ld & 3) == 0 && ((reinterpret_cast<uintptr_t>(pc) | reinterpret_cast<uintptr_t>(a) |
                                                      reinterpret_cast<uintptr_t>(b)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(gc) & (4 * sizeof(G) - 1)) == 0 && vm == nullptr;
  if (vec) {
    for (int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); i < P; i += 4 * stride) {
      float pv[4], gv[4], av[4] = {0.f, 0.f, 0.f, 0.f}, bv[4] = {0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<float4*>(pv) = *reinterpret_cast<const float4*>(pc + i);
      if constexpr (sizeof(G) == 4) {
        *reinterpret_cast<float4*>(gv) = *reinterpret_cast<const float4*>(gc + i);
      } else {
        const uint2 r = *reinterpret_cast<const uint2*>(gc + i);
        gv[0] = bf16_to_f32((uint16_t)(r.x & 0xffff));
        gv[1] = bf16_to_f32((uint16_t)(r.x >> 16));
        gv[2] = bf16_to_f32((uint16_t)(r.y & 0xffff));
        gv[3] = bf16_to_f32((uint16_t)(r.y >> 16));
      }
      if (!fresh) {
        *reinterpret_cast<float4*>(av) = *reinterpret_cast<const float4*>(a + i);
        *reinterpret_cast<float4*>(bv) = *reinterpret_cast<const float4*>(b + i);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pj = pv[e], g = gv[e];
        if (wd != 0.f) {
          if (decoupled) pj *= (1.f - lr * wd);
          else g += wd * pj;
        }
        float ma = (1.f - beta1) * g;
        float mb = (1.f - beta2) * g * g;
        if (!fresh) {
          ma += beta1 * av[e];
          mb += beta2 * bv[e];
        }
        av[e] = ma;
        bv[e] = mb;
        pv[e] = pj - step_size * ma / (sqrtf(mb) / bc2_sqrt + eps);
      }
      *reinterpret_cast<float4*>(a + i) = *reinterpret_cast<const float4*>(av);
      *reinterpret_cast<float4*>(b + i) = *reinterpret_cast<const float4*>(bv);
      *reinterpret_cast<float4*>(pc + i) = *reinterpret_cast<const float4*>(pv);
      if (shadow) {
        uint2 o;
        o.x = (uint32_t)f32_to_bf16(pv[0]) | ((uint32_t)f32_to_bf16(pv[1]) << 16);
        o.y = (uint32_t)f32_to_bf16(pv[2]) | ((uint32_t)f32_to_bf16(pv[3]) << 16);
        *reinterpret_cast<uint2*>(shadow + (int64_t)c * ld + i) = o;
      }
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    float p = pc[i];
    float g = load1<G>(gc + i);
    if (wd != 0.f) {
      if (decoupled) p *= (1.f - lr * wd);
      else g += wd * p;
    }
    float ma = (1.f - beta1) * g;
    float mb = (1.f - beta2) * g * g;
    if (!fresh) {
      ma += beta1 * a[i];
      mb += beta2 * b[i];
    }
    a[i] = ma;
    b[i] = mb;
    float den;
    if (vm) {
      float v = fresh ? mb : fmaxf(vm[i], mb);
      vm[i] = v;
      den = sqrtf(v) / bc2_sqrt + eps;
    } else {
      den = sqrtf(mb) / bc2_sqrt + eps;
    }
    const float np = p - step_size * ma / den;
    pc[i] = np;
    if (shadow) shadow[(int64_t)c * ld + i] = f32_to_bf16(np);   // bf16 weight copy for the next forward
  }
}

FA_EXPORT int fa_adam_step(float* param, const void* grad, int grad_is_bf16, float* m1, float* m2, float* vmax,
                           const float* step, int C, int64_t P, int64_t ld, float lr, float beta1, float beta2,
                           float eps, float wd, int decoupled, const float* active, void* shadow,
                           hipStream_t stream) {
  dim3 grid(fa_grid(P, 256, 1024), C);
  if (grad_is_bf16)
    hipLaunchKernelGGL(adam_kernel<uint16_t>, grid, dim3(256), 0, stream, param, (const uint16_t*)grad, m1, m2, vmax,
                       step, P, ld, lr, beta1, beta2, eps, wd, decoupled, active, (uint16_t*)shadow);
  else
    hipLaunchKernelGGL(adam_kernel<float>, grid, dim3(256), 0, stream, param, (const float*)grad, m1, m2, vmax, step,
                       P, ld, lr, beta1, beta2, eps, wd, decoupled, active, (uint16_t*)shadow);
  return (int)hipGetLastError();
}

// dst[c][:] = src[:] for every row c of a [C, P] stack (row stride ld): the global model into every client
// slot. float4 stores when the rows are 16-B aligned; the source row stays in L2 across the C rows.
// blockIdx.y takes BR_ROWS destination rows: each source vector is read once per BR_ROWS rows (a 32-client
// transformer arena: 1.4 instead of 11 GB of source reads, the source row being larger than the MALL)
// (FEDML_AMD_BCAST_ROWS overrides the 8, for A/B runs)
__global__ __launch_bounds__(256) void broadcast_rows_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                             int64_t P, int64_t ld, int vec, int C, int rows) {
  const int r0 = blockIdx.y * rows, nr = min(rows, C - r0);
  float* d = dst + (int64_t)r0 * ld;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    const int64_t n4 = P / 4, ld4 = ld / 4;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(d);
    for (int64_t i = i0; i < n4; i += stride) {
      const float4 v = s4[i];
      for (int r = 0; r < nr; ++r) d4[r * ld4 + i] = v;
    }
    for (int64_t i = n4 * 4 + i0; i < P; i += stride)
      for (int r = 0; r < nr; ++r) d[r * ld + i] = src[i];
  } else {
    for (int64_t i = i0; i < P; i += stride) {
      const float v = src[i];
      for (int r = 0; r < nr; ++r) d[r * ld + i] = v;
    }
  }
}

// Zero columns [off, off + len) of every row of a [C, ld] fp32 stack for the nseg (off, len) pairs of `segs`
// (device int64 table): the gradient-arena columns that are accumulated into (everything but the
// first-touch weight-gradient rows) in one launch. grid = (chunks, C, nseg).
__global__ __launch_bounds__(256) void zero_segments_kernel(float* __restrict__ base, int64_t ld,
                                                            const int64_t* __restrict__ segs) {
  const int64_t off = segs[2 * blockIdx.z], len = segs[2 * blockIdx.z + 1];
  float* d = base + (int64_t)blockIdx.y * ld + off;
  const int64_t head = min<int64_t>(len, (int64_t)((16 - ((uintptr_t)d & 15)) & 15) / 4);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 < head) d[i0] = 0.f;
  const int64_t n4 = (len - head) / 4;
  float4* d4 = reinterpret_cast<float4*>(d + head);
  for (int64_t i = i0; i < n4; i += stride) d4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = head + 4 * n4 + i0; i < len; i += stride) d[i] = 0.f;
}

FA_EXPORT int fa_zero_segments(float* base, int64_t ld, int C, const int64_t* segs_dev, int nseg, int64_t max_len,
                               hipStream_t stream) {
  if (C <= 0 || nseg <= 0 || max_len <= 0) return 0;
  if (nseg > 65535 || C > 65535) return (int)hipErrorInvalidValue;
  dim3 grid(fa_grid((max_len + 3) / 4, 256, 512), C, nseg);
  hipLaunchKernelGGL(zero_segments_kernel, grid, dim3(256), 0, stream, base, ld, segs_dev);
  return (int)hipGetLastError();
}

// Embedding-table gradient of a client-stacked lookup: dst[c][ids[c][t]][:] += g[c][t][:] with fp32 atomics
// (vector-memory global atomics), dst = client c's [V][d] table at base + c·ld. torch's accumulating
// index_put_ on the strided arena view copies the whole [C, V, d] table out and back (2 × 3 GB per DistilBERT
// step). One workgroup per token row; tokens of one client hitting the same row add in any order.
__global__ __launch_bounds__(256) void embedding_grad_kernel(float* __restrict__ base, int64_t ld,
                                                             const int64_t* __restrict__ ids, const float* __restrict__ g,
                                                             int T, int V, int d) {
  const int64_t row = blockIdx.x;            // c·T + t
  const int c = (int)(row / T);
  const int64_t id = ids[row];
  if (id < 0 || id >= V) return;             // out-of-range ids contribute nothing (torch would raise earlier)
  float* dst = base + (int64_t)c * ld + id * d;
  const float* src = g + row * d;
  for (int k = threadIdx.x; k < d; k += blockDim.x) atomicAdd(dst + k, src[k]);
}

FA_EXPORT int fa_embedding_grad_f32(float* base, int64_t ld, const int64_t* ids, const float* g, int C, int T, int V,
                                    int d, hipStream_t stream) {
  if (C <= 0 || T <= 0 || d <= 0) return 0;
  hipLaunchKernelGGL(embedding_grad_kernel, dim3((unsigned)((int64_t)C * T)), dim3(d >= 256 ? 256 : 64), 0, stream,
                     base, ld, ids, g, T, V, d);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_broadcast_rows(float* dst, const float* src, int C, int64_t P, int64_t ld, hipStream_t stream) {
  if (C <= 0 || P <= 0) return 0;
  const int vec = ((uintptr_t)dst % 16 == 0) && ((uintptr_t)src % 16 == 0) && (ld % 4 == 0);
  static int rows = -1;
  if (rows < 0) {
    const char* e = getenv("FEDML_AMD_BCAST_ROWS");
    rows = e && atoi(e) > 0 ? atoi(e) : 8;
  }
  dim3 grid(fa_grid(vec ? (P + 3) / 4 : P, 256, 1024), (C + rows - 1) / rows);
  hipLaunchKernelGGL(broadcast_rows_kernel, grid, dim3(256), 0, stream, dst, src, P, ld, vec, C, rows);
  return (int)hipGetLastError();
}

// =====================================================================================
// K10  Fused server step for FedOpt: avg = Σ w_c X_c;  g = global - avg (pseudo-gradient,
//      `mpi_p2p_mp/fedopt/FedOptAggregator.py:120-134`); then one of
//      0 SGD(+momentum) [FedAvgM], 1 Adam [FedAdam], 2 Yogi [FedYogi], 3 Adagrad [FedAdagrad]
//      applied to `global` in place — one pass over [C, P], no materialised average.
// =====================================================================================
__global__ __launch_bounds__(256) void fedopt_kernel(const float* __restrict__ X, int64_t ldx, int C,
                                                     const float* __restrict__ w, float* __restrict__ glob,
                                                     float* __restrict__ s1, float* __restrict__ s2, int64_t P, int opt,
                                                     float lr, float b1, float b2, float eps, float bc1, float bc2,
                                                     float momentum, int nesterov, int first_step) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    float avg = 0.f;
    for (int c = 0; c < C; ++c) avg += w[c] * X[(int64_t)c * ldx + i];
    const float p = glob[i];
    const float g = p - avg;
    float np;
    if (opt == 0) {
      float d = g;
      if (momentum != 0.f) {
        float b = first_step ? g : momentum * s1[i] + g;
        s1[i] = b;
        d = nesterov ? g + momentum * b : b;
      }
      np = p - lr * d;
    } else if (opt == 1 || opt == 2) {
      float m = b1 * s1[i] + (1.f - b1) * g;
      float v;
      if (opt == 1) {
        v = b2 * s2[i] + (1.f - b2) * g * g;
      } else {  // Yogi: v = v - (1-b2) * g^2 * sign(v - g^2)
        const float g2 = g * g;
        const float vo = s2[i];
        v = vo - (1.f - b2) * g2 * copysignf(1.f, vo - g2);
      }
      s1[i] = m;
      s2[i] = v;
      np = p - lr * (m / bc1) / (sqrtf(fmaxf(v, 0.f) / bc2) + eps);
    } else {  // Adagrad
      float v = s2[i] + g * g;
      s2[i] = v;
      np = p - lr * g / (sqrtf(v) + eps);
    }
    glob[i] = np;
  }
}

FA_EXPORT int fa_fedopt_step(const float* X, int64_t ldx, int C, const float* w, float* glob, float* s1, float* s2,
                             int64_t P, int opt, float lr, float b1, float b2, float eps, float bc1, float bc2,
                             float momentum, int nesterov, int first_step, hipStream_t stream) {
  hipLaunchKernelGGL(fedopt_kernel, dim3(fa_grid(P, 256, 2048)), dim3(256), 0, stream, X, ldx, C, w, glob, s1, s2, P,
                     opt, lr, b1, b2, eps, bc1, bc2, momentum, nesterov, first_step);
  return (int)hipGetLastError();
}

// =====================================================================================
// K11  FedNova server step (`single_process/fednova/fednova_trainer.py` aggregate, Wang et al. 2020) on
//      the all-reduced coefficient-weighted client sum wsum = Σ_i coef_i·w_i, coef_i = τ_eff·p_i / a_i,
//      S = Σ_i coef_i (device scalar: no host sync):
//        cum = S·g − wsum                 (τ_eff · Σ p_i (g − w_i)/a_i, the normalised cumulative update)
//        gmf = 0:  g ← g − cum
//        gmf > 0:  buf ← first ? cum/lr : gmf·buf + cum/lr;   g ← g − lr·buf   (server momentum)
//      one pass over P instead of the reference's per-tensor loops.
// =====================================================================================
__global__ __launch_bounds__(256) void fednova_server_kernel(float* __restrict__ glob, const float* __restrict__ wsum,
                                                             const float* __restrict__ S_ptr, float* __restrict__ buf,
                                                             int64_t P, float gmf, float lr, int first) {
  const float S = *S_ptr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    const float g = glob[i];
    const float cum = S * g - wsum[i];
    if (gmf != 0.f) {
      const float b = first ? cum / lr : gmf * buf[i] + cum / lr;
      buf[i] = b;
      glob[i] = g - lr * b;
    } else {
      glob[i] = g - cum;
    }
  }
}

FA_EXPORT int fa_fednova_server_step(float* glob, const float* wsum, const float* S, float* buf, int64_t P, float gmf,
                                     float lr, int first, hipStream_t stream) {
  if (gmf != 0.f && (!buf || lr == 0.f)) return -1;
  hipLaunchKernelGGL(fednova_server_kernel, dim3(fa_grid(P, 256, 2048)), dim3(256), 0, stream, glob, wsum, S, buf, P,
                     gmf, lr, first);
  return (int)hipGetLastError();
}

// =====================================================================================
// K9  Robust aggregation (`core/robustness/robust_aggregation.py`)
//   per-client squared L2 norm of (X_c - G) restricted to a mask of "weight" coordinates
//   (BN running stats excluded, `is_weight_param`), deterministic two-level reduction:
//   fixed 64 partial slots per client, then an ordered finalize.
// =====================================================================================
constexpr int kNormSlots = 64;

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(const float* __restrict__ X, int64_t ldx,
                                                             const float* __restrict__ G,
                                                             const uint8_t* __restrict__ mask, int64_t P,
                                                             float* __restrict__ partial) {
  __shared__ float red[4];
  const int c = blockIdx.y;
  const float* xc = X + (int64_t)c * ldx;
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    if (mask && !mask[i]) continue;
    float d = xc[i] - (G ? G[i] : 0.f);
    acc += d * d;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partial[c * kNormSlots + blockIdx.x] = acc;
}

__global__ void sqnorm_finalize_kernel(const float* __restrict__ partial, float* __restrict__ out, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int j = 0; j < kNormSlots; ++j) s += partial[c * kNormSlots + j];
  out[c] = s;
}

// `partial` scratch must hold C*64 floats.
FA_EXPORT int fa_client_sqnorm(const float* X, int64_t ldx, int C, const float* G, const uint8_t* mask, int64_t P,
                               float* partial, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(kNormSlots, C), dim3(256), 0, stream, X, ldx, G, mask, P, partial);
  hipLaunchKernelGGL(sqnorm_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, stream, partial, out, C);
  return (int)hipGetLastError();
}

// X_c ← G + (X_c - G) / max(1, ||X_c - G|| / bound)   (masked coordinates only)
__global__ __launch_bounds__(256) void clip_kernel(float* __restrict__ X, int64_t ldx, const float* __restrict__ G,
                                                   const uint8_t* __restrict__ mask, const float* __restrict__ sqn,
                                                   int64_t P, float bound) {
  const int c = blockIdx.y;
  const float nrm = sqrtf(sqn[c]);
  const float s = 1.f / fmaxf(1.f, nrm / bound);
  if (s == 1.f) return;
  float* xc = X + (int64_t)c * ldx;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    if (mask && !mask[i]) continue;
    const float g = G ? G[i] : 0.f;
    xc[i] = g + (xc[i] - g) * s;
  }
}

FA_EXPORT int fa_norm_clip(float* X, int64_t ldx, int C, const float* G, const uint8_t* mask, const float* sqn,
                           int64_t P, float bound, hipStream_t stream) {
  hipLaunchKernelGGL(clip_kernel, dim3(fa_grid(P, 256, 1024), C), dim3(256), 0, stream, X, ldx, G, mask, sqn, P,
                     bound);
  return (int)hipGetLastError();
}

// x += stddev * N(0,1), Box–Muller on Philox(seed, offset + i)
__global__ __launch_bounds__(256) void gauss_noise_kernel(float* __restrict__ x, const uint8_t* __restrict__ mask,
                                                          int64_t n, float stddev, uint32_t seed_lo, uint32_t seed_hi,
                                                          uint64_t offset) {
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    const uint64_t ctr = offset + (uint64_t)i;
    Philox4 r = philox4x32((uint32_t)ctr, (uint32_t)(ctr >> 32), 0x5eed, 0, seed_lo, seed_hi);
    const float u1 = u01(r.v[0]), u2 = u01(r.v[1]), u3 = u01(r.v[2]), u4 = u01(r.v[3]);
    const float m1 = sqrtf(-2.f * __logf(u1)), m2 = sqrtf(-2.f * __logf(u3));
    float z[4];
    z[0] = m1 * __cosf(6.2831853f * u2);
    z[1] = m1 * __sinf(6.2831853f * u2);
    z[2] = m2 * __cosf(6.2831853f * u4);
    z[3] = m2 * __sinf(6.2831853f * u4);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j < n && (!mask || mask[i + j])) x[i + j] += stddev * z[j];
  }
}

FA_EXPORT int fa_gaussian_noise(float* x, const uint8_t* mask, int64_t n, float stddev, uint64_t seed,
                                uint64_t offset, hipStream_t stream) {
  hipLaunchKernelGGL(gauss_noise_kernel, dim3(fa_grid((n + 3) / 4, 256, 2048)), dim3(256), 0, stream, x, mask, n,
                     stddev, (uint32_t)seed, (uint32_t)(seed >> 32), offset);
  return (int)hipGetLastError();
}

// Coordinate-wise median over C clients (torch.median convention: lower median).
// One coordinate per lane, values held in registers, fully unrolled bitonic network
// over NMAX (padded with +inf) so every index is compile-time → no scratch.
template <int NMAX>
__global__ __launch_bounds__(256) void median_kernel(const float* __restrict__ X, int64_t ldx, int C, int64_t P,
                                                     float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float v[NMAX];
#pragma unroll
  for (int c = 0; c < NMAX; ++c) v[c] = (c < C) ? X[(int64_t)c * ldx + i] : INFINITY;
#pragma unroll
  for (int k = 2; k <= NMAX; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int a = 0; a < NMAX; ++a) {
        const int b = a ^ j;
        if (b > a) {
          const bool up = ((a & k) == 0);
          const float x = v[a], y = v[b];
          const float lo = fminf(x, y), hi = fmaxf(x, y);
          v[a] = up ? lo : hi;
          v[b] = up ? hi : lo;
        }
      }
    }
  }
  const int mid = (C - 1) / 2;
  float r = v[0];
#pragma unroll
  for (int c = 1; c < NMAX; ++c)
    if (c == mid) r = v[c];
  out[i] = r;
}

FA_EXPORT int fa_coordinate_median(const float* X, int64_t ldx, int C, int64_t P, float* out, hipStream_t stream) {
  const int grid = (int)((P + 255) / 256);
  if (C <= 8) hipLaunchKernelGGL(median_kernel<8>, dim3(grid), dim3(256), 0, stream, X, ldx, C, P, out);
  else if (C <= 16) hipLaunchKernelGGL(median_kernel<16>, dim3(grid), dim3(256), 0, stream, X, ldx, C, P, out);
  else if (C <= 32) hipLaunchKernelGGL(median_kernel<32>, dim3(grid), dim3(256), 0, stream, X, ldx, C, P, out);
  else if (C <= 64) hipLaunchKernelGGL(median_kernel<64>, dim3(grid), dim3(256), 0, stream, X, ldx, C, P, out);
  else return -1;
  return (int)hipGetLastError();
}

// =====================================================================================
// K15  Update compression (absent in the reference; required by the north star)
//   (a) block-scaled int8 with stochastic rounding + error feedback
//   (b) block-scaled fp8 (OCP e4m3fn, gfx950 hardware convert)
//   (c) exact top-k by |x| via 3-pass radix select on the float bits, device-resident state
// =====================================================================================
// one wave per quantisation block of 256 values (4 per lane)
__global__ __launch_bounds__(256) void quant_int8_kernel(const float* __restrict__ x, float* __restrict__ residual,
                                                         int8_t* __restrict__ q, float* __restrict__ scales, int64_t n,
                                                         int stochastic, uint32_t seed_lo, uint32_t seed_hi) {
  const int lane = threadIdx.x & 63;
  const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t base = blk * 256 + lane * 4;
  if (blk * 256 >= n) return;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = base + j;
    v[j] = (i < n) ? x[i] + (residual ? residual[i] : 0.f) : 0.f;
  }
  float amax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
  amax = wave_max(amax);
  const float scale = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / scale;
  Philox4 r = philox4x32((uint32_t)base, (uint32_t)(base >> 32), 0x0a11, 0, seed_lo, seed_hi);
  char4 packed;
  int8_t qq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float t = v[j] * inv;
    t = stochastic ? floorf(t + u01(r.v[j]) - 1e-7f) : rintf(t);
    t = fminf(fmaxf(t, -127.f), 127.f);
    qq[j] = (int8_t)t;
    if (residual && base + j < n) residual[base + j] = v[j] - t * scale;
  }
  packed.x = qq[0]; packed.y = qq[1]; packed.z = qq[2]; packed.w = qq[3];
  if (base + 3 < n) {
    *reinterpret_cast<char4*>(q + base) = packed;
  } else {
    for (int j = 0; j < 4; ++j)
      if (base + j < n) q[base + j] = qq[j];
  }
  if (lane == 0) scales[blk] = scale;
}

FA_EXPORT int fa_quant_int8(const float* x, float* residual, int8_t* q, float* scales, int64_t n, int stochastic,
                            uint64_t seed, hipStream_t stream) {
  const int64_t nblk = (n + 255) / 256;
  hipLaunchKernelGGL(quant_int8_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, stream, x, residual, q,
                     scales, n, stochastic, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (int)hipGetLastError();
}

// acc[i] += w * q[i] * scale[i/256]
__global__ __launch_bounds__(256) void dequant_int8_axpy_kernel(const int8_t* __restrict__ q,
                                                                const float* __restrict__ scales, float w,
                                                                float* __restrict__ acc, int64_t n) {
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    const float s = w * scales[i >> 8];
    if (i + 3 < n) {
      const char4 c = *reinterpret_cast<const char4*>(q + i);
      f32x4* a = reinterpret_cast<f32x4*>(acc + i);
      f32x4 t = *a;
      t.x += s * c.x; t.y += s * c.y; t.z += s * c.z; t.w += s * c.w;
      *a = t;
    } else {
      for (int j = 0; j < 4 && i + j < n; ++j) acc[i + j] += s * q[i + j];
    }
  }
}

FA_EXPORT int fa_dequant_int8_axpy(const int8_t* q, const float* scales, float w, float* acc, int64_t n,
                                   hipStream_t stream) {
  hipLaunchKernelGGL(dequant_int8_axpy_kernel, dim3(fa_grid((n + 3) / 4, 256, 2048)), dim3(256), 0, stream, q, scales,
                     w, acc, n);
  return (int)hipGetLastError();
}

// fp8 e4m3fn (OCP; max finite 448) with a per-256 block scale
__global__ __launch_bounds__(256) void quant_fp8_kernel(const float* __restrict__ x, float* __restrict__ residual,
                                                        uint8_t* __restrict__ q, float* __restrict__ scales,
                                                        int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t base = blk * 256 + lane * 4;
  if (blk * 256 >= n) return;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = base + j;
    v[j] = (i < n) ? x[i] + (residual ? residual[i] : 0.f) : 0.f;
  }
  float amax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
  amax = wave_max(amax);
  const float scale = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / scale;
  float t[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = fminf(fmaxf(v[j] * inv, -448.f), 448.f);
  int pk = __builtin_amdgcn_cvt_pk_fp8_f32(t[0], t[1], 0, false);
  pk = __builtin_amdgcn_cvt_pk_fp8_f32(t[2], t[3], pk, true);
  if (residual) {
    float back[4];
    back[0] = __builtin_amdgcn_cvt_f32_fp8(pk, 0);
    back[1] = __builtin_amdgcn_cvt_f32_fp8(pk, 1);
    back[2] = __builtin_amdgcn_cvt_f32_fp8(pk, 2);
    back[3] = __builtin_amdgcn_cvt_f32_fp8(pk, 3);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (base + j < n) residual[base + j] = v[j] - back[j] * scale;
  }
  if (base + 3 < n) {
    *reinterpret_cast<int*>(q + base) = pk;
  } else {
    for (int j = 0; j < 4; ++j)
      if (base + j < n) q[base + j] = (uint8_t)((pk >> (8 * j)) & 0xff);
  }
  if (lane == 0) scales[blk] = scale;
}

FA_EXPORT int fa_quant_fp8(const float* x, float* residual, uint8_t* q, float* scales, int64_t n,
                           hipStream_t stream) {
  const int64_t nblk = (n + 255) / 256;
  hipLaunchKernelGGL(quant_fp8_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, stream, x, residual, q, scales,
                     n);
  return (int)hipGetLastError();
}

__global__ __launch_bounds__(256) void dequant_fp8_axpy_kernel(const uint8_t* __restrict__ q,
                                                               const float* __restrict__ scales, float w,
                                                               float* __restrict__ acc, int64_t n) {
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    const float s = w * scales[i >> 8];
    if (i + 3 < n) {
      const int pk = *reinterpret_cast<const int*>(q + i);
      f32x4* a = reinterpret_cast<f32x4*>(acc + i);
      f32x4 t = *a;
      t.x += s * __builtin_amdgcn_cvt_f32_fp8(pk, 0);
      t.y += s * __builtin_amdgcn_cvt_f32_fp8(pk, 1);
      t.z += s * __builtin_amdgcn_cvt_f32_fp8(pk, 2);
      t.w += s * __builtin_amdgcn_cvt_f32_fp8(pk, 3);
      *a = t;
    } else {
      for (int j = 0; j < 4 && i + j < n; ++j) acc[i + j] += s * __builtin_amdgcn_cvt_f32_fp8((int)q[i + j], 0);
    }
  }
}

FA_EXPORT int fa_dequant_fp8_axpy(const uint8_t* q, const float* scales, float w, float* acc, int64_t n,
                                  hipStream_t stream) {
  hipLaunchKernelGGL(dequant_fp8_axpy_kernel, dim3(fa_grid((n + 3) / 4, 256, 2048)), dim3(256), 0, stream, q, scales,
                     w, acc, n);
  return (int)hipGetLastError();
}

// ---- all clients of a GPU in ONE launch: compress (int8 stochastic | fp8) Δ_c = w_c − w_global with
// error feedback, decompress straight into the aggregate: acc = Σ_c n_c·(w_global + D(C(Δ_c + r_c))),
// r_c ← Δ_c + r_c − D(C(·)). One wave per 256-value quantisation block loops over the C clients, so acc
// is written once per element (no atomics, no [C, P] intermediate, no per-client host loop).
// residual_rows[c] = the client's residual row (0 = none); weights / client ids read on the device.
template <int MODE>  // 0 int8 stochastic, 1 fp8 e4m3fn
__global__ __launch_bounds__(256) void compress_accumulate_kernel(
    const float* __restrict__ params, int64_t ldp, int C, const float* __restrict__ glob,
    const uint64_t* __restrict__ residual_rows, const float* __restrict__ weights, const int64_t* __restrict__ ids,
    float* __restrict__ acc, int64_t n, uint32_t seed_lo, uint32_t seed_hi) {
  const int lane = threadIdx.x & 63;
  const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t base = blk * 256 + lane * 4;
  if (blk * 256 >= n) return;
  float g[4], a[4] = {0.f, 0.f, 0.f, 0.f};
  float wsum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) g[j] = (base + j < n) ? glob[base + j] : 0.f;
  for (int c = 0; c < C; ++c) {
    const float w = weights[c];
    if (w == 0.f) continue;   // wave-uniform
    wsum += w;
    float* res = reinterpret_cast<float*>(residual_rows ? residual_rows[c] : 0ull);
    const float* pc = params + (int64_t)c * ldp;
    float v[4];
    // 16-B accesses when this lane's 4 values are in range and the rows are 16-B aligned (one load per operand
    // instead of four: the kernel is a stream over [C, P] params + residuals)
    const bool vec = base + 3 < n && (((uintptr_t)(pc + base) | (uintptr_t)(res ? res + base : pc + base)) & 15) == 0;
    if (vec) {
      const float4 p4 = *reinterpret_cast<const float4*>(pc + base);
      const float4 r4 = res ? *reinterpret_cast<const float4*>(res + base) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[0] = p4.x - g[0] + r4.x;
      v[1] = p4.y - g[1] + r4.y;
      v[2] = p4.z - g[2] + r4.z;
      v[3] = p4.w - g[3] + r4.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t i = base + j;
        v[j] = (i < n) ? pc[i] - g[j] + (res ? res[i] : 0.f) : 0.f;
      }
    }
    float amax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    amax = wave_max(amax);
    float back[4];
    if (MODE == 0) {
      const float scale = amax > 0.f ? amax / 127.f : 1.f;
      const float inv = 1.f / scale;
      const uint32_t cid = (uint32_t)ids[c];
      Philox4 r = philox4x32((uint32_t)base, (uint32_t)(base >> 32), 0x0a11, cid, seed_lo, seed_hi);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float t = floorf(v[j] * inv + u01(r.v[j]) - 1e-7f);
        t = fminf(fmaxf(t, -127.f), 127.f);
        back[j] = t * scale;
      }
    } else {
      const float scale = amax > 0.f ? amax / 448.f : 1.f;
      const float inv = 1.f / scale;
      float t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = fminf(fmaxf(v[j] * inv, -448.f), 448.f);
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(t[0], t[1], 0, false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(t[2], t[3], pk, true);
      back[0] = __builtin_amdgcn_cvt_f32_fp8(pk, 0) * scale;
      back[1] = __builtin_amdgcn_cvt_f32_fp8(pk, 1) * scale;
      back[2] = __builtin_amdgcn_cvt_f32_fp8(pk, 2) * scale;
      back[3] = __builtin_amdgcn_cvt_f32_fp8(pk, 3) * scale;
    }
    if (vec && res) {
      *reinterpret_cast<float4*>(res + base) = make_float4(v[0] - back[0], v[1] - back[1], v[2] - back[2], v[3] - back[3]);
    } else if (res) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (base + j < n) res[base + j] = v[j] - back[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] += w * back[j];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (base + j < n) acc[base + j] = a[j] + wsum * g[j];
}

FA_EXPORT int fa_compress_accumulate(const float* params, int64_t ldp, int C, const float* glob,
                                     const uint64_t* residual_rows, const float* weights, const int64_t* ids,
                                     float* acc, int64_t n, int mode, uint64_t seed, hipStream_t stream) {
  const int64_t nblk = (n + 255) / 256;
  const dim3 grid((unsigned)((nblk + 3) / 4));
  if (mode == 0)
    hipLaunchKernelGGL(compress_accumulate_kernel<0>, grid, dim3(256), 0, stream, params, ldp, C, glob, residual_rows,
                       weights, ids, acc, n, (uint32_t)seed, (uint32_t)(seed >> 32));
  else if (mode == 1)
    hipLaunchKernelGGL(compress_accumulate_kernel<1>, grid, dim3(256), 0, stream, params, ldp, C, glob, residual_rows,
                       weights, ids, acc, n, (uint32_t)seed, (uint32_t)(seed >> 32));
  else
    return -2;
  return (int)hipGetLastError();
}

// ---- top-k: radix select over |x| float bits (31 significant bits: 11 + 11 + 9) ----
// state[0] = prefix bits fixed so far, state[1] = k still to take inside the prefix,
// state[2] = output cursor, state[3] = tie cursor, state[4] = threshold bits (final)
struct TopkPass {
  int shift;  // low bit of the digit
  int bits;   // digit width
};
__constant__ TopkPass kTopkPasses[3] = {{20, 11}, {9, 11}, {0, 9}};

__global__ __launch_bounds__(256) void topk_hist_kernel(const float* __restrict__ x, int64_t n, int pass,
                                                        const uint32_t* __restrict__ state,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[2048];
  const TopkPass ps = kTopkPasses[pass];
  const int nb = 1 << ps.bits;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t prefix = state[0];
  const int hi_shift = ps.shift + ps.bits;  // bits above the digit must match prefix
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t a = __float_as_uint(x[i]) & 0x7fffffffu;
    if (hi_shift < 31 && (a >> hi_shift) != (prefix >> hi_shift)) continue;
    atomicAdd(&h[(a >> ps.shift) & (nb - 1)], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// single workgroup: walk the histogram from the top, fix the digit holding the k-th element
__global__ void topk_select_kernel(uint32_t* __restrict__ hist, int pass, uint32_t* __restrict__ state) {
  if (threadIdx.x != 0) return;
  const TopkPass ps = kTopkPasses[pass];
  const int nb = 1 << ps.bits;
  uint32_t k = state[1];
  uint32_t cum = 0;
  int digit = 0;
  for (int b = nb - 1; b >= 0; --b) {
    if (cum + hist[b] >= k) {
      digit = b;
      break;
    }
    cum += hist[b];
  }
  state[0] |= ((uint32_t)digit << ps.shift);
  state[1] = k - cum;
  for (int b = 0; b < nb; ++b) hist[b] = 0;  // ready for the next pass
}

// compaction: |x| > T → take; |x| == T → take the first `state[1]` ties
__global__ __launch_bounds__(256) void topk_compact_kernel(const float* __restrict__ x, int64_t n,
                                                           uint32_t* __restrict__ state, int32_t* __restrict__ idx,
                                                           float* __restrict__ val, float* __restrict__ residual,
                                                           int64_t kmax) {
  const uint32_t T = state[0];
  const uint32_t ties = state[1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    const uint32_t a = __float_as_uint(v) & 0x7fffffffu;
    bool take = a > T;
    if (!take && a == T) take = atomicAdd(&state[3], 1u) < ties;
    if (take) {
      const uint32_t slot = atomicAdd(&state[2], 1u);
      if (slot < kmax) {
        idx[slot] = (int32_t)i;
        val[slot] = v;
      }
      if (residual) residual[i] = 0.f;
    } else if (residual) {
      residual[i] = v;
    }
  }
}

__global__ void topk_init_kernel(uint32_t* __restrict__ state, uint32_t* __restrict__ hist, uint32_t k) {
  for (int b = threadIdx.x; b < 2048; b += blockDim.x) hist[b] = 0;
  if (threadIdx.x < 8) state[threadIdx.x] = (threadIdx.x == 1) ? k : 0u;
}

// state: 8 uint32 device scratch; hist: 2048 uint32 scratch (both zeroed by the caller once)
FA_EXPORT int fa_topk_abs(const float* x, int64_t n, int64_t k, uint32_t* state, uint32_t* hist, int32_t* idx,
                          float* val, float* residual, hipStream_t stream) {
  hipLaunchKernelGGL(topk_init_kernel, dim3(1), dim3(256), 0, stream, state, hist, (uint32_t)k);
  const int grid = fa_grid(n, 256, 1024);
  for (int pass = 0; pass < 3; ++pass) {
    hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(256), 0, stream, x, n, pass, state, hist);
    hipLaunchKernelGGL(topk_select_kernel, dim3(1), dim3(64), 0, stream, hist, pass, state);
  }
  hipLaunchKernelGGL(topk_compact_kernel, dim3(grid), dim3(256), 0, stream, x, n, state, idx, val, residual, k);
  return (int)hipGetLastError();
}

// ---- batched top-k with error feedback over the [C, P] client stack (8 launches for any C) ----
// Client c's update Δ_c = params_c − glob + r_c keeps its k largest |Δ_c| entries; the rest becomes its new
// residual r_c. The same 3-pass radix select as topk_abs, but every pass runs all clients in ONE grid
// (blockIdx.y = client, per-client histogram and state), Δ_c is recomputed from the arenas in each pass
// (reading params + residual costs less than writing and re-reading a [C, P] scratch), and the final pass
// applies the selection and accumulates acc = Σ_c w_c·(glob + topk(Δ_c)) with one thread per element
// looping over the clients — no atomics on acc, no per-client host loop.
// state[c][0] prefix bits, [1] k left inside the prefix, [3] tie cursor.
__global__ __launch_bounds__(256) void topkb_init_kernel(uint32_t* __restrict__ state, uint32_t* __restrict__ hist,
                                                         int C, uint32_t k) {
  const int c = blockIdx.x;
  for (int b = threadIdx.x; b < 2048; b += blockDim.x) hist[(int64_t)c * 2048 + b] = 0;
  if (threadIdx.x < 8) state[c * 8 + threadIdx.x] = (threadIdx.x == 1) ? k : 0u;
}

__device__ __forceinline__ float4 topkb_delta(const float* __restrict__ pc, const float* __restrict__ glob,
                                              const float* __restrict__ res, int64_t i) {
  const float4 p = *reinterpret_cast<const float4*>(pc + i);
  const float4 g = *reinterpret_cast<const float4*>(glob + i);
  float4 v = make_float4(p.x - g.x, p.y - g.y, p.z - g.z, p.w - g.w);
  if (res) {
    const float4 r = *reinterpret_cast<const float4*>(res + i);
    v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
  }
  return v;
}

// grid (blocks per client, C); n % 4 == 0, rows 16-byte aligned
__global__ __launch_bounds__(256) void topkb_hist_kernel(const float* __restrict__ params, int64_t ldp,
                                                         const float* __restrict__ glob,
                                                         const uint64_t* __restrict__ rows,
                                                         const float* __restrict__ weights, int64_t n, int pass,
                                                         const uint32_t* __restrict__ state,
                                                         uint32_t* __restrict__ hist) {
  const int c = blockIdx.y;
  if (weights[c] == 0.f) return;   // block-uniform: padding / dropped slots
  __shared__ uint32_t h[2048];
  const TopkPass ps = kTopkPasses[pass];
  const int nb = 1 << ps.bits;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t prefix = state[c * 8];
  const int hi_shift = ps.shift + ps.bits;
  const float* pc = params + (int64_t)c * ldp;
  const float* res = reinterpret_cast<const float*>(rows ? rows[c] : 0ull);
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    const float4 v = topkb_delta(pc, glob, res, i);
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t a = __float_as_uint(e[j]) & 0x7fffffffu;
      if (hi_shift < 31 && (a >> hi_shift) != (prefix >> hi_shift)) continue;
      atomicAdd(&h[(a >> ps.shift) & (nb - 1)], 1u);
    }
  }
  __syncthreads();
  uint32_t* hc = hist + (int64_t)c * 2048;
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&hc[b], h[b]);
}

// one wave per client: lane l owns 32 bins counted from the top, a wave prefix sum finds the lane holding
// the k-th element, that lane walks its bins; the histogram is cleared for the next pass
__global__ __launch_bounds__(64) void topkb_select_kernel(uint32_t* __restrict__ hist, int pass,
                                                          uint32_t* __restrict__ state,
                                                          const float* __restrict__ weights) {
  const int c = blockIdx.x;
  if (weights[c] == 0.f) return;
  const TopkPass ps = kTopkPasses[pass];
  const int nb = 1 << ps.bits;
  const int per = nb / 64;   // 32 (11-bit passes) or 8 (9-bit pass)
  uint32_t* hc = hist + (int64_t)c * 2048;
  const int lane = threadIdx.x;
  const int top = nb - 1 - lane * per;   // this lane's bins: top, top-1, …, top-per+1
  uint32_t mine = 0;
  for (int j = 0; j < per; ++j) mine += hc[top - j];
  uint32_t incl = mine;   // inclusive scan from lane 0 (the highest bins)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const uint32_t k = state[c * 8 + 1];
  const uint64_t hit = __ballot(incl >= k);
  const int owner = hit ? __ffsll((long long)hit) - 1 : 63;
  if (lane == owner) {
    uint32_t cum = incl - mine;
    int digit = top - per + 1;
    for (int j = 0; j < per; ++j) {
      const uint32_t hb = hc[top - j];
      if (cum + hb >= k) {
        digit = top - j;
        break;
      }
      cum += hb;
    }
    state[c * 8] |= ((uint32_t)digit << ps.shift);
    state[c * 8 + 1] = k - cum;
  }
  __syncthreads();
  for (int b = lane; b < nb; b += 64) hc[b] = 0;
}

// one thread per 4 elements, looping over the clients: take |Δ| > T_c and the first `ties` entries equal
// to T_c; acc = wsum·glob + Σ w_c·taken Δ_c; residual ← untaken Δ_c (0 where taken)
__global__ __launch_bounds__(256) void topkb_apply_kernel(const float* __restrict__ params, int64_t ldp, int C,
                                                          const float* __restrict__ glob,
                                                          const uint64_t* __restrict__ rows,
                                                          const float* __restrict__ weights, int64_t n,
                                                          uint32_t* __restrict__ state, float* __restrict__ acc) {
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    const float4 g = *reinterpret_cast<const float4*>(glob + i);
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    float wsum = 0.f;
    for (int c = 0; c < C; ++c) {
      const float w = weights[c];
      if (w == 0.f) continue;
      wsum += w;
      float* res = reinterpret_cast<float*>(rows ? rows[c] : 0ull);
      const float4 v4 = topkb_delta(params + (int64_t)c * ldp, glob, res, i);
      const uint32_t T = state[c * 8], ties = state[c * 8 + 1];
      float e[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t bits = __float_as_uint(e[j]) & 0x7fffffffu;
        bool take = bits > T;
        if (!take && bits == T) take = atomicAdd(&state[c * 8 + 3], 1u) < ties;
        if (take) {
          a[j] += w * e[j];
          e[j] = 0.f;
        }
      }
      if (res) *reinterpret_cast<float4*>(res + i) = make_float4(e[0], e[1], e[2], e[3]);
    }
    *reinterpret_cast<float4*>(acc + i) =
        make_float4(a[0] + wsum * g.x, a[1] + wsum * g.y, a[2] + wsum * g.z, a[3] + wsum * g.w);
  }
}

// state: C·8 uint32, hist: C·2048 uint32 scratch; rows: C residual-row pointers (0 = none) or null
FA_EXPORT int fa_topk_compress_accumulate(const float* params, int64_t ldp, int C, const float* glob,
                                          const uint64_t* rows, const float* weights, int64_t n, int64_t k,
                                          uint32_t* state, uint32_t* hist, float* acc, hipStream_t stream) {
  if (C <= 0 || C > 65535 || n <= 0 || (n & 3) || (ldp & 3) || k <= 0 || k > n || k > 0xffffffffll)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(topkb_init_kernel, dim3(C), dim3(256), 0, stream, state, hist, C, (uint32_t)k);
  const int per_client = (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + 255) / 256, std::max(1, 4096 / C)));
  for (int pass = 0; pass < 3; ++pass) {
    hipLaunchKernelGGL(topkb_hist_kernel, dim3(per_client, C), dim3(256), 0, stream, params, ldp, glob, rows,
                       weights, n, pass, state, hist);
    hipLaunchKernelGGL(topkb_select_kernel, dim3(C), dim3(64), 0, stream, hist, pass, state, weights);
  }
  hipLaunchKernelGGL(topkb_apply_kernel, dim3(fa_grid(n / 4, 256, 8192)), dim3(256), 0, stream, params, ldp, C, glob,
                     rows, weights, n, state, acc);
  return (int)hipGetLastError();
}

// acc[idx[j]] += w * val[j]   (indices of one client are unique → no atomics needed)
__global__ __launch_bounds__(256) void scatter_axpy_kernel(const int32_t* __restrict__ idx,
                                                           const float* __restrict__ val, int64_t k, float w,
                                                           float* __restrict__ acc) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += (int64_t)gridDim.x * blockDim.x)
    acc[idx[j]] += w * val[j];
}

FA_EXPORT int fa_scatter_axpy(const int32_t* idx, const float* val, int64_t k, float w, float* acc,
                              hipStream_t stream) {
  hipLaunchKernelGGL(scatter_axpy_kernel, dim3(fa_grid(k, 256, 2048)), dim3(256), 0, stream, idx, val, k, w, acc);
  return (int)hipGetLastError();
}

// =====================================================================================
// K7  Fused softmax cross-entropy forward+backward (one wave per row).
//   loss_row = -cw[y] * log softmax(z)[y];  dz = cw[y] * (softmax(z) - onehot(y)) * row_scale
//   ignore_index rows give 0 loss / 0 grad (NWP padding, `my_model_trainer_nwp.py`).
// =====================================================================================
template <typename T>
__global__ __launch_bounds__(256) void xent_kernel(const T* __restrict__ z, const int64_t* __restrict__ y,
                                                   const float* __restrict__ cw, const float* __restrict__ row_scale,
                                                   T* __restrict__ dz, float* __restrict__ loss, int64_t R, int K,
                                                   int64_t ignore_index) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* zr = z + row * K;
  const int64_t lbl = y[row];
  const bool ign = (lbl == ignore_index) || lbl < 0 || lbl >= K;
  float m = -INFINITY;
  for (int j = lane; j < K; j += 64) m = fmaxf(m, load1<T>(zr + j));
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < K; j += 64) s += __expf(load1<T>(zr + j) - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
  const float w = ign ? 0.f : (cw ? cw[lbl] : 1.f);
  const float rs = row_scale ? row_scale[row] : 1.f;
  if (dz) {
    T* dr = dz + row * K;
    const float inv = 1.f / s;
    for (int j = lane; j < K; j += 64) {
      float p = __expf(load1<T>(zr + j) - m) * inv;
      float g = w * rs * (p - (j == lbl ? 1.f : 0.f));
      if constexpr (sizeof(T) == 4) dr[j] = g;
      else dr[j] = f32_to_bf16(g);
    }
  }
  if (lane == 0) loss[row] = ign ? 0.f : w * (lse - load1<T>(zr + lbl));
}

FA_EXPORT int fa_softmax_xent(const void* z, int is_bf16, const int64_t* y, const float* cw, const float* row_scale,
                              void* dz, float* loss, int64_t R, int K, int64_t ignore_index, hipStream_t stream) {
  const unsigned grid = (unsigned)((R + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL(xent_kernel<uint16_t>, dim3(grid), dim3(256), 0, stream, (const uint16_t*)z, y, cw, row_scale,
                       (uint16_t*)dz, loss, R, K, ignore_index);
  else
    hipLaunchKernelGGL(xent_kernel<float>, dim3(grid), dim3(256), 0, stream, (const float*)z, y, cw, row_scale,
                       (float*)dz, loss, R, K, ignore_index);
  return (int)hipGetLastError();
}

// =====================================================================================
// K8  On-device evaluation: argmax + confusion matrix per client (one wave per row),
//     replacing the reference's per-batch `.cpu().numpy()` counting
//     (`single_process/fedavg/my_model_trainer_classification.py:113-154`).
//     cm[group][label][pred] += 1, group = row / rows_per_group.
// =====================================================================================
template <typename T>
__global__ __launch_bounds__(256) void confusion_kernel(const T* __restrict__ z, const int64_t* __restrict__ y,
                                                        int32_t* __restrict__ cm, int64_t R, int K,
                                                        int64_t rows_per_group) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* zr = z + row * K;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = lane; j < K; j += 64) {
    const float v = load1<T>(zr + j);
    if (v > best || (v == best && j < bi)) { best = v; bi = j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  const int64_t lbl = y[row];
  if (lane == 0 && lbl >= 0 && lbl < K) {
    const int64_t g = row / rows_per_group;
    atomicAdd(&cm[(g * K + lbl) * K + bi], 1);
  }
}

FA_EXPORT int fa_confusion(const void* z, int is_bf16, const int64_t* y, int32_t* cm, int64_t R, int K,
                           int64_t rows_per_group, hipStream_t stream) {
  const unsigned grid = (unsigned)((R + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL(confusion_kernel<uint16_t>, dim3(grid), dim3(256), 0, stream, (const uint16_t*)z, y, cm, R, K,
                       rows_per_group);
  else
    hipLaunchKernelGGL(confusion_kernel<float>, dim3(grid), dim3(256), 0, stream, (const float*)z, y, cm, R, K,
                       rows_per_group);
  return (int)hipGetLastError();
}

// K8b  Evaluation statistics of a logits block in one pass (one wave per row): argmax, the row's cross-entropy
//      (log-sum-exp − z[y]) and, per group g = grp[row] (a client; null → group 0), the sums
//      sums[g] = (correct, loss, rows) and optionally per-class counts cls[g] = (true positives[K], actual[K],
//      predicted[K]) — what the fork's trainer test() derives per batch on the host
//      (`my_model_trainer_classification.py:113-154`, `fedavg_api.py:143-177`). Rows with a label outside
//      [0, K) or a negative group are padding and skipped.
template <typename T>
__global__ __launch_bounds__(256) void eval_stats_kernel(const T* __restrict__ z, const int64_t* __restrict__ y,
                                                         const int32_t* __restrict__ grp, float* __restrict__ sums,
                                                         int32_t* __restrict__ cls, int64_t R, int K) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int64_t lbl = y[row];
  const int g = grp != nullptr ? grp[row] : 0;
  if (lbl < 0 || lbl >= K || g < 0) return;          // uniform per wave: the whole wave leaves
  const T* zr = z + row * K;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = lane; j < K; j += 64) {
    const float v = load1<T>(zr + j);
    if (v > best || (v == best && j < bi)) { best = v; bi = j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  float se = 0.f;
  for (int j = lane; j < K; j += 64) se += __expf(load1<T>(zr + j) - best);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
  if (lane == 0) {
    const float loss = __logf(se) + best - load1<T>(zr + lbl);
    const int hit = bi == (int)lbl;
    atomicAdd(&sums[3 * g + 0], (float)hit);
    atomicAdd(&sums[3 * g + 1], loss);
    atomicAdd(&sums[3 * g + 2], 1.f);
    if (cls != nullptr) {
      int32_t* c = cls + (int64_t)g * 3 * K;
      if (hit) atomicAdd(&c[lbl], 1);
      atomicAdd(&c[K + lbl], 1);
      atomicAdd(&c[2 * K + bi], 1);
    }
  }
}

FA_EXPORT int fa_eval_stats(const void* z, int is_bf16, const int64_t* y, const int32_t* grp, float* sums,
                            int32_t* cls, int64_t R, int K, hipStream_t stream) {
  if (R <= 0) return 0;
  const unsigned grid = (unsigned)((R + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL(eval_stats_kernel<uint16_t>, dim3(grid), dim3(256), 0, stream, (const uint16_t*)z, y, grp, sums,
                       cls, R, K);
  else
    hipLaunchKernelGGL(eval_stats_kernel<float>, dim3(grid), dim3(256), 0, stream, (const float*)z, y, grp, sums, cls,
                       R, K);
  return (int)hipGetLastError();
}

// misc: fp32 → bf16 cast of a flat buffer (weights for bf16 compute)
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                        int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f32_to_bf16(x[i]);
}
FA_EXPORT int fa_cast_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t stream) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(fa_grid(n, 256, 2048)), dim3(256), 0, stream, x, y, n);
  return (int)hipGetLastError();
}

// =====================================================================================
// bf16 channels-last shadow of conv weights for the per-client (library conv) path: one launch
// writes every conv layer's OIHW fp32 master as bf16 OHWI (= an NCHW tensor with channels_last
// strides), so MIOpen's NHWC convolutions read it without a per-layer cast + layout copy.
// =====================================================================================
struct ShadowSeg {
  int64_t off;    // element offset of the weight slot in a client row (same in both arenas)
  int O, I, KH, KW;
};

__global__ __launch_bounds__(256) void pack_conv_shadow_kernel(const float* __restrict__ params, int64_t ldp,
                                                               uint16_t* __restrict__ shadow, int64_t lds,
                                                               const ShadowSeg* __restrict__ segs) {
  const ShadowSeg sg = segs[blockIdx.z];
  const int c = blockIdx.y;
  const int KK = sg.KH * sg.KW;
  const int n = sg.O * sg.I * KK;
  const float* src = params + (int64_t)c * ldp + sg.off;
  uint16_t* dst = shadow + (int64_t)c * lds + sg.off;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    // j indexes the OHWI destination: o, (h, w), i
    const int i = j % sg.I;
    const int t = j / sg.I;
    const int hw = t % KK;
    const int o = t / KK;
    dst[j] = f32_to_bf16(src[((int64_t)o * sg.I + i) * KK + hw]);
  }
}

FA_EXPORT int fa_pack_conv_shadow(const float* params, int64_t ldp, void* shadow, int64_t lds, const void* segs,
                                  int nseg, int max_n, int C, hipStream_t stream) {
  if (nseg <= 0) return 0;
  if (nseg > 65535 || C > 65535) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_conv_shadow_kernel, dim3(fa_grid(max_n, 256, 128), C, nseg), dim3(256), 0, stream, params,
                     ldp, (uint16_t*)shadow, lds, (const ShadowSeg*)segs);
  return (int)hipGetLastError();
}
