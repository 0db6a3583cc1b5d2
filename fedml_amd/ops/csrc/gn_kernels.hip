// GroupNorm forward / backward (reference: model/cv/group_normalization.py:7-93, which
// builds GroupNorm out of F.batch_norm on a reshaped input — three passes and a [1, N·G, ·] copy).
//
// Layout: x [N][R][L] contiguous, R = groups (summed over all clients of a client-stacked batch),
// L = cpg · HW (a group's channels are contiguous in NCHW). One workgroup per (n, r) row: the row is
// read for the two-pass mean/variance (second read from L2), normalised and written with the
// per-channel affine (optionally fused ReLU). Affine parameters may live in the fp32 client arena:
// channel ch of the stacked tensor belongs to client ch / chpc and reads w[client · w_cs + ch % chpc]
// (w_cs = 0 for a single model).
//
// Backward per row: Σ g and Σ g·x̂ (g = dy·γ) for dx = rstd·(g − mean(g) − x̂·mean(g·x̂)); dγ / dβ per
// channel are reduced over the row's HW positions in the workgroup and added with one fp32 atomic per
// channel and row into dense [R·cpg] accumulators.
#include "common.h"

namespace gnk {

constexpr int NT = 256;

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }

template <typename T>
__device__ __forceinline__ void st(T* p, int64_t i, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, int64_t i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st<uint16_t>(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }

struct Affine {
  const float* w;
  const float* b;
  int64_t w_cs, b_cs;
  int chpc;
  __device__ __forceinline__ float wv(int ch) const { return w ? w[(int64_t)(ch / chpc) * w_cs + ch % chpc] : 1.f; }
  __device__ __forceinline__ float bv(int ch) const { return b ? b[(int64_t)(ch / chpc) * b_cs + ch % chpc] : 0.f; }
};

template <typename T>
__global__ __launch_bounds__(NT) void gn_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, Affine af,
                                                    float* __restrict__ mean_out, float* __restrict__ rstd_out, int R,
                                                    int cpg, int HW, float eps, int relu) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const int r = row % R;
  const int L = cpg * HW;
  const int64_t base = (int64_t)row * L;
  float s = 0.f;
  for (int i = threadIdx.x; i < L; i += NT) s += ld(x, base + i);
  const float mean = block_sum(s, red) / (float)L;
  float q = 0.f;
  for (int i = threadIdx.x; i < L; i += NT) {
    const float d = ld(x, base + i) - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)L + eps);
  for (int j = 0; j < cpg; ++j) {
    const int ch = r * cpg + j;
    const float a = af.wv(ch) * rstd;
    const float c = af.bv(ch) - mean * a;
    for (int k = threadIdx.x; k < HW; k += NT) {
      const int64_t i = base + (int64_t)j * HW + k;
      float v = ld(x, i) * a + c;
      if (relu) v = fmaxf(v, 0.f);
      st(y, i, v);
    }
  }
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void gn_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x, Affine af,
                                                    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                    T* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
                                                    int R, int cpg, int HW) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const int r = row % R;
  const int L = cpg * HW;
  const int64_t base = (int64_t)row * L;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float s1 = 0.f, s2 = 0.f;
  for (int j = 0; j < cpg; ++j) {
    const int ch = r * cpg + j;
    const float w = af.wv(ch);
    float pw = 0.f, pb = 0.f;
    for (int k = threadIdx.x; k < HW; k += NT) {
      const int64_t i = base + (int64_t)j * HW + k;
      const float g = ld(dy, i);
      const float xh = (ld(x, i) - mean) * rstd;
      pw += g * xh;
      pb += g;
    }
    s1 += w * pb;
    s2 += w * pw;
    if (dw != nullptr || db != nullptr) {
      pw = block_sum(pw, red);
      pb = block_sum(pb, red);
      if (threadIdx.x == 0) {
        if (dw) atomicAdd(dw + ch, pw);
        if (db) atomicAdd(db + ch, pb);
      }
    }
  }
  const float m1 = block_sum(s1, red) / (float)L;
  const float m2 = block_sum(s2, red) / (float)L;
  for (int j = 0; j < cpg; ++j) {
    const int ch = r * cpg + j;
    const float w = af.wv(ch);
    for (int k = threadIdx.x; k < HW; k += NT) {
      const int64_t i = base + (int64_t)j * HW + k;
      const float xh = (ld(x, i) - mean) * rstd;
      st(dx, i, rstd * (w * ld(dy, i) - m1 - xh * m2));
    }
  }
}

}  // namespace gnk

// dtype: 0 = fp32, 1 = bf16. rows = N·R. w / b may be null (no affine).
FA_EXPORT int fa_gn_fwd(const void* x, void* y, const float* w, int64_t w_cs, const float* b, int64_t b_cs, int chpc,
                        float* mean, float* rstd, int64_t rows, int R, int cpg, int HW, float eps, int relu, int dtype,
                        hipStream_t stream) {
  using namespace gnk;
  if (rows <= 0 || rows > 0x7fffffff || R <= 0 || cpg <= 0 || HW <= 0 || chpc <= 0 || (int64_t)cpg * HW > 0x7fffffff)
    return (int)hipErrorInvalidValue;
  Affine af{w, b, w_cs, b_cs, chpc};
  if (dtype == 1)
    hipLaunchKernelGGL(gn_fwd_kernel<uint16_t>, dim3((unsigned)rows), dim3(NT), 0, stream, (const uint16_t*)x,
                       (uint16_t*)y, af, mean, rstd, R, cpg, HW, eps, relu);
  else
    hipLaunchKernelGGL(gn_fwd_kernel<float>, dim3((unsigned)rows), dim3(NT), 0, stream, (const float*)x, (float*)y, af,
                       mean, rstd, R, cpg, HW, eps, relu);
  return (int)hipGetLastError();
}

// dw / db: dense fp32 [R·cpg] accumulators (zeroed by the caller), may be null.
FA_EXPORT int fa_gn_bwd(const void* dy, const void* x, const float* w, int64_t w_cs, int chpc, const float* mean,
                        const float* rstd, void* dx, float* dw, float* db, int64_t rows, int R, int cpg, int HW,
                        int dtype, hipStream_t stream) {
  using namespace gnk;
  if (rows <= 0 || rows > 0x7fffffff || R <= 0 || cpg <= 0 || HW <= 0 || chpc <= 0 || (int64_t)cpg * HW > 0x7fffffff)
    return (int)hipErrorInvalidValue;
  Affine af{w, nullptr, w_cs, 0, chpc};
  if (dtype == 1)
    hipLaunchKernelGGL(gn_bwd_kernel<uint16_t>, dim3((unsigned)rows), dim3(NT), 0, stream, (const uint16_t*)dy,
                       (const uint16_t*)x, af, mean, rstd, (uint16_t*)dx, dw, db, R, cpg, HW);
  else
    hipLaunchKernelGGL(gn_bwd_kernel<float>, dim3((unsigned)rows), dim3(NT), 0, stream, (const float*)dy,
                       (const float*)x, af, mean, rstd, (float*)dx, dw, db, R, cpg, HW);
  return (int)hipGetLastError();
}
