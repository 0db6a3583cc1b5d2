// Shared helpers for the fedml_amd HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define FA_EXPORT extern "C" __attribute__((visibility("default")))

// CDNA wavefront = 64 lanes (never 32)
constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// round-to-nearest-even f32 → bf16: a plain cast, which hipcc -O3 lowers to the gfx950
// v_cvt_pk_bf16_f32 instruction (one per pair, NaN-preserving) instead of ~6 integer ops per value
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  const __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x multiple of 64 (≤1024); `red` needs blockDim.x/64 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  const int nw = blockDim.x >> 6;
  float t = (threadIdx.x < (unsigned)nw) ? red[threadIdx.x] : 0.f;
  if (wid == 0) t = wave_sum(t);
  __syncthreads();
  if (threadIdx.x == 0) red[0] = t;
  __syncthreads();
  float r = red[0];
  __syncthreads();
  return r;
}

// ---- counter-based RNG (Philox4x32-10) for noise / stochastic rounding ----
struct Philox4 {
  uint32_t v[4];
};
__device__ __forceinline__ Philox4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0; k1 += W1;
  }
  Philox4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}
__device__ __forceinline__ float u01(uint32_t x) {  // (0,1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

static inline int fa_grid(int64_t work, int block, int cap = 4096) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// Deterministic mode (utils/determinism.py): every client-batched launcher plans its work split (pixel chunks,
// workgroup targets, tile shapes) for this fixed client count instead of the launch's C, so the fp32 partial
// sums of one client — and so its bits — do not depend on how many clients share its GPU (a world-size
// invariant run). 0 (default): plan for the launch's own C. Set by fa_set_plan_clients (det_kernels.hip).
extern "C" int fa_plan_clients;
static inline int fa_plan_c(int C) { return fa_plan_clients > 0 ? fa_plan_clients : C; }
