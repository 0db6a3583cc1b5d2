// Finite-field kernels for secure aggregation (TurboAggregate / SecAgg).
//
// fa_mod_matmul: out[M,N] = (A[M,K] @ B[K,N]) mod p over int64 residues in [0,p), p < 2^31.
// Shapes in practice: A is a small Lagrange/Vandermonde coefficient matrix (M,K <= 64),
// B is K shares of a model-sized vector (N ~ 1e6..1e8) -> HBM-bound streaming over B.
// Each thread owns one column and up to MR rows, so every B element is read once per
// MR-row chunk; A lives in LDS. Products of residues are < 2^62, so one u64 multiply and a
// reduction per term is exact. p = 2^31-1 takes the shift-add Mersenne reduction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"

namespace {

constexpr int MR = 8;
constexpr uint64_t MERSENNE31 = 2147483647ull;

template <bool MERSENNE>
__device__ __forceinline__ uint64_t reduce(uint64_t x, uint64_t p) {
  if (MERSENNE) {
    x = (x & MERSENNE31) + (x >> 31);
    x = (x & MERSENNE31) + (x >> 31);
    return x >= MERSENNE31 ? x - MERSENNE31 : x;
  }
  return x % p;
}

template <bool MERSENNE>
__global__ __launch_bounds__(256) void mod_matmul_kernel(const int64_t* __restrict__ A, const int64_t* __restrict__ B,
                                                         int64_t* __restrict__ out, int M, int K, int64_t N,
                                                         uint64_t p) {
  extern __shared__ uint64_t sA[];  // [MR][K]
  const int m0 = blockIdx.y * MR;
  const int mr = min(MR, M - m0);
  for (int i = threadIdx.x; i < mr * K; i += blockDim.x) sA[i] = (uint64_t)A[(int64_t)(m0 + i / K) * K + i % K];
  __syncthreads();
  for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
    uint64_t acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[r] = 0;
    for (int k = 0; k < K; ++k) {
      const uint64_t b = (uint64_t)B[(int64_t)k * N + n];
#pragma unroll
      for (int r = 0; r < MR; ++r)
        if (r < mr) acc[r] = reduce<MERSENNE>(acc[r] + reduce<MERSENNE>(sA[r * K + k] * b, p), p);
    }
#pragma unroll
    for (int r = 0; r < MR; ++r)
      if (r < mr) out[(int64_t)(m0 + r) * N + n] = (int64_t)acc[r];
  }
}

// out[n] = (sum_c X[c,n]) mod p   (server-side sum of masked uploads)
template <bool MERSENNE>
__global__ __launch_bounds__(256) void mod_sum_kernel(const int64_t* __restrict__ X, int64_t* __restrict__ out,
                                                      int C, int64_t N, uint64_t p) {
  for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
    uint64_t acc = 0;
    for (int c = 0; c < C; ++c) acc = reduce<MERSENNE>(acc + (uint64_t)X[(int64_t)c * N + n], p);
    out[n] = (int64_t)acc;
  }
}

}  // namespace

FA_EXPORT int fa_mod_matmul(const int64_t* A, const int64_t* B, int64_t* out, int M, int K, int64_t N, int64_t p,
                            hipStream_t stream) {
  if (M <= 0 || K <= 0 || N <= 0) return 0;
  if (p <= 1 || p >= (1ll << 31) || K > 512) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)fa_grid(N, 256, 4096), (unsigned)((M + MR - 1) / MR));
  size_t lds = (size_t)MR * K * sizeof(uint64_t);
  if (p == (int64_t)MERSENNE31)
    hipLaunchKernelGGL(mod_matmul_kernel<true>, grid, dim3(256), lds, stream, A, B, out, M, K, N, (uint64_t)p);
  else
    hipLaunchKernelGGL(mod_matmul_kernel<false>, grid, dim3(256), lds, stream, A, B, out, M, K, N, (uint64_t)p);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_mod_sum(const int64_t* X, int64_t* out, int C, int64_t N, int64_t p, hipStream_t stream) {
  if (N <= 0) return 0;
  if (p <= 1 || p >= (1ll << 31) || C > (1 << 30)) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)fa_grid(N, 256, 4096));
  if (p == (int64_t)MERSENNE31)
    hipLaunchKernelGGL(mod_sum_kernel<true>, grid, dim3(256), 0, stream, X, out, C, N, (uint64_t)p);
  else
    hipLaunchKernelGGL(mod_sum_kernel<false>, grid, dim3(256), 0, stream, X, out, C, N, (uint64_t)p);
  return (int)hipGetLastError();
}
