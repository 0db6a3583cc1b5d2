// Flush of the deterministic fixed-point accumulators (detacc.h): dst[i] += round_f32(acc[i] · 2^-80),
// acc[i] = 0. The 128-bit sum goes through fp64 (hi · 2^64 + lo, then · 2^-80) and rounds once more to
// fp32 — a pure function of the integer sum, so the result is the same bits for any arrival order.
#include "common.h"
#include "detacc.h"
#include "bnlazy.h"

__global__ __launch_bounds__(256) void det_flush_kernel(float* __restrict__ dst, unsigned long long* __restrict__ acc,
                                                        int64_t n, const unsigned int* __restrict__ bad) {
  const bool poisoned = bad != nullptr && *bad != 0u;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const unsigned long long lo = acc[2 * i], hi = acc[2 * i + 1];
    if (poisoned) {
      dst[i] = __builtin_nanf("");
    } else if ((lo | hi) != 0ull) {
      const double d = (double)(long long)hi * 18446744073709551616.0 + (double)lo;
      dst[i] += (float)(d * 8.271806125530277e-25);   // 2^-80
    } else {
      continue;
    }
    acc[2 * i] = 0ull;
    acc[2 * i + 1] = 0ull;
  }
}

extern "C" int fa_det_flush(float* dst, void* acc, int64_t n, unsigned int* bad, hipStream_t stream) {
  if (n <= 0) return 0;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(det_flush_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, stream, dst,
                     (unsigned long long*)acc, n, bad);
  return (int)hipGetLastError();
}

extern "C" int fa_plan_clients = 0;

// deferred BatchNorm finalisation (bnlazy.h): descriptors for the next consumer launch (slot 0: the vectors the
// kernel reads as scale/shift or α/β/γ; slot 1: a second BN — the downsample branch of a block-output prologue)
static const void* g_lazy[2] = {nullptr, nullptr};
extern "C" int fa_set_lazy(const void* d0, const void* d1) {
  g_lazy[0] = d0;
  g_lazy[1] = d1;
  return 0;
}
extern "C" const BnLazy* fa_take_lazy(int slot) {
  const void* d = g_lazy[slot];
  g_lazy[slot] = nullptr;
  return reinterpret_cast<const BnLazy*>(d);
}
extern "C" int fa_set_plan_clients(int c) {
  fa_plan_clients = c > 0 ? c : 0;
  return 0;
}

FA_DET_EXPORT(det)
