// Deterministic fp32 accumulation for the kernels that reduce with global atomics (BN statistics,
// split-K / pixel-chunked weight gradients).
//
// fp32 atomicAdd is order-dependent: the same step run twice can differ in the last bit, and a ReLU
// pre-activation sitting at the threshold then flips (tests/test_native_resnet_fp32_gpu.py). In
// deterministic mode (utils/determinism.py) every registered fp32 target gets a shadow of 128-bit
// two's-complement fixed-point accumulators (LSB 2^-80, range ±2^47; an addend of magnitude ≥ 2^46
// or a non-finite one poisons the run: the flush then writes NaN, which the engine's guards catch): each addend is converted
// exactly-or-truncated to fixed point (a pure function of the addend), and integer addition is
// associative, so the sum is the same bits whatever order the workgroups arrive in. A flush kernel
// (fa_det_flush) rounds each accumulator to fp32, adds it to the target and clears the shadow.
//
// The registry is a per-translation-unit __device__ table (kernels are built without RDC): every
// TU that accumulates includes this header and exports its setter with FA_DET_EXPORT(name);
// the host sets the same table in all of them (ops/det_ops.py). n == 0 (the default) keeps the
// plain fp32 atomics at the cost of one uniform load and branch per call site.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fa_det {
constexpr int MAXR = 16;
constexpr int FRAC = 80;   // fixed-point fraction bits
struct Table {
  int64_t n;                        // registered ranges (0: deterministic mode off)
  const float* lo[MAXR];            // fp32 target ranges [lo, lo + len)
  int64_t len[MAXR];
  unsigned long long* acc[MAXR];    // [len][2] accumulators (low word, high word)
  unsigned int* bad;                // set when a non-finite addend arrived (flush then writes NaN)
};

// false: not representable (non-finite, or |v| ≥ 2^46 where a few sums could wrap the range)
__device__ __forceinline__ bool to_fixed(float v, unsigned long long& lo, unsigned long long& hi) {
  const uint32_t b = __float_as_uint(v);
  const int ex = (int)((b >> 23) & 0xff);
  lo = 0ull;
  hi = 0ull;
  if (ex == 0) return true;                             // zero / subnormal (< 2^-126): below the LSB
  const unsigned long long man = (unsigned long long)((b & 0x7fffffu) | 0x800000u);
  const int sh = ex - 150 + FRAC;                       // value = man · 2^(ex - 150)
  if (ex == 255 || sh > 102) return false;
  if (sh <= -24) return true;
  if (sh < 0) {
    lo = man >> (-sh);
  } else if (sh < 64) {
    lo = man << sh;
    hi = sh > 40 ? (man >> (64 - sh)) : 0ull;
  } else {
    hi = man << (sh - 64);
  }
  if (b >> 31) {                                        // two's complement negate
    lo = ~lo + 1ull;
    hi = ~hi + (lo == 0ull ? 1ull : 0ull);
  }
  return true;
}

__device__ __forceinline__ void add_fixed(unsigned long long* a, float v, unsigned int* bad) {
  unsigned long long lo, hi;
  if (!to_fixed(v, lo, hi)) {
    atomicOr(bad, 1u);
    return;
  }
  if ((lo | hi) == 0ull) return;
  const unsigned long long old = atomicAdd(a, lo);
  const unsigned long long carry = (old + lo) < old ? 1ull : 0ull;
  if (hi + carry) atomicAdd(a + 1, hi + carry);
}
}  // namespace fa_det

// __constant__: kernels never write it, so its loads are invariant across the atomics they guard — one load per
// kernel instead of one load + wait per atomic call site (a __device__ table was reloaded after every atomic)
static __constant__ fa_det::Table g_fa_det;

// the deterministic branch: out of line (one copy per translation unit, not one per unrolled call site)
__device__ __attribute__((noinline)) static void fa_acc_add_det(float* p, float v) {
  unsigned long long* slot = nullptr;
  for (int r = 0; r < (int)g_fa_det.n; ++r) {
    const int64_t i = p - g_fa_det.lo[r];
    if (i >= 0 && i < g_fa_det.len[r]) {
      slot = g_fa_det.acc[r] + 2 * i;
      break;
    }
  }
  if (slot)
    fa_det::add_fixed(slot, v, g_fa_det.bad);
  else
    atomicAdd(p, v);   // unregistered target
}

// atomicAdd(p, v), or its deterministic fixed-point twin when p lies in a registered range
__device__ __forceinline__ void fa_acc_add(float* p, float v) {
  if (__builtin_expect(g_fa_det.n == 0, 1))
    atomicAdd(p, v);
  else
    fa_acc_add_det(p, v);
}

// per-TU setter: FA_DET_EXPORT(conv) → extern "C" int fa_det_set_conv(const fa_det::Table* host)
#define FA_DET_EXPORT(name)                                                                  \
  static fa_det::Table g_fa_det_host_##name;                                                 \
  extern "C" __attribute__((visibility("default"))) int fa_det_set_##name(const void* host) { \
    g_fa_det_host_##name = *reinterpret_cast<const fa_det::Table*>(host);                    \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fa_det), host, sizeof(fa_det::Table));        \
  }

// host: round a registered range's accumulators into fp32 (dst += Σ) and clear them (det_kernels.hip)
extern "C" int fa_det_flush(float* dst, void* acc, int64_t n, unsigned int* bad, hipStream_t stream);

// host helper for a TU that must flush between two of its own launches (e.g. a scratch that a second
// kernel scatters): flushes [p, p + n) if it lies in a registered range of that TU's table
static inline int fa_det_flush_if_registered(const fa_det::Table& t, float* p, int64_t n, hipStream_t stream) {
  for (int r = 0; r < t.n && r < fa_det::MAXR; ++r) {
    const int64_t i = p - t.lo[r];
    if (i >= 0 && i + n <= t.len[r]) return fa_det_flush(p, t.acc[r] + 2 * i, n, t.bad, stream);
  }
  return 0;
}
