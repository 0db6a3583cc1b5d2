// Counter-hash dropout shared by the bf16 and fp32 transformer kernels (and mirrored in
// ops/transformer_ops.py:dropout_keep): keep ⇔ fmix32(fmix32(a ^ seed) + b·φ) ≥ p·2³². Forward and
// backward regenerate the same mask from (seed, a, b), so no mask is ever stored.
#pragma once
#include <stdint.h>

namespace fa_drop {

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ bool keep(uint32_t seed, uint32_t a, uint32_t b, uint32_t thr) {
  return fmix32(fmix32(a ^ seed) + b * 0x9E3779B1u) >= thr;
}

}  // namespace fa_drop
