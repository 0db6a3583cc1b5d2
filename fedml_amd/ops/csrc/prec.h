// Storage-precision policies of the native client-batched ResNet kernels (gfx950, wave64).
//
// The conv / BN kernels are written once against a policy P and instantiated twice:
//
//   P = prec::BF16  activations and packed weights bf16, v_mfma_f32_16x16x32_bf16
//                   (one MFMA per 8-element K fragment)
//   P = prec::F32   activations and packed weights fp32, v_mfma_f32_16x16x4_f32 — exact fp32
//                   products with fp32 accumulation (a k-ordered fmaf chain, no xf32 on gfx950);
//                   the reference trains in fp32 (simulation/single_process/fedavg/
//                   my_model_trainer_classification.py:18-93), so this is the reference-precision path.
//
// A "chunk" is one 16-byte vector (uint4): P::VEC elements (8 bf16 | 4 fp32); global staging and
// LDS tile stores move chunks. An MFMA "fragment" is 8 K-elements per lane for both policies:
//   row fragment  frag(p)             lane (g = lane>>4, r = lane&15) holds K = 8g + j, j = 0..7, read
//                                     from 8 consecutive elements (bf16: one ds_read_b128; fp32: two);
//   pixel fragment frag_tr(tile, ...) lane holds pixel ROWS row0 + 8g + j of one column of a natural
//                                     [pixel][ld] tile (the weight-gradient operands):
//                                     bf16: two ds_read_b64_tr_b16 (column 4·(lane&3) + transpose);
//                                     fp32: eight ds_read_b32 of column lane&15 — with ld ≡ 2 (mod 4)
//                                     dwords the two lane groups of each LDS cycle hit disjoint banks.
// Both operands of one product always use the same fragment kind, so the K order matches.
// mma(a, b, c): bf16 one 16x16x32 MFMA; fp32 eight 16x16x4 MFMAs (element j of every lane is the
// K = 4-slice j). The C/D layout is the same for both (col = lane&15, row = 4(lane>>4) + i).
#pragma once
#include "common.h"

namespace prec {

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short v4i16v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16v lds_v4i16v;
typedef float f32x8v __attribute__((ext_vector_type(8)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

struct BF16 {
  using T = uint16_t;
  static constexpr int VEC = 8;     // elements per 16-B chunk
  static constexpr int ES = 2;      // bytes per element
  static constexpr bool kF32 = false;
  using frag_t = bf16x8v;

  static __device__ __forceinline__ float to_f(T h) { return __uint_as_float(((uint32_t)h) << 16); }
  static __device__ __forceinline__ T from_f(float f) { return f32_to_bf16(f); }
  static __device__ __forceinline__ float round(float f) { return to_f(from_f(f)); }
  static __device__ __forceinline__ void unpack(uint4 v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
  }
  // one v_cvt_pk_bf16_f32 for the pair (the same RNE conversion as two scalar casts, which the compiler
  // emitted as two converts plus an OR)
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    const f32x2v v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
  }
  // 4 consecutive elements (one accumulator quad) ↔ fp32; store rounds, returns the stored values
  static __device__ __forceinline__ void load4(const T* p, float* f) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  }
  static __device__ __forceinline__ void store4(T* p, float* f) {
    const uint2 v = make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
    *reinterpret_cast<uint2*>(p) = v;
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  }
  static __device__ __forceinline__ frag_t frag(const T* p) {
    union { uint4 u; frag_t b; } c;
    c.u = *reinterpret_cast<const uint4*>(p);
    return c.b;
  }
  // pixel fragment: this lane's first pixel row / column offset, then the read at that address with
  // `step` elements between consecutive pixels
  static __device__ __forceinline__ int px_row(int lane) { return 8 * (lane >> 4) + ((lane & 15) >> 2); }
  static __device__ __forceinline__ int px_col(int lane) { return 4 * (lane & 3); }
  static __device__ __forceinline__ frag_t frag_px(const T* a0, int step) {
    const v4i16v r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16v*)(a0));
    const v4i16v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16v*)(a0 + 4 * step));
    union { short s[8]; frag_t b; } u;
    u.s[0] = r0[0]; u.s[1] = r0[1]; u.s[2] = r0[2]; u.s[3] = r0[3];
    u.s[4] = r1[0]; u.s[5] = r1[1]; u.s[6] = r1[2]; u.s[7] = r1[3];
    return u.b;
  }
  static __device__ __forceinline__ frag_t frag_tr(const T* tile, int ld, int row0, int col0, int lane) {
    return frag_px(tile + (row0 + px_row(lane)) * ld + col0 + px_col(lane), ld);
  }
  // one 16-B chunk into a frag_tr tile
  static __device__ __forceinline__ void st_chunk(T* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
  // row fragment from a frag_tr tile (pitch_tr: 8-B aligned rows for fp32)
  static __device__ __forceinline__ frag_t frag_a8(const T* p) { return frag(p); }
  // 8 consecutive elements ↔ fp32, and a fragment built from 8 fp32 values (rounded to storage)
  static __device__ __forceinline__ void load8(const T* p, float* f) { unpack(*reinterpret_cast<const uint4*>(p), f); }
  static __device__ __forceinline__ frag_t frag8(const float* f) {
    union { uint4 u; frag_t b; } c;
    c.u = pack(f);
    return c.b;
  }
  static __device__ __forceinline__ f32x4 mma(const frag_t& a, const frag_t& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  // row-tile staging pair (K-streamed kernels): chunk `col` (16 B, K offset col·VEC from an 8-element-aligned
  // row start) into the LDS tile, and the 8-element row fragment back out — identity layouts here
  static __device__ __forceinline__ void st_tile(T* p, int, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
  static __device__ __forceinline__ frag_t frag_tile(const T* p) { return frag(p); }
  // LDS row pitch (elements) of a [rows][ch] tile: 16-B aligned, bank-spread for the bf16 reads
  static constexpr int pitch(int ch) { return ch + 8; }
  // pitch of tiles read with frag_tr
  static constexpr int pitch_tr(int ch) { return ch + 8; }
};

struct F32 {
  using T = float;
  static constexpr int VEC = 4;
  static constexpr int ES = 4;
  static constexpr bool kF32 = true;
  using frag_t = f32x8v;

  static __device__ __forceinline__ float to_f(T h) { return h; }
  static __device__ __forceinline__ T from_f(float f) { return f; }
  static __device__ __forceinline__ float round(float f) { return f; }
  static __device__ __forceinline__ void unpack(uint4 v, float* f) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
  static __device__ __forceinline__ void load4(const T* p, float* f) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  static __device__ __forceinline__ void store4(T* p, float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
  static __device__ __forceinline__ frag_t frag(const T* p) {
    const float4 lo = *reinterpret_cast<const float4*>(p);
    const float4 hi = *reinterpret_cast<const float4*>(p + 4);
    return frag_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  }
  static __device__ __forceinline__ int px_row(int lane) { return 8 * (lane >> 4); }
  static __device__ __forceinline__ int px_col(int lane) { return lane & 15; }
  static __device__ __forceinline__ frag_t frag_px(const T* a, int step) {
    frag_t f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = a[j * step];
    return f;
  }
  static __device__ __forceinline__ frag_t frag_tr(const T* tile, int ld, int row0, int col0, int lane) {
    return frag_px(tile + (row0 + px_row(lane)) * ld + col0 + px_col(lane), ld);
  }
  static __device__ __forceinline__ frag_t frag_a8(const T* p) {
    const float2 a = reinterpret_cast<const float2*>(p)[0], b = reinterpret_cast<const float2*>(p)[1];
    const float2 c = reinterpret_cast<const float2*>(p)[2], d = reinterpret_cast<const float2*>(p)[3];
    return frag_t{a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
  }
  static __device__ __forceinline__ void load8(const T* p, float* f) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  static __device__ __forceinline__ frag_t frag8(const float* f) {
    return frag_t{f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]};
  }
  // frag_tr tiles have an 8-B-aligned pitch: chunks go in as two 8-B stores
  static __device__ __forceinline__ void st_chunk(T* p, uint4 v) {
    reinterpret_cast<uint2*>(p)[0] = make_uint2(v.x, v.y);
    reinterpret_cast<uint2*>(p)[1] = make_uint2(v.z, v.w);
  }
  static __device__ __forceinline__ f32x4 mma(const frag_t& a, const frag_t& b, f32x4 c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
    return c;
  }
  static __device__ __forceinline__ void st_tile(T* p, int, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
  static __device__ __forceinline__ frag_t frag_tile(const T* p) { return frag(p); }
  static constexpr int pitch(int ch) { return ch + 4; }
  // ≡ 2 (mod 4) dwords: rows 8 apart (lane groups g and g + 1 of one frag_px read) are 16 banks apart
  static constexpr int pitch_tr(int ch) { return ch + 2; }
};

// fp32 storage, products on the bf16 matrix cores as a three-term split (Ootomo & Yokota style):
//   a = a_hi + a_lo,  a_hi = bf16(a),  a_lo = bf16(a − a_hi)     (same for b)
//   a·b ≈ a_lo·b_hi + a_hi·b_lo + a_hi·b_hi                         (a_lo·b_lo, ~2⁻¹⁸ relative, dropped)
// Each product keeps ~16 significant bits (relative error ≲ 2⁻¹⁶ ≈ 1.5e-5 per product, fp32 accumulation):
// ~8 bits more than TF32 — what cuDNN uses for "fp32" convolutions by default (torch.backends.cudnn.allow_tf32)
// — and 3 v_mfma_f32_16x16x32_bf16 instead of 8 v_mfma_f32_16x16x4_f32 per 8-element fragment
// (≈ 5× the matrix throughput). Storage, epilogues, statistics and everything outside the MFMA stay fp32.
// The split is done once per fragment load, so operand reuse across the wave's tile amortises it.
struct F32X3 : F32 {
  struct frag_t {
    bf16x8v hi, lo;
  };
  static __device__ __forceinline__ frag_t split(const f32x8v& f) {
    frag_t s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const __bf16 h = (__bf16)f[j];
      s.hi[j] = h;
      s.lo[j] = (__bf16)(f[j] - (float)h);
    }
    return s;
  }
  static __device__ __forceinline__ frag_t frag(const T* p) { return split(F32::frag(p)); }
  static __device__ __forceinline__ frag_t frag_px(const T* a, int step) { return split(F32::frag_px(a, step)); }
  static __device__ __forceinline__ frag_t frag_tr(const T* tile, int ld, int row0, int col0, int lane) {
    return split(F32::frag_tr(tile, ld, row0, col0, lane));
  }
  static __device__ __forceinline__ frag_t frag_a8(const T* p) { return split(F32::frag_a8(p)); }
  static __device__ __forceinline__ frag_t frag8(const float* f) { return split(F32::frag8(f)); }
  // pre-split row tiles: each 8-element K group (32 B, two chunks) is stored as [hi 0-7 | lo 0-7] bf16, so
  // a fragment is two ds_read_b128 with no conversion; the split happens once per element at staging
  // instead of once per fragment use
  static __device__ __forceinline__ void st_tile(T* p, int col, uint4 v) {
    char* g = reinterpret_cast<char*>(p - 4 * (col & 1)) + 8 * (col & 1);
    const float f[4] = {__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
    uint16_t h[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const __bf16 b = (__bf16)f[j];
      h[j] = __builtin_bit_cast(uint16_t, b);
      l[j] = __builtin_bit_cast(uint16_t, (__bf16)(f[j] - (float)b));
    }
    *reinterpret_cast<uint2*>(g) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
    *reinterpret_cast<uint2*>(g + 16) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
  }
  static __device__ __forceinline__ frag_t frag_tile(const T* p) {
    frag_t s;
    s.hi = *reinterpret_cast<const bf16x8v*>(p);
    s.lo = *reinterpret_cast<const bf16x8v*>(reinterpret_cast<const char*>(p) + 16);
    return s;
  }
  static __device__ __forceinline__ f32x4 mma(const frag_t& a, const frag_t& b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, c, 0, 0, 0);
  }
};

// fp32 matrix-core mode of the `_f32` entry points: 0 = exact (F32), 1 = split bf16 (F32X3). One flag per
// process (inline function → a single COMDAT object across the kernel translation units).
inline int& f32_mma_mode() {
  static int mode = 0;
  return mode;
}

}  // namespace prec

// dispatch an `_f32` launcher body on the fp32 matrix-core mode: EXPR uses the policy name PX
#define FA_F32_DISPATCH(NS, EXPR)                   \
  do {                                              \
    if (prec::f32_mma_mode() == 1) {                \
      using PX = NS::F32X3;                         \
      return EXPR;                                  \
    }                                               \
    using PX = NS::F32;                             \
    return EXPR;                                    \
  } while (0)
