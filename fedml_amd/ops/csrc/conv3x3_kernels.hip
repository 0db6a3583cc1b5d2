// Spatially tiled 3×3 / stride-1 / pad-1 convolution kernels for the client-batched ResNet
// (gfx950, wave64, v_mfma_f32_16x16x32_bf16).
//
// Why a dedicated path: the generic implicit-GEMM kernels gather every A element per tap from
// global memory (9 × the input bytes through L2, an integer divide per K step, the BatchNorm
// operand transform re-applied 9 times) and reach only 5–15 % of HBM bandwidth on the 3×3 layers
// of ResNet-56 (16/32/64 channels at 32²/16²/8²). Here a workgroup stages whole images of one
// client ONCE into LDS — already transformed (relu(x·s+t) forward, α·g+β·y+γ backward), with a
// zero halo of one pixel — and all nine taps read the tile from LDS:
//
//   conv3x3_gemm_kernel  forward (out = conv(act(x)), epilogue BN statistics Σy, Σy²)  and
//                        backward-data (dx = convᵀ(dy), epilogue ReLU mask of the previous BN
//                        + its backward statistics Σg', Σg'·x)  — taps flipped via the halo index
//   conv3x3_wgrad_kernel dW[co][tap][ci] = Σ_p dy[p][co] · act(x)[p ⊕ tap][ci]; both operands are
//                        read pixel-major with gfx950's transposing LDS read ds_read_b64_tr_b16,
//                        the im2col shift is only an address offset into the haloed tile.
//
// LDS pixel stride = channels + 8 (bf16): 16-B-aligned for the vector staging writes and
// bank-spread for both the row reads (ds_read_b128) and the transposed reads.
#include "common.h"

#include <cstdlib>

#ifndef TAP_UNROLL
#define TAP_UNROLL 3
#endif

namespace c3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) {
  union { uint4 u; bf16x8 b; } c;
  c.u = v;
  return c.b;
}
__device__ __forceinline__ void unpack8(uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2(f[0], f[1]); r.y = pack2(f[2], f[3]); r.z = pack2(f[4], f[5]); r.w = pack2(f[6], f[7]);
  return r;
}

enum { XF_NONE = 0, XF_BNRELU = 1, XF_DY = 2 };
enum { EPI_FWD = 0, EPI_MASK = 2 };

// Exact n / d for 0 ≤ n < 2^26 by multiply-high (branch-free libdivide form; d ≥ 1): the tile
// index math runs per 16-B chunk and per 16-pixel MFMA tile, where a runtime integer divide
// (≈ 30 VALU instructions) used to cost more issue slots than the MFMAs it fed.
struct FastDiv {
  uint32_t m, s;
};
static inline FastDiv make_fdiv(uint32_t d) {
  uint32_t sh = 0;
  while ((1u << sh) < d) ++sh;
  const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << sh) - d)) / d + 1;
  return FastDiv{(uint32_t)m, sh};
}
__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return (int)((__umulhi((uint32_t)n, f.m) + (uint32_t)n) >> f.s);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Operand transform of one 16-B chunk (8 channels from ch0) with the per-channel vectors in LDS,
// two channels per packed-fp32 instruction.
template <int XF>
struct ChunkVec {
  const float *v0, *v1, *v2;
  int ch0;
  __device__ __forceinline__ void load(const float* a, const float* b, const float* c, int ch) {
    v0 = a; v1 = b; v2 = c; ch0 = ch;
  }
  // XF_BNRELU: relu(x·s + t);  XF_DY: α·g + β·y + γ
  __device__ __forceinline__ uint4 apply(uint4 v, uint4 w) const {
    if (XF == XF_NONE) return v;
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
    const f32x2* A = reinterpret_cast<const f32x2*>(v0 + ch0);
    const f32x2* B = reinterpret_cast<const f32x2*>(v1 + ch0);
    const f32x2* Cv = reinterpret_cast<const f32x2*>(v2 + ch0);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2 x = f32x2{__uint_as_float(vv[j] << 16), __uint_as_float(vv[j] & 0xffff0000u)};
      f32x2 r;
      if (XF == XF_BNRELU) {
        r = x * A[j] + B[j];
        r.x = fmaxf(r.x, 0.f);
        r.y = fmaxf(r.y, 0.f);
      } else {
        const f32x2 y = f32x2{__uint_as_float(ww[j] << 16), __uint_as_float(ww[j] & 0xffff0000u)};
        r = x * A[j] + (y * B[j] + Cv[j]);
      }
      o[j] = pack2(r.x, r.y);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
  }
};

// Stage one work unit of a client into an LDS tile [ns][TR][TW][KC+8] with the operand transform
// applied. Tile row tr / column tc hold source pixel (t0 + tr, tc − 1); outside the source image
// the tile is zero (the convolution's zero padding). UPS: the source is read zero-upsampled by 2
// (stride-2 backward-data: dy sits at the even positions of the dx grid). `src`/`src2` already
// point at the client. `cv` holds the transform vectors of channel chunk threadIdx.x % (KC/8).
template <int KC, int XF, int UPS>
__device__ __forceinline__ void stage_tile(uint16_t* tile, const uint16_t* __restrict__ src,
                                           const uint16_t* __restrict__ src2, const ChunkVec<XF>& cv, int img0,
                                           int ns, int t0, int TR, int TW, FastDiv fd_trtw, FastDiv fd_tw, int Hs,
                                           int Ws) {
  constexpr int LD = KC + 8;
  constexpr int CG = KC / 8;
  static_assert(256 % CG == 0, "fixed chunk per thread");
  const int TRTW = TR * TW;
  const int total = ns * TRTW * CG;
  const int cg = threadIdx.x % CG;
  for (int i = threadIdx.x; i < total; i += 256) {
    const int pix = i / CG;
    const int im = fdiv(pix, fd_trtw);
    const int r = pix - im * TRTW;
    const int tr = fdiv(r, fd_tw);
    int t = t0 + tr, u = r - tr * TW - 1;
    bool ok;
    if (UPS) {
      ok = t >= 0 && u >= 0 && !(t & 1) && !(u & 1);
      t >>= 1;
      u >>= 1;
      ok = ok && t < Hs && u < Ws;
    } else {
      ok = t >= 0 && t < Hs && u >= 0 && u < Ws;
    }
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ok) {
      const int64_t off = ((((int64_t)(img0 + im) * Hs) + t) * Ws + u) * KC + cg * 8;
      const uint4 raw = *reinterpret_cast<const uint4*>(src + off);
      uint4 raw2 = make_uint4(0, 0, 0, 0);
      if (XF == XF_DY) raw2 = *reinterpret_cast<const uint4*>(src2 + off);
      v = cv.apply(raw, raw2);
    }
    *reinterpret_cast<uint4*>(tile + (int64_t)pix * LD + cg * 8) = v;
  }
}

// Register-prefetching form of stage_tile: load() issues every global read of a unit (≤ MAXC
// 16-B chunks per thread, checked on the host) into registers, store() transforms and writes the
// tile. The unit loops call load() for unit u+1 right after the tile of unit u is in LDS, so the
// HBM latency of the next unit overlaps this unit's MFMA work instead of being paid serially.
template <int KC, int XF, int UPS, int MAXC>
struct TileLoader {
  static constexpr int CG = KC / 8;
  uint4 r1[MAXC], r2[XF == XF_DY ? MAXC : 1];
  uint32_t okm;
  int total;
  __device__ __forceinline__ void load(const uint16_t* __restrict__ src, const uint16_t* __restrict__ src2, int img0,
                                       int ns, int t0, int TR, int TW, FastDiv fd_trtw, FastDiv fd_tw, int Hs,
                                       int Ws) {
    const int TRTW = TR * TW;
    total = ns * TRTW * CG;
    const int cg = threadIdx.x % CG;
    okm = 0;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int i = threadIdx.x + j * 256;
      const int pix = i / CG;
      const int im = fdiv(pix, fd_trtw);
      const int r = pix - im * TRTW;
      const int tr = fdiv(r, fd_tw);
      int t = t0 + tr, u = r - tr * TW - 1;
      bool ok;
      if (UPS) {
        ok = t >= 0 && u >= 0 && !(t & 1) && !(u & 1);
        t >>= 1;
        u >>= 1;
        ok = ok && t < Hs && u < Ws;
      } else {
        ok = t >= 0 && t < Hs && u >= 0 && u < Ws;
      }
      ok = ok && i < total;
      r1[j] = make_uint4(0, 0, 0, 0);
      if (XF == XF_DY) r2[j] = make_uint4(0, 0, 0, 0);
      if (ok) {
        const int64_t off = ((((int64_t)(img0 + im) * Hs) + t) * Ws + u) * KC + cg * 8;
        r1[j] = *reinterpret_cast<const uint4*>(src + off);
        if (XF == XF_DY) r2[j] = *reinterpret_cast<const uint4*>(src2 + off);
        okm |= 1u << j;
      }
    }
  }
  __device__ __forceinline__ void store(uint16_t* tile, const ChunkVec<XF>& cv) const {
    constexpr int LD = KC + 8;
    const int cg = threadIdx.x % CG;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int i = threadIdx.x + j * 256;
      if (i < total) {
        const uint4 v = (okm >> j) & 1u ? cv.apply(r1[j], XF == XF_DY ? r2[j] : r1[j]) : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(tile + (int64_t)(i / CG) * LD + cg * 8) = v;
      }
    }
  }
};

// dy = α·g + β·y + γ staged pixel-major without halo (weight gradient), prefetched the same way.
template <int COUT, int MAXD>
struct DyLoader {
  static constexpr int CGD = COUT / 8;
  uint4 rg[MAXD], ry[MAXD];
  int total;
  __device__ __forceinline__ void load(const uint16_t* __restrict__ gc, const uint16_t* __restrict__ yc, int64_t pix0,
                                       int npix) {
    total = npix * CGD;
    const int cg = threadIdx.x % CGD;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      const int i = threadIdx.x + j * 256;
      rg[j] = ry[j] = make_uint4(0, 0, 0, 0);
      if (i < total) {
        const int64_t off = (pix0 + i / CGD) * COUT + cg * 8;
        rg[j] = *reinterpret_cast<const uint4*>(gc + off);
        ry[j] = *reinterpret_cast<const uint4*>(yc + off);
      }
    }
  }
  __device__ __forceinline__ void store(uint16_t* dyL, const ChunkVec<XF_DY>& dv) const {
    constexpr int LDD = COUT + 8;
    const int cg = threadIdx.x % CGD;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      const int i = threadIdx.x + j * 256;
      if (i < total) *reinterpret_cast<uint4*>(dyL + (size_t)(i / CGD) * LDD + cg * 8) = dv.apply(rg[j], ry[j]);
    }
  }
};

// Work unit u of a client: S > 1 → images [u·S, u·S + S) whole; S == 1 → image u / (H/R),
// output rows [(u mod H/R)·R, +R).
__device__ __forceinline__ void unit_geom(int u, int N, int H, int R, int S, int& img0, int& ns, int& r0) {
  if (S > 1) {
    img0 = u * S;
    ns = min(S, N - img0);
    r0 = 0;
  } else {
    const int rb = H / R;
    img0 = u / rb;
    ns = 1;
    r0 = (u % rb) * R;
  }
}

struct Args {
  const uint16_t* src;   // x (forward) or g (backward-data)        [C][N][H][W][KC]
  const uint16_t* src2;  // y for XF_DY
  const uint16_t* wpk;   // packed weights [C][NOUT][ldk], k = tap·KC + kc
  int64_t wpk_ld;
  const float* vec0;     // scale | α
  const float* vec1;     // shift | β
  const float* vec2;     //       | γ
  uint16_t* out;         // [C][N][H][W][NOUT]
  const uint16_t* e_x;   // EPI_MASK: previous raw activation [C][N][H][W][NOUT]
  const float* e_s;
  const float* e_t;
  float* stats;          // [C][NOUT][NS]
  int NS;
  int N, H, W;                    // output (iteration) geometry
  int Hs, Ws;                     // A-operand source geometry (≠ H, W for stride 2)
  int ldk;
  int R, S, units, units_per_wg;  // stage geometry (see unit_geom) and work split
  int nout_total;                 // output channels of the layer (a workgroup computes NOUT of them)
  FastDiv fd_trtw, fd_tw, fd_rw, fd_w;  // ÷ TR·TW, ÷ TW (tile), ÷ R·W, ÷ W (output unit)
};

// MTW 16-pixel tiles per wave share every B fragment read.
// ST = stride: forward stride 2 reads the input at (2·p + tap); backward-data stride 2 reads a
// zero-upsampled dy tile at the dx resolution (then it is a stride-1 correlation).
//
// The MFMA computes the TRANSPOSED tile D[channel][pixel] (weights as the A operand, the haloed
// activation tile as B): each lane then owns 4 consecutive channels of one pixel, so the epilogue
// works straight from the accumulators — one 8-B store per lane, per-lane BN vectors and
// statistics in registers — with no LDS staging pass. A-operand reads are unconditional: rows past
// the unit read pixel 0 (discarded in the epilogue) and K-steps past 9·KC read tap 0 against the
// zero K-padding of the packed weights.
template <int KC, int NOUT, int XF, int BWD, int EPI, int MTW, int ST, int MAXC>
__global__ __launch_bounds__(256) void conv3x3_gemm_kernel(Args a) {
  constexpr int NT = NOUT / 16;
  constexpr int LD = KC + 8;
  constexpr int K = 9 * KC;
  constexpr int KSTEPS = (K + 31) / 32;
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int H = a.H, W = a.W, HW = H * W;
  const int Hs = a.Hs, Ws = a.Ws;
  constexpr int SP = (!BWD && ST == 2) ? 2 : 1;   // source-pixel step per output pixel
  constexpr bool UPS = BWD && ST == 2;
  const int TW = (UPS ? W : Ws) + 2;             // tile width incl. halo

  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* wl = reinterpret_cast<uint16_t*>(smem);                        // [NOUT][ldk]
  float* v0 = reinterpret_cast<float*>(smem + (size_t)NOUT * a.ldk * 2);   // [KC] ×3
  float* v1 = v0 + KC;
  float* v2 = v1 + KC;
  float* red = v2 + KC;                                                     // [4][NOUT][2]
  float* esL = red + 4 * NOUT * 2;                                          // [NOUT] ×2 (EPI_MASK)
  float* etL = esL + NOUT;
  uint16_t* tile = reinterpret_cast<uint16_t*>(etL + NOUT);                // [S][TR][TW][LD]

  const int ch_base = blockIdx.z * NOUT;  // output-channel slice of this workgroup
  const int NO = a.nout_total;
  {
    const uint4* s = reinterpret_cast<const uint4*>(a.wpk + (int64_t)c * a.wpk_ld + (int64_t)ch_base * a.ldk);
    uint4* d = reinterpret_cast<uint4*>(wl);
    const int n16 = NOUT * a.ldk / 8;
    for (int i = threadIdx.x; i < n16; i += 256) d[i] = s[i];
    if (XF != XF_NONE)
      for (int i = threadIdx.x; i < KC; i += 256) {
        v0[i] = a.vec0[(int64_t)c * KC + i];
        v1[i] = a.vec1[(int64_t)c * KC + i];
        if (XF == XF_DY) v2[i] = a.vec2[(int64_t)c * KC + i];
      }
    if (EPI == EPI_MASK)
      for (int i = threadIdx.x; i < NOUT; i += 256) {
        esL[i] = a.e_s[(int64_t)c * NO + ch_base + i];
        etL[i] = a.e_t[(int64_t)c * NO + ch_base + i];
      }
  }
  __syncthreads();
  ChunkVec<XF> cvec;
  cvec.load(v0, v1, v2, (threadIdx.x % (KC / 8)) * 8);

  const uint16_t* src = a.src + (int64_t)c * a.N * Hs * Ws * KC;
  const uint16_t* src2 = (XF == XF_DY) ? a.src2 + (int64_t)c * a.N * Hs * Ws * KC : nullptr;
  uint16_t* out = a.out + (int64_t)c * a.N * HW * NO;
  const uint16_t* ex = (EPI == EPI_MASK) ? a.e_x + (int64_t)c * a.N * HW * NO : nullptr;

  // per-lane epilogue state: channels ch_base + nt·16 + 4g + i
  float st0[NT][4], st1[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st0[nt][i] = 0.f;
      st1[nt][i] = 0.f;
    }

  // loop-invariant A-operand tap offsets of this lane (one per K-step)
  int toff[KC >= 32 ? 1 : KSTEPS];
#pragma unroll
  for (int ks = 0; ks < (KC >= 32 ? 0 : KSTEPS); ++ks) {
    const int k = ks * 32 + 8 * g;
    const int tap = k / KC, ci = k % KC;
    const int kh = tap / 3, kw = tap % 3;
    // forward reads x_pad(pr + kh, pc + kw); backward reads dy_pad(pr + 2 − kh, pc + 2 − kw)
    const int o = BWD ? ((2 - kh) * TW + (2 - kw)) * LD + ci : (kh * TW + kw) * LD + ci;
    toff[ks] = k < K ? o : 0;
  }
  const uint16_t* wrow = wl + (lane & 15) * a.ldk + 8 * g;

  const int R = a.R, RW = R * W;
  const int TR = SP == 2 ? 2 * R + 1 : R + 2;    // tile rows incl. halo
  const int u_lo = blockIdx.x * a.units_per_wg;
  const int u_hi = min(a.units, u_lo + a.units_per_wg);
  TileLoader<KC, XF, UPS, MAXC> ld;
  if (u_lo < u_hi) {
    int img0, ns, r0;
    unit_geom(u_lo, a.N, H, R, a.S, img0, ns, r0);
    ld.load(src, src2, img0, ns, SP * r0 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
  }
  for (int u = u_lo; u < u_hi; ++u) {
    int img0, ns, r0;
    unit_geom(u, a.N, H, R, a.S, img0, ns, r0);
    const int64_t pix0 = (int64_t)img0 * HW + (int64_t)r0 * W;  // first output pixel of the unit
    __syncthreads();  // previous unit fully consumed
    ld.store(tile, cvec);
    __syncthreads();
    if (u + 1 < u_hi) {  // next unit's global reads in flight during this unit's MFMAs
      int img1, ns1, r1;
      unit_geom(u + 1, a.N, H, R, a.S, img1, ns1, r1);
      ld.load(src, src2, img1, ns1, SP * r1 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
    }
    const int P = ns * RW;
    const int ntile = (P + 15) / 16;
    for (int t0 = wid * MTW; t0 < ntile; t0 += 4 * MTW) {
      int base[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        const int p = (t0 + mt) * 16 + (lane & 15);
        const int pp = p < P ? p : 0;
        const int im = fdiv(pp, a.fd_rw);
        const int r = pp - im * RW;
        const int rr = fdiv(r, a.fd_w);
        base[mt] = ((im * TR + SP * rr) * TW + SP * (r - rr * W)) * LD;
      }
      f32x4 acc[MTW][NT];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (KC >= 32) {
        // one tap per group of KC/32 K-steps: the tap offset is wave-uniform (scalar ALU)
#pragma unroll TAP_UNROLL
        for (int tap = 0; tap < 9; ++tap) {
          const int kh = tap / 3, kw = tap - 3 * (tap / 3);
          const int tapoff = (BWD ? ((2 - kh) * TW + (2 - kw)) : (kh * TW + kw)) * LD + 8 * g;
#pragma unroll
          for (int cc = 0; cc < KC / 32; ++cc) {
            bf16x8 af[MTW];
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
              af[mt] = *reinterpret_cast<const bf16x8*>(tile + base[mt] + tapoff + cc * 32);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              const bf16x8 bw =
                  *reinterpret_cast<const bf16x8*>(wrow + nt * 16 * a.ldk + (tap * (KC / 32) + cc) * 32);
#pragma unroll
              for (int mt = 0; mt < MTW; ++mt)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw, af[mt], acc[mt][nt], 0, 0, 0);
            }
          }
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
          bf16x8 af[MTW];
#pragma unroll
          for (int mt = 0; mt < MTW; ++mt) af[mt] = *reinterpret_cast<const bf16x8*>(tile + base[mt] + toff[ks]);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const bf16x8 bw = *reinterpret_cast<const bf16x8*>(wrow + nt * 16 * a.ldk + ks * 32);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw, af[mt], acc[mt][nt], 0, 0, 0);
          }
        }
      }
      // ---- epilogue from the accumulators: lane = (pixel lane&15, channels 4g..4g+3 of each nt) ----
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        const int p = (t0 + mt) * 16 + (lane & 15);
        if (p >= P) continue;
        const int64_t prow = (pix0 + p) * NO + ch_base + 4 * g;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          uint2 pk = make_uint2(pack2(acc[mt][nt][0], acc[mt][nt][1]), pack2(acc[mt][nt][2], acc[mt][nt][3]));
          float f[4] = {__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                        __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
          if (EPI == EPI_FWD) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { st0[nt][i] += f[i]; st1[nt][i] += f[i] * f[i]; }
          } else {
            const uint2 xr = *reinterpret_cast<const uint2*>(ex + prow + nt * 16);
            const float xv[4] = {__uint_as_float(xr.x << 16), __uint_as_float(xr.x & 0xffff0000u),
                                 __uint_as_float(xr.y << 16), __uint_as_float(xr.y & 0xffff0000u)};
            const float4 es = *reinterpret_cast<const float4*>(esL + nt * 16 + 4 * g);
            const float4 et = *reinterpret_cast<const float4*>(etL + nt * 16 + 4 * g);
            f[0] = (xv[0] * es.x + et.x > 0.f) ? f[0] : 0.f;
            f[1] = (xv[1] * es.y + et.y > 0.f) ? f[1] : 0.f;
            f[2] = (xv[2] * es.z + et.z > 0.f) ? f[2] : 0.f;
            f[3] = (xv[3] * es.w + et.w > 0.f) ? f[3] : 0.f;
            pk = make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));  // masking keeps values exact
#pragma unroll
            for (int i = 0; i < 4; ++i) { st0[nt][i] += f[i]; st1[nt][i] += f[i] * xv[i]; }
          }
          *reinterpret_cast<uint2*>(out + prow + nt * 16) = pk;
        }
      }
    }
  }

  // ---- statistics: the 16 lanes of a channel quad (xor 1..8) → waves (LDS) → one atomic each ----
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st0[nt][i] += __shfl_xor(st0[nt][i], o, 64);
        st1[nt][i] += __shfl_xor(st1[nt][i], o, 64);
      }
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[(wid * NOUT + nt * 16 + 4 * g + i) * 2 + 0] = st0[nt][i];
        red[(wid * NOUT + nt * 16 + 4 * g + i) * 2 + 1] = st1[nt][i];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NOUT * 2; i += 256) {
    const int ch = i / 2, q = i % 2;
    const float s = red[(0 * NOUT + ch) * 2 + q] + red[(1 * NOUT + ch) * 2 + q] + red[(2 * NOUT + ch) * 2 + q] +
                    red[(3 * NOUT + ch) * 2 + q];
    atomicAdd(&a.stats[((int64_t)c * NO + ch_base + ch) * a.NS + q], s);
  }
}

// ---------------------------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------------------------
// 8 consecutive pixels × 16 columns, transposed read from a natural [pixel][ld] LDS tile: lane
// (g, i = q·4 + p) addresses pixel row0 + 8g + q, columns col0 + 4p (and pixel + 4).
__device__ __forceinline__ bf16x8 tr_read(const uint16_t* a0, int ld4) {
  const v4i16 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  const v4i16 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0 + ld4));
  union { short s[8]; bf16x8 b; } u;
  u.s[0] = r0[0]; u.s[1] = r0[1]; u.s[2] = r0[2]; u.s[3] = r0[3];
  u.s[4] = r1[0]; u.s[5] = r1[1]; u.s[6] = r1[2]; u.s[7] = r1[3];
  return u.b;
}

struct WArgs {
  const uint16_t* g;      // [C][N][H][W][COUT]
  const uint16_t* yv;
  const float* alpha;
  const float* beta;
  const float* gamma;
  const uint16_t* x;      // [C][N][H][W][CIN]
  const float* ps;
  const float* pt;
  float* dw;              // GEMM-layout scratch [C][COUT][9·CIN]
  int N, H, W;            // dy (output) geometry
  int Hs, Ws;             // x (input) geometry
  int R, S, units, units_per_wg;
  int nt_per_z;           // GEMM column tiles (16 wide) per blockIdx.z
  FastDiv fd_trtw, fd_tw, fd_rw, fd_w;
};

// WN waves split the column tiles of this z-slice, WK = 4/WN waves split the pixel K-steps.
template <int CIN, int COUT, int PRO, int WN, int TPW, int ST, int MAXC, int MAXD>
__global__ __launch_bounds__(256) void conv3x3_wgrad_kernel(WArgs a) {
  constexpr int WK = 4 / WN;
  constexpr int MT = COUT / 16;
  constexpr int LDX = CIN + 8, LDD = COUT + 8;
  constexpr int K = 9 * CIN;
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int kgrp = wid / WN, ngrp = wid % WN;
  const int H = a.H, W = a.W, HW = H * W;
  const int Hs = a.Hs, Ws = a.Ws, TW = Ws + 2;
  const int nt_lo = blockIdx.z * a.nt_per_z;
  const int nt_hi = min(K / 16, nt_lo + a.nt_per_z);
  const int my_nt0 = nt_lo + ngrp * TPW;  // this wave's column tiles [my_nt0, my_nt0 + TPW) ∩ [.., nt_hi)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* vv = reinterpret_cast<float*>(smem);                          // α β γ [COUT], s t [CIN]
  uint16_t* dyL = reinterpret_cast<uint16_t*>(vv + 3 * COUT + 2 * CIN);  // [S·HW][LDD]
  uint16_t* xt = dyL + (size_t)a.S * a.R * W * LDD;                    // [S][TR][TW][LDX]

  for (int i = threadIdx.x; i < COUT; i += 256) {
    vv[i] = a.alpha[(int64_t)c * COUT + i];
    vv[COUT + i] = a.beta[(int64_t)c * COUT + i];
    vv[2 * COUT + i] = a.gamma[(int64_t)c * COUT + i];
  }
  if (PRO)
    for (int i = threadIdx.x; i < CIN; i += 256) {
      vv[3 * COUT + i] = a.ps[(int64_t)c * CIN + i];
      vv[3 * COUT + CIN + i] = a.pt[(int64_t)c * CIN + i];
    }

  f32x4 acc[MT][TPW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[m][t] = {0.f, 0.f, 0.f, 0.f};

  const uint16_t* gc = a.g + (int64_t)c * a.N * HW * COUT;
  const uint16_t* yc = a.yv + (int64_t)c * a.N * HW * COUT;
  const uint16_t* xc = a.x + (int64_t)c * a.N * Hs * Ws * CIN;
  const int R = a.R, RW = R * W;
  const int TR = ST == 2 ? 2 * R + 1 : R + 2;
  const int u_lo = blockIdx.x * a.units_per_wg;
  const int u_hi = min(a.units, u_lo + a.units_per_wg);

  constexpr int CGD = COUT / 8;
  static_assert(256 % CGD == 0, "fixed chunk per thread");
  __syncthreads();  // vectors
  ChunkVec<XF_DY> dvec;
  dvec.load(vv, vv + COUT, vv + 2 * COUT, (threadIdx.x % CGD) * 8);
  ChunkVec<PRO ? XF_BNRELU : XF_NONE> xvec;
  xvec.load(vv + 3 * COUT, vv + 3 * COUT + CIN, nullptr, (threadIdx.x % (CIN / 8)) * 8);
  TileLoader<CIN, PRO ? XF_BNRELU : XF_NONE, 0, MAXC> xld;
  DyLoader<COUT, MAXD> dld;
  if (u_lo < u_hi) {
    int img0, ns, r0;
    unit_geom(u_lo, a.N, H, R, a.S, img0, ns, r0);
    dld.load(gc, yc, (int64_t)img0 * HW + (int64_t)r0 * W, ns * RW);
    xld.load(xc, nullptr, img0, ns, ST * r0 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
  }
  for (int u = u_lo; u < u_hi; ++u) {
    int img0, ns, r0;
    unit_geom(u, a.N, H, R, a.S, img0, ns, r0);
    __syncthreads();
    dld.store(dyL, dvec);  // dy = α·g + β·y + γ, natural [pixel][co] (no halo)
    xld.store(xt, xvec);
    __syncthreads();
    if (u + 1 < u_hi) {
      int img1, ns1, r1;
      unit_geom(u + 1, a.N, H, R, a.S, img1, ns1, r1);
      dld.load(gc, yc, (int64_t)img1 * HW + (int64_t)r1 * W, ns1 * RW);
      xld.load(xc, nullptr, img1, ns1, ST * r1 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
    }
    const int KS = ns * RW / 32;  // R·W is a multiple of 32
    for (int ks = kgrp; ks < KS; ks += WK) {
      const int p0 = ks * 32;
      // this lane's pixel row of the fragment (8-pixel groups never straddle an image row: W % 8 == 0)
      const int pix = p0 + 8 * g + q;
      const int im = fdiv(pix, a.fd_rw);
      const int r = pix - im * RW;
      const int rr = fdiv(r, a.fd_w);
      const uint16_t* xrow = xt + (size_t)((im * TR + ST * rr) * TW + ST * (r - rr * W)) * LDX + 4 * pq;
      const uint16_t* drow = dyL + (size_t)pix * LDD + 4 * pq;
      bf16x8 af[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) af[m] = tr_read(drow + m * 16, 4 * LDD);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int nt = my_nt0 + t;
        if (nt < nt_hi) {
          const int k0 = nt * 16;
          const int tap = k0 / CIN, ci0 = k0 % CIN;
          const int kh = tap / 3, kw = tap % 3;
          const bf16x8 bf = tr_read(xrow + (kh * TW + kw) * LDX + ci0, 4 * ST * LDX);
#pragma unroll
          for (int m = 0; m < MT; ++m)
            acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bf, acc[m][t], 0, 0, 0);
        }
      }
    }
  }

  // ---- reduce the WK pixel groups through LDS, then contiguous fp32 atomics (GEMM layout) ----
  float* dwc = a.dw + (int64_t)c * COUT * K;
  if (WK > 1) {
    __syncthreads();
    float* rbuf = reinterpret_cast<float*>(dyL);  // [WK-1][WN][MT][TPW][4][64]
    if (kgrp > 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            rbuf[((((kgrp - 1) * WN + ngrp) * MT + m) * TPW + t) * 256 + i * 64 + lane] = acc[m][t][i];
    }
    __syncthreads();
    if (kgrp == 0) {
      for (int kg2 = 1; kg2 < WK; ++kg2)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[m][t][i] += rbuf[((((kg2 - 1) * WN + ngrp) * MT + m) * TPW + t) * 256 + i * 64 + lane];
    }
  }
  if (kgrp == 0) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int nt = my_nt0 + t;
      if (nt < nt_hi) {
        const int k = nt * 16 + (lane & 15);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(&dwc[(int64_t)(m * 16 + 4 * g + i) * K + k], acc[m][t][i]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct Plan {
  int R, S, units, units_per_wg, gx;
};

// Stage ≈ `target_px` output pixels: whole images when they are small (S images), otherwise a
// block of R rows of one image (R·W a multiple of 32). ~`target_wgs` workgroups in total, each
// looping over a contiguous run of units (amortises the weight staging).
static Plan make_plan(int N, int H, int W, int C, int target_px, int target_wgs) {
  Plan p;
  const int hw = H * W;
  if (hw <= target_px) {
    p.R = H;
    p.S = max(1, min(N, target_px / hw));
    p.units = (N + p.S - 1) / p.S;
  } else {
    p.S = 1;
    p.R = 1;
    for (int r = H; r >= 1; --r)
      if (H % r == 0 && r * W <= target_px && (r * W) % 32 == 0) { p.R = r; break; }
    p.units = N * (H / p.R);
  }
  const int wpc = max(1, (target_wgs + C - 1) / C);
  p.units_per_wg = max(1, (p.units + wpc - 1) / wpc);
  p.gx = (p.units + p.units_per_wg - 1) / p.units_per_wg;
  return p;
}

static size_t gemm_smem(int kc, int nout, int ldk, const Plan& p, int TR, int TW) {
  return (size_t)nout * ldk * 2 + (size_t)3 * kc * 4 + (size_t)4 * nout * 2 * 4 + (size_t)2 * nout * 4 +
         (size_t)p.S * TR * TW * (kc + 8) * 2;
}

// NOUT_WG output channels per workgroup (blockIdx.z slices the layer's NOUT)
template <int KC, int NOUT_WG, int XF, int BWD, int EPI, int ST>
static int launch_gemm(Args a, int nout, int C, int target_px, hipStream_t stream) {
  constexpr int MTW = NOUT_WG >= 64 ? 2 : 4;
  static const int wgs = [] {   // FEDML_AMD_C3G_WGS: workgroup target of the fwd / bwd-data kernels
    const char* e = getenv("FEDML_AMD_C3G_WGS");
    return e ? atoi(e) : 2048;
  }();
  Plan p = make_plan(a.N, a.H, a.W, C, target_px, wgs);
  {  // a unit's tile must fit the loader's register budget (≤ 12 16-B chunks per thread)
    const bool f2 = !BWD && ST == 2;
    while (target_px > 8) {
      const int tr = f2 ? 2 * p.R + 1 : p.R + 2, tw = (BWD ? a.W : a.Ws) + 2;
      if ((p.S * tr * tw * (KC / 8) + 255) / 256 <= 12) break;
      target_px /= 2;
      p = make_plan(a.N, a.H, a.W, C, target_px, wgs);
    }
  }
  a.R = p.R; a.S = p.S; a.units = p.units; a.units_per_wg = p.units_per_wg; a.nout_total = nout;
  const bool fwd2 = !BWD && ST == 2;
  const int TR = fwd2 ? 2 * p.R + 1 : p.R + 2;
  const int TW = (BWD ? a.W : a.Ws) + 2;
  const size_t smem = gemm_smem(KC, NOUT_WG, a.ldk, p, TR, TW);
  if (smem > 160 * 1024) return -5;
  a.fd_trtw = make_fdiv(TR * TW); a.fd_tw = make_fdiv(TW); a.fd_rw = make_fdiv(p.R * a.W); a.fd_w = make_fdiv(a.W);
  const int need = (p.S * TR * TW * (KC / 8) + 255) / 256;  // 16-B chunks per thread per unit
  auto kern = need <= 2 ? conv3x3_gemm_kernel<KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 2>
            : need <= 4 ? conv3x3_gemm_kernel<KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 4>
            : need <= 8 ? conv3x3_gemm_kernel<KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 8>
                        : conv3x3_gemm_kernel<KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 12>;
  if (need > 12) return -7;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(p.gx, C, nout / NOUT_WG), dim3(256), smem, stream, a);
  return (int)hipGetLastError();
}

// tuning override of the unit size (output pixels per LDS tile): FEDML_AMD_C3_PX
static int px_override() {
  static const int v = [] {
    const char* e = getenv("FEDML_AMD_C3_PX");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <int XF, int BWD, int EPI, int ST>
static int dispatch_gemm(int kc, int nout, const Args& a, int C, hipStream_t s) {
  if (kc != nout) return -2;
  if (px_override() > 0) {
    const int o = px_override();
    switch (kc) {
      case 16: return launch_gemm<16, 16, XF, BWD, EPI, ST>(a, nout, C, o, s);
      case 32: return launch_gemm<32, 32, XF, BWD, EPI, ST>(a, nout, C, o, s);
      case 64: return launch_gemm<64, 32, XF, BWD, EPI, ST>(a, nout, C, o, s);
      default: return -2;
    }
  }
  // unit sizes measured with FEDML_AMD_C3_PX sweeps (profiles/r1_c3_unit_sweep.txt)
  constexpr int PX = ST == 2 ? 128 : 256;
  switch (kc) {
    case 16: return launch_gemm<16, 16, XF, BWD, EPI, ST>(a, nout, C, (BWD && ST == 1) ? 512 : PX, s);
    case 32: return launch_gemm<32, 32, XF, BWD, EPI, ST>(a, nout, C, PX, s);
    case 64: return launch_gemm<64, 32, XF, BWD, EPI, ST>(a, nout, C, ST == 2 ? 64 : 128, s);  // weights split over z
    default: return -2;
  }
}

}  // namespace c3

// forward 3×3 / pad 1 / stride 1|2: y = conv(pro(x)); stats[c][co][2] += (Σy, Σy²).
// (H, W) = input resolution. Returns < 0 if unsupported.
FA_EXPORT int fa_conv3x3_fwd(const uint16_t* x, const uint16_t* wpk, int64_t wpk_ld, const float* pscale,
                             const float* pshift, uint16_t* y, float* stats, int C, int N, int H, int W, int Cin,
                             int Cout, int ldk, int stride, hipStream_t stream) {
  if ((stride != 1 && stride != 2) || H % stride || W % stride || (W / stride) % 8 != 0) return -3;
  c3::Args a = {};
  a.src = x; a.wpk = wpk; a.wpk_ld = wpk_ld; a.vec0 = pscale; a.vec1 = pshift; a.out = y; a.stats = stats; a.NS = 2;
  a.N = N; a.H = H / stride; a.W = W / stride; a.Hs = H; a.Ws = W; a.ldk = ldk;
  if (stride == 2) {
    if (pscale) return c3::dispatch_gemm<c3::XF_BNRELU, 0, c3::EPI_FWD, 2>(Cin, Cout, a, C, stream);
    return c3::dispatch_gemm<c3::XF_NONE, 0, c3::EPI_FWD, 2>(Cin, Cout, a, C, stream);
  }
  if (pscale) return c3::dispatch_gemm<c3::XF_BNRELU, 0, c3::EPI_FWD, 1>(Cin, Cout, a, C, stream);
  return c3::dispatch_gemm<c3::XF_NONE, 0, c3::EPI_FWD, 1>(Cin, Cout, a, C, stream);
}

// backward-data 3×3 / pad 1 / stride 1|2 with the ReLU-mask epilogue (EPI_MASK of the generic kernel):
//   g' = convᵀ(α·g + β·y + γ) · [e_x·e_s + e_t > 0];  stats[c][ci][3] += (Σg', Σg'·e_x, ·)
// (Hx, Wx) = dx resolution; dy is (Hx/stride, Wx/stride).
FA_EXPORT int fa_conv3x3_bwd_data(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                                  const float* gamma, const uint16_t* wpk_b, int64_t wpk_ld, uint16_t* dx,
                                  const uint16_t* e_x, const float* e_s, const float* e_t, float* stats, int C, int N,
                                  int Hx, int Wx, int Cout, int Cin, int ldk2, int stride, hipStream_t stream) {
  if ((stride != 1 && stride != 2) || Hx % stride || Wx % stride || Wx % 8 != 0) return -3;
  c3::Args a = {};
  a.src = g; a.src2 = yv; a.wpk = wpk_b; a.wpk_ld = wpk_ld; a.vec0 = alpha; a.vec1 = beta; a.vec2 = gamma;
  a.out = dx; a.e_x = e_x; a.e_s = e_s; a.e_t = e_t; a.stats = stats; a.NS = 3;
  a.N = N; a.H = Hx; a.W = Wx; a.Hs = Hx / stride; a.Ws = Wx / stride; a.ldk = ldk2;
  if (stride == 2) return c3::dispatch_gemm<c3::XF_DY, 1, c3::EPI_MASK, 2>(Cout, Cin, a, C, stream);
  return c3::dispatch_gemm<c3::XF_DY, 1, c3::EPI_MASK, 1>(Cout, Cin, a, C, stream);
}

// weight gradient 3×3 / pad 1 / stride 1|2 into the GEMM-layout scratch `dw` [C][Cout][9·Cin] (zero
// on entry); the caller runs the scatter pass (fa_wgrad_scatter) into the OIHW arena.
// (H, W) = input (x) resolution.
FA_EXPORT int fa_conv3x3_wgrad(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                               const float* gamma, const uint16_t* x, const float* ps, const float* pt, float* dw,
                               int C, int N, int H, int W, int Cin, int Cout, int stride, hipStream_t stream) {
  if ((stride != 1 && stride != 2) || H % stride || W % stride || Cin != Cout) return -3;
  const int Ho = H / stride, Wo = W / stride;
  if (Wo % 8 != 0 || (Ho * Wo) % 32 != 0) return -3;
  c3::WArgs a = {};
  a.g = g; a.yv = yv; a.alpha = alpha; a.beta = beta; a.gamma = gamma; a.x = x; a.ps = ps; a.pt = pt; a.dw = dw;
  a.N = N; a.H = Ho; a.W = Wo; a.Hs = H; a.Ws = W;
  // units sized so one unit's operands fit the loaders' register budget (x tile ≤ 8, dy ≤ 4 chunks/thread)
  int tpx = Cin >= 64 ? (stride == 2 ? 64 : 128) : (stride == 2 ? 128 : 256);
  // Target workgroup count: every workgroup adds its Cout×9·Cin partial sums with fp32 atomics, so
  // more, shorter workgroups cost atomics per client (FEDML_AMD_C3W_WGS overrides, for tuning;
  // scripts/gpu_c3w_sweep*.sh)
  static const int wgs = [] {
    const char* e = getenv("FEDML_AMD_C3W_WGS");
    return e ? atoi(e) : 256;   // measured: +2/+3/+6 % rounds/s at 50/25/13 clients per GPU, neutral at 100
  }();
  c3::Plan p = c3::make_plan(N, Ho, Wo, C, tpx, wgs);
  while (tpx > 8) {
    const int tr = stride == 2 ? 2 * p.R + 1 : p.R + 2;
    if ((p.S * tr * (W + 2) * (Cin / 8) + 255) / 256 <= 8 && (p.S * p.R * Wo * (Cout / 8) + 255) / 256 <= 4) break;
    tpx /= 2;
    p = c3::make_plan(N, Ho, Wo, C, tpx, wgs);
  }
  a.R = p.R; a.S = p.S; a.units = p.units; a.units_per_wg = p.units_per_wg;
  const int TR = stride == 2 ? 2 * p.R + 1 : p.R + 2;
  a.fd_trtw = c3::make_fdiv(TR * (W + 2)); a.fd_tw = c3::make_fdiv(W + 2); a.fd_rw = c3::make_fdiv(p.R * Wo);
  a.fd_w = c3::make_fdiv(Wo);
  const int NTK = 9 * Cin / 16;
  const size_t vv = (size_t)(3 * Cout + 2 * Cin) * 4;
  const size_t smem_base = vv + (size_t)p.S * p.R * Wo * (Cout + 8) * 2 +
                           (size_t)p.S * TR * (W + 2) * (Cin + 8) * 2;
  const int needx = (p.S * TR * (W + 2) * (Cin / 8) + 255) / 256;
  const int needd = (p.S * p.R * Wo * (Cout / 8) + 255) / 256;
  if (needx > 8 || needd > 4) return -7;
#define W3_LAUNCH(CI, CO, WN, TPW, NZ, ST)                                                                     \
  {                                                                                                            \
    a.nt_per_z = (NTK + (NZ) - 1) / (NZ);                                                                      \
    auto kern = needx <= 4 ? (ps ? c3::conv3x3_wgrad_kernel<CI, CO, 1, WN, TPW, ST, 4, 4>                      \
                                 : c3::conv3x3_wgrad_kernel<CI, CO, 0, WN, TPW, ST, 4, 4>)                     \
                           : (ps ? c3::conv3x3_wgrad_kernel<CI, CO, 1, WN, TPW, ST, 8, 4>                      \
                                 : c3::conv3x3_wgrad_kernel<CI, CO, 0, WN, TPW, ST, 8, 4>);                    \
    const size_t red = (size_t)(4 / (WN) - 1) * (WN) * ((CO) / 16) * (TPW) * 256 * 4;                          \
    const size_t smem = smem_base > red + vv ? smem_base : red + vv;                                           \
    if (smem > 160 * 1024) return -5;                                                                          \
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);       \
    hipLaunchKernelGGL(kern, dim3(p.gx, C, NZ), dim3(256), smem, stream, a);                                   \
    return (int)hipGetLastError();                                                                             \
  }
#define W3_ALL(ST)                                                                                             \
  switch (Cin) {                                                                                               \
    case 16: W3_LAUNCH(16, 16, 1, 9, 1, ST)                                                                    \
    case 32: W3_LAUNCH(32, 32, 2, 9, 1, ST)                                                                    \
    case 64: W3_LAUNCH(64, 64, 4, 5, 2, ST)                                                                    \
    default: return -2;                                                                                        \
  }
  if (stride == 2) {
    W3_ALL(2)
  }
  W3_ALL(1)
#undef W3_ALL
#undef W3_LAUNCH
}
