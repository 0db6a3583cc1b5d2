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
// LDS pixel stride = P::pitch(channels) (bf16: +8, fp32: +4; P::pitch_tr for the weight-gradient
// tiles): 16-B-aligned for the vector staging writes and bank-spread for the fragment reads.
// Every kernel is instantiated for bf16 and fp32 storage (prec.h); the fp32 instances are the
// reference-precision path (exact fp32 MFMA products, fp32 activations).
#include "prec.h"
#include "detacc.h"
#include "bnlazy.h"
#include <algorithm>

#include <cstdlib>

FA_DET_EXPORT(conv3x3)

#ifndef TAP_UNROLL
#define TAP_UNROLL 3
#endif
// Weight-gradient kernels with ≤ 8 prefetched x chunks per thread run ≥ 2 waves per SIMD: the fp32 instances
// otherwise allocate 270-290 registers (VGPR + AGPR: loader prefetch registers, 20 accumulator tiles) and run ONE
// wave per SIMD, so every barrier and exposed load stalls the matrix pipe. Measured (C=100 headline): 64-channel
// wgrad 880 → 651 µs, 32-channel 590 → 444 µs. The forward / backward-data kernels and the 16-chunk wgrad variants
// keep the compiler's choice: forced to 256 registers they spill (stage-2 backward-data 452 → 594 µs).
#ifndef C3W_MIN_WAVES
#define C3W_MIN_WAVES 2
#endif

namespace c3 {

using prec::BF16;
using prec::F32;
using prec::F32X3;

enum { XF_NONE = 0, XF_BNRELU = 1, XF_DY = 2 };
enum { EPI_FWD = 0, EPI_MASK = 2, EPI_BLOCK = 3 };

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

// Operand transform of one 16-B chunk (P::VEC channels from ch0) with the per-channel vectors in
// LDS, two channels per packed-fp32 instruction.
template <class P, int XF>
struct ChunkVec {
  const float *v0, *v1, *v2;
  int ch0;
  __device__ __forceinline__ void load(const float* a, const float* b, const float* c, int ch) {
    v0 = a; v1 = b; v2 = c; ch0 = ch;
  }
  // XF_BNRELU: relu(x·s + t);  XF_DY: α·g + β·y + γ
  __device__ __forceinline__ uint4 apply(uint4 v, uint4 w) const {
    if (XF == XF_NONE) return v;
    float x[P::VEC], o[P::VEC];
    P::unpack(v, x);
    const f32x2* A = reinterpret_cast<const f32x2*>(v0 + ch0);
    const f32x2* B = reinterpret_cast<const f32x2*>(v1 + ch0);
    const f32x2* Cv = reinterpret_cast<const f32x2*>(v2 + ch0);
    if (XF == XF_BNRELU) {
#pragma unroll
      for (int j = 0; j < P::VEC / 2; ++j) {
        f32x2 r = f32x2{x[2 * j], x[2 * j + 1]} * A[j] + B[j];
        o[2 * j] = fmaxf(r.x, 0.f);
        o[2 * j + 1] = fmaxf(r.y, 0.f);
      }
    } else {
      float y[P::VEC];
      P::unpack(w, y);
#pragma unroll
      for (int j = 0; j < P::VEC / 2; ++j) {
        const f32x2 r = f32x2{x[2 * j], x[2 * j + 1]} * A[j] + (f32x2{y[2 * j], y[2 * j + 1]} * B[j] + Cv[j]);
        o[2 * j] = r.x;
        o[2 * j + 1] = r.y;
      }
    }
    return P::pack(o);
  }
};

// Stage one work unit of a client into an LDS tile [ns][TR][TW][LD] with the operand transform
// applied. Tile row tr / column tc hold source pixel (t0 + tr, tc − 1); outside the source image
// the tile is zero (the convolution's zero padding). UPS: the source is read zero-upsampled by 2
// (stride-2 backward-data: dy sits at the even positions of the dx grid). `src`/`src2` already
// point at the client. Register-prefetching: load() issues every global read of a unit (≤ MAXC
// 16-B chunks per thread, checked on the host) into registers, store() transforms and writes the
// tile. The unit loops call load() for unit u+1 right after the tile of unit u is in LDS, so the
// HBM latency of the next unit overlaps this unit's MFMA work instead of being paid serially.
template <class P, int KC, int XF, int UPS, int MAXC, bool TR = false>
struct TileLoader {
  using T = typename P::T;
  static constexpr int CG = KC / P::VEC;
  static constexpr int LD = TR ? P::pitch_tr(KC) : P::pitch(KC);
  uint4 r1[MAXC], r2[XF == XF_DY ? MAXC : 1];
  uint32_t okm;
  int total;
  __device__ __forceinline__ void load(const T* __restrict__ src, const T* __restrict__ src2, int img0,
                                       int ns, int t0, int TR_, int TW, FastDiv fd_trtw, FastDiv fd_tw, int Hs,
                                       int Ws) {
    const int TRTW = TR_ * TW;
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
        const int64_t off = ((((int64_t)(img0 + im) * Hs) + t) * Ws + u) * KC + cg * P::VEC;
        r1[j] = *reinterpret_cast<const uint4*>(src + off);
        if (XF == XF_DY) r2[j] = *reinterpret_cast<const uint4*>(src2 + off);
        okm |= 1u << j;
      }
    }
  }
  __device__ __forceinline__ void store(T* tile, const ChunkVec<P, XF>& cv) const {
    const int cg = threadIdx.x % CG;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int i = threadIdx.x + j * 256;
      if (i < total) {
        const uint4 v = (okm >> j) & 1u ? cv.apply(r1[j], XF == XF_DY ? r2[j] : r1[j]) : make_uint4(0, 0, 0, 0);
        T* dst = tile + (int64_t)(i / CG) * LD + cg * P::VEC;
        if (TR) P::st_chunk(dst, v);
        else *reinterpret_cast<uint4*>(dst) = v;
      }
    }
  }
};

// dy = α·g + β·y + γ staged pixel-major without halo (weight gradient), prefetched the same way.
template <class P, int COUT, int MAXD>
struct DyLoader {
  using T = typename P::T;
  static constexpr int CGD = COUT / P::VEC;
  uint4 rg[MAXD], ry[MAXD];
  int total;
  __device__ __forceinline__ void load(const T* __restrict__ gc, const T* __restrict__ yc, int64_t pix0,
                                       int npix) {
    total = npix * CGD;
    const int cg = threadIdx.x % CGD;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      const int i = threadIdx.x + j * 256;
      rg[j] = ry[j] = make_uint4(0, 0, 0, 0);
      if (i < total) {
        const int64_t off = (pix0 + i / CGD) * COUT + cg * P::VEC;
        rg[j] = *reinterpret_cast<const uint4*>(gc + off);
        ry[j] = *reinterpret_cast<const uint4*>(yc + off);
      }
    }
  }
  __device__ __forceinline__ void store(T* dyL, const ChunkVec<P, XF_DY>& dv) const {
    constexpr int LDD = P::pitch_tr(COUT);
    const int cg = threadIdx.x % CGD;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      const int i = threadIdx.x + j * 256;
      if (i < total) P::st_chunk(dyL + (size_t)(i / CGD) * LDD + cg * P::VEC, dv.apply(rg[j], ry[j]));
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

// Valid images of client c (heterogeneous batches: images past nimg[c] are padding and never touched)
// and the work units they span.
__device__ __forceinline__ int client_images(const int* nimg, int c, int N) { return nimg ? min(N, nimg[c]) : N; }
__device__ __forceinline__ int client_units(int Ne, int H, int R, int S) { return S > 1 ? (Ne + S - 1) / S : Ne * (H / R); }

struct Args {              // tensors are P::T (bf16 | fp32) unless noted
  const void* src;       // x (forward) or g (backward-data)        [C][N][H][W][KC]
  const void* src2;      // y for XF_DY
  const void* wpk;       // packed weights [C][NOUT][ldk], k = tap·KC + kc
  int64_t wpk_ld;
  const float* vec0;     // scale | α
  const float* vec1;     // shift | β
  const float* vec2;     //       | γ
  void* out;             // [C][N][H][W][NOUT]
  const void* e_x;       // EPI_MASK: previous raw activation [C][N][H][W][NOUT]; EPI_BLOCK: block input (mask)
  const void* e_add;     // EPI_BLOCK: shortcut gradient added before the mask
  const void* e_y1;      // EPI_BLOCK: previous block's last-BN input (Σg'·y1; null: not accumulated)
  const void* e_y2;      // EPI_BLOCK: previous block's shortcut-BN input (Σg'·y2; null: none)
  const float* e_s;
  const float* e_t;
  float* stats;          // [C][NOUT][NS]
  const float* pivot;    // EPI_FWD: per-(client, channel) shift subtracted from the stored output (or null)
  const int* nimg;       // per-client valid images (null: all N) — heterogeneous client batches
  int NS;
  int N, H, W;                    // output (iteration) geometry
  int Hs, Ws;                     // A-operand source geometry (≠ H, W for stride 2)
  int ldk;
  int R, S, units, units_per_wg;  // stage geometry (see unit_geom) and work split
  int nout_total;                 // output channels of the layer (a workgroup computes NOUT of them)
  FastDiv fd_trtw, fd_tw, fd_rw, fd_w;  // ÷ TR·TW, ÷ TW (tile), ÷ R·W, ÷ W (output unit)
  const BnLazy* lz0;              // XF_BNRELU: deferred finalisation of the prologue BN (bnlazy.h) or null
  int xcd;                        // XCD-aware block order (FEDML_AMD_C3_XCD, default on)
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
template <class P, int KC, int NOUT, int XF, int BWD, int EPI, int MTW, int ST, int MAXC>
__global__ __launch_bounds__(256) void conv3x3_gemm_kernel(Args a) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  constexpr int NT = NOUT / 16;
  constexpr int LD = P::pitch(KC);
  constexpr int K = 9 * KC;
  constexpr int KSTEPS = (K + 31) / 32;
  // XCD-aware order: workgroups go round-robin over the 8 XCDs (linear id mod 8). Remap so each XCD runs a
  // contiguous client-major run of (unit block, output slice) with the slice fastest: the NOUT/32 slices of one
  // unit block — which stage the SAME input tile — then run back to back on one XCD and the later ones read the
  // tile from that XCD's L2 instead of HBM
  int bx = blockIdx.x, bz = blockIdx.z, c = blockIdx.y;
  if (a.xcd) {
    const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
    const int total = gx * gy * gz, full = total / 8 * 8;
    int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    if (lin < full) lin = (lin % 8) * (full / 8) + lin / 8;
    bz = lin % gz;
    bx = (lin / gz) % gx;
    c = lin / (gz * gx);
  }
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int H = a.H, W = a.W, HW = H * W;
  const int Hs = a.Hs, Ws = a.Ws;
  constexpr int SP = (!BWD && ST == 2) ? 2 : 1;   // source-pixel step per output pixel
  constexpr bool UPS = BWD && ST == 2;
  const int TW = (UPS ? W : Ws) + 2;             // tile width incl. halo
  const int Ne = client_images(a.nimg, c, a.N);
  const int u_lo = bx * a.units_per_wg;
  const int u_hi = min(client_units(Ne, H, a.R, a.S), u_lo + a.units_per_wg);
  if (u_lo >= u_hi) return;   // no valid images in this workgroup's units (uniform: whole workgroup)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* wl = reinterpret_cast<T*>(smem);                                             // [NOUT][ldk]
  float* v0 = reinterpret_cast<float*>(smem + (size_t)NOUT * a.ldk * P::ES);     // [KC] ×3
  float* v1 = v0 + KC;
  float* v2 = v1 + KC;
  float* red = v2 + KC;                                                           // [4][NOUT][3]
  float* esL = red + 4 * NOUT * 3;                                                // [NOUT] ×2 (EPI_MASK)
  float* etL = esL + NOUT;
  T* tile = reinterpret_cast<T*>(etL + NOUT);                                     // [S][TR][TW][LD]

  const int ch_base = bz * NOUT;  // output-channel slice of this workgroup
  const int NO = a.nout_total;
  {
    const uint4* s = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.wpk) + (int64_t)c * a.wpk_ld +
                                                    (int64_t)ch_base * a.ldk);
    uint4* d = reinterpret_cast<uint4*>(wl);
    const int n16 = NOUT * a.ldk / P::VEC;
    for (int i = threadIdx.x; i < n16; i += 256) d[i] = s[i];
    if (XF != XF_NONE)
      for (int i = threadIdx.x; i < KC; i += 256) {
        if (XF == XF_BNRELU && a.lz0) {
          bn_lazy_fwd(a.lz0, c, i, bx == 0 && bz == 0, v0[i], v1[i]);
        } else {
          v0[i] = a.vec0[(int64_t)c * KC + i];
          v1[i] = a.vec1[(int64_t)c * KC + i];
        }
        if (XF == XF_DY) v2[i] = a.vec2[(int64_t)c * KC + i];
      }
    if (EPI == EPI_MASK)
      for (int i = threadIdx.x; i < NOUT; i += 256) {
        esL[i] = a.e_s[(int64_t)c * NO + ch_base + i];
        etL[i] = a.e_t[(int64_t)c * NO + ch_base + i];
      }
  }
  __syncthreads();
  ChunkVec<P, XF> cvec;
  cvec.load(v0, v1, v2, (threadIdx.x % (KC / P::VEC)) * P::VEC);

  const T* src = reinterpret_cast<const T*>(a.src) + (int64_t)c * a.N * Hs * Ws * KC;
  const T* src2 = (XF == XF_DY) ? reinterpret_cast<const T*>(a.src2) + (int64_t)c * a.N * Hs * Ws * KC : nullptr;
  T* out = reinterpret_cast<T*>(a.out) + (int64_t)c * a.N * HW * NO;
  const int64_t eo = (int64_t)c * a.N * HW * NO;
  const T* ex = (EPI != EPI_FWD) ? reinterpret_cast<const T*>(a.e_x) + eo : nullptr;
  const T* ea = (EPI == EPI_BLOCK) ? reinterpret_cast<const T*>(a.e_add) + eo : nullptr;
  const T* ey1 = (EPI == EPI_BLOCK && a.e_y1) ? reinterpret_cast<const T*>(a.e_y1) + eo : nullptr;
  const T* ey2 = (EPI == EPI_BLOCK && a.e_y2) ? reinterpret_cast<const T*>(a.e_y2) + eo : nullptr;

  // per-lane epilogue state: channels ch_base + nt·16 + 4g + i; forward outputs are stored as y − K with a
  // per-channel pivot K ≈ the batch mean (BatchNorm statistics and the folded backward then work on
  // values centred near 0: no E[y²] − mean² cancellation)
  float st0[NT][4], st1[NT][4], st2[EPI == EPI_BLOCK ? NT : 1][4], piv[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      piv[nt][i] = (EPI == EPI_FWD && a.pivot) ? a.pivot[(int64_t)c * NO + ch_base + nt * 16 + 4 * g + i] : 0.f;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st0[nt][i] = 0.f;
      st1[nt][i] = 0.f;
      if (EPI == EPI_BLOCK) st2[EPI == EPI_BLOCK ? nt : 0][i] = 0.f;
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
  const T* wrow = wl + (lane & 15) * a.ldk + 8 * g;

  const int R = a.R, RW = R * W;
  const int TR = SP == 2 ? 2 * R + 1 : R + 2;    // tile rows incl. halo
  TileLoader<P, KC, XF, UPS, MAXC> ld;
  {
    int img0, ns, r0;
    unit_geom(u_lo, Ne, H, R, a.S, img0, ns, r0);
    ld.load(src, src2, img0, ns, SP * r0 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
  }
  for (int u = u_lo; u < u_hi; ++u) {
    int img0, ns, r0;
    unit_geom(u, Ne, H, R, a.S, img0, ns, r0);
    const int64_t pix0 = (int64_t)img0 * HW + (int64_t)r0 * W;  // first output pixel of the unit
    __syncthreads();  // previous unit fully consumed
    ld.store(tile, cvec);
    __syncthreads();
    if (u + 1 < u_hi) {  // next unit's global reads in flight during this unit's MFMAs
      int img1, ns1, r1;
      unit_geom(u + 1, Ne, H, R, a.S, img1, ns1, r1);
      ld.load(src, src2, img1, ns1, SP * r1 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
    }
    const int P_ = ns * RW;
    const int ntile = (P_ + 15) / 16;
    for (int t0 = wid * MTW; t0 < ntile; t0 += 4 * MTW) {
      int base[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        const int p = (t0 + mt) * 16 + (lane & 15);
        const int pp = p < P_ ? p : 0;
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
            frag_t af[MTW];
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt) af[mt] = P::frag(tile + base[mt] + tapoff + cc * 32);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              const frag_t bw = P::frag(wrow + nt * 16 * a.ldk + (tap * (KC / 32) + cc) * 32);
#pragma unroll
              for (int mt = 0; mt < MTW; ++mt) acc[mt][nt] = P::mma(bw, af[mt], acc[mt][nt]);
            }
          }
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
          frag_t af[MTW];
#pragma unroll
          for (int mt = 0; mt < MTW; ++mt) af[mt] = P::frag(tile + base[mt] + toff[ks]);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const frag_t bw = P::frag(wrow + nt * 16 * a.ldk + ks * 32);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt) acc[mt][nt] = P::mma(bw, af[mt], acc[mt][nt]);
          }
        }
      }
      // ---- epilogue from the accumulators: lane = (pixel lane&15, channels 4g..4g+3 of each nt) ----
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        const int p = (t0 + mt) * 16 + (lane & 15);
        if (p >= P_) continue;
        const int64_t prow = (pix0 + p) * NO + ch_base + 4 * g;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          float f[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
          if (EPI == EPI_FWD) {
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] -= piv[nt][i];
            P::store4(out + prow + nt * 16, f);   // f ← the stored (rounded) values
#pragma unroll
            for (int i = 0; i < 4; ++i) { st0[nt][i] += f[i]; st1[nt][i] += f[i] * f[i]; }
          } else if (EPI == EPI_BLOCK) {   // g' = (dx + shortcut gradient) · [block input > 0]
            float xv[4], ev[4];
            P::load4(ex + prow + nt * 16, xv);
            P::load4(ea + prow + nt * 16, ev);
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] = xv[i] > 0.f ? f[i] + ev[i] : 0.f;
            P::store4(out + prow + nt * 16, f);   // f ← the stored (rounded) values
#pragma unroll
            for (int i = 0; i < 4; ++i) st0[nt][i] += f[i];
            if (ey1) {
              float y1[4];
              P::load4(ey1 + prow + nt * 16, y1);
#pragma unroll
              for (int i = 0; i < 4; ++i) st1[nt][i] += f[i] * y1[i];
            }
            if (ey2) {
              float y2[4];
              P::load4(ey2 + prow + nt * 16, y2);
#pragma unroll
              for (int i = 0; i < 4; ++i) st2[EPI == EPI_BLOCK ? nt : 0][i] += f[i] * y2[i];
            }
          } else {
            float xv[4];
            P::load4(ex + prow + nt * 16, xv);
            const float4 es = *reinterpret_cast<const float4*>(esL + nt * 16 + 4 * g);
            const float4 et = *reinterpret_cast<const float4*>(etL + nt * 16 + 4 * g);
            f[0] = (xv[0] * es.x + et.x > 0.f) ? f[0] : 0.f;
            f[1] = (xv[1] * es.y + et.y > 0.f) ? f[1] : 0.f;
            f[2] = (xv[2] * es.z + et.z > 0.f) ? f[2] : 0.f;
            f[3] = (xv[3] * es.w + et.w > 0.f) ? f[3] : 0.f;
            P::store4(out + prow + nt * 16, f);
#pragma unroll
            for (int i = 0; i < 4; ++i) { st0[nt][i] += f[i]; st1[nt][i] += f[i] * xv[i]; }
          }
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
        if (EPI == EPI_BLOCK) st2[EPI == EPI_BLOCK ? nt : 0][i] += __shfl_xor(st2[EPI == EPI_BLOCK ? nt : 0][i], o, 64);
      }
  }
  constexpr int NQ = EPI == EPI_BLOCK ? 3 : 2;   // statistics columns written
  if ((lane & 15) == 0) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[(wid * NOUT + nt * 16 + 4 * g + i) * 3 + 0] = st0[nt][i];
        red[(wid * NOUT + nt * 16 + 4 * g + i) * 3 + 1] = st1[nt][i];
        if (EPI == EPI_BLOCK) red[(wid * NOUT + nt * 16 + 4 * g + i) * 3 + 2] = st2[EPI == EPI_BLOCK ? nt : 0][i];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NOUT * NQ; i += 256) {
    const int ch = i / NQ, q = i % NQ;
    if (EPI == EPI_BLOCK && q == 2 && !ey2) continue;
    const float s = red[(0 * NOUT + ch) * 3 + q] + red[(1 * NOUT + ch) * 3 + q] + red[(2 * NOUT + ch) * 3 + q] +
                    red[(3 * NOUT + ch) * 3 + q];
    fa_acc_add(&a.stats[((int64_t)c * NO + ch_base + ch) * a.NS + q], s);
  }
}

// ---------------------------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------------------------
// per-layer operands of a multi-layer weight-gradient launch (conv3x3_wgrad_multi): same geometry, own tensors
struct WPtrs {
  const void* g;
  const void* yv;
  const float* alpha;
  const float* beta;
  const float* gamma;
  const void* x;
  const float* ps;
  const float* pt;
  float* dw;
};

struct WArgs {           // activations are P::T
  const WPtrs* tab;       // multi-layer launch: nl layers × C clients along blockIdx.y (null: one layer, these below)
  int nl;
  const void* g;          // [C][N][H][W][COUT]
  const void* yv;
  const float* alpha;
  const float* beta;
  const float* gamma;
  const void* x;          // [C][N][H][W][CIN]
  const float* ps;
  const float* pt;
  float* dw;              // GEMM-layout scratch [C][COUT][9·CIN]
  const int* nimg;        // per-client valid images (null: all N)
  const BnLazy* lz0;      // deferred backward finalisation of the BN whose α/β/γ this kernel reads (or null)
  int N, H, W;            // dy (output) geometry
  int Hs, Ws;             // x (input) geometry
  int R, S, units, units_per_wg;
  int nt_per_z;           // GEMM column tiles (16 wide) per blockIdx.z
  FastDiv fd_trtw, fd_tw, fd_rw, fd_w;
  int xcd;                // XCD-aware block order (FEDML_AMD_C3_XCD, default on)
};

// WN waves split the column tiles of this z-slice, WK = 4/WN waves split the pixel K-steps.
template <class P, int CIN, int COUT, int PRO, int WN, int TPW, int ST, int MAXC, int MAXD>
__global__ __launch_bounds__(256, (MAXC <= 8 ? C3W_MIN_WAVES : 1)) void conv3x3_wgrad_kernel(WArgs a) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  constexpr int WK = 4 / WN;
  constexpr int MT = COUT / 16;
  constexpr int LDX = P::pitch_tr(CIN), LDD = P::pitch_tr(COUT);
  constexpr int K = 9 * CIN;
  // XCD-aware order as in conv3x3_gemm_kernel: the column slices (z) of one pixel chunk stage the same dy and x
  // tiles, so they run back to back on one XCD and share its L2
  int bx = blockIdx.x, bz = blockIdx.z, c = blockIdx.y;
  if (a.xcd) {
    const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
    const int total = gx * gy * gz, full = total / 8 * 8;
    int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    if (lin < full) lin = (lin % 8) * (full / 8) + lin / 8;
    bz = lin % gz;
    bx = (lin / gz) % gx;
    c = lin / (gz * gx);
  }
  if (a.tab) {   // layer l = (block row) / C (uniform: scalar loads of its operand pointers)
    const int Cc = gridDim.y / a.nl, l = c / Cc;
    c -= l * Cc;
    const WPtrs q = a.tab[l];
    a.g = q.g; a.yv = q.yv; a.alpha = q.alpha; a.beta = q.beta; a.gamma = q.gamma;
    a.x = q.x; a.ps = q.ps; a.pt = q.pt; a.dw = q.dw;
  }
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int kgrp = wid / WN, ngrp = wid % WN;
  const int H = a.H, W = a.W, HW = H * W;
  const int Hs = a.Hs, Ws = a.Ws, TW = Ws + 2;
  const int nt_lo = bz * a.nt_per_z;
  const int nt_hi = min(K / 16, nt_lo + a.nt_per_z);
  const int my_nt0 = nt_lo + ngrp * TPW;  // this wave's column tiles [my_nt0, my_nt0 + TPW) ∩ [.., nt_hi)
  const int Ne = client_images(a.nimg, c, a.N);
  const int u_lo = bx * a.units_per_wg;
  const int u_hi = min(client_units(Ne, H, a.R, a.S), u_lo + a.units_per_wg);
  if (u_lo >= u_hi) return;   // nothing to add (uniform: whole workgroup)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* vv = reinterpret_cast<float*>(smem);                          // α β γ [COUT], s t [CIN]
  T* dyL = reinterpret_cast<T*>(vv + 3 * COUT + 2 * CIN);             // [S·HW][LDD]
  T* xt = dyL + (size_t)a.S * a.R * W * LDD;                           // [S][TR][TW][LDX]

  for (int i = threadIdx.x; i < COUT; i += 256) {
    if (a.lz0) {
      bn_lazy_bwd(a.lz0, c, i, bx == 0 && bz == 0, vv[i], vv[COUT + i], vv[2 * COUT + i]);
    } else {
      vv[i] = a.alpha[(int64_t)c * COUT + i];
      vv[COUT + i] = a.beta[(int64_t)c * COUT + i];
      vv[2 * COUT + i] = a.gamma[(int64_t)c * COUT + i];
    }
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

  const T* gc = reinterpret_cast<const T*>(a.g) + (int64_t)c * a.N * HW * COUT;
  const T* yc = reinterpret_cast<const T*>(a.yv) + (int64_t)c * a.N * HW * COUT;
  const T* xc = reinterpret_cast<const T*>(a.x) + (int64_t)c * a.N * Hs * Ws * CIN;
  const int R = a.R, RW = R * W;
  const int TR = ST == 2 ? 2 * R + 1 : R + 2;

  constexpr int CGD = COUT / P::VEC;
  static_assert(256 % CGD == 0, "fixed chunk per thread");
  __syncthreads();  // vectors
  ChunkVec<P, XF_DY> dvec;
  dvec.load(vv, vv + COUT, vv + 2 * COUT, (threadIdx.x % CGD) * P::VEC);
  ChunkVec<P, PRO ? XF_BNRELU : XF_NONE> xvec;
  xvec.load(vv + 3 * COUT, vv + 3 * COUT + CIN, nullptr, (threadIdx.x % (CIN / P::VEC)) * P::VEC);
  TileLoader<P, CIN, PRO ? XF_BNRELU : XF_NONE, 0, MAXC, true> xld;
  DyLoader<P, COUT, MAXD> dld;
  {
    int img0, ns, r0;
    unit_geom(u_lo, Ne, H, R, a.S, img0, ns, r0);
    dld.load(gc, yc, (int64_t)img0 * HW + (int64_t)r0 * W, ns * RW);
    xld.load(xc, nullptr, img0, ns, ST * r0 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
  }
  for (int u = u_lo; u < u_hi; ++u) {
    int img0, ns, r0;
    unit_geom(u, Ne, H, R, a.S, img0, ns, r0);
    __syncthreads();
    dld.store(dyL, dvec);  // dy = α·g + β·y + γ, natural [pixel][co] (no halo)
    xld.store(xt, xvec);
    __syncthreads();
    if (u + 1 < u_hi) {
      int img1, ns1, r1;
      unit_geom(u + 1, Ne, H, R, a.S, img1, ns1, r1);
      dld.load(gc, yc, (int64_t)img1 * HW + (int64_t)r1 * W, ns1 * RW);
      xld.load(xc, nullptr, img1, ns1, ST * r1 - 1, TR, TW, a.fd_trtw, a.fd_tw, Hs, Ws);
    }
    const int KS = ns * RW / 32;  // R·W is a multiple of 32
    for (int ks = kgrp; ks < KS; ks += WK) {
      const int p0 = ks * 32;
      // this lane's first pixel of the fragment (its 8 pixels 8g..8g+7 never straddle an image row:
      // W % 8 == 0)
      const int pix = p0 + P::px_row(lane);
      const int im = fdiv(pix, a.fd_rw);
      const int r = pix - im * RW;
      const int rr = fdiv(r, a.fd_w);
      const T* xrow = xt + (size_t)((im * TR + ST * rr) * TW + ST * (r - rr * W)) * LDX + P::px_col(lane);
      const T* drow = dyL + (size_t)pix * LDD + P::px_col(lane);
      frag_t af[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) af[m] = P::frag_px(drow + m * 16, LDD);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        // branch-free: a tile past the slice end recomputes its last tile (the epilogue discards it), so all
        // TPW fragment reads issue ahead of the MFMAs — behind a per-tile branch each read's LDS latency was
        // exposed before its 4 MFMAs (s_waitcnt lgkmcnt(0) per tile)
        const int nt = min(my_nt0 + t, nt_hi - 1);
        const int k0 = nt * 16;
        const int tap = k0 / CIN, ci0 = k0 % CIN;
        const int kh = tap / 3, kw = tap % 3;
        const frag_t bf = P::frag_px(xrow + (kh * TW + kw) * LDX + ci0, ST * LDX);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][t] = P::mma(af[m], bf, acc[m][t]);
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
          for (int i = 0; i < 4; ++i) fa_acc_add(&dwc[(int64_t)(m * 16 + 4 * g + i) * K + k], acc[m][t][i]);
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

template <class P>
static size_t gemm_smem(int kc, int nout, int ldk, const Plan& p, int TR, int TW) {
  return (size_t)nout * ldk * P::ES + (size_t)3 * kc * 4 + (size_t)4 * nout * 3 * 4 + (size_t)2 * nout * 4 +
         (size_t)p.S * TR * TW * P::pitch(kc) * P::ES;
}

// FEDML_AMD_C3_XCD=0: hardware block order in the 3×3 tile kernels (A/B of the XCD-aware remap)
static int c3_xcd() {
  static const int v = [] {
    const char* e = getenv("FEDML_AMD_C3_XCD");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <class P, int KC, int NOUT_WG, int XF, int BWD, int EPI, int MTW, int ST>
static auto gemm_variant(int need) {
  return need <= 4 ? conv3x3_gemm_kernel<P, KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 4>
       : need <= 8 ? conv3x3_gemm_kernel<P, KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 8>
                   : conv3x3_gemm_kernel<P, KC, NOUT_WG, XF, BWD, EPI, MTW, ST, 12>;
}

// NOUT_WG output channels per workgroup (blockIdx.z slices the layer's NOUT)
template <class P, int KC, int NOUT_WG, int XF, int BWD, int EPI, int ST>
static int launch_gemm(Args a, int nout, int C, int target_px, hipStream_t stream) {
  constexpr int CG = KC / P::VEC;
  static const int wgs_env = [] {   // FEDML_AMD_C3G_WGS: workgroup target of the fwd / bwd-data kernels
    const char* e = getenv("FEDML_AMD_C3G_WGS");
    return e ? atoi(e) : 0;
  }();
  // fp32: ~40 workgroups per client (512..2048): the 13-client share wants 512 (fwd 1.72 → 1.52, bwd-data
  // 1.86 → 1.61 ms/step), 100 clients keep 2048 (scripts/gpu_c3g_small_c.sh)
  const int PC = fa_plan_c(C);
  int wgs = wgs_env > 0 ? wgs_env : (P::kF32 ? std::min(2048, std::max(512, 40 * PC)) : 2048);
  // fp32 64-channel layers over many pixels (ResNet-18's 32² stage: 64 Ki pixels per client) want ~640 pixels
  // per workgroup: 512 → 1024 workgroups at 10 clients, −0.2 ms/step (profiles/r4_c3_r18_fp32_sweep.txt)
  if (P::kF32 && KC == 64 && wgs_env <= 0)
    wgs = std::max(wgs, (int)std::min<int64_t>(2048, (int64_t)PC * a.N * a.H * a.W / 640));
  Plan p = make_plan(a.N, a.H, a.W, PC, target_px, wgs);
  {  // a unit's tile must fit the loader's register budget (≤ 12 16-B chunks per thread)
    const bool f2 = !BWD && ST == 2;
    while (target_px > 8) {
      const int tr = f2 ? 2 * p.R + 1 : p.R + 2, tw = (BWD ? a.W : a.Ws) + 2;
      if ((p.S * tr * tw * CG + 255) / 256 <= 12) break;
      target_px /= 2;
      p = make_plan(a.N, a.H, a.W, PC, target_px, wgs);
    }
  }
  a.R = p.R; a.S = p.S; a.units = p.units; a.units_per_wg = p.units_per_wg; a.nout_total = nout;
  a.xcd = c3_xcd();
  const bool fwd2 = !BWD && ST == 2;
  const int TR = fwd2 ? 2 * p.R + 1 : p.R + 2;
  const int TW = (BWD ? a.W : a.Ws) + 2;
  const size_t smem = gemm_smem<P>(KC, NOUT_WG, a.ldk, p, TR, TW);
  if (smem > 160 * 1024) return -5;
  a.fd_trtw = make_fdiv(TR * TW); a.fd_tw = make_fdiv(TW); a.fd_rw = make_fdiv(p.R * a.W); a.fd_w = make_fdiv(a.W);
  const int need = (p.S * TR * TW * CG + 255) / 256;  // 16-B chunks per thread per unit
  if (need > 12) return -7;
  // 16-pixel tiles per wave: as many as keep all 4 waves busy on one unit. A unit of ONE 8×8 image (the
  // 64-channel fp32 layers: two would not fit the loader's registers) has 4 tiles, so MTW = 4 used to run
  // it on a single wave while three waited at the barrier.
  const int ntile = p.S * p.R * a.W / 16;
  auto kern = gemm_variant<P, KC, NOUT_WG, XF, BWD, EPI, 1, ST>(need);
  if (ntile >= 8) kern = gemm_variant<P, KC, NOUT_WG, XF, BWD, EPI, 2, ST>(need);
  if constexpr (NOUT_WG < 64)
    if (ntile >= 16) kern = gemm_variant<P, KC, NOUT_WG, XF, BWD, EPI, 4, ST>(need);
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

// per-channel-count unit override (tuning): FEDML_AMD_C3_PX16 / _PX32 / _PX64 (output pixels per LDS tile)
static int px_override_kc(int kc) {
  static const int v16 = [] { const char* e = getenv("FEDML_AMD_C3_PX16"); return e ? atoi(e) : 0; }();
  static const int v32 = [] { const char* e = getenv("FEDML_AMD_C3_PX32"); return e ? atoi(e) : 0; }();
  static const int v64 = [] { const char* e = getenv("FEDML_AMD_C3_PX64"); return e ? atoi(e) : 0; }();
  return kc == 16 ? v16 : kc == 32 ? v32 : kc == 64 ? v64 : 0;
}

// tuning override of the fp32 64-channel output slice per workgroup: FEDML_AMD_C3_N64=32 (default 16)
static int n64_override() {
  static const int v = [] {
    const char* e = getenv("FEDML_AMD_C3_N64");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <class P, int XF, int BWD, int EPI, int ST>
static int dispatch_gemm(int kc, int nout, const Args& a, int C, hipStream_t s) {
  if (kc != nout) return -2;
  if constexpr (P::kF32) {
    if (kc == 64 && n64_override() == 32) {
      const int r = launch_gemm<P, 64, 32, XF, BWD, EPI, ST>(
          a, nout, C, px_override() > 0 ? px_override() : (ST == 2 ? (BWD ? 256 : 64) : 128), s);
      if (r != -5) return r;   // -5: the 32-channel fp32 weight slice does not fit LDS with this unit
    }
  }
  // fp32: half the output channels per workgroup on the 64-channel layers (the fp32 weight slice of
  // 32 channels alone would take 75 KB of LDS)
  constexpr int N64 = P::kF32 ? 16 : 32;
  if (px_override() > 0) {
    const int o = px_override();
    switch (kc) {
      case 16: return launch_gemm<P, 16, 16, XF, BWD, EPI, ST>(a, nout, C, o, s);
      case 32: return launch_gemm<P, 32, 32, XF, BWD, EPI, ST>(a, nout, C, o, s);
      case 64: return launch_gemm<P, 64, N64, XF, BWD, EPI, ST>(a, nout, C, o, s);
      default: return -2;
    }
  }
  // unit sizes measured with FEDML_AMD_C3_PX sweeps (bf16: profiles/r1_c3_unit_sweep.txt; fp32:
  // profiles/r2_c3_sweep_fp32.txt — 256-px units for the fp32 backward, stride 2 included)
  constexpr int PX = ST == 2 ? ((P::kF32 && BWD) ? 256 : 128) : 256;
  if (ST == 1 && px_override_kc(kc) > 0) {
    const int o = px_override_kc(kc);
    switch (kc) {
      case 16: return launch_gemm<P, 16, 16, XF, BWD, EPI, ST>(a, nout, C, o, s);
      case 32: return launch_gemm<P, 32, 32, XF, BWD, EPI, ST>(a, nout, C, o, s);
      case 64: return launch_gemm<P, 64, N64, XF, BWD, EPI, ST>(a, nout, C, o, s);
      default: return -2;
    }
  }
  switch (kc) {
    case 16: return launch_gemm<P, 16, 16, XF, BWD, EPI, ST>(a, nout, C, (BWD && ST == 1 && !P::kF32) ? 512 : PX, s);
    // fp32 32-channel stride-1 layers: 64-px units (4 rows of 16²) — the loader then prefetches ≤ 8 chunks per
    // thread and the kernel keeps 2 waves per SIMD (256-px units: 12 chunks, 272-290 registers, 1 wave);
    // profiles/r3_c3_px_sweep.txt: fwd 0.416 → 0.361 ms, bwd 0.480 → 0.388 ms at C = 100
    case 32: return launch_gemm<P, 32, 32, XF, BWD, EPI, ST>(a, nout, C, (P::kF32 && ST == 1) ? 64 : PX, s);
    case 64: return launch_gemm<P, 64, N64, XF, BWD, EPI, ST>(a, nout, C, ST == 2 ? ((P::kF32 && BWD) ? 256 : 64) : 128,
                                                               s);  // weights split over z
    default: return -2;
  }
}

template <class P>
static int conv3x3_fwd(const void* x, const void* wpk, int64_t wpk_ld, const float* pscale, const float* pshift,
                       void* y, float* stats, int C, int N, int H, int W, int Cin, int Cout, int ldk, int stride,
                       const float* pivot, const int* nimg, hipStream_t stream) {
  if ((stride != 1 && stride != 2) || H % stride || W % stride || (W / stride) % 8 != 0) return -3;
  Args a = {};
  a.src = x; a.wpk = wpk; a.wpk_ld = wpk_ld; a.vec0 = pscale; a.vec1 = pshift; a.out = y; a.stats = stats; a.NS = 2;
  a.pivot = pivot; a.nimg = nimg; a.lz0 = fa_take_lazy(0);
  a.N = N; a.H = H / stride; a.W = W / stride; a.Hs = H; a.Ws = W; a.ldk = ldk;
  if (stride == 2) {
    if (pscale) return dispatch_gemm<P, XF_BNRELU, 0, EPI_FWD, 2>(Cin, Cout, a, C, stream);
    return dispatch_gemm<P, XF_NONE, 0, EPI_FWD, 2>(Cin, Cout, a, C, stream);
  }
  if (pscale) return dispatch_gemm<P, XF_BNRELU, 0, EPI_FWD, 1>(Cin, Cout, a, C, stream);
  return dispatch_gemm<P, XF_NONE, 0, EPI_FWD, 1>(Cin, Cout, a, C, stream);
}

template <class P>
static int conv3x3_bwd_data(const void* g, const void* yv, const float* alpha, const float* beta, const float* gamma,
                            const void* wpk_b, int64_t wpk_ld, void* dx, const void* e_x, const float* e_s,
                            const float* e_t, float* stats, int C, int N, int Hx, int Wx, int Cout, int Cin, int ldk2,
                            int stride, const int* nimg, hipStream_t stream, const void* e_add = nullptr,
                            const void* e_y1 = nullptr, const void* e_y2 = nullptr) {
  if ((stride != 1 && stride != 2) || Hx % stride || Wx % stride || Wx % 8 != 0) return -3;
  Args a = {};
  a.src = g; a.src2 = yv; a.wpk = wpk_b; a.wpk_ld = wpk_ld; a.vec0 = alpha; a.vec1 = beta; a.vec2 = gamma;
  a.out = dx; a.e_x = e_x; a.e_s = e_s; a.e_t = e_t; a.stats = stats; a.NS = 3; a.nimg = nimg;
  a.e_add = e_add; a.e_y1 = e_y1; a.e_y2 = e_y2;
  a.N = N; a.H = Hx; a.W = Wx; a.Hs = Hx / stride; a.Ws = Wx / stride; a.ldk = ldk2;
  if (e_add) {   // EPI_BLOCK (stride 1: the block's first conv keeps the channel count)
    if (stride != 1) return -3;
    return dispatch_gemm<P, XF_DY, 1, EPI_BLOCK, 1>(Cout, Cin, a, C, stream);
  }
  if (stride == 2) return dispatch_gemm<P, XF_DY, 1, EPI_MASK, 2>(Cout, Cin, a, C, stream);
  return dispatch_gemm<P, XF_DY, 1, EPI_MASK, 1>(Cout, Cin, a, C, stream);
}

template <class P>
static int conv3x3_wgrad(const void* g, const void* yv, const float* alpha, const float* beta, const float* gamma,
                         const void* x, const float* ps, const float* pt, float* dw, int C, int N, int H, int W,
                         int Cin, int Cout, int stride, const int* nimg, hipStream_t stream,
                         const WPtrs* tab = nullptr, int nl = 1, int has_ps = 0) {
  if ((stride != 1 && stride != 2) || H % stride || W % stride || Cin != Cout) return -3;
  const int Ho = H / stride, Wo = W / stride;
  if (Wo % 8 != 0 || (Ho * Wo) % 32 != 0) return -3;
  WArgs a = {};
  a.xcd = c3_xcd();
  a.g = g; a.yv = yv; a.alpha = alpha; a.beta = beta; a.gamma = gamma; a.x = x; a.ps = ps; a.pt = pt; a.dw = dw;
  a.tab = tab; a.nl = nl;
  a.lz0 = tab ? nullptr : fa_take_lazy(0);
  if (tab) ps = has_ps ? reinterpret_cast<const float*>(tab) : nullptr;   // selects the prologue variant below
  a.nimg = nimg;
  a.N = N; a.H = Ho; a.W = Wo; a.Hs = H; a.Ws = W;
  // units sized so one unit's operands fit the loaders' register budget (x tile ≤ 8, dy ≤ 4 chunks/thread)
  int tpx = Cin >= 64 ? (stride == 2 ? 64 : 128) : (stride == 2 ? 128 : 256);
  if (P::kF32) tpx /= 2;
  // Target workgroup count: every workgroup adds its Cout×9·Cin partial sums with fp32 atomics, so
  // more, shorter workgroups cost atomics per client (FEDML_AMD_C3W_WGS overrides, for tuning;
  // scripts/gpu_c3w_sweep*.sh)
  // bf16 256: +2/+3/+6 % rounds/s at 50/25/13 clients per GPU, neutral at 100 (fewer fp32 atomics per
  // client); fp32 2048: the MFMA work per workgroup dominates the atomics (wgrad 0.72 → 0.54 ms at 16×32²,
  // profiles/r2_c3_sweep_fp32.txt)
  // fp32 scales with the clients on this GPU (~20 workgroups per client, 256..2048): at 13 clients (the
  // 8-GPU share of the headline) 2048 workgroups spend the kernel on atomics — 256 cuts wgrad 2.16 → 1.67
  // ms/step, while 100 clients still want 2048 (scripts/gpu_c3w_small_c.sh)
  static const int wgs_env = [] {
    const char* e = getenv("FEDML_AMD_C3W_WGS");
    return e ? atoi(e) : 0;
  }();
  const int PC = fa_plan_c(C);
  int wgs = wgs_env > 0 ? wgs_env : (P::kF32 ? std::min(2048, std::max(256, 20 * PC)) : 256);
  // fp32 64-channel layers over many pixels: ~640 pixels per workgroup (ResNet-18 at 10 clients: 256 → 1024
  // workgroups, wgrad −0.6 ms/step; the 8² ResNet-56 layers keep the client-count rule; r4_c3_r18_fp32_sweep.txt)
  // and at most 1024 (100 clients, 64 channels at 8²: 2000 → 1024 workgroups, 2.78 → 2.43 ms/step; the 16- and
  // 32-channel layers keep 2000, profiles/r4_c3w_c100_sweep.txt)
  if (P::kF32 && Cin == 64 && wgs_env <= 0)
    wgs = std::max(std::min(wgs, 1024), (int)std::min<int64_t>(2048, (int64_t)PC * N * Ho * Wo / 640));
  const int CGX = Cin / P::VEC, CGD = Cout / P::VEC;
  constexpr int XMAX = P::kF32 ? 16 : 8;   // x-tile 16-B chunks per thread (fp32: twice the chunks per pixel)
  Plan p = make_plan(N, Ho, Wo, PC, tpx, wgs);
  while (tpx > 8) {
    const int tr = stride == 2 ? 2 * p.R + 1 : p.R + 2;
    if ((p.S * tr * (W + 2) * CGX + 255) / 256 <= XMAX && (p.S * p.R * Wo * CGD + 255) / 256 <= 4) break;
    tpx /= 2;
    p = make_plan(N, Ho, Wo, PC, tpx, wgs);
  }
  if ((p.R * Wo) % 32 != 0) return -7;   // a unit must hold whole 32-pixel K-steps
  a.R = p.R; a.S = p.S; a.units = p.units; a.units_per_wg = p.units_per_wg;
  const int TR = stride == 2 ? 2 * p.R + 1 : p.R + 2;
  a.fd_trtw = make_fdiv(TR * (W + 2)); a.fd_tw = make_fdiv(W + 2); a.fd_rw = make_fdiv(p.R * Wo);
  a.fd_w = make_fdiv(Wo);
  const int NTK = 9 * Cin / 16;
  const size_t vv = (size_t)(3 * Cout + 2 * Cin) * 4;
  const size_t smem_base = vv + (size_t)p.S * p.R * Wo * P::pitch_tr(Cout) * P::ES +
                           (size_t)p.S * TR * (W + 2) * P::pitch_tr(Cin) * P::ES;
  const int needx = (p.S * TR * (W + 2) * CGX + 255) / 256;
  const int needd = (p.S * p.R * Wo * CGD + 255) / 256;
  if (needx > XMAX || needd > 4) return -7;
  constexpr int XLO = P::kF32 ? 8 : 4;
#define W3_LAUNCH(CI, CO, WN, TPW, NZ, ST)                                                                     \
  {                                                                                                            \
    a.nt_per_z = (NTK + (NZ) - 1) / (NZ);                                                                      \
    auto kern = needx <= XLO ? (ps ? conv3x3_wgrad_kernel<P, CI, CO, 1, WN, TPW, ST, XLO, 4>                   \
                                   : conv3x3_wgrad_kernel<P, CI, CO, 0, WN, TPW, ST, XLO, 4>)                  \
                             : (ps ? conv3x3_wgrad_kernel<P, CI, CO, 1, WN, TPW, ST, XMAX, 4>                  \
                                   : conv3x3_wgrad_kernel<P, CI, CO, 0, WN, TPW, ST, XMAX, 4>);                \
    const size_t red = (size_t)(4 / (WN) - 1) * (WN) * ((CO) / 16) * (TPW) * 256 * 4;                          \
    const size_t smem = smem_base > red + vv ? smem_base : red + vv;                                           \
    if (smem > 160 * 1024) return -5;                                                                          \
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);       \
    hipLaunchKernelGGL(kern, dim3(p.gx, C * nl, NZ), dim3(256), smem, stream, a);                              \
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

}  // namespace c3

// forward 3×3 / pad 1 / stride 1|2: y = conv(pro(x)) − K; stats[c][co][2] += (Σy, Σy²) of the stored y.
// K = pivot[c][co] (null: 0). (H, W) = input resolution. Returns < 0 if unsupported.
// `_f32`: fp32 activations / packed weights.
FA_EXPORT int fa_conv3x3_fwd(const uint16_t* x, const uint16_t* wpk, int64_t wpk_ld, const float* pscale,
                             const float* pshift, uint16_t* y, float* stats, int C, int N, int H, int W, int Cin,
                             int Cout, int ldk, int stride, const float* pivot, const int* nimg,
                             hipStream_t stream) {
  return c3::conv3x3_fwd<c3::BF16>(x, wpk, wpk_ld, pscale, pshift, y, stats, C, N, H, W, Cin, Cout, ldk, stride,
                                   pivot, nimg, stream);
}
FA_EXPORT int fa_conv3x3_fwd_f32(const float* x, const float* wpk, int64_t wpk_ld, const float* pscale,
                                 const float* pshift, float* y, float* stats, int C, int N, int H, int W, int Cin,
                                 int Cout, int ldk, int stride, const float* pivot, const int* nimg,
                                 hipStream_t stream) {
  FA_F32_DISPATCH(c3, c3::conv3x3_fwd<PX>(x, wpk, wpk_ld, pscale, pshift, y, stats, C, N, H, W, Cin, Cout, ldk, stride,
                                  pivot, nimg, stream));
}

// backward-data 3×3 / pad 1 / stride 1|2 with the ReLU-mask epilogue (EPI_MASK of the generic kernel):
//   g' = convᵀ(α·g + β·y + γ) · [e_x·e_s + e_t > 0];  stats[c][ci][3] += (Σg', Σg'·e_x, ·)
// (Hx, Wx) = dx resolution; dy is (Hx/stride, Wx/stride).
FA_EXPORT int fa_conv3x3_bwd_data(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                                  const float* gamma, const uint16_t* wpk_b, int64_t wpk_ld, uint16_t* dx,
                                  const uint16_t* e_x, const float* e_s, const float* e_t, float* stats, int C, int N,
                                  int Hx, int Wx, int Cout, int Cin, int ldk2, int stride, const int* nimg,
                                  hipStream_t stream) {
  return c3::conv3x3_bwd_data<c3::BF16>(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, e_x, e_s, e_t, stats, C, N, Hx,
                                        Wx, Cout, Cin, ldk2, stride, nimg, stream);
}
FA_EXPORT int fa_conv3x3_bwd_data_f32(const float* g, const float* yv, const float* alpha, const float* beta,
                                      const float* gamma, const float* wpk_b, int64_t wpk_ld, float* dx,
                                      const float* e_x, const float* e_s, const float* e_t, float* stats, int C, int N,
                                      int Hx, int Wx, int Cout, int Cin, int ldk2, int stride, const int* nimg,
                                      hipStream_t stream) {
  FA_F32_DISPATCH(c3, c3::conv3x3_bwd_data<PX>(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, e_x, e_s, e_t, stats, C, N, Hx,
                                       Wx, Cout, Cin, ldk2, stride, nimg, stream));
}

// backward-data 3×3 / pad 1 / stride 1 of a block's first conv with the block epilogue (EPI_BLOCK of the
// generic kernel):  g' = (convᵀ(α·g + β·y + γ) + e_add) · [e_x > 0];  stats[c][ci][3] += (Σg', Σg'·e_y1, Σg'·e_y2)
// (e_y1 / e_y2 null: that column is left alone)
FA_EXPORT int fa_conv3x3_bwd_data_block(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                                        const float* gamma, const uint16_t* wpk_b, int64_t wpk_ld, uint16_t* dx,
                                        const uint16_t* e_x, const uint16_t* e_add, const uint16_t* e_y1,
                                        const uint16_t* e_y2, float* stats, int C, int N, int Hx, int Wx, int Cout,
                                        int Cin, int ldk2, const int* nimg, hipStream_t stream) {
  if (!e_add) return -3;
  return c3::conv3x3_bwd_data<c3::BF16>(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, e_x, nullptr, nullptr, stats, C,
                                        N, Hx, Wx, Cout, Cin, ldk2, 1, nimg, stream, e_add, e_y1, e_y2);
}
FA_EXPORT int fa_conv3x3_bwd_data_block_f32(const float* g, const float* yv, const float* alpha, const float* beta,
                                            const float* gamma, const float* wpk_b, int64_t wpk_ld, float* dx,
                                            const float* e_x, const float* e_add, const float* e_y1, const float* e_y2,
                                            float* stats, int C, int N, int Hx, int Wx, int Cout, int Cin, int ldk2,
                                            const int* nimg, hipStream_t stream) {
  if (!e_add) return -3;
  FA_F32_DISPATCH(c3, c3::conv3x3_bwd_data<PX>(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, e_x, nullptr, nullptr, stats,
                                       C, N, Hx, Wx, Cout, Cin, ldk2, 1, nimg, stream, e_add, e_y1, e_y2));
}

// weight gradient 3×3 / pad 1 / stride 1|2 into the GEMM-layout scratch `dw` [C][Cout][9·Cin] (zero
// on entry); the caller runs the scatter pass (fa_wgrad_scatter) into the OIHW arena.
// (H, W) = input (x) resolution.
FA_EXPORT int fa_conv3x3_wgrad(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                               const float* gamma, const uint16_t* x, const float* ps, const float* pt, float* dw,
                               int C, int N, int H, int W, int Cin, int Cout, int stride, const int* nimg,
                               hipStream_t stream) {
  return c3::conv3x3_wgrad<c3::BF16>(g, yv, alpha, beta, gamma, x, ps, pt, dw, C, N, H, W, Cin, Cout, stride, nimg,
                                     stream);
}
// the same weight gradient for nl layers of one geometry in ONE launch (`tab`: device table of nl WPtrs; has_ps:
// every layer has the BN + ReLU prologue on x): nl × the workgroups of one layer — the small-grid layers of a
// 13-client share fill the GPU together
FA_EXPORT int fa_conv3x3_wgrad_multi_f32(const void* tab, int nl, int has_ps, int C, int N, int H, int W, int Cin,
                                         int Cout, int stride, const int* nimg, hipStream_t stream) {
  if (!tab || nl < 1 || nl > 64) return -3;
  const c3::WPtrs* t = reinterpret_cast<const c3::WPtrs*>(tab);
  FA_F32_DISPATCH(c3, c3::conv3x3_wgrad<PX>(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                            nullptr, C, N, H, W, Cin, Cout, stride, nimg, stream, t, nl, has_ps));
}
FA_EXPORT int fa_conv3x3_wgrad_f32(const float* g, const float* yv, const float* alpha, const float* beta,
                                   const float* gamma, const float* x, const float* ps, const float* pt, float* dw,
                                   int C, int N, int H, int W, int Cin, int Cout, int stride, const int* nimg,
                                   hipStream_t stream) {
  FA_F32_DISPATCH(c3, c3::conv3x3_wgrad<PX>(g, yv, alpha, beta, gamma, x, ps, pt, dw, C, N, H, W, Cin, Cout, stride, nimg,
                                    stream));
}
