// 1×1 / stride-1 weight gradient for the client-batched ResNet (gfx950, bf16 MFMA).
//
//   dW[c][co][ci] += Σ_p dy[c][p][co] · act(x)[c][p][ci]
//   dy = α·g + β·y + γ (folded BN backward), act = PRO ? relu(x·s + t) : x
//
// A plain GEMM over pixels, so both operands are staged pixel-major in their natural layout and
// read with the transposing LDS read (ds_read_b64_tr_b16). Unlike the generic weight-gradient
// kernel (one fragment pair per output tile), each wave owns an MTW × NTW block of output tiles
// and reuses every A fragment NTW times and every B fragment MTW times; the next pixel chunk is
// prefetched into registers while the current one is multiplied. For 1×1 convolutions the GEMM
// layout [co][ci] IS the OIHW layout, so the partial sums go straight into the gradient arena
// with fp32 atomics — no scratch / scatter pass.
#include "prec.h"
#include "detacc.h"
#include "bnlazy.h"

FA_DET_EXPORT(conv1x1)

namespace c1 {

using prec::BF16;
using prec::F32;
using prec::F32X3;

// WM × WN waves tile the (COUT/16) × (CIN/16) output tiles; WK = 4/(WM·WN) waves split the pixels.
template <class P, int CIN, int COUT, int PRO, int WM, int WN, int PT>
__global__ __launch_bounds__(256) void conv1x1_wgrad_kernel(const typename P::T* __restrict__ g,
                                                            const typename P::T* __restrict__ yv,
                                                            const float* __restrict__ alpha,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ gamma,
                                                            const typename P::T* __restrict__ x,
                                                            const float* __restrict__ ps, const float* __restrict__ pt,
                                                            float* __restrict__ garena, int64_t ldw, int64_t woff,
                                                            int M, int pix_per_wg, const int* __restrict__ nimg,
                                                            int hw, const BnLazy* __restrict__ lz) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  constexpr int V = P::VEC;
  constexpr int WK = 4 / (WM * WN);
  constexpr int MTW = COUT / 16 / WM, NTW = CIN / 16 / WN;
  constexpr int LDD = P::pitch_tr(COUT), LDX = P::pitch_tr(CIN);
  constexpr int DCH = PT * COUT / V, XCH = PT * CIN / V;            // 16-B chunks per stage
  constexpr int DI = (DCH + 255) / 256, XI = (XCH + 255) / 256;    // per thread
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g4 = lane >> 4;
  const int kgrp = wid / (WM * WN), mgrp = (wid % (WM * WN)) / WN, ngrp = wid % WN;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* vv = reinterpret_cast<float*>(smem);                              // α β γ [COUT], s t [CIN]
  T* dyL = reinterpret_cast<T*>(vv + 3 * COUT + 2 * CIN);                  // [PT][LDD]
  T* xL = dyL + PT * LDD;                                                  // [PT][LDX]

  const bool raw = yv == nullptr;   // dy = g as stored (e.g. Gᵀ·act(x) of a recomputed-y bottleneck)
  if (!raw)
    for (int i = threadIdx.x; i < COUT; i += 256) {
      if (lz) {
        bn_lazy_bwd(lz, c, i, blockIdx.x == 0, vv[i], vv[COUT + i], vv[2 * COUT + i]);
      } else {
        vv[i] = alpha[(int64_t)c * COUT + i];
        vv[COUT + i] = beta[(int64_t)c * COUT + i];
        vv[2 * COUT + i] = gamma[(int64_t)c * COUT + i];
      }
    }
  if (PRO)
    for (int i = threadIdx.x; i < CIN; i += 256) {
      vv[3 * COUT + i] = ps[(int64_t)c * CIN + i];
      vv[3 * COUT + CIN + i] = pt[(int64_t)c * CIN + i];
    }

  const T* gc = g + (int64_t)c * M * COUT;
  const T* yc = raw ? nullptr : yv + (int64_t)c * M * COUT;
  const T* xc = x + (int64_t)c * M * CIN;
  const int p_begin = blockIdx.x * pix_per_wg;
  const int p_end = min(nimg ? min(M, nimg[c] * hw) : M, p_begin + pix_per_wg);   // valid pixels of client c
  if (p_begin >= p_end) return;

  uint4 rg[DI], ry[DI], rx[XI];
  auto load = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * 256;
      rg[it] = make_uint4(0, 0, 0, 0);
      ry[it] = make_uint4(0, 0, 0, 0);
      if (i < DCH) {
        const int p = p0 + i / (COUT / V);
        if (p < p_end) {
          const int64_t off = (int64_t)p * COUT + (i % (COUT / V)) * V;
          rg[it] = *reinterpret_cast<const uint4*>(gc + off);
          if (!raw) ry[it] = *reinterpret_cast<const uint4*>(yc + off);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * 256;
      rx[it] = make_uint4(0, 0, 0, 0);
      if (i < XCH) {
        const int p = p0 + i / (CIN / V);
        if (p < p_end) rx[it] = *reinterpret_cast<const uint4*>(xc + (int64_t)p * CIN + (i % (CIN / V)) * V);
      }
    }
  };
  auto store = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < DCH) {
        const int pp = i / (COUT / V), co0 = (i % (COUT / V)) * V;
        float gf[V], yf[V];
        P::unpack(rg[it], gf);
        P::unpack(ry[it], yf);
        const bool live = p0 + pp < p_end;
#pragma unroll
        for (int j = 0; j < V; ++j)
          gf[j] = !live ? 0.f : raw ? gf[j] : vv[co0 + j] * gf[j] + vv[COUT + co0 + j] * yf[j] + vv[2 * COUT + co0 + j];
        P::st_chunk(dyL + pp * LDD + co0, P::pack(gf));
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < XCH) {
        const int pp = i / (CIN / V), ci0 = (i % (CIN / V)) * V;
        uint4 v = rx[it];
        if (PRO && p0 + pp < p_end) {
          float f[V];
          P::unpack(v, f);
#pragma unroll
          for (int j = 0; j < V; ++j) f[j] = fmaxf(f[j] * vv[3 * COUT + ci0 + j] + vv[3 * COUT + CIN + ci0 + j], 0.f);
          v = P::pack(f);
        }
        P::st_chunk(xL + pp * LDX + ci0, v);
      }
    }
  };

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = {0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // vectors
  if (p_begin < p_end) load(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += PT) {
    store(p0);
    __syncthreads();
    if (p0 + PT < p_end) load(p0 + PT);
#pragma unroll
    for (int ks = kgrp; ks < PT / 32; ks += WK) {
      frag_t af[MTW], bfr[NTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) af[m] = P::frag_tr(dyL, LDD, ks * 32, (mgrp * MTW + m) * 16, lane);
#pragma unroll
      for (int n = 0; n < NTW; ++n) bfr[n] = P::frag_tr(xL, LDX, ks * 32, (ngrp * NTW + n) * 16, lane);
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n) acc[m][n] = P::mma(af[m], bfr[n], acc[m][n]);
    }
    __syncthreads();
  }

  // ---- reduce pixel groups through LDS, then atomics straight into the OIHW arena ----
  if (WK > 1) {
    float* rbuf = reinterpret_cast<float*>(dyL);
    if (kgrp > 0) {
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            rbuf[((((kgrp - 1) * (WM * WN) + mgrp * WN + ngrp) * MTW + m) * NTW + n) * 256 + i * 64 + lane] =
                acc[m][n][i];
    }
    __syncthreads();
    if (kgrp == 0)
      for (int k2 = 1; k2 < WK; ++k2)
#pragma unroll
        for (int m = 0; m < MTW; ++m)
#pragma unroll
          for (int n = 0; n < NTW; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[m][n][i] += rbuf[((((k2 - 1) * (WM * WN) + mgrp * WN + ngrp) * MTW + m) * NTW + n) * 256 + i * 64 + lane];
  }
  if (kgrp == 0) {
    float* gw = garena + (int64_t)c * ldw + woff;
#pragma unroll
    for (int m = 0; m < MTW; ++m)
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const int ci = (ngrp * NTW + n) * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = (mgrp * MTW + m) * 16 + 4 * g4 + i;
          fa_acc_add(&gw[(int64_t)co * CIN + ci], acc[m][n][i]);
        }
      }
  }
}

template <class P, int CIN, int COUT, int WM, int WN, int PT>
static int launch(const void* g_, const void* yv_, const float* al, const float* be, const float* ga,
                  const void* x_, const float* ps, const float* pt, float* garena, int64_t ldw, int64_t woff, int C,
                  int M, int pix_per_wg, const int* nimg, int hw, hipStream_t stream) {
  using T = typename P::T;
  const T* g = (const T*)g_;
  const T* yv = (const T*)yv_;
  const T* x = (const T*)x_;
  constexpr int WK = 4 / (WM * WN);
  const size_t vv = (size_t)(3 * COUT + 2 * CIN) * 4;
  const size_t tiles = (size_t)PT * (P::pitch_tr(COUT) + P::pitch_tr(CIN)) * P::ES;
  const size_t red = (size_t)(WK - 1) * (WM * WN) * (COUT / 16 / WM) * (CIN / 16 / WN) * 256 * 4;
  const size_t smem = vv + (tiles > red ? tiles : red);
  if (smem > 160 * 1024) return -5;
  auto kern = ps ? conv1x1_wgrad_kernel<P, CIN, COUT, 1, WM, WN, PT> : conv1x1_wgrad_kernel<P, CIN, COUT, 0, WM, WN, PT>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  const int gx = (M + pix_per_wg - 1) / pix_per_wg;
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(256), smem, stream, g, yv, al, be, ga, x, ps, pt, garena, ldw, woff, M,
                     pix_per_wg, nimg, hw, fa_take_lazy(0));
  return (int)hipGetLastError();
}

}  // namespace c1

// weight gradient of a 1×1 / stride-1 convolution, accumulated (+=) into the OIHW arena
// (cin must equal the stored weight's input channels). Returns < 0 for unsupported shapes.
template <class P>
static int conv1x1_wgrad(const void* g, const void* yv, const float* alpha, const float* beta, const float* gamma,
                         const void* x, const float* ps, const float* pt, float* garena, int64_t ldw, int64_t woff,
                         int C, int M, int Cin, int Cout, int pix_per_wg, const int* nimg, int hw,
                         hipStream_t stream) {
#define C1(CI, CO, WM, WN, PT)                                                                                 \
  if (Cin == CI && Cout == CO)                                                                                 \
    return c1::launch<P, CI, CO, WM, WN, PT>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, M,    \
                                             pix_per_wg, nimg, hw, stream);
  C1(16, 64, 1, 1, 128)    // 4 tiles: 4 pixel groups
  C1(64, 16, 1, 1, 128)
  C1(16, 16, 1, 1, 128)
  C1(32, 128, 2, 1, 128)   // 16 tiles: 2 co-groups × 2 pixel groups
  C1(128, 32, 1, 2, 128)
  C1(32, 32, 1, 1, 128)
  C1(64, 256, 4, 1, 64)    // 64 tiles: 4 co-groups (16 tiles per wave)
  C1(256, 64, 1, 4, 64)
  C1(64, 64, 2, 2, 128)
  C1(128, 128, 2, 2, 64)
  C1(64, 128, 2, 1, 128)
#undef C1
  return -2;
}

FA_EXPORT int fa_conv1x1_wgrad(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                               const float* gamma, const uint16_t* x, const float* ps, const float* pt, float* garena,
                               int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int pix_per_wg,
                               const int* nimg, int hw, hipStream_t stream) {
  return conv1x1_wgrad<c1::BF16>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, M, Cin, Cout, pix_per_wg,
                                 nimg, hw, stream);
}
FA_EXPORT int fa_conv1x1_wgrad_f32(const float* g, const float* yv, const float* alpha, const float* beta,
                                   const float* gamma, const float* x, const float* ps, const float* pt, float* garena,
                                   int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int pix_per_wg,
                                   const int* nimg, int hw, hipStream_t stream) {
  FA_F32_DISPATCH(c1, conv1x1_wgrad<PX>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, M, Cin, Cout, pix_per_wg,
                                nimg, hw, stream));
}

// ============================================================================================
// Fused backward of a 1×1 / stride-1 bottleneck convolution: data gradient (with the block
// epilogue of the generic kernel) AND weight gradient from ONE pass over the operands.
//
//   dy  = α·g + β·y + γ                                   (folded BN backward of this conv's BN)
//   dx  = dy · W                     → epilogue E (below) → out, statistics of the previous BN
//   dW += dyᵀ · act(e_x)             act = relu(e_x·s + t) (EPI_MASK) | e_x (EPI_BLOCK)
//
//   EPI_MASK  (conv2 of a block: dx feeds conv1's BN)  g' = dx·[e_x·s + t > 0];  Σg', Σg'·e_x
//   EPI_BLOCK (conv0: dx is the block-input gradient)  g' = (dx + e_add)·[e_x > 0];  Σg', Σg'·e_y1, Σg'·e_y2
//
// The separate kernels read g, y and e_x twice (once for dx, once for dW); here every pixel chunk
// is loaded once (register-prefetched one stage ahead), dy is formed once in LDS and feeds both
// MFMA products, and the dx tile goes through an LDS staging buffer so the epilogue runs on 16-B
// vectors in the same thread↔chunk mapping as the loads (the raw e_x chunk stays in registers).
// Reference parity: the backward of ResNet bottleneck blocks trained by the reference's
// ModelTrainerCLS (reference: python/fedml/model/cv/resnet.py Bottleneck, ml/trainer/my_model_trainer_classification.py).
// ============================================================================================
namespace c1f {
using prec::BF16;
using prec::F32;
using prec::F32X3;

struct Args {             // activations are P::T (bf16 | fp32)
  const void* g;          // [C][M][CO]
  const void* y;          // [C][M][CO]
  const float* alpha;     // [C][CO]
  const float* beta;
  const float* gamma;
  const void* wb;         // packed backward weights, client c at wb + c·wb_ld: [CI][roundup(CO, 32) + 8]
  int64_t wb_ld;
  const void* e_x;        // [C][M][CI]
  const float* e_s;       // [C][CI] (EPI_MASK)
  const float* e_t;
  const void* e_add;      // [C][M][CI] (EPI_BLOCK)
  const void* e_y1;
  const void* e_y2;       // optional
  void* out;              // [C][M][CI]
  float* stats;           // [C][CI][NS]
  int NS;
  float* garena;
  int64_t ldw, woff;
  int M, pix_per_wg;
  float* part;            // optional [C][G][CO·CI + 3·CI] per-workgroup partials (no atomics)
  const int* nimg;        // per-client valid images (null: all) and pixels per image
  int hw;
  const float* pivot;     // RY: [C][CO] shift K of the conv's forward output (y − K is what α, β, γ assume)
  const BnLazy* lz;       // deferred backward finalisation of this conv's BN (α, β, γ; bnlazy.h) or null
};

enum { EPI_MASK = 2, EPI_BLOCK = 3 };

// NW waves per workgroup: the weight-gradient accumulators (CO·CI fp32 per workgroup) are spread
// over NW waves, so the 64/256-channel layers use 8 waves to stay off the 256-VGPR cliff.
// LDS: dyL is read both ways (pixel fragments for dW, row fragments for dx), so it takes the
// frag_tr pitch and its row fragments are read 8-B aligned (P::frag_a8).
// RY (recomputed y, EPI_MASK, fp32 storage): the conv's forward output y is not stored — it is recomputed
// per stage from the staged act(e_x) tile (the conv input) and the weights already in LDS (wL holds Wᵀ:
// read transposed it is W), as y − K straight into the dy tile, which is then turned into dy in place.
// This replaces a 4·planes-channel read of y with MFMA work on data the kernel holds anyway.
template <class P, int CI, int CO, int EPI, int WM, int WN, int PT, int NW, bool RY = false>
__global__ __launch_bounds__(64 * NW) void conv1x1_bwd_kernel(Args a) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  constexpr int V = P::VEC;
  constexpr int NT = 64 * NW;
  constexpr int WK = NW / (WM * WN);
  constexpr int MTW = CO / 16 / WM, NTW = CI / 16 / WN;  // weight-gradient tiles per wave
  constexpr int KP = (CO + 31) / 32 * 32;            // dx GEMM depth (zero-padded to the MFMA K)
  // RY with CI < 32: the recompute GEMM's K is padded to 32 with zero columns of act(x) and zero rows of W
  constexpr int KCI = RY ? (CI + 31) / 32 * 32 : CI;
  // weight tile pitch: the packed global rows are KP + 8 long; in LDS the fp32 rows take KP + 4 (≡ 4 mod 8 dwords:
  // the 16 rows of a ds_read_b128 fragment read land on 16 distinct 4-bank groups — at KP + 8 rows r and r + 8
  // shared banks, a 2-way conflict on every dgrad B fragment); bf16 rows keep KP + 8 (already ≡ 4 mod 8 dwords)
  constexpr int LDWG = KP + 8, LDW = P::kF32 ? KP + 4 : KP + 8;
  constexpr int LDD = P::pitch_tr(KP), LDX = P::pitch_tr(KCI), LDS_ = P::pitch(CI);
  constexpr int DCH = PT * CO / V, XCH = PT * CI / V;
  constexpr int DI = (DCH + NT - 1) / NT, XI = (XCH + NT - 1) / NT;
  constexpr int MT = PT / 16;                       // dx row tiles per stage
  constexpr int MPW = MT >= NW ? MT / NW : 1;       // row tiles per wave
  constexpr int WPM = MT >= NW ? 1 : NW / MT;       // waves sharing a row tile (split columns)
  constexpr int NTX = CI / 16 / WPM;                // dx column tiles per wave
  constexpr int CGX = CI / V;                       // 16-B chunks per e_x row
  static_assert(WK >= 1 && NW % (WM * WN) == 0, "wave grid");
  static_assert((CI / 16) % WPM == 0 && NTX >= 1, "dx column split");
  static_assert(NT % CGX == 0, "fixed channel chunk per thread");
  static_assert(PT % 32 == 0 && (PT / 32) % WK == 0, "pixel k-steps per wave group");
  constexpr bool PRO = (EPI == EPI_MASK);
  constexpr bool BLK = (EPI == EPI_BLOCK);
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g4 = lane >> 4;
  const int kgrp = wid / (WM * WN), mgrp = (wid % (WM * WN)) / WN, ngrp = wid % WN;
  // workgroups past the client's valid pixels have nothing to add (the partial-sum mode still writes its
  // zero partials below)
  if (!a.part && (int)(blockIdx.x * a.pix_per_wg) >= (a.nimg ? min(a.M, a.nimg[c] * a.hw) : a.M)) return;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* vv = reinterpret_cast<float*>(smem);                            // α β γ [CO], s t [CI]
  T* wL = reinterpret_cast<T*>(vv + 3 * CO + 2 * CI + (RY ? CO : 0));    // [CI][LDW]
  T* sL = wL + KCI * LDW;                                                // [PT][LDS_] dx staging
  T* dyL = sL + PT * LDS_;                                               // [PT][LDD]
  T* xL = dyL + PT * LDD;                                                // [PT][LDX]  act(e_x)

  for (int i = threadIdx.x; i < CO; i += NT) {
    if (a.lz) {
      bn_lazy_bwd(a.lz, c, i, blockIdx.x == 0, vv[i], vv[CO + i], vv[2 * CO + i]);
    } else {
      vv[i] = a.alpha[(int64_t)c * CO + i];
      vv[CO + i] = a.beta[(int64_t)c * CO + i];
      vv[2 * CO + i] = a.gamma[(int64_t)c * CO + i];
    }
  }
  if (PRO)
    for (int i = threadIdx.x; i < CI; i += NT) {
      vv[3 * CO + i] = a.e_s[(int64_t)c * CI + i];
      vv[3 * CO + CI + i] = a.e_t[(int64_t)c * CI + i];
    }
  float* pivL = vv + 3 * CO + 2 * CI;   // RY: [CO] (the weight tile below starts after it)
  if (RY)
    for (int i = threadIdx.x; i < CO; i += NT) pivL[i] = a.pivot ? a.pivot[(int64_t)c * CO + i] : 0.f;
  {
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.wb) + (int64_t)c * a.wb_ld);
    uint4* dst = reinterpret_cast<uint4*>(wL);
    if (LDW == LDWG) {
      for (int i = threadIdx.x; i < CI * LDW / V; i += NT) dst[i] = src[i];
    } else {      // re-pitched rows (K padding columns are never read: fragments stop at KP)
      constexpr int RC = KP / V;   // 16-B chunks per row
      for (int i = threadIdx.x; i < CI * RC; i += NT) {
        const int r = i / RC, q = i - r * RC;
        dst[r * (LDW / V) + q] = src[r * (LDWG / V) + q];
      }
    }
  }
  if (KP > CO)  // zero K-padding columns of the dy tile (never rewritten by the stage stores)
    for (int i = threadIdx.x; i < PT * (KP - CO); i += NT) dyL[(i / (KP - CO)) * LDD + CO + i % (KP - CO)] = 0;
  if (KCI > CI) {   // RY, CI < 32: zero K padding of the recompute operands (never rewritten either)
    for (int i = threadIdx.x; i < (KCI - CI) * LDW; i += NT) wL[CI * LDW + i] = 0;
    for (int i = threadIdx.x; i < PT * (KCI - CI); i += NT) xL[(i / (KCI - CI)) * LDX + CI + i % (KCI - CI)] = 0;
  }

  const int M = a.M;
  const int Mc = a.nimg ? min(M, a.nimg[c] * a.hw) : M;   // this client's valid pixels
  const T* gc = reinterpret_cast<const T*>(a.g) + (int64_t)c * M * CO;
  const T* yc = reinterpret_cast<const T*>(a.y) + (int64_t)c * M * CO;
  const T* e_x = reinterpret_cast<const T*>(a.e_x);
  const T* e_add = reinterpret_cast<const T*>(a.e_add);
  const T* e_y1 = reinterpret_cast<const T*>(a.e_y1);
  const T* e_y2 = reinterpret_cast<const T*>(a.e_y2);
  T* outp = reinterpret_cast<T*>(a.out);
  const int64_t xbase = (int64_t)c * M * CI;
  const int p_begin = blockIdx.x * a.pix_per_wg;
  const int p_end = min(Mc, p_begin + a.pix_per_wg);
  const int ci0 = (threadIdx.x % CGX) * V;  // this thread's channel chunk in every e_x-shaped pass
  const bool has_y2 = BLK && e_y2 != nullptr;
  const bool has_y1 = BLK && e_y1 != nullptr;   // null: the previous BN's Σg·y comes from elsewhere

  // registers: next stage (r*) and current stage (e*) — every operand is fetched one stage ahead
  uint4 rg[DI], ry[DI], rx[XI], ra[XI], r1[XI], r2[XI];
  uint4 ex_[XI], ea[XI], e1[XI], e2[XI];
  auto load = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * NT;
      rg[it] = make_uint4(0, 0, 0, 0);
      ry[it] = make_uint4(0, 0, 0, 0);
      if (i < DCH) {
        const int p = p0 + i / (CO / V);
        if (p < p_end) {
          const int64_t off = (int64_t)p * CO + (i % (CO / V)) * V;
          rg[it] = *reinterpret_cast<const uint4*>(gc + off);
          if (!RY) ry[it] = *reinterpret_cast<const uint4*>(yc + off);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * NT;
      const int p = p0 + i / CGX;
      rx[it] = ra[it] = r1[it] = r2[it] = make_uint4(0, 0, 0, 0);
      if (i < XCH && p < p_end) {
        const int64_t off = xbase + (int64_t)p * CI + ci0;
        rx[it] = *reinterpret_cast<const uint4*>(e_x + off);
        if (BLK) {
          ra[it] = *reinterpret_cast<const uint4*>(e_add + off);
          if (has_y1) r1[it] = *reinterpret_cast<const uint4*>(e_y1 + off);
          if (has_y2) r2[it] = *reinterpret_cast<const uint4*>(e_y2 + off);
        }
      }
    }
  };
  auto form_dy = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * NT;
      if (i < DCH) {
        const int pp = i / (CO / V), co0 = (i % (CO / V)) * V;
        float gf[V], yf[V];
        P::unpack(rg[it], gf);
        if (RY) {   // y − K recomputed into this very chunk of the dy tile (8-B aligned rows)
          const uint2 lo = reinterpret_cast<const uint2*>(dyL + pp * LDD + co0)[0];
          const uint2 hi = reinterpret_cast<const uint2*>(dyL + pp * LDD + co0)[1];
          P::unpack(make_uint4(lo.x, lo.y, hi.x, hi.y), yf);
        } else {
          P::unpack(ry[it], yf);
        }
        const bool live = p0 + pp < p_end;
#pragma unroll
        for (int j = 0; j < V; ++j)
          gf[j] = live ? vv[co0 + j] * gf[j] + vv[CO + co0 + j] * yf[j] + vv[2 * CO + co0 + j] : 0.f;
        P::st_chunk(dyL + pp * LDD + co0, P::pack(gf));
      }
    }
  };
  // RY: y − K = act(x) · Wᵀ − K for the stage's PT pixels, one 16 × 16 tile per wave iteration
  auto recompute_y = [&]() {
    constexpr int NCT = CO / 16;
#pragma unroll 1
    for (int t = wid; t < (PT / 16) * NCT; t += NW) {
      const int mt = t / NCT, nt = t % NCT;
      f32x4 yacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < KCI; k0 += 32) {
        const frag_t af = P::frag_a8(xL + (mt * 16 + (lane & 15)) * LDX + k0 + 8 * g4);
        const frag_t bw = P::frag_tr(wL, LDW, k0, nt * 16, lane);
        yacc = P::mma(af, bw, yacc);
      }
      const int col = nt * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) dyL[(mt * 16 + 4 * g4 + i) * LDD + col] = P::from_f(yacc[i] - pivL[col]);
    }
  };
  auto store = [&](int p0) {
    if (!RY) form_dy(p0);
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * NT;
      ex_[it] = rx[it];
      if (BLK) { ea[it] = ra[it]; e1[it] = r1[it]; e2[it] = r2[it]; }
      if (i < XCH) {
        const int pp = i / CGX;
        uint4 v = rx[it];
        if (PRO && p0 + pp < p_end) {
          float f[V];
          P::unpack(v, f);
#pragma unroll
          for (int j = 0; j < V; ++j) f[j] = fmaxf(f[j] * vv[3 * CO + ci0 + j] + vv[3 * CO + CI + ci0 + j], 0.f);
          v = P::pack(f);
        }
        P::st_chunk(xL + pp * LDX + ci0, v);
      }
    }
    if (RY) {
      __syncthreads();   // act(x) staged
      recompute_y();
      __syncthreads();   // y − K staged
      form_dy(p0);
    }
  };

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = {0.f, 0.f, 0.f, 0.f};
  float st0[V], st1[V], st2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { st0[j] = 0.f; st1[j] = 0.f; st2[j] = 0.f; }

  __syncthreads();  // vectors + weights
  if (p_begin < p_end) load(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += PT) {
    store(p0);
    __syncthreads();
    if (p0 + PT < p_end) load(p0 + PT);
    // ---- weight gradient: acc += dyᵀ · act(x) over this stage's pixels ----
#pragma unroll
    for (int ks = kgrp; ks < PT / 32; ks += WK) {
      frag_t af[MTW], bfr[NTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) af[m] = P::frag_tr(dyL, LDD, ks * 32, (mgrp * MTW + m) * 16, lane);
#pragma unroll
      for (int n = 0; n < NTW; ++n) bfr[n] = P::frag_tr(xL, LDX, ks * 32, (ngrp * NTW + n) * 16, lane);
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n) acc[m][n] = P::mma(af[m], bfr[n], acc[m][n]);
    }
    // ---- data gradient: dx = dy · W, staged to LDS in storage precision ----
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi) {
      const int mt = MT >= NW ? wid + NW * mi : wid / WPM;
      const int n0 = MT >= NW ? 0 : (wid % WPM) * NTX;
      f32x4 dacc[NTX];
#pragma unroll
      for (int n = 0; n < NTX; ++n) dacc[n] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < KP; k0 += 32) {
        const frag_t af = P::frag_a8(dyL + (mt * 16 + (lane & 15)) * LDD + k0 + 8 * g4);
#pragma unroll
        for (int n = 0; n < NTX; ++n) {
          const frag_t bw = P::frag(wL + ((n0 + n) * 16 + (lane & 15)) * LDW + k0 + 8 * g4);
          dacc[n] = P::mma(af, bw, dacc[n]);
        }
      }
#pragma unroll
      for (int n = 0; n < NTX; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sL[(mt * 16 + 4 * g4 + i) * LDS_ + (n0 + n) * 16 + (lane & 15)] = P::from_f(dacc[n][i]);
    }
    __syncthreads();  // dx staged; dyL / xL free for the next stage
    // ---- epilogue on 16-B chunks (same mapping as the e_x loads) ----
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * NT;
      const int pp = i / CGX;
      if (i < XCH && p0 + pp < p_end) {
        float gv[V], xv[V];
        P::unpack(*reinterpret_cast<const uint4*>(sL + pp * LDS_ + ci0), gv);
        P::unpack(ex_[it], xv);
        if (PRO) {
#pragma unroll
          for (int j = 0; j < V; ++j)
            gv[j] = (xv[j] * vv[3 * CO + ci0 + j] + vv[3 * CO + CI + ci0 + j] > 0.f) ? gv[j] : 0.f;
        } else {
          float ex[V];
          P::unpack(ea[it], ex);
#pragma unroll
          for (int j = 0; j < V; ++j) gv[j] = (xv[j] > 0.f) ? gv[j] + ex[j] : 0.f;
        }
        const uint4 gp = P::pack(gv);
        *reinterpret_cast<uint4*>(outp + xbase + (int64_t)(p0 + pp) * CI + ci0) = gp;
        float gr[V];
        P::unpack(gp, gr);
        if (PRO) {
#pragma unroll
          for (int j = 0; j < V; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * xv[j]; }
        } else {
          float y1[V], y2[V];
          P::unpack(e1[it], y1);
          P::unpack(e2[it], y2);
#pragma unroll
          for (int j = 0; j < V; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * y1[j]; st2[j] += gr[j] * y2[j]; }
        }
      }
    }
  }

  // ---- statistics: lanes sharing a chunk (shuffles), then waves (LDS) ----
#pragma unroll
  for (int o = CGX; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      st0[j] += __shfl_xor(st0[j], o, 64);
      st1[j] += __shfl_xor(st1[j], o, 64);
      if (BLK) st2[j] += __shfl_xor(st2[j], o, 64);
    }
  }
  __syncthreads();  // every wave is past its last epilogue: the tile region is free
  float* sred = reinterpret_cast<float*>(sL);  // [NW][CI][3]
  if (lane < CGX) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sred[(wid * CI + ci0 + j) * 3 + 0] = st0[j];
      sred[(wid * CI + ci0 + j) * 3 + 1] = st1[j];
      sred[(wid * CI + ci0 + j) * 3 + 2] = st2[j];
    }
  }
  __syncthreads();
  const int64_t E = (int64_t)CO * CI + 3 * CI;
  float* mypart = a.part ? a.part + ((int64_t)c * gridDim.x + blockIdx.x) * E : nullptr;
  for (int i = threadIdx.x; i < 3 * CI; i += NT) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += sred[w * CI * 3 + i];
    if (mypart) {
      mypart[(int64_t)CO * CI + i] = v;
    } else if (p_begin < p_end && (i % 3 < 2 || has_y2)) {
      fa_acc_add(a.stats + (int64_t)c * CI * a.NS + (i / 3) * a.NS + i % 3, v);
    }
  }

  // ---- weight gradient: reduce pixel groups through LDS, then partials or atomics ----
  if (WK > 1) {
    __syncthreads();
    float* rbuf = reinterpret_cast<float*>(sL);
    if (kgrp > 0) {
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            rbuf[((((kgrp - 1) * (WM * WN) + mgrp * WN + ngrp) * MTW + m) * NTW + n) * 256 + i * 64 + lane] =
                acc[m][n][i];
    }
    __syncthreads();
    if (kgrp == 0)
      for (int k2 = 1; k2 < WK; ++k2)
#pragma unroll
        for (int m = 0; m < MTW; ++m)
#pragma unroll
          for (int n = 0; n < NTW; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[m][n][i] += rbuf[((((k2 - 1) * (WM * WN) + mgrp * WN + ngrp) * MTW + m) * NTW + n) * 256 + i * 64 + lane];
  }
  if (kgrp == 0) {
    float* gw = a.garena + (int64_t)c * a.ldw + a.woff;
#pragma unroll
    for (int m = 0; m < MTW; ++m)
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const int ci = (ngrp * NTW + n) * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = (mgrp * MTW + m) * 16 + 4 * g4 + i;
          if (mypart)
            mypart[(int64_t)co * CI + ci] = acc[m][n][i];
          else if (p_begin < p_end)
            fa_acc_add(&gw[(int64_t)co * CI + ci], acc[m][n][i]);
        }
      }
  }
}

// second pass of the partial-sum mode: Σ over the G workgroups of a client, added (single writer
// per element, deterministic order) into the OIHW arena rows and the [C][CI][NS] statistics.
__global__ __launch_bounds__(256) void partial_reduce_kernel(const float* __restrict__ part, int G, int CO, int CI,
                                                             float* __restrict__ garena, int64_t ldw, int64_t woff,
                                                             float* __restrict__ stats, int NS, int has_q2) {
  const int c = blockIdx.y;
  const int64_t E = (int64_t)CO * CI + 3 * CI;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  const float* p = part + (int64_t)c * G * E + e;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int g = 0;
  for (; g + 4 <= G; g += 4) {
    s0 += p[(int64_t)g * E];
    s1 += p[(int64_t)(g + 1) * E];
    s2 += p[(int64_t)(g + 2) * E];
    s3 += p[(int64_t)(g + 3) * E];
  }
  for (; g < G; ++g) s0 += p[(int64_t)g * E];
  const float v = (s0 + s1) + (s2 + s3);
  if (e < (int64_t)CO * CI) {
    garena[(int64_t)c * ldw + woff + e] += v;
  } else {
    const int i = (int)(e - (int64_t)CO * CI);
    const int ci = i / 3, q = i % 3;
    if (q < 2 || has_q2) stats[((int64_t)c * CI + ci) * NS + q] += v;
  }
}

template <class P, int CI, int CO, int EPI, int WM, int WN, int PT, int NW, bool RY = false>
static int launch(const Args& a, int C, hipStream_t stream) {
  constexpr int WK = NW / (WM * WN);
  constexpr int KP = (CO + 31) / 32 * 32;
  constexpr int KCI = RY ? (CI + 31) / 32 * 32 : CI;
  const size_t vv = (size_t)(3 * CO + 2 * CI + (RY ? CO : 0)) * 4;
  const size_t wl = (size_t)KCI * (KP + 8) * P::ES;
  const size_t stage = (size_t)PT * P::pitch(CI) * P::ES;
  const size_t tiles = (size_t)PT * (P::pitch_tr(KP) + P::pitch_tr(KCI)) * P::ES;
  const size_t red = (size_t)(WK - 1) * (WM * WN) * (CO / 16 / WM) * (CI / 16 / WN) * 256 * 4;
  const size_t sred = (size_t)NW * CI * 3 * 4;
  size_t region = stage + tiles;   // the reduction buffers reuse the stage + tile region
  region = region > red ? region : red;
  region = region > sred ? region : sred;
  const size_t smem = vv + wl + region;
  if (smem > 160 * 1024) return -5;
  if (a.NS < 2 || (EPI == EPI_BLOCK && a.e_y2 && a.NS < 3)) return -4;
  auto kern = conv1x1_bwd_kernel<P, CI, CO, EPI, WM, WN, PT, NW, RY>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  const int gx = (a.M + a.pix_per_wg - 1) / a.pix_per_wg;
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(64 * NW), smem, stream, a);
  if (a.part) {
    const int64_t E = (int64_t)CO * CI + 3 * CI;
    hipLaunchKernelGGL(partial_reduce_kernel, dim3((unsigned)((E + 255) / 256), C), dim3(256), 0, stream, a.part, gx,
                       CO, CI, a.garena, a.ldw, a.woff, a.stats, a.NS, (EPI == EPI_BLOCK && a.e_y2) ? 1 : 0);
  }
  return (int)hipGetLastError();
}

template <class P>
static int bwd_fused(const void* g, const void* y, const float* alpha, const float* beta, const float* gamma,
                     const void* wb, int64_t wb_ld, int ldk2, const void* e_x, const float* e_s, const float* e_t,
                     const void* e_add, const void* e_y1, const void* e_y2, void* out, float* stats, int NS,
                     float* garena, int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int epi,
                     int pix_per_wg, float* part, const int* nimg, int hw, const float* pivot, hipStream_t stream) {
  if (ldk2 != (Cout + 31) / 32 * 32 + 8 || pix_per_wg <= 0) return -3;
  if (epi == EPI_MASK && (!e_s || !e_t)) return -4;
  if (epi == EPI_BLOCK && !e_add) return -4;
  // y == null: recompute y from the staged input (EPI_MASK, fp32 storage only)
  if (!y && (epi != EPI_MASK || !P::kF32)) return -4;
  Args a{g, y, alpha, beta, gamma, wb, wb_ld, e_x, e_s, e_t, e_add, e_y1, e_y2, out, stats, NS, garena, ldw,
         woff, M, pix_per_wg, part, nimg, hw, pivot, fa_take_lazy(0)};
#define C1F(CI, CO, E, WM, WN, PT, NW)                                              \
  if (Cin == CI && Cout == CO && epi == E) {                                       \
    if constexpr (E == EPI_MASK && P::kF32)                                        \
      if (!y) return launch<P, CI, CO, E, WM, WN, PT, NW, true>(a, C, stream);     \
    return launch<P, CI, CO, E, WM, WN, PT, NW>(a, C, stream);                     \
  }
  // conv2 of a bottleneck (planes → 4·planes): mask epilogue, BN-ReLU prologue on the wgrad operand
  C1F(16, 64, 2, 2, 1, 64, 4)
  C1F(32, 128, 2, 4, 1, 64, 4)
  C1F(64, 256, 2, 8, 1, 32, 8)
  // conv0 (in → planes): block epilogue
  C1F(64, 16, 3, 1, 2, 64, 4)
  C1F(128, 32, 3, 1, 8, 64, 8)
  C1F(256, 64, 3, 1, 8, 32, 8)
  C1F(16, 16, 3, 1, 1, 128, 4)
  C1F(64, 32, 3, 1, 4, 64, 4)
  C1F(128, 64, 3, 2, 4, 32, 8)
#undef C1F
  return -2;
}

}  // namespace c1f

// fused data + weight gradient of a 1×1 / stride-1 bottleneck convolution (Cin = dx channels,
// Cout = g channels). epi: 2 = BN-ReLU mask epilogue, 3 = block epilogue. With ``part`` (≥ C·G·
// (Cout·Cin + 3·Cin) floats, G = ceil(M / pix_per_wg)) the per-workgroup weight-gradient and
// statistics partials are written out and summed by a second pass instead of fp32 atomics:
// cheaper at many workgroups (atomic contention on the CO·CI addresses) and deterministic.
// Returns < 0 for unsupported shapes / arguments. `_f32`: fp32 activations / packed weights.
FA_EXPORT int fa_conv1x1_bwd_fused(const uint16_t* g, const uint16_t* y, const float* alpha, const float* beta,
                                   const float* gamma, const uint16_t* wb, int64_t wb_ld, int ldk2, const uint16_t* e_x,
                                   const float* e_s, const float* e_t, const uint16_t* e_add, const uint16_t* e_y1,
                                   const uint16_t* e_y2, uint16_t* out, float* stats, int NS, float* garena,
                                   int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int epi, int pix_per_wg,
                                   float* part, const int* nimg, int hw, hipStream_t stream) {
  return c1f::bwd_fused<c1f::BF16>(g, y, alpha, beta, gamma, wb, wb_ld, ldk2, e_x, e_s, e_t, e_add, e_y1, e_y2, out,
                                   stats, NS, garena, ldw, woff, C, M, Cin, Cout, epi, pix_per_wg, part, nimg, hw,
                                   nullptr, stream);
}
FA_EXPORT int fa_conv1x1_bwd_fused_f32(const float* g, const float* y, const float* alpha, const float* beta,
                                       const float* gamma, const float* wb, int64_t wb_ld, int ldk2, const float* e_x,
                                       const float* e_s, const float* e_t, const float* e_add, const float* e_y1,
                                       const float* e_y2, float* out, float* stats, int NS, float* garena,
                                       int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int epi,
                                       int pix_per_wg, float* part, const int* nimg, int hw, hipStream_t stream) {
  FA_F32_DISPATCH(c1f, c1f::bwd_fused<PX>(g, y, alpha, beta, gamma, wb, wb_ld, ldk2, e_x, e_s, e_t, e_add, e_y1, e_y2, out,
                                  stats, NS, garena, ldw, woff, C, M, Cin, Cout, epi, pix_per_wg, part, nimg, hw,
                                  nullptr, stream));
}
// recomputed-y variant (EPI_MASK): `y` is not read — y − pivot is rebuilt from e_x and the weights
FA_EXPORT int fa_conv1x1_bwd_fused_ry_f32(const float* g, const float* alpha, const float* beta, const float* gamma,
                                          const float* pivot, const float* wb, int64_t wb_ld, int ldk2,
                                          const float* e_x, const float* e_s, const float* e_t, float* out,
                                          float* stats, int NS, float* garena, int64_t ldw, int64_t woff, int C, int M,
                                          int Cin, int Cout, int pix_per_wg, float* part, const int* nimg, int hw,
                                          hipStream_t stream) {
  FA_F32_DISPATCH(c1f, c1f::bwd_fused<PX>(g, nullptr, alpha, beta, gamma, wb, wb_ld, ldk2, e_x, e_s, e_t, nullptr,
                                  nullptr, nullptr, out, stats, NS, garena, ldw, woff, C, M, Cin, Cout, c1f::EPI_MASK,
                                  pix_per_wg, part, nimg, hw, pivot, stream));
}
