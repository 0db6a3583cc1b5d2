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
#include "common.h"

namespace c1 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ void unpack8(uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = (uint32_t)f32_to_bf16(f[0]) | ((uint32_t)f32_to_bf16(f[1]) << 16);
  r.y = (uint32_t)f32_to_bf16(f[2]) | ((uint32_t)f32_to_bf16(f[3]) << 16);
  r.z = (uint32_t)f32_to_bf16(f[4]) | ((uint32_t)f32_to_bf16(f[5]) << 16);
  r.w = (uint32_t)f32_to_bf16(f[6]) | ((uint32_t)f32_to_bf16(f[7]) << 16);
  return r;
}
__device__ __forceinline__ bf16x8 tr_read(const uint16_t* a0, int ld4) {
  const v4i16 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  const v4i16 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0 + ld4));
  union { short s[8]; bf16x8 b; } u;
  u.s[0] = r0[0]; u.s[1] = r0[1]; u.s[2] = r0[2]; u.s[3] = r0[3];
  u.s[4] = r1[0]; u.s[5] = r1[1]; u.s[6] = r1[2]; u.s[7] = r1[3];
  return u.b;
}

// WM × WN waves tile the (COUT/16) × (CIN/16) output tiles; WK = 4/(WM·WN) waves split the pixels.
template <int CIN, int COUT, int PRO, int WM, int WN, int PT>
__global__ __launch_bounds__(256) void conv1x1_wgrad_kernel(const uint16_t* __restrict__ g,
                                                            const uint16_t* __restrict__ yv,
                                                            const float* __restrict__ alpha,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ gamma,
                                                            const uint16_t* __restrict__ x,
                                                            const float* __restrict__ ps, const float* __restrict__ pt,
                                                            float* __restrict__ garena, int64_t ldw, int64_t woff,
                                                            int M, int pix_per_wg) {
  constexpr int WK = 4 / (WM * WN);
  constexpr int MTW = COUT / 16 / WM, NTW = CIN / 16 / WN;
  constexpr int LDD = COUT + 8, LDX = CIN + 8;
  constexpr int DCH = PT * COUT / 8, XCH = PT * CIN / 8;            // 16-B chunks per stage
  constexpr int DI = (DCH + 255) / 256, XI = (XCH + 255) / 256;    // per thread
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int kgrp = wid / (WM * WN), mgrp = (wid % (WM * WN)) / WN, ngrp = wid % WN;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* vv = reinterpret_cast<float*>(smem);                              // α β γ [COUT], s t [CIN]
  uint16_t* dyL = reinterpret_cast<uint16_t*>(vv + 3 * COUT + 2 * CIN);    // [PT][LDD]
  uint16_t* xL = dyL + PT * LDD;                                           // [PT][LDX]

  for (int i = threadIdx.x; i < COUT; i += 256) {
    vv[i] = alpha[(int64_t)c * COUT + i];
    vv[COUT + i] = beta[(int64_t)c * COUT + i];
    vv[2 * COUT + i] = gamma[(int64_t)c * COUT + i];
  }
  if (PRO)
    for (int i = threadIdx.x; i < CIN; i += 256) {
      vv[3 * COUT + i] = ps[(int64_t)c * CIN + i];
      vv[3 * COUT + CIN + i] = pt[(int64_t)c * CIN + i];
    }

  const uint16_t* gc = g + (int64_t)c * M * COUT;
  const uint16_t* yc = yv + (int64_t)c * M * COUT;
  const uint16_t* xc = x + (int64_t)c * M * CIN;
  const int p_begin = blockIdx.x * pix_per_wg;
  const int p_end = min(M, p_begin + pix_per_wg);

  uint4 rg[DI], ry[DI], rx[XI];
  auto load = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * 256;
      rg[it] = make_uint4(0, 0, 0, 0);
      ry[it] = make_uint4(0, 0, 0, 0);
      if (i < DCH) {
        const int p = p0 + i / (COUT / 8);
        if (p < p_end) {
          const int64_t off = (int64_t)p * COUT + (i % (COUT / 8)) * 8;
          rg[it] = *reinterpret_cast<const uint4*>(gc + off);
          ry[it] = *reinterpret_cast<const uint4*>(yc + off);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * 256;
      rx[it] = make_uint4(0, 0, 0, 0);
      if (i < XCH) {
        const int p = p0 + i / (CIN / 8);
        if (p < p_end) rx[it] = *reinterpret_cast<const uint4*>(xc + (int64_t)p * CIN + (i % (CIN / 8)) * 8);
      }
    }
  };
  auto store = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < DCH) {
        const int pp = i / (COUT / 8), co0 = (i % (COUT / 8)) * 8;
        float gf[8], yf[8];
        unpack8(rg[it], gf);
        unpack8(ry[it], yf);
        const bool live = p0 + pp < p_end;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          gf[j] = live ? vv[co0 + j] * gf[j] + vv[COUT + co0 + j] * yf[j] + vv[2 * COUT + co0 + j] : 0.f;
        *reinterpret_cast<uint4*>(dyL + pp * LDD + co0) = pack8(gf);
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < XCH) {
        const int pp = i / (CIN / 8), ci0 = (i % (CIN / 8)) * 8;
        uint4 v = rx[it];
        if (PRO && p0 + pp < p_end) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j] * vv[3 * COUT + ci0 + j] + vv[3 * COUT + CIN + ci0 + j], 0.f);
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(xL + pp * LDX + ci0) = v;
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
      const int row = ks * 32 + 8 * g4 + q;
      bf16x8 af[MTW], bfr[NTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) af[m] = tr_read(dyL + row * LDD + (mgrp * MTW + m) * 16 + 4 * pq, 4 * LDD);
#pragma unroll
      for (int n = 0; n < NTW; ++n) bfr[n] = tr_read(xL + row * LDX + (ngrp * NTW + n) * 16 + 4 * pq, 4 * LDX);
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
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
          atomicAdd(&gw[(int64_t)co * CIN + ci], acc[m][n][i]);
        }
      }
  }
}

template <int CIN, int COUT, int WM, int WN, int PT>
static int launch(const uint16_t* g, const uint16_t* yv, const float* al, const float* be, const float* ga,
                  const uint16_t* x, const float* ps, const float* pt, float* garena, int64_t ldw, int64_t woff, int C,
                  int M, int pix_per_wg, hipStream_t stream) {
  constexpr int WK = 4 / (WM * WN);
  const size_t vv = (size_t)(3 * COUT + 2 * CIN) * 4;
  const size_t tiles = (size_t)PT * ((COUT + 8) + (CIN + 8)) * 2;
  const size_t red = (size_t)(WK - 1) * (WM * WN) * (COUT / 16 / WM) * (CIN / 16 / WN) * 256 * 4;
  const size_t smem = vv + (tiles > red ? tiles : red);
  if (smem > 160 * 1024) return -5;
  auto kern = ps ? conv1x1_wgrad_kernel<CIN, COUT, 1, WM, WN, PT> : conv1x1_wgrad_kernel<CIN, COUT, 0, WM, WN, PT>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  const int gx = (M + pix_per_wg - 1) / pix_per_wg;
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(256), smem, stream, g, yv, al, be, ga, x, ps, pt, garena, ldw, woff, M,
                     pix_per_wg);
  return (int)hipGetLastError();
}

}  // namespace c1

// weight gradient of a 1×1 / stride-1 convolution, accumulated (+=) into the OIHW arena
// (cin must equal the stored weight's input channels). Returns < 0 for unsupported shapes.
FA_EXPORT int fa_conv1x1_wgrad(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                               const float* gamma, const uint16_t* x, const float* ps, const float* pt, float* garena,
                               int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int pix_per_wg,
                               hipStream_t stream) {
#define C1(CI, CO, WM, WN, PT)                                                                                 \
  if (Cin == CI && Cout == CO)                                                                                 \
    return c1::launch<CI, CO, WM, WN, PT>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, M,       \
                                          pix_per_wg, stream);
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
using c1::bf16x8;
using c1::pack8;
using c1::tr_read;
using c1::unpack8;

struct Args {
  const uint16_t* g;      // [C][M][CO]
  const uint16_t* y;      // [C][M][CO]
  const float* alpha;     // [C][CO]
  const float* beta;
  const float* gamma;
  const uint16_t* wb;     // packed backward weights, client c at wb + c·wb_ld: [CI][roundup(CO, 32) + 8]
  int64_t wb_ld;
  const uint16_t* e_x;    // [C][M][CI]
  const float* e_s;       // [C][CI] (EPI_MASK)
  const float* e_t;
  const uint16_t* e_add;  // [C][M][CI] (EPI_BLOCK)
  const uint16_t* e_y1;
  const uint16_t* e_y2;   // optional
  uint16_t* out;          // [C][M][CI]
  float* stats;           // [C][CI][NS]
  int NS;
  float* garena;
  int64_t ldw, woff;
  int M, pix_per_wg;
  float* part;            // optional [C][G][CO·CI + 3·CI] per-workgroup partials (no atomics)
};

enum { EPI_MASK = 2, EPI_BLOCK = 3 };

// NW waves per workgroup: the weight-gradient accumulators (CO·CI fp32 per workgroup) are spread
// over NW waves, so the 64/256-channel layers use 8 waves to stay off the 256-VGPR cliff.
template <int CI, int CO, int EPI, int WM, int WN, int PT, int NW>
__global__ __launch_bounds__(64 * NW) void conv1x1_bwd_kernel(Args a) {
  constexpr int NT = 64 * NW;
  constexpr int WK = NW / (WM * WN);
  constexpr int MTW = CO / 16 / WM, NTW = CI / 16 / WN;  // weight-gradient tiles per wave
  constexpr int KP = (CO + 31) / 32 * 32;            // dx GEMM depth (zero-padded to the MFMA K)
  constexpr int LDD = KP + 8, LDX = CI + 8, LDW = KP + 8;
  constexpr int DCH = PT * CO / 8, XCH = PT * CI / 8;
  constexpr int DI = (DCH + NT - 1) / NT, XI = (XCH + NT - 1) / NT;
  constexpr int MT = PT / 16;                       // dx row tiles per stage
  constexpr int MPW = MT >= NW ? MT / NW : 1;       // row tiles per wave
  constexpr int WPM = MT >= NW ? 1 : NW / MT;       // waves sharing a row tile (split columns)
  constexpr int NTX = CI / 16 / WPM;                // dx column tiles per wave
  constexpr int CGX = CI / 8;                       // 16-B chunks per e_x row
  static_assert(WK >= 1 && NW % (WM * WN) == 0, "wave grid");
  static_assert((CI / 16) % WPM == 0 && NTX >= 1, "dx column split");
  static_assert(NT % CGX == 0, "fixed channel chunk per thread");
  static_assert(PT % 32 == 0 && (PT / 32) % WK == 0, "pixel k-steps per wave group");
  constexpr bool PRO = (EPI == EPI_MASK);
  constexpr bool BLK = (EPI == EPI_BLOCK);
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int kgrp = wid / (WM * WN), mgrp = (wid % (WM * WN)) / WN, ngrp = wid % WN;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* vv = reinterpret_cast<float*>(smem);                            // α β γ [CO], s t [CI]
  uint16_t* wL = reinterpret_cast<uint16_t*>(vv + 3 * CO + 2 * CI);      // [CI][LDW]
  uint16_t* dyL = wL + CI * LDW;                                         // [PT][LDD]
  uint16_t* xL = dyL + PT * LDD;                                         // [PT][LDX]  act(e_x)
  uint16_t* sL = xL + PT * LDX;                                          // [PT][LDX]  dx staging

  for (int i = threadIdx.x; i < CO; i += NT) {
    vv[i] = a.alpha[(int64_t)c * CO + i];
    vv[CO + i] = a.beta[(int64_t)c * CO + i];
    vv[2 * CO + i] = a.gamma[(int64_t)c * CO + i];
  }
  if (PRO)
    for (int i = threadIdx.x; i < CI; i += NT) {
      vv[3 * CO + i] = a.e_s[(int64_t)c * CI + i];
      vv[3 * CO + CI + i] = a.e_t[(int64_t)c * CI + i];
    }
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.wb + (int64_t)c * a.wb_ld);
    uint4* dst = reinterpret_cast<uint4*>(wL);
    for (int i = threadIdx.x; i < CI * LDW / 8; i += NT) dst[i] = src[i];
  }
  if (KP > CO)  // zero K-padding columns of the dy tile (never rewritten by the stage stores)
    for (int i = threadIdx.x; i < PT * (KP - CO); i += NT) dyL[(i / (KP - CO)) * LDD + CO + i % (KP - CO)] = 0;

  const int M = a.M;
  const uint16_t* gc = a.g + (int64_t)c * M * CO;
  const uint16_t* yc = a.y + (int64_t)c * M * CO;
  const int64_t xbase = (int64_t)c * M * CI;
  const int p_begin = blockIdx.x * a.pix_per_wg;
  const int p_end = min(M, p_begin + a.pix_per_wg);
  const int ci0 = (threadIdx.x % CGX) * 8;  // this thread's channel chunk in every e_x-shaped pass
  const bool has_y2 = BLK && a.e_y2 != nullptr;

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
        const int p = p0 + i / (CO / 8);
        if (p < p_end) {
          const int64_t off = (int64_t)p * CO + (i % (CO / 8)) * 8;
          rg[it] = *reinterpret_cast<const uint4*>(gc + off);
          ry[it] = *reinterpret_cast<const uint4*>(yc + off);
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
        rx[it] = *reinterpret_cast<const uint4*>(a.e_x + off);
        if (BLK) {
          ra[it] = *reinterpret_cast<const uint4*>(a.e_add + off);
          r1[it] = *reinterpret_cast<const uint4*>(a.e_y1 + off);
          if (has_y2) r2[it] = *reinterpret_cast<const uint4*>(a.e_y2 + off);
        }
      }
    }
  };
  auto store = [&](int p0) {
#pragma unroll
    for (int it = 0; it < DI; ++it) {
      const int i = threadIdx.x + it * NT;
      if (i < DCH) {
        const int pp = i / (CO / 8), co0 = (i % (CO / 8)) * 8;
        float gf[8], yf[8];
        unpack8(rg[it], gf);
        unpack8(ry[it], yf);
        const bool live = p0 + pp < p_end;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          gf[j] = live ? vv[co0 + j] * gf[j] + vv[CO + co0 + j] * yf[j] + vv[2 * CO + co0 + j] : 0.f;
        *reinterpret_cast<uint4*>(dyL + pp * LDD + co0) = pack8(gf);
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * NT;
      ex_[it] = rx[it];
      if (BLK) { ea[it] = ra[it]; e1[it] = r1[it]; e2[it] = r2[it]; }
      if (i < XCH) {
        const int pp = i / CGX;
        uint4 v = rx[it];
        if (PRO && p0 + pp < p_end) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j] * vv[3 * CO + ci0 + j] + vv[3 * CO + CI + ci0 + j], 0.f);
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(xL + pp * LDX + ci0) = v;
      }
    }
  };

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = {0.f, 0.f, 0.f, 0.f};
  float st0[8], st1[8], st2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st0[j] = 0.f; st1[j] = 0.f; st2[j] = 0.f; }

  __syncthreads();  // vectors + weights
  if (p_begin < p_end) load(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += PT) {
    store(p0);
    __syncthreads();
    if (p0 + PT < p_end) load(p0 + PT);
    // ---- weight gradient: acc += dyᵀ · act(x) over this stage's pixels ----
#pragma unroll
    for (int ks = kgrp; ks < PT / 32; ks += WK) {
      const int row = ks * 32 + 8 * g4 + q;
      bf16x8 af[MTW], bfr[NTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) af[m] = tr_read(dyL + row * LDD + (mgrp * MTW + m) * 16 + 4 * pq, 4 * LDD);
#pragma unroll
      for (int n = 0; n < NTW; ++n) bfr[n] = tr_read(xL + row * LDX + (ngrp * NTW + n) * 16 + 4 * pq, 4 * LDX);
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
    // ---- data gradient: dx = dy · W, staged to LDS as bf16 ----
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi) {
      const int mt = MT >= NW ? wid + NW * mi : wid / WPM;
      const int n0 = MT >= NW ? 0 : (wid % WPM) * NTX;
      f32x4 dacc[NTX];
#pragma unroll
      for (int n = 0; n < NTX; ++n) dacc[n] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < KP; k0 += 32) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(dyL + (mt * 16 + (lane & 15)) * LDD + k0 + 8 * g4);
#pragma unroll
        for (int n = 0; n < NTX; ++n) {
          const bf16x8 bw = *reinterpret_cast<const bf16x8*>(wL + ((n0 + n) * 16 + (lane & 15)) * LDW + k0 + 8 * g4);
          dacc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw, dacc[n], 0, 0, 0);
        }
      }
#pragma unroll
      for (int n = 0; n < NTX; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sL[(mt * 16 + 4 * g4 + i) * LDX + (n0 + n) * 16 + (lane & 15)] = f32_to_bf16(dacc[n][i]);
    }
    __syncthreads();  // dx staged; dyL / xL free for the next stage
    // ---- epilogue on 16-B chunks (same mapping as the e_x loads) ----
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int i = threadIdx.x + it * NT;
      const int pp = i / CGX;
      if (i < XCH && p0 + pp < p_end) {
        float gv[8], xv[8];
        unpack8(*reinterpret_cast<const uint4*>(sL + pp * LDX + ci0), gv);
        unpack8(ex_[it], xv);
        if (PRO) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            gv[j] = (xv[j] * vv[3 * CO + ci0 + j] + vv[3 * CO + CI + ci0 + j] > 0.f) ? gv[j] : 0.f;
        } else {
          float ex[8];
          unpack8(ea[it], ex);
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] = (xv[j] > 0.f) ? gv[j] + ex[j] : 0.f;
        }
        const uint4 gp = pack8(gv);
        *reinterpret_cast<uint4*>(a.out + xbase + (int64_t)(p0 + pp) * CI + ci0) = gp;
        float gr[8];
        unpack8(gp, gr);
        if (PRO) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * xv[j]; }
        } else {
          float y1[8], y2[8];
          unpack8(e1[it], y1);
          unpack8(e2[it], y2);
#pragma unroll
          for (int j = 0; j < 8; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * y1[j]; st2[j] += gr[j] * y2[j]; }
        }
      }
    }
  }

  // ---- statistics: lanes sharing a chunk (shuffles), then waves (LDS) ----
#pragma unroll
  for (int o = CGX; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      st0[j] += __shfl_xor(st0[j], o, 64);
      st1[j] += __shfl_xor(st1[j], o, 64);
      if (BLK) st2[j] += __shfl_xor(st2[j], o, 64);
    }
  }
  __syncthreads();  // every wave is past its last epilogue: the tile region is free
  float* sred = reinterpret_cast<float*>(dyL);  // [NW][CI][3]
  if (lane < CGX) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
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
      atomicAdd(a.stats + (int64_t)c * CI * a.NS + (i / 3) * a.NS + i % 3, v);
    }
  }

  // ---- weight gradient: reduce pixel groups through LDS, then partials or atomics ----
  if (WK > 1) {
    __syncthreads();
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
            atomicAdd(&gw[(int64_t)co * CI + ci], acc[m][n][i]);
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

template <int CI, int CO, int EPI, int WM, int WN, int PT, int NW>
static int launch(const Args& a, int C, hipStream_t stream) {
  constexpr int WK = NW / (WM * WN);
  constexpr int KP = (CO + 31) / 32 * 32;
  const size_t vv = (size_t)(3 * CO + 2 * CI) * 4;
  const size_t wl = (size_t)CI * (KP + 8) * 2;
  const size_t tiles = (size_t)PT * ((KP + 8) + 2 * (CI + 8)) * 2;
  const size_t red = (size_t)(WK - 1) * (WM * WN) * (CO / 16 / WM) * (CI / 16 / WN) * 256 * 4;
  const size_t sred = (size_t)NW * CI * 3 * 4;
  size_t region = tiles > red ? tiles : red;
  region = region > sred ? region : sred;
  const size_t smem = vv + wl + region;
  if (smem > 160 * 1024) return -5;
  if (a.NS < 2 || (EPI == EPI_BLOCK && a.e_y2 && a.NS < 3)) return -4;
  auto kern = conv1x1_bwd_kernel<CI, CO, EPI, WM, WN, PT, NW>;
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

}  // namespace c1f

// fused data + weight gradient of a 1×1 / stride-1 bottleneck convolution (Cin = dx channels,
// Cout = g channels). epi: 2 = BN-ReLU mask epilogue, 3 = block epilogue. With ``part`` (≥ C·G·
// (Cout·Cin + 3·Cin) floats, G = ceil(M / pix_per_wg)) the per-workgroup weight-gradient and
// statistics partials are written out and summed by a second pass instead of fp32 atomics:
// cheaper at many workgroups (atomic contention on the CO·CI addresses) and deterministic.
// Returns < 0 for unsupported shapes / arguments.
FA_EXPORT int fa_conv1x1_bwd_fused(const uint16_t* g, const uint16_t* y, const float* alpha, const float* beta,
                                   const float* gamma, const uint16_t* wb, int64_t wb_ld, int ldk2, const uint16_t* e_x,
                                   const float* e_s, const float* e_t, const uint16_t* e_add, const uint16_t* e_y1,
                                   const uint16_t* e_y2, uint16_t* out, float* stats, int NS, float* garena,
                                   int64_t ldw, int64_t woff, int C, int M, int Cin, int Cout, int epi, int pix_per_wg,
                                   float* part, hipStream_t stream) {
  if (ldk2 != (Cout + 31) / 32 * 32 + 8 || pix_per_wg <= 0) return -3;
  if (epi == c1f::EPI_MASK && (!e_s || !e_t)) return -4;
  if (epi == c1f::EPI_BLOCK && (!e_add || !e_y1)) return -4;
  c1f::Args a{g, y, alpha, beta, gamma, wb, wb_ld, e_x, e_s, e_t, e_add, e_y1, e_y2, out, stats, NS, garena, ldw,
              woff, M, pix_per_wg, part};
#define C1F(CI, CO, E, WM, WN, PT, NW) \
  if (Cin == CI && Cout == CO && epi == E) return c1f::launch<CI, CO, E, WM, WN, PT, NW>(a, C, stream);
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
