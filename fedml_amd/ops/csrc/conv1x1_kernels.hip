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
