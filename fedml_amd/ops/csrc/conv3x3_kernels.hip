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

// Stage one work unit of a client into an LDS tile [ns][TR][TW][KC+8] with the operand transform
// applied. Tile row tr / column tc hold source pixel (t0 + tr, tc − 1); outside the source image
// the tile is zero (the convolution's zero padding). UPS: the source is read zero-upsampled by 2
// (stride-2 backward-data: dy sits at the even positions of the dx grid). `src`/`src2` already
// point at the client.
template <int KC, int XF, int UPS>
__device__ __forceinline__ void stage_tile(uint16_t* tile, const uint16_t* __restrict__ src,
                                           const uint16_t* __restrict__ src2, const float* v0, const float* v1,
                                           const float* v2, int img0, int ns, int t0, int TR, int TW, int Hs,
                                           int Ws) {
  constexpr int LD = KC + 8;
  constexpr int CG = KC / 8;
  const int total = ns * TR * TW * CG;
  for (int i = threadIdx.x; i < total; i += 256) {
    const int cg = i % CG;
    const int pix = i / CG;
    const int im = pix / (TR * TW);
    const int r = pix % (TR * TW);
    int t = t0 + r / TW, u = r % TW - 1;
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
      v = *reinterpret_cast<const uint4*>(src + off);
      if (XF != XF_NONE) {
        float f[8];
        unpack8(v, f);
        if (XF == XF_BNRELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j] * v0[cg * 8 + j] + v1[cg * 8 + j], 0.f);
        } else {
          float y[8];
          unpack8(*reinterpret_cast<const uint4*>(src2 + off), y);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = v0[cg * 8 + j] * f[j] + v1[cg * 8 + j] * y[j] + v2[cg * 8 + j];
        }
        v = pack8(f);
      }
    }
    *reinterpret_cast<uint4*>(tile + (int64_t)pix * LD + cg * 8) = v;
  }
}

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
};

// MTW 16-pixel tiles per wave share every B fragment read.
// ST = stride: forward stride 2 reads the input at (2·p + tap); backward-data stride 2 reads a
// zero-upsampled dy tile at the dx resolution (then it is a stride-1 correlation).
template <int KC, int NOUT, int XF, int BWD, int EPI, int MTW, int ST>
__global__ __launch_bounds__(256) void conv3x3_gemm_kernel(Args a) {
  constexpr int NT = NOUT / 16;
  constexpr int LD = KC + 8;
  constexpr int K = 9 * KC;
  constexpr int KSTEPS = (K + 31) / 32;
  constexpr int CG = NOUT / 8;
  constexpr int ROWS_PER_PASS = 64 / CG;
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
  float* red = v2 + KC;                                                     // [4][NOUT][3]
  uint16_t* stage = reinterpret_cast<uint16_t*>(red + 4 * NOUT * 3);       // [4][16][NOUT]
  uint16_t* my_stage = stage + wid * 16 * NOUT;
  uint16_t* tile = stage + 4 * 16 * NOUT;                                   // [S][H+2][W+2][LD]

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
    for (int i = threadIdx.x; i < 4 * NOUT * 3; i += 256) red[i] = 0.f;
  }

  const uint16_t* src = a.src + (int64_t)c * a.N * Hs * Ws * KC;
  const uint16_t* src2 = (XF == XF_DY) ? a.src2 + (int64_t)c * a.N * Hs * Ws * KC : nullptr;
  uint16_t* out = a.out + (int64_t)c * a.N * HW * NO;

  float st0[8], st1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st0[j] = 0.f; st1[j] = 0.f; }
  const int my_cg = lane % CG;

  const int R = a.R, RW = R * W;
  const int TR = SP == 2 ? 2 * R + 1 : R + 2;    // tile rows incl. halo
  const int u_lo = blockIdx.x * a.units_per_wg;
  const int u_hi = min(a.units, u_lo + a.units_per_wg);
  for (int u = u_lo; u < u_hi; ++u) {
    int img0, ns, r0;
    unit_geom(u, a.N, H, R, a.S, img0, ns, r0);
    const int64_t pix0 = (int64_t)img0 * HW + (int64_t)r0 * W;  // first output pixel of the unit
    __syncthreads();  // previous unit fully consumed (and, first time, weights/vectors visible)
    stage_tile<KC, XF, UPS>(tile, src, src2, v0, v1, v2, img0, ns, SP * r0 - 1, TR, TW, Hs, Ws);
    __syncthreads();
    const int P = ns * RW;
    const int ntile = (P + 15) / 16;
    for (int t0 = wid * MTW; t0 < ntile; t0 += 4 * MTW) {
      int base[MTW];
      bool valid[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        const int p = (t0 + mt) * 16 + (lane & 15);
        valid[mt] = (t0 + mt) < ntile && p < P;
        const int pp = valid[mt] ? p : 0;
        const int im = pp / RW, r = pp % RW;
        base[mt] = ((im * TR + SP * (r / W)) * TW + SP * (r % W)) * LD;
      }
      f32x4 acc[MTW][NT];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int k = ks * 32 + 8 * g;
        const int tap = k / KC, ci = k % KC;
        const int kh = tap / 3, kw = tap % 3;
        // forward reads x_pad(pr + kh, pc + kw); backward reads dy_pad(pr + 2 − kh, pc + 2 − kw)
        const int toff = BWD ? ((2 - kh) * TW + (2 - kw)) * LD + ci : (kh * TW + kw) * LD + ci;
        const bool kin = k < K;
        bf16x8 af[MTW];
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) {
          uint4 v = make_uint4(0, 0, 0, 0);
          if (valid[mt] && kin) v = *reinterpret_cast<const uint4*>(tile + base[mt] + toff);
          af[mt] = as_bf16x8(v);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint4 bv = *reinterpret_cast<const uint4*>(wl + (nt * 16 + (lane & 15)) * a.ldk + ks * 32 + 8 * g);
#pragma unroll
          for (int mt = 0; mt < MTW; ++mt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], as_bf16x8(bv), acc[mt][nt], 0, 0, 0);
        }
      }
      // ---- epilogue, one 16-pixel tile at a time ----
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        if (t0 + mt >= ntile) break;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) my_stage[(4 * g + i) * NOUT + nt * 16 + (lane & 15)] = f32_to_bf16(acc[mt][nt][i]);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int rows_valid = min(16, P - (t0 + mt) * 16);
#pragma unroll
        for (int pass = 0; pass < (16 + ROWS_PER_PASS - 1) / ROWS_PER_PASS; ++pass) {
          const int row = pass * ROWS_PER_PASS + lane / CG;
          if (lane / CG < ROWS_PER_PASS && row < rows_valid) {
            const int ch0 = my_cg * 8;
            const uint4 dv = *reinterpret_cast<const uint4*>(my_stage + row * NOUT + ch0);
            const int64_t goff = (pix0 + (t0 + mt) * 16 + row) * NO + ch_base + ch0;
            if (EPI == EPI_FWD) {
              *reinterpret_cast<uint4*>(out + goff) = dv;
              float f[8];
              unpack8(dv, f);
#pragma unroll
              for (int j = 0; j < 8; ++j) { st0[j] += f[j]; st1[j] += f[j] * f[j]; }
            } else {
              const int64_t eoff = (int64_t)c * a.N * HW * NO + goff;
              float gv[8], xv[8];
              unpack8(dv, gv);
              unpack8(*reinterpret_cast<const uint4*>(a.e_x + eoff), xv);
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const int ch = ch0 + j;
                const bool on = xv[j] * a.e_s[(int64_t)c * NO + ch_base + ch] + a.e_t[(int64_t)c * NO + ch_base + ch] > 0.f;
                gv[j] = on ? gv[j] : 0.f;
              }
              const uint4 gp = pack8(gv);
              *reinterpret_cast<uint4*>(out + goff) = gp;
              float gr[8];
              unpack8(gp, gr);
#pragma unroll
              for (int j = 0; j < 8; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * xv[j]; }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
  }

  // ---- statistics: lanes sharing a channel group → waves → one atomic per (client, channel) ----
#pragma unroll
  for (int o = CG; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      st0[j] += __shfl_xor(st0[j], o, 64);
      st1[j] += __shfl_xor(st1[j], o, 64);
    }
  }
  if (lane < CG) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wid * NOUT + lane * 8 + j) * 3 + 0] = st0[j];
      red[(wid * NOUT + lane * 8 + j) * 3 + 1] = st1[j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NOUT * 2; i += 256) {
    const int ch = i / 2, q = i % 2;
    const float s = red[(0 * NOUT + ch) * 3 + q] + red[(1 * NOUT + ch) * 3 + q] + red[(2 * NOUT + ch) * 3 + q] +
                    red[(3 * NOUT + ch) * 3 + q];
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
};

// WN waves split the column tiles of this z-slice, WK = 4/WN waves split the pixel K-steps.
template <int CIN, int COUT, int PRO, int WN, int TPW, int ST>
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

  for (int u = u_lo; u < u_hi; ++u) {
    int img0, ns, r0;
    unit_geom(u, a.N, H, R, a.S, img0, ns, r0);
    const int64_t pix0 = (int64_t)img0 * HW + (int64_t)r0 * W;
    __syncthreads();
    // dy = α·g + β·y + γ, natural [pixel][co] (no halo)
    {
      constexpr int CGD = COUT / 8;
      const int total = ns * RW * CGD;
      for (int i = threadIdx.x; i < total; i += 256) {
        const int cg = i % CGD, p = i / CGD;
        const int64_t off = (pix0 + p) * COUT + cg * 8;
        float gf[8], yf[8];
        unpack8(*reinterpret_cast<const uint4*>(gc + off), gf);
        unpack8(*reinterpret_cast<const uint4*>(yc + off), yf);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          gf[j] = vv[cg * 8 + j] * gf[j] + vv[COUT + cg * 8 + j] * yf[j] + vv[2 * COUT + cg * 8 + j];
        *reinterpret_cast<uint4*>(dyL + (size_t)p * LDD + cg * 8) = pack8(gf);
      }
    }
    stage_tile<CIN, PRO ? XF_BNRELU : XF_NONE, 0>(xt, xc, nullptr, vv + 3 * COUT, vv + 3 * COUT + CIN, nullptr,
                                                 img0, ns, ST * r0 - 1, TR, TW, Hs, Ws);
    __syncthreads();
    const int KS = ns * RW / 32;  // R·W is a multiple of 32
    for (int ks = kgrp; ks < KS; ks += WK) {
      const int p0 = ks * 32;
      // this lane's pixel row of the fragment (8-pixel groups never straddle an image row: W % 8 == 0)
      const int pix = p0 + 8 * g + q;
      const int im = pix / RW, r = pix % RW;
      const uint16_t* xrow = xt + (size_t)((im * TR + ST * (r / W)) * TW + ST * (r % W)) * LDX + 4 * pq;
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
  return (size_t)nout * ldk * 2 + (size_t)3 * kc * 4 + (size_t)4 * nout * 3 * 4 + (size_t)4 * 16 * nout * 2 +
         (size_t)p.S * TR * TW * (kc + 8) * 2;
}

// NOUT_WG output channels per workgroup (blockIdx.z slices the layer's NOUT)
template <int KC, int NOUT_WG, int XF, int BWD, int EPI, int ST>
static int launch_gemm(Args a, int nout, int C, int target_px, hipStream_t stream) {
  constexpr int MTW = NOUT_WG >= 64 ? 2 : 4;
  const Plan p = make_plan(a.N, a.H, a.W, C, target_px, 2048);
  a.R = p.R; a.S = p.S; a.units = p.units; a.units_per_wg = p.units_per_wg; a.nout_total = nout;
  const bool fwd2 = !BWD && ST == 2;
  const int TR = fwd2 ? 2 * p.R + 1 : p.R + 2;
  const int TW = (BWD ? a.W : a.Ws) + 2;
  const size_t smem = gemm_smem(KC, NOUT_WG, a.ldk, p, TR, TW);
  if (smem > 160 * 1024) return -5;
  auto kern = conv3x3_gemm_kernel<KC, NOUT_WG, XF, BWD, EPI, MTW, ST>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(p.gx, C, nout / NOUT_WG), dim3(256), smem, stream, a);
  return (int)hipGetLastError();
}

template <int XF, int BWD, int EPI, int ST>
static int dispatch_gemm(int kc, int nout, const Args& a, int C, hipStream_t s) {
  if (kc != nout) return -2;
  constexpr int PX = ST == 2 ? 128 : 256;
  switch (kc) {
    case 16: return launch_gemm<16, 16, XF, BWD, EPI, ST>(a, nout, C, PX, s);
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
  const c3::Plan p = c3::make_plan(N, Ho, Wo, C, Cin >= 64 ? (stride == 2 ? 64 : 128) : (stride == 2 ? 128 : 256),
                                   2048);
  a.R = p.R; a.S = p.S; a.units = p.units; a.units_per_wg = p.units_per_wg;
  const int TR = stride == 2 ? 2 * p.R + 1 : p.R + 2;
  const int NTK = 9 * Cin / 16;
  const size_t vv = (size_t)(3 * Cout + 2 * Cin) * 4;
  const size_t smem_base = vv + (size_t)p.S * p.R * Wo * (Cout + 8) * 2 +
                           (size_t)p.S * TR * (W + 2) * (Cin + 8) * 2;
#define W3_LAUNCH(CI, CO, WN, TPW, NZ, ST)                                                                     \
  {                                                                                                            \
    a.nt_per_z = (NTK + (NZ) - 1) / (NZ);                                                                      \
    auto kern = ps ? c3::conv3x3_wgrad_kernel<CI, CO, 1, WN, TPW, ST>                                          \
                   : c3::conv3x3_wgrad_kernel<CI, CO, 0, WN, TPW, ST>;                                         \
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
