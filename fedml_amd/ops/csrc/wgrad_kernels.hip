// Backward-weight kernel for the client-batched convolutions (gfx950, bf16 MFMA).
//
//   dW[c][co][tap][ci] += Σ_p dy[c][p][co] · act(x)[c][p ⊕ tap][ci]
//   dy = α·g + β·y + γ   (the following BatchNorm's backward, folded)
//   act = PRO ? relu(x·s + t) : x   (the preceding BatchNorm + ReLU, recomputed — never stored)
//
// The reduction runs over pixels, so both MFMA operands must be pixel-major per lane
// (A = dyᵀ: lane holds 8 consecutive pixels of one output channel; B = im2col(act): 8
// consecutive pixels of one (tap, ci)). Tiles are staged into LDS in their NATURAL layout
// ([pixel][channel], 16-B vector writes after the operand transform) and the fragments are
// read with gfx950's transposing LDS read `ds_read_b64_tr_b16` (two per operand: pixels
// 8g..8g+3 and 8g+4..8g+7 of column l&15), so no scalar transposed LDS traffic is needed.
// A workgroup owns one client and a contiguous pixel chunk; its 4 waves split the Cout×K output
// tiles and keep them in registers for the whole chunk; the partial dW is added (fp32 atomics)
// into the client-stacked gradient arena at the OIHW position of each element.
#include "prec.h"
#include "detacc.h"
#include "bnlazy.h"

#include <stdlib.h>
#include <type_traits>

FA_DET_EXPORT(wgrad)

using prec::BF16;
using prec::F32;
using prec::F32X3;

// One workgroup = (client c, pixel chunk, K-slice z). The K-slice keeps the per-wave output
// tile count ≤ 16 (≤ 64 accumulator registers) and means each workgroup only stages the im2col
// columns it needs. Raw global data of sub-tile i+1 is prefetched into registers while the
// MFMAs of sub-tile i run. Partial dW goes to a GEMM-layout fp32 scratch [C][Cout][K] with
// row-contiguous atomics (16 consecutive k per lane group), then one scatter pass adds it into
// the OIHW gradient arena.
template <class P, int TPW, int DYI, int AI>
__global__ __launch_bounds__(256) void conv_wgrad_tr_kernel(
    const typename P::T* __restrict__ g, const typename P::T* __restrict__ yv, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ gamma, const typename P::T* __restrict__ x,
    const float* __restrict__ ps, const float* __restrict__ pt, float* __restrict__ dw, int Nb, int H, int W,
    int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int pix_per_wg, int nt_per_z,
    const int* __restrict__ nimg, int co_slice, const BnLazy* __restrict__ lz) {
  using T = typename P::T;
  const bool PRO = ps != nullptr;   // runtime flag: halves the instantiations (uniform branch)
  using frag_t = typename P::frag_t;
  constexpr int V = P::VEC;
  constexpr int PT = P::kF32 ? 32 : 64;   // pixels per staged sub-tile (fp32: half → same register budget)
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int K = KH * KW * Cin;
  // this client's valid output pixels (images past nimg[c] are padding)
  const int Mv = nimg ? min(Nb * Ho * Wo, nimg[c] * Ho * Wo) : Nb * Ho * Wo;
  if ((int)(blockIdx.x * pix_per_wg) >= Mv) return;   // uniform: whole workgroup idle
  const int NT2 = (K + 15) / 16;
  // blockIdx.z = (K-slice, output-channel slice): wide layers (Cout > 256) split their Cout into
  // co_slice-wide slices so the staged dy tile and the per-wave tile count stay bounded
  const int nco = Cout / co_slice;
  const int co_lo = (blockIdx.z % nco) * co_slice;
  const int Cs = co_slice;
  const int nt_lo = (blockIdx.z / nco) * nt_per_z;
  const int nt_hi = min(NT2, nt_lo + nt_per_z);
  const int k_lo = nt_lo * 16;
  const int k_hi = min(K, nt_hi * 16);
  const int kw_ = (nt_hi - nt_lo) * 16;     // staged columns (zero beyond K)
  const int M = Nb * Ho * Wo;
  const int ldd = P::pitch_tr(Cs);
  const int lda = P::pitch_tr(kw_);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* dyL = reinterpret_cast<T*>(smem);                  // [PT][ldd]
  T* aL = dyL + PT * ldd;                               // [PT][lda]
  float* vv = reinterpret_cast<float*>(aL + PT * lda);  // α β γ [Cs] (this slice), s t [Cin]

  for (int i = threadIdx.x; i < Cs; i += 256) {
    if (lz) {   // one writer per output-channel slice: the first pixel chunk of its first K-slice
      bn_lazy_bwd(lz, c, co_lo + i, blockIdx.x == 0 && (int)blockIdx.z < nco, vv[i], vv[Cs + i], vv[2 * Cs + i]);
    } else {
      vv[i] = alpha[(int64_t)c * Cout + co_lo + i];
      vv[Cs + i] = beta[(int64_t)c * Cout + co_lo + i];
      vv[2 * Cs + i] = gamma[(int64_t)c * Cout + co_lo + i];
    }
  }
  if (PRO)
    for (int i = threadIdx.x; i < Cin; i += 256) {
      vv[3 * Cs + i] = ps[(int64_t)c * Cin + i];
      vv[3 * Cs + Cin + i] = pt[(int64_t)c * Cin + i];
    }
  const int padc = kw_ - (k_hi - k_lo);
  for (int i = threadIdx.x; i < PT * padc; i += 256) aL[(i / padc) * lda + (k_hi - k_lo) + i % padc] = 0;

  const int MT = Cs / 16, NTZ = nt_hi - nt_lo;
  const int ntiles = MT * NTZ;
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};

  const T* gc = g + (int64_t)c * M * Cout;
  const T* yc = yv + (int64_t)c * M * Cout;
  const T* xc = x + (int64_t)c * Nb * H * W * Cin;
  const int p_begin = blockIdx.x * pix_per_wg;
  const int p_end = min(Mv, p_begin + pix_per_wg);
  const int cg = Cs / V, kg = (k_hi - k_lo) / V;
  const int n_dy = PT * cg, n_a = PT * kg;
  __syncthreads();

  uint4 rg[DYI], ry[DYI], rx[AI];
  uint32_t dvalid = 0, avalid = 0;
  auto load_sub = [&](int p0) {
    dvalid = 0;
    avalid = 0;
#pragma unroll
    for (int it = 0; it < DYI; ++it) {
      const int i = threadIdx.x + it * 256;
      rg[it] = make_uint4(0, 0, 0, 0);
      ry[it] = make_uint4(0, 0, 0, 0);
      if (i < n_dy) {
        const int p = p0 + i / cg, co0 = (i % cg) * V;
        if (p < p_end) {
          rg[it] = *reinterpret_cast<const uint4*>(gc + (int64_t)p * Cout + co_lo + co0);
          ry[it] = *reinterpret_cast<const uint4*>(yc + (int64_t)p * Cout + co_lo + co0);
          dvalid |= 1u << it;
        }
      }
    }
#pragma unroll
    for (int it = 0; it < AI; ++it) {
      const int i = threadIdx.x + it * 256;
      rx[it] = make_uint4(0, 0, 0, 0);
      if (i < n_a) {
        const int p = p0 + i / kg, k0 = k_lo + (i % kg) * V;
        if (p < p_end) {
          const int tap = k0 / Cin, ci0 = k0 % Cin;
          const int n = p / (Ho * Wo), r = p % (Ho * Wo);
          const int oh = r / Wo, ow = r % Wo;
          const int ih = oh * stride - pad + tap / KW, iw = ow * stride - pad + tap % KW;
          if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
            rx[it] = *reinterpret_cast<const uint4*>(xc + (((int64_t)n * H + ih) * W + iw) * Cin + ci0);
            avalid |= 1u << it;
          }
        }
      }
    }
  };
  auto store_sub = [&]() {
#pragma unroll
    for (int it = 0; it < DYI; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < n_dy) {
        const int pp = i / cg, co0 = (i % cg) * V;
        float gf[V], yf[V], d[V];
        P::unpack(rg[it], gf);
        P::unpack(ry[it], yf);
        const bool live = (dvalid >> it) & 1u;
#pragma unroll
        for (int j = 0; j < V; ++j)
          d[j] = live ? vv[co0 + j] * gf[j] + vv[Cs + co0 + j] * yf[j] + vv[2 * Cs + co0 + j] : 0.f;
        P::st_chunk(dyL + pp * ldd + co0, P::pack(d));
      }
    }
#pragma unroll
    for (int it = 0; it < AI; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < n_a) {
        const int pp = i / kg, kk = (i % kg) * V;
        uint4 v = rx[it];
        if (!((avalid >> it) & 1u)) {
          v = make_uint4(0, 0, 0, 0);   // zero padding / out-of-range pixel (not relu(shift))
        } else if (PRO) {
          const int ci0 = (k_lo + kk) % Cin;
          float f[V];
          P::unpack(v, f);
#pragma unroll
          for (int j = 0; j < V; ++j) f[j] = fmaxf(f[j] * vv[3 * Cs + ci0 + j] + vv[3 * Cs + Cin + ci0 + j], 0.f);
          v = P::pack(f);
        }
        P::st_chunk(aL + pp * lda + kk, v);
      }
    }
  };

  if (p_begin < p_end) load_sub(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += PT) {
    store_sub();
    __syncthreads();
    if (p0 + PT < p_end) load_sub(p0 + PT);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = wid + 4 * t;
      if (tile < ntiles) {
        const int mt = tile / NTZ, nt = tile % NTZ;
#pragma unroll
        for (int ks = 0; ks < PT / 32; ++ks) {
          const frag_t af = P::frag_tr(dyL, ldd, ks * 32, mt * 16, lane);
          const frag_t bf = P::frag_tr(aL, lda, ks * 32, nt * 16, lane);
          acc[t] = P::mma(af, bf, acc[t]);
        }
      }
    }
    __syncthreads();
  }
  float* dwc = dw + (int64_t)c * Cout * K;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = wid + 4 * t;
    if (tile < ntiles) {
      const int mt = tile / NTZ, nt = tile % NTZ;
      const int k = k_lo + nt * 16 + (lane & 15);
      if (k < K) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = co_lo + mt * 16 + 4 * (lane >> 4) + i;
          fa_acc_add(&dwc[(int64_t)co * K + k], acc[t][i]);
        }
      }
    }
  }
}

__global__ void wgrad_scatter_kernel(float* __restrict__ dw, float* __restrict__ garena, int64_t ldw, int64_t woff,
                                     int Cout, int Cin, int taps, int cin_src);

// GEMM-layout dW row [tap·Cin + ci] of one (client, co) → OIHW row [ci][tap] (+=), through LDS so both
// the read and the write are contiguous (the element-wise scatter writes with a stride of `taps`), and
// the scratch row is cleared for the next layer. One workgroup per (co, client).
__global__ __launch_bounds__(256) void wgrad_scatter_rows_kernel(float* __restrict__ dw, float* __restrict__ garena,
                                                                 int64_t ldw, int64_t woff, int Cout, int Cin,
                                                                 int taps, int cin_src) {
  extern __shared__ float row[];
  const int co = blockIdx.x, c = blockIdx.y;
  const int K = taps * Cin;
  float* d = dw + ((int64_t)c * Cout + co) * K;
  for (int i = threadIdx.x; i < K; i += 256) {
    row[i] = d[i];
    d[i] = 0.f;
  }
  __syncthreads();
  float* gw = garena + (int64_t)c * ldw + woff + (int64_t)co * cin_src * taps;
  for (int i = threadIdx.x; i < cin_src * taps; i += 256) {
    const int ci = i / taps, tap = i - ci * taps;
    gw[i] += row[tap * Cin + ci];
  }
}

static int wgrad_scatter_rows(float* dw, float* garena, int64_t ldw, int64_t woff, int C, int Cout, int Cin, int taps,
                              int cin_src, hipStream_t stream) {
  const size_t smem = (size_t)taps * Cin * 4;
  if (smem > 64 * 1024 || Cout > 65535 || C > 65535) {
    hipLaunchKernelGGL(wgrad_scatter_kernel, dim3(fa_grid((int64_t)Cout * taps * Cin, 256, 64), C), dim3(256), 0,
                       stream, dw, garena, ldw, woff, Cout, Cin, taps, cin_src);
  } else {
    hipLaunchKernelGGL(wgrad_scatter_rows_kernel, dim3(Cout, C), dim3(256), smem, stream, dw, garena, ldw, woff, Cout,
                       Cin, taps, cin_src);
  }
  return (int)hipGetLastError();
}

// ---- wide layers (Cout ≥ 128: ResNet-18 stages 2-4) ----
// One workgroup owns a 128 (co) × 128 (k) dW tile of one client and reduces it over a pixel chunk;
// its 4 waves form a 2 × 2 grid of 64 × 64 sub-tiles (4 × 4 MFMA tiles each), so per 32-pixel K step
// a wave reads 4 dy fragments + 4 im2col fragments (transposing LDS reads) for 16 MFMAs — the
// generic kernel above re-reads both per MFMA. The next sub-tile's global data is prefetched into
// registers during the MFMAs. When one chunk covers the client's pixels (the deep, small-image
// stages: 4·4·64 px) the tile is owned by exactly one workgroup and is added straight into the
// OIHW gradient arena — no fp32 atomics, no scratch, no scatter pass.
template <class P>
__global__ __launch_bounds__(256) void wgrad_wide_kernel(
    const typename P::T* __restrict__ g, const typename P::T* __restrict__ yv, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ gamma, const typename P::T* __restrict__ x,
    const float* __restrict__ ps, const float* __restrict__ pt, float* __restrict__ dw, float* __restrict__ garena,
    int64_t ldw, int64_t woff, int cin_src, int Nb, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW,
    int stride, int pad, int pix_per_wg, const int* __restrict__ nimg, int direct) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  constexpr int V = P::VEC;
  constexpr int PT = P::kF32 ? 32 : 64;
  constexpr int TS = 128;                       // tile edge (co and k)
  constexpr int NI = PT * (TS / V) / 256;       // 16-B chunks per thread per operand and sub-tile (4)
  const bool PRO = ps != nullptr;
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int K = KH * KW * Cin;
  const int nks = (K + TS - 1) / TS;
  const int co_lo = (blockIdx.z / nks) * TS;
  const int k_lo = (blockIdx.z % nks) * TS;
  const int kn = min(TS, K - k_lo);             // multiple of 8 (Cin % 8 == 0)
  const int M = Nb * Ho * Wo;
  const int Mv = nimg ? min(M, nimg[c] * Ho * Wo) : M;
  const int p_begin = blockIdx.x * pix_per_wg;
  if (p_begin >= Mv) return;   // uniform: whole workgroup idle
  const int p_end = min(Mv, p_begin + pix_per_wg);
  constexpr int LD = P::pitch_tr(TS);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* dyL = reinterpret_cast<T*>(smem);                 // [PT][LD]
  T* aL = dyL + PT * LD;                               // [PT][LD]

  // Each thread always stages the same 16-B column chunk (channels col..col+V-1 of dy and k-columns
  // k_lo+col.. of im2col) for rows pp0 + RPI·it: its folded-BN coefficients, tap and prologue
  // scale/shift are loop invariants kept in registers; per row only the pixel is decoded (float-
  // reciprocal divmod — the runtime integer divisions made this loop VALU-bound).
  constexpr int CPR = TS / V;   // chunks per staged row
  constexpr int RPI = 256 / CPR;
  const int col = (threadIdx.x % CPR) * V;
  const int pp0 = threadIdx.x / CPR;
  float ca[V], cb[V], cc[V], cs[V], ct[V];
  const bool DYM = yv == nullptr;   // g holds the materialised dy (dy_apply): no transform, no y stream
#pragma unroll
  for (int j = 0; j < V; ++j) {
    ca[j] = DYM ? 1.f : alpha[(int64_t)c * Cout + co_lo + col + j];
    cb[j] = DYM ? 0.f : beta[(int64_t)c * Cout + co_lo + col + j];
    cc[j] = DYM ? 0.f : gamma[(int64_t)c * Cout + co_lo + col + j];
  }
  const bool kval = col < kn;
  const int k0 = k_lo + (kval ? col : 0);
  const int tap = k0 / Cin, ci0 = k0 % Cin;
  const int kh = tap / KW, kw = tap % KW;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    cs[j] = PRO ? ps[(int64_t)c * Cin + ci0 + j] : 1.f;
    ct[j] = PRO ? pt[(int64_t)c * Cin + ci0 + j] : 0.f;
  }
  const int HWo = Ho * Wo;
  const float inv_hw = 1.f / (float)HWo, inv_w = 1.f / (float)Wo;
  auto fdiv = [](int a, int b, float inv_b) {   // exact for 0 ≤ a < 2^22
    int q = (int)((float)a * inv_b);
    const int r = a - q * b;
    return q + (r >= b) - (r < 0);
  };

  // buffer descriptors over this client's operands (wave-uniform inputs made provably uniform by readfirstlane,
  // else hipcc wraps each buffer op in a waterfall loop): per-row 32-bit byte offsets, one VALU add each, and an
  // offset past num_records loads zeros (rows past the chunk, out-of-image taps) without a branch
  auto rsrc = [](const void* base, int64_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
  };
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  auto bl = [](__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
  };
  constexpr uint32_t kOOB = 0x80000000u;   // ≥ every num_records (the launcher keeps them below 2^31 bytes)
  const int64_t dy_bytes = (int64_t)M * Cout * (int64_t)sizeof(T);
  const __amdgpu_buffer_rsrc_t sg = rsrc(g + (int64_t)c * M * Cout, dy_bytes);
  const __amdgpu_buffer_rsrc_t sy = rsrc(DYM ? g + (int64_t)c * M * Cout : yv + (int64_t)c * M * Cout, dy_bytes);
  const __amdgpu_buffer_rsrc_t sx = rsrc(x + (int64_t)c * Nb * H * W * Cin, (int64_t)Nb * H * W * Cin * (int64_t)sizeof(T));
  // Per staged row: the pixel decoded by shifts when Ho·Wo and Wo are powers of two — the 64-bit offsets and
  // float-reciprocal divisions cost ~60 VALU instructions per row, which made this kernel VALU-issue-bound
  // (~380 VALU per 32 MFMAs of a sub-tile; profiles/r5_convk_valu.txt)
  const int sh_w = (Wo & (Wo - 1)) == 0 ? __builtin_ctz(Wo) : -1;
  const int sh_hw = (sh_w >= 0 && (HWo & (HWo - 1)) == 0) ? __builtin_ctz(HWo) : -1;
  const int xh = kh - pad, xw = kw - pad;
  uint4 rg[NI], ry[NI], rx[NI];
  uint32_t dvalid = 0, avalid = 0;
  auto load_sub = [&](int p0) {
    dvalid = 0;
    avalid = 0;
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int p = p0 + pp0 + RPI * it;
      if (DYM) ry[it] = make_uint4(0, 0, 0, 0);
      const bool pv = p < p_end;
      dvalid |= (uint32_t)pv << it;
      const uint32_t go = pv ? (uint32_t)(p * Cout + co_lo + col) * (uint32_t)sizeof(T) : kOOB;
      rg[it] = bl(sg, go);
      if (!DYM) ry[it] = bl(sy, go);
      int n, oh, ow;
      if (sh_hw >= 0) {
        n = p >> sh_hw;
        const int r = p & (HWo - 1);
        oh = r >> sh_w;
        ow = r & (Wo - 1);
      } else {
        n = fdiv(p, HWo, inv_hw);
        const int r = p - n * HWo;
        oh = fdiv(r, Wo, inv_w);
        ow = r - oh * Wo;
      }
      const int ih = oh * stride + xh, iw = ow * stride + xw;
      const bool ok = pv && kval && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      rx[it] = bl(sx, ok ? (uint32_t)(((n * H + ih) * W + iw) * Cin + ci0) * (uint32_t)sizeof(T) : kOOB);
      avalid |= (uint32_t)ok << it;
    }
  };
  auto store_sub = [&]() {
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int pp = pp0 + RPI * it;
      const bool live = (dvalid >> it) & 1u;   // pixels past the chunk: dy = 0 (not γ)
      if (DYM) {
        P::st_chunk(dyL + pp * LD + col, rg[it]);   // zero-filled when not live
      } else {
        float gf[V], yf[V], d[V];
        P::unpack(rg[it], gf);
        P::unpack(ry[it], yf);
#pragma unroll
        for (int j = 0; j < V; ++j) d[j] = live ? ca[j] * gf[j] + cb[j] * yf[j] + cc[j] : 0.f;
        P::st_chunk(dyL + pp * LD + col, P::pack(d));
      }
      uint4 v = rx[it];   // out-of-image taps / past-K columns stay 0 (zero padding, not relu(shift))
      if (PRO && ((avalid >> it) & 1u)) {
        float f[V];
        P::unpack(v, f);
#pragma unroll
        for (int j = 0; j < V; ++j) f[j] = fmaxf(f[j] * cs[j] + ct[j], 0.f);
        v = P::pack(f);
      }
      P::st_chunk(aL + pp * LD + col, v);
    }
  };

  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  load_sub(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += PT) {
    store_sub();
    __syncthreads();
    if (p0 + PT < p_end) load_sub(p0 + PT);
#pragma unroll
    for (int ks = 0; ks < PT / 32; ++ks) {
      frag_t af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = P::frag_tr(dyL, LD, ks * 32, (wm * 4 + i) * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = P::frag_tr(aL, LD, ks * 32, (wn * 4 + j) * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = P::mma(af[i], bf[j], acc[i][j]);
    }
    __syncthreads();
  }
  const int taps = KH * KW;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kk = (wn * 4 + j) * 16 + (lane & 15);
    if (kk >= kn) continue;
    const int k = k_lo + kk;
    const int tap = k / Cin, ci = k % Cin;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co_lo + (wm * 4 + i) * 16 + 4 * (lane >> 4) + r;
        if (direct) {
          if (ci < cin_src) garena[(int64_t)c * ldw + woff + ((int64_t)co * cin_src + ci) * taps + tap] += acc[i][j][r];
        } else {   // several pixel chunks per tile: row-contiguous atomics into the GEMM-layout scratch
          fa_acc_add(&dw[((int64_t)c * Cout + co) * K + k], acc[i][j][r]);
        }
      }
    }
  }
}

template <class P>
static int wgrad_wide(const typename P::T* g, const typename P::T* yv, const float* alpha, const float* beta,
                      const float* gamma, const typename P::T* x, const float* ps, const float* pt, float* garena,
                      int64_t ldw, int64_t woff, int C, int Nb, int H, int W, int Cin, int Ho, int Wo, int Cout,
                      int KH, int KW, int stride, int pad, int cin_src, float* dw, const int* nimg,
                      hipStream_t stream) {
  constexpr int PT = P::kF32 ? 32 : 64;
  const int K = KH * KW * Cin;
  const int nks = (K + 127) / 128;
  const int base = fa_plan_c(C) * nks * (Cout / 128);
  const int M = Nb * Ho * Wo;
  // the kernel's buffer descriptors and per-row byte offsets are 32-bit
  if ((int64_t)M * Cout * P::ES >= (1ll << 31) || (int64_t)Nb * H * W * Cin * P::ES >= (1ll << 31)) return -8;
  // pixel chunks: enough workgroups to fill the chip (FEDML_AMD_WGW_WGS; measured on ResNet-18 ×10: fp32 2048,
  // bf16 1024 — 1.257 → 1.282 rounds/s), chunks of ≥ 512 pixels. One chunk (gx = 1) writes the gradient arena
  // directly — no fp32-atomic scratch and no scatter pass.
  static const int env_target = [] {
    const char* e = getenv("FEDML_AMD_WGW_WGS");
    return e ? atoi(e) : 0;
  }();
  const int target = env_target > 0 ? env_target : (P::kF32 ? 2048 : 1024);
  int gx = max(1, min((target + base - 1) / base, (M + 511) / 512));
  int ppw = ((M + gx - 1) / gx + PT - 1) / PT * PT;
  gx = (M + ppw - 1) / ppw;
  const int direct = gx == 1;
  const size_t smem = (size_t)2 * PT * P::pitch_tr(128) * P::ES;
  auto kern = wgrad_wide_kernel<P>;
  if (smem > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C, nks * (Cout / 128)), dim3(256), smem, stream, g, yv, alpha, beta, gamma, x,
                     ps, pt, dw, garena, ldw, woff, cin_src, Nb, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ppw,
                     nimg, direct);
  if (!direct) {
    fa_det_flush_if_registered(g_fa_det_host_wgrad, dw, (int64_t)C * Cout * K, stream);
    return wgrad_scatter_rows(dw, garena, ldw, woff, C, Cout, Cin, KH * KW, cin_src, stream);
  }
  return (int)hipGetLastError();
}

// dW GEMM layout [c][co][tap*Cin + ci] → OIHW gradient arena (+=), and clear the scratch
__global__ __launch_bounds__(256) void wgrad_scatter_kernel(float* __restrict__ dw, float* __restrict__ garena,
                                                            int64_t ldw, int64_t woff, int Cout, int Cin, int taps,
                                                            int cin_src) {
  const int c = blockIdx.y;
  const int K = taps * Cin;
  const int n = Cout * K;
  float* d = dw + (int64_t)c * n;
  float* gw = garena + (int64_t)c * ldw + woff;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int co = i / K, k = i % K;
    const int tap = k / Cin, ci = k % Cin;
    if (ci < cin_src) gw[((int64_t)co * cin_src + ci) * taps + tap] += d[i];
    d[i] = 0.f;
  }
}

// `dw` scratch: C × Cout × K fp32, zero on entry (left zeroed on exit by the scatter pass)
template <class P>
static int conv_wgrad(const typename P::T* g, const typename P::T* yv, const float* alpha, const float* beta,
                      const float* gamma, const typename P::T* x, const float* ps, const float* pt, float* garena,
                      int64_t ldw, int64_t woff, int C, int Nb, int H, int W, int Cin, int Ho, int Wo, int Cout,
                      int KH, int KW, int stride, int pad, int pix_per_wg, int cin_src, float* dw,
                      const int* nimg, hipStream_t stream) {
  constexpr int V = P::VEC;
  constexpr int PT = P::kF32 ? 32 : 64;
  if (Cin % 8 != 0 || Cout % 16 != 0) return -3;
  const BnLazy* lz = fa_take_lazy(0);   // deferred BN finalisation: the tiled kernel only (not wgrad_wide)
  {
    // FEDML_AMD_WGRAD_WIDE: 0 off, 1 (default) wide layers with K ≥ 256 or Cout > 256, 2 every Cout % 128 == 0
    static int mode = -1;
    if (mode < 0) {
      const char* e = getenv("FEDML_AMD_WGRAD_WIDE");
      mode = e ? atoi(e) : 2;   // measured: +1.8 % on the fp32 headline (downsample convs)
    }
    const int K = KH * KW * Cin;
    if (Cout % 128 == 0 && ((mode == 1 && (K >= 256 || Cout > 256)) || mode == 2)) {
      if (lz) return -9;
      return wgrad_wide<P>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, Nb, H, W, Cin, Ho, Wo, Cout, KH,
                           KW, stride, pad, cin_src, dw, nimg, stream);
    }
  }
  if (!yv) return -7;   // a materialised dy is only consumed by the wide kernel
  const int co_slice = Cout > 256 ? 128 : Cout;   // wide layers: 128-channel dy slices
  if (Cout % co_slice != 0) return -3;
  const int K = KH * KW * Cin;
  const int NT2 = (K + 15) / 16;
  const int MT = co_slice / 16;
  // ≤ 64 tiles per workgroup → ≤ 16 per wave; ≤ 32 column tiles so the A staging fits the largest instantiation
  // (a 16-wide output slice over a long K — squeeze-excite / narrow 1×1 layers — would otherwise ask for 22+)
  const int nt_per_z = max(1, min(min(NT2, 64 / MT), 256 * V / PT));
  const int nz = (NT2 + nt_per_z - 1) / nt_per_z * (Cout / co_slice);
  const int tpw = (MT * nt_per_z + 3) / 4;
  const int M = Nb * Ho * Wo;
  const int gx = (M + pix_per_wg - 1) / pix_per_wg;
  const int kw_ = nt_per_z * 16;
  const int dyi = (PT * (co_slice / V) + 255) / 256;
  const int ai = (PT * (kw_ / V) + 255) / 256;
  // the staging loops cover DYI·256 / AI·256 16-B chunks: a sub-tile larger than the largest
  // instantiation would leave LDS rows unwritten
  if (dyi > 8 || ai > 16) return -6;
  const size_t smem =
      (size_t)PT * (P::pitch_tr(co_slice) + P::pitch_tr(kw_)) * P::ES + (size_t)(3 * co_slice + 2 * Cin) * 4;
  if (smem > 160 * 1024) return -5;
  dim3 grid(gx, C, nz);
  auto go = [&](auto kern) {
    if (smem > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    hipLaunchKernelGGL(kern, grid, dim3(256), smem, stream, g, yv, alpha, beta, gamma, x, ps, pt, dw, Nb, H, W, Cin,
                       Ho, Wo, Cout, KH, KW, stride, pad, pix_per_wg, nt_per_z, nimg, co_slice, lz);
  };
  // instantiated register budgets: dy chunks/thread D ∈ {2, 8}, A chunks/thread ∈ {2, 4, 8, 16}
  auto by_a = [&](auto tpw_c, auto d_c) {
    constexpr int T_ = decltype(tpw_c)::value, D_ = decltype(d_c)::value;
    if (ai <= 2) go(conv_wgrad_tr_kernel<P, T_, D_, 2>);
    else if (ai <= 4) go(conv_wgrad_tr_kernel<P, T_, D_, 4>);
    else if (ai <= 8) go(conv_wgrad_tr_kernel<P, T_, D_, 8>);
    else go(conv_wgrad_tr_kernel<P, T_, D_, 16>);
  };
  auto by_d = [&](auto tpw_c) {
    if (dyi <= 2) by_a(tpw_c, std::integral_constant<int, 2>{});
    else by_a(tpw_c, std::integral_constant<int, 8>{});
  };
  if (tpw <= 4) by_d(std::integral_constant<int, 4>{});
  else if (tpw <= 8) by_d(std::integral_constant<int, 8>{});
  else by_d(std::integral_constant<int, 16>{});
  fa_det_flush_if_registered(g_fa_det_host_wgrad, dw, (int64_t)C * Cout * K, stream);
  return wgrad_scatter_rows(dw, garena, ldw, woff, C, Cout, Cin, KH * KW, cin_src, stream);
}

FA_EXPORT int fa_conv_wgrad(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                            const float* gamma, const uint16_t* x, const float* ps, const float* pt, float* garena,
                            int64_t ldw, int64_t woff, int C, int Nb, int H, int W, int Cin, int Ho, int Wo, int Cout,
                            int KH, int KW, int stride, int pad, int pix_per_wg, int cin_src, float* dw,
                            const int* nimg, hipStream_t stream) {
  return conv_wgrad<BF16>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, Nb, H, W, Cin, Ho, Wo, Cout, KH,
                          KW, stride, pad, pix_per_wg, cin_src, dw, nimg, stream);
}
FA_EXPORT int fa_conv_wgrad_f32(const float* g, const float* yv, const float* alpha, const float* beta,
                                const float* gamma, const float* x, const float* ps, const float* pt, float* garena,
                                int64_t ldw, int64_t woff, int C, int Nb, int H, int W, int Cin, int Ho, int Wo,
                                int Cout, int KH, int KW, int stride, int pad, int pix_per_wg, int cin_src, float* dw,
                                const int* nimg, hipStream_t stream) {
  FA_F32_DISPATCH(prec, conv_wgrad<PX>(g, yv, alpha, beta, gamma, x, ps, pt, garena, ldw, woff, C, Nb, H, W, Cin, Ho, Wo, Cout, KH,
                         KW, stride, pad, pix_per_wg, cin_src, dw, nimg, stream));
}

// scatter a GEMM-layout dW scratch [C][Cout][taps·Cin] into the OIHW arena (+=) and clear it
FA_EXPORT int fa_wgrad_scatter(float* dw, float* garena, int64_t ldw, int64_t woff, int C, int Cout, int Cin,
                               int taps, int cin_src, hipStream_t stream) {
  hipLaunchKernelGGL(wgrad_scatter_kernel, dim3(fa_grid((int64_t)Cout * taps * Cin, 256, 64), C), dim3(256), 0,
                     stream, dw, garena, ldw, woff, Cout, Cin, taps, cin_src);
  return (int)hipGetLastError();
}

// ---- deferred scatter of every 3×3 layer's dW in ONE launch at the end of backward ----
// Each layer owns its GEMM-layout scratch [C][Cout][9·Cin] at `src_off` of one buffer; blockIdx.z
// selects the layer (replaces one scatter launch per 3×3 layer and step).
struct ScatterSeg {
  int64_t src_off;   // element offset of the layer's [C][Cout][9·Cin] scratch
  int64_t woff;      // OIHW weight offset inside a client row of the gradient arena
  int cout, cin, cin_src, pad_;
};

__global__ __launch_bounds__(256) void wgrad_scatter_multi_kernel(float* __restrict__ dw, float* __restrict__ garena,
                                                                  int64_t ldw, const ScatterSeg* __restrict__ segs) {
  const ScatterSeg sg = segs[blockIdx.z];
  const int c = blockIdx.y;
  const int K = 9 * sg.cin;
  const int n = sg.cout * K;
  float* d = dw + sg.src_off + (int64_t)c * n;
  float* gw = garena + (int64_t)c * ldw + sg.woff;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int co = i / K, k = i - co * K;
    const int tap = k / sg.cin, ci = k - tap * sg.cin;
    if (ci < sg.cin_src) gw[((int64_t)co * sg.cin_src + ci) * 9 + tap] += d[i];
    d[i] = 0.f;
  }
}

// segs: device array of `nseg` ScatterSeg; max_n = the largest Cout·9·Cin among them
FA_EXPORT int fa_wgrad_scatter_multi(float* dw, float* garena, int64_t ldw, const void* segs, int nseg, int max_n,
                                     int C, hipStream_t stream) {
  if (nseg <= 0) return 0;
  if (nseg > 65535 || C > 65535) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wgrad_scatter_multi_kernel, dim3(fa_grid(max_n, 256, 64), C, nseg), dim3(256), 0, stream, dw,
                     garena, ldw, (const ScatterSeg*)segs);
  return (int)hipGetLastError();
}
