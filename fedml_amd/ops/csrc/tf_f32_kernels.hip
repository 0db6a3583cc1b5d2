// Client-batched transformer kernels at fp32 storage — the reference's training precision
// (simulation/single_process/fedavg/my_model_trainer_classification.py:26-37 trains in fp32) — for the
// DistilBERT / ViT virtual-client engine. The bf16 counterparts are
// bgemm_kernels.hip and transformer_kernels.hip; these keep every activation, statistic and
// gradient in fp32 and put the products on the matrix cores through the prec.h policies:
//
//   P = prec::F32    exact fp32 products, v_mfma_f32_16x16x4_f32 (bit-for-bit a k-ordered fmaf chain)
//   P = prec::F32X3  split-bf16 products (3 × v_mfma_f32_16x16x32_bf16, ~2⁻¹⁶ relative per product)
//
// selected per process by prec::f32_mma_mode() (the `fp32_mma` config key), like the conv kernels.
//
// * client-batched GEMM  D[c] = A[c] · B[c]ᵀ over per-client weights read straight from the fp32
//   client arena (row segments: a fused q/k/v projection reads three arena slots), forward with
//   fused bias (+ exact-erf GELU), backward-data, and backward-weight accumulated straight into the
//   gradient arena. Block tile 128×128×32, 4 waves × 64×64, register-prefetched double-buffered
//   LDS, XCD-aware block order. Rows whose storage runs along the reduction index ("TR":
//   backward operands) are staged as-is and read with strided ds_read_b32 fragments (prec.h
//   frag_tr); K-major rows are read with two ds_read_b128 (F32X3: pre-split hi/lo at staging).
//   Any N / K is accepted: the VEC = 0 instantiation stages and stores element by element (the
//   classifier heads, N = #labels).
// * fused residual + dropout + LayerNorm forward / backward, per-client gamma/beta
// * exact-erf GELU forward / backward
// * attention (S ≤ 256, head dim 64): exact two-pass row softmax with all scores of a 16-row
//   query slice in registers, K/V streamed through LDS in 64-key chunks; backward as dQ and dK/dV
//   kernels; attention dropout from the shared counter hash (dropout.h).
#include <initializer_list>

#include "prec.h"
#include "dropout.h"
#include "detacc.h"

FA_DET_EXPORT(tf_f32)

namespace tff {

using prec::F32;
using prec::F32X3;

// =========================================================================================
// client-batched GEMM
// =========================================================================================
constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int LDR = BK + 4;      // K-major row tile [128][36]: 16-B aligned rows, 16 rows on distinct banks
constexpr int LDT = BM + 2;      // TR tile [32][130]: ≡ 2 (mod 4) → the two lane groups of a frag_tr read split banks
constexpr int TILE = BM * LDR;   // floats per operand image
static_assert(BK * LDT <= TILE, "TR image must fit the tile slot");

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_ACC = 2, EPI_DGELU = 3 };   // DGELU: D ⊙ gelu'(R) (a GELU's input grad)

struct Segs {        // row segments of an operand (≤ 4 arena slots); one segment = a plain matrix
  int64_t off[4];    // element offset of segment s's first row, relative to the client base
  int lo[5];         // first logical row of segment s (lo[n] = total rows)
  int n;
};

// Constant-index selects only: a runtime index into the by-value kernel-argument struct would be lowered to
// a global load of the kernarg segment plus an s_waitcnt vmcnt(0) — which also waits for every prefetch
// load in flight, serialising the K loop.
__device__ __forceinline__ int64_t seg_row(const Segs& s, int r, int rowlen) {
  int64_t off = s.off[0];
  int lo = s.lo[0];
  if (s.n > 1 && r >= s.lo[1]) { off = s.off[1]; lo = s.lo[1]; }
  if (s.n > 2 && r >= s.lo[2]) { off = s.off[2]; lo = s.lo[2]; }
  if (s.n > 3 && r >= s.lo[3]) { off = s.off[3]; lo = s.lo[3]; }
  return off + (int64_t)(r - lo) * rowlen;
}

struct Args {
  const float* A;    // !A_TR: storage [M][K] (rows m)        A_TR: storage [K][M] (rows = reduction)
  int64_t a_bs;
  int lda;
  const float* B;    // !B_TR: storage rows n (segmented) × K  B_TR: storage rows k (segmented) × N
  int64_t b_bs;
  int ldb;
  Segs bseg;
  float* Cp;         // STORE/GELU: [C][M][ldc]; ACC: rows m of a segmented arena (row length ldc)
  int64_t c_bs;
  int ldc;
  Segs cseg;
  const float* bias; // segmented [N] per client (may be null)
  int64_t bias_bs;
  Segs biasseg;
  float* C2;         // GELU: gelu(D + b); Cp keeps the pre-activation for the backward
  float* bg;         // ACC with A_TR (weight gradient): optional bias gradient += Σ_t A[t][m] (segmented rows)
  int64_t bg_bs;
  Segs bgseg;
  const float* R;    // STORE: optional residual addend [C][M][ldr] (D = A·Bᵀ + b + R: a pre-LN block's x + f(x))
  int64_t r_bs;
  int ldr;
  int M, N, K;
  int tiles_m, tiles_n, nclients;
  int acc_store;     // ACC: the first (and only) writer of these gradient rows — store instead of +=, so the
                     // arena rows need no zero fill (each element has exactly one producing tile: no split-K)
  int stage_epi;     // VEC: epilogue through LDS, row-contiguous 16-B chunks (FEDML_AMD_TF_STAGE_EPI=0: off)
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x, float g) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return g * (cdf + x * pdf);
}


// Stage one operand tile into registers (4 float4 per thread):
//   TR = 0: logical rows [r0, r0+128) × k [k0, k0+32) of storage S[row][k]          (row segmented)
//   TR = 1: storage rows k [k0, k0+32) (segmented) × logical cols [r0, r0+128)
// VEC = 1: every row start and extent is a multiple of 4 floats (one float4 per chunk); VEC = 0:
// element-wise loads with bounds on every element.
// CHECK = 0: the tile lies inside the operand (interior blocks, K % 32 == 0) — unpredicated loads.
template <int TR, int VEC, int CHECK = 1>
__device__ __forceinline__ void load_tile(float4 (&r)[4], const float* __restrict__ base, const Segs& sg, int ld,
                                          int rows, int K, int r0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    int srow, col, lim;
    bool rok;
    if (!TR) {
      srow = r0 + (v >> 3);
      col = k0 + 4 * (v & 7);
      rok = srow < rows;
      lim = K;
    } else {
      srow = k0 + (v >> 5);
      col = r0 + 4 * (v & 31);
      rok = srow < K;
      lim = rows;
    }
    if (!CHECK) {
      r[i] = *reinterpret_cast<const float4*>(base + seg_row(sg, srow, ld) + col);
      continue;
    }
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rok) {
      const float* p = base + seg_row(sg, srow, ld) + col;
      if (VEC) {
        if (col < lim) x = *reinterpret_cast<const float4*>(p);
      } else {
        if (col < lim) x.x = p[0];
        if (col + 1 < lim) x.y = p[1];
        if (col + 2 < lim) x.z = p[2];
        if (col + 3 < lim) x.w = p[3];
      }
    }
    r[i] = x;
  }
}

template <class P, int TR>
__device__ __forceinline__ void store_tile(float* tile, const float4 (&r)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    const uint4 u = make_uint4(__float_as_uint(r[i].x), __float_as_uint(r[i].y), __float_as_uint(r[i].z),
                               __float_as_uint(r[i].w));
    if (!TR) P::st_tile(tile + (v >> 3) * LDR + 4 * (v & 7), v & 7, u);
    else F32::st_chunk(tile + (v >> 5) * LDT + 4 * (v & 31), u);
  }
}

template <class P, int TR>
__device__ __forceinline__ typename P::frag_t frag_of(const float* tile, int row0, int lane) {
  if (TR) return P::frag_tr(tile, LDT, 0, row0, lane);
  return P::frag_tile(tile + (row0 + (lane & 15)) * LDR + 8 * (lane >> 4));
}

// BSUM (weight gradient, A_TR): also sum the staged A chunks of this thread (its 4 rows t of 4 columns m) —
// the bias gradient Σ_t dy[t][m] comes out of the same operand reads
template <class P, int A_TR, int B_TR, int VEC, int CHECK, int BSUM = 0>
__device__ __forceinline__ void gemm_mainloop(f32x4 (&acc)[4][4], const float* A, const Segs& aseg, const float* B,
                                              const Args& p, int m0, int n0, int nk, float* SA0, float* SB0, int tid,
                                              int lane, int wm, int wn, float4& bs) {
  float4 ra[4], rb[4];
  auto bsum = [&]() {
    if constexpr (BSUM != 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { bs.x += ra[i].x; bs.y += ra[i].y; bs.z += ra[i].z; bs.w += ra[i].w; }
    }
  };
  load_tile<A_TR, VEC, CHECK>(ra, A, aseg, p.lda, p.M, p.K, m0, 0, tid);
  bsum();
  load_tile<B_TR, VEC, CHECK>(rb, B, p.bseg, p.ldb, p.N, p.K, n0, 0, tid);
  store_tile<P, A_TR>(SA0, ra, tid);
  store_tile<P, B_TR>(SB0, rb, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {   // the next K-step's global reads fly under this step's MFMAs
      load_tile<A_TR, VEC, CHECK>(ra, A, aseg, p.lda, p.M, p.K, m0, (kt + 1) * BK, tid);
      load_tile<B_TR, VEC, CHECK>(rb, B, p.bseg, p.ldb, p.N, p.K, n0, (kt + 1) * BK, tid);
      bsum();
    }
    const float* ta = SA0 + cur * TILE;
    const float* tb = SB0 + cur * TILE;
    typename P::frag_t bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag_of<P, B_TR>(tb, wn + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const typename P::frag_t af = frag_of<P, A_TR>(ta, wm + 16 * i, lane);
      // operands swapped: the MFMA computes the transposed tile, so a lane owns 4 consecutive
      // output columns n of one row m (16-byte epilogue accesses)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = P::mma(bfr[j], af, acc[i][j]);
    }
    if (more) {
      store_tile<P, A_TR>(SA0 + (cur ^ 1) * TILE, ra, tid);
      store_tile<P, B_TR>(SB0 + (cur ^ 1) * TILE, rb, tid);
    }
    __syncthreads();
  }
}

template <class P, int A_TR, int B_TR, int EPI, int VEC>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const Args p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];   // [A0][A1][B0][B1]
  float* const SA0 = smem;
  float* const SB0 = smem + 2 * TILE;

  // XCD-aware order: consecutive logical tiles (the n-tiles of one client row block, which share
  // the A rows) land on one XCD's L2 under round-robin block placement
  const int total = p.tiles_m * p.tiles_n * p.nclients;
  int L = blockIdx.x;
  if ((total & 7) == 0) L = (L & 7) * (total >> 3) + (L >> 3);
  const int tn = L % p.tiles_n;
  const int tm = (L / p.tiles_n) % p.tiles_m;
  const int c = L / (p.tiles_n * p.tiles_m);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;

  const float* A = p.A + (int64_t)c * p.a_bs;
  const float* B = p.B + (int64_t)c * p.b_bs;
  Segs aseg;
  aseg.n = 1;
  aseg.off[0] = 0;
  aseg.lo[0] = 0;
#pragma unroll
  for (int t = 1; t < 4; ++t) aseg.off[t] = 0;
#pragma unroll
  for (int t = 1; t < 5; ++t) aseg.lo[t] = 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  float4 bs = make_float4(0.f, 0.f, 0.f, 0.f);
  // interior blocks (the vast majority) stage their tiles with unpredicated vector loads
  const bool interior = VEC && m0 + BM <= p.M && n0 + BN <= p.N && (p.K % BK) == 0;
  if constexpr (EPI == EPI_ACC && A_TR == 1 && VEC == 1) {
    // weight gradient with a fused bias gradient: the first column-block of every row-block sums its A operand
    if (p.bg != nullptr && tn == 0) {
      if (interior)
        gemm_mainloop<P, A_TR, B_TR, VEC, 0, 1>(acc, A, aseg, B, p, m0, n0, nk, SA0, SB0, tid, lane, wm, wn, bs);
      else
        gemm_mainloop<P, A_TR, B_TR, VEC, 1, 1>(acc, A, aseg, B, p, m0, n0, nk, SA0, SB0, tid, lane, wm, wn, bs);
      // the 8 threads holding the same 4 columns (tid & 31) combine through LDS (free after the main loop)
      float4* red = reinterpret_cast<float4*>(smem);
      red[tid] = bs;
      __syncthreads();
      if (tid < 32) {
        float4 t4 = red[tid];
#pragma unroll
        for (int g8 = 1; g8 < NT / 32; ++g8) {
          const float4 u = red[g8 * 32 + tid];
          t4.x += u.x; t4.y += u.y; t4.z += u.z; t4.w += u.w;
        }
        const int m = m0 + 4 * tid;
        if (m < p.M) {   // m .. m+3 in one segment (segment bounds are multiples of 4 on the VEC path)
          float4* bp = reinterpret_cast<float4*>(p.bg + (int64_t)c * p.bg_bs + seg_row(p.bgseg, m, 1));
          if (p.acc_store) {
            *bp = t4;
          } else {
            float4 o = *bp;
            o.x += t4.x; o.y += t4.y; o.z += t4.z; o.w += t4.w;
            *bp = o;
          }
        }
      }
    } else if (interior) {
      gemm_mainloop<P, A_TR, B_TR, VEC, 0>(acc, A, aseg, B, p, m0, n0, nk, SA0, SB0, tid, lane, wm, wn, bs);
    } else {
      gemm_mainloop<P, A_TR, B_TR, VEC, 1>(acc, A, aseg, B, p, m0, n0, nk, SA0, SB0, tid, lane, wm, wn, bs);
    }
  } else {
    if (interior)
      gemm_mainloop<P, A_TR, B_TR, VEC, 0>(acc, A, aseg, B, p, m0, n0, nk, SA0, SB0, tid, lane, wm, wn, bs);
    else
      gemm_mainloop<P, A_TR, B_TR, VEC, 1>(acc, A, aseg, B, p, m0, n0, nk, SA0, SB0, tid, lane, wm, wn, bs);
  }

  if (VEC && p.stage_epi) {
    // the tile through LDS (free after the main loop; the bias-sum scratch above is consumed): each 64-row half
    // staged by the two waves that own it, then written by all 256 threads as 16-B chunks of whole 512-B rows —
    // the MFMA layout stores 64-B row pieces
    constexpr int SLD = BN + 4;
    float* stg = smem;   // [64][SLD]
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if ((wm >> 6) == h) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 v = acc[i][j];
            *reinterpret_cast<float4*>(stg + (16 * i + (lane & 15)) * SLD + wn + 16 * j + 4 * (lane >> 4)) =
                make_float4(v[0], v[1], v[2], v[3]);
          }
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int q = tid + NT * t, row = q >> 5, col = 4 * (q & 31);
        const int m = m0 + 64 * h + row, n = n0 + col;
        if (m >= p.M || n >= p.N) continue;
        float4 v = *reinterpret_cast<const float4*>(stg + row * SLD + col);
        if (EPI == EPI_ACC) {
          float* dst = p.Cp + (int64_t)c * p.c_bs + seg_row(p.cseg, m, p.ldc) + n;
          if (!p.acc_store) {
            const float4 q4 = *reinterpret_cast<const float4*>(dst);
            v.x += q4.x; v.y += q4.y; v.z += q4.z; v.w += q4.w;
          }
          *reinterpret_cast<float4*>(dst) = v;
          continue;
        }
        if (p.bias) {
          const float4 b = *reinterpret_cast<const float4*>(p.bias + (int64_t)c * p.bias_bs + seg_row(p.biasseg, n, 1));
          v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
        }
        if (EPI == EPI_DGELU) {
          const float4 x4 = *reinterpret_cast<const float4*>(p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldr + n);
          v.x = gelu_grad(x4.x, v.x); v.y = gelu_grad(x4.y, v.y);
          v.z = gelu_grad(x4.z, v.z); v.w = gelu_grad(x4.w, v.w);
        }
        if (EPI == EPI_STORE && p.R) {
          const float4 r4 = *reinterpret_cast<const float4*>(p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldr + n);
          v.x += r4.x; v.y += r4.y; v.z += r4.z; v.w += r4.w;
        }
        const int64_t o = (int64_t)c * p.c_bs + (int64_t)m * p.ldc + n;
        *reinterpret_cast<float4*>(p.Cp + o) = v;
        if (EPI == EPI_GELU)
          *reinterpret_cast<float4*>(p.C2 + o) = make_float4(gelu_erf(v.x), gelu_erf(v.y), gelu_erf(v.z), gelu_erf(v.w));
      }
      __syncthreads();
    }
    return;
  }

  // epilogue: lane owns row m = m0 + wm + 16i + (lane & 15), cols n .. n+3, n = n0 + wn + 16j + 4(lane >> 4)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm + 16 * i + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + 16 * j + 4 * (lane >> 4);
      if (n >= p.N) continue;
      f32x4 v = acc[i][j];
      if (EPI == EPI_ACC) {
        float* dst = p.Cp + (int64_t)c * p.c_bs + seg_row(p.cseg, m, p.ldc) + n;
        if (VEC) {
          float4 o = make_float4(v[0], v[1], v[2], v[3]);
          if (!p.acc_store) {
            const float4 q = *reinterpret_cast<const float4*>(dst);
            o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
          }
          *reinterpret_cast<float4*>(dst) = o;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = p.acc_store ? v[r] : dst[r] + v[r];
        }
      } else {
        if (p.bias) {
          const float* bp = p.bias + (int64_t)c * p.bias_bs;
          if (VEC) {
            const float4 b = *reinterpret_cast<const float4*>(bp + seg_row(p.biasseg, n, 1));
            v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) v[r] += bp[seg_row(p.biasseg, n + r, 1)];
          }
        }
        if (EPI == EPI_DGELU) {   // the data gradient of a GELU'd linear's output, through the GELU
          const float* rp = p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldr + n;
          if (VEC) {
            const float4 x4 = *reinterpret_cast<const float4*>(rp);
            v[0] = gelu_grad(x4.x, v[0]); v[1] = gelu_grad(x4.y, v[1]);
            v[2] = gelu_grad(x4.z, v[2]); v[3] = gelu_grad(x4.w, v[3]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) v[r] = gelu_grad(rp[r], v[r]);
          }
        }
        if (EPI == EPI_STORE && p.R) {
          const float* rp = p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldr + n;
          if (VEC) {
            const float4 r4 = *reinterpret_cast<const float4*>(rp);
            v[0] += r4.x; v[1] += r4.y; v[2] += r4.z; v[3] += r4.w;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) v[r] += rp[r];
          }
        }
        const int64_t o = (int64_t)c * p.c_bs + (int64_t)m * p.ldc + n;
        if (VEC) {
          *reinterpret_cast<float4*>(p.Cp + o) = make_float4(v[0], v[1], v[2], v[3]);
          if (EPI == EPI_GELU)
            *reinterpret_cast<float4*>(p.C2 + o) = make_float4(gelu_erf(v[0]), gelu_erf(v[1]), gelu_erf(v[2]),
                                                               gelu_erf(v[3]));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) {
              p.Cp[o + r] = v[r];
              if (EPI == EPI_GELU) p.C2[o + r] = gelu_erf(v[r]);
            }
        }
      }
    }
  }
}

template <class P, int A_TR, int B_TR, int EPI>
int launch_gemm(const Args& a, bool vec, hipStream_t st) {
  const int64_t blocks = (int64_t)a.tiles_m * a.tiles_n * a.nclients;
  if (blocks <= 0 || blocks > 0x7fffffff) return (int)hipErrorInvalidValue;
  const size_t smem = 4 * TILE * sizeof(float);   // 72 KiB: 2 blocks per CU (≥ the 33 KiB epilogue staging)
  static_assert(4 * TILE >= 64 * (BN + 4), "epilogue staging must fit the operand images");
  auto kern = vec ? gemm_kernel<P, A_TR, B_TR, EPI, 1> : gemm_kernel<P, A_TR, B_TR, EPI, 0>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  Args b = a;
  const char* se = getenv("FEDML_AMD_TF_STAGE_EPI");
  b.stage_epi = se ? atoi(se) != 0 : 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NT), smem, st, b);
  return (int)hipGetLastError();
}

inline void fill_segs(Segs& s, const int64_t* off, const int* lo, int n) {
  s.n = n < 1 ? 1 : n;
  for (int i = 0; i < 4; ++i) s.off[i] = (off && i < n) ? off[i] : 0;
  for (int i = 0; i < 5; ++i) s.lo[i] = (lo && i <= n) ? lo[i] : 0;
}

// every value a multiple of 4 floats (16-byte vectors everywhere)
inline bool al4(std::initializer_list<int64_t> v) {
  for (int64_t x : v)
    if (x & 3) return false;
  return true;
}
inline bool al16(std::initializer_list<const void*> v) {
  for (const void* x : v)
    if (reinterpret_cast<uintptr_t>(x) & 15) return false;
  return true;
}
inline bool segs_al4(const Segs& s) {
  for (int i = 0; i < s.n; ++i)
    if ((s.off[i] & 3) || (s.lo[i] & 3)) return false;
  return (s.lo[s.n] & 3) == 0;
}

// =========================================================================================
// LayerNorm / GELU (fp32)
// =========================================================================================
// forward: x = res + dropout(h) (both optional), y = LN(x)·γ_c + β_c. One wave per row, NV float4
// chunks per lane (d ≤ 256·NV, d % 4 == 0).
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ h, const float* __restrict__ res, int R,
                                                     int d, int rpc, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, uint32_t thr,
                                                     float dscale, uint32_t seed, float* __restrict__ y,
                                                     float* __restrict__ xsum, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, const uint32_t* __restrict__ seedp,
                                                     int64_t gcs) {
  if (seedp) seed += *seedp * 1000003u;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int c = row / rpc;
  float x[NV][4];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 4;
    if (col < d) {
      const float4 a = *reinterpret_cast<const float4*>(h + (size_t)row * d + col);
      x[v][0] = a.x; x[v][1] = a.y; x[v][2] = a.z; x[v][3] = a.w;
      if (thr) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[v][j] = fa_drop::keep(seed, (uint32_t)row, (uint32_t)(col + j), thr) ? x[v][j] * dscale : 0.f;
      }
      if (res) {
        const float4 b = *reinterpret_cast<const float4*>(res + (size_t)row * d + col);
        x[v][0] += b.x; x[v][1] += b.y; x[v][2] += b.z; x[v][3] += b.w;
      }
      if (xsum && (res || thr))
        *reinterpret_cast<float4*>(xsum + (size_t)row * d + col) = make_float4(x[v][0], x[v][1], x[v][2], x[v][3]);
#pragma unroll
      for (int j = 0; j < 4; ++j) s += x[v][j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[v][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 4;
    if (col < d) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = x[v][j] - mean;
        q += t * t;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)d + eps);
  const float* g = gamma + (int64_t)c * gcs;   // per-client γ/β rows: the arena views (client stride gcs)
  const float* b = beta + (int64_t)c * gcs;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 4;
    if (col < d) {
      const float4 gg = *reinterpret_cast<const float4*>(g + col);
      const float4 bb = *reinterpret_cast<const float4*>(b + col);
      *reinterpret_cast<float4*>(y + (size_t)row * d + col) =
          make_float4((x[v][0] - mean) * rstd * gg.x + bb.x, (x[v][1] - mean) * rstd * gg.y + bb.y,
                      (x[v][2] - mean) * rstd * gg.z + bb.z, (x[v][3] - mean) * rstd * gg.w + bb.w);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// backward: grid (blocks_per_client, C); each wave walks rows of one client keeping the d-wide
// dγ/dβ partial sums in registers; the 4 waves combine in LDS, one fp32 atomic per column and block
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     int rpc, int d, const float* __restrict__ gamma,
                                                     float* __restrict__ dx, float* __restrict__ dh, uint32_t thr,
                                                     float dscale, uint32_t seed, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta, const uint32_t* __restrict__ seedp,
                                                     int64_t gcs, int64_t dgcs, const float* __restrict__ dadd) {
  if (seedp) seed += *seedp * 1000003u;
  extern __shared__ float red[];   // [4][2][d]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.y;
  const float* g = gamma + (int64_t)c * gcs;
  float ag[NV][4], ab[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 4; ++j) ag[v][j] = ab[v][j] = 0.f;
  for (int r = blockIdx.x * 4 + wid; r < rpc; r += gridDim.x * 4) {
    const size_t row = (size_t)c * rpc + r;
    const float mu = mean[row], rs = rstd[row];
    float xh[NV][4], gd[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int col = (v * 64 + lane) * 4;
      if (col < d) {
        const float4 xv = *reinterpret_cast<const float4*>(x + row * d + col);
        const float4 gv = *reinterpret_cast<const float4*>(dy + row * d + col);
        const float4 gg = *reinterpret_cast<const float4*>(g + col);
        const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gy[4] = {gv.x, gv.y, gv.z, gv.w};
        const float gm[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[v][j] = (xs[j] - mu) * rs;
          gd[v][j] = gy[j] * gm[j];
          s1 += gd[v][j];
          s2 += gd[v][j] * xh[v][j];
          ag[v][j] += gy[j] * xh[v][j];
          ab[v][j] += gy[j];
        }
      }
    }
    s1 = wave_sum(s1) / (float)d;
    s2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int col = (v * 64 + lane) * 4;
      if (col < d) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = rs * (gd[v][j] - s1 - xh[v][j] * s2);
        if (dx) *reinterpret_cast<float4*>(dx + row * d + col) = make_float4(o[0], o[1], o[2], o[3]);
        if (dh) {
          if (thr) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              o[j] = fa_drop::keep(seed, (uint32_t)row, (uint32_t)(col + j), thr) ? o[j] * dscale : 0.f;
          }
          if (dadd) {   // the other consumer's gradient of the LN input (pre-LN residual stream)
            const float4 a4 = *reinterpret_cast<const float4*>(dadd + row * d + col);
            o[0] += a4.x; o[1] += a4.y; o[2] += a4.z; o[3] += a4.w;
          }
          *reinterpret_cast<float4*>(dh + row * d + col) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 4;
    if (col < d) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[(wid * 2 + 0) * d + col + j] = ag[v][j];
        red[(wid * 2 + 1) * d + col + j] = ab[v][j];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sg += red[(w * 2 + 0) * d + i];
      sb += red[(w * 2 + 1) * d + i];
    }
    fa_acc_add(dgamma + (int64_t)c * dgcs + i, sg);   // straight into the gradient arena rows when dgcs = ld
    fa_acc_add(dbeta + (int64_t)c * dgcs + i, sb);
  }
}

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<float4*>(y)[i] = make_float4(gelu_erf(v.x), gelu_erf(v.y), gelu_erf(v.z), gelu_erf(v.w));
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                                       float* __restrict__ gx, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const float4 g = reinterpret_cast<const float4*>(gy)[i];
    reinterpret_cast<float4*>(gx)[i] =
        make_float4(gelu_grad(v.x, g.x), gelu_grad(v.y, g.y), gelu_grad(v.z, g.z), gelu_grad(v.w, g.w));
  }
}

// db[c][n] += Σ_m g[c][m][n]: each thread owns one column (VEC = 4: four, as float4) of a row chunk, with
// independent partial sums so several row loads are in flight (a one-accumulator chain left the kernel
// latency-bound: 96 % of wave time waiting on memory); one fp32 atomic per column into the gradient arena
template <int VEC>
__global__ __launch_bounds__(256) void bias_grad_kernel(const float* __restrict__ g, int64_t g_bs, int ldg,
                                                        float* __restrict__ out, int64_t o_cs, Segs seg, int M, int N,
                                                        int rows_per_block) {
  const int c = blockIdx.z;
  const int n = (blockIdx.x * 256 + threadIdx.x) * VEC;
  if (n >= N) return;
  const int m0 = blockIdx.y * rows_per_block;
  const int m1 = min(M, m0 + rows_per_block);
  const float* gp = g + (int64_t)c * g_bs + n;
  float a[4][VEC];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < VEC; ++j) a[u][j] = 0.f;
  int m = m0;
  for (; m + 4 <= m1; m += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (VEC == 4) {
        const float4 v = *reinterpret_cast<const float4*>(gp + (int64_t)(m + u) * ldg);
        a[u][0] += v.x; a[u][1] += v.y; a[u][2] += v.z; a[u][3] += v.w;
      } else {
        a[u][0] += gp[(int64_t)(m + u) * ldg];
      }
    }
  }
  for (; m < m1; ++m) {
    if (VEC == 4) {
      const float4 v = *reinterpret_cast<const float4*>(gp + (int64_t)m * ldg);
      a[0][0] += v.x; a[0][1] += v.y; a[0][2] += v.z; a[0][3] += v.w;
    } else {
      a[0][0] += gp[(int64_t)m * ldg];
    }
  }
  // columns n .. n+3 share a segment (segment bounds are multiples of 4 on the VEC path)
  float* o = out + (int64_t)c * o_cs + seg_row(seg, n, 1);
#pragma unroll
  for (int j = 0; j < VEC; ++j) fa_acc_add(o + j, (a[0][j] + a[1][j]) + (a[2][j] + a[3][j]));
}

// =========================================================================================
// attention (fp32, head dim 64, S ≤ 256)
// =========================================================================================
constexpr float kLog2e = 1.4426950408889634f;
constexpr int AKP = 68;   // [64][68] chunks read as row fragments (and frag_tr): 16-B aligned rows
constexpr int AVP = 66;   // [64][66] chunks read only through frag_tr (≡ 2 mod 4: no 2-way bank split)

// rows [r0, r0+64) of one head's 64 columns into LDS (zero rows past S)
template <int PITCH>
__device__ __forceinline__ void stage64(float* dst, const float* src, int ld, int r0, int S) {
  for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
    const int r = i >> 4, ch = i & 15;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < S) v = *reinterpret_cast<const float4*>(src + (size_t)(r0 + r) * ld + 4 * ch);
    float* d = dst + r * PITCH + 4 * ch;
    if (PITCH % 4 == 0) {
      *reinterpret_cast<float4*>(d) = v;
    } else {
      reinterpret_cast<float2*>(d)[0] = make_float2(v.x, v.y);
      reinterpret_cast<float2*>(d)[1] = make_float2(v.z, v.w);
    }
  }
}

template <class P>
__device__ __forceinline__ typename P::frag_t zero_frag() {
  const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  return P::frag8(z);
}

// forward: grid (ceil(S/64), H, CB), 4 waves; wave w owns query rows q0 + 16w + [0, 16). All NB·16
// scores of the slice stay in registers (exact softmax over the full row), K then V stream through
// LDS in 64-key chunks; P goes through a per-wave LDS slice to become an A operand.
template <class P, int NB>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const float* __restrict__ q, int ldq,
                                                          const float* __restrict__ k, int ldk,
                                                          const float* __restrict__ v, int ldv, float* __restrict__ o,
                                                          int ldo, const uint8_t* __restrict__ kmask,
                                                          float* __restrict__ lse2, int S, int H, float scale,
                                                          uint32_t thr, float dscale, uint32_t seed,
                                                          const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  constexpr int NC = NB / 4;   // 64-key chunks
  __shared__ __attribute__((aligned(16))) float Ks[64 * AKP];
  __shared__ __attribute__((aligned(16))) float Vs[64 * AVP];
  __shared__ __attribute__((aligned(16))) float Ps[4 * 16 * AKP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int q0 = blockIdx.x * 64, h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const int qr = q0 + 16 * w + (lane & 15);   // A-operand row of this lane
  // wave-uniform skips of work that only touches padding (S not a multiple of 64, e.g. ViT's 197 tokens):
  // a wave whose 16 query rows are all ≥ S, and 16-key blocks / 32-key halves entirely ≥ S (their scores are
  // −∞ and their probabilities 0: skipping them leaves every result bit unchanged)
  const bool wrows = q0 + 16 * w < S;
  typename P::frag_t qf[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    qf[t] = qr < S ? P::frag(q + (tok0 + qr) * ldq + h * 64 + 32 * t + 8 * g) : zero_frag<P>();
  const float c2 = scale * kLog2e;

  f32x4 sc[NB];
#pragma unroll
  for (int kc = 0; kc < NC; ++kc) {
    __syncthreads();
    stage64<AKP>(Ks, k + tok0 * ldk + h * 64, ldk, kc * 64, S);
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (wrows && kc * 64 + nb * 16 < S) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc = P::mma(qf[t], P::frag(Ks + (nb * 16 + (lane & 15)) * AKP + 32 * t + 8 * g), acc);
      }
      const int key = kc * 64 + nb * 16 + (lane & 15);
      const bool valid = key < S && (kmask == nullptr || kmask[tok0 + key] != 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[kc * 4 + nb][r] = valid ? acc[r] * c2 : -INFINITY;
    }
  }
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float mx = -INFINITY;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) mx = fmaxf(mx, sc[nb][r]);
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    m[r] = mx;
    l[r] = 0.f;
  }
  const int qbase = q0 + 16 * w + 4 * g;   // C-layout query row of reg 0
  const uint32_t bh = (uint32_t)(cb * H + h);
  float* Pw = Ps + w * 16 * AKP;
  f32x4 ao[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) ao[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < NC; ++kc) {
    __syncthreads();   // every wave is done with the previous V chunk
    stage64<AVP>(Vs, v + tok0 * ldv + h * 64, ldv, kc * 64, S);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int kl = nb * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pr = m[r] == -INFINITY ? 0.f : exp2f(sc[kc * 4 + nb][r] - m[r]);
        l[r] += pr;
        if (thr) pr = fa_drop::keep(seed, bh * 65536u + (uint32_t)(qbase + r), (uint32_t)(kc * 64 + kl), thr) ? pr * dscale : 0.f;
        Pw[(4 * g + r) * AKP + kl] = pr;
      }
    }
    __syncthreads();
    if (wrows) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (kc * 64 + 32 * kt >= S) continue;
#pragma unroll
        for (int db = 0; db < 4; ++db)
          ao[db] = P::mma(P::frag(Pw + (lane & 15) * AKP + 32 * kt + 8 * g),
                          P::frag_tr(Vs, AVP, 32 * kt, 16 * db, lane), ao[db]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) l[r] += __shfl_xor(l[r], off, 64);
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qq = qbase + r;
      if (qq < S) o[(tok0 + qq) * ldo + h * 64 + 16 * db + (lane & 15)] = l[r] > 0.f ? ao[db][r] / l[r] : 0.f;
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qq = qbase + r;
      if (qq < S) lse2[((size_t)cb * H + h) * S + qq] = l[r] > 0.f ? m[r] + log2f(l[r]) : INFINITY;
    }
  }
}

// D[cb, h, q] = Σ_dim dO·O  (one thread per (token, head))
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const float* __restrict__ o, int ldo,
                                                            const float* __restrict__ dout, int lddo,
                                                            float* __restrict__ D, int CBS, int S, int H) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)CBS * H) return;
  const int h = (int)(i % H);
  const int64_t tok = i / H;
  float s = 0.f;
#pragma unroll
  for (int ch = 0; ch < 16; ++ch) {
    const float4 a = *reinterpret_cast<const float4*>(o + tok * ldo + h * 64 + 4 * ch);
    const float4 b = *reinterpret_cast<const float4*>(dout + tok * lddo + h * 64 + 4 * ch);
    s += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
  }
  const int64_t cb = tok / S, qq = tok % S;
  D[(cb * H + h) * S + qq] = s;
}

// dQ: grid (ceil(S/64), H, CB); wave w owns 16 query rows, loops over 64-key chunks
template <class P>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(const float* __restrict__ q, int ldq,
                                                             const float* __restrict__ k, int ldk,
                                                             const float* __restrict__ v, int ldv,
                                                             const float* __restrict__ dout, int lddo,
                                                             const uint8_t* __restrict__ kmask,
                                                             const float* __restrict__ lse2,
                                                             const float* __restrict__ D, float* __restrict__ dq,
                                                             int lddq, int S, int H, float scale, uint32_t thr,
                                                             float dscale, uint32_t seed,
                                                             const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  __shared__ __attribute__((aligned(16))) float Ks[64 * AKP];
  __shared__ __attribute__((aligned(16))) float Vs[64 * AKP];
  __shared__ __attribute__((aligned(16))) float dSs[4 * 16 * AKP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const size_t bhS = ((size_t)cb * H + h) * S;
  const int qr = blockIdx.x * 64 + 16 * w + (lane & 15);
  const bool wrows = blockIdx.x * 64 + 16 * w < S;   // wave-uniform padding skips, as in the forward
  typename P::frag_t qf[2], df[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    qf[t] = qr < S ? P::frag(q + (tok0 + qr) * ldq + h * 64 + 32 * t + 8 * g) : zero_frag<P>();
    df[t] = qr < S ? P::frag(dout + (tok0 + qr) * lddo + h * 64 + 32 * t + 8 * g) : zero_frag<P>();
  }
  const int qbase = blockIdx.x * 64 + 16 * w + 4 * g;
  float Lr[4], Dr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qq = qbase + r;
    Lr[r] = qq < S ? lse2[bhS + qq] : INFINITY;
    Dr[r] = qq < S ? D[bhS + qq] : 0.f;
  }
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  float* dS = dSs + w * 16 * AKP;
  f32x4 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) acc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < S; k0 += 64) {
    __syncthreads();
    stage64<AKP>(Ks, k + tok0 * ldk + h * 64, ldk, k0, S);
    stage64<AKP>(Vs, v + tok0 * ldv + h * 64, ldv, k0, S);
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      if (wrows && k0 + nb * 16 < S) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int off = (nb * 16 + (lane & 15)) * AKP + 32 * t + 8 * g;
          s = P::mma(qf[t], P::frag(Ks + off), s);
          dp = P::mma(df[t], P::frag(Vs + off), dp);
        }
      }
      const int key = k0 + nb * 16 + (lane & 15);
      const bool valid = key < S && (kmask == nullptr || kmask[tok0 + key] != 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = valid ? exp2f(s[r] * c2 - Lr[r]) : 0.f;
        float gr = dp[r];
        if (thr) gr = fa_drop::keep(seed, bh * 65536u + (uint32_t)(qbase + r), (uint32_t)key, thr) ? gr * dscale : 0.f;
        dS[(4 * g + r) * AKP + nb * 16 + (lane & 15)] = pr * (gr - Dr[r]);
      }
    }
    __syncthreads();
    if (wrows) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (k0 + 32 * kt >= S) continue;
#pragma unroll
        for (int db = 0; db < 4; ++db)
          acc[db] = P::mma(P::frag(dS + (lane & 15) * AKP + 32 * kt + 8 * g),
                           P::frag_tr(Ks, AKP, 32 * kt, 16 * db, lane), acc[db]);
      }
    }
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qq = qbase + r;
      if (qq < S) dq[(tok0 + qq) * lddq + h * 64 + 16 * db + (lane & 15)] = acc[db][r] * scale;
    }
}

// dK, dV: grid (ceil(S/64), H, CB); wave w owns 16 keys, loops over 64-query chunks
template <class P>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_kernel(const float* __restrict__ q, int ldq,
                                                              const float* __restrict__ k, int ldk,
                                                              const float* __restrict__ v, int ldv,
                                                              const float* __restrict__ dout, int lddo,
                                                              const uint8_t* __restrict__ kmask,
                                                              const float* __restrict__ lse2,
                                                              const float* __restrict__ D, float* __restrict__ dk,
                                                              int lddk, float* __restrict__ dv, int lddv, int S, int H,
                                                              float scale, uint32_t thr, float dscale, uint32_t seed,
                                                              const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  __shared__ __attribute__((aligned(16))) float Qs[64 * AKP];
  __shared__ __attribute__((aligned(16))) float dOs[64 * AKP];
  __shared__ __attribute__((aligned(16))) float Pst[4 * 16 * AKP];
  __shared__ __attribute__((aligned(16))) float dSt[4 * 16 * AKP];
  __shared__ float Ls[64], Dsh[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const size_t bhS = ((size_t)cb * H + h) * S;
  const int kr = blockIdx.x * 64 + 16 * w + (lane & 15);
  const bool wkeys = blockIdx.x * 64 + 16 * w < S;   // wave-uniform padding skips, as in the forward
  typename P::frag_t kf[2], vf[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    kf[t] = kr < S ? P::frag(k + (tok0 + kr) * ldk + h * 64 + 32 * t + 8 * g) : zero_frag<P>();
    vf[t] = kr < S ? P::frag(v + (tok0 + kr) * ldv + h * 64 + 32 * t + 8 * g) : zero_frag<P>();
  }
  const int kbase = blockIdx.x * 64 + 16 * w + 4 * g;   // C-layout key of reg 0
  bool kvalid[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kk = kbase + r;
    kvalid[r] = kk < S && (kmask == nullptr || kmask[tok0 + kk] != 0);
  }
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  float* Pw = Pst + w * 16 * AKP;
  float* dSw = dSt + w * 16 * AKP;
  f32x4 adk[4], adv[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) adk[db] = adv[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int q0 = 0; q0 < S; q0 += 64) {
    __syncthreads();
    stage64<AKP>(Qs, q + tok0 * ldq + h * 64, ldq, q0, S);
    stage64<AKP>(dOs, dout + tok0 * lddo + h * 64, lddo, q0, S);
    if (threadIdx.x < 64) {
      const int qq = q0 + threadIdx.x;
      Ls[threadIdx.x] = qq < S ? lse2[bhS + qq] : INFINITY;
      Dsh[threadIdx.x] = qq < S ? D[bhS + qq] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
      if (wkeys && q0 + nb * 16 < S) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int off = (nb * 16 + (lane & 15)) * AKP + 32 * t + 8 * g;
          st = P::mma(kf[t], P::frag(Qs + off), st);
          dpt = P::mma(vf[t], P::frag(dOs + off), dpt);
        }
      }
      const int ql = nb * 16 + (lane & 15);
      const int qq = q0 + ql;
      const float Lq = Ls[ql], Dq = Dsh[ql];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = kvalid[r] && qq < S;
        const float pr = valid ? exp2f(st[r] * c2 - Lq) : 0.f;
        float pd = pr, gr = dpt[r];
        if (thr) {
          const bool kp = fa_drop::keep(seed, bh * 65536u + (uint32_t)qq, (uint32_t)(kbase + r), thr);
          pd = kp ? pr * dscale : 0.f;
          gr = kp ? gr * dscale : 0.f;
        }
        Pw[(4 * g + r) * AKP + ql] = pd;
        dSw[(4 * g + r) * AKP + ql] = pr * (gr - Dq);
      }
    }
    __syncthreads();
    if (wkeys) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (q0 + 32 * kt >= S) continue;
        const int ao = (lane & 15) * AKP + 32 * kt + 8 * g;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          adv[db] = P::mma(P::frag(Pw + ao), P::frag_tr(dOs, AKP, 32 * kt, 16 * db, lane), adv[db]);
          adk[db] = P::mma(P::frag(dSw + ao), P::frag_tr(Qs, AKP, 32 * kt, 16 * db, lane), adk[db]);
        }
      }
    }
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kk = kbase + r;
      if (kk < S) {
        dk[(tok0 + kk) * lddk + h * 64 + 16 * db + (lane & 15)] = adk[db][r] * scale;
        dv[(tok0 + kk) * lddv + h * 64 + 16 * db + (lane & 15)] = adv[db][r];
      }
    }
}

template <class P, int NB>
int launch_attn_fwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, float* o, int ldo,
                    const uint8_t* kmask, float* lse2, int CB, int S, int H, float scale, uint32_t thr, float dscale,
                    uint32_t seed, const uint32_t* seedp, hipStream_t st) {
  hipLaunchKernelGGL((attn_fwd_kernel<P, NB>), dim3((S + 63) / 64, H, CB), dim3(256), 0, st, q, ldq, k, ldk, v, ldv,
                     o, ldo, kmask, lse2, S, H, scale, thr, dscale, seed, seedp);
  return (int)hipGetLastError();
}

template <class P>
int attn_fwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, float* o, int ldo,
             const uint8_t* kmask, float* lse2, int CB, int S, int H, float scale, uint32_t thr, float dscale,
             uint32_t seed, const uint32_t* seedp, hipStream_t st) {
  if (S <= 64) return launch_attn_fwd<P, 4>(q, ldq, k, ldk, v, ldv, o, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, st);
  if (S <= 128) return launch_attn_fwd<P, 8>(q, ldq, k, ldk, v, ldv, o, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, st);
  if (S <= 192) return launch_attn_fwd<P, 12>(q, ldq, k, ldk, v, ldv, o, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, st);
  return launch_attn_fwd<P, 16>(q, ldq, k, ldk, v, ldv, o, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, st);
}

template <class P>
int attn_bwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, const float* dout, int lddo,
             const uint8_t* kmask, const float* lse2, const float* D, float* dq, int lddq, float* dk, int lddk,
             float* dv, int lddv, int CB, int S, int H, float scale, uint32_t thr, float dscale, uint32_t seed,
             const uint32_t* seedp, hipStream_t st) {
  const dim3 grid((S + 63) / 64, H, CB);
  hipLaunchKernelGGL(attn_bwd_dq_kernel<P>, grid, dim3(256), 0, st, q, ldq, k, ldk, v, ldv, dout, lddo, kmask, lse2,
                     D, dq, lddq, S, H, scale, thr, dscale, seed, seedp);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<P>, grid, dim3(256), 0, st, q, ldq, k, ldk, v, ldv, dout, lddo, kmask, lse2,
                     D, dk, lddk, dv, lddv, S, H, scale, thr, dscale, seed, seedp);
  return (int)hipGetLastError();
}

}  // namespace tff

// =========================================================================================
// C ABI (checked by ops/transformer_ops.py before launch)
// =========================================================================================
// y[c] = x[c] · W[c]ᵀ + b[c] (gelu: y2 = gelu(y)); W, b: fp32 arena row segments
FA_EXPORT int fa_bgemm_fwd_f32(const float* x, int64_t x_bs, int ldx, const float* w_base, int64_t w_cs,
                               const int64_t* w_off, const float* b_base, int64_t b_cs, const int64_t* b_off,
                               const int* seg_lo, int nseg, float* y, int64_t y_bs, int ldy, float* y2, int C, int M,
                               int N, int K, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = x; a.a_bs = x_bs; a.lda = ldx;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = y; a.c_bs = y_bs; a.ldc = ldy;
  a.bias = b_base; a.bias_bs = b_cs;
  fill_segs(a.biasseg, b_off, seg_lo, nseg);
  a.C2 = y2;
  a.M = M; a.N = N; a.K = K;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (N + BN - 1) / BN; a.nclients = C;
  const bool vec = al4({x_bs, ldx, K, w_cs, b_cs, y_bs, ldy, N}) && segs_al4(a.bseg) && (!b_base || segs_al4(a.biasseg)) &&
                   al16({x, w_base, b_base, y, y2});
  if (y2) FA_F32_DISPATCH(tff, (launch_gemm<PX, 0, 0, EPI_GELU>(a, vec, stream)));
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 0, 0, EPI_STORE>(a, vec, stream)));
}

// y[c] = x[c] · W[c]ᵀ + b[c] + res[c]   (no GELU; res [C][M][ldr], may alias nothing it reads)
FA_EXPORT int fa_bgemm_fwd_res_f32(const float* x, int64_t x_bs, int ldx, const float* w_base, int64_t w_cs,
                                   const int64_t* w_off, const float* b_base, int64_t b_cs, const int64_t* b_off,
                                   const int* seg_lo, int nseg, float* y, int64_t y_bs, int ldy, const float* res,
                                   int64_t r_bs, int ldr, int C, int M, int N, int K, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || M <= 0 || N <= 0 || K <= 0 || !res) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = x; a.a_bs = x_bs; a.lda = ldx;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = y; a.c_bs = y_bs; a.ldc = ldy;
  a.bias = b_base; a.bias_bs = b_cs;
  fill_segs(a.biasseg, b_off, seg_lo, nseg);
  a.R = res; a.r_bs = r_bs; a.ldr = ldr;
  a.M = M; a.N = N; a.K = K;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (N + BN - 1) / BN; a.nclients = C;
  const bool vec = al4({x_bs, ldx, K, w_cs, b_cs, y_bs, ldy, N, r_bs, ldr}) && segs_al4(a.bseg) &&
                   (!b_base || segs_al4(a.biasseg)) && al16({x, w_base, b_base, y, res});
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 0, 0, EPI_STORE>(a, vec, stream)));
}

// dx[c] = dy[c] · W[c]    dy [M][N], W [N][K] arena segments (rows n = the reduction index), dx [M][K]
FA_EXPORT int fa_bgemm_dgrad_f32(const float* dy, int64_t dy_bs, int lddy, const float* w_base, int64_t w_cs,
                                 const int64_t* w_off, const int* seg_lo, int nseg, float* dx, int64_t dx_bs, int lddx,
                                 int C, int M, int N, int K, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = dx; a.c_bs = dx_bs; a.ldc = lddx;
  a.M = M; a.N = K; a.K = N;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  const bool vec = al4({dy_bs, lddy, N, w_cs, K, dx_bs, lddx}) && segs_al4(a.bseg) && al16({dy, w_base, dx});
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 0, 1, EPI_STORE>(a, vec, stream)));
}

// dx[c] = (dy[c] · W[c]) ⊙ gelu'(pre[c])   pre [C][M][K] (the pre-activation of the GELU that produced x)
FA_EXPORT int fa_bgemm_dgrad_dgelu_f32(const float* dy, int64_t dy_bs, int lddy, const float* w_base, int64_t w_cs,
                                       const int64_t* w_off, const int* seg_lo, int nseg, float* dx, int64_t dx_bs,
                                       int lddx, const float* pre, int C, int M, int N, int K, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || M <= 0 || N <= 0 || K <= 0 || !pre) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = dx; a.c_bs = dx_bs; a.ldc = lddx;
  a.R = pre; a.r_bs = dx_bs; a.ldr = lddx;
  a.M = M; a.N = K; a.K = N;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  const bool vec = al4({dy_bs, lddy, N, w_cs, K, dx_bs, lddx}) && segs_al4(a.bseg) && al16({dy, w_base, dx, pre});
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 0, 1, EPI_DGELU>(a, vec, stream)));
}

// dx[c] += dy[c] · W[c]   (accumulating form: the residual-stream gradient the caller already holds in dx —
// a post-LN block's input feeds both the next LayerNorm's residual and this linear)
FA_EXPORT int fa_bgemm_dgrad_acc_f32(const float* dy, int64_t dy_bs, int lddy, const float* w_base, int64_t w_cs,
                                     const int64_t* w_off, const int* seg_lo, int nseg, float* dx, int64_t dx_bs,
                                     int lddx, int C, int M, int N, int K, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = dx; a.c_bs = dx_bs; a.ldc = lddx;
  fill_segs(a.cseg, nullptr, nullptr, 1);   // one plain [M][lddx] matrix per client
  a.M = M; a.N = K; a.K = N;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  const bool vec = al4({dy_bs, lddy, N, w_cs, K, dx_bs, lddx}) && segs_al4(a.bseg) && al16({dy, w_base, dx});
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 0, 1, EPI_ACC>(a, vec, stream)));
}

// dW[c] += dy[c]ᵀ · x[c]    dy [T][N], x [T][K]; dW [N][K] gradient-arena segments (rows n)
FA_EXPORT int fa_bgemm_wgrad_st_f32(const float* dy, int64_t dy_bs, int lddy, const float* x, int64_t x_bs, int ldx,
                                    float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo, int nseg,
                                    int C, int T, int N, int K, int store, hipStream_t stream);
FA_EXPORT int fa_bgemm_wgrad_f32(const float* dy, int64_t dy_bs, int lddy, const float* x, int64_t x_bs, int ldx,
                                 float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo, int nseg, int C,
                                 int T, int N, int K, hipStream_t stream) {
  return fa_bgemm_wgrad_st_f32(dy, dy_bs, lddy, x, x_bs, ldx, g_base, g_cs, g_off, seg_lo, nseg, C, T, N, K, 0, stream);
}
// store = 1: dW[c] = dy[c]ᵀ · x[c] (the rows' first writer: no zero fill needed), else dW[c] += …
FA_EXPORT int fa_bgemm_wgrad_st_f32(const float* dy, int64_t dy_bs, int lddy, const float* x, int64_t x_bs, int ldx,
                                    float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo, int nseg,
                                    int C, int T, int N, int K, int store, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || T <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = x; a.b_bs = x_bs; a.ldb = ldx;
  fill_segs(a.bseg, nullptr, nullptr, 1);
  a.Cp = g_base; a.c_bs = g_cs; a.ldc = K;
  fill_segs(a.cseg, g_off, seg_lo, nseg);
  a.M = N; a.N = K; a.K = T;
  a.tiles_m = (N + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  a.acc_store = store;
  const bool vec = al4({dy_bs, lddy, N, x_bs, ldx, K, g_cs}) && segs_al4(a.cseg) && al16({dy, x, g_base});
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 1, 1, EPI_ACC>(a, vec, stream)));
}

// dW[c] += dy[c]ᵀ · x[c] and db[c] += Σ_t dy[c][t][:] in one pass over dy (bias segments share seg_lo);
// store = 1: = instead of += for both (the rows' first writer)
FA_EXPORT int fa_bgemm_wgrad_bias_f32(const float* dy, int64_t dy_bs, int lddy, const float* x, int64_t x_bs,
                                      int ldx, float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo,
                                      int nseg, float* b_base, int64_t b_cs, const int64_t* b_off, int C, int T, int N,
                                      int K, int store, hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || T <= 0 || N <= 0 || K <= 0 || !b_base) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = x; a.b_bs = x_bs; a.ldb = ldx;
  fill_segs(a.bseg, nullptr, nullptr, 1);
  a.Cp = g_base; a.c_bs = g_cs; a.ldc = K;
  fill_segs(a.cseg, g_off, seg_lo, nseg);
  a.bg = b_base; a.bg_bs = b_cs;
  fill_segs(a.bgseg, b_off, seg_lo, nseg);
  a.M = N; a.N = K; a.K = T;
  a.tiles_m = (N + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  a.acc_store = store;
  const bool vec = al4({dy_bs, lddy, N, x_bs, ldx, K, g_cs, b_cs}) && segs_al4(a.cseg) && segs_al4(a.bgseg) &&
                   al16({dy, x, g_base, b_base});
  if (!vec) return -2;   // the caller falls back to the separate bias reduction
  FA_F32_DISPATCH(tff, (launch_gemm<PX, 1, 1, EPI_ACC>(a, vec, stream)));
}

// db[c] += Σ_m dy[c][m][:]   dy fp32 [C][M][N]; db: fp32 arena segments
FA_EXPORT int fa_bias_grad_f32(const float* dy, int64_t dy_bs, int lddy, float* o_base, int64_t o_cs,
                               const int64_t* o_off, const int* seg_lo, int nseg, int C, int M, int N,
                               hipStream_t stream) {
  using namespace tff;
  if (nseg < 1 || nseg > 4 || C <= 0 || M <= 0 || N <= 0 || C > 65535) return (int)hipErrorInvalidValue;
  Segs sg;
  fill_segs(sg, o_off, seg_lo, nseg);
  const int rpb = 128;
  const bool vec = al4({dy_bs, lddy, N}) && segs_al4(sg) && al16({dy});
  const int cols = vec ? N / 4 : N;
  dim3 grid((unsigned)((cols + 255) / 256), (unsigned)((M + rpb - 1) / rpb), (unsigned)C);
  if (vec)
    hipLaunchKernelGGL(bias_grad_kernel<4>, grid, dim3(256), 0, stream, dy, dy_bs, lddy, o_base, o_cs, sg, M, N, rpb);
  else
    hipLaunchKernelGGL(bias_grad_kernel<1>, grid, dim3(256), 0, stream, dy, dy_bs, lddy, o_base, o_cs, sg, M, N, rpb);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_ln_fwd_f32(const float* h, const float* res, int R, int d, int rows_per_client, const float* gamma,
                            const float* beta, float eps, uint32_t thr, float dscale, uint32_t seed, float* y,
                            float* xsum, float* mean, float* rstd, const uint32_t* seedp, int64_t gcs,
                            hipStream_t stream) {
  using namespace tff;
  if (d % 4 != 0 || d > 2048 || R <= 0 || gcs % 4 != 0) return (int)hipErrorInvalidValue;
  const dim3 grid((R + 3) / 4);
#define TFF_LNF(NV) \
  hipLaunchKernelGGL(ln_fwd_kernel<NV>, grid, dim3(256), 0, stream, h, res, R, d, rows_per_client, gamma, beta, eps, \
                     thr, dscale, seed, y, xsum, mean, rstd, seedp, gcs)
  if (d <= 256) TFF_LNF(1);
  else if (d <= 512) TFF_LNF(2);
  else if (d <= 768) TFF_LNF(3);
  else if (d <= 1024) TFF_LNF(4);
  else TFF_LNF(8);
#undef TFF_LNF
  return (int)hipGetLastError();
}

// dadd (optional): added to dh (the gradient of the LN input h) — the residual stream's other gradient
FA_EXPORT int fa_ln_bwd_add_f32(const float* dy, const float* x, const float* mean, const float* rstd, int C,
                                int rows_per_client, int d, const float* gamma, float* dx, float* dh, uint32_t thr,
                                float dscale, uint32_t seed, float* dgamma, float* dbeta, const uint32_t* seedp,
                                int64_t gcs, int64_t dgcs, const float* dadd, hipStream_t stream);

FA_EXPORT int fa_ln_bwd_f32(const float* dy, const float* x, const float* mean, const float* rstd, int C,
                            int rows_per_client, int d, const float* gamma, float* dx, float* dh, uint32_t thr,
                            float dscale, uint32_t seed, float* dgamma, float* dbeta, const uint32_t* seedp,
                            int64_t gcs, int64_t dgcs, hipStream_t stream) {
  return fa_ln_bwd_add_f32(dy, x, mean, rstd, C, rows_per_client, d, gamma, dx, dh, thr, dscale, seed, dgamma, dbeta,
                           seedp, gcs, dgcs, nullptr, stream);
}

FA_EXPORT int fa_ln_bwd_add_f32(const float* dy, const float* x, const float* mean, const float* rstd, int C,
                                int rows_per_client, int d, const float* gamma, float* dx, float* dh, uint32_t thr,
                                float dscale, uint32_t seed, float* dgamma, float* dbeta, const uint32_t* seedp,
                                int64_t gcs, int64_t dgcs, const float* dadd, hipStream_t stream) {
  using namespace tff;
  if (d % 4 != 0 || d > 2048 || C <= 0 || C > 65535 || gcs % 4 != 0) return (int)hipErrorInvalidValue;
  int bpc = (rows_per_client + 31) / 32;   // ≥ 8 rows per wave
  if (bpc < 1) bpc = 1;
  if (bpc > 1024) bpc = 1024;
  const dim3 grid(bpc, C);
  const size_t sm = 8 * (size_t)d * sizeof(float);
#define TFF_LNB(NV) \
  hipLaunchKernelGGL(ln_bwd_kernel<NV>, grid, dim3(256), sm, stream, dy, x, mean, rstd, rows_per_client, d, gamma, dx, \
                     dh, thr, dscale, seed, dgamma, dbeta, seedp, gcs, dgcs, dadd)
  if (d <= 256) TFF_LNB(1);
  else if (d <= 512) TFF_LNB(2);
  else if (d <= 768) TFF_LNB(3);
  else if (d <= 1024) TFF_LNB(4);
  else TFF_LNB(8);
#undef TFF_LNB
  return (int)hipGetLastError();
}

FA_EXPORT int fa_gelu_fwd_f32(const float* x, float* y, int64_t n, hipStream_t stream) {
  if (n % 4 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tff::gelu_fwd_kernel, dim3(fa_grid(n / 4, 256, 8192)), dim3(256), 0, stream, x, y, n / 4);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_gelu_bwd_f32(const float* x, const float* gy, float* gx, int64_t n, hipStream_t stream) {
  if (n % 4 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tff::gelu_bwd_kernel, dim3(fa_grid(n / 4, 256, 8192)), dim3(256), 0, stream, x, gy, gx, n / 4);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_attn_fwd_f32(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, float* o,
                              int ldo, const uint8_t* kmask, float* lse2, int CB, int S, int H, float scale,
                              uint32_t thr, float dscale, uint32_t seed, const uint32_t* seedp, hipStream_t stream) {
  if (S <= 0 || S > 256 || H <= 0 || H > 65535 || CB <= 0 || CB > 65535 || (ldq | ldk | ldv | ldo) % 4 != 0)
    return (int)hipErrorInvalidValue;
  FA_F32_DISPATCH(tff, tff::attn_fwd<PX>(q, ldq, k, ldk, v, ldv, o, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed,
                                         seedp, stream));
}

FA_EXPORT int fa_attn_bwd_f32(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, const float* o,
                              int ldo, const float* dout, int lddo, const uint8_t* kmask, const float* lse2, float* Dbuf,
                              float* dq, int lddq, float* dk, int lddk, float* dv, int lddv, int CB, int S, int H,
                              float scale, uint32_t thr, float dscale, uint32_t seed, const uint32_t* seedp,
                              hipStream_t stream) {
  if (S <= 0 || S > 4096 || H <= 0 || H > 65535 || CB <= 0 || CB > 65535 ||
      (ldq | ldk | ldv | ldo | lddo | lddq | lddk | lddv) % 4 != 0)
    return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)CB * S * H;
  hipLaunchKernelGGL(tff::attn_bwd_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, o, ldo, dout,
                     lddo, Dbuf, CB * S, S, H);
  FA_F32_DISPATCH(tff, tff::attn_bwd<PX>(q, ldq, k, ldk, v, ldv, dout, lddo, kmask, lse2, Dbuf, dq, lddq, dk, lddk, dv,
                                         lddv, CB, S, H, scale, thr, dscale, seed, seedp, stream));
}
