// Client-batched GEMMs for the transformer linears of the virtual-client engine
// (gfx950, wave64, bf16 MFMA v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// Every virtual client c owns private weights that live in the fp32 client arena [C][P]
// (row stride P, one slot per state_dict key). One launch runs the same linear for all C
// clients; the weights are read straight from the arena (converted to bf16 while staging
// into LDS — no per-step bf16 weight copies) and weight gradients are added straight into
// the fp32 gradient arena. A fused q/k/v projection is ONE GEMM whose weight rows come from
// three arena slots ("segments").
//
//   logical GEMM per client:  D[m][n] = Σ_k A(m, k) · B(n, k)
//   forward      y  = x · Wᵀ + b      A = x  [M][K]            B = W  [N][K] (arena, fp32)
//   bwd-data     dx = dy · W          A = dy [M][N]            B = Wᵀ: storage W[n][k], k-major → "TR"
//   bwd-weight   dW += dyᵀ · x        A = dyᵀ: storage dy[t][n] "TR"  B = xᵀ: storage x[t][k] "TR"
//
// An operand whose storage rows run along the REDUCTION index ("TR") is staged into LDS in its
// natural layout and its MFMA fragments are read with gfx950's transposing LDS read
// ds_read_b64_tr_b16; a K-major operand is read with plain 16-byte LDS reads.
// Block tile 128×128×64, 4 waves × (64×64), register-staged double-buffered LDS, XCD-aware
// block order (consecutive tiles of one client/row-block on one XCD → shared A rows in its L2).
// The MFMA computes the transposed tile D[n][m], so each lane owns 4 consecutive output columns
// of one row: 8-byte bf16 / 16-byte fp32 epilogue accesses, bias as one float4.
#include "common.h"
#include <cstdlib>
#include "detacc.h"

FA_DET_EXPORT(bgemm)

namespace bg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int LDK = BK + 8;    // K-major tile [128 rows][64 k] row pitch (elements)
constexpr int LDT = BM + 16;   // TR tile [64 k][128 cols] row pitch (elements)
constexpr int TILE_ELEMS = 128 * LDK;  // == 64 * LDT (18 KiB per operand tile)
static_assert(128 * LDK == 64 * LDT, "tile images must be the same size");

// EPI_DGELU: the data gradient of a GELU'd linear's output taken through the GELU, D ⊙ gelu'(R) (R = its bf16
// pre-activation) — the consumer's dgrad absorbs the GELU backward pass
enum { EPI_BF16 = 0, EPI_GELU = 1, EPI_ACC32 = 2, EPI_DGELU = 3 };

struct Segs {        // row segments of an fp32 arena operand (≤ 4 slots)
  int64_t off[4];    // element offset of segment s's first row, relative to the base pointer
  int lo[5];         // first logical row of segment s (lo[n] = total rows)
  int n;
};

struct Args {
  const uint16_t* A;
  int64_t a_bs;
  int lda;
  const void* B;     // bf16 [C][..] (b_bs, ldb) or fp32 arena base (b_bs = client stride, ldb = row length)
  int64_t b_bs;
  int ldb;
  Segs bseg;
  void* Cp;          // bf16 [C][M][ldc] (EPI_BF16/GELU) or fp32 arena base (EPI_ACC32, rows = segs)
  int64_t c_bs;
  int ldc;
  Segs cseg;
  const float* bias; // fp32 arena base (client stride bias_bs), rows = n segments (may be null)
  int64_t bias_bs;
  Segs biasseg;
  uint16_t* C2;      // EPI_GELU: gelu(D + b) (C keeps the pre-activation for the backward)
  int64_t c2_bs;
  const uint16_t* R; // EPI_BF16: optional residual addend [C][M][ldc] (D = A·Bᵀ + b + R); EPI_DGELU: pre-activation
  int64_t r_bs;
  float* bg;         // EPI_ACC32 (weight gradient): optional bias gradient Σ_t A[t][m] (segmented rows, tn == 0 blocks)
  int64_t bg_bs;
  Segs bgseg;
  int M, N, K;
  int tiles_m, tiles_n, nclients;
  int acc_store;     // EPI_ACC32: the rows' first (only) writer — store instead of += (no zero fill of those rows)
  int64_t a_bytes, b_bytes;   // LDS-DMA kernel: per-client operand extents its buffer descriptors bound
  int stage_epi;              // LDS-DMA kernel: bf16 epilogue staged through LDS (16-B row-contiguous stores)
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

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

__device__ __forceinline__ bf16x8 row_frag(const uint16_t* tile, int row, int k) {
  return *reinterpret_cast<const bf16x8*>(tile + row * LDK + k);
}

// 8 consecutive reduction rows (row0 + 8·(lane>>4) + j) of column col0 + (lane & 15)
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* tile, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const uint16_t* a0 = tile + (row0 + 8 * g + q) * LDT + col0 + 4 * p;
  const v4i16 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  const v4i16 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0 + 4 * LDT));
  union {
    short s[8];
    bf16x8 b;
  } u;
  u.s[0] = r0[0]; u.s[1] = r0[1]; u.s[2] = r0[2]; u.s[3] = r0[3];
  u.s[4] = r1[0]; u.s[5] = r1[1]; u.s[6] = r1[2]; u.s[7] = r1[3];
  return u.b;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x, float g) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return g * (cdf + x * pdf);
}

// ---- staging of one bf16 operand tile (4 × 16-byte vectors per thread) ----
// TR = 0: logical rows [r0, r0+128) × k [k0, k0+64) of storage S[row][k]  (pitch ld)
// TR = 1: storage S[k][col]: k rows [k0, k0+64) × cols [r0, r0+128)       (pitch ld)
template <int TR>
__device__ __forceinline__ void load_bf16(uint4 (&r)[4], const uint16_t* __restrict__ S, int ld, int rows, int K,
                                          int r0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    int row, col;
    bool ok;
    if (!TR) {
      row = r0 + (v >> 3);
      col = k0 + 8 * (v & 7);
      ok = row < rows && col < K;
    } else {
      row = k0 + (v >> 4);
      col = r0 + 8 * (v & 15);
      ok = row < K && col < rows;
    }
    r[i] = ok ? *reinterpret_cast<const uint4*>(S + (int64_t)row * ld + col) : make_uint4(0, 0, 0, 0);
  }
}

// B operand in bf16 with segmented rows (the bf16 weight shadow of the arena, or a plain [rows][ld]
// matrix as one segment at offset 0)
template <int TR>
__device__ __forceinline__ void load_bf16_seg(uint4 (&r)[4], const uint16_t* __restrict__ base, const Segs& sg,
                                              int rowlen, int rows, int K, int r0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    int srow, col;
    bool ok;
    if (!TR) {
      srow = r0 + (v >> 3);
      col = k0 + 8 * (v & 7);
      ok = srow < rows && col < K;
    } else {
      srow = k0 + (v >> 4);
      col = r0 + 8 * (v & 15);
      ok = srow < K && col < rows;
    }
    r[i] = ok ? *reinterpret_cast<const uint4*>(base + seg_row(sg, srow, rowlen) + col) : make_uint4(0, 0, 0, 0);
  }
}

template <int TR>
__device__ __forceinline__ void store_bf16(uint16_t* tile, const uint4 (&r)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    const int off = TR ? (v >> 4) * LDT + 8 * (v & 15) : (v >> 3) * LDK + 8 * (v & 7);
    *reinterpret_cast<uint4*>(tile + off) = r[i];
  }
}

// ---- fp32 arena operand (segmented rows), converted to bf16 at the LDS write ----
// TR = 0: storage row = logical row n (segmented), elements k.   TR = 1: storage row = k (segmented), cols n.
template <int TR>
__device__ __forceinline__ void load_f32(float4 (&r)[8], const float* __restrict__ base, const Segs& sg, int rowlen,
                                         int rows, int K, int r0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    int srow, col;
    bool ok;
    if (!TR) {
      const int n = r0 + (v >> 3);
      col = k0 + 8 * (v & 7);
      ok = n < rows && col < K;
      srow = n;
    } else {
      const int k = k0 + (v >> 4);
      col = r0 + 8 * (v & 15);
      ok = k < K && col < rows;
      srow = k;
    }
    if (ok) {
      const float* p = base + seg_row(sg, srow, rowlen) + col;
      r[2 * i] = *reinterpret_cast<const float4*>(p);
      r[2 * i + 1] = *reinterpret_cast<const float4*>(p + 4);
    } else {
      r[2 * i] = make_float4(0.f, 0.f, 0.f, 0.f);
      r[2 * i + 1] = r[2 * i];
    }
  }
}

template <int TR>
__device__ __forceinline__ void store_f32(uint16_t* tile, const float4 (&r)[8], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    const int off = TR ? (v >> 4) * LDT + 8 * (v & 15) : (v >> 3) * LDK + 8 * (v & 7);
    const float4 a = r[2 * i], b = r[2 * i + 1];
    uint4 o;
    o.x = pk2(a.x, a.y); o.y = pk2(a.z, a.w); o.z = pk2(b.x, b.y); o.w = pk2(b.z, b.w);
    *reinterpret_cast<uint4*>(tile + off) = o;
  }
}

// DB = 1: double-buffered LDS (72 KiB, one barrier per K-step, 2 blocks/CU).
// DB = 0: single LDS buffer (36 KiB, two barriers per K-step) at 3 waves/SIMD → 3 blocks/CU; the
//         next tile still streams into registers under the current tile's MFMAs.
template <int A_TR, int B_TR, int B_F32, int EPI, int BSEG, int DB>
__global__ __launch_bounds__(NT, 3) void bgemm_kernel(const Args p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // DB: [A buf 0][A buf 1][B buf 0][B buf 1]      !DB: [A][B]
#define SA(b) (smem + (DB ? (b) : 0) * TILE_ELEMS)
#define SB(b) (smem + (DB ? (2 + (b)) : 1) * TILE_ELEMS)

  // XCD-aware order: the 8 XCDs take blocks round-robin, so give each XCD a contiguous range of
  // (client, m-tile, n-tile) tiles — the n-tiles of one row block then share A in that XCD's L2.
  const int total = p.tiles_m * p.tiles_n * p.nclients;
  int L = blockIdx.x;
  if ((total & 7) == 0) L = (L & 7) * (total >> 3) + (L >> 3);
  const int tn = L % p.tiles_n;
  const int tm = (L / p.tiles_n) % p.tiles_m;
  const int c = L / (p.tiles_n * p.tiles_m);
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;

  const uint16_t* A = p.A + (int64_t)c * p.a_bs;
  // a single-segment bf16 B is a plain matrix at offset off[0] (no per-vector segment search)
  const uint16_t* Bh = B_F32 ? nullptr : (const uint16_t*)p.B + (int64_t)c * p.b_bs + (BSEG ? 0 : p.bseg.off[0]);
  const float* Bf = B_F32 ? (const float*)p.B + (int64_t)c * p.b_bs : nullptr;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4];
  uint4 rbh[4];
  float4 rbf[8];
  const int nk = (p.K + BK - 1) / BK;
  // weight gradient with a fused bias gradient: the first column-block of every row-block sums its A (dy) tiles
  // — thread tid's 4 staging vectors all hold columns 8·(tid & 15) .. +7 of the A tile (TR layout)
  const bool bsum = EPI == EPI_ACC32 && A_TR == 1 && p.bg != nullptr && tn == 0;
  float bs8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs8[e] = 0.f;
  auto bias_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t w[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bs8[2 * e] += bf16_to_f32((uint16_t)(w[e] & 0xffff));
        bs8[2 * e + 1] += bf16_to_f32((uint16_t)(w[e] >> 16));
      }
    }
  };

  load_bf16<A_TR>(ra, A, p.lda, p.M, p.K, m0, 0, tid);
  if (bsum) bias_acc();
  if (B_F32) load_f32<B_TR>(rbf, Bf, p.bseg, p.ldb, p.N, p.K, n0, 0, tid);
  else if (BSEG) load_bf16_seg<B_TR>(rbh, Bh, p.bseg, p.ldb, p.N, p.K, n0, 0, tid);
      else load_bf16<B_TR>(rbh, Bh, p.ldb, p.N, p.K, n0, 0, tid);
  store_bf16<A_TR>(SA(0), ra, tid);
  if (B_F32) store_f32<B_TR>(SB(0), rbf, tid);
  else store_bf16<B_TR>(SB(0), rbh, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {   // next tile's global reads fly while this tile's MFMAs run
      load_bf16<A_TR>(ra, A, p.lda, p.M, p.K, m0, (kt + 1) * BK, tid);
      if (bsum) bias_acc();
      if (B_F32) load_f32<B_TR>(rbf, Bf, p.bseg, p.ldb, p.N, p.K, n0, (kt + 1) * BK, tid);
      else if (BSEG) load_bf16_seg<B_TR>(rbh, Bh, p.bseg, p.ldb, p.N, p.K, n0, (kt + 1) * BK, tid);
      else load_bf16<B_TR>(rbh, Bh, p.ldb, p.N, p.K, n0, (kt + 1) * BK, tid);
    }
    const uint16_t* ta = SA(cur);
    const uint16_t* tb = SB(cur);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = A_TR ? tr_frag(ta, kk * 32, wm + 16 * i, lane)
                     : row_frag(ta, wm + 16 * i + (lane & 15), kk * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = B_TR ? tr_frag(tb, kk * 32, wn + 16 * j, lane)
                      : row_frag(tb, wn + 16 * j + (lane & 15), kk * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (!DB && more) __syncthreads();   // every wave is done reading the single buffer
    if (more) {
      store_bf16<A_TR>(SA(cur ^ 1), ra, tid);
      if (B_F32) store_f32<B_TR>(SB(cur ^ 1), rbf, tid);
      else store_bf16<B_TR>(SB(cur ^ 1), rbh, tid);
    }
    __syncthreads();
  }

  if (EPI == EPI_ACC32 && A_TR == 1 && bsum) {
    // the 16 threads holding the same 8 columns (tid & 15) combine through LDS (free after the K loop)
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid * 8 + e] = bs8[e];
    __syncthreads();
    if (tid < 128) {   // column m0 + tid: group tid >> 3, element tid & 7
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) t += red[(r * 16 + (tid >> 3)) * 8 + (tid & 7)];
      const int m = m0 + tid;
      if (m < p.M) {
        float* bp = p.bg + (int64_t)c * p.bg_bs + seg_row(p.bgseg, m, 1);
        *bp = p.acc_store ? t : *bp + t;
      }
    }
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
      if (EPI == EPI_ACC32) {
        float* dst = (float*)p.Cp + (int64_t)c * p.c_bs + seg_row(p.cseg, m, p.ldc) + n;
        float4 o = make_float4(v[0], v[1], v[2], v[3]);
        if (!p.acc_store) {
          const float4 q = *reinterpret_cast<const float4*>(dst);
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        *reinterpret_cast<float4*>(dst) = o;
      } else {
        if (p.bias) {
          const float4 b = *reinterpret_cast<const float4*>(p.bias + (int64_t)c * p.bias_bs + seg_row(p.biasseg, n, 1));
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (p.R) {   // EPI_BF16: residual addend; EPI_DGELU: the pre-activation of the GELU
          const uint2 rr = *reinterpret_cast<const uint2*>(p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldc + n);
          const float r4[4] = {bf16_to_f32((uint16_t)(rr.x & 0xffff)), bf16_to_f32((uint16_t)(rr.x >> 16)),
                               bf16_to_f32((uint16_t)(rr.y & 0xffff)), bf16_to_f32((uint16_t)(rr.y >> 16))};
          if (EPI == EPI_DGELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu_grad(r4[e], v[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += r4[e];
          }
        }
        uint2 o;
        o.x = pk2(v[0], v[1]);
        o.y = pk2(v[2], v[3]);
        *reinterpret_cast<uint2*>((uint16_t*)p.Cp + (int64_t)c * p.c_bs + (int64_t)m * p.ldc + n) = o;
        if (EPI == EPI_GELU) {
          // GELU of the bf16-rounded pre-activation (what the backward recomputes from)
          float r[4];
          r[0] = bf16_to_f32((uint16_t)(o.x & 0xffff)); r[1] = bf16_to_f32((uint16_t)(o.x >> 16));
          r[2] = bf16_to_f32((uint16_t)(o.y & 0xffff)); r[3] = bf16_to_f32((uint16_t)(o.y >> 16));
          uint2 g;
          g.x = pk2(gelu_erf(r[0]), gelu_erf(r[1]));
          g.y = pk2(gelu_erf(r[2]), gelu_erf(r[3]));
          *reinterpret_cast<uint2*>(p.C2 + (int64_t)c * p.c2_bs + (int64_t)m * p.ldc + n) = g;
        }
      }
    }
  }
}

#undef SA
#undef SB

// db[c][n] += Σ_m g[c][m][n] for bf16 g [C][M][ldg]: each thread owns 2 adjacent columns of a
// 256-row chunk (4-byte coalesced loads), one fp32 atomic pair per thread into the (segmented)
// fp32 gradient arena — no fp32 copy of g and no separate accumulate kernel.
__global__ __launch_bounds__(256) void bias_grad_kernel(const uint16_t* __restrict__ g, int64_t g_bs, int ldg,
                                                        float* __restrict__ out, int64_t o_cs, Segs seg, int M, int N,
                                                        int rows_per_block) {
  const int c = blockIdx.z;
  const int n = 2 * (blockIdx.x * 256 + threadIdx.x);
  if (n >= N) return;
  const int m0 = blockIdx.y * rows_per_block;
  const int m1 = min(M, m0 + rows_per_block);
  const uint16_t* gp = g + (int64_t)c * g_bs + n;
  float a0 = 0.f, a1 = 0.f;
  for (int m = m0; m < m1; ++m) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(gp + (int64_t)m * ldg);
    a0 += bf16_to_f32((uint16_t)(v & 0xffff));
    a1 += bf16_to_f32((uint16_t)(v >> 16));
  }
  float* o = out + (int64_t)c * o_cs;
  fa_acc_add(o + seg_row(seg, n, 1), a0);
  fa_acc_add(o + seg_row(seg, n + 1, 1), a1);
}

// ---------------------------------------------------------------------------------------------------------------
// LDS-DMA variant for bf16 operands (activations, the arena's bf16 shadow): the same 128 × 128 × 64 block tile and
// wave layout, but the tiles travel global → LDS by `buffer_load_dwordx4 … lds` (no staging registers, no
// ds_write pass). The LDS image is lane-linear per wave instruction, so bank spreading is an XOR swizzle of the
// SOURCE address: K-major [128 rows][64 k] images put 16-B chunk q of row r at q ^ ((r >> 1) & 7) (ds_read_b128
// conflict-free), TR [64 k][128 cols] images put 32-B chunk h of row r at h ^ ((r & 3) | ((r >> 1) & 4))
// (ds_read_b64_tr_b16 conflict-free). Buffer descriptors bound each client's operand: reads past it return 0, which
// zero-fills the reduction tail of the weight gradient (T % 64) and every ragged row for free.
// DB = 1: two images per operand (64 KiB), next K-step's DMA in flight under this one's MFMAs;
// DB = 0: one image (32 KiB, more blocks per CU), load → wait → compute.
constexpr int GIMG = 128 * 64;   // elements of one operand image (16 KiB)
constexpr int kStgLd = 128 + 4;  // fp32 epilogue staging row pitch (16-B rows, 4-bank shift per row)

__device__ __forceinline__ int swz_nt(int r, int q) { return q ^ ((r >> 1) & 7); }
__device__ __forceinline__ int swz_tr(int r, int h) { return h ^ ((r & 3) | ((r >> 1) & 4)); }

__device__ __forceinline__ bf16x8 row_frag_s(const uint16_t* tile, int row, int q) {
  return *reinterpret_cast<const bf16x8*>(tile + row * 64 + 8 * swz_nt(row, q));
}

__device__ __forceinline__ bf16x8 tr_frag_s(const uint16_t* tile, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r = row0 + 8 * g + q, h = col0 >> 4;
  const uint16_t* a0 = tile + r * 128 + 16 * swz_tr(r, h) + 4 * p;
  const uint16_t* a1 = tile + (r + 4) * 128 + 16 * swz_tr(r + 4, h) + 4 * p;
  const v4i16 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  const v4i16 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a1));
  union {
    short s[8];
    bf16x8 b;
  } u;
  u.s[0] = r0[0]; u.s[1] = r0[1]; u.s[2] = r0[2]; u.s[3] = r0[3];
  u.s[4] = r1[0]; u.s[5] = r1[1]; u.s[6] = r1[2]; u.s[7] = r1[3];
  return u.b;
}

// per-lane byte offsets (relative to the K-step's first reduction row / column) of the 4 DMA instructions a wave
// issues for one operand image; instruction i of wave w fills LDS bytes [(4w + i)·1 KiB, +1 KiB)
template <int TR>
__device__ __forceinline__ void dma_offsets(uint32_t (&vo)[4], const Segs& sg, bool seg, int ld, int r0, int wid,
                                            int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int P = (wid * 4 + i) * 1024 + lane * 16;
    if (!TR) {   // image row r = logical row r0 + r (an output row / col), stored chunk → source chunk
      const int r = P >> 7;
      const int q = ((P >> 4) & 7) ^ ((r >> 1) & 7);
      const int64_t row = seg ? seg_row(sg, r0 + r, ld) : (int64_t)(r0 + r) * ld;
      vo[i] = (uint32_t)((row + 8 * q) * 2);
    } else {     // image row r = reduction row k0 + r, cols r0 .. r0 + 127
      const int r = P >> 8;
      const int h = ((P >> 5) & 7) ^ ((r & 3) | ((r >> 1) & 4));
      const int col = r0 + 16 * h + 8 * ((P >> 4) & 1);
      vo[i] = (uint32_t)(((int64_t)r * ld + col) * 2);
    }
  }
}

template <int A_TR, int B_TR, int EPI, int BSEG, int DB>
__global__ __launch_bounds__(NT, 2) void bgemm_dma_kernel(const Args p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // [A img 0][B img 0]([A img 1][B img 1])
  const int total = p.tiles_m * p.tiles_n * p.nclients;
  int L = blockIdx.x;
  {   // contiguous tile ranges per XCD (bijective for any total)
    const int q = total >> 3, r = total & 7, x = L & 7;
    L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
  }
  const int tn = L % p.tiles_n;
  const int tm = (L / p.tiles_n) % p.tiles_m;
  const int c = L / (p.tiles_n * p.tiles_m);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;

  // descriptors from PROVABLY wave-uniform inputs (readfirstlane), else hipcc wraps every buffer op in a waterfall
  // loop (cdna_hip_programming.md T20)
  auto rsrc = [](const void* base, int64_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t ra = rsrc(p.A + (int64_t)c * p.a_bs, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = rsrc((const uint16_t*)p.B + (int64_t)c * p.b_bs, p.b_bytes);
  uint32_t voa[4], vob[4];
  dma_offsets<A_TR>(voa, p.bseg, false, p.lda, m0, wid, lane);
  dma_offsets<B_TR>(vob, p.bseg, BSEG && !B_TR, p.ldb, n0, wid, lane);

  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BK;
    // uniform advance of the K-step: along the row (K-major) or down the rows (TR; a segmented TR operand's 64
    // reduction rows sit inside one segment — the host checks the boundaries)
    const uint32_t sa = __builtin_amdgcn_readfirstlane(A_TR ? (uint32_t)((int64_t)k0 * p.lda * 2) : (uint32_t)(k0 * 2));
    const uint32_t sb = __builtin_amdgcn_readfirstlane(
        B_TR ? (uint32_t)((BSEG ? seg_row(p.bseg, k0, p.ldb) : (int64_t)k0 * p.ldb) * 2) : (uint32_t)(k0 * 2));
    uint16_t* ia = smem + (DB ? buf : 0) * 2 * GIMG;
    uint16_t* ib = ia + GIMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(ia + (wid * 4 + i) * 512),
                                               16, voa[i], sa, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(ib + (wid * 4 + i) * 512),
                                               16, vob[i], sb, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (p.K + BK - 1) / BK;
  // weight gradient with a fused bias gradient: the first column-block of every row-block sums its A (dy) images
  const bool bsum = EPI == EPI_ACC32 && A_TR == 1 && p.bg != nullptr && tn == 0;
  float bs = 0.f;

  if (DB) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = DB ? (kt & 1) : 0;
    if (DB) {
      if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
    } else {
      issue(kt, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const uint16_t* ta = smem + cur * 2 * GIMG;
    const uint16_t* tb = ta + GIMG;
    if (bsum) {   // column tid & 127 of the dy image, rows 32·(tid >> 7) .. +31
      const int col = tid & 127;
#pragma unroll 8
      for (int r = 32 * (tid >> 7); r < 32 * (tid >> 7) + 32; ++r)
        bs += bf16_to_f32(ta[r * 128 + 16 * swz_tr(r, col >> 4) + (col & 15)]);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = A_TR ? tr_frag_s(ta, kk * 32, wm + 16 * i, lane)
                     : row_frag_s(ta, wm + 16 * i + (lane & 15), kk * 4 + (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = B_TR ? tr_frag_s(tb, kk * 32, wn + 16 * j, lane)
                      : row_frag_s(tb, wn + 16 * j + (lane & 15), kk * 4 + (lane >> 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (DB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next image has landed (this wave's part)
    __syncthreads();    // ... every wave's part; and nobody reads the image the next DMA overwrites
  }

  if (EPI == EPI_ACC32 && A_TR == 1 && bsum) {
    float* red = reinterpret_cast<float*>(smem);
    red[tid] = bs;
    __syncthreads();
    if (tid < 128) {
      const int m = m0 + tid;
      if (m < p.M) {
        float* bp = p.bg + (int64_t)c * p.bg_bs + seg_row(p.bgseg, m, 1);
        const float t = red[tid] + red[tid + 128];
        *bp = p.acc_store ? t : *bp + t;
      }
    }
    __syncthreads();   // the reduction scratch is the epilogue staging area
  }

  if (p.stage_epi) {
    // outputs through LDS: each 64-row half of the tile is staged in fp32 by the two waves that own it, then
    // written by all 256 threads as 16-B chunks of whole rows (the MFMA layout stores 32-B (bf16) / 64-B (fp32)
    // row pieces)
    float* stg = reinterpret_cast<float*>(smem);   // [64][kStgLd] fp32
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if ((wm >> 6) == h) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 v = acc[i][j];
            *reinterpret_cast<float4*>(stg + (16 * i + (lane & 15)) * kStgLd + wn + 16 * j + 4 * (lane >> 4)) =
                make_float4(v[0], v[1], v[2], v[3]);
          }
      }
      __syncthreads();
      if (EPI == EPI_ACC32) {   // fp32 weight gradient rows of the arena: += (or = for the first writer)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int q = tid + NT * t, row = q >> 5, col = 4 * (q & 31);
          const int m = m0 + 64 * h + row, n = n0 + col;
          if (m < p.M && n < p.N) {
            float4 o = *reinterpret_cast<const float4*>(stg + row * kStgLd + col);
            float* dst = (float*)p.Cp + (int64_t)c * p.c_bs + seg_row(p.cseg, m, p.ldc) + n;
            if (!p.acc_store) {
              const float4 q4 = *reinterpret_cast<const float4*>(dst);
              o.x += q4.x; o.y += q4.y; o.z += q4.z; o.w += q4.w;
            }
            *reinterpret_cast<float4*>(dst) = o;
          }
        }
        __syncthreads();
        continue;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = tid + NT * t, row = q >> 4, col = 8 * (q & 15);
        const int m = m0 + 64 * h + row, n = n0 + col;
        if (m < p.M && n < p.N) {
          const float4 a0 = *reinterpret_cast<const float4*>(stg + row * kStgLd + col);
          const float4 a1 = *reinterpret_cast<const float4*>(stg + row * kStgLd + col + 4);
          float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
          if (p.bias) {
            const float* bp = p.bias + (int64_t)c * p.bias_bs + seg_row(p.biasseg, n, 1);
            const float4 b0 = *reinterpret_cast<const float4*>(bp), b1 = *reinterpret_cast<const float4*>(bp + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
          }
          if (p.R) {
            const uint4 rr = *reinterpret_cast<const uint4*>(p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldc + n);
            const uint32_t w4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = bf16_to_f32((uint16_t)(w4[e] & 0xffff)), hi = bf16_to_f32((uint16_t)(w4[e] >> 16));
              if (EPI == EPI_DGELU) {
                v[2 * e] = gelu_grad(lo, v[2 * e]);
                v[2 * e + 1] = gelu_grad(hi, v[2 * e + 1]);
              } else {
                v[2 * e] += lo;
                v[2 * e + 1] += hi;
              }
            }
          }
          uint4 o;
          o.x = pk2(v[0], v[1]); o.y = pk2(v[2], v[3]); o.z = pk2(v[4], v[5]); o.w = pk2(v[6], v[7]);
          *reinterpret_cast<uint4*>((uint16_t*)p.Cp + (int64_t)c * p.c_bs + (int64_t)m * p.ldc + n) = o;
          if (EPI == EPI_GELU) {   // GELU of the bf16-rounded pre-activation (what the backward recomputes from)
            const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
            uint32_t g4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              g4[e] = pk2(gelu_erf(bf16_to_f32((uint16_t)(w4[e] & 0xffff))),
                          gelu_erf(bf16_to_f32((uint16_t)(w4[e] >> 16))));
            *reinterpret_cast<uint4*>(p.C2 + (int64_t)c * p.c2_bs + (int64_t)m * p.ldc + n) =
                make_uint4(g4[0], g4[1], g4[2], g4[3]);
          }
        }
      }
      __syncthreads();   // the staging rows are rewritten by the next half
    }
    return;
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm + 16 * i + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + 16 * j + 4 * (lane >> 4);
      if (n >= p.N) continue;
      f32x4 v = acc[i][j];
      if (EPI == EPI_ACC32) {
        float* dst = (float*)p.Cp + (int64_t)c * p.c_bs + seg_row(p.cseg, m, p.ldc) + n;
        float4 o = make_float4(v[0], v[1], v[2], v[3]);
        if (!p.acc_store) {
          const float4 q = *reinterpret_cast<const float4*>(dst);
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        *reinterpret_cast<float4*>(dst) = o;
      } else {
        if (p.bias) {
          const float4 b = *reinterpret_cast<const float4*>(p.bias + (int64_t)c * p.bias_bs + seg_row(p.biasseg, n, 1));
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (p.R) {
          const uint2 rr = *reinterpret_cast<const uint2*>(p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldc + n);
          const float r4[4] = {bf16_to_f32((uint16_t)(rr.x & 0xffff)), bf16_to_f32((uint16_t)(rr.x >> 16)),
                               bf16_to_f32((uint16_t)(rr.y & 0xffff)), bf16_to_f32((uint16_t)(rr.y >> 16))};
          if (EPI == EPI_DGELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu_grad(r4[e], v[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += r4[e];
          }
        }
        uint2 o;
        o.x = pk2(v[0], v[1]);
        o.y = pk2(v[2], v[3]);
        *reinterpret_cast<uint2*>((uint16_t*)p.Cp + (int64_t)c * p.c_bs + (int64_t)m * p.ldc + n) = o;
        if (EPI == EPI_GELU) {
          float r[4];
          r[0] = bf16_to_f32((uint16_t)(o.x & 0xffff)); r[1] = bf16_to_f32((uint16_t)(o.x >> 16));
          r[2] = bf16_to_f32((uint16_t)(o.y & 0xffff)); r[3] = bf16_to_f32((uint16_t)(o.y >> 16));
          uint2 g;
          g.x = pk2(gelu_erf(r[0]), gelu_erf(r[1]));
          g.y = pk2(gelu_erf(r[2]), gelu_erf(r[3]));
          *reinterpret_cast<uint2*>(p.C2 + (int64_t)c * p.c2_bs + (int64_t)m * p.ldc + n) = g;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// 256 × 256 × 64 block tile on the same LDS-DMA images: 8 waves (2 along M × 4 along N, 128 × 64 outputs and 128
// accumulator registers each — two waves per SIMD), the block's A and B tiles as two 128-wide half images each
// (the 128 × 128 kernel's swizzled layouts), two buffers (128 KiB). The next K-step's four half images are DMA'd
// at the start of this K-step, under its four quadrant phases of MFMAs; one wait + raw barrier per K-step. Half the L2 bytes
// per MFMA of the 128 × 128 tile. (cdna_hip_programming.md §5: 256² tiles with the prefetch in flight across the
// barrier.)
template <int A_TR, int B_TR, int EPI, int BSEG>
__global__ __launch_bounds__(512, 1) void bgemm_dma256_kernel(const Args p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // buffer b: [A0][A1][B0][B1] images at smem + b·4·GIMG
  const int total = p.tiles_m * p.tiles_n * p.nclients;
  int L = blockIdx.x;
  {
    const int q = total >> 3, r = total & 7, x = L & 7;
    L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
  }
  const int tn = L % p.tiles_n;
  const int tm = (L / p.tiles_n) % p.tiles_m;
  const int c = L / (p.tiles_n * p.tiles_m);
  const int m0 = tm * 256, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;   // rows wr·128 (A half wr), cols wc·64 (B half wc >> 1)

  auto rsrc = [](const void* base, int64_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t ra = rsrc(p.A + (int64_t)c * p.a_bs, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = rsrc((const uint16_t*)p.B + (int64_t)c * p.b_bs, p.b_bytes);
  // per-lane offsets: half image h (0, 1: A halves; 2, 3: B halves), instruction i of this wave (2 per wave)
  uint32_t vo[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int P = (wid * 2 + i) * 1024 + lane * 16;
      const bool isA = h < 2;
      const int TR = isA ? A_TR : B_TR;
      const int ld = isA ? p.lda : p.ldb;
      const int r0 = (isA ? m0 : n0) + (h & 1) * 128;
      if (!TR) {
        const int r = P >> 7;
        const int q = ((P >> 4) & 7) ^ ((r >> 1) & 7);
        const int64_t row = (!isA && BSEG) ? seg_row(p.bseg, r0 + r, ld) : (int64_t)(r0 + r) * ld;
        vo[h][i] = (uint32_t)((row + 8 * q) * 2);
      } else {
        const int r = P >> 8;
        const int hh = ((P >> 5) & 7) ^ ((r & 3) | ((r >> 1) & 4));
        const int col = r0 + 16 * hh + 8 * ((P >> 4) & 1);
        vo[h][i] = (uint32_t)(((int64_t)r * ld + col) * 2);
      }
    }
  auto issue_half = [&](int kt, int buf, int h) {
    const int k0 = kt * BK;
    uint32_t so;
    if (h < 2) so = A_TR ? (uint32_t)((int64_t)k0 * p.lda * 2) : (uint32_t)(k0 * 2);
    else so = B_TR ? (uint32_t)((BSEG ? seg_row(p.bseg, k0, p.ldb) : (int64_t)k0 * p.ldb) * 2) : (uint32_t)(k0 * 2);
    so = __builtin_amdgcn_readfirstlane(so);
    uint16_t* img = smem + (buf * 4 + h) * GIMG;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? ra : rb,
                                               (__attribute__((address_space(3))) void*)(img + (wid * 2 + i) * 512),
                                               16, vo[h][i], so, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (p.K + BK - 1) / BK;
  const bool bsum = EPI == EPI_ACC32 && A_TR == 1 && p.bg != nullptr && tn == 0;
  float bs = 0.f;

#pragma unroll
  for (int h = 0; h < 4; ++h) issue_half(0, 0, h);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    const uint16_t* ta = smem + (cur * 4 + wr) * GIMG;
    const uint16_t* tb = smem + (cur * 4 + 2 + (wc >> 1)) * GIMG;
    const int cb = (wc & 1) * 64;     // this wave's columns inside its B half image
    if (bsum) {   // column tid & 255 of the block's dy (A half (tid & 255) >> 7), rows 32·(tid >> 8) .. +31
      const int col = tid & 127;
      const uint16_t* th = smem + (cur * 4 + ((tid >> 7) & 1)) * GIMG;
#pragma unroll 8
      for (int r = 32 * (tid >> 8); r < 32 * (tid >> 8) + 32; ++r)
        bs += bf16_to_f32(th[r * 128 + 16 * swz_tr(r, col >> 4) + (col & 15)]);
    }
    bf16x8 af[4][2];
    if (more) {   // the whole next K-step in flight from the start of this one (the most lead time 2 buffers give)
#pragma unroll
      for (int h = 0; h < 4; ++h) issue_half(kt + 1, cur ^ 1, h);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {     // quadrant (qm, qn): rows qm·64, cols qn·32 of the wave's 128 × 64 tile
      const int qm = q >> 1, qn = (q == 1 || q == 2) ? 1 : 0;
      if (q == 0 || q == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            af[i][kk] = A_TR ? tr_frag_s(ta, kk * 32, qm * 64 + 16 * i, lane)
                             : row_frag_s(ta, qm * 64 + 16 * i + (lane & 15), kk * 4 + (lane >> 4));
      }
      bf16x8 bfr[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          bfr[j][kk] = B_TR ? tr_frag_s(tb, kk * 32, cb + qn * 32 + 16 * j, lane)
                            : row_frag_s(tb, cb + qn * 32 + 16 * j + (lane & 15), kk * 4 + (lane >> 4));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qm * 4 + i][qn * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // this wave's DMA of the next K-step landed
    __builtin_amdgcn_s_barrier();                                  // ... every wave's; nobody reads buf cur again
  }

  if (EPI == EPI_ACC32 && A_TR == 1 && bsum) {
    float* red = reinterpret_cast<float*>(smem);
    red[tid] = bs;
    __syncthreads();
    if (tid < 256) {
      const int m = m0 + tid;
      if (m < p.M) {
        float* bp = p.bg + (int64_t)c * p.bg_bs + seg_row(p.bgseg, m, 1);
        const float t = red[tid] + red[tid + 256];
        *bp = p.acc_store ? t : *bp + t;
      }
    }
  }

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + 16 * i + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + 16 * j + 4 * (lane >> 4);
      if (n >= p.N) continue;
      f32x4 v = acc[i][j];
      if (EPI == EPI_ACC32) {
        float* dst = (float*)p.Cp + (int64_t)c * p.c_bs + seg_row(p.cseg, m, p.ldc) + n;
        float4 o = make_float4(v[0], v[1], v[2], v[3]);
        if (!p.acc_store) {
          const float4 q = *reinterpret_cast<const float4*>(dst);
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        *reinterpret_cast<float4*>(dst) = o;
      } else {
        if (p.bias) {
          const float4 b = *reinterpret_cast<const float4*>(p.bias + (int64_t)c * p.bias_bs + seg_row(p.biasseg, n, 1));
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (p.R) {
          const uint2 rr = *reinterpret_cast<const uint2*>(p.R + (int64_t)c * p.r_bs + (int64_t)m * p.ldc + n);
          const float r4[4] = {bf16_to_f32((uint16_t)(rr.x & 0xffff)), bf16_to_f32((uint16_t)(rr.x >> 16)),
                               bf16_to_f32((uint16_t)(rr.y & 0xffff)), bf16_to_f32((uint16_t)(rr.y >> 16))};
          if (EPI == EPI_DGELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu_grad(r4[e], v[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += r4[e];
          }
        }
        uint2 o;
        o.x = pk2(v[0], v[1]);
        o.y = pk2(v[2], v[3]);
        *reinterpret_cast<uint2*>((uint16_t*)p.Cp + (int64_t)c * p.c_bs + (int64_t)m * p.ldc + n) = o;
        if (EPI == EPI_GELU) {
          float r[4];
          r[0] = bf16_to_f32((uint16_t)(o.x & 0xffff)); r[1] = bf16_to_f32((uint16_t)(o.x >> 16));
          r[2] = bf16_to_f32((uint16_t)(o.y & 0xffff)); r[3] = bf16_to_f32((uint16_t)(o.y >> 16));
          uint2 g;
          g.x = pk2(gelu_erf(r[0]), gelu_erf(r[1]));
          g.y = pk2(gelu_erf(r[2]), gelu_erf(r[3]));
          *reinterpret_cast<uint2*>(p.C2 + (int64_t)c * p.c2_bs + (int64_t)m * p.ldc + n) = g;
        }
      }
    }
  }
}

// operand extent (bytes from the client's base) the DMA descriptors bound: rows × ld of a plain matrix, or the end
// of the last segment row
inline int64_t seg_extent(const Segs& s, int rows, int ld) {
  int64_t e = 0;
  for (int i = 0; i < s.n; ++i) {
    const int lo = s.lo[i], hi = (i + 1 < s.n) ? s.lo[i + 1] : rows;
    e = std::max<int64_t>(e, s.off[i] + (int64_t)(hi - lo) * ld);
  }
  return e * 2;
}

template <int A_TR, int B_TR, int B_F32, int EPI>
int launch(const Args& a, hipStream_t st) {
  const int64_t blocks = (int64_t)a.tiles_m * a.tiles_n * a.nclients;
  if (blocks <= 0 || blocks > 0x7fffffff) return (int)hipErrorInvalidValue;
  static const int db = [] {
    const char* e = getenv("FEDML_AMD_BGEMM_DB");
    return e ? atoi(e) : 0;
  }();
  const bool seg = !B_F32 && a.bseg.n > 1;
  // bf16 operands: the LDS-DMA kernel (FEDML_AMD_BGEMM_DMA=0: never; 1: double-buffered; 2: single image, default)
  // (single image measured faster: ViT-B/16 bf16 3.84 vs 3.50 rounds/s double-buffered, 3.71 register-staged;
  // profiles/r5_bgemm_dma_micro.txt)
  const char* dma_env = getenv("FEDML_AMD_BGEMM_DMA");
  const int dma = dma_env ? atoi(dma_env) : 2;
  if (!B_F32 && dma) {
    Args b = a;
    // A: [M][lda] (K-major) or [K][lda] (TR); B: [N][ldb] / segments (K-major) or [K][ldb] / segments (TR)
    b.a_bytes = (int64_t)(A_TR ? a.K : a.M) * a.lda * 2;
    const int brows = B_TR ? a.K : a.N;
    b.b_bytes = seg_extent(a.bseg, brows, a.ldb);
    bool ok = b.a_bytes < (1ll << 31) && b.b_bytes < (1ll << 31);
    // a K-major operand's reduction runs along its rows: a K tail would read the next row, not zeros
    if ((!A_TR || !B_TR) && a.K % BK != 0) ok = false;
    if (B_TR && seg)   // a K-step's 64 reduction rows must not straddle a segment boundary
      for (int i = 1; i < a.bseg.n; ++i) ok = ok && (a.bseg.lo[i] % BK == 0);
    // FEDML_AMD_BGEMM_256=1: the 256 × 256 tile when it still gives ≥ 256 blocks (one per CU)
    const char* e256 = getenv("FEDML_AMD_BGEMM_256");
    const int t256 = e256 ? atoi(e256) : 0;
    if (ok && t256) {
      Args b2 = b;
      b2.tiles_m = (a.M + 255) / 256;
      b2.tiles_n = (a.N + 255) / 256;
      const int64_t nb = (int64_t)b2.tiles_m * b2.tiles_n * b2.nclients;
      // 1: K-major operands only (a transposing ds_read_b64_tr_b16 after an in-flight LDS-DMA gets a conservative
      // vmcnt(0) from hipcc, which serialises the phase pipeline); 2: every layout, any grid (tests)
      const bool ok2 = t256 == 2 || (nb >= 256 && !A_TR && !B_TR);
      if (ok2) {
        auto kern = seg ? bgemm_dma256_kernel<A_TR, B_TR, EPI, 1> : bgemm_dma256_kernel<A_TR, B_TR, EPI, 0>;
        const size_t smem3 = 8 * GIMG * sizeof(uint16_t);   // 128 KiB
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem3);
        hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(512), smem3, st, b2);
        return (int)hipGetLastError();
      }
    }
    {   // staged epilogue: 16-B chunks need 8-element aligned rows / client strides / output columns
      const char* se = getenv("FEDML_AMD_BGEMM_STAGE_EPI");
      const bool want = se ? atoi(se) != 0 : true;
      b.stage_epi = want && (EPI == EPI_ACC32
                                 ? (a.ldc % 4 == 0 && a.c_bs % 4 == 0 && a.N % 4 == 0)
                                 : (a.ldc % 8 == 0 && a.c_bs % 8 == 0 && a.N % 8 == 0 && (!a.R || a.r_bs % 8 == 0) &&
                                    (!a.C2 || a.c2_bs % 8 == 0)));
    }
    if (ok) {
      auto pick = [&](auto k1, auto k0) { return dma == 2 ? k0 : k1; };
      auto kern = seg ? pick(bgemm_dma_kernel<A_TR, B_TR, EPI, 1, 1>, bgemm_dma_kernel<A_TR, B_TR, EPI, 1, 0>)
                      : pick(bgemm_dma_kernel<A_TR, B_TR, EPI, 0, 1>, bgemm_dma_kernel<A_TR, B_TR, EPI, 0, 0>);
      const size_t smem2 = std::max<size_t>((dma == 2 ? 2 : 4) * GIMG * sizeof(uint16_t),
                                            b.stage_epi ? 64 * kStgLd * sizeof(float) : 0);
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem2);
      hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NT), smem2, st, b);
      return (int)hipGetLastError();
    }
  }
  const size_t smem = (db ? 4 : 2) * TILE_ELEMS * sizeof(uint16_t);   // 72 KiB (2 blocks/CU) | 36 KiB (3)
  auto kern = db ? (seg ? bgemm_kernel<A_TR, B_TR, B_F32, EPI, 1, 1> : bgemm_kernel<A_TR, B_TR, B_F32, EPI, 0, 1>)
                 : (seg ? bgemm_kernel<A_TR, B_TR, B_F32, EPI, 1, 0> : bgemm_kernel<A_TR, B_TR, B_F32, EPI, 0, 0>);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NT), smem, st, a);
  return (int)hipGetLastError();
}

inline void fill_segs(Segs& s, const int64_t* off, const int* lo, int n) {
  s.n = n < 1 ? 1 : n;
  for (int i = 0; i < 4; ++i) s.off[i] = (off && i < n) ? off[i] : 0;
  for (int i = 0; i < 5; ++i) s.lo[i] = (lo && i <= n) ? lo[i] : 0;
}

}  // namespace bg

// Host-side contract (checked by the Python wrapper before launch): K % 8 == 0; TR operands'
// contiguous (column) extent % 8 == 0; N % 4 == 0; ldc % 4 == 0; segment boundaries % 8 == 0;
// every pointer 16-byte aligned. nseg ≤ 4.
//
// y[c] = x[c] · W[c]ᵀ + b[c]   (W: fp32 arena segments, or — w_bf16 — the same segments of the arena's
// bf16 shadow; b: fp32 arena segments; y bf16; gelu → y2 = gelu(y))
FA_EXPORT int fa_bgemm_fwd_res(const void* x, int64_t x_bs, int ldx, const void* w_base, int w_bf16, int64_t w_cs,
                               const int64_t* w_off, const float* b_base, int64_t b_cs, const int64_t* b_off,
                               const int* seg_lo, int nseg, void* y, int64_t y_bs, int ldy, void* y2, const void* res,
                               int C, int M, int N, int K, hipStream_t stream);
FA_EXPORT int fa_bgemm_fwd(const void* x, int64_t x_bs, int ldx, const void* w_base, int w_bf16, int64_t w_cs,
                           const int64_t* w_off, const float* b_base, int64_t b_cs, const int64_t* b_off,
                           const int* seg_lo, int nseg, void* y, int64_t y_bs, int ldy, void* y2, int C, int M, int N,
                           int K, hipStream_t stream) {
  return fa_bgemm_fwd_res(x, x_bs, ldx, w_base, w_bf16, w_cs, w_off, b_base, b_cs, b_off, seg_lo, nseg, y, y_bs, ldy,
                          y2, nullptr, C, M, N, K, stream);
}
// res (no GELU): y = x·Wᵀ + b + res, res bf16 with y's layout (a pre-LN block's residual stream in the epilogue)
FA_EXPORT int fa_bgemm_fwd_res(const void* x, int64_t x_bs, int ldx, const void* w_base, int w_bf16, int64_t w_cs,
                               const int64_t* w_off, const float* b_base, int64_t b_cs, const int64_t* b_off,
                               const int* seg_lo, int nseg, void* y, int64_t y_bs, int ldy, void* y2, const void* res,
                               int C, int M, int N, int K, hipStream_t stream) {
  using namespace bg;
  if (nseg < 1 || nseg > 4 || (res && y2)) return (int)hipErrorInvalidValue;
  Args a{};
  a.R = (const uint16_t*)res; a.r_bs = y_bs;
  a.A = (const uint16_t*)x; a.a_bs = x_bs; a.lda = ldx;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = y; a.c_bs = y_bs; a.ldc = ldy;
  a.bias = b_base; a.bias_bs = b_cs;
  fill_segs(a.biasseg, b_off, seg_lo, nseg);
  a.C2 = (uint16_t*)y2; a.c2_bs = y_bs;
  a.M = M; a.N = N; a.K = K;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (N + BN - 1) / BN; a.nclients = C;
  if (w_bf16) return y2 ? launch<0, 0, 0, EPI_GELU>(a, stream) : launch<0, 0, 0, EPI_BF16>(a, stream);
  return y2 ? launch<0, 0, 1, EPI_GELU>(a, stream) : launch<0, 0, 1, EPI_BF16>(a, stream);
}

// dx[c] = dy[c] · W[c]      dy [M][N] bf16, W [N][K] fp32 arena segments (rows n), dx [M][K] bf16
FA_EXPORT int fa_bgemm_dgrad_dgelu(const void* dy, int64_t dy_bs, int lddy, const void* w_base, int w_bf16,
                                   int64_t w_cs, const int64_t* w_off, const int* seg_lo, int nseg, void* dx,
                                   int64_t dx_bs, int lddx, const void* pre, int C, int M, int N, int K,
                                   hipStream_t stream);
FA_EXPORT int fa_bgemm_dgrad(const void* dy, int64_t dy_bs, int lddy, const void* w_base, int w_bf16, int64_t w_cs,
                             const int64_t* w_off, const int* seg_lo, int nseg, void* dx, int64_t dx_bs, int lddx, int C,
                             int M, int N, int K, hipStream_t stream) {
  return fa_bgemm_dgrad_dgelu(dy, dy_bs, lddy, w_base, w_bf16, w_cs, w_off, seg_lo, nseg, dx, dx_bs, lddx, nullptr, C, M,
                              N, K, stream);
}
// dx = dy · W + add   (add bf16 with dx's layout; may alias dx — each element is read, then written, by one lane):
// the residual-stream gradient of x's other consumer folded into this dgrad's epilogue
FA_EXPORT int fa_bgemm_dgrad_add(const void* dy, int64_t dy_bs, int lddy, const void* w_base, int w_bf16,
                                 int64_t w_cs, const int64_t* w_off, const int* seg_lo, int nseg, void* dx,
                                 int64_t dx_bs, int lddx, const void* add, int C, int M, int N, int K,
                                 hipStream_t stream) {
  using namespace bg;
  if (nseg < 1 || nseg > 4 || !add) return (int)hipErrorInvalidValue;
  Args a{};
  a.R = (const uint16_t*)add; a.r_bs = dx_bs;
  a.A = (const uint16_t*)dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = dx; a.c_bs = dx_bs; a.ldc = lddx;
  a.M = M; a.N = K; a.K = N;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  return w_bf16 ? launch<0, 1, 0, EPI_BF16>(a, stream) : launch<0, 1, 1, EPI_BF16>(a, stream);
}
// pre != null: dx = (dy · W) ⊙ gelu'(pre) — pre [C][M][lddx] bf16, the GELU input that produced this linear's x
FA_EXPORT int fa_bgemm_dgrad_dgelu(const void* dy, int64_t dy_bs, int lddy, const void* w_base, int w_bf16,
                                   int64_t w_cs, const int64_t* w_off, const int* seg_lo, int nseg, void* dx,
                                   int64_t dx_bs, int lddx, const void* pre, int C, int M, int N, int K,
                                   hipStream_t stream) {
  using namespace bg;
  if (nseg < 1 || nseg > 4) return (int)hipErrorInvalidValue;
  Args a{};
  a.R = (const uint16_t*)pre; a.r_bs = dx_bs;
  // GEMM: D[m][k] = Σ_n dy(m, n) · W(n, k): reduction = n (storage rows of W → TR)
  a.A = (const uint16_t*)dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = w_base; a.b_bs = w_cs; a.ldb = K;
  fill_segs(a.bseg, w_off, seg_lo, nseg);
  a.Cp = dx; a.c_bs = dx_bs; a.ldc = lddx;
  a.M = M; a.N = K; a.K = N;
  a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  if (pre) return w_bf16 ? launch<0, 1, 0, EPI_DGELU>(a, stream) : launch<0, 1, 1, EPI_DGELU>(a, stream);
  return w_bf16 ? launch<0, 1, 0, EPI_BF16>(a, stream) : launch<0, 1, 1, EPI_BF16>(a, stream);
}

FA_EXPORT int fa_bgemm_wgrad_bias(const void* dy, int64_t dy_bs, int lddy, const void* x, int64_t x_bs, int ldx,
                                  float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo, int nseg,
                                  float* b_base, int64_t b_cs, const int64_t* b_off, int C, int T, int N, int K,
                                  int store, hipStream_t stream);
// dW[c] += dy[c]ᵀ · x[c]    dy [T][N], x [T][K] bf16; dW [N][K] fp32 gradient-arena segments (rows n)
FA_EXPORT int fa_bgemm_wgrad(const void* dy, int64_t dy_bs, int lddy, const void* x, int64_t x_bs, int ldx,
                             float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo, int nseg, int C,
                             int T, int N, int K, hipStream_t stream) {
  return fa_bgemm_wgrad_bias(dy, dy_bs, lddy, x, x_bs, ldx, g_base, g_cs, g_off, seg_lo, nseg, nullptr, 0, nullptr, C, T,
                             N, K, 0, stream);
}
// b_base != null: also db[c] (+)= Σ_t dy[c][t][:] (bias segments share seg_lo) from the GEMM's own dy tiles;
// store = 1: = instead of += for dW and db (the rows' first writer)
FA_EXPORT int fa_bgemm_wgrad_bias(const void* dy, int64_t dy_bs, int lddy, const void* x, int64_t x_bs, int ldx,
                                  float* g_base, int64_t g_cs, const int64_t* g_off, const int* seg_lo, int nseg,
                                  float* b_base, int64_t b_cs, const int64_t* b_off, int C, int T, int N, int K,
                                  int store, hipStream_t stream) {
  using namespace bg;
  if (nseg < 1 || nseg > 4) return (int)hipErrorInvalidValue;
  Args a{};
  a.bg = b_base; a.bg_bs = b_cs;
  if (b_base) fill_segs(a.bgseg, b_off, seg_lo, nseg);
  a.acc_store = store;
  // GEMM: D[n][k] = Σ_t dy(t, n) · x(t, k): both operands have storage rows along t (TR)
  a.A = (const uint16_t*)dy; a.a_bs = dy_bs; a.lda = lddy;
  a.B = x; a.b_bs = x_bs; a.ldb = ldx;
  fill_segs(a.bseg, nullptr, nullptr, 1);   // plain [T][K] storage: one segment at offset 0
  a.Cp = g_base; a.c_bs = g_cs; a.ldc = K;
  fill_segs(a.cseg, g_off, seg_lo, nseg);
  a.M = N; a.N = K; a.K = T;
  a.tiles_m = (N + BM - 1) / BM; a.tiles_n = (K + BN - 1) / BN; a.nclients = C;
  return launch<1, 1, 0, EPI_ACC32>(a, stream);
}

// db[c] += Σ_m dy[c][m][:]   dy bf16 [C][M][N] (N even, segment boundaries even); db: fp32 arena segments
FA_EXPORT int fa_bias_grad(const void* dy, int64_t dy_bs, int lddy, float* o_base, int64_t o_cs, const int64_t* o_off,
                           const int* seg_lo, int nseg, int C, int M, int N, hipStream_t stream) {
  using namespace bg;
  if (nseg < 1 || nseg > 4 || (N & 1) || C <= 0 || M <= 0 || C > 65535) return (int)hipErrorInvalidValue;
  Segs sg;
  fill_segs(sg, o_off, seg_lo, nseg);
  const int rpb = 128;
  dim3 grid((unsigned)((N / 2 + 255) / 256), (unsigned)((M + rpb - 1) / rpb), (unsigned)C);
  hipLaunchKernelGGL(bias_grad_kernel, grid, dim3(256), 0, stream, (const uint16_t*)dy, dy_bs, lddy, o_base, o_cs, sg,
                     M, N, rpb);
  return (int)hipGetLastError();
}
