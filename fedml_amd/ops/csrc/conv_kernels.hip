// Client-batched convolution kernels for the virtual-client engine (gfx950, wave64, bf16 MFMA).
//
// Layouts (per virtual client c, all clients of a GPU in one launch, grid.y = client):
//   activations  X [C][N][H][W][Ch]   bf16, NHWC inside a client
//   packed fwd W  Wf[C][Cout][ldk]    bf16, k = (kh*KW + kw)*Cin + ci, zero padded to Kp
//   packed bwd W  Wb[C][Cin][ldk2]    bf16, k = (kh*KW + kw)*Cout + co (taps NOT flipped: the data
//                                            kernel maps each tap to the dy pixel it came from)
//   BN / scale vectors [C][Ch] fp32; BN statistics [C][Ch][NS] fp32 (atomics)
//
// Every conv is an implicit GEMM per client: M = N·Ho·Wo pixels, N = Cout, K = KH·KW·Cin.
// ResNet-56 channels are 16–256, so these GEMMs are skinny and HBM-bound; the kernels are
// built to move each activation byte once:
//   * forward : A operand = relu(x·s + t) of the PREVIOUS conv's raw output (its BatchNorm
//               folded into this conv's operand load), epilogue writes the raw output once
//               and accumulates this layer's BN statistics (Σy, Σy²) per (client, channel).
//   * bwd-data: A operand = dy = α·g + β·y + γ (the BN backward of the following BN folded
//               into the load), epilogue applies the previous ReLU mask and accumulates the
//               previous BN's backward statistics (Σg, Σg·x), writing g once.
//   * bwd-weight: dW = Σ_pixels dyᵀ ⊗ act(x), pixel-chunk per workgroup, fp32 atomics
//               straight into the client-stacked gradient arena (OIHW positions, stride ldw).
// MFMA: v_mfma_f32_16x16x32_bf16. Lane l holds A[row l&15][k 8(l>>4)..+7], B[k 8(l>>4)..+7][col l&15];
// D: col = l&15, row = 4(l>>4) + i.
#include "lds_swz.h"
#include "prec.h"
#include "detacc.h"
#include "bnlazy.h"
#include <algorithm>
#include <type_traits>

FA_DET_EXPORT(conv)

using prec::BF16;
using prec::F32;
using prec::F32X3;

// PRO_BOUT (conv_gemm_kernel, 1×1 / stride 1 forward only): the previous block's output is formed in the operand
//   load, a = relu(y·s + t + r) with r = src2 (identity shortcut) | src2·rs + rt (downsample BN) — the same
//   operation order as block_out_kernel — and written once to `pro_out` by the blockIdx.z == 0 workgroups: the
//   block output pass of that block (read y and r, write out, then this conv reads out again) disappears.
enum { PRO_NONE = 0, PRO_BNRELU = 1, PRO_BOUT = 2 };
// EPI_BOUT (conv_gemm_kernel only): the bottleneck block output straight from the last conv's accumulators,
//   out = relu((acc − K)·e_s + e_t + r),  r = e_add (identity shortcut) | e_add·e_rs + e_rt (downsample BN)
// — the conv's output y itself is never stored (its BN statistics come from a stats-only EPI_FWD pass)
enum { EPI_FWD = 0, EPI_STORE = 1, EPI_MASK = 2, EPI_BLOCK = 3, EPI_BOUT = 4 };

// =====================================================================================
// Weight packing: fp32 OIHW (client-stacked arena, stride ldw) → bf16 | fp32 GEMM layouts.
// One launch packs every conv layer of the model (segment table), both directions.
// =====================================================================================
struct PackSeg {
  int64_t src_off;   // offset of the OIHW weight inside one client's arena row
  int64_t dst_f;     // offset of this layer's Wf block (elements, per client stride = dst_ld)
  int64_t dst_b;     // offset of this layer's Wb block
  int cout, cin, kh, kw, ldk, ldk2;
  int cin_src;       // channels of the stored weight (cin may be padded up to a multiple of 8)
};

template <class P>
__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ arena, int64_t ldw,
                                                           const PackSeg* __restrict__ segs, int nseg,
                                                           typename P::T* __restrict__ dst, int64_t dst_ld) {
  using T = typename P::T;
  const int c = blockIdx.y;
  const PackSeg s = segs[blockIdx.z];
  const float* w = arena + (int64_t)c * ldw + s.src_off;
  T* df = dst + (int64_t)c * dst_ld + s.dst_f;
  T* db = dst + (int64_t)c * dst_ld + s.dst_b;
  const int taps = s.kh * s.kw;
  const int nf = s.cout * s.ldk;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += gridDim.x * blockDim.x) {
    const int co = i / s.ldk, k = i % s.ldk;
    float v = 0.f;
    if (k < taps * s.cin) {
      const int tap = k / s.cin, ci = k % s.cin;
      if (ci < s.cin_src) v = w[((int64_t)co * s.cin_src + ci) * taps + tap];
    }
    df[i] = P::from_f(v);
  }
  if (s.dst_b >= 0) {
    const int nb = s.cin * s.ldk2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) {
      const int ci = i / s.ldk2, k = i % s.ldk2;
      float v = 0.f;
      if (k < taps * s.cout) {
        const int tap = k / s.cout, co = k % s.cout;
        if (ci < s.cin_src) v = w[((int64_t)co * s.cin_src + ci) * taps + tap];
      }
      db[i] = P::from_f(v);
    }
  }
}

// Tiled packing: one workgroup moves a 32 (co) × 32 (ci) × taps block through LDS — coalesced
// reads of the OIHW rows, coalesced writes of both GEMM layouts (k = tap·cin + ci rows of Wf, and
// the co-contiguous rows of Wb, a transpose). The element-wise kernel above reads OIHW with a stride
// of `taps` floats and issues one integer division chain per element (ResNet-18: 1.45 ms per step).
constexpr int PK_T = 32;
constexpr int PK_MAXTAPS = 9;

// grid.x enumerates the (segment, tile) pairs of all layers back to back (no idle workgroups: one
// launch per model, the ResNet-18 table has 21 segments from 1 to 256 tiles)
template <class P>
__global__ __launch_bounds__(256) void pack_weights_tiled_kernel(const float* __restrict__ arena, int64_t ldw,
                                                                 const PackSeg* __restrict__ segs, int nseg,
                                                                 typename P::T* __restrict__ dst, int64_t dst_ld) {
  using T = typename P::T;
  __shared__ float tile[PK_T][PK_T * PK_MAXTAPS + 1];
  const int c = blockIdx.y;
  int si = 0, t0 = 0;
  for (;;) {   // segment of this tile (uniform per workgroup)
    const int nt = ((segs[si].cout + PK_T - 1) / PK_T) * ((segs[si].cin + PK_T - 1) / PK_T);
    if ((int)blockIdx.x < t0 + nt || si == nseg - 1) break;
    t0 += nt;
    ++si;
  }
  const PackSeg s = segs[si];
  const int taps = s.kh * s.kw;
  const int nco = (s.cout + PK_T - 1) / PK_T, nci = (s.cin + PK_T - 1) / PK_T;
  const int tix = blockIdx.x - t0;
  if (tix >= nco * nci) return;
  const int co0 = (tix / nci) * PK_T, ci0 = (tix % nci) * PK_T;
  const int tco = min(PK_T, s.cout - co0), tci = min(PK_T, s.cin - ci0);
  const float* w = arena + (int64_t)c * ldw + s.src_off;
  // load: row co holds (ci, tap) pairs ci0.. contiguous in the source (ci < cin_src; padding → 0).
  // PK_U independent loads per thread are in flight before the first LDS write: one load → wait → write per
  // iteration left the kernel HBM-latency bound (36 round trips per thread for a full 3×3 tile; ResNet-18
  // bf16 0.47 ms per step at 1.4 TB/s)
  constexpr int PK_U = 36;
  const int rowlen = tci * taps, n = tco * rowlen;
  for (int base = 0; base < n; base += 256 * PK_U) {
    float v[PK_U];
#pragma unroll
    for (int u = 0; u < PK_U; ++u) {
      const int i = base + u * 256 + (int)threadIdx.x;
      v[u] = 0.f;
      if (i < n) {
        const int r = i / rowlen, q = i - r * rowlen;
        if (ci0 + q / taps < s.cin_src) v[u] = w[((int64_t)(co0 + r) * s.cin_src + ci0) * taps + q];
      }
    }
#pragma unroll
    for (int u = 0; u < PK_U; ++u) {
      const int i = base + u * 256 + (int)threadIdx.x;
      if (i < n) {
        const int r = i / rowlen;
        tile[r][i - r * rowlen] = v[u];
      }
    }
  }
  __syncthreads();
  T* df = dst + (int64_t)c * dst_ld + s.dst_f;
  // Wf[co][tap·cin + ci]: ci fastest, 4 consecutive elements per store (8 B bf16 / 16 B fp32 — single
  // 2-byte stores made this kernel store-issue-bound); cin, cout are multiples of 8 and 16
  const int tci4 = tci / 4, tco4 = tco / 4;
  for (int i = threadIdx.x; i < tco * taps * tci4; i += 256) {
    const int ci = (i % tci4) * 4, rt = i / tci4;
    const int tap = rt % taps, r = rt / taps;
    float f[4] = {tile[r][ci * taps + tap], tile[r][(ci + 1) * taps + tap], tile[r][(ci + 2) * taps + tap],
                  tile[r][(ci + 3) * taps + tap]};
    P::store4(df + (int64_t)(co0 + r) * s.ldk + tap * s.cin + ci0 + ci, f);
  }
  if (ci0 == 0) {   // zero the K padding of these rows
    const int kp = s.ldk - taps * s.cin;
    for (int i = threadIdx.x; i < tco * kp; i += 256)
      df[(int64_t)(co0 + i / kp) * s.ldk + taps * s.cin + i % kp] = P::from_f(0.f);
  }
  if (s.dst_b >= 0) {
    T* db = dst + (int64_t)c * dst_ld + s.dst_b;
    // Wb[ci][tap·cout + co]: co fastest, 4 per store
    for (int i = threadIdx.x; i < tci * taps * tco4; i += 256) {
      const int r = (i % tco4) * 4, ct = i / tco4;
      const int tap = ct % taps, ci = ct / taps;
      const int q = ci * taps + tap;
      float f[4] = {tile[r][q], tile[r + 1][q], tile[r + 2][q], tile[r + 3][q]};
      P::store4(db + (int64_t)(ci0 + ci) * s.ldk2 + tap * s.cout + co0 + r, f);
    }
    if (co0 == 0) {
      const int kp = s.ldk2 - taps * s.cout;
      for (int i = threadIdx.x; i < tci * kp; i += 256)
        db[(int64_t)(ci0 + i / kp) * s.ldk2 + taps * s.cout + i % kp] = P::from_f(0.f);
    }
  }
}

// total_tiles: Σ ceil(cout/32)·ceil(cin/32) over the segments (0 → the element-wise kernel)
template <class P>
static int pack_weights(const float* arena, int64_t ldw, const void* segs_dev, int nseg, typename P::T* dst,
                        int64_t dst_ld, int C, int total_tiles, int max_taps, hipStream_t stream) {
  if (total_tiles > 0 && max_taps <= PK_MAXTAPS && total_tiles <= (1 << 30))
    hipLaunchKernelGGL(pack_weights_tiled_kernel<P>, dim3(total_tiles, C), dim3(256), 0, stream, arena, ldw,
                       (const PackSeg*)segs_dev, nseg, dst, dst_ld);
  else
    hipLaunchKernelGGL(pack_weights_kernel<P>, dim3(16, C, nseg), dim3(256), 0, stream, arena, ldw,
                       (const PackSeg*)segs_dev, nseg, dst, dst_ld);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_pack_weights(const float* arena, int64_t ldw, const void* segs_dev, int nseg, uint16_t* dst,
                              int64_t dst_ld, int C, int max_tiles, int max_taps, hipStream_t stream) {
  return pack_weights<BF16>(arena, ldw, segs_dev, nseg, dst, dst_ld, C, max_tiles, max_taps, stream);
}
FA_EXPORT int fa_pack_weights_f32(const float* arena, int64_t ldw, const void* segs_dev, int nseg, float* dst,
                                  int64_t dst_ld, int C, int max_tiles, int max_taps, hipStream_t stream) {
  return pack_weights<F32>(arena, ldw, segs_dev, nseg, dst, dst_ld, C, max_tiles, max_taps, stream);
}

// =====================================================================================
// Implicit-GEMM convolution (forward and backward-data share this body).
//
//   out[c][m][n] = Σ_k A[c][m][k] · B[c][n][k],   m = output pixel, n = output channel
//
// A is gathered on the fly from `src` ([C][N][Hs][Ws][KC]) at the input pixel each tap maps
// to, with the operand transform chosen by AOP:
//   AOP_ACT   : a = PRO ? relu(x·s + t) : x           (forward; s,t = previous BN folded)
//   AOP_DY    : a = α·g + β·y + γ                       (bwd-data; g = `src`, y = `src2`)
// Geometry: MODE_FWD  → input pixel = o·stride − pad + tap offset (bounds → 0)
//           MODE_BWD  → dy pixel = (i + pad − tap)/stride when divisible and in range (else 0)
// The workgroup owns one client and a run of 16-pixel tiles; 4 waves, each wave a 16 × NOUT tile
// per iteration; B (packed weights) and the per-channel vectors live in LDS.
// =====================================================================================
enum { AOP_ACT = 0, AOP_DY = 1 };
// MODE_BWD2: backward-data of a 1×1 / stride-2 / pad-0 convolution (the downsample shortcut): iterates
// over the dy pixels (a quarter of the dx grid), writes dx(2i, 2j) = Wᵀ·dy(i, j) and zeros at the three
// other pixels of each 2×2 cell — the generic MODE_BWD runs MFMAs over those zero pixels (4× the work).
// MODE_BWDS2 (K-streamed kernel only): backward-data of a 3×3 / stride-2 / pad-1 convolution split into the
// four parity classes of dx pixels: dx(i, j) only receives taps kh ≡ (i + pad), kw ≡ (j + pad) (mod 2), so
// each class runs a GEMM over its 1, 2, 2 or 4 taps (2.25 on average) instead of 9 taps of which 3/4
// are zero — grid.z carries (N-tile, class).
enum { MODE_FWD = 0, MODE_BWD = 1, MODE_BWD2 = 2, MODE_BWDS2 = 3 };

struct ConvArgs {        // activations / packed weights are P::T (bf16 | fp32)
  const void* src;       // A source activations / g
  const void* src2;      // y for AOP_DY
  const void* wpk;       // packed B [C][NOUT][ldk]
  int64_t wpk_ld;        // per-client stride of the packed weights (elements)
  const float* vec0;     // PRO scale  | α
  const float* vec1;     // PRO shift  | β
  const float* vec2;     //            | γ       | PRO_BOUT: shortcut-BN scale (null: identity)
  const float* vec3;     // PRO_BOUT: shortcut-BN shift
  void* pro_out;         // PRO_BOUT: the formed block output [C][Nb][Hs][Ws][KC]
  void* out;             // [C][M][NOUT]
  // epilogue inputs
  const void* e_x;       // EPI_MASK: previous raw activation (mask + Σg·x); EPI_BLOCK: block input (mask)
  const float* e_s;      // EPI_MASK: previous BN scale
  const float* e_t;      // EPI_MASK: previous BN shift
  const void* e_add;     // EPI_BLOCK: extra gradient (downsample / identity path)
  const void* e_y1;      // EPI_BLOCK: previous block's bn3 input (Σg·y)
  const void* e_y2;      // EPI_BLOCK: previous block's downsample-bn input (optional)
  float* stats;          // [C][NOUT][NS]
  const float* pivot;    // EPI_FWD / EPI_BOUT: per-(client, channel) shift subtracted from the output (or null)
  const float* e_rs;     // EPI_BOUT: downsample-BN scale / shift of the shortcut (null: identity shortcut)
  const float* e_rt;
  const int* nimg;       // per-client valid images (null: all Nb) — heterogeneous client batches
  int NS;
  int Nb, Hs, Ws, KC;    // source geometry (KC = channels of the A source = GEMM K per tap)
  int Ho, Wo;            // output geometry
  int KH, KW, stride, pad;
  int ldk;               // packed row length (≥ K, multiple of 32, +8 pad)
  int Kp;                // K rounded to 32
  int tiles_per_wave;
  int nout_total;        // output channels of the layer; a workgroup computes NOUT of them (blockIdx.z)
  const BnLazy* lz0;     // PRO: deferred finalisation of the prologue BN (vec0/vec1; bnlazy.h) or null
  const BnLazy* lz1;     // PRO_BOUT: ... of the shortcut BN (vec2/vec3)
};

template <class P, int NT, int AOP, int PRO, int MODE, int EPI>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  constexpr int V = P::VEC;
  constexpr int NOUT = NT * 16;
  const int c = blockIdx.y;
  const int NO = a.nout_total;
  const int ch_base = blockIdx.z * NOUT;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int K = a.KH * a.KW * a.KC;
  const int Mo = a.Nb * a.Ho * a.Wo;                             // output pixels per client (tensor layout)
  const int HWi = MODE == MODE_BWD2 ? a.Hs * a.Ws : a.Ho * a.Wo;   // iteration pixels per image
  const int M = MODE == MODE_BWD2 ? a.Nb * HWi : Mo;
  // this client's valid iteration pixels: images past nimg[c] are padding (never read or written)
  const int Mv = a.nimg ? min(M, a.nimg[c] * HWi) : M;
  if ((int)(blockIdx.x * 4 * a.tiles_per_wave) * 16 >= Mv) return;   // uniform: whole workgroup idle

  extern __shared__ __attribute__((aligned(16))) char smem[];
  // fp32: the weight slice is staged as the bank-conflict-free swizzled image of lds_swz.h
  const int wl_ld = P::kF32 ? lswz::pitch(a.Kp) : a.ldk;
  T* wl = reinterpret_cast<T*>(smem);                                            // [NOUT][wl_ld]
  float* v0 = reinterpret_cast<float*>(smem + (size_t)NOUT * wl_ld * P::ES);    // [KC]
  float* v1 = v0 + a.KC;
  float* v2 = v1 + a.KC;
  float* v3 = v2 + a.KC;
  float* red = v3 + a.KC;                                                         // [4][NOUT][3]
  T* stage = reinterpret_cast<T*>(red + 4 * NOUT * 3);                           // [4][16][NOUT]
  T* my_stage = stage + wid * 16 * NOUT;

  // ---- stage packed weights (16-B copies) and per-channel vectors ----
  {
    const T* wsrc = reinterpret_cast<const T*>(a.wpk) + (int64_t)c * a.wpk_ld + (int64_t)ch_base * a.ldk;
    if constexpr (P::kF32) {
      lswz::stage(reinterpret_cast<float*>(wl), reinterpret_cast<const float*>(wsrc), a.ldk, NOUT, a.Kp, threadIdx.x,
                  256);
    } else {
      const uint4* src = reinterpret_cast<const uint4*>(wsrc);
      uint4* dst = reinterpret_cast<uint4*>(wl);
      const int n16 = NOUT * a.ldk / V;
      for (int i = threadIdx.x; i < n16; i += 256) dst[i] = src[i];
    }
    if (AOP == AOP_DY || PRO != PRO_NONE) {
      for (int i = threadIdx.x; i < a.KC; i += 256) {
        if (PRO != PRO_NONE && a.lz0) {
          bn_lazy_fwd(a.lz0, c, i, blockIdx.x == 0 && blockIdx.z == 0, v0[i], v1[i]);
        } else {
          v0[i] = a.vec0[(int64_t)c * a.KC + i];
          v1[i] = a.vec1[(int64_t)c * a.KC + i];
        }
        if (PRO == PRO_BOUT && a.vec2 && a.lz1) {
          bn_lazy_fwd(a.lz1, c, i, blockIdx.x == 0 && blockIdx.z == 0, v2[i], v3[i]);
        } else {
          if (AOP == AOP_DY || (PRO == PRO_BOUT && a.vec2)) v2[i] = a.vec2[(int64_t)c * a.KC + i];
          if (PRO == PRO_BOUT && a.vec2) v3[i] = a.vec3[(int64_t)c * a.KC + i];
        }
      }
    }
    for (int i = threadIdx.x; i < 4 * NOUT * 3; i += 256) red[i] = 0.f;
  }
  __syncthreads();

  const int64_t src_client = (int64_t)c * a.Nb * a.Hs * a.Ws * a.KC;
  const T* src = reinterpret_cast<const T*>(a.src) + src_client;
  const T* src2 = (AOP == AOP_DY || PRO == PRO_BOUT) ? reinterpret_cast<const T*>(a.src2) + src_client : nullptr;
  T* out = a.out ? reinterpret_cast<T*>(a.out) + (int64_t)c * Mo * NO : nullptr;   // null: statistics only (EPI_FWD)
  T* pro_out = (PRO == PRO_BOUT && blockIdx.z == 0) ? reinterpret_cast<T*>(a.pro_out) + src_client : nullptr;
  const T* e_x = reinterpret_cast<const T*>(a.e_x);
  const T* e_add = reinterpret_cast<const T*>(a.e_add);
  const T* e_y1 = reinterpret_cast<const T*>(a.e_y1);
  const T* e_y2 = reinterpret_cast<const T*>(a.e_y2);

  // epilogue per-lane statistics: lane owns the V channels (lane % (NOUT/V))*V .. +V-1
  constexpr int CG = NOUT / V;                 // 16-B chunks per output row
  constexpr int ROWS_PER_PASS = 64 / CG;       // rows covered by one 64-lane pass (CG ≤ 64)
  float st0[V], st1[V], st2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { st0[j] = 0.f; st1[j] = 0.f; st2[j] = 0.f; }
  const int my_cg = lane % CG;
  constexpr int NPASS = (16 + ROWS_PER_PASS - 1) / ROWS_PER_PASS;
  // EPI_BOUT: this lane's BN3 / shortcut-BN vectors (its channel chunk is fixed for the whole kernel)
  float bs[V], bt[V], brs[V], brt[V];
  if (EPI == EPI_BOUT) {
    const int64_t vo = (int64_t)c * NO + ch_base + my_cg * V;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      bs[j] = a.e_s[vo + j];
      bt[j] = a.e_t[vo + j];
      brs[j] = a.e_rs ? a.e_rs[vo + j] : 0.f;
      brt[j] = a.e_rs ? a.e_rt[vo + j] : 0.f;
    }
  }

  const int tiles_total = (Mv + 15) / 16;
  const int tile0 = (blockIdx.x * 4 + wid) * a.tiles_per_wave;
  const int tile_end = min(tiles_total, tile0 + a.tiles_per_wave);
  const int IW = MODE == MODE_BWD2 ? a.Ws : a.Wo;
  // One-deep software pipeline over the wave's (tile, K-chunk) sequence: the raw global operand of the NEXT
  // chunk — the next tile's first chunk at a tile's last one — is issued before this chunk's transform, MFMAs
  // and (at a tile's end) epilogue, so its HBM latency hides behind them instead of stalling the wave.
  constexpr bool TWO = AOP == AOP_DY || PRO == PRO_BOUT;   // second operand stream (y | shortcut)
  int p_tile = tile0, p_k0 = 0, p_on = 0, p_oh = 0, p_ow = 0, p_ci = 0;
  bool p_mvalid = false, p_ok = false;
  int64_t p_off = 0;
  float pf[8], pr[TWO ? 8 : 1];
  auto coords = [&](int tile) {
    const int m = tile * 16 + (lane & 15);
    p_mvalid = m < Mv;
    const int mm = p_mvalid ? m : 0;
    p_on = mm / HWi;
    const int orem = mm % HWi;
    p_oh = orem / IW;
    p_ow = orem % IW;
  };
  auto gather = [&]() {
    p_ok = false;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = 0.f;
    const int k = p_k0 + 8 * (lane >> 4);
    if (p_tile >= tile_end || !p_mvalid || k >= K) return;
    const int tap = k / a.KC, ci = k % a.KC;
    const int kh = tap / a.KW, kw = tap % a.KW;
    int ih, iw;
    bool ok;
    if (MODE == MODE_BWD2) {   // the iteration pixel IS the dy pixel
      ih = p_oh;
      iw = p_ow;
      ok = true;
    } else if (MODE == MODE_FWD) {
      ih = p_oh * a.stride - a.pad + kh;
      iw = p_ow * a.stride - a.pad + kw;
      ok = ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws;
    } else {
      const int th = p_oh + a.pad - kh, tw = p_ow + a.pad - kw;
      ok = th >= 0 && tw >= 0 && (th % a.stride) == 0 && (tw % a.stride) == 0;
      ih = th / a.stride;
      iw = tw / a.stride;
      ok = ok && ih < a.Hs && iw < a.Ws;
    }
    if (!ok) return;
    p_off = (((int64_t)p_on * a.Hs + ih) * a.Ws + iw) * a.KC + ci;
    p_ci = ci;
    p_ok = true;
    P::load8(src + p_off, pf);
    if (TWO) P::load8(src2 + p_off, pr);
  };
  if (tile0 < tile_end) {
    coords(tile0);
    gather();
  }
  for (int tile = tile0; tile < tile_end; ++tile) {
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
    // EPI_BOUT: the shortcut rows of this tile's epilogue, in flight during the K loop
    uint4 rres[EPI == EPI_BOUT ? NPASS : 1];
    if (EPI == EPI_BOUT) {
      const int rv = min(16, Mv - tile * 16);
#pragma unroll
      for (int pass = 0; pass < NPASS; ++pass) {
        const int row = pass * ROWS_PER_PASS + lane / CG;
        rres[pass] = make_uint4(0, 0, 0, 0);
        if (lane / CG < ROWS_PER_PASS && row < rv)
          rres[pass] = *reinterpret_cast<const uint4*>(e_add + (int64_t)c * Mo * NO +
                                                       (int64_t)(tile * 16 + row) * NO + ch_base + my_cg * V);
      }
    }

    for (int k0 = 0; k0 < a.Kp; k0 += 32) {
      float f[8], r[TWO ? 8 : 1];
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = pf[j];
      if (TWO) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = pr[j];
      }
      const bool ok = p_ok;
      const int ci = p_ci;
      const int64_t off = p_off;
      p_k0 += 32;   // advance the pipeline and issue the next chunk's loads
      if (p_k0 >= a.Kp) {
        p_k0 = 0;
        if (++p_tile < tile_end) coords(p_tile);
      }
      gather();
      if (ok) {
        if (AOP == AOP_ACT && PRO == PRO_BNRELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j] * v0[ci + j] + v1[ci + j], 0.f);
        } else if (AOP == AOP_ACT && PRO == PRO_BOUT) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] * v0[ci + j] + v1[ci + j];
          if (a.vec2) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += r[j] * v2[ci + j] + v3[ci + j];
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += r[j];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = P::round(fmaxf(f[j], 0.f));   // the operand = the stored value
          if (pro_out) {
#pragma unroll
            for (int q = 0; q < 8 / V; ++q) *reinterpret_cast<uint4*>(pro_out + off + q * V) = P::pack(f + q * V);
          }
        } else if (AOP == AOP_DY) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = v0[ci + j] * f[j] + v1[ci + j] * r[j] + v2[ci + j];
        }
      }
      const frag_t afrag = P::frag8(f);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        frag_t bv;
        if constexpr (P::kF32) {
          float wf[8];
          lswz::load8(reinterpret_cast<const float*>(wl), a.Kp, nt * 16 + (lane & 15), k0 + 8 * (lane >> 4), wf);
          bv = P::frag8(wf);
        } else {
          bv = P::frag(wl + (nt * 16 + (lane & 15)) * a.ldk + k0 + 8 * (lane >> 4));
        }
        acc[nt] = P::mma(afrag, bv, acc[nt]);
      }
    }

    // ---- stage the 16 × NOUT tile (storage precision) in LDS; forward outputs as y − K (pivot) ----
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float k = ((EPI == EPI_FWD || EPI == EPI_BOUT) && a.pivot)
                          ? a.pivot[(int64_t)c * NO + ch_base + nt * 16 + (lane & 15)] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 4 * (lane >> 4) + i;
        my_stage[row * NOUT + nt * 16 + (lane & 15)] = P::from_f(acc[nt][i] - k);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes visible to this wave
    __builtin_amdgcn_wave_barrier();

    // ---- vectorised epilogue: each lane handles V channels of one row per pass ----
    const int rows_valid = min(16, Mv - tile * 16);
#pragma unroll
    for (int pass = 0; pass < (16 + ROWS_PER_PASS - 1) / ROWS_PER_PASS; ++pass) {
      const int row = pass * ROWS_PER_PASS + lane / CG;
      if (lane / CG < ROWS_PER_PASS && row < rows_valid) {
        const int ch0 = my_cg * V;
        const uint4 dv = *reinterpret_cast<const uint4*>(my_stage + row * NOUT + ch0);
        int64_t goff = ((int64_t)(tile * 16 + row)) * NO + ch_base + ch0;
        if (MODE == MODE_BWD2) {   // dy pixel → dx (2i, 2j); zeros at the other three pixels of the cell
          const int pm = tile * 16 + row;
          const int n_ = pm / HWi, r_ = pm % HWi;
          const int64_t px = ((int64_t)n_ * a.Ho + 2 * (r_ / a.Ws)) * a.Wo + 2 * (r_ % a.Ws);
          goff = px * NO + ch_base + ch0;
          const uint4 z = make_uint4(0, 0, 0, 0);
          *reinterpret_cast<uint4*>(out + goff + NO) = z;
          *reinterpret_cast<uint4*>(out + goff + (int64_t)a.Wo * NO) = z;
          *reinterpret_cast<uint4*>(out + goff + (int64_t)(a.Wo + 1) * NO) = z;
        }
        if (EPI == EPI_BOUT) {
          float f[V], r[V];
          P::unpack(dv, f);
          P::unpack(rres[EPI == EPI_BOUT ? pass : 0], r);
#pragma unroll
          for (int j = 0; j < V; ++j) {
            f[j] = f[j] * bs[j] + bt[j];   // same operation order as block_out_kernel
            f[j] += a.e_rs ? r[j] * brs[j] + brt[j] : r[j];
            f[j] = fmaxf(f[j], 0.f);
          }
          *reinterpret_cast<uint4*>(out + goff) = P::pack(f);
        } else if (EPI == EPI_FWD || EPI == EPI_STORE) {
          if (EPI == EPI_STORE || out) *reinterpret_cast<uint4*>(out + goff) = dv;
          if (EPI == EPI_FWD) {
            float f[V];
            P::unpack(dv, f);
#pragma unroll
            for (int j = 0; j < V; ++j) { st0[j] += f[j]; st1[j] += f[j] * f[j]; }
          }
        } else {
          const int64_t eoff = (int64_t)c * Mo * NO + goff;
          float g[V], xv[V];
          P::unpack(dv, g);
          P::unpack(*reinterpret_cast<const uint4*>(e_x + eoff), xv);
          if (EPI == EPI_MASK) {
#pragma unroll
            for (int j = 0; j < V; ++j) {
              const int ch = ch0 + j;
              const bool on_ = xv[j] * a.e_s[(int64_t)c * NO + ch_base + ch] + a.e_t[(int64_t)c * NO + ch_base + ch] > 0.f;
              g[j] = on_ ? g[j] : 0.f;
            }
          } else {  // EPI_BLOCK: g = (g + extra) · [block_input > 0]
            float ex[V];
            P::unpack(*reinterpret_cast<const uint4*>(e_add + eoff), ex);
#pragma unroll
            for (int j = 0; j < V; ++j) g[j] = (xv[j] > 0.f) ? g[j] + ex[j] : 0.f;
          }
          const uint4 gp = P::pack(g);
          *reinterpret_cast<uint4*>(out + goff) = gp;
          float gr[V];
          P::unpack(gp, gr);
          if (EPI == EPI_MASK) {
#pragma unroll
            for (int j = 0; j < V; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * xv[j]; }
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) st0[j] += gr[j];
            if (e_y1) {   // null: the previous BN's Σg·y comes from elsewhere (recomputed-y bottlenecks)
              float y1[V];
              P::unpack(*reinterpret_cast<const uint4*>(e_y1 + eoff), y1);
#pragma unroll
              for (int j = 0; j < V; ++j) st1[j] += gr[j] * y1[j];
            }
            if (e_y2) {
              float y2[V];
              P::unpack(*reinterpret_cast<const uint4*>(e_y2 + eoff), y2);
#pragma unroll
              for (int j = 0; j < V; ++j) st2[j] += gr[j] * y2[j];
            }
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ---- statistics: reduce lanes sharing a channel group, then waves, then one atomic ----
  if (EPI != EPI_STORE && EPI != EPI_BOUT) {
#pragma unroll
    for (int o = CG; o < 64; o <<= 1) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        st0[j] += __shfl_xor(st0[j], o, 64);
        st1[j] += __shfl_xor(st1[j], o, 64);
        if (EPI == EPI_BLOCK) st2[j] += __shfl_xor(st2[j], o, 64);
      }
    }
    if (lane < CG) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int ch = lane * V + j;
        red[(wid * NOUT + ch) * 3 + 0] = st0[j];
        red[(wid * NOUT + ch) * 3 + 1] = st1[j];
        red[(wid * NOUT + ch) * 3 + 2] = st2[j];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NOUT * a.NS; i += 256) {
      const int ch = i / a.NS, q = i % a.NS;
      const float s = red[(0 * NOUT + ch) * 3 + q] + red[(1 * NOUT + ch) * 3 + q] + red[(2 * NOUT + ch) * 3 + q] +
                      red[(3 * NOUT + ch) * 3 + q];
      fa_acc_add(&a.stats[((int64_t)c * NO + ch_base + ch) * a.NS + q], s);
    }
  }
}

template <class P>
static size_t conv_smem_bytes(int nout, int ldk, int kc, int Kp) {
  if (P::kF32) ldk = lswz::pitch(Kp);   // the swizzled weight image (lds_swz.h)
  return (size_t)nout * ldk * P::ES + (size_t)4 * kc * 4 + (size_t)4 * nout * 3 * 4 + (size_t)4 * 16 * nout * P::ES;
}

// =====================================================================================
// K-streamed implicit GEMM for WIDE layers (ResNet-18: 64–512 channels, K = 9·Cin up to 4608).
//
// conv_gemm_kernel keeps the whole [NOUT][K] weight slice resident in LDS, which stops fitting
// (fp32: 64 × 4608 × 4 B = 1.2 MB) or leaves one workgroup per CU. Here BOTH operands stream through
// LDS in K-chunks: the workgroup tile is BM = 64·TPW pixels × 64 output channels, wave w owns
// pixel rows [16·TPW·w, 16·TPW·(w+1)) × all 64 channels (TPW × 4 MFMA tiles). Per chunk every thread
//   * has the chunk's global data already in registers (issued one whole chunk earlier: the
//     gathers' latency hides behind a chunk of MFMAs, not one K step),
//   * stores it to LDS applying the operand transform (BN+ReLU prologue | folded BN backward),
//   * issues the next chunk's loads, then runs the chunk's MFMAs from LDS
//     (per 32-K step: TPW + 4 fragment reads for 4·TPW MFMAs).
// Coalesced staging: 16-B vectors, consecutive lanes read consecutive channels of one pixel.
// Epilogue as conv_gemm_kernel (stage the tile in LDS, vectorised stores, statistics).
// =====================================================================================
template <class P, int TM, int WN>
struct ConvK {
  static constexpr int WM = 4 / WN;                                        // waves along M
  static constexpr int KB = 64 / (P::kF32 ? 2 : 1);                        // K elements per chunk (128 B rows)
  static constexpr int LD = KB + (P::kF32 ? 4 : 8);                        // LDS pitch (elements)
  static constexpr int BN = 64 * WN;                                       // output channels per workgroup
  static constexpr int BM = 16 * TM * WM;                                  // pixels per workgroup
  static constexpr int CPR = KB / P::VEC;                                  // 16-B chunks per row (8)
  static constexpr int RPI = 256 / CPR;                                    // rows per thread pass (32)
  static constexpr int NA = BM / RPI;                                      // A chunks per thread
  static constexpr int NB = BN / RPI;                                      // B chunks per thread
  static_assert(NA >= 1 && NB >= 1, "tile too small for the staging map");
  static_assert(4 * 16 * 64 <= (BM + BN) * LD, "epilogue staging must fit the operand tiles");
  static size_t smem(int kc) { return (size_t)(BM + BN) * LD * P::ES + (size_t)4 * kc * 4 + (size_t)4 * 64 * 3 * 4; }
};

// wave (wm, wn) = (wid / WN, wid % WN) owns pixel rows [16·TM·wm, +16·TM) × channels [64·wn, +64) of the
// workgroup tile: TM × 4 MFMA tiles, TM + 4 fragment reads per 4·TM MFMAs per 32-K step.
template <class P, int TM, int WN, int AOP, int PRO, int MODE, int EPI>
__global__ __launch_bounds__(256) void convk_gemm_kernel(ConvArgs a) {
  using T = typename P::T;
  using frag_t = typename P::frag_t;
  using CK = ConvK<P, TM, WN>;
  constexpr int V = P::VEC;
  constexpr int NT = 4;
  constexpr int NOUT = 64;      // channels per wave (epilogue unit)
  constexpr int KB = CK::KB;
  constexpr int LD = CK::LD;
  constexpr bool DY = AOP == AOP_DY;
  // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs (linear id mod 8); remap so
  // each XCD runs a contiguous run of (client, N-tile, M-tile) — the tiles that share one client's
  // weights and activations hit the same L2
  const int gx = gridDim.x, gz = gridDim.z;
  const int total = gx * gridDim.y * gz;
  int lin = blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z);
  const int full = total / 8 * 8;
  if (lin < full) lin = (lin % 8) * (full / 8) + lin / 8;
  const int bx = lin % gx;
  const int bzz = (lin / gx) % gz;
  const int c = lin / (gx * gz);
  constexpr bool S2 = MODE == MODE_BWDS2;
  const int bz = S2 ? bzz >> 2 : bzz;
  // stride-2 parity class: dx rows i ≡ r0, cols j ≡ c0 (mod 2); taps kh = qh + 2t (t < nth), kw = qw + 2u
  const int qh = (bzz >> 1) & 1, qw = bzz & 1;
  const int r0 = S2 ? (qh + a.pad) & 1 : 0, c0 = S2 ? (qw + a.pad) & 1 : 0;
  const int nth = S2 ? (a.KH - qh + 1) / 2 : 1, ntw = S2 ? (a.KW - qw + 1) / 2 : 1;
  const int Hc = S2 ? (a.Ho - r0 + 1) / 2 : 0, Wc = S2 ? (a.Wo - c0 + 1) / 2 : 0;
  const int NO = a.nout_total;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ch_base = bz * CK::BN;
  const int ch_w = ch_base + wn * 64;
  const int K = S2 ? nth * ntw * a.KC : a.KH * a.KW * a.KC;
  const int Kp = S2 ? (K + 31) / 32 * 32 : a.Kp;
  const int Mo = a.Nb * a.Ho * a.Wo;
  const int HWi = MODE == MODE_BWD2 ? a.Hs * a.Ws : (S2 ? Hc * Wc : a.Ho * a.Wo);
  const int M = (MODE == MODE_BWD2 || S2) ? a.Nb * HWi : Mo;
  const int Mv = a.nimg ? min(M, a.nimg[c] * HWi) : M;
  const int m0 = bx * CK::BM;
  if (m0 >= Mv) return;   // uniform: whole workgroup idle (also: classes smaller than the grid)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* al = reinterpret_cast<T*>(smem);                                               // [BM][LD]
  T* wl = al + CK::BM * LD;                                                         // [BN][LD]
  float* v0 = reinterpret_cast<float*>(wl + CK::BN * LD);                          // [KC]
  float* v1 = v0 + a.KC;
  float* v2 = v1 + a.KC;
  float* v3 = v2 + a.KC;                                                            // PRO_BOUT: shortcut-BN shift
  float* red = v3 + a.KC;                                                           // [4 waves][64][3]
  T* my_stage = al + wid * 16 * NOUT;   // epilogue staging [4][16][64] reuses the operand tiles
  // PRO_BOUT (1×1 / stride 1): the operand is the previous block's output relu(y·s + t + r), r = src2 | src2·v2 + v3,
  // formed at staging (same operation order as block_out_kernel) and written once to pro_out by the first
  // N-tile's workgroups
  constexpr bool BOUT = PRO == PRO_BOUT;
  if (DY || PRO == PRO_BNRELU || BOUT) {
    for (int i = threadIdx.x; i < a.KC; i += 256) {
      if (!DY && a.lz0) {
        bn_lazy_fwd(a.lz0, c, i, bx == 0 && bzz == 0, v0[i], v1[i]);
      } else {
        v0[i] = a.vec0[(int64_t)c * a.KC + i];
        v1[i] = a.vec1[(int64_t)c * a.KC + i];
      }
      if (DY) v2[i] = a.vec2[(int64_t)c * a.KC + i];
      if (BOUT && a.vec2) {
        if (a.lz1) {
          bn_lazy_fwd(a.lz1, c, i, bx == 0 && bzz == 0, v2[i], v3[i]);
        } else {
          v2[i] = a.vec2[(int64_t)c * a.KC + i];
          v3[i] = a.vec3[(int64_t)c * a.KC + i];
        }
      }
    }
  }
  for (int i = threadIdx.x; i < 4 * NOUT * 3; i += 256) red[i] = 0.f;

  const int64_t src_client = (int64_t)c * a.Nb * a.Hs * a.Ws * a.KC;
  const T* src = reinterpret_cast<const T*>(a.src) + src_client;
  constexpr bool TWO = DY || BOUT;   // second operand stream (y | shortcut)
  const T* src2 = TWO ? reinterpret_cast<const T*>(a.src2) + src_client : nullptr;
  T* pro_out = (BOUT && bz == 0) ? reinterpret_cast<T*>(a.pro_out) + src_client : nullptr;
  // null: statistics only (EPI_FWD; the recomputed-y backward takes a conv's BN statistics from the same kernel)
  T* out = a.out ? reinterpret_cast<T*>(a.out) + (int64_t)c * Mo * NO : nullptr;
  const T* wsrc = reinterpret_cast<const T*>(a.wpk) + (int64_t)c * a.wpk_ld + (int64_t)ch_base * a.ldk;

  // this thread's staging slots: column chunk `col` of rows row0 + RPI·j
  const int col = threadIdx.x % CK::CPR;
  const int row0 = threadIdx.x / CK::CPR;
  const int IW = MODE == MODE_BWD2 ? a.Ws : (S2 ? Wc : a.Wo);
  // Uniform-tap path (every ResNet-18 wide layer: KC % KB == 0): a K-chunk then lies inside ONE tap, so the
  // tap, its pixel delta and the channel base are wave-uniform. Each staged row keeps its base element
  // offset and a validity bit per tap (computed once), and a chunk's gather costs one add and one bit test
  // per row — the generic decode below (two runtime divisions, bounds and 64-bit offsets per row and chunk)
  // made this kernel VALU-issue-bound: ~420 VALU instructions per 32 MFMAs of a chunk (profiles/r5_convk_valu.txt).
  const int ntap = S2 ? nth * ntw : a.KH * a.KW;
  const bool UT = (a.KC % KB == 0) && ntap <= 32 && (MODE != MODE_BWD || a.stride == 1) &&
                  (int64_t)a.Nb * a.Hs * a.Ws * a.KC < (1ll << 31);   // 32-bit element offsets
  int rn[CK::NA], rhw[CK::NA];   // image index, (h << 16 | w) of the row's iteration pixel; rn < 0: invalid
  int rbase[CK::NA];             // UT: element offset of the row's tap-(0,0) source pixel + this thread's column
  uint32_t rmask[CK::NA];        // UT: bit t = tap t of this row reads inside the image
#pragma unroll
  for (int j = 0; j < CK::NA; ++j) {
    const int m = m0 + row0 + CK::RPI * j;
    rbase[j] = 0;
    rmask[j] = 0;
    if (m < Mv) {
      rn[j] = m / HWi;
      const int r = m % HWi;
      const int ph = r / IW, pw = r % IW;
      rhw[j] = (ph << 16) | pw;
      if (UT) {
        // source pixel of tap t = (h0 + dh(t), w0 + dw(t)), dh/dw as in tap_delta below
        int h0, w0;
        if (MODE == MODE_FWD) { h0 = ph * a.stride - a.pad; w0 = pw * a.stride - a.pad; }
        else if (MODE == MODE_BWD) { h0 = ph + a.pad; w0 = pw + a.pad; }
        else if (MODE == MODE_BWD2) { h0 = ph; w0 = pw; }
        else { h0 = ph + ((r0 + a.pad - qh) >> 1); w0 = pw + ((c0 + a.pad - qw) >> 1); }
        rbase[j] = ((rn[j] * a.Hs + h0) * a.Ws + w0) * a.KC + col * V;
        for (int t = 0; t < ntap; ++t) {
          const int tr = S2 ? t / ntw : t / a.KW, tc = S2 ? t % ntw : t % a.KW;
          const int ih = MODE == MODE_FWD ? h0 + tr : h0 - tr, iw = MODE == MODE_FWD ? w0 + tc : w0 - tc;
          if ((unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws) rmask[j] |= 1u << t;
        }
      }
    } else {
      rn[j] = -1;
      rhw[j] = 0;
    }
  }
  // UT chunk state (uniform): tap index and channel base of the chunk fetched last, advanced per fetch
  int u_tap = 0, u_ci0 = 0, u_tr = 0, u_tc = 0;
  const int u_tcn = S2 ? ntw : a.KW;   // taps per tap row
  const int wrow = row0 * a.ldk + col * V;

  f32x4 acc[TM][NT];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[t][nt] = {0.f, 0.f, 0.f, 0.f};

  uint4 ra[CK::NA], ry[TWO ? CK::NA : 1], rb[CK::NB];
  int64_t aoff[BOUT ? CK::NA : 1];   // PRO_BOUT: the operand element's position (pro_out write)
  uint32_t aval = 0;
  int p_ci = 0;                      // channel of this thread's first element in the fetched chunk
  auto fetch = [&](int kbase) {
    if (UT) {
      if (kbase == 0) { u_tap = 0; u_ci0 = 0; u_tr = 0; u_tc = 0; }
      const int dh = MODE == MODE_FWD ? u_tr : -u_tr, dw = MODE == MODE_FWD ? u_tc : -u_tc;
      const int uoff = (dh * a.Ws + dw) * a.KC + u_ci0;
      const int kh = S2 ? qh + 2 * u_tr : u_tr, kw = S2 ? qw + 2 * u_tc : u_tc;
      const int kcol = (kh * a.KW + kw) * a.KC + u_ci0;   // column of the packed weights (chunk start)
      p_ci = u_ci0 + col * V;
      aval = 0;
#pragma unroll
      for (int j = 0; j < CK::NA; ++j) {
        ra[j] = make_uint4(0, 0, 0, 0);
        if (TWO) ry[j] = make_uint4(0, 0, 0, 0);
        if ((rmask[j] >> u_tap) & 1u) {
          const int off = rbase[j] + uoff;
          ra[j] = *reinterpret_cast<const uint4*>(src + off);
          if (TWO) ry[j] = *reinterpret_cast<const uint4*>(src2 + off);
          if constexpr (BOUT) aoff[j] = off;
          aval |= 1u << j;
        }
      }
#pragma unroll
      for (int j = 0; j < CK::NB; ++j)
        rb[j] = *reinterpret_cast<const uint4*>(wsrc + kcol + (wrow + CK::RPI * j * a.ldk));
      // advance to the next chunk: channel base, then tap (column, row)
      u_ci0 += KB;
      if (u_ci0 == a.KC) {
        u_ci0 = 0;
        ++u_tap;
        if (++u_tc == u_tcn) { u_tc = 0; ++u_tr; }
      }
      return;
    }
    const int k = kbase + col * V;
    const bool kval = k < K;
    const int tap = kval ? k / a.KC : 0, ci = kval ? k % a.KC : 0;
    const int kh = S2 ? qh + 2 * (tap / ntw) : tap / a.KW, kw = S2 ? qw + 2 * (tap % ntw) : tap % a.KW;
    const int kcol = S2 ? (kh * a.KW + kw) * a.KC + ci : k;   // column of the packed weights
    p_ci = ci;
    aval = 0;
#pragma unroll
    for (int j = 0; j < CK::NA; ++j) {
      ra[j] = make_uint4(0, 0, 0, 0);
      if (TWO) ry[j] = make_uint4(0, 0, 0, 0);
      if (rn[j] >= 0 && kval) {
        const int ph = rhw[j] >> 16, pw = rhw[j] & 0xffff;
        int ih, iw;
        bool ok;
        if (MODE == MODE_BWD2) {
          ih = ph; iw = pw; ok = true;
        } else if (MODE == MODE_FWD) {
          ih = ph * a.stride - a.pad + kh;
          iw = pw * a.stride - a.pad + kw;
          ok = ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws;
        } else if (S2) {   // dx (2ph + r0, 2pw + c0): the parity makes (i + pad − kh) even by construction
          ih = (2 * ph + r0 + a.pad - kh) >> 1;
          iw = (2 * pw + c0 + a.pad - kw) >> 1;
          ok = 2 * ph + r0 + a.pad - kh >= 0 && 2 * pw + c0 + a.pad - kw >= 0 && ih < a.Hs && iw < a.Ws;
        } else {
          const int th = ph + a.pad - kh, tw = pw + a.pad - kw;
          ok = th >= 0 && tw >= 0 && (th % a.stride) == 0 && (tw % a.stride) == 0;
          ih = th / a.stride;
          iw = tw / a.stride;
          ok = ok && ih < a.Hs && iw < a.Ws;
        }
        if (ok) {
          const int64_t off = (((int64_t)rn[j] * a.Hs + ih) * a.Ws + iw) * a.KC + ci;
          ra[j] = *reinterpret_cast<const uint4*>(src + off);
          if (TWO) ry[j] = *reinterpret_cast<const uint4*>(src2 + off);
          if constexpr (BOUT) aoff[j] = off;
          aval |= 1u << j;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < CK::NB; ++j)
      rb[j] = kval ? *reinterpret_cast<const uint4*>(wsrc + (int64_t)(row0 + CK::RPI * j) * a.ldk + kcol)
                   : make_uint4(0, 0, 0, 0);
  };
  auto put = [&](int) {
    const int ci = p_ci;
    // the chunk's per-channel coefficients, read from LDS once for all NA rows (the row loop's LDS stores
    // otherwise make the compiler re-read them per row)
    float c0v[(PRO == PRO_BNRELU || DY) ? V : 1], c1v[(PRO == PRO_BNRELU || DY) ? V : 1], c2v[DY ? V : 1];
    if constexpr (PRO == PRO_BNRELU || DY) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        c0v[e] = v0[ci + e];
        c1v[e] = v1[ci + e];
        if (DY) c2v[e] = v2[ci + e];
      }
    }
#pragma unroll
    for (int j = 0; j < CK::NA; ++j) {
      uint4 v = make_uint4(0, 0, 0, 0);   // out-of-image taps / padding rows: 0 (not the transform of 0)
      if ((aval >> j) & 1u) {
        if constexpr (BOUT) {
          float f[V], r[V];
          P::unpack(ra[j], f);
          P::unpack(ry[j], r);
#pragma unroll
          for (int e = 0; e < V; ++e) {
            f[e] = f[e] * v0[ci + e] + v1[ci + e];
            f[e] += a.vec2 ? r[e] * v2[ci + e] + v3[ci + e] : r[e];
            f[e] = P::round(fmaxf(f[e], 0.f));   // the operand = the stored value
          }
          v = P::pack(f);
          if (pro_out) *reinterpret_cast<uint4*>(pro_out + aoff[j]) = v;
        } else if (PRO == PRO_BNRELU || DY) {
          float f[V];
          P::unpack(ra[j], f);
          if (DY) {
            float yv[V];
            P::unpack(ry[j], yv);
#pragma unroll
            for (int e = 0; e < V; ++e) f[e] = c0v[e] * f[e] + c1v[e] * yv[e] + c2v[e];
          } else {
#pragma unroll
            for (int e = 0; e < V; ++e) f[e] = fmaxf(f[e] * c0v[e] + c1v[e], 0.f);
          }
          v = P::pack(f);
        } else {
          v = ra[j];
        }
      }
      P::st_tile(al + (row0 + CK::RPI * j) * LD + col * V, col, v);
    }
#pragma unroll
    for (int j = 0; j < CK::NB; ++j) P::st_tile(wl + (row0 + CK::RPI * j) * LD + col * V, col, rb[j]);
  };

  const T* my_a = al + (wm * 16 * TM + (lane & 15)) * LD + 8 * (lane >> 4);
  const T* my_b = wl + (wn * 64 + (lane & 15)) * LD + 8 * (lane >> 4);
  __syncthreads();   // prologue vectors visible to put()
  fetch(0);
  for (int kbase = 0; kbase < Kp; kbase += KB) {
    const int kn = min(KB, Kp - kbase);     // multiple of 32
    if (kbase) __syncthreads();             // previous chunk fully consumed
    put(kbase);
    __syncthreads();
    if (kbase + KB < Kp) fetch(kbase + KB);
    for (int k0 = 0; k0 < kn; k0 += 32) {
      frag_t af[TM];
#pragma unroll
      for (int t = 0; t < TM; ++t) af[t] = P::frag_tile(my_a + t * 16 * LD + k0);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const frag_t bv = P::frag_tile(my_b + nt * 16 * LD + k0);
#pragma unroll
        for (int t = 0; t < TM; ++t) acc[t][nt] = P::mma(af[t], bv, acc[t][nt]);
      }
    }
  }
  __syncthreads();   // every wave done with the operand tiles before they hold the epilogue staging
  const int tiles_total = (Mv + 15) / 16;
  const int tile0 = m0 / 16 + wm * TM;
  const T* e_x = reinterpret_cast<const T*>(a.e_x);
  const T* e_add = reinterpret_cast<const T*>(a.e_add);
  const T* e_y1 = reinterpret_cast<const T*>(a.e_y1);
  const T* e_y2 = reinterpret_cast<const T*>(a.e_y2);
  constexpr int CG = NOUT / V;
  constexpr int ROWS_PER_PASS = 64 / CG;
  float st0[V], st1[V], st2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { st0[j] = 0.f; st1[j] = 0.f; st2[j] = 0.f; }
  const int my_cg = lane % CG;
  float kpiv[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    kpiv[nt] = (EPI == EPI_FWD && a.pivot) ? a.pivot[(int64_t)c * NO + ch_w + nt * 16 + (lane & 15)] : 0.f;

#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int tile = tile0 + t;
    if (tile >= tiles_total) break;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        my_stage[(4 * (lane >> 4) + i) * NOUT + nt * 16 + (lane & 15)] = P::from_f(acc[t][nt][i] - kpiv[nt]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int rows_valid = min(16, Mv - tile * 16);
#pragma unroll
    for (int pass = 0; pass < (16 + ROWS_PER_PASS - 1) / ROWS_PER_PASS; ++pass) {
      const int row = pass * ROWS_PER_PASS + lane / CG;
      if (lane / CG < ROWS_PER_PASS && row < rows_valid) {
        const int ch0 = my_cg * V;
        const uint4 dv = *reinterpret_cast<const uint4*>(my_stage + row * NOUT + ch0);
        int64_t goff = ((int64_t)(tile * 16 + row)) * NO + ch_w + ch0;
        if (S2) {   // class pixel (n, a, b) → dx (2a + r0, 2b + c0)
          const int pm = tile * 16 + row;
          const int n_ = pm / HWi, r_ = pm % HWi;
          goff = (((int64_t)n_ * a.Ho + 2 * (r_ / Wc) + r0) * a.Wo + 2 * (r_ % Wc) + c0) * NO + ch_w + ch0;
        }
        if (MODE == MODE_BWD2) {
          const int pm = tile * 16 + row;
          const int n_ = pm / HWi, r_ = pm % HWi;
          const int64_t px = ((int64_t)n_ * a.Ho + 2 * (r_ / a.Ws)) * a.Wo + 2 * (r_ % a.Ws);
          goff = px * NO + ch_w + ch0;
          const uint4 z = make_uint4(0, 0, 0, 0);
          *reinterpret_cast<uint4*>(out + goff + NO) = z;
          *reinterpret_cast<uint4*>(out + goff + (int64_t)a.Wo * NO) = z;
          *reinterpret_cast<uint4*>(out + goff + (int64_t)(a.Wo + 1) * NO) = z;
        }
        if (EPI == EPI_FWD || EPI == EPI_STORE) {
          if (EPI == EPI_STORE || out) *reinterpret_cast<uint4*>(out + goff) = dv;
          if (EPI == EPI_FWD) {
            float f[V];
            P::unpack(dv, f);
#pragma unroll
            for (int j = 0; j < V; ++j) { st0[j] += f[j]; st1[j] += f[j] * f[j]; }
          }
        } else {
          const int64_t eoff = (int64_t)c * Mo * NO + goff;
          float g[V], xv[V];
          P::unpack(dv, g);
          P::unpack(*reinterpret_cast<const uint4*>(e_x + eoff), xv);
          if (EPI == EPI_MASK) {
#pragma unroll
            for (int j = 0; j < V; ++j) {
              const int ch = ch_w + ch0 + j;
              const bool on_ = xv[j] * a.e_s[(int64_t)c * NO + ch] + a.e_t[(int64_t)c * NO + ch] > 0.f;
              g[j] = on_ ? g[j] : 0.f;
            }
          } else {
            float ex[V];
            P::unpack(*reinterpret_cast<const uint4*>(e_add + eoff), ex);
#pragma unroll
            for (int j = 0; j < V; ++j) g[j] = (xv[j] > 0.f) ? g[j] + ex[j] : 0.f;
          }
          const uint4 gp = P::pack(g);
          *reinterpret_cast<uint4*>(out + goff) = gp;
          float gr[V];
          P::unpack(gp, gr);
          if (EPI == EPI_MASK) {
#pragma unroll
            for (int j = 0; j < V; ++j) { st0[j] += gr[j]; st1[j] += gr[j] * xv[j]; }
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) st0[j] += gr[j];
            if (e_y1) {   // null: the previous BN's Σg·y comes from elsewhere (recomputed-y bottlenecks)
              float y1[V];
              P::unpack(*reinterpret_cast<const uint4*>(e_y1 + eoff), y1);
#pragma unroll
              for (int j = 0; j < V; ++j) st1[j] += gr[j] * y1[j];
            }
            if (e_y2) {
              float y2[V];
              P::unpack(*reinterpret_cast<const uint4*>(e_y2 + eoff), y2);
#pragma unroll
              for (int j = 0; j < V; ++j) st2[j] += gr[j] * y2[j];
            }
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  if (EPI != EPI_STORE) {
#pragma unroll
    for (int o = CG; o < 64; o <<= 1) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        st0[j] += __shfl_xor(st0[j], o, 64);
        st1[j] += __shfl_xor(st1[j], o, 64);
        if (EPI == EPI_BLOCK) st2[j] += __shfl_xor(st2[j], o, 64);
      }
    }
    if (lane < CG) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int ch = lane * V + j;
        red[(wid * NOUT + ch) * 3 + 0] = st0[j];
        red[(wid * NOUT + ch) * 3 + 1] = st1[j];
        red[(wid * NOUT + ch) * 3 + 2] = st2[j];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < CK::BN * a.NS; i += 256) {
      const int chb = i / a.NS, q = i % a.NS;
      const int wn_ = chb / 64, ch = chb % 64;
      float s = 0.f;
#pragma unroll
      for (int m_ = 0; m_ < CK::WM; ++m_) s += red[((m_ * WN + wn_) * NOUT + ch) * 3 + q];
      fa_acc_add(&a.stats[((int64_t)c * NO + ch_base + chb) * a.NS + q], s);
    }
  }
}

// K above which (or outputs above 256) the K-streamed kernel runs; FEDML_AMD_CONVK_MIN_K overrides
static int convk_min_k() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FEDML_AMD_CONVK_MIN_K");
    // 256 → 128 (round 4): the 256 → 64 block-output 1×1 of the headline's 8² stage runs faster as the K-streamed
    // GEMM plus a separate block-output pass than as the fused generic kernel — headline fp32 +0.8 %, 13-client share
    // +1.4 %, MobileNet +2 %, ResNet-18 neutral (profiles/r4_bench_convk_min_k.jsonl); 256 in round 3: ResNet-18 +9 %.
    // 128 → 32 (round 5, after the K-streamed kernel's uniform-tap gather): 13-client share 10.09 → 10.21 rounds/s
    // over three alternating pairs, headline unchanged (profiles/r5_convk_min_k_ab.txt)
    v = e ? atoi(e) : 32;
  }
  return v;
}

template <class P, int TM, int WN, int AOP, int PRO, int MODE, int EPI>
static int launch_convk_t(ConvArgs a, int nout, int C, hipStream_t stream) {
  using CK = ConvK<P, TM, WN>;
  a.nout_total = nout;
  if (nout % CK::BN != 0) return -2;
  // MODE_BWDS2: the largest parity class sets grid.x; grid.z = N-tiles × 4 classes
  const int M = MODE == MODE_BWD2 ? a.Nb * a.Hs * a.Ws
                                  : (MODE == MODE_BWDS2 ? a.Nb * ((a.Ho + 1) / 2) * ((a.Wo + 1) / 2) : a.Nb * a.Ho * a.Wo);
  const int gx = (M + CK::BM - 1) / CK::BM;
  const size_t smem = CK::smem(a.KC);
  if (smem > 160 * 1024) return -5;
  auto kern = convk_gemm_kernel<P, TM, WN, AOP, PRO, MODE, EPI>;
  if (smem > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C, nout / CK::BN * (MODE == MODE_BWDS2 ? 4 : 1)), dim3(256), smem, stream, a);
  return (int)hipGetLastError();
}

// tile shape: 128 × 128 (2 × 2 waves of 64 × 64) for ≥ 128 outputs; 64-output layers 256 / 128 / 64 × 64
// by the workgroup count (FEDML_AMD_CONVK_TILE forces 0: 128x128, 1: 256x64, 2: 128x64, 3: 64x64)
template <class P, int AOP, int PRO, int MODE, int EPI>
static int launch_convk(ConvArgs a, int nout, int C, hipStream_t s) {
  static int force = -2;
  if (force == -2) {
    const char* e = getenv("FEDML_AMD_CONVK_TILE");
    force = e ? atoi(e) : -1;
  }
  if (nout % 64 != 0) return -2;
  const int M = MODE == MODE_BWD2 ? a.Nb * a.Hs * a.Ws : a.Nb * a.Ho * a.Wo;   // (BWDS2: all 4 classes)
  const int64_t wgs1 = (int64_t)((M + 63) / 64) * fa_plan_c(C) * (nout / 64);   // workgroups of a 64 × 64 tile
  int pick = force;
  // fp32 wide layers take 64 × 64 tiles too: the fp32 128 × 128 tile (operands twice the bytes, 16 accumulator
  // tiles per wave) runs fewer waves per CU — ResNet-18 preset fp32 0.392 → 0.410 rounds/s, bf16 keeps 128 × 128
  // (1.124 vs 1.055 rounds/s with 64 × 64; profiles/r3_bench_secondary_final.jsonl)
  if (pick < 0) pick = nout % 128 == 0 ? (P::kF32 ? 3 : 0) : (wgs1 >= 4096 ? 1 : (wgs1 >= 1024 ? 2 : 3));
  switch (pick) {
    case 0: return launch_convk_t<P, 4, 2, AOP, PRO, MODE, EPI>(a, nout, C, s);
    case 1: return launch_convk_t<P, 4, 1, AOP, PRO, MODE, EPI>(a, nout, C, s);
    case 2: return launch_convk_t<P, 2, 1, AOP, PRO, MODE, EPI>(a, nout, C, s);
    default: return launch_convk_t<P, 1, 1, AOP, PRO, MODE, EPI>(a, nout, C, s);
  }
}

template <class P, int NT, int AOP, int PRO, int MODE, int EPI>
static int launch_conv(ConvArgs a, int nout, int C, hipStream_t stream) {
  a.nout_total = nout;
  const int M = MODE == MODE_BWD2 ? a.Nb * a.Hs * a.Ws : a.Nb * a.Ho * a.Wo;
  const int tiles = (M + 15) / 16;
  const int per_wg = 4 * a.tiles_per_wave;
  const int gx = (tiles + per_wg - 1) / per_wg;
  const size_t smem = conv_smem_bytes<P>(NT * 16, a.ldk, a.KC, a.Kp);
  if (smem > 160 * 1024) return -5;
  auto kern = conv_gemm_kernel<P, NT, AOP, PRO, MODE, EPI>;
  if (smem > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C, nout / (NT * 16)), dim3(256), smem, stream, a);
  return (int)hipGetLastError();
}

// Wide outputs (128/256 channels) are split over blockIdx.z in 64-channel slices: the per-WG weight
// and epilogue-staging LDS shrinks 2–4× (several workgroups per CU instead of one), at the cost of
// re-reading the (narrow) A operand once per slice.
template <class P, int AOP, int PRO, int MODE, int EPI>
static int dispatch_nt(int nout, const ConvArgs& a, int C, hipStream_t s) {
  // wide layers (ResNet-18 stages 2-4): weights streamed through LDS in K-chunks
  if (nout % 64 == 0 && (nout > 256 || a.KH * a.KW * a.KC > convk_min_k()))
    return launch_convk<P, AOP, PRO, MODE, EPI>(a, nout, C, s);
  switch (nout) {
    case 16: return launch_conv<P, 1, AOP, PRO, MODE, EPI>(a, nout, C, s);
    case 32: return launch_conv<P, 2, AOP, PRO, MODE, EPI>(a, nout, C, s);
    case 64:
    case 128:
    case 256:
      // 64-channel slices; narrower when the packed-weight slice would not fit the LDS (fp32, K ≥ 576)
      if (conv_smem_bytes<P>(64, a.ldk, a.KC, a.Kp) <= 160 * 1024)
        return launch_conv<P, 4, AOP, PRO, MODE, EPI>(a, nout, C, s);
      if (conv_smem_bytes<P>(32, a.ldk, a.KC, a.Kp) <= 160 * 1024)
        return launch_conv<P, 2, AOP, PRO, MODE, EPI>(a, nout, C, s);
      return launch_conv<P, 1, AOP, PRO, MODE, EPI>(a, nout, C, s);
    default: return -2;
  }
}

// =====================================================================================
// fp32 1×1 / stride-1 "expand" forward: the bottleneck's last conv, planes → 4·planes (ResNet-56/110: 16 → 64 at
// 32², 32 → 128 at 16², 64 → 256 at 8²), y = conv(pro(x)) − K with the BN statistics of the stored y
// (reference block: python/fedml/model/cv/resnet.py:110 conv3, :127 in forward; its conv1, :106 / :119, is the
// block-output-forming kernel below).
//
// The generic conv_gemm_kernel pads K to 32 (half of every 16-channel layer's MFMAs multiply zeros), stages each
// 16 × 64 output tile through LDS and keeps one 1-KB operand load in flight per wave: 3.8–4.0 TB/s on a layer that
// is 80 % output writes (profiles/r5_resnet56_fp32_c100_layer_roofline.txt). Here, per wave:
//   * the weights of its 64-channel output slice stay in registers for the whole launch (Cin VGPRs),
//   * the MFMA computes the TRANSPOSED tile D[channel][pixel] (A = W, B = xᵀ), so a lane owns 4 consecutive
//     channels of one pixel: the epilogue is one 16-B store per lane and MFMA tile, no LDS staging,
//   * the 4-wide K slice of MFMA (kb, j) is input channel 16·kb + 4·(lane>>4) + j: every lane's operand is one
//     16-B load per 16 input channels, and K = Cin exactly (no padding),
//   * U pixel tiles of 16 per iteration, the next iteration's operands loaded before this one's MFMAs.
// Workgroup = 4 waves; S = Cout / 64 of them take the S channel slices of the SAME pixel tiles (the operand is
// read once from HBM, the other slices hit the CU's L1/L2), 4 / S wave rows split the workgroup's pixel run.
// Exact fp32 products (v_mfma_f32_16x16x4_f32), fp32 accumulation; statistics reduced lane → wave → workgroup →
// one fa_acc_add per (channel, moment) (fixed point in deterministic mode).
// =====================================================================================
namespace c1x {

// 16-B output store; nt: non-temporal (streaming) — the layer's output is far larger than L2 / MALL at C = 100
__device__ __forceinline__ void st4(float* p, float4 v, int nt) {
  if (nt) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}

template <int CIN, int S, int PRO, int U>
__global__ __launch_bounds__(256, 2) void conv1x1_expand_f32_kernel(ConvArgs a, int gpw, int nts) {
  constexpr int KB = CIN / 16;           // 16-channel input blocks
  constexpr int R = 4 / S;               // wave rows per workgroup
  constexpr int NO = 64 * S;             // output channels (= Cout)
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, px_l = lane & 15;
  const int slice = wid % S, row = wid / S;
  const int M = a.Nb * a.Ho * a.Wo;
  const int Mv = a.nimg ? min(M, a.nimg[c] * a.Ho * a.Wo) : M;
  const int groups = (Mv + 16 * U - 1) / (16 * U);
  if ((int)blockIdx.x * R * gpw >= groups) return;   // uniform: the whole workgroup is idle

  __shared__ float vs[CIN], vt[CIN];
  __shared__ float red[4][64][2];
  if (PRO == PRO_BNRELU) {
    for (int i = threadIdx.x; i < CIN; i += 256) {
      float s_, t_;
      if (a.lz0) {
        bn_lazy_fwd(a.lz0, c, i, blockIdx.x == 0, s_, t_);
      } else {
        s_ = a.vec0[(int64_t)c * CIN + i];
        t_ = a.vec1[(int64_t)c * CIN + i];
      }
      vs[i] = s_;
      vt[i] = t_;
    }
  }
  __syncthreads();

  // per-lane constants: weights W[co = 64·slice + 16·nt + px_l][16·kb + 4·g + 0..3], BN fold, pivot
  float4 w[4][KB];
  const float* wsrc = reinterpret_cast<const float*>(a.wpk) + (int64_t)c * a.wpk_ld;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      w[nt][kb] = *reinterpret_cast<const float4*>(wsrc + (int64_t)(64 * slice + 16 * nt + px_l) * a.ldk + 16 * kb +
                                                   4 * g);
  float4 s4[KB], t4[KB];
  if (PRO == PRO_BNRELU) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      s4[kb] = *reinterpret_cast<const float4*>(vs + 16 * kb + 4 * g);
      t4[kb] = *reinterpret_cast<const float4*>(vt + 16 * kb + 4 * g);
    }
  }
  float4 kp[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
    kp[nt] = a.pivot ? *reinterpret_cast<const float4*>(a.pivot + (int64_t)c * NO + 64 * slice + 16 * nt + 4 * g)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  float st0[4][4], st1[4][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) st0[nt][r] = st1[nt][r] = 0.f;

  const float* src = reinterpret_cast<const float*>(a.src) + (int64_t)c * M * CIN;
  float* out = a.out ? reinterpret_cast<float*>(a.out) + (int64_t)c * M * NO : nullptr;
  const int gbeg = ((int)blockIdx.x * R + row) * gpw;
  const int gend = min(groups, gbeg + gpw);

  float4 xb[U][KB];
  auto load = [&](int gi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int px = (gi * U + u) * 16 + px_l;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        xb[u][kb] = px < Mv ? *reinterpret_cast<const float4*>(src + (int64_t)px * CIN + 16 * kb + 4 * g)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  if (gbeg < gend) load(gbeg);
  for (int gi = gbeg; gi < gend; ++gi) {
    float4 xc[U][KB];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) xc[u][kb] = xb[u][kb];
    if (gi + 1 < gend) load(gi + 1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p0 = (gi * U + u) * 16;
      if (p0 >= Mv) break;   // uniform: Mv is a multiple of 16 (whole images)
      f32x4 acc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        float xv[4] = {xc[u][kb].x, xc[u][kb].y, xc[u][kb].z, xc[u][kb].w};
        if (PRO == PRO_BNRELU) {
          xv[0] = fmaxf(xv[0] * s4[kb].x + t4[kb].x, 0.f);
          xv[1] = fmaxf(xv[1] * s4[kb].y + t4[kb].y, 0.f);
          xv[2] = fmaxf(xv[2] * s4[kb].z + t4[kb].z, 0.f);
          xv[3] = fmaxf(xv[3] * s4[kb].w + t4[kb].w, 0.f);
        }
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const float wv[4] = {w[nt][kb].x, w[nt][kb].y, w[nt][kb].z, w[nt][kb].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[j], xv[j], acc[nt], 0, 0, 0);
        }
      }
      const int64_t px = p0 + px_l;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float y0 = acc[nt][0] - kp[nt].x, y1 = acc[nt][1] - kp[nt].y;
        const float y2 = acc[nt][2] - kp[nt].z, y3 = acc[nt][3] - kp[nt].w;
        if (out) st4(out + px * NO + 64 * slice + 16 * nt + 4 * g, make_float4(y0, y1, y2, y3), nts);
        st0[nt][0] += y0; st1[nt][0] += y0 * y0;
        st0[nt][1] += y1; st1[nt][1] += y1 * y1;
        st0[nt][2] += y2; st1[nt][2] += y2 * y2;
        st0[nt][3] += y3; st1[nt][3] += y3 * y3;
      }
    }
  }

  // statistics: the 16 lanes of a lane group hold the same 16 channels (4 per MFMA tile) → xor-reduce, then the
  // wave rows of a slice through LDS, then one atomic per (channel, moment)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st0[nt][r] += __shfl_xor(st0[nt][r], o, 64);
        st1[nt][r] += __shfl_xor(st1[nt][r], o, 64);
      }
  if (px_l == 0) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wid][16 * nt + 4 * g + r][0] = st0[nt][r];
        red[wid][16 * nt + 4 * g + r][1] = st1[nt][r];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NO * 2; i += 256) {
    const int sl = i / 128, ch = (i >> 1) & 63, q = i & 1;
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < R; ++rr) s += red[rr * S + sl][ch][q];
    fa_acc_add(&a.stats[((int64_t)c * NO + 64 * sl + ch) * 2 + q], s);
  }
}

// fp32 1×1 / stride-1 forward with the previous block's output formed in the operand load (PRO_BOUT): the
// bottleneck's first conv, 4·planes (or 2·planes at a stage entry) → planes. Per 16-pixel tile a lane loads its
// 4-channel pieces of y and the shortcut r for every 16-channel input block, forms a = relu(y·s + t + r)
// (r → r·rs + rt behind a downsample BN; block_out_kernel's operation order, so the same bits), writes the block
// output once and feeds the transposed MFMA (D[channel][pixel]) from registers; the weights
// [COUT][CIN] sit in LDS (pitch CIN + 8, bank-conflict free), the BN
// vectors too. The operands stream in 64-channel chunks (8 16-B loads per lane), one chunk ahead.
// BOUT = false: the plain 1×1 forward of the same shapes (operand = the stored block output as is, nothing written
// but y): the unfused path's conv then sums in exactly the fused kernel's order — both paths give the same bits
template <int CIN, int COUT, bool BOUT>
__global__ __launch_bounds__(256, 2) void conv1x1_pbout_f32_kernel(ConvArgs a, int gpw, int nts) {
  // LDW ≡ 8 (mod 64) dwords: the 16 rows × 4 lane groups of a ds_read_b128 fragment read (row px_l, column 4·g)
  // land on 16 distinct 4-bank slots (CIN + 4 measured 56–64 % bank-conflict cycles)
  constexpr int KB = CIN / 16, NT = COUT / 16, LDW = CIN + 8;
  const int c = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, px_l = lane & 15;
  const int M = a.Nb * a.Ho * a.Wo;
  const int Mv = a.nimg ? min(M, a.nimg[c] * a.Ho * a.Wo) : M;
  const int tiles = Mv / 16;
  if ((int)blockIdx.x * 4 * gpw >= tiles) return;   // uniform

  __shared__ __attribute__((aligned(16))) float wl[COUT * LDW];
  __shared__ __attribute__((aligned(16))) float vs[CIN], vt[CIN], vrs[CIN], vrt[CIN];
  __shared__ float red[4][COUT][2];
  const bool ds = BOUT && a.vec2 != nullptr;   // downsample-BN shortcut
  for (int i = threadIdx.x; i < (BOUT ? CIN : 0); i += 256) {
    float s_, t_;
    if (a.lz0) {
      bn_lazy_fwd(a.lz0, c, i, blockIdx.x == 0, s_, t_);
    } else {
      s_ = a.vec0[(int64_t)c * CIN + i];
      t_ = a.vec1[(int64_t)c * CIN + i];
    }
    vs[i] = s_;
    vt[i] = t_;
    if (ds) {
      if (a.lz1) {
        bn_lazy_fwd(a.lz1, c, i, blockIdx.x == 0, s_, t_);
      } else {
        s_ = a.vec2[(int64_t)c * CIN + i];
        t_ = a.vec3[(int64_t)c * CIN + i];
      }
      vrs[i] = s_;
      vrt[i] = t_;
    }
  }
  {
    const float* wsrc = reinterpret_cast<const float*>(a.wpk) + (int64_t)c * a.wpk_ld;
    for (int i = threadIdx.x; i < COUT * CIN / 4; i += 256) {
      const int co = i / (CIN / 4), k4 = i % (CIN / 4);
      *reinterpret_cast<float4*>(wl + co * LDW + 4 * k4) =
          *reinterpret_cast<const float4*>(wsrc + (int64_t)co * a.ldk + 4 * k4);
    }
  }
  __syncthreads();

  float4 kp[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    kp[nt] = a.pivot ? *reinterpret_cast<const float4*>(a.pivot + (int64_t)c * COUT + 16 * nt + 4 * g)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  float st0[NT][4], st1[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) st0[nt][r] = st1[nt][r] = 0.f;

  const int64_t cin_off = (int64_t)c * M * CIN;
  const float* ysrc = reinterpret_cast<const float*>(a.src) + cin_off;
  const float* rsrc = BOUT ? reinterpret_cast<const float*>(a.src2) + cin_off : nullptr;
  float* bout = BOUT ? reinterpret_cast<float*>(a.pro_out) + cin_off : nullptr;
  float* out = reinterpret_cast<float*>(a.out) + (int64_t)c * M * COUT;
  const int tbeg = ((int)blockIdx.x * 4 + wid) * gpw;
  const int tend = min(tiles, tbeg + gpw);
  // (tile, 64-channel chunk) sequence, one chunk's 8 operand loads in flight ahead of the chunk being computed
  constexpr int NQ = KB / 4;   // chunks per tile
  float4 py[4], pr[4];
  auto load = [&](int tile, int q) {
    const int64_t px = (int64_t)tile * 16 + px_l;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      py[k] = *reinterpret_cast<const float4*>(ysrc + px * CIN + 64 * q + 16 * k + 4 * g);
      if (BOUT) pr[k] = *reinterpret_cast<const float4*>(rsrc + px * CIN + 64 * q + 16 * k + 4 * g);
    }
  };
  if (tbeg < tend) load(tbeg, 0);
  for (int tile = tbeg; tile < tend; ++tile) {
    const int64_t px = (int64_t)tile * 16 + px_l;
    // LDS offsets made opaque per tile: the weight / BN-vector reads are loop-invariant, and hoisted out of the
    // tile loop they would hold CIN·COUT/16 + CIN/2 VGPRs (spills at CIN ≥ 128)
    int lo = 4 * g;
    asm volatile("" : "+v"(lo));
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float4 yv[4], rv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) { yv[k] = py[k]; rv[k] = BOUT ? pr[k] : py[k]; }
      if (q + 1 < NQ) load(tile, q + 1);
      else if (tile + 1 < tend) load(tile + 1, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ci = 64 * q + 16 * k + 4 * g;
        const int cl = 64 * q + 16 * k + lo;   // == ci
        float f[4] = {yv[k].x, yv[k].y, yv[k].z, yv[k].w};
        if (BOUT) {
        const float4 s4 = *reinterpret_cast<const float4*>(vs + cl), t4 = *reinterpret_cast<const float4*>(vt + cl);
        const float r[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
        const float sv[4] = {s4.x, s4.y, s4.z, s4.w}, tv[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = f[j] * sv[j] + tv[j];
        if (ds) {
          const float4 a4 = *reinterpret_cast<const float4*>(vrs + cl), b4 = *reinterpret_cast<const float4*>(vrt + cl);
          const float rs[4] = {a4.x, a4.y, a4.z, a4.w}, rt[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) f[j] += r[j] * rs[j] + rt[j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) f[j] += r[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = fmaxf(f[j], 0.f);
        st4(bout + px * CIN + ci, make_float4(f[0], f[1], f[2], f[3]), nts);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const float4 w4 = *reinterpret_cast<const float4*>(wl + (16 * nt + px_l) * LDW + cl);
          const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[j], f[j], acc[nt], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float y0 = acc[nt][0] - kp[nt].x, y1 = acc[nt][1] - kp[nt].y;
      const float y2 = acc[nt][2] - kp[nt].z, y3 = acc[nt][3] - kp[nt].w;
      st4(out + px * COUT + 16 * nt + 4 * g, make_float4(y0, y1, y2, y3), nts);
      st0[nt][0] += y0; st1[nt][0] += y0 * y0;
      st0[nt][1] += y1; st1[nt][1] += y1 * y1;
      st0[nt][2] += y2; st1[nt][2] += y2 * y2;
      st0[nt][3] += y3; st1[nt][3] += y3 * y3;
    }
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st0[nt][r] += __shfl_xor(st0[nt][r], o, 64);
        st1[nt][r] += __shfl_xor(st1[nt][r], o, 64);
      }
  if (px_l == 0) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wid][16 * nt + 4 * g + r][0] = st0[nt][r];
        red[wid][16 * nt + 4 * g + r][1] = st1[nt][r];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < COUT * 2; i += 256) {
    const int ch = i >> 1, q = i & 1;
    const float s = red[0][ch][q] + red[1][ch][q] + red[2][ch][q] + red[3][ch][q];
    fa_acc_add(&a.stats[((int64_t)c * COUT + ch) * 2 + q], s);
  }
}

static int g_enable = -1;   // FEDML_AMD_C1X (default on); fa_set_c1x overrides
// launch sizing (tuning): total workgroup target and the minimum pixels per wave, which bounds how often a wave
// refills its weight slice (16 KB per wave at 64 input channels) for few clients
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
// measured at C = 100 (profiles/r6_c1x_wgs.txt): 8192 workgroups for the 32² expand (473 → 428 µs) and the 16²
// block-output-forming kernels (588 → 552, 627 → 569 µs); 2048 for the rest (the 8² block-output kernel 304 → 349 µs
// and the 16² expand 248 → 262 µs at 8192)
static int wg_target(int dflt) {
  static int v = -2;
  if (v == -2) v = env_int("FEDML_AMD_C1X_WGS", -1);
  return std::max(64, v > 0 ? v : dflt);
}
// expand: ≥ 128 px per wave (13 clients, 8² stage: 41 → 34 µs per call); block-output-forming: no minimum (its
// 8² stage measured 63 → 80 µs at 128) — profiles/r6_c1x_sizing.txt
static int min_px_per_wave(bool expand) {
  static int v[2] = {-1, -1};
  if (v[expand] < 0) v[expand] = std::max(16, env_int(expand ? "FEDML_AMD_C1X_MINPX" : "FEDML_AMD_C1X_PB_MINPX",
                                                      expand ? 128 : 16));
  return v[expand];
}
static int nt_stores() {     // FEDML_AMD_C1X_NT: non-temporal output stores (measured slower: off; profiles/r6_c1x_ab.txt)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FEDML_AMD_C1X_NT");
    v = e ? (atoi(e) != 0) : 0;
  }
  return v;
}

template <int CIN, int S, int PRO>
static int launch_t(const ConvArgs& a, int C, hipStream_t stream) {
  constexpr int U = CIN >= 64 ? 2 : 4;
  constexpr int R = 4 / S;
  const int M = a.Nb * a.Ho * a.Wo;
  const int groups = (M + 16 * U - 1) / (16 * U);
  // ≈ 2048 workgroups over the launch (8 per CU), ≥ 2 pixel groups per wave
  const int pc = fa_plan_c(C);
  const int wgs_target = std::max(1, (wg_target(CIN == 16 ? 8192 : 2048) + pc - 1) / pc);
  const int gpw = std::max(std::max(2, min_px_per_wave(true) / (16 * U)), (groups + wgs_target * R - 1) / (wgs_target * R));
  const int gx = (groups + R * gpw - 1) / (R * gpw);
  hipLaunchKernelGGL((conv1x1_expand_f32_kernel<CIN, S, PRO, U>), dim3(gx, C), dim3(256), 0, stream, a, gpw,
                     nt_stores());
  return (int)hipGetLastError();
}

// 1 when the expand kernel took the launch; 0: not its shape (the caller runs the generic kernels)
template <class P>
static int try_launch(const ConvArgs& a, int Cin, int Cout, int KH, int KW, int stride, int pad, int C, bool bnrelu,
                      hipStream_t stream, int* rc) {
  if (g_enable < 0) {
    const char* e = getenv("FEDML_AMD_C1X");
    g_enable = e ? (atoi(e) != 0) : 1;
  }
  // a null output is the statistics-only pass of the recomputed-y bottleneck, whose EPI_BOUT pass re-runs the
  // generic kernel: both must sum in the same order, so it stays there
  if (!g_enable || !std::is_same<P, prec::F32>::value || !a.out) return 0;
  if (KH != 1 || KW != 1 || stride != 1 || pad != 0 || a.Ho != a.Hs || a.Wo != a.Ws || Cout != 4 * Cin) return 0;
  // whole 16-pixel tiles per image: a tile never straddles the valid / padding boundary of a ragged client
  if (a.ldk % 4 != 0 || a.wpk_ld % 4 != 0 || (a.Ho * a.Wo) % 16 != 0) return 0;
  switch ((Cin << 1) | (bnrelu ? 1 : 0)) {
    case (16 << 1) | 1: *rc = launch_t<16, 1, PRO_BNRELU>(a, C, stream); return 1;
    case (32 << 1) | 1: *rc = launch_t<32, 2, PRO_BNRELU>(a, C, stream); return 1;
    case (64 << 1) | 1: *rc = launch_t<64, 4, PRO_BNRELU>(a, C, stream); return 1;
    case (16 << 1): *rc = launch_t<16, 1, PRO_NONE>(a, C, stream); return 1;
    case (32 << 1): *rc = launch_t<32, 2, PRO_NONE>(a, C, stream); return 1;
    case (64 << 1): *rc = launch_t<64, 4, PRO_NONE>(a, C, stream); return 1;
    default: return 0;
  }
}

template <int CIN, int COUT, bool BOUT = true>
static int launch_pbout_t(const ConvArgs& a, int C, hipStream_t stream) {
  const int tiles = a.Nb * a.Ho * a.Wo / 16;
  const int pc = fa_plan_c(C);
  const int wgs_target = std::max(1, (wg_target(CIN == 128 ? 8192 : 2048) + pc - 1) / pc);
  const int gpw = std::max(min_px_per_wave(false) / 16, (tiles + wgs_target * 4 - 1) / (wgs_target * 4));
  const int gx = (tiles + 4 * gpw - 1) / (4 * gpw);
  hipLaunchKernelGGL((conv1x1_pbout_f32_kernel<CIN, COUT, BOUT>), dim3(gx, C), dim3(256), 0, stream, a, gpw,
                     nt_stores());
  return (int)hipGetLastError();
}

template <class P>
static int try_pbout(const ConvArgs& a, int Cin, int Cout, int C, hipStream_t stream, int* rc) {
  if (g_enable < 0) {
    const char* e = getenv("FEDML_AMD_C1X");
    g_enable = e ? (atoi(e) != 0) : 1;
  }
  if (!g_enable || !std::is_same<P, prec::F32>::value || !a.out) return 0;
  if (a.ldk % 4 != 0 || a.wpk_ld % 4 != 0 || (a.Ho * a.Wo) % 16 != 0) return 0;
  // 64-channel inputs (the 32² stage) stay on the generic kernel: measured 1151 vs 1112 µs (64 → 16) and 1311 vs
  // 1089 µs (64 → 32) per call at C = 100; the 16² / 8² stages gain (567 vs 594, 307 vs 338, 609 vs 694 µs)
  if (getenv("FEDML_AMD_C1X_PB64") && atoi(getenv("FEDML_AMD_C1X_PB64"))) {
    if (Cin * 1000 + Cout == 64016) { *rc = launch_pbout_t<64, 16>(a, C, stream); return 1; }
    if (Cin * 1000 + Cout == 64032) { *rc = launch_pbout_t<64, 32>(a, C, stream); return 1; }
  }
  switch (Cin * 1000 + Cout) {
    case 128032: *rc = launch_pbout_t<128, 32>(a, C, stream); return 1;
    case 256064: *rc = launch_pbout_t<256, 64>(a, C, stream); return 1;
    case 128064: *rc = launch_pbout_t<128, 64>(a, C, stream); return 1;
    default: return 0;
  }
}

// the plain (PRO_NONE) 1×1 / stride-1 forward of the block-output-forming shapes: same kernel, same sums
template <class P>
static int try_plain_reduce(const ConvArgs& a, int Cin, int Cout, int KH, int KW, int stride, int pad, int C,
                            hipStream_t stream, int* rc) {
  if (g_enable < 0) {
    const char* e = getenv("FEDML_AMD_C1X");
    g_enable = e ? (atoi(e) != 0) : 1;
  }
  if (!g_enable || !std::is_same<P, prec::F32>::value || !a.out) return 0;
  if (KH != 1 || KW != 1 || stride != 1 || pad != 0 || a.Ho != a.Hs || a.Wo != a.Ws) return 0;
  if (a.ldk % 4 != 0 || a.wpk_ld % 4 != 0 || (a.Ho * a.Wo) % 16 != 0) return 0;
  switch (Cin * 1000 + Cout) {
    case 128032: *rc = launch_pbout_t<128, 32, false>(a, C, stream); return 1;
    case 256064: *rc = launch_pbout_t<256, 64, false>(a, C, stream); return 1;
    case 128064: *rc = launch_pbout_t<128, 64, false>(a, C, stream); return 1;
    default: return 0;
  }
}

}  // namespace c1x

// FEDML_AMD_C1X override (tests / A-B runs): 1 on, 0 off (generic kernels); returns the previous setting
FA_EXPORT int fa_set_c1x(int on) {
  const int prev = c1x::g_enable;
  c1x::g_enable = on ? 1 : 0;
  return prev;
}

template <class P>
static int conv_fwd(const void* x, const void* wpk, int64_t wpk_ld, const float* pscale, const float* pshift, void* y,
                    float* stats, int C, int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                    int Ho, int Wo, int ldk, int tiles_per_wave, const float* pivot, const int* nimg,
                    hipStream_t stream) {
  if (Cin % 8 != 0) return -3;
  ConvArgs a = {};
  a.src = x; a.wpk = wpk; a.wpk_ld = wpk_ld; a.vec0 = pscale; a.vec1 = pshift; a.out = y; a.stats = stats; a.NS = 2;
  a.pivot = pivot; a.nimg = nimg;
  a.Nb = Nb; a.Hs = H; a.Ws = W; a.KC = Cin; a.Ho = Ho; a.Wo = Wo; a.KH = KH; a.KW = KW; a.stride = stride;
  a.pad = pad; a.ldk = ldk; a.Kp = (KH * KW * Cin + 31) / 32 * 32; a.tiles_per_wave = tiles_per_wave;
  a.lz0 = fa_take_lazy(0);
  a.lz1 = fa_take_lazy(1);
  int rc = 0;
  if (c1x::try_launch<P>(a, Cin, Cout, KH, KW, stride, pad, C, pscale != nullptr, stream, &rc)) return rc;
  if (!pscale && c1x::try_plain_reduce<P>(a, Cin, Cout, KH, KW, stride, pad, C, stream, &rc)) return rc;
  if (pscale)
    return dispatch_nt<P, AOP_ACT, PRO_BNRELU, MODE_FWD, EPI_FWD>(Cout, a, C, stream);
  return dispatch_nt<P, AOP_ACT, PRO_NONE, MODE_FWD, EPI_FWD>(Cout, a, C, stream);
}

// 1×1 / stride-1 forward whose operand is the previous block's output formed on the fly (PRO_BOUT), written to
// `bout` on the way: bout = relu(yp·s + t + r), r = res | res·rs + rt;  y = conv(bout) − K, stats as conv_fwd
template <class P>
static int conv_fwd_pbout(const void* yp, const float* s, const float* t, const void* res, const float* rs,
                          const float* rt, void* bout, const void* wpk, int64_t wpk_ld, void* y, float* stats, int C,
                          int Nb, int H, int W, int Cin, int Cout, int ldk, int tiles_per_wave, const float* pivot,
                          const int* nimg, hipStream_t stream) {
  if (Cin % 8 != 0 || !s || !t || !res || !bout || (rs && !rt)) return -3;
  ConvArgs a = {};
  a.src = yp; a.src2 = res; a.vec0 = s; a.vec1 = t; a.vec2 = rs; a.vec3 = rt; a.pro_out = bout;
  a.wpk = wpk; a.wpk_ld = wpk_ld; a.out = y; a.stats = stats; a.NS = 2; a.pivot = pivot; a.nimg = nimg;
  a.Nb = Nb; a.Hs = H; a.Ws = W; a.KC = Cin; a.Ho = H; a.Wo = W; a.KH = 1; a.KW = 1; a.stride = 1;
  a.pad = 0; a.ldk = ldk; a.Kp = (Cin + 31) / 32 * 32; a.tiles_per_wave = tiles_per_wave;
  a.lz0 = fa_take_lazy(0);
  a.lz1 = fa_take_lazy(1);
  int rc = 0;
  if (c1x::try_pbout<P>(a, Cin, Cout, C, stream, &rc)) return rc;
  // wide layers: the K-streamed kernel forms the operand at its LDS staging (dispatch_nt routes them there)
  return dispatch_nt<P, AOP_ACT, PRO_BOUT, MODE_FWD, EPI_FWD>(Cout, a, C, stream);
}

// bottleneck block output from the last 1×1 conv (EPI_BOUT): out = relu(BN(conv(relu(x·ps + pt)) − K) + shortcut)
template <class P>
static int conv_fwd_bout(const void* x, const void* wpk, int64_t wpk_ld, const float* pscale, const float* pshift,
                         void* out, const float* s, const float* t, const float* pivot, const void* res, const float* rs,
                         const float* rt, int C, int Nb, int H, int W, int Cin, int Cout, int ldk, int tiles_per_wave,
                         const int* nimg, hipStream_t stream) {
  if (Cin % 8 != 0 || Cout % 64 != 0 || !pscale || !s || !t || !res || (rs && !rt)) return -3;
  ConvArgs a = {};
  a.src = x; a.wpk = wpk; a.wpk_ld = wpk_ld; a.vec0 = pscale; a.vec1 = pshift; a.out = out; a.NS = 2;
  a.e_s = s; a.e_t = t; a.pivot = pivot; a.e_add = res; a.e_rs = rs; a.e_rt = rt; a.nimg = nimg;
  a.Nb = Nb; a.Hs = H; a.Ws = W; a.KC = Cin; a.Ho = H; a.Wo = W; a.KH = 1; a.KW = 1; a.stride = 1;
  a.pad = 0; a.ldk = ldk; a.Kp = (Cin + 31) / 32 * 32; a.tiles_per_wave = tiles_per_wave;
  if (conv_smem_bytes<P>(64, a.ldk, a.KC, a.Kp) > 160 * 1024) return -5;
  return launch_conv<P, 4, AOP_ACT, PRO_BNRELU, MODE_FWD, EPI_BOUT>(a, Cout, C, stream);
}

template <class P, int AOP>
static int conv_bwd_data_dispatch(const ConvArgs& a, int epi, int C, int Cin, int Cout, int KH, int KW, int stride,
                                  int pad, int Hx, int Wx, int Hy, int Wy, hipStream_t stream) {
  // 3×3 / stride-2 / pad-1 (ResNet-18 stage entries): parity-class GEMMs over the valid taps only
  if (KH == 3 && KW == 3 && stride == 2 && pad == 1 && Cin % 64 == 0 && Cout % 64 == 0) {
    switch (epi) {
      case EPI_STORE: return launch_convk<P, AOP, PRO_NONE, MODE_BWDS2, EPI_STORE>(a, Cin, C, stream);
      case EPI_MASK: return launch_convk<P, AOP, PRO_NONE, MODE_BWDS2, EPI_MASK>(a, Cin, C, stream);
      case EPI_BLOCK: return launch_convk<P, AOP, PRO_NONE, MODE_BWDS2, EPI_BLOCK>(a, Cin, C, stream);
      default: return -4;
    }
  }
  switch (epi) {
    case EPI_STORE:
      if (KH == 1 && KW == 1 && stride == 2 && pad == 0 && Hx == 2 * Hy && Wx == 2 * Wy)
        return dispatch_nt<P, AOP, PRO_NONE, MODE_BWD2, EPI_STORE>(Cin, a, C, stream);
      return dispatch_nt<P, AOP, PRO_NONE, MODE_BWD, EPI_STORE>(Cin, a, C, stream);
    case EPI_MASK: return dispatch_nt<P, AOP, PRO_NONE, MODE_BWD, EPI_MASK>(Cin, a, C, stream);
    case EPI_BLOCK: return dispatch_nt<P, AOP, PRO_NONE, MODE_BWD, EPI_BLOCK>(Cin, a, C, stream);
    default: return -4;
  }
}

template <class P>
static int conv_bwd_data(const void* g, const void* yv, const float* alpha, const float* beta, const float* gamma,
                         const void* wpk_b, int64_t wpk_ld, void* dx, int epi, const void* e_x, const float* e_s,
                         const float* e_t, const void* e_add, const void* e_y1, const void* e_y2, float* stats, int C,
                         int Nb, int Hy, int Wy, int Cout, int Cin, int KH, int KW, int stride, int pad, int Hx, int Wx,
                         int ldk2, int tiles_per_wave, const int* nimg, hipStream_t stream) {
  if (Cout % 8 != 0) return -3;
  ConvArgs a = {};
  a.nimg = nimg;
  a.src = g; a.src2 = yv; a.wpk = wpk_b; a.wpk_ld = wpk_ld; a.vec0 = alpha; a.vec1 = beta; a.vec2 = gamma;
  a.out = dx; a.e_x = e_x; a.e_s = e_s; a.e_t = e_t; a.e_add = e_add; a.e_y1 = e_y1; a.e_y2 = e_y2;
  a.stats = stats; a.NS = 3;  // backward statistics are always laid out [C][Ch][3]
  a.Nb = Nb; a.Hs = Hy; a.Ws = Wy; a.KC = Cout; a.Ho = Hx; a.Wo = Wx; a.KH = KH; a.KW = KW; a.stride = stride;
  a.pad = pad; a.ldk = ldk2; a.Kp = (KH * KW * Cout + 31) / 32 * 32; a.tiles_per_wave = tiles_per_wave;
  // yv == null: `g` already holds the materialised dy (dy_apply), the operand is loaded as is
  if (!yv) return conv_bwd_data_dispatch<P, AOP_ACT>(a, epi, C, Cin, Cout, KH, KW, stride, pad, Hx, Wx, Hy, Wy, stream);
  return conv_bwd_data_dispatch<P, AOP_DY>(a, epi, C, Cin, Cout, KH, KW, stride, pad, Hx, Wx, Hy, Wy, stream);
}

// forward: y = conv(pro(x)) − K, stats[c][co][2] += (Σy, Σy²) of the stored y; K = pivot[c][co] (null: 0).
// `_f32`: fp32 activations / packed weights.
FA_EXPORT int fa_conv_fwd(const uint16_t* x, const uint16_t* wpk, int64_t wpk_ld, const float* pscale,
                          const float* pshift, uint16_t* y, float* stats, int C, int Nb, int H, int W, int Cin,
                          int Cout, int KH, int KW, int stride, int pad, int Ho, int Wo, int ldk, int tiles_per_wave,
                          const float* pivot, const int* nimg, hipStream_t stream) {
  return conv_fwd<BF16>(x, wpk, wpk_ld, pscale, pshift, y, stats, C, Nb, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo,
                        ldk, tiles_per_wave, pivot, nimg, stream);
}
FA_EXPORT int fa_conv_fwd_f32(const float* x, const float* wpk, int64_t wpk_ld, const float* pscale,
                              const float* pshift, float* y, float* stats, int C, int Nb, int H, int W, int Cin,
                              int Cout, int KH, int KW, int stride, int pad, int Ho, int Wo, int ldk,
                              int tiles_per_wave, const float* pivot, const int* nimg, hipStream_t stream) {
  FA_F32_DISPATCH(prec, conv_fwd<PX>(x, wpk, wpk_ld, pscale, pshift, y, stats, C, Nb, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo,
                       ldk, tiles_per_wave, pivot, nimg, stream));
}

FA_EXPORT int fa_conv_fwd_bout_f32(const float* x, const float* wpk, int64_t wpk_ld, const float* pscale,
                                   const float* pshift, float* out, const float* s, const float* t, const float* pivot,
                                   const float* res, const float* rs, const float* rt, int C, int Nb, int H, int W,
                                   int Cin, int Cout, int ldk, int tiles_per_wave, const int* nimg, hipStream_t stream) {
  FA_F32_DISPATCH(prec, conv_fwd_bout<PX>(x, wpk, wpk_ld, pscale, pshift, out, s, t, pivot, res, rs, rt, C, Nb, H, W,
                                          Cin, Cout, ldk, tiles_per_wave, nimg, stream));
}

FA_EXPORT int fa_conv_fwd_pbout(const uint16_t* yp, const float* s, const float* t, const uint16_t* res,
                                const float* rs, const float* rt, uint16_t* bout, const uint16_t* wpk, int64_t wpk_ld,
                                uint16_t* y, float* stats, int C, int Nb, int H, int W, int Cin, int Cout, int ldk,
                                int tiles_per_wave, const float* pivot, const int* nimg, hipStream_t stream) {
  return conv_fwd_pbout<BF16>(yp, s, t, res, rs, rt, bout, wpk, wpk_ld, y, stats, C, Nb, H, W, Cin, Cout, ldk,
                              tiles_per_wave, pivot, nimg, stream);
}
FA_EXPORT int fa_conv_fwd_pbout_f32(const float* yp, const float* s, const float* t, const float* res,
                                    const float* rs, const float* rt, float* bout, const float* wpk, int64_t wpk_ld,
                                    float* y, float* stats, int C, int Nb, int H, int W, int Cin, int Cout, int ldk,
                                    int tiles_per_wave, const float* pivot, const int* nimg, hipStream_t stream) {
  FA_F32_DISPATCH(prec, conv_fwd_pbout<PX>(yp, s, t, res, rs, rt, bout, wpk, wpk_ld, y, stats, C, Nb, H, W, Cin, Cout,
                                           ldk, tiles_per_wave, pivot, nimg, stream));
}

// backward-data: dx = convᵀ(α·g + β·y + γ) with epilogue
//   epi 1 (STORE): out = dx
//   epi 2 (MASK) : out = g' = dx·[e_x·e_s + e_t > 0];  stats (Σg', Σg'·e_x)
//   epi 3 (BLOCK): out = g' = (dx + e_add)·[e_x > 0];   stats (Σg', Σg'·e_y1, Σg'·e_y2)
FA_EXPORT int fa_conv_bwd_data(const uint16_t* g, const uint16_t* yv, const float* alpha, const float* beta,
                               const float* gamma, const uint16_t* wpk_b, int64_t wpk_ld, uint16_t* dx, int epi,
                               const uint16_t* e_x, const float* e_s, const float* e_t, const uint16_t* e_add,
                               const uint16_t* e_y1, const uint16_t* e_y2, float* stats, int C, int Nb, int Hy,
                               int Wy, int Cout, int Cin, int KH, int KW, int stride, int pad, int Hx, int Wx,
                               int ldk2, int tiles_per_wave, const int* nimg, hipStream_t stream) {
  return conv_bwd_data<BF16>(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, epi, e_x, e_s, e_t, e_add, e_y1, e_y2,
                             stats, C, Nb, Hy, Wy, Cout, Cin, KH, KW, stride, pad, Hx, Wx, ldk2, tiles_per_wave, nimg,
                             stream);
}
FA_EXPORT int fa_conv_bwd_data_f32(const float* g, const float* yv, const float* alpha, const float* beta,
                                   const float* gamma, const float* wpk_b, int64_t wpk_ld, float* dx, int epi,
                                   const float* e_x, const float* e_s, const float* e_t, const float* e_add,
                                   const float* e_y1, const float* e_y2, float* stats, int C, int Nb, int Hy,
                                   int Wy, int Cout, int Cin, int KH, int KW, int stride, int pad, int Hx, int Wx,
                                   int ldk2, int tiles_per_wave, const int* nimg, hipStream_t stream) {
  FA_F32_DISPATCH(prec, conv_bwd_data<PX>(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, epi, e_x, e_s, e_t, e_add, e_y1, e_y2,
                            stats, C, Nb, Hy, Wy, Cout, Cin, KH, KW, stride, pad, Hx, Wx, ldk2, tiles_per_wave, nimg,
                            stream));
}

// fp32 matrix-core mode of every `_f32` conv launcher (prec.h): 0 exact v_mfma_f32_16x16x4_f32,
// 1 split-bf16 (three v_mfma_f32_16x16x32_bf16 per fragment). Returns the previous mode.
FA_EXPORT int fa_set_f32_mma_mode(int mode) {
  const int prev = prec::f32_mma_mode();
  prec::f32_mma_mode() = mode ? 1 : 0;
  return prev;
}
