// Transformer kernels for the client-batched DistilBERT / ViT path:
//   * fused (residual + dropout +) LayerNorm forward / backward with per-client gamma/beta
//   * exact-erf GELU forward / backward
//   * short-sequence attention (S <= 256, head dim 64) forward and backward on
//     v_mfma_f32_16x16x32_bf16, K/V (or Q/dO) tiles staged in LDS, exact row softmax in
//     registers, attention-probability dropout from a counter hash (regenerated in backward).
//
// Layouts: token-major activations [rows = clients·batch·seq][d] in bf16 (the output of the
// per-client batched GEMMs), heads interleaved along d (head h = columns 64h..64h+63).
// MFMA 16x16x32 bf16 operand maps (gfx950): lane l holds A[row l&15][k 8(l>>4)..+7],
// B[k 8(l>>4)..+7][col l&15]; C/D: col = l&15, row = 4(l>>4) + reg.
#include "common.h"
#include <cstdlib>
#include <type_traits>
#include "dropout.h"
#include "detacc.h"

FA_DET_EXPORT(transformer)

typedef __bf16 bf16x8_mf __attribute__((ext_vector_type(8)));

namespace {


__device__ __forceinline__ void unpack8(const uint4 u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f32_to_bf16(f[2 * i]) | ((uint32_t)f32_to_bf16(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ------------------------------------------------------------------------------------------
// LayerNorm forward: x = bf16(res + dropout(h)) (res/dropout optional), y = LN(x)*g + b.
// One wave per row, NV chunks of 8 columns per lane (d <= NV*512, d % 8 == 0).
// ------------------------------------------------------------------------------------------
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const uint16_t* __restrict__ h, const uint16_t* __restrict__ res,
                                                     int R, int d, int rows_per_client, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, uint32_t thr,
                                                     float dscale, uint32_t seed, uint16_t* __restrict__ y,
                                                     uint16_t* __restrict__ xsum, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out,
                                                     const uint32_t* __restrict__ seedp, int64_t gcs) {
  if (seedp) seed += *seedp * 1000003u;   // device step counter (graph-captured steps)
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int c = row / rows_per_client;
  float x[NV][8];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 8;
    if (col < d) {
      unpack8(*(const uint4*)(h + (size_t)row * d + col), x[v]);
      if (thr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[v][j] = fa_drop::keep(seed, (uint32_t)row, (uint32_t)(col + j), thr) ? x[v][j] * dscale : 0.f;
      }
      if (res) {
        float r8[8];
        unpack8(*(const uint4*)(res + (size_t)row * d + col), r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[v][j] += r8[j];
      }
      if (res || thr) {  // the sum is materialised in bf16 (as a bf16 torch graph would): round first
        const uint4 p = pack8(x[v]);
        unpack8(p, x[v]);
        if (xsum) *(uint4*)(xsum + (size_t)row * d + col) = p;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[v][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[v][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 8;
    if (col < d) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = x[v][j] - mean;
        q += t * t;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)d + eps);
  const float* g = gamma + (int64_t)c * gcs;
  const float* b = beta + (int64_t)c * gcs;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 8;
    if (col < d) {
      float o[8];
      const float4 g0 = *(const float4*)(g + col), g1 = *(const float4*)(g + col + 4);
      const float4 b0 = *(const float4*)(b + col), b1 = *(const float4*)(b + col + 4);
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (x[v][j] - mean) * rstd * gg[j] + bb[j];
      *(uint4*)(y + (size_t)row * d + col) = pack8(o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// LayerNorm backward. grid (blocks_per_client, C); each wave walks rows of one client and keeps
// the d-wide dgamma/dbeta partial sums in registers; the 4 waves combine in LDS and one fp32
// atomic per column and block lands in dgamma/dbeta [C, d].
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     int rows_per_client, int d, const float* __restrict__ gamma,
                                                     uint16_t* __restrict__ dx, uint16_t* __restrict__ dh,
                                                     uint32_t thr, float dscale, uint32_t seed,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                     const uint32_t* __restrict__ seedp, int64_t gcs, int64_t dgcs,
                                                     const uint16_t* __restrict__ dadd) {
  if (seedp) seed += *seedp * 1000003u;
  extern __shared__ float red[];  // [4][2][d]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.y;
  const float* g = gamma + (int64_t)c * gcs;
  float ag[NV][8], ab[NV][8];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) ag[v][j] = ab[v][j] = 0.f;
  for (int r = blockIdx.x * 4 + wid; r < rows_per_client; r += gridDim.x * 4) {
    const size_t row = (size_t)c * rows_per_client + r;
    const float mu = mean[row], rs = rstd[row];
    float xh[NV][8], gy[NV][8], gd[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int col = (v * 64 + lane) * 8;
      if (col < d) {
        float xv[8];
        unpack8(*(const uint4*)(x + row * d + col), xv);
        unpack8(*(const uint4*)(dy + row * d + col), gy[v]);
        const float4 g0 = *(const float4*)(g + col), g1 = *(const float4*)(g + col + 4);
        const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[v][j] = (xv[j] - mu) * rs;
          gd[v][j] = gy[v][j] * gg[j];
          s1 += gd[v][j];
          s2 += gd[v][j] * xh[v][j];
          ag[v][j] += gy[v][j] * xh[v][j];
          ab[v][j] += gy[v][j];
        }
      }
    }
    s1 = wave_sum(s1) / (float)d;
    s2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int col = (v * 64 + lane) * 8;
      if (col < d) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (gd[v][j] - s1 - xh[v][j] * s2);
        if (dx) *(uint4*)(dx + row * d + col) = pack8(o);
        if (dh) {
          if (thr) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
              o[j] = fa_drop::keep(seed, (uint32_t)row, (uint32_t)(col + j), thr) ? o[j] * dscale : 0.f;
          }
          if (dadd) {   // the other consumer's gradient of the LN input (pre-LN residual stream)
            float a8[8];
            unpack8(*(const uint4*)(dadd + row * d + col), a8);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += a8[j];
          }
          *(uint4*)(dh + row * d + col) = pack8(o);
        }
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 8;
    if (col < d) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
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
    fa_acc_add(dgamma + (int64_t)c * dgcs + i, sg);
    fa_acc_add(dbeta + (int64_t)c * dgcs + i, sb);
  }
}

// ------------------------------------------------------------------------------------------
// GELU (erf form, as torch.nn.functional.gelu's default), 8 bf16 per thread
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                       int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    unpack8(*(const uint4*)(x + i * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.5f * v[j] * (1.f + erff(v[j] * 0.70710678118654752f));
    *(uint4*)(y + i * 8) = pack8(v);
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ gy,
                                                       uint16_t* __restrict__ gx, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8], g[8];
    unpack8(*(const uint4*)(x + i * 8), v);
    unpack8(*(const uint4*)(gy + i * 8), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cdf = 0.5f * (1.f + erff(v[j] * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * v[j] * v[j]);
      g[j] = g[j] * (cdf + v[j] * pdf);
    }
    *(uint4*)(gx + i * 8) = pack8(g);
  }
}

// ------------------------------------------------------------------------------------------
// Attention. q/k/v/o: token-major bf16 with row strides ld*, head h at column 64h.
// lse2: [CB, H, S] fp32, log2-domain log-sum-exp of the scaled scores (+inf for empty rows).
// ------------------------------------------------------------------------------------------
constexpr float kLog2e = 1.4426950408889634f;
constexpr int KST = 72;  // LDS row stride (bf16) of [rows][64] tiles: 144 B, 16-B aligned

__device__ __forceinline__ bf16x8_mf lds8(const uint16_t* p) { return __builtin_bit_cast(bf16x8_mf, *(const uint4*)p); }
__device__ __forceinline__ bf16x8_mf g8(const uint16_t* p) { return __builtin_bit_cast(bf16x8_mf, *(const uint4*)p); }
__device__ __forceinline__ bf16x8_mf zero8() { return __builtin_bit_cast(bf16x8_mf, make_uint4(0, 0, 0, 0)); }

typedef short v4i16_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16_t lds_v4i16_t;

// MFMA operand fragment "8 consecutive rows row0 + 8·(lane>>4) + j of column col0 + (lane & 15)" of a
// ROW-MAJOR LDS tile (pitch ld elements) via gfx950's transposing LDS read ds_read_b64_tr_b16: the
// k-strided operands of P·V, dS·K, Pᵀ·dO and dSᵀ·Q come straight from the row-major K/V/Q/dO
// images — no transposed copies staged with 2-byte LDS stores.
__device__ __forceinline__ bf16x8_mf tr8(const uint16_t* tile, int ld, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const uint16_t* a0 = tile + (row0 + 8 * g + q) * ld + col0 + 4 * p;
  const v4i16_t r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(a0));
  const v4i16_t r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(a0 + 4 * ld));
  union {
    short s[8];
    bf16x8_mf b;
  } u;
  u.s[0] = r0[0]; u.s[1] = r0[1]; u.s[2] = r0[2]; u.s[3] = r0[3];
  u.s[4] = r1[0]; u.s[5] = r1[1]; u.s[6] = r1[2]; u.s[7] = r1[3];
  return u.b;
}

// stage rows [r0, r0+nrows) of one head's 64 columns into LDS, row-major [nrows][KST]
__device__ __forceinline__ void stage_rows(uint16_t* dst, const uint16_t* src, int ld, int r0, int nrows, int S) {
  for (int i = threadIdx.x; i < nrows * 8; i += blockDim.x) {
    const int r = i >> 3, ch = i & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < S) v = *(const uint4*)(src + (size_t)(r0 + r) * ld + ch * 8);
    *(uint4*)(dst + r * KST + ch * 8) = v;
  }
}
// Forward: grid (H, CB), 4 waves. K and V of the (sequence, head) are staged ONCE (row-major) and the
// workgroup loops over 64-query chunks; wave w owns query rows q0 + 16w + [0,16). Whole key range in
// LDS (SP = padded S), exact softmax over the row in registers.
template <int SP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const uint16_t* __restrict__ q, int ldq,
                                                       const uint16_t* __restrict__ k, int ldk,
                                                       const uint16_t* __restrict__ v, int ldv,
                                                       uint16_t* __restrict__ o, int ldo,
                                                       const uint8_t* __restrict__ kmask, float* __restrict__ lse2,
                                                       int S, int H, float scale, uint32_t thr, float dscale,
                                                       uint32_t seed, const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  constexpr int NB = SP / 16;
  constexpr int VST = SP + 8;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[SP * KST];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[SP * KST];
  __shared__ __attribute__((aligned(16))) uint16_t Ps[4 * 16 * VST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = blockIdx.x, cb = blockIdx.y;
  const size_t tok0 = (size_t)cb * S;
  stage_rows(Ks, k + tok0 * ldk + h * 64, ldk, 0, SP, S);
  stage_rows(Vs, v + tok0 * ldv + h * 64, ldv, 0, SP, S);
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  uint16_t* P = Ps + w * 16 * VST;
  bool kval[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int key = nb * 16 + (lane & 15);
    kval[nb] = key < S && (kmask == nullptr || kmask[tok0 + key] != 0);
  }
  for (int q0 = 0; q0 < S; q0 += 64) {
    const int qr = q0 + w * 16 + (lane & 15);  // A-operand row of this lane
    // wave-uniform skips of padding-only work (query waves past S, 16-key blocks / 32-key halves past S):
    // their scores are −∞ and probabilities 0, so every result bit is unchanged
    const bool wrows = q0 + w * 16 < S;
    bf16x8_mf qf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
      qf[t] = qr < S ? g8(q + (tok0 + qr) * ldq + h * 64 + 32 * t + 8 * (lane >> 4)) : zero8();
    __syncthreads();   // staging done (first chunk) / previous chunk's P reads done
    f32x4 sc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (wrows && nb * 16 < S) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              qf[t], lds8(Ks + (nb * 16 + (lane & 15)) * KST + 32 * t + 8 * (lane >> 4)), acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = kval[nb] ? acc[r] * c2 : -INFINITY;
      sc[nb] = acc;
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
    const int qbase = q0 + w * 16 + 4 * (lane >> 4);  // C-layout query row of reg 0
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int key = nb * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = m[r] == -INFINITY ? 0.f : exp2f(sc[nb][r] - m[r]);
        l[r] += p;
        if (thr) p = fa_drop::keep(seed, bh * 65536u + (uint32_t)(qbase + r), (uint32_t)key, thr) ? p * dscale : 0.f;
        P[(4 * (lane >> 4) + r) * VST + key] = f32_to_bf16(p);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) l[r] += __shfl_xor(l[r], off, 64);
    }
    __syncthreads();
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < SP / 32; ++kt)
        if (wrows && kt * 32 < S)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(P + (lane & 15) * VST + kt * 32 + 8 * (lane >> 4)),
                                                         tr8(Vs, KST, kt * 32, db * 16, lane), acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qrow = qbase + r;
        if (qrow < S) {
          const float val = l[r] > 0.f ? acc[r] / l[r] : 0.f;
          o[(tok0 + qrow) * ldo + h * 64 + db * 16 + (lane & 15)] = f32_to_bf16(val);
        }
      }
    }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qrow = qbase + r;
        if (qrow < S) lse2[((size_t)cb * H + h) * S + qrow] = l[r] > 0.f ? m[r] + log2f(l[r]) : INFINITY;
      }
    }
  }
}

// Forward with the probabilities kept in registers: the scores are computed transposed, Sᵀ = K·Qᵀ
// (mfma_16x16x32: A = K rows, B = Q rows), so a lane holds ONE query (its column) and keys 4g … 4g+3 of every
// 16-key block in its 4 accumulators. The softmax of a query is then an in-lane max / sum over its 4·NB scores
// plus two cross-group shuffles, and the bf16 probabilities of a block ARE the B operand of the 16×16×16 MFMA
// (B[k = 4g + j][col]) for Oᵀ = Vᵀ·Pᵀ — no LDS round trip for P. Vᵀ's A fragment (A[row = dim][k = 4g + j]) is one
// ds_read_b64_tr_b16 of the row-major V image (16-lane group g: rows 4g … 4g+3 of the key block). K and V of the
// (sequence, head) stay in LDS for all its query chunks; 64 KB at S ≤ 224, two workgroups per CU. Same
// results as attn_fwd_kernel up to the order of the fp32 sums (the backward kernels are shared).
template <int SP>
__global__ __launch_bounds__(256, 2) void attn_fwd_rp_kernel(const uint16_t* __restrict__ q, int ldq,
                                                          const uint16_t* __restrict__ k, int ldk,
                                                          const uint16_t* __restrict__ v, int ldv,
                                                          uint16_t* __restrict__ o, int ldo,
                                                          const uint8_t* __restrict__ kmask, float* __restrict__ lse2,
                                                          int S, int H, float scale, uint32_t thr, float dscale,
                                                          uint32_t seed, const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  constexpr int NB = SP / 16;
  static_assert(NB <= 16, "key-validity bits");
  __shared__ __attribute__((aligned(16))) uint16_t Ks[SP * KST];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[SP * KST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int h = blockIdx.x, cb = blockIdx.y;
  const size_t tok0 = (size_t)cb * S;
  stage_rows(Ks, k + tok0 * ldk + h * 64, ldk, 0, SP, S);
  stage_rows(Vs, v + tok0 * ldv + h * 64, ldv, 0, SP, S);
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  uint64_t kv = 0;   // bit 4·nb + r: key nb·16 + 4g + r exists and is not masked
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = nb * 16 + 4 * g + r;
      if (key < S && (kmask == nullptr || kmask[tok0 + key] != 0)) kv |= 1ull << (4 * nb + r);
    }
  // V^T fragment address of this lane inside a 16-key block (lane 4q + p of its group: row 4g + q, cols 4p..4p+3)
  const int vrow = 4 * g + (i16 >> 2), vcol = 4 * (i16 & 3);
  __syncthreads();
  for (int q0 = 0; q0 < S; q0 += 64) {
    const int qr = q0 + w * 16 + i16;          // this lane's query (the B / C column)
    const bool wrows = q0 + w * 16 < S;        // wave-uniform: whole 16-query tile past S → skip its MFMAs
    bf16x8_mf qf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) qf[t] = qr < S ? g8(q + (tok0 + qr) * ldq + h * 64 + 32 * t + 8 * g) : zero8();
    f32x4 sc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (wrows && nb * 16 < S) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(Ks + (nb * 16 + i16) * KST + 32 * t + 8 * g), qf[t], acc,
                                                         0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = ((kv >> (4 * nb + r)) & 1) ? acc[r] * c2 : -INFINITY;
      sc[nb] = acc;
    }
    float m = -INFINITY;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, sc[nb][r]);
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
    v4i16_t pt[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = m == -INFINITY ? 0.f : exp2f(sc[nb][r] - m);
        l += p;
        if (thr) p = fa_drop::keep(seed, bh * 65536u + (uint32_t)qr, (uint32_t)(nb * 16 + 4 * g + r), thr) ? p * dscale : 0.f;
        pt[nb][r] = (short)f32_to_bf16(p);
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    f32x4 oacc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if (wrows && nb * 16 < S) {   // wave-uniform (the transposing read needs every lane active)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const v4i16_t va =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(Vs + (nb * 16 + vrow) * KST + db * 16 + vcol));
          oacc[db] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pt[nb], oacc[db], 0, 0, 0);
        }
      }
    }
    if (qr < S) {
      const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        uint2 ov;
        ov.x = (uint32_t)f32_to_bf16(oacc[db][0] * inv) | ((uint32_t)f32_to_bf16(oacc[db][1] * inv) << 16);
        ov.y = (uint32_t)f32_to_bf16(oacc[db][2] * inv) | ((uint32_t)f32_to_bf16(oacc[db][3] * inv) << 16);
        *reinterpret_cast<uint2*>(o + (tok0 + qr) * ldo + h * 64 + db * 16 + 4 * g) = ov;
      }
      if (g == 0) lse2[((size_t)cb * H + h) * S + qr] = l > 0.f ? m + log2f(l) : INFINITY;
    }
  }
}

// D[cb,h,q] = Σ_dim dO·O  (one thread per (token, head))
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const uint16_t* __restrict__ o, int ldo,
                                                            const uint16_t* __restrict__ dout, int lddo,
                                                            float* __restrict__ D, int CBS, int S, int H) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)CBS * H) return;
  const int h = (int)(i % H);
  const int64_t tok = i / H;
  float s = 0.f;
#pragma unroll
  for (int ch = 0; ch < 8; ++ch) {
    float a[8], b[8];
    unpack8(*(const uint4*)(o + tok * ldo + h * 64 + ch * 8), a);
    unpack8(*(const uint4*)(dout + tok * lddo + h * 64 + ch * 8), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * b[j];
  }
  const int64_t cb = tok / S, qq = tok % S;
  D[(cb * H + h) * S + qq] = s;
}

// dQ: grid (ceil(S/64), H, CB); wave w owns 16 query rows, loops over key chunks of 64.
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const uint16_t* __restrict__ q, int ldq,
                                                          const uint16_t* __restrict__ k, int ldk,
                                                          const uint16_t* __restrict__ v, int ldv,
                                                          const uint16_t* __restrict__ dout, int lddo,
                                                          const uint8_t* __restrict__ kmask,
                                                          const float* __restrict__ lse2, const float* __restrict__ D,
                                                          uint16_t* __restrict__ dq, int lddq, int S, int H,
                                                          float scale, uint32_t thr, float dscale, uint32_t seed,
                                                          const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[64 * KST];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[64 * KST];
  __shared__ __attribute__((aligned(16))) uint16_t dSs[4 * 16 * KST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const size_t bhS = ((size_t)cb * H + h) * S;
  const int qr = blockIdx.x * 64 + w * 16 + (lane & 15);
  const bool wrows = blockIdx.x * 64 + w * 16 < S;   // wave-uniform padding skips, as in the forward
  bf16x8_mf qf[2], df[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    qf[t] = qr < S ? g8(q + (tok0 + qr) * ldq + h * 64 + 32 * t + 8 * (lane >> 4)) : zero8();
    df[t] = qr < S ? g8(dout + (tok0 + qr) * lddo + h * 64 + 32 * t + 8 * (lane >> 4)) : zero8();
  }
  const int qbase = blockIdx.x * 64 + w * 16 + 4 * (lane >> 4);
  float L[4], Dr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qq = qbase + r;
    L[r] = qq < S ? lse2[bhS + qq] : INFINITY;
    Dr[r] = qq < S ? D[bhS + qq] : 0.f;
  }
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  uint16_t* dS = dSs + w * 16 * KST;
  f32x4 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) acc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < S; k0 += 64) {
    __syncthreads();
    stage_rows(Ks, k + tok0 * ldk + h * 64, ldk, k0, 64, S);
    stage_rows(Vs, v + tok0 * ldv + h * 64, ldv, k0, 64, S);
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      if (wrows && k0 + nb * 16 < S) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int off = (nb * 16 + (lane & 15)) * KST + 32 * t + 8 * (lane >> 4);
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[t], lds8(Ks + off), s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(df[t], lds8(Vs + off), dp, 0, 0, 0);
        }
      }
      const int key = k0 + nb * 16 + (lane & 15);
      const bool valid = key < S && (kmask == nullptr || kmask[tok0 + key] != 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = valid ? exp2f(s[r] * c2 - L[r]) : 0.f;
        float g = dp[r];
        if (thr) g = fa_drop::keep(seed, bh * 65536u + (uint32_t)(qbase + r), (uint32_t)key, thr) ? g * dscale : 0.f;
        dS[(4 * (lane >> 4) + r) * KST + nb * 16 + (lane & 15)] = f32_to_bf16(p * (g - Dr[r]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
        if (wrows && k0 + kt * 32 < S)
          acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(dS + (lane & 15) * KST + kt * 32 + 8 * (lane >> 4)),
                                                            tr8(Ks, KST, kt * 32, db * 16, lane), acc[db], 0, 0, 0);
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qq = qbase + r;
      if (qq < S) dq[(tok0 + qq) * lddq + h * 64 + db * 16 + (lane & 15)] = f32_to_bf16(acc[db][r] * scale);
    }
}

// dK, dV: grid (ceil(S/64), H, CB); wave w owns 16 keys, loops over query chunks of 64.
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(const uint16_t* __restrict__ q, int ldq,
                                                           const uint16_t* __restrict__ k, int ldk,
                                                           const uint16_t* __restrict__ v, int ldv,
                                                           const uint16_t* __restrict__ dout, int lddo,
                                                           const uint8_t* __restrict__ kmask,
                                                           const float* __restrict__ lse2, const float* __restrict__ D,
                                                           uint16_t* __restrict__ dk, int lddk,
                                                           uint16_t* __restrict__ dv, int lddv, int S, int H,
                                                           float scale, uint32_t thr, float dscale, uint32_t seed,
                                                           const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  __shared__ __attribute__((aligned(16))) uint16_t Qs[64 * KST];
  __shared__ __attribute__((aligned(16))) uint16_t dOs[64 * KST];
  __shared__ __attribute__((aligned(16))) uint16_t Pst[4 * 16 * KST];
  __shared__ __attribute__((aligned(16))) uint16_t dSt[4 * 16 * KST];
  __shared__ float Ls[64], Dsh[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const size_t bhS = ((size_t)cb * H + h) * S;
  const int kr = blockIdx.x * 64 + w * 16 + (lane & 15);
  const bool wkeys = blockIdx.x * 64 + w * 16 < S;   // wave-uniform padding skips, as in the forward
  bf16x8_mf kf[2], vf[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    kf[t] = kr < S ? g8(k + (tok0 + kr) * ldk + h * 64 + 32 * t + 8 * (lane >> 4)) : zero8();
    vf[t] = kr < S ? g8(v + (tok0 + kr) * ldv + h * 64 + 32 * t + 8 * (lane >> 4)) : zero8();
  }
  const int kbase = blockIdx.x * 64 + w * 16 + 4 * (lane >> 4);  // C-layout key of reg 0
  bool kvalid[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kk = kbase + r;
    kvalid[r] = kk < S && (kmask == nullptr || kmask[tok0 + kk] != 0);
  }
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  uint16_t* Pw = Pst + w * 16 * KST;
  uint16_t* dSw = dSt + w * 16 * KST;
  f32x4 adk[4], adv[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) adk[db] = adv[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int q0 = 0; q0 < S; q0 += 64) {
    __syncthreads();
    stage_rows(Qs, q + tok0 * ldq + h * 64, ldq, q0, 64, S);
    stage_rows(dOs, dout + tok0 * lddo + h * 64, lddo, q0, 64, S);
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
          const int off = (nb * 16 + (lane & 15)) * KST + 32 * t + 8 * (lane >> 4);
          st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t], lds8(Qs + off), st, 0, 0, 0);
          dpt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[t], lds8(dOs + off), dpt, 0, 0, 0);
        }
      }
      const int ql = nb * 16 + (lane & 15);
      const int qq = q0 + ql;
      const float Lq = Ls[ql], Dq = Dsh[ql];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = kvalid[r] && qq < S;
        const float p = valid ? exp2f(st[r] * c2 - Lq) : 0.f;
        float pd = p, g = dpt[r];
        if (thr) {
          const bool kp = fa_drop::keep(seed, bh * 65536u + (uint32_t)qq, (uint32_t)(kbase + r), thr);
          pd = kp ? p * dscale : 0.f;
          g = kp ? g * dscale : 0.f;
        }
        Pw[(4 * (lane >> 4) + r) * KST + ql] = f32_to_bf16(pd);
        dSw[(4 * (lane >> 4) + r) * KST + ql] = f32_to_bf16(p * (g - Dq));
      }
    }
    __syncthreads();
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (!wkeys || q0 + kt * 32 >= S) continue;
        const int ao = (lane & 15) * KST + kt * 32 + 8 * (lane >> 4);
        adv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(Pw + ao), tr8(dOs, KST, kt * 32, db * 16, lane),
                                                          adv[db], 0, 0, 0);
        adk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(dSw + ao), tr8(Qs, KST, kt * 32, db * 16, lane),
                                                          adk[db], 0, 0, 0);
      }
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kk = kbase + r;
      if (kk < S) {
        dk[(tok0 + kk) * lddk + h * 64 + db * 16 + (lane & 15)] = f32_to_bf16(adk[db][r] * scale);
        dv[(tok0 + kk) * lddv + h * 64 + db * 16 + (lane & 15)] = f32_to_bf16(adv[db][r]);
      }
    }
}

// Backward with the probabilities in registers (the orientation trick of attn_fwd_rp_kernel).
// dQ: scores and dP transposed (Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ: lane = one query, keys 4g … 4g+3 of a 16-key block), so
// dSᵀ = Pᵀ ∘ (dPᵀ − D) is the B operand of dQᵀ = Kᵀ·dSᵀ (16×16×16; Kᵀ by a transposing read) — no dS staging.
template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_dq_rp_kernel(const uint16_t* __restrict__ q, int ldq,
                                                             const uint16_t* __restrict__ k, int ldk,
                                                             const uint16_t* __restrict__ v, int ldv,
                                                             const uint16_t* __restrict__ dout, int lddo,
                                                             const uint8_t* __restrict__ kmask,
                                                             const float* __restrict__ lse2, const float* __restrict__ D,
                                                             uint16_t* __restrict__ dq, int lddq, int S, int H,
                                                             float scale, uint32_t thr, float dscale, uint32_t seed,
                                                             const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[CH * KST];   // CH keys at a time (CH ≥ S: staged once)
  __shared__ __attribute__((aligned(16))) uint16_t Vs[CH * KST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const size_t bhS = ((size_t)cb * H + h) * S;
  const int qr = blockIdx.x * 64 + w * 16 + i16;     // this lane's query
  const bool wrows = blockIdx.x * 64 + w * 16 < S;   // wave-uniform
  bf16x8_mf qf[2], df[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    qf[t] = qr < S ? g8(q + (tok0 + qr) * ldq + h * 64 + 32 * t + 8 * g) : zero8();
    df[t] = qr < S ? g8(dout + (tok0 + qr) * lddo + h * 64 + 32 * t + 8 * g) : zero8();
  }
  const float L = qr < S ? lse2[bhS + qr] : INFINITY;
  const float Dq = qr < S ? D[bhS + qr] : 0.f;
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  const int trow = 4 * g + (i16 >> 2), tcol = 4 * (i16 & 3);   // transposing-read address of this lane
  f32x4 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) acc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < S; k0 += CH) {
    __syncthreads();
    stage_rows(Ks, k + tok0 * ldk + h * 64, ldk, k0, CH, S);
    stage_rows(Vs, v + tok0 * ldv + h * 64, ldv, k0, CH, S);
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < CH / 16; ++nb) {
      if (!wrows || k0 + nb * 16 >= S) continue;   // wave-uniform
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int off = (nb * 16 + i16) * KST + 32 * t + 8 * g;
        st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(Ks + off), qf[t], st, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(Vs + off), df[t], dpt, 0, 0, 0);
      }
      v4i16_t ds;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + nb * 16 + 4 * g + r;
        const bool valid = key < S && (kmask == nullptr || kmask[tok0 + key] != 0);
        const float p = valid ? exp2f(st[r] * c2 - L) : 0.f;
        float gg = dpt[r];
        if (thr) gg = fa_drop::keep(seed, bh * 65536u + (uint32_t)qr, (uint32_t)key, thr) ? gg * dscale : 0.f;
        ds[r] = (short)f32_to_bf16(p * (gg - Dq));
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const v4i16_t ka =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(Ks + (nb * 16 + trow) * KST + db * 16 + tcol));
        acc[db] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, ds, acc[db], 0, 0, 0);
      }
    }
  }
  if (qr < S) {
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      uint2 ov;
      ov.x = (uint32_t)f32_to_bf16(acc[db][0] * scale) | ((uint32_t)f32_to_bf16(acc[db][1] * scale) << 16);
      ov.y = (uint32_t)f32_to_bf16(acc[db][2] * scale) | ((uint32_t)f32_to_bf16(acc[db][3] * scale) << 16);
      *reinterpret_cast<uint2*>(dq + (tok0 + qr) * lddq + h * 64 + db * 16 + 4 * g) = ov;
    }
  }
}

// dK, dV: scores in the natural orientation (S = Q·Kᵀ, dP = dO·Vᵀ: lane = one key, queries 4g … 4g+3 of a
// 16-query block), so P and dS = P ∘ (dP − D) are the B operands of dVᵀ = dOᵀ·P and dKᵀ = Qᵀ·dS (16×16×16; dOᵀ and
// Qᵀ by transposing reads of the staged row-major tiles) — no P / dS staging.
template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_dkv_rp_kernel(const uint16_t* __restrict__ q, int ldq,
                                                              const uint16_t* __restrict__ k, int ldk,
                                                              const uint16_t* __restrict__ v, int ldv,
                                                              const uint16_t* __restrict__ dout, int lddo,
                                                              const uint8_t* __restrict__ kmask,
                                                              const float* __restrict__ lse2,
                                                              const float* __restrict__ D, uint16_t* __restrict__ dk,
                                                              int lddk, uint16_t* __restrict__ dv, int lddv, int S,
                                                              int H, float scale, uint32_t thr, float dscale,
                                                              uint32_t seed, const uint32_t* __restrict__ seedp) {
  if (seedp) seed += *seedp * 1000003u;
  __shared__ __attribute__((aligned(16))) uint16_t Qs[CH * KST];   // CH queries at a time (CH ≥ S: staged once)
  __shared__ __attribute__((aligned(16))) uint16_t dOs[CH * KST];
  __shared__ __attribute__((aligned(16))) float Ls[CH], Dsh[CH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int h = blockIdx.y, cb = blockIdx.z;
  const size_t tok0 = (size_t)cb * S;
  const size_t bhS = ((size_t)cb * H + h) * S;
  const int kr = blockIdx.x * 64 + w * 16 + i16;     // this lane's key
  const bool wkeys = blockIdx.x * 64 + w * 16 < S;   // wave-uniform
  bf16x8_mf kf[2], vf[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    kf[t] = kr < S ? g8(k + (tok0 + kr) * ldk + h * 64 + 32 * t + 8 * g) : zero8();
    vf[t] = kr < S ? g8(v + (tok0 + kr) * ldv + h * 64 + 32 * t + 8 * g) : zero8();
  }
  const bool kvalid = kr < S && (kmask == nullptr || kmask[tok0 + kr] != 0);
  const float c2 = scale * kLog2e;
  const uint32_t bh = (uint32_t)(cb * H + h);
  const int trow = 4 * g + (i16 >> 2), tcol = 4 * (i16 & 3);
  f32x4 adk[4], adv[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) adk[db] = adv[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int q0 = 0; q0 < S; q0 += CH) {
    __syncthreads();
    stage_rows(Qs, q + tok0 * ldq + h * 64, ldq, q0, CH, S);
    stage_rows(dOs, dout + tok0 * lddo + h * 64, lddo, q0, CH, S);
    for (int i = threadIdx.x; i < CH; i += 256) {
      Ls[i] = q0 + i < S ? lse2[bhS + q0 + i] : INFINITY;
      Dsh[i] = q0 + i < S ? D[bhS + q0 + i] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < CH / 16; ++nb) {
      if (!wkeys || q0 + nb * 16 >= S) continue;   // wave-uniform
      f32x4 s_ = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int off = (nb * 16 + i16) * KST + 32 * t + 8 * g;
        s_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(Qs + off), kf[t], s_, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(dOs + off), vf[t], dp, 0, 0, 0);
      }
      const float4 Lq = *reinterpret_cast<const float4*>(Ls + nb * 16 + 4 * g);
      const float4 Dq = *reinterpret_cast<const float4*>(Dsh + nb * 16 + 4 * g);
      const float Lr[4] = {Lq.x, Lq.y, Lq.z, Lq.w}, Dr[4] = {Dq.x, Dq.y, Dq.z, Dq.w};
      v4i16_t pp, dss;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + nb * 16 + 4 * g + r;
        const bool valid = kvalid && qq < S;
        const float p = valid ? exp2f(s_[r] * c2 - Lr[r]) : 0.f;
        float pd = p, gg = dp[r];
        if (thr) {
          const bool kp = fa_drop::keep(seed, bh * 65536u + (uint32_t)qq, (uint32_t)kr, thr);
          pd = kp ? p * dscale : 0.f;
          gg = kp ? gg * dscale : 0.f;
        }
        pp[r] = (short)f32_to_bf16(pd);
        dss[r] = (short)f32_to_bf16(p * (gg - Dr[r]));
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int ao = (nb * 16 + trow) * KST + db * 16 + tcol;
        const v4i16_t oa = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(dOs + ao));
        const v4i16_t qa = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(Qs + ao));
        adv[db] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(oa, pp, adv[db], 0, 0, 0);
        adk[db] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(qa, dss, adk[db], 0, 0, 0);
      }
    }
  }
  if (kr < S) {
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      uint2 kv2, vv2;
      kv2.x = (uint32_t)f32_to_bf16(adk[db][0] * scale) | ((uint32_t)f32_to_bf16(adk[db][1] * scale) << 16);
      kv2.y = (uint32_t)f32_to_bf16(adk[db][2] * scale) | ((uint32_t)f32_to_bf16(adk[db][3] * scale) << 16);
      vv2.x = (uint32_t)f32_to_bf16(adv[db][0]) | ((uint32_t)f32_to_bf16(adv[db][1]) << 16);
      vv2.y = (uint32_t)f32_to_bf16(adv[db][2]) | ((uint32_t)f32_to_bf16(adv[db][3]) << 16);
      *reinterpret_cast<uint2*>(dk + (tok0 + kr) * lddk + h * 64 + db * 16 + 4 * g) = kv2;
      *reinterpret_cast<uint2*>(dv + (tok0 + kr) * lddv + h * 64 + db * 16 + 4 * g) = vv2;
    }
  }
}

template <int NV>
int launch_ln_fwd(const uint16_t* h, const uint16_t* res, int R, int d, int rpc, const float* g, const float* b,
                  float eps, uint32_t thr, float dscale, uint32_t seed, const uint32_t* seedp, uint16_t* y,
                  uint16_t* xsum, float* mean,
                  float* rstd, int64_t gcs, hipStream_t st) {
  hipLaunchKernelGGL(ln_fwd_kernel<NV>, dim3((R + 3) / 4), dim3(256), 0, st, h, res, R, d, rpc, g, b, eps, thr,
                     dscale, seed, y, xsum, mean, rstd, seedp, gcs);
  return (int)hipGetLastError();
}
template <int NV>
int launch_ln_bwd(const uint16_t* dy, const uint16_t* x, const float* mean, const float* rstd, int C, int rpc, int d,
                  const float* g, uint16_t* dx, uint16_t* dh, uint32_t thr, float dscale, uint32_t seed,
                  const uint32_t* seedp, float* dg,
                  float* db, int64_t gcs, int64_t dgcs, hipStream_t st, const uint16_t* dadd = nullptr) {
  int bpc = (rpc + 31) / 32;  // ≥8 rows per wave
  if (bpc < 1) bpc = 1;
  if (bpc > 1024) bpc = 1024;
  hipLaunchKernelGGL(ln_bwd_kernel<NV>, dim3(bpc, C), dim3(256), 8 * d * sizeof(float), st, dy, x, mean, rstd, rpc,
                     d, g, dx, dh, thr, dscale, seed, dg, db, seedp, gcs, dgcs, dadd);
  return (int)hipGetLastError();
}

template <int SP>
int launch_attn_fwd(const uint16_t* q, int ldq, const uint16_t* k, int ldk, const uint16_t* v, int ldv, uint16_t* o,
                    int ldo, const uint8_t* kmask, float* lse2, int CB, int S, int H, float scale, uint32_t thr,
                    float dscale, uint32_t seed, const uint32_t* seedp, hipStream_t st) {
  // FEDML_AMD_ATTN_RP=0: the LDS-staged-probability forward (A/B)
  static const bool rp = [] {
    const char* e = getenv("FEDML_AMD_ATTN_RP");
    return !(e && e[0] == '0');
  }();
  if (rp)
    hipLaunchKernelGGL(attn_fwd_rp_kernel<SP>, dim3(H, CB), dim3(256), 0, st, q, ldq, k, ldk, v, ldv, o,
                       ldo, kmask, lse2, S, H, scale, thr, dscale, seed, seedp);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<SP>, dim3(H, CB), dim3(256), 0, st, q, ldq, k, ldk, v, ldv, o,
                       ldo, kmask, lse2, S, H, scale, thr, dscale, seed, seedp);
  return (int)hipGetLastError();
}

}  // namespace

FA_EXPORT int fa_ln_fwd(const void* h, const void* res, int R, int d, int rows_per_client, const float* gamma,
                        const float* beta, float eps, uint32_t thr, float dscale, uint32_t seed, void* y, void* xsum,
                        float* mean, float* rstd, const uint32_t* seedp, int64_t gcs, hipStream_t stream) {
  if (d % 8 != 0 || d > 2048 || gcs % 4 != 0) return (int)hipErrorInvalidValue;
  auto H = (const uint16_t*)h;
  auto Rs = (const uint16_t*)res;
  auto Y = (uint16_t*)y;
  auto X = (uint16_t*)xsum;
  if (d <= 512) return launch_ln_fwd<1>(H, Rs, R, d, rows_per_client, gamma, beta, eps, thr, dscale, seed, seedp, Y, X, mean, rstd, gcs, stream);
  if (d <= 1024) return launch_ln_fwd<2>(H, Rs, R, d, rows_per_client, gamma, beta, eps, thr, dscale, seed, seedp, Y, X, mean, rstd, gcs, stream);
  return launch_ln_fwd<4>(H, Rs, R, d, rows_per_client, gamma, beta, eps, thr, dscale, seed, seedp, Y, X, mean, rstd, gcs, stream);
}

FA_EXPORT int fa_ln_bwd_add(const void* dy, const void* x, const float* mean, const float* rstd, int C,
                            int rows_per_client, int d, const float* gamma, void* dx, void* dh, uint32_t thr,
                            float dscale, uint32_t seed, float* dgamma, float* dbeta, const uint32_t* seedp,
                            int64_t gcs, int64_t dgcs, const void* dadd, hipStream_t stream);
FA_EXPORT int fa_ln_bwd(const void* dy, const void* x, const float* mean, const float* rstd, int C,
                        int rows_per_client, int d, const float* gamma, void* dx, void* dh, uint32_t thr, float dscale,
                        uint32_t seed, float* dgamma, float* dbeta, const uint32_t* seedp, int64_t gcs,
                        int64_t dgcs, hipStream_t stream) {
  return fa_ln_bwd_add(dy, x, mean, rstd, C, rows_per_client, d, gamma, dx, dh, thr, dscale, seed, dgamma, dbeta, seedp,
                       gcs, dgcs, nullptr, stream);
}
// dadd (optional, bf16 like dh): added to dh — the residual stream's other gradient (pre-LN)
FA_EXPORT int fa_ln_bwd_add(const void* dy, const void* x, const float* mean, const float* rstd, int C,
                            int rows_per_client, int d, const float* gamma, void* dx, void* dh, uint32_t thr,
                            float dscale, uint32_t seed, float* dgamma, float* dbeta, const uint32_t* seedp,
                            int64_t gcs, int64_t dgcs, const void* dadd, hipStream_t stream) {
  if (d % 8 != 0 || d > 2048 || gcs % 4 != 0) return (int)hipErrorInvalidValue;
  auto DY = (const uint16_t*)dy;
  auto X = (const uint16_t*)x;
  auto DX = (uint16_t*)dx;
  auto DH = (uint16_t*)dh;
  auto DA = (const uint16_t*)dadd;
  if (d <= 512) return launch_ln_bwd<1>(DY, X, mean, rstd, C, rows_per_client, d, gamma, DX, DH, thr, dscale, seed, seedp, dgamma, dbeta, gcs, dgcs, stream, DA);
  if (d <= 1024) return launch_ln_bwd<2>(DY, X, mean, rstd, C, rows_per_client, d, gamma, DX, DH, thr, dscale, seed, seedp, dgamma, dbeta, gcs, dgcs, stream, DA);
  return launch_ln_bwd<4>(DY, X, mean, rstd, C, rows_per_client, d, gamma, DX, DH, thr, dscale, seed, seedp, dgamma, dbeta, gcs, dgcs, stream, DA);
}

FA_EXPORT int fa_gelu_fwd(const void* x, void* y, int64_t n, hipStream_t stream) {
  if (n % 8 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(fa_grid(n / 8, 256, 8192)), dim3(256), 0, stream, (const uint16_t*)x,
                     (uint16_t*)y, n / 8);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_gelu_bwd(const void* x, const void* gy, void* gx, int64_t n, hipStream_t stream) {
  if (n % 8 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(fa_grid(n / 8, 256, 8192)), dim3(256), 0, stream, (const uint16_t*)x,
                     (const uint16_t*)gy, (uint16_t*)gx, n / 8);
  return (int)hipGetLastError();
}

FA_EXPORT int fa_attn_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                          const uint8_t* kmask, float* lse2, int CB, int S, int H, float scale, uint32_t thr,
                          float dscale, uint32_t seed, const uint32_t* seedp, hipStream_t stream) {
  auto Q = (const uint16_t*)q;
  auto K = (const uint16_t*)k;
  auto V = (const uint16_t*)v;
  auto O = (uint16_t*)o;
  if (S <= 0 || S > 256 || (ldq | ldk | ldv | ldo) % 8 != 0) return (int)hipErrorInvalidValue;
  if (S <= 64) return launch_attn_fwd<64>(Q, ldq, K, ldk, V, ldv, O, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, stream);
  if (S <= 128) return launch_attn_fwd<128>(Q, ldq, K, ldk, V, ldv, O, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, stream);
  if (S <= 160) return launch_attn_fwd<160>(Q, ldq, K, ldk, V, ldv, O, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, stream);
  if (S <= 192) return launch_attn_fwd<192>(Q, ldq, K, ldk, V, ldv, O, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, stream);
  if (S <= 224) return launch_attn_fwd<224>(Q, ldq, K, ldk, V, ldv, O, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, stream);
  return launch_attn_fwd<256>(Q, ldq, K, ldk, V, ldv, O, ldo, kmask, lse2, CB, S, H, scale, thr, dscale, seed, seedp, stream);
}

FA_EXPORT int fa_attn_bwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, const void* o,
                          int ldo, const void* dout, int lddo, const uint8_t* kmask, const float* lse2, float* Dbuf,
                          void* dq, int lddq, void* dk, int lddk, void* dv, int lddv, int CB, int S, int H,
                          float scale, uint32_t thr, float dscale, uint32_t seed, const uint32_t* seedp, hipStream_t stream) {
  if (S <= 0 || S > 4096 || (ldq | ldk | ldv | ldo | lddo | lddq | lddk | lddv) % 8 != 0)
    return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)CB * S * H;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const uint16_t*)o, ldo, (const uint16_t*)dout, lddo, Dbuf, CB * S, S, H);
  const dim3 grid((S + 63) / 64, H, CB);
  static const bool rp = [] {   // FEDML_AMD_ATTN_RP=0: the LDS-staged dS / P kernels (A/B)
    const char* e = getenv("FEDML_AMD_ATTN_RP");
    return !(e && e[0] == '0');
  }();
  auto Q = (const uint16_t*)q;
  auto K = (const uint16_t*)k;
  auto V = (const uint16_t*)v;
  auto DO = (const uint16_t*)dout;
  if (rp) {   // S ≤ 128: the whole sequence staged once per workgroup; longer: 64-row chunks (more workgroups per
             // CU — measured faster at S = 197, slower at 128; profiles/r6_attention_rp.txt)
    auto go = [&](auto sp) {
      constexpr int SP = decltype(sp)::value;
      hipLaunchKernelGGL(attn_bwd_dq_rp_kernel<SP>, grid, dim3(256), 0, stream, Q, ldq, K, ldk, V, ldv, DO, lddo,
                         kmask, lse2, Dbuf, (uint16_t*)dq, lddq, S, H, scale, thr, dscale, seed, seedp);
      hipLaunchKernelGGL(attn_bwd_dkv_rp_kernel<SP>, grid, dim3(256), 0, stream, Q, ldq, K, ldk, V, ldv, DO, lddo,
                         kmask, lse2, Dbuf, (uint16_t*)dk, lddk, (uint16_t*)dv, lddv, S, H, scale, thr, dscale, seed,
                         seedp);
    };
    if (S <= 64) go(std::integral_constant<int, 64>{});
    else if (S <= 128) go(std::integral_constant<int, 128>{});
    else go(std::integral_constant<int, 64>{});
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(256), 0, stream, Q, ldq, K, ldk, V, ldv, DO, lddo, kmask, lse2,
                     Dbuf, (uint16_t*)dq, lddq, S, H, scale, thr, dscale, seed, seedp);
  hipLaunchKernelGGL(attn_bwd_dkv_kernel, grid, dim3(256), 0, stream, Q, ldq, K, ldk, V, ldv, DO, lddo, kmask, lse2,
                     Dbuf, (uint16_t*)dk, lddk, (uint16_t*)dv, lddv, S, H, scale, thr, dscale, seed, seedp);
  return (int)hipGetLastError();
}
