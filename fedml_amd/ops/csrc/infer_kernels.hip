// Inference-only fused bottleneck for the client-batched native ResNet forward (gfx950, wave64, exact fp32
// v_mfma_f32_16x16x4_f32): evaluation of the global model and the Shapley valuation's coalition models
// (NativeResNetStep.forward_eval; core/valuation.py, simulation/rccl/evaluation.py).
//
// The training forward runs a bottleneck (reference model/cv/resnet.py:87-137) as separate kernels — 1×1 conv,
// 3×3 conv, 1×1 conv, block output — with every intermediate written to and re-read from HBM and batch statistics
// accumulated on the way. Inference needs none of that: BatchNorm is a per-channel scale / shift from the running
// statistics (bn_eval_fold), so one workgroup takes a band of R output rows of one image of one model and runs
//
//   m1 = relu(s1·(x ⊛ W1) + t1)      rows r0−1 .. r0+R (halo), zero outside the image     → LDS
//   m2 = relu(s2·(m1 ⊛ W2) + t2)     3×3, stride 1, pad 1                                  → LDS
//   y  = relu(s3·(m2 ⊛ W3) + t3 + x)                                                        → HBM
//
// reading x once (plus its L2-resident residual re-read) and writing y once. The model's three packed weight
// matrices stay in LDS (bneck_eval_kernel) or, by default, in each wave's registers (bneck_eval_rw_kernel) for all
// the units of that model the workgroup processes.
//
// MFMA operand convention (K16 fragments): in one K-step of 16, lane group g = lane>>4 holds k = 4g..4g+3 as a
// float4 and MFMA j (0..3) consumes element j — A = weights (row = output channel lane&15), B = activations
// (column = pixel lane&15), so D[channel][pixel] leaves each lane 4 consecutive channels of one pixel (one
// float4 store per tile, per-lane scale / shift).
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace infer {

struct BArgs {
  const float* x;      // block input  [C][N][H][W][CIN]
  float* out;          // block output [C][N][H][W][CIN]
  const float* wpk;    // packed forward weights, model c at wpk + c·wpk_ld
  int64_t wpk_ld;
  int64_t off1, off2, off3;   // 1×1 (CM × CIN), 3×3 (CM × 9·CM, tap-major), 1×1 (CIN × CM)
  int ldk1, ldk2, ldk3;
  const float *s1, *t1, *s2, *t2, *s3, *t3;   // folded BatchNorm [C][CM] ×4, [C][CIN] ×2
  int N, units_per_wg;
  float* pool;   // bneck3 only: non-null → write the global average pool [C][N][CIN] instead of y
};

__device__ __forceinline__ f32x4 mma4(const float4 a, const float4 b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
}

// two independent accumulator chains interleaved (the 16x16x4 f32 MFMA has a 40-cycle dependent latency and a
// 32-cycle issue: one chain alone leaves the matrix pipe idle between its MFMAs)
__device__ __forceinline__ void mma4x2(const float4 a0, const float4 b0, f32x4& c0, const float4 a1, const float4 b1,
                                       f32x4& c1) {
  c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, c1, 0, 0, 0);
}

template <int CM, int HW, int R>
struct Geo {
  static constexpr int CIN = 4 * CM;
  static constexpr int H = HW, W = HW;
  static constexpr int BANDS = H / R;
  static constexpr int TW = W + 2;                 // m1 tile width incl. the zero halo columns
  static constexpr int P1 = (R + 2) * W;           // conv1 outputs (halo rows included)
  static constexpr int P2 = R * W;
  static constexpr int LW1 = CIN + 4, LW2 = 9 * CM + 4, LW3 = CM + 4, LM = CM + 4;   // LDS pitches (floats)
  static constexpr int FLOATS = CM * LW1 + CM * LW2 + CIN * LW3 + 4 * CM + 2 * CIN + (R + 2) * TW * LM + P2 * LM;
};

template <int CM, int HW, int R, int NW>
__global__ __launch_bounds__(64 * NW) void bneck_eval_kernel(BArgs a) {
  using G = Geo<CM, HW, R>;
  constexpr int CIN = G::CIN, H = G::H, W = G::W, TW = G::TW, LM = G::LM;
  constexpr int LW1 = G::LW1, LW2 = G::LW2, LW3 = G::LW3;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* w1 = sm;                        // [CM][LW1]
  float* w2 = w1 + CM * LW1;             // [CM][LW2]
  float* w3 = w2 + CM * LW2;             // [CIN][LW3]
  float* vs = w3 + CIN * LW3;            // s1 t1 s2 t2 [CM], s3 t3 [CIN]
  float* m1 = vs + 4 * CM + 2 * CIN;     // [R+2][TW][LM]
  float* m2 = m1 + (R + 2) * TW * LM;    // [P2][LM]
  const int c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int units = a.N * G::BANDS;
  const int u_lo = blockIdx.x * a.units_per_wg;
  if (u_lo >= units) return;   // uniform: whole workgroup
  const int u_hi = min(units, u_lo + a.units_per_wg);
  {
    const float* pk = a.wpk + (int64_t)c * a.wpk_ld;
    for (int i = tid; i < CM * CIN; i += 64 * NW) {
      const int n = i / CIN, k = i - n * CIN;
      w1[n * LW1 + k] = pk[a.off1 + (int64_t)n * a.ldk1 + k];
    }
    for (int i = tid; i < CM * 9 * CM; i += 64 * NW) {
      const int n = i / (9 * CM), k = i - n * (9 * CM);
      w2[n * LW2 + k] = pk[a.off2 + (int64_t)n * a.ldk2 + k];
    }
    for (int i = tid; i < CIN * CM; i += 64 * NW) {
      const int n = i / CM, k = i - n * CM;
      w3[n * LW3 + k] = pk[a.off3 + (int64_t)n * a.ldk3 + k];
    }
    for (int i = tid; i < CM; i += 64 * NW) {
      vs[i] = a.s1[(int64_t)c * CM + i];
      vs[CM + i] = a.t1[(int64_t)c * CM + i];
      vs[2 * CM + i] = a.s2[(int64_t)c * CM + i];
      vs[3 * CM + i] = a.t2[(int64_t)c * CM + i];
    }
    for (int i = tid; i < CIN; i += 64 * NW) {
      vs[4 * CM + i] = a.s3[(int64_t)c * CIN + i];
      vs[4 * CM + CIN + i] = a.t3[(int64_t)c * CIN + i];
    }
    // the zero halo columns of m1 (conv1 never writes them)
    for (int i = tid; i < (R + 2) * 2 * CM; i += 64 * NW) {
      const int r = i / (2 * CM), side = (i / CM) & 1, ch = i % CM;
      m1[(r * TW + (side ? W + 1 : 0)) * LM + ch] = 0.f;
    }
  }
  __syncthreads();
  const float* s1 = vs;
  const float* t1 = vs + CM;
  const float* s2 = vs + 2 * CM;
  const float* t2 = vs + 3 * CM;
  const float* s3 = vs + 4 * CM;
  const float* t3 = vs + 4 * CM + CIN;

  for (int u = u_lo; u < u_hi; ++u) {
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    const int64_t img = ((int64_t)c * a.N + n) * H * W * CIN;
    const float* xin = a.x + img;
    float* yout = a.out + img;

    // ---- conv1 + bn1 + relu: rows r0−1 .. r0+R → m1 ----
    for (int t = wid; t < (G::P1 / 16) * (CM / 16); t += NW) {
      const int pt = t / (CM / 16), nt = t - pt * (CM / 16);
      const int p = pt * 16 + l16, pr = p / W, pc = p - pr * W;
      const int row = r0 - 1 + pr;
      const bool inside = row >= 0 && row < H;
      const float* xp = xin + ((int64_t)(inside ? row : 0) * W + pc) * CIN + 4 * g;
      float4 bx[CIN / 16];
#pragma unroll
      for (int ks = 0; ks < CIN / 16; ++ks)
        bx[ks] = inside ? *reinterpret_cast<const float4*>(xp + 16 * ks) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float* wr = w1 + (nt * 16 + l16) * LW1 + 4 * g;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < CIN / 16; ++ks) acc = mma4(*reinterpret_cast<const float4*>(wr + 16 * ks), bx[ks], acc);
      const int ch = nt * 16 + 4 * g;
      float4 v;
      v.x = inside ? fmaxf(acc[0] * s1[ch] + t1[ch], 0.f) : 0.f;
      v.y = inside ? fmaxf(acc[1] * s1[ch + 1] + t1[ch + 1], 0.f) : 0.f;
      v.z = inside ? fmaxf(acc[2] * s1[ch + 2] + t1[ch + 2], 0.f) : 0.f;
      v.w = inside ? fmaxf(acc[3] * s1[ch + 3] + t1[ch + 3], 0.f) : 0.f;
      *reinterpret_cast<float4*>(m1 + (pr * TW + pc + 1) * LM + ch) = v;
    }
    __syncthreads();

    // ---- conv2 (3×3) + bn2 + relu → m2: two tiles per wave iteration (T2 is a multiple of 8) ----
    static_assert(((G::P2 / 16) * (CM / 16)) % (2 * NW) == 0, "conv2 tiles");
    for (int t = wid; t < (G::P2 / 16) * (CM / 16); t += 2 * NW) {
      int p[2], ch[2];
      const float* wr[2];
      const float* mp[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int th = t + NW * h;
        const int pt = th / (CM / 16), nt = th - pt * (CM / 16);
        p[h] = pt * 16 + l16;
        const int pr = p[h] / W, pc = p[h] - pr * W;
        wr[h] = w2 + (nt * 16 + l16) * LW2 + 4 * g;
        mp[h] = m1 + (pr * TW + pc) * LM + 4 * g;
        ch[h] = nt * 16 + 4 * g;
      }
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap - 3 * (tap / 3);
        const int mo = (kh * TW + kw) * LM;
#pragma unroll
        for (int cc = 0; cc < CM / 16; ++cc)
          mma4x2(*reinterpret_cast<const float4*>(wr[0] + tap * CM + 16 * cc),
                 *reinterpret_cast<const float4*>(mp[0] + mo + 16 * cc), acc0,
                 *reinterpret_cast<const float4*>(wr[1] + tap * CM + 16 * cc),
                 *reinterpret_cast<const float4*>(mp[1] + mo + 16 * cc), acc1);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 acc = h ? acc1 : acc0;
        const int c0 = ch[h];
        float4 v;
        v.x = fmaxf(acc[0] * s2[c0] + t2[c0], 0.f);
        v.y = fmaxf(acc[1] * s2[c0 + 1] + t2[c0 + 1], 0.f);
        v.z = fmaxf(acc[2] * s2[c0 + 2] + t2[c0 + 2], 0.f);
        v.w = fmaxf(acc[3] * s2[c0 + 3] + t2[c0 + 3], 0.f);
        *reinterpret_cast<float4*>(m2 + p[h] * LM + c0) = v;
      }
    }
    __syncthreads();

    // ---- conv3 (1×1) + bn3 + residual + relu → y: two tiles per wave iteration ----
    static_assert(((G::P2 / 16) * (CIN / 16)) % (2 * NW) == 0, "conv3 tiles");
    for (int t = wid; t < (G::P2 / 16) * (CIN / 16); t += 2 * NW) {
      int p[2], ch[2];
      const float* wr[2];
      const float* mp[2];
      float4 res[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int th = t + NW * h;
        const int pt = th / (CIN / 16), nt = th - pt * (CIN / 16);
        p[h] = pt * 16 + l16;
        wr[h] = w3 + (nt * 16 + l16) * LW3 + 4 * g;
        mp[h] = m2 + p[h] * LM + 4 * g;
        ch[h] = nt * 16 + 4 * g;
        const int pr = p[h] / W, pc = p[h] - pr * W;
        res[h] = *reinterpret_cast<const float4*>(xin + ((int64_t)(r0 + pr) * W + pc) * CIN + ch[h]);   // early
      }
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < CM / 16; ++ks)
        mma4x2(*reinterpret_cast<const float4*>(wr[0] + 16 * ks), *reinterpret_cast<const float4*>(mp[0] + 16 * ks),
               acc0, *reinterpret_cast<const float4*>(wr[1] + 16 * ks),
               *reinterpret_cast<const float4*>(mp[1] + 16 * ks), acc1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 acc = h ? acc1 : acc0;
        const int c0 = ch[h];
        const int pr = p[h] / W, pc = p[h] - pr * W;
        float4 v;
        v.x = fmaxf(acc[0] * s3[c0] + t3[c0] + res[h].x, 0.f);
        v.y = fmaxf(acc[1] * s3[c0 + 1] + t3[c0 + 1] + res[h].y, 0.f);
        v.z = fmaxf(acc[2] * s3[c0 + 2] + t3[c0 + 2] + res[h].z, 0.f);
        v.w = fmaxf(acc[3] * s3[c0 + 3] + t3[c0 + 3] + res[h].w, 0.f);
        *reinterpret_cast<float4*>(yout + ((int64_t)(r0 + pr) * W + pc) * CIN + c0) = v;
      }
    }
    __syncthreads();   // m1 / m2 are rewritten by the next unit
  }
}

// ---- register-resident weights (variant 3) ----
// Every wave keeps ONE output-channel tile per conv for the whole kernel (conv1 / conv2: nt = wave mod CM/16, conv3:
// nt = wave mod CIN/16), so the three A-fragment sets live in VGPRs — loaded once from the packed weights, no LDS
// weight reads in the MFMA loops (half the LDS traffic of conv2, none in conv1 / conv3) and no 73 KB weight stage
// in LDS. conv1's x tiles are software-pipelined one tile ahead (the last tile of a unit prefetches the next unit's
// first, in flight across conv2 / conv3); its K is split over two accumulators so the MFMA chain never waits on
// itself.
//
// BAND (the memory-bound 32×32 stage): the unit's whole input band (R+2 rows × W × CIN) is staged in LDS from
// registers that were loaded during the PREVIOUS unit — HBM reads spread over the whole unit instead of bursting in
// conv1, ~80 KB in flight per CU — and the residual comes from the band too (x is read from HBM exactly once).
template <int CM, int HW, int R, bool BAND, bool PIPE>
struct GeoR {
  static constexpr int CIN = 4 * CM, H = HW, W = HW, BANDS = H / R, TW = W + 2;
  static constexpr int P1 = (R + 2) * W, P2 = R * W, PT1 = P1 / 16, PT2 = P2 / 16;
  static constexpr int NT1 = CM / 16, NT3 = CIN / 16, LM = CM + 4, LX = CIN + 4;
  static constexpr int NF4 = P1 * CIN / 4;   // band float4s
  static constexpr int M1F = (R + 2) * TW * LM, M2F = P2 * LM, NB = PIPE ? 2 : 1;   // m1 / m2 floats; buffers
  static constexpr int FLOATS = 4 * CM + 2 * CIN + NB * (M1F + M2F) + (BAND ? P1 * LX : 0);
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// NW = 8: one workgroup per CU; NW = 4 (smaller R): two per CU, so one workgroup's barrier waits overlap the
// other's MFMAs. conv3 gives a wave NT3/NW channel tiles when the waves are fewer than CIN/16.
template <int CM, int HW, int R, bool BAND, bool PIPE, int NW, int Q2>
__global__ __launch_bounds__(64 * NW, NW == 4 ? (BAND ? 1 : 3) : 2) void bneck_eval_rw_kernel(BArgs a) {   // waves per SIMD
  using G = GeoR<CM, HW, R, BAND, PIPE>;
  static_assert(!(BAND && PIPE), "the band is read by conv1 and conv3 of one unit");
  constexpr int CIN = G::CIN, H = G::H, W = G::W, TW = G::TW, LM = G::LM, NT1 = G::NT1, NT3 = G::NT3;
  constexpr int NTW3 = NT3 > NW ? NT3 / NW : 1;   // conv3 channel tiles per wave
  constexpr int PS1 = NW / NT1, PS3 = NT3 >= NW ? 1 : NW / NT3;   // pixel-tile strides of conv1/conv2 and conv3
  constexpr int PF = (G::NF4 + 64 * NW - 1) / (64 * NW);          // BAND float4s per thread
  static_assert(NW % NT1 == 0 && (NW % NT3 == 0 || NT3 % NW == 0), "wave split");
  static_assert(G::PT2 % (Q2 * PS1) == 0 && G::PT2 % (2 * PS3) == 0, "Q2 / two pixel tiles per wave iteration");
  static_assert((CIN / 16) % 2 == 0 && Q2 % 2 == 0, "conv1 K split; conv2 chains in pairs");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* vs = sm;                          // s1 t1 s2 t2 [CM], s3 t3 [CIN]
  float* m1 = vs + 4 * CM + 2 * CIN;       // [NB][R+2][TW][LM]
  float* m2 = m1 + G::NB * G::M1F;         // [NB][P2][LM]
  float* xb = m2 + G::NB * G::M2F;         // BAND: [P1][LX]
  constexpr int LX = G::LX;
  const int c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int units = a.N * G::BANDS;
  const int u_lo = blockIdx.x * a.units_per_wg;
  if (u_lo >= units) return;   // uniform: whole workgroup
  const int u_hi = min(units, u_lo + a.units_per_wg);
  const int nt1 = wid % NT1, pg1 = wid / NT1, nt3 = wid % NT3, pg3 = NT3 >= NW ? 0 : wid / NT3;

  const float* pk = a.wpk + (int64_t)c * a.wpk_ld;
  float4 a1[CIN / 16], a2[9 * NT1], a3[NTW3][NT1];
  {
    const float* w1 = pk + a.off1 + (int64_t)(nt1 * 16 + l16) * a.ldk1 + 4 * g;
    const float* w2 = pk + a.off2 + (int64_t)(nt1 * 16 + l16) * a.ldk2 + 4 * g;
    const float* w3 = pk + a.off3 + (int64_t)(nt3 * 16 + l16) * a.ldk3 + 4 * g;   // + NW·16 rows per extra tile
#pragma unroll
    for (int ks = 0; ks < CIN / 16; ++ks) a1[ks] = ld4(w1 + 16 * ks);
#pragma unroll
    for (int j = 0; j < 9 * NT1; ++j) a2[j] = ld4(w2 + (j / NT1) * CM + 16 * (j % NT1));
#pragma unroll
    for (int j = 0; j < NTW3; ++j)
#pragma unroll
      for (int ks = 0; ks < NT1; ++ks) a3[j][ks] = ld4(w3 + (int64_t)j * NW * 16 * a.ldk3 + 16 * ks);
  }
  for (int i = tid; i < CM; i += 64 * NW) {
    vs[i] = a.s1[(int64_t)c * CM + i];
    vs[CM + i] = a.t1[(int64_t)c * CM + i];
    vs[2 * CM + i] = a.s2[(int64_t)c * CM + i];
    vs[3 * CM + i] = a.t2[(int64_t)c * CM + i];
  }
  for (int i = tid; i < CIN; i += 64 * NW) {
    vs[4 * CM + i] = a.s3[(int64_t)c * CIN + i];
    vs[4 * CM + CIN + i] = a.t3[(int64_t)c * CIN + i];
  }
  for (int i = tid; i < G::NB * (R + 2) * 2 * CM; i += 64 * NW) {   // m1's zero halo columns (never written)
    const int b = i / ((R + 2) * 2 * CM), r = (i / (2 * CM)) % (R + 2), side = (i / CM) & 1, ch = i % CM;
    m1[b * G::M1F + (r * TW + (side ? W + 1 : 0)) * LM + ch] = 0.f;
  }
  const float* s1 = vs;
  const float* t1 = vs + CM;
  const float* s2 = vs + 2 * CM;
  const float* t2 = vs + 3 * CM;
  const float* s3 = vs + 4 * CM;
  const float* t3 = vs + 4 * CM + CIN;

  // x tile `pt` of unit u (rows r0−1 .. r0+R; rows outside the image read a clamped in-image row — conv1 zeroes
  // their outputs, so only the address has to be valid)
  float4 bx[CIN / 16];
  float4 pf[BAND ? PF : 1];
  // BAND: thread tid holds float4s f = tid + 512·i of the band (pixel f / (CIN/4), channels 4·(f mod CIN/4)):
  // consecutive threads read consecutive 16 B of HBM. Rows outside the image are not loaded (conv1 zeroes them).
  auto load_band = [&](int u) {
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    const float* xi = a.x + ((int64_t)c * a.N + n) * H * W * CIN;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int f = tid + 64 * NW * i, q = f / (CIN / 4), row = r0 - 1 + q / W;
      if (f < G::NF4 && row >= 0 && row < H)
        pf[i] = ld4(xi + ((int64_t)row * W + q % W) * CIN + 4 * (f % (CIN / 4)));
    }
  };
  auto store_band = [&]() {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int f = tid + 64 * NW * i;
      if (f < G::NF4) *reinterpret_cast<float4*>(xb + (f / (CIN / 4)) * LX + 4 * (f % (CIN / 4))) = pf[i];
    }
  };
  auto load_x = [&](int u, int pt) {
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    const int p = pt * 16 + l16, pr = p / W, pc = p - pr * W;
    const int row = min(max(r0 - 1 + pr, 0), H - 1);
    const float* xp = a.x + (((int64_t)c * a.N + n) * H * W + (int64_t)row * W + pc) * CIN + 4 * g;
#pragma unroll
    for (int ks = 0; ks < CIN / 16; ++ks) bx[ks] = ld4(xp + 16 * ks);
  };
  // ---- conv1 + bn1 + relu: unit u → m1b ----
  auto conv1 = [&](int u, float* m1b) {
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    for (int pt = pg1; pt < G::PT1; pt += PS1) {
      float4 cur[CIN / 16];
      if constexpr (BAND) {
        const float* xp = xb + (pt * 16 + l16) * LX + 4 * g;
#pragma unroll
        for (int ks = 0; ks < CIN / 16; ++ks) cur[ks] = ld4(xp + 16 * ks);
      } else {
#pragma unroll
        for (int ks = 0; ks < CIN / 16; ++ks) cur[ks] = bx[ks];
        if (pt + PS1 < G::PT1) load_x(u, pt + PS1);
        else if (u + 1 < u_hi) load_x(u + 1, pg1);
      }
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < CIN / 16; ks += 2) mma4x2(a1[ks], cur[ks], acc0, a1[ks + 1], cur[ks + 1], acc1);
      const int p = pt * 16 + l16, pr = p / W, pc = p - pr * W;
      const int row = r0 - 1 + pr;
      const bool inside = row >= 0 && row < H;
      const int ch = nt1 * 16 + 4 * g;
      float4 v;
      v.x = inside ? fmaxf((acc0[0] + acc1[0]) * s1[ch] + t1[ch], 0.f) : 0.f;
      v.y = inside ? fmaxf((acc0[1] + acc1[1]) * s1[ch + 1] + t1[ch + 1], 0.f) : 0.f;
      v.z = inside ? fmaxf((acc0[2] + acc1[2]) * s1[ch + 2] + t1[ch + 2], 0.f) : 0.f;
      v.w = inside ? fmaxf((acc0[3] + acc1[3]) * s1[ch + 3] + t1[ch + 3], 0.f) : 0.f;
      *reinterpret_cast<float4*>(m1b + (pr * TW + pc + 1) * LM + ch) = v;
    }
  };

  // ---- conv2 (3×3) + bn2 + relu: m1b → m2b, pixel tiles pt and pt + PS1 per iteration ----
  auto conv2 = [&](const float* m1b, float* m2b) {
    for (int pt = pg1; pt < G::PT2; pt += Q2 * PS1) {
      const float* mp[Q2];
      int p[Q2];
#pragma unroll
      for (int h = 0; h < Q2; ++h) {
        p[h] = (pt + h * PS1) * 16 + l16;
        const int pr = p[h] / W, pc = p[h] - pr * W;
        mp[h] = m1b + (pr * TW + pc) * LM + 4 * g;
      }
      f32x4 acc[Q2];
#pragma unroll
      for (int h = 0; h < Q2; ++h) acc[h] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int mo = ((tap / 3) * TW + tap % 3) * LM;
#pragma unroll
        for (int cc = 0; cc < NT1; ++cc)
#pragma unroll
          for (int h = 0; h < Q2; h += 2)
            mma4x2(a2[tap * NT1 + cc], ld4(mp[h] + mo + 16 * cc), acc[h], a2[tap * NT1 + cc],
                   ld4(mp[h + 1] + mo + 16 * cc), acc[h + 1]);
      }
      const int c0 = nt1 * 16 + 4 * g;
#pragma unroll
      for (int h = 0; h < Q2; ++h) {
        float4 v;
        v.x = fmaxf(acc[h][0] * s2[c0] + t2[c0], 0.f);
        v.y = fmaxf(acc[h][1] * s2[c0 + 1] + t2[c0 + 1], 0.f);
        v.z = fmaxf(acc[h][2] * s2[c0 + 2] + t2[c0 + 2], 0.f);
        v.w = fmaxf(acc[h][3] * s2[c0 + 3] + t2[c0 + 3], 0.f);
        *reinterpret_cast<float4*>(m2b + p[h] * LM + c0) = v;
      }
    }
  };

  // ---- conv3 (1×1) + bn3 + residual + relu: m2b → y of unit u, pixel tiles pt and pt + PS3 per iteration ----
  auto conv3 = [&](int u, const float* m2b) {
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    const int64_t img = ((int64_t)c * a.N + n) * H * W * CIN + (int64_t)r0 * W * CIN;
#pragma unroll
    for (int j = 0; j < NTW3; ++j) {
      const int c0 = (nt3 + j * NW) * 16 + 4 * g;
      for (int pt = pg3; pt < G::PT2; pt += 2 * PS3) {
        int p[2];
        float4 res[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          p[h] = (pt + h * PS3) * 16 + l16;
          res[h] = BAND ? ld4(xb + (W + p[h]) * LX + c0)             // the band's centre rows
                        : ld4(a.x + img + (int64_t)p[h] * CIN + c0);   // early: hides under the MFMAs
        }
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NT1; ++ks)
          mma4x2(a3[j][ks], ld4(m2b + p[0] * LM + 16 * ks + 4 * g), acc0, a3[j][ks],
                 ld4(m2b + p[1] * LM + 16 * ks + 4 * g), acc1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 acc = h ? acc1 : acc0;
          float4 v;
          v.x = fmaxf(acc[0] * s3[c0] + t3[c0] + res[h].x, 0.f);
          v.y = fmaxf(acc[1] * s3[c0 + 1] + t3[c0 + 1] + res[h].y, 0.f);
          v.z = fmaxf(acc[2] * s3[c0 + 2] + t3[c0 + 2] + res[h].z, 0.f);
          v.w = fmaxf(acc[3] * s3[c0 + 3] + t3[c0 + 3] + res[h].w, 0.f);
          *reinterpret_cast<float4*>(a.out + img + (int64_t)p[h] * CIN + c0) = v;
        }
      }
    }
  };

  if constexpr (BAND) load_band(u_lo);
  else if (pg1 < G::PT1) load_x(u_lo, pg1);
  __syncthreads();

  if constexpr (PIPE) {
    // interval k: conv1 of unit k, conv2 of unit k−1, conv3 of unit k−2 (m1 / m2 double-buffered): one barrier per
    // unit, and every interval carries a whole bottleneck's work, so the waves stay balanced between barriers
    const int nu = u_hi - u_lo;
    for (int k = 0; k < nu + 2; ++k) {
      if (k < nu) conv1(u_lo + k, m1 + (k & 1) * G::M1F);
      if (k >= 1 && k - 1 < nu) conv2(m1 + ((k - 1) & 1) * G::M1F, m2 + ((k - 1) & 1) * G::M2F);
      if (k >= 2) conv3(u_lo + k - 2, m2 + (k & 1) * G::M2F);
      __syncthreads();
    }
  } else {
    for (int u = u_lo; u < u_hi; ++u) {
      if constexpr (BAND) {
        store_band();
        __syncthreads();
        if (u + 1 < u_hi) load_band(u + 1);   // in flight for the whole unit
      }
      conv1(u, m1);
      __syncthreads();
      conv2(m1, m2);
      __syncthreads();
      conv3(u, m2);
      __syncthreads();   // m1 / m2 are rewritten by the next unit
    }
  }
}

template <int CM, int HW, int R, bool BAND, bool PIPE, int NW, int Q2 = 2>
static int launch_rw(BArgs a, int C, hipStream_t stream) {
  using G = GeoR<CM, HW, R, BAND, PIPE>;
  const size_t smem = (size_t)G::FLOATS * 4;
  if (smem > 160 * 1024) return -5;
  const int units = a.N * G::BANDS;
  // one 8-wave (two 4-wave) workgroups per CU (the weight fragments take ~60-120 VGPRs a wave): ~2 workgroups per
  // CU over all models, each looping over a contiguous run of one model's units
  const int target = NW == 4 ? 1024 : 512;
  const int per_model = std::max(1, std::min(units, (target + C - 1) / C));
  a.units_per_wg = (units + per_model - 1) / per_model;
  const int gx = (units + a.units_per_wg - 1) / a.units_per_wg;
  auto kern = bneck_eval_rw_kernel<CM, HW, R, BAND, PIPE, NW, Q2>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(64 * NW), smem, stream, a);
  return (int)hipGetLastError();
}

template <int CM, int HW, int R, int NW>
static int launch(BArgs a, int C, hipStream_t stream) {
  using G = Geo<CM, HW, R>;
  const size_t smem = (size_t)G::FLOATS * 4;
  if (smem > 160 * 1024) return -5;
  const int units = a.N * G::BANDS;
  // ~1024 workgroups over all models (4 per CU), each looping over a contiguous run of one model's units: the
  // model's weights are staged once per workgroup
  const int per_model = std::max(1, std::min(units, (1024 + C - 1) / C));
  a.units_per_wg = (units + per_model - 1) / per_model;
  const int gx = (units + a.units_per_wg - 1) / a.units_per_wg;
  auto kern = bneck_eval_kernel<CM, HW, R, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(64 * NW), smem, stream, a);
  return (int)hipGetLastError();
}

// ---- stage-entry bottleneck with a downsample shortcut (register-resident weights) ----
// y = relu(s3·(m2 ⊛ W3) + t3 + sd·(x ⊛_S Wd) + td), m2 = relu(bn2(conv2_S(relu(bn1(x ⊛ W1))))): the first block of a
// stage (reference model/cv/resnet.py:113-121 — stride S on the 3×3, a 1×1 stride-S projection shortcut). x has CX
// channels at HW², y has CO = 4·CM at (HW/S)². A unit is a band of R output rows; conv1 runs on the S·(R−1)+3 input
// rows the band's 3×3 windows touch. The projection's operands are the x pixels conv1 just read (L2-resident).
template <int CX, int CM, int HW, int S, int R>
struct GeoD {
  static constexpr int CO = 4 * CM, H = HW, W = HW, HO = HW / S, WO = HW / S, BANDS = HO / R, TW = W + 2;
  static constexpr int RI = S * (R - 1) + 3, P1 = RI * W, P2 = R * WO, PT1 = P1 / 16, PT2 = P2 / 16;
  static constexpr int NT1 = CM / 16, NT3 = CO / 16, KX = CX / 16, LM = CM + 4;
  static constexpr int M1F = RI * TW * LM, M2F = P2 * LM;
  static constexpr int FLOATS = 4 * CM + 4 * CO + M1F + M2F;
};

struct DArgs {
  BArgs b;
  int64_t offd;
  int ldkd;
  const float *sd, *td;   // folded shortcut BatchNorm [C][CO]
};

template <int CX, int CM, int HW, int S, int R>
__global__ __launch_bounds__(512, 2) void bneck_ds_eval_kernel(DArgs d) {
  using G = GeoD<CX, CM, HW, S, R>;
  constexpr int NW = 8, CO = G::CO, H = G::H, W = G::W, WO = G::WO, TW = G::TW, LM = G::LM;
  constexpr int NT1 = G::NT1, NT3 = G::NT3, KX = G::KX;
  constexpr int NTW3 = NT3 > NW ? NT3 / NW : 1;
  constexpr int PS1 = NW / NT1, PS3 = NT3 >= NW ? 1 : NW / NT3;
  static_assert(CX % 16 == 0 && G::P1 % 16 == 0 && G::P2 % 16 == 0 && HW % S == 0 && G::HO % R == 0, "geometry");
  static_assert(NW % NT1 == 0 && (NW % NT3 == 0 || NT3 % NW == 0), "wave split");
  static_assert(G::PT2 % (2 * PS1) == 0 && G::PT2 % (2 * PS3) == 0, "two pixel tiles per wave iteration");
  const BArgs& a = d.b;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* vs = sm;                          // s1 t1 s2 t2 [CM], s3 t3 sd td [CO]
  float* m1 = vs + 4 * CM + 4 * CO;        // [RI][TW][LM]
  float* m2 = m1 + G::M1F;                 // [P2][LM]
  const int c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int units = a.N * G::BANDS;
  const int u_lo = blockIdx.x * a.units_per_wg;
  if (u_lo >= units) return;   // uniform: whole workgroup
  const int u_hi = min(units, u_lo + a.units_per_wg);
  const int nt1 = wid % NT1, pg1 = wid / NT1, nt3 = wid % NT3, pg3 = NT3 >= NW ? 0 : wid / NT3;

  const float* pk = a.wpk + (int64_t)c * a.wpk_ld;
  float4 a1[KX], a2[9 * NT1], a3[NTW3][NT1], ad[NTW3][KX];
  {
    const float* w1 = pk + a.off1 + (int64_t)(nt1 * 16 + l16) * a.ldk1 + 4 * g;
    const float* w2 = pk + a.off2 + (int64_t)(nt1 * 16 + l16) * a.ldk2 + 4 * g;
    const float* w3 = pk + a.off3 + (int64_t)(nt3 * 16 + l16) * a.ldk3 + 4 * g;
    const float* wd = pk + d.offd + (int64_t)(nt3 * 16 + l16) * d.ldkd + 4 * g;
#pragma unroll
    for (int ks = 0; ks < KX; ++ks) a1[ks] = ld4(w1 + 16 * ks);
#pragma unroll
    for (int j = 0; j < 9 * NT1; ++j) a2[j] = ld4(w2 + (j / NT1) * CM + 16 * (j % NT1));
#pragma unroll
    for (int j = 0; j < NTW3; ++j) {
#pragma unroll
      for (int ks = 0; ks < NT1; ++ks) a3[j][ks] = ld4(w3 + (int64_t)j * NW * 16 * a.ldk3 + 16 * ks);
#pragma unroll
      for (int ks = 0; ks < KX; ++ks) ad[j][ks] = ld4(wd + (int64_t)j * NW * 16 * d.ldkd + 16 * ks);
    }
  }
  for (int i = tid; i < CM; i += 64 * NW) {
    vs[i] = a.s1[(int64_t)c * CM + i];
    vs[CM + i] = a.t1[(int64_t)c * CM + i];
    vs[2 * CM + i] = a.s2[(int64_t)c * CM + i];
    vs[3 * CM + i] = a.t2[(int64_t)c * CM + i];
  }
  for (int i = tid; i < CO; i += 64 * NW) {
    vs[4 * CM + i] = a.s3[(int64_t)c * CO + i];
    vs[4 * CM + CO + i] = a.t3[(int64_t)c * CO + i];
    vs[4 * CM + 2 * CO + i] = d.sd[(int64_t)c * CO + i];
    vs[4 * CM + 3 * CO + i] = d.td[(int64_t)c * CO + i];
  }
  for (int i = tid; i < G::RI * 2 * CM; i += 64 * NW) {   // m1's zero halo columns (conv1 never writes them)
    const int r = i / (2 * CM), side = (i / CM) & 1, ch = i % CM;
    m1[(r * TW + (side ? W + 1 : 0)) * LM + ch] = 0.f;
  }
  const float* s1 = vs;
  const float* t1 = vs + CM;
  const float* s2 = vs + 2 * CM;
  const float* t2 = vs + 3 * CM;
  const float* s3 = vs + 4 * CM;
  const float* t3 = vs + 4 * CM + CO;
  const float* sdv = vs + 4 * CM + 2 * CO;
  const float* tdv = vs + 4 * CM + 3 * CO;

  float4 bx[KX];
  auto load_x = [&](int u, int pt) {   // conv1 input tile pt of unit u (a clamped in-image row outside the image)
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    const int p = pt * 16 + l16, pr = p / W, pc = p - pr * W;
    const int row = min(max(S * r0 - 1 + pr, 0), H - 1);
    const float* xp = a.x + (((int64_t)c * a.N + n) * H * W + (int64_t)row * W + pc) * CX + 4 * g;
#pragma unroll
    for (int ks = 0; ks < KX; ++ks) bx[ks] = ld4(xp + 16 * ks);
  };
  if (pg1 < G::PT1) load_x(u_lo, pg1);
  __syncthreads();

  for (int u = u_lo; u < u_hi; ++u) {
    const int n = u / G::BANDS, r0 = (u - n * G::BANDS) * R;
    const float* xi = a.x + ((int64_t)c * a.N + n) * H * W * CX;
    float* yo = a.out + (((int64_t)c * a.N + n) * G::HO + r0) * WO * CO;

    // ---- conv1 + bn1 + relu on input rows S·r0−1 .. S·(r0+R−1)+1 → m1 ----
    for (int pt = pg1; pt < G::PT1; pt += PS1) {
      float4 cur[KX];
#pragma unroll
      for (int ks = 0; ks < KX; ++ks) cur[ks] = bx[ks];
      if (pt + PS1 < G::PT1) load_x(u, pt + PS1);
      else if (u + 1 < u_hi) load_x(u + 1, pg1);
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (KX % 2 == 0) {
#pragma unroll
        for (int ks = 0; ks < KX; ks += 2) mma4x2(a1[ks], cur[ks], acc0, a1[ks + 1], cur[ks + 1], acc1);
      } else {
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) acc0 = mma4(a1[ks], cur[ks], acc0);
      }
      const int p = pt * 16 + l16, pr = p / W, pc = p - pr * W;
      const int row = S * r0 - 1 + pr;
      const bool inside = row >= 0 && row < H;
      const int ch = nt1 * 16 + 4 * g;
      float4 v;
      v.x = inside ? fmaxf((acc0[0] + acc1[0]) * s1[ch] + t1[ch], 0.f) : 0.f;
      v.y = inside ? fmaxf((acc0[1] + acc1[1]) * s1[ch + 1] + t1[ch + 1], 0.f) : 0.f;
      v.z = inside ? fmaxf((acc0[2] + acc1[2]) * s1[ch + 2] + t1[ch + 2], 0.f) : 0.f;
      v.w = inside ? fmaxf((acc0[3] + acc1[3]) * s1[ch + 3] + t1[ch + 3], 0.f) : 0.f;
      *reinterpret_cast<float4*>(m1 + (pr * TW + pc + 1) * LM + ch) = v;
    }
    __syncthreads();

    // ---- conv2 (3×3, stride S) + bn2 + relu → m2 ----
    for (int pt = pg1; pt < G::PT2; pt += 2 * PS1) {
      const float* mp[2];
      int q[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        q[h] = (pt + h * PS1) * 16 + l16;
        const int orow = q[h] / WO, ocol = q[h] - orow * WO;
        mp[h] = m1 + (S * orow * TW + S * ocol) * LM + 4 * g;
      }
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int mo = ((tap / 3) * TW + tap % 3) * LM;
#pragma unroll
        for (int cc = 0; cc < NT1; ++cc)
          mma4x2(a2[tap * NT1 + cc], ld4(mp[0] + mo + 16 * cc), acc0, a2[tap * NT1 + cc], ld4(mp[1] + mo + 16 * cc),
                 acc1);
      }
      const int c0 = nt1 * 16 + 4 * g;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 acc = h ? acc1 : acc0;
        float4 v;
        v.x = fmaxf(acc[0] * s2[c0] + t2[c0], 0.f);
        v.y = fmaxf(acc[1] * s2[c0 + 1] + t2[c0 + 1], 0.f);
        v.z = fmaxf(acc[2] * s2[c0 + 2] + t2[c0 + 2], 0.f);
        v.w = fmaxf(acc[3] * s2[c0 + 3] + t2[c0 + 3], 0.f);
        *reinterpret_cast<float4*>(m2 + q[h] * LM + c0) = v;
      }
    }
    __syncthreads();

    // ---- conv3 + bn3 and the stride-S projection + bn_d, summed, relu → y ----
#pragma unroll
    for (int j = 0; j < NTW3; ++j) {
      const int c0 = (nt3 + j * NW) * 16 + 4 * g;
      for (int pt = pg3; pt < G::PT2; pt += 2 * PS3) {
        int q[2];
        float4 xs[2][KX];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          q[h] = (pt + h * PS3) * 16 + l16;
          const int orow = q[h] / WO, ocol = q[h] - orow * WO;
          const float* xp = xi + ((int64_t)S * (r0 + orow) * W + S * ocol) * CX + 4 * g;
#pragma unroll
          for (int ks = 0; ks < KX; ++ks) xs[h][ks] = ld4(xp + 16 * ks);   // early: hides under conv3's MFMAs
        }
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        f32x4 dac0 = {0.f, 0.f, 0.f, 0.f}, dac1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NT1; ++ks)
          mma4x2(a3[j][ks], ld4(m2 + q[0] * LM + 16 * ks + 4 * g), acc0, a3[j][ks],
                 ld4(m2 + q[1] * LM + 16 * ks + 4 * g), acc1);
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) mma4x2(ad[j][ks], xs[0][ks], dac0, ad[j][ks], xs[1][ks], dac1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 acc = h ? acc1 : acc0;
          const f32x4 dac = h ? dac1 : dac0;
          float4 v;
          v.x = fmaxf(acc[0] * s3[c0] + t3[c0] + dac[0] * sdv[c0] + tdv[c0], 0.f);
          v.y = fmaxf(acc[1] * s3[c0 + 1] + t3[c0 + 1] + dac[1] * sdv[c0 + 1] + tdv[c0 + 1], 0.f);
          v.z = fmaxf(acc[2] * s3[c0 + 2] + t3[c0 + 2] + dac[2] * sdv[c0 + 2] + tdv[c0 + 2], 0.f);
          v.w = fmaxf(acc[3] * s3[c0 + 3] + t3[c0 + 3] + dac[3] * sdv[c0 + 3] + tdv[c0 + 3], 0.f);
          *reinterpret_cast<float4*>(yo + (int64_t)q[h] * CO + c0) = v;
        }
      }
    }
    __syncthreads();   // m1 / m2 are rewritten by the next unit
  }
}

template <int CX, int CM, int HW, int S, int R>
static int launch_ds(DArgs d, int C, hipStream_t stream) {
  using G = GeoD<CX, CM, HW, S, R>;
  const size_t smem = (size_t)G::FLOATS * 4;
  if (smem > 160 * 1024) return -5;
  const int units = d.b.N * G::BANDS;
  const int per_model = std::max(1, std::min(units, (512 + C - 1) / C));
  d.b.units_per_wg = (units + per_model - 1) / per_model;
  const int gx = (units + d.b.units_per_wg - 1) / d.b.units_per_wg;
  auto kern = bneck_ds_eval_kernel<CX, CM, HW, S, R>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(512), smem, stream, d);
  return (int)hipGetLastError();
}

// ---- stage-3 bottleneck (64-wide, 8×8): one wave per SIMD, every weight in registers ----
// The 64-wide stage's weights (W1 64×256, W2 64×576, W3 256×64: 272 KB fp32) fit neither LDS nor the 2-waves-per-SIMD
// register budget, but split over FOUR waves (wave w owns conv1 / conv2 output tile w and conv3 output tiles
// w + 4j) they are 68 float4 = 272 VGPRs a wave: one 4-wave workgroup per CU, one wave per SIMD with the 512-entry
// register file. A unit is one 8×8 image: its x (64 px × 256 ch, 64 KB) is staged in LDS from registers loaded
// during the PREVIOUS image, so HBM reads overlap the MFMAs and the residual comes from LDS; four pixel tiles per
// wave give four independent accumulator chains (the 40-cycle MFMA dependency hides behind the other three).
template <int CM>
struct Geo3 {
  static constexpr int CIN = 4 * CM, HW = 8, P = HW * HW, TW = HW + 2, NT1 = CM / 16, NT3 = CIN / 16;
  static constexpr int LX = CIN + 4, LM = CM + 4;
  static constexpr int XF = P * LX, M1F = TW * TW * LM, M2F = P * LM;
  static constexpr int FLOATS = 4 * CM + 2 * CIN + XF + M1F + M2F;
  static constexpr int PF = P * CIN / 4 / 256;   // x float4s per thread
};

template <int CM>
__global__ __launch_bounds__(256, 1) void bneck3_eval_kernel(BArgs a) {
  using G = Geo3<CM>;
  constexpr int CIN = G::CIN, HW = G::HW, P = G::P, TW = G::TW, LX = G::LX, LM = G::LM;
  constexpr int NW = 4, NT1 = G::NT1, NTW3 = G::NT3 / NW, PT = P / 16;
  static_assert(NT1 == NW && G::NT3 % NW == 0 && PT == 4 && (P * CIN / 4) % 256 == 0, "one tile a wave");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* vs = sm;                          // s1 t1 s2 t2 [CM], s3 t3 [CIN]
  float* xs = vs + 4 * CM + 2 * CIN;       // [P][LX]
  float* m1 = xs + G::XF;                  // [TW][TW][LM], zero ring
  float* m2 = m1 + G::M1F;                 // [P][LM]
  const int c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int u_lo = blockIdx.x * a.units_per_wg;
  if (u_lo >= a.N) return;   // uniform: whole workgroup
  const int u_hi = min(a.N, u_lo + a.units_per_wg);

  const float* pk = a.wpk + (int64_t)c * a.wpk_ld;
  float4 a1[CIN / 16], a2[9 * NT1], a3[NTW3][NT1];
  {
    const float* w1 = pk + a.off1 + (int64_t)(wid * 16 + l16) * a.ldk1 + 4 * g;
    const float* w2 = pk + a.off2 + (int64_t)(wid * 16 + l16) * a.ldk2 + 4 * g;
    const float* w3 = pk + a.off3 + (int64_t)(wid * 16 + l16) * a.ldk3 + 4 * g;
#pragma unroll
    for (int ks = 0; ks < CIN / 16; ++ks) a1[ks] = ld4(w1 + 16 * ks);
#pragma unroll
    for (int j = 0; j < 9 * NT1; ++j) a2[j] = ld4(w2 + (j / NT1) * CM + 16 * (j % NT1));
#pragma unroll
    for (int j = 0; j < NTW3; ++j)
#pragma unroll
      for (int ks = 0; ks < NT1; ++ks) a3[j][ks] = ld4(w3 + (int64_t)j * NW * 16 * a.ldk3 + 16 * ks);
  }
  for (int i = tid; i < CM; i += 256) {
    vs[i] = a.s1[(int64_t)c * CM + i];
    vs[CM + i] = a.t1[(int64_t)c * CM + i];
    vs[2 * CM + i] = a.s2[(int64_t)c * CM + i];
    vs[3 * CM + i] = a.t2[(int64_t)c * CM + i];
  }
  for (int i = tid; i < CIN; i += 256) {
    vs[4 * CM + i] = a.s3[(int64_t)c * CIN + i];
    vs[4 * CM + CIN + i] = a.t3[(int64_t)c * CIN + i];
  }
  for (int i = tid; i < G::M1F; i += 256) m1[i] = 0.f;   // the zero ring (conv1 rewrites the interior)
  const float* s1 = vs;
  const float* t1 = vs + CM;
  const float* s2 = vs + 2 * CM;
  const float* t2 = vs + 3 * CM;
  const float* s3 = vs + 4 * CM;
  const float* t3 = vs + 4 * CM + CIN;

  float4 pf[G::PF];   // float4 f = tid + 256·i of an image: pixel f / (CIN/4), channels 4·(f mod CIN/4)
  auto load_img = [&](int n) {
    const float* xi = a.x + ((int64_t)c * a.N + n) * P * CIN;
#pragma unroll
    for (int i = 0; i < G::PF; ++i) pf[i] = ld4(xi + 4 * (int64_t)(tid + 256 * i));
  };
  load_img(u_lo);
  __syncthreads();

  for (int n = u_lo; n < u_hi; ++n) {
#pragma unroll
    for (int i = 0; i < G::PF; ++i) {
      const int f = tid + 256 * i;
      *reinterpret_cast<float4*>(xs + (f / (CIN / 4)) * LX + 4 * (f % (CIN / 4))) = pf[i];
    }
    __syncthreads();
    if (n + 1 < u_hi) load_img(n + 1);   // in flight for the whole image

    // ---- conv1 + bn1 + relu → m1 interior: output tile `wid`, all four pixel tiles ----
    {
      f32x4 acc[PT];
#pragma unroll
      for (int t = 0; t < PT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* xp = xs + l16 * LX + 4 * g;
#pragma unroll
      for (int ks = 0; ks < CIN / 16; ++ks)
#pragma unroll
        for (int t = 0; t < PT; ++t) acc[t] = mma4(a1[ks], ld4(xp + 16 * t * LX + 16 * ks), acc[t]);
      const int ch = wid * 16 + 4 * g;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int p = 16 * t + l16, r = p / HW, col = p % HW;
        float4 v;
        v.x = fmaxf(acc[t][0] * s1[ch] + t1[ch], 0.f);
        v.y = fmaxf(acc[t][1] * s1[ch + 1] + t1[ch + 1], 0.f);
        v.z = fmaxf(acc[t][2] * s1[ch + 2] + t1[ch + 2], 0.f);
        v.w = fmaxf(acc[t][3] * s1[ch + 3] + t1[ch + 3], 0.f);
        *reinterpret_cast<float4*>(m1 + ((r + 1) * TW + col + 1) * LM + ch) = v;
      }
    }
    __syncthreads();

    // ---- conv2 (3×3) + bn2 + relu → m2 ----
    {
      f32x4 acc[PT];
#pragma unroll
      for (int t = 0; t < PT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* mp[PT];
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int p = 16 * t + l16, r = p / HW, col = p % HW;
        mp[t] = m1 + (r * TW + col) * LM + 4 * g;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int mo = ((tap / 3) * TW + tap % 3) * LM;
#pragma unroll
        for (int cc = 0; cc < NT1; ++cc)
#pragma unroll
          for (int t = 0; t < PT; ++t) acc[t] = mma4(a2[tap * NT1 + cc], ld4(mp[t] + mo + 16 * cc), acc[t]);
      }
      const int ch = wid * 16 + 4 * g;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        float4 v;
        v.x = fmaxf(acc[t][0] * s2[ch] + t2[ch], 0.f);
        v.y = fmaxf(acc[t][1] * s2[ch + 1] + t2[ch + 1], 0.f);
        v.z = fmaxf(acc[t][2] * s2[ch + 2] + t2[ch + 2], 0.f);
        v.w = fmaxf(acc[t][3] * s2[ch + 3] + t2[ch + 3], 0.f);
        *reinterpret_cast<float4*>(m2 + (16 * t + l16) * LM + ch) = v;
      }
    }
    __syncthreads();

    // ---- conv3 + bn3 + residual (from the staged x) + relu → y: output tiles wid + 4j (the network's last block
    // with a.pool: the 64-pixel average instead, summed over the four tiles in-lane and over the 16 pixel lanes
    // by butterfly shuffles — y is never written and no pooling pass runs) ----
    float* yo = a.out + ((int64_t)c * a.N + n) * P * CIN;
#pragma unroll
    for (int j = 0; j < NTW3; ++j) {
      const int c0 = (wid + NW * j) * 16 + 4 * g;
      f32x4 acc[PT];
#pragma unroll
      for (int t = 0; t < PT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NT1; ++ks)
#pragma unroll
        for (int t = 0; t < PT; ++t)
          acc[t] = mma4(a3[j][ks], ld4(m2 + (16 * t + l16) * LM + 16 * ks + 4 * g), acc[t]);
      float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int p = 16 * t + l16;
        const float4 res = ld4(xs + p * LX + c0);
        float4 v;
        v.x = fmaxf(acc[t][0] * s3[c0] + t3[c0] + res.x, 0.f);
        v.y = fmaxf(acc[t][1] * s3[c0 + 1] + t3[c0 + 1] + res.y, 0.f);
        v.z = fmaxf(acc[t][2] * s3[c0 + 2] + t3[c0 + 2] + res.z, 0.f);
        v.w = fmaxf(acc[t][3] * s3[c0 + 3] + t3[c0 + 3] + res.w, 0.f);
        if (a.pool) {
          sum.x += v.x;
          sum.y += v.y;
          sum.z += v.z;
          sum.w += v.w;
        } else {
          *reinterpret_cast<float4*>(yo + (int64_t)p * CIN + c0) = v;
        }
      }
      if (a.pool) {   // uniform branch
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          sum.x += __shfl_xor(sum.x, o);
          sum.y += __shfl_xor(sum.y, o);
          sum.z += __shfl_xor(sum.z, o);
          sum.w += __shfl_xor(sum.w, o);
        }
        if (l16 == 0) {
          constexpr float inv = 1.f / P;
          *reinterpret_cast<float4*>(a.pool + ((int64_t)c * a.N + n) * CIN + c0) =
              make_float4(sum.x * inv, sum.y * inv, sum.z * inv, sum.w * inv);
        }
      }
    }
    __syncthreads();   // xs / m1 / m2 are rewritten by the next image
  }
}

template <int CM>
static int launch3(BArgs a, int C, hipStream_t stream) {
  using G = Geo3<CM>;
  const size_t smem = (size_t)G::FLOATS * 4;
  if (smem > 160 * 1024) return -5;
  // one workgroup per CU: ~512 workgroups over all models, each looping over a contiguous run of one model's images
  const int per_model = std::max(1, std::min(a.N, (512 + C - 1) / C));
  a.units_per_wg = (a.N + per_model - 1) / per_model;
  const int gx = (a.N + a.units_per_wg - 1) / a.units_per_wg;
  auto kern = bneck3_eval_kernel<CM>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(kern, dim3(gx, C), dim3(256), smem, stream, a);
  return (int)hipGetLastError();
}

// ---- stage-3 entry (16² × 128 → 8² × 256, stride-2 3×3, projection shortcut): one wave per SIMD ----
// As bneck3_eval_kernel: wave w keeps ALL of conv1's weights (it takes four input rows for every output tile), conv2
// output tile w and conv3 output tiles w + 4j in registers (32 + 36 + 16 = 84 float4 = 336 VGPRs); the projection's
// fragments (32 float4 more would spill) are re-read from L2 per image, each tile's ahead of its conv3 MFMAs. A unit
// is one image: conv1
// reads x straight from global memory (L2 after the first wave) for the 16 input rows; wave 0 also copies the
// stride-2 pixels' fragments to LDS, where conv3's shortcut operand is read from with m2.
struct Geo3D {
  static constexpr int CX = 128, CM = 64, CO = 256, H = 16, W = 16, HO = 8, WO = 8, TW = W + 2, RI = H + 1;
  static constexpr int LM = CM + 4, LX = CX + 4, P1 = H * W, P2 = HO * WO;
  static constexpr int M1F = RI * TW * LM, M2F = P2 * LM, XSF = P2 * LX;
  static constexpr int FLOATS = 4 * CM + 4 * CO + M1F + M2F + XSF;
};

__global__ __launch_bounds__(256, 1) void bneck3_ds_eval_kernel(DArgs d) {
  using G = Geo3D;
  constexpr int CX = G::CX, CM = G::CM, CO = G::CO, W = G::W, WO = G::WO, TW = G::TW, LM = G::LM, LX = G::LX;
  constexpr int NW = 4, KX = CX / 16, NT1 = CM / 16, NTW3 = CO / 16 / NW, PT1 = G::P1 / 16, PT2 = G::P2 / 16;
  static_assert(NT1 == NW && PT2 == 4 && PT1 == 16, "one output tile a wave");
  const BArgs& a = d.b;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* vs = sm;                      // s1 t1 s2 t2 [CM], s3 t3 sd td [CO]
  float* m1 = vs + 4 * CM + 4 * CO;    // [RI][TW][LM]: input row r ↦ r + 1, col c ↦ c + 1; row 0 / col 0 zero
  float* m2 = m1 + G::M1F;             // [P2][LM]
  float* xs = m2 + G::M2F;             // [P2][LX]: x at the stride-2 pixels (the shortcut's operand)
  const int c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int u_lo = blockIdx.x * a.units_per_wg;
  if (u_lo >= a.N) return;   // uniform: whole workgroup
  const int u_hi = min(a.N, u_lo + a.units_per_wg);

  const float* pk = a.wpk + (int64_t)c * a.wpk_ld;
  float4 a1[NT1][KX], a2[9 * NT1], a3[NTW3][NT1];
  const float* wd = pk + d.offd + (int64_t)(wid * 16 + l16) * d.ldkd + 4 * g;   // + NW·16 rows per tile j
  {
    const float* w1 = pk + a.off1 + (int64_t)l16 * a.ldk1 + 4 * g;
    const float* w2 = pk + a.off2 + (int64_t)(wid * 16 + l16) * a.ldk2 + 4 * g;
    const float* w3 = pk + a.off3 + (int64_t)(wid * 16 + l16) * a.ldk3 + 4 * g;
#pragma unroll
    for (int o = 0; o < NT1; ++o)
#pragma unroll
      for (int ks = 0; ks < KX; ++ks) a1[o][ks] = ld4(w1 + (int64_t)o * 16 * a.ldk1 + 16 * ks);
#pragma unroll
    for (int j = 0; j < 9 * NT1; ++j) a2[j] = ld4(w2 + (j / NT1) * CM + 16 * (j % NT1));
#pragma unroll
    for (int j = 0; j < NTW3; ++j)
#pragma unroll
      for (int ks = 0; ks < NT1; ++ks) a3[j][ks] = ld4(w3 + (int64_t)j * NW * 16 * a.ldk3 + 16 * ks);
  }
  for (int i = tid; i < CM; i += 256) {
    vs[i] = a.s1[(int64_t)c * CM + i];
    vs[CM + i] = a.t1[(int64_t)c * CM + i];
    vs[2 * CM + i] = a.s2[(int64_t)c * CM + i];
    vs[3 * CM + i] = a.t2[(int64_t)c * CM + i];
  }
  for (int i = tid; i < CO; i += 256) {
    vs[4 * CM + i] = a.s3[(int64_t)c * CO + i];
    vs[4 * CM + CO + i] = a.t3[(int64_t)c * CO + i];
    vs[4 * CM + 2 * CO + i] = d.sd[(int64_t)c * CO + i];
    vs[4 * CM + 3 * CO + i] = d.td[(int64_t)c * CO + i];
  }
  for (int i = tid; i < G::M1F; i += 256) m1[i] = 0.f;   // the zero row 0 / column 0 (conv1 writes the rest)
  const float* s1 = vs;
  const float* t1 = vs + CM;
  const float* s2 = vs + 2 * CM;
  const float* t2 = vs + 3 * CM;
  const float* s3 = vs + 4 * CM;
  const float* t3 = vs + 4 * CM + CO;
  const float* sdv = vs + 4 * CM + 2 * CO;
  const float* tdv = vs + 4 * CM + 3 * CO;
  __syncthreads();

  for (int n = u_lo; n < u_hi; ++n) {
    const float* xi = a.x + ((int64_t)c * a.N + n) * G::P1 * CX;

    // ---- conv1 + bn1 + relu over the 16 input rows → m1: wave w takes input rows 4w..4w+3 (pixel tile = row)
    // for all four output tiles, so x is read once per workgroup and every B fragment feeds four MFMA chains; the
    // stride-2 pixels' fragments are kept in LDS for the shortcut ----
    {
      f32x4 acc[NT1][4];
#pragma unroll
      for (int o = 0; o < NT1; ++o)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[o][q] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* xr = xi + (int64_t)(4 * wid * W + l16) * CX + 4 * g;
#pragma unroll
      for (int ks = 0; ks < KX; ++ks) {
        float4 b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = ld4(xr + (int64_t)q * W * CX + 16 * ks);
#pragma unroll
        for (int o = 0; o < NT1; ++o)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[o][q] = mma4(a1[o][ks], b[q], acc[o][q]);
        if ((l16 & 1) == 0) {
#pragma unroll
          for (int q = 0; q < 4; q += 2)
            *reinterpret_cast<float4*>(xs + ((2 * wid + q / 2) * WO + (l16 >> 1)) * LX + 16 * ks + 4 * g) = b[q];
        }
      }
#pragma unroll
      for (int o = 0; o < NT1; ++o) {
        const int ch = o * 16 + 4 * g;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 v;
          v.x = fmaxf(acc[o][q][0] * s1[ch] + t1[ch], 0.f);
          v.y = fmaxf(acc[o][q][1] * s1[ch + 1] + t1[ch + 1], 0.f);
          v.z = fmaxf(acc[o][q][2] * s1[ch + 2] + t1[ch + 2], 0.f);
          v.w = fmaxf(acc[o][q][3] * s1[ch + 3] + t1[ch + 3], 0.f);
          *reinterpret_cast<float4*>(m1 + ((4 * wid + q + 1) * TW + l16 + 1) * LM + ch) = v;
        }
      }
    }
    __syncthreads();

    // ---- conv2 (3×3, stride 2) + bn2 + relu → m2 ----
    {
      const int ch1 = wid * 16 + 4 * g;
      f32x4 acc[PT2];
      const float* mp[PT2];
#pragma unroll
      for (int t = 0; t < PT2; ++t) {
        acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int p = 16 * t + l16, orow = p / WO, ocol = p % WO;
        mp[t] = m1 + (2 * orow * TW + 2 * ocol) * LM + 4 * g;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int mo = ((tap / 3) * TW + tap % 3) * LM;
#pragma unroll
        for (int cc = 0; cc < NT1; ++cc)
#pragma unroll
          for (int t = 0; t < PT2; ++t) acc[t] = mma4(a2[tap * NT1 + cc], ld4(mp[t] + mo + 16 * cc), acc[t]);
      }
#pragma unroll
      for (int t = 0; t < PT2; ++t) {
        float4 v;
        v.x = fmaxf(acc[t][0] * s2[ch1] + t2[ch1], 0.f);
        v.y = fmaxf(acc[t][1] * s2[ch1 + 1] + t2[ch1 + 1], 0.f);
        v.z = fmaxf(acc[t][2] * s2[ch1 + 2] + t2[ch1 + 2], 0.f);
        v.w = fmaxf(acc[t][3] * s2[ch1 + 3] + t2[ch1 + 3], 0.f);
        *reinterpret_cast<float4*>(m2 + (16 * t + l16) * LM + ch1) = v;
      }
    }
    __syncthreads();

    // ---- conv3 + bn3 + shortcut conv + bn_d, summed, relu → y ----
    float* yo = a.out + ((int64_t)c * a.N + n) * G::P2 * CO;
#pragma unroll
    for (int j = 0; j < NTW3; ++j) {
      const int c0 = (wid + NW * j) * 16 + 4 * g;
      float4 adj[KX];   // issued before conv3's MFMAs, consumed after them
      __builtin_amdgcn_sched_barrier(0);   // keep the next tile's fragment loads out of this one (register budget)
#pragma unroll
      for (int ks = 0; ks < KX; ++ks) adj[ks] = ld4(wd + (int64_t)j * NW * 16 * d.ldkd + 16 * ks);
      f32x4 acc[PT2], dac[PT2];
#pragma unroll
      for (int t = 0; t < PT2; ++t) acc[t] = dac[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NT1; ++ks)
#pragma unroll
        for (int t = 0; t < PT2; ++t)
          acc[t] = mma4(a3[j][ks], ld4(m2 + (16 * t + l16) * LM + 16 * ks + 4 * g), acc[t]);
#pragma unroll
      for (int ks = 0; ks < KX; ++ks)
#pragma unroll
        for (int t = 0; t < PT2; ++t)
          dac[t] = mma4(adj[ks], ld4(xs + (16 * t + l16) * LX + 16 * ks + 4 * g), dac[t]);
#pragma unroll
      for (int t = 0; t < PT2; ++t) {
        float4 v;
        v.x = fmaxf(acc[t][0] * s3[c0] + t3[c0] + dac[t][0] * sdv[c0] + tdv[c0], 0.f);
        v.y = fmaxf(acc[t][1] * s3[c0 + 1] + t3[c0 + 1] + dac[t][1] * sdv[c0 + 1] + tdv[c0 + 1], 0.f);
        v.z = fmaxf(acc[t][2] * s3[c0 + 2] + t3[c0 + 2] + dac[t][2] * sdv[c0 + 2] + tdv[c0 + 2], 0.f);
        v.w = fmaxf(acc[t][3] * s3[c0 + 3] + t3[c0 + 3] + dac[t][3] * sdv[c0 + 3] + tdv[c0 + 3], 0.f);
        *reinterpret_cast<float4*>(yo + (int64_t)(16 * t + l16) * CO + c0) = v;
      }
    }
    __syncthreads();   // m1 / m2 / xs are rewritten by the next image
  }
}

static int launch3_ds(DArgs d, int C, hipStream_t stream) {
  const size_t smem = (size_t)Geo3D::FLOATS * 4;
  if (smem > 160 * 1024) return -5;
  const int per_model = std::max(1, std::min(d.b.N, (512 + C - 1) / C));
  d.b.units_per_wg = (d.b.N + per_model - 1) / per_model;
  const int gx = (d.b.N + d.b.units_per_wg - 1) / d.b.units_per_wg;
  (void)hipFuncSetAttribute((const void*)bneck3_ds_eval_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(bneck3_ds_eval_kernel, dim3(gx, C), dim3(256), smem, stream, d);
  return (int)hipGetLastError();
}

// ---- stem: NCHW image → 3×3 conv (≤ 4 input channels, 16 outputs) → BN → ReLU → NHWC ----
// Replaces the layout pass, the stem conv (a 16-output GEMM that cannot fill a tile) and the BN/ReLU pass of the
// training path with one memory-bound kernel. A workgroup takes a band of 8 rows of one 32-wide image: the input
// rows (+1 halo row above and below, zero columns left and right) are staged in LDS as [row][col][4 channels];
// MFMA K-step t is tap t (lane group g = input channel g, the 4th channel zero), so each 16-pixel × 16-channel
// tile is 9 MFMAs, four tiles per wave interleaved.
__global__ __launch_bounds__(256) void stem_eval_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                        const float* __restrict__ wpk, int64_t wpk_ld, int64_t off,
                                                        int ldk, int cin_pad, const float* __restrict__ s,
                                                        const float* __restrict__ t, int N, int H, int cin) {
  constexpr int W = 32, R = 8, TW = W + 2, CO = 16, PT = R * W / 16 / 4;   // 4 pixel tiles a wave
  __shared__ __attribute__((aligned(16))) float xs[(R + 2) * TW * 4];
  const int c = blockIdx.y;
  const int bands = H / R;
  const int n = blockIdx.x / bands, r0 = (blockIdx.x - n * bands) * R;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const float* xi = x + ((int64_t)c * N + n) * cin * H * W;
  for (int i = tid; i < (R + 2) * TW * 4; i += 256) {
    const int ch = i & 3, col = (i >> 2) % TW - 1, row = r0 - 1 + (i >> 2) / TW;
    xs[i] = (ch < cin && col >= 0 && col < W && row >= 0 && row < H) ? xi[((int64_t)ch * H + row) * W + col] : 0.f;
  }
  float a[9];
  const float* wp = wpk + (int64_t)c * wpk_ld + off + (int64_t)l16 * ldk + g;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) a[tap] = g < cin ? wp[tap * cin_pad] : 0.f;
  __syncthreads();
  f32x4 acc[PT];
#pragma unroll
  for (int q = 0; q < PT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int p = (wid * PT + q) * 16 + l16, pr = p / W, pc = p % W;
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tap], xs[((pr + kh) * TW + pc + kw) * 4 + g], acc[q], 0, 0, 0);
    }
  }
  const float* sv = s + (int64_t)c * CO + 4 * g;
  const float* tv = t + (int64_t)c * CO + 4 * g;
  float* yo = out + (((int64_t)c * N + n) * H + r0) * W * CO + 4 * g;
#pragma unroll
  for (int q = 0; q < PT; ++q) {
    const int p = (wid * PT + q) * 16 + l16;
    float4 v;
    v.x = fmaxf(acc[q][0] * sv[0] + tv[0], 0.f);
    v.y = fmaxf(acc[q][1] * sv[1] + tv[1], 0.f);
    v.z = fmaxf(acc[q][2] * sv[2] + tv[2], 0.f);
    v.w = fmaxf(acc[q][3] * sv[3] + tv[3], 0.f);
    *reinterpret_cast<float4*>(yo + (int64_t)p * CO) = v;
  }
}

}  // namespace infer

// y = relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1(x)))))))) + x) for a stride-1, downsample-free bottleneck of
// C models at once; mid width cm ∈ {16, 32, 64} at hw = 32 / 16 / 8 (the ResNet-56/110 CIFAR stages 1-3). pool
// (cm 64 only; else null): write the global average pool of y [C][N][4·cm] instead of y. Returns -2 for a geometry
// without an instantiation (the caller keeps the unfused forward).
FA_EXPORT int fa_bneck_eval_f32(const float* x, float* out, const float* wpk, int64_t wpk_ld, int64_t off1, int ldk1,
                                int64_t off2, int ldk2, int64_t off3, int ldk3, const float* s1, const float* t1,
                                const float* s2, const float* t2, const float* s3, const float* t3, int C, int N, int H,
                                int W, int cm, float* pool, hipStream_t stream) {
  if (C <= 0 || N <= 0 || H != W || C > 65535) return (int)hipErrorInvalidValue;
  infer::BArgs a = {x, out, wpk, wpk_ld, off1, off2, off3, ldk1, ldk2, ldk3, s1, t1, s2, t2, s3, t3, N, 1, pool};
  if (pool && !(cm == 64 && H == 8 && ((off1 | off2 | off3 | ldk1 | ldk2 | ldk3 | wpk_ld) & 3) == 0 &&
                (reinterpret_cast<uintptr_t>(wpk) & 15) == 0))
    return -2;   // the pooled epilogue exists in the stage-3 kernel only
  // FEDML_AMD_BNECK_EVAL_VARIANT (A/B of the tilings; ms per 128-model × 64-image ResNet-56 forward on MI355X,
  // profiles/r6_fused_eval_variants.txt): 0 = LDS-resident weights, 4 waves, R = 8 (27.9); 1 = 8 waves, R = 16 / 8
  // (26.4); 2 = 8 waves, R = 8 / 16 (26.0); 3 = register-resident weights, R = 16 (25.3); 4 = same, R = 8 (25.4);
  // 5 (default) = 3 with the stage-1 input band staged in LDS one unit ahead (24.4); 6 = 4-wave workgroups, R = 4
  // band (25.6); 7 = three-stage unit pipeline, one barrier per unit (26.5)
  static const int variant = [] {
    const char* e = getenv("FEDML_AMD_BNECK_EVAL_VARIANT");
    return e ? atoi(e) : 5;
  }();
  if (variant >= 3 && ((off1 | off2 | off3 | ldk1 | ldk2 | ldk3 | wpk_ld) & 3) == 0 &&
      (reinterpret_cast<uintptr_t>(wpk) & 15) == 0) {   // float4 weight-fragment loads
    if (cm == 16 && H == 32) {
      if (variant == 3) return infer::launch_rw<16, 32, 16, false, false, 8>(a, C, stream);
      if (variant == 4) return infer::launch_rw<16, 32, 8, false, false, 8>(a, C, stream);
      if (variant == 6) return infer::launch_rw<16, 32, 4, true, false, 4>(a, C, stream);
      if (variant == 7) return infer::launch_rw<16, 32, 8, false, true, 8>(a, C, stream);
      if (variant == 9) return infer::launch_rw<16, 32, 8, false, false, 4>(a, C, stream);
      if (variant == 11) return infer::launch_rw<16, 32, 8, true, false, 4, 4>(a, C, stream);
      if (variant == 12) return infer::launch_rw<16, 32, 8, false, false, 4, 4>(a, C, stream);
      return infer::launch_rw<16, 32, 8, true, false, 8>(a, C, stream);
    }
    if (cm == 64 && H == 8 && variant != 8) return infer::launch3<64>(a, C, stream);
    if (cm == 32 && H == 16) {
      if (variant == 4) return infer::launch_rw<32, 16, 8, false, false, 8>(a, C, stream);
      if (variant == 10) return infer::launch_rw<32, 16, 16, false, false, 8, 4>(a, C, stream);
      if (variant == 6 || variant == 7) return infer::launch_rw<32, 16, 8, false, true, 8>(a, C, stream);
      return infer::launch_rw<32, 16, 16, false, false, 8>(a, C, stream);
    }
  }
  if (cm == 16 && H == 32) {
    if (variant == 0) return infer::launch<16, 32, 8, 4>(a, C, stream);
    if (variant == 2) return infer::launch<16, 32, 8, 8>(a, C, stream);
    return infer::launch<16, 32, 16, 8>(a, C, stream);
  }
  if (cm == 32 && H == 16) {
    if (variant == 0) return infer::launch<32, 16, 8, 4>(a, C, stream);
    if (variant == 2) return infer::launch<32, 16, 16, 8>(a, C, stream);
    return infer::launch<32, 16, 8, 8>(a, C, stream);
  }
  return -2;
}

// The stage-entry bottleneck (projection shortcut, stride on the 3×3) of C models at once: x [C][N][H][W][cx] →
// out [C][N][H/stride][W/stride][4·cm]. Instantiated for the CIFAR ResNet-56/110 stage-1 (cx 16, cm 16, 32², stride
// 1), stage-2 (cx 64, cm 32, 32², stride 2) and stage-3 (cx 128, cm 64, 16², stride 2) entries; -2 for any other
// geometry (the caller keeps the unfused forward).
FA_EXPORT int fa_bneck_ds_eval_f32(const float* x, float* out, const float* wpk, int64_t wpk_ld, int64_t off1, int ldk1,
                                   int64_t off2, int ldk2, int64_t off3, int ldk3, int64_t offd, int ldkd,
                                   const float* s1, const float* t1, const float* s2, const float* t2, const float* s3,
                                   const float* t3, const float* sd, const float* td, int C, int N, int H, int W,
                                   int cx, int cm, int stride, hipStream_t stream) {
  if (C <= 0 || N <= 0 || H != W || C > 65535) return (int)hipErrorInvalidValue;
  if (((off1 | off2 | off3 | offd | ldk1 | ldk2 | ldk3 | ldkd | wpk_ld) & 3) != 0 ||
      (reinterpret_cast<uintptr_t>(wpk) & 15) != 0)
    return -2;
  infer::DArgs d = {{x, out, wpk, wpk_ld, off1, off2, off3, ldk1, ldk2, ldk3, s1, t1, s2, t2, s3, t3, N, 1, nullptr},
                    offd, ldkd, sd, td};
  if (cx == 16 && cm == 16 && H == 32 && stride == 1) return infer::launch_ds<16, 16, 32, 1, 8>(d, C, stream);
  if (cx == 64 && cm == 32 && H == 32 && stride == 2) return infer::launch_ds<64, 32, 32, 2, 8>(d, C, stream);
  if (cx == 128 && cm == 64 && H == 16 && stride == 2) return infer::launch3_ds(d, C, stream);
  return -2;
}

// relu(bn(conv3×3(x))) of the CIFAR stem for C models at once: x [C][N][cin][H][32] fp32 (NCHW, cin ≤ 4) →
// out [C][N][H][32][16] (NHWC), BN folded (s, t [C][16]); weights from the packed forward layout (k = tap·cin_pad +
// ci). -2 for any other geometry (the caller keeps the layout pass + conv + block-output path).
FA_EXPORT int fa_stem_eval_f32(const float* x, float* out, const float* wpk, int64_t wpk_ld, int64_t off, int ldk,
                               int cin_pad, const float* s, const float* t, int C, int N, int cin, int H, int W,
                               int cout, hipStream_t stream) {
  if (C <= 0 || N <= 0 || C > 65535) return (int)hipErrorInvalidValue;
  if (W != 32 || H % 8 != 0 || cin > 4 || cin < 1 || cout != 16 || cin_pad < cin) return -2;
  hipLaunchKernelGGL(infer::stem_eval_kernel, dim3(N * (H / 8), C), dim3(256), 0, stream, x, out, wpk, wpk_ld, off,
                     ldk, cin_pad, s, t, N, H, cin);
  return (int)hipGetLastError();
}
