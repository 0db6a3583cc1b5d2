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
// matrices stay in LDS for all the units of that model the workgroup processes.
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

}  // namespace infer

// y = relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1(x)))))))) + x) for a stride-1, downsample-free bottleneck of
// C models at once; mid width cm ∈ {16, 32} at hw = 32 / 16 (the ResNet-56/110 CIFAR stages 1 and 2). Returns -2
// for a geometry without an instantiation (the caller keeps the unfused forward).
FA_EXPORT int fa_bneck_eval_f32(const float* x, float* out, const float* wpk, int64_t wpk_ld, int64_t off1, int ldk1,
                                int64_t off2, int ldk2, int64_t off3, int ldk3, const float* s1, const float* t1,
                                const float* s2, const float* t2, const float* s3, const float* t3, int C, int N, int H,
                                int W, int cm, hipStream_t stream) {
  if (C <= 0 || N <= 0 || H != W || C > 65535) return (int)hipErrorInvalidValue;
  infer::BArgs a = {x, out, wpk, wpk_ld, off1, off2, off3, ldk1, ldk2, ldk3, s1, t1, s2, t2, s3, t3, N, 1};
  // 8 waves per workgroup: two per SIMD share the staged weights (the 32-wide stage's 73 KB of weights leave room
  // for one workgroup per CU), so one wave's LDS / HBM waits overlap the other's MFMAs
  static const int variant = [] {
    const char* e = getenv("FEDML_AMD_BNECK_EVAL_VARIANT");
    return e ? atoi(e) : 1;
  }();
  if (cm == 16 && H == 32)
    return variant == 0 ? infer::launch<16, 32, 8, 4>(a, C, stream) : infer::launch<16, 32, 16, 8>(a, C, stream);
  if (cm == 32 && H == 16)
    return variant == 0 ? infer::launch<32, 16, 8, 4>(a, C, stream) : infer::launch<32, 16, 8, 8>(a, C, stream);
  return -2;
}
