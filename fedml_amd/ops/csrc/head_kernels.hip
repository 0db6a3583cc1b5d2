// Fused classifier head of the client-batched ResNet step (fp32, one 1024-thread workgroup per client):
//
//   Z  = P·Wᵀ + b                        logits            P [N][F] pooled features, W [K][F], b [K] (arena)
//   dl = rs·(softmax(Z) − onehot(y))     CE backward       rs = the row's scale (1/batch, 0 for padding rows)
//   gW += dlᵀ·P,  gb += Σ_n dl,  dP = dl·W                  (gradient arena rows; dP for the pooled backward)
//   loss_c[c] = Σ_n rs·(lse − Z[y])
//
// P and Z/dl stay in LDS across the phases: one launch instead of the library batched GEMMs + the
// separate CE / column-sum / accumulate kernels, no logits or dlogits round trip, and no atomics — every
// reduction runs in a fixed order (bit-reproducible, independent of how many clients share the GPU).
// Reference model: `model/cv/resnet.py:137` (self.fc) + `my_model_trainer_classification.py:52` (CE loss).
#include "common.h"

namespace fch {

constexpr int kThreads = 1024;   // 16 waves: the phases are latency-bound chains of W / LDS reads (one block per
                                 // client: 13 per GPU at the 8-GPU headline share), 4× the 256-thread block's waves

__global__ __launch_bounds__(kThreads) void fc_head_xent_kernel(const float* __restrict__ pooled,
                                                           const float* __restrict__ arena, int64_t lda, int64_t ow,
                                                           int64_t ob, const int64_t* __restrict__ labels,
                                                           const float* __restrict__ row_scale,
                                                           float* __restrict__ garena, int64_t ldg,
                                                           float* __restrict__ dpool, float* __restrict__ loss_c, int N,
                                                           int F, int K) {
  extern __shared__ float4 smem4[];
  float* sm = reinterpret_cast<float*>(smem4);
  const int FP = F + 4;                 // padded row: float4 reads of 64 rows hit distinct bank groups
  float* P = sm;                        // [N][FP]
  float* Z = sm + (size_t)N * FP;       // [N][K]: logits, then dl
  __shared__ float red[kThreads / 64];
  const int c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* Pg = pooled + (int64_t)c * N * F;
  const float* W = arena + (int64_t)c * lda + ow;
  const float* b = arena + (int64_t)c * lda + ob;
  const int F4 = F >> 2;
  for (int i = tid; i < N * F4; i += kThreads) {
    const int n = i / F4, f = (i - n * F4) * 4;
    *reinterpret_cast<float4*>(P + n * FP + f) = *reinterpret_cast<const float4*>(Pg + (int64_t)n * F + f);
  }
  __syncthreads();
  // logits: a thread owns 4 consecutive classes of one row; lanes run over rows (W loads are wave-uniform)
  const int K4 = (K + 3) >> 2;
  for (int i = tid; i < N * K4; i += kThreads) {
    const int kq = i / N, n = i - kq * N, k0 = kq * 4;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    const float* pr = P + n * FP;
    const float* w0 = W + (int64_t)min(k0, K - 1) * F;
    const float* w1 = W + (int64_t)min(k0 + 1, K - 1) * F;
    const float* w2 = W + (int64_t)min(k0 + 2, K - 1) * F;
    const float* w3 = W + (int64_t)min(k0 + 3, K - 1) * F;
    for (int f = 0; f < F; f += 4) {
      const float4 p = *reinterpret_cast<const float4*>(pr + f);
      acc0 = fmaf(p.x, w0[f], acc0); acc0 = fmaf(p.y, w0[f + 1], acc0);
      acc0 = fmaf(p.z, w0[f + 2], acc0); acc0 = fmaf(p.w, w0[f + 3], acc0);
      acc1 = fmaf(p.x, w1[f], acc1); acc1 = fmaf(p.y, w1[f + 1], acc1);
      acc1 = fmaf(p.z, w1[f + 2], acc1); acc1 = fmaf(p.w, w1[f + 3], acc1);
      acc2 = fmaf(p.x, w2[f], acc2); acc2 = fmaf(p.y, w2[f + 1], acc2);
      acc2 = fmaf(p.z, w2[f + 2], acc2); acc2 = fmaf(p.w, w2[f + 3], acc2);
      acc3 = fmaf(p.x, w3[f], acc3); acc3 = fmaf(p.y, w3[f + 1], acc3);
      acc3 = fmaf(p.z, w3[f + 2], acc3); acc3 = fmaf(p.w, w3[f + 3], acc3);
    }
    float* zr = Z + n * K;
    if (k0 < K) zr[k0] = acc0 + b[k0];
    if (k0 + 1 < K) zr[k0 + 1] = acc1 + b[k0 + 1];
    if (k0 + 2 < K) zr[k0 + 2] = acc2 + b[k0 + 2];
    if (k0 + 3 < K) zr[k0 + 3] = acc3 + b[k0 + 3];
  }
  __syncthreads();
  // softmax cross-entropy, one wave per row; Z becomes dl in place
  float lsum = 0.f;
  for (int n = wv; n < N; n += kThreads / 64) {
    float* zr = Z + n * K;
    const float rs = row_scale[(int64_t)c * N + n];
    const int64_t lbl = labels[(int64_t)c * N + n];
    if (rs == 0.f || lbl < 0 || lbl >= K) {      // padding / ignored row: no loss, no gradient
      for (int j = lane; j < K; j += 64) zr[j] = 0.f;
      continue;
    }
    float m = -INFINITY;
    for (int j = lane; j < K; j += 64) m = fmaxf(m, zr[j]);
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < K; j += 64) s += __expf(zr[j] - m);
    s = wave_sum(s);
    const float zl = zr[lbl];
    const float inv = 1.f / s;
    for (int j = lane; j < K; j += 64) zr[j] = rs * (__expf(zr[j] - m) * inv - (j == lbl ? 1.f : 0.f));
    lsum += rs * (m + __logf(s) - zl);
  }
  if (lane == 0) red[wv] = lsum;
  __syncthreads();
  if (tid == 0) {   // fixed order
    float t = 0.f;
    for (int w = 0; w < kThreads / 64; ++w) t += red[w];
    loss_c[c] = t;
  }
  // gW += dlᵀ·P: a thread owns (class k, 4 features); lanes run over features
  float* gW = garena + (int64_t)c * ldg + ow;
  for (int i = tid; i < K * F4; i += kThreads) {
    const int k = i / F4, f = (i - k * F4) * 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int n = 0; n < N; ++n) {
      const float d = Z[n * K + k];
      const float4 p = *reinterpret_cast<const float4*>(P + n * FP + f);
      a0 = fmaf(d, p.x, a0); a1 = fmaf(d, p.y, a1); a2 = fmaf(d, p.z, a2); a3 = fmaf(d, p.w, a3);
    }
    float* g = gW + (int64_t)k * F + f;
    g[0] += a0; g[1] += a1; g[2] += a2; g[3] += a3;
  }
  float* gb = garena + (int64_t)c * ldg + ob;
  for (int k = tid; k < K; k += kThreads) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += Z[n * K + k];
    gb[k] += s;
  }
  // dP = dl·W: a thread owns (row n, 4 features)
  float* dp = dpool + (int64_t)c * N * F;
  for (int i = tid; i < N * F4; i += kThreads) {
    const int n = i / F4, f = (i - n * F4) * 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const float* zr = Z + n * K;
    for (int k = 0; k < K; ++k) {
      const float d = zr[k];
      const float* w = W + (int64_t)k * F + f;
      a0 = fmaf(d, w[0], a0); a1 = fmaf(d, w[1], a1); a2 = fmaf(d, w[2], a2); a3 = fmaf(d, w[3], a3);
    }
    *reinterpret_cast<float4*>(dp + (int64_t)n * F + f) = make_float4(a0, a1, a2, a3);
  }
}

}  // namespace fch

extern "C" size_t fa_fc_head_smem(int N, int F, int K) {
  return ((size_t)N * (F + 4) + (size_t)N * K) * sizeof(float);
}

// pooled [C][N][F] fp32 (16-B aligned, F % 4 == 0); W / b at offsets ow / ob of every arena row (stride lda);
// gradients added at the same offsets of the gradient arena (stride ldg); dpool [C][N][F]; loss_c [C].
// Returns -5 when P and the logits do not fit one workgroup's LDS (the caller keeps the library path).
FA_EXPORT int fa_fc_head_xent_f32(const float* pooled, const float* arena, int64_t lda, int64_t ow, int64_t ob,
                                  const int64_t* labels, const float* row_scale, float* garena, int64_t ldg,
                                  float* dpool, float* loss_c, int C, int N, int F, int K, hipStream_t stream) {
  if (F % 4 != 0 || N <= 0 || K <= 0) return -3;
  const size_t smem = fa_fc_head_smem(N, F, K);
  if (smem > 160 * 1024) return -5;
  if (smem > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)fch::fc_head_xent_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)smem);
  hipLaunchKernelGGL(fch::fc_head_xent_kernel, dim3(C), dim3(fch::kThreads), smem, stream, pooled, arena, lda, ow, ob, labels,
                     row_scale, garena, ldg, dpool, loss_c, N, F, K);
  return (int)hipGetLastError();
}
