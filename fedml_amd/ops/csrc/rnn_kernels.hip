// Client-batched LSTM cell (fp32) for the recurrent FL models (reference `model/nlp/rnn.py:5-86`:
// RNN_OriginalFedAvg, RNN_StackOverFlow), driven by ops/rnn_ops.py.
//
// Layout [C][T][B][X] (client, time, batch, feature). The recurrent GEMMs (h·W_hhᵀ per step, and the
// whole-sequence input projection / weight gradients) run as client-batched library GEMMs; the gate
// nonlinearities, the cell update and their backward are these fused elementwise passes — one launch per
// time step each way instead of ~12 autograd ops, and the gate activations are stored once for backward.
//
// forward   G = x·W_ihᵀ + h·W_hhᵀ + b (gate order i, f, g, o):  i,f,o = σ(·), g = tanh(·)
//           c_t = f·c_{t−1} + i·g,  h_t = o·tanh(c_t);          A_t = (i, f, g, o) kept for backward
// backward  dc = dc_next + dh·o·(1 − tanh²c_t);  dG = (dc·g·i(1−i), dc·c_{t−1}·f(1−f), dc·i·(1−g²),
//           dh·tanh c_t·o(1−o));  dc_next ← dc·f
#include "common.h"

namespace rnn {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// G [C][B][4H] contiguous; c_prev / c_out / h_out / A with client strides (elements) cs_c / cs_h / cs_a
__global__ __launch_bounds__(256) void lstm_cell_fwd_kernel(const float* __restrict__ G,
                                                            const float* __restrict__ c_prev, int64_t cs_cp,
                                                            float* __restrict__ c_out, float* __restrict__ h_out,
                                                            int64_t cs_ch, float* __restrict__ A, int64_t cs_a,
                                                            int C, int B, int H) {
  const int64_t n = (int64_t)C * B * H;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int j = (int)(e % H);
    const int64_t cb = e / H;
    const int b = (int)(cb % B), c = (int)(cb / B);
    const float* g = G + cb * 4 * H;
    const float gi = sigm(g[j]), gf = sigm(g[H + j]), gg = tanhf(g[2 * H + j]), go = sigm(g[3 * H + j]);
    const float cp = c_prev ? c_prev[c * cs_cp + (int64_t)b * H + j] : 0.f;
    const float cn = fmaf(gf, cp, gi * gg);
    const int64_t o = c * cs_ch + (int64_t)b * H + j;
    c_out[o] = cn;
    h_out[o] = go * tanhf(cn);
    float* a = A + c * cs_a + (int64_t)b * 4 * H;
    a[j] = gi;
    a[H + j] = gf;
    a[2 * H + j] = gg;
    a[3 * H + j] = go;
  }
}

// dh [C][B][H] contiguous (output gradient + recurrent term); dc [C][B][H] contiguous, in: dc_next (ignored
// when first), out: dc for step t−1; dG out with client stride cs_a
__global__ __launch_bounds__(256) void lstm_cell_bwd_kernel(const float* __restrict__ dh, float* __restrict__ dc,
                                                            int first, const float* __restrict__ A, int64_t cs_a,
                                                            const float* __restrict__ c_cur,
                                                            const float* __restrict__ c_prev, int64_t cs_c,
                                                            float* __restrict__ dG, int C, int B, int H) {
  const int64_t n = (int64_t)C * B * H;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int j = (int)(e % H);
    const int64_t cb = e / H;
    const int b = (int)(cb % B), c = (int)(cb / B);
    const float* a = A + c * cs_a + (int64_t)b * 4 * H;
    const float gi = a[j], gf = a[H + j], gg = a[2 * H + j], go = a[3 * H + j];
    const int64_t oc = c * cs_c + (int64_t)b * H + j;
    const float tc = tanhf(c_cur[oc]);
    const float cp = c_prev ? c_prev[oc - (int64_t)B * H] : 0.f;   // c_{t−1}: one time slice earlier
    const float g = dh[e];
    const float d = (first ? 0.f : dc[e]) + g * go * (1.f - tc * tc);
    float* o = dG + c * cs_a + (int64_t)b * 4 * H;
    o[j] = d * gg * gi * (1.f - gi);
    o[H + j] = d * cp * gf * (1.f - gf);
    o[2 * H + j] = d * gi * (1.f - gg * gg);
    o[3 * H + j] = g * tc * go * (1.f - go);
    dc[e] = d * gf;
  }
}

}  // namespace rnn

FA_EXPORT int fa_lstm_cell_fwd(const float* G, const float* c_prev, int64_t cs_cp, float* c_out, float* h_out,
                               int64_t cs_ch, float* A, int64_t cs_a, int C, int B, int H, hipStream_t stream) {
  const int64_t n = (int64_t)C * B * H;
  hipLaunchKernelGGL(rnn::lstm_cell_fwd_kernel, dim3(fa_grid(n, 256, 8192)), dim3(256), 0, stream, G, c_prev, cs_cp,
                     c_out, h_out, cs_ch, A, cs_a, C, B, H);
  return (int)hipGetLastError();
}

// c_prev: pointer to c_{t−1}'s slice (same client stride as c_cur) or null at t = 0 (the kernel indexes it as
// c_cur − B·H, so pass the c_cur slice itself as a non-null marker)
FA_EXPORT int fa_lstm_cell_bwd(const float* dh, float* dc, int first, const float* A, int64_t cs_a,
                               const float* c_cur, int has_prev, int64_t cs_c, float* dG, int C, int B, int H,
                               hipStream_t stream) {
  const int64_t n = (int64_t)C * B * H;
  hipLaunchKernelGGL(rnn::lstm_cell_bwd_kernel, dim3(fa_grid(n, 256, 8192)), dim3(256), 0, stream, dh, dc, first, A,
                     cs_a, c_cur, has_prev ? c_cur : nullptr, cs_c, dG, C, B, H);
  return (int)hipGetLastError();
}
