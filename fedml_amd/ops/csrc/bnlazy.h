// Deferred ("lazy") BatchNorm finalisation for the native client-batched ResNet step.
//
// The explicit path runs one tiny kernel per BatchNorm and direction (bn_fwd_finalize / bn_bwd_finalize in
// bn_kernels.hip) between a statistics producer and its consumer: 2 × 58 launches per ResNet-56 step, each a
// few µs of kernel plus a dependent-launch boundary — at the 13-client share of an 8-GPU run that is ~7 % of the
// step. Here the FIRST consumer of a BatchNorm's folded vectors computes them itself, per workgroup, in its
// prologue, from the finished statistics (they are complete: the producer kernel has ended), with exactly the
// explicit kernel's arithmetic (same bits). One designated workgroup per client (the consumer's first
// pixel-chunk / output-slice workgroup of that client, passed as `writer`) also writes everything the explicit
// kernel writes — the folded rows read by the later consumers, running statistics, pivot, num_batches_tracked
// (forward) or dγ/dβ into the gradient arena (backward) — so the rest of the step is unchanged. No in-launch
// hand-off: nothing another workgroup of the SAME kernel reads is written.
//
// The host selects the descriptor for a consumer launch with fa_set_lazy (csrc/det_kernels.hip): the launcher
// takes it (fa_take_lazy) and clears it, so it never leaks into another launch. Deterministic mode keeps the
// explicit path (its statistics live in fixed-point shadows until a flush).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct BnLazy {
  int kind;                 // 0: forward (scale, shift) | 1: backward (α, β, γc)
  int Ch, NS, q_gy, hw, update_running;
  float n, momentum, eps;
  const float* stats;       // fwd [C][Ch][2] (Σy, Σy²) | bwd [C][Ch][NS] (Σg at 0, Σg·y at q_gy)
  float* arena;             // parameter arena (γ, β, running statistics)
  float* garena;            // gradient arena (bwd: dγ, dβ)
  int64_t ldw, off_gamma, off_beta, off_rm, off_rv, off_nbt;
  const float* active;      // [C] (fwd running-statistics update) or null
  const int* nimg;          // [C] valid images per client or null
  float* r0;                // fwd: scale | bwd: α
  float* r1;                // fwd: shift | bwd: β
  float* r2;                // fwd: mean  | bwd: γc
  float* r3;                // fwd: rstd
  float* pivot;             // fwd: [C][Ch] in/out (null: none)
  const float* mean_in;     // bwd: forward mean / rstd rows
  const float* rstd_in;
};

extern "C" const BnLazy* fa_take_lazy(int slot);   // host side: the descriptor set for this launch (or null)

// The folding arithmetic shared by the explicit finalize kernels (bn_kernels.hip) and the deferred path, written
// with explicitly rounded operations so that no FMA contraction can differ between the kernels it is inlined
// into: both paths produce the same bits.
struct BnFwdFold {
  float mean, var, rstd, scale, shift;
};
__device__ __forceinline__ BnFwdFold bn_fold_fwd(float s1, float s2, float n, float eps, float g, float b) {
  BnFwdFold f;
  f.mean = __fdiv_rn(s1, n);
  f.var = fmaxf(__fsub_rn(__fdiv_rn(s2, n), __fmul_rn(f.mean, f.mean)), 0.f);
  f.rstd = rsqrtf(__fadd_rn(f.var, eps));
  f.scale = __fmul_rn(g, f.rstd);
  f.shift = __fsub_rn(b, __fmul_rn(__fmul_rn(f.mean, g), f.rstd));
  return f;
}
struct BnBwdFold {
  float dgamma, dbeta, a, b, c;
};
__device__ __forceinline__ BnBwdFold bn_fold_bwd(float sg, float sgy, float mu, float r, float g, float n) {
  BnBwdFold f;
  f.dbeta = sg;
  f.dgamma = __fmul_rn(r, __fsub_rn(sgy, __fmul_rn(mu, sg)));
  f.a = __fmul_rn(g, r);
  f.b = __fdiv_rn(__fmul_rn(__fmul_rn(__fmul_rn(-g, r), r), f.dgamma), n);
  f.c = __fsub_rn(__fdiv_rn(__fmul_rn(-f.a, f.dbeta), n), __fmul_rn(f.b, mu));
  return f;
}
__device__ __forceinline__ float bn_running_update(float old, float mom, float v) {
  return __fadd_rn(__fmul_rn(__fsub_rn(1.f, mom), old), __fmul_rn(mom, v));
}
__device__ __forceinline__ float bn_unbiased(float var, float n) {
  return __fdiv_rn(__fmul_rn(var, n), fmaxf(__fsub_rn(n, 1.f), 1.f));
}

// forward: (scale, shift) of client c, channel ch — bn_fwd_finalize_kernel's arithmetic
__device__ __forceinline__ void bn_lazy_fwd(const BnLazy* L, int c, int ch, bool writer, float& s_out, float& t_out) {
  float n = L->n;
  if (L->nimg) n = (float)L->nimg[c] * (float)L->hw;
  if (n <= 0.f) {            // client without data this step: nothing to normalise (its kernels exit early)
    s_out = 0.f;
    t_out = 0.f;
    return;
  }
  const int Ch = L->Ch;
  float* pa = L->arena + (int64_t)c * L->ldw;
  const int64_t v = (int64_t)c * Ch + ch;
  const float g = L->off_gamma >= 0 ? pa[L->off_gamma + ch] : 1.f;
  const float b = L->off_beta >= 0 ? pa[L->off_beta + ch] : 0.f;
  const BnFwdFold f = bn_fold_fwd(L->stats[v * 2 + 0], L->stats[v * 2 + 1], n, L->eps, g, b);
  s_out = f.scale;
  t_out = f.shift;
  if (!writer) return;
  const float k = L->pivot ? L->pivot[v] : 0.f;
  const float true_mean = __fadd_rn(f.mean, k);
  L->r0[v] = s_out;
  L->r1[v] = t_out;
  L->r2[v] = f.mean;
  L->r3[v] = f.rstd;
  const bool on = L->active ? L->active[c] > 0.f : true;
  if (L->pivot && on) L->pivot[v] = true_mean;
  if (L->update_running && on) {
    const float mom = L->momentum;
    if (L->off_rm >= 0) pa[L->off_rm + ch] = bn_running_update(pa[L->off_rm + ch], mom, true_mean);
    if (L->off_rv >= 0) pa[L->off_rv + ch] = bn_running_update(pa[L->off_rv + ch], mom, bn_unbiased(f.var, n));
    if (L->off_nbt >= 0 && ch == 0) pa[L->off_nbt] += 1.f;
  }
}

// backward: (α, β, γc) of dy = α·g + β·y + γc — bn_bwd_finalize_kernel's arithmetic
__device__ __forceinline__ void bn_lazy_bwd(const BnLazy* L, int c, int ch, bool writer, float& a_out, float& b_out,
                                            float& g_out) {
  float n = L->n;
  if (L->nimg) n = (float)L->nimg[c] * (float)L->hw;
  if (n <= 0.f) {
    a_out = b_out = g_out = 0.f;
    return;
  }
  const int64_t v = (int64_t)c * L->Ch + ch;
  const float g = L->off_gamma >= 0 ? L->arena[(int64_t)c * L->ldw + L->off_gamma + ch] : 1.f;
  const BnBwdFold f = bn_fold_bwd(L->stats[v * L->NS + 0], L->stats[v * L->NS + L->q_gy], L->mean_in[v],
                                  L->rstd_in[v], g, n);
  a_out = f.a;
  b_out = f.b;
  g_out = f.c;
  if (!writer) return;
  if (L->off_gamma >= 0) L->garena[(int64_t)c * L->ldw + L->off_gamma + ch] += f.dgamma;
  if (L->off_beta >= 0) L->garena[(int64_t)c * L->ldw + L->off_beta + ch] += f.dbeta;
  L->r0[v] = a_out;
  L->r1[v] = b_out;
  L->r2[v] = g_out;
}
