// torch.optim.Adam's per-element update (BS/trainers/base.py:225-228; the single-tensor path of torch/optim/adam.py)
// for the optimizer sweeps (misc.hip): one definition, every fused multiply-add spelled out, so any kernel that
// inlines it produces the same bits.
#pragma once
#include "common.h"

// Bias corrections of step t exactly as torch.optim.Adam forms them: the hyperparameters are Python doubles there,
// bias_correction1 = 1 - beta1 ** step, step_size = lr / bias_correction1, bias_correction2_sqrt = sqrt(1 - beta2 **
// step) in double, each cast to float where it meets the fp32 tensors.  hyper is double[5] for that reason: with fp32
// betas, 1 - 0.999f is 1.3e-5 (relative) off torch's float(1 - 0.999) -- a systematic bias in every v update and in
// sqrt(bc2) that a 1000-step curve amplified.
struct AdamScalars { float step_size, bc2s, gs; };
__device__ __forceinline__ AdamScalars adam_scalars(double t, const double* hyper, const float* divisor) {
  const double lr = hyper[0], b1 = hyper[1], b2 = hyper[2];
  const double bc1 = 1.0 - pow(b1, t), bc2 = 1.0 - pow(b2, t);
  return {(float)(lr / bc1), (float)sqrt(bc2), divisor ? 1.f / divisor[0] : 1.f};
}
// the per-element scalars: float(beta2) (exp_avg_sq.mul_(beta2)), float(1 - beta1) (lerp weight), float(1 - beta2)
// (addcmul value), float(eps), float(weight_decay)
struct AdamElem { float b2, omb1, omb2, eps, wd; };
__device__ __forceinline__ AdamElem adam_elem(const double* hyper) {
  return {(float)hyper[2], (float)(1.0 - hyper[1]), (float)(1.0 - hyper[2]), (float)hyper[3], (float)hyper[4]};
}
// one element: gradient scale (1 / the data-parallel count), weight decay, exp_avg.lerp_(grad, 1-beta1),
// exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2), param.addcdiv_(exp_avg, sqrt(exp_avg_sq) / bc2s + eps, -step_size).
// Every fused multiply-add is spelled out and no other contraction is allowed: the compiler's own contraction
// choices differed between two kernels inlining the same expression (1 ulp in 0.5 % of the parameters; round 6's
// dE GEMM with the update in its epilogue, measured and removed: DESIGN.md §4).
__device__ __forceinline__ void adam_elem_update(float& P, float G, float& Mv, float& Vv, const AdamElem& h,
                                                 float step_size, float bc2s, float gs) {
#pragma clang fp contract(off)
  float gj = gs == 1.f ? G : G * gs;
  if (h.wd != 0.f) gj = __builtin_fmaf(h.wd, P, gj);
  Mv = __builtin_fmaf(h.omb1, gj - Mv, Mv);
  Vv = __builtin_fmaf(h.omb2 * gj, gj, Vv * h.b2);
  const float denom = sqrtf(Vv) / bc2s + h.eps;
  P = __builtin_fmaf(-step_size, Mv / denom, P);
}
