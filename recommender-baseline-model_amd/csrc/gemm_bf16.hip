// bf16 GEMM dispatch (gfx950): epilogue-class selection, tile choice, split-K weight-gradient
// launches.  The kernel template is gemm_bf16_impl.h; its forward (A . W^T) and input-gradient
// (dY . W) instantiations are compiled in gemm_bf16_fwd.hip / gemm_bf16_dgrad.hip.
#include "gemm_bf16_impl.h"

namespace gbf {

int epi_class(const GemmArgs& a) {
  const rs_epilogue& e = a.epi;
  if (!a.vec_ok || e.alpha != 1.0f) return EC_GENERIC;
  int ec = 0;
  if (e.bias) ec |= EB;
  if (e.drop_p > 0.f) ec |= ED;
  if (e.resid) ec |= ER;
  if (e.rowmask_ids) ec |= EM;
  if (e.post_drop_p > 0.f) ec |= EP;
  if (e.accumulate) ec |= EA;
  if (a.c_f32) ec |= EF;
  if (e.act < 0 || e.act > 4) return EC_GENERIC;
  if ((e.act == 3 || e.act == 4) && !e.aux) return EC_GENERIC;
  return ec | (e.act << 8);
}

#ifndef GBF_ANY_MIN
#define GBF_ANY_MIN 512
#endif
template <bool AK, bool BK, int EC>
hipError_t launch_any(GemmArgs& a, hipStream_t s) {
  auto blocks = [&](int bm, int bn) { return cdiv(a.M, bm) * cdiv(a.N, bn) * a.split_k; };
  if (blocks(128, 128) >= GBF_ANY_MIN) return launch_cfg<AK, BK, 128, 128, EC>(a, s);
  if (a.N >= 128 && blocks(64, 128) >= 512) return launch_cfg<AK, BK, 64, 128, EC>(a, s);
  if (blocks(128, 64) >= 512) return launch_cfg<AK, BK, 128, 64, EC>(a, s);
  return launch_cfg<AK, BK, 64, 64, EC>(a, s);
}

hipError_t launch_fwd(GemmArgs& a, hipStream_t s);    // gemm_bf16_fwd.hip
hipError_t launch_fwd_ln(GemmArgs& a, hipStream_t s); // gemm_bf16_fwd.hip
hipError_t launch_dgrad(GemmArgs& a, hipStream_t s);  // gemm_bf16_dgrad.hip

}  // namespace gbf

hipError_t gemm_bf16_launch(int ak, int bk, GemmArgs& a, hipStream_t s) {
  using namespace gbf;
  const rs_epilogue& e = a.epi;
  a.vec_ok = !a.slab && (a.ldc % 8 == 0) && ((uintptr_t)a.C % 16 == 0) &&
             (!e.bias || (uintptr_t)e.bias % 16 == 0) &&
             (!e.resid || (e.ldres % 8 == 0 && (uintptr_t)e.resid % 16 == 0)) &&
             (!(e.aux || e.aux_out) || (e.ldaux % 8 == 0 && (uintptr_t)(e.aux ? e.aux : e.aux_out) % 16 == 0));
  if (a.slab) {
    if (ak && bk) return launch_any<true, true, EC_SLAB>(a, s);
    if (!ak && !bk) return launch_any<false, false, EC_SLAB>(a, s);
    if (!ak && bk) return launch_any<false, true, EC_SLAB>(a, s);
    return launch_any<true, false, EC_SLAB>(a, s);
  }
  if (!ak && !bk) return launch_fwd(a, s);
  if (!ak && bk) return launch_dgrad(a, s);
  if (ak && bk) {
    const hipError_t e = dma::launch_wgrad(a, s);
    if (e != hipErrorNotSupported) return e;
    return launch_any<true, true, EC_GENERIC>(a, s);
  }
  return launch_any<true, false, EC_GENERIC>(a, s);
}

extern "C" {

// C = epi(LN(X) W^T), the BERT LayerNorm (variant 1: a_2 (x - mean) / (std_unbiased + eps) + b_2,
// BS/models/bert_modules/utils/layer_norm.py:14-17) formed in the GEMM's prologue -- replaces rs_layernorm_fwd +
// rs_gemm for the sublayers' LN -> Linear pairs (utils/sublayer.py:16-18 into attention/multi_head.py:18-19 and
// utils/feed_forward.py:15-16).  See recsys_hip.h.
int rs_gemm_ln(int64_t M, int64_t N, int64_t K, const void* X, int64_t ldx, const float* gamma, const float* beta,
               float eps, const void* W, int64_t ldw, void* C, int64_t ldc, const rs_epilogue* epi, void* h,
               int64_t ldh, float* mean, float* rinv, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !X || !W || !C || !gamma || !beta || !epi) return RS_ERR_ARG;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = X; a.lda = ldx; a.B = W; a.ldb = ldw; a.C = C; a.ldc = ldc;
  a.c_f32 = 0; a.split_k = 1; a.k_per_split = K;
  a.epi = *epi;
  a.ln.gamma = gamma; a.ln.beta = beta; a.ln.eps = eps; a.ln.h = h; a.ln.ldh = ldh; a.ln.mean = mean;
  a.ln.rinv = rinv;
  const rs_epilogue& e = a.epi;
  a.vec_ok = (a.ldc % 8 == 0) && ((uintptr_t)a.C % 16 == 0) && (!e.bias || (uintptr_t)e.bias % 16 == 0) &&
             (!(e.aux || e.aux_out) || (e.ldaux % 8 == 0 && (uintptr_t)(e.aux ? e.aux : e.aux_out) % 16 == 0));
  const hipError_t r = gbf::launch_fwd_ln(a, (hipStream_t)stream);
  return r == hipErrorNotSupported ? RS_ERR_UNSUPPORTED : (int)r;
}

}  // extern "C"
