// bf16 GEMM, forward orientation C = A . B^T (activations x torch Linear weight [out,in]),
// all hot-path epilogue classes (gemm_bf16_impl.h).
#include "gemm_bf16_impl.h"

namespace gbf {
hipError_t launch_fwd(GemmArgs& a, hipStream_t s) { return launch_classes<false, false>(a, s); }

// LN(X) . W^T with the BERT LayerNorm in the GEMM's prologue (rs_gemm_ln): the classes of the QKV projection (bias)
// and FFN1 (bias + GELU, + dropout in training); hipErrorNotSupported for any other
hipError_t launch_fwd_ln(GemmArgs& a, hipStream_t s) {
  switch (epi_class(a)) {
    case EB: return dma::launch_ln<EB>(a, s);
    case EB | (2 << 8): return dma::launch_ln<EB | (2 << 8)>(a, s);
    case EB | ED | (2 << 8): return dma::launch_ln<EB | ED | (2 << 8)>(a, s);
    default: return hipErrorNotSupported;
  }
}
}  // namespace gbf
