// bf16 GEMM, forward orientation C = A . B^T (activations x torch Linear weight [out,in]),
// all hot-path epilogue classes (gemm_bf16_impl.h).
#include "gemm_bf16_impl.h"

namespace gbf {
hipError_t launch_fwd(GemmArgs& a, hipStream_t s) { return launch_classes<false, false>(a, s); }
}  // namespace gbf
