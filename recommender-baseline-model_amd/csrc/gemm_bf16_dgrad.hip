// bf16 GEMM, input-gradient orientation dX = dY . W (B operand k-major, read with
// ds_read_b64_tr_b16), all hot-path epilogue classes (gemm_bf16_impl.h).
#include "gemm_bf16_impl.h"

namespace gbf {
hipError_t launch_dgrad(GemmArgs& a, hipStream_t s) { return launch_classes<false, true>(a, s); }
}  // namespace gbf
