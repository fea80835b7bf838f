// SASRec's parameter-norm regulariser (gfx950).
//
// Replaces BS/trainers/sas.py:51-52:
//     for param in self.model.parameters():
//         loss += self.l2_emb * torch.norm(param)
// i.e. l2 * sum_p ||p||_2 over EVERY parameter tensor, whose gradient is l2 * p / ||p|| (torch's
// norm backward masks a zero norm to a zero gradient).  The parameters live in one flat fp32 buffer
// (flat.py); the caller describes it as chunks of at most RS_L2_CHUNK elements, each tagged with its
// parameter (segment) -- desc (device int64 [nchunk][4]) = {lo, hi, first chunk of the segment, chunks
// of the segment}, segments in order, chunks of one segment consecutive.
//
//   pass 1 (one workgroup per chunk): ws[c] = sum_{i in chunk c} p[i]^2          (fp32, fixed order)
//   pass 2 (one workgroup): per segment ||p_seg|| = sqrt(block sum of its chunk sums) -> ws[nchunk + first
//          chunk]; adds l2 * sum_seg ||p_seg|| (segments in order) to *loss
//   pass 3 (one workgroup per chunk): g[i] += scale * l2 * p[i] / ||p_seg||  (one norm read per chunk)
// ws holds 2 * nchunk floats.
// Deterministic (no atomics).  scale: a device float (the data-parallel step's global count: the
// optimizer divides the summed gradient by it, so the penalty's gradient is pre-multiplied) or null = 1.
#include "common.h"
#include "../../include/recsys_hip.h"

namespace pen {

constexpr int NT = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) s += red[i];
    red[NT / 64] = s;
  }
  __syncthreads();
  s = red[NT / 64];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(NT) void sumsq_kernel(const float* __restrict__ p, const int64_t* __restrict__ desc,
                                                   float* __restrict__ ws) {
  __shared__ float red[NT / 64 + 1];
  const int64_t c = blockIdx.x;
  const int64_t lo = desc[4 * c], hi = desc[4 * c + 1];
  float s = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += NT) {
    const float x = p[i];
    s = __builtin_fmaf(x, x, s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[c] = s;
}

// one workgroup: every segment's norm (its chunk sums reduced by the whole workgroup, fixed order) and the loss
__global__ __launch_bounds__(NT) void norm_kernel(const int64_t* __restrict__ desc, int64_t nchunk,
                                                  float* __restrict__ ws, float l2, float* __restrict__ loss) {
  __shared__ float red[NT / 64 + 1];
  float tot = 0.f;
  for (int64_t c0 = 0; c0 < nchunk;) {
    const int64_t nc = desc[4 * c0 + 3];
    float s = 0.f;
    for (int64_t k = threadIdx.x; k < nc; k += NT) s += ws[c0 + k];
    s = block_sum(s, red);
    const float nrm = sqrtf(s);
    tot += nrm;
    if (threadIdx.x == 0) ws[nchunk + c0] = nrm;
    c0 += nc > 0 ? nc : 1;
  }
  if (threadIdx.x == 0 && loss) *loss += l2 * tot;
}

__global__ __launch_bounds__(NT) void apply_kernel(const float* __restrict__ p, float* __restrict__ g,
                                                   const int64_t* __restrict__ desc, int64_t nchunk,
                                                   const float* __restrict__ ws, float l2,
                                                   const float* __restrict__ scale) {
  const int64_t c = blockIdx.x;
  const int64_t lo = desc[4 * c], hi = desc[4 * c + 1];
  const float nrm = ws[nchunk + desc[4 * c + 2]];
  const float k = nrm > 0.f ? l2 * (scale ? *scale : 1.f) / nrm : 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += NT) g[i] = __builtin_fmaf(k, p[i], g[i]);
}

}  // namespace pen

extern "C" {

int rs_l2_penalty(const float* p, float* g, const int64_t* desc, int64_t nchunk, float l2, const float* scale,
                  float* ws, float* loss, void* stream) {
  if (!p || !desc || !ws || nchunk <= 0 || nchunk > (int64_t)1 << 30) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pen::sumsq_kernel, dim3((unsigned)nchunk), dim3(pen::NT), 0, s, p, desc, ws);
  hipLaunchKernelGGL(pen::norm_kernel, dim3(1), dim3(pen::NT), 0, s, desc, nchunk, ws, l2, loss);
  if (g)
    hipLaunchKernelGGL(pen::apply_kernel, dim3((unsigned)nchunk), dim3(pen::NT), 0, s, p, g, desc, nchunk, ws, l2,
                       scale);
  return (int)hipGetLastError();
}

}  // extern "C"
