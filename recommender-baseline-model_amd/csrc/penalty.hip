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
//   pass 2 (one workgroup per chunk): ||p_seg|| = sqrt(sum of the segment's ws, in chunk order);
//          g[i] += scale * l2 * p[i] / ||p_seg||; workgroup 0 also adds l2 * sum_seg ||p_seg|| to *loss.
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

__device__ __forceinline__ float seg_norm(const int64_t* desc, const float* ws, int64_t c) {
  const int64_t c0 = desc[4 * c + 2], nc = desc[4 * c + 3];
  float s = 0.f;
  for (int64_t k = 0; k < nc; ++k) s += ws[c0 + k];
  return sqrtf(s);
}

__global__ __launch_bounds__(NT) void apply_kernel(const float* __restrict__ p, float* __restrict__ g,
                                                   const int64_t* __restrict__ desc, int64_t nchunk,
                                                   const float* __restrict__ ws, float l2,
                                                   const float* __restrict__ scale, float* __restrict__ loss) {
  __shared__ float red[NT / 64 + 1];
  const int64_t c = blockIdx.x;
  const int64_t lo = desc[4 * c], hi = desc[4 * c + 1];
  const float nrm = seg_norm(desc, ws, c);
  const float k = nrm > 0.f ? l2 * (scale ? *scale : 1.f) / nrm : 0.f;
  if (g)
    for (int64_t i = lo + threadIdx.x; i < hi; i += NT) g[i] = __builtin_fmaf(k, p[i], g[i]);
  if (c == 0 && loss) {
    // sum of the segment norms, segments in order (each counted at its first chunk)
    float s = 0.f;
    for (int64_t j = threadIdx.x; j < nchunk; j += NT)
      if (desc[4 * j + 2] == j) s += seg_norm(desc, ws, j);
    s = block_sum(s, red);
    if (threadIdx.x == 0) *loss += l2 * s;
  }
}

}  // namespace pen

extern "C" {

int rs_l2_penalty(const float* p, float* g, const int64_t* desc, int64_t nchunk, float l2, const float* scale,
                  float* ws, float* loss, void* stream) {
  if (!p || !desc || !ws || nchunk <= 0 || nchunk > (int64_t)1 << 30) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pen::sumsq_kernel, dim3((unsigned)nchunk), dim3(pen::NT), 0, s, p, desc, ws);
  hipLaunchKernelGGL(pen::apply_kernel, dim3((unsigned)nchunk), dim3(pen::NT), 0, s, p, g, desc, nchunk, ws, l2,
                     scale, loss);
  return (int)hipGetLastError();
}

}  // extern "C"
