// Deterministic slab reductions (gfx950): the second pass of every two-level
// reduction in the library (split-K weight gradients, bias / LayerNorm-affine
// column sums, the embedding positional gradient).
//
//   out0[i]      (+)= sum_z slab[z*n + i]        for i <  n0
//   out1[i - n0] (+)= sum_z slab[z*n + i]        for n0 <= i < n
//
// Layout of one block: C float4 columns x G split-groups (C*G = 256 threads).
// Each thread sums the splits g, g+G, ... of its float4 column (4 independent
// 16-byte loads in flight per iteration), the G group partials are combined
// through LDS in a fixed order, so the result is bitwise reproducible.  Small
// n (bias / LN vectors of 128-512 floats) gets wide G so that the serial chain
// per thread stays short; large n (d x d weight slabs) gets C = 64.
#include "common.h"
#include "../../include/recsys_hip.h"

template <int C>
__global__ __launch_bounds__(256) void reduce_slabs_v4_kernel(const float4* __restrict__ slab, int splits, int64_t n4,
                                                              int64_t n04, float4* __restrict__ out0,
                                                              float4* __restrict__ out1, int accumulate) {
  constexpr int G = 256 / C;
  const int col = threadIdx.x % C, grp = threadIdx.x / C;
  const int64_t i = (int64_t)blockIdx.x * C + col;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    int z = grp;
    for (; z + 3 * G < splits; z += 4 * G) {
      const float4 a = slab[(int64_t)z * n4 + i];
      const float4 b = slab[(int64_t)(z + G) * n4 + i];
      const float4 c = slab[(int64_t)(z + 2 * G) * n4 + i];
      const float4 d = slab[(int64_t)(z + 3 * G) * n4 + i];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
      s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
      s.x += c.x; s.y += c.y; s.z += c.z; s.w += c.w;
      s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
    }
    for (; z < splits; z += G) {
      const float4 a = slab[(int64_t)z * n4 + i];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  __shared__ float4 red[G][C];
  red[grp][col] = s;
  __syncthreads();
  if (grp == 0 && i < n4) {
    float4 t = red[0][col];
#pragma unroll
    for (int g = 1; g < G; ++g) {
      const float4 u = red[g][col];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    float4* base = i < n04 ? out0 : out1;
    if (base == nullptr) return;
    float4* o = i < n04 ? out0 + i : out1 + (i - n04);
    if (accumulate) {
      const float4 p = *o;
      t.x += p.x; t.y += p.y; t.z += p.z; t.w += p.w;
    }
    *o = t;
  }
}

// scalar fallback (n or n0 not a multiple of 4, or unaligned outputs)
__global__ __launch_bounds__(256) void reduce_slabs_scalar_kernel(const float* __restrict__ slab, int splits, int64_t n,
                                                                  int64_t n0, float* __restrict__ out0,
                                                                  float* __restrict__ out1, int accumulate) {
  constexpr int C = 64, G = 4;
  const int col = threadIdx.x % C, grp = threadIdx.x / C;
  const int64_t i = (int64_t)blockIdx.x * C + col;
  float s = 0.f;
  if (i < n) {
    // eight splits' loads in flight, summed in the same order (z = grp, grp + G, ...): the same bits as one at a time
    int z = grp;
    for (; z + 7 * G < splits; z += 8 * G) {
      float u[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = slab[(int64_t)(z + t * G) * n + i];
#pragma unroll
      for (int t = 0; t < 8; ++t) s += u[t];
    }
    for (; z < splits; z += G) s += slab[(int64_t)z * n + i];
  }
  __shared__ float red[G][C];
  red[grp][col] = s;
  __syncthreads();
  if (grp == 0 && i < n) {
    const float t = red[0][col] + red[1][col] + red[2][col] + red[3][col];
    float* o = i < n0 ? (out0 ? out0 + i : nullptr) : (out1 ? out1 + (i - n0) : nullptr);
    if (o) *o = accumulate ? *o + t : t;
  }
}

hipError_t launch_reduce_slabs(const float* slab, int splits, int64_t n, int64_t n0, float* out0, float* out1,
                               int accumulate, hipStream_t s) {
  const bool vec = (n % 4 == 0) && (n0 % 4 == 0) && ((uintptr_t)slab % 16 == 0) &&
                   ((uintptr_t)out0 % 16 == 0) && ((uintptr_t)out1 % 16 == 0);
  if (!vec) {
    hipLaunchKernelGGL(reduce_slabs_scalar_kernel, dim3((unsigned)cdiv(n, 64)), dim3(256), 0, s, slab, splits, n, n0,
                       out0, out1, accumulate);
    return hipGetLastError();
  }
  const int64_t n4 = n / 4, n04 = n0 / 4;
  const float4* s4 = reinterpret_cast<const float4*>(slab);
  float4* o0 = reinterpret_cast<float4*>(out0);
  float4* o1 = reinterpret_cast<float4*>(out1);
  if (n4 <= 16)
    hipLaunchKernelGGL((reduce_slabs_v4_kernel<16>), dim3((unsigned)cdiv(n4, 16)), dim3(256), 0, s, s4, splits, n4,
                       n04, o0, o1, accumulate);
  else if (n4 <= 32 * 8)
    hipLaunchKernelGGL((reduce_slabs_v4_kernel<32>), dim3((unsigned)cdiv(n4, 32)), dim3(256), 0, s, s4, splits, n4,
                       n04, o0, o1, accumulate);
  else
    hipLaunchKernelGGL((reduce_slabs_v4_kernel<64>), dim3((unsigned)cdiv(n4, 64)), dim3(256), 0, s, s4, splits, n4,
                       n04, o0, o1, accumulate);
  return hipGetLastError();
}

extern "C" {

int rs_reduce_slabs(const float* slab, int splits, int64_t n, float* out, int accumulate, void* stream) {
  if (n <= 0 || splits < 1 || !slab || !out) return RS_ERR_ARG;
  return (int)launch_reduce_slabs(slab, splits, n, n, out, nullptr, accumulate, (hipStream_t)stream);
}

int rs_reduce_slabs2(const float* slab, int splits, int64_t n0, float* out0, int64_t n1, float* out1, int accumulate,
                     void* stream) {
  if (n0 < 0 || n1 < 0 || n0 + n1 <= 0 || splits < 1 || !slab) return RS_ERR_ARG;
  return (int)launch_reduce_slabs(slab, splits, n0 + n1, n0, out0, out1, accumulate, (hipStream_t)stream);
}

}  // extern "C"
