// Union-of-touched-rows exchange of an embedding-table gradient (data parallel).
//
// A step touches few rows of a large table (BERT at 1M items: B*T = 12,800 token rows per rank of
// 1,000,002), and every other row of the table's gradient is zero on every rank.  Instead of an
// all-reduce of the dense table gradient (1 GB at cfg5), the ranks all-gather their batch ids, build the
// same sorted union of touched rows on every rank, pack those rows of their gradient into a compact
// buffer, all-reduce that, and unpack it.  Rows outside the union stay zero, as the dense all-reduce would
// leave them.  Everything here is graph-capturable (no host sync): the union size stays on the device and
// the compact buffer has a fixed capacity (the gathered id count, capped at the table size).
//
//   rs_touched_rows : flags[v] = v occurs in ids; index[v] = rank of v among the flagged rows (ascending
//                     row order) or -1; *count = number of flagged rows.  Two-level exclusive scan.
//   rs_rows_pack    : compact[index[v]] = src[v] for flagged v; compact rows [count, cap) zeroed.
//   rs_rows_unpack  : dst[v] = compact[index[v]] for flagged v.
#include "common.h"
#include "../../include/recsys_hip.h"

namespace sr {

constexpr int NT = 256;
constexpr int PER = 8;                // flags per thread
constexpr int CH = NT * PER;          // flags per scan block

__global__ __launch_bounds__(NT) void zero_kernel(int32_t* __restrict__ flags, int64_t rows) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < rows; i += (int64_t)gridDim.x * NT) flags[i] = 0;
}

__global__ __launch_bounds__(NT) void mark_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t rows,
                                                  int32_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t v = ids[i];
    if (v >= 0 && v < rows) flags[v] = 1;      // benign race: every writer stores 1
  }
}

// block-wide exclusive scan of one value per thread; returns the exclusive prefix, *total = block sum
__device__ __forceinline__ int32_t block_scan(int32_t x, int32_t* sh, int32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int32_t v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) sh[w] = v;
  __syncthreads();
  int32_t wofs = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    if (k < w) wofs += sh[k];
    tot += sh[k];
  }
  __syncthreads();
  *total = tot;
  return wofs + v - x;
}

// per-block flag counts
__global__ __launch_bounds__(NT) void count_kernel(const int32_t* __restrict__ flags, int64_t rows,
                                                   int32_t* __restrict__ bsum) {
  __shared__ int32_t sh[NT / 64];
  const int64_t base = (int64_t)blockIdx.x * CH + threadIdx.x * PER;
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) c += (base + k < rows) ? flags[base + k] : 0;
  int32_t tot;
  block_scan(c, sh, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// exclusive scan of the block counts (one workgroup, any number of blocks) -> bofs, *count
__global__ __launch_bounds__(NT) void scan_blocks_kernel(const int32_t* __restrict__ bsum, int64_t nb,
                                                         int32_t* __restrict__ bofs, int32_t* __restrict__ count) {
  __shared__ int32_t sh[NT / 64];
  int32_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += NT) {
    const int64_t b = b0 + threadIdx.x;
    const int32_t x = b < nb ? bsum[b] : 0;
    int32_t tot;
    const int32_t ex = block_scan(x, sh, &tot);
    if (b < nb) bofs[b] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *count = carry;
}

__global__ __launch_bounds__(NT) void index_kernel(const int32_t* __restrict__ flags, int64_t rows,
                                                   const int32_t* __restrict__ bofs, int32_t* __restrict__ index) {
  __shared__ int32_t sh[NT / 64];
  const int64_t base = (int64_t)blockIdx.x * CH + threadIdx.x * PER;
  int32_t f[PER], c = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    f[k] = (base + k < rows) ? flags[base + k] : 0;
    c += f[k];
  }
  int32_t tot;
  int32_t pos = bofs[blockIdx.x] + block_scan(c, sh, &tot);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (base + k < rows) index[base + k] = f[k] ? pos : -1;
    pos += f[k];
  }
}

// one wave per table row (d fp32, 16-byte chunks); pack: src rows -> compact, unpack: compact -> dst rows
template <bool PACK>
__global__ __launch_bounds__(NT) void move_kernel(float* __restrict__ table, int64_t rows, int64_t d,
                                                  const int32_t* __restrict__ index, float* __restrict__ compact) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (NT / 64);
  for (int64_t v = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6); v < rows; v += nw) {
    const int32_t c = index[v];
    if (c < 0) continue;
    float4* t = reinterpret_cast<float4*>(table + v * d);
    float4* k = reinterpret_cast<float4*>(compact + (int64_t)c * d);
    for (int64_t j = lane; j < d / 4; j += 64) {
      if (PACK) k[j] = t[j];
      else t[j] = k[j];
    }
  }
}

// compact rows [*count, cap) = 0
__global__ __launch_bounds__(NT) void zero_tail_kernel(float* __restrict__ compact, int64_t cap, int64_t d,
                                                       const int32_t* __restrict__ count) {
  const int64_t lo = (int64_t)(*count) * d, hi = cap * d;
  for (int64_t i = lo + (int64_t)blockIdx.x * NT + threadIdx.x; i < hi; i += (int64_t)gridDim.x * NT) compact[i] = 0.f;
}

static unsigned grid_rows(int64_t work, int64_t per_block) {
  const int64_t g = cdiv(work, per_block);
  return (unsigned)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

}  // namespace sr

extern "C" {

int64_t rs_touched_rows_ws_numel(int64_t rows) { return 2 * cdiv(rows, sr::CH); }

int rs_touched_rows(const int64_t* ids, int64_t n, int64_t rows, int32_t* flags, int32_t* index, int32_t* count,
                    int32_t* ws, void* stream) {
  if (n < 0 || rows <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nb = cdiv(rows, sr::CH);
  int32_t* bsum = ws;
  int32_t* bofs = ws + nb;
  hipLaunchKernelGGL(sr::zero_kernel, dim3(sr::grid_rows(rows, sr::NT * 4)), dim3(sr::NT), 0, s, flags, rows);
  if (n > 0)
    hipLaunchKernelGGL(sr::mark_kernel, dim3(sr::grid_rows(n, sr::NT * 4)), dim3(sr::NT), 0, s, ids, n, rows, flags);
  hipLaunchKernelGGL(sr::count_kernel, dim3((unsigned)nb), dim3(sr::NT), 0, s, flags, rows, bsum);
  hipLaunchKernelGGL(sr::scan_blocks_kernel, dim3(1), dim3(sr::NT), 0, s, bsum, nb, bofs, count);
  hipLaunchKernelGGL(sr::index_kernel, dim3((unsigned)nb), dim3(sr::NT), 0, s, flags, rows, bofs, index);
  return (int)hipGetLastError();
}

int rs_rows_pack(const float* src, int64_t rows, int64_t d, const int32_t* index, const int32_t* count,
                 float* compact, int64_t cap, void* stream) {
  if (rows <= 0 || d <= 0 || d % 4 || cap <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sr::zero_tail_kernel, dim3(sr::grid_rows(cap * d, sr::NT * 8)), dim3(sr::NT), 0, s, compact, cap,
                     d, count);
  hipLaunchKernelGGL(sr::move_kernel<true>, dim3(sr::grid_rows(rows, sr::NT / 64 * 4)), dim3(sr::NT), 0, s,
                     const_cast<float*>(src), rows, d, index, compact);
  return (int)hipGetLastError();
}

int rs_rows_unpack(float* dst, int64_t rows, int64_t d, const int32_t* index, const float* compact, void* stream) {
  if (rows <= 0 || d <= 0 || d % 4) return RS_ERR_ARG;
  hipLaunchKernelGGL(sr::move_kernel<false>, dim3(sr::grid_rows(rows, sr::NT / 64 * 4)), dim3(sr::NT), 0,
                     (hipStream_t)stream, dst, rows, d, index, const_cast<float*>(compact));
  return (int)hipGetLastError();
}

}  // extern "C"
