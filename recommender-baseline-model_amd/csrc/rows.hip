// Labelled-row compaction for the BERT4Rec loss head (gfx950).
//
// The reference computes the full-vocabulary logits of EVERY position and lets
// CrossEntropyLoss(ignore_index=0) drop the unlabelled ones
// (BS/models/bert.py:16, BS/trainers/bert.py:36-40).  Rows with label 0
// contribute neither loss nor gradient, so the build runs the vocabulary GEMMs
// only on the labelled rows: these kernels build the ordered list of those rows
// on the device (no host sync, graph-capturable), gather their hidden states,
// and scatter the hidden-state gradient back.  The compacted row count stays on
// the device (rows_dev) and bounds the following GEMMs.
#include "common.h"
#include "../../include/recsys_hip.h"

// one 1024-row block per workgroup, no cross-workgroup synchronisation: workgroup b first counts the labelled rows
// before its block (coalesced strided loads, one block reduction), then places its own rows by wave ballots (lane
// prefix = popcount of the lower lanes' bits) and the waves' totals scanned in LDS.  Rows keep their order.  (The
// round-1 form -- ONE 1024-thread workgroup, a contiguous chunk per thread, Hillis-Steele scan -- took 20.7 us at
// cfg3's 12,800 rows on the BERT step's critical path.)
__global__ __launch_bounds__(1024) void compact_kernel(const int64_t* __restrict__ labels, int64_t n,
                                                       int64_t cap, int32_t* __restrict__ idx,
                                                       int32_t* __restrict__ rank, int32_t* __restrict__ count) {
  __shared__ int32_t wb[16], wo[16], wpre[18];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * 1024, r = base + tid;
  const bool lab = r < n && labels[r] != 0;
  int32_t c = 0;
  for (int64_t q = tid; q < base; q += 1024) c += labels[q] != 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  const uint64_t bal = __ballot(lab);
  if (lane == 0) {
    wb[w] = c;
    wo[w] = (int32_t)__popcll(bal);
  }
  __syncthreads();
  if (tid == 0) {
    int32_t before = 0, own = 0;
    for (int k = 0; k < 16; ++k) {
      wpre[k] = own;
      before += wb[k];
      own += wo[k];
    }
    wpre[16] = before;
    wpre[17] = own;
  }
  __syncthreads();
  const int32_t before = wpre[16], own = wpre[17];
  const int32_t pos = before + wpre[w] + (int32_t)__popcll(bal & ((1ull << lane) - 1ull));
  if (r < n) {
    if (lab && pos < cap) {
      idx[pos] = (int32_t)r;
      rank[r] = pos;
    } else {
      rank[r] = -1;
    }
  }
  if (blockIdx.x == gridDim.x - 1) {
    const int64_t total = (int64_t)before + own;
    if (tid == 0) *count = (int32_t)min(total, cap);
    // unused slots of the list point nowhere (never read for real rows: bounded by count)
    for (int64_t i = total + tid; i < cap; i += 1024) idx[i] = -1;
  }
}

// dst[i] = src[idx[i]] for i < count, zero rows for count <= i < cap; lab_out[i] = labels[idx[i]] or 0
template <typename T>
__global__ __launch_bounds__(256) void gather_rows_kernel(const T* __restrict__ src, int64_t lds, int64_t d,
                                                          const int32_t* __restrict__ idx,
                                                          const int32_t* __restrict__ count, int64_t cap,
                                                          T* __restrict__ dst, int64_t ldd,
                                                          const int64_t* __restrict__ labels,
                                                          int64_t* __restrict__ lab_out) {
  constexpr int V = Vec<T>::N;
  const int64_t cpr = d / V;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= cap * cpr) return;
  const int64_t r = i / cpr, c = (i % cpr) * V;
  const int32_t n = *count;
  float v[V];
  if (r < n) {
    const int64_t s = idx[r];
    load_chunk<T>(v, src + s * lds + c);
    if (c == 0 && lab_out) lab_out[r] = labels[s];
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = 0.f;
    if (c == 0 && lab_out) lab_out[r] = 0;
  }
  store_chunk<T>(dst + r * ldd + c, v);
}

// dst[r] = rank[r] >= 0 ? src[rank[r]] : 0   over all n rows
template <typename T>
__global__ __launch_bounds__(256) void scatter_rows_kernel(const T* __restrict__ src, int64_t lds, int64_t d,
                                                           const int32_t* __restrict__ rank, int64_t n,
                                                           T* __restrict__ dst, int64_t ldd) {
  constexpr int V = Vec<T>::N;
  const int64_t cpr = d / V;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n * cpr) return;
  const int64_t r = i / cpr, c = (i % cpr) * V;
  const int32_t k = rank[r];
  float v[V];
  if (k >= 0) load_chunk<T>(v, src + (int64_t)k * lds + c);
  else {
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = 0.f;
  }
  store_chunk<T>(dst + r * ldd + c, v);
}

// dst[r] = rank[r] >= 0 ? T(sum_z slab[z][rank[r]]) : 0 over all n rows: the split-K reduction, the cast
// and the scatter of a compacted-row GEMM output in one pass (only live rows read the slabs)
template <typename T>
__global__ __launch_bounds__(256) void splitk_scatter_kernel(const float* __restrict__ slab, int splits,
                                                             int64_t slab_stride, int64_t d,
                                                             const int32_t* __restrict__ rank, int64_t n,
                                                             T* __restrict__ dst, int64_t ldd) {
  const int64_t cpr = d / 4;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n * cpr) return;
  const int64_t r = i / cpr, c = (i % cpr) * 4;
  const int32_t k = rank[r];
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (k >= 0) {
    const float* p = slab + (int64_t)k * d + c;
    int z = 0;
    for (; z + 8 <= splits; z += 8) {   // 8 splits' loads in flight, summed in split order (same bits)
      float4 u[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = *reinterpret_cast<const float4*>(p + (int64_t)(z + t) * slab_stride);
#pragma unroll
      for (int t = 0; t < 8; ++t) { v[0] += u[t].x; v[1] += u[t].y; v[2] += u[t].z; v[3] += u[t].w; }
    }
    for (; z < splits; ++z) {
      const float4 u = *reinterpret_cast<const float4*>(p + (int64_t)z * slab_stride);
      v[0] += u.x; v[1] += u.y; v[2] += u.z; v[3] += u.w;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) dst[r * ldd + c + j] = from_f<T>(v[j]);
}

// Eval scores at candidate ids: out[b][c] = <h[b], E[cand[b][c]]> (+ bias[cand[b][c]]).  SAS.predict
// (BS/models/sas_model/sas.py:107-118: last-position features . item_emb[candidates]) and BERT's validation
// scores (BS/trainers/bert.py:43-49: the last position's logits gathered at the candidates) without forming the
// (B, V+1) logits -- cfg5's full-vocabulary eval would be 51 GB fp32.  One wave per (row, candidate): lanes
// stride over the d features, fp32 products summed lane-wise in feature order then by a fixed butterfly.
// A candidate outside [0, V) scores NaN (the reference indexes out of range and raises; the Python wrapper checks).
template <typename T>
__global__ __launch_bounds__(256) void cand_scores_kernel(const T* __restrict__ h, int64_t ldh, int64_t B, int64_t d,
                                                          const T* __restrict__ E, const float* __restrict__ bias,
                                                          const int64_t* __restrict__ cand, int64_t C, int64_t V,
                                                          float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= B * C) return;
  const int64_t b = q / C, v = cand[q];
  if (v < 0 || v >= V) {
    if (lane == 0) out[q] = __builtin_nanf("");
    return;
  }
  const T* hr = h + b * ldh;
  const T* er = E + v * d;
  float acc = 0.f;
  for (int64_t k = lane; k < d; k += 64) acc = fmaf(to_f(hr[k]), to_f(er[k]), acc);
  acc = wave_sum(acc);
  if (lane == 0) out[q] = bias ? acc + bias[v] : acc;
}

extern "C" {

int rs_splitk_scatter_rows(int dtype, const float* slab, int splits, int64_t cap, int64_t d, const int32_t* rank,
                           int64_t n, void* dst, int64_t ldd, void* stream) {
  if (splits < 1 || cap <= 0 || d <= 0 || d % 4 || n <= 0 || !slab || !rank || !dst || ((uintptr_t)slab % 16))
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)cdiv(n * (d / 4), 256));
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((splitk_scatter_kernel<__bf16>), g, dim3(256), 0, s, slab, splits, cap * d, d, rank, n,
                       (__bf16*)dst, ldd);
  else
    hipLaunchKernelGGL((splitk_scatter_kernel<float>), g, dim3(256), 0, s, slab, splits, cap * d, d, rank, n,
                       (float*)dst, ldd);
  return (int)hipGetLastError();
}

int rs_compact_rows(const int64_t* labels, int64_t n, int64_t cap, int32_t* idx, int32_t* rank, int32_t* count,
                    void* stream) {
  if (n <= 0 || cap <= 0) return RS_ERR_ARG;
  if (n >= ((int64_t)1 << 31)) return RS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)cdiv(n, (int64_t)1024)), dim3(1024), 0, (hipStream_t)stream, labels,
                     n, cap, idx, rank, count);
  return (int)hipGetLastError();
}

int rs_gather_rows(int dtype, const void* src, int64_t lds, int64_t d, const int32_t* idx, const int32_t* count,
                   int64_t cap, void* dst, int64_t ldd, const int64_t* labels, int64_t* lab_out, void* stream) {
  const int vec = dtype == RS_DTYPE_BF16 ? 8 : 4;
  if (cap <= 0 || d <= 0 || d % vec || lds % vec || ldd % vec) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = cap * (d / vec);
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((gather_rows_kernel<__bf16>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s,
                       (const __bf16*)src, lds, d, idx, count, cap, (__bf16*)dst, ldd, labels, lab_out);
  else
    hipLaunchKernelGGL((gather_rows_kernel<float>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s,
                       (const float*)src, lds, d, idx, count, cap, (float*)dst, ldd, labels, lab_out);
  return (int)hipGetLastError();
}

int rs_scatter_rows(int dtype, const void* src, int64_t lds, int64_t d, const int32_t* rank, int64_t n, void* dst,
                    int64_t ldd, void* stream) {
  const int vec = dtype == RS_DTYPE_BF16 ? 8 : 4;
  if (n <= 0 || d <= 0 || d % vec || lds % vec || ldd % vec) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t m = n * (d / vec);
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((scatter_rows_kernel<__bf16>), dim3((unsigned)cdiv(m, 256)), dim3(256), 0, s,
                       (const __bf16*)src, lds, d, rank, n, (__bf16*)dst, ldd);
  else
    hipLaunchKernelGGL((scatter_rows_kernel<float>), dim3((unsigned)cdiv(m, 256)), dim3(256), 0, s,
                       (const float*)src, lds, d, rank, n, (float*)dst, ldd);
  return (int)hipGetLastError();
}

int rs_candidate_scores(int dtype, const void* h, int64_t ldh, int64_t B, int64_t d, const void* E, const float* bias,
                        const int64_t* cand, int64_t C, int64_t V, float* out, void* stream) {
  if (B <= 0 || C <= 0 || d <= 0 || V <= 0 || ldh < d || !h || !E || !cand || !out) return RS_ERR_ARG;
  const dim3 g((unsigned)cdiv(B * C, 4)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL(cand_scores_kernel<__bf16>, g, blk, 0, s, (const __bf16*)h, ldh, B, d, (const __bf16*)E, bias,
                       cand, C, V, out);
  else if (dtype == RS_DTYPE_F32)
    hipLaunchKernelGGL(cand_scores_kernel<float>, g, blk, 0, s, (const float*)h, ldh, B, d, (const float*)E, bias, cand,
                       C, V, out);
  else
    return RS_ERR_ARG;
  return (int)hipGetLastError();
}

}  // extern "C"
