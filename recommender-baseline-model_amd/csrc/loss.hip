// Loss heads (gfx950).
//
//   rs_bce_fwd / rs_bce_bwd  SAS: BCEWithLogits(pos_logits[valid], 1) + BCEWithLogits(neg_logits[valid], 0),
//                            each a mean over valid = (pos != 0)   (BS/trainers/sas.py:13,40,49)
//   rs_ce_fwd  / rs_ce_bwd   BERT: CrossEntropyLoss(ignore_index=0) over rows of vocabulary logits
//                            (BS/trainers/bert.py:11,36-40)
//
// Reductions are two-level (per-block partials to a small slab, then one block
// adds them in a fixed order), so the loss is deterministic.  The divisor is
// the valid-row count of this batch, or -- for data-parallel training -- a
// caller-provided global count (count_override), which makes the per-rank
// gradients sum exactly to the single-device mean's gradient.
#include "common.h"
#include "../../include/recsys_hip.h"

__device__ __forceinline__ float softplus(float z) { return fmaxf(z, 0.f) + log1pf(expf(-fabsf(z))); }
__device__ __forceinline__ float sigmoidf(float z) { return 1.f / (1.f + expf(-z)); }

#define BCE_BLOCKS 256

__global__ __launch_bounds__(256) void bce_partial_kernel(const float* __restrict__ pl, const float* __restrict__ nl,
                                                          const int64_t* __restrict__ pos, int64_t M,
                                                          float* __restrict__ ws) {
  float sp = 0.f, sn = 0.f, cnt = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    if (pos[i] != 0) {
      sp += softplus(-pl[i]);   // BCEWithLogits(x, 1)
      sn += softplus(nl[i]);    // BCEWithLogits(x, 0)
      cnt += 1.f;
    }
  }
  __shared__ float red[3][4];
  sp = wave_sum(sp); sn = wave_sum(sn); cnt = wave_sum(cnt);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = sp; red[1][w] = sn; red[2][w] = cnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    ws[blockIdx.x * 3 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    ws[blockIdx.x * 3 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    ws[blockIdx.x * 3 + 2] = red[2][0] + red[2][1] + red[2][2] + red[2][3];
  }
}

__global__ void bce_finish_kernel(const float* __restrict__ ws, int nblk, const float* __restrict__ count_override,
                                  float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float sp = 0.f, sn = 0.f, c = 0.f;
  for (int b = 0; b < nblk; ++b) { sp += ws[b * 3]; sn += ws[b * 3 + 1]; c += ws[b * 3 + 2]; }
  const float cc = count_override ? *count_override : c;
  out[0] = sp + sn;
  out[1] = c;
  out[2] = sp / cc + sn / cc;   // mean over valid positions, pos term + neg term
  out[3] = sn;
}

__global__ __launch_bounds__(256) void bce_bwd_kernel(const float* __restrict__ pl, const float* __restrict__ nl,
                                                      const int64_t* __restrict__ pos, int64_t M,
                                                      const float* __restrict__ count, const float* __restrict__ dloss,
                                                      float* __restrict__ dpl, float* __restrict__ dnl) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= M) return;
  const float s = (dloss ? *dloss : 1.f) / *count;
  const bool v = pos[i] != 0;
  dpl[i] = v ? (sigmoidf(pl[i]) - 1.f) * s : 0.f;
  dnl[i] = v ? sigmoidf(nl[i]) * s : 0.f;
}

// ---- cross entropy: one block per row, online (max, sum) over the vocabulary
__global__ __launch_bounds__(256) void ce_row_kernel(const float* __restrict__ logits, int64_t R, int64_t V1,
                                                     int64_t ldl, const int64_t* __restrict__ labels,
                                                     float* __restrict__ lse_out, float* __restrict__ part,
                                                     const int* __restrict__ rows_dev) {
  const int64_t r = blockIdx.x;
  if (rows_dev && r >= *rows_dev) {
    if (threadIdx.x == 0) { lse_out[r] = 0.f; part[r * 2] = 0.f; part[r * 2 + 1] = 0.f; }
    return;
  }
  const int64_t lab = labels[r];
  const float* x = logits + r * ldl;
  float m = -__builtin_inff(), s = 0.f;
  if (lab != 0) {
    for (int64_t j = threadIdx.x; j < V1; j += blockDim.x) {
      const float v = x[j];
      if (v > m) { s = s * expf(m - v) + 1.f; m = v; }
      else s += expf(v - m);
    }
  }
  // combine (m, s) across the block
  __shared__ float sm[256], ss[256];
  sm[threadIdx.x] = m; ss[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float m1 = sm[threadIdx.x], m2 = sm[threadIdx.x + o];
      const float s1 = ss[threadIdx.x], s2 = ss[threadIdx.x + o];
      const float mm = fmaxf(m1, m2);
      const float t = (mm == -__builtin_inff()) ? 0.f : s1 * expf(m1 - mm) + s2 * expf(m2 - mm);
      sm[threadIdx.x] = mm; ss[threadIdx.x] = t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float lse = lab != 0 ? sm[0] + logf(ss[0]) : 0.f;
    lse_out[r] = lse;
    part[r * 2 + 0] = lab != 0 ? lse - x[lab] : 0.f;
    part[r * 2 + 1] = lab != 0 ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(256) void ce_finish_kernel(const float* __restrict__ part, int64_t R,
                                                        const float* __restrict__ count_override,
                                                        float* __restrict__ out) {
  float s = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < R; i += blockDim.x) { s += part[i * 2]; c += part[i * 2 + 1]; }
  __shared__ float rs[4], rc[4];
  s = wave_sum(s); c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = s; rc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S = rs[0] + rs[1] + rs[2] + rs[3], C = rc[0] + rc[1] + rc[2] + rc[3];
    out[0] = S;
    out[1] = C;
    out[2] = S / (count_override ? *count_override : C);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits, int64_t R, int64_t V1,
                                                     int64_t ldl, const int64_t* __restrict__ labels,
                                                     const float* __restrict__ count, const float* __restrict__ dloss,
                                                     const float* __restrict__ lse, T* __restrict__ dl, int64_t lddl,
                                                     const int* __restrict__ rows_dev) {
  const int64_t r = blockIdx.y;
  if (rows_dev && r >= *rows_dev) return;
  const int64_t lab = labels[r];
  const float sc = (dloss ? *dloss : 1.f) / *count;
  const float L = lse[r];
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < V1; j += (int64_t)gridDim.x * blockDim.x) {
    float g = 0.f;
    if (lab != 0) g = (expf(logits[r * ldl + j] - L) - (j == lab ? 1.f : 0.f)) * sc;
    dl[r * lddl + j] = from_f<T>(g);
  }
}

extern "C" {

int rs_bce_fwd(const float* pl, const float* nl, const int64_t* pos, int64_t M, const float* count_override,
               float* ws, float* out, void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (int)std::min<int64_t>(BCE_BLOCKS, cdiv(M, 256));
  hipLaunchKernelGGL(bce_partial_kernel, dim3(nblk), dim3(256), 0, s, pl, nl, pos, M, ws);
  hipLaunchKernelGGL(bce_finish_kernel, dim3(1), dim3(64), 0, s, ws, nblk, count_override, out);
  return (int)hipGetLastError();
}

int rs_bce_bwd(const float* pl, const float* nl, const int64_t* pos, int64_t M, const float* count,
               const float* dloss, float* dpl, float* dnl, void* stream) {
  if (M <= 0 || !count) return RS_ERR_ARG;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3((unsigned)cdiv(M, 256)), dim3(256), 0, (hipStream_t)stream, pl, nl, pos,
                     M, count, dloss, dpl, dnl);
  return (int)hipGetLastError();
}

int rs_ce_fwd(const float* logits, int64_t R, int64_t V1, int64_t ldl, const int64_t* labels,
              const float* count_override, float* ws, float* out, const int* rows_dev, void* stream) {
  // ws layout: [R] lse, then [R][2] partials
  if (R <= 0 || V1 <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_row_kernel, dim3((unsigned)R), dim3(256), 0, s, logits, R, V1, ldl, labels, ws, ws + R, rows_dev);
  hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(256), 0, s, ws + R, R, count_override, out);
  return (int)hipGetLastError();
}

int rs_ce_bwd(int dtype, const float* logits, int64_t R, int64_t V1, int64_t ldl, const int64_t* labels,
              const float* count, const float* dloss, const float* ws, void* dlogits, int64_t lddl,
              const int* rows_dev, void* stream) {
  if (R <= 0 || V1 <= 0 || !count) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)std::min<int64_t>(cdiv(V1, 256), 64), (unsigned)R);
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((ce_bwd_kernel<__bf16>), grid, dim3(256), 0, s, logits, R, V1, ldl, labels, count, dloss, ws,
                       (__bf16*)dlogits, lddl, rows_dev);
  else
    hipLaunchKernelGGL((ce_bwd_kernel<float>), grid, dim3(256), 0, s, logits, R, V1, ldl, labels, count, dloss, ws,
                       (float*)dlogits, lddl, rows_dev);
  return (int)hipGetLastError();
}

}  // extern "C"
