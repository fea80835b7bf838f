// rs-build: included by grad_tail.hip (compiled once, as part of that translation unit)
// Embedding stage and the SAS sampled-logit head (gfx950).  HBM-bound row
// gathers / scatters: 16-byte vector loads along d, one row per 2..8 lanes.
//
//   rs_embed_fwd / rs_embed_bwd      BS/models/sas_model/sas.py:60-67 (SAS) and
//                                    BS/models/bert_modules/embedding/bert.py:29-31 (BERT)
//   rs_sampled_logits_fwd / _bwd     BS/models/sas_model/sas.py:93-100 (tied item_emb logits)
//
// Gradient scatter into the fp32 tables uses no-return float atomics (one
// dword per lane, 256 contiguous bytes per wave-instruction when d >= 64);
// rows with id 0 are skipped, which is torch's padding_idx=0 semantics
// (sas.py:30, bert_modules/embedding/token.py:6).  The positional-table
// gradient is a deterministic per-position sum over the batch.
#include "common.h"
#include "../../include/recsys_hip.h"

// count_ids (optional): wave w (global index) also writes count_parts[w] = the number of its rows r with
// count_ids[r] != 0 (SAS: the valid positions, pos != 0, the loss's divisor -- known here, long before the fused
// head needs it).  The id load is issued with the gathers and the count is a wave ballot: no barrier.
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, int64_t rows, int64_t T_,
                                                        const T* __restrict__ table, const T* __restrict__ pos,
                                                        int64_t d, float scale, int mode, float drop_p,
                                                        uint64_t salt, const uint64_t* seed_base, T* __restrict__ out,
                                                        const int64_t* __restrict__ count_ids,
                                                        int* __restrict__ count_parts) {
  const uint64_t seed = eff_seed(salt, seed_base);
  constexpr int V = Vec<T>::N;
  const int64_t cpr = d / V;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool in = i < rows * cpr;
  const bool head = count_ids && in && i % cpr == 0;
  const int64_t cid = head ? count_ids[i / cpr] : 0;
  if (in) {
    const int64_t r = i / cpr, c = (i % cpr) * V, t = r % T_;
    const int64_t id = ids[r];
    float e[V], p[V], o[V];
    load_chunk<T>(e, table + id * d + c);
    load_chunk<T>(p, pos + t * d + c);
    const float keep = (mode == 0 && id == 0) ? 0.f : 1.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float x = mode == 0 ? e[j] * scale + p[j] : e[j] + p[j];
      if (drop_p > 0.f) x *= drop_mul(drop_p, seed, (uint64_t)(r * d + c + j));
      o[j] = x * keep;
    }
    store_chunk<T>(out + r * d + c, o);
  }
  if (count_ids) {   // grid-uniform
    const int n = __popcll(__ballot(head && cid != 0));
    if ((threadIdx.x & 63) == 0) count_parts[(blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6] = n;
  }
}

// any width / alignment (e.g. the reference's default SAS d = 50): one element per thread, same math
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_any_kernel(const int64_t* __restrict__ ids, int64_t rows,
                                                            int64_t T_, const T* __restrict__ table,
                                                            const T* __restrict__ pos, int64_t d, float scale,
                                                            int mode, float drop_p, uint64_t salt,
                                                            const uint64_t* seed_base, T* __restrict__ out) {
  const uint64_t seed = eff_seed(salt, seed_base);
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= rows * d) return;
  const int64_t r = i / d, c = i % d, t = r % T_;
  const int64_t id = ids[r];
  const float e = to_f(table[id * d + c]), p = to_f(pos[t * d + c]);
  float x = mode == 0 ? e * scale + p : e + p;
  if (drop_p > 0.f) x *= drop_mul(drop_p, seed, (uint64_t)i);
  out[i] = from_f<T>((mode == 0 && id == 0) ? 0.f : x);
}

template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_table_kernel(const int64_t* __restrict__ ids, int64_t rows,
                                                              const T* __restrict__ dx, int64_t d, float scale,
                                                              float drop_p, uint64_t salt, const uint64_t* seed_base,
                                                              float* __restrict__ dtable) {
  const uint64_t seed = eff_seed(salt, seed_base);
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= rows * d) return;
  const int64_t r = i / d, c = i % d;
  const int64_t id = ids[r];
  if (id == 0) return;  // padding_idx = 0 (and the SAS timeline mask)
  float g = to_f(dx[i]) * scale;
  if (drop_p > 0.f) g *= drop_mul(drop_p, seed, (uint64_t)i);
  if (g != 0.f) atomicAdd(dtable + id * d + c, g);
}

template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(const int64_t* __restrict__ ids, int64_t rows,
                                                            int64_t T_, const T* __restrict__ dx, int64_t d,
                                                            int mode, float drop_p, uint64_t salt,
                                                            const uint64_t* seed_base, float* __restrict__ dpos,
                                                            int accumulate) {
  const uint64_t seed = eff_seed(salt, seed_base);
  // block = one position t, threads over columns; sum over the batch in order
  const int64_t t = blockIdx.x;
  const int64_t nb = rows / T_;
  for (int64_t c = threadIdx.x; c < d; c += blockDim.x) {
    float s = 0.f;
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t r = b * T_ + t;
      if (mode == 0 && ids[r] == 0) continue;  // SAS timeline mask zeroes padded rows
      float g = to_f(dx[r * d + c]);
      if (drop_p > 0.f) g *= drop_mul(drop_p, seed, (uint64_t)(r * d + c));
      s += g;
    }
    dpos[t * d + c] = accumulate ? dpos[t * d + c] + s : s;
  }
}

// vectorized positional-gradient sum: block = position t, 256 threads = CPR chunk-columns x RG
// batch groups, fixed-order LDS combine (deterministic)
template <typename T, int CPR, int NTB = 256>
__device__ __forceinline__ void embed_pos_body(const int64_t* __restrict__ ids, int64_t rows, int64_t T_,
                                               const T* __restrict__ dx, int64_t d, int mode, float drop_p,
                                               uint64_t salt, const uint64_t* seed_base, float* __restrict__ dpos,
                                               int accumulate, int64_t t) {
  constexpr int V = Vec<T>::N, RG = NTB / CPR;
  const uint64_t seed = eff_seed(salt, seed_base);
  const int64_t nb = rows / T_;
  const int cc = threadIdx.x % CPR, rg = threadIdx.x / CPR;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  if (cc * V < d) {
    // U rows per iteration, every load issued before any use (a branch around a load on the
    // row's id would make hipcc wait for each load in turn)
    constexpr int U = 8;
    const uint32_t s32 = seed32(seed);
    for (int64_t b0 = rg; b0 < nb; b0 += (int64_t)RG * U) {
      float g[U][V];
      bool keep[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t b = b0 + (int64_t)u * RG;
        const int64_t r = (b < nb ? b : nb - 1) * T_ + t;
        keep[u] = b < nb && (mode != 0 || ids[r] != 0);
        load_chunk<T>(g[u], dx + r * d + cc * V);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = (b0 + (int64_t)u * RG) * T_ + t;
        float dm[V];
#pragma unroll
        for (int j = 0; j < V; j += 2) {
          if (drop_p > 0.f) drop_mul2(drop_p, s32, (uint64_t)(r * d + cc * V + j), dm[j], dm[j + 1]);
          else dm[j] = dm[j + 1] = 1.f;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += keep[u] ? g[u][j] * dm[j] : 0.f;
      }
    }
  }
  __shared__ float red[RG][CPR * V];
#pragma unroll
  for (int j = 0; j < V; ++j) red[rg][cc * V + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += NTB) {
    float sum = 0.f;
    for (int g2 = 0; g2 < RG; ++g2) sum += red[g2][c];
    dpos[t * d + c] = accumulate ? dpos[t * d + c] + sum : sum;
  }
}

template <typename T, int CPR, int NTB = 256>
__global__ __launch_bounds__(NTB) void embed_bwd_pos_v_kernel(const int64_t* __restrict__ ids, int64_t rows,
                                                              int64_t T_, const T* __restrict__ dx, int64_t d,
                                                              int mode, float drop_p, uint64_t salt,
                                                              const uint64_t* seed_base, float* __restrict__ dpos,
                                                              int accumulate) {
  embed_pos_body<T, CPR, NTB>(ids, rows, T_, dx, d, mode, drop_p, salt, seed_base, dpos, accumulate, blockIdx.x);
}

// one wave per row m
template <typename T>
__global__ __launch_bounds__(256) void sampled_logits_fwd_kernel(const T* __restrict__ f, int64_t M, int64_t d,
                                                                 const T* __restrict__ E, const int64_t* __restrict__ pos,
                                                                 const int64_t* __restrict__ neg, float* __restrict__ pl,
                                                                 float* __restrict__ nl) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const T* fr = f + m * d;
  const T* ep = E + pos[m] * d;
  const T* en = E + neg[m] * d;
  float sp = 0.f, sn = 0.f;
  for (int64_t c = lane; c < d; c += 64) {
    const float x = to_f(fr[c]);
    sp += x * to_f(ep[c]);
    sn += x * to_f(en[c]);
  }
  sp = wave_sum(sp);
  sn = wave_sum(sn);
  if (lane == 0) {
    pl[m] = sp;
    nl[m] = sn;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void sampled_logits_bwd_kernel(const T* __restrict__ f, int64_t M, int64_t d,
                                                                 const T* __restrict__ E, const int64_t* __restrict__ pos,
                                                                 const int64_t* __restrict__ neg,
                                                                 const float* __restrict__ dpl,
                                                                 const float* __restrict__ dnl, T* __restrict__ df,
                                                                 int accumulate, float* __restrict__ dE) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const int64_t ip = pos[m], in = neg[m];
  const float gp = dpl[m], gn = dnl[m];
  const T* fr = f + m * d;
  const T* ep = E + ip * d;
  const T* en = E + in * d;
  T* dfr = df + m * d;
  for (int64_t c = lane; c < d; c += 64) {
    const float x = to_f(fr[c]);
    float g = gp * to_f(ep[c]) + gn * to_f(en[c]);
    if (accumulate) g += to_f(dfr[c]);
    dfr[c] = from_f<T>(g);
    if (dE == nullptr) continue;   // table gradient by rs_item_grad instead
    if (ip != 0 && gp != 0.f) atomicAdd(dE + ip * d + c, gp * x);
    if (in != 0 && gn != 0.f) atomicAdd(dE + in * d + c, gn * x);
  }
}

template <typename T>
static hipError_t embed_fwd_t(int mode, const int64_t* ids, int64_t rows, int64_t T_, const void* table,
                              const void* pos, int64_t d, float scale, float drop_p, uint64_t seed,
                              const uint64_t* seed_base, void* out, hipStream_t s,
                              const int64_t* count_ids = nullptr, int* count_parts = nullptr) {
  const bool vec = d % Vec<T>::N == 0 && ((uintptr_t)table | (uintptr_t)pos | (uintptr_t)out) % 16 == 0;
  if (!vec) {
    if (count_ids) return hipErrorInvalidValue;
    hipLaunchKernelGGL((embed_fwd_any_kernel<T>), dim3((unsigned)cdiv(rows * d, 256)), dim3(256), 0, s, ids, rows, T_,
                       (const T*)table, (const T*)pos, d, scale, mode, drop_p, seed, seed_base, (T*)out);
    return hipGetLastError();
  }
  const int64_t n = rows * (d / Vec<T>::N);
  hipLaunchKernelGGL((embed_fwd_kernel<T>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, ids, rows, T_,
                     (const T*)table, (const T*)pos, d, scale, mode, drop_p, seed, seed_base, (T*)out, count_ids,
                     count_parts);
  return hipGetLastError();
}

template <typename T>
static hipError_t embed_bwd_t(int mode, const int64_t* ids, int64_t rows, int64_t T_, const void* dx, int64_t d,
                              float scale, float drop_p, uint64_t seed, const uint64_t* seed_base, float* dtable,
                              float* dpos, int acc_pos, hipStream_t s) {
  if (dtable)
    hipLaunchKernelGGL((embed_bwd_table_kernel<T>), dim3((unsigned)cdiv(rows * d, 256)), dim3(256), 0, s, ids, rows,
                       (const T*)dx, d, mode == 0 ? scale : 1.0f, drop_p, seed, seed_base, dtable);
  if (dpos) {
    constexpr int V = Vec<T>::N;
    const int64_t cpr = d / V;
    const bool vec = (d % V == 0) && ((uintptr_t)dx % 16 == 0);
    if (vec && cpr <= 16)   // 512 threads: 32 batch groups, each row's loads and mask hashes spread over 8 waves
      hipLaunchKernelGGL((embed_bwd_pos_v_kernel<T, 16, 512>), dim3((unsigned)T_), dim3(512), 0, s, ids, rows, T_,
                         (const T*)dx, d, mode, drop_p, seed, seed_base, dpos, acc_pos);
    else if (vec && cpr <= 32)
      hipLaunchKernelGGL((embed_bwd_pos_v_kernel<T, 32>), dim3((unsigned)T_), dim3(256), 0, s, ids, rows, T_,
                         (const T*)dx, d, mode, drop_p, seed, seed_base, dpos, acc_pos);
    else if (vec && cpr <= 64)
      hipLaunchKernelGGL((embed_bwd_pos_v_kernel<T, 64>), dim3((unsigned)T_), dim3(256), 0, s, ids, rows, T_,
                         (const T*)dx, d, mode, drop_p, seed, seed_base, dpos, acc_pos);
    else
      hipLaunchKernelGGL((embed_bwd_pos_kernel<T>), dim3((unsigned)T_), dim3(d >= 256 ? 256 : 128), 0, s, ids, rows,
                         T_, (const T*)dx, d, mode, drop_p, seed, seed_base, dpos, acc_pos);
  }
  return hipGetLastError();
}

extern "C" {

int rs_embed_fwd(int dtype, int mode, const int64_t* ids, int64_t rows, int64_t T, const void* table,
                 const void* pos, int64_t d, float scale, float drop_p, uint64_t seed, const uint64_t* seed_base,
                 void* out, void* stream) {
  if (rows <= 0 || T <= 0 || rows % T || d <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  return (int)(dtype == RS_DTYPE_BF16
                   ? embed_fwd_t<__bf16>(mode, ids, rows, T, table, pos, d, scale, drop_p, seed, seed_base, out, s)
                   : embed_fwd_t<float>(mode, ids, rows, T, table, pos, d, scale, drop_p, seed, seed_base, out, s));
}

int rs_embed_bwd(int dtype, int mode, const int64_t* ids, int64_t rows, int64_t T, const void* dx, int64_t d,
                 float scale, float drop_p, uint64_t seed, const uint64_t* seed_base, float* dtable, float* dpos,
                 int accumulate_pos, void* stream) {
  if (rows <= 0 || T <= 0 || rows % T) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  return (int)(dtype == RS_DTYPE_BF16
                   ? embed_bwd_t<__bf16>(mode, ids, rows, T, dx, d, scale, drop_p, seed, seed_base, dtable, dpos, accumulate_pos, s)
                   : embed_bwd_t<float>(mode, ids, rows, T, dx, d, scale, drop_p, seed, seed_base, dtable, dpos, accumulate_pos, s));
}

int rs_sampled_logits_fwd(int dtype, const void* f, int64_t M, int64_t d, const void* E, const int64_t* pos,
                          const int64_t* neg, float* pl, float* nl, void* stream) {
  if (M <= 0 || d <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)cdiv(M, 4));
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((sampled_logits_fwd_kernel<__bf16>), grid, dim3(256), 0, s, (const __bf16*)f, M, d,
                       (const __bf16*)E, pos, neg, pl, nl);
  else
    hipLaunchKernelGGL((sampled_logits_fwd_kernel<float>), grid, dim3(256), 0, s, (const float*)f, M, d,
                       (const float*)E, pos, neg, pl, nl);
  return (int)hipGetLastError();
}

int rs_sampled_logits_bwd(int dtype, const void* f, int64_t M, int64_t d, const void* E, const int64_t* pos,
                          const int64_t* neg, const float* dpl, const float* dnl, void* df, int accumulate_df,
                          float* dE, void* stream) {
  if (M <= 0 || d <= 0) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)cdiv(M, 4));
  if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL((sampled_logits_bwd_kernel<__bf16>), grid, dim3(256), 0, s, (const __bf16*)f, M, d,
                       (const __bf16*)E, pos, neg, dpl, dnl, (__bf16*)df, accumulate_df, dE);
  else
    hipLaunchKernelGGL((sampled_logits_bwd_kernel<float>), grid, dim3(256), 0, s, (const float*)f, M, d,
                       (const float*)E, pos, neg, dpl, dnl, (float*)df, accumulate_df, dE);
  return (int)hipGetLastError();
}

}  // extern "C"
