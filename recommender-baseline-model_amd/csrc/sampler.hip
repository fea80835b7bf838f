// On-device SASRec training-batch sampler and ranking metrics (gfx950).
//
// rs_sas_sample replaces the reference's WarpSampler worker (BS/dataloaders/sas.py:65-91):
//   user u ~ uniform over the users;  train = history[u][-max_len:];
//   seq = [0]*pad + train[:-1],  pos = [0]*pad + train[1:],  pad = max_len - len(train) + 1
//   neg = [0]*pad + (len(train)-1) draws uniform over {0..item_num} \ set(train)
// (random_neq, sas.py:60-62: uniform over the complement; item 0 is a legal negative).
// One workgroup per sequence: the window's items go into an LDS hash set, negatives are drawn by
// rejection against it (expected draws (V+1)/(V+1-|set|)).  Counter-based RNG (splitmix64 of the
// device step seed, the sequence and position, the attempt): graph-capturable, reproducible.  The
// reference's numpy stream cannot be reproduced; the distribution is the same.
//
// rs_bert_mask replaces BertTrainDataset's per-token Python masking (BS/dataloaders/bert.py:77-110).
//
// The *_draws forms also record the random draws each row consumed (user index, candidate negatives / the
// masking uniform and replacement item), so tests replay the reference's construction on them
// (oracle/sampling.py) and compare the batch bit for bit.
//
// rs_rank_metrics restates recalls_ndcgs_and_mrr_for_ks (BS/trainers/utils.py:28-57) on the GPU:
// per row the rank of every positive among the candidates (score descending, ties by index as a
// stable sort), then Recall@k / NDCG@k / MRR@k summed over rows in a fixed order.
#include "common.h"
#include "../../include/recsys_hip.h"

namespace smp {

constexpr int HS = 1024;   // LDS hash-set slots (>= 2 * window)
constexpr int NA = 256;    // negative-draw attempts per position (the rejection loop's bound; a draws record keeps all)

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int slot_of(int64_t v) { return (int)(((uint64_t)v * 0x9E3779B97F4A7C15ull) >> 54); }

__device__ __forceinline__ bool contains(const int64_t* tab, int64_t v) {
  int s = slot_of(v);
  for (int p = 0; p < HS; ++p) {
    const int64_t x = tab[s];
    if (x == v) return true;
    if (x < 0) return false;
    s = (s + 1) & (HS - 1);
  }
  return false;
}

__global__ __launch_bounds__(256) void sas_sample_kernel(const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ items, int64_t n_users,
                                                         int64_t item_num, int T, const uint64_t* seed_base,
                                                         uint64_t salt, int64_t* __restrict__ seq,
                                                         int64_t* __restrict__ pos, int64_t* __restrict__ neg,
                                                         int64_t* __restrict__ draws) {
  __shared__ int64_t tab[HS];
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  const uint64_t seed = salt ^ ((seed_base ? *seed_base : 0ull) * 0xD1B54A32D192ED03ull);
  const int64_t u = (int64_t)__umul64hi(splitmix64(seed ^ (0xA0761D6478BD642Full * (uint64_t)(b + 1))),
                                        (uint64_t)n_users);
  const int64_t s0 = off[u], L = off[u + 1] - s0;
  const int64_t n = L < T ? L : T;          // window = the last n items (history[-max_len:])
  const int64_t w0 = s0 + L - n;
  const int64_t pad = T - n + 1;
  // draws (tests): per row {u, then per position the first NA candidate negatives, -1 where no negative is drawn}
  int64_t* dr = draws ? draws + b * (1 + (int64_t)T * NA) : nullptr;
  if (dr && tid == 0) dr[0] = u;
  for (int i = tid; i < HS; i += 256) tab[i] = -1;
  __syncthreads();
  for (int64_t i = tid; i < n; i += 256) {
    const int64_t v = items[w0 + i];
    int s = slot_of(v);
    for (int p = 0; p < HS; ++p) {
      const unsigned long long prev =
          atomicCAS(reinterpret_cast<unsigned long long*>(&tab[s]), ~0ull, (unsigned long long)v);
      if (prev == ~0ull || (int64_t)prev == v) break;
      s = (s + 1) & (HS - 1);
    }
  }
  __syncthreads();
  const uint64_t V1 = (uint64_t)item_num + 1;
  for (int t = tid; t < T; t += 256) {
    const int64_t o = t - pad;                 // position in the window of seq[t]
    int64_t sv = 0, pv = 0, nv = 0;
    if (o >= 0) {
      sv = items[w0 + o];
      pv = items[w0 + o + 1];
      const uint64_t base = seed + (((uint64_t)b * (uint64_t)T + (uint64_t)t) << 20);
      int64_t v = (int64_t)__umul64hi(splitmix64(base), V1);
      for (int a = 1; a < NA && contains(tab, v); ++a) v = (int64_t)__umul64hi(splitmix64(base + a), V1);
      for (int64_t k = 0; k < (int64_t)V1 && contains(tab, v); ++k) v = (v + 1) % (int64_t)V1;   // never reached in practice
      nv = v;
    }
    if (dr)
      for (int a = 0; a < NA; ++a)
        dr[1 + (int64_t)t * NA + a] = o >= 0 ? (int64_t)__umul64hi(splitmix64(seed + (((uint64_t)b * (uint64_t)T + (uint64_t)t) << 20) + a), V1) : -1;
    seq[b * T + t] = sv;
    pos[b * T + t] = pv;
    neg[b * T + t] = nv;
  }
}

__global__ void seed_step_kernel(uint64_t* s) {
  if (threadIdx.x == 0) *s += 1;
}

// BERT4Rec cloze masking (BertTrainDataset.__getitem__, BS/dataloaders/bert.py:77-110): the row's user is
// perm[(cursor * batch + b) mod n_users] (an epoch's shuffled order); every kept item (the last max_len of
// the history) is masked with probability p -- then, with prob' = u / p, [MASK] if prob' < 0.8, a uniform
// item of 1..num_items if prob' < 0.9, else itself -- and labelled with itself; other positions keep
// their item with label 0; rows are left padded with 0.  state = {step seed, cursor}, advanced first.
__global__ __launch_bounds__(256) void bert_mask_kernel(const int64_t* __restrict__ off,
                                                        const int64_t* __restrict__ items, int64_t n_users,
                                                        int64_t num_items, int T, double p,
                                                        const int64_t* __restrict__ perm,
                                                        const uint64_t* __restrict__ state, uint64_t salt,
                                                        int64_t* __restrict__ tokens, int64_t* __restrict__ labels,
                                                        int64_t* __restrict__ draws) {
  const int64_t b = blockIdx.x;
  const uint64_t seed = salt ^ (state[0] * 0xD1B54A32D192ED03ull);
  const int64_t slot = (int64_t)(((state[1] - 1) * (uint64_t)gridDim.x + (uint64_t)b) % (uint64_t)n_users);
  const int64_t u = perm ? perm[slot] : slot;
  const int64_t s0 = off[u], L = off[u + 1] - s0;
  const int64_t n = L < T ? L : T;
  const int64_t w0 = s0 + L - n, pad = T - n;
  const int64_t mask_token = num_items + 1;
  // the reference's decision (prob = rng.rand(); prob < mask_prob; prob /= mask_prob; < 0.8; < 0.9) in double on
  // the 24-bit uniform k / 2^24, exactly as Python evaluates it on that value (mask_prob arrives as the Python double)
  const double pd = p;
  // draws (tests): per row {u, then per position (k, the replacement item), -1 on padding}
  int64_t* dr = draws ? draws + b * (1 + 2 * (int64_t)T) : nullptr;
  if (dr && threadIdx.x == 0) dr[0] = u;
  for (int t = threadIdx.x; t < T; t += 256) {
    int64_t tok = 0, lab = 0, dk = -1, di = -1;
    if (t >= pad) {
      const int64_t it = items[w0 + t - pad];
      const uint64_t h = splitmix64(seed + (((uint64_t)b * (uint64_t)T + (uint64_t)t) << 8));
      const double prob = (double)(h >> 40) * (1.0 / 16777216.0);      // 24-bit uniform [0, 1), exact in double
      const int64_t rnd = 1 + (int64_t)__umul64hi(splitmix64(h ^ 0x9E3779B97F4A7C15ull), (uint64_t)num_items);
      tok = it;
      if (prob < pd) {
        const double q = prob / pd;
        if (q < 0.8) tok = mask_token;
        else if (q < 0.9) tok = rnd;
        lab = it;
      }
      dk = (int64_t)(h >> 40);
      di = rnd;
    }
    tokens[b * T + t] = tok;
    labels[b * T + t] = lab;
    if (dr) {
      dr[1 + 2 * t] = dk;
      dr[2 + 2 * t] = di;
    }
  }
}

__global__ void mask_step_kernel(uint64_t* s) {
  if (threadIdx.x == 0) {
    s[0] += 1;
    s[1] += 1;
  }
}

// ---------------------------------------------------------------------------------- metrics
constexpr int MAXK = 8;

// one wave per row: partial[row][3*nk] = (recall, ndcg, mrr) per k
__global__ __launch_bounds__(256) void rank_rows_kernel(const float* __restrict__ scores, const float* __restrict__ labels,
                                                        int64_t R, int64_t C, int nk, const int* __restrict__ ks_dev,
                                                        float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* s = scores + r * C;
  const float* l = labels + r * C;
  int ks[MAXK];
  for (int q = 0; q < nk; ++q) ks[q] = ks_dev[q];
  float rec[MAXK], dcg[MAXK], mrr[MAXK];
  for (int q = 0; q < MAXK; ++q) rec[q] = dcg[q] = mrr[q] = 0.f;
  float npos = 0.f;
  for (int64_t j = 0; j < C; ++j) {
    const float lj = l[j];
    if (lj == 0.f) continue;                  // wave-uniform
    npos += lj;
    const float sj = s[j];
    int cnt = 0;
    for (int64_t i = lane; i < C; i += 64) {
      const float si = s[i];
      cnt += (si > sj || (si == sj && i < j)) ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    const int p = cnt + 1;                    // 1-based position after a stable descending sort
    for (int q = 0; q < nk; ++q)
      if (p <= ks[q]) {
        rec[q] += lj;
        dcg[q] += lj / log2f((float)p + 1.f);
        mrr[q] += lj / (float)p;
      }
  }
  if (lane != 0) return;
  for (int q = 0; q < nk; ++q) {
    float idcg = 0.f;
    const int m = (int)fminf(npos, (float)ks[q]);
    for (int i = 0; i < m; ++i) idcg += 1.f / log2f((float)i + 2.f);
    partial[r * 3 * nk + 3 * q + 0] = rec[q] / npos;
    partial[r * 3 * nk + 3 * q + 1] = dcg[q] / idcg;
    partial[r * 3 * nk + 3 * q + 2] = mrr[q];
  }
}

// mean over rows, fixed order (one workgroup)
__global__ __launch_bounds__(256) void rank_mean_kernel(const float* __restrict__ partial, int64_t R, int m,
                                                        float* __restrict__ out) {
  __shared__ double red[256];
  for (int c = 0; c < m; ++c) {
    double acc = 0.0;
    for (int64_t r = threadIdx.x; r < R; r += 256) acc += (double)partial[r * m + c];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = (float)(red[0] / (double)R);
    __syncthreads();
  }
}

}  // namespace smp

extern "C" {

int rs_sas_sample_draws(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t item_num,
                        int64_t batch, int64_t max_len, uint64_t* seed_base, uint64_t salt, int64_t* seq, int64_t* pos,
                        int64_t* neg, int64_t* draws, void* stream) {
  if (n_users <= 0 || item_num <= 0 || batch <= 0 || max_len <= 0 || max_len > smp::HS / 2 || !user_offsets ||
      !user_items || !seq || !pos || !neg)
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (seed_base) hipLaunchKernelGGL(smp::seed_step_kernel, dim3(1), dim3(64), 0, s, seed_base);
  hipLaunchKernelGGL(smp::sas_sample_kernel, dim3((unsigned)batch), dim3(256), 0, s, user_offsets, user_items, n_users,
                     item_num, (int)max_len, seed_base, salt, seq, pos, neg, draws);
  return (int)hipGetLastError();
}

int rs_sas_sample(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t item_num,
                  int64_t batch, int64_t max_len, uint64_t* seed_base, uint64_t salt, int64_t* seq, int64_t* pos,
                  int64_t* neg, void* stream) {
  return rs_sas_sample_draws(user_offsets, user_items, n_users, item_num, batch, max_len, seed_base, salt, seq, pos,
                             neg, nullptr, stream);
}

int rs_bert_mask_draws(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t num_items,
                       int64_t batch, int64_t max_len, double mask_prob, const int64_t* perm, uint64_t* state,
                       uint64_t salt, int64_t* tokens, int64_t* labels, int64_t* draws, void* stream) {
  if (n_users <= 0 || num_items <= 0 || batch <= 0 || max_len <= 0 || !(mask_prob >= 0.0 && mask_prob <= 1.0) ||
      !user_offsets || !user_items || !state || !tokens || !labels)
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(smp::mask_step_kernel, dim3(1), dim3(64), 0, s, state);
  hipLaunchKernelGGL(smp::bert_mask_kernel, dim3((unsigned)batch), dim3(256), 0, s, user_offsets, user_items, n_users,
                     num_items, (int)max_len, mask_prob, perm, state, salt, tokens, labels, draws);
  return (int)hipGetLastError();
}

int rs_bert_mask(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t num_items,
                 int64_t batch, int64_t max_len, double mask_prob, const int64_t* perm, uint64_t* state, uint64_t salt,
                 int64_t* tokens, int64_t* labels, void* stream) {
  return rs_bert_mask_draws(user_offsets, user_items, n_users, num_items, batch, max_len, mask_prob, perm, state, salt,
                            tokens, labels, nullptr, stream);
}

int rs_rank_metrics(const float* scores, const float* labels, int64_t rows, int64_t cands, int nk, const int* ks,
                    float* ws, float* out, void* stream) {
  if (rows <= 0 || cands <= 0 || nk <= 0 || nk > smp::MAXK || !scores || !labels || !ks || !ws || !out)
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(smp::rank_rows_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, s, scores, labels, rows, cands,
                     nk, ks, ws);
  hipLaunchKernelGGL(smp::rank_mean_kernel, dim3(1), dim3(256), 0, s, ws, rows, 3 * nk, out);
  return (int)hipGetLastError();
}

}  // extern "C"
