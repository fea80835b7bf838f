// rs-build: included by grad_tail.hip (compiled once, as part of that translation unit)
// SASRec output head, fused (bf16 activations, fp32 math; gfx950).
//
// Forward (BS/models/sas_model/sas.py:87-100 + the BCE of BS/trainers/sas.py:40-49):
//   f = last_layernorm(x_L)          [saved: f, mean, rstd]
//   pos_logits = <f, E[pos]>, neg_logits = <f, E[neg]>      (E = item_emb, tied)
//   per-64-row-block partial sums of softplus(-pos_logit), softplus(neg_logit) and the
//   valid count (pos != 0)  -> part[block][3]
// Backward:
//   every workgroup sums the count partials in block order (deterministic, no finish
//   kernel), dpl = (sigmoid(pl) - 1)/count, dnl = sigmoid(nl)/count on valid rows (or the
//   caller's dpl/dnl), df = dpl E[pos] + dnl E[neg], dx_L = LN'(x_L, df) and the LayerNorm
//   affine partials; workgroup 0 also writes the loss statistics.
// One kernel each way replaces LN fwd + sampled logits + 2 BCE kernels, and BCE bwd + sampled
// logits bwd + LN bwd (+ its reduce): the item-table gradient of the logits is rs_item_grad's.
#include "common.h"
#include "../../include/recsys_hip.h"

namespace hd {

typedef __bf16 bf16;
constexpr int RB = 64;   // rows per workgroup

__device__ __forceinline__ float softplus(float z) { return fmaxf(z, 0.f) + log1pf(expf(-fabsf(z))); }
__device__ __forceinline__ float sigmoidf(float z) { return 1.f / (1.f + expf(-z)); }

template <int D>
__global__ __launch_bounds__(256) void head_fwd_kernel(int64_t M, const bf16* __restrict__ x,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, bf16* __restrict__ f, float* __restrict__ mean,
                                                       float* __restrict__ rstd, const bf16* __restrict__ E,
                                                       const int64_t* __restrict__ pos, const int64_t* __restrict__ neg,
                                                       float* __restrict__ pl, float* __restrict__ nl,
                                                       float* __restrict__ part) {
  constexpr int LPR = D / 8, RPP = 256 / LPR, NP = RB / RPP;
  const int tid = threadIdx.x, sub = tid % LPR, c0 = sub * 8;
  const int64_t row0 = (int64_t)blockIdx.x * RB;
  float gm[8], bt[8];
  load_chunk<float>(gm, gamma + c0);
  load_chunk<float>(gm + 4, gamma + c0 + 4);
  load_chunk<float>(bt, beta + c0);
  load_chunk<float>(bt + 4, beta + c0 + 4);
  float xv[NP][8], ep[NP][8], en[NP][8];
  int64_t ip[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int64_t m0 = row0 + k * RPP + tid / LPR;
    const int64_t m = m0 < M ? m0 : M - 1;
    ip[k] = pos[m];
    load_chunk<bf16>(xv[k], x + m * D + c0);
    load_chunk<bf16>(ep[k], E + ip[k] * D + c0);
    load_chunk<bf16>(en[k], E + neg[m] * D + c0);
  }
  float sp = 0.f, sn = 0.f, cnt = 0.f;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int64_t m = row0 + k * RPP + tid / LPR;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += xv[k][j];
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mu = s / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float u = xv[k][j] - mu;
      q += u * u;
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rs = 1.0f / sqrtf(q / (float)D + eps);
    float y[8];
    float dp = 0.f, dn = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y[j] = (xv[k][j] - mu) * rs * gm[j] + bt[j];
      y[j] = (float)(bf16)y[j];                // the logits read the stored (bf16) features
      dp += y[j] * ep[k][j];
      dn += y[j] * en[k][j];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) {
      dp += __shfl_xor(dp, o, 64);
      dn += __shfl_xor(dn, o, 64);
    }
    if (m < M) {
      store_chunk<bf16>(f + m * D + c0, y);
      if (sub == 0) {
        mean[m] = mu;
        rstd[m] = rs;
        pl[m] = dp;
        nl[m] = dn;
        if (ip[k] != 0) {
          sp += softplus(-dp);
          sn += softplus(dn);
          cnt += 1.f;
        }
      }
    }
  }
  // block partials in a fixed order: lanes -> waves -> LDS
  sp = wave_sum(sp);
  sn = wave_sum(sn);
  cnt = wave_sum(cnt);
  __shared__ float red[3][4];
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    red[0][w] = sp;
    red[1][w] = sn;
    red[2][w] = cnt;
  }
  __syncthreads();
  if (tid < 3) part[blockIdx.x * 3 + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}

template <int D>
__global__ __launch_bounds__(256) void head_bwd_kernel(int64_t M, int nblk, const float* __restrict__ part,
                                                       const float* __restrict__ divisor, float* __restrict__ out,
                                                       const float* __restrict__ pl, const float* __restrict__ nl,
                                                       const float* __restrict__ dpl_in, const float* __restrict__ dnl_in,
                                                       float* __restrict__ dpl, float* __restrict__ dnl,
                                                       const int64_t* __restrict__ pos, const int64_t* __restrict__ neg,
                                                       const bf16* __restrict__ E, const bf16* __restrict__ x,
                                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, bf16* __restrict__ dx,
                                                       float* __restrict__ lnpart) {
  constexpr int LPR = D / 8, RPP = 256 / LPR, NP = RB / RPP;
  const int tid = threadIdx.x, sub = tid % LPR, c0 = sub * 8;
  const int64_t row0 = (int64_t)blockIdx.x * RB;
  __shared__ float red[8][256];
  float gm[8];
  load_chunk<float>(gm, gamma + c0);
  load_chunk<float>(gm + 4, gamma + c0 + 4);
  // all row loads first; the loss statistics below overlap their latency
  float xv[NP][8], ep[NP][8], en[NP][8], gp[NP], gn[NP], mu[NP], ra[NP];
  bool vrow[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int64_t m0 = row0 + k * RPP + tid / LPR;
    const int64_t m = m0 < M ? m0 : M - 1;
    const int64_t ipos = pos[m];
    load_chunk<bf16>(xv[k], x + m * D + c0);
    load_chunk<bf16>(ep[k], E + ipos * D + c0);
    load_chunk<bf16>(en[k], E + neg[m] * D + c0);
    mu[k] = mean[m];
    ra[k] = rstd[m];
    vrow[k] = ipos != 0;
    gp[k] = dpl_in ? dpl_in[m] : pl[m];
    gn[k] = dpl_in ? dnl_in[m] : nl[m];
  }
  // loss statistics / gradient scale from the forward partials (fixed order: identical in every block)
  if (!dpl_in) {
    float c = 0.f, a = 0.f, b = 0.f;
    for (int i = tid; i < nblk; i += 256) {
      a += part[i * 3];
      b += part[i * 3 + 1];
      c += part[i * 3 + 2];
    }
    red[0][tid] = a;
    red[1][tid] = b;
    red[2][tid] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) {
        red[0][tid] += red[0][tid + s];
        red[1][tid] += red[1][tid + s];
        red[2][tid] += red[2][tid + s];
      }
      __syncthreads();
    }
    const float cc = divisor ? *divisor : red[2][0];
    const float scale = 1.f / cc;
    if (blockIdx.x == 0 && tid == 0) {
      out[0] = red[0][0] + red[1][0];
      out[1] = red[2][0];
      out[2] = red[0][0] / cc + red[1][0] / cc;
      out[3] = red[1][0];
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      gp[k] = vrow[k] ? (sigmoidf(gp[k]) - 1.f) * scale : 0.f;
      gn[k] = vrow[k] ? sigmoidf(gn[k]) * scale : 0.f;
    }
  }
  float pg[8], pb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pg[j] = pb[j] = 0.f;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int64_t m = row0 + k * RPP + tid / LPR;
    const bool valid = m < M;
    const float a = ra[k];
    float u[8], gq[8], sg = 0.f, sgu = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = valid ? gp[k] * ep[k][j] + gn[k] * en[k][j] : 0.f;   // df
      u[j] = xv[k][j] - mu[k];
      gq[j] = g * gm[j];
      pg[j] += g * (u[j] * a);
      pb[j] += g;
      sg += gq[j];
      sgu += gq[j] * u[j];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) {
      sg += __shfl_xor(sg, o, 64);
      sgu += __shfl_xor(sgu, o, 64);
    }
    const float mg = sg / (float)D;
    const float coef = a * a * a * sgu / (float)D;
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = a * (gq[j] - mg) - coef * u[j];
    if (valid) {
      store_chunk<bf16>(dx + m * D + c0, t);
      if (sub == 0 && !dpl_in) {
        dpl[m] = gp[k];
        dnl[m] = gn[k];
      }
    }
  }
  // affine partials of the block: RPP row groups combined in a fixed order
  float* r = &red[0][0];   // [RPP][D] = 2048 floats
  const int grp = tid / LPR;
  for (int which = 0; which < 2; ++which) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) r[grp * D + c0 + j] = which == 0 ? pg[j] : pb[j];
    __syncthreads();
    if (tid < D) {
      float s = 0.f;
      for (int g = 0; g < RPP; ++g) s += r[g * D + tid];
      lnpart[((int64_t)blockIdx.x * 2 + which) * D + tid] = s;
    }
  }
}

// the loss statistics of the head's block partials (as head_bwd_kernel's workgroup 0 forms them), by one workgroup:
// out = [sum of the BCE terms, valid count, loss = mean pos term + mean neg term, neg sum]
__device__ void head_stats(int nblk, const float* __restrict__ part, const float* __restrict__ divisor,
                           float* __restrict__ out, float (*red)[256], float* __restrict__ aux = nullptr) {
  const int tid = threadIdx.x;
  float c = 0.f, a = 0.f, b = 0.f;
  for (int i = tid; i < nblk; i += 256) {
    a += part[i * 3];
    b += part[i * 3 + 1];
    c += part[i * 3 + 2];
  }
  red[0][tid] = a;
  red[1][tid] = b;
  red[2][tid] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      red[0][tid] += red[0][tid + s];
      red[1][tid] += red[1][tid + s];
      red[2][tid] += red[2][tid + s];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float cc = divisor ? *divisor : red[2][0];
    out[0] = red[0][0] + red[1][0];
    out[1] = red[2][0];
    out[2] = red[0][0] / cc + red[1][0] / cc;
    out[3] = red[1][0];
    if (aux) {   // data parallel: (loss sum, count) straight into the gradient buffer's all-reduced tail
      aux[0] = out[0];
      aux[1] = out[1];
    }
  }
}

__global__ __launch_bounds__(256) void head_finish_kernel(int nblk, const float* __restrict__ part,
                                                          const float* __restrict__ divisor, float* __restrict__ out) {
  __shared__ float red[3][256];
  head_stats(nblk, part, divisor, out, red);
}

}  // namespace hd

extern "C" {

int rs_sas_head_finish(int64_t nblk, const float* part, const float* divisor, float* out, void* stream) {
  if (nblk <= 0 || !part || !out) return RS_ERR_ARG;
  hipLaunchKernelGGL(hd::head_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, (int)nblk, part,
                     divisor, out);
  return (int)hipGetLastError();
}

int rs_sas_head_fwd(int64_t M, int64_t d, const void* x, const float* ln_w, const float* ln_b, float eps, void* f,
                    float* mean, float* rstd, const void* E, const int64_t* pos, const int64_t* neg, float* pl,
                    float* nl, float* part, void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  const dim3 grid((unsigned)cdiv(M, hd::RB));
  hipStream_t s = (hipStream_t)stream;
#define HF(D)                                                                                                \
  hipLaunchKernelGGL(hd::head_fwd_kernel<D>, grid, dim3(256), 0, s, M, (const __bf16*)x, ln_w, ln_b, eps,   \
                     (__bf16*)f, mean, rstd, (const __bf16*)E, pos, neg, pl, nl, part)
  if (d == 64) HF(64);
  else if (d == 128) HF(128);
  else if (d == 256) HF(256);
  else return RS_ERR_UNSUPPORTED;
#undef HF
  return (int)hipGetLastError();
}

int rs_sas_head_bwd(int64_t M, int64_t d, const float* part, const float* divisor, float* out, const float* pl,
                    const float* nl, const float* dpl_in, const float* dnl_in, float* dpl, float* dnl,
                    const int64_t* pos, const int64_t* neg, const void* E, const void* x, const float* ln_w,
                    const float* mean, const float* rstd, void* dx, float* lnpart, void* stream) {
  if (M <= 0 || (!dpl_in && (!part || !out || !dpl || !dnl))) return RS_ERR_ARG;
  const int nblk = (int)cdiv(M, hd::RB);
  const dim3 grid((unsigned)nblk);
  hipStream_t s = (hipStream_t)stream;
#define HB(D)                                                                                                 \
  hipLaunchKernelGGL(hd::head_bwd_kernel<D>, grid, dim3(256), 0, s, M, nblk, part, divisor, out, pl, nl,     \
                     dpl_in, dnl_in, dpl, dnl, pos, neg, (const __bf16*)E, (const __bf16*)x, ln_w, mean, rstd, \
                     (__bf16*)dx, lnpart)
  if (d == 64) HB(64);
  else if (d == 128) HB(128);
  else if (d == 256) HB(256);
  else return RS_ERR_UNSUPPORTED;
#undef HB
  return (int)hipGetLastError();
}

}  // extern "C"
