// LayerNorm forward/backward, both reference variants (gfx950).
//
// variant 0 -- torch.nn.LayerNorm(d, eps=1e-8): biased variance, eps inside the sqrt
//              (BS/models/sas_model/sas.py:39,42,50,74,82,86)
// variant 1 -- BERT custom LN: a_2*(x-mean)/(std_unbiased+eps)+b_2, eps=1e-6
//              (BS/models/bert_modules/utils/layer_norm.py:14-17)
//
// One wave per row (rows of d <= 1024 live in registers, two-pass statistics
// in fp32).  The affine-parameter gradients are column sums over all M rows:
// every block keeps per-column partials in registers for its rows, the
// partials go to a [blocks][2][d] slab and a second kernel adds them in a
// fixed order (deterministic, no atomics).
#include "common.h"
#include "../../include/recsys_hip.h"

#define LN_MAXV 16  // d <= 64*16
#define LN_BWD_BLOCKS 512  // affine-partial slabs per LN backward (ws >= 2*d*LN_BWD_BLOCKS floats)

template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ X, int64_t ldx, int64_t M, int d,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, int variant, T* __restrict__ Y, int64_t ldy,
                                                     float* __restrict__ mean_out, float* __restrict__ rinv_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* x = X + row * ldx;
  float v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < d ? to_f(x[c]) : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    const float u = c < d ? v[i] - mu : 0.f;
    q += u * u;
  }
  q = wave_sum(q);
  float rinv;
  if (variant == 0) rinv = 1.0f / sqrtf(q / (float)d + eps);
  else rinv = 1.0f / (sqrtf(q / (float)(d - 1)) + eps);
  T* y = Y + row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < d) {
      const float u = v[i] - mu;
      float o = variant == 0 ? u * rinv * gamma[c] + beta[c] : gamma[c] * (u * rinv) + beta[c];
      y[c] = from_f<T>(o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rinv_out[row] = rinv;
  }
}

template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ X, int64_t ldx, const T* __restrict__ dY,
                                                     int64_t lddy, int64_t M, int d, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rinv,
                                                     float eps, int variant, T* __restrict__ dX, int64_t lddx,
                                                     int accumulate, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[NV], pb[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < M; row += stride) {
    const T* x = X + row * ldx;
    const T* dy = dY + row * lddy;
    const float mu = mean[row], a = rinv[row];
    float u[NV], gq[NV];
    float sg = 0.f, sgu = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < d) {
        u[i] = to_f(x[c]) - mu;
        const float dyc = to_f(dy[c]);
        gq[i] = dyc * gamma[c];
        pg[i] += dyc * (u[i] * a);
        pb[i] += dyc;
      } else {
        u[i] = 0.f;
        gq[i] = 0.f;
      }
      sg += gq[i];
      sgu += gq[i] * u[i];
    }
    sg = wave_sum(sg);
    sgu = wave_sum(sgu);
    const float mg = sg / (float)d;
    float coef;  // dx = a*(g - mean(g)) - coef*u
    if (variant == 0) {
      coef = a * a * a * sgu / (float)d;                      // a * xhat * mean(g*xhat)
    } else {
      const float sd = 1.0f / a - eps;                        // unbiased std
      coef = sd > 0.f ? a * a * sgu / ((float)(d - 1) * sd) : 0.f;
    }
    T* dx = dX + row * lddx;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < d) {
        float o = a * (gq[i] - mg) - coef * u[i];
        if (accumulate) o += to_f(dx[c]);
        dx[c] = from_f<T>(o);
      }
    }
  }
  // block-level reduction of the affine partials through LDS
  __shared__ float red[4][2][64 * LN_MAXV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    red[wave][0][lane + 64 * i] = pg[i];
    red[wave][1][lane + 64 * i] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 256) {
    float g0 = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    float b0 = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    part[((int64_t)blockIdx.x * 2 + 0) * d + c] = g0;
    part[((int64_t)blockIdx.x * 2 + 1) * d + c] = b0;
  }
}

// ---- vectorized kernels: LPR lanes per row, NCH 16-byte chunks per lane (d = LPR*NCH*V),
// 64/LPR rows per wave; statistics by shuffles inside the LPR-lane group.
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (hipcc pitfall: a per-element `variant ? a : b` around the gamma/beta loads made it branch and
// wait vmcnt(0) per element -- 16 dependent L2 round trips, 4x the kernel time; the variant is a
// template parameter and gamma/beta are loaded as float4 vectors up front)
template <typename T, int LPR, int NCH, int VAR>
__global__ __launch_bounds__(256) void ln_fwd_v_kernel(const T* __restrict__ X, int64_t ldx, int64_t M, int d,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, T* __restrict__ Y, int64_t ldy,
                                                       float* __restrict__ mean_out, float* __restrict__ rinv_out) {
  // contraction spelled out (fmaf below, nothing else fused): gemm_dma.h's LayerNorm prologue repeats this
  // arithmetic and must produce the same bits
#pragma clang fp contract(off)
  constexpr int V = Vec<T>::N, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (row >= M) return;
  const T* x = X + row * ldx;
  float v[NCH][V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    load_chunk<T>(v[i], x + (i * LPR + sub) * V);
#pragma unroll
    for (int j = 0; j < V; ++j) s += v[i][j];
  }
  const float mu = group_sum<LPR>(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float u = v[i][j] - mu;
      q = __builtin_fmaf(u, u, q);
    }
  q = group_sum<LPR>(q);
  const float rinv = VAR == 0 ? 1.0f / sqrtf(q / (float)d + eps) : 1.0f / (sqrtf(q / (float)(d - 1)) + eps);
  T* y = Y + row * ldy;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c0 = (i * LPR + sub) * V;
    float gm[V], bt[V], o[V];
    load_chunk<float>(gm, gamma + c0);
    load_chunk<float>(bt, beta + c0);
    if (V == 8) {
      load_chunk<float>(gm + 4, gamma + c0 + 4);
      load_chunk<float>(bt + 4, beta + c0 + 4);
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float u = v[i][j] - mu;
      o[j] = VAR == 0 ? __builtin_fmaf(u * rinv, gm[j], bt[j]) : __builtin_fmaf(gm[j], u * rinv, bt[j]);
    }
    store_chunk<T>(y + c0, o);
  }
  if (sub == 0) {
    mean_out[row] = mu;
    rinv_out[row] = rinv;
  }
}

// backward; the affine partials of each lane's columns are accumulated over all rows the lane
// group visits (grid-stride), combined over the block's row groups in LDS (fixed order) and
// written to part[block][2][d] for the deterministic slab reduce.
// DROP (BERT's backward): the dropout site(s) that consume dX, applied to dX as stored -- 1: out1 = drop(dX; s1)
// (rs_dropout_rowmask without row mask), 2: out1 = drop(dX; s1), out2 = drop(out1; s2) (rs_dropout2) -- with the
// same hash indices (row * d + column) and roundings as those kernels: one launch instead of two.
struct LnDrop {
  float p;
  uint64_t salt1, salt2;
  const uint64_t* seed_base;   // the device step word (graph replays advance it): seeds formed in the kernel
  void* out1;
  void* out2;
};
template <typename T, int LPR, int NCH, int VAR, bool ACC, int DROP = 0>
__global__ __launch_bounds__(256) void ln_bwd_v_kernel(const T* __restrict__ X, int64_t ldx, const T* __restrict__ dY,
                                                       int64_t lddy, int64_t M, int d, const float* __restrict__ gamma,
                                                       const float* __restrict__ mean, const float* __restrict__ rinv,
                                                       float eps, T* __restrict__ dX, int64_t lddx,
                                                       float* __restrict__ part, LnDrop dr = LnDrop{}) {
  constexpr int V = Vec<T>::N, RPW = 64 / LPR, RPB = 4 * RPW;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int rgrp = (threadIdx.x >> 6) * RPW + lane / LPR;  // row group within the block
  uint32_t ds1 = 0u, ds2 = 0u;
  if constexpr (DROP > 0) {
    if (dr.p > 0.f) {
      ds1 = seed32(eff_seed(dr.salt1, dr.seed_base));
      if constexpr (DROP == 2) ds2 = seed32(eff_seed(dr.salt2, dr.seed_base));
    }
  }
  float pg[NCH][V], pb[NCH][V], gm[NCH][V];
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      pg[i][j] = 0.f;
      pb[i][j] = 0.f;
      gm[i][j] = gamma[(i * LPR + sub) * V + j];
    }
  // U rows per lane group per iteration, all their loads issued before any of them is used
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * RPB;
  for (int64_t row0 = (int64_t)blockIdx.x * RPB + rgrp; row0 < M; row0 += stride * U) {
    float xv[U][NCH][V], dyv[U][NCH][V], ov[U][NCH][V], mu[U], ra[U];
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
      const int64_t row = row0 + uu * stride;
      const int64_t rr = row < M ? row : M - 1;
      mu[uu] = mean[rr];
      ra[uu] = rinv[rr];
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int c0 = (i * LPR + sub) * V;
        load_chunk<T>(xv[uu][i], X + rr * ldx + c0);
        load_chunk<T>(dyv[uu][i], dY + rr * lddy + c0);
        if constexpr (ACC) load_chunk<T>(ov[uu][i], dX + rr * lddx + c0);
      }
    }
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
      const int64_t row = row0 + uu * stride;
      const bool valid = row < M;
      const float a = ra[uu];
      float u[NCH][V], gq[NCH][V];
      float sg = 0.f, sgu = 0.f;
#pragma unroll
      for (int i = 0; i < NCH; ++i)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float dy = valid ? dyv[uu][i][j] : 0.f;
          u[i][j] = xv[uu][i][j] - mu[uu];
          gq[i][j] = dy * gm[i][j];
          pg[i][j] += dy * (u[i][j] * a);
          pb[i][j] += dy;
          sg += gq[i][j];
          sgu += gq[i][j] * u[i][j];
        }
      sg = group_sum<LPR>(sg);
      sgu = group_sum<LPR>(sgu);
      const float mg = sg / (float)d;
      float coef;
      if (VAR == 0) {
        coef = a * a * a * sgu / (float)d;
      } else {
        const float sd = 1.0f / a - eps;
        coef = sd > 0.f ? a * a * sgu / ((float)(d - 1) * sd) : 0.f;
      }
      if (valid) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
          const int c0 = (i * LPR + sub) * V;
          float o[V];
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const float t = a * (gq[i][j] - mg) - coef * u[i][j];
            if constexpr (ACC) o[j] = ov[uu][i][j] + t;
            else o[j] = t;
          }
          store_chunk<T>(dX + row * lddx + c0, o);
          if constexpr (DROP > 0) {
            const uint64_t base = (uint64_t)(row * d + c0);
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = to_f(from_f<T>(o[j]));   // dX as stored
            if (dr.p > 0.f) {
#pragma unroll
              for (int j = 0; j < V; j += 2) {
                float m0, m1;
                drop_mul2(dr.p, ds1, base + j, m0, m1);
                o[j] = to_f(from_f<T>(o[j] * m0));
                o[j + 1] = to_f(from_f<T>(o[j + 1] * m1));
              }
            }
            store_chunk<T>(reinterpret_cast<T*>(dr.out1) + row * d + c0, o);
            if constexpr (DROP == 2) {
              if (dr.p > 0.f) {
#pragma unroll
                for (int j = 0; j < V; j += 2) {
                  float m0, m1;
                  drop_mul2(dr.p, ds2, base + j, m0, m1);
                  o[j] *= m0;
                  o[j + 1] *= m1;
                }
              }
              store_chunk<T>(reinterpret_cast<T*>(dr.out2) + row * d + c0, o);
            }
          }
        }
      }
    }
  }
  // combine the RPB row groups: LDS [RPB][d] twice (gamma, beta) in two rounds to bound LDS
  __shared__ float red[RPB * LPR * NCH * V];
  for (int which = 0; which < 2; ++which) {
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int j = 0; j < V; ++j) red[rgrp * d + (i * LPR + sub) * V + j] = which == 0 ? pg[i][j] : pb[i][j];
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += 256) {
      float t = 0.f;
      for (int g = 0; g < RPB; ++g) t += red[g * d + c];
      part[((int64_t)blockIdx.x * 2 + which) * d + c] = t;
    }
    __syncthreads();
  }
}

template <typename T>
static hipError_t ln_fwd_t(const void* X, int64_t ldx, int64_t M, int d, const float* gamma, const float* beta,
                           float eps, int variant, void* Y, int64_t ldy, float* mean, float* rinv, hipStream_t s) {
  const T* x = (const T*)X;
  T* y = (T*)Y;
  {
    constexpr int V = Vec<T>::N;
    const bool vec = (d % V == 0) && (ldx % V == 0) && (ldy % V == 0) && ((uintptr_t)X % 16 == 0) &&
                     ((uintptr_t)Y % 16 == 0) && ((uintptr_t)gamma % 16 == 0) && ((uintptr_t)beta % 16 == 0);
    const int cpr = d / V;
#define LNFV(LPR, NCH)                                                                                       \
  do {                                                                                                       \
    if (variant == 0)                                                                                        \
      hipLaunchKernelGGL((ln_fwd_v_kernel<T, LPR, NCH, 0>), dim3((unsigned)cdiv(M, 4 * (64 / LPR))), dim3(256), \
                         0, s, x, ldx, M, d, gamma, beta, eps, y, ldy, mean, rinv);                          \
    else                                                                                                     \
      hipLaunchKernelGGL((ln_fwd_v_kernel<T, LPR, NCH, 1>), dim3((unsigned)cdiv(M, 4 * (64 / LPR))), dim3(256), \
                         0, s, x, ldx, M, d, gamma, beta, eps, y, ldy, mean, rinv);                          \
  } while (0)
    if (vec) {
      if (cpr == 4) { LNFV(4, 1); return hipGetLastError(); }
      if (cpr == 8) { LNFV(8, 1); return hipGetLastError(); }
      if (cpr == 16) { LNFV(16, 1); return hipGetLastError(); }
      if (cpr == 32) { LNFV(32, 1); return hipGetLastError(); }
      if (cpr == 64) { LNFV(64, 1); return hipGetLastError(); }
      if (cpr == 128) { LNFV(64, 2); return hipGetLastError(); }
    }
#undef LNFV
  }
  dim3 grid((unsigned)cdiv(M, 4)), block(256);
#define LNF(NV) hipLaunchKernelGGL((ln_fwd_kernel<T, NV>), grid, block, 0, s, x, ldx, M, d, gamma, beta, eps, variant, y, ldy, mean, rinv)
  if (d <= 64) LNF(1);
  else if (d <= 128) LNF(2);
  else if (d <= 256) LNF(4);
  else if (d <= 512) LNF(8);
  else LNF(16);
#undef LNF
  return hipGetLastError();
}

template <typename T>
static hipError_t ln_bwd_t(const void* X, int64_t ldx, const void* dY, int64_t lddy, int64_t M, int d,
                           const float* gamma, const float* mean, const float* rinv, float eps, int variant,
                           void* dX, int64_t lddx, int acc, float* dgamma, float* dbeta, float* ws, hipStream_t s,
                           int drop = 0, LnDrop dr = LnDrop{}) {
  const T* x = (const T*)X;
  const T* dy = (const T*)dY;
  T* dx = (T*)dX;
  {
    constexpr int V = Vec<T>::N;
    const bool vec = (d % V == 0) && (ldx % V == 0) && (lddy % V == 0) && (lddx % V == 0) &&
                     ((uintptr_t)X % 16 == 0) && ((uintptr_t)dY % 16 == 0) && ((uintptr_t)dX % 16 == 0);
    const int cpr = d / V;
    int lpr = 0, nch = 1;
    if (vec) {
      if (cpr == 4 || cpr == 8 || cpr == 16 || cpr == 32 || cpr == 64) lpr = cpr;
      else if (cpr == 128) { lpr = 64; nch = 2; }
    }
    if (lpr) {
      const int64_t rpb = 4 * (64 / lpr);
      // every row group's rows in ONE iteration of 4 (one dependent round trip per workgroup): up to 512
      // workgroups (cfg3, 12,800 rows of 256: 400 -- 256 ran two iterations each)
      const int nb = (int)std::min<int64_t>(LN_BWD_BLOCKS, cdiv(M, rpb * 4));
#define LNBV1D(LPR, NCH, VAR, ACC, DR)                                                                      \
  hipLaunchKernelGGL((ln_bwd_v_kernel<T, LPR, NCH, VAR, ACC, DR>), dim3(nb), dim3(256), 0, s, x, ldx, dy, lddy, M, \
                     d, gamma, mean, rinv, eps, dx, lddx, ws, dr)
#define LNBV1(LPR, NCH, VAR, ACC)                     \
  do {                                                \
    if (drop == 0) LNBV1D(LPR, NCH, VAR, ACC, 0);     \
    else if (drop == 1) LNBV1D(LPR, NCH, VAR, ACC, 1); \
    else LNBV1D(LPR, NCH, VAR, ACC, 2);               \
  } while (0)
#define LNBV(LPR, NCH)                                                \
  do {                                                                \
    if (variant == 0) {                                               \
      if (acc) LNBV1(LPR, NCH, 0, true); else LNBV1(LPR, NCH, 0, false); \
    } else {                                                          \
      if (acc) LNBV1(LPR, NCH, 1, true); else LNBV1(LPR, NCH, 1, false); \
    }                                                                 \
  } while (0)
      if (lpr == 4) LNBV(4, 1);
      else if (lpr == 8) LNBV(8, 1);
      else if (lpr == 16) LNBV(16, 1);
      else if (lpr == 32) LNBV(32, 1);
      else if (nch == 1) LNBV(64, 1);
      else LNBV(64, 2);
#undef LNBV
#undef LNBV1
#undef LNBV1D
      hipError_t e = hipGetLastError();
      if (e != hipSuccess || !(dgamma || dbeta)) return e;
      return launch_reduce_slabs(ws, nb, 2 * (int64_t)d, d, dgamma, dbeta, 1, s);
    }
  }
  if (drop) return hipErrorInvalidValue;   // the dropout epilogue is the vectorised path's (callers fall back)
  const int nblk = (int)std::min<int64_t>(LN_BWD_BLOCKS, cdiv(M, 4));
  dim3 grid(nblk), block(256);
#define LNB(NV) hipLaunchKernelGGL((ln_bwd_kernel<T, NV>), grid, block, 0, s, x, ldx, dy, lddy, M, d, gamma, mean, rinv, eps, variant, dx, lddx, acc, ws)
  if (d <= 64) LNB(1);
  else if (d <= 128) LNB(2);
  else if (d <= 256) LNB(4);
  else if (d <= 512) LNB(8);
  else LNB(16);
#undef LNB
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !(dgamma || dbeta)) return e;
  return launch_reduce_slabs(ws, nblk, 2 * (int64_t)d, d, dgamma, dbeta, 1, s);
}

extern "C" {

int rs_layernorm_fwd(int dtype, int variant, const void* X, int64_t ldx, int64_t M, int64_t d,
                     const float* gamma, const float* beta, float eps, void* Y, int64_t ldy,
                     float* mean, float* rinv, void* stream) {
  if (M <= 0 || d <= 1 || d > 64 * LN_MAXV) return RS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  return (int)(dtype == RS_DTYPE_BF16
                   ? ln_fwd_t<__bf16>(X, ldx, M, (int)d, gamma, beta, eps, variant, Y, ldy, mean, rinv, s)
                   : ln_fwd_t<float>(X, ldx, M, (int)d, gamma, beta, eps, variant, Y, ldy, mean, rinv, s));
}

int64_t rs_layernorm_bwd_nparts(int dtype, int64_t M, int64_t d) {
  const int V = dtype == RS_DTYPE_BF16 ? Vec<__bf16>::N : Vec<float>::N;
  if (M <= 0 || d <= 1 || d % V) return 0;
  const int64_t cpr = d / V;
  const int64_t lpr = (cpr == 4 || cpr == 8 || cpr == 16 || cpr == 32 || cpr == 64) ? cpr : cpr == 128 ? 64 : 0;
  if (!lpr) return 0;
  const int64_t rpb = 4 * (64 / lpr);
  return std::min<int64_t>(LN_BWD_BLOCKS, cdiv(M, rpb * 4));
}

int rs_layernorm_bwd_drop(int dtype, int variant, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                          int64_t M, int64_t d, const float* gamma, const float* mean, const float* rinv, float eps,
                          void* dX, int64_t lddx, int accumulate_dx, float* dgamma, float* dbeta, float* ws,
                          float drop_p, uint64_t salt1, uint64_t salt2, const uint64_t* seed_base, void* out1,
                          void* out2, void* stream) {
  if (M <= 0 || d <= 1 || d > 64 * LN_MAXV || !out1) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int drop = out2 ? 2 : 1;
  const int V = dtype == RS_DTYPE_BF16 ? 8 : 4;
  const bool al = ((uintptr_t)out1 | (uintptr_t)(out2 ? out2 : out1)) % 16 == 0 && d % V == 0;
  if (al) {
    const LnDrop dr{drop_p, salt1, salt2, seed_base, out1, out2};
    const hipError_t e =
        dtype == RS_DTYPE_BF16
            ? ln_bwd_t<__bf16>(X, ldx, dY, lddy, M, (int)d, gamma, mean, rinv, eps, variant, dX, lddx, accumulate_dx,
                               dgamma, dbeta, ws, s, drop, dr)
            : ln_bwd_t<float>(X, ldx, dY, lddy, M, (int)d, gamma, mean, rinv, eps, variant, dX, lddx, accumulate_dx,
                              dgamma, dbeta, ws, s, drop, dr);
    if (e != hipErrorInvalidValue) return (int)e;
  }
  // not the vectorised path: the two launches (same results)
  if (int r = rs_layernorm_bwd(dtype, variant, X, ldx, dY, lddy, M, d, gamma, mean, rinv, eps, dX, lddx,
                               accumulate_dx, dgamma, dbeta, ws, stream))
    return r;
  return out2 ? rs_dropout2(dtype, dX, M, d, lddx, drop_p, salt1, salt2, seed_base, d, out1, out2, stream)
              : rs_dropout_rowmask(dtype, dX, M, d, lddx, drop_p, salt1, seed_base, d, nullptr, out1, nullptr, stream);
}

int rs_layernorm_bwd(int dtype, int variant, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                     int64_t M, int64_t d, const float* gamma, const float* mean, const float* rinv, float eps,
                     void* dX, int64_t lddx, int accumulate_dx, float* dgamma, float* dbeta, float* ws,
                     void* stream) {
  if (M <= 0 || d <= 1 || d > 64 * LN_MAXV) return RS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  return (int)(dtype == RS_DTYPE_BF16
                   ? ln_bwd_t<__bf16>(X, ldx, dY, lddy, M, (int)d, gamma, mean, rinv, eps, variant, dX, lddx,
                                      accumulate_dx, dgamma, dbeta, ws, s)
                   : ln_bwd_t<float>(X, ldx, dY, lddy, M, (int)d, gamma, mean, rinv, eps, variant, dX, lddx,
                                     accumulate_dx, dgamma, dbeta, ws, s));
}

}  // extern "C"
