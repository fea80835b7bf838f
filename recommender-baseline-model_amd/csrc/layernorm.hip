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

__global__ void ln_affine_reduce_kernel(const float* __restrict__ part, int nblk, int d, float* __restrict__ dgamma,
                                        float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * d) return;
  const int which = c / d, col = c % d;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[((int64_t)b * 2 + which) * d + col];
  float* dst = which == 0 ? dgamma : dbeta;
  if (dst) dst[col] += s;
}

template <typename T>
static hipError_t ln_fwd_t(const void* X, int64_t ldx, int64_t M, int d, const float* gamma, const float* beta,
                           float eps, int variant, void* Y, int64_t ldy, float* mean, float* rinv, hipStream_t s) {
  dim3 grid((unsigned)cdiv(M, 4)), block(256);
  const T* x = (const T*)X;
  T* y = (T*)Y;
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
                           void* dX, int64_t lddx, int acc, float* dgamma, float* dbeta, float* ws, hipStream_t s) {
  const int nblk = (int)std::min<int64_t>(256, cdiv(M, 4));
  dim3 grid(nblk), block(256);
  const T* x = (const T*)X;
  const T* dy = (const T*)dY;
  T* dx = (T*)dX;
#define LNB(NV) hipLaunchKernelGGL((ln_bwd_kernel<T, NV>), grid, block, 0, s, x, ldx, dy, lddy, M, d, gamma, mean, rinv, eps, variant, dx, lddx, acc, ws)
  if (d <= 64) LNB(1);
  else if (d <= 128) LNB(2);
  else if (d <= 256) LNB(4);
  else if (d <= 512) LNB(8);
  else LNB(16);
#undef LNB
  if (dgamma || dbeta)
    hipLaunchKernelGGL(ln_affine_reduce_kernel, dim3((unsigned)cdiv(2 * d, 256)), dim3(256), 0, s, ws, nblk, d,
                       dgamma, dbeta);
  return hipGetLastError();
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
