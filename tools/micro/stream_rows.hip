// Micro-benchmark: streaming row kernels over a (25600 x 128) bf16 matrix (the SAS cfg2
// activation), to find what bounds the row-wise kernels (LayerNorm, embedding, elementwise).
// Build: hipcc --offload-arch=gfx950 -O3 stream_rows.hip -o stream_rows
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "recsys_hip.h"
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;

__global__ __launch_bounds__(256) void copy1(const bf16x8* __restrict__ x, bf16x8* __restrict__ y, long n) {
  long i = blockIdx.x * 256L + threadIdx.x;
  if (i < n) y[i] = x[i];
}
template <int U>
__global__ __launch_bounds__(256) void copyU(const bf16x8* __restrict__ x, bf16x8* __restrict__ y, long n) {
  long i0 = (blockIdx.x * 256L) * U + threadIdx.x;
  bf16x8 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (i0 + u * 256 < n) v[u] = x[i0 + u * 256];
#pragma unroll
  for (int u = 0; u < U; ++u) if (i0 + u * 256 < n) y[i0 + u * 256] = v[u];
}
__global__ __launch_bounds__(256) void copy_gs(const bf16x8* __restrict__ x, bf16x8* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) y[i] = x[i];
}
// LayerNorm-like: 16 lanes per row, shuffles, gamma/beta
template <bool VECGB>
__global__ __launch_bounds__(256) void lnlike(const bf16x8* __restrict__ x, bf16x8* __restrict__ y,
                                              const float* __restrict__ gm, const float* __restrict__ bt, long rows) {
  const int lane = threadIdx.x & 63, sub = lane & 15;
  long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + lane / 16;
  if (row >= rows) return;
  bf16x8 v = x[row * 16 + sub];
  float f[8], s = 0.f;
  for (int j = 0; j < 8; ++j) { f[j] = (float)v[j]; s += f[j]; }
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  float mu = s / 128.f, q = 0.f;
  for (int j = 0; j < 8; ++j) { float u = f[j] - mu; q += u * u; }
  for (int o = 8; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  float r = 1.f / sqrtf(q / 128.f + 1e-8f);
  float g[8], b[8];
  if (VECGB) {
    f4 g0 = *(const f4*)(gm + sub * 8), g1 = *(const f4*)(gm + sub * 8 + 4);
    f4 b0 = *(const f4*)(bt + sub * 8), b1 = *(const f4*)(bt + sub * 8 + 4);
    for (int j = 0; j < 4; ++j) { g[j] = g0[j]; g[j + 4] = g1[j]; b[j] = b0[j]; b[j + 4] = b1[j]; }
  } else {
    for (int j = 0; j < 8; ++j) { g[j] = gm[sub * 8 + j]; b[j] = bt[sub * 8 + j]; }
  }
  bf16x8 o;
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)((f[j] - mu) * r * g[j] + b[j]);
  y[row * 16 + sub] = o;
}

int main() {
  const long rows = 25600, n = rows * 16;  // 16 chunks of 8 bf16 per row
  bf16x8 *x, *y;
  float *g, *b;
  hipMalloc(&x, n * 16); hipMalloc(&y, n * 16); hipMalloc(&g, 512); hipMalloc(&b, 512);
  hipMemset(x, 0, n * 16); hipMemset(g, 0, 512); hipMemset(b, 0, 512);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto T = [&](const char* name, auto launch) {
    for (int i = 0; i < 10; ++i) launch();
    hipEventRecord(e0);
    const int R = 200;
    for (int i = 0; i < R; ++i) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double us = ms * 1e3 / R;
    printf("%-40s %8.2f us  %7.0f GB/s\n", name, us, 2.0 * n * 16 / (us * 1e-6) / 1e9);
  };
  T("copy 1 chunk/thread (1600 blk)", [&] { copy1<<<(n + 255) / 256, 256>>>(x, y, n); });
  T("copy 4 chunks/thread (400 blk)", [&] { copyU<4><<<(n + 1023) / 1024, 256>>>(x, y, n); });
  T("copy 8 chunks/thread (200 blk)", [&] { copyU<8><<<(n + 2047) / 2048, 256>>>(x, y, n); });
  T("copy grid-stride 1024 blk", [&] { copy_gs<<<1024, 256>>>(x, y, n); });
  T("copy grid-stride 2048 blk", [&] { copy_gs<<<2048, 256>>>(x, y, n); });
  T("lnlike scalar gamma (1600 blk)", [&] { lnlike<false><<<(rows + 15) / 16, 256>>>(x, y, g, b, rows); });
  T("lnlike vec gamma (1600 blk)", [&] { lnlike<true><<<(rows + 15) / 16, 256>>>(x, y, g, b, rows); });
  float *mu, *ri; hipMalloc(&mu, rows * 4); hipMalloc(&ri, rows * 4);
  T("rs_layernorm_fwd (library)", [&] { rs_layernorm_fwd(1, 0, x, 128, rows, 128, g, b, 1e-8f, y, 128, mu, ri, nullptr); });
  __bf16 *W; hipMalloc(&W, 128 * 128 * 2); hipMemset(W, 0, 128 * 128 * 2);
  T("rs_gemm d->d (library)", [&] { rs_gemm(1, 0, 0, rows, 128, 128, x, 128, W, 128, y, 128, 0, nullptr, 1, nullptr, nullptr); });
  // bigger problem: 8x (to see size effects)
  bf16x8 *X, *Y; long N = n * 8; hipMalloc(&X, N * 16); hipMalloc(&Y, N * 16); hipMemset(X, 0, N * 16);
  for (int i = 0; i < 10; ++i) copy1<<<(N + 255) / 256, 256>>>(X, Y, N);
  hipEventRecord(e0); for (int i = 0; i < 50; ++i) copy1<<<(N + 255) / 256, 256>>>(X, Y, N); hipEventRecord(e1);
  hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("%-40s %8.2f us  %7.0f GB/s\n", "copy 8x size (52 MB each way)", ms * 1e3 / 50, 2.0 * N * 16 / (ms * 1e-3 / 50) / 1e9);
  return 0;
}
