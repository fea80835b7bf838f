// Cold instruction-fetch cost on MI355X: the same VALU work as one long straight-line body (~32 KB of
// code) vs a rolled loop (a few dozen bytes), 256 workgroups x 512 threads, hipEvent-timed.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ __launch_bounds__(512) void big_kernel(float* out, float a) {
  float x = a + threadIdx.x, y = a * 2.f;
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(y));
  if (x == 12345.f) out[0] = x;
}
__global__ __launch_bounds__(512) void loop_kernel(float* out, float a, int n) {
  float x = a + threadIdx.x, y = a * 2.f;
#pragma unroll 1
  for (int i = 0; i < n; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(y));
  if (x == 12345.f) out[0] = x;
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  float* d;
  hipMalloc(&d, 4096);
  printf("big 4000 (32 KB code): %7.2f us\n", timeit([&] { hipLaunchKernelGGL(big_kernel<4000>, 256, 512, 0, 0, d, 1.f); }, 100));
  printf("big 1000 ( 8 KB code): %7.2f us\n", timeit([&] { hipLaunchKernelGGL(big_kernel<1000>, 256, 512, 0, 0, d, 1.f); }, 100));
  printf("loop 4000:             %7.2f us\n", timeit([&] { hipLaunchKernelGGL(loop_kernel, 256, 512, 0, 0, d, 1.f, 4000); }, 100));
  printf("loop 1000:             %7.2f us\n", timeit([&] { hipLaunchKernelGGL(loop_kernel, 256, 512, 0, 0, d, 1.f, 1000); }, 100));
  // alternate two different big kernels so neither stays warm in the instruction cache
  printf("big 4000 alternating with big 3999: %7.2f us per launch\n", timeit([&] {
           hipLaunchKernelGGL(big_kernel<4000>, 256, 512, 0, 0, d, 1.f);
           hipLaunchKernelGGL(big_kernel<3999>, 256, 512, 0, 0, d, 1.f);
         }, 100) / 2);
  return 0;
}
