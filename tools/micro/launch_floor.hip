// Per-launch floor on MI355X: back-to-back launches of near-empty kernels, timed with hipEvents.
//   hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o launch_floor && ./launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1234567) p[0] = 1;
}
__global__ void lds_kernel(int* p) {
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (s[(threadIdx.x + 1) % blockDim.x] == 1234567) p[0] = 1;
}
__global__ void touch_kernel(const int4* __restrict__ src, int4* __restrict__ dst, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  int* d;
  hipMalloc(&d, 64 << 20);
  hipFuncSetAttribute((const void*)lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  printf("empty 1x64:          %7.2f us\n", timeit([&] { hipLaunchKernelGGL(empty_kernel, 1, 64, 0, 0, d); }, 200));
  printf("empty 256x512:       %7.2f us\n", timeit([&] { hipLaunchKernelGGL(empty_kernel, 256, 512, 0, 0, d); }, 200));
  printf("empty 2048x256:      %7.2f us\n", timeit([&] { hipLaunchKernelGGL(empty_kernel, 2048, 256, 0, 0, d); }, 200));
  for (int kb : {0, 32, 64, 128, 150}) {
    printf("lds %3d KB 256x512:  %7.2f us\n", kb,
           timeit([&] { hipLaunchKernelGGL(lds_kernel, 256, 512, kb * 1024, 0, d); }, 200));
  }
  const long n = (6553600) / 16;
  int4* src = (int4*)d;
  int4* dst = (int4*)(d + (16 << 20) / 4 * 1);
  printf("copy 6.5MB:          %7.2f us\n",
         timeit([&] { hipLaunchKernelGGL(touch_kernel, (unsigned)((n + 255) / 256), 256, 0, 0, src, dst, n); }, 200));
  return 0;
}
