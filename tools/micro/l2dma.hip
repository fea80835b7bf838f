// Micro-benchmark: LDS-DMA (global_load_lds_dwordx4) read bandwidth from an L2 / MALL-resident footprint for the
// stage-piece shapes of the DMA GEMMs: 16 rows x 64 B (a 32-deep bf16 k stage of 512-B rows, gemm_dma.h kc_piece),
// 8 rows x 128 B (a 64-deep stage), 1 KB contiguous.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/l2dma.hip -o tools/micro/l2dma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void* lds_vptr;
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)(lds_vptr)p; }
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}

template <int PAT>
__global__ __launch_bounds__(256) void dmark(const char* __restrict__ x, uint64_t pieces, int iters, int* out) {
  __shared__ __attribute__((aligned(1024))) char lds[4][8][1024];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = blockIdx.x * 4ull + wave, nw = gridDim.x * 4ull;
  const uint32_t base = lds_u32(&lds[wave][0][0]);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t c = (gw + (uint64_t)(it * 8 + u) * nw) % pieces;
      uint64_t off;
      if (PAT == 0) off = c * 1024 + lane * 16;                                            // contiguous
      else if (PAT == 1) off = (c >> 3) * 8192 + (lane >> 2) * 512 + (c & 7) * 64 + (lane & 3) * 16;   // 16 x 64 B
      else off = (c >> 2) * 4096 + (lane >> 3) * 512 + (c & 3) * 128 + (lane & 7) * 16;      // 8 x 128 B
      dma16(x + off, __builtin_amdgcn_readfirstlane(base + u * 1024));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (lds[wave][lane & 7][lane] == 0x7f && iters < 0) out[0] = 1;
}

int main() {
  const uint64_t maxb = 256ull << 20;
  char* x;
  int* o;
  hipMalloc(&x, maxb);
  hipMalloc(&o, 4);
  hipMemset(x, 1, maxb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t sizes[] = {2ull << 20, 8ull << 20, 64ull << 20};
  const char* names[] = {"contiguous 1KB", "16 rows x 64B", "8 rows x 128B"};
  for (uint64_t S : sizes)
    for (int wgs : {256, 768, 1536})
      for (int pat = 0; pat < 3; ++pat) {
        const uint64_t pieces = S / 1024;
        const int iters = (int)((2ull << 30) / (1024ull * wgs * 4 * 8));
        auto launch = [&] {
          if (pat == 0) hipLaunchKernelGGL((dmark<0>), dim3(wgs), dim3(256), 0, 0, x, pieces, iters, o);
          else if (pat == 1) hipLaunchKernelGGL((dmark<1>), dim3(wgs), dim3(256), 0, 0, x, pieces, iters, o);
          else hipLaunchKernelGGL((dmark<2>), dim3(wgs), dim3(256), 0, 0, x, pieces, iters, o);
        };
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 5.0 * 1024.0 * wgs * 4 * 8 * iters;
        printf("%-15s footprint %4.0f MB  wgs %5d  %7.2f TB/s\n", names[pat], S / 1048576.0, wgs,
               bytes / (ms * 1e-3) / 1e12);
      }
  return 0;
}
