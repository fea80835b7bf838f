// Micro-benchmark: aggregate read bandwidth of the cache hierarchy as seen by the CUs, for the
// access patterns of the bf16 GEMMs: (a) coalesced (a wave's 64 lanes read 1 KB contiguous),
// (b) MFMA-fragment pattern (lane l reads 16 B of row l%16 at 16-B chunk l/16 + 4j: one load
// instruction touches 16 rows x 64 B, row stride 512 B), over a footprint that is L2-resident
// (2 MB), MALL-resident (96 MB) or HBM (2 GB).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/l2bw.hip -o tools/micro/l2bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

template <int PAT, int U>
__global__ __launch_bounds__(256) void rd(const u4* __restrict__ x, uint64_t chunks_1k, int iters, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (blockIdx.x * 4ull + (threadIdx.x >> 6));
  const uint64_t nw = gridDim.x * 4ull;
  u4 acc = {0, 0, 0, 0};
  // lane offset inside a 1 KB piece (in 16 B units)
  int off;
  if (PAT == 0) off = lane;                               // contiguous
  else off = (lane & 15) * 32 + (lane >> 4);              // 16 rows (512 B stride) x 4 chunks of 16 B
  for (int it = 0; it < iters; ++it) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t c = (wave + (uint64_t)(it * U + u) * nw) % chunks_1k;
      if (PAT == 0) v[u] = x[c * 64 + off];
      else {
        // 8 instructions per 8 KB "tile" (16 rows x 512 B): piece c selects tile c/8, step c%8 -> chunk 4*(c%8)
        const uint64_t tile = c >> 3, step = c & 7;
        v[u] = x[tile * 512 + off + step * 4];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

int main() {
  const uint64_t maxb = 2ull << 30;
  u4* x;
  uint32_t* o;
  hipMalloc(&x, maxb);
  hipMalloc(&o, 4);
  hipMemset(x, 1, maxb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t sizes[] = {2ull << 20, 96ull << 20, 2ull << 30};
  for (int pat = 0; pat < 2; ++pat)
    for (uint64_t S : sizes)
      for (int wgs : {256, 512, 1024, 2048}) {
        const uint64_t chunks = S / 1024;
        const int U = 8;
        // ~4 GB of loads per launch
        const int iters = (int)((4ull << 30) / (1024ull * wgs * 4 * U));
        auto launch = [&] {
          if (pat == 0) hipLaunchKernelGGL((rd<0, 8>), dim3(wgs), dim3(256), 0, 0, x, chunks, iters, o);
          else hipLaunchKernelGGL((rd<1, 8>), dim3(wgs), dim3(256), 0, 0, x, chunks, iters, o);
        };
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 5.0 * 1024.0 * wgs * 4 * U * iters;
        printf("%-11s footprint %6.0f MB  wgs %5d  %8.2f TB/s\n", pat ? "frag16x64B" : "contiguous", S / 1048576.0,
               wgs, bytes / (ms * 1e-3) / 1e12);
      }
  return 0;
}
