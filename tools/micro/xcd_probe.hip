// XCD placement / L2 locality probe.  (1) Which XCD (s_getreg HW_REG_XCC_ID) each block of a 256-block launch lands
// on, over several launches: is block b -> XCD a fixed function of b % 8?  (2) A producer kernel writes a 26 MB
// activation-sized buffer, block w writing chunk w % 8; a consumer then reads it (64 KB per block, the row-chain
// prologue's burst) with block w reading chunk (w + s) % 8 for s = 0 (same XCD as the writer) and s = 1..7: how much
// faster is an XCD-local read right after its producer?
//   hipcc --offload-arch=gfx950 -O3 tools/micro/xcd_probe.hip -o tools/micro/xcd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
__global__ void where(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}
typedef __attribute__((ext_vector_type(4))) unsigned u4;
// buffer = 8 chunks; block w handles rows of chunk (w + shift) % 8, local index w / 8
__global__ __launch_bounds__(512) void produce(u4* buf, int64_t chunk_u4, int shift) {
  const int w = blockIdx.x, c = (w + shift) & 7, l = w >> 3, nl = gridDim.x >> 3;
  u4* p = buf + c * chunk_u4;
  for (int64_t i = l * 512 + threadIdx.x; i < chunk_u4; i += (int64_t)nl * 512) p[i] = (u4){(unsigned)i, 1u, 2u, 3u};
}
__global__ __launch_bounds__(512) void consume(const u4* buf, int64_t chunk_u4, int shift, int per_thread, u4* sink,
                                               unsigned long long* t) {
  const int w = blockIdx.x, c = (w + shift) & 7, l = w >> 3, nl = gridDim.x >> 3;
  const u4* p = buf + c * chunk_u4;
  unsigned long long t0 = wall_clock64();
  u4 acc = {0, 0, 0, 0};
  u4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t i = (l * 8 + k) * 512 + threadIdx.x;   // 8 x 16 B per thread = 64 KB per block
    v[k] = p[i % chunk_u4];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) acc += v[k];
  if (acc.x == 0xdeadbeef) sink[0] = acc;
  __syncthreads();
  if (threadIdx.x == 0) t[w] = wall_clock64() - t0;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 4096 * 4);
  std::vector<unsigned> h(4096);
  int fixed = 1;
  for (int it = 0; it < 6; ++it) {
    hipLaunchKernelGGL(where, dim3(256), dim3(512), 0, 0, d);
    hipMemcpy(h.data(), d, 256 * 4, hipMemcpyDeviceToHost);
    printf("launch %d: block 0..15 -> xcc", it);
    for (int b = 0; b < 16; ++b) printf(" %u", h[b]);
    int ok = 1;
    for (int b = 8; b < 256; ++b) ok &= h[b] == h[b % 8];
    printf("  (b and b%%8 share an XCC: %s)\n", ok ? "yes" : "NO");
    static unsigned first[8];
    if (it == 0) for (int b = 0; b < 8; ++b) first[b] = h[b];
    for (int b = 0; b < 8; ++b) fixed &= h[b] == first[b];
  }
  printf("block %% 8 -> xcc fixed across launches: %s\n", fixed ? "yes" : "NO");
  const int64_t bytes = 26214400, chunk_u4 = bytes / 16 / 8;
  u4 *buf, *sink;
  unsigned long long* t;
  hipMalloc(&buf, bytes);
  hipMalloc(&sink, 64);
  hipMalloc(&t, 256 * 8);
  std::vector<unsigned long long> ht(256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int s = 0; s < 8; ++s) {
    double ev = 0, med = 0;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(produce, dim3(256), dim3(512), 0, 0, buf, chunk_u4, 0);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(consume, dim3(256), dim3(512), 0, 0, buf, chunk_u4, s, 8, sink, t);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ev += ms * 1e3 / reps;
      hipMemcpy(ht.data(), t, 256 * 8, hipMemcpyDeviceToHost);
      std::vector<unsigned long long> v(ht);
      std::sort(v.begin(), v.end());
      med += v[128] * 0.01 / reps;   // 100 MHz ticks -> us
    }
    printf("consumer reads chunk (w + %d) %% 8 of the producer's (w %% 8): event %.2f us, block read p50 %.2f us\n", s,
           ev, med);
  }
  return 0;
}
