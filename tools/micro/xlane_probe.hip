// Cross-lane reduction forms (common.h): the permlane / DPP versions against the __shfl_xor butterflies they
// replace, bit for bit, on random data with all lanes active.
//   hipcc --offload-arch=gfx950 -O3 -I recommender-baseline-model_amd/csrc tools/micro/xlane_probe.hip -o tools/micro/xlane_probe
#include "common.h"
#include <cstdio>
#include <vector>
#include <random>

__global__ void probe(const float* in, unsigned* bad) {
  const float v = in[blockIdx.x * 64 + threadIdx.x];
  float a = v, b = v;
  a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
  b = add_xor32(add_xor16(b));
  if (__builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b)) atomicAdd(&bad[0], 1u);
  a = v; b = v;
  a = fmaxf(a, __shfl_xor(a, 16, 64)); a = fmaxf(a, __shfl_xor(a, 32, 64));
  b = max_xor32(max_xor16(b));
  if (a != b) atomicAdd(&bad[1], 1u);
  a = v; b = v;
  for (int o = 1; o < 16; o <<= 1) a += __shfl_xor(a, o, 64);
  b = row16_sum_up(b);
  if (__builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b)) atomicAdd(&bad[2], 1u);
  a = v; b = v;
  for (int o = 8; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  b = group16_sum_full(b);
  if (__builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b)) atomicAdd(&bad[3], 1u);
  a = v; b = v;
  a += __shfl_xor(a, 16, 64);
  b = add_xor16(b);
  if (__builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b)) atomicAdd(&bad[4], 1u);
  a = v; b = v;
  a += __shfl_xor(a, 32, 64);
  b = add_xor32(b);
  if (__builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b)) atomicAdd(&bad[5], 1u);
}

int main() {
  const int n = 4096 * 64;
  std::vector<float> h(n);
  std::mt19937 g(1);
  std::normal_distribution<float> d;
  for (auto& x : h) x = d(g);
  float* in;
  unsigned* bad;
  hipMalloc(&in, n * 4);
  hipMalloc(&bad, 64);
  hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice);
  hipMemset(bad, 0, 64);
  hipLaunchKernelGGL(probe, dim3(4096), dim3(64), 0, 0, in, bad);
  unsigned hb[6];
  hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
  printf("mismatching lanes of %d: add16+32 %u, max16+32 %u, row16_sum_up %u, group16_sum_full %u, add16 %u, add32 %u\n",
         n, hb[0], hb[1], hb[2], hb[3], hb[4], hb[5]);
  return 0;
}
