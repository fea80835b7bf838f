// Loader-wave flag hand-off probe (rowchain.hip WLoad / WReady): wave 7 of each 8-wave workgroup publishes three LDS
// flags after (mode 0) nothing, (mode 1) LDS-DMA of three 32 KB images as WLoad does; the other waves spin on them
// (bounded) and record the spins each flag took (-1: not seen).
//   hipcc --offload-arch=gfx950 -O3 -I include -I recommender-baseline-model_amd/csrc tools/micro/flag_probe.hip -o tools/micro/flag_probe
#include "../../recommender-baseline-model_amd/csrc/rowchain.hip"
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void probe(int mode, const __bf16* W, int* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int* wflag = reinterpret_cast<int*>(smem + 3 * 32768 + 4096);
  const __bf16* const Ws[3] = {W, W + 128 * 128, W + 2 * 128 * 128};
  const int64_t ldw[3] = {128, 128, 128};
  if (mode >= 1 && wave == rc::LOADER) rc::WLoad<128>::prime(smem, Ws, ldw, lane);
  if (tid < 3) wflag[tid] = 0;
  rc::lds_barrier();
  if (wave == rc::LOADER) {
    if (mode >= 1) rc::WLoad<128>::stream(smem, Ws, ldw, wflag, lane);
    else for (int m = 0; m < 3; ++m) rc::publish(wflag, m, lane);
    return;
  }
  for (int m = 0; m < 3; ++m) {
    int spin = 0;
    while (spin < (1 << 16) && __hip_atomic_load(&wflag[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      __builtin_amdgcn_s_sleep(1);
      ++spin;
    }
    if (lane == 0) out[(blockIdx.x * 8 + wave) * 3 + m] = spin < (1 << 16) ? spin : -1;
  }
}

int main() {
  __bf16* W;
  int* out;
  hipMalloc(&W, 3 * 128 * 128 * 2);
  hipMemset(W, 0x3c, 3 * 128 * 128 * 2);
  hipMalloc(&out, 256 * 8 * 3 * 4);
  const size_t lds = 3 * 32768 + 4096 + 16;
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(out, 0x7f, 256 * 8 * 3 * 4);
    hipLaunchKernelGGL(probe, dim3(256), dim3(512), lds, 0, mode, (const __bf16*)W, out);
    hipError_t e = hipDeviceSynchronize();
    std::vector<int> h(256 * 8 * 3);
    hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
    int miss[3] = {0, 0, 0}, maxs[3] = {0, 0, 0};
    for (int b = 0; b < 256; ++b)
      for (int w = 0; w < 7; ++w)
        for (int m = 0; m < 3; ++m) {
          const int v = h[(b * 8 + w) * 3 + m];
          if (v < 0) ++miss[m];
          else if (v > maxs[m]) maxs[m] = v;
        }
    printf("mode %d (%s): missed %d/%d/%d of 1792, max spins %d/%d/%d\n", mode, hipGetErrorString(e), miss[0],
           miss[1], miss[2], maxs[0], maxs[1], maxs[2]);
  }
  return 0;
}
