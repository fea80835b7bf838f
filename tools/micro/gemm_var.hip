// Micro-benchmark of rs_gemm variants at the SAS cfg2 shape (M=25600, N=K=128, bf16) through the
// C ABI, hipEvent-timed back-to-back launches (device time per call).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "recsys_hip.h"
int main() {
  const long M = 25600, N = 128, K = 128;
  __bf16 *x, *w, *y, *r; float *b; long *ids; unsigned long long *sb;
  hipMalloc(&x, M * K * 2); hipMalloc(&w, N * K * 4); hipMalloc(&y, M * 4 * N * 2); hipMalloc(&r, M * N * 2);
  hipMalloc(&b, 4 * N * 4); hipMalloc(&ids, M * 8); hipMalloc(&sb, 8);
  hipMemset(x, 0x3c, M * K * 2); hipMemset(w, 0x3c, N * K * 4); hipMemset(r, 0, M * N * 2); hipMemset(b, 0, 4 * N * 4);
  hipMemset(ids, 1, M * 8); hipMemset(sb, 0, 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto T = [&](const char* name, rs_epilogue* ep, long n = N) {
    for (int i = 0; i < 10; ++i) rs_gemm(1, 0, 0, M, n, K, x, K, w, K, y, n, 0, ep, 1, nullptr, nullptr);
    hipEventRecord(e0);
    for (int i = 0; i < 200; ++i) rs_gemm(1, 0, 0, M, n, K, x, K, w, K, y, n, 0, ep, 1, nullptr, nullptr);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double us = ms * 1e3 / 200;
    printf("%-44s %8.2f us  %7.0f GB/s\n", name, us, (M * K * 2.0 + M * n * 2.0) / (us * 1e-6) / 1e9);
  };
  rs_epilogue e; memset(&e, 0, sizeof(e)); e.alpha = 1.f;
  T("plain", &e);
  e.bias = b; T("+bias", &e);
  e.drop_p = 0.2f; e.drop_seed = 7; e.seed_base = (const uint64_t*)sb; e.drop_ld = N; T("+bias+dropout", &e);
  e.resid = r; e.ldres = N; T("+bias+dropout+resid", &e);
  e.rowmask_ids = (const int64_t*)ids; T("+bias+dropout+resid+rowmask", &e);
  memset(&e, 0, sizeof(e)); e.alpha = 1.f;
  T("plain N=256", &e, 256);
  T("plain N=512", &e, 512);
  return 0;
}
