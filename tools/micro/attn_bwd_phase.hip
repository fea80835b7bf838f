// Phase timing of the LDS attention backward (wall_clock64 stamps per wave): dQ kernel entry / K,V staged /
// done, dK/dV kernel entry / Q,dO staged / done.
//   hipcc --offload-arch=gfx950 -O3 -DATTN_PROF -I include -I recommender-baseline-model_amd/csrc \
//         tools/micro/attn_bwd_phase.hip -o tools/micro/attn_bwd_phase
#include "../../recommender-baseline-model_amd/csrc/attention_lds.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

KStamp kstamp_next(int) { return KStamp{nullptr, nullptr, 0}; }

static void run(int B, int T) {
  const int H = 1, Dh = 128, d = 128;
  const size_t M = (size_t)B * T;
  void *q, *kv, *o, *dout, *dq, *dkv;
  float *lse, *delta;
  uint64_t* sb;
  hipMalloc(&q, M * d * 2); hipMalloc(&kv, M * 2 * d * 2); hipMalloc(&o, M * d * 2); hipMalloc(&dout, M * d * 2);
  hipMalloc(&dq, M * d * 2); hipMalloc(&dkv, M * 2 * d * 2);
  hipMalloc(&lse, M * 4); hipMalloc(&delta, M * 4); hipMalloc(&sb, 8);
  hipMemset(q, 0x3c, M * d * 2); hipMemset(kv, 0x3c, M * 2 * d * 2); hipMemset(o, 0x3c, M * d * 2);
  hipMemset(dout, 0x3c, M * d * 2); hipMemset(lse, 0, M * 4); hipMemset(sb, 0, 8);
  std::vector<unsigned long long> p(8192 * NW * 10);
  for (int it = 0; it < 5; ++it) {
    hipMemcpyToSymbol(HIP_SYMBOL(g_attn_prof), p.data(), p.size() * 8);   // zero
    attn_lds_bwd(B, T, H, Dh, q, d, kv, 2 * d, (char*)kv + d * 2, 2 * d, o, d, dout, d, lse, dq, d, dkv, 2 * d,
                 (char*)dkv + d * 2, 2 * d, 0.088f, 0, nullptr, 0.2f, 7, sb, delta, 0);
  }
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(p.data(), HIP_SYMBOL(g_attn_prof), p.size() * 8);
  const int nq = (T + 15) / 16;
  int ns = 1;
  while ((int64_t)B * H * ns < 256 && ns * 2 <= std::max(1, nq / 4)) ns *= 2;
  const int nblk = ns * B * H;
  unsigned long long t0 = ~0ull, t1 = 0;
  double sum[6] = {0};
  int nw = 0;
  std::vector<double> st, cq, ck;
  for (int k = 0; k < 2; ++k) {}
  for (int b = 0; b < nblk; ++b)
    for (int w = 0; w < NW; ++w) {
      const unsigned long long* x = &p[((size_t)b * NW + w) * 10];
      if (!x[4] || !x[6] || !x[7] || !x[9]) continue;
      t0 = std::min(t0, x[4]);
      t1 = std::max(t1, x[9]);
    }
  double dq_end = 0, dkv_start = 1e30;
  for (int b = 0; b < nblk; ++b)
    for (int w = 0; w < NW; ++w) {
      const unsigned long long* x = &p[((size_t)b * NW + w) * 10];
      if (!x[4] || !x[6] || !x[7] || !x[9]) continue;
      sum[0] += x[4] - t0; sum[1] += x[5] - x[4]; sum[2] += x[6] - x[5];
      sum[3] += x[7] - t0; sum[4] += x[8] - x[7]; sum[5] += x[9] - x[8];
      cq.push_back(x[6] - x[5]); ck.push_back(x[9] - x[8]);
      dq_end = std::max(dq_end, (double)(x[6] - t0)); dkv_start = std::min(dkv_start, (double)(x[7] - t0));
      ++nw;
    }
  std::sort(cq.begin(), cq.end()); std::sort(ck.begin(), ck.end());
  const double u = 0.01;   // 100 MHz ticks -> us
  printf("B=%d T=%d nsplit=%d blocks=%d waves=%d: span %.2f us\n", B, T, ns, nblk, nw, (t1 - t0) * u);
  printf("  dQ : entry +%.2f  staging %.2f  compute %.2f (p50 %.2f max %.2f)  last wave done %.2f\n", sum[0] / nw * u,
         sum[1] / nw * u, sum[2] / nw * u, cq[cq.size() / 2] * u, cq.back() * u, dq_end * u);
  printf("  dKV: first entry %.2f mean entry +%.2f  staging %.2f  compute %.2f (p50 %.2f max %.2f)\n", dkv_start * u,
         sum[3] / nw * u, sum[4] / nw * u, sum[5] / nw * u, ck[ck.size() / 2] * u, ck.back() * u);
  hipFree(q); hipFree(kv); hipFree(o); hipFree(dout); hipFree(dq); hipFree(dkv); hipFree(lse); hipFree(delta); hipFree(sb);
}

int main() {
  run(128, 200);
  run(128, 50);
  return 0;
}
