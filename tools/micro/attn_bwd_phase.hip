// Phase timing of the LDS attention backward (wall_clock64 stamps per wave): dQ kernel entry / K,V staged /
// done, dK/dV kernel entry / Q,dO staged / done.
//   hipcc --offload-arch=gfx950 -O3 -DATTN_PROF -I include -I recommender-baseline-model_amd/csrc \
//         tools/micro/attn_bwd_phase.hip -o tools/micro/attn_bwd_phase
#include "../../recommender-baseline-model_amd/csrc/attention_lds.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

KStamp kstamp_next(int) { return KStamp{nullptr, nullptr, 0}; }

static void run(int B, int T, float drop, int mk = 0) {
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
                 (char*)dkv + d * 2, 2 * d, 0.088f, mk, nullptr, drop, 7, sb, delta, 0);
  }
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(p.data(), HIP_SYMBOL(g_attn_prof), p.size() * 8);
  const int nq = (T + 15) / 16;
  int ns = 1;
  while (2 * (int64_t)B * H * ns * 2 <= 256 && ns * 2 <= std::max(1, nq / 4)) ns *= 2;   // pick_split_bwd (merged)
  const int nblk = ns * B * H;
  // merged launch: blocks [0, nblk) are dQ workgroups (stamps 4/5/6), [nblk, 2 nblk) dK/dV ones (7/8/9)
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < 2 * nblk; ++b)
    for (int w = 0; w < NW; ++w) {
      const unsigned long long* x = &p[((size_t)b * NW + w) * 10];
      const unsigned long long e = b < nblk ? x[4] : x[7], f = b < nblk ? x[6] : x[9];
      if (!e || !f) continue;
      t0 = std::min(t0, e);
      t1 = std::max(t1, f);
    }
  const double u = 0.01;   // 100 MHz ticks -> us
  printf("B=%d T=%d p=%.1f delta_in=%d nsplit=%d blocks=2x%d: span %.2f us\n", B, T, drop, mk != 0, ns, nblk, (t1 - t0) * u);
  for (int kind = 0; kind < 2; ++kind) {
    std::vector<double> ent, stg, cmp, fin;
    for (int b = kind * nblk; b < (kind + 1) * nblk; ++b)
      for (int w = 0; w < NW; ++w) {
        const unsigned long long* x = &p[((size_t)b * NW + w) * 10 + (kind ? 7 : 4)];
        if (!x[0] || !x[2]) continue;
        ent.push_back((x[0] - t0) * u); stg.push_back((x[1] - x[0]) * u); cmp.push_back((x[2] - x[1]) * u);
        fin.push_back((x[2] - t0) * u);
      }
    auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
    printf("  %s: entry p50 %.2f max %.2f | staging p50 %.2f max %.2f | compute p50 %.2f max %.2f | end p50 %.2f max %.2f\n",
           kind ? "dKV" : "dQ ", q(ent, .5), q(ent, 1), q(stg, .5), q(stg, 1), q(cmp, .5), q(cmp, 1), q(fin, .5), q(fin, 1));
  }
  hipFree(q); hipFree(kv); hipFree(o); hipFree(dout); hipFree(dq); hipFree(dkv); hipFree(lse); hipFree(delta); hipFree(sb);
}

int main() {
  run(128, 200, 0.2f);
  run(128, 200, 0.2f, RS_ATTN_DELTA_IN);
  run(128, 200, 0.0f, RS_ATTN_DELTA_IN);
  run(128, 50, 0.2f);
  run(128, 50, 0.2f, RS_ATTN_DELTA_IN);
  return 0;
}
