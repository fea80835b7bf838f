// Phase timing of the LDS attention forward (wall_clock64 stamps per wave: entry, staged, done).
//   hipcc --offload-arch=gfx950 -O3 -DATTN_PROF -I include -I recommender-baseline-model_amd/csrc \
//         tools/micro/attn_phase.hip -o tools/micro/attn_phase
#include "../../recommender-baseline-model_amd/csrc/attention_lds.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

KStamp kstamp_next(int) { return KStamp{nullptr, nullptr, 0}; }

static void run(int B, int T) {
  const int H = 1, Dh = 128, d = 128;
  const size_t M = (size_t)B * T;
  void *q, *kv, *o;
  float* lse;
  uint64_t* sb;
  hipMalloc(&q, M * d * 2);
  hipMalloc(&kv, M * 2 * d * 2);
  hipMalloc(&o, M * d * 2);
  hipMalloc(&lse, M * 4);
  hipMalloc(&sb, 8);
  hipMemset(q, 0x3c, M * d * 2);
  hipMemset(kv, 0x3c, M * 2 * d * 2);
  hipMemset(sb, 0, 8);
  for (int it = 0; it < 5; ++it)
    attn_lds_fwd(B, T, H, Dh, q, d, kv, 2 * d, (char*)kv + d * 2, 2 * d, o, d, lse, 0.088f, 0, nullptr, 0.2f, 7, sb, 0);
  hipDeviceSynchronize();
  std::vector<unsigned long long> p(8192 * NW * 10);
  hipMemcpyFromSymbol(p.data(), HIP_SYMBOL(g_attn_prof), p.size() * 8);
  const int nq = (T + 15) / 16;
  int ns = 1;
  while ((int64_t)B * H * ns < 256 && ns * 2 <= std::max(1, nq / 4)) ns *= 2;
  const int nblk = ns * B * H;
  unsigned long long t0 = ~0ull, t1 = 0;
  double stage = 0, comp = 0, ramp = 0;
  int nw = 0;
  std::vector<double> comps;
  for (int b = 0; b < nblk; ++b)
    for (int w = 0; w < NW; ++w) {
      const unsigned long long* x = &p[((size_t)b * NW + w) * 10];
      if (!x[0] || !x[2]) continue;
      t0 = std::min(t0, x[0]);
      t1 = std::max(t1, x[2]);
    }
  for (int b = 0; b < nblk; ++b)
    for (int w = 0; w < NW; ++w) {
      const unsigned long long* x = &p[((size_t)b * NW + w) * 10];
      if (!x[0] || !x[2]) continue;
      stage += x[1] - x[0];
      comp += x[2] - x[1];
      ramp += x[0] - t0;
      comps.push_back(x[2] - x[1]);
      ++nw;
    }
  std::sort(comps.begin(), comps.end());
  const double tick_us = 0.01;   // wall_clock64: 100 MHz
  printf("B=%d T=%d nsplit=%d blocks=%d: span %.2f us | mean entry offset %.2f, staging %.2f, compute %.2f "
         "(p50 %.2f, max %.2f) us\n",
         B, T, ns, nblk, (t1 - t0) * tick_us, ramp / nw * tick_us, stage / nw * tick_us, comp / nw * tick_us,
         comps[comps.size() / 2] * tick_us, comps.back() * tick_us);
  // block 0: per wave, item durations (us) after staging
  for (int w = 0; w < NW; ++w) {
    const unsigned long long* x = &p[(size_t)w * 10];
    printf("  blk0 wave %d: staged +%.2f", w, (x[1] - x[0]) * tick_us);
    unsigned long long prev = x[1];
    for (int j = 0; j < 7; ++j) {
      if (!x[3 + j] || x[3 + j] < prev) break;
      printf("  item%d %.2f", j, (x[3 + j] - prev) * tick_us);
      prev = x[3 + j];
    }
    printf("  | end +%.2f\n", (x[2] - x[0]) * tick_us);
  }
  hipFree(q); hipFree(kv); hipFree(o); hipFree(lse); hipFree(sb);
}

int main() {
  run(128, 200);
  run(128, 64);
  run(128, 50);
  run(64, 200);
  run(256, 200);
  return 0;
}
