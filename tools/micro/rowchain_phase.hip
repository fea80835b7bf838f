// Phase timing of the row-chain block_out kernel (rowchain.hip, wall_clock64 stamps per wave): entry,
// weights staged, first GEMM done (its inputs arrived), x1 stored, chain done, exit.
//   hipcc --offload-arch=gfx950 -O3 -DRC_PROF -I include -I recommender-baseline-model_amd/csrc \
//         tools/micro/rowchain_phase.hip -o tools/micro/rowchain_phase
#include "../../recommender-baseline-model_amd/csrc/rowchain.hip"

#include <algorithm>
#include <cstdio>
#include <vector>
#include <string>

static void pct(const char* name, std::vector<double> v) {
  if (v.empty()) return;
  std::sort(v.begin(), v.end());
  auto q = [&](double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
  printf("  %-26s n=%5zu  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", name, v.size(), q(0.1), q(0.5), q(0.9),
         v.back());
}

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 25600, d = 128;
  void *o, *Q, *W, *x1, *z, *h1, *xn;
  float *b, *lw, *lb, *mu, *rs;
  int64_t* ids;
  uint64_t* sb;
  hipMalloc(&o, M * d * 2); hipMalloc(&Q, M * d * 2); hipMalloc(&W, 3 * d * d * 2); hipMalloc(&x1, M * d * 2);
  hipMalloc(&z, M * d * 2); hipMalloc(&h1, M * d * 2); hipMalloc(&xn, M * d * 2);
  hipMalloc(&b, d * 4); hipMalloc(&lw, d * 4); hipMalloc(&lb, d * 4); hipMalloc(&mu, M * 4); hipMalloc(&rs, M * 4);
  hipMalloc(&ids, M * 8); hipMalloc(&sb, 8);
  hipMemset(o, 0x3c, M * d * 2); hipMemset(Q, 0x3c, M * d * 2); hipMemset(W, 0x3c, 3 * d * d * 2);
  hipMemset(b, 0, d * 4); hipMemset(lw, 0, d * 4); hipMemset(lb, 0, d * 4); hipMemset(ids, 1, M * 8);
  hipMemset(sb, 0, 8);
  const __bf16* Wb = (const __bf16*)W;
  // --head (argv[2] = "head"): the last block's kernel with the SAS head (rs_sas_block_out_head), 3,416 items
  const bool head = argc > 2 && std::string(argv[2]) == "head";
  const int G = (int)rc::grid_for(M);
  void *E, *f, *dx;
  int64_t *pos, *neg;
  int* cnt;
  float *pl, *nl, *dpl, *dnl, *lnpart, *part;
  hipMalloc(&E, 3417 * d * 2); hipMalloc(&f, M * d * 2); hipMalloc(&dx, M * d * 2);
  hipMalloc(&pos, M * 8); hipMalloc(&neg, M * 8); hipMalloc(&cnt, G * 8 * 4);
  hipMalloc(&pl, M * 4); hipMalloc(&nl, M * 4); hipMalloc(&dpl, M * 4); hipMalloc(&dnl, M * 4);
  hipMalloc(&lnpart, G * 2 * d * 4); hipMalloc(&part, G * 3 * 4);
  {
    std::vector<int64_t> ip(M), in(M);
    for (int64_t i = 0; i < M; ++i) { ip[i] = 1 + (i * 7919) % 3416; in[i] = 1 + (i * 104729) % 3416; }
    hipMemcpy(pos, ip.data(), M * 8, hipMemcpyHostToDevice);
    hipMemcpy(neg, in.data(), M * 8, hipMemcpyHostToDevice);
    std::vector<int> c(G, 96);
    hipMemcpy(cnt, c.data(), G * 4, hipMemcpyHostToDevice);
    hipMemset(E, 0x3c, 3417 * d * 2);
  }
  std::vector<unsigned long long> p(4096 * 8 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float ms = 0.f;
  for (int it = 0; it < 20; ++it) {
    hipMemcpyToSymbol(HIP_SYMBOL(rc::g_rc_prof), p.data(), p.size() * 8);   // zero
    hipEventRecord(e0, 0);
    if (head)
      rs_sas_block_out_head(M, d, o, Q, Wb, b, x1, lw, lb, 1e-8f, z, mu, rs, Wb + d * d, b, h1, Wb + 2 * d * d, b, xn,
                            ids, 0.2f, 3, 5, sb, E, pos, neg, lw, lb, cnt, G, nullptr, f, pl, nl, dpl, dnl, dx,
                            lnpart, part, 0);
    else
      rs_sas_block_out(M, d, o, Q, Wb, b, x1, lw, lb, 1e-8f, z, mu, rs, Wb + d * d, b, h1, Wb + 2 * d * d, b, xn,
                       ids, 0.2f, 3, 5, sb, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  hipMemcpyFromSymbol(p.data(), HIP_SYMBOL(rc::g_rc_prof), p.size() * 8);
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b_ = 0; b_ < G; ++b_)
    for (int w = 0; w < 8; ++w) {
      const unsigned long long* x = &p[((size_t)b_ * 8 + w) * 16];
      if (x[0]) t0 = std::min(t0, x[0]);
      if (x[5]) t1 = std::max(t1, x[5]);
    }
  const double u = 0.01;   // 100 MHz ticks -> us
  printf("block_out M=%lld grid=%d: event %.2f us, first entry -> last exit %.2f us\n", (long long)M, G, ms * 1e3,
         (t1 - t0) * u);
  std::vector<double> ent, stg, ga, gb, ex, tot;
  for (int b_ = 0; b_ < G; ++b_)
    for (int w = 0; w < 8; ++w) {
      const unsigned long long* x = &p[((size_t)b_ * 8 + w) * 16];
      if (!x[0]) continue;
      ent.push_back((x[0] - t0) * u);
      stg.push_back((x[1] - x[0]) * u);
      if (x[2]) {
        ga.push_back((x[2] - x[1]) * u);
        gb.push_back((x[4] - x[2]) * u);
      }
      ex.push_back((x[5] - t0) * u);
      tot.push_back((x[5] - x[0]) * u);
    }
  pct("entry after first", ent);
  pct("weight staging (+barrier)", stg);
  pct("x1, LN2, GEMM W1 (tile 1)", ga);
  pct("GEMM W2 + stores (tile 1)", gb);
  pct("exit after first entry", ex);
  pct("wave lifetime", tot);
  if (head) {
    std::vector<double> hd;
    for (int b_ = 0; b_ < G; ++b_)
      for (int w = 0; w < 8; ++w) {
        const unsigned long long* x = &p[((size_t)b_ * 8 + w) * 16];
        if (x[6] && x[4]) hd.push_back((x[6] - x[4]) * u);
      }
    pct("head (tile 1)", hd);
  }
  return 0;
}
