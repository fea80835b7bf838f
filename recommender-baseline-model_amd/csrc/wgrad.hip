// rs-build: included by grad_tail.hip (compiled once, as part of that translation unit)
// Grouped weight-gradient GEMMs + grouped slab reduction (bf16 operands, fp32 results).
//
// In a SASRec / BERT4Rec backward every Linear / Conv1d(k=1) weight gradient is
//   dW[N][K] += sum_m dY[m][n] X[m][k],   db[N] += sum_m dY[m][n]
// with M = B*T token rows (25.6k at the headline shape) and N, K = d or 2d (<= 256): a tall-skinny
// reduction whose output is tiny.  One launch per weight (the generic split-K GEMM + a reduce
// launch each) is latency-bound: every workgroup runs a handful of 64-row stages between a cold
// prologue and a slab epilogue.  Here ALL weight gradients of the backward pass run in ONE launch
// (problems x output tiles x row splits workgroups, each streaming its row range through
// double-buffered LDS stages and MFMA-accumulating a whole 64x64 / 128x128 output tile), and ALL
// their split partials -- plus any extra partial sets such as the LayerNorm affine partials the
// fused row-block kernels leave -- are summed by ONE deterministic grouped reduction.
//
// Bias gradients ride on the same MFMAs (dY^T against a ones operand) in the k-tile-0 blocks.
#include "gemm_bf16_impl.h"
#include "dma256.h"

namespace wg {

typedef __bf16 bf16;
constexpr int MAXP = 16;

struct Prob {
  const bf16* dY;
  const bf16* X;
  int64_t lddy, ldx;
  int N, K, tiles_k, tile0;    // tile0: first global tile index of this problem
  int64_t slab_off;            // float offset of split 0; split stride = N*K + N
};

struct Args {
  Prob p[MAXP];
  int nprob, ntiles, splits, rows_per_split;
  int64_t M;
  float* slab;
  KStamp ks;                   // begin stamp of a stamped rs_wgrad_grouped launch
};

template <int T>
constexpr int group_lds_bytes() { return 2 * 2 * gbf::Img<true, T>::ELEMS * (int)sizeof(bf16); }

// one (split, output tile) of the grouped launch; bid_raw / nwg: this workgroup's index among the launch's
// nwg weight-gradient workgroups (dispatch order, before the XCD remap)
template <int T>
__device__ __forceinline__ void group_tile(const Args& a, unsigned bid_raw, unsigned nwg, bf16* smem) {
  using I = gbf::Img<true, T>;          // k-major stage image [64 rows][T + 8]
  constexpr int STAGE = 2 * I::ELEMS;
  constexpr int BKT = gbf::BKT;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wave >> 1, wn = wave & 1;
  constexpr int FM = T / 32, FN = T / 32;

  // XCD-aware: workgroup b runs on XCD b % 8; give each XCD a contiguous range of (split, tile) pairs, so
  // the tiles that share a row range's dY / X column slices read them through ONE XCD's L2 (round-robin
  // dealing had every XCD fetch its own copy: ~2.5x the algorithmic HBM bytes at the BERT shapes)
  unsigned bid = bid_raw;
  {
    const unsigned q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int t = (int)(bid % (unsigned)a.ntiles);
  const int s = (int)(bid / (unsigned)a.ntiles);
  int pi = 0;
#pragma unroll 1
  for (int q = 1; q < a.nprob; ++q)
    if (t >= a.p[q].tile0) pi = q;
  const Prob& P = a.p[pi];
  const int lt = t - P.tile0;
  const int tn = lt / P.tiles_k, tk = lt - tn * P.tiles_k;
  const int64_t n0 = (int64_t)tn * T, c0 = (int64_t)tk * T;
  const int64_t kbeg = (int64_t)s * a.rows_per_split;
  const int64_t kend = min(a.M, kbeg + a.rows_per_split);
  const int nk = kend > kbeg ? (int)((kend - kbeg + BKT - 1) / BKT) : 0;
  const bool do_colsum = tk == 0 && wn == 0;

  f32x4 acc[FM][FN], accb[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    accb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  // the MFMAs of one 64-deep LDS stage image (dY^T tile x X tile, + the bias column sums against ones)
  auto mma_stage = [&](const bf16* cur) {
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = gbf::frag<true, T>(cur, wm * (T / 2) + 16 * i, ss, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = gbf::frag<true, T>(cur + I::ELEMS, wn * (T / 2) + 16 * j, ss, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (do_colsum) {
#pragma unroll
        for (int i = 0; i < FM; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb[i], 0, 0, 0);
      }
    }
  };

  const bool interior = ((kend - kbeg) % BKT) == 0;
  // ragged row ranges (M not a multiple of 64): bounds-checked loads, one stage in flight
  auto edge_loop = [&]() {
    gbf::Stage<true, T> sa, sb;
    sa.tid_ = tid;
    sb.tid_ = tid;
    auto issue = [&](int64_t k0) {
      sa.load_checked(P.dY, P.lddy, k0, n0, kend, P.N, tid);
      sb.load_checked(P.X, P.ldx, k0, c0, kend, P.K, tid);
    };
    issue(kbeg);
    sa.store(smem, tid);
    sb.store(smem + I::ELEMS, tid);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) issue(kbeg + (int64_t)(kt + 1) * BKT);
      mma_stage(smem + (kt & 1) * STAGE);
      if (more) {
        bf16* nxt = smem + ((kt + 1) & 1) * STAGE;
        sa.store(nxt, tid);
        sb.store(nxt + I::ELEMS, tid);
      }
      __syncthreads();
    }
  };

  // interior tiles: two stages in flight in registers (a ring of 2 register slots feeding the 2 LDS buffers), so
  // each stage's L2 / HBM round trip hides under two stages of MFMAs instead of one.  Every iteration issues
  // its loads unconditionally (past the last stage every lane re-reads the tile's first word), so the wait
  // before an LDS store covers exactly the older slot's loads.  cfg3 (16 BERT weights, 384 workgroups of 100
  // stages): 170 -> 166 us for the launch + reduction, interleaved A/B; the step and cfg2 within noise -- the
  // launch streams ~475 MB at ~3.6 TB/s, so one stage of prefetch was not what bounded it.  The deeper ring raises
  // the launch's HBM fetches 475 -> 536 MB (PMC; more stages in flight per XCD's L2 evict tiles' shared rows
  // before their neighbours read them): kept for the time, the launch is latency- not bandwidth-bound.
  auto ring = [&]() {
    static_assert(I::NCH % 256 == 0, "whole 16-B chunks per thread");
    constexpr int PT = I::PER_T;
    bf16x8 ra[2][PT], rb[2][PT];
    const bf16* pa[PT];
    const bf16* pb[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + 256 * i, rr = ch / I::CPR, cc = (ch % I::CPR) * 8;
      pa[i] = P.dY + (kbeg + rr) * P.lddy + n0 + cc;
      pb[i] = P.X + (kbeg + rr) * P.ldx + c0 + cc;
    }
    const int64_t sta = (int64_t)BKT * P.lddy, stb = (int64_t)BKT * P.ldx;
    int at = 0;   // stage the pointers address (stops at nk - 1)
    auto load = [&](auto S) {
      constexpr int sl = decltype(S)::value;
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        ra[sl][i] = *reinterpret_cast<const bf16x8*>(pa[i]);
        rb[sl][i] = *reinterpret_cast<const bf16x8*>(pb[i]);
      }
      const bool adv = at + 1 < nk;
      at += adv ? 1 : 0;
#pragma unroll
      for (int i = 0; i < PT; ++i) {   // past the last stage: every lane re-reads one 16-B word (one line per wave)
        pa[i] = adv ? pa[i] + sta : P.dY + kbeg * P.lddy + n0;
        pb[i] = adv ? pb[i] + stb : P.X + kbeg * P.ldx + c0;
      }
    };
    auto store = [&](auto S, bf16* img) {
      constexpr int sl = decltype(S)::value;
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int ch = tid + 256 * i, rr = ch / I::CPR, cc = (ch % I::CPR) * 8;
        *reinterpret_cast<bf16x8*>(img + rr * I::LD + cc) = ra[sl][i];
        *reinterpret_cast<bf16x8*>(img + I::ELEMS + rr * I::LD + cc) = rb[sl][i];
      }
    };
    load(std::integral_constant<int, 0>{});
    load(std::integral_constant<int, 1>{});
    store(std::integral_constant<int, 0>{}, smem);
    __syncthreads();
    auto body = [&](int kt, auto S) {
      constexpr int sl = decltype(S)::value;      // == kt & 1
      load(S);                                    // stage kt + 2 (or the one-word dummy past the last)
      mma_stage(smem + sl * STAGE);
      if (kt + 1 < nk) store(std::integral_constant<int, 1 - sl>{}, smem + (1 - sl) * STAGE);
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      body(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < nk) body(kt + 1, std::integral_constant<int, 1>{});
    }
  };
  if (nk > 0) {
    if (interior) ring();
    else edge_loop();
  }

  // split partial -> slab (each 16-lane group stores 64 contiguous bytes per row)
  float* S = a.slab + P.slab_off + (int64_t)s * ((int64_t)P.N * P.K + P.N);
  const int g = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t n = n0 + wm * (T / 2) + 16 * i + 4 * g + r;
#pragma unroll
      for (int j = 0; j < FN; ++j) S[n * P.K + c0 + wn * (T / 2) + 16 * j + cl] = acc[i][j][r];
      if (do_colsum && cl == 0) S[(int64_t)P.N * P.K + n] = accb[i][r];
    }
}

template <int T>
__global__ __launch_bounds__(256, 2) void wgrad_group_kernel(Args a) {
  KStampBegin stamp_(a.ks);
  __shared__ __attribute__((aligned(16))) bf16 smem[group_lds_bytes<T>() / sizeof(bf16)];
  group_tile<T>(a, blockIdx.x, gridDim.x, smem);
}

// 256 x 256 output tiles (every dimension of the problems a multiple of 256: the BERT d = 256 layer's QKV, output,
// FFN1 and FFN2 weights).  With 128 x 128 tiles each 64-row stage moves 32 KB from L2 per 2.1 MFLOP and the 12,800-row
// operands of width 1,024 / 768 are re-read by every 128-wide tile across them (FFN1's X 8x, dY 2x per split): the
// launch ran at ~8.6 TB/s of L2->CU operand traffic (148 us at cfg3, 0.2 of MFMA).  A 256 x 256 tile halves the
// stage bytes per flop and reads the 256-wide side once per split.  The tile is gemm_n256's (dma256.h): 8 waves,
// each a 128 x 64 quadrant, 32-deep stages of both k-major operands by LDS-DMA into four buffers, three in flight;
// bias column sums on MFMAs against ones (column tile 0); the fp32 partial tile staged through LDS into the split's
// slab in the layout the grouped reduction sums (same slabs as the 64 / 128 tiles; summation order within a split
// differs: 32-deep MFMA steps in row order).
struct Args256 {
  Prob p[MAXP];
  int nprob, ntiles, splits, rows_per_split;
  int64_t M;
  float* slab;
  KStamp ks;
};
__global__ __launch_bounds__(g256::NTH) void wgrad_group256_kernel(Args256 a) {
  using namespace g256;
  KStampBegin stamp_(a.ks);
  constexpr int LDC = BN + 4;
  constexpr int LDS_BYTES = NBUF * DSTAGE > (BM / 2) * LDC * 4 ? NBUF * DSTAGE : (BM / 2) * LDC * 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  constexpr int FM = 8, FN = 4;
  // XCD-contiguous (split, tile) ranges (as group_tile): the tiles of one row split, which share its operand rows,
  // read them through one XCD's L2
  unsigned bid = blockIdx.x;
  {
    const unsigned nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int t = (int)(bid % (unsigned)a.ntiles);
  const int s = (int)(bid / (unsigned)a.ntiles);
  int pi = 0;
#pragma unroll 1
  for (int q = 1; q < a.nprob; ++q)
    if (t >= a.p[q].tile0) pi = q;
  const Prob& P = a.p[pi];
  const int lt = t - P.tile0;
  const int tm = lt / P.tiles_k, tn = lt - tm * P.tiles_k;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)s * a.rows_per_split;
  const int64_t kend = min(a.M, kbeg + a.rows_per_split);
  const int nk = kend > kbeg ? (int)((kend - kbeg + DBK - 1) / DBK) : 0;
  const uint32_t lds0 = lds_u32(smem);
  const bool do_colsum = tn == 0;

  f32x4 acc[FM][FN], accb[2];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  accb[0] = accb[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;

  auto issue = [&](int st) {
    const uint32_t buf = lds0 + (uint32_t)((st % NBUF) * DSTAGE);
    const int64_t k0 = kbeg + (int64_t)st * DBK;
#pragma unroll
    for (int j = 0; j < 2; ++j) km_piece(P.dY, P.lddy, k0, m0, kend, P.N, 2 * wave + j, lane, buf);
#pragma unroll
    for (int j = 0; j < 2; ++j) km_piece(P.X, P.ldx, k0, n0, kend, P.K, 2 * wave + j, lane, buf + IMG_BYTES);
  };
  auto zero_tail = [&](int st) {
    char* buf = smem + (st % NBUF) * DSTAGE;
    const int kv = (int)(kend - (kbeg + (int64_t)st * DBK));
    for (int e = tid; e < (DBK - kv) * 256; e += NTH) {
      const int r = kv + e / 256, c = e % 256;
      *reinterpret_cast<__bf16*>(buf + IMG_BYTES + km_off(r, c)) = (__bf16)0.0f;
      *reinterpret_cast<__bf16*>(buf + km_off(r, c)) = (__bf16)0.0f;
    }
  };
  auto compute = [&](int st) {
    const char* buf = smem + (st % NBUF) * DSTAGE;
    bf16x8 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = km_frag(buf, wm * 128 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = km_frag(buf + IMG_BYTES, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (do_colsum) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
        if ((i >> 1) == wn) accb[i & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb[i & 1], 0, 0, 0);
    }
  };
  const bool tail = ((kend - kbeg) % DBK) != 0;
  for (int st = 0; st < min(nk, DIST); ++st) issue(st);
  for (int st = 0; st < nk; ++st) {
    const int after = min(nk - 1, st + DIST - 1) - st;
    vm_wait_stages(after);
    raw_barrier();
    if (st + DIST < nk) issue(st + DIST);
    if (tail && st == nk - 1) {
      zero_tail(st);
      raw_barrier();
    }
    compute(st);
  }
  vm_wait<0>();

  // epilogue: the partial tile into split s's slab, [N][K] rows of the weight (+ the bias partial after them)
  float* S = a.slab + P.slab_off + (int64_t)s * ((int64_t)P.N * P.K + P.N);
  float* Cs = reinterpret_cast<float*>(smem);
  const int g = lane >> 4, cl = lane & 15;
  if (do_colsum && cl == 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[(int64_t)P.N * P.K + m0 + wm * 128 + 16 * (2 * wn + u) + 4 * g + r] = accb[u][r];
  }
  constexpr int TPR = BN / 8, RPP = NTH / TPR;
  const int c8 = (tid % TPR) * 8;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
    if (wm == half) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) Cs[(16 * i + 4 * g + r) * LDC + wn * 64 + 16 * j + cl] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int row = tid / TPR; row < BM / 2; row += RPP) {
      const int64_t m = m0 + half * 128 + row;
      const float4 v0 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8 + 4);
      float* dst = S + m * P.K + n0 + c8;
      *reinterpret_cast<float4*>(dst) = v0;
      *reinterpret_cast<float4*>(dst + 4) = v1;
    }
  }
}

// the grouped launch (T = output tile edge)
inline void launch_group(const Args& a, int T, hipStream_t s) {
  const dim3 grid((unsigned)(a.ntiles * a.splits));
  if (T == 256) {
    Args256 b;
    static_assert(sizeof(b.p) == sizeof(a.p), "same problem table");
    memcpy(b.p, a.p, sizeof(a.p));
    b.nprob = a.nprob; b.ntiles = a.ntiles; b.splits = a.splits; b.rows_per_split = a.rows_per_split;
    b.M = a.M; b.slab = a.slab; b.ks = a.ks;
    hipLaunchKernelGGL(wgrad_group256_kernel, grid, dim3(g256::NTH), 0, s, b);
  } else if (T == 128) hipLaunchKernelGGL(wgrad_group_kernel<128>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wgrad_group_kernel<64>, grid, dim3(256), 0, s, a);
}

// ---------------------------------------------------------------- grouped slab reduction
constexpr int MAXS = 64;
struct Seg {
  const float* src;   // split z at src + z*stride
  int64_t stride;
  int splits, n;      // n floats (multiple of 4, 16-byte aligned src/out)
  float* out;
  int cols;           // columns per thread of the column form (1, or 4 for large few-split segments), 0: split
                      // groups + LDS tree
};
constexpr int COLS_MAX = 32;   // splits up to which a segment is summed column per thread
struct RArgs {
  Seg s[MAXS];
  int blk0[MAXS + 1];
  int nseg, accumulate;
  KStamp ks;                   // end stamp (last reduction launch of a stamped rs_wgrad_grouped)
};

// block = C float4 columns x G split groups (C*G = 256): group g sums splits g, g+G, ... (4 loads in flight),
// then a fixed LDS tree combines the groups (deterministic).  C = 16 for the weight-gradient slabs (tens of
// splits); segments with many splits -- the LayerNorm affine partials, one row per 64-token block (400 at cfg2)
// -- take C = 4, G = 64: 4x the workgroups and a quarter of the serial loads per thread (with C = 16 those
// few blocks summed 25 splits per thread and set the reduction launch's length)
constexpr int RED_C = 16, RED_G = 16;
__device__ __forceinline__ int seg_cols(int splits) { return splits > 64 ? 4 : RED_C; }

__device__ __forceinline__ void reduce_segments_block(const RArgs& a, int b, float4 (*red2)[RED_C]) {
  float4* red = &red2[0][0];
  int si = 0;
#pragma unroll 1
  for (int q = 1; q < a.nseg; ++q)
    if (b >= a.blk0[q]) si = q;
  const Seg& S = a.s[si];
  const int C = seg_cols(S.splits), G = 256 / C;
  const int col = threadIdx.x % C, grp = threadIdx.x / C;
  const int64_t i4 = (int64_t)(b - a.blk0[si]) * C + col;
  const int64_t n4 = S.n / 4;
  const float4* src = reinterpret_cast<const float4*>(S.src);
  const int64_t st4 = S.stride / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    int z = grp;
    for (; z + 3 * G < S.splits; z += 4 * G) {
      const float4 u0 = src[(int64_t)z * st4 + i4];
      const float4 u1 = src[(int64_t)(z + G) * st4 + i4];
      const float4 u2 = src[(int64_t)(z + 2 * G) * st4 + i4];
      const float4 u3 = src[(int64_t)(z + 3 * G) * st4 + i4];
      acc.x += u0.x; acc.y += u0.y; acc.z += u0.z; acc.w += u0.w;
      acc.x += u1.x; acc.y += u1.y; acc.z += u1.z; acc.w += u1.w;
      acc.x += u2.x; acc.y += u2.y; acc.z += u2.z; acc.w += u2.w;
      acc.x += u3.x; acc.y += u3.y; acc.z += u3.z; acc.w += u3.w;
    }
    for (; z < S.splits; z += G) {
      const float4 u = src[(int64_t)z * st4 + i4];
      acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w;
    }
  }
  red[grp * C + col] = acc;
  __syncthreads();
  for (int h = G / 2; h > 0; h >>= 1) {
    if (grp < h) {
      const float4 u = red[(grp + h) * C + col];
      float4 t = red[grp * C + col];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      red[grp * C + col] = t;
    }
    __syncthreads();
  }
  if (grp == 0 && i4 < n4) {
    float4 tot = red[col];
    float4* o = reinterpret_cast<float4*>(S.out) + i4;
    if (a.accumulate) {
      const float4 p = *o;
      tot.x += p.x; tot.y += p.y; tot.z += p.z; tot.w += p.w;
    }
    *o = tot;
  }
}

__device__ __forceinline__ void reduce_cols_block(const RArgs& a, int b);
// a launch mixing both forms: each segment's blocks take its own (block-uniform branch)
__device__ __forceinline__ void reduce_any_block(const RArgs& a, int b, float4 (*red2)[RED_C]) {
  int si = 0;
#pragma unroll 1
  for (int q = 1; q < a.nseg; ++q)
    if (b >= a.blk0[q]) si = q;
  if (a.s[si].cols) reduce_cols_block(a, b);
  else reduce_segments_block(a, b, red2);
}

__global__ __launch_bounds__(256) void reduce_segments_kernel(RArgs a) {
  KStampEnd stamp_(a.ks);
  __shared__ float4 red[RED_G][RED_C];
  reduce_any_block(a, blockIdx.x, red);
}

// few splits (<= 32): one float4 column per thread, all splits summed in order by that thread (4 loads
// in flight), 1024 columns per block -- the large BERT-size segments stream at HBM rate
__device__ __forceinline__ void reduce_cols_block(const RArgs& a, int b) {
  int si = 0;
#pragma unroll 1
  for (int q = 1; q < a.nseg; ++q)
    if (b >= a.blk0[q]) si = q;
  const Seg& S = a.s[si];
  const int64_t n4 = S.n / 4;
  if (S.cols == 4) {
    // large segments of at most 4 splits (the BERT weight slabs): 4 columns per thread, every split's loads of
    // all 4 issued before the first sum (16 float4 in flight instead of 2-4); each column still summed in split
    // order, then the old value -- the same bits as the one-column form
    const int64_t i0 = (int64_t)(b - a.blk0[si]) * 1024 + threadIdx.x;
    const float4* src = reinterpret_cast<const float4*>(S.src);
    const int64_t st4 = S.stride / 4;
    float4 u[4][4];
#pragma unroll
    for (int z = 0; z < 4; ++z)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i4 = i0 + 256 * k;
        u[z][k] = (z < S.splits && i4 < n4) ? src[(int64_t)z * st4 + i4] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    float4 old[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i4 = i0 + 256 * k;
      old[k] = (a.accumulate && i4 < n4) ? reinterpret_cast<const float4*>(S.out)[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i4 = i0 + 256 * k;
      if (i4 >= n4) continue;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int z = 0; z < 4; ++z)
        if (z < S.splits) { acc.x += u[z][k].x; acc.y += u[z][k].y; acc.z += u[z][k].z; acc.w += u[z][k].w; }
      if (a.accumulate) { acc.x += old[k].x; acc.y += old[k].y; acc.z += old[k].z; acc.w += old[k].w; }
      reinterpret_cast<float4*>(S.out)[i4] = acc;
    }
    return;
  }
  const int64_t i4 = (int64_t)(b - a.blk0[si]) * 256 + threadIdx.x;
  if (i4 >= n4) return;
  const float4* src = reinterpret_cast<const float4*>(S.src) + i4;
  const int64_t st4 = S.stride / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int z = 0;
  for (; z + 4 <= S.splits; z += 4) {
    const float4 u0 = src[(int64_t)z * st4], u1 = src[(int64_t)(z + 1) * st4];
    const float4 u2 = src[(int64_t)(z + 2) * st4], u3 = src[(int64_t)(z + 3) * st4];
    acc.x += u0.x; acc.y += u0.y; acc.z += u0.z; acc.w += u0.w;
    acc.x += u1.x; acc.y += u1.y; acc.z += u1.z; acc.w += u1.w;
    acc.x += u2.x; acc.y += u2.y; acc.z += u2.z; acc.w += u2.w;
    acc.x += u3.x; acc.y += u3.y; acc.z += u3.z; acc.w += u3.w;
  }
  for (; z < S.splits; ++z) {
    const float4 u = src[(int64_t)z * st4];
    acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w;
  }
  float4* o = reinterpret_cast<float4*>(S.out) + i4;
  if (a.accumulate) {
    const float4 p = *o;
    acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
  }
  *o = acc;
}

__global__ __launch_bounds__(256) void reduce_cols_kernel(RArgs a) {
  KStampEnd stamp_(a.ks);
  reduce_cols_block(a, blockIdx.x);
}

}  // namespace wg

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// one reduction launch's arguments for segs[0, nseg <= MAXS): RS_ERR_ARG on a bad segment; blk = workgroups,
// cols = every segment takes the column-per-thread form (reduce_cols_kernel; else the mixed launch).  Each
// segment picks its form by its split count: the weight-gradient slabs (tens of splits) stream a column per
// thread at HBM rate, the LayerNorm partial sets (one per row-chain workgroup: 256) take split groups + a tree
static int reduce_args(int nseg, const rs_reduce_segment* segs, int accumulate, wg::RArgs& ra, int& blk, bool& cols) {
  ra = wg::RArgs{};
  ra.nseg = nseg;
  ra.accumulate = accumulate;
  cols = true;
  blk = 0;
  for (int q = 0; q < nseg; ++q) {
    const rs_reduce_segment& g = segs[q];
    if (g.n <= 0 || g.n % 4 || g.stride % 4 || g.splits < 1 || !al16(g.src) || !al16(g.out)) return RS_ERR_ARG;
    const int c = g.splits > wg::COLS_MAX ? 0 : (g.splits <= 4 && g.n / 4 >= 16384) ? 4 : 1;
    cols = cols && c;
    ra.s[q] = {g.src, g.stride, (int)g.splits, (int)g.n, g.out, c};
    ra.blk0[q] = blk;
    blk += (int)cdiv(g.n / 4, c ? 256 * c : (g.splits > 64 ? 4 : wg::RED_C));
  }
  ra.blk0[nseg] = blk;
  return 0;
}

static int launch_segments(int nseg, const rs_reduce_segment* segs, int accumulate, hipStream_t s,
                           KStamp end = KStamp{}) {
  if (nseg <= 0) return 0;
  for (int base = 0; base < nseg; base += wg::MAXS) {
    wg::RArgs ra;
    int blk;
    bool cols;
    if (int e = reduce_args(min(wg::MAXS, nseg - base), segs + base, accumulate, ra, blk, cols)) return e;
    if (base + wg::MAXS >= nseg) ra.ks = end;
    if (cols) hipLaunchKernelGGL(wg::reduce_cols_kernel, dim3((unsigned)blk), dim3(256), 0, s, ra);
    else hipLaunchKernelGGL(wg::reduce_segments_kernel, dim3((unsigned)blk), dim3(256), 0, s, ra);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

extern "C" {

int64_t rs_wgrad_grouped_slab_numel(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split) {
  if (nprob <= 0 || M <= 0 || rows_per_split <= 0) return -1;
  const int64_t splits = cdiv(M, rows_per_split);
  int64_t tot = 0;
  for (int q = 0; q < nprob; ++q) tot += splits * (probs[q].N * probs[q].K + probs[q].N);
  return tot;
}

int rs_reduce_segments(int nseg, const rs_reduce_segment* segs, int accumulate, void* stream) {
  return launch_segments(nseg, segs, accumulate, (hipStream_t)stream);
}

}  // extern "C"

// the grouped launch's arguments (T = output tile edge) and its reduction segments (problems' W and bias
// segments, then the caller's extra ones)
// output tile edge of a grouped launch: 256 when every problem's N and K are multiples of 256, else 128, else 64 --
// at most max_tile (the caller's cap: a launch sharing the chip with a streaming kernel takes the 128-wide tiles)
static int64_t wgrad_tile(int nprob, const rs_wgrad_problem* probs, int64_t max_tile) {
  int64_t T = max_tile >= 256 ? 256 : max_tile >= 128 ? 128 : 64;
  for (int q = 0; q < nprob; ++q)
    while (probs[q].N % T || probs[q].K % T) T /= 2;
  return T < 64 ? 64 : T;
}

static int wgrad_group_args(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                            int64_t slab_numel, int nextra, const rs_reduce_segment* extra, wg::Args& a, int& T_,
                            rs_reduce_segment* segs, int& ns, int64_t max_tile) {
  if (nprob <= 0 || nprob > wg::MAXP || M <= 0 || rows_per_split <= 0 || rows_per_split % 64 || !slab)
    return RS_ERR_ARG;
  int64_t T = wgrad_tile(nprob, probs, max_tile);
  const int64_t splits = cdiv(M, rows_per_split);
  a = wg::Args{};
  a.nprob = nprob;
  a.M = M;
  a.rows_per_split = (int)rows_per_split;
  a.splits = (int)splits;
  a.slab = slab;
  int tiles = 0;
  int64_t off = 0;
  for (int q = 0; q < nprob; ++q) {
    const rs_wgrad_problem& p = probs[q];
    if (p.N <= 0 || p.K <= 0 || p.N % T || p.K % T || p.lddy % 8 || p.ldx % 8 || !al16(p.dY) || !al16(p.X) ||
        !p.dW)
      return RS_ERR_UNSUPPORTED;
    a.p[q] = {(const __bf16*)p.dY, (const __bf16*)p.X, p.lddy, p.ldx, (int)p.N, (int)p.K, (int)(p.K / T), tiles, off};
    tiles += (int)((p.N / T) * (p.K / T));
    off += splits * (p.N * p.K + p.N);
  }
  if (off > slab_numel) return RS_ERR_ARG;
  a.ntiles = tiles;
  T_ = (int)T;
  ns = 0;
  off = 0;
  for (int q = 0; q < nprob; ++q) {
    const rs_wgrad_problem& p = probs[q];
    const int64_t stride = p.N * p.K + p.N;
    segs[ns++] = {slab + off, stride, splits, p.N * p.K, p.dW};
    if (p.db) segs[ns++] = {slab + off + p.N * p.K, stride, splits, p.N, p.db};
    off += splits * stride;
  }
  if (nextra < 0 || nextra > wg::MAXS) return RS_ERR_ARG;
  for (int q = 0; q < nextra; ++q) segs[ns++] = extra[q];
  return 0;
}

extern "C" {

int rs_wgrad_grouped_tile_max(int nprob, const rs_wgrad_problem* probs, int max_tile) {
  if (nprob <= 0 || nprob > wg::MAXP || !probs || max_tile < 64) return -1;
  return (int)wgrad_tile(nprob, probs, max_tile);
}

int rs_wgrad_grouped_tile(int nprob, const rs_wgrad_problem* probs) {
  return rs_wgrad_grouped_tile_max(nprob, probs, 256);
}

int rs_wgrad_grouped_max(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                         int64_t slab_numel, int nextra, const rs_reduce_segment* extra, int max_tile, void* stream) {
  wg::Args a;
  int T, ns;
  rs_reduce_segment segs[2 * wg::MAXP + wg::MAXS];
  if (max_tile < 64) return RS_ERR_ARG;
  if (int e = wgrad_group_args(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, a, T, segs, ns,
                               max_tile))
    return e;
  a.ks = kstamp_next(RS_STAMP_WGRAD_GROUPED);
  hipStream_t s = (hipStream_t)stream;
  wg::launch_group(a, T, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return launch_segments(ns, segs, 1, s, a.ks);
}

int rs_wgrad_grouped(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                     int64_t slab_numel, int nextra, const rs_reduce_segment* extra, void* stream) {
  return rs_wgrad_grouped_max(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, 256, stream);
}

}  // extern "C"
