// Large-tile bf16 GEMM for the vocabulary head's two weight-sized products (gfx950), output width N = 256:
//
//   dE[v][:] = sum_r dlogits[r][v] h[r][:]      (A k-major: the gradient of out.weight, BS/models/bert.py:10,16;
//   db[v]    = sum_r dlogits[r][v]                the bias gradient rides along as MFMAs against ones)
//   dh[r][:] = sum_v dlogits[r][v] E[v][:]      (A k-contiguous, split over the vocabulary into fp32 slabs that
//                                                rs_splitk_scatter_rows sums, casts and scatters to the tokens)
//
// At the cfg5 shape (1M classes x 256 x ~1.8k labelled rows) both are ~0.9 TFLOP and stream the 3.6 GB dlogits
// once: arithmetic intensity ~256 flop/B, just under the bf16 ridge, so the floor is HBM (~0.5 ms each).  The
// generic 128x128 kernel (gemm_bf16_impl.h) covers only half of N per tile, so dE read dlogits TWICE, and its
// 4-wave 64x64 per-wave tiles pay one LDS fragment read per 2 MFMAs.  Here:
//
//  * a 256 x 256 output tile (the whole N) per 8-wave workgroup: A streams from HBM exactly once; each wave owns a
//    128 x 64 quadrant (8 x 4 accumulator tiles of mfma_f32_16x16x32_bf16: 3 fragment reads per 8 MFMAs);
//  * 32-deep k stages loaded by LDS-DMA into four stage buffers, three in flight (below); k-major operands read
//    with ds_read_b64_tr_b16 (the transposing LDS read);
//  * dh's split-K workgroups are dealt so that the row tiles of one vocabulary slice share an XCD (its L2 holds
//    the slice of E they all read);
//  * the epilogue stages the fp32 tile through LDS in two 128-row halves and stores 1 KB rows.
#include "common.h"
#include "dma256.h"
#include "../../include/recsys_hip.h"

namespace g256 {

struct Args {
  int64_t M, K;                   // N = 256
  const __bf16* A; int64_t lda;   // A(m, k) = A[k*lda + m] (a_kmajor) or A[m*lda + k]
  const __bf16* B; int64_t ldb;   // B(k, n) = B[k*ldb + n]
  float* C; int64_t ldc;          // C[z*cz + m*ldc + n]
  int64_t cz, k_per_split;
  float* colsum;                  // a_kmajor: colsum[m] = sum_k A(m, k) (nullable)
  const int* rows_dev;            // a_kmajor: bound on K; else bound on M (nullable)
};

template <bool AK>
__global__ __launch_bounds__(NTH) void gemm_n256_dma_kernel(Args a) {
  constexpr int LDC = BN + 4;
  constexpr int LDS_BYTES = NBUF * DSTAGE > (BM / 2) * LDC * 4 ? NBUF * DSTAGE : (BM / 2) * LDC * 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  constexpr int FM = 8, FN = 4;

  const int64_t Mb = (!AK && a.rows_dev) ? min(a.M, (int64_t)*a.rows_dev) : a.M;
  const int64_t Kb = (AK && a.rows_dev) ? min(a.K, (int64_t)*a.rows_dev) : a.K;
  const unsigned tiles_m = (unsigned)((a.M + BM - 1) / BM);
  unsigned tm, z;
  {
    const unsigned tot = gridDim.x, L = blockIdx.x, q = tot >> 3, r = tot & 7, x = L & 7;
    const unsigned lg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
    z = lg / tiles_m;
    tm = lg - z * tiles_m;
  }
  const int64_t m0 = (int64_t)tm * BM;
  if (m0 >= Mb) return;
  const int64_t kbeg = (int64_t)z * a.k_per_split;
  const int64_t kend = min(Kb, kbeg + a.k_per_split);
  const int nk = kend > kbeg ? (int)((kend - kbeg + DBK - 1) / DBK) : 0;
  const uint32_t lds0 = lds_u32(smem);

  f32x4 acc[FM][FN], accb[2];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  accb[0] = accb[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  const bool do_colsum = AK && a.colsum != nullptr;
  // A's column bound for clamping: the allocated row length (k-major A: the m extent; the k-contiguous A: k)
  const int64_t a_cols = a.lda;

  // this wave's 4 DMA pieces of stage t (A pieces 2w, 2w+1; B pieces 2w, 2w+1)
  auto issue = [&](int t) {
    const uint32_t buf = lds0 + (uint32_t)((t % NBUF) * DSTAGE);
    const int64_t k0 = kbeg + (int64_t)t * DBK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j;
      if (AK) km_piece(a.A, a.lda, k0, m0, kend, a_cols, pc, lane, buf);
      else kc_piece(a.A, a.lda, m0, k0, a.M, a_cols, pc, lane, buf);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) km_piece(a.B, a.ldb, k0, 0, kend, a.ldb, 2 * wave + j, lane, buf + IMG_BYTES);
  };
  // zero the k positions past kend of stage t's images (the last stage only)
  auto zero_tail = [&](int t) {
    char* buf = smem + (t % NBUF) * DSTAGE;
    const int kv = (int)(kend - (kbeg + (int64_t)t * DBK));      // valid k in this stage, 1..31
    // k-major images: rows >= kv, 256 columns each (B always; A when AK)
    for (int e = tid; e < (DBK - kv) * 256; e += NTH) {
      const int r = kv + e / 256, c = e % 256;
      *reinterpret_cast<__bf16*>(buf + IMG_BYTES + km_off(r, c)) = (__bf16)0.0f;
      if (AK) *reinterpret_cast<__bf16*>(buf + km_off(r, c)) = (__bf16)0.0f;
    }
    if (!AK)
      for (int e = tid; e < BM * (DBK - kv); e += NTH) {
        const int m = e / (DBK - kv), k = kv + e % (DBK - kv);
        *reinterpret_cast<__bf16*>(buf + kc_off(m, k)) = (__bf16)0.0f;
      }
  };
  auto compute = [&](int t) {
    const char* buf = smem + (t % NBUF) * DSTAGE;
    bf16x8 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = AK ? km_frag(buf, wm * 128 + 16 * i, lane) : kc_frag(buf, wm * 128 + 16 * i, lane);
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
  for (int t = 0; t < min(nk, DIST); ++t) issue(t);
  for (int t = 0; t < nk; ++t) {
    const int after = min(nk - 1, t + DIST - 1) - t;   // stages issued after t, allowed to stay in flight
    vm_wait_stages(after);
    raw_barrier();                                      // stage t landed everywhere; buffer (t - 1) % NBUF free
    if (t + DIST < nk) issue(t + DIST);
    if (tail && t == nk - 1) {
      zero_tail(t);
      raw_barrier();
    }
    compute(t);
  }
  vm_wait<0>();

  // ---- epilogue: as the register-staged kernel's
  float* Cs = reinterpret_cast<float*>(smem);
  float* Cz = a.C + (int64_t)z * a.cz;
  const int g = lane >> 4, cl = lane & 15;
  if (do_colsum && cl == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 128 + 16 * (2 * wn + t) + 4 * g + r;
        if (m < a.M) a.colsum[m] = accb[t][r];
      }
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
      if (m >= a.M) break;
      const float4 v0 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8 + 4);
      float* dst = Cz + m * a.ldc + c8;
      *reinterpret_cast<float4*>(dst) = v0;
      *reinterpret_cast<float4*>(dst + 4) = v1;
    }
  }
}

// the k split of a k-contiguous product (dh): as many splits as fill the 256 CUs with whole row tiles, each a
// multiple of the 64-deep stage
static void splits_for(int64_t M, int64_t K, int& splits, int64_t& kps) {
  const int64_t tiles = (M + BM - 1) / BM;
  int64_t s = std::max<int64_t>(1, 256 / tiles);
  s = std::min<int64_t>(s, (K + BKT - 1) / BKT);
  kps = ((K + s - 1) / s + BKT - 1) / BKT * BKT;
  splits = (int)((K + kps - 1) / kps);
}

}  // namespace g256

extern "C" {

int rs_gemm_n256_splits(int64_t M, int64_t K) {
  if (M <= 0 || K <= 0) return -1;
  int s;
  int64_t kps;
  g256::splits_for(M, K, s, kps);
  return s;
}

int rs_gemm_n256(int a_kmajor, int64_t M, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                 int64_t ldc, int split, int64_t c_split_stride, float* colsum, const int* rows_dev, void* stream) {
  if (M <= 0 || K <= 0 || !A || !B || !C || ldb < 256 || ldc < 256 || (colsum && !a_kmajor) ||
      (lda % 8) || (ldb % 8) || (ldc % 4) || ((uintptr_t)A % 16) || ((uintptr_t)B % 16) || ((uintptr_t)C % 16))
    return RS_ERR_ARG;
  if (a_kmajor ? lda < M : lda < K) return RS_ERR_ARG;
  g256::Args a{M, K, (const __bf16*)A, lda, (const __bf16*)B, ldb, C, ldc, c_split_stride, K, colsum, rows_dev};
  int splits = 1;
  if (split) {
    g256::splits_for(M, K, splits, a.k_per_split);
    if (splits > 1 && c_split_stride < M * ldc) return RS_ERR_ARG;
  }
  const dim3 grid((unsigned)(((M + g256::BM - 1) / g256::BM) * splits)), blk(g256::NTH);
  hipStream_t s = (hipStream_t)stream;
  if (a_kmajor) hipLaunchKernelGGL(g256::gemm_n256_dma_kernel<true>, grid, blk, 0, s, a);
  else hipLaunchKernelGGL(g256::gemm_n256_dma_kernel<false>, grid, blk, 0, s, a);
  return (int)hipGetLastError();
}

}  // extern "C"
