// LDS-DMA pipelined form of the bf16 block GEMM (gfx950), included by gemm_bf16_impl.h before its tile dispatch.
//
// The BERT block products (M = B*T = 12,800 token rows, N / K = 256 / 768 / 1,024: QKV, output projection, FFN
// in both orientations) are short in K (8-32 stages of 32) and wide in M, so the register-staged kernel above
// spends its time waiting: one stage in flight, and HBM / L2 latency under load (~1-2 us) paid once per stage.
// Here, as in gemm_n256.hip's vocabulary GEMM:
//
//  * 32-deep k stages loaded by global_load_lds_dwordx4 straight into FOUR LDS stage buffers, three stages in
//    flight per wave (counted vmcnt, never drained in the main loop), one raw s_barrier per stage;
//  * no staging registers: the images are lane-linear 1-KB DMA pieces, so the bank-conflict-free layouts move to
//    the SOURCE address -- k-contiguous images [rows][32 k] (64-B rows) with chunk g of row m at g ^ h((m >> 2) & 3),
//    h = {0, 2, 3, 1}; the k-major weight image of the input-gradient products [32 k][128 n] in 8-row x 32-column
//    subtiles (read by ds_read_b64_tr_b16);
//  * tiles BM x 128 (BM = 64 or 128) over 4 waves (2 x 2), 2 workgroups per CU; every k stage is one
//    mfma_f32_16x16x32_bf16 step, in k order -- so each output element sees exactly the register-staged kernel's
//    accumulation sequence (bit-identical results, tests/test_gemm_dma_gpu.py);
//  * the epilogue is the register-staged kernel's epi_rows (all compile-time epilogue classes), staged through LDS
//    64 rows at a time.
//
// Taken for A k-contiguous (forward X.W^T and input gradient dY.W), N % 128 == 0, K % 32 == 0, no split-K, a
// compile-time epilogue class.  RS_GEMM_DMA=0 selects the register-staged kernel (read per launch, for A/B);
// RS_GEMM_DMA_BM=128 takes 128-row tiles.  Measured at the cfg3 shapes (tools/diag/gemm_epi.py, M = 12,800, same
// session; register-staged -> DMA 128-row -> DMA 64-row tiles, us): QKV + bias 24.7 -> 16.2 -> 15.2, QKV input
// gradient 16.5 -> 14.4 -> 12.9, FFN1 + bias + GELU + dropout + pre-activation 24.9 -> 25.9 -> 22.5, FFN2 + bias +
// dropout + residual + post-dropout 20.2 -> 17.7 -> 17.7, FFN2 input gradient + GELU' + dropout 26.0 -> 27.4 -> 22.9,
// FFN1 input gradient 19.0 -> 16.7 -> 15.0, output projection 9.1 / 9.0 / 9.0 (both orientations); whole cfg3 step
// 41.1k -> 43.3k seq/s.  64-row tiles (3 workgroups per CU) are the default.
// (included inside namespace gbf: epi_rows, GemmArgs and the epilogue classes are those above)
#pragma once

namespace dma {

constexpr int DBK = 32, NBUF = 4, DIST = 3, BN = 128, NTH = 256;
constexpr int IMG_B = BN * DBK * 2;   // the B operand's stage image (8 KB, either orientation)

__device__ __forceinline__ uint32_t kc_swz(int m) { return (uint32_t)((0x1320u >> (4 * ((m >> 2) & 3))) & 3u); }
// byte offset of element (row m, k) of a k-contiguous stage image [rows][32]
__device__ __forceinline__ uint32_t kc_off(int m, int k) {
  return (uint32_t)(64 * m + 16 * ((uint32_t)(k >> 3) ^ kc_swz(m)) + 2 * (k & 7));
}
// byte offset of element (k row r, column c < 128) of the k-major stage image [32][128]: 8-row x 32-column subtiles
// of 512 B, chunk (ch & 3) ^ ((r >> 2) & 3) inside its 64-B subtile row (cdna_hip_programming.md T10, image (a))
__device__ __forceinline__ uint32_t km_off(int r, int c) {
  const int ch = c >> 3;
  return (uint32_t)(2048 * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3)) + 2 * (c & 7));
}

typedef __attribute__((address_space(3))) void* lds_vptr;
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)(lds_vptr)p; }
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// piece j of a k-contiguous image: rows 16j .. 16j+15 (64 B each); lane l stores chunk position l & 3 of row
// 16j + (l >> 2), which holds logical chunk (l & 3) ^ h(row).  Rows past rlim read row rlim - 1 (finite; their
// outputs are never stored).
__device__ __forceinline__ void kc_piece(const __bf16* base, int64_t ld, int64_t r0, int64_t k0, int64_t rlim, int j,
                                         int lane, uint32_t img) {
  const int r = 16 * j + (lane >> 2);
  const int ch = (lane & 3) ^ (int)kc_swz(r);
  const int64_t row = min(r0 + r, rlim - 1);
  dma16(base + row * ld + k0 + 8 * ch, __builtin_amdgcn_readfirstlane(img + (uint32_t)j * 1024));
}
// piece j (0..7) of the k-major image: byte b = 1024 j + 16 l holds (k row r, logical chunk ch) of the subtile layout
__device__ __forceinline__ void km_piece(const __bf16* base, int64_t ld, int64_t k0, int64_t c0, int j, int lane,
                                         uint32_t img) {
  const int b = 1024 * j + 16 * lane;
  const int r = 8 * (b >> 11) + ((b >> 6) & 7);
  const int ch = 4 * ((b >> 9) & 3) + (((b >> 4) & 3) ^ ((r >> 2) & 3));
  dma16(base + (k0 + r) * ld + c0 + 8 * ch, __builtin_amdgcn_readfirstlane(img + (uint32_t)j * 1024));
}
__device__ __forceinline__ bf16x8 kc_frag(const char* img, int row0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  return *reinterpret_cast<const bf16x8*>(img + kc_off(row0 + li, 8 * g));
}
__device__ __forceinline__ bf16x8 km_frag(const char* img, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int c = col0 + 4 * p, r = 8 * g + q;
  const bf4 x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)(img + km_off(r, c)));
  const bf4 y =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)(img + km_off(r + 4, c)));
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

// LNA: the A operand is the BERT LayerNorm (BS/models/bert_modules/utils/layer_norm.py:14-17) of the rows of X
// (a.A, K = d = 256), formed in the prologue instead of by a launch of its own (rs_layernorm_fwd variant 1 +
// rs_gemm): thread t holds row t / 4's 16-B chunks 4 j + t % 4 (j = 0..7: stage j's chunk of that row), so
// (a) the row statistics follow ln_fwd_v_kernel's arithmetic exactly -- per-chunk sums in element order, then the
//     32-chunk butterfly (chunk c with c ^ 16, ^ 8, ^ 4 inside the thread, ^ 2 and ^ 1 by lane shuffles) -- and the
//     normalised values, hence the GEMM, are bit-identical to the two-launch form;
// (b) stage j's A image is one 16-B LDS write per thread (the k-contiguous swizzled layout), issued with the
//     stage's B DMA; no A DMAs at all;
// (c) the column-tile-0 workgroups store h and (mean, rinv) after the main loop (stores count in vmcnt: issued
//     earlier they would lengthen the stage waits).
template <bool BK, int BM, int EC, bool LNA = false>
__global__ __launch_bounds__(NTH, 2) void gemm_dma_kernel(GemmArgs a) {
  KStampBegin stamp_b_(a.ks);
  KStampEnd stamp_e_(a.ks);
  static_assert(!LNA || (BM == 64 && !BK), "the LayerNorm prologue: forward orientation, 64-row tiles");
  constexpr int IMG_A = BM * DBK * 2, DSTAGE = IMG_A + IMG_B;
  constexpr int LDC = BN + 4, HR = 64;            // epilogue: 64 rows of the fp32 tile per LDS pass
  constexpr int LDS_MAIN = NBUF * DSTAGE > HR * LDC * 4 ? NBUF * DSTAGE : HR * LDC * 4;
  constexpr int LDS_BYTES = LDS_MAIN + (LNA ? 2 * 256 * 4 : 0);   // LNA: gamma, beta (fp32) after the stages
  constexpr int PA = LNA ? 0 : BM / 64, PB = 2, PPS = PA + PB;   // DMA pieces per wave per stage (A, B)
  constexpr int FM = BM / 32, FN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // block -> tile as the register-staged kernel (XCD-contiguous ranges, shorter tile axis fastest)
  const unsigned tiles_n = (unsigned)(a.N / BN);
  const int64_t Mb = a.epi.rows_dev ? min(a.M, (int64_t)*a.epi.rows_dev) : a.M;
  unsigned tiles_m = gridDim.x / tiles_n, bid = blockIdx.x, nwg = gridDim.x;
  if (a.epi.rows_dev) {
    tiles_m = (unsigned)((Mb + BM - 1) / BM);
    nwg = tiles_m * tiles_n;
    if (bid >= nwg) return;
  }
  {
    const unsigned q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  unsigned tm, tn;
  if (tiles_m < tiles_n) {
    tn = bid / tiles_m;
    tm = bid - tn * tiles_m;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  if (m0 >= Mb) return;
  const int nk = (int)(a.K / DBK);
  const __bf16* A = reinterpret_cast<const __bf16*>(a.A);
  const __bf16* B = reinterpret_cast<const __bf16*>(a.B);
  const uint32_t lds0 = lds_u32(smem);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // LNA: this thread's normalised A chunks (row lr, chunk 4 j + lq of stage j), kept for the h store
  bf16x8 hq[LNA ? 8 : 1];
  const int lr = tid >> 2, lq = tid & 3;
  auto issue = [&](int t) {
    const uint32_t buf = lds0 + (uint32_t)((t % NBUF) * DSTAGE);
    const int64_t k0 = (int64_t)t * DBK;
    if constexpr (LNA) {
      *reinterpret_cast<bf16x8*>(smem + (t % NBUF) * DSTAGE + 64 * lr + 16 * ((uint32_t)lq ^ kc_swz(lr))) = hq[t];
    }
#pragma unroll
    for (int j = 0; j < PA; ++j) kc_piece(A, a.lda, m0, k0, a.M, wave * PA + j, lane, buf);
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      if (BK) km_piece(B, a.ldb, k0, n0, wave * PB + j, lane, buf + IMG_A);
      else kc_piece(B, a.ldb, n0, k0, a.N, wave * PB + j, lane, buf + IMG_A);
    }
  };
  auto compute = [&](int t) {
    const char* buf = smem + (t % NBUF) * DSTAGE;
    bf16x8 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = kc_frag(buf, wm * (BM / 2) + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      fb[j] = BK ? km_frag(buf + IMG_A, wn * 64 + 16 * j, lane) : kc_frag(buf + IMG_A, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };

  float ln_mu = 0.f, ln_r = 0.f;
  if constexpr (LNA) {
    // ln_fwd_v_kernel's arithmetic, contraction spelled out the same way (fmaf where it has fmaf, nothing else)
#pragma clang fp contract(off)
    // the row's chunks and the matching gamma / beta, then the first stages' B DMAs: every load before the stats
    const int64_t xr = min(m0 + lr, a.M - 1);
    const __bf16* xp = A + xr * a.lda + 8 * lq;
    bf16x8 xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = *reinterpret_cast<const bf16x8*>(xp + 32 * j);
    // gamma / beta to LDS (one float4 per thread: 128 threads each), read back per chunk for the normalisation
    // (held in registers they pushed the kernel to 172 VGPRs: two workgroups per CU instead of three)
    float* lnp = reinterpret_cast<float*>(smem + LDS_MAIN);
    const float4 gb = tid < 64 ? reinterpret_cast<const float4*>(a.ln.gamma)[tid]
                               : reinterpret_cast<const float4*>(a.ln.beta)[(tid - 64) & 63];
#pragma unroll
    for (int t = 0; t < DIST; ++t) {                    // B only (the A writes need the stats)
#pragma unroll
      for (int j = 0; j < PB; ++j) kc_piece(B, a.ldb, n0, (int64_t)t * DBK, a.N, wave * PB + j, lane,
                                            lds0 + (uint32_t)(t * DSTAGE) + IMG_A);
    }
    vm_wait<DIST * PB>();                               // the x / gamma / beta loads (older than the DMAs)
    if (tid < 128) reinterpret_cast<float4*>(lnp)[tid] = gb;
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s[j] += (float)xv[j][e];
    }
    // ln_fwd_v_kernel<bf16, 32, 1, 1>: group_sum<32> over the row's 32 chunk sums, chunk c in lane c; here
    // chunk c = 4 j + lq: c ^ 16 / ^ 8 / ^ 4 = j ^ 4 / ^ 2 / ^ 1 (this thread), c ^ 2 / ^ 1 = lanes tid ^ 2 / ^ 1
    auto tree = [&](float* v) {
      float l1[4], l2[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) l1[j] = v[j] + v[j + 4];
#pragma unroll
      for (int j = 0; j < 2; ++j) l2[j] = l1[j] + l1[j + 2];
      float l3 = l2[0] + l2[1];
      l3 += __shfl_xor(l3, 2, 64);
      l3 += __shfl_xor(l3, 1, 64);
      return l3;
    };
    const float mu = tree(s) / 256.f;
    float qs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      qs[j] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float u = (float)xv[j][e] - mu;
        qs[j] = __builtin_fmaf(u, u, qs[j]);
      }
    }
    const float q = tree(qs);
    const float rinv = 1.0f / (sqrtf(q / 255.f) + a.ln.eps);
    ln_mu = mu;
    ln_r = rinv;
    __syncthreads();                                    // gamma / beta in LDS
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c0 = 32 * j + 8 * lq;
      const float4 g0 = *reinterpret_cast<const float4*>(lnp + c0), g1 = *reinterpret_cast<const float4*>(lnp + c0 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(lnp + 256 + c0);
      const float4 b1 = *reinterpret_cast<const float4*>(lnp + 256 + c0 + 4);
      const float gm[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bt[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float u = (float)xv[j][e] - mu;
        hq[j][e] = (__bf16)__builtin_fmaf(gm[e], u * rinv, bt[e]);
      }
    }
#pragma unroll
    for (int t = 0; t < DIST; ++t)
      *reinterpret_cast<bf16x8*>(smem + t * DSTAGE + 64 * lr + 16 * ((uint32_t)lq ^ kc_swz(lr))) = hq[t];
  } else {
    for (int t = 0; t < min(nk, DIST); ++t) issue(t);
  }
  auto step = [&](int t, int nkk) {
    const int after = min(nkk - 1, t + DIST - 1) - t;  // stages issued after t, allowed to stay in flight
    if (after >= 2) vm_wait<2 * PPS>();
    else if (after == 1) vm_wait<PPS>();
    else vm_wait<0>();
    raw_barrier();                                      // stage t landed everywhere; buffer (t - 1) % NBUF free
    if (t + DIST < nkk) issue(t + DIST);
    compute(t);
  };
  if constexpr (LNA) {
    // K = 256: eight stages, unrolled so the register chunks hq[t] are indexed statically (a runtime index would
    // put the array in scratch memory)
#pragma unroll
    for (int t = 0; t < 8; ++t) step(t, 8);
  } else {
    for (int t = 0; t < nk; ++t) step(t, nk);
  }
  if constexpr (LNA) {
    // column tile 0: the LayerNorm output and its row statistics (the backward's operands)
    const int64_t row = m0 + lr;
    if (tn == 0 && row < Mb) {
      if (a.ln.h) {
        __bf16* hp = reinterpret_cast<__bf16*>(a.ln.h) + row * a.ln.ldh + 8 * lq;
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<bf16x8*>(hp + 32 * j) = hq[j];
      }
      if (lq == 0) {
        if (a.ln.mean) a.ln.mean[row] = ln_mu;
        if (a.ln.rinv) a.ln.rinv[row] = ln_r;
      }
    }
  }

  // ---- epilogue through LDS, 64 rows per pass
  float* Cs = reinterpret_cast<float*>(smem);
  const int g = lane >> 4, cl = lane & 15;
  constexpr int TPR = BN / 8, RPP = NTH / TPR;          // 16 threads per row, 16 rows per pass
  const int c8 = (tid % TPR) * 8;
  const int64_t n = n0 + c8;
  uint32_t s1 = 0, s2 = 0;
  if constexpr ((EC & ED) != 0) s1 = seed32(eff_seed(a.epi.drop_seed, a.epi.seed_base));
  if constexpr ((EC & EP) != 0) s2 = seed32(eff_seed(a.epi.post_drop_seed, a.epi.seed_base));
#pragma unroll
  for (int half = 0; half < BM / HR; ++half) {
    __syncthreads();
    if (BM == HR || wm == half) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[((BM == HR ? wm * (BM / 2) : 0) + 16 * i + 4 * g + r) * LDC + wn * 64 + 16 * j + cl] = acc[i][j][r];
    }
    __syncthreads();
    epi_rows<EC, HR / RPP, RPP, LDC>(a, Cs, tid / TPR, c8, m0 + half * HR, Mb, n, s1, s2);
  }
}

// Weight-gradient orientation, one split (the BERT vocabulary head's dE = dlogits^T h below the 64k classes where
// gemm_n256 takes over; rs_linear_wgrad's direct path): C[m][n] (+)= sum_k A[k][m] B[k][n], both operands k-major
// ([32 k][128] stage images, transposing reads), 128 x 128 tiles, the k bound from the device row count, the last
// partial stage zeroed in LDS; the bias column sums colsum_out[m] ride on MFMAs against ones in the tiles of column
// tile 0 (as the register-staged kernel); fp32 C stored from the accumulators.
template <int UNUSED = 0>   // a template: the header is compiled into several translation units
__global__ __launch_bounds__(NTH, 2) void gemm_dma_wgrad_kernel(GemmArgs a) {
  KStampBegin stamp_b_(a.ks);
  KStampEnd stamp_e_(a.ks);
  constexpr int IMG = 32 * 128 * 2, DSTAGE = 2 * IMG, PPS = 4, FM = 4, FN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * DSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const unsigned tiles_n = (unsigned)(a.N / BN), tiles_m = gridDim.x / tiles_n;
  unsigned bid = blockIdx.x;
  {
    const unsigned nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  unsigned tm, tn;
  if (tiles_m < tiles_n) {
    tn = bid / tiles_m;
    tm = bid - tn * tiles_m;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
  const int64_t m0 = (int64_t)tm * 128, n0 = (int64_t)tn * BN;
  const int64_t Kb = a.epi.rows_dev ? min(a.K, (int64_t)*a.epi.rows_dev) : a.K;
  const int nk = Kb > 0 ? (int)((Kb + DBK - 1) / DBK) : 0;
  const __bf16* A = reinterpret_cast<const __bf16*>(a.A);
  const __bf16* B = reinterpret_cast<const __bf16*>(a.B);
  const bool do_colsum = a.colsum_out != nullptr && tn == 0 && wn == 0;
  const uint32_t lds0 = lds_u32(smem);
  f32x4 acc[FM][FN], accb[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    accb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  auto issue = [&](int t) {
    const uint32_t buf = lds0 + (uint32_t)((t % NBUF) * DSTAGE);
    const int64_t k0 = (int64_t)t * DBK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j, b = 1024 * pc + 16 * lane;
      const int r = 8 * (b >> 11) + ((b >> 6) & 7);
      const int ch = 4 * ((b >> 9) & 3) + (((b >> 4) & 3) ^ ((r >> 2) & 3));
      const int64_t k = min(k0 + r, Kb - 1);
      const int64_t ca = min(m0 + 8 * ch, a.lda - 8);        // columns past M: inside the row, never stored
      dma16(A + k * a.lda + ca, __builtin_amdgcn_readfirstlane(buf + (uint32_t)pc * 1024));
      dma16(B + k * a.ldb + n0 + 8 * ch, __builtin_amdgcn_readfirstlane(buf + IMG + (uint32_t)pc * 1024));
    }
  };
  auto zero_tail = [&](int t) {
    char* buf = smem + (t % NBUF) * DSTAGE;
    const int kv = (int)(Kb - (int64_t)t * DBK);
    for (int e = tid; e < (DBK - kv) * 128; e += NTH) {
      const int r = kv + e / 128, c = e % 128;
      *reinterpret_cast<__bf16*>(buf + km_off(r, c)) = (__bf16)0.0f;
      *reinterpret_cast<__bf16*>(buf + IMG + km_off(r, c)) = (__bf16)0.0f;
    }
  };
  auto compute = [&](int t) {
    const char* buf = smem + (t % NBUF) * DSTAGE;
    bf16x8 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = km_frag(buf, wm * 64 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = km_frag(buf + IMG, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (do_colsum) {
#pragma unroll
      for (int i = 0; i < FM; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb[i], 0, 0, 0);
    }
  };
  const bool tail = (Kb % DBK) != 0;
  for (int t = 0; t < min(nk, DIST); ++t) issue(t);
  for (int t = 0; t < nk; ++t) {
    const int after = min(nk - 1, t + DIST - 1) - t;
    if (after >= 2) vm_wait<2 * PPS>();
    else if (after == 1) vm_wait<PPS>();
    else vm_wait<0>();
    raw_barrier();
    if (t + DIST < nk) issue(t + DIST);
    if (tail && t == nk - 1) {
      zero_tail(t);
      raw_barrier();
    }
    compute(t);
  }
  vm_wait<0>();
  float* C = reinterpret_cast<float*>(a.C);
  const int g = lane >> 4, cl = lane & 15;
  const bool accum = a.epi.accumulate != 0;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float* c = C + m * a.ldc + n0 + wn * 64 + 16 * j + cl;
        *c = accum ? *c + acc[i][j][r] : acc[i][j][r];
      }
      if (do_colsum && cl == 0) a.colsum_out[m] = (accum ? a.colsum_out[m] : 0.f) + accb[i][r];
    }
}

inline bool enabled() {
  const char* e = getenv("RS_GEMM_DMA");
  return e ? atoi(e) != 0 : true;
}

// launch the DMA form when the call fits it (returns hipErrorNotSupported otherwise)
template <bool BK, int EC>
hipError_t launch(GemmArgs& a, hipStream_t s) {
  if (!enabled() || a.split_k != 1 || a.N % BN || a.K % DBK || a.K < DBK || a.lda % 8 || a.ldb % 8 ||
      ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15))
    return hipErrorNotSupported;
  const char* f = getenv("RS_GEMM_DMA_BM");
  const int force = f ? atoi(f) : 0;
  const int64_t big = cdiv(a.M, 128) * (a.N / BN);
  const bool bm128 = force == 128;   // 64-row tiles by default: at every cfg3 shape as fast or faster (header)
  if (bm128) {
    hipLaunchKernelGGL((gemm_dma_kernel<BK, 128, EC>), dim3((unsigned)big), dim3(NTH), 0, s, a);
  } else {
    hipLaunchKernelGGL((gemm_dma_kernel<BK, 64, EC>), dim3((unsigned)(cdiv(a.M, 64) * (a.N / BN))), dim3(NTH), 0, s,
                       a);
  }
  return hipGetLastError();
}

// C = epi(LN(X) W^T) with the LayerNorm in the prologue (gemm_dma_kernel LNA): K = 256 (the whole row in one tile
// row), N % 128 == 0, no split; hipErrorNotSupported otherwise
template <int EC>
hipError_t launch_ln(GemmArgs& a, hipStream_t s) {
  if (a.split_k != 1 || a.N % BN || a.K != 256 || a.lda % 8 || a.ldb % 8 || ((uintptr_t)a.A & 15) ||
      ((uintptr_t)a.B & 15) || !a.ln.gamma || !a.ln.beta || ((uintptr_t)a.ln.gamma & 15) ||
      ((uintptr_t)a.ln.beta & 15) || (a.ln.h && (a.ln.ldh % 8 || ((uintptr_t)a.ln.h & 15))))
    return hipErrorNotSupported;
  hipLaunchKernelGGL((gemm_dma_kernel<false, 64, EC, true>), dim3((unsigned)(cdiv(a.M, 64) * (a.N / BN))), dim3(NTH),
                     0, s, a);
  return hipGetLastError();
}

// the weight-gradient form when the call fits it (hipErrorNotSupported otherwise): one split, fp32 C, alpha 1, no
// other epilogue, N % 128 == 0
inline hipError_t launch_wgrad(GemmArgs& a, hipStream_t s) {
  const rs_epilogue& e = a.epi;
  if (!enabled() || a.split_k != 1 || a.slab || !a.c_f32 || e.alpha != 1.0f || e.bias || e.act || e.aux ||
      e.aux_out || e.drop_p > 0.f || e.resid || e.rowmask_ids || e.post_drop_p > 0.f || a.N % BN || a.M < 8 ||
      a.lda % 8 || a.ldb % 8 || a.lda < a.M || ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15))
    return hipErrorNotSupported;
  hipLaunchKernelGGL(gemm_dma_wgrad_kernel<0>, dim3((unsigned)(cdiv(a.M, 128) * (a.N / BN))), dim3(NTH), 0, s, a);
  return hipGetLastError();
}

}  // namespace dma
