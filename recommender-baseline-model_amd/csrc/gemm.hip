// MFMA GEMM with fused epilogues for the recsys hot path (gfx950).
//
// C[M,N] = epilogue( alpha * A[M,K] . B[N,K]^T )
//
// Operand storage (template flags):
//   AK = false : A(m,k) at A[m*lda + k]   (row-major activations, "X")
//   AK = true  : A(m,k) at A[k*lda + m]   (transposed view, e.g. dY^T for dW)
//   BK = false : B(n,k) at B[n*ldb + k]   (torch Linear weight [out,in])
//   BK = true  : B(n,k) at B[k*ldb + n]   (weight used as W, or activations for dW)
// Uses in the hot path (reference call sites in BS/models/**):
//   Linear / Conv1d(k=1) forward  Y = X W^T       AK=0 BK=0
//   input gradient               dX = dY W        AK=0 BK=1
//   weight gradient              dW = dY^T X      AK=1 BK=1 (split-K into fp32 slabs)
//
// Tiling: 256 threads = 4 waves (2x2), block tile BM x BN, BK = 32 (one MFMA
// k-chunk), LDS images keep the global orientation (k-contiguous rows for
// AK/BK = 0, m/n-contiguous rows for AK/BK = 1), register-staged prefetch of
// tile k+1 under the MFMAs of tile k.  The block->tile map is XCD-aware: blocks
// b and b+8 share an XCD, so consecutive tile ids go to the same XCD's L2.
#include "gemm_common.h"

template <typename T, bool KMAJ, int ROWS, bool ALIGNED = true>
struct TileLoader {
  // Tile of logical (ROWS x 32) over (row, k).  Global chunks are 16 B along
  // the contiguous axis.  For KMAJ=false: R=ROWS rows of 32 k; for KMAJ=true:
  // 32 k-rows of ROWS elements.
  static constexpr int V = Vec<T>::N;
  static constexpr int GR = KMAJ ? 32 : ROWS;       // global rows in tile
  static constexpr int GC = KMAJ ? ROWS : 32;       // contiguous elements per global row
  static constexpr int CPR = GC / V;                // chunks per row
  static constexpr int NCH = GR * CPR;              // chunks per tile
  static constexpr int PER_T = (NCH + 255) / 256;
  static constexpr int PAD = V;                     // one 16-B chunk of padding per LDS row
  static constexpr int LD = GC + PAD;               // LDS row length
  static constexpr int LDS_ELEMS = GR * LD;
  float buf[PER_T][V];

  __device__ __forceinline__ void load(const T* base, int64_t ld, int64_t r0, int64_t c0,
                                       int64_t rlim, int64_t clim, int tid) {
    // (r0, c0) = global (row, col) origin of the tile in storage orientation
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int ch = tid + i * 256;
      if (ch < NCH) {
        int r = ch / CPR, c = (ch % CPR) * V;
        int64_t gr = r0 + r, gc = c0 + c;
        if (ALIGNED && gr < rlim && gc + V <= clim) {
          load_chunk<T>(buf[i], base + gr * ld + gc);
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j)
            buf[i][j] = (gr < rlim && gc + j < clim) ? to_f(base[gr * ld + gc + j]) : 0.0f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(T* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int ch = tid + i * 256;
      if (ch < NCH) {
        int r = ch / CPR, c = (ch % CPR) * V;
        store_chunk<T>(lds + r * LD + c, buf[i]);
      }
    }
  }
  // fragment for tile-row `row` (0..ROWS-1), k chunk base kb = 8*(lane>>4)
  __device__ __forceinline__ void frag(Frag<T>& f, const T* lds, int row, int kb) const {
    if (!KMAJ) frag_load_vec(f, lds + row * LD + kb);
    else frag_load_strided(f, lds + kb * LD + row, LD);
  }
};

template <typename T>
__device__ __forceinline__ void epilogue_store(const GemmArgs& a, int64_t m, int64_t n, float acc) {
  const rs_epilogue& e = a.epi;
  float v = acc * e.alpha;
  if (e.bias) v += e.bias[n];
  if (e.act == ACT_RELU || e.act == ACT_GELU) {
    if (e.aux_out) reinterpret_cast<T*>(e.aux_out)[m * e.ldaux + n] = from_f<T>(v);
    v = (e.act == ACT_RELU) ? fmaxf(v, 0.0f) : gelu_tanh(v);
  } else if (e.act == ACT_RELU_BWD) {
    v = to_f(reinterpret_cast<const T*>(e.aux)[m * e.ldaux + n]) > 0.0f ? v : 0.0f;
  } else if (e.act == ACT_GELU_BWD) {
    v *= gelu_tanh_grad(to_f(reinterpret_cast<const T*>(e.aux)[m * e.ldaux + n]));
  }
  if (e.drop_p > 0.0f) v *= drop_mul(e.drop_p, eff_seed(e.drop_seed, e.seed_base), (uint64_t)(m * e.drop_ld + n));
  if (e.resid) v += to_f(reinterpret_cast<const T*>(e.resid)[m * e.ldres + n]);
  if (e.rowmask_ids) v = (e.rowmask_ids[m] != 0) ? v : 0.0f;
  if (e.post_drop_p > 0.0f)
    v *= drop_mul(e.post_drop_p, eff_seed(e.post_drop_seed, e.seed_base), (uint64_t)(m * e.drop_ld + n));
  if (a.c_f32) {
    float* C = reinterpret_cast<float*>(a.C) + m * a.ldc + n;
    *C = e.accumulate ? *C + v : v;
  } else {
    T* C = reinterpret_cast<T*>(a.C) + m * a.ldc + n;
    *C = from_f<T>(e.accumulate ? to_f(*C) + v : v);
  }
}

// ALIGNED = false: operands whose leading dimensions / base addresses are not 16-byte multiples (e.g. the
// reference's default SAS width d = 50) are read element by element; everything else is the same kernel.
template <typename T, bool AK, bool BK, int BM, int BN, bool ALIGNED = true>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs a) {
  using LA = TileLoader<T, AK, BM, ALIGNED>;
  using LB = TileLoader<T, BK, BN, ALIGNED>;
  __shared__ __attribute__((aligned(16))) T lds[LA::LDS_ELEMS + LB::LDS_ELEMS];
  T* As = lds;
  T* Bs = lds + LA::LDS_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int FM = BM / 32, FN = BN / 32;  // 16x16 fragments per wave per dim

  // XCD-aware tile mapping (bijective): blocks sharing blockIdx.x % 8 share an XCD.
  const int64_t tiles_n = cdiv(a.N, BN);
  const int64_t nwg = (int64_t)gridDim.x;
  int64_t bid = blockIdx.x;
  {
    int64_t q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int64_t m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;
  const int z = blockIdx.z;
  // device-side row bound (rows of a compaction): M rows for the A-row-major GEMMs, K for wgrad
  const int64_t Mb = (!AK && a.epi.rows_dev) ? min(a.M, (int64_t)*a.epi.rows_dev) : a.M;
  const int64_t Kb = (AK && a.epi.rows_dev) ? min(a.K, (int64_t)*a.epi.rows_dev) : a.K;
  if (m0 >= Mb) return;
  const int64_t kbeg = (int64_t)z * a.k_per_split;
  const int64_t kend = min(Kb, kbeg + a.k_per_split);

  const T* A = reinterpret_cast<const T*>(a.A);
  const T* B = reinterpret_cast<const T*>(a.B);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  LA la;
  LB lb;
  auto issue = [&](int64_t k0) {
    if (!AK) la.load(A, a.lda, m0, k0, Mb, kend, tid);
    else la.load(A, a.lda, k0, m0, kend, a.M, tid);
    if (!BK) lb.load(B, a.ldb, n0, k0, a.N, kend, tid);
    else lb.load(B, a.ldb, k0, n0, kend, a.N, tid);
  };

  // bias gradient fused into the weight-gradient GEMM: the blocks of output
  // column tile 0 also sum their A (= dY^T, k-major) tiles over k
  const bool do_colsum = AK && a.bias_colsum && (bid % tiles_n) == 0;
  float csum = 0.f;
  auto colsum_tile = [&]() {
    if (do_colsum && tid < BM) {
#pragma unroll 8
      for (int kk = 0; kk < 32; ++kk) csum += to_f(As[kk * LA::LD + tid]);
    }
  };

  if (kbeg < kend) {
    issue(kbeg);
    la.store(As, tid);
    lb.store(Bs, tid);
    __syncthreads();
    colsum_tile();
    const int kb = 8 * (lane >> 4), rl = lane & 15;
    for (int64_t k0 = kbeg; k0 < kend; k0 += 32) {
      const bool more = k0 + 32 < kend;
      if (more) issue(k0 + 32);
      Frag<T> fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) la.frag(fa[i], As, wm * (BM / 2) + i * 16 + rl, kb);
#pragma unroll
      for (int j = 0; j < FN; ++j) lb.frag(fb[j], Bs, wn * (BN / 2) + j * 16 + rl, kb);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma(fa[i], fb[j], acc[i][j]);
      __syncthreads();
      if (more) {
        la.store(As, tid);
        lb.store(Bs, tid);
        __syncthreads();
        colsum_tile();
      }
    }
  }

  const int rq = 4 * (lane >> 4), cl = lane & 15;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t n = n0 + wn * (BN / 2) + j * 16 + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * (BM / 2) + i * 16 + rq + r;
        if (m < Mb && n < a.N) {
          if (a.slab) a.slab[(int64_t)z * a.slab_stride + m * a.N + n] = acc[i][j][r];
          else epilogue_store<T>(a, m, n, acc[i][j][r]);
        }
      }
    }
  if (do_colsum && tid < BM && m0 + tid < a.M)
    a.slab[(int64_t)z * a.slab_stride + a.M * a.N + m0 + tid] = csum;
}

template <typename T, bool AK, bool BK>
static hipError_t launch_t(GemmArgs& a, hipStream_t s) {
  const int64_t big = cdiv(a.M, 128) * cdiv(a.N, 128) * a.split_k;
  if (big >= 512) {
    dim3 grid((unsigned)(cdiv(a.M, 128) * cdiv(a.N, 128)), 1, a.split_k);
    hipLaunchKernelGGL((gemm_kernel<T, AK, BK, 128, 128>), grid, dim3(256), 0, s, a);
  } else {
    dim3 grid((unsigned)(cdiv(a.M, 64) * cdiv(a.N, 64)), 1, a.split_k);
    hipLaunchKernelGGL((gemm_kernel<T, AK, BK, 64, 64>), grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

template <typename T, bool AK, bool BK>
static hipError_t launch_unaligned_t(GemmArgs& a, hipStream_t s) {
  dim3 grid((unsigned)(cdiv(a.M, 64) * cdiv(a.N, 64)), 1, a.split_k);
  hipLaunchKernelGGL((gemm_kernel<T, AK, BK, 64, 64, false>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename T>
static hipError_t launch_unaligned(int ak, int bk, GemmArgs& a, hipStream_t s) {
  if (!ak && !bk) return launch_unaligned_t<T, false, false>(a, s);
  if (!ak && bk) return launch_unaligned_t<T, false, true>(a, s);
  if (ak && bk) return launch_unaligned_t<T, true, true>(a, s);
  return launch_unaligned_t<T, true, false>(a, s);
}

template <typename T>
static hipError_t launch_dt(int ak, int bk, GemmArgs& a, hipStream_t s) {
  if (!ak && !bk) return launch_t<T, false, false>(a, s);
  if (!ak && bk) return launch_t<T, false, true>(a, s);
  if (ak && bk) return launch_t<T, true, true>(a, s);
  return launch_t<T, true, false>(a, s);
}

extern "C" {

int rs_gemm(int dtype, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
            const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int c_f32,
            const rs_epilogue* epi, int split_k, float* slab, void* stream) {
  if (M <= 0 || N <= 0 || K < 0 || split_k < 1) return RS_ERR_ARG;
  const int esz = dtype == RS_DTYPE_BF16 ? 2 : 4;
  const int vec = 16 / esz;
  const bool aligned = !((lda % vec) || (ldb % vec) || ((uintptr_t)A % 16) || ((uintptr_t)B % 16));
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % esz) return RS_ERR_ARG;
  if (split_k > 1 && !slab) return RS_ERR_ARG;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
  a.c_f32 = c_f32; a.split_k = split_k;
  a.k_per_split = split_k > 1 ? cdiv(cdiv(K, split_k), 64) * 64 : (K > 0 ? K : 1);
  a.slab = slab;
  a.slab_stride = M * N;
  a.bias_colsum = 0;
  if (epi) a.epi = *epi;
  else { a.epi = rs_epilogue{}; a.epi.alpha = 1.0f; }
  hipStream_t s = (hipStream_t)stream;
  if (!aligned)
    return (int)(dtype == RS_DTYPE_BF16 ? launch_unaligned<__bf16>(a_kmajor, b_kmajor, a, s)
                                        : launch_unaligned<float>(a_kmajor, b_kmajor, a, s));
  hipError_t err = dtype == RS_DTYPE_BF16 ? gemm_bf16_launch(a_kmajor, b_kmajor, a, s)
                                          : launch_dt<float>(a_kmajor, b_kmajor, a, s);
  return (int)err;
}

// dW[N,K] (+)= sum_m dY[m,:]^T X[m,:]  and  db[N] (+)= sum_m dY[m,:]  (split-K over the M token
// rows into fp32 slabs, bias column sums fused into the GEMM, one deterministic reduce pass)
int rs_linear_wgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dY, int64_t lddy, const void* X,
                    int64_t ldx, float* dW, float* db, int accumulate, int splits, float* slab, const int* rows_dev,
                    void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1 || !slab || !dW) return RS_ERR_ARG;
  const int esz = dtype == RS_DTYPE_BF16 ? 2 : 4;
  const int vec = 16 / esz;
  const bool aligned = !((lddy % vec) || (ldx % vec) || ((uintptr_t)dY % 16) || ((uintptr_t)X % 16));
  if (((uintptr_t)slab % 16) || ((uintptr_t)dY | (uintptr_t)X) % esz) return RS_ERR_ARG;
  GemmArgs a{};
  hipStream_t s = (hipStream_t)stream;
  if (aligned && dtype == RS_DTYPE_BF16 && splits == 1 && K % 8 == 0 && ((uintptr_t)dW % 16) == 0) {
    // one split: the tiles accumulate straight into dW (and the ones-operand column sums into db)
    a.M = N; a.N = K; a.K = M; a.A = dY; a.lda = lddy; a.B = X; a.ldb = ldx; a.C = dW; a.ldc = K;
    a.c_f32 = 1; a.split_k = 1; a.k_per_split = M;
    a.bias_colsum = db ? 1 : 0;
    a.colsum_out = db;
    a.epi = rs_epilogue{};
    a.epi.alpha = 1.0f;
    a.epi.accumulate = accumulate;
    a.epi.rows_dev = rows_dev;
    return (int)gemm_bf16_launch(1, 1, a, s);
  }
  a.M = N; a.N = K; a.K = M; a.A = dY; a.lda = lddy; a.B = X; a.ldb = ldx; a.C = nullptr; a.ldc = 0;
  a.c_f32 = 1; a.split_k = splits;
  a.k_per_split = cdiv(cdiv(M, splits), 64) * 64;
  a.slab = slab;
  a.slab_stride = N * K + (db ? N : 0);
  a.bias_colsum = db ? 1 : 0;
  a.epi = rs_epilogue{};
  a.epi.alpha = 1.0f;
  a.epi.rows_dev = rows_dev;
  hipError_t err = !aligned ? (dtype == RS_DTYPE_BF16 ? launch_unaligned_t<__bf16, true, true>(a, s)
                                                     : launch_unaligned_t<float, true, true>(a, s))
                  : dtype == RS_DTYPE_BF16 ? gemm_bf16_launch(1, 1, a, s) : launch_t<float, true, true>(a, s);
  if (err != hipSuccess) return (int)err;
  // one pass over the slabs: columns [0, N*K) -> dW, [N*K, N*K+N) -> db
  return (int)launch_reduce_slabs(slab, splits, a.slab_stride, N * K, dW, db, accumulate, s);
}

}  // extern "C"
