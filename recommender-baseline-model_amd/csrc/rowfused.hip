// Row-block fused SASRec sublayers (bf16, gfx950).
//
// Everything in a SAS block except the attention core is row-local: LayerNorm, the
// Linear / Conv1d(k=1) GEMMs (K = N = d <= 256), bias, ReLU, dropout, residuals and the
// timeline mask.  One workgroup owns 64 token rows and runs a whole chain with the
// activations in LDS, reading weights straight from L2 as MFMA B fragments:
//
//   rs_sas_block_in   (sas.py:73-76 before the attention core)
//        X -> Q = LN1(X) [saved], q = Q Wq^T + bq, kv = X Wkv^T + bkv
//   rs_sas_block_out  (sas.py:75-84 after the attention core)
//        O -> x1 = Q + O Wo^T + bo [saved], z = LN2(x1) [saved],
//             h1 = relu(drop(z W1^T + b1)) [saved], x' = (drop(h1 W2^T + b2) + z) * (ids != 0)
//
// The saved tensors, their layout and every dropout index (m*d + n per site salt) are
// exactly those of the unfused kernels, so the backward pass is shared.  Per 64-row tile
// this replaces 3 + 5 launches and 7 activation round trips through HBM with 2 launches.
//
// Tile GEMM: 4 waves split the N output columns (wave w: columns [wN/4, (w+1)N/4)), all
// 64 rows; A fragments from the LDS tile (ds_read_b128), B fragments = 16-byte rows of the
// torch [N][K] weight loaded from global/L2 for the whole K at once, MFMA 16x16x32 bf16,
// fp32 accumulate; results go through an LDS tile for coalesced 16-byte global stores.
#include "common.h"
#include "../../include/recsys_hip.h"

namespace rf {

typedef __bf16 bf16;
constexpr int BMR = 64;   // rows per workgroup

template <int D> struct Tile { static constexpr int LD = D + 8; static constexpr int ELEMS = BMR * LD; };

// global [row0, row0+64) x D  ->  LDS tile (rows >= M zero)
template <int D>
__device__ __forceinline__ void tile_load(bf16* t, const bf16* g, int64_t ldg, int64_t row0, int64_t M, int tid) {
  constexpr int CPR = D / 8, NCH = BMR * CPR, PT = NCH / 256;
  bf16x8 v[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    const int64_t gr = row0 + r < M ? row0 + r : M - 1;
    v[i] = *reinterpret_cast<const bf16x8*>(g + gr * ldg + c);
    if (row0 + r >= M) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = (bf16)0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    *reinterpret_cast<bf16x8*>(t + r * Tile<D>::LD + c) = v[i];
  }
}

template <int D>
__device__ __forceinline__ void tile_store(const bf16* t, bf16* g, int64_t ldg, int64_t row0, int64_t M, int tid) {
  constexpr int CPR = D / 8, NCH = BMR * CPR, PT = NCH / 256;
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    if (row0 + r < M) *reinterpret_cast<bf16x8*>(g + (row0 + r) * ldg + c) = *reinterpret_cast<const bf16x8*>(t + r * Tile<D>::LD + c);
  }
}

// torch.nn.LayerNorm (biased variance, eps inside the sqrt) over the 64 rows of an LDS tile
template <int D>
__device__ __forceinline__ void tile_ln(const bf16* in, bf16* out, const float* __restrict__ gamma,
                                        const float* __restrict__ beta, float eps, float* mean_g, float* rstd_g,
                                        int64_t row0, int64_t M, int tid) {
  constexpr int LPR = D / 8, RPP = 256 / LPR;   // lanes per row, rows per pass
  const int sub = tid % LPR;
  float gm[8], bt[8];
  load_chunk<float>(gm, gamma + sub * 8);
  load_chunk<float>(gm + 4, gamma + sub * 8 + 4);
  load_chunk<float>(bt, beta + sub * 8);
  load_chunk<float>(bt + 4, beta + sub * 8 + 4);
#pragma unroll
  for (int r0 = 0; r0 < BMR; r0 += RPP) {
    const int r = r0 + tid / LPR;
    float v[8];
    load_chunk<bf16>(v, in + r * Tile<D>::LD + sub * 8);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mu = s / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float u = v[j] - mu;
      q += u * u;
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rs = 1.0f / sqrtf(q / (float)D + eps);
    float y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = (v[j] - mu) * rs * gm[j] + bt[j];
    store_chunk<bf16>(out + r * Tile<D>::LD + sub * 8, y);
    if (sub == 0 && row0 + r < M) {
      mean_g[row0 + r] = mu;
      rstd_g[row0 + r] = rs;
    }
  }
}

// acc[i][j] (rows 16i + 4g + r, columns c0w + 16j + cl) += A_tile[64 x K] . W[n][k]^T
template <int K, int FN>
__device__ __forceinline__ void tile_mm(const bf16* A, int lda, const bf16* __restrict__ W, int64_t ldw, int c0w,
                                        f32x4 (&acc)[4][FN], int lane) {
  const int g = lane >> 4, cl = lane & 15;
  constexpr int KS = K / 32;
  bf16x8 b[KS][FN];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      b[ks][j] = *reinterpret_cast<const bf16x8*>(W + (int64_t)(c0w + 16 * j + cl) * ldw + 32 * ks + 8 * g);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(A + (16 * i + cl) * lda + 32 * ks + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[ks][j], acc[i][j], 0, 0, 0);
  }
}

// drop_mul (common.h) with the site seed already folded to 32 bits
__device__ __forceinline__ float drop_mul32(float p, uint32_t s32, uint64_t idx) {
  const uint32_t h = pair_hash(s32, idx);
  const uint32_t u = (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
  return u >= drop_thr(p) ? 1.0f / (1.0f - p) : 0.0f;
}

template <int FN>
__device__ __forceinline__ void acc_zero(f32x4 (&acc)[4][FN]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
}

// ------------------------------------------------------------------ block input side
struct InArgs {
  int64_t M;
  const bf16* x; int64_t ldx;
  const float* ln_w; const float* ln_b; float eps;
  bf16* Q; float* mean; float* rstd;
  const bf16* Wq; const float* bq; bf16* q;
  const bf16* Wkv; const float* bkv; bf16* kv;
};

template <int D>
__global__ __launch_bounds__(256) void sas_block_in_kernel(InArgs a) {
  constexpr int LD = Tile<D>::LD;
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * Tile<D>::ELEMS];
  bf16* X = smem;
  bf16* Qt = smem + Tile<D>::ELEMS;
  bf16* S = smem + 2 * Tile<D>::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * BMR;
  tile_load<D>(X, a.x, a.ldx, row0, a.M, tid);
  __syncthreads();
  tile_ln<D>(X, Qt, a.ln_w, a.ln_b, a.eps, a.mean, a.rstd, row0, a.M, tid);
  __syncthreads();
  tile_store<D>(Qt, a.Q, D, row0, a.M, tid);
  // q = Q Wq^T + bq     (wave w: columns [wD/4, (w+1)D/4))
  {
    constexpr int FN = D / 64;
    f32x4 acc[4][FN];
    acc_zero(acc);
    const int c0w = wave * (D / 4);
    tile_mm<D, FN>(Qt, LD, a.Wq, D, c0w, acc, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = c0w + 16 * j + cl;
      const float bb = a.bq[c];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) S[(16 * i + 4 * g + r) * LD + c] = (bf16)(acc[i][j][r] + bb);
    }
  }
  __syncthreads();
  tile_store<D>(S, a.q, D, row0, a.M, tid);
  // kv = X Wkv^T + bkv  (N = 2D: waves 0-1 produce k, waves 2-3 v)
  {
    constexpr int FN = 2 * D / 64;
    f32x4 acc[4][FN];
    acc_zero(acc);
    const int c0w = wave * (2 * D / 4);
    tile_mm<D, FN>(X, LD, a.Wkv, D, c0w, acc, lane);
    __syncthreads();   // X and S are free once every wave is past its MFMAs and the q store
    bf16* dst = wave < 2 ? S : X;
    const int cb = wave < 2 ? 0 : D;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = c0w + 16 * j + cl;
      const float bb = a.bkv[c];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(16 * i + 4 * g + r) * LD + c - cb] = (bf16)(acc[i][j][r] + bb);
    }
  }
  __syncthreads();
  tile_store<D>(S, a.kv, 2 * D, row0, a.M, tid);
  tile_store<D>(X, a.kv + D, 2 * D, row0, a.M, tid);
}

// ------------------------------------------------------------------ block output side
struct OutArgs {
  int64_t M;
  const bf16* o; const bf16* Q;
  const bf16* Wo; const float* bo; bf16* x1;
  const float* ln_w; const float* ln_b; float eps; bf16* z; float* mean; float* rstd;
  const bf16* W1; const float* b1; bf16* h1;
  const bf16* W2; const float* b2; bf16* xn;
  const int64_t* ids;
  float drop_p; uint64_t salt1, salt2; const uint64_t* seed_base;
};

template <int D>
__global__ __launch_bounds__(256) void sas_block_out_kernel(OutArgs a) {
  constexpr int LD = Tile<D>::LD, FN = D / 64;
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * Tile<D>::ELEMS];
  bf16* T0 = smem;
  bf16* T1 = smem + Tile<D>::ELEMS;
  bf16* T2 = smem + 2 * Tile<D>::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * BMR;
  const int c0w = wave * (D / 4);
  const bool drop = a.drop_p > 0.f;
  const uint32_t s1 = drop ? seed32(eff_seed(a.salt1, a.seed_base)) : 0u;
  const uint32_t s2 = drop ? seed32(eff_seed(a.salt2, a.seed_base)) : 0u;
  tile_load<D>(T0, a.o, D, row0, a.M, tid);
  tile_load<D>(T1, a.Q, D, row0, a.M, tid);
  __syncthreads();
  f32x4 acc[4][FN];
  // x1 = Q + o Wo^T + bo  -> T2
  acc_zero(acc);
  tile_mm<D, FN>(T0, LD, a.Wo, D, c0w, acc, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
    const float bb = a.bo[c];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 16 * i + 4 * g + r;
        T2[rr * LD + c] = (bf16)(acc[i][j][r] + bb + (float)T1[rr * LD + c]);
      }
  }
  __syncthreads();
  tile_store<D>(T2, a.x1, D, row0, a.M, tid);
  // z = LN2(x1) -> T0
  tile_ln<D>(T2, T0, a.ln_w, a.ln_b, a.eps, a.mean, a.rstd, row0, a.M, tid);
  __syncthreads();
  tile_store<D>(T0, a.z, D, row0, a.M, tid);
  // h1 = relu(drop(z W1^T + b1)) -> T1
  acc_zero(acc);
  tile_mm<D, FN>(T0, LD, a.W1, D, c0w, acc, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
    const float bb = a.b1[c];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 16 * i + 4 * g + r;
        float v = fmaxf(acc[i][j][r] + bb, 0.f);
        if (drop) v *= drop_mul32(a.drop_p, s1, (uint64_t)((row0 + rr) * D + c));
        T1[rr * LD + c] = (bf16)v;
      }
  }
  __syncthreads();
  tile_store<D>(T1, a.h1, D, row0, a.M, tid);
  // x' = (drop(h1 W2^T + b2) + z) * (ids != 0) -> T2
  acc_zero(acc);
  tile_mm<D, FN>(T1, LD, a.W2, D, c0w, acc, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 16 * i + 4 * g + r;
      const int64_t m = row0 + rr;
      const bool keep = m < a.M && a.ids[m < a.M ? m : 0] != 0;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = c0w + 16 * j + cl;
        const float dm = drop ? drop_mul32(a.drop_p, s2, (uint64_t)(m * D + c)) : 1.0f;
        // fma as rs_gemm's epilogue (explicit there too): one rounding of drop(v) + z
        const float v = __builtin_fmaf(acc[i][j][r] + a.b2[c], dm, (float)T0[rr * LD + c]);
        T2[rr * LD + c] = (bf16)(keep ? v : 0.f);
      }
    }
  __syncthreads();
  tile_store<D>(T2, a.xn, D, row0, a.M, tid);
}

}  // namespace rf

extern "C" {

int rs_sas_block_in(int64_t M, int64_t d, const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps,
                    void* Q, float* mean, float* rstd, const void* Wq, const float* bq, void* q, const void* Wkv,
                    const float* bkv, void* kv, void* stream) {
  if (M <= 0 || ldx % 8) return RS_ERR_ARG;
  rf::InArgs a = {M, (const __bf16*)x, ldx, ln_w, ln_b, eps, (__bf16*)Q, mean, rstd, (const __bf16*)Wq, bq,
                  (__bf16*)q, (const __bf16*)Wkv, bkv, (__bf16*)kv};
  dim3 grid((unsigned)cdiv(M, rf::BMR));
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) hipLaunchKernelGGL(rf::sas_block_in_kernel<64>, grid, dim3(256), 0, s, a);
  else if (d == 128) hipLaunchKernelGGL(rf::sas_block_in_kernel<128>, grid, dim3(256), 0, s, a);
  else return RS_ERR_UNSUPPORTED;
  return (int)hipGetLastError();
}

int rs_sas_block_out(int64_t M, int64_t d, const void* o, const void* Q, const void* Wo, const float* bo, void* x1,
                     const float* ln_w, const float* ln_b, float eps, void* z, float* mean, float* rstd,
                     const void* W1, const float* b1, void* h1, const void* W2, const float* b2, void* xn,
                     const int64_t* ids, float drop_p, uint64_t salt1, uint64_t salt2, const uint64_t* seed_base,
                     void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  rf::OutArgs a = {M, (const __bf16*)o, (const __bf16*)Q, (const __bf16*)Wo, bo, (__bf16*)x1, ln_w, ln_b, eps,
                   (__bf16*)z, mean, rstd, (const __bf16*)W1, b1, (__bf16*)h1, (const __bf16*)W2, b2, (__bf16*)xn,
                   ids, drop_p, salt1, salt2, seed_base};
  dim3 grid((unsigned)cdiv(M, rf::BMR));
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) hipLaunchKernelGGL(rf::sas_block_out_kernel<64>, grid, dim3(256), 0, s, a);
  else if (d == 128) hipLaunchKernelGGL(rf::sas_block_out_kernel<128>, grid, dim3(256), 0, s, a);
  else return RS_ERR_UNSUPPORTED;
  return (int)hipGetLastError();
}

}  // extern "C"
