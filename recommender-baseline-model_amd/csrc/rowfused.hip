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

// B fragments of a wave's output columns [c0w, c0w + 16 FN) for the whole K: rows of the torch
// [N][K] weight, 16 bytes per lane per fragment, straight from L2.  Loaded ahead of the GEMM that
// uses them (the kernels below issue the next GEMM's fragments under the current phase).
template <int K, int FN>
struct BFr {
  bf16x8 b[K / 32][FN];
  __device__ __forceinline__ void load(const bf16* __restrict__ W, int64_t ldw, int c0w, int lane) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[ks][j] = *reinterpret_cast<const bf16x8*>(W + (int64_t)(c0w + 16 * j + cl) * ldw + 32 * ks + 8 * g);
  }
};

// acc[i][j] (rows 16i + 4g + r, columns c0w + 16j + cl) += A_tile[64 x K] . W[n][k]^T
template <int K, int FN>
__device__ __forceinline__ void tile_mm_b(const bf16* A, int lda, const BFr<K, FN>& B, f32x4 (&acc)[4][FN],
                                          int lane) {
  const int g = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks) {
    bf16x8 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(A + (16 * i + cl) * lda + 32 * ks + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], B.b[ks][j], acc[i][j], 0, 0, 0);
  }
}

template <int FN>
__device__ __forceinline__ void load_bias(float (&bv)[FN], const float* __restrict__ bias, int c0w, int lane) {
#pragma unroll
  for (int j = 0; j < FN; ++j) bv[j] = bias[c0w + 16 * j + (lane & 15)];
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
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * BMR;
  constexpr int FQ = D / 64, FKV = 2 * D / 64;
  BFr<D, FQ> wq;
  float bqv[FQ];
  wq.load(a.Wq, D, wave * (D / 4), lane);
  load_bias(bqv, a.bq, wave * (D / 4), lane);
  tile_load<D>(X, a.x, a.ldx, row0, a.M, tid);
  __syncthreads();
  tile_ln<D>(X, Qt, a.ln_w, a.ln_b, a.eps, a.mean, a.rstd, row0, a.M, tid);
  __syncthreads();
  tile_store<D>(Qt, a.Q, D, row0, a.M, tid);
  BFr<D, FKV> wkv;
  float bkvv[FKV];
  // q = Q Wq^T + bq     (wave w: columns [wD/4, (w+1)D/4))
  {
    constexpr int FN = FQ;
    f32x4 acc[4][FN];
    acc_zero(acc);
    const int c0w = wave * (D / 4);
    tile_mm_b<D, FN>(Qt, LD, wq, acc, lane);
    wkv.load(a.Wkv, D, wave * (2 * D / 4), lane);     // next GEMM's weights, under this epilogue
    load_bias(bkvv, a.bkv, wave * (2 * D / 4), lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = c0w + 16 * j + cl;
      const float bb = bqv[j];
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
    tile_mm_b<D, FN>(X, LD, wkv, acc, lane);
    __syncthreads();   // X and S are free once every wave is past its MFMAs and the q store
    bf16* dst = wave < 2 ? S : X;
    const int cb = wave < 2 ? 0 : D;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = c0w + 16 * j + cl;
      const float bb = bkvv[j];
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
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * BMR;
  const int c0w = wave * (D / 4);
  const bool drop = a.drop_p > 0.f;
  const uint32_t s1 = drop ? seed32(eff_seed(a.salt1, a.seed_base)) : 0u;
  const uint32_t s2 = drop ? seed32(eff_seed(a.salt2, a.seed_base)) : 0u;
  __shared__ bool keep_s[BMR];
  // everything the block reads besides its two input tiles is requested up front: the first two
  // GEMMs' weight fragments, the biases, the timeline-mask ids
  BFr<D, FN> wo, w1, w2;
  float bov[FN], b1v[FN], b2v[FN];
  wo.load(a.Wo, D, c0w, lane);
  w1.load(a.W1, D, c0w, lane);
  load_bias(bov, a.bo, c0w, lane);
  load_bias(b1v, a.b1, c0w, lane);
  load_bias(b2v, a.b2, c0w, lane);
  if (tid < BMR) keep_s[tid] = row0 + tid < a.M && a.ids[row0 + tid < a.M ? row0 + tid : 0] != 0;
  tile_load<D>(T0, a.o, D, row0, a.M, tid);
  tile_load<D>(T1, a.Q, D, row0, a.M, tid);
  __syncthreads();
  f32x4 acc[4][FN];
  // x1 = Q + o Wo^T + bo  -> T2
  acc_zero(acc);
  tile_mm_b<D, FN>(T0, LD, wo, acc, lane);
  w2.load(a.W2, D, c0w, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
    const float bb = bov[j];
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
  tile_mm_b<D, FN>(T0, LD, w1, acc, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
    const float bb = b1v[j];
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
  tile_mm_b<D, FN>(T1, LD, w2, acc, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 16 * i + 4 * g + r;
      const int64_t m = row0 + rr;
      const bool keep = keep_s[rr];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = c0w + 16 * j + cl;
        const float dm = drop ? drop_mul32(a.drop_p, s2, (uint64_t)(m * D + c)) : 1.0f;
        // fma as rs_gemm's epilogue (explicit there too): one rounding of drop(v) + z
        const float v = __builtin_fmaf(acc[i][j][r] + b2v[j], dm, (float)T0[rr * LD + c]);
        T2[rr * LD + c] = (bf16)(keep ? v : 0.f);
      }
    }
  __syncthreads();
  tile_store<D>(T2, a.xn, D, row0, a.M, tid);
}

// ------------------------------------------------------------------ backward helpers
// LayerNorm backward over the 64 rows of LDS tiles (the arithmetic of layernorm.hip's
// ln_bwd_v_kernel, VAR 0): t = rstd*(dy*g - mean(dy*g)) - rstd^3*mean(dy*g*u)*u, u = x - mean.
// out(r, c0, t[8]) consumes each row chunk; pg/pb accumulate this lane's dgamma/dbeta columns.
template <int D, typename Out>
__device__ __forceinline__ void tile_ln_bwd(const bf16* dY, const bf16* X, const float* __restrict__ gamma,
                                            const float* __restrict__ mean, const float* __restrict__ rstd,
                                            int64_t row0, int64_t M, int tid, float (&pg)[8], float (&pb)[8], Out out) {
  constexpr int LPR = D / 8, RPP = 256 / LPR;
  const int sub = tid % LPR, c0 = sub * 8;
  float gm[8];
  load_chunk<float>(gm, gamma + c0);
  load_chunk<float>(gm + 4, gamma + c0 + 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) pg[j] = pb[j] = 0.f;
  float mu[BMR / RPP], ra[BMR / RPP];
#pragma unroll
  for (int k = 0; k < BMR / RPP; ++k) {
    const int64_t m = row0 + k * RPP + tid / LPR;
    mu[k] = mean[m < M ? m : M - 1];
    ra[k] = rstd[m < M ? m : M - 1];
  }
#pragma unroll
  for (int k = 0; k < BMR / RPP; ++k) {
    const int r = k * RPP + tid / LPR;
    const bool valid = row0 + r < M;
    float xv[8], dy[8], u[8], gq[8];
    load_chunk<bf16>(xv, X + r * Tile<D>::LD + c0);
    load_chunk<bf16>(dy, dY + r * Tile<D>::LD + c0);
    const float a = ra[k];
    float sg = 0.f, sgu = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = valid ? dy[j] : 0.f;
      u[j] = xv[j] - mu[k];
      gq[j] = g * gm[j];
      pg[j] += g * (u[j] * a);
      pb[j] += g;
      sg += gq[j];
      sgu += gq[j] * u[j];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) {
      sg += __shfl_xor(sg, o, 64);
      sgu += __shfl_xor(sgu, o, 64);
    }
    const float mg = sg / (float)D;
    const float coef = a * a * a * sgu / (float)D;
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = a * (gq[j] - mg) - coef * u[j];
    if (valid) out(r, c0, t);
  }
}

// combine the RPP row groups' dgamma/dbeta partials (fixed order) -> part[block][2][D]
template <int D>
__device__ __forceinline__ void tile_ln_partials(float* red, const float (&pg)[8], const float (&pb)[8], float* part,
                                                 int tid) {
  constexpr int LPR = D / 8, RPP = 256 / LPR;
  const int grp = tid / LPR, c0 = (tid % LPR) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[grp * D + c0 + j] = pg[j];
    red[RPP * D + grp * D + c0 + j] = pb[j];
  }
  __syncthreads();
  if (tid < 2 * D) {
    const int which = tid / D, c = tid % D;
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < RPP; ++g) t += red[which * RPP * D + g * D + c];
    part[((int64_t)blockIdx.x * 2 + which) * D + c] = t;
  }
}

// ------------------------------------------------------------------ block output side, backward
struct OutBwdArgs {
  int64_t M;
  const bf16* dxn; const int64_t* ids;
  const bf16* h1; const bf16* x1; const float* mean2; const float* rstd2; const float* ln_w;
  const bf16* W2T; const bf16* W1T; const bf16* WoT;      // transposed [in][out] copies
  bf16* dy2; bf16* da1; bf16* dx1; bf16* dout; float* part;
  float drop_p; uint64_t salt1, salt2; const uint64_t* seed_base;
};

template <int D>
__global__ __launch_bounds__(256) void sas_block_out_bwd_kernel(OutBwdArgs a) {
  constexpr int LD = Tile<D>::LD, FN = D / 64, CPR = D / 8, PT = BMR * CPR / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * Tile<D>::ELEMS];
  bf16* T0 = smem;
  bf16* T1 = smem + Tile<D>::ELEMS;
  bf16* T2 = smem + 2 * Tile<D>::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * BMR;
  const int c0w = wave * (D / 4);
  const bool drop = a.drop_p > 0.f;
  const uint32_t s1 = drop ? seed32(eff_seed(a.salt1, a.seed_base)) : 0u;
  const uint32_t s2 = drop ? seed32(eff_seed(a.salt2, a.seed_base)) : 0u;
  BFr<D, FN> w2t, w1t, wot;
  w2t.load(a.W2T, D, c0w, lane);
  w1t.load(a.W1T, D, c0w, lane);
  // 1. dzres = dxn * mask -> T0; dy2 = drop2(dzres) -> T1 (+ global); h1 -> T2
  {
    bf16x8 v[PT], hv[PT];
    bool keep[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
      const int64_t m = row0 + r < a.M ? row0 + r : a.M - 1;
      v[i] = *reinterpret_cast<const bf16x8*>(a.dxn + m * D + c);
      hv[i] = *reinterpret_cast<const bf16x8*>(a.h1 + m * D + c);
      keep[i] = row0 + r < a.M && a.ids[m] != 0;
    }
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
      const int64_t m = row0 + r;
      float x[8], y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = keep[i] ? (float)v[i][j] : 0.f;
      float dm[8];
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        if (drop) drop_mul2(a.drop_p, s2, (uint64_t)(m * D + c + j), dm[j], dm[j + 1]);
        else dm[j] = dm[j + 1] = 1.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = x[j] * dm[j];
      store_chunk<bf16>(T0 + r * LD + c, x);
      store_chunk<bf16>(T1 + r * LD + c, y);
      *reinterpret_cast<bf16x8*>(T2 + r * LD + c) = hv[i];
      if (m < a.M) store_chunk<bf16>(a.dy2 + m * D + c, y);
    }
  }
  __syncthreads();
  f32x4 acc[4][FN];
  // 2. da1 = relu'(h1) * drop1(dy2 W2) -> T2 in place of h1
  acc_zero(acc);
  tile_mm_b<D, FN>(T1, LD, w2t, acc, lane);
  wot.load(a.WoT, D, c0w, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 16 * i + 4 * g + r;
        float x = (float)T2[rr * LD + c] > 0.f ? acc[i][j][r] : 0.f;
        if (drop) x *= drop_mul32(a.drop_p, s1, (uint64_t)((row0 + rr) * D + c));
        T2[rr * LD + c] = (bf16)x;
      }
  }
  __syncthreads();
  tile_store<D>(T2, a.da1, D, row0, a.M, tid);
  // 3. dz = da1 W1 + dzres -> T0 in place; x1 -> T1
  bf16x8 xv[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    const int64_t m = row0 + r < a.M ? row0 + r : a.M - 1;
    xv[i] = *reinterpret_cast<const bf16x8*>(a.x1 + m * D + c);
  }
  acc_zero(acc);
  tile_mm_b<D, FN>(T2, LD, w1t, acc, lane);
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    *reinterpret_cast<bf16x8*>(T1 + r * LD + c) = xv[i];
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 16 * i + 4 * g + r;
        T0[rr * LD + c] = (bf16)(acc[i][j][r] + (float)T0[rr * LD + c]);
      }
  }
  __syncthreads();
  // 4. dx1 = LN2'(x1, dz) -> T2
  float pg[8], pb[8];
  tile_ln_bwd<D>(T0, T1, a.ln_w, a.mean2, a.rstd2, row0, a.M, tid, pg, pb,
                 [&](int r, int c0, const float* t) { store_chunk<bf16>(T2 + r * LD + c0, t); });
  // rows >= M of T2 are never written: zero them so the next GEMM reads defined data
  if (row0 + BMR > a.M) {
    constexpr int LPR = D / 8, RPP = 256 / LPR;
    for (int r = tid / LPR; r < BMR; r += RPP)
      if (row0 + r >= a.M) {
        float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        store_chunk<bf16>(T2 + r * LD + (tid % LPR) * 8, z);
      }
  }
  __syncthreads();
  tile_ln_partials<D>(reinterpret_cast<float*>(T0), pg, pb, a.part, tid);
  tile_store<D>(T2, a.dx1, D, row0, a.M, tid);
  // 5. dout = dx1 Wo
  acc_zero(acc);
  tile_mm_b<D, FN>(T2, LD, wot, acc, lane);
  __syncthreads();   // T0 (partials scratch) free
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) T0[(16 * i + 4 * g + r) * LD + c] = (bf16)acc[i][j][r];
  }
  __syncthreads();
  tile_store<D>(T0, a.dout, D, row0, a.M, tid);
}

// ------------------------------------------------------------------ block input side, backward
struct InBwdArgs {
  int64_t M;
  const bf16* dq; const bf16* dkv; const bf16* dx1; const bf16* x;
  const float* mean1; const float* rstd1; const float* ln_w;
  const bf16* WinT; int64_t ldwt;                       // in_proj^T [d][3d]
  bf16* dx; float* part;
};

template <int D>
__global__ __launch_bounds__(256) void sas_block_in_bwd_kernel(InBwdArgs a) {
  constexpr int LD = Tile<D>::LD, FN = D / 64, CPR = D / 8, PT = BMR * CPR / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * Tile<D>::ELEMS];
  bf16* T0 = smem;
  bf16* T1 = smem + Tile<D>::ELEMS;
  bf16* T2 = smem + 2 * Tile<D>::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4, cl = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * BMR;
  const int c0w = wave * (D / 4);
  BFr<D, FN> wk, wv, wq;
  wk.load(a.WinT + D, a.ldwt, c0w, lane);
  wv.load(a.WinT + 2 * D, a.ldwt, c0w, lane);
  // 1. dx_kv = dk Wk + dv Wv -> T2
  tile_load<D>(T0, a.dkv, 2 * D, row0, a.M, tid);
  tile_load<D>(T1, a.dkv + D, 2 * D, row0, a.M, tid);
  __syncthreads();
  bf16x8 qv[PT], rv[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    const bool ok = row0 + r < a.M;
    const int64_t m = ok ? row0 + r : a.M - 1;
    qv[i] = *reinterpret_cast<const bf16x8*>(a.dq + m * D + c);
    rv[i] = *reinterpret_cast<const bf16x8*>(a.dx1 + m * D + c);
    if (!ok) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[i][j] = (bf16)0.f;
    }
  }
  f32x4 acc[4][FN];
  acc_zero(acc);
  tile_mm_b<D, FN>(T0, LD, wk, acc, lane);
  tile_mm_b<D, FN>(T1, LD, wv, acc, lane);
  wq.load(a.WinT, a.ldwt, c0w, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) T2[(16 * i + 4 * g + r) * LD + c] = (bf16)acc[i][j][r];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    *reinterpret_cast<bf16x8*>(T0 + r * LD + c) = qv[i];
    *reinterpret_cast<bf16x8*>(T1 + r * LD + c) = rv[i];
  }
  __syncthreads();
  // 2. dQ = dq Wq + dx1 -> T1 in place; x -> T0
  bf16x8 xv[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    const int64_t m = row0 + r < a.M ? row0 + r : a.M - 1;
    xv[i] = *reinterpret_cast<const bf16x8*>(a.x + m * D + c);
  }
  acc_zero(acc);
  tile_mm_b<D, FN>(T0, LD, wq, acc, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = c0w + 16 * j + cl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 16 * i + 4 * g + r;
        T1[rr * LD + c] = (bf16)(acc[i][j][r] + (float)T1[rr * LD + c]);
      }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int ch = tid + i * 256, r = ch / CPR, c = (ch % CPR) * 8;
    *reinterpret_cast<bf16x8*>(T0 + r * LD + c) = xv[i];
  }
  __syncthreads();
  // 3. dx = dx_kv + LN1'(x, dQ)
  float pg[8], pb[8];
  tile_ln_bwd<D>(T1, T0, a.ln_w, a.mean1, a.rstd1, row0, a.M, tid, pg, pb, [&](int r, int c0, const float* t) {
    float o[8];
    load_chunk<bf16>(o, T2 + r * LD + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] += t[j];
    store_chunk<bf16>(a.dx + (row0 + r) * D + c0, o);
  });
  __syncthreads();
  tile_ln_partials<D>(reinterpret_cast<float*>(T0), pg, pb, a.part, tid);
}

// ------------------------------------------------------------------ batched bf16 transpose
// dst[m][c][r] = src[m][r][c] for the SAS block weight matrices (desc: rows, cols, src_off, lds,
// dst_off, ldd in elements); 64x64 tiles through LDS.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const int64_t* __restrict__ desc, const bf16* src,
                                                             bf16* dst) {
  __shared__ bf16 t[64][66];
  const int64_t* dsc = desc + 6 * blockIdx.y;
  const int64_t rows = dsc[0], cols = dsc[1];
  const int64_t tc = cdiv(cols, 64);
  const int64_t tr = blockIdx.x / tc, tcc = blockIdx.x % tc;
  if (tr * 64 >= rows) return;
  const bf16* s = src + dsc[2];
  bf16* d = dst + dsc[4];
  const int64_t lds = dsc[3], ldd = dsc[5];
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e / 64, c = e % 64;
    const int64_t gr = tr * 64 + r, gc = tcc * 64 + c;
    t[r][c] = (gr < rows && gc < cols) ? s[gr * lds + gc] : (bf16)0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int c = e / 64, r = e % 64;
    const int64_t gr = tr * 64 + r, gc = tcc * 64 + c;
    if (gr < rows && gc < cols) d[gc * ldd + gr] = t[r][c];
  }
}

}  // namespace rf

// 64-row-tile launchers, called by rowchain.hip's C-ABI entry points when RS_ROWCHAIN=0
int rf_sas_block_in(int64_t M, int64_t d, const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps,
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

int rf_sas_block_out(int64_t M, int64_t d, const void* o, const void* Q, const void* Wo, const float* bo, void* x1,
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

int rf_sas_block_out_bwd(int64_t M, int64_t d, const void* dxn, const int64_t* ids, const void* h1, const void* x1,
                         const float* mean2, const float* rstd2, const float* ln_w, const void* W2T, const void* W1T,
                         const void* WoT, void* dy2, void* da1, void* dx1, void* dout, float* part, float drop_p,
                         uint64_t salt1, uint64_t salt2, const uint64_t* seed_base, void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  rf::OutBwdArgs a = {M, (const __bf16*)dxn, ids, (const __bf16*)h1, (const __bf16*)x1, mean2, rstd2, ln_w,
                      (const __bf16*)W2T, (const __bf16*)W1T, (const __bf16*)WoT, (__bf16*)dy2, (__bf16*)da1,
                      (__bf16*)dx1, (__bf16*)dout, part, drop_p, salt1, salt2, seed_base};
  const int nb = (int)cdiv(M, rf::BMR);
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) hipLaunchKernelGGL(rf::sas_block_out_bwd_kernel<64>, dim3(nb), dim3(256), 0, s, a);
  else if (d == 128) hipLaunchKernelGGL(rf::sas_block_out_bwd_kernel<128>, dim3(nb), dim3(256), 0, s, a);
  else return RS_ERR_UNSUPPORTED;
  return (int)hipGetLastError();
}

int rf_sas_block_in_bwd(int64_t M, int64_t d, const void* dq, const void* dkv, const void* dx1, const void* x,
                        const float* mean1, const float* rstd1, const float* ln_w, const void* WinT, void* dx,
                        float* part, void* stream) {
  if (M <= 0) return RS_ERR_ARG;
  rf::InBwdArgs a = {M, (const __bf16*)dq, (const __bf16*)dkv, (const __bf16*)dx1, (const __bf16*)x, mean1, rstd1,
                     ln_w, (const __bf16*)WinT, 3 * d, (__bf16*)dx, part};
  const int nb = (int)cdiv(M, rf::BMR);
  hipStream_t s = (hipStream_t)stream;
  if (d == 64) hipLaunchKernelGGL(rf::sas_block_in_bwd_kernel<64>, dim3(nb), dim3(256), 0, s, a);
  else if (d == 128) hipLaunchKernelGGL(rf::sas_block_in_bwd_kernel<128>, dim3(nb), dim3(256), 0, s, a);
  else return RS_ERR_UNSUPPORTED;
  return (int)hipGetLastError();
}

extern "C" {

int rs_transpose_bf16(int64_t nmat, const int64_t* desc, int64_t max_tiles, const void* src, void* dst,
                      void* stream) {
  if (nmat <= 0 || max_tiles <= 0) return RS_ERR_ARG;
  hipLaunchKernelGGL(rf::transpose_bf16_kernel, dim3((unsigned)max_tiles, (unsigned)nmat), dim3(256), 0,
                     (hipStream_t)stream, desc, (const __bf16*)src, (__bf16*)dst);
  return (int)hipGetLastError();
}

}  // extern "C"
