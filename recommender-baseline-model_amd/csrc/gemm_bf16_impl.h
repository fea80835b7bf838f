// bf16 MFMA GEMM for the throughput path (gfx950); fp32 (parity) stays in gemm.hip.
//
// C[M,N] = epilogue( alpha * A[M,K] . B[N,K]^T ), same operand conventions, epilogue
// and split-K slab semantics as gemm.hip (GemmArgs in gemm_common.h).  What is different:
//
//  * 64-deep k stages, double-buffered LDS images, ONE barrier per stage; the next
//    stage's 16-byte global loads are issued before the current stage's MFMAs
//    (register-staged, stored into the other buffer after them);
//  * operand images keep the global orientation; fragments of k-contiguous images
//    are ds_read_b128, fragments of m/n-contiguous ("k-major") images are two
//    ds_read_b64_tr_b16 (hardware transpose), so dX = dY.W and dW = dY^T.X read
//    their transposed operands at full LDS rate;
//  * the epilogue goes through LDS: the fp32 accumulator tile is staged, then each
//    thread owns 8 consecutive columns of a row -> 16-byte loads of bias / residual /
//    pre-activation and 16-byte (bf16) or 2x16-byte (fp32) coalesced stores;
//  * wgrad (A = dY^T) sums the bias gradient with extra MFMAs against a ones operand
//    in the blocks of output column tile 0 (no separate column-sum pass).
#pragma once
#include "gemm_common.h"
#include <cstdio>
#include <cstdlib>
#include <type_traits>

typedef __attribute__((ext_vector_type(4))) __bf16 bf4;

namespace gbf {

constexpr int BKT = 64;  // k per stage

template <bool KMAJ, int ROWS>
struct Img {
  // k-contiguous: [ROWS][BKT + 8];  k-major: [BKT][ROWS + 8]   (bf16 elements)
  static constexpr int LD = KMAJ ? ROWS + 8 : BKT + 8;
  static constexpr int ELEMS = (KMAJ ? BKT : ROWS) * LD;
  static constexpr int GR = KMAJ ? BKT : ROWS;      // global rows per stage
  static constexpr int CPR = (KMAJ ? ROWS : BKT) / 8;  // 16-B chunks per global row
  static constexpr int NCH = GR * CPR;
  static constexpr int PER_T = (NCH + 255) / 256;
};

template <bool KMAJ, int ROWS>
struct Stage {
  using I = Img<KMAJ, ROWS>;
  bf16x8 r[I::PER_T];
  const __bf16* p[I::PER_T];   // interior path: per-chunk source pointers, advanced one stage at a time
  int64_t step;                // elements per 64-deep stage along k
  // interior tiles: set up the per-thread chunk pointers once (k origin c0/r0 = first stage)
  __device__ __forceinline__ void init(const __bf16* base, int64_t ld, int64_t r0, int64_t c0, int tid) {
#pragma unroll
    for (int i = 0; i < I::PER_T; ++i) {
      const int ch = min(tid + i * 256, I::NCH - 1);
      const int rr = ch / I::CPR, cc = (ch % I::CPR) * 8;
      p[i] = base + (r0 + rr) * ld + c0 + cc;
    }
    step = KMAJ ? (int64_t)BKT * ld : (int64_t)BKT;
  }
  __device__ __forceinline__ void load_next() {
#pragma unroll
    for (int i = 0; i < I::PER_T; ++i) {
      if (I::NCH % 256 == 0 || tid_ok(i)) r[i] = *reinterpret_cast<const bf16x8*>(p[i]);
      p[i] += step;
    }
  }
  int tid_;
  __device__ __forceinline__ bool tid_ok(int i) const { return tid_ + i * 256 < I::NCH; }
  // (r0, c0): global origin in storage orientation; rlim/clim: bounds.
  // Interior tiles (the block-uniform common case) take plain unconditional 16-B loads: a per-lane
  // "vector load or element-wise fallback" branch makes hipcc wait vmcnt(0) after every chunk,
  // serialising the loads of a stage.  Only edge tiles take the checked path.
  __device__ __forceinline__ void load_checked(const __bf16* base, int64_t ld, int64_t r0, int64_t c0,
                                               int64_t rlim, int64_t clim, int tid) {
#pragma unroll
    for (int i = 0; i < I::PER_T; ++i) {
      const int ch = tid + i * 256;
      if (ch < I::NCH) {
        const int rr = ch / I::CPR, cc = (ch % I::CPR) * 8;
        const int64_t gr = r0 + rr, gc = c0 + cc;
        if (gr < rlim && gc + 8 <= clim) {
          r[i] = *reinterpret_cast<const bf16x8*>(base + gr * ld + gc);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) r[i][j] = (gr < rlim && gc + j < clim) ? base[gr * ld + gc + j] : (__bf16)0.0f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(__bf16* img, int tid) const {
#pragma unroll
    for (int i = 0; i < I::PER_T; ++i) {
      const int ch = tid + i * 256;
      if (ch < I::NCH) {
        const int rr = ch / I::CPR, cc = (ch % I::CPR) * 8;
        *reinterpret_cast<bf16x8*>(img + rr * I::LD + cc) = r[i];
      }
    }
  }
};

// fragment of operand rows [row0, row0+16) for k sub-step s (32 deep) of the stage image
template <bool KMAJ, int ROWS>
__device__ __forceinline__ bf16x8 frag(const __bf16* img, int row0, int s, int lane) {
  using I = Img<KMAJ, ROWS>;
  const int g = lane >> 4, li = lane & 15;
  if (!KMAJ) return *reinterpret_cast<const bf16x8*>(img + (row0 + li) * I::LD + 32 * s + 8 * g);
  const int q = li >> 2, p = li & 3;
  const __bf16* a0 = img + (32 * s + 8 * g + q) * I::LD + row0 + 4 * p;
  const bf4 x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)a0);
  const bf4 y = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf4*)(a0 + 4 * I::LD));
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

// epilogue for 8 consecutive columns n..n+7 of row m (vector path: all 8 in range and aligned)
template <typename TC>
__device__ __forceinline__ void epi8(const GemmArgs& a, int64_t m, int64_t n, float* v, bool vec_ok) {
  const rs_epilogue& e = a.epi;
  const __bf16* aux = reinterpret_cast<const __bf16*>(e.aux);
  __bf16* aux_out = reinterpret_cast<__bf16*>(e.aux_out);
  const __bf16* res = reinterpret_cast<const __bf16*>(e.resid);
  const bool rowkeep = e.rowmask_ids ? e.rowmask_ids[m] != 0 : true;
  const uint64_t s1 = e.drop_p > 0.f ? eff_seed(e.drop_seed, e.seed_base) : 0;
  const uint64_t s2 = e.post_drop_p > 0.f ? eff_seed(e.post_drop_seed, e.seed_base) : 0;
  float bias[8], auxv[8], resv[8];
  if (vec_ok) {
    if (e.bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(e.bias + n);
      const float4 b1 = *reinterpret_cast<const float4*>(e.bias + n + 4);
      bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
      bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
    }
    if (e.act >= 3) load_chunk<__bf16>(auxv, aux + m * e.ldaux + n);
    if (res) load_chunk<__bf16>(resv, res + m * e.ldres + n);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in = n + j < a.N;
      bias[j] = (e.bias && in) ? e.bias[n + j] : 0.f;
      auxv[j] = (e.act >= 3 && in) ? (float)aux[m * e.ldaux + n + j] : 0.f;
      resv[j] = (res && in) ? (float)res[m * e.ldres + n + j] : 0.f;
    }
  }
  float pre[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = v[j] * e.alpha;
    if (e.bias) x += bias[j];
    pre[j] = x;
    if (e.act == 1) x = fmaxf(x, 0.f);
    else if (e.act == 2) x = gelu_tanh_fast(x);
    else if (e.act == 3) x = auxv[j] > 0.f ? x : 0.f;
    else if (e.act == 4) x *= gelu_tanh_grad_fast(auxv[j]);
    const float dmj = e.drop_p > 0.f ? drop_mul(e.drop_p, s1, (uint64_t)(m * e.drop_ld + n + j)) : 1.0f;
    x = res ? __builtin_fmaf(x, dmj, resv[j]) : x * dmj;
    if (!rowkeep) x = 0.f;
    if (e.post_drop_p > 0.f) x *= drop_mul(e.post_drop_p, s2, (uint64_t)(m * e.drop_ld + n + j));
    v[j] = x;
  }
  if ((e.act == 1 || e.act == 2) && aux_out) {
    if (vec_ok) store_chunk<__bf16>(aux_out + m * e.ldaux + n, pre);
    else
      for (int j = 0; j < 8; ++j)
        if (n + j < a.N) aux_out[m * e.ldaux + n + j] = (__bf16)pre[j];
  }
  TC* C = reinterpret_cast<TC*>(a.C) + m * a.ldc + n;
  if (vec_ok) {
    if (e.accumulate) {
      float old[8];
      if constexpr (sizeof(TC) == 4) {
        load_chunk<float>(old, reinterpret_cast<const float*>(C));
        load_chunk<float>(old + 4, reinterpret_cast<const float*>(C) + 4);
      } else {
        load_chunk<__bf16>(old, reinterpret_cast<const __bf16*>(C));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += old[j];
    }
    if constexpr (sizeof(TC) == 4) {
      store_chunk<float>(reinterpret_cast<float*>(C), v);
      store_chunk<float>(reinterpret_cast<float*>(C) + 4, v + 4);
    } else {
      store_chunk<__bf16>(reinterpret_cast<__bf16*>(C), v);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (n + j < a.N) {
        float x = v[j];
        if (e.accumulate) x += (float)C[j];
        C[j] = (TC)x;
      }
  }
}

// ---- compile-time epilogue classes: the runtime-flag epilogue (epi8) made hipcc spill SGPRs
// into VGPR lanes and roughly tripled the per-wave instruction count of these short GEMMs
enum : int { EB = 1, ED = 2, ER = 4, EM = 8, EP = 16, EA = 32, EF = 64 };  // bias drop resid rowmask post acc f32C
constexpr int EC_GENERIC = -1, EC_SLAB = -2, EC_CE_PART = -3, EC_CE_GRAD = -4;
constexpr int ec_act(int ec) { return (ec >> 8) & 7; }

template <int EC>
__device__ __forceinline__ void epi8_t(const GemmArgs& a, int64_t m, int64_t n, float* v, uint32_t s1, uint32_t s2) {
  constexpr int ACT = ec_act(EC);
  const rs_epilogue& e = a.epi;
  float bias[8], auxv[8], resv[8];
  if constexpr ((EC & EB) != 0) {
    load_chunk<float>(bias, e.bias + n);
    load_chunk<float>(bias + 4, e.bias + n + 4);
  }
  if constexpr (ACT >= 3) load_chunk<__bf16>(auxv, reinterpret_cast<const __bf16*>(e.aux) + m * e.ldaux + n);
  if constexpr ((EC & ER) != 0) load_chunk<__bf16>(resv, reinterpret_cast<const __bf16*>(e.resid) + m * e.ldres + n);
  bool keep = true;
  if constexpr ((EC & EM) != 0) keep = e.rowmask_ids[m] != 0;
  float dm[8], pm[8];
  if constexpr ((EC & ED) != 0) {
    const uint64_t base = (uint64_t)(m * e.drop_ld + n);
#pragma unroll
    for (int j = 0; j < 8; j += 2) drop_mul2(e.drop_p, s1, base + j, dm[j], dm[j + 1]);
  }
  if constexpr ((EC & EP) != 0) {
    const uint64_t base = (uint64_t)(m * e.drop_ld + n);
#pragma unroll
    for (int j = 0; j < 8; j += 2) drop_mul2(e.post_drop_p, s2, base + j, pm[j], pm[j + 1]);
  }
  float pre[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = v[j];
    if constexpr ((EC & EB) != 0) x += bias[j];
    pre[j] = x;
    if constexpr (ACT == 1) x = fmaxf(x, 0.f);
    if constexpr (ACT == 2) x = gelu_tanh_fast(x);
    if constexpr (ACT == 3) x = auxv[j] > 0.f ? x : 0.f;
    if constexpr (ACT == 4) x *= gelu_tanh_grad_fast(auxv[j]);
    if constexpr ((EC & ED) != 0 && (EC & ER) != 0) x = __builtin_fmaf(x, dm[j], resv[j]);  // one rounding
    else if constexpr ((EC & ED) != 0) x *= dm[j];
    else if constexpr ((EC & ER) != 0) x += resv[j];
    if constexpr ((EC & EM) != 0) x = keep ? x : 0.f;
    if constexpr ((EC & EP) != 0) x *= pm[j];
    v[j] = x;
  }
  if constexpr (ACT == 1 || ACT == 2) {
    if (e.aux_out) store_chunk<__bf16>(reinterpret_cast<__bf16*>(e.aux_out) + m * e.ldaux + n, pre);
  }
  if constexpr ((EC & EF) != 0) {
    float* C = reinterpret_cast<float*>(a.C) + m * a.ldc + n;
    if constexpr ((EC & EA) != 0) {
      float old[8];
      load_chunk<float>(old, C);
      load_chunk<float>(old + 4, C + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += old[j];
    }
    store_chunk<float>(C, v);
    store_chunk<float>(C + 4, v + 4);
  } else {
    __bf16* C = reinterpret_cast<__bf16*>(a.C) + m * a.ldc + n;
    if constexpr ((EC & EA) != 0) {
      float old[8];
      load_chunk<__bf16>(old, C);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += old[j];
    }
    store_chunk<__bf16>(C, v);
  }
}

__device__ __forceinline__ void bf8_to_f(const bf16x8& x, float* o) {
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)x[j];
}

// Whole-tile epilogue of a compile-time class, columns n..n+7 in range: every global operand of the
// thread's NP rows (pre-activation, residual, row-mask id, old C) is loaded before any row is
// finished, so the tile pays one memory round trip instead of one per row.
template <int EC, int NP, int RPP, int LDC>
__device__ __forceinline__ void epi_rows(const GemmArgs& a, const float* Cs, int row0, int c8, int64_t m0, int64_t Mb,
                                         int64_t n, uint32_t s1, uint32_t s2) {
  constexpr int ACT = ec_act(EC);
  const rs_epilogue& e = a.epi;
  float bias[8];
  if constexpr ((EC & EB) != 0) {
    load_chunk<float>(bias, e.bias + n);
    load_chunk<float>(bias + 4, e.bias + n + 4);
  }
  bf16x8 auxr[NP], resr[NP], oldr[NP];
  int64_t idr[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int64_t m = m0 + row0 + p * RPP;
    if (m < Mb) {
      if constexpr (ACT >= 3) auxr[p] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(e.aux) + m * e.ldaux + n);
      if constexpr ((EC & ER) != 0) resr[p] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(e.resid) + m * e.ldres + n);
      if constexpr ((EC & EM) != 0) idr[p] = e.rowmask_ids[m];
      if constexpr ((EC & EA) != 0 && (EC & EF) == 0) oldr[p] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(a.C) + m * a.ldc + n);
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int row = row0 + p * RPP;
    const int64_t m = m0 + row;
    if (m >= Mb) break;
    float v[8];
    {
      const float4 v0 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8 + 4);
      v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    }
    float auxv[8], resv[8], dm[8], pm[8];
    if constexpr (ACT >= 3) bf8_to_f(auxr[p], auxv);
    if constexpr ((EC & ER) != 0) bf8_to_f(resr[p], resv);
    if constexpr ((EC & ED) != 0) {
      const uint64_t base = (uint64_t)(m * e.drop_ld + n);
#pragma unroll
      for (int j = 0; j < 8; j += 2) drop_mul2(e.drop_p, s1, base + j, dm[j], dm[j + 1]);
    }
    if constexpr ((EC & EP) != 0) {
      const uint64_t base = (uint64_t)(m * e.drop_ld + n);
#pragma unroll
      for (int j = 0; j < 8; j += 2) drop_mul2(e.post_drop_p, s2, base + j, pm[j], pm[j + 1]);
    }
    bool keep = true;
    if constexpr ((EC & EM) != 0) keep = idr[p] != 0;
    float pre[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = v[j];
      if constexpr ((EC & EB) != 0) x += bias[j];
      pre[j] = x;
      if constexpr (ACT == 1) x = fmaxf(x, 0.f);
      if constexpr (ACT == 2) x = gelu_tanh_fast(x);
      if constexpr (ACT == 3) x = auxv[j] > 0.f ? x : 0.f;
      if constexpr (ACT == 4) x *= gelu_tanh_grad_fast(auxv[j]);
      if constexpr ((EC & ED) != 0 && (EC & ER) != 0) x = __builtin_fmaf(x, dm[j], resv[j]);  // one rounding
      else if constexpr ((EC & ED) != 0) x *= dm[j];
      else if constexpr ((EC & ER) != 0) x += resv[j];
      if constexpr ((EC & EM) != 0) x = keep ? x : 0.f;
      if constexpr ((EC & EP) != 0) x *= pm[j];
      v[j] = x;
    }
    if constexpr (ACT == 1 || ACT == 2) {
      if (e.aux_out) store_chunk<__bf16>(reinterpret_cast<__bf16*>(e.aux_out) + m * e.ldaux + n, pre);
    }
    if constexpr ((EC & EF) != 0) {
      float* C = reinterpret_cast<float*>(a.C) + m * a.ldc + n;
      if constexpr ((EC & EA) != 0) {
        float old[8];
        load_chunk<float>(old, C);
        load_chunk<float>(old + 4, C + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += old[j];
      }
      store_chunk<float>(C, v);
      store_chunk<float>(C + 4, v + 4);
    } else {
      if constexpr ((EC & EA) != 0) {
        float old[8];
        bf8_to_f(oldr[p], old);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += old[j];
      }
      store_chunk<__bf16>(reinterpret_cast<__bf16*>(a.C) + m * a.ldc + n, v);
    }
  }
}

// Vocabulary cross-entropy epilogues (vocab_ce.hip).  Columns n..n+7 of rows row0 + p*RPP (the 16
// threads of a row hold its 128 columns; columns >= N are masked).
//  EC_CE_PART: per (row, column tile) the online-softmax pair (max, sum exp(x - max)) of the
//              tile's logits x = acc + bias, and the label's logit when it falls in the tile;
//  EC_CE_GRAD: dlogits = (exp(x - lse[row]) - [col == label]) * dloss / count as bf16 (ce_bwd_kernel's
//              arithmetic, loss.hip), so the fp32 logits are never written.
template <int EC, int NP, int RPP, int LDC, int TPR>
__device__ __forceinline__ void ce_rows(const GemmArgs& a, const float* Cs, int row0, int c8, int64_t m0, int64_t Mb,
                                        int64_t n, unsigned tn) {
  float bias[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = (a.epi.bias && n + j < a.N) ? a.epi.bias[n + j] : 0.f;
  int64_t lab[NP];
  float lse[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int64_t m = m0 + row0 + p * RPP;
    lab[p] = m < Mb ? a.ce.labels[m] : 0;
    if constexpr (EC == EC_CE_GRAD) lse[p] = m < Mb ? a.ce.lse[m] : 0.f;
  }
  float sc = 0.f;
  if constexpr (EC == EC_CE_GRAD) sc = (a.ce.dloss ? *a.ce.dloss : 1.f) / *a.ce.count;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int row = row0 + p * RPP;
    const int64_t m = m0 + row;
    if (m >= Mb) break;     // uniform over the TPR threads of a row
    float v[8];
    {
      const float4 v0 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8 + 4);
      v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += bias[j];
    if constexpr (EC == EC_CE_PART) {
      float mx = -__builtin_inff(), sm = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (n + j < a.N) mx = fmaxf(mx, v[j]);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (n + j < a.N) sm += __expf(v[j] - mx);
#pragma unroll
      for (int o = TPR / 2; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(mx, o, TPR), s2 = __shfl_xor(sm, o, TPR);
        const float mm = fmaxf(mx, m2);
        sm = (mm == -__builtin_inff()) ? 0.f : sm * __expf(mx - mm) + s2 * __expf(m2 - mm);
        mx = mm;
      }
      if (c8 == 0) {
        a.ce.part[(m * a.ce.ntn + tn) * 2 + 0] = mx;
        a.ce.part[(m * a.ce.ntn + tn) * 2 + 1] = sm;
      }
      const int64_t l = lab[p];
      if (l >= n && l < n + 8 && l < a.N) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (l == n + j) a.ce.tgt[m] = v[j];
      }
    } else {
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        g[j] = lab[p] != 0 ? (__expf(v[j] - lse[p]) - (n + j == lab[p] ? 1.f : 0.f)) * sc : 0.f;
      __bf16* C = reinterpret_cast<__bf16*>(a.C) + m * a.ldc + n;
      if (n + 8 <= a.N) {
        store_chunk<__bf16>(C, g);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (n + j < a.N) C[j] = (__bf16)g[j];
      }
    }
  }
}

template <bool AK, bool BK, int BM, int BN, int EC>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmArgs a) {
  KStampBegin stamp_b_(a.ks);
  KStampEnd stamp_e_(a.ks);
  using IA = Img<AK, BM>;
  using IB = Img<BK, BN>;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  constexpr int LDC = BN + 4;
  constexpr int LDS_BYTES = (2 * STAGE * 2 > BM * LDC * 4) ? 2 * STAGE * 2 : BM * LDC * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  __bf16* stage0 = reinterpret_cast<__bf16*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int FM = BM / 32, FN = BN / 32;

  // block -> tile (32-bit: every block index fits); XCD-aware: blocks b and b+8 share an XCD, so
  // consecutive tiles (which share A rows / B columns) go to one XCD's L2
  const unsigned tiles_n = (unsigned)((a.N + BN - 1) / BN);
  const int64_t Mb = (!AK && a.epi.rows_dev) ? min(a.M, (int64_t)*a.epi.rows_dev) : a.M;
  unsigned bid = blockIdx.x;
  unsigned tiles_m = gridDim.x / tiles_n;
  int z = blockIdx.z;
  if (gridDim.z > 1) {
    // split-K: the tiles of one k slice share its B columns (the vocabulary GEMM dh = dlogits.E: a 16k-row
    // slice of the 512 MB weight per split), so deal whole k slices to XCDs -- workgroups are dispatched
    // x-fastest then z, round robin over the 8 XCDs -- instead of every XCD fetching every slice (cfg5:
    // 1.32 -> 1.30 ms; the MALL serves most of the re-reads)
    const unsigned tot = gridDim.x * gridDim.z, L = blockIdx.x + gridDim.x * blockIdx.z;
    const unsigned q = tot >> 3, r = tot & 7, x = L & 7;
    const unsigned lg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
    z = (int)(lg / gridDim.x);
    bid = lg - (unsigned)z * gridDim.x;
    if (!AK && a.epi.rows_dev) {
      tiles_m = (unsigned)((Mb + BM - 1) / BM);
      if (bid >= tiles_m * tiles_n) return;
    }
  } else {
    // a device row count (compacted rows) leaves only the first cdiv(Mb, BM) row tiles live: remap over
    // those, so the live tiles spread over all XCDs instead of the first few XCDs' contiguous ranges
    unsigned nwg = gridDim.x;
    if (!AK && a.epi.rows_dev) {
      tiles_m = (unsigned)((Mb + BM - 1) / BM);
      nwg = tiles_m * tiles_n;
      if (bid >= nwg) return;
    }
    const unsigned q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  // walk the shorter tile axis fastest: an XCD's contiguous range of tiles then shares the tiles of
  // the LONG axis's operand in its L2, and that operand streams from HBM once (the 1M-column vocabulary
  // GEMMs: 14 row tiles x 7.8k column tiles; row-major order re-read the 512 MB weight 14 times)
  unsigned tm, tn;
  if (tiles_m < tiles_n) {
    tn = bid / tiles_m;
    tm = bid - tn * tiles_m;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t Kb = (AK && a.epi.rows_dev) ? min(a.K, (int64_t)*a.epi.rows_dev) : a.K;
  if (m0 >= Mb) return;
  const int64_t kbeg = (int64_t)z * a.k_per_split;
  const int64_t kend = min(Kb, kbeg + a.k_per_split);
  const int nk = kend > kbeg ? (int)((kend - kbeg + BKT - 1) / BKT) : 0;

  const __bf16* A = reinterpret_cast<const __bf16*>(a.A);
  const __bf16* B = reinterpret_cast<const __bf16*>(a.B);
  const bool do_colsum = AK && a.bias_colsum && tn == 0 && wn == 0;

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

  Stage<AK, BM> sa;
  Stage<BK, BN> sb;
  sa.tid_ = tid;
  sb.tid_ = tid;
  // Two instantiations of the k loop: interior blocks (whole BM x BN tile and whole 64-deep stages
  // in bounds: unconditional loads through per-thread pointers set up once, so the next stage's
  // loads stay in flight under the MFMAs) and edge blocks (checked loads).  Mixing both in one loop
  // made hipcc wait vmcnt(0) before the MFMAs.
  const bool interior = (m0 + BM <= (AK ? a.M : Mb)) && (n0 + BN <= a.N) && ((kend - kbeg) % BKT == 0);
  auto kloop = [&](auto edge_tag) {
    constexpr bool EDGE = decltype(edge_tag)::value;
    auto issue = [&](int64_t k0) {
      if (!EDGE) {
        sa.load_next();
        sb.load_next();
        return;
      }
      if (!AK) sa.load_checked(A, a.lda, m0, k0, Mb, kend, tid);
      else sa.load_checked(A, a.lda, k0, m0, kend, a.M, tid);
      if (!BK) sb.load_checked(B, a.ldb, n0, k0, a.N, kend, tid);
      else sb.load_checked(B, a.ldb, k0, n0, kend, a.N, tid);
    };
    if (!EDGE) {
      if (!AK) sa.init(A, a.lda, m0, kbeg, tid);
      else sa.init(A, a.lda, kbeg, m0, tid);
      if (!BK) sb.init(B, a.ldb, n0, kbeg, tid);
      else sb.init(B, a.ldb, kbeg, n0, tid);
    }
    issue(kbeg);
    sa.store(stage0, tid);
    sb.store(stage0 + IA::ELEMS, tid);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const __bf16* cur = stage0 + (kt & 1) * STAGE;
      const bool more = kt + 1 < nk;
      if (more) issue(kbeg + (int64_t)(kt + 1) * BKT);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = frag<AK, BM>(cur, wm * (BM / 2) + 16 * i, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = frag<BK, BN>(cur + IA::ELEMS, wn * (BN / 2) + 16 * j, s, lane);
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
      if (more) {
        __bf16* nxt = stage0 + ((kt + 1) & 1) * STAGE;
        sa.store(nxt, tid);
        sb.store(nxt + IA::ELEMS, tid);
      }
      __syncthreads();
    }
  };
  if (nk > 0) {
    if (interior) kloop(std::integral_constant<bool, false>{});
    else kloop(std::integral_constant<bool, true>{});
  }

  // ---- epilogue through LDS
  float* Cs = reinterpret_cast<float*>(smem);
  __syncthreads();
  {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(wm * (BM / 2) + 16 * i + 4 * g + r) * LDC + wn * (BN / 2) + 16 * j + cl] = acc[i][j][r];
    if (do_colsum && cl == 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t m = m0 + wm * (BM / 2) + 16 * i + 4 * g + r;
          if (m < a.M) {
            if (a.colsum_out) a.colsum_out[m] = (a.epi.accumulate ? a.colsum_out[m] : 0.f) + accb[i][r];
            else a.slab[(int64_t)z * a.slab_stride + a.M * a.N + m] = accb[i][r];
          }
        }
    }
  }
  __syncthreads();
  constexpr int TPR = BN / 8;         // threads per row
  constexpr int RPP = 256 / TPR;      // rows per pass
  const int c8 = (tid % TPR) * 8;
  const int64_t n = n0 + c8;
  if constexpr (EC == EC_CE_PART || EC == EC_CE_GRAD) {
    ce_rows<EC, BM / RPP, RPP, LDC, TPR>(a, Cs, tid / TPR, c8, m0, Mb, n, tn);
    return;
  }
  if (n >= a.N) return;
  uint32_t s1 = 0, s2 = 0;
  if constexpr (EC >= 0) {
    if constexpr ((EC & ED) != 0) s1 = seed32(eff_seed(a.epi.drop_seed, a.epi.seed_base));
    if constexpr ((EC & EP) != 0) s2 = seed32(eff_seed(a.epi.post_drop_seed, a.epi.seed_base));
    if (n + 8 <= a.N) {
      epi_rows<EC, BM / RPP, RPP, LDC>(a, Cs, tid / TPR, c8, m0, Mb, n, s1, s2);
      return;
    }
  }
  for (int row = tid / TPR; row < BM; row += RPP) {
    const int64_t m = m0 + row;
    if (m >= Mb) break;
    float v[8];
    const float4 v0 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8);
    const float4 v1 = *reinterpret_cast<const float4*>(Cs + row * LDC + c8 + 4);
    v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    if constexpr (EC == EC_SLAB) {
      float* S = a.slab + ((int64_t)z * a.slab_stride + m * a.N + n);
      if (n + 8 <= a.N && (a.N % 4) == 0) {
        *reinterpret_cast<float4*>(S) = v0;
        *reinterpret_cast<float4*>(S + 4) = v1;
      } else {
        for (int j = 0; j < 8; ++j)
          if (n + j < a.N) S[j] = v[j];
      }
      continue;
    }
    if constexpr (EC >= 0) {
      if (n + 8 <= a.N) {
        epi8_t<EC>(a, m, n, v, s1, s2);
        continue;
      }
    }
    if constexpr (EC != EC_SLAB) {
      const bool vec_ok = (n + 8 <= a.N) && a.vec_ok;
      if (a.c_f32) epi8<float>(a, m, n, v, vec_ok);
      else epi8<__bf16>(a, m, n, v, vec_ok);
    }
  }
}

template <bool AK, bool BK, int BM, int BN, int EC>
hipError_t launch_cfg(GemmArgs& a, hipStream_t s) {
  dim3 grid((unsigned)(cdiv(a.M, BM) * cdiv(a.N, BN)), 1, a.split_k);
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BK, BM, BN, EC>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// tile choice: 128x128 when that still gives >= 512 workgroups (2 per CU), else 64x64; the GELU /
// GELU' + dropout epilogues (BERT FFN1 forward, FFN2 input gradient) always take 64x64: their VALU work
// (tanh, the dropout hash) then overlaps the loads of the other resident workgroups (12800 x 1024 x 256:
// 25.9 -> 24.3 us and 27.6 -> 25.6 us, tools/diag/gemm_epi.py)
#include "gemm_dma.h"

template <bool AK, bool BK, int EC>
hipError_t launch_tiles(GemmArgs& a, hipStream_t s) {
  if constexpr (!AK && EC >= 0) {
    const hipError_t e = dma::launch<BK, EC>(a, s);
    if (e != hipErrorNotSupported) return e;
  }
  constexpr bool heavy_epi = EC >= 0 && (ec_act(EC) == 2 || ec_act(EC) == 4) && (EC & ED) != 0;
  if (!heavy_epi && cdiv(a.M, 128) * cdiv(a.N, 128) * a.split_k >= 512) return launch_cfg<AK, BK, 128, 128, EC>(a, s);
#ifdef GBF_MID_MIN
  if (!heavy_epi && a.N >= 128 && cdiv(a.M, 64) * cdiv(a.N, 128) * a.split_k >= GBF_MID_MIN)
    return launch_cfg<AK, BK, 64, 128, EC>(a, s);
#endif
  return launch_cfg<AK, BK, 64, 64, EC>(a, s);
}

// the epilogue classes of the hot path (SAS / BERT forward and input-gradient GEMMs)
#define GBF_EC_LIST(X)                                                                                     \
  X(0) X(EB) X(EB | ER) X(EB | ED | (1 << 8)) X(EB | (1 << 8)) X(EB | ED | ER | EM) X(EB | ER | EM)        \
  X(EB | ED | (2 << 8)) X(EB | (2 << 8)) X(EB | ED | ER) X(EB | ED | ER | EP) X(EF | EB) X(ER)              \
  X(ED | (3 << 8)) X((3 << 8)) X(ED | (4 << 8)) X((4 << 8)) X(EA)

int epi_class(const GemmArgs& a);

template <bool AK, bool BK>
hipError_t launch_classes(GemmArgs& a, hipStream_t s) {
  const int ec = epi_class(a);
#define GBF_CASE(E) case (E): return launch_tiles<AK, BK, (E)>(a, s);
  switch (ec) {
    GBF_EC_LIST(GBF_CASE)
    default: break;
  }
#undef GBF_CASE
  return launch_tiles<AK, BK, EC_GENERIC>(a, s);
}

}  // namespace gbf
