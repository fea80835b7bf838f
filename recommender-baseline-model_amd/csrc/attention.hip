// Fused masked scaled-dot-product attention, forward + backward (gfx950).
//
// Replaces the attention core of
//   SAS : torch F.multi_head_attention_forward (need_weights=True path) called at
//         BS/models/sas_model/sas.py:75 -- q*1/sqrt(Dh), baddbmm(causal -inf mask, q, k^T),
//         softmax, dropout(P), bmm(P, v)
//   BERT: BS/models/bert_modules/attention/single.py:13-35 -- q.k^T/sqrt(Dh),
//         masked_fill(key padding, -1e9), softmax, dropout(P), P.v
//
// These are the generic kernels: fp32 (the parity mode) and any bf16 shape the LDS-resident kernels
// (attention_lds.hip: bf16, T <= 256, Dh in {32, 64, 128}) do not take -- any head dim Dh <= 256 (the
// reference's default SAS width is d = 50 with one head) and any sequence length T (`--max_len 300` ...).
//
// Layout: token-major rows (row = b*T + t), head h in columns [h*Dh, (h+1)*Dh) of q/k/v/o (any leading
// dimension; rows that are not 16-byte aligned are read element by element).  The head dim is padded to
// DHP in {32, 64, 128, 256} inside the kernel (zero fragments; the padding contributes nothing to q.k or
// P.v and is never stored).  One 64-lane wave per workgroup owns 16 query rows (forward, dQ) or 16 key rows
// (dK/dV) and walks the other axis in 32-wide chunks: the forward with an online softmax (running row max
// and sum, O rescaled per chunk), the backward recomputing P from the saved row logsumexp.  Dropout masks
// are regenerated from the counter-based RNG with index ((b*H + h)*T + query)*Tp + key, Tp = T rounded up
// to even (every mask row starts on a hash pair, so the paired-hash kernels of attention_lds.hip draw the
// same masks for odd T).
#include "common.h"
#include "../../include/recsys_hip.h"

struct AttnArgs {
  int64_t B, T, H;
  int Dh;          // real head dim (<= the kernel's DHP)
  int vec;         // every operand row 16-byte aligned and ld a multiple of the vector width
  const void* q; int64_t ldq;
  const void* k; int64_t ldk;
  const void* v; int64_t ldv;
  void* o; int64_t ldo;
  const void* dout; int64_t lddo;
  void* dq; int64_t lddq;
  void* dk; int64_t lddk;
  void* dv; int64_t lddv;
  float* lse;
  const float* lse_in;
  float* delta;
  float scale;
  int mask_kind;  // 0 causal (-inf), 1 key padding (-1e9)
  const int64_t* ids;
  float drop_p;
  uint64_t seed;
  const uint64_t* seed_base;
};

#define NEG_INF (-__builtin_inff())

__device__ __forceinline__ int64_t mask_pitch(int64_t T) { return T + (T & 1); }

// masked, scaled score for (query row, key) -- exactly the reference's masking
__device__ __forceinline__ float masked_score(const AttnArgs& a, int64_t b, int64_t qrow, int64_t key, float s) {
  if (key >= a.T) return NEG_INF;                                   // beyond the sequence: not a key
  if (a.mask_kind == 0) return key > qrow ? NEG_INF : s;            // causal (sas.py:70)
  return a.ids[b * a.T + key] == 0 ? -1e9f : s;                     // key padding (single.py:28)
}

// 8 elements of row `row`, columns [col, col+8) (zero past rlim rows / dh columns)
// exp / log of the generic kernels: the fp32 (parity) instantiations use the accurate libm forms, as the reference's
// torch softmax does (the fast forms' argument rounding -- exp2(x * log2 e) -- adds noise that a 1000-step training
// curve amplifies); bf16 keeps the fast hardware forms
template <typename T> __device__ __forceinline__ float aexp(float x) { return __expf(x); }
template <> __device__ __forceinline__ float aexp<float>(float x) { return expf(x); }
template <typename T> __device__ __forceinline__ float alog(float x) { return __logf(x); }
template <> __device__ __forceinline__ float alog<float>(float x) { return logf(x); }

template <typename T>
__device__ __forceinline__ void load_frag_rows(Frag<T>& f, const T* base, int64_t ld, int64_t row, int64_t rlim,
                                               int col, int dh, int vec) {
  if (row < rlim && vec && col + 8 <= dh) {
    frag_load_vec(f, base + row * ld + col);
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) frag_set(f, j, (row < rlim && col + j < dh) ? to_f(base[row * ld + col + j]) : 0.0f);
}

// stage a 32-row x DHP chunk (rows r0.., row-major in global) transposed into LDS: dst[dim][row] (ld = 32+PADT)
template <typename T, int DHP>
__device__ __forceinline__ void stage_transposed(T* dst, int ldd, const T* src, int64_t ld, int64_t r0,
                                                 int64_t rlim, int lane, int dh, int vec) {
  constexpr int V = Vec<T>::N;
  constexpr int CPR = DHP / V;          // chunks per row
  constexpr int NCH = 32 * CPR;
#pragma unroll
  for (int i = 0; i < NCH / 64; ++i) {
    int ch = lane + i * 64;
    int r = ch / CPR, c = (ch % CPR) * V;
    float buf[V];
    if (r0 + r < rlim && vec && c + V <= dh) load_chunk<T>(buf, src + (r0 + r) * ld + c);
    else {
#pragma unroll
      for (int j = 0; j < V; ++j) buf[j] = (r0 + r < rlim && c + j < dh) ? to_f(src[(r0 + r) * ld + c + j]) : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < V; ++j) dst[(c + j) * ldd + r] = from_f<T>(buf[j]);
  }
}

// ------------------------------------------------------------------ forward (online softmax over 32-key chunks)
template <typename T, int DHP>
__global__ __launch_bounds__(64) void attn_fwd_kernel(AttnArgs a) {
  constexpr int PLD = 32 + Vec<T>::N;            // P chunk row stride in LDS
  constexpr int VLD = 32 + Vec<T>::N;            // V^T chunk row stride
  __shared__ __attribute__((aligned(16))) T Ps[16 * PLD];
  __shared__ __attribute__((aligned(16))) T Vt[DHP * VLD];

  const int lane = threadIdx.x;
  const int64_t bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int64_t q0 = (int64_t)blockIdx.x * 16;
  const uint64_t seed = eff_seed(a.seed, a.seed_base);
  const int64_t Dh = a.Dh, tp = mask_pitch(a.T);
  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.T * a.ldq + h * Dh;
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.T * a.ldk + h * Dh;
  const T* Vp = reinterpret_cast<const T*>(a.v) + b * a.T * a.ldv + h * Dh;
  const int g = lane >> 4, cl = lane & 15;

  // keys this wave can see
  const int64_t kend = a.mask_kind == 0 ? min(a.T, q0 + 16) : a.T;
  const int nkc = (int)((kend + 31) / 32);

  Frag<T> qf[DHP / 32];
#pragma unroll
  for (int kk = 0; kk < DHP / 32; ++kk) load_frag_rows(qf[kk], Q, a.ldq, q0 + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);

  float mx[4], sm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mx[r] = NEG_INF; sm[r] = 0.f; }
  f32x4 o[DHP / 16];
#pragma unroll
  for (int nt = 0; nt < DHP / 16; ++nt) o[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < nkc; ++kc) {
    f32x4 s[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      s[hf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < DHP / 32; ++kk) {
        Frag<T> kf;
        load_frag_rows(kf, K, a.ldk, (int64_t)kc * 32 + hf * 16 + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
        s[hf] = mma(qf[kk], kf, s[hf]);
      }
    }
    // mask + scale, chunk row max, rescale the running state
    float cm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t qrow = q0 + 4 * g + r;
      cm[r] = NEG_INF;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int64_t key = (int64_t)kc * 32 + hf * 16 + cl;
        const float x = masked_score(a, b, qrow, key, s[hf][r] * a.scale);
        s[hf][r] = x;
        cm[r] = fmaxf(cm[r], x);
      }
      cm[r] = group16_max(cm[r]);
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float nm = fmaxf(mx[r], cm[r]);
      alpha[r] = (mx[r] == NEG_INF) ? 0.f : aexp<T>(mx[r] - nm);
      mx[r] = nm;
      float rs = 0.f;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float e = (s[hf][r] == NEG_INF || nm == NEG_INF) ? 0.0f : aexp<T>(s[hf][r] - nm);
        s[hf][r] = e;
        rs += e;
      }
      sm[r] = sm[r] * alpha[r] + group16_sum(rs);
    }
#pragma unroll
    for (int nt = 0; nt < DHP / 16; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[nt][r] *= alpha[r];
    // P (unnormalised, + dropout) -> LDS [row][key]; V^T chunk -> LDS; O += P.V
    __syncthreads();
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t qrow = q0 + 4 * g + r, key = (int64_t)kc * 32 + hf * 16 + cl;
        float p = s[hf][r];
        if (a.drop_p > 0.f) p *= drop_mul(a.drop_p, seed, (uint64_t)((bh * a.T + qrow) * tp + key));
        Ps[(4 * g + r) * PLD + hf * 16 + cl] = from_f<T>(p);
      }
    stage_transposed<T, DHP>(Vt, VLD, Vp, a.ldv, (int64_t)kc * 32, a.T, lane, a.Dh, a.vec);
    __syncthreads();
    Frag<T> pa;
    frag_load_vec(pa, Ps + cl * PLD + 8 * g);
#pragma unroll
    for (int nt = 0; nt < DHP / 16; ++nt) {
      Frag<T> vb;
      frag_load_vec(vb, Vt + (nt * 16 + cl) * VLD + 8 * g);
      o[nt] = mma(pa, vb, o[nt]);
    }
  }
  if (cl == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t qrow = q0 + 4 * g + r;
      if (qrow < a.T) a.lse[bh * a.T + qrow] = mx[r] + alog<T>(sm[r]);
    }
  }
  T* O = reinterpret_cast<T*>(a.o) + b * a.T * a.ldo + h * Dh;
  float inv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) inv[r] = sm[r] > 0.f ? 1.0f / sm[r] : 0.f;
#pragma unroll
  for (int nt = 0; nt < DHP / 16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t qrow = q0 + 4 * g + r;
      const int col = nt * 16 + cl;
      if (qrow < a.T && col < a.Dh) O[qrow * a.ldo + col] = from_f<T>(o[nt][r] * inv[r]);
    }
}

// ------------------------------------------------------------------ backward: delta = rowsum(dO * O)
template <typename T>
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnArgs a) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // over B*T*H (bh-major)
  const int lane = threadIdx.x & 63;
  if (row >= a.B * a.H * a.T) return;
  const int64_t bh = row / a.T, t = row % a.T, b = bh / a.H, h = bh % a.H;
  const T* O = reinterpret_cast<const T*>(a.o) + (b * a.T + t) * a.ldo + h * a.Dh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (b * a.T + t) * a.lddo + h * a.Dh;
  float s = 0.f;
  for (int c = lane; c < a.Dh; c += 64) s += to_f(O[c]) * to_f(dO[c]);
  s = wave_sum(s);
  if (lane == 0) a.delta[row] = s;
}

// ------------------------------------------------------------------ backward: dQ
template <typename T, int DHP>
__global__ __launch_bounds__(64) void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int SLD = 32 + Vec<T>::N;
  __shared__ __attribute__((aligned(16))) T dSs[16 * SLD];
  __shared__ __attribute__((aligned(16))) T Kt[DHP * SLD];
  const int lane = threadIdx.x, g = lane >> 4, cl = lane & 15;
  const int64_t bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const uint64_t seed = eff_seed(a.seed, a.seed_base);
  const int64_t q0 = (int64_t)blockIdx.x * 16, Dh = a.Dh, tp = mask_pitch(a.T);
  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.T * a.ldq + h * Dh;
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.T * a.ldk + h * Dh;
  const T* Vp = reinterpret_cast<const T*>(a.v) + b * a.T * a.ldv + h * Dh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + b * a.T * a.lddo + h * Dh;

  Frag<T> qf[DHP / 32], df[DHP / 32];
#pragma unroll
  for (int kk = 0; kk < DHP / 32; ++kk) {
    load_frag_rows(qf[kk], Q, a.ldq, q0 + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
    load_frag_rows(df[kk], dO, a.lddo, q0 + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
  }
  float lse[4], dl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qrow = q0 + 4 * g + r;
    lse[r] = qrow < a.T ? a.lse_in[bh * a.T + qrow] : 0.f;
    dl[r] = qrow < a.T ? a.delta[bh * a.T + qrow] : 0.f;
  }
  const int64_t kend = a.mask_kind == 0 ? min(a.T, q0 + 16) : a.T;
  const int nkc = (int)((kend + 31) / 32);
  f32x4 acc[DHP / 16];
#pragma unroll
  for (int nt = 0; nt < DHP / 16; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int64_t kbase = (int64_t)kc * 32 + half * 16;
      f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f}, dp = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < DHP / 32; ++kk) {
        Frag<T> kf, vf;
        load_frag_rows(kf, K, a.ldk, kbase + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
        load_frag_rows(vf, Vp, a.ldv, kbase + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
        s = mma(qf[kk], kf, s);
        dp = mma(df[kk], vf, dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t qrow = q0 + 4 * g + r, key = kbase + cl;
        float x = masked_score(a, b, qrow, key, s[r] * a.scale);
        float p = (x == NEG_INF || qrow >= a.T) ? 0.f : aexp<T>(x - lse[r]);
        float dpe = dp[r];
        if (a.drop_p > 0.f) dpe *= drop_mul(a.drop_p, seed, (uint64_t)((bh * a.T + qrow) * tp + key));
        dSs[(4 * g + r) * SLD + half * 16 + cl] = from_f<T>(p * (dpe - dl[r]) * a.scale);
      }
    }
    stage_transposed<T, DHP>(Kt, SLD, K, a.ldk, (int64_t)kc * 32, a.T, lane, a.Dh, a.vec);
    __syncthreads();
    Frag<T> sa;
    frag_load_vec(sa, dSs + cl * SLD + 8 * g);
#pragma unroll
    for (int nt = 0; nt < DHP / 16; ++nt) {
      Frag<T> kb;
      frag_load_vec(kb, Kt + (nt * 16 + cl) * SLD + 8 * g);
      acc[nt] = mma(sa, kb, acc[nt]);
    }
  }
  T* dQ = reinterpret_cast<T*>(a.dq) + b * a.T * a.lddq + h * Dh;
#pragma unroll
  for (int nt = 0; nt < DHP / 16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t qrow = q0 + 4 * g + r;
      const int col = nt * 16 + cl;
      if (qrow < a.T && col < a.Dh) dQ[qrow * a.lddq + col] = from_f<T>(acc[nt][r]);
    }
}

// ------------------------------------------------------------------ backward: dK, dV
template <typename T, int DHP>
__global__ __launch_bounds__(64) void attn_bwd_dkv_kernel(AttnArgs a) {
  constexpr int SLD = 32 + Vec<T>::N;
  __shared__ __attribute__((aligned(16))) T Pt[16 * SLD];
  __shared__ __attribute__((aligned(16))) T dSt[16 * SLD];
  __shared__ __attribute__((aligned(16))) T Qt[DHP * SLD];
  __shared__ __attribute__((aligned(16))) T dOt[DHP * SLD];
  const int lane = threadIdx.x, g = lane >> 4, cl = lane & 15;
  const int64_t bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const uint64_t seed = eff_seed(a.seed, a.seed_base);
  const int64_t k0 = (int64_t)blockIdx.x * 16, Dh = a.Dh, tp = mask_pitch(a.T);
  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.T * a.ldq + h * Dh;
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.T * a.ldk + h * Dh;
  const T* Vp = reinterpret_cast<const T*>(a.v) + b * a.T * a.ldv + h * Dh;
  const T* dO = reinterpret_cast<const T*>(a.dout) + b * a.T * a.lddo + h * Dh;

  Frag<T> kf[DHP / 32], vf[DHP / 32];
#pragma unroll
  for (int kk = 0; kk < DHP / 32; ++kk) {
    load_frag_rows(kf[kk], K, a.ldk, k0 + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
    load_frag_rows(vf[kk], Vp, a.ldv, k0 + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
  }
  f32x4 accv[DHP / 16], acck[DHP / 16];
#pragma unroll
  for (int nt = 0; nt < DHP / 16; ++nt) {
    accv[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    acck[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // queries that can see these keys
  const int64_t qbeg = a.mask_kind == 0 ? (k0 / 32) * 32 : 0;
  for (int64_t qc = qbeg; qc < a.T; qc += 32) {
    __syncthreads();
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int64_t qb = qc + half * 16;
      f32x4 st = (f32x4){0.f, 0.f, 0.f, 0.f}, dpt = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < DHP / 32; ++kk) {
        Frag<T> qfr, dfr;
        load_frag_rows(qfr, Q, a.ldq, qb + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
        load_frag_rows(dfr, dO, a.lddo, qb + cl, a.T, kk * 32 + 8 * g, a.Dh, a.vec);
        st = mma(kf[kk], qfr, st);      // S^T[key][query]
        dpt = mma(vf[kk], dfr, dpt);    // dP^T[key][query]
      }
      const int64_t qrow = qb + cl;     // column = query
      const float lq = qrow < a.T ? a.lse_in[bh * a.T + qrow] : 0.f;
      const float dq = qrow < a.T ? a.delta[bh * a.T + qrow] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t key = k0 + 4 * g + r;
        float x = masked_score(a, b, qrow, key, st[r] * a.scale);
        float p = (x == NEG_INF || qrow >= a.T || key >= a.T) ? 0.f : aexp<T>(x - lq);
        float dm = a.drop_p > 0.f ? drop_mul(a.drop_p, seed, (uint64_t)((bh * a.T + qrow) * tp + key)) : 1.f;
        Pt[(4 * g + r) * SLD + half * 16 + cl] = from_f<T>(p * dm);
        dSt[(4 * g + r) * SLD + half * 16 + cl] = from_f<T>(p * (dpt[r] * dm - dq) * a.scale);
      }
    }
    stage_transposed<T, DHP>(Qt, SLD, Q, a.ldq, qc, a.T, lane, a.Dh, a.vec);
    stage_transposed<T, DHP>(dOt, SLD, dO, a.lddo, qc, a.T, lane, a.Dh, a.vec);
    __syncthreads();
    Frag<T> pa, sa;
    frag_load_vec(pa, Pt + cl * SLD + 8 * g);
    frag_load_vec(sa, dSt + cl * SLD + 8 * g);
#pragma unroll
    for (int nt = 0; nt < DHP / 16; ++nt) {
      Frag<T> ob, qb2;
      frag_load_vec(ob, dOt + (nt * 16 + cl) * SLD + 8 * g);
      frag_load_vec(qb2, Qt + (nt * 16 + cl) * SLD + 8 * g);
      accv[nt] = mma(pa, ob, accv[nt]);
      acck[nt] = mma(sa, qb2, acck[nt]);
    }
  }
  T* dK = reinterpret_cast<T*>(a.dk) + b * a.T * a.lddk + h * Dh;
  T* dV = reinterpret_cast<T*>(a.dv) + b * a.T * a.lddv + h * Dh;
#pragma unroll
  for (int nt = 0; nt < DHP / 16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t key = k0 + 4 * g + r;
      const int col = nt * 16 + cl;
      if (key < a.T && col < a.Dh) {
        dK[key * a.lddk + col] = from_f<T>(acck[nt][r]);
        dV[key * a.lddv + col] = from_f<T>(accv[nt][r]);
      }
    }
}

// ------------------------------------------------------------------ launchers
template <typename T, int DHP>
static hipError_t fwd_dh(AttnArgs& a, hipStream_t s) {
  dim3 grid((unsigned)cdiv(a.T, 16), (unsigned)(a.B * a.H));
  hipLaunchKernelGGL((attn_fwd_kernel<T, DHP>), grid, dim3(64), 0, s, a);
  return hipGetLastError();
}
template <typename T, int DHP>
static hipError_t bwd_dh(AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((attn_delta_kernel<T>), dim3((unsigned)cdiv(a.B * a.H * a.T, 4)), dim3(256), 0, s, a);
  dim3 grid((unsigned)cdiv(a.T, 16), (unsigned)(a.B * a.H));
  hipLaunchKernelGGL((attn_bwd_dq_kernel<T, DHP>), grid, dim3(64), 0, s, a);
  hipLaunchKernelGGL((attn_bwd_dkv_kernel<T, DHP>), grid, dim3(64), 0, s, a);
  return hipGetLastError();
}
template <typename T>
static hipError_t dispatch(bool fwd, int64_t Dh, AttnArgs& a, hipStream_t s) {
  if (Dh <= 32) return fwd ? fwd_dh<T, 32>(a, s) : bwd_dh<T, 32>(a, s);
  if (Dh <= 64) return fwd ? fwd_dh<T, 64>(a, s) : bwd_dh<T, 64>(a, s);
  if (Dh <= 128) return fwd ? fwd_dh<T, 128>(a, s) : bwd_dh<T, 128>(a, s);
  if (Dh <= 256) return fwd ? fwd_dh<T, 256>(a, s) : bwd_dh<T, 256>(a, s);
  return hipErrorInvalidValue;
}

bool attn_lds_supported(int64_t T, int64_t Dh);
hipError_t attn_lds_fwd(int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq, const void* k,
                        int64_t ldk, const void* v, int64_t ldv, void* o, int64_t ldo, float* lse, float scale,
                        int mask_kind, const int64_t* ids, float drop_p, uint64_t seed, const uint64_t* seed_base,
                        hipStream_t s);
hipError_t attn_lds_bwd(int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq, const void* k,
                        int64_t ldk, const void* v, int64_t ldv, const void* o, int64_t ldo, const void* dout,
                        int64_t lddo, const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv,
                        int64_t lddv, float scale, int mask_kind, const int64_t* ids, float drop_p, uint64_t seed,
                        const uint64_t* seed_base, float* delta, hipStream_t s);

// bf16 storage with T <= 256 takes the LDS-resident kernels (attention_lds.hip); fp32 (the
// parity mode) and anything else the register/LDS-chunk kernels above.
static bool use_lds_path(int dtype, int64_t BH, int64_t T, int64_t Dh) {
  // the LDS kernels form the dropout-mask element index in 32 bits
  const bool idx32 = BH * T * (T + (T & 1)) < ((int64_t)1 << 32);
  return dtype == RS_DTYPE_BF16 && idx32 && attn_lds_supported(T, Dh);
}

static int check(int64_t B, int64_t T, int64_t H, int64_t Dh) {
  if (B <= 0 || H <= 0 || T <= 0 || Dh <= 0 || Dh > 256) return RS_ERR_UNSUPPORTED;
  return RS_OK;
}

// 16-byte vector loads need every row start aligned: base pointers and leading dims (and the head offset Dh)
static int vec_ok(int dtype, int64_t Dh, const void* const* ptrs, int np, const int64_t* lds, int n) {
  const int vec = dtype == RS_DTYPE_BF16 ? 8 : 4;
  if (Dh % vec) return 0;
  for (int i = 0; i < n; ++i)
    if (lds[i] % vec) return 0;
  for (int i = 0; i < np; ++i)
    if ((uintptr_t)ptrs[i] % 16) return 0;
  return 1;
}

// delta[(b*H + h)*T + t] = sum over the head's Dh columns of dO * O (the attention backward's row term), one wave
// per (token row, head); the values as stored (bf16 or fp32)
template <typename E>
__global__ __launch_bounds__(256) void row_delta_kernel(int64_t M, int64_t T, int64_t H, int64_t Dh, const E* dout,
                                                        int64_t lddo, const E* o, int64_t ldo, float* delta) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= M * H) return;
  const int64_t m = w / H, h = w % H;
  const E* a = dout + m * lddo + h * Dh;
  const E* b = o + m * ldo + h * Dh;
  float s = 0.f;
  for (int64_t c = lane; c < Dh; c += 64) s = __builtin_fmaf((float)a[c], (float)b[c], s);
#pragma unroll
  for (int x = 32; x > 0; x >>= 1) s += __shfl_xor(s, x, 64);
  if (lane == 0) {
    const int64_t bb = m / T, t = m % T;
    delta[(bb * H + h) * T + t] = s;
  }
}

// bf16, Dh a multiple of 8 and 16-byte aligned rows: 16 lanes per (row, head), 16 B per lane per step
__global__ __launch_bounds__(256) void row_delta_v8_kernel(int64_t M, int64_t T, int64_t H, int64_t Dh,
                                                           const __bf16* dout, int64_t lddo, const __bf16* o,
                                                           int64_t ldo, float* delta) {
  const int64_t w = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;   // (row, head) of this 16-lane group
  const int l = threadIdx.x & 15;
  const bool ok = w < M * H;
  const int64_t ww = ok ? w : M * H - 1;
  const int64_t m = ww / H, h = ww % H;
  const __bf16* a = dout + m * lddo + h * Dh;
  const __bf16* b = o + m * ldo + h * Dh;
  float s = 0.f;
  for (int64_t c = 8 * l; c < Dh; c += 128) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(a + c), y = *reinterpret_cast<const bf16x8*>(b + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) s = __builtin_fmaf((float)x[j], (float)y[j], s);
  }
#pragma unroll
  for (int x = 8; x > 0; x >>= 1) s += __shfl_xor(s, x, 64);
  if (ok && l == 0) {
    const int64_t bb = m / T, t = m % T;
    delta[(bb * H + h) * T + t] = s;
  }
}

extern "C" {

int rs_attn_row_delta(int dtype, int64_t B, int64_t T, int64_t H, int64_t Dh, const void* dout, int64_t lddo,
                      const void* o, int64_t ldo, float* delta, void* stream) {
  if (B <= 0 || T <= 0 || H <= 0 || Dh <= 0 || !dout || !o || !delta) return RS_ERR_ARG;
  const int64_t M = B * T;
  const dim3 grid((unsigned)((M * H + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const bool v8 = Dh % 8 == 0 && lddo % 8 == 0 && ldo % 8 == 0 && ((uintptr_t)dout & 15) == 0 && ((uintptr_t)o & 15) == 0;
  if (dtype == RS_DTYPE_BF16 && v8)
    hipLaunchKernelGGL(row_delta_v8_kernel, dim3((unsigned)((M * H * 16 + 255) / 256)), dim3(256), 0, s, M, T, H,
                       Dh, (const __bf16*)dout, lddo, (const __bf16*)o, ldo, delta);
  else if (dtype == RS_DTYPE_BF16)
    hipLaunchKernelGGL(row_delta_kernel<__bf16>, grid, dim3(256), 0, s, M, T, H, Dh, (const __bf16*)dout, lddo,
                       (const __bf16*)o, ldo, delta);
  else
    hipLaunchKernelGGL(row_delta_kernel<float>, grid, dim3(256), 0, s, M, T, H, Dh, (const float*)dout, lddo,
                       (const float*)o, ldo, delta);
  return (int)hipGetLastError();
}

int rs_attn_fwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq,
                const void* k, int64_t ldk, const void* v, int64_t ldv, void* o, int64_t ldo, float* lse,
                float scale, int mask_kind, const int64_t* ids, float drop_p, uint64_t seed,
                const uint64_t* seed_base, void* stream) {
  const int64_t lds[4] = {ldq, ldk, ldv, ldo};
  int c = check(B, T, H, Dh);
  if (c) return c;
  if (mask_kind == 1 && !ids) return RS_ERR_ARG;
  const void* ptrs[4] = {q, k, v, o};
  const int vec = vec_ok(dtype, Dh, ptrs, 4, lds, 4);
  AttnArgs a = {};
  hipStream_t s = (hipStream_t)stream;
  if (vec && use_lds_path(dtype, B * H, T, Dh))
    return (int)attn_lds_fwd(B, T, H, Dh, q, ldq, k, ldk, v, ldv, o, ldo, lse, scale, mask_kind, ids, drop_p, seed,
                             seed_base, s);
  a.B = B; a.T = T; a.H = H; a.Dh = (int)Dh; a.vec = vec;
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv;
  a.o = o; a.ldo = ldo; a.lse = lse; a.scale = scale; a.mask_kind = mask_kind; a.ids = ids;
  a.drop_p = drop_p; a.seed = seed; a.seed_base = seed_base;
  return (int)(dtype == RS_DTYPE_BF16 ? dispatch<__bf16>(true, Dh, a, s) : dispatch<float>(true, Dh, a, s));
}

int rs_attn_bwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq,
                const void* k, int64_t ldk, const void* v, int64_t ldv, const void* o, int64_t ldo,
                const void* dout, int64_t lddo, const float* lse, void* dq, int64_t lddq, void* dk,
                int64_t lddk, void* dv, int64_t lddv, float scale, int mask_kind, const int64_t* ids,
                float drop_p, uint64_t seed, const uint64_t* seed_base, float* ws, void* stream) {
  const int64_t lds[8] = {ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv};
  const int delta_in = mask_kind & RS_ATTN_DELTA_IN;
  mask_kind &= ~RS_ATTN_DELTA_IN;
  int c = check(B, T, H, Dh);
  if (c) return c;
  if (mask_kind == 1 && !ids) return RS_ERR_ARG;
  const void* ptrs[8] = {q, k, v, o, dout, dq, dk, dv};
  const int vec = vec_ok(dtype, Dh, ptrs, 8, lds, 8);
  if (vec && use_lds_path(dtype, B * H, T, Dh))
    return (int)attn_lds_bwd(B, T, H, Dh, q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv,
                             lddv, scale, mask_kind | delta_in, ids, drop_p, seed, seed_base, ws, (hipStream_t)stream);
  // the generic kernels always form delta themselves (into ws)
  AttnArgs a = {};
  a.B = B; a.T = T; a.H = H; a.Dh = (int)Dh; a.vec = vec;
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv;
  a.o = const_cast<void*>(o); a.ldo = ldo; a.dout = dout; a.lddo = lddo; a.dq = dq; a.lddq = lddq;
  a.dk = dk; a.lddk = lddk; a.dv = dv; a.lddv = lddv; a.lse_in = lse; a.delta = ws; a.scale = scale;
  a.mask_kind = mask_kind; a.ids = ids; a.drop_p = drop_p; a.seed = seed; a.seed_base = seed_base;
  hipStream_t s = (hipStream_t)stream;
  return (int)(dtype == RS_DTYPE_BF16 ? dispatch<__bf16>(false, Dh, a, s) : dispatch<float>(false, Dh, a, s));
}

}  // extern "C"
