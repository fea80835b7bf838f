// BERT4Rec vocabulary head + CrossEntropyLoss(ignore_index=0) without materialising the logits (bf16).
//
// The reference computes logits = out(x) over the whole vocabulary (BS/models/bert.py:16) and
// CrossEntropyLoss(ignore_index=0) on them (BS/trainers/bert.py:11,36-40).  The fused training step
// already keeps only the labelled rows (R of B*T); for those, the unfused sequence wrote R x (V+1)
// fp32 logits, re-read them for the row log-sum-exp and again for the gradient (3 passes over
// 190 MB at the cfg3 shape).  Here:
//   rs_vocab_ce_fwd: GEMM h . E^T + b whose epilogue (EC_CE_PART, gemm_bf16_impl.h) leaves per
//                    (row, 128-column tile) online-softmax pairs and the label logit; one wave per
//                    row combines them into lse and the row loss; a fixed-order block sum gives
//                    out = {loss sum, labelled count, mean} (ce_finish_kernel, loss.hip semantics);
//   rs_vocab_ce_bwd: the same GEMM again, epilogue EC_CE_GRAD writing dlogits = (softmax - onehot)
//                    * dloss / count straight as bf16 (the operand of the weight and input gradients).
// The recompute costs one more 2*R*(V+1)*d GEMM and saves ~580 MB of HBM traffic per step.
#include "gemm_bf16_impl.h"

namespace vce {

// one wave per row: combine the row's tile partials (lane-strided, then a fixed butterfly)
// tgt: the label logits from the GEMM epilogue, or (lh != null) computed here as <h[r], E[label]> + b[label]
struct LabelDot {
  const __bf16* h; int64_t ldh;
  const __bf16* E; int64_t lde;
  const float* bias;
  int64_t d;
};

__global__ __launch_bounds__(256) void ce_tiles_kernel(const float* __restrict__ part, int64_t ntn, int64_t R,
                                                       const int64_t* __restrict__ labels,
                                                       const float* __restrict__ tgt, const int* __restrict__ rows_dev,
                                                       float* __restrict__ lse, float* __restrict__ rowp, LabelDot lh) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const bool live = (!rows_dev || r < *rows_dev) && labels[r] != 0;
  if (!live) {
    if (lane == 0) { lse[r] = 0.f; rowp[2 * r] = 0.f; rowp[2 * r + 1] = 0.f; }
    return;
  }
  float mx = -__builtin_inff(), sm = 0.f;
  const float2* pr = reinterpret_cast<const float2*>(part + r * ntn * 2);
  int64_t ti = lane;
  // 8 tiles' (max, sum) pairs in flight per lane, folded against their common max (1M classes: 7.8k tiles per
  // row; one dependent round trip per tile made the launch ~60 us)
  constexpr int U = 8;
  for (; ti + 64 * (U - 1) < ntn; ti += 64 * U) {
    float2 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = pr[ti + 64 * u];
    float mm = mx;
#pragma unroll
    for (int u = 0; u < U; ++u) mm = fmaxf(mm, q[u].x);
    if (mm != -__builtin_inff()) {
      float acc = sm * __expf(mx - mm);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += q[u].y * __expf(q[u].x - mm);
      sm = acc;
      mx = mm;
    }
  }
  for (; ti < ntn; ti += 64) {
    const float m2 = pr[ti].x, s2 = pr[ti].y;
    const float mm = fmaxf(mx, m2);
    sm = (mm == -__builtin_inff()) ? 0.f : sm * __expf(mx - mm) + s2 * __expf(m2 - mm);
    mx = mm;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(sm, o, 64);
    const float mm = fmaxf(mx, m2);
    sm = (mm == -__builtin_inff()) ? 0.f : sm * __expf(mx - mm) + s2 * __expf(m2 - mm);
    mx = mm;
  }
  float t = 0.f;
  if (lh.h) {
    const int64_t lb = labels[r];
    float dot = 0.f;
    for (int64_t k = lane; k < lh.d; k += 64) dot += (float)lh.h[r * lh.ldh + k] * (float)lh.E[lb * lh.lde + k];
    t = wave_sum(dot) + (lh.bias ? lh.bias[lb] : 0.f);
  }
  if (lane == 0) {
    const float L = mx + __logf(sm);
    lse[r] = L;
    rowp[2 * r] = L - (lh.h ? t : tgt[r]);
    rowp[2 * r + 1] = 1.f;
  }
}

__global__ __launch_bounds__(256) void ce_sum_kernel(const float* __restrict__ rowp, int64_t R,
                                                     const float* __restrict__ count_override, float* __restrict__ out) {
  float s = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < R; i += blockDim.x) { s += rowp[i * 2]; c += rowp[i * 2 + 1]; }
  __shared__ float rs[4], rc[4];
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = s; rc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S = rs[0] + rs[1] + rs[2] + rs[3], C = rc[0] + rc[1] + rc[2] + rc[3];
    out[0] = S;
    out[1] = C;
    out[2] = S / (count_override ? *count_override : C);
  }
}

constexpr int BN = 128;

inline int64_t ntn_of(int64_t V1) { return cdiv(V1, BN); }

// ws layout (floats): part [R][ntn][2] | tgt [R] | lse [R] | rowp [R][2]
struct Ws {
  float *part, *tgt, *lse, *rowp;
  Ws(float* ws, int64_t R, int64_t V1) {
    part = ws;
    tgt = part + R * ntn_of(V1) * 2;
    lse = tgt + R;
    rowp = lse + R;
  }
};

bool args_ok(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde) {
  return R > 0 && V1 > 0 && d > 0 && d % 8 == 0 && ldh % 8 == 0 && lde % 8 == 0 && ((uintptr_t)h % 16) == 0 &&
         ((uintptr_t)E % 16) == 0;
}

GemmArgs gemm_args(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                   const float* bias, const int64_t* labels, const int* rows_dev) {
  GemmArgs a{};
  a.M = R; a.N = V1; a.K = d;
  a.A = h; a.lda = ldh; a.B = E; a.ldb = lde;
  a.split_k = 1; a.k_per_split = d;
  a.epi.alpha = 1.0f;
  a.epi.bias = bias;
  a.epi.rows_dev = rows_dev;
  a.ce.labels = labels;
  a.ce.ntn = ntn_of(V1);
  return a;
}

}  // namespace vce

hipError_t vce_finish(const float* part, int64_t ntn, int64_t R, const int64_t* labels, const float* tgt,
                      const int* rows_dev, float* lse, float* rowp, const float* count_override, float* out,
                      hipStream_t s, const void* h, int64_t ldh, const void* E, int64_t lde, const float* bias,
                      int64_t d) {
  const vce::LabelDot lh{(const __bf16*)h, ldh, (const __bf16*)E, lde, bias, d};
  hipLaunchKernelGGL(vce::ce_tiles_kernel, dim3((unsigned)cdiv(R, 4)), dim3(256), 0, s, part, ntn, R, labels, tgt,
                     rows_dev, lse, rowp, lh);
  hipLaunchKernelGGL(vce::ce_sum_kernel, dim3(1), dim3(256), 0, s, rowp, R, count_override, out);
  return hipGetLastError();
}

extern "C" {

int64_t rs_vocab_ce_ws_numel(int64_t R, int64_t V1) {
  if (R <= 0 || V1 <= 0) return -1;
  return R * vce::ntn_of(V1) * 2 + 4 * R;
}

int rs_vocab_ce_fwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                    const float* bias, const int64_t* labels, const int* rows_dev, const float* count_override,
                    float* ws, float* out, void* stream) {
  if (!vce::args_ok(R, V1, d, h, ldh, E, lde) || !labels || !ws || !out) return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  vce::Ws w(ws, R, V1);
  GemmArgs a = vce::gemm_args(R, V1, d, h, ldh, E, lde, bias, labels, rows_dev);
  a.ce.part = w.part;
  a.ce.tgt = w.tgt;
  a.ks = kstamp_next(RS_STAMP_VOCAB_CE_FWD);
  hipError_t e = gbf::launch_cfg<false, false, 128, vce::BN, gbf::EC_CE_PART>(a, s);
  if (e != hipSuccess) return (int)e;
  return (int)vce_finish(w.part, a.ce.ntn, R, labels, w.tgt, rows_dev, w.lse, w.rowp, count_override, out, s,
                         nullptr, 0, nullptr, 0, nullptr, 0);
}

int rs_vocab_ce_bwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                    const float* bias, const int64_t* labels, const int* rows_dev, const float* count,
                    const float* dloss, const float* ws, void* dlogits, int64_t lddl, void* stream) {
  if (!vce::args_ok(R, V1, d, h, ldh, E, lde) || !labels || !ws || !count || !dlogits || lddl % 8 ||
      ((uintptr_t)dlogits % 16))
    return RS_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  vce::Ws w(const_cast<float*>(ws), R, V1);
  GemmArgs a = vce::gemm_args(R, V1, d, h, ldh, E, lde, bias, labels, rows_dev);
  a.C = dlogits;
  a.ldc = lddl;
  a.ce.lse = w.lse;
  a.ce.count = count;
  a.ce.dloss = dloss;
  return (int)gbf::launch_cfg<false, false, 128, vce::BN, gbf::EC_CE_GRAD>(a, s);
}

}  // extern "C"
