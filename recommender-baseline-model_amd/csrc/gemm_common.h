// Shared declarations of the two GEMM implementations (gemm.hip: fp32 parity path and generic;
// gemm_bf16.hip: the bf16 throughput path).
#pragma once
#include "common.h"
#include "../../include/recsys_hip.h"

#define ACT_NONE 0
#define ACT_RELU 1
#define ACT_GELU 2
#define ACT_RELU_BWD 3
#define ACT_GELU_BWD 4

struct GemmArgs {
  int64_t M, N, K;
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  int c_f32;
  int split_k; int64_t k_per_split;
  float* slab;  // when non-null: write raw fp32 partials to slab[z*slab_stride + m*N + n]
  int64_t slab_stride;
  int bias_colsum;  // (AK only) also write sum_k A(m,k) of this split to slab[z*slab_stride + M*N + m]
  float* colsum_out;  // (bf16 path, no slab) ... or add it to colsum_out[m] (epi.accumulate) / store it there
  rs_epilogue epi;
  int vec_ok;  // (bf16 path) 8-column vectorised epilogue legal for this call
  // (bf16 path, vocabulary cross-entropy epilogues of vocab_ce.hip) row labels; per (row, column
  // tile) (max, sum exp) partials [M][ntn][2]; label logits [M]; row log-sum-exp [M]; loss divisor
  struct {
    const int64_t* labels;
    float* part;
    float* tgt;
    const float* lse;
    const float* count;
    const float* dloss;
    int64_t ntn;
  } ce;
  KStamp ks;  // (bf16 path) in-kernel begin/end stamps of this launch (bench.py timing), buf null = off
  // (bf16 DMA path, rs_gemm_ln) A = BERT LayerNorm of the rows of A formed in the GEMM's prologue: gamma / beta
  // (fp32, K = d entries), eps; the column-tile-0 workgroups also store the LayerNorm output h (bf16, ldh) and the
  // row statistics mean / rinv (each nullable)
  struct {
    const float* gamma;
    const float* beta;
    float eps;
    void* h;
    int64_t ldh;
    float* mean;
    float* rinv;
  } ln;
};


hipError_t gemm_bf16_launch(int ak, int bk, GemmArgs& a, hipStream_t s);
