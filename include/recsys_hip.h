/*
 * recsys_hip.h -- C ABI of librecsys_hip.so, the MI355X (gfx950) hot path for
 * SASRec / BERT4Rec training.
 *
 * The reference (Furyton/Recommender-Baseline-Model, NerualNetwork/bert4rec&sas4rec,
 * "BS/" below) has no native code and no FFI: every op on its hot path is a
 * stock PyTorch module call.  Each entry point here replaces the reference
 * call(s) cited on it; the Python host side (rbm_amd.ops, bound with ctypes)
 * keeps the reference's model/trainer API on top.
 *
 * Conventions (every function):
 *   - raw device pointers + sizes, plus a hipStream_t passed as void*; the
 *     caller passes torch.cuda.current_stream().cuda_stream;
 *   - nothing is allocated or freed; every buffer, including workspace, is
 *     owned by the caller (graph-capturable: no sync, no malloc);
 *   - returns 0 on success, a hipError_t value, or RS_ERR_* (1001 bad argument,
 *     1002 unsupported shape/dtype);
 *   - dtype: 0 = fp32 (parity mode: exact f32-input MFMA), 1 = bf16 (storage
 *     and MFMA operands; fp32 accumulate).  Gradients, LN/softmax statistics,
 *     biases, LN affine params and the loss are always fp32.
 *   - ids are int64 (the reference feeds torch.LongTensor / int64 numpy).
 */
#ifndef RECSYS_HIP_H
#define RECSYS_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define RS_ERR_ARG 1001
#define RS_ERR_UNSUPPORTED 1002

/* Fused GEMM epilogue, applied per output element in this order:
 *   v = alpha*acc (+ bias[n])
 *   act: 1 relu / 2 gelu_tanh (pre-activation stored to aux_out if set),
 *        3 relu_bwd (v *= aux>0), 4 gelu_bwd (v *= gelu'(aux))
 *   dropout: v *= keep(drop_seed, m*drop_ld+n) / (1-drop_p)
 *   v += resid[m*ldres+n];  v *= (rowmask_ids[m] != 0);
 *   post dropout: v *= keep(post_drop_seed, m*drop_ld+n) / (1-post_drop_p);  v += C (accumulate)
 * rows_dev (nullable, device int): only rows m < min(M, *rows_dev) are computed/stored -- the
 * row count of a device-side compaction (BERT labelled rows) without a host sync.           */
typedef struct rs_epilogue {
  const float* bias;
  float alpha;
  int act;
  const void* aux;
  void* aux_out;
  int64_t ldaux;
  float drop_p;
  uint64_t drop_seed;          /* site salt */
  const uint64_t* seed_base;   /* device step seed (nullable) */
  int64_t drop_ld;
  const void* resid;
  int64_t ldres;
  const int64_t* rowmask_ids;
  int accumulate;
  float post_drop_p;
  uint64_t post_drop_seed;
  const int* rows_dev;
} rs_epilogue;

/* C[M,N] = epi(A . B^T).  a_kmajor: A(m,k) at A[k*lda+m] (else A[m*lda+k]);
 * b_kmajor: B(n,k) at B[k*ldb+n] (else B[n*ldb+k]).  c_f32 selects an fp32 C.
 * split_k > 1 writes raw fp32 partials to slab[split_k][M][N] (epi ignored);
 * finish with rs_reduce_slabs.
 * Replaces: nn.Linear / nn.Conv1d(k=1) forward and autograd backward
 *   (BS/models/sas_model/sas.py:10-17, torch F.multi_head_attention_forward
 *   in_proj/out_proj via sas.py:45-47,75; BS/models/bert_modules/attention/
 *   multi_head.py:18-19,29,40; utils/feed_forward.py:10-16; BS/models/bert.py:10,16). */
int rs_gemm(int dtype, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
            const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int c_f32,
            const rs_epilogue* epi, int split_k, float* slab, void* stream);

/* C = epi(LN(X) W^T) with the BERT LayerNorm (variant 1 of rs_layernorm_fwd: gamma (x - mean) / (std_unbiased + eps)
 * + beta) formed in the GEMM's prologue (bf16 X / W / C, K = d = 256, N % 128 == 0; epilogues: bias, bias + GELU
 * (+ dropout, aux_out = the pre-activation)).  h (bf16 [M][ldh]), mean, rinv (fp32 [M]) receive the LayerNorm output
 * and row statistics exactly as rs_layernorm_fwd writes them (each nullable); C is bit-identical to rs_layernorm_fwd
 * + rs_gemm.  RS_ERR_UNSUPPORTED for other shapes / epilogues (the caller runs the two launches).
 * Replaces: utils/sublayer.py:16-18's norm(x) feeding attention/multi_head.py:18-19 (the q/k/v Linears) and
 * utils/feed_forward.py:15-16 (w_1 + GELU + dropout). */
int rs_gemm_ln(int64_t M, int64_t N, int64_t K, const void* X, int64_t ldx, const float* gamma, const float* beta,
               float eps, const void* W, int64_t ldw, void* C, int64_t ldc, const rs_epilogue* epi, void* h,
               int64_t ldh, float* mean, float* rinv, void* stream);

/* out[i] (+)= sum_z slab[z*n+i], fixed order (deterministic split-K finish). */
int rs_reduce_slabs(const float* slab, int splits, int64_t n, float* out, int accumulate, void* stream);
/* Same over slabs of n0+n1 floats: the first n0 columns go to out0, the rest to out1. */
int rs_reduce_slabs2(const float* slab, int splits, int64_t n0, float* out0, int64_t n1, float* out1, int accumulate,
                     void* stream);

/* Weight + bias gradient of a Linear / Conv1d(k=1) layer over M token rows:
 *   dW[N,K] (+)= sum_m dY[m,:]^T X[m,:];   db[N] (+)= sum_m dY[m,:]   (db nullable)
 * split-K over the rows into `splits` fp32 slabs (slab >= splits*(N*K + N) floats), the bias
 * column sums fused into the GEMM, then one deterministic reduce.  accumulate: += into dW/db.
 * rows_dev (nullable, device int): only the first min(M, *rows_dev) rows contribute.
 * Replaces the autograd weight/bias gradients of nn.Linear / nn.Conv1d / in_proj / out_proj
 * (BS/models/sas_model/sas.py:10-17,45-47; BS/models/bert_modules/attention/multi_head.py:18-19;
 * utils/feed_forward.py:10-11; BS/models/bert.py:10). */
int rs_linear_wgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dY, int64_t lddy, const void* X,
                    int64_t ldx, float* dW, float* db, int accumulate, int splits, float* slab, const int* rows_dev,
                    void* stream);

/* out[n] (+)= sum_m X[m*ldx+n] over M rows (bias gradients).  ws: >= 64*N floats. */
int rs_colsum(int dtype, const void* X, int64_t M, int64_t N, int64_t ldx, float* ws, float* out,
              int accumulate, void* stream);

/* Embedding stage.  mode 0 = SAS (BS/models/sas_model/sas.py:60-67):
 *   x = table[ids]*scale + pos[t]; dropout; x *= (ids != 0)
 * mode 1 = BERT (BS/models/bert_modules/embedding/bert.py:29-31):
 *   x = table[ids] + pos[t]; dropout.        t = row % T, rows = B*T. */
int rs_embed_fwd(int dtype, int mode, const int64_t* ids, int64_t rows, int64_t T, const void* table,
                 const void* pos, int64_t d, float scale, float drop_p, uint64_t seed, const uint64_t* seed_base,
                 void* out, void* stream);
/* dtable[ids[r]] += dX*mask*scale (rows with id 0 skipped: padding_idx=0, fp32 atomics);
 * dpos[t] (+)= sum_b dX[b,t] * mask (deterministic; accumulate flag). */
int rs_embed_bwd(int dtype, int mode, const int64_t* ids, int64_t rows, int64_t T, const void* dx,
                 int64_t d, float scale, float drop_p, uint64_t seed, const uint64_t* seed_base,
                 float* dtable, float* dpos, int accumulate_pos, void* stream);

/* LayerNorm over rows of d.  variant 0 = torch.nn.LayerNorm (biased var,
 * eps in sqrt; BS/models/sas_model/sas.py:39,42,50); variant 1 = BERT custom
 * a2*(x-mean)/(std_unbiased+eps)+b2 (BS/models/bert_modules/utils/layer_norm.py:14-17).
 * Saves mean[M] and rinv[M] (1/sqrt(var+eps), or 1/(std+eps)). */
int rs_layernorm_fwd(int dtype, int variant, const void* X, int64_t ldx, int64_t M, int64_t d,
                     const float* gamma, const float* beta, float eps, void* Y, int64_t ldy,
                     float* mean, float* rinv, void* stream);
/* dX (+)= LN backward; dgamma/dbeta += column sums (deterministic, ws >= 2*d*512 floats). */
int rs_layernorm_bwd(int dtype, int variant, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                     int64_t M, int64_t d, const float* gamma, const float* mean, const float* rinv, float eps,
                     void* dX, int64_t lddx, int accumulate_dx, float* dgamma, float* dbeta, float* ws,
                     void* stream);
/* The affine-gradient partial count of rs_layernorm_bwd's vectorised path (d a multiple of 8 bf16 / 4 fp32 with
 * 16-byte aligned rows and leading dimensions): with dgamma = dbeta = NULL it leaves ws[nparts][2][d] (gamma
 * terms, then beta terms) unreduced, for a later grouped reduction (rs_reduce_segments / rs_wgrad_grouped's extra
 * segments).  0 = the shape takes the other path (pass dgamma/dbeta). */
int64_t rs_layernorm_bwd_nparts(int dtype, int64_t M, int64_t d);
/* rs_layernorm_bwd followed by the dropout site(s) that consume dX, in one launch (vectorised path; other shapes
 * run the two launches): out2 == NULL -- out1 = drop(dX; salt1) as rs_dropout_rowmask without a row mask;
 * else out1 = drop(dX; salt1), out2 = drop(out1; salt2) as rs_dropout2.  dX as stored (accumulated) is the
 * input; hash index row * d + column; out1/out2 dense [M][d].  (BERT: bert_modules/utils/sublayer.py:18 and
 * transformer.py:32 backward.) */
int rs_layernorm_bwd_drop(int dtype, int variant, const void* X, int64_t ldx, const void* dY, int64_t lddy,
                          int64_t M, int64_t d, const float* gamma, const float* mean, const float* rinv, float eps,
                          void* dX, int64_t lddx, int accumulate_dx, float* dgamma, float* dbeta, float* ws,
                          float drop_p, uint64_t salt1, uint64_t salt2, const uint64_t* seed_base, void* out1,
                          void* out2, void* stream);

/* Fused scaled-dot-product attention per (sequence, head), T keys, head dim Dh.
 * q/k/v/o rows are tokens (b*T + t); head h occupies columns [h*Dh, (h+1)*Dh).
 * mask_kind 0 = causal, -inf above the diagonal (SAS, sas.py:70 + torch MHA baddbmm);
 * mask_kind 1 = key padding, scores of keys with ids==0 replaced by -1e9 (BERT,
 * bert_modules/bert.py:38 + attention/single.py:28).  S = scale * q.k^T;
 * P = softmax(S); P = dropout(P); O = P.v.  lse[(b*H+h)*T + t] = row logsumexp.
 * Dropout keep(seed, idx) of P[b,h,q,k] uses idx = ((b*H + h)*T + q)*Tp + k, Tp = T + (T & 1) (even row
 * pitch), i.e. rs_dropout_rowmask over a (B*H*T, Tp) tensor draws the same mask (tests materialise it). */
int rs_attn_fwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq,
                const void* k, int64_t ldk, const void* v, int64_t ldv, void* o, int64_t ldo, float* lse,
                float scale, int mask_kind, const int64_t* ids, float drop_p, uint64_t seed,
                const uint64_t* seed_base, void* stream);
/* Backward: dq, dk, dv (overwritten).  ws: >= B*H*T floats (row deltas).  mask_kind | RS_ATTN_DELTA_IN: ws
 * already holds delta[(b*H+h)*T + t] = rowsum(dO * O) over the head's columns (rs_sas_block_out_bwd with o given
 * forms it); the bf16 LDS path then reads neither O nor recomputes it (other paths recompute it into ws). */
#define RS_ATTN_DELTA_IN 0x100
/* delta[(b*H+h)*T + t] = rowsum over head h's Dh columns of dout * o (values as stored; dtype as rs_attn_bwd) --
 * the RS_ATTN_DELTA_IN input when no fused kernel forms it (BERT: after the output projection's input gradient,
 * bert_modules/attention/multi_head.py + single.py reversed). */
int rs_attn_row_delta(int dtype, int64_t B, int64_t T, int64_t H, int64_t Dh, const void* dout, int64_t lddo,
                      const void* o, int64_t ldo, float* delta, void* stream);
int rs_attn_bwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t Dh, const void* q, int64_t ldq,
                const void* k, int64_t ldk, const void* v, int64_t ldv, const void* o, int64_t ldo,
                const void* dout, int64_t lddo, const float* lse, void* dq, int64_t lddq, void* dk,
                int64_t lddk, void* dv, int64_t lddv, float scale, int mask_kind, const int64_t* ids,
                float drop_p, uint64_t seed, const uint64_t* seed_base, float* ws, void* stream);

/* SAS sampled tied logits (sas.py:93-100): pl[m] = <f[m], E[pos[m]]>, nl likewise (fp32 out). */
int rs_sampled_logits_fwd(int dtype, const void* f, int64_t M, int64_t d, const void* E,
                          const int64_t* pos, const int64_t* neg, float* pl, float* nl, void* stream);
/* df[m] (+)= dpl*E[pos]+dnl*E[neg];  dE[pos] += dpl*f, dE[neg] += dnl*f (id 0 skipped). */
int rs_sampled_logits_bwd(int dtype, const void* f, int64_t M, int64_t d, const void* E,
                          const int64_t* pos, const int64_t* neg, const float* dpl, const float* dnl,
                          void* df, int accumulate_df, float* dE, void* stream);
/* SAS loss (BS/trainers/sas.py:40-49): mean BCEWithLogits(pl,1) + mean BCEWithLogits(nl,0)
 * over valid = (pos != 0).  Writes out[0] = sum of terms, out[1] = count, out[2] = loss
 * (= pos_sum/count + neg_sum/count, count taken from count_override if non-null -- the DP
 * global count), out[3] = neg_sum.  out needs 4 floats; ws >= 3*256 floats. */
int rs_bce_fwd(const float* pl, const float* nl, const int64_t* pos, int64_t M, const float* count_override,
               float* ws, float* out, void* stream);
/* dpl, dnl = dloss * (sigmoid(x) - y) / count on valid positions, 0 elsewhere. */
int rs_bce_bwd(const float* pl, const float* nl, const int64_t* pos, int64_t M, const float* count,
               const float* dloss, float* dpl, float* dnl, void* stream);

/* BERT loss (BS/trainers/bert.py:36-40): CrossEntropyLoss(ignore_index=0) over
 * R rows of V1 fp32 logits (leading dim ldl).  out[0] = sum of -log p(label),
 * out[1] = count, out[2] = loss (count_override as in rs_bce_fwd).
 * ws >= 3*R floats (row lse + partials).  rows_dev (nullable): rows >= *rows_dev are skipped (the
 * tail of a labelled-row compaction, see rs_compact_rows). */
int rs_ce_fwd(const float* logits, int64_t R, int64_t V1, int64_t ldl, const int64_t* labels,
              const float* count_override, float* ws, float* out, const int* rows_dev, void* stream);
/* dlogits (may alias logits) = dloss * (softmax - onehot)/count on labelled rows, 0 else; dtype of
 * dlogits selected by dtype (fp32 or bf16 copy for the following GEMMs). */
int rs_ce_bwd(int dtype, const float* logits, int64_t R, int64_t V1, int64_t ldl, const int64_t* labels,
              const float* count, const float* dloss, const float* ws, void* dlogits, int64_t lddl,
              const int* rows_dev, void* stream);

/* Labelled-row compaction for the BERT loss head (BS/trainers/bert.py:36-40 drops label-0 rows).
 * idx[i] = i-th row with labels != 0 (ascending, i < cap), rank[r] = position of row r in idx or -1,
 * *count = min(#labelled, cap) -- all on the device (the count bounds later GEMMs via rows_dev). */
int rs_compact_rows(const int64_t* labels, int64_t n, int64_t cap, int32_t* idx, int32_t* rank, int32_t* count,
                    void* stream);
/* dst[i,:] = src[idx[i],:] for i < *count, zero rows up to cap; lab_out[i] = labels[idx[i]] (0 beyond). */
int rs_gather_rows(int dtype, const void* src, int64_t lds, int64_t d, const int32_t* idx, const int32_t* count,
                   int64_t cap, void* dst, int64_t ldd, const int64_t* labels, int64_t* lab_out, void* stream);
/* dst[r,:] = rank[r] >= 0 ? src[rank[r],:] : 0 for r < n (the hidden-state gradient scattered back). */
int rs_scatter_rows(int dtype, const void* src, int64_t lds, int64_t d, const int32_t* rank, int64_t n, void* dst,
                    int64_t ldd, void* stream);

/* dst[r] = rank[r] >= 0 ? sum_z slab[z][rank[r]][:] : 0 (cast to dtype) for r < n: the split-K partials
 * (slab[splits][cap][d] fp32, rs_gemm split_k of a compacted-row GEMM) reduced, cast and scattered back
 * to the token rows in one pass (replaces rs_reduce_slabs + rs_cast_bf16 + rs_scatter_rows). */
int rs_splitk_scatter_rows(int dtype, const float* slab, int splits, int64_t cap, int64_t d, const int32_t* rank,
                           int64_t n, void* dst, int64_t ldd, void* stream);

/* Large-tile bf16 GEMM with a 256-wide output (gemm_n256.hip; the vocabulary head's weight-sized products at
 * d = 256, BS/models/bert.py:10,16 + BS/trainers/bert.py:36-40): C[m][0..256) = sum_k A(m, k) B(k, n), fp32 out.
 * A(m, k) = A[k*lda + m] (a_kmajor: dE = dlogits^T h) or A[m*lda + k] (dh = dlogits E); B(k, n) = B[k*ldb + n].
 * colsum (a_kmajor only, nullable): colsum[m] = sum_k A(m, k) (the bias gradient).  rows_dev (nullable, device int):
 * bounds K (a_kmajor) or M (else) -- the labelled-row count of a compacted batch.  split != 0 splits K into
 * rs_gemm_n256_splits(M, K) slices written to C + z * c_split_stride (fp32 partial slabs).  16-B aligned operands,
 * lda / ldb multiples of 8. */
int rs_gemm_n256_splits(int64_t M, int64_t K);
int rs_gemm_n256(int a_kmajor, int64_t M, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                 int64_t ldc, int split, int64_t c_split_stride, float* colsum, const int* rows_dev, void* stream);

/* Eval scores at candidate ids (replaces SAS.predict's item_emb(candidates).matmul(final_feat), BS/models/sas_model/
 * sas.py:107-118, and BERTTrainer.calculate_metrics' logits[:, -1, :].gather(1, candidates), BS/trainers/bert.py:
 * 43-49): out[b][c] = <h[b*ldh .. + d], E[cand[b][c]]> (+ bias[cand[b][c]] when bias != NULL), fp32.  h, E in dtype
 * (RS_DTYPE_*); cand int64 [B][C] in [0, V) (others score NaN). */
int rs_candidate_scores(int dtype, const void* h, int64_t ldh, int64_t B, int64_t d, const void* E, const float* bias,
                        const int64_t* cand, int64_t C, int64_t V, float* out, void* stream);

/* torch.optim.Adam step (BS/trainers/base.py:225-228; amsgrad=False) over a
 * flat fp32 buffer.  hyper (device double[5]) = {lr, beta1, beta2, eps, weight_decay} (doubles, as torch's Python
 * floats: the scalars are formed in double and cast to float where they meet the tensors, like torch's).
 * state (device double[8]; double[144] for rs_adam_prepare_step; zero-initialised): rs_adam_prepare does state[0] += 1 (the step count t)
 * and forms state[1] = float(lr/(1-beta1^t)), state[2] = float(sqrt(1-beta2^t)) (double math), state[3] = 1/(*grad_divisor) (1 when null: the
 * data-parallel step all-reduces UNnormalised gradients plus the valid-position count and
 * divides here, so the summed gradient equals the single-device mean's).  rs_adam_step then
 * updates (grad scaled by state[3])
 * p, m, v (and writes the bf16 copy of p to p_bf16 when non-null); zero_grad != 0 also clears g
 * (the next step's accumulation starts from zero without a separate fill).  rs_adam_prepare
 * also advances *seed_base when non-null (the next step's dropout masks, as rs_seed_advance).
 * rs_adam_prepare_step = rs_adam_prepare + rs_adam_step in ONE launch (every workgroup derives step
 * t's scalars; the last to finish publishes them; state[7] and state[16 + 16 k], k < 8, are its arrival
 * counters and must be 0 between launches); further ranges of the same step then use rs_adam_step.  ntd > 0 (with p_bf16): the bf16
 * result is also written TRANSPOSED for ntd matrices of the buffer, tdesc (device int64 [ntd][6]) = rows,
 * cols, src_off (element offset of the matrix in the flat buffer whose element tbase is p[0]), lds
 * (% 4 == 0), dst_off, ldd: wT[dst_off + c*ldd + r] = bf16(p[src_off + r*lds + c]) (rs_transpose_bf16's
 * output, so the SAS backward's transposed weights need no separate launch).  Same results bit for bit. */
int rs_adam_prepare(double* state, const double* hyper, const float* grad_divisor, uint64_t* seed_base,
                    void* stream);
int rs_adam_step(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16,
                 const double* state, const double* hyper, int zero_grad, void* stream);
/* rs_adam_step on at most max_wg workgroups (grid-stride; same results bit for bit): a range updated on a side
 * stream beside other kernels (BERT's out.weight during the encoder backward) takes a bounded share of the CUs.
 * Replaces the same torch.optim.Adam step (BS/trainers/base.py:225-228) over that range. */
int rs_adam_step_wg(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, const double* state,
                    const double* hyper, int zero_grad, int max_wg, void* stream);
int rs_adam_prepare_step(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, double* state,
                         const double* hyper, int zero_grad, const float* grad_divisor, uint64_t* seed_base,
                         const int64_t* tdesc, int ntd, int64_t tbase, void* wT, void* stream);
/* rs_adam_prepare_step that also writes *loss_out = *loss_sum / *grad_divisor (data parallel: the step's mean
 * loss from the all-reduced gradient tail) in the same launch. */
int rs_adam_prepare_step_loss(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, double* state,
                              const double* hyper, int zero_grad, const float* grad_divisor, uint64_t* seed_base,
                              const int64_t* tdesc, int ntd, int64_t tbase, void* wT, const float* loss_sum,
                              float* loss_out, void* stream);
/* rs_adam_step_wg / rs_adam_prepare_step_loss over a range holding (part of) a table whose gradient only
 * rs_item_grad_marked writes: table row r is launch element moff + r * 2^dshift (moff may be negative), mrows rows,
 * 5 <= dshift <= 16 (rows of at least 32 elements: a wave tests its rows' marks from one 16-byte window; smaller
 * dshift returns RS_ERR_ARG);
 * a row with row_marks[r] != *epoch has a zero gradient this step, so its gradient is not read (nor cleared: it
 * is zero already).  Same results bit for bit as the unmarked launches.  row_marks == NULL: the unmarked launch.
 * row_marks: 16-byte aligned, (mrows + 15) / 16 * 16 + 16 + 1024 bytes, the bytes past the stamps zero (the
 * sweep's scalar mark loads run up to 16 bytes past a row; unstamped rows' gradient loads read the zero tail).
 * Only valid while nothing but the marked item gradient writes that table's gradient rows (single device, no
 * l2 regulariser, no exchange). */
int rs_adam_step_marked(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, const double* state,
                        const double* hyper, int zero_grad, int max_wg, const uint8_t* row_marks, const uint8_t* epoch,
                        int64_t moff, int64_t mrows, int dshift, void* stream);
int rs_adam_prepare_step_marked(int64_t n, float* p, float* g, float* m, float* v, void* p_bf16, double* state,
                                const double* hyper, int zero_grad, const float* grad_divisor, uint64_t* seed_base,
                                const int64_t* tdesc, int ntd, int64_t tbase, void* wT, const float* loss_sum,
                                float* loss_out, const uint8_t* row_marks, const uint8_t* epoch, int64_t moff,
                                int64_t mrows, int dshift, void* stream);

/* SASRec's parameter-norm regulariser, BS/trainers/sas.py:51-52 (loss += l2_emb * torch.norm(p) for every
 * parameter p): *loss += l2 * sum_seg ||p_seg||_2 and g += scale * l2 * p / ||p_seg|| (0 where the norm is 0,
 * as torch's norm backward).  desc: device int64 [nchunk][4] = {lo, hi, first chunk of the segment, chunks of
 * the segment} over the flat parameter buffer (chunks of one segment consecutive); ws: fp32 [2 * nchunk]; scale:
 * device float or null (= 1; the data-parallel step passes the global count its optimizer divides by);
 * g and loss nullable.  Deterministic. */
int rs_l2_penalty(const float* p, float* g, const int64_t* desc, int64_t nchunk, float l2, const float* scale,
                  float* ws, float* loss, void* stream);

/* dst_bf16[i] = bf16(src[i]) */
int rs_cast_bf16(int64_t n, const float* src, void* dst, void* stream);

/* out = x * keep(seed, m*drop_ld+n)/(1-p) * (rowmask_ids[m] != 0); also (optional)
 * out_masked = x * (rowmask != 0).  Elementwise backward helper for dropout sites
 * that feed GEMMs (SAS FFN dropout2 + timeline mask, sas.py:17,84). */
int rs_dropout_rowmask(int dtype, const void* x, int64_t M, int64_t N, int64_t ld, float drop_p,
                       uint64_t seed, const uint64_t* seed_base, int64_t drop_ld, const int64_t* rowmask_ids,
                       void* out, void* out_masked, void* stream);

/* Two stacked dropout sites' backward in one pass (bert.py encode_backward: block-output then
 * residual dropout of BERT4Rec's SublayerConnection/TransformerBlock, BS/models/bert_modules/
 * transformer.py:32, utils/sublayer.py:18): out1 = x * keep(salt1)/(1-p),
 * out2 = out1 * keep(salt2)/(1-p), each rounded to the dtype.  N, ld multiples of 8. */
int rs_dropout2(int dtype, const void* x, int64_t M, int64_t N, int64_t ld, float drop_p, uint64_t salt1,
                uint64_t salt2, const uint64_t* seed_base, int64_t drop_ld, void* out1, void* out2, void* stream);

/* ---- BERT vocabulary head + CrossEntropyLoss(ignore_index=0), logits never materialised (bf16;
 * vocab_ce.hip).  Replaces, for the labelled rows of the fused step, rs_gemm (logits = h E^T + b,
 * BS/models/bert.py:16) + rs_ce_fwd + rs_ce_bwd (BS/trainers/bert.py:11,36-40).
 * h [R][d] bf16 (ldh), E [V1][d] bf16 (lde), bias [V1] fp32, labels [R] (0 = ignored), rows_dev:
 * device row count (rows >= it are skipped; nullable).  ws: rs_vocab_ce_ws_numel floats, written by
 * fwd and read by bwd.  fwd: out = {loss sum, labelled count, sum / (count_override or count)};
 * bwd: dlogits [R][V1] bf16 (lddl, 16-B aligned rows) = (softmax - onehot) * (dloss or 1) / count. */
int64_t rs_vocab_ce_ws_numel(int64_t R, int64_t V1);
int rs_vocab_ce_fwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                    const float* bias, const int64_t* labels, const int* rows_dev, const float* count_override,
                    float* ws, float* out, void* stream);
int rs_vocab_ce_bwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                    const float* bias, const int64_t* labels, const int* rows_dev, const float* count,
                    const float* dloss, const float* ws, void* dlogits, int64_t lddl, void* stream);

/* ---- vocabulary head, vocabulary-tile-stationary (vocab_head.hip; bf16, d in {64, 128, 256}) -----
 * Same math and workspace layout (rs_vocab_ce_ws_numel) as rs_vocab_ce_fwd/bwd, for the same reference
 * lines (BS/models/bert.py:10,16, BS/trainers/bert.py:11,36-40); one persistent workgroup per CU keeps a
 * 256- (fwd) / 128-entry (bwd) tile of E in LDS and walks every 128-row tile of h against it, so E streams
 * from HBM once and the short d-deep products run back to back instead of one cold tile at a time.
 * rs_vocab_head_fwd: out = {loss sum, labelled count, sum / (count_override or count)}, ws keeps lse.
 * rs_vocab_head_bwd: dlogits [R][V1] bf16 (rows < live count) = (softmax - onehot) * (dloss or 1) / count. */
int rs_vocab_head_supported(int64_t d);
int rs_vocab_head_fwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                      const float* bias, const int64_t* labels, const int* rows_dev, const float* count_override,
                      float* ws, float* out, void* stream);
int rs_vocab_head_bwd(int64_t R, int64_t V1, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                      const float* bias, const int64_t* labels, const int* rows_dev, const float* count,
                      const float* dloss, const float* ws, void* dlogits, int64_t lddl, int64_t voff, void* stream);

/* Vocabulary-sharded head (data-parallel rank r owns rows [v0, v1) of E = out.weight and b;
 * every rank holds the labelled rows h of ALL ranks, all-gathered).  Labels stay absolute vocabulary ids
 * (0 = not labelled); rs_vocab_head_bwd's voff = v0 places E's rows.
 * rs_vocab_shard_lse: per row, log-sum-exp of h E_shard^T + b_shard (0 for unlabelled rows); ws as
 *   rs_vocab_ce_ws_numel(R, v1 - v0).
 * rs_vocab_shard_label_logits: tgt[r] = <h[r], E[label - v0]> + b[label - v0] where this shard holds the label,
 *   else 0 (summed over ranks: every row's label logit).
 * rs_vocab_shard_combine: lse_parts [N][R] (every shard's lse, all-gathered) -> lse [R] over the whole
 *   vocabulary; out = {loss sum, labelled count, mean} of CE over the labelled rows. */
int rs_vocab_shard_lse(int64_t R, int64_t V1s, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                       const float* bias, const int64_t* labels, float* ws, float* lse, void* stream);
int rs_vocab_shard_label_logits(int64_t R, int64_t d, const void* h, int64_t ldh, const void* E, int64_t lde,
                                const float* bias, const int64_t* labels, int64_t v0, int64_t v1, float* tgt,
                                void* stream);
int rs_vocab_shard_combine(int N, int64_t R, const float* lse_parts, const float* tgt, const int64_t* labels,
                           float* lse, float* out, void* stream);

/* Host-only: the causal attention backward's work plan for (B, T, H) -- per (split < 4, wave < 8, item < 6) a
 * uint32 (valid << 31 | slot << 26 | role << 24 | chunk end << 16 | chunk begin << 8 | tile; attention_lds.hip
 * make_plan) of the dK/dV (dkv = 1) or dQ pass; *nsplit = workgroups per sequence.  Returns RS_ERR_UNSUPPORTED
 * where the kernels fall back to one tile per wave (T < 128 or no plan fits). */
int rs_attn_bwd_plan(int64_t B, int64_t T, int64_t H, int dkv, uint32_t* plan, int* nsplit);

/* Kernel stamps (bench.py's in-step timing of the dominant launch; not on the reference's path).
 * While enabled (buf != NULL), rs_attn_bwd (bf16 LDS path), rs_wgrad_grouped and rs_vocab_ce_fwd (its
 * logits GEMM) launches of the kinds in kind_mask (bit RS_STAMP_*) are stamped -- marks numbered in launch order from 0, fixed into the kernel
 * arguments, so a captured graph keeps stamping on every replay.  buf (device u64) = {base step, steps
 * held, marks per step, W, then per (slot = (int64)*step - base, mark) a record {begin, end lanes
 * 0 .. W-1}} in s_memrealtime ticks (begin: the first dispatched workgroup's start; each wave raises
 * end lane (wave index mod W) to its exit time; the launch ends at the max over the lanes).  step: the optimizer's device step count (double, rs_adam_prepare's
 * state[0]).  rs_kernel_stamps(NULL, NULL, 0) disables.  rs_kernel_stamp_count / rs_kernel_stamp_kinds:
 * the marks handed out since the last enable and their kinds.  rs_wall_clock_khz: tick rate. */
#define RS_STAMP_ATTN_BWD 1
#define RS_STAMP_WGRAD_GROUPED 2
#define RS_STAMP_VOCAB_CE_FWD 3   /* the logits GEMM of rs_vocab_ce_fwd / the rs_vocab_head_fwd kernel */
int rs_kernel_stamps(uint64_t* buf, const double* step, int kind_mask);
int rs_kernel_stamp_count(void);
int rs_kernel_stamp_kinds(int* kinds, int n);
int rs_wall_clock_khz(int* khz);

/* *seed_base += 1 on the stream (advances every dropout mask; capturable). */
int rs_seed_advance(uint64_t* seed_base, void* stream);
/* Upload an instantiated step graph (hipGraphExec_t) to the device ahead of its first launch (hipGraphUpload):
 * graph preparation, no step runs.  Infrastructure of the captured training step (BS/trainers/base.py:114-123's
 * loop body replayed as one graph), not a reference op. */
int rs_graph_upload(void* graph_exec, void* stream);

/* ---- fused SAS sublayers (bf16, d in {64, 128}; rowchain.hip) ----------------------------
 * One workgroup per CU stages the block's weights in LDS once, each wave carries 16 tokens
 * through the whole chain in registers.
 * Same outputs, saved tensors and dropout masks as the unfused kernel sequence, so rs_* backward
 * kernels consume them unchanged.
 *
 * Replaces, for SASRec block i (BS/models/sas_model/sas.py:73-76, the attention input side):
 *   Q = LN1(x) [mean/rstd saved];  q = Q Wq^T + bq;  kv = x Wkv^T + bkv   (kv: [M][2d])
 * Wq = in_proj_weight[:d], Wkv = in_proj_weight[d:] (bf16, torch [out][in] layout).
 * Returns RS_ERR_UNSUPPORTED for other d: callers fall back to the unfused sequence. */
int rs_sas_block_in(int64_t M, int64_t d, const void* x, int64_t ldx, const float* ln_w, const float* ln_b,
                    float eps, void* Q, float* mean, float* rstd, const void* Wq, const float* bq, void* q,
                    const void* Wkv, const float* bkv, void* kv, void* stream);
/* The first block's input side with the embedding stage folded in (rowchain: one launch instead of two): x0 =
 * (item_emb[ids]*scale + pos_emb[t]) -> dropout(p, salt) -> *(ids != 0), exactly as rs_embed_fwd mode 0, stored
 * to x0 [M][d] and fed to rs_sas_block_in's chain; with count_ids, count_parts[rs_sas_block_in_count_parts(M)]
 * (int32) receives per-workgroup counts of count_ids != 0 (the BCE divisor for rs_sas_block_out_head).  d in {64, 128}
 * and 16-byte aligned tables / x0, else RS_ERR_ARG. */
int64_t rs_sas_block_in_count_parts(int64_t M);
int rs_sas_block_in_embed(int64_t M, int64_t d, const int64_t* ids, int64_t T, const void* item_emb, const void* pos_emb,
                          float scale, float drop_p, uint64_t salt, const uint64_t* seed_base, void* x0,
                          const int64_t* count_ids, int* count_parts, const float* ln_w, const float* ln_b, float eps,
                          void* Q, float* mean, float* rstd, const void* Wq, const float* bq, void* q, const void* Wkv,
                          const float* bkv, void* kv, void* stream);
/* The output side (sas.py:75-84, PointWiseFeedForward sas.py:8-24):
 *   x1 = Q + o Wo^T + bo;  z = LN2(x1);  h1 = relu(drop(z W1^T + b1, salt1));
 *   xn = (drop(h1 W2^T + b2, salt2) + z) * (ids != 0)
 * Dropout element index m*d + n, seeds eff_seed(salt, *seed_base) as rs_gemm's epilogue. */
int rs_sas_block_out(int64_t M, int64_t d, const void* o, const void* Q, const void* Wo, const float* bo, void* x1,
                     const float* ln_w, const float* ln_b, float eps, void* z, float* mean, float* rstd,
                     const void* W1, const float* b1, void* h1, const void* W2, const float* b2, void* xn,
                     const int64_t* ids, float drop_p, uint64_t salt1, uint64_t salt2, const uint64_t* seed_base,
                     void* stream);
/* rs_sas_block_out for the LAST block with the SAS head riding in the same kernel (token-local once the BCE
 * divisor c = *divisor or the sum of count_parts[ncount] from rs_sas_block_in_embed is known): per token, after
 * xn: f = LN_last(xn) [saved], pl/nl = <f, E[pos]>/<f, E[neg]>, dpl = (sigmoid(pl)-1)/c, dnl = sigmoid(nl)/c on
 * pos != 0 [saved], dx = LN_last'(xn, dpl E[pos] + dnl E[neg]) [saved, bf16].  Per workgroup
 * (rs_sas_block_grid(M) of them): lnpart[b][2][d] LN affine partials, part[b][3] BCE partials (sum softplus(-pl),
 * sum softplus(nl), count) for rs_wgrad_grouped_pos_stats.  RS_ERR_UNSUPPORTED for d not in {64, 128}. */
int64_t rs_sas_block_grid(int64_t M);
int rs_sas_block_out_head(int64_t M, int64_t d, const void* o, const void* Q, const void* Wo, const float* bo,
                          void* x1, const float* ln_w, const float* ln_b, float eps, void* z, float* mean, float* rstd,
                          const void* W1, const float* b1, void* h1, const void* W2, const float* b2, void* xn,
                          const int64_t* ids, float drop_p, uint64_t salt1, uint64_t salt2,
                          const uint64_t* seed_base, const void* E, const int64_t* pos, const int64_t* neg,
                          const float* lnl_w, const float* lnl_b, const int* count_parts, int64_t ncount,
                          const float* divisor, void* f, float* pl, float* nl, float* dpl, float* dnl, void* dx,
                          float* lnpart, float* part, void* stream);

/* Union-of-touched-rows exchange of an embedding-table gradient (sparse_rows.hip; data parallel,
 * replaces the dense all-reduce of the token / item table gradient -- the reference has no
 * multi-GPU path, BS/trainers/base.py:32-34).  rs_touched_rows: flags[v] = (v occurs in ids[0..n)),
 * index[v] = rank of v among flagged rows (ascending) or -1, *count = flagged rows; flags/index int32[rows],
 * ws int32[rs_touched_rows_ws_numel(rows)].  rs_rows_pack: compact[index[v]][:] = src[v][:] for flagged v,
 * compact rows [*count, cap) zeroed (cap >= *count).  rs_rows_unpack: dst[v][:] = compact[index[v]][:].
 * fp32 rows of d (d % 4 == 0, 16-B aligned). */
int64_t rs_touched_rows_ws_numel(int64_t rows);
int rs_touched_rows(const int64_t* ids, int64_t n, int64_t rows, int32_t* flags, int32_t* index, int32_t* count,
                    int32_t* ws, void* stream);
int rs_rows_pack(const float* src, int64_t rows, int64_t d, const int32_t* index, const int32_t* count,
                 float* compact, int64_t cap, void* stream);
int rs_rows_unpack(float* dst, int64_t rows, int64_t d, const int32_t* index, const float* compact, void* stream);

/* Number of LayerNorm affine partial sets the two backward kernels below write for M token rows
 * (one per workgroup). */
int64_t rs_sas_block_parts(int64_t M);
/* Backward of rs_sas_block_out (sas.py:75-84 reversed):
 *   dzres = dxn*(ids!=0); dy2 = drop2(dzres) [out]; da1 = relu'(h1)*drop1(dy2 W2) [out];
 *   dz = da1 W1 + dzres; dx1 = LN2'(x1, dz) [out]; dout = dx1 Wo [out];
 *   part[b][0][:] / part[b][1][:] = LN2 dgamma / dbeta partial set b (part >= 2*d*rs_sas_block_parts(M)
 *   floats; sum them with rs_reduce_segments / rs_wgrad_grouped: stride 2d, splits rs_sas_block_parts(M)).
 *   W*T are bf16 TRANSPOSED weights ([in][out], rs_transpose_bf16).
 * Replaces rs_dropout_rowmask + 3 rs_gemm dgrads + rs_layernorm_bwd of the unfused sequence. */
int rs_sas_block_out_bwd(int64_t M, int64_t d, const void* dxn, const int64_t* ids, const void* h1, const void* x1,
                         const float* mean2, const float* rstd2, const float* ln_w, const void* W2T, const void* W1T,
                         const void* WoT, void* dy2, void* da1, void* dx1, void* dout, float* part, float drop_p,
                         uint64_t salt1, uint64_t salt2, const uint64_t* seed_base, void* stream);
/* rs_sas_block_out_bwd, and with o (the attention output [M][d] bf16, one head) also
 * delta[m] = rowsum(dout[m] * o[m]) -- the attention backward's row term, so rs_attn_bwd (mask_kind |
 * RS_ATTN_DELTA_IN, ws = delta) reads neither o nor recomputes it.  o and delta: both or neither. */
int rs_sas_block_out_bwd_delta(int64_t M, int64_t d, const void* dxn, const int64_t* ids, const void* h1,
                               const void* x1, const float* mean2, const float* rstd2, const float* ln_w,
                               const void* W2T, const void* W1T, const void* WoT, void* dy2, void* da1, void* dx1,
                               void* dout, float* part, float drop_p, uint64_t salt1, uint64_t salt2,
                               const uint64_t* seed_base, const void* o, float* delta, void* stream);
/* Backward of rs_sas_block_in (sas.py:73-76 reversed):
 *   dQ = dq Wq + dx1;  dx = dk Wk + dv Wv + LN1'(x, dQ) [out];  LN1 affine partials -> part (as above).
 * WinT = in_proj_weight^T ([d][3d] bf16). */
int rs_sas_block_in_bwd(int64_t M, int64_t d, const void* dq, const void* dkv, const void* dx1, const void* x,
                        const float* mean1, const float* rstd1, const float* ln_w, const void* WinT, void* dx,
                        float* part, void* stream);
/* Batched bf16 transpose: for m < nmat, desc[6m..6m+5] = {rows, cols, src_off, lds, dst_off, ldd}
 * (elements): dst[dst_off + c*ldd + r] = src[src_off + r*lds + c].  Grid x = max_tiles >= the
 * largest ceil(rows/64)*ceil(cols/64). */
int rs_transpose_bf16(int64_t nmat, const int64_t* desc, int64_t max_tiles, const void* src, void* dst,
                      void* stream);

/* ---- grouped weight gradients (wgrad.hip) ---------------------------------------------------
 * Every Linear / Conv1d(k=1) weight gradient of a backward pass, dW[N][K] += dY^T X and
 * db[N] += colsum(dY) over the M token rows (the autograd accumulation of nn.Linear's backward,
 * BS/models/sas_model/sas.py:8-24,67-84; bert_modules/...), in ONE GEMM launch (problems x output
 * tiles x row splits) followed by ONE deterministic grouped reduction of the split partials.
 * bf16 dY/X (16-byte aligned, ld % 8 == 0), fp32 dW/db accumulated; N, K multiples of 64. */
typedef struct {
  const void* dY; int64_t lddy;   /* [M][N] bf16 */
  const void* X;  int64_t ldx;    /* [M][K] bf16 */
  int64_t N, K;
  float* dW;                      /* [N][K] fp32, += */
  float* db;                      /* [N] fp32, += (or NULL) */
} rs_wgrad_problem;
/* A partial-sum set: out[i] (+)= sum_{z < splits} src[z*stride + i], i < n (n, stride multiples
 * of 4; src/out 16-byte aligned). */
typedef struct {
  const float* src; int64_t stride; int64_t splits; int64_t n; float* out;
} rs_reduce_segment;
/* slab floats needed by rs_wgrad_grouped for these problems (splits = ceil(M / rows_per_split)). */
int64_t rs_wgrad_grouped_slab_numel(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split);
/* output tile edge rs_wgrad_grouped uses for these problems (reads N and K only): 256 when every N and K is a
 * multiple of 256 (the BERT d = 256 layer's weights), else 128 or 64; -1 on bad arguments.  Callers size the row
 * splits by it (about one 256-tile workgroup per CU in total). */
int rs_wgrad_grouped_tile(int nprob, const rs_wgrad_problem* probs);
/* the same with the tile edge capped at max_tile (>= 64) */
int rs_wgrad_grouped_tile_max(int nprob, const rs_wgrad_problem* probs, int max_tile);
/* nprob <= 16 problems; rows_per_split % 64 == 0; the extra segments (<= 64, e.g. LayerNorm
 * affine partials from rs_sas_block_*_bwd) are summed into their outputs (+=) by the same
 * reduction launch.  Returns RS_ERR_UNSUPPORTED for shapes outside the contract. */
int rs_wgrad_grouped(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                     int64_t slab_numel, int nextra, const rs_reduce_segment* extra, void* stream);
/* rs_wgrad_grouped with the output tile edge capped at max_tile (>= 64; rs_wgrad_grouped = 256): a launch that runs
 * beside a streaming kernel (the BERT token table's optimizer update) takes 128-wide tiles -- the 256-wide form's
 * one-workgroup-per-CU LDS-DMA pipeline measured 10x slower sharing the chip with it (cfg5). */
int rs_wgrad_grouped_max(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                         int64_t slab_numel, int nextra, const rs_reduce_segment* extra, int max_tile, void* stream);

/* rs_wgrad_grouped followed by rs_embed_bwd's positional part (bf16, SAS mode 0, scale 1, dpos +=): the
 * positional table's gradient rides in the grouped reduction's launch as T extra workgroups (grad_tail.hip). */
int rs_wgrad_grouped_pos(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                         int64_t slab_numel, int nextra, const rs_reduce_segment* extra, const int64_t* ids,
                         int64_t T, const void* dx, int64_t d, float drop_p, uint64_t salt,
                         const uint64_t* seed_base, float* dpos, void* stream);
/* rs_wgrad_grouped_pos whose reduction launch also carries rs_sas_head_finish (one more workgroup): the SAS
 * head's loss statistics loss_out[0..3] from the head's partials (head_part[head_blocks][3]); aux_out (optional,
 * data parallel): (loss sum, count) written there too -- the all-reduced tail of the gradient buffer. */
int rs_wgrad_grouped_pos_stats(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split,
                               float* slab, int64_t slab_numel, int nextra, const rs_reduce_segment* extra,
                               const int64_t* ids, int64_t T, const void* dx, int64_t d, float drop_p, uint64_t salt,
                               const uint64_t* seed_base, float* dpos, const float* head_part, int64_t head_blocks,
                               const float* head_divisor, float* loss_out, float* aux_out, void* stream);
/* The reduction alone: out (+)= sum over splits, for nseg segments (any number, 64 per launch). */
int rs_reduce_segments(int nseg, const rs_reduce_segment* segs, int accumulate, void* stream);

/* ---- item-table gradient by inverted index (itemgrad.hip) ------------------------------------
 * dtable[v] += sum over the rows keyed v of: source 0  scale * dropout(m*d + c) * dx[m]  (the
 * embedding lookup, sas.py:59-66), source 1  w1[m] * f[m], source 2  w2[m] * f[m]  (the tied
 * sampled logits, sas.py:91-98); key 0 (padding_idx) skipped.  Deterministic: a stable radix
 * sort of the keys, per-key sums in fixed order, one writer per table row, no float atomics.
 * Build the index once per batch (the keys are step inputs), then rs_item_grad after the
 * backward pass.  ws: rs_item_index_ws_bytes() bytes (device). */
int64_t rs_item_index_ws_bytes(int nsrc, int64_t rows, int64_t table_rows, int64_t d);
int rs_item_index_build(int nsrc, const int64_t* keys0, const int64_t* keys1, const int64_t* keys2, int64_t rows,
                        int64_t table_rows, int64_t d, void* ws, int64_t ws_bytes, void* stream);
/* Where the built index lives in ws (for tests and tools): out[0..3] = byte offsets of the sorted keys (u32 [n]),
 * the sorted entries (u32 [n], entry = source * rows + row), start (int [table_rows + 1]), and the sort path
 * (0 counting sort, 1 / 2 one-workgroup LDS radix sort with u32 / u64 words, 3 multi-workgroup radix sort). */
int rs_item_index_layout(int nsrc, int64_t rows, int64_t table_rows, int64_t d, int64_t* out);
/* dx, f: bf16 [rows][d] (d in {64, 128, 256}); w1, w2: fp32 [rows]; dtable fp32 [table_rows][d]. */
int rs_item_grad(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const void* dx, float scale,
                 float drop_p, uint64_t salt, const uint64_t* seed_base, const void* f, const float* w1,
                 const float* w2, float* dtable, void* stream);
/* rs_item_grad that also marks the table rows it writes: row_marks[v] = epoch for every key v of the batch and
 * *epoch_out = epoch, epoch = the low byte of *seed_base (0 without one): the step's stamp for rs_adam_*_marked.
 * row_marks: the rs_adam_*_marked layout over table_rows (stamps: any initial contents). */
int rs_item_grad_marked(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const void* dx,
                        float scale, float drop_p, uint64_t salt, const uint64_t* seed_base, const void* f,
                        const float* w1, const float* w2, float* dtable, uint8_t* row_marks, uint8_t* epoch_out,
                        void* stream);
/* The same for fp32 dx, f (the fp32 parity path, any d): each key run summed in sorted-entry order inside 32-entry
 * chunks, a run crossing chunks as its chunk partials in chunk order (the index workspace's partial region). */
int rs_item_grad_f32(const void* ws, int nsrc, int64_t rows, int64_t table_rows, int64_t d, const float* dx, float scale,
                     float drop_p, uint64_t salt, const uint64_t* seed_base, const float* f, const float* w1,
                     const float* w2, float* dtable, void* stream);

/* ---- fused SASRec output head (head.hip), bf16, d in {64, 128, 256} ----------------------------
 * Forward (sas.py:87-100 + BCE of trainers/sas.py:40-49): f = LN_last(x) [f, mean, rstd saved];
 * pl = <f, E[pos]>, nl = <f, E[neg]> (E = item_emb); part[b][3] = per-64-row-block sums of
 * softplus(-pl), softplus(nl) and the valid count (pos != 0).  part >= 3*ceil(M/64) floats. */
int rs_sas_head_fwd(int64_t M, int64_t d, const void* x, const float* ln_w, const float* ln_b, float eps, void* f,
                    float* mean, float* rstd, const void* E, const int64_t* pos, const int64_t* neg, float* pl,
                    float* nl, float* part, void* stream);
/* Backward: with dpl_in == NULL the BCE gradient is formed here: dpl = (sigmoid(pl)-1)/c,
 * dnl = sigmoid(nl)/c on valid rows, c = *divisor or the forward's valid count, written to
 * dpl/dnl, and out[0..3] = {loss sum, count, mean loss (as rs_bce_fwd), neg-term sum}; with
 * dpl_in/dnl_in given (autograd) those are used.  Then df = dpl E[pos] + dnl E[neg] and
 * dx = LN'(x, df) (bf16); lnpart[b][2][d] = LN affine partials (reduce with rs_reduce_segments).
 * The item-table gradient of the logits is left to rs_item_grad. */
int rs_sas_head_bwd(int64_t M, int64_t d, const float* part, const float* divisor, float* out, const float* pl,
                    const float* nl, const float* dpl_in, const float* dnl_in, float* dpl, float* dnl,
                    const int64_t* pos, const int64_t* neg, const void* E, const void* x, const float* ln_w,
                    const float* mean, const float* rstd, void* dx, float* lnpart, void* stream);
/* out[0..3] from a head's BCE partials part[nblk][3] exactly as rs_sas_head_bwd forms them (one workgroup; the
 * unfused form of rs_wgrad_grouped_pos_stats' statistics). */
int rs_sas_head_finish(int64_t nblk, const float* part, const float* divisor, float* out, void* stream);

/* ---- on-device SAS sampler and ranking metrics (sampler.hip) ----------------------------------
 * rs_sas_sample: one training batch as WarpSampler's workers build it (BS/dataloaders/sas.py:65-91):
 * per row a uniform user, its last max_len items, seq/pos = the window shifted by one, left padded
 * with 0, neg = uniform draws over {0..item_num} minus the window's items.  Histories are a CSR pair
 * (user_offsets[n_users+1], user_items).  *seed_base is advanced first (device counter; graph-
 * capturable); salt separates samplers.  seq/pos/neg: int64 [batch][max_len]; max_len <= 512. */
int rs_sas_sample(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t item_num,
                  int64_t batch, int64_t max_len, uint64_t* seed_base, uint64_t salt, int64_t* seq, int64_t* pos,
                  int64_t* neg, void* stream);
/* rs_bert_mask: one BERT4Rec training batch as BertTrainDataset builds it (BS/dataloaders/bert.py:77-110):
 * row b's user = perm[(cursor*batch + b) mod n_users] (perm nullable = identity), its last max_len items
 * cloze-masked (prob mask_prob, a double: the reference's Python float; then 80 % [MASK] = num_items+1, 10 % a uniform item, 10 % kept;
 * label = the item, 0 elsewhere), left padded.  state[2] = {step seed, cursor} on the device, both
 * advanced by 1 before sampling (graph-capturable; reset state[1] to 0 at an epoch start). */
int rs_bert_mask(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t num_items,
                 int64_t batch, int64_t max_len, double mask_prob, const int64_t* perm, uint64_t* state, uint64_t salt,
                 int64_t* tokens, int64_t* labels, void* stream);
/* The same two samplers, also recording the draws each row consumed (tests replay the reference's construction
 * on them, oracle/sampling.py).  SAS: draws int64 [batch][1 + max_len*256] = {user, then per position the 256
 * candidate negatives the rejection loop may try, in draw order (-1 where the position draws none)}.  BERT: draws int64 [batch][1 + 2*max_len]
 * = {user, then per position (k, item): the masking uniform is k / 2^24, the replacement item is item; -1 on
 * padding}. */
int rs_sas_sample_draws(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t item_num,
                        int64_t batch, int64_t max_len, uint64_t* seed_base, uint64_t salt, int64_t* seq, int64_t* pos,
                        int64_t* neg, int64_t* draws, void* stream);
int rs_bert_mask_draws(const int64_t* user_offsets, const int64_t* user_items, int64_t n_users, int64_t num_items,
                       int64_t batch, int64_t max_len, double mask_prob, const int64_t* perm, uint64_t* state,
                       uint64_t salt, int64_t* tokens, int64_t* labels, int64_t* draws, void* stream);

/* rs_rank_metrics: recalls_ndcgs_and_mrr_for_ks (BS/trainers/utils.py:28-57) over scores/labels
 * fp32 [rows][cands] (labels 0/1 weights), ks: device int[nk] (nk <= 8).  out[3*q + {0,1,2}] =
 * mean Recall@k, NDCG@k, MRR@k for ks[q]; ws >= 3*nk*rows floats.  Ranks follow a stable
 * descending sort (ties by candidate index). */
int rs_rank_metrics(const float* scores, const float* labels, int64_t rows, int64_t cands, int nk, const int* ks,
                    float* ws, float* out, void* stream);

/* ABI version of this header/library pair. */
int rs_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
