// The SAS backward's gradient tail: rs_wgrad_grouped_pos(_stats) = the grouped weight gradients (wgrad.hip) with
// the positional table's gradient (embedding.hip, BS/models/sas_model/sas.py:63) and the SAS head's loss statistics
// (head.hip, BS/trainers/sas.py:49) riding in the grouped reduction's launch -- same arithmetic in the same order,
// bit for bit, as the functions one after the other (their fallback when the shapes do not fit the fused form).
// The item table's gradient (itemgrad.hip, rs_item_grad) runs beside it on the step's side queue.
#include "wgrad.hip"
#include "itemgrad.hip"
#include "embedding.hip"
#include "head.hip"

namespace gt {

// the grouped slab reduction AND the positional table's gradient (rs_embed_bwd's positional part, SAS mode) AND,
// optionally, the SAS head's loss statistics (head_stats): workgroup 0 forms those when hs.out, workgroups
// [h, h + T_) sum one position each, the next rblk reduce
struct HeadStats {
  int nblk;
  const float* part;
  const float* divisor;
  float* out;
  float* aux;   // optional second copy of (loss sum, count)
};
__global__ __launch_bounds__(256) void reduce_pos_kernel(wg::RArgs r, int rblk, int cols, const int64_t* ids,
                                                         int64_t rows, int64_t T_, const __bf16* dx, int64_t d,
                                                         float drop_p, uint64_t salt, const uint64_t* seed_base,
                                                         float* dpos, HeadStats hs) {
  KStampEnd stamp_(r.ks);
  __shared__ float4 red[wg::RED_G][wg::RED_C];
  const int h = hs.out ? 1 : 0;
  if (h && blockIdx.x == 0) {
    static_assert(sizeof(red) >= 3 * 256 * sizeof(float), "head_stats scratch");
    hd::head_stats(hs.nblk, hs.part, hs.divisor, hs.out, reinterpret_cast<float(*)[256]>(&red[0][0]), hs.aux);
    return;
  }
  // the positions' workgroups (long: a 128-row column sum each) are dispatched first, the many short
  // reduction workgroups fill the CUs around them
  if ((int64_t)blockIdx.x - h < T_) {
    embed_pos_body<__bf16, 16, 256>(ids, rows, T_, dx, d, 0, drop_p, salt, seed_base, dpos, 1, blockIdx.x - h);
  } else {
    const int b = (int)(blockIdx.x - h - T_);
    if (cols) wg::reduce_cols_block(r, b);
    else wg::reduce_any_block(r, b, red);
  }
}

}  // namespace gt

extern "C" {

int rs_wgrad_grouped_pos(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                         int64_t slab_numel, int nextra, const rs_reduce_segment* extra, const int64_t* ids,
                         int64_t T_, const void* dx, int64_t d, float drop_p, uint64_t salt,
                         const uint64_t* seed_base, float* dpos, void* stream) {
  return rs_wgrad_grouped_pos_stats(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, ids, T_, dx, d,
                                    drop_p, salt, seed_base, dpos, nullptr, 0, nullptr, nullptr, nullptr, stream);
}

int rs_wgrad_grouped_pos_stats(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split,
                               float* slab, int64_t slab_numel, int nextra, const rs_reduce_segment* extra,
                               const int64_t* ids, int64_t T_, const void* dx, int64_t d, float drop_p, uint64_t salt,
                               const uint64_t* seed_base, float* dpos, const float* head_part, int64_t head_blocks,
                               const float* head_divisor, float* loss_out, float* aux_out, void* stream) {
  if (!ids || !dx || !dpos || T_ <= 0 || M % T_ || !head_part != !loss_out || (loss_out && head_blocks <= 0))
    return RS_ERR_ARG;
  wg::Args a;
  int T, ns;
  rs_reduce_segment segs[2 * wg::MAXP + wg::MAXS];
  if (int e = wgrad_group_args(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, a, T, segs, ns, 256))
    return e;
  const bool vec = d % 8 == 0 && d / 8 <= 16 && ((uintptr_t)dx % 16) == 0;
  if (ns > wg::MAXS || !vec) {   // unfused: the functions one after the other
    if (int e = rs_wgrad_grouped(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, stream)) return e;
    if (int e = rs_embed_bwd(RS_DTYPE_BF16, 0, ids, M, T_, dx, d, 1.f, drop_p, salt, seed_base, nullptr, dpos, 1,
                             stream))
      return e;
    if (!loss_out) return 0;
    if (int e = rs_sas_head_finish(head_blocks, head_part, head_divisor, loss_out, stream)) return e;
    return aux_out ? (int)hipMemcpyAsync(aux_out, loss_out, 2 * sizeof(float), hipMemcpyDeviceToDevice,
                                         (hipStream_t)stream)
                   : 0;
  }
  wg::RArgs r;
  int rblk;
  bool cols;
  if (int e = reduce_args(ns, segs, 1, r, rblk, cols)) return e;
  a.ks = kstamp_next(RS_STAMP_WGRAD_GROUPED);
  r.ks = a.ks;
  hipStream_t s = (hipStream_t)stream;
  wg::launch_group(a, T, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const gt::HeadStats hs{(int)head_blocks, head_part, head_divisor, loss_out, aux_out};
  hipLaunchKernelGGL(gt::reduce_pos_kernel, dim3((unsigned)(rblk + T_ + (loss_out ? 1 : 0))), dim3(256), 0, s, r, rblk,
                     (int)cols, ids, M, T_, (const __bf16*)dx, d, drop_p, salt, seed_base, dpos, hs);
  return (int)hipGetLastError();
}

}  // extern "C"
