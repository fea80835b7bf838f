// The backward's gradient tail in two launches on ONE queue instead of four on two.
//
//   rs_wgrad_grouped_items = rs_wgrad_grouped + rs_item_grad:
//     launch 1: the grouped weight-gradient tiles (wgrad.hip) AND the item-gradient chunks (itemgrad.hip) --
//               workgroups [0, n_w) are weight-gradient ones, dispatched first, the rest item chunks, which
//               fill the CUs beside them (both latency-bound; one LDS union sized for the larger)
//     launch 2: the grouped slab reduction AND the item-gradient span pass (keys crossing chunks)
//   Same arithmetic in the same order, bit for bit, as the two functions called one after the other; on one
//   queue it replaces a cross-queue fork + join of the step graph (~6 us of idle each, measured).
#include "wgrad.hip"
#include "itemgrad.hip"
#include "embedding.hip"
#include "head.hip"

namespace gt {

template <int T, int D>
union TailLds {
  __bf16 w[wg::group_lds_bytes<T>() / sizeof(__bf16)];
  ig::ChunkLds<D> c;
};

template <int T, int D>
__global__ __launch_bounds__(256, 2) void wgrad_items_kernel(wg::Args a, ig::GradArgs g, unsigned nw) {
  KStampBegin stamp_(a.ks);
  __shared__ __attribute__((aligned(16))) TailLds<T, D> L;
  if (blockIdx.x < nw) wg::group_tile<T>(a, blockIdx.x, nw, L.w);
  else ig::item_chunk<D>(g, (int64_t)(blockIdx.x - nw), L.c);
}

template <int D>
__global__ __launch_bounds__(256) void reduce_span_kernel(wg::RArgs r, int rblk, int cols, ig::GradArgs g,
                                                          int64_t nchunks) {
  KStampEnd stamp_(r.ks);
  __shared__ float4 red[wg::RED_G][wg::RED_C];
  if ((int)blockIdx.x < rblk) {
    if (cols) wg::reduce_cols_block(r, blockIdx.x);
    else wg::reduce_any_block(r, blockIdx.x, red);
  } else {
    ig::item_span<D>(g, nchunks, (int64_t)blockIdx.x - rblk);
  }
}

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

template <int T, int D>
static hipError_t launch(const wg::Args& a, const ig::GradArgs& g, const wg::RArgs& r, int rblk, bool cols,
                         int64_t nchunks, hipStream_t s) {
  const unsigned nw = (unsigned)(a.ntiles * a.splits);
  hipLaunchKernelGGL((wgrad_items_kernel<T, D>), dim3(nw + (unsigned)nchunks), dim3(256), 0, s, a, g, nw);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((reduce_span_kernel<D>), dim3((unsigned)(rblk + cdiv(nchunks, 4))), dim3(256), 0, s, r, rblk,
                     (int)cols, g, nchunks);
  return hipGetLastError();
}

}  // namespace gt

extern "C" {

int rs_wgrad_grouped_items(int nprob, const rs_wgrad_problem* probs, int64_t M, int64_t rows_per_split, float* slab,
                           int64_t slab_numel, int nextra, const rs_reduce_segment* extra, const void* ws, int nsrc,
                           int64_t rows, int64_t table_rows, int64_t d, const void* dx, float scale, float drop_p,
                           uint64_t salt, const uint64_t* seed_base, const void* f, const float* w1, const float* w2,
                           float* dtable, void* stream) {
  wg::Args a;
  int T, ns;
  rs_reduce_segment segs[2 * wg::MAXP + wg::MAXS];
  if (int e = wgrad_group_args(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, a, T, segs, ns))
    return e;
  ig::GradArgs g;
  ig::Layout L;
  if (int e = item_grad_args(ws, nsrc, rows, table_rows, d, dx, scale, drop_p, salt, seed_base, f, w1, w2, dtable, g,
                             L))
    return e;
  if (ns > wg::MAXS || (d != 64 && d != 128 && d != 256)) {   // more than one reduction launch: unfused
    if (int e = rs_wgrad_grouped(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, stream)) return e;
    return rs_item_grad(ws, nsrc, rows, table_rows, d, dx, scale, drop_p, salt, seed_base, f, w1, w2, dtable, stream);
  }
  wg::RArgs r;
  int rblk;
  bool cols;
  if (int e = reduce_args(ns, segs, 1, r, rblk, cols)) return e;
  a.ks = kstamp_next(RS_STAMP_WGRAD_GROUPED);
  r.ks = a.ks;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (T == 128)
    e = d == 64 ? gt::launch<128, 64>(a, g, r, rblk, cols, L.nchunks, s)
      : d == 128 ? gt::launch<128, 128>(a, g, r, rblk, cols, L.nchunks, s)
                 : gt::launch<128, 256>(a, g, r, rblk, cols, L.nchunks, s);
  else
    e = d == 64 ? gt::launch<64, 64>(a, g, r, rblk, cols, L.nchunks, s)
      : d == 128 ? gt::launch<64, 128>(a, g, r, rblk, cols, L.nchunks, s)
                 : gt::launch<64, 256>(a, g, r, rblk, cols, L.nchunks, s);
  return (int)e;
}

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
  if (int e = wgrad_group_args(nprob, probs, M, rows_per_split, slab, slab_numel, nextra, extra, a, T, segs, ns))
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
  const dim3 grid((unsigned)(a.ntiles * a.splits));
  if (T == 128) hipLaunchKernelGGL(wg::wgrad_group_kernel<128>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wg::wgrad_group_kernel<64>, grid, dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const gt::HeadStats hs{(int)head_blocks, head_part, head_divisor, loss_out, aux_out};
  hipLaunchKernelGGL(gt::reduce_pos_kernel, dim3((unsigned)(rblk + T_ + (loss_out ? 1 : 0))), dim3(256), 0, s, r, rblk,
                     (int)cols, ids, M, T_, (const __bf16*)dx, d, drop_p, salt, seed_base, dpos, hs);
  return (int)hipGetLastError();
}

}  // extern "C"
