"""Thin tensor-level wrappers over the C ABI (librecsys_hip.so).

Every function launches HIP kernels on the current torch stream and returns
nothing; outputs are caller-allocated tensors (the C ABI allocates nothing).
2-D tensors are passed with their row stride as the leading dimension.
"""
import ctypes as C
import os

import torch

from . import _lib
from ._lib import BF16, F32, Epilogue, call, ptr, stream

ACT_NONE, ACT_RELU, ACT_GELU, ACT_RELU_BWD, ACT_GELU_BWD = (
    _lib.ACT_NONE, _lib.ACT_RELU, _lib.ACT_GELU, _lib.ACT_RELU_BWD, _lib.ACT_GELU_BWD)


# ------------------------------------------------------------------ kernel stamps
STAMP_KINDS = {1: "attn_bwd", 2: "wgrad_grouped", 3: "vocab_ce_fwd"}


def kernel_stamps(buf, step, kinds=()):
    """Enable (buf: int64 device tensor, step: the optimizer's float64 device step count, kinds: names from
    STAMP_KINDS) or disable (None, None) the in-kernel begin/end stamps of rs_attn_bwd / rs_wgrad_grouped
    launches (layout in include/recsys_hip.h).  Launches captured into a graph while enabled keep stamping
    on every replay."""
    mask = sum(1 << k for k, n in STAMP_KINDS.items() if n in kinds)
    call("rs_kernel_stamps", ptr(buf), ptr(step), mask)


def read_kernel_stamps(buf, khz):
    """[(mark, step slot, µs)] of every complete record in a stamp buffer (after the stamped work finished)."""
    import numpy as np
    h = buf.cpu().numpy().view(np.uint64)
    steps, marks, W = int(h[1]), int(h[2]), int(h[3])
    rec = h[4:4 + steps * marks * (1 + W)].reshape(steps, marks, 1 + W)
    out = []
    for st in range(steps):
        for m in range(marks):
            b, e = int(rec[st, m, 0]), int(rec[st, m, 1:].max())
            if b and e > b:
                out.append((m, st, (e - b) / khz * 1e3))
    return out


def kernel_stamp_kinds():
    """Kind name of every mark handed out since the last kernel_stamps(buf, step), in mark order."""
    n = _lib.lib().rs_kernel_stamp_count()
    arr = (C.c_int * max(n, 1))()
    call("rs_kernel_stamp_kinds", arr, n)
    return [STAMP_KINDS.get(arr[i], "?") for i in range(n)]


# ------------------------------------------------------------------ HIP-event launch timing
_EVENTS = {"kinds": (), "pairs": []}


def event_timing(kinds=()):
    """Bracket every launch of the named kinds (STAMP_KINDS names) with a pair of timing HIP events on the current
    stream (eager launches; bench.py's roofline leg).  Returns the list collecting (kind, begin event, end event);
    kinds=() disables."""
    _EVENTS["kinds"], _EVENTS["pairs"] = tuple(kinds), []
    return _EVENTS["pairs"]


def _ev_begin(kind):
    if kind not in _EVENTS["kinds"]:
        return None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _EVENTS["pairs"].append((kind, e0, e1))
    return e1


def _ev_end(e1):
    if e1 is not None:
        e1.record()


def wall_clock_khz():
    k = C.c_int()
    call("rs_wall_clock_khz", C.byref(k))
    return k.value


def dtype_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


def ld(t):
    return t.stride(0) if t.dim() == 2 else t.shape[-1]


def epilogue(bias=None, alpha=1.0, act=ACT_NONE, aux=None, aux_out=None, drop_p=0.0, drop_seed=0,
             seed_base=None, drop_ld=0, resid=None, rowmask_ids=None, accumulate=False, post_drop_p=0.0,
             post_drop_seed=0, rows_dev=None):
    e = Epilogue()
    e.bias = ptr(bias)
    e.alpha = alpha
    e.act = act
    e.aux = ptr(aux)
    e.aux_out = ptr(aux_out)
    a = aux if aux is not None else aux_out
    e.ldaux = ld(a) if a is not None else 0
    e.drop_p = drop_p
    e.drop_seed = drop_seed
    e.seed_base = ptr(seed_base)
    e.drop_ld = drop_ld
    e.resid = ptr(resid)
    e.ldres = ld(resid) if resid is not None else 0
    e.rowmask_ids = ptr(rowmask_ids)
    e.accumulate = 1 if accumulate else 0
    e.post_drop_p = post_drop_p
    e.post_drop_seed = post_drop_seed
    e.rows_dev = ptr(rows_dev)
    return e


def gemm(A, B, Cout, M, N, K, a_kmajor=False, b_kmajor=False, epi=None, split_k=1, slab=None):
    """Cout[M,N] = epi(A . B^T) with the storage conventions of rs_gemm (C may be fp32 for bf16 A/B)."""
    assert A.dtype == B.dtype, "A and B must share the compute dtype"
    call("rs_gemm", dtype_code(A), int(a_kmajor), int(b_kmajor), M, N, K, ptr(A), ld(A), ptr(B), ld(B),
         ptr(Cout), ld(Cout), int(Cout.dtype == torch.float32),
         C.byref(epi) if epi is not None else None, split_k, ptr(slab), stream())


def linear_fwd(X, W, Y, bias=None, **epi_kw):
    """Y = X W^T (+ fused epilogue).  X [M,K], W [N,K], Y [M,N]."""
    M, K = X.shape
    N = W.shape[0]
    gemm(X, W, Y, M, N, K, False, False, epilogue(bias=bias, **epi_kw))


RS_ERR_UNSUPPORTED = 1002


def linear_fwd_ln(X, gamma, beta, eps, W, Y, h=None, mean=None, rinv=None, bias=None, **epi_kw):
    """Y = epi(LN(X) W^T) with the BERT LayerNorm (variant 1) in the GEMM's prologue (rs_gemm_ln); h / mean / rinv
    receive what rs_layernorm_fwd would write.  Returns False (nothing launched) when the shape or epilogue is not
    one the fused kernel covers -- the caller then runs layernorm_fwd + linear_fwd."""
    M, K = X.shape
    N = W.shape[0]
    e = epilogue(bias=bias, **epi_kw)
    rc = _lib.lib().rs_gemm_ln(M, N, K, ptr(X), ld(X), ptr(gamma), ptr(beta), eps, ptr(W), ld(W), ptr(Y), ld(Y),
                               C.byref(e), ptr(h), ld(h) if h is not None else 0, ptr(mean), ptr(rinv), stream())
    if rc == RS_ERR_UNSUPPORTED:
        return False
    if rc != 0:
        raise RuntimeError(f"rs_gemm_ln failed with code {rc}")
    return True


def linear_dgrad(dY, W, dX, **epi_kw):
    """dX = dY W (+ epilogue).  dY [M,N], W [N,K], dX [M,K]."""
    M, N = dY.shape
    K = W.shape[1]
    gemm(dY, W, dX, M, K, N, False, True, epilogue(**epi_kw))


def linear_dgrad_splitk(dY, W, dX, slab, splits, acc_f32=None, rows_dev=None):
    """dX = dY W for a long contraction (dY [M,N] with N >> M, e.g. the vocabulary gradient):
    split-K into fp32 slabs (rs_gemm with split_k) + one deterministic reduce (+ cast when dX is
    bf16, through ``acc_f32`` [M,K] fp32)."""
    M, N = dY.shape
    K = W.shape[1]
    assert slab.numel() >= splits * M * K
    gemm(dY, W, slab, M, K, N, False, True, epilogue(rows_dev=rows_dev), split_k=splits, slab=slab)
    out = dX if dX.dtype == torch.float32 else acc_f32
    assert out is not None and out.is_contiguous() and out.shape == (M, K)
    call("rs_reduce_slabs", ptr(slab), splits, M * K, ptr(out), 0, stream())
    if out is not dX:
        cast_bf16(out, dX)


def split_for(M_tok, n_out, k_in):
    """Split-K factor of the weight-gradient GEMM: ~1024 blocks of 64x64 output tiles, >= 256 rows each."""
    tiles = -(-n_out // 64) * -(-k_in // 64)
    return int(max(1, min(-(-1024 // tiles), -(-M_tok // 256))))


def wgrad_slab_numel(M_tok, n_out, k_in):
    return split_for(M_tok, n_out, k_in) * (n_out * k_in + n_out)


def linear_wgrad(dY, X, dW, slab, db=None, split_k=None, accumulate=True, rows_dev=None):
    """dW [N,K] (+)= dY^T X and db [N] (+)= colsum(dY) over M token rows (rs_linear_wgrad)."""
    M, N = dY.shape
    K = X.shape[1]
    s = split_k or split_for(M, N, K)
    direct = s == 1 and dY.dtype == torch.bfloat16 and K % 8 == 0 and dW.data_ptr() % 16 == 0  # no slab used
    assert direct or slab.numel() >= s * (N * K + N), "slab workspace too small"
    assert dY.dtype == X.dtype
    call("rs_linear_wgrad", dtype_code(dY), M, N, K, ptr(dY), ld(dY), ptr(X), ld(X), ptr(dW), ptr(db),
         int(accumulate), s, ptr(slab), ptr(rows_dev), stream())


def colsum(X, out, ws, accumulate=True):
    M, N = X.shape
    call("rs_colsum", dtype_code(X), ptr(X), M, N, ld(X), ptr(ws), ptr(out), int(accumulate), stream())


def layernorm_fwd(X, gamma, beta, eps, Y, mean, rinv, variant):
    M, d = X.shape
    call("rs_layernorm_fwd", dtype_code(X), variant, ptr(X), ld(X), M, d, ptr(gamma), ptr(beta), eps,
         ptr(Y), ld(Y), ptr(mean), ptr(rinv), stream())


def layernorm_bwd_nparts(X):
    """Partial count layernorm_bwd leaves in ws when called with dgamma = dbeta = None (0: not deferrable)."""
    M, d = X.shape
    ok = X.data_ptr() % 16 == 0 and ld(X) % (8 if X.dtype == torch.bfloat16 else 4) == 0
    return int(_lib.lib().rs_layernorm_bwd_nparts(dtype_code(X), M, d)) if ok else 0


def layernorm_bwd_drop(X, dY, gamma, mean, rinv, eps, dX, dgamma, dbeta, ws, variant, drop_p, salt1, salt2, seed_base,
                       out1, out2=None, accumulate=False):
    """layernorm_bwd, then out1 = drop(dX; salt1) (and out2 = drop(out1; salt2)) in the same launch."""
    M, d = X.shape
    assert out1.shape == (M, d) and out1.is_contiguous() and (out2 is None or out2.is_contiguous())
    call("rs_layernorm_bwd_drop", dtype_code(X), variant, ptr(X), ld(X), ptr(dY), ld(dY), M, d, ptr(gamma),
         ptr(mean), ptr(rinv), eps, ptr(dX), ld(dX), int(accumulate), ptr(dgamma), ptr(dbeta), ptr(ws), drop_p, salt1,
         salt2, ptr(seed_base), ptr(out1), ptr(out2), stream())


def layernorm_bwd(X, dY, gamma, mean, rinv, eps, dX, dgamma, dbeta, ws, variant, accumulate=False):
    M, d = X.shape
    call("rs_layernorm_bwd", dtype_code(X), variant, ptr(X), ld(X), ptr(dY), ld(dY), M, d, ptr(gamma),
         ptr(mean), ptr(rinv), eps, ptr(dX), ld(dX), int(accumulate), ptr(dgamma), ptr(dbeta), ptr(ws), stream())


def embed_fwd(mode, ids, T, table, pos, scale, drop_p, seed, seed_base, out):
    rows = ids.numel()
    d = table.shape[1]
    call("rs_embed_fwd", dtype_code(table), mode, ptr(ids), rows, T, ptr(table), ptr(pos), d, scale, drop_p,
         seed, ptr(seed_base), ptr(out), stream())


def embed_bwd(mode, ids, T, dx, scale, drop_p, seed, seed_base, dtable, dpos, accumulate_pos=True):
    rows = ids.numel()
    d = dx.shape[-1]
    call("rs_embed_bwd", dtype_code(dx), mode, ptr(ids), rows, T, ptr(dx), d, scale, drop_p, seed,
         ptr(seed_base), ptr(dtable), ptr(dpos), int(accumulate_pos), stream())


def attn_fwd(B, T, H, Dh, q, k, v, o, lse, scale, mask_kind, ids, drop_p, seed, seed_base):
    call("rs_attn_fwd", dtype_code(q), B, T, H, Dh, ptr(q), ld(q), ptr(k), ld(k), ptr(v), ld(v), ptr(o), ld(o),
         ptr(lse), scale, mask_kind, ptr(ids), drop_p, seed, ptr(seed_base), stream())


RS_ATTN_DELTA_IN = 0x100


def attn_row_delta(B, T, H, Dh, do, o, delta):
    """delta[(b*H+h)*T + t] = sum over head h's columns of do * o (the input of attn_bwd(delta_in=True))."""
    call("rs_attn_row_delta", dtype_code(do), B, T, H, Dh, ptr(do), ld(do), ptr(o), ld(o), ptr(delta), stream())


def attn_bwd(B, T, H, Dh, q, k, v, o, do, lse, dq, dk, dv, scale, mask_kind, ids, drop_p, seed, seed_base, ws,
             delta_in=False):
    """delta_in: ws already holds delta = rowsum(dO * O) per (b, h, t) (sas_block_out_bwd with o=)."""
    mk = mask_kind | (RS_ATTN_DELTA_IN if delta_in else 0)
    ev = _ev_begin("attn_bwd")
    call("rs_attn_bwd", dtype_code(q), B, T, H, Dh, ptr(q), ld(q), ptr(k), ld(k), ptr(v), ld(v), ptr(o), ld(o),
         ptr(do), ld(do), ptr(lse), ptr(dq), ld(dq), ptr(dk), ld(dk), ptr(dv), ld(dv), scale, mk, ptr(ids),
         drop_p, seed, ptr(seed_base), ptr(ws), stream())
    _ev_end(ev)


def sampled_logits_fwd(f, E, pos, neg, pl, nl):
    M, d = f.shape
    call("rs_sampled_logits_fwd", dtype_code(f), ptr(f), M, d, ptr(E), ptr(pos), ptr(neg), ptr(pl), ptr(nl),
         stream())


def sampled_logits_bwd(f, E, pos, neg, dpl, dnl, df, dE, accumulate_df=False):
    M, d = f.shape
    call("rs_sampled_logits_bwd", dtype_code(f), ptr(f), M, d, ptr(E), ptr(pos), ptr(neg), ptr(dpl), ptr(dnl),
         ptr(df), int(accumulate_df), ptr(dE), stream())


def bce_fwd(pl, nl, pos, ws, out, count_override=None):
    call("rs_bce_fwd", ptr(pl), ptr(nl), ptr(pos), pl.numel(), ptr(count_override), ptr(ws), ptr(out), stream())


def bce_bwd(pl, nl, pos, count, dloss, dpl, dnl):
    call("rs_bce_bwd", ptr(pl), ptr(nl), ptr(pos), pl.numel(), ptr(count), ptr(dloss), ptr(dpl), ptr(dnl),
         stream())


def ce_fwd(logits, labels, ws, out, count_override=None, rows_dev=None):
    R, V1 = logits.shape
    call("rs_ce_fwd", ptr(logits), R, V1, ld(logits), ptr(labels), ptr(count_override), ptr(ws), ptr(out),
         ptr(rows_dev), stream())


def ce_bwd(logits, labels, count, dloss, ws, dlogits, rows_dev=None):
    R, V1 = logits.shape
    call("rs_ce_bwd", dtype_code(dlogits), ptr(logits), R, V1, ld(logits), ptr(labels), ptr(count), ptr(dloss),
         ptr(ws), ptr(dlogits), ld(dlogits), ptr(rows_dev), stream())


def compact_rows(labels, cap, idx, rank, count):
    call("rs_compact_rows", ptr(labels), labels.numel(), cap, ptr(idx), ptr(rank), ptr(count), stream())


def gather_rows(src, idx, count, cap, dst, labels=None, lab_out=None):
    d = src.shape[1]
    call("rs_gather_rows", dtype_code(src), ptr(src), ld(src), d, ptr(idx), ptr(count), cap, ptr(dst), ld(dst),
         ptr(labels), ptr(lab_out), stream())


def scatter_rows(src, rank, dst):
    n, d = dst.shape
    call("rs_scatter_rows", dtype_code(src), ptr(src), ld(src), d, ptr(rank), n, ptr(dst), ld(dst), stream())


def reduce_slabs(slab, splits, out, accumulate=False):
    """out (+)= sum over the `splits` leading slabs of slab (fixed order)."""
    n = out.numel()
    call("rs_reduce_slabs", ptr(slab), splits, n, ptr(out), int(accumulate), stream())


def splitk_scatter_rows(slab, splits, cap, rank, dst):
    """dst[r] = sum_z slab[z][rank[r]] (0 where rank < 0): split-K reduce + cast + scatter, one launch."""
    n, d = dst.shape
    call("rs_splitk_scatter_rows", dtype_code(dst), ptr(slab), splits, cap, d, ptr(rank), n, ptr(dst), ld(dst),
         stream())


def adam_prepare(state, hyper, grad_divisor=None, seed_base=None):
    call("rs_adam_prepare", ptr(state), ptr(hyper), ptr(grad_divisor), ptr(seed_base), stream())


def row_marks_bytes(rows):
    """Size of a row-marks array (rs_item_grad_marked / rs_adam_*_marked): the rows' stamps, padding to 16 B + 16
    (the sweep's scalar mark loads run past the last row) and a 1 KB zero tail (the unstamped rows' gradient
    loads read it).  Allocate zeroed, 16-byte aligned."""
    return (rows + 15) // 16 * 16 + 16 + 1024


def adam_step(p, g, m, v, p_bf16, state, hyper, zero_grad=False, max_wg=None, marks=None):
    """marks: (row_marks u8, epoch u8, moff, rows, dshift) of a marked table inside this range (rs_adam_step_marked)."""
    if marks is not None:
        rm, ep, moff, rows, dshift = marks
        call("rs_adam_step_marked", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), ptr(state), ptr(hyper),
             int(zero_grad), int(max_wg or 8192), ptr(rm), ptr(ep), int(moff), int(rows), int(dshift), stream())
        return
    if max_wg:
        call("rs_adam_step_wg", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), ptr(state), ptr(hyper),
             int(zero_grad), int(max_wg), stream())
        return
    call("rs_adam_step", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), ptr(state), ptr(hyper),
         int(zero_grad), stream())


def adam_prepare_step(p, g, m, v, p_bf16, state, hyper, zero_grad=False, grad_divisor=None, seed_base=None,
                      transposed=None, loss_sum=None, loss_out=None, tbase=0, marks=None):
    """adam_prepare + adam_step in one launch (state: double[144]; state[7], state[16 + 16 k] arrival counters).
    transposed: (desc int64 device [n][6] as transpose_bf16's, its host copy, dst bf16 tensor) -- the bf16
    result of those matrices is also written transposed; the descriptors' offsets are flat-buffer elements and
    p[0] is element `tbase` of the flat buffer (every matrix must lie inside [tbase, tbase + p.numel()))."""
    if state.numel() < 144:
        raise ValueError("adam_prepare_step needs the 144-entry optimizer state")
    td, nt, wt = None, 0, None
    if transposed is not None:
        td, host, wt = transposed
        nt = len(host)
        for rows, cols, off, lds, doff, ldd in host:
            if lds % 4 or off % 4 or tbase % 4 or off < tbase or off + rows * lds > tbase + (p.numel() // 4) * 4 \
                    or doff + (cols - 1) * ldd + rows > wt.numel() or rows * lds >= 2 ** 31:
                raise ValueError("adam_prepare_step: transposed matrix outside the buffers or misaligned")
        if p_bf16 is None:
            raise ValueError("adam_prepare_step: transposed copies need the bf16 output")
    if marks is not None:      # a marked table inside the range (rs_adam_prepare_step_marked)
        rm, ep, moff, rows, dshift = marks
        call("rs_adam_prepare_step_marked", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), ptr(state),
             ptr(hyper), int(zero_grad), ptr(grad_divisor), ptr(seed_base), ptr(td), nt, int(tbase), ptr(wt),
             ptr(loss_sum), ptr(loss_out), ptr(rm), ptr(ep), int(moff), int(rows), int(dshift), stream())
        return
    if loss_out is not None:   # + loss_out = loss_sum / grad_divisor in the same launch
        call("rs_adam_prepare_step_loss", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), ptr(state),
             ptr(hyper), int(zero_grad), ptr(grad_divisor), ptr(seed_base), ptr(td), nt, int(tbase), ptr(wt), ptr(loss_sum),
             ptr(loss_out), stream())
        return
    call("rs_adam_prepare_step", p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), ptr(state), ptr(hyper),
         int(zero_grad), ptr(grad_divisor), ptr(seed_base), ptr(td), nt, int(tbase), ptr(wt), stream())


L2_CHUNK = 16384


def l2_chunk_desc(flat, device):
    """rs_l2_penalty's chunk descriptor over a FlatParams buffer: one segment per parameter tensor (its exact
    elements, alignment padding excluded), cut into chunks of at most L2_CHUNK elements.  int64 [n][4]."""
    rows = []
    for n in flat.names:
        lo = flat.offsets[n]
        cnt = 1
        for s in flat.shapes[n]:
            cnt *= s
        first, nch = len(rows), max(1, -(-cnt // L2_CHUNK))
        for k in range(nch):
            rows.append([lo + k * L2_CHUNK, lo + min(cnt, (k + 1) * L2_CHUNK), first, nch])
    return torch.tensor(rows, dtype=torch.int64, device=device)


def l2_penalty(p, g, desc, l2, ws, loss=None, scale=None):
    """loss += l2 * sum ||p_seg||, g += scale * l2 * p / ||p_seg|| (BS/trainers/sas.py:51-52; rs_l2_penalty)."""
    assert ws.numel() >= 2 * desc.shape[0] and ws.dtype == torch.float32   # chunk sums + segment norms
    call("rs_l2_penalty", ptr(p), ptr(g), ptr(desc), desc.shape[0], float(l2), ptr(scale), ptr(ws), ptr(loss),
         stream())


def cast_bf16(src, dst):
    call("rs_cast_bf16", src.numel(), ptr(src), ptr(dst), stream())


def dropout_rowmask(x, drop_p, seed, seed_base, rowmask_ids, out, out_masked=None):
    M, N = x.shape
    call("rs_dropout_rowmask", dtype_code(x), ptr(x), M, N, ld(x), drop_p, seed, ptr(seed_base), N,
         ptr(rowmask_ids), ptr(out), ptr(out_masked), stream())


def dropout2(x, drop_p, salt1, salt2, seed_base, out1, out2):
    """out1 = drop(x; salt1), out2 = drop(out1; salt2): two stacked dropout sites' backward, one pass."""
    M, N = x.shape
    call("rs_dropout2", dtype_code(x), ptr(x), M, N, ld(x), drop_p, salt1, salt2, ptr(seed_base), N, ptr(out1),
         ptr(out2), stream())


# ---- BERT vocabulary head + cross entropy, logits not materialised (vocab_ce.hip) -----------
def vocab_ce_ws_numel(R, V1):
    n = _lib.lib().rs_vocab_ce_ws_numel(R, V1)
    if n < 0:
        raise RuntimeError("rs_vocab_ce_ws_numel: bad arguments")
    return n


def vocab_ce_fwd(h, E, bias, labels, ws, out, rows_dev=None, count_override=None):
    """out[0:3] = (loss sum, labelled count, mean) of CE(h E^T + bias, labels, ignore_index=0); ws keeps
    the row log-sum-exp for vocab_ce_bwd."""
    R, d = h.shape
    V1 = E.shape[0]
    call("rs_vocab_ce_fwd", R, V1, d, ptr(h), ld(h), ptr(E), ld(E), ptr(bias), ptr(labels), ptr(rows_dev),
         ptr(count_override), ptr(ws), ptr(out), stream())


def vocab_head_supported(d):
    return bool(_lib.lib().rs_vocab_head_supported(d))


def vocab_head_fwd(h, E, bias, labels, ws, out, rows_dev=None, count_override=None):
    """vocab_ce_fwd's result from the vocabulary-tile-stationary kernel (rs_vocab_head_fwd)."""
    R, d = h.shape
    V1 = E.shape[0]
    ev = _ev_begin("vocab_ce_fwd")
    call("rs_vocab_head_fwd", R, V1, d, ptr(h), ld(h), ptr(E), ld(E), ptr(bias), ptr(labels), ptr(rows_dev),
         ptr(count_override), ptr(ws), ptr(out), stream())
    _ev_end(ev)


def vocab_head_bwd(h, E, bias, labels, ws, count, dl, rows_dev=None, dloss=None, voff=0):
    """vocab_ce_bwd's dlogits from the vocabulary-tile-stationary kernel (rs_vocab_head_bwd); E may be a shard of
    the table starting at vocabulary id voff (labels stay absolute)."""
    R, d = h.shape
    V1 = E.shape[0]
    call("rs_vocab_head_bwd", R, V1, d, ptr(h), ld(h), ptr(E), ld(E), ptr(bias), ptr(labels), ptr(rows_dev),
         ptr(count), ptr(dloss), ptr(ws), ptr(dl), ld(dl), int(voff), stream())


def vocab_shard_lse(h, E, bias, labels, ws, lse):
    R, d = h.shape
    call("rs_vocab_shard_lse", R, E.shape[0], d, ptr(h), ld(h), ptr(E), ld(E), ptr(bias), ptr(labels), ptr(ws),
         ptr(lse), stream())


def vocab_shard_label_logits(h, E, bias, labels, v0, v1, tgt):
    R, d = h.shape
    call("rs_vocab_shard_label_logits", R, d, ptr(h), ld(h), ptr(E), ld(E), ptr(bias), ptr(labels), int(v0), int(v1),
         ptr(tgt), stream())


def vocab_shard_combine(lse_parts, tgt, labels, lse, out):
    N, R = lse_parts.shape
    call("rs_vocab_shard_combine", N, R, ptr(lse_parts), ptr(tgt), ptr(labels), ptr(lse), ptr(out), stream())


def vocab_ce_bwd(h, E, bias, labels, ws, count, dl, rows_dev=None, dloss=None):
    """dl [R, V1] bf16 = (softmax(h E^T + bias) - onehot(labels)) * dloss / count."""
    R, d = h.shape
    V1 = E.shape[0]
    call("rs_vocab_ce_bwd", R, V1, d, ptr(h), ld(h), ptr(E), ld(E), ptr(bias), ptr(labels), ptr(rows_dev),
         ptr(count), ptr(dloss), ptr(ws), ptr(dl), ld(dl), stream())


def graph_upload(graph):
    """hipGraphUpload of a captured torch.cuda.CUDAGraph's executable (rs_graph_upload) on the current stream."""
    call("rs_graph_upload", C.c_void_p(int(graph.raw_cuda_graph_exec())), stream())


def seed_advance(seed_base):
    call("rs_seed_advance", ptr(seed_base), stream())


# ---- fused SAS sublayers (rowchain.hip) ----------------------------------------------------
def sas_block_fused_ok(d, dtype):
    """rs_sas_block_in/out cover bf16 with d in {64, 128}; anything else runs the unfused kernels."""
    return dtype == torch.bfloat16 and d in (64, 128)


def sas_block_in(x, ln_w, ln_b, eps, Q, mean, rstd, Wq, bq, q, Wkv, bkv, kv):
    M, d = x.shape
    call("rs_sas_block_in", M, d, ptr(x), ld(x), ptr(ln_w), ptr(ln_b), eps, ptr(Q), ptr(mean), ptr(rstd),
         ptr(Wq), ptr(bq), ptr(q), ptr(Wkv), ptr(bkv), ptr(kv), stream())


def sas_block_in_count_parts(M):
    return int(_lib.lib().rs_sas_block_in_count_parts(M))


def sas_block_in_embed(ids, T, item_emb, pos_emb, scale, drop_p, salt, seed_base, x0, count_ids, count_parts,
                       ln_w, ln_b, eps, Q, mean, rstd, Wq, bq, q, Wkv, bkv, kv):
    """embed_fwd(_counted) (mode 0) + sas_block_in in one launch (rowchain); x0 receives the embedding output."""
    M, d = x0.shape
    assert ids.numel() == M and item_emb.dtype == torch.bfloat16 and x0.dtype == torch.bfloat16
    if count_parts is not None:
        assert count_parts.dtype == torch.int32 and count_parts.numel() >= sas_block_in_count_parts(M)
    call("rs_sas_block_in_embed", M, d, ptr(ids), T, ptr(item_emb), ptr(pos_emb), scale, drop_p, salt,
         ptr(seed_base), ptr(x0), ptr(count_ids), ptr(count_parts), ptr(ln_w), ptr(ln_b), eps, ptr(Q), ptr(mean),
         ptr(rstd), ptr(Wq), ptr(bq), ptr(q), ptr(Wkv), ptr(bkv), ptr(kv), stream())


def sas_block_grid(M):
    return int(_lib.lib().rs_sas_block_grid(M))


def sas_block_out_head(out_args, E, pos, neg, lnl_w, lnl_b, count_parts, divisor, f, pl, nl, dpl, dnl, dx, lnpart,
                       part):
    """sas_block_out(*out_args) for the last block with the SAS head in the same launch (rowchain);
    lnpart [G][2][d], part [G][3] with G = sas_block_grid(M)."""
    (o, Q, Wo, bo, x1, ln_w, ln_b, eps, z, mean, rstd, W1, b1, h1, W2, b2, xn, ids, drop_p, salt1, salt2,
     seed_base) = out_args
    M, d = o.shape
    G = sas_block_grid(M)
    assert part.numel() == 3 * G and lnpart.numel() >= 2 * d * G and count_parts.dtype == torch.int32
    call("rs_sas_block_out_head", M, d, ptr(o), ptr(Q), ptr(Wo), ptr(bo), ptr(x1), ptr(ln_w), ptr(ln_b), eps, ptr(z),
         ptr(mean), ptr(rstd), ptr(W1), ptr(b1), ptr(h1), ptr(W2), ptr(b2), ptr(xn), ptr(ids), drop_p, salt1, salt2,
         ptr(seed_base), ptr(E), ptr(pos), ptr(neg), ptr(lnl_w), ptr(lnl_b), ptr(count_parts), count_parts.numel(),
         ptr(divisor), ptr(f), ptr(pl), ptr(nl), ptr(dpl), ptr(dnl), ptr(dx), ptr(lnpart), ptr(part), stream())


def sas_block_out(o, Q, Wo, bo, x1, ln_w, ln_b, eps, z, mean, rstd, W1, b1, h1, W2, b2, xn, ids, drop_p,
                  salt1, salt2, seed_base):
    M, d = o.shape
    call("rs_sas_block_out", M, d, ptr(o), ptr(Q), ptr(Wo), ptr(bo), ptr(x1), ptr(ln_w), ptr(ln_b), eps, ptr(z),
         ptr(mean), ptr(rstd), ptr(W1), ptr(b1), ptr(h1), ptr(W2), ptr(b2), ptr(xn), ptr(ids), drop_p, salt1,
         salt2, ptr(seed_base), stream())


def sas_block_out_bwd(dxn, ids, h1, x1, mean2, rstd2, ln_w, W2T, W1T, WoT, dy2, da1, dx1, dout, part, drop_p, salt1,
                      salt2, seed_base, o=None, delta=None):
    """part: fp32 >= 2*d*sas_block_parts(M), receives the LN2 affine partials (ln_partial_segments).  o, delta
    (one-head attention output [M, d] bf16, fp32 [M]): also delta = rowsum(dout * o) for attn_bwd(delta_in=True)."""
    M, d = dxn.shape
    call("rs_sas_block_out_bwd_delta", M, d, ptr(dxn), ptr(ids), ptr(h1), ptr(x1), ptr(mean2), ptr(rstd2),
         ptr(ln_w), ptr(W2T), ptr(W1T), ptr(WoT), ptr(dy2), ptr(da1), ptr(dx1), ptr(dout), ptr(part), drop_p, salt1,
         salt2, ptr(seed_base), ptr(o), ptr(delta), stream())


def sas_block_in_bwd(dq, dkv, dx1, x, mean1, rstd1, ln_w, WinT, dx, part):
    M, d = dq.shape
    call("rs_sas_block_in_bwd", M, d, ptr(dq), ptr(dkv), ptr(dx1), ptr(x), ptr(mean1), ptr(rstd1), ptr(ln_w),
         ptr(WinT), ptr(dx), ptr(part), stream())


# ---- union-of-touched-rows table-gradient exchange (sparse_rows.hip) -------------------------
def touched_rows_ws_numel(rows):
    return int(_lib.lib().rs_touched_rows_ws_numel(rows))


def touched_rows(ids, rows, flags, index, count, ws):
    """flags/index int32[rows]: index[v] = rank of table row v among the rows occurring in ids (ascending), else
    -1; count int32[1] = their number (device-side, no sync)."""
    call("rs_touched_rows", ptr(ids), ids.numel(), rows, ptr(flags), ptr(index), ptr(count), ptr(ws), stream())


def rows_pack(src, index, count, compact):
    """compact[index[v]] = src[v] for the touched rows; compact rows [count, cap) = 0.  src fp32 [rows, d]."""
    rows, d = src.shape
    call("rs_rows_pack", ptr(src), rows, d, ptr(index), ptr(count), ptr(compact), compact.shape[0], stream())


def rows_unpack(dst, index, compact):
    """dst[v] = compact[index[v]] for the touched rows (the others are left as they are)."""
    rows, d = dst.shape
    call("rs_rows_unpack", ptr(dst), rows, d, ptr(index), ptr(compact), stream())


def sas_block_parts(M):
    """LayerNorm affine partial sets written by rs_sas_block_out_bwd / rs_sas_block_in_bwd for M rows."""
    return int(_lib.lib().rs_sas_block_parts(M))


def ln_partial_segments(part, M, d, dgamma, dbeta, nb=None):
    """The two reduce segments of a fused kernel's LayerNorm partials (part[b][2][d], b < nb; default: the
    SAS row-block backward kernels' set count)."""
    nb = sas_block_parts(M) if nb is None else nb
    return [(part, 2 * d, nb, d, dgamma), (part[d:], 2 * d, nb, d, dbeta)]


def _segments(segs):
    arr = (_lib.ReduceSegment * max(1, len(segs)))()
    for i, (src, stride, splits, n, out) in enumerate(segs):
        arr[i] = _lib.ReduceSegment(ptr(src), stride, splits, n, ptr(out))
    return arr


def wgrad_grouped(problems, M, rows_per_split, slab, extra=(), pos=None, max_tile=256):
    ev = _ev_begin("wgrad_grouped")
    _wgrad_grouped(problems, M, rows_per_split, slab, extra, pos, max_tile)
    _ev_end(ev)


def _wgrad_grouped(problems, M, rows_per_split, slab, extra=(), pos=None, max_tile=256):
    """problems: [(dY, X, dW, db|None)] with dW [N][K] fp32 (+=); extra: reduce segments
    (src, stride, splits, n, out) summed (+=) in the same reduction launch.  pos: (ids, T, dx, drop_p, salt, seed_base, dpos) -- the SAS positional
    table's gradient (embed_bwd mode 0, scale 1, +=) then rides in the reduction launch (rs_wgrad_grouped_pos);
    pos + (head_part, divisor, loss_out): the SAS head's loss statistics too (rs_wgrad_grouped_pos_stats)."""
    arr = (_lib.WgradProblem * len(problems))()
    for i, (dY, X, dW, db) in enumerate(problems):
        N, K = dY.shape[1], X.shape[1]
        assert dW.numel() == N * K and dY.shape[0] >= M and X.shape[0] >= M
        arr[i] = _lib.WgradProblem(ptr(dY), ld(dY), ptr(X), ld(X), N, K, ptr(dW), ptr(db) if db is not None else None)
    segs = _segments(list(extra))
    if pos is not None:
        assert max_tile == 256, "the positional form takes the default tiles"
        ids, T, dx, drop_p, salt, seed_base, dpos, *st = pos
        if st:
            hp, hdiv, lout, *aux = st
            call("rs_wgrad_grouped_pos_stats", len(problems), arr, M, rows_per_split, ptr(slab), slab.numel(),
                 len(extra), segs, ptr(ids), T, ptr(dx), dx.shape[-1], drop_p, salt, ptr(seed_base), ptr(dpos),
                 ptr(hp), hp.numel() // 3, ptr(hdiv), ptr(lout), ptr(aux[0] if aux else None), stream())
            return
        call("rs_wgrad_grouped_pos", len(problems), arr, M, rows_per_split, ptr(slab), slab.numel(), len(extra),
             segs, ptr(ids), T, ptr(dx), dx.shape[-1], drop_p, salt, ptr(seed_base), ptr(dpos), stream())
        return
    call("rs_wgrad_grouped_max", len(problems), arr, M, rows_per_split, ptr(slab), slab.numel(), len(extra), segs,
         int(max_tile), stream())


def wgrad_grouped_tile(shapes, max_tile=256):
    """Output tile edge rs_wgrad_grouped uses for problems of these (N, K) shapes (256, 128 or 64; at most
    max_tile)."""
    arr = (_lib.WgradProblem * len(shapes))()
    for i, (N, K) in enumerate(shapes):
        arr[i] = _lib.WgradProblem(None, 0, None, 0, N, K, None, None)
    t = int(_lib.lib().rs_wgrad_grouped_tile_max(len(shapes), arr, int(max_tile)))
    if t <= 0:
        raise RuntimeError("rs_wgrad_grouped_tile: bad arguments")
    return t


def wgrad_grouped_slab_numel(shapes, M, rows_per_split):
    """shapes: [(N, K)] of the problems."""
    splits = -(-M // rows_per_split)
    return sum(splits * (N * K + N) for N, K in shapes)


def reduce_segments(segs, accumulate=True):
    call("rs_reduce_segments", len(segs), _segments(list(segs)), int(accumulate), stream())


def transpose_bf16(desc, max_tiles, src, dst):
    """desc: int64 device tensor [nmat][6] (rows, cols, src_off, lds, dst_off, ldd)."""
    call("rs_transpose_bf16", desc.shape[0], ptr(desc), max_tiles, ptr(src), ptr(dst), stream())


# ---- item-table gradient by inverted index (itemgrad.hip) ----------------------------------
def item_index_ws_bytes(nsrc, rows, table_rows, d):
    n = _lib.lib().rs_item_index_ws_bytes(nsrc, rows, table_rows, d)
    if n < 0:
        raise RuntimeError("rs_item_index_ws_bytes: bad arguments")
    return n


def item_index_build(keys, table_rows, d, ws):
    """keys: 1-3 int64 device tensors of the same numel (ids, pos, neg)."""
    rows = keys[0].numel()
    kp = [ptr(k) for k in keys] + [None] * (3 - len(keys))
    call("rs_item_index_build", len(keys), kp[0], kp[1], kp[2], rows, table_rows, d, ptr(ws), ws.numel(), stream())


def item_index_view(nsrc, rows, table_rows, d, ws):
    """(sorted keys, sorted entries, start, sort path) of a built index: views into ws (tests and tools); start
    (first sorted position of each key) exists on the counting-sort path only, else None."""
    out = (_lib.i64 * 4)()
    call("rs_item_index_layout", nsrc, rows, table_rows, d, out)
    n = nsrc * rows
    sk = ws[out[0]:out[0] + 4 * n].view(torch.int32)
    sv = ws[out[1]:out[1] + 4 * n].view(torch.int32)
    start = ws[out[2]:out[2] + 4 * (table_rows + 1)].view(torch.int32) if out[2] >= 0 else None
    return sk, sv, start, int(out[3])


def item_grad(ws, nsrc, rows, dx, scale, drop_p, salt, seed_base, f, w1, w2, dtable, marks=None):
    """marks: (row_marks u8 [table_rows], epoch u8 [1]) -- rs_item_grad_marked stamps the rows it writes (bf16)."""
    table_rows, d = dtable.shape
    if marks is not None and dx.dtype != torch.float32:
        call("rs_item_grad_marked", ptr(ws), nsrc, rows, table_rows, d, ptr(dx), scale, drop_p, salt, ptr(seed_base),
             ptr(f) if f is not None else None, ptr(w1) if w1 is not None else None,
             ptr(w2) if w2 is not None else None, ptr(dtable), ptr(marks[0]), ptr(marks[1]), stream())
        return
    # fp32 (the parity path): chunk + span kernels at any width; bf16: the LDS chunk kernels (d in {64, 128, 256})
    call("rs_item_grad_f32" if dx.dtype == torch.float32 else "rs_item_grad", ptr(ws), nsrc, rows, table_rows, d,
         ptr(dx), scale, drop_p, salt, ptr(seed_base),
         ptr(f) if f is not None else None, ptr(w1) if w1 is not None else None,
         ptr(w2) if w2 is not None else None, ptr(dtable), stream())


def gemm_n256_splits(M, K):
    return int(_lib.lib().rs_gemm_n256_splits(M, K))


def gemm_n256(A, B, C, a_kmajor, M, K, split=False, colsum=None, rows_dev=None):
    """C[m, :256] = sum_k A(m, k) B(k, :) fp32 (rs_gemm_n256).  A: bf16 2-D view, A(m, k) = A[k, m] (a_kmajor) or
    A[m, k]; B: bf16 (K, 256) rows (row stride ld(B)); C: fp32 rows of 256 (ld(C)); split: C is a [splits, M, 256]
    slab (one k slice each, gemm_n256_splits(M, K) of them)."""
    cz = C[0].numel() if split else 0
    Cm = C[0] if split else C
    call("rs_gemm_n256", int(a_kmajor), M, K, ptr(A), ld(A), ptr(B), ld(B), ptr(C), ld(Cm), int(split), cz,
         ptr(colsum), ptr(rows_dev), stream())


def candidate_scores(h, E, cand, bias=None):
    """(B, C) fp32 scores <h[b], E[cand[b, c]]> (+ bias[cand[b, c]]): rs_candidate_scores.  h: (B, d) rows (row stride
    may exceed d), E: (V, d) in h's dtype, cand: (B, C) int64 on the device; raises on an id outside [0, V) like
    the reference's embedding / gather."""
    B, d = h.shape
    V = E.shape[0]
    cand = cand.contiguous()
    if bool(((cand < 0) | (cand >= V)).any()):
        raise IndexError("candidate id out of range")
    out = torch.empty(cand.shape, dtype=torch.float32, device=h.device)
    call("rs_candidate_scores", dtype_code(h), ptr(h), h.stride(0), B, d, ptr(E), ptr(bias), ptr(cand), cand.shape[1], V,
         ptr(out), stream())
    return out


# ---- fused SAS output head (head.hip) --------------------------------------------------------
def sas_head_fwd(x, ln_w, ln_b, eps, f, mean, rstd, E, pos, neg, pl, nl, part):
    M, d = x.shape
    call("rs_sas_head_fwd", M, d, ptr(x), ptr(ln_w), ptr(ln_b), eps, ptr(f), ptr(mean), ptr(rstd), ptr(E), ptr(pos),
         ptr(neg), ptr(pl), ptr(nl), ptr(part), stream())


def sas_head_bwd(part, divisor, out, pl, nl, dpl_in, dnl_in, dpl, dnl, pos, neg, E, x, ln_w, mean, rstd, dx, lnpart):
    M, d = x.shape
    call("rs_sas_head_bwd", M, d, ptr(part), ptr(divisor), ptr(out), ptr(pl), ptr(nl), ptr(dpl_in), ptr(dnl_in),
         ptr(dpl), ptr(dnl), ptr(pos), ptr(neg), ptr(E), ptr(x), ptr(ln_w), ptr(mean), ptr(rstd), ptr(dx),
         ptr(lnpart), stream())


def sas_head_finish(part, divisor, out):
    """Loss statistics out[0..3] from the head's BCE partials part[nblk][3] (one workgroup)."""
    call("rs_sas_head_finish", part.numel() // 3, ptr(part), ptr(divisor), ptr(out), stream())


# ---- on-device sampler and ranking metrics (sampler.hip) -----------------------------------
def sas_sample(user_offsets, user_items, n_users, item_num, seed_base, salt, seq, pos, neg, draws=None):
    """draws (optional, tests): int64 (batch, 1 + 256 * max_len) record of the draws (rs_sas_sample_draws)."""
    B, T = seq.shape
    if draws is not None:
        call("rs_sas_sample_draws", ptr(user_offsets), ptr(user_items), n_users, item_num, B, T, ptr(seed_base), salt,
             ptr(seq), ptr(pos), ptr(neg), ptr(draws), stream())
        return
    call("rs_sas_sample", ptr(user_offsets), ptr(user_items), n_users, item_num, B, T, ptr(seed_base), salt,
         ptr(seq), ptr(pos), ptr(neg), stream())


def bert_mask(offsets, items, n_users, num_items, mask_prob, perm, state, salt, tokens, labels, draws=None):
    """rs_bert_mask: the next (tokens, labels) batch into (batch, max_len) int64 device tensors; draws (optional,
    tests): int64 (batch, 1 + 2 * max_len) record of the draws (rs_bert_mask_draws)."""
    B, T = tokens.shape
    if draws is not None:
        call("rs_bert_mask_draws", ptr(offsets), ptr(items), n_users, num_items, B, T, mask_prob, ptr(perm),
             ptr(state), salt, ptr(tokens), ptr(labels), ptr(draws), stream())
        return
    call("rs_bert_mask", ptr(offsets), ptr(items), n_users, num_items, B, T, mask_prob, ptr(perm), ptr(state), salt,
         ptr(tokens), ptr(labels), stream())


def rank_metrics(scores, labels, ks_dev, ws, out):
    R, C = scores.shape
    call("rs_rank_metrics", ptr(scores), ptr(labels), R, C, ks_dev.numel(), ptr(ks_dev), ptr(ws), ptr(out), stream())
