"""Data-parallel gradient exchange (one process per GPU, torch.distributed over RCCL/xGMI).

The reference has no working multi-GPU path for SAS (``nn.DataParallel`` replicates the numpy
batch, BS/trainers/base.py:32-34 + BS/trainers/sas.py:36-37), so the target is the single-device
math on the global batch: both losses are MEANS over the valid positions of
the whole batch (BS/trainers/sas.py:49, BS/trainers/bert.py:40).  Each rank therefore
back-propagates its UNnormalised loss sum, writes (loss sum, valid count) into the two aux
floats at the tail of its flat gradient buffer, and ONE all-reduce(SUM) of that buffer yields
the global gradient sum, loss sum and count; the optimizer divides by the count
(rs_adam_prepare's grad_divisor).  Averaging per-rank means instead is wrong whenever ranks see
different valid counts.

Overlap with backward: the flat buffer is split into buckets that become final at
different points of the backward -- BERT: the vocabulary head (out.weight, out.bias, + aux) right after its
weight gradient, then everything else.  (The fused SAS backward finishes all its gradients in its last launches,
so it exchanges one bucket: see FusedTrainStep._buckets.)  BucketedExchange starts each
bucket's all-reduce (async, on the backend's stream, ordered after the work already issued on the
current stream) as soon as it is final, so it overlaps the rest of the backward; finish() makes the
current stream wait for all of them before the optimizer.

Large embedding tables (SparseRowExchange): a step touches few rows of a 1M-row token table,
and the others' gradients are zero on every rank.  The ranks all-gather their batch ids, build the same sorted
union of touched rows on the device (rs_touched_rows: no host sync, graph-capturable), pack those rows of the
table gradient into a fixed-capacity compact buffer (capacity = gathered id count, at most the table), all-reduce
that instead of the dense table, and unpack it.  Rows outside the union stay zero, as the dense all-reduce leaves
them; every element is summed over the same ranks (two ranks: bit for bit the dense result).  Bytes per rank at
cfg5 on 8 GPUs (1,000,002 x 256 fp32 table, 12,800 token ids per rank): 1,024 MB dense -> at most 102,400 rows x
1 KB = 105 MB + 0.8 MB of ids.

Sharded table optimizer (ShardedRows): the SAS item table is most of the gradient buffer (cfg4:
54,543 x 128 fp32 = 27.9 of 28.7 MB) and every rank's Adam over it is the same work.  Instead of the dense all-reduce, the
table's gradient is REDUCE-SCATTERED (each rank receives the global sum of its 1/N of the table), each rank runs Adam on
that part only, and the updated compute rows (bf16, or fp32 without a bf16 copy) are ALL-GATHERED back before the next
forward.  The fp32 master and Adam moments of the other ranks' parts are not kept current on this rank (they stay
allocated: this is for exchange bytes and optimizer time, not memory); gather_masters() all-gathers them (checkpoints).
Ring bytes sent per rank and step at cfg4 on 8 GPUs: dense all-reduce 2 x 7/8 x 28.7 MB = 50.2 MB; sharded: 7/8 x 27.9 MB
reduce-scatter + 7/8 x 14.0 MB bf16 all-gather + 2 x 7/8 x 0.8 MB for the rest = 38.1 MB, and 1/8 of the table's Adam.
The split is by elements (Adam and the copies are elementwise), in equal 64-element-aligned parts; the table's last few
elements that do not fill a part ride in the dense all-reduce.  Under gloo (the CPU tests) the reduce-scatter is an
all-reduce of the region whose own part is then used -- the same values -- since gloo has no reduce-scatter.

The bucket helpers only move tensors (gloo on CPU in the tests); SparseRowExchange's index/pack kernels need the
HIP library.
"""
import torch
import torch.distributed as dist

LOSS_SUM, COUNT = 0, 1   # aux slots


def world(group=None):
    """World size of `group` (default: the global group); 1 without torch.distributed."""
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def backend(group=None):
    """The process group's backend name ("nccl" = RCCL on ROCm, "gloo"), None without torch.distributed."""
    return str(dist.get_backend(group)).lower() if dist.is_available() and dist.is_initialized() else None


def agree(ok, group=None):
    """True on every rank iff `ok` is true on every rank (an eager MIN all-reduce of one flag; a no-op without
    torch.distributed).  Used where a rank-local outcome (a graph capture that may refuse a collective) decides
    which collectives every rank issues next: the ranks must take the same branch or the next collective hangs."""
    if world(group) == 1:
        return bool(ok)
    dev = "cuda" if backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def replicas_equal(t, group=None):
    """True iff the tensor `t` holds the same bits on every rank (the data-parallel replicas' parameters after a
    step): MAX and MIN all-reduces of an exact integer checksum of its bits."""
    if world(group) == 1:
        return True
    x = t.detach().reshape(-1).view(torch.int32).to(torch.int64)
    w = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.int64) % 65521 + 1
    c = torch.stack([(x * w).sum(), x.sum()])
    if backend(group) != "nccl":
        c = c.cpu()
    hi, lo = c.clone(), c.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    return bool(torch.equal(hi, lo))


def allreduce_grads(flat_grad, group=None, bucket_numel=None):
    """SUM all-reduce of the flat gradient buffer (parameters + aux tail), in place.

    bucket_numel: split into buckets of that many floats (None = one call); buckets are issued
    back to back on the current stream, RCCL pipelines them over the xGMI links."""
    if world(group) == 1:
        return flat_grad
    if not bucket_numel or bucket_numel >= flat_grad.numel():
        dist.all_reduce(flat_grad, group=group)
        return flat_grad
    for o in range(0, flat_grad.numel(), bucket_numel):
        dist.all_reduce(flat_grad[o:o + bucket_numel], group=group)
    return flat_grad


def global_mean_loss(aux):
    """Loss of the global batch from an all-reduced aux tail (a device scalar, no sync)."""
    return aux[LOSS_SUM:LOSS_SUM + 1] / aux[COUNT:COUNT + 1]


class BucketedExchange:
    """All-reduce(SUM) of a flat gradient buffer bucket by bucket, each launched when it is final.

    buckets: {tag: (lo, hi)} disjoint slices covering the buffer.  launch(tag) issues that slice's
    all-reduce asynchronously; finish() waits for every launched one (on the current stream for
    NCCL/RCCL: no host block) and checks that every bucket went out exactly once."""

    def __init__(self, flat_grad, buckets, group=None, partial=False, extra=None):
        """buckets: {tag: (lo, hi) or [(lo, hi), ...]}.  partial: the buckets may leave parts of the buffer out
        (rank-owned regions, e.g. a vocabulary shard, or a table exchanged by SparseRowExchange / ShardedRows); else
        they must cover it.  extra: {tag: callable() -> work or None}, a further collective issued with that tag's
        all-reduce (ShardedRows.scatter)."""
        self.flat_grad = flat_grad
        self.extra = dict(extra or {})
        self.buckets = {t: ([r] if isinstance(r, tuple) else list(r)) for t, r in dict(buckets).items()}
        self.group = group
        spans = sorted(x for rs in self.buckets.values() for x in rs)
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), "buckets must be disjoint"
        assert all(0 <= lo < hi <= flat_grad.numel() for lo, hi in spans), "bucket out of the buffer"
        if not partial:
            assert spans[0][0] == 0 and spans[-1][1] == flat_grad.numel(), "buckets must cover the buffer"
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:])), "buckets must be contiguous"
        self.works = []
        self.sent = []

    def launch(self, tag):
        self.sent.append(tag)
        for lo, hi in self.buckets[tag]:
            self.works.append(dist.all_reduce(self.flat_grad[lo:hi], group=self.group, async_op=True))
        if tag in self.extra:
            w = self.extra[tag]()
            if w is not None:
                self.works.append(w)

    def finish(self):
        assert sorted(self.sent) == sorted(self.buckets), (self.sent, list(self.buckets))
        for w in self.works:
            w.wait()
        self.works, self.sent = [], []
        return self.flat_grad


def carve(buckets, lo, hi):
    """The buckets {tag: (lo, hi) | [ranges]} with [lo, hi) removed from every range (a region exchanged another
    way); tags left with no range are dropped."""
    out = {}
    for tag, rs in buckets.items():
        rs = [rs] if isinstance(rs, tuple) else list(rs)
        keep = []
        for a, b in rs:
            if b <= lo or a >= hi:
                keep.append((a, b))
                continue
            if a < lo:
                keep.append((a, lo))
            if b > hi:
                keep.append((hi, b))
        if keep:
            out[tag] = keep
    return out


class SparseRowExchange:
    """Union-of-touched-rows all-reduce of one embedding table's gradient (see the module docstring).

    grad_rows: the table's fp32 gradient rows [rows, d] (a view into the flat gradient buffer); n_local: ids per
    rank per step.  Per step: gather_ids(ids) (collective) -> index_rows() -> [table gradient complete] ->
    pack() -> allreduce() (collective) -> unpack().  Collectives run on the current stream's order (eager, between
    graph segments); the kernels are graph-capturable."""

    def __init__(self, grad_rows, n_local, group=None):
        from . import ops
        self.ops = ops
        self.g = grad_rows
        self.rows, self.d = grad_rows.shape
        self.W = world(group)
        self.n_local = int(n_local)
        self.group = group
        self.cap = min(self.rows, self.W * self.n_local)
        dev = grad_rows.device
        self.ids_all = torch.zeros(self.W * self.n_local, dtype=torch.int64, device=dev)
        self.flags = torch.zeros(self.rows, dtype=torch.int32, device=dev)
        self.index = torch.zeros(self.rows, dtype=torch.int32, device=dev)
        self.count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ws = torch.zeros(ops.touched_rows_ws_numel(self.rows), dtype=torch.int32, device=dev)
        self.compact = torch.zeros(self.cap, self.d, dtype=torch.float32, device=dev)

    @staticmethod
    def worthwhile(rows, n_local, n_ranks):
        """Sparse when the compact buffer is at most half the dense table."""
        return n_ranks > 1 and n_ranks * n_local <= rows // 2

    def bytes_per_step(self):
        """(dense all-reduce bytes, sparse all-reduce + all-gather bytes) of this table."""
        return self.rows * self.d * 4, self.cap * self.d * 4 + self.W * self.n_local * 8

    def gather_ids(self, ids):
        flat = ids.reshape(-1)
        assert flat.numel() == self.n_local, (flat.numel(), self.n_local)
        dist.all_gather(list(self.ids_all.view(self.W, self.n_local).unbind(0)), flat, group=self.group)

    def index_rows(self):
        self.ops.touched_rows(self.ids_all, self.rows, self.flags, self.index, self.count, self.ws)

    def pack(self):
        self.ops.rows_pack(self.g, self.index, self.count, self.compact)

    def allreduce(self):
        dist.all_reduce(self.compact, group=self.group)

    def unpack(self):
        self.ops.rows_unpack(self.g, self.index, self.compact)


class ShardedRows:
    """Reduce-scatter / rank-local Adam / all-gather of one table of a FlatParams buffer (see the module docstring).

    The table's elements [lo, hi) (hi = lo + N x part, the largest N-fold multiple of 64 elements inside the table)
    are cut into N equal parts; rank r owns [lo + r part, lo + (r + 1) part).  Per step: scatter() (collective, with
    the dense all-reduce) -> Adam over ranges() -> zero_foreign() -> gather() (collective) of the compute copy."""

    ALIGN = 64

    def __init__(self, flat, name, group=None):
        self.flat = flat
        self.name = name
        self.group = group
        self.W = world(group)
        self.rank = dist.get_rank(group) if self.W > 1 else 0
        self.lo = flat.offsets[name]
        n = 1
        for s in flat.shapes[name]:
            n *= s
        self.table_end = self.lo + n
        A = self.ALIGN
        assert self.lo % A == 0, self.lo
        self.part = (n // (self.W * A)) * A
        self.hi = self.lo + self.W * self.part
        self.own = (self.lo + self.rank * self.part, self.lo + (self.rank + 1) * self.part)
        self.nccl = backend(group) == "nccl"

    @staticmethod
    def worthwhile(numel, n_ranks):
        """Shard when every rank's part is at least 64k elements (smaller tables: the extra collective's latency
        outweighs the bytes)."""
        return n_ranks > 1 and numel // n_ranks >= 65536

    def foreign(self):
        """The sharded region's ranges this rank does not own."""
        a, b = self.own
        return [(x, y) for x, y in ((self.lo, a), (b, self.hi)) if y > x]

    def dense_ranges(self, total):
        """[0, total) without the sharded region (what the all-reduce and the full-buffer optimizer launch cover)."""
        return [(x, y) for x, y in ((0, self.lo), (self.hi, total)) if y > x]

    def adam_ranges(self, total):
        """The optimizer's ranges: the dense parts first (the first launch prepares the step's scalars and writes the
        transposed block weights: it must cover them), then the owned part."""
        return self.dense_ranges(total) + [self.own]

    @classmethod
    def ring_bytes(cls, total, table, n_ranks, compute_bytes):
        """(dense all-reduce bytes, sharded-table bytes) sent per rank and step by ring collectives: a buffer of
        `total` fp32 elements holding a `table`-element table whose compute copy has `compute_bytes` bytes per
        element.  Sharded: reduce-scatter (fp32) + all-gather (compute copy) of the parts, all-reduce of the rest."""
        f = (n_ranks - 1) / n_ranks
        sharded = n_ranks * ((table // (n_ranks * cls.ALIGN)) * cls.ALIGN)
        return 2 * f * total * 4, f * sharded * (4 + compute_bytes) + 2 * f * (total - sharded) * 4

    def bytes_per_step(self):
        """ring_bytes for this buffer and table."""
        f = self.flat
        return self.ring_bytes(f.numel, self.table_end - self.lo, self.W, 2 if f.bf16 is not None else 4)

    def scatter(self, async_op=True):
        """Reduce-scatter(SUM) of the sharded region of the gradient, in place: the owned part receives the global
        sum (RCCL: reduce_scatter_tensor; gloo: an all-reduce of the region)."""
        g = self.flat.grad
        if self.nccl:
            a, b = self.own
            return dist.reduce_scatter_tensor(g[a:b], g[self.lo:self.hi], group=self.group, async_op=async_op)
        return dist.all_reduce(g[self.lo:self.hi], group=self.group, async_op=async_op)

    def zero_foreign(self):
        """Clear the gradient outside the owned part (the optimizer clears the owned part): the next backward
        accumulates into zeros."""
        for a, b in self.foreign():
            self.flat.grad[a:b].zero_()

    def gather(self, buf):
        """All-gather of the sharded region of `buf` (every rank contributes its owned part), in place."""
        a, b = self.own
        full = buf[self.lo:self.hi]
        if self.nccl:
            dist.all_gather_into_tensor(full, buf[a:b], group=self.group)
        else:
            dist.all_gather(list(full.view(self.W, self.part).unbind(0)), buf[a:b].clone(), group=self.group)

    def gather_compute(self):
        """The step's all-gather: the rows the forward reads (the bf16 copy when there is one, else the master)."""
        f = self.flat
        self.gather(f.bf16 if f.bf16 is not None else f.data)

    def gather_masters(self, bufs):
        """All-gather the sharded region of each fp32 buffer (master weights, Adam moments): afterwards every rank
        holds the full, current table (collective)."""
        for b in bufs:
            self.gather(b)

    def stale_ranges(self):
        """Ranges of the fp32 master that are not current on this rank after a step (bf16 copy: the foreign parts;
        fp32 compute: none -- the master itself is gathered)."""
        return self.foreign() if self.flat.bf16 is not None else []
