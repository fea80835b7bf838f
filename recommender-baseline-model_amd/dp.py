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
different points of the backward -- SAS: the dense block / LayerNorm weights (+ aux) after the grouped
weight-gradient launch, then the item / positional tables; BERT: the vocabulary head (out.weight,
out.bias, + aux) right after its weight gradient, then everything else.  BucketedExchange starts each
bucket's all-reduce (async, on the backend's stream, ordered after the work already issued on the
current stream) as soon as it is final, so it overlaps the rest of the backward; finish() makes the
current stream wait for all of them before the optimizer.

These helpers only move tensors; they work for any device / backend (gloo on CPU in the tests).
"""
import torch
import torch.distributed as dist

LOSS_SUM, COUNT = 0, 1   # aux slots


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_grads(flat_grad, group=None, bucket_numel=None):
    """SUM all-reduce of the flat gradient buffer (parameters + aux tail), in place.

    bucket_numel: split into buckets of that many floats (None = one call); buckets are issued
    back to back on the current stream, RCCL pipelines them over the xGMI links."""
    if world() == 1:
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

    def __init__(self, flat_grad, buckets, group=None, partial=False):
        """partial: the buckets may leave parts of the buffer out (rank-owned regions, e.g. a vocabulary shard);
        else they must cover it."""
        self.flat_grad = flat_grad
        self.buckets = dict(buckets)
        self.group = group
        spans = sorted(self.buckets.values())
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), "buckets must be disjoint"
        assert all(0 <= lo < hi <= flat_grad.numel() for lo, hi in spans), "bucket out of the buffer"
        if not partial:
            assert spans[0][0] == 0 and spans[-1][1] == flat_grad.numel(), "buckets must cover the buffer"
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:])), "buckets must be contiguous"
        self.works = []
        self.sent = []

    def launch(self, tag):
        lo, hi = self.buckets[tag]
        self.sent.append(tag)
        self.works.append(dist.all_reduce(self.flat_grad[lo:hi], group=self.group, async_op=True))

    def finish(self):
        assert sorted(self.sent) == sorted(self.buckets), (self.sent, list(self.buckets))
        for w in self.works:
            w.wait()
        self.works, self.sent = [], []
        return self.flat_grad
