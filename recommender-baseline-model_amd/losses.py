"""Loss heads as autograd Functions over the HIP kernels.

* :func:`sampled_bce` -- ``BS/trainers/sas.py:38-49``: BCEWithLogits(pos_logits[pos!=0], 1)
  + BCEWithLogits(neg_logits[pos!=0], 0), each averaged over the valid positions.
* :func:`cross_entropy` -- ``BS/trainers/bert.py:11,36-40``: CrossEntropyLoss(ignore_index=0).

Both take an optional ``global_count`` (a 1-element fp32 device tensor): the
valid-position count of the whole data-parallel batch, so per-rank losses and
gradients sum to the single-device mean.
"""
import torch

from . import ops


class _SampledBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pl, nl, pos, global_count):
        pl, nl = pl.contiguous(), nl.contiguous()
        out = torch.empty(4, dtype=torch.float32, device=pl.device)
        ws = torch.empty(3 * 256, dtype=torch.float32, device=pl.device)
        ops.bce_fwd(pl, nl, pos, ws, out, global_count)
        count = global_count if global_count is not None else out[1:2]
        ctx.save_for_backward(pl, nl, pos, count)
        return out[2].clone()

    @staticmethod
    def backward(ctx, dloss):
        pl, nl, pos, count = ctx.saved_tensors
        dpl, dnl = torch.empty_like(pl), torch.empty_like(nl)
        ops.bce_bwd(pl, nl, pos, count, dloss.contiguous().float(), dpl, dnl)
        return dpl, dnl, None, None


def sampled_bce(pos_logits, neg_logits, pos_ids, global_count=None):
    return _SampledBCE.apply(pos_logits, neg_logits, pos_ids.contiguous(), global_count)


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, global_count):
        R, V1 = logits.shape
        out = torch.empty(4, dtype=torch.float32, device=logits.device)
        ws = torch.empty(3 * R, dtype=torch.float32, device=logits.device)
        ops.ce_fwd(logits, labels, ws, out, global_count)
        count = global_count if global_count is not None else out[1:2]
        ctx.save_for_backward(logits, labels, count, ws)
        return out[2].clone()

    @staticmethod
    def backward(ctx, dloss):
        logits, labels, count, ws = ctx.saved_tensors
        dl = torch.empty_like(logits)
        ops.ce_bwd(logits, labels, count, dloss.contiguous().float(), ws, dl)
        return dl, None, None


def cross_entropy(logits, labels, global_count=None):
    """logits (R, V+1) fp32 (row stride may be padded), labels (R,) int64; ignore_index = 0."""
    return _CrossEntropy.apply(logits, labels.reshape(-1).contiguous(), global_count)
