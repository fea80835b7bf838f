"""Vocabulary-sharded BERT output layer for data-parallel training.

With the BERT vocabulary at 1M items the output layer (out.weight [V+1, d], BS/models/bert.py:10) is 257M
parameters: replicated, every rank computes the whole R x (V+1) head and every step all-reduces a 1 GB
gradient.  Sharded, data-parallel rank r owns rows [v0, v1) of out.weight / out.bias (128-aligned slices):

  1. all-gather the labelled rows h and their labels of every rank            (N * cap * d bf16)
  2. per row, log-sum-exp over this shard (rs_vocab_shard_lse) and the label's logit where this
     shard holds the label (rs_vocab_shard_label_logits)
  3. all-gather the per-shard lse, all-reduce the label logits                   (N * cap floats each)
  4. lse over the whole vocabulary and the loss of the global batch (rs_vocab_shard_combine): every rank
     holds the same loss and labelled count, so the gradients below are already those of the global mean
  5. dlogits on the shard (rs_vocab_head_bwd, voff = v0) -> dE_shard = dlogits^T H, db_shard: complete
     gradients of the owned rows, no collective
  6. dH = dlogits E_shard summed over shards (all-reduce, N * cap * d fp32); each rank keeps its own rows
     and continues its encoder backward.

The owned rows' gradients never enter the data-parallel all-reduce, and the optimizer updates only the owned
rows (FusedTrainStep); the other ranks' rows of this rank's out.weight copy are never read.  The collectives
run eagerly between captured graph segments (the engine's split(tag, action) points).
"""
import torch
import torch.distributed as dist

ALIGN = 128


class VocabShard:
    """This rank's slice [v0, v1) of the output vocabulary (V1 = num_items + 1 rows)."""

    def __init__(self, V1, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        per = -(-(-(-V1 // self.world)) // ALIGN) * ALIGN
        self.v0 = min(V1, self.rank * per)
        self.v1 = min(V1, self.v0 + per)
        self.V1 = V1
        if self.v1 <= self.v0:
            raise ValueError(f"vocabulary of {V1} rows too small for {self.world} shards of {per}")

    def owned_ranges(self, offset, d):
        """Flat-buffer float ranges of out.weight rows this rank owns (out.weight at flat offset `offset`)."""
        return offset + self.v0 * d, offset + self.v1 * d

    def all_gather(self, out, inp):
        """out = concatenation of every rank's inp (equal sizes)."""
        dist.all_gather(list(out.view(self.world, -1).unbind(0)), inp.reshape(-1), group=self.group)

    def all_reduce(self, t):
        dist.all_reduce(t, group=self.group)

    def gather_rows(self, full, rows_per_rank=None):
        """Make every rank's copy of a vocabulary-major tensor `full` [V1, ...] hold the owners' rows (in place):
        the reference-layout parameter (or optimizer state) for a checkpoint."""
        per = -(-(-(-self.V1 // self.world)) // ALIGN) * ALIGN
        inner = full[0].numel() if full.dim() > 1 else 1
        buf = torch.zeros(self.world * per * inner, dtype=full.dtype, device=full.device)
        mine = torch.zeros(per * inner, dtype=full.dtype, device=full.device)
        mine[:(self.v1 - self.v0) * inner] = full[self.v0:self.v1].reshape(-1)
        self.all_gather(buf, mine)
        flat = full.view(-1)
        for r in range(self.world):
            v0 = min(self.V1, r * per)
            v1 = min(self.V1, v0 + per)
            if v1 > v0:
                flat[v0 * inner:v1 * inner] = buf[r * per * inner:(r * per + v1 - v0) * inner]
        return full
