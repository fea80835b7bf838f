"""On-device SAS training sampler: the reference's ``WarpSampler`` (BS/dataloaders/sas.py:93-122) with the
per-sequence work of ``sample_function`` (:65-91) done by one HIP kernel (rs_sas_sample).

Same contract as the reference loader: iterate ``len(sampler) = len(user_train) // batch_size`` batches
of (seq, pos, neg), each (batch_size, max_len); a row is a uniformly drawn user's last ``max_len``
items shifted by one (seq/pos), left-padded with 0, and negatives drawn uniformly from
{0..item_num} minus that window (item 0 is a legal negative, as ``random_neq`` allows).  Unlike the
reference the batch is produced on the device (int64 tensors) by a counter-based RNG: no worker
processes, no host round trip, and ``sample_into`` can be captured in the training step's HIP graph.
"""
import torch

from . import ops


class DeviceWarpSampler:
    def __init__(self, user_train, item_num, batch_size, max_len, device="cuda", num_workers=None, seed=None):
        """user_train: list (per user) of item-id lists, as ``data_partition`` builds it.
        num_workers is accepted for signature compatibility and ignored."""
        lens = [len(s) for s in user_train]
        if not lens or min(lens) < 1:
            raise ValueError("every user needs at least one training item")
        if max_len > 512:
            raise ValueError("max_len must be <= 512")
        self.device = torch.device(device)
        off = torch.zeros(len(lens) + 1, dtype=torch.int64)
        off[1:] = torch.cumsum(torch.tensor(lens, dtype=torch.int64), 0)
        self.offsets = off.to(self.device)
        self.items = torch.tensor([i for s in user_train for i in s], dtype=torch.int64, device=self.device)
        self.n_users = len(lens)
        self.item_num = int(item_num)
        self.batch_size = int(batch_size)
        self.max_len = int(max_len)
        self.num_batch = self.n_users // self.batch_size
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        self.salt = int(torch.randint(0, 2 ** 62, (1,), generator=g).item())
        self.seed_base = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.cnt = 0

    def sample_into(self, seq, pos, neg):
        """Write the next batch into existing (batch_size, max_len) int64 device tensors."""
        ops.sas_sample(self.offsets, self.items, self.n_users, self.item_num, self.seed_base, self.salt, seq, pos, neg)

    def sample(self):
        shape = (self.batch_size, self.max_len)
        seq, pos, neg = (torch.empty(shape, dtype=torch.int64, device=self.device) for _ in range(3))
        self.sample_into(seq, pos, neg)
        return seq, pos, neg

    # ---- the reference loader's iterator protocol (BS/dataloaders/sas.py:111-122)
    def __iter__(self):
        self.cnt = 0
        return self

    def __next__(self):
        if self.cnt < self.num_batch:
            self.cnt += 1
            return self.sample()
        raise StopIteration

    def __len__(self):
        return self.num_batch

    def close(self):
        pass
