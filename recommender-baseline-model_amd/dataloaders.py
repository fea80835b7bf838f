"""On-device training samplers.

DeviceWarpSampler (SAS): the reference's ``WarpSampler`` (BS/dataloaders/sas.py:93-122) with the
per-sequence work of ``sample_function`` (:65-91) done by one HIP kernel (rs_sas_sample).

Same contract as the reference loader: iterate ``len(sampler) = len(user_train) // batch_size`` batches
of (seq, pos, neg), each (batch_size, max_len); a row is a uniformly drawn user's last ``max_len``
items shifted by one (seq/pos), left-padded with 0, and negatives drawn uniformly from
{0..item_num} minus that window (item 0 is a legal negative, as ``random_neq`` allows).  Unlike the
reference the batch is produced on the device (int64 tensors) by a counter-based RNG: no worker
processes, no host round trip, and ``sample_into`` can be captured in the training step's HIP graph.

DeviceBertMasker (BERT4Rec): the reference's ``BertTrainDataset`` + shuffling ``DataLoader``
(BS/dataloaders/bert.py:64-110) with the per-token cloze masking done by rs_bert_mask.  An epoch visits
the users in a fresh random order (``torch.randperm`` on the device at ``__iter__``), ``len(masker) =
n_users // batch_size`` full batches (the fixed batch shape a captured graph needs; the reference's
last partial batch is dropped), each row = that user's last ``max_len`` items cloze-masked at
``mask_prob`` (80 % [MASK] = num_items+1, 10 % random item, 10 % kept), labels = the masked items.
"""
import torch

from . import ops


def _flatten(histories, device):
    lens = [len(s) for s in histories]
    if not lens or min(lens) < 1:
        raise ValueError("every user needs at least one training item")
    off = torch.zeros(len(lens) + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(torch.tensor(lens, dtype=torch.int64), 0)
    items = torch.tensor([i for s in histories for i in s], dtype=torch.int64, device=device)
    return off.to(device), items, len(lens)


class DeviceWarpSampler:
    n_outputs = 3

    def __init__(self, user_train, item_num, batch_size, max_len, device="cuda", num_workers=None, seed=None):
        """user_train: list (per user) of item-id lists, as ``data_partition`` builds it.
        num_workers is accepted for signature compatibility and ignored."""
        if max_len > 512:
            raise ValueError("max_len must be <= 512")
        self.device = torch.device(device)
        self.offsets, self.items, self.n_users = _flatten(user_train, self.device)
        self.item_num = int(item_num)
        self.batch_size = int(batch_size)
        self.max_len = int(max_len)
        self.num_batch = self.n_users // self.batch_size
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        self.salt = int(torch.randint(0, 2 ** 62, (1,), generator=g).item())
        self.seed_base = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.cnt = 0

    def sample_into(self, seq, pos, neg, draws=None):
        """Write the next batch into existing (batch_size, max_len) int64 device tensors (draws: see
        ops.sas_sample)."""
        ops.sas_sample(self.offsets, self.items, self.n_users, self.item_num, self.seed_base, self.salt, seq, pos, neg,
                       draws)

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


class DeviceBertMasker:
    n_outputs = 2

    def __init__(self, u2seq, num_items, batch_size, max_len, mask_prob, device="cuda", seed=None):
        """u2seq: list (per user) of training item-id lists (the reference's ``train`` dict values in user
        order).  The [MASK] token is num_items + 1, as BERTEmbedding's table (V+2 rows) expects."""
        self.device = torch.device(device)
        self.offsets, self.items, self.n_users = _flatten(u2seq, self.device)
        self.num_items = int(num_items)
        self.batch_size = int(batch_size)
        self.max_len = int(max_len)
        self.mask_prob = float(mask_prob)
        self.num_batch = self.n_users // self.batch_size
        self.gen = torch.Generator(device=self.device)
        g = torch.Generator()
        if seed is not None:
            g.manual_seed(seed)
            self.gen.manual_seed(seed)
        self.salt = int(torch.randint(0, 2 ** 62, (1,), generator=g).item())
        self.state = torch.zeros(2, dtype=torch.int64, device=self.device)   # {step seed, cursor}
        self.perm = torch.arange(self.n_users, dtype=torch.int64, device=self.device)
        self.cnt = 0

    def new_epoch(self):
        """Reshuffle the user order in place and restart the cursor (device work; graphs see it)."""
        torch.randperm(self.n_users, generator=self.gen, device=self.device, out=self.perm)
        self.state[1:2].zero_()

    def sample_into(self, tokens, labels, draws=None):
        ops.bert_mask(self.offsets, self.items, self.n_users, self.num_items, self.mask_prob, self.perm, self.state,
                      self.salt, tokens, labels, draws)

    def sample(self):
        shape = (self.batch_size, self.max_len)
        tokens, labels = (torch.empty(shape, dtype=torch.int64, device=self.device) for _ in range(2))
        self.sample_into(tokens, labels)
        return tokens, labels

    def __iter__(self):
        self.new_epoch()
        self.cnt = 0
        return self

    def __next__(self):
        if self.cnt < self.num_batch:
            self.cnt += 1
            return self.sample()
        raise StopIteration

    def __len__(self):
        return self.num_batch
