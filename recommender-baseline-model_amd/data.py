"""Synthetic interaction streams shaped like the reference's training batches.

Host-side numpy generator (no GPU, no reference import) used by the bench, the
parity tests and the golden-fixture script.  Semantics follow the reference
samplers:

* SAS  -- ``BS/dataloaders/sas.py:70-86``: a user history of length n gives
  ``seq = pad + h[:-1]``, ``pos = pad + h[1:]``, ``neg = pad + random items not
  in h``; left padding with item 0 to ``max_len``.
* BERT -- ``BS/dataloaders/bert.py:230-263``: cloze masking with probability
  ``mask_prob``; of the masked tokens 80 % become ``[MASK] = V+1``, 10 % a
  random item, 10 % stay; ``labels`` hold the original item at masked
  positions and 0 elsewhere; left padding to ``max_len``.

Item ids are Zipf(s=1) over 1..V (hot head, long tail) as SURVEY.md §8(d)
prescribes, so gathers see a realistic hot set.
"""
import numpy as np


class ZipfItems:
    def __init__(self, num_items, s=1.0):
        w = 1.0 / np.arange(1, num_items + 1, dtype=np.float64) ** s
        self.cdf = np.cumsum(w) / w.sum()
        self.num_items = num_items

    def sample(self, rng, size):
        u = rng.random(size)
        return np.minimum(np.searchsorted(self.cdf, u), self.num_items - 1).astype(np.int64) + 1


def history_lengths(rng, n, max_len, shape="ml-1m"):
    """Valid history lengths (items per user window, including the last target).

    ml-1m : lognormal around 100 interactions, clipped to [20, max_len+1]
    beauty: heavy-tailed short sessions (mean ~9), clipped to [5, max_len+1]
    """
    if shape == "ml-1m":
        L = np.exp(rng.normal(np.log(120.0), 0.9, size=n))
        return np.clip(np.round(L), 21, max_len + 1).astype(np.int64)
    if shape == "beauty":
        L = 5 + rng.geometric(1.0 / 4.5, size=n)
        return np.clip(L, 5, max_len + 1).astype(np.int64)
    if shape == "full":
        return np.full(n, max_len + 1, dtype=np.int64)
    raise ValueError(shape)


def sas_batch(rng, batch, max_len, num_items, shape="ml-1m", zipf=None):
    """Returns (seq, pos, neg) int64 arrays of shape (batch, max_len)."""
    zipf = zipf or ZipfItems(num_items)
    seq = np.zeros((batch, max_len), np.int64)
    pos = np.zeros((batch, max_len), np.int64)
    neg = np.zeros((batch, max_len), np.int64)
    lens = history_lengths(rng, batch, max_len, shape)
    for b in range(batch):
        n = int(lens[b])
        h = zipf.sample(rng, n)
        seen = set(h.tolist())
        ng = rng.integers(1, num_items + 1, size=n - 1)
        for j in range(n - 1):               # resample collisions with the history
            while int(ng[j]) in seen and len(seen) < num_items:
                ng[j] = rng.integers(1, num_items + 1)
        pad = max_len - (n - 1)
        seq[b, pad:] = h[:-1]
        pos[b, pad:] = h[1:]
        neg[b, pad:] = ng
    return seq, pos, neg


def bert_batch(rng, batch, max_len, num_items, mask_prob=0.2, shape="ml-1m", zipf=None):
    """Returns (tokens, labels) int64 arrays of shape (batch, max_len)."""
    zipf = zipf or ZipfItems(num_items)
    tokens = np.zeros((batch, max_len), np.int64)
    labels = np.zeros((batch, max_len), np.int64)
    lens = np.minimum(history_lengths(rng, batch, max_len, shape), max_len)
    mask_token = num_items + 1
    for b in range(batch):
        n = int(lens[b])
        s = zipf.sample(rng, n)
        pr = rng.random(n)
        hit = pr < mask_prob
        sub = pr / mask_prob
        tok = s.copy()
        tok[hit & (sub < 0.8)] = mask_token
        rnd = hit & (sub >= 0.8) & (sub < 0.9)
        tok[rnd] = rng.integers(1, num_items + 1, size=int(rnd.sum()))
        lab = np.where(hit, s, 0)
        tokens[b, max_len - n:] = tok
        labels[b, max_len - n:] = lab
    return tokens, labels


def user_histories(rng, n_users, max_len, num_items, shape="ml-1m", zipf=None):
    """Synthetic per-user training histories (list of item-id lists, as ``data_partition`` yields
    ``user_train``): config-shaped lengths, Zipf item ids.  Input of rbm_amd.dataloaders.DeviceWarpSampler."""
    zipf = zipf or ZipfItems(num_items)
    lens = history_lengths(rng, n_users, max_len, shape)
    return [zipf.sample(rng, int(n)).tolist() for n in lens]
