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


# ------------------------------------------------------------------------------------------------------------------
# Leave-one-out train / eval streams with sequential structure (the HR@10 parity run at the benchmarked shape).
# Zipf-only histories teach a model item popularity and nothing else; here each item has a few fixed successors, so
# ranking the held-out item needs the attention over the history.  Split and candidates follow the reference:
# ``BS/dataloaders`` data_partition (train = all but the last two items, val = second last, test = last),
# ``WarpSampler`` batches (``BS/dataloaders/sas.py:65-79``), ``SASEvalDataset`` (``:125-153``: the last max_len
# items, left padding, candidates = answer + negatives) with ``RandomNegativeSampler``'s 100 negatives per user
# (uniform over 1..V, not seen by the user, no repeats; ``BS/dataloaders/negative_samplers/random.py``).

def loo_users(rng, n_users, max_len, num_items, follow=0.7, n_succ=3, shape="ml-1m", zipf=None):
    """Per-user histories (train, val, test): history lengths as `history_lengths` + 2; the first item Zipf, each
    next item one of its predecessor's `n_succ` fixed successors with probability `follow`, else Zipf."""
    zipf = zipf or ZipfItems(num_items)
    succ = zipf.sample(rng, (num_items + 1, n_succ))
    lens = history_lengths(rng, n_users, max_len, shape) + 2
    train, val, test = [], [], []
    for n in lens.tolist():
        h = np.empty(n, np.int64)
        h[0] = zipf.sample(rng, 1)[0]
        jump = rng.random(n) < follow
        k = rng.integers(0, n_succ, size=n)
        z = zipf.sample(rng, n)
        for j in range(1, n):
            h[j] = succ[h[j - 1], k[j]] if jump[j] else z[j]
        train.append(h[:-2])
        val.append(int(h[-2]))
        test.append(int(h[-1]))
    return train, val, test


def loo_train_batch(rng, train, batch, max_len, num_items):
    """One WarpSampler batch (seq, pos, neg) over the users' train histories: a uniform user, seq = its history
    shifted by one, pos the next items, neg uniform items outside the history, the last max_len positions, left
    padding."""
    seq = np.zeros((batch, max_len), np.int64)
    pos = np.zeros((batch, max_len), np.int64)
    neg = np.zeros((batch, max_len), np.int64)
    users = rng.integers(0, len(train), size=batch)
    for b, u in enumerate(users.tolist()):
        h = train[u]
        n = min(len(h) - 1, max_len)
        seen = set(h.tolist())
        ng = rng.integers(1, num_items + 1, size=n)
        for j in range(n):
            while int(ng[j]) in seen and len(seen) < num_items:
                ng[j] = rng.integers(1, num_items + 1)
        seq[b, max_len - n:] = h[-n - 1:-1]
        pos[b, max_len - n:] = h[-n:]
        neg[b, max_len - n:] = ng
    return seq, pos, neg


def loo_eval_set(rng, train, val, test, max_len, num_items, n_neg=100):
    """The test split as SASEvalDataset serves it: seq = (train + val)[-max_len:] left-padded, candidates = [test]
    + n_neg negatives never seen by the user (no repeats), labels = [1, 0 ... 0].  Returns int64 arrays."""
    U = len(train)
    seq = np.zeros((U, max_len), np.int64)
    cand = np.zeros((U, 1 + n_neg), np.int64)
    for u in range(U):
        h = np.append(train[u], val[u])[-max_len:]
        seq[u, max_len - len(h):] = h
        seen = set(train[u].tolist()) | {val[u], test[u]}
        negs = []
        while len(negs) < n_neg:
            i = int(rng.integers(1, num_items + 1))
            if i not in seen and i not in negs:
                negs.append(i)
        cand[u, 0] = test[u]
        cand[u, 1:] = negs
    labels = np.zeros_like(cand)
    labels[:, 0] = 1
    return seq, cand, labels
