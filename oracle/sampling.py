"""Training-batch construction oracle (TEST INFRASTRUCTURE ONLY).

Replays the reference's batch builders on the random draws the device samplers recorded
(``rs_sas_sample_draws`` / ``rs_bert_mask_draws``), so the construction itself -- window, truncation,
padding, the one-step shift, negatives drawn outside the window with item 0 allowed, the 80/10/10 cloze
rule, labels, the epoch's user order -- is compared bit for bit with the device batch:

- ``sas_sample`` restates ``sample_function.sample`` (``BS/dataloaders/sas.py:71-79``) and ``random_neq``
  (``:65-67``);
- ``bert_getitem`` restates ``BertTrainDataset.__getitem__`` (``BS/dataloaders/bert.py:77-110``);
- ``bert_epoch_user`` restates the shuffling ``DataLoader`` order (``bert.py:27-28``): batch c, row b of an
  epoch reads user perm[c * batch + b].

Where the reference calls numpy's stream (``np.random.randint`` for the user, ``np.random.randint`` indexing
the complement for a negative, ``rng.rand`` / ``rng.randint`` for masking), each call site here consumes the
next recorded device draw instead.  ``random_neq`` draws uniformly from the complement of the window by
indexing a list; the device draws uniformly from {0..item_num} and rejects values inside the window, which
is the same distribution -- the replay takes the first recorded candidate outside the window (the
distributional equality itself is checked separately, tests/test_sampler_gpu.py's chi-square test).
"""


def random_neq(l, r, exclusive, size, candidates):
    """``random_neq(l, r, exclusive, size)`` (sas.py:65-67) with the uniform index into the complement replaced
    by rejection over the recorded candidates: per draw, the first of ``candidates[j]`` in [l, r] outside
    ``exclusive`` (None if every recorded candidate was rejected)."""
    out = []
    for j in range(size):
        pick = None
        for c in candidates[j]:
            if l <= c <= r and c not in exclusive:
                pick = int(c)
                break
        out.append(pick)
    return out


def sas_sample(user_train, user, item_num, max_len, candidates):
    """``sample()`` of sample_function (sas.py:71-79) for the drawn ``user``; candidates[t] = the recorded
    negative candidates of output position t (t = padding_len .. max_len - 1 are used)."""
    train = list(user_train[user])[-max_len:]
    padding_len = max_len - len(train) + 1

    seq = padding_len * [0] + train[:-1]
    pos = padding_len * [0] + train[1:]
    neg = padding_len * [0] + random_neq(0, item_num, set(train), len(train) - 1, candidates[padding_len:])
    return seq, pos, neg


def bert_getitem(u2seq, user, max_len, mask_prob, mask_token, draws):
    """``BertTrainDataset.__getitem__`` (bert.py:77-110).  draws[i] = (prob, item) for item i of the user's FULL
    history: the reference's ``rng.rand()`` for that item and, where the 10 % branch calls it,
    ``rng.randint(1, num_items + 1)`` (None elsewhere).  (The device sampler draws only for the items the final
    ``[-max_len:]`` keeps -- the masking of a dropped item cannot reach the output -- and its recorded uniform is
    k / 2^24; tests pass prob = 1.0, i.e. unmasked, for the dropped items.)"""
    seq = list(u2seq[user])

    tokens = []
    labels = []
    for i, s in enumerate(seq):
        prob, rnd = draws[i]
        if prob < mask_prob:
            prob /= mask_prob

            if prob < 0.8:
                tokens.append(mask_token)
            elif prob < 0.9:
                tokens.append(int(rnd))
            else:
                tokens.append(s)

            labels.append(s)
        else:
            tokens.append(s)
            labels.append(0)

    tokens = tokens[-max_len:]
    labels = labels[-max_len:]

    mask_len = max_len - len(tokens)

    tokens = [0] * mask_len + tokens
    labels = [0] * mask_len + labels
    return tokens, labels


def device_bert_draws(history_len, max_len, rec):
    """Full-history draws for bert_getitem from a device record row rec[t] = (k, item) per output position t (-1 on
    padding): prob = k / 2^24 for the kept tail, 1.0 (unmasked) for the items truncation drops."""
    kept = min(history_len, max_len)
    pad = max_len - kept
    out = [(1.0, None)] * (history_len - kept)
    for t in range(pad, max_len):
        k, item = rec[t]
        out.append((float(k) / 16777216.0, int(item)))
    return out


def bert_epoch_user(perm, batch_size, batch_index, row):
    """The user a shuffled epoch's batch ``batch_index`` (0-based) reads at ``row``: DataLoader(shuffle=True)
    walks one permutation of the users in order (bert.py:27-28); the fixed-shape device loader wraps modulo
    the user count."""
    return int(perm[(batch_index * batch_size + row) % len(perm)])
