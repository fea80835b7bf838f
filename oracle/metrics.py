"""Ranking-metric oracle (TEST INFRASTRUCTURE ONLY).

Restates ``recalls_ndcgs_and_mrr_for_ks`` (``BS/trainers/utils.py:28-57``) in
numpy: Recall@k (= HR@k with one positive), NDCG@k, MRR@k over (B, C) score /
0-1 label matrices.  Ties are broken like ``torch.argsort`` on CPU for the
distinct scores used in the fixtures (stable descending order).
"""
import numpy as np


def recalls_ndcgs_and_mrr_for_ks(scores, labels, ks):
    scores = np.asarray(scores, dtype=np.float64)
    labels = np.asarray(labels, dtype=np.float64)
    answer_count = labels.sum(1)
    rank = np.argsort(-scores, axis=1, kind="stable")
    out = {}
    for k in sorted(ks, reverse=True):
        cut = rank[:, :k]
        hits = np.take_along_axis(labels, cut, axis=1)
        out["Recall@%d" % k] = float((hits.sum(1) / answer_count).mean())
        w = 1.0 / np.log2(np.arange(2, 2 + k, dtype=np.float64))
        dcg = (hits * w).sum(1)
        idcg = np.array([w[:int(min(n, k))].sum() for n in answer_count])
        out["NDCG@%d" % k] = float((dcg / idcg).mean())
        out["MRR@%d" % k] = float((hits * (1.0 / np.arange(1, k + 1))).sum(1).mean())
    return out
