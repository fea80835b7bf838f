"""Ranking metrics on the GPU: ``recalls_ndcgs_and_mrr_for_ks`` (BS/trainers/utils.py:28-57) through
rs_rank_metrics.  Same inputs (scores, labels: (B, C)) and the same dict keys; ranks follow a stable
descending sort (ties by candidate index)."""
import torch

from . import ops
from .engine_util import as_ids


def recalls_ndcgs_and_mrr_for_ks(scores, labels, ks):
    dev = scores.device
    if dev.type != "cuda":
        raise RuntimeError("rbm_amd.metrics runs on the GPU (rs_rank_metrics); there is no CPU fallback")
    ks = sorted(ks, reverse=True)
    s = scores.detach().float().contiguous()
    lab = labels.detach().to(device=dev, dtype=torch.float32).contiguous()
    R = s.shape[0]
    ks_dev = torch.tensor(ks, dtype=torch.int32, device=dev)
    ws = torch.empty(3 * len(ks) * R, dtype=torch.float32, device=dev)
    out = torch.empty(3 * len(ks), dtype=torch.float32, device=dev)
    ops.rank_metrics(s, lab, ks_dev, ws, out)
    v = out.cpu().tolist()
    res = {}
    for q, k in enumerate(ks):
        res["Recall@%d" % k] = v[3 * q]
        res["NDCG@%d" % k] = v[3 * q + 1]
        res["MRR@%d" % k] = v[3 * q + 2]
    return res


def calculate_metrics(model, batch, metric_ks):
    """The trainers' ``calculate_metrics`` (BS/trainers/sas.py:56-62, BS/trainers/bert.py:43-52) on the GPU: the
    model's scores at the candidates -- ``SASModel.predict`` / ``BERTModel.predict`` (the last position only, no
    (B, T, V+1) logits) -- ranked by rs_rank_metrics.  batch = (seqs, candidates, labels) as the eval loaders
    yield it."""
    seqs, candidates, labels = batch
    dev = model.engine().flat.device if hasattr(model, "engine") else next(model.parameters()).device
    with torch.no_grad():
        scores = model.predict(as_ids(seqs, dev), as_ids(candidates, dev))
    return recalls_ndcgs_and_mrr_for_ks(scores, torch.as_tensor(labels).to(dev), metric_ks)
