"""HR@10 parity (BASELINE.json metric: "... HR@10 parity").

The reference's validation computes candidate scores with the model (SAS.predict,
BS/models/sas_model/sas.py:107-118; BERT last-position logits gathered at the candidates,
BS/trainers/bert.py:43-52) and ranks them with recalls_ndcgs_and_mrr_for_ks
(BS/trainers/utils.py:28-57; Recall@k = HR@k with one positive).  Here the HIP path's scores and
the fp64 oracle's scores on the SAME weights and candidates give identical HR/NDCG@k in fp32 mode
and HR@10 within one user's worth in bf16 mode.  The SAS weights are the REFERENCE's own trained
weights after 1000 Adam steps (tests/golden/sas_curve.npz "final/"), so the ranking is a real one.
The ranking function is the oracle restatement pinned to the reference by tests/test_oracle.py.
"""
import argparse

import numpy as np
import pytest
import torch

from conftest import load_golden, rel

pytestmark = pytest.mark.gpu
KS = [1, 5, 10]


def _eval_batch(V, T, B, C, seed):
    import rbm_amd.data as synth
    rng = np.random.default_rng(seed)
    seq, pos, _ = synth.sas_batch(rng, B, T, V, zipf=synth.ZipfItems(V))
    target = pos[:, -1]
    neg = np.stack([rng.choice(np.setdiff1d(np.arange(1, V + 1), [t]), C - 1, replace=False) for t in target])
    cand = np.concatenate([target[:, None], neg], axis=1)
    labels = np.zeros_like(cand)
    labels[:, 0] = 1
    return seq, cand, labels


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_sas_hr_at_10_matches_oracle(dtype):
    import rbm_amd  # noqa: F401
    from oracle import metrics as om
    from oracle import sas as osas
    from rbm_amd.models import model_factory
    z = load_golden("sas_curve")
    V, T, d, L, h = (int(z[k]) for k in ("V", "T", "d", "L", "h"))
    a = argparse.Namespace(model_code="sas", num_items=V, max_len=T, device="cuda", sas_hidden_units=d,
                           sas_num_blocks=L, sas_heads=h, sas_dropout=0.0, l2_emb=0.0, rs_dtype=dtype)
    m = model_factory(a)
    m.load_state_dict({k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("final/")})
    m.eval()
    B, C = 256, 21
    seq, cand, labels = _eval_batch(V, T, B, C, seed=123)
    ours = m.predict(torch.from_numpy(seq).int(), torch.from_numpy(cand).int()).cpu().numpy()
    P = {k[6:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("final/")}
    ref = osas.predict(P, torch.from_numpy(seq), torch.from_numpy(cand), L, h).numpy()
    mo, mr = om.recalls_ndcgs_and_mrr_for_ks(ours, labels, KS), om.recalls_ndcgs_and_mrr_for_ks(ref, labels, KS)
    assert mr["Recall@10"] > 0.75           # trained (0.83) vs 0.61 at init, 0.48 by chance
    if dtype == "fp32":
        assert rel(ours, ref) < 1e-5
        assert mo == mr, (mo, mr)
    else:
        assert rel(ours, ref) < 3e-2
        assert abs(mo["Recall@10"] - mr["Recall@10"]) <= 2.0 / B, (mo, mr)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_bert_hr_at_10_matches_oracle(dtype):
    import rbm_amd  # noqa: F401
    from oracle import bert as obert
    from oracle import metrics as om
    from rbm_amd.models import model_factory
    z = load_golden("bert_mid")
    V, T, d, L, h = (int(z[k]) for k in ("V", "T", "d", "L", "h"))
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=d,
                           bert_num_blocks=L, bert_num_heads=h, bert_dropout=0.0, bert_hidden_dropout=0.0,
                           bert_mask_prob=0.2, model_init_seed=4, rs_dtype=dtype)
    m = model_factory(a)
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p/")})
    m.eval()
    B, C = 64, 101
    seq, cand, labels = _eval_batch(V, T, B, C, seed=7)
    seq = np.concatenate([seq[:, 1:], np.full((B, 1), V + 1)], axis=1)   # eval appends [MASK] (dataloaders/bert.py:128-142)
    with torch.no_grad():                                           # validate() runs under no_grad (base.py:151-183)
        logits = m(torch.from_numpy(seq).cuda())
        ours = logits[:, -1, :].gather(1, torch.from_numpy(cand).cuda()).cpu().numpy()    # trainers/bert.py:47-49
    P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
    ref = obert.forward(P, torch.from_numpy(seq), L, h)[:, -1, :].gather(1, torch.from_numpy(cand)).numpy()
    mo, mr = om.recalls_ndcgs_and_mrr_for_ks(ours, labels, KS), om.recalls_ndcgs_and_mrr_for_ks(ref, labels, KS)
    if dtype == "fp32":
        assert rel(ours, ref) < 1e-5
        assert mo == mr, (mo, mr)
    else:
        assert rel(ours, ref) < 3e-2
        assert abs(mo["Recall@10"] - mr["Recall@10"]) <= 2.0 / B, (mo, mr)
    # the eval route without full-vocabulary logits (BERTModel.predict -> rs_candidate_scores) gives the same scores
    # as the gathered logits (same encoder; only the head's summation order differs) and the same metrics
    from rbm_amd.metrics import calculate_metrics
    pred = m.predict(torch.from_numpy(seq), torch.from_numpy(cand)).cpu().numpy()
    assert rel(pred, ours) < (1e-6 if dtype == "fp32" else 1e-2)
    mp = calculate_metrics(m, (torch.from_numpy(seq), torch.from_numpy(cand), torch.from_numpy(labels)), KS)
    mg = {k: v for k, v in om.recalls_ndcgs_and_mrr_for_ks(ours, labels, KS).items()}
    for k in mg:
        if dtype == "fp32":
            assert abs(mp[k] - mg[k]) < 1e-6, (k, mp[k], mg[k])
        elif k.startswith("Recall"):
            assert abs(mp[k] - mg[k]) <= 1.0 / B + 1e-6, (k, mp[k], mg[k])


def test_bert_predict_at_1m_items_without_full_logits():
    """cfg5's eval shape (V = 1,000,000, T = 200, d = 256, 4 blocks, B = 64, 101 candidates): BERTModel.predict
    allocates no (B, T, V+1) logits (51 GB fp32) and equals the last position's hidden state times the gathered
    out.weight rows plus out.bias (torch fp64 on the same hidden state)."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    V, T, d, L, h, B, C = 1_000_000, 200, 256, 4, 2, 64, 101
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=d,
                           bert_num_blocks=L, bert_num_heads=h, bert_dropout=0.1, bert_hidden_dropout=0.1,
                           bert_mask_prob=0.2, model_init_seed=0, rs_dtype="bf16")
    m = model_factory(a)
    m.eval()
    rng = np.random.default_rng(3)
    seq = rng.integers(1, V + 1, size=(B, T))
    seq[:, :50] = 0
    seq[:, -1] = V + 1
    cand = rng.integers(1, V + 1, size=(B, C))
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    scores = m.predict(torch.from_numpy(seq), torch.from_numpy(cand))
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated() - base < 2 * 1024 ** 3
    eng = m.engine()
    xL, _ = eng.encode(torch.from_numpy(seq).cuda(), False)
    hl = xL.view(B, T, d)[:, -1, :].double()
    W = eng.W("out.weight").double()[torch.from_numpy(cand).cuda()]
    ref = torch.einsum("bd,bcd->bc", hl, W) + eng.Wf("out.bias").double()[torch.from_numpy(cand).cuda()]
    assert rel(scores.cpu().numpy(), ref.cpu().numpy()) < 1e-5
    assert torch.isfinite(scores).all()
    with pytest.raises(IndexError):
        m.predict(torch.from_numpy(seq), torch.from_numpy(cand + V))
