"""Pin the CPU oracle against golden vectors generated from the reference itself
(tools/gen_golden.py imports BS/models + BS/trainers).  CPU-only."""
import numpy as np
import pytest
import torch

from conftest import golden_params, load_golden, rel
from oracle import bert as obert
from oracle import metrics as ometrics
from oracle import optim as ooptim
from oracle import sas as osas


@pytest.mark.parametrize("name", ["sas_tiny", "sas_mid"])
def test_sas_oracle_matches_reference(name):
    z = load_golden(name)
    P = golden_params(z)
    seq, pos, neg = (torch.from_numpy(z[k]) for k in ("seq", "pos", "neg"))
    loss, pl, nl, grads = osas.loss_and_grads(P, seq, pos, neg, int(z["L"]), int(z["h"]))
    assert rel(pl, z["pos_logits"]) < 1e-5
    assert rel(nl, z["neg_logits"]) < 1e-5
    assert abs(loss.item() - float(z["loss"])) < 1e-5 * max(1.0, abs(float(z["loss"])))
    gscale = max(np.linalg.norm(z["g/" + k]) for k in P)
    for k, g in grads.items():
        ref = z["g/" + k]
        if k.endswith("in_proj_bias"):
            # key-bias rows d..2d are analytically zero (softmax shift invariance)
            d = int(z["d"])
            assert np.linalg.norm(g[d:2 * d].numpy()) <= 1e-5 * gscale
            g, ref = torch.cat([g[:d], g[2 * d:]]), np.concatenate([ref[:d], ref[2 * d:]])
        assert rel(g, ref) < 1e-4, k


def test_sas_oracle_predict():
    z = load_golden("sas_tiny")
    P = golden_params(z)
    s = osas.predict(P, torch.from_numpy(z["seq"]), torch.from_numpy(z["cand"]), int(z["L"]), int(z["h"]))
    assert rel(s, z["cand_scores"]) < 1e-5


@pytest.mark.parametrize("name", ["bert_tiny", "bert_mid"])
def test_bert_oracle_matches_reference(name):
    z = load_golden(name)
    P = golden_params(z)
    tok, lab = torch.from_numpy(z["tokens"]), torch.from_numpy(z["labels"])
    loss, logits, grads = obert.loss_and_grads(P, tok, lab, int(z["L"]), int(z["h"]))
    assert rel(logits, z["logits"]) < 1e-5
    assert abs(loss.item() - float(z["loss"])) < 1e-5 * max(1.0, float(z["loss"]))
    for k, g in grads.items():
        ref = z["g/" + k]
        if np.linalg.norm(ref) == 0:
            assert np.linalg.norm(g.numpy()) == 0, k
            continue
        if "linear_layers.1.bias" in k:   # key bias: analytically zero gradient
            continue
        assert rel(g, ref) < 1e-4, k


@pytest.mark.parametrize("name", ["bert_tiny", "bert_mid"])
def test_bert_oracle_labelled_rows_head_equals_full(name):
    """The oracle's labelled-rows output layer (what the 1M-class tests use) against its full form and the
    reference's goldens: same loss, logits of the labelled rows, every gradient."""
    z = load_golden(name)
    P = golden_params(z)
    tok, lab = torch.from_numpy(z["tokens"]), torch.from_numpy(z["labels"])
    loss, logits, grads = obert.loss_and_grads(P, tok, lab, int(z["L"]), int(z["h"]), labelled_only=True)
    full = z["logits"].reshape(-1, z["logits"].shape[-1])[lab.reshape(-1).numpy() != 0]
    assert logits.shape == full.shape and rel(logits, full) < 1e-5
    assert abs(loss.item() - float(z["loss"])) < 1e-5 * max(1.0, float(z["loss"]))
    _, _, g_full = obert.loss_and_grads(P, tok, lab, int(z["L"]), int(z["h"]))
    for k, g in grads.items():
        if float(g_full[k].norm()) == 0:
            assert float(g.norm()) == 0, k
            continue
        assert rel(g, g_full[k]) < 1e-5, k     # fp32 parameters: the summation order of the head's reductions


def test_adam_oracle_matches_torch():
    torch.manual_seed(0)
    p0 = [torch.randn(7, 5), torch.randn(11)]
    a = [t.clone().requires_grad_(True) for t in p0]
    b = [t.clone() for t in p0]
    opt = torch.optim.Adam(a, lr=1e-3, weight_decay=0.01)
    ora = ooptim.AdamOracle(b, lr=1e-3, weight_decay=0.01)
    for _ in range(5):
        gs = [torch.randn_like(t) for t in p0]
        for t, g in zip(a, gs):
            t.grad = g.clone()
        opt.step()
        ora.step(gs)
    for x, y in zip(a, b):
        assert torch.equal(x.detach(), y)


def test_metrics_oracle_matches_reference():
    z = load_golden("metrics")
    m = ometrics.recalls_ndcgs_and_mrr_for_ks(z["scores"], z["labels"], list(z["ks"]))
    for k in m:
        assert abs(m[k] - float(z["m/" + k])) < 1e-6, k


def test_sas_curve_first_steps_oracle():
    """Replay the first 20 steps of the 1000-step reference curve with oracle + AdamOracle."""
    import rbm_amd.data as synth
    z = load_golden("sas_curve")
    P = {k: v.clone() for k, v in golden_params(z).items()}
    V, T, B = int(z["V"]), int(z["T"]), int(z["B"])
    rng = np.random.default_rng(int(z["seed"]))
    zipf = synth.ZipfItems(V)
    opt = ooptim.AdamOracle(list(P.values()), lr=float(z["lr"]))
    for step in range(20):
        seq, pos, neg = (torch.from_numpy(a) for a in synth.sas_batch(rng, B, T, V, zipf=zipf))
        loss, _, _, grads = osas.loss_and_grads(P, seq, pos, neg, int(z["L"]), int(z["h"]))
        assert abs(loss.item() - z["losses"][step]) < 1e-4, step
        opt.step([grads[k] for k in P])
