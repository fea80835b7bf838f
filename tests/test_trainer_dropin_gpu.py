"""Drop-in check: the REFERENCE's trainer code path, unchanged, on top of the HIP models.

Restates BS/trainers/sas.py:34-54 (numpy batch -> model(seq,pos,neg) -> BCEWithLogits on
np.where(pos != 0) -> + l2_emb * ||p||) and BS/trainers/bert.py:30-41 (model(seqs) -> view ->
CrossEntropyLoss(ignore_index=0)) with torch.optim.Adam over model.parameters() created AFTER
model.to(device) as BS/trainers/base.py:21,38 does, and compares 3 training steps against the CPU
oracle + oracle Adam (fp32 parity mode)."""
import argparse

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import load_golden, rel

pytestmark = pytest.mark.gpu


def _sas_calculate_loss(model, batch, l2_emb=0.0):
    seq, pos, neg = batch
    seq, pos, neg = np.array(seq), np.array(pos), np.array(neg)              # sas.py:36
    pos_logits, neg_logits = model(seq, pos, neg)                            # :37
    pos_labels = torch.ones(pos_logits.shape, device="cuda")                 # :38
    neg_labels = torch.zeros(neg_logits.shape, device="cuda")
    indices = np.where(pos != 0)                                              # :40
    bce = nn.BCEWithLogitsLoss()
    loss = bce(pos_logits[indices], pos_labels[indices])                      # :49
    loss += bce(neg_logits[indices], neg_labels[indices])
    for param in model.parameters():                                          # :51-52
        loss += l2_emb * torch.norm(param)
    return loss


def test_reference_sas_trainer_loop_on_hip_model():
    import rbm_amd  # noqa: F401
    from oracle import sas as osas
    from oracle.optim import AdamOracle
    from rbm_amd.models import model_factory
    z = load_golden("sas_mid")
    a = argparse.Namespace(model_code="sas", num_items=int(z["V"]), max_len=int(z["T"]), device="cpu",
                           sas_hidden_units=int(z["d"]), sas_num_blocks=int(z["L"]), sas_heads=int(z["h"]),
                           sas_dropout=0.0, l2_emb=0.0, rs_dtype="fp32")
    model = model_factory(a)
    model.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p/")})
    model = model.to("cuda")                                                  # base.py:21
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=0.0)     # base.py:228
    P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
    oopt = AdamOracle(list(P.values()), lr=1e-3)
    batch = (z["seq"], z["pos"], z["neg"])
    for _ in range(3):
        opt.zero_grad()                                                        # base.py:114-123
        loss = _sas_calculate_loss(model, batch)
        loss.backward()
        opt.step()
        l64, _, _, g = osas.loss_and_grads(P, *(torch.from_numpy(x) for x in batch), int(z["L"]), int(z["h"]))
        oopt.step([g[k] for k in P])
        assert abs(loss.item() - l64.item()) < 1e-4 * max(1.0, abs(l64.item()))
    sd = model.state_dict()
    d = int(z["d"])
    for k in P:
        a, b = sd[k].cpu().numpy(), P[k].numpy()
        if k.endswith("in_proj_bias"):   # the key-bias third: noise-level gradient, Adam steps it by ~lr
            a, b = np.concatenate([a[:d], a[2 * d:]]), np.concatenate([b[:d], b[2 * d:]])
        assert rel(a, b) < 1e-4, k


def test_reference_bert_trainer_loop_on_hip_model():
    import rbm_amd  # noqa: F401
    from oracle import bert as obert
    from oracle.optim import AdamOracle
    from rbm_amd.models import model_factory
    z = load_golden("bert_mid")
    a = argparse.Namespace(model_code="bert", num_items=int(z["V"]), max_len=int(z["T"]), device="cpu",
                           bert_hidden_units=int(z["d"]), bert_num_blocks=int(z["L"]), bert_num_heads=int(z["h"]),
                           bert_dropout=0.0, bert_hidden_dropout=0.0, bert_mask_prob=0.2, model_init_seed=4,
                           rs_dtype="fp32")
    model = model_factory(a).to("cuda")
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    ce = nn.CrossEntropyLoss(ignore_index=0)                                   # bert.py:11
    P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
    oopt = AdamOracle(list(P.values()), lr=1e-3)
    seqs, labels = torch.from_numpy(z["tokens"]), torch.from_numpy(z["labels"])
    for _ in range(3):
        opt.zero_grad()
        logits = model(seqs.cuda())                                            # bert.py:34
        loss = ce(logits.view(-1, logits.size(-1)), labels.cuda().view(-1))    # :36-40
        loss.backward()
        opt.step()
        l64, _, g = obert.loss_and_grads(P, seqs, labels, int(z["L"]), int(z["h"]))
        oopt.step([g[k] for k in P])
        assert abs(loss.item() - l64.item()) < 1e-4 * max(1.0, abs(l64.item()))
    sd = model.state_dict()
    for k in P:
        if "linear_layers.1.bias" in k:   # Adam turns the noise-level key-bias gradient into lr steps
            continue
        assert rel(sd[k].cpu().numpy(), P[k].numpy()) < 1e-4, k
