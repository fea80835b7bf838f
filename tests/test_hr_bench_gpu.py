"""HR@10 parity at the BENCHMARKED configuration (BASELINE.json metric "... HR@10 parity"; configs[1]: 3,416 items,
T = 200, d = 128, 2 blocks, 1 head, B = 128, dropout 0.2).

tests/golden/sas_hr_bench.npz (tools/gen_golden.py --bench-hr) holds the REFERENCE's own run: its SASModel trained by
its own SASTrainer.calculate_loss + Adam (BS/trainers/sas.py:34-54, BS/trainers/base.py:114-123,225-228) for 1000
steps on leave-one-out WarpSampler batches (rbm_amd.data.loo_*: histories with fixed item successors, so ranking
needs the attention, not just popularity), then evaluated as its validate() does (BS/trainers/sas.py:56-62,
BS/dataloaders/sas.py:125-153) on all 6,040 users with 1 + 100 candidates by recalls_ndcgs_and_mrr_for_ks
(BS/trainers/utils.py:28-57).  Recall@10 = HR@10 (one positive per row).

(a) the HIP eval path (SASModel.predict -> rs_candidate_scores, rs_rank_metrics) on the reference's trained weights
    gives the reference's metrics: fp32 the same hit count at every k, bf16 HR@10 within a stated few users;
(b) the FUSED TRAINER (the benchmarked bf16 step, and the fp32 parity mode) from the reference's initial weights
    over the same 1000 batches ends at the reference-trained model's HR@10 within 0.01.

Measured (MI355X): the reference trains HR@10 0.166 -> 0.886 (5,353 of 6,040 users hit).  (a) fp32: the same hits at
k = 1 / 5 / 10 / 20, scores 7e-7 from the reference's; bf16: HR@10 the same 5,353 hits (k = 1: 4,122 vs 4,126),
scores 1.2e-2.  (b) bf16 fused trainer HR@10 0.8877 (gap +0.0015), NDCG@10 0.7833 vs 0.7838, last-100-step mean loss
0.51927 vs 0.51914; fp32 fused trainer 0.8882 (gap +0.0020)."""
import argparse

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _data(z):
    import rbm_amd.data as synth
    V, T = int(z["V"]), int(z["T"])
    train, val, test = synth.loo_users(np.random.default_rng(int(z["data_seed"])), int(z["users"]), T, V)
    seq, cand, labels = synth.loo_eval_set(np.random.default_rng(int(z["eval_seed"])), train, val, test, T, V)
    assert int((seq * 31 + 7).sum() + (cand * 131).sum()) == int(z["eval_checksum"])
    return train, seq, cand, labels


def _model(z, dtype, p=0.0):
    from rbm_amd.models import model_factory
    torch.manual_seed(int(z["init_seed"]))         # the reference's initial weights (pinned: test_hr_bench_fixture)
    a = argparse.Namespace(model_code="sas", num_items=int(z["V"]), max_len=int(z["T"]), device="cuda",
                           sas_hidden_units=int(z["d"]), sas_num_blocks=int(z["L"]), sas_heads=int(z["h"]),
                           sas_dropout=p, l2_emb=0.0, rs_dtype=dtype)
    return model_factory(a)


def _eval(m, seq, cand, labels, ks):
    """All users' candidate scores (SASModel.predict) ranked once by rs_rank_metrics, as the reference ranks its
    whole eval set; the trainers' calculate_metrics route is checked on one eval batch against the same scores."""
    from rbm_amd.metrics import calculate_metrics, recalls_ndcgs_and_mrr_for_ks
    m.eval()
    with torch.no_grad():
        sc = torch.cat([m.predict(torch.from_numpy(seq[i:i + 1024]), torch.from_numpy(cand[i:i + 1024]))
                        for i in range(0, len(seq), 1024)])
    out = recalls_ndcgs_and_mrr_for_ks(sc, torch.from_numpy(labels).cuda(), ks)
    mb = calculate_metrics(m, (seq[:256], cand[:256], labels[:256]), ks)
    mr = recalls_ndcgs_and_mrr_for_ks(sc[:256], torch.from_numpy(labels[:256]).cuda(), ks)
    assert all(abs(mb[k] - mr[k]) < 1e-6 for k in mb), (mb, mr)
    m.train()
    return sc.cpu().numpy(), out


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_hr_at_10_on_reference_trained_weights(dtype):
    import rbm_amd  # noqa: F401
    z = load_golden("sas_hr_bench")
    ks = [int(k) for k in z["ks"]]
    _, seq, cand, labels = _data(z)
    U = len(seq)
    m = _model(z, dtype)
    m.load_state_dict({k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("final/")})
    sc, mo = _eval(m, seq, cand, labels, ks)
    ref = {k[2:]: float(z[k]) for k in z.files if k.startswith("m/")}
    head = z["scores_head"]
    srel = np.linalg.norm(sc[:512] - head) / np.linalg.norm(head)
    hits = {k: (round(mo[f"Recall@{k}"] * U), round(ref[f"Recall@{k}"] * U)) for k in ks}
    print(dtype, "HR@10 ours", mo["Recall@10"], "reference", ref["Recall@10"], "hits", hits, "score rel", srel)
    assert ref["Recall@10"] > float(z["m0/Recall@10"]) + 0.1          # a trained ranking, not the init's
    if dtype == "fp32":
        assert srel < 1e-5
        for k in ks:                         # the same number of users hit at every k
            assert hits[k][0] == hits[k][1], (k, hits[k])
            assert abs(mo[f"NDCG@{k}"] - ref[f"NDCG@{k}"]) < 1e-5 and abs(mo[f"MRR@{k}"] - ref[f"MRR@{k}"]) < 1e-5
    else:
        # bf16 scores (2e-3 relative) reorder near-tied candidates of a few users
        assert srel < 3e-2
        assert abs(hits[10][0] - hits[10][1]) <= 12, hits[10]          # <= 0.2 % of the 6,040 users


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_fused_trainer_reaches_reference_hr_at_10(dtype):
    """The benchmarked fused step (bf16) and the fp32 parity mode, trained like the reference (same initial weights,
    the same 1000 batches, dropout 0.2 -- masks from the kernels' counter hash, not torch's bernoulli stream -- Adam
    lr 1e-3), end within 0.01 HR@10 of the reference-trained model on the same eval set."""
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    z = load_golden("sas_hr_bench")
    ks = [int(k) for k in z["ks"]]
    train, seq, cand, labels = _data(z)
    V, T, B = int(z["V"]), int(z["T"]), int(z["B"])
    m = _model(z, dtype, p=float(z["p"]))
    m.train()
    tr = FusedTrainStep(m, lr=float(z["lr"]))
    rng = np.random.default_rng(int(z["batch_seed"]))
    losses, csum = [], 0
    for _ in range(int(z["steps"])):
        batch = synth.loo_train_batch(rng, train, B, T, V)
        csum += int(sum(((j + 1) * x).sum() for j, x in enumerate(batch)) % (1 << 40))
        losses.append(tr.step(*(torch.from_numpy(x).cuda() for x in batch)).clone())
    assert csum == int(z["batch_checksum"])                          # the reference's batches
    losses = np.array([float(x.item()) for x in losses])
    ref_l = z["losses"]
    _, mo = _eval(m, seq, cand, labels, ks)
    ref = {k[2:]: float(z[k]) for k in z.files if k.startswith("m/")}
    gap = mo["Recall@10"] - ref["Recall@10"]
    print(dtype, "trained HR@10", mo["Recall@10"], "reference", ref["Recall@10"], "gap", gap, "NDCG@10",
          mo["NDCG@10"], ref["NDCG@10"], "last-100 mean loss", losses[-100:].mean(), ref_l[-100:].mean())
    assert abs(gap) <= 0.01, (mo, ref)
    assert abs(mo["NDCG@10"] - ref["NDCG@10"]) <= 0.01
    assert abs(losses[-100:].mean() - ref_l[-100:].mean()) <= 0.01 * ref_l[-100:].mean()
