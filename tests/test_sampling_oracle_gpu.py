"""On-device batch builders vs the oracle's replay of the reference construction, bit for bit.

rs_sas_sample_draws / rs_bert_mask_draws record the draws each row consumed (user, candidate negatives,
masking uniforms and replacement items); oracle/sampling.py replays sample_function (BS/dataloaders/sas.py:65-79)
and BertTrainDataset.__getitem__ (BS/dataloaders/bert.py:77-110) on them.  The batches the training step reads
(seq, pos, neg / tokens, labels) must equal the replay exactly, and the plain entry points (no record) must
produce the same batch as the recording ones.
"""
import numpy as np
import pytest
import torch

from oracle import sampling as osmp

pytestmark = pytest.mark.gpu


def _histories(n_users, V, rng, min_len=1, max_len=300):
    return [list(map(int, rng.integers(1, V + 1, size=int(rng.integers(min_len, max_len + 1)))))
            for _ in range(n_users)]


# (users, V, max_len, batch, history lengths): windows shorter / longer than max_len (truncation, the first
# position always padding), 1-item histories (all padding), a small catalogue where most draws are rejected
# (V = 60 against windows of up to 50), and the cfg2 shape (V = 3,416, T = 200, B = 128)
@pytest.mark.parametrize("n_users,V,T,B,lo,hi", [(200, 500, 50, 64, 1, 300), (40, 60, 50, 32, 1, 120),
                                                 (300, 3416, 200, 128, 20, 400), (16, 100, 8, 16, 1, 2)])
def test_sas_sampler_equals_reference_construction(n_users, V, T, B, lo, hi):
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceWarpSampler
    rng = np.random.default_rng(V + T)
    users = _histories(n_users, V, rng, lo, hi)
    smp = DeviceWarpSampler(users, V, B, T, seed=7)
    twin = DeviceWarpSampler(users, V, B, T, seed=7)
    for step in range(3):
        seq, pos, neg = (torch.empty(B, T, dtype=torch.int64, device="cuda") for _ in range(3))
        draws = torch.empty(B, 1 + 256 * T, dtype=torch.int64, device="cuda")
        smp.sample_into(seq, pos, neg, draws)
        plain = twin.sample()
        got = [x.cpu().numpy() for x in (seq, pos, neg)]
        for a, b in zip(got, plain):
            assert np.array_equal(a, b.cpu().numpy()), "recording changed the batch"
        dr = draws.cpu().numpy()
        for b in range(B):
            u = int(dr[b, 0])
            assert 0 <= u < n_users
            cands = dr[b, 1:].reshape(T, 256)
            rs, rp, rn = osmp.sas_sample(users, u, V, T, cands)
            assert None not in rn, "every recorded candidate rejected"
            assert got[0][b].tolist() == rs, (step, b, "seq")
            assert got[1][b].tolist() == rp, (step, b, "pos")
            assert got[2][b].tolist() == rn, (step, b, "neg")


@pytest.mark.parametrize("n_users,V,T,B,p,lo,hi", [(64, 700, 40, 16, 0.3, 1, 90), (256, 26744, 200, 64, 0.2, 5, 400),
                                                   (20, 50, 10, 8, 1.0, 1, 30), (24, 300, 16, 8, 0.15, 1, 3)])
def test_bert_masker_equals_reference_construction(n_users, V, T, B, p, lo, hi):
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceBertMasker
    rng = np.random.default_rng(V + T)
    users = _histories(n_users, V, rng, lo, hi)
    m = DeviceBertMasker(users, V, B, T, p, seed=5)
    twin = DeviceBertMasker(users, V, B, T, p, seed=5)
    m.new_epoch()
    twin.new_epoch()
    assert torch.equal(m.perm, twin.perm)
    perm = m.perm.cpu().numpy()
    assert sorted(perm.tolist()) == list(range(n_users))
    pf = float(np.float32(p))               # the ABI's fp32 mask_prob, as the kernel compares it
    for c in range(len(m) + 1):             # one batch past the epoch wraps to its start
        tok, lab = (torch.empty(B, T, dtype=torch.int64, device="cuda") for _ in range(2))
        draws = torch.empty(B, 1 + 2 * T, dtype=torch.int64, device="cuda")
        m.sample_into(tok, lab, draws)
        pt, pl = twin.sample()
        tok, lab, dr = tok.cpu().numpy(), lab.cpu().numpy(), draws.cpu().numpy()
        assert np.array_equal(tok, pt.cpu().numpy()) and np.array_equal(lab, pl.cpu().numpy())
        for b in range(B):
            u = int(dr[b, 0])
            assert u == osmp.bert_epoch_user(perm, B, c, b)
            d = dr[b, 1:].reshape(T, 2)
            live = d[:, 0] >= 0
            assert ((d[live, 1] >= 1) & (d[live, 1] <= V)).all(), "replacement item outside 1..num_items"
            rt, rl = osmp.bert_getitem(users, u, T, pf, V + 1, osmp.device_bert_draws(len(users[u]), T, d))
            assert tok[b].tolist() == rt, (c, b, "tokens")
            assert lab[b].tolist() == rl, (c, b, "labels")
