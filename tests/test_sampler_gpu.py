"""On-device SAS sampler (rs_sas_sample) and GPU ranking metrics (rs_rank_metrics).

The sampler cannot reproduce the reference's numpy stream (BS/dataloaders/sas.py:65-91), so it is
checked against the sampler's definition: every row is some user's last max_len items shifted by one
and left padded; negatives avoid that window, may be 0, and are uniform over the allowed set; users
are uniform.  The metrics are checked against the oracle restatement of
recalls_ndcgs_and_mrr_for_ks (pinned to the reference's known answers in tests/test_oracle.py).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _histories(n_users, V, rng, max_hist=300):
    return [list(rng.integers(1, V + 1, size=int(rng.integers(1, max_hist)))) for _ in range(n_users)]


def test_sampler_rows_follow_the_reference_construction():
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceWarpSampler
    rng = np.random.default_rng(0)
    V, T, B = 500, 50, 64
    users = _histories(200, V, rng)
    windows = {}
    for u, h in enumerate(users):
        windows.setdefault(tuple(h[-T:]), []).append(u)
    s = DeviceWarpSampler(users, V, B, T, seed=1)
    assert len(s) == 200 // B
    for seq, pos, neg in list(iter(s))[:3]:
        seq, pos, neg = (x.cpu().numpy() for x in (seq, pos, neg))
        assert seq.shape == (B, T) and seq.dtype == np.int64
        for b in range(B):
            nz = np.nonzero(pos[b])[0]
            pad = T - len(nz)
            assert (nz == np.arange(pad, T)).all(), "left padding"
            # window = seq tail + last pos item; it must be some user's last min(L, T) items
            win = tuple(list(seq[b, pad:]) + [pos[b, -1]]) if len(nz) else None
            if win is None:
                continue
            assert win in windows, "row is not a user's window"
            assert (seq[b, pad + 1:] == pos[b, pad:-1]).all(), "pos = seq shifted by one"
            assert (seq[b, :pad] == 0).all() and (neg[b, :pad] == 0).all()
            w = set(win)
            assert all(0 <= v <= V and v not in w for v in neg[b, pad:]), "negative inside the window"


def test_sampler_negatives_and_users_are_uniform():
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceWarpSampler
    V, T, B = 20, 8, 256
    users = [[1, 2, 3, 4, 5, 6, 7, 8, 9, 10] for _ in range(4)] + [[11, 12]]
    s = DeviceWarpSampler(users, V, B, T, seed=3)
    last, negs10 = [], []
    for _ in range(80):
        seq, pos, neg = (x.cpu().numpy() for x in s.sample())
        last.append(pos[:, -1])
        m = (pos != 0) & (pos[:, -1:] == 10)
        negs10.append(neg[m])
        assert ((neg >= 0) & (neg <= V)).all()
    last = np.concatenate(last)
    frac12 = (last == 12).mean()                 # users are uniform: 1 of 5 is the 2-item user
    assert abs(frac12 - 0.2) < 0.02, frac12
    # the 10-item users' window is their last T=8 items {3..10}: negatives uniform over {0, 1, 2, 11..20}
    allowed = [0, 1, 2, *range(11, 21)]
    v = np.concatenate(negs10)
    assert set(np.unique(v)) <= set(allowed)
    cnt = np.array([(v == k).sum() for k in allowed], dtype=np.float64)
    exp = v.size / len(allowed)
    chi2 = ((cnt - exp) ** 2 / exp).sum()
    assert chi2 < 50.0, (chi2, cnt)              # 12 degrees of freedom: mean 12, ~4 sigma margin


def test_sampler_is_reproducible_and_advances():
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceWarpSampler
    rng = np.random.default_rng(5)
    users = _histories(50, 300, rng)
    a = DeviceWarpSampler(users, 300, 32, 40, seed=9)
    b = DeviceWarpSampler(users, 300, 32, 40, seed=9)
    x1, x2 = a.sample(), a.sample()
    y1 = b.sample()
    assert all(torch.equal(u, v) for u, v in zip(x1, y1))
    assert not torch.equal(x1[2], x2[2])


@pytest.mark.parametrize("R,C,ks", [(256, 101, [1, 5, 10, 20]), (64, 21, [10]), (7, 5, [1, 3, 5])])
def test_rank_metrics_match_oracle(R, C, ks):
    import rbm_amd  # noqa: F401
    from oracle import metrics as om
    from rbm_amd import metrics as gm
    rng = np.random.default_rng(R)
    scores = np.round(rng.normal(size=(R, C)), 1).astype(np.float32)     # rounding creates ties
    labels = np.zeros((R, C), np.float32)
    labels[:, 0] = 1
    labels[::3, 2] = 1                                                    # some rows with two positives
    ours = gm.recalls_ndcgs_and_mrr_for_ks(torch.from_numpy(scores).cuda(), torch.from_numpy(labels).cuda(), ks)
    ref = om.recalls_ndcgs_and_mrr_for_ks(scores, labels, ks)
    assert ours.keys() == ref.keys()
    for k in ref:
        assert abs(ours[k] - ref[k]) < 1e-5, (k, ours[k], ref[k])


def test_sampled_step_graph_equals_eager():
    """The sampler captured in the step's graph (capture_sampled/replay_sampled) reproduces, bit for bit,
    eager sampling + eager steps from the same initial state and sampler seed."""
    import argparse
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceWarpSampler
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    rng = np.random.default_rng(11)
    V, T, B = 400, 64, 32
    users = _histories(300, V, rng, max_hist=120)
    a = argparse.Namespace(model_code="sas", num_items=V, max_len=T, device="cuda", sas_hidden_units=64,
                           sas_num_blocks=2, sas_heads=1, sas_dropout=0.2, l2_emb=0.0, rs_dtype="bf16")
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        m = model_factory(a)
        st = FusedTrainStep(m, lr=1e-3)
        smp = DeviceWarpSampler(users, V, B, T, seed=4)
        losses = []
        if graph:
            st.capture_sampled(smp, warmup=2)
            for _ in range(5):
                losses.append(st.replay_sampled().item())
        else:
            buf = [torch.zeros(B, T, dtype=torch.int64, device="cuda") for _ in range(3)]
            for _ in range(7):
                smp.sample_into(*buf)
                losses.append(st.step(*buf).item())
            losses = losses[2:]
        runs.append((losses, m.sas.engine().flat.data.clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1])
    assert all(np.isfinite(runs[0][0]))


def _originals(tok, lab):
    return np.where(lab != 0, lab, tok)


def test_bert_masker_rows_and_epoch():
    """rs_bert_mask rows follow BertTrainDataset.__getitem__ (BS/dataloaders/bert.py:77-110): a user's last
    max_len items, left padded; labels only at masked positions and equal to the item; unmasked tokens are
    the item itself; one epoch visits every user once (shuffled)."""
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceBertMasker
    rng = np.random.default_rng(2)
    V, T, B = 700, 40, 16
    users = _histories(64, V, rng, max_hist=90)
    windows = {tuple(h[-T:]): u for u, h in enumerate(users)}
    m = DeviceBertMasker(users, V, B, T, 0.3, seed=3)
    assert len(m) == 4
    seen = []
    for tok, lab in m:
        tok, lab = tok.cpu().numpy(), lab.cpu().numpy()
        orig = _originals(tok, lab)
        for b in range(B):
            nz = np.nonzero(orig[b])[0]
            pad = T - len(nz)
            assert (nz == np.arange(pad, T)).all(), "left padding"
            w = tuple(orig[b, pad:])
            assert w in windows, "row is not a user's window"
            seen.append(windows[w])
            masked = lab[b] != 0
            assert ((tok[b][~masked] == orig[b][~masked])).all()
            assert ((tok[b][masked] >= 1) & (tok[b][masked] <= V + 1)).all()
    assert sorted(seen) == list(range(64)), "an epoch visits every user once"


def test_bert_masker_rates():
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceBertMasker
    V, T, B = 5000, 100, 128
    users = [list(range(1 + u, 201 + u)) for u in range(256)]
    m = DeviceBertMasker(users, V, B, T, 0.2, seed=4)
    m.new_epoch()
    n_tok = n_mask = n_mtok = n_keep = 0
    for _ in range(20):
        tok, lab = (x.cpu().numpy() for x in m.sample())
        masked = lab != 0
        n_tok += tok.size
        n_mask += masked.sum()
        n_mtok += (tok[masked] == V + 1).sum()
        n_keep += (tok[masked] == lab[masked]).sum()
    f = n_mask / n_tok
    assert abs(f - 0.2) < 0.005, f
    assert abs(n_mtok / n_mask - 0.8) < 0.01 and abs(n_keep / n_mask - 0.1) < 0.01, (n_mtok / n_mask, n_keep / n_mask)


def test_bert_sampled_step_graph_equals_eager():
    import argparse
    import rbm_amd  # noqa: F401
    from rbm_amd.dataloaders import DeviceBertMasker
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    rng = np.random.default_rng(12)
    V, T, B = 500, 32, 16
    users = _histories(100, V, rng, max_hist=60)
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=64,
                           bert_num_blocks=1, bert_num_heads=2, bert_dropout=0.1, bert_hidden_dropout=0.1,
                           bert_mask_prob=0.2, model_init_seed=0, rs_dtype="bf16")
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        m = model_factory(a)
        st = FusedTrainStep(m, lr=1e-3)
        smp = DeviceBertMasker(users, V, B, T, 0.2, seed=6)
        smp.new_epoch()
        losses = []
        if graph:
            st.capture_sampled(smp, warmup=2)
            for _ in range(4):
                losses.append(st.replay_sampled().item())
        else:
            buf = [torch.zeros(B, T, dtype=torch.int64, device="cuda") for _ in range(2)]
            for _ in range(6):
                smp.sample_into(*buf)
                losses.append(st.step(*buf).item())
            losses = losses[2:]
        runs.append((losses, m.engine().flat.data.clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1])
