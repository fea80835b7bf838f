"""Unrolled step graphs (FusedTrainStep.capture / capture_sampled with steps_per_graph=S): one replay runs S
whole training steps, each on its own batch with its own Adam update, and must equal S single-step replays
bit for bit (same kernels, same order, same seeds)."""
import argparse

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(kind, dtype="bf16", p=0.2, l2=0.0):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    torch.manual_seed(0)
    if kind == "sas":
        a = argparse.Namespace(model_code="sas", num_items=600, max_len=64, device="cuda", sas_hidden_units=64,
                               sas_num_blocks=2, sas_heads=1, sas_dropout=p, l2_emb=l2, rs_dtype=dtype)
    else:
        a = argparse.Namespace(model_code="bert", num_items=600, max_len=64, device="cuda", bert_hidden_units=64,
                               bert_num_blocks=2, bert_num_heads=2, bert_dropout=p, bert_hidden_dropout=p,
                               bert_mask_prob=0.2, model_init_seed=0, rs_dtype=dtype)
    return model_factory(a)


def _batches(kind, n):
    import rbm_amd.data as synth
    rng = np.random.default_rng(5)
    out = []
    for _ in range(n):
        b = synth.sas_batch(rng, 16, 64, 600) if kind == "sas" else synth.bert_batch(rng, 16, 64, 600)
        out.append(torch.stack([torch.from_numpy(x) for x in b]).cuda())
    return out


@pytest.mark.parametrize("kind,l2", [("sas", 0.0), ("sas", 0.01), ("bert", 0.0)])
def test_unrolled_graph_equals_single_step_replays(kind, l2):
    """unroll 0 = eager steps (no graph); l2 > 0: the SAS parameter-norm term (rs_l2_penalty) in every unrolled
    step, its loss landing in that step's row."""
    from rbm_amd.train_step import FusedTrainStep
    S, rounds = 4, 2
    bs = _batches(kind, S * rounds)
    runs = []
    for unroll in (0, 1, S):
        m = _model(kind, l2=l2)
        st = FusedTrainStep(m, lr=1e-3)
        losses = []
        if unroll == 0:
            for b in bs[:1] * 2:       # the capture's two warmup steps
                st.step(*b.unbind(0))
            for b in bs:
                losses.append(st.step(*b.unbind(0)).item())
            runs.append((losses, st.flat.data.clone(), int(st.opt.state[0].item())))
            continue
        st.capture(*bs[0].unbind(0), warmup=2, steps_per_graph=unroll)
        if unroll == 1:
            for b in bs:
                losses.append(st.replay_packed(b).item())
        else:
            for r in range(rounds):
                losses += st.replay_packed(torch.stack(bs[r * S:(r + 1) * S])).tolist()
        runs.append((losses, st.flat.data.clone(), int(st.opt.state[0].item())))
    assert runs[0][2] == runs[1][2] == runs[2][2] == 2 + S * rounds
    for r in runs[1:]:
        assert r[0] == runs[0][0], (r[0], runs[0][0])
        assert torch.equal(r[1], runs[0][1])
    assert all(np.isfinite(runs[0][0]))


def test_unrolled_sampled_graph_equals_single_step_replays():
    from rbm_amd.dataloaders import DeviceWarpSampler
    from rbm_amd.train_step import FusedTrainStep
    import rbm_amd.data as synth
    users = synth.user_histories(np.random.default_rng(3), 200, 64, 600)
    S = 4
    runs = []
    for unroll in (1, S):
        m = _model("sas")
        st = FusedTrainStep(m, lr=1e-3)
        st.capture_sampled(DeviceWarpSampler(users, 600, 16, 64, seed=9), warmup=2, steps_per_graph=unroll)
        losses = []
        for _ in range(S // unroll):
            losses += st.replay_sampled().reshape(-1).tolist()
        runs.append((losses, st.flat.data.clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1])


def test_unrolled_rejects_wrong_shapes():
    from rbm_amd.train_step import FusedTrainStep
    bs = _batches("sas", 2)
    st = FusedTrainStep(_model("sas"), lr=1e-3)
    st.capture(*bs[0].unbind(0), warmup=1, steps_per_graph=2)
    with pytest.raises(ValueError):
        st.replay_packed(bs[0])
    with pytest.raises(ValueError):
        st.replay(*bs[0].unbind(0))
