"""Checkpoint interop: the fused trainer's checkpoint has the reference's layout
({'model_state_dict', 'optimizer_state_dict', 'epoch'}, BS/trainers/base.py:255-259, BS/loggers.py:48-58),
its optimizer state loads into torch.optim.Adam (the reference's optimizer, base.py:225-228) and continues
identically, and a fused trainer resumes from it bit for bit (both paths' gradients are deterministic: the fp32
unfused path sums the item-embedding gradient by the inverted index, rs_item_grad_f32, not with float atomics)."""
import argparse
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _args(dt="fp32"):
    return argparse.Namespace(model_code="sas", num_items=300, max_len=32, device="cuda", sas_hidden_units=64,
                              sas_num_blocks=2, sas_heads=2, sas_dropout=0.0, l2_emb=0.0, rs_dtype=dt)


def _batch(seed):
    import rbm_amd.data as synth
    rng = np.random.default_rng(seed)
    return tuple(torch.from_numpy(a).cuda() for a in synth.sas_batch(rng, 8, 32, 300))


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_checkpoint_resumes_in_torch_adam_and_in_the_fused_trainer(dt):
    import rbm_amd  # noqa: F401
    from rbm_amd.losses import sampled_bce
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    torch.manual_seed(0)
    m = model_factory(_args(dt))
    st = FusedTrainStep(m, lr=2e-3, weight_decay=0.0)
    for i in range(3):
        st.step(*_batch(i))
    buf = io.BytesIO()
    torch.save(st.checkpoint(epoch=1), buf)
    buf.seek(0)
    ck = torch.load(buf, weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "epoch"}
    assert set(ck["model_state_dict"]) == set(m.state_dict())

    # reference side: a plain module + torch.optim.Adam resumed from the checkpoint
    m2 = model_factory(_args(dt))
    m2.load_state_dict(ck["model_state_dict"])
    opt2 = torch.optim.Adam(m2.parameters(), lr=1.0)
    opt2.load_state_dict(ck["optimizer_state_dict"])
    assert opt2.param_groups[0]["lr"] == pytest.approx(2e-3)
    seq, pos, neg = _batch(10)
    opt2.zero_grad()
    pl, nl = m2(seq, pos, neg)
    sampled_bce(pl, nl, pos).backward()
    opt2.step()

    # fused side: a fresh trainer resumed from the same checkpoint, and the original trainer
    m3 = model_factory(_args(dt))
    st3 = FusedTrainStep(m3, lr=1.0)
    buf.seek(0)                        # a fresh copy: torch's Adam.step() advanced ck's 'step' tensors in place
    st3.load_checkpoint(torch.load(buf, weights_only=True))
    st3.step(seq, pos, neg)
    st.step(seq, pos, neg)
    torch.cuda.synchronize()
    p1 = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    p2 = torch.cat([p.detach().reshape(-1) for p in m2.parameters()])
    p3 = torch.cat([p.detach().reshape(-1) for p in m3.parameters()])
    assert torch.equal(p1, p3), "fused resume must be bit-identical"
    rel = ((p1 - p2).norm() / p1.norm()).item()
    assert rel < (1e-6 if dt == "fp32" else 1e-3), rel
