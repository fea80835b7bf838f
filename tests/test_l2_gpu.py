"""SASRec's parameter-norm regulariser l2_emb * sum_p ||p||_2 (BS/trainers/sas.py:51-52) in the fused training step
(rs_l2_penalty): loss and gradient against the fp64 oracle, single device; the data-parallel path (scale = the
global count) is covered by tests/test_dp_multirank_gpu.py (its SAS model trains with l2_emb > 0)."""
import argparse

import numpy as np
import pytest
import torch

from conftest import check_bf16_grads, rel

pytestmark = pytest.mark.gpu


def _model(dtype, l2):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    torch.manual_seed(8)
    a = argparse.Namespace(model_code="sas", num_items=400, max_len=40, device="cuda", sas_hidden_units=64,
                           sas_num_blocks=2, sas_heads=1, sas_dropout=0.0, l2_emb=l2, rs_dtype=dtype)
    return model_factory(a)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_l2_penalty_loss_and_grad_match_oracle(dtype):
    import rbm_amd.data as synth
    from oracle import sas as osas
    from rbm_amd.train_step import FusedTrainStep
    l2 = 0.05
    m = _model(dtype, l2)
    tr = FusedTrainStep(m, lr=1e-3)
    assert tr.l2 == l2
    rng = np.random.default_rng(2)
    seq, pos, neg = (torch.from_numpy(a).cuda() for a in synth.sas_batch(rng, 5, 40, 400))
    tr._compute(seq, pos, neg)
    tr._l2(tr.loss_out[2:3])          # what _update runs before the optimizer
    torch.cuda.synchronize()
    loss = float(tr.loss_out[2].item())
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    l64, _, _, g64 = osas.loss_and_grads(P, seq.cpu(), pos.cpu(), neg.cpu(), 2, 1, l2_emb=l2)
    pen = l2 * sum(float(torch.norm(v)) for v in P.values())
    assert pen > 1.0                                  # the term is a visible part of the loss
    ftol = 1e-5 if dtype == "fp32" else 3e-2
    assert abs(loss - l64.item()) < ftol * abs(l64.item()), (loss, l64.item())
    d = 64
    if dtype == "bf16":
        _, _, _, ge = osas.loss_and_grads(P, seq.cpu(), pos.cpu(), neg.cpu(), 2, 1, l2_emb=l2, emu=osas.BF16Storage())
        check_bf16_grads(lambda n: tr.flat.view(n, tr.flat.grad).cpu().numpy(), ge, g64, d,
                         kbias=lambda n: n.endswith("in_proj_bias"), strip="sas.")
        return
    for k, ref in g64.items():
        g = tr.flat.view(k[4:], tr.flat.grad).cpu().numpy().astype(np.float64)
        r = ref.numpy()
        if k.endswith("in_proj_bias"):
            g, r = np.concatenate([g[:d], g[2 * d:]]), np.concatenate([r[:d], r[2 * d:]])
        assert rel(g, r) < 1e-4, (k, rel(g, r))


def test_l2_zero_norm_parameter_gets_zero_gradient():
    """torch.norm's backward masks a zero norm: a parameter that is all zero (here an LN bias) gets no NaN."""
    from rbm_amd import ops
    m = _model("fp32", 0.1)
    eng = m.sas.engine()
    fl = eng.flat
    fl.view("last_layernorm.bias").zero_()
    desc = ops.l2_chunk_desc(fl, fl.device)
    ws = torch.zeros(2 * desc.shape[0], device="cuda")
    g = torch.zeros(fl.numel, device="cuda")
    loss = torch.zeros(1, device="cuda")
    ops.l2_penalty(fl.data, g, desc, 0.1, ws, loss=loss)
    torch.cuda.synchronize()
    assert torch.isfinite(g).all()
    assert not fl.view("last_layernorm.bias", g).any()
    w = fl.view("item_emb.weight")
    assert torch.allclose(fl.view("item_emb.weight", g), 0.1 * w / torch.norm(w), rtol=1e-5, atol=1e-8)
    ref = 0.1 * sum(float(torch.norm(p.detach().double())) for p in m.parameters())
    assert abs(loss.item() - ref) < 1e-5 * ref
