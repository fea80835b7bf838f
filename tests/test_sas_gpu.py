"""SASRec HIP path vs the reference (golden vectors) and the CPU oracle.

GPU tests: the whole forward / loss / backward goes through librecsys_hip.so
(C ABI).  fp32 mode must match the reference within the fp32 tolerance stated
here; bf16 mode within the bf16 tolerance.
"""
import argparse

import numpy as np
import pytest
import torch

from conftest import check_bf16_grads, golden_params, load_golden, rel

pytestmark = pytest.mark.gpu

# tolerances (norm-relative): fp32 mode vs the reference's fp32 outputs
FWD_TOL_F32 = 1e-5
GRAD_TOL_F32 = 1e-4
# bf16 storage / MFMA operands, fp32 accumulate
FWD_TOL_BF16 = 3e-2  # bf16 storage of weights/activations/activation-gradients
# bf16 gradients: conftest.check_bf16_grads (vs the bf16-storage emulation within EMU_TOL, vs the exact math
# within max(3e-2, 2 x the format's own error for that tensor))


def sas_args(V, T, d, L, h, p=0.0, dtype="fp32"):
    return argparse.Namespace(model_code="sas", num_items=V, max_len=T, device="cuda", sas_hidden_units=d,
                              sas_num_blocks=L, sas_heads=h, sas_dropout=p, l2_emb=0.0, rs_dtype=dtype)


def make_model(z, dtype="fp32"):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    m = model_factory(sas_args(int(z["V"]), int(z["T"]), int(z["d"]), int(z["L"]), int(z["h"]), dtype=dtype))
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p/")})
    return m


def run_step(m, seq, pos, neg):
    from rbm_amd.losses import sampled_bce
    m.train()
    m.zero_grad(set_to_none=True)
    pl, nl = m(seq, pos, neg)
    loss = sampled_bce(pl, nl, torch.from_numpy(pos).cuda())
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()}
    return pl.detach().cpu().numpy(), nl.detach().cpu().numpy(), float(loss.item()), grads


def check_grads(grads, ref, d, tol, scale_ref):
    for k, g in grads.items():
        r = ref[k]
        if k.endswith("in_proj_bias"):
            # key-bias gradient is analytically zero (softmax shift invariance): compare on scale
            assert np.linalg.norm(g[d:2 * d]) <= max(1e-5, tol) * scale_ref, k
            g, r = np.concatenate([g[:d], g[2 * d:]]), np.concatenate([r[:d], r[2 * d:]])
        assert rel(g, r) < tol, (k, rel(g, r))


@pytest.mark.parametrize("name", ["sas_tiny", "sas_mid"])
def test_sas_fp32_matches_reference(name):
    z = load_golden(name)
    m = make_model(z, "fp32")
    pl, nl, loss, grads = run_step(m, z["seq"], z["pos"], z["neg"])
    assert rel(pl, z["pos_logits"]) < FWD_TOL_F32
    assert rel(nl, z["neg_logits"]) < FWD_TOL_F32
    assert abs(loss - float(z["loss"])) < FWD_TOL_F32 * max(1.0, abs(float(z["loss"])))
    ref = {k: z["g/sas." + k[4:]] if k.startswith("sas.") else z["g/" + k] for k in grads}
    scale = max(np.linalg.norm(v) for v in ref.values())
    check_grads(grads, ref, int(z["d"]), GRAD_TOL_F32, scale)


@pytest.mark.parametrize("name", ["sas_tiny", "sas_mid"])
def test_sas_bf16_matches_reference(name):
    """bf16 fused path on the reference's golden batches: forward vs the reference outputs; gradients vs the
    bf16-storage emulation (the kernels' own error) and vs the reference's fp32 gradients (+ the format's)."""
    from oracle import sas as osas
    z = load_golden(name)
    m = make_model(z, "bf16")
    pl, nl, loss, grads = run_step(m, z["seq"], z["pos"], z["neg"])
    assert rel(pl, z["pos_logits"]) < FWD_TOL_BF16
    assert rel(nl, z["neg_logits"]) < FWD_TOL_BF16
    assert abs(loss - float(z["loss"])) < FWD_TOL_BF16 * max(1.0, abs(float(z["loss"])))
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    L, h = int(z["L"]), int(z["h"])
    args = [torch.from_numpy(z[k]) for k in ("seq", "pos", "neg")]
    _, _, _, ge = osas.loss_and_grads(P, *args, L, h, emu=osas.BF16Storage())
    ref = {("sas." + k[4:] if k.startswith("sas.") else k): torch.from_numpy(z["g/" + k].astype(np.float64))
           for k in grads}
    ge = {k: ge[k] for k in ref}
    out = check_bf16_grads(lambda n: grads[n], ge, ref, int(z["d"]), kbias=lambda n: n.endswith("in_proj_bias"))
    print(name, "worst vs emulation", max(out.items(), key=lambda kv: kv[1][0]),
          "worst vs reference", max(out.items(), key=lambda kv: kv[1][1]))


def test_sas_predict_matches_reference():
    z = load_golden("sas_tiny")
    m = make_model(z, "fp32")
    m.eval()
    s = m.predict(torch.from_numpy(z["seq"]).int(), torch.from_numpy(z["cand"]).int())
    assert rel(s.cpu().numpy(), z["cand_scores"]) < FWD_TOL_F32


@pytest.mark.parametrize("V,T,d,L,h,B", [(3416, 200, 128, 2, 1, 3), (500, 50, 64, 2, 2, 5),
                                         (300, 37, 128, 1, 4, 2), (1000, 200, 256, 2, 2, 2),
                                         # BASELINE configs[0] = the reference's default config (BS/config.json:
                                         # d = 50, 1 head, T = 200), its 2-head variant (Dh = 25), --max_len 300
                                         (3416, 200, 50, 2, 1, 4), (400, 60, 50, 2, 2, 3), (500, 300, 64, 2, 1, 2)])
def test_sas_fp32_matches_oracle_shapes(V, T, d, L, h, B):
    """Random weights / batches at several shapes (odd T, Dh 25/32/50/64/128, T up to 300) vs the fp64 oracle."""
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from rbm_amd.models import model_factory
    from oracle import sas as osas
    torch.manual_seed(V + T)
    m = model_factory(sas_args(V, T, d, L, h))
    rng = np.random.default_rng(T)
    seq, pos, neg = synth.sas_batch(rng, B, T, V)
    pl, nl, loss, grads = run_step(m, seq, pos, neg)
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    l64, pl64, nl64, g64 = osas.loss_and_grads(P, torch.from_numpy(seq), torch.from_numpy(pos),
                                               torch.from_numpy(neg), L, h)
    assert rel(pl, pl64) < FWD_TOL_F32 and rel(nl, nl64) < FWD_TOL_F32
    assert abs(loss - l64.item()) < 1e-5 * max(1, abs(l64.item()))
    ref = {k: g64[k].numpy() for k in grads}
    scale = max(np.linalg.norm(v) for v in ref.values())
    check_grads(grads, ref, d, GRAD_TOL_F32, scale)


def test_sas_all_padding_rows_and_zero_negatives():
    """Edge cases the reference handles: fully padded sequences and neg id 0 (random_neq can return 0)."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    from oracle import sas as osas
    torch.manual_seed(0)
    V, T, d, L, h, B = 60, 16, 64, 2, 1, 4
    m = model_factory(sas_args(V, T, d, L, h))
    rng = np.random.default_rng(1)
    seq = np.zeros((B, T), np.int64)
    pos = np.zeros((B, T), np.int64)
    neg = np.zeros((B, T), np.int64)
    seq[1, 3:] = rng.integers(1, V + 1, T - 3)
    pos[1, 3:] = rng.integers(1, V + 1, T - 3)
    neg[1, 3:] = rng.integers(0, 3, T - 3)           # includes padding id 0
    seq[2, :] = rng.integers(1, V + 1, T)
    pos[2, :] = rng.integers(1, V + 1, T)
    neg[2, :] = rng.integers(1, V + 1, T)
    pl, nl, loss, grads = run_step(m, seq, pos, neg)
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    l64, pl64, nl64, g64 = osas.loss_and_grads(P, *(torch.from_numpy(a) for a in (seq, pos, neg)), L, h)
    assert rel(pl, pl64) < FWD_TOL_F32 and rel(nl, nl64) < FWD_TOL_F32
    assert abs(loss - l64.item()) < 1e-5 * max(1, abs(l64.item()))
    assert grads["sas.item_emb.weight"][0].any() == False  # noqa: E712  padding row never updated
    ref = {k: g64[k].numpy() for k in grads}
    scale = max(np.linalg.norm(v) for v in ref.values())
    check_grads(grads, ref, d, GRAD_TOL_F32, scale)


@pytest.mark.parametrize("V,T,d,L,h,B", [(500, 37, 64, 2, 2, 3), (400, 200, 128, 2, 1, 5), (300, 50, 128, 1, 4, 2)])
def test_sas_autograd_bf16_dropout_matches_oracle(V, T, d, L, h, B):
    """The reference forward API in bf16 (SASModel.forward -> pos/neg logits, then the BCE and autograd backward:
    the row-chain block kernels with the split head rs_sas_head_fwd / rs_sas_head_bwd) at p = 0.2, with fully padded
    leading positions, padded targets and a ragged last row tile, against the oracle replaying the same dropout
    masks: logits and loss within the bf16 forward bar, every gradient against the bf16-storage emulation
    (conftest.check_bf16_grads).  The fused training step's form of the same kernels (embedding inside the first
    block's input kernel, head inside the last block's output kernel) is tested in test_dropout_parity_gpu."""
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from oracle import sas as osas
    from rbm_amd.losses import sampled_bce
    from rbm_amd.models import model_factory
    from test_dropout_parity_gpu import sas_masks
    torch.manual_seed(V)
    p = 0.2
    m = model_factory(sas_args(V, T, d, L, h, p=p, dtype="bf16"))
    m.train()
    eng = m.sas.engine()
    assert eng.fused_head
    rng = np.random.default_rng(T)
    seq, pos, neg = (torch.from_numpy(a) for a in synth.sas_batch(rng, B, T, V))
    seq[0, :11] = 0
    pos[0, :10] = 0
    pos[-1, -1] = 0
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    eng.seed_base.fill_(40)
    pl, nl = m(seq.numpy(), pos.numpy(), neg.numpy())
    sb = eng.seed_base.clone()            # the forward advanced the step seed once: its masks use this value
    loss = sampled_bce(pl, nl, pos.cuda())
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: q.grad.detach().cpu().numpy() for k, q in m.named_parameters()}
    masks = {k: v.cpu().double() for k, v in sas_masks(eng, B, T, sb).items()}
    le, ple, nle, ge = osas.loss_and_grads(P, seq, pos, neg, L, h, p=p, masks=masks, emu=osas.BF16Storage())
    l64, pl64, nl64, g64 = osas.loss_and_grads(P, seq, pos, neg, L, h, p=p, masks=masks)
    valid = (pos != 0).numpy()
    assert rel(pl.detach().cpu().numpy()[valid], pl64.numpy()[valid]) < FWD_TOL_BF16
    assert rel(nl.detach().cpu().numpy()[valid], nl64.numpy()[valid]) < FWD_TOL_BF16
    assert abs(loss.item() - le.item()) < 2e-3 * abs(le.item()), (loss.item(), le.item())
    ge = {k: ge[k] for k in g64}
    out = check_bf16_grads(lambda n: grads[n], ge, g64, d, kbias=lambda n: n.endswith("in_proj_bias"))
    assert not grads["sas.item_emb.weight"][0].any()          # padding row never updated
    print((V, T, d, B), "worst vs emulation", max(out.items(), key=lambda kv: kv[1][0]))
