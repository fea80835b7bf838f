"""BERT4Rec: the HIP path vs the reference (golden vectors) and the CPU oracle.

* CPU: ``BERTModel(args)`` builds bit-identical initial weights to the reference for the
  same ``model_init_seed`` (BS/models/bert_modules/bert.py:12 seeds before construction) and
  the same state_dict keys -- checked against the weights the reference itself produced.
* GPU: forward logits / CE loss / every gradient through librecsys_hip.so, both through the
  reference API (``model(x)`` full-vocabulary logits + torch CE on top) and through the fused
  labelled-rows-only training step; fp32 within the fp32 tolerance, bf16 within the bf16 one.
"""
import argparse

import numpy as np
import pytest
import torch

from conftest import golden_params, load_golden, rel

FWD_TOL_F32, GRAD_TOL_F32 = 1e-5, 1e-4
FWD_TOL_BF16, GRAD_TOL_BF16 = 3e-2, 3e-2   # BERT bf16 gradients measure <= 1e-2 (no ReLU: GELU)
SEEDS = {"bert_tiny": 3, "bert_mid": 4, "bert_curve": 7}   # tools/gen_golden.py


def bert_args(z, device="cuda", dtype="fp32", seed=0, p=0.0, hp=0.0):
    return argparse.Namespace(model_code="bert", num_items=int(z["V"]), max_len=int(z["T"]), device=device,
                              bert_hidden_units=int(z["d"]), bert_num_blocks=int(z["L"]), bert_num_heads=int(z["h"]),
                              bert_dropout=p, bert_hidden_dropout=hp, bert_mask_prob=0.2, model_init_seed=seed,
                              rs_dtype=dtype)


@pytest.mark.parametrize("name", ["bert_tiny", "bert_mid", "bert_curve"])
def test_bert_init_matches_reference(name):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    z = load_golden(name)
    m = model_factory(bert_args(z, device="cpu", seed=SEEDS[name]))
    sd = m.state_dict()
    ref = golden_params(z)
    assert sorted(sd) == sorted(ref)
    for k in ref:
        assert torch.equal(sd[k], ref[k]), k


def make_model(z, dtype):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    m = model_factory(bert_args(z, dtype=dtype))
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p/")})
    return m


def check_grads(grads, z, tol):
    scale = max(np.linalg.norm(z["g/" + k]) for k in grads)
    for k, g in grads.items():
        r = z["g/" + k]
        if "linear_layers.1.bias" in k:       # key bias: analytically zero (softmax shift invariance)
            assert np.linalg.norm(g) <= max(1e-5, tol) * scale, k
            continue
        if np.linalg.norm(r) == 0:
            assert np.linalg.norm(g) <= 1e-6 * scale, k
            continue
        assert rel(g, r) < tol, (k, rel(g, r))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("name", ["bert_tiny", "bert_mid"])
def test_bert_api_matches_reference(name, dtype):
    """model(x) -> (B,T,V+1) logits, torch CE(ignore_index=0) on top, backward through the HIP path."""
    z = load_golden(name)
    m = make_model(z, dtype)
    m.train()
    tok = torch.from_numpy(z["tokens"]).cuda()
    lab = torch.from_numpy(z["labels"]).cuda()
    logits = m(tok)
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), lab.reshape(-1), ignore_index=0)
    loss.backward()
    torch.cuda.synchronize()
    ftol, gtol = (FWD_TOL_F32, GRAD_TOL_F32) if dtype == "fp32" else (FWD_TOL_BF16, GRAD_TOL_BF16)
    assert rel(logits.detach().cpu().numpy(), z["logits"]) < ftol
    assert abs(loss.item() - float(z["loss"])) < ftol * max(1.0, float(z["loss"]))
    check_grads({k: p.grad.cpu().numpy() for k, p in m.named_parameters()}, z, gtol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("name", ["bert_tiny", "bert_mid"])
def test_bert_fused_step_matches_reference(name, dtype):
    """The fused training step (labelled-row compaction + vocab GEMM + CE on those rows only)
    gives the reference loss and gradients."""
    from rbm_amd.train_step import FusedTrainStep
    z = load_golden(name)
    m = make_model(z, dtype)
    m.train()
    tr = FusedTrainStep(m, lr=0.0)
    tok = torch.from_numpy(z["tokens"]).cuda()
    lab = torch.from_numpy(z["labels"]).cuda()
    tr.flat.grad.zero_()
    tr.engine.sync_compute_weights()
    tr.engine.train_loss_and_backward(tok, lab, tr.loss_out, tr._divisor, tr.flat.grad)
    torch.cuda.synchronize()
    ftol, gtol = (FWD_TOL_F32, GRAD_TOL_F32) if dtype == "fp32" else (FWD_TOL_BF16, GRAD_TOL_BF16)
    loss = float(tr.loss_out[2].item())
    assert abs(loss - float(z["loss"])) < ftol * max(1.0, float(z["loss"]))
    assert int(tr.loss_out[1].item()) == int((z["labels"] != 0).sum())
    check_grads({k: tr.flat.view(k, tr.flat.grad).cpu().numpy() for k, _ in m.named_parameters()}, z, gtol)


@pytest.mark.gpu
@pytest.mark.parametrize("V,T,d,L,h,B,cap", [(26744, 200, 256, 2, 2, 2, None), (500, 50, 64, 1, 1, 3, 64),
                                             (300, 37, 128, 2, 4, 2, None)])
def test_bert_fp32_matches_oracle_shapes(V, T, d, L, h, B, cap):
    """cfg3 shape (V=26,744, T=200, d=256, 2 heads) and odd shapes vs the fp64 oracle, fused step,
    including a compaction cap above the labelled count."""
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from oracle import bert as obert
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=d,
                           bert_num_blocks=L, bert_num_heads=h, bert_dropout=0.0, bert_hidden_dropout=0.0,
                           bert_mask_prob=0.2, model_init_seed=V, rs_dtype="fp32")
    m = model_factory(a)
    rng = np.random.default_rng(T)
    tok, lab = synth.bert_batch(rng, B, T, V, mask_prob=0.2)
    tr = FusedTrainStep(m, lr=0.0, max_labelled=cap)
    tr.flat.grad.zero_()
    tr.engine.train_loss_and_backward(torch.from_numpy(tok).cuda(), torch.from_numpy(lab).cuda(), tr.loss_out,
                                      tr._divisor, tr.flat.grad, max_labelled=cap)
    torch.cuda.synchronize()
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    l64, _, g64 = obert.loss_and_grads(P, torch.from_numpy(tok), torch.from_numpy(lab), L, h)
    assert abs(tr.loss_out[2].item() - l64.item()) < 1e-5 * max(1, abs(l64.item()))
    scale = max(float(v.norm()) for v in g64.values())
    for k in g64:
        g = tr.flat.view(k, tr.flat.grad).cpu().double()
        if "linear_layers.1.bias" in k or float(g64[k].norm()) == 0:
            assert float(g.norm()) <= 1e-5 * scale, k
            continue
        assert rel(g.numpy(), g64[k].numpy()) < GRAD_TOL_F32, (k, rel(g.numpy(), g64[k].numpy()))


def _bert(V, T, d, L, h, p, dtype, seed):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=d,
                           bert_num_blocks=L, bert_num_heads=h, bert_dropout=p, bert_hidden_dropout=p,
                           bert_mask_prob=0.2, model_init_seed=seed, rs_dtype=dtype)
    return model_factory(a)


def _bert_step_vs_oracle(m, tok, lab, L, h, p, cap=None, seed=4242, labelled_only=False):
    """One fused bf16 training step's loss and gradient (FusedTrainStep._compute, before the optimizer) against the
    fp64 oracle replaying the step's dropout masks.  Returns (loss, oracle loss, {name: norm-relative error})."""
    from oracle import bert as obert
    from rbm_amd.train_step import FusedTrainStep
    from test_dropout_parity_gpu import bert_masks
    tr = FusedTrainStep(m, lr=0.0, max_labelled=cap)
    tr.engine.seed_base.fill_(seed)
    tr.flat.grad.zero_()
    tr._compute(tok, lab)
    torch.cuda.synchronize()
    loss = float(tr.loss_out[2].item())
    assert float(tr.loss_out[1].item()) == int((lab != 0).sum())
    B, T = tok.shape
    sb = torch.full((1,), seed, dtype=torch.int64, device="cuda")
    masks = {k: v.cpu().double() for k, v in bert_masks(tr.engine, B, T, sb).items()} if p > 0 else None
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    torch.set_num_threads(16)
    l64, _, g64 = obert.loss_and_grads(P, tok.cpu(), lab.cpu(), L, h, p=p, hp=p, masks=masks,
                                       labelled_only=labelled_only)
    scale = max(float(g.norm()) for g in g64.values())
    worst = {}
    for k, r in g64.items():
        g = tr.flat.view(k, tr.flat.grad).cpu().double()
        if "linear_layers.1.bias" in k:          # the attention key bias: analytically zero gradient
            assert float(g.norm()) <= 1e-2 * scale, k
            continue
        worst[k] = rel(g.numpy(), r.numpy())
    return loss, float(l64), worst


@pytest.mark.gpu
@pytest.mark.parametrize("d,B,cap", [(64, 16, 256), (256, 40, 512), (128, 3, 128), (96, 8, 256)])
def test_bert_vocab_head_matches_oracle(d, B, cap):
    """bf16: the vocabulary head without materialised logits -- rs_vocab_head_fwd/bwd (vocabulary-tile-stationary,
    d in {64, 128, 256}) or, for other widths (d = 96), rs_vocab_ce_fwd/bwd (GEMM epilogues) -- at the cfg3
    vocabulary (26,745 classes: a ragged last column tile), ragged / partial row tiles and labelled-row caps above
    the labelled count, against the fp64 oracle's full-vocabulary CE (BS/models/bert.py:16, BS/trainers/bert.py:
    36-40)."""
    import rbm_amd.data as synth
    from rbm_amd import ops
    m = _bert(26744, 50, d, 1, 2, 0.0, "bf16", seed=1)
    assert ops.vocab_head_supported(d) == (d != 96)
    rng = np.random.default_rng(1)
    tok, lab = (torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, 50, 26744, mask_prob=0.2))
    assert int((lab != 0).sum()) <= cap
    loss, l64, worst = _bert_step_vs_oracle(m, tok, lab, 1, 2, 0.0, cap=cap)
    assert abs(loss - l64) < FWD_TOL_BF16 * abs(l64), (loss, l64)
    bad = {k: v for k, v in worst.items() if v >= GRAD_TOL_BF16}
    assert not bad, bad


@pytest.mark.gpu
def test_bert_cfg3_bench_step_matches_oracle():
    """BASELINE configs[2] at its benchmarked shape and dtype: BERT4Rec, 26,744 items, T = 200, d = 256, 4 blocks,
    2 heads, dropout 0.1 at every site (injected into the oracle), bf16 fused training step -- grouped weight
    gradients (rs_wgrad_grouped), LayerNorm-backward dropout fusion, delta-in attention backward, the
    vocabulary-tile-stationary head -- at the bench's batch (64) and labelled-row cap (1,792) against the fp64
    oracle (BS/models/bert.py:10,16, BS/trainers/bert.py:30-41; its output layer on the labelled rows only, the same
    loss and gradients)."""
    import rbm_amd.data as synth
    m = _bert(26744, 200, 256, 4, 2, 0.1, "bf16", seed=3)
    rng = np.random.default_rng(7)
    tok, lab = (torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, 64, 200, 26744, mask_prob=0.2))
    n_lab = int((lab != 0).sum())
    assert 1024 < n_lab <= 1792, n_lab
    loss, l64, worst = _bert_step_vs_oracle(m, tok, lab, 4, 2, 0.1, cap=1792, labelled_only=True)
    print("cfg3 bf16 step, rows", n_lab, ": loss", loss, l64, "worst", max(worst.items(), key=lambda kv: kv[1]))
    assert abs(loss - l64) < FWD_TOL_BF16 * abs(l64), (loss, l64)
    bad = {k: v for k, v in worst.items() if v >= GRAD_TOL_BF16}
    assert not bad, bad


@pytest.mark.gpu
def test_bert_cfg5_bench_step_matches_oracle():
    """BASELINE configs[4] at its benchmarked shape and dtype: 1,000,000 items (out.weight 1,000,001 x 256, the token
    table 1,000,002 x 256), T = 200, d = 256, 4 blocks, 2 heads, dropout 0.1 (injected into the oracle), bf16 fused
    training step (vocabulary-tile-stationary head rs_vocab_head_fwd/bwd + the dE / dh GEMMs; token-table gradient
    by inverted index) at batch 1 (the labelled-row cap 128 covers it) against the fp64 oracle's CE over the full
    vocabulary (BS/models/bert.py:16, BS/trainers/bert.py:36-40): loss, out.weight / out.bias gradients (dense over
    all 1M rows), the token table and every block weight."""
    import rbm_amd.data as synth
    V, T, B, L = 1_000_000, 200, 1, 4
    m = _bert(V, T, 256, L, 2, 0.1, "bf16", seed=5)
    rng = np.random.default_rng(6)
    tok, lab = (torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, T, V, mask_prob=0.2))
    n_lab = int((lab != 0).sum())
    assert 0 < n_lab <= 128
    loss, l64, worst = _bert_step_vs_oracle(m, tok, lab, L, 2, 0.1, cap=128)
    print("cfg5 bf16 step: loss", loss, l64, "worst", max(worst.items(), key=lambda kv: kv[1]))
    assert abs(loss - l64) < FWD_TOL_BF16 * abs(l64), (loss, l64)
    bad = {k: v for k, v in worst.items() if v >= GRAD_TOL_BF16}
    assert not bad, bad


@pytest.mark.gpu
def test_bert_cfg5_bench_cap_step_matches_oracle():
    """The same 1M-item step at the bench's own batch (64) and labelled-row cap (1,792): ~1,450 labelled rows, so
    the head's row tiles, the dE / dh GEMMs' row dimension and the token table's inverted index run at the
    benchmarked size (the batch-1 test above fits one tile).  The fp64 oracle applies the output layer to the
    labelled rows only (oracle.bert.loss_and_grads(labelled_only=True): the same loss and gradients, pinned against
    its full form on the goldens), which keeps its logits at R x 1M (~12 GB fp64; ~60 GB host memory in all)."""
    import rbm_amd.data as synth
    V, T, B, L = 1_000_000, 200, 64, 4
    m = _bert(V, T, 256, L, 2, 0.1, "bf16", seed=5)
    rng = np.random.default_rng(8)
    tok, lab = (torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, T, V, mask_prob=0.2))
    n_lab = int((lab != 0).sum())
    assert 1024 < n_lab <= 1792, n_lab
    loss, l64, worst = _bert_step_vs_oracle(m, tok, lab, L, 2, 0.1, cap=1792, labelled_only=True)
    print("cfg5 bf16 step, rows", n_lab, ": loss", loss, l64, "worst", max(worst.items(), key=lambda kv: kv[1]))
    assert abs(loss - l64) < FWD_TOL_BF16 * abs(l64), (loss, l64)
    bad = {k: v for k, v in worst.items() if v >= GRAD_TOL_BF16}
    assert not bad, bad


@pytest.mark.gpu
def test_bert_cfg5_token_table_gradient_touches_batch_rows_only():
    """1M-item vocabulary: rows of out.weight no labelled row's softmax touches still get the dense softmax
    gradient; the token table gets gradient only on the batch's tokens (padding_idx 0 excluded)."""
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    V, T, B = 1_000_000, 20, 2
    m = _bert(V, T, 256, 1, 2, 0.0, "bf16", seed=5)
    tr = FusedTrainStep(m, lr=1e-3, max_labelled=128)
    rng = np.random.default_rng(6)
    tok, lab = (torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, T, V, mask_prob=0.3))
    tr.flat.grad.zero_()
    tr._compute(tok, lab)
    torch.cuda.synchronize()
    tok_rows = torch.unique(tok.cpu())
    gt = tr.flat.view("bert.embedding.token.weight", tr.flat.grad).cpu()
    untouched = torch.ones(gt.shape[0], dtype=torch.bool)
    untouched[tok_rows] = False
    assert gt[untouched].abs().max().item() == 0.0
    assert gt[0].abs().max().item() == 0.0
    go = tr.flat.view("out.weight", tr.flat.grad).cpu()
    assert (go.abs().sum(1) > 0).float().mean().item() > 0.99


@pytest.mark.gpu
def test_bert_large_vocab_overwritten_head_grads_match_zeroed():
    """Large vocabulary (V * d >= 2^24): out.weight / out.bias get their whole gradient written every step (dE GEMM
    without accumulate) and the optimizer updates that range in its own launch without zeroing it
    (FusedAdam.step keep, BERTEngine.overwritten_grads).  Three steps must give the same bits as the same steps
    with the range zeroed like the rest of the buffer."""
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    V, T, B = 70000, 40, 8
    rng = np.random.default_rng(3)
    batches = [tuple(torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, T, V, mask_prob=0.2))
               for _ in range(3)]
    params = []
    for keep in (True, False):
        torch.manual_seed(0)     # the engine draws its dropout-site salts from torch's generator
        m = _bert(V, T, 256, 1, 2, 0.1, "bf16", seed=11)
        tr = FusedTrainStep(m, lr=1e-3, max_labelled=128)
        assert (tr.engine.overwritten_grads() is not None) or not keep
        if not keep:
            tr.engine.overwritten_grads = lambda: None
        tr.engine.seed_base.fill_(99)
        for tok, lab in batches:
            tr.step(tok, lab)
        torch.cuda.synchronize()
        params.append(tr.flat.data.clone())
        if keep:   # the kept range holds the last step's gradient, the rest is zero
            lo, hi = tr.engine.overwritten_grads()
            assert float(tr.flat.grad[lo:hi].abs().sum()) > 0
            assert float(tr.flat.grad[:lo].abs().sum()) == 0
    diff = {k: float((tr.flat.view(k, params[0]) - tr.flat.view(k, params[1])).abs().max()) for k in tr.flat.names}
    assert torch.equal(params[0], params[1]), {k: v for k, v in diff.items() if v}


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_bert_early_head_adam_equals_end_of_step(graph, monkeypatch):
    """The out.weight / out.bias update forked onto a side stream right after the head's dE / dh (beside the encoder's
    backward; FusedTrainStep._early_head_update, RS_EARLY_HEAD_ADAM) gives the same bits as the update at the end of
    the step -- and the token table's update forked after its gradient, beside the grouped weight gradients
    (RS_EARLY_TOKEN_ADAM): three steps, eager and graph-replayed (two steps unrolled per replay), with the head's
    gradient range left unzeroed (V * d >= 2^24: the only vocabularies the early update runs at)."""
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    V, T, B = 70000, 40, 8
    rng = np.random.default_rng(5)
    batches = [tuple(torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, T, V, mask_prob=0.2))
               for _ in range(4)]
    res = []
    for early in ("1", "0"):
        monkeypatch.setenv("RS_EARLY_HEAD_ADAM", early)
        monkeypatch.setenv("RS_EARLY_TOKEN_ADAM", early)
        torch.manual_seed(0)
        m = _bert(V, T, 256, 1, 2, 0.1, "bf16", seed=12)
        tr = FusedTrainStep(m, lr=1e-3, max_labelled=128)
        assert tr._early_ok == (early == "1")
        tr.engine.seed_base.fill_(77)
        if graph:
            tr.capture(*batches[0], warmup=1, steps_per_graph=2)
            pk = lambda bs: torch.stack([torch.stack(b) for b in bs])   # noqa: E731  [S, 2, B, T]
            losses = [tr.replay_packed(pk(batches[0:2])).cpu().tolist(),
                      tr.replay_packed(pk(batches[2:4])).cpu().tolist()]
        else:
            losses = [float(tr.step(tok, lab).item()) for tok, lab in batches[:3]]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.clone(), tr.opt.m.clone(), tr.opt.v.clone(), tr.opt.state.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)





@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_bert_ln_in_gemm_equals_separate_launches(graph, monkeypatch):
    """The sublayers' LayerNorms inside the QKV / FFN1 GEMMs (rs_gemm_ln, RS_GEMM_LN=1) give the same bits as
    rs_layernorm_fwd + rs_gemm (RS_GEMM_LN=0) over whole training steps: losses, parameters, Adam moments (d = 256,
    dropout on, eager and graph-replayed)."""
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    V, T, B = 3000, 64, 8
    rng = np.random.default_rng(17)
    batches = [tuple(torch.from_numpy(t).cuda() for t in synth.bert_batch(rng, B, T, V, mask_prob=0.2))
               for _ in range(3)]
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("RS_GEMM_LN", on)
        torch.manual_seed(0)
        m = _bert(V, T, 256, 2, 2, 0.1, "bf16", seed=5)
        tr = FusedTrainStep(m, lr=1e-3, max_labelled=B * T)
        tr.engine.seed_base.fill_(41)
        if graph:
            tr.capture(*batches[0], warmup=1)
            losses = [float(tr.replay(*b).item()) for b in batches[1:]]
        else:
            losses = [float(tr.step(*b).item()) for b in batches]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.clone(), tr.opt.m.clone(), tr.opt.v.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)
