"""Row-marked optimizer sweeps (rs_item_grad_marked + rs_adam_*_marked): the inverted-index gradient stamps the
table rows it writes and the Adam sweep skips the gradient loads of the other rows.  Same bits as the unmarked
sweep: kernel level (a table inside the range, a range starting inside the table, stale stamps of an older step)
and whole training steps (SAS item table, BERT token table with its update forked beside the weight gradients),
eager and graph-replayed."""
import argparse

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prep", [False, True])
@pytest.mark.parametrize("moff", [1000, -4 * 128 * 3, 900_004 - 5000 * 64 + 12])
@pytest.mark.parametrize("dshift", [6, 7, 8])
def test_marked_sweep_equals_unmarked(prep, moff, dshift):
    """moff: the table starts mid-wave inside the range, the range starts inside the table, the table runs past the
    range's end; d = 64 / 128 / 256 (a wave's 256 elements span up to 5 / 3 / 2 rows)."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    rows = 5000
    d = 1 << dshift
    n = 900_004
    gen = torch.Generator(device="cuda").manual_seed(3)
    p0 = torch.randn(n, generator=gen, device="cuda")
    m0 = torch.randn(n, generator=gen, device="cuda").abs() * 1e-3
    v0 = torch.randn(n, generator=gen, device="cuda").abs() * 1e-6
    g0 = torch.randn(n, generator=gen, device="cuda")
    # rows of the table [moff, moff + rows * d) ∩ [0, n): a third stamped this step, the rest with zero gradient,
    # some of those carrying an older stamp
    marks = torch.zeros(ops.row_marks_bytes(rows), dtype=torch.uint8, device="cuda")
    marks[:rows] = torch.randint(0, 256, (rows,), generator=gen, device="cuda", dtype=torch.int64).to(torch.uint8)
    epoch = torch.tensor([77], dtype=torch.uint8, device="cuda")
    touched = torch.rand(rows, generator=gen, device="cuda") < 0.33
    mv = marks[:rows]
    mv[touched] = 77
    mv[~touched & (mv == 77)] = 78
    r = (torch.arange(n, device="cuda") - moff) // d
    inside = (r >= 0) & (r < rows)
    zero = inside & ~touched[r.clamp(0, rows - 1)]
    g0[zero] = 0.0
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01], dtype=torch.float64, device="cuda")
    outs = []
    for mk in (None, (marks, epoch, moff, rows, dshift)):
        p, m, v, g = p0.clone(), m0.clone(), v0.clone(), g0.clone()
        pb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(144, dtype=torch.float64, device="cuda")
        st[0] = 4.0
        if prep:
            ops.adam_prepare_step(p, g, m, v, pb, st, hyper, zero_grad=True, marks=mk)
        else:
            ops.adam_prepare(st, hyper)
            ops.adam_step(p, g, m, v, pb, st, hyper, zero_grad=True, max_wg=300, marks=mk)
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(g)) == 0
        outs.append((p, m, v, pb, st[:4].clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_item_grad_marks_every_written_row():
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    import rbm_amd.data as synth
    V, T, B, d = 20000, 50, 16, 128
    rng = np.random.default_rng(1)
    seq, pos, neg = (torch.from_numpy(x).cuda() for x in synth.sas_batch(rng, B, T, V))
    M = B * T
    iws = torch.empty(ops.item_index_ws_bytes(3, M, V + 1, d), dtype=torch.uint8, device="cuda")
    ops.item_index_build([seq.reshape(-1), pos.reshape(-1), neg.reshape(-1)], V + 1, d, iws)
    dx = torch.randn(M, d, device="cuda").to(torch.bfloat16)
    f = torch.randn(M, d, device="cuda").to(torch.bfloat16)
    w1, w2 = torch.randn(M, device="cuda"), torch.randn(M, device="cuda")
    sb = torch.tensor([0x1234_5678_9A], dtype=torch.int64, device="cuda")
    outs = []
    for marked in (False, True):
        dt = torch.zeros(V + 1, d, device="cuda")
        rm = torch.zeros(ops.row_marks_bytes(V + 1), dtype=torch.uint8, device="cuda")
        rm[:V + 1] = 3
        ep = torch.zeros(1, dtype=torch.uint8, device="cuda")
        ops.item_grad(iws, 3, M, dx, 2.0, 0.2, 99, sb, f, w1, w2, dt, marks=(rm, ep) if marked else None)
        torch.cuda.synchronize()
        outs.append((dt, rm, ep))
    assert torch.equal(outs[0][0], outs[1][0])            # the marks change no gradient bit
    dt, rm, ep = outs[1]
    assert int(ep.item()) == 0x9A                         # the seed's low byte
    keys = torch.unique(torch.cat([seq.reshape(-1), pos.reshape(-1), neg.reshape(-1)]))
    keys = keys[keys != 0]
    stamped = rm[:V + 1] == 0x9A
    assert bool(stamped[keys].all())
    assert int(stamped.sum()) == keys.numel()             # only the batch's keys
    assert not bool(dt[~stamped].any())                   # every row with a gradient is stamped


def _sas(V):
    from rbm_amd.models import model_factory
    torch.manual_seed(0)
    a = argparse.Namespace(model_code="sas", num_items=V, max_len=32, device="cuda", sas_hidden_units=128,
                           sas_num_blocks=2, sas_heads=1, sas_dropout=0.2, l2_emb=0.0, rs_dtype="bf16")
    return model_factory(a)


def _bert(V):
    from rbm_amd.models import model_factory
    torch.manual_seed(0)
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=40, device="cuda", bert_hidden_units=256,
                           bert_num_blocks=1, bert_num_heads=2, bert_dropout=0.1, bert_hidden_dropout=0.1,
                           bert_mask_prob=0.2, model_init_seed=12, rs_dtype="bf16")
    return model_factory(a)


@pytest.mark.parametrize("kind", ["sas", "bert"])
@pytest.mark.parametrize("graph", [False, True])
def test_training_with_row_marks_equals_unmarked(kind, graph, monkeypatch):
    """SAS: a 20k-item table (the marked sweep inside the step's one prepared launch); BERT: a 70k-token vocabulary
    (the early out.weight update and the token table's update forked beside the weight gradients, marked)."""
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    V = 20000 if kind == "sas" else 70000
    rng = np.random.default_rng(5)
    if kind == "sas":
        batches = [torch.stack([torch.from_numpy(x) for x in synth.sas_batch(rng, 16, 32, V)]).cuda()
                   for _ in range(4)]
    else:
        batches = [torch.stack([torch.from_numpy(x) for x in synth.bert_batch(rng, 8, 40, V, mask_prob=0.2)]).cuda()
                   for _ in range(4)]
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("RS_ROW_MARKS", on)
        m = _sas(V) if kind == "sas" else _bert(V)
        tr = FusedTrainStep(m, lr=1e-3, **({} if kind == "sas" else {"max_labelled": 128}))
        assert (tr.opt.marks is not None) == (on == "1")
        if kind == "bert":
            assert tr._early_token
        tr.engine.seed_base.fill_(250)        # the stamp byte wraps (255 -> 0) inside the run
        if graph:
            tr.capture(*batches[0].unbind(0), warmup=1, steps_per_graph=2)
            losses = tr.replay_packed(torch.stack(batches[0:2])).tolist() + \
                tr.replay_packed(torch.stack(batches[2:4])).tolist()
        else:
            losses = [float(tr.step(*b.unbind(0)).item()) for b in batches]
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(tr.flat.grad[:tr.flat.offsets["out.weight"]] if kind == "bert"
                                       else tr.flat.grad)) == 0
        res.append((losses, tr.flat.data.clone(), tr.opt.m.clone(), tr.opt.v.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dshift", [2, 4])
def test_marked_sweep_rejects_narrow_rows(dshift):
    """A wave tests its rows' marks from one 16-byte window of the marks array: rows narrower than 32 elements would
    put more than 9 rows under one wave, so the ABI refuses them (RS_ERR_ARG -> RuntimeError) instead of skipping
    stamped rows."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    n, rows = 4096, 64
    p, g, m, v = (torch.zeros(n, device="cuda") for _ in range(4))
    pb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    st = torch.zeros(144, dtype=torch.float64, device="cuda")
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0], dtype=torch.float64, device="cuda")
    marks = torch.zeros(ops.row_marks_bytes(rows), dtype=torch.uint8, device="cuda")
    epoch = torch.zeros(1, dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError):
        ops.adam_step(p, g, m, v, pb, st, hyper, zero_grad=True, max_wg=8, marks=(marks, epoch, 0, rows, dshift))
