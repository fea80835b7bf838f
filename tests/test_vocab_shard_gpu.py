"""Vocabulary-sharded BERT output layer (rbm_amd.vocab_parallel): two data-parallel
ranks -- processes on ONE GPU, gloo moving the tensors (the product uses RCCL; one GPU per test box) -- each
own half of out.weight / out.bias.  Their losses and, after the shards are gathered, their parameters equal the
single-process step on the concatenated batch (bf16 tolerance: the shard kernels sum in a different order)."""
import argparse
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, rel

pytestmark = pytest.mark.gpu

V, T, D, BR = 3000, 50, 64, 6      # items, max_len, hidden, sequences per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(V=V):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=D,
                           bert_num_blocks=1, bert_num_heads=2, bert_dropout=0.0, bert_hidden_dropout=0.0,
                           bert_mask_prob=0.2, model_init_seed=7, rs_dtype="bf16")
    return model_factory(a)


def _batches(world, steps, V=V):
    import rbm_amd.data as synth
    rng = np.random.default_rng(3)
    return [[synth.bert_batch(rng, BR, T, V, mask_prob=0.3) for _ in range(world)] for _ in range(steps)]


def _worker(rank, world, port, graph, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rbm_amd.train_step import FusedTrainStep
        m = _model()
        tr = FusedTrainStep(m, lr=1e-3, vocab_shard=True, max_labelled=BR * T)
        assert tr.vshard.v1 - tr.vshard.v0 < V + 1
        batches = [[tuple(torch.from_numpy(x).cuda() for x in b[rank])] for b in _batches(world, 3)]
        if graph:
            tr.capture(*batches[0][0])
            tr.load_checkpoint(tr.checkpoint())       # (capture ran warm-up steps) -- exercises the gather too
            m0 = _model()
            m.load_state_dict(m0.state_dict())
            tr.engine.sync_compute_weights()
            tr.opt.m.zero_(); tr.opt.v.zero_(); tr.opt.state.zero_()
        losses = []
        for b in batches:
            losses.append(float((tr.replay(*b[0]) if graph else tr.step(*b[0])).item()))
        ck = tr.checkpoint()
        torch.save({"losses": losses, "sd": {k: v.detach().cpu() for k, v in ck["model_state_dict"].items()}},
                   os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("graph", [False, True])
def test_vocab_sharded_head_equals_single_process(tmp_path, graph):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), graph, str(tmp_path)), nprocs=world, join=True)
    from rbm_amd.train_step import FusedTrainStep
    m = _model()
    tr = FusedTrainStep(m, lr=1e-3, max_labelled=world * BR * T)
    ref_losses = []
    for b in _batches(world, 3):
        tok = torch.from_numpy(np.concatenate([x[0] for x in b])).cuda()
        lab = torch.from_numpy(np.concatenate([x[1] for x in b])).cuda()
        ref_losses.append(float(tr.step(tok, lab).item()))
    ref = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["losses"] == r1["losses"]
    assert np.allclose(r0["losses"], ref_losses, rtol=2e-3), (r0["losses"], ref_losses)
    for k in ref:
        assert torch.equal(r0["sd"][k], r1["sd"][k]), k                # replicas agree after the gather
        if "linear_layers.1.bias" in k:
            continue    # attention key bias: analytically zero gradient, Adam amplifies rounding noise (see test_dp_gpu)
        assert rel(r0["sd"][k].float().numpy(), ref[k].float().numpy()) < 5e-3, (k, rel(r0["sd"][k].numpy(), ref[k].numpy()))


# ---------------------------------------------------------------------------------------------------------------
# The sharded step's gradient against the ORACLE (oracle/bert.py: the float64 restatement of the reference's BERT4Rec
# forward and CE(ignore_index=0), BS/models/bert.py:10,16, BS/trainers/bert.py:36-40) on the concatenated batch.
# V = 100,000: 100,001 output rows, split at row 50,048 (128-aligned, inside one 256-entry forward vocabulary tile of
# the ping-pong head); each rank's owned rows of out.weight / out.bias hold complete gradients of the global mean, the
# rest of the buffer the all-reduced encoder gradients (FusedTrainStep.step up to the optimizer).

VB = 100_000


def _grad_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rbm_amd.train_step import FusedTrainStep
        m = _model(VB)
        tr = FusedTrainStep(m, lr=0.0, vocab_shard=True, max_labelled=BR * T)
        b = tuple(torch.from_numpy(x).cuda() for x in _batches(world, 1, VB)[0][rank])
        tr.flat.grad.zero_()
        tr._compute(*b, split=tr._eager_split, update=True)
        tr.exchange.launch("final")
        tr.exchange.finish()
        torch.cuda.synchronize()
        grads = {k: tr.flat.view(k, tr.flat.grad).detach().cpu().clone() for k in m.state_dict()}
        torch.save({"v0": tr.vshard.v0, "v1": tr.vshard.v1, "loss": float(tr.loss_out[2].item()),
                    "count": float(tr.loss_out[1].item()), "grads": grads}, os.path.join(out_dir, f"g{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_vocab_sharded_gradient_equals_oracle(tmp_path):
    """Loss, labelled count and every gradient tensor (out.weight / out.bias assembled from the owners' rows) against
    the float64 oracle on the concatenated batch, at the bf16 bars of the single-device BERT oracle tests
    (test_bert.py: 3e-2 loss / per tensor); the attention key bias (analytically zero) against the gradient scale."""
    from oracle import bert as obert
    world = 2
    mp.spawn(_grad_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"g{i}.pt", weights_only=True) for i in range(world)]
    assert (r[0]["v0"], r[0]["v1"], r[1]["v0"], r[1]["v1"]) == (0, 50048, 50048, VB + 1)
    assert r[0]["loss"] == r[1]["loss"] and r[0]["count"] == r[1]["count"]
    b = _batches(world, 1, VB)[0]
    tok = torch.from_numpy(np.concatenate([x[0] for x in b]))
    lab = torch.from_numpy(np.concatenate([x[1] for x in b]))
    assert r[0]["count"] == float((lab != 0).sum())
    P = {k: v.detach().cpu().double() for k, v in _model(VB).state_dict().items()}
    torch.set_num_threads(16)
    l64, _, g64 = obert.loss_and_grads(P, tok, lab, 1, 2)
    assert abs(r[0]["loss"] - float(l64)) <= 3e-2 * abs(float(l64)), (r[0]["loss"], float(l64))
    scale = max(float(v.norm()) for v in g64.values())
    errs = {}
    for k, ref in g64.items():
        if k in ("out.weight", "out.bias"):
            g = torch.cat([r[i]["grads"][k][r[i]["v0"]:r[i]["v1"]] for i in range(world)])
        else:
            assert torch.equal(r[0]["grads"][k], r[1]["grads"][k]), k
            g = r[0]["grads"][k]
        g = g.double().numpy()
        if "linear_layers.1.bias" in k:
            assert np.linalg.norm(g) <= 1e-2 * scale, k
            continue
        errs[k] = rel(g, ref.numpy())
    worst = max(errs, key=errs.get)
    print("vocab-sharded head vs oracle: worst", worst, errs[worst])
    assert errs[worst] < 3e-2, (worst, errs[worst])
