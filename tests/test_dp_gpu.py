"""The data-parallel training step on the GPU through RCCL (a world_size-1 'nccl' process group:
one MI355X per test box), eager and HIP-graph-captured: unnormalised backward + aux
(loss sum, count) + all-reduce + Adam-side division gives the same update as the
single-device step (which divides inside the loss kernel like the reference)."""
import argparse
import warnings
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _model(kind, seed):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    torch.manual_seed(seed)
    if kind == "sas":
        a = argparse.Namespace(model_code="sas", num_items=500, max_len=50, device="cuda", sas_hidden_units=64,
                               sas_num_blocks=2, sas_heads=1, sas_dropout=0.0, l2_emb=0.0, rs_dtype="fp32")
    else:
        a = argparse.Namespace(model_code="bert", num_items=500, max_len=50, device="cuda", bert_hidden_units=64,
                               bert_num_blocks=2, bert_num_heads=2, bert_dropout=0.0, bert_hidden_dropout=0.0,
                               bert_mask_prob=0.2, model_init_seed=seed, rs_dtype="fp32")
    return model_factory(a)


def _batches(kind, n):
    import rbm_amd.data as synth
    rng = np.random.default_rng(11)
    out = []
    for _ in range(n):
        b = synth.sas_batch(rng, 6, 50, 500) if kind == "sas" else synth.bert_batch(rng, 6, 50, 500)
        out.append(tuple(torch.from_numpy(x).cuda() for x in b))
    return out


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("kind", ["sas", "bert"])
def test_dp_step_equals_single_device_step(nccl_group, kind, graph, overlap):
    """overlap: bucket all-reduces launched between graph segments as the backward finishes them
    (dp.BucketedExchange); else one bucketed all-reduce after the backward."""
    from rbm_amd.train_step import FusedTrainStep
    batches = _batches(kind, 4)
    res = {}
    for dp in (False, True):
        m = _model(kind, 3)
        tr = FusedTrainStep(m, lr=1e-3, dp=dp, bucket_numel=None if (overlap or not dp) else 8192,
                            overlap=overlap if dp else None)
        if dp and overlap and kind == "bert":
            assert len(tr.exchange.buckets) == 2          # vocabulary head first, then the rest
        if graph:
            tr.capture(*batches[0])
            # capture() ran warm-up steps: restart from the same weights for both arms
        losses = []
        for b in batches:
            losses.append(float((tr.replay(*b) if graph else tr.step(*b)).item()))
        res[dp] = (losses, tr.flat.data.detach().cpu().clone())
    l0, p0 = res[False]
    l1, p1 = res[True]
    assert np.allclose(l0, l1, rtol=1e-5, atol=1e-6), (l0, l1)
    # Adam turns rounding-level gradient differences into lr-sized steps where the true gradient is
    # ~0 (the attention key bias: analytically zero, numerically noise), so the parameters agree to
    # ~1e-5 relative, not to the last bit
    assert rel(p1.numpy(), p0.numpy()) < 3e-4


@pytest.mark.parametrize("kind", ["sas", "bert"])
def test_dp_overlap_bitwise_equals_single_allreduce_bf16(nccl_group, kind):
    """bf16 fused steps (SAS: one bucket, issued by the exchange after the backward; BERT: the vocabulary head's
    bucket cut after its weight gradient): the overlapped, segment-captured DP step gives bit-identical parameters
    to the one-all-reduce DP step."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    batches = _batches(kind, 3)
    res = []
    for overlap in (False, True):
        torch.manual_seed(5)
        if kind == "sas":
            a = argparse.Namespace(model_code="sas", num_items=500, max_len=50, device="cuda", sas_hidden_units=128,
                                   sas_num_blocks=2, sas_heads=1, sas_dropout=0.1, l2_emb=0.0, rs_dtype="bf16")
        else:
            a = argparse.Namespace(model_code="bert", num_items=500, max_len=50, device="cuda", bert_hidden_units=64,
                                   bert_num_blocks=2, bert_num_heads=2, bert_dropout=0.1, bert_hidden_dropout=0.1,
                                   bert_mask_prob=0.2, model_init_seed=5, rs_dtype="bf16")
        m = model_factory(a)
        tr = FusedTrainStep(m, lr=1e-3, dp=True, overlap=overlap, bucket_numel=None if overlap else 1 << 30)
        assert len(tr.exchange.buckets) == (1 if kind == "sas" else 2) if overlap else tr.exchange is None
        tr.capture(*batches[0])
        losses = [float(tr.replay(*b).item()) for b in batches]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.detach().cpu().clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_dp_graph_collectives_equal_segmented(nccl_group, monkeypatch):
    """SAS under DP with the all-reduce captured inside the step graph (one step per replay, and two steps
    unrolled into one replay) against the segmented form (step graph, all-reduce between replays, optimizer
    graph): bit-identical parameters and losses (bf16 fused step, dropout on, l2_emb > 0)."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    batches = _batches("sas", 4)
    res = []
    for mode, S in (("0", 1), ("1", 1), ("1", 2)):
        monkeypatch.setenv("RS_DP_GRAPH_COLLECTIVES", mode)
        torch.manual_seed(5)
        a = argparse.Namespace(model_code="sas", num_items=500, max_len=50, device="cuda", sas_hidden_units=128,
                               sas_num_blocks=2, sas_heads=1, sas_dropout=0.1, l2_emb=0.01, rs_dtype="bf16")
        tr = FusedTrainStep(model_factory(a), lr=1e-3, dp=True)
        assert tr.graph_collectives == (mode == "1")
        tr.capture(*batches[0], steps_per_graph=S)
        assert len(tr.graphs) == (1 if mode == "1" else 2)
        if S == 1:
            losses = [float(tr.replay(*b).item()) for b in batches]
        else:
            losses = []
            for j in range(0, len(batches), S):
                packed = torch.stack([torch.stack(b) for b in batches[j:j + S]])
                losses += [float(x) for x in tr.replay_packed(packed).cpu()]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.detach().cpu().clone()))
    for losses, params in res[1:]:
        assert losses == res[0][0], (losses, res[0][0])
        assert torch.equal(params, res[0][1])


@pytest.mark.parametrize("variant", ["buckets", "sparse", "vocab_shard"])
def test_dp_graph_collectives_equal_segmented_bert(nccl_group, monkeypatch, variant):
    """BERT under DP with every collective captured inside the step graph -- the vocabulary head's bucket issued at
    its point of the backward (forked onto the process group's stream, joined before Adam), the sparse token-table
    exchange's id gather and compact all-reduce, or the vocabulary-sharded head's gathers / reductions -- one step
    per replay and two steps unrolled, against the segmented form (collectives issued between segment graphs):
    bit-identical losses and parameters (bf16 fused step, dropout on)."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    batches = _batches("bert", 4)
    res = []
    for mode, S in (("0", 1), ("1", 1), ("1", 2)):
        monkeypatch.setenv("RS_DP_GRAPH_COLLECTIVES", mode)
        torch.manual_seed(5)
        a = argparse.Namespace(model_code="bert", num_items=500, max_len=50, device="cuda", bert_hidden_units=64,
                               bert_num_blocks=2, bert_num_heads=2, bert_dropout=0.1, bert_hidden_dropout=0.1,
                               bert_mask_prob=0.2, model_init_seed=5, rs_dtype="bf16")
        tr = FusedTrainStep(model_factory(a), lr=1e-3, dp=True, vocab_shard=variant == "vocab_shard",
                            sparse_rows="on" if variant == "sparse" else "off")
        assert tr.graph_collectives == (mode == "1")
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            tr.capture(*batches[0], steps_per_graph=S)
        # no segment graph captures nothing (the sparse form's leading id all-gather used to leave an empty one)
        assert not [str(w.message) for w in caught if "Graph is empty" in str(w.message)]
        if mode == "0":
            assert all(g is not None for g in tr.graphs)
        if variant == "sparse":
            assert tr.sparse is not None
        if mode == "1":
            assert len(tr.graphs) == 1
        if S == 1:
            losses = [float(tr.replay(*b).item()) for b in batches]
        else:
            losses = []
            for j in range(0, len(batches), S):
                packed = torch.stack([torch.stack(b) for b in batches[j:j + S]])
                losses += [float(x) for x in tr.replay_packed(packed).cpu()]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.detach().cpu().clone()))
    for losses, params in res[1:]:
        assert losses == res[0][0], (losses, res[0][0])
        assert torch.equal(params, res[0][1])


def test_dp_large_vocab_unzeroed_head_grads_equal_zeroed(nccl_group):
    """DP (in-graph all-reduce) with a vocabulary large enough (V * d >= 2^24) that the optimizer leaves the output
    layer's gradient range unzeroed (BERTEngine.overwritten_grads -> FusedAdam.step keep): the bucket holding that
    range is all-reduced IN PLACE every step, so the head must overwrite it whole before the exchange.  Three
    graph-replayed steps equal, bit for bit, the same steps with the range zeroed by the optimizer."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    V, T, d, B = 262_144, 32, 64, 4
    rng = np.random.default_rng(9)
    import rbm_amd.data as synth
    batches = [tuple(torch.from_numpy(x).cuda() for x in synth.bert_batch(rng, B, T, V, mask_prob=0.3))
               for _ in range(3)]
    res = []
    for keep in (True, False):
        torch.manual_seed(6)
        a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=d,
                               bert_num_blocks=1, bert_num_heads=2, bert_dropout=0.1, bert_hidden_dropout=0.1,
                               bert_mask_prob=0.3, model_init_seed=6, rs_dtype="bf16")
        tr = FusedTrainStep(model_factory(a), lr=1e-3, dp=True)
        assert tr.engine.overwritten_grads() is not None
        if not keep:
            tr.engine.overwritten_grads = lambda: None
        tr.capture(*batches[0], warmup=1)
        losses = [float(tr.replay(*b).item()) for b in batches]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.detach().cpu().clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_dp_sharded_item_table_equals_dense_rccl(nccl_group, monkeypatch):
    """The sharded item-table optimizer (dp.ShardedRows: in-place RCCL reduce_scatter_tensor of the table's gradient,
    Adam over the owned part, in-place all_gather_into_tensor of the bf16 rows) through RCCL -- eager, segmented
    graphs, the collectives captured in the step graph, and two steps unrolled into one graph -- against the dense
    all-reduce step: bit-identical losses and parameters (world size 1 here: the two-rank form against the oracle is
    tests/test_dp_multirank_gpu.py::test_two_rank_sharded_item_table)."""
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    batches = _batches("sas", 4)
    res = []
    runs = (("off", "1", 1), ("on", "0", 1), ("on", "1", 1), ("on", "1", 2), ("off", None, 1), ("on", None, 1))
    for shard, mode, S in runs:
        monkeypatch.setenv("RS_DP_GRAPH_COLLECTIVES", mode or "1")
        torch.manual_seed(5)
        a = argparse.Namespace(model_code="sas", num_items=500, max_len=50, device="cuda", sas_hidden_units=128,
                               sas_num_blocks=2, sas_heads=1, sas_dropout=0.1, l2_emb=0.0, rs_dtype="bf16")
        tr = FusedTrainStep(model_factory(a), lr=1e-3, dp=True, shard_rows=shard)
        assert (tr.rshard is not None) == (shard == "on")
        if mode is None:                       # eager steps
            losses = [float(tr.step(*b).item()) for b in batches]
        else:
            tr.capture(*batches[0], steps_per_graph=S)
            if S == 1:
                losses = [float(tr.replay(*b).item()) for b in batches]
            else:
                losses = []
                for j in range(0, len(batches), S):
                    packed = torch.stack([torch.stack(b) for b in batches[j:j + S]])
                    losses += [float(x) for x in tr.replay_packed(packed).cpu()]
        assert tr.replicas_equal()
        tr.gather_shards()
        torch.cuda.synchronize()
        res.append((losses, tr.flat.data.detach().cpu().clone(), tr.flat.bf16.detach().cpu().clone()))
    # the captured forms (warm-up steps before the measured ones) against the captured dense step; eager against eager
    for k, ref in ((1, 0), (2, 0), (3, 0), (5, 4)):
        assert res[k][0] == res[ref][0], (runs[k], res[k][0], res[ref][0])
        assert torch.equal(res[k][1], res[ref][1]), runs[k]
        assert torch.equal(res[k][2], res[ref][2]), runs[k]
