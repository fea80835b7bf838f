"""Data-parallel exchange on CPU (gloo, world_size 2): the product's rbm_amd.dp helpers applied to
per-rank UNnormalised gradients + (loss sum, count) aux give exactly the single-process gradient
of the mean loss on the concatenated batch -- the reference's semantics (BS/trainers/sas.py:49,
BS/trainers/bert.py:40) -- even when the ranks hold different valid counts.  The per-rank
gradients come from the CPU oracle (the GPU kernels compute the same quantity; the single-GPU
DP path is covered by tests/test_dp_gpu.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, load_golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat(grads, names, loss_sum, count):
    v = torch.cat([grads[k].reshape(-1) for k in names] + [torch.tensor([loss_sum, count], dtype=grads[names[0]].dtype)])
    return v


def _worker(rank, world, port, kind, bucket, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import rbm_amd  # noqa: F401
    from rbm_amd import dp
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names, flat, _ = _local(kind, rank, world)
        dp.allreduce_grads(flat, bucket_numel=bucket)
        loss = dp.global_mean_loss(flat[-2:])
        g = flat[:-2] / flat[-1]
        torch.save({"g": g, "loss": loss}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _local(kind, rank, world):
    """This rank's share of the batch (rank r takes rows r, r+world, ...): unnormalised grads."""
    from oracle import bert as obert
    from oracle import sas as osas
    if kind == "sas":
        z = load_golden("sas_mid")
        P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
        seq, pos, neg = (torch.from_numpy(z[k])[rank::world] for k in ("seq", "pos", "neg"))
        loss, _, _, g = osas.loss_and_grads(P, seq, pos, neg, int(z["L"]), int(z["h"]))
        cnt = float((pos != 0).sum())
    else:
        z = load_golden("bert_mid")
        P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
        tok, lab = (torch.from_numpy(z[k])[rank::world] for k in ("tokens", "labels"))
        loss, _, g = obert.loss_and_grads(P, tok, lab, int(z["L"]), int(z["h"]))
        cnt = float((lab != 0).sum())
    names = list(P)
    ung = {k: g[k] * cnt for k in names}          # gradient of the loss SUM
    return names, _flat(ung, names, float(loss) * cnt, cnt), cnt


@pytest.mark.parametrize("kind", ["sas", "bert"])
@pytest.mark.parametrize("bucket", [None, 4096])
def test_dp_two_ranks_equal_single_device(kind, bucket, tmp_path):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import bert as obert
    from oracle import sas as osas
    port = _free_port()
    mp.spawn(_worker, args=(2, port, kind, bucket, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert torch.equal(r0["g"], r1["g"])                  # replicas apply the same update
    if kind == "sas":
        z = load_golden("sas_mid")
        P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
        loss, _, _, g = osas.loss_and_grads(P, *(torch.from_numpy(z[k]) for k in ("seq", "pos", "neg")),
                                            int(z["L"]), int(z["h"]))
    else:
        z = load_golden("bert_mid")
        P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
        loss, _, g = obert.loss_and_grads(P, torch.from_numpy(z["tokens"]), torch.from_numpy(z["labels"]),
                                          int(z["L"]), int(z["h"]))
    ref = torch.cat([g[k].reshape(-1) for k in P])
    assert abs(float(r0["loss"]) - float(loss)) < 1e-10 * max(1.0, abs(float(loss)))
    assert float((r0["g"] - ref).norm() / ref.norm()) < 1e-12


def _bucket_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import rbm_amd  # noqa: F401
    from rbm_amd import dp
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(rank)
        flat = torch.randn(1000, generator=g)
        ref = flat.clone()
        dist.all_reduce(ref)
        ex = dp.BucketedExchange(flat, {"final": (0, 300), "dense": (300, 1000)})
        ex.launch("dense")                # launched as soon as final, out of buffer order
        flat[:300] *= 1.0                 # (the rest of the backward writing the other bucket)
        ex.launch("final")
        ex.finish()
        torch.save({"flat": flat, "ref": ref}, os.path.join(out_dir, f"b{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_bucketed_exchange_equals_one_allreduce(tmp_path):
    """dp.BucketedExchange (the data-parallel step's all-reduce, bucket by bucket as the backward finishes them)
    sums exactly what one all-reduce of the whole buffer sums, on every rank."""
    port = _free_port()
    mp.spawn(_bucket_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"b{r}.pt", weights_only=True)
        assert torch.equal(d["flat"], d["ref"])


def test_bucketed_exchange_rejects_bad_buckets():
    import sys
    sys.path.insert(0, ROOT)
    from rbm_amd import dp
    with pytest.raises(AssertionError):
        dp.BucketedExchange(torch.zeros(10), {"a": (0, 4), "b": (5, 10)})     # gap
    with pytest.raises(AssertionError):
        dp.BucketedExchange(torch.zeros(10), {"a": (0, 4)})                    # does not cover


def test_ranks_have_different_counts():
    """The case the global-count normalisation exists for: per-rank means would be wrong."""
    z = load_golden("sas_mid")
    pos = z["pos"]
    counts = [int((pos[r::2] != 0).sum()) for r in range(2)]
    assert counts[0] != counts[1]
    _ = np


def _shard_worker(rank, world, port, V1, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import rbm_amd  # noqa: F401
    from rbm_amd.vocab_parallel import VocabShard
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vs = VocabShard(V1)
        full = torch.full((V1, 3), -1.0)
        full[vs.v0:vs.v1] = torch.arange(vs.v0, vs.v1, dtype=torch.float32)[:, None]   # only owned rows are valid
        vs.gather_rows(full)
        torch.save({"v": (vs.v0, vs.v1), "full": full}, os.path.join(out_dir, f"s{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,V1", [(2, 1001), (3, 300), (2, 129)])
def test_vocab_shard_ranges_and_gather(tmp_path, world, V1):
    """rbm_amd.vocab_parallel.VocabShard: 128-aligned disjoint shards covering [0, V1); gather_rows assembles
    the owners' rows on every rank (the checkpoint layout of the vocabulary-sharded BERT head)."""
    mp.spawn(_shard_worker, args=(world, _free_port(), V1, str(tmp_path)), nprocs=world, join=True)
    spans = []
    for r in range(world):
        d = torch.load(tmp_path / f"s{r}.pt", weights_only=True)
        spans.append(tuple(d["v"]))
        assert torch.equal(d["full"], torch.arange(V1, dtype=torch.float32)[:, None].expand(V1, 3))
    assert spans[0][0] == 0 and spans[-1][1] == V1
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert all(v0 % 128 == 0 for v0, _ in spans)


def _carve_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import rbm_amd  # noqa: F401
    from rbm_amd import dp
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(rank)
        flat = torch.randn(1000, generator=g)
        mine = flat.clone()
        ref = flat.clone()
        dist.all_reduce(ref)
        # the table region [100, 400) leaves the dense buckets (exchanged by dp.SparseRowExchange instead)
        b = dp.carve({"final": (0, 600), "out": (600, 1000)}, 100, 400)
        assert b == {"final": [(0, 100), (400, 600)], "out": [(600, 1000)]}, b
        ex = dp.BucketedExchange(flat, b, partial=True)
        ex.launch("out")
        ex.launch("final")
        ex.finish()
        torch.save({"flat": flat, "ref": ref, "mine": mine}, os.path.join(out_dir, f"c{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_carved_buckets_leave_the_table_region(tmp_path):
    """dp.carve + multi-range buckets (the BERT step with a sparse token-table exchange): every range but the carved
    one is all-reduced exactly as one dense all-reduce sums it; the carved region keeps this rank's values."""
    mp.spawn(_carve_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"c{r}.pt", weights_only=True)
        out = torch.ones(1000, dtype=torch.bool)
        out[100:400] = False
        assert torch.equal(d["flat"][out], d["ref"][out])
        assert torch.equal(d["flat"][100:400], d["mine"][100:400])


def test_sparse_exchange_sizing():
    """The bytes the union-of-touched-rows exchange moves at cfg5 on 8 GPUs, and when it is used."""
    import sys
    sys.path.insert(0, ROOT)
    from rbm_amd import dp
    rows, d, n = 1_000_002, 256, 64 * 200
    assert dp.SparseRowExchange.worthwhile(rows, n, 8)
    assert not dp.SparseRowExchange.worthwhile(rows, n, 1)
    assert not dp.SparseRowExchange.worthwhile(54_543, 128 * 50 * 3, 8)     # SAS cfg4 item table: dense
    cap = min(rows, 8 * n)
    assert cap * d * 4 == 104_857_600 and rows * d * 4 == 1_024_002_048


def _rows_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import rbm_amd  # noqa: F401
    from rbm_amd import dp
    from rbm_amd.flat import FlatParams
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        mod = torch.nn.Module()
        mod.item_emb = torch.nn.Embedding(1001, 3)          # 3,003 elements: 1,003 of them past the N x 64 parts
        mod.lin = torch.nn.Linear(5, 7)
        flat = FlatParams(mod, "cpu")
        rs = dp.ShardedRows(flat, "item_emb.weight")
        g = torch.Generator().manual_seed(rank)
        flat.grad.copy_(torch.randn(flat.grad.numel(), generator=g))
        ref = flat.grad.clone()
        dist.all_reduce(ref)
        ex = dp.BucketedExchange(flat.grad, dp.carve({"final": (0, flat.grad.numel())}, rs.lo, rs.hi), partial=True,
                                 extra={"final": rs.scatter})
        ex.launch("final")
        ex.finish()
        a, b = rs.own
        got = {"own": (a, b), "lo": rs.lo, "hi": rs.hi, "dense": rs.dense_ranges(flat.numel),
               "adam": rs.adam_ranges(flat.numel), "foreign": rs.foreign(),
               "grad_own": flat.grad[a:b].clone(), "ref": ref}
        rs.zero_foreign()
        got["zeroed"] = all(bool((flat.grad[x:y] == 0).all()) for x, y in rs.foreign())
        got["grad_dense"] = rs.dense_ranges(flat.grad.numel())
        got["dense_grads"] = [flat.grad[x:y].clone() for x, y in got["grad_dense"]]
        # the owner's update: each rank writes only its part, then the gather makes the region whole everywhere
        flat.data[rs.lo:rs.hi] = -1.0
        flat.data[a:b] = torch.arange(a, b, dtype=torch.float32)
        rs.gather(flat.data)
        got["data"] = flat.data[rs.lo:rs.hi].clone()
        torch.save(got, os.path.join(out_dir, f"w{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_rows_scatter_gather(tmp_path, world):
    """dp.ShardedRows (the sharded item-table optimizer of the SAS DP step): equal 64-aligned parts tile the sharded
    region; after the exchange each rank's part holds the global gradient sum and the dense ranges (the table's tail
    included) the all-reduced values; zero_foreign clears the rest; gather assembles the owners' parts everywhere."""
    mp.spawn(_rows_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = []
    for r in range(world):
        d = torch.load(tmp_path / f"w{r}.pt", weights_only=True)
        a, b = d["own"]
        parts.append((a, b))
        assert (b - a) % 64 == 0 and b - a == (3003 // (world * 64)) * 64
        # two ranks: a + b in either collective; three: gloo may associate the sums differently per buffer size
        same = torch.equal if world == 2 else (lambda x, y: torch.allclose(x, y, rtol=1e-6, atol=1e-6))
        assert same(d["grad_own"], d["ref"][a:b])
        assert d["dense"][0] == (d["hi"], d["dense"][0][1]) and d["lo"] == 0
        assert d["adam"] == d["dense"] + [(a, b)]
        assert d["zeroed"]
        assert d["grad_dense"][-1][1] == d["ref"].numel()          # the aux tail rides in the dense all-reduce
        for got, (x, y) in zip(d["dense_grads"], d["grad_dense"]):
            assert same(got, d["ref"][x:y])
        assert torch.equal(d["data"], torch.arange(d["lo"], d["hi"], dtype=torch.float32))
    assert parts[0][0] == 0 and all(p[1] == q[0] for p, q in zip(parts, parts[1:]))


def test_sharded_rows_sizing():
    """The cfg4 exchange (SAS, 54,543 x 128 item table, 8 GPUs) with the sharded item-table optimizer against the dense
    all-reduce: ring bytes sent per rank and step."""
    import sys
    sys.path.insert(0, ROOT)
    from rbm_amd import dp
    n_item = 54_543 * 128
    assert dp.ShardedRows.worthwhile(n_item, 8) and not dp.ShardedRows.worthwhile(n_item, 1)
    assert not dp.ShardedRows.worthwhile(501 * 64, 2)
    total = 7_187_328                        # the cfg4 flat buffer (fp32 elements, FlatParams layout)
    dense, sharded = dp.ShardedRows.ring_bytes(total, n_item, 8, 2)
    assert 50.0e6 < dense < 50.5e6 and 37.5e6 < sharded < 38.5e6, (dense, sharded)
