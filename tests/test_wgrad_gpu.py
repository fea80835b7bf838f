"""Grouped weight-gradient GEMMs + grouped reduction (wgrad.hip) vs a torch fp32 reference.

dW[N][K] += dY^T X and db[N] += colsum(dY) for several problems in one launch, with ragged
row counts (the last split partial) and extra partial-sum segments reduced by the same launch.
Operands are bf16, accumulation fp32: the reference is the fp32 product of the same bf16 values.
"""
import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,M,rows", [(128, 25600, 640), (128, 1000, 128), (64, 111, 64), (64, 3000, 256)])
def test_wgrad_grouped_matches_torch(d, M, rows):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    g = torch.Generator(device="cuda").manual_seed(d + M)
    dev = "cuda"
    shapes = [(d, d), (2 * d, d), (d, d)]
    probs, refs = [], []
    for N, K in shapes:
        dY = torch.randn(M, N, device=dev, generator=g).bfloat16()
        X = torch.randn(M, K, device=dev, generator=g).bfloat16()
        dW = torch.randn(N, K, device=dev, generator=g)
        db = torch.randn(N, device=dev, generator=g)
        refs.append((dW + dY.float().t() @ X.float(), db + dY.float().sum(0)))
        probs.append((dY, X, dW, db))
    probs[2] = probs[2][:3] + (None,)                       # a problem without a bias
    # an extra segment set: 37 partials of 2*64 floats each summed into two outputs
    part = torch.randn(37, 2, 64, device=dev, generator=g)
    o1, o2 = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    e1, e2 = o1 + part[:, 0].sum(0), o2 + part[:, 1].sum(0)
    extra = [(part.view(-1), 128, 37, 64, o1), (part.view(-1)[64:], 128, 37, 64, o2)]
    slab = torch.empty(ops.wgrad_grouped_slab_numel(shapes, M, rows), device=dev)
    ops.wgrad_grouped(probs, M, rows, slab, extra=extra)
    torch.cuda.synchronize()
    for i, ((dY, X, dW, db), (rW, rb)) in enumerate(zip(probs, refs)):
        assert rel(dW.cpu().numpy(), rW.cpu().numpy()) < 1e-5, i
        if db is not None:
            assert rel(db.cpu().numpy(), rb.cpu().numpy()) < 1e-5, i
    assert rel(o1.cpu().numpy(), e1.cpu().numpy()) < 1e-6 and rel(o2.cpu().numpy(), e2.cpu().numpy()) < 1e-6


def test_wgrad_grouped_is_deterministic():
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    M, d = 5000, 128
    dY = torch.randn(M, d, device="cuda").bfloat16()
    X = torch.randn(M, d, device="cuda").bfloat16()
    outs = []
    for _ in range(2):
        dW = torch.zeros(d, d, device="cuda")
        db = torch.zeros(d, device="cuda")
        slab = torch.empty(ops.wgrad_grouped_slab_numel([(d, d)], M, 128), device="cuda")
        ops.wgrad_grouped([(dY, X, dW, db)], M, 128, slab)
        outs.append((dW.clone(), db.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("M,N,K,acc", [(1792, 26745, 256, True), (300, 1000, 64, False), (1000, 130, 128, True)])
def test_linear_wgrad_single_split_direct(M, N, K, acc):
    """rs_linear_wgrad with one split accumulates straight into dW / db (no slab): the BERT vocabulary
    weight gradient (N = |items|+1 not a multiple of 8), with a device row count below M."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    g = torch.Generator(device="cuda").manual_seed(M + N)
    Np = -(-N // 64) * 64                                   # row pitch: a multiple of 8 elements, as the ABI asks
    dY = torch.randn(M, Np, device="cuda", generator=g).bfloat16()[:, :N]
    X = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    dW0 = torch.randn(N, K, device="cuda", generator=g)
    db0 = torch.randn(N, device="cuda", generator=g)
    rows = M - 37
    rows_dev = torch.tensor([rows], dtype=torch.int32, device="cuda")
    dW, db = dW0.clone(), db0.clone()
    slab = torch.empty(1, device="cuda")
    ops.linear_wgrad(dY, X, dW, slab, db=db, split_k=1, accumulate=acc, rows_dev=rows_dev)
    torch.cuda.synchronize()
    ref_w = dY[:rows].float().t() @ X[:rows].float() + (dW0 if acc else 0)
    ref_b = dY[:rows].float().sum(0) + (db0 if acc else 0)
    assert rel(dW.cpu().numpy(), ref_w.cpu().numpy()) < 1e-5
    assert rel(db.cpu().numpy(), ref_b.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("M,rows,d,tmax", [(25600, 1280, 128, 256), (12800, 6400, 256, 256), (1000, 192, 128, 256),
                                           (777, 128, 256, 256), (12800, 3200, 256, 128)])
def test_wgrad_grouped_bench_shapes(M, rows, d, tmax):
    """The grouped launch at the SAS shape (cfg2: 12 d x d weights... here 6, 20 splits) and the BERT layer's four
    weights (cfg3: QKV, output, FFN1, FFN2), with ragged last splits: every weight and bias gradient against float64,
    and two launches give the same bits (fixed-order split reduction)."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    g = torch.Generator(device="cuda").manual_seed(M + d)
    shapes = [(3 * d, d), (d, d), (4 * d, d), (d, 4 * d)] if d == 256 else [(d, d)] * 6
    ops_in = [(torch.randn(M, N, device="cuda", generator=g).bfloat16(),
               torch.randn(M, K, device="cuda", generator=g).bfloat16()) for N, K in shapes]
    outs = []
    for _ in range(2):
        probs = [(dY, X, torch.zeros(N, K, device="cuda"), torch.zeros(N, device="cuda"))
                 for (dY, X), (N, K) in zip(ops_in, shapes)]
        slab = torch.empty(ops.wgrad_grouped_slab_numel(shapes, M, rows), device="cuda")
        ops.wgrad_grouped(probs, M, rows, slab, max_tile=tmax)   # tmax 128 at d = 256: the capped (beside) form
        torch.cuda.synchronize()
        outs.append([(dW.clone(), db.clone()) for _, _, dW, db in probs])
    for (a, b), (c, e) in zip(outs[0], outs[1]):
        assert torch.equal(a, c) and torch.equal(b, e)
    for (dY, X), (dW, db) in zip(ops_in, outs[0]):
        assert rel(dW.double().cpu().numpy(), (dY.double().t() @ X.double()).cpu().numpy()) < 1e-5
        assert rel(db.double().cpu().numpy(), dY.double().sum(0).cpu().numpy()) < 1e-5
