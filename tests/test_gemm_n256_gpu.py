"""Large-tile N = 256 GEMM (gemm_n256.hip) for the vocabulary head's dE = dlogits^T h (+ bias column sums) and
dh = dlogits E (split over the vocabulary), against torch float64 on the same bf16 operands: edge row tiles, partial
k stages, a device row-count bound, bit-for-bit repeatable."""
import numpy as np
import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu


def _bf(shape, scale=1.0, seed=0, pad_cols=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    full = (torch.randn(shape[0], shape[1] + pad_cols, device="cuda", generator=g) * scale).bfloat16()
    return full[:, :shape[1]]


@pytest.mark.parametrize("R,V,count", [(1750, 5000, None), (512, 1024, None), (1792, 26745, 1700), (64, 300, 40),
                                       (130, 257, None)])
def test_dE_and_bias_match_float64(R, V, count):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    dl = _bf((R, V), 1e-2, seed=1, pad_cols=(-V) % 64)        # row stride padded to 64 like the workspace
    h = _bf((R, 256), 1.0, seed=2)
    dE = torch.full((V, 256), float("nan"), device="cuda")
    db = torch.full((V,), float("nan"), device="cuda")
    rows = None if count is None else torch.tensor([count], dtype=torch.int32, device="cuda")
    ops.gemm_n256(dl, h, dE, True, V, R, colsum=db, rows_dev=rows)
    k = R if count is None else count
    ref = dl[:k].double().t() @ h[:k].double()
    rb = dl[:k].double().sum(0)
    assert rel(dE.cpu().numpy(), ref.cpu().numpy()) < 2e-6
    assert rel(db.cpu().numpy(), rb.cpu().numpy()) < 2e-6
    again = torch.empty_like(dE)
    ops.gemm_n256(dl, h, again, True, V, R, colsum=None, rows_dev=rows)
    assert torch.equal(again, dE)


@pytest.mark.parametrize("R,V,count", [(1792, 1000001, 1750), (512, 26745, None), (300, 70000, 200), (256, 64, None)])
def test_dh_split_matches_float64(R, V, count):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    dl = _bf((R, V), 1e-2, seed=3, pad_cols=(-V) % 64)
    E = _bf((V, 256), 0.05, seed=4)
    S = ops.gemm_n256_splits(R, V)
    assert S >= 1
    slab = torch.full((S, R, 256), float("nan"), device="cuda")
    rows = None if count is None else torch.tensor([count], dtype=torch.int32, device="cuda")
    ops.gemm_n256(dl, E, slab, False, R, V, split=True, rows_dev=rows)
    m = R if count is None else count
    got = slab[:, :m].double().sum(0)
    ref = dl[:m].double() @ E.double()
    assert rel(got.cpu().numpy(), ref.cpu().numpy()) < 2e-6
    again = torch.empty_like(slab)
    ops.gemm_n256(dl, E, again, False, R, V, split=True, rows_dev=rows)
    assert torch.equal(again[:, :m], slab[:, :m])


@pytest.mark.parametrize("R,V,count,max_wg", [(1750, 5000, None, 0), (300, 70001, 200, 64), (130, 257, None, 1),
                                              (1750, 5000, None, 7)])
def test_dE_adam_epilogue_equals_gemm_then_sweep(R, V, count, max_wg):
    """rs_gemm_n256_adam (dE with torch.optim.Adam applied to the parameter rows in the epilogue) = rs_gemm_n256 into
    a gradient buffer followed by rs_adam_step over those rows: the same bits in p, m, v, the bf16 copy and the bias
    column sums -- one workgroup per row tile (max_wg 0) or a bounded grid walking them."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    dl = _bf((R, V), 1e-2, seed=5, pad_cols=(-V) % 64)
    h = _bf((R, 256), 1.0, seed=6)
    g = torch.Generator(device="cuda").manual_seed(7)
    p0 = torch.randn(V, 256, device="cuda", generator=g) * 0.05
    m0 = torch.randn(V, 256, device="cuda", generator=g) * 1e-3
    v0 = torch.rand(V, 256, device="cuda", generator=g) * 1e-6
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0], dtype=torch.float64, device="cuda")
    rows = None if count is None else torch.tensor([count], dtype=torch.int32, device="cuda")
    outs = []
    for fused in (True, False):
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        pb = torch.empty(V, 256, dtype=torch.bfloat16, device="cuda")
        db = torch.full((V,), float("nan"), device="cuda")
        st = torch.zeros(144, dtype=torch.float64, device="cuda")
        st[0] = 6.0
        ops.adam_prepare(st, hyper)
        if fused:
            ops.gemm_n256_adam(dl, h, V, R, p, m, v, pb, st, hyper, colsum=db, rows_dev=rows, max_wg=max_wg)
        else:
            gr = torch.empty(V, 256, device="cuda")
            ops.gemm_n256(dl, h, gr, True, V, R, colsum=db, rows_dev=rows)
            ops.adam_step(p.view(-1), gr.view(-1), m.view(-1), v.view(-1), pb.view(-1), st, hyper)
        torch.cuda.synchronize()
        outs.append((p, m, v, pb, db))
    for name, a, b in zip(("p", "m", "v", "pb", "db"), *outs):
        assert torch.equal(a, b), (name, float((a.float() - b.float()).abs().max()),
                                   int((a != b).sum()), (a != b).nonzero()[:4].tolist())
