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
