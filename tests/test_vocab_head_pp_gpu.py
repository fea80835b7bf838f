"""The ping-pong vocabulary-head forward (vocab_head.hip ``pp::fwd_kernel``: E held in registers, whole h row tiles
by LDS-DMA, two wave groups half an interval apart) against the lock-step form (``RS_VHEAD_PP=0``) and an fp32
torch restatement of the reference's CE over the full vocabulary (BS/models/bert.py:16, BS/trainers/bert.py:36-40):
loss sum, labelled count, mean, and the per-row log-sum-exp the backward reads."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(h, E, bias, lab, rows_dev, pp):
    from rbm_amd import ops
    R, V1 = h.shape[0], E.shape[0]
    ws = torch.full((ops.vocab_ce_ws_numel(R, V1),), float("nan"), device="cuda")
    out = torch.zeros(4, device="cuda")
    old = os.environ.get("RS_VHEAD_PP")
    os.environ["RS_VHEAD_PP"] = str(pp)
    try:
        ops.vocab_head_fwd(h, E, bias, lab, ws, out, rows_dev=rows_dev)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("RS_VHEAD_PP")
        else:
            os.environ["RS_VHEAD_PP"] = old
    ntn = -(-V1 // 128)
    lse = ws[R * ntn * 2 + R: R * ntn * 2 + 2 * R]
    return out.cpu(), lse.cpu()


# (R, V1, d, live rows): the cfg3 vocabulary (ragged last 256-entry tile), a vocabulary smaller than one tile, an
# odd row count with a partial last 32-row tile, fewer live rows than R (rows_dev), a vocabulary of one tile + 1
@pytest.mark.parametrize("R,V1,d,live", [(1750, 26745, 256, 1750), (37, 200, 64, 37), (130, 5001, 128, 101),
                                         (300, 257, 256, 300), (64, 70001, 256, 61)])
def test_vocab_head_pp_fwd_matches_lockstep_and_fp32(R, V1, d, live):
    import rbm_amd  # noqa: F401
    g = torch.Generator(device="cuda").manual_seed(R + V1)
    h = torch.randn(R, d, device="cuda", generator=g).bfloat16()
    E = (0.08 * torch.randn(V1, d, device="cuda", generator=g)).bfloat16()
    bias = 0.3 * torch.randn(V1, device="cuda", generator=g)
    lab = torch.randint(0, V1, (R,), device="cuda", generator=g)
    lab[::7] = 0                                              # ignore_index rows
    rows_dev = torch.tensor([live], dtype=torch.int32, device="cuda")
    o_pp, l_pp = _run(h, E, bias, lab, rows_dev, 1)
    o_ls, l_ls = _run(h, E, bias, lab, rows_dev, 0)
    logits = h[:live].float() @ E.float().t() + bias
    lse = torch.logsumexp(logits, 1).cpu()
    lv = lab[:live]
    keep = (lv != 0).cpu()
    tgt = logits.gather(1, lv[:, None]).squeeze(1).cpu()
    loss = float((lse - tgt)[keep].sum())
    assert float(o_pp[1]) == float(keep.sum()) == float(o_ls[1])
    assert abs(float(o_pp[0]) - loss) <= 2e-5 * abs(loss) + 1e-3, (float(o_pp[0]), loss)
    assert abs(float(o_pp[0]) - float(o_ls[0])) <= 1e-5 * abs(loss) + 1e-3
    live_rows = torch.arange(live)[keep]
    assert torch.allclose(l_pp[live_rows], lse[live_rows], rtol=0, atol=2e-4)
    assert torch.allclose(l_pp[live_rows], l_ls[live_rows], rtol=0, atol=1e-4)


def _bwd(h, E, bias, lab, ws, cnt, rows_dev, pp, voff=0):
    from rbm_amd import ops
    R, V1 = h.shape[0], E.shape[0]
    V1p = -(-V1 // 8) * 8
    dl = torch.full((R, V1p), 7.0, device="cuda", dtype=torch.bfloat16)[:, :V1]
    old = os.environ.get("RS_VHEAD_PP")
    os.environ["RS_VHEAD_PP"] = str(pp)
    try:
        ops.vocab_head_bwd(h, E, bias, lab, ws, cnt, dl, rows_dev=rows_dev, voff=voff)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("RS_VHEAD_PP")
        else:
            os.environ["RS_VHEAD_PP"] = old
    return dl.float().cpu()


@pytest.mark.parametrize("R,V1,d,live", [(1750, 26745, 256, 1750), (37, 200, 64, 37), (130, 5001, 128, 101),
                                         (300, 257, 256, 300), (64, 70001, 256, 61)])
def test_vocab_head_pp_bwd_matches_lockstep_and_fp32(R, V1, d, live):
    """dlogits = (softmax - onehot(label)) / count (BS/trainers/bert.py:36-40 backward): the ping-pong form against
    the fp32 restatement within bf16 rounding, against the lock-step form, label-0 rows exactly zero, rows past the
    live count untouched."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    g = torch.Generator(device="cuda").manual_seed(R * 3 + V1)
    h = torch.randn(R, d, device="cuda", generator=g).bfloat16()
    E = (0.08 * torch.randn(V1, d, device="cuda", generator=g)).bfloat16()
    bias = 0.3 * torch.randn(V1, device="cuda", generator=g)
    lab = torch.randint(0, V1, (R,), device="cuda", generator=g)
    lab[::5] = 0
    rows_dev = torch.tensor([live], dtype=torch.int32, device="cuda")
    ws = torch.empty(ops.vocab_ce_ws_numel(R, V1), device="cuda")
    out = torch.zeros(4, device="cuda")
    ops.vocab_head_fwd(h, E, bias, lab, ws, out, rows_dev=rows_dev)
    cnt = out[1:2].clone()
    d_pp = _bwd(h, E, bias, lab, ws, cnt, rows_dev, 1)
    d_ls = _bwd(h, E, bias, lab, ws, cnt, rows_dev, 0)
    logits = h[:live].float() @ E.float().t() + bias
    ref = torch.softmax(logits, 1)
    lv = lab[:live]
    ref[torch.arange(live, device="cuda"), lv] -= 1.0
    ref = (ref * (lv != 0)[:, None] / float(cnt)).cpu()
    assert torch.equal(d_pp[live:], torch.full_like(d_pp[live:], 7.0)), "rows past the live count written"
    dead = (lv == 0).cpu()
    assert torch.equal(d_pp[:live][dead], torch.zeros_like(d_pp[:live][dead]))
    tol = 2.0 ** -7 * ref.abs() + 1e-6 / float(cnt)
    assert bool(((d_pp[:live] - ref).abs() <= tol).all()), float((d_pp[:live] - ref).abs().max())
    assert bool(((d_pp[:live] - d_ls[:live]).abs() <= tol).all())


def test_vocab_head_cfg5_vocabulary_full_path_matches_fp64():
    """The whole bf16 vocabulary head at the cfg5 vocabulary (1,000,001 classes, d = 256) with 1,100 labelled rows --
    35 of the ping-pong kernels' 32-row tiles (34 full + a partial one), rows with label 0 among them: the forward
    (loss sum, count, per-row log-sum-exp), dlogits, dE = dlogits^T h with db (rs_gemm_n256, k-major), dh = dlogits
    E (rs_gemm_n256 split over the vocabulary + rs_splitk_scatter_rows), against a float64 torch restatement of the
    reference's CE over the full vocabulary (BS/models/bert.py:10,16, BS/trainers/bert.py:36-40), formed in 64k-class
    chunks."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    R, V1, d = 1100, 1_000_001, 256
    g = torch.Generator(device="cuda").manual_seed(1100)
    h = torch.randn(R, d, device="cuda", generator=g).bfloat16()
    E = (0.06 * torch.randn(V1, d, device="cuda", generator=g)).bfloat16()
    bias = 0.3 * torch.randn(V1, device="cuda", generator=g)
    lab = torch.randint(1, V1, (R,), device="cuda", generator=g)
    lab[::9] = 0
    rows_dev = torch.tensor([R], dtype=torch.int32, device="cuda")
    ws = torch.empty(ops.vocab_ce_ws_numel(R, V1), device="cuda")
    out = torch.zeros(4, device="cuda")
    ops.vocab_head_fwd(h, E, bias, lab, ws, out, rows_dev=rows_dev)
    cnt = out[1:2].clone()
    V1p = -(-V1 // 8) * 8
    dl = torch.empty((R, V1p), device="cuda", dtype=torch.bfloat16)[:, :V1]
    ops.vocab_head_bwd(h, E, bias, lab, ws, cnt, dl, rows_dev=rows_dev)
    dE = torch.empty(V1, d, device="cuda")
    db = torch.empty(V1, device="cuda")
    ops.gemm_n256(dl, h, dE, True, V1, R, colsum=db, rows_dev=rows_dev)
    sk = ops.gemm_n256_splits(R, V1)
    slab = torch.empty(sk * R * d, device="cuda")
    ops.gemm_n256(dl, E, slab.view(sk, R, d), False, R, V1, split=True, rows_dev=rows_dev)
    dh = torch.empty(R, d, device="cuda", dtype=torch.bfloat16)
    ops.splitk_scatter_rows(slab, sk, R, torch.arange(R, dtype=torch.int32, device="cuda"), dh)
    torch.cuda.synchronize()
    ntn = -(-V1 // 128)
    lse_k = ws[R * ntn * 2 + R: R * ntn * 2 + 2 * R].double()
    # float64 reference, 64k classes at a time
    h64, keep = h.double(), (lab != 0)
    n = float(keep.sum())
    C = 1 << 16
    m = torch.full((R,), -float("inf"), device="cuda", dtype=torch.float64)
    s = torch.zeros(R, device="cuda", dtype=torch.float64)
    tgt = torch.zeros(R, device="cuda", dtype=torch.float64)
    for c0 in range(0, V1, C):
        z = h64 @ E[c0:c0 + C].double().t() + bias[c0:c0 + C].double()
        mc = torch.maximum(m, z.max(1).values)
        s = s * torch.exp(m - mc) + torch.exp(z - mc[:, None]).sum(1)
        m = mc
        inside = (lab >= c0) & (lab < c0 + z.shape[1])
        tgt[inside] = z[inside, lab[inside] - c0]
    lse = m + torch.log(s)
    loss = float((lse - tgt)[keep].sum())
    dE64 = torch.empty(V1, d, device="cuda", dtype=torch.float64)
    db64 = torch.empty(V1, device="cuda", dtype=torch.float64)
    dh64 = torch.zeros(R, d, device="cuda", dtype=torch.float64)
    err_dl = 0.0
    for c0 in range(0, V1, C):
        z = h64 @ E[c0:c0 + C].double().t() + bias[c0:c0 + C].double()
        p = torch.exp(z - lse[:, None])
        inside = (lab >= c0) & (lab < c0 + z.shape[1])
        p[inside, lab[inside] - c0] -= 1.0
        p *= keep[:, None].double() / n
        err_dl = max(err_dl, float(((dl[:, c0:c0 + C].double() - p).abs() - 2.0 ** -8 * p.abs()).max()))
        dE64[c0:c0 + C] = p.t() @ h64
        db64[c0:c0 + C] = p.sum(0)
        dh64 += p @ E[c0:c0 + C].double()
    assert float(out[1]) == n
    assert abs(float(out[0]) - loss) <= 2e-5 * abs(loss), (float(out[0]), loss)
    assert float((lse_k - lse)[keep].abs().max()) <= 2e-4
    assert err_dl <= 1e-6 / n, err_dl                           # dlogits: bf16 rounding of the exact value
    rel64 = lambda a, b: float((a.double() - b).norm() / b.norm())   # noqa: E731
    assert rel64(dE, dE64) < 1e-2, rel64(dE, dE64)
    assert rel64(db, db64) < 1e-2, rel64(db, db64)
    assert rel64(dh, dh64) < 1e-2, rel64(dh, dh64)
    print("cfg5 head:", rel64(dE, dE64), rel64(db, db64), rel64(dh, dh64))
