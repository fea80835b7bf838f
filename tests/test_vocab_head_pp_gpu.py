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
