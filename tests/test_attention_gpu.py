"""rs_attn_fwd / rs_attn_bwd vs a plain PyTorch fp32 reference of the same op.

The reference op is the attention core both models run:
  SAS  (mask_kind 0): torch F.multi_head_attention_forward's baddbmm(-inf causal mask) /
       softmax / bmm, called at BS/models/sas_model/sas.py:75
  BERT (mask_kind 1): BS/models/bert_modules/attention/single.py:13-35 -- masked_fill(key
       padding, -1e9) / softmax / matmul
bf16 runs the LDS-resident kernels (attention_lds.hip), fp32 the chunked kernels.
"""
import math

import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2}


def ref_attention(q, k, v, ids, B, T, H, Dh, mask_kind):
    """q,k,v: (B*T, H*Dh) fp32 -> o (B*T, H*Dh)"""
    def heads(x):
        return x.view(B, T, H, Dh).transpose(1, 2)
    s = heads(q) @ heads(k).transpose(-1, -2) / math.sqrt(Dh)
    if mask_kind == 0:
        blocked = torch.triu(torch.ones(T, T, dtype=torch.bool, device=q.device), 1)
        s = s.masked_fill(blocked, float("-inf"))
    else:
        s = s.masked_fill((ids == 0).view(B, 1, 1, T), -1e9)
    p = torch.softmax(s, -1)
    return (p @ heads(v)).transpose(1, 2).reshape(B * T, H * Dh)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("mask_kind", [0, 1])
@pytest.mark.parametrize("B,T,H,Dh", [(3, 200, 1, 128), (2, 50, 2, 64), (2, 16, 2, 32), (2, 256, 2, 128),
                                      (3, 37, 1, 64), (2, 200, 2, 128),
                                      # any head dim / length (generic kernels): the reference's default SAS
                                      # width d = 50 (1 or 2 heads), --max_len 300, T > 256, Dh = 256, d = 300
                                      (2, 200, 1, 50), (2, 200, 2, 25), (2, 300, 1, 128), (1, 513, 2, 64),
                                      (2, 64, 1, 256), (2, 40, 3, 100), (3, 1, 1, 64)])
def test_attention_matches_torch(dtype, mask_kind, B, T, H, Dh):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    torch.manual_seed(B * T + H * Dh + mask_kind)
    d = H * Dh
    dev = "cuda"
    ids = torch.randint(1, 50, (B, T), device=dev)
    for b in range(B):                   # left padding of different lengths (the reference pads left)
        ids[b, : (b * T) // (B + 1)] = 0
    q = torch.randn(B * T, d, device=dev)
    kv = torch.randn(B * T, 2 * d, device=dev)
    q16, kv16 = q.to(dtype), kv.to(dtype)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q16, kv16[:, :d], kv16[:, d:]))
    o_ref = ref_attention(qr, kr, vr, ids, B, T, H, Dh, mask_kind)
    do = torch.randn_like(o_ref).to(dtype)
    o_ref.backward(do.float())

    o = torch.empty(B * T, d, device=dev, dtype=dtype)
    lse = torch.empty(B * H * T, device=dev)
    sc = 1.0 / math.sqrt(Dh)
    ops.attn_fwd(B, T, H, Dh, q16, kv16[:, :d], kv16[:, d:], o, lse, sc, mask_kind, ids, 0.0, 0, None)
    dq = torch.empty_like(q16)
    dkv = torch.empty_like(kv16)
    ws = torch.empty(B * H * T, device=dev)
    ops.attn_bwd(B, T, H, Dh, q16, kv16[:, :d], kv16[:, d:], o, do, lse, dq, dkv[:, :d], dkv[:, d:], sc, mask_kind,
                 ids, 0.0, 0, None, ws)
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel(o.float().cpu(), o_ref.detach().cpu()) < tol
    if T == 1:      # one key: dq is exactly 0 (softmax of one score); the kernel's is rounding noise
        assert dq.float().abs().max().item() < 1e-5 * do.float().abs().max().item() * kv.float().abs().max().item()
    else:
        assert rel(dq.float().cpu(), qr.grad.cpu()) < 2 * tol
    assert rel(dkv[:, :d].float().cpu(), kr.grad.cpu()) < 2 * tol or T == 1
    assert rel(dkv[:, d:].float().cpu(), vr.grad.cpu()) < 2 * tol


@pytest.mark.parametrize("mask_kind", [0, 1])
def test_attention_dropout_is_consistent_between_fwd_and_bwd(mask_kind):
    """With dropout on, the backward must regenerate exactly the forward's mask: check the
    bf16 kernels against the fp32 kernels run with the same seed (same counter-based RNG)."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    torch.manual_seed(5)
    B, T, H, Dh = 2, 200, 1, 128
    d = H * Dh
    dev = "cuda"
    ids = torch.randint(1, 50, (B, T), device=dev)
    ids[0, :60] = 0
    q = torch.randn(B * T, d, device=dev)
    kv = torch.randn(B * T, 2 * d, device=dev)
    do = torch.randn(B * T, d, device=dev)
    sb = torch.full((1,), 3, dtype=torch.int64, device=dev)
    outs = {}
    for dt in (torch.float32, torch.bfloat16):
        qq, kk, dd = q.to(dt), kv.to(dt), do.to(dt)
        o = torch.empty(B * T, d, device=dev, dtype=dt)
        lse = torch.empty(B * H * T, device=dev)
        ops.attn_fwd(B, T, H, Dh, qq, kk[:, :d], kk[:, d:], o, lse, 0.1, mask_kind, ids, 0.2, 77, sb)
        dq, dkv = torch.empty_like(qq), torch.empty_like(kk)
        ws = torch.empty(B * H * T, device=dev)
        ops.attn_bwd(B, T, H, Dh, qq, kk[:, :d], kk[:, d:], o, dd, lse, dq, dkv[:, :d], dkv[:, d:], 0.1, mask_kind,
                     ids, 0.2, 77, sb, ws)
        outs[dt] = [t.float().cpu() for t in (o, dq, dkv)]
    torch.cuda.synchronize()
    for a, b in zip(outs[torch.bfloat16], outs[torch.float32]):
        assert rel(a, b) < 3e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("mask_kind", [0, 1])
@pytest.mark.parametrize("B,T,H,Dh", [(3, 200, 1, 128), (3, 37, 2, 64), (2, 200, 1, 50), (2, 300, 1, 128)])
def test_attention_dropout_matches_torch_with_the_kernels_mask(dtype, mask_kind, B, T, H, Dh):
    """Attention-probability dropout (sas.py:75 MHA dropout, single.py:33) at p = 0.2: the keep mask the kernels
    draw (materialised through rs_dropout_rowmask with the documented index ((b*H+h)*T+q)*Tp + k) applied in the
    torch reference gives the kernels' outputs and gradients -- LDS-resident (bf16 T <= 256) and generic kernels."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    torch.manual_seed(T + Dh)
    p, salt = 0.2, 0x1234567
    d = H * Dh
    dev = "cuda"
    ids = torch.randint(1, 50, (B, T), device=dev)
    ids[0, : T // 3] = 0
    sb = torch.full((1,), 99, dtype=torch.int64, device=dev)
    Tp = T + (T & 1)
    ones = torch.ones(B * H * T, Tp, device=dev)
    mult = torch.empty_like(ones)
    ops.dropout_rowmask(ones, p, salt, sb, None, mult)
    mask = (mult[:, :T] > 0).float().view(B, H, T, T)
    q = torch.randn(B * T, d, device=dev).to(dtype)
    kv = torch.randn(B * T, 2 * d, device=dev).to(dtype)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, kv[:, :d], kv[:, d:]))

    def heads(x):
        return x.view(B, T, H, Dh).transpose(1, 2)
    s_ = heads(qr) @ heads(kr).transpose(-1, -2) / math.sqrt(Dh)
    if mask_kind == 0:
        s_ = s_.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=dev), 1), float("-inf"))
    else:
        s_ = s_.masked_fill((ids == 0).view(B, 1, 1, T), -1e9)
    pr = torch.softmax(s_, -1) * mask / (1 - p)
    o_ref = (pr @ heads(vr)).transpose(1, 2).reshape(B * T, d)
    do = torch.randn_like(o_ref).to(dtype)
    o_ref.backward(do.float())
    o = torch.empty(B * T, d, device=dev, dtype=dtype)
    lse = torch.empty(B * H * T, device=dev)
    sc = 1.0 / math.sqrt(Dh)
    ops.attn_fwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, lse, sc, mask_kind, ids, p, salt, sb)
    dq, dkv = torch.empty_like(q), torch.empty_like(kv)
    ws = torch.empty(B * H * T, device=dev)
    ops.attn_bwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, do, lse, dq, dkv[:, :d], dkv[:, d:], sc, mask_kind, ids, p,
                 salt, sb, ws)
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel(o.float().cpu(), o_ref.detach().cpu()) < tol
    assert rel(dq.float().cpu(), qr.grad.cpu()) < 2 * tol
    assert rel(dkv[:, :d].float().cpu(), kr.grad.cpu()) < 2 * tol
    assert rel(dkv[:, d:].float().cpu(), vr.grad.cpu()) < 2 * tol


@pytest.mark.parametrize("mask_kind", [0, 1])
@pytest.mark.parametrize("B,T,H,Dh,p", [(4, 200, 1, 128, 0.2), (3, 50, 2, 64, 0.0), (2, 37, 1, 32, 0.1)])
def test_attention_bwd_with_given_delta(mask_kind, B, T, H, Dh, p):
    """mask_kind | RS_ATTN_DELTA_IN: the backward takes delta = rowsum(dO * O) from the caller (the SAS out-side
    backward forms it) instead of reading O; same gradients as forming it itself (delta's fp32 summation order is
    the only difference) and still the torch reference's within the bf16 bound."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    torch.manual_seed(7 + T)
    d, dev, dt = H * Dh, "cuda", torch.bfloat16
    ids = torch.randint(1, 50, (B, T), device=dev)
    ids[0, : T // 3] = 0
    q = torch.randn(B * T, d, device=dev).to(dt)
    kv = torch.randn(B * T, 2 * d, device=dev).to(dt)
    o = torch.empty(B * T, d, device=dev, dtype=dt)
    lse = torch.empty(B * H * T, device=dev)
    sc, sb = 1.0 / math.sqrt(Dh), torch.zeros(1, dtype=torch.int64, device=dev)
    ops.attn_fwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, lse, sc, mask_kind, ids, p, 11, sb)
    do = torch.randn(B * T, d, device=dev).to(dt)
    outs = []
    for given in (False, True):
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        ws = torch.empty(B * H * T, device=dev)
        if given:   # rs_attn_row_delta, checked against torch
            ops.attn_row_delta(B, T, H, Dh, do, o, ws)
            ref = (do.float() * o.float()).view(B, T, H, Dh).sum(-1).transpose(1, 2).reshape(-1)
            assert rel(ws.cpu(), ref.cpu()) < 1e-5
        o_arg = torch.full_like(o, float("nan")) if given else o       # O must not be read
        ops.attn_bwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o_arg, do, lse, dq, dkv[:, :d], dkv[:, d:], sc, mask_kind,
                     ids, p, 11, sb, ws, delta_in=given)
        outs.append((dq.float(), dkv.float()))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.isfinite(b).all()
        assert rel(b.cpu(), a.cpu()) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,T,H,Dh", [(2, 37, 2, 64), (3, 20, 1, 50), (2, 9, 3, 128)])
def test_attn_row_delta_matches_torch(dtype, B, T, H, Dh):
    """rs_attn_row_delta (the RS_ATTN_DELTA_IN input BERT forms after its output projection's input gradient):
    vectorised (bf16, Dh % 8 == 0) and scalar forms against torch."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    torch.manual_seed(B + T + H + Dh)
    do = torch.randn(B * T, H * Dh, device="cuda").to(dtype)
    o = torch.randn(B * T, H * Dh, device="cuda").to(dtype)
    ws = torch.empty(B * H * T, device="cuda")
    ops.attn_row_delta(B, T, H, Dh, do, o, ws)
    ref = (do.double() * o.double()).view(B, T, H, Dh).sum(-1).transpose(1, 2).reshape(-1)
    assert rel(ws.cpu(), ref.cpu()) < 1e-5
