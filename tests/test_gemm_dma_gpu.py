"""LDS-DMA pipelined bf16 GEMM (csrc/gemm_dma.h) for the BERT block products: the same call with RS_GEMM_DMA=1
(the DMA form, both row tiles) and RS_GEMM_DMA=0 (the register-staged kernel) gives the SAME bits -- every output
element takes the same sequence of 32-deep MFMA steps in k order and the same epilogue -- at the cfg3 shapes
(BS/models/bert_modules/attention/multi_head.py:24-40 QKV / output projection, utils/feed_forward.py:15-16 FFN), in
both orientations, with every epilogue class the BERT layer uses, ragged M and a device row count; and the plain
product matches torch float64 on the same bf16 operands."""
import os

import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu


def _bf(shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, device="cuda", generator=g) * scale).bfloat16()


def _run(fn, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _three_ways(fn):
    """(register-staged, DMA 128-row tiles, DMA 64-row tiles) results of fn()."""
    ref = _run(fn, {"RS_GEMM_DMA": "0"})
    d128 = _run(fn, {"RS_GEMM_DMA": "1", "RS_GEMM_DMA_BM": "128"})
    d64 = _run(fn, {"RS_GEMM_DMA": "1", "RS_GEMM_DMA_BM": "64"})
    return ref, d128, d64


def _same(outs):
    ref = outs[0]
    for o in outs[1:]:
        if isinstance(ref, tuple):
            for x, y in zip(ref, o):
                assert torch.equal(x, y)
        else:
            assert torch.equal(ref, o)


CASES = [  # M, N (output width), K
    (12800, 768, 256),    # QKV forward
    (12800, 256, 256),    # output projection forward / its input gradient
    (12800, 1024, 256),   # FFN1 forward / FFN2 input gradient
    (12800, 256, 1024),   # FFN2 forward / FFN1 input gradient
    (12800, 256, 768),    # QKV input gradient
    (1000, 384, 96),      # ragged rows, 3 k stages
    (70, 128, 32),        # one partial row tile, one stage
]


@pytest.mark.parametrize("M,N,K", CASES)
def test_forward_plain_bitwise_and_float64(M, N, K):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    x, W = _bf((M, K), 1.0, 1), _bf((N, K), 0.05, 2)

    def f():
        y = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        ops.linear_fwd(x, W, y)
        torch.cuda.synchronize()
        return y
    outs = _three_ways(f)
    _same(outs)
    ref = x.double() @ W.double().t()
    assert rel(outs[1].double().cpu().numpy(), ref.cpu().numpy()) < 5e-3   # bf16 output rounding


@pytest.mark.parametrize("M,N,K", CASES)
def test_dgrad_plain_bitwise_and_float64(M, N, K):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    dy, W = _bf((M, K), 1.0, 3), _bf((K, N), 0.05, 4)    # dX[M,N] = dY[M,K] . W[K,N]

    def f():
        dx = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        ops.linear_dgrad(dy, W, dx)
        torch.cuda.synchronize()
        return dx
    outs = _three_ways(f)
    _same(outs)
    ref = dy.double() @ W.double()
    assert rel(outs[1].double().cpu().numpy(), ref.cpu().numpy()) < 5e-3


def test_bert_layer_epilogues_bitwise():
    """The fused epilogues of the BERT layer (tools/diag/gemm_epi.py's set): bias + GELU + dropout + saved
    pre-activation (FFN1), bias + dropout + residual + post-dropout (FFN2), GELU' + dropout (FFN2 input gradient),
    bias + dropout + residual (output projection), bias (QKV), accumulate, fp32 output; a device row count."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    B, T, d, ff = 16, 200, 256, 1024
    M = B * T
    sb = torch.tensor([5], dtype=torch.int64, device="cuda")
    x, W1, W2, Wq, Wo = _bf((M, d), 1, 5), _bf((ff, d), .05, 6), _bf((d, ff), .05, 7), _bf((3 * d, d), .05, 8), \
        _bf((d, d), .05, 9)
    b1, b2, bq = (torch.randn(n, device="cuda") for n in (ff, d, 3 * d))
    z, dy2 = _bf((M, d), 1, 10), _bf((M, d), 1, 11)
    dk = dict(drop_p=0.1, drop_seed=7, seed_base=sb)
    rows = torch.tensor([M - 77], dtype=torch.int32, device="cuda")

    def f():
        h = torch.zeros(M, ff, device="cuda", dtype=torch.bfloat16)
        pre = torch.zeros_like(h)
        ops.linear_fwd(x, W1, h, bias=b1, act=ops.ACT_GELU, aux_out=pre, drop_ld=ff, **dk)
        y = torch.zeros(M, d, device="cuda", dtype=torch.bfloat16)
        ops.linear_fwd(h, W2, y, bias=b2, drop_ld=d, resid=z, post_drop_p=0.1, post_drop_seed=8, **dk)
        dh = torch.zeros(M, ff, device="cuda", dtype=torch.bfloat16)
        ops.linear_dgrad(dy2, W2, dh, act=ops.ACT_GELU_BWD, aux=pre, drop_ld=ff, **dk)
        o = torch.zeros(M, d, device="cuda", dtype=torch.bfloat16)
        ops.linear_fwd(x, Wo, o, bias=b2, drop_ld=d, resid=z, **dk)
        q = torch.zeros(M, 3 * d, device="cuda", dtype=torch.bfloat16)
        ops.linear_fwd(x, Wq, q, bias=bq)
        acc = z.clone()
        ops.linear_fwd(x, Wo, acc, accumulate=True)
        f32 = torch.zeros(M, d, device="cuda", dtype=torch.float32)
        ops.linear_fwd(x, Wo, f32, bias=b2)
        rd = torch.full((M, d), 3.0, device="cuda", dtype=torch.bfloat16)
        ops.linear_fwd(x, Wo, rd, rows_dev=rows)
        torch.cuda.synchronize()
        return h, pre, y, dh, o, q, acc, f32, rd
    outs = _three_ways(f)
    _same(outs)
    rd = outs[1][-1]
    assert torch.all(rd[M - 77:] == 3.0)          # rows past the device count untouched


@pytest.mark.parametrize("R,V,count,accumulate", [(2600, 26745, 2531, False), (512, 1000, None, True),
                                                  (77, 300, 40, False)])
def test_wgrad_direct_bitwise(R, V, count, accumulate):
    """rs_linear_wgrad's one-split path (the BERT vocabulary head's dE = dlogits^T h + the bias column sums below the
    64k classes, BS/models/bert.py:10,16) on the DMA weight-gradient kernel equals the register-staged kernel bit for
    bit: ragged vocabulary tiles, a device row count with a partial last stage, accumulate on and off."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    Vp = V + (-V) % 64
    dl = _bf((R, Vp), 1e-2, 21)[:, :V]
    h = _bf((R, 256), 1.0, 22)
    rows = None if count is None else torch.tensor([count], dtype=torch.int32, device="cuda")
    slab = torch.empty(1, device="cuda")

    def f():
        dE = torch.full((V, 256), 0.5, device="cuda")
        db = torch.full((V,), 0.25, device="cuda")
        ops.linear_wgrad(dl, h, dE, slab, db=db, split_k=1, accumulate=accumulate, rows_dev=rows)
        torch.cuda.synchronize()
        return dE, db
    outs = _three_ways(f)
    _same(outs)
    k = R if count is None else count
    ref = dl[:k].double().t() @ h[:k].double() + (0.5 if accumulate else 0.0)
    assert rel(outs[1][0].double().cpu().numpy(), ref.cpu().numpy()) < 2e-6


@pytest.mark.parametrize("M", [12800, 1000, 37])
@pytest.mark.parametrize("kind", ["qkv", "ffn1", "ffn1_eval"])
def test_gemm_ln_equals_layernorm_then_gemm(M, kind):
    """rs_gemm_ln (the BERT LayerNorm formed in the DMA GEMM's prologue) = rs_layernorm_fwd (variant 1) + rs_gemm, bit
    for bit: the product, the LayerNorm output h and the row statistics -- QKV (bias) and FFN1 (bias + GELU + dropout
    + pre-activation; eval: no dropout) at the cfg3 shapes, ragged M (a partial last row tile)."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    d = 256
    N = 768 if kind == "qkv" else 1024
    x = _bf((M, d), 2.0, seed=11) + 0.3
    W = _bf((N, d), 0.05, seed=12)
    g = torch.Generator(device="cuda").manual_seed(13)
    gamma = 1.0 + 0.1 * torch.randn(d, device="cuda", generator=g)
    beta = 0.1 * torch.randn(d, device="cuda", generator=g)
    bias = 0.1 * torch.randn(N, device="cuda", generator=g)
    sb = torch.tensor([12345], dtype=torch.int64, device="cuda")
    kw = dict(bias=bias)
    if kind != "qkv":
        kw.update(act=ops.ACT_GELU, drop_p=0.1 if kind == "ffn1" else 0.0, drop_seed=77, seed_base=sb, drop_ld=N)
    outs = []
    for fused in (True, False):
        y = torch.full((M, N), float("nan"), device="cuda").bfloat16()
        h = torch.full((M, d), float("nan"), device="cuda").bfloat16()
        mu, r = torch.full((M,), float("nan"), device="cuda"), torch.full((M,), float("nan"), device="cuda")
        aux = torch.full((M, N), float("nan"), device="cuda").bfloat16() if kind != "qkv" else None
        kk = dict(kw, aux_out=aux) if aux is not None else kw
        if fused:
            assert ops.linear_fwd_ln(x, gamma, beta, 1e-6, W, y, h, mu, r, **kk)
        else:
            ops.layernorm_fwd(x, gamma, beta, 1e-6, h, mu, r, 1)
            ops.linear_fwd(h, W, y, **kk)
        torch.cuda.synchronize()
        outs.append((y, h, mu, r) + ((aux,) if aux is not None else ()))
    for name, a, b in zip(("y", "h", "mean", "rinv", "aux"), *outs):
        assert torch.equal(a, b), (name, float((a.float() - b.float()).abs().max()), int((a != b).sum()))
