"""Dropout-ON parity of the training step (the benchmarked configuration runs SAS at p = 0.2, BERT at 0.1).

The HIP kernels draw every dropout mask from a counter-based hash of (site salt, device step seed, element
index) and regenerate it in the backward (common.h drop_mul).  The masks a training step used are materialised
here through the C ABI -- rs_dropout_rowmask over a tensor of ones, with the site's salt, the step's seed and
the site's element indexing (include/recsys_hip.h: token sites m*ld + c, attention ((b*H+h)*T+q)*Tp + k) -- and
injected into the oracle, which then replays the reference's dropout sites exactly:

  SAS  (BS/models/sas_model/sas.py)  emb :64, attn{i} (MHA attention-prob dropout) :75, ffn1_{i} / ffn2_{i} :17-19
  BERT (BS/models/bert_modules/)     emb embedding/bert.py:31, attn{i} attention/single.py:33,
                                     res1_{i} / res2_{i} utils/sublayer.py:18, ffn_{i} utils/feed_forward.py:16,
                                     blk_{i} transformer.py:32

fp32 mode is held to the fp32 bars (1e-5 forward / loss, 1e-4 gradients, norm-relative); the bf16 fused path
(the one bench.py times) to its bf16 bars.  Statistical tests check every site's keep rate and that masks
are uncorrelated across sites, steps (the optimizer advances the device seed) and data-parallel ranks (rank r
starts its seed at r << 40, train_step.py).
"""
import argparse
import math

import numpy as np
import pytest
import torch

from conftest import check_bf16_grads, rel

pytestmark = pytest.mark.gpu

FWD_TOL_F32, GRAD_TOL_F32 = 1e-5, 1e-4
FWD_TOL_BF16, GRAD_TOL_BF16 = 3e-2, 3e-2   # GRAD_TOL_BF16: BERT (SAS: conftest.check_bf16_grads)


def _ones_mask(M, N, p, salt, sb):
    """keep mask (bool, [M, N]) of a site with element index m*N + c."""
    from rbm_amd import ops
    ones = torch.ones(M, N, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ones)
    ops.dropout_rowmask(ones, p, salt, sb, None, out)
    return out > 0


def token_mask(M, N, p, salt, sb):
    return _ones_mask(M, N, p, salt, sb)


def attn_mask(B, H, T, p, salt, sb):
    Tp = T + (T & 1)
    return _ones_mask(B * H * T, Tp, p, salt, sb)[:, :T].reshape(B, H, T, T)


def sas_masks(eng, B, T, sb):
    d, H, p = eng.d, eng.H, eng.p
    M = B * T
    out = {"emb": token_mask(M, d, p, eng.salt["emb"], sb).view(B, T, d)}
    for i in range(eng.L):
        out[f"attn{i}"] = attn_mask(B, H, T, p, eng.salt[f"attn{i}"], sb)
        out[f"ffn1_{i}"] = token_mask(M, d, p, eng.salt[f"ffn1_{i}"], sb).view(B, T, d)
        out[f"ffn2_{i}"] = token_mask(M, d, p, eng.salt[f"ffn2_{i}"], sb).view(B, T, d)
    return out


def bert_masks(eng, B, T, sb):
    d, H, p, hp, Fd = eng.d, eng.H, eng.p, eng.hp, eng.F
    M = B * T
    out = {"emb": token_mask(M, d, hp, eng.salt["emb"], sb).view(B, T, d)}
    for i in range(eng.L):
        out[f"attn{i}"] = attn_mask(B, H, T, p, eng.salt[f"attn{i}"], sb)
        out[f"res1_{i}"] = token_mask(M, d, hp, eng.salt[f"res1{i}"], sb).view(B, T, d)
        out[f"ffn_{i}"] = token_mask(M, Fd, hp, eng.salt[f"ffn{i}"], sb).view(B, T, Fd)
        out[f"res2_{i}"] = token_mask(M, d, hp, eng.salt[f"res2{i}"], sb).view(B, T, d)
        out[f"blk_{i}"] = token_mask(M, d, hp, eng.salt[f"blk{i}"], sb).view(B, T, d)
    return out


def _sas_model(V, T, d, L, h, p, dtype, seed):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    torch.manual_seed(seed)
    a = argparse.Namespace(model_code="sas", num_items=V, max_len=T, device="cuda", sas_hidden_units=d,
                           sas_num_blocks=L, sas_heads=h, sas_dropout=p, l2_emb=0.0, rs_dtype=dtype)
    return model_factory(a)


def _bert_model(V, T, d, L, h, p, dtype, seed):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    a = argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cuda", bert_hidden_units=d,
                           bert_num_blocks=L, bert_num_heads=h, bert_dropout=p, bert_hidden_dropout=p,
                           bert_mask_prob=0.2, model_init_seed=seed, rs_dtype=dtype)
    return model_factory(a)


def _step_grads(tr, batch, seed):
    """One training step's loss and gradient (before the optimizer) exactly as FusedTrainStep computes it."""
    tr.engine.seed_base.fill_(seed)
    tr.flat.grad.zero_()
    tr._compute(*batch)
    torch.cuda.synchronize()
    return float(tr.loss_out[2].item()), tr.flat.grad[:tr.flat.numel].clone()


def _check(grads, g64, flat, tol, d=None, kbias=None):
    scale = max(float(np.linalg.norm(v.numpy())) for v in g64.values())
    worst = {}
    for k, ref in g64.items():
        name = k[4:] if k.startswith("sas.") else k
        g = flat.view(name, grads).cpu().numpy().astype(np.float64)
        r = ref.numpy()
        if kbias is not None and kbias(name):
            # the attention key bias: analytically zero gradient (softmax shift invariance); on scale
            assert np.linalg.norm(g[d:2 * d] if g.shape[0] == 3 * d else g) <= max(1e-5, tol) * scale, name
            if g.shape[0] != 3 * d:
                continue
            g, r = np.concatenate([g[:d], g[2 * d:]]), np.concatenate([r[:d], r[2 * d:]])
        worst[name] = rel(g, r)
    bad = {k: v for k, v in worst.items() if v >= tol}
    assert not bad, (bad, max(worst.values()))
    return worst


@pytest.mark.parametrize("dtype,V,T,d,L,h,B", [
    ("fp32", 500, 50, 64, 2, 1, 4),      # sas_mid-like, fp32 parity kernels
    ("fp32", 300, 37, 64, 2, 2, 3),      # odd T (mask row pitch), two heads
    ("bf16", 500, 50, 64, 2, 1, 4),      # fused bf16 kernels (bench path)
    ("bf16", 300, 37, 128, 2, 1, 8),     # fused, odd T.  At this small shape the kernel's distance to the
                                         # emulation depends on the dropout draw's conditioning
                                         # (tools/diag/dropout_seed_sweep.py, 16 draws: B = 3 worst 4.9 %, median
                                         # 0.9 %; B = 8 worst 3.4 %, median 1.0 %, 2 draws above 2 % -- with the
                                         # emulation itself 6-12 % from the exact math there); the test's draw
                                         # (seed 977) at B = 8: 1.1 %
    ("bf16", 3416, 200, 128, 2, 1, 8),   # cfg2 shape, small batch
    ("bf16", 3416, 200, 128, 2, 1, 128), # cfg2 exactly: the benchmarked configuration (B = 128, p = 0.2)
    ("fp32", 3416, 200, 50, 2, 1, 4),    # cfg1: the reference's default width d = 50 (generic kernels)
    ("bf16", 3416, 200, 50, 2, 1, 4),    # cfg1 in bf16 (generic kernels, unaligned rows)
    ("fp32", 400, 300, 64, 2, 1, 2),     # --max_len 300 (T > 256)
    ("bf16", 54542, 50, 128, 2, 1, 128), # cfg4 exactly (Amazon-Beauty shape): the benchmarked per-GPU step
])
def test_sas_dropout_step_matches_oracle(dtype, V, T, d, L, h, B):
    import rbm_amd.data as synth
    from oracle import sas as osas
    from rbm_amd.train_step import FusedTrainStep
    p = 0.2
    m = _sas_model(V, T, d, L, h, p, dtype, seed=V + T)
    tr = FusedTrainStep(m, lr=1e-3)
    rng = np.random.default_rng(T)
    seq, pos, neg = (torch.from_numpy(a).cuda() for a in synth.sas_batch(rng, B, T, V))
    seed = 977
    loss, grads = _step_grads(tr, (seq, pos, neg), seed)
    sb = torch.full((1,), seed, dtype=torch.int64, device="cuda")
    masks = {k: v.cpu().double() for k, v in sas_masks(tr.engine, B, T, sb).items()}
    for k, v in masks.items():          # the sites really drop ~p of their elements
        assert abs(1 - v.mean().item() - p) < 0.05, k
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    torch.set_num_threads(16)
    l64, _, _, g64 = osas.loss_and_grads(P, seq.cpu(), pos.cpu(), neg.cpu(), L, h, p=p, masks=masks)
    ftol = FWD_TOL_F32 if dtype == "fp32" else FWD_TOL_BF16
    assert abs(loss - l64.item()) < ftol * max(1.0, abs(l64.item())), (loss, l64.item())
    if dtype == "fp32":
        worst = _check(grads, g64, tr.flat, GRAD_TOL_F32, d=d, kbias=lambda n: n.endswith("in_proj_bias"))
        print(dtype, (V, T, d, B), "loss", loss, float(l64), "worst grad rel", max(worst.items(), key=lambda kv: kv[1]))
        return
    le, _, _, ge = osas.loss_and_grads(P, seq.cpu(), pos.cpu(), neg.cpu(), L, h, p=p, masks=masks,
                                       emu=osas.BF16Storage())
    assert abs(loss - le.item()) < 2e-3 * abs(le.item()), (loss, le.item())
    from rbm_amd import ops
    out = check_bf16_grads(lambda n: tr.flat.view(n, grads).cpu().numpy(), ge, g64, d,
                           kbias=lambda n: n.endswith("in_proj_bias"), strip="sas.",
                           emu_tol=2e-2 if ops.sas_block_fused_ok(d, torch.bfloat16) else 0.1)
    w_emu = max(out.items(), key=lambda kv: kv[1][0])
    w_ex = max(out.items(), key=lambda kv: kv[1][1])
    print(dtype, (V, T, d, B), "loss", loss, float(le), float(l64), "worst vs bf16 emulation", w_emu,
          "worst vs exact", w_ex)


@pytest.mark.parametrize("dtype,V,T,d,L,h,B", [
    ("fp32", 200, 30, 64, 2, 2, 3),
    ("bf16", 200, 30, 64, 2, 2, 3),
])
def test_bert_dropout_step_matches_oracle(dtype, V, T, d, L, h, B):
    import rbm_amd.data as synth
    from oracle import bert as obert
    from rbm_amd.train_step import FusedTrainStep
    p = 0.1
    m = _bert_model(V, T, d, L, h, p, dtype, seed=3)
    tr = FusedTrainStep(m, lr=1e-3)
    rng = np.random.default_rng(4)
    tok, lab = (torch.from_numpy(a).cuda() for a in synth.bert_batch(rng, B, T, V, mask_prob=0.3))
    seed = 4242
    loss, grads = _step_grads(tr, (tok, lab), seed)
    sb = torch.full((1,), seed, dtype=torch.int64, device="cuda")
    masks = {k: v.cpu().double() for k, v in bert_masks(tr.engine, B, T, sb).items()}
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    l64, _, g64 = obert.loss_and_grads(P, tok.cpu(), lab.cpu(), L, h, p=p, hp=p, masks=masks)
    ftol, gtol = (FWD_TOL_F32, GRAD_TOL_F32) if dtype == "fp32" else (FWD_TOL_BF16, GRAD_TOL_BF16)
    assert abs(loss - l64.item()) < ftol * max(1.0, abs(l64.item())), (loss, l64.item())
    worst = _check(grads, g64, tr.flat, gtol, d=d, kbias=lambda n: "linear_layers.1.bias" in n)
    print(dtype, "BERT loss", loss, float(l64), "worst grad rel", max(worst.items(), key=lambda kv: kv[1]))


def _corr(a, b):
    a = a.double().flatten() - a.double().mean()
    b = b.double().flatten() - b.double().mean()
    return float((a * b).sum() / math.sqrt(float((a * a).sum() * (b * b).sum())))


def test_dropout_masks_statistics():
    """Keep rate 1-p within 4 sigma at every SAS site; masks uncorrelated (|r| < 4/sqrt(n)) across sites, across
    consecutive steps (seed + 1, what the optimizer kernel advances) and across data-parallel ranks
    (seed + (1 << 40))."""
    m = _sas_model(3416, 200, 128, 2, 1, 0.2, "bf16", seed=1)
    eng = m.sas.engine()
    B, T, p = 16, 200, 0.2
    sb0 = torch.full((1,), 5, dtype=torch.int64, device="cuda")
    sb_next = torch.full((1,), 6, dtype=torch.int64, device="cuda")
    sb_rank = torch.full((1,), 5 + (1 << 40), dtype=torch.int64, device="cuda")
    a = sas_masks(eng, B, T, sb0)
    nxt = sas_masks(eng, B, T, sb_next)
    rk = sas_masks(eng, B, T, sb_rank)
    for k, v in a.items():
        n = v.numel()
        keep = v.double().mean().item()
        assert abs(keep - (1 - p)) < 4 * math.sqrt(p * (1 - p) / n), (k, keep)
        lim = 4 / math.sqrt(n)
        assert abs(_corr(v, nxt[k])) < lim, (k, "step", _corr(v, nxt[k]))
        assert abs(_corr(v, rk[k])) < lim, (k, "rank", _corr(v, rk[k]))
    tok = [k for k in a if not k.startswith("attn")]
    for i, k1 in enumerate(tok):
        for k2 in tok[i + 1:]:
            r = _corr(a[k1], a[k2])
            assert abs(r) < 4 / math.sqrt(a[k1].numel()), (k1, k2, r)
    r = _corr(a["attn0"], a["attn1"])
    assert abs(r) < 4 / math.sqrt(a["attn0"].numel()), r


def test_dropout_seed_advances_per_step_and_differs_per_rank():
    """FusedTrainStep: the optimizer kernel advances the device seed by one per step (so every step draws new
    masks, also inside replayed graphs), and a data-parallel rank r starts at r << 40."""
    import rbm_amd.data as synth
    from rbm_amd.train_step import FusedTrainStep
    m = _sas_model(500, 50, 64, 2, 1, 0.2, "bf16", seed=2)
    tr = FusedTrainStep(m, lr=1e-3)
    rng = np.random.default_rng(0)
    b = tuple(torch.from_numpy(x).cuda() for x in synth.sas_batch(rng, 4, 50, 500))
    s0 = int(tr.engine.seed_base.item())
    tr.step(*b)
    tr.step(*b)
    assert int(tr.engine.seed_base.item()) == s0 + 2
    tr.capture(*b, warmup=1)
    s1 = int(tr.engine.seed_base.item())
    tr.replay(*b)
    tr.replay(*b)
    assert int(tr.engine.seed_base.item()) == s1 + 2


@pytest.mark.parametrize("dist", [1, 2, 3, 37, 1000])
def test_dropout_masks_of_nearby_seeds_are_not_shifted_copies(dist):
    """Two sites (or steps) whose 32-bit seeds differ by a small XOR distance d: with the seed entering the pair hash
    only by XOR, mask_B(pair j) was exactly mask_A(pair j ^ d) -- a permuted copy.  The seed-dependent first
    multiplier (common.h pair_hash) makes them unrelated: the d-aligned masks correlate at the independent rate."""
    from rbm_amd import ops
    M, N, p = 512, 512, 0.2
    x = torch.ones(M, N, device="cuda")
    salt = 0x5A5A_1234_0000_0000
    ma, mb = torch.empty_like(x), torch.empty_like(x)
    ops.dropout_rowmask(x, p, salt, None, None, ma)
    ops.dropout_rowmask(x, p, salt ^ dist, None, None, mb)
    a, b = (t.ne(0).flatten() for t in (ma, mb))
    idx = torch.arange(a.numel(), device="cuda")
    a_aligned = a[((idx >> 1) ^ dist) << 1 | (idx & 1)]
    lim = 4 / math.sqrt(a.numel())
    assert abs(_corr(b, a_aligned)) < lim, _corr(b, a_aligned)
    assert abs(_corr(a, b)) < lim
    assert abs(a.double().mean().item() - (1 - p)) < 4 * math.sqrt(p * (1 - p) / a.numel())
