"""Item-table gradient by inverted index (itemgrad.hip) vs the atomic scatter kernels and torch.

Sources: the embedding lookup's rows (scale * dropout * dx) and the tied sampled-logit rows
(dpl * f, dnl * f), keyed by Zipf-distributed item ids so hot ids span many 64-entry chunks.
"""
import numpy as np
import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu


def _inputs(M, V1, d, seed):
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, V1) ** 1.1
    w /= w.sum()

    def keys():
        k = rng.choice(np.arange(1, V1), size=M, p=w)
        k[rng.random(M) < 0.15] = 0                      # padding rows
        return torch.from_numpy(k).cuda()
    ids, pos, neg = keys(), keys(), keys()
    g = torch.Generator(device="cuda").manual_seed(seed)
    dx = torch.randn(M, d, device="cuda", generator=g).bfloat16()
    f = torch.randn(M, d, device="cuda", generator=g).bfloat16()
    dpl = torch.randn(M, device="cuda", generator=g)
    dnl = torch.randn(M, device="cuda", generator=g)
    return ids, pos, neg, dx, f, dpl, dnl


def _radix_path(M, V1):
    """True when itemgrad.hip's layout() takes the hand-written radix sort instead of the counting sort: tables
    over the LDS histogram's 32k rows, (512-entry sort blocks) x (table rows) > 2^26 histogram ints, or keys wider
    than 22 bits."""
    nb = -(-3 * M // 512)
    return V1 > 32768 or nb * V1 > (1 << 26) or (V1 - 1).bit_length() > 22


# tables over 32k rows (40,000; 54,543; 800,000) -> the radix sort (one workgroup in LDS for 9,000 / 19,200 entries,
# multi-workgroup for 90,000); the rest -> the counting sort
@pytest.mark.parametrize("M,V1,d,p", [(25600, 3417, 128, 0.2), (5000, 300, 64, 0.0), (777, 50, 256, 0.1),
                                      (64, 5, 128, 0.0), (3000, 40000, 64, 0.0), (6400, 54543, 128, 0.2),
                                      (30000, 800000, 64, 0.0)])
def test_item_grad_matches_atomic_scatter(M, V1, d, p):
    assert _radix_path(M, V1) == (V1 > 32768)
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    ids, pos, neg, dx, f, dpl, dnl = _inputs(M, V1, d, seed=M + d)
    T = 200 if M % 200 == 0 else M
    seed_base = torch.full((1,), 7, dtype=torch.int64, device="cuda")
    salt, scale = 12345, float(np.sqrt(d))
    base = torch.randn(V1, d, device="cuda")
    ours = base.clone()
    ws = torch.empty(ops.item_index_ws_bytes(3, M, V1, d), dtype=torch.uint8, device="cuda")
    ops.item_index_build([ids, pos, neg], V1, d, ws)
    ops.item_grad(ws, 3, M, dx, scale, p, salt, seed_base, f, dpl, dnl, ours)
    ref = base.clone()
    ops.embed_bwd(0, ids, T, dx, scale, p, salt, seed_base, ref, None)
    E = torch.randn(V1, d, device="cuda").bfloat16()
    df = torch.empty(M, d, device="cuda").bfloat16()
    ops.sampled_logits_bwd(f, E, pos, neg, dpl, dnl, df, ref)
    torch.cuda.synchronize()
    assert rel(ours.cpu().numpy(), ref.cpu().numpy()) < 1e-5
    assert torch.equal(ours[0], base[0])                         # padding row untouched
    if p == 0.0:
        t = base.double().clone()
        for k, w, src in ((ids, None, dx), (pos, dpl, f), (neg, dnl, f)):
            rows = src.double() * (scale if w is None else w.double()[:, None])
            keep = k != 0
            t.index_add_(0, k[keep], rows[keep])
        assert rel(ours.cpu().numpy(), t.cpu().numpy()) < 1e-5
    # reproducible bit for bit
    again = base.clone()
    ops.item_index_build([ids, pos, neg], V1, d, ws)
    ops.item_grad(ws, 3, M, dx, scale, p, salt, seed_base, f, dpl, dnl, again)
    assert torch.equal(again, ours)


def _index_keys(nsrc, M, V1, pad, seed):
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, V1) ** 1.05
    w /= w.sum()
    ks = []
    for _ in range(nsrc):
        k = rng.choice(np.arange(1, V1), size=M, p=w)
        k[rng.random(M) < pad] = 0
        ks.append(k)
    return ks


# (nsrc, rows, table rows, padding share, expected sort path): 0 counting sort, 3 radix sort (2,048-entry tiles; up
# to 64 tiles the scatter workgroups scan the tile counts themselves, past that a scan launch: 131,072 = 64 tiles,
# 133,121 = 66).  cfg4 = 3 x 6,400 entries over 54,543 rows (~80 % padding); cfg5 = 12,800 token ids over 1,000,002
# rows (20-bit keys: three 7-bit passes).
@pytest.mark.parametrize("nsrc,M,V1,pad,path", [
    (3, 25600, 3417, 0.2, 0), (3, 6400, 54543, 0.8, 3), (3, 3000, 40000, 0.15, 3), (1, 12800, 1000002, 0.28, 3),
    (3, 30000, 800000, 0.15, 3), (1, 300000, 1000002, 0.3, 3), (3, 12272, 54543, 0.0, 3), (1, 1, 40000, 0.0, 3),
    (3, 6400, 54543, 1.0, 3), (1, 131072, 1000002, 0.0, 3), (1, 133121, 1000002, 0.0, 3)])
def test_item_index_is_the_stable_sort(nsrc, M, V1, pad, path):
    """The built index equals numpy's stable argsort of the concatenated keys bit for bit (sorted keys, entries,
    and on the counting-sort path start[v] = first position of key >= v), on every sort path incl. all-padding
    and single-entry batches."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    d = 128
    ks = _index_keys(nsrc, M, V1, pad, seed=M + V1)
    dev = [torch.from_numpy(k).cuda() for k in ks]
    ws = torch.empty(ops.item_index_ws_bytes(nsrc, M, V1, d), dtype=torch.uint8, device="cuda")
    ops.item_index_build(dev, V1, d, ws)
    sk, sv, start, got_path = ops.item_index_view(nsrc, M, V1, d, ws)
    torch.cuda.synchronize()
    assert got_path == path
    allk = np.concatenate(ks)
    order = np.argsort(allk, kind="stable")
    srt = allk[order]
    assert np.array_equal(sk.cpu().numpy().astype(np.int64), srt)
    assert np.array_equal(sv.cpu().numpy().astype(np.int64), order)
    assert (start is not None) == (path == 0)
    if start is not None:
        assert np.array_equal(start.cpu().numpy().astype(np.int64), np.searchsorted(srt, np.arange(V1 + 1), "left"))
    # a second build over the same workspace: the same bits (no state carried between builds)
    ws2 = ws.clone()
    ops.item_index_build(dev, V1, d, ws2)
    sk2, sv2, _, _ = ops.item_index_view(nsrc, M, V1, d, ws2)
    assert torch.equal(sk2, sk) and torch.equal(sv2, sv)


# the fp32 parity path (rs_item_grad_f32: chunk sums + chunk-order span sums, any width): Zipf-hot keys spanning
# many chunks, padding keys, odd widths, both index paths
@pytest.mark.parametrize("M,V1,d,p", [(25600, 3417, 128, 0.2), (25600, 3417, 50, 0.0), (777, 50, 256, 0.1),
                                      (64, 5, 96, 0.0), (6400, 54543, 128, 0.2), (5000, 300, 300, 0.0)])
def test_item_grad_f32_matches_atomic_scatter(M, V1, d, p):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    ids, pos, neg, dx, f, dpl, dnl = _inputs(M, V1, d, seed=M + d + 1)
    dx, f = dx.float(), f.float()
    T = 200 if M % 200 == 0 else M
    seed_base = torch.full((1,), 7, dtype=torch.int64, device="cuda")
    salt, scale = 12345, float(np.sqrt(d))
    base = torch.randn(V1, d, device="cuda")
    ours = base.clone()
    ws = torch.empty(ops.item_index_ws_bytes(3, M, V1, d), dtype=torch.uint8, device="cuda")
    ops.item_index_build([ids, pos, neg], V1, d, ws)
    ops.item_grad(ws, 3, M, dx, scale, p, salt, seed_base, f, dpl, dnl, ours)
    ref = base.clone()
    ops.embed_bwd(0, ids, T, dx, scale, p, salt, seed_base, ref, None)
    E = torch.randn(V1, d, device="cuda")
    df = torch.empty(M, d, device="cuda")
    ops.sampled_logits_bwd(f, E, pos, neg, dpl, dnl, df, ref)
    torch.cuda.synchronize()
    assert rel(ours.cpu().numpy(), ref.cpu().numpy()) < 1e-5   # both fp32 sums, different orders
    assert torch.equal(ours[0], base[0])                         # padding row untouched
    if p == 0.0:
        t = base.double().clone()
        for k, w, src in ((ids, None, dx), (pos, dpl, f), (neg, dnl, f)):
            rows = src.double() * (scale if w is None else w.double()[:, None])
            keep = k != 0
            t.index_add_(0, k[keep], rows[keep])
        assert rel(ours.cpu().numpy(), t.cpu().numpy()) < 1e-5
    again = base.clone()
    ops.item_index_build([ids, pos, neg], V1, d, ws)
    ops.item_grad(ws, 3, M, dx, scale, p, salt, seed_base, f, dpl, dnl, again)
    assert torch.equal(again, ours)                              # reproducible bit for bit
