#!/usr/bin/env python
"""Per-op micro-benchmark of the C-ABI kernels at a config's shapes (GPU only).

    python tools/kbench.py [--config cfg2] [--dtype bf16] [--reps 50]

Each op is launched `reps` times back to back on one stream and timed with HIP
events on that stream; prints avg microseconds and the algorithmic HBM rate.
"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import rbm_amd  # noqa: E402,F401
from rbm_amd import ops  # noqa: E402

SHAPES = {"cfg2": dict(B=128, T=200, d=128, V=3416, H=1, ff=128),
          "cfg3": dict(B=64, T=200, d=256, V=26744, H=2, ff=1024),
          "cfg4": dict(B=128, T=50, d=128, V=54542, H=1, ff=128),
          "cfg5": dict(B=64, T=200, d=256, V=1000000, H=2, ff=1024)}


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--adam-params", type=int, default=662400, help="parameter count of the adam_step entry")
    ap.add_argument("--drop", type=float, default=0.2, help="dropout rate of the dropout-carrying ops")
    ap.add_argument("--only", default="", help="time only the ops whose name contains one of these |-separated strings")
    a = ap.parse_args()
    c = SHAPES[a.config]
    B, T, d, V, H, ff = c["B"], c["T"], c["d"], c["V"], c["H"], c["ff"]
    M = B * T
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    es = 2 if dt == torch.bfloat16 else 4
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def rn(*shape, dtype=dt):
        return torch.randn(*shape, device=dev, generator=g).to(dtype)

    ids = torch.randint(1, V + 1, (B, T), device=dev, generator=g)
    ids[:, :40] = 0
    pos = torch.randint(1, V + 1, (B, T), device=dev, generator=g)
    neg = torch.randint(1, V + 1, (B, T), device=dev, generator=g)
    x, y, z = rn(M, d), rn(M, d), rn(M, d)
    W, Wff, bias, bff = rn(d, d), rn(ff, d), torch.randn(d, device=dev), torch.randn(ff, device=dev)
    yff = rn(M, ff)
    sb = torch.zeros(1, dtype=torch.int64, device=dev)
    rows = []

    def run(name, fn, nbytes, flops=0.0):
        if a.only and not any(o in name for o in a.only.split("|")):
            return
        us = timeit(fn, a.reps)
        rows.append((name, us, nbytes / (us * 1e-6) / 1e9, flops / (us * 1e-6) / 1e12))

    mb = M * d * es
    run("linear_fwd d->d +bias",lambda: ops.linear_fwd(x, W, y, bias=bias), 2 * mb, 2 * M * d * d)
    run("linear_fwd d->ff +bias+relu+drop",lambda: ops.linear_fwd(
        x, Wff, yff, bias=bff, act=ops.ACT_RELU, drop_p=0.2, drop_seed=7, seed_base=sb, drop_ld=ff),
        mb + M * ff * es, 2 * M * d * ff)
    run("linear_fwd d->d +bias+drop+resid+rowmask",lambda: ops.linear_fwd(
        x, W, y, bias=bias, drop_p=0.2, drop_seed=7, seed_base=sb, drop_ld=d, resid=z, rowmask_ids=ids),
        3 * mb, 2 * M * d * d)
    run("linear_dgrad d<-d",lambda: ops.linear_dgrad(y, W, z), 2 * mb, 2 * M * d * d)
    dW = torch.zeros(d, d, device=dev)
    db = torch.zeros(d, device=dev)
    for sk in (None, 16, 32, 64, 128):
        s = sk or ops.split_for(M, d, d)
        slab = torch.empty(s * (d * d + d), device=dev)
        run(f"linear_wgrad+bias split={s}",lambda: ops.linear_wgrad(y, x, dW, slab, db=db, split_k=s), 2 * mb, 2 * M * d * d)
    gam, bet = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    mu, ri = torch.empty(M, device=dev), torch.empty(M, device=dev)
    run("layernorm_fwd",lambda: ops.layernorm_fwd(x, gam, bet, 1e-8, y, mu, ri, 0), 2 * mb)
    ws = torch.empty(2 * 512 * d, device=dev)
    dg, dbt = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
    run("layernorm_bwd",lambda: ops.layernorm_bwd(x, y, gam, mu, ri, 1e-8, z, dg, dbt, ws, 0),
        3 * mb)
    wsc = torch.empty(64 * d, device=dev)
    run("colsum",lambda: ops.colsum(y, db, wsc), mb)
    table = rn(V + 1, d)
    pe = rn(T, d)
    run("embed_fwd",lambda: ops.embed_fwd(0, ids, T, table, pe, math.sqrt(d), 0.2, 5, sb, x), 2 * mb)
    dtab = torch.zeros(V + 1, d, device=dev)
    dpos = torch.zeros(T, d, device=dev)
    run("embed_bwd (table atomics + pos)",lambda: ops.embed_bwd(0, ids, T, y, math.sqrt(d), 0.2, 5, sb, dtab,
                                                                      dpos), mb + M * d * 4)
    run("embed_bwd pos only",lambda: ops.embed_bwd(0, ids, T, y, math.sqrt(d), 0.2, 5, sb, None, dpos), mb)
    pl, nl = torch.empty(M, device=dev), torch.empty(M, device=dev)
    run("sampled_logits_fwd",lambda: ops.sampled_logits_fwd(x, table, pos, neg, pl, nl), 3 * mb)
    run("sampled_logits_bwd",lambda: ops.sampled_logits_bwd(x, table, pos, neg, pl, nl, y, dtab),
        4 * mb + 2 * M * d * 4)
    Dh = d // H
    q, kv, o = rn(M, d), rn(M, 2 * d), rn(M, d)
    lse = torch.empty(B * H * T, device=dev)
    aflops = 2.0 * T * (T + 1) * Dh * B * H
    run("attn_fwd causal drop",lambda: ops.attn_fwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, lse,
                                                            1 / math.sqrt(Dh), 0, ids, a.drop, 9, sb),
        4 * mb, aflops)
    dq, dkv = rn(M, d), rn(M, 2 * d)
    wat = torch.empty(B * H * T, device=dev)
    # the step's variant (sas.py / bert.py): delta = rowsum(dO * O) handed in, O not read -- 7 activation tensors
    ops.attn_row_delta(B, T, H, Dh, y, o, wat)
    run("attn_bwd causal drop",lambda: ops.attn_bwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, y, lse, dq,
                                                            dkv[:, :d], dkv[:, d:], 1 / math.sqrt(Dh), 0, ids, a.drop,
                                                            9, sb, wat, delta_in=True), 7 * mb, 2.0 * aflops)
    if a.config in ("cfg3", "cfg5"):
        # BERT block GEMMs with their fused epilogues (bert.py encode / encode_backward)
        hg, apre, gg = rn(M, d), rn(M, ff), rn(M, ff)
        Wqkv, bqkv, qkv = rn(3 * d, d), torch.randn(3 * d, device=dev), rn(M, 3 * d)
        W1b, W2b = rn(ff, d), rn(d, ff)
        run("bert qkv fwd +bias", lambda: ops.linear_fwd(hg, Wqkv, qkv, bias=bqkv), 4 * mb, 6 * M * d * d)
        run("bert out fwd +bias+drop+resid", lambda: ops.linear_fwd(
            x, W, y, bias=bias, drop_p=0.1, drop_seed=7, seed_base=sb, drop_ld=d, resid=z), 3 * mb, 2 * M * d * d)
        run("bert ffn1 fwd +bias+gelu+drop+aux", lambda: ops.linear_fwd(
            hg, W1b, gg, bias=bff, act=ops.ACT_GELU, aux_out=apre, drop_p=0.1, drop_seed=7, seed_base=sb,
            drop_ld=ff), mb + 2 * M * ff * es, 2 * M * d * ff)
        run("bert ffn2 fwd +bias+drop+resid+post", lambda: ops.linear_fwd(
            gg, W2b, y, bias=bias, drop_p=0.1, drop_seed=7, seed_base=sb, drop_ld=d, resid=z, post_drop_p=0.1,
            post_drop_seed=8), M * ff * es + 2 * mb, 2 * M * d * ff)
        run("bert ffn2 dgrad +gelu'+drop", lambda: ops.linear_dgrad(
            y, W2b, gg, act=ops.ACT_GELU_BWD, aux=apre, drop_p=0.1, drop_seed=7, seed_base=sb, drop_ld=ff),
            mb + 2 * M * ff * es, 2 * M * d * ff)
        run("bert ffn1 dgrad", lambda: ops.linear_dgrad(gg, W1b, z), M * ff * es + mb, 2 * M * d * ff)
        run("bert qkv dgrad", lambda: ops.linear_dgrad(qkv, Wqkv, z), 4 * mb, 6 * M * d * d)
        from rbm_amd.models.bert_model.bert import BERTEngine
        bshapes = [(d, ff), (ff, d), (d, d), (3 * d, d)] * 4
        bprobs = [(rn(M, n), rn(M, k), torch.zeros(n, k, device=dev), torch.zeros(n, device=dev)) for n, k in bshapes]
        brows = BERTEngine._wgrad_rows(M, bshapes)
        bslab = torch.empty(ops.wgrad_grouped_slab_numel(bshapes, M, brows), device=dev)
        run("bert wgrad_grouped 16 problems", lambda: ops.wgrad_grouped(bprobs, M, brows, bslab),
            sum(M * (n + k) * es for n, k in bshapes), sum(2 * M * n * k for n, k in bshapes))
        V1 = V + 1
        R = 1792
        V1p = -(-V1 // 64) * 64
        h = rn(R, d)
        Wo = (0.05 * torch.randn(V1, d, device=dev, generator=g)).to(dt)
        bo = torch.zeros(V1, device=dev)
        lg = torch.empty(R, V1p, device=dev)[:, :V1]
        run("vocab logits fwd (fp32 out)",lambda: ops.linear_fwd(h, Wo, lg, bias=bo),
            R * V1 * 4 + V1 * d * es, 2 * R * V1 * d)
        dl = torch.randn(R, V1p, device=dev, generator=g).to(dt)[:, :V1]
        dh = rn(R, d)
        run("vocab dgrad",lambda: ops.linear_dgrad(dl, Wo, dh), R * V1 * es + V1 * d * es,
            2 * R * V1 * d)
        sk = int(max(1, min(64, -(-V1 // 2048))))
        slab_dh = torch.empty(sk * R * d, device=dev)
        run(f"vocab dh split-K={sk}", lambda: ops.gemm(dl, Wo, slab_dh, R, d, V1, False, True, ops.epilogue(),
                                                        split_k=sk, slab=slab_dh), R * V1 * es + V1 * d * es,
            2 * R * V1 * d)
        if ops.vocab_head_supported(d):
            # the bench's cfg5 roofline kernel at its shape (R = the batches' mean labelled count, bench.py roofline)
            Rh = 1574 if V1 > 500000 else R
            hh = rn(Rh, d)
            labh = torch.randint(1, V1, (Rh,), device=dev, generator=g)
            wsh = torch.empty(ops.vocab_ce_ws_numel(Rh, V1), device=dev)
            outh = torch.empty(4, device=dev)
            run("vocab_head_fwd (E-stationary, online-softmax partials)",
                lambda: ops.vocab_head_fwd(hh, Wo, bo, labh, wsh, outh),
                (V1 * d + Rh * d) * es + Rh * -(-V1 // 128) * 8, 2 * Rh * V1 * d)
        dWo = torch.zeros(V1, d, device=dev)
        slab_o = torch.empty(ops.wgrad_slab_numel(R, V1, d), device=dev)
        run("vocab wgrad+bias",lambda: ops.linear_wgrad(dl, h, dWo, slab_o, db=bo),
            R * V1 * es + V1 * d * 4, 2 * R * V1 * d)
    if d in (64, 128) and dt == torch.bfloat16:
        # fused SAS row-block kernels, grouped weight gradients, item-table gradient, fused head
        Win, bin_ = rn(3 * d, d), torch.randn(3 * d, device=dev)
        Q, qq, kvb, oo = rn(M, d), rn(M, d), rn(M, 2 * d), rn(M, d)
        x1, zz, h1, xn = rn(M, d), rn(M, d), rn(M, d), rn(M, d)
        m1_, r1_ = torch.zeros(M, device=dev), torch.ones(M, device=dev)
        run("fused block_in", lambda: ops.sas_block_in(x, gam, bet, 1e-8, Q, m1_, r1_, Win[:d], bin_[:d], qq, Win[d:],
                                                        bin_[d:], kvb), 6 * mb)
        run("fused block_out", lambda: ops.sas_block_out(oo, Q, W, bias, x1, gam, bet, 1e-8, zz, m1_, r1_, W, bias, h1,
                                                          W, bias, xn, ids, a.drop, 3, 4, sb), 6 * mb)
        WT, WinT = rn(d, d), rn(d, 3 * d)
        dy2, da1, dx1, do_ = rn(M, d), rn(M, d), rn(M, d), rn(M, d)
        part = torch.empty(2 * d * max(-(-M // 64), ops.sas_block_parts(M)), device=dev)
        run("fused block_out_bwd", lambda: ops.sas_block_out_bwd(y, ids, h1, x1, m1_, r1_, gam, WT, WT, WT, dy2, da1,
                                                                  dx1, do_, part, a.drop, 3, 4, sb), 8 * mb)
        dqkv = rn(M, 2 * d)
        run("fused block_in_bwd", lambda: ops.sas_block_in_bwd(qq, dqkv, dx1, x, m1_, r1_, gam, WinT, z, part),
            6 * mb)
        probs = []
        for _ in range(2):
            probs += [(dy2, h1, torch.zeros(d, d, device=dev), torch.zeros(d, device=dev)),
                      (da1, zz, torch.zeros(d, d, device=dev), torch.zeros(d, device=dev)),
                      (dx1, oo, torch.zeros(d, d, device=dev), torch.zeros(d, device=dev)),
                      (qq, Q, torch.zeros(d, d, device=dev), torch.zeros(d, device=dev)),
                      (dqkv, x, torch.zeros(2 * d, d, device=dev), torch.zeros(2 * d, device=dev))]
        for rows_ in (640, 1280, 2560):
            wsl = torch.empty(ops.wgrad_grouped_slab_numel([(d, d)] * 8 + [(2 * d, d)] * 2, M, rows_), device=dev)
            run(f"wgrad_grouped 10 problems rows={rows_}", lambda: ops.wgrad_grouped(probs, M, rows_, wsl),
                24 * mb, 2 * M * d * d * 12)
        zw = 1.0 / torch.arange(1, V + 1, dtype=torch.float64) ** 1.1
        kk = [torch.multinomial(zw, M, replacement=True, generator=torch.Generator().manual_seed(5 + i)).add(1)
              .view(B, T).to(dev) for i in range(3)]
        iws = torch.empty(ops.item_index_ws_bytes(3, M, V + 1, d), dtype=torch.uint8, device=dev)
        run("item_index_build (zipf)", lambda: ops.item_index_build(kk, V + 1, d, iws), 3 * M * 8)
        ops.item_index_build(kk, V + 1, d, iws)
        dtab2 = torch.zeros(V + 1, d, device=dev)
        run("item_grad (zipf)", lambda: ops.item_grad(iws, 3, M, y, math.sqrt(d), 0.2, 5, sb, x, pl, nl, dtab2),
            3 * mb)
        hp = torch.empty(3 * (-(-M // 64)), device=dev)
        run("head_fwd", lambda: ops.sas_head_fwd(x, gam, bet, 1e-8, y, mu, ri, table, pos, neg, pl, nl, hp), 4 * mb)
        lout = torch.empty(4, device=dev)
        dpl_, dnl_ = torch.empty(M, device=dev), torch.empty(M, device=dev)
        run("head_bwd", lambda: ops.sas_head_bwd(hp, None, lout, pl, nl, None, None, dpl_, dnl_, pos, neg, table, x,
                                                 gam, mu, ri, z, part), 4 * mb)
    n = a.adam_params
    p, gg, m1, v1 = (torch.randn(n, device=dev) for _ in range(4))
    v1.abs_()
    pbf = torch.empty(n, dtype=torch.bfloat16, device=dev)
    st = torch.tensor([1.0, 0.001, 1.0, 1.0], dtype=torch.float64, device=dev)
    hy = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0], dtype=torch.float64, device=dev)
    run(f"adam_step ({n} params)",lambda: ops.adam_step(p, gg, m1, v1, pbf, st, hy, zero_grad=True), n * 4 * 8 + n * 2)
    st144 = torch.zeros(144, dtype=torch.float64, device=dev)
    run(f"adam_prepare_step ({n} params)", lambda: ops.adam_prepare_step(p, gg, m1, v1, pbf, st144, hy, zero_grad=True),
        n * 4 * 8 + n * 2)
    if a.config in ("cfg2", "cfg4"):
        # the SAS step's form: + the transposed bf16 block weights (rs_transpose_bf16's descriptors, 2 blocks x
        # in_proj / out_proj / conv1 / conv2 at the flat buffer's offsets)
        dd, L = c["d"], 2
        desc, off = [], n - L * 6 * dd * dd
        for i in range(L):
            for rows_, o in ((3 * dd, 0), (dd, 3 * dd * dd), (dd, 4 * dd * dd), (dd, 5 * dd * dd)):
                desc.append([rows_, dd, off + i * 6 * dd * dd + o, dd, i * 6 * dd * dd + o, rows_])
        td = torch.tensor(desc, dtype=torch.int64, device=dev)
        wT = torch.empty(L * 6 * dd * dd, dtype=torch.bfloat16, device=dev)
        run(f"adam_prepare_step +transposes ({n} params)", lambda: ops.adam_prepare_step(
            p, gg, m1, v1, pbf, st144, hy, zero_grad=True, transposed=(td, desc, wT)), n * 4 * 8 + n * 2)
    print(f"{'op':45s} {'us':>9s} {'GB/s':>9s} {'TFLOP/s':>8s}")
    for name, us, gbs, tf in rows:
        print(f"{name:45s} {us:9.2f} {gbs:9.1f} {tf:8.2f}")


if __name__ == "__main__":
    main()
