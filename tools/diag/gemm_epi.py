#!/usr/bin/env python
"""Epilogue cost of the BERT block GEMMs (cfg3 shapes): the same GEMM timed with progressively
heavier fused epilogues, so the mainloop and each epilogue stage can be told apart (GPU only).

    python tools/diag/gemm_epi.py [--reps 50]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import rbm_amd  # noqa: E402,F401
from rbm_amd import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--envs", default="", help="';'-separated environment sets (',' between K=V pairs) to time "
                    "every library op under, e.g. 'RS_GEMM_PD=1;' (empty set = defaults)")
    a = ap.parse_args()
    B, T, d, ff = 64, 200, 256, 1024
    M = B * T
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rn = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    sb = torch.zeros(1, dtype=torch.int64, device=dev)
    x, W1, W2 = rn(M, d), rn(ff, d), rn(d, ff)
    b1, b2 = torch.randn(ff, device=dev), torch.randn(d, device=dev)
    h, pre, y, z = rn(M, ff), rn(M, ff), rn(M, d), rn(M, d)
    dk = dict(drop_p=0.1, drop_seed=7, seed_base=sb)
    rows = []

    envs = [e for e in a.envs.split(";")] if a.envs else [""]

    def run(name, fn, nbytes, flops):
        for es in (envs if not name.startswith("torch") else [""]):
            kv = [p.split("=", 1) for p in es.split(",") if p]
            for k, v in kv:
                os.environ[k] = v
            us = timeit(fn, a.reps)
            for k, _ in kv:
                os.environ.pop(k, None)
            tag = f" [{es or 'default'}]" if len(envs) > 1 and not name.startswith("torch") else ""
            rows.append((name + tag, us, nbytes / us / 1e3, flops / us / 1e6))

    mb, fb = M * d * 2, M * ff * 2
    f1 = 2.0 * M * d * ff
    run("ffn1 plain", lambda: ops.linear_fwd(x, W1, h), mb + fb, f1)
    run("ffn1 +bias", lambda: ops.linear_fwd(x, W1, h, bias=b1), mb + fb, f1)
    run("ffn1 +bias+gelu", lambda: ops.linear_fwd(x, W1, h, bias=b1, act=ops.ACT_GELU), mb + fb, f1)
    run("ffn1 +bias+gelu+aux", lambda: ops.linear_fwd(x, W1, h, bias=b1, act=ops.ACT_GELU, aux_out=pre),
        mb + 2 * fb, f1)
    run("ffn1 +bias+drop", lambda: ops.linear_fwd(x, W1, h, bias=b1, drop_ld=ff, **dk), mb + fb, f1)
    run("ffn1 +bias+gelu+drop+aux", lambda: ops.linear_fwd(x, W1, h, bias=b1, act=ops.ACT_GELU, aux_out=pre,
                                                           drop_ld=ff, **dk), mb + 2 * fb, f1)
    run("ffn2 plain", lambda: ops.linear_fwd(h, W2, y), fb + mb, f1)
    run("ffn2 +bias+drop+resid+post", lambda: ops.linear_fwd(h, W2, y, bias=b2, drop_ld=d, resid=z, post_drop_p=0.1,
                                                             post_drop_seed=8, **dk), fb + 3 * mb, f1)
    run("ffn2 dgrad plain", lambda: ops.linear_dgrad(y, W2, h), mb + fb, f1)
    run("ffn2 dgrad +gelu'+drop", lambda: ops.linear_dgrad(y, W2, h, act=ops.ACT_GELU_BWD, aux=pre, drop_ld=ff, **dk),
        mb + 2 * fb, f1)
    run("ffn1 dgrad plain", lambda: ops.linear_dgrad(h, W1, y), fb + mb, f1)
    # the library bar (hipBLASLt through torch) for the same plain products
    W1t, W2t = W1.t().contiguous(), W2.t().contiguous()
    run("torch.mm ffn1 (x W1^T)", lambda: torch.mm(x, W1.t(), out=h), mb + fb, f1)
    run("torch.mm ffn2 (h W2^T)", lambda: torch.mm(h, W2.t(), out=y), fb + mb, f1)
    run("torch.mm ffn2 dgrad (y W2)", lambda: torch.mm(y, W2, out=h), mb + fb, f1)
    run("torch.mm ffn1 dgrad (h W1)", lambda: torch.mm(h, W1, out=y), fb + mb, f1)
    run("torch.mm ffn1 (x W1t)", lambda: torch.mm(x, W1t, out=h), mb + fb, f1)
    Wq = rn(3 * d, d)
    qkv = rn(M, 3 * d)
    run("qkv plain", lambda: ops.linear_fwd(x, Wq, qkv), mb * 4, 6.0 * M * d * d)
    run("torch.mm qkv", lambda: torch.mm(x, Wq.t(), out=qkv), mb * 4, 6.0 * M * d * d)
    Wo = rn(d, d)
    run("out plain", lambda: ops.linear_fwd(x, Wo, y), mb * 2, 2.0 * M * d * d)
    run("qkv dgrad plain", lambda: ops.linear_dgrad(qkv, Wq, y), mb * 4, 6.0 * M * d * d)
    run("out dgrad plain", lambda: ops.linear_dgrad(z, Wo, y), mb * 2, 2.0 * M * d * d)
    run("out +bias+drop+resid", lambda: ops.linear_fwd(x, Wo, y, bias=b2, drop_ld=d, resid=z, **dk), mb * 3,
        2.0 * M * d * d)
    run("qkv +bias", lambda: ops.linear_fwd(x, Wq, qkv, bias=torch.zeros(3 * d, device=dev)), mb * 4,
        6.0 * M * d * d)
    run("torch.mm out", lambda: torch.mm(x, Wo.t(), out=y), mb * 2, 2.0 * M * d * d)
    torch.cuda.synchronize()
    print(f"{'op':60s} {'us':>8s} {'GB/s':>8s} {'TFLOP/s':>8s}")
    for n, us, bw, tf in rows:
        print(f"{n:60s} {us:8.2f} {bw:8.0f} {tf:8.1f}")


if __name__ == "__main__":
    main()
