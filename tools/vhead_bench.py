#!/usr/bin/env python
"""Micro-benchmark of the BERT vocabulary-head kernels at a vocabulary size (GPU only).

    python tools/vhead_bench.py [--V 1000000] [--R 1750] [--d 256] [--reps 10] [--only fwd,bwd,wgrad,dgrad]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rbm_amd  # noqa: E402,F401
from rbm_amd import ops  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=1000000)
    ap.add_argument("--R", type=int, default=1750)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="fwd,bwd,wgrad,dgrad")
    ap.add_argument("--sk", default="", help="','-separated split-K counts to time the dgrad at (default: the step's)")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    R, V1, d = a.R, a.V + 1, a.d
    h = torch.randn(R, d, device="cuda", generator=g).bfloat16()
    E = (0.05 * torch.randn(V1, d, device="cuda", generator=g)).bfloat16()
    bias = torch.zeros(V1, device="cuda")
    lab = torch.randint(1, V1, (R,), device="cuda", generator=g)
    ws = torch.empty(ops.vocab_ce_ws_numel(R, V1), device="cuda")
    out = torch.empty(4, device="cuda")
    cnt = torch.tensor([float(R)], device="cuda")
    V1p = -(-V1 // 8) * 8
    dl = torch.empty(R, V1p, device="cuda", dtype=torch.bfloat16)[:, :V1]
    dE = torch.zeros(V1, d, device="cuda")
    db = torch.zeros(V1, device="cuda")
    fl = 2.0 * R * V1 * d
    only = a.only.split(",")
    ops.vocab_head_fwd(h, E, bias, lab, ws, out)
    torch.cuda.synchronize()
    if "fwd" in only:
        for pp in ("1", "0"):     # RS_VHEAD_PP: the ping-pong form, then the lock-step form
            os.environ["RS_VHEAD_PP"] = pp
            us = timeit(lambda: ops.vocab_head_fwd(h, E, bias, lab, ws, out), a.reps)
            print(f"vocab_head_fwd   {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s  (RS_VHEAD_PP={pp}) loss {float(out[0]):.6e}")
        os.environ.pop("RS_VHEAD_PP")
    if "bwd" in only:
        for pp in ("1", "0"):
            os.environ["RS_VHEAD_PP"] = pp
            us = timeit(lambda: ops.vocab_head_bwd(h, E, bias, lab, ws, cnt, dl), a.reps)
            print(f"vocab_head_bwd   {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s  (RS_VHEAD_PP={pp})")
        os.environ.pop("RS_VHEAD_PP")
    if "wgrad" in only:
        slab = torch.empty(1, device="cuda")
        us = timeit(lambda: ops.linear_wgrad(dl, h, dE, slab, db=db), a.reps)
        print(f"wgrad dE=dl^T h  {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
    if "dgrad" in only:
        for sk in ([int(x) for x in a.sk.split(",")] if a.sk else [int(max(1, min(64, -(-V1 // 2048))))]):
            slab_d = torch.empty(sk * R * d, device="cuda")
            us = timeit(lambda: ops.gemm(dl, E, slab_d, R, d, V1, False, True, ops.epilogue(), split_k=sk,
                                         slab=slab_d), a.reps)
            print(f"dgrad dh=dl E    {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s (split-K {sk} slabs, reduction not incl.)")


if __name__ == "__main__":
    main()
