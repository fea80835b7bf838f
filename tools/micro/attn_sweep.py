"""Attention kernel timing sweep over sequence lengths (GPU): where does the time go?"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import rbm_amd  # noqa: E402,F401
from rbm_amd import ops  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    d, H = 128, 1
    for B, T, mk in [(128, 200, 0), (128, 200, 1), (128, 112, 0), (228, 112, 0), (128, 64, 0), (400, 64, 0),
                     (128, 256, 0), (64, 200, 0), (256, 200, 0)]:
        M = B * T
        q = torch.randn(M, d, device="cuda").bfloat16()
        kv = torch.randn(M, 2 * d, device="cuda").bfloat16()
        o = torch.empty(M, d, device="cuda").bfloat16()
        do = torch.randn(M, d, device="cuda").bfloat16()
        lse = torch.empty(B * T, device="cuda")
        ids = torch.ones(B, T, dtype=torch.int64, device="cuda")
        sb = torch.zeros(1, dtype=torch.int64, device="cuda")
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        ws = torch.empty(B * T, device="cuda")
        sc = 1 / math.sqrt(d)
        tf = timeit(lambda: ops.attn_fwd(B, T, H, d, q, kv[:, :d], kv[:, d:], o, lse, sc, mk, ids, 0.2, 5, sb))
        tb = timeit(lambda: ops.attn_bwd(B, T, H, d, q, kv[:, :d], kv[:, d:], o, do, lse, dq, dkv[:, :d], dkv[:, d:],
                                         sc, mk, ids, 0.2, 5, sb, ws))
        print(f"B={B:4d} T={T:4d} mask={mk}  fwd {tf:7.2f} us  bwd {tb:7.2f} us   per 1k tokens: fwd {tf / M * 1e3:6.3f} "
              f"bwd {tb / M * 1e3:6.3f}")


if __name__ == "__main__":
    main()
