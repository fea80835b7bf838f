"""Rates of the cfg5 vocabulary-head GEMMs: the build's kernels (rs_linear_wgrad for dE = dlogits^T h, split-K rs_gemm
for dh = dlogits E) against hipBLASLt through torch.mm on the same shapes (bf16 in; torch.mm writes bf16), as a
reference point for what the matrix cores sustain on these shapes.

    python tools/diag/vocab_gemm_probe.py [--R 1792] [--V 1000001] [--d 256]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


REPS = [20]


def timed(fn, reps=None):
    reps = reps or REPS[0]
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=1792)
    ap.add_argument("--V", type=int, default=1000001)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--only", default="", help="run only the n256 kernels ('n256')")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    R, V, d = a.R, a.V, a.d
    REPS[0] = a.reps
    Vp = -(-V // 64) * 64
    dl = (torch.randn(R, Vp, device="cuda") * 1e-3).bfloat16()[:, :V]
    h = torch.randn(R, d, device="cuda").bfloat16()
    E = (torch.randn(V, d, device="cuda") * 0.02).bfloat16()
    fl = 2.0 * R * V * d
    dE = torch.empty(V, d, device="cuda")
    db = torch.empty(V, device="cuda")
    if a.only != "n256":
        slab = torch.empty(ops.wgrad_slab_numel(R, V, d), device="cuda")
        us = timed(lambda: ops.linear_wgrad(dl, h, dE, slab, db=db, accumulate=False))
        print(f"dE  rs_linear_wgrad      {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
        sk = int(max(1, min(64, -(-V // 2048))))
        slab_d = torch.empty(sk * R * d, device="cuda")
        us = timed(lambda: ops.gemm(dl, E, slab_d, R, d, V, False, True, ops.epilogue(), split_k=sk, slab=slab_d))
        print(f"dh  rs_gemm split-K {sk:3d} {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
    us = timed(lambda: ops.gemm_n256(dl, h, dE, True, V, R, colsum=db))
    print(f"dE  rs_gemm_n256         {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
    S = ops.gemm_n256_splits(R, V)
    slab2 = torch.empty(S, R, d, device="cuda")
    us = timed(lambda: ops.gemm_n256(dl, E, slab2, False, R, V, split=True))
    print(f"dh  rs_gemm_n256 x{S:3d}    {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
    if a.only == "n256":
        return
    dlc = dl.contiguous()
    us = timed(lambda: torch.mm(dlc.t(), h))
    print(f"dE  torch.mm (hipBLASLt) {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
    us = timed(lambda: torch.mm(dlc, E))
    print(f"dh  torch.mm (hipBLASLt) {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
    x = torch.randn(8192, 8192, device="cuda").bfloat16()
    us = timed(lambda: torch.mm(x, x), 10)
    print(f"8192^3 torch.mm          {us:9.1f} us  {2 * 8192 ** 3 / us / 1e6:7.1f} TFLOP/s")


if __name__ == "__main__":
    main()
