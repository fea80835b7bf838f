"""Time the fused SAS training step at any width / dtype (GPU only) -- e.g. the reference's default d = 50
(BASELINE configs[0]'s model on the GPU), which takes the generic kernels, not the row-chain ones.

    python tools/width_step.py --d 50 --dtype bf16 [--B 64 --T 200 --V 3416 --steps 50]

Prints ms/step (HIP graph of one step, replayed); run it under `rocprofv3 --kernel-trace --stats` for the kernel
breakdown.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=50)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--V", type=int, default=3416)
    ap.add_argument("--L", type=int, default=2)
    ap.add_argument("--h", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import rbm_amd.data as synth
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    args = argparse.Namespace(model_code="sas", num_items=a.V, max_len=a.T, device="cuda", sas_hidden_units=a.d,
                              sas_num_blocks=a.L, sas_heads=a.h, sas_dropout=0.2, l2_emb=0.0, rs_dtype=a.dtype)
    torch.manual_seed(0)
    m = model_factory(args)
    m.train()
    tr = FusedTrainStep(m, lr=1e-3)
    rng = np.random.default_rng(0)
    batch = [torch.from_numpy(x).cuda() for x in synth.sas_batch(rng, a.B, a.T, a.V)]
    tr.capture(*batch)
    for _ in range(5):
        tr.replay(*batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.replay(*batch)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    print(f"SAS d={a.d} {a.dtype} B={a.B} T={a.T} V={a.V}: {ms:.4f} ms/step, {a.B / ms * 1e3:.0f} seq/s")


if __name__ == "__main__":
    main()
