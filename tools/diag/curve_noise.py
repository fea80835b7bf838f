"""How far do two fp32 implementations of the same math drift apart over the bench-shape 1000-step run?
Replays tests/golden/sas_curve_bench.npz with the oracle (this repo's CPU restatement) in fp32 and fp64 and
compares with the reference's own fp32 / fp64 runs (diagnostic; not a test).

    python tools/diag/curve_noise.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import rbm_amd.data as synth  # noqa: E402
from oracle import sas as osas  # noqa: E402
from oracle.optim import AdamOracle  # noqa: E402


def run(z, dtype, steps, ulp_seed=None):
    """ulp_seed: flip the last mantissa bit of a random half of the initial weights (a one-ulp perturbation: the
    spread of such runs is the fp32 rounding noise of the trajectory itself)."""
    V, T, d, L, h, B = (int(z[k]) for k in ("V", "T", "d", "L", "h", "B"))
    P = {k[2:]: torch.from_numpy(z[k]).to(dtype) for k in z.files if k.startswith("p/")}
    if ulp_seed is not None:
        g = torch.Generator().manual_seed(ulp_seed)
        for k, v in P.items():
            bits = v.view(torch.int32)
            bits ^= torch.randint(0, 2, v.shape, generator=g, dtype=torch.int32)
    opt = AdamOracle(list(P.values()), lr=float(z["lr"]))
    rng = np.random.default_rng(int(z["seed"]))
    zipf = synth.ZipfItems(V)
    out = []
    for _ in range(steps):
        seq, pos, neg = (torch.from_numpy(x) for x in synth.sas_batch(rng, B, T, V, zipf=zipf))
        loss, _, _, g = osas.loss_and_grads(P, seq, pos, neg, L, h)
        out.append(loss.item())
        opt.step([g[k] for k in P])
    return np.array(out)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sweep":
    # distribution of the fp32 drift: thread counts (BLAS reduction orders) and one-ulp weight perturbations
    z = np.load(os.path.join(ROOT, "tests", "golden", "sas_curve_bench.npz"))
    r32, r64 = z["losses"], z["losses64"]
    for nt, us in [(8, None), (4, None), (2, None), (8, 1), (8, 2), (8, 3), (8, 4)]:
        torch.set_num_threads(nt)
        o = run(z, torch.float32, int(z["steps"]), ulp_seed=us)
        print(f"threads {nt} ulp {us}: vs ref32 max {np.abs(o - r32).max():.2e}  vs ref64 max {np.abs(o - r64).max():.2e}"
              f" mean {np.abs(o - r64).mean():.2e}", flush=True)
    sys.exit(0)

if __name__ == "__main__":
    torch.set_num_threads(8)
    z = np.load(os.path.join(ROOT, "tests", "golden", "sas_curve_bench.npz"))
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else int(z["steps"])
    o32 = run(z, torch.float32, steps)
    o64 = run(z, torch.float64, steps)
    r32, r64 = z["losses"][:steps], z["losses64"][:steps]
    for name, a, b in [("oracle32 vs ref32", o32, r32), ("oracle32 vs ref64", o32, r64),
                       ("oracle64 vs ref64", o64, r64), ("ref32 vs ref64", r32, r64)]:
        e = np.abs(a - b)
        print(f"{name:20s} max {e.max():.2e} mean {e.mean():.2e} frac>1e-3 {(e > 1e-3).mean():.3f}")
    np.savez_compressed("/tmp/curve_noise.npz", o32=o32, o64=o64)
