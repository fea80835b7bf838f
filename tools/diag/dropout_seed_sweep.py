"""bf16 fused SAS step vs the oracle's bf16-storage emulation and the exact math, over several dropout seeds of one
shape (tests/test_dropout_parity_gpu.py's construction): is a large kernel-vs-emulation error a kernel error or an
ill-conditioned draw (then the emulation's own distance to the exact math, fmt, is large too)?

    python tools/diag/dropout_seed_sweep.py --V 300 --T 37 --d 128 --B 3 --seeds 970-985
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=300)
    ap.add_argument("--T", type=int, default=37)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--B", type=int, default=3)
    ap.add_argument("--seeds", default="970-985")
    a = ap.parse_args()
    import rbm_amd.data as synth
    import test_dropout_parity_gpu as tp
    from conftest import rel
    from oracle import sas as osas
    from rbm_amd.train_step import FusedTrainStep
    lo, hi = (int(x) for x in a.seeds.split("-"))
    p, L, h = 0.2, 2, 1
    m = tp._sas_model(a.V, a.T, a.d, L, h, p, "bf16", seed=a.V + a.T)
    tr = FusedTrainStep(m, lr=1e-3)
    rng = np.random.default_rng(a.T)
    seq, pos, neg = (torch.from_numpy(x).cuda() for x in synth.sas_batch(rng, a.B, a.T, a.V))
    P = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    torch.set_num_threads(16)
    for seed in range(lo, hi + 1):
        _, grads = tp._step_grads(tr, (seq, pos, neg), seed)
        sb = torch.full((1,), seed, dtype=torch.int64, device="cuda")
        masks = {k: v.cpu().double() for k, v in tp.sas_masks(tr.engine, a.B, a.T, sb).items()}
        _, _, _, g64 = osas.loss_and_grads(P, seq.cpu(), pos.cpu(), neg.cpu(), L, h, p=p, masks=masks)
        _, _, _, ge = osas.loss_and_grads(P, seq.cpu(), pos.cpu(), neg.cpu(), L, h, p=p, masks=masks,
                                          emu=osas.BF16Storage())
        emu, fmt = [], []
        for k in g64:
            name = k[4:]
            if name.endswith("in_proj_bias"):
                continue
            g = tr.flat.view(name, grads).cpu().numpy().astype(np.float64)
            emu.append((rel(g, ge[k].numpy()), name))
            fmt.append((rel(ge[k].numpy(), g64[k].numpy()), name))
        print(f"seed {seed}: worst kernel-vs-emulation {max(emu)[0]:.4f} ({max(emu)[1]}), median {np.median([e for e, _ in emu]):.4f}; "
              f"worst emulation-vs-exact {max(fmt)[0]:.4f} ({max(fmt)[1]}), median {np.median([f for f, _ in fmt]):.4f}",
              flush=True)


if __name__ == "__main__":
    main()
