"""Which bf16 store drives the benchmarked path's loss-curve drift?  (diagnostic; not a test)

Replays tests/golden/sas_curve_bench.npz -- the reference's own 1000-step run at the bench shape (3,416 items, T 200,
d 128, 2 blocks, B 16, lr 1e-3, dropout 0) -- with tools/diag/bf16_budget.py's emulation of the fused bf16 step
(fp64 math, bf16 rounding exactly where the HIP path stores bf16, in rounding groups) and an fp64 Adam
(oracle/optim.py), once with every group on and once per group with THAT group kept exact, and reports each curve
against the reference's fp32 losses: max |dloss|, mean, and the 50-step moving-average deviation.

    python tools/diag/bf16_curve_budget.py [--steps 1000] [--jobs 4] [--variants all,all-W,...] > out.txt
"""
import argparse
import concurrent.futures as cf
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "diag"))


def run(variant, steps, threads):
    import torch
    torch.set_num_threads(threads)
    import bf16_budget as bb
    import rbm_amd.data as synth
    from oracle.optim import AdamOracle
    bb.ON.clear()
    if variant == "exact":
        pass
    elif variant == "all":
        bb.ON.update(bb.GROUPS)
    elif variant.startswith("all-"):
        bb.ON.update(set(bb.GROUPS) - set(variant[4:].split("+")))
    elif variant.startswith("only-"):
        bb.ON.update(variant[5:].split("+"))
    z = np.load(os.path.join(ROOT, "tests", "golden", "sas_curve_bench.npz"))
    V, T, d, L, h, B = (int(z[k]) for k in ("V", "T", "d", "L", "h", "B"))
    P = {k[2:]: torch.from_numpy(z[k]).double() for k in z.files if k.startswith("p/")}
    names = list(P)
    opt = AdamOracle([P[k] for k in names], lr=float(z["lr"]))
    rng = np.random.default_rng(int(z["seed"]))
    zipf = synth.ZipfItems(V)
    losses = []
    for _ in range(steps):
        seq, pos, neg = (torch.from_numpy(x) for x in synth.sas_batch(rng, B, T, V, zipf=zipf))
        loss, g = bb.loss_and_grads(P, seq, pos, neg, L, h)
        g["sas.item_emb.weight"][0] = 0.0          # padding_idx row: no gradient (nn.Embedding)
        opt.step([g[k] for k in names])
        losses.append(loss)
    ref = z["losses"][:steps]
    err = np.abs(np.array(losses) - ref)
    ma = lambda x: np.convolve(x, np.ones(50) / 50, mode="valid")  # noqa: E731
    dma = np.abs(ma(np.array(losses)) - ma(ref)).max() if steps >= 50 else float("nan")
    return variant, float(err.max()), float(err.mean()), float(dma)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()
    import bf16_budget as bb
    variants = args.variants.split(",") if args.variants else \
        ["exact", "all"] + [f"all-{g}" for g in bb.GROUPS]
    threads = max(1, (os.cpu_count() or 8) // args.jobs)
    with cf.ProcessPoolExecutor(args.jobs) as ex:
        futs = [ex.submit(run, v, args.steps, threads) for v in variants]
        for f in cf.as_completed(futs):
            v, mx, mean, dma = f.result()
            print(f"{v:14s} max {mx:.3e}  mean {mean:.3e}  ma50 {dma:.3e}", flush=True)


if __name__ == "__main__":
    main()
