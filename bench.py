#!/usr/bin/env python
"""Training-throughput benchmark of the SASRec / BERT4Rec HIP hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2] [--batch B]

For N > 1 launch one process per GPU (torchrun; RANK/LOCAL_RANK/WORLD_SIZE from the
env), RCCL all-reduce of the flat gradient each step, weak scaling (B sequences per
GPU).  One "step" = zero_grad + forward + loss + backward (+ all-reduce) + Adam on
one synthetic batch, captured once in a HIP graph and replayed (inputs resident in
HBM; each replay first copies its batch into the graph's static input buffers).
Rank 0 prints ONE JSON line (metric/value/unit/... + roofline + cpu_baseline).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_HBM_GBS = 8000.0          # spec peak (MI355X_MICROARCH.md)
MI355X_BF16_TFLOPS = 2500.0      # dense bf16 MFMA peak (spec, no sparsity)
MI355X_F32_TFLOPS = 157.3        # f32-input MFMA peak

CONFIGS = {
    # BASELINE.json configs[1] -- the metric's config: SASRec ML-1M shape, d=128, T=200, 2 blocks
    "cfg2": dict(model="sas", V=3416, T=200, d=128, L=2, h=1, p=0.2, B=128, shape="ml-1m",
                 name="SASRec ML-1M shape (|items|=3416, seq_len=200, d=128, 2 blocks, 1 head, dropout 0.2)"),
    # configs[3] shape (per-GPU part of the 8-GPU DP config)
    "cfg4": dict(model="sas", V=54542, T=50, d=128, L=2, h=1, p=0.2, B=128, shape="beauty",
                 name="SASRec Amazon-Beauty shape (|items|=54542, seq_len=50, d=128, 2 blocks, 1 head)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="sequences per GPU (default: the config's)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-graph", action="store_true")
    return ap.parse_args()


def make_model(cfg, dtype):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    a = argparse.Namespace(model_code=cfg["model"], num_items=cfg["V"], max_len=cfg["T"], device="cuda",
                           sas_hidden_units=cfg["d"], sas_num_blocks=cfg["L"], sas_heads=cfg["h"],
                           sas_dropout=cfg["p"], l2_emb=0.0, rs_dtype=dtype)
    return model_factory(a)


def make_batches(cfg, B, n, seed):
    import rbm_amd.data as synth
    rng = np.random.default_rng(seed)
    zipf = synth.ZipfItems(cfg["V"])
    out = []
    for _ in range(n):
        seq, pos, neg = synth.sas_batch(rng, B, cfg["T"], cfg["V"], shape=cfg["shape"], zipf=zipf)
        out.append(tuple(torch.from_numpy(a).cuda() for a in (seq, pos, neg)))
    return out


def attn_fwd_roofline(model, batch, cfg, dtype, reps=50):
    """Dominant-kernel roofline: time rs_attn_fwd alone with HIP events on its own stream."""
    from rbm_amd import ops
    eng = model.sas.engine()
    seq = batch[0]
    B, T = seq.shape
    d, H = cfg["d"], cfg["h"]
    Dh = d // H
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B * T, d, device="cuda", generator=g).to(dt)
    kv = torch.randn(B * T, 2 * d, device="cuda", generator=g).to(dt)
    o = torch.empty(B * T, d, device="cuda", dtype=dt)
    lse = torch.empty(B * H * T, device="cuda", dtype=torch.float32)
    s = torch.cuda.current_stream()
    args = (B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, lse, 1.0 / math.sqrt(Dh), 0, seq, cfg["p"], 123, eng.seed_base)
    for _ in range(5):
        ops.attn_fwd(*args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        ops.attn_fwd(*args)
    e1.record(s)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    flops = 2.0 * T * (T + 1) * Dh * B * H        # QK^T + PV over the causal triangle, 2 flop/MAC
    peak = MI355X_BF16_TFLOPS if dtype == "bf16" else MI355X_F32_TFLOPS
    achieved = flops / (us * 1e-6) / 1e12
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic_attn_fwd.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")
    return {"kernel": "attn_fwd_kernel (rs_attn_fwd)", "bound": "mfma", "achieved": round(achieved, 2),
            "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
            "avg_launch_us": round(us, 2), "flops_per_launch": flops}


def cpu_baseline(cfg, B, seconds):
    """The CPU oracle (PyTorch-CPU fp32 restatement of the reference math, dropout at the
    config value via torch bernoulli like the reference) timed on this host's cores."""
    import rbm_amd.data as synth
    from oracle import sas as osas
    from oracle.optim import AdamOracle
    cores = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    model = make_model_cpu(cfg)
    P = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = AdamOracle(list(P.values()))
    rng = np.random.default_rng(99)
    batch = [torch.from_numpy(a) for a in synth.sas_batch(rng, B, cfg["T"], cfg["V"], shape=cfg["shape"])]
    osas.loss_and_grads(P, *batch, cfg["L"], cfg["h"], p=cfg["p"], masks=osas.RandomDropout())  # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        _, _, _, g = osas.loss_and_grads(P, *batch, cfg["L"], cfg["h"], p=cfg["p"], masks=osas.RandomDropout())
        opt.step([g[k] for k in P])
        steps += 1
        if time.perf_counter() - t0 > seconds and steps >= 2:
            break
    dt = time.perf_counter() - t0
    return {"value": round(steps * B / dt, 2), "unit": "sequences/s", "cores": cores, "kind": "port",
            "sample": f"{steps} full train steps (fwd+BCE+bwd+Adam, fp32, dropout {cfg['p']}) of the "
                      f"workload at batch {B} with the oracle (oracle/sas.py), {dt:.1f} s"}


def make_model_cpu(cfg):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    a = argparse.Namespace(model_code="sas", num_items=cfg["V"], max_len=cfg["T"], device="cpu",
                           sas_hidden_units=cfg["d"], sas_num_blocks=cfg["L"], sas_heads=cfg["h"],
                           sas_dropout=cfg["p"], l2_emb=0.0)
    return model_factory(a)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    cfg = dict(CONFIGS[args.config])
    B = args.batch or cfg["B"]
    torch.manual_seed(1234)               # identical initial weights on every rank
    model = make_model(cfg, args.dtype)
    model.train()
    from rbm_amd.train_step import FusedTrainStep
    trainer = FusedTrainStep(model, lr=1e-3)
    batches = make_batches(cfg, B, 8, seed=1000 + rank)

    if args.no_graph:
        run = trainer.step
    else:
        trainer.capture(*batches[0])
        run = trainer.replay
    for i in range(args.warmup):
        loss = run(*batches[i % len(batches)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = run(*batches[i % len(batches)])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = tt.item()
    final_loss = float(loss.float().sum().item())

    roof = attn_fwd_roofline(model, batches[0], cfg, args.dtype)
    if rank == 0:
        cpu = cpu_baseline(cfg, B, args.cpu_baseline_seconds) if world == 1 and args.cpu_baseline_seconds > 0 \
            else None
        line = {
            "metric": "training sequences/sec, SASRec L=200 d=128 (HR@10 parity tested separately)",
            "value": round(world * B * args.steps / elapsed, 1),
            "unit": "sequences/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (Zipf item ids, ML-1M-shaped history lengths, random-init weights)",
            "config": {"workload": cfg["name"], "model": "SASRec", "global_batch": world * B, "per_gpu_batch": B,
                       "seq_len": cfg["T"], "hidden": cfg["d"], "blocks": cfg["L"], "heads": cfg["h"],
                       "num_items": cfg["V"], "parallelism": f"dp{world}", "hip_graph": not args.no_graph},
            "final_loss": round(final_loss, 5),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
