#!/usr/bin/env python
"""Training-throughput benchmark of the SASRec / BERT4Rec HIP hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5] [--batch B]

BASELINE.json's metric is training sequences/sec for SASRec T=200 d=128 (configs[1] = cfg2,
the default).  For N > 1 one process runs per GPU: either the driver's torchrun starts them
(RANK / LOCAL_RANK / WORLD_SIZE from the env; WORLD_SIZE must equal --gpus), or `bench.py --gpus N`
started alone launches the N ranks itself (torch.distributed.run children, before any GPU call).
Data parallel, RCCL all-reduce of the flat gradient (+ loss-sum/count aux) each step, weak
scaling (B sequences per GPU).

One "step" = zero_grad + forward + loss + backward (+ all-reduce) + Adam on one synthetic batch
already resident in HBM: the step is captured once in HIP graphs and replayed; each replay first
copies its batch into the graph's static input buffers (device to device).  Rank 0 prints ONE
JSON line with metric/value/unit/... plus
  roofline     -- the dominant kernel (most device time per step, from the rocprof profile
                  committed under profiles/), re-timed here with HIP events on its own stream,
                  algorithmic bytes or flops per launch / average launch time vs the chip peak;
  cpu_baseline -- the CPU oracle (PyTorch-CPU fp32 restatement of the reference math, dropout
                  at the config value) timed on this host for a bounded sample of the workload.
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
RIDGE_BF16 = MI355X_BF16_TFLOPS * 1e12 / (MI355X_HBM_GBS * 1e9)   # flop/B

CONFIGS = {
    # BASELINE.json configs[1] -- the metric's config
    "cfg2": dict(model="sas", V=3416, T=200, d=128, L=2, h=1, p=0.2, B=128, shape="ml-1m",
                 name="SASRec ML-1M shape (|items|=3416, seq_len=200, d=128, 2 blocks, 1 head, dropout 0.2)"),
    # configs[2]
    "cfg3": dict(model="bert", V=26744, T=200, d=256, L=4, h=2, p=0.1, B=64, shape="ml-1m", mask=0.2,
                 name="BERT4Rec ML-20M shape (|items|=26744, seq_len=200, d=256, 4 blocks, 2 heads, mask 0.2, "
                      "dropout 0.1)"),
    # configs[3] (per-GPU share of the 8-GPU DP config)
    "cfg4": dict(model="sas", V=54542, T=50, d=128, L=2, h=1, p=0.2, B=128, shape="beauty",
                 name="SASRec Amazon-Beauty shape (|items|=54542, seq_len=50, d=128, 2 blocks, 1 head)"),
    # configs[4] (per-GPU share)
    "cfg5": dict(model="bert", V=1000000, T=200, d=256, L=4, h=2, p=0.1, B=64, shape="ml-1m", mask=0.2,
                 name="BERT4Rec synthetic 1M-item catalog (seq_len=200, d=256, 4 blocks, 2 heads, mask 0.2)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=24)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="sequences per GPU (default: the config's)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--vocab-shard", default="auto", choices=["auto", "on", "off"],
                    help="BERT, N > 1: shard out.weight over the ranks (auto: on for vocabularies >= 100k)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-process path with several ranks on one GPU)")
    ap.add_argument("--steps-per-graph", default="auto",
                    help="training steps unrolled into one graph replay (single GPU; 'auto' = the largest of "
                         "20/10/8/5/4/2 dividing --steps, else 1); every step still runs on its own batch with its own "
                         "Adam update; warmup steps beyond a multiple of it run as eager steps")
    ap.add_argument("--roofline-replays", type=int, default=20,
                    help="eager training steps after the timed ones with HIP timing events around the dominant "
                         "kernel's launches (0 = none: the in-kernel stamps of the timed steps then give "
                         "avg_launch_us)")
    ap.add_argument("--nbatches", type=int, default=8, help="distinct synthetic batches cycled through")
    ap.add_argument("--sampler", default="host", choices=["host", "device"],
                    help="SAS: 'device' = batches drawn each step by the on-device WarpSampler "
                         "(rs_sas_sample) inside the step's graph, from synthetic user histories")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


# ------------------------------------------------------------------------------------ rank launcher
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` started WITHOUT a torchrun environment (no WORLD_SIZE): start the N data-parallel
    ranks as child processes -- torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1 -- and
    return the worst exit status.  Called before anything touches the GPU (this process never initialises
    HIP; the children do), and the children are started, never exec'd into.  The reference picks its device
    count from the device list (`BS/utils.py:74-76`, `BS/trainers/base.py:32-34`)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC: RCCL / CUDA-tensor sharing across ranks
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def world_from_env(gpus):
    """(world, rank, local_rank) of this process; under torchrun WORLD_SIZE must equal --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {gpus}: start N ranks with `bench.py --gpus N` "
                         f"(it launches them) or torchrun --nproc-per-node N ... bench.py --gpus N")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def launch_selftest(args):
    """CPU check of the launcher's plumbing (tests/test_bench_launch.py): every rank joins a gloo group of the
    launched size, the ranks all-reduce their rank ids, and rank 0 prints one line with the live world size."""
    world, rank, _ = world_from_env(args.gpus)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank)])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "parallelism": f"dp{world}", "rank_sum": t.item()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def model_args(cfg, dtype, device):
    if cfg["model"] == "sas":
        return argparse.Namespace(model_code="sas", num_items=cfg["V"], max_len=cfg["T"], device=device,
                                  sas_hidden_units=cfg["d"], sas_num_blocks=cfg["L"], sas_heads=cfg["h"],
                                  sas_dropout=cfg["p"], l2_emb=0.0, rs_dtype=dtype)
    return argparse.Namespace(model_code="bert", num_items=cfg["V"], max_len=cfg["T"], device=device,
                              bert_hidden_units=cfg["d"], bert_num_blocks=cfg["L"], bert_num_heads=cfg["h"],
                              bert_dropout=cfg["p"], bert_hidden_dropout=cfg["p"], bert_mask_prob=cfg["mask"],
                              model_init_seed=0, rs_dtype=dtype)


def make_model(cfg, dtype, device="cuda"):
    import rbm_amd  # noqa: F401
    from rbm_amd.models import model_factory
    return model_factory(model_args(cfg, dtype, device))


def make_batches(cfg, B, n, seed):
    """Synthetic interaction streams (rbm_amd.data): Zipf item ids, config-shaped history lengths."""
    import rbm_amd.data as synth
    rng = np.random.default_rng(seed)
    zipf = synth.ZipfItems(cfg["V"])
    out = []
    for _ in range(n):
        if cfg["model"] == "sas":
            b = synth.sas_batch(rng, B, cfg["T"], cfg["V"], shape=cfg["shape"], zipf=zipf)
        else:
            b = synth.bert_batch(rng, B, cfg["T"], cfg["V"], mask_prob=cfg["mask"], shape=cfg["shape"], zipf=zipf)
        out.append(b)
    return out


CFG_NAME = "cfg2"

# ------------------------------------------------------------------------------------ roofline
def _time_on_stream(fn, reps, stream):
    with torch.cuda.stream(stream):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def _roof(kernel, us, flops, nbytes, dtype, note, live_us=None, live_expected=None, event_us=None):
    iso_us = us
    stamp_us = sum(live_us) / len(live_us) if live_us else None
    if event_us:
        us = sum(event_us) / len(event_us)
        note += (f"; avg_launch_us = mean of {len(event_us)} launches inside training steps of the same trainer run "
                 f"after the timed ones, each bracketed by HIP timing events on the stream it runs on, minus the "
                 f"median time of an empty event pair queued the same way (event_pair_cost_us)")
        if live_us:
            note += (f"; stamp_launch_us = mean of {len(live_us)} launches of the timed steps themselves (in-kernel "
                     f"s_memrealtime stamps: first wave in to last wave out, so without dispatch ramp and drain)")
    elif live_us:
        us = stamp_us
        note += (f"; avg_launch_us = mean of {len(live_us)} launches timed inside the timed steps (in-kernel "
                 f"s_memrealtime stamps: first wave in to last wave out of the launch)")
    note += "; isolated_launch_us = the same launch re-timed alone, back to back, with HIP events"
    ai = flops / nbytes if nbytes else float("inf")
    peak_f = MI355X_BF16_TFLOPS if dtype == "bf16" else MI355X_F32_TFLOPS
    # both utilisations of the same live launch time, whichever bound the arithmetic intensity selects
    util = {"mfma_util": round(flops / (us * 1e-6) / 1e12 / peak_f, 4),
            "hbm_util": round(nbytes / (us * 1e-6) / 1e9 / MI355X_HBM_GBS, 4)}
    ridge = peak_f * 1e12 / (MI355X_HBM_GBS * 1e9)
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):   # measured HBM bytes per launch at this config (tools/make_traffic.py)
        traffic = json.load(open(tpath)).get(CFG_NAME, {}).get(kernel)
    if ai < ridge:
        ach = nbytes / (us * 1e-6) / 1e9
        return {"kernel": kernel, "bound": "hbm", "achieved": round(ach, 1), "peak": MI355X_HBM_GBS, "unit": "GB/s",
                "frac": round(ach / MI355X_HBM_GBS, 4), "traffic": traffic, "avg_launch_us": round(us, 2),
                "isolated_launch_us": round(iso_us, 2),
                "stamp_launch_us": round(stamp_us, 2) if stamp_us else None, "event_samples": len(event_us or ()),
                "live_samples": len(live_us or ()),
                "live_samples_expected": live_expected,
                "algorithmic_bytes_per_launch": int(nbytes), "algorithmic_flops_per_launch": int(flops),
                "arith_intensity": round(ai, 1), **util, "note": note}
    ach = flops / (us * 1e-6) / 1e12
    return {"kernel": kernel, "bound": "mfma", "achieved": round(ach, 2), "peak": peak_f, "unit": "TFLOP/s",
            "frac": round(ach / peak_f, 4), "traffic": traffic, "avg_launch_us": round(us, 2),
            "isolated_launch_us": round(iso_us, 2),
            "stamp_launch_us": round(stamp_us, 2) if stamp_us else None, "event_samples": len(event_us or ()),
            "live_samples": len(live_us or ()),
            "live_samples_expected": live_expected,
            "algorithmic_bytes_per_launch": int(nbytes), "algorithmic_flops_per_launch": int(flops),
            "arith_intensity": round(ai, 1), **util, "note": note}


# ops wrapper of the dominant kernel per config (most device time per step in the rocprof profiles):
# SAS -> the attention backward; BERT at 27k items -> the grouped block weight gradients; BERT at 1M items ->
# the vocabulary-logits GEMM (rs_vocab_ce_fwd; its backward twin recomputes the same product)
def dominant(cfg):
    if cfg["model"] == "sas":
        return "attn_bwd"
    return "vocab_ce_fwd" if cfg["V"] >= 100000 else "wgrad_grouped"


def roofline(cfg, B, dtype, live_us=None, reps=50, labelled=None, live_expected=None, event_us=None):
    """Dominant kernel of the step (by rocprof device time).  SAS: the attention backward (rs_attn_bwd:
    dQ+delta and dK/dV kernels); BERT: the grouped block weight gradients (rs_wgrad_grouped).
    live_us: its launch durations measured INSIDE the timed step replays (in-kernel begin/end stamps of
    every launch of every timed step, ops.kernel_stamps; event-record nodes in a ROCm graph add a ~6 us
    barrier each, so HIP events inside the graph would perturb the step they time) -- `achieved` is
    computed from their mean.  The same launch is also re-timed alone here with HIP
    events on a dedicated stream (`isolated_launch_us`, a cross-check)."""
    from rbm_amd import ops
    es = 2 if dtype == "bf16" else 4
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(0)
    stream = torch.cuda.Stream()
    T, d, H = cfg["T"], cfg["d"], cfg["h"]
    Dh = d // H
    if cfg["model"] == "sas":
        M = B * T
        q = torch.randn(M, d, device="cuda", generator=g).to(dt)
        kv = torch.randn(M, 2 * d, device="cuda", generator=g).to(dt)
        o = torch.randn(M, d, device="cuda", generator=g).to(dt)
        do = torch.randn(M, d, device="cuda", generator=g).to(dt)
        lse = torch.zeros(B * H * T, device="cuda")
        ids = torch.ones(B, T, dtype=torch.int64, device="cuda")
        sb = torch.zeros(1, dtype=torch.int64, device="cuda")
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        ws = torch.empty(B * H * T, device="cuda")
        with torch.cuda.stream(stream):
            ops.attn_fwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, lse, 1 / math.sqrt(Dh), 0, ids, cfg["p"], 5, sb)
            # the step's variant: delta = rowsum(dO*O) handed in by the out-side backward (sas.py, delta_in=True),
            # so the launch timed here reads neither O nor forms delta, exactly like the live-stamped one
            ops.attn_row_delta(B, T, H, Dh, do, o, ws)
        us = _time_on_stream(lambda: ops.attn_bwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, do, lse, dq, dkv[:, :d],
                                                  dkv[:, d:], 1 / math.sqrt(Dh), 0, ids, cfg["p"], 5, sb, ws,
                                                  delta_in=True),
                             reps, stream)
        # algorithmic: dV, dP, dQ, dK products over the causal triangle (2 flop/MAC); bytes: read
        # q, k, v, dO + lse, delta, write dq, dk, dv once (7 activation tensors of M x d)
        flops = 4 * 2.0 * (T * (T + 1) / 2) * Dh * B * H
        nbytes = 7 * M * d * es + B * H * T * 4 * 2
        return _roof("rs_attn_bwd (attn_bwd_lds: dQ + dK/dV workgroups)", us, flops, nbytes, dtype,
                     f"causal attention backward (delta_in: no O read), B={B} T={T} Dh={Dh} dropout {cfg['p']}; "
                     f"one launch, both passes", live_us, live_expected, event_us)
    if dominant(cfg) == "vocab_ce_fwd":
        # BERT, 1M-item vocabulary: h[R,d] . E^T + b with the online-softmax partial epilogue over the labelled
        # rows (R = the batches' mean labelled count), E = out.weight [V+1, d] bf16
        R, V1 = int(round(labelled)), cfg["V"] + 1
        h = torch.randn(R, d, device="cuda", generator=g).to(dt)
        E = (0.05 * torch.randn(V1, d, device="cuda", generator=g)).to(dt)
        bias = torch.zeros(V1, device="cuda")
        lab = torch.randint(1, V1, (R,), device="cuda", generator=g)
        ws = torch.empty(ops.vocab_ce_ws_numel(R, V1), device="cuda")
        out = torch.empty(4, device="cuda")
        us = _time_on_stream(lambda: ops.vocab_head_fwd(h, E, bias, lab, ws, out), reps, stream)
        flops = 2.0 * R * V1 * d
        nbytes = (V1 * d + R * d) * es + R * -(-V1 // 128) * 2 * 4     # E, h once; (max, sum) partials
        return _roof("rs_vocab_head_fwd (E-tile-stationary logits + online-softmax partials)", us, flops, nbytes, dtype,
                     f"R={R} labelled rows (batch mean) x V+1={V1} x d={d}", live_us, live_expected, event_us)
    # BERT: the grouped weight-gradient launch of all block weights (rs_wgrad_grouped: GEMM + reduction),
    # the largest single kernel of the step
    from rbm_amd.models.bert_model.bert import BERTEngine
    M, Fd, L = B * T, 4 * d, cfg["L"]
    rn = lambda *s: torch.randn(*s, device="cuda", generator=g).to(dt)  # noqa: E731
    shapes = [(d, Fd), (Fd, d), (d, d), (3 * d, d)] * L        # W2, W1, Wo, Wqkv  (N, K)
    probs = [(rn(M, n), rn(M, k), torch.zeros(n, k, device="cuda"), torch.zeros(n, device="cuda"))
             for n, k in shapes]
    rows = BERTEngine._wgrad_rows(M, shapes)
    slab = torch.empty(ops.wgrad_grouped_slab_numel(shapes, M, rows), device="cuda")
    us = _time_on_stream(lambda: ops.wgrad_grouped(probs, M, rows, slab), reps, stream)
    flops = sum(2.0 * M * n * k for n, k in shapes)
    nbytes = sum(M * (n + k) * es + (n * k + n) * 4 * 2 for n, k in shapes)   # dY, X once; dW, db read+write
    kern = "wgrad_group256_kernel" if ops.wgrad_grouped_tile(shapes) == 256 else "wgrad_group_kernel"
    return _roof(f"rs_wgrad_grouped ({kern} + reduce_cols_kernel)", us, flops, nbytes, dtype,
                 f"{len(shapes)} block weight gradients of M={M} token rows (d={d}, ff={Fd}, L={L}), "
                 f"{-(-M // rows)} row splits; 2 kernels per launch", live_us, live_expected, event_us)


# ------------------------------------------------------------------------------------ CPU baseline
def _cgroup_cpu_quota():
    """CPUs granted by the cgroup's CPU quota (v2 cpu.max, v1 cfs_quota_us / cfs_period_us), None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def host_cpu_share():
    """The CPU share this process may use, from what the host actually grants it: the scheduler affinity mask, the
    cgroup CPU quota and the job's OMP_NUM_THREADS limit (the GPU box sets it to its per-GPU share); the baseline
    runs on the smallest of them.  os.cpu_count() is the whole host's count and is reported, not used."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cgroup_cpu_quota()
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    lim = [aff] + ([max(1, int(quota))] if quota else []) + ([omp] if omp else [])
    return {"threads": max(1, min(lim)), "affinity_cpus": aff,
            "cgroup_quota_cpus": round(quota, 2) if quota else None, "omp_num_threads": omp,
            "host_logical_cpus": os.cpu_count()}


def cpu_baseline(cfg, B, seconds):
    """The CPU oracle (PyTorch-CPU fp32 restatement of the reference math, torch bernoulli dropout
    at the config value like the reference) timed on this host's cores: full train steps
    (forward + loss + backward + Adam) on a batch of the workload, for a bounded time."""
    from oracle import bert as obert
    from oracle import sas as osas
    from oracle.optim import AdamOracle
    share = host_cpu_share()
    cores = share["threads"]
    try:
        import psutil
        physical = psutil.cpu_count(logical=False)
    except Exception:   # noqa: BLE001 -- informational only
        physical = None
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    m = make_model(cfg, "fp32", device="cpu")
    P = {k: v.detach().clone() for k, v in m.state_dict().items()}
    opt = AdamOracle(list(P.values()))
    # bounded sample: the workload's batch, except at a 1M-item vocabulary, where the oracle (like the reference)
    # materialises all-position logits B*T*(V+1) fp32 -- 51 GB at B = 64 -- so it runs batch 2 there
    Bc = B if (cfg["model"] == "sas" or cfg["V"] < 100000) else max(1, min(B, 2))
    batch = [torch.from_numpy(a) for a in make_batches(cfg, Bc, 1, 99)[0]]

    def one():
        if cfg["model"] == "sas":
            _, _, _, g = osas.loss_and_grads(P, *batch, cfg["L"], cfg["h"], p=cfg["p"], masks=osas.RandomDropout())
        else:
            _, _, g = obert.loss_and_grads(P, *batch, cfg["L"], cfg["h"], p=cfg["p"], hp=cfg["p"],
                                           masks=osas.RandomDropout())
        opt.step([g[k] for k in P])

    one()   # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        one()
        steps += 1
        if time.perf_counter() - t0 > seconds and steps >= 2:
            break
    dt = time.perf_counter() - t0
    return {"value": round(steps * Bc / dt, 2), "unit": "sequences/s", "cores": cores, "kind": "port",
            "sample": f"{steps} full train steps (fwd+loss+bwd+Adam, fp32, dropout {cfg['p']}) at batch {Bc} of the "
                      f"workload with the CPU oracle (oracle/{cfg['model']}.py), {dt:.1f} s on {cores} threads"
                      f" (host: {os.cpu_count()} logical / {physical} physical cores)",
            "cpu_share": share}


# ------------------------------------------------------------------------------------ main
def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # N ranks requested without a launcher: start them (torch.distributed.run children) and report the worst rc
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_selftest:
        return launch_selftest(args)
    world, rank, local = world_from_env(args.gpus)
    dev = local % max(1, torch.cuda.device_count())     # one GPU per rank (ranks > GPUs: gloo rehearsal only)
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    global CFG_NAME
    CFG_NAME = args.config
    cfg = dict(CONFIGS[args.config])
    B = args.batch or cfg["B"]
    torch.manual_seed(1234)               # identical initial weights on every rank
    model = make_model(cfg, args.dtype)
    model.train()
    host_batches = make_batches(cfg, B, args.nbatches, seed=1000 + rank)
    max_lab = None
    if cfg["model"] == "bert" and args.sampler == "host":
        cnt = max(int((lab != 0).sum()) for _, lab in host_batches)
        if world > 1:
            t = torch.tensor([cnt], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            cnt = int(t.item())
        max_lab = -(-cnt // 128) * 128
    batches = [tuple(torch.from_numpy(a).cuda() for a in b) for b in host_batches]
    from rbm_amd.train_step import FusedTrainStep
    vshard = cfg["model"] == "bert" and world > 1 and (
        args.vocab_shard == "on" or (args.vocab_shard == "auto" and cfg["V"] >= 100000))
    trainer = FusedTrainStep(model, lr=1e-3, max_labelled=max_lab, vocab_shard=vshard)
    # the dominant kernel is timed live, inside every timed step: the step graph is captured with kernel
    # stamps on (first wave in / last wave out s_memrealtime ticks of each stamped launch, per step)
    from rbm_amd import ops
    NMARK, WAVES = 8, 16384
    sbuf = None if args.no_graph else torch.zeros(4 + args.steps * NMARK * (1 + WAVES), dtype=torch.int64,
                                                  device="cuda")
    stamps = None if sbuf is None else (sbuf, (dominant(cfg),))

    if args.steps_per_graph == "auto":
        # the largest of 20 / 10 / 8 / 5 / 4 / 2 steps per replay that divides the timed count (a replay boundary costs
        # ~25 us; the driver's 20 timed steps at cfg2: 20 per replay 422.9-430.4k against 10 per replay
        # 418.2-426.2k seq/s, four interleaved rounds); the warmup need not be a multiple: its remainder runs as eager steps (below)
        # (data parallel: when the trainer captures its all-reduce inside the step graph -- SAS)
        unroll = (world == 1 or trainer.graph_collectives) and not args.no_graph
        S = next((u for u in (20, 10, 8, 5, 4, 2) if args.steps % u == 0), 1) if unroll else 1
    else:
        S = int(args.steps_per_graph)
        if S > 1 and ((world > 1 and not trainer.graph_collectives) or args.no_graph or args.steps % S):
            raise SystemExit("--steps-per-graph > 1 needs graphs (with the all-reduce inside them under DP) and "
                             "--steps a multiple of it")

    def capture(fn):
        """fn(S) captures the step graphs; under DP, an all-reduce that refuses capture in an unrolled graph falls
        back to one step per replay with the collectives between segment graphs (every rank alike)."""
        nonlocal S
        try:
            fn(S)
        except Exception as e:
            if world == 1 or S == 1:
                raise
            print(f"rank {rank}: unrolled DP capture failed ({e}); one step per replay", file=sys.stderr)
            torch.cuda.synchronize()
            trainer.graph_collectives = False
            if trainer.exchange is not None:
                trainer.exchange.works, trainer.exchange.sent = [], []
            S = 1
            fn(S)

    if args.sampler == "device" and cfg["model"] == "sas":
        import rbm_amd.data as synth
        from rbm_amd.dataloaders import DeviceWarpSampler
        users = synth.user_histories(np.random.default_rng(77 + rank), cfg.get("users", 6040), cfg["T"], cfg["V"],
                                     shape=cfg["shape"])
        sampler = DeviceWarpSampler(users, cfg["V"], B, cfg["T"], seed=5 + rank)
        capture(lambda s: trainer.capture_sampled(sampler, stamps=stamps, steps_per_graph=s))
        batches = [()]
        run = trainer.replay_sampled
        eager = lambda i: (sampler.sample_into(*trainer.static), trainer.step(*trainer.static))  # noqa: E731
    elif args.sampler == "device":
        # BERT: on-device cloze masking (rs_bert_mask) in the step graph; the labelled-row cap stays
        # B*T (default), every vocabulary GEMM is bounded by the device-side labelled count
        import rbm_amd.data as synth
        from rbm_amd.dataloaders import DeviceBertMasker
        users = synth.user_histories(np.random.default_rng(77 + rank), cfg.get("users", 6040), cfg["T"], cfg["V"],
                                     shape=cfg["shape"])
        sampler = DeviceBertMasker(users, cfg["V"], B, cfg["T"], cfg["mask"], seed=5 + rank)
        sampler.new_epoch()
        capture(lambda s: trainer.capture_sampled(sampler, stamps=stamps, steps_per_graph=s))
        batches = [()]
        run = trainer.replay_sampled
        eager = lambda i: (sampler.sample_into(*trainer.static), trainer.step(*trainer.static))  # noqa: E731
    elif args.no_graph:
        run = trainer.step
    else:
        capture(lambda s: trainer.capture(*batches[0], stamps=stamps, steps_per_graph=s))
        step_batches = batches
        eager = lambda i: trainer.step(*step_batches[i % len(step_batches)])  # noqa: E731
        batches = [torch.stack(b) for b in batches]     # one device copy per replay (replay_packed)
        if S > 1:   # S consecutive batches per replay, still cycling through all of them
            batches = [torch.stack([batches[(j * S + k) % len(batches)] for k in range(S)])
                       for j in range(max(1, len(batches) // S))]
        batches = [(b,) for b in batches]
        run = trainer.replay_packed
    # stamped launches per training step (mark numbering restarts at every unrolled step)
    marks_per_step = len(ops.kernel_stamp_kinds()) if sbuf is not None else 0
    if marks_per_step > NMARK:
        raise SystemExit(f"{marks_per_step} stamped launches per step exceed the stamp buffer's {NMARK} marks")
    # W warmup steps: whole replays, then the remainder (W mod S) as eager steps of the same trainer -- every
    # warmup step is a full training step with its own Adam update
    for i in range(args.warmup // S):
        loss = run(*batches[i % len(batches)])
    for i in range(args.warmup % S):
        loss = eager(i)
    torch.cuda.synchronize()
    replicas_checked = False
    if world > 1:
        # the replicas must hold the same parameter bits after the warmup steps (one all-reduced gradient per
        # step): checks the exchange -- in-graph or segmented -- end to end before anything is timed
        if not trainer.replicas_equal():
            raise SystemExit(f"rank {rank}: data-parallel replicas diverged during warmup")
        replicas_checked = True
        dist.barrier()
    torch.cuda.synchronize()
    if sbuf is not None:
        sbuf.zero_()
        sbuf[:4] = torch.tensor([int(trainer.opt.state[0].item()), args.steps, NMARK, WAVES], dtype=torch.int64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps // S):
        loss = run(*batches[i % len(batches)])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = tt.item()
    final_loss = float(loss.float().reshape(-1)[-1].item())

    live, live_expected = None, None
    if sbuf is not None:
        live = [us for _, _, us in ops.read_kernel_stamps(sbuf, ops.wall_clock_khz())]
        live_expected = args.steps * marks_per_step
        del sbuf
    # the dominant kernel's launch time by HIP events: after the timed steps, training steps of the same trainer run
    # eagerly with a pair of timing events recorded around each of its launches on the stream it runs on (event nodes
    # inside a ROCm graph cost the step a few us each, so they stay out of the timed replays, whose own launches
    # carry the in-kernel stamps above).  A spin kernel first holds the queue while the host issues the whole step,
    # so its launches then run back to back as in a replay and the events see device time only.  Every rank alike
    # (under DP the steps hold the collectives).
    event_us, ev_cost, event_raw = None, None, None
    if not args.no_graph and args.roofline_replays > 0:
        pairs = ops.event_timing((dominant(cfg),))
        empty = []
        try:
            for i in range(args.roofline_replays):
                torch.cuda._sleep(5_000_000)
                # an empty event pair queued the same way: the events' own cost, subtracted from every bracket
                c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                c0.record()
                c1.record()
                empty.append((c0, c1))
                eager(i)
                torch.cuda.synchronize()
        finally:
            ops.event_timing(())
        ev_cost = sorted(c0.elapsed_time(c1) * 1e3 for c0, c1 in empty)[len(empty) // 2]
        event_us = [e0.elapsed_time(e1) * 1e3 - ev_cost for _, e0, e1 in pairs]
        event_raw = sum(e0.elapsed_time(e1) * 1e3 for _, e0, e1 in pairs) / max(1, len(pairs))
    labelled = (sum(float((lab != 0).sum()) for _, lab in host_batches) / len(host_batches)
                if cfg["model"] == "bert" else None)
    roof = roofline(cfg, B, args.dtype, live_us=live, labelled=labelled, live_expected=live_expected,
                    event_us=event_us) if rank == 0 else None
    if roof is not None and event_us:
        roof["event_pair_raw_us"] = round(event_raw, 2)
        roof["event_pair_cost_us"] = round(ev_cost, 2)
    if rank == 0:
        cpu = cpu_baseline(cfg, B, args.cpu_baseline_seconds) if world == 1 and args.cpu_baseline_seconds > 0 \
            else None
        line = {
            "metric": "training sequences/sec, SASRec L=200 d=128 at 1/2/4/8 MI355X; HR@10 parity",
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
            "data": "synthetic (Zipf item ids, ML-1M/Beauty-shaped history lengths, random-init weights); "
                    "HR@10 parity is tested in tests/ (predict + recalls_ndcgs_and_mrr_for_ks)",
            "config": {"workload": cfg["name"], "model": "SASRec" if cfg["model"] == "sas" else "BERT4Rec",
                       "global_batch": world * B, "per_gpu_batch": B, "seq_len": cfg["T"], "hidden": cfg["d"],
                       "blocks": cfg["L"], "heads": cfg["h"], "num_items": cfg["V"], "parallelism": f"dp{world}",
                       "hip_graph": not args.no_graph, "bench_config": args.config,
                       "sampler": args.sampler, "steps_per_graph": S},
            "final_loss": round(final_loss, 5),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if max_lab is not None:
            line["config"]["labelled_rows_cap"] = max_lab
        if vshard:
            line["config"]["vocab_sharded_head"] = True
        if world > 1:
            # every rank compared its parameters with rank 0's after the warmup steps (SystemExit otherwise)
            line["dp"] = {"backend": args.dist_backend, "replicas_equal_after_warmup": replicas_checked,
                          "graph_collectives": bool(trainer.graph_collectives),
                          "sharded_item_table": trainer.rshard is not None}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
