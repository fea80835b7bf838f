"""Structural cost of the data-parallel step on ONE GPU: the bench workload (cfg2 by default, device sampler) as
FusedTrainStep(dp=True) in a world-size-1 RCCL group (RS_DP_GRAPH_COLLECTIVES=0: segment graphs, the bucket
all-reduce issued between replays, a separate optimizer graph; default: the all-reduce inside the step graph) against
the single-GPU step graph (S steps per replay).  The world-1
all-reduce moves no bytes over xGMI, so the difference is what the DP step structure costs per step.
    python tools/dp_overhead.py [cfg2] [steps]"""
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def run(cfg, dp, S, steps):
    import rbm_amd.data as synth
    from rbm_amd.dataloaders import DeviceWarpSampler
    from rbm_amd.train_step import FusedTrainStep
    torch.manual_seed(1234)
    model = bench.make_model(cfg, "bf16")
    model.train()
    tr = FusedTrainStep(model, lr=1e-3, dp=dp)
    users = synth.user_histories(np.random.default_rng(77), cfg.get("users", 6040), cfg["T"], cfg["V"],
                                 shape=cfg["shape"])
    sampler = DeviceWarpSampler(users, cfg["V"], cfg["B"], cfg["T"], seed=5)
    tr.capture_sampled(sampler, steps_per_graph=S)
    for _ in range(20 // S):
        tr.replay_sampled()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // S):
        loss = tr.replay_sampled()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    return ms, float(loss.float().reshape(-1)[-1].item())


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    bench.CFG_NAME = name
    cfg = dict(bench.CONFIGS[name])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    for label, dp, S in (("single, 10 steps/replay", False, 10), ("single, 1 step/replay", False, 1),
                         ("dp world 1, 1 step/replay", True, 1), ("dp world 1, 10 steps/replay", True, 10)):
        ms, loss = run(cfg, dp, S, steps)
        print(f"{name} {label:28s} {ms:.4f} ms/step  loss {loss:.4f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
