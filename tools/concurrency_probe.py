#!/usr/bin/env python
"""Probe: do two half-batch SAS train steps on two streams overlap on the GPU (latency-bound kernels)?
Times (a) one FusedTrainStep graph at B, (b) two independent FusedTrainStep graphs at B/2 replayed on two
streams concurrently, (c) the same two replayed back to back on one stream."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    cfg = dict(bench.CONFIGS[a.config])
    B = cfg["B"]
    from rbm_amd.train_step import FusedTrainStep

    def trainer(b):
        torch.manual_seed(0)
        m = bench.make_model(cfg, "bf16")
        batch = [torch.from_numpy(x).cuda() for x in bench.make_batches(cfg, b, 1, 3)[0]]
        t = FusedTrainStep(m, lr=1e-3)
        t.capture(*batch)
        return t

    def timeit(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e6

    full = trainer(B)
    h1, h2 = trainer(B // 2), trainer(B // 2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def two_streams():
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        with torch.cuda.stream(s1):
            h1.g_compute.replay()
        with torch.cuda.stream(s2):
            h2.g_compute.replay()
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

    def one_stream():
        h1.g_compute.replay()
        h2.g_compute.replay()

    print(f"full B={B}: {timeit(lambda: full.g_compute.replay()):.1f} us/step")
    print(f"2 x B={B // 2}, one stream: {timeit(one_stream):.1f} us")
    print(f"2 x B={B // 2}, two streams: {timeit(two_streams):.1f} us")
    print(f"1 x B={B // 2}: {timeit(lambda: h1.g_compute.replay()):.1f} us")


if __name__ == "__main__":
    main()
