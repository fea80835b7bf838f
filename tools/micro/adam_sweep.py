"""Standalone Adam sweep rate: rs_adam_step_wg over n fp32 elements (+ bf16 copy) at several workgroup caps.
Usage: python tools/micro/adam_sweep.py [n_millions]   (ranges of >= 64M elements take the nontemporal form)"""
import os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import rbm_amd  # noqa: F401
from rbm_amd import ops

n = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 256 * 1024 * 1024
dev = "cuda"
p = torch.randn(n, device=dev); g = torch.randn(n, device=dev) * 1e-3
m = torch.zeros(n, device=dev); v = torch.zeros(n, device=dev); pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0], dtype=torch.float64, device=dev)
state = torch.zeros(144, dtype=torch.float64, device=dev)
ops.adam_prepare(state, hyper)
nbytes = n * 30
for wg in [256, 512, 1024, 2048, 8192]:
    for _ in range(2):
        ops.adam_step(p, g, m, v, pb, state, hyper, max_wg=wg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.adam_step(p, g, m, v, pb, state, hyper, max_wg=wg)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 5
    print(f"n={n} wg={wg}: {us:.1f} us  {nbytes / us / 1e6:.2f} TB/s", flush=True)
