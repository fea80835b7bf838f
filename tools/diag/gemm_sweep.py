"""Epilogue-cost sweep of the bf16 GEMM at the BERT FFN shape (M=12800, K=256, N=1024)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
import rbm_amd  # noqa
from rbm_amd import ops
sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
from kbench import timeit
dev = "cuda"
M, K, N = int(os.environ.get("M", 12800)), int(os.environ.get("K", 256)), int(os.environ.get("N", 1024))
x = torch.randn(M, K, device=dev).bfloat16()
W = torch.randn(N, K, device=dev).bfloat16()
b = torch.randn(N, device=dev)
y = torch.empty(M, N, device=dev).bfloat16()
aux = torch.empty(M, N, device=dev).bfloat16()
yf = torch.empty(M, N, device=dev)
sb = torch.zeros(1, dtype=torch.int64, device=dev)
cases = [("plain", lambda: ops.linear_fwd(x, W, y)),
         ("bias", lambda: ops.linear_fwd(x, W, y, bias=b)),
         ("bias gelu", lambda: ops.linear_fwd(x, W, y, bias=b, act=ops.ACT_GELU)),
         ("bias gelu aux", lambda: ops.linear_fwd(x, W, y, bias=b, act=ops.ACT_GELU, aux_out=aux)),
         ("bias gelu aux drop", lambda: ops.linear_fwd(x, W, y, bias=b, act=ops.ACT_GELU, aux_out=aux, drop_p=0.1,
                                                       drop_seed=3, seed_base=sb, drop_ld=N)),
         ("bias drop", lambda: ops.linear_fwd(x, W, y, bias=b, drop_p=0.1, drop_seed=3, seed_base=sb, drop_ld=N)),
         ("fp32 out bias", lambda: ops.linear_fwd(x, W, yf, bias=b))]
for name, fn in cases:
    us = timeit(fn, 50)
    print(f"{name:24s} {us:8.2f} us  {2*M*N*K/us/1e6:7.1f} TFLOP/s")
