"""Adam oracle (TEST INFRASTRUCTURE ONLY).

Restates ``torch.optim.Adam`` (single-tensor path, amsgrad=False) as the
reference constructs it in ``BS/trainers/base.py:225-228``
(``optim.Adam(params, lr=args.lr, weight_decay=args.weight_decay)``, betas
(0.9, 0.999), eps 1e-8).  Bias corrections are formed in double precision on
the host, exactly like torch does with Python floats.
"""
import math

import torch


class AdamOracle:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.params = list(params)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self, grads):
        self.t += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        step_size = self.lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        for p, g, m, v in zip(self.params, grads, self.m, self.v):
            if self.wd != 0:
                g = g + self.wd * p
            m.lerp_(g, 1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / bc2_sqrt).add_(self.eps)
            p.addcdiv_(m, denom, value=-step_size)
