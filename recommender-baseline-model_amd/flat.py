"""Flat parameter storage: every model parameter is a view into ONE fp32 buffer.

Why: Adam becomes one fused kernel over one buffer (rs_adam_step), the
data-parallel gradient all-reduce is one contiguous RCCL call (or a few
buckets), and the bf16 weight copy the MFMA GEMMs read is one cast.  The
``nn.Parameter`` objects (and so ``state_dict()`` keys/shapes) are exactly the
reference's; only their storage is shared.  Each region starts on a 64-element
(256-byte) boundary so every kernel can use 16-byte vector accesses.
"""
import torch
import torch.nn as nn

ALIGN = 64
AUX = 64   # fp32 scalars riding at the tail of the gradient buffer (DP: loss sum, valid count)


class FlatParams:
    def __init__(self, module: nn.Module, device, order=None):
        """order: optional callable(list of names) -> the same names in storage order (e.g. to keep the
        q/k/v projection weights of a block adjacent so that one GEMM computes all three)."""
        named = list(module.named_parameters())
        if order is not None:
            pos = {n: i for i, (n, _) in enumerate(named)}
            names = order([n for n, _ in named])
            assert sorted(names) == sorted(pos), "order() must permute the parameter names"
            named = [named[pos[n]] for n in names]
        self.names = [n for n, _ in named]
        self.shapes = {n: tuple(p.shape) for n, p in named}
        self.offsets = {}
        off = 0
        for n, p in named:
            self.offsets[n] = off
            off += -(-p.numel() // ALIGN) * ALIGN
        self.numel = off
        self.device = torch.device(device)
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        # the gradient buffer carries AUX extra floats after the parameters: the data-parallel step
        # puts its local loss sum and valid-position count there, so ONE all-reduce sums both
        self.grad = torch.zeros(self.numel + AUX, dtype=torch.float32, device=self.device)
        self.aux = self.grad[self.numel:]
        self.bf16 = None
        # ranges of the fp32 master that are not current on this rank (a data-parallel step that shards a table's
        # optimizer, dp.ShardedRows: the compute copy of those rows was all-gathered, the master was not)
        self.stale = []
        for n, p in named:
            if p.dtype != torch.float32:
                raise TypeError(f"parameter {n} must be fp32 (master weights), got {p.dtype}")
            self.view(n).copy_(p.detach().to(self.device))
        self.rebind(module)

    def view(self, name, buf=None):
        buf = self.data if buf is None else buf
        o = self.offsets[name]
        shp = self.shapes[name]
        n = 1
        for s in shp:
            n *= s
        return buf[o:o + n].view(shp)

    def gview(self, name):
        return self.view(name, self.grad)

    def cview(self, name):
        """compute-dtype view (bf16 copy when present, else fp32 master)."""
        return self.view(name, self.bf16 if self.bf16 is not None else self.data)

    def rebind(self, module: nn.Module):
        """Point every registered nn.Parameter of ``module`` at its flat-buffer view."""
        for n in self.names:
            *path, leaf = n.split(".")
            m = module
            for part in path:
                m = getattr(m, part)
            old = getattr(m, leaf)
            newp = nn.Parameter(self.view(n), requires_grad=old.requires_grad)
            setattr(m, leaf, newp)

    def enable_bf16(self):
        if self.bf16 is None:
            self.bf16 = torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device)

    def adjacent(self, names):
        """True when the listed parameters are stored back to back (one contiguous region)."""
        off = self.offsets[names[0]]
        for n in names:
            if self.offsets[n] != off:
                return False
            k = 1
            for s in self.shapes[n]:
                k *= s
            off += k
        return True

    def span(self, names, buf=None, rows=None):
        """A 2-D view over adjacent parameters (concatenated along dim 0)."""
        assert self.adjacent(names), names
        buf = self.data if buf is None else buf
        o = self.offsets[names[0]]
        n = sum(self.shapes[k][0] for k in names)
        inner = 1
        for s in self.shapes[names[0]][1:]:
            inner *= s
        t = buf[o:o + n * inner]
        return t.view(n, inner) if inner > 1 else t

    def is_bound(self, module: nn.Module):
        for n, p in module.named_parameters():
            if n not in self.offsets:
                return False
            v = self.view(n)
            if p.data_ptr() != v.data_ptr() or p.device != v.device:
                return False
        return True
