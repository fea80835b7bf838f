"""Fused, graph-capturable training step for the SAS / BERT HIP engines.

One call = the reference trainer's inner-loop body (``BS/trainers/base.py:114-123``):
``optimizer.zero_grad(); loss = calculate_loss(batch); loss.backward();
optimizer.step()`` -- with every op a HIP kernel on the current stream and no
host synchronisation (the reference's ``loss.item()`` is left to the caller).

Data parallel (one process per GPU, ``torch.distributed`` over RCCL):
  1. the loss kernel produces this rank's valid-position count;
  2. one all-reduce of that scalar gives the global count, which is the
     divisor of every rank's loss gradient (so the summed gradients equal the
     single-device mean's gradient exactly);
  3. one all-reduce (SUM) of the flat fp32 gradient buffer, then the fused Adam
     sweep -- identical on every rank, so the replicas stay bit-identical.

The step can be captured once into a HIP graph (``capture``) and replayed
(``replay``) with new batches copied into its static input buffers; the
dropout step-seed lives in device memory and is advanced inside the graph.
"""
import torch
import torch.distributed as dist

from . import ops


class FusedAdam:
    """Device-side torch.optim.Adam over a FlatParams buffer (rs_adam_prepare/step)."""

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        dev = flat.device
        self.flat = flat
        self.m = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        self.v = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        self.state = torch.zeros(4, dtype=torch.float64, device=dev)
        self.hyper = torch.tensor([lr, betas[0], betas[1], eps, weight_decay], dtype=torch.float32, device=dev)

    def set_lr(self, lr):
        self.hyper[0] = lr

    def step(self):
        ops.adam_prepare(self.state, self.hyper)
        ops.adam_step(self.flat.data, self.flat.grad, self.m, self.v, self.flat.bf16, self.state, self.hyper)


class FusedTrainStep:
    def __init__(self, model, lr=1e-3, weight_decay=0.0, process_group=None, dp=None, max_labelled=None):
        """model: rbm_amd SASModel or BERTModel on a CUDA device.  max_labelled (BERT): upper bound
        on labelled rows per batch (sizes the compacted vocabulary-logit buffers; default B*T)."""
        self.model = model
        self.kind = model.code()
        self.engine = model.sas.engine() if self.kind == "sas" else model.engine()
        self.flat = self.engine.flat
        self.engine.sync_compute_weights()
        self.opt = FusedAdam(self.flat, lr=lr, weight_decay=weight_decay)
        self.pg = process_group
        self.dp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 if dp is None else dp
        dev = self.flat.device
        self.loss_out = torch.zeros(4, dtype=torch.float32, device=dev)
        self.count = torch.zeros(1, dtype=torch.float32, device=dev)
        self.graph = None
        self.static = None
        self.max_labelled = max_labelled

    # ---------------------------------------------------------------- one step
    def step(self, *batch):
        """batch: SAS (seq, pos, neg) / BERT (tokens, labels) int64 device tensors.  Returns the
        device loss tensor (this rank's share of the global mean under DP)."""
        self.flat.grad.zero_()
        eng = self.engine
        if self.kind == "sas":
            seq, pos, neg = batch
            pl, nl, saved = eng.forward(seq, pos, neg, True)
            ws = eng.ws.get("bce", (3 * 256,), torch.float32)
            ops.bce_fwd(pl, nl, pos, ws, self.loss_out)
            cnt = self._global_count(self.loss_out[1:2])
            dpl, dnl = torch.empty_like(pl), torch.empty_like(nl)
            ops.bce_bwd(pl, nl, pos, cnt, None, dpl, dnl)
            eng.backward(saved, dpl, dnl, self.flat.grad)
        else:
            tokens, labels = batch
            eng.train_loss_and_backward(tokens, labels, self.loss_out, self._global_count, self.flat.grad,
                                        max_labelled=self.max_labelled)
        if self.dp:
            dist.all_reduce(self.flat.grad, group=self.pg)
        self.opt.step()
        return self.loss_out[0:1] / self.count if self.dp else self.loss_out[2:3]

    def _global_count(self, local_count):
        if not self.dp:
            self.count.copy_(local_count)
            return self.count
        self.count.copy_(local_count)
        dist.all_reduce(self.count, group=self.pg)
        return self.count

    # ---------------------------------------------------------------- HIP graph
    def capture(self, *example_batch, warmup=2):
        """Capture one step into a HIP graph.  example_batch fixes the shapes."""
        self.static = [t.clone() for t in example_batch]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step(*self.static)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_loss = self.step(*self.static)
        return self

    def replay(self, *batch):
        for dst, src in zip(self.static, batch):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_loss
