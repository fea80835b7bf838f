"""Fused, graph-capturable training step for the SAS / BERT HIP engines.

One call = the reference trainer's inner-loop body (``BS/trainers/base.py:114-123``):
``optimizer.zero_grad(); loss = calculate_loss(batch); loss.backward();
optimizer.step()`` -- every op a HIP kernel on the current stream, no host
synchronisation (the reference's ``loss.item()`` is left to the caller).

Single device: the loss kernels divide by the batch's valid-position count
exactly like the reference's mean (BS/trainers/sas.py:49, BS/trainers/bert.py:40).

Data parallel (one process per GPU, ``torch.distributed`` over RCCL; see
:mod:`rbm_amd.dp`): each rank back-propagates its UNnormalised loss sum, puts
(loss sum, valid count) into the aux tail of its flat gradient buffer, ONE
all-reduce(SUM) of the buffer follows, and the fused Adam divides by the global
count -- the summed gradient then equals the single-device mean's gradient
 and the replicas stay bit-identical.

``capture`` records the step into HIP graphs (one graph on a single device;
compute and optimizer graphs around the eager RCCL call under DP) and
``replay`` runs it on new batches copied into the graphs' static inputs; the
dropout step-seed lives in device memory and is advanced inside the graph.
"""
import gc
import os
import warnings

import torch

from . import dp as dpx
from . import ops
from .engine_util import capture_event, release_capture_events


# thread-local capture: the process group's watchdog thread polls its collectives' events while a step graph is
# being captured, which global capture mode forbids (hipErrorStreamCaptureUnsupported aborts the process)
CAPTURE_MODE = "thread_local"


class FusedAdam:
    """Device-side torch.optim.Adam over a FlatParams buffer (rs_adam_prepare_step / rs_adam_step)."""

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        dev = flat.device
        self.flat = flat
        self.m = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        self.v = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        # [t, lr/bc1, sqrt(bc2), grad scale, -, -, -, arrival counters of rs_adam_prepare_step (state[7],
        # state[16 + 16 k], k < 8)]
        self.state = torch.zeros(144, dtype=torch.float64, device=dev)
        self.hyper = torch.tensor([lr, betas[0], betas[1], eps, weight_decay], dtype=torch.float64, device=dev)
        # (table lo, rows, log2 d, row marks, epoch): a table whose gradient rows only the marked item gradient
        # writes -- the sweep skips the gradient loads of the rows it did not stamp (rs_adam_*_marked)
        self.marks = None

    def _marks(self, lo, hi):
        if self.marks is None:
            return None
        tlo, rows, dshift, rm, ep = self.marks
        if hi <= tlo or lo >= tlo + (rows << dshift):
            return None
        return rm, ep, tlo - lo, rows, dshift

    def set_lr(self, lr):
        """StepLR hook (BS/trainers/base.py:40,87): lives on the device, so graph replays see it."""
        self.hyper[0] = lr

    def step(self, grad_divisor=None, seed_base=None, ranges=None, transposed=None, loss=None, keep=None):
        """One Adam update; also clears the gradient buffer (the next step accumulates from zero) and
        advances the dropout step seed when given.  ranges: [(lo, hi)] flat slices to update (default all; a
        vocabulary-sharded rank skips the output rows other ranks own).  loss = (sum, out): out = sum / grad_divisor
        in the first launch.  transposed (the SAS block weights' transposed bf16 copies) rides in the first range's
        launch, which must cover those matrices.  keep = (lo, hi): a slice the backward OVERWRITES every step
        (BERT's out.weight / out.bias with a large vocabulary): updated by its own launch that leaves its gradient
        in place -- no zero written by this sweep, none read back by the next step's dE GEMM (2 GB per step at 1M
        items)."""
        f = self.flat
        segs = [(lo, hi, True) for lo, hi in (ranges or [(0, f.numel)])]
        if keep is not None and ranges is None:
            klo, khi = keep
            assert 0 < klo < khi <= f.numel and klo % 4 == 0 and khi % 4 == 0, keep
            segs = [(0, klo, True), (klo, khi, False)] + ([(khi, f.numel, True)] if khi < f.numel else [])
        for k, (lo, hi, zg) in enumerate(segs):
            bf = f.bf16[lo:hi] if f.bf16 is not None else None
            if k == 0:   # the first range's launch also prepares the step's scalars (rs_adam_prepare_step)
                ops.adam_prepare_step(f.data[lo:hi], f.grad[lo:hi], self.m[lo:hi], self.v[lo:hi], bf, self.state,
                                      self.hyper, zero_grad=zg, grad_divisor=grad_divisor, seed_base=seed_base,
                                      transposed=transposed, tbase=lo,
                                      loss_sum=loss[0] if loss else None, loss_out=loss[1] if loss else None,
                                      marks=self._marks(lo, hi))
            else:
                ops.adam_step(f.data[lo:hi], f.grad[lo:hi], self.m[lo:hi], self.v[lo:hi], bf, self.state,
                              self.hyper, zero_grad=zg, marks=self._marks(lo, hi))


    def step_keep_early(self, keep, max_wg=None, zero_grad=False, prep_event=None):
        """The first part of a step whose `keep` range is final before the rest of the backward (BERT's out.weight /
        out.bias, after the head's dE / dh): rs_adam_prepare (t += 1 and the step's scalars; no seed advance -- the
        backward still draws this step's dropout masks) and that range's update, gradient left in place.
        step_rest() finishes the step: the same per-element math as step(keep=...), bit for bit."""
        lo, hi = keep
        f = self.flat
        ops.adam_prepare(self.state, self.hyper)
        if prep_event is not None:
            prep_event.record(torch.cuda.current_stream())
        bf = f.bf16[lo:hi] if f.bf16 is not None else None
        ops.adam_step(f.data[lo:hi], f.grad[lo:hi], self.m[lo:hi], self.v[lo:hi], bf, self.state, self.hyper,
                      zero_grad=zero_grad, max_wg=max_wg, marks=self._marks(lo, hi))

    def step_range(self, lo, hi, zero_grad=True, max_wg=None):
        """rs_adam_step over [lo, hi) with the step's scalars already prepared (a step_keep_early step)."""
        f = self.flat
        bf = f.bf16[lo:hi] if f.bf16 is not None else None
        ops.adam_step(f.data[lo:hi], f.grad[lo:hi], self.m[lo:hi], self.v[lo:hi], bf, self.state, self.hyper,
                      zero_grad=zero_grad, max_wg=max_wg, marks=self._marks(lo, hi))

    def step_rest(self, keep, seed_base=None, done=()):
        """The rest of a step_keep_early step: every range outside `keep` and the ranges in `done` (already updated
        by step_range) with the gradient cleared, then the seed."""
        f = self.flat
        cuts = sorted([tuple(keep)] + [tuple(r) for r in done])
        a = 0
        for lo, hi in cuts + [(f.numel, f.numel)]:
            assert lo >= a, (cuts, a)
            if lo > a:
                self.step_range(a, lo)
            a = hi
        if seed_base is not None:
            ops.seed_advance(seed_base)


class FusedStepLR:
    """``torch.optim.lr_scheduler.StepLR(optimizer, step_size, gamma)`` for a FusedAdam (BS/trainers/base.py:40, stepped
    once per epoch at :87): every ``step_size``-th ``step()`` multiplies the learning rate by ``gamma`` -- chained in
    Python floats exactly as torch's StepLR forms it -- and writes it into the optimizer's device hyperparameters, so
    captured step graphs replayed afterwards use it without re-capture."""

    def __init__(self, optimizer, step_size, gamma=0.1):
        self.optimizer = optimizer.opt if isinstance(optimizer, FusedTrainStep) else optimizer
        self.step_size = int(step_size)
        self.gamma = float(gamma)
        self.base_lr = float(self.optimizer.hyper[0].item())
        self.lr = self.base_lr
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        if self.last_epoch % self.step_size == 0:
            self.lr = self.lr * self.gamma
            self.optimizer.set_lr(self.lr)

    def get_last_lr(self):
        return [self.lr]

    def state_dict(self):
        return {"step_size": self.step_size, "gamma": self.gamma, "base_lrs": [self.base_lr],
                "last_epoch": self.last_epoch, "_last_lr": [self.lr]}


class FusedTrainStep:
    def __init__(self, model, lr=1e-3, weight_decay=0.0, process_group=None, dp=None, max_labelled=None,
                 bucket_numel=None, overlap=None, vocab_shard=False, sparse_rows="auto", shard_rows="auto"):
        """model: rbm_amd SASModel or BERTModel on a CUDA device.
        dp: data-parallel mode (default: torch.distributed initialised with world size > 1).
        max_labelled (BERT): upper bound on labelled rows per batch (sizes the compacted
        vocabulary-logit buffers; default B*T).  overlap (DP, default on unless bucket_numel is given): each
        gradient bucket's all-reduce starts as soon as the backward has finished it (dp.BucketedExchange);
        bucket_numel: otherwise ONE all-reduce after the backward, in buckets of that many floats.
        vocab_shard (BERT, DP): out.weight / out.bias sharded over the ranks (rbm_amd.vocab_parallel).
        sparse_rows (BERT, DP with overlap): "auto" (default: when the gathered ids are at most half the table),
        "on" or "off" -- the token table's gradient is exchanged as the union of the rows the ranks touched
        (dp.SparseRowExchange) instead of inside the dense buckets.
        shard_rows (SAS, DP): "auto" (default: when each rank's part of the item table is >= 64k elements, gloo
        only -- off over RCCL until a multi-GPU run verifies it), "on" or "off" -- the item table's optimizer is sharded over the ranks (dp.ShardedRows): its gradient is
        reduce-scattered, each rank updates its part, the compute rows are all-gathered.  The other ranks' parts of
        the fp32 master and Adam moments are then not current on this rank: checkpoint() / gather_shards() gather
        them (needs l2_emb == 0: the regulariser reads every master row)."""
        self.model = model
        self.kind = model.code()
        self.engine = model.sas.engine() if self.kind == "sas" else model.engine()
        self.flat = self.engine.flat
        self.engine.sync_compute_weights()
        self.engine.external_seed = True       # advanced by the optimizer kernel at the end of each step
        if hasattr(self.engine, "adam_transposes"):
            self.engine.adam_transposes = True  # SAS: the optimizer kernel also writes the transposed block weights
        self.flat.grad.zero_()                 # then kept zero by the optimizer (zero_grad)
        self.opt = FusedAdam(self.flat, lr=lr, weight_decay=weight_decay)
        self.pg = process_group
        self.dp = dpx.world() > 1 if dp is None else bool(dp)
        self.bucket_numel = bucket_numel
        self.overlap = self.dp and (bucket_numel is None if overlap is None else bool(overlap))
        if self.dp:
            # dropout masks hash (site salt, step seed, local element index): without a per-rank seed every rank
            # would draw the same masks for its local rows; rank r starts its step seed at r << 40
            import torch.distributed as dist
            r = dist.get_rank(self.pg)
            if r:
                self.engine.seed_base.fill_(r << 40)
        self.vshard = None
        if vocab_shard:
            from .vocab_parallel import VocabShard
            if not (self.dp and self.kind == "bert"):
                raise ValueError("vocab_shard needs a data-parallel BERT step")
            self.vshard = VocabShard(self.flat.shapes["out.weight"][0], self.pg)
            self.engine.vocab_shard = self.vshard
            self.overlap = True
        self.max_labelled = max_labelled
        dev = self.flat.device
        # SAS's parameter-norm regulariser (BS/trainers/sas.py:51-52: loss += l2_emb * ||p|| for every
        # parameter); the BERT trainer has none (BS/trainers/bert.py:30-41)
        self.l2 = float(getattr(model.sas, "l2_emb", 0.0)) if self.kind == "sas" else 0.0
        if self.l2:
            self.l2_desc = ops.l2_chunk_desc(self.flat, dev)
            self.l2_ws = torch.zeros(2 * self.l2_desc.shape[0], dtype=torch.float32, device=dev)
        self.loss_out = torch.zeros(4, dtype=torch.float32, device=dev)
        self.count = torch.zeros(1, dtype=torch.float32, device=dev)
        self.one = torch.ones(1, dtype=torch.float32, device=dev)
        self.loss_val = torch.zeros(1, dtype=torch.float32, device=dev)
        self.graphs = None
        self.static = None
        self.steps_per_graph = 1
        self._stamps = None
        self.rshard = None
        # "auto" stays off over RCCL: its in-place reduce-scatter / all-gather are checked at world size 1 and over
        # gloo with two ranks only (one GPU reaches this builder, and RCCL refuses two ranks on one device), so the
        # sharded form is an explicit opt-in there until a multi-GPU run pins it to the dense exchange
        auto_ok = dpx.backend(self.pg) != "nccl" if self.dp else False
        if self.dp and self.kind == "sas" and shard_rows != "off":
            name = "item_emb.weight"
            n = self.flat.view(name).numel()
            if shard_rows == "on" or (auto_ok and dpx.ShardedRows.worthwhile(n, dpx.world(self.pg))):
                if self.l2:
                    if shard_rows == "on":
                        raise ValueError("shard_rows needs l2_emb == 0 (the regulariser reads every master row)")
                else:
                    self.rshard = dpx.ShardedRows(self.flat, name, self.pg)
        self.exchange = None
        if self.overlap:
            b, extra = self._buckets(), None
            if self.rshard is not None:
                b, extra = dpx.carve(b, self.rshard.lo, self.rshard.hi), {"final": self.rshard.scatter}
            self.exchange = dpx.BucketedExchange(self.flat.grad, b, self.pg, extra=extra,
                                                 partial=self.vshard is not None or self.rshard is not None)
        # Under DP over RCCL the collectives are captured INSIDE the step graph (RCCL collectives are graph
        # capturable; thread-local capture mode lets the process group's watchdog poll meanwhile), so a replay is
        # forward + backward + exchange + Adam with no host round trip, and several steps unroll into one graph as
        # on one device.  A bucket the backward finishes early (BERT's vocabulary head), the vocabulary-sharded
        # head's collectives and the sparse token-table exchange are issued at their point of the captured
        # backward: the collective runs on the process group's stream, forked from the capture stream there and
        # joined before the optimizer, so it overlaps the rest of the backward inside the graph.  Measured on one
        # GPU (world-1 group, tools/dp_overhead.py, SAS cfg2): the segmented form -- step graph, all-reduce issued
        # between replays, optimizer graph -- costs 0.355 against 0.308 ms/step.  RCCL only (gloo's collectives on
        # device tensors synchronise with the host: not capturable); RS_DP_GRAPH_COLLECTIVES=0: the segmented form.
        self.graph_collectives = (self.dp and os.environ.get("RS_DP_GRAPH_COLLECTIVES", "1") != "0"
                                  and dpx.backend(self.pg) == "nccl")
        self.sparse_mode = sparse_rows
        self.sparse = None
        self._sparse_checked = False
        # BERT on one device with a vocabulary whose head gradient the backward overwrites whole (overwritten_grads:
        # the 1M-item head): out.weight / out.bias are final once the head's dE / dh are formed, so their Adam update
        # (256M elements: ~1 ms of HBM streaming at cfg5) runs on a side stream BESIDE the encoder's backward, on a
        # bounded grid, and joins before the rest of the optimizer (RS_EARLY_HEAD_ADAM=0: at the end, as before).
        self._early_kp = None
        self._early_ev = None
        self._early_ok = (self.kind == "bert" and not self.dp and self.vshard is None and not self.l2
                          and os.environ.get("RS_EARLY_HEAD_ADAM", "1") != "0"
                          and hasattr(self.engine, "overwritten_grads"))
        self._opt_stream = torch.cuda.Stream(device=self.flat.device) if self._early_ok else None

        self._early_done = []
        # (below the unzeroed-head vocabulary size -- cfg3's 27k classes -- the early update measured slower: 44.2-44.4k
        # -> 43.6-43.7k seq/s, three interleaved rounds; it runs only with the overwritten-gradient head)
        # ... and the token table's update (256M elements at cfg5) beside the grouped weight gradients: cfg5
        # 7,140 / 7,043 / 7,051 -> 7,144 / 7,167 / 7,195 seq/s (three interleaved rounds)
        self._early_token = self._early_ok and os.environ.get("RS_EARLY_TOKEN_ADAM", "1") != "0"
        # single device, bf16: the item / token table's gradient rows come only from the inverted-index kernels,
        # which stamp the rows they write; the optimizer then reads the gradient of those rows only (4 of its 30
        # bytes per element elsewhere).  Not under data parallel (other ranks' rows arrive by the exchange) nor
        # with the l2 regulariser (it writes every row); tables below ROW_MARKS_MIN rows are mostly touched.
        if (not self.dp and not self.l2 and os.environ.get("RS_ROW_MARKS", "1") != "0"
                and hasattr(self.engine, "enable_row_marks")):
            r = self.engine.enable_row_marks(self.ROW_MARKS_MIN)
            if r is not None:
                name, rm, ep = r
                rows, d = self.flat.shapes[name]
                self.opt.marks = (self.flat.offsets[name], rows, d.bit_length() - 1, rm, ep)

    # ---------------------------------------------------------------- pieces
    def _divisor(self, local_count):
        """Divisor of the loss gradient: the local count (single device, = reference mean) or 1
        (DP: unnormalised; the optimizer divides by the all-reduced global count)."""
        return self.one if self.dp else local_count

    def _buckets(self):
        """Data-parallel all-reduce buckets, {tag: (lo, hi)} of the flat gradient buffer (+ aux tail): the one
        final first (tag named by the engine's split call) and "final" (the rest, after the backward)."""
        f = self.flat
        if self.kind == "sas" and self.engine.fused_head:
            # ONE bucket: the fused SAS backward finishes every gradient in its last launches (the grouped weight
            # gradients with the positional table's, the item table's beside them on the side queue, joined
            # before the step ends), so a dense-block bucket cut there would go out back to back with the tables'
            # -- two collectives' latency and a graph-segment boundary for no overlap (2.65 MB fp32 at cfg2)
            return {"final": (0, f.grad.numel())}
        if self.kind == "bert" and getattr(self, "vshard", None) is not None:
            # the output layer's rows are rank-owned (complete gradients, no exchange); the loss is global already
            return {"final": (0, f.offsets["out.weight"])}
        if self.kind == "bert":
            cut = f.offsets["out.weight"]
            assert f.offsets["out.bias"] > cut and all(o < cut for n, o in f.offsets.items()
                                                       if n not in ("out.weight", "out.bias"))
            return {"final": (0, cut), "out": (cut, f.grad.numel())}
        return {"final": (0, f.grad.numel())}

    def _maybe_sparse(self, tokens):
        """Decide (once, at the first batch: the exchange is sized by its id count) whether the BERT token table's
        gradient goes through dp.SparseRowExchange; if so, carve it out of the dense buckets."""
        if self._sparse_checked:
            return
        self._sparse_checked = True
        if not (self.dp and self.overlap and self.kind == "bert") or self.sparse_mode == "off":
            return
        name = "bert.embedding.token.weight"
        rows, d = self.flat.shapes[name]
        n = tokens.numel()
        if self.sparse_mode == "auto" and not dpx.SparseRowExchange.worthwhile(rows, n, dpx.world(self.pg)):
            return
        self.sparse = dpx.SparseRowExchange(self.flat.view(name, self.flat.grad), n, self.pg)
        self.engine.sparse_tok = self.sparse
        lo = self.flat.offsets[name]
        self.exchange = dpx.BucketedExchange(self.flat.grad, dpx.carve(self._buckets(), lo, lo + rows * d), self.pg,
                                             partial=True)

    def _compute(self, *batch, split=None, update=False):
        # the early optimizer hooks are live only inside this trainer's own steps, whose _update joins them
        # (update=True); a bare forward + backward (tests reading the gradient, the engine driven directly) runs none
        if not (self._early_ok and update):
            return self._compute_impl(*batch, split=split)
        self.engine.after_head_grads = self._early_head_update
        self.engine.after_token_grads = self._early_token_update if self._early_token else None
        done = False
        try:
            out = self._compute_impl(*batch, split=split)
            done = True
            return out
        finally:
            self.engine.after_head_grads = None
            self.engine.after_token_grads = None
            if not done:
                # an aborted compute (e.g. a capture failing after the fork) must not leave a forked update for the
                # next step's _update to join
                self._early_ev = None
                self._early_done = []

    def _compute_impl(self, *batch, split=None):
        """Forward + loss + backward into the flat gradient.  split(tag): called by the engine when the bucket
        `tag` is final (DP only: the aux tail -- loss sum, count -- is written before it).

        The aux tail is written exactly ONCE per step, before the all-reduce of the bucket holding it is issued:
        by sp() when the engine finishes a bucket mid-backward (that bucket's all-reduce may still be running, or
        be done, when the backward returns: writing the local values again then would overwrite the global
        sums), else after the backward, before the all-reduce of the last bucket."""
        eng = self.engine
        sp = None
        aux_written = [False]

        def write_aux():
            if self.dp and not aux_written[0]:
                self.flat.aux[dpx.LOSS_SUM:dpx.COUNT + 1].copy_(self.loss_out[0:2])
                aux_written[0] = True
        if split is not None:
            def sp(tag, action=None):
                if action is None:
                    write_aux()
                split(tag, action)
        if self.kind == "sas":
            seq, pos, neg = batch
            pl, nl, saved = eng.forward(seq, pos, neg, True, clone_seed=False, fuse_head=eng.fused_head,
                                        head_divisor=self.one if self.dp else None)
            if eng.fused_head:
                # BCE forward/backward inside the fused head kernels (head.hip)
                # DP: the loss sum and count go to the buffer's tail in the tail's reduction launch (no copy node)
                if eng.backward(saved, None, None, self.flat.grad, loss_out=self.loss_out,
                                divisor=self.one if self.dp else None,
                                split=sp if self.exchange is not None and "dense" in self.exchange.buckets else None,
                                aux_out=self.flat.aux[dpx.LOSS_SUM:dpx.COUNT + 1] if self.dp else None):
                    aux_written[0] = True
                write_aux()
                return
            ws = eng.ws.get("bce", (3 * 256,), torch.float32)
            ops.bce_fwd(pl, nl, pos, ws, self.loss_out)
            div = self._divisor(self.loss_out[1:2])
            dpl, dnl = eng.ws.get("dpl", pl.shape, torch.float32), eng.ws.get("dnl", nl.shape, torch.float32)
            ops.bce_bwd(pl, nl, pos, div, None, dpl, dnl)
            eng.backward(saved, dpl, dnl, self.flat.grad)
        else:
            tokens, labels = batch
            self._maybe_sparse(tokens)
            if self.sparse is not None and split is None:
                raise RuntimeError("the sparse token-table exchange needs the overlapped (segmented) step")
            eng.train_loss_and_backward(tokens, labels, self.loss_out, self._divisor, self.flat.grad,
                                        max_labelled=self.max_labelled, split=sp)
        write_aux()

    def _exchange(self):
        if not self.dp:
            return
        if self.rshard is None:
            dpx.allreduce_grads(self.flat.grad, self.pg, self.bucket_numel)
            return
        for lo, hi in self.rshard.dense_ranges(self.flat.grad.numel()):
            dpx.allreduce_grads(self.flat.grad[lo:hi], self.pg, self.bucket_numel)
        self.rshard.scatter(async_op=False)

    def _adam_ranges(self):
        if self.rshard is not None:
            return self.rshard.adam_ranges(self.flat.numel)
        if self.vshard is None:
            return None
        f, vs = self.flat, self.vshard
        ow = f.offsets["out.weight"]
        V1, d = f.shapes["out.weight"]
        lo, hi = vs.owned_ranges(ow, d)
        # everything before out.weight, the owned rows, then out.bias (updated whole: 16-B aligned ranges) and on
        return [(0, ow), (lo, hi), (ow + V1 * d, f.numel)]

    def _l2(self, loss, scale=None):
        """The regulariser's loss term and gradient, added after the gradient exchange (every rank adds the same
        term once; `scale` = the divisor the optimizer applies to the summed gradient)."""
        if self.l2:
            ops.l2_penalty(self.flat.data, self.flat.grad, self.l2_desc, self.l2, self.l2_ws, loss=loss, scale=scale)

    def _update(self, post=True):
        """The optimizer (graph-capturable).  post: then the sharded item table's all-gather (_post_update; a
        collective -- the segmented DP graphs run it eagerly after the optimizer's graph instead)."""
        sb = self.engine.seed_base
        if self.vshard is not None:
            # the sharded head normalised by the global count already; the loss is the global batch's
            self.loss_val.copy_(self.loss_out[2:3])
            self.opt.step(seed_base=sb, ranges=self._adam_ranges())
        else:
            tr = self.engine.transposed_spec() if hasattr(self.engine, "transposed_spec") else None
            kp = self.engine.overwritten_grads() if hasattr(self.engine, "overwritten_grads") else None
            if self.dp:
                lsum, cnt = self.flat.aux[dpx.LOSS_SUM:dpx.LOSS_SUM + 1], self.flat.aux[dpx.COUNT:dpx.COUNT + 1]
                rg = self._adam_ranges()
                if self.l2:
                    torch.div(lsum, cnt, out=self.loss_val)
                    self._l2(self.loss_val, scale=cnt)
                    self.opt.step(grad_divisor=cnt, seed_base=sb, transposed=tr, keep=kp, ranges=rg)
                else:   # the loss division rides in the optimizer's launch
                    self.opt.step(grad_divisor=cnt, seed_base=sb, transposed=tr, loss=(lsum, self.loss_val), keep=kp,
                                  ranges=rg)
                if self.rshard is not None:
                    self.rshard.zero_foreign()
                    if post:
                        self._post_update()
            elif self._early_ev is not None:
                assert tr is None and kp in (None, self._early_kp), (kp, self._early_kp)
                cur = torch.cuda.current_stream()
                done, self._early_done = self._early_done, []
                cur.wait_event(self._early_ev)
                self.opt.step_rest(self._early_kp, seed_base=sb, done=done)
                self._early_ev = None
            else:
                self._l2(self.loss_out[2:3])
                self.opt.step(seed_base=sb, transposed=tr, keep=kp)

    def _post_update(self):
        """Sharded item table: all-gather the updated compute rows; the other ranks' master rows are stale now."""
        if self.rshard is not None:
            self.rshard.gather_compute()
            self.flat.stale = self.rshard.stale_ranges()

    # max workgroups of the early out.weight update: a bounded share of the CUs beside the encoder's backward.  cfg5
    # (two interleaved rounds, seq/s): end of step 6,776 / 6,607; early on 128 workgroups 6,573 / 6,444, 256: 7,184 /
    # 7,130, 512: 6,889 / 6,858, 1,024: 6,801 / 6,695 (1,024 took the CUs from the encoder's first backward GEMM)
    EARLY_HEAD_ADAM_WG = int(os.environ.get("RS_EARLY_HEAD_ADAM_WG", "256"))

    EARLY_TOKEN_ADAM_WG = int(os.environ.get("RS_EARLY_TOKEN_ADAM_WG", "256"))

    ROW_MARKS_MIN = 16384

    def _early_token_update(self, name):
        """Engine hook (BERTEngine: right after the token table's gradient, before the grouped weight gradients): that
        range's update follows the early head update on the side stream (same prepared scalars, gradient cleared),
        beside the grouped weight-gradient launch; step_rest skips it.  Returns True when it forked that update."""
        if self._early_ev is None:
            return False
        f = self.flat
        lo = f.offsets[name]
        hi = min(lo + -(-f.view(name).numel() // 4) * 4, f.numel)
        kp = self._early_kp
        if not (hi <= kp[0] or lo >= kp[1]) or lo % 4:
            return False
        ev = capture_event()
        ev.record(torch.cuda.current_stream())
        self._opt_stream.wait_event(ev)
        with torch.cuda.stream(self._opt_stream):
            self.opt.step_range(lo, hi, zero_grad=True, max_wg=self.EARLY_TOKEN_ADAM_WG)
            self._early_ev = capture_event()
            self._early_ev.record(self._opt_stream)
        self._early_done.append((lo, hi))
        return True

    def _early_head_update(self):
        """Engine hook (BERTEngine: right after the head's dE / dh): fork the out.weight / out.bias update onto the
        optimizer's side stream; _update joins it."""
        rng = self.engine.head_grad_range()
        if rng is None:
            return
        # the unzeroed-gradient contract (overwritten_grads) only at large vocabularies: elsewhere the early update
        # clears the range's gradient like the rest of the buffer
        if self.engine.overwritten_grads() is None:
            return
        self._early_kp = rng
        self._early_done = []
        cur = torch.cuda.current_stream()
        ev = capture_event()
        ev.record(cur)
        self._opt_stream.wait_event(ev)
        with torch.cuda.stream(self._opt_stream):
            self.opt.step_keep_early(rng, max_wg=self.EARLY_HEAD_ADAM_WG)
            self._early_ev = capture_event()
            self._early_ev.record(self._opt_stream)

    # ---------------------------------------------------------------- one step
    def step(self, *batch):
        """batch: SAS (seq, pos, neg) / BERT (tokens, labels) int64 device tensors.  Returns the
        device loss (the global batch's mean loss, as the reference's calculate_loss)."""
        if self.overlap:
            self._compute(*batch, split=self._eager_split, update=True)
            self.exchange.launch("final")
            self.exchange.finish()
        else:
            self._compute(*batch, update=True)
            self._exchange()
        self._update()
        return self.loss_val if self.dp else self.loss_out[2:3]

    def replicas_equal(self):
        """Data parallel: True iff every rank holds the same parameter bits (collective; call on every rank).  The
        replicas start equal and every step applies the same all-reduced gradient, so a difference means an
        exchange went wrong (bench.py checks it after its warmup).  Sharded item table: the master outside the
        table and the table's all-gathered compute rows (what every rank's next forward reads)."""
        if not self.dp:
            return True
        if self.rshard is None:
            return dpx.replicas_equal(self.flat.data, self.pg)
        f, rs = self.flat, self.rshard
        cb = f.bf16 if f.bf16 is not None else f.data
        oks = [dpx.replicas_equal(f.data[a:b], self.pg) for a, b in rs.dense_ranges(f.numel)]
        oks.append(dpx.replicas_equal(cb[rs.lo:rs.hi], self.pg))
        return all(oks)

    def gather_shards(self):
        """Make this rank's parameters and Adam moments whole: the vocabulary shards (gather_vocab_shards) and the
        sharded item table's master / moment rows.  Collective: call on every rank."""
        self.gather_vocab_shards()
        if self.rshard is not None:
            torch.cuda.synchronize()
            self.rshard.gather_masters([self.flat.data, self.opt.m, self.opt.v])
            self.flat.stale = []

    def masters_loaded(self):
        """Call after writing the parameters directly (model.load_state_dict on every rank): the fp32 masters are
        whole and current again, and the compute copy is re-derived from them."""
        self.flat.stale = []
        self.engine.sync_compute_weights()

    # ---------------------------------------------------------------- checkpoints
    def _param_slices(self):
        """(nn.Parameter, offset) of every model parameter in the reference's optimizer order
        (model.parameters(), BS/trainers/base.py:225-228); offsets index the flat buffers."""
        base = self.flat.data.data_ptr()
        out = []
        for p in self.model.parameters():
            off = (p.data_ptr() - base) // 4
            if not 0 <= off < self.flat.numel:
                raise RuntimeError("parameter is not a view of the flat buffer")
            out.append((p, off))
        return out

    def optimizer_state_dict(self):
        """The optimizer state in torch.optim.Adam's state_dict() layout (param_groups from a real Adam over
        the same parameters; per-parameter 'step', 'exp_avg', 'exp_avg_sq'), so the reference trainer can
        resume from it (BS/trainers/base.py:255-259, 'optimizer_state_dict').  With the sharded item table and stale
        rows (after a step) this is COLLECTIVE: call it on every rank, not from rank 0 alone."""
        if self.rshard is not None and self.flat.stale:
            self.gather_shards()
        torch.cuda.synchronize()
        hy = self.opt.hyper.cpu().tolist()
        ref = torch.optim.Adam(self.model.parameters(), lr=hy[0], betas=(hy[1], hy[2]), eps=hy[3], weight_decay=hy[4])
        sd = ref.state_dict()
        step = float(self.opt.state[0].item())
        if step > 0:
            for i, (p, off) in enumerate(self._param_slices()):
                n = p.numel()
                sd["state"][i] = {"step": torch.tensor(step),
                                  "exp_avg": self.opt.m[off:off + n].view(p.shape).detach().cpu().clone(),
                                  "exp_avg_sq": self.opt.v[off:off + n].view(p.shape).detach().cpu().clone()}
        return sd

    def load_optimizer_state_dict(self, sd):
        """Resume from a torch.optim.Adam state_dict (e.g. a reference checkpoint's 'optimizer_state_dict')."""
        g = sd["param_groups"][0]
        self.opt.hyper.copy_(torch.tensor([g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"]],
                                          dtype=torch.float64))
        slices = self._param_slices()
        steps = set()
        self.opt.m.zero_()
        self.opt.v.zero_()
        for i, (p, off) in enumerate(slices):
            st = sd["state"].get(i)
            if not st:
                continue
            n = p.numel()
            self.opt.m[off:off + n].copy_(st["exp_avg"].reshape(-1))
            self.opt.v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
            steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError("per-parameter Adam step counts differ; the fused optimizer keeps one")
        self.opt.state.zero_()
        self.opt.state[0] = steps.pop() if steps else 0.0

    def gather_vocab_shards(self):
        """Vocabulary-sharded step: make this rank's out.weight / out.bias (and their Adam moments) hold every
        owner's rows -- the reference layout a checkpoint stores.  Collective: call on every rank."""
        if self.vshard is None:
            return
        torch.cuda.synchronize()
        for name in ("out.weight", "out.bias"):
            for buf in (self.flat.data, self.opt.m, self.opt.v):
                self.vshard.gather_rows(self.flat.view(name, buf))
        self.engine.sync_compute_weights()

    def state_dict(self):
        """model.state_dict() with every row current: under a sharded optimizer (vocabulary / item table) the other
        ranks' fp32 master rows are stale on this rank after a step (flat.stale), so they are gathered first.
        Collective when sharded: call on every rank.  Read the weights through this (or checkpoint()), not through
        model.state_dict() / model.parameters() directly, whenever shard_rows / vocab_shard is on."""
        self.gather_shards()
        return self.model.state_dict()

    def checkpoint(self, epoch=None):
        """{'model_state_dict', 'optimizer_state_dict'[, 'epoch']} as the reference's loggers save it
        (BS/trainers/base.py:255-259, BS/loggers.py:48-58).  Sharded (vocabulary / item table): collective."""
        self.gather_shards()
        d = {"model_state_dict": self.model.state_dict(), "optimizer_state_dict": self.optimizer_state_dict()}
        if epoch is not None:
            d["epoch"] = epoch
        return d

    def load_checkpoint(self, d):
        self.model.load_state_dict(d["model_state_dict"])
        self.masters_loaded()
        self.load_optimizer_state_dict(d["optimizer_state_dict"])

    # ---------------------------------------------------------------- HIP graphs
    def capture(self, *example_batch, warmup=2, stamps=None, steps_per_graph=1):
        """Capture the step into HIP graphs; example_batch fixes the shapes.
        stamps: (int64 device buffer, kind names): the compute graph is captured with kernel stamps enabled
        for those kinds (ops.kernel_stamps against the optimizer's step count), so every replay records the
        begin/end ticks of its rs_attn_bwd / rs_wgrad_grouped launches there (bench.py's in-step timing).
        steps_per_graph=S > 1 (single device): S whole training steps -- each on its own batch, each with its
        own Adam update -- are unrolled into ONE graph, so a replay costs one launch and one input copy per S
        steps; replay_packed() then takes the S batches stacked as [S, n_inputs, ...] and returns the S
        steps' losses."""
        S = self._unroll_check(steps_per_graph)
        # one packed static buffer when the inputs share shape and dtype: replay_packed() then refills
        # all of them with ONE device copy (the bench stacks its batches the same way)
        same = all(t.shape == example_batch[0].shape and t.dtype == example_batch[0].dtype for t in example_batch)
        if S > 1 and not same:
            raise ValueError("steps_per_graph > 1 needs inputs of one shape and dtype (one packed buffer)")
        if same:
            one = torch.stack([t for t in example_batch])
            self.packed = (torch.stack([one] * S) if S > 1 else one).contiguous()
            self.static_steps = [list(p.unbind(0)) for p in (self.packed.unbind(0) if S > 1 else [self.packed])]
            self.static = self.static_steps[0]
        else:
            self.packed = None
            self.static = [t.clone() for t in example_batch]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step(*self.static)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if S > 1:
            self._capture_graphs(self._unrolled(lambda k: self.static_steps[k]), stamps, unrolled=True)
        else:
            self._capture_graphs(lambda split=None: self._compute(*self.static, split=split, update=True), stamps)
        return self

    def _unroll_check(self, steps_per_graph):
        S = int(steps_per_graph)
        if S < 1:
            raise ValueError("steps_per_graph must be >= 1")
        if S > 1 and self.dp and not self.graph_collectives:
            raise ValueError("steps_per_graph > 1 under DP needs the all-reduce inside the graph (graph_collectives)")
        self.steps_per_graph = S
        # one loss-statistics row per unrolled step: the step's kernels write its own row (a copy node between
        # Adam and the next step's first kernel cost ~9 us of idle per step in the graph)
        self.loss_rows = torch.zeros(S, 4, dtype=torch.float32, device=self.flat.device)
        self.loss_steps = self.loss_rows[:, 2]
        return S

    def _unrolled(self, inputs, sample=None):
        """compute() for an unrolled graph: S x (sample, forward + backward, Adam, keep the loss)."""
        def compute(split=None):
            base, base_val = self.loss_out, self.loss_val
            try:
                for k in range(self.steps_per_graph):
                    if k and self._stamps is not None:
                        # restart the stamp marks: each unrolled step records under its own step slot with
                        # marks numbered from 0, so every step's launches fit the per-step mark capacity
                        ops.kernel_stamps(self._stamps[0], self.opt.state, self._stamps[1])
                    self.loss_out = self.loss_rows[k]
                    self.loss_val = self.loss_rows[k, 2:3]    # DP: the global mean loss lands in the step's row
                    if sample is not None:
                        sample()
                    self._compute(*inputs(k), split=self._inline_split(), update=True)
                    self._graph_exchange()
                    self._update()
            finally:
                self.loss_out, self.loss_val = base, base_val
        return compute

    def _inline_split(self):
        """split() for a step whose collectives are captured with it: a bucket's all-reduce (or the computation's
        own collective) is issued right where the backward finishes it (None: no mid-backward exchange)."""
        return self._eager_split if self.graph_collectives and self.overlap else None

    def _graph_exchange(self):
        """DP with graph collectives: the buckets not yet launched mid-backward, then the join, issued inside the
        step being captured."""
        if not self.dp:
            return
        if self.exchange is not None:
            for tag in self.exchange.buckets:
                if tag not in self.exchange.sent:
                    self.exchange.launch(tag)
            self.exchange.finish()
        else:
            self._exchange()

    def _release_graphs(self):
        """Drop every graph (and the exchange's pending work handles) of an earlier capture and let their HIP objects
        go NOW, with no stream capturing: graph executables, their memory pools and the events of earlier eager steps
        are destroyed here, before a new capture begins, instead of whenever Python's collector happens to run --
        a collection that landed mid-capture and destroyed such an object aborted the process once (round 3)."""
        torch.cuda.synchronize()
        self.g_compute = self.g_segments = self.g_update = None
        self.graphs = None
        self._empty_graphs = []
        if self.exchange is not None:
            self.exchange.works, self.exchange.sent = [], []
        gc.collect()
        torch.cuda.synchronize()

    def _capture_graphs(self, compute, stamps=None, unrolled=False):
        """The compute graph (+ the optimizer in the same graph on one device).  DP: the compute graph is cut at
        every bucket the backward finishes (overlap: segments replayed with that bucket's all-reduce launched
        between them) or ends after the backward, and the optimizer is a separate graph after the exchange.
        The previous capture's objects are released explicitly first (_release_graphs); the cyclic collector is
        also held off for the capture itself, so no collection can run while a stream is capturing."""
        self._release_graphs()
        gc_on = gc.isenabled()
        gc.disable()
        try:
            r = self._capture_graphs_impl(compute, stamps, unrolled)
        finally:
            release_capture_events()     # the graphs are instantiated: the capture's fork / join events may go
            if gc_on:
                gc.enable()
        if os.environ.get("RS_GRAPH_UPLOAD", "1") != "0":
            # the executables go to the device now, not at their first replay (hipGraphUpload; preparation only, no
            # step runs): the bench's driver shape (20 timed steps, the first replay inside them) 420.2-420.9k ->
            # 422.0-426.5k seq/s over four interleaved rounds at cfg2
            try:
                for g in self.graphs or ():
                    ops.graph_upload(g)
            except (RuntimeError, AttributeError):   # an optimisation only: a graph that cannot be uploaded replays
                pass
            torch.cuda.synchronize()
        return r

    def _capture_graphs_impl(self, compute, stamps=None, unrolled=False):
        self._stamps = stamps
        if stamps is not None:
            ops.kernel_stamps(stamps[0], self.opt.state, stamps[1])
        try:
            if self.graph_collectives:
                # one graph: compute, the all-reduce, the optimizer (unrolled: S of those)
                err = None
                try:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                        compute(self._inline_split()) if not unrolled else compute()
                        if not unrolled:
                            self._graph_exchange()
                            self._update()
                except Exception as e:   # the collective refused capture on this rank
                    err = e
                torch.cuda.synchronize()
                if self.exchange is not None:
                    self.exchange.works, self.exchange.sent = [], []
                # the ranks agree on the outcome (eager MIN of a flag) before anything else is issued: a rank that
                # fell back alone would run eager / segmented collectives against the others' captured ones.
                # Unverified beyond that flag: after a MIXED outcome the ranks that captured hold collectives that
                # never run (their graphs are dropped), the failed rank fewer; RCCL orders a communicator's
                # collectives by issue, and a captured-but-never-launched one is not expected to take a slot, but
                # no test covers it (every test succeeds or fails on all ranks together).  If that ever misbehaves,
                # re-capture on a fresh process subgroup instead of self.pg.
                if not dpx.agree(err is None, self.pg):
                    self.graph_collectives = False
                    if self.steps_per_graph > 1:   # every rank raises alike; the caller re-captures with S = 1
                        raise RuntimeError(f"all-reduce capture failed on some rank ({err or 'not this one'})")
                    import warnings
                    warnings.warn(f"all-reduce capture failed on some rank ({err or 'not this one'}); falling back "
                                  f"to segmented DP graphs on every rank")
                    return self._capture_graphs_impl(compute, stamps, unrolled)
                self.g_compute = g
                self.g_segments = None
            elif self.overlap:
                self.g_segments = self._capture_segments(compute)
                self.g_compute = None
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                    compute()
                    if not self.dp and not unrolled:
                        self._update()
                self.g_compute = g
                self.g_segments = None
        finally:
            if stamps is not None:
                ops.kernel_stamps(None, None)
            self._stamps = None
        self.g_update = None
        if self.graph_collectives:
            self.graphs = (self.g_compute,)
            return
        if self.dp:
            self.g_update = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_update, capture_error_mode=CAPTURE_MODE):
                self._update(post=False)
        segs = [seg[0] for seg in self.g_segments if seg[0] is not None] if self.g_segments else [self.g_compute]
        self.graphs = tuple(segs) + ((self.g_update,) if self.dp else ())

    def _capture_segments(self, compute):
        """Capture compute(split) as consecutive graphs, a new one begun at every split(tag, action):
        [(graph, tag, action)], the last tagged "final".  At replay, after each graph: its action (a collective of
        the computation) or its bucket's all-reduce.  All segments share one memory pool and one capture stream."""
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        segs, cur = [], [torch.cuda.CUDAGraph()]
        self._empty_graphs = []

        def end():
            # a segment that captured no work (a split point right at the start, e.g. the sparse token-table
            # exchange's id all-gather before the first kernel) is not replayed: its action still runs.  The empty
            # graph object itself is kept alive with the others (destroying it here releases the shared memory
            # pool's use count out of order: torch's caching allocator asserts)
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                cur[0].capture_end()
            empty = any("Graph is empty" in str(x.message) for x in w)
            for x in w:
                if "Graph is empty" not in str(x.message):
                    warnings.warn_explicit(x.message, x.category, x.filename, x.lineno)
            if empty:
                self._empty_graphs.append(cur[0])
                return None
            return cur[0]
        with torch.cuda.stream(s):
            cur[0].capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)

            def split(tag, action=None):
                segs.append((end(), tag, action))
                cur[0] = torch.cuda.CUDAGraph()
                cur[0].capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)
            try:
                compute(split)
            finally:
                last = end()
            segs.append((last, "final", None))
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        return segs

    def _eager_split(self, tag, action=None):
        if action is not None:
            action()
        else:
            self.exchange.launch(tag)

    def _replay_graphs(self):
        if self.graph_collectives:
            self.g_compute.replay()
            if self.rshard is not None:
                self.flat.stale = self.rshard.stale_ranges()
            return self.loss_steps if self.steps_per_graph > 1 else self.loss_val
        if self.overlap:
            for g, tag, action in self.g_segments:
                if g is not None:
                    g.replay()
                if action is not None:
                    action()                  # a collective of the computation itself (vocabulary shards)
                elif tag in self.exchange.buckets:
                    self.exchange.launch(tag)  # RCCL all-reduce of the bucket, overlapping the next segment
            self.exchange.finish()
            self.g_update.replay()
            self._post_update()
            return self.loss_val
        self.g_compute.replay()
        if self.steps_per_graph > 1:
            return self.loss_steps
        if self.dp:
            self._exchange()            # RCCL all-reduce, eager, on the current stream
            self.g_update.replay()
            self._post_update()
        return self.loss_val if self.dp else self.loss_out[2:3]

    def capture_sampled(self, sampler, warmup=2, stamps=None, steps_per_graph=1):
        """Capture sampling (rbm_amd.dataloaders.DeviceWarpSampler for SAS, DeviceBertMasker for BERT, into
        static buffers) together with the step, so ``replay_sampled()`` runs a whole training iteration --
        batch construction included -- as one graph replay (the reference's sampler / DataLoader +
        train_one_epoch body, BS/trainers/base.py:114-123)."""
        want = 3 if self.kind == "sas" else 2
        if getattr(sampler, "n_outputs", None) != want:
            raise ValueError(f"the {self.kind} step needs a sampler producing {want} tensors")
        S = self._unroll_check(steps_per_graph)
        self.sampler = sampler
        shape = (sampler.batch_size, sampler.max_len)
        self.packed = torch.zeros((want,) + shape, dtype=torch.int64, device=self.flat.device)
        self.static = list(self.packed.unbind(0))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                sampler.sample_into(*self.static)
                self.step(*self.static)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

        if S > 1:
            self._capture_graphs(self._unrolled(lambda k: self.static, lambda: sampler.sample_into(*self.static)),
                                 stamps, unrolled=True)
            return self

        def compute(split=None):
            sampler.sample_into(*self.static)
            self._compute(*self.static, split=split, update=True)
        self._capture_graphs(compute, stamps)
        return self

    def replay_sampled(self):
        """One training iteration on a freshly sampled batch (after capture_sampled)."""
        return self._replay_graphs()

    def replay_packed(self, packed):
        """replay() for a batch already stacked as one tensor [n_inputs, ...] (see capture); with
        steps_per_graph=S > 1, S batches stacked as [S, n_inputs, ...] -> the S steps' losses."""
        if self.steps_per_graph > 1 and packed.shape != self.packed.shape:
            raise ValueError(f"replay_packed: expected {tuple(self.packed.shape)} (steps_per_graph batches), "
                             f"got {tuple(packed.shape)}")
        if self.packed is None:
            return self.replay(*packed.unbind(0))
        self.packed.copy_(packed, non_blocking=True)
        return self._replay_graphs()

    def replay(self, *batch):
        if self.steps_per_graph > 1:
            raise ValueError("an unrolled graph (steps_per_graph > 1) replays through replay_packed()")
        for dst, src in zip(self.static, batch):
            dst.copy_(src, non_blocking=True)
        return self._replay_graphs()
