"""SASRec on the MI355X HIP path.

Same constructor arguments, parameter modules, initialisation and
``state_dict`` keys as the reference ``BS/models/sas_model/sas.py:23-57`` (the
torch modules below are only parameter containers and initialisers: they never
run), same ``forward``/``predict`` results (``sas.py:59-118``).  The math runs
as HIP kernels through the C ABI, orchestrated by :class:`SASEngine`:

bf16 fused step (FusedTrainStep, d in {64, 128}: the benchmarked path) -- per block two row-chain kernels per
direction (rowchain.hip: one workgroup per CU, the block's three d x d weights in LDS, each wave carrying 16-token
tiles through the sublayer chain in registers) around the LDS-resident attention (attention_lds.hip):
  x = emb*sqrt(d)+pos, drop, mask;  Q = LN1(x);      rs_sas_block_in_embed (first block) / rs_sas_block_in
  q = Q Wq^T+bq;  kv = x Wkv^T+bkv                   (same launch; sas.py:59-67, 73-76)
  o = attn(q, k, v) causal, dropout on P             rs_attn_fwd (mask_kind 0; sas.py:75)
  x1 = Q + o Wo^T + bo;  z = LN2(x1);                rs_sas_block_out (sas.py:75-84, PointWiseFeedForward)
  x = (drop(relu(drop(z W1^T+b1)) W2^T+b2) + z)*m    (same launch)
  f = LN(x); pl/nl = <f, E[pos/neg]>; BCE + grads   rs_sas_block_out_head (the last block's output kernel)
backward: rs_sas_block_out_bwd_delta -> rs_attn_bwd (dQ and dK/dV workgroups in one launch) ->
rs_sas_block_in_bwd per block, then ONE grouped launch of every weight / bias / LayerNorm-affine gradient
(rs_wgrad_grouped_pos_stats, with the positional table's gradient and the loss statistics) beside the item-table
gradient by inverted index (rs_item_index_build on a side stream during the forward, rs_item_grad), then the fused
Adam (rs_adam_prepare_step_loss).
fp32 parity mode and other widths run the generic unfused kernels: rs_embed_fwd, rs_layernorm_fwd/bwd (variant 0,
eps 1e-8), rs_gemm (MFMA, fused bias / ReLU / dropout / residual / row-mask epilogues), rs_attn_fwd/bwd,
rs_sampled_logits_fwd/bwd, rs_bce_*, split-K weight gradients.
"""
import math

import torch
import torch.nn as nn

from ... import ops
from ...engine_util import Workspace, as_ids, capture_event, compute_dtype, require_cuda, site_salt
from ...flat import FlatParams

LN_EPS = 1e-8


class PointWiseFeedForward(nn.Module):
    """Parameter container mirroring ``sas.py:6-14`` (conv1 / conv2 = Conv1d(d, d, 1))."""

    def __init__(self, hidden_units, dropout_rate):
        super().__init__()
        self.conv1 = nn.Conv1d(hidden_units, hidden_units, kernel_size=1)
        self.conv2 = nn.Conv1d(hidden_units, hidden_units, kernel_size=1)
        self.dropout_rate = dropout_rate


class SAS(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.item_num = args.num_items
        self.device = args.device
        self.max_len = args.max_len
        self.hidden = args.sas_hidden_units
        self.num_blocks = args.sas_num_blocks
        self.heads = args.sas_heads
        self.dropout_rate = args.sas_dropout
        # the trainer's l2 regulariser weight (BS/trainers/sas.py:14,51-52), applied by FusedTrainStep
        self.l2_emb = float(getattr(args, "l2_emb", 0.0) or 0.0)
        self.cdtype = compute_dtype(args)
        d = self.hidden
        if d % self.heads:
            raise ValueError("sas_hidden_units must be divisible by sas_heads")

        self.item_emb = nn.Embedding(self.item_num + 1, d, padding_idx=0)
        self.pos_emb = nn.Embedding(args.max_len, d)
        self.attention_layernorms = nn.ModuleList()
        self.attention_layers = nn.ModuleList()
        self.forward_layernorms = nn.ModuleList()
        self.forward_layers = nn.ModuleList()
        self.last_layernorm = nn.LayerNorm(d, eps=LN_EPS)
        for _ in range(self.num_blocks):
            self.attention_layernorms.append(nn.LayerNorm(d, eps=LN_EPS))
            self.attention_layers.append(nn.MultiheadAttention(d, self.heads, self.dropout_rate))
            self.forward_layernorms.append(nn.LayerNorm(d, eps=LN_EPS))
            self.forward_layers.append(PointWiseFeedForward(d, self.dropout_rate))

        self._flat = None
        self._engine = None
        if torch.device(self.device).type == "cuda":
            self.to(self.device)

    # ---- flat-buffer management ------------------------------------------------------
    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        p = next(self.parameters())
        self._flat = FlatParams(self, p.device) if p.device.type == "cuda" else None
        self._engine = None
        return self

    def engine(self):
        p = self.item_emb.weight
        require_cuda(p.device)
        if self._flat is None or not self._flat.is_bound(self):
            self._flat = FlatParams(self, p.device)
            self._engine = None
        if self._engine is None:
            self._engine = SASEngine(self, self._flat)
        return self._engine

    # ---- reference API ---------------------------------------------------------------
    def forward(self, log_seqs, pos_seqs, neg_seqs):
        eng = self.engine()
        dev = self._flat.device
        ids, pos, neg = as_ids(log_seqs, dev), as_ids(pos_seqs, dev), as_ids(neg_seqs, dev)
        params = [p for _, p in self.named_parameters()]
        return _SASFunction.apply(eng, ids, pos, neg, self.training, *params)

    def log2feats(self, log_seqs):
        eng = self.engine()
        ids = as_ids(log_seqs, self._flat.device)
        with torch.no_grad():
            return eng.features(ids).clone()

    @torch.no_grad()
    def predict(self, log_seqs, item_indices):
        eng = self.engine()
        dev = self._flat.device
        return eng.predict(as_ids(log_seqs, dev), as_ids(item_indices, dev))


class _SASFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, ids, pos, neg, training, *params):
        engine.sync_compute_weights()
        pl, nl, saved = engine.forward(ids, pos, neg, training)
        ctx.engine = engine
        ctx.saved = saved
        return pl, nl

    @staticmethod
    def backward(ctx, dpl, dnl):
        eng = ctx.engine
        grad = torch.zeros(eng.flat.numel, dtype=torch.float32, device=eng.flat.device)
        eng.backward(ctx.saved, dpl.contiguous().float(), dnl.contiguous().float(), grad)
        ctx.saved = None
        grads = [eng.flat.view(n, grad) for n in eng.flat.names]
        return (None, None, None, None, None, *grads)


class SASEngine:
    """Owns workspaces and issues the HIP kernels of one SAS model."""

    def __init__(self, model: SAS, flat: FlatParams):
        self.m = model
        self.flat = flat
        self.d = model.hidden
        self.L = model.num_blocks
        self.H = model.heads
        self.Dh = self.d // self.H
        self.p = float(model.dropout_rate)
        self.dt = model.cdtype
        self.dev = flat.device
        if self.dt == torch.bfloat16:
            flat.enable_bf16()
        self.ws = Workspace(self.dev)
        self.seed_base = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.external_seed = False    # True: the fused train step's optimizer advances seed_base
        # True: the fused train step's optimizer also writes the transposed bf16 block weights (transposed_spec),
        # so the forward's side branch builds only the item index and the backward needs no join for it
        self.adam_transposes = False
        self._wT = None
        salt0 = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.salt = {"emb": site_salt(salt0, 0)}
        for i in range(self.L):
            self.salt[f"attn{i}"] = site_salt(salt0, 1 + 4 * i)
            self.salt[f"ffn1_{i}"] = site_salt(salt0, 2 + 4 * i)
            self.salt[f"ffn2_{i}"] = site_salt(salt0, 3 + 4 * i)

    # compute-dtype weights
    def sync_compute_weights(self):
        f = self.flat
        if f.bf16 is not None:
            if not f.stale:
                ops.cast_bf16(f.data, f.bf16)
            else:   # the compute copy of stale master rows (a sharded item table) is the current one: keep it
                a = 0
                for lo, hi in sorted(f.stale) + [(f.numel, f.numel)]:
                    if lo > a:
                        ops.cast_bf16(f.data[a:lo], f.bf16[a:lo])
                    a = max(a, hi)
            if self._wT is not None:
                self._refresh_transposed()

    def transposed_spec(self):
        """(desc, host desc, destination) of the backward's transposed block weights, for an optimizer that
        writes them itself (rs_adam_prepare_step; adam_transposes=True), or None before they exist."""
        if not self.adam_transposes or self._wT is None:
            return None
        return self._wT_desc, self._wT_desc_host, self._wT

    def W(self, n):
        return self.flat.cview(n)

    def Wf(self, n):
        return self.flat.view(n)

    def _buf(self, name, shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.dt, device=self.dev)

    # ---- forward -------------------------------------------------------------------
    def forward(self, ids, pos, neg, training, need_logits=True, clone_seed=True, fuse_head=False,
                head_divisor=None):
        """fuse_head (the fused training step, whose backward forms the BCE gradient itself): the head's forward
        and backward run as one pass per token inside the last block's output kernel (rs_sas_block_out_head); the
        returned pl / nl are filled by then.  The first block's input kernel counts the valid positions (the BCE
        divisor) for it; head_divisor (device scalar, data parallel: 1) replaces that count and must be the divisor
        later passed to backward."""
        B, T = ids.shape
        M, d, H, Dh, L = B * T, self.d, self.H, self.Dh, self.L
        p = self.p if training else 0.0
        if p > 0 and not self.external_seed:
            ops.seed_advance(self.seed_base)
        # this step's masks, replayed by backward (the fused step runs backward before the next
        # advance, so it reads the live word; the autograd API may interleave forwards: snapshot)
        sb = self.seed_base.clone() if clone_seed else self.seed_base
        e = self._buf
        s = {"B": B, "T": T, "p": p, "ids": ids, "pos": pos, "neg": neg, "sb": sb,
             "x": [], "Q": [], "mu1": [], "r1": [], "q": [], "kv": [], "o": [], "lse": [],
             "x1": [], "z": [], "mu2": [], "r2": [], "h1": []}
        fused = ops.sas_block_fused_ok(d, self.dt)
        side = fused and training and pos is not None
        if side:
            fork = capture_event()
            fork.record()
        x = e("x0", (M, d))
        # the fused training step: the head's forward and backward inside the last block's output kernel, the
        # embedding stage inside the first block's input kernel, which counts the valid positions (the BCE divisor)
        fuse_head = fuse_head and side and need_logits
        cntp = None
        if fuse_head:
            cntp = self.ws.get("cntp", (ops.sas_block_in_count_parts(M),), torch.int32)
            s["cntp"] = cntp
        emb = None
        if fused:
            emb = (ids, T, self.W("item_emb.weight"), self.W("pos_emb.weight"), math.sqrt(d), p, self.salt["emb"], sb,
                   x, pos if cntp is not None else None, cntp)
        else:
            ops.embed_fwd(0, ids, T, self.W("item_emb.weight"), self.W("pos_emb.weight"), math.sqrt(d), p,
                          self.salt["emb"], sb, x)

        def after_first():
            if side:
                # issued after the first forward launch: in the captured graph the forward chain is then the
                # first child of the step's root and keeps the launch queue; the side branch gets the second
                s["side"] = self._side_prologue(ids, pos, neg, after=fork)
        head = None
        if cntp is not None:
            # the head inside the last block's output kernel: its outputs, per-workgroup partials
            Gb = ops.sas_block_grid(M)
            f32 = torch.float32
            s.update(head_in_block=True, hdiv=head_divisor, f=e("f", (M, d)), pl=e("pl", (B, T), f32),
                     nl=e("nl", (B, T), f32), dpl=e("dpl", (B, T), f32), dnl=e("dnl", (B, T), f32),
                     hdx=e("dx", (M, d)), lnh=self.ws.get("lnh_blk", (2 * d * Gb,), f32),
                     headp=e("headp", (3 * Gb,), f32))
            head = (self.W("item_emb.weight"), pos, neg, self.Wf("last_layernorm.weight"),
                    self.Wf("last_layernorm.bias"), cntp, head_divisor, s["f"], s["pl"], s["nl"], s["dpl"], s["dnl"],
                    s["hdx"], s["lnh"], s["headp"])
        if fused:
            x = self._forward_blocks_fused(s, x, emb=emb, after_first=after_first, head=head)
        else:
            for i in range(L):
                pre = f"attention_layers.{i}."
                Q, mu1, r1 = e("Q", (M, d)), e("mu", (M,), torch.float32), e("r", (M,), torch.float32)
                Win, bin_ = self.W(pre + "in_proj_weight"), self.Wf(pre + "in_proj_bias")
                q, kv = e("q", (M, d)), e("kv", (M, 2 * d))
                o, lse = e("o", (M, d)), e("lse", (B * H * T,), torch.float32)
                x1 = e("x1", (M, d))
                z, mu2, r2 = e("z", (M, d)), e("mu", (M,), torch.float32), e("r", (M,), torch.float32)
                fw = f"forward_layers.{i}."
                h1, xn = e("h1", (M, d)), e("x", (M, d))
                ops.layernorm_fwd(x, self.Wf(f"attention_layernorms.{i}.weight"),
                                  self.Wf(f"attention_layernorms.{i}.bias"), LN_EPS, Q, mu1, r1, 0)
                ops.linear_fwd(Q, Win[:d], q, bias=bin_[:d])
                ops.linear_fwd(x, Win[d:], kv, bias=bin_[d:])
                ops.attn_fwd(B, T, H, Dh, q, kv[:, :d], kv[:, d:], o, lse, 1.0 / math.sqrt(Dh), 0, ids, p,
                             self.salt[f"attn{i}"], sb)
                ops.linear_fwd(o, self.W(pre + "out_proj.weight"), x1, bias=self.Wf(pre + "out_proj.bias"), resid=Q)
                ops.layernorm_fwd(x1, self.Wf(f"forward_layernorms.{i}.weight"),
                                  self.Wf(f"forward_layernorms.{i}.bias"), LN_EPS, z, mu2, r2, 0)
                ops.linear_fwd(z, self.W(fw + "conv1.weight").view(d, d), h1, bias=self.Wf(fw + "conv1.bias"),
                               act=ops.ACT_RELU, drop_p=p, drop_seed=self.salt[f"ffn1_{i}"], seed_base=sb, drop_ld=d)
                ops.linear_fwd(h1, self.W(fw + "conv2.weight").view(d, d), xn, bias=self.Wf(fw + "conv2.bias"),
                               drop_p=p, drop_seed=self.salt[f"ffn2_{i}"], seed_base=sb, drop_ld=d, resid=z,
                               rowmask_ids=ids)
                for k_, v_ in (("x", x), ("Q", Q), ("mu1", mu1), ("r1", r1), ("q", q), ("kv", kv), ("o", o),
                               ("lse", lse), ("x1", x1), ("z", z), ("mu2", mu2), ("r2", r2), ("h1", h1)):
                    s[k_].append(v_)
                x = xn
        if "head_in_block" in s:
            s.update(xL=x)
            return s["pl"], s["nl"], s
        f, muf, rf = e("f", (M, d)), e("mu", (M,), torch.float32), e("r", (M,), torch.float32)
        s.update(xL=x, f=f, muf=muf, rf=rf)
        if fused and need_logits:
            # last LayerNorm + tied sampled logits + BCE partial sums in one kernel (head.hip)
            pl, nl = e("pl", (B, T), torch.float32), e("nl", (B, T), torch.float32)
            headp = e("headp", (3 * (-(-M // 64)),), torch.float32)
            ops.sas_head_fwd(x, self.Wf("last_layernorm.weight"), self.Wf("last_layernorm.bias"), LN_EPS, f, muf, rf,
                             self.W("item_emb.weight"), pos, neg, pl, nl, headp)
            s.update(pl=pl, nl=nl, headp=headp)
            return pl, nl, s
        ops.layernorm_fwd(x, self.Wf("last_layernorm.weight"), self.Wf("last_layernorm.bias"), LN_EPS, f, muf, rf, 0)
        if not need_logits:
            return None, None, s
        pl, nl = e("pl", (B, T), torch.float32), e("nl", (B, T), torch.float32)
        ops.sampled_logits_fwd(f, self.W("item_emb.weight"), pos, neg, pl, nl)
        return pl, nl, s

    def _forward_blocks_fused(self, s, x, emb=None, after_first=None, head=None):
        """SAS blocks' forward with the row-chain kernels (rowchain.hip) on each side of the attention core
        (rs_sas_block_in, rs_attn_fwd, rs_sas_block_out per block).  Fills s's per-block saved tensors; returns the
        last block's output.  emb: sas_block_in_embed's embedding arguments (x is then its x0 output, formed by the
        first launch); after_first(): called after the first launch; head: sas_block_out_head's head arguments
        (the last block's output kernel then also runs the SAS head)."""
        B, T, p, ids, sb = s["B"], s["T"], s["p"], s["ids"], s["sb"]
        M, d, H, Dh, L = B * T, self.d, self.H, self.Dh, self.L
        e = self._buf
        f32 = torch.float32
        lay = [dict(Q=e("Q", (M, d)), mu1=e("mu", (M,), f32), r1=e("r", (M,), f32), q=e("q", (M, d)),
                    kv=e("kv", (M, 2 * d)), o=e("o", (M, d)), lse=e("lse", (B * H * T,), f32), x1=e("x1", (M, d)),
                    z=e("z", (M, d)), mu2=e("mu", (M,), f32), r2=e("r", (M,), f32), h1=e("h1", (M, d)),
                    xn=e("x", (M, d))) for _ in range(L)]

        def in_args(i):
            pre = f"attention_layers.{i}."
            Win, bin_ = self.W(pre + "in_proj_weight"), self.Wf(pre + "in_proj_bias")
            b = lay[i]
            return (self.Wf(f"attention_layernorms.{i}.weight"), self.Wf(f"attention_layernorms.{i}.bias"),
                    b["Q"], b["mu1"], b["r1"], Win[:d], bin_[:d], b["q"], Win[d:], bin_[d:], b["kv"])

        def out_args(i):
            pre, fw, b = f"attention_layers.{i}.", f"forward_layers.{i}.", lay[i]
            return (b["o"], b["Q"], self.W(pre + "out_proj.weight"), self.Wf(pre + "out_proj.bias"), b["x1"],
                    self.Wf(f"forward_layernorms.{i}.weight"), self.Wf(f"forward_layernorms.{i}.bias"), LN_EPS,
                    b["z"], b["mu2"], b["r2"], self.W(fw + "conv1.weight"), self.Wf(fw + "conv1.bias"), b["h1"],
                    self.W(fw + "conv2.weight"), self.Wf(fw + "conv2.bias"), b["xn"], ids, p,
                    self.salt[f"ffn1_{i}"], self.salt[f"ffn2_{i}"], sb)

        ln_w, ln_b, Q, mu1, r1, Wq, bq, q, Wkv, bkv, kv = in_args(0)
        if emb is not None:
            ops.sas_block_in_embed(*emb, ln_w, ln_b, LN_EPS, Q, mu1, r1, Wq, bq, q, Wkv, bkv, kv)
        else:
            ops.sas_block_in(x, ln_w, ln_b, LN_EPS, Q, mu1, r1, Wq, bq, q, Wkv, bkv, kv)
        if after_first is not None:
            after_first()
        xs = [x]
        for i in range(L):
            b = lay[i]
            ops.attn_fwd(B, T, H, Dh, b["q"], b["kv"][:, :d], b["kv"][:, d:], b["o"], b["lse"], 1.0 / math.sqrt(Dh),
                         0, ids, p, self.salt[f"attn{i}"], sb)
            if head is not None and i == L - 1:
                ops.sas_block_out_head(out_args(i), *head)
            else:
                ops.sas_block_out(*out_args(i))
            if i + 1 < L:
                ln_w, ln_b, Q, mu1, r1, Wq, bq, q, Wkv, bkv, kv = in_args(i + 1)
                ops.sas_block_in(b["xn"], ln_w, ln_b, LN_EPS, Q, mu1, r1, Wq, bq, q, Wkv, bkv, kv)
            xs.append(b["xn"])
        for i in range(L):
            b = lay[i]
            for k_ in ("Q", "mu1", "r1", "q", "kv", "o", "lse", "x1", "z", "mu2", "r2", "h1"):
                s[k_].append(b[k_])
            s["x"].append(xs[i])
        return xs[L]

    @property
    def fused_head(self):
        """True when forward/backward take the fused bf16 path (head.hip, rowchain.hip, itemgrad.hip)."""
        return ops.sas_block_fused_ok(self.d, self.dt)

    # ---- backward ------------------------------------------------------------------
    def backward(self, s, dpl, dnl, grad, loss_out=None, divisor=None, split=None, aux_out=None):
        """Accumulates every parameter gradient into the flat fp32 buffer ``grad``.  dpl/dnl: the
        logits' gradients; None (fused path only) = form the BCE gradient of the forward's logits here,
        writing the loss statistics to loss_out (divisor: device count, None = this batch's).  aux_out (data
        parallel, fused head): (loss sum, count) also written there by the same launch; returns True if it was."""
        B, T, p, ids = s["B"], s["T"], s["p"], s["ids"]
        M, d, H, Dh, L = B * T, self.d, self.H, self.Dh, self.L
        sb = s["sb"]
        e = self._buf
        G = lambda n: self.flat.view(n, grad)  # noqa: E731
        slab = self.ws.get("slab", (ops.wgrad_slab_numel(M, 2 * d, d),), torch.float32)
        wln = self.ws.get("ln", (2 * 512 * d,), torch.float32)
        wat = self.ws.get("attn", (B * H * T,), torch.float32)

        fused = ops.sas_block_fused_ok(d, self.dt)
        if fused:
            # the side-stream prologue of forward built the item index and the transposed weights; the head
            # backward needs neither, so the join waits until the blocks' backward
            ev, iws = s["side"] if "side" in s else self._side_prologue(ids, s["pos"], s["neg"])
        if fused:
            dx = e("dx", (M, d))
            lnh = self.ws.get("lnh", (2 * d * (-(-M // 64)),), torch.float32)
            E, gl = self.W("item_emb.weight"), self.Wf("last_layernorm.weight")
            stats = ()
            nb = -(-M // 64)
            if dpl is None and "head_in_block" in s:
                # the head ran inside the last block's output kernel (forward)
                assert s["hdiv"] is divisor, "backward's divisor must be the one forward's head used"
                dx, dpl, dnl, lnh = s["hdx"], s["dpl"], s["dnl"], s["lnh"]
                nb = s["headp"].numel() // 3
                if loss_out is not None:
                    stats = (s["headp"], divisor, loss_out) + ((aux_out,) if aux_out is not None else ())
            elif dpl is None:
                dpl, dnl = e("dpl", (B, T), torch.float32), e("dnl", (B, T), torch.float32)
                ops.sas_head_bwd(s["headp"], divisor, loss_out, s["pl"], s["nl"], None, None, dpl, dnl, s["pos"],
                                 s["neg"], E, s["xL"], gl, s["muf"], s["rf"], dx, lnh)
            else:
                ops.sas_head_bwd(None, None, None, None, None, dpl, dnl, None, None, s["pos"], s["neg"], E, s["xL"],
                                 gl, s["muf"], s["rf"], dx, lnh)
            segs = ops.ln_partial_segments(lnh, M, d, G("last_layernorm.weight"), G("last_layernorm.bias"), nb=nb)
            # the item table's gradient (rs_item_grad, ~40 us) runs on the side stream beside the grouped weight
            # gradients (both latency-bound; measured: inside those launches on one queue 0.367 vs 0.356 ms/step at
            # cfg2, the item chunks queue behind the weight-gradient tiles); the positional table's gradient and the
            # head's loss statistics ride in the grouped reduction's launch on the main one, so both branches end
            # together and the join's cross-queue latency is hidden
            if self._side_refreshed:
                # the blocks' backward reads the transposed weights the side branch wrote this step (otherwise
                # the previous step's optimizer wrote them)
                torch.cuda.current_stream().wait_event(ev)

            def item_grads(dx):
                ops.item_grad(iws, 3, M, dx, math.sqrt(d), p, self.salt["emb"], sb, s["f"], dpl, dnl,
                              G("item_emb.weight"), marks=getattr(self, "row_marks", None))
            dx = self._backward_blocks_fused(s, dx, grad, segs, tail=item_grads,
                                             pos=lambda dx: (ids, T, dx, p, self.salt["emb"], sb,
                                                             G("pos_emb.weight")) + stats)
            torch.cuda.current_stream().wait_event(self._tail_join)
            if split is not None:
                split("dense")          # every parameter gradient is final (data-parallel overlap)
            return len(stats) > 3
        df = e("df", (M, d))
        # the item table's gradient (lookup + tied logits) by the inverted index after the blocks (rs_item_grad /
        # rs_item_grad_f32): one writer per table row in a fixed order, so the unfused (fp32 parity) step is
        # deterministic -- the float-atomic scatter made every fp32 curve its own chaotic draw
        by_index = self.dt == torch.float32 or d in (64, 128, 256)   # else (bf16, other d): atomic scatter
        ops.sampled_logits_bwd(s["f"], self.W("item_emb.weight"), s["pos"], s["neg"], dpl, dnl, df,
                               None if by_index else G("item_emb.weight"))
        dx = e("dx", (M, d))
        ops.layernorm_bwd(s["xL"], df, self.Wf("last_layernorm.weight"), s["muf"], s["rf"], LN_EPS, dx,
                          G("last_layernorm.weight"), G("last_layernorm.bias"), wln, 0)
        for i in reversed(range(L)):
            pre = f"attention_layers.{i}."
            fw = f"forward_layers.{i}."
            # x_{i+1} = (drop2(h1 W2^T + b2) + z) * mask
            dy2, dzres = e("dy2", (M, d)), e("dzres", (M, d))
            ops.dropout_rowmask(dx, p, self.salt[f"ffn2_{i}"], sb, ids, dy2, dzres)
            ops.linear_wgrad(dy2, s["h1"][i], G(fw + "conv2.weight").view(d, d), slab, db=G(fw + "conv2.bias"))
            da1 = e("da1", (M, d))
            ops.linear_dgrad(dy2, self.W(fw + "conv2.weight").view(d, d), da1, act=ops.ACT_RELU_BWD,
                             aux=s["h1"][i], drop_p=p, drop_seed=self.salt[f"ffn1_{i}"], seed_base=sb, drop_ld=d)
            ops.linear_wgrad(da1, s["z"][i], G(fw + "conv1.weight").view(d, d), slab, db=G(fw + "conv1.bias"))
            dz = e("dz", (M, d))
            ops.linear_dgrad(da1, self.W(fw + "conv1.weight").view(d, d), dz, resid=dzres)
            dx1 = e("dx1", (M, d))
            ops.layernorm_bwd(s["x1"][i], dz, self.Wf(f"forward_layernorms.{i}.weight"), s["mu2"][i], s["r2"][i],
                              LN_EPS, dx1, G(f"forward_layernorms.{i}.weight"), G(f"forward_layernorms.{i}.bias"),
                              wln, 0)
            # x1 = Q + o Wo^T + bo
            ops.linear_wgrad(dx1, s["o"][i], G(pre + "out_proj.weight"), slab, db=G(pre + "out_proj.bias"))
            do = e("do", (M, d))
            ops.linear_dgrad(dx1, self.W(pre + "out_proj.weight"), do)
            dq, dkv = e("dq", (M, d)), e("dkv", (M, 2 * d))
            kv = s["kv"][i]
            ops.attn_bwd(B, T, H, Dh, s["q"][i], kv[:, :d], kv[:, d:], s["o"][i], do, s["lse"][i], dq,
                         dkv[:, :d], dkv[:, d:], 1.0 / math.sqrt(Dh), 0, ids, p, self.salt[f"attn{i}"], sb, wat)
            Gin, Gb = G(pre + "in_proj_weight"), G(pre + "in_proj_bias")
            Win = self.W(pre + "in_proj_weight")
            ops.linear_wgrad(dq, s["Q"][i], Gin[:d], slab, db=Gb[:d])
            ops.linear_wgrad(dkv, s["x"][i], Gin[d:], slab, db=Gb[d:])
            dQ = e("dQ", (M, d))
            ops.linear_dgrad(dq, Win[:d], dQ, resid=dx1)
            dxi = e("dxi", (M, d))
            ops.linear_dgrad(dkv, Win[d:], dxi)
            ops.layernorm_bwd(s["x"][i], dQ, self.Wf(f"attention_layernorms.{i}.weight"), s["mu1"][i], s["r1"][i],
                              LN_EPS, dxi, G(f"attention_layernorms.{i}.weight"),
                              G(f"attention_layernorms.{i}.bias"), wln, 0, accumulate=True)
            dx = dxi
        ops.embed_bwd(0, ids, T, dx, math.sqrt(d), p, self.salt["emb"], sb, None if by_index else G("item_emb.weight"),
                      G("pos_emb.weight"))
        if by_index:
            V1 = self.flat.shapes["item_emb.weight"][0]
            iws = self.ws.get("itemidx", (ops.item_index_ws_bytes(3, M, V1, d),), torch.uint8)
            ops.item_index_build([ids, s["pos"], s["neg"]], V1, d, iws)
            ops.item_grad(iws, 3, M, dx, math.sqrt(d), p, self.salt["emb"], sb, s["f"], dpl, dnl,
                          G("item_emb.weight"), marks=getattr(self, "row_marks", None))

    def enable_row_marks(self, min_rows=0):
        """Stamp the rows the inverted-index gradient writes (rs_item_grad_marked) so the optimizer can skip the
        gradient loads of the others: (table name, row marks u8 [rows], epoch u8 [1]), or None where that
        gradient is not the index path's alone (fp32 / other widths) or the table is below min_rows."""
        name = "item_emb.weight"
        rows, d = self.flat.shapes[name]
        if not (self.dt == torch.bfloat16 and d in (64, 128, 256)) or d & (d - 1) or rows < min_rows:
            self.row_marks = None
            return None
        self.row_marks = (torch.zeros(ops.row_marks_bytes(rows), dtype=torch.uint8, device=self.dev),
                          torch.zeros(1, dtype=torch.uint8, device=self.dev))
        return (name,) + self.row_marks

    def _side_prologue(self, ids, pos, neg, after=None):
        """Work of the fused backward that depends only on the batch's keys and the weights, issued on a
        side stream so it overlaps the forward pass: the item-gradient index (rs_item_index_build) and
        the transposed block weights (rs_transpose_bf16).  Returns (event, index workspace)."""
        cur = torch.cuda.current_stream()
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.dev)
        if after is not None:
            self._side.wait_event(after)
        else:
            self._side.wait_stream(cur)
        B, T = ids.shape
        M, d = B * T, self.d
        V1 = self.flat.shapes["item_emb.weight"][0]
        with torch.cuda.stream(self._side):
            iws = self.ws.get("itemidx", (ops.item_index_ws_bytes(3, M, V1, d),), torch.uint8)
            ops.item_index_build([ids, pos, neg], V1, d, iws)
            self._side_refreshed = not self.adam_transposes or self._wT is None
            if self._side_refreshed:
                self._refresh_transposed()
            ev = capture_event()
            ev.record(self._side)
        return ev, iws

    def _refresh_transposed(self):
        """bf16 [in][out] copies of the block weights for the fused backward's input-gradient
        GEMMs (rs_transpose_bf16, one launch); per layer: in_proj^T [d][3d], out_proj^T, conv1^T,
        conv2^T [d][d]."""
        d, L = self.d, self.L
        if self._wT is None:
            self._wT = torch.empty(L * 6 * d * d, dtype=torch.bfloat16, device=self.dev)
            desc = []
            for i in range(L):
                base = i * 6 * d * d
                pre, fw = f"attention_layers.{i}.", f"forward_layers.{i}."
                for name, rows, off in ((pre + "in_proj_weight", 3 * d, 0), (pre + "out_proj.weight", d, 3 * d * d),
                                        (fw + "conv1.weight", d, 4 * d * d), (fw + "conv2.weight", d, 5 * d * d)):
                    desc.append([rows, d, self.flat.offsets[name], d, base + off, rows])
            self._wT_desc = torch.tensor(desc, dtype=torch.int64, device=self.dev)
            self._wT_desc_host = desc
            self._wT_tiles = max(-(-r // 64) * -(-c // 64) for r, c, *_ in desc)
        ops.transpose_bf16(self._wT_desc, self._wT_tiles, self.flat.bf16, self._wT)
        return self._wT

    def _backward_blocks_fused(self, s, dx, grad, extra_segs=(), tail=None, pos=None):
        """SAS blocks' backward with rs_sas_block_out_bwd / rs_sas_block_in_bwd (rowchain.hip) for the
        row-local chains; then ALL ten weight gradients and the four LayerNorm affine partial sets in
        one grouped GEMM launch + one grouped reduction (rs_wgrad_grouped, wgrad.hip).  Returns the
        gradient at the embedding output.  tail(dx): work on that gradient alone (the item table's
        gradient), issued on the side stream so it runs beside the grouped weight-gradient launch (both are
        latency-bound); the caller joins self._tail_join.  pos(dx): the positional table's gradient (and the head's
        loss statistics) in the grouped reduction's launch (ops.wgrad_grouped pos=)."""
        B, T, p, ids, sb = s["B"], s["T"], s["p"], s["ids"], s["sb"]
        M, d, H, Dh, L = B * T, self.d, self.H, self.Dh, self.L
        e = self._buf
        G = lambda n: self.flat.view(n, grad)  # noqa: E731
        wT = self._wT.view(L, 6, d, d)              # refreshed by _side_prologue
        nb = ops.sas_block_parts(M)
        lnp = self.ws.get("lnp", (L, 2, 2 * d * nb), torch.float32)
        wat = self.ws.get("attn", (B * H * T,), torch.float32)
        probs, segs = [], list(extra_segs)
        # per block: the out-side backward's outputs (dy2, da1, dx1, do) and the attention backward's (dq, dkv)
        g = [dict(dy2=e("dy2", (M, d)), da1=e("da1", (M, d)), dx1=e("dx1", (M, d)), do=e("do", (M, d)),
                  dq=e("dq", (M, d)), dkv=e("dkv", (M, 2 * d))) for _ in range(L)]

        # one head: the out-side backward also forms the attention backward's row term delta = rowsum(dO * O)
        # (the attention kernels then read neither O nor recompute it)
        dl = [self.ws.get(f"attn_delta{i}", (B * H * T,), torch.float32) for i in range(L)] if H == 1 else None

        def out_bwd_args(i):
            return (ids, s["h1"][i], s["x1"][i], s["mu2"][i], s["r2"][i], self.Wf(f"forward_layernorms.{i}.weight"),
                    wT[i, 5], wT[i, 4], wT[i, 3], g[i]["dy2"], g[i]["da1"], g[i]["dx1"], g[i]["do"], lnp[i, 0], p,
                    self.salt[f"ffn1_{i}"], self.salt[f"ffn2_{i}"], sb, s["o"][i] if dl else None, dl[i] if dl else None)

        def in_bwd_args(i):
            return (g[i]["dq"], g[i]["dkv"], g[i]["dx1"], s["x"][i], s["mu1"][i], s["r1"][i],
                    self.Wf(f"attention_layernorms.{i}.weight"), wT[i, 0:3].reshape(d, 3 * d))

        ops.sas_block_out_bwd(dx, *out_bwd_args(L - 1))
        for i in reversed(range(L)):
            pre, fw = f"attention_layers.{i}.", f"forward_layers.{i}."
            dq, dkv, kv = g[i]["dq"], g[i]["dkv"], s["kv"][i]
            ops.attn_bwd(B, T, H, Dh, s["q"][i], kv[:, :d], kv[:, d:], s["o"][i], g[i]["do"], s["lse"][i], dq,
                         dkv[:, :d], dkv[:, d:], 1.0 / math.sqrt(Dh), 0, ids, p, self.salt[f"attn{i}"], sb,
                         dl[i] if dl else wat, delta_in=bool(dl))
            dxi = e("dxi", (M, d))
            ops.sas_block_in_bwd(*in_bwd_args(i), dxi, lnp[i, 1])
            if i > 0:
                ops.sas_block_out_bwd(dxi, *out_bwd_args(i - 1))
            dx = dxi
            Gin, Gb = G(pre + "in_proj_weight"), G(pre + "in_proj_bias")
            probs += [(g[i]["dy2"], s["h1"][i], G(fw + "conv2.weight"), G(fw + "conv2.bias")),
                      (g[i]["da1"], s["z"][i], G(fw + "conv1.weight"), G(fw + "conv1.bias")),
                      (g[i]["dx1"], s["o"][i], G(pre + "out_proj.weight"), G(pre + "out_proj.bias")),
                      (dq, s["Q"][i], Gin[:d], Gb[:d]),
                      (dkv, s["x"][i], Gin[d:], Gb[d:])]
            segs += ops.ln_partial_segments(lnp[i, 0], M, d, G(f"forward_layernorms.{i}.weight"),
                                            G(f"forward_layernorms.{i}.bias"))
            segs += ops.ln_partial_segments(lnp[i, 1], M, d, G(f"attention_layernorms.{i}.weight"),
                                            G(f"attention_layernorms.{i}.bias"))
        rows = self._wgrad_rows(M, 6 * L)
        wslab = self.ws.get("wslab", (ops.wgrad_grouped_slab_numel([(d, d)] * 4 * L + [(2 * d, d)] * L, M, rows),),
                            torch.float32)
        join, fork = None, None
        if tail is not None:
            fork = capture_event()
            fork.record(torch.cuda.current_stream())
        # the grouped launch is captured BEFORE the side branch: a HIP graph keeps a node's first child on its
        # queue, so the weight gradients follow the blocks' backward with no cross-queue hop (side branch
        # first: 11 us of fork latency before rs_wgrad_grouped and 11 us of join latency before Adam)
        ops.wgrad_grouped(probs, M, rows, wslab, extra=segs, pos=pos(dx) if pos is not None else None)
        if tail is not None:
            self._side.wait_event(fork)
            with torch.cuda.stream(self._side):
                tail(dx)
                join = capture_event()
                join.record(self._side)
            self._tail_join = join
        return dx

    @staticmethod
    def _wgrad_rows(M, tiles):
        """rows per split of the grouped weight-gradient launch: ~256 workgroups (the 128x128-tile kernel
        runs one per CU), fewer splits also shrink the partial slab the reduction reads."""
        splits = max(1, 256 // tiles)
        return max(64, -(-(-(-M // splits)) // 64) * 64)

    # ---- eval ----------------------------------------------------------------------
    def features(self, ids):
        self.sync_compute_weights()
        _, _, s = self.forward(ids, None, None, False, need_logits=False)
        B, T = ids.shape
        return s["f"].view(B, T, self.d)

    def predict(self, ids, cand):
        f = self.features(ids)[:, -1, :]                    # sas.py:110 (a strided view: row stride T*d)
        # candidate scores <f_b, item_emb[c]> (sas.py:112-114): one wave per (row, candidate), rs_candidate_scores
        return ops.candidate_scores(f, self.W("item_emb.weight"), cand)
