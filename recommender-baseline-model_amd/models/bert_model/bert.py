"""BERT4Rec on the MI355X HIP path.

Parameter modules, construction order (so ``model_init_seed`` gives the
reference's exact initial weights) and ``state_dict`` keys are those of the
reference ``BS/models/bert.py:6-16`` + ``BS/models/bert_modules/**``; the torch
modules here are only parameter containers and initialisers.  The math runs as
HIP kernels through the C ABI (include/recsys_hip.h), issued by
:class:`BERTEngine`:

forward (per step)                         kernels
  x = tok[ids] + pe; drop                    rs_embed_fwd (mode 1)          embedding/bert.py:29-31
  per block: h = LN1(x)                      rs_layernorm_fwd (variant 1)   utils/layer_norm.py:14-17
             qkv = h Wqkv^T + b              rs_gemm (one GEMM, q/k/v weights stored adjacent)
             o = attn(q,k,v) key-padding     rs_attn_fwd (mask_kind 1)      attention/single.py:13-35
             x1 = x + drop(o Wo^T + bo)      rs_gemm (+bias+dropout+residual)  sublayer.py:16-18
             g = drop(gelu(LN2(x1) W1^T+b1)) rs_layernorm_fwd, rs_gemm (+bias+gelu+dropout) feed_forward.py:15-16
             x = drop(x1 + drop(g W2^T+b2))  rs_gemm (+bias+dropout+residual+post-dropout) transformer.py:28-32
  logits = x Wout^T + bout                   rs_gemm                        BS/models/bert.py:16
training loss (BS/trainers/bert.py:30-41): CE(ignore_index=0) only needs the
labelled rows, so the fused step compacts them on the device (rs_compact_rows /
rs_gather_rows), runs the vocabulary GEMM + CE on those rows only, and scatters
the hidden-state gradient back (rs_scatter_rows).
"""
import math
import os
import random

import numpy as np
import torch
import torch.nn as nn

from ... import ops
from ...engine_util import Workspace, as_ids, capture_event, compute_dtype, require_cuda, site_salt
from ...flat import ALIGN, FlatParams

LN_EPS = 1e-6  # utils/layer_norm.py:8


# ---------------------------------------------------------------- parameter containers (reference layout)
class LayerNorm(nn.Module):
    def __init__(self, features):
        super().__init__()
        self.a_2 = nn.Parameter(torch.ones(features))
        self.b_2 = nn.Parameter(torch.zeros(features))


class SublayerConnection(nn.Module):
    def __init__(self, size):
        super().__init__()
        self.norm = LayerNorm(size)


class MultiHeadedAttention(nn.Module):
    def __init__(self, h, d_model):
        super().__init__()
        assert d_model % h == 0
        self.d_k = d_model // h
        self.h = h
        self.linear_layers = nn.ModuleList([nn.Linear(d_model, d_model) for _ in range(3)])
        self.output_linear = nn.Linear(d_model, d_model)


class PositionwiseFeedForward(nn.Module):
    def __init__(self, d_model, d_ff):
        super().__init__()
        self.w_1 = nn.Linear(d_model, d_ff)
        self.w_2 = nn.Linear(d_ff, d_model)


class TransformerBlock(nn.Module):
    def __init__(self, hidden, attn_heads, feed_forward_hidden):
        super().__init__()
        self.attention = MultiHeadedAttention(h=attn_heads, d_model=hidden)
        self.feed_forward = PositionwiseFeedForward(d_model=hidden, d_ff=feed_forward_hidden)
        self.input_sublayer = SublayerConnection(size=hidden)
        self.output_sublayer = SublayerConnection(size=hidden)


class PositionalEmbedding(nn.Module):
    def __init__(self, max_len, d_model):
        super().__init__()
        self.pe = nn.Embedding(max_len, d_model)


class BERTEmbedding(nn.Module):
    def __init__(self, vocab_size, embed_size, max_len):
        super().__init__()
        self.token = nn.Embedding(vocab_size, embed_size, padding_idx=0)
        self.position = PositionalEmbedding(max_len=max_len, d_model=embed_size)


def fix_random_seed_as(seed):
    """BS/utils.py:65-71 (called by BERT.__init__, bert_modules/bert.py:12)."""
    random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


class BERT(nn.Module):
    """Mirror of ``bert_modules/bert.py:8-46`` (parameters only)."""

    def __init__(self, args):
        super().__init__()
        fix_random_seed_as(args.model_init_seed)
        self.max_len = args.max_len
        self.hidden = args.bert_hidden_units
        self.heads = args.bert_num_heads
        self.num_blocks = args.bert_num_blocks
        self.dropout = float(args.bert_dropout)
        self.hidden_dropout = float(args.bert_hidden_dropout)
        vocab_size = args.num_items + 2          # [MASK] = num_items + 1, padding = 0
        self.embedding = BERTEmbedding(vocab_size=vocab_size, embed_size=self.hidden, max_len=self.max_len)
        self.transformer_blocks = nn.ModuleList(
            [TransformerBlock(self.hidden, self.heads, self.hidden * 4) for _ in range(self.num_blocks)])


def _storage_order(names):
    """Keep each block's q/k/v weights (then biases) adjacent so one GEMM computes all three."""
    out, seen = [], set()
    for n in names:
        if n in seen:
            continue
        if ".attention.linear_layers.0." in n:
            stem, leaf = n.split(".attention.linear_layers.0.")
            group = [f"{stem}.attention.linear_layers.{j}.{leaf}" for j in range(3)]
            out += group
            seen.update(group)
        elif ".attention.linear_layers." in n:
            continue   # emitted with its .0. sibling
        else:
            out.append(n)
            seen.add(n)
    return out


N256_MIN_V1 = 1 << 16   # see BERTEngine._n256_head


class BERTEngine:
    """Owns workspaces and issues the HIP kernels of one BERT4Rec model."""

    def __init__(self, model, flat: FlatParams):
        self.m = model
        self.flat = flat
        b = model.bert
        self.d = b.hidden
        self.L = b.num_blocks
        self.H = b.heads
        self.Dh = self.d // self.H
        self.F = 4 * self.d
        self.p = b.dropout
        self.hp = b.hidden_dropout
        self.T = b.max_len
        self.V1 = model.out.weight.shape[0]
        self.V1p = -(-self.V1 // 64) * 64
        self.dt = model.cdtype
        self.dev = flat.device
        if self.dt == torch.bfloat16:
            flat.enable_bf16()
        self.ws = Workspace(self.dev)
        self.seed_base = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.external_seed = False    # True: the fused train step's optimizer advances seed_base
        salt0 = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.salt = {"emb": site_salt(salt0, 0)}
        for i in range(self.L):
            for j, k in enumerate(("attn", "res1", "ffn", "res2", "blk")):
                self.salt[f"{k}{i}"] = site_salt(salt0, 1 + 5 * i + j)
        self.qkv_fused = all(flat.adjacent([self._qkv(i, j, leaf) for j in range(3)])
                             for i in range(self.L) for leaf in ("weight", "bias"))

    @staticmethod
    def _qkv(i, j, leaf):
        return f"bert.transformer_blocks.{i}.attention.linear_layers.{j}.{leaf}"

    def sync_compute_weights(self):
        if self.flat.bf16 is not None:
            ops.cast_bf16(self.flat.data, self.flat.bf16)

    def W(self, n):
        return self.flat.cview(n)

    def Wf(self, n):
        return self.flat.view(n)

    def _buf(self, shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.dt, device=self.dev)

    def Wqkv(self, i, buf=None):
        names = [self._qkv(i, j, "weight") for j in range(3)]
        return self.flat.span(names, buf if buf is not None else (self.flat.bf16 if self.flat.bf16 is not None
                                                                   else self.flat.data))

    def bqkv(self, i, buf=None):
        return self.flat.span([self._qkv(i, j, "bias") for j in range(3)], buf)

    # ---- encoder forward -------------------------------------------------------------
    def encode(self, ids, training, clone_seed=True, after_first=None):
        B, T = ids.shape
        if T != self.T:
            raise ValueError(f"sequence length {T} must equal max_len {self.T} (position.py:14-16 adds the "
                             "whole positional table)")
        M, d, H, Dh, L, Fd = B * T, self.d, self.H, self.Dh, self.L, self.F
        p = self.p if training else 0.0
        hp = self.hp if training else 0.0
        if (p > 0 or hp > 0) and not self.external_seed:
            ops.seed_advance(self.seed_base)
        sb = self.seed_base.clone() if clone_seed else self.seed_base
        e = self._buf
        s = {"B": B, "T": T, "p": p, "hp": hp, "ids": ids, "sb": sb, "blocks": []}
        x = e((M, d))
        ops.embed_fwd(1, ids, T, self.W("bert.embedding.token.weight"), self.W("bert.embedding.position.pe.weight"),
                      1.0, hp, self.salt["emb"], sb, x)
        if after_first is not None:
            after_first()
        for i in range(L):
            pre = f"bert.transformer_blocks.{i}."
            h, mu1, r1 = e((M, d)), e((M,), torch.float32), e((M,), torch.float32)
            qkv = e((M, 3 * d))
            g1, b1 = self.Wf(pre + "input_sublayer.norm.a_2"), self.Wf(pre + "input_sublayer.norm.b_2")
            # LN1 inside the QKV GEMM's prologue (rs_gemm_ln: h, mean, rinv as rs_layernorm_fwd writes them)
            if self.qkv_fused and self._ln_gemm() and ops.linear_fwd_ln(x, g1, b1, LN_EPS, self.Wqkv(i), qkv, h, mu1,
                                                                        r1, bias=self.bqkv(i)):
                pass
            elif self.qkv_fused:
                ops.layernorm_fwd(x, g1, b1, LN_EPS, h, mu1, r1, 1)
                ops.linear_fwd(h, self.Wqkv(i), qkv, bias=self.bqkv(i))
            else:
                ops.layernorm_fwd(x, g1, b1, LN_EPS, h, mu1, r1, 1)
                for j in range(3):
                    ops.linear_fwd(h, self.W(self._qkv(i, j, "weight")), qkv[:, j * d:(j + 1) * d],
                                   bias=self.Wf(self._qkv(i, j, "bias")))
            o, lse = e((M, d)), e((B * H * T,), torch.float32)
            ops.attn_fwd(B, T, H, Dh, qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, lse, 1.0 / math.sqrt(Dh), 1,
                         ids, p, self.salt[f"attn{i}"], sb)
            x1 = e((M, d))
            ops.linear_fwd(o, self.W(pre + "attention.output_linear.weight"), x1,
                           bias=self.Wf(pre + "attention.output_linear.bias"), drop_p=hp,
                           drop_seed=self.salt[f"res1{i}"], seed_base=sb, drop_ld=d, resid=x)
            h2, mu2, r2 = e((M, d)), e((M,), torch.float32), e((M,), torch.float32)
            g2, b2 = self.Wf(pre + "output_sublayer.norm.a_2"), self.Wf(pre + "output_sublayer.norm.b_2")
            a_pre, g = e((M, Fd)), e((M, Fd))
            ffn1 = dict(bias=self.Wf(pre + "feed_forward.w_1.bias"), act=ops.ACT_GELU, aux_out=a_pre, drop_p=hp,
                        drop_seed=self.salt[f"ffn{i}"], seed_base=sb, drop_ld=Fd)
            # LN2 inside the FFN1 GEMM's prologue
            if not (self._ln_gemm() and ops.linear_fwd_ln(x1, g2, b2, LN_EPS, self.W(pre + "feed_forward.w_1.weight"),
                                                          g, h2, mu2, r2, **ffn1)):
                ops.layernorm_fwd(x1, g2, b2, LN_EPS, h2, mu2, r2, 1)
                ops.linear_fwd(h2, self.W(pre + "feed_forward.w_1.weight"), g, **ffn1)
            xn = e((M, d))
            ops.linear_fwd(g, self.W(pre + "feed_forward.w_2.weight"), xn, bias=self.Wf(pre + "feed_forward.w_2.bias"),
                           drop_p=hp, drop_seed=self.salt[f"res2{i}"], seed_base=sb, drop_ld=d, resid=x1,
                           post_drop_p=hp, post_drop_seed=self.salt[f"blk{i}"])
            s["blocks"].append(dict(x=x, h=h, mu1=mu1, r1=r1, qkv=qkv, o=o, lse=lse, x1=x1, h2=h2, mu2=mu2, r2=r2,
                                    a_pre=a_pre, g=g))
            x = xn
        s["xL"] = x
        return x, s

    # ---- encoder backward ------------------------------------------------------------
    def encode_backward(self, s, dx, grad):
        """dx: (M, d) compute-dtype gradient of the last hidden state; accumulates parameter grads."""
        B, T, hp, ids, sb = s["B"], s["T"], s["hp"], s["ids"], s["sb"]
        M, d, H, Dh, L, Fd = B * T, self.d, self.H, self.Dh, self.L, self.F
        e = self._buf
        G = lambda n: self.flat.view(n, grad)  # noqa: E731
        slab = self.ws.get("slab", (max(ops.wgrad_slab_numel(M, Fd, d), ops.wgrad_slab_numel(M, d, Fd),
                                        ops.wgrad_slab_numel(M, 3 * d, d)),), torch.float32)
        wln = self.ws.get("ln", (2 * 512 * d,), torch.float32)
        wat = self.ws.get("attn", (B * H * T,), torch.float32)
        # bf16: every block weight gradient is deferred into ONE grouped launch + ONE reduction
        # (rs_wgrad_grouped, wgrad.hip) after the last block's input gradient
        grouped = self.dt == torch.bfloat16 and self.qkv_fused and d % 64 == 0 and Fd % 64 == 0
        probs = []
        ln_segs = []

        def ln_bwd(X, dY, gname, bname, mean, rstd, dX, tag, drop=None):
            """LayerNorm backward; grouped: its affine partials are summed by the grouped launch's reduction (no
            reduction launch per LayerNorm on the backward's critical path).  drop = (salt1, salt2 | None, out1,
            out2 | None): the dropout site(s) consuming dX, in the same launch (rs_layernorm_bwd_drop)."""
            nparts = ops.layernorm_bwd_nparts(X) if grouped else 0
            part = self.ws.get(f"lnpart_{tag}", (2 * d * nparts,), torch.float32) if nparts else wln
            dg, db = (None, None) if nparts else (G(gname), G(bname))
            if drop is not None:
                s1, s2, o1, o2 = drop
                ops.layernorm_bwd_drop(X, dY, self.Wf(gname), mean, rstd, LN_EPS, dX, dg, db, part, 1, hp, s1,
                                       s2 if s2 is not None else 0, sb, o1, o2, accumulate=True)
            else:
                ops.layernorm_bwd(X, dY, self.Wf(gname), mean, rstd, LN_EPS, dX, dg, db, part, 1, accumulate=True)
            if nparts:
                ln_segs.extend(ops.ln_partial_segments(part, M, d, G(gname), G(bname), nb=nparts))

        def wgrad(dY, X, dW, db):
            if grouped:
                probs.append((dY, X, dW, db))
            else:
                ops.linear_wgrad(dY, X, dW, slab, db=db)

        pending = None
        for i in reversed(range(L)):
            a = s["blocks"][i]
            pre = f"bert.transformer_blocks.{i}."
            # x_out = drop_blk(x1 + drop_res2(g W2^T + b2))
            # (the deferred weight gradients need dy / dyo to outlive the in-place LayerNorm-backward
            # accumulations into dx2: separate buffers even without dropout)
            if pending is not None:
                dx2, dy = pending        # formed by the block above's input LayerNorm backward
                pending = None
            elif hp > 0 or grouped:
                dx2, dy = e((M, d)), e((M, d))
                ops.dropout2(dx, hp, self.salt[f"blk{i}"], self.salt[f"res2{i}"], sb, dx2, dy)
            else:
                dx2, dy = dx, dx
            wgrad(dy, a["g"], G(pre + "feed_forward.w_2.weight"), G(pre + "feed_forward.w_2.bias"))
            da = e((M, Fd))
            ops.linear_dgrad(dy, self.W(pre + "feed_forward.w_2.weight"), da, act=ops.ACT_GELU_BWD, aux=a["a_pre"],
                             drop_p=hp, drop_seed=self.salt[f"ffn{i}"], seed_base=sb, drop_ld=Fd)
            wgrad(da, a["h2"], G(pre + "feed_forward.w_1.weight"), G(pre + "feed_forward.w_1.bias"))
            dh2 = e((M, d))
            ops.linear_dgrad(da, self.W(pre + "feed_forward.w_1.weight"), dh2)
            # x1 = x + drop_res1(o Wo^T + bo): dyo = drop_res1(dx2) formed by the LayerNorm backward's launch
            if grouped:
                dyo = e((M, d))
                ln_bwd(a["x1"], dh2, pre + "output_sublayer.norm.a_2", pre + "output_sublayer.norm.b_2", a["mu2"],
                       a["r2"], dx2, f"{i}o", drop=(self.salt[f"res1{i}"], None, dyo, None))
            else:
                ln_bwd(a["x1"], dh2, pre + "output_sublayer.norm.a_2", pre + "output_sublayer.norm.b_2", a["mu2"],
                       a["r2"], dx2, f"{i}o")
                if hp > 0:
                    dyo = e((M, d))
                    ops.dropout_rowmask(dx2, hp, self.salt[f"res1{i}"], sb, None, dyo)
                else:
                    dyo = dx2
            wgrad(dyo, a["o"], G(pre + "attention.output_linear.weight"), G(pre + "attention.output_linear.bias"))
            do = e((M, d))
            ops.linear_dgrad(dyo, self.W(pre + "attention.output_linear.weight"), do)
            qkv = a["qkv"]
            dqkv = e((M, 3 * d))
            # the attention backward's row term delta = rowsum(dO * O) per head, formed once here: neither
            # attention pass then reads O, and the dK/dV pass streams its Q/dO images while it computes
            ops.attn_row_delta(B, T, H, Dh, do, a["o"], wat)
            ops.attn_bwd(B, T, H, Dh, qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], a["o"], do, a["lse"],
                         dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:], 1.0 / math.sqrt(Dh), 1, ids, s["p"],
                         self.salt[f"attn{i}"], sb, wat, delta_in=True)
            dh = e((M, d))
            if self.qkv_fused:
                wgrad(dqkv, a["h"], self.Wqkv(i, grad), self.bqkv(i, grad))
                ops.linear_dgrad(dqkv, self.Wqkv(i), dh)
            else:
                for j in range(3):
                    ops.linear_wgrad(dqkv[:, j * d:(j + 1) * d], a["h"], G(self._qkv(i, j, "weight")), slab,
                                     db=G(self._qkv(i, j, "bias")))
                    ops.linear_dgrad(dqkv[:, j * d:(j + 1) * d], self.W(self._qkv(i, j, "weight")), dh,
                                     accumulate=j > 0)
            if grouped and i > 0:
                # the block below starts with dropout2 of this dX (its blk and res2 sites): same launch
                pending = (e((M, d)), e((M, d)))
                ln_bwd(a["x"], dh, pre + "input_sublayer.norm.a_2", pre + "input_sublayer.norm.b_2", a["mu1"],
                       a["r1"], dx2, f"{i}i",
                       drop=(self.salt[f"blk{i - 1}"], self.salt[f"res2{i - 1}"], pending[0], pending[1]))
            else:
                ln_bwd(a["x"], dh, pre + "input_sublayer.norm.a_2", pre + "input_sublayer.norm.b_2", a["mu1"],
                       a["r1"], dx2, f"{i}i")
            dx = dx2
        if self._det_table():
            # token-table gradient by inverted index (rs_item_grad: sorted keys, per-row sums, no float
            # atomics -- deterministic); the index comes from the side stream when the step issued it
            ev, iws = s["side"] if "side" in s else self._token_index(ids, side=False)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
            ops.embed_bwd(1, ids, T, dx, 1.0, hp, self.salt["emb"], sb, None, G("bert.embedding.position.pe.weight"))
            ops.item_grad(iws, 1, M, dx, 1.0, hp, self.salt["emb"], sb, None, None, None,
                          G("bert.embedding.token.weight"), marks=getattr(self, "row_marks", None))
        else:
            ops.embed_bwd(1, ids, T, dx, 1.0, hp, self.salt["emb"], sb, G("bert.embedding.token.weight"),
                          G("bert.embedding.position.pe.weight"))
        hook = getattr(self, "after_token_grads", None)
        # the token table's gradient is final; True: the trainer's optimizer update of it now runs beside the grouped
        # weight gradients, which then take 128-wide tiles (the 256-wide form slowed 10x sharing the chip with that
        # stream at cfg5: 1,377 against 280 us; cfg5 5.8k -> 7.07k seq/s)
        beside = bool(hook("bert.embedding.token.weight")) if hook is not None else False
        tmax = 128 if beside else 256
        ex, sp = getattr(self, "sparse_tok", None), getattr(self, "_split", None)
        if ex is not None and sp is not None:
            # data parallel, union-of-touched-rows exchange of the token table's gradient (dp.SparseRowExchange):
            # its all-reduce runs beside the grouped weight-gradient launches below
            ex.pack()
            sp("tok_rows", ex.allreduce)
            ex.unpack()
        for c in range(0, len(probs), 16):              # rs_wgrad_grouped takes up to 16 problems
            chunk = probs[c:c + 16]
            shapes = [(p[0].shape[1], p[1].shape[1]) for p in chunk]
            rows = self._wgrad_rows(M, shapes, tmax)
            wslab = self.ws.get(f"wslab{c}_{tmax}", (ops.wgrad_grouped_slab_numel(shapes, M, rows),), torch.float32)
            ops.wgrad_grouped(chunk, M, rows, wslab, extra=ln_segs if c == 0 else (), max_tile=tmax)

    def overwritten_grads(self):
        """(lo, hi) flat range whose gradient the fused step writes whole every step (out.weight then out.bias,
        train_loss_and_backward): the optimizer leaves it unzeroed (FusedAdam.step keep) when it is large enough
        for the saved sweep (8 B per element) to pay for the extra launch -- the 1M-item vocabulary (256M
        elements), not the 27k one.  Contract: every head path WRITES this whole range (dE = dlogits^T h and the
        bias column sums with accumulate off; rows without labelled logits get exact zeros) and nothing else
        accumulates into it -- a head variant that accumulated would double-count the previous step's gradient
        (tests/test_bert.py ...overwritten_head_grads_match_zeroed, tests/test_dp_gpu.py
        ...unzeroed_head_grads_equal_zeroed under the in-place all-reduce)."""
        if self.V1 * self.d < (1 << 24):
            return None
        return self.head_grad_range()

    def head_grad_range(self):
        """(lo, hi) flat range of out.weight then out.bias (their gradient is final once the head's dE / dh are
        formed), or None when the layout does not make it one 16-B aligned range (or the head is sharded)."""
        f = self.flat
        ow, ob = f.offsets["out.weight"], f.offsets["out.bias"]
        A = ALIGN   # FlatParams pads every parameter to a multiple of ALIGN floats
        end = ob + -(-self.V1 // A) * A
        if getattr(self, "vocab_shard", None) is not None:
            return None
        if ob != ow + -(-self.V1 * self.d // A) * A or end > f.numel or ow % 4 or end % 4:
            return None
        return ow, min(end, f.numel)

    def _ln_gemm(self):
        """The sublayers' LayerNorms inside the GEMMs they feed (rs_gemm_ln: bf16, d = 256)?  RS_GEMM_LN=0 (read per
        call, for A/B): rs_layernorm_fwd + rs_gemm, the same bits."""
        return self.dt == torch.bfloat16 and self.d == 256 and os.environ.get("RS_GEMM_LN", "1") != "0"

    def _det_table(self):
        return self.dt == torch.bfloat16 and self.d in (64, 128, 256)

    def enable_row_marks(self, min_rows=0):
        """Stamp the rows the inverted-index gradient writes (rs_item_grad_marked) so the optimizer can skip the
        gradient loads of the others: (table name, row marks u8 [rows], epoch u8 [1]), or None where that
        gradient is not the index path's alone (fp32 / other widths) or the table is below min_rows."""
        name = "bert.embedding.token.weight"
        rows, d = self.flat.shapes[name]
        if not self._det_table() or d & (d - 1) or rows < min_rows:
            self.row_marks = None
            return None
        self.row_marks = (torch.zeros(ops.row_marks_bytes(rows), dtype=torch.uint8, device=self.dev),
                          torch.zeros(1, dtype=torch.uint8, device=self.dev))
        return (name,) + self.row_marks

    def _token_index(self, ids, side=True, after=None):
        """rs_item_index_build over the batch's token ids (the token-table gradient's inverted index); on a
        side stream overlapping the forward pass when ``side``, ordered after the event ``after`` (else after the
        current stream's work).  Returns (event or None, workspace)."""
        M = ids.numel()
        rows = self.flat.shapes["bert.embedding.token.weight"][0]
        iws = self.ws.get("tokidx", (ops.item_index_ws_bytes(1, M, rows, self.d),), torch.uint8)
        if not side:
            ops.item_index_build([ids], rows, self.d, iws)
            return None, iws
        cur = torch.cuda.current_stream()
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.dev)
        if after is not None:
            self._side.wait_event(after)
        else:
            self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            ops.item_index_build([ids], rows, self.d, iws)
            ev = capture_event()
            ev.record(self._side)
        return ev, iws

    @staticmethod
    def _wgrad_rows(M, shapes, max_tile=256):
        """rows per split of the grouped weight-gradient launch.  128 x 128 tiles: about one and a half workgroups per
        CU in total (cfg3: 192 tiles x 2 splits; 4 splits measured 156 against 153 us for the launch, 1 split 219 us);
        256 x 256 tiles (every dimension a multiple of 256, rs_wgrad_grouped_tile; one 8-wave workgroup per CU): about
        one per CU (cfg3: 48 tiles x 5 splits)."""
        t = ops.wgrad_grouped_tile(shapes, max_tile)
        tiles = sum(-(-n // t) * -(-k // t) for n, k in shapes)
        splits = max(1, round((256 if t == 256 else 384) / tiles))
        return max(64, -(-(-(-M // splits)) // 64) * 64)

    # ---- eval scores at candidates (BS/trainers/bert.py:43-49 without the (B, T, V+1) logits) --------
    def predict(self, ids, cand):
        """logits[:, -1, :].gather(1, cand) of the reference's validation: the encoder in eval mode (no dropout),
        then only the last position's scores at the candidates (out.weight rows . h_last + out.bias)."""
        self.sync_compute_weights()
        B, T = ids.shape
        xL, _ = self.encode(ids, False)
        h = xL.view(B, T, self.d)[:, -1, :]
        return ops.candidate_scores(h, self.W("out.weight"), cand, bias=self.Wf("out.bias"))

    def _n256_head(self):
        """(dE, dh) on the 256-wide-tile GEMM (gemm_n256.hip)?  bf16 and d = 256 only.  dh = dlogits E (split over
        the vocabulary) at every vocabulary size; dE = dlogits^T h from N256_MIN_V1 classes on (3.9k row tiles at
        1M classes; the 27k-class cfg3 head has 105, under the 256 CUs, where the 128x128 kernel's 418 tiles are
        faster).  Measured (tools/diag/vocab_gemm_probe.py, R = 1,792): 1M classes dE 1,745 -> 1,278 us, dh 1,262 ->
        1,059 us; 26,745 classes dh 60.5 -> 41.1 us, dE 94.8 -> 112.7 us.  RS_N256_HEAD=0/1 forces both off / on."""
        ok = self.dt == torch.bfloat16 and self.d == 256
        env = os.environ.get("RS_N256_HEAD")
        if env is not None:
            return (ok and env == "1",) * 2
        return ok and self.V1 >= N256_MIN_V1, ok

    # ---- full-vocabulary logits (the reference forward API) ---------------------------
    def logits(self, xL):
        M = xL.shape[0]
        out = torch.empty((M, self.V1p), dtype=torch.float32, device=self.dev)[:, :self.V1]
        ops.linear_fwd(xL, self.W("out.weight"), out, bias=self.Wf("out.bias"))
        return out

    def logits_backward(self, xL, dlogits, grad):
        """dlogits (M, V+1) fp32 -> out.weight/out.bias grads and dx_L (compute dtype)."""
        M = xL.shape[0]
        d = self.d
        dl = self.ws.get("dlogits_full", (M, self.V1p), self.dt)[:, :self.V1]
        dl.copy_(dlogits)
        slab = self.ws.get("slab_out", (ops.wgrad_slab_numel(M, self.V1, d),), torch.float32)
        ops.linear_wgrad(dl, xL, self.flat.view("out.weight", grad), slab, db=self.flat.view("out.bias", grad))
        dx = self._buf((M, d))
        ops.linear_dgrad(dl, self.W("out.weight"), dx)
        return dx

    # ---- fused training loss (labelled rows only) -------------------------------------
    def train_loss_and_backward(self, tokens, labels, loss_out, global_count, grad, max_labelled=None, split=None):
        """Forward + CE(ignore_index=0) + backward of one batch.  loss_out[0] = loss sum, [1] = local
        labelled count, [2] = local mean; ``global_count(local)`` returns the divisor (DP).
        split(tag, action): data-parallel segment points (train_step.FusedTrainStep); with a sparse token-table
        exchange (self.sparse_tok) the step starts with the all-gather of the batch ids."""
        ex = getattr(self, "sparse_tok", None)
        self._split = split
        if ex is not None and split is not None:
            split("tok_ids", lambda: ex.gather_ids(tokens))
            ex.index_rows()
        # the token index on the side stream, issued after the first forward launch but ordered only after what
        # preceded it: in a captured graph the forward chain is then the first child of the step's root and keeps
        # the launch queue, and the side branch takes the second (issued first, it kept the queue and the whole
        # encoder moved: cfg3 paid ~7 us before the embedding and ~12 us at the token gradient's queue hop;
        # three interleaved rounds: 1.4145 / 1.4142 / 1.4149 -> 1.3983 / 1.4052 / 1.3978 ms/step)
        side_box = {}
        if self._det_table():
            fork = capture_event()
            fork.record()
            side_box["fork"] = fork

        def after_first():
            if "fork" in side_box:
                side_box["side"] = self._token_index(tokens, after=side_box["fork"])
        xL, s = self.encode(tokens, True, clone_seed=False, after_first=after_first)
        side = side_box.get("side")
        if side is not None:
            s["side"] = side
        B, T = tokens.shape
        M, d = B * T, self.d
        cap = int(max_labelled or M)
        idx = self.ws.get("cidx", (cap,), torch.int32)
        rank = self.ws.get("crank", (M,), torch.int32)
        cnt = self.ws.get("ccount", (1,), torch.int32)
        ops.compact_rows(labels, cap, idx, rank, cnt)
        hl = self.ws.get("hl", (cap, d), self.dt)
        lab = self.ws.get("lab", (cap,), torch.int64)
        if getattr(self, "vocab_shard", None) is not None:
            return self._sharded_head_and_backward(s, xL, hl, lab, idx, rank, cnt, labels, cap, loss_out, grad, split)
        ops.gather_rows(xL, idx, cnt, cap, hl, labels, lab)
        hook = getattr(self, "before_head", None)
        if hook is not None:
            hook()                      # out.weight / out.bias are read from here on
        if self.dt == torch.bfloat16 and ops.vocab_head_supported(d):
            # vocabulary-tile-stationary kernels (vocab_head.hip): logits never materialised
            wce = self.ws.get("vce", (ops.vocab_ce_ws_numel(cap, self.V1),), torch.float32)
            ops.vocab_head_fwd(hl, self.W("out.weight"), self.Wf("out.bias"), lab, wce, loss_out, rows_dev=cnt)
            count = global_count(loss_out[1:2])
            dl = self.ws.get("dlogits", (cap, self.V1p), self.dt)[:, :self.V1]
            ops.vocab_head_bwd(hl, self.W("out.weight"), self.Wf("out.bias"), lab, wce, count, dl, rows_dev=cnt)
        elif self.dt == torch.bfloat16:
            # widths the tile head does not cover: logits never materialised either -- GEMM + online-softmax
            # partials, then GEMM + dlogits (vocab_ce.hip)
            wce = self.ws.get("vce", (ops.vocab_ce_ws_numel(cap, self.V1),), torch.float32)
            ops.vocab_ce_fwd(hl, self.W("out.weight"), self.Wf("out.bias"), lab, wce, loss_out, rows_dev=cnt)
            count = global_count(loss_out[1:2])
            dl = self.ws.get("dlogits", (cap, self.V1p), self.dt)[:, :self.V1]
            ops.vocab_ce_bwd(hl, self.W("out.weight"), self.Wf("out.bias"), lab, wce, count, dl, rows_dev=cnt)
        else:
            logits = self.ws.get("logits", (cap, self.V1p), torch.float32)[:, :self.V1]
            ops.linear_fwd(hl, self.W("out.weight"), logits, bias=self.Wf("out.bias"), rows_dev=cnt)
            wce = self.ws.get("wce", (3 * cap,), torch.float32)
            ops.ce_fwd(logits, lab, wce, loss_out, None, rows_dev=cnt)
            count = global_count(loss_out[1:2])
            if self.dt == torch.float32:
                dl = logits                                   # in place
            else:
                dl = self.ws.get("dlogits", (cap, self.V1p), self.dt)[:, :self.V1]
            ops.ce_bwd(logits, lab, count, None, wce, dl, rows_dev=cnt)
        big_dE, big_dh = self._n256_head()
        # out.weight / out.bias get their whole gradient here: written, not accumulated (no read of the old
        # values; see overwritten_grads)
        if big_dE:  # 256-wide tiles: dlogits streams once (gemm_n256.hip)
            ops.gemm_n256(dl, hl, self.flat.view("out.weight", grad), True, self.V1, cap,
                          colsum=self.flat.view("out.bias", grad), rows_dev=cnt)
        else:
            slab = self.ws.get("slab_out", (ops.wgrad_slab_numel(cap, self.V1, d),), torch.float32)
            ops.linear_wgrad(dl, hl, self.flat.view("out.weight", grad), slab, db=self.flat.view("out.bias", grad),
                             rows_dev=cnt, accumulate=False)
        if split is not None:
            # join the side stream's token index here: a captured graph segment must not end with forked work
            if s.get("side") is not None and s["side"][0] is not None:
                torch.cuda.current_stream().wait_event(s["side"][0])
                s["side"] = (None, s["side"][1])
            split("out")                # the vocabulary head's gradient is final (data-parallel overlap)
        # contraction over the whole vocabulary with few rows: split-K into slabs, then ONE pass that sums
        # the live rows' partials in a fixed order, casts and scatters them back to the token rows
        if big_dh:
            sk = ops.gemm_n256_splits(cap, self.V1)
            slab_d = self.ws.get("slab_dh", (sk * cap * d,), torch.float32)
            ops.gemm_n256(dl, self.W("out.weight"), slab_d.view(sk, cap, d), False, cap, self.V1, split=True,
                          rows_dev=cnt)
        else:
            sk = int(max(1, min(64, -(-self.V1 // 2048))))
            slab_d = self.ws.get("slab_dh", (sk * cap * d,), torch.float32)
            ops.gemm(dl, self.W("out.weight"), slab_d, cap, d, self.V1, False, True, ops.epilogue(rows_dev=cnt),
                     split_k=sk, slab=slab_d)
        hook = getattr(self, "after_head_grads", None)
        if hook is not None:
            hook()                      # out.weight / out.bias are final and no longer read this step
        dxL = self._buf((M, d))
        ops.splitk_scatter_rows(slab_d, sk, cap, rank, dxL)
        self.encode_backward(s, dxL, grad)


    def _sharded_head_and_backward(self, s, xL, hl, lab, idx, rank, cnt, labels, cap, loss_out, grad, split):
        """The vocabulary head with out.weight / out.bias sharded over the data-parallel ranks (vocab_parallel.py):
        loss_out = (loss sum, labelled count, mean) of the GLOBAL batch on every rank; gradients are those of the
        global mean (no later division); this rank's out.weight rows get complete gradients, the rest none."""
        vs = self.vocab_shard
        if not (self.dt == torch.bfloat16 and ops.vocab_head_supported(self.d)):
            raise RuntimeError("the vocabulary-sharded head needs the bf16 path and d in {64, 128, 256}")
        B, T = xL.shape[0] // self.T, self.T
        M, d, N = xL.shape[0], self.d, vs.world
        R = N * cap
        v0, v1 = vs.v0, vs.v1
        V1s = v1 - v0
        hl.zero_()                       # rows past the labelled count: zero (they meet dlogits = 0 in dE)
        lab.zero_()
        ops.gather_rows(xL, idx, cnt, cap, hl, labels, lab)
        H = self.ws.get("vs_H", (R, d), self.dt)
        L = self.ws.get("vs_L", (R,), torch.int64)

        def sync(tag, action):
            if split is None:
                action()
            else:
                if s.get("side") is not None and s["side"][0] is not None:     # join the side stream first
                    torch.cuda.current_stream().wait_event(s["side"][0])
                    s["side"] = (None, s["side"][1])
                split(tag, action)

        sync("vocab_gather", lambda: (vs.all_gather(H, hl), vs.all_gather(L, lab)))
        Es, bs = self.W("out.weight")[v0:v1], self.Wf("out.bias")[v0:v1]
        wce = self.ws.get("vs_ce", (ops.vocab_ce_ws_numel(R, V1s),), torch.float32)
        lse_r = self.ws.get("vs_lse_r", (R,), torch.float32)
        tgt = self.ws.get("vs_tgt", (R,), torch.float32)
        ops.vocab_shard_lse(H, Es, bs, L, wce, lse_r)
        ops.vocab_shard_label_logits(H, Es, bs, L, v0, v1, tgt)
        lse_parts = self.ws.get("vs_lse_parts", (N, R), torch.float32)
        sync("vocab_lse", lambda: (vs.all_gather(lse_parts.view(-1), lse_r), vs.all_reduce(tgt)))
        ntn = -(-V1s // 128)
        lse = wce[R * ntn * 2 + R:R * ntn * 2 + 2 * R]      # where rs_vocab_head_bwd reads the row lse
        ops.vocab_shard_combine(lse_parts, tgt, L, lse, loss_out)
        count = loss_out[1:2]
        V1sp = -(-V1s // 8) * 8
        dl = self.ws.get("vs_dlogits", (R, V1sp), self.dt)[:, :V1s]
        ops.vocab_head_bwd(H, Es, bs, L, wce, count, dl, voff=v0)
        slab = self.ws.get("vs_slab_out", (ops.wgrad_slab_numel(R, V1s, d),), torch.float32)
        ops.linear_wgrad(dl, H, self.flat.view("out.weight", grad)[v0:v1], slab,
                         db=self.flat.view("out.bias", grad)[v0:v1])
        sk = int(max(1, min(64, -(-V1s // 2048))))
        slab_d = self.ws.get("vs_slab_dh", (sk * R * d,), torch.float32)
        ops.gemm(dl, Es, slab_d, R, d, V1s, False, True, ops.epilogue(), split_k=sk, slab=slab_d)
        dH = self.ws.get("vs_dH", (R, d), torch.float32)
        ops.reduce_slabs(slab_d, sk, dH)
        sync("vocab_dh", lambda: vs.all_reduce(dH))
        dxL = self._buf((M, d))
        ops.splitk_scatter_rows(dH[vs.rank * cap:(vs.rank + 1) * cap], 1, cap, rank, dxL)
        self.encode_backward(s, dxL, grad)


class _BERTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, ids, training, *params):
        engine.sync_compute_weights()
        xL, s = engine.encode(ids, training)
        logits = engine.logits(xL)
        ctx.engine, ctx.saved, ctx.xL = engine, s, xL
        B, T = ids.shape
        return logits.view(B, T, -1)

    @staticmethod
    def backward(ctx, dlogits):
        eng = ctx.engine
        grad = torch.zeros(eng.flat.numel, dtype=torch.float32, device=eng.flat.device)
        B, T, V1 = dlogits.shape
        dx = eng.logits_backward(ctx.xL, dlogits.reshape(B * T, V1), grad)
        eng.encode_backward(ctx.saved, dx, grad)
        ctx.saved = None
        return (None, None, None, *[eng.flat.view(n, grad) for n in eng.flat.names_in_module_order])


def build_flat(model, device):
    flat = FlatParams(model, device, order=_storage_order)
    flat.names_in_module_order = [n for n, _ in model.named_parameters()]
    return flat


def require(model):
    p = model.out.weight
    require_cuda(p.device)
    return p.device


__all__ = ["BERT", "BERTEngine", "_BERTFunction", "build_flat", "as_ids", "compute_dtype", "require"]
