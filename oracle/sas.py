"""SASRec oracle: functional CPU restatement (TEST INFRASTRUCTURE ONLY).

Follows ``BS/models/sas_model/sas.py`` (reference ``NerualNetwork/bert4rec&sas4rec``):

* embedding stage          ``sas.py:60-67``  (item_emb * sqrt(d) + pos_emb, dropout, timeline mask)
* causal mask              ``sas.py:69-70``  (True above the diagonal -> -inf)
* attention sublayer       ``sas.py:72-80``  (Q = LN(x); k, v from the *un-normalised* x;
                                              torch ``F.multi_head_attention_forward`` need_weights=True
                                              path: q*1/sqrt(E), baddbmm(mask, q, k^T), softmax,
                                              dropout, bmm(P, v), out_proj; residual onto Q)
* FFN sublayer             ``sas.py:6-20, 82-84`` (LN -> conv1 -> dropout -> relu -> conv2 -> dropout,
                                              + LN output, timeline mask)
* last LayerNorm           ``sas.py:86``     (eps 1e-8, biased variance)
* sampled tied logits      ``sas.py:90-105``
* candidate scoring        ``sas.py:107-118``
* loss                     ``BS/trainers/sas.py:34-54`` (BCEWithLogits mean over pos != 0, + l2_emb * sum ||p||)

Parameters are passed as a dict keyed exactly like ``SASModel.state_dict()``
(``sas.item_emb.weight`` ...).  Dropout masks may be injected per site
(``masks`` dict) so that the HIP path's dropout can be replayed; with no masks
and ``p == 0`` the math is the deterministic eval/parity path.

``emu=BF16Storage()`` re-runs the same math (in fp64) with bf16 rounding at the
points where the HIP bf16 path stores a tensor in bf16 -- the weights' compute
copies, every saved activation, the activation gradients handed between kernels,
the attention's packed P and dS MFMA operands -- so the fused bf16 kernels can be
held to the arithmetic of a bf16-storage model (tight), separately from the
format's own error against the exact math (tests/test_sas_gpu.py).
"""
import math

import torch
import torch.nn.functional as F

LN_EPS = 1e-8  # torch.nn.LayerNorm(eps=1e-8), sas.py:39,42,50


def layer_norm(x, w, b, eps=LN_EPS):
    """torch.nn.LayerNorm: biased variance, eps inside the sqrt."""
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def _dropout(x, p, mask):
    if mask is False:                # CPU-baseline timing: torch's own bernoulli dropout, as the reference
        return F.dropout(x, p, training=True) if p > 0 else x
    if mask is not None:
        return x * mask / (1.0 - p)
    if p > 0:
        raise ValueError("oracle dropout with p>0 needs an injected mask")
    return x


class _RoundFwd(torch.autograd.Function):
    """value rounded to bf16; gradient passed through (a tensor the kernels store in bf16)."""
    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """value unchanged; the gradient arriving here rounded to bf16 (a gradient handed between kernels in bf16)."""
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class Exact:
    """No rounding: the reference math."""
    def w(self, t):
        return t

    def a(self, t):
        return t

    def g(self, t):
        return t


class BF16Storage(Exact):
    """The HIP bf16 path's storage roundings (rowchain.hip, attention_lds.hip, head.hip, embedding.hip)."""
    def w(self, t):
        return _RoundFwd.apply(t)

    def a(self, t):
        return _RoundFwd.apply(t)

    def g(self, t):
        return _RoundGrad.apply(t)


class RandomDropout(dict):
    """``masks=RandomDropout()``: every dropout site draws torch bernoulli masks, like the
    reference's nn.Dropout (used only to time the CPU baseline at the config dropout)."""

    def get(self, key, default=None):
        return False


def log2feats(P, log_seqs, num_blocks, heads, p=0.0, masks=None, emu=None):
    """sas.py:59-88.  log_seqs: (B,T) int64 tensor.  Returns (B,T,d).  emu: Exact() (default) or
    BF16Storage() -- the HIP bf16 path's rounding points, marked R below (W = weight copy, A = stored
    activation, G = gradient handed between kernels)."""
    masks = {} if masks is None else masks
    R = emu or Exact()
    E = R.w(P["sas.item_emb.weight"])                                # R:W
    d = E.shape[1]
    B, T = log_seqs.shape
    x = F.embedding(log_seqs, E, padding_idx=0) * (d ** 0.5)           # :60-61 (padding_idx=0, :30)
    x = x + R.w(P["sas.pos_emb.weight"])[:T].unsqueeze(0)           # :62-63
    x = _dropout(x, p, masks.get("emb"))                            # :64
    keep = (log_seqs != 0).unsqueeze(-1).to(x.dtype)                # :66-67
    x = R.g(R.a(x * keep))                                           # R:A embedding out, R:G its gradient
    causal = torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1)  # :70 (~tril)
    neg_inf = torch.zeros(T, T, dtype=x.dtype).masked_fill(causal, float("-inf"))
    hd = d // heads
    for i in range(num_blocks):
        pre = f"sas.attention_layers.{i}."
        Q = R.a(layer_norm(x, P[f"sas.attention_layernorms.{i}.weight"],
                           P[f"sas.attention_layernorms.{i}.bias"]))  # :74
        W, bW = R.w(P[pre + "in_proj_weight"]), P[pre + "in_proj_bias"]
        q = R.g(R.a(Q @ W[:d].T + bW[:d]))                            # R:A q, kv; R:G dq, dkv
        k = R.g(R.a(x @ W[d:2 * d].T + bW[d:2 * d]))
        v = R.g(R.a(x @ W[2 * d:].T + bW[2 * d:]))
        q = q.view(B, T, heads, hd).transpose(1, 2) * math.sqrt(1.0 / hd)
        k = k.view(B, T, heads, hd).transpose(1, 2)
        v = v.view(B, T, heads, hd).transpose(1, 2)
        S = neg_inf + R.g(q @ k.transpose(-1, -2))                   # baddbmm(mask, q, k^T); R:G dS operand
        Pm = torch.softmax(S, dim=-1)
        Pm = R.a(_dropout(Pm, p, masks.get(f"attn{i}")))             # R:A P operand of the PV MFMA
        O = R.g(R.a((Pm @ v).transpose(1, 2).reshape(B, T, d)))      # R:A o, R:G do
        y = O @ R.w(P[pre + "out_proj.weight"]).T + P[pre + "out_proj.bias"]
        x = R.g(R.a(Q + y))                                          # :79; R:A x1, R:G dx1
        z = R.a(layer_norm(x, P[f"sas.forward_layernorms.{i}.weight"],
                           P[f"sas.forward_layernorms.{i}.bias"]))    # :82
        z = R.g(z)                                                   # R:G dz (LN2's backward input)
        fw = f"sas.forward_layers.{i}."
        a1 = z @ R.w(P[fw + "conv1.weight"])[:, :, 0].T + P[fw + "conv1.bias"]
        h1 = R.g(R.a(torch.relu(_dropout(a1, p, masks.get(f"ffn1_{i}")))))   # relu(dropout1(conv1)); R:A/G
        a2 = R.g(h1 @ R.w(P[fw + "conv2.weight"])[:, :, 0].T + P[fw + "conv2.bias"])   # R:G dy2
        x = R.g(R.a((_dropout(a2, p, masks.get(f"ffn2_{i}")) + z) * keep))   # :16-20, :84; R:A/G
    f = layer_norm(x, P["sas.last_layernorm.weight"], P["sas.last_layernorm.bias"])  # :86
    return R.a(f)                                                    # R:A the head's stored features


def forward(P, log_seqs, pos_seqs, neg_seqs, num_blocks, heads, p=0.0, masks=None, emu=None):
    """sas.py:90-105 -> (pos_logits, neg_logits), each (B,T)."""
    f = log2feats(P, log_seqs, num_blocks, heads, p, masks, emu)
    E = (emu or Exact()).w(P["sas.item_emb.weight"])
    pe = F.embedding(pos_seqs, E, padding_idx=0)   # padding_idx=0 blocks the row-0 gradient (sas.py:30)
    ne = F.embedding(neg_seqs, E, padding_idx=0)
    return (f * pe).sum(-1), (f * ne).sum(-1)


def predict(P, log_seqs, item_indices, num_blocks, heads):
    """sas.py:107-118 -> (B, C) candidate scores from the last position."""
    f = log2feats(P, log_seqs, num_blocks, heads)[:, -1, :]
    return (P["sas.item_emb.weight"][item_indices] @ f.unsqueeze(-1)).squeeze(-1)


def bce_loss(pos_logits, neg_logits, pos_seqs, params=None, l2_emb=0.0):
    """BS/trainers/sas.py:34-54: BCEWithLogits means over valid = (pos != 0)."""
    valid = pos_seqs != 0
    pl, nl = pos_logits[valid], neg_logits[valid]
    loss = (F.binary_cross_entropy_with_logits(pl, torch.ones_like(pl))
            + F.binary_cross_entropy_with_logits(nl, torch.zeros_like(nl)))
    if l2_emb and params is not None:
        for t in params.values():
            loss = loss + l2_emb * torch.norm(t)
    return loss


def loss_and_grads(P, seq, pos, neg, num_blocks, heads, p=0.0, masks=None, l2_emb=0.0, emu=None):
    """One training-step gradient: returns (loss, pos_logits, neg_logits, grads dict)."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    pl, nl = forward(leaves, seq, pos, neg, num_blocks, heads, p, masks, emu)
    loss = bce_loss(pl, nl, pos, leaves, l2_emb)
    loss.backward()
    return loss.detach(), pl.detach(), nl.detach(), {k: v.grad for k, v in leaves.items()}
