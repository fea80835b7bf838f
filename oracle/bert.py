"""BERT4Rec oracle: functional CPU restatement (TEST INFRASTRUCTURE ONLY).

Follows the reference ``NerualNetwork/bert4rec&sas4rec`` (``BS/``):

* key-padding mask         ``BS/models/bert_modules/bert.py:38``  ((x > 0) over keys)
* embedding                ``embedding/bert.py:29-31``, ``token.py:4-6``, ``position.py:14-16``
                           (token(x) + the whole positional table; dropout)
* transformer block        ``transformer.py:28-32``  (x + drop(MHA(LN(x))); x + drop(FFN(LN(x))); drop(x))
* LayerNorm                ``utils/layer_norm.py:14-17`` (a_2 (x-mean)/(std_unbiased + 1e-6) + b_2)
* attention                ``attention/multi_head.py:24-40``, ``attention/single.py:13-35``
                           (scores/sqrt(d_k), masked_fill(mask==0, -1e9), softmax, dropout, P v)
* feed-forward             ``utils/feed_forward.py:15-16``, ``utils/gelu.py:11-12`` (tanh GELU)
* output layer             ``BS/models/bert.py:10,16`` (untied Linear(d, V+1) on every position)
* loss                     ``BS/trainers/bert.py:30-41`` (CrossEntropyLoss(ignore_index=0))

Parameters are a dict keyed like ``BERTModel.state_dict()``.
"""
import math

import torch
import torch.nn.functional as F

LN_EPS = 1e-6  # utils/layer_norm.py:8


def layer_norm(x, a2, b2, eps=LN_EPS):
    mean = x.mean(-1, keepdim=True)
    std = x.std(-1, keepdim=True)            # unbiased (N-1)
    return a2 * (x - mean) / (std + eps) + b2


def gelu(x):
    return 0.5 * x * (1 + torch.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * torch.pow(x, 3))))


def _dropout(x, p, mask):
    if mask is False:                # CPU-baseline timing: torch's own bernoulli dropout, as the reference
        return F.dropout(x, p, training=True) if p > 0 else x
    if mask is not None:
        return x * mask / (1.0 - p)
    if p > 0:
        raise ValueError("oracle dropout with p>0 needs an injected mask")
    return x


def encode(P, x_ids, num_blocks, heads, p=0.0, hp=0.0, masks=None):
    """BERT.forward (bert_modules/bert.py:36-43) -> hidden (B,T,d).  masks: per-site dropout masks,
    or ``oracle.sas.RandomDropout()`` for torch bernoulli dropout (CPU-baseline timing only)."""
    masks = {} if masks is None else masks
    B, T = x_ids.shape
    key_ok = (x_ids > 0).view(B, 1, 1, T)
    x = F.embedding(x_ids, P["bert.embedding.token.weight"], padding_idx=0) + P["bert.embedding.position.pe.weight"].unsqueeze(0)
    x = _dropout(x, hp, masks.get("emb"))
    d = x.shape[-1]
    dk = d // heads
    for i in range(num_blocks):
        pre = f"bert.transformer_blocks.{i}."
        h = layer_norm(x, P[pre + "input_sublayer.norm.a_2"], P[pre + "input_sublayer.norm.b_2"])
        lin = [(P[pre + f"attention.linear_layers.{j}.weight"], P[pre + f"attention.linear_layers.{j}.bias"])
               for j in range(3)]
        q, k, v = [(h @ w.T + b).view(B, T, heads, dk).transpose(1, 2) for (w, b) in lin]
        scores = (q @ k.transpose(-2, -1)) / math.sqrt(dk)
        scores = scores.masked_fill(~key_ok, -1e9)
        pa = torch.softmax(scores, dim=-1)
        pa = _dropout(pa, p, masks.get(f"attn{i}"))
        o = (pa @ v).transpose(1, 2).contiguous().view(B, T, d)
        y = o @ P[pre + "attention.output_linear.weight"].T + P[pre + "attention.output_linear.bias"]
        x = x + _dropout(y, hp, masks.get(f"res1_{i}"))
        h = layer_norm(x, P[pre + "output_sublayer.norm.a_2"], P[pre + "output_sublayer.norm.b_2"])
        a = h @ P[pre + "feed_forward.w_1.weight"].T + P[pre + "feed_forward.w_1.bias"]
        g = _dropout(gelu(a), hp, masks.get(f"ffn_{i}"))
        y = g @ P[pre + "feed_forward.w_2.weight"].T + P[pre + "feed_forward.w_2.bias"]
        x = x + _dropout(y, hp, masks.get(f"res2_{i}"))
        x = _dropout(x, hp, masks.get(f"blk_{i}"))
    return x


def forward(P, x_ids, num_blocks, heads, p=0.0, hp=0.0, masks=None):
    """BERTModel.forward (BS/models/bert.py:15-16) -> logits (B,T,V+1)."""
    h = encode(P, x_ids, num_blocks, heads, p, hp, masks)
    return h @ P["out.weight"].T + P["out.bias"]


def ce_loss(logits, labels):
    """BS/trainers/bert.py:36-40."""
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), ignore_index=0)


def loss_and_grads(P, x_ids, labels, num_blocks, heads, p=0.0, hp=0.0, masks=None, labelled_only=False):
    """(loss, logits, {name: gradient}).  labelled_only: the output layer on the labelled rows alone (logits
    (R, V+1) in row-major order of the labelled positions) -- the same loss and gradients, since CrossEntropyLoss's
    ignore_index rows (BS/trainers/bert.py:36-40) neither enter the mean nor receive a logit gradient; what a 1M-class
    vocabulary needs to stay within the CPU's memory and seconds (pinned against the full form on the goldens,
    tests/test_oracle.py)."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    if labelled_only:
        h = encode(leaves, x_ids, num_blocks, heads, p, hp, masks)
        lab = labels.reshape(-1)
        rows = torch.nonzero(lab != 0).flatten()
        logits = h.reshape(-1, h.shape[-1])[rows] @ leaves["out.weight"].T + leaves["out.bias"]
        loss = F.cross_entropy(logits, lab[rows])
    else:
        logits = forward(leaves, x_ids, num_blocks, heads, p, hp, masks)
        loss = ce_loss(logits, labels)
    loss.backward()
    return loss.detach(), logits.detach(), {k: v.grad for k, v in leaves.items()}
