"""bf16 error budget of the fused SAS training step, emulated on the CPU (diagnostic; not a test).

Re-runs the oracle's SAS math in fp64 with bf16 rounding inserted where the HIP bf16 path stores a tensor in
bf16 (weights' compute copies, saved activations, activation gradients between kernels, the attention's packed
P / dS MFMA operands).  Each rounding group can be switched off to see how much of the per-tensor gradient
error (vs exact fp64) it causes.

    python tools/diag/bf16_budget.py [--B 4 --T 50 --d 64 --V 500]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

GROUPS = ("W", "WE", "Ax", "AQ", "Aqkv", "Ao", "Ax1", "Az", "Ah1", "G", "P", "DS", "LNG")
ON = set(GROUPS)


def rb(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _RF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return rb(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _RG(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return rb(g)


def RF(x, grp="A"):
    return _RF.apply(x) if grp in ON else x


def RG(x, grp="G"):
    return _RG.apply(x) if grp in ON else x


def ln(x, w, b, eps=1e-8):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def forward(P, seq, pos, neg, L, heads):
    W = lambda k: RF(P[k], "W")  # noqa: E731   bf16 compute copy of a block weight (MFMA operand)
    E = P["sas.item_emb.weight"]
    d = E.shape[1]
    B, T = seq.shape
    Eb = RF(E, "WE")                   # the tables' bf16 copies: the embedding gather and the tied logits (VALU)
    x = F.embedding(seq, Eb) * math.sqrt(d) + RF(P["sas.pos_emb.weight"], "WE")[:T]
    keep = (seq != 0).unsqueeze(-1).double()
    x = x * keep
    x = RG(RF(x, "Ax"))                # x0 stored bf16; its gradient dx (block_in_bwd output) bf16
    causal = torch.triu(torch.ones(T, T, dtype=torch.bool), 1)
    hd = d // heads
    for i in range(L):
        pre = f"sas.attention_layers.{i}."
        Q = RF(ln(x, P[f"sas.attention_layernorms.{i}.weight"], P[f"sas.attention_layernorms.{i}.bias"]), "AQ")
        Win, b = W(pre + "in_proj_weight"), P[pre + "in_proj_bias"]
        q = RG(RF(Q @ Win[:d].T + b[:d], "Aqkv"))                   # dq bf16 (attention bwd output)
        k = RG(RF(x @ Win[d:2 * d].T + b[d:2 * d], "Aqkv"))
        v = RG(RF(x @ Win[2 * d:].T + b[2 * d:], "Aqkv"))
        qh = q.view(B, T, heads, hd).transpose(1, 2)
        kh = k.view(B, T, heads, hd).transpose(1, 2)
        vh = v.view(B, T, heads, hd).transpose(1, 2)
        S = (qh @ kh.transpose(-1, -2)) / math.sqrt(hd)
        S = RG(S, "DS")                                       # dS packed to bf16 for the dQ / dK MFMAs
        S = S.masked_fill(causal, float("-inf"))
        Pm = RF(torch.softmax(S, -1), "P")                    # P packed to bf16 for the PV MFMA
        O = (Pm @ vh).transpose(1, 2).reshape(B, T, d)
        O = RG(RF(O, "Ao"))                                          # o saved bf16; do (dout) bf16
        x1 = RG(RF(Q + O @ W(pre + "out_proj.weight").T + P[pre + "out_proj.bias"], "Ax1"))   # dx1 bf16
        z = RF(ln(x1, P[f"sas.forward_layernorms.{i}.weight"], P[f"sas.forward_layernorms.{i}.bias"]), "Az")
        z = RG(z, "LNG")                                      # dz rounded in LDS before LN2's backward
        fw = f"sas.forward_layers.{i}."
        a1 = z @ W(fw + "conv1.weight")[:, :, 0].T + P[fw + "conv1.bias"]
        h1 = RG(RF(torch.relu(a1), "Ah1"))                           # h1 saved bf16; da1 bf16
        a2 = h1 @ W(fw + "conv2.weight")[:, :, 0].T + P[fw + "conv2.bias"]
        a2 = RG(a2)                                           # dy2 bf16
        x = RG(RF((a2 + z) * keep, "Ax"))                           # block output bf16; its gradient dxn bf16
    f = ln(x, P["sas.last_layernorm.weight"], P["sas.last_layernorm.bias"])
    pe, ne = F.embedding(pos, Eb), F.embedding(neg, Eb)
    return (f * pe).sum(-1), (f * ne).sum(-1)


def loss_and_grads(P, seq, pos, neg, L, h):
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    pl, nl = forward(leaves, seq, pos, neg, L, h)
    valid = pos != 0
    loss = (F.binary_cross_entropy_with_logits(pl[valid], torch.ones_like(pl[valid]))
            + F.binary_cross_entropy_with_logits(nl[valid], torch.zeros_like(nl[valid])))
    loss.backward()
    return loss.item(), {k: v.grad.clone() for k, v in leaves.items()}


def rel(a, b):
    return float((a - b).norm() / max(b.norm(), 1e-300))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--V", type=int, default=500)
    ap.add_argument("--L", type=int, default=2)
    args = ap.parse_args()
    import rbm_amd.data as synth
    from rbm_amd.models.sas_model.sas import SAS
    torch.manual_seed(args.V + args.T)
    a = argparse.Namespace(num_items=args.V, max_len=args.T, device="cpu", sas_hidden_units=args.d,
                           sas_num_blocks=args.L, sas_heads=1, sas_dropout=0.0, l2_emb=0.0, rs_dtype="fp32")
    m = SAS(a)
    P = {"sas." + k: v.detach().double() for k, v in m.state_dict().items()}
    rng = np.random.default_rng(args.T)
    seq, pos, neg = (torch.from_numpy(x) for x in synth.sas_batch(rng, args.B, args.T, args.V))
    ON.clear()
    l64, g64 = loss_and_grads(P, seq, pos, neg, args.L, 1)
    rows = []
    for label, on in [("all", set(GROUPS))] + [(f"all-{g}", set(GROUPS) - {g}) for g in GROUPS] + \
            [(f"only-{g}", {g}) for g in GROUPS]:
        ON.clear()
        ON.update(on)
        l, g = loss_and_grads(P, seq, pos, neg, args.L, 1)
        errs = {}
        for k in g64:
            u, r = g[k], g64[k]
            if k.endswith("in_proj_bias"):
                d = args.d
                u, r = torch.cat([u[:d], u[2 * d:]]), torch.cat([r[:d], r[2 * d:]])
            errs[k] = rel(u, r)
        worst = max(errs, key=errs.get)
        rows.append((label, abs(l - l64) / abs(l64), worst, errs[worst], float(np.median(list(errs.values())))))
    for r in rows:
        print(f"{r[0]:10s} loss {r[1]:.2e}  worst {r[3]:.4f} ({r[2]})  median {r[4]:.4f}")


if __name__ == "__main__":
    main()
