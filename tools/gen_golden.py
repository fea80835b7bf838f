"""Generate golden vectors by importing the REFERENCE code (container-only).

Runs the reference's own ``SASModel`` / ``BERTModel`` (``BS/models``) and the
reference trainers' ``calculate_loss`` (``BS/trainers/sas.py:34-54``,
``BS/trainers/bert.py:30-41``) on small seeded inputs and writes
``tests/golden/*.npz``: weights, inputs, logits, loss, every gradient (fp32, plus
an fp64 re-run for the tolerance floor), a 1000-step SAS Adam loss curve, a
300-step BERT loss curve and ranking-metric known answers
(``BS/trainers/utils.py:28-57``).

The reference never travels to the GPU box; this script refuses to run when
``/root/reference`` is absent.  Nothing is written into the reference tree:
bytecode writing is disabled and the CWD is switched to a temp dir.

    python tools/gen_golden.py                 # all fixtures
    python tools/gen_golden.py --bench-curve   # the 1000-step loss curve at the benchmarked shape
    python tools/gen_golden.py --bench-hr      # 1000 training steps + HR@10 at the benchmarked configuration
"""
import argparse
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
REF = "/root/reference/NerualNetwork/bert4rec&sas4rec"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")

if not os.path.isdir(REF):
    raise SystemExit("gen_golden: /root/reference is absent; fixtures are generated in the build container only")

import numpy as np  # noqa: E402
import torch  # noqa: E402

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object          # BS/trainers/base.py:10 imports it; tensorboard is not installed
sys.modules["torch.utils.tensorboard"] = _tb
sys.path.insert(0, REF)
sys.path.insert(0, ROOT)
os.chdir(tempfile.mkdtemp())

from models import model_factory  # noqa: E402  (reference)
from trainers.sas import SASTrainer  # noqa: E402  (reference)
from trainers.bert import BERTTrainer  # noqa: E402  (reference)
from trainers.utils import recalls_ndcgs_and_mrr_for_ks  # noqa: E402  (reference)
import rbm_amd.data as synth  # noqa: E402  (this repo: synthetic batches)

torch.set_num_threads(8)


def sas_args(V, T, d, L, h, p=0.0):
    return argparse.Namespace(model_code="sas", num_items=V, max_len=T, device="cpu", sas_hidden_units=d,
                              sas_num_blocks=L, sas_heads=h, sas_dropout=p, l2_emb=0.0)


def bert_args(V, T, d, L, h, p=0.0, hp=0.0, seed=0):
    return argparse.Namespace(model_code="bert", num_items=V, max_len=T, device="cpu", bert_hidden_units=d,
                              bert_num_blocks=L, bert_num_heads=h, bert_dropout=p, bert_hidden_dropout=hp,
                              bert_mask_prob=0.2, model_init_seed=seed)


class _FakeSAS:   # the attributes SASTrainer.calculate_loss reads
    def __init__(self, model, args):
        self.model, self.args = model, args
        self.bce_criterion = torch.nn.BCEWithLogitsLoss()
        self.l2_emb = args.l2_emb


class _FakeBERT:  # the attributes BERTTrainer.calculate_loss reads
    def __init__(self, model, args):
        self.model, self.args, self.device = model, args, args.device
        self.ce = torch.nn.CrossEntropyLoss(ignore_index=0)


def _pack(prefix, sd):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in sd.items()}


def sas_case(name, V, T, d, L, h, B, seed, shape="ml-1m"):
    torch.manual_seed(seed)
    args = sas_args(V, T, d, L, h)
    model = model_factory(args)
    model.train()
    rng = np.random.default_rng(seed)
    seq, pos, neg = synth.sas_batch(rng, B, T, V, shape=shape)
    out = {"V": V, "T": T, "d": d, "L": L, "h": h, "B": B, "seq": seq, "pos": pos, "neg": neg}
    out.update(_pack("p/", model.state_dict()))
    model.zero_grad()
    pl, nl = model(seq, pos, neg)
    loss = SASTrainer.calculate_loss(_FakeSAS(model, args), (seq, pos, neg))
    loss.backward()
    out.update({"pos_logits": pl.detach().numpy(), "neg_logits": nl.detach().numpy(),
                "loss": np.float64(loss.item())})
    out.update({"g/" + k: p.grad.numpy().copy() for k, p in model.named_parameters()})
    # candidate scoring (SAS.predict, sas.py:107-118) on 1 positive + 20 negatives
    cand = np.concatenate([pos[:, -1:], rng.integers(1, V + 1, size=(B, 20))], axis=1)
    with torch.no_grad():
        model.eval()
        out["cand"] = cand
        out["cand_scores"] = model.predict(seq, cand).numpy()
        model.train()
    # fp64 re-run of the same math: the reference's own fp32 noise floor
    m64 = model.double()
    m64.zero_grad()
    pl64, nl64 = m64(seq, pos, neg)
    idx = np.where(pos != 0)
    bce = torch.nn.BCEWithLogitsLoss()
    l64 = bce(pl64[idx], torch.ones_like(pl64[idx])) + bce(nl64[idx], torch.zeros_like(nl64[idx]))
    l64.backward()
    out.update({"pos_logits64": pl64.detach().numpy(), "neg_logits64": nl64.detach().numpy(),
                "loss64": np.float64(l64.item())})
    out.update(_drift(out, m64))
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "loss", loss.item(), "loss64", l64.item())


def _drift(out, m64):
    """Per-tensor norm-relative fp32-vs-fp64 gradient drift of the reference itself."""
    res = {}
    for k, p in m64.named_parameters():
        g64 = p.grad.numpy()
        res["drift/" + k] = np.float64(np.linalg.norm(out["g/" + k] - g64) / max(np.linalg.norm(g64), 1e-30))
    return res


def bert_case(name, V, T, d, L, h, B, seed):
    args = bert_args(V, T, d, L, h, seed=seed)
    model = model_factory(args)      # BERT.__init__ seeds with model_init_seed (bert.py:12)
    model.train()
    rng = np.random.default_rng(seed + 100)
    tokens, labels = synth.bert_batch(rng, B, T, V, mask_prob=0.3)
    out = {"V": V, "T": T, "d": d, "L": L, "h": h, "B": B, "tokens": tokens, "labels": labels}
    out.update(_pack("p/", model.state_dict()))
    model.zero_grad()
    batch = (torch.from_numpy(tokens), torch.from_numpy(labels))
    logits = model(batch[0])
    loss = BERTTrainer.calculate_loss(_FakeBERT(model, args), batch)
    loss.backward()
    out.update({"logits": logits.detach().numpy(), "loss": np.float64(loss.item())})
    out.update({"g/" + k: p.grad.numpy().copy() for k, p in model.named_parameters()})
    m64 = model.double()
    m64.zero_grad()
    lg64 = m64(batch[0])
    l64 = torch.nn.functional.cross_entropy(lg64.view(-1, lg64.shape[-1]), batch[1].view(-1), ignore_index=0)
    l64.backward()
    lg = lg64.detach().numpy()
    out.update({"logits_drift": np.float64(np.linalg.norm(out["logits"] - lg) / np.linalg.norm(lg)),
                "loss64": np.float64(l64.item())})
    out.update(_drift(out, m64))
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "loss", loss.item(), "loss64", l64.item())


def _sas_train(model, args, B, T, V, steps, seed, lr):
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=0)   # BS/trainers/base.py:228
    fake = _FakeSAS(model, args)
    rng = np.random.default_rng(seed)
    zipf = synth.ZipfItems(V)
    losses = []
    for _ in range(steps):                                             # BS/trainers/base.py:114-123
        batch = synth.sas_batch(rng, B, T, V, zipf=zipf)
        opt.zero_grad()
        loss = SASTrainer.calculate_loss(fake, batch)
        losses.append(loss.item())
        loss.backward()
        opt.step()
    return np.array(losses, np.float64)


def sas_curve(name, V, T, d, L, h, B, steps, seed, lr=1e-3, final=True, also64=False):
    """The reference's own training run (SASTrainer.calculate_loss + backward + Adam) on the deterministic batch
    stream; also64: the same run with the reference modules in float64 (its exact-math trajectory)."""
    torch.manual_seed(seed)
    args = sas_args(V, T, d, L, h)
    model = model_factory(args)
    model.train()
    out = {"V": V, "T": T, "d": d, "L": L, "h": h, "B": B, "steps": steps, "seed": seed, "lr": lr}
    out.update(_pack("p/", model.state_dict()))
    m64 = None
    if also64:
        import copy
        m64 = copy.deepcopy(model).double()
    out["losses"] = _sas_train(model, args, B, T, V, steps, seed, lr)
    if final:
        out.update(_pack("final/", model.state_dict()))
    if m64 is not None:
        torch.set_default_dtype(torch.float64)    # the trainer's label tensors follow the logits' dtype
        try:
            out["losses64"] = _sas_train(m64, args, B, T, V, steps, seed, lr)
        finally:
            torch.set_default_dtype(torch.float32)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, out["losses"][0], "->", out["losses"][-1],
          "" if m64 is None else f"max |fp32 - fp64| {np.abs(out['losses'] - out['losses64']).max():.2e}")


def bert_curve(name, V, T, d, L, h, B, steps, seed, lr=1e-3):
    args = bert_args(V, T, d, L, h, seed=seed)
    model = model_factory(args)
    model.train()
    out = {"V": V, "T": T, "d": d, "L": L, "h": h, "B": B, "steps": steps, "seed": seed, "lr": lr}
    out.update(_pack("p/", model.state_dict()))
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=0)
    fake = _FakeBERT(model, args)
    rng = np.random.default_rng(seed)
    zipf = synth.ZipfItems(V)
    losses = []
    for _ in range(steps):
        tok, lab = synth.bert_batch(rng, B, T, V, mask_prob=0.3, zipf=zipf)
        opt.zero_grad()
        loss = BERTTrainer.calculate_loss(fake, (torch.from_numpy(tok), torch.from_numpy(lab)))
        losses.append(loss.item())
        loss.backward()
        opt.step()
    out["losses"] = np.array(losses, np.float64)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, losses[0], "->", losses[-1])


def metrics_case(name):
    rng = np.random.default_rng(5)
    B, C = 32, 101
    scores = rng.standard_normal((B, C)).astype(np.float32)
    labels = np.zeros((B, C), np.int64)
    labels[:, 0] = 1
    labels[:4, 1:3] = 1                 # a few multi-positive rows
    scores[5:9, 0] += 3.0               # a few confident hits
    ks = [1, 5, 10, 20]
    m = recalls_ndcgs_and_mrr_for_ks(torch.from_numpy(scores), torch.from_numpy(labels), ks)
    out = {"scores": scores, "labels": labels, "ks": np.array(ks)}
    out.update({"m/" + k: np.float64(v) for k, v in m.items()})
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, m["Recall@10"], m["NDCG@10"])


def _hashes(sd):
    """sha256 of each tensor's float32 bytes: pins an initialisation without storing it."""
    import hashlib
    return {k: hashlib.sha256(v.detach().cpu().float().numpy().tobytes()).hexdigest() for k, v in sd.items()}


def _ref_eval(model, seq, cand, labels, ks, chunk=512):
    """The reference's validate() scoring (BS/trainers/sas.py:56-62: model.predict on the candidates) over the whole
    eval set, ranked once by its recalls_ndcgs_and_mrr_for_ks (BS/trainers/utils.py:28-57)."""
    model.eval()
    with torch.no_grad():
        sc = torch.cat([model.predict(torch.from_numpy(seq[i:i + chunk]), torch.from_numpy(cand[i:i + chunk]))
                        for i in range(0, len(seq), chunk)])
    model.train()
    return sc.numpy(), recalls_ndcgs_and_mrr_for_ks(sc, torch.from_numpy(labels), ks)


HR = dict(V=3416, T=200, d=128, L=2, h=1, B=128, p=0.2, steps=1000, lr=1e-3, users=6040, init_seed=8, data_seed=11,
          batch_seed=12, eval_seed=13)


def sas_hr_bench(name="sas_hr_bench"):
    """HR@10 at the benchmarked configuration (BASELINE configs[1]: V 3,416, T 200, d 128, 2 blocks, 1 head, B 128,
    dropout 0.2): the reference's own SASModel trained by its own calculate_loss + Adam for 1000 steps on
    leave-one-out WarpSampler batches (rbm_amd.data.loo_*), then evaluated as its validate() does on all users with
    1 + 100 candidates.  Stores the reference's init hashes, final weights, losses and metrics (init and final)."""
    c = HR
    V, T, d, L, h, B = c["V"], c["T"], c["d"], c["L"], c["h"], c["B"]
    ks = [1, 5, 10, 20]
    train, val, test = synth.loo_users(np.random.default_rng(c["data_seed"]), c["users"], T, V)
    seq, cand, labels = synth.loo_eval_set(np.random.default_rng(c["eval_seed"]), train, val, test, T, V)
    torch.manual_seed(c["init_seed"])
    args = sas_args(V, T, d, L, h, p=c["p"])
    model = model_factory(args)
    model.train()
    out = {k: np.float64(v) if isinstance(v, float) else np.int64(v) for k, v in c.items()}
    out["ks"] = np.array(ks)
    out.update({"init_sha/" + k: np.array(v) for k, v in _hashes(model.state_dict()).items()})
    out["eval_checksum"] = np.int64(int((seq * 31 + 7).sum() + (cand * 131).sum()))
    sc0, m0 = _ref_eval(model, seq, cand, labels, ks)
    out.update({"m0/" + k: np.float64(v) for k, v in m0.items()})
    opt = torch.optim.Adam(model.parameters(), lr=c["lr"], weight_decay=0)   # BS/trainers/base.py:225-228
    fake = _FakeSAS(model, args)
    rng = np.random.default_rng(c["batch_seed"])
    losses, csum = [], 0
    for i in range(c["steps"]):                                              # BS/trainers/base.py:114-123
        batch = synth.loo_train_batch(rng, train, B, T, V)
        csum += int(sum(((j + 1) * x).sum() for j, x in enumerate(batch)) % (1 << 40))
        opt.zero_grad()
        loss = SASTrainer.calculate_loss(fake, batch)
        losses.append(loss.item())
        loss.backward()
        opt.step()
        if i % 100 == 0:
            print(name, "step", i, losses[-1], flush=True)
    out["batch_checksum"] = np.int64(csum)
    out["losses"] = np.array(losses, np.float64)
    out.update(_pack("final/", model.state_dict()))
    sc1, m1 = _ref_eval(model, seq, cand, labels, ks)
    out.update({"m/" + k: np.float64(v) for k, v in m1.items()})
    out["scores_head"] = sc1[:512]                   # the reference's fp32 scores of the first 512 users
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "Recall@10 init", m0["Recall@10"], "trained", m1["Recall@10"], "loss", losses[0], "->", losses[-1])


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    if "--bench-hr" in sys.argv:
        sas_hr_bench()
        raise SystemExit(0)
    if "--bench-curve" in sys.argv:
        # the benchmarked SAS shape (BASELINE configs[1]: ML-1M items, T = 200, d = 128, 2 blocks, 1 head)
        sas_curve("sas_curve_bench", V=3416, T=200, d=128, L=2, h=1, B=16, steps=1000, seed=8, final=False,
                  also64=True)
        raise SystemExit(0)
    sas_case("sas_tiny", V=50, T=16, d=64, L=2, h=2, B=4, seed=1)
    sas_case("sas_mid", V=400, T=200, d=128, L=2, h=1, B=3, seed=2)
    bert_case("bert_tiny", V=50, T=16, d=64, L=2, h=2, B=4, seed=3)
    bert_case("bert_mid", V=300, T=64, d=128, L=2, h=2, B=3, seed=4)
    sas_curve("sas_curve", V=50, T=16, d=64, L=2, h=2, B=8, steps=1000, seed=6)
    bert_curve("bert_curve", V=50, T=16, d=64, L=2, h=2, B=8, steps=300, seed=7)
    metrics_case("metrics")
