"""Golden vectors for oracle/sampling.py from the REFERENCE's batch builders (container-only).

Runs the reference's ``sample_function`` (``BS/dataloaders/sas.py:65-86``: ``sample()`` + ``random_neq``) and
``BertTrainDataset.__getitem__`` (``BS/dataloaders/bert.py:64-110``) on small seeded histories, recording every
random draw they consume (numpy's ``randint`` for the SAS user and negative indices; the dataset's ``rng.rand`` /
``rng.randint`` for masking), and writes ``tests/golden/sampling.npz``: the histories, the draws, and the
reference's batches.  ``tests/test_oracle_sampling.py`` replays the oracle on those draws and must reproduce the
reference's batches exactly -- the pin of the oracle the GPU sampler tests compare against.

The reference never travels to the GPU box; this script refuses to run when ``/root/reference`` is absent and
writes nothing into the reference tree (no bytecode, temp CWD).

    python tools/gen_golden_sampling.py
"""
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
REF = "/root/reference/NerualNetwork/bert4rec&sas4rec"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "sampling.npz")

if not os.path.isdir(REF):
    raise SystemExit("gen_golden_sampling: /root/reference is absent; fixtures are generated in the build container")

import numpy as np  # noqa: E402

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb
sys.path.insert(0, REF)
os.chdir(tempfile.mkdtemp())

import dataloaders.sas as ref_sas  # noqa: E402  (reference)
from dataloaders.bert import BertTrainDataset  # noqa: E402  (reference)


class _Stop(Exception):
    pass


class _OneBatch:
    """result_queue for sample_function: keeps the first batch, then stops the worker's infinite loop."""
    def __init__(self):
        self.batch = None

    def put(self, item):
        self.batch = [list(x) for x in item]
        raise _Stop


def _histories(rng, n, V, lo, hi):
    return [list(map(int, rng.integers(1, V + 1, size=int(rng.integers(lo, hi + 1))))) for _ in range(n)]


def _csr(hist):
    off = np.zeros(len(hist) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hist])
    return off, np.array([i for h in hist for i in h], np.int64)


def sas_case(seed, n_users, V, T, B, lo, hi):
    rng = np.random.default_rng(seed)
    users = _histories(rng, n_users, V, lo, hi)
    calls = []
    real = np.random.randint

    def rec(*a, **k):
        out = real(*a, **k)
        calls.append(np.array(out, np.int64).reshape(-1))
        return out
    np.random.seed(seed)
    ref_sas.np.random.randint = rec
    q = _OneBatch()
    try:
        ref_sas.sample_function(users, V, B, T, q)
    except _Stop:
        pass
    finally:
        ref_sas.np.random.randint = real
    seqs, poss, negs = (np.array(x, np.int64) for x in q.batch)
    assert len(calls) == 2 * B, len(calls)
    u = np.array([int(calls[2 * b][0]) for b in range(B)], np.int64)
    return users, u, seqs, poss, negs


def bert_case(seed, n_users, V, T, p, lo, hi):
    rng = np.random.default_rng(seed)
    users = _histories(rng, n_users, V, lo, hi)
    log = []

    class RecRng:
        def rand(self):
            x = np.random.rand()
            log.append(("r", float(x)))
            return x

        def randint(self, a, b):
            x = np.random.randint(a, b)
            log.append(("i", int(x)))
            return x
    np.random.seed(seed)
    ds = BertTrainDataset(users, T, p, V + 1, V, RecRng())
    toks, labs, draws = [], [], []
    for u in range(n_users):
        start = len(log)
        t, lab = ds[u]
        per = []
        for kind, x in log[start:]:
            if kind == "r":
                per.append([x, -1.0])
            else:
                per[-1][1] = float(x)
        assert len(per) == len(users[u])
        toks.append(t.numpy())
        labs.append(lab.numpy())
        draws.append(np.array(per, np.float64))
    return users, np.stack(toks), np.stack(labs), draws


def main():
    out = {}
    for name, args in {"sas_a": (11, 40, 60, 50, 32, 1, 120), "sas_b": (12, 100, 3416, 200, 16, 1, 400),
                       "sas_c": (13, 20, 30, 8, 20, 1, 3)}.items():
        users, u, s, p_, n = sas_case(*args)
        off, items = _csr(users)
        out.update({f"{name}/off": off, f"{name}/items": items, f"{name}/user": u, f"{name}/seq": s,
                    f"{name}/pos": p_, f"{name}/neg": n, f"{name}/V": np.int64(args[2]), f"{name}/T": np.int64(args[3])})
    for name, args in {"bert_a": (21, 30, 700, 40, 0.3, 1, 90), "bert_b": (22, 12, 26744, 200, 0.2, 150, 400),
                       "bert_c": (23, 10, 50, 10, 1.0, 1, 30)}.items():
        users, t, lab, draws = bert_case(*args)
        off, items = _csr(users)
        out.update({f"{name}/off": off, f"{name}/items": items, f"{name}/tokens": t, f"{name}/labels": lab,
                    f"{name}/draws": np.concatenate(draws), f"{name}/V": np.int64(args[2]),
                    f"{name}/T": np.int64(args[3]), f"{name}/p": np.float64(args[4])})
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sum(v.nbytes for v in out.values()), "bytes")


if __name__ == "__main__":
    main()
