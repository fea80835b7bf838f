"""BERTModel -- same API as the reference ``BS/models/bert.py:6-16``.

``forward(x)`` returns the full-vocabulary logits (B, T, V+1) like the
reference; training through :class:`rbm_amd.train_step.FusedTrainStep` uses the
labelled-rows-only loss head instead (same loss and gradients).  ``predict(x,
candidates)`` gives the validation scores ``forward(x)[:, -1, :].gather(1,
candidates)`` (``BS/trainers/bert.py:43-49``) without forming the (B, T, V+1)
logits (51 GB fp32 at a 1M-item catalogue and B = 64).
"""
import torch
import torch.nn as nn

from ..engine_util import as_ids, compute_dtype, require_cuda
from .base import BaseModel
from .bert_model.bert import BERT, BERTEngine, _BERTFunction, build_flat


class BERTModel(BaseModel):
    def __init__(self, args):
        super().__init__(args)
        self.bert = BERT(args)
        self.out = nn.Linear(self.bert.hidden, args.num_items + 1)
        self.cdtype = compute_dtype(args)
        self._flat = None
        self._engine = None
        if torch.device(getattr(args, "device", "cpu")).type == "cuda":
            self.to(args.device)

    @classmethod
    def code(cls):
        return 'bert'

    def _apply(self, fn, recurse=True):
        # (re)build the flat parameter buffer eagerly on .to(cuda), before any optimizer is created over
        # model.parameters() (the reference builds its Adam after model.to(device), base.py:21,38)
        super()._apply(fn, recurse)
        p = self.out.weight
        self._flat = build_flat(self, p.device) if p.device.type == "cuda" else None
        self._engine = None
        return self

    def engine(self):
        p = self.out.weight
        require_cuda(p.device)
        if self._flat is None or not self._flat.is_bound(self):
            self._flat = build_flat(self, p.device)
            self._engine = None
        if self._engine is None:
            self._engine = BERTEngine(self, self._flat)
        return self._engine

    @torch.no_grad()
    def predict(self, x, candidates):
        """(B, C) fp32 scores of the last position at ``candidates`` (long ids): the same values as
        ``self(x)[:, -1, :].gather(1, candidates)`` (the reference's calculate_metrics), eval-mode encoder."""
        eng = self.engine()
        dev = self._flat.device
        return eng.predict(as_ids(x, dev), as_ids(candidates, dev))

    def forward(self, x):
        eng = self.engine()
        ids = as_ids(x, self._flat.device)
        params = [p for _, p in self.named_parameters()]
        return _BERTFunction.apply(eng, ids, self.training, *params)
