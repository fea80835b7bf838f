"""CPU oracle for the SASRec / BERT4Rec training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this
module; only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of ``bench.py`` use it, and only as the checker / the CPU baseline.

What it is: a from-scratch functional restatement, in PyTorch-CPU (fp32 or
fp64), of the reference math in Furyton/Recommender-Baseline-Model
``NerualNetwork/bert4rec&sas4rec`` (abbreviated ``BS/`` in citations):

* :mod:`oracle.sas`     -- ``BS/models/sas_model/sas.py`` + ``BS/trainers/sas.py``
* :mod:`oracle.bert`    -- ``BS/models/bert_modules/**`` + ``BS/models/bert.py``
                           + ``BS/trainers/bert.py``
* :mod:`oracle.optim`   -- ``torch.optim.Adam`` as used by ``BS/trainers/base.py:225-233``
* :mod:`oracle.metrics` -- ``BS/trainers/utils.py:28-57``

Pinning: every function here is checked against golden vectors produced by
importing the reference itself in the build container
(``tools/gen_golden.py`` -> ``tests/golden/*.npz``; ``tests/test_oracle.py``).
Backward passes are torch autograd over the restated forward math.
"""
