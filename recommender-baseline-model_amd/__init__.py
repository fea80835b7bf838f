"""MI355X-native SASRec / BERT4Rec training hot path (package ``rbm_amd``).

Mirrors the reference ``NerualNetwork/bert4rec&sas4rec`` model/trainer API
(``models.model_factory``, ``SASModel``, ``BERTModel``) while the per-step
hot path runs as hand-written HIP kernels for gfx950 behind the C ABI declared
in ``include/recsys_hip.h`` (``librecsys_hip.so``).  The reference trainer's
step body (``BS/trainers/base.py:114-123``) is ``train_step.FusedTrainStep``.

Importing the package does not load the native library; the first op call
does, and fails loudly if it is missing.
"""
__all__ = ["data", "models", "train_step"]
