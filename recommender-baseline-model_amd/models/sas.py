"""SASModel wrapper -- same API as the reference ``BS/models/sas.py:6-19``."""
from .base import BaseModel
from .sas_model.sas import SAS


class SASModel(BaseModel):
    def __init__(self, args):
        super().__init__(args)
        self.sas = SAS(args)

    @classmethod
    def code(cls):
        return 'sas'

    def forward(self, log_seqs, pos_seqs, neg_seqs):  # for training
        return self.sas(log_seqs, pos_seqs, neg_seqs)

    def predict(self, log_seqs, item_indices):  # for inference
        return self.sas.predict(log_seqs, item_indices)
