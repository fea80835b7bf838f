"""BERTModel wrapper -- same API as the reference ``BS/models/bert.py:6-16``."""
from .base import BaseModel


class BERTModel(BaseModel):
    def __init__(self, args):
        super().__init__(args)
        raise NotImplementedError("BERT4Rec HIP path: in progress")

    @classmethod
    def code(cls):
        return 'bert'
