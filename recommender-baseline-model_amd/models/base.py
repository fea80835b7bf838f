"""BaseModel -- same contract as the reference ``BS/models/base.py:6-14``."""
from abc import ABCMeta, abstractmethod

import torch.nn as nn


class BaseModel(nn.Module, metaclass=ABCMeta):
    def __init__(self, args):
        super().__init__()
        self.args = args

    @classmethod
    @abstractmethod
    def code(cls):
        pass
