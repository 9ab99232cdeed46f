"""Xavier initialisation hooks (common/init.py:7-42), applied with ``module.apply``."""
import torch.nn as nn
from torch.nn.init import constant_, xavier_normal_, xavier_uniform_


def xavier_normal_initialization(module):
    if isinstance(module, nn.Embedding):
        xavier_normal_(module.weight.data)
    elif isinstance(module, nn.Linear):
        xavier_normal_(module.weight.data)
        if module.bias is not None:
            constant_(module.bias.data, 0)


def xavier_uniform_initialization(module):
    # note: overwrites the padding_idx row of an Embedding too (SURVEY parity quirk 9)
    if isinstance(module, (nn.Embedding, nn.Parameter)):
        xavier_uniform_(module.weight.data)
    elif isinstance(module, nn.Linear):
        xavier_uniform_(module.weight.data)
        if module.bias is not None:
            constant_(module.bias.data, 0)
