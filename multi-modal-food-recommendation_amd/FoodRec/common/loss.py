"""Loss modules with the reference's semantics (common/loss.py:8-60).

These are the forms unchanged reference models call (they compute the scores themselves).
Engine-native models use FoodRec.engine.ops.bpr_emb_loss, which fuses the gathers, dot
products, BPR and EmbLoss into two HIP kernels.
"""
import torch
import torch.nn as nn


class BPRLoss(nn.Module):
    """-log(gamma + sigmoid(pos - neg)).mean(); gamma kept for parity (loss.py:29-34)."""

    def __init__(self, gamma=1e-10):
        super().__init__()
        self.gamma = gamma

    def forward(self, pos_score, neg_score):
        return -torch.log(self.gamma + torch.sigmoid(pos_score - neg_score)).mean()


class EmbLoss(nn.Module):
    """Sum of (un-squared) Frobenius norms / rows of the LAST argument; shape [1] (loss.py:37-50)."""

    def __init__(self, norm=2):
        super().__init__()
        self.norm = norm

    def forward(self, *embeddings):
        emb_loss = torch.zeros(1, device=embeddings[-1].device)
        for embedding in embeddings:
            emb_loss = emb_loss + torch.norm(embedding, p=self.norm)
        return emb_loss / embeddings[-1].shape[0]


class L2Loss(nn.Module):
    def forward(self, *embeddings):
        l2 = torch.zeros(1, device=embeddings[-1].device)
        for embedding in embeddings:
            l2 = l2 + torch.sum(embedding ** 2) * 0.5
        return l2
