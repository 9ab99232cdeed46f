"""BPRMF (BASELINE config 1) on the MI355X engine.

The reference ships no BPRMF; semantics follow its plugin style:
LightGCN (models/lightgcn.py) with zero propagation layers and ID item embeddings, BPRLoss +
reg_weight * EmbLoss on the same rows.  Training runs entirely in the fused BPR kernels.
"""
import torch
from torch import nn

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.init import xavier_uniform_initialization
from FoodRec.common.loss import BPRLoss, EmbLoss
from FoodRec.engine import ops


class BPRMF(GeneralRecommender):
    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.dataset = dataset
        self.latent_dim = config["embedding_size"]
        self.reg_weight = config["reg_weight"]
        self.user_embedding = nn.Embedding(self.n_users, self.latent_dim)
        self.item_embedding = nn.Embedding(self.n_items, self.latent_dim)
        self.mf_loss = BPRLoss()
        self.reg_loss = EmbLoss()
        self.apply(xavier_uniform_initialization)

    def forward(self):
        return self.user_embedding.weight, self.item_embedding.weight, None

    def calculate_loss(self, batch_data):
        U, I = self.user_embedding.weight, self.item_embedding.weight
        mf, emb = ops.bpr_emb_loss(U, I, U, I, batch_data["u_id"], batch_data["pos_i_id"], batch_data["neg_i_id"])
        return mf, self.reg_weight * emb

    # inference_fast below is the plain gather-dot of forward()'s tables: the trainer may score the
    # evaluation lists with fr_score_segments instead (no [n, 64] gathers)
    fused_scores = True

    def inference_fast(self, batch_data, user_emb, item_emb):
        return torch.mul(user_emb[batch_data["user_input"]], item_emb[batch_data["item_input"]]).sum(dim=1)

    def inference_by_user(self, batch_data):
        u, i, _ = self.forward()
        return self.inference_fast(batch_data, u, i)
