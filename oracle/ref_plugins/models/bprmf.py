"""ORACLE plugin (test infrastructure only): BPRMF written in the reference's plugin style.

BASELINE config 1 names BPRMF, but the reference ships no such model.  This
file is authored here (not copied) so the reference's own Trainer can run it in the golden
harness: `models` is a namespace package in the reference, so putting this directory on
sys.path makes get_model('BPRMF') (utils/utils.py:27-40) resolve it.  Semantics = LightGCN
(models/lightgcn.py) with zero propagation layers and ID item embeddings.
"""
import torch
from torch import nn

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.init import xavier_uniform_initialization
from FoodRec.common.loss import BPRLoss, EmbLoss


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
        user, pos, neg = batch_data['u_id'], batch_data['pos_i_id'], batch_data['neg_i_id']
        u_all, i_all, _ = self.forward()
        u, p, n = u_all[user], i_all[pos], i_all[neg]
        mf = self.mf_loss(torch.mul(u, p).sum(dim=1), torch.mul(u, n).sum(dim=1))
        reg = self.reg_weight * self.reg_loss(u, p, n)
        return mf, reg

    def inference_fast(self, batch_data, user_emb, item_emb):
        return torch.mul(user_emb[batch_data['user_input']], item_emb[batch_data['item_input']]).sum(dim=1)

    def inference_by_user(self, batch_data):
        u_all, i_all, _ = self.forward()
        return self.inference_fast(batch_data, u_all, i_all)
