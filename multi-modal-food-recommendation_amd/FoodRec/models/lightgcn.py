"""LightGCN on the MI355X engine (reference: models/lightgcn.py).

Same parameters, init order and state_dict keys as the reference; forward() is the fused
propagation (one HIP SpMM per layer with the layer mean in the epilogue) and calculate_loss
the fused gather-dot-BPR + EmbLoss kernels.  Reference quirks kept: ego item rows are
``image_trs(text features)`` and ``image_trs`` keeps torch's default init (created after the
xavier pass, lightgcn.py:73-74,129); EmbLoss regularises the (otherwise unused)
``item_embedding`` rows.
"""
import torch
from torch import nn

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.init import xavier_uniform_initialization
from FoodRec.common.loss import BPRLoss, EmbLoss
from FoodRec.engine import ops
from FoodRec.models._graphs import ui_adjacency


class LightGCN(GeneralRecommender):
    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.config = config
        self.dataset = dataset
        self.device = config["device"]
        self.latent_dim = config["embedding_size"]
        self.n_layers = config["n_layers"]
        self.reg_weight = config["reg_weight"]
        self.user_embedding = nn.Embedding(self.n_users, self.latent_dim)
        self.item_embedding = nn.Embedding(self.n_items, self.latent_dim)
        self.mf_loss = BPRLoss()
        self.reg_loss = EmbLoss()
        self.restore_user_e = None
        self.restore_item_e = None
        self.norm_adj_matrix = ui_adjacency(dataset, self.n_users, self.n_items, self.device)
        self.apply(xavier_uniform_initialization)
        self.other_parameter_name = ["restore_user_e", "restore_item_e"]
        self.image_embedding = nn.Embedding.from_pretrained(self.t_feat, freeze=False)
        self.image_trs = nn.Linear(self.t_feat.shape[1], self.latent_dim)

    def get_ego_embeddings(self):
        return torch.cat([self.user_embedding.weight, self.image_trs(self.image_embedding.weight)], dim=0)

    def forward(self):
        out = ops.propagate_mean(self.norm_adj_matrix, self.get_ego_embeddings(), self.n_layers)
        user_all, item_all = torch.split(out, [self.n_users, self.n_items])
        return user_all, item_all

    def calculate_loss(self, batch_data):
        self.restore_user_e = self.restore_item_e = None
        user_all, item_all = self.forward()
        mf, emb = ops.bpr_emb_loss(user_all, item_all, self.user_embedding.weight, self.item_embedding.weight,
                                   batch_data["u_id"], batch_data["pos_i_id"], batch_data["neg_i_id"])
        return mf, self.reg_weight * emb

    # inference_fast below is the plain gather-dot of forward()'s tables: the trainer may score the
    # evaluation lists with fr_score_segments instead (no [n, 64] gathers)
    fused_scores = True

    def inference_fast(self, batch_data, user_emb, item_emb):
        return torch.mul(user_emb[batch_data["user_input"]], item_emb[batch_data["item_input"]]).sum(dim=1)

    def inference_by_user(self, batch_data):
        user_all, item_all = self.forward()
        return self.inference_fast(batch_data, user_all, item_all)
