"""A model written the way the reference's plugins are (test fixture, not product code).

It subclasses the plugin API's ``GeneralRecommender``, keeps its normalised adjacency as a plain
torch sparse COO attribute and propagates with ``torch.sparse.mm(self.norm_adj_matrix, x)`` followed
by ``torch.stack(...).mean(1)`` -- the operator boundary of reference lightgcn.py:134-147 /
cikm_model.py:187,199.  Nothing in it knows about the engine: the Trainer's
``swap_sparse_attributes`` replaces the COO attribute by an ``Adjacency`` and the same calls then
dispatch (with autograd) to the HIP SpMM.

Its computation is LightGCN's (ego = [user table ; Linear(text table)], L layers, BPR + EmbLoss on
the ego rows, lightgcn.py:122-179), with the parameters and the adjacency taken from the reference's
golden (tests/golden/model_LightGCN.npz) instead of being initialised here.
"""
import torch
from torch import nn

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.loss import BPRLoss, EmbLoss


class PropagationStub(GeneralRecommender):
    def __init__(self, config, dataset, golden):
        super().__init__(config, dataset)
        self.n_layers = config["n_layers"]
        self.reg_weight = config["reg_weight"]
        sd = {k[3:]: torch.from_numpy(golden[k].copy()) for k in golden.files if k.startswith("sd/")}
        self.user_embedding = nn.Embedding.from_pretrained(sd["user_embedding.weight"], freeze=False)
        self.item_embedding = nn.Embedding.from_pretrained(sd["item_embedding.weight"], freeze=False)
        self.image_embedding = nn.Embedding.from_pretrained(sd["image_embedding.weight"], freeze=False)
        self.image_trs = nn.Linear(*sd["image_trs.weight"].shape[::-1])
        with torch.no_grad():
            self.image_trs.weight.copy_(sd["image_trs.weight"])
            self.image_trs.bias.copy_(sd["image_trs.bias"])
        idx = torch.from_numpy(golden["adj/norm_adj_matrix/indices"].copy())
        val = torch.from_numpy(golden["adj/norm_adj_matrix/values"].copy())
        shape = tuple(int(x) for x in golden["adj/norm_adj_matrix/shape"])
        self.norm_adj_matrix = torch.sparse_coo_tensor(idx, val, shape).coalesce().to(self.device)
        self.mf_loss = BPRLoss()
        self.reg_loss = EmbLoss()

    def forward(self):
        x = torch.cat([self.user_embedding.weight, self.image_trs(self.image_embedding.weight)], dim=0)
        layers = [x]
        for _ in range(self.n_layers):
            x = torch.sparse.mm(self.norm_adj_matrix, x)
            layers.append(x)
        out = torch.stack(layers, dim=1).mean(dim=1)
        return torch.split(out, [self.n_users, self.n_items])

    def calculate_loss(self, batch):
        user, pos, neg = batch["u_id"], batch["pos_i_id"], batch["neg_i_id"]
        users, items = self.forward()
        u = users[user]
        s_pos = (u * items[pos]).sum(dim=1)
        s_neg = (u * items[neg]).sum(dim=1)
        reg = self.reg_weight * self.reg_loss(self.user_embedding(user), self.item_embedding(pos),
                                              self.item_embedding(neg))
        return self.mf_loss(s_pos, s_neg), reg
