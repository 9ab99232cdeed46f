"""SCHGN on the engine (reference models/schgn.py).

The reference file itself drops in unchanged (``get_model`` resolves ``models.schgn`` first; its
``import torch_geometric`` binds to FoodRec.engine.geometric's GCNConv when PyG is absent).  This is
the engine-native restatement used when the reference's ``models/`` is not on sys.path, with the
same parameters (state_dict keys), module registration order and seeded initialisation:

  * graph (schgn.py:139-151): edges item->user (uRecipe), ingredient->item (rIngre) and calorie
    level->item (rCalories) over the node space [users | items | ingredients | levels], built
    vectorised; one GCNConv(64, 64) + tanh over the concatenated tables (:29-41, 229-238) runs as
    one HIP SpMM per direction;
  * compute_score (:225-256): id + GCN embeddings, ingredient-level attention with the 1e12 length
    mask (:160-183), component attention over (id, ingredient, image, calorie) (:185-204), the
    W_concat / dropout(0.5) / ReLU / output_mlp head;
  * calculate_loss (:272-316): summed BPR log-sigmoid, the L2 terms, and the masked-ingredient SSL
    loss through the BERT encoder (:211-223);
  * inference_by_user / full_sort_predict / sample_sort_predict (:318-389).

One deliberate difference: the full-graph GCN output, identical for the positive and the negative
pass (no dropout inside), is computed once per training step and shared (the reference computes it
twice); values are the same, the two backward contributions are summed by autograd.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.module import Encoder, LayerNorm
from FoodRec.engine.geometric import GCNConv


def l2_loss(t):
    return torch.sum(t ** 2)


def truncated_normal_(tensor, mean=0.0, std=0.01):
    """schgn.py:18-26: per element, the first of four N(0, 1) draws inside (-2, 2) (the first draw
    when none is), scaled by std and shifted by mean.  Consumes 4 normals per element."""
    with torch.no_grad():
        draws = tensor.new_empty(tuple(tensor.shape) + (4,)).normal_()
        inside = (draws < 2) & (draws > -2)
        first = inside.max(-1, keepdim=True)[1]
        tensor.data.copy_(draws.gather(-1, first).squeeze(-1))
        tensor.data.mul_(std).add_(mean)
    return tensor


class GraphConv(nn.Module):
    """GCNConv + tanh with the reference's truncated-normal re-initialisation (:29-41)."""

    def __init__(self, in_channel, out_channel):
        super().__init__()
        self.in_channel, self.out_channel = in_channel, out_channel
        self.conv1 = GCNConv(in_channel, out_channel)
        std = float(np.sqrt(2.0 / (in_channel + out_channel)))
        truncated_normal_(self.conv1.lin.weight, std=std)
        truncated_normal_(self.conv1.bias, std=std)

    def forward(self, x, edge_index):
        return torch.tanh(self.conv1(x, edge_index))


def _tn_linear(lin: nn.Linear, w_std: float, b_std: float | None):
    truncated_normal_(lin.weight, std=w_std)
    if b_std is not None:
        truncated_normal_(lin.bias, std=b_std)


class SCHGN(GeneralRecommender):
    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.device = config["device"]
        self.config = config
        self.dataset = dataset
        self.n_users = dataset.n_users
        self.n_items = dataset.n_items
        self.n_cold = dataset.cold_num
        self.n_health = dataset.num_calories_level
        self.n_ingredients = dataset.num_ingredients
        self.img_size = dataset.image_size

        self.ingre_encoder = Encoder(n_layers=config["num_hidden_layers"], n_heads=config["num_attention_heads"],
                                     hidden_size=config["embedding_size"], inner_size=config["inner_size"],
                                     hidden_dropout_prob=config["hidden_dropout_prob"],
                                     attn_dropout_prob=config["attention_probs_dropout_prob"],
                                     hidden_act=config["hidden_act"], layer_norm_eps=1e-12)
        self.apply(self.init_weights)

        self.g2i_edges, self.i2u_edges = self.load_graph(dataset)
        self.new_gcn = GraphConv(64, 64)

        e = config["embedding_size"]
        self.emb_size = e
        self.regs = config["regs"]
        self.reg_image = config["reg_image"]
        self.reg_w = config["reg_w"]
        self.reg_g = config["reg_g"]
        self.reg_health = config["reg_health"]
        self.ssl = config["ssl"]

        # storage only; drawn by _init_weight below, after every Linear (the reference's order)
        self.user_embed = nn.Parameter(torch.empty(self.n_users, e), requires_grad=True)
        self.item_embed = nn.Parameter(torch.empty(self.n_items, e), requires_grad=True)
        self.ingre_embed_first = nn.Parameter(torch.empty(self.n_ingredients, e), requires_grad=True)
        self.ingre_embed_second = nn.Parameter(torch.zeros(1, e), requires_grad=False)  # padding row
        self.ingre_embed_mask = nn.Parameter(torch.empty(1, e), requires_grad=True)     # [MASK] row
        self.health_embed = nn.Parameter(torch.empty(self.n_health, e), requires_grad=True)

        self.img_trans = nn.Linear(self.img_size, e)
        s_img = float(np.sqrt(2.0 / (self.img_size + e)))
        _tn_linear(self.img_trans, s_img, s_img)
        s2 = float(np.sqrt(2.0 / (2 * e)))
        self.W_att_ingre = nn.Linear(3 * e, e)
        _tn_linear(self.W_att_ingre, float(np.sqrt(2.0 / (4 * e))), s2)
        self.h_att_ingre = nn.Linear(e, 1, bias=False)
        nn.init.ones_(self.h_att_ingre.weight)
        self.W_att_comp = nn.Linear(2 * e, e)
        _tn_linear(self.W_att_comp, float(np.sqrt(2.0 / (3 * e))), s2)
        self.h_att_comp = nn.Linear(e, 1, bias=False)
        nn.init.ones_(self.h_att_comp.weight)
        self.W_concat = nn.Linear(3 * e, e)
        _tn_linear(self.W_concat, float(np.sqrt(2.0 / (4 * e))), s2)
        self.output_mlp = nn.Linear(e, 1, bias=False)
        _tn_linear(self.output_mlp, s2, None)
        self.mip_norm = nn.Linear(e, e)
        self.criterion = nn.BCELoss(reduction="none")
        self._init_weight()

    def _init_weight(self):
        for p in (self.user_embed, self.item_embed, self.ingre_embed_first, self.ingre_embed_mask, self.health_embed):
            truncated_normal_(p, std=0.01)

    def init_weights(self, module):
        if isinstance(module, nn.Linear):
            truncated_normal_(module.weight, std=0.01)
        elif isinstance(module, LayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    def load_graph(self, dataset):
        """schgn.py:139-151, vectorised: (source, target) rows item->user, then ingredient->item and
        level->item, in the reference's edge order."""
        U, I, NI = self.n_users, self.n_items, self.n_ingredients
        ur = np.asarray(dataset.uRecipe_triples, np.int64).reshape(-1, 2)
        ri = np.asarray(dataset.rIngre_triples, np.int64).reshape(-1, 2)
        rc = np.asarray(dataset.rCalories_triples, np.int64).reshape(-1, 2)
        i2u = np.stack([ur[:, 1] + U, ur[:, 0]], 1)
        g2i = np.concatenate([np.stack([ri[:, 1] + U + I, ri[:, 0] + U], 1),
                              np.stack([rc[:, 1] + U + I + NI, rc[:, 0] + U], 1)])
        # the reference's (swapped) attribute names: g2i_edges holds item->user, i2u_edges the rest
        return (torch.from_numpy(i2u).to(self.device, dtype=torch.long),
                torch.from_numpy(g2i).to(self.device, dtype=torch.long))

    # ----------------------------------------------------------------------------- layers
    def sequence_mask(self, lengths, max_len):
        return (torch.arange(0, max_len, 1, device=lengths.device) < lengths.unsqueeze(-1)).float()

    def attention_ingredient_level(self, ingre_emb, u_emb, img_emb, ingre_num):
        n = ingre_emb.shape[1]
        ctx = torch.cat([ingre_emb, u_emb.unsqueeze(1).repeat(1, n, 1), img_emb.unsqueeze(1).repeat(1, n, 1)], dim=2)
        logits = self.h_att_ingre(torch.tanh(self.W_att_ingre(ctx))).squeeze()
        pad = (torch.ones_like(self.sequence_mask(ingre_num, n)) - self.sequence_mask(ingre_num, n)) * -1e12
        att = F.softmax(logits + pad, dim=1).unsqueeze(2)
        return torch.sum(att * ingre_emb, dim=1)

    def attention_id_ingre_image(self, u_emb, i_emb, ingre_att_emb, img_emb, hl_emb):
        b = u_emb.shape[0]
        parts = (i_emb, ingre_att_emb, img_emb, hl_emb)
        pairs = torch.cat([torch.cat([u_emb, c], dim=1) for c in parts], dim=0)
        w = F.softmax(self.h_att_comp(torch.tanh(self.W_att_comp(pairs))).view(b, -1), dim=1).unsqueeze(2)
        return torch.sum(w * torch.stack(parts, dim=1), dim=1)

    def masked_ingre_prediction(self, ingre_emb, target_emb):
        h = self.mip_norm(ingre_emb.view(-1, self.emb_size))
        return torch.sigmoid(torch.sum(h * target_emb.view(-1, self.emb_size), -1))

    def compute_ssl_loss(self, ingre_embedding, ingre_embedding_gcn, masked_ingre_seq, pos_ingre, neg_ingre):
        seq_mask = ((masked_ingre_seq == self.n_ingredients).float() * -1e8).unsqueeze(1).unsqueeze(1)
        encoded = self.ingre_encoder(ingre_embedding_gcn[masked_ingre_seq], seq_mask, output_all_encoded_layers=True)[-1]
        pos_score = self.masked_ingre_prediction(encoded, ingre_embedding[pos_ingre])
        neg_score = self.masked_ingre_prediction(encoded, ingre_embedding[neg_ingre])
        dist = torch.sigmoid(pos_score - neg_score)
        loss = self.criterion(dist, torch.ones_like(dist, dtype=torch.float32))
        masked = (masked_ingre_seq == self.n_ingredients + 1).float()
        return torch.sum(loss * masked.flatten())

    def _gcn(self):
        """tanh(GCNConv(x)) over [users | items | ingredients | levels] (schgn.py:229-238)."""
        x = torch.cat([self.user_embed, self.item_embed, self.ingre_embed_first, self.health_embed], dim=0)
        edge_index = torch.cat([self.g2i_edges, self.i2u_edges], dim=0).t().contiguous()
        return self.new_gcn(x, edge_index)

    def compute_score(self, user, item, ingre, ingre_num, img, hl, is_training, g2i_edges, i2u_edges, ingre_embedding,
                      gcn_emb=None):
        u_emb = self.user_embed[user]
        i_emb = self.item_embed[item]
        ingre_emb = ingre_embedding[ingre]
        hl_emb = self.health_embed[hl]
        img_emb = self.img_trans(img.to(torch.float32))
        if gcn_emb is None:
            gcn_emb = self._gcn()
        u_g, i_g, ing_g, hl_g = torch.split(gcn_emb, [self.n_users, self.n_items, self.n_ingredients, self.n_health])
        ingre_embedding_gcn = torch.cat([ing_g, self.ingre_embed_second, self.ingre_embed_mask], dim=0)
        u_f = u_emb + u_g[user]
        i_f = i_emb + i_g[item]
        ing_f = ingre_emb + ingre_embedding_gcn[ingre]
        hl_f = hl_emb + hl_g[hl]
        ingre_att = self.attention_ingredient_level(ing_f, u_f, img_emb, ingre_num)
        item_att = self.attention_id_ingre_image(u_f, i_f, ingre_att, img_emb, hl_f)
        hidden = self.W_concat(torch.cat([u_f, item_att, u_f * item_att], dim=1))
        score = self.output_mlp(F.relu(F.dropout(hidden, p=0.5, training=is_training))).squeeze()
        return score, u_emb, i_emb, ingre_emb, hl_emb, ingre_embedding_gcn, item_att

    def calculate_loss(self, batch_data):
        user = batch_data["u_id"]
        pos_item, pos_ingre, pos_num, pos_img = (batch_data["pos_i_id"], batch_data["pos_ingre_code"],
                                                 batch_data["pos_ingre_num"], batch_data["pos_img"])
        neg_item, neg_ingre, neg_num, neg_img = (batch_data["neg_i_id"], batch_data["neg_ingre_code"],
                                                 batch_data["neg_ingre_num"], batch_data["neg_img"])
        pos_hl, neg_hl = batch_data["pos_cl"].long(), batch_data["neg_cl"].long()
        ingre_embedding = torch.cat([self.ingre_embed_first, self.ingre_embed_second, self.ingre_embed_mask], dim=0)
        gcn = self._gcn()  # shared by the positive and the negative pass
        pos_s, u_e, pi_e, p_ing, p_hl, ing_g, _ = self.compute_score(user, pos_item, pos_ingre, pos_num, pos_img, pos_hl,
                                                                     True, None, None, ingre_embedding, gcn)
        neg_s, u_e, ni_e, n_ing, n_hl, _, _ = self.compute_score(user, neg_item, neg_ingre, neg_num, neg_img, neg_hl,
                                                                 True, None, None, ingre_embedding, gcn)
        ssl_loss = self.ssl * self.compute_ssl_loss(ingre_embedding, ing_g, batch_data["masked_ingre_seq"],
                                                    batch_data["pos_ingre_seq"], batch_data["neg_ingre_seq"])
        bpr_loss = -torch.sum(torch.log(torch.sigmoid(pos_s - neg_s)))
        reg_loss = self.regs * (l2_loss(u_e) + l2_loss(pi_e) + l2_loss(ni_e) + l2_loss(p_ing) + l2_loss(n_ing))
        reg_loss += self.reg_health * (l2_loss(p_hl) + l2_loss(n_hl))
        reg_loss += self.reg_image * l2_loss(self.img_trans.weight)
        reg_loss += self.reg_w * (l2_loss(self.W_concat.weight) + l2_loss(self.output_mlp.weight))
        reg_loss += self.reg_g * l2_loss(self.new_gcn.conv1.lin.weight)
        return bpr_loss, reg_loss, ssl_loss

    # ----------------------------------------------------------------------------- inference
    def _item_inputs(self, item):
        """ingredient codes / counts, image rows and calorie levels of ``item`` (the reference reads
        dataset.ingredientCodeDict / ingredientNum / embImage / cal_level)."""
        f = self.__dict__.get("_fr_item_tables")
        if f is None or f[0].device != item.device:
            ds = self.dataset
            cal = np.zeros(self.n_items, np.int64)
            for i, lv in ds.cal_level.items():
                if 0 <= int(i) < self.n_items:
                    cal[int(i)] = int(lv)
            f = (torch.as_tensor(np.asarray(ds.ingredientCodeDict, np.int64)[:self.n_items], device=item.device),
                 torch.as_tensor(np.asarray(ds.ingredientNum, np.int64)[:self.n_items], device=item.device),
                 torch.as_tensor(np.asarray(ds.embImage)[:self.n_items], dtype=torch.float32, device=item.device),
                 torch.as_tensor(cal, device=item.device))
            self.__dict__["_fr_item_tables"] = f
        return f[0][item], f[1][item], f[2][item], f[3][item]

    def _eval_embedding(self):
        return torch.cat([self.ingre_embed_first, self.ingre_embed_second], dim=0)

    def full_sort_predict(self, batch_data):
        item = torch.arange(self.n_items, device=self.user_embed.device)
        user = batch_data["u_id"].repeat(self.n_items)
        ingre, num, img, hl = self._item_inputs(item)
        return self.compute_score(user, item, ingre, num, img, hl, False, None, None, self._eval_embedding())[0]

    def sample_sort_predict(self, batch_data):
        user = batch_data["u_id"]
        items = torch.cat([batch_data["neg_i_id"], batch_data["pos_i_id"].unsqueeze(1)], dim=1).view(-1)
        nb = items.shape[0]
        ingres = torch.cat([batch_data["neg_ingre_code"], batch_data["pos_ingre_code"].unsqueeze(1)], dim=1).view(nb, -1)
        nums = torch.cat([batch_data["neg_ingre_num"], batch_data["pos_ingre_num"].unsqueeze(1)], dim=1).view(-1)
        img = torch.cat([batch_data["neg_img"], batch_data["pos_img"].unsqueeze(1)], dim=1).view(nb, -1)
        hl = torch.cat([batch_data["neg_cl"].long(), batch_data["pos_cl"].long().unsqueeze(1)], dim=1).view(-1)
        n, m = user.size(0), self.config["neg_sample_num"] + 1
        users = user.view(n, 1).expand(n, m).contiguous().view(-1)
        return self.compute_score(users, items, ingres, nums, img, hl, False, None, None,
                                  self._eval_embedding())[0].view(n, m)

    def inference_by_user(self, batch_data):
        item = batch_data["item_input"]
        if "img_input" in batch_data:
            ingre, num, img, hl = (batch_data["ingre_input"], batch_data["ingre_num_input"], batch_data["img_input"],
                                   batch_data["cal_level_input"])
        else:
            ingre, num, img, hl = self._item_inputs(item)
        return self.compute_score(batch_data["user_input"], item, ingre, num, img, hl, False, None, None,
                                  self._eval_embedding())[0]
