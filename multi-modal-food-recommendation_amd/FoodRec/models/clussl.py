"""CLUSSL (PRICAI'24) on the MI355X engine — the reference's ``PRICAI_ModelX``
(models/pricai_modelx.py).

Parameters, construction order and state_dict keys are the reference's.  forward() runs the
three item-side propagations (ingredient, image-cluster, text-cluster graphs; n_ri_layers each)
and the user-item propagation (n_ui_layers) as fused HIP SpMM chains (:179-232).  The SSL term is
the fused multi-view distance-correlation kernel: the three reference calls
dcor(image,text) + dcor(image,ingre) + dcor(ingre,text) (:263) share one set of distance tiles.
``ssl_mode: infonce`` switches to the (in the reference commented-out) InfoNCE form over the same
view pairs, run by the fused InfoNCE kernel (CL_loss, :354-378).
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.init import xavier_uniform_initialization
from FoodRec.common.loss import BPRLoss, EmbLoss
from FoodRec.engine import ops
from FoodRec.models._graphs import side_adjacency, ui_adjacency

# (image, text), (image, ingre), (ingre, text) with views ordered [image, text, ingre]
_DCOR_PAIRS = ((0, 1), (0, 2), (2, 1))


class CLUSSL(GeneralRecommender):
    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.device = config["device"]
        self.config = config
        self.dataset = dataset
        self.n_ingredients = dataset.num_ingredients
        self.n_cal_level = dataset.num_calories_level
        self.n_health_level = len(dataset.health_level_multi_hot[0]) if config["use_health_level_multi_hot"] \
            else dataset.num_health_level
        self.interaction_matrix = dataset.train_coo_matrix
        d = config["embedding_size"]
        self.latent_dim = d
        self.n_ri_layers = config["n_ri_layers"]
        self.n_mm_layers = config["n_mm_layers"]
        self.n_ui_layers = config["n_ui_layers"]
        self.reg_weight = config["reg_weight"]
        self.loss_cl = config["loss_cl"]
        self.knn_k = config["knn_k"]
        self.mm_image_weight = config["mm_image_weight"]
        self.n_cluster = config["n_cluster"]
        self.ssl_mode = (config["ssl_mode"] or "dcor").lower()
        self.user_embedding = nn.Embedding(self.n_users, d)
        self.item_embedding = nn.Embedding(self.n_items, d)
        self.ingre_embedding = nn.Embedding(self.n_ingredients + 1, d, padding_idx=self.n_ingredients)
        self.mf_loss = BPRLoss()
        self.reg_loss = EmbLoss()
        self.norm_adj_matrix = ui_adjacency(dataset, self.n_users, self.n_items, self.device)
        self.image_norm_adj = side_adjacency(dataset.image_cluster_triples, self.n_items, self.n_cluster, self.device)
        self.text_norm_adj = side_adjacency(dataset.text_cluster_triples, self.n_items, self.n_cluster, self.device)
        self.ingre_norm_adj = side_adjacency(dataset.rIngre_triples, self.n_items, self.n_ingredients, self.device)
        self.proj_ingre = nn.Linear(d, d)
        self.proj_text = nn.Linear(d, d)
        self.proj_image = nn.Linear(d, d)
        self.image_prototype_embedding = nn.Embedding(self.n_cluster, d)
        self.text_prototype_embedding = nn.Embedding(self.n_cluster, d)
        self.apply(xavier_uniform_initialization)
        self.v_center, self.t_center = None, None
        if config["use_center_embedding"]:
            import numpy as np
            base = config["interaction_data_path"] + "mm_cluster/"
            self.v_center = torch.tensor(np.load(base + "image_center.npy").astype(np.float32)).to(self.device)
            self.t_center = torch.tensor(np.load(base + "text_center.npy").astype(np.float32)).to(self.device)
            self.image_prototype_embedding = nn.Embedding.from_pretrained(self.v_center, freeze=False)
            self.image_trs = nn.Linear(self.v_center.shape[1], d)
            nn.init.xavier_normal_(self.image_trs.weight)
            self.text_prototype_embedding = nn.Embedding.from_pretrained(self.t_center, freeze=False)
            self.text_trs = nn.Linear(self.t_center.shape[1], d)
            nn.init.xavier_normal_(self.text_trs.weight)

    def _view(self, adj, side_table):
        # split(propagate(cat(item, side)))[0] (pricai_modelx.py:183-226): on the GPU the item rows
        # only, on the bipartite item-side graph (ops.propagate_lo: half-graph last layer and backward).
        # The side table is passed whole: rows past the graph (the ingredient padding row the
        # reference slices off, weight[:-1]) are never read and get a zero gradient, without the
        # slice's zero-filled backward copy
        return ops.propagate_lo(adj, self.item_embedding.weight, side_table, self.n_ri_layers)

    def _views(self, adjs, side_tables):
        # the three views as one node (ops.propagate_lo_views: the item-row gradients summed in the
        # SpMM epilogue); FR_CLUSSL_VIEWS_NODE=0: one node per view
        if os.environ.get("FR_CLUSSL_VIEWS_NODE", "1") == "0":
            return [self._view(a, t) for a, t in zip(adjs, side_tables)]
        return ops.propagate_lo_views(adjs, self.item_embedding.weight, side_tables, self.n_ri_layers)

    def forward(self):
        return self._forward()[:3]

    def _forward(self, ssl_ids=None):
        """forward(); with ``ssl_ids`` also the three views gathered there (image, text, ingre),
        the sum and the gathers as one node (ops.views_sum_gather)."""
        img_side = self.image_trs(self.image_prototype_embedding.weight) if self.v_center is not None \
            else self.image_prototype_embedding.weight
        txt_side = self.text_trs(self.text_prototype_embedding.weight) if self.t_center is not None \
            else self.text_prototype_embedding.weight
        item_ingre, item_image, item_text = self._views(
            (self.ingre_norm_adj, self.image_norm_adj, self.text_norm_adj),
            (self.ingre_embedding.weight, img_side, txt_side))
        gathered = None
        if ssl_ids is not None:
            item_emb, (g_ing, g_img, g_txt) = ops.views_sum_gather([item_ingre, item_image, item_text], ssl_ids)
            gathered = [g_img, g_txt, g_ing]
        else:
            item_emb = item_ingre + item_image + item_text
        if ssl_ids is not None and self.n_ui_layers == 1:
            # the loss evaluates the UI layer at its batch rows only (ops.ui_bpr): item_emb is its input
            return None, item_emb, (item_image, item_text, item_ingre), gathered
        # propagate(cat([user, item_emb])) with the concatenation folded into the SpMM addressing
        ui = ops.propagate_mean_split(self.norm_adj_matrix, self.user_embedding.weight, item_emb, self.n_ui_layers)
        if ssl_ids is not None:  # the loss reads the one table (bpr_emb_loss item_offset): no split backward
            return ui, None, (item_image, item_text, item_ingre), gathered
        user_all, item_all = torch.split(ui, [self.n_users, self.n_items])
        return user_all, item_all, (item_image, item_text, item_ingre), gathered

    def calculate_loss(self, batch_data):
        user, pos_item, neg_item = batch_data["u_id"], batch_data["pos_i_id"], batch_data["neg_i_id"]
        # [pos; neg] as the engine feed laid it out (a graphed step's batch), else concatenated
        all_item = dict.get(batch_data, "pn_i_id") if isinstance(batch_data, dict) else None
        if all_item is None:
            all_item = torch.cat([pos_item, neg_item], dim=0)
        ui, item_emb, _, views = self._forward(all_item)  # views at the batch items: image, text, ingre
        # the loss weights (reg_weight, loss_cl) are applied inside the kernels: no multiply launches
        if ui is None:  # one UI layer: propagation at the batch rows + BPR + EmbLoss as one node
            mf_loss, reg = ops.ui_bpr(self.norm_adj_matrix, self.user_embedding.weight, item_emb,
                                      self.item_embedding.weight, user, pos_item, neg_item, w_emb=self.reg_weight)
        else:
            mf_loss, reg = ops.bpr_emb_loss(ui, None, self.user_embedding.weight, self.item_embedding.weight,
                                            user, pos_item, neg_item, item_offset=self.n_users, w_emb=self.reg_weight)
        if self.ssl_mode == "infonce":
            # sum over the pairs of CL_loss(cat([views[a], views[b]])): one fused node for all pairs
            cl = ops.infonce_pairs(views, _DCOR_PAIRS, 0.5, weight=self.loss_cl)
        else:
            cl = ops.dcor_loss(views, _DCOR_PAIRS, weight=self.loss_cl)
        return mf_loss, cl, reg

    # inference_fast below is the plain gather-dot of forward()'s tables: the trainer may score the
    # evaluation lists with fr_score_segments instead (no [n, 64] gathers)
    fused_scores = True

    def inference_fast(self, batch_data, user_emb, item_emb):
        return torch.mul(user_emb[batch_data["user_input"]], item_emb[batch_data["item_input"]]).sum(dim=1)

    def inference_by_user(self, batch_data):
        u, i, _ = self.forward()
        return self.inference_fast(batch_data, u, i)

    def CL_loss(self, hidden, hidden_norm=True, temperature=0.5):
        if not hidden_norm:
            raise NotImplementedError("the fused InfoNCE kernel implements hidden_norm=True")
        return ops.infonce_loss(hidden, temperature)

    def correlation_distance(self, x, y):
        return ops.dcor_loss([x, y], [(0, 1)])


PRICAI_ModelX = CLUSSL
