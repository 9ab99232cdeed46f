"""LightGCN with ID embeddings on a synthetic interaction graph -- BASELINE config 4 (SURVEY 8(a)
a15 template: models/lightgcn.py with the ego item rows = item_embedding).

One training step: ego = [user_emb; item_emb] (one [U+I, d] table), L-layer propagation with the
layer mean (``ops.propagate_mean``: one HIP SpMM per layer, mean in the epilogue), BPRLoss on the
propagated rows + reg_weight * EmbLoss on the ego rows of the batch (``ops.bpr_emb_loss``, fused;
item ids offset by U into the same table so users and items share one gradient buffer), backward
(L SpMMs), fused Adam.  Users and items live in one parameter so no [U+I, d] concatenation is
materialised per step; ``user_embedding`` / ``item_embedding`` are views of it, and the state_dict
carries them under the reference LightGCN's keys.

``embedding_dtype: bf16`` (BASELINE config 5, d=256): the ego table and every propagated table are
bf16 in HBM (half the gather bytes of the HBM-bound SpMM); SpMM / BPR arithmetic is fp32 in the
kernels and Adam runs on an fp32 master copy with fp32 moments (``FusedAdam``).
``full_sort_topk`` ranks all items for a batch of users on the matrix cores (MFMA) with the
training items masked and the top-k selection fused into the GEMM.
"""
import torch
from torch import nn

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.engine import ops


class _TableView:
    """``.weight`` view of a row block of the ego table (the reference's nn.Embedding attribute)."""

    def __init__(self, owner, lo, hi):
        self._owner, self._lo, self._hi = owner, lo, hi

    @property
    def weight(self):
        return self._owner.ego[self._lo:self._hi]


class LightGCN_ID(GeneralRecommender):
    # the row-list propagation (ops.propagate_rows) sizes its launches from host reads: Trainer steps
    # this model eagerly (inside an explicit capture the full propagation runs instead)
    graph_capturable = False

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.latent_dim = config["embedding_size"]
        self.n_layers = config["n_layers"]
        self.reg_weight = config["reg_weight"]
        U, I, d = self.n_users, self.n_items, self.latent_dim
        dev = torch.device(config["device"]) if config["device"] is not None else dataset.adj.rowptr.device
        # BASELINE config 5: bf16 tables (the optimiser keeps an fp32 master copy and fp32 moments)
        self.table_dtype = torch.bfloat16 if str(config["embedding_dtype"] or "fp32") == "bf16" else torch.float32
        ego = torch.empty(U + I, d, device=dev)
        with torch.no_grad():  # xavier_uniform_ of each nn.Embedding weight (common/init.py)
            nn.init.xavier_uniform_(ego[:U])
            nn.init.xavier_uniform_(ego[U:])
        self.ego = nn.Parameter(ego.to(self.table_dtype))
        del ego
        self.norm_adj_matrix = dataset.adj
        self.user_embedding = _TableView(self, 0, U)
        self.item_embedding = _TableView(self, U, U + I)

    def state_dict(self, *args, **kwargs):
        sd = super().state_dict(*args, **kwargs)
        ego = sd.pop("ego")
        sd["user_embedding.weight"] = ego[:self.n_users]
        sd["item_embedding.weight"] = ego[self.n_users:]
        return sd

    def load_state_dict(self, state_dict, strict=True, assign=False):
        sd = dict(state_dict)
        if "user_embedding.weight" in sd:
            sd["ego"] = torch.cat([sd.pop("user_embedding.weight"), sd.pop("item_embedding.weight")])
        return super().load_state_dict(sd, strict=strict, assign=assign)

    def forward(self):
        out = ops.propagate_mean(self.norm_adj_matrix, self.ego, self.n_layers)
        return out[:self.n_users], out[self.n_users:]

    def calculate_loss(self, batch_data):
        U = self.n_users
        u, p, n = batch_data["u_id"], batch_data["pos_i_id"], batch_data["neg_i_id"]
        # the loss reads the propagated table at the batch's users and items only: the last layer is
        # evaluated there and the backward starts from those rows (ops.propagate_rows)
        out = ops.propagate_rows(self.norm_adj_matrix, self.ego, self.n_layers, [(u, 0), (p, U), (n, U)])
        mf, emb = ops.bpr_emb_loss(out, out, self.ego, self.ego, u, p + U, n + U)
        return mf, self.reg_weight * emb

    def full_sort_predict(self, batch_data):
        """Dense scores of the batch users against every item (common/abstract_recommender.py:39-50)."""
        user_all, item_all = self.forward()
        return torch.matmul(user_all[batch_data["u_id"]].float(), item_all.float().t())

    def full_sort_topk(self, users, k, exclude_train=True, held_out=None, tables=None):
        """Fused full-sort top-k on the matrix cores (engine.ops.full_sort_topk): scores of ``users``
        against all items with the user's training items masked (``exclude_train``), top ``k``.
        ``tables``: precomputed (user_all, item_all) to score several user batches per propagation."""
        user_all, item_all = tables if tables is not None else self.forward()
        users = users.to(device=user_all.device, dtype=torch.int64)
        ex = None
        if exclude_train:
            adj = self.norm_adj_matrix
            ex = (adj.rowptr, adj.col, self.n_users)  # user rows of the adjacency hold U + item
        return ops.full_sort_topk(user_all[users], item_all, k, user_ids=users, exclude=ex, held_out=held_out)

    # inference_fast below is the plain gather-dot of forward()'s tables: the trainer may score the
    # evaluation lists with fr_score_segments instead (no [n, 64] gathers)
    fused_scores = True

    def inference_fast(self, batch_data, user_emb, item_emb):
        return torch.mul(user_emb[batch_data["user_input"]], item_emb[batch_data["item_input"]]).sum(dim=1)

    def inference_by_user(self, batch_data):
        user_all, item_all = self.forward()
        return self.inference_fast(batch_data, user_all, item_all)
