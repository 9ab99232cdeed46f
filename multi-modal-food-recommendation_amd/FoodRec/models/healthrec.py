"""HealthRec (CIKM'24) on the MI355X engine — the reference's ``CIKM_Model`` (models/cikm_model.py).

``get_model('CIKM_Model')`` resolves here unless the reference file itself is on the path.
Parameters, construction order (so seeded init is bit-identical) and state_dict keys are the
reference's.  Execution differs where the math allows:

* forward(): RI propagation (n_layers) and UI propagation (ui_layers) run as fused HIP SpMM
  chains with the layer mean in the epilogue (cikm_model.py:182-208);
* BPR + the user/item EmbLoss terms run in the fused gather-dot-BPR kernels (:255-279);
* text_trs / image_trs are applied to the 2B gathered feature rows instead of the full item
  tables (:240-243).  A row-wise Linear commutes with the row gather, so the loss and every
  gradient (including the dense feature-table gradients that Adam then applies to all rows)
  are the same; it removes ~36 GFLOP of discarded projection work per step at Allrecipes shape.
* the ingredient Transformer, target attention, KD and health heads are PyTorch-ROCm ops
  with the reference's exact quirks (F.normalize over dim=1, raw ingre_embedding for the
  encoder, padding mask constant -(2**32)+1, KD threshold via max(0, kd - thr)).
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.functional import cosine_similarity

from FoodRec.common.abstract_recommender import GeneralRecommender
from FoodRec.common.init import xavier_uniform_initialization
from FoodRec.common.loss import BPRLoss, EmbLoss
from FoodRec.engine import layers, ops
from FoodRec.models._graphs import side_adjacency, ui_adjacency

# FR_FUSED_FUSION=0 keeps the unfused (torch + engine ops) target-attention path for A/B comparisons
FUSED_FUSION = os.environ.get("FR_FUSED_FUSION", "1") != "0"
# FR_FUSED_HEAD=0 keeps the torch health-MLP / BCE / cosine loss head
FUSED_HEAD = os.environ.get("FR_FUSED_HEAD", "1") != "0"
# FR_FUSED_PROJECTION=0 keeps gather + ops.linear for the image / text projections
FUSED_PROJECTION = os.environ.get("FR_FUSED_PROJECTION", "1") != "0"
# FR_FUSED_LOSS_HEAD=0 keeps the modal fusion and the health / KD head as two nodes (four kernels)
FUSED_LOSS_HEAD = os.environ.get("FR_FUSED_LOSS_HEAD", "1") != "0"
# FR_PROJECTION_FIRST=1: the modal projections before the encoder (their backward after the encoder's)
PROJECTION_FIRST = os.environ.get("FR_PROJECTION_FIRST", "0") == "1"
# FR_FUSED_GRAPH=0 keeps the concatenated-ego propagation + separate BPR op (full UI propagation)
FUSED_GRAPH = os.environ.get("FR_FUSED_GRAPH", "1") != "0"


class TargetAttention(nn.Module):
    """Head-split scaled dot attention with a shared LayerNorm on Q and K
    (target_attention_layer, cikm_model.py:311-369); parameter names kept for state_dict."""

    def __init__(self, model_dims, hidden, num_head, linear_projection, atten_mode, padding_idx):
        super().__init__()
        self.linear_projection = linear_projection
        self.num_split = int(hidden / num_head)
        self.num_head = num_head
        self.q_fc = nn.Linear(model_dims, hidden)
        self.k_fc = nn.Linear(model_dims, hidden)
        self.v_fc = nn.Linear(model_dims, hidden)
        self.atten_mode = atten_mode
        self.padding_idx = padding_idx
        if atten_mode == "ln":
            self.ln = nn.LayerNorm(self.num_split, eps=1e-12)

    def forward(self, target_query, item_vec, seq_ids=None):
        q, k, v = target_query, item_vec, item_vec
        if self.linear_projection:
            q, k, v = self.q_fc(q), self.k_fc(k), self.v_fc(v)
        h = self.num_head
        # heads stacked along the batch axis: [h*N, L, d/h]
        qh = torch.cat(torch.chunk(q, h, dim=2), dim=0)
        kh = torch.cat(torch.chunk(k, h, dim=2), dim=0)
        vh = torch.cat(torch.chunk(v, h, dim=2), dim=0)
        if self.atten_mode == "ln":
            ln = self.ln
            qh = ops.layer_norm(qh, ln.normalized_shape, ln.weight, ln.bias, ln.eps)
            kh = ops.layer_norm(kh, ln.normalized_shape, ln.weight, ln.bias, ln.eps)
        scores = torch.matmul(qh, kh.transpose(1, 2)) * (kh.shape[-1] ** (-0.5))
        if seq_ids is not None:
            lq, lk = q.shape[1], k.shape[1]
            pad = (seq_ids == self.padding_idx).float().view(-1, 1, lk).repeat(h, lq, 1)
            keep = (seq_ids != self.padding_idx).float().view(-1, 1, lk).repeat(h, lq, 1)
            scores = keep * scores + pad * (-2 ** 32 + 1)
        att = torch.softmax(scores, dim=-1)
        out = torch.matmul(att, vh)
        return torch.cat(torch.chunk(out, h, dim=0), dim=2).squeeze(), att


class HealthRec(GeneralRecommender):
    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.device = config["device"]
        self.config = config
        self.dataset = dataset
        self.n_ingredients = dataset.num_ingredients
        self.n_cal_level = dataset.num_calories_level
        self.n_health_level = len(dataset.health_level_multi_hot[0]) if config["use_health_level_multi_hot"] \
            else dataset.num_health_level
        d = config["embedding_size"]
        # module construction order == the reference's (seeded init parity)
        self.encoder_layer = layers.TransformerEncoderLayer(d_model=d, nhead=config["num_attention_heads"],
                                                        dim_feedforward=4 * d,
                                                        dropout=config["attention_probs_dropout_prob"],
                                                        activation=config["hidden_act"])
        self.ingr_encoder = nn.TransformerEncoder(self.encoder_layer, num_layers=config["num_hidden_layers"],
                                                  enable_nested_tensor=False)
        for k, layer in enumerate(self.ingr_encoder.layers):  # dropout-hash salt of the fused layer
            layer.__dict__["_fr_salt"] = k
        self.mm_target_atten = TargetAttention(d, d, config["num_attention_heads"], False, "ln", self.n_ingredients)
        self.ingre_target_atten = TargetAttention(d, d, config["num_attention_heads"], False, "ln", self.n_ingredients)
        self.health_mlp = nn.Sequential(nn.Linear(d, d), nn.ReLU(), nn.Linear(d, self.n_health_level))
        self.criterion = nn.BCELoss(reduction="none")
        self.interaction_matrix = dataset.train_coo_matrix
        self.latent_dim = d
        self.n_layers = config["n_layers"]
        self.ui_layers = config["ui_layers"]
        self.reg_weight = config["reg_weight"]
        self.loss_kd = config["loss_kd"]
        self.loss_health = config["loss_health"]
        self.kd_threshold = config["kd_threshold"]
        self.user_embedding = nn.Embedding(self.n_users, d)
        self.item_embedding = nn.Embedding(self.n_items, d)
        self.ingre_embedding = nn.Embedding(self.n_ingredients + 1, d, padding_idx=self.n_ingredients)
        self.mf_loss = BPRLoss()
        self.reg_loss = EmbLoss()
        self.norm_adj_matrix = ui_adjacency(dataset, self.n_users, self.n_items, self.device)
        self.ri_norm_adj = side_adjacency(dataset.rIngre_triples, self.n_items, self.n_ingredients, self.device)
        self.apply(xavier_uniform_initialization)
        if self.v_feat is not None:
            self.image_embedding = nn.Embedding.from_pretrained(self.v_feat, freeze=False)
            self.image_trs = nn.Linear(self.v_feat.shape[1], d)
            nn.init.xavier_normal_(self.image_trs.weight)
        if self.t_feat is not None:
            self.text_embedding = nn.Embedding.from_pretrained(self.t_feat, freeze=False)
            self.text_trs = nn.Linear(self.t_feat.shape[1], d)
            nn.init.xavier_normal_(self.text_trs.weight)

    def _propagate(self):
        """[users | items] after both propagations (cikm_model.py:185-205), and the discarded
        propagated ingredients."""
        ir_ego = torch.cat((self.item_embedding.weight, self.ingre_embedding.weight[:-1, :]), dim=0)
        ir_all = ops.propagate_mean(self.ri_norm_adj, ir_ego, self.n_layers)
        item_ir, ingre_ir = torch.split(ir_all, [self.n_items, self.n_ingredients])
        ui_ego = torch.cat([self.user_embedding.weight, item_ir], dim=0)
        return ops.propagate_mean(self.norm_adj_matrix, ui_ego, self.ui_layers), ingre_ir

    def forward(self):
        ui_all, ingre_ir = self._propagate()
        user_all, item_all = torch.split(ui_all, [self.n_users, self.n_items])
        return user_all, item_all, ingre_ir

    def calculate_loss(self, batch_data):
        user, pos_item, neg_item = batch_data["u_id"], batch_data["pos_i_id"], batch_data["neg_i_id"]
        all_item = _pn(batch_data, "i_id")
        xg = self.__dict__.get("_fr_exchange")  # row-gradient exchange (FusedAdam / data parallel)
        # lazily updated image/text rows of this batch: caught up on a side stream (ALU-bound) while
        # the propagation (memory-bound, other tables) runs (data parallel: RowExchange hands it to
        # its sink, the same FusedAdam row state)
        join = xg.prefetch_rows([(t.weight, all_item) for t in self._row_tables()]) \
            if xg is not None and hasattr(xg, "prefetch_rows") and self._fused_projection(all_item) \
            else (lambda stream=None: None)
        fused_graph = self._fused_graph(user)
        if fused_graph:
            # both propagations + BPR + the user/item EmbLoss terms as one node: split-table reads and
            # writes (no cat / split glue), the UI propagation evaluated at the batch rows only.  Started
            # on a branch stream: the encoder / projection / fusion work below overlaps it (and its
            # backward overlaps theirs); joined before the KD head reads its item rows
            branch = ops.graph_bpr_begin(self.user_embedding.weight, self.item_embedding.weight,
                                         self.ingre_embedding.weight, user, pos_item, neg_item, all_item,
                                         self.ri_norm_adj, self.norm_adj_matrix, self.n_layers, self.ui_layers)
        else:
            ui_all, _ = self._propagate()  # one [users | items] table: one gradient buffer in the BPR backward
        # the modal projections read only the (caught-up) image / text rows: on a second branch
        # stream they overlap the encoder forward, and autograd runs their backward there too, beside
        # the encoder backward; joined before the fusion reads mm_query
        proj = self._fused_projection(all_item)
        aux = ops.aux_stream(all_item.device) if proj else None
        if aux is not None:
            main = torch.cuda.current_stream(all_item.device)
            aux.wait_stream(main)
            join(aux)
            all_item.record_stream(aux)
            with torch.cuda.stream(aux):
                mm_query = ops.modal_projection(all_item, [(self.image_embedding.weight, self.image_trs),
                                                           (self.text_embedding.weight, self.text_trs)], exchange=xg)
                projected = torch.cuda.Event()
                projected.record(aux)
        elif proj and PROJECTION_FIRST:
            # projected before the encoder: its autograd node is then older than the encoder's, and the
            # engine runs the younger of two ready nodes first -- the encoder's backward, then the
            # projection backward (dW + the factored table rows, read only by the optimiser)
            join()
            mm_query = ops.modal_projection(all_item, [(self.image_embedding.weight, self.image_trs),
                                                       (self.text_embedding.weight, self.text_trs)], exchange=xg)
        ingr_all = self.ingre_embedding.weight  # the reference discards the propagated ingredients
        health_level = _pn(batch_data, "hl_mh")
        ingredients = _pn(batch_data, "ingre_code")
        ingre_num = _pn(batch_data, "ingre_num")
        B = user.shape[0]
        # ingr_all[ingredients] (grad reaches the pad row too, cikm_model.py:230) and the EmbLoss
        # norms of ingre_embedding(pos / neg ingredients) with padding_idx (:270-279): the same
        # gather, so one gather and one combined deterministic scatter (fr_embedding_bwd)
        # (the norms' finalize is left to the loss's reg_combine launch: they feed nothing before it)
        ingr_emb, ing_norms = ops.embedding_norms(ingredients, ingr_all, self.n_ingredients, B, defer_norms=True)
        mask = batch_data.get("pn_pad_kpm")  # additive key mask gathered with the codes (engine batch), else computed
        if mask is None:
            mask = ingredients == self.n_ingredients
        encoded = layers.run_encoder(self.ingr_encoder, ingr_emb.permute(1, 0, 2), src_key_padding_mask=mask)
        encoded = encoded.permute(1, 0, 2).contiguous()
        if xg is not None and hasattr(xg, "background_rest"):
            xg.background_rest()  # the rest of the lazy-Adam background slice beside the loss head

        # gather-then-project == project-then-gather for a row-wise Linear (module docstring)
        if aux is not None:
            main.wait_event(projected)
            mm_query.record_stream(main)
        elif proj and PROJECTION_FIRST:
            pass
        elif proj:
            join()
            # gathers folded into the projection GEMMs; the tables' gradient stays factored (dY, W)
            mm_query = ops.modal_projection(all_item, [(self.image_embedding.weight, self.image_trs),
                                                       (self.text_embedding.weight, self.text_trs)], exchange=xg)
        else:
            img_q = ops.linear(ops.embedding(all_item, self.image_embedding.weight, exchange=xg),
                               self.image_trs.weight, self.image_trs.bias).unsqueeze(1)
            txt_q = ops.linear(ops.embedding(all_item, self.text_embedding.weight, exchange=xg),
                               self.text_trs.weight, self.text_trs.bias).unsqueeze(1)
            mm_query = torch.cat([img_q, txt_q], dim=1)
        if FUSED_LOSS_HEAD and self._fused_fusion(encoded, mm_query) and self._fused_head(encoded, health_level):
            # the target attentions, normalize heads, health MLP / BCE and KD cosine as ONE node
            # (fr_modal_head_*: 2 launches forward, 2 backward; know / hin never leave the registers)
            if fused_graph:
                mf_loss, emb3, item_rows = ops.graph_bpr_end(branch)
            else:
                mf_loss, emb3, item_rows = ops.bpr_emb_loss(ui_all, None, self.user_embedding.weight,
                                                            self.item_embedding.weight, user, pos_item, neg_item,
                                                            item_rows=True, item_offset=self.n_users)
            health_term, kd_term = ops.modal_head(encoded, mm_query, ingredients, ingre_num, self.n_ingredients,
                                                  item_rows, health_level, self.mm_target_atten.ln,
                                                  self.ingre_target_atten.ln, self.health_mlp, self.kd_threshold,
                                                  self.loss_health, self.loss_kd)
            return self._losses(mf_loss, health_term, kd_term, emb3, ing_norms, B)
        if self._fused_fusion(encoded, mm_query):
            # both target attentions + the normalize heads in one HIP kernel pair (fr_modal_fusion_*)
            item_know, health_in = ops.modal_fusion(encoded, mm_query, ingredients, ingre_num, self.n_ingredients,
                                                    self.mm_target_atten.ln, self.ingre_target_atten.ln)
        else:
            item_health, _ = self.mm_target_atten(mm_query, encoded, ingredients)
            item_mm, _ = self.ingre_target_atten(encoded, mm_query)
            item_know = F.normalize(item_mm).sum(1) / ingre_num.unsqueeze(1)
            health_in = F.normalize(item_health).mean(dim=1)
        # torch.cat([item_all[pos], item_all[neg]]) (cikm_model.py:256-257, 263): the BPR kernel's own
        # item rows; their KD gradient is added inside the BPR backward's scatter
        if fused_graph:
            mf_loss, emb3, item_rows = ops.graph_bpr_end(branch)
        else:
            mf_loss, emb3, item_rows = ops.bpr_emb_loss(ui_all, None, self.user_embedding.weight,
                                                        self.item_embedding.weight, user, pos_item, neg_item,
                                                        item_rows=True, item_offset=self.n_users)
        if self._fused_head(health_in, health_level):
            # health MLP + BCE sum and the KD cosine term, weighted, in one HIP kernel per direction
            health_term, kd_term = ops.health_kd_loss(health_in, item_know, item_rows, health_level, self.health_mlp,
                                                      self.kd_threshold, self.loss_health, self.loss_kd)
        else:
            health_pred = torch.sigmoid(self.health_mlp(health_in))
            health_term = self.loss_health * torch.sum(self.criterion(health_pred, health_level))
            kd = 1 - cosine_similarity(item_know, item_rows, dim=-1).mean()
            kd_term = self.loss_kd * self.norm_loss(kd, self.kd_threshold)

        return self._losses(mf_loss, health_term, kd_term, emb3, ing_norms, B)

    def _losses(self, mf_loss, health_term, kd_term, emb3, ing_norms, B):
        # EmbLoss over 5 blocks, / rows of the last block (= B): fused part carries 3 of them
        if emb3.is_cuda and ing_norms.is_cuda and emb3.dtype == torch.float32 and ing_norms.dtype == torch.float32:
            # the head's and the norms' deferred finalizes, the EmbLoss assembly and (in a trainer step)
            # the step's bookkeeping in one launch (ops.healthrec_loss_finalize)
            return mf_loss, health_term, kd_term, ops.healthrec_loss_finalize(mf_loss, health_term, kd_term, emb3,
                                                                              ing_norms, B, self.reg_weight)
        ops.finalize_norms(ing_norms)
        reg = emb3 + ing_norms.sum() / B  # (= ing_norms[0] + ing_norms[1]; sum's backward is a view, no fills)
        return mf_loss, health_term, kd_term, self.reg_weight * reg

    def _fused_fusion(self, encoded, mm_query) -> bool:
        """The fused modal-fusion kernels cover the reference's configuration: d=64, 2 heads, 'ln'
        attention without projections, 2 modal queries, fp32 on the GPU."""
        a, b = self.mm_target_atten, self.ingre_target_atten
        return (FUSED_FUSION and encoded.is_cuda and encoded.dtype == torch.float32 and encoded.shape[-1] == 64
                and mm_query.shape[1] == 2 and encoded.shape[1] in ops.ENCODER_LENGTHS
                and all(m.num_head == 2 and m.atten_mode == "ln" and not m.linear_projection for m in (a, b))
                and a.ln.eps == b.ln.eps)

    @torch.no_grad()
    def engine_layout(self):
        """Place item_embedding and ingre_embedding in ONE device buffer, [items ; ingredients (+ pad)]
        -- the RI propagation's ego table [item ; ingre[:-1]] (cikm_model.py:185) is then a plain
        contiguous view: the first SpMM of every step gathers from one table instead of two.  Called
        by the Trainer before the optimiser exists (the parameter objects stay the same; state_dict
        and load_state_dict are unaffected)."""
        iw, gw = self.item_embedding.weight, self.ingre_embedding.weight
        if not (iw.is_cuda and gw.is_cuda and iw.dtype == gw.dtype and iw.shape[1] == gw.shape[1]):
            return
        if iw.is_contiguous() and gw.is_contiguous() and gw.data_ptr() == iw.data_ptr() + iw.numel() * iw.element_size():
            return
        big = torch.cat([iw.detach(), gw.detach()], dim=0)
        iw.data = big[:iw.shape[0]]
        gw.data = big[iw.shape[0]:]

    def _fused_graph(self, ids) -> bool:
        """ops.graph_bpr covers the GPU configuration: fp32 d=64 contiguous tables, CSR adjacencies
        (the Trainer's swap), at least one layer of each propagation."""
        from FoodRec.engine.graph import Adjacency
        ws = (self.user_embedding.weight, self.item_embedding.weight, self.ingre_embedding.weight)
        return (FUSED_GRAPH and ids.is_cuda and all(w.is_cuda and w.dtype == torch.float32 and w.shape[1] == 64
                                                     and w.is_contiguous() for w in ws)
                and isinstance(self.norm_adj_matrix, Adjacency) and isinstance(self.ri_norm_adj, Adjacency)
                and self.n_layers >= 1 and self.ui_layers >= 1)

    def _row_tables(self):
        return [getattr(self, n) for n in ("image_embedding", "text_embedding") if hasattr(self, n)]

    def _fused_projection(self, ids) -> bool:
        """Both modal tables present, fp32 on the GPU, Linear(K -> 64) with K a multiple of 16."""
        if not (FUSED_PROJECTION and ids.is_cuda and hasattr(self, "image_embedding") and hasattr(self, "text_embedding")):
            return False
        return all(t.weight.dtype == torch.float32 and t.weight.is_contiguous() and lin.out_features == 64
                   and lin.in_features % 16 == 0 and lin.bias is not None
                   for t, lin in ((self.image_embedding, self.image_trs), (self.text_embedding, self.text_trs)))

    def _fused_head(self, health_in, health_level) -> bool:
        """The fused loss head covers health_mlp = Linear(64, 64), ReLU, Linear(64, H <= 16) with
        BCELoss(reduction='none') summed, fp32 on the GPU."""
        m = self.health_mlp
        return (FUSED_HEAD and health_in.is_cuda and health_in.dtype == torch.float32 and health_in.shape[-1] == 64
                and len(m) == 3 and isinstance(m[0], nn.Linear) and isinstance(m[1], nn.ReLU)
                and isinstance(m[2], nn.Linear) and m[0].in_features == 64 and m[0].out_features == 64
                and m[2].in_features == 64 and 1 <= m[2].out_features <= 16 and m[0].bias is not None
                and m[2].bias is not None and health_level.dim() == 2
                and health_level.shape[1] == m[2].out_features
                and isinstance(self.criterion, nn.BCELoss) and self.criterion.weight is None)

    def row_sparse_tables(self):
        """Parameters whose only use on the training step is a row gather (engine.dist exchanges
        their data-parallel gradient as rows)."""
        return [getattr(self, n).weight for n in ("image_embedding", "text_embedding") if hasattr(self, n)]

    def inference_by_user(self, batch_data):
        user_all, item_all, _ = self.forward()
        return self.inference_fast(batch_data, user_all, item_all)

    # inference_fast below is the plain gather-dot of forward()'s tables: the trainer may score the
    # evaluation lists with fr_score_segments instead (no [n, 64] gathers)
    fused_scores = True

    def inference_fast(self, batch_data, user_emb, item_emb):
        return torch.mul(user_emb[batch_data["user_input"]], item_emb[batch_data["item_input"]]).sum(dim=1)

    def norm_loss(self, kd_loss, threshold):
        # torch.max(tensor(0.), kd - thr) (cikm_model.py:304-308) with a cached device zero, so the
        # step issues no host->device scalar copy (graph-capturable)
        zero = self.__dict__.get("_zero")
        if zero is None or zero.device != kd_loss.device:
            zero = torch.zeros((), dtype=kd_loss.dtype, device=kd_loss.device)
            self.__dict__["_zero"] = zero
        return torch.max(zero, kd_loss - threshold)


def _pn(batch, what):
    """torch.cat([batch['pos_' + what], batch['neg_' + what]]) -- read directly when the engine's
    batch (sampler.LazyBatch) provides it stacked."""
    v = batch.get("pn_" + what)
    return v if v is not None else torch.cat([batch["pos_" + what], batch["neg_" + what]], dim=0)


# the reference's names
CIKM_Model = HealthRec
target_attention_layer = TargetAttention
