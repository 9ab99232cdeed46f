"""Normalised adjacencies the models propagate over, built straight into HBM-resident CSR.

Same graphs as the reference's per-model dok/scipy builders (value-for-value, see
FoodRec.engine.graph), without the O(nnz) Python dicts:
  ui_adjacency    get_norm_adj_mat            (lightgcn.py:76-120, cikm_model.py:136-180)
  side_adjacency  load_graph + get_norm_adj_recipe_ing/_infor (cikm_model.py:91-134,
                  pricai_modelx.py:88-131): node ids [0, n_items) items, n_items + side id
"""
import numpy as np

from FoodRec.engine.graph import Adjacency, DEFAULT_CHUNK


def ui_adjacency(dataset, n_users, n_items, device, chunk=DEFAULT_CHUNK) -> Adjacency:
    coo = dataset.train_coo_matrix
    rows = np.asarray(coo.row, np.int64)
    cols = np.asarray(coo.col, np.int64) + n_users
    adj = Adjacency.sym_normalized(n_users + n_items, rows, cols, device=device, chunk=chunk)
    # users connect only to items and items only to users
    adj.mark_bipartite(n_users)
    return adj


def side_adjacency(triples, n_items, n_side, device, chunk=DEFAULT_CHUNK) -> Adjacency:
    t = np.asarray(triples)
    rows = t[:, 1].astype(np.int64) + n_items
    cols = t[:, 0].astype(np.int64)
    adj = Adjacency.sym_normalized(n_items + n_side, rows, cols, device=device, chunk=chunk)
    # items connect only to side nodes and side nodes only to items
    adj.mark_bipartite(n_items)
    return adj
