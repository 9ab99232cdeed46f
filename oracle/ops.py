"""ORACLE (test infrastructure only): CPU restatement of the hot-path arithmetic.

Each function names the reference file:line it restates (paths under /root/reference/FoodRec).
torch-CPU is used for the float ops because the reference itself is PyTorch (its arithmetic
lives in ATen); numpy/scipy for the integer graph construction.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch


# ----------------------------------------------------------------------------- row gathers
def embedding_bwd_f64(idx, G, num_rows: int, padding_idx=None) -> np.ndarray:
    """Weight gradient of a row gather ``W[idx]`` / ``nn.Embedding(idx)`` in float64.

    Restates the autograd of ``ingr_all_embeddings[ingredients]`` (cikm_model.py:230; index
    backward = index_put_ accumulate) and of ``self.ingre_embedding(...)`` with
    ``padding_idx=self.n_ingredients`` (cikm_model.py:67-68, 270-271; embedding backward leaves the
    padding row's gradient zero): dW[r] = sum_{i : idx[i] == r, r != padding_idx} G[i].
    """
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    G = np.asarray(G, dtype=np.float64)
    G = G.reshape(idx.shape[0], G.shape[-1])
    keep = idx != (-1 if padding_idx is None else int(padding_idx))
    out = np.zeros((num_rows, G.shape[1]), np.float64)
    np.add.at(out, idx[keep], G[keep])
    return out


# ----------------------------------------------------------------------------- adjacency
def norm_adj_coo(n_nodes: int, rows, cols):
    """D^-1/2 A D^-1/2 of the symmetrised binary graph.

    Restates get_norm_adj_mat (models/lightgcn.py:76-120, cikm_model.py:136-180) and
    get_norm_adj_recipe_ing / _infor (cikm_model.py:112-134, pricai_modelx.py:109-131):
    dok insert of (r,c) and (c,r) with value 1 (duplicates collapse), deg = (A>0).sum(1) + 1e-7,
    diag = deg^-0.5 (float64), L = D*A*D, coo order, values cast to float32.
    Returns (row int64, col int64, val float32) in row-major sorted order.
    """
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    A = sp.coo_matrix((np.ones(2 * len(rows), np.float32),
                       (np.concatenate([rows, cols]), np.concatenate([cols, rows]))),
                      shape=(n_nodes, n_nodes)).tocsr()
    A.data[:] = 1.0  # binary: the dok dict keeps one entry per (r, c)
    deg = np.asarray((A > 0).sum(axis=1)).ravel() + 1e-7
    D = sp.diags(np.power(deg, -0.5))
    L = sp.coo_matrix(D * A * D)
    order = np.lexsort((L.col, L.row))
    return L.row[order].astype(np.int64), L.col[order].astype(np.int64), L.data[order].astype(np.float32)


def coo_to_torch(n_nodes, row, col, val) -> torch.Tensor:
    i = torch.from_numpy(np.stack([row, col]))
    return torch.sparse_coo_tensor(i, torch.from_numpy(val), (n_nodes, n_nodes)).coalesce()


# ----------------------------------------------------------------------------- propagation
def propagate_mean(adj: torch.Tensor, ego: torch.Tensor, n_layers: int) -> torch.Tensor:
    """LightGCN layer stack + mean (models/lightgcn.py:134-144, cikm_model.py:182-208)."""
    out = [ego]
    x = ego
    for _ in range(n_layers):
        x = torch.sparse.mm(adj, x)
        out.append(x)
    return torch.stack(out, dim=1).mean(dim=1)


def spmm_f64(row, col, val, n_rows, X: np.ndarray) -> np.ndarray:
    A = sp.csr_matrix((val.astype(np.float64), (row, col)), shape=(n_rows, X.shape[0]))
    return A @ X.astype(np.float64)


# ----------------------------------------------------------------------------- losses
def bpr_loss(pos_score: torch.Tensor, neg_score: torch.Tensor, gamma: float = 1e-10) -> torch.Tensor:
    """common/loss.py:29-34."""
    return -torch.log(gamma + torch.sigmoid(pos_score - neg_score)).mean()


def emb_loss(*embeddings: torch.Tensor) -> torch.Tensor:
    """common/loss.py:45-50: sum of Frobenius norms / rows of the LAST argument, shape [1]."""
    total = torch.zeros(1, dtype=embeddings[-1].dtype)
    for e in embeddings:
        total = total + torch.norm(e, p=2)
    return total / embeddings[-1].shape[0]


def correlation_distance(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """models/pricai_modelx.py:409-437 (distance correlation of two [n,d] views), shape [1]."""
    zero = torch.zeros(1, dtype=x.dtype)

    def centred(X):
        r = (X * X).sum(1, keepdim=True)
        q = r - 2 * X @ X.t() + r.t()
        D = torch.sqrt(torch.maximum(q, zero) + 1e-8)
        return D - D.mean(0, keepdim=True) - D.mean(1, keepdim=True) + D.mean()

    def dcov(D1, D2):
        n = D1.shape[0]
        s = (D1 * D2).sum() / (torch.ones(1, dtype=x.dtype) * n * n)
        return torch.sqrt(torch.maximum(s, zero) + 1e-8)

    A, B = centred(x), centred(y)
    c12, c11, c22 = dcov(A, B), dcov(A, A), dcov(B, B)
    return c12 / torch.sqrt(torch.maximum(c11 * c22, zero) + 1e-10)


def cl_loss(hidden: torch.Tensor, temperature: float = 0.5) -> torch.Tensor:
    """models/pricai_modelx.py:354-378 (InfoNCE over two halves, hidden_norm=True)."""
    b = hidden.shape[0] // 2
    h = torch.nn.functional.normalize(hidden, p=2, dim=-1)
    h1, h2 = h[:b], h[b:2 * b]
    labels = torch.arange(b)
    mask = torch.eye(b, dtype=hidden.dtype) * 1e9
    aa = h1 @ h1.t() / temperature - mask
    bb = h2 @ h2.t() / temperature - mask
    ab = h1 @ h2.t() / temperature
    ba = h2 @ h1.t() / temperature
    la = torch.nn.functional.cross_entropy(torch.cat([ab, aa], 1), labels)
    lb = torch.nn.functional.cross_entropy(torch.cat([ba, bb], 1), labels)
    return (la + lb) / b


def bpr_step_reference(U_all, I_all, U_ego, I_ego, user, pos, neg, reg_weight, gamma=1e-10):
    """Gather/dot/BPR + weighted EmbLoss exactly as models/lightgcn.py:158-177 composes them."""
    u, p, n = U_all[user], I_all[pos], I_all[neg]
    mf = bpr_loss((u * p).sum(1), (u * n).sum(1), gamma)
    reg = reg_weight * emb_loss(U_ego[user], I_ego[pos], I_ego[neg])
    return mf, reg


# ----------------------------------------------------------------------------- full-sort top-k
def full_sort_topk(U: np.ndarray, I: np.ndarray, k: int, exclude=None, held_out=None):
    """Full-sort ranking of every item for each user row of U.

    Restates Trainer.evaluate (common/trainer.py:476-503): scores = full_sort_predict (the dense
    user @ item.T of common/abstract_recommender.py:39-50), torch.topk(scores, max(topk)); with
    the MMRec history mask (scores of ``exclude[u]`` items set to -inf before the top-k) when
    ``exclude`` is given; hits = ``i in pos_items`` of TopKEvaluator.evaluate
    (utils/topk_evaluator.py:104-107) against ``held_out[u]``.  Scores in float64 on the given
    values; ties ordered by item id (a stable descending sort: torch.topk leaves tie order
    unspecified).  Returns (scores [n,k] f64, items [n,k] int64, hits [n,k] bool or None).
    """
    S = np.asarray(U, np.float64) @ np.asarray(I, np.float64).T
    n = S.shape[0]
    if exclude is not None:
        for u in range(n):
            ex = np.asarray(list(exclude[u]), np.int64)
            if ex.size:
                S[u, ex] = -np.inf
    order = np.argsort(-S, axis=1, kind="stable")[:, :k]
    scores = np.take_along_axis(S, order, 1)
    hits = None
    if held_out is not None:
        hits = np.array([[i in set(held_out[u]) for i in order[u]] for u in range(n)], dtype=bool)
    return scores, order.astype(np.int64), hits


def bf16_round(x) -> np.ndarray:
    """float32 values rounded to bfloat16 (round to nearest even), returned as float32."""
    return torch.as_tensor(np.asarray(x, np.float32)).to(torch.bfloat16).float().numpy()
