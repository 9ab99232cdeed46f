"""ORACLE (test infrastructure only): torch-CPU implementations of the engine ops.

``installed()`` swaps FoodRec.engine.ops' functions for the oracle's CPU restatements (torch
sparse COO SpMM, the reference's loss formulas), so an engine model can run its training step
on the host.  Used ONLY by bench.py's ``cpu_baseline`` leg (timed on the GPU box's host cores)
and by CPU tests; the product never imports this module and never falls back to it.
"""
from __future__ import annotations

import contextlib

import torch

from oracle import ops as O


def _coo(adj):
    t = adj.__dict__.get("_oracle_coo")
    if t is None:
        rows = torch.repeat_interleave(torch.arange(adj.shape[0]), (adj.rowptr[1:] - adj.rowptr[:-1]).cpu())
        t = torch.sparse_coo_tensor(torch.stack([rows, adj.col.cpu().long()]), adj.val.cpu(), adj.shape).coalesce()
        adj.__dict__["_oracle_coo"] = t
    return t


def spmm_launch(adj, X, Y1=None, Y2=None, alpha=1.0, A1=None, beta1=0.0, A2=None, beta2=0.0, stream=None):
    """fr_spmm_csr's epilogue contract on torch sparse: Y1 = adj@X; Y2 = alpha*adj@X + beta1*A1 + beta2*A2."""
    Z = torch.sparse.mm(_coo(adj), X)
    if Y1 is not None:
        Y1.copy_(Z)
    if Y2 is not None:
        r = alpha * Z
        if A1 is not None:
            r = r + beta1 * A1
        if A2 is not None:
            r = r + beta2 * A2
        Y2.copy_(r)


def scatter_rows(ids, G, num_rows, padding_idx=None):
    """fr_embedding_bwd: dense row scatter-add (ids outside [0, num_rows) or == padding_idx skipped)."""
    d = G.shape[-1]
    G = G.reshape(-1, d)
    ids = ids.reshape(-1).to(torch.int64)
    keep = (ids >= 0) & (ids < num_rows)
    if padding_idx is not None:
        keep &= ids != padding_idx
    return torch.zeros(num_rows, d, dtype=G.dtype).index_add_(0, ids[keep], G[keep])


def spmm(adj, X):
    return torch.sparse.mm(_coo(adj), X)


def propagate_mean(adj, ego, n_layers):
    if n_layers == 0:
        return ego
    return O.propagate_mean(_coo(adj), ego, n_layers)


def bpr_emb_loss(U, I, Ue, Ie, user, pos, neg, gamma=1e-10, deterministic=False, item_rows=False,
                 item_offset=None, w_emb=1.0):
    if item_offset is not None:
        I = U[item_offset:]
    u, p, n = U[user], I[pos], I[neg]
    mf = O.bpr_loss((u * p).sum(1), (u * n).sum(1), gamma)
    emb = torch.zeros(1) if Ue is None else O.emb_loss(Ue[user], Ie[pos], Ie[neg])
    if w_emb != 1.0:
        emb = w_emb * emb  # the model's reg_weight * EmbLoss (pricai_modelx.py:267)
    return (mf, emb, torch.cat([p, n])) if item_rows else (mf, emb)


def ui_bpr(ui_adj, user_w, item_hi, item_w, u, p, n, gamma=1e-10, w_emb=1.0):
    # the UI layer (pricai_modelx.py:226-232) and BPR + EmbLoss (:252-267) as the reference computes them
    ui = propagate_mean(ui_adj, torch.cat([user_w, item_hi], dim=0), 1)
    return bpr_emb_loss(ui, None, user_w, item_w, u, p, n, gamma=gamma, item_offset=user_w.shape[0], w_emb=w_emb)


def dcor_loss(views, pairs, weight=1.0):
    s = sum(O.correlation_distance(views[a], views[b]) for a, b in pairs)
    return s if weight == 1.0 else weight * s  # loss_cl * SSL term (pricai_modelx.py:263-267)


def infonce_pairs(views, pairs, tau=0.5, weight=1.0):
    s = sum(O.cl_loss(torch.cat([views[a], views[b]]), tau) for a, b in pairs)
    return s if weight == 1.0 else weight * s


def infonce_loss(H, tau=0.5):
    return O.cl_loss(H, tau)


def embedding(idx, weight, padding_idx=None, exchange=None):
    # ingr_all[ingredients] / nn.Embedding(padding_idx) (cikm_model.py:230, 270-271); the data-
    # parallel row exchange is a GPU-only optimisation of the same mean gradient (the CPU baseline
    # runs one process)
    return torch.nn.functional.embedding(idx, weight, padding_idx=padding_idx)


def embedding_norms(idx, weight, padding_idx, half, defer_norms=False):
    # ingr_all[ingredients] (cikm_model.py:230) and the EmbLoss norms of ingre_embedding(pos / neg)
    # with padding_idx (cikm_model.py:270-279), as the reference computes them
    E = torch.nn.functional.embedding(idx, weight)
    P = torch.nn.functional.embedding(idx, weight, padding_idx=padding_idx)
    return E, torch.stack([torch.norm(P[:half]), torch.norm(P[half:])])


def linear(x, W, b=None):
    return torch.nn.functional.linear(x, W, b)


_PATCH = {"embedding": embedding, "embedding_norms": embedding_norms, "linear": linear, "spmm_launch": spmm_launch, "scatter_rows": scatter_rows, "spmm": spmm, "propagate_mean": propagate_mean, "bpr_emb_loss": bpr_emb_loss,
          "dcor_loss": dcor_loss, "infonce_loss": infonce_loss, "infonce_pairs": infonce_pairs,
          "ui_bpr": ui_bpr}


@contextlib.contextmanager
def installed():
    from FoodRec.engine import ops
    saved = {k: getattr(ops, k) for k in _PATCH}
    for k, v in _PATCH.items():
        setattr(ops, k, v)
    try:
        yield
    finally:
        for k, v in saved.items():
            setattr(ops, k, v)
