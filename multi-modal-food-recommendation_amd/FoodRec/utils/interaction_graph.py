"""BASELINE config 4 data: a synthetic user-item interaction graph built directly in HBM.

U users with Poisson(mean_deg - 1) + 1 interactions each, items drawn from a Zipf-like popularity
((rank + 10)^-0.8 over a random item ranking), duplicate pairs removed -- SURVEY 8(d) config 4
(10M users x 1M items x ~200M interactions).  The graph is kept only as the symmetric normalised
adjacency the model propagates over (``Adjacency``, CSR): its user rows [0, U) hold exactly the E
interactions (columns U + item, sorted), so

* positives: one device permutation of the E interactions per epoch (the reference's shuffled
  DataLoader over the positive list, dataloader.py:12-48 / trainer.py:401-402); the user of
  interaction e is the CSR row containing e;
* negatives: ``fr_sample_negatives_csr`` draws uniform item ids and rejects the user's training
  items by bisection in that same CSR row (get_random_neg, dataloader.py:145-151).

The reference's host pipeline (dok matrices, per-sample Python) cannot hold 200M interactions; the
semantics of a training triple are the same.
"""
from __future__ import annotations

import torch

from FoodRec.engine import native
from FoodRec.engine.graph import DEFAULT_CHUNK, Adjacency, bipartite_norm_csr_torch


def synth_bipartite(n_users, n_items, mean_deg=20.0, seed=0, device="cuda"):
    """(user, item) pairs of the config-4 generator (duplicates removed later by the CSR build)."""
    g = torch.Generator(device=device).manual_seed(seed)
    deg = torch.poisson(torch.full((n_users,), mean_deg - 1.0, device=device), generator=g).to(torch.int64) + 1
    u = torch.repeat_interleave(torch.arange(n_users, device=device), deg)
    p = (torch.randperm(n_items, device=device, generator=g).to(torch.float64) + 10.0) ** -0.8
    cdf = torch.cumsum(p / p.sum(), 0)
    r = torch.rand(u.numel(), device=device, generator=g, dtype=torch.float64)
    i = torch.searchsorted(cdf, r).clamp_(max=n_items - 1)
    return u, i


def uniform_bipartite(n_users, n_items, mean_deg=20.0, seed=0, device="cuda"):
    """(user, item) pairs with config 4's user degrees but uniformly popular items: no item row is
    hot, so a gather over an item table far beyond the Infinity Cache misses it (a DRAM-level SpMM
    measurement; duplicates removed later by the CSR build)."""
    g = torch.Generator(device=device).manual_seed(seed)
    deg = torch.poisson(torch.full((n_users,), mean_deg - 1.0, device=device), generator=g).to(torch.int64) + 1
    u = torch.repeat_interleave(torch.arange(n_users, device=device), deg)
    i = torch.randint(0, n_items, (u.numel(),), device=device, generator=g)
    return u, i


class InteractionGraph:
    """Dataset object for LightGCN_ID: n_users / n_items (what GeneralRecommender reads), the
    normalised adjacency ``adj`` and a device triple sampler."""

    def __init__(self, n_users=10_000_000, n_items=1_000_000, mean_deg=20.0, seed=0, device="cuda",
                 chunk=DEFAULT_CHUNK, pairs=None):
        dev = torch.device(device)
        native.require_device(torch.empty(0, device=dev))
        if pairs is None:
            u, i = synth_bipartite(n_users, n_items, mean_deg, seed, dev)
        else:
            u, i = (torch.as_tensor(x, dtype=torch.int64, device=dev) for x in pairs)
        rp, col, val = bipartite_norm_csr_torch(n_users, n_items, u, i)
        del u, i
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.n_edges = int(rp[n_users].item())
        self.adj = Adjacency(rp, col, val, (n_users + n_items, n_users + n_items), device=dev, chunk=chunk,
                             symmetric=True)
        self.adj.mark_bipartite(n_users)  # users connect to items only and items to users only
        self.device = dev
        self.seed = int(seed)
        self._perm = None
        self._pos = 0
        self._epoch = 0
        self._draws = 0

    # ------------------------------------------------------------------ triple sampler
    def _new_epoch(self):
        g = torch.Generator(device=self.device).manual_seed(self.seed * 1_000_003 + self._epoch)
        self._perm = torch.randperm(self.n_edges, device=self.device, generator=g)
        self._pos = 0
        self._epoch += 1

    def triples(self, batch_size: int):
        """Next (user, pos_item, neg_item) batch, int64 on the device (the epoch's ragged tail is
        skipped, like a drop_last loader; a new permutation starts)."""
        B = int(batch_size)
        if self._perm is None or self._pos + B > self.n_edges:
            self._new_epoch()
        e = self._perm[self._pos:self._pos + B]
        self._pos += B
        rp, col = self.adj.rowptr, self.adj.col
        u = torch.searchsorted(rp[:self.n_users + 1], e, right=True) - 1
        p = col[e].to(torch.int64) - self.n_users
        n = self.negatives(u)
        return u, p, n

    def negatives(self, users: torch.Tensor, max_tries: int = 64) -> torch.Tensor:
        users = users.to(torch.int64).contiguous()
        out = torch.empty_like(users)
        seed = (self.seed * 0x9E3779B1 + self._draws) & ((1 << 64) - 1)
        self._draws += 1
        native.check(native.lib().fr_sample_negatives_csr(
            self.adj.rowptr.data_ptr(), self.adj.col.data_ptr(), self.n_users, users.data_ptr(), users.numel(),
            self.n_items, self.n_users, seed, max_tries, out.data_ptr(), native.stream_of(users)),
            "fr_sample_negatives_csr")
        return out
