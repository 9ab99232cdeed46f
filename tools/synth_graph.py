"""Synthetic user-item interaction graphs on the device (BASELINE config 4 shape by default):
U users with Poisson(mean_deg) >= 1 interactions each, items drawn from a Zipf-like popularity
(rank + 10)^-0.8, duplicates removed (so E is slightly below U * mean_deg)."""
import torch


def synth_bipartite(n_users=10_000_000, n_items=1_000_000, mean_deg=20.0, seed=0, device="cuda"):
    g = torch.Generator(device=device).manual_seed(seed)
    deg = torch.poisson(torch.full((n_users,), mean_deg - 1.0, device=device), generator=g).to(torch.int64) + 1
    u = torch.repeat_interleave(torch.arange(n_users, device=device), deg)
    p = (torch.randperm(n_items, device=device, generator=g).to(torch.float64) + 10.0) ** -0.8
    cdf = torch.cumsum(p / p.sum(), 0)
    r = torch.rand(u.numel(), device=device, generator=g, dtype=torch.float64)
    i = torch.searchsorted(cdf, r).clamp_(max=n_items - 1)
    return u, i
