"""SCHGN drop-in on the CPU.

* the engine's torch_geometric.nn.GCNConv provider against a float64 per-edge restatement of PyG's
  documented GCNConv (oracle.ops.gcn_conv_f64; PyG is not installed here, so GCNConv parity with
  PyG itself is unpinned), its parameters and its seeded RNG consumption;
* the masked-ingredient SSL batches against the reference's own TrainDataLoader.ssl_task and
  get_neg_ingre (loaded from /root/reference by file, Python's random seeded alike);
* the reference's models/schgn.py imported UNCHANGED (its FoodRec imports bind to this package,
  torch_geometric to the provider) against the engine-native FoodRec.models.schgn: identical
  state_dict under the seed, identical losses, gradients and evaluation scores.
Engine ops run through oracle.cpu_backend (the CPU restatement of the HIP ops).
"""
import importlib.util
import os
import random

import numpy as np
import pytest
import torch

from oracle import cpu_backend
from oracle import ops as O

REF = "/root/reference/FoodRec"


def _load(alias, path):
    spec = importlib.util.spec_from_file_location(alias, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_torch_geometric_resolves_to_engine_provider():
    import FoodRec  # noqa: F401  (installs the provider when PyG is absent)
    import torch_geometric
    from FoodRec.engine import geometric
    if not getattr(torch_geometric, "__fr_engine__", False):
        pytest.skip("a real torch_geometric is installed")
    assert torch_geometric.nn.GCNConv is geometric.GCNConv
    conv = torch_geometric.nn.GCNConv(8, 5)
    assert sorted(conv.state_dict()) == ["bias", "lin.weight"]
    assert tuple(conv.lin.weight.shape) == (5, 8) and not isinstance(conv.lin, torch.nn.Linear)
    # glorot drawn twice (Linear's reset, then GCNConv.reset_parameters), bias zero
    torch.manual_seed(3)
    c2 = geometric.GCNConv(8, 5)
    after = torch.rand(1)
    torch.manual_seed(3)
    a = (6.0 / 13) ** 0.5
    torch.empty(5, 8).uniform_(-a, a)
    w = torch.empty(5, 8).uniform_(-a, a)
    assert torch.equal(c2.lin.weight.detach(), w) and torch.equal(torch.rand(1), after)
    assert torch.count_nonzero(c2.bias) == 0


@pytest.mark.parametrize("improved", [False, True])
def test_gcn_conv_matches_per_edge_restatement(improved):
    from FoodRec.engine.geometric import GCNConv
    g = torch.Generator().manual_seed(7)
    N, E = 40, 150
    src = torch.randint(0, N, (E,), generator=g)
    dst = torch.randint(0, N, (E,), generator=g)
    src[:3] = dst[:3]                 # existing self-loops keep their own weight
    src[3:6], dst[3:6] = src[6:9], dst[6:9]  # duplicate edges are separate messages
    ei = torch.stack([src, dst])
    ew = torch.rand(E, generator=g) + 0.5
    x = torch.randn(N, 12, generator=g)
    torch.manual_seed(0)
    conv = GCNConv(12, 6, improved=improved)
    with torch.no_grad():
        conv.bias.copy_(torch.randn(6, generator=g))
    with cpu_backend.installed():
        for weights in (None, ew):
            out = conv(x, ei, weights)
            ref = O.gcn_conv_f64(x.numpy(), ei.numpy(), conv.lin.weight.detach().numpy(), conv.bias.detach().numpy(),
                                 None if weights is None else weights.numpy(), improved)
            np.testing.assert_allclose(out.detach().numpy(), ref, rtol=1e-5, atol=1e-5)
        # the cached normalised graph is reused only for an identical edge_index
        out2 = conv(x, ei.flip(0))
        ref2 = O.gcn_conv_f64(x.numpy(), ei.flip(0).numpy(), conv.lin.weight.detach().numpy(),
                              conv.bias.detach().numpy(), None, improved)
        np.testing.assert_allclose(out2.detach().numpy(), ref2, rtol=1e-5, atol=1e-5)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_ssl_sequences_replay_reference_stream():
    from FoodRec.engine.sampler import ssl_sequences
    ref_utils = _load("_ref_utils", os.path.join(REF, "utils", "utils.py"))
    ref_dl = _load("_ref_dataloader", os.path.join(REF, "utils", "dataloader.py"))
    ref_dl.get_neg_ingre = ref_utils.get_neg_ingre
    rng = np.random.default_rng(0)
    NI, B, L = 37, 64, 20
    nums = rng.integers(1, L + 1, B)
    codes = np.full((B, L), NI, np.int64)
    for b in range(B):
        codes[b, :nums[b]] = rng.choice(NI, nums[b], replace=False)

    class _Self:
        n_ingredients, masked_p, max_len = NI, 0.2, L

    random.seed(11)
    want = [ref_dl.TrainDataLoader.ssl_task(_Self(), codes[b], int(nums[b])) for b in range(B)]
    after_ref = random.random()
    random.seed(11)
    got = ssl_sequences(codes, nums, NI)
    assert random.random() == after_ref  # the same number of draws
    for k in range(3):
        assert np.array_equal(got[k], np.stack([w[k].numpy() for w in want]))
    assert (got[0] == NI + 1).any()


def _schgn_data():
    from helpers import tiny_config, tiny_data
    cfg = tiny_config("SCHGN", False)
    return cfg, tiny_data(cfg)


def _batch(data, n=48, seed=5):
    from FoodRec.engine.sampler import BatchFeatures
    feats = BatchFeatures(data, "cpu", ssl=True)
    pairs = data.train_pairs[:n]
    g = torch.Generator().manual_seed(seed)
    neg = torch.randint(0, data.n_items, (n,), generator=g)
    random.seed(seed)
    b = feats.batch(torch.from_numpy(pairs[:, 0].copy()), torch.from_numpy(pairs[:, 1].copy()), neg)
    keys = ("u_id", "pos_i_id", "neg_i_id", "pos_ingre_code", "neg_ingre_code", "pos_ingre_num", "neg_ingre_num",
            "pos_img", "neg_img", "pos_cl", "neg_cl", "masked_ingre_seq", "pos_ingre_seq", "neg_ingre_seq")
    return {k: b[k] for k in keys}, feats


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_schgn_drops_in_and_matches_engine_model():
    from FoodRec.engine.sampler import EvalBatch
    from FoodRec.models.schgn import SCHGN
    from FoodRec.utils.utils import init_seed
    cfg, data = _schgn_data()
    ref_mod = _load("_ref_schgn", os.path.join(REF, "models", "schgn.py"))  # unchanged reference file
    init_seed(999)
    ref = ref_mod.SCHGN(cfg, data)
    init_seed(999)
    nat = SCHGN(cfg, data)
    rs, ns = ref.state_dict(), nat.state_dict()
    assert list(rs) == list(ns)
    for k in rs:
        assert torch.equal(rs[k], ns[k]), k
    batch, feats = _batch(data)
    with cpu_backend.installed():
        torch.manual_seed(1)
        lr = ref.calculate_loss(batch)
        sum(lr).backward()
        torch.manual_seed(1)
        ln = nat.calculate_loss(batch)
        sum(ln).backward()
        for a, b in zip(lr, ln):
            torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-7)
        rp, np_ = dict(ref.named_parameters()), dict(nat.named_parameters())
        for k, p in rp.items():
            if p.grad is None:
                assert np_[k].grad is None, k
                continue
            scale = p.grad.abs().max().item()
            err = (np_[k].grad - p.grad).abs().max().item()
            assert err <= 1e-5 * scale + 1e-9, f"{k}: {err} vs {scale}"
        ref.eval()
        nat.eval()
        with torch.no_grad():
            users = torch.arange(data.n_users).repeat_interleave(3)[:120]
            items = torch.randint(0, data.n_items, (120,), generator=torch.Generator().manual_seed(2))
            sr = ref.inference_by_user(EvalBatch(feats, users, items))
            sn = nat.inference_by_user(EvalBatch(feats, users, items))
            torch.testing.assert_close(sn, sr, rtol=1e-6, atol=1e-6)


def test_engine_schgn_trains_on_cpu_backend():
    """get_model('SCHGN') resolves the engine-native model; two optimiser steps on the CPU
    restatement lower the loss on a fixed batch."""
    from FoodRec.utils.utils import get_model, init_seed
    cfg, data = _schgn_data()
    init_seed(999)
    model = get_model("SCHGN")(cfg, data)
    batch, _ = _batch(data)
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    losses = []
    with cpu_backend.installed():
        model.train()
        for _ in range(3):
            torch.manual_seed(1)
            loss = sum(model.calculate_loss(batch))
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]
