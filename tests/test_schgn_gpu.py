"""SCHGN on the GPU: the engine's GCNConv (HIP SpMM over the normalised
target-row CSR) and the engine-native SCHGN against their CPU restatements.

Oracles: oracle.ops.gcn_conv_f64 (PyG's documented GCNConv, per-edge float64) for the layer; the same
model on oracle.cpu_backend (torch-CPU) for the full SCHGN step, dropout disabled on both sides (the
GPU and CPU dropout streams differ).  PyG itself is absent, so parity with PyG is unpinned.

Tolerances: GCNConv forward 1e-5 rel; gradients <= 1e-4 * max|ref| + 1e-7; SCHGN losses 1e-4 rel,
parameter gradients <= 2e-4 * max|ref| + 1e-7 (fp32 SpMM / GEMM order vs torch-CPU).
"""
import random

import numpy as np
import pytest
import torch

from oracle import cpu_backend
from oracle import ops as O

pytestmark = pytest.mark.gpu


def test_gcn_conv_gpu_matches_oracle(cuda):
    from FoodRec.engine.geometric import GCNConv
    g = torch.Generator().manual_seed(4)
    N, E = 3000, 20000
    ei = torch.stack([torch.randint(0, N, (E,), generator=g), torch.randint(0, N, (E,), generator=g)])
    ei[:, :5] = ei[0, :5]  # a few self-loops
    x = torch.randn(N, 64, generator=g)
    torch.manual_seed(0)
    conv = GCNConv(64, 64)
    with torch.no_grad():
        conv.bias.copy_(torch.randn(64, generator=g))
    ref = O.gcn_conv_f64(x.numpy(), ei.numpy(), conv.lin.weight.detach().numpy(), conv.bias.detach().numpy())
    gout = torch.randn(N, 64, generator=g)
    # CPU restatement for the gradients
    cpu = GCNConv(64, 64)
    cpu.load_state_dict(conv.state_dict())
    xc = x.clone().requires_grad_(True)
    with cpu_backend.installed():
        (cpu(xc, ei) * gout).sum().backward()
    gpu = conv.to(cuda)
    xg = x.to(cuda).requires_grad_(True)
    out = gpu(xg, ei.to(cuda))
    (out * gout.to(cuda)).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    for a, b in ((xg.grad, xc.grad), (gpu.lin.weight.grad, cpu.lin.weight.grad), (gpu.bias.grad, cpu.bias.grad)):
        err = (a.cpu() - b).abs().max().item()
        assert err <= 1e-4 * b.abs().max().item() + 1e-7


def _setup(device):
    from helpers import tiny_config, tiny_data
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("SCHGN", device == "cuda")
    cfg["device"] = torch.device(device)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("SCHGN")(cfg, data).to(device)
    return cfg, data, model


def _batch(data, device, n=64, seed=5):
    from FoodRec.engine.sampler import BatchFeatures
    feats = BatchFeatures(data, device, ssl=True)
    pairs = data.train_pairs[:n]
    neg = torch.randint(0, data.n_items, (n,), generator=torch.Generator().manual_seed(seed))
    random.seed(seed)
    b = feats.batch(torch.from_numpy(pairs[:, 0].copy()).to(device), torch.from_numpy(pairs[:, 1].copy()).to(device),
                    neg.to(device))
    keys = ("u_id", "pos_i_id", "neg_i_id", "pos_ingre_code", "neg_ingre_code", "pos_ingre_num", "neg_ingre_num",
            "pos_img", "neg_img", "pos_cl", "neg_cl", "masked_ingre_seq", "pos_ingre_seq", "neg_ingre_seq")
    return {k: b[k] for k in keys}


def test_schgn_step_gpu_matches_cpu_restatement(cuda, monkeypatch):
    monkeypatch.setattr(torch.nn.functional, "dropout", lambda x, p=0.5, training=True, inplace=False: x)
    _, data, m_gpu = _setup("cuda")
    _, _, m_cpu = _setup("cpu")
    for k, v in m_cpu.state_dict().items():
        assert torch.equal(v, m_gpu.state_dict()[k].cpu()), k
    lg = m_gpu.calculate_loss(_batch(data, "cuda"))
    sum(lg).backward()
    with cpu_backend.installed():
        lc = m_cpu.calculate_loss(_batch(data, "cpu"))
        sum(lc).backward()
    for a, b in zip(lg, lc):
        torch.testing.assert_close(a.detach().cpu(), b.detach(), rtol=1e-4, atol=1e-6)
    pg = dict(m_gpu.named_parameters())
    for k, p in m_cpu.named_parameters():
        if p.grad is None:
            continue
        err = (pg[k].grad.cpu() - p.grad).abs().max().item()
        assert err <= 2e-4 * p.grad.abs().max().item() + 1e-7, f"{k}: {err}"


def test_schgn_trainer_epoch_and_eval_gpu(cuda):
    """One epoch through the Trainer (SSL batches, FusedAdam) and the by-user evaluation (chunked
    EvalBatch with the reference's side inputs); metrics finite."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sampler import TripleSampler
    cfg, data, model = _setup("cuda")
    tr = Trainer(cfg, model)
    assert not tr.use_graph  # SSL batches are host-generated: eager steps
    tr.EVAL_CHUNK_ROWS = 4096  # several chunks on the tiny data
    tr._dataset = data
    sampler = TripleSampler(data, cfg["train_batch_size"], cuda)
    loss = tr._train_epoch(sampler, 0)[0]
    assert np.all(np.isfinite(np.asarray(loss, dtype=np.float64)))
    res = tr._valid_by_user_epoch(is_test=True)
    vals = np.asarray(list(res[1].values()) if isinstance(res, tuple) else list(res.values()), dtype=np.float64)
    assert np.all(np.isfinite(vals))
