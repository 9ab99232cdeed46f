"""The operator boundary on the MI355X: a reference-style model (tests/ref_style/propagation_stub.py:
plain torch sparse COO attribute, ``torch.sparse.mm`` + ``stack().mean(1)``) under the Trainer.

Trainer(...) swaps the COO attribute for an ``Adjacency`` (engine/graph.py ``swap_sparse_attributes``),
so ``torch.sparse.mm(self.norm_adj_matrix, x)`` dispatches through ``Adjacency.__torch_function__``
to the HIP SpMM (fr_spmm_csr) with autograd (backward = A^T G = A G, the adjacency is symmetric).
Against the reference's LightGCN golden (same parameters, adjacency and batch): forward tables rel
1e-5, loss components rel 1e-5, gradients <= 2e-4 of the tensor's max, and a fused-Adam step taken
through the trainer moves the parameters.
"""
import numpy as np
import pytest
import torch

from helpers import golden, tiny_config, tiny_data

pytestmark = pytest.mark.gpu


def test_reference_style_sparse_mm_dispatches_to_hip_spmm(cuda):
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import native, profiling
    from FoodRec.engine.graph import Adjacency
    from ref_style.propagation_stub import PropagationStub
    g = golden("model_LightGCN.npz")
    cfg = tiny_config("LightGCN", True, cuda_graph=False)
    data = tiny_data(cfg)
    model = PropagationStub(cfg, data, g).to(cuda)
    assert model.norm_adj_matrix.layout == torch.sparse_coo
    tr = Trainer(cfg, model)
    assert tr.swapped_adjacencies == ["norm_adj_matrix"]
    assert isinstance(model.norm_adj_matrix, Adjacency) and model.norm_adj_matrix.device == cuda
    native.lib()
    with profiling.timing() as timer:
        with torch.no_grad():
            users, items = model.forward()
        torch.cuda.synchronize()
    assert timer.summary().get("spmm", {}).get("launches", 0) >= 1, "torch.sparse.mm did not reach fr_spmm_csr"
    np.testing.assert_allclose(users.cpu().numpy(), g["fwd/user"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(items.cpu().numpy(), g["fwd/item"], rtol=1e-5, atol=1e-6)
    batch = {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}
    tr.optimizer.zero_grad()
    losses = model.calculate_loss(batch)
    np.testing.assert_allclose([float(x) for x in losses], g["loss"], rtol=1e-5)
    sum(losses).backward()
    n = 0
    for k, p in model.named_parameters():
        if "grad/" + k in g.files:
            ref = g["grad/" + k]
            err = np.abs(p.grad.cpu().numpy() - ref).max()
            assert err <= 2e-4 * np.abs(ref).max() + 1e-8, (k, err)
            n += 1
    assert n == 5
    before = model.user_embedding.weight.detach().clone()
    tr.optimizer.step()
    assert not torch.equal(before, model.user_embedding.weight.detach())
