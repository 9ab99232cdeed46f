"""BASELINE config 4 path (LightGCN_ID on a synthetic interaction graph) at test scale: the device
triple sampler and one training step vs the oracle's CPU restatement.

Tolerances: losses rel 1e-5; ego gradient |err| <= 1e-4 * max|grad| (fp32 SpMM/scatter order);
the graph's CSR equals the numpy builder's bit for bit (tests/test_gpu_kernels covers Adam)."""
import numpy as np
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu

U, I = 3000, 800


def _graph(cuda, seed=1):
    from FoodRec.utils.interaction_graph import InteractionGraph
    return InteractionGraph(U, I, mean_deg=8.0, seed=seed, device=cuda, chunk=64)


def _config(cuda, **over):
    from FoodRec.utils.configurator import Config
    cd = {"use_gpu": True, "seed": 999, "reg_weight": 0.1, "n_layers": 2, "embedding_size": 64}
    cd.update(over)
    cfg = Config("LightGCN_ID", "Synthetic", cd)
    cfg["device"] = cuda
    return cfg


def test_interaction_graph_sampler(cuda):
    g = _graph(cuda)
    rp, col = g.adj.rowptr.cpu().numpy(), g.adj.col.cpu().numpy()
    assert rp[U] == g.n_edges and np.all(col[:g.n_edges] >= U)
    items = {u: set(col[rp[u]:rp[u + 1]] - U) for u in range(U)}
    seen = 0
    for _ in range(5):
        u, p, n = (x.cpu().numpy() for x in g.triples(512))
        for a, b, c in zip(u, p, n):
            assert b in items[a], "positive must be a training interaction"
            assert c not in items[a], "negative must not be a training interaction"
            assert 0 <= c < I
        seen += len(u)
    assert seen == 2560
    # negatives are uniform over items minus the user's: a chi-square-free sanity check on spread
    n = torch.cat([g.negatives(torch.randint(0, U, (20000,), device=cuda)) for _ in range(3)]).cpu().numpy()
    counts = np.bincount(n, minlength=I)
    assert counts.min() > 0 and counts.max() < 4 * counts.mean()


def test_interaction_graph_csr_matches_numpy_builder(cuda):
    from FoodRec.engine.graph import sym_norm_csr_np
    from FoodRec.utils.interaction_graph import synth_bipartite
    u, i = synth_bipartite(U, I, 8.0, seed=1, device=cuda)
    g = _graph(cuda)
    rp, col, val = sym_norm_csr_np(U + I, u.cpu().numpy(), i.cpu().numpy() + U)
    assert np.array_equal(g.adj.rowptr.cpu().numpy(), rp)
    assert np.array_equal(g.adj.col.cpu().numpy(), col)
    assert np.array_equal(g.adj.val.cpu().numpy(), val)


def test_lightgcn_id_step_matches_oracle(cuda):
    from FoodRec.models.lightgcn_id import LightGCN_ID
    g = _graph(cuda)
    torch.manual_seed(0)
    model = LightGCN_ID(_config(cuda), g)
    u, p, n = g.triples(512)
    ego0 = model.ego.detach().cpu().clone()
    mf, reg = model.calculate_loss({"u_id": u, "pos_i_id": p, "neg_i_id": n})
    (mf + reg).backward()
    grad = model.ego.grad.cpu()
    # oracle: the reference LightGCN arithmetic on CPU (lightgcn.py:134-177, loss.py)
    rp, col, val = (t.cpu().numpy() for t in (g.adj.rowptr, g.adj.col, g.adj.val))
    rows = np.repeat(np.arange(U + I), np.diff(rp))
    A = O.coo_to_torch(U + I, rows, col.astype(np.int64), val)
    E = ego0.clone().requires_grad_(True)
    out = O.propagate_mean(A, E, 2)
    uc, pc, nc = u.cpu(), p.cpu() + U, n.cpu() + U
    mf_r = O.bpr_loss((out[uc] * out[pc]).sum(1), (out[uc] * out[nc]).sum(1))
    reg_r = 0.1 * O.emb_loss(E[uc], E[pc], E[nc])
    (mf_r + reg_r).backward()
    torch.testing.assert_close(mf.detach().cpu(), mf_r.detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(reg.detach().cpu().reshape(-1), reg_r.detach().reshape(-1), rtol=1e-5, atol=1e-7)
    assert (grad - E.grad).abs().max() <= 1e-4 * E.grad.abs().max()


def test_lightgcn_id_state_dict_uses_reference_keys(cuda):
    from FoodRec.models.lightgcn_id import LightGCN_ID
    g = _graph(cuda)
    m = LightGCN_ID(_config(cuda), g)
    sd = m.state_dict()
    assert set(sd) == {"user_embedding.weight", "item_embedding.weight"}
    assert sd["user_embedding.weight"].shape == (U, 64) and sd["item_embedding.weight"].shape == (I, 64)
    m2 = LightGCN_ID(_config(cuda), g)
    m2.load_state_dict(sd)
    assert torch.equal(m2.ego, m.ego)


def test_lightgcn_id_steps_eagerly_and_captures_on_the_full_path(cuda):
    """The row-list propagation reads sizes back to the host, so the Trainer steps LightGCN_ID
    eagerly (use_graph False), and an explicit capture (graphed_step) falls back to the full
    propagation inside the graph: its steps match the eager rows-form steps (losses rel 1e-5,
    parameters 1e-5 * max after 4 Adam steps; float-atomic scatter order differs)."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.models.lightgcn_id import LightGCN_ID
    g = _graph(cuda)
    torch.manual_seed(0)
    me = LightGCN_ID(_config(cuda), g)
    mg = LightGCN_ID(_config(cuda), g)
    mg.load_state_dict(me.state_dict())
    te, tg = Trainer(_config(cuda), me), Trainer(_config(cuda), mg)
    assert not te.use_graph
    graphed = tg.graphed_step(512, warmup=1)
    se, sg = te.new_step_state(), graphed.state
    for k in range(4):
        u, p, n = g.triples(512)
        before = None if sg["acc"] is None else sg["acc"].clone()
        graphed(u, p, n, k, sg)
        ae = None if se["acc"] is None else se["acc"].clone()
        te.train_step({"u_id": u, "pos_i_id": p, "neg_i_id": n}, k, se)
        dg = sg["acc"] - (0 if before is None else before)
        de = se["acc"] - (0 if ae is None else ae)
        torch.testing.assert_close(dg, de, rtol=1e-5, atol=1e-7)
    assert graphed.graph is not None
    assert (mg.ego - me.ego).abs().max() <= 1e-5 * me.ego.abs().max()


def test_fused_step_returns_its_loss(cuda):
    """the fused-bookkeeping train_step returns the step's loss (a device fp32 scalar =
    the sum of the loss parts, as the reference's step returns loss), not None."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.models.lightgcn_id import LightGCN_ID
    g = _graph(cuda)
    torch.manual_seed(0)
    m = LightGCN_ID(_config(cuda), g)
    tr = Trainer(_config(cuda), m)
    st = tr.new_step_state()
    u, p, n = g.triples(512)
    with torch.no_grad():
        mf, reg = m.calculate_loss({"u_id": u, "pos_i_id": p, "neg_i_id": n})
    loss = tr.train_step({"u_id": u, "pos_i_id": p, "neg_i_id": n}, 0, st)
    assert torch.is_tensor(loss) and loss.is_cuda and loss.dtype == torch.float32
    assert float(loss) == pytest.approx(float(mf.reshape(-1)[0] + reg.reshape(-1)[0]), rel=1e-6)
    assert float(loss) == pytest.approx(float(st["acc"].sum()), rel=1e-6)
