"""Model- and trainer-level parity on the MI355X against goldens produced by the reference.

Tolerances: forward tables rel 1e-5 (abs 1e-6); loss components rel 1e-5; gradients rel 2e-4
of the tensor's max; one fused-Adam step applied to the reference's gradients <= 4 ulp of the
reference's parameters; training: per-epoch
loss trace rel 1e-4, final Recall/NDCG/AUC abs 1e-3 (the north-star parity bar).

HealthRec's trajectory is chaotic at the fp32-rounding level: its first Adam steps are sign(g) on
elements whose gradient is ~1e-5 of the tensor's max, and the reference's OWN 3-epoch trace moves
by up to 6e-3 (epoch 3) when its encoder layers' outputs are perturbed by one ulp or by +-4e-7 of
their max -- the fused layer's measured distance from float64 (tests/golden/
train_CIKM_Model_spread.npz, oracle/gen_golden.py --only spread).  Its trace and metrics are
therefore checked against that envelope: |ours - golden| <= max(1e-4 rel, the reference's largest
deviation over the perturbed runs) per epoch, metrics likewise with a 1e-3 floor.  The kernel
itself is held to float64 per layer (tests/test_encoder_gpu.py).
"""
import numpy as np
import pytest
import torch

from helpers import golden, tiny_config, tiny_data

pytestmark = pytest.mark.gpu

MODELS = ["LightGCN", "BPRMF", "CIKM_Model", "PRICAI_ModelX"]
# exact-stream training parity (HealthRec with the reference's attention dropout set to 0: the
# reference's CPU dropout masks cannot be reproduced on the device)
TRAINED = ["LightGCN", "BPRMF", "PRICAI_ModelX", "CIKM_Model"]


def _load_model(name, cuda):
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config(name, True)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model(name)(cfg, data).to(cfg["device"])
    return cfg, data, model


def _batch(g, cuda):
    return {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}


@pytest.mark.parametrize("name", MODELS)
def test_init_forward_loss_grad_adam(cuda, name):
    g = golden(f"model_{name}.npz")
    cfg, data, model = _load_model(name, cuda)
    for k, v in model.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), g["sd/" + k], err_msg=k)
    model.eval()
    with torch.no_grad():
        out = model.forward()
    np.testing.assert_allclose(out[0].detach().cpu().numpy(), g["fwd/user"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out[1].detach().cpu().numpy(), g["fwd/item"], rtol=1e-5, atol=1e-6)
    if "fwd/view_image" in g.files:
        for t, k in zip(out[2], ("image", "text", "ingre")):
            np.testing.assert_allclose(t.detach().cpu().numpy(), g["fwd/view_" + k], rtol=1e-5, atol=1e-6)
    from FoodRec.common.trainer import Trainer
    tr = Trainer(cfg, model)
    tr.optimizer.zero_grad()
    losses = model.calculate_loss(_batch(g, cuda))
    got = np.array([float(x.detach().reshape(-1)[0]) for x in losses])
    # EmbLoss norms over [B,20,64] ingredient blocks: torch-CPU's fp32 norm reduction is itself
    # ~1e-5 relative accurate at 655k elements (ours accumulates in fp64)
    np.testing.assert_allclose(got, g["loss"], rtol=5e-5)
    sum(losses).backward()
    tr.optimizer.materialize_row_grads()  # HealthRec's image/text tables hand Adam their rows
    for k, p in model.named_parameters():
        if "grad/" + k in g.files:
            ref = g["grad/" + k]
            assert p.grad is not None, k
            err = np.abs(p.grad.cpu().numpy() - ref).max()
            assert err <= 2e-4 * np.abs(ref).max() + 1e-8, (k, err)
    # optimiser-step parity in model context: our fused Adam applied to the REFERENCE's gradients
    # must reproduce the reference's parameters after its first step (<= 4 ulp; the gradients
    # themselves are checked above)
    for k, p in model.named_parameters():
        p.grad = torch.from_numpy(g["grad/" + k]).to(cuda) if "grad/" + k in g.files else None
    tr.optimizer.step()
    for k, p in model.named_parameters():
        got_p, ref_p = p.detach().cpu().numpy(), g["adam1/" + k]
        err = np.abs(got_p - ref_p)
        assert np.all(err <= 4 * np.spacing(np.abs(ref_p)) + 4 * np.spacing(np.float32(cfg["learning_rate"]))), \
            (k, err.max())


def _bars(name, g):
    """Per-epoch trace tolerance and per-metric tolerance: rel 1e-4 / abs 1e-3, widened for
    HealthRec to the reference's own spread under fp32-level perturbations (module docstring)."""
    ref = g["train_loss"]
    tr_tol = 1e-4 * np.abs(ref)
    met_tol = {k: 1e-3 for k in g["test_keys"].tolist()}
    if name == "CIKM_Model":
        sp = golden("train_CIKM_Model_spread.npz")
        tr_tol = np.maximum(tr_tol, np.abs(sp["train_loss"] - ref).max(axis=0))
        for j, k in enumerate(sp["test_keys"].tolist()):
            met_tol[k] = max(1e-3, float(np.abs(sp["test"][:, j] - g["test"][j]).max()))
    return tr_tol, met_tol


def _check_trace(name, g, trace):
    tr_tol, _ = _bars(name, g)
    assert np.all(np.abs(trace - g["train_loss"]) <= tr_tol), (name, trace, g["train_loss"], tr_tol)


@pytest.mark.parametrize("name", TRAINED)
def test_training_matches_reference(cuda, name):
    from FoodRec.common.trainer import Trainer
    g = golden(f"train_{name}.npz")
    cfg, data, model = _load_model(name, cuda)
    tr = Trainer(cfg, model)
    bv, bvr, btr = tr.fit(data, hyper_tuple=(999,), saved=True, verbose=False)
    trace = np.array([tr.train_loss_dict[e] for e in sorted(tr.train_loss_dict)])
    _check_trace(name, g, trace)
    _, met_tol = _bars(name, g)
    for keys, vals, got in ((g["valid_keys"], g["valid"], bvr), (g["test_keys"], g["test"], btr)):
        for k, v in zip(keys.tolist(), vals.tolist()):
            assert abs(got[k] - v) <= met_tol.get(k, 1e-3), (name, k, got[k], v)


@pytest.mark.parametrize("name", ["LightGCN", "PRICAI_ModelX", "CIKM_Model"])
def test_graphed_training_matches_reference(cuda, name):
    """The HIP-graph-captured step (cuda_graph=True) trains exactly like the eager one."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    g = golden(f"train_{name}.npz")
    cfg = tiny_config(name, True, cuda_graph=True, cuda_graph_warmup=1)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model(name)(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model)
    bv, bvr, btr = tr.fit(data, hyper_tuple=(999,), saved=True, verbose=False)
    assert tr._graphed is not None and tr._graphed.graph is not None, "graph was never captured"
    trace = np.array([tr.train_loss_dict[e] for e in sorted(tr.train_loss_dict)])
    _check_trace(name, g, trace)
    _, met_tol = _bars(name, g)
    for k, v in zip(g["test_keys"].tolist(), g["test"].tolist()):
        assert abs(btr[k] - v) <= met_tol[k], (name, k, btr[k], v)


def test_mirror_gradient_training_matches_reference(cuda):
    """--mg (trainer.py:195-212): every beta-th batch steps on alpha1*loss, recomputes the loss on
    the same batch and back-propagates -alpha2*loss before the regular step; mg.yaml resolved to
    its first hyper-parameter values (alpha1 1, alpha2 0.1, beta 3) as quick_start does."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("train_mg_LightGCN.npz")
    cfg = tiny_config("LightGCN", True, mg=True)
    assert (cfg["alpha1"], cfg["alpha2"], cfg["beta"]) == (float(g["alpha1"]), float(g["alpha2"]), int(g["beta"]))
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("LightGCN")(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model, mg=True)
    bv, bvr, btr = tr.fit(data, hyper_tuple=(999,), saved=True, verbose=False)
    trace = np.array([tr.train_loss_dict[e] for e in sorted(tr.train_loss_dict)])
    np.testing.assert_allclose(trace, g["train_loss"], rtol=1e-4)
    for keys, vals, got in ((g["valid_keys"], g["valid"], bvr), (g["test_keys"], g["test"], btr)):
        for k, v in zip(keys.tolist(), vals.tolist()):
            assert abs(got[k] - v) <= 1e-3, ("mg", k, got[k], v)


@pytest.mark.parametrize("drop", [0.0, 0.5])
def test_healthrec_graphed_lazy_equals_eager_dense(cuda, drop):
    """The HealthRec step bench.py times (captured graph, DeviceFeed batch gather, lazy row Adam with
    the side-stream catch-up, automatic flushes of a small history ring) against the eager step with
    the every-row Adam, over 2 epochs of 24 steps (B = 32: 23 graph replays + the ragged eager
    batch per epoch), attention dropout 0 and the bench's 0.5 (the replayed graph must draw the
    same per-step encoder keep-masks as the eager steps: device counters advance alike).  Both runs are made run-to-run reproducible (config
    ``deterministic``: owner-slot BPR scatter; torch's deterministic index_add_): Adam turns last-bit
    noise in near-zero gradients into +-lr steps, so atomics alone would make any two runs differ.
    Per-epoch loss sums and every parameter and Adam moment after the epochs (flushed) agree to
    fp32 round-off (rel 1e-6)."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    runs = []
    det0 = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        _graphed_vs_eager_runs(runs, Trainer, TripleSampler, get_model, init_seed, drop)
    finally:
        torch.use_deterministic_algorithms(det0)
    (la, sa, oa, ma), (lb, sb, ob, mb) = runs
    np.testing.assert_allclose(lb, la, rtol=1e-6)
    for k in sa:
        torch.testing.assert_close(sb[k], sa[k], rtol=1e-6, atol=1e-7, msg=k)
    for (k, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        if pa in oa.state:
            for s_ in ("exp_avg", "exp_avg_sq"):
                torch.testing.assert_close(ob.state[pb][s_], oa.state[pa][s_], rtol=1e-6, atol=1e-9, msg=(k, s_))


def _graphed_vs_eager_runs(runs, Trainer, TripleSampler, get_model, init_seed, drop=0.0):
    for graphed in (False, True):
        cfg = tiny_config("CIKM_Model", True, train_batch_size=32, cuda_graph=graphed, cuda_graph_warmup=2,
                          lazy_row_adam=graphed, deterministic=True, attention_probs_dropout_prob=drop)
        data = tiny_data(cfg)
        init_seed(999)
        model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
        tr = Trainer(cfg, model)
        assert tr.optimizer.lazy_rows == graphed
        tr.optimizer.hist_cap = 7  # ring wraps every 5 steps: automatic flushes inside the epochs
        sampler = TripleSampler(data, 32, cfg["device"])
        assert len(sampler) == 24
        losses = [tr._train_epoch(sampler, e)[0] for e in range(2)]
        if graphed:
            assert tr._graphed is not None and tr._graphed.graph is not None
        runs.append((np.array(losses), model.state_dict(), tr.optimizer, model))
