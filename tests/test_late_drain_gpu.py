"""HealthRec's deferred ingredient rows added inside FusedAdam.step (ops.late_drain: the update of
every other tensor launched first, the rows scattered beside it on the branch stream, then the
ingredient table's update) against the rows added at the end of the backward pass: the same step
on the same batch leaves every gradient the step read within float-atomic reordering of the other
(1e-5 of its max; parameters are not compared -- Adam's first step is a sign step, so gradients
near zero may round either way)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _one_step(cuda, late, monkeypatch):
    from helpers import golden, tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import ops
    from FoodRec.utils.utils import get_model, init_seed
    monkeypatch.setattr(ops, "LATE_DRAIN", late)
    g = golden("model_CIKM_Model.npz")
    batch = {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}
    cfg = tiny_config("CIKM_Model", True)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(cuda)
    tr = Trainer(cfg, model)
    st = tr.new_step_state()
    seen = {}
    orig = ops.run_pending_drains

    def spy(**kw):
        seen["pending"] = seen.get("pending", 0) + len(ops._PENDING_DRAINS)
        return orig(**kw)
    monkeypatch.setattr(ops, "run_pending_drains", spy)
    tr.train_step(batch, 0, st)
    torch.cuda.synchronize()
    assert not ops._PENDING_DRAINS
    return ({k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None},
            seen.get("pending", 0))


def test_late_drain_step_matches_end_of_pass_drain(cuda, monkeypatch):
    a, n_late = _one_step(cuda, True, monkeypatch)
    b, n_eager = _one_step(cuda, False, monkeypatch)
    assert n_late >= 1 and n_eager == 0  # the late path actually ran (and only there)
    assert a.keys() == b.keys()
    assert "ingre_embedding.weight" in a
    for k in a:
        err = (a[k] - b[k]).abs().max().item()
        assert err <= 1e-5 * b[k].abs().max().item() + 1e-9, (k, err)


def _held_lazy_run(cuda, monkeypatch, branch, late):
    """A lazily updated table (lazy_rows) that takes some dense steps, each with deferred rows left for
    FusedAdam.step's drain (late) or already added into .grad on the host (not late), beside a dense
    tensor; flushed at the end.  Returns the table, the dense tensor and both tables' moments."""
    from FoodRec.engine import ops, optim
    from FoodRec.engine.optim import FusedAdam
    monkeypatch.setattr(optim, "HELD_ON_BRANCH", branch)
    torch.manual_seed(11)
    R, d = 300, 64
    w = torch.nn.Parameter(torch.randn(R, d).to(cuda))
    v = torch.nn.Parameter(torch.randn(4096, d).to(cuda))
    o = FusedAdam([w, v], lr=3e-3, lazy_rows=True, hist_cap=16)
    dense_at = {3, 4, 8, 11}
    for k in range(13):
        g = torch.Generator().manual_seed(500 + k)
        ids = torch.arange(R) if k == 0 else torch.randint(0, 70, (40,), generator=g)
        G = torch.randn(ids.numel(), d, generator=g)
        o.zero_grad()
        v.grad = torch.randn(v.shape, generator=g).to(cuda)
        if k in dense_at:
            # the dense part, plus rows (unique ids: atomic order cannot matter) drained late or added here
            rid = torch.randperm(R, generator=g)[:50]
            RG = torch.randn(50, d, generator=g)
            dense = torch.zeros(R, d).index_add_(0, ids, G)
            if late:
                w.grad = dense.to(cuda)
                defer = ops._DeferredRows()
                defer.put(rid.to(cuda), RG.to(cuda), None)
                fork = torch.cuda.Event()
                fork.record()
                ops._PENDING_DRAINS.append((fork, defer, w))
            else:
                w.grad = dense.index_add_(0, rid, RG).to(cuda)
        else:
            o.row_grads.stash(w, None, ids.to(cuda), G.to(cuda))
        o.step()
        assert not ops._PENDING_DRAINS
    o.flush()
    torch.cuda.synchronize()
    assert "lazy_last" in o.state[w]
    return [w.detach().clone(), v.detach().clone()] + [o.state[p][s].clone() for p in (w, v)
                                                       for s in ("exp_avg", "exp_avg_sq")]


def test_held_lazy_table_update_follows_its_flush(cuda, monkeypatch):
    """a late-drained table that carries lazy state, taking a dense step, is flushed (its
    deferred row steps replayed) on the current stream; with FR_HELD_ON_BRANCH its own update runs on
    the branch stream and must wait for that flush, not only for the point before the first update
    launch.  Parameters and moments after 13 steps (4 of them dense with late rows) are bit-identical
    with the held update on the branch stream, on the current stream, and with the rows added into
    .grad before the step."""
    ref = _held_lazy_run(cuda, monkeypatch, False, False)
    for branch in (True, False):
        got = _held_lazy_run(cuda, monkeypatch, branch, True)
        for a, b in zip(got, ref):
            assert torch.equal(a, b), branch
