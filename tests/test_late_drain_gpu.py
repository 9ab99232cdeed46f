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
