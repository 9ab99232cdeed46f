"""GraphedStep.prepare(): every graph a timed loop replays is captured before it (bench.py's
timed region holds no capture whatever --warmup says), and the unrolled graph keeps the lazy-Adam
history ring from wrapping (FusedAdam.reserve_replays).

Reference: the step loop being timed, /root/reference/FoodRec/common/trainer.py:156-229."""
import numpy as np
import pytest
import torch

from helpers import tiny_config, tiny_data

pytestmark = pytest.mark.gpu


def _graphed(cuda, unroll, **over):
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("CIKM_Model", True, train_batch_size=32, cuda_graph=True, **over)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model)
    sampler = TripleSampler(data, 32, cfg["device"])
    g = tr.graphed_step(32, warmup=2, unroll=unroll)
    feed = g.attach_feed(sampler)

    def batches():
        while True:
            for t in sampler.epoch(out=g.inputs, feed=feed):
                yield t

    return tr, g, batches()


@pytest.mark.parametrize("unroll", [1, 4])
def test_prepare_leaves_no_capture_for_later_calls(cuda, unroll):
    tr, g, it = _graphed(cuda, unroll)
    state = g.state
    n = g.prepare(lambda: next(it), state)
    assert g.graph is not None
    assert (g.graph_n is not None) == (unroll > 1)
    assert g.captures == (2 if unroll > 1 else 1)
    assert g.pending == 0
    assert n == 2 + unroll + (1 if unroll > 1 else 0)  # warm-up, capture call(s), the one-step replay
    c0 = g.captures
    for i in range(20):  # crosses the 24-step epoch: a ragged eager batch and a restage on the way
        g(*next(it), n + i, state)
    g.flush()
    torch.cuda.synchronize()
    assert g.captures == c0, "a call after prepare() captured a graph"
    assert not int(state["nan"].item())


def test_unrolled_replay_never_wraps_the_lazy_ring(cuda):
    """hist_cap 6: an unroll-4 replay is exactly the ring's bound (hist_cap - 2); without the flush
    ahead of the replay the pending count would reach 7.  Parameters after 30 steps equal the
    unroll-1 run's (same graphs per step, deterministic scatters)."""
    out = []
    det0 = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        for unroll in (1, 4):
            tr, g, it = _graphed(cuda, unroll, lazy_row_adam=True, deterministic=True)
            tr.optimizer.hist_cap = 6
            seen = []
            orig = tr.optimizer.flush

            def flush(orig=orig, opt=tr.optimizer):
                seen.append(opt._lazy_pending)
                orig()

            tr.optimizer.flush = flush
            state = g.state
            n = g.prepare(lambda: next(it), state)
            for i in range(30):
                g(*next(it), n + i, state)
                assert tr.optimizer._lazy_pending <= tr.optimizer.hist_cap - 2
            g.flush()
            tr.flush_optimizer()
            torch.cuda.synchronize()
            assert max(seen) <= tr.optimizer.hist_cap - 2, seen
            out.append({k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()})
    finally:
        torch.use_deterministic_algorithms(det0)
    for k in out[0]:
        np.testing.assert_allclose(out[1][k].numpy(), out[0][k].numpy(), rtol=1e-6, atol=1e-7, err_msg=k)
