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


def test_stamp_timer_inside_a_graph(cuda):
    """profiling.StampTimer (fr_stamp wall-clock stamps around a region, the roofline pass's timing
    inside a graph replay): a region captured in a graph reports a positive duration close to the
    same kernel's event-timed duration outside the graph; regions issued outside the capture are not
    reported."""
    from FoodRec.engine import profiling
    x = torch.randn(1 << 25, device=cuda)
    y = torch.empty_like(x)
    for _ in range(3):
        torch.mul(x, 2.0, out=y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.mul(x, 2.0, out=y)
    e1.record()
    torch.cuda.synchronize()
    eager_us = e0.elapsed_time(e1) / 10 * 1e3
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with profiling.stamping(cuda) as st:
        with torch.cuda.stream(side):
            with profiling.region("warm", 0):  # eager: stamped, not reported
                torch.mul(x, 2.0, out=y)
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(g):
            with profiling.region("mul", 8 * x.numel()):
                torch.mul(x, 2.0, out=y)
    assert st.hz > 0
    durs = []
    for _ in range(5):
        g.replay()
        got = st.read()
        assert [n for n, _, _ in got] == ["mul"]
        durs.append(got[0][1])
    med = sorted(durs)[2]
    assert 0.5 * eager_us < med < 2.0 * eager_us + 20.0, (med, eager_us)
