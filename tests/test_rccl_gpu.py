"""RCCL on the MI355X (the one-GPU box allows one rank: RCCL refuses two ranks on one device, so the
multi-rank runs are the driver's 8-GPU bench; the same code paths run here with every collective
forced through RCCL at world 1).

* the C-ABI communicator (fr_comm_unique_id / fr_comm_init / fr_allreduce_f32 / fr_allgather_f32,
  engine/comm.py): in-place sum and gather on data a kernel wrote on the caller's stream, issued
  both on that stream and asynchronously on the communicator's stream (wait() orders the caller);
  a collective captured in a HIP graph and replayed;
* the row-sharded config-4 step (engine/sharded.py) through a torch.distributed "nccl" (= RCCL)
  group and through the C-ABI communicator, collectives forced at world 1: the item all-reduce of
  every layer (async, overlapping the user SpMM) and the owner gathers; losses rel 1e-5 and
  gradients 1e-4 * max against the same step without collectives and the single-GPU LightGCN_ID;
* HealthRec's data-parallel step (engine/dist.py GradAllReduce with the row exchange forced on,
  Trainer.GraphedDPStep: graph A -> RCCL all-gather of the row stashes -> async RCCL all-reduce of
  the dense buffer overlapped with graph B1 -> graph B2) against the single-process graphed step,
  deterministic mode: per-step losses and all parameters after 6 steps rel 1e-6.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group(cuda):
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group already exists")
    store = dist.FileStore(os.path.join(tempfile.mkdtemp(prefix="frpg_"), "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=cuda)
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.destroy_process_group()


def test_cabi_comm_world_one(cuda):
    from FoodRec.engine import native
    from FoodRec.engine.comm import RcclComm
    assert native.lib().fr_comm_available() == 1
    comm = RcclComm(0, 1, RcclComm.unique_id())
    torch.manual_seed(0)
    x = torch.randn(1 << 20, device=cuda)
    ref = x.clone()
    y = x.mul(3.0)               # a kernel on the current stream produces the collective's input
    comm.all_reduce(y)
    torch.testing.assert_close(y, ref * 3.0, rtol=0, atol=0)
    z = x.add(1.0)
    work = comm.all_reduce(z, async_op=True)
    work.wait()
    z.mul_(2.0)                  # ordered after the collective by wait()
    torch.testing.assert_close(z, (ref + 1.0) * 2.0, rtol=0, atol=0)
    recv = torch.full((1, 4096), -1.0, device=cuda)
    send = x[:4096].contiguous()
    comm.all_gather(recv, send)
    torch.testing.assert_close(recv[0], send, rtol=0, atol=0)
    # a collective inside a captured HIP graph, replayed
    buf = torch.zeros(8192, device=cuda)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        buf.add_(1.0)
        comm.all_reduce(buf)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        buf.add_(1.0)
        comm.all_reduce(buf)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.all(buf == 4.0)  # 1 (eager warm-up) + 3 replays; capture itself executes nothing
    comm.close()


def _sharded_case(cuda, U=20000, I=3000):
    from FoodRec.engine.sharded import ShardedGraph
    from FoodRec.utils.interaction_graph import synth_bipartite
    u, i = synth_bipartite(U, I, 10.0, seed=3, device=cuda)
    return u, i, ShardedGraph(U, I, u, i, 0, 1, cuda, chunk=64)


def _close(a, b, rel):
    err = (a - b).abs().max().item()
    assert err <= rel * b.abs().max().item() + 1e-7, (err, b.abs().max().item())


@pytest.mark.parametrize("kind", ["torch_nccl", "cabi"])
def test_sharded_step_through_rccl_world_one(cuda, nccl_group, kind):
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import sharded
    from FoodRec.engine.comm import RcclComm
    from FoodRec.engine.sharded import ShardedLightGCN
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.interaction_graph import InteractionGraph
    U, I, d, B = 20000, 3000, 64, 512
    u, i, g1 = _sharded_case(cuda, U, I)
    group = nccl_group if kind == "torch_nccl" else RcclComm.from_process_group(nccl_group)
    calls = []
    real = sharded._all_reduce

    def counting(t, grp, async_op=False):
        calls.append(grp is not None)  # a group was handed over: the collective is issued (forced)
        return real(t, grp, async_op)

    sharded._all_reduce = counting
    try:
        with sharded.collectives_at_world_one():
            mR = ShardedLightGCN(g1, d, 2, 0.1, group=group, seed=7)
            m0 = ShardedLightGCN(g1, d, 2, 0.1, group=None, seed=7)
            uu, pp, nn_ = g1.triples(B, 5, 0)
            batch = {"u_id": uu, "pos_i_id": pp, "neg_i_id": nn_}
            mfR, regR = mR.calculate_loss(batch)
            (mfR + regR.sum()).backward()
            n_rccl = sum(calls)
            mf0, reg0 = m0.calculate_loss(batch)
            (mf0 + reg0.sum()).backward()
            # rows form (L = 2): forward the item flags, the layer-1 item rows at S and the 2B batch
            # item rows; backward the first layer's item rows at S + the second layer per item-row
            # block; + the owner gather of the batch users' propagated and ego rows (one [2B, d]);
            # + the |S| cross-check (check_same_count: one P-slot all-reduce)
            nb = len(g1.iu_blocks)
            assert nb >= 2 and n_rccl == nb + 6, (nb, calls)
            _close(mfR.detach(), mf0.detach(), 1e-5)
            _close(regR.detach(), reg0.detach(), 1e-5)
            _close(mR.ego_i.grad, m0.ego_i.grad, 1e-4)
            _close(mR.ego_u.grad, m0.ego_u.grad, 1e-4)
            g = InteractionGraph(U, I, pairs=(u, i), device=cuda, chunk=64)
            cfg = Config("LightGCN_ID", "Synthetic", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                      "ckp_root": "/tmp/frckp/"})
            cfg["device"] = cuda
            ms = LightGCN_ID(cfg, g)
            with torch.no_grad():
                ms.ego.copy_(torch.cat([m0.ego_u, m0.ego_i]))
            mfS, regS = ms.calculate_loss(batch)
            (mfS + regS.sum()).backward()
            _close(mfR.detach(), mfS.detach(), 1e-5)
            _close(torch.cat([mR.ego_u.grad, mR.ego_i.grad]), ms.ego.grad, 1e-4)
            # three trainer steps through RCCL stay finite and move the tables
            mR.zero_grad(set_to_none=True)
            tr = Trainer(cfg, mR)
            state = tr.new_step_state()
            before = mR.ego_i.detach().clone()
            for k in range(3):
                a, b, c = g1.triples(B, 5, 1 + k)
                tr.train_step({"u_id": a, "pos_i_id": b, "neg_i_id": c}, k, state)
            torch.cuda.synchronize()
            assert not int(state["nan"].item()) and not torch.equal(before, mR.ego_i.detach())
    finally:
        sharded._all_reduce = real
        if isinstance(group, RcclComm):
            group.close()


def test_healthrec_graphed_dp_step_through_rccl_world_one(cuda, nccl_group):
    from helpers import tiny_config, tiny_data
    from FoodRec.common.trainer import GraphedDPStep, Trainer
    from FoodRec.engine.dist import GradAllReduce
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    det0 = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    runs = []
    try:
        for dp in (False, True):
            cfg = tiny_config("CIKM_Model", True, train_batch_size=32, cuda_graph=True, deterministic=True)
            data = tiny_data(cfg)
            init_seed(999)
            model = get_model("CIKM_Model")(cfg, data).to(cuda)
            tr = Trainer(cfg, model)
            if dp:
                hook = GradAllReduce(model, 1, group=nccl_group, exchange_rows=True)
                assert hook.rows is not None
                tr.grad_hook = hook
            sampler = TripleSampler(data, 32, cuda)
            step = tr.graphed_step(32, warmup=2)
            assert isinstance(step, GraphedDPStep) == dp
            state = step.state
            trace = []
            for k, (u, p, n) in enumerate(sampler.epoch()):
                if k == 6:
                    break
                step(u, p, n, k, state)
                trace.append(state["acc"].cpu().numpy().copy())
            tr.flush_optimizer()
            runs.append((np.array(trace), {k: v.detach().clone() for k, v in model.state_dict().items()}))
    finally:
        torch.use_deterministic_algorithms(det0)
    (ta, sa), (tb, sb) = runs
    np.testing.assert_allclose(tb, ta, rtol=1e-6)
    for k in sa:
        torch.testing.assert_close(sb[k], sa[k], rtol=1e-6, atol=1e-7, msg=k)
