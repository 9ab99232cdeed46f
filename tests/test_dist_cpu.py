"""Multi-process data-parallel path on CPU (gloo, world_size 2): the gradient all-reduce hook that
bench.py / Trainer use for N>1 (engine/dist.py).  No GPU needed."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from FoodRec.engine.dist import GradAllReduce, init_from_env
    r, w, _ = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Embedding(50, 8), torch.nn.Linear(8, 3))
    unused = torch.nn.Parameter(torch.zeros(4))  # never receives a gradient
    model.register_parameter("unused", unused)
    hook = GradAllReduce(model, world)
    for step in range(2):
        model.zero_grad(set_to_none=True)
        g = torch.Generator().manual_seed(100 * step + rank)  # each rank its own batch
        ids = torch.randint(0, 50, (16,), generator=g)
        model[1](model[0](ids)).pow(2).sum().backward()
        local = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
        hook(model)
        torch.save({"local": local,
                    "reduced": {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None},
                    "unused_grad": unused.grad},
                   os.path.join(out_dir, f"r{rank}_s{step}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_gloo_world2(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for step in range(2):
        res = [torch.load(tmp_path / f"r{r}_s{step}.pt", weights_only=True) for r in range(world)]
        for name in res[0]["local"]:
            mean = sum(res[r]["local"][name] for r in range(world)) / world
            for r in range(world):
                torch.testing.assert_close(res[r]["reduced"][name], mean, rtol=1e-6, atol=1e-7)
            # replicas stay bit-identical: every rank holds the same averaged gradient
            assert torch.equal(res[0]["reduced"][name], res[1]["reduced"][name])
        assert res[0]["unused_grad"] is None


class _Sink:
    """Records what RowExchange.apply hands a FusedAdam row-gradient collector."""

    def __init__(self):
        self.calls = []

    def stash_factored(self, w, pad, ids, dY, W):
        self.calls.append((w, ids, dY.clone(), dY.data_ptr(), W))


def _row_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from FoodRec.engine.dist import RowExchange, init_from_env
    init_from_env(backend="gloo")
    img, txt = torch.zeros(40, 32), torch.zeros(40, 16)  # two row tables gathered at the same ids
    Wi, Wt = torch.randn(64, 32), torch.randn(64, 16)
    xg = RowExchange(dist.group.WORLD, world)
    xg.sink = _Sink()
    out = []
    for step in range(2):
        g = torch.Generator().manual_seed(10 * step + rank)
        ids = torch.randint(0, 40, (6,), generator=g)
        dYi, dYt = torch.randn(6, 64, generator=g), torch.randn(6, 64, generator=g)
        xg.stash_factored(img, None, ids, dYi, Wi)
        xg.stash_factored(txt, None, ids, dYt, Wt)
        xg.exchange()
        xg.sink.calls.clear()
        xg.apply()
        out.append({"ids": ids, "dYi": dYi, "dYt": dYt,
                    "calls": [(c[0] is img, c[1], c[2], c[3]) for c in xg.sink.calls],
                    "same_ids": xg.sink.calls[0][1] is xg.sink.calls[1][1]})
    torch.save(out, os.path.join(out_dir, f"rows_r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_row_exchange_gloo_world2_shared_ids(tmp_path):
    """RowExchange over gloo, two factored tables stashed with one ids tensor (HealthRec's image /
    text projections): one ids region on the wire; apply hands the sink ONE ids tensor (all ranks'
    ids, rank-major) and the rows mean-scaled, as adjacent 64-column views of one buffer."""
    world = 2
    mp.start_processes(_row_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [torch.load(tmp_path / f"rows_r{r}.pt", weights_only=False) for r in range(world)]
    for step in range(2):
        ids_all = torch.cat([res[r][step]["ids"] for r in range(world)])
        for r in range(world):
            st = res[r][step]
            assert st["same_ids"]
            (img_first, ids_i, dyi, pi), (_, ids_t, dyt, pt) = st["calls"]
            assert img_first and torch.equal(ids_i, ids_all) and torch.equal(ids_t, ids_all)
            assert pt == pi + 4 * 64  # adjacent column blocks of one buffer
            torch.testing.assert_close(dyi, torch.cat([res[q][step]["dYi"] for q in range(world)]) / world)
            torch.testing.assert_close(dyt, torch.cat([res[q][step]["dYt"] for q in range(world)]) / world)


def _distinct_ids_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from FoodRec.engine.dist import RowExchange, init_from_env
    init_from_env(backend="gloo")
    a, b = torch.zeros(40, 32), torch.zeros(40, 16)
    Wa, Wb = torch.randn(64, 32), torch.randn(64, 16)
    xg = RowExchange(dist.group.WORLD, world)
    xg.sink = _Sink()
    out = []
    for step in range(3):
        g = torch.Generator().manual_seed(10 * step + rank)
        # two tables with DIFFERENT ids of the same shape, each ids tensor a temporary freed right
        # after its stash (the pattern under which a recycled Python id() grouped them as shared);
        # at step 2 they share one ids tensor (the packed layout must change back)
        ia = torch.randint(0, 40, (6,), generator=g)
        ib = ia if step == 2 else torch.randint(0, 40, (6,), generator=g)
        dYa, dYb = torch.randn(6, 64, generator=g), torch.randn(6, 64, generator=g)
        xg.stash_factored(a, None, ia.reshape(-1).to(torch.int64) + 0, dYa, Wa)
        xg.stash_factored(b, None, (ib.reshape(-1).to(torch.int64) + 0) if step != 2 else ia, dYb, Wb)
        xg.exchange()
        xg.sink.calls.clear()
        xg.apply()
        calls = {c[0] is a: c[1].clone() for c in xg.sink.calls}
        out.append({"ia": ia, "ib": ib, "got_a": calls[True], "got_b": calls[False]})
    torch.save(out, os.path.join(out_dir, f"distinct_r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_row_exchange_distinct_ids_same_shape(tmp_path):
    """two tables stashed in one backward with different ids of equal shape are never
    grouped as sharing ids; each gets every rank's own ids back."""
    world = 2
    mp.start_processes(_distinct_ids_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [torch.load(tmp_path / f"distinct_r{r}.pt", weights_only=False) for r in range(world)]
    for step in range(3):
        ia = torch.cat([res[r][step]["ia"] for r in range(world)])
        ib = torch.cat([res[r][step]["ib"] for r in range(world)])
        for r in range(world):
            assert torch.equal(res[r][step]["got_a"].reshape(-1), ia)
            assert torch.equal(res[r][step]["got_b"].reshape(-1), ib)
