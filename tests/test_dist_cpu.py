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
