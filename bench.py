"""Benchmark: BPR training triples/sec on MI355X (BASELINE.json metric), one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload healthrec_allrecipes]

Workload (N=1 line = BASELINE configs[1]): HealthRec (reference CIKM_Model) on a seeded synthetic
Allrecipes-shaped dataset (U=68,768, I=45,630, ~677k train pairs, NI=19,987, 2048-d image /
512-d text features, 7-bit health), d=64, B=512 triples per step per GPU.  A "step" is the
reference's full training step on one batch: native triple sampling (exact reference RNG
stream), forward (RI + UI SpMM propagation, ingredient Transformer, target attention, KD and
health heads), the fused BPR/EmbLoss, backward, and the fused Adam update over all 125.7M
parameters.  Inputs are resident in HBM before timing; the host->device copy of each batch's
sampled indices is inside the step.

N>1 (torch.distributed.run, RCCL): data-parallel replicas, each rank steps its own 512-triple
batch and the dense gradient buffer is all-reduced over xGMI every step ("scaling": "weak";
value = triples of all ranks / max-over-ranks time).

Extra objects on the line:
  roofline      dominant kernel (by measured time over the timed steps, HIP events on the launch
                stream): algorithmic bytes per launch / average launch time vs 8 TB/s HBM peak
  spmm          the propagation SpMM's own achieved GB/s (the metric's "SpMM HBM GB/s")
  cpu_baseline  the oracle's CPU restatement of the same step (torch-CPU, oracle/cpu_backend.py)
                timed on this host's cores on a bounded number of steps (rank 0, N=1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); N > 1 without a torch.distributed environment starts "
                         "the N ranks itself under torch.distributed.run (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="healthrec_allrecipes", choices=["healthrec_allrecipes"])
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--cpu-baseline-steps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes/launch of the dominant kernel from rocprofv3 PMC (profiles/)")
    ap.add_argument("--eager", action="store_true", help="do not capture the step in a HIP graph")
    ap.add_argument("--kernel-steps", type=int, default=10,
                    help="eager steps of the per-kernel HIP-event timing pass (roofline)")
    ap.add_argument("--no-spmm-10m", action="store_true",  # also skips the config-4 training step
                    help="skip the SpMM measurement on the 10M x 1M x 200M synthetic graph")
    ap.add_argument("--check-launch", action="store_true",
                    help="launcher self-test: start the ranks, join the process group (gloo, CPU), assert "
                         "the world size and print the n_gpus line -- no GPU work")
    ap.add_argument("--config-json", default=None, help="extra config keys for the HealthRec step (JSON)")
    ap.add_argument("--no-config3", action="store_true",
                    help="skip BASELINE config 3 (CLUSSL on Foodcom-shape data, dCor and InfoNCE SSL)")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip BASELINE config 5 (d=256 bf16 tables, full-sort top-k on MFMA)")
    ap.add_argument("--no-config1", action="store_true",
                    help="skip BASELINE config 1 (BPRMF on Allrecipes-shape data, GPU step + CPU oracle)")
    ap.add_argument("--no-eval", action="store_true",
                    help="skip the per-epoch evaluation leg (68,768 test users ranked on the device)")
    return ap.parse_args()


def build(device, batch, seed=0, dataset_seed=0, extra=None):
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.synthetic import make_synthetic
    from FoodRec.utils.utils import get_model, init_seed
    ds = make_synthetic("allrecipes", dataset_seed, negatives=False)
    data = FoodData.from_synthetic(ds)
    cfg = Config("CIKM_Model", "Allrecipes", {"use_gpu": device.type == "cuda", "seed": 999, "cuda_graph": True,
                                             "train_batch_size": batch, "log_root": "/tmp/frlog/",
                                             "ckp_root": "/tmp/frckp/", **(extra or {}),
                                             # FR_BENCH_CFG: JSON config overrides for A/B runs
                                             **json.loads(os.environ.get("FR_BENCH_CFG", "{}"))})
    cfg["device"] = device
    data.args_config = cfg
    init_seed(999 + seed)
    model = get_model("CIKM_Model")(cfg, data).to(device)
    return cfg, data, model


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_command(gpus: int, argv, port: int):
    """The child command that starts ``gpus`` ranks of this script (one process per GPU, rendezvous on
    127.0.0.1): torch.distributed.run with the caller's own arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(gpus)}",
            "--master-addr", "127.0.0.1", "--master-port", str(int(port)), os.path.abspath(__file__), *argv]


def spawn_ranks(gpus: int, argv) -> int:
    """``--gpus N > 1`` run outside torch.distributed: start the N ranks as a CHILD process and return
    its exit status.  This process imports nothing that touches HIP (the ranks own the GPUs); rank 0
    prints the JSON line on the shared stdout."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only (RCCL across processes)
    return subprocess.run(launch_command(gpus, argv, _free_port()), env=env).returncode


def resolve_world(gpus, environ) -> int:
    """Ranks this process belongs to: WORLD_SIZE when launched by torch.distributed.run (it must equal
    ``--gpus`` when both are given), else ``--gpus`` (default 1)."""
    if "WORLD_SIZE" in environ:
        world = int(environ["WORLD_SIZE"])
        if gpus is not None and int(gpus) != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: the launcher started a "
                             f"different number of ranks")
        return world
    return 1 if gpus is None else int(gpus)


def _check_launch(args, world, rank):
    """--check-launch: the process-group half of a multi-rank run on the CPU (gloo)."""
    import torch.distributed as dist
    from FoodRec.engine.dist import init_process_group  # explicit collective timeout (FR_PG_TIMEOUT_S)
    if world > 1:
        init_process_group("gloo")
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
        got = dist.get_world_size()
        dist.destroy_process_group()
    else:
        got = 1
    if rank == 0:
        print(json.dumps({"check_launch": True, "n_gpus": got, "gpus_requested": args.gpus,
                          "backend": "gloo" if world > 1 else None}), flush=True)
    return 0


def main():
    args = _args()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        return spawn_ranks(args.gpus, sys.argv[1:])
    world = resolve_world(args.gpus, os.environ)
    args.gpus = world
    rank = int(os.environ.get("RANK", "0"))
    if args.check_launch:
        return _check_launch(args, world, rank)
    import numpy as np
    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FR_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks sharing one GPU (the driver's
    # multi-GPU runs use RCCL, one rank per GPU)
    backend = os.environ.get("FR_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    if world > 1 and backend == "nccl" and ndev < world:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, {ndev} visible "
                         f"(FR_BENCH_BACKEND=gloo rehearses several ranks on one GPU)")
    local = local % ndev
    # FR_BENCH_DP1=1: the data-parallel step (row exchange + dense all-reduce through RCCL, graphs A /
    # B1 / B2 around the collectives) at world 1 -- the per-rank cost of the N > 1 path on one GPU
    dp1 = world == 1 and os.environ.get("FR_BENCH_DP1") == "1"
    from FoodRec.engine.dist import init_process_group  # explicit collective timeout (FR_PG_TIMEOUT_S)
    if dp1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        init_process_group("nccl", torch.device("cuda", local), rank=0, world_size=1)
    if world > 1:
        torch.cuda.set_device(local)
        init_process_group(backend, torch.device("cuda", local) if backend == "nccl" else None)
        # the job really runs ``world`` ranks: checked against the process group itself
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    device = torch.device("cuda", local)
    ranks = _rank_report(world, backend, device) if world > 1 else None

    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import profiling
    from FoodRec.engine.dist import GradAllReduce
    from FoodRec.engine.sampler import TripleSampler

    cfg, data, model = build(device, args.batch, extra=json.loads(args.config_json) if args.config_json else None)
    trainer = Trainer(cfg, model)
    if world > 1 or dp1:
        trainer.grad_hook = GradAllReduce(model, world, exchange_rows=True if dp1 else None)
    np.random.seed(1000 + rank)  # each replica draws its own triple stream
    sampler = TripleSampler(data, args.batch, device, replay_python_random=False)
    feats = trainer._features()
    state = trainer.new_step_state()
    model.train()

    use_graph = not args.eager  # N>1: two graphs per step, gradient collectives between them
    graphed = trainer.graphed_step(args.batch, warmup=3) if use_graph else None
    feed = None
    if graphed is not None:
        # the sampler stages each epoch's permutation and negatives on the device and the graph
        # gathers its own batch (DeviceFeed) and accumulates into its own state: per step the host
        # only replays the graph
        state = graphed.state
        feed = graphed.attach_feed(sampler)

    def batches():
        while True:
            for t in sampler.epoch(out=graphed.inputs if graphed is not None else None, feed=feed, prefetch=True):
                yield t

    it = batches()
    # per-epoch sampling (permutation, the epoch's negatives in one native call, H2D copy, staging),
    # once per 1,323-step epoch.  As in the trainer on a GPU, the host draws of epoch e + 1 run on a
    # host thread during epoch e (TripleSampler.prefetch); what the epoch boundary still costs (the
    # prefetched draws' copy to the device and the feed's staging) is timed here and amortised into
    # `value` (epoch_sampling.ms_per_epoch / steps_per_epoch per step); the draw itself is timed on
    # its thread (host_draw_ms), and the timed steps below run with such a draw in flight.
    # (the median of three boundaries, so one noisy host sample does not move `value`)
    probes, draws = [], []
    for _ in range(3):
        sampler.prefetch()
        sampler.wait_prefetch()  # the previous epoch's steps have covered the draw
        draws.append(sampler.last_draw_ms)
        torch.cuda.synchronize()
        te0 = time.perf_counter()
        probe = sampler.epoch(out=graphed.inputs if graphed is not None else None, feed=feed)
        next(probe)
        torch.cuda.synchronize()
        probes.append((time.perf_counter() - te0) * 1e3)
        del probe
    epoch_ms = sorted(probes)[1]
    draw_ms = sorted(draws)[1]
    steps_per_epoch = len(sampler)

    def do_step(i):
        u, p, n = next(it)
        if graphed is not None:
            graphed(u, p, n, i, state)
        else:
            trainer.train_step(feats.batch(u, p, n), i, state)

    # every HIP graph the timed steps replay (the one-step graph and the unrolled graph) is captured
    # and replayed once here, whatever --warmup says: no capture lands inside the timed region
    prep_steps = graphed.prepare(lambda: next(it), state) if graphed is not None else 0
    for i in range(args.warmup):
        do_step(prep_steps + i)
    if graphed is not None:
        graphed.flush()  # no warm-up step left pending for the timed region
    captures0 = graphed.captures if graphed is not None else 0
    # a next-epoch draw in flight on its host thread while the steps run (the trainer's steady state
    # for the first ~40 steps of every epoch; here over the whole timed region)
    sampler.discard_prefetch()
    sampler.prefetch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        do_step(prep_steps + args.warmup + i)
    if graphed is not None:
        graphed.flush()  # steps of an unrolled graph not yet replayed run inside the timed region
    t_submit = time.perf_counter() - t0  # host time to issue the steps (graph replays): < elapsed when GPU-bound
    torch.cuda.synchronize()
    t_steps = time.perf_counter() - t0
    captures_timed = (graphed.captures - captures0) if graphed is not None else 0
    assert captures_timed == 0, f"{captures_timed} graph capture(s) inside the timed region"
    # the deferred zero-gradient row steps of the lazily updated tables (FusedAdam lazy rows): the
    # trainer applies them once per epoch (_train_epoch's flush_optimizer, before evaluation); here
    # they run right after the steps, inside the bracket, and are timed on their own: `value`
    # charges them per epoch like the epoch's sampling (every parameter holds its dense-Adam value
    # when the bracket closes)
    trainer.flush_optimizer()
    torch.cuda.synchronize()
    t_flushed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, t_steps, t_flushed - t_steps], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, t_steps, flush_s = (float(x) for x in t.tolist())
    else:
        flush_s = t_flushed - t_steps
    assert not int(state["nan"].item()), "NaN loss during bench"
    # per-kernel HIP-event timing (roofline): the same kernels, launched eagerly on the same
    # stream right after the timed region (events cannot bracket single kernels inside a replay)
    with profiling.timing() as timer:
        tk0 = time.perf_counter()
        for i in range(args.kernel_steps):
            u, p, n = next(it)
            if feed is not None and u is graphed.inputs[0]:
                feed.fill(u, p, n)  # eager step: gather the batch the graph would have gathered
            trainer.train_step(feats.batch(u, p, n), i, state)
        torch.cuda.synchronize()
        eager_elapsed = time.perf_counter() - tk0
    kern = timer.summary()
    ksteps = max(1, args.kernel_steps)
    # the same eager pass with the propagation branch serialised (nothing runs beside the encoder):
    # the kernels' own durations, next to the in-step ones above (stretched by the branch's SpMMs)
    from FoodRec.engine import ops as _ops_mod
    branch0 = _ops_mod.BRANCH_STREAMS
    _ops_mod.BRANCH_STREAMS = False
    try:
        with profiling.timing() as timer_iso:
            for i in range(args.kernel_steps):
                u, p, n = next(it)
                if feed is not None and u is graphed.inputs[0]:
                    feed.fill(u, p, n)
                trainer.train_step(feats.batch(u, p, n), i, state)
            torch.cuda.synchronize()
        kern_iso = timer_iso.summary()
    finally:
        _ops_mod.BRANCH_STREAMS = branch0

    # the same regions inside a graph replay: a one-step graph of the training step captured with
    # device wall-clock stamps around every region (timing events cannot be recorded in a graph)
    kern_graph = None
    if graphed is not None and world == 1 and not dp1 and args.kernel_steps > 0:
        kern_graph = graph_region_pass(trainer, args.batch, sampler, device, args.kernel_steps)

    ms_steps = t_steps / args.steps * 1e3
    flush_ms = flush_s * 1e3
    ms_per_step = ms_steps + (epoch_ms + flush_ms) / steps_per_epoch
    triples = args.batch * args.steps * world
    value = triples / (ms_per_step * 1e-3 * args.steps)

    # dominance by median launch x launches: one launch stretched by a host stall does not move it
    dom_name = max(kern, key=lambda k: kern[k]["median_ms"] * kern[k]["launches"]) if kern else None
    traffic = args.traffic if args.traffic is not None else pmc_traffic(dom_name)
    roofline = None
    if dom_name is not None:
        d = dict(kern[dom_name])
        eager_d = dict(d)
        src = ("HIP events per launch on the launch stream, eager pass of "
               f"{ksteps} steps right after the timed region (kernels.{dom_name})")
        if kern_graph is not None and dom_name in kern_graph:
            gd = kern_graph[dom_name]
            d.update(avg_ms=gd["avg_ms"], total_ms=gd["avg_ms"] * gd["launches_per_step"] * ksteps,
                     launches=gd["launches_per_step"] * ksteps)
            src = ("device wall-clock stamps (fr_stamp) around each call inside a graph replay: a one-step graph "
                   f"of the training step captured with the stamps, {gd['replays']} replays (kernels_in_graph."
                   f"{dom_name}; includes the stamps' launch gaps)")
        common = {"kernel": dom_name, "avg_launch_ms": round(d["avg_ms"], 4), "launches_per_step": d["launches"] / ksteps,
                  "share_of_step": round(d["total_ms"] / ksteps / ms_per_step, 3), "timing_source": src}
        if dom_name.startswith("encoder_"):
            # the fused Transformer layer: fp32 MFMA GEMMs (v_mfma_f32_16x16x4_f32) -> an MFMA roofline
            from FoodRec.engine import ops as _ops
            fl = _ops.encoder_flops(2 * args.batch, 20, dom_name.endswith("bwd"))
            tf = fl / (d["avg_ms"] * 1e-3) / 1e12
            roofline = {**common, "bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_F32_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(tf / MFMA_F32_PEAK_TFLOPS, 4), "traffic": traffic,
                        "flops_per_launch": fl, "bytes_per_launch": int(d["bytes_per_launch"]),
                        "region_kernels": ("enc_bwd_kernel<20> + its layer's ordered weight-gradient reduction "
                                           "(enc_reduce_kernel), one fr_encoder_bwd call per layer; avg_launch_ms "
                                           "averages the two layers' calls"
                                           if dom_name.endswith("bwd") else "enc_fwd_kernel<20>"),
                        "note": "dense fp32 MFMA peak; the layer's 20x20 attention, LayerNorms, GELU and dropout "
                                "hash run on the VALU between the GEMMs (latency-bound at 1 workgroup per CU)"}
            tfe = fl / (eager_d["avg_ms"] * 1e-3) / 1e12
            roofline["eager"] = {"avg_launch_ms": round(eager_d["avg_ms"], 4), "achieved": round(tfe, 2),
                                 "frac": round(tfe / MFMA_F32_PEAK_TFLOPS, 4),
                                 "note": "HIP events in the eager pass (other streams' kernels overlap it differently "
                                         "than in the graph)"}
            iso = kern_iso.get(dom_name)
            if iso is not None:
                tfi = fl / (iso["avg_ms"] * 1e-3) / 1e12
                roofline["isolated"] = {"avg_launch_ms": round(iso["avg_ms"], 4), "achieved": round(tfi, 2),
                                        "frac": round(tfi / MFMA_F32_PEAK_TFLOPS, 4),
                                        "note": "same eager pass with the propagation branch serialised (FR_BRANCH_"
                                                "STREAMS off): the launch without the RI / UI SpMMs beside it"}
        else:
            achieved = d["gbps"]
            roofline = {**common, "bound": "hbm", "achieved": round(achieved, 1),
                        "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                        "traffic": traffic, "bytes_per_launch": int(d["bytes_per_launch"]),
                        "residency": ("the gathered X tables (<= 29 MB) sit in the 256 MB Infinity Cache (MALL): "
                                      "this is a cache-level rate; the HBM-level SpMM roofline is config4_10m.spmm"
                                      if dom_name == "spmm" else None)}
    # the propagation SpMM's own figures (the metric's "SpMM HBM GB/s") are in `spmm` below
    # step-level figure: algorithmic bytes of every timed region per step / the graphed step time
    step_bytes = sum(v["bytes_per_launch"] * v["launches"] for v in kern.values()) / ksteps
    step_fig = {"algorithmic_bytes_per_step": int(step_bytes),
                "achieved_gbps": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                "frac_of_hbm_peak": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "note": "sum over the engine's timed regions (their byte models) per step; latency-bound "
                        "step: ~80 launches of mostly L2/MALL-resident work"}
    spmm = None
    if "spmm" in kern:
        s = kern["spmm"]
        spmm = {"achieved_gbps": round(s["gbps"], 1), "avg_launch_ms": round(s["avg_ms"], 4),
                "bytes_per_launch": int(s["bytes_per_launch"]), "launches_per_step": s["launches"] / ksteps,
                "frac_of_hbm_peak": round(s["gbps"] / HBM_PEAK_GBPS, 4),
                "note": "Allrecipes-shape X tables (<=29 MB) are Infinity-Cache resident"}
    kernels = {k: {"avg_ms": round(v["avg_ms"], 4), "per_step_ms": round(v["total_ms"] / ksteps, 4),
                   "gbps": round(v["gbps"], 1)} for k, v in kern.items()}
    graph_unroll = (graphed.unroll if world == 1 and not dp1 else 1) if graphed is not None else 0
    if kern_graph is not None:
        kernels["_in_graph"] = kern_graph
    kernels["_timing"] = {"step_execution": "hip_graph_replay" if use_graph else "eager",
                          "kernel_pass": f"{ksteps} eager steps, HIP events on the launch stream",
                          "eager_ms_per_step": round(eager_elapsed / ksteps * 1e3, 4)}

    c3 = None
    if world == 1 and not args.no_config3:
        del graphed, state
        c3 = config3(device, cpu=not args.no_cpu_baseline)
        graphed = state = None
    c4 = None
    if not args.no_spmm_10m:
        del trainer, model, sampler, state, graphed
        torch.cuda.empty_cache()
        if world == 1:
            c4 = config4(device, cpu=not args.no_cpu_baseline)
            # the row-sharded step at P = 1 (no collectives): the denominator of the N-GPU runs'
            # config4_10m line (the driver's multi-GPU bench runs config4_sharded at P = N)
            c4["sharded_p1"] = config4_sharded(device, 1, 0)
        else:
            c4 = config4_sharded(device, world, rank)
    c5 = None
    if world == 1 and not args.no_config5:
        c5 = config5(device)
    c1 = None
    if world == 1 and not args.no_config1:
        c1 = config1(device, cpu=not args.no_cpu_baseline)
    ev = None
    if world == 1 and not args.no_eval:
        ev = eval_leg(device)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    # the config-4 row-sharded step at a fixed global batch (strong scaling): the north star's
    # "10M-user/1M-item" scaling figure, beside the HealthRec data-parallel `value` (weak scaling)
    c4_scaling = None
    if c4 is not None:
        sh = c4.get("sharded_p1") if world == 1 else c4
        c4_scaling = {"workload": "config4_10m LightGCN_ID row-sharded (U=10M, I=1M, E=200M, d=64)",
                      "scaling": "strong", "ranks": world,
                      "per_global_batch": {b: {"ms_per_step": v["ms_per_step"], "triples_per_s": v["triples_per_s"]}
                                           for b, v in sh["step"].items()},
                      "note": "every rank steps the same global batch B; triples_per_s = B / max-over-ranks "
                              "step time; compare across n_gpus at equal B"}
    n_pg = dist.get_world_size() if world > 1 else 1
    if rank == 0:
        line = {"metric": "BPR triples/sec + SpMM HBM GB/s, Allrecipes d=64, 1/2/4/8 MI355X",
                "value": round(value, 1), "unit": "triples/s", "n_gpus": n_pg, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                "config": {"workload": "healthrec_allrecipes", "model": "HealthRec (CIKM_Model)",
                           "dataset": "Allrecipes-shape synthetic (U=68768, I=45630, train=677054)",
                           "embedding_size": 64, "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                           "parallelism": f"dp{world}" if world > 1 else ("dp1 (forced exchange)" if dp1 else "single"),
                           "graph_steps_per_replay": graph_unroll},
                "roofline": roofline, "ranks": ranks, "scaling_config4": c4_scaling, "step_bytes": step_fig,
                "timed_region": {"graph_captures_in_timed_region": captures_timed,
                                 "prepare_steps": prep_steps, "warmup_steps": args.warmup,
                                 "elapsed_s": round(elapsed, 6), "steps_s": round(t_steps, 6),
                                 "note": "GraphedStep.prepare() captured and replayed every graph before t0 "
                                         "(prepare_steps untimed training steps, then --warmup steps)"},
                "epoch_sampling": {"ms_per_epoch": round(epoch_ms, 2), "probes_ms": [round(x, 2) for x in probes],
                                   "steps_per_epoch": steps_per_epoch,
                                   "ms_per_step_without": round(ms_steps, 4),
                                   "host_submit_ms_per_step": round(t_submit / args.steps * 1e3, 4),
                                   "steps_ms_per_step": round(t_steps / args.steps * 1e3, 4),
                                   "lazy_flush_ms_per_epoch": round(flush_ms, 3),
                                   "host_draw_ms": round(draw_ms, 2), "prefetch": True,
                                   "note": "value and ms_per_step = the timed steps + (epoch_sampling.ms_per_epoch, "
                                           "the median of three epoch boundaries, + the once-per-epoch lazy-row "
                                           "flush, timed inside the bracket after the steps) / steps_per_epoch; "
                                           "the epoch's host draws (host_draw_ms: permutation + negatives) run on "
                                           "a host thread during the previous epoch, as in the trainer on a GPU "
                                           "(TripleSampler.prefetch), and the timed steps ran with one in flight; "
                                           "ms_per_epoch is what the boundary still costs (the draws' H2D copy "
                                           "and the feed's staging)"},
                "spmm": spmm, "config1_bprmf_allrecipes": c1, "config3_clussl_foodcom": c3, "config4_10m": c4,
                "config5_10m_bf16": c5, "eval_healthrec_allrecipes": ev, "kernels": kernels, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if world > 1 or dp1:
        dist.destroy_process_group()


# the kernels each engine timing region launches on HEAD (tools/pmc_regions.py REGION_KERNELS): a
# committed PMC file sampled from other kernels is stale and is not used
REGION_KERNELS = {"encoder_bwd": ["enc_bwd_kernel", "enc_reduce_kernel"], "encoder_fwd": ["enc_fwd_kernel"],
                  "spmm": ["spmm_plain16_kernel"], "spmm_masked": ["spmm_sparse_kernel"],
                  "spmm_rows": ["spmm_rows_kernel"], "adam": ["adam_kernel<false, false>"],
                  "adam_rows": ["adam_lazy_rows_kernel<false>"]}


def pmc_traffic(kernel):
    """HBM bytes per launch of region ``kernel`` measured by rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE,
    the gfx950 calibration) in separate profiling passes, committed under profiles/ (newest round),
    or None when that file's region was sampled from other kernels than the region launches today."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    if not files or kernel is None:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    if d.get("region_kernels", {}).get(kernel) != REGION_KERNELS.get(kernel):
        return None
    return d.get("per_region_bytes", {}).get(kernel)


def config4_bytes_per_step(N, nnz, P, B, L=2, d=64, s=4, adam=28):
    """SURVEY 8(d) algorithmic bytes of one LightGCN-ID step (no-reuse gather model).  ``adam``:
    bytes per parameter of the optimiser pass (28 fp32; 30 for bf16 params + fp32 master/m/v)."""
    b_spmm = 8 * (N + 1) + nnz * 8 + nnz * d * s + N * d * s
    return 2 * L * b_spmm + 2 * (L + 1) * N * d * s + adam * P + B * (3 * 8 + 3 * d * s) * 2, b_spmm


def config4_bytes_rows(N, nnz, P, B, deg_rows, layer1=None, d=64, s=4, adam=28):
    """Algorithmic bytes of the LightGCN-ID step as the engine runs it (L = 2, ops.propagate_rows):
    layer 1 over the full graph, or (``layer1`` = (rows, edges) it covers) over the user block plus
    the items layer 2 reads; layer 2 only at the 3B loss rows (their edges: ``deg_rows`` = the sum of
    their degrees); BPR + EmbLoss with a dense zero-filled gradient table; the backward's first layer
    as the sparse-upstream launch (all col/val scanned, X gathered at the hits, H written in full);
    its second layer over the full graph (+ the G addend); Adam over every parameter."""
    b_full = 8 * (N + 1) + nnz * 8 + nnz * d * s + N * d * s
    l1_rows, l1_edges = layer1 if layer1 is not None else (N, nnz)
    b_l1 = 8 * (l1_rows + 1) + l1_edges * 8 + l1_edges * d * s + l1_rows * d * s
    rows = 3 * B
    fwd = b_l1 + 16 * rows + deg_rows * (8 + d * s) + rows * d * s * 3
    loss = B * (3 * 8 + 3 * d * s) * 2 + N * d * s  # + the dense gradient table's zero fill
    bwd = (8 * (N + 1) + 8 * nnz + deg_rows * d * s + N * d * s + rows * d * s) + (b_full + N * d * s)
    return fwd + loss + bwd + adam * P


MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md; no sparsity)
MFMA_F32_PEAK_TFLOPS = 157.3


def config5(device, batches=(512, 8192), steps=3, warmup=2, spmm_iters=5, topk_users=32768, k=20):
    """BASELINE config 5: the config-4 graph at d=256 with bf16 tables.  (1) fr_spmm_csr_bf16 alone
    (HBM-bound gather, s=2), (2) the LightGCN-ID training step with bf16 tables (fp32 master + moments
    in Adam), SURVEY 8(d) byte model with s=2 and 30 B/param Adam, (3) the fused full-sort top-k
    (fr_topk_scores: MFMA user x item GEMM + running top-k, training items masked) for
    ``topk_users`` users against all 1M items, as TFLOP/s of the dense score GEMM vs the bf16 peak."""
    import torch
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import ops
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.interaction_graph import InteractionGraph
    U, I, d = 10_000_000, 1_000_000, 256
    t0 = time.perf_counter()
    g = InteractionGraph(U, I, 20.0, seed=0, device=device)
    build_s = time.perf_counter() - t0
    adj = g.adj
    N = U + I
    X = torch.randn(N, d, device=device).to(torch.bfloat16)
    Y = torch.empty_like(X)
    ops.spmm_launch(adj, X, Y1=Y)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(spmm_iters):
        ops.spmm_launch(adj, X, Y1=Y)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / spmm_iters
    b = ops.spmm_bytes(adj, d, 1, 2)
    spmm = {"avg_launch_ms": round(ms, 3), "bytes_per_launch": b, "achieved_gbps": round(b / ms / 1e6, 1),
            "peak": HBM_PEAK_GBPS, "frac": round(b / ms / 1e6 / HBM_PEAK_GBPS, 4), "chunk": adj.chunk}
    del X, Y
    torch.cuda.empty_cache()
    cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                 "ckp_root": "/tmp/frckp/", "embedding_size": d,
                                                 "embedding_dtype": "bf16"})
    cfg["device"] = device
    torch.manual_seed(999)
    model = LightGCN_ID(cfg, g)
    trainer = Trainer(cfg, model)
    P = sum(p.numel() for p in model.parameters())
    steps_out = {}
    for B in batches:
        state = trainer.new_step_state()

        def step(i):
            u, p, n = g.triples(B)
            trainer.train_step({"u_id": u, "pos_i_id": p, "neg_i_id": n}, i, state)

        for i in range(warmup):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(warmup + i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        assert not int(state["nan"].item()), "NaN loss in the config-5 step"
        bstep, _ = config4_bytes_per_step(N, adj.nnz, P, B, d=d, s=2, adam=30)
        steps_out[str(B)] = {"ms_per_step": round(dt * 1e3, 3), "triples_per_s": round(B / dt, 1),
                             "bytes_per_step": bstep, "achieved_gbps": round(bstep / dt / 1e9, 1),
                             "roofline_frac": round(bstep / dt / 1e9 / HBM_PEAK_GBPS, 4),
                             "roofline_triples_per_s": round(B / (bstep / (HBM_PEAK_GBPS * 1e9)), 1)}
    trainer.optimizer.state.clear()
    del trainer
    torch.cuda.empty_cache()
    # full-sort top-k over all items for a batch of users (propagated tables computed once)
    with torch.no_grad():
        tables = model.forward()
        gen = torch.Generator(device=device).manual_seed(7)
        users = torch.randint(0, U, (topk_users,), device=device, generator=gen)
        model.full_sort_topk(users, k, tables=tables)
        torch.cuda.synchronize()
        reps = 3
        ev0.record()
        for _ in range(reps):
            s_, i_, _h = model.full_sort_topk(users, k, tables=tables)
        ev1.record()
        torch.cuda.synchronize()
    tk_ms = ev0.elapsed_time(ev1) / reps
    flops = ops.topk_flops(topk_users, I, d)
    topk = {"users": topk_users, "items": I, "k": k, "mask": "training items", "avg_call_ms": round(tk_ms, 3),
            "flops_per_call": flops, "achieved_tflops": round(flops / tk_ms / 1e9, 1),
            "peak_tflops": MFMA_BF16_PEAK_TFLOPS,
            "frac": round(flops / tk_ms / 1e9 / MFMA_BF16_PEAK_TFLOPS, 4),
            "users_per_s": round(topk_users / tk_ms * 1e3, 1),
            "kernel": "fr_topk_scores (v_mfma_f32_32x32x16_bf16 + fused running top-k + merge)"}
    out = {"graph": "synthetic U=10M I=1M E=%d (nnz=%d), built on device in %.1f s" % (g.n_edges, adj.nnz, build_s),
           "model": "LightGCN_ID (L=2, d=256, bf16 tables, fp32 master/moments Adam, BPR + EmbLoss)",
           "params": P, "steps_timed": steps, "spmm_bf16": spmm, "step": steps_out, "full_sort_topk": topk,
           "byte_model": "SURVEY 8(d) with s=2: 2L*B_spmm + 2(L+1)*N*d*2 + 30*P + B*(3*8+3*d*2)*2"}
    del model, g, adj, tables
    torch.cuda.empty_cache()
    return out


def graph_region_pass(trainer, B, sampler, device, reps):
    """Per-region durations INSIDE a graph replay: a one-step graph of the same training step (unroll
    1, batches copied into its inputs) captured while profiling.StampTimer brackets every region with
    device wall-clock stamps, then replayed ``reps`` times; {region: avg_ms, launches_per_step, ...}."""
    from collections import defaultdict
    from FoodRec.engine import profiling
    g2 = trainer.graphed_step(B, warmup=3, unroll=1)
    st2 = g2.state

    def batches():
        while True:
            for t in sampler.epoch(out=g2.inputs):
                yield t

    it2 = batches()
    with profiling.stamping(device) as stamps:
        n0 = g2.prepare(lambda: next(it2), st2)
    per = defaultdict(list)
    for r in range(reps):
        g2(*next(it2), n0 + r, st2)
        step = defaultdict(list)
        for name, us, _ in stamps.read():
            step[name].append(us)
        for name, v in step.items():
            per[name].append(v)
    out = {}
    for name, steps in per.items():
        flat = [x for v in steps for x in v]
        out[name] = {"avg_ms": round(sum(flat) / len(flat) / 1e3, 4), "launches_per_step": len(steps[0]),
                     "median_ms": round(sorted(flat)[len(flat) // 2] / 1e3, 4), "replays": len(steps)}
    del g2, st2, it2
    return out


def config3(device, steps=30, warmup=5, ssl_iters=20, cpu=True, cpu_steps=5):
    """BASELINE config 3 on one GPU: CLUSSL (reference PRICAI_ModelX) on a Foodcom-shaped synthetic
    dataset (U=7,596, I=29,943, ~192k train pairs, 2,000 image / text k-means clusters, NI=4,963),
    d=64, B=512: the full graphed training step (3 item-side propagations with n_ri_layers=2, the
    UI propagation, BPR + EmbLoss, the SSL term, backward, Adam) with the reference's distance-
    correlation SSL (:263) and with the InfoNCE variant (CL_loss, :354-378), plus the fused SSL
    kernels alone (forward + backward over the three [2B, 64] views)."""
    import numpy as np
    import torch
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import ops
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.models.clussl import _DCOR_PAIRS
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.synthetic import make_synthetic
    from FoodRec.utils.utils import get_model, init_seed
    B = 512
    data = FoodData.from_synthetic(make_synthetic("foodcom", 0, negatives=False))
    out = {"dataset": "Foodcom-shape synthetic (U=%d, I=%d, train=%d, clusters=2000)"
                      % (data.n_users, data.n_items, int(data.train_coo_matrix.nnz)),
           "model": "CLUSSL (PRICAI_ModelX), n_ri_layers=2, n_ui_layers=1, d=64", "batch": B, "steps_timed": steps}
    for mode in ("dcor", "infonce"):
        cfg = Config("PRICAI_ModelX", "Foodcom", {"use_gpu": True, "seed": 999, "cuda_graph": True,
                                                  "train_batch_size": B, "ssl_mode": mode, "n_cluster": 2000,
                                                  "log_root": "/tmp/frlog/", "ckp_root": "/tmp/frckp/"})
        cfg["device"] = device
        init_seed(999)
        model = get_model("PRICAI_ModelX")(cfg, data).to(device)
        tr = Trainer(cfg, model)
        np.random.seed(2000)
        sampler = TripleSampler(data, B, device, replay_python_random=False)
        g = tr.graphed_step(B, warmup=3)
        feed = g.attach_feed(sampler)
        state = g.state
        model.train()

        def batches():
            while True:
                for t in sampler.epoch(out=g.inputs, feed=feed):
                    yield t

        it = batches()
        prep = g.prepare(lambda: next(it), state)  # every graph captured and replayed before t0
        for i in range(warmup):
            g(*next(it), prep + i, state)
        g.flush()
        captures0 = g.captures
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            g(*next(it), prep + warmup + i, state)
        g.flush()
        tr.flush_optimizer()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        assert g.captures == captures0, "graph capture inside the config-3 timed region"
        assert not int(state["nan"].item()), "NaN loss in the config-3 step"
        out[mode] = {"ms_per_step": round(dt * 1e3, 4), "triples_per_s": round(B / dt, 1),
                     "graph_captures_in_timed_region": g.captures - captures0, "prepare_steps": prep}
        del tr, model, g, sampler, state, it
        torch.cuda.empty_cache()
    torch.manual_seed(0)
    views = [torch.randn(2 * B, 64, device=device, requires_grad=True) for _ in range(3)]
    for name, fn in (("dcor_fwd_bwd_ms", lambda: ops.dcor_loss(views, _DCOR_PAIRS).backward()),
                     ("infonce_fwd_bwd_ms", lambda: ops.infonce_pairs(views, _DCOR_PAIRS, 0.5).backward())):
        # eager (host-issued: Python + autograd per call) and the same call captured in a HIP graph
        # and replayed (the kernels' GPU time, as the graphed training step runs them)
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ssl_iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name.replace("_ms", "_eager_ms")] = round(e0.elapsed_time(e1) / ssl_iters, 4)
        for v in views:
            v.grad = None  # (the capture adopts fresh .grad buffers: replays overwrite, no accumulate kernel)
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            fn()
            for v in views:
                v.grad = None
        torch.cuda.current_stream(device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fn()
        graph.replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(ssl_iters):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) / ssl_iters, 4)
        del graph
        for v in views:
            v.grad = None
    # MFMA roofline of the SSL kernels (fp32 v_mfma_f32_16x16x4_f32 Gram tiles): algorithmic FLOPs of
    # one forward + backward over the three [2B, 64] views / the graph-replay GPU time
    n_views, n_pairs = len(views), len(_DCOR_PAIRS)
    for key, fl, name, kern in (
            ("roofline", ops.infonce_flops(2 * B, 64, n_pairs), "infonce_fwd_bwd_ms",
             "nce_lse_mfma + nce_bwd_mfma (+ their finalize launches): fr_infonce_multi_fwd_ex / _bwd"),
            ("roofline_dcor", ops.dcor_flops(2 * B, 64, n_views), "dcor_fwd_bwd_ms",
             "dcor tiles + means + finalize, dcor backward + finalize: fr_dcor_fwd_ex / fr_dcor_bwd_ex")):
        tf = fl / (out[name] * 1e-3) / 1e12
        out[key] = {"kernel": kern, "bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_F32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tf / MFMA_F32_PEAK_TFLOPS, 4), "traffic": None,
                    "flops_per_call": fl, "avg_call_ms": out[name],
                    "timing_source": f"HIP events around {ssl_iters} replays of one captured fwd+bwd call "
                                     f"(config3_clussl_foodcom.{name})",
                    "flop_model": ("per pair: the (2n)^2 logit Gram forward + dH = S H, S^T H backward, "
                                   "2 (2n)^2 d each, n = 2B = 1024 rows per view, d = 64"
                                   if key == "roofline" else
                                   "per view: the n^2 distance Gram forward + the m X product backward, "
                                   "2 n^2 d each, n = 2B = 1024, d = 64")}
    if cpu:
        out["cpu_baseline"] = config3_cpu(data, B, cpu_steps)
    return out


def _cpu_threads():
    """The CPU threads a baseline uses: the box's per-GPU share (OMP_NUM_THREADS=16 there), at most 16."""
    return min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1, 16)


def config3_cpu(data, B, steps):
    """The config-3 step (CLUSSL, dCor SSL) of the torch-CPU oracle on this host's CPU share:
    the engine model on oracle/cpu_backend (the reference's formulas in torch-CPU ops)."""
    import numpy as np
    import torch
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.utils import get_model, init_seed
    from oracle import cpu_backend
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    with cpu_backend.installed():
        cfg = Config("PRICAI_ModelX", "Foodcom", {"use_gpu": False, "seed": 999, "train_batch_size": B,
                                                  "ssl_mode": "dcor", "n_cluster": 2000, "log_root": "/tmp/frlog/",
                                                  "ckp_root": "/tmp/frckp/"})
        cfg["device"] = torch.device("cpu")
        init_seed(999)
        model = get_model("PRICAI_ModelX")(cfg, data)
        tr = Trainer(cfg, model)
        np.random.seed(2001)
        sampler = TripleSampler(data, B, "cpu", replay_python_random=False)
        feats = tr._features()
        st = tr.new_step_state()
        it = sampler.epoch()
        u, p, n = next(it)
        tr.train_step(feats.batch(u, p, n), 0, st)  # warm-up
        c0 = time.perf_counter()
        for i in range(steps):
            u, p, n = next(it)
            tr.train_step(feats.batch(u, p, n), 1 + i, st)
        dt = (time.perf_counter() - c0) / steps
    return {"value": round(B / dt, 1), "unit": "triples/s", "cores": threads, "kind": "port",
            "host_cores_total": os.cpu_count(), "ms_per_step": round(dt * 1e3, 1),
            "sample": f"{steps} CLUSSL dCor training steps (B={B}) of the torch-CPU oracle after 1 warm-up"}


def config4_cpu(adj, n_users, P, batches, threads=None, sample_nnz=16_000_000):
    """The reference's compute path for the config-4 step (lightgcn.py:134-177 with common/loss.py and
    torch.optim.Adam) on this host's CPU share, as a bounded sample.  The reference multiplies by the
    normalised adjacency as a coalesced COO tensor (torch.sparse.mm), ~0.3 us per non-zero on the
    CPU here: one full product over the 400M non-zeros would take minutes.  So every s-th row of A
    (s = nnz / sample_nnz: ~16M non-zeros, users and Zipf-heavy items alike) is multiplied with the
    full [N, 64] table and the time is scaled by nnz / sampled non-zeros (the COO product is a loop
    over the non-zeros).  The step is composed as 2L = 4 such products (forward; backward = the same
    product, A symmetric) + Adam over the P parameters (a P/16 slice timed, scaled) + BPR / EmbLoss on
    the B rows (timed).  Returns None when the host lacks the memory."""
    import torch
    threads = threads or _cpu_threads()
    torch.set_num_threads(threads)
    N, nnz = adj.shape[0], adj.nnz
    try:
        import psutil
        if psutil.virtual_memory().available < 4 * N * 64 * 4 + 40 * sample_nnz:
            return None
    except ImportError:
        pass
    rp = adj.rowptr
    stride = max(1, -(-nnz // sample_nnz))
    sel = torch.arange(0, N, stride, device=rp.device)
    lens = rp[sel + 1] - rp[sel]
    tot = int(lens.sum().item())
    first = torch.cumsum(lens, 0) - lens
    pos = torch.repeat_interleave(rp[sel] - first, lens) + torch.arange(tot, device=rp.device)
    rows = torch.repeat_interleave(torch.arange(sel.numel(), device=rp.device), lens)
    idx = torch.stack([rows, adj.col[pos].to(torch.int64)]).cpu()
    vals = adj.val[pos].cpu()
    n_sel = int(sel.numel())
    del pos, rows, lens, first, sel
    A = torch.sparse_coo_tensor(idx, vals, (n_sel, N), is_coalesced=True)
    del idx, vals
    gen = torch.Generator().manual_seed(0)
    X = torch.randn(N, 64, generator=gen)
    t0 = time.perf_counter()
    Y = torch.sparse.mm(A, X)
    t_sample = time.perf_counter() - t0
    t_spmm = t_sample * nnz / max(tot, 1)
    del Y, A, X
    # Adam on a slice of the parameters, scaled to P (the update is elementwise: linear in P)
    m = max(1, P // 16)
    w = torch.nn.Parameter(torch.randn(m, generator=gen))
    w.grad = torch.randn(m, generator=gen)
    opt = torch.optim.Adam([w], lr=1e-3)
    opt.step()
    t0 = time.perf_counter()
    opt.step()
    t_adam = (time.perf_counter() - t0) * (P / m)
    del w, opt
    out = {"spmm_s": round(t_spmm, 3), "adam_s": round(t_adam, 3), "cores": threads, "host_cores_total": os.cpu_count(),
           "kind": "port", "step": {}}
    E = torch.randn(n_users + 64, 64, generator=gen)
    for B in batches:
        ue, pe, ne = (E[torch.randint(0, E.shape[0], (B,), generator=gen)].requires_grad_(True) for _ in range(3))
        t0 = time.perf_counter()
        pos_s, neg_s = (ue * pe).sum(1), (ue * ne).sum(1)
        mf = -torch.log(1e-10 + torch.sigmoid(pos_s - neg_s)).mean()
        reg = (ue.norm(2).pow(2) + pe.norm(2).pow(2) + ne.norm(2).pow(2)) / B
        (mf + 1e-4 * reg).backward()
        t_loss = time.perf_counter() - t0
        step_s = 4 * t_spmm + t_adam + t_loss
        out["step"][str(B)] = {"value": round(B / step_s, 2), "unit": "triples/s", "ms_per_step": round(step_s * 1e3, 1)}
    out["sample"] = ("torch.sparse.mm (coalesced COO, as the reference) over every %d-th row of A: %d of %d non-zeros "
                     "x [%d, 64], %.2f s, scaled by non-zeros; x 4 (2 layers forward + backward) + torch.optim.Adam "
                     "over %d params (a 1/16 slice timed, scaled) + BPRLoss / EmbLoss on B rows"
                     % (stride, tot, nnz, N, t_sample, P))
    return out


def config4(device, batches=(512, 8192), steps=5, warmup=2, spmm_iters=10, cpu=True):
    """BASELINE config 4 on one GPU: the synthetic 10M users x 1M items x ~200M interactions graph.
    (1) fr_spmm_csr alone (the propagation kernel in its HBM-bound regime; the Allrecipes tables fit
    the Infinity Cache), (2) the full LightGCN-ID training step (device triple sampling, 2-layer
    propagation + layer mean, fused BPR + EmbLoss, backward, fused Adam over (U+I) x 64) timed over
    ``steps`` steps per batch size, roofline from SURVEY 8(d)'s per-step byte model."""
    import torch
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import ops
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.interaction_graph import InteractionGraph
    U, I, d = 10_000_000, 1_000_000, 64
    t0 = time.perf_counter()
    g = InteractionGraph(U, I, 20.0, seed=0, device=device)
    build_s = time.perf_counter() - t0
    adj = g.adj
    N = U + I
    X = torch.randn(N, d, device=device)
    Y = torch.empty_like(X)
    ops.spmm_launch(adj, X, Y1=Y)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(spmm_iters):
        ops.spmm_launch(adj, X, Y1=Y)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / spmm_iters
    b = ops.spmm_bytes(adj, d, 1)
    spmm = {"avg_launch_ms": round(ms, 3), "bytes_per_launch": b, "achieved_gbps": round(b / ms / 1e6, 1),
            "peak": HBM_PEAK_GBPS, "frac": round(b / ms / 1e6 / HBM_PEAK_GBPS, 4), "chunk": adj.chunk,
            **spmm_traffic("config4", ms)}
    del X, Y
    torch.cuda.empty_cache()
    cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                 "ckp_root": "/tmp/frckp/"})
    cfg["device"] = device
    torch.manual_seed(999)
    model = LightGCN_ID(cfg, g)
    trainer = Trainer(cfg, model)
    P = sum(p.numel() for p in model.parameters())
    steps_out = {}
    for B in batches:
        state = trainer.new_step_state()

        def step(i):
            u, p, n = g.triples(B)
            trainer.train_step({"u_id": u, "pos_i_id": p, "neg_i_id": n}, i, state)

        for i in range(warmup):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(warmup + i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        assert not int(state["nan"].item()), "NaN loss in the config-4 step"
        # the loss rows' degree sum, averaged over 8 sampled batches (same sampler)
        deg = adj.rowptr[1:] - adj.rowptr[:-1]
        dsum = l1r = l1e = 0
        for _ in range(8):
            u, p, n = g.triples(B)
            dsum += int(torch.cat([deg[u], deg[p + U], deg[n + U]]).sum().item())
            S = ops._bipartite_layer1_rows(adj, [(u, 0), (p, U), (n, U)], U)  # layer 1's item rows
            l1r += int(S.numel())
            l1e += int(deg[S].sum().item())
        del deg
        deg_rows = dsum // 8
        layer1 = (U + l1r // 8, adj.nnz_below_split + l1e // 8)
        bstep = config4_bytes_rows(N, adj.nnz, P, B, deg_rows, layer1)
        dense_eq, _ = config4_bytes_per_step(N, adj.nnz, P, B)
        steps_out[str(B)] = {"ms_per_step": round(dt * 1e3, 3), "triples_per_s": round(B / dt, 1),
                             "bytes_per_step": bstep, "loss_rows_degree_sum": deg_rows,
                             "layer1_rows_edges": list(layer1),
                             "achieved_gbps": round(bstep / dt / 1e9, 1),
                             "roofline_frac": round(bstep / dt / 1e9 / HBM_PEAK_GBPS, 4),
                             "roofline_triples_per_s": round(B / (bstep / (HBM_PEAK_GBPS * 1e9)), 1),
                             "survey_8d_dense_bytes": dense_eq,
                             "survey_8d_dense_roofline_triples_per_s":
                                 round(B / (dense_eq / (HBM_PEAK_GBPS * 1e9)), 1)}
    out = {"graph": "synthetic U=10M I=1M E=%d (nnz=%d, N=%d), built on device in %.1f s"
                    % (g.n_edges, adj.nnz, N, build_s),
           "model": "LightGCN_ID (L=2, d=64, fp32, BPR + EmbLoss, Adam)", "params": P, "steps_timed": steps,
           "spmm": spmm, "step": steps_out,
           "byte_model": "config4_bytes_rows: full layer 1 + layer 2 at the 3B loss rows (their edges) + "
                         "BPR/EmbLoss with a dense zero-filled gradient + sparse-upstream backward layer (col/val "
                         "scan, hits, H write) + full backward layer + 28*P Adam; survey_8d_dense_bytes = SURVEY "
                         "8(d)'s 2L*B_spmm + 2(L+1)*N*d*s + 28*P + B*(3*8+3*d*s)*2 (every layer over the full graph)"}
    if cpu:
        out["cpu_baseline"] = config4_cpu(adj, U, P, batches)
    del trainer, model, g, adj
    torch.cuda.empty_cache()
    bm = out["spmm_dram_uniform"] = spmm_dram_uniform(device)
    # the DRAM figure comes from a graph whose gathers miss the Infinity Cache: on config 4's 1M-item
    # graph the 256 MB item block is MALL-sized, and even the PMC beyond-L2 bytes (FETCH_SIZE counts
    # MALL hits, MI355X_MICROARCH.md) are partly cache hits -- so this graph's rate is reported as
    # cache-assisted / beyond-L2, never as DRAM.  spmm_dram_uniform: 10M users x 16M uniformly popular
    # items (4 GB item block, no hot rows): min(model, PMC) bytes / launch time is a DRAM rate.
    sp = out["spmm"]
    dram_bytes = min(bm["bytes_per_launch"], bm.get("traffic") or bm["bytes_per_launch"])
    dram_gbps = dram_bytes / bm["avg_launch_ms"] / 1e6
    sp.update({"achieved_gbps_cache_assisted": sp["achieved_gbps"], "frac_cache_assisted": sp["frac"],
               "achieved_gbps_dram": round(dram_gbps, 1), "frac_dram": round(dram_gbps / HBM_PEAK_GBPS, 4),
               "frac": round(dram_gbps / HBM_PEAK_GBPS, 4),
               "frac_note": "frac = frac_dram: the same kernel on a 10M x 16M uniform-popularity graph "
                            "(spmm_dram_uniform: 4 GB item block, every gather beyond the Infinity Cache), "
                            "min(model, PMC) bytes / launch time; *_cache_assisted: this graph's no-reuse byte "
                            "model, whose Zipf-hot item rows the Infinity Cache holds; frac_beyond_l2: PMC bytes "
                            "that left the L2 (DRAM + Infinity-Cache hits) -- neither is a DRAM rate"})
    if sp["frac_dram"] * HBM_PEAK_GBPS > 6300:
        sp["frac_note"] += "; WARNING: frac_dram above the guide's 6.29 TB/s streaming ceiling"
    return out


def spmm_traffic(key, ms):
    """PMC bytes per launch of the config-4 SpMM (``key``: config4 | dram_uniform) from the newest
    profiles/r*/pmc_spmm10m.json (tools/pmc_spmm10m.py: FETCH_SIZE x 2 + WRITE_SIZE, bytes that left
    the L2 -- DRAM plus Infinity Cache hits) and the rate they imply at this run's launch time
    (``frac_beyond_l2``: that rate / the 8 TB/s peak -- DRAM plus Infinity-Cache hits)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_spmm10m.json")))
    if not files:
        return {"traffic": None}
    with open(files[-1]) as f:
        d = json.load(f).get(key)
    if not d:
        return {"traffic": None}
    t = int(d["bytes_per_launch"])
    return {"traffic": t, "traffic_gbps": round(t / ms / 1e6, 1),
            "frac_beyond_l2": round(t / ms / 1e6 / HBM_PEAK_GBPS, 4), "traffic_source": os.path.relpath(files[-1], ROOT)}


def spmm_dram_uniform(device, iters=5):
    """The config-4 SpMM with every gather beyond the 256 MB Infinity Cache: 10M users x 16M
    uniformly popular items (uniform_bipartite: config 4's user degrees, ~200M interactions; the item
    block of X is 4 GB, the user block 2.56 GB, no hot rows), d=64 fp32 -- the byte model then counts
    DRAM traffic (checked against the PMC beyond-L2 bytes of tools/spmm10m.py --uniform)."""
    import torch
    from FoodRec.engine import ops
    from FoodRec.utils.interaction_graph import InteractionGraph, uniform_bipartite
    U, I, d = 10_000_000, 16_000_000, 64
    g = InteractionGraph(U, I, 20.0, seed=1, device=device, pairs=uniform_bipartite(U, I, 20.0, 1, device))
    adj = g.adj
    X = torch.randn(U + I, d, device=device)
    Y = torch.empty_like(X)
    ops.spmm_launch(adj, X, Y1=Y)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        ops.spmm_launch(adj, X, Y1=Y)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / iters
    b = ops.spmm_bytes(adj, d, 1)
    out = {"graph": "synthetic uniform U=10M I=16M E=%d (nnz=%d)" % (g.n_edges, adj.nnz),
           "item_table_mb": I * d * 4 / 2**20, "avg_launch_ms": round(ms, 3), "bytes_per_launch": b,
           "achieved_gbps": round(b / ms / 1e6, 1), "peak": HBM_PEAK_GBPS,
           "frac": round(b / ms / 1e6 / HBM_PEAK_GBPS, 4), **spmm_traffic("dram_uniform", ms)}
    del X, Y, g, adj
    torch.cuda.empty_cache()
    return out


def config4_sharded(device, world, rank, batches=(512, 8192), steps=5, warmup=2):
    """BASELINE config 4 row-sharded over the job's ranks (engine/sharded.py): users in
    nnz-balanced blocks, items replicated, one RCCL all-reduce of the item block per propagation
    layer (forward and backward).  Every rank builds the same graph from the same seed and keeps
    its slice; every rank samples the same global batch.  Time = max over ranks."""
    import torch
    import torch.distributed as dist
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sharded import ShardedGraph, ShardedLightGCN
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.interaction_graph import synth_bipartite
    U, I, d = 10_000_000, 1_000_000, 64
    t0 = time.perf_counter()
    u, i = synth_bipartite(U, I, 20.0, seed=0, device=device)
    g = ShardedGraph(U, I, u, i, rank, world, device)
    del u, i
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                 "ckp_root": "/tmp/frckp/"})
    cfg["device"] = device
    dist_on = world > 1 or (dist.is_available() and dist.is_initialized())
    sync = (lambda: dist.barrier()) if dist_on else (lambda: None)  # noqa: E731
    model = ShardedLightGCN(g, d, 2, 0.1, group=dist.group.WORLD if dist_on else None, seed=999)
    trainer = Trainer(cfg, model)
    P_local = sum(p.numel() for p in model.parameters())
    deg_u = g.A_ui.rowptr[1:] - g.A_ui.rowptr[:-1]   # this rank's users (global degrees)
    deg_i = g.A_iu.rowptr[1:] - g.A_iu.rowptr[:-1]   # items, this rank's share of their degrees
    out_steps = {}
    for B in batches:
        state = trainer.new_step_state()

        def step(k):
            uu, pp, nn_ = g.triples(B, 999, k)
            trainer.train_step({"u_id": uu, "pos_i_id": pp, "neg_i_id": nn_}, k, state)

        for k in range(warmup):
            step(k)
        torch.cuda.synchronize()
        sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            step(warmup + k)
        torch.cuda.synchronize()
        sync()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
        if dist_on:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item()) / steps
        assert not int(state["nan"].item()), "NaN loss in the sharded config-4 step"
        # global degree sum of the loss rows (owned users' degrees + every rank's share of the items')
        from FoodRec.engine.sharded import _neighbour_items
        ds = torch.zeros(3, dtype=torch.float64, device=device)  # loss rows' degrees, |S|, S's degrees
        for k in range(4):
            uu, pp, nn_ = g.triples(B, 999, 1000 + k)
            own, loc = g.owner_index(uu)
            flags = torch.zeros(I, dtype=torch.float32, device=device)
            flags[_neighbour_items(g, loc)] = 1.0
            flags[torch.cat([pp, nn_])] = 1.0
            if dist_on:
                dist.all_reduce(flags)
            S = torch.nonzero(flags > 0).reshape(-1)
            ds[0] += (deg_u[loc[own]].sum() + deg_i[pp].sum() + deg_i[nn_].sum()).double()
            ds[1] += float(S.numel()) / (world if dist_on else 1)
            ds[2] += deg_i[S].sum().double()
        if dist_on:
            dist.all_reduce(ds)
        deg_rows = int(ds[0].item() / 4)
        layer1 = (U + int(ds[1].item() / 4), g.n_edges + int(ds[2].item() / 4))
        # the single-GPU byte model of the whole step (work is divided, not changed, by sharding)
        bstep = config4_bytes_rows(U + I, 2 * g.n_edges, (U + I) * d, B, deg_rows, layer1)
        out_steps[str(B)] = {"ms_per_step": round(dt * 1e3, 3), "triples_per_s": round(B / dt, 1),
                             "bytes_per_step_global": bstep, "loss_rows_degree_sum": deg_rows,
                             "achieved_gbps_per_gpu": round(bstep / dt / 1e9 / world, 1),
                             "roofline_frac_per_gpu": round(bstep / dt / 1e9 / world / HBM_PEAK_GBPS, 4)}
    nnz = torch.tensor([g.local_nnz], device=device, dtype=torch.float64)
    if dist_on:
        nnz_all = [torch.zeros_like(nnz) for _ in range(world)]
        dist.all_gather(nnz_all, nnz)
    else:
        nnz_all = [nnz]
    out = {"graph": "synthetic U=10M I=1M E=%d, row-sharded over %d ranks (built in %.1f s)"
                    % (g.n_edges, world, build_s),
           "model": "LightGCN_ID row-sharded (users in nnz-balanced blocks, items replicated), rows form",
           "collectives_per_step": "1 all-reduce of I x d fp32 (256 MB: the last backward layer's item partial, "
                                   "cut into item-row blocks) + the item flags (I floats) + 2 of the |S| layer-1 "
                                   "item rows + 1 of the 2B batch item rows + 1 owner gather of the batch users' propagated and ego rows (2B x d)",
           "byte_model": "config4_bytes_rows (the single-GPU step's algorithmic bytes)",
           "local_params_rank0": P_local, "local_nnz_per_rank": [int(x.item()) for x in nnz_all],
           "steps_timed": steps, "step": out_steps}
    del trainer, model, g
    torch.cuda.empty_cache()
    return out


def cpu_baseline(args):
    """Time the oracle's CPU restatement of the same step on this host, as BASELINE.md section 3 states
    it: every host core (torch.set_num_threads(os.cpu_count())), ``--cpu-baseline-steps`` (20) timed
    steps after 3 warm-ups.  The per-GPU share of the host (the GPU box gives one GPU's job 16 CPUs,
    OMP_NUM_THREADS=16) is timed beside it on a shorter sample (``per_gpu_share``)."""
    import torch
    from oracle import cpu_backend
    all_cores = os.cpu_count() or 1
    share = _cpu_threads()
    with cpu_backend.installed():
        from FoodRec.common.trainer import Trainer
        from FoodRec.engine.sampler import TripleSampler
        cfg, data, model = build(torch.device("cpu"), args.batch)
        trainer = Trainer(cfg, model)
        sampler = TripleSampler(data, args.batch, "cpu", replay_python_random=False)
        feats = trainer._features()
        state = trainer.new_step_state()
        it = sampler.epoch()
        step = [0]

        def run(threads, warm, k):
            torch.set_num_threads(threads)
            for _ in range(warm):
                u, p, n = next(it)
                trainer.train_step(feats.batch(u, p, n), step[0], state)
                step[0] += 1
            t0 = time.perf_counter()
            for _ in range(k):
                u, p, n = next(it)
                trainer.train_step(feats.batch(u, p, n), step[0], state)
                step[0] += 1
            return time.perf_counter() - t0

        k = max(1, args.cpu_baseline_steps)
        dt = run(all_cores, 3, k)
        ks = 4
        dts = run(share, 1, ks)
    torch.set_num_threads(share)
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    quota = None
    try:  # the cgroup's CPU quota (cpu.max "QUOTA PERIOD"): what the threads can actually run on
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"value": round(args.batch * k / dt, 2), "unit": "triples/s", "cores": all_cores, "kind": "port",
            "host_cores_total": all_cores, "cores_in_affinity": affinity, "cgroup_cpu_quota": quota,
            "sample": f"{k} HealthRec training steps (B={args.batch}) of the torch-CPU oracle after 3 warm-ups, "
                      f"torch.set_num_threads({all_cores})",
            "ms_per_step": round(dt / k * 1e3, 1),
            "note": "BASELINE.md section 3: every host core; where the cgroup quota is below the core count the "
                    "threads oversubscribe it and per_gpu_share (threads = the quota) is the faster CPU figure",
            "per_gpu_share": {"value": round(args.batch * ks / dts, 2), "cores": share,
                              "ms_per_step": round(dts / ks * 1e3, 1),
                              "sample": f"{ks} steps after 1 warm-up, torch.set_num_threads({share})"}}


def config1(device, steps=50, warmup=5, cpu=True, cpu_steps=20):
    """BASELINE config 1: BPRMF (ID embeddings, no graph: the reference-style plugin of
    oracle/ref_plugins) on the Allrecipes-shape synthetic data, d=64, B=1024 (overall.yaml's batch:
    the reference ships no BPRMF.yaml), graphed training step on the GPU; beside it the torch-CPU
    oracle of the same step on this host's CPU share (the reference's CPU trainer path)."""
    import numpy as np
    import torch
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.synthetic import make_synthetic
    from FoodRec.utils.utils import get_model, init_seed
    from oracle import cpu_backend
    B = 1024
    data = FoodData.from_synthetic(make_synthetic("allrecipes", 0, negatives=False))

    def make(dev):
        cfg = Config("BPRMF", "Allrecipes", {"use_gpu": dev.type == "cuda", "seed": 999, "cuda_graph": True,
                                             "train_batch_size": B, "reg_weight": 0.1, "log_root": "/tmp/frlog/",
                                             "ckp_root": "/tmp/frckp/"})
        cfg["device"] = dev
        init_seed(999)
        return cfg, get_model("BPRMF")(cfg, data).to(dev)

    cfg, model = make(device)
    tr = Trainer(cfg, model)
    np.random.seed(3000)
    sampler = TripleSampler(data, B, device, replay_python_random=False)
    g = tr.graphed_step(B, warmup=3)
    feed = g.attach_feed(sampler)
    state = g.state
    model.train()

    def batches():
        while True:
            for t in sampler.epoch(out=g.inputs, feed=feed):
                yield t

    it = batches()
    prep = g.prepare(lambda: next(it), state)  # every graph captured and replayed before t0
    for i in range(warmup):
        g(*next(it), prep + i, state)
    g.flush()
    captures0 = g.captures
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        g(*next(it), prep + warmup + i, state)
    g.flush()
    tr.flush_optimizer()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    assert g.captures == captures0, "graph capture inside the config-1 timed region"
    assert not int(state["nan"].item()), "NaN loss in the config-1 step"
    out = {"model": "BPRMF (ID-only, no graph), d=64, B=1024", "dataset": "Allrecipes-shape synthetic",
           "steps_timed": steps, "ms_per_step": round(dt * 1e3, 4), "triples_per_s": round(B / dt, 1)}
    del tr, model, g, sampler, state, it
    torch.cuda.empty_cache()
    if cpu:
        threads = min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1, 16)
        torch.set_num_threads(threads)
        with cpu_backend.installed():
            ccfg, cmodel = make(torch.device("cpu"))
            ctr = Trainer(ccfg, cmodel)
            cs = TripleSampler(data, B, "cpu", replay_python_random=False)
            feats = ctr._features()
            st = ctr.new_step_state()
            cit = cs.epoch()
            u, p, n = next(cit)
            ctr.train_step(feats.batch(u, p, n), 0, st)
            c0 = time.perf_counter()
            for i in range(cpu_steps):
                u, p, n = next(cit)
                ctr.train_step(feats.batch(u, p, n), 1 + i, st)
            cdt = (time.perf_counter() - c0) / cpu_steps
        out["cpu_baseline"] = {"value": round(B / cdt, 1), "unit": "triples/s", "cores": threads, "kind": "port",
                               "sample": f"{cpu_steps} BPRMF steps (B={B}) of the torch-CPU oracle after 1 warm-up",
                               "ms_per_step": round(cdt * 1e3, 2)}
    return out


def _fast_negatives(rng, user_ids, train_keys, I, neg=500, over=640):
    """Bench-only evaluation candidates: ``neg`` distinct uniform item draws per user excluding its
    train items (the synthetic generator's popularity^0.7 lists take ~1 min at Allrecipes shape; the
    ranking's cost depends on the list lengths, not on which items they hold)."""
    import numpy as np
    out = np.empty((len(user_ids), neg), np.int64)
    for c0 in range(0, len(user_ids), 8192):
        uu = np.asarray(user_ids[c0:c0 + 8192], np.int64)
        cand = np.sort(rng.integers(0, I, size=(len(uu), over)), axis=1)
        key = uu[:, None] * I + cand
        pos = np.searchsorted(train_keys, key)
        ok = train_keys[np.minimum(pos, len(train_keys) - 1)] != key
        ok[:, 1:] &= cand[:, 1:] != cand[:, :-1]
        rank = np.cumsum(ok, axis=1)
        assert np.all(rank[:, -1] >= neg), "increase `over`"
        sel = ok & (rank <= neg)
        rows = cand[sel].reshape(len(uu), neg)
        out[c0:c0 + len(uu)] = rng.permuted(rows, axis=1)
    return out


def eval_leg(device, host_users=3000, reps=3):
    """HealthRec's per-epoch evaluation at Allrecipes shape (EvalByUserDataloader + the trainer's
    _valid_by_user_epoch, reference trainer.py:231-282,49-69, dataloader.py:228-302): all 68,768 test
    users x (|test pos| + 500 negatives) scored on the device and ranked by fr_rank_metrics, beside
    the reference-style per-user numpy loop (argsort / metrics_by_user / get_auc_fast) timed on a
    sample of users and checked bit-equal to the device metrics on that sample."""
    import numpy as np
    import torch
    from FoodRec.common.trainer import Trainer, metrics_from_hits, rank_user_host
    from FoodRec.engine import ops
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.synthetic import make_synthetic
    from FoodRec.utils.utils import get_model, init_seed
    ds = make_synthetic("allrecipes", 0, negatives=False)
    I = ds.n_items
    train_keys = np.unique(ds.train[:, 0] * I + ds.train[:, 1])
    rng = np.random.default_rng(7)
    ds.test_neg = _fast_negatives(rng, np.arange(ds.n_users), train_keys, I)
    ds.valid_neg = _fast_negatives(rng, ds.valid_users, train_keys, I)
    data = FoodData.from_synthetic(ds)
    cfg = Config("CIKM_Model", "Allrecipes", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                             "ckp_root": "/tmp/frckp/"})
    cfg["device"] = device
    data.args_config = cfg
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(device)
    tr = Trainer(cfg, model)
    model.eval()
    neg_num = cfg["neg_sample_num"]
    out = {}
    fused = tr._fused_scoring()
    for name, is_test in (("test", True), ("valid", False)):
        w0 = time.perf_counter()
        tr._valid_by_user_epoch(is_test=is_test)  # first call: builds (and, fused, uploads) the lists
        torch.cuda.synchronize()
        first_s = time.perf_counter() - w0
        walls = []
        for _ in range(reps):
            t0 = time.perf_counter()
            tr._valid_by_user_epoch(is_test=is_test)
            walls.append(time.perf_counter() - t0)
        # the same call's parts
        t0 = time.perf_counter()
        if fused:
            dc = tr._device_candidates(is_test)  # (kept on the device since the first call)
            users, items, lens, npos = dc["users"], dc["items_host"], dc["lens"], dc["npos"]
        else:
            users, items, lens, npos = tr._candidates(is_test)
        t1 = time.perf_counter()
        sc = tr._score_fused(dc) if fused else tr._score(users, items, on_device=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        hits, aucc, flags = ops.rank_metrics(sc, lens, npos, 20)
        res = metrics_from_hits(hits, lens, npos, aucc, neg_num)
        t3 = time.perf_counter()
        host = sc.cpu().numpy()
        off = np.zeros(len(lens) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        nh = min(host_users, len(lens))
        h0 = time.perf_counter()
        ref = np.stack([rank_user_host(host[off[k]:off[k + 1]].copy(), int(npos[k]), neg_num) for k in range(nh)])
        h1 = time.perf_counter()
        ok = [k for k in range(nh) if not flags[k]]
        host_loop_s = (h1 - h0) / nh * len(lens)
        out[name] = {"users": int(len(lens)), "candidates": int(len(items)),
                     "wall_s": round(sorted(walls)[len(walls) // 2], 4), "first_call_s": round(first_s, 4),
                     "scoring": "fr_score_segments (cached device lists)" if fused else "inference_fast (torch)",
                     "parts_s": {"candidates": round(t1 - t0, 4), "score_device": round(t2 - t1, 4),
                                 "rank_device_and_metrics": round(t3 - t2, 4)},
                     "tie_users_routed_to_host": int(flags.sum()),
                     "reference_style_host_loop_s": round(host_loop_s, 3),
                     "host_loop_sample_users": nh,
                     "device_vs_host_loop_speedup_rank": round(host_loop_s / max(t3 - t2, 1e-9), 1),
                     "metrics_bit_equal_on_sample": bool(np.array_equal(res[ok], ref[ok]))}
    del tr, model
    torch.cuda.empty_cache()
    out["note"] = ("wall_s = Trainer._valid_by_user_epoch (median of %d): lazy-row flush + candidate lists (built "
                   "and uploaded by the first call, first_call_s, then kept on the device) + forward() + "
                   "fr_score_segments + fr_rank_metrics + float64 metrics; score_device = forward() + scoring; "
                   "the reference-style loop is timed on %d users and scaled to all users" % (reps, host_users))
    return out


def _rank_report(world, backend, device):
    """What the job runs on, from the process group: its size, backend, the distinct GPUs behind the
    ranks (PCI bus ids), and -- over RCCL -- the rank count of an engine C-ABI communicator
    (fr_comm_init) joined by every rank."""
    import torch
    import torch.distributed as dist
    props = torch.cuda.get_device_properties(device)
    ident = f"{getattr(props, 'pci_bus_id', '?')}:{getattr(props, 'pci_device_id', '?')}:{device.index}"
    allid = [None] * world
    dist.all_gather_object(allid, ident)
    rep = {"process_group_world_size": dist.get_world_size(), "backend": dist.get_backend(),
           "distinct_gpus": len(set(allid)), "rccl_comm_ranks": None}
    if backend == "nccl":
        from FoodRec.engine.comm import RcclComm
        comm = RcclComm.from_process_group()
        one = torch.ones(1, device=device)
        comm.all_reduce(one)  # every rank contributes 1: the communicator's rank count
        rep["rccl_comm_ranks"] = int(one.item())
        assert comm.world == world and rep["rccl_comm_ranks"] == world, rep
        comm.close()
    return rep


if __name__ == "__main__":
    sys.exit(main())
