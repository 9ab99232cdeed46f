"""Trainer — the reference's training engine (common/trainer.py:71-474) on the MI355X engine.

Same public surface and semantics: ``fit`` (epoch loop, LambdaLR per epoch, evaluation every
``eval_step``, early stopping, checkpoint on improvement, final test on the best checkpoint),
``_train_epoch`` (returns the per-component loss sums), ``_valid_by_user_epoch`` (sampled
candidate Recall/NDCG@{10,20} + AUC), mirror-gradient variant (``mg``), NaN stop.

What changes is the execution, not the results:
  * triples come from FoodRec.engine.sampler.TripleSampler: the reference's exact RNG stream,
    drawn natively per epoch, batches assembled on the device (no per-sample Python, no
    per-step deepcopy unless ``mg``);
  * Adam is the fused multi-tensor HIP kernel (FoodRec.engine.optim.FusedAdam);
  * no host synchronisation inside the step loop: loss components accumulate on the device
    and the NaN check is a device flag that turns the optimiser step into a no-op, read once
    per epoch (the reference reads 4 .item()s and a NaN flag every step);
  * evaluation scores every user's candidate list in one batched gather-dot on the device; the
    ranking metrics then follow the reference's numpy code per user (same argsort tie order).
Unchanged reference models (torch.sparse.mm users) are supported: their sparse adjacency
attributes are swapped for HIP-backed Adjacency objects at construction.
"""
from __future__ import annotations

import copy
import itertools
import math
import os
from logging import getLogger
from time import time

import numpy as np
import torch
import torch.optim as optim
from torch.nn.utils.clip_grad import clip_grad_norm_

from FoodRec.engine import ops
from FoodRec.engine.graph import swap_sparse_attributes
from FoodRec.engine.optim import FusedAdam
from FoodRec.engine.sampler import BatchFeatures, EvalBatch, TripleSampler
from FoodRec.utils.textio import eval_candidates
from FoodRec.utils.utils import dict2str, early_stopping


def get_auc_fast(rel_list, predictions, neg_num):
    """trainer.py:49-52."""
    neg_predictions = predictions[len(rel_list):]
    auc_value = np.sum([np.sum(neg_predictions < predictions[idx]) for idx in rel_list])
    return auc_value / (len(rel_list) * neg_num)


def metrics_by_user(doc_list, rel_list):
    """trainer.py:55-69: Recall and NDCG of a ranked list against the relevant index set."""
    rel = set(rel_list)
    dcg, hits = 0.0, 0.0
    for i, doc in enumerate(doc_list):
        if doc in rel:
            dcg += 1 / (math.log(i + 2) / math.log(2))
            hits += 1
    idcg = 0.0
    for i in range(min(len(doc_list), len(rel_list))):
        idcg += 1 / (math.log(i + 2) / math.log(2))
    return hits / len(rel_list), dcg / idcg


# 1 / log2(i + 2): the DCG discount of rank i, the same Python float expression as metrics_by_user
_DISCOUNT = [1 / (math.log(i + 2) / math.log(2)) for i in range(31)]


def rank_user_host(pr, npo, neg_num, ks=(10, 20)):
    """One user's (recall, ndcg, auc) per k by the reference's own code path (trainer.py:231-282):
    numpy's argsort order, metrics_by_user, get_auc_fast."""
    gt = range(npo)
    order = np.argsort(pr)[::-1]
    auc = get_auc_fast(gt, pr, neg_num)
    out = np.zeros((3, len(ks)))
    for j, topk in enumerate(ks):
        r, nd = metrics_by_user(order[:topk], gt)
        out[0, j], out[1, j], out[2, j] = r, nd, auc
    return out


def metrics_from_hits(hits, lens, npos, auc_cnt, neg_num, ks=(10, 20)):
    """Per-user [recall, ndcg, auc] x ks from the device ranking (fr_rank_metrics: bit t of hits[u]
    = rank t is a positive; auc_cnt[u] = the strict positive-over-negative count), evaluated with
    metrics_by_user / get_auc_fast's float64 operations in their order (DCG summed over ranks in
    increasing order, the other ranks adding 0.0), so every value equals the host loop's bit for bit."""
    U = len(lens)
    res = np.zeros((U, 3, len(ks)))
    hits = np.asarray(hits).astype(np.int64)
    lens = np.asarray(lens, np.int64)
    npos = np.asarray(npos, np.int64)
    auc = np.asarray(auc_cnt, np.int64) / (npos * int(neg_num))
    for j, k in enumerate(ks):
        dcg, hitn, idcg = np.zeros(U), np.zeros(U), np.zeros(U)
        lim = np.minimum(np.minimum(lens, k), npos)  # min(len(order[:k]), len(gt))
        for i in range(k):
            b = ((hits >> i) & 1).astype(bool)
            dcg = dcg + np.where(b, _DISCOUNT[i], 0.0)
            hitn = hitn + b
            idcg = idcg + np.where(i < lim, _DISCOUNT[i], 0.0)
        res[:, 0, j] = hitn / npos
        res[:, 1, j] = dcg / idcg
        res[:, 2, j] = auc
    return res


def book_step(parts, acc, nan_flag, accumulate=True):
    """fr_step_book over the loss parts (device float scalars): acc (+)= parts, nan |= isnan(sum),
    and the step's deferred device counters (ops.defer_increment) advanced in the same launch.
    Returns the step's loss (the fp32 sum of the parts, a fresh device scalar; no host sync)."""
    import ctypes
    from FoodRec.engine import native
    n = len(parts)
    ptrs = (ctypes.c_void_p * n)(*[x.data_ptr() for x in parts])
    ctrs = ops.take_pending_counters()
    cptr = (ctypes.c_void_p * max(1, len(ctrs)))(*[c.data_ptr() for c in ctrs])
    loss = torch.empty((), dtype=torch.float32, device=acc.device)
    native.check(native.lib().fr_step_book(ptrs, n, acc.data_ptr(), int(bool(accumulate)), nan_flag.data_ptr(),
                                           cptr, len(ctrs), loss.data_ptr(), native.stream_of(acc)), "fr_step_book")
    return loss


# Captures are thread-local: the process group's watchdog thread polls its collectives' events
# (hipEventQuery) at any time, which a global-mode capture on another thread turns into a fatal
# "operation not permitted when stream is capturing" (seen under rocprofv3 at world 1).
_CAPTURE_MODE = "thread_local"


class GraphedStep:
    """Trainer.train_step captured once in a HIP graph and replayed per batch.

    The batch's (u, pos, neg) ids are copied into static device buffers; the graph holds the
    whole step: side-feature gathers, forward (HIP SpMM chains, Transformer, heads), fused
    BPR/EmbLoss, backward, and the fused Adam update (device-side step counters and lr).  The
    first ``warmup`` calls run eagerly on a side stream (lazy workspaces, BLAS handles), the next
    call captures and replays.  Batches of another size (the epoch's last) run eagerly.

    ``unroll`` > 1 (with a device feed and the graph's own state): a second graph holds ``unroll``
    consecutive steps and is replayed once per ``unroll`` calls, so the per-replay launch gap
    (~25 us between graphs on MI355X) is paid once per ``unroll`` steps.  Calls in between only count
    the step; ``flush`` (run by the feed before it stages the next epoch, before a ragged batch, and
    by the trainer at the epoch's end) replays the one-step graph for the steps still pending.
    """

    def __init__(self, trainer, batch_size, warmup=3, unroll=1):
        self.tr = trainer
        self.B = int(batch_size)
        self.warmup = max(1, int(warmup))
        self.unroll = max(1, int(unroll))
        self.graph_n = None   # the unrolled graph (unroll steps)
        self.pending = 0      # steps called but not yet replayed (unroll > 1)
        dev = torch.device(trainer.device)
        self.u = torch.zeros(self.B, dtype=torch.int64, device=dev)
        self.p = torch.zeros_like(self.u)
        self.n = torch.zeros_like(self.u)
        self.graph = None
        self.calls = 0
        self.captures = 0     # graph captures so far (a timed region must not contain one)
        self.static_loss = None
        # the graph's own state: each replay adds the step's loss vector to gstate["acc"] and ORs
        # the NaN flag into gstate["nan"].  Callers that pass this dict (``.state``) as their epoch
        # state pay no per-step copies; any other state dict is folded in around each replay.
        self.gstate = {"acc": None, "nan": torch.zeros((), dtype=torch.int32, device=dev)}
        self.feed = None  # engine.sampler.DeviceFeed: full batches are gathered inside the graph

    def attach_feed(self, sampler):
        """Gather full batches inside the step from ``sampler``'s staged epoch (pass the returned feed
        to ``sampler.epoch(out=self.inputs, feed=...)``)."""
        if self.graph is not None or self.calls:
            raise RuntimeError("attach_feed before the first step")
        if sampler.batch_size != self.B:
            raise ValueError("sampler batch size differs from the graphed step's")
        self.feed = sampler.device_feed()
        self.feed.on_stage = self.flush  # pending steps read the epoch being replaced
        return self.feed

    def flush(self):
        """Replay the one-step graph for the steps an unrolled graph has not run yet."""
        while self.pending:
            self.pending -= 1
            self.graph.replay()
            self._note()

    def _unrolls(self, state) -> bool:
        return state is self.gstate and self.unroll > 1 and self.feed is not None

    def prepare(self, next_batch, state, first_idx=0) -> int:
        """Run the eager warm-up calls and capture every graph later calls replay -- the one-step
        graph and, when steps are unrolled, the ``unroll``-step graph -- replaying each at least
        once, then flush.  ``next_batch()`` yields the (u, pos, neg) of one call (training steps:
        the warm-up steps train).  Afterwards calls only replay (``captures`` does not move), so a
        timed region that starts here measures the steady state whatever its length.  Returns the
        number of steps taken."""
        i = first_idx
        while self.graph is None or (self._unrolls(state) and self.graph_n is None):
            self(*next_batch(), i, state)
            i += 1
        if self._unrolls(state):
            self.flush()
            self(*next_batch(), i, state)  # pending 1: the one-step graph's first replay is the flush's
            i += 1
        self.flush()
        return i - first_idx

    @property
    def state(self):
        return self.gstate

    @property
    def inputs(self):
        """The static (u, pos, neg) buffers: a sampler writing into them saves the per-step copies."""
        return self.u, self.p, self.n

    def _note(self):
        if isinstance(self.tr.optimizer, FusedAdam):
            self.tr.optimizer.note_replay()

    def _body(self, batch_idx, state, accumulate=True):
        feats = self.tr._features()
        pre = None
        ops.defer_counters(True)  # the feed cursor advances in the step's fr_step_book launch
        if self.feed is not None:
            # (u, pos, neg) and the [pos; neg] item features gathered in one launch (fr_feed_batch)
            pre = self.feed.fill(self.u, self.p, self.n, feats if not feats.ssl else None)
        return self.tr.train_step(feats.batch(self.u, self.p, self.n, pre=pre), batch_idx, state,
                                  accumulate=accumulate)

    def __call__(self, u, p, n, batch_idx, state):
        if u.numel() != self.B:
            self.flush()
            return self.tr.train_step(self.tr._features().batch(u, p, n), batch_idx, state)
        for src, dst in ((u, self.u), (p, self.p), (n, self.n)):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.calls += 1
        if self.graph is None and self.calls <= self.warmup:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                out = self._body(batch_idx, state)
            torch.cuda.current_stream().wait_stream(side)
            self.n_parts = state["acc"].numel()
            return out
        own = state is self.gstate
        if self.graph is None:
            acc0 = self.gstate["acc"] if own else None  # the warm-up steps' sums when state is ours
            self.gstate["acc"] = torch.zeros(self.n_parts, dtype=torch.float64, device=self.u.device)
            self.tr.optimizer.zero_grad()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                self.static_loss = self._body(batch_idx, self.gstate, accumulate=True)
            self.graph = g
            self.captures += 1
            if acc0 is not None:
                self.gstate["acc"].copy_(acc0)
        if self._unrolls(state):
            self.pending += 1
            if self.pending < self.unroll:
                return self.static_loss
            if self.graph_n is None:
                # the same body unroll times in one capture, sharing the one-step graph's memory pool
                # (the two graphs replay in stream order)
                gn = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gn, pool=self.graph.pool(), capture_error_mode=_CAPTURE_MODE):
                    for k in range(self.unroll):
                        self.static_loss_n = self._body(batch_idx + k, self.gstate, accumulate=True)
                self.graph_n = gn
                self.captures += 1
            self.pending = 0
            if isinstance(self.tr.optimizer, FusedAdam):
                # the replay runs ``unroll`` lazy steps before note_replay can flush: keep the
                # history ring from wrapping inside it
                self.tr.optimizer.reserve_replays(self.unroll)
            self.graph_n.replay()
            for _ in range(self.unroll):
                self._note()
            return self.static_loss_n
        if own:
            self.flush()
            self.graph.replay()
            self._note()
            return self.static_loss
        self.flush()
        self.gstate["nan"].copy_(state["nan"])
        self.gstate["acc"].zero_()
        self.graph.replay()
        self._note()
        state["nan"].copy_(self.gstate["nan"])
        if state["acc"] is None:
            state["acc"] = self.gstate["acc"].clone()
        else:
            state["acc"].add_(self.gstate["acc"])
        return self.static_loss


class GraphedDPStep(GraphedStep):
    """Data-parallel step (Trainer.grad_hook = engine.dist.GradAllReduce) as HIP graphs with the
    collectives between them, so no RCCL call is ever captured:

      graph A  zero_grad, forward, loss, backward (row-gathered tables stash their (ids, rows)),
               pack the dense gradients into the flat buffer
      eager    RowExchange all-gathers (64-wide rows), then the all-reduce of the flat buffer issued
               asynchronously
      graph B1 (row-exchanged tables + FusedAdam) the tables' mean rows and their Adam update, which
               runs while the all-reduce is in flight
      graph B2 after the all-reduce: average + unpack the dense gradients, dense Adam
      (otherwise: both collectives, then one graph B: average + unpack, the tables' mean rows,
      fused Adam)

    The first ``warmup`` calls run the same phases eagerly (side stream for the graphed parts),
    which also creates the hook's static buffers before capture."""

    def __init__(self, trainer, batch_size, warmup=3):
        super().__init__(trainer, batch_size, warmup)
        self.graph_b = None

    def _part_a(self, batch_idx, state, accumulate):
        tr = self.tr
        feats = tr._features()
        pre = None
        ops.defer_counters(True)
        if self.feed is not None:
            pre = self.feed.fill(self.u, self.p, self.n, feats if not feats.ssl else None)
        tr.optimizer.zero_grad()
        try:
            ops.book_request(state, accumulate)
            losses = tr.model.calculate_loss(feats.batch(self.u, self.p, self.n, pre=pre))
            ops.finalize_pending()
            parts = losses if isinstance(losses, tuple) else (losses,)
            fused = tr._book_fused(state, parts, accumulate) is not None
        finally:
            ops.book_taken()
            ops.drop_pending_finalizes()
            ops.defer_counters(False)
        if fused:
            torch.autograd.backward(list(parts), grad_tensors=tr._ones_like(parts))
            ops.loss_side_join()
            tr.grad_hook.pack()
            return None
        ops.loss_side_join()
        loss = sum(parts)
        vec = torch.stack([x.detach().reshape(-1)[0].double() for x in parts])
        if state.get("acc") is None:
            state["acc"] = vec.clone()
        elif accumulate:
            state["acc"].add_(vec)
        else:
            state["acc"].copy_(vec)
        state["nan"] |= torch.isnan(loss.detach().reshape(-1)[0]).to(torch.int32)
        loss.backward()
        tr.grad_hook.pack()
        return loss.detach()

    def _part_b(self, state):
        self.tr.grad_hook.unpack()
        self.tr._opt_step(state["nan"])

    def _split_b(self) -> bool:
        """Row-exchanged tables + FusedAdam: their update (graph B1) runs while the dense
        all-reduce is in flight, the dense update (graph B2) after it."""
        hook = self.tr.grad_hook
        return getattr(hook, "rows", None) is not None and isinstance(self.tr.optimizer, FusedAdam)

    def _part_b1(self, state):
        self.tr.grad_hook.unpack_rows()
        self.tr.optimizer.step(skip_flag=state["nan"], part="rows")

    def _part_b2(self, state):
        self.tr.grad_hook.unpack_dense()
        self.tr.optimizer.step(skip_flag=state["nan"], part="dense")

    def _comm_and_b(self, run_b1, run_b2, run_b):
        hook = self.tr.grad_hook
        if self._split_b():
            hook.communicate_rows()
            work = hook.communicate_dense(async_op=True)
            run_b1()
            work.wait()
            run_b2()
        else:
            hook.communicate()
            run_b()

    def __call__(self, u, p, n, batch_idx, state):
        tr = self.tr
        if u.numel() != self.B:
            return tr.train_step(tr._features().batch(u, p, n), batch_idx, state)
        for src, dst in ((u, self.u), (p, self.p), (n, self.n)):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.calls += 1
        if self.graph is None and self.calls <= self.warmup:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                out = self._part_a(batch_idx, state, True)
            torch.cuda.current_stream().wait_stream(side)

            def on_side(fn):
                def run():
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        fn(state)
                    torch.cuda.current_stream().wait_stream(side)
                return run
            self._comm_and_b(on_side(self._part_b1), on_side(self._part_b2), on_side(self._part_b))
            self.n_parts = state["acc"].numel()
            return out
        own = state is self.gstate
        if self.graph is None:
            acc0 = self.gstate["acc"] if own else None
            self.gstate["acc"] = torch.zeros(self.n_parts, dtype=torch.float64, device=self.u.device)
            tr.optimizer.zero_grad()
            ga = torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga, capture_error_mode=_CAPTURE_MODE):
                self.static_loss = self._part_a(batch_idx, self.gstate, True)
            if self._split_b():
                gb1, gb2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb1, pool=ga.pool(), capture_error_mode=_CAPTURE_MODE):
                    self._part_b1(self.gstate)
                with torch.cuda.graph(gb2, pool=ga.pool(), capture_error_mode=_CAPTURE_MODE):
                    self._part_b2(self.gstate)
                self.graph_b = (gb1, gb2)
            else:
                gb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb, pool=ga.pool(), capture_error_mode=_CAPTURE_MODE):
                    self._part_b(self.gstate)
                self.graph_b = (gb,)
            self.graph = ga
            if acc0 is not None:
                self.gstate["acc"].copy_(acc0)
        gb = self.graph_b
        replay_b = (lambda: gb[0].replay(), lambda: gb[1].replay(), None) if len(gb) == 2 else \
            (None, None, lambda: gb[0].replay())
        if own:
            self.graph.replay()
            self._comm_and_b(*replay_b)
            self._note()
            return self.static_loss
        self.flush()
        self.gstate["nan"].copy_(state["nan"])
        self.gstate["acc"].zero_()
        self.graph.replay()
        self._comm_and_b(*replay_b)
        self._note()
        state["nan"].copy_(self.gstate["nan"])
        if state["acc"] is None:
            state["acc"] = self.gstate["acc"].clone()
        else:
            state["acc"].add_(self.gstate["acc"])
        return self.static_loss


class AbstractTrainer:
    def __init__(self, config, model):
        self.config = config
        self.model = model

    def fit(self, train_data):
        raise NotImplementedError("Method [next] should be implemented.")

    def evaluate(self, eval_data):
        raise NotImplementedError("Method [next] should be implemented.")


class Trainer(AbstractTrainer):
    def __init__(self, config, model, mg=False):
        super().__init__(config, model)
        self.logger = getLogger()
        self.learner = config["learner"]
        self.learning_rate = config["learning_rate"]
        self.epochs = config["epochs"]
        self.eval_step = min(config["eval_step"], self.epochs)
        self.test_step = min(config["test_step"] or self.epochs, self.epochs)
        self.stopping_step = config["stopping_step"]
        self.clip_grad_norm = config["clip_grad_norm"]
        self.valid_metric = (config["valid_metric"] or "NDCG@20").lower()
        self.valid_metric_bigger = config["valid_metric_bigger"]
        self.test_batch_size = config["eval_batch_size"]
        self.device = config["device"]
        wd = config["weight_decay"]
        self.weight_decay = (float(eval(wd)) if isinstance(wd, str) else float(wd)) if wd is not None else 0.0
        self.req_training = config["req_training"]
        self.start_epoch = 0
        self.cur_step = 0
        tmp = {f"{j.lower()}@{k}": 0.0 for j, k in itertools.product(config["metrics"] or [], config["topk"] or [])}
        self.best_valid_score = -1
        self.best_valid_result = tmp
        self.best_test_upon_valid = tmp
        self.train_loss_dict = {}
        self.swapped_adjacencies = []
        ops.set_deterministic(bool(config["deterministic"]))  # reproducible scatters (engine-wide)
        if self._on_gpu():
            self.swapped_adjacencies = swap_sparse_attributes(model)
            prep = getattr(model, "engine_layout", None)  # engine-native models lay out their tables
            if callable(prep):
                prep()
        self.optimizer = self._build_optimizer()
        if isinstance(self.optimizer, FusedAdam) and self.optimizer.lazy_rows:
            model.__dict__["_fr_flush"] = self.optimizer.flush  # model.state_dict() applies deferred rows
        sched = config["learning_rate_scheduler"] or [1.0, 50]
        self.lr_scheduler = optim.lr_scheduler.LambdaLR(self.optimizer,
                                                        lr_lambda=lambda e: sched[0] ** (e / sched[1]))
        self.eval_type = config["eval_type"]
        self.mg = mg
        self.alpha1, self.alpha2, self.beta = config["alpha1"], config["alpha2"], config["beta"]
        self._feats = None
        # row-gathered feature tables hand the optimiser (ids, rows) instead of a dense gradient
        # (FusedAdam.row_grads; a data-parallel GradAllReduce routes its RowExchange there too)
        self._row_grads_on = isinstance(self.optimizer, FusedAdam) and (
            config["row_grad_tables"] is None or bool(config["row_grad_tables"]))
        if self._row_grads_on:
            model._fr_exchange = self.optimizer.row_grads
        # optional callable(model) run between backward and the optimiser step (e.g. the
        # data-parallel gradient all-reduce of FoodRec.engine.dist)
        self.grad_hook = None
        # capture the training step in a HIP graph (config key cuda_graph; GPU, single process)
        # host-side batch work (SCHGN's masked-ingredient SSL draws Python's random per batch) cannot
        # be captured: those configurations step eagerly
        # (and only the fused Adam reads the NaN flag on the device: other optimisers step eagerly)
        # and a model whose step sizes launches from host reads (graph_capturable = False: the
        # row-list propagation of LightGCN_ID / ShardedLightGCN) steps eagerly too
        self.use_graph = (bool(config["cuda_graph"]) and self._on_gpu() and not config["SCHGN_ssl"]
                          and isinstance(self.optimizer, FusedAdam) and getattr(model, "graph_capturable", True))
        self._graphed = None

    @property
    def grad_hook(self):
        return self._grad_hook

    @grad_hook.setter
    def grad_hook(self, hook):
        self._grad_hook = hook
        rows = getattr(hook, "rows", None)
        if rows is not None and self._row_grads_on:
            rows.sink = self.optimizer.row_grads

    def _on_gpu(self) -> bool:
        return torch.device(self.device).type == "cuda"

    def _build_optimizer(self):
        params = self.model.parameters()
        name = (self.learner or "adam").lower()
        if name == "adam":
            if self._on_gpu():
                lazy = self.config["lazy_row_adam"]
                slices = self.config["lazy_row_slices"]
                return FusedAdam(params, lr=self.learning_rate, weight_decay=self.weight_decay,
                                 lazy_rows=True if lazy is None else bool(lazy),
                                 lazy_slices=0 if slices is None else int(slices))
            return optim.Adam(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == "sgd":
            return optim.SGD(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == "adagrad":
            return optim.Adagrad(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == "rmsprop":
            return optim.RMSprop(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        self.logger.warning("Received unrecognized optimizer, set default Adam optimizer")
        return FusedAdam(params, lr=self.learning_rate) if self._on_gpu() else optim.Adam(params, lr=self.learning_rate)

    # ------------------------------------------------------------------------------ training
    def _features(self):
        if self._feats is None:
            ds = self.model.dataset if hasattr(self.model, "dataset") else getattr(self, "_dataset", None)
            if ds is None or not hasattr(ds, "ingredientCodeDict"):
                from FoodRec.engine.sampler import IdFeatures  # ids-only graph (InteractionGraph)
                self._feats = IdFeatures(self.device)
            else:
                self._feats = BatchFeatures(ds, self.device, ssl=bool(self.config["SCHGN_ssl"]))
        return self._feats

    def _opt_step(self, skip_flag):
        if isinstance(self.optimizer, FusedAdam):
            self.optimizer.step(skip_flag=skip_flag)  # the kernels read the NaN flag on the device
            ops.run_pending_drains()  # (no-op: the step ran them)
        elif not int(skip_flag.item()):
            # other optimisers: the reference returns before optimizer.step() at the first NaN batch
            # (trainer.py:191-193), so the flag is read on the host before stepping
            self.optimizer.step()

    def train_step(self, interaction, batch_idx, state, loss_func=None, accumulate=True):
        """One optimisation step on one batch (the body of the reference's step loop,
        trainer.py:177-227), with no host synchronisation.  ``state`` carries the device-side
        loss accumulator and NaN flag across steps (``accumulate=False``: overwrite, for capture)."""
        loss_func = loss_func or self.model.calculate_loss
        self.optimizer.zero_grad()
        second_inter = copy.copy(interaction) if (self.mg and batch_idx % self.beta == 0) else None
        ops.defer_counters(True)  # device step counters advance in the step's fr_step_book launch
        try:
            if second_inter is None:
                ops.book_request(state, accumulate)  # a fused loss op may book the step in its own launch
            losses = loss_func(interaction)
            ops.finalize_pending()
            parts = losses if isinstance(losses, tuple) else (losses,)
            booked = self._book_fused(state, parts, accumulate) if second_inter is None else None
        finally:
            ops.book_taken()  # (clears a request nothing answered)
            ops.drop_pending_finalizes()  # (partials a raising loss left behind)
            ops.defer_counters(False)  # (applies the increments eagerly when the step was not booked)
        if booked is not None:
            # the loss sum is never materialised for autograd: each part back-propagates with a
            # cached ones seed; the returned loss is fr_step_book's fp32 sum of the parts
            ops.late_drain(self._late_drain_ok())
            try:
                torch.autograd.backward(list(parts), grad_tensors=self._ones_like(parts))
            finally:
                ops.late_drain(False)
            ops.loss_side_join()
            self._finish_step(state)
            return booked
        ops.loss_side_join()
        loss = sum(parts)
        vec = torch.stack([x.detach().reshape(-1)[0].double() for x in parts])
        if state.get("acc") is None:
            state["acc"] = vec.clone()
        elif accumulate:
            state["acc"].add_(vec)
        else:
            state["acc"].copy_(vec)
        nan_flag = state["nan"]
        nan_flag |= torch.isnan(loss.detach().reshape(-1)[0]).to(torch.int32)
        if second_inter is not None:
            (self.alpha1 * loss).backward()
            self._opt_step(nan_flag)
            self.optimizer.zero_grad()
            l2 = loss_func(second_inter)
            l2 = sum(l2) if isinstance(l2, tuple) else l2
            nan_flag |= torch.isnan(l2.detach().reshape(-1)[0]).to(torch.int32)
            (-1 * self.alpha2 * l2).backward()
        else:
            ops.late_drain(self._late_drain_ok())
            try:
                loss.backward()
            finally:
                ops.late_drain(False)
        self._finish_step(state)
        return loss.detach()

    def _late_drain_ok(self) -> bool:
        """Whether the step's gradients go straight to FusedAdam.step (no clipping, no gradient
        hook): deferred gradient rows may then be added inside the step (ops.late_drain)."""
        return not self.clip_grad_norm and self.grad_hook is None and isinstance(self.optimizer, FusedAdam)

    def _finish_step(self, state):
        """Gradient hook / clipping, then the optimiser step (common/trainer.py:215-224)."""
        if self.clip_grad_norm or self.grad_hook is not None:
            if isinstance(self.optimizer, FusedAdam):
                self.optimizer.materialize_row_grads()  # dense .grad for the norm / the hook
        if self.clip_grad_norm:
            clip_grad_norm_(self.model.parameters(), **self.clip_grad_norm)
        if self.grad_hook is not None:
            self.grad_hook(self.model)
        self._opt_step(state["nan"])
        return None

    def _book_fused(self, state, parts, accumulate):
        """Per-step loss bookkeeping in one HIP launch (fr_step_book): state['acc'] (float64 sums
        of every loss part) and the sticky NaN flag of sum(parts).  Returns the step's loss (the
        fp32 sum, a device scalar), or None when it does not apply (CPU, more than 8 parts,
        non-fp32 or non-scalar parts)."""
        done = ops.book_taken()
        if done is not None:  # a fused loss op booked the step in its launch (ops.healthrec_loss_finalize)
            if len(done[0]) != len(parts) or any(a is not b for a, b in zip(done[0], parts)):
                raise RuntimeError("a loss op booked other loss parts than calculate_loss returned")
            return done[1]
        if not (len(parts) <= 8 and all(torch.is_tensor(x) and x.is_cuda and x.dtype == torch.float32
                                          and x.numel() == 1 and x.is_contiguous() and x.requires_grad
                                          for x in parts)):
            return None
        if state.get("acc") is None:
            state["acc"] = torch.zeros(len(parts), dtype=torch.float64, device=parts[0].device)
            accumulate = False
        elif state["acc"].numel() != len(parts):
            return None
        side = ops.loss_side_stream()  # a loss op forked the side stream: book there too (joined after the backward)
        if side is None:
            return book_step(parts, state["acc"], state["nan"], accumulate)
        side.wait_stream(torch.cuda.current_stream(parts[0].device))
        for x in parts:
            x.record_stream(side)
        with torch.cuda.stream(side):
            return book_step(parts, state["acc"], state["nan"], accumulate)

    def _ones_like(self, parts):
        cache = self.__dict__.setdefault("_ones_cache", {})
        out = []
        for x in parts:
            key = (tuple(x.shape), x.dtype, x.device)
            t = cache.get(key)
            if t is None:
                t = torch.ones(x.shape, dtype=x.dtype, device=x.device)
                t._fr_unit = True  # exactly one, never written: engine backwards skip their device scale
                cache[key] = t
            out.append(t)
        return out

    def graphed_step(self, batch_size: int, warmup: int = 3, unroll: int | None = None):
        """A callable (u, p, n, batch_idx, state) running train_step through captured HIP graphs
        (data parallel: two graphs with the gradient collectives between them; single process:
        ``unroll`` steps per replay, default config ``cuda_graph_unroll``)."""
        if self.grad_hook is not None and hasattr(self.grad_hook, "communicate"):
            return GraphedDPStep(self, batch_size, warmup)
        if unroll is None:
            unroll = int(self.config["cuda_graph_unroll"] or 1) if "cuda_graph_unroll" in self.config else 1
        return GraphedStep(self, batch_size, warmup, unroll=unroll)

    def new_step_state(self):
        return {"acc": None, "nan": torch.zeros((), dtype=torch.int32, device=torch.device(self.device))}

    def _train_epoch(self, train_data, epoch_idx, loss_func=None):
        """One epoch.  ``train_data`` is a TripleSampler (engine path).  Returns
        (per-component loss sums | tensor on NaN, per-batch losses, similarity sums)."""
        if not self.req_training:
            return 0.0, [], None
        self.model.train()
        feats = self._features()
        state = self.new_step_state()
        loss_batches = []
        if self.use_graph and loss_func is None and not self.mg:
            if self._graphed is None:
                self._graphed = self.graphed_step(train_data.batch_size, int(self.config["cuda_graph_warmup"] or 3))
            step = self._graphed
            state = step.state  # the graph accumulates into its own state: reset it for this epoch
            if state["acc"] is not None:
                state["acc"].zero_()
            state["nan"].zero_()
            if step.feed is None and hasattr(train_data, "device_feed"):
                step.attach_feed(train_data)
            for batch_idx, (u, p, n) in enumerate(train_data.epoch(out=step.inputs, feed=step.feed,
                                                                   prefetch=self._prefetch_ok(train_data, epoch_idx))):
                loss_batches.append(step(u, p, n, batch_idx, state))
            step.flush()
        else:
            for batch_idx, (u, p, n) in enumerate(train_data.epoch(prefetch=self._prefetch_ok(train_data, epoch_idx))):
                loss_batches.append(self.train_step(feats.batch(u, p, n), batch_idx, state, loss_func))
        self.flush_optimizer()
        if hasattr(feats, "check_ids"):
            feats.check_ids()
        if state["acc"] is None:
            return 0.0, loss_batches, None
        if int(state["nan"].item()):
            self.logger.info("Loss is nan at epoch: {}. Exiting.".format(epoch_idx))
            return torch.tensor(float("nan")), torch.tensor(0.0), None
        total = tuple(state["acc"].cpu().tolist())
        return (total if len(total) > 1 else total[0]), loss_batches, None

    def _prefetch_ok(self, train_data, epoch_idx) -> bool:
        """Draw the next epoch's permutation and negatives on a host thread during this epoch
        (TripleSampler.prefetch): on a GPU, where nothing in a training epoch draws from the torch CPU
        or np.random generators (dropout runs on the device), so the streams are the reference's;
        not after the last epoch.  Config ``sampler_prefetch`` (default on) turns it off."""
        on = self.config["sampler_prefetch"] if "sampler_prefetch" in self.config else None
        return (hasattr(train_data, "prefetch") and self._on_gpu() and on is not False
                and epoch_idx + 1 < self.epochs)

    # ------------------------------------------------------------------------------ evaluation
    def _candidates(self, is_test):
        """EvalByUserDataloader (dataloader.py:228-302): per user, pos + negatives with the
        positives removed (the removal persists in the dataset's RaggedIds, as the reference's
        in-place list.remove does); native pass in csrc/fr_io.cpp."""
        ds = self.model.dataset
        if not is_test:
            users, pos_lists, neg_lists = ds.valid_users, ds.validRatings, ds.validNegatives
        else:
            users, pos_lists, neg_lists = list(range(ds.num_users)), ds.testRatings, ds.testNegatives
        return eval_candidates(users, pos_lists, neg_lists)

    EVAL_CHUNK_ROWS = 1 << 18

    @torch.no_grad()
    def _score(self, users, items, on_device=False):
        """Scores of the (user, candidate) rows.  The fast graph path gathers from one forward; the
        per-row path (inference_by_user) runs over chunks of ``eval_chunk_rows`` rows (a model
        attribute, else EVAL_CHUNK_ROWS), each an EvalBatch with the reference's side inputs.
        ``on_device``: return the fp32 scores as a device tensor (the device ranking's input)."""
        dev = torch.device(self.device)
        fin = (lambda t: t.float().reshape(-1).contiguous()) if on_device else (lambda t: t.float().reshape(-1).cpu())
        if self.config["graph_inference_fast"]:
            batch = {"user_input": torch.from_numpy(users).to(dev), "item_input": torch.from_numpy(items).to(dev)}
            out = self.model.forward()
            sc = fin(self.model.inference_fast(batch, out[0], out[1]))
            return sc if on_device else sc.numpy()
        step = int(getattr(self.model, "eval_chunk_rows", None) or self.EVAL_CHUNK_ROWS)
        feats = self._features()
        parts = []
        for s in range(0, len(users), step):
            batch = EvalBatch(feats, torch.from_numpy(users[s:s + step]).to(dev),
                              torch.from_numpy(items[s:s + step]).to(dev))
            parts.append(fin(self.model.inference_by_user(batch)))
        if on_device:
            return torch.cat(parts) if parts else torch.zeros(0, dtype=torch.float32, device=dev)
        return torch.cat(parts).numpy() if parts else np.zeros(0, np.float32)

    def flush_optimizer(self):
        """Apply the optimiser's deferred zero-gradient row steps (FusedAdam lazy rows) so every
        parameter holds its dense-Adam value; called at each epoch end and before evaluation."""
        if isinstance(self.optimizer, FusedAdam):
            self.optimizer.flush()

    def _device_candidates(self, is_test):
        """The evaluation lists on the device (uid / offsets / items per user segment, plus the host
        lens / npos), built once per split and kept: after the first pass removed the positives from
        the negatives in place, every later EvalByUserDataloader pass yields the same lists."""
        ds = self.model.dataset
        neg = ds.testNegatives if is_test else ds.validNegatives
        cache = self.__dict__.setdefault("_dev_candidates", {})
        ent = cache.get(bool(is_test))
        if ent is None or ent["neg"] is not neg:
            users, items, lens, npos = self._candidates(is_test)
            dev = torch.device(self.device)
            off = np.zeros(len(lens) + 1, np.int64)
            np.cumsum(lens, out=off[1:])
            uid = users[off[:-1][lens > 0]] if (lens > 0).all() else None
            ent = {"neg": neg, "lens": lens, "npos": npos, "n": int(off[-1]),
                   "uid": None if uid is None else torch.from_numpy(np.ascontiguousarray(uid)).to(dev),
                   "off": torch.from_numpy(off).to(dev), "items": torch.from_numpy(items).to(dev),
                   "users": users, "items_host": items}
            cache[bool(is_test)] = ent
        return ent

    def _fused_scoring(self) -> bool:
        """The model's inference_fast is the plain gather-dot of its forward() tables (engine models
        declare it: ``fused_scores``) and the evaluation runs on the device: fr_score_segments."""
        return (self._on_gpu() and bool(self.config["graph_inference_fast"])
                and getattr(type(self.model), "fused_scores", False))

    @torch.no_grad()
    def _score_fused(self, dc):
        """Device scores of the cached evaluation lists (fr_score_segments over forward()'s tables),
        or None when those tables are not the kernel's fp32 [*, 64] (another embedding_size, bf16
        tables): the caller then scores through the model's inference_fast."""
        out = self.model.forward()
        if not ops.score_segments_ok(out[0], out[1]):
            return None
        return ops.score_segments(out[0], out[1], dc["uid"], dc["off"], dc["items"])

    def _valid_by_user_epoch(self, valid_data=None, is_test=False):
        self.flush_optimizer()
        neg_num = self.config["neg_sample_num"]
        if self._fused_scoring():
            dc = self._device_candidates(is_test)
            sc = self._score_fused(dc) if dc["uid"] is not None else None
            if sc is not None:
                res = self._rank_scores(sc, dc["lens"], dc["npos"], neg_num)
                recalls, ndcgs, aucs = res.mean(axis=0).tolist()
                metrics = {"AUC": aucs[0], "Recall@10": recalls[0], "Recall@20": recalls[1],
                           "NDCG@10": ndcgs[0], "NDCG@20": ndcgs[1]}
                return metrics["NDCG@20"], metrics
        users, items, lens, npos = self._candidates(is_test)
        if self._on_gpu():
            res = self._rank_on_device(users, items, lens, npos, neg_num)
        else:
            preds = self._score(users, items)
            res = np.zeros((len(lens), 3, 2))
            off = 0
            for k, (ln, npo) in enumerate(zip(lens.tolist(), npos.tolist())):
                res[k] = rank_user_host(preds[off:off + ln].copy(), npo, neg_num)
                off += ln
        recalls, ndcgs, aucs = res.mean(axis=0).tolist()
        metrics = {"AUC": aucs[0], "Recall@10": recalls[0], "Recall@20": recalls[1],
                   "NDCG@10": ndcgs[0], "NDCG@20": ndcgs[1]}
        return metrics["NDCG@20"], metrics

    def _rank_on_device(self, users, items, lens, npos, neg_num):
        """Scores stay on the device; fr_rank_metrics ranks every user (top-20 hit masks + the AUC
        counts) and the host turns them into the reference's float64 metrics (metrics_from_hits).
        Users whose top-21 scores tie (numpy's argsort tie order decides) are ranked by the host's
        numpy path on their own scores."""
        return self._rank_scores(self._score(users, items, on_device=True), lens, npos, neg_num)

    def _rank_scores(self, sc, lens, npos, neg_num):
        """fr_rank_metrics over device scores + the reference's float64 metric assembly; users whose
        top-21 scores tie go to the host's numpy path on their own scores."""
        hits, aucc, flags = ops.rank_metrics(sc, lens, npos, 20)
        res = metrics_from_hits(hits, lens, npos, aucc, neg_num)
        redo = np.nonzero(flags)[0]
        if len(redo):
            off = np.zeros(len(lens) + 1, np.int64)
            np.cumsum(lens, out=off[1:])
            host = sc.cpu().numpy()
            for k in redo.tolist():
                res[k] = rank_user_host(host[off[k]:off[k + 1]].copy(), int(npos[k]), neg_num)
        self.last_eval_host_users = int(len(redo))
        return res

    # ------------------------------------------------------------------------------ fit
    def _generate_train_loss_output(self, epoch_idx, s_time, e_time, losses):
        out = "epoch %d training [time: %.2fs, " % (epoch_idx, e_time - s_time)
        if isinstance(losses, tuple):
            out += ", ".join("train_loss%d: %.4f" % (i + 1, l) for i, l in enumerate(losses))
        else:
            out += "train loss: %.4f" % losses
        return out + "]"

    def fit(self, dataset, valid_data=None, test_data=None, hyper_tuple=None, saved=False, verbose=True):
        self._dataset = dataset
        ckpt_name = "{}-{}-{}={}.pt".format(self.config["model"], self.config["dataset"],
                                           self.config["hyper_parameters"], hyper_tuple)
        ckroot = self.config["ckp_root"] or "./ckp/"
        os.makedirs(ckroot, exist_ok=True)
        ckpt = os.path.join(ckroot, ckpt_name)
        sampler = TripleSampler(dataset, self.config["train_batch_size"], self.device)
        saved_once = False
        finished = False
        try:
            for epoch_idx in range(self.start_epoch, self.epochs):
                t0 = time()
                self.model.pre_epoch_processing()
                train_loss, _, _ = self._train_epoch(sampler, epoch_idx)
                if torch.is_tensor(train_loss):
                    break
                for group in self.optimizer.param_groups:
                    self.logger.info("======lr: %f" % group["lr"])
                self.lr_scheduler.step()
                if isinstance(self.optimizer, FusedAdam):
                    self.optimizer.sync_lr()
                self.train_loss_dict[epoch_idx] = sum(train_loss) if isinstance(train_loss, tuple) else train_loss
                t1 = time()
                post = self.model.post_epoch_processing()
                if verbose:
                    self.logger.info(self._generate_train_loss_output(epoch_idx, t0, t1, train_loss))
                    if post is not None:
                        self.logger.info(post)
                if (epoch_idx + 1) % self.eval_step == 0:
                    v0 = time()
                    valid_score, valid_result = self._valid_by_user_epoch(is_test=False)
                    self.best_valid_score, self.cur_step, stop_flag, update_flag = early_stopping(
                        valid_score, self.best_valid_score, self.cur_step, max_step=self.stopping_step,
                        bigger=self.valid_metric_bigger)
                    v1 = time()
                    if verbose:
                        self.logger.info("epoch %d evaluating [time: %.2fs, valid_score: %f]" % (epoch_idx, v1 - v0, valid_score))
                        self.logger.info("valid result: \n" + dict2str(valid_result))
                    if update_flag:
                        torch.save(self.model.state_dict(), ckpt)
                        saved_once = True
                        if verbose:
                            self.logger.info("██ " + str(self.config["model"]) + "--Best validation results updated!!!")
                        self.best_valid_result = valid_result
                    if stop_flag:
                        if verbose:
                            self.logger.info("+++++Finished training, best eval result in epoch %d" %
                                             (epoch_idx - self.cur_step * self.eval_step))
                        break
            finished = True
        finally:
            # early stop, the NaN break or an exception: the sampler's prefetch thread is joined here,
            # so no host draw outlives fit() (a grid search reseeds before its next run)
            if finished:
                sampler.close()
            else:
                try:
                    sampler.close()
                except Exception:  # (the exception already raised is the one to report)
                    pass
        if saved_once:
            self.model.load_state_dict(torch.load(ckpt, weights_only=True))
        _, test_result = self._valid_by_user_epoch(is_test=True)
        self.logger.info("test result: \n" + dict2str(test_result))
        self.best_test_upon_valid = test_result
        return self.best_valid_score, self.best_valid_result, self.best_test_upon_valid
