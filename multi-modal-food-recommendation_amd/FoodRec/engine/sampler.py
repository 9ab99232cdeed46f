"""Batch triple sampler with the reference's exact RNG stream.

Reference order of random draws inside Trainer.fit (common/trainer.py:398-404):
  1. TrainDataLoader(use_neg_list=False) and TrainDataLoader(use_neg_list=True) each run
     init_neg_list (utils/dataloader.py:40-48): one rejection-sampled negative per training
     pair from np.random, in trainMatrix.keys() order, then random.sample(neg_list, n);
  2. every epoch, DataLoader.__iter__ draws a base seed (torch global RNG), RandomSampler
     draws a second int64 that seeds a private generator for torch.randperm(n);
  3. __getitem__ per index (permutation order) draws that pair's negative from np.random:
     randint(num_items) rejected while in trainList[u] or validTestRatings[u] (:145-151).

Here step 1 and each epoch's negatives are drawn in one native call (fr_sampler_negatives, the
same MT19937 masked-rejection stream as numpy's legacy RandomState; the np.random state is read
and written back so the global stream stays in sync), and torch's own randperm is used for the
permutation.  Batches are materialised on the device by index gathers.
"""
from __future__ import annotations

import ctypes
import random

import numpy as np
import torch

from . import native


def _np_state():
    st = np.random.get_state()
    assert st[0] == "MT19937"
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = np.array([st[2]], dtype=np.int32)
    return st, key, pos


def draw_negatives(users: np.ndarray, num_items: int, excl_ptr, excl_items, excl2_ptr, excl2_items,
                   perm: np.ndarray | None = None, out: np.ndarray | None = None) -> np.ndarray:
    """np.random-stream-exact rejection sampling for every user in ``users`` (in order), or for
    ``users[perm]`` with ``perm`` (no permuted copy); ``out``: a caller's int64 buffer (e.g. a pinned
    staging tensor's numpy view) of the draws' length."""
    users = np.ascontiguousarray(users, dtype=np.int64)
    n = len(users) if perm is None else len(perm)
    if perm is not None:
        perm = np.ascontiguousarray(perm, dtype=np.int64)  # (entries range-checked by the native loop)
    if out is None:
        out = np.empty(n, np.int64)
    elif out.dtype != np.int64 or out.shape != (n,) or not out.flags.c_contiguous:
        raise native.EngineError("draw_negatives: out must be a contiguous int64 array of the draws' length")
    excl_ptr = np.ascontiguousarray(excl_ptr, np.int64)
    n_users = len(excl_ptr) - 1
    if n_users < 0 or (excl2_ptr is not None and len(excl2_ptr) != len(excl_ptr)):
        raise native.EngineError("draw_negatives: the exclusion row pointers need n_users + 1 entries each")
    st, key, pos = _np_state()
    lib = native.lib()
    tail = (n_users, excl_ptr.ctypes.data, np.ascontiguousarray(excl_items, np.int64).ctypes.data,
            None if excl2_ptr is None else np.ascontiguousarray(excl2_ptr, np.int64).ctypes.data,
            None if excl2_items is None else np.ascontiguousarray(excl2_items, np.int64).ctypes.data, out.ctypes.data)
    kp = (key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), pos.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
          int(num_items))
    if perm is None:
        rc = lib.fr_sampler_negatives(*kp, users.ctypes.data, n, *tail)
    else:
        rc = lib.fr_sampler_negatives_perm(*kp, users.ctypes.data, len(users), perm.ctypes.data, n, *tail)
    native.check(rc, "fr_sampler_negatives")
    np.random.set_state((st[0], key, int(pos[0]), st[3], st[4]))
    return out


class TripleSampler:
    """Epoch iterator over (user, pos, neg) batches, identical to the reference DataLoader."""

    def __init__(self, dataset, batch_size: int, device=None, replay_python_random: bool = True):
        self.ds = dataset
        self.batch_size = int(batch_size)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.users = np.ascontiguousarray(dataset.train_pairs[:, 0], np.int64)
        self.items = np.ascontiguousarray(dataset.train_pairs[:, 1], np.int64)
        self.n = len(self.users)
        # the two TrainDataLoader constructions of Trainer.fit (init_neg_list x 2)
        self.neg_list_pre = self._init_neg_list(replay_python_random)
        self.neg_list_post = self._init_neg_list(replay_python_random)
        self._dev_users = torch.from_numpy(self.users).to(self.device)
        self._dev_items = torch.from_numpy(self.items).to(self.device)
        self._pending = None    # the next epoch's host draws, in flight on a host thread (prefetch)
        self._pool = None
        self._slot = 0          # pinned staging buffer of the next draw (two alternate)
        self._pins = [None, None]
        self._pin_copied = [None, None]
        self.last_draw_ms = None

    def _negatives(self, users, perm=None, out=None):
        d = self.ds
        return draw_negatives(users, d.num_items, d.excl_train_ptr, d.excl_train_items,
                              d.excl_vt_ptr, d.excl_vt_items, perm=perm, out=out)

    def _init_neg_list(self, replay_python_random):
        negs = self._negatives(self.users)
        if replay_python_random:
            # random.sample(neg_list, n) consumes Python's RNG as a function of n only
            shuffled = random.sample(range(self.n), self.n)
            return negs[np.asarray(shuffled, dtype=np.int64)]
        return negs

    def __len__(self):
        return (self.n + self.batch_size - 1) // self.batch_size

    def epoch_order(self) -> torch.Tensor:
        """Consume the torch global RNG like DataLoader(RandomSampler) and return the permutation."""
        torch.empty((), dtype=torch.int64).random_()           # _BaseDataLoaderIter._base_seed
        seed = int(torch.empty((), dtype=torch.int64).random_().item())  # RandomSampler
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(self.n, generator=g)

    def device_feed(self):
        """A DeviceFeed over this sampler's device arrays (for a graphed step that gathers its own
        batches: see DeviceFeed)."""
        return DeviceFeed(self._dev_users, self._dev_items, self.n, self.batch_size, self.device)

    def _draw_host(self, slot):
        """One epoch's host draws: the permutation and every pair's negative, in the reference's
        order; on a GPU into pinned staging buffer ``slot`` (after its previous copy has finished)."""
        import time
        t0 = time.perf_counter()
        perm = self.epoch_order().numpy()
        if self.device.type == "cuda":
            if self._pins[slot] is None or self._pins[slot].numel() != self.n:
                self._pins[slot] = torch.empty(self.n, dtype=torch.int64, pin_memory=True)
                self._pin_copied[slot] = None
            if self._pin_copied[slot] is not None:
                self._pin_copied[slot].synchronize()  # this buffer's previous copy to the device is done
            self._negatives(self.users, perm=perm, out=self._pins[slot].numpy())
            negs = self._pins[slot]
        else:
            negs = torch.from_numpy(self._negatives(self.users, perm=perm))
        self.last_draw_ms = (time.perf_counter() - t0) * 1e3
        return perm, negs, slot

    def prefetch(self):
        """Start the next epoch's host draws (torch's permutation, np.random's negatives) on a host
        thread, so they overlap this epoch's steps; the next ``epoch()`` takes them.  The streams are
        those of drawing at the next epoch's start provided nothing else draws from the torch CPU or
        np.random global generators meanwhile -- true of a GPU training epoch (device dropout), which is
        where the trainer uses it.  The native sampler and randperm release the GIL."""
        if self._pending is not None:
            return
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="fr-sampler")
        slot, self._slot = self._slot, self._slot ^ 1
        self._pending = self._pool.submit(self._draw_host, slot)

    def wait_prefetch(self):
        """Block until a prefetch in flight has finished (its draws stay queued for ``epoch()``)."""
        if self._pending is not None:
            self._pending.result()

    def discard_prefetch(self):
        """Wait for a prefetch in flight and drop its draws (the generators have advanced past them:
        measurement use only)."""
        if self._pending is not None:
            self._pending.result()
            self._pending = None

    def close(self):
        """Join a prefetch in flight (its draws are dropped; an exception the host thread raised is
        re-raised here) and shut the thread down, so no draw outlives the caller's training run (a
        later run's init_seed could otherwise be overwritten by a late np.random.set_state)."""
        pend, self._pending = self._pending, None
        try:
            if pend is not None:
                pend.result()
        finally:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
                self._pool = None

    def epoch(self, out=None, feed=None, prefetch: bool = False):
        """Yield (u, pos, neg) int64 device tensors per batch for one epoch.  Negatives are drawn
        per batch (same stream as the reference's per-sample draws, in permutation order).  With
        ``out`` = three [batch_size] device buffers (a graphed step's static inputs), full batches
        are written into them and the buffers are yielded.  ``prefetch``: once this epoch is staged,
        start the next epoch's host draws on a host thread (``prefetch()``)."""
        # the whole epoch's negatives in one native call and one host->device copy: the same draws in
        # the same order as per-batch (or the reference's per-sample) drawing, since nothing else
        # consumes np.random during an epoch; the steps then only index device arrays.  On a GPU the
        # draws land in one of two persistent pinned staging buffers (no pageable copy / pin per epoch)
        if self._pending is not None:
            perm, negs_h, slot = self._pending.result()
            self._pending = None
        else:
            slot, self._slot = self._slot, self._slot ^ 1
            perm, negs_h, slot = self._draw_host(slot)
        perm_d = torch.from_numpy(perm).to(self.device, non_blocking=True)
        if self.device.type == "cuda":
            negs_d = negs_h.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._pin_copied[slot] = ev
        else:
            negs_d = negs_h
        if feed is not None and out is not None:
            feed.stage(perm_d, negs_d)
        if prefetch:
            self.prefetch()
        for s in range(0, self.n, self.batch_size):
            idx = perm_d[s:s + self.batch_size]
            negs = negs_d[s:s + self.batch_size]
            if out is not None and idx.numel() == out[0].numel():
                if feed is not None:  # the consumer's graph gathers this batch itself
                    yield out
                    continue
                torch.index_select(self._dev_users, 0, idx, out=out[0])
                torch.index_select(self._dev_items, 0, idx, out=out[1])
                out[2].copy_(negs)
                yield out
            else:
                yield self._dev_users[idx], self._dev_items[idx], negs


class DeviceFeed:
    """The epoch's permutation and negatives staged in fixed device buffers plus a device batch
    cursor, so a captured step gathers its own (u, pos, neg) batch (``fill``, inside the graph):
    the host only replays the graph per step, no kernels between replays.  ``stage`` (once per
    epoch, outside the graph) copies the epoch in and rewinds the cursor."""

    def __init__(self, dev_users, dev_items, n, batch_size, device):
        self.users, self.items = dev_users, dev_items
        self.B = int(batch_size)
        self.perm = torch.zeros(n, dtype=torch.int64, device=device)
        self.negs = torch.zeros(n, dtype=torch.int64, device=device)
        self.cursor = torch.zeros((), dtype=torch.int64, device=device)
        self.offs = torch.arange(self.B, dtype=torch.int64, device=device)
        self._pos = torch.empty(self.B, dtype=torch.int64, device=device)
        self._idx = torch.empty(self.B, dtype=torch.int64, device=device)
        self.on_stage = None  # called before a new epoch is staged (a graphed step's pending steps)

    def stage(self, perm_d, negs_d):
        from . import ops
        if self.on_stage is not None:
            self.on_stage()
        ops.drop_pending(self.cursor)
        self.perm.copy_(perm_d)
        self.negs.copy_(negs_d)
        self.cursor.zero_()

    def fill(self, u, p, n, feats=None):
        """Gather batch ``cursor`` into (u, p, n) and advance the cursor.  With ``feats`` (a
        BatchFeatures on the GPU) the [pos; neg] item features are gathered in the same launch
        (fr_feed_batch) into feats' static buffers, which are returned for ``feats.batch(..., pre=)``."""
        from . import ops
        ops.settle_counter(self.cursor)
        if feats is not None and feats.native_ok():
            pre = feats.pn_buffers(self.B)
            feats.launch_feed(self, u, p, n, pre)
            ops.defer_increment(self.cursor)  # advanced by the step's fr_step_book
            return pre
        torch.add(self.offs, self.cursor * self.B, out=self._pos)
        torch.index_select(self.perm, 0, self._pos, out=self._idx)
        torch.index_select(self.users, 0, self._idx, out=u)
        torch.index_select(self.items, 0, self._idx, out=p)
        torch.index_select(self.negs, 0, self._pos, out=n)
        ops.defer_increment(self.cursor)
        return None


SSL_MASKED_P = 0.2   # TrainDataLoader.masked_p (dataloader.py:19)
SSL_MAX_LEN = 20     # TrainDataLoader.max_len


def ssl_sequences(codes: np.ndarray, nums: np.ndarray, n_ingredients: int, rnd=random):
    """TrainDataLoader.ssl_task + utils.get_neg_ingre (dataloader.py:117-143, utils/utils.py:186-190)
    for a batch of positives in sample order, drawing from Python's ``random`` exactly as the
    reference's per-sample __getitem__ does: per valid ingredient one random() < 0.2 masks it
    (token n_ingredients + 1) and draws a negative ingredient by randint rejection against the
    recipe's own ingredients.  Returns (masked, pos, neg) int64 [B, L]."""
    B, L = codes.shape
    masked = codes.copy()
    neg = codes.copy()
    mask_tok = n_ingredients + 1
    for b in range(B):
        k = int(nums[b])
        row = codes[b].tolist()
        own = set(row[:k])
        for t in range(min(k, L)):
            if rnd.random() < SSL_MASKED_P:
                masked[b, t] = mask_tok
                j = rnd.randint(0, n_ingredients - 1)
                while j in own:
                    j = rnd.randint(0, n_ingredients - 1)
                neg[b, t] = j
    return masked, codes.copy(), neg


class IdFeatures:
    """Batch assembly for an interaction graph without item side tables (LightGCN_ID on an
    InteractionGraph): the batch is the (u, pos, neg) ids alone."""

    ssl = False

    def __init__(self, device):
        self.device = torch.device(device)

    def native_ok(self) -> bool:
        return False

    def batch(self, u, p, n, pre=None):
        return {"u_id": u, "pos_i_id": p, "neg_i_id": n}


class BatchFeatures:
    """Device-resident per-item side tables used to assemble the reference's batch dict
    (dataloader.py:50-115): ingredient codes/counts, health multi-hot, image rows, calorie levels;
    with ``ssl`` (config SCHGN_ssl) the masked-ingredient sequences of every batch."""

    def __init__(self, dataset, device, ssl: bool = False):
        self.device = torch.device(device)
        self.ingre_code = torch.from_numpy(np.asarray(dataset.ingredientCodeDict, np.int64)).to(self.device)
        self.ingre_num = torch.tensor(dataset.ingredientNum, dtype=torch.int64, device=self.device)
        self.health = None
        if getattr(dataset, "health_level_multi_hot", None) is not None:
            self.health = torch.from_numpy(dataset.health_matrix()).to(self.device)
        self.cal = None
        cal = getattr(dataset, "cal_level", None)
        if cal is not None:
            dense = np.zeros(len(dataset.ingredientNum), np.int64)
            for i, lv in (cal.items() if isinstance(cal, dict) else enumerate(cal)):
                if 0 <= int(i) < len(dense):
                    dense[int(i)] = int(lv)
            self.cal = torch.from_numpy(dense).to(self.device)
        self.ssl = bool(ssl)
        if self.ssl:
            self._codes_np = np.asarray(dataset.ingredientCodeDict, np.int64)
            self._nums_np = np.asarray(dataset.ingredientNum, np.int64)
            self._n_ingre = int(dataset.num_ingredients)
        self._image = None
        self._ds = dataset
        self.pad_id = int(getattr(dataset, "num_ingredients", -1) or -1)  # HealthRec's ingredient padding id

    def image(self):
        if self._image is None:
            self._image = torch.from_numpy(np.asarray(self._ds.embImage, np.float64)).to(self.device)
        return self._image

    # ------------------------------------------------------------------ [pos; neg] features (fr_feed_batch)
    def native_ok(self) -> bool:
        return self.device.type == "cuda" and self.ingre_code.dim() == 2 and self.ingre_code.shape[1] >= 1

    def _pn_alloc(self, B):
        dev = self.device
        L = self.ingre_code.shape[1]
        out = {"pn_i_id": torch.empty(2 * B, dtype=torch.int64, device=dev),
               "pn_ingre_code": torch.empty(2 * B, L, dtype=torch.int64, device=dev),
               "pn_ingre_num": torch.empty(2 * B, dtype=torch.int64, device=dev),
               "pn_pad_kpm": torch.empty(2 * B, L, dtype=torch.float32, device=dev)}
        if self.health is not None:
            out["pn_hl_mh"] = torch.empty(2 * B, self.health.shape[1], dtype=self.health.dtype, device=dev)
        return out

    def pn_buffers(self, B):
        """Static [pos; neg] feature buffers for batch size B (a graphed step's inputs)."""
        cache = self.__dict__.setdefault("_pn_static", {})
        if B not in cache:
            cache[B] = self._pn_alloc(B)
        return cache[B]

    def _launch(self, perm, users, items, negs, cursor, B, u, p, n, out):
        from . import native
        h = self.health
        H = 0 if h is None else h.shape[1]
        native.check(native.lib().fr_feed_batch(
            native.ptr(perm), native.ptr(users), native.ptr(items), native.ptr(negs), native.ptr(cursor), B,
            native.ptr(u), p.data_ptr(), n.data_ptr(), self.ingre_code.data_ptr(), self.ingre_code.shape[1],
            self.ingre_num.data_ptr(), native.ptr(h), H, self.ingre_code.shape[0], self.pad_id,
            out["pn_i_id"].data_ptr(), out["pn_ingre_code"].data_ptr(), out["pn_ingre_num"].data_ptr(),
            native.ptr(out.get("pn_hl_mh")), out["pn_pad_kpm"].data_ptr(), self.id_error_flag().data_ptr(),
            native.stream_of(p)), "fr_feed_batch")

    def id_error_flag(self):
        """Sticky device flag fr_feed_batch sets when a batch carried an item id outside the item
        table (replaced by item 0); the trainer checks it at epoch end (one host read)."""
        f = self.__dict__.get("_id_err")
        if f is None:
            f = self._id_err = torch.zeros((), dtype=torch.int32, device=self.device)
        return f

    def check_ids(self):
        f = self.__dict__.get("_id_err")
        if f is not None and int(f.item()):
            f.zero_()
            raise RuntimeError("fr_feed_batch met item ids outside the item table (sampler or staging bug); "
                               "they were replaced by item 0")

    def launch_feed(self, feed, u, p, n, out):
        self._launch(feed.perm, feed.users, feed.items, feed.negs, feed.cursor, feed.B, u, p, n, out)

    def gather_pn(self, p, n) -> dict:
        """The [pos; neg] item features of a batch in one launch (fresh tensors)."""
        p, n = p.to(torch.int64).contiguous(), n.to(torch.int64).contiguous()
        out = self._pn_alloc(p.numel())
        self._launch(None, None, None, None, None, p.numel(), None, p, n, out)
        return out

    def batch(self, u, p, n, pre=None) -> "LazyBatch":
        b = LazyBatch(self, u, p, n)
        if pre is not None:
            dict.update(b, pre)
        if self.ssl:  # eager, like the reference's per-sample __getitem__ (the RNG stream advances per batch)
            pi = p.cpu().numpy()
            seqs = ssl_sequences(self._codes_np[pi], self._nums_np[pi], self._n_ingre)
            for key, arr in zip(("masked_ingre_seq", "pos_ingre_seq", "neg_ingre_seq"), seqs):
                b[key] = torch.from_numpy(arr).to(self.device)
        return b


class LazyBatch(dict):
    """dict with the reference batch keys; side features are gathered on first access."""

    _LAZY = ("pos_ingre_code", "pos_ingre_num", "pos_hl_mh", "pos_img", "pos_cl",
             "neg_ingre_code", "neg_ingre_num", "neg_hl_mh", "neg_img", "neg_cl",
             # engine extras: [pos; neg] stacked, gathered together in one launch (fr_feed_batch), and
             # the ingredient key-padding mask of the stacked codes in the additive float form
             # (-inf at padding, 0 elsewhere) the Transformer layer consumes as it is
             "pn_i_id", "pn_ingre_code", "pn_ingre_num", "pn_hl_mh", "pn_pad_kpm")

    def __init__(self, feats: BatchFeatures, u, p, n):
        super().__init__(u_id=u, pos_i_id=p, neg_i_id=n)
        self._f = feats

    def _make(self, key):
        if key.startswith("pn_") and self._f.native_ok():
            got = self._f.gather_pn(self["pos_i_id"], self["neg_i_id"])  # every pn_ key in one launch
            for k, v in got.items():
                if not dict.__contains__(self, k):
                    dict.__setitem__(self, k, v)
            if key not in got:
                raise KeyError(key)
            return got[key]
        if key == "pn_i_id":
            return torch.cat([self["pos_i_id"], self["neg_i_id"]])
        if key == "pn_pad_kpm":
            codes = self["pn_ingre_code"]
            return torch.zeros(codes.shape, dtype=torch.float32, device=codes.device).masked_fill_(
                codes == self._f.pad_id, float("-inf"))
        side, what = key.split("_", 1)
        idx = {"pos": self["pos_i_id"], "neg": self["neg_i_id"]}.get(side)
        if idx is None:
            idx = self["pn_i_id"]
        f = self._f
        if what == "ingre_code":
            return f.ingre_code[idx]
        if what == "ingre_num":
            return f.ingre_num[idx]
        if what == "hl_mh":
            if f.health is None:
                raise KeyError(key)
            return f.health[idx]
        if what == "img":
            return f.image()[idx]
        if what == "cl":
            if f.cal is None:
                raise KeyError(key)
            return f.cal[idx]
        raise KeyError(key)

    def __missing__(self, key):
        if key in self._LAZY:
            v = self._make(key)
            self[key] = v
            return v
        raise KeyError(key)

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def __contains__(self, key):
        if dict.__contains__(self, key):
            return True
        if key not in self._LAZY:
            return False
        if key in ("pos_hl_mh", "neg_hl_mh", "pn_hl_mh"):
            return self._f.health is not None
        if key in ("pos_cl", "neg_cl"):
            return self._f.cal is not None
        return True

    def keys(self):
        return list(dict.keys(self)) + [k for k in self._LAZY if k not in dict.keys(self) and k in self]

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def __copy__(self):
        """The trainer's ``second_inter`` (trainer.py:181, for --mg): the same tensors, lazy keys
        still lazy (the reference deep-copies; nothing here mutates a batch tensor in place)."""
        out = LazyBatch.__new__(LazyBatch)
        dict.update(out, dict.items(self))
        out._f = self._f
        return out


class EvalBatch(dict):
    """The per-user evaluation batch of EvalByUserDataloader (dataloader.py:228-302) for a chunk of
    (user, candidate) rows: ``user_input`` / ``item_input`` plus, gathered on first access, the
    candidates' ``img_input`` (float32), ``ingre_input``, ``ingre_num_input``, ``cal_level_input``
    and ``health_level_input`` (the reference fills the latter with the calorie level too)."""

    def __init__(self, feats: BatchFeatures, users, items):
        super().__init__(user_input=users, item_input=items)
        self._f = feats

    def _make(self, key):
        f, it = self._f, self["item_input"]
        if key == "img_input":
            return f.image()[it].to(torch.float32)
        if key == "ingre_input":
            return f.ingre_code[it]
        if key == "ingre_num_input":
            return f.ingre_num[it]
        if key in ("cal_level_input", "health_level_input") and f.cal is not None:
            return f.cal[it]
        raise KeyError(key)

    def __missing__(self, key):
        v = self._make(key)
        self[key] = v
        return v

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def __contains__(self, key):
        if dict.__contains__(self, key):
            return True
        if key in ("img_input", "ingre_input", "ingre_num_input"):
            return True
        return key in ("cal_level_input", "health_level_input") and self._f.cal is not None
