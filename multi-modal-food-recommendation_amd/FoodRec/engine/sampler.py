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


def draw_negatives(users: np.ndarray, num_items: int, excl_ptr, excl_items, excl2_ptr, excl2_items) -> np.ndarray:
    """np.random-stream-exact rejection sampling for every user in ``users`` (in order)."""
    users = np.ascontiguousarray(users, dtype=np.int64)
    out = np.empty(len(users), np.int64)
    st, key, pos = _np_state()
    lib = native.lib()
    rc = lib.fr_sampler_negatives(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                  pos.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(num_items),
                                  users.ctypes.data, len(users),
                                  np.ascontiguousarray(excl_ptr, np.int64).ctypes.data,
                                  np.ascontiguousarray(excl_items, np.int64).ctypes.data,
                                  None if excl2_ptr is None else np.ascontiguousarray(excl2_ptr, np.int64).ctypes.data,
                                  None if excl2_items is None else np.ascontiguousarray(excl2_items, np.int64).ctypes.data,
                                  out.ctypes.data)
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

    def _negatives(self, users):
        d = self.ds
        return draw_negatives(users, d.num_items, d.excl_train_ptr, d.excl_train_items,
                              d.excl_vt_ptr, d.excl_vt_items)

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

    def epoch(self):
        """Yield (u, pos, neg) int64 device tensors per batch for one epoch.  Negatives are drawn
        per batch (same stream as the reference's per-sample draws, in permutation order)."""
        perm = self.epoch_order().numpy()
        perm_d = torch.from_numpy(perm).to(self.device, non_blocking=True)
        pin = self.device.type == "cuda"
        for s in range(0, self.n, self.batch_size):
            negs = torch.from_numpy(self._negatives(self.users[perm[s:s + self.batch_size]]))
            if pin:
                negs = negs.pin_memory()
            idx = perm_d[s:s + self.batch_size]
            yield self._dev_users[idx], self._dev_items[idx], negs.to(self.device, non_blocking=True)


class BatchFeatures:
    """Device-resident per-item side tables used to assemble the reference's batch dict
    (dataloader.py:50-115): ingredient codes/counts, health multi-hot, image rows."""

    def __init__(self, dataset, device):
        self.device = torch.device(device)
        self.ingre_code = torch.from_numpy(np.asarray(dataset.ingredientCodeDict, np.int64)).to(self.device)
        self.ingre_num = torch.tensor(dataset.ingredientNum, dtype=torch.int64, device=self.device)
        self.health = None
        if getattr(dataset, "health_level_multi_hot", None) is not None:
            self.health = torch.from_numpy(dataset.health_matrix()).to(self.device)
        self._image = None
        self._ds = dataset

    def image(self):
        if self._image is None:
            self._image = torch.from_numpy(np.asarray(self._ds.embImage, np.float64)).to(self.device)
        return self._image

    def batch(self, u, p, n) -> "LazyBatch":
        return LazyBatch(self, u, p, n)


class LazyBatch(dict):
    """dict with the reference batch keys; side features are gathered on first access."""

    _LAZY = ("pos_ingre_code", "pos_ingre_num", "pos_hl_mh", "pos_img",
             "neg_ingre_code", "neg_ingre_num", "neg_hl_mh", "neg_img",
             # engine extras: [pos; neg] stacked (one gather instead of two gathers and a cat)
             "pn_i_id", "pn_ingre_code", "pn_ingre_num", "pn_hl_mh")

    def __init__(self, feats: BatchFeatures, u, p, n):
        super().__init__(u_id=u, pos_i_id=p, neg_i_id=n)
        self._f = feats

    def _make(self, key):
        if key == "pn_i_id":
            return torch.cat([self["pos_i_id"], self["neg_i_id"]])
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
        return dict.__contains__(self, key) or (key in self._LAZY and (key not in ("pos_hl_mh", "neg_hl_mh") or self._f.health is not None))

    def keys(self):
        return list(dict.keys(self)) + [k for k in self._LAZY if k not in dict.keys(self) and k in self]

    def items(self):
        return [(k, self[k]) for k in self.keys()]
