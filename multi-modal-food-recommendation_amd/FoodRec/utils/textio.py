"""Native readers of the reference's interaction text files and the ragged id lists they fill.

The reference parses ``data.*.negative`` / ``data.*.rating`` line by line in Python
(utils/dataset.py:93-176,245-256) and keeps each negative file as a list of Python lists; at the
Allrecipes shape that is 97,768 lists x 999 ids and most of its load time.  Here the C-ABI
readers (``fr_io_open`` / ``fr_io_fill``, csrc/fr_io.cpp) parse the files in parallel straight into
int64 arrays, and :class:`RaggedIds` keeps them as (values, offsets) with an alive mask standing in
for the reference's in-place ``list.remove`` (dataloader.py:228-302): indexing a user returns that
user's list as Python ints, exactly what ``testNegatives[u]`` returned in the reference.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ..engine import native

FR_IO_NEGATIVE = 0
FR_IO_RATING = 1


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def _threads() -> int:
    return int(os.environ.get("FR_IO_THREADS", "0"))


def _read(path: str, mode: int, with_aux: bool):
    lib = native.lib()
    table = ctypes.c_void_p()
    rows, vals = ctypes.c_int64(), ctypes.c_int64()
    rc = lib.fr_io_open(os.fsencode(path), mode, _threads(), ctypes.byref(table), ctypes.byref(rows),
                        ctypes.byref(vals))
    if rc == 5:  # FR_EIO: the reference's open() raises FileNotFoundError / OSError
        msg = lib.fr_last_error().decode()
        raise FileNotFoundError(msg) if not os.path.exists(path) else OSError(msg)
    native.check(rc, "fr_io_open")
    try:
        values = np.empty(vals.value, np.int64)
        offsets = np.empty(rows.value + 1, np.int64) if mode == FR_IO_NEGATIVE else None
        aux = np.empty(rows.value, np.float64) if with_aux else None
        bad = ctypes.c_int64()
        rc = lib.fr_io_fill(table, _p(values), _p(offsets), _p(aux), ctypes.byref(bad))
        if rc == 6:  # FR_EPARSE: the reference's int()/float() raise ValueError
            raise ValueError(f"{path}: {lib.fr_last_error().decode()}")
        native.check(rc, "fr_io_fill")
    finally:
        lib.fr_io_close(table)
    return values, offsets, aux


def read_negatives(path: str) -> "RaggedIds":
    """``InteractionData.load_negative_file`` (utils/dataset.py:245-256): per line, the int() ids
    after the first tab-separated field."""
    values, offsets, _ = _read(path, FR_IO_NEGATIVE, False)
    return RaggedIds(values, offsets)


def read_ratings(path: str, with_rating: bool = True):
    """``u\\ti\\trating`` lines (utils/dataset.py:93-176) -> ([n, 2] int64 (u, i), [n] float64 rating or
    None).  A training file line without a rating field raises IndexError, as ``arr[2]`` does."""
    values, _, aux = _read(path, FR_IO_RATING, with_rating)
    pairs = values.reshape(-1, 2)
    if with_rating and len(aux) and np.isnan(aux).any():
        line = int(np.flatnonzero(np.isnan(aux))[0]) + 1
        raise IndexError(f"{path}: line {line}: list index out of range (no rating field)")
    return pairs, aux


class RaggedIds:
    """Per-user id lists as flat int64 ``values`` with ``offsets[n + 1]`` and an ``alive`` mask.

    Sequence protocol of the reference's list of lists: ``len()``, ``[u]`` -> list of Python ints
    (the alive ids of row u in file order), iteration.  Rows are read-only views; the one in-place
    edit the reference makes, removing evaluation positives (dataloader.py:228-302), is
    :meth:`remove_positives`, which persists like the reference's mutation of its lists.
    """

    __slots__ = ("values", "offsets", "alive", "_all_alive")

    def __init__(self, values: np.ndarray, offsets: np.ndarray, alive: np.ndarray | None = None):
        self.values = np.ascontiguousarray(values, dtype=np.int64)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.alive = np.ones(len(self.values), np.uint8) if alive is None else np.ascontiguousarray(alive, np.uint8)
        self._all_alive = alive is None

    @classmethod
    def from_dense(cls, rows: np.ndarray) -> "RaggedIds":
        rows = np.asarray(rows, dtype=np.int64)
        n, k = rows.shape if rows.ndim == 2 else (len(rows), 0)
        return cls(rows.reshape(-1), np.arange(n + 1, dtype=np.int64) * k)

    @classmethod
    def from_lists(cls, lists) -> "RaggedIds":
        lens = np.fromiter((len(x) for x in lists), np.int64, count=len(lists))
        offsets = np.zeros(len(lens) + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        values = (np.fromiter((v for x in lists for v in x), np.int64, count=int(offsets[-1]))
                  if offsets[-1] else np.zeros(0, np.int64))
        return cls(values, offsets)

    def __len__(self) -> int:
        return len(self.offsets) - 1

    def row(self, u: int) -> np.ndarray:
        b, e = self.offsets[u], self.offsets[u + 1]
        v = self.values[b:e]
        return v if self._all_alive else v[self.alive[b:e].astype(bool)]

    def __getitem__(self, u):
        if isinstance(u, slice):
            return [self[i] for i in range(*u.indices(len(self)))]
        u = int(u)
        if u < 0:
            u += len(self)
        if not 0 <= u < len(self):
            raise IndexError("list index out of range")
        return self.row(u).tolist()

    def __iter__(self):
        for u in range(len(self)):
            yield self.row(u).tolist()

    def tolist(self) -> list:
        return list(self)

    def lengths(self) -> np.ndarray:
        if self._all_alive:
            return np.diff(self.offsets)
        c = np.zeros(len(self.values) + 1, np.int64)
        np.cumsum(self.alive, out=c[1:])
        return c[self.offsets[1:]] - c[self.offsets[:-1]]

    def compact(self) -> "RaggedIds":
        """The alive ids only, as a fresh RaggedIds."""
        if self._all_alive:
            return self
        offsets = np.zeros(len(self) + 1, np.int64)
        np.cumsum(self.lengths(), out=offsets[1:])
        return RaggedIds(self.values[self.alive.astype(bool)], offsets)

    def remove_positives(self, pos: "RaggedIds") -> np.ndarray:
        """For each row u and each id p of pos[u] in order: drop the first alive occurrence of p in
        row u (``if item in neg: neg.remove(item)``).  Returns lens[u] = |pos[u]| + alive ids of u."""
        if len(pos) != len(self):
            raise ValueError(f"{len(pos)} positive rows for {len(self)} negative rows")
        pos = pos.compact()
        lens = np.empty(len(self), np.int64)
        total = ctypes.c_int64()
        native.check(native.lib().fr_io_remove_positives(
            _p(self.values), _p(self.offsets), _p(self.alive), _p(pos.values), _p(pos.offsets), len(self),
            _p(lens), ctypes.byref(total), _threads()), "fr_io_remove_positives")
        self._all_alive = False
        return lens


def eval_candidates(users, pos_lists, neg: RaggedIds):
    """EvalByUserDataloader candidates (utils/dataloader.py:228-302): per user, ``items = pos + neg``
    after removing each positive from the negatives in place.  Returns (users, items, lens, npos)
    as flat int64 arrays, the layout the trainer scores in one pass."""
    pos = (pos_lists if isinstance(pos_lists, RaggedIds) else RaggedIds.from_lists(pos_lists)).compact()
    users = np.asarray(users, dtype=np.int64)
    if len(users) != len(pos):
        raise ValueError(f"{len(users)} users for {len(pos)} positive rows")
    lens = neg.remove_positives(pos)
    cand_off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=cand_off[1:])
    out_users = np.empty(int(cand_off[-1]), np.int64)
    out_items = np.empty(int(cand_off[-1]), np.int64)
    native.check(native.lib().fr_io_candidates(
        _p(neg.values), _p(neg.offsets), _p(neg.alive), _p(pos.values), _p(pos.offsets), _p(users), len(lens),
        _p(cand_off), _p(out_users), _p(out_items), _threads()), "fr_io_candidates")
    return out_users, out_items, lens, np.diff(pos.offsets)
