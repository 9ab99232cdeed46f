"""FoodData: the reference's dataset object (utils/dataset.py:11-370), loaded vectorised.

Exposes the same attribute names the reference models and trainer read (SURVEY 8(b) "Dataset
attributes models read") with the same values and orders, plus array views the engine uses:

  train_pairs [E,2] int64   (u, i) in file order == trainMatrix.keys() order (dok insertion)
  excl_train_ptr/items      per-user sorted train items (CSR)       -> negative-sampler exclusions
  excl_vt_ptr/items         per-user sorted valid+test items (CSR)

Pickled inputs (inter_coo_matrix.pkl, health dicts) are read with a restricted unpickler that
only reconstructs numpy arrays, scipy COO matrices and plain containers.
"""
from __future__ import annotations

import io
import os
import pickle
from collections import defaultdict

import numpy as np
import scipy.sparse as sp

from .textio import RaggedIds, read_negatives, read_ratings

_SAFE = {
    ("builtins", "dict"), ("builtins", "list"), ("builtins", "set"), ("builtins", "tuple"),
    ("builtins", "int"), ("builtins", "float"), ("builtins", "bool"), ("builtins", "frozenset"),
    ("collections", "OrderedDict"), ("collections", "defaultdict"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "scalar"), ("numpy", "int64"), ("numpy", "float64"),
    ("scipy.sparse._coo", "coo_matrix"), ("scipy.sparse.coo", "coo_matrix"),
    ("scipy.sparse._arrays", "coo_array"), ("scipy.sparse._coo", "coo_array"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _SAFE:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a data pickle")


def safe_pickle_load(path: str):
    with open(path, "rb") as f:
        return _SafeUnpickler(io.BytesIO(f.read())).load()


def _read_pairs(path: str, with_rating: bool = False):
    """``u\ti\trating`` lines -> ([n,2] int64 (u, i), [n] float64 rating or None); native parallel
    reader (utils/textio.py, csrc/fr_io.cpp)."""
    return read_ratings(path, with_rating)


def _read_negatives(path: str) -> RaggedIds:
    return read_negatives(path)


def _as_ragged(x) -> RaggedIds:
    if isinstance(x, RaggedIds):
        return x
    if isinstance(x, np.ndarray):
        return RaggedIds.from_dense(x)
    return RaggedIds.from_lists(x)


def _csr_sets(users: np.ndarray, items: np.ndarray, n_users: int):
    """per-user sorted unique item lists as (ptr [n_users+1], items)."""
    key = np.unique(users.astype(np.int64) * (np.int64(items.max(initial=0)) + 1) + items)
    m = np.int64(items.max(initial=0)) + 1
    u, it = key // m, key % m
    ptr = np.zeros(n_users + 1, np.int64)
    np.cumsum(np.bincount(u, minlength=n_users), out=ptr[1:])
    return ptr, it.astype(np.int64)


def _group_training(pairs: np.ndarray) -> RaggedIds:
    """load_training_file_as_list (reference utils/dataset.py:138-155): a new list starts at a line
    whose user exceeds the counter u_, and u_ then grows by ONE (not to that user), so a user id gap
    inserts empty lists.  Files whose users run 0, 1, 2, ... take the vectorised path."""
    n = len(pairs)
    if n == 0:
        return RaggedIds(np.zeros(0, np.int64), np.zeros(2, np.int64))  # [[]]
    u = pairs[:, 0]
    step = np.diff(u)
    if u[0] == 0 and ((step == 0) | (step == 1)).all():
        starts = np.flatnonzero(step) + 1
    else:
        starts, u_ = [], 0
        for k, uk in enumerate(u.tolist()):
            if u_ < uk:
                starts.append(k)
                u_ += 1
        starts = np.asarray(starts, np.int64)
    offsets = np.concatenate([[0], starts, [n]]).astype(np.int64)
    return RaggedIds(pairs[:, 1], offsets)


def _group_valid(pairs: np.ndarray):
    """load_valid_file_as_list (reference utils/dataset.py:115-136): a new list starts when the user
    exceeds the current list's user (a running maximum); users = each list's user, except that the
    last entry is the final line's user.  (An empty file, where the reference's int('') raises, gives
    no lists.)"""
    n = len(pairs)
    if n == 0:
        return RaggedIds(np.zeros(0, np.int64), np.zeros(1, np.int64)), []
    u = pairs[:, 0]
    prev_max = np.maximum.accumulate(u)
    starts = np.concatenate([[0], np.flatnonzero(u[1:] > prev_max[:-1]) + 1]).astype(np.int64)
    users = u[starts].copy()
    users[-1] = u[-1]
    return RaggedIds(pairs[:, 1], np.append(starts, n)), users.tolist()


class _TrainMatrix:
    """Stands in for the reference's dok trainMatrix: shape + keys() in insertion order."""

    def __init__(self, pairs: np.ndarray, shape):
        self._pairs = pairs
        self.shape = shape

    def keys(self):
        return [tuple(x) for x in self._pairs.tolist()]

    def __len__(self):
        return len(self._pairs)


class FoodData:
    def __init__(self, args_config=None, _arrays=None):
        self.args_config = args_config
        if _arrays is None:
            _arrays = self._read_files(args_config)
        self._build(_arrays, args_config)

    # ----------------------------------------------------------------------------- input
    @staticmethod
    def _read_files(cfg) -> dict:
        ip = cfg["interaction_data_path"]
        gp = cfg["graph_data_path"]
        ingre_path = cfg["ingre_data_path"] or ip
        a = {}
        tr, rating = _read_pairs(ip + "data.train.rating", with_rating=True)
        # dok assignment keeps rating > 0 rows, first occurrence position (dataset.py:167-176)
        a["train_raw"] = tr
        a["train_rating_pos"] = rating > 0
        a["valid"] = _read_pairs(ip + "data.valid.rating")[0]
        a["test"] = _read_pairs(ip + "data.test.rating")[0]
        a["valid_neg"] = _read_negatives(ip + "data.valid.negative")
        a["test_neg"] = _read_negatives(ip + "data.test.negative")
        a["image"] = np.load(ip + "data_image_features_float.npy")
        a["text"] = np.load(ingre_path + "data_text_features_t5.npy")
        a["ingre_num"] = np.loadtxt(ingre_path + "data_id_ingre_num_file", dtype=np.int64, ndmin=2)[:, 1]
        a["ingre_code"] = np.load(ingre_path + "data_ingre_code_file.npy")
        coo_path = (ip if ip != gp else gp) + "inter_coo_matrix.pkl"
        a["coo"] = safe_pickle_load(coo_path) if os.path.exists(coo_path) else None
        ri_dir = ingre_path if cfg["small_ingre"] else gp
        if cfg["load_RecipeIngre_graph"]:
            a["ri"] = np.loadtxt(ri_dir + "ri_graph.txt", dtype=np.int64, ndmin=2)
        if cfg["load_ImageCluster_graph"]:
            a["image_cluster"] = np.loadtxt(ip + "cluster/image_cluster_edge.txt", ndmin=2)
        if cfg["load_TextCluster_graph"]:
            a["text_cluster"] = np.loadtxt(ip + "cluster/text_cluster_edge.txt", ndmin=2)
        if cfg["use_health_level_multi_hot"]:
            a["health"] = safe_pickle_load(gp + "recipe_health_level_multi_hot_dict.pkl")
        for flag, key, name in (("load_UserRecipe_graph", "ur", "ur_graph.txt"),
                                ("load_RecipeRecipe_graph", "rr", "rr_graph.txt"),
                                ("load_IngreIngre_graph", "ii", "ii_graph.txt"),
                                ("load_RecipeCalories_graph", "rc", "rc_graph.txt"),
                                ("load_RecipeHealth_graph", "rh", "rh_graph.txt")):
            if cfg[flag]:
                a[key] = np.loadtxt(gp + name, dtype=np.int64, ndmin=2)
        if cfg["use_cal_level"]:
            a["cal_level"] = safe_pickle_load(gp + "recipe_cal_level_dict.pkl")
        if cfg["use_health_level"]:
            a["health_level"] = safe_pickle_load(gp + "recipe_health_level_dict.pkl")
        return a

    @classmethod
    def from_synthetic(cls, ds, args_config=None, flags=("ri", "image_cluster", "text_cluster", "health")):
        """Build directly from a FoodRec.utils.synthetic.SyntheticFood (no files)."""
        import scipy.sparse as sps
        a = {"train_raw": ds.train, "train_rating_pos": np.ones(len(ds.train), bool),
             "valid": ds.valid, "test": ds.test,
             "valid_neg": ds.valid_neg, "test_neg": ds.test_neg,
             "image": ds.image, "text": ds.text, "ingre_num": ds.ingre_num, "ingre_code": ds.ingre_code,
             "coo": sps.coo_matrix((np.ones(len(ds.train)), (ds.train[:, 0], ds.train[:, 1])),
                                   shape=(ds.n_users, ds.n_items))}
        if "ri" in flags:
            ri = np.stack([np.repeat(np.arange(ds.n_items), 20), ds.ingre_code.reshape(-1)], 1)
            a["ri"] = ri[ri[:, 1] != ds.n_ingredients]
        if "image_cluster" in flags:
            a["image_cluster"] = ds.image_cluster.astype(np.float64)
        if "text_cluster" in flags:
            a["text_cluster"] = ds.text_cluster.astype(np.float64)
        if "health" in flags:
            a["health"] = {i: row for i, row in enumerate(ds.health.tolist())}
        if "schgn" in flags:  # SCHGN's user-recipe and recipe-calorie graphs + calorie levels
            cal = ds.extra["cal_level"]
            a["ur"] = np.asarray(ds.train, np.int64)
            a["rc"] = np.stack([np.arange(ds.n_items, dtype=np.int64), cal], 1)
            a["cal_level"] = {i: int(v) for i, v in enumerate(cal.tolist())}
        return cls(args_config, _arrays=a)

    # ----------------------------------------------------------------------------- build
    def _build(self, a: dict, cfg):
        raw = a["train_raw"][a["train_rating_pos"]]
        # first occurrence of each (u,i), in file order (dok insertion order)
        ncol = np.int64(raw[:, 1].max(initial=0)) + 1
        _, first = np.unique(raw[:, 0] * ncol + raw[:, 1], return_index=True)
        self.train_pairs = raw[np.sort(first)]
        tr_all, va_all, te_all = a["train_raw"], a["valid"], a["test"]
        self.num_users = int(tr_all[:, 0].max()) + 1
        self.num_items = int(tr_all[:, 1].max()) + 1
        self.trainMatrix = _TrainMatrix(self.train_pairs, (self.num_users, self.num_items))
        self._tr_all, self._va_all, self._te_all = tr_all, va_all, te_all
        # per-user lists as RaggedIds (the reference's list-of-lists protocol over flat arrays)
        self.testRatings = _group_training(te_all)
        self.testNegatives = _as_ragged(a["test_neg"])
        self.validRatings, self.valid_users = _group_valid(va_all)
        self.validNegatives = _as_ragged(a["valid_neg"])
        assert len(self.testRatings) == len(self.testNegatives)
        assert len(self.validRatings) == len(self.validNegatives)
        train_items = set(tr_all[:, 1].tolist())
        vt_items = set(va_all[:, 1].tolist()) | set(te_all[:, 1].tolist())
        self.cold_list = list(vt_items - train_items)
        self.cold_num = len(self.cold_list)
        self.train_item_list = list(train_items)

        nu_all = int(max(tr_all[:, 0].max(), va_all[:, 0].max(initial=0), te_all[:, 0].max())) + 1
        self.train_data = tr_all.copy()
        self.valid_data = va_all.copy()
        self.test_data = te_all.copy()
        for d in (self.train_data, self.valid_data, self.test_data):
            d[:, 1] += nu_all

        self.embImage = a["image"]
        self.image_size = self.embImage.shape[1]
        self.embText = a["text"]
        self.text_size = self.embText.shape[1]
        self.ingredientNum = [int(x) for x in np.asarray(a["ingre_num"]).tolist()]
        self.ingredientCodeDict = np.asarray(a["ingre_code"])
        self.num_ingredients = int(np.max(self.ingredientCodeDict))

        cat = np.concatenate([self.train_data, self.valid_data, self.test_data])
        self.user_range = (int(cat[:, 0].min()), int(cat[:, 0].max()))
        self.n_users = self.user_range[1] - self.user_range[0] + 1
        self.item_range = (int(cat[:, 1].min()), int(cat[:, 1].max()))
        self.n_items = self.item_range[1] - self.item_range[0] + 1
        self.n_train, self.n_valid, self.n_test = len(self.train_data), len(self.valid_data), len(self.test_data)
        self.inter_num = self.n_train + self.n_valid + self.n_test

        coo = a.get("coo")
        if coo is None:
            coo = sp.coo_matrix((np.ones(len(self.train_pairs)), (self.train_pairs[:, 0], self.train_pairs[:, 1])),
                                shape=(self.num_users, self.n_items))
        self.train_coo_matrix = sp.coo_matrix(coo).astype(np.float32)

        # GraphData part (dataset.py:273-348)
        self.num_health_level = 0
        self.num_calories_level = 0
        self.n_relations = 0
        for key, attr in (("ur", "uRecipe_triples"), ("rr", "rRecipe_triples"), ("ri", "rIngre_triples"),
                          ("ii", "iIngre_triples"), ("rc", "rCalories_triples"), ("rh", "rHealth_triples"),
                          ("image_cluster", "image_cluster_triples"), ("text_cluster", "text_cluster_triples")):
            if key in a:
                setattr(self, attr, a[key])
                self.n_relations += 1
        if "rc" in a:
            self.num_calories_level = int(a["rc"][:, 1].max()) + 1
        if "rh" in a:
            self.num_health_level = int(a["rh"][:, 1].max()) + 1
        if "health" in a:
            self.health_level_multi_hot = a["health"]
        if "cal_level" in a:
            self.cal_level = a["cal_level"]
        if "health_level" in a:
            self.health_level = a["health_level"]

        # engine views: exclusion sets of the negative sampler (dataloader.py:145-151)
        self.excl_train_ptr, self.excl_train_items = _csr_sets(tr_all[:, 0], tr_all[:, 1], self.num_users)
        vt = np.concatenate([va_all, te_all])
        vt = vt[vt[:, 0] < self.num_users]
        self.excl_vt_ptr, self.excl_vt_items = _csr_sets(vt[:, 0], vt[:, 1], self.num_users)

    # --- per-user Python structures of the reference API, built on first use (the engine's
    # sampler and evaluator use the array views instead)
    @property
    def trainList(self):
        if "_trainList" not in self.__dict__:
            self._trainList = _group_training(self._tr_all)
        return self._trainList

    @property
    def validTestRatings(self):
        if "_vtr" not in self.__dict__:
            vtr = {u: set() for u in range(self.num_users)}
            for u, i in np.concatenate([self._va_all, self._te_all]).tolist():
                vtr.setdefault(u, set()).add(i)
            self._vtr = vtr
        return self._vtr

    @property
    def train_user_dict(self):
        if "_tud" not in self.__dict__:
            self._tud = self._user_dict(self.train_data)
        return self._tud

    @property
    def valid_user_dict(self):
        if "_vud" not in self.__dict__:
            self._vud = self._user_dict(self.valid_data)
        return self._vud

    @property
    def test_user_dict(self):
        if "_teud" not in self.__dict__:
            self._teud = self._user_dict(self.test_data)
        return self._teud

    @staticmethod
    def _user_dict(inter):
        d = defaultdict(list)
        for u, i in inter.tolist():
            d[u].append(i)
        return d

    def health_matrix(self) -> np.ndarray:
        """[n_items, bits] float32 of health_level_multi_hot (items without an entry -> 0)."""
        hm = self.health_level_multi_hot
        bits = len(hm[next(iter(hm))])
        out = np.zeros((self.n_items, bits), np.float32)
        for i, row in hm.items():
            if 0 <= int(i) < self.n_items:
                out[int(i)] = row
        return out

    def __str__(self):
        info = [str(self.args_config["dataset"]) if self.args_config is not None else "FoodData",
                f"The number of users: {self.n_users}",
                f"Average actions of users: {self.inter_num / self.n_users}",
                f"The number of items: {self.n_items}",
                f"Average actions of items: {self.inter_num / self.n_items}",
                f"The number of inters: {self.inter_num}",
                f"The sparsity of the dataset: {(1 - self.inter_num / self.n_users / self.n_items) * 100}%"]
        return "\n".join(info)
