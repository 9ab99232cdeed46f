"""Seeded synthetic datasets in the reference's on-disk format.

The processed Allrecipes / Foodcom datasets are not available offline
(reference README.md:10), so every fixture, test and bench input is generated
here.  The generator reproduces the *shapes and file formats* that
`dataset_process/allrecipes_process.ipynb` writes and that
`FoodRec/utils/dataset.py` reads:

========================================  ===========================================
file                                      format (reader in reference utils/dataset.py)
========================================  ===========================================
data.{train,valid,test}.rating            ``u\\ti\\trating`` users contiguous (:137-176)
data.{valid,test}.negative                ``(u,i)\\tn1\\tn2...`` one line per user (:245)
data_image_features_float.npy             [I, 2048] float64 (:45)
data_text_features_t5.npy                 [I, 512] float64 (:48)
data_ingre_code_file.npy                  [I, 20] int64, pad = NI (:52-53)
data_id_ingre_num_file                    ``i\\tnum`` (:207-213)
ri_graph.txt (+ graph_edge/ri_graph.txt)  ``item ingre`` (:294, notebook cell 23)
cluster/{image,text}_cluster_edge.txt     ``item cluster`` (:330-337)
inter_coo_matrix.pkl                      pickled scipy coo U x I (:56-60, cell 21)
graph_edge/recipe_health_level_...pkl     {item: [bits]} (:316-317, cell 28)
========================================  ===========================================

Shapes: Allrecipes U=68,768 I=45,630 train~677k, NI=19,987,
7 health bits; Foodcom U=7,596 I=29,943 train~192k, NI=4,963, 6 health bits.
"""
from __future__ import annotations

import os
import pickle
from dataclasses import dataclass, field

import numpy as np

SHAPES = {
    # name: users, items, mean train per user, valid-user fraction, mean valid, mean test,
    #       ingredients, clusters, image dim, text dim, health bits
    "tiny": dict(U=120, I=90, train=6.0, vfrac=0.5, valid=2.0, test=2.0, NI=40, C=12,
                 img=32, txt=16, health=7, neg=30),
    "small": dict(U=2000, I=1500, train=10.0, vfrac=0.45, valid=3.0, test=3.0, NI=400, C=60,
                  img=64, txt=32, health=7, neg=100),
    "foodcom": dict(U=7596, I=29943, train=25.26, vfrac=0.635, valid=7.29, test=12.66,
                    NI=4963, C=2000, img=2048, txt=512, health=6, neg=500),
    "allrecipes": dict(U=68768, I=45630, train=9.84, vfrac=0.426, valid=4.55, test=4.12,
                       NI=19987, C=2000, img=2048, txt=512, health=7, neg=500),
}


@dataclass
class SyntheticFood:
    """In-memory synthetic dataset (arrays only; no Python per-row objects)."""
    name: str
    n_users: int
    n_items: int
    n_ingredients: int
    n_cluster: int
    train: np.ndarray          # [E,2] int64 (u, i), users contiguous, file order
    valid: np.ndarray          # [Ev,2]
    test: np.ndarray           # [Et,2]
    valid_users: np.ndarray    # [Vu]
    valid_neg: np.ndarray      # [Vu, neg] int64
    test_neg: np.ndarray       # [U, neg] int64
    ingre_code: np.ndarray     # [I,20] int64, pad = NI
    ingre_num: np.ndarray      # [I] int64
    image: np.ndarray          # [I, img] float64
    text: np.ndarray           # [I, txt] float64
    image_cluster: np.ndarray  # [Ec,2] (item, cluster)
    text_cluster: np.ndarray   # [Ec,2]
    health: np.ndarray         # [I, bits] int64 0/1
    extra: dict = field(default_factory=dict)


def _popularity(n_items: int, rng: np.random.Generator, s: float = 0.8) -> np.ndarray:
    # popularity ~ (rank + 10)^-s over a random rank permutation
    rank = rng.permutation(n_items)
    p = (rank + 10.0) ** (-s)
    return p / p.sum()


def make_synthetic(shape: str = "tiny", seed: int = 0, negatives: bool = True, **overrides) -> SyntheticFood:
    """``negatives=False`` skips the 500-per-user evaluation candidate lists (training-only
    inputs, e.g. bench.py) — they are the slowest part to generate at Allrecipes shape."""
    cfg = dict(SHAPES[shape])
    cfg.update(overrides)
    rng = np.random.default_rng(seed)
    U, I, NI, C = cfg["U"], cfg["I"], cfg["NI"], cfg["C"]
    pop = _popularity(I, rng)

    is_valid_user = rng.random(U) < cfg["vfrac"]
    n_tr = 1 + rng.poisson(max(cfg["train"] - 1.0, 0.1), U)
    n_te = 1 + rng.poisson(max(cfg["test"] - 1.0, 0.1), U)
    n_va = np.where(is_valid_user, 1 + rng.poisson(max(cfg["valid"] - 1.0, 0.1), U), 0)
    want = n_tr + n_te + n_va
    # oversample then de-duplicate per user
    draw = (want * 1.3 + 4).astype(np.int64)
    users = np.repeat(np.arange(U, dtype=np.int64), draw)
    items = rng.choice(I, size=users.shape[0], p=pop).astype(np.int64)
    key = np.unique(users * I + items)
    # shuffle within user: random sort key then stable sort by user
    order = np.lexsort((rng.random(key.shape[0]), key // I))
    key = key[order]
    u_all, i_all = key // I, key % I
    starts = np.searchsorted(u_all, np.arange(U))
    ends = np.searchsorted(u_all, np.arange(U), side="right")
    have = ends - starts
    pos_in_user = np.arange(key.shape[0]) - np.repeat(starts, have)
    # role assignment: first n_tr train, then n_te test, then n_va valid (truncated to what exists)
    tr_k = np.minimum(n_tr, np.maximum(have - 1, 1))
    te_k = np.minimum(n_te, np.maximum(have - tr_k, 0))
    va_k = np.minimum(n_va, np.maximum(have - tr_k - te_k, 0))
    tr_k_r, te_k_r, va_k_r = (np.repeat(x, have) for x in (tr_k, te_k, va_k))
    role = np.full(key.shape[0], -1)
    role[pos_in_user < tr_k_r] = 0
    role[(pos_in_user >= tr_k_r) & (pos_in_user < tr_k_r + te_k_r)] = 1
    role[(pos_in_user >= tr_k_r + te_k_r) & (pos_in_user < tr_k_r + te_k_r + va_k_r)] = 2
    assert np.all(tr_k >= 1) and np.all(te_k >= 1), "every user needs a train and a test row"

    def _split(r):
        m = role == r
        return np.stack([u_all[m], i_all[m]], 1)

    train, test, valid = _split(0), _split(1), _split(2)
    # the reference sizes items by the id range over all splits (dataset.py:216-227) and the
    # negative sampler by max train id + 1 (dataset.py:30): make sure ids 0 and I-1 occur in train
    for must in (0, I - 1):
        if not np.any(train[:, 1] == must):
            train[0 if must == 0 else -1, 1] = must
    train = _dedupe_sorted(train, I)
    valid_users = np.unique(valid[:, 0]) if valid.shape[0] else np.zeros(0, np.int64)

    # popularity^0.7 candidate negatives (allrecipes_process.ipynb cell 15), excluding train items
    tr_count = np.bincount(train[:, 1], minlength=I).astype(np.float64)
    p07 = np.where(tr_count > 0, (tr_count / tr_count.sum()) ** 0.7, 0.0)
    p07 /= p07.sum()
    neg = cfg["neg"]
    tr_ptr = np.concatenate([[0], np.cumsum(np.bincount(train[:, 0], minlength=U))])

    train_keys = np.unique(train[:, 0] * I + train[:, 1])

    def _negatives(user_ids, chunk=4096):
        """neg distinct popularity^0.7 draws per user excluding its train items (vectorised)."""
        out = np.empty((len(user_ids), neg), np.int64)
        for c0 in range(0, len(user_ids), chunk):
            uu = np.asarray(user_ids[c0:c0 + chunk], np.int64)
            cand = rng.choice(I, size=(len(uu), 3 * neg), p=p07)
            key = uu[:, None] * I + cand
            pos = np.searchsorted(train_keys, key)
            excl = train_keys[np.minimum(pos, len(train_keys) - 1)] == key
            order = np.argsort(cand, axis=1, kind="stable")
            srt = np.take_along_axis(cand, order, 1)
            dup_s = np.zeros_like(srt, dtype=bool)
            dup_s[:, 1:] = srt[:, 1:] == srt[:, :-1]
            dup = np.empty_like(dup_s)
            np.put_along_axis(dup, order, dup_s, 1)
            ok = ~excl & ~dup
            rank = np.cumsum(ok, axis=1)
            full = rank[:, -1] >= neg
            sel = ok & (rank <= neg)
            out_rows = np.where(full)[0]
            out[c0 + out_rows] = cand[out_rows][sel[out_rows]].reshape(len(out_rows), neg)
            for r in np.where(~full)[0]:  # rare: too few distinct candidates, top up one by one
                u = int(uu[r])
                own = set(train[tr_ptr[u]:tr_ptr[u + 1], 1].tolist())
                got = list(dict.fromkeys(c for c in cand[r].tolist() if c not in own))
                while len(got) < neg:
                    c = int(rng.integers(I))
                    if c not in own and c not in got:
                        got.append(c)
                out[c0 + r] = got[:neg]
        return out

    if negatives:
        valid_neg = _negatives(valid_users)
        test_neg = _negatives(np.arange(U))
    else:
        valid_neg = np.zeros((len(valid_users), 0), np.int64)
        test_neg = np.zeros((U, 0), np.int64)

    # ingredients: 1..20 distinct per item, padded with NI (notebook cell 6)
    k = rng.integers(1, 21, size=I)
    k[rng.integers(I)] = 19  # guarantee at least one padded row -> max code == NI
    code = np.full((I, 20), NI, np.int64)
    raw = _distinct_rows(rng, I, NI, 20)
    mask = np.arange(20)[None, :] < k[:, None]
    code[mask] = raw[mask]
    image = rng.standard_normal((I, cfg["img"]))
    text = rng.standard_normal((I, cfg["txt"]))
    ne = min(6, C)
    img_c = _distinct_rows(rng, I, C, ne)
    txt_c = _distinct_rows(rng, I, C, ne)
    item_ids = np.repeat(np.arange(I, dtype=np.int64), ne)
    image_cluster = np.stack([item_ids, img_c.reshape(-1)], 1)
    text_cluster = np.stack([item_ids, txt_c.reshape(-1)], 1)
    health = (rng.random((I, cfg["health"])) < 0.35).astype(np.int64)
    # SCHGN's calorie level per recipe (0..5), from its own generator: the main stream (and the
    # goldens' dataset digest) is unchanged
    cal_level = np.random.default_rng([seed, 0xCA1]).integers(0, 6, I).astype(np.int64)
    return SyntheticFood(shape, U, I, NI, C, train, valid, test, valid_users.astype(np.int64),
                         valid_neg, test_neg, code, k.astype(np.int64), image, text,
                         image_cluster, text_cluster, health, extra={"cal_level": cal_level})


def _distinct_rows(rng, rows: int, n: int, k: int) -> np.ndarray:
    """[rows, k] int64, each row k distinct values of [0, n) in random order (vectorised)."""
    if n <= 256:
        return np.argsort(rng.random((rows, n)), axis=1)[:, :k].astype(np.int64)
    m = 2 * k + 8
    out = np.empty((rows, k), np.int64)
    cand = rng.integers(0, n, size=(rows, m))
    order = np.argsort(cand, axis=1, kind="stable")
    srt = np.take_along_axis(cand, order, 1)
    dup_s = np.zeros_like(srt, dtype=bool)
    dup_s[:, 1:] = srt[:, 1:] == srt[:, :-1]
    dup = np.empty_like(dup_s)
    np.put_along_axis(dup, order, dup_s, 1)
    ok = ~dup
    rank = np.cumsum(ok, axis=1)
    full = rank[:, -1] >= k
    rows_ok = np.where(full)[0]
    out[rows_ok] = cand[rows_ok][(ok & (rank <= k))[rows_ok]].reshape(len(rows_ok), k)
    for r in np.where(~full)[0]:
        out[r] = rng.choice(n, k, replace=False)
    return out


def _dedupe_sorted(pairs: np.ndarray, n_items: int) -> np.ndarray:
    """Drop duplicate (u,i) rows keeping first occurrence and the file order."""
    key = pairs[:, 0] * n_items + pairs[:, 1]
    _, first = np.unique(key, return_index=True)
    keep = np.sort(first)
    out = pairs[keep]
    # users must stay contiguous (file is grouped by user)
    order = np.argsort(out[:, 0], kind="stable")
    return out[order]


def write_reference_format(ds: SyntheticFood, data_path: str, dataset: str) -> str:
    """Write `ds` under ``data_path/dataset/processed_dataset/`` exactly as the
    preprocessing notebooks do.  Returns that directory."""
    root = os.path.join(data_path, dataset, "processed_dataset") + os.sep
    os.makedirs(root + "graph_edge", exist_ok=True)
    os.makedirs(root + "cluster", exist_ok=True)

    def _rating(path, pairs):
        with open(path, "w") as f:
            f.write("".join(f"{u}\t{i}\t1\n" for u, i in pairs.tolist()))

    _rating(root + "data.train.rating", ds.train)
    _rating(root + "data.valid.rating", ds.valid)
    _rating(root + "data.test.rating", ds.test)

    def _neg(path, users, negs, split):
        first = {}
        for u, i in split.tolist():
            first.setdefault(u, i)
        with open(path, "w") as f:
            for u, row in zip(users.tolist(), negs.tolist()):
                f.write(f"({u},{first.get(u, 0)})\t" + "\t".join(map(str, row)) + "\n")

    _neg(root + "data.valid.negative", ds.valid_users, ds.valid_neg, ds.valid)
    _neg(root + "data.test.negative", np.arange(ds.n_users), ds.test_neg, ds.test)
    np.save(root + "data_image_features_float.npy", ds.image)
    np.save(root + "data_text_features_t5.npy", ds.text)
    np.save(root + "data_ingre_code_file.npy", ds.ingre_code)
    with open(root + "data_id_ingre_num_file", "w") as f:
        f.write("".join(f"{i}\t{n}\n" for i, n in enumerate(ds.ingre_num.tolist())))
    ri = np.stack([np.repeat(np.arange(ds.n_items), 20), ds.ingre_code.reshape(-1)], 1)
    ri = ri[ri[:, 1] != ds.n_ingredients]
    for p in (root + "ri_graph.txt", root + "graph_edge/ri_graph.txt"):
        np.savetxt(p, ri, fmt="%d")
    np.savetxt(root + "cluster/image_cluster_edge.txt", ds.image_cluster, fmt="%d")
    np.savetxt(root + "cluster/text_cluster_edge.txt", ds.text_cluster, fmt="%d")
    import scipy.sparse as sp
    mat = sp.coo_matrix((np.ones(len(ds.train)), (ds.train[:, 0], ds.train[:, 1])),
                        shape=(ds.n_users, ds.n_items))
    with open(root + "inter_coo_matrix.pkl", "wb") as f:
        pickle.dump(mat, f)
    with open(root + "graph_edge/recipe_health_level_multi_hot_dict.pkl", "wb") as f:
        pickle.dump({i: row for i, row in enumerate(ds.health.tolist())}, f)
    # SCHGN's graphs: user-recipe (the training interactions), recipe-calorie level, level dict
    np.savetxt(root + "graph_edge/ur_graph.txt", ds.train, fmt="%d")
    cal = ds.extra["cal_level"]
    np.savetxt(root + "graph_edge/rc_graph.txt", np.stack([np.arange(ds.n_items), cal], 1), fmt="%d")
    with open(root + "graph_edge/recipe_cal_level_dict.pkl", "wb") as f:
        pickle.dump({i: int(v) for i, v in enumerate(cal.tolist())}, f)
    return root
