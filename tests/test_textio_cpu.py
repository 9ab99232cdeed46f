"""Native text readers (csrc/fr_io.cpp via FoodRec/utils/textio.py) against the pure-Python
restatement of the reference loaders (oracle/textio.py): same lists on the same files, the same
errors on malformed fields, and the evaluation candidates' in-place positive removal."""
import os

import numpy as np
import pytest

from oracle import textio as ref
from FoodRec.utils import textio
from FoodRec.utils.dataset import _group_training, _group_valid

THREADS = (1, 3, 7)


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_bytes(text.encode())
    return str(p)


@pytest.fixture(params=THREADS)
def threads(request, monkeypatch):
    monkeypatch.setenv("FR_IO_THREADS", str(request.param))
    return request.param


def _random_negative_text(rng, users=200):
    lines = []
    for u in range(users):
        k = int(rng.integers(0, 40))
        ids = rng.integers(0, 5000, size=k).tolist()
        sep = "\t".join(str(x) for x in ids)
        lines.append(f"({u},{int(rng.integers(0, 5000))})" + ("\t" + sep if k else ""))
    return "\n".join(lines) + "\n"


def test_negatives_match_reference_loader(tmp_path, threads):
    rng = np.random.default_rng(threads)
    text = _random_negative_text(rng)
    # reference-compatible variants: CRLF line, padded fields, signs, underscores, no final newline
    text += "(200,1)\t 12\t+7\t3_4\r\n(201,2)\n(202,3)\t-5\t0009"
    path = _write(tmp_path, "data.test.negative", text)
    got = textio.read_negatives(path)
    want = ref.load_negative_file(path)
    assert len(got) == len(want)
    assert [got[u] for u in range(len(got))] == want
    assert got[-1] == [-5, 9] and got[201] == [] and got[200] == [12, 7, 34]
    assert list(got.lengths()) == [len(x) for x in want]


@pytest.mark.parametrize("bad", ["(0,1)\t1\t\n", "(0,1)\t1\tx\n", "(0,1)\t1\t\t2\n", "(0,1)\t1.5\n", "(0,1)\t_1\n"])
def test_negatives_malformed_field_raises_like_int(tmp_path, bad):
    path = _write(tmp_path, "bad.negative", "(0,0)\t1\t2\n" + bad)
    with pytest.raises(ValueError):
        ref.load_negative_file(path)
    with pytest.raises(ValueError, match="line 2"):
        textio.read_negatives(path)


def test_missing_file_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        textio.read_negatives(str(tmp_path / "absent.negative"))


def _rating_text(users, per_user, rng):
    lines = []
    for u in users:
        for _ in range(per_user(u)):
            lines.append(f"{u}\t{int(rng.integers(0, 900))}\t{float(rng.integers(0, 5))}\t{int(rng.integers(1e9))}")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("users", [list(range(50)), [0, 1, 3, 4, 9, 10], [2, 3, 5], [0, 0, 1, 1, 4]])
def test_rating_lists_match_reference_grouping(tmp_path, threads, users):
    rng = np.random.default_rng(len(users))
    text = _rating_text(sorted(set(users)), lambda u: 1 + (u * 7) % 5, rng)
    path = _write(tmp_path, "data.test.rating", text)
    pairs, rating = textio.read_ratings(path, with_rating=True)
    want_r = ref.training_ratings(path)
    assert pairs.tolist() == [[u, i] for u, i, _ in want_r]
    assert rating.tolist() == [r for _, _, r in want_r]
    assert list(_group_training(pairs)) == ref.load_training_file_as_list(path)
    got_lists, got_users = _group_valid(pairs)
    want_lists, want_users = ref.load_valid_file_as_list(path)
    assert list(got_lists) == want_lists and got_users == want_users


def test_valid_grouping_non_monotone_users(tmp_path):
    # a user id lower than the current list's user joins the current list (running maximum)
    path = _write(tmp_path, "data.valid.rating", "3\t1\t1\n3\t2\t1\n1\t5\t1\n4\t6\t1\n2\t7\t1\n")
    pairs, _ = textio.read_ratings(path, with_rating=False)
    got_lists, got_users = _group_valid(pairs)
    want_lists, want_users = ref.load_valid_file_as_list(path)
    assert list(got_lists) == want_lists and got_users == want_users
    assert list(_group_training(pairs)) == ref.load_training_file_as_list(path)


def test_training_rating_needs_third_field(tmp_path):
    path = _write(tmp_path, "data.train.rating", "0\t1\t1\n0\t2\n")
    with pytest.raises(IndexError):
        textio.read_ratings(path, with_rating=True)
    pairs, _ = textio.read_ratings(path, with_rating=False)
    assert pairs.tolist() == [[0, 1], [0, 2]]


def test_eval_candidates_match_reference_and_persist(tmp_path):
    rng = np.random.default_rng(5)
    n_users = 300
    neg_lists = [rng.integers(0, 60, size=int(rng.integers(0, 30))).tolist() for _ in range(n_users)]
    pos_lists = [rng.integers(0, 60, size=int(rng.integers(1, 6))).tolist() for _ in range(n_users)]
    pos_lists[0] = [7, 7, 7]          # duplicate positives remove successive occurrences
    neg_lists[0] = [7, 1, 7, 2]
    users = list(range(100, 100 + n_users))
    neg = textio.RaggedIds.from_lists(neg_lists)
    ref_neg = [list(x) for x in neg_lists]
    for _ in range(2):  # the removal persists into the next evaluation, as in the reference
        got = textio.eval_candidates(users, pos_lists, neg)
        want = ref.eval_candidates(users, pos_lists, ref_neg)
        for g, w in zip(got, want):
            assert np.asarray(g).tolist() == list(w)
        assert list(neg) == ref_neg
    assert neg[0] == [1, 2]


def test_dataset_lists_are_reference_lists(tmp_path):
    """FoodData on the reference's on-disk format: per-user lists equal the reference loaders'."""
    from helpers import tiny_config, tiny_data
    cfg = tiny_config("LightGCN", False)
    data = tiny_data(cfg)
    ip = cfg["interaction_data_path"]
    assert [data.testNegatives[u] for u in range(len(data.testNegatives))] == \
        ref.load_negative_file(ip + "data.test.negative")
    assert list(data.validNegatives) == ref.load_negative_file(ip + "data.valid.negative")
    assert list(data.testRatings) == ref.load_training_file_as_list(ip + "data.test.rating")
    assert list(data.trainList) == ref.load_training_file_as_list(ip + "data.train.rating")
    lists, users = ref.load_valid_file_as_list(ip + "data.valid.rating")
    assert list(data.validRatings) == lists and data.valid_users == users
