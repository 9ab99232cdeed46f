"""ORACLE (test infrastructure only): pure-Python restatement of the reference's text loaders and
evaluation candidate lists, line by line as the reference reads them.

Paths under /root/reference/FoodRec.  The product path is FoodRec/utils/textio.py over the C-ABI
readers of csrc/fr_io.cpp; tests/test_textio_cpu.py compares the two on the same files.
"""
from __future__ import annotations


def load_negative_file(filename):
    """InteractionData.load_negative_file (utils/dataset.py:245-256)."""
    negative_list = []
    with open(filename, "r") as f:
        line = f.readline()
        while line is not None and line != "":
            fields = line.split("\t")
            negative_list.append([int(x) for x in fields[1:]])
            line = f.readline()
    return negative_list


def load_training_file_as_list(filename):
    """InteractionData.load_training_file_as_list (utils/dataset.py:138-155): the counter u_ grows by
    one per new list, whatever the user id."""
    u_ = 0
    lists, items = [], []
    with open(filename, "r") as f:
        line = f.readline()
        while line is not None and line != "":
            fields = line.split("\t")
            u, i = int(fields[0]), int(fields[1])
            if u_ < u:
                lists.append(items)
                items = []
                u_ += 1
            items.append(i)
            line = f.readline()
    lists.append(items)
    return lists


def load_valid_file_as_list(filename):
    """InteractionData.load_valid_file_as_list (utils/dataset.py:115-136)."""
    lists, items, user_list = [], [], []
    with open(filename, "r") as f:
        line = f.readline()
        last_u = int(line.split("\t")[0])
        u = last_u
        while line is not None and line != "":
            fields = line.split("\t")
            u, i = int(fields[0]), int(fields[1])
            if last_u < u:
                lists.append(items)
                user_list.append(last_u)
                items = []
                last_u = u
            items.append(i)
            line = f.readline()
    lists.append(items)
    user_list.append(u)
    return lists, user_list


def training_ratings(filename):
    """(u, i, float(rating)) per line, as load_training_file_as_matrix parses them
    (utils/dataset.py:158-176)."""
    out = []
    with open(filename, "r") as f:
        for line in f:
            fields = line.split("\t")
            out.append((int(fields[0]), int(fields[1]), float(fields[2])))
    return out


def eval_candidates(users, pos_lists, neg_lists):
    """EvalByUserDataloader (utils/dataloader.py:228-302): per user, each positive is removed from
    the negatives in place (list.remove, first occurrence), then items = pos + neg.  Mutates
    neg_lists like the reference."""
    out_users, out_items, lens, npos = [], [], [], []
    for idx, user in enumerate(users):
        pos, neg = pos_lists[idx], neg_lists[idx]
        for item in pos:
            if item in neg:
                neg.remove(item)
        items = pos + neg
        out_users += [user] * len(items)
        out_items += items
        lens.append(len(items))
        npos.append(len(pos))
    return out_users, out_items, lens, npos
