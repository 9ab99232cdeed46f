"""Shared fixtures: the seeded 'tiny' dataset written in the reference's on-disk format and a
config resolved the way oracle/gen_golden.py resolved the reference's."""
import os
import tempfile

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_TMP = {}

BASE = {"seed": 999, "epochs": 3, "eval_step": 1, "n_cluster": 12, "neg_sample_num": 30}
# the reference has no BPRMF.yaml: its golden ran on overall.yaml (batch 1024, lazy eval path)
EXTRA = {"BPRMF": {"reg_weight": 0.1, "train_batch_size": 1024, "graph_inference_fast": False}, "CIKM_Model": {"attention_probs_dropout_prob": 0.0}}


def tiny_dir():
    if "tiny" not in _TMP:
        from FoodRec.utils.synthetic import make_synthetic, write_reference_format
        tmp = tempfile.mkdtemp(prefix="frtiny_")
        write_reference_format(make_synthetic("tiny", 0), tmp + "/", "Tiny")
        _TMP["tiny"] = tmp
    return _TMP["tiny"]


def tiny_config(model, use_gpu, mg=False, **over):
    from FoodRec.utils.configurator import Config
    tmp = tiny_dir()
    cd = dict(BASE)
    cd.update(EXTRA.get(model, {}))
    cd.update({"data_path": tmp + "/", "log_root": tmp + "/log/", "ckp_root": tmp + "/ckp/", "use_gpu": use_gpu})
    cd.update(over)
    cfg = Config(model, "Tiny", cd, mg)
    root = tmp + "/Tiny/processed_dataset/"
    cfg["interaction_data_path"] = root
    cfg["graph_data_path"] = root + "graph_edge/"
    cfg["ingre_data_path"] = root
    for k in cfg["hyper_parameters"]:
        if isinstance(cfg[k], list):
            cfg[k] = cfg[k][0]
    return cfg


def tiny_data(cfg):
    from FoodRec.utils.dataset import FoodData
    return FoodData(cfg)


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
