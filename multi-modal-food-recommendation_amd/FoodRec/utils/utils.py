"""Driver helpers with the reference's semantics (utils/utils.py:14-113)."""
from __future__ import annotations

import datetime
import importlib
import random

import numpy as np
import torch

# reference model names served by engine-native implementations when the user has not put the
# reference model file itself on the path (drop-in files always win: see get_model)
ENGINE_MODELS = {
    "lightgcn": ("FoodRec.models.lightgcn", "LightGCN"),
    "bprmf": ("FoodRec.models.bprmf", "BPRMF"),
    "cikm_model": ("FoodRec.models.healthrec", "HealthRec"),
    "healthrec": ("FoodRec.models.healthrec", "HealthRec"),
    "pricai_modelx": ("FoodRec.models.clussl", "CLUSSL"),
    "clussl": ("FoodRec.models.clussl", "CLUSSL"),
    "lightgcn_id": ("FoodRec.models.lightgcn_id", "LightGCN_ID"),
    "schgn": ("FoodRec.models.schgn", "SCHGN"),
}


def get_local_time() -> str:
    return datetime.datetime.now().strftime("%b-%d-%Y-%H-%M-%S")


def get_model(model_name: str):
    """Resolve a model class by name (utils/utils.py:27-40).

    Order: ``models.<name.lower()>`` on sys.path (the reference's namespace-package lookup, so
    unchanged reference model files drop in), then the engine-native implementations.
    """
    mod_name = model_name.lower()
    try:
        if importlib.util.find_spec("models." + mod_name) is not None:
            module = importlib.import_module("models." + mod_name)
            if hasattr(module, model_name):
                return getattr(module, model_name)
    except (ModuleNotFoundError, ValueError):
        pass
    if mod_name in ENGINE_MODELS:
        path, cls = ENGINE_MODELS[mod_name]
        return getattr(importlib.import_module(path), cls)
    module = importlib.import_module("FoodRec.models." + mod_name)
    return getattr(module, model_name)


def get_trainer():
    return getattr(importlib.import_module("FoodRec.common.trainer"), "Trainer")


def init_seed(seed):
    """random / np.random / torch (+cuda) seeding in the reference's order (:47-53)."""
    random.seed(seed)
    np.random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    torch.manual_seed(seed)


def early_stopping(value, best, cur_step, max_step, bigger=True):
    """(:56-97) -> (best, cur_step, stop_flag, update_flag)."""
    improved = value > best if bigger else value < best
    if improved:
        return value, 0, False, True
    cur_step += 1
    return best, cur_step, cur_step > max_step, False


def dict2str(result_dict) -> str:
    return "".join(f"{k}: {v:.04f}    " for k, v in result_dict.items())


def get_neg_ingre(ingre_set, ingre_size):
    """utils/utils.py:186-190: an ingredient id uniform in [0, ingre_size) not in ``ingre_set``,
    by rejection on Python's random.randint."""
    ingre_id = random.randint(0, ingre_size - 1)
    while ingre_id in ingre_set:
        ingre_id = random.randint(0, ingre_size - 1)
    return ingre_id
