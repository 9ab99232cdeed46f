"""Driver: config -> data -> hyper-parameter grid -> model -> Trainer.fit (utils/quick_start.py:17-106).

Same seed/RNG order as the reference: init_seed(seed) immediately before model construction,
so parameter init and the sampler stream match the reference's for the same seed.
"""
from __future__ import annotations

import os
import platform
from itertools import product
from logging import getLogger

from FoodRec.utils.configurator import Config
from FoodRec.utils.dataset import FoodData
from FoodRec.utils.logger import init_logger
from FoodRec.utils.utils import dict2str, get_model, get_trainer, init_seed


def quick_start(model, dataset, config_dict, save_model=True, mg=False):
    config = Config(model, dataset, config_dict, mg)
    config["interaction_data_path"] = config["data_path"] + dataset + "/processed_dataset/"
    config["graph_data_path"] = config["data_path"] + dataset + "/processed_dataset/graph_edge/"
    config["ingre_data_path"] = config["data_path"] + dataset + "/processed_dataset/"
    init_logger(config)
    logger = getLogger()
    logger.info("██Server: \t" + platform.node())
    logger.info("██Dir: \t" + os.getcwd() + "\n")
    logger.info(config)

    data = FoodData(config)
    logger.info(str(data))

    hyper_ret = []
    val_metric = config["valid_metric"]
    best_test_value, best_test_idx = 0.0, 0
    logger.info("\n\n=================================\n\n")
    if "seed" not in config["hyper_parameters"]:
        config["hyper_parameters"] = ["seed"] + config["hyper_parameters"]
    hyper_ls = [config[i] if isinstance(config[i], list) else [config[i]] for i in config["hyper_parameters"]]
    combos = list(product(*hyper_ls))
    for idx, hyper_tuple in enumerate(combos):
        for j, k in zip(config["hyper_parameters"], hyper_tuple):
            config[j] = k
        init_seed(config["seed"])
        logger.info("========={}/{}: Parameters:{}={}=======".format(idx + 1, len(combos),
                                                                        config["hyper_parameters"], hyper_tuple))
        net = get_model(config["model"])(config, data).to(config["device"])
        logger.info(net)
        trainer = get_trainer()(config, net, mg)
        _, best_valid_result, best_test_upon_valid = trainer.fit(data, hyper_tuple=hyper_tuple, saved=save_model)
        hyper_ret.append((hyper_tuple, best_valid_result, best_test_upon_valid))
        if best_test_upon_valid[val_metric] > best_test_value:
            best_test_value, best_test_idx = best_test_upon_valid[val_metric], idx
        logger.info("best valid result: {}".format(dict2str(best_valid_result)))
        logger.info("test result: {}".format(dict2str(best_test_upon_valid)))
    logger.info("\n============All Over=====================")
    for (p, k, v) in hyper_ret:
        logger.info("Parameters: {}={},\n best valid: {},\n best test: {}".format(
            config["hyper_parameters"], p, dict2str(k), dict2str(v)))
    if hyper_ret:
        p, k, v = hyper_ret[best_test_idx]
        logger.info("\n\n█████████████ BEST ████████████████")
        logger.info("\tParameters: {}={},\nValid: {},\nTest: {}\n\n".format(
            config["hyper_parameters"], p, dict2str(k), dict2str(v)))
    return hyper_ret
