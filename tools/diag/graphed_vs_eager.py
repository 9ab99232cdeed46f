"""Diagnose: HealthRec tiny, B=32, 2 epochs under (graph, lazy rows, history ring) variants."""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "..", "multi-modal-food-recommendation_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import numpy as np
import torch
from helpers import tiny_config, tiny_data
from FoodRec.common.trainer import Trainer
from FoodRec.engine.sampler import TripleSampler
from FoodRec.utils.utils import get_model, init_seed

B = int(os.environ.get("B", "32"))
torch.use_deterministic_algorithms(os.environ.get("DET", "1") == "1")
for graphed, lazy, cap, warm in [(False, False, 8192, 2), (False, False, 8192, 2), (False, True, 8192, 2),
                                 (False, True, 7, 2), (True, False, 8192, 2), (True, True, 8192, 2),
                                 (True, True, 7, 2)]:
    cfg = tiny_config("CIKM_Model", True, train_batch_size=B, cuda_graph=graphed, cuda_graph_warmup=warm,
                      lazy_row_adam=lazy, deterministic=os.environ.get('DET', '1') == '1')
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model)
    tr.optimizer.hist_cap = cap
    sampler = TripleSampler(data, B, cfg["device"])
    losses = [tr._train_epoch(sampler, e)[0] for e in range(2)]
    print(f"graph={graphed} lazy={lazy} cap={cap} warm={warm}:", np.array(losses).round(5).tolist(), flush=True)
