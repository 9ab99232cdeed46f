"""Plugin API — AbstractRecommender / GeneralRecommender (common/abstract_recommender.py:8-91).

The drop-in boundary: reference model files subclass GeneralRecommender unchanged.  After
construction the engine swaps their torch sparse adjacency attributes for HIP-backed CSR
``Adjacency`` objects (FoodRec.engine.graph.swap_sparse_attributes), so their
``torch.sparse.mm`` calls run the MI355X SpMM.
"""
import numpy as np
import torch
import torch.nn as nn


class AbstractRecommender(nn.Module):
    def pre_epoch_processing(self):
        pass

    def post_epoch_processing(self):
        pass

    def calculate_loss(self, interaction):
        raise NotImplementedError

    def predict(self, interaction):
        raise NotImplementedError

    def full_sort_predict(self, interaction):
        raise NotImplementedError

    def __str__(self):
        params = sum(int(np.prod(p.size())) for p in self.parameters())
        return super().__str__() + "\nTrainable parameters: {}".format(params)


class GeneralRecommender(AbstractRecommender):
    def state_dict(self, *args, **kwargs):
        """The training engine may hold deferred parameter updates (FusedAdam lazy rows): a trainer
        registers its flush here so a checkpoint always holds the dense-Adam values."""
        flush = self.__dict__.get("_fr_flush")
        if flush is not None:
            flush()
        return super().state_dict(*args, **kwargs)

    def __init__(self, config, dataset):
        super().__init__()
        self.n_users = dataset.n_users
        self.n_items = dataset.n_items
        self.batch_size = config["train_batch_size"]
        self.device = config["device"]
        self.v_feat, self.t_feat = None, None
        if not config["end2end"] and config["is_multimodal_model"]:
            # fp64 features cast to fp32 on the device (abstract_recommender.py:84-91)
            self.v_feat = torch.tensor(np.asarray(dataset.embImage).astype(np.float32)).to(self.device)
            self.t_feat = torch.tensor(np.asarray(dataset.embText).astype(np.float32)).to(self.device)
            assert self.v_feat is not None or self.t_feat is not None, "Features all NONE"
