"""HealthRec's training step WITH the bench's attention dropout (p = 0.5, configs/model/CIKM_Model.yaml:7)
checked end to end: the fused two-layer encoder stack inside the model (per-layer hash seeds and device
counters, the ingredient key-padding mask, the backward through both layers) against the float64
restatement oracle.ops.encoder_layer_f64 driven by the SAME keep-masks (oracle.ops.encoder_keep_masks).

The reference's torch-CPU dropout masks cannot be reproduced on the device, so the reference-golden
training parity (tests/test_models_gpu.py) runs HealthRec at p = 0; this test covers the p = 0.5 path
the benchmark measures.  Both runs share every non-encoder op (the engine's own), so a difference here
is the fused stack's.  Tolerances: loss components rel 1e-5; every gradient within 1e-4 of its
tensor's max (+1e-7); the layer itself is held to float64 in tests/test_encoder_gpu.py.
"""
import numpy as np
import pytest
import torch

import oracle.ops as O
from helpers import golden, tiny_config, tiny_data

pytestmark = pytest.mark.gpu


def _run_step(tr, model, batch):
    tr.optimizer.zero_grad()
    losses = model.calculate_loss(batch)
    vals = np.array([float(x.detach().reshape(-1)[0]) for x in losses])
    sum(losses).backward()
    tr.optimizer.materialize_row_grads()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    return vals, grads


def test_healthrec_dropout_step_matches_mask_restatement(cuda, monkeypatch):
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import layers
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("CIKM_Model", True, attention_probs_dropout_prob=0.5)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
    model.train()
    tr = Trainer(cfg, model)
    g = golden("model_CIKM_Model.npz")
    batch = {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}
    enc_layers = list(model.ingr_encoder.layers)
    cfgs = [m._fused_cfg(cuda) for m in enc_layers]
    assert all(c.drop[0] == pytest.approx(0.5) for c in cfgs)
    before = [int(c.counter.item()) for c in cfgs]

    got_loss, got_grads = _run_step(tr, model, batch)
    after = [int(c.counter.item()) for c in cfgs]
    assert after == [b + 1 for b in before], (before, after)  # each layer drew one step of masks
    assert len({c.seed for c in cfgs}) == len(cfgs)           # and its own hash stream

    calls = []

    def restated(encoder, src, src_key_padding_mask=None):
        kpm = torch.nn.functional._canonical_mask(mask=src_key_padding_mask, mask_name="src_key_padding_mask",
                                                  other_type=None, other_name="", target_type=src.dtype)
        x = src.transpose(0, 1).to("cpu", torch.float64)
        NS, L, _ = x.shape
        mask = None if kpm is None else kpm.to("cpu", torch.float64)
        for m, c, ctr in zip(encoder.layers, cfgs, before):
            drop = tuple(float(p) for p in c.drop)
            masks = O.encoder_keep_masks(c.seed, ctr, NS, L, drop)
            params = [p.to("cpu", torch.float64) for p in m._fused_params()]
            x = O.encoder_layer_f64(x, mask, params, masks, drop, eps=(m.norm1.eps, m.norm2.eps),
                                    gelu=bool(c.gelu))
        calls.append((NS, L))
        return x.to(src.device, torch.float32).transpose(0, 1)

    monkeypatch.setattr(layers, "run_encoder", restated)
    ref_loss, ref_grads = _run_step(tr, model, batch)
    assert calls, "the restated encoder was not called"
    np.testing.assert_allclose(got_loss, ref_loss, rtol=1e-5)
    assert set(got_grads) == set(ref_grads)
    enc_keys = [k for k in got_grads if k.startswith("ingr_encoder.")]
    assert enc_keys, "no encoder gradients"
    for k, ref in ref_grads.items():
        err = float((got_grads[k] - ref).abs().max())
        assert err <= 1e-4 * float(ref.abs().max()) + 1e-7, (k, err, float(ref.abs().max()))
