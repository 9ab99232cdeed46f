"""ORACLE (test infrastructure only): generate golden vectors by running the REFERENCE itself.

Runs ONLY in the build container, where the reference is mounted read-only at /root/reference
(importable, with one harness-side shim for scipy>=1.13's removed
dok_matrix._update).  Writes small .npz fixtures to tests/golden/; the tests and the GPU box use
only those files.  Re-run:  python oracle/gen_golden.py

Fixtures (all on the seeded synthetic 'tiny' dataset of FoodRec/utils/synthetic.py):
  adj_*.npz         reference normalised adjacencies (UI, RI, image/text/ingre cluster graphs)
  model_<M>.npz     init state_dict under seed 999, forward() outputs, loss components and
                    parameter gradients on the first training batch, params after 1 Adam step
  stream.npz        the reference sampler's (u, pos, neg) triples for epochs 0 and 1
  train_<M>.npz     per-epoch loss trace + final valid/test metrics of Trainer.fit
  ops.npz           correlation_distance / CL_loss / BPRLoss / EmbLoss values + grads
  metrics.npz       metrics_by_user / get_auc_fast on fixed rankings
  train_CIKM_Model_spread.npz  HealthRec's train trace + test metrics under torch CPU thread counts
                    1, 2, 3, 8, under 1-ulp random perturbations of the encoder layers' outputs and
                    under +-4e-7*max noise there (the reference's own spread over equally valid fp32
                    roundings)
  train_mg_LightGCN.npz  the same, trained by the reference's mirror-gradient trainer (--mg,
                    trainer.py:195-212; mg.yaml resolved to alpha1=1, alpha2=0.1, beta=3)

Fixtures at BASELINE widths (seeded synthetic data at the Allrecipes / Foodcom shapes, written in
the reference's format and read by the reference's own loader; only small slices are stored):
  wide_CIKM_Model_allrecipes.npz   HealthRec (p=0): first K training steps of Trainer.fit's stream
  wide_PRICAI_ModelX_foodcom.npz   CLUSSL, 2,000 clusters: first K training steps
  wide_PRICAI_ModelX_infonce_foodcom.npz   the same with the InfoNCE SSL term of the commented
                                   pricai_modelx.py:259 (CL_loss over the three view pairs)
  wide_BPRMF_allrecipes.npz        BPRMF (the authored plugin, BASELINE config 1), B = 1024
    per step: the batch ids and every loss component; step 0: every gradient of the small
    parameters, sampled rows of the large ones; init and after K Adam steps: sampled parameter rows

Re-generate a subset:  python oracle/gen_golden.py --only train=CIKM_Model,mg,wide
(sections: model, stream, train[=M1+M2], spread, mg, ops, metrics, wide[=M1+M2])
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "multi-modal-food-recommendation_amd"))

EPOCHS = 3


def _setup_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    # torch imports torch._dynamo lazily (first optimiser construction) and walks sys.modules with
    # inspect, which cannot place the reference's namespace package 'FoodRec': import it up front
    import torch._dynamo  # noqa: F401
    # our synthetic generator is imported BEFORE the reference takes the 'FoodRec' name
    from FoodRec.utils.synthetic import make_synthetic, write_reference_format
    for k in [k for k in sys.modules if k == "FoodRec" or k.startswith("FoodRec.")]:
        del sys.modules[k]
    sys.path.remove(os.path.join(ROOT, "multi-modal-food-recommendation_amd"))
    sys.path[:0] = [os.path.join(HERE, "ref_plugins"), REF, REF + "/FoodRec"]
    import scipy.sparse as sp
    if not hasattr(sp.dok_matrix, "_update"):
        sp.dok_matrix._update = lambda self, d: self._dict.update(d)  # SURVEY 8(c) shim
    os.chdir(REF + "/FoodRec")  # Config reads ./configs (utils/configurator.py:68-72)
    return make_synthetic, write_reference_format


def dataset_digest(ds) -> str:
    h = hashlib.sha256()
    for a in (ds.train, ds.valid, ds.test, ds.valid_neg, ds.test_neg, ds.ingre_code,
              ds.image_cluster, ds.text_cluster, ds.health):
        h.update(np.ascontiguousarray(a).tobytes())
    h.update(np.ascontiguousarray(ds.image).tobytes())
    return h.hexdigest()


def _sections(argv):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="model,stream,train,mg,ops,metrics,wide")
    want = {}
    for item in ap.parse_args(argv).only.split(","):
        name, _, arg = item.partition("=")
        want[name.strip()] = [a for a in arg.split("+") if a] or None
    return want


def main(argv=None):
    want = _sections(argv)
    make_synthetic, write_reference_format = _setup_reference()
    import torch
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.utils import init_seed, get_model
    from FoodRec.utils.dataloader import TrainDataLoader
    from FoodRec.common.trainer import Trainer, metrics_by_user, get_auc_fast
    from torch.utils.data import RandomSampler, DataLoader
    import logging

    logging.basicConfig(level=logging.WARNING)
    torch.set_num_threads(4)
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="frgold_")
    ds_syn = make_synthetic("tiny", 0)
    write_reference_format(ds_syn, tmp + "/", "Tiny")
    digest = dataset_digest(ds_syn)

    base = {"data_path": tmp + "/", "log_root": tmp + "/log/", "ckp_root": tmp + "/ckp/",
            "use_gpu": False, "seed": [999], "epochs": EPOCHS, "eval_step": 1, "n_cluster": [12],
            "neg_sample_num": 30}

    def make_config(model, extra=None, mg=False, root=None, dsname="Tiny", over_base=None):
        cd = dict(base if over_base is None else over_base)
        cd.update(extra or {})
        cfg = Config(model, dsname, cd, mg)
        root = root or tmp + "/Tiny/processed_dataset/"
        cfg["interaction_data_path"] = root
        cfg["graph_data_path"] = root + "graph_edge/"
        cfg["ingre_data_path"] = root
        # hyper-parameter lists resolved as quick_start.py:57-66 would for a single combo
        for k in cfg["hyper_parameters"]:
            if isinstance(cfg[k], list):
                cfg[k] = cfg[k][0]
        return cfg

    models = {
        "LightGCN": {},
        "BPRMF": {"reg_weight": 0.1},
        "CIKM_Model": {"attention_probs_dropout_prob": 0.0},
        "PRICAI_ModelX": {},
    }

    # ---------------------------------------------------------------- model-level goldens
    for name, extra in (models.items() if "model" in want else ()):
        cfg = make_config(name, extra)
        data = FoodData(cfg)
        init_seed(cfg["seed"])
        model = get_model(name)(cfg, data)
        sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        out = {f"sd/{k}": v.numpy() for k, v in sd0.items()}
        out["digest"] = np.array(digest)
        # adjacency goldens (the reference's own construction)
        for attr in ("norm_adj_matrix", "ri_norm_adj", "image_norm_adj", "text_norm_adj", "ingre_norm_adj"):
            if hasattr(model, attr):
                A = getattr(model, attr).coalesce()
                out[f"adj/{attr}/indices"] = A.indices().numpy()
                out[f"adj/{attr}/values"] = A.values().numpy()
                out[f"adj/{attr}/shape"] = np.array(A.shape)
        # first training batch in fit() order (trainer.py:398-402)
        trainer = Trainer(cfg, model)
        pre = TrainDataLoader(cfg, data, use_neg_list=False)
        TrainDataLoader(cfg, data, use_neg_list=True)
        dl = DataLoader(pre, sampler=RandomSampler(pre), batch_size=cfg["train_batch_size"])
        batch = next(iter(dl))
        for k, v in batch.items():
            out[f"batch/{k}"] = v.numpy()
        model.eval()  # dropout off (CIKM is also configured with p = 0)
        with torch.no_grad():
            fw = model.forward()
        out["fwd/user"] = fw[0].detach().numpy().copy()
        out["fwd/item"] = fw[1].detach().numpy().copy()
        if name == "PRICAI_ModelX":
            out["fwd/view_image"], out["fwd/view_text"], out["fwd/view_ingre"] = (x.numpy().copy() for x in fw[2])
        trainer.optimizer.zero_grad()
        losses = model.calculate_loss(batch)
        losses = losses if isinstance(losses, tuple) else (losses,)
        out["loss"] = np.array([float(l.detach().reshape(-1)[0]) for l in losses])
        sum(losses).backward()
        for k, p in model.named_parameters():
            if p.grad is not None:
                out[f"grad/{k}"] = p.grad.numpy().copy()
        trainer.optimizer.step()
        for k, p in model.named_parameters():
            out[f"adam1/{k}"] = p.detach().numpy().copy()
        np.savez_compressed(os.path.join(OUT, f"model_{name}.npz"), **out)
        print("model", name, out["loss"])

    # ---------------------------------------------------------------- sampler stream
    if "stream" in want:
        stream_golden(make_config, FoodData, init_seed, get_model, TrainDataLoader, DataLoader, RandomSampler)
    # ---------------------------------------------------------------- end-to-end training
    for name in (want["train"] or ("LightGCN", "BPRMF", "PRICAI_ModelX", "CIKM_Model")) if "train" in want else ():
        train_golden(f"train_{name}.npz", make_config(name, models[name]), name, FoodData, init_seed, get_model,
                     Trainer)
    if "spread" in want:
        train_spread("train_CIKM_Model_spread.npz", make_config("CIKM_Model", models["CIKM_Model"]), "CIKM_Model",
                     FoodData, init_seed, get_model, Trainer)
    if "mg" in want:
        # the reference's --mg cascade (configurator.py:64-86 adds configs/mg.yaml; quick_start.py:54-88
        # takes the first value of each hyper-parameter list) and Trainer(config, model, mg=True)
        train_golden("train_mg_LightGCN.npz", make_config("LightGCN", models["LightGCN"], mg=True), "LightGCN",
                     FoodData, init_seed, get_model, Trainer, mg=True)
    if "wide" in want:
        for name in want["wide"] or tuple(WIDE):
            wide_golden(name, make_synthetic, write_reference_format, make_config, FoodData, init_seed, get_model,
                        Trainer, TrainDataLoader, DataLoader, RandomSampler)
    if "ops" in want:
        ops_golden()
    if "metrics" in want:
        metrics_golden(metrics_by_user, get_auc_fast)
    print("wrote", sorted(os.listdir(OUT)))


def stream_golden(make_config, FoodData, init_seed, get_model, TrainDataLoader, DataLoader, RandomSampler):
    cfg = make_config("LightGCN")
    data = FoodData(cfg)
    init_seed(cfg["seed"])
    get_model("LightGCN")(cfg, data)  # consumes the torch RNG exactly as quick_start does
    pre = TrainDataLoader(cfg, data, use_neg_list=False)
    post = TrainDataLoader(cfg, data, use_neg_list=True)
    dl = DataLoader(pre, sampler=RandomSampler(pre), batch_size=cfg["train_batch_size"])
    st = {"pos_list_order_u": np.array(pre._user_input), "pos_list_order_i": np.array(pre._item_input_pos),
          "neg_list_post": np.array(post.neg_list), "num_items": np.array(data.num_items),
          "batch_size": np.array(cfg["train_batch_size"])}
    for ep in range(2):
        us, ps, ns = [], [], []
        for b in dl:
            us.append(b["u_id"].numpy()); ps.append(b["pos_i_id"].numpy()); ns.append(b["neg_i_id"].numpy())
        st[f"ep{ep}/u"] = np.concatenate(us)
        st[f"ep{ep}/p"] = np.concatenate(ps)
        st[f"ep{ep}/n"] = np.concatenate(ns)
    np.savez_compressed(os.path.join(OUT, "stream.npz"), **st)
    print("stream", st["ep0/u"][:8], st["ep0/n"][:8])



def train_spread(fname, cfg, name, FoodData, init_seed, get_model, Trainer, threads=(1, 2, 3, 8),
                 ulp_seeds=(1, 2, 3, 4, 5, 6), noise_seeds=tuple(range(1, 13))):
    """The reference's own sensitivity to fp32 rounding: the same Trainer.fit (same seed, data and
    batches) (a) under several torch CPU thread counts, whose reductions order their partial sums
    differently, and (b) with every Transformer encoder layer's output moved by ONE ulp, up or down
    at random (a seeded generator of its own; gradients unchanged) -- the size of the difference
    between any two correct fp32 implementations of the layer -- and (c) by uniform noise of
    +-4e-7 * max|output|, the fused MI355X layer's measured distance from float64 (tools/diag_enc.py).
    Stores every run's loss trace and final test metrics."""
    import torch
    traces, tests, kinds = [], [], []
    layer_cls = torch.nn.TransformerEncoderLayer
    orig_forward = layer_cls.forward

    def ulp_forward(gen):
        def fwd(self, *a, **kw):
            out = orig_forward(self, *a, **kw)
            with torch.no_grad():  # every output element moved by one ulp up or down (own generator)
                up = torch.rand(out.shape, generator=gen) < 0.5
                to = torch.where(up, torch.full_like(out, float("inf")), torch.full_like(out, float("-inf")))
                delta = torch.nextafter(out, to) - out
            return out + delta
        return fwd

    def noise_forward(gen):
        def fwd(self, *a, **kw):
            out = orig_forward(self, *a, **kw)
            with torch.no_grad():  # uniform +-4e-7 * max|out|: the fused kernel's measured error vs float64
                eps = 4e-7 * float(out.abs().max())
                delta = (torch.rand(out.shape, generator=gen) * 2 - 1) * eps
            return out + delta
        return fwd

    runs = ([("threads", t) for t in threads] + [("ulp", k) for k in ulp_seeds] +
            [("noise", k) for k in noise_seeds])
    for kind, t in runs:
        torch.set_num_threads(t if kind == "threads" else 4)
        if kind == "ulp":
            layer_cls.forward = ulp_forward(torch.Generator().manual_seed(int(t)))
        elif kind == "noise":
            layer_cls.forward = noise_forward(torch.Generator().manual_seed(1000 + int(t)))
        data = FoodData(cfg)
        init_seed(cfg["seed"])
        model = get_model(name)(cfg, data)
        tr = Trainer(cfg, model)
        bv, bvr, btr = tr.fit(data, hyper_tuple=(999,), saved=True, verbose=False)
        layer_cls.forward = orig_forward
        traces.append([tr.train_loss_dict[e] for e in sorted(tr.train_loss_dict)])
        tests.append(list(btr.values()))
        kinds.append(f"{kind}={t}")
        print("spread", name, kind, t, traces[-1], list(btr.values()))
    torch.set_num_threads(4)
    np.savez_compressed(os.path.join(OUT, fname), runs=np.array(kinds), train_loss=np.array(traces),
                        test_keys=np.array(list(btr.keys())), test=np.array(tests))


def train_golden(fname, cfg, name, FoodData, init_seed, get_model, Trainer, mg=False):
    data = FoodData(cfg)
    init_seed(cfg["seed"])
    model = get_model(name)(cfg, data)
    tr = Trainer(cfg, model, mg) if mg else Trainer(cfg, model)
    bv, bvr, btr = tr.fit(data, hyper_tuple=(999,), saved=True, verbose=False)
    out = {"train_loss": np.array([tr.train_loss_dict[e] for e in sorted(tr.train_loss_dict)]),
           "valid_keys": np.array(list(bvr.keys())), "valid": np.array(list(bvr.values())),
           "test_keys": np.array(list(btr.keys())), "test": np.array(list(btr.values())),
           "best_valid_score": np.array(bv)}
    if mg:
        out.update({"alpha1": np.array(cfg["alpha1"]), "alpha2": np.array(cfg["alpha2"]), "beta": np.array(cfg["beta"])})
    np.savez_compressed(os.path.join(OUT, fname), **out)
    print("train", fname, out["train_loss"], btr)


WIDE = {  # case -> (model, synthetic shape, dataset name, training steps, config overrides, loss)
    "CIKM_Model": ("CIKM_Model", "allrecipes", "Allrecipes", 3, {"attention_probs_dropout_prob": 0.0}, None),
    "PRICAI_ModelX": ("PRICAI_ModelX", "foodcom", "Foodcom", 4, {}, None),
    # the InfoNCE SSL variant: the reference's commented line pricai_modelx.py:259 (CL_loss over the
    # three view pairs), computed by the harness with the reference model's own methods
    "PRICAI_ModelX_infonce": ("PRICAI_ModelX", "foodcom", "Foodcom", 3, {}, "infonce"),
    # BASELINE config 1: the authored BPRMF plugin (oracle/ref_plugins) on the reference trainer at
    # the Allrecipes shape, overall.yaml's batch (1024: the reference ships no BPRMF.yaml)
    "BPRMF": ("BPRMF", "allrecipes", "Allrecipes", 4, {"reg_weight": 0.1}, None),
}


def clussl_infonce_losses(model, batch):
    """PRICAI_ModelX.calculate_loss (pricai_modelx.py:234-276) with its SSL term replaced by the
    commented InfoNCE line (:259): CL_loss(cat([image, text])) + CL_loss(cat([image, ingre])) +
    CL_loss(cat([ingre, text])) over the batch items' views.  The BPR and EmbLoss terms are the
    reference's own calculate_loss outputs; the views come from a second reference forward()
    (deterministic: the same values, and the gradients of both graphs sum into the parameters)."""
    import torch
    mf, _, reg = model.calculate_loss(batch)
    all_item = torch.cat([batch["pos_i_id"], batch["neg_i_id"]], dim=0)
    _, _, (image, text, ingre) = model.forward()
    a, b, c = image[all_item], text[all_item], ingre[all_item]
    cl = model.CL_loss(torch.cat([a, b], dim=0)) + model.CL_loss(torch.cat([a, c], dim=0)) + \
        model.CL_loss(torch.cat([c, b], dim=0))
    return mf, model.loss_cl * cl, reg


WIDE_LOSS = {None: lambda model, batch: model.calculate_loss(batch), "infonce": clussl_infonce_losses}
WIDE_ROWS = 48          # sampled rows per large parameter
WIDE_BIG = 1 << 16      # parameters with more elements than this are stored as sampled rows


def wide_digest(ds) -> str:
    """Digest of the training inputs of a BASELINE-width synthetic dataset (not its evaluation
    negatives: the fixtures come from negatives=False data, as bench.py uses)."""
    h = hashlib.sha256()
    for a in (ds.train, ds.valid, ds.test, ds.ingre_code, ds.ingre_num, ds.image_cluster, ds.text_cluster,
              ds.health, ds.image[::997], ds.text[::997]):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def wide_rows(name, shape0, batch_ids):
    """Rows stored for a large parameter: a fixed sample plus rows the first batch touches."""
    import zlib
    rng = np.random.default_rng(zlib.crc32(name.encode()) + shape0)
    fixed = rng.choice(shape0, size=min(WIDE_ROWS // 2, shape0), replace=False)
    touched = np.unique(batch_ids[batch_ids < shape0])[: WIDE_ROWS // 2]
    return np.unique(np.concatenate([fixed, touched])).astype(np.int64)


def wide_golden(name, make_synthetic, write_reference_format, make_config, FoodData, init_seed, get_model,
                Trainer, TrainDataLoader, DataLoader, RandomSampler):
    """The reference's first K training steps at a BASELINE width:
    Trainer.fit's order (init_seed -> model -> Trainer -> two TrainDataLoaders -> RandomSampler),
    then the step loop of trainer.py:177-224 (zero_grad, calculate_loss, sum, backward, Adam)."""
    import torch
    case = name
    name, shape, dsname, steps, extra, loss_kind = WIDE[case]
    loss_fn = WIDE_LOSS[loss_kind]
    ds = make_synthetic(shape, 0, negatives=False)
    digest = wide_digest(ds)
    # the reference's .negative reader needs >= 1 candidate per line (dataset.py:245-256); the
    # evaluation lists are not used by these fixtures
    ds.valid_neg = np.zeros((len(ds.valid_users), 1), np.int64)
    ds.test_neg = np.zeros((ds.n_users, 1), np.int64)
    root = tempfile.mkdtemp(prefix=f"frwide_{shape}_")
    write_reference_format(ds, root + "/", dsname)
    wbase = {"data_path": root + "/", "log_root": root + "/log/", "ckp_root": root + "/ckp/", "use_gpu": False,
             "seed": [999], "n_cluster": [ds.n_cluster]}
    cfg = make_config(name, extra, root=root + f"/{dsname}/processed_dataset/", dsname=dsname, over_base=wbase)
    data = FoodData(cfg)
    init_seed(cfg["seed"])
    model = get_model(name)(cfg, data)
    trainer = Trainer(cfg, model)
    pre = TrainDataLoader(cfg, data, use_neg_list=False)
    TrainDataLoader(cfg, data, use_neg_list=True)
    dl = DataLoader(pre, sampler=RandomSampler(pre), batch_size=cfg["train_batch_size"])
    out = {"digest": np.array(digest), "steps": np.array(steps), "batch_size": np.array(cfg["train_batch_size"])}
    it = iter(dl)
    model.train()
    rows = {}
    for k in range(steps):
        batch = next(it)
        for key in ("u_id", "pos_i_id", "neg_i_id"):
            out[f"step{k}/{key}"] = batch[key].numpy()
        if k == 0:
            ids = np.concatenate([batch[key].numpy() for key in ("u_id", "pos_i_id", "neg_i_id")])
            for pn, p in model.named_parameters():
                if p.numel() > WIDE_BIG:
                    rows[pn] = wide_rows(pn, p.shape[0], ids)
                    out[f"rows/{pn}"] = rows[pn]
            for pn, v in model.state_dict().items():
                out[f"sd0/{pn}"] = (v[torch.from_numpy(rows[pn])] if pn in rows else v).numpy().copy()
        if k == 0:
            _wide_f64_step(model, batch, rows, out, loss_fn)
        trainer.optimizer.zero_grad()
        losses = loss_fn(model, batch)
        losses = losses if isinstance(losses, tuple) else (losses,)
        out[f"step{k}/loss"] = np.array([float(l.detach().reshape(-1)[0]) for l in losses])
        sum(losses).backward()
        if k == 0:
            for pn, p in model.named_parameters():
                if p.grad is not None:
                    g = p.grad
                    out[f"grad0/{pn}"] = (g[torch.from_numpy(rows[pn])] if pn in rows else g).numpy().copy()
        trainer.optimizer.step()
        print("wide", case, "step", k, out[f"step{k}/loss"], flush=True)
    for pn, p in model.named_parameters():
        v = p.detach()
        out[f"final/{pn}"] = (v[torch.from_numpy(rows[pn])] if pn in rows else v).numpy().copy()
    np.savez_compressed(os.path.join(OUT, f"wide_{case}_{shape}.npz"), **out)


def _wide_f64_step(model, batch, rows, out, loss_fn):
    """The same first step of the reference model evaluated in float64 (a deep copy: parameters,
    feature tensors and adjacencies cast): ``step0/loss_f64`` and ``grad0_f64/*``.  At these widths
    the reference's own fp32 CPU gradients carry ~1e-4 - 4e-4 relative error upstream of the health
    head (fp32 sums over 1,024 items x 7 labels and 20,480 tokens), so the GPU is also pinned against
    the float64 evaluation of the reference's arithmetic."""
    import copy
    import torch
    m64 = copy.deepcopy(model).double()
    for k, v in list(vars(m64).items()):
        if torch.is_tensor(v) and v.is_floating_point():
            setattr(m64, k, v.double())
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
    m64.train()
    losses = loss_fn(m64, b64)
    losses = losses if isinstance(losses, tuple) else (losses,)
    out["step0/loss_f64"] = np.array([float(l.detach().reshape(-1)[0]) for l in losses])
    sum(losses).backward()
    for pn, p in m64.named_parameters():
        if p.grad is not None:
            g = p.grad
            # stored rounded to fp32 (6e-8 relative): far below the differences it is compared at
            out[f"grad0_f64/{pn}"] = (g[torch.from_numpy(rows[pn])] if pn in rows else g).numpy().astype(np.float32)
    del m64


def ops_golden():
    import torch
    from FoodRec.models.pricai_modelx import PRICAI_ModelX
    from FoodRec.common.loss import BPRLoss, EmbLoss
    g = torch.Generator().manual_seed(1234)
    ops = {}
    x = torch.randn(256, 64, generator=g, requires_grad=True)
    y = torch.randn(256, 64, generator=g, requires_grad=True)
    dc = PRICAI_ModelX.correlation_distance(None, x, y)
    dc.sum().backward()
    ops.update({"dcor/x": x.detach().numpy(), "dcor/y": y.detach().numpy(), "dcor/out": dc.detach().numpy(),
                "dcor/gx": x.grad.numpy(), "dcor/gy": y.grad.numpy()})
    h = torch.randn(2 * 128, 64, generator=g, requires_grad=True)
    cl = PRICAI_ModelX.CL_loss(None, h)
    cl.backward()
    ops.update({"cl/h": h.detach().numpy(), "cl/out": cl.detach().numpy(), "cl/gh": h.grad.numpy()})
    ps_ = torch.randn(100, generator=g, requires_grad=True)
    ns_ = torch.randn(100, generator=g, requires_grad=True)
    bl = BPRLoss()(ps_, ns_)
    bl.backward()
    ops.update({"bpr/pos": ps_.detach().numpy(), "bpr/neg": ns_.detach().numpy(), "bpr/out": bl.detach().numpy(),
                "bpr/gpos": ps_.grad.numpy()})
    es = [torch.randn(50, 64, generator=g, requires_grad=True) for _ in range(3)]
    el = EmbLoss()(*es)
    el.sum().backward()
    ops.update({"emb/e0": es[0].detach().numpy(), "emb/e1": es[1].detach().numpy(),
                "emb/e2": es[2].detach().numpy(), "emb/out": el.detach().numpy(),
                "emb/g0": es[0].grad.numpy()})
    np.savez_compressed(os.path.join(OUT, "ops.npz"), **ops)


def metrics_golden(metrics_by_user, get_auc_fast):
    rng = np.random.default_rng(7)
    mt = {}
    for k in range(20):
        n_pos = int(rng.integers(1, 6))
        pred = rng.standard_normal(n_pos + 30).astype(np.float32)
        if k % 5 == 0:
            pred[3] = pred[7]  # a tie
        order = np.argsort(pred)[::-1]
        rec, nd = [], []
        for kk in (10, 20):
            r_, n_ = metrics_by_user(order[:kk], range(n_pos))
            rec.append(r_); nd.append(n_)
        mt[f"u{k}/pred"] = pred
        mt[f"u{k}/npos"] = np.array(n_pos)
        mt[f"u{k}/recall"] = np.array(rec)
        mt[f"u{k}/ndcg"] = np.array(nd)
        mt[f"u{k}/auc"] = np.array(get_auc_fast(range(n_pos), pred, 30))
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), **mt)


if __name__ == "__main__":
    main()
