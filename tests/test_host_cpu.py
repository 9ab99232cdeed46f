"""CPU tests: host logic against the reference's goldens (no GPU, no compute kernels).

Covers the dataset loader, config cascade, exact-RNG triple sampler (MT19937 stream + torch
permutation), model init parity (state_dict bit-identical under seed 999), normalised
adjacency construction (bit-identical to the reference's scipy build), evaluation metrics,
and the C-ABI library exporting every symbol of include/fr_engine.h.
"""
import os
import re

import numpy as np
import pytest
import torch

from helpers import golden, tiny_config, tiny_data, tiny_dir

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dataset_digest_matches_goldens():
    """The goldens were produced on make_synthetic('tiny', 0); a generator change must regenerate them."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from gen_golden import dataset_digest
    from FoodRec.utils.synthetic import make_synthetic
    assert str(golden("model_LightGCN.npz")["digest"]) == dataset_digest(make_synthetic("tiny", 0))


def test_library_exports_header_symbols():
    from FoodRec.engine import native
    header = open(os.path.join(ROOT, "include", "fr_engine.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|void|const char\*)\s+(fr_\w+)\s*\(", header, re.M))
    assert declared == set(native.EXPORTED_SYMBOLS)
    lib = native.lib()
    for name in declared:
        assert hasattr(lib, name)
    assert lib.fr_version() >= 1


def test_config_cascade_semantics():
    from FoodRec.utils.configurator import Config
    cfg = Config("CIKM_Model", "Allrecipes", {"learning_rate": 0.123, "use_gpu": False})
    assert cfg["learning_rate"] == 0.123          # config_dict overrides files
    assert cfg["train_batch_size"] == 512          # model yaml overrides overall.yaml (1024)
    assert cfg["definitely_missing_key"] is None   # missing keys read as None
    assert cfg["hyper_parameters"][-1] == "seed"   # seed appended
    assert cfg["valid_metric_bigger"] is True
    lg = Config("LightGCN", "x", {"use_gpu": False})
    assert isinstance(lg["reg_weight"], float) and lg["reg_weight"] == 0.1   # '1e-01' is a float


def test_dataset_matches_reference_structures():
    g = golden("stream.npz")
    data = tiny_data(tiny_config("LightGCN", False))
    np.testing.assert_array_equal(data.train_pairs[:, 0], g["pos_list_order_u"])
    np.testing.assert_array_equal(data.train_pairs[:, 1], g["pos_list_order_i"])
    assert data.num_items == int(g["num_items"])
    assert len(data.trainList) == data.num_users
    assert all(isinstance(x, int) for x in data.testNegatives[0])


def test_sampler_stream_bit_exact():
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("stream.npz")
    cfg = tiny_config("LightGCN", False)
    data = tiny_data(cfg)
    init_seed(999)
    get_model("LightGCN")(cfg, data)          # consumes torch's RNG like quick_start
    s = TripleSampler(data, int(g["batch_size"]))
    np.testing.assert_array_equal(s.neg_list_post, g["neg_list_post"])
    for ep in range(2):
        u, p, n = (np.concatenate(x) for x in zip(*[(a.numpy(), b.numpy(), c.numpy()) for a, b, c in s.epoch()]))
        np.testing.assert_array_equal(u, g[f"ep{ep}/u"])
        np.testing.assert_array_equal(p, g[f"ep{ep}/p"])
        np.testing.assert_array_equal(n, g[f"ep{ep}/n"])


def test_sampler_close_joins_the_prefetch_thread(monkeypatch):
    """TripleSampler.close (Trainer.fit's finally): a prefetch in flight is joined, its host thread
    shut down, and an exception the thread raised reaches the caller instead of being dropped."""
    import threading
    from FoodRec.engine.sampler import TripleSampler
    cfg = tiny_config("LightGCN", False)
    data = tiny_data(cfg)
    s = TripleSampler(data, 64)
    s.prefetch()
    s.close()
    assert s._pending is None and s._pool is None
    assert not [t for t in threading.enumerate() if t.name.startswith("fr-sampler")]

    def boom(slot):
        raise RuntimeError("draw failed")
    monkeypatch.setattr(s, "_draw_host", boom)
    s.prefetch()
    with pytest.raises(RuntimeError, match="draw failed"):
        s.close()
    assert s._pool is None


def test_sampler_prefetch_keeps_the_stream():
    """TripleSampler.prefetch (the next epoch's permutation and negatives drawn on a host thread
    while this epoch's batches are consumed) yields the reference stream: the golden epochs, and the
    global RNG states after them, equal those of drawing at each epoch's start."""
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("stream.npz")
    cfg = tiny_config("LightGCN", False)
    data = tiny_data(cfg)
    init_seed(999)
    get_model("LightGCN")(cfg, data)
    s = TripleSampler(data, int(g["batch_size"]))
    for ep in range(2):
        u, p, n = (np.concatenate(x) for x in zip(*[(a.numpy(), b.numpy(), c.numpy())
                                                     for a, b, c in s.epoch(prefetch=ep == 0)]))
        np.testing.assert_array_equal(u, g[f"ep{ep}/u"])
        np.testing.assert_array_equal(p, g[f"ep{ep}/p"])
        np.testing.assert_array_equal(n, g[f"ep{ep}/n"])
    assert s._pending is None
    after = (torch.get_rng_state(), np.random.get_state()[1].copy())
    init_seed(999)
    get_model("LightGCN")(cfg, data)
    s2 = TripleSampler(data, int(g["batch_size"]))
    for _ in range(2):
        list(s2.epoch())
    assert torch.equal(after[0], torch.get_rng_state())
    np.testing.assert_array_equal(after[1], np.random.get_state()[1])


def test_randint_stream_equals_numpy():
    from FoodRec.engine.sampler import draw_negatives
    import ctypes
    from FoodRec.engine import native
    for high in (1, 2, 7, 90, 45630, 2 ** 31 + 11, 2 ** 40 + 3):
        np.random.seed(high % 1000)
        ref = [np.random.randint(high) for _ in range(500)]
        np.random.seed(high % 1000)
        st = np.random.get_state()
        key = np.array(st[1], np.uint32)
        pos = np.array([st[2]], np.int32)
        out = np.empty(500, np.int64)
        native.check(native.lib().fr_sampler_randint(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                      pos.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                      high, 500, out.ctypes.data), "randint")
        np.testing.assert_array_equal(out, ref)
        np.random.set_state((st[0], key, int(pos[0]), st[3], st[4]))
        assert np.random.randint(1 << 30) == (lambda: (np.random.seed(high % 1000), [np.random.randint(high) for _ in range(500)], np.random.randint(1 << 30))[2])()


@pytest.mark.parametrize("name", ["LightGCN", "BPRMF", "CIKM_Model", "PRICAI_ModelX"])
def test_model_init_and_adjacency_bit_exact(name):
    from FoodRec.utils.utils import get_model, init_seed
    g = golden(f"model_{name}.npz")
    cfg = tiny_config(name, False)
    data = tiny_data(cfg)
    init_seed(999)
    m = get_model(name)(cfg, data)
    sd = m.state_dict()
    assert sorted(sd) == sorted(k[3:] for k in g.files if k.startswith("sd/"))
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), g["sd/" + k], err_msg=k)
    for attr in ("norm_adj_matrix", "ri_norm_adj", "image_norm_adj", "text_norm_adj", "ingre_norm_adj"):
        if f"adj/{attr}/values" not in g.files:
            continue
        A = getattr(m, attr)
        rows = np.repeat(np.arange(A.shape[0]), np.diff(A.rowptr.numpy()))
        idx = g[f"adj/{attr}/indices"]
        np.testing.assert_array_equal(rows, idx[0])
        np.testing.assert_array_equal(A.col.numpy(), idx[1])
        np.testing.assert_array_equal(A.val.numpy(), g[f"adj/{attr}/values"])
        assert tuple(A.shape) == tuple(g[f"adj/{attr}/shape"])


def test_metrics_match_reference():
    from FoodRec.common.trainer import get_auc_fast, metrics_by_user
    g = golden("metrics.npz")
    for k in range(20):
        pred, npos = g[f"u{k}/pred"], int(g[f"u{k}/npos"])
        order = np.argsort(pred)[::-1]
        for j, topk in enumerate((10, 20)):
            r, nd = metrics_by_user(order[:topk], range(npos))
            assert r == g[f"u{k}/recall"][j] and nd == g[f"u{k}/ndcg"][j]
        assert get_auc_fast(range(npos), pred, 30) == g[f"u{k}/auc"]


def test_oracle_pinned_against_reference_ops():
    """The oracle's restatements reproduce the reference's own op outputs (ops.npz)."""
    from oracle import ops as O
    g = golden("ops.npz")
    x = torch.tensor(g["dcor/x"], requires_grad=True)
    y = torch.tensor(g["dcor/y"], requires_grad=True)
    d = O.correlation_distance(x, y)
    d.sum().backward()
    np.testing.assert_allclose(d.detach().numpy(), g["dcor/out"], rtol=1e-6)
    np.testing.assert_allclose(x.grad.numpy(), g["dcor/gx"], rtol=1e-5, atol=1e-7)
    h = torch.tensor(g["cl/h"], requires_grad=True)
    c = O.cl_loss(h)
    c.backward()
    np.testing.assert_allclose(c.detach().numpy(), g["cl/out"], rtol=1e-6)
    np.testing.assert_allclose(h.grad.numpy(), g["cl/gh"], rtol=1e-5, atol=1e-8)
    b = O.bpr_loss(torch.tensor(g["bpr/pos"]), torch.tensor(g["bpr/neg"]))
    np.testing.assert_allclose(b.numpy(), g["bpr/out"], rtol=1e-7)
    e = O.emb_loss(*(torch.tensor(g[f"emb/e{i}"]) for i in range(3)))
    np.testing.assert_allclose(e.numpy(), g["emb/out"], rtol=1e-7)
    A = golden("model_LightGCN.npz")
    idx, val = A["adj/norm_adj_matrix/indices"], A["adj/norm_adj_matrix/values"]
    n = int(A["adj/norm_adj_matrix/shape"][0])
    upper = idx[0] < idx[1]
    r, c, v = O.norm_adj_coo(n, idx[0][upper], idx[1][upper])
    np.testing.assert_array_equal(r, idx[0])
    np.testing.assert_array_equal(c, idx[1])
    np.testing.assert_array_equal(v, val)


def test_engine_refuses_cpu_tensors():
    from FoodRec.engine import native, ops
    with pytest.raises(native.EngineError):
        ops.bpr_emb_loss(torch.randn(4, 8), torch.randn(4, 8), None, None,
                         torch.zeros(2, dtype=torch.long), torch.zeros(2, dtype=torch.long),
                         torch.zeros(2, dtype=torch.long))


def test_safe_unpickler_refuses_code():
    import pickle
    from FoodRec.utils.dataset import safe_pickle_load
    path = os.path.join(tiny_dir(), "evil.pkl")
    with open(path, "wb") as f:
        pickle.dump(os.getcwd, f)   # a callable: must not be reconstructed
    with pytest.raises(pickle.UnpicklingError):
        safe_pickle_load(path)


@pytest.mark.parametrize("act", ["gelu", "relu"])
def test_engine_encoder_layer_restates_torch(act):
    """engine.layers.TransformerEncoderLayer: same parameters/init as torch's, and its restated
    training forward (post-norm, packed in-projection, per-head key-padding mask, SDPA) gives the
    same outputs and gradients as torch's module (cikm_model.py:33-35 builds this layer)."""
    import torch
    import torch.nn as nn
    from FoodRec.engine import layers
    torch.manual_seed(0)
    ref = nn.TransformerEncoder(nn.TransformerEncoderLayer(64, 2, 256, dropout=0.0, activation=act),
                                num_layers=2, enable_nested_tensor=False)
    torch.manual_seed(0)
    eng = nn.TransformerEncoder(layers.TransformerEncoderLayer(64, 2, 256, dropout=0.0, activation=act),
                                num_layers=2, enable_nested_tensor=False)
    sr, se = ref.state_dict(), eng.state_dict()
    assert list(sr) == list(se) and all(torch.equal(sr[k], se[k]) for k in sr)
    for layer in eng.layers:  # force the restated path on CPU (ops.linear -> F.linear below 1024 rows)
        layer._engine_path = lambda *a: True
    g = torch.Generator().manual_seed(1)
    x = torch.randn(20, 7, 64, generator=g)
    mask = torch.rand(7, 20, generator=g) < 0.4
    mask[:, 0] = False
    xr, xe = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    yr = ref(xr, src_key_padding_mask=mask)
    ye = eng(xe, src_key_padding_mask=mask)
    torch.testing.assert_close(ye, yr, rtol=1e-6, atol=1e-6)
    w = torch.randn(yr.shape, generator=g)
    (yr * w).sum().backward()
    (ye * w).sum().backward()
    torch.testing.assert_close(xe.grad, xr.grad, rtol=1e-5, atol=1e-6)
    for (n, pr), (_, pe) in zip(ref.named_parameters(), eng.named_parameters()):
        torch.testing.assert_close(pe.grad, pr.grad, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.parametrize("model", ["CIKM_Model", "PRICAI_ModelX", "LightGCN", "BPRMF"])
def test_oracle_cpu_backend_covers_engine_models(model):
    """bench.py's cpu_baseline leg runs engine models on the host through oracle.cpu_backend: every
    engine op a model calls must have a CPU restatement there (one training step, finite losses)."""
    import torch
    from oracle import cpu_backend
    from helpers import tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    with cpu_backend.installed():
        cfg = tiny_config(model, False)
        cfg["device"] = torch.device("cpu")
        data = tiny_data(cfg)
        init_seed(999)
        m = get_model(model)(cfg, data)
        trainer = Trainer(cfg, m)
        sampler = TripleSampler(data, 512, "cpu", replay_python_random=False)  # 2B = 1024 rows: ops.linear's engine path
        state = trainer.new_step_state()
        u, p, n = next(iter(sampler.epoch()))
        trainer.train_step(trainer._features().batch(u, p, n), 0, state)
        assert torch.isfinite(state["acc"]).all() and int(state["nan"]) == 0


@pytest.mark.parametrize("name,shape", [("CIKM_Model", "allrecipes"), ("PRICAI_ModelX", "foodcom"),
                                        ("BPRMF", "allrecipes")])
def test_wide_goldens_match_generator(name, shape):
    """The BASELINE-width reference fixtures (tests/golden/wide_*.npz) were produced on
    make_synthetic(shape, 0, negatives=False), the data bench.py trains on."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from gen_golden import wide_digest
    from FoodRec.utils.synthetic import make_synthetic
    assert str(golden(f"wide_{name}_{shape}.npz")["digest"]) == wide_digest(make_synthetic(shape, 0, negatives=False))


@pytest.mark.parametrize("edges", [64, 2048])
def test_sparse_block_plan_covers_every_edge_once(edges):
    """ops.sparse_block_plan (the sparse-upstream kernel's edge-balanced row blocks): every edge in
    exactly one block, blocks of at most 64 whole rows and 2 x ``edges`` edges, heavy rows (more than
    ``edges`` edges) cut into consecutive chunks of at most ``edges`` edges and listed once in
    split_rows, empty rows and a trailing empty row covered."""
    from FoodRec.engine.ops import sparse_block_plan
    rng = np.random.default_rng(edges)
    deg = np.concatenate([rng.integers(0, 30, 3000), [5 * edges + 3, 0, 0, edges, edges + 1],
                          rng.zipf(1.6, 500).clip(max=40 * edges), [0]])
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    blocks, split_rows = sparse_block_plan(rp, 64, edges)
    cover = np.zeros(rp[-1], np.int32)
    rows_seen = np.zeros(len(deg), np.int32)
    for r0, r1, e0, e1 in blocks:
        cover[e0:e1] += 1
        if e0 == rp[r0] and e1 == rp[r1]:  # whole rows
            assert 0 < r1 - r0 <= 64 and e1 - e0 <= 2 * edges
            rows_seen[r0:r1] += 1
        else:  # a chunk of one heavy row
            assert r1 - r0 == 1 and r0 in split_rows and 0 < e1 - e0 <= edges
            assert rp[r0] <= e0 < e1 <= rp[r1]
    assert (cover == 1).all()
    assert np.array_equal(np.sort(split_rows), np.nonzero(deg > edges)[0])
    assert (rows_seen[deg <= edges] == 1).all() and (rows_seen[deg > edges] == 0).all()
    assert (np.diff(blocks[:, 2]) >= 0).all()  # in edge order


def test_sparse_block_rows_exported_and_plans_refused():
    """The sparse-upstream kernel's row limit comes from the library (fr_spmm_sparse_block_rows, the
    kernel's kSpRows = 64; no GPU call), sparse_block_plan refuses a wider block size, and
    check_sparse_plan refuses a 65-row block, rows past the adjacency and an edge range outside its
    rows -- the same conditions the kernel flags in fr_spmm_plan_status."""
    from FoodRec.engine import native, ops
    assert native.lib().fr_spmm_sparse_block_rows() == 64 == ops.sparse_block_rows()
    rp = np.arange(0, 301 * 3, 3, dtype=np.int64)  # 300 rows of 3 edges
    with pytest.raises(native.EngineError):
        ops.sparse_block_plan(rp, 65, 2048)
    blocks, _ = ops.sparse_block_plan(rp)
    assert (blocks[:, 1] - blocks[:, 0]).max() == 64
    ops.check_sparse_plan(blocks, rp, 64)
    for bad in ([[0, 65, 0, 195]], [[290, 301, 870, 903]], [[0, 10, 0, 33]], [[5, 7, 16, 20]]):
        with pytest.raises(native.EngineError):
            ops.check_sparse_plan(np.asarray(bad), rp, 64)
    ops.check_sparse_plan(np.asarray([[5, 6, 16, 17], [5, 6, 17, 18]]), rp, 64)  # chunks of one row


def test_plain_chunk_widens_light_graphs_only():
    """graph.plain_chunk: a graph whose heaviest row fits PLAIN_MAX_DEGREE gets a chunk covering it
    (no split rows: the single-launch row walk), a heavier graph keeps the auto chunk."""
    from FoodRec.engine import graph
    if graph.PLAIN_MAX_DEGREE == 0:
        pytest.skip("FR_PLAIN_CHUNK=0")
    assert graph.plain_chunk(32, 20) == 32
    assert graph.plain_chunk(32, 125) == 128
    assert graph.plain_chunk(64, 65) == 128
    assert graph.plain_chunk(32, 256) == 256
    assert graph.plain_chunk(32, 257) == 32
    assert graph.plain_chunk(128, 2928) == 128
    rng = np.random.default_rng(0)
    rows = rng.integers(0, 300, 6000)
    cols = 300 + rng.integers(0, 40, 6000)  # 40 side nodes of ~150 edges each
    adj = graph.Adjacency.sym_normalized(340, torch.as_tensor(rows), torch.as_tensor(cols))
    deg = np.diff(adj.rowptr.numpy())
    assert 128 < deg.max() <= 256 and adj.chunk == 256 and adj.n_split == 0 and adj.n_plain == 340


def test_reserve_replays_flushes_before_the_ring_could_wrap():
    """FusedAdam.reserve_replays: an unrolled graph runs ``n`` lazy steps before
    note_replay sees them, so the optimiser flushes first when pending + n would pass hist_cap - 2."""
    import torch
    from FoodRec.engine.optim import FusedAdam
    opt = FusedAdam([torch.nn.Parameter(torch.zeros(4, 4))], lazy_rows=True, hist_cap=8)
    calls = []
    opt.flush = lambda: (calls.append(opt._lazy_pending), setattr(opt, "_lazy_pending", 0))
    opt.reserve_replays(4)  # nothing launched yet: nothing to flush
    assert calls == []
    opt._lazy_launched = True
    opt._lazy_pending = 2
    opt.reserve_replays(4)  # 2 + 4 = 6 = hist_cap - 2: within the bound
    assert calls == []
    opt._lazy_pending = 3
    opt.reserve_replays(4)  # 3 + 4 = 7 > 6: flush first
    assert calls == [3] and opt._lazy_pending == 0
    with pytest.raises(ValueError):
        opt.reserve_replays(7)  # more steps per replay than the ring can ever hold


def test_bookkeeping_launches_refuse_repeated_counters():
    """fr_step_book / fr_healthrec_loss_finalize load every counter before advancing any (one
    memory round trip), so a counter named twice would advance once: the ABI refuses it before
    any launch (host-side check; no device needed)."""
    import ctypes
    from FoodRec.engine import native
    lib = native.lib()
    parts = (ctypes.c_void_p * 1)(0x1000)
    twice = (ctypes.c_void_p * 2)(0x2000, 0x2000)
    with pytest.raises(native.EngineError, match="distinct"):
        native.check(lib.fr_step_book(parts, 1, 0x3000, 0, 0x4000, twice, 2, None, None), "fr_step_book")
    with pytest.raises(native.EngineError, match="distinct"):
        native.check(lib.fr_healthrec_loss_finalize(0x1000, 16, 0.5, 1.0, 1.0, 0x1100, 0x1200, 64, 0x1300, 512.0,
                                                    1e-3, 0x1400, 0x1500, 0x1600, 0x1700, 0, 0x1800, twice, 2,
                                                    None, None), "fr_healthrec_loss_finalize")


def test_region_byte_models():
    """The byte models of the regions that used to report none: row-list SpMM at
    each side's mean degree, the RI frontier's expected size, the sparse-upstream scan + write, the
    scatter-upstream, and the BPR backward / finish kernels -- pinned on a small bipartite shape."""
    from types import SimpleNamespace
    import torch
    from FoodRec.engine import ops
    adj = SimpleNamespace(shape=(100, 100), nnz=600, bipartite_split=40, nnz_below_split=300)
    assert ops.mean_degree(adj, 0) == 7.5 and ops.mean_degree(adj, 40) == 5.0
    flat = SimpleNamespace(shape=(100, 100), nnz=600, bipartite_split=None, nnz_below_split=0)
    assert ops.mean_degree(flat, 77) == 6.0
    ids = torch.zeros(10, dtype=torch.int64)
    # users (side 0) and items (offset 40: side 1), one output written each
    want = 10 * (16 + 7.5 * (8 + 256) + 256) + 10 * (16 + 5.0 * (8 + 256) + 256)
    assert ops.rows_bytes(adj, [(ids, 0), (ids, 40)], 64, 1) == int(want)
    assert ops.rows_bytes(adj, 10, 64, 3) == int(10 * (16 + 7.5 * 264 + 3 * 256))
    assert ops.frontier_rows(adj, 4, 60) == 38 and ops.frontier_rows(adj, 40, 60) == 60
    assert ops.sparse_upstream_bytes(adj) == 8 * 101 + 8 * 600 + 256 * 100
    assert ops.scatter_upstream_bytes(adj, [(ids, 40)]) == int(10 * (16 + 256 + 5.0 * (8 + 512)))
    assert ops.bpr_bwd_bytes(512) == 3 * 512 * (8 + 1024)
    assert ops.bpr_finish_bytes(512) == 3 * 512 * (9 + 768)
