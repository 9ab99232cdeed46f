"""Row gradients of row-gathered tables (fr_embedding_rowgrad + fr_adam_step_rows) vs the dense path.

HealthRec's image / text feature tables (cikm_model.py:83-87) are only row-gathered on the step, so
FusedAdam takes their gradient as (row -> slot map, one summed row per distinct id).  Bar: the
parameters and both Adam moments after several steps are BIT-IDENTICAL to the dense-gradient
update (same per-row sums in the same order, zero gradient elsewhere), and the compact rows equal
the float64 scatter of the oracle within 1e-6 of each row's sum of |G| (fp32 summation).
"""
import numpy as np
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


def _case(R, d, n, pad, seed):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, R, (n,), generator=g)
    ids[: n // 10] = ids[n // 2]  # a hot row
    if pad is not None:
        ids[1::17] = pad
    G = torch.randn(n, d, generator=g)
    return ids, G


@pytest.mark.parametrize("R,d,n,pad", [(45630, 2048, 1024, None), (45630, 512, 1024, None), (1000, 64, 4096, 7),
                                       (300, 4, 1, None), (45630, 512, 8192, None), (2000, 64, 20480, 1999)])
def test_rowgrad_matches_scatter(cuda, R, d, n, pad):
    from FoodRec.engine import native
    ids, G = _case(R, d, n, pad, 1)
    idg, Gg = ids.to(cuda), G.to(cuda)
    rmap = torch.empty(R, dtype=torch.int32, device=cuda)
    rows = torch.empty(n, d, device=cuda)
    lib = native.lib()
    ws = native.workspace(lib.fr_embedding_rowgrad_workspace(n, R, d), cuda)
    native.check(lib.fr_embedding_rowgrad(idg.data_ptr(), n, Gg.data_ptr(), d, d, R, -1 if pad is None else pad,
                                          rmap.data_ptr(), rows.data_ptr(), ws.data_ptr(), ws.numel(),
                                          torch.cuda.current_stream().cuda_stream), "rowgrad")
    ref = O.embedding_bwd_f64(ids.numpy(), G.numpy(), R, pad)
    rm = rmap.cpu().numpy()
    present = np.unique(ids.numpy()[ids.numpy() != (-1 if pad is None else pad)])
    assert set(np.nonzero(rm >= 0)[0].tolist()) == set(present.tolist())
    # the slot of a row is its first position
    first = {}
    for i, r in enumerate(ids.numpy().tolist()):
        first.setdefault(r, i)
    assert all(rm[r] == first[r] for r in present.tolist())
    got = rows.cpu().numpy()[rm[present]]
    scale = O.embedding_bwd_f64(ids.numpy(), np.abs(G.numpy()), R, pad)[present]  # sum of |G| per row
    assert np.all(np.abs(got - ref[present]) <= 1e-6 * scale + 1e-7)


@pytest.mark.parametrize("d", [2048, 64])
def test_row_adam_bit_identical_to_dense(cuda, d):
    from FoodRec.engine import ops
    from FoodRec.engine.optim import FusedAdam
    R, n = 5000, 1024
    torch.manual_seed(0)
    w0 = torch.randn(R, d) * 0.1
    extra = torch.randn(33, 7)  # a dense parameter in the same step
    pa, pb = (torch.nn.Parameter(w0.clone().to(cuda)) for _ in range(2))
    ea, eb = (torch.nn.Parameter(extra.clone().to(cuda)) for _ in range(2))
    oa, ob = FusedAdam([pa, ea], lr=3e-3), FusedAdam([pb, eb], lr=3e-3)
    for step in range(3):
        ids, G = _case(R, d, n, 11, 10 + step)
        idg, Gg = ids.to(cuda), G.to(cuda)
        ge = torch.randn(33, 7, generator=torch.Generator().manual_seed(step)).to(cuda)
        oa.zero_grad()
        pa.grad = ops.scatter_rows(idg, Gg, R, 11)  # dense path
        ea.grad = ge.clone()
        oa.step()
        ob.zero_grad()
        ob.row_grads.stash(pb, 11, idg, Gg)      # row path
        eb.grad = ge.clone()
        ob.step()
        assert torch.equal(pa, pb), step
        assert torch.equal(oa.state[pa]["exp_avg"], ob.state[pb]["exp_avg"])
        assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])
        assert torch.equal(ea, eb)


def test_rowgrad_sort_path_matches_dense_bitwise(cuda):
    """n > 4096 (the 8-rank data-parallel exchange: 8 x 1024 rows) takes the counting-sort path in
    compact mode; its rows equal the dense path's rows bit for bit."""
    from FoodRec.engine import native, ops
    R, d, n = 45630, 512, 8192
    ids, G = _case(R, d, n, None, 9)
    idg, Gg = ids.to(cuda), G.to(cuda)
    dense = ops.scatter_rows(idg, Gg, R, None)
    lib = native.lib()
    rmap = torch.empty(R, dtype=torch.int32, device=cuda)
    rows = torch.empty(n, d, device=cuda)
    ws = native.workspace(lib.fr_embedding_rowgrad_workspace(n, R, d), cuda)
    native.check(lib.fr_embedding_rowgrad(idg.data_ptr(), n, Gg.data_ptr(), d, d, R, -1, rmap.data_ptr(),
                                          rows.data_ptr(), ws.data_ptr(), ws.numel(),
                                          torch.cuda.current_stream().cuda_stream), "rowgrad")
    present = torch.nonzero(rmap >= 0).squeeze(1)
    assert torch.equal(rows[rmap[present].long()], dense[present])
    assert int((dense.abs().sum(1) > 0).sum()) <= present.numel()


def test_row_adam_accumulates_like_dense(cuda):
    from FoodRec.engine import ops
    from FoodRec.engine.optim import FusedAdam
    R, d = 777, 128
    torch.manual_seed(1)
    w0 = torch.randn(R, d)
    pa, pb = (torch.nn.Parameter(w0.clone().to(cuda)) for _ in range(2))
    oa, ob = FusedAdam([pa], lr=1e-2), FusedAdam([pb], lr=1e-2)
    ids1, G1 = _case(R, d, 500, None, 3)
    ids2, G2 = _case(R, d, 300, None, 4)
    i1, g1, i2, g2 = ids1.to(cuda), G1.to(cuda), ids2.to(cuda), G2.to(cuda)
    oa.zero_grad()
    pa.grad = ops.scatter_rows(torch.cat([i1, i2]), torch.cat([g1, g2]), R, None)
    oa.step()
    ob.zero_grad()
    ob.row_grads.stash(pb, None, i1, g1)
    ob.row_grads.stash(pb, None, i2, g2)
    ob.step()
    assert torch.equal(pa, pb)
    assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])


def test_healthrec_step_row_vs_dense(cuda):
    """One HealthRec training step with row_grad_tables on and off: the image / text tables and their
    Adam moments are bit-identical.  (Other parameters are not compared after the step: the BPR
    gradient scatter uses float atomics, and a first Adam step moves each element by ~lr * sign(g),
    so last-bit gradient noise can flip near-zero elements.)"""
    from helpers import golden, tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("model_CIKM_Model.npz")
    batch = {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}
    runs = []
    for rows in (True, False):
        cfg = tiny_config("CIKM_Model", True, row_grad_tables=rows, cuda_graph=False)
        data = tiny_data(cfg)
        init_seed(999)
        model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
        tr = Trainer(cfg, model)
        assert (model.__dict__.get("_fr_exchange") is tr.optimizer.row_grads) == rows
        tr.train_step(batch, 0, tr.new_step_state())
        runs.append((model, tr.optimizer))
    (ma, oa), (mb, ob) = runs
    for (k, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
        if k.startswith(("image_embedding", "text_embedding")):
            assert torch.equal(a, b), k
            for s_ in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(oa.state[a][s_], ob.state[b][s_]), (k, s_)


@pytest.mark.parametrize("wd,cap", [(0.0, 8192), (0.01, 8), (0.0, 5)])
def test_lazy_row_adam_equals_eager_rows(cuda, wd, cap):
    """fr_adam_step_rows_lazy (deferred zero-gradient row steps) vs fr_adam_step_rows over 23 steps
    on two tables with sparse, repeating row sets, an lr change mid-way (LambdaLR between epochs),
    weight decay, and a history ring small enough to force the automatic flushes: after each flush
    p, exp_avg and exp_avg_sq are BIT-IDENTICAL to the every-row update."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(2)
    shapes = [(613, 256), (301, 64)]
    w0 = [torch.randn(R, d) for R, d in shapes]
    pa = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    pb = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    oa = FusedAdam(pa, lr=3e-3, weight_decay=wd)
    ob = FusedAdam(pb, lr=3e-3, weight_decay=wd, lazy_rows=True, hist_cap=cap)
    for step in range(23):
        if step == 11:
            for o in (oa, ob):
                o.param_groups[0]["lr"] = 1.5e-3
                o.sync_lr()
        oa.zero_grad()
        ob.zero_grad()
        for k, ((R, d), a, b) in enumerate(zip(shapes, pa, pb)):
            n = 40 if step % 3 else 5
            ids, G = _case(R, d, n, None, 100 * step + k)
            # step 0 touches every row (non-zero moments everywhere), later steps a third of them:
            # the other rows only decay, through deferred steps
            ids = torch.arange(R) if step == 0 else ids % (R // 3)
            G = torch.randn(R, d) if step == 0 else G
            ids, G = ids.to(cuda), G.to(cuda)
            oa.row_grads.stash(a, None, ids, G)
            ob.row_grads.stash(b, None, ids, G)
        oa.step()
        ob.step()
        if step in (6, 22):
            ob.flush()
            for a, b in zip(pa, pb):
                assert torch.equal(a, b)
                for s_ in ("exp_avg", "exp_avg_sq"):
                    assert torch.equal(oa.state[a][s_], ob.state[b][s_]), s_
    # lazy state really skipped rows between flushes
    assert "lazy_last" in ob.state[pb[0]]


def test_lazy_row_adam_graph_replay(cuda):
    """The lazy update captured in a HIP graph and replayed: step counter, history ring and row
    replays run from device state; note_replay counts the replays, flush() equals the eager rows."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(3)
    R, d = 517, 128
    w0 = torch.randn(R, d)
    pa = torch.nn.Parameter(w0.clone().to(cuda))
    pb = torch.nn.Parameter(w0.clone().to(cuda))
    oa = FusedAdam([pa], lr=2e-3)
    ob = FusedAdam([pb], lr=2e-3, lazy_rows=True, hist_cap=16)
    ids_s = torch.zeros(64, dtype=torch.int64, device=cuda)
    G_s = torch.zeros(64, d, device=cuda)

    def body():
        ob.zero_grad()
        ob.row_grads.stash(pb, None, ids_s, G_s)
        ob.step()

    cases = [_case(R, d, 64, None, 700 + k) for k in range(20)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ids_s.copy_(cases[0][0].to(cuda) % 100)
        G_s.copy_(cases[0][1].to(cuda))
        body()  # eager warm-up step (state creation)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for k, (ids, G) in enumerate(cases):
        oa.zero_grad()
        oa.row_grads.stash(pa, None, ids.to(cuda) % 100, G.to(cuda))
        oa.step()
        if k == 0:
            continue
        ids_s.copy_(ids.to(cuda) % 100)
        G_s.copy_(G.to(cuda))
        g.replay()
        ob.note_replay()
    ob.flush()
    torch.cuda.synchronize()
    assert torch.equal(pa, pb)
    assert torch.equal(oa.state[pa]["exp_avg"], ob.state[pb]["exp_avg"])
    assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])
    assert int(ob.state[pb]["step"].item()) == 20


def test_lazy_row_catch_up_before_gather(cuda):
    """Rows read by a step (ids with duplicates) are caught up before the gather: they equal the
    every-row update's rows right away, without a flush; the other rows are still deferred."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(4)
    R, d = 400, 512
    w0 = torch.randn(R, d)
    pa = torch.nn.Parameter(w0.clone().to(cuda))
    pb = torch.nn.Parameter(w0.clone().to(cuda))
    oa = FusedAdam([pa], lr=4e-3)
    ob = FusedAdam([pb], lr=4e-3, lazy_rows=True)
    for k in range(9):
        ids, G = _case(R, d, 50, None, 900 + k)
        ids = torch.arange(R) if k == 0 else ids % 50  # every row has moments after step 1
        G = torch.randn(R, d) if k == 0 else G
        ids, G = ids.to(cuda), G.to(cuda)
        for o, p in ((oa, pa), (ob, pb)):
            o.zero_grad()
            o.row_grads.stash(p, None, ids, G)
            o.step()
    read = torch.tensor([3, 3, 77, 391, 120, 77], dtype=torch.int64, device=cuda)  # 77+: untouched rows
    ob.row_grads.catch_up_rows(pb, read)
    assert torch.equal(pa[read], pb[read])
    assert not torch.equal(pa[200:], pb[200:])  # deferred
    ob.row_grads.catch_up_rows(pb, read)  # idempotent
    assert torch.equal(pa[read], pb[read])
    ob.flush()
    assert torch.equal(pa, pb)
    assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])


def test_device_feed_stream_bit_exact(cuda):
    """GraphedStep's DeviceFeed (epoch staged on the device, batches gathered inside the captured
    step) yields the reference's triple stream: the golden 2-epoch stream of dataloader.py's
    sampler, full batches via DeviceFeed.fill, the ragged last batch as tensors."""
    from helpers import golden, tiny_config, tiny_data
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("stream.npz")
    cfg = tiny_config("LightGCN", False)
    data = tiny_data(cfg)
    init_seed(999)
    get_model("LightGCN")(cfg, data)
    B = int(g["batch_size"])
    s = TripleSampler(data, B, cuda)
    feed = s.device_feed()
    out = tuple(torch.zeros(B, dtype=torch.int64, device=cuda) for _ in range(3))
    for ep in range(2):
        got = []
        for u, p, n in s.epoch(out=out, feed=feed):
            if u is out[0]:
                feed.fill(*out)
            got.append([x.cpu().numpy().copy() for x in (u, p, n)])
        for k, key in enumerate("upn"):
            np.testing.assert_array_equal(np.concatenate([b[k] for b in got]), g[f"ep{ep}/{key}"])


def test_lazy_row_prefetch_multi(cuda):
    """RowGrads.prefetch_rows (side stream, both tables in one fr_adam_catch_up_rows_multi launch)
    catches the rows up exactly like per-table catch-up; the later per-table call is skipped."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(5)
    shapes = [(300, 256), (300, 64)]
    w0 = [torch.randn(R, d) for R, d in shapes]
    pa = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    pb = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    oa = FusedAdam(pa, lr=4e-3)
    ob = FusedAdam(pb, lr=4e-3, lazy_rows=True)
    for k in range(7):
        for o, ps in ((oa, pa), (ob, pb)):
            o.zero_grad()
            for t, ((R, d), p) in enumerate(zip(shapes, ps)):
                ids, G = _case(R, d, 40, None, 1000 + 10 * k + t)
                ids = torch.arange(R) if k == 0 else ids % 30
                G = torch.randn(R, d, generator=torch.Generator().manual_seed(k)) if k == 0 else G
                o.row_grads.stash(p, None, ids.to(cuda), G.to(cuda))
            o.step()
    ob.zero_grad()
    read = torch.tensor([5, 250, 250, 77, 3, 299], dtype=torch.int64, device=cuda)
    join = ob.row_grads.prefetch_rows([(p, read) for p in pb])
    join()
    for a, b in zip(pa, pb):
        assert torch.equal(a[read], b[read])
    assert any(w is pb[0] and i is read for w, i in ob.row_grads._prefetched)
    ob.flush()
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)


def test_healthrec_lazy_state_dict_flushes(cuda):
    """The trainer registers its optimiser's flush on the model: model.state_dict() (a checkpoint)
    holds the dense-Adam values of a lazily updated table, not the deferred ones."""
    from helpers import tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("CIKM_Model", True, cuda_graph=False)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model)
    opt = tr.optimizer
    assert opt.lazy_rows
    w = model.image_embedding.weight
    R, d = w.shape
    ref = torch.nn.Parameter(w.detach().clone())
    from FoodRec.engine.optim import FusedAdam
    oref = FusedAdam([ref], lr=opt.param_groups[0]["lr"])
    for k in range(4):  # first step touches every row, later ones alternate between two row sets
        ids = torch.arange(R, device=cuda) if k == 0 else torch.arange(k % 2, R, 2, device=cuda)
        G = torch.randn(ids.numel(), d, device=cuda)
        for o, p in ((opt, w), (oref, ref)):
            o.zero_grad()
            o.row_grads.stash(p, None, ids, G)
            o.step()
    raw = w.detach().clone()
    assert not torch.equal(raw, ref)  # deferred steps pending
    sd = model.state_dict()
    assert torch.equal(sd["image_embedding.weight"], ref)


def _row_or_dense(o, p, ids, G, dense):
    """Hand one step's gradient to ``o`` as rows (the row path) or as a dense .grad (summed on the
    host in a fixed order, so both optimisers see the same bits)."""
    o.zero_grad()
    if dense:
        p.grad = torch.zeros(p.shape).index_add_(0, ids.cpu(), G.cpu()).to(p.device)
    else:
        o.row_grads.stash(p, None, ids, G)


def test_lazy_rows_interleaved_dense_steps(cuda):
    """A lazily updated table that also takes dense steps (a dense .grad: clipping, a hook, more ids
    than the row path takes): the deferred steps are replayed before the dense update and every row
    is current through it afterwards.  Bit-identical to the every-row update after each flush, with
    several lazy steps pending before each dense one (stale history slots)."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(6)
    R, d = 257, 64
    w0 = torch.randn(R, d)
    pa = torch.nn.Parameter(w0.clone().to(cuda))
    pb = torch.nn.Parameter(w0.clone().to(cuda))
    oa = FusedAdam([pa], lr=3e-3)
    ob = FusedAdam([pb], lr=3e-3, lazy_rows=True, hist_cap=16)
    dense_at = {4, 5, 9, 15}
    for k in range(18):
        ids, G = _case(R, d, 30, None, 1300 + k)
        ids = torch.arange(R) if k == 0 else ids % 60
        G = torch.randn(R, d) if k == 0 else G
        ids, G = ids.to(cuda), G.to(cuda)
        for o, p in ((oa, pa), (ob, pb)):
            _row_or_dense(o, p, ids, G, k in dense_at)
            o.step()
        if k in (5, 12, 17):
            ob.flush()
            assert torch.equal(pa, pb), k
            for s_ in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(oa.state[pa][s_], ob.state[pb][s_]), (k, s_)
    assert int(ob.state[pb]["step"].item()) == 18


def test_lazy_rows_more_than_16_tables(cuda):
    """More lazy tables than one launch's argument block holds (16): the row update is split into
    launches of 16 and stays lazy for all of them (no fallback to a non-lazy update)."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(7)
    shapes = [(97 + 3 * t, 64 if t % 2 else 128) for t in range(19)]
    w0 = [torch.randn(R, d) for R, d in shapes]
    pa = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    pb = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    oa = FusedAdam(pa, lr=2e-3)
    ob = FusedAdam(pb, lr=2e-3, lazy_rows=True)
    for k in range(6):
        for o, ps in ((oa, pa), (ob, pb)):
            o.zero_grad()
            for t, ((R, d), p) in enumerate(zip(shapes, ps)):
                ids, G = _case(R, d, 20, None, 2000 + 50 * k + t)
                ids = torch.arange(R) if k == 0 else ids % 40
                G = torch.randn(R, d, generator=torch.Generator().manual_seed(k * 100 + t)) if k == 0 else G
                o.row_grads.stash(p, None, ids.to(cuda), G.to(cuda))
            o.step()
    assert all("lazy_last" in ob.state[p] for p in pb)
    assert not torch.equal(pa[0], pb[0])  # rows 40+ deferred
    ob.flush()
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
        assert torch.equal(oa.state[a]["exp_avg_sq"], ob.state[b]["exp_avg_sq"])


def test_lazy_rows_state_dict_round_trip(cuda):
    """optimizer.state_dict() -> torch.save -> torch.load -> load_state_dict() into a fresh FusedAdam,
    then more lazy steps: bit-identical to the uninterrupted run.  (torch's loader would cast the
    int32 per-row step index to float32 and leave 'step' on the host)"""
    import io
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(8)
    R, d = 300, 128
    w0 = torch.randn(R, d)
    pa = torch.nn.Parameter(w0.clone().to(cuda))
    pb = torch.nn.Parameter(w0.clone().to(cuda))
    oa = FusedAdam([pa], lr=3e-3, lazy_rows=True)
    ob = FusedAdam([pb], lr=3e-3, lazy_rows=True)
    cases = []
    for k in range(10):
        ids, G = _case(R, d, 25, None, 2500 + k)
        cases.append(((torch.arange(R) if k == 0 else ids % 70).to(cuda),
                      (torch.randn(R, d) if k == 0 else G).to(cuda)))
    for k in range(10):
        for o, p in ((oa, pa), (ob, pb)):
            if o is ob and k == 5:
                buf = io.BytesIO()
                torch.save(ob.state_dict(), buf)
                buf.seek(0)
                sd = torch.load(buf, weights_only=True)
                pb_new = torch.nn.Parameter(pb.detach().clone())
                ob = FusedAdam([pb_new], lr=3e-3, lazy_rows=True)
                ob.load_state_dict(sd)
                st = ob.state[pb_new]
                assert st["step"].dtype == torch.int64 and st["step"].is_cuda
                assert "lazy_last" not in st and st["exp_avg"].dtype == torch.float32
                pb, o, p = pb_new, ob, pb_new
            o.zero_grad()
            o.row_grads.stash(p, None, *cases[k])
            o.step()
    oa.flush()
    ob.flush()
    assert torch.equal(pa, pb)
    for s_ in ("exp_avg", "exp_avg_sq"):
        assert torch.equal(oa.state[pa][s_], ob.state[pb][s_]), s_
    assert int(ob.state[pb]["step"].item()) == 10


def test_feed_batch_one_launch_matches_gathers(cuda):
    """fr_feed_batch (DeviceFeed.fill with the batch features): (u, pos, neg) equal to the golden
    reference stream and to the index_select feed, and the [pos; neg] features (item ids, ingredient
    codes, counts, health multi-hot, padding mask) equal to torch gathers of the side tables; the
    plain-mode gather (LazyBatch pn_ keys) equal too."""
    from helpers import golden, tiny_config, tiny_data
    from FoodRec.engine.sampler import BatchFeatures, TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("stream.npz")
    cfg = tiny_config("CIKM_Model", False)
    data = tiny_data(cfg)
    init_seed(999)
    get_model("LightGCN")(tiny_config("LightGCN", False), tiny_data(tiny_config("LightGCN", False)))
    B = int(g["batch_size"])
    s = TripleSampler(data, B, cuda)
    feed = s.device_feed()
    feats = BatchFeatures(data, cuda)
    out = tuple(torch.zeros(B, dtype=torch.int64, device=cuda) for _ in range(3))
    got = []
    for u, p, n in s.epoch(out=out, feed=feed):
        if u is out[0]:
            pre = feed.fill(*out, feats)
            assert pre is not None
            pn = torch.cat([out[1], out[2]])
            assert torch.equal(pre["pn_i_id"], pn)
            assert torch.equal(pre["pn_ingre_code"], feats.ingre_code[pn])
            assert torch.equal(pre["pn_ingre_num"], feats.ingre_num[pn])
            assert torch.equal(pre["pn_hl_mh"], feats.health[pn])
            assert torch.equal(pre["pn_pad_kpm"] == float("-inf"), feats.ingre_code[pn] == data.num_ingredients)
            assert torch.all((pre["pn_pad_kpm"] == 0) | (pre["pn_pad_kpm"] == float("-inf")))
            lb = feats.batch(out[0].clone(), out[1].clone(), out[2].clone())  # plain mode (lazy keys)
            for k in ("pn_i_id", "pn_ingre_code", "pn_ingre_num", "pn_hl_mh", "pn_pad_kpm"):
                assert torch.equal(lb[k], pre[k]), k
        got.append([x.cpu().numpy().copy() for x in (u, p, n)])
    for k, key in enumerate("upn"):
        np.testing.assert_array_equal(np.concatenate([b[k] for b in got]), g[f"ep0/{key}"])


def test_feed_batch_bad_id_is_reported(cuda):
    """fr_feed_batch replaces an out-of-range item id by item 0 in every output (in feed
    mode p / n too, so they agree with pn and the features) and sets the sticky flag the trainer
    reads at epoch end (BatchFeatures.check_ids raises)."""
    from helpers import tiny_config, tiny_data
    from FoodRec.engine.sampler import BatchFeatures, TripleSampler
    cfg = tiny_config("CIKM_Model", False)
    data = tiny_data(cfg)
    B = 64
    s = TripleSampler(data, B, cuda, replay_python_random=False)
    feed = s.device_feed()
    feats = BatchFeatures(data, cuda)
    out = tuple(torch.zeros(B, dtype=torch.int64, device=cuda) for _ in range(3))
    it = s.epoch(out=out, feed=feed)
    next(it)
    feed.negs[3] = feats.ingre_code.shape[0] + 7  # corrupt staged negative of batch 0, row 3
    pre = feed.fill(*out, feats)
    torch.cuda.synchronize()
    assert int(out[2][3]) == 0 and int(pre["pn_i_id"][B + 3]) == 0
    assert torch.equal(pre["pn_i_id"], torch.cat([out[1], out[2]]))
    assert torch.equal(pre["pn_ingre_code"][B + 3], feats.ingre_code[0])
    with pytest.raises(RuntimeError, match="outside the item table"):
        feats.check_ids()
    feats.check_ids()  # the flag was cleared by the report
    lb = feats.batch(out[0].clone(), out[1].clone(), out[2].clone())  # a clean batch: no report
    torch.cuda.synchronize()
    assert torch.equal(lb["pn_i_id"], pre["pn_i_id"])
    feats.check_ids()


@pytest.mark.parametrize("n", [1024 * 20, 1000, 17])
@pytest.mark.parametrize("hot", [None, 19987, 5])
def test_embedding_bwd_atomic_matches_sorted(cuda, hot, n):
    """fr_embedding_bwd_atomic (float atomics, the hot row pre-summed per workgroup) against the
    deterministic counting-sort scatter: equal to fp32 rounding (rel 1e-5 of the row scale), the
    padding_idx row skipped, out-of-range ids ignored; HealthRec's shape ([1024 x 20] positions,
    about half of them the padding ingredient 19987, into 19988 rows), and a ragged position count."""
    from FoodRec.engine import ops
    g = torch.Generator().manual_seed(3)
    R = 19988
    ids = torch.randint(0, R - 1, (n,), generator=g)
    ids[torch.rand(n, generator=g) < 0.5] = 19987
    ids[7] = R + 5  # out of range: skipped by both paths
    G = torch.randn(n, 64, generator=g)
    idc, Gc = ids.to(cuda), G.to(cuda)
    ref = ops.scatter_rows(idc, Gc, R, None)
    got = ops.scatter_rows(idc, Gc, R, None, hot_row=hot)
    scale = ops.scatter_rows(idc, Gc.abs(), R, None)
    assert torch.all((got - ref).abs() <= 1e-5 * scale + 1e-6)
    pad_ref = ops.scatter_rows(idc, Gc, R, 11)
    pad_got = ops.scatter_rows(idc, Gc, R, 11, hot_row=hot)
    assert torch.all(pad_got[11] == 0)
    assert torch.all((pad_got - pad_ref).abs() <= 1e-5 * scale + 1e-6)


@pytest.mark.parametrize("n", [1024 * 20, 1000, 17])
def test_norms_bwd_scatter_matches_two_launches(cuda, n):
    """fr_norms_bwd_scatter (HealthRec's deferred ingredient rows formed inside the scatter) against
    fr_norms_bwd_coef + the deterministic scatter: equal to fp32 rounding (rel 1e-5 of the row
    scale); the padding positions take G only (pre-summed into the pad row), the two halves their
    own coefficient, out-of-range ids skipped, a zero norm gives a zero coefficient."""
    from FoodRec.engine import native, ops
    g = torch.Generator().manual_seed(5)
    R, pad = 19988, 19987
    ids = torch.randint(0, R - 1, (n,), generator=g)
    ids[torch.rand(n, generator=g) < 0.5] = pad
    ids[min(7, n - 1)] = R + 5
    G = torch.randn(n, 64, generator=g)
    E = torch.randn(n, 64, generator=g)
    half = n // 2
    for nrm_h, gn_h in (([3.0, 2.0], [0.7, -1.3]), ([0.0, 2.0], [0.7, -1.3])):
        idc, Gc, Ec = ids.to(cuda), G.to(cuda), E.to(cuda)
        nrm, gn = torch.tensor(nrm_h, device=cuda), torch.tensor(gn_h, device=cuda)
        rows = torch.empty_like(Gc)
        native.check(native.lib().fr_norms_bwd_coef(idc.data_ptr(), n, half, pad, Gc.data_ptr(), Ec.data_ptr(),
                                                    gn.data_ptr(), 1, nrm.data_ptr(), rows.data_ptr(), 0), "coef")
        ref = ops.scatter_rows(idc, rows, R, None)
        got = torch.zeros(R, 64, device=cuda)
        ops.norms_scatter_into(idc, Gc, Ec, gn, nrm, half, pad, got)
        scale = ops.scatter_rows(idc, rows.abs(), R, None) + ops.scatter_rows(idc, Ec.abs(), R, None)
        assert torch.all((got - ref).abs() <= 1e-5 * scale + 1e-6)


@pytest.mark.parametrize("slices", [1, 3, 8])
def test_lazy_rows_background_slices(cuda, slices):
    """Background slice replay (fr_adam_catch_up_slice, issued by prefetch_rows behind the batch's
    catch-up on the side stream and joined before the optimiser step): each step one slice of
    every table replays its backlog.  Without any flush, every row is current within ``slices``
    steps; after a flush the tables, moments and step counters are bit-identical to the every-row
    update.  Two tables of different widths in one launch, rows gathered before the step."""
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(8)
    shapes = [(1001, 128), (1001, 32)]
    w0 = [torch.randn(R, d) for R, d in shapes]
    pa = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    pb = [torch.nn.Parameter(w.clone().to(cuda)) for w in w0]
    oa = FusedAdam(pa, lr=3e-3)
    ob = FusedAdam(pb, lr=3e-3, lazy_rows=True, lazy_slices=slices)
    for k in range(14):
        ids, _ = _case(1001, 4, 40, None, 3100 + k)
        ids = ids.to(cuda)
        Gs = [torch.randn(40, d, generator=torch.Generator().manual_seed(3200 + 7 * k + d)).to(cuda)
              for _, d in shapes]
        for o, ps in ((oa, pa), (ob, pb)):
            o.zero_grad()
            join = o.row_grads.prefetch_rows([(p, ids) for p in ps])
            join()
            for p, G in zip(ps, Gs):
                o.row_grads.stash(p, None, ids, G)
            o.step()
        if k >= slices:  # every row replayed within the last `slices` steps (before this step)
            for p in pb:
                st = ob.state[p]
                lag = int(st["step"].item()) - int(st["lazy_last"].min().item())
                assert lag <= slices, (k, lag)
        if k in (6, 13):
            ob.flush()
            for a_, b_ in zip(pa, pb):
                assert torch.equal(a_, b_), k
                for s_ in ("exp_avg", "exp_avg_sq"):
                    assert torch.equal(oa.state[a_][s_], ob.state[b_][s_]), (k, s_)


def test_rounding_shortcuts_bit_exact(cuda):
    """The lazy-row replay's in-range forms (v_rcp + fma chain division without the scale / fix-up
    steps, bare v_sqrt_f32 + residual selection) and sqrt_rn's small-input scaling return the IEEE
    correctly rounded fp32 result: 2^24 random operand sets per form on the device, zero mismatches
    (division vs __fdiv_rn; sqrt vs the correctly rounded double root, denormals included)."""
    from FoodRec.engine import native
    bad = torch.zeros(3, dtype=torch.int64, device=cuda)
    for seed in (1, 2):
        native.check(native.lib().fr_adam_rounding_selftest(1 << 23, seed, bad.data_ptr(),
                                                            native.stream_of(bad)), "fr_adam_rounding_selftest")
    assert bad.tolist() == [0, 0, 0]


def test_rows_side_stream_first_steps_equal_inline(cuda):
    """FusedAdam.step's row-table update on the side stream (FR_ROWS_SIDE_STREAM=1, the default) vs
    on the current stream, over the first two HealthRec steps (lazy rows, deterministic scatters).
    Step 1 is the one that creates the Adam state, the lazy bookkeeping, the lr scalar and the ticket
    words on the current stream: the side stream must be ordered after them (else it reads
    uninitialised moments and the queued zero fills overwrite its update).  Every parameter and
    moment agrees (rel 1e-6)."""
    from helpers import golden, tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import optim
    from FoodRec.utils.utils import get_model, init_seed
    g = golden("model_CIKM_Model.npz")
    batch = {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}
    runs = []
    det0 = torch.are_deterministic_algorithms_enabled()
    side0 = optim.ROWS_SIDE_STREAM
    torch.use_deterministic_algorithms(True)
    try:
        for side in (True, False):
            optim.ROWS_SIDE_STREAM = side
            cfg = tiny_config("CIKM_Model", True, cuda_graph=False, lazy_row_adam=True, deterministic=True)
            data = tiny_data(cfg)
            init_seed(999)
            model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
            tr = Trainer(cfg, model)
            st = tr.new_step_state()
            for k in range(2):
                tr.train_step(batch, k, st)
            tr.optimizer.flush()
            torch.cuda.synchronize()
            runs.append((model, tr.optimizer))
    finally:
        optim.ROWS_SIDE_STREAM = side0
        torch.use_deterministic_algorithms(det0)
    (ma, oa), (mb, ob) = runs
    for (k, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-9, msg=k)
        if a in oa.state:
            assert int(oa.state[a]["step"]) == int(ob.state[b]["step"]) == 2, k
            for s_ in ("exp_avg", "exp_avg_sq"):
                torch.testing.assert_close(oa.state[a][s_], ob.state[b][s_], rtol=1e-6, atol=1e-12, msg=(k, s_))
