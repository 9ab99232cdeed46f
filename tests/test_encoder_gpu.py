"""Fused Transformer encoder layer (fr_encoder_fwd / fr_encoder_bwd) vs the oracle.

The layer replaces nn.TransformerEncoderLayer(64, 2, 256, dropout=p, activation=gelu) of HealthRec's
ingredient encoder (cikm_model.py:33-35, 232-238).  Oracle: oracle.ops.encoder_layer_f64, a float64
restatement of torch's post-norm training forward (pinned against torch's own module by
tests/test_encoder_cpu.py), fed the kernel's dropout keep-masks regenerated on the host by
oracle.ops.encoder_keep_masks.

Tolerances (fp32 MFMA GEMMs + fp32 softmax/LayerNorm vs float64):
  outputs              : |err| <= 2e-5 * max|ref| + 2e-6
  dx, parameter grads  : |err| <= 1e-4 * max|ref grad| + 1e-6
  dropout masks        : exact (the same hash)
"""
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


def _params(gen, scale=0.15):
    shapes = [(192, 64), (192,), (64, 64), (64,), (64,), (64,), (256, 64), (256,), (64, 256), (64,), (64,), (64,)]
    ps = []
    for k, s in enumerate(shapes):
        t = torch.randn(s, generator=gen, dtype=torch.float64) * scale
        if k in (4, 10):  # LayerNorm gammas around 1
            t = 1.0 + t
        ps.append(t)
    return ps


def _run(cuda, NS, L, drop, gelu=True, with_mask=True, seed=1234, counter=0):
    from FoodRec.engine import ops
    gen = torch.Generator().manual_seed(NS * 31 + L)
    x = torch.randn(NS, L, 64, generator=gen, dtype=torch.float64)
    mask = None
    if with_mask:
        pad = torch.rand(NS, L, generator=gen) < 0.4
        pad[:, 0] = False
        mask = torch.zeros(NS, L, dtype=torch.float64).masked_fill(pad, float("-inf"))
    params = _params(gen)
    gout = torch.randn(NS, L, 64, generator=gen, dtype=torch.float64)

    cfg = ops.EncoderConfig((1e-5, 1e-5), drop, gelu, seed, cuda)
    cfg.counter.fill_(counter)
    xg = x.float().to(cuda).requires_grad_(True)
    pg = [p.float().to(cuda).requires_grad_(True) for p in params]
    out = ops.encoder_layer(xg, None if mask is None else mask.float().to(cuda), cfg, pg)
    out.backward(gout.float().to(cuda))
    assert int(cfg.counter.item()) == counter + 1

    masks = O.encoder_keep_masks(seed, counter, NS, L, drop)
    xr = x.clone().requires_grad_(True)
    pr = [p.clone().requires_grad_(True) for p in params]
    ref = O.encoder_layer_f64(xr, mask, pr, masks, drop, gelu=gelu)
    ref.backward(gout)
    return out, xg, pg, ref, xr, pr


def _check(out, xg, pg, ref, xr, pr):
    o = out.detach().double().cpu()
    assert (o - ref.detach()).abs().max() <= 2e-5 * ref.abs().max() + 2e-6
    names = ["x", "in_proj_weight", "in_proj_bias", "out_proj.weight", "out_proj.bias", "norm1.weight",
             "norm1.bias", "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias", "norm2.weight",
             "norm2.bias"]
    for name, a, b in zip(names, [xg] + pg, [xr] + pr):
        ga, gb = a.grad.double().cpu(), b.grad
        assert (ga - gb).abs().max() <= 1e-4 * gb.abs().max() + 1e-6, name


@pytest.mark.parametrize("NS,L", [(1024, 20), (1027, 20), (333, 16), (101, 8), (50, 5), (7, 20)])
def test_encoder_layer_no_dropout(cuda, NS, L):
    """p = 0 (the reference goldens' setting): outputs and all 13 gradients vs float64, including a
    partial last workgroup (NS not a multiple of 80 / L)."""
    _check(*_run(cuda, NS, L, (0.0, 0.0, 0.0, 0.0)))


@pytest.mark.parametrize("gelu", [True, False])
def test_encoder_layer_dropout_masks(cuda, gelu):
    """p = 0.5 at all four sites (HealthRec's attention_probs_dropout_prob): the kernel's masks are
    regenerated on the host from the same hash, so forward and backward match exactly-masked float64."""
    _check(*_run(cuda, 257, 20, (0.5, 0.5, 0.5, 0.5), gelu=gelu, counter=7))


def test_encoder_layer_mixed_dropout_no_mask(cuda):
    _check(*_run(cuda, 96, 10, (0.1, 0.0, 0.3, 0.2), with_mask=False, seed=99, counter=3))


def test_encoder_in_cuda_graph(cuda):
    """Captured once, replayed twice: every replay reads the device counter, so masks differ
    between replays and the backward of each replay uses its own forward's masks."""
    from FoodRec.engine import ops
    gen = torch.Generator().manual_seed(0)
    params = [p.float().to(cuda).requires_grad_(True) for p in _params(gen)]
    x = torch.randn(200, 20, 64, generator=gen).to(cuda).requires_grad_(True)
    cfg = ops.EncoderConfig((1e-5, 1e-5), (0.5, 0.5, 0.5, 0.5), True, 77, cuda)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):  # warm-up (allocator, autograd)
            ops.encoder_layer(x, None, cfg, params).sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    x.grad = None
    with torch.cuda.graph(g):
        out = ops.encoder_layer(x, None, cfg, params)
        out.sum().backward()
    outs, dxs = [], []
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        outs.append(out.detach().clone())
        dxs.append(x.grad.detach().clone())
    assert not torch.equal(outs[0], outs[1])
    c = int(cfg.counter.item())
    for k, (o, dx) in enumerate(zip(outs, dxs)):
        masks = O.encoder_keep_masks(77, c - 2 + k, 200, 20, (0.5,) * 4)
        xr = x.detach().double().cpu().requires_grad_(True)
        pr = [p.detach().double().cpu() for p in params]
        ref = O.encoder_layer_f64(xr, None, pr, masks, (0.5,) * 4)
        ref.sum().backward()
        assert (o.double().cpu() - ref.detach()).abs().max() <= 2e-5 * ref.abs().max() + 2e-6
        assert (dx.double().cpu() - xr.grad).abs().max() <= 1e-4 * xr.grad.abs().max() + 1e-6


def test_encoder_deterministic(cuda):
    a = _run(cuda, 300, 20, (0.5, 0.5, 0.5, 0.5), counter=2)
    b = _run(cuda, 300, 20, (0.5, 0.5, 0.5, 0.5), counter=2)
    assert torch.equal(a[0], b[0])
    for pa, pb in zip([a[1]] + a[2], [b[1]] + b[2]):
        assert torch.equal(pa.grad, pb.grad)


@pytest.mark.parametrize("NS,L", [(474, 20), (1027, 20), (7, 20), (333, 16), (101, 8), (50, 5), (33, 10), (9, 4)])
def test_encoder_writes_stay_in_bounds(cuda, NS, L):
    """Every buffer of fr_encoder_fwd / fr_encoder_bwd sits between guard zones of a sentinel value:
    the kernels write only inside their outputs (no row of a partial workgroup or padding tile lands
    past an output's end or in front of it) and never write their inputs or the saved tensors."""
    import ctypes

    from FoodRec.engine import native, ops
    lib = native.lib()
    G = 4096
    SENT = 12345.0
    T = NS * L
    gen = torch.Generator().manual_seed(NS + L)

    def guarded(n, fill=None):
        buf = torch.full((n + 2 * G,), SENT, dtype=torch.float32, device=cuda)
        if fill is not None:
            buf[G:G + n] = fill.reshape(-1).to(cuda)
        return buf, buf[G:G + n]

    def intact(buf, n):
        return bool((buf[:G] == SENT).all()) and bool((buf[G + n:] == SENT).all())

    x_b, x = guarded(T * 64, torch.randn(T * 64, generator=gen))
    pad = torch.rand(NS, L, generator=gen) < 0.3
    pad[:, 0] = False
    m_b, m = guarded(T, torch.zeros(NS, L).masked_fill(pad, float("-inf")))
    params = [p.float() for p in _params(gen)]
    pbufs = [guarded(p.numel(), p) for p in params]
    pp = (ctypes.c_void_p * 12)(*[v.data_ptr() for _, v in pbufs])
    eps = (ctypes.c_float * 2)(1e-5, 1e-5)
    drop = (ctypes.c_float * 4)(0.1, 0.1, 0.1, 0.1)
    counter = torch.zeros(1, dtype=torch.int64, device=cuda)
    seed_used = torch.zeros(1, dtype=torch.int64, device=cuda)
    sizes = {"out": T * 64, "qkv": T * 192, "ctx": T * 64, "y1": T * 64, "fact": T * 256,
             "dact": int(lib.fr_encoder_dact_numel(NS, L)), "y2": T * 64, "st1": T * 2, "st2": T * 2}
    outs = {k: guarded(n) for k, n in sizes.items()}
    s = native.stream_of(x)
    native.check(lib.fr_encoder_fwd(x.data_ptr(), m.data_ptr(), NS, L, pp, eps, drop, 5, 1, counter.data_ptr(),
                                    seed_used.data_ptr(), *[outs[k][1].data_ptr() for k in sizes], s),
                 "fr_encoder_fwd")
    torch.cuda.synchronize()
    for k, n in sizes.items():
        assert intact(outs[k][0], n), f"forward wrote outside {k}"
    snap = {k: v[0].clone() for k, v in outs.items()}
    g_b, g = guarded(T * 64, torch.randn(T * 64, generator=gen))
    g_snap = g_b.clone()
    dx_b, dx = guarded(T * 64)
    gr_b, gr = guarded(int(lib.fr_encoder_grad_numel()))
    nparts = int(lib.fr_encoder_partials(NS, L))
    pa_b, pa = guarded(nparts)
    native.check(lib.fr_encoder_bwd(g.data_ptr(), x.data_ptr(), m.data_ptr(), NS, L, pp, eps, drop, 5, 1,
                                    seed_used.data_ptr(), *[outs[k][1].data_ptr() for k in list(sizes)[1:]],
                                    dx.data_ptr(), gr.data_ptr(), pa.data_ptr(), nparts, None, None, s),
                 "fr_encoder_bwd")
    torch.cuda.synchronize()
    assert intact(dx_b, T * 64), "backward wrote outside dx"
    assert intact(gr_b, int(lib.fr_encoder_grad_numel())), "backward wrote outside the gradient"
    assert intact(pa_b, nparts), "backward wrote outside the partials"
    # the same backward again, reducing the first call's partials in its own launch (a stacked
    # encoder's folded reduction) and leaving its own unreduced: the folded sum stays inside its
    # output, equals fr_encoder_reduce's to fp32 reassociation, and the first partials are not written
    pa_snap = pa_b.clone()
    pb_b, pb = guarded(nparts)
    gf_b, gf = guarded(int(lib.fr_encoder_grad_numel()))
    dx2_b, dx2 = guarded(T * 64)
    native.check(lib.fr_encoder_bwd(g.data_ptr(), x.data_ptr(), m.data_ptr(), NS, L, pp, eps, drop, 5, 1,
                                    seed_used.data_ptr(), *[outs[k][1].data_ptr() for k in list(sizes)[1:]],
                                    dx2.data_ptr(), None, pb.data_ptr(), nparts, pa.data_ptr(), gf.data_ptr(), s),
                 "fr_encoder_bwd (folded reduction)")
    torch.cuda.synchronize()
    assert intact(gf_b, int(lib.fr_encoder_grad_numel())) and intact(pb_b, nparts) and intact(dx2_b, T * 64)
    assert torch.equal(pa_b, pa_snap), "the folded reduction wrote the partials it reads"
    assert torch.equal(dx2, dx) and torch.equal(pb, pa), "the backward itself must not change"
    torch.testing.assert_close(gf, gr, rtol=1e-5, atol=1e-6 * float(gr.abs().max()))
    assert torch.equal(g_b, g_snap), "backward wrote its upstream gradient"
    for k in sizes:
        assert torch.equal(outs[k][0], snap[k]), f"backward wrote the saved {k}"
    for (b, v), p in zip(pbufs, params):
        assert intact(b, p.numel()) and torch.equal(v.cpu(), p.reshape(-1)), "a parameter was written"
    assert intact(x_b, T * 64) and intact(m_b, T)
    assert torch.isfinite(dx).all() and torch.isfinite(gr).all()


@pytest.mark.parametrize("NS,L,drop", [(1024, 20, (0.5, 0.5, 0.5, 0.5)), (257, 20, (0.0,) * 4), (101, 8, (0.1, 0.2, 0.3, 0.4))])
def test_encoder_stack_two_layers(cuda, NS, L, drop):
    """ops.encoder_stack (HealthRec's 2-layer ingredient encoder as ONE autograd node, layer 2's
    weight-gradient reduction folded into layer 1's backward launch) vs two float64 layers with the
    kernels' own masks: output 2e-5 * max, dx and all 24 parameter gradients 1e-4 * max."""
    from FoodRec.engine import ops
    gen = torch.Generator().manual_seed(NS + 7 * L)
    x = torch.randn(NS, L, 64, generator=gen, dtype=torch.float64)
    pad = torch.rand(NS, L, generator=gen) < 0.4
    pad[:, 0] = False
    mask = torch.zeros(NS, L, dtype=torch.float64).masked_fill(pad, float("-inf"))
    params = [_params(gen), _params(gen)]
    gout = torch.randn(NS, L, 64, generator=gen, dtype=torch.float64)
    cfgs = [ops.EncoderConfig((1e-5, 1e-5), drop, True, 100 + k, cuda) for k in range(2)]
    for k, c in enumerate(cfgs):
        c.counter.fill_(3 + k)
    xg = x.float().to(cuda).requires_grad_(True)
    pg = [[p.float().to(cuda).requires_grad_(True) for p in ps] for ps in params]
    out = ops.encoder_stack(xg, mask.float().to(cuda), cfgs, pg)
    out.backward(gout.float().to(cuda))
    xr = x.clone().requires_grad_(True)
    pr = [[p.clone().requires_grad_(True) for p in ps] for ps in params]
    h = xr
    for k in range(2):
        masks = O.encoder_keep_masks(100 + k, 3 + k, NS, L, drop)
        h = O.encoder_layer_f64(h, mask, pr[k], masks, drop, gelu=True)
    h.backward(gout)
    o = out.detach().double().cpu()
    assert (o - h.detach()).abs().max() <= 2e-5 * h.abs().max() + 2e-6
    for a, b in zip([xg] + pg[0] + pg[1], [xr] + pr[0] + pr[1]):
        ga, gb = a.grad.double().cpu(), b.grad
        assert (ga - gb).abs().max() <= 1e-4 * gb.abs().max() + 1e-6
