"""Micro-benchmark of the fused encoder layer (fr_encoder_fwd / fr_encoder_bwd) at HealthRec's shape
(2B = 1024 sequences x 20 tokens, d=64, 2 heads, FF 256, dropout 0.5) vs torch's
nn.TransformerEncoderLayer on the same device.  Prints one JSON line (per-call ms, HIP events on
the launch stream)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-food-recommendation_amd"))

import torch  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", type=int, default=1024)
    ap.add_argument("--L", type=int, default=20)
    ap.add_argument("--p", type=float, default=0.5)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--phases", action="store_true", help="per-phase s_memtime stamps of workgroup 0")
    ap.add_argument("--reduce-mode", type=int, default=-1,
                    help="fr_encoder_options: 0 column-slice partial reduction (default), 1 row-streaming")
    ap.add_argument("--no-torch", action="store_true", help="skip torch's own layer")
    args = ap.parse_args()
    from FoodRec.engine import native, ops
    native.check(native.lib().fr_encoder_options(args.reduce_mode), "fr_encoder_options")
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    layer = torch.nn.TransformerEncoderLayer(64, 2, 256, dropout=args.p, activation="gelu").to(dev)
    params = [layer.self_attn.in_proj_weight, layer.self_attn.in_proj_bias, layer.self_attn.out_proj.weight,
              layer.self_attn.out_proj.bias, layer.norm1.weight, layer.norm1.bias, layer.linear1.weight,
              layer.linear1.bias, layer.linear2.weight, layer.linear2.bias, layer.norm2.weight, layer.norm2.bias]
    x = torch.randn(args.ns, args.L, 64, device=dev, requires_grad=True)
    pad = torch.rand(args.ns, args.L, device=dev) < 0.4
    pad[:, 0] = False
    mask = torch.zeros(args.ns, args.L, device=dev).masked_fill(pad, float("-inf"))
    cfg = ops.EncoderConfig((1e-5, 1e-5), (args.p,) * 4, True, 1, dev)
    g = torch.randn(args.ns, args.L, 64, device=dev)

    holder = {}

    def fwd():
        holder["y"] = ops.encoder_layer(x, mask, cfg, params)

    def fwd_bwd():
        ops.encoder_layer(x, mask, cfg, params).backward(g)

    xs = x.detach().transpose(0, 1).contiguous().requires_grad_(True)

    def torch_fwd_bwd():
        layer(xs, src_key_padding_mask=pad).backward(g.transpose(0, 1))

    with torch.no_grad():
        t_fwd = timed(fwd, args.iters)
    t_fb = timed(fwd_bwd, args.iters)
    t_torch = 0.0 if args.no_torch else timed(torch_fwd_bwd, args.iters)
    phases = None
    if args.phases:
        import ctypes
        import numpy as np
        lib = native.lib()
        native.check(lib.fr_encoder_profile(1, None), "fr_encoder_profile")
        for _ in range(3):
            fwd_bwd()
        torch.cuda.synchronize()
        marks = np.zeros((2, 32), np.uint64)
        native.check(lib.fr_encoder_profile(0, ctypes.c_void_p(marks.ctypes.data)), "fr_encoder_profile")
        phases = {}
        for kind, name in ((0, "fwd"), (1, "bwd")):
            m = marks[kind].astype(np.int64)
            idx = sorted((k for k in range(32) if m[k] != 0), key=lambda k: m[k])  # in time order
            phases[name] = {f"{a}->{b}": int(m[b] - m[a]) for a, b in zip(idx, idx[1:])}
            phases[name]["total"] = int(m[idx[-1]] - m[idx[0]])
    print(json.dumps({"ns": args.ns, "L": args.L, "p": args.p, "fused_fwd_ms": round(t_fwd, 4),
                      "fused_fwd_bwd_ms": round(t_fb, 4), "fused_bwd_ms": round(t_fb - t_fwd, 4),
                      "torch_fwd_bwd_ms": round(t_torch, 4), "phases_cycles": phases}))


if __name__ == "__main__":
    main()
