"""Time fr_topk_scores (fused full-sort top-k) on synthetic tables: variants by k, masking, d, dtype.

    python tools/bench_topk.py [--users 32768] [--items 1000000] [--d 256] [--k 20] [--reps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=32768)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--only", default=None, help="k,mask (e.g. 20,0) to run one variant")
    args = ap.parse_args()
    import torch
    from FoodRec.engine import ops
    dev = torch.device("cuda:0")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    g = torch.Generator(device=dev).manual_seed(0)
    U = (torch.randn(args.users, args.d, device=dev, generator=g) * 0.1).to(dt)
    I = (torch.randn(args.items, args.d, device=dev, generator=g) * 0.1).to(dt)
    # exclusion CSR: 20 random items per user (sorted)
    ex_items = torch.sort(torch.randint(0, args.items, (args.users, 20), device=dev, generator=g), dim=1).values
    rp = torch.arange(0, 20 * args.users + 1, 20, device=dev, dtype=torch.int64)
    ex = (rp, ex_items.reshape(-1).to(torch.int32).contiguous(), 0)
    flops = ops.topk_flops(args.users, args.items, args.d)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    variants = ((20, True), (20, False), (1, False), (32, False))
    if args.only:
        kk, mm = args.only.split(",")
        variants = ((int(kk), bool(int(mm))),)
    for k, mask in variants:
        kw = {"exclude": ex} if mask else {}
        ops.full_sort_topk(U, I, k, **kw)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.reps):
            ops.full_sort_topk(U, I, k, **kw)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(f"k={k:2d} mask={mask!s:5} d={args.d} {args.dtype}: {ms:8.3f} ms  "
              f"{flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
