"""Average duration of named kernels inside the graphed training steps of a rocprofv3 kernel trace
of bench.py (steps delimited by feed_batch launches; the last ``eager`` feed launches belong to the
eager kernel passes and are skipped), for comparison with the bench line's in-graph stamps.

    python tools/graph_kernel_avg.py run_kernel_trace.csv [eager=20] [steps=20]
"""
import csv
import json
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    eager = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    feeds = [i for i, r in enumerate(rows) if "feed_batch_kernel" in r["Kernel_Name"]]
    bounds = feeds[-eager - nsteps - 1:-eager]
    per = {}
    for a, b in zip(bounds, bounds[1:]):
        for r in rows[a:b]:
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            per.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    steps = len(bounds) - 1
    out = {n: {"calls_per_step": len(v) / steps, "avg_us": round(sum(v) / len(v), 2)} for n, v in per.items()}
    eb, er = out.get("enc_bwd_kernel<20>"), out.get("enc_reduce_kernel")
    if eb and er:
        out["_encoder_bwd_call_us"] = round(eb["avg_us"] + er["avg_us"], 2)
    out["_steps"] = steps
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
