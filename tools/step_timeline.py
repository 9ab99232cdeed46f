"""One graphed step's kernel timeline from a rocprofv3 kernel trace: start offset, duration and
queue of every kernel between two consecutive feed_batch launches (the step boundary), to read the
critical path of a multi-stream step.

    python tools/step_timeline.py run_kernel_trace.csv [step_index_from_end]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    feeds = [i for i, r in enumerate(rows) if "feed_batch_kernel" in r["Kernel_Name"]]
    a, b = feeds[-k - 1], feeds[-k]
    t0 = int(rows[a]["Start_Timestamp"])
    queues = {}
    for r in rows[a:b]:
        q = queues.setdefault(r["Queue_Id"], len(queues))
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        print(f"q{q} {s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name}")
    print("step", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3, "us")


if __name__ == "__main__":
    main()
