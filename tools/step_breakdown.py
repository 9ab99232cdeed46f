"""Per-step GPU time by kernel from a rocprofv3 kernel trace: the window between the first and the
last Adam launch (the training steps), normalised per step.  Usage: step_breakdown.py trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("(anonymous namespace)::adam_kernel")]
lo, hi = adam[0], adam[-1]
# steps = number of Adam launch groups (launches of one step are back-to-back)
steps = 1 + sum(1 for a, b in zip(adam, adam[1:]) if b - a > 3)
agg = defaultdict(lambda: [0, 0.0])
busy = 0.0
for r in rows[lo:hi + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"]
    for key in ("Cijk_", "rocprim", "__amd_rocclr"):
        if name.startswith(key) or key in name[:40]:
            name = name[:60]
    agg[name][0] += 1
    agg[name][1] += d
    busy += d
span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3
print(f"steps {steps}  window {span/1e3:.1f} ms  kernel-busy {busy/1e3:.1f} ms  per step: busy {busy/steps:.0f} us, "
      f"launches {sum(v[0] for v in agg.values())/steps:.0f}")
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{n/steps:6.1f}/step {t/steps:8.1f} us/step {t/n:8.1f} us/launch  {name[:110]}")
