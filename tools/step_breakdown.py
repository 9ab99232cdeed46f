"""Per-step GPU time by kernel from a rocprofv3 kernel trace: the window between the first Adam
launch and the last Adam launch of the first `--steps` step groups (the HealthRec training steps;
later groups belong to other bench legs), normalised per step.
Usage: step_breakdown.py trace.csv [top] [--steps K]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
max_steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else None
if max_steps is not None:
    args = [a for a in args if a != str(max_steps)]
rows = list(csv.DictReader(open(args[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# one optimiser launch per step marks the step: the row-gradient Adam when present, else the dense one
adam = ([i for i, r in enumerate(rows) if "::adam_lazy_rows_kernel<false>" in r["Kernel_Name"]]
        or [i for i, r in enumerate(rows) if "::adam_kernel<true," in r["Kernel_Name"]]
        or [i for i, r in enumerate(rows) if "::adam_kernel" in r["Kernel_Name"]])
# step groups: Adam launches of one step are back-to-back
groups = [[adam[0]]]
for a, b in zip(adam, adam[1:]):
    if b - a > 3:
        groups.append([])
    groups[-1].append(b)
if max_steps is not None:
    groups = groups[:max_steps]
lo, hi = groups[0][0], groups[-1][-1]
steps = len(groups)
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
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(args[1]) if len(args) > 1 else 30]:
    print(f"{n/steps:6.1f}/step {t/steps:8.1f} us/step {t/n:8.1f} us/launch  {name[:110]}")
