"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one line per kernel name):
python tools/sqpmc_sum.py <counter_collection.csv> [name-filter-regex]"""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
for k, d in acc.items():
    if pat and not pat.search(k):
        continue
    calls = max(n[(k, c)] for c in d)
    print(k, "calls", calls, {c: round(v / calls) for c, v in sorted(d.items())})
