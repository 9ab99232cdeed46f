"""Summarise rocprofv3 PMC passes over tools/spmm10m.py into the beyond-L2 bytes per config-4 SpMM
launch (profiles/r*/pmc_spmm10m.json, read by bench.py's config4_10m.spmm block).

Per launch: FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half of a wide coalesced read stream,
MI355X_MICROARCH.md's HBM section) + WRITE_SIZE, summed over the kernels one spmm_launch issues (the
unit kernel and, for split rows, the ordered fix-up), averaged over the launches.  These are bytes
that left the L2: DRAM traffic plus Infinity Cache (MALL) hits -- an upper bound on DRAM bytes.

usage: python tools/pmc_spmm10m.py FETCH_DIR WRITE_DIR OUT_JSON KEY [note]   (KEY: config4 | dram_uniform)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    agg = defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and "spmm" in r["Kernel_Name"]:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    fd, wd, out, key = sys.argv[1:5]
    note = sys.argv[5] if len(sys.argv) > 5 else ""
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    kernels = {}
    total = 0.0
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        if not f:
            continue
        fkb, wkb = sum(f) / len(f), (sum(w) / len(w) if w else 0.0)
        b = (2 * fkb + wkb) * 1024
        kernels[name] = {"launches": len(f), "fetch_kb_raw": round(fkb, 1), "write_kb": round(wkb, 1), "bytes": b}
        total += b
    res = json.load(open(out)) if os.path.exists(out) else {}
    res[key] = {"bytes_per_launch": int(total), "kernels": kernels,
                "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes with --kernel-trace, over "
                          "tools/spmm10m.py (bench.py's graph); FETCH_SIZE doubled (gfx950). " + note}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(key, int(total), {k: int(v["bytes"]) for k, v in kernels.items()})


if __name__ == "__main__":
    main()
