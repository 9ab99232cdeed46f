"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into HBM bytes per launch per kernel.

gfx950 calibration (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) reports half of the bytes of
a wide coalesced read stream, so it is doubled; WRITE_SIZE (KB) is taken as is.
usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [kernel-substring ...]
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    agg = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    keys = sys.argv[3:] or ["adam_kernel", "spmm_units_kernel"]
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    for k in keys:
        fv = [v for n, vs in fetch.items() if k in n for v in vs]
        wv = [v for n, vs in write.items() if k in n for v in vs]
        if not fv:
            print(k, "no samples")
            continue
        f_kb = sum(fv) / len(fv)
        w_kb = sum(wv) / len(wv) if wv else 0.0
        print(f"{k}: launches={len(fv)} FETCH_SIZE={f_kb:.0f}KB (x2 calibrated) WRITE_SIZE={w_kb:.0f}KB "
              f"-> HBM bytes/launch ~ {(2 * f_kb + w_kb) * 1024:.4e}")


if __name__ == "__main__":
    main()
