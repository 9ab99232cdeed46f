"""rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes -> HBM bytes per launch of each engine timing region
(the regions bench.py's `kernels` reports), written with the kernel names each region was sampled
from so bench.py can refuse a stale file (profiles/r*/pmc_traffic.json).

gfx950 calibration (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) reports half of the bytes of a
wide coalesced read stream, so it is doubled; WRITE_SIZE (KB) is taken as is.  A region spanning
several launches per call (fr_encoder_bwd = enc_bwd_kernel + enc_reduce_kernel) sums its kernels.

usage: python tools/pmc_regions.py FETCH_DIR WRITE_DIR OUT_JSON [source note]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

# engine timing region -> the kernels (name substrings) one call of it launches on HEAD
REGION_KERNELS = {
    "encoder_bwd": ["enc_bwd_kernel", "enc_reduce_kernel"],
    "encoder_fwd": ["enc_fwd_kernel"],
    "spmm": ["spmm_plain16_kernel"],
    "spmm_masked": ["spmm_sparse_kernel"],
    "spmm_rows": ["spmm_rows_kernel"],
    "adam": ["adam_kernel<false, false>"],
    "adam_rows": ["adam_lazy_rows_kernel<false>"],
    "adam_rows_catch_up": ["adam_catch_up_multi_kernel"],
    "adam_rows_slice": ["adam_catch_up_slice_kernel"],
    "modal_fusion": ["fusion_fwd_kernel", "fusion_bwd_kernel"],
    "embedding_bwd": ["emb_atomic_kernel"],
}


def load(d, counter):
    agg = defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def per_kernel(fetch, write, sub):
    fv = [v for n, vs in fetch.items() if sub in n for v in vs]
    wv = [v for n, vs in write.items() if sub in n for v in vs]
    names = sorted({n for n in list(fetch) + list(write) if sub in n})
    if not fv:
        return None
    f_kb = sum(fv) / len(fv)
    w_kb = sum(wv) / len(wv) if wv else 0.0
    return {"names": names, "launches": len(fv), "fetch_kb_raw": round(f_kb, 1), "write_kb": round(w_kb, 1),
            "bytes": (2 * f_kb + w_kb) * 1024}


def main():
    fd, wd, out = sys.argv[1], sys.argv[2], sys.argv[3]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (--kernel-trace only); "
                     "FETCH_SIZE doubled per MI355X_MICROARCH.md's HBM section; averages over every launch. " + note,
           "per_region_bytes": {}, "region_kernels": {}, "kernels": {}}
    for region, subs in REGION_KERNELS.items():
        parts = [per_kernel(fetch, write, s) for s in subs]
        if any(p is None for p in parts):
            continue
        res["per_region_bytes"][region] = int(sum(p["bytes"] for p in parts))
        res["region_kernels"][region] = subs
        for s, p in zip(subs, parts):
            res["kernels"][s] = p
            print(f"{region:20s} {s:32s} launches={p['launches']:4d} bytes/launch={p['bytes']:.4e}")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
