#!/usr/bin/env python
"""Summarise a scripts/gpu_profile.sh run into profiles/.

  python scripts/pmc_traffic.py gpurun_out/<tag> profiles/<round>_<tag>
writes <out>_kernel_stats.csv (copy of rocprofv3 --stats) and
profiles/pmc_traffic.json: per kernel family, HBM bytes per launch from the
FETCH_SIZE / WRITE_SIZE passes (KB units).  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B wide read
request, i.e. half of a coalesced stream -> doubled here; WRITE_SIZE is taken
as is.  Families follow bench.py's kernel kinds.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def family(name):
    # split-f16 kernels (dstd_hilo.hip) are families of their own: the
    # 64->64 launches whose bytes bench.py's roofline divides
    if "k_block_fused" in name:
        return "block_split"
    if "k_spatial_hl" in name:
        return "spatial_gc_split"
    if "k_temporal_hl" in name or "k_temporal_fused" in name:
        return "temporal_gc_split"
    if "k_adj_hl<0" in name:
        return "adj_spatial_split"
    if "k_adj_hl<1" in name:
        return "adj_temporal_split"
    if "k_hl_prep" in name:
        return "hl_prep"
    if "k_spatial" in name:
        return "spatial_gc"
    if "k_temporal" in name:
        return "temporal_gc"
    if "k_adj_fast<0" in name:
        return "adj_spatial"
    if "k_adj_fast<1" in name:
        return "adj_temporal"
    if "k_adj<" in name:
        return "adj_generic"
    if "k_pq" in name:
        return "prep"
    if "k_fold" in name:
        return "fold"
    return None


def short(name):
    """'void dstd::k_spatial_hl<22, 64, 64>(dstd::SpatialHLArgs)' -> 'k_spatial_hl<22, 64, 64>'"""
    name = name.split("(")[0].replace("void ", "")
    return name.split("::")[-1] if "<" not in name else name[name.index("k_"):] if "k_" in name else name


def per_launch(path, counter, key=family):
    tot, ids = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        f = key(r["Kernel_Name"])
        if f is None:
            continue
        tot[f] += float(r["Counter_Value"])
        ids[f].add(r["Dispatch_Id"])
    return {f: tot[f] / len(ids[f]) for f in tot}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), dst + "_kernel_stats.csv")
    fetch = write = None
    fetch_k = write_k = {}
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc") or not os.path.exists(p):
            continue
        names = {r["Counter_Name"] for r in csv.DictReader(open(p))}
        if "FETCH_SIZE" in names:
            fetch = per_launch(p, "FETCH_SIZE")
            fetch_k = per_launch(p, "FETCH_SIZE", short)
        if "WRITE_SIZE" in names:
            write = per_launch(p, "WRITE_SIZE")
            write_k = per_launch(p, "WRITE_SIZE", short)
    out = {"_note": "HBM bytes per launch, averaged over every launch of the family in the profiled bench run; "
                    "FETCH_SIZE doubled (gfx950 half-count of wide reads), WRITE_SIZE as reported; KB = 1024 B",
           "_source": os.path.basename(dst)}
    for f in sorted(set(fetch or {}) | set(write or {})):
        fb = 2 * 1024 * (fetch or {}).get(f, 0.0)
        wb = 1024 * (write or {}).get(f, 0.0)
        out[f] = {"fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                  "hbm_bytes_per_launch": round(fb + wb)}
    out["by_kernel"] = {}
    for k in sorted(set(fetch_k) | set(write_k)):
        fb = 2 * 1024 * fetch_k.get(k, 0.0)
        wb = 1024 * write_k.get(k, 0.0)
        out["by_kernel"][k] = {"fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                               "hbm_bytes_per_launch": round(fb + wb)}
    with open(os.path.join(os.path.dirname(dst) or ".", "pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
