#!/usr/bin/env python
"""HBM bytes per action of the headline workload from two rocprofv3 passes
(--pmc FETCH_SIZE, --pmc WRITE_SIZE, --kernel-include-regex
"k_poisson_apply|k_seam_sum") into the JSON bench.py reads
(bench_traffic/pmc_traffic_nodal_p8_1024x1024.json).

  python tools/bench_traffic.py FETCH.csv WRITE.csv OUT.json "workload text" "source"

Per kernel: FETCH_SIZE x 2 (the gfx950 correction, confirmed per access shape
by tools/pmc_calib.cpp: profiles/r04/calib/) and WRITE_SIZE as is, both KB
x 1024, averaged over the dispatches; one action = one dispatch of each."""
import collections
import csv
import json
import sys

KERNELS = ("k_poisson_apply", "k_seam_sum")


def per_kernel(path, counter):
    vals = collections.defaultdict(dict)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        for k in KERNELS:
            if k in row["Kernel_Name"]:
                d = int(row["Dispatch_Id"])
                vals[k][d] = vals[k].get(d, 0.0) + float(row["Counter_Value"]) * 1024.0
    return {k: list(v.values()) for k, v in vals.items()}


def main():
    fcsv, wcsv, out, workload, source = sys.argv[1:6]
    f = per_kernel(fcsv, "FETCH_SIZE")
    w = per_kernel(wcsv, "WRITE_SIZE")
    pk, total = {}, 0.0
    for k in KERNELS:
        fv, wv = f.get(k, []), w.get(k, [])
        if not fv or not wv:
            continue
        fb = 2.0 * sum(fv) / len(fv)
        wb = sum(wv) / len(wv)
        pk[k] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "dispatches": min(len(fv), len(wv))}
        total += fb + wb
    res = {"kernels": list(pk), "launches_per_action": len(pk), "hbm_bytes_per_launch": total,
           "per_kernel": pk, "workload": workload,
           "note": "per action = one dispatch of each kernel; FETCH_SIZE x2 (gfx950 correction, "
                   "calibrated per access shape: profiles/r04/calib/), WRITE_SIZE as is; KB "
                   "x1024; separate rocprofv3 passes (%s)" % source}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
