#!/usr/bin/env python
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs of the element
kernel into HBM bytes per action (one sem_apply = one launch per colour).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of wide coalesced reads, so the read side is doubled; WRITE_SIZE is
taken as is.  Both are KB (x1024).  FETCH_SIZE also counts Infinity-Cache
hits, so this is memory-side traffic (an upper bound on HBM reads).

  python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json [--kernel k_poisson_apply]
"""
import argparse
import collections
import csv
import json


def per_dispatch(path, counter, kernel):
    vals = collections.OrderedDict()
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or kernel not in row["Kernel_Name"]:
            continue
        vals[int(row["Dispatch_Id"])] = vals.get(int(row["Dispatch_Id"]), 0.0) + \
            float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="k_poisson_apply")
    ap.add_argument("--launches-per-action", type=int, default=None,
                    help="colour launches per sem_apply (default: from the bench JSON)")
    ap.add_argument("--bench-json", default=None)
    a = ap.parse_args()
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    lpa = a.launches_per_action
    if lpa is None and a.bench_json:
        cfg = json.load(open(a.bench_json))["config"]
        lpa = cfg["scatter_plan"]["colours"]
    lpa = lpa or 1
    n = min(len(f), len(w)) // lpa * lpa
    fetch = sum(f[:n]) * 1024 * 2 / (n // lpa)
    write = sum(w[:n]) * 1024 / (n // lpa)
    res = {"kernel": a.kernel, "launches_per_action": lpa, "actions": n // lpa,
           "fetch_bytes_per_action_corrected": fetch, "write_bytes_per_action": write,
           "hbm_bytes_per_launch": fetch + write,
           "note": "per action (all colour launches); FETCH_SIZE x2 (gfx950 wide-read "
                   "correction), includes Infinity-Cache hits"}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
