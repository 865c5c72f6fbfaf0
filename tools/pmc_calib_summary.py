#!/usr/bin/env python
"""Correction factors of FETCH_SIZE / WRITE_SIZE per access shape, from the
two rocprofv3 passes over tools/pmc_calib.bin (one counter per pass) and the
program's own stdout (shape, bytes touched per launch, ms of the second
launch), in dispatch order: every shape is launched twice.

  python tools/pmc_calib_summary.py FETCH_csv WRITE_csv calib_stdout out.json

factor = counter bytes per launch / bytes touched per launch (the counters are
reported in KiB).  A byte count of the operator kernels measured with a shape
of this table is corrected by dividing by its factor."""
import csv
import json
import sys


def per_dispatch(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        # the calibration kernels only (hipMemset's fill kernel runs first)
        if r.get("Counter_Name") == counter and "k_" in r["Kernel_Name"]:
            rows.append((int(r.get("Dispatch_Id", len(rows))), r["Kernel_Name"],
                         float(r["Counter_Value"]) * 1024.0))
    rows.sort()
    return rows


def main():
    fcsv, wcsv, out_txt, dst = sys.argv[1:5]
    shapes = []
    for ln in open(out_txt):
        if ln.startswith("#") or not ln.strip():
            continue
        name, nbytes, ms = ln.split()
        shapes.append((name, int(nbytes), float(ms)))
    F = per_dispatch(fcsv, "FETCH_SIZE")
    W = per_dispatch(wcsv, "WRITE_SIZE")
    assert len(F) == len(W) == 2 * len(shapes), (len(F), len(W), len(shapes))
    res = {}
    for i, (name, nb, ms) in enumerate(shapes):
        f = F[2 * i + 1][2]  # the second (timed) launch
        w = W[2 * i + 1][2]
        res[name] = dict(bytes_touched=nb, kernel=F[2 * i + 1][1][:80], fetch_bytes=f,
                         write_bytes=w, fetch_factor=f / nb, write_factor=w / nb, ms=ms,
                         gb_per_s=nb / ms / 1e6)
    json.dump(res, open(dst, "w"), indent=1)
    print("%-18s %14s %8s %8s %8s" % ("shape", "bytes", "fetch/B", "write/B", "GB/s"))
    for k, v in res.items():
        print("%-18s %14d %8.3f %8.3f %8.0f" % (k, v["bytes_touched"], v["fetch_factor"],
                                                v["write_factor"], v["gb_per_s"]))


if __name__ == "__main__":
    main()
