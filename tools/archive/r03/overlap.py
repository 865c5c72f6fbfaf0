#!/usr/bin/env python
"""Overlap of the decomposition's side-stream work with the interior
elements, from rocprofv3 --kernel-trace CSVs of bench.py ranks (one CSV per
rank; the side stream is the queue that runs k_gather / k_scatter_add_peer).

  python tools/r03/overlap.py TRACE.csv [TRACE.csv ...] > summary.json
"""
import csv
import json
import sys


def main(paths):
    out = {}
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Stream_Id") or r["Queue_Id"]) for r in rows)
        side = {q for s, e, n, q in ks if "k_scatter_add_peer" in n}
        interior = [(s, e) for s, e, n, q in ks if "k_poisson_apply" in n and q not in side]
        side_k = [(s, e, n) for s, e, n, q in ks if q in side and "semk" in n or
                  (q in side and "namespace" in n)]
        tot = ov = 0
        for s, e, n in side_k:
            tot += e - s
            for a, b in interior:
                ov += max(0, min(e, b) - max(s, a))
        out[path] = dict(side_stream_kernels=len(side_k), side_kernel_us=tot / 1e3,
                         overlapped_with_interior_us=ov / 1e3,
                         overlap_fraction=ov / tot if tot else None,
                         interior_launches=len(interior),
                         interior_us_avg=sum(b - a for a, b in interior) / max(1, len(interior)) / 1e3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
