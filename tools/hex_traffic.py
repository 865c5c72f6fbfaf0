#!/usr/bin/env python
"""HBM bytes per hexahedral action (k_hex_poisson + k_hex_seam_sum, one
launch each per sem_apply) from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes, with the gfx950 FETCH_SIZE x2 correction (tools/pmc_traffic.py).
  python tools/hex_traffic.py FETCH.csv WRITE.csv OUT.json"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import per_dispatch  # noqa: E402


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    res = {"kernels": {}, "note": "per action = one launch of each kernel; FETCH_SIZE x2 "
                                  "(gfx950 wide-read correction), includes Infinity-Cache hits"}
    tot = 0.0
    for k in ("k_hex_poisson", "k_hex_seam_sum"):
        f = per_dispatch(fetch_csv, "FETCH_SIZE", k)
        w = per_dispatch(write_csv, "WRITE_SIZE", k)
        fb = sum(f) / len(f) * 1024 * 2
        wb = sum(w) / len(w) * 1024
        res["kernels"][k] = {"dispatches": len(f), "fetch_bytes_corrected": fb,
                             "write_bytes": wb}
        tot += fb + wb
    res["hbm_bytes_per_launch"] = tot
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
