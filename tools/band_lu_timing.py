"""Timing of sem_band_lu_solve (one workgroup, n dependent elimination steps)
over sizes, to state its size limit in DESIGN.md §4.7.  Random banded
non-symmetric matrices with a dominant diagonal (pivoting still exercised by
the random off-diagonals); the order is kept as given (no RCM: the band is
the one built).  Prints one JSON line per case: n, kl, ku, seconds of the
device call (hipMalloc + fill + factor/solve + copy back), error vs spsolve
where spsolve finishes quickly.

  python tools/band_lu_timing.py"""
import json
import os
import sys
import time

import numpy as np
import torch
from scipy import sparse
from scipy.sparse import linalg as spla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402
from spectralelementmethod_amd import _lib  # noqa: E402


def run(n, bw, dev, check=True):
    rng = np.random.default_rng(n + bw)
    offs = list(range(-bw, bw + 1))
    A = sparse.diags([rng.standard_normal(n - abs(k)) for k in offs], offs, format="csr")
    A = A + sparse.diags(np.full(n, 4.0 * bw))
    A = A.tocsr()
    b = rng.standard_normal(n)
    lib = _lib.load()
    rp = torch.from_numpy(A.indptr.astype(np.int64)).to(dev)
    ci = torch.from_numpy(A.indices.astype(np.int32)).to(dev)
    va = torch.from_numpy(A.data.astype(np.float64)).to(dev)
    bd = torch.from_numpy(b).to(dev)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    info = C.c_int(0)
    best = None
    for _ in range(2):  # first call loads the code object
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(lib.sem_band_lu_solve(n, bw, bw, _lib.tptr(rp), _lib.tptr(ci), _lib.tptr(va),
                                         _lib.tptr(bd), _lib.tptr(x), C.byref(info),
                                         _lib.stream_ptr()))
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    out = dict(n=n, kl=bw, ku=bw, seconds=best, info=info.value,
               us_per_step=best / n * 1e6)
    if check:
        ref = spla.spsolve(A.tocsc(), b)
        xv = x.cpu().numpy()
        out["rel_l2_vs_spsolve"] = float(np.linalg.norm(xv - ref) / np.linalg.norm(ref))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # both schedules (SEM_BAND_LU_STEPS 0: one workgroup; 1: two launches per step)
    for mode in ("0", "1"):
        os.environ["SEM_BAND_LU_STEPS"] = mode
        print(json.dumps({"schedule": "one workgroup" if mode == "0" else "launches per step"}),
              flush=True)
        for n, bw in [(2000, 8), (20000, 8), (20000, 32), (20000, 48), (20000, 64),
                      (20000, 96), (20000, 128), (20000, 256), (5000, 1024)]:
            if mode == "0" and bw >= 1024:
                n = 2000
            run(n, bw, dev, check=n * bw <= 5_000_000)
