"""Host-side enqueue cost of the library calls on one step (diagnostic for
strong scaling: at 8 GPUs a rank's device work per step is ~85 us)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spectralelementmethod_amd import _lib, meshgen  # noqa: E402
from spectralelementmethod_amd.operators import SEMOperator  # noqa: E402

p = 8
for nex in (1024, 128):
    nodes, e2n = meshgen.structured_square(nex, 1024, p, warp=0.05)
    op = SEMOperator(p, e2n, nodes)
    op.compute_geometry()
    u = torch.randn(op.ndof, dtype=torch.float64, device="cuda")
    y = torch.empty_like(u)
    lib = _lib.load()
    sp = _lib.stream_ptr()
    up, yp = _lib.tptr(u), _lib.tptr(y)
    for _ in range(5):
        lib.sem_apply(op._ctx, 0, up, yp, 0, sp)
    torch.cuda.synchronize()
    K = 200
    t0 = time.perf_counter()
    for _ in range(K):
        lib.sem_apply(op._ctx, 0, up, yp, 0, sp)
    t_enq = (time.perf_counter() - t0) / K
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / K
    idx = torch.arange(100000, dtype=torch.int32, device="cuda")
    buf = torch.empty(100000, dtype=torch.float64, device="cuda")
    t0 = time.perf_counter()
    for _ in range(K):
        lib.sem_gather(yp, _lib.tptr(idx), 100000, _lib.tptr(buf), sp)
    t_g = (time.perf_counter() - t0) / K
    torch.cuda.synchronize()
    ev = torch.cuda.Event()
    t0 = time.perf_counter()
    for _ in range(K):
        ev.record()
    t_ev = (time.perf_counter() - t0) / K
    print("nex %d: sem_apply enqueue %.1f us (device %.1f us/step incl.), sem_gather enqueue %.1f us, "
          "torch event record %.1f us, plan %s" % (nex, t_enq * 1e6, t_all * 1e6, t_g * 1e6,
                                                   t_ev * 1e6, op.plan_info()["colours"]))
