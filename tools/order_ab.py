"""Element-order experiment for the chain planner: chains covering several
element columns (rounds = columns, each round one 28-element block of one
column) vs the natural column-major order.  Usage:
  SEM_CHAIN_ROUNDS=R python tools/order_ab.py R"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spectralelementmethod_amd import meshgen  # noqa: E402
from spectralelementmethod_amd.operators import SEMOperator  # noqa: E402

R = int(sys.argv[1])
p, nex, ney = 8, 1024, 1024
nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
blk = 28  # 4 groups of 7 elements
if R > 1:
    ids = np.arange(nex * ney).reshape(nex, ney)  # [ex, ey]
    order = []
    for X in range(0, nex, R):
        for b in range(0, ney, blk):
            for c in range(X, min(X + R, nex)):
                order.append(ids[c, b:b + blk])
    order = np.concatenate(order)
    assert order.size == nex * ney
    e2n = np.ascontiguousarray(e2n[order])
op = SEMOperator(p, e2n, nodes)
op.compute_geometry()
u = torch.randn(op.ndof, dtype=torch.float64, device="cuda")
y = torch.empty_like(u)
for _ in range(5):
    op.apply(u, out=y)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
K = 30
ev[0].record()
for _ in range(K):
    op.apply(u, out=y)
ev[1].record()
torch.cuda.synchronize()
pl = op.plan_info()
print("rounds %d: %.4f ms/action, colours %d, atomic groups %d, map %d B, plan %s" % (
    R, ev[0].elapsed_time(ev[1]) / K, pl["colours"], pl["atomic_groups"], pl["map_entry_bytes"],
    pl["plan"]), flush=True)
