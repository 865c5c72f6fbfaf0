"""Planner and throughput on unstructured meshes (profiles/r02/unstructured.json):
colours, atomic-fallback groups, map entry width and DOF/s per mesh kind."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spectralelementmethod_amd import meshgen  # noqa: E402
from spectralelementmethod_amd.operators import SEMOperator  # noqa: E402


def mesh(kind, p):
    if kind == "structured":
        return meshgen.structured_square(300, 300, p, warp=0.05)
    if kind == "shuffled_elems":
        n, e = meshgen.structured_square(300, 300, p, warp=0.05)
        return n, meshgen.shuffle_elements(e, 5)
    if kind == "shuffled_nodes":
        return meshgen.shuffle_nodes(*meshgen.structured_square(300, 300, p, warp=0.05), 6)
    nodes, e2n = meshgen.quads_from_triangles(120, 100, p, seed=3)   # 72,000 quads
    if kind == "split_tri":
        return nodes, e2n
    sh = meshgen.shuffle_nodes(nodes, meshgen.shuffle_elements(e2n, 1), 2)
    return sh if kind == "split_tri_shuffled" else meshgen.rcm_renumber(*sh)


out = []
for p in (4, 8):
    for kind in ("structured", "shuffled_elems", "shuffled_nodes", "split_tri",
                 "split_tri_shuffled", "split_tri_rcm"):
        nodes, e2n = mesh(kind, p)
        t0 = time.perf_counter()
        op = SEMOperator(p, e2n, nodes)
        op.compute_geometry()
        torch.cuda.synchronize()
        t_setup = time.perf_counter() - t0
        u = torch.randn(op.ndof, dtype=torch.float64, device="cuda")
        y = torch.empty_like(u)
        for _ in range(3):
            op.apply(u, out=y)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        K = 20
        ev[0].record()
        for _ in range(K):
            op.apply(u, out=y)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / K
        plan = op.plan_info()
        rec = dict(kind=kind, p=p, n_elem=int(e2n.shape[0]), ndof=op.ndof, ms_per_action=ms,
                   dof_per_s=op.ndof / ms * 1e3, setup_s=t_setup,
                   **{k: plan[k] for k in ("colours", "chains_per_colour", "atomic_groups",
                                           "zero_list", "map_entry_bytes", "geometry", "kernel", "plan")})
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del op
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "unstructured.json"), "w") as f:
    json.dump(out, f, indent=1)
