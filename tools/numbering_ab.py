#!/usr/bin/env python
"""Element-kernel time of one structured mesh under several node numberings
(same elements, same element order): lexicographic, the reference's default
RCM, first touch in element order, first touch in the kernel's (group, row,
lane) order, lexicographic with element-interior nodes first.  Also the cost
of one device gather permutation of a node vector.

  python tools/numbering_ab.py [--nex 256] [--p 8] > out.json"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def first_touch(order_ids, n_node):
    """new id of each node = rank of its first appearance in order_ids."""
    _, first = np.unique(order_ids, return_index=True)
    nodes_in_order = order_ids[np.sort(first)]
    inv = np.empty(n_node, dtype=np.int64)
    inv[nodes_in_order] = np.arange(n_node)
    return inv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nex", type=int, default=256)
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default=None, help="comma list of numberings")
    a = ap.parse_args()
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.discrete import rcm_permutation
    from spectralelementmethod_amd.operators import SEMOperator
    p, n = a.p, a.p + 1
    nodes, e2n = meshgen.structured_square(a.nex, a.nex, p, warp=0.05)
    e2n = e2n.astype(np.int64)
    N, E = nodes.shape[1], e2n.shape[0]
    epw = 64 // n
    nums = {"lex": np.arange(N)}
    perm = rcm_permutation(e2n.reshape(E, -1), N)
    inv = np.empty(N, dtype=np.int64)
    inv[perm] = np.arange(N)
    nums["rcm"] = inv.copy()
    nums["first_touch_element"] = first_touch(e2n.reshape(-1), N)
    g = np.full((-(-E // epw)) * epw, -1)
    g[:E] = np.arange(E)
    g = g.reshape(-1, epw)
    wave = np.concatenate([e2n[g[:, k]][:, :, :].transpose(0, 1, 2)[:, None] for k in range(epw)],
                          axis=1)  # [group, k, r, jj]
    wave = np.where((g >= 0)[:, :, None, None], wave, -1).transpose(0, 2, 1, 3).reshape(-1)
    nums["first_touch_wave_row"] = first_touch(wave[wave >= 0], N)
    bnd = np.zeros(N, bool)
    e3 = e2n.reshape(E, n, n)
    for sl in (e3[:, 0, :], e3[:, -1, :], e3[:, :, 0], e3[:, :, -1]):
        bnd[sl.reshape(-1)] = True
    split = np.concatenate([np.flatnonzero(~bnd), np.flatnonzero(bnd)])
    inv = np.empty(N, dtype=np.int64)
    inv[split] = np.arange(N)
    nums["lex_interior_first"] = inv
    if a.only:
        nums = {k: v for k, v in nums.items() if k in a.only.split(",")}
    dev = torch.device("cuda:0")
    u0 = np.random.default_rng(0).standard_normal(N)
    out = {"mesh": "%dx%d p=%d" % (a.nex, a.nex, p), "ndof": N}
    ref = None
    for name, newid in nums.items():
        nn = np.empty_like(nodes)
        nn[:, newid] = nodes
        m = newid[e2n].astype(np.uint32)
        op = SEMOperator(p, m, nn, device=dev)
        u = torch.empty(N, dtype=torch.float64, device=dev)
        u[torch.from_numpy(newid).to(dev)] = torch.from_numpy(u0).to(dev)
        y = torch.empty_like(u)
        for _ in range(10):
            op.apply(u, out=y)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.reps)]
        torch.cuda.synchronize()
        for s, e in ev:
            s.record()
            op.apply(u, out=y)
            e.record()
        torch.cuda.synchronize()
        t = sorted(s.elapsed_time(e) for s, e in ev)
        t_ren = None
        if name == "rcm":  # the action through the solver numbering (2 gathers)
            yr = torch.empty_like(u)
            for _ in range(5):
                op.apply(u, out=yr, renumber=True)
            torch.cuda.synchronize()
            for s, e in ev:
                s.record()
                op.apply(u, out=yr, renumber=True)
                e.record()
            torch.cuda.synchronize()
            t_ren = sorted(s.elapsed_time(e) for s, e in ev)[len(ev) // 2]
            assert float((yr - y).norm() / y.norm()) < 1e-12
        yv = y[torch.from_numpy(newid).to(dev)].cpu().numpy()
        if ref is None:
            ref = yv
        info = op.plan_info()
        out[name] = {"ms_median": t[len(t) // 2], "ms_min": t[0],
                     "map_entry_bytes": info["map_entry_bytes"], "blocks": info["blocks"],
                     "seam_nodes": info.get("seam_nodes"),
                     "rel_vs_lex": float(np.linalg.norm(yv - ref) / np.linalg.norm(ref)),
                     "ms_median_renumbered_action": t_ren}
        print(name, out[name], file=sys.stderr, flush=True)
        op.close()
        del op
    # one gather permutation of a node vector (sem_gather, uint32 index)
    from spectralelementmethod_amd import _lib
    lib = _lib.load()
    idx = torch.from_numpy(nums["rcm"].astype(np.uint32).view(np.int32)).to(dev)
    src = torch.randn(N, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    for _ in range(5):
        lib.sem_gather(_lib.tptr(src), _lib.tptr(idx), N, _lib.tptr(dst), _lib.stream_ptr())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(a.reps):
        lib.sem_gather(_lib.tptr(src), _lib.tptr(idx), N, _lib.tptr(dst), _lib.stream_ptr())
    e.record()
    torch.cuda.synchronize()
    out["gather_permute_ms"] = s.elapsed_time(e) / a.reps
    print(json.dumps(out))


if __name__ == "__main__":
    main()
