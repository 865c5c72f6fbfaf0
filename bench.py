#!/usr/bin/env python
"""Benchmark: global Poisson stiffness action, DOF-updates/s (BASELINE.json
metric), on synthetic structured quad meshes of order p, elements split in
column strips across ranks (one process per GPU).

A step = one global action y = K u over one batch of synthetic input: the
element kernels and, with several ranks, the interface sum with the
neighbouring ranks (RCCL send/recv over xGMI, hidden behind the interior
elements; csrc/sem_dd.hip).  Inputs are resident in HBM before the timed
region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--p 8] [--nex 1024] [--ney 1024]
                  [--scaling strong|weak] [--op poisson|axisym_stokes|axisym_ns|pcg]
  python bench.py --dim 3 [--p 8] [--hex-ne 27] [--hex-nex L] [--gpus N]
                  [--hex-decomp block|slab]
                  (hexahedra, bench_hex; N ranks = slabs of element layers along x,
                  or boxes on a near-cubic rank grid)

--gpus N without a launcher: this process starts N rank processes (before
touching the GPU) and waits for them; under torchrun (WORLD_SIZE set) each
process is one rank.  --scaling strong (default): the nex x ney mesh is the
GLOBAL mesh split into N strips (BASELINE config 3: 1024 x 1024 over 8
GPUs); weak: every rank owns nex x ney elements.

Rank 0 prints ONE JSON line (the driver's contract) with a ``roofline``
object for the element kernel (algorithmic bytes of SURVEY.md §8(d) / HIP
event time on the launch stream), a ``parity`` spot check of the timed
output against the NumPy oracle, and, at N = 1, a ``cpu_baseline`` object
(the oracle of the reference path timed on this host's cores on bounded
samples, in a child process with OMP_NUM_THREADS pinned).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "global stiffness-action DOF-updates/s (and % HBM roofline), Poisson p=8"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP64_PEAK_TFLOPS = 78.6  # MI355X vector fp64 (256 CUs x 128 FLOP/clk x 2.4 GHz)
# PMC-measured HBM bytes per action of the headline workload (separate
# rocprofv3 --pmc passes, FETCH_SIZE x2 + WRITE_SIZE, all launches of one
# action), per geometry mode: copies of profiles/r01/pmc_traffic_p8_1024x1024.json
# and profiles/r03/pmc_default/traffic_per_action.json in bench_traffic/, which
# travels to the GPU box; profiles/ does not
DEFAULT_TRAFFIC = {"stored": "pmc_traffic_stored_p8_1024x1024.json",
                   "nodal": "pmc_traffic_nodal_p8_1024x1024.json"}


JSON_OUT = sys.stdout  # the driver's JSON line (rank 0)


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- byte models
def alg_bytes_s8d(kind, n_nodes, n_elem, p):
    """SURVEY.md §8(d), the problem's algorithmic bytes: Poisson
    B = 16*ndof + 28*E*(p+1)^2 (u read once, y written once, 3 fp64 geometric
    factors + one uint32 map entry per element node); axisymmetric
    B = 32*n_nodes + 60*E*(p+1)^2 (Navier-Stokes residual: 9 factors, 76)."""
    n2 = (p + 1) ** 2
    if kind == "poisson":
        return 16 * n_nodes + 28 * n_elem * n2
    if kind == "axisym_ns":
        return 32 * n_nodes + 76 * n_elem * n2
    return 32 * n_nodes + 60 * n_elem * n2


def streamed_bytes(kind, n_nodes, n_elem, p, geometry, map_bytes, map_patterns=0):
    """The least the kernel as built must stream: with NODAL geometry the
    factors are replaced by x_phys per global node (16 B) gathered like u;
    map_bytes = 2: 16-bit packed map plus one uint32 base per group row;
    map_patterns > 0: the bases and the pattern table only."""
    n = p + 1
    n2 = n * n
    m = map_bytes * n_elem * n2
    if map_bytes == 2:
        epw = 64 // n
        m += 4 * n * n_elem // epw
        if map_patterns:
            m = 4 * n * n_elem // epw + 2 * map_patterns * n * epw * n
    if kind != "poisson":
        if geometry == "nodal":  # (psi, omega) read + written, x_phys read
            return 48 * n_nodes + m
        return alg_bytes_s8d(kind, n_nodes, n_elem, p)
    if geometry == "nodal":
        return 32 * n_nodes + m
    return 16 * n_nodes + 24 * n_elem * n2 + m


def alg_flops(kind, n_elem, p, geometry="stored"):
    """fp64 FLOP per action: the four sum-factorised contractions (2 n^3 each)
    plus pointwise work; nodal geometry adds the four derivatives of x_phys
    and the per-node det / inverse / detJxW (15 n^2 incl. one division)."""
    n = p + 1
    extra = 8 * n ** 3 + 15 * n ** 2 if geometry == "nodal" else 0
    if kind == "poisson":
        return n_elem * (8 * n ** 3 + 7 * n ** 2 + extra)
    if geometry == "nodal":  # + the seven factors from J and rho (two reciprocals)
        extra += 16 * n ** 2
    return n_elem * (16 * n ** 3 + (30 if kind == "axisym_ns" else 22) * n ** 2 + extra)


# ---------------------------------------------------------------- CPU baseline
def _faithful_worker(args):
    """One worker of the multi-process reference-faithful action: builds the
    dense Lse of its element slice, then times its per-element einsum +
    np.add.at passes (after a barrier shared with the other workers)."""
    p, nex, warp, w, nw, reps, barrier = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    nodes, e2n = meshgen.structured_square(nex, nex, p, warp=warp)
    prob = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True)
    E = e2n.shape[0]
    sl = np.arange(w * E // nw, (w + 1) * E // nw)
    Lse = prob.element_matrices(sl)
    u = np.random.default_rng(0).standard_normal(prob.ndof)
    sem_oracle.apply_element_matrices(Lse, prob.e2n[sl], u, prob.ndof)  # warm-up
    ts = []
    for _ in range(reps):
        barrier.wait()
        t0 = time.perf_counter()
        sem_oracle.apply_element_matrices(Lse, prob.e2n[sl], u, prob.ndof)
        ts.append(time.perf_counter() - t0)
    return ts


def cpu_baseline(p, warp, budget_s=20.0, workers=16):
    """The reference path on this host (oracle/sem_oracle.py restates it;
    BASELINE.md §3), OMP_NUM_THREADS pinned to 1 per process:
    (1) reference-faithful per-element dense Lse (examples/poisson.py:168-193)
        applied with einsum('pqrs,rs') + np.add.at (squirmer:286), one
        process on 64 x 64, and `workers` processes on 128 x 128 (elements
        split evenly, partial vectors summed; the sum is timed too);
    (2) batched element-matrix (einsum + bincount) on 64 x 64;
    (3) batched sum-factorised NumPy on 256 x 256 (config 2)."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    half = gll["half_%d" % p]
    out = {}

    def timed(fn, min_reps=3, max_reps=20, budget=budget_s / 4):
        fn()
        ts, t_start = [], time.perf_counter()
        while len(ts) < min_reps or (time.perf_counter() - t_start < budget and len(ts) < max_reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), len(ts)

    nodes, e2n = meshgen.structured_square(64, 64, p, warp=warp)
    t0 = time.perf_counter()
    prob = sem_oracle.PoissonProblem(nodes, e2n, half, batched_geometry=True)
    Lse = prob.element_matrices()
    t_setup = time.perf_counter() - t0
    u = np.random.default_rng(0).standard_normal(prob.ndof)
    t1, r1 = timed(lambda: sem_oracle.apply_element_matrices(Lse, prob.e2n, u, prob.ndof))
    out["faithful_1"] = dict(ndof=prob.ndof, n_elem=e2n.shape[0], sec_per_action=t1,
                             dof_per_s=prob.ndof / t1, reps=r1,
                             setup_sec_per_elem=t_setup / e2n.shape[0])
    t2, r2 = timed(lambda: sem_oracle.apply_element_matrices_batched(Lse, prob.e2n, u, prob.ndof))
    out["batched_elem_matrix"] = dict(ndof=prob.ndof, sec_per_action=t2, dof_per_s=prob.ndof / t2,
                                      reps=r2)
    del Lse
    nodes, e2n = meshgen.structured_square(256, 256, p, warp=warp)
    prob = sem_oracle.PoissonProblem(nodes, e2n, half, batched_geometry=True)
    u = np.random.default_rng(0).standard_normal(prob.ndof)
    t3, r3 = timed(lambda: prob.apply(u), max_reps=5)
    out["batched_sumfact"] = dict(ndof=prob.ndof, sec_per_action=t3, dof_per_s=prob.ndof / t3,
                                  reps=r3)
    # (1) on `workers` processes
    nw = max(1, min(workers, os.cpu_count() or 1))
    nex_mp = 128
    reps = 5
    ctx = mp.get_context("fork")
    barrier = ctx.Manager().Barrier(nw)
    with ctx.Pool(nw) as pool:
        res = pool.map(_faithful_worker, [(p, nex_mp, warp, w, nw, reps, barrier)
                                          for w in range(nw)])
    t_max = [max(r[k] for r in res) for k in range(reps)]
    ndof_mp = (nex_mp * p + 1) ** 2
    parts = [np.random.default_rng(w).standard_normal(ndof_mp) for w in range(nw)]
    t0 = time.perf_counter()
    np.add.reduce(parts)
    t_sum = time.perf_counter() - t0
    t_mp = float(np.median(t_max)) + t_sum
    out["faithful_mp"] = dict(ndof=ndof_mp, n_elem=nex_mp * nex_mp, workers=nw,
                              sec_per_action=t_mp, dof_per_s=ndof_mp / t_mp, reps=reps)
    return out


def alg_bytes_hex(n_nodes, n_elem, p):
    """The 3-D form of SURVEY.md §8(d): u read once and y written once (16
    per DOF), 6 fp64 geometric factors + one uint32 map entry per element
    node (52 B): B = 16*ndof + 52*E*(p+1)^3."""
    return 16 * n_nodes + 52 * n_elem * (p + 1) ** 3


def alg_flops_hex(n_elem, p):
    """fp64 FLOP per hexahedral action: six sum-factorised contractions
    (2 n^4 each) + 15 per node for the 3x3 factor product."""
    n = p + 1
    return n_elem * (12 * n ** 4 + 15 * n ** 3)


def _faithful_hex_worker(args):
    """One worker of the multi-process reference-faithful hexahedral action:
    dense element Laplacians (the 3-D form of examples/poisson.py:168-193) of
    its element slice, applied per element + np.add.at, timed after a barrier."""
    p, ne, warp, w, nw, reps, barrier = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    nodes, e2n = meshgen.structured_cube(ne, ne, ne, p, warp=warp)
    prob = sem_oracle.HexPoissonProblem(nodes, e2n, gll["half_%d" % p])
    E = e2n.shape[0]
    sl = np.arange(w * E // nw, (w + 1) * E // nw)
    L = prob.element_matrices(sl)
    loc = prob.e2n[sl].reshape(len(sl), -1)
    u = np.random.default_rng(0).standard_normal(prob.ndof)

    def run():
        y = np.zeros(prob.ndof)
        for k in range(len(sl)):
            np.add.at(y, loc[k], L[k] @ u[loc[k]])
        return y
    run()
    ts = []
    for _ in range(reps):
        barrier.wait()
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    return ts


def cpu_baseline_hex(p, warp, budget_s=20.0, workers=16):
    """The reference path on hexahedra on this host (oracle restatement,
    OMP_NUM_THREADS = 1 per process): (1) per-element dense Laplacian applied
    element by element + np.add.at, `workers` processes over an 8^3 mesh;
    (2) batched sum-factorised NumPy on 12^3 (one process)."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    out = {}
    nodes, e2n = meshgen.structured_cube(12, 12, 12, p, warp=warp)
    prob = sem_oracle.HexPoissonProblem(nodes, e2n, gll["half_%d" % p])
    u = np.random.default_rng(0).standard_normal(prob.ndof)
    prob.apply(u)
    ts, t_start = [], time.perf_counter()
    while len(ts) < 3 or (time.perf_counter() - t_start < budget_s / 2 and len(ts) < 10):
        t0 = time.perf_counter()
        prob.apply(u)
        ts.append(time.perf_counter() - t0)
    t3 = float(np.median(ts))
    out["batched_sumfact"] = dict(ndof=prob.ndof, sec_per_action=t3, dof_per_s=prob.ndof / t3,
                                  reps=len(ts))
    del prob
    nw = max(1, min(workers, os.cpu_count() or 1))
    ne, reps = 8, 5
    ctx = mp.get_context("fork")
    barrier = ctx.Manager().Barrier(nw)
    with ctx.Pool(nw) as pool:
        res = pool.map(_faithful_hex_worker, [(p, ne, warp, w, nw, reps, barrier)
                                              for w in range(nw)])
    t_max = [max(r[k] for r in res) for k in range(reps)]
    ndof = (ne * p + 1) ** 3
    parts = [np.random.default_rng(w).standard_normal(ndof) for w in range(nw)]
    t0 = time.perf_counter()
    np.add.reduce(parts)
    t_mp = float(np.median(t_max)) + time.perf_counter() - t0
    out["faithful_mp"] = dict(ndof=ndof, n_elem=ne ** 3, workers=nw, sec_per_action=t_mp,
                              dof_per_s=ndof / t_mp, reps=reps)
    return out


def _hex_partition(args, world, rank):
    """The hexahedral workload split over `world` ranks (row N3): --hex-ne^3
    warped hexahedra (--hex-nex elements along x if given).  --hex-decomp
    slab (default): slabs of element layers along x (SlabPartition); block:
    boxes on the distributed.block_grid(world) rank grid (BlockPartition;
    2 x 2 x 2 at 8 ranks; ahead of slabs from about 54^3 on, behind them at
    27^3).  --scaling weak multiplies the mesh by the rank
    grid, so every rank keeps the one-GPU mesh."""
    from spectralelementmethod_amd.distributed import BlockPartition, SlabPartition, block_grid
    ne = args.hex_ne
    nex, ney, nez = args.hex_nex or ne, ne, ne
    if args.hex_decomp == "slab" or world == 1:
        if args.scaling == "weak":
            nex *= world
        return SlabPartition(nex, ney, nez, args.p, world, rank)
    grid = block_grid(world)
    if args.scaling == "weak":
        nex, ney, nez = nex * grid[0], ney * grid[1], nez * grid[2]
    return BlockPartition(nex, ney, nez, args.p, grid, rank)


def _hex_ranges(part):
    """Element ranges per axis of a rank's part (slab or box)."""
    if hasattr(part, "ranges"):
        return [tuple(r) for r in part.ranges]
    return [(part.ex0, part.ex1), (0, part.ney), (0, part.nez)]


def _hex_desc(part):
    r = _hex_ranges(part)
    kind = "box" if hasattr(part, "ranges") else "slab"
    return "%s %s" % (kind, " x ".join("[%d,%d)" % a for a in r))


def _hex_gid_to_local(part, gids):
    """Local node ids of global ids that lie in the rank's node box."""
    p = part.p
    r = _hex_ranges(part)
    shape = [(b - a) * p + 1 for a, b in r]
    iz = gids % part.Nz
    iy = (gids // part.Nz) % part.Ny
    ix = gids // (part.Nz * part.Ny)
    lx, ly, lz = ix - r[0][0] * p, iy - r[1][0] * p, iz - r[2][0] * p
    assert (lx >= 0).all() and (lx < shape[0]).all() and (ly >= 0).all() and \
        (ly < shape[1]).all() and (lz >= 0).all() and (lz < shape[2]).all()
    return (lx * shape[1] + ly) * shape[2] + lz


def _hex_sub_box(part, box, keep_lo_x=True):
    """Nodes of the element box `box` (3 element ranges) whose value the box's
    elements alone determine: along each axis the box's first and last node
    index are dropped unless they lie on the mesh boundary (or, with
    keep_lo_x False, the first x index is always dropped)."""
    p = part.p
    Ns = ((part.nex * p + 1), part.Ny, part.Nz)
    keep = []
    for a, (c0, c1) in enumerate(box):
        idx = np.arange(c0 * p, c1 * p + 1)
        m = np.ones(idx.size, dtype=bool)
        if (c0 > 0) or (a == 0 and not keep_lo_x):
            m[0] = False
        if c1 * p < Ns[a] - 1:
            m[-1] = False
        keep.append(m)
    return (keep[0][:, None, None] & keep[1][None, :, None] & keep[2][None, None, :]).ravel()


def hex_parity_checks(op, y, u, part, p, warp, dev, world):
    """Parity of the timed hexahedral output against the NumPy oracle
    (HexPoissonProblem).  One rank: the whole mesh.  Several ranks: (a) a box
    of two elements per axis in the middle of the rank's part, compared on
    the nodes the box's elements alone determine; (b) the two element layers
    across the rank's +x face, [ex1 - 1, ex1 + 1) (x two elements in the
    middle of the rank's y/z range for a box, the whole y/z extent for a
    slab; the neighbour's u regenerated from the global field), compared on
    this rank's nodes of that box, the last x layer being the shared face
    whose value exists only after the exchange."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    half = gll["half_%d" % p]

    def rel(a, b):
        return float(np.linalg.norm(a - b) / np.linalg.norm(b))
    t0 = time.perf_counter()
    ext = p > 10  # the extended-precision oracle, on blocks

    def oracle(nodes, e2n, u_sub):
        if ext:
            return np.asarray(sem_oracle.hex_poisson_apply_extended(nodes, e2n, half, u_sub),
                              dtype=np.float64)
        return sem_oracle.HexPoissonProblem(nodes, e2n, half).apply(u_sub)
    vs = ("oracle/sem_oracle.py hex_poisson_apply_extended (x87 extended precision; the "
          "float64 transform is ill-conditioned above p = 10)" if ext else
          "oracle/sem_oracle.py HexPoissonProblem")
    if world == 1 and not ext:
        nodes, e2n = part.local_mesh(warp)
        ref = sem_oracle.HexPoissonProblem(nodes, e2n, half).apply(u.cpu().numpy())
        return {"rel_l2": rel(y.cpu().numpy(), ref), "tolerance": 1e-10,
                "vs": "oracle/sem_oracle.py HexPoissonProblem (whole mesh)",
                "oracle_sec": time.perf_counter() - t0}, None
    rng = _hex_ranges(part)  # (world 1 above p = 10: a block, not the whole mesh)
    slab = not hasattr(part, "ranges")

    def middle(a):
        r0, r1 = rng[a]
        if slab and a > 0:
            return (r0, r1)
        c0 = r0 + max(0, (r1 - r0 - 2) // 2)
        return (c0, min(r1, c0 + 2))
    box = [middle(0), middle(1), middle(2)]
    nodes, e2n, gids = meshgen.structured_box(part.nex, part.ney, part.nez, p, *box, warp=warp)
    loc = _hex_gid_to_local(part, gids)
    y_ref = oracle(nodes, e2n, u[torch_index(loc, dev)].cpu().numpy())
    inner = np.flatnonzero(_hex_sub_box(part, box))
    block = {"rel_l2": rel(y[torch_index(loc[inner], dev)].cpu().numpy(), y_ref[inner]),
             "tolerance": 1e-10, "nodes_checked": int(inner.size),
             "block": "elements %s of the rank's %s" % (
                 " x ".join("[%d,%d)" % b for b in box), _hex_desc(part)), "vs": vs,
             "oracle_sec": time.perf_counter() - t0}
    iface = None
    if rng[0][1] < part.nex:
        c0 = rng[0][1] - 1
        box = [(c0, c0 + 2), middle(1), middle(2)]
        nodes, e2n, gids = meshgen.structured_box(part.nex, part.ney, part.nez, p, *box,
                                                  warp=warp)
        y_ref = oracle(nodes, e2n, global_field_at(part, gids, dev).cpu().numpy())
        sel = _hex_sub_box(part, box, keep_lo_x=False)
        sel &= (gids // (part.Ny * part.Nz)) <= rng[0][1] * p  # this rank's x layers
        own = np.flatnonzero(sel)
        face = int(((gids // (part.Ny * part.Nz))[own] == rng[0][1] * p).sum())
        iface = {"rel_l2": rel(y[torch_index(_hex_gid_to_local(part, gids[own]),
                                             dev)].cpu().numpy(), y_ref[own]),
                 "tolerance": 1e-10, "nodes_checked": int(own.size), "interface_nodes": face,
                 "block": "elements %s across the rank's +x face" % (
                     " x ".join("[%d,%d)" % b for b in box))}
    return block, iface


def bench_hex(args):
    """Hexahedral Poisson action (rows N2 / N3: north_star's "structured
    quad/hex meshes ... at 1/2/4/8 GPUs"): --hex-ne^3 warped hexahedra of
    order p (default p = 8, 27^3 = 19,683 elements, 10,218,313 DOF, ~1e7 DOF
    like config 4).  One GPU: a step = one sem_apply (element kernel + seam
    sum).  N ranks: the mesh in N slabs along x (SlabPartition), a step = one
    sem_dd_apply per rank (interface elements + RCCL face exchange on a side
    stream, interior elements on the caller's stream, the finish)."""
    import torch
    import torch.distributed as dist
    from spectralelementmethod_amd.distributed import OverlappedOperator
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_one_gpu:
        local_rank = 0
        args.transport = "torch"
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        _init_process_group(args, dev)
    p = args.p
    part = _hex_partition(args, world, rank)
    t0 = time.time()
    nodes, e2n = part.local_mesh(args.warp)
    log("rank %d: hex %s of %dx%dx%d p=%d: %d elements, %d nodes (%.1fs)" % (
        rank, _hex_desc(part), part.nex, part.ney, part.nez, p, e2n.shape[0],
        nodes.shape[1], time.time() - t0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    op = OverlappedOperator(p, nodes, e2n, part.neighbors if world > 1 else {}, 1, dev,
                            owned=part.owned, transport=args.transport, world=world, rank=rank)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    del nodes, e2n
    plan = op.plan_info()
    log("rank %d: hex plan %s; %d interface + %d interior elements; transport %s; setup %.2fs"
        % (rank, plan, op.n_iface_elem, op.n_interior_elem, op.transport, t_setup))
    u = global_random_field(part, 1, 0, op.ndof, dev)
    y = torch.empty_like(u)
    for _ in range(args.warmup):
        op.step(u, y)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    events = [(ev(), ev()) for _ in range(args.steps)]
    region = (ev(), ev())
    each = args.step_events == "each"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        if each:
            op.step(u, y, events[k])
        else:
            op.step(u, y, (region[0] if k == 0 else None,
                           region[1] if k == args.steps - 1 else None))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if not each:  # untimed: per-action quartiles
        for k in range(args.steps):
            op.step(u, y, events[k])
        torch.cuda.synchronize()
    kern_ms = [a.elapsed_time(b) for a, b in events]
    kern_avg_s = (float(np.mean(kern_ms)) if each else
                  region[0].elapsed_time(region[1]) / args.steps) / 1e3
    per_rank_ms = [elapsed / args.steps * 1e3]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank_ms[0])
        per_rank_ms = gathered
    parity, parity_iface, parity_ranks = None, None, None
    if not args.no_check:
        parity, parity_iface = hex_parity_checks(op, y, u, part, p, args.warp, dev, world)
        log("rank %d: hex parity %s; interface %s" % (rank, parity, parity_iface))
        assert parity["rel_l2"] < parity["tolerance"], parity
        if parity_iface is not None:
            assert parity_iface["rel_l2"] < parity_iface["tolerance"], parity_iface
        if world > 1:
            parity_ranks = [None] * world
            dist.all_gather_object(parity_ranks, (parity["rel_l2"], None if parity_iface is None
                                                  else parity_iface["rel_l2"]))
    n_nodes, E = op.ndof, op.n_elem
    ndof_global = part.global_nodes
    B = alg_bytes_hex(n_nodes, E, p)
    F = alg_flops_hex(E, p)
    achieved = B / kern_avg_s / 1e9
    traffic, traffic_src = None, args.traffic_json
    if traffic_src is None and (p, part.nex, part.ney) == (8, 27, 27) and world == 1:
        traffic_src = os.path.join(ROOT, "bench_traffic", "pmc_traffic_hex_p8_27.json")
    if traffic_src and os.path.exists(traffic_src):
        with open(traffic_src) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    hk = plan.get("hex_kernel", "three_block")
    result = {
        "metric": METRIC.replace("Poisson p=8", "Poisson p=%d on hexahedra" % p),
        "value": ndof_global * args.steps / elapsed, "unit": "DOF/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (structured warped hexahedral mesh, u ~ N(0,1))",
        "config": {
            "workload": "poisson hex p=%d, %dx%dx%d hexahedra%s (rows N2/N3, north_star "
                        "'quad/hex')" % (p, part.nex, part.ney, part.nez,
                                         (" in %d %s" % (world, "boxes %s" % "x".join(
                                             str(g) for g in part.grid) if hasattr(part, "grid")
                                             else "slabs")) if world > 1 else ""),
            "p": p, "ndim": 3, "geometry": "stored", "n_elem_global": part.nex * part.ney *
            part.nez, "n_elem_per_gpu": E, "ndof_global": ndof_global, "ndof_per_gpu": n_nodes,
            "ranks_seen": world,
            "parallelism": "single GPU" if world == 1 else (
                "%s x%d; interface elements on a side stream, shared-node exchange "
                "(transport %s) overlapped with the interior elements" % (
                    ("boxes on a %s rank grid" % "x".join(str(g) for g in part.grid))
                    if hasattr(part, "grid") else "slabs of element layers along x",
                    world, op.transport)),
            "per_rank_ms_per_step": per_rank_ms,
            "exchange_bytes_per_step_per_rank": 2 * op.exchange_bytes,
            "interface_elements": op.n_iface_elem,
            "kernel_ms_avg": kern_avg_s * 1e3, "kernel_ms_min": float(np.min(kern_ms)),
            "kernel_ms_quartiles": [float(q) for q in np.percentile(kern_ms, [25, 50, 75])],
            "kernel_ms_note": ("HIP events around each step on the launch stream" if each else
                               "HIP events around the K timed steps / K (element kernel + seam "
                               "sum + the gaps); min / quartiles from per-step events of a "
                               "second, untimed pass"),
            "step_events": args.step_events,
            "decomposition": op.dd_info(),
            "gflops_kernel": F / kern_avg_s / 1e9, "gpu_setup_sec": t_setup,
            "plan": plan,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": os.path.relpath(traffic_src, ROOT) if traffic is not None else None,
            "bytes_model": "16*ndof + 52*E*(p+1)^3 (u, y, 6 factors + uint32 map per element node)",
            "alg_bytes_per_launch": B, "kernel": "%s<%d,0> + k_hex_seam_sum" % (
                "k_hex_rows" if hk == "rows" else "k_hex_poisson", p + 1),
            "fp64_tflops": F / kern_avg_s / 1e12, "fp64_peak_tflops": FP64_PEAK_TFLOPS,
        },
    }
    if parity is not None:
        result["parity"] = parity
    if parity_iface is not None or parity_ranks is not None:
        result["parity_interface"] = parity_iface
        result["parity_per_rank"] = parity_ranks
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing CPU baseline (hexahedral NumPy oracle, child process)...")
        env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1",
                   MKL_NUM_THREADS="1")
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-only",
                              "--dim", "3", "--p", str(p), "--warp", str(args.warp),
                              "--cpu-budget", str(args.cpu_budget), "--cpu-workers",
                              str(args.cpu_workers)],
                             env=env, capture_output=True, text=True, check=True)
        cb = json.loads(out.stdout.strip().splitlines()[-1])
        fm = cb["faithful_mp"]
        result["cpu_baseline"] = {
            "value": fm["dof_per_s"], "unit": "DOF/s", "cores": fm["workers"], "kind": "port",
            "sample": "per-element dense 3-D Laplacian applied element by element + np.add.at "
                      "(the hexahedral form of examples/poisson.py:168-193 / squirmer:286), %d "
                      "processes x OMP_NUM_THREADS=1 over an 8^3 p=%d warped mesh (%d DOF); "
                      "host os.cpu_count()=%d" % (fm["workers"], p, fm["ndof"], os.cpu_count()),
            "batched_sumfact_1thread_dof_per_s": cb["batched_sumfact"]["dof_per_s"],
            "batched_sumfact_sample": "12^3 p=%d (%d DOF)" % (p, cb["batched_sumfact"]["ndof"]),
        }
    if rank == 0:
        print(json.dumps(result), file=JSON_OUT, flush=True)
    op.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def _init_process_group(args, dev):
    """One rank's process group (gloo for CPU-side objects, NCCL = RCCL for
    device tensors), stdout kept for the JSON line."""
    import datetime
    import torch.distributed as dist
    # keep stdout for the one JSON line: gloo / RCCL print connection
    # banners on file descriptor 1 from C++ (they go to stderr instead)
    global JSON_OUT
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    pg_timeout = datetime.timedelta(seconds=args.deadline)
    if args.rehearse_one_gpu:
        dist.init_process_group("gloo", timeout=pg_timeout)
    else:
        dist.init_process_group("cpu:gloo,cuda:nccl", device_id=dev, timeout=pg_timeout)
    dist.barrier()


# ---------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, deadline_s):
    """Start n rank processes of this script (before any GPU call here), each
    in its own process group, and watch them: the first rank that exits
    non-zero (RCCL init, OOM, a bad partition) or the deadline ends the run --
    the others are killed (they would otherwise wait in a collective for a
    peer that is gone) and the launcher returns non-zero within seconds.
    Rank 0 prints the JSON line."""
    import signal
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, start_new_session=True))

    def kill_all():
        for pr in procs:
            if pr.poll() is None:
                try:
                    os.killpg(pr.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        for pr in procs:
            pr.wait()

    t_end = time.monotonic() + deadline_s
    while True:
        codes = [pr.poll() for pr in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            log("rank %d exited with status %d: stopping the other ranks" % bad[0])
            kill_all()
            return 1
        if all(c == 0 for c in codes):
            return 0
        if time.monotonic() > t_end:
            log("deadline of %.0f s reached: stopping all ranks" % deadline_s)
            kill_all()
            return 124
        time.sleep(0.2)


def _inject_failure(rank):
    """Test hook (tests/test_bench_launcher.py): SEM_BENCH_INJECT=fail:<r>
    makes rank r exit with status 3 at start-up and every other rank wait as
    if blocked in a collective on the missing peer."""
    spec = os.environ.get("SEM_BENCH_INJECT", "")
    if spec.startswith("fail:"):
        if rank == int(spec[5:]):
            log("rank %d: injected failure" % rank)
            sys.exit(3)
        time.sleep(3600)


# ---------------------------------------------------------------- parity spot check
def parity_spot_check(op, y, u, part, p, warp, cols=2):
    """Recompute the action on a block of `cols` element columns in the
    middle of this rank's strip with the NumPy oracle (float64) and compare
    with the timed output on the block's inner nodes (its left/right node
    lines also receive contributions from outside the block)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    ncol = part.ex1 - part.ex0
    cols = min(cols, ncol)
    c0 = part.ex0 + (ncol - cols) // 2
    nodes, e2n, off = meshgen.structured_strip(part.nex, part.ney, p, c0, c0 + cols, warp)
    loc = off - part.node_offset + np.arange(nodes.shape[1])
    u_sub = u[torch_index(loc, u.device)].cpu().numpy()
    half = gll["half_%d" % p]
    y_ref = sem_oracle.PoissonProblem(nodes, e2n, half, batched_geometry=True).apply(u_sub)
    Ny = part.Ny
    inner = np.arange(Ny, nodes.shape[1] - Ny)
    y_gpu = y[torch_index(loc[inner], y.device)].cpu().numpy()
    ref = y_ref[inner]

    def rel(a, b):
        return float(np.linalg.norm(a - b) / np.linalg.norm(b))
    out = dict(rel_l2=rel(y_gpu, ref), nodes_checked=int(inner.size),
               block="element columns [%d, %d) x %d rows" % (c0, c0 + cols, part.ney),
               against="float64 NumPy oracle of the reference path")
    if p > 10:
        # above p = 10 the reference's own float64 geometry (equispaced->GLL
        # transform, cond(V_eq) 1e3..1e5) is the inaccurate side (DESIGN.md
        # §6): the criterion is the extended-precision evaluation of the same
        # action from the same float64 inputs, at the same 1e-10
        ext = np.asarray(sem_oracle.poisson_apply_extended(nodes, e2n, half, u_sub),
                         dtype=np.float64)[inner]
        out.update(rel_l2_float64_oracle=out["rel_l2"], rel_l2=rel(y_gpu, ext),
                   oracle_float64_vs_extended=rel(ref, ext),
                   against="extended-precision oracle (poisson_apply_extended)")
    return out


def global_field_at(part, gids, dev):
    """u at arbitrary GLOBAL node ids (e.g. a neighbour's nodes next to the
    interface): the global field of global_random_field regenerated chunk by
    chunk on the device (the same Philox stream), entries picked."""
    import torch
    g = torch.Generator(device=dev).manual_seed(1234)
    gids = torch_index(gids, dev)
    out = torch.empty(gids.numel(), dtype=torch.float64, device=dev)
    chunk, pos, n_glob = 1 << 24, 0, part.global_nodes
    while pos < n_glob:
        m = min(chunk, n_glob - pos)
        v = torch.randn(m, dtype=torch.float64, device=dev, generator=g)
        sel = (gids >= pos) & (gids < pos + m)
        out[sel] = v[gids[sel] - pos]
        pos += m
    return out


def parity_interface_check(y, part, p, warp, dev):
    """The interface sum, checked against the oracle: the two element columns
    on either side of this rank's right interface, [ex1 - 1, ex1 + 1),
    recomputed by the NumPy oracle (u of the neighbour's column regenerated
    from the global field) and compared on this rank's own inner nodes of the
    block -- node lines (ex1 - 1) p + 1 .. ex1 p, the last one being the
    shared line whose value this rank only has after the exchange."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    if part.rank == part.world - 1:
        return None
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    c0 = part.ex1 - 1
    nodes, e2n, off = meshgen.structured_strip(part.nex, part.ney, p, c0, c0 + 2, warp)
    gids = off + np.arange(nodes.shape[1])
    u_sub = global_field_at(part, gids, dev).cpu().numpy()
    y_ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p],
                                      batched_geometry=True).apply(u_sub)
    Ny = part.Ny
    own = np.arange(Ny, (p + 1) * Ny)  # block node lines 1 .. p
    loc = gids[own] - part.node_offset
    y_gpu = y[torch_index(loc, y.device)].cpu().numpy()
    ref = y_ref[own]
    return dict(rel_l2=float(np.linalg.norm(y_gpu - ref) / np.linalg.norm(ref)),
                nodes_checked=int(own.size), interface_nodes=int(Ny),
                block="element columns [%d, %d) x %d rows across the interface with rank %d" % (
                    c0, c0 + 2, part.ney, part.rank + 1),
                against="float64 NumPy oracle of the reference path")


def torch_index(a, device):
    import torch
    return torch.from_numpy(np.asarray(a, dtype=np.int64)).to(device)


# ---------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the driver's own command (--steps 20 --warmup 5); the per-action kernel
    # time quartiles in the JSON show the clock under sustained fp64 load
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--nex", type=int, default=1024,
                    help="element columns of the global mesh (strong) or per rank (weak)")
    ap.add_argument("--ney", type=int, default=1024)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--warp", type=float, default=0.05)
    ap.add_argument("--op", choices=["poisson", "axisym_stokes", "axisym_ns", "pcg"],
                    default="poisson")
    ap.add_argument("--re", type=float, default=10.0, help="Reynolds number for --op axisym_ns")
    ap.add_argument("--geometry", choices=["auto", "nodal", "stored"], default="auto",
                    help="Poisson geometric factors: re-derived from x_phys per node, or "
                         "streamed; auto = the library's per-order choice")
    ap.add_argument("--kernel", choices=["auto", "column", "mfma"], default="auto",
                    help="Poisson kernel family: LDS column kernel or fp64-MFMA element kernel; "
                         "auto = the library's measured choice")
    ap.add_argument("--transport", choices=["auto", "rccl", "torch"], default="auto",
                    help="interface sum with several ranks: native RCCL or torch.distributed")
    ap.add_argument("--pcg-rtol", type=float, default=0.0,
                    help="--op pcg: 0 = time exactly --steps iterations; > 0 = solve to it")
    # region (default): one HIP event pair around the K timed actions; a pair
    # around every action costs the step ~10 us of queue markers (one rank of
    # the 8-strip split: 0.107 against 0.095-0.098 ms per step; the driver
    # command 0.636-0.644 against 0.622-0.637, profiles/r05/step_events/)
    ap.add_argument("--step-events", choices=["each", "region"], default="region",
                    help="one HIP event pair around the timed region (per-action quartiles "
                         "then from an untimed pass), or a pair around every timed action")
    ap.add_argument("--kernel-series", action="store_true",
                    help="also write every timed action's HIP-event time into the JSON")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the parity spot check (timing-only diagnostic builds)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--deadline", type=float, default=900.0,
                    help="seconds: the whole multi-rank run (launcher kills every rank after it) "
                         "and the process-group timeout of each rank")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="diagnostic: every rank on cuda:0, gloo process group, torch transport "
                         "(exercises the multi-rank flow on a one-GPU box; timings meaningless)")
    ap.add_argument("--time-rank", type=int, default=None, metavar="R",
                    help="diagnostic: time rank R of the --gpus N strip decomposition ALONE on "
                         "this GPU (loopback transport: the exchange returns the rank's own "
                         "values; kernels, streams and host enqueue of the real step)")
    ap.add_argument("--time-rank-transport", choices=["loopback", "rccl_self"],
                    default="rccl_self",
                    help="--time-rank: the exchange as RCCL send/recv to this rank itself on a "
                         "one-rank communicator (default) or the loopback copy kernel")
    ap.add_argument("--dump-interface", default=None, metavar="DIR",
                    help="test hook: every rank writes y at its interface node lines (global "
                         "ids, values) to DIR/iface_rank<r>.npz after the timed steps")
    ap.add_argument("--traffic-json", default=None,
                    help="JSON with PMC-measured HBM bytes per launch (profiles/)")
    ap.add_argument("--numbering", choices=["lex", "rcm"], default="lex",
                    help="rcm: the reference DOFManager's default node order (reverse "
                         "Cuthill-McKee of the element-clique graph, sem/discrete.py:169-178), "
                         "element order unchanged; one GPU, Poisson")
    ap.add_argument("--renumber", choices=["auto", "off"], default="auto",
                    help="--op pcg on one GPU: solve in the kernel's traversal numbering "
                         "when it reads fewer lines (auto) or keep the caller's (off)")
    ap.add_argument("--dim", type=int, choices=[2, 3], default=2,
                    help="3: the hexahedral Poisson action (bench_hex)")
    ap.add_argument("--hex-ne", type=int, default=27, help="--dim 3: hexahedra per side")
    ap.add_argument("--hex-nex", type=int, default=None,
                    help="--dim 3: element layers along x (the slab axis; default --hex-ne), "
                         "per rank with --scaling weak")
    ap.add_argument("--hex-decomp", choices=["block", "slab"], default="slab",
                    help="--dim 3 on N ranks: slabs of element layers along x (slab) or "
                         "boxes on a near-cubic rank grid (block)")
    args = ap.parse_args()

    if args.cpu_baseline_only:  # child process: no GPU
        fn = cpu_baseline_hex if args.dim == 3 else cpu_baseline
        print(json.dumps(fn(args.p, args.warp, args.cpu_budget, args.cpu_workers)))
        return 0
    if args.time_rank is not None:
        return time_rank(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, args.deadline)
    if args.dim == 3:
        return bench_hex(args)

    import torch
    import torch.distributed as dist
    from spectralelementmethod_amd import _lib  # noqa: F401
    from spectralelementmethod_amd.distributed import StripPartition, OverlappedOperator
    from spectralelementmethod_amd.operators import POISSON, AXISYM_STOKES, AXISYM_NS

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    _inject_failure(rank)
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    if args.rehearse_one_gpu:
        local_rank = 0
        args.transport = "torch"
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        _init_process_group(args, dev)

    opname = args.op
    kind = {"poisson": POISSON, "pcg": POISSON, "axisym_stokes": AXISYM_STOKES,
            "axisym_ns": AXISYM_NS}[opname]
    kname = "poisson" if kind == POISSON else opname
    dpn = 1 if kind == POISSON else 2
    p = args.p
    nex_global = args.nex * world if args.scaling == "weak" else args.nex
    part = StripPartition(nex_global, args.ney, p, world, rank, dofs_per_node=dpn)
    t0 = time.time()
    if kind == POISSON:
        nodes, e2n = part.local_mesh(args.warp)
        if args.numbering == "rcm":
            if world != 1:
                raise SystemExit("--numbering rcm is single-GPU")
            from spectralelementmethod_amd.discrete import rcm_permutation
            t0 = time.time()
            # what DOFManager(mesh, ...) does by default (rcm_order=True):
            # scipy's RCM of the graph joining every two nodes of a cell
            # (sem/discrete.py:142-178), walked on the cell map natively
            # (equal to scipy's permutation, tests/test_order.py)
            perm = rcm_permutation(e2n.reshape(e2n.shape[0], -1), nodes.shape[1])
            inv = np.empty_like(perm)
            inv[perm] = np.arange(perm.size, dtype=perm.dtype)
            nodes = nodes[:, perm].copy()
            e2n = inv[e2n].astype(np.uint32)
            log("RCM numbering (reference default): %.1fs" % (time.time() - t0))
    else:
        from spectralelementmethod_amd import meshgen
        if world != 1:
            raise SystemExit("axisymmetric bench is single-GPU")
        nodes, e2n = meshgen.annulus(args.nex, args.ney, p)
    t_mesh = time.time() - t0
    log("rank %d: mesh %d elements, %d nodes (%.1fs)" % (rank, e2n.shape[0], nodes.shape[1],
                                                          t_mesh))
    geometry = args.geometry if kind in (POISSON, AXISYM_STOKES) else "stored"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    op = OverlappedOperator(p, nodes, e2n, part.neighbors if world > 1 else {}, dpn, dev,
                            geometry=geometry, kind=kind, kernel=args.kernel, owned=part.owned,
                            transport=args.transport, world=world, rank=rank)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    if kind == AXISYM_NS:
        for o in op.ops:
            o.set_reynolds(args.re)
    plan = op.plan_info()
    # as the library resolved it
    geometry = (plan["geometry"] if kind == POISSON else
                plan["geometry_axisym"] if kind == AXISYM_STOKES else "stored")
    log("rank %d: plan %s; %d interface + %d interior elements; transport %s; setup %.2fs" % (
        rank, plan, op.n_iface_elem, op.n_interior_elem, op.transport, t_setup))
    n_elem_local = op.n_elem
    n_nodes_local = op.ndof // dpn
    ndof_global = part.global_nodes * dpn if kind == POISSON else op.ndof

    if opname == "pcg":
        return bench_pcg(args, op, part, nodes, dev, world, rank, ndof_global, t_setup)
    rcm_nodes, rcm_e2n = (nodes, e2n) if args.numbering == "rcm" else (None, None)
    del nodes, e2n

    # u from one global field so shared DOFs agree on both sides of an interface
    u = global_random_field(part, dpn, kind, op.ndof, dev)
    if args.numbering == "rcm":  # the same field, renumbered
        u = u[torch_index(perm, dev)].contiguous()
    y = torch.empty_like(u)

    for _ in range(args.warmup):
        op.step(u, y)
    torch.cuda.synchronize()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    # --step-events each: a HIP event pair around every timed action;
    # region: one pair around the K actions (per-action average = region / K),
    # the per-action quartiles from a second, untimed pass of K actions
    events = [(ev(), ev()) for _ in range(args.steps)]
    region = (ev(), ev())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        if args.step_events == "each":
            op.step(u, y, events[k])
        else:
            op.step(u, y, (region[0] if k == 0 else None,
                           region[1] if k == args.steps - 1 else None))
    t_enqueue = time.perf_counter() - t_start  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    region_ms = None
    if args.step_events == "region":
        region_ms = region[0].elapsed_time(region[1]) / args.steps
        for k in range(args.steps):  # untimed: per-action quartiles
            op.step(u, y, events[k])
        torch.cuda.synchronize()
    kern_ms = [a.elapsed_time(b) for a, b in events]
    per_rank_ms = [elapsed / args.steps * 1e3]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank_ms[0])
        per_rank_ms = gathered
    kern_avg_s = (region_ms if region_ms is not None else float(np.mean(kern_ms))) / 1e3

    parity, parity_ranks, parity_iface = None, None, None
    if not args.no_check and args.numbering == "rcm":
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import sem_oracle
        gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
        P = sem_oracle.PoissonProblem(rcm_nodes, rcm_e2n, gll["half_%d" % p],
                                      batched_geometry=True)
        ref = P.apply(u.cpu().numpy())
        parity = {"rel_l2": float(np.linalg.norm(y.cpu().numpy() - ref) / np.linalg.norm(ref)),
                  "vs": "oracle on the whole RCM-numbered mesh", "tolerance": 1e-10}
        log("parity %s" % parity)
        assert parity["rel_l2"] < parity["tolerance"], parity
    elif not args.no_check:
        assert torch.isfinite(y).all().item(), "non-finite output"
        if kind == POISSON:
            parity = parity_spot_check(op, y, u, part, p, args.warp)
            parity["tolerance"] = 1e-10
            log("rank %d: parity spot check %s" % (rank, parity))
            assert parity["rel_l2"] < parity["tolerance"], parity
            iface = parity_interface_check(y, part, p, args.warp, dev) if world > 1 else None
            if iface is not None:
                iface["tolerance"] = 1e-10
                log("rank %d: interface parity %s" % (rank, iface))
                assert iface["rel_l2"] < iface["tolerance"], iface
            if world > 1:
                parity_ranks = [None] * world
                dist.all_gather_object(parity_ranks, parity["rel_l2"])
                parity_iface = [None] * world
                dist.all_gather_object(parity_iface, None if iface is None else iface["rel_l2"])
    if args.dump_interface and kind == POISSON:
        lines = [k for k in sorted(part.neighbors)]
        loc = np.concatenate([part.neighbors[k] for k in lines]) if lines else np.zeros(0, int)
        np.savez(os.path.join(args.dump_interface, "iface_rank%d.npz" % rank),
                 gid=part.node_offset + loc, y=y[torch_index(loc, dev)].cpu().numpy())

    value = ndof_global * args.steps / elapsed
    map_bytes = plan.get("map_entry_bytes", 4) if (
        plan["kernel"] == "column" and (kind == POISSON or geometry == "nodal")) else 4
    B = alg_bytes_s8d(kname, n_nodes_local, n_elem_local, p)
    B_stream = streamed_bytes(kname, n_nodes_local, n_elem_local, p, geometry, map_bytes,
                              plan.get("map_patterns", 0) if map_bytes == 2 else 0)
    F = alg_flops(kname, n_elem_local, p, geometry)
    achieved = B / kern_avg_s / 1e9
    traffic, traffic_src = None, args.traffic_json
    if (traffic_src is None and kind == POISSON and plan["kernel"] == "column" and world == 1
            and (p, args.nex, args.ney) == (8, 1024, 1024) and args.numbering == "lex"):
        traffic_src = os.path.join(ROOT, "bench_traffic", DEFAULT_TRAFFIC[geometry])
    if traffic_src and os.path.exists(traffic_src):
        with open(traffic_src) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    headline = (args.nex, args.ney, p) == (1024, 1024, 8)
    result = {
        "metric": METRIC if kind == POISSON else METRIC.replace(
            "Poisson p=8", ("axisymmetric Stokes p=%d" if kind == AXISYM_STOKES else
                            "axisymmetric Navier-Stokes residual p=%d") % p),
        "value": value,
        "unit": "DOF/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (structured warped quad mesh, u ~ N(0,1))",
        "config": {
            "numbering": args.numbering,
            "workload": "%s p=%d, %dx%d elements %s (%s)" % (
                opname, p, args.nex, args.ney,
                "global mesh in %d strip(s)" % world if args.scaling == "strong"
                else "per GPU", "BASELINE config 3, the 10^6-element north-star mesh"
                if headline and args.scaling == "strong" else "custom"),
            "p": p, "geometry": geometry, "ranks_seen": world,
            "n_elem_global": part.nex * part.ney if kind == POISSON else n_elem_local,
            "n_elem_per_gpu": n_elem_local, "ndof_global": ndof_global,
            "ndof_per_gpu": op.ndof,
            "parallelism": ("element column strips x%d; interface elements on a side stream, "
                            "RCCL send/recv interface sum overlapped with the interior elements "
                            "(transport %s)" % (world, op.transport)) if world > 1 else
            "single GPU",
            "per_rank_ms_per_step": per_rank_ms,
            "exchange_bytes_per_step_per_rank": 2 * op.exchange_bytes,
            "interface_elements": op.n_iface_elem,
            "kernel_ms_avg": kern_avg_s * 1e3, "kernel_ms_min": float(np.min(kern_ms)),
            "kernel_ms_note": ("avg = mean of the timed actions' HIP-event times, including the "
                               "shader-clock ramp of the first actions (it must match the "
                               "rocprofv3 average); the median is kernel_ms_quartiles[1]"
                               if region_ms is None else
                               "avg = HIP events around the K timed actions / K (gaps between "
                               "the launches included; the rocprofv3 averages sum to at most "
                               "it); min / quartiles / max from per-action events of a second, "
                               "untimed pass"),
            "step_events": args.step_events,
            "kernel_ms_quartiles": [float(q) for q in np.percentile(kern_ms, [25, 50, 75])],
            "kernel_ms_max": float(np.max(kern_ms)),
            "kernel_ms_series": [round(float(x), 5) for x in kern_ms] if args.kernel_series
            else None,
            "host_enqueue_ms_per_step": t_enqueue / args.steps * 1e3,
            "decomposition": op.dd_info(),
            "gflops_kernel": F / kern_avg_s / 1e9,
            "kernel_family": plan["kernel"], "map_entry_bytes": map_bytes,
            "gpu_setup_sec": t_setup, "gpu_setup_sec_per_elem": t_setup / max(1, n_elem_local),
            "scatter_plan": {k: plan[k] for k in ("plan", "colours", "chains_per_colour", "rounds",
                                                  "zero_list", "atomic_groups", "seam_nodes",
                                                  "map_patterns") if k in plan},
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "bytes_model": "SURVEY.md §8(d): 16*ndof + 28*E*(p+1)^2" if kind == POISSON else
            "SURVEY.md §8(d) axisymmetric: 32*n_nodes + (60|76)*E*(p+1)^2",
            "alg_bytes_per_launch": B,
            "streamed_bytes_per_launch": B_stream,
            "frac_streamed_min": B_stream / kern_avg_s / 1e9 / HBM_PEAK_GBS,
            "kernel": (("k_poisson_mfma<%d>" if plan["kernel"] == "mfma" else
                        "k_poisson_apply<%d>") % (p + 1) if kind == POISSON else
                       ("k_axisym_nodal<%d>" if geometry == "nodal" else "k_axisym_apply<%d>")
                       % (p + 1)),
            "launch": ("one sem_apply = one launch of %d chains + k_seam_sum over %d seam nodes"
                       % (plan["chains_per_colour"][0], plan["seam_nodes"])
                       if plan["plan"] == "chains-seams" else
                       "one sem_apply = %d colour launches" % plan["colours"]) if world == 1 else
            "one sem_dd_apply (interface + interior elements + exchange), per rank",
            "fp64_tflops": F / kern_avg_s / 1e12, "fp64_peak_tflops": FP64_PEAK_TFLOPS,
            "traffic_source": os.path.relpath(traffic_src, ROOT) if traffic is not None else None,
        },
    }
    if parity is not None:
        result["parity"] = parity
    if parity_ranks is not None:
        result["parity_per_rank"] = parity_ranks
        result["parity_interface_per_rank"] = parity_iface
    if rank == 0 and world == 1 and not args.no_cpu_baseline and kind == POISSON:
        log("timing CPU baseline (NumPy oracle of the reference path, child process)...")
        env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1",
                   MKL_NUM_THREADS="1")
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-only",
                              "--p", str(p), "--warp", str(args.warp), "--cpu-budget",
                              str(args.cpu_budget), "--cpu-workers", str(args.cpu_workers)],
                             env=env, capture_output=True, text=True, check=True)
        cb = json.loads(out.stdout.strip().splitlines()[-1])
        f1, fm = cb["faithful_1"], cb["faithful_mp"]
        result["cpu_baseline"] = {
            "value": fm["dof_per_s"], "unit": "DOF/s", "cores": fm["workers"], "kind": "port",
            "sample": "reference-faithful per-element Lse einsum('pqrs,rs') + np.add.at "
                      "(examples/poisson.py:168-193, squirmer:286), %d processes x "
                      "OMP_NUM_THREADS=1 over a 128x128 p=%d warped mesh (%d DOF), element "
                      "slices summed; median of %d; host os.cpu_count()=%d" % (
                          fm["workers"], p, fm["ndof"], fm["reps"], os.cpu_count()),
            "faithful_1thread_dof_per_s": f1["dof_per_s"],
            "faithful_1thread_sample": "64x64 p=%d (%d DOF), median of %d" % (p, f1["ndof"],
                                                                               f1["reps"]),
            "batched_elem_matrix_1thread_dof_per_s": cb["batched_elem_matrix"]["dof_per_s"],
            "batched_sumfact_1thread_dof_per_s": cb["batched_sumfact"]["dof_per_s"],
            "batched_sumfact_sample": "256x256 p=%d (%d DOF)" % (p, cb["batched_sumfact"]["ndof"]),
            "full_host_extrapolated": {
                "value": fm["dof_per_s"] * (os.cpu_count() or 1) / fm["workers"],
                "cores": os.cpu_count(),
                "note": "the %d-process figure scaled linearly to every core of the host: an "
                        "upper bound, not a measurement (the box's CPU share for one GPU is "
                        "%d processes; the other cores belong to other GPUs' jobs)" % (
                            fm["workers"], fm["workers"])},
            "faithful_setup_sec_per_elem": f1["setup_sec_per_elem"],
            "gpu_setup_sec_per_elem": t_setup / max(1, n_elem_local),
        }
    if rank == 0:
        print(json.dumps(result), file=JSON_OUT, flush=True)
    op.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def time_rank(args):
    """One rank of the N-strip decomposition of the nex x ney mesh, alone on
    this GPU.  --time-rank-transport rccl_self (default, sem_dd_set_rccl_self):
    every exchange is RCCL send/recv per peer addressed to this rank itself on
    a one-rank communicator -- RCCL's host enqueue and side-stream work in the
    real step; loopback (sem_dd_set_loopback): a copy kernel in their place.
    The kernels, streams and host enqueue are those of the real step, the
    values are NOT the global action.  Reports the step
    (wall clock and HIP events on the caller's stream), the interior elements
    alone, the side-stream chain alone (gather, interface elements, pack),
    the exposed time of the side stream and the finish, the host enqueue split
    by sem_dd_info, and the single-GPU step of the whole mesh on the same box:
    strong scaling to N GPUs at >= S x needs the rank's step <= T_1 / S."""
    import torch
    from spectralelementmethod_amd import _lib
    from spectralelementmethod_amd.distributed import StripPartition, OverlappedOperator
    N, R, p = args.gpus, args.time_rank, args.p
    if not (0 <= R < N):
        raise SystemExit("--time-rank needs 0 <= R < --gpus")
    # keep stdout for the one JSON line: RCCL prints its banner on file
    # descriptor 1 from C++ when the communicator is created (to stderr instead)
    global JSON_OUT
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hexa = args.dim == 3
    part = _hex_partition(args, N, R) if hexa else StripPartition(args.nex, args.ney, p, N, R)
    nodes, e2n = part.local_mesh(args.warp)
    op = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, dev, owned=part.owned,
                            transport=args.time_rank_transport, world=1, rank=0, decompose=True)
    del nodes, e2n
    u = global_random_field(part, 1, 0, op.ndof, dev)
    y = torch.empty_like(u)
    lib = _lib.load()
    main = torch.cuda.current_stream(dev)
    sp = _lib.stream_ptr(main)

    def timed(fn, steps, warmup, after_warmup=None):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        if after_warmup is not None:
            after_warmup()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        each = args.step_events == "each"  # region: one pair around the steps
        t0 = time.perf_counter()
        for k, (a, b) in enumerate(ev):
            if each or k == 0:
                a.record(main)
            fn()
            if each or k == steps - 1:
                b.record(main)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms = ([a.elapsed_time(b) for a, b in ev] if each else
              [ev[0][0].elapsed_time(ev[-1][1]) / steps])
        return dict(wall_ms_per_step=wall / steps * 1e3, event_ms_avg=float(np.mean(ms)),
                    event_ms_quartiles=[float(q) for q in np.percentile(ms, [25, 50, 75])],
                    host_enqueue_ms_per_step=t_enq / steps * 1e3)

    K, W = max(1, args.steps), max(1, args.warmup)
    info0 = []  # sem_dd_info after the warm-up (first launches load code objects)
    step = timed(lambda: op.step(u, y), K, W, lambda: info0.append(op.dd_info()))
    i0, i1 = info0[0], op.dd_info()
    n_app = i1["applies"] - i0["applies"]
    d_us = {k: (i1[k] - i0[k]) / n_app / 1e3 for k in
            ("host_ns", "host_ns_transport", "host_ns_side", "host_ns_interior", "host_ns_finish")}
    host_split = dict(host_us_per_apply=d_us["host_ns"],
                      host_us_per_apply_excl_transport=d_us["host_ns"] - d_us["host_ns_transport"],
                      host_us_transport=d_us["host_ns_transport"],
                      host_us_side=d_us["host_ns_side"], host_us_interior=d_us["host_ns_interior"],
                      host_us_finish=d_us["host_ns_finish"])
    # the interior elements alone, as sem_dd_apply launches them
    flags = 2 if i1["zero_list_in_finish"] else 0  # SEM_APPLY_SKIP_ZERO (seam sum included)
    interior = None
    if op.interior is not None:
        interior = timed(lambda: _lib.check(lib.sem_apply(op.interior._ctx, 0, _lib.tptr(u),
                                                          _lib.tptr(y), flags, sp)), K, W)
    # the side-stream chain alone (on the caller's stream here)
    side = None
    if op.iface is not None:
        # as sem_dd_apply's side stream runs it: the interface elements over
        # the rank's numbering (zero list skipped), then the pack
        pl = op.plan
        sidx = torch.from_numpy(pl.iface_dofs[pl.peer_dofs].view(np.int32)).to(dev)
        yc = torch.empty_like(u)
        send = torch.empty(max(1, sidx.numel()), dtype=torch.float64, device=dev)

        def side_chain():
            _lib.check(lib.sem_apply(op.iface._ctx, 0, _lib.tptr(u), _lib.tptr(yc), 2, sp))
            _lib.check(lib.sem_gather(_lib.tptr(yc), _lib.tptr(sidx), sidx.numel(),
                                      _lib.tptr(send), sp))
        side = timed(side_chain, K, W)
    iface_elems, interior_elems = op.n_iface_elem, op.n_interior_elem
    exch_bytes = op.exchange_bytes
    plan_int = op.interior.plan_info() if op.interior is not None else None
    plan_if = op.iface.plan_info() if op.iface is not None else None
    ndof = op.ndof
    op.close()
    del op, u, y
    torch.cuda.empty_cache()
    # the single-GPU step of the whole mesh on this box (the strong-scaling base)
    single = None
    if not args.no_check:
        full = _hex_partition(args, 1, 0) if hexa else StripPartition(args.nex, args.ney, p, 1, 0)
        nodes, e2n = full.local_mesh(args.warp)
        op1 = OverlappedOperator(p, nodes, e2n, {}, 1, dev, world=1, rank=0)
        del nodes, e2n
        u1 = global_random_field(full, 1, 0, op1.ndof, dev)
        y1 = torch.empty_like(u1)
        single = timed(lambda: op1.step(u1, y1), K, W)
        op1.close()
    step_ms = step["wall_ms_per_step"]
    res = {
        "mode": "time-rank (%s transport: the exchange returns this rank's own values; "
                "timing only, the result is NOT the global action)" % args.time_rank_transport,
        "transport": args.time_rank_transport,
        "rank": R, "of_ranks": N, "p": p,
        "mesh": ("%dx%dx%d hexahedra (%s scaling)" % (part.nex, part.ney, part.nez, args.scaling)
                 if hexa else "%dx%d" % (args.nex, args.ney)),
        "strip_elements": (_hex_desc(part) if hexa
                           else "%d x %d" % (part.ex1 - part.ex0, part.ney)), "ndof_rank": ndof,
        "exchange_bytes_per_step": 2 * exch_bytes,
        "peers": sorted(part.neighbors), "interface_elements": iface_elems,
        "interior_elements": interior_elems, "steps": K, "warmup": W,
        "step": step, "interior_alone": interior, "side_chain_alone": side,
        "exposed_beyond_interior_ms": (step["event_ms_avg"] - interior["event_ms_avg"])
        if interior else None,
        "host": host_split, "plan_interior": plan_int, "plan_iface": plan_if,
        "single_gpu_whole_mesh": single,
    }
    if single is not None:
        t1 = single["wall_ms_per_step"]
        for S in (6, 7, N):
            res["budget_ms_for_%dx" % S] = t1 / S
        res["fits_6x"] = step_ms <= t1 / 6
        res["projected_speedup_if_ranks_equal"] = t1 / step_ms
    print(json.dumps(res), file=JSON_OUT, flush=True)
    return 0


def global_random_field(part, dpn, kind, ndof, dev):
    """u ~ N(0,1) drawn per GLOBAL node id (counter-based, so every rank
    draws the same value for a shared node): Philox via torch on the device."""
    import torch
    if kind != 0:
        g = torch.Generator(device=dev).manual_seed(1234)
        return torch.randn(ndof, dtype=torch.float64, device=dev, generator=g)
    if not hasattr(part, "node_offset"):  # a box: not one contiguous global range
        return global_field_at(part, part.local_to_global(), dev)
    # the strip's nodes are the contiguous global range [node_offset, +n_nodes)
    g = torch.Generator(device=dev).manual_seed(1234)
    n_glob = part.global_nodes
    lo = part.node_offset
    # draw the global vector in chunks, keep the rank's window (cheap at 67M)
    out = torch.empty(ndof, dtype=torch.float64, device=dev)
    chunk = 1 << 24
    pos = 0
    while pos < n_glob:
        m = min(chunk, n_glob - pos)
        v = torch.randn(m, dtype=torch.float64, device=dev, generator=g)
        a, b = max(pos, lo), min(pos + m, lo + ndof)
        if a < b:
            out[a - lo:b - lo] = v[a - pos:b - pos]
        pos += m
    return out


def bench_pcg(args, op, part, nodes, dev, world, rank, ndof_global, t_setup):
    """Assembled Poisson solve (DOFManagerSC.solve,
    sem/discrete.py:502-528) by device-resident Jacobi-PCG.  Manufactured
    problem: x* = sin(pi x/2) cos(pi y/2) + x y at the nodes, b = K x*
    (computed by the same distributed operator, so shared DOFs agree),
    Dirichlet x = x* on the square's boundary, x0 = 0 inside.  --pcg-rtol 0:
    a step = one PCG iteration (iterations/s); else solve to the tolerance
    and report time to solution and the error against x*."""
    import torch
    import torch.distributed as dist
    x_n, y_n = torch.from_numpy(nodes[0]).to(dev), torch.from_numpy(nodes[1]).to(dev)
    xs = torch.sin(0.5 * np.pi * x_n) * torch.cos(0.5 * np.pi * y_n) + x_n * y_n
    on = (torch.abs(x_n.abs() - 1) < 1e-9) | (torch.abs(y_n.abs() - 1) < 1e-9)
    # warped mesh: the boundary is still the square's boundary (warp vanishes there)
    b = op.apply(xs)
    x = torch.where(on, xs, torch.zeros_like(xs))
    rtol = args.pcg_rtol
    iters = args.steps
    # warm-up (also builds the diagonal once per call, included in timing below)
    ren = "auto" if args.renumber == "auto" else False
    op.pcg_solve(b, x.clone(), on, rtol=0.0, max_iter=max(1, args.warmup), renumber=ren)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    x_run = x.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, its, rel = op.pcg_solve(b, x_run, on, rtol=rtol, max_iter=iters if rtol == 0 else 200000,
                               renumber=ren)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    own = torch.from_numpy(part.owned).to(dev)
    err_num = torch.sum((x_run - xs)[own] ** 2)
    err_den = torch.sum(xs[own] ** 2)
    if world > 1:
        t = torch.stack([err_num, err_den]).cpu()
        dist.all_reduce(t)
        err_num, err_den = t[0], t[1]
    err = float(torch.sqrt(err_num / err_den))
    solver_numbering = None
    sop = None if op.dd else op.ops[0]
    if sop is not None and sop._solver is not None:
        solver_numbering = {"row_lines_gain": sop.solver_gain,
                            "renumbered": sop._solver[0] is not None,
                            "rule": "traversal numbering when the caller's numbering reads "
                                    ">= 1.3x the 64-byte lines per wavefront row"}
    result = {
        "metric": "assembled Poisson Jacobi-PCG, DOF-iterations/s, p=%d" % args.p,
        "value": ndof_global * its / elapsed, "unit": "DOF*iterations/s", "n_gpus": world,
        "steps": its, "warmup": args.warmup, "ms_per_step": elapsed / max(its, 1) * 1e3,
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic manufactured solution on the structured warped quad mesh",
        "config": {"workload": "pcg p=%d, %dx%d elements (%s)" % (
            args.p, args.nex, args.ney, "fixed iterations" if rtol == 0 else
            "solve to rtol %g" % rtol), "ndof_global": ndof_global, "ranks_seen": world,
            "numbering": args.numbering,
            "transport": op.transport},
        "pcg": {"iterations": its, "iterations_per_s": its / elapsed, "seconds": elapsed,
                "final_relres": rel, "rel_l2_error_vs_manufactured": err,
                "check_every": 16, "gpu_setup_sec": t_setup,
                "solver_numbering": solver_numbering},
    }
    if rank == 0:
        print(json.dumps(result), file=JSON_OUT, flush=True)
    op.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
