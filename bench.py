#!/usr/bin/env python
"""Benchmark: global Poisson stiffness action, DOF-updates/s (BASELINE.json
metric), on synthetic structured quad meshes of order p, elements split in
column strips across ranks (one process per GPU, weak scaling: every rank owns
nex x ney elements).

A step = one global action y = K u over one batch of synthetic input:
  sem_zero_shared(y) -> sem_apply (the element kernel) -> interface sum with
  the neighbouring ranks (RCCL point-to-point; nothing at N = 1).
Inputs are resident in HBM before the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--p 8] [--nex 1024] [--ney 1024]

Rank 0 prints ONE JSON line (the driver's contract) with a ``roofline``
object for the element kernel (algorithmic bytes / HIP-event kernel time,
SURVEY.md §8(d)) and, at N = 1, a ``cpu_baseline`` object (the NumPy oracle
of the reference path timed on this host's cores on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from spectralelementmethod_amd import _lib  # noqa: E402
from spectralelementmethod_amd.distributed import StripPartition, OverlappedOperator  # noqa: E402
from spectralelementmethod_amd.operators import POISSON, AXISYM_STOKES, AXISYM_NS  # noqa: E402

METRIC = "global stiffness-action DOF-updates/s (and % HBM roofline), Poisson p=8"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP64_PEAK_TFLOPS = 78.6  # MI355X vector fp64 (256 CUs x 128 FLOP/clk x 2.4 GHz)
# PMC-measured HBM bytes of the headline workload, per geometry mode
DEFAULT_TRAFFIC = {"stored": "r01/pmc_traffic_p8_1024x1024.json",
                   "nodal": "r01c/pmc_traffic_nodal_p8_1024x1024.json"}


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def alg_bytes(kind, ndof_nodes, n_elem, p, geometry="stored", map_bytes=4):
    """Poisson with stored factors B = 16*ndof + 28*E*(p+1)^2
    (u read, y written, 3 fp64 factors + one uint32 map entry per local
    node); with nodal geometry the factors are replaced by x_phys per global
    node: B = 32*ndof + 4*E*(p+1)^2; axisymmetric B = 32*n_nodes +
    60*E*(p+1)^2 (Navier-Stokes residual: 9 factors, 76*E*(p+1)^2).
    map_bytes = 2: the column kernel streams 16-bit map entries plus one
    uint32 base per group row (4*(p+1) bytes per floor(64/(p+1)) elements)."""
    n = p + 1
    n2 = n * n
    if kind == POISSON:
        m = map_bytes * n_elem * n2
        if map_bytes == 2:
            m += 4 * n * n_elem // (64 // n)
        if geometry == "nodal":
            return 32 * ndof_nodes + m
        return 16 * ndof_nodes + 24 * n_elem * n2 + m
    if kind == AXISYM_NS:
        return 32 * ndof_nodes + 76 * n_elem * n2
    return 32 * ndof_nodes + 60 * n_elem * n2


def alg_flops(kind, n_elem, p, geometry="stored"):
    """fp64 FLOP per action: the four sum-factorised contractions (2 n^3 each)
    plus pointwise work; nodal geometry adds the four derivatives of x_phys
    and the per-node det / inverse / detJxW (15 n^2 incl. one division)."""
    n = p + 1
    if kind == POISSON:
        extra = 8 * n ** 3 + 15 * n ** 2 if geometry == "nodal" else 0
        return n_elem * (8 * n ** 3 + 7 * n ** 2 + extra)
    return n_elem * (16 * n ** 3 + (30 if kind == AXISYM_NS else 22) * n ** 2)


def cpu_baseline(p, warp, budget_s=20.0):
    """Reference path on the host: the NumPy oracle (oracle/sem_oracle.py),
    single-threaded.  (1) reference-faithful: per-element precomputed dense
    Lse (examples/poisson.py:168-193) applied with einsum('pqrs,rs') +
    np.add.at (squirmer-axisymmetric.py:286), on a 64 x 64 sample of the
    same p / warp; (2) batched sum-factorised NumPy on 256 x 256 (config 2)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
    half = gll["half_%d" % p]
    out = {}
    nodes, e2n = meshgen.structured_square(64, 64, p, warp=warp)
    prob = sem_oracle.PoissonProblem(nodes, e2n, half, batched_geometry=True)
    t0 = time.perf_counter()
    Lse = prob.element_matrices()
    t_setup = time.perf_counter() - t0
    u = np.random.default_rng(0).standard_normal(prob.ndof)
    sem_oracle.apply_element_matrices(Lse, prob.e2n, u, prob.ndof)  # warm-up
    reps, ts = 0, []
    t_start = time.perf_counter()
    while reps < 3 or (time.perf_counter() - t_start < budget_s / 3 and reps < 20):
        t0 = time.perf_counter()
        sem_oracle.apply_element_matrices(Lse, prob.e2n, u, prob.ndof)
        ts.append(time.perf_counter() - t0)
        reps += 1
    t_faith = float(np.median(ts))
    out["faithful"] = dict(ndof=prob.ndof, n_elem=e2n.shape[0], sec_per_action=t_faith,
                           dof_per_s=prob.ndof / t_faith, setup_sec=t_setup, reps=reps)
    del Lse
    nodes, e2n = meshgen.structured_square(256, 256, p, warp=warp)
    prob = sem_oracle.PoissonProblem(nodes, e2n, half, batched_geometry=True)
    u = np.random.default_rng(0).standard_normal(prob.ndof)
    prob.apply(u)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        prob.apply(u)
        ts.append(time.perf_counter() - t0)
    t_b = float(np.median(ts))
    out["batched_sumfact"] = dict(ndof=prob.ndof, n_elem=e2n.shape[0], sec_per_action=t_b,
                                  dof_per_s=prob.ndof / t_b)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--nex", type=int, default=1024, help="element columns per rank")
    ap.add_argument("--ney", type=int, default=1024)
    ap.add_argument("--warp", type=float, default=0.05)
    ap.add_argument("--op", choices=["poisson", "axisym_stokes", "axisym_ns"], default="poisson")
    ap.add_argument("--re", type=float, default=10.0, help="Reynolds number for --op axisym_ns")
    ap.add_argument("--geometry", choices=["auto", "nodal", "stored"], default="auto",
                    help="Poisson geometric factors: re-derived from x_phys per node, or "
                         "streamed; auto = nodal for p <= 8 (the library's default)")
    ap.add_argument("--kernel", choices=["auto", "column", "mfma"], default="auto",
                    help="Poisson kernel family: LDS column kernel or fp64-MFMA element kernel; "
                         "auto = the library's measured choice")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the finiteness check (timing-only diagnostic builds)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--traffic-json", default=None,
                    help="JSON with PMC-measured HBM bytes per launch (profiles/)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        dist.barrier()

    kind = {"poisson": POISSON, "axisym_stokes": AXISYM_STOKES, "axisym_ns": AXISYM_NS}[args.op]
    dpn = 1 if kind == POISSON else 2
    p = args.p
    nex_global = args.nex * world
    part = StripPartition(nex_global, args.ney, p, world, rank, dofs_per_node=dpn)
    t0 = time.time()
    if kind == POISSON:
        nodes, e2n = part.local_mesh(args.warp)
    else:
        from spectralelementmethod_amd import meshgen
        if world != 1:
            raise SystemExit("axisymmetric bench is single-GPU")
        nodes, e2n = meshgen.annulus(args.nex, args.ney, p)
    log("rank %d: mesh %d elements, %d nodes (%.1fs)" % (rank, e2n.shape[0], nodes.shape[1],
                                                          time.time() - t0))
    geometry = args.geometry if kind == POISSON else "stored"
    # interface elements first, RCCL interface sum on a side stream while the
    # interior elements run (one plain operator when there is no neighbour)
    op = OverlappedOperator(p, nodes, e2n, part.neighbors if world > 1 else {}, dpn, dev,
                            geometry=geometry, kind=kind, kernel=args.kernel)
    if kind == AXISYM_NS:
        for o in op.ops:
            o.set_reynolds(args.re)
    plan = op.plan_info()
    geometry = plan["geometry"] if kind == POISSON else "stored"  # as the library resolved it
    log("rank %d: plan %s; %d interface + %d interior elements" % (
        rank, plan, op.n_iface_elem, op.n_interior_elem))
    n_elem_local = op.n_elem
    del nodes, e2n
    log("rank %d: operator ready (%.1fs)" % (rank, time.time() - t0))

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    u = torch.randn(op.ndof, dtype=torch.float64, device=dev, generator=g)
    y = torch.empty_like(u)

    def step(ev=None):
        op.step(u, y, ev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = [a.elapsed_time(b) for a, b in events]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    kern_avg_s = float(np.mean(kern_ms)) / 1e3

    # correctness spot check of the timed output (cheap, outside the timing):
    # y must be finite and u.Ku > 0 on this rank's block
    assert args.no_check or torch.isfinite(y).all().item()

    n_nodes_local = op.ndof // dpn
    ndof_global = part.global_nodes * dpn if kind == POISSON else op.ndof
    value = ndof_global * args.steps / elapsed
    map_bytes = plan.get("map_entry_bytes", 4) if (plan["kernel"] == "column"
                                                  and kind == POISSON) else 4
    # algorithmic bytes keep SURVEY.md §8(d)'s uint32 map (the problem's
    # input); the bytes the kernel streams with a 16-bit packed map are
    # reported beside them
    B = alg_bytes(kind, n_nodes_local, n_elem_local, p, geometry)
    B_stream = alg_bytes(kind, n_nodes_local, n_elem_local, p, geometry, map_bytes)
    F = alg_flops(kind, n_elem_local, p, geometry)
    achieved = B / kern_avg_s / 1e9
    traffic = None
    traffic_src = args.traffic_json
    if (traffic_src is None and kind == POISSON and plan["kernel"] == "column"
            and (p, args.nex, args.ney) == (8, 1024, 1024)):
        # PMC measurement of this workload (separate FETCH_SIZE / WRITE_SIZE
        # passes, tools/gpu_profile.sh + tools/pmc_traffic.py)
        traffic_src = os.path.join(ROOT, "profiles", DEFAULT_TRAFFIC[geometry])
    if traffic_src and os.path.exists(traffic_src):
        with open(traffic_src) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
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
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (structured warped quad mesh, u ~ N(0,1))",
        "config": {
            "workload": "%s p=%d, %dx%d elements per GPU (%s)" % (
                args.op, p, args.nex, args.ney,
                "10^6-element north-star mesh" if (args.nex, args.ney, p) == (1024, 1024, 8)
                else "custom"),
            "p": p, "geometry": geometry, "n_elem_per_gpu": n_elem_local, "ndof_global": ndof_global,
            "ndof_per_gpu": op.ndof, "parallelism": "element column strips x%d, RCCL P2P "
                                                    "interface sum overlapped with interior "
                                                    "elements" % world if world > 1 else
            "single GPU",
            "kernel_ms_avg": kern_avg_s * 1e3, "kernel_ms_min": float(np.min(kern_ms)),
            "gflops_kernel": F / kern_avg_s / 1e9,
            "kernel_family": plan["kernel"], "map_entry_bytes": map_bytes,
            "scatter_plan": {k: plan[k] for k in ("colours", "chains_per_colour", "rounds", "zero_list",
                                                  "atomic_groups")},
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": ("k_poisson_mfma<%d>" if plan["kernel"] == "mfma" else "k_poisson_apply<%d>")
                      % (p + 1) if kind == POISSON else "k_axisym_apply<%d>" % (p + 1),
            "alg_bytes_per_launch": B, "streamed_bytes_per_launch": B_stream,
            "fp64_tflops": F / kern_avg_s / 1e12, "fp64_peak_tflops": FP64_PEAK_TFLOPS,
            "launch": "one sem_apply = %d colour launches" % plan["colours"],
            "traffic_source": os.path.relpath(traffic_src, ROOT) if traffic is not None else None,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and kind == POISSON:
        log("timing CPU baseline (NumPy oracle, 1 thread)...")
        cb = cpu_baseline(p, args.warp, args.cpu_budget)
        result["cpu_baseline"] = {
            "value": cb["faithful"]["dof_per_s"], "unit": "DOF/s", "cores": 1, "kind": "port",
            "sample": "reference-faithful per-element Lse einsum + np.add.at, 64x64 p=%d warped "
                      "(%d DOF), median of %d; host os.cpu_count()=%d" % (
                          p, cb["faithful"]["ndof"], cb["faithful"]["reps"], os.cpu_count()),
            "batched_sumfact_dof_per_s": cb["batched_sumfact"]["dof_per_s"],
            "batched_sumfact_sample": "256x256 p=%d (%d DOF)" % (p, cb["batched_sumfact"]["ndof"]),
            "faithful_setup_sec_per_elem": cb["faithful"]["setup_sec"] / cb["faithful"]["n_elem"],
        }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
