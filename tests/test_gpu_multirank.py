"""GPU tests of the multi-GPU path (csrc/sem_dd.hip through the C ABI) and of
the device-resident assembled solve.

Several ranks run on ONE device here (the box has one GPU; RCCL refuses two
ranks on one GPU), so the interface sum goes through the caller-supplied
transport (TorchTransport over gloo, staged through host memory).  Every
other part of the step is the production path: interface elements on the
side stream over the compact numbering, pack, exchange, unpack, interior
elements on the caller's stream, final add -- and the PCG loop of
sem_dd_pcg_solve with its global dot products.  The native RCCL transport
differs only in the two transport calls (ncclSend/ncclRecv, ncclAllReduce).

Tolerances: the multi-rank action equals the single-GPU action to 1e-13
relative (only the summation order of the few shared DOFs differs); the
solve matches the oracle's direct solve to 1e-10 (the north-star bar)."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _manufactured(nodes, dev):
    x = torch.from_numpy(nodes[0]).to(dev)
    y = torch.from_numpy(nodes[1]).to(dev)
    xs = torch.sin(0.5 * np.pi * x) * torch.cos(0.5 * np.pi * y) + x * y
    on = (torch.abs(x.abs() - 1) < 1e-9) | (torch.abs(y.abs() - 1) < 1e-9)
    return xs, on


def _rank_worker(rank, world, port, mode, p, nex, ney, q):
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import (GenericPartition, OverlappedOperator,
                                                           StripPartition)
        from spectralelementmethod_amd.operators import SEMOperator
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if mode == "sfc":  # irregular-valence mesh, Morton-curve partition
            from spectralelementmethod_amd.distributed import partition_elements
            gnodes, ge2n = meshgen.quads_from_triangles(nex, ney, p, seed=4)
        else:
            gnodes, ge2n = meshgen.structured_square(nex, ney, p, warp=0.05)
        if mode == "strip":
            part = StripPartition(nex, ney, p, world, rank)
            nodes, e2n = part.local_mesh(0.05)
        elif mode == "sfc":
            part = GenericPartition(ge2n, partition_elements(ge2n, gnodes, world, "sfc"), world,
                                    rank)
            e2n, nodes = part.e2n_local, gnodes[:, part.l2g]
        else:
            elem_rank = np.random.default_rng(8).integers(0, world, size=ge2n.shape[0])
            part = GenericPartition(ge2n, elem_rank, world, rank)
            e2n, nodes = part.e2n_local, gnodes[:, part.l2g]
        l2g = torch.from_numpy(part.local_to_global().astype(np.int64)).to(dev)
        op = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, dev, owned=part.owned,
                                transport="torch", world=world, rank=rank)
        full = SEMOperator(p, ge2n, gnodes, device=dev)
        g = torch.Generator(device=dev).manual_seed(21)
        u_glob = torch.randn(full.ndof, dtype=torch.float64, device=dev, generator=g)
        y_ref = full.apply(u_glob)[l2g]
        u = u_glob[l2g].contiguous()
        y = torch.full_like(u, 7.0)
        errs = []
        for _ in range(3):  # repeated steps reuse the buffers and the side stream
            op.step(u, y)
            errs.append(((y - y_ref).norm() / y_ref.norm()).item())
        d = op.diag()
        d_ref = full.diag()[l2g]
        err_diag = ((d - d_ref).norm() / d_ref.norm()).item()
        # device-resident PCG over the decomposition vs the single-GPU solve
        xs_g, on_g = _manufactured(gnodes, dev)
        b = full.apply(xs_g)
        x_single = torch.where(on_g, xs_g, torch.zeros_like(xs_g))
        x_single, its1, _ = full.pcg_solve(b, x_single, on_g, rtol=1e-12)
        xs, on = xs_g[l2g], on_g[l2g]
        x = torch.where(on, xs, torch.zeros_like(xs))
        x, its, rel = op.pcg_solve(b[l2g].contiguous(), x, on, rtol=1e-12, check_every=4)
        err_pcg = ((x - x_single[l2g]).norm() / x_single[l2g].norm()).item()
        err_exact = ((x - xs).norm() / xs.norm()).item()
        q.put((rank, max(errs), err_diag, err_pcg, err_exact, its, its1, op.transport,
               op.n_iface_elem, op.n_interior_elem))
        op.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,p,nex,ney", [(2, "strip", 8, 12, 6), (3, "strip", 4, 10, 5),
                                                  (3, "generic", 3, 7, 6),
                                                  (4, "sfc", 4, 6, 5),
                                                  # constant-D kernels on both contexts
                                                  (2, "strip", 12, 8, 6)])
def test_overlapped_operator_ranks_on_one_gpu(gpu, world, mode, p, nex, ney):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, mode, p, nex, ney, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        res = [q.get(timeout=150) for _ in range(world)]
    finally:
        for pr in procs:
            pr.join(timeout=60)
    for pr in procs:
        assert pr.exitcode == 0
    its_all = set()
    for rank, err, err_d, err_pcg, err_x, its, its1, tr, n_if, n_in in res:
        assert tr == "torch-host"
        assert err < 1e-13, (rank, err)
        assert err_d < 1e-13, (rank, err_d)
        assert err_pcg < 1e-9 and err_x < 1e-9, (rank, err_pcg, err_x)
        assert n_if > 0
        its_all.add(its)
    assert len(its_all) == 1  # every rank ran the same iterations (global dots)


def test_single_rank_overlapped_is_plain_operator(gpu):
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import OverlappedOperator
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(9, 7, 5, warp=0.05)
    op = OverlappedOperator(5, nodes, e2n, {}, 1, gpu, world=1, rank=0)
    full = SEMOperator(5, e2n, nodes, device=gpu)
    u = torch.randn(full.ndof, dtype=torch.float64, device=gpu,
                    generator=torch.Generator(device=gpu).manual_seed(3))
    # (this small mesh has atomic-fallback groups: equal up to summation order)
    a, b = op.apply(u), full.apply(u)
    assert (a - b).norm().item() <= 1e-14 * b.norm().item()
    assert op.dd is None and op.transport == "none"


@pytest.mark.parametrize("p,nex", [(2, 256), (4, 64)])
def test_pcg_vs_oracle_direct_solve(gpu, gll, p, nex):
    """Device-resident PCG (sem_pcg_solve) vs the oracle's assembled direct
    solve (what DOFManagerSC.solve computes, sem/discrete.py:502-528) of the
    restated examples/poisson.py problem (f = 1: rhs = assembled detJxW,
    u = 0.2((x+1)+(y+1)) on the left and bottom edges): 256 x 256 p = 2 is
    65,536 elements, 263,169 DOF.  Tolerance 1e-10 relative L2."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(nex, nex, p, warp=0.05)
    prob = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True)
    Lse = sem_oracle.poisson_Lse_batched(prob.invJ, prob.detJxW, prob.D)
    K = sem_oracle.assemble_poisson_matrix(Lse, prob.e2n, prob.ndof)
    rhs = np.bincount(prob.e2n.ravel(), weights=prob.detJxW.ravel(), minlength=prob.ndof)
    ebc, vals = meshgen.square_dirichlet_left_bottom(nodes)
    ref = sem_oracle.poisson_solve_direct(K, rhs, ebc, vals)
    op = SEMOperator(p, e2n, nodes, device=gpu)
    # rhs assembled on the device from the device geometry (sem_assemble)
    JxW = op.geometry_fields()["detJxW"]
    b = op.assemble(JxW)
    assert rel_l2(b.cpu().numpy(), rhs) < 1e-13
    x = torch.from_numpy(np.where(ebc, vals, 0.0)).to(gpu)
    x, its, rel = op.pcg_solve(b, x, ebc, rtol=1e-13, max_iter=50000)
    assert rel <= 1e-13
    assert rel_l2(x.cpu().numpy(), ref) < 1e-10, (its, rel_l2(x.cpu().numpy(), ref))


def test_pcg_fixed_iterations_and_errors(gpu):
    """rtol = 0 runs exactly max_iter iterations; a non-converged solve
    raises ValueError (SEM_E_INVALID) like the reference's solver failure."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(16, 16, 4, warp=0.05)
    op = SEMOperator(4, e2n, nodes, device=gpu)
    xs, on = _manufactured(nodes, gpu)
    b = op.apply(xs)
    x = torch.where(on, xs, torch.zeros_like(xs))
    _, its, rel = op.pcg_solve(b, x.clone(), on, rtol=0.0, max_iter=37)
    assert its == 37 and 0 < rel < 1
    with pytest.raises(ValueError):
        op.pcg_solve(b, x.clone(), on, rtol=1e-14, max_iter=5)
    x, its, rel = op.pcg_solve(b, x, on, rtol=1e-12)
    assert rel <= 1e-12 and ((x - xs).norm() / xs.norm()).item() < 1e-9


@pytest.mark.parametrize("iters", [1, 36, 37])
def test_pcg_x_pairs_bitwise(gpu, monkeypatch, iters):
    """x updated every second iteration (default: x += a' p' + a p as two
    fused multiply-adds in order, a flush after an odd count) is bitwise the
    x of the every-iteration update (SEM_PCG_X_EVERY=1), read per solve."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(16, 16, 4, warp=0.05)
    op = SEMOperator(4, e2n, nodes, device=gpu)
    xs, on = _manufactured(nodes, gpu)
    b = op.apply(xs)
    x0 = torch.where(on, xs, torch.zeros_like(xs))
    out = {}
    for every in ("1", "0"):
        monkeypatch.setenv("SEM_PCG_X_EVERY", every)
        out[every] = op.pcg_solve(b, x0.clone(), on, rtol=0.0, max_iter=iters)
    assert out["1"][1] == out["0"][1] == iters
    assert torch.equal(out["1"][0], out["0"][0])
    assert out["1"][2] == out["0"][2]
    # and a converged solve with the default
    monkeypatch.delenv("SEM_PCG_X_EVERY")
    x, its, rel = op.pcg_solve(b, x0.clone(), on, rtol=1e-12)
    assert rel <= 1e-12 and ((x - xs).norm() / xs.norm()).item() < 1e-9


def _native_rccl_worker(q):
    """One rank through the bench's process-group setup and the native RCCL
    transport of sem_dd (communicator init, ncclAllReduce in the PCG; no peer
    to send to at world size 1)."""
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                      WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("cpu:gloo,cuda:nccl", device_id=dev)  # as bench.py
    try:
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
        from spectralelementmethod_amd.operators import SEMOperator
        dist.barrier()
        part = StripPartition(10, 6, 4, 1, 0)
        nodes, e2n = part.local_mesh(0.05)
        op = OverlappedOperator(4, nodes, e2n, {}, 1, dev, owned=part.owned, transport="rccl",
                                world=1, rank=0, decompose=True)
        full = SEMOperator(4, e2n, nodes, device=dev)
        u = torch.randn(full.ndof, dtype=torch.float64, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(2))
        err = ((op.apply(u) - full.apply(u)).norm() / full.apply(u).norm()).item()
        xs, on = _manufactured(nodes, dev)
        b = full.apply(xs)
        x1, its1, _ = full.pcg_solve(b, torch.where(on, xs, torch.zeros_like(xs)), on, rtol=1e-12)
        x2, its2, _ = op.pcg_solve(b, torch.where(on, xs, torch.zeros_like(xs)), on, rtol=1e-12)
        t = torch.tensor([1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)       # bench's timing reduction (gloo)
        got = [None]
        dist.all_gather_object(got, 3.5)
        q.put((op.transport, err, ((x2 - x1).norm() / x1.norm()).item(), its1, its2, got[0]))
        op.close()
    finally:
        dist.destroy_process_group()


def test_native_rccl_transport_single_rank(gpu):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_native_rccl_worker, args=(q,))
    pr.start()
    try:
        tr, err, err_pcg, its1, its2, got = q.get(timeout=150)
    finally:
        pr.join(timeout=60)
    assert pr.exitcode == 0
    assert tr == "rccl"
    assert err < 1e-14 and err_pcg < 1e-12 and its1 == its2 and got == 3.5


def _axisym_worker(rank, world, port, q):
    """The decomposition with two DOFs per node (interleaved psi, omega):
    the axisymmetric Stokes block over theta-strips of a curved annulus."""
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import GenericPartition, OverlappedOperator
        from spectralelementmethod_amd.operators import AXISYM_STOKES, SEMOperator
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        p, nth, nr = 6, 9, 5
        gnodes, ge2n = meshgen.annulus(nth, nr, p)
        elem_rank = (np.arange(ge2n.shape[0]) * world) // ge2n.shape[0]  # theta strips
        part = GenericPartition(ge2n, elem_rank, world, rank, dofs_per_node=2)
        nodes, e2n = gnodes[:, part.l2g], part.e2n_local
        op = OverlappedOperator(p, nodes, e2n, part.neighbors, 2, dev, owned=part.owned,
                                kind=AXISYM_STOKES, transport="torch", world=world, rank=rank)
        full = SEMOperator(p, ge2n, gnodes, dofs_per_node=2, device=dev)
        g = torch.Generator(device=dev).manual_seed(9)
        s = torch.randn(full.ndof, dtype=torch.float64, device=dev, generator=g)
        ref = full.apply(s, kind="axisym_stokes")
        dof = torch.from_numpy((part.l2g[:, None] * 2 + np.arange(2)).ravel()).to(dev)
        y = op.apply(s[dof].contiguous())
        q.put((rank, ((y - ref[dof]).norm() / ref[dof].norm()).item(), op.exchange_bytes))
        op.close()
    finally:
        dist.destroy_process_group()


def test_overlapped_axisym_two_dofs_per_node(gpu):
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_axisym_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        res = [q.get(timeout=150) for _ in range(world)]
    finally:
        for pr in procs:
            pr.join(timeout=60)
    for pr in procs:
        assert pr.exitcode == 0
    for rank, err, nbytes in res:
        assert err < 1e-13, (rank, err)
        assert nbytes > 0


def _graph_worker(rank, world, port, q):
    """One rank's step eager and as captured graphs (sem_dd_set_graphs):
    bitwise equal actions (same kernels, same order), equal PCG solves, and
    the host-enqueue time per step of both."""
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        p = 8
        part = StripPartition(32, 24, p, world, rank)
        nodes, e2n = part.local_mesh(0.05)
        op = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, dev, owned=part.owned,
                                transport="torch", world=world, rank=rank)
        g = torch.Generator(device=dev).manual_seed(5 + rank)
        u = torch.randn(op.ndof, dtype=torch.float64, device=dev, generator=g)
        out, enq = {}, {}
        for mode in (False, True):
            op.set_graphs(mode)
            y = torch.full_like(u, 3.0)
            op.step(u, y)  # (re)capture
            torch.cuda.synchronize()
            dist.barrier()
            i0 = op.dd_info()
            for _ in range(10):
                op.step(u, y)
            i1 = op.dd_info()
            # host enqueue time of the library's own launches per step (the
            # gloo transport, which waits for the device, left out)
            enq[mode] = ((i1["host_ns"] - i0["host_ns"]) -
                         (i1["host_ns_transport"] - i0["host_ns_transport"])) / 10 * 1e-9
            torch.cuda.synchronize()
            out[mode] = y.clone()
        info = op.dd_info()
        xs, on = _manufactured(nodes, dev)
        b = op.apply(xs)
        sol = {}
        for mode in (False, True):
            op.set_graphs(mode)
            x = torch.where(on, xs, torch.zeros_like(xs))
            x, its, rel = op.pcg_solve(b, x, on, rtol=1e-11)
            sol[mode] = (x, its)
        # the Jacobi diagonal is summed with atomics (setup, sem_diag): the two
        # solves differ at rounding level, not in their iteration count
        dx = ((sol[False][0] - sol[True][0]).norm() / sol[True][0].norm()).item()
        # a context state change between two captured steps
        # (new coordinates, geometry switched to stored factors) must
        # re-capture; a stale graph would replay the old x_phys kernel
        from spectralelementmethod_amd import _lib
        op.set_graphs(True)
        y_g = torch.zeros_like(u)
        op.step(u, y_g)  # captured on the current state
        for o in op.ops:
            o.nodes[0].mul_(1.5)
            _lib.check(o._lib.sem_set_geom_mode(o._ctx, _lib.GEOM_STORED))
            o.compute_geometry()
        op.step(u, y_g)
        op.set_graphs(False)
        y_e = torch.zeros_like(u)
        op.step(u, y_e)
        torch.cuda.synchronize()
        recapture = (torch.equal(y_g, y_e), not torch.allclose(y_e, out[False]),
                     op.dd_info()["captures"])
        q.put((rank, torch.equal(out[False], out[True]), info, dx, sol[False][1], sol[True][1],
               enq[False] * 1e6, enq[True] * 1e6, recapture))
        op.close()
    finally:
        dist.destroy_process_group()


def test_captured_step_equals_eager(gpu):
    """sem_dd_apply through its captured graphs (opt-in) equals the
    eager enqueue bit for bit on 2 ranks of one device (torch transport
    between the graph segments); the PCG over the decomposition agrees to
    rounding (its Jacobi diagonal is an atomic sum)."""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        res = [q.get(timeout=150) for _ in range(world)]
    finally:
        for pr in procs:
            pr.join(timeout=60)
    for pr in procs:
        assert pr.exitcode == 0
    for rank, same, info, dx, its0, its1, us_eager, us_graph, recap in res:
        assert same, rank
        assert recap[0] and recap[1], (rank, recap)  # re-captured after the state change
        assert recap[2] > info["captures"], (rank, recap, info)
        assert info["graphs"] and info["replays"] >= 10 and info["captures"] >= 1, info
        assert dx < 1e-12 and abs(its0 - its1) <= 16, (rank, dx, its0, its1)
        print("rank %d host enqueue per step (transport call excluded): eager %.1f us, "
              "graphs %.1f us" % (rank, us_eager, us_graph))


def _remap_worker(rank, world, port, q):
    """sem_set_map on both contexts of a live decomposition
    rebuilds its finish tables (freed once, reallocated); the next step must
    equal a freshly built decomposition bit for bit, eager and captured."""
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spectralelementmethod_amd import _lib
        from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        p = 8
        part = StripPartition(24, 16, p, world, rank)
        nodes, e2n = part.local_mesh(0.05)
        kw = dict(owned=part.owned, transport="torch", world=world, rank=rank)
        op = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, dev, **kw)
        g = torch.Generator(device=dev).manual_seed(11 + rank)
        u = torch.randn(op.ndof, dtype=torch.float64, device=dev, generator=g)
        y = torch.zeros_like(u)
        op.step(u, y)
        for o in op.ops:  # the same map again: a new plan, new finish tables
            _lib.check(o._lib.sem_set_map(o._ctx, _lib.tptr(o.e2n), _lib.stream_ptr()))
            o.compute_geometry()
        ys = {}
        for mode in (False, True):
            op.set_graphs(mode)
            yy = torch.full_like(u, 5.0)
            for _ in range(3):
                op.step(u, yy)
            torch.cuda.synchronize()
            ys[mode] = yy.clone()
        op.set_graphs(False)
        fresh = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, dev, **kw)
        y_ref = torch.zeros_like(u)
        fresh.step(u, y_ref)
        torch.cuda.synchronize()
        q.put((rank, torch.equal(ys[False], y_ref), torch.equal(ys[True], y_ref)))
        fresh.close()
        op.close()
    finally:
        dist.destroy_process_group()


def test_remap_rebuilds_finish_bitwise(gpu):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_remap_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        res = [q.get(timeout=150) for _ in range(world)]
    finally:
        for pr in procs:
            pr.join(timeout=60)
    for pr in procs:
        assert pr.exitcode == 0
    for rank, eager_ok, graph_ok in res:
        assert eager_ok and graph_ok, (rank, eager_ok, graph_ok)
