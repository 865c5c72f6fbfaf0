"""World-size-2 (and 3) tests of the multi-GPU path's host logic on CPU with the
gloo backend: strip / generic partitions, the interface exchange protocol and
the assembled global action.  The rank-local operator is a CPU stand-in built
from the oracle (the real one is SEMOperator on a GPU); everything else is
the product code in spectralelementmethod_amd.distributed."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class OracleLocalOp(object):
    """CPU stand-in for SEMOperator.apply on the rank-local mesh."""

    def __init__(self, nodes, e2n, half):
        import sem_oracle
        self.prob = sem_oracle.PoissonProblem(nodes, e2n, half)
        self.device = torch.device("cpu")

    def apply(self, u, out=None, kind=0):
        y = torch.from_numpy(self.prob.apply(u.numpy()))
        if out is not None:
            out.copy_(y)
            return out
        return y


def _worker(rank, world, port, mode, q):
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sem_oracle
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import (DistributedOperator, GenericPartition,
                                                           StripPartition)
        gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
        p, nex, ney = 4, 7, 3
        half = gll["half_%d" % p]
        gnodes, ge2n = meshgen.structured_square(nex, ney, p, warp=0.05)
        u_glob = np.random.default_rng(11).standard_normal(gnodes.shape[1])
        y_glob = sem_oracle.PoissonProblem(gnodes, ge2n, half).apply(u_glob)
        if mode == "strip":
            part = StripPartition(nex, ney, p, world, rank)
            nodes, e2n = part.local_mesh(0.05)
        else:
            rng = np.random.default_rng(3)
            elem_rank = rng.integers(0, world, size=ge2n.shape[0])
            part = GenericPartition(ge2n, elem_rank, world, rank)
            e2n = part.e2n_local
            nodes = gnodes[:, part.l2g]
        l2g = part.local_to_global()
        op = DistributedOperator(OracleLocalOp(nodes, e2n, half), part)
        u = torch.from_numpy(u_glob[l2g].copy())
        y = op.apply(u)
        err = np.abs(y.numpy() - y_glob[l2g]).max() / np.abs(y_glob).max()
        # owned-entry dot product reduces to the global one
        d = op.global_dot(u, y)
        q.put((rank, err, d, float(np.dot(u_glob, y_glob)), op.xchg.bytes_per_exchange))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "strip"), (3, "strip"), (2, "generic"),
                                        (3, "generic")])
def test_distributed_action_gloo(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, err, d, d_ref, nbytes in res:
        assert err < 1e-14, (rank, err)
        assert abs(d - d_ref) <= 1e-12 * abs(d_ref)
        assert nbytes > 0


def test_strip_partition_bookkeeping():
    from spectralelementmethod_amd.distributed import StripPartition
    nex, ney, p, world = 10, 4, 8, 4
    parts = [StripPartition(nex, ney, p, world, r) for r in range(world)]
    assert sum(pt.n_elem for pt in parts) == nex * ney
    owned = sum(int(pt.owned.sum()) for pt in parts)
    assert owned == parts[0].global_nodes
    for a, b in zip(parts[:-1], parts[1:]):
        # the right line of a == the left line of b in global numbering
        ga = a.local_to_global()[a.neighbors[b.rank]]
        gb = b.local_to_global()[b.neighbors[a.rank]]
        assert np.array_equal(ga, gb)
    with pytest.raises(ValueError):
        StripPartition(3, 4, 2, 4, 0)


def _dd_worker(rank, world, port, mode, q):
    """The overlapped multi-GPU step's protocol (DDPlan + the sequence
    sem_dd_apply enqueues, dd_step_reference) with oracle stand-ins for the
    two device operators, under gloo."""
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sem_oracle
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import (DDPlan, GenericPartition,
                                                           StripPartition, dd_step_reference,
                                                           torch_p2p_exchange)
        gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
        p, nex, ney = 3, 9, 4
        half = gll["half_%d" % p]
        gnodes, ge2n = meshgen.structured_square(nex, ney, p, warp=0.05)
        u_glob = np.random.default_rng(5).standard_normal(gnodes.shape[1])
        y_glob = sem_oracle.PoissonProblem(gnodes, ge2n, half).apply(u_glob)
        if mode == "strip":
            part = StripPartition(nex, ney, p, world, rank)
            nodes, e2n = part.local_mesh(0.05)
        else:
            rng = np.random.default_rng(8)
            elem_rank = rng.integers(0, world, size=ge2n.shape[0])
            part = GenericPartition(ge2n, elem_rank, world, rank)
            e2n, nodes = part.e2n_local, gnodes[:, part.l2g]
        plan = DDPlan(e2n, nodes.shape[1], part.neighbors, 1, part.owned)
        # interface elements over the compact node numbering, interior over the local one
        op_i = sem_oracle.PoissonProblem(nodes[:, plan.iface_nodes], plan.e2n_iface, half) \
            if plan.iface_elems.size else None
        op_b = sem_oracle.PoissonProblem(nodes, e2n[plan.interior_elems], half) \
            if plan.interior_elems.size else None
        l2g = part.local_to_global()
        u = torch.from_numpy(u_glob[l2g].copy())
        y = dd_step_reference(
            plan, u, lambda uc: torch.from_numpy(op_i.apply(uc.numpy())),
            lambda ul: torch.from_numpy(op_b.apply(ul.numpy())),
            lambda send, peers, counts: torch_p2p_exchange(send, peers, counts))
        err = np.abs(y.numpy() - y_glob[l2g]).max() / np.abs(y_glob).max()
        own = torch.from_numpy(np.asarray(plan.not_owned == 0))
        d = torch.sum(u[own] * y[own]).reshape(1)
        dist.all_reduce(d)
        q.put((rank, err, d.item(), float(np.dot(u_glob, y_glob)),
               plan.exchanged_per_direction, len(plan.peers)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "strip"), (3, "strip"), (2, "generic"),
                                        (4, "generic")])
def test_overlapped_protocol_gloo(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dd_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, err, d, d_ref, nx, npeer in res:
        assert err < 1e-14, (rank, err)
        assert abs(d - d_ref) <= 1e-12 * abs(d_ref)
        assert nx > 0 and npeer >= 1


def test_ddplan_bookkeeping():
    """DDPlan (host side of sem_dd): compact interface numbering, peer lists
    in compact DOFs that map back to the partition's shared nodes, owned DOFs,
    and dpn = 2 interleaving."""
    from spectralelementmethod_amd.distributed import DDPlan, StripPartition
    for dpn in (1, 2):
        for rank in range(3):
            part = StripPartition(12, 4, 3, 3, rank, dofs_per_node=dpn)
            nodes, e2n = part.local_mesh(0.05)
            pl = DDPlan(e2n, part.n_nodes, part.neighbors, dpn, part.owned)
            assert pl.iface_elems.size == len(part.neighbors) * part.ney
            assert np.union1d(pl.iface_elems, pl.interior_elems).size == e2n.shape[0]
            # compact map reproduces the local map of the interface elements
            assert np.array_equal(pl.iface_nodes[pl.e2n_iface], e2n[pl.iface_elems])
            assert pl.iface_dofs.size == dpn * pl.iface_nodes.size
            off = np.concatenate([[0], np.cumsum(pl.peer_counts)])
            for k, r in enumerate(pl.peers):
                cd = pl.peer_dofs[off[k]:off[k + 1]].astype(np.int64)
                ld = pl.iface_dofs[cd].astype(np.int64)
                nodes_back = ld[::dpn] // dpn
                assert np.array_equal(nodes_back, part.neighbors[r])
                assert np.array_equal(ld % dpn, np.tile(np.arange(dpn), part.Ny))
            # shared nodes are touched by interface elements only
            iface = np.concatenate(list(part.neighbors.values()))
            assert not np.isin(iface, e2n[pl.interior_elems]).any()
            assert pl.not_owned.sum() == (dpn * part.Ny if rank > 0 else 0)
    with pytest.raises(ValueError):  # a shared node no element of the rank references
        DDPlan(e2n, part.n_nodes + 1, {0: np.array([0, part.n_nodes])}, 1)


def test_split_interface_elements():
    """Interface / interior element split and node states of the overlapped
    multi-GPU operator (host logic)."""
    from spectralelementmethod_amd import _lib
    from spectralelementmethod_amd.distributed import StripPartition, split_interface_elements
    for rank in range(3):
        part = StripPartition(12, 4, 3, 3, rank)
        nodes, e2n = part.local_mesh(0.05)
        ie, be, st_i, st_b = split_interface_elements(e2n, part.neighbors)
        assert np.union1d(ie, be).size == e2n.shape[0] and np.intersect1d(ie, be).size == 0
        n_nb = len(part.neighbors)
        assert ie.size == n_nb * part.ney  # one element column per interface
        iface = np.concatenate(list(part.neighbors.values()))
        # interface nodes belong to interface elements only
        assert not np.isin(iface, e2n[be]).any()
        in_i = np.zeros(part.n_nodes, bool)
        in_i[e2n[ie].ravel()] = True
        assert (st_b[in_i] == _lib.NODE_PRIOR).all()
        only_b = np.zeros(part.n_nodes, bool)
        only_b[e2n[be].ravel()] = True
        only_b &= ~in_i
        assert (st_i[only_b] == _lib.NODE_OTHER).all() and (st_b[only_b] == 0).all()
        assert (st_i[in_i] == 0).all()


@pytest.mark.parametrize("method", ["sfc", "rcm"])
def test_partition_elements(method):
    """SFC / RCM element -> rank assignment: balanced pieces, and far fewer
    shared nodes than a random assignment on an irregular-valence mesh."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import GenericPartition, partition_elements
    nodes, e2n = meshgen.quads_from_triangles(12, 10, 3, seed=2)
    world = 4
    er = partition_elements(e2n, nodes, world, method)
    sizes = np.bincount(er, minlength=world)
    assert sizes.max() - sizes.min() <= 1

    def shared(elem_rank):
        return sum(int(sum(v.size for v in GenericPartition(e2n, elem_rank, world, r)
                           .neighbors.values())) for r in range(world))
    rnd = np.random.default_rng(0).integers(0, world, e2n.shape[0])
    assert shared(er) < 0.25 * shared(rnd)
    with pytest.raises(ValueError):
        partition_elements(e2n, nodes, world, "metis")


def _dd_worker_unstructured(rank, world, port, q):
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sem_oracle
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import (DDPlan, GenericPartition,
                                                           dd_step_reference, partition_elements,
                                                           torch_p2p_exchange)
        gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
        p = 4
        half = gll["half_%d" % p]
        gnodes, ge2n = meshgen.quads_from_triangles(7, 6, p, seed=1)
        u_glob = np.random.default_rng(2).standard_normal(gnodes.shape[1])
        y_glob = sem_oracle.PoissonProblem(gnodes, ge2n, half).apply(u_glob)
        part = GenericPartition(ge2n, partition_elements(ge2n, gnodes, world, "sfc"), world, rank)
        e2n, nodes = part.e2n_local, gnodes[:, part.l2g]
        plan = DDPlan(e2n, nodes.shape[1], part.neighbors, 1, part.owned)
        op_i = sem_oracle.PoissonProblem(nodes[:, plan.iface_nodes], plan.e2n_iface, half)
        op_b = sem_oracle.PoissonProblem(nodes, e2n[plan.interior_elems], half) \
            if plan.interior_elems.size else None
        u = torch.from_numpy(u_glob[part.l2g].copy())
        y = dd_step_reference(
            plan, u, lambda uc: torch.from_numpy(op_i.apply(uc.numpy())),
            lambda ul: torch.from_numpy(op_b.apply(ul.numpy())),
            lambda send, peers, counts: torch_p2p_exchange(send, peers, counts))
        err = np.abs(y.numpy() - y_glob[part.l2g]).max() / np.abs(y_glob).max()
        q.put((rank, err, len(plan.peers)))
    finally:
        dist.destroy_process_group()


def test_overlapped_protocol_unstructured_sfc_gloo():
    """The multi-GPU protocol on an irregular-valence mesh partitioned along
    the Morton curve (vertices shared by three or more ranks)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dd_worker_unstructured, args=(r, world, port, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, err, npeer in res:
        assert err < 1e-14, (rank, err)
        assert npeer >= 1


# ---------------------------------------------------------------- hexahedra (row N3)
def test_slab_partition_bookkeeping():
    """SlabPartition (hexahedral slabs along x): element and owned-node
    counts add up to the cube, neighbouring slabs agree on their shared face
    in global numbering, and every slab's local mesh is the global cube's
    nodes and element map at its global ids, bit for bit."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import SlabPartition
    nex, ney, nez, p, world = 7, 3, 2, 3, 3
    gnodes, ge2n = meshgen.structured_cube(nex, ney, nez, p, warp=0.05)
    parts = [SlabPartition(nex, ney, nez, p, world, r) for r in range(world)]
    assert sum(pt.n_elem for pt in parts) == nex * ney * nez
    assert sum(int(pt.owned.sum()) for pt in parts) == parts[0].global_nodes == gnodes.shape[1]
    e0 = 0
    for pt in parts:
        nodes, e2n = pt.local_mesh(0.05)
        l2g = pt.local_to_global()
        assert np.array_equal(nodes, gnodes[:, l2g])  # bitwise, incl. the warp
        ge = ge2n[e0:e0 + pt.n_elem].astype(np.int64)
        assert np.array_equal(l2g[e2n.astype(np.int64)], ge)
        e0 += pt.n_elem
    for a, b in zip(parts[:-1], parts[1:]):
        ga = a.local_to_global()[a.neighbors[b.rank]]
        gb = b.local_to_global()[b.neighbors[a.rank]]
        assert np.array_equal(ga, gb) and ga.size == a.Ny * a.Nz
    with pytest.raises(ValueError):
        SlabPartition(2, 3, 3, 2, 4, 0)


def test_block_partition_bookkeeping():
    """BlockPartition (hexahedral boxes on a rank grid): element and
    owned-node counts add up to the cube, every pair of ranks agrees on its
    shared nodes (faces, edges, corners) in global numbering, and every box's
    local mesh is the global cube's nodes and element map at its global ids,
    bit for bit."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import BlockPartition, block_grid
    assert block_grid(8) == (2, 2, 2) and block_grid(4) == (2, 2, 1)
    assert block_grid(2) == (2, 1, 1) and block_grid(1) == (1, 1, 1)
    assert block_grid(12) == (3, 2, 2)
    nex, ney, nez, p = 5, 4, 3, 2
    gnodes, ge2n = meshgen.structured_cube(nex, ney, nez, p, warp=0.05)
    gpos = {tuple(r): i for i, r in enumerate(ge2n.reshape(ge2n.shape[0], -1)[:, [0, -1]])}
    for grid in [(2, 2, 2), (3, 2, 1), (1, 1, 3), (2, 1, 1)]:
        world = int(np.prod(grid))
        parts = [BlockPartition(nex, ney, nez, p, grid, r) for r in range(world)]
        assert sum(pt.n_elem for pt in parts) == nex * ney * nez
        assert sum(int(pt.owned.sum()) for pt in parts) == gnodes.shape[1]
        seen = set()
        for pt in parts:
            nodes, e2n = pt.local_mesh(0.05)
            l2g = pt.local_to_global()
            assert np.array_equal(nodes, gnodes[:, l2g])  # bitwise, incl. the warp
            ge = l2g[e2n.astype(np.int64)].reshape(e2n.shape[0], -1)
            for row in ge:  # every local element is a global element, once
                k = gpos[(row[0], row[-1])]
                assert np.array_equal(row, ge2n[k].ravel()) and k not in seen
                seen.add(k)
            for q, loc in pt.neighbors.items():
                ga = l2g[loc]
                gb = parts[q].local_to_global()[parts[q].neighbors[pt.rank]]
                assert np.array_equal(ga, gb) and np.all(np.diff(ga) > 0)
            # a node is shared with exactly the ranks whose node boxes hold it
            cnt = np.zeros(pt.n_nodes, dtype=np.int64)
            for loc in pt.neighbors.values():
                cnt[loc] += 1
            holders = np.zeros(gnodes.shape[1], dtype=np.int64)
            for o in parts:
                holders[o.local_to_global()] += 1
            assert np.array_equal(cnt + 1, holders[l2g])
        assert len(seen) == ge2n.shape[0]
    assert len(BlockPartition(nex, ney, nez, p, (2, 2, 2), 0).neighbors) == 7  # faces+edges+corner
    with pytest.raises(ValueError):
        BlockPartition(1, 3, 3, 2, (2, 1, 1), 0)


def _dd_worker_hex(rank, world, port, mode, q):
    """The overlapped step's protocol (DDPlan + dd_step_reference) on a
    hexahedral slab / generic partition, hexahedral oracle stand-ins for the
    two device operators, under gloo."""
    import sys
    for pth in (ROOT, os.path.join(ROOT, "oracle")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sem_oracle
        from spectralelementmethod_amd import meshgen
        from spectralelementmethod_amd.distributed import (BlockPartition, DDPlan,
                                                           GenericPartition, SlabPartition,
                                                           block_grid, dd_step_reference,
                                                           partition_elements, torch_p2p_exchange)
        gll = np.load(os.path.join(ROOT, "tests", "golden", "gll.npz"))
        p, nex, ney, nez = 3, 5, 2, 2
        half = gll["half_%d" % p]
        gnodes, ge2n = meshgen.structured_cube(nex, ney, nez, p, warp=0.05)
        u_glob = np.random.default_rng(6).standard_normal(gnodes.shape[1])
        y_glob = sem_oracle.HexPoissonProblem(gnodes, ge2n, half).apply(u_glob)
        if mode == "slab":
            part = SlabPartition(nex, ney, nez, p, world, rank)
            nodes, e2n = part.local_mesh(0.05)
        elif mode == "block":
            part = BlockPartition(nex, ney, nez, p, block_grid(world), rank)
            nodes, e2n = part.local_mesh(0.05)
        else:
            part = GenericPartition(ge2n, partition_elements(ge2n, gnodes, world, "sfc"), world,
                                    rank)
            e2n, nodes = part.e2n_local, gnodes[:, part.l2g]
        plan = DDPlan(e2n, nodes.shape[1], part.neighbors, 1, part.owned)
        op_i = sem_oracle.HexPoissonProblem(nodes[:, plan.iface_nodes], plan.e2n_iface, half)
        op_b = sem_oracle.HexPoissonProblem(nodes, e2n[plan.interior_elems], half) \
            if plan.interior_elems.size else None
        l2g = part.local_to_global()
        u = torch.from_numpy(u_glob[l2g].copy())
        y = dd_step_reference(
            plan, u, lambda uc: torch.from_numpy(op_i.apply(uc.numpy())),
            lambda ul: torch.from_numpy(op_b.apply(ul.numpy())),
            lambda send, peers, counts: torch_p2p_exchange(send, peers, counts))
        err = np.abs(y.numpy() - y_glob[l2g]).max() / np.abs(y_glob).max()
        own = torch.from_numpy(np.asarray(plan.not_owned == 0))
        d = torch.sum(u[own] * y[own]).reshape(1)
        dist.all_reduce(d)
        q.put((rank, err, d.item(), float(np.dot(u_glob, y_glob)), plan.exchanged_per_direction,
               plan.iface_elems.size, plan.interior_elems.size))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "slab"), (3, "slab"), (2, "generic"), (4, "block"),
                                        (8, "block")])
def test_overlapped_protocol_hex_gloo(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dd_worker_hex, args=(r, world, port, mode, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, err, d, d_ref, nx, n_if, n_in in res:
        assert err < 1e-14, (rank, err)
        assert abs(d - d_ref) <= 1e-12 * abs(d_ref)
        assert nx > 0 and n_if > 0


def test_ddplan_hex_slabs():
    """DDPlan on hexahedral slabs: one element layer per shared face is the
    interface, the shared faces are touched by interface elements only."""
    from spectralelementmethod_amd.distributed import DDPlan, SlabPartition
    for rank in range(3):
        part = SlabPartition(9, 3, 2, 2, 3, rank)
        nodes, e2n = part.local_mesh()
        pl = DDPlan(e2n, part.n_nodes, part.neighbors, 1, part.owned)
        assert pl.iface_elems.size == len(part.neighbors) * part.ney * part.nez
        assert np.array_equal(pl.iface_nodes[pl.e2n_iface], e2n[pl.iface_elems])
        iface = np.concatenate(list(part.neighbors.values()))
        assert not np.isin(iface, e2n[pl.interior_elems]).any()
        assert pl.exchanged_per_direction == len(part.neighbors) * part.face
        assert pl.not_owned.sum() == (part.face if rank > 0 else 0)
