"""Element partitioning across GPUs and the shared-DOF interface sum.

The reference has no parallelism at all (single-threaded Python loops,
sem/discrete.py:208-209).  Its element loop is embarrassingly parallel except
for the final scatter-add: a node on the boundary between two partitions gets
contributions from elements on both sides.  This module splits the elements
over ranks (one process per GPU), applies the operator locally with
``SEMOperator`` and then sums ONLY the interface entries between neighbouring
ranks -- never the full vector.

Exchange: point-to-point with each neighbour over ``torch.distributed``
(RCCL over xGMI for the "nccl" backend), 8 B per shared node and direction.
Packing and unpacking use the library's gather / scatter-add kernels on
device tensors.  CPU tensors are accepted by the exchange layer only so that
its protocol can be tested under the "gloo" backend; the operator itself has
no CPU path.
"""
import ctypes as C
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from . import meshgen


# ---------------------------------------------------------------- partitions
class StripPartition(object):
    """Contiguous strips of element columns of a structured nex x ney mesh
    (meshgen.structured_square numbering): rank r owns columns
    [ex0, ex1) and the contiguous global node range
    [node_offset, node_offset + n_nodes).  Neighbours share one node line of
    Ny = ney*p + 1 nodes."""

    def __init__(self, nex, ney, p, world, rank, dofs_per_node=1):
        if world < 1 or not (0 <= rank < world):
            raise ValueError("bad world/rank")
        if nex < world:
            raise ValueError("fewer element columns than ranks")
        self.nex, self.ney, self.p, self.world, self.rank = nex, ney, p, world, rank
        self.dpn = dofs_per_node
        base, extra = divmod(nex, world)
        cols = [base + (1 if r < extra else 0) for r in range(world)]
        starts = np.concatenate([[0], np.cumsum(cols)])
        self.ex0, self.ex1 = int(starts[rank]), int(starts[rank + 1])
        self.Ny = ney * p + 1
        self.n_nodes = ((self.ex1 - self.ex0) * p + 1) * self.Ny
        self.node_offset = self.ex0 * p * self.Ny
        self.n_elem = (self.ex1 - self.ex0) * ney
        self.neighbors = {}
        line = np.arange(self.Ny, dtype=np.int64)
        if rank > 0:
            self.neighbors[rank - 1] = line.copy()
        if rank < world - 1:
            self.neighbors[rank + 1] = self.n_nodes - self.Ny + line
        # each shared node is owned by exactly one rank (lowest rank) for
        # global reductions / gathers
        self.owned = np.ones(self.n_nodes, dtype=bool)
        if rank > 0:
            self.owned[:self.Ny] = False

    @property
    def global_nodes(self):
        return (self.nex * self.p + 1) * self.Ny

    def local_mesh(self, warp=0.0):
        nodes, e2n, off = meshgen.structured_strip(self.nex, self.ney, self.p, self.ex0, self.ex1,
                                                   warp)
        assert off == self.node_offset and nodes.shape[1] == self.n_nodes
        return nodes, e2n

    def local_to_global(self):
        return self.node_offset + np.arange(self.n_nodes, dtype=np.int64)


class SlabPartition(object):
    """Hexahedral twin of StripPartition (row N3): contiguous slabs of element
    layers along x of a structured nex x ney x nez cube
    (meshgen.structured_cube numbering): rank r owns layers [ex0, ex1), the
    contiguous global node range [node_offset, node_offset + n_nodes), and
    shares one node face of Ny*Nz nodes with each neighbouring slab.  The
    reference's loop this splits is the serial ``for cell in
    self._mesh.cells`` (sem/discrete.py:189-209) over its N-D tensor layer
    (sem/basis_functions.py:626-650).  The hexahedral chains run along xi0 =
    x, so a slab of L layers gives chains of L elements (the planner cuts
    longer ones anyway, csrc/sem_hex.hip hex_build_plan)."""

    def __init__(self, nex, ney, nez, p, world, rank):
        if world < 1 or not (0 <= rank < world):
            raise ValueError("bad world/rank")
        if nex < world:
            raise ValueError("fewer element layers than ranks")
        self.nex, self.ney, self.nez, self.p = nex, ney, nez, p
        self.world, self.rank, self.dpn = world, rank, 1
        base, extra = divmod(nex, world)
        layers = [base + (1 if r < extra else 0) for r in range(world)]
        starts = np.concatenate([[0], np.cumsum(layers)])
        self.ex0, self.ex1 = int(starts[rank]), int(starts[rank + 1])
        self.Ny, self.Nz = ney * p + 1, nez * p + 1
        self.face = self.Ny * self.Nz
        self.n_nodes = ((self.ex1 - self.ex0) * p + 1) * self.face
        self.node_offset = self.ex0 * p * self.face
        self.n_elem = (self.ex1 - self.ex0) * ney * nez
        self.neighbors = {}
        face = np.arange(self.face, dtype=np.int64)
        if rank > 0:
            self.neighbors[rank - 1] = face.copy()
        if rank < world - 1:
            self.neighbors[rank + 1] = self.n_nodes - self.face + face
        # a shared node belongs to the lower rank (global dot products)
        self.owned = np.ones(self.n_nodes, dtype=bool)
        if rank > 0:
            self.owned[:self.face] = False

    @property
    def global_nodes(self):
        return (self.nex * self.p + 1) * self.face

    def local_mesh(self, warp=0.0):
        nodes, e2n, off = meshgen.structured_slab(self.nex, self.ney, self.nez, self.p, self.ex0,
                                                  self.ex1, warp)
        assert off == self.node_offset and nodes.shape[1] == self.n_nodes
        return nodes, e2n

    def local_to_global(self):
        return self.node_offset + np.arange(self.n_nodes, dtype=np.int64)


def _split(n, parts):
    base, extra = divmod(n, parts)
    sizes = [base + (1 if r < extra else 0) for r in range(parts)]
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)


def block_grid(world):
    """px x py x pz = world with the factors as equal as possible (8 -> 2 x 2
    x 2, 4 -> 2 x 2 x 1, 6 -> 3 x 2 x 1), the largest along x."""
    best = None
    for px in range(1, world + 1):
        if world % px:
            continue
        for py in range(1, world // px + 1):
            if (world // px) % py:
                continue
            pz = world // px // py
            g = tuple(sorted((px, py, pz), reverse=True))
            key = (max(g) - min(g), -g[0])
            if best is None or key < best[0]:
                best = (key, g)
    return best[1]


class BlockPartition(object):
    """Hexahedral boxes of a structured nex x ney x nez cube on a px x py x
    pz grid of ranks (rank = (rx * py + ry) * pz + rz): each rank's elements
    are a box, its nodes the box's node box, numbered locally x-major as in
    the cube (meshgen.structured_box).  Against SlabPartition a box exposes
    fewer interface elements per element at the price of more peers (faces,
    edges and corners: up to 26): at 27^3 over 8 ranks 2 x 2 x 2 boxes of
    13-14 elements per side put about a fifth of a rank's elements on its
    interface, 8 slabs two thirds.  Shared nodes are listed per peer in
    global-id order on both sides; a shared node belongs to the lowest rank
    holding it."""

    def __init__(self, nex, ney, nez, p, grid, rank):
        px, py, pz = (int(g) for g in grid)
        self.world = world = px * py * pz
        if not (0 <= rank < world):
            raise ValueError("bad world/rank")
        if nex < px or ney < py or nez < pz:
            raise ValueError("fewer elements than ranks along an axis")
        self.nex, self.ney, self.nez, self.p, self.rank, self.dpn = nex, ney, nez, p, rank, 1
        self.grid = (px, py, pz)
        cuts = [_split(nex, px), _split(ney, py), _split(nez, pz)]

        def box(q):  # element ranges of rank q
            c = np.unravel_index(q, (px, py, pz))
            return [(int(cuts[a][c[a]]), int(cuts[a][c[a] + 1])) for a in range(3)]
        self.ranges = box(rank)
        self.Ny, self.Nz = ney * p + 1, nez * p + 1
        nb = [(e0 * p, e1 * p) for e0, e1 in self.ranges]  # inclusive node ranges
        self.shape = tuple(b - a + 1 for a, b in nb)
        self.n_nodes = int(np.prod(self.shape))
        self.n_elem = int(np.prod([e1 - e0 for e0, e1 in self.ranges]))
        self.neighbors = {}
        self.owned = np.ones(self.n_nodes, dtype=bool)
        for q in range(world):
            if q == rank:
                continue
            qb = [(e0 * p, e1 * p) for e0, e1 in box(q)]
            inter = [(max(a[0], b[0]), min(a[1], b[1])) for a, b in zip(nb, qb)]
            if any(lo > hi for lo, hi in inter):
                continue
            ax = [np.arange(lo, hi + 1) - nb[a][0] for a, (lo, hi) in enumerate(inter)]
            loc = ((ax[0][:, None, None] * self.shape[1] + ax[1][None, :, None]) * self.shape[2]
                   + ax[2][None, None, :]).ravel()
            self.neighbors[q] = loc
            if q < rank:
                self.owned[loc] = False

    @property
    def global_nodes(self):
        return (self.nex * self.p + 1) * self.Ny * self.Nz

    def local_mesh(self, warp=0.0):
        nodes, e2n, _ = meshgen.structured_box(self.nex, self.ney, self.nez, self.p,
                                               *self.ranges, warp=warp)
        return nodes, e2n

    def local_to_global(self):
        (x0, x1), (y0, y1), (z0, z1) = [(e0 * self.p, e1 * self.p) for e0, e1 in self.ranges]
        ix, iy, iz = np.arange(x0, x1 + 1), np.arange(y0, y1 + 1), np.arange(z0, z1 + 1)
        return ((ix[:, None, None] * self.Ny + iy[None, :, None]) * self.Nz
                + iz[None, None, :]).ravel()


def partition_elements(e2n, nodes, world, method="sfc"):
    """Element -> rank assignment of an arbitrary mesh in equal contiguous
    pieces of a locality-preserving element order:

    * "sfc": the Morton (Z-order) curve through the element centroids;
    * "rcm": reverse Cuthill-McKee order of the element adjacency graph
      (elements sharing a node), the ordering the reference applies to nodes
      (sem/discrete.py:169-178).

    Returns int64 [E] with values 0..world-1, the pieces differing in size by
    at most one element."""
    e2n = np.asarray(e2n)
    E = e2n.shape[0]
    if world < 1 or E < world:
        raise ValueError("need 1 <= world <= number of elements")
    flat = e2n.reshape(E, -1).astype(np.int64)
    if method == "sfc":
        c = np.asarray(nodes, dtype=np.float64)[:, flat].mean(axis=2)  # [ndim, E]
        lo = c.min(axis=1, keepdims=True)
        span = np.maximum(c.max(axis=1, keepdims=True) - lo, 1e-300)
        U = np.uint64
        if c.shape[0] == 3:  # hexahedra: 21 bits per axis, every third of 63
            q = np.minimum((c - lo) / span * 2097151.0, 2097151.0).astype(np.uint64)

            def spread3(v):
                v = (v | (v << U(32))) & U(0x1F00000000FFFF)
                v = (v | (v << U(16))) & U(0x1F0000FF0000FF)
                v = (v | (v << U(8))) & U(0x100F00F00F00F00F)
                v = (v | (v << U(4))) & U(0x10C30C30C30C30C3)
                return (v | (v << U(2))) & U(0x1249249249249249)
            key = spread3(q[0]) | (spread3(q[1]) << U(1)) | (spread3(q[2]) << U(2))
        else:
            q = np.minimum((c - lo) / span * 65535.0, 65535.0).astype(np.uint64)

            def spread(v):  # 16 bits -> every other of 32
                v = (v | (v << U(8))) & U(0x00FF00FF)
                v = (v | (v << U(4))) & U(0x0F0F0F0F)
                v = (v | (v << U(2))) & U(0x33333333)
                return (v | (v << U(1))) & U(0x55555555)
            key = spread(q[0]) | (spread(q[1]) << U(1))
        order = np.argsort(key, kind="stable")
    elif method == "rcm":
        from scipy import sparse
        from scipy.sparse import csgraph
        n_node = int(flat.max()) + 1
        B = sparse.csr_matrix((np.ones(flat.size, np.int8),
                               (np.repeat(np.arange(E), flat.shape[1]), flat.ravel())),
                              shape=(E, n_node))
        A = (B @ B.T).tocsr()
        order = csgraph.reverse_cuthill_mckee(A, symmetric_mode=True)
    else:
        raise ValueError("method must be 'sfc' or 'rcm'")
    rank = np.empty(E, dtype=np.int64)
    bounds = (np.arange(world + 1) * E) // world
    for r in range(world):
        rank[order[bounds[r]:bounds[r + 1]]] = r
    return rank


class GenericPartition(object):
    """Any element -> rank assignment of an arbitrary mesh.  Local nodes are
    the sorted global ids the rank's elements touch; the interface with each
    neighbour is their intersection, in global-id order on both sides."""

    def __init__(self, e2n, elem_rank, world, rank, dofs_per_node=1):
        e2n = np.asarray(e2n)
        elem_rank = np.asarray(elem_rank)
        self.world, self.rank, self.dpn = world, rank, dofs_per_node
        mine = np.nonzero(elem_rank == rank)[0]
        self.elements = mine
        self.l2g = np.unique(e2n[mine])
        g2l = {g: i for i, g in enumerate(self.l2g.tolist())}
        self.e2n_local = np.vectorize(g2l.__getitem__, otypes=[np.uint32])(e2n[mine]) \
            if mine.size else np.zeros((0,) + e2n.shape[1:], np.uint32)
        self.n_nodes = self.l2g.size
        self.n_elem = mine.size
        self.neighbors = {}
        # rank owning each node = lowest rank touching it
        owner = np.full(int(e2n.max()) + 1, world, dtype=np.int64)
        for r in range(world):
            nodes_r = np.unique(e2n[elem_rank == r])
            owner[nodes_r] = np.minimum(owner[nodes_r], r)
            if r == rank:
                continue
            shared = np.intersect1d(self.l2g, nodes_r, assume_unique=True)
            if shared.size:
                self.neighbors[r] = np.searchsorted(self.l2g, shared)
        self.owned = owner[self.l2g] == rank

    def local_to_global(self):
        return self.l2g


# ---------------------------------------------------------------- exchange
class InterfaceExchange(object):
    """Sums the shared entries of a rank-local vector with its neighbours:
    y[iface_k] += y_neighbour[iface_k] for every neighbour k (dpn components
    per node).  One isend/irecv pair per neighbour, batched."""

    def __init__(self, neighbors, dofs_per_node=1, device=None, group=None):
        self.group = group
        self.dpn = dofs_per_node
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.peers = sorted(neighbors)
        self.idx = {}
        self.send = {}
        self.recv = {}
        for r in self.peers:
            nodes = np.asarray(neighbors[r], dtype=np.int64)
            dof = (nodes[:, None] * self.dpn + np.arange(self.dpn)[None, :]).ravel()
            if self.device.type == "cuda":
                self.idx[r] = torch.from_numpy(dof.astype(np.uint32).view(np.int32)).to(self.device)
            else:
                self.idx[r] = torch.from_numpy(dof)
            self.send[r] = torch.empty(dof.size, dtype=torch.float64, device=self.device)
            self.recv[r] = torch.empty(dof.size, dtype=torch.float64, device=self.device)
        self.bytes_per_exchange = sum(8 * t.numel() for t in self.send.values())

    def _pack(self, y, r):
        if y.is_cuda:
            _lib.check(_lib.load().sem_gather(_lib.tptr(y), _lib.tptr(self.idx[r]),
                                              self.idx[r].numel(), _lib.tptr(self.send[r]),
                                              _lib.stream_ptr()))
        else:
            torch.index_select(y, 0, self.idx[r], out=self.send[r])

    def _unpack(self, y, r):
        if y.is_cuda:
            _lib.check(_lib.load().sem_scatter_add(_lib.tptr(y), _lib.tptr(self.idx[r]),
                                                   self.idx[r].numel(), _lib.tptr(self.recv[r]),
                                                   _lib.stream_ptr()))
        else:
            y.index_add_(0, self.idx[r], self.recv[r])

    def exchange(self, y):
        if not self.peers:
            return y
        for r in self.peers:
            self._pack(y, r)
        ops = []
        for r in self.peers:
            ops.append(dist.P2POp(dist.isend, self.send[r], r, group=self.group))
            ops.append(dist.P2POp(dist.irecv, self.recv[r], r, group=self.group))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        for r in self.peers:
            self._unpack(y, r)
        return y


class DistributedOperator(object):
    """Rank-local operator + interface sum = the global action restricted to
    this rank's nodes.  ``local_op`` is any object with
    ``apply(u, out=None, kind=...)`` (normally SEMOperator)."""

    def __init__(self, local_op, partition, group=None, device=None):
        self.op = local_op
        self.part = partition
        dev = device if device is not None else getattr(local_op, "device", None)
        self.xchg = InterfaceExchange(partition.neighbors, partition.dpn, dev, group)

    def apply(self, u, out=None, kind=0):
        y = self.op.apply(u, out=out, kind=kind)
        return self.xchg.exchange(y)

    def global_dot(self, a, b, group=None):
        """Owned-entry dot product reduced over ranks."""
        own = torch.from_numpy(np.repeat(self.part.owned, self.part.dpn)).to(a.device)
        s = torch.sum(a[own] * b[own]).reshape(1)
        dist.all_reduce(s, group=group)
        return s.item()


# ---------------------------------------------------------------- overlap
def split_interface_elements(e2n, neighbors):
    """Split a rank's elements into the ones touching a partition interface
    and the interior ones, with the node states of include/sem_hip.h
    sem_set_map_shared for applying the two sets IN ORDER into one y
    (interface first): returns (iface_elems, interior_elems, state_iface,
    state_interior).  The multi-GPU step (OverlappedOperator) instead runs
    the two sets CONCURRENTLY into separate vectors (DDPlan)."""
    e2n = np.asarray(e2n)
    n_elem = e2n.shape[0]
    flat = e2n.reshape(n_elem, -1)
    n_node = int(flat.max()) + 1 if flat.size else 0
    iface = np.zeros(n_node, dtype=bool)
    for nodes in neighbors.values():
        iface[np.asarray(nodes, dtype=np.int64)] = True
    touch = iface[flat].any(axis=1)
    ie = np.nonzero(touch)[0]
    be = np.nonzero(~touch)[0]
    in_i = np.zeros(n_node, dtype=bool)
    in_b = np.zeros(n_node, dtype=bool)
    in_i[flat[ie].ravel()] = True
    in_b[flat[be].ravel()] = True
    state_i = np.where(in_b & ~in_i, _lib.NODE_OTHER, 0).astype(np.uint8)
    # interior operator: everything the interface operator wrote is PRIOR;
    # nodes neither references were zeroed by the interface operator
    state_b = np.where(in_i, _lib.NODE_PRIOR, np.where(in_b, 0, _lib.NODE_OTHER)).astype(np.uint8)
    return ie, be, state_i, state_b


class DDPlan(object):
    """Host plan of one rank's ``sem_dd`` (include/sem_hip.h): which elements
    touch a node shared with another rank (computed first, over a compact
    renumbering of their nodes, on a side stream) and which are interior;
    the compact <-> local DOF map; the compact DOFs exchanged with each peer
    (in the order of ``neighbors[peer]``, which both sides agree on); the
    DOFs another rank owns (left out of global dot products).

    e2n: local element map [E, n, n]; neighbors: {peer rank: local node ids};
    owned: bool [n_node] (None = all owned)."""

    def __init__(self, e2n, n_node, neighbors, dofs_per_node=1, owned=None):
        e2n = np.asarray(e2n)
        self.dpn = dpn = int(dofs_per_node)
        self.n_node = int(n_node)
        self.ndof = dpn * self.n_node
        flat = e2n.reshape(e2n.shape[0], -1).astype(np.int64)
        shared = np.zeros(self.n_node, dtype=bool)
        for nodes in neighbors.values():
            shared[np.asarray(nodes, dtype=np.int64)] = True
        touch = shared[flat].any(axis=1)
        self.iface_elems = np.nonzero(touch)[0]
        self.interior_elems = np.nonzero(~touch)[0]
        self.iface_nodes = np.unique(flat[self.iface_elems])  # sorted local ids
        self.e2n_iface = np.searchsorted(self.iface_nodes, flat[self.iface_elems]).astype(
            np.uint32).reshape((self.iface_elems.size,) + e2n.shape[1:])
        comp = np.arange(dpn, dtype=np.int64)
        self.iface_dofs = (self.iface_nodes[:, None] * dpn + comp[None, :]).ravel().astype(
            np.uint32)
        self.peers = sorted(int(r) for r in neighbors)
        counts, dofs = [], []
        for r in self.peers:
            nodes = np.asarray(neighbors[r], dtype=np.int64)
            c = np.searchsorted(self.iface_nodes, nodes)
            if nodes.size and (c.max() >= self.iface_nodes.size
                               or not np.array_equal(self.iface_nodes[c], nodes)):
                raise ValueError("shared node of peer %d is not on an element of this rank" % r)
            dofs.append((c[:, None] * dpn + comp[None, :]).ravel())
            counts.append(dofs[-1].size)
        self.peer_counts = np.asarray(counts, dtype=np.int64)
        self.peer_dofs = (np.concatenate(dofs) if dofs else np.zeros(0, np.int64)).astype(
            np.uint32)
        self.not_owned = None if owned is None else np.repeat(
            ~np.asarray(owned, dtype=bool), dpn).astype(np.uint8)

    @property
    def exchanged_per_direction(self):
        return int(self.peer_counts.sum())


def dd_step_reference(plan, u, apply_iface, apply_interior, exchange):
    """The sequence ``sem_dd_apply`` enqueues (csrc/sem_dd.hip), restated on
    host tensors so the protocol can be checked under gloo without a GPU:
    interface elements on the compact vector, pack, exchange, unpack, then
    the interior result plus the interface result.  ``exchange(send, peers,
    counts)`` returns the received buffer."""
    cidx = torch.from_numpy(plan.iface_dofs.astype(np.int64))
    pidx = torch.from_numpy(plan.peer_dofs.astype(np.int64))
    y_c = apply_iface(u[cidx]) if cidx.numel() else torch.zeros(0, dtype=u.dtype)
    send = y_c[pidx]
    y = apply_interior(u) if plan.interior_elems.size else torch.zeros_like(u)
    recv = exchange(send, plan.peers, plan.peer_counts)
    off = np.concatenate([[0], np.cumsum(plan.peer_counts)])
    for k in range(len(plan.peers)):  # one pass per peer: a DOF may have several
        y_c.index_add_(0, pidx[off[k]:off[k + 1]], recv[off[k]:off[k + 1]])
    y.index_add_(0, cidx, y_c)
    return y


def torch_p2p_exchange(send, peers, counts, group=None, recv=None):
    """Point-to-point exchange of the packed interface values with every peer
    through torch.distributed (one isend/irecv pair per peer, batched)."""
    if recv is None:
        recv = torch.empty_like(send)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    ops = []
    for k, r in enumerate(peers):
        a, b = int(off[k]), int(off[k + 1])
        ops.append(dist.P2POp(dist.isend, send[a:b], r, group=group))
        ops.append(dist.P2POp(dist.irecv, recv[a:b], r, group=group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return recv


class TorchTransport(object):
    """Caller-supplied transport of a ``sem_dd`` (sem_dd_set_transport) over
    torch.distributed: the fallback when the native RCCL communicator cannot
    be created, and the path the gloo tests drive on one GPU (several ranks
    on one device; RCCL refuses duplicate GPUs).  With an NCCL (RCCL) process
    group the buffers stay on the device and the collectives are ordered on
    the library's side stream; with gloo they are staged through host
    memory."""

    def __init__(self, device, group=None):
        self.lib = _lib.load()
        self.group = group
        self.device = torch.device(device)
        self.on_device = "nccl" in str(dist.get_backend(group)).lower()
        self._xfn = _lib.EXCHANGE_FN(self._exchange)
        self._rfn = _lib.ALLREDUCE_FN(self._allreduce)
        self._cache = {}
        self.error = None
        self._fullsync = os.environ.get("SEM_TT_FULLSYNC") == "1"  # diagnostic

    def _bufs(self, key, n, stream):
        """persistent staging buffers (allocated once, under the stream that
        uses them, so the caching allocator never hands them to other work)"""
        b = self._cache.get(key)
        if b is None or b[0].numel() < n:
            if self.on_device:
                with torch.cuda.stream(stream):
                    b = tuple(torch.empty(max(n, 1), dtype=torch.float64, device=self.device)
                              for _ in range(2))
            else:
                b = tuple(torch.empty(max(n, 1), dtype=torch.float64).pin_memory()
                          for _ in range(2))
            self._cache[key] = b
        return b[0][:n], b[1][:n]

    def _sync(self, stream):
        if self._fullsync:
            torch.cuda.synchronize(self.device)
        else:
            stream.synchronize()

    def _exchange(self, user, n_peers, peers, off, d_send, d_recv, side):
        try:
            peers_l = [peers[k] for k in range(n_peers)]
            total = off[n_peers]
            counts = [off[k + 1] - off[k] for k in range(n_peers)]
            nb = 8 * total
            stream = torch.cuda.ExternalStream(side, device=self.device) if side else \
                torch.cuda.default_stream(self.device)
            send, recv = self._bufs("x", total, stream)
            _lib.check(self.lib.sem_copy_async(send.data_ptr(), d_send, nb, side))
            if self.on_device:
                with torch.cuda.stream(stream):
                    torch_p2p_exchange(send, peers_l, counts, self.group, recv)
                    _lib.check(self.lib.sem_copy_async(d_recv, recv.data_ptr(), nb, side))
            else:
                self._sync(stream)
                torch_p2p_exchange(send, peers_l, counts, self.group, recv)
                _lib.check(self.lib.sem_copy_async(d_recv, recv.data_ptr(), nb, side))
                self._sync(stream)  # the host buffer is reused by the next call
            return 0
        except Exception as e:  # reported through the library's return code
            self.error = e
            return 1

    def _allreduce(self, user, d_buf, count, st):
        try:
            nb = 8 * count
            # NULL (None here) is the legacy default stream
            stream = torch.cuda.ExternalStream(st, device=self.device) if st else \
                torch.cuda.default_stream(self.device)
            t, _ = self._bufs("r%d" % (st or 0), count, stream)
            if self.on_device:
                with torch.cuda.stream(stream):
                    _lib.check(self.lib.sem_copy_async(t.data_ptr(), d_buf, nb, st))
                    dist.all_reduce(t, group=self.group)
                    _lib.check(self.lib.sem_copy_async(d_buf, t.data_ptr(), nb, st))
            else:
                _lib.check(self.lib.sem_copy_async(t.data_ptr(), d_buf, nb, st))
                self._sync(stream)
                dist.all_reduce(t, group=self.group)
                _lib.check(self.lib.sem_copy_async(d_buf, t.data_ptr(), nb, st))
                self._sync(stream)
            return 0
        except Exception as e:
            self.error = e
            return 1

    def install(self, dd, world, rank):
        _lib.check(self.lib.sem_dd_set_transport(dd, C.cast(self._xfn, C.c_void_p),
                                                 C.cast(self._rfn, C.c_void_p), None, world,
                                                 rank))


def init_rccl(dd, world, rank, group=None):
    """Native transport: one RCCL communicator over all ranks (collective:
    every rank calls it).  Rank 0 draws the id, torch.distributed carries it."""
    lib = _lib.load()
    buf = C.create_string_buffer(_lib.RCCL_ID_BYTES)
    if rank == 0:
        _lib.check(lib.sem_rccl_unique_id(buf, _lib.RCCL_ID_BYTES))
    obj = [buf.raw if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    buf = C.create_string_buffer(obj[0], _lib.RCCL_ID_BYTES)
    _lib.check(lib.sem_dd_init_rccl(dd, buf, world, rank))


class OverlappedOperator(object):
    """One rank's part of the global operator.

    Single rank (``world`` 1): one ``SEMOperator``.  Several ranks: a native
    ``sem_dd`` (csrc/sem_dd.hip) holding two operators -- the interface
    elements over a compact numbering of their nodes, applied on a side
    stream and summed with the neighbours, and the interior elements applied
    meanwhile on the caller's stream -- so one ``step`` is one C call.

    transport: "rccl" (native RCCL send/recv + all-reduce), "torch"
    (torch.distributed point-to-point, see TorchTransport), or "auto"
    (RCCL when the process group is NCCL and the communicator comes up,
    torch otherwise), or "loopback" (diagnostic, sem_dd_set_loopback: each
    exchange returns this rank's own interface values, so ONE rank of a
    decomposition runs and is timed alone on one GPU; the result is not the
    global action).  decompose (default: world > 1) forces the sem_dd path
    (tests run it on one rank to exercise the native RCCL calls)."""

    def __init__(self, p, nodes, e2n, neighbors, dofs_per_node=1, device=None, group=None,
                 geometry="auto", kind=0, kernel="auto", owned=None, transport="auto",
                 world=None, rank=None, decompose=None):
        from .operators import SEMOperator
        self.dpn = dofs_per_node
        self.kind = kind
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self._lib = _lib.load()
        e2n = np.asarray(e2n)
        nodes = np.asarray(nodes)
        n_node = nodes.shape[1]
        self.world = world if world is not None else (
            dist.get_world_size(group) if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized()
                                                   else 0)
        self.n_elem = e2n.shape[0]
        self.ndof = dofs_per_node * n_node
        self.dd = None
        self.transport = "none"
        self.exchange_bytes = 0
        kw = dict(dofs_per_node=dofs_per_node, device=self.device, geometry=geometry,
                  kernel=kernel)
        if decompose is None:
            decompose = self.world > 1
        if not decompose:
            self.ops = [SEMOperator(p, e2n, nodes, **kw)]
            self.n_iface_elem, self.n_interior_elem = 0, self.n_elem
            self.plan = None
        else:
            self.plan = pl = DDPlan(e2n, n_node, neighbors, dofs_per_node, owned)
            self.n_iface_elem, self.n_interior_elem = pl.iface_elems.size, pl.interior_elems.size
            # the interface elements over the rank's own numbering: they read
            # u directly (no gather of a compact copy) and write a private
            # rank-sized y_c (sem_dd_create's local mode)
            self.iface = SEMOperator(p, e2n[pl.iface_elems], nodes, **kw) \
                if pl.iface_elems.size else None
            # a local-mode interface plan with atomic first
            # writers zeroes its whole zero list (nearly every node of the
            # rank) on every step; such plans (generic / unstructured
            # partitions) take the compact numbering of the interface DOFs
            # instead (sem_dd_create's compact mode)
            self.iface_compact = False
            if (self.iface is not None and dofs_per_node == 1 and
                    self.iface.plan_info().get("atomic_groups", 0) > 0):
                self.iface.close()
                self.iface = SEMOperator(p, pl.e2n_iface, np.asarray(nodes)[:, pl.iface_nodes],
                                         **kw)
                self.iface_compact = True
            self.interior = SEMOperator(p, e2n[pl.interior_elems], nodes, **kw) \
                if pl.interior_elems.size else None
            self.ops = [o for o in (self.iface, self.interior) if o is not None]
            dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
            cidx = dev(pl.iface_dofs.view(np.int32))
            pidx = dev(pl.peer_dofs.view(np.int32))
            notown = dev(pl.not_owned) if pl.not_owned is not None else None
            peers = (C.c_int * max(1, len(pl.peers)))(*pl.peers)
            counts = (C.c_int64 * max(1, len(pl.peers)))(*pl.peer_counts.tolist())
            dd = C.c_void_p()
            _lib.check(self._lib.sem_dd_create(
                C.byref(dd), self.iface._ctx if self.iface else None,
                self.interior._ctx if self.interior else None, self.ndof, _lib.tptr(cidx),
                int(pl.iface_dofs.size), len(pl.peers), peers, counts, _lib.tptr(pidx),
                _lib.tptr(notown), self.device.index))
            self.dd = dd
            self.exchange_bytes = 8 * pl.exchanged_per_direction
            self._install_transport(transport, group)
        for op in self.ops:
            op.compute_geometry(kind)

    def _install_transport(self, transport, group):
        backend = str(dist.get_backend(group)).lower() if dist.is_initialized() else ""
        if transport not in ("auto", "rccl", "torch", "loopback", "rccl_self"):
            raise ValueError("transport must be auto, rccl, torch, loopback or rccl_self")
        if transport == "loopback":  # diagnostic: one rank timed alone (sem_dd_set_loopback)
            _lib.check(self._lib.sem_dd_set_loopback(self.dd))
            self.world, self.rank = 1, 0
            self.transport = "loopback"
            return
        if transport == "rccl_self":  # timing: RCCL send/recv to self (sem_dd_set_rccl_self)
            _lib.check(self._lib.sem_dd_set_rccl_self(self.dd))
            self.world, self.rank = 1, 0
            self.transport = "rccl_self"
            return
        if transport == "rccl" or (transport == "auto" and "nccl" in backend):
            try:
                init_rccl(self.dd, self.world, self.rank, group)
                self.transport = "rccl"
                return
            except Exception as e:
                if transport == "rccl":
                    raise
                import sys
                print("[sem] native RCCL transport unavailable (%s); using torch.distributed" % e,
                      file=sys.stderr, flush=True)
        self._torch = TorchTransport(self.device, group)
        self._torch.install(self.dd, self.world, self.rank)
        self.transport = "torch-" + ("device" if self._torch.on_device else "host")

    def close(self):
        if self.dd:
            self._lib.sem_dd_destroy(self.dd)
            self.dd = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc and getattr(self, "_torch", None) is not None and self._torch.error is not None:
            err, self._torch.error = self._torch.error, None
            raise RuntimeError("interface transport failed: %r" % (err,))
        _lib.check(rc)

    def plan_info(self):
        return (self.interior or self.iface).plan_info() if self.dd else self.ops[0].plan_info()

    def dd_info(self):
        """The decomposition's sem_dd_info as a dict (None on one rank)."""
        if not self.dd:
            return None
        v = (C.c_int64 * 16)()
        _lib.check(self._lib.sem_dd_info(self.dd, v, 16))
        steps = max(1, v[9])
        return dict(ndof=v[0], iface_dofs=v[1], peers=v[2], exchanged=v[3],
                    transport=("none", "rccl", "callbacks", "loopback", "rccl_self")[v[4]],
                    interior=bool(v[5]), graphs=bool(v[6]), captures=v[7], replays=v[8],
                    applies=v[9], host_ns=v[10], host_ns_transport=v[11],
                    host_us_per_apply=v[10] / steps / 1e3,
                    host_us_per_apply_excl_transport=(v[10] - v[11]) / steps / 1e3,
                    host_ns_side=v[12], host_ns_interior=v[13], host_ns_finish=v[14],
                    host_us_side=v[12] / steps / 1e3, host_us_interior=v[13] / steps / 1e3,
                    host_us_finish=v[14] / steps / 1e3, zero_list_in_finish=bool(v[15] & 1),
                    seam_sum_in_finish=bool(v[15] & 2), seam_sum_in_pack=bool(v[15] & 4),
                    split_finish=bool(v[15] & 8),
                    event_fence="device" if v[15] & 16 else "system")

    def set_graphs(self, enable):
        """Captured step on / off (sem_dd_set_graphs)."""
        if self.dd:
            _lib.check(self._lib.sem_dd_set_graphs(self.dd, 1 if enable else 0))
        return self

    def step(self, u, y, events=None):
        """y = K u on this rank's DOFs, shared DOFs summed over all ranks.
        ``events`` (start, end) bracket the step on the caller's stream
        (either may be None)."""
        main = torch.cuda.current_stream(self.device)
        sp = _lib.stream_ptr(main)
        if events is not None and events[0] is not None:
            events[0].record(main)
        if self.dd:
            self._check(self._lib.sem_dd_apply(self.dd, self.kind, _lib.tptr(u), _lib.tptr(y),
                                               sp))
        else:
            _lib.check(self._lib.sem_apply(self.ops[0]._ctx, self.kind, _lib.tptr(u),
                                           _lib.tptr(y), 0, sp))
        if events is not None and events[1] is not None:
            events[1].record(main)
        return y

    def apply(self, u, out=None):
        if out is None:
            out = torch.empty_like(u)
        return self.step(u, out)

    def diag(self):
        d = torch.empty(self.ndof, dtype=torch.float64, device=self.device)
        sp = _lib.stream_ptr(torch.cuda.current_stream(self.device))
        if self.dd:
            self._check(self._lib.sem_dd_diag(self.dd, self.kind, _lib.tptr(d), sp))
        else:
            _lib.check(self._lib.sem_diag(self.ops[0]._ctx, self.kind, _lib.tptr(d), sp))
        return d

    def pcg_solve(self, rhs, x, dirichlet, rtol=1e-13, max_iter=20000,
                  check_every=_lib.PCG_CHECK_EVERY, renumber="auto"):
        """Jacobi-PCG for K x = rhs on this rank's DOFs (dirichlet: bool mask;
        x holds the Dirichlet values and the initial guess, updated in place).
        Returns (x, iterations executed, final relative residual).  One rank
        without the decomposition: SEMOperator.pcg_solve (renumber: its
        solver numbering)."""
        if self.dd and self.world > 1 and self.plan.not_owned is None:
            # every rank would count its copies of the shared DOFs in the
            # global dot products: a wrong inner product, silently
            raise ValueError("pcg_solve on several ranks needs the ownership mask (owned=...)")
        mask = torch.as_tensor(dirichlet, dtype=torch.bool).to(self.device).to(torch.uint8)
        its, rel = C.c_int(0), C.c_double(0.0)
        sp = _lib.stream_ptr(torch.cuda.current_stream(self.device))
        if self.dd:
            self._check(self._lib.sem_dd_pcg_solve(
                self.dd, self.kind, _lib.tptr(rhs), _lib.tptr(x), _lib.tptr(mask), float(rtol),
                int(max_iter), int(check_every), C.byref(its), C.byref(rel), sp))
        else:
            return self.ops[0].pcg_solve(rhs, x, dirichlet, rtol=rtol, max_iter=max_iter,
                                         kind=self.kind,
                                         stream=torch.cuda.current_stream(self.device),
                                         renumber=renumber)
        return x, its.value, rel.value


DomainOperator = OverlappedOperator
