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
    (computed first, so the interface sum can start) and the interior ones,
    with the node states of include/sem_hip.h sem_set_map_shared:
    returns (iface_elems, interior_elems, state_iface, state_interior)."""
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


class OverlappedOperator(object):
    """Rank-local operator whose interface sum overlaps the interior
    elements: interface elements are applied first, an
    event releases the RCCL exchange on a side stream, and the interior
    elements run meanwhile on the caller's stream.  Interface nodes are
    touched only by interface elements, so the exchange's scatter-add never
    races the interior kernel."""

    def __init__(self, p, nodes, e2n, neighbors, dofs_per_node=1, device=None, group=None,
                 geometry="auto", kind=0, kernel="auto"):
        from .operators import SEMOperator
        self.dpn = dofs_per_node
        self.kind = kind
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        e2n = np.asarray(e2n)
        n_node = np.asarray(nodes).shape[1]
        ie, be, st_i, st_b = split_interface_elements(e2n, neighbors)
        if st_i.size < n_node:  # nodes beyond the last referenced one
            pad = n_node - st_i.size
            st_i = np.concatenate([st_i, np.zeros(pad, np.uint8)])
            st_b = np.concatenate([st_b, np.full(pad, _lib.NODE_OTHER, np.uint8)])
        self.n_iface_elem, self.n_interior_elem = ie.size, be.size
        if ie.size == 0 or be.size == 0:  # nothing to overlap
            self.ops = [SEMOperator(p, e2n, nodes, dofs_per_node, device=self.device,
                                    geometry=geometry, kernel=kernel)]
        else:
            self.ops = [SEMOperator(p, e2n[ie], nodes, dofs_per_node, device=self.device,
                                    geometry=geometry, node_state=st_i, kernel=kernel),
                        SEMOperator(p, e2n[be], nodes, dofs_per_node, device=self.device,
                                    geometry=geometry, node_state=st_b, kernel=kernel)]
        for op in self.ops:
            op.compute_geometry(kind)
        self.ndof = self.ops[0].ndof
        self.n_elem = e2n.shape[0]
        self.xchg = InterfaceExchange(neighbors, dofs_per_node, self.device, group) \
            if neighbors else None
        self.side = torch.cuda.Stream(device=self.device)
        self.ready = torch.cuda.Event()
        self._lib = _lib.load()

    def plan_info(self):
        return self.ops[-1].plan_info()

    def step(self, u, y, events=None):
        """y = K u on this rank's nodes, interface sum included.  ``events``
        (start, end) bracket the element kernels on the caller's stream."""
        main = torch.cuda.current_stream(self.device)
        sp = _lib.stream_ptr(main)
        up, yp = _lib.tptr(u), _lib.tptr(y)
        last = len(self.ops) - 1
        for i, op in enumerate(self.ops):
            _lib.check(self._lib.sem_zero_shared(op._ctx, yp, sp))
            if events is not None and i == 0:
                events[0].record(main)
            _lib.check(self._lib.sem_apply(op._ctx, self.kind, up, yp, _lib.APPLY_SKIP_ZERO, sp))
            if i == 0 and self.xchg is not None:
                self.ready.record(main)
            if events is not None and i == last:
                events[1].record(main)
        if self.xchg is not None:
            with torch.cuda.stream(self.side):
                self.side.wait_event(self.ready)
                self.xchg.exchange(y)
            main.wait_stream(self.side)
        return y

    def apply(self, u, out=None):
        if out is None:
            out = torch.empty_like(u)
        return self.step(u, out)
