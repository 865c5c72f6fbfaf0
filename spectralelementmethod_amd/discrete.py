"""Meshes, DOF managers and finite elements (mirror of sem/discrete.py).

Same class names, constructor arguments, properties and exceptions as the
reference: ``Mesh`` (:920-1127), ``Cell`` (:857-882), ``DOFManager``
(:44-280), ``DOFManagerSC`` (:283-528) and ``FiniteElement`` (:531-705).

What changes is where the work happens.  The reference builds a Mapping and
dense element operators per element inside a Python generator and applies
them one element at a time.  Here the element loop is one GPU launch:

* ``DOFManager.stiffness_action(u)`` / ``operator_action(kind, u)`` -- the
  global matrix-free action (csrc/sem_kernels.h), new batched entry points;
* ``finite_elements()`` still yields per-element ``FiniteElement`` objects
  with the reference's properties, but their geometry (x_phys, J, invJ,
  detJ, detJxW) comes from one batched device computation;
* ``DOFManagerSC`` keeps the reference's static-condensation API
  (init_global_linear_system, reorder_local_system_hier,
  compute_local_sc_system, assemble_global_sc_system, solve; :404-528) with
  the element Schur complements and interior back-solves as batched device
  launches and the condensed system solved by device PCG;
  ``DOFManagerSC.solve_poisson`` solves the same assembled Poisson system
  matrix-free (Jacobi-PCG on the GPU, no element matrices at all).

Node reorderings (RCM, static-condensation ordering) are host-side setup and
reproduce the reference's permutations exactly.
"""
from collections import namedtuple

import numpy as np
from scipy import sparse

from .geometry import NCube, Quadrilateral
from .mapping import Mapping, OutsideDomain  # noqa: F401

_CELL_CHUNK = 4096


class Static_COO_Matrix(object):
    """COO triplets (sem/discrete.py:26-41)."""

    def __init__(self, data, row_col, shape):
        self.data = data
        self.row_col = row_col
        self.row = row_col[0]
        self.col = row_col[1]
        self.shape = shape

    def tocoo(self):
        return sparse.coo_matrix((self.data, self.row_col))


# ---------------------------------------------------------------------------
class CellBase(object):
    """Part of a mesh whose nodes define a cell (sem/discrete.py:777-855)."""

    def __init__(self, mesh, geometry, node_map):
        self._mesh = mesh
        self._geometry = geometry
        self._node_map = node_map

    @property
    def ndim(self):
        return self._geometry.ndim

    @property
    def n_nodes(self):
        return self._geometry.n_nodes

    @property
    def n_exterior_nodes(self):
        return self._geometry.n_exterior_nodes

    @property
    def n_interior_nodes(self):
        return self._geometry.n_interior_nodes

    @property
    def geometry(self):
        return self._geometry

    @property
    def node_ind_lexicographic(self):
        return self._node_map

    @property
    def nodes_lexicographic(self):
        return self._mesh.nodes[:, self._node_map]

    @property
    def node_ind_hierarchical(self):
        return self._node_map.flat[self._geometry.hierarchical_node_order]

    @property
    def nodes_hierarchical(self):
        return self._mesh.nodes[:, self.node_ind_hierarchical]

    @property
    def vertex_node_ind(self):
        return self._node_map.flat[self._geometry.vertex_node_ind]

    @property
    def vertex_nodes(self):
        return self._mesh.nodes[:, self.vertex_node_ind]

    @property
    def exterior_node_ind(self):
        return self._node_map.flat[self._geometry.exterior_node_ind]

    @property
    def exterior_nodes(self):
        return self._mesh.nodes[:, self.exterior_node_ind]

    @property
    def interior_node_ind(self):
        return self._node_map.flat[self._geometry.interior_node_ind]

    @property
    def interior_nodes(self):
        return self._mesh.nodes[:, self.interior_node_ind]


class Cell(CellBase):
    def __init__(self, mesh, geometry, node_map, region_id, adj_map, boundary_data):
        CellBase.__init__(self, mesh, geometry, node_map)
        self._region_id = region_id
        self._adj_map = adj_map
        self._boundary_data = boundary_data

    @property
    def region_id(self):
        return self._region_id

    @property
    def region_name(self):
        return self._mesh._region_names[self._region_id]


class Mesh(object):
    """Finite element mesh (sem/discrete.py:920-1127).  Node maps of all cells
    live in one uint32 array [n_cells, *shape] so the device path can take it
    whole (``element_map``)."""

    CellData = namedtuple("CellData", ["geometry_id", "region_id", "node_map"])
    BoundaryData = namedtuple("BoundaryData", ["ndim", "index"])

    def __init__(self, ndim):
        self._ndim = ndim
        self._geometries = []
        self._maps = []            # pending per-cell node maps (add_cell)
        self._blocks = []          # consolidated uint32 arrays
        self._geom_ids = []
        self._region_ids = []
        self._region_names = []
        self._region_id_lookup = {}
        self._boundary_names = []
        self._boundary_id_lookup = {}
        self._boundary_map = {}
        self._boundary_cells = []
        self._adj = None           # [E, n_sides] neighbour cell per side, -1 on a boundary
        self._e2n = None
        self.condensed = False
        self.version = 0           # bumped whenever nodes are permuted
        self.nodes = np.zeros((ndim, 0))

    @classmethod
    def from_arrays(cls, nodes, e2n, region="*"):
        """Mesh of identical cells from nodes [d, N] and an element map [E,
        n0, .., n_{d-1}] (the batched form of add_cell): quadrilaterals for
        d = 2, hexahedra (NCube of three axes) for d = 3."""
        e2n = np.array(e2n, dtype=np.uint32, order="C")  # a copy: node permutations
        nodes = np.array(nodes, dtype=np.float64)         # must not reach the caller's
        d = nodes.shape[0]
        if e2n.ndim != d + 1 or d not in (2, 3):
            raise ValueError("nodes [d, N] with d = 2 or 3 and an element map [E] + [n] * d")
        mesh = cls(d)
        mesh.set_nodes(nodes)
        gid = mesh.add_geometry(Quadrilateral(*e2n.shape[1:]) if d == 2 else NCube(*e2n.shape[1:]))
        rid = mesh.new_region(region)
        mesh.add_cells(e2n, gid, rid)
        return mesh

    @property
    def ndim(self):
        return self._ndim

    @property
    def n_nodes(self):
        return self.nodes.shape[1]

    @property
    def n_cells(self):
        return len(self._geom_ids)

    @property
    def n_boundary_cells(self):
        return len(self._boundary_map)

    def add_geometry(self, geometry):
        if geometry.ndim > self.ndim:
            raise ValueError("Cell geometry has more dimensions than the mesh.")
        self._geometries.append(geometry)
        return len(self._geometries) - 1

    def get_geometries(self):
        return self._geometries

    def new_region(self, name):
        rid = len(self._region_names)
        self._region_names.append(name)
        self._region_id_lookup[name] = rid
        return rid

    def new_boundary(self, name):
        bid = len(self._boundary_names)
        self._boundary_names.append(name)
        self._boundary_id_lookup[name] = bid
        self._boundary_cells.append(set())
        return bid

    def set_nodes(self, nodes):
        nodes = np.asarray(nodes)
        if nodes.shape[0] != self.ndim:
            raise ValueError("Points have the wrong number of dimensions.")
        self.nodes = nodes

    def add_cell(self, node_ind, geometry_id, region_id):
        node_ind = np.asarray(node_ind, dtype=np.uint32)
        geo = self._geometries[geometry_id]
        node_ind = node_ind.reshape(geo.shape)
        self._maps.append(node_ind)
        self._geom_ids.append(geometry_id)
        self._region_ids.append(region_id)
        self._e2n = None

    def add_cells(self, e2n, geometry_id, region_id):
        """Batched add_cell: e2n [k, *shape]; region_id one id or k ids."""
        e2n = np.ascontiguousarray(e2n, dtype=np.uint32)
        geo = self._geometries[geometry_id]
        if tuple(e2n.shape[1:]) != tuple(geo.shape):
            raise ValueError("cell maps do not match the geometry shape")
        self._flush()
        self._blocks.append(e2n)
        self._geom_ids.extend([geometry_id] * e2n.shape[0])
        if np.ndim(region_id) == 0:
            self._region_ids.extend([region_id] * e2n.shape[0])
        else:
            region_id = [int(r) for r in region_id]
            if len(region_id) != e2n.shape[0]:
                raise ValueError("one region id per cell expected")
            self._region_ids.extend(region_id)
        self._e2n = None

    def set_adjacency(self, adj):
        """Neighbour cell across each side ([E, n_sides], -1 where the side is
        on the mesh boundary): the reference's per-cell _adj_map
        (sem/discrete.py:1048; filled by sem/grid_importers.py:268)."""
        adj = np.asarray(adj, dtype=np.int64)
        if adj.shape[0] != self.n_cells:
            raise ValueError("one adjacency row per cell expected")
        self._adj = adj

    def adjacency(self, i):
        """[neighbour or None per side] of cell i (reference _adj_map[i])."""
        if self._adj is None:
            geo = self._geometries[self._geom_ids[i]]
            return [None] * geo.n_sub_geometries()
        return [int(a) if a >= 0 else None for a in self._adj[i]]

    def add_boundary_cell(self, cell_number, bnd_id, ndim, index):
        cell = self._boundary_map.setdefault(cell_number, {})
        cell.setdefault(bnd_id, []).append(Mesh.BoundaryData(ndim, index))
        self._boundary_cells[bnd_id].add(cell_number)

    def _flush(self):
        if self._maps:
            shapes = {m.shape for m in self._maps}
            if len(shapes) == 1:
                self._blocks.append(np.stack(self._maps))
            else:
                self._blocks.extend(m[None] for m in self._maps)
            self._maps = []

    def element_map(self):
        """uint32 [n_cells, n0, n1] (all cells must share one shape)."""
        if self._e2n is None:
            self._flush()
            if not self._blocks:
                raise ValueError("mesh has no cells")
            shapes = {b.shape[1:] for b in self._blocks}
            if len(shapes) != 1:
                raise NotImplementedError("meshes mixing cell shapes are not supported")
            self._e2n = self._blocks[0] if len(self._blocks) == 1 else \
                np.concatenate(self._blocks)
            self._blocks = [self._e2n]
        return self._e2n

    def get_cell(self, i):
        e2n = self.element_map()
        geo = self._geometries[self._geom_ids[i]]
        return Cell(self, geo, e2n[i], self._region_ids[i], self.adjacency(i),
                    self._boundary_map.get(i, {}))

    @property
    def cells(self):
        for i in range(self.n_cells):
            yield self.get_cell(i)

    def cells_on_boundary(self, name):
        bid = self._boundary_id_lookup[name]
        for i in sorted(self._boundary_cells[bid]):
            yield self.get_cell(i)

    def _compute_cell_centroids(self):
        e2n = self.element_map()
        geo = self._geometries[self._geom_ids[0]]
        v = e2n.reshape(e2n.shape[0], -1)[:, geo.vertex_node_ind]
        self._centroids = self.nodes[:, v].mean(axis=2).T

    def _permute_nodes(self, perm):
        """New node k is old node perm[k] (sem/discrete.py:1115-1127)."""
        perm = np.asarray(perm)
        self.nodes[:, :perm.size] = self.nodes[:, perm]
        inv = np.zeros_like(perm)
        inv[perm] = np.arange(perm.size, dtype=perm.dtype)
        e2n = self.element_map()
        e2n[...] = inv[e2n]
        self.version += 1


# ---------------------------------------------------------------------------
def _pair_graph(maps, n):
    """Boolean CSR graph with an edge between every two nodes of a cell."""
    E, k = maps.shape
    rows, cols = [], []
    for s in range(0, E, _CELL_CHUNK):
        m = maps[s:s + _CELL_CHUNK].astype(np.int64)
        rows.append(np.repeat(m, k, axis=1).ravel())
        cols.append(np.tile(m, (1, k)).ravel())
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    g = sparse.coo_matrix((np.ones(r.size, dtype=bool), (r, c)), shape=(n, n))
    return g.tocsr()


def rcm_permutation(maps, n):
    """scipy.sparse.csgraph.reverse_cuthill_mckee(_pair_graph(maps, n), True)
    without the pair graph (sem_node_degrees / sem_cuthill_mckee in
    libsem_hip.so walk the cell map; the graph has sum_cells nloc^2 entries
    and no longer fits a host at 1024^2 cells of order 8).  Degree ties are
    broken by numpy's argsort, as scipy does; equal to scipy's permutation
    (tests/test_order.py).  Without the built library (host-only use of
    DOFManager) scipy's RCM of the pair graph gives the same permutation."""
    import ctypes as C
    from . import _lib
    try:
        lib = _lib.load()
    except (ImportError, OSError):
        from scipy.sparse import csgraph
        return csgraph.reverse_cuthill_mckee(_pair_graph(np.asarray(maps), n), True)
    cells = np.ascontiguousarray(maps, dtype=np.uint32)
    E, k = cells.shape
    deg = np.empty(n, dtype=np.int32)
    _lib.check(lib.sem_node_degrees(cells.ctypes.data_as(C.c_void_p), E, k, n,
                                    deg.ctypes.data_as(C.c_void_p)))
    seeds = np.argsort(deg).astype(np.int64)
    order = np.empty(n, dtype=np.int64)
    _lib.check(lib.sem_cuthill_mckee(cells.ctypes.data_as(C.c_void_p), E, k, n,
                                     deg.ctypes.data_as(C.c_void_p),
                                     seeds.ctypes.data_as(C.c_void_p),
                                     order.ctypes.data_as(C.c_void_p)))
    return order[::-1].astype(np.int32)


class DOFManager(object):
    """Degrees of freedom on a mesh (sem/discrete.py:44-280) plus the
    batched device operator path."""

    _compute_flag_keys = {"x_phys", "Jacobian"}
    default_compute_flags = dict.fromkeys(_compute_flag_keys, False)

    def __init__(self, mesh, dofs_per_node=1, basis=None, mapping_basis=None, rcm_order=True,
                 device=None):
        self._mesh = mesh
        self._dpn = dofs_per_node
        self._mesh._compute_cell_centroids()
        self._basis = basis
        self._map_basis = basis if mapping_basis is None else mapping_basis
        self._device = device
        self._op = None
        self._op_version = None
        self._fields = None
        if rcm_order:
            self._reorder_nodes_rcm()

    @property
    def ndof_per_node(self):
        return self._dpn

    @property
    def ndof(self):
        return self._dpn * self._mesh.n_nodes

    @property
    def mesh(self):
        return self._mesh

    @property
    def basis(self):
        return self._basis

    def _resolve_cmpflag_dependencies(self, compute_flags):
        bad = set(compute_flags) - self._compute_flag_keys
        if bad:
            raise ValueError("Unrecognized flags {}.".format(bad))
        for flag, default in self.default_compute_flags.items():
            compute_flags.setdefault(flag, default)
        if compute_flags["Jacobian"]:
            compute_flags["x_phys"] = True

    def _get_connectivity_graph(self):
        e2n = self._mesh.element_map()
        return _pair_graph(e2n.reshape(e2n.shape[0], -1), self._mesh.n_nodes)

    def _reorder_nodes_rcm(self):
        """Reverse Cuthill-McKee node order (sem/discrete.py:169-178), the
        graph walked on the cell map natively (rcm_permutation)."""
        e2n = self._mesh.element_map()
        self._mesh._permute_nodes(rcm_permutation(e2n.reshape(e2n.shape[0], -1),
                                                  self._mesh.n_nodes))

    # ------------------------------------------------------------------ device
    def operator(self):
        """The device operator context for this mesh and basis."""
        from .operators import SEMOperator
        if self._basis is None:
            raise ValueError("Basis must be initialized")
        if self._map_basis is not self._basis and \
                self._map_basis.coeff_shape != self._basis.coeff_shape:
            raise NotImplementedError("only isoparametric mappings are supported on the device")
        if self._op is None or self._op_version != self._mesh.version:
            p = self._basis.coeff_shape[0] - 1
            self._op = SEMOperator(p, self._mesh.element_map(), self._mesh.nodes,
                                   dofs_per_node=self._dpn, basis=self._basis,
                                   device=self._device)
            self._op_version = self._mesh.version
            self._fields = None
        return self._op

    def stiffness_action(self, u, out=None, accumulate=False):
        """Global Poisson stiffness action K u (matrix-free, one launch):
        the loop examples/poisson.py:168-193 + einsum('pqrs,rs') + scatter."""
        return self.operator().apply(u, out=out, kind="poisson", accumulate=accumulate)

    def operator_action(self, kind, u, out=None, accumulate=False):
        """Global action of ``kind`` ('poisson' or 'axisym_stokes')."""
        return self.operator().apply(u, out=out, kind=kind, accumulate=accumulate)

    def geometry_fields(self):
        """Host copies of x_phys, J, invJ, detJ, detJxW for every cell."""
        op = self.operator()
        if self._fields is None:
            f = op.geometry_fields()
            self._fields = {k: v.cpu().numpy() for k, v in f.items()}
        return self._fields

    # ------------------------------------------------------------------ reference API
    def get_finite_element(self, i, **compute_flags):
        self._resolve_cmpflag_dependencies(compute_flags)
        return FiniteElement(self, self._mesh.get_cell(i), compute_flags, i)

    def finite_elements(self, **compute_flags):
        """Iterate over all finite elements (sem/discrete.py:189-209); the
        geometry of all cells is computed once on the device."""
        self._resolve_cmpflag_dependencies(compute_flags)
        for i in range(self._mesh.n_cells):
            yield FiniteElement(self, self._mesh.get_cell(i), compute_flags, i)

    def boundary_elements(self, name, **compute_flags):
        raise NotImplementedError("boundary sub-elements (sem/discrete.py:211-219) are out of "
                                  "scope for the operator engine")

    def values_at_nodes(self, coeffs):
        """Values at the equispaced element nodes (sem/discrete.py:235-258),
        all cells in one device launch."""
        e2n = self._mesh.element_map()
        coeffs = np.asarray(coeffs, dtype=np.float64)
        vals = np.empty_like(coeffs)
        loc = coeffs[..., e2n]
        out = self._basis.interpolate_on_grid_eq(loc)
        vals[..., e2n] = out
        return vals

    def interpolate(self, coeffs, x_phys):
        raise NotImplementedError("point location (sem/discrete.py:221-233) is out of scope")

    def find_elem_containing_point(self, point):
        raise NotImplementedError("point location (sem/discrete.py:263-280) is out of scope")


def band_order(A):
    """Reverse Cuthill-McKee order of a square sparse matrix (on the
    symmetrised pattern) and its lower / upper bandwidths in that order:
    (perm, A[perm][:, perm] as CSR, kl, ku)."""
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    A = sparse.csr_matrix(A)
    pat = (abs(A) + abs(A.T)).tocsr()
    perm = np.asarray(reverse_cuthill_mckee(pat, symmetric_mode=True), dtype=np.int64)
    Ap = A[perm][:, perm].tocoo()
    kl = int(max(0, (Ap.row - Ap.col).max(initial=0)))
    ku = int(max(0, (Ap.col - Ap.row).max(initial=0)))
    return perm, Ap.tocsr(), kl, ku


def band_lu_solve(A, b, device):
    """x = A^-1 b for a square sparse matrix on the device: reverse
    Cuthill-McKee order (host, scipy.sparse.csgraph, as the reference orders
    its nodes: sem/discrete.py:169-178), then banded LU with partial pivoting
    (sem_band_lu_solve).  Stands in for the reference's
    scipy.sparse.linalg.spsolve (sem/discrete.py:511): a singular matrix
    gives a MatrixRankWarning and a NaN solution, as there."""
    import ctypes as C
    import warnings
    import torch
    from . import _lib
    A = sparse.csr_matrix(A)
    n = A.shape[0]
    if n == 0:
        return np.zeros(0)
    perm, Ap, kl, ku = band_order(A)
    lib = _lib.load()
    rp = torch.from_numpy(Ap.indptr.astype(np.int64)).to(device)
    ci = torch.from_numpy(Ap.indices.astype(np.int32)).to(device)
    va = torch.from_numpy(Ap.data.astype(np.float64)).to(device)
    bp = torch.from_numpy(np.ascontiguousarray(np.asarray(b, dtype=np.float64)[perm])).to(device)
    xp = torch.empty(n, dtype=torch.float64, device=device)
    info = C.c_int(0)
    with torch.cuda.device(device):
        _lib.check(lib.sem_band_lu_solve(n, kl, ku, _lib.tptr(rp), _lib.tptr(ci), _lib.tptr(va),
                                         _lib.tptr(bp), _lib.tptr(xp), C.byref(info),
                                         _lib.stream_ptr()))
    x = np.empty(n)
    if info.value:
        from scipy.sparse.linalg import MatrixRankWarning
        warnings.warn("Matrix is exactly singular", MatrixRankWarning, stacklevel=3)
        x.fill(np.nan)
        return x
    x[perm] = xp.cpu().numpy()
    return x


class DOFManagerSC(DOFManager):
    """DOFs ordered for static condensation: element-exterior nodes first
    (sem/discrete.py:283-528)."""

    @property
    def ndof_exterior(self):
        return self._mesh.n_nodes_cell_exterior * self._dpn

    @property
    def ndof_interior(self):
        return self._mesh.n_nodes_cell_interior * self._dpn

    def __init__(self, mesh, dofs_per_node=1, basis=None, mapping_basis=None, rcm_order=True,
                 device=None):
        super(DOFManagerSC, self).__init__(mesh, dofs_per_node, basis, mapping_basis,
                                           rcm_order=False, device=device)
        self._do_static_condensation()
        if rcm_order:
            self._reorder_nodes_rcm()

    def _do_static_condensation(self):
        """Exterior nodes (sorted) first, then interior (sorted)
        (sem/discrete.py:314-359)."""
        mesh = self._mesh
        e2n = mesh.element_map()
        geo = mesh._geometries[mesh._geom_ids[0]]
        flat = e2n.reshape(e2n.shape[0], -1)
        ext = np.unique(flat[:, geo.exterior_node_ind])
        itr = np.sort(flat[:, geo.interior_node_ind].ravel())
        ix_map = np.concatenate((ext, itr)).astype(np.int64)
        assert ix_map.size == mesh.n_nodes
        mesh._permute_nodes(ix_map)
        mesh.n_nodes_cell_exterior = ext.size
        mesh.n_nodes_cell_interior = itr.size
        mesh.condensed = True

    def _get_connectivity_graph(self):
        e2n = self._mesh.element_map()
        geo = self._mesh._geometries[self._mesh._geom_ids[0]]
        ext = e2n.reshape(e2n.shape[0], -1)[:, geo.exterior_node_ind]
        return _pair_graph(ext, self._mesh.n_nodes_cell_exterior)

    def _reorder_nodes_rcm(self):
        """RCM on the exterior graph only (sem/discrete.py:389-402)."""
        mesh = self._mesh
        n_ext = mesh.n_nodes_cell_exterior
        perm = np.empty(mesh.n_nodes, np.uint32)
        e2n = mesh.element_map()
        geo = mesh._geometries[mesh._geom_ids[0]]
        perm[:n_ext] = rcm_permutation(e2n.reshape(e2n.shape[0], -1)[:, geo.exterior_node_ind],
                                       n_ext)
        perm[n_ext:] = np.arange(n_ext, mesh.n_nodes)
        mesh._permute_nodes(perm)

    # -------------------------------------------------- static condensation
    # The reference's API (sem/discrete.py:404-528), same names, arguments and
    # results; the per-element dense linear algebra runs as one batched device
    # launch (csrc/sem_sc.hip) instead of a Python loop of scipy.linalg.solve.
    def _cell_dofs_hier(self):
        """Global DOFs of every cell in hierarchical order (exterior first):
        FiniteElement.global_dof_ind_hier for all cells, [E, n_nodes * dpn]."""
        mesh = self._mesh
        geo = mesh._geometries[mesh._geom_ids[0]]
        e2n = mesh.element_map()
        h = geo.hierarchical_node_order
        nodes = e2n.reshape(e2n.shape[0], -1)[:, h].astype(np.int64)
        dpn = self._dpn
        return (nodes[:, :, None] * dpn + np.arange(dpn)[None, None, :]).reshape(
            nodes.shape[0], -1), geo.n_exterior_nodes * dpn

    def init_global_linear_system(self):
        """Zero COO matrix over the element-exterior DOFs and a zero RHS
        (sem/discrete.py:404-426)."""
        _, ne = self._cell_dofs_hier()
        n_mat_entries = self._mesh.n_cells * ne ** 2
        row_col = np.zeros((2, n_mat_entries), dtype=np.uint32)
        entries = np.zeros(n_mat_entries, dtype=np.float64)
        ndof_ext = self.ndof_exterior
        return Static_COO_Matrix(entries, row_col, (ndof_ext, ndof_ext)), \
            np.zeros(ndof_ext, dtype=np.float64)

    @staticmethod
    def reorder_local_system_hier(fe, local_system):
        """Lexicographic local system -> hierarchical DOF order, exterior
        first (sem/discrete.py:428-436)."""
        lmat, lrhs = local_system
        hier = fe.loc_dof_ind_hier
        return lmat[np.ix_(hier, hier)], lrhs[hier]

    @staticmethod
    def compute_local_sc_system(fe, local_system):
        """Schur complement system of one element's hierarchical local system
        (sem/discrete.py:438-472), on the device."""
        S, s, _ = _schur_batched([local_system], fe.ndof_exterior)
        return S[0].cpu().numpy(), s[0].cpu().numpy()

    def assemble_global_sc_system(self, global_sc_system, local_systems):
        """Element Schur complements of all local systems (one batched
        device launch) assembled into the COO system from
        init_global_linear_system (sem/discrete.py:474-500)."""
        gmat, grhs = global_sc_system
        dofs, ne = self._cell_dofs_hier()
        local_systems = list(local_systems) if not isinstance(local_systems, list) \
            else local_systems
        S, s, work = _schur_batched(local_systems, ne, self._device)
        ext = dofs[:, :ne]
        E = ext.shape[0]
        gmat.row[:] = np.repeat(ext, ne, axis=1).ravel()
        gmat.col[:] = np.tile(ext, (1, ne)).ravel()
        gmat.data[:] = S.reshape(E, -1).cpu().numpy().ravel()
        grhs += np.bincount(ext.ravel(), weights=s.cpu().numpy().ravel(), minlength=grhs.size)
        self._sc_state = (local_systems, local_systems[0] if local_systems else None, work, ne)

    def _solve_boundary_dofs(self, global_sc_system, dof_vec, on_ebc, rtol=1e-13):
        """Solve the condensed exterior system with the essential BCs
        (sem/discrete.py:502-510).  Symmetric systems (Poisson): Jacobi-PCG on
        the device over the assembled CSR matrix; otherwise (the axisymmetric
        Stokes / Navier-Stokes block) a direct solve like the reference's
        spsolve: banded LU with partial pivoting on the device, the unknowns
        ordered by reverse Cuthill-McKee (sem_band_lu_solve)."""
        import torch
        from . import _lib
        sc_mat, sc_rhs = global_sc_system
        is_unk = ~np.asarray(on_ebc, dtype=bool)
        n = self.ndof_exterior
        ext_dofs = dof_vec[:n]
        A = sparse.coo_matrix((sc_mat.data, (sc_mat.row, sc_mat.col)), shape=(n, n)).tocsr()
        A.sum_duplicates()
        asym = abs(A - A.T)
        if asym.nnz == 0 or asym.max() <= 1e-12 * abs(A).max():
            dev = self.operator().device
            lib = _lib.load()
            rp = torch.from_numpy(A.indptr.astype(np.int64)).to(dev)
            ci = torch.from_numpy(A.indices.astype(np.int32)).to(dev)
            va = torch.from_numpy(A.data.astype(np.float64)).to(dev)
            b = torch.from_numpy(np.asarray(sc_rhs, dtype=np.float64)).to(dev)
            x = torch.from_numpy(np.where(is_unk, 0.0, ext_dofs)).to(dev)
            mask = torch.from_numpy((~is_unk).astype(np.uint8)).to(dev)
            import ctypes as C
            its, rel = C.c_int(0), C.c_double(0.0)
            with torch.cuda.device(dev):
                _lib.check(lib.sem_csr_pcg_solve(n, _lib.tptr(rp), _lib.tptr(ci), _lib.tptr(va),
                                                 _lib.tptr(b), _lib.tptr(x), _lib.tptr(mask),
                                                 float(rtol), 100000, C.byref(its), C.byref(rel),
                                                 dev.index, _lib.stream_ptr()))
            ext_dofs[is_unk] = x.cpu().numpy()[is_unk]
            return its.value, rel.value
        A1 = A[is_unk]
        rhs1 = sc_rhs[is_unk] - A1[:, ~is_unk].dot(ext_dofs[~is_unk])
        ext_dofs[is_unk] = band_lu_solve(A1[:, is_unk], rhs1, self.operator().device)
        return None, None

    def _solve_interior_dofs(self, local_systems, dof_vec):
        """Interior DOFs of every element from its exterior DOFs
        (sem/discrete.py:512-524), one batched device launch reusing the
        eliminations of assemble_global_sc_system."""
        import torch
        from . import _lib
        dofs, ne = self._cell_dofs_hier()
        st = getattr(self, "_sc_state", None)
        if st is None or st[0] is not local_systems or \
                (local_systems and st[1] is not local_systems[0]):
            _, _, work = _schur_batched(list(local_systems), ne, self._device)
        else:
            work = st[2]
        E, nl = dofs.shape
        if nl == ne:
            return
        xe = torch.from_numpy(np.ascontiguousarray(dof_vec[dofs[:, :ne]])).to(work.device)
        xi = torch.empty(E, nl - ne, dtype=torch.float64, device=work.device)
        lib = _lib.load()
        with torch.cuda.device(work.device):
            _lib.check(lib.sem_schur_backsolve(E, nl, ne, _lib.tptr(work), _lib.tptr(xe),
                                               _lib.tptr(xi), _lib.stream_ptr()))
        dof_vec[dofs[:, ne:]] = xi.cpu().numpy()

    def solve(self, global_sc_system, local_systems, dof_vec, on_ebc):
        """Static-condensation solve (sem/discrete.py:526-528): exterior DOFs
        from the condensed system, then the element interiors; dof_vec
        holds the essential BC values on entry and the solution on exit."""
        self._solve_boundary_dofs(global_sc_system, dof_vec, on_ebc)
        self._solve_interior_dofs(local_systems, dof_vec)

    def solve_poisson(self, rhs, dof_vec, on_ebc, rtol=1e-13, max_iter=20000):
        """Assembled Poisson solve K u = rhs with essential BCs: the result of
        DOFManagerSC.solve (sem/discrete.py:502-528) computed matrix-free with
        Jacobi-PCG on the GPU.  ``dof_vec`` holds the EBC values (updated in
        place); ``on_ebc`` masks the exterior DOFs (reference convention) or
        all DOFs.  Returns (dof_vec, iterations, relative residual)."""
        import torch
        if self._dpn != 1:
            raise NotImplementedError("solve_poisson: scalar problems (dofs_per_node == 1)")
        mask = np.zeros(self.ndof, dtype=bool)
        on_ebc = np.asarray(on_ebc, dtype=bool)
        mask[:on_ebc.size] = on_ebc
        op = self.operator()
        x = torch.from_numpy(np.where(mask, dof_vec, 0.0)).to(op.device)
        b = torch.from_numpy(np.asarray(rhs, dtype=np.float64)).to(op.device)
        x, its, rel = op.pcg_solve(b, x, mask, rtol=rtol, max_iter=max_iter)
        dof_vec[...] = x.cpu().numpy()
        return dof_vec, its, rel


def _schur_batched(local_systems, ne, device=None):
    """Device Schur complements of hierarchical local systems (list of
    (lmat [nl, nl], lrhs [nl])): returns S [E, ne, ne], s [E, ne] and the
    elimination workspace (A_ii^-1 [A_ie | b_i]) as device tensors."""
    import ctypes as C
    import torch
    from . import _lib
    from .operators import _device_index
    dev = torch.device("cuda", _device_index(device))
    mats = torch.from_numpy(np.ascontiguousarray(
        np.stack([np.asarray(m, dtype=np.float64) for m, _ in local_systems]))).to(dev)
    rhs = torch.from_numpy(np.ascontiguousarray(
        np.stack([np.asarray(r, dtype=np.float64) for _, r in local_systems]))).to(dev)
    E, nl = rhs.shape
    if mats.shape != (E, nl, nl) or not (0 <= ne <= nl):
        raise ValueError("local systems must be [nl, nl] matrices and [nl] vectors")
    S = torch.empty(E, ne, ne, dtype=torch.float64, device=dev)
    s = torch.empty(E, ne, dtype=torch.float64, device=dev)
    work = torch.empty(E, max(nl - ne, 1), nl + 1, dtype=torch.float64, device=dev)
    bad = C.c_int64(0)
    lib = _lib.load()
    with torch.cuda.device(dev):
        rc = lib.sem_schur_batched(E, nl, ne, _lib.tptr(mats), _lib.tptr(rhs), _lib.tptr(work),
                                   _lib.tptr(S), _lib.tptr(s), C.byref(bad), _lib.stream_ptr())
    if rc == _lib.SEM_E_INVALID and bad.value:
        raise np.linalg.LinAlgError("Singular matrix (%d elements)" % bad.value)
    _lib.check(rc)
    return S, s, work


class FiniteElement(object):
    """One element of a DOFManager (sem/discrete.py:531-705)."""

    def __init__(self, dof_mngr, cell, compute_flags, index):
        self._cell = cell
        self._dpn = dof_mngr._dpn
        self._basis = dof_mngr._basis
        self._quad_rule = self._basis.quad_rule
        self._cmpflags = compute_flags
        self._index = index
        fields = dof_mngr.geometry_fields() if compute_flags.get("x_phys") else {}
        self._mapping = Mapping(dof_mngr._map_basis, fields, index, compute_flags)
        self._l_dof_ind_hier, self._g_dof_ind_hier = self._compute_hier_dofs()

    def _compute_hier_dofs(self):
        dpn = self._dpn
        lh = self._cell.geometry.hierarchical_node_order
        gh = self._cell.node_ind_hierarchical
        ld = (dpn * lh[:, None].astype(np.uint32) + np.arange(dpn, dtype=np.uint32)).ravel()
        gd = (dpn * gh[:, None].astype(np.uint32) + np.arange(dpn, dtype=np.uint32)).ravel()
        return ld.astype(np.uint32), gd.astype(np.uint32)

    @property
    def ndim(self):
        return self._basis.ndim

    @property
    def x_phys(self):
        return self._mapping.x_phys

    @property
    def J(self):
        return self._mapping.J

    @property
    def invJ(self):
        return self._mapping.invJ

    @property
    def detJxW(self):
        return self._mapping._get("detJxW", "Jacobian")

    @property
    def ndof(self):
        return self.n_nodes * self._dpn

    @property
    def ndof_exterior(self):
        return self.n_exterior_nodes * self._dpn

    @property
    def ndof_interior(self):
        return self.n_interior_nodes * self._dpn

    @property
    def loc_dof_ind_hier(self):
        return self._l_dof_ind_hier

    @property
    def global_dof_ind_hier(self):
        return self._g_dof_ind_hier

    @property
    def exterior_dof_ind(self):
        return self._g_dof_ind_hier[:self.ndof_exterior]

    @property
    def interior_dof_ind(self):
        return self._g_dof_ind_hier[self.ndof_exterior:]

    @property
    def n_nodes(self):
        return self._cell.n_nodes

    @property
    def n_exterior_nodes(self):
        return self._cell.n_exterior_nodes

    @property
    def n_interior_nodes(self):
        return self._cell.n_interior_nodes

    @property
    def basis(self):
        return self._basis

    @property
    def mapping(self):
        return self._mapping

    @property
    def quadrature(self):
        return self._quad_rule

    @property
    def node_ind(self):
        return self._cell.node_ind_lexicographic

    def local(self, arr):
        return arr[self.node_ind]

    def gradient(self, coeffs):
        """Physical gradient invJ^T . grad_xi (sem/discrete.py:680-684);
        the reference-coordinate gradient runs on the device."""
        g = np.asarray(self._basis.gradient(np.asarray(coeffs, dtype=np.float64)))
        return np.einsum("ij...,i...->j...", self.invJ, g)

    def deriv(self, coeffs, dim):
        g = np.asarray(self._basis.gradient(np.asarray(coeffs, dtype=np.float64)))
        return np.einsum("i...,i...", self.invJ[:, dim], g)

    def integrate(self, coeffs):
        return (coeffs * self.detJxW).sum()

    def values_at_nodes(self, coeffs):
        return self._basis.interpolate_on_grid_eq(coeffs)
