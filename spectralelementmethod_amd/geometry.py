"""Cell geometries and their node orderings (host-side setup).

Mirror of sem/geometry.py: ``NCube`` (:32-216), ``Line`` (:219-236) and
``Quadrilateral`` (:239-259).  Only the orderings the operator path needs are
here: lexicographic shape, vertex / exterior / interior node sets and the
hierarchical order (vertices, then each edge's interior, then the cell
interior; sem/geometry.py:197-212) used by static condensation
(sem/discrete.py:561-576).
"""
import itertools as itt
from math import comb

import numpy as np


class Geometry(object):
    pass


class NCube(Geometry):
    """Orthotope cell with ``shape`` nodes per direction."""

    @property
    def ndim(self):
        return len(self._shape)

    @property
    def shape(self):
        return self._shape

    @property
    def n_nodes(self):
        return self._n_nodes

    @property
    def n_exterior_nodes(self):
        return self._n_exterior_nodes

    @property
    def n_interior_nodes(self):
        return self._n_interior_nodes

    @property
    def vertex_node_ind(self):
        return self._hier_node_order[:2 ** self.ndim]

    @property
    def hierarchical_node_order(self):
        return self._hier_node_order

    @property
    def exterior_node_ind(self):
        return self._hier_node_order[:self._n_exterior_nodes]

    @property
    def interior_node_ind(self):
        return self._hier_node_order[self._n_exterior_nodes:]

    @property
    def nodes(self):
        return self._node_locations

    def __init__(self, *shape):
        if not all(isinstance(s, (int, np.integer)) and s > 0 for s in shape):
            raise ValueError("shape entries must be positive integers")
        self._shape = tuple(int(s) for s in shape)
        self._n_nodes = int(np.prod(self._shape))
        self._n_interior_nodes = int(np.prod([max(s - 2, 0) for s in self._shape]))
        self._n_exterior_nodes = self._n_nodes - self._n_interior_nodes
        self._node_locations = np.meshgrid(*(np.linspace(-1, 1, s) for s in self._shape),
                                           indexing="ij", sparse=True)
        self._hier_node_order = self._compute_hierarchical_node_ordering()
        self._sub_geo_class = NCube

    def n_sub_geometries(self, dim=-1):
        """Number of dim-dimensional boundary pieces: 2^(n-dim) C(n, dim)."""
        if dim < 0:
            dim = self.ndim + dim
        if dim > self.ndim or dim < 0:
            raise ValueError("No {}D sub-geometry in a {}D parent geometry".format(dim, self.ndim))
        n = self.ndim
        return 2 ** (n - dim) * comb(n, dim)

    def sub_geometry_ix_exps(self, dim=None, inclusive=True):
        """Index expressions of every dim-dimensional piece: fixed axes in
        itertools.combinations order, each fixed at its first / last index
        (itertools.product order); free axes full (inclusive) or interior."""
        if dim is None:
            dim = self.ndim - 1
        if dim > self.ndim or dim < 0:
            raise ValueError("No {}D sub-geometry on a {}D parent geometry".format(dim, self.ndim))
        out = []
        for fixed in itt.combinations(range(self.ndim), self.ndim - dim):
            for consts in itt.product(*[(0, self._shape[a] - 1) for a in fixed]):
                idx, shp = [], []
                cmap = dict(zip(fixed, consts))
                for d in range(self.ndim):
                    if d in cmap:
                        idx.append(cmap[d])
                    elif inclusive:
                        idx.append(slice(0, self._shape[d]))
                        shp.append(self._shape[d])
                    else:
                        idx.append(slice(1, self._shape[d] - 1))
                        shp.append(self._shape[d] - 2)
                out.append((tuple(shp), tuple(idx)))
        return out

    def _compute_hierarchical_node_ordering(self):
        lin = np.arange(self._n_nodes).reshape(self._shape)
        parts = [np.atleast_1d(lin[ix]).ravel() for _, ix in self.sub_geometry_ix_exps(0, False)]
        for d in range(1, self.ndim + 1):
            parts.extend(lin[ix].ravel() for _, ix in self.sub_geometry_ix_exps(d, False))
        order = np.concatenate(parts).astype(np.uint32)
        assert order.size == self._n_nodes
        return order

    def sub_geometry(self, axis):
        return self._sub_geo_class(*(self._shape[axis + 1:] + self._shape[:axis]))


class Line(NCube):
    corner_verts = [np.array([True, False]), np.array([False, True])]

    @property
    def ndim(self):
        return 1

    def __init__(self, shape_u):
        NCube.__init__(self, shape_u)
        self._sub_geo_class = None

    def sub_geometry(self, axis=0):
        raise NotImplementedError("The sub-geometry of a line is a single point.")


class Quadrilateral(NCube):
    """Vertex/edge enumeration as sem/geometry.py:245-255."""

    corner_verts = [np.array([1, 1, 0, 0], dtype=bool), np.array([0, 0, 1, 1], dtype=bool),
                    np.array([1, 0, 1, 0], dtype=bool), np.array([0, 1, 0, 1], dtype=bool)]

    @property
    def ndim(self):
        return 2

    def __init__(self, shape_u, shape_v):
        NCube.__init__(self, shape_u, shape_v)
        self._sub_geo_class = Line
