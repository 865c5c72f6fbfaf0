"""Gmsh 2.2 binary ``.msh`` reader and a writer for
synthetic meshes.

Reader: ``load_msh(file_path, ndim)`` mirrors sem/grid_importers.py:45-68 --
same sections, the same format checks and exceptions (``FileFormatError``;
ASCII files raise ``NotImplementedError``), the same node renumbering to
0-based ids, the same Gmsh -> lexicographic reorder of each cell's nodes
(:273-332), the same regions / boundaries (:104-133) and the same cell
adjacency and boundary-side bookkeeping (:221-270).  What differs is the
work: element blocks are decoded and reordered as whole arrays (one gather
per block instead of a Python loop per cell), and neighbours are found by
hashing vertex pairs instead of the reference's O(E^2) centroid-distance
search (:221-270); for a conforming mesh both produce the same adjacency, and
boundary sides are recorded in the reference's order (closest boundary cell
first).  The result is a ``discrete.Mesh`` whose element map feeds the device
operators directly.

Writer: ``write_msh`` produces binary 2.2 files (quadrilateral cells of any
supported order, tagged boundary lines) -- the inverse of the reader's
reorder -- so synthetic meshes can take the reference's file path (no
``.msh`` file is bundled with the reference and gmsh is not installed).
"""
import struct

import numpy as np

from . import discrete
from .geometry import Line, Quadrilateral


class FileFormatError(Exception):
    """Raised when a mesh file does not follow the Gmsh 2.2 layout
    (sem/grid_importers.py:9-12)."""


# Gmsh element type -> cell geometry (sem/grid_importers.py:19-42)
LINE_TYPES = {1: 2, 8: 3, 26: 4, 27: 5, 28: 6, 62: 7, 63: 8, 64: 9, 65: 10, 66: 11}
QUAD_TYPES = {3: 2, 10: 3, 36: 4, 37: 5, 38: 6, 47: 7, 48: 8, 49: 9, 50: 10, 51: 11}
construct_geometry = dict(
    [(t, (lambda n: (lambda: Line(n)))(n)) for t, n in LINE_TYPES.items()] +
    [(t, (lambda n: (lambda: Quadrilateral(n, n)))(n)) for t, n in QUAD_TYPES.items()])
_TYPE_OF_QUAD = {n: t for t, n in QUAD_TYPES.items()}
_TYPE_OF_LINE = {n: t for t, n in LINE_TYPES.items()}


def gmsh_to_lexicographic(shape):
    """Index map of _convert_ix_order_to_lexicographic (sem/grid_importers.py:
    273-332): lexicographic entry k of a cell is Gmsh entry idxmap.flat[k].
    Gmsh numbers vertices first, then edges counter-clockwise, then the
    interior recursively."""
    if len(shape) == 0:
        return np.zeros((), dtype=np.int64)
    if len(shape) == 1:
        M, N = shape[0], 1
    elif len(shape) == 2:
        M, N = shape
    else:
        raise NotImplementedError("Can only take 2 arguments for now...")
    idxmap = np.zeros((M, N), dtype=np.int64)
    k = 0
    ring = 0
    while ring < min(M, N) // 2:
        lo, hi = ring, -ring - 1
        idxmap[lo, lo], idxmap[hi, lo], idxmap[hi, hi], idxmap[lo, hi] = k, k + 1, k + 2, k + 3
        k += 4
        p_ns = M - 2 * (ring + 1)       # south edge, increasing
        idxmap[lo + 1:hi, lo] = np.arange(k, k + p_ns)
        k += p_ns
        p_ew = N - 2 * (ring + 1)       # east edge, increasing
        idxmap[hi, lo + 1:hi] = np.arange(k, k + p_ew)
        k += p_ew
        idxmap[lo + 1:hi, hi] = np.arange(k + p_ns - 1, k - 1, -1)   # north, decreasing
        k += p_ns
        idxmap[lo, lo + 1:hi] = np.arange(k + p_ew - 1, k - 1, -1)   # west, decreasing
        k += p_ew
        ring += 1
    if (M % 2 or N % 2) and min(M, N) != 2:
        lo, hi = ring, -ring - 1
        if M > N:      # a line of nodes on the horizontal centre line
            idxmap[lo, lo], idxmap[hi, lo] = k, k + 1
            k += 2
            idxmap[lo + 1:hi, lo] = np.arange(k, M * N)
        elif M < N:    # ... on the vertical centre line
            idxmap[lo, lo], idxmap[lo, hi] = k, k + 1
            k += 2
            idxmap[lo, lo + 1:hi] = np.arange(k, M * N)
        else:          # the single centre node
            idxmap[lo, lo] = M * N - 1
    return idxmap.squeeze()


class _Reader(object):
    def __init__(self, data):
        self.data = data
        self.pos = 0

    def readline(self):
        end = self.data.find(b"\n", self.pos)
        end = len(self.data) if end < 0 else end + 1
        line = self.data[self.pos:end]
        self.pos = end
        return line

    def take(self, dtype, count):
        dtype = np.dtype(dtype)
        nbytes = dtype.itemsize * count
        if self.pos + nbytes > len(self.data):
            raise FileFormatError("Unexpected end of binary data")
        out = np.frombuffer(self.data, dtype, count, self.pos)
        self.pos += nbytes
        return out


def parse_format(f):
    """$MeshFormat: version 2.2, binary flag, data size 8
    (sem/grid_importers.py:71-101).  Returns is_binary."""
    if not f.readline().startswith(b"$MeshFormat"):
        raise FileFormatError("Expected 'MeshFormat' data")
    version, is_binary, data_size = f.readline().split()
    if version != b"2.2":
        raise FileFormatError("Expected Gmsh file format version 2.2, but got {} instead"
                              .format(version.decode("utf-8")))
    if is_binary not in (b"0", b"1"):
        raise FileFormatError("Unable to recognize file format")
    is_binary = bool(int(is_binary))
    if data_size != b"8":
        raise FileFormatError("Expected a data size of 8, but got {} instead"
                              .format(data_size.decode("utf-8")))
    if is_binary:
        f.readline()  # the binary int 1 (endianness marker)
    if not f.readline().startswith(b"$EndMeshFormat"):
        raise FileFormatError("Malformed mesh format specification")
    return is_binary


def parse_physical_names(f, mesh):
    """$PhysicalNames (sem/grid_importers.py:104-133): ndim-dimensional names
    become regions, lower-dimensional ones boundaries.  Returns the maps
    physical id -> region id / boundary id."""
    if not f.readline().startswith(b"$PhysicalNames"):
        raise FileFormatError("Expected 'PhysicalNames' data")
    n_phys = int(f.readline().rstrip())
    region_id_map, boundary_id_map = {}, {}
    for i in range(n_phys):
        parts = f.readline().split()
        dim, phys_id = int(parts[0]), int(parts[1]) - 1
        if phys_id != i:
            raise FileFormatError("physical ids must be numbered consecutively from 1")
        name = parts[2].strip(b'"').decode("utf-8")
        if dim == mesh.ndim:
            region_id_map[phys_id] = mesh.new_region(name)
        elif dim < mesh.ndim:
            boundary_id_map[phys_id] = mesh.new_boundary(name)
    if not f.readline().startswith(b"$EndPhysicalNames"):
        raise FileFormatError("Wrong number of physical names specifed")
    return region_id_map, boundary_id_map


def parse_nodes_bin(f, mesh):
    """$Nodes, binary (sem/grid_importers.py:136-156)."""
    if not f.readline().startswith(b"$Nodes"):
        raise FileFormatError("Expected 'Nodes' data")
    n_nodes = int(f.readline().rstrip())
    rec = f.take(np.dtype([("index", "<i4"), ("coord", "<f8", 3)]), n_nodes)
    f.readline()
    if not f.readline().startswith(b"$EndNodes"):
        raise FileFormatError("Expected end of 'Nodes' data")
    if not np.array_equal(rec["index"], np.arange(1, n_nodes + 1)):
        raise FileFormatError("nodes must be numbered consecutively from 1")
    mesh.set_nodes(np.ascontiguousarray(rec["coord"][:, :mesh.ndim].T))


def parse_elements_bin(f, mesh, region_id_map, boundary_id_map):
    """$Elements, binary (sem/grid_importers.py:159-218).  Bulk cells go to
    the mesh (lexicographic node maps); lower-dimensional cells are returned
    as boundary cells [(boundary id, node map), ...] for the neighbour
    search."""
    if not f.readline().startswith(b"$Elements"):
        raise FileFormatError("Expected 'Elements' data")
    n_elems = int(f.readline().rstrip())
    n_read = 0
    geo_ids = {}
    bnd = []
    while n_read < n_elems:
        elem_type, n_follow, n_tags = (int(v) for v in f.take("<i4", 3))
        if elem_type not in construct_geometry:
            raise NotImplementedError("Gmsh element type %d is not supported" % elem_type)
        geometry = construct_geometry[elem_type]()
        n_nodes = geometry.n_nodes
        block = f.take("<u4", n_follow * (1 + n_tags + n_nodes)).reshape(n_follow, -1)
        if not np.array_equal(block[:, 0], np.arange(n_read + 1, n_read + n_follow + 1)):
            raise FileFormatError("elements must be numbered consecutively from 1")
        phys = block[:, 1].astype(np.int64) - 1
        idx = gmsh_to_lexicographic(geometry.shape).ravel()
        node_ix = (block[:, 1 + n_tags:].astype(np.int64) - 1)[:, idx]
        node_ix = node_ix.reshape((n_follow,) + tuple(geometry.shape)).astype(np.uint32)
        if geometry.ndim == mesh.ndim:
            if elem_type not in geo_ids:
                geo_ids[elem_type] = mesh.add_geometry(geometry)
            regions = np.array([region_id_map[int(t)] for t in phys], dtype=np.int64)
            mesh.add_cells(node_ix, geo_ids[elem_type], regions)
        elif geometry.ndim < mesh.ndim:
            for t, nm in zip(phys, node_ix):
                bnd.append((boundary_id_map[int(t)], geometry, nm))
        n_read += n_follow
    f.readline()
    if not f.readline().startswith(b"$EndElements"):
        raise FileFormatError("Expected 'Elements' data")
    return bnd


def find_cell_neighbors(mesh, bnd_cells):
    """Cell adjacency and boundary sides (sem/grid_importers.py:221-270):
    side s of cell i (Quadrilateral.corner_verts[s] selects its two vertices)
    borders the cell sharing the same two vertices, or a boundary line with
    those end points.  Boundary sides of one cell are recorded closest
    boundary-cell centroid first, as the reference's distance search does."""
    e2n = mesh.element_map()
    E = e2n.shape[0]
    geo = mesh.get_geometries()[mesh._geom_ids[0]]
    verts = e2n.reshape(E, -1)[:, geo.vertex_node_ind].astype(np.int64)   # [E, 4]
    n_sides = len(geo.corner_verts)
    sides = np.stack([np.sort(verts[:, m], axis=1) for m in geo.corner_verts], axis=1)  # [E, 4, 2]
    keys = sides[..., 0] * (np.int64(mesh.n_nodes) + 1) + sides[..., 1]
    flat = keys.ravel()
    order = np.argsort(flat, kind="stable")
    sk = flat[order]
    adj = np.full(E * n_sides, -1, dtype=np.int64)
    same = np.nonzero(sk[1:] == sk[:-1])[0]
    a, b = order[same], order[same + 1]
    adj[a] = b // n_sides
    adj[b] = a // n_sides
    mesh.set_adjacency(adj.reshape(E, n_sides))
    if not bnd_cells:
        return
    lookup = dict(zip(flat.tolist(), range(flat.size)))
    centroids = mesh.nodes[:, e2n.reshape(E, -1)].mean(axis=2).T                 # [E, ndim]
    found = {}
    for bid, bgeo, nm in bnd_cells:
        v = np.sort(nm.ravel()[bgeo.vertex_node_ind].astype(np.int64))
        key = int(v[0]) * (mesh.n_nodes + 1) + int(v[1])
        hit = lookup.get(key)
        if hit is None:
            continue
        cell, side = divmod(hit, n_sides)
        dist = float(np.linalg.norm(mesh.nodes[:, nm.ravel()].mean(axis=1) - centroids[cell]))
        found.setdefault(cell, []).append((dist, bid, bgeo.ndim, side))
    for cell in sorted(found):
        for dist, bid, nd, side in sorted(found[cell], key=lambda t: t[0]):
            mesh.add_boundary_cell(cell, bid, nd, side)


def load_msh(file_path, ndim):
    """Read a Gmsh 2.2 binary mesh into a ``discrete.Mesh`` (sem/grid_importers.py:45-68)."""
    with open(file_path, "rb") as fh:
        data = fh.read()
    f = _Reader(data)
    is_binary = parse_format(f)
    if not is_binary:
        raise NotImplementedError("Reading ASCII *.msh files is not yet supported. Save the "
                                  "mesh in binary format and try again.")
    mesh = discrete.Mesh(ndim)
    region_id_map, boundary_id_map = parse_physical_names(f, mesh)
    parse_nodes_bin(f, mesh)
    bnd = parse_elements_bin(f, mesh, region_id_map, boundary_id_map)
    find_cell_neighbors(mesh, bnd)
    return mesh


# --------------------------------------------------------------------------
def write_msh(file_path, nodes, cells, regions, physical_names, boundary_lines=()):
    """Write a Gmsh 2.2 binary mesh.

    nodes           float [ndim, N] (2-D; z = 0 is written)
    cells           uint [E, n, n] lexicographic quadrilateral node maps
    regions         int [E] physical id (1-based) of each cell
    physical_names  [(dim, physical id, name), ...]
    boundary_lines  [(physical id, uint [n] lexicographic line node map), ...]
    """
    nodes = np.asarray(nodes, dtype=np.float64)
    cells = np.asarray(cells)
    E, n = cells.shape[0], cells.shape[1]
    N = nodes.shape[1]
    out = bytearray()
    out += b"$MeshFormat\n2.2 1 8\n" + struct.pack("<i", 1) + b"\n$EndMeshFormat\n"
    out += b"$PhysicalNames\n%d\n" % len(physical_names)
    for dim, pid, name in physical_names:
        out += b'%d %d "%s"\n' % (dim, pid, name.encode())
    out += b"$EndPhysicalNames\n$Nodes\n%d\n" % N
    rec = np.zeros(N, dtype=np.dtype([("index", "<i4"), ("coord", "<f8", 3)]))
    rec["index"] = np.arange(1, N + 1)
    rec["coord"][:, :nodes.shape[0]] = nodes.T
    out += rec.tobytes() + b"\n$EndNodes\n"
    n_lines = len(boundary_lines)
    out += b"$Elements\n%d\n" % (n_lines + E)
    eid = 1
    if n_lines:
        nl = len(boundary_lines[0][1])
        out += np.array([_TYPE_OF_LINE[nl], n_lines, 2], dtype="<i4").tobytes()
        blk = np.zeros((n_lines, 3 + nl), dtype="<u4")
        for i, (pid, nm) in enumerate(boundary_lines):
            g = np.empty(nl, dtype=np.int64)
            g[gmsh_to_lexicographic((nl,)).ravel()] = np.asarray(nm, dtype=np.int64).ravel()
            blk[i] = [eid + i, pid, pid] + list(g + 1)
        out += blk.tobytes()
        eid += n_lines
    idx = gmsh_to_lexicographic((n, n)).ravel()
    g = np.empty((E, n * n), dtype=np.int64)
    g[:, idx] = cells.reshape(E, -1).astype(np.int64)
    blk = np.empty((E, 3 + n * n), dtype="<u4")
    blk[:, 0] = np.arange(eid, eid + E)
    blk[:, 1] = regions
    blk[:, 2] = regions
    blk[:, 3:] = g + 1
    out += np.array([_TYPE_OF_QUAD[n], E, 2], dtype="<i4").tobytes() + blk.tobytes()
    out += b"\n$EndElements\n"
    with open(file_path, "wb") as fh:
        fh.write(bytes(out))
