"""Synthetic meshes for tests and benchmarks.

The reference ships only Gmsh ``.geo`` sources (examples/meshes/*.geo) and
no ``.msh``; gmsh is absent here.  These generators produce the same kind of
mesh in memory, following the in-memory fixture pattern of
tests/test_discrete.py:19-33 (nodes via np.mgrid, x-major global ids):

* ``structured_square``: [-1,1]^2 with nex x ney quads of order p and
  equispaced element nodes (Gmsh high-order node placement), optional warp
  x,y += a sin(pi x) sin(pi y) for non-constant Jacobians
  (examples/meshes/square.geo:1-15 stand-in).
* ``annulus``: curved half-annulus in (rho, z), r in [r0, r1],
  theta in [th0, pi - th0] (examples/meshes/donut.geo:1-22 stand-in).

Both return ``nodes`` float64 [2, n_nodes] and ``e2n`` uint32 [E, n, n]
(lexicographic (xi0, xi1), sem/discrete.py:1044).

Hexahedra (``north_star``: "synthetic structured quad/hex meshes"):

* ``structured_cube``: [-1,1]^3 with nex x ney x nez hexahedra of order p,
  equispaced element nodes, optional warp x,y,z += a sin(pi x) sin(pi y)
  sin(pi z);
* ``extrude``: a quad mesh swept along z in nez uniform layers (the mesh of
  the extrusion identity the hexahedral parity tests use).

They return ``nodes`` float64 [3, n_nodes] and ``e2n`` uint32 [E, n, n, n]
(lexicographic (xi0, xi1, xi2), xi2 fastest, as the reference's N-D
``TensorProduct`` lays out an [n, n, n] coefficient block,
sem/basis_functions.py:408-448, 626-650).
"""
import numpy as np


def _element_map(n_a, n_b, p, stride):
    """e2n[ea*n_b + eb, i, j] = (ea*p + i)*stride + eb*p + j."""
    n = p + 1
    ea = np.arange(n_a, dtype=np.int64)[:, None, None, None]
    eb = np.arange(n_b, dtype=np.int64)[None, :, None, None]
    i = np.arange(n, dtype=np.int64)[None, None, :, None]
    j = np.arange(n, dtype=np.int64)[None, None, None, :]
    ids = (ea * p + i) * stride + eb * p + j
    return ids.reshape(n_a * n_b, n, n).astype(np.uint32)


def structured_square(nex, ney, p, warp=0.0, x0=-1.0, x1=1.0, y0=-1.0, y1=1.0):
    """Structured quad mesh.  Node (ix, iy) -> id ix*Ny + iy with
    Ny = ney*p + 1; element (ex, ey) -> id ex*ney + ey.  A strip of element
    columns [ex0, ex1) therefore owns the contiguous node range
    [ex0*p*Ny, (ex1*p + 1)*Ny)."""
    Nx, Ny = nex * p + 1, ney * p + 1
    if Nx * Ny >= 2 ** 32:
        raise ValueError("mesh too large for a uint32 element map")
    x = np.linspace(x0, x1, Nx)
    y = np.linspace(y0, y1, Ny)
    X, Y = np.meshgrid(x, y, indexing="ij")
    if warp:
        s = warp * np.sin(np.pi * X) * np.sin(np.pi * Y)
        X = X + s
        Y = Y + s
    nodes = np.stack([X.ravel(), Y.ravel()])
    return nodes, _element_map(nex, ney, p, Ny)


def _element_map3(n_a, n_b, n_c, p, Nb, Nc):
    """e2n[(ea*n_b + eb)*n_c + ec, i, j, k] = ((ea*p + i)*Nb + eb*p + j)*Nc + ec*p + k."""
    n = p + 1
    ea = np.arange(n_a, dtype=np.int64)[:, None, None, None, None, None]
    eb = np.arange(n_b, dtype=np.int64)[None, :, None, None, None, None]
    ec = np.arange(n_c, dtype=np.int64)[None, None, :, None, None, None]
    i = np.arange(n, dtype=np.int64)[None, None, None, :, None, None]
    j = np.arange(n, dtype=np.int64)[None, None, None, None, :, None]
    k = np.arange(n, dtype=np.int64)[None, None, None, None, None, :]
    ids = ((ea * p + i) * Nb + eb * p + j) * Nc + ec * p + k
    return ids.reshape(n_a * n_b * n_c, n, n, n).astype(np.uint32)


def structured_cube(nex, ney, nez, p, warp=0.0, lo=-1.0, hi=1.0):
    """Structured hexahedral mesh of [lo, hi]^3.  Node (ix, iy, iz) -> id
    (ix*Ny + iy)*Nz + iz; element (ex, ey, ez) -> id (ex*ney + ey)*nez + ez;
    local node (a, b, c) of element (ex, ey, ez) is node
    (ex*p + a, ey*p + b, ez*p + c)."""
    Nx, Ny, Nz = nex * p + 1, ney * p + 1, nez * p + 1
    if Nx * Ny * Nz >= 2 ** 32:
        raise ValueError("mesh too large for a uint32 element map")
    X, Y, Z = np.meshgrid(np.linspace(lo, hi, Nx), np.linspace(lo, hi, Ny),
                          np.linspace(lo, hi, Nz), indexing="ij")
    if warp:
        s = warp * np.sin(np.pi * X) * np.sin(np.pi * Y) * np.sin(np.pi * Z)
        X = X + s
        Y = Y + 0.5 * s
        Z = Z - s
    nodes = np.stack([X.ravel(), Y.ravel(), Z.ravel()])
    return nodes, _element_map3(nex, ney, nez, p, Ny, Nz)


def structured_slab(nex, ney, nez, p, ex0, ex1, warp=0.0, lo=-1.0, hi=1.0):
    """Element layers [ex0, ex1) along x of ``structured_cube(nex, ney, nez,
    p, warp, lo, hi)`` with the nodes renumbered locally: local id = global id
    - ex0*p*Ny*Nz (the slab's nodes are one contiguous global range, x-major).
    The coordinates are slices of the same global linspaces with the same
    warp expression, so a node on a slab face has bit-identical coordinates
    in both neighbouring slabs.  Returns nodes [3, n_local], e2n
    [E_local, n, n, n] (element (ex - ex0, ey, ez) -> id ((ex - ex0)*ney +
    ey)*nez + ez, as in the cube) and node_offset."""
    if not (0 <= ex0 < ex1 <= nex):
        raise ValueError("bad slab [%d, %d) of %d layers" % (ex0, ex1, nex))
    Nx, Ny, Nz = nex * p + 1, ney * p + 1, nez * p + 1
    if Nx * Ny * Nz >= 2 ** 32:
        raise ValueError("mesh too large for a uint32 element map")
    ix0, ix1 = ex0 * p, ex1 * p + 1
    X, Y, Z = np.meshgrid(np.linspace(lo, hi, Nx)[ix0:ix1], np.linspace(lo, hi, Ny),
                          np.linspace(lo, hi, Nz), indexing="ij")
    if warp:
        s = warp * np.sin(np.pi * X) * np.sin(np.pi * Y) * np.sin(np.pi * Z)
        X = X + s
        Y = Y + 0.5 * s
        Z = Z - s
    nodes = np.stack([X.ravel(), Y.ravel(), Z.ravel()])
    return nodes, _element_map3(ex1 - ex0, ney, nez, p, Ny, Nz), ix0 * Ny * Nz


def structured_box(nex, ney, nez, p, rx, ry, rz, warp=0.0, lo=-1.0, hi=1.0):
    """The element box rx x ry x rz (half-open element ranges per axis) of
    ``structured_cube(nex, ney, nez, p, warp, lo, hi)`` with its nodes
    numbered locally (x-major, z fastest, as in the cube).  Coordinates are
    slices of the same global linspaces with the same warp expression, so a
    node shared by two boxes has bit-identical coordinates in both.  Returns
    nodes [3, n_local], e2n [E_local, n, n, n] and the global node ids
    [n_local]."""
    (ex0, ex1), (ey0, ey1), (ez0, ez1) = rx, ry, rz
    for (a, b), m in ((rx, nex), (ry, ney), (rz, nez)):
        if not (0 <= a < b <= m):
            raise ValueError("bad element range [%d, %d) of %d" % (a, b, m))
    Nx, Ny, Nz = nex * p + 1, ney * p + 1, nez * p + 1
    if Nx * Ny * Nz >= 2 ** 32:
        raise ValueError("mesh too large for a uint32 element map")
    ix = np.arange(ex0 * p, ex1 * p + 1)
    iy = np.arange(ey0 * p, ey1 * p + 1)
    iz = np.arange(ez0 * p, ez1 * p + 1)
    X, Y, Z = np.meshgrid(np.linspace(lo, hi, Nx)[ix], np.linspace(lo, hi, Ny)[iy],
                          np.linspace(lo, hi, Nz)[iz], indexing="ij")
    if warp:
        s = warp * np.sin(np.pi * X) * np.sin(np.pi * Y) * np.sin(np.pi * Z)
        X = X + s
        Y = Y + 0.5 * s
        Z = Z - s
    nodes = np.stack([X.ravel(), Y.ravel(), Z.ravel()])
    e2n = _element_map3(ex1 - ex0, ey1 - ey0, ez1 - ez0, p, iy.size, iz.size)
    gids = ((ix[:, None, None] * Ny + iy[None, :, None]) * Nz + iz[None, None, :]).ravel()
    return nodes, e2n, gids


def extrude(nodes2, e2n2, nez, p, z0=0.0, z1=1.0):
    """Sweep a quad mesh (nodes2 [2, N2], e2n2 [E2, n, n]) along z in nez
    uniform layers of order-p elements over [z0, z1].  Node (i2, kz) -> id
    i2*Nz + kz (Nz = nez*p + 1); element (e2, ez) -> id e2*nez + ez, local
    node (a, b, c) = (2-D local node (a, b), layer node ez*p + c)."""
    nodes2 = np.asarray(nodes2, dtype=np.float64)
    e2n2 = np.asarray(e2n2).astype(np.int64)
    E2, n = e2n2.shape[0], e2n2.shape[1]
    Nz = nez * p + 1
    z = np.linspace(z0, z1, Nz)
    N2 = nodes2.shape[1]
    nodes = np.stack([np.repeat(nodes2[0], Nz), np.repeat(nodes2[1], Nz), np.tile(z, N2)])
    ez = np.arange(nez, dtype=np.int64)[None, :, None, None, None]
    c = np.arange(n, dtype=np.int64)[None, None, None, None, :]
    ids = e2n2[:, None, :, :, None] * Nz + ez * p + c
    if N2 * Nz >= 2 ** 32:
        raise ValueError("mesh too large for a uint32 element map")
    return nodes, ids.reshape(E2 * nez, n, n, n).astype(np.uint32)


def structured_strip(nex, ney, p, ex0, ex1, warp=0.0):
    """Element columns [ex0, ex1) of ``structured_square(nex, ney, p, warp)``
    with nodes renumbered locally: local id = global id - ex0*p*Ny.  The
    coordinates are slices of the same global linspace, so a node on a strip
    boundary has bit-identical coordinates in both neighbouring strips.
    Returns nodes [2, n_local], e2n [E_local, n, n], node_offset."""
    if not (0 <= ex0 < ex1 <= nex):
        raise ValueError("bad strip [%d, %d) of %d columns" % (ex0, ex1, nex))
    Nx, Ny = nex * p + 1, ney * p + 1
    ix0, ix1 = ex0 * p, ex1 * p + 1
    x = np.linspace(-1.0, 1.0, Nx)[ix0:ix1]
    y = np.linspace(-1.0, 1.0, Ny)
    X, Y = np.meshgrid(x, y, indexing="ij")
    if warp:
        s = warp * np.sin(np.pi * X) * np.sin(np.pi * Y)
        X = X + s
        Y = Y + s
    nodes = np.stack([X.ravel(), Y.ravel()])
    return nodes, _element_map(ex1 - ex0, ney, p, Ny), ix0 * Ny


def annulus(nth, nr, p, r0=1.0, r1=4.0, th0=0.05, th1=np.pi - 0.05):
    """Curved annulus: xi0 <-> theta, xi1 <-> r (positive Jacobian).
    Node (it, ir) -> id it*Nr + ir."""
    Nt, Nr = nth * p + 1, nr * p + 1
    th = np.linspace(th0, th1, Nt)
    r = np.linspace(r0, r1, Nr)
    TH, R = np.meshgrid(th, r, indexing="ij")
    nodes = np.stack([(R * np.sin(TH)).ravel(), (R * np.cos(TH)).ravel()])
    return nodes, _element_map(nth, nr, p, Nr)


def square_dirichlet_left_bottom(nodes, tol=1e-12):
    """Essential-BC mask and values of the restated Poisson example:
    u = 0.2((x+1) + (y+1)) on the left and bottom edges
    (examples/poisson.py:137-140)."""
    x, y = nodes
    on = (np.abs(x + 1) < tol) | (np.abs(y + 1) < tol)
    vals = np.zeros(x.shape)
    vals[on] = 0.2 * ((x[on] + 1) + (y[on] + 1))
    return on, vals


def square_boundary_lines(e2n, nex, ney):
    """Lexicographic node maps of the boundary sides of a structured_square
    mesh, keyed by side: 'left' (x = x0), 'right', 'bottom' (y = y0), 'top'.
    Element (ex, ey) has id ex*ney + ey; its row r runs along x, column j
    along y."""
    e2n = np.asarray(e2n)
    out = {"left": [], "right": [], "bottom": [], "top": []}
    for ey in range(ney):
        out["left"].append(e2n[ey][0, :])
        out["right"].append(e2n[(nex - 1) * ney + ey][-1, :])
    for ex in range(nex):
        out["bottom"].append(e2n[ex * ney][:, 0])
        out["top"].append(e2n[ex * ney + ney - 1][:, -1])
    return out


def write_square_msh(path, nex, ney, p, warp=0.0):
    """The square.geo stand-in as a Gmsh 2.2 binary file: region 'interior',
    boundaries 'ebc' (left + bottom) and 'nbc' (top + right), the tags of
    examples/meshes/square.geo:1-15.  Returns (nodes, e2n)."""
    from .grid_importers import write_msh
    nodes, e2n = structured_square(nex, ney, p, warp)
    sides = square_boundary_lines(e2n, nex, ney)
    lines = [(1, m) for m in sides["left"] + sides["bottom"]] + \
            [(2, m) for m in sides["top"] + sides["right"]]
    names = [(1, 1, "ebc"), (1, 2, "nbc"), (2, 3, "interior")]
    write_msh(path, nodes, e2n, np.full(e2n.shape[0], 3), names, lines)
    return nodes, e2n


# ---------------------------------------------------------------------------
# Unstructured quad meshes (planner / partitioner coverage)
# ---------------------------------------------------------------------------
def _order_p_quads(corners, p):
    """Order-p lexicographic element nodes of straight-sided quads with CCW
    corners [E, 4, 2] (c0 -> c1 along xi0, c0 -> c3 along xi1), equispaced
    (Gmsh high-order placement); shared nodes merged by position.
    Returns nodes [2, n_nodes], e2n uint32 [E, p+1, p+1]."""
    corners = np.asarray(corners, dtype=np.float64)
    E = corners.shape[0]
    t = np.linspace(0.0, 1.0, p + 1)
    s0 = t[:, None]   # xi0 (row index i)
    s1 = t[None, :]   # xi1 (column index j)
    c0, c1, c2, c3 = (corners[:, k, :][:, None, None, :] for k in range(4))
    X = ((1 - s0) * (1 - s1))[None, :, :, None] * c0 + (s0 * (1 - s1))[None, :, :, None] * c1 \
        + (s0 * s1)[None, :, :, None] * c2 + ((1 - s0) * s1)[None, :, :, None] * c3
    pts = X.reshape(-1, 2)
    scale = max(1.0, float(np.abs(pts).max()))
    key = np.round(pts / scale * 1e9).astype(np.int64)
    _, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    # number nodes in order of first appearance (element-major: locality)
    order = np.argsort(first)
    rank = np.empty_like(order)
    rank[order] = np.arange(order.size)
    ids = rank[inv.ravel()]
    nodes = pts[first[order]].T.copy()
    return nodes, ids.reshape(E, p + 1, p + 1).astype(np.uint32)


def quads_from_triangles(nx, ny, p, jitter=0.2, seed=0):
    """Irregular-valence quad mesh of [-1,1]^2: a jittered nx x ny grid is
    split into triangles (alternating diagonals), and every triangle into
    three quads through its centroid and edge midpoints -- interior vertices
    of valence 3 (centroids), 4 (edge midpoints) and 6 or more (grid points),
    unlike any structured mesh.  Elements are numbered triangle by triangle
    (a locality-preserving but non-lexicographic order)."""
    rng = np.random.default_rng(seed)
    x = np.linspace(-1, 1, nx + 1)
    y = np.linspace(-1, 1, ny + 1)
    X, Y = np.meshgrid(x, y, indexing="ij")
    h = min(2.0 / nx, 2.0 / ny)
    inner = np.zeros_like(X, dtype=bool)
    inner[1:-1, 1:-1] = True
    X = X + np.where(inner, rng.uniform(-jitter, jitter, X.shape) * h, 0.0)
    Y = Y + np.where(inner, rng.uniform(-jitter, jitter, Y.shape) * h, 0.0)
    P = np.stack([X, Y], axis=-1)
    tris = []
    for i in range(nx):
        for j in range(ny):
            a, b, c, d = P[i, j], P[i + 1, j], P[i + 1, j + 1], P[i, j + 1]
            if (i + j) % 2 == 0:
                tris += [(a, b, c), (a, c, d)]
            else:
                tris += [(a, b, d), (b, c, d)]
    quads = []
    for (a, b, c) in tris:  # CCW triangles -> 3 CCW quads
        g = (a + b + c) / 3.0
        mab, mbc, mca = (a + b) / 2, (b + c) / 2, (c + a) / 2
        quads += [(a, mab, g, mca), (b, mbc, g, mab), (c, mca, g, mbc)]
    return _order_p_quads(np.array(quads), p)


def shuffle_elements(e2n, seed=0):
    """The same mesh with its elements in random order (destroys the
    locality the chain planner exploits)."""
    perm = np.random.default_rng(seed).permutation(np.asarray(e2n).shape[0])
    return np.ascontiguousarray(np.asarray(e2n)[perm])


def shuffle_nodes(nodes, e2n, seed=0):
    """The same mesh with its nodes renumbered at random (rows of a group then
    span far more than the 4096 ids of the 16-bit packed map)."""
    n = nodes.shape[1]
    perm = np.random.default_rng(seed).permutation(n)  # new id of old node
    new_nodes = np.empty_like(nodes)
    new_nodes[:, perm] = nodes
    return new_nodes, perm[np.asarray(e2n).astype(np.int64)].astype(np.uint32)


def rcm_renumber(nodes, e2n):
    """Reverse Cuthill-McKee renumbering of the nodes (what DOFManager does by
    default, sem/discrete.py:169-178), then elements sorted by their smallest
    node: restores locality after shuffling."""
    from scipy import sparse
    from scipy.sparse import csgraph
    e2n = np.asarray(e2n).astype(np.int64)
    E = e2n.shape[0]
    n = nodes.shape[1]
    flat = e2n.reshape(E, -1)
    rows = np.repeat(flat, flat.shape[1], axis=1).ravel()
    cols = np.tile(flat, (1, flat.shape[1])).ravel()
    g = sparse.csr_matrix((np.ones(rows.size, np.int8), (rows, cols)), shape=(n, n))
    order = csgraph.reverse_cuthill_mckee(g, symmetric_mode=True)
    new_id = np.empty(n, dtype=np.int64)
    new_id[order] = np.arange(n)
    e_new = new_id[flat]
    e_order = np.argsort(e_new.min(axis=1), kind="stable")
    return nodes[:, order].copy(), e_new[e_order].reshape(e2n.shape).astype(np.uint32)
