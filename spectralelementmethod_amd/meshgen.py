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
