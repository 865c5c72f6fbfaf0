#!/usr/bin/env python
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

This script is test infrastructure.  It runs only in the build container,
where the reference checkout lives at /root/reference (read-only).  It is
never run on the GPU box and nothing in the product imports it.  Only its
OUTPUTS (small .npz files of inputs and expected outputs) are committed.

How the reference is imported:
  * ``h5py`` is absent from this image.  The reference imports it at module
    level (sem/basis_functions.py:11, sem/basis_data.py:16) and reads
    sem/data/basis-data.hdf5 through ``h5py.File`` (sem/basis_functions.py:
    362-370).  A runtime stand-in module decodes that file's contiguous
    float64 payload (105 values at byte offset 2216, datasets for orders
    1..10 in order, each shaped (3, p//2+1)).  The decode is checked against
    the reference's own numpy ``quadratures.GaussLobatto`` below.
  * SciPy >= 1.15 made ``comb(..., exact)`` keyword-only, which breaks
    sem/geometry.py:149; the positional ``exact`` is forwarded as a keyword.
  * Byte-code writing is disabled so nothing is written under /root/reference.
Orders 11..16 are produced by the reference's own arbitrary-precision
generator ``sem.basis_data.gauss_legendre_lobatto`` (sem/basis_data.py:19-109)
and served through the same stand-in ("extended-order oracle").

The operator definitions are RESTATED from the reference examples because
the examples cannot run as written:
  * Poisson element Laplacian Lse: examples/poisson.py:168-193,
    applied as einsum('pqrs,rs') (examples/squirmer-axisymmetric.py:286) and
    scatter-added through FiniteElement.node_ind (sem/discrete.py:658-663).
  * Axisymmetric E2e, Lve, Me: examples/squirmer-axisymmetric.py:193-254.
  * Assembled Poisson solution: DOFManagerSC (sem/discrete.py:283-528) with
    the local systems of examples/poisson.py:200-256.

Usage:  python tests/golden/make_goldens.py   (writes tests/golden/*.npz)
"""
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
HDF5_PAYLOAD_OFFSET = 2216
HDF5_N_VALUES = 105
MAX_ORDER_EXT = 16


# --------------------------------------------------------------------------
# runtime environment gaps (no edits to /root/reference)
# --------------------------------------------------------------------------
def decode_basis_hdf5():
    raw = open(os.path.join(REF, "sem", "data", "basis-data.hdf5"), "rb").read()
    vals = np.frombuffer(raw[HDF5_PAYLOAD_OFFSET:HDF5_PAYLOAD_OFFSET + 8 * HDF5_N_VALUES], "<f8")
    tables, off = {}, 0
    for order in range(1, 11):
        m = order // 2 + 1
        tables[order] = vals[off:off + 3 * m].reshape(3, m).copy()
        off += 3 * m
    assert off == HDF5_N_VALUES
    return tables


_TABLES = {}


class _Group(dict):
    def __init__(self, tables, max_order):
        super().__init__({str(k): v for k, v in tables.items()})
        self.attrs = {"max_order": max_order}


class _File(object):
    def __init__(self, path, mode="r"):
        assert mode == "r"
        self._root = {"GaussLegendreLobatto": _Group(_TABLES, max(_TABLES))}

    def __getitem__(self, key):
        return self._root[key]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def install_runtime_shims():
    h5 = types.ModuleType("h5py")
    h5.File = _File
    sys.modules["h5py"] = h5
    import scipy.special as sf
    _comb = sf.comb

    def comb(N, k, *args, **kw):
        if args:
            kw["exact"] = args[0]
        return _comb(N, k, **kw)

    sf.comb = comb
    sys.path.insert(0, REF)


# --------------------------------------------------------------------------
# synthetic meshes (same convention as spectralelementmethod_amd.meshgen)
# --------------------------------------------------------------------------
def structured_square(nex, ney, p, warp=0.0):
    """[-1,1]^2, nex x ney elements of order p, equispaced element nodes.
    Global node (ix, iy) has id ix*Ny + iy (x-major, as np.mgrid in
    tests/test_discrete.py:26-28); element (ex, ey) has id ex*ney + ey."""
    n = p + 1
    Nx, Ny = nex * p + 1, ney * p + 1
    x = np.linspace(-1.0, 1.0, Nx)
    y = np.linspace(-1.0, 1.0, Ny)
    X, Y = np.meshgrid(x, y, indexing="ij")
    if warp:
        s = warp * np.sin(np.pi * X) * np.sin(np.pi * Y)
        X, Y = X + s, Y + s
    nodes = np.stack([X.ravel(), Y.ravel()])
    ids = np.arange(Nx * Ny, dtype=np.uint32).reshape(Nx, Ny)
    e2n = np.empty((nex * ney, n, n), dtype=np.uint32)
    for ex in range(nex):
        for ey in range(ney):
            e2n[ex * ney + ey] = ids[ex * p:ex * p + n, ey * p:ey * p + n]
    return nodes, e2n


def annulus(nth, nr, p, r0=1.0, r1=4.0, th0=0.05, th1=np.pi - 0.05):
    """Curved annulus in the (rho, z) half plane: xi0 <-> theta, xi1 <-> r
    (positive Jacobian).  Global node (it, ir) has id it*Nr + ir."""
    n = p + 1
    Nt, Nr = nth * p + 1, nr * p + 1
    th = np.linspace(th0, th1, Nt)
    r = np.linspace(r0, r1, Nr)
    TH, R = np.meshgrid(th, r, indexing="ij")
    nodes = np.stack([(R * np.sin(TH)).ravel(), (R * np.cos(TH)).ravel()])
    ids = np.arange(Nt * Nr, dtype=np.uint32).reshape(Nt, Nr)
    e2n = np.empty((nth * nr, n, n), dtype=np.uint32)
    for et in range(nth):
        for er in range(nr):
            e2n[et * nr + er] = ids[et * p:et * p + n, er * p:er * p + n]
    return nodes, e2n


def ref_mesh(nodes, e2n):
    from sem.discrete import Mesh
    from sem.geometry import Quadrilateral
    n = e2n.shape[1]
    geo = Quadrilateral(n, n)
    mesh = Mesh(geo.ndim)
    mesh.set_nodes(nodes.copy())
    mesh.add_geometry(geo)
    mesh.new_region("*")
    for e in range(e2n.shape[0]):
        mesh.add_cell(e2n[e].copy(), 0, 0)
    return mesh


def ref_basis(p):
    import sem.basis_functions as bf
    b1 = bf.LagrangeGaussLobatto(p)
    return b1, bf.TensorProductQS(b1, b1)


def mesh_map(mesh):
    return np.stack([mesh.get_cell(i).node_ind_lexicographic for i in range(mesh.n_cells)]).astype(np.uint32)


# --------------------------------------------------------------------------
# restated reference operators
# --------------------------------------------------------------------------
def poisson_Lse(fe):
    """examples/poisson.py:166-193 with current names."""
    n = fe.basis.coeff_shape[0]
    dmats = fe.basis.get_D1_matrices()
    invJ = fe.invJ
    gradh_xi0 = np.einsum("mp,imn->imnp", dmats[0], invJ[0, ...])
    gradh_xi1 = np.einsum("nq,imn->imnq", dmats[1], invJ[1, ...])
    JxW = fe.detJxW
    Lse = np.zeros((n, n, n, n))
    p, q, r = np.ogrid[[slice(n)] * 3]
    Lse[p, q, r, q] += np.einsum("mn,imnp,imnr->pnr", JxW, gradh_xi0, gradh_xi0)
    Lse += np.einsum("mn,imnp,imns->pnms", JxW, gradh_xi0, gradh_xi1)
    Lse += np.einsum("mn,imnq,imnr->mqrn", JxW, gradh_xi1, gradh_xi0)
    Lse[p, q, p, r] += np.einsum("mn,imnq,imns->mqs", JxW, gradh_xi1, gradh_xi1)
    return Lse, JxW


def axisym_ops(fe):
    """examples/squirmer-axisymmetric.py:186-254 at Re = 0 (Ae omitted)."""
    x = fe.x_phys
    JxW = fe.detJxW
    invJ = fe.invJ
    dmats = fe.basis.get_D1_matrices()
    n = fe.basis.coeff_shape[0]
    gradh_xi0 = np.einsum("imn,mp->imnp", invJ[0, :], dmats[0])
    gradh_xi1 = np.einsum("imn,nq->imnq", invJ[1, :], dmats[1])
    E2e = np.zeros((n, n, n, n))
    rho_JxW = x[0] * JxW
    p, q, r = np.ogrid[[slice(n)] * 3]
    E2e[p, q, r, q] += np.einsum("mn,imnp,imnr->pnr", rho_JxW, gradh_xi0, gradh_xi0)
    E2e += np.einsum("mn,imnp,imns->pnms", rho_JxW, gradh_xi0, gradh_xi1)
    E2e += np.einsum("mn,imnq,imnr->mqrn", rho_JxW, gradh_xi1, gradh_xi0)
    E2e[p, q, p, r] += np.einsum("mn,imnq,imns->mqs", rho_JxW, gradh_xi1, gradh_xi1)
    p2, q2 = np.ogrid[[slice(n)] * 2]
    Lve = E2e.copy()
    Lve[p2, q2, p2, q2] += JxW / x[0]
    p, q, r = np.ogrid[[slice(n)] * 3]
    E2e[p, q, r, q] += 2 * np.einsum("mn,mnr->mnr", JxW, gradh_xi0[0])
    E2e[p, q, p, r] += 2 * np.einsum("mn,mns->mns", JxW, gradh_xi1[0])
    Me_diag = rho_JxW * x[0]
    return E2e, Lve, Me_diag


def scatter_action(dm, u, op):
    y = np.zeros(dm.ndof)
    for fe in dm.finite_elements(x_phys=True, Jacobian=True):
        loc = fe.node_ind
        y_e = np.einsum("pqrs,rs", op(fe), u[loc])
        np.add.at(y, loc, y_e)
    return y


# --------------------------------------------------------------------------
def gen_gll():
    import sem.basis_data as bd
    import sem.basis_functions as bf
    import sem.quadratures as quad
    out = {}
    # decoded HDF5 vs the reference's numpy GaussLobatto (validates the decode)
    for p in range(1, 11):
        g = quad.GaussLobatto(p + 1)
        m = p // 2 + 1
        assert np.abs(_TABLES[p][0] - g.abscissa[-m:]).max() < 2e-16
        assert np.abs(_TABLES[p][2] - g.weights[-m:]).max() < 2e-14
    for p in range(11, MAX_ORDER_EXT + 1):
        nodes, bary, qw = bd.gauss_legendre_lobatto(p + 1)
        _TABLES[p] = np.array([[float(v) for v in mat] for mat in (nodes, bary, qw)])
    for p in range(1, MAX_ORDER_EXT + 1):
        b = bf.LagrangeGaussLobatto(p)
        out["half_%d" % p] = _TABLES[p]
        out["nodes_%d" % p] = b.nodes
        out["bary_%d" % p] = b.bary_wts
        out["quad_%d" % p] = b.quad_rule.weights
        out["D1_%d" % p] = b.D1
        out["Veq_%d" % p] = b._interp_eq_mat
    # barycentric known answer (sem/bary_interp.c:95-99 restated through the
    # reference's Python twin)
    b4 = bf.LagrangeGaussLobatto(4)
    f = np.array([-1, -0.65465, 0, 0.65465, 1.0])
    out["bary_known_f"] = f
    out["bary_known_x"] = np.array(0.654)
    out["bary_known_value"] = np.array(b4.interpolate(f, np.array(0.654)))
    # interpolation at a sweep of points (incl. exact nodes) for n = 2..9
    rng = np.random.default_rng(7)
    for p in range(1, 9):
        b = bf.LagrangeGaussLobatto(p)
        xs = np.concatenate([np.linspace(-1, 1, 17), b.nodes, rng.uniform(-1, 1, 8)])
        fv = rng.standard_normal(p + 1)
        out["interp_x_%d" % p] = xs
        out["interp_f_%d" % p] = fv
        # vector x: the reference's scalar-x exact-node branch (basis_functions.py:331-332)
        # indexes a 0-d result and raises, so points are passed as one 1-D array
        out["interp_y_%d" % p] = np.asarray(b.interpolate(fv, xs))
    np.savez_compressed(os.path.join(OUT, "gll.npz"), **out)
    print("gll.npz: p=1..%d" % MAX_ORDER_EXT)


def gen_tensor_ops():
    """TensorProduct.deriv / gradient / compute_coeffs_grid_eq on random data
    (sem/basis_functions.py:599-650)."""
    rng = np.random.default_rng(3)
    out = {}
    for p in (2, 4, 8, 12):
        _, tb = ref_basis(p)
        c = rng.standard_normal((5, p + 1, p + 1))
        out["c_%d" % p] = c
        out["grad_%d" % p] = tb.gradient(c)
        out["coeffs_eq_%d" % p] = tb.compute_coeffs_grid_eq(c)
    np.savez_compressed(os.path.join(OUT, "tensor_ops.npz"), **out)
    print("tensor_ops.npz")


def gen_poisson_action():
    from sem.discrete import DOFManager
    out = {}
    cases = [("p4_4x4", 4, 4, 4, 0.0, False), ("p8_8x8w", 8, 8, 8, 0.05, False),
             ("p8_8x8w_rcm", 8, 8, 8, 0.05, True), ("p2_6x5", 2, 6, 5, 0.05, False),
             ("p6_3x4w", 6, 3, 4, 0.05, False), ("p12_3x3w", 12, 3, 3, 0.05, False),
             ("p16_2x2w", 16, 2, 2, 0.05, False)]
    rng = np.random.default_rng(0)
    for name, p, nex, ney, warp, rcm in cases:
        nodes, e2n = structured_square(nex, ney, p, warp)
        mesh = ref_mesh(nodes, e2n)
        _, tb = ref_basis(p)
        dm = DOFManager(mesh, 1, tb, rcm_order=rcm)
        u = rng.standard_normal(dm.ndof)
        y = scatter_action(dm, u, lambda fe: poisson_Lse(fe)[0])
        out[name + "_nodes"] = mesh.nodes.copy()
        out[name + "_e2n"] = mesh_map(mesh)
        out[name + "_u"] = u
        out[name + "_y"] = y
        out[name + "_p"] = np.array(p)
        print("  action %s ndof=%d |y|=%.6e" % (name, dm.ndof, np.linalg.norm(y)))
        if name in ("p8_8x8w", "p4_4x4", "p12_3x3w", "p16_2x2w"):
            fields = {k: [] for k in ("x_phys", "J", "invJ", "detJ", "detJxW")}
            for fe in dm.finite_elements(x_phys=True, Jacobian=True):
                fields["x_phys"].append(fe.x_phys)
                fields["J"].append(fe.J)
                fields["invJ"].append(fe.invJ)
                fields["detJ"].append(fe.mapping.detJ)
                fields["detJxW"].append(fe.detJxW)
            for k, v in fields.items():
                out[name + "_geom_" + k] = np.stack(v)
    np.savez_compressed(os.path.join(OUT, "poisson_action.npz"), **out)
    print("poisson_action.npz")


def gen_poisson_solution():
    """Assembled Poisson solution through DOFManagerSC (config 1 stand-in:
    structured 8x8 p=4 on [-1,1]^2; EBC u = 0.2((x+1)+(y+1)) on the left and
    bottom edges (examples/poisson.py:137-140), f = 1 so lrhs = JxW
    (examples/poisson.py:200), homogeneous Neumann elsewhere)."""
    from sem.discrete import DOFManagerSC
    out = {}
    for name, p, nex, ney, warp in [("p4_8x8", 4, 8, 8, 0.0), ("p8_4x4w", 8, 4, 4, 0.05)]:
        nodes, e2n = structured_square(nex, ney, p, warp)
        mesh = ref_mesh(nodes, e2n)
        _, tb = ref_basis(p)
        dm = DOFManagerSC(mesh, 1, tb)  # default rcm_order=True
        local_systems = []
        n2 = (p + 1) ** 2
        for fe in dm.finite_elements(x_phys=True, Jacobian=True):
            Lse, JxW = poisson_Lse(fe)
            loc = (Lse.reshape(n2, n2), JxW.reshape(n2).copy())
            local_systems.append(dm.reorder_local_system_hier(fe, loc))
        gsys = dm.init_global_linear_system()
        dm.assemble_global_sc_system(gsys, local_systems)
        xg = mesh.nodes[0]
        yg = mesh.nodes[1]
        tol = 1e-12
        ebc_node = (np.abs(xg + 1) < tol) | (np.abs(yg + 1) < tol)
        dof = np.zeros(dm.ndof)
        dof[ebc_node] = 0.2 * ((xg[ebc_node] + 1) + (yg[ebc_node] + 1))
        on_ebc = ebc_node[:dm.ndof_exterior].copy()
        assert not ebc_node[dm.ndof_exterior:].any()
        dm.solve(gsys, local_systems, dof, on_ebc)
        # global RHS vector F = sum_e scatter(JxW) (f = 1) for matrix-free solvers
        F = np.zeros(dm.ndof)
        for fe in dm.finite_elements(x_phys=True, Jacobian=True):
            np.add.at(F, fe.node_ind, fe.detJxW)
        out[name + "_nodes"] = mesh.nodes.copy()
        out[name + "_e2n"] = mesh_map(mesh)
        out[name + "_ebc"] = ebc_node
        out[name + "_rhs"] = F
        out[name + "_soln"] = dof
        out[name + "_p"] = np.array(p)
        out[name + "_n_ext"] = np.array(dm.ndof_exterior)
        print("  SC solve %s ndof=%d ext=%d |u|=%.16g max=%.16g" % (
            name, dm.ndof, dm.ndof_exterior, np.linalg.norm(dof), dof.max()))
    np.savez_compressed(os.path.join(OUT, "poisson_solution.npz"), **out)
    print("poisson_solution.npz")


def gen_axisym():
    from sem.discrete import DOFManager
    out = {}
    rng = np.random.default_rng(1)
    for name, p, nth, nr in [("p6_4x8", 6, 4, 8), ("p4_3x2", 4, 3, 2)]:
        nodes, e2n = annulus(nth, nr, p)
        mesh = ref_mesh(nodes, e2n)
        _, tb = ref_basis(p)
        dm = DOFManager(mesh, 2, tb, rcm_order=False)
        nn = mesh.n_nodes
        psi = rng.standard_normal(nn)
        om = rng.standard_normal(nn)
        yE = np.zeros(nn)
        yL = np.zeros(nn)
        yM = np.zeros(nn)
        for fe in dm.finite_elements(x_phys=True, Jacobian=True):
            E2e, Lve, Me_d = axisym_ops(fe)
            loc = fe.node_ind
            np.add.at(yE, loc, np.einsum("pqrs,rs", E2e, psi[loc]))
            np.add.at(yL, loc, np.einsum("pqrs,rs", Lve, om[loc]))
            np.add.at(yM, loc, Me_d * om[loc])
        # Stokes block (Re = 0), dpn = 2 interleaved (squirmer:97-98, 278-295):
        # y[2k] = Lve.omega ; y[2k+1] = E2e.psi - Me.omega
        sol = np.empty(2 * nn)
        sol[0::2] = psi
        sol[1::2] = om
        yb = np.empty(2 * nn)
        yb[0::2] = yL
        yb[1::2] = yE - yM
        out[name + "_nodes"] = mesh.nodes.copy()
        out[name + "_e2n"] = mesh_map(mesh)
        out[name + "_psi"] = psi
        out[name + "_omega"] = om
        out[name + "_E2e_psi"] = yE
        out[name + "_Lve_omega"] = yL
        out[name + "_Me_omega"] = yM
        out[name + "_soln"] = sol
        out[name + "_block"] = yb
        out[name + "_p"] = np.array(p)
        print("  axisym %s nodes=%d |yE|=%.6e |yL|=%.6e" % (name, nn, np.linalg.norm(yE), np.linalg.norm(yL)))
    np.savez_compressed(os.path.join(OUT, "axisym_action.npz"), **out)
    print("axisym_action.npz")


def axisym_Ae(fe, n_rey):
    """Advection operator of examples/squirmer-axisymmetric.py:229-250 (built
    with the reference's own KroneckerArray, sem/sp_array.py:11-113)."""
    from sem.sp_array import KroneckerArray
    JxW = fe.detJxW
    invJ = fe.invJ
    x = fe.x_phys
    dmats = fe.basis.get_D1_matrices()
    gradh_xi0 = np.einsum("imn,mp->imnp", invJ[0, :], dmats[0])
    gradh_xi1 = np.einsum("imn,nq->imnq", invJ[1, :], dmats[1])
    Ae = KroneckerArray(shape=fe.basis.coeff_shape * 3)
    Ae.add_diag(n_rey * (np.einsum("mn,mnr,mnu->mnru", JxW, gradh_xi0[0], gradh_xi1[1]) -
                         np.einsum("mn,mnr,mnu->mnru", JxW, gradh_xi0[1], gradh_xi1[0])),
                [0, 1, 2, 1, 0, 3])
    Ae.add_diag(n_rey * (np.einsum("mn,mns,mnt->mnst", JxW, gradh_xi1[0], gradh_xi0[1]) -
                         np.einsum("mn,mns,mnt->mnst", JxW, gradh_xi1[1], gradh_xi0[0])),
                [0, 1, 0, 2, 3, 1])
    Ae.add_diag(n_rey * np.einsum("mn,mnr->mnr", JxW / x[0], gradh_xi0[1]), [0, 1, 2, 1, 0, 1])
    Ae.add_diag(n_rey * np.einsum("mn,mns->mns", JxW / x[0], gradh_xi1[1]), [0, 1, 0, 2, 0, 1])
    return Ae


def gen_axisym_ns():
    """Navier-Stokes (Re > 0) squirmer residual and its Newton Jacobian:
    compute_local_system (examples/squirmer-axisymmetric.py:259-297) with
    the operators of pre_assembly (:193-254), Ae as the reference's
    KroneckerArray.  res[0::2] = Ae.w.psi + Lve.w, res[1::2] = E2e.psi -
    Me.w; the dense local Jacobian jac_l is assembled and applied to a
    random direction (the JVP golden)."""
    from sem.discrete import DOFManager
    from sem.sp_array import KroneckerArray
    np.float = float  # sem/sp_array.py:39 (NumPy >= 1.24 removed np.float)
    out = {}
    rng = np.random.default_rng(7)
    for name, p, nth, nr, n_rey in [("p6_4x8", 6, 4, 8, 3.7), ("p4_3x2", 4, 3, 2, 12.5)]:
        nodes, e2n = annulus(nth, nr, p)
        mesh = ref_mesh(nodes, e2n)
        _, tb = ref_basis(p)
        dm = DOFManager(mesh, 2, tb, rcm_order=False)
        nn = mesh.n_nodes
        sfn = rng.standard_normal(nn)
        vort = rng.standard_normal(nn)
        delta = rng.standard_normal(2 * nn)
        res = np.zeros(2 * nn)
        jvp = np.zeros(2 * nn)
        for fe in dm.finite_elements(x_phys=True, Jacobian=True):
            E2e, Lve, Me_d = axisym_ops(fe)
            Ae = axisym_Ae(fe, n_rey)
            Me = KroneckerArray(shape=fe.basis.coeff_shape * 2)
            Me.add_diag(Me_d, [0, 1, 0, 1])
            loc = fe.node_ind
            s_l, w_l = sfn[loc], vort[loc]
            n_nodes = loc.size
            Ae_w = Ae.dot_dense(w_l, [4, 5])
            r0 = Ae_w.dot_dense(s_l, [2, 3]).to_array() + np.einsum("pqrs,rs", Lve, w_l)
            r1 = np.einsum("pqrs,rs", E2e, s_l) - Me.dot_dense(w_l, [2, 3]).to_array()
            jac = np.zeros((2 * n_nodes, 2 * n_nodes))
            jac[0::2, 0::2] = Ae_w.to_array().reshape(n_nodes, n_nodes)
            jac[0::2, 1::2] = (Ae.dot_dense(s_l, [2, 3]).to_array() + Lve).reshape(n_nodes, n_nodes)
            jac[1::2, 0::2] = E2e.reshape(n_nodes, n_nodes)
            jac[1::2, 1::2] = -Me.to_array().reshape(n_nodes, n_nodes)
            dofs = (2 * loc.ravel()[:, None] + np.arange(2)[None, :]).ravel()
            np.add.at(res, 2 * loc.ravel(), r0.ravel())
            np.add.at(res, 2 * loc.ravel() + 1, r1.ravel())
            np.add.at(jvp, dofs, jac @ delta[dofs])
        sol = np.empty(2 * nn)
        sol[0::2], sol[1::2] = sfn, vort
        out[name + "_nodes"] = mesh.nodes.copy()
        out[name + "_e2n"] = mesh_map(mesh)
        out[name + "_p"] = np.array(p)
        out[name + "_re"] = np.array(n_rey)
        out[name + "_soln"] = sol
        out[name + "_res"] = res
        out[name + "_delta"] = delta
        out[name + "_jvp"] = jvp
        print("  axisym NS %s Re=%g |res|=%.6e |jvp|=%.6e" % (name, n_rey, np.linalg.norm(res),
                                                           np.linalg.norm(jvp)))
    np.savez_compressed(os.path.join(OUT, "axisym_ns.npz"), **out)
    print("axisym_ns.npz")


def gen_geometry():
    """Node orderings of sem/geometry.py (NCube hierarchical order :197-212,
    exterior/interior sets) and the DOFManagerSC condensation permutation
    (sem/discrete.py:314-359) on a small mesh."""
    from sem.geometry import Quadrilateral
    from sem.discrete import DOFManagerSC, DOFManager
    out = {}
    for shp in [(2, 2), (3, 3), (5, 5), (9, 9), (17, 17), (5, 6), (4, 7)]:
        q = Quadrilateral(*shp)
        key = "%dx%d" % shp
        out["hier_" + key] = q.hierarchical_node_order
        out["next_" + key] = np.array(q.n_exterior_nodes)
        out["nsub_" + key] = np.array([q.n_sub_geometries(d) for d in range(3)])
    nodes, e2n = structured_square(3, 2, 4, 0.0)
    for rcm in (False, True):
        mesh = ref_mesh(nodes, e2n)
        _, tb = ref_basis(4)
        dm = DOFManagerSC(mesh, 1, tb, rcm_order=rcm)
        out["sc_nodes_rcm%d" % rcm] = mesh.nodes.copy()
        out["sc_e2n_rcm%d" % rcm] = mesh_map(mesh)
        out["sc_next_rcm%d" % rcm] = np.array(dm.ndof_exterior)
        fe = next(dm.finite_elements())
        out["sc_gdof_hier_rcm%d" % rcm] = np.stack(
            [f.global_dof_ind_hier for f in dm.finite_elements()])
        out["sc_ldof_hier_rcm%d" % rcm] = fe.loc_dof_ind_hier
    mesh = ref_mesh(nodes, e2n)
    _, tb = ref_basis(4)
    DOFManager(mesh, 1, tb, rcm_order=True)
    out["rcm_nodes"] = mesh.nodes.copy()
    out["rcm_e2n"] = mesh_map(mesh)
    np.savez_compressed(os.path.join(OUT, "geometry.npz"), **out)
    print("geometry.npz")


def gen_msh():
    """Gmsh 2.2 binary meshes written by the package's writer
    (spectralelementmethod_amd.meshgen.write_square_msh: the square.geo
    stand-in) and read by the REFERENCE reader load_msh
    (sem/grid_importers.py:45-68).  The .msh files are committed as input
    fixtures; msh_reference.npz holds what the reference reader built."""
    sys.path.insert(1, os.path.dirname(os.path.dirname(OUT)))
    from spectralelementmethod_amd import meshgen
    import sem.grid_importers as gi
    out = {}
    cases = {"sq_p4": (3, 2, 4, 0.05), "sq_p2": (4, 3, 2, 0.0), "sq_p8": (2, 3, 8, 0.05)}
    for name, (nex, ney, p, warp) in cases.items():
        path = os.path.join(OUT, "mesh_%s.msh" % name)
        meshgen.write_square_msh(path, nex, ney, p, warp)
        mesh = gi.load_msh(path, 2)
        out[name + "_nodes"] = np.asarray(mesh.nodes, dtype=np.float64)
        out[name + "_e2n"] = mesh_map(mesh)
        out[name + "_region"] = np.array([cd.region_id for cd in mesh._cell_data])
        out[name + "_adj"] = np.array([[-1 if a is None else a for a in row]
                                       for row in mesh._adj_map], dtype=np.int64)
        rows = []
        for cell in sorted(mesh._boundary_map):
            for bid in sorted(mesh._boundary_map[cell]):
                for k, bd in enumerate(mesh._boundary_map[cell][bid]):
                    rows.append((cell, bid, k, bd.ndim, bd.index))
        out[name + "_bnd"] = np.array(rows, dtype=np.int64)
        out[name + "_region_names"] = np.array(mesh._region_names)
        out[name + "_boundary_names"] = np.array(mesh._boundary_names)
    np.savez_compressed(os.path.join(OUT, "msh_reference.npz"), **out)
    print("msh_reference.npz")


def ref_basis3(p):
    import sem.basis_functions as bf
    b1 = bf.LagrangeGaussLobatto(p)
    return b1, bf.TensorProductQS(b1, b1, b1)


def hex_Lse(invJ, JxW, D):
    """3-D element Laplacian [n^3, n^3] (RESTATED: examples/poisson.py:166-193
    with gradh = invJ . D per direction, written with Kronecker factors; the
    reference has no 3-D example)."""
    n = D.shape[0]
    I = np.eye(n)
    dphi = [np.kron(np.kron(D, I), I), np.kron(np.kron(I, D), I), np.kron(np.kron(I, I), D)]
    W = JxW.ravel()
    L = np.zeros((n ** 3, n ** 3))
    for x in range(3):
        g = sum(invJ[d, x].ravel()[:, None] * dphi[d] for d in range(3))
        L += g.T @ (W[:, None] * g)
    return L


def gen_hex():
    """Hexahedral goldens from the reference's N-dimensional basis layer:
    TensorProductQS(b, b, b).gradient / compute_coeffs_grid_eq
    (sem/basis_functions.py:599-650) and quad_rule.xweight
    (sem/quadratures.py:268-275) on random data, and Poisson actions on small
    warped hexahedral meshes whose per-element ingredients come from the same
    reference calls: x_phys = compute_coeffs_grid_eq(element nodes)
    (Mapping._compute_x_phys, sem/mapping.py:98-103), J = gradient(x_phys)
    .swapaxes(0, 1) (sem/mapping.py:113-114), detJxW = xweight(detJ)
    (sem/discrete.py:594-597).  The 3x3 det / inverse (numpy.linalg) and the
    element Laplacian (hex_Lse) are restatements: the reference stops at 2-D
    there (sem/mapping.py:110-111)."""
    sys.path.insert(1, os.path.dirname(os.path.dirname(OUT)))
    from spectralelementmethod_amd import meshgen
    rng = np.random.default_rng(11)
    out = {}
    for p in (2, 4, 8):
        _, tb = ref_basis3(p)
        c = rng.standard_normal((3, p + 1, p + 1, p + 1))
        out["c_%d" % p] = c
        out["grad_%d" % p] = tb.gradient(c)
        out["coeffs_eq_%d" % p] = tb.compute_coeffs_grid_eq(c)
        out["xweight_%d" % p] = tb.quad_rule.xweight(c)
    cases = [("p2_3x2x2w", 2, (3, 2, 2)), ("p3_2x2x2w", 3, (2, 2, 2)),
             ("p4_2x2x1w", 4, (2, 2, 1)), ("p5_1x2x1w", 5, (1, 2, 1))]
    for name, p, (nx, ny, nz) in cases:
        nodes, e2n = meshgen.structured_cube(nx, ny, nz, p, warp=0.05)
        _, tb = ref_basis3(p)
        D = tb.get_D1_matrices()[0]
        ndof = nodes.shape[1]
        u = rng.standard_normal(ndof)
        y = np.zeros(ndof)
        fields = {k: [] for k in ("x_phys", "J", "invJ", "detJ", "detJxW")}
        for e in range(e2n.shape[0]):
            X = nodes[:, e2n[e]]
            xp = tb.compute_coeffs_grid_eq(X)
            J = tb.gradient(xp).swapaxes(0, 1)
            Jm = np.moveaxis(J, (0, 1), (-2, -1))
            detJ = np.linalg.det(Jm)
            invJ = np.moveaxis(np.linalg.inv(Jm), (-2, -1), (0, 1))
            JxW = tb.quad_rule.xweight(detJ)
            L = hex_Lse(invJ, JxW, D)
            np.add.at(y, e2n[e].ravel(), L @ u[e2n[e]].ravel())
            for k, v in (("x_phys", xp), ("J", J), ("invJ", invJ), ("detJ", detJ),
                         ("detJxW", JxW)):
                fields[k].append(v)
        out[name + "_nodes"] = nodes
        out[name + "_e2n"] = e2n
        out[name + "_u"] = u
        out[name + "_y"] = y
        out[name + "_p"] = np.array(p)
        for k, v in fields.items():
            out[name + "_geom_" + k] = np.stack(v)
        print("  hex action %s ndof=%d |y|=%.6e" % (name, ndof, np.linalg.norm(y)))
    np.savez_compressed(os.path.join(OUT, "hex.npz"), **out)
    print("hex.npz")


GENERATORS = {"gll": gen_gll, "tensor_ops": gen_tensor_ops, "poisson_action": gen_poisson_action,
              "poisson_solution": gen_poisson_solution, "axisym": gen_axisym,
              "geometry": gen_geometry, "msh": gen_msh, "axisym_ns": gen_axisym_ns,
              "hex": gen_hex}


def main(names=None):
    _TABLES.update(decode_basis_hdf5())
    install_runtime_shims()
    for name in (names or list(GENERATORS)):
        if name not in ("gll", "msh") and len(_TABLES) < 16:
            # extended-order tables are needed by every generator
            import sem.basis_data as bd
            for p in range(11, MAX_ORDER_EXT + 1):
                nodes, bary, qw = bd.gauss_legendre_lobatto(p + 1)
                _TABLES[p] = np.array([[float(v) for v in mat] for mat in (nodes, bary, qw)])
        GENERATORS[name]()


if __name__ == "__main__":
    main(sys.argv[1:] or None)
