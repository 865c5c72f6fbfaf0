"""GPU parity of the hexahedral (3-D) Poisson path: libsem_hip.so through the
C ABI (sem_ctx_create_nd, ndim = 3) against

* the goldens built from the reference's own N-D basis calls
  (tests/golden/hex.npz: TensorProductQS(b, b, b).compute_coeffs_grid_eq /
  gradient / quad_rule.xweight, sem/basis_functions.py:599-650,
  sem/quadratures.py:268-275), p = 2..5, warped hexahedra;
* the extrusion identity K3 (u (x) 1) = (K2 u) (x) (M_z 1) on the reference's
  2-D golden meshes swept along z: the 3-D action pinned to the reference's
  own 2-D action output;
* the NumPy oracle (oracle/sem_oracle.py, HexPoissonProblem, itself pinned to
  the two above) at every built order p = 1..16 (above p = 10 its extended-
  precision twin), on broken-chain numberings and at ~1e7 DOF (p = 8, 27^3
  hexahedra; p = 16, 13^3) at the north-star 1e-10.

The 3x3 determinant / inverse and the 3-D element operator have no reference
counterpart (sem/mapping.py:110-111 stops at 2-D): beyond the extrusion
identity they are "parity unpinned" restatements."""
import numpy as np
import pytest

from conftest import rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-12        # small meshes, vs reference goldens / oracle
TOL_FULL = 1e-10   # BASELINE.json north_star at ~1e7 DOF
TOL_HI = 1e-11     # p = 11..16 vs the extended-precision oracle (small meshes)
HEX_CASES = ["p2_3x2x2w", "p3_2x2x2w", "p4_2x2x1w", "p5_1x2x1w"]


@pytest.fixture(scope="module")
def sem():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from spectralelementmethod_amd import operators
    return operators


def _oracle(gll, nodes, e2n, p):
    import sem_oracle
    return sem_oracle.HexPoissonProblem(nodes, e2n, gll["half_%d" % p])


@pytest.mark.parametrize("name", HEX_CASES)
def test_hex_action_golden(sem, hex_golden, name):
    p = int(hex_golden[name + "_p"])
    op = sem.SEMOperator(p, hex_golden[name + "_e2n"], hex_golden[name + "_nodes"])
    assert op.ndim == 3
    y = op.apply(torch.from_numpy(hex_golden[name + "_u"]).cuda()).cpu().numpy()
    assert rel_l2(y, hex_golden[name + "_y"]) < TOL


@pytest.mark.parametrize("name", HEX_CASES)
def test_hex_geometry_fields_golden(sem, hex_golden, name):
    p = int(hex_golden[name + "_p"])
    op = sem.SEMOperator(p, hex_golden[name + "_e2n"], hex_golden[name + "_nodes"])
    f = op.geometry_fields()
    for k in ("x_phys", "J", "invJ", "detJ", "detJxW"):
        assert rel_l2(f[k].cpu().numpy(), hex_golden[name + "_geom_" + k]) < TOL, k


@pytest.mark.parametrize("name,nez", [("p8_8x8w", 3), ("p4_4x4", 5), ("p6_3x4w", 2),
                                      ("p2_6x5", 4)])
def test_hex_extrusion_identity(sem, gll, poisson_action, name, nez):
    """3-D action of u2 (x) 1 on the extruded reference mesh = the
    reference's 2-D golden action times the assembled z mass."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    p = int(poisson_action[name + "_p"])
    z0, z1 = -0.5, 0.25
    nodes3, e2n3 = meshgen.extrude(poisson_action[name + "_nodes"], poisson_action[name + "_e2n"],
                                   nez, p, z0, z1)
    op = sem.SEMOperator(p, e2n3, nodes3)
    Nz = nez * p + 1
    u = torch.from_numpy(np.repeat(poisson_action[name + "_u"], Nz)).cuda()
    y = op.apply(u).cpu().numpy()
    _, _, quad = sem_oracle.gll_unfold(gll["half_%d" % p])
    mz = np.zeros(Nz)
    for ez in range(nez):
        mz[ez * p:ez * p + p + 1] += 0.5 * (z1 - z0) / nez * quad
    assert rel_l2(y, np.outer(poisson_action[name + "_y"], mz).ravel()) < TOL


@pytest.mark.parametrize("p", range(1, 17))
def test_hex_orders_vs_oracle(sem, gll, p):
    """Every built order.  Above p = 10 the equispaced->GLL transform is
    ill-conditioned and the float64 oracle itself is off by
    7e-12 (p = 12) to 1e-8 (p = 16): the yardstick there is the extended-
    precision evaluation of the same action from the same float64 inputs
    (hex_poisson_apply_extended), and the device (compensated transform,
    k_hex_eq2gll_pass) must be within TOL_HI of it and no further from it
    than the float64 oracle."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    ne = {1: 6, 2: 5, 3: 4, 4: 3, 5: 3}.get(p, 2)
    nodes, e2n = meshgen.structured_cube(ne + 1, ne, ne - 1 if ne > 2 else 2, p, warp=0.05)
    P = _oracle(gll, nodes, e2n, p)
    op = sem.SEMOperator(p, e2n, nodes)
    u = np.random.default_rng(p).standard_normal(P.ndof)
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    if p <= 10:
        assert rel_l2(y, P.apply(u)) < TOL
    else:
        ext = np.asarray(sem_oracle.hex_poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u),
                         dtype=np.float64)
        err, err_f64 = rel_l2(y, ext), rel_l2(P.apply(u), ext)
        print("p=%d device vs extended %.2e, float64 oracle vs extended %.2e" % (p, err, err_f64))
        assert err < TOL_HI and err <= max(err_f64, TOL)
    info = op.plan_info()
    assert info["ndim"] == 3 and info["chains"] == ne * (ne - 1 if ne > 2 else 2)
    assert info["hex_kernel"] == ("rows" if p >= 13 else "three_block")


def test_hex_full_size_p16(sem, gll):
    """~1e7 DOF at the highest order: p = 16, 13^3 warped hexahedra
    (9,129,329 DOF) against the extended-precision oracle at the north-star
    1e-10 (the float64 oracle's own error there is ~1e-8)."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    p, ne = 16, 13
    nodes, e2n = meshgen.structured_cube(ne, ne, ne, p, warp=0.05)
    op = sem.SEMOperator(p, e2n, nodes)
    u = np.random.default_rng(16).standard_normal(nodes.shape[1])
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    ext = np.asarray(sem_oracle.hex_poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u),
                     dtype=np.float64)
    err = rel_l2(y, ext)
    print("p=16 13^3: device vs extended %.2e" % err)
    assert err < TOL_FULL


@pytest.mark.parametrize("p", [3, 6, 8, 10])
@pytest.mark.parametrize("form", ["rows_zmerge", "rows", "three_block_zmerge", "three_block"])
def test_hex_kernel_forms_vs_oracle(sem, gll, monkeypatch, p, form):
    """Both action kernels at every order class, whatever AUTO picks: the row
    form and the three-block kernel, each with and without the xi2-face
    z-merge, overwrite and accumulate, on a warped mesh with several slots
    per workgroup and broken sub-chains."""
    from spectralelementmethod_amd import meshgen
    monkeypatch.setenv("SEM_HEX_ROWS", "1" if form.startswith("rows") else "0")
    monkeypatch.setenv("SEM_HEX_ZMERGE", "1" if form.endswith("zmerge") else "0")
    ne = {3: 4, 6: 3}.get(p, 2)
    nodes, e2n = meshgen.structured_cube(ne + 2, ne + 1, ne, p, warp=0.05)
    P = _oracle(gll, nodes, e2n, p)
    op = sem.SEMOperator(p, e2n, nodes)
    rng = np.random.default_rng(10 + p)
    u = rng.standard_normal(P.ndof)
    y0 = rng.standard_normal(P.ndof)
    ref = P.apply(u)
    info = op.plan_info()
    assert info["hex_kernel"] == ("rows" if form.startswith("rows") else "three_block")
    assert info["zmerge"] == form.endswith("zmerge")
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    assert rel_l2(y, ref) < TOL
    yt = torch.from_numpy(y0.copy()).cuda()
    op.apply(torch.from_numpy(u).cuda(), out=yt, accumulate=True)
    assert rel_l2(yt.cpu().numpy(), y0 + ref) < TOL
    if form.endswith("zmerge") and p <= 6:  # the diagonal runs on the z-merged plan too
        L = P.element_matrices()
        dref = np.bincount(P.e2n.reshape(P.e2n.shape[0], -1).ravel(),
                           weights=np.einsum("eii->ei", L).ravel(), minlength=P.ndof)
        assert rel_l2(op.diag().cpu().numpy(), dref) < TOL


@pytest.mark.parametrize("p,gy,gz", [(1, 8, 8), (2, 4, 7), (3, 4, 4), (4, 2, 5), (7, 2, 2)])
def test_hex_ymerge_vs_oracle(sem, gll, monkeypatch, p, gy, gz):
    """The y-merge (the workgroup's slots as a gy x gz grid, xi1 faces between
    its rows summed in LDS as well as the xi2 faces within a row): action,
    accumulate and diagonal against the oracle with it on and off, on a
    warped mesh sized so that full grids, a grid cut short at the mesh edge
    and the 1-D fallback all occur; fewer seam nodes with it on."""
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_cube(3, 2 * gy + 1, gz + 1, p, warp=0.05)
    P = _oracle(gll, nodes, e2n, p)
    rng = np.random.default_rng(40 + p)
    u = rng.standard_normal(P.ndof)
    y0 = rng.standard_normal(P.ndof)
    ref = P.apply(u)
    L = P.element_matrices()
    dref = np.bincount(P.e2n.reshape(P.e2n.shape[0], -1).ravel(),
                       weights=np.einsum("eii->ei", L).ravel(), minlength=P.ndof)
    seams = {}
    monkeypatch.setenv("SEM_HEX_ROWS", "0")
    monkeypatch.setenv("SEM_HEX_ZMERGE", "1")
    for ym in ("1", "0"):
        monkeypatch.setenv("SEM_HEX_YMERGE", ym)
        op = sem.SEMOperator(p, e2n, nodes)
        info = op.plan_info()
        assert info["ymerge"] == (ym == "1")
        if ym == "1":
            assert tuple(info["slot_grid"]) == (gy, gz)
        seams[ym] = info["seam_nodes"]
        y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
        assert rel_l2(y, ref) < TOL, ym
        yt = torch.from_numpy(y0.copy()).cuda()
        op.apply(torch.from_numpy(u).cuda(), out=yt, accumulate=True)
        assert rel_l2(yt.cpu().numpy(), y0 + ref) < TOL, ym
        assert rel_l2(op.diag().cpu().numpy(), dref) < TOL, ym
    assert seams["1"] < seams["0"], seams


@pytest.mark.parametrize("rows", ["0", "1"])
@pytest.mark.parametrize("p", [2, 5, 8])
def test_hex_template_map_bitwise(sem, monkeypatch, p, rows):
    """The template map (one base per element, the column's offsets in
    registers) gives the per-element map's action and diagonal bit for bit
    on a structured cube, in both kernel forms; shuffled node ids keep the
    map."""
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_cube(5, 4, 3, p, warp=0.05)
    u = torch.from_numpy(np.random.default_rng(p).standard_normal(nodes.shape[1])).cuda()
    out = {}
    monkeypatch.setenv("SEM_HEX_ROWS", rows)
    for tm in ("1", "0"):
        monkeypatch.setenv("SEM_HEX_TMAP", tm)
        op = sem.SEMOperator(p, e2n, nodes)
        assert op.plan_info()["template_map"] == (tm == "1")
        out[tm] = (op.apply(u).cpu().numpy(), op.diag().cpu().numpy())
    assert np.array_equal(out["1"][0], out["0"][0])
    assert np.array_equal(out["1"][1], out["0"][1])
    monkeypatch.delenv("SEM_HEX_TMAP")
    perm = np.random.default_rng(1).permutation(nodes.shape[1])
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size)
    op = sem.SEMOperator(p, inv[e2n.astype(np.int64)].astype(np.uint32), nodes[:, perm])
    assert not op.plan_info()["template_map"]


def _permute_local(e2n, rng, frac=0.5):
    """Re-orient a fraction of the elements (swap / reverse local axes): the
    mesh is the same, the xi0 chains break wherever orientations differ."""
    e2n = e2n.copy()
    for e in np.flatnonzero(rng.random(e2n.shape[0]) < frac):
        perm = rng.permutation(3)
        flips = rng.random(3) < 0.5
        # orientation-preserving only (a reflection would make detJ < 0)
        sign = np.linalg.det(np.eye(3)[perm]) * (-1) ** int(flips.sum())
        if sign < 0:
            flips[0] = not flips[0]
        t = np.transpose(e2n[e], perm)
        for ax in range(3):
            if flips[ax]:
                t = np.flip(t, axis=ax)
        e2n[e] = t
    return e2n


@pytest.mark.parametrize("case", ["shuffle_elements", "shuffle_nodes", "reoriented",
                                  "reoriented_shuffled"])
def test_hex_broken_chains_vs_oracle(sem, gll, case):
    """The planner on numberings that defeat the chains: still exact."""
    from spectralelementmethod_amd import meshgen
    p = 4
    nodes, e2n = meshgen.structured_cube(4, 3, 3, p, warp=0.05)
    rng = np.random.default_rng(5)
    if case in ("shuffle_elements", "reoriented_shuffled"):
        e2n = meshgen.shuffle_elements(e2n, seed=3)
    if case == "shuffle_nodes":
        nodes, e2n = meshgen.shuffle_nodes(nodes, e2n, seed=4)
    if case.startswith("reoriented"):
        e2n = _permute_local(e2n, rng)
    P = _oracle(gll, nodes, e2n, p)
    op = sem.SEMOperator(p, e2n, nodes)
    u = rng.standard_normal(P.ndof)
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    assert rel_l2(y, P.apply(u)) < TOL


def test_hex_accumulate_diag_assemble_and_set_geometry(sem, gll):
    from spectralelementmethod_amd import meshgen
    p = 5
    nodes, e2n = meshgen.structured_cube(3, 2, 2, p, warp=0.05)
    P = _oracle(gll, nodes, e2n, p)
    op = sem.SEMOperator(p, e2n, nodes)
    rng = np.random.default_rng(9)
    u = torch.from_numpy(rng.standard_normal(P.ndof)).cuda()
    y0 = torch.from_numpy(rng.standard_normal(P.ndof)).cuda()
    y = y0.clone()
    op.apply(u, out=y, accumulate=True)
    ref = y0.cpu().numpy() + P.apply(u.cpu().numpy())
    assert rel_l2(y.cpu().numpy(), ref) < TOL
    # diagonal of the assembled operator
    L = P.element_matrices()
    dref = np.bincount(P.e2n.reshape(P.e2n.shape[0], -1).ravel(),
                       weights=np.einsum("eii->ei", L).ravel(), minlength=P.ndof)
    assert rel_l2(op.diag().cpu().numpy(), dref) < TOL
    # load vector of f = 1 (sem_assemble of detJxW)
    f = op.geometry_fields()["detJxW"]
    F = op.assemble(f).cpu().numpy()
    Fref = np.bincount(P.e2n.ravel(), weights=P.detJxW.ravel(), minlength=P.ndof)
    assert rel_l2(F, Fref) < TOL
    # caller-installed factors give the same action
    op2 = sem.SEMOperator(p, e2n, nodes)
    op2.set_geometry(P.G)
    assert rel_l2(op2.apply(u).cpu().numpy(), ref - y0.cpu().numpy()) < TOL


def test_hex_apply_is_deterministic(sem):
    from spectralelementmethod_amd import meshgen
    p = 6
    nodes, e2n = meshgen.structured_cube(5, 4, 3, p, warp=0.05)
    op = sem.SEMOperator(p, e2n, nodes)
    u = torch.from_numpy(np.random.default_rng(1).standard_normal(nodes.shape[1])).cuda()
    y1 = op.apply(u).clone()
    for _ in range(3):
        assert torch.equal(op.apply(u), y1)


def test_hex_detj_nonpositive_raises(sem):
    from spectralelementmethod_amd import meshgen
    p = 3
    nodes, e2n = meshgen.structured_cube(2, 2, 2, p)
    e2n = e2n.copy()
    e2n[1] = e2n[1][::-1]  # mirrored element: detJ < 0
    op = sem.SEMOperator(p, e2n, nodes)
    with pytest.raises(AssertionError):
        op.compute_geometry()


def test_hex_pcg_vs_direct_solve(sem, gll):
    """Assembled 3-D Poisson solve on the device (Jacobi-PCG, sem_pcg_solve)
    against a direct sparse solve of the oracle's assembled K (u = 0.2 (x +
    y + z + 3) on the x = -1 and y = -1 faces, f = 1)."""
    import scipy.sparse as sps
    import scipy.sparse.linalg as spsl
    from spectralelementmethod_amd import meshgen
    p = 4
    nodes, e2n = meshgen.structured_cube(3, 3, 2, p, warp=0.05)
    P = _oracle(gll, nodes, e2n, p)
    L = P.element_matrices()
    E, nl = L.shape[0], L.shape[1]
    loc = P.e2n.reshape(E, nl)
    K = sps.coo_matrix((L.ravel(), (np.repeat(loc, nl, axis=1).ravel(),
                                    np.tile(loc, (1, nl)).ravel())),
                       shape=(P.ndof, P.ndof)).tocsr()
    F = np.bincount(P.e2n.ravel(), weights=P.detJxW.ravel(), minlength=P.ndof)
    x, yv, zv = nodes
    ebc = (np.abs(x + 1) < 1e-12) | (np.abs(yv + 1) < 1e-12)
    g = np.where(ebc, 0.2 * (x + yv + zv + 3), 0.0)
    free = ~ebc
    ref = g.copy()
    ref[free] = spsl.spsolve(K[free][:, free].tocsc(), F[free] - K[free][:, ebc] @ g[ebc])
    op = sem.SEMOperator(p, e2n, nodes)
    xd = torch.from_numpy(g.copy()).cuda()
    xd, its, rel = op.pcg_solve(torch.from_numpy(F).cuda(), xd, ebc, rtol=1e-14,
                                max_iter=5000)
    assert rel_l2(xd.cpu().numpy(), ref) < 1e-10, (its, rel)


def test_hex_full_size_p8(sem, gll):
    """~1e7 DOF: p = 8, 27^3 warped hexahedra (10,218,313 DOF) vs the oracle
    at the north-star 1e-10; the plan forms chains along xi0."""
    from spectralelementmethod_amd import meshgen
    p, ne = 8, 27
    nodes, e2n = meshgen.structured_cube(ne, ne, ne, p, warp=0.05)
    P = _oracle(gll, nodes, e2n, p)
    op = sem.SEMOperator(p, e2n, nodes)
    u = np.random.default_rng(27).standard_normal(P.ndof)
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    assert rel_l2(y, P.apply(u)) < TOL_FULL
    info = op.plan_info()
    assert info["chains"] == ne * ne and info["plain_stores"] > 0
