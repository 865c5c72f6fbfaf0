"""GPU parity: libsem_hip.so (through the C ABI) vs the reference's golden
vectors and the NumPy oracle.  Tolerances: the north-star bar is 1e-10
relative L2 for the stiffness action and the assembled solution; the kernels
meet 1e-12 on every golden case (fp64 throughout)."""
import numpy as np
import pytest

from conftest import rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL_ACTION = 1e-12      # Poisson stiffness action vs reference golden
TOL_AXISYM = 1e-12      # axisymmetric block vs reference golden
TOL_GEOM = 1e-12        # x_phys, J, invJ, detJ, detJxW vs reference golden
TOL_SOLVE = 1e-10       # assembled Poisson solution vs reference DOFManagerSC.solve

ACTION_CASES = ["p4_4x4", "p8_8x8w", "p8_8x8w_rcm", "p2_6x5", "p6_3x4w", "p12_3x3w", "p16_2x2w"]


@pytest.fixture(scope="module")
def sem():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from spectralelementmethod_amd import operators
    return operators


GEOMETRY = ["nodal", "stored"]


def make_op(sem, fx, name, dpn=1, geometry="nodal"):
    p = int(fx[name + "_p"])
    return sem.SEMOperator(p, fx[name + "_e2n"], fx[name + "_nodes"], dofs_per_node=dpn,
                           geometry=geometry)


def assert_parity(y, y_ref, y_ext, tol):
    """Pass when y matches the reference within ``tol`` relative L2; where
    the reference's own float64 rounding (measured against the
    extended-precision oracle y_ext) exceeds tol (p > 10: cond(V_eq) * eps),
    y must be at least as accurate as the reference and agree with it to
    twice the reference's own error."""
    e_ref = rel_l2(y, y_ref)
    if e_ref < tol:
        return
    assert y_ext is not None, e_ref
    e_self = rel_l2(y, y_ext)
    e_refx = rel_l2(y_ref, y_ext)
    assert e_self <= max(1.5 * e_refx, tol), (e_self, e_refx)
    assert e_ref <= 2.0 * e_refx + tol, (e_ref, e_refx)


@pytest.mark.parametrize("geometry", GEOMETRY)
@pytest.mark.parametrize("name", ACTION_CASES)
def test_poisson_action_golden(sem, poisson_action, gll, name, geometry):
    import sem_oracle
    op = make_op(sem, poisson_action, name, geometry=geometry)
    u = torch.from_numpy(poisson_action[name + "_u"]).cuda()
    y = op.apply(u).cpu().numpy()
    p = int(poisson_action[name + "_p"])
    y_ext = None
    if p > 10:
        y_ext = sem_oracle.poisson_apply_extended(poisson_action[name + "_nodes"],
                                                  poisson_action[name + "_e2n"],
                                                  gll["half_%d" % p], poisson_action[name + "_u"])
    assert_parity(y, poisson_action[name + "_y"], y_ext, TOL_ACTION)


def test_poisson_accumulate(sem, poisson_action):
    name = "p8_8x8w"
    op = make_op(sem, poisson_action, name)
    u = torch.from_numpy(poisson_action[name + "_u"]).cuda()
    y0 = torch.linspace(-1, 1, u.numel(), dtype=torch.float64, device="cuda")
    y = y0.clone()
    op.apply(u, out=y, accumulate=True)
    ref = y0.cpu().numpy() + poisson_action[name + "_y"]
    assert rel_l2(y.cpu().numpy(), ref) < TOL_ACTION
    # overwrite mode must not depend on the previous contents of out
    y.fill_(123.0)
    op.apply(u, out=y, accumulate=False)
    assert rel_l2(y.cpu().numpy(), poisson_action[name + "_y"]) < TOL_ACTION


@pytest.mark.parametrize("name", ["p4_4x4", "p8_8x8w"])
def test_geometry_fields_golden(sem, poisson_action, name):
    op = make_op(sem, poisson_action, name)
    f = op.geometry_fields()
    for key in ("x_phys", "J", "invJ", "detJ", "detJxW"):
        got = f[key].cpu().numpy()
        ref = poisson_action[name + "_geom_" + key]
        assert got.shape == ref.shape, key
        assert rel_l2(got, ref) < TOL_GEOM, key


@pytest.mark.parametrize("geometry", GEOMETRY)
@pytest.mark.parametrize("name", ["p6_4x8", "p4_3x2"])
def test_axisym_block_golden(sem, axisym_action, name, geometry):
    op = make_op(sem, axisym_action, name, dpn=2, geometry=geometry)
    sol = torch.from_numpy(axisym_action[name + "_soln"]).cuda()
    y = op.apply(sol, kind="axisym_stokes").cpu().numpy()
    assert op.plan_info()["geometry_axisym"] == geometry
    ref = axisym_action[name + "_block"]
    assert rel_l2(y[0::2], ref[0::2]) < TOL_AXISYM     # Lve . omega
    assert rel_l2(y[1::2], ref[1::2]) < TOL_AXISYM     # E2e . psi - Me . omega


@pytest.mark.parametrize("geometry", GEOMETRY)
def test_axisym_components_golden(sem, axisym_action, geometry):
    """Separate E2e.psi, Lve.omega and Me.omega via zeroed inputs."""
    name = "p6_4x8"
    op = make_op(sem, axisym_action, name, dpn=2, geometry=geometry)
    psi = axisym_action[name + "_psi"]
    om = axisym_action[name + "_omega"]
    z = np.zeros_like(psi)
    s = np.empty(2 * psi.size)
    s[0::2], s[1::2] = psi, z
    y = op.apply(torch.from_numpy(s).cuda(), kind="axisym_stokes").cpu().numpy()
    assert rel_l2(y[1::2], axisym_action[name + "_E2e_psi"]) < TOL_AXISYM
    assert np.abs(y[0::2]).max() == 0.0
    s[0::2], s[1::2] = z, om
    y = op.apply(torch.from_numpy(s).cuda(), kind="axisym_stokes").cpu().numpy()
    assert rel_l2(y[0::2], axisym_action[name + "_Lve_omega"]) < TOL_AXISYM
    assert rel_l2(-y[1::2], axisym_action[name + "_Me_omega"]) < TOL_AXISYM


@pytest.mark.parametrize("geometry", GEOMETRY)
def test_poisson_vs_oracle_larger(sem, gll, geometry):
    """128 x 96 warped mesh at p = 8 vs the batched NumPy oracle (and the
    extended-precision oracle: small elements make J = D x_phys cancel
    O(1) coordinates against O(h) variations in the reference algorithm)."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    p = 8
    nodes, e2n = meshgen.structured_square(128, 96, p, warp=0.05)
    prob = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True)
    u = np.random.default_rng(5).standard_normal(prob.ndof)
    op = sem.SEMOperator(p, e2n, nodes, geometry=geometry)
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    y_ext = sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u)
    assert_parity(y, prob.apply(u), y_ext, TOL_ACTION)


@pytest.mark.parametrize("p", [1, 2, 3, 5, 7, 9, 10, 11, 13, 14, 15])
def test_poisson_all_orders_vs_oracle(sem, gll, p):
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_square(5, 4, p, warp=0.05)
    prob = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p])
    u = np.random.default_rng(p).standard_normal(prob.ndof)
    op = sem.SEMOperator(p, e2n, nodes)
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    y_ext = sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u)
    assert_parity(y, prob.apply(u), y_ext, TOL_ACTION)


@pytest.mark.parametrize("geometry", GEOMETRY)
@pytest.mark.parametrize("p,ney", [(8, 14), (8, 143), (4, 36), (6, 27)])
def test_map16_matches_32bit_map(sem, gll, monkeypatch, p, ney, geometry):
    """16-bit packed map (one base per group row) against the
    32-bit map: the same arithmetic in the same order (the two kernel
    instantiations may contract FMAs differently: agreement to 1e-14), both
    within tolerance of the oracle.  ney = 143 at p = 8 makes ~5 % of the
    groups wrap into the next element column: those read the 32-bit map
    inside the same launch (per-group fallback)."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_square(max(6, ney // 4), ney, p, warp=0.05)
    u = np.random.default_rng(p + ney).standard_normal(nodes.shape[1])
    # chains of consecutive elements (at p = 4, ney = 36 a chain spans two
    # element columns and the planner would pick element-coloured chains)
    monkeypatch.setenv("SEM_PLAN", "0")
    op16 = sem.SEMOperator(p, e2n, nodes, geometry=geometry)
    assert op16.plan_info()["map_entry_bytes"] == 2
    y16 = op16.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    monkeypatch.setenv("SEM_MAP16", "0")
    op32 = sem.SEMOperator(p, e2n, nodes, geometry=geometry)
    assert op32.plan_info()["map_entry_bytes"] == 4
    y32 = op32.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    assert rel_l2(y16, y32) < 1e-14
    ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p]).apply(u)
    # small elements: the oracle's float64 geometry (O(1) coordinates, as in
    # the reference) loses digits; judge both against extended precision
    y_ext = sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u)
    assert_parity(y16, ref, y_ext, TOL_ACTION)
    assert_parity(y32, ref, y_ext, TOL_ACTION)


def test_properties_full_size(sem):
    """Size-independent properties on a 512 x 512 p = 8 mesh (16.8M DOF):
    constants in the kernel, symmetry, linearity, run-to-run agreement."""
    from spectralelementmethod_amd import meshgen
    p = 8
    nodes, e2n = meshgen.structured_square(512, 512, p, warp=0.05)
    op = sem.SEMOperator(p, e2n, nodes)
    g = torch.Generator(device="cuda").manual_seed(1)
    u = torch.randn(op.ndof, dtype=torch.float64, device="cuda", generator=g)
    v = torch.randn(op.ndof, dtype=torch.float64, device="cuda", generator=g)
    Ku = op.apply(u)
    Kv = op.apply(v)
    # symmetric positive semi-definite stiffness
    a, b = torch.dot(v, Ku).item(), torch.dot(u, Kv).item()
    assert abs(a - b) <= 1e-11 * max(abs(a), abs(b))
    assert torch.dot(u, Ku).item() > 0
    # Neumann Laplacian annihilates constants
    ones = torch.ones_like(u)
    K1 = op.apply(ones)
    assert K1.abs().max().item() < 1e-10 * Ku.abs().max().item()
    # linearity
    K_lin = op.apply(2.0 * u - 3.0 * v)
    assert (K_lin - (2.0 * Ku - 3.0 * Kv)).norm().item() < 1e-13 * K_lin.norm().item()
    # repeated application agrees (atomics may reorder fp adds: <= 1e-14)
    Ku2 = op.apply(u)
    assert (Ku2 - Ku).norm().item() <= 1e-14 * Ku.norm().item()


def test_nodal_vs_stored_full_size(sem):
    """The two geometry modes agree at 16.8M DOF (they differ only in where
    x_phys is rounded to absolute coordinates)."""
    from spectralelementmethod_amd import meshgen
    p = 8
    nodes, e2n = meshgen.structured_square(512, 512, p, warp=0.05)
    g = torch.Generator(device="cuda").manual_seed(3)
    ys = []
    for geometry in GEOMETRY:
        op = sem.SEMOperator(p, e2n, nodes, geometry=geometry)
        u = torch.randn(op.ndof, dtype=torch.float64, device="cuda",
                        generator=g.manual_seed(3))
        ys.append(op.apply(u))
        del op
    assert (ys[0] - ys[1]).norm().item() < 1e-11 * ys[1].norm().item()


def test_detj_nonpositive_raises(sem, poisson_action):
    name = "p4_4x4"
    e2n = poisson_action[name + "_e2n"].copy()
    e2n[3] = e2n[3][::-1, :]  # mirror one element: negative orientation
    with pytest.raises(AssertionError):
        op = sem.SEMOperator(4, e2n, poisson_action[name + "_nodes"])
        op.compute_geometry()


def test_bad_inputs_raise(sem, poisson_action):
    name = "p4_4x4"
    nodes = poisson_action[name + "_nodes"]
    e2n = poisson_action[name + "_e2n"]
    with pytest.raises(ValueError):
        sem.SEMOperator(4, e2n[:, :3, :3], nodes)
    bad = e2n.copy()
    bad[0, 0, 0] = nodes.shape[1] + 5
    with pytest.raises(ValueError):
        sem.SEMOperator(4, bad, nodes)
    op = sem.SEMOperator(4, e2n, nodes)
    with pytest.raises(ValueError):
        op.apply(torch.zeros(7, dtype=torch.float64, device="cuda"))
    with pytest.raises(ValueError):
        op.apply(torch.zeros(op.ndof, dtype=torch.float64, device="cuda"), kind="axisym_stokes")


def test_unreferenced_nodes_zeroed(sem, poisson_action):
    """Nodes no element references get y = 0 in overwrite mode."""
    name = "p4_4x4"
    nodes = poisson_action[name + "_nodes"]
    extra = np.concatenate([nodes, np.array([[5.0, 6.0], [5.0, 6.0]])], axis=1)
    op = sem.SEMOperator(4, poisson_action[name + "_e2n"], extra)
    u = np.concatenate([poisson_action[name + "_u"], [1.0, 2.0]])
    y = torch.full((op.ndof,), 7.0, dtype=torch.float64, device="cuda")
    op.apply(torch.from_numpy(u).cuda(), out=y)
    y = y.cpu().numpy()
    assert y[-2] == 0.0 and y[-1] == 0.0
    assert rel_l2(y[:-2], poisson_action[name + "_y"]) < TOL_ACTION


def test_nonconforming_map_all_atomic(sem, poisson_action, gll):
    """A map where an element-interior node is shared falls back to the
    all-atomic kernel and still matches the oracle."""
    import sem_oracle
    name = "p4_4x4"
    nodes = poisson_action[name + "_nodes"]
    e2n = poisson_action[name + "_e2n"].copy()
    e2n = np.concatenate([e2n, e2n[:2]])  # duplicate two elements
    op = sem.SEMOperator(4, e2n, nodes)
    prob = sem_oracle.PoissonProblem(nodes, e2n, gll["half_4"])
    u = poisson_action[name + "_u"]
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    assert rel_l2(y, prob.apply(u)) < TOL_ACTION


@pytest.mark.parametrize("p", [2, 4, 8, 12])
def test_tensor_ops_golden(sem, tensor_ops, p):
    from spectralelementmethod_amd.basis_functions import gll_basis_2d
    tb = gll_basis_2d(p)
    c = tensor_ops["c_%d" % p]
    assert rel_l2(tb.gradient(c), tensor_ops["grad_%d" % p]) < 1e-13
    assert rel_l2(tb.compute_coeffs_grid_eq(c), tensor_ops["coeffs_eq_%d" % p]) < 1e-12
    back = tb.interpolate_on_grid_eq(tb.compute_coeffs_grid_eq(c))
    assert rel_l2(back, c) < 1e-12


def test_poisson_solution_golden(sem, poisson_solution):
    """Assembled Poisson solution (matrix-free PCG on the GPU) vs the
    reference's static-condensation solve DOFManagerSC.solve."""
    for name in ("p4_8x8", "p8_4x4w"):
        fx = poisson_solution
        p = int(fx[name + "_p"])
        op = sem.SEMOperator(p, fx[name + "_e2n"], fx[name + "_nodes"])
        ebc = fx[name + "_ebc"]
        x = torch.zeros(op.ndof, dtype=torch.float64, device="cuda")
        ref = fx[name + "_soln"]
        x[torch.from_numpy(ebc).cuda()] = torch.from_numpy(ref[ebc]).cuda()
        x, its, rel = op.pcg_solve(torch.from_numpy(fx[name + "_rhs"]).cuda(), x, ebc, rtol=1e-13)
        assert rel_l2(x.cpu().numpy(), ref) < TOL_SOLVE, (name, its, rel)


@pytest.mark.parametrize("geometry", GEOMETRY)
def test_shared_output_split(sem, gll, geometry):
    """Interface elements first, interior elements second into the same y
    (sem_set_map_shared node states) == the single operator, in overwrite
    and in accumulate mode."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import split_interface_elements
    p, nex, ney = 6, 9, 5
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    Ny = ney * p + 1
    nn = nodes.shape[1]
    neighbors = {1: np.arange(nn - Ny, nn)}  # right edge line as the "interface"
    ie, be, st_i, st_b = split_interface_elements(e2n, neighbors)
    assert ie.size == ney and be.size == (nex - 1) * ney
    full = sem.SEMOperator(p, e2n, nodes, geometry=geometry)
    op_i = sem.SEMOperator(p, e2n[ie], nodes, geometry=geometry, node_state=st_i)
    op_b = sem.SEMOperator(p, e2n[be], nodes, geometry=geometry, node_state=st_b)
    u = torch.randn(full.ndof, dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(7))
    ref = full.apply(u)
    y = torch.full_like(u, 3.0)
    op_i.apply(u, out=y)
    op_b.apply(u, out=y)
    assert (y - ref).norm().item() <= 1e-13 * ref.norm().item()
    y0 = torch.linspace(-1, 1, u.numel(), dtype=torch.float64, device="cuda")
    y = y0.clone()
    op_i.apply(u, out=y, accumulate=True)
    op_b.apply(u, out=y, accumulate=True)
    assert (y - y0 - ref).norm().item() <= 1e-13 * ref.norm().item()


# ---------------------------------------------------------------------------
# fp64 matrix-core kernel (k_poisson_mfma, sem_set_kernel SEM_KERNEL_MFMA)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("geometry", GEOMETRY)
@pytest.mark.parametrize("name", ACTION_CASES)
def test_poisson_action_golden_mfma(sem, poisson_action, gll, name, geometry):
    import sem_oracle
    fx = poisson_action
    p = int(fx[name + "_p"])
    if p == 16 and geometry == "nodal":
        pytest.skip("the n = 17 MFMA kernel takes stored factors (nodal: test_mfma_auto_selection_and_limits)")
    op = sem.SEMOperator(p, fx[name + "_e2n"], fx[name + "_nodes"], kernel="mfma",
                         geometry=geometry)
    assert op.plan_info()["kernel"] == "mfma"
    y = op.apply(torch.from_numpy(fx[name + "_u"]).cuda()).cpu().numpy()
    y_ext = None
    if p > 10:
        y_ext = sem_oracle.poisson_apply_extended(fx[name + "_nodes"], fx[name + "_e2n"],
                                                  gll["half_%d" % p], fx[name + "_u"])
    assert_parity(y, fx[name + "_y"], y_ext, TOL_ACTION)


@pytest.mark.parametrize("geometry", GEOMETRY)
@pytest.mark.parametrize("p", list(range(1, 17)))
def test_poisson_all_orders_mfma(sem, gll, p, geometry):
    """Every tile packing: 16 // (p + 1) elements per tile side for p <= 7
    (block-diagonal D), one element per tile above, three elements' lines
    flattened over four tiles at p = 16 (k_poisson_mfma17p); the 7 x 5 mesh
    leaves partly filled tiles / wavefronts at the end of every colour."""
    import sem_oracle
    if p == 16 and geometry == "nodal":
        pytest.skip("the n = 17 MFMA kernel takes stored factors")
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_square(7, 5, p, warp=0.05)
    prob = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p])
    u = np.random.default_rng(p).standard_normal(prob.ndof)
    op = sem.SEMOperator(p, e2n, nodes, kernel="mfma", geometry=geometry)
    y = op.apply(torch.from_numpy(u).cuda()).cpu().numpy()
    y_ext = sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u)
    assert_parity(y, prob.apply(u), y_ext, TOL_ACTION)


def test_mfma_auto_selection_and_limits(sem, poisson_action):
    from spectralelementmethod_amd import meshgen
    # the column kernel on the seam plan measured ahead of the MFMA kernel at
    # every order: AUTO never picks MFMA
    for p, expect in ((8, "column"), (11, "column"), (12, "column"), (13, "column"),
                      (15, "column"), (16, "column")):
        nodes, e2n = meshgen.structured_square(3, 2, p)
        assert sem.SEMOperator(p, e2n, nodes).plan_info()["kernel"] == expect, p
    # AUTO geometry per order: only the orders with a clear measured win are
    # pinned (p = 3, 5, 6, 7 were within 2-3 % in the sweep)
    for p, expect in ((2, "nodal"), (4, "nodal"), (8, "nodal"), (12, "stored")):
        nodes, e2n = meshgen.structured_square(3, 2, p)
        assert sem.SEMOperator(p, e2n, nodes).plan_info()["geometry"] == expect, p
    # axisymmetric Stokes block: NODAL at p <= 6 and p = 16, STORED at 8..12
    for p, expect in ((2, "nodal"), (6, "nodal"), (10, "stored")):
        nodes, e2n = meshgen.annulus(3, 2, p)
        op = sem.SEMOperator(p, e2n, nodes, dofs_per_node=2)
        op.apply(torch.zeros(op.ndof, dtype=torch.float64, device="cuda"), kind="axisym_stokes")
        assert op.plan_info()["geometry_axisym"] == expect, p
    # nodal geometry requested explicitly keeps the column kernel under auto
    nodes, e2n = meshgen.structured_square(3, 2, 12)
    assert sem.SEMOperator(12, e2n, nodes, geometry="nodal").plan_info()["kernel"] == "column"
    # p = 16 (n = 17): the folded multi-element MFMA kernel, stored factors only
    nodes, e2n = meshgen.structured_square(2, 2, 16)
    op = sem.SEMOperator(16, e2n, nodes, kernel="mfma")
    assert op.plan_info()["kernel"] == "mfma" and op.plan_info()["geometry"] == "stored"
    assert op.plan_info()["plan"] == "element"  # colour launches (seams measured slower)
    op = sem.SEMOperator(16, e2n, nodes, kernel="mfma", geometry="nodal")
    with pytest.raises(NotImplementedError):
        op.apply(torch.zeros(op.ndof, dtype=torch.float64, device="cuda"))
    fx = poisson_action
    with pytest.raises(NotImplementedError):
        sem.SEMOperator(4, fx["p4_4x4_e2n"], fx["p4_4x4_nodes"], dofs_per_node=2, kernel="mfma")
    with pytest.raises(ValueError):
        sem.SEMOperator(4, fx["p4_4x4_e2n"], fx["p4_4x4_nodes"], kernel="bogus")


def test_mfma_accumulate_unreferenced_nonconforming(sem, poisson_action, gll):
    import sem_oracle
    fx = poisson_action
    name = "p4_4x4"
    nodes, e2n, u = fx[name + "_nodes"], fx[name + "_e2n"], fx[name + "_u"]
    op = sem.SEMOperator(4, e2n, nodes, kernel="mfma")
    ut = torch.from_numpy(u).cuda()
    y0 = torch.linspace(-1, 1, u.size, dtype=torch.float64, device="cuda")
    y = y0.clone()
    op.apply(ut, out=y, accumulate=True)
    assert rel_l2(y.cpu().numpy(), y0.cpu().numpy() + fx[name + "_y"]) < TOL_ACTION
    y.fill_(123.0)
    op.apply(ut, out=y)
    assert rel_l2(y.cpu().numpy(), fx[name + "_y"]) < TOL_ACTION
    # unreferenced trailing nodes are zeroed in overwrite mode
    extra = np.concatenate([nodes, np.array([[5.0, 6.0], [5.0, 6.0]])], axis=1)
    op = sem.SEMOperator(4, e2n, extra, kernel="mfma")
    y = torch.full((op.ndof,), 7.0, dtype=torch.float64, device="cuda")
    op.apply(torch.from_numpy(np.concatenate([u, [1.0, 2.0]])).cuda(), out=y)
    y = y.cpu().numpy()
    assert y[-2] == 0.0 and y[-1] == 0.0
    assert rel_l2(y[:-2], fx[name + "_y"]) < TOL_ACTION
    # duplicated elements (shared interior nodes): non-conforming map, the
    # colouring then separates elements sharing any node
    e2d = np.concatenate([e2n, e2n[:2]])
    op = sem.SEMOperator(4, e2d, nodes, kernel="mfma")
    assert not op.plan_info()["conforming"]
    y = op.apply(ut).cpu().numpy()
    assert rel_l2(y, sem_oracle.PoissonProblem(nodes, e2d, gll["half_4"]).apply(u)) < TOL_ACTION


@pytest.mark.parametrize("p,geometry", [(10, "stored"), (4, "nodal"), (3, "stored"), (16, "stored")])
def test_mfma_shared_output_split(sem, p, geometry):
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import split_interface_elements
    nex, ney = 7, 4
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    Ny = ney * p + 1
    nn = nodes.shape[1]
    ie, be, st_i, st_b = split_interface_elements(e2n, {1: np.arange(nn - Ny, nn)})
    full = sem.SEMOperator(p, e2n, nodes, kernel="column", geometry="stored")
    op_i = sem.SEMOperator(p, e2n[ie], nodes, node_state=st_i, kernel="mfma", geometry=geometry)
    op_b = sem.SEMOperator(p, e2n[be], nodes, node_state=st_b, kernel="mfma", geometry=geometry)
    u = torch.randn(full.ndof, dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(9))
    ref = full.apply(u)
    y = torch.full_like(u, 3.0)
    op_i.apply(u, out=y)
    op_b.apply(u, out=y)
    assert (y - ref).norm().item() <= 1e-13 * ref.norm().item()


@pytest.mark.parametrize("nex,ney", [(40, 30), (13, 7)])
def test_mfma17_vs_column(sem, nex, ney):
    """p = 16: the MFMA kernel (k_poisson_mfma17p: three elements per
    wavefront, folded 17-point contractions) against the column kernel, in
    overwrite and accumulate mode; symmetric, annihilates constants."""
    from spectralelementmethod_amd import meshgen
    p = 16
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    g = torch.Generator(device="cuda").manual_seed(17)
    col = sem.SEMOperator(p, e2n, nodes, kernel="column", geometry="stored")
    mf = sem.SEMOperator(p, e2n, nodes, kernel="mfma")
    assert mf.plan_info()["kernel"] == "mfma"
    u = torch.randn(col.ndof, dtype=torch.float64, device="cuda", generator=g)
    v = torch.randn(col.ndof, dtype=torch.float64, device="cuda", generator=g)
    ya, yb = col.apply(u), mf.apply(u)
    assert (ya - yb).norm().item() < 1e-12 * ya.norm().item()
    y = v.clone()
    mf.apply(u, out=y, accumulate=True)
    assert (y - v - ya).norm().item() < 1e-12 * ya.norm().item()
    Kv = mf.apply(v)
    a, b = torch.dot(v, yb).item(), torch.dot(u, Kv).item()
    assert abs(a - b) <= 1e-11 * max(abs(a), abs(b))
    K1 = mf.apply(torch.ones_like(u))
    assert K1.abs().max().item() < 1e-9 * yb.abs().max().item()


def test_mfma_vs_column_larger(sem):
    """The two kernel families agree at 2.4M DOF (p = 12, 128 x 96 warped),
    and the MFMA action is symmetric and annihilates constants."""
    from spectralelementmethod_amd import meshgen
    p = 12
    nodes, e2n = meshgen.structured_square(128, 96, p, warp=0.05)
    g = torch.Generator(device="cuda").manual_seed(4)
    col = sem.SEMOperator(p, e2n, nodes, kernel="column", geometry="stored")
    mf = sem.SEMOperator(p, e2n, nodes, kernel="mfma")
    u = torch.randn(col.ndof, dtype=torch.float64, device="cuda", generator=g)
    v = torch.randn(col.ndof, dtype=torch.float64, device="cuda", generator=g)
    ya, yb = col.apply(u), mf.apply(u)
    assert (ya - yb).norm().item() < 1e-13 * ya.norm().item()
    Kv = mf.apply(v)
    a, b = torch.dot(v, yb).item(), torch.dot(u, Kv).item()
    assert abs(a - b) <= 1e-11 * max(abs(a), abs(b))
    K1 = mf.apply(torch.ones_like(u))
    assert K1.abs().max().item() < 1e-10 * yb.abs().max().item()


# ---------------------------------------------------------------------------
# Navier-Stokes squirmer residual (Re > 0) and its Newton Jacobian product
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["p6_4x8", "p4_3x2"])
def test_axisym_ns_golden(sem, axisym_ns, name):
    """Residual vs the reference's compute_local_system with the
    KroneckerArray Ae (squirmer:229-297); Jacobian-vector product vs its
    assembled dense jac_l."""
    fx = axisym_ns
    p = int(fx[name + "_p"])
    op = sem.SEMOperator(p, fx[name + "_e2n"], fx[name + "_nodes"], dofs_per_node=2)
    op.set_reynolds(float(fx[name + "_re"]))
    sol = torch.from_numpy(fx[name + "_soln"]).cuda()
    with pytest.raises(Exception):
        op.apply(sol, kind="axisym_ns_jvp")  # no linearisation recorded yet
    res = op.apply(sol, kind="axisym_ns", linearize=True).cpu().numpy()
    assert rel_l2(res, fx[name + "_res"]) < TOL_AXISYM
    jvp = op.apply(torch.from_numpy(fx[name + "_delta"]).cuda(), kind="axisym_ns_jvp")
    assert rel_l2(jvp.cpu().numpy(), fx[name + "_jvp"]) < TOL_AXISYM


def test_axisym_ns_properties():
    """Re = 0 gives the Stokes block; the residual is quadratic in the state,
    so the central difference (F(s + d) - F(s - d)) / 2 is exactly J(s) d
    (rounding only), on a 96 x 64 curved annulus at p = 6."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    p = 6
    nodes, e2n = meshgen.annulus(96, 64, p)
    op = SEMOperator(p, e2n, nodes, dofs_per_node=2)
    g = torch.Generator(device="cuda").manual_seed(5)
    s = torch.randn(op.ndof, dtype=torch.float64, device="cuda", generator=g)
    d = torch.randn(op.ndof, dtype=torch.float64, device="cuda", generator=g)
    op.set_reynolds(0.0)
    stokes = op.apply(s, kind="axisym_stokes")
    assert (op.apply(s, kind="axisym_ns") - stokes).norm().item() <= 1e-13 * stokes.norm().item()
    op.set_reynolds(25.0)
    op.apply(s, kind="axisym_ns", linearize=True)
    jd = op.apply(d, kind="axisym_ns_jvp")
    cd = 0.5 * (op.apply(s + d, kind="axisym_ns") - op.apply(s - d, kind="axisym_ns"))
    assert (jd - cd).norm().item() <= 1e-12 * jd.norm().item()


def test_apply_rejects_aliased_output(sem, poisson_action):
    """u and y must not alias: the kernels read u while other workgroups
    write y (include/sem_hip.h sem_apply); both the facade and the C ABI
    refuse it."""
    from spectralelementmethod_amd import _lib
    fx = poisson_action
    op = sem.SEMOperator(4, fx["p4_4x4_e2n"], fx["p4_4x4_nodes"])
    u = torch.from_numpy(fx["p4_4x4_u"]).cuda()
    with pytest.raises(ValueError):
        op.apply(u, out=u)
    op.compute_geometry()
    rc = _lib.load().sem_apply(op._ctx, 0, _lib.tptr(u), _lib.tptr(u), 0, _lib.stream_ptr())
    assert rc == _lib.SEM_E_INVALID and "overlap" in _lib.last_error()


def test_basis_must_be_symmetric(sem):
    """The kernels apply D in even-odd form and assume a node set symmetric
    about 0 (GLL): sem_set_basis refuses a D that is not centro-antisymmetric
    or weights that are not symmetric (ValueError) instead of computing a
    wrong action silently."""
    from types import SimpleNamespace
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.basis_functions import gll_basis_2d
    p = 4
    good = gll_basis_2d(p)
    nodes, e2n = meshgen.structured_square(2, 2, p)
    D = good.get_D1_matrices()[0].copy()
    w = np.array(good.quad_rule.weights[0], dtype=np.float64)

    def fake(D, w):
        sub = SimpleNamespace(_interp_eq_inv=good._subbases[0]._interp_eq_inv)
        return SimpleNamespace(get_D1_matrices=lambda: (D, D), _subbases=[sub, sub],
                               quad_rule=SimpleNamespace(weights=[w, w]))

    sem.SEMOperator(p, e2n, nodes, basis=fake(D, w))  # the GLL basis itself passes
    Db = D.copy()
    Db[0, 1] += 1e-6
    with pytest.raises(ValueError, match="symmetric"):
        sem.SEMOperator(p, e2n, nodes, basis=fake(Db, w))
    wb = w.copy()
    wb[0] *= 1.0 + 1e-9
    with pytest.raises(ValueError, match="symmetric"):
        sem.SEMOperator(p, e2n, nodes, basis=fake(D, wb))
