"""The block layout of the chain plans (groups_blocks in
csrc/sem_device.hip, the row carry in chain_emit, csrc/sem_kernels.h).

On a structured numbering a chain is R stacked element lines x 4 groups, and
the node row between two rounds is handed from round to round in registers
(code SKIP | CARRY) instead of being stored by one chain and read-modified-
written by another.  The carried node receives the same two partial sums,
added in the other order (exact: addition commutes), so the block plans agree
with the consecutive-group plan to rounding of the multi-way corner sums
(1e-14), and both meet the oracle (1e-12; the north-star bar is 1e-10).
Meshes include partial segments (line length not a multiple of 28 elements)
and partial blocks (line count not a multiple of R)."""
import numpy as np
import pytest

from conftest import rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-12
SAME = 1e-14


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _op(monkeypatch, rounds, seam, *args, **kw):
    from spectralelementmethod_amd.operators import SEMOperator
    monkeypatch.setenv("SEM_BLOCK_ROUNDS", str(rounds))
    monkeypatch.setenv("SEM_SEAM", seam)
    monkeypatch.setenv("SEM_PLAN", "0")
    return SEMOperator(*args, **kw)


@pytest.mark.parametrize("p,nex,ney,geometry", [(2, 9, 61, "auto"), (4, 11, 40, "nodal"),
                                                (6, 7, 30, "stored"), (8, 13, 33, "nodal"),
                                                (8, 10, 57, "stored"), (12, 6, 9, "auto"),
                                                (16, 5, 7, "auto")])
@pytest.mark.parametrize("seam", ["0", "1"])
def test_blocks_match_consecutive_groups(gpu, gll, monkeypatch, p, nex, ney, geometry, seam):
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    u = torch.from_numpy(np.random.default_rng(p).standard_normal(nodes.shape[1])).to(gpu)
    y0 = torch.from_numpy(np.random.default_rng(3).standard_normal(nodes.shape[1])).to(gpu)
    base = _op(monkeypatch, 0, "0", p, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
    assert not base.plan_info()["blocks"]
    yb = base.apply(u).cpu().numpy()
    ab = y0.clone()
    base.apply(u, out=ab, accumulate=True)
    ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True).apply(
        u.cpu().numpy())
    for R in (2, 3, 4):
        op = _op(monkeypatch, R, seam, p, e2n, nodes, device=gpu, kernel="column",
                 geometry=geometry)
        info = op.plan_info()
        assert info["blocks"] and info["rounds"] == R and info["row_carries"] > 0, info
        assert info["atomic_groups"] == 0 and info["zero_list"] == 0, info
        assert info["plan"] == ("chains-seams" if seam == "1" else "chains"), info
        y = op.apply(u).cpu().numpy()
        assert rel_l2(y, yb) <= SAME, (R, rel_l2(y, yb))
        a = y0.clone()
        op.apply(u, out=a, accumulate=True)
        assert rel_l2(a.cpu().numpy(), ab.cpu().numpy()) <= SAME
        if p <= 10:
            assert rel_l2(y, ref) < TOL


def test_blocks_rcm_numbering_falls_back(gpu, gll, monkeypatch):
    """A numbering without stacked lines (RCM-renumbered nodes, elements sorted
    by their smallest node) keeps consecutive groups, exactly."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    nodes, e2n = meshgen.structured_square(12, 10, 4, warp=0.05)
    nodes, e2n = meshgen.rcm_renumber(nodes, meshgen.shuffle_elements(e2n, seed=2))
    u = np.random.default_rng(0).standard_normal(nodes.shape[1])
    op = _op(monkeypatch, 4, "0", 4, e2n, nodes, device=gpu)
    y = op.apply(torch.from_numpy(u).to(gpu)).cpu().numpy()
    assert rel_l2(y, sem_oracle.PoissonProblem(nodes, e2n, gll["half_4"]).apply(u)) < TOL


@pytest.mark.parametrize("geometry", ["nodal", "stored"])
def test_blocks_axisymmetric(gpu, monkeypatch, geometry):
    """Two DOFs per node: the Stokes block, the Navier-Stokes residual and its
    Jacobian-vector product on the block layout (row carry of both fields)
    equal the consecutive-group plan."""
    from spectralelementmethod_amd import meshgen
    p = 6
    nodes, e2n = meshgen.annulus(13, 37, p)
    rng = np.random.default_rng(8)
    sol = torch.from_numpy(rng.standard_normal(2 * nodes.shape[1])).to(gpu)
    dirn = torch.from_numpy(rng.standard_normal(2 * nodes.shape[1])).to(gpu)
    out = {}
    for R, seam in ((0, "0"), (4, "0"), (4, "1"), (3, "0")):
        op = _op(monkeypatch, R, seam, p, e2n, nodes, dofs_per_node=2, device=gpu,
                 geometry=geometry)
        assert op.plan_info()["blocks"] == (R > 0)
        op.set_reynolds(5.0)
        ys = op.apply(sol, kind="axisym_stokes")
        yn = op.apply(sol, kind="axisym_ns", linearize=True)
        yj = op.apply(dirn, kind="axisym_ns_jvp")
        out[(R, seam)] = [t.cpu().numpy() for t in (ys, yn, yj)]
    for key, vals in out.items():
        for a, b in zip(vals, out[(0, "0")]):
            assert rel_l2(a, b) <= SAME, key


@pytest.mark.parametrize("seam", ["0", "1"])
def test_blocks_multirank_one_gpu(gpu, monkeypatch, seam):
    """The decomposition's interior and interface operators on the block
    layout (shared-output node states): the 2- and 3-rank actions on one
    device equal the single-operator action."""
    import importlib
    monkeypatch.setenv("SEM_BLOCK_ROUNDS", "4")
    monkeypatch.setenv("SEM_SEAM", seam)
    mr = importlib.import_module("test_gpu_multirank")
    mr.test_overlapped_operator_ranks_on_one_gpu(gpu, 2, "strip", 8, 24, 20)
    mr.test_overlapped_operator_ranks_on_one_gpu(gpu, 3, "strip", 8, 24, 20)


def test_seams_with_rounds_of_consecutive_groups(gpu, gll, monkeypatch):
    """two rounds of consecutive groups on the seam plan.  A
    seam node the same chain touches again in a later round would be stored
    twice into its slot; the planner falls back to the colour launches
    instead, and the action is exact."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    p = 8
    nodes, e2n = meshgen.structured_square(32, 32, p, warp=0.05)
    u = np.random.default_rng(4).standard_normal(nodes.shape[1])
    monkeypatch.setenv("SEM_CHAIN_ROUNDS", "2")
    op = _op(monkeypatch, 0, "1", p, e2n, nodes, device=gpu, kernel="column")
    y = op.apply(torch.from_numpy(u).to(gpu)).cpu().numpy()
    ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True).apply(u)
    assert rel_l2(y, ref) < TOL
