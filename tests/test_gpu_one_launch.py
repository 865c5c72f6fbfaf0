"""The one-launch scatter plan of the chain kernels (SEM_DF=1; DESIGN.md §5,
DFPlan in csrc/sem_kernels.h; measured slower than one launch per colour,
so not the default): every chain in one launch, workgroups taking
chains from a ticket counter, a chain starting once the chains that wrote its
shared nodes earlier in ticket order have published their flags.

Checked against the NumPy oracle (north-star tolerance 1e-10 relative L2, the
kernels meet 1e-12) and against the one-launch-per-colour plan (SEM_DF=0),
whose per-node summation order differs: agreement to 1e-13.  The lag sweep
includes lag 1, where the ticket order is close to the element order and
almost every chain really waits on a neighbour taken just before it: the
hand-off (sc1 stores, drained waves, flag; sc1 operand loads) is exercised
under uneven load, every node compared."""
import numpy as np
import pytest

from conftest import rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-12


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _mesh(p, nex, ney):
    from spectralelementmethod_amd import meshgen
    return meshgen.structured_square(nex, ney, p, warp=0.05)


def _oracle(gll, nodes, e2n, p, u):
    import sem_oracle
    return (sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True).apply(u),
            sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u))


def _check(y, ref, ext):
    e = rel_l2(y, ref)
    if e >= TOL:  # high order: judge against extended precision (test_gpu_parity.assert_parity)
        assert rel_l2(y, ext) <= max(1.5 * rel_l2(ref, ext), TOL), e


@pytest.mark.parametrize("p,nex,ney", [(2, 40, 33), (4, 30, 29), (6, 21, 17), (8, 64, 48),
                                       (12, 13, 11), (16, 9, 8)])
def test_one_launch_vs_colour_launches(gpu, gll, monkeypatch, p, nex, ney):
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = _mesh(p, nex, ney)
    u = np.random.default_rng(p).standard_normal(nodes.shape[1])
    ut = torch.from_numpy(u).to(gpu)
    monkeypatch.setenv("SEM_PLAN", "0")
    monkeypatch.setenv("SEM_SEAM", "0")
    monkeypatch.setenv("SEM_DF", "1")
    monkeypatch.setenv("SEM_DF_LAG", "4")  # small mesh: a lag below the chain count
    op1 = SEMOperator(p, e2n, nodes, device=gpu, kernel="column")
    info = op1.plan_info()
    assert info["plan"] == "chains-one-launch", info
    assert info["colours"] == 1 and info["dependencies"] > 0
    y1 = op1.apply(ut).cpu().numpy()
    monkeypatch.setenv("SEM_DF", "0")
    op4 = SEMOperator(p, e2n, nodes, device=gpu, kernel="column")
    assert op4.plan_info()["plan"] == "chains"
    y4 = op4.apply(ut).cpu().numpy()
    assert rel_l2(y1, y4) < 1e-13
    ref, ext = _oracle(gll, nodes, e2n, p, u)
    _check(y1, ref, ext)
    assert op1.plan_info()["wait_timeouts"] == 0


@pytest.mark.parametrize("lag,ticket", [(1, "1"), (1, "0"), (64, "1"), (100000, "1")])
@pytest.mark.parametrize("geometry", ["nodal", "stored"])
def test_one_launch_lag_and_dispatch(gpu, gll, monkeypatch, lag, ticket, geometry):
    """128 x 96 p = 8: every lag gives the oracle's action, run after run
    bitwise identical (each node's writers run in ticket order, whatever the
    timing), and no wait hits its spin limit.  SEM_DF_TICKET=0 takes the
    chain from blockIdx instead of the ticket counter (a timing experiment;
    it relies on in-order dispatch)."""
    from spectralelementmethod_amd.operators import SEMOperator
    p = 8
    nodes, e2n = _mesh(p, 128, 96)
    u = np.random.default_rng(11).standard_normal(nodes.shape[1])
    monkeypatch.setenv("SEM_SEAM", "0")
    monkeypatch.setenv("SEM_DF", "1")
    monkeypatch.setenv("SEM_DF_LAG", str(lag))
    monkeypatch.setenv("SEM_DF_TICKET", ticket)
    op = SEMOperator(p, e2n, nodes, device=gpu, geometry=geometry)
    assert op.plan_info()["plan"] == "chains-one-launch"
    assert op.plan_info()["lag"] == lag
    ut = torch.from_numpy(u).to(gpu)
    ys = [op.apply(ut) for _ in range(3)]
    torch.cuda.synchronize()
    for y in ys[1:]:
        assert torch.equal(y, ys[0])
    ref, ext = _oracle(gll, nodes, e2n, p, u)
    _check(ys[0].cpu().numpy(), ref, ext)
    assert op.plan_info()["wait_timeouts"] == 0


def test_one_launch_accumulate_and_graph_replay(gpu, gll, monkeypatch):
    """accumulate mode (first writers read y too), and the action captured in
    a HIP graph: the epoch lives on the device, so every replay waits for the
    flags of ITS OWN launch."""
    from spectralelementmethod_amd.operators import SEMOperator
    p = 6
    nodes, e2n = _mesh(p, 48, 40)
    monkeypatch.setenv("SEM_SEAM", "0")
    monkeypatch.setenv("SEM_DF", "1")
    op = SEMOperator(p, e2n, nodes, device=gpu)
    assert op.plan_info()["plan"] == "chains-one-launch"
    g = torch.Generator(device=gpu).manual_seed(4)
    u = torch.randn(op.ndof, dtype=torch.float64, device=gpu, generator=g)
    y0 = torch.randn(op.ndof, dtype=torch.float64, device=gpu, generator=g)
    Ku = op.apply(u)
    y = y0.clone()
    op.apply(u, out=y, accumulate=True)
    assert (y - (y0 + Ku)).norm().item() <= 1e-14 * y.norm().item()
    # graph capture of the action on a side stream, replayed with new inputs
    s = torch.cuda.Stream(device=gpu)
    us = torch.zeros_like(u)
    ys = torch.zeros_like(u)
    s.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(s):
        op.apply(us, out=ys, stream=s)  # warm-up outside the capture
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            op.apply(us, out=ys, stream=s)
    torch.cuda.current_stream(gpu).wait_stream(s)
    ref, ext = _oracle(gll, nodes, e2n, p, u.cpu().numpy())
    for k in range(3):
        us.copy_(u * (k + 1))
        graph.replay()
        torch.cuda.synchronize()
        _check(ys.cpu().numpy() / (k + 1), ref, ext)
    assert op.plan_info()["wait_timeouts"] == 0


@pytest.mark.parametrize("geometry", ["nodal", "stored"])
def test_one_launch_axisymmetric(gpu, gll, monkeypatch, geometry):
    """The axisymmetric Stokes block (two DOFs per node, 16-B read-modify-
    writes) and the Navier-Stokes residual / Jacobian-vector product in one
    launch: equal to the per-colour launches to 1e-13, the Stokes block to the
    oracle at 1e-12."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    p = 6
    nodes, e2n = meshgen.annulus(40, 36, p)
    rng = np.random.default_rng(8)
    sol = torch.from_numpy(rng.standard_normal(2 * nodes.shape[1])).to(gpu)
    dirn = torch.from_numpy(rng.standard_normal(2 * nodes.shape[1])).to(gpu)
    monkeypatch.setenv("SEM_DF_LAG", "8")
    monkeypatch.setenv("SEM_SEAM", "0")
    out = {}
    for df in ("1", "0"):
        monkeypatch.setenv("SEM_DF", df)
        op = SEMOperator(p, e2n, nodes, dofs_per_node=2, device=gpu, geometry=geometry)
        assert op.plan_info()["plan"] == ("chains-one-launch" if df == "1" else "chains")
        op.set_reynolds(5.0)
        ys = op.apply(sol, kind="axisym_stokes")
        yn = op.apply(sol, kind="axisym_ns", linearize=True)
        yj = op.apply(dirn, kind="axisym_ns_jvp")
        out[df] = [t.cpu().numpy() for t in (ys, yn, yj)]
        assert op.plan_info()["wait_timeouts"] == 0
    for a, b in zip(out["1"], out["0"]):
        assert rel_l2(a, b) < 1e-13
    nodes_1d, bary, quad = sem_oracle.gll_unfold(gll["half_%d" % p])
    D = sem_oracle.diff_matrix(nodes_1d, bary)
    _, lu = sem_oracle.interp_eq_lu(nodes_1d, bary)
    e2n64 = e2n.astype(np.int64)
    xp, _, invJ, _, detJxW = sem_oracle.geometry(nodes, e2n64, D, quad, lu, batched=True)
    F = sem_oracle.axisym_factors(xp, invJ, detJxW)
    ref = sem_oracle.axisym_apply(F, D, e2n64, sol.cpu().numpy(), nodes.shape[1])
    assert rel_l2(out["1"][0], ref) < TOL
