"""The seam plan of the Poisson column kernel (SEM_SEAM=1; DESIGN.md §5,
SeamPlan / k_seam_sum in csrc/sem_kernels.h): every chain in ONE launch in
element order, nodes written by several chains stored per writer colour and
summed by a second launch in colour order.

The seam sums add the same partial sums in the same order as the colour
launches' read-modify-writes, so the two plans agree to the last bit on the
structured meshes (checked at 1e-15 to stay robust to a compiler contracting
a multiply-add differently in the two kernel instantiations), and both meet
the oracle (1e-12; the north-star bar is 1e-10)."""
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


def _oracle(gll, nodes, e2n, p, u):
    import sem_oracle
    return (sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True).apply(u),
            sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u))


# ney = whole chains per element column (chains that wrap into the next
# column share nodes irregularly: atomic chains, and no seam plan)
@pytest.mark.parametrize("p,nex,ney,geometry", [(2, 7, 168, "auto"), (4, 9, 96, "auto"),
                                                (6, 8, 72, "stored"), (8, 17, 112, "nodal"),
                                                (8, 17, 112, "stored"), (12, 9, 32, "auto"),
                                                (16, 7, 12, "auto")])
def test_seams_match_colour_launches(gpu, gll, monkeypatch, p, nex, ney, geometry):
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    u = np.random.default_rng(p).standard_normal(nodes.shape[1])
    ut = torch.from_numpy(u).to(gpu)
    monkeypatch.setenv("SEM_PLAN", "0")
    monkeypatch.setenv("SEM_SEAM", "1")
    ops = SEMOperator(p, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
    info = ops.plan_info()
    assert info["plan"] == "chains-seams", info
    assert info["seam_nodes"] > 0 and info["colours"] == 1
    ys = ops.apply(ut)
    monkeypatch.setenv("SEM_SEAM", "0")
    opc = SEMOperator(p, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
    assert opc.plan_info()["plan"] == "chains"
    yc = opc.apply(ut)
    assert rel_l2(ys.cpu().numpy(), yc.cpu().numpy()) <= 1e-15
    # accumulate: y0 + K u in both plans
    y0 = torch.from_numpy(np.random.default_rng(3).standard_normal(nodes.shape[1])).to(gpu)
    a_s, a_c = y0.clone(), y0.clone()
    ops.apply(ut, out=a_s, accumulate=True)
    opc.apply(ut, out=a_c, accumulate=True)
    assert rel_l2(a_s.cpu().numpy(), a_c.cpu().numpy()) <= 1e-15
    ref, ext = _oracle(gll, nodes, e2n, p, u)
    y = ys.cpu().numpy()
    if rel_l2(y, ref) >= TOL:  # p > 10: judge against extended precision
        assert rel_l2(y, ext) <= max(1.5 * rel_l2(ref, ext), TOL)


def test_seams_fall_back_on_irregular_meshes(gpu, gll, monkeypatch):
    """Split-triangle quads: in-round sharing the chains cannot express; the
    planner drops the seam plan (element-coloured chains or the atomic
    fallback instead) and the action stays exact."""
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    monkeypatch.setenv("SEM_SEAM", "1")
    nodes, e2n = meshgen.quads_from_triangles(14, 11, 4, seed=3)
    u = np.random.default_rng(1).standard_normal(nodes.shape[1])
    op = SEMOperator(4, e2n, nodes, device=gpu)
    assert op.plan_info()["plan"] != "chains-seams"
    y = op.apply(torch.from_numpy(u).to(gpu)).cpu().numpy()
    assert rel_l2(y, sem_oracle.PoissonProblem(nodes, e2n, gll["half_4"]).apply(u)) < TOL


def test_seams_multirank_one_gpu(gpu, monkeypatch):
    """The decomposition's interior and interface operators on the seam plan
    (shared-output node states: interface nodes PRIOR for the interior
    operator): the 2-rank action on one device equals the single-operator
    action."""
    import importlib
    monkeypatch.setenv("SEM_SEAM", "1")
    mr = importlib.import_module("test_gpu_multirank")
    mr.test_overlapped_operator_ranks_on_one_gpu(gpu, 2, "strip", 8, 24, 20)


@pytest.mark.parametrize("geometry", ["nodal", "stored"])
def test_seams_axisymmetric(gpu, monkeypatch, geometry):
    """Two DOFs per node (16-B slots, k_seam_sum2): the Stokes block and the
    Navier-Stokes residual / Jacobian-vector product on the seam plan equal
    the colour launches (same partial sums, same order)."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    p = 6
    nodes, e2n = meshgen.annulus(16, 72, p)
    rng = np.random.default_rng(8)
    sol = torch.from_numpy(rng.standard_normal(2 * nodes.shape[1])).to(gpu)
    dirn = torch.from_numpy(rng.standard_normal(2 * nodes.shape[1])).to(gpu)
    monkeypatch.setenv("SEM_PLAN", "0")
    out = {}
    for seam in ("1", "0"):
        monkeypatch.setenv("SEM_SEAM", seam)
        op = SEMOperator(p, e2n, nodes, dofs_per_node=2, device=gpu, geometry=geometry)
        assert op.plan_info()["plan"] == ("chains-seams" if seam == "1" else "chains")
        op.set_reynolds(5.0)
        ys = op.apply(sol, kind="axisym_stokes")
        yn = op.apply(sol, kind="axisym_ns", linearize=True)
        yj = op.apply(dirn, kind="axisym_ns_jvp")
        out[seam] = [t.cpu().numpy() for t in (ys, yn, yj)]
    for a, b in zip(out["1"], out["0"]):
        assert rel_l2(a, b) <= 1e-15


@pytest.mark.parametrize("nex,ney", [(7, 12), (20, 9)])
def test_mfma17_seams_match_colour_launches(gpu, gll, monkeypatch, nex, ney):
    """p = 16 MFMA kernel (k_poisson_mfma17p): the element seam plan (one
    launch in breadth-first element order + seam sums; SEM_SEAM=1) against
    its colour launches, overwrite and accumulate, and against the oracle."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    p = 16
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    u = np.random.default_rng(p).standard_normal(nodes.shape[1])
    ut = torch.from_numpy(u).to(gpu)
    monkeypatch.setenv("SEM_SEAM", "1")
    ops = SEMOperator(p, e2n, nodes, device=gpu, kernel="mfma")
    info = ops.plan_info()
    assert info["plan"] == "element-seams" and info["seam_nodes"] > 0, info
    ys = ops.apply(ut)
    monkeypatch.setenv("SEM_SEAM", "0")
    opc = SEMOperator(p, e2n, nodes, device=gpu, kernel="mfma")
    assert opc.plan_info()["plan"] == "element"
    yc = opc.apply(ut)
    assert rel_l2(ys.cpu().numpy(), yc.cpu().numpy()) <= 1e-15
    y0 = torch.from_numpy(np.random.default_rng(3).standard_normal(nodes.shape[1])).to(gpu)
    a_s, a_c = y0.clone(), y0.clone()
    ops.apply(ut, out=a_s, accumulate=True)
    opc.apply(ut, out=a_c, accumulate=True)
    assert rel_l2(a_s.cpu().numpy(), a_c.cpu().numpy()) <= 1e-15
    ref, ext = _oracle(gll, nodes, e2n, p, u)
    y = ys.cpu().numpy()
    assert rel_l2(y, ext) <= max(1.5 * rel_l2(ref, ext), TOL)


@pytest.mark.parametrize("geometry", ["nodal", "stored"])
def test_chain_swizzle_is_bitwise_neutral(gpu, monkeypatch, geometry):
    """The planner's XCD-contiguous chain order (chain_swizzle in
    csrc/sem_device.hip, seam launches of <= 2,400 chains) only permutes the
    chain blocks of the packed arrays: the action equals the unpermuted
    plan's bit for bit, with nodal and with stored (packed by element
    position) factors."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(20, 112, 8, warp=0.05)  # whole chains per column
    u = torch.from_numpy(np.random.default_rng(4).standard_normal(nodes.shape[1])).to(gpu)
    monkeypatch.setenv("SEM_SEAM", "1")
    monkeypatch.setenv("SEM_CHAIN_SWIZZLE_MAX", "0")
    ref = SEMOperator(8, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
    monkeypatch.setenv("SEM_CHAIN_SWIZZLE_MAX", "100000")
    swz = SEMOperator(8, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
    assert swz.plan_info()["plan"] == "chains-seams"
    assert torch.equal(ref.apply(u), swz.apply(u))


@pytest.mark.parametrize("rank", [0, 2])
def test_dd_fused_seam_finish_is_bitwise(gpu, monkeypatch, rank):
    """sem_dd's finish fused with the interior's seam sum (one launch) equals
    the interior's own seam sum followed by k_dd_finish bit for bit, on one
    rank of a 4-strip split with the loopback transport (both peers'
    exchanges exercised; the values are not the global action, the same in
    both forms)."""
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    part = StripPartition(24, 112, 8, 4, rank)  # whole chains per element column
    nodes, e2n = part.local_mesh(0.05)
    u = torch.from_numpy(np.random.default_rng(5).standard_normal(nodes.shape[1])).to(gpu)
    monkeypatch.setenv("SEM_SEAM", "1")
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("SEM_DD_FUSE_SEAM", fuse)
        op = OverlappedOperator(8, nodes, e2n, part.neighbors, 1, gpu, owned=part.owned,
                                transport="loopback", world=1, rank=0, decompose=True)
        y = torch.full_like(u, 7.0)
        op.step(u, y)
        op.step(u, y)
        torch.cuda.synchronize()
        out[fuse] = (y.clone(), op.dd_info())
        op.close()
    assert out["1"][1]["seam_sum_in_finish"] and not out["0"][1]["seam_sum_in_finish"]
    assert torch.equal(out["1"][0], out["0"][0])


def test_dd_rccl_self_transport_equals_loopback(gpu):
    """The timing transport over RCCL (sem_dd_set_rccl_self: send/recv per
    peer to this rank itself on a one-rank communicator, on the side stream)
    moves the same bytes as the loopback copy: bitwise the same step."""
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    part = StripPartition(24, 112, 8, 4, 1)
    nodes, e2n = part.local_mesh(0.05)
    u = torch.from_numpy(np.random.default_rng(6).standard_normal(nodes.shape[1])).to(gpu)
    out = {}
    for tr in ("loopback", "rccl_self"):
        op = OverlappedOperator(8, nodes, e2n, part.neighbors, 1, gpu, owned=part.owned,
                                transport=tr, world=1, rank=0, decompose=True)
        assert op.transport == tr and op.dd_info()["transport"] == tr
        y = torch.full_like(u, 7.0)
        for _ in range(3):
            op.step(u, y)
        torch.cuda.synchronize()
        out[tr] = y.clone()
        op.close()
    assert torch.equal(out["loopback"], out["rccl_self"])


@pytest.mark.parametrize("rank", [0, 2])
@pytest.mark.parametrize("transport", ["loopback", "rccl_self"])
def test_dd_fused_seam_pack_is_bitwise(gpu, monkeypatch, rank, transport):
    """The interface context's seam sum fused with the pack of the send
    buffer (one launch on the side stream) equals its own seam-sum launch
    followed by the gather, bit for bit, on one rank of a 4-strip split."""
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    part = StripPartition(24, 112, 8, 4, rank)
    nodes, e2n = part.local_mesh(0.05)
    u = torch.from_numpy(np.random.default_rng(7).standard_normal(nodes.shape[1])).to(gpu)
    monkeypatch.setenv("SEM_SEAM", "1")
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("SEM_DD_FUSE_PACK", fuse)
        op = OverlappedOperator(8, nodes, e2n, part.neighbors, 1, gpu, owned=part.owned,
                                transport=transport, world=1, rank=0, decompose=True)
        y = torch.full_like(u, 7.0)
        op.step(u, y)
        op.step(u, y)
        torch.cuda.synchronize()
        out[fuse] = (y.clone(), op.dd_info())
        op.close()
    assert out["1"][1]["seam_sum_in_pack"] and not out["0"][1]["seam_sum_in_pack"]
    assert torch.equal(out["1"][0], out["0"][0])


@pytest.mark.parametrize("rank", [0, 2])
def test_dd_split_finish_is_bitwise(gpu, monkeypatch, rank):
    """The fused finish split around the join (the interior's seam nodes off
    the interface and the zero list before the side stream is waited for, the
    rest after it) equals the one-launch finish bit for bit."""
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    part = StripPartition(24, 112, 8, 4, rank)
    nodes, e2n = part.local_mesh(0.05)
    u = torch.from_numpy(np.random.default_rng(8).standard_normal(nodes.shape[1])).to(gpu)
    monkeypatch.setenv("SEM_SEAM", "1")
    out = {}
    for split in ("1", "0"):
        monkeypatch.setenv("SEM_DD_SPLIT_FINISH", split)
        op = OverlappedOperator(8, nodes, e2n, part.neighbors, 1, gpu, owned=part.owned,
                                transport="rccl_self", world=1, rank=0, decompose=True)
        y = torch.full_like(u, 7.0)
        op.step(u, y)
        op.step(u, y)
        torch.cuda.synchronize()
        out[split] = (y.clone(), op.dd_info())
        op.close()
    assert out["1"][1]["split_finish"] and not out["0"][1]["split_finish"]
    assert out["1"][1]["seam_sum_in_finish"]
    assert torch.equal(out["1"][0], out["0"][0])


@pytest.mark.parametrize("transport", ["loopback", "rccl_self"])
def test_dd_event_fence_scope(gpu, monkeypatch, transport):
    """The stream-join events carry the system-scope fence unless the
    transport keeps every writer on this device (loopback, RCCL to self:
    device scope by default); SEM_DD_EVENT_FENCE forces either scope, and the
    step is bitwise the same under both."""
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    part = StripPartition(24, 112, 8, 4, 2)
    nodes, e2n = part.local_mesh(0.05)
    u = torch.from_numpy(np.random.default_rng(9).standard_normal(nodes.shape[1])).to(gpu)
    out = {}
    for scope in ("auto", "system", "device"):
        if scope == "auto":
            monkeypatch.delenv("SEM_DD_EVENT_FENCE", raising=False)
        else:
            monkeypatch.setenv("SEM_DD_EVENT_FENCE", scope)
        op = OverlappedOperator(8, nodes, e2n, part.neighbors, 1, gpu, owned=part.owned,
                                transport=transport, world=1, rank=0, decompose=True)
        y = torch.full_like(u, 7.0)
        for _ in range(3):
            op.step(u, y)
        torch.cuda.synchronize()
        out[scope] = (y.clone(), op.dd_info()["event_fence"])
        op.close()
    assert out["auto"][1] == "device" and out["system"][1] == "system"
    assert out["device"][1] == "device"
    assert torch.equal(out["auto"][0], out["system"][0])
    assert torch.equal(out["auto"][0], out["device"][0])


@pytest.mark.parametrize("rank", [0, 1, 3])
def test_dd_hex_slab_rank_equals_single_gpu_interior(gpu, rank):
    """One rank of a hexahedral slab split (row N3) through sem_dd with the
    RCCL-to-self timing transport (bench.py --dim 3 --time-rank): away from
    the shared faces (where the loopback adds the rank's own values, not the
    neighbour's) every node equals the single-GPU action of the whole cube."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.distributed import OverlappedOperator, SlabPartition
    from spectralelementmethod_amd.operators import SEMOperator
    p, nex, ney, nez, world = 6, 12, 3, 3, 4
    part = SlabPartition(nex, ney, nez, p, world, rank)
    nodes, e2n = part.local_mesh(0.05)
    gnodes, ge2n = meshgen.structured_cube(nex, ney, nez, p, warp=0.05)
    u_glob = torch.from_numpy(np.random.default_rng(12).standard_normal(gnodes.shape[1])).to(gpu)
    y_glob = SEMOperator(p, ge2n, gnodes, device=gpu).apply(u_glob)
    l2g = torch.from_numpy(part.local_to_global()).to(gpu)
    op = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, gpu, owned=part.owned,
                            transport="rccl_self", world=1, rank=0, decompose=True)
    y = torch.full((op.ndof,), 7.0, dtype=torch.float64, device=gpu)
    op.step(u_glob[l2g].contiguous(), y)
    torch.cuda.synchronize()
    inner = torch.ones(op.ndof, dtype=torch.bool, device=gpu)
    for nb in part.neighbors.values():
        inner[torch.from_numpy(nb).to(gpu)] = False
    ref = y_glob[l2g]
    assert ((y - ref)[inner].norm() / ref[inner].norm()).item() < 1e-12
    assert op.dd_info()["event_fence"] == "device" and op.plan_info()["ndim"] == 3
    op.close()
