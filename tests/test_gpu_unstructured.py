"""GPU parity on meshes the chain planner was not shaped for (the oracle is
mesh-agnostic): irregular-valence quads from split triangles, randomly
ordered elements, randomly numbered nodes (group rows spanning far more than
the 16-bit map's 4096-id window), and the RCM renumbering that restores
locality.  Tolerance 1e-12 relative L2 (fp64; scatter order may differ where
the planner falls back to atomics)."""
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


def make_mesh(kind, p):
    from spectralelementmethod_amd import meshgen
    if kind == "split_tri":
        return meshgen.quads_from_triangles(14, 11, p, seed=3)
    if kind == "split_tri_shuffled":
        nodes, e2n = meshgen.quads_from_triangles(14, 11, p, seed=3)
        return meshgen.shuffle_nodes(nodes, meshgen.shuffle_elements(e2n, 1), 2)
    if kind == "split_tri_rcm":
        nodes, e2n = meshgen.quads_from_triangles(14, 11, p, seed=3)
        return meshgen.rcm_renumber(*meshgen.shuffle_nodes(nodes, meshgen.shuffle_elements(e2n, 1),
                                                           2))
    nodes, e2n = meshgen.structured_square(40, 30, p, warp=0.05)
    if kind == "shuffled_elems":
        return nodes, meshgen.shuffle_elements(e2n, 5)
    if kind == "shuffled_nodes":
        return meshgen.shuffle_nodes(nodes, e2n, 6)
    raise ValueError(kind)


KINDS = ["split_tri", "split_tri_shuffled", "split_tri_rcm", "shuffled_elems", "shuffled_nodes"]


@pytest.mark.parametrize("geometry", ["nodal", "stored"])
@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("kind", KINDS)
def test_unstructured_action_vs_oracle(gpu, gll, kind, p, geometry):
    import sem_oracle
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = make_mesh(kind, p)
    u = np.random.default_rng(p).standard_normal(nodes.shape[1])
    ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True).apply(u)
    op = SEMOperator(p, e2n, nodes, device=gpu, geometry=geometry, kernel="column")
    plan = op.plan_info()
    assert plan["conforming"] and plan["colours"] <= 9
    y = op.apply(torch.from_numpy(u).to(gpu)).cpu().numpy()
    assert rel_l2(y, ref) < TOL, (kind, p, geometry, plan)
    if kind == "shuffled_nodes" and p == 8:
        assert plan["map_entry_bytes"] == 4  # rows span far beyond the 16-bit window
    if kind in ("split_tri", "split_tri_shuffled", "shuffled_elems"):
        # the element order defeats the chain patterns: element-coloured chains
        # (greedy colouring in breadth-first order fits these in 8 colours), no
        # atomics on these conforming meshes
        assert plan["plan"] == "element-coloured" and plan["atomic_groups"] == 0, plan


@pytest.mark.parametrize("p", [4, 12])
@pytest.mark.parametrize("kind", ["split_tri", "split_tri_shuffled"])
def test_unstructured_mfma_vs_oracle(gpu, gll, kind, p):
    import sem_oracle
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = make_mesh(kind, p)
    u = np.random.default_rng(p).standard_normal(nodes.shape[1])
    ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p], batched_geometry=True).apply(u)
    op = SEMOperator(p, e2n, nodes, device=gpu, kernel="mfma")
    y = op.apply(torch.from_numpy(u).to(gpu)).cpu().numpy()
    assert op.plan_info()["kernel"] == "mfma"
    # above p = 10 the reference's equispaced->GLL transform (cond(V_eq) ~1e3 at
    # p = 12) limits the oracle itself to ~1e-11 on these small elements
    # (DESIGN.md §6); the north-star bar 1e-10 applies
    assert rel_l2(y, ref) < (TOL if p <= 10 else 1e-10), (kind, p)


@pytest.mark.parametrize("plan_env", ["1", "0"])
def test_forced_plan_structured(gpu, gll, monkeypatch, plan_env):
    """SEM_PLAN=1 forces the element-coloured plan on a structured mesh,
    SEM_PLAN=0 the chain plan with its atomic fallback on split triangles:
    both give the oracle's action."""
    import sem_oracle
    from spectralelementmethod_amd.operators import SEMOperator
    monkeypatch.setenv("SEM_PLAN", plan_env)
    for kind in ("shuffled_elems", "split_tri"):
        nodes, e2n = make_mesh(kind, 4)
        u = np.random.default_rng(1).standard_normal(nodes.shape[1])
        ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_4"]).apply(u)
        op = SEMOperator(4, e2n, nodes, device=gpu)
        plan = op.plan_info()["plan"]
        assert plan == "element-coloured" if plan_env == "1" else plan.startswith("chains")
        y = op.apply(torch.from_numpy(u).to(gpu)).cpu().numpy()
        assert rel_l2(y, ref) < TOL
