"""sem_apply_dot: the Poisson action with u . K u summed inside its own
launches on the seam plan (each node's final value is stored exactly once:
u[gid] * value at that store, per-workgroup partials, one fixed-order sum),
and the separate-pass fallback on the other plans.  The action equals
sem_apply bit for bit; the dot equals torch's u . y to rounding (1e-13
relative: a different summation order) and is the same run to run."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("p,nex,ney,env", [
    (8, 40, 70, {"SEM_SEAM": "1"}),                             # consecutive groups, seams
    (8, 40, 70, {"SEM_SEAM": "1", "SEM_BLOCK_ROUNDS": "4"}),    # block layout, seams
    (4, 30, 50, {"SEM_SEAM": "1", "SEM_BLOCK_ROUNDS": "3"}),
    (12, 9, 14, {"SEM_SEAM": "1"}),
    (16, 6, 7, {}),                                             # AUTO (seams at high order)
    (8, 40, 70, {"SEM_SEAM": "0"}),                             # colour launches: fallback
])
@pytest.mark.parametrize("geometry", ["nodal", "stored"])
def test_apply_dot(gpu, monkeypatch, p, nex, ney, env, geometry):
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    op = SEMOperator(p, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
    u = torch.from_numpy(np.random.default_rng(p).standard_normal(nodes.shape[1])).to(gpu)
    y_ref = op.apply(u)
    y, dot = op.apply_dot(u)
    assert torch.equal(y, y_ref)
    ref = torch.dot(u, y_ref).item()
    assert abs(dot.item() - ref) <= 1e-13 * abs(ref), (dot.item(), ref)
    _, dot2 = op.apply_dot(u)
    assert dot2.item() == dot.item()  # fixed-order partial sums
