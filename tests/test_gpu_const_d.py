"""D of the standard GLL basis as compile-time constants in the Poisson
column kernels (csrc/deo_const.h, tools/gen_deo_const.py).

sem_set_basis compares the context's D with the baked table bit for bit and
only then runs the constant-D instantiations (at the orders const_d_order
picks, or at every order with SEM_CONST_D=1, as here) (the contractions, their order
of operations and their FMAs are those of the argument form): the results
must equal the argument form (SEM_CONST_D=0) exactly, for every plan and
geometry, with the fused dot, in accumulate mode, and against the oracle.
A basis that is not the baked one (a perturbed D) runs the argument form."""
import numpy as np
import pytest

from conftest import rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


CASES = [(1, 9, 64, "auto", "1"), (2, 7, 168, "auto", "1"), (4, 9, 96, "auto", "0"),
         (6, 8, 72, "auto", "1"), (8, 17, 112, "nodal", "1"), (8, 17, 112, "stored", "1"),
         (8, 9, 40, "nodal", "0"), (10, 5, 30, "auto", "1"), (12, 9, 32, "auto", "1"),
         (14, 6, 16, "auto", "0"), (16, 7, 12, "auto", "1")]


@pytest.mark.parametrize("p,nex,ney,geometry,seam", CASES)
def test_const_d_is_bitwise_the_argument_form(gpu, gll, monkeypatch, p, nex, ney, geometry,
                                              seam):
    import sem_oracle
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp=0.05)
    rng = np.random.default_rng(p)
    u = rng.standard_normal(nodes.shape[1])
    y0 = rng.standard_normal(nodes.shape[1])
    ut, y0t = torch.from_numpy(u).to(gpu), torch.from_numpy(y0).to(gpu)
    monkeypatch.setenv("SEM_SEAM", seam)
    out = {}
    for cd in ("1", "0"):
        monkeypatch.setenv("SEM_CONST_D", cd)
        op = SEMOperator(p, e2n, nodes, device=gpu, kernel="column", geometry=geometry)
        info = op.plan_info()
        assert info["const_d"] == (cd == "1"), info
        y = op.apply(ut)
        ya = op.apply(ut, y0t.clone(), accumulate=True)
        dot = op.apply_dot(ut)[1].item()
        out[cd] = (y, ya, dot, info["plan"])
    assert out["1"][3] == out["0"][3]
    assert torch.equal(out["1"][0], out["0"][0])
    assert torch.equal(out["1"][1], out["0"][1])
    assert out["1"][2] == out["0"][2]
    # above p = 10 against the extended-precision evaluation (the
    # reference's float64 geometry transform is itself the larger error
    # there)
    if p <= 10:
        ref = sem_oracle.PoissonProblem(nodes, e2n, gll["half_%d" % p],
                                        batched_geometry=True).apply(u)
    else:
        ref = sem_oracle.poisson_apply_extended(nodes, e2n, gll["half_%d" % p], u)
    assert rel_l2(out["1"][0].cpu().numpy(), ref) < 1e-10


def test_other_basis_runs_the_argument_form(gpu, monkeypatch):
    """A D that differs from the baked one in one bit is not taken as
    constant: the kernels read the caller's D (and agree with the oracle's
    use of that same D)."""
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.operators import SEMOperator
    monkeypatch.setenv("SEM_CONST_D", "1")
    p = 8
    nodes, e2n = meshgen.structured_square(17, 112, p, warp=0.05)
    op = SEMOperator(p, e2n, nodes, device=gpu, kernel="column")
    assert op.plan_info()["const_d"]
    D = op.D.copy()
    D[1, 2] = np.nextafter(D[1, 2], 1.0)
    D[p - 1, p - 2] = -D[1, 2]  # keep the centro-antisymmetry sem_set_basis checks
    lib = op._lib
    from spectralelementmethod_amd import _lib
    _lib.check(lib.sem_set_basis(op._ctx, _lib.dptr(np.ascontiguousarray(D)),
                                 _lib.dptr(op.w)))
    assert not op.plan_info()["const_d"]
