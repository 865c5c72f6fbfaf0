"""Host logic of the discrete facade (CPU): cell geometry orderings, the
reference's node permutations (RCM, static condensation) and hierarchical
DOF numbering, checked against goldens from the reference
(tests/golden/geometry.npz).  Mirrors tests/test_discrete.py of the
reference (single 9x9-node quad built in memory)."""
import numpy as np
import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def geo():
    return load_golden("geometry.npz")


@pytest.mark.parametrize("shp", [(2, 2), (3, 3), (5, 5), (9, 9), (17, 17), (5, 6), (4, 7)])
def test_quadrilateral_orderings(geo, shp):
    from spectralelementmethod_amd.geometry import Quadrilateral
    q = Quadrilateral(*shp)
    key = "%dx%d" % shp
    assert np.array_equal(q.hierarchical_node_order, geo["hier_" + key])
    assert q.n_exterior_nodes == int(geo["next_" + key])
    assert [q.n_sub_geometries(d) for d in range(3)] == list(geo["nsub_" + key])
    assert q.n_interior_nodes == max(shp[0] - 2, 0) * max(shp[1] - 2, 0)


def _mesh():
    from spectralelementmethod_amd import meshgen
    from spectralelementmethod_amd.discrete import Mesh
    nodes, e2n = meshgen.structured_square(3, 2, 4, 0.0)
    return Mesh.from_arrays(nodes, e2n)


def _basis():
    from spectralelementmethod_amd.basis_functions import gll_basis_2d
    return gll_basis_2d(4)


@pytest.mark.parametrize("rcm", [0, 1])
def test_static_condensation_order(geo, rcm):
    from spectralelementmethod_amd.discrete import DOFManagerSC
    mesh = _mesh()
    dm = DOFManagerSC(mesh, 1, _basis(), rcm_order=bool(rcm))
    assert dm.ndof_exterior == int(geo["sc_next_rcm%d" % rcm])
    assert np.array_equal(mesh.element_map(), geo["sc_e2n_rcm%d" % rcm])
    assert np.array_equal(mesh.nodes, geo["sc_nodes_rcm%d" % rcm])
    g = np.stack([fe.global_dof_ind_hier for fe in dm.finite_elements()])
    assert np.array_equal(g, geo["sc_gdof_hier_rcm%d" % rcm])
    fe = next(dm.finite_elements())
    assert np.array_equal(fe.loc_dof_ind_hier, geo["sc_ldof_hier_rcm%d" % rcm])


def test_rcm_order(geo):
    from spectralelementmethod_amd.discrete import DOFManager
    mesh = _mesh()
    DOFManager(mesh, 1, _basis(), rcm_order=True)
    assert np.array_equal(mesh.element_map(), geo["rcm_e2n"])
    assert np.array_equal(mesh.nodes, geo["rcm_nodes"])


def test_single_cell_fixture_and_flags():
    """tests/test_discrete.py:19-41 pattern: one 9x9-node quad on [-1,1]^2."""
    from spectralelementmethod_amd.basis_functions import gll_basis_2d
    from spectralelementmethod_amd.discrete import DOFManager, Mesh
    from spectralelementmethod_amd.geometry import Quadrilateral
    geometry = Quadrilateral(9, 9)
    mesh = Mesh(geometry.ndim)
    nodes = np.mgrid[tuple(slice(-1, 1, s * 1j) for s in geometry.shape)].reshape(2, -1)
    mesh.set_nodes(nodes)
    mesh.add_geometry(geometry)
    mesh.new_region("*")
    mesh.add_cell(np.arange(geometry.n_nodes).reshape(geometry.shape), 0, 0)
    dm = DOFManager(mesh, basis=gll_basis_2d(8))
    assert dm.ndof == 81 and mesh.n_cells == 1
    fe = next(dm.finite_elements())
    assert fe.n_nodes == 81 and fe.n_exterior_nodes == 32 and fe.n_interior_nodes == 49
    # default rcm_order=True renumbers the nodes (sem/discrete.py:123-124)
    assert np.array_equal(np.sort(fe.node_ind.ravel()), np.arange(81))
    assert np.array_equal(fe.node_ind, np.arange(81)[::-1].reshape(9, 9))
    with pytest.raises(ValueError):
        next(dm.finite_elements(bogus=True))
    with pytest.raises(AttributeError):
        fe.x_phys  # not requested
    with pytest.raises(ValueError):
        mesh.set_nodes(np.zeros((3, 4)))


def test_band_order_recovers_band():
    """band_order (the host half of the device direct solve of the condensed
    system): reverse Cuthill-McKee brings a randomly permuted banded,
    non-symmetric matrix back to a small bandwidth, and the permuted matrix
    is the original one reordered."""
    import numpy as np
    from scipy import sparse
    from spectralelementmethod_amd.discrete import band_order
    rng = np.random.default_rng(3)
    n, bw = 500, 6
    A = sparse.diags([rng.standard_normal(n - abs(k)) for k in range(-bw, bw + 1)],
                     list(range(-bw, bw + 1)), format="csr")
    q = rng.permutation(n)
    Aq = A[q][:, q]
    perm, Ap, kl, ku = band_order(Aq)
    assert sorted(perm.tolist()) == list(range(n))
    assert kl <= 2 * bw and ku <= 2 * bw
    assert abs(Ap - Aq[perm][:, perm]).max() == 0.0
