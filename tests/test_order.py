"""Native reverse Cuthill-McKee (sem_node_degrees / sem_cuthill_mckee,
discrete.rcm_permutation) against the reference's own recipe: scipy's
reverse_cuthill_mckee on the boolean graph joining every two nodes of a cell
(sem/discrete.py:142-178, DOFManagerSC: :361-402).  Host only."""
import numpy as np
import pytest
from scipy.sparse import csgraph

from spectralelementmethod_amd import meshgen
from spectralelementmethod_amd.discrete import _pair_graph, rcm_permutation


def _cases():
    out = []
    for p, ne in [(1, 5), (2, 7), (3, 9), (4, 16), (8, 24)]:
        nodes, e2n = meshgen.structured_square(ne, ne + 1, p, warp=0.05)
        out.append(("square_p%d" % p, e2n.reshape(e2n.shape[0], -1), nodes.shape[1]))
    nodes, e2n = meshgen.structured_square(12, 10, 4)
    e2 = meshgen.shuffle_elements(e2n, seed=3)
    n2, e3 = meshgen.shuffle_nodes(nodes, e2, seed=4)
    out.append(("shuffled", e3.reshape(e3.shape[0], -1), n2.shape[1]))
    nodes, e2n = meshgen.structured_cube(4, 3, 3, 3)
    out.append(("cube_p3", e2n.reshape(e2n.shape[0], -1), nodes.shape[1]))
    nodes, e2n = meshgen.annulus(8, 6, 4)
    out.append(("annulus_p4", e2n.reshape(e2n.shape[0], -1), nodes.shape[1]))
    # two components and an unreferenced node
    nodes, e2n = meshgen.structured_square(3, 3, 2)
    m = e2n.reshape(e2n.shape[0], -1)
    out.append(("two_components", np.concatenate([m, m + nodes.shape[1] + 1]),
                2 * nodes.shape[1] + 1))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_rcm_equals_scipy(case):
    _, maps, n = case
    ref = csgraph.reverse_cuthill_mckee(_pair_graph(maps, n), True)
    got = rcm_permutation(maps, n)
    assert got.dtype == ref.dtype
    np.testing.assert_array_equal(got, ref)


def test_degrees_equal_scipy():
    import ctypes as C
    from spectralelementmethod_amd import _lib
    nodes, e2n = meshgen.structured_square(6, 5, 4, warp=0.05)
    m = np.ascontiguousarray(e2n.reshape(e2n.shape[0], -1), dtype=np.uint32)
    g = _pair_graph(m, nodes.shape[1])
    deg = np.empty(nodes.shape[1], dtype=np.int32)
    _lib.check(_lib.load().sem_node_degrees(m.ctypes.data_as(C.c_void_p), m.shape[0],
                                            m.shape[1], nodes.shape[1],
                                            deg.ctypes.data_as(C.c_void_p)))
    # scipy's _node_degrees: row length, the diagonal counted twice
    np.testing.assert_array_equal(deg, np.diff(g.indptr) + 1)


def test_rcm_rejects_bad_map():
    with pytest.raises(ValueError):
        rcm_permutation(np.array([[0, 1, 5]]), 3)



def test_dofmanager_hex_rcm_numbering():
    """DOFManager's default RCM on a hexahedral mesh built with
    Mesh.from_arrays: scipy's permutation of the 3-D pair graph; the caller's
    arrays are left alone."""
    from spectralelementmethod_amd.basis_functions import LagrangeGaussLobatto, TensorProductQS
    from spectralelementmethod_amd.discrete import DOFManager, Mesh
    p = 3
    nodes, e2n = meshgen.structured_cube(3, 2, 2, p, warp=0.05)
    e2n0, nodes0 = e2n.copy(), nodes.copy()
    mesh = Mesh.from_arrays(nodes, e2n)
    b = LagrangeGaussLobatto(p)
    DOFManager(mesh, 1, TensorProductQS(b, b, b))
    perm = csgraph.reverse_cuthill_mckee(_pair_graph(e2n.reshape(e2n.shape[0], -1),
                                                     nodes.shape[1]), True)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size, dtype=perm.dtype)
    assert np.array_equal(e2n, e2n0) and np.array_equal(nodes, nodes0)
    assert np.array_equal(mesh.nodes, nodes[:, perm])
    assert np.array_equal(mesh.element_map(), inv[e2n])


def test_rcm_equals_scipy_cfg2_size():
    """BASELINE config 2's mesh (256^2 cells, p = 8, 4.2M nodes): the native
    walk still reproduces scipy's permutation exactly."""
    nodes, e2n = meshgen.structured_square(256, 256, 8, warp=0.05)
    maps = e2n.reshape(e2n.shape[0], -1)
    ref = csgraph.reverse_cuthill_mckee(_pair_graph(maps, nodes.shape[1]), True)
    np.testing.assert_array_equal(rcm_permutation(maps, nodes.shape[1]), ref)
