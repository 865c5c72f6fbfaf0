"""CPU checks of libsem_hip.so's host side and the Python facade's host
logic: the C ABI loads and exports every symbol include/sem_hip.h declares,
the host basis functions match the reference goldens, and the synthetic mesh
generators reproduce the golden meshes.  No GPU compute is called here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, rel_l2


@pytest.fixture(scope="module")
def lib():
    from spectralelementmethod_amd import _lib
    return _lib.load()


def header_symbols():
    src = open(os.path.join(ROOT, "include", "sem_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sem_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol(lib):
    from spectralelementmethod_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, "no ctypes signature for %s" % s
    assert lib.sem_version().decode().startswith("sem_hip")


def test_library_targets_gfx950():
    from spectralelementmethod_amd._build import LIB_PATH
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("p", range(1, 17))
def test_gll_table_bitwise(lib, gll, p):
    from spectralelementmethod_amd import _lib
    n = p + 1
    x, b, w = np.empty(n), np.empty(n), np.empty(n)
    _lib.check(lib.sem_gll_table(p, _lib.dptr(x), _lib.dptr(b), _lib.dptr(w)))
    assert np.array_equal(x, gll["nodes_%d" % p])
    assert np.array_equal(b, gll["bary_%d" % p])
    assert np.array_equal(w, gll["quad_%d" % p])
    D = np.empty((n, n))
    _lib.check(lib.sem_diff_matrix(n, _lib.dptr(x), _lib.dptr(b), _lib.dptr(D)))
    assert rel_l2(D, gll["D1_%d" % p]) < 1e-15
    V, Vi = np.empty((n, n)), np.empty((n, n))
    _lib.check(lib.sem_interp_eq_matrix(n, _lib.dptr(x), _lib.dptr(b), _lib.dptr(V),
                                        _lib.dptr(Vi)))
    assert np.abs(V - gll["Veq_%d" % p]).max() < 1e-15
    assert np.abs(Vi @ V - np.eye(n)).max() < 1e-9 * max(1.0, np.abs(Vi).max())


def test_gll_table_errors(lib):
    from spectralelementmethod_amd import _lib
    x = np.empty(20)
    with pytest.raises(ValueError):
        _lib.check(lib.sem_gll_table(0, _lib.dptr(x), _lib.dptr(x), _lib.dptr(x)))
    with pytest.raises(NotImplementedError):
        _lib.check(lib.sem_gll_table(17, _lib.dptr(x), _lib.dptr(x), _lib.dptr(x)))


def test_barycentric_known_answer(lib, gll):
    """C twin of sem/bary_interp.c:93-100."""
    from spectralelementmethod_amd import _lib
    f = np.ascontiguousarray(gll["bary_known_f"])
    v = lib.sem_barycentric_lagrange(_lib.dptr(f), 5, 0.654)
    assert v == float(gll["bary_known_value"])
    assert "%g" % v == "0.653996"


@pytest.mark.parametrize("p", range(1, 9))
def test_barycentric_sweep(lib, gll, p):
    from spectralelementmethod_amd import _lib
    f = np.ascontiguousarray(gll["interp_f_%d" % p])
    got = np.array([lib.sem_barycentric_lagrange(_lib.dptr(f), p + 1, x)
                    for x in gll["interp_x_%d" % p]])
    assert np.allclose(got, gll["interp_y_%d" % p], rtol=1e-13, atol=1e-14)


def test_legeval(lib):
    from numpy.polynomial import legendre
    for n in range(0, 14):
        for x in np.linspace(-1, 1, 7):
            assert abs(lib.sem_legeval(x, n) - legendre.legval(x, [0] * n + [1])) < 1e-14


def test_facade_basis_host(gll):
    from spectralelementmethod_amd.basis_functions import (LagrangeGaussLobatto, TensorProductQS)
    for p in (1, 4, 9, 16):
        b = LagrangeGaussLobatto(p)
        assert np.array_equal(b.nodes, gll["nodes_%d" % p])
        assert b.deg == p and b.n_coeffs == p + 1
        # Kronecker property (tests/test_basis.py:60-66, :122-128)
        assert np.allclose(b(b.nodes), np.eye(p + 1), atol=0)
        tb = TensorProductQS(b, b)
        assert tb.coeff_shape == (p + 1, p + 1) and tb.ndim == 2
        assert np.array_equal(tb.get_D1_matrices()[0], b.D1)
        W = tb.quad_rule.get_weights()
        assert W.shape == (p + 1, p + 1)
        # integral of (x+1)(y+1) over [-1,1]^2 = 4 (tests/test_basis.py:100-105 in 2-D)
        X, Y = tb.nodegrid()
        assert abs(tb.quad_rule.integrate((X + 1) * (Y + 1)) - 4.0) < 1e-13
    with pytest.raises(ValueError):
        LagrangeGaussLobatto(0)
    with pytest.raises(NotImplementedError):
        LagrangeGaussLobatto(17)


def test_interpolate_sin(gll):
    """tests/test_basis.py:68-98: interpolation / derivative of sin(pi x)."""
    from spectralelementmethod_amd.basis_functions import LagrangeGaussLobatto
    b = LagrangeGaussLobatto(9)
    xx = np.linspace(-1, 1, 50)
    f = np.sin(np.pi * b.nodes)
    assert np.allclose(b.interpolate(f, xx), np.sin(np.pi * xx), rtol=1e-2, atol=1e-4)
    assert np.allclose(b.D1 @ f, np.pi * np.cos(np.pi * b.nodes), rtol=1e-2, atol=1e-3)


def test_meshgen_matches_golden(poisson_action, axisym_action):
    from spectralelementmethod_amd import meshgen
    for name, (p, nex, ney, w) in {"p4_4x4": (4, 4, 4, 0.0), "p8_8x8w": (8, 8, 8, 0.05),
                                   "p2_6x5": (2, 6, 5, 0.05), "p16_2x2w": (16, 2, 2, 0.05)}.items():
        nodes, e2n = meshgen.structured_square(nex, ney, p, warp=w)
        assert np.array_equal(nodes, poisson_action[name + "_nodes"])
        assert np.array_equal(e2n, poisson_action[name + "_e2n"])
    nodes, e2n = meshgen.annulus(4, 8, 6)
    assert np.array_equal(nodes, axisym_action["p6_4x8_nodes"])
    assert np.array_equal(e2n, axisym_action["p6_4x8_e2n"])


@pytest.mark.parametrize("split", [(0, 3), (3, 7), (0, 7), (5, 7)])
def test_structured_strip(split):
    from spectralelementmethod_amd import meshgen
    p, nex, ney = 4, 7, 3
    gn, ge = meshgen.structured_square(nex, ney, p, warp=0.05)
    ex0, ex1 = split
    ln, le, off = meshgen.structured_strip(nex, ney, p, ex0, ex1, warp=0.05)
    sel = ge[ex0 * ney:ex1 * ney]
    assert np.array_equal(le.astype(np.int64) + off, sel.astype(np.int64))
    assert np.array_equal(ln, gn[:, off:off + ln.shape[1]])
