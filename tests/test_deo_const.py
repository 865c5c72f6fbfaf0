"""The baked D table of the constant-D kernels (csrc/deo_const.h, written by
tools/gen_deo_const.py) against the library's own host computation of D
(sem_gll_table + sem_diff_matrix through LagrangeGaussLobatto, what
SEMOperator hands to sem_set_basis): bit for bit at every order, and its
even-odd halves as make_deo_data (csrc/sem_ctx.h) forms them.  sem_set_basis
compares the context's D with this table and only then takes the
constant-D kernels, so a stale table costs speed, never results -- this
test keeps it from going stale.  CPU only."""
import os
import re

import numpy as np

from conftest import ROOT

HDR = os.path.join(ROOT, "spectralelementmethod_amd", "csrc", "deo_const.h")


def _arrays():
    src = open(HDR).read()
    out = {}
    for n, body in re.findall(r"struct DEOConstData<(\d+)> \{\n(.*?)\n\};", src, flags=re.S):
        d = {}
        for name, vals in re.findall(r"static constexpr double (\w+)\[\d+\] = \{(.*?)\};", body):
            d[name] = np.array([float.fromhex(v.strip()) for v in vals.split(",")])
        out[int(n)] = d
    full = {int(n): np.array([float.fromhex(v.strip()) for v in vals.split(",")])
            for n, vals in re.findall(r"sem_deo_const_d(\d+)\[\d+\] = \{(.*?)\};", src)}
    return out, full


def test_baked_d_is_the_library_d_bitwise():
    from spectralelementmethod_amd.operators import _basis_arrays
    halves, full = _arrays()
    assert sorted(full) == list(range(2, 18)) == sorted(halves)
    for n in range(2, 18):
        _, D, _, _ = _basis_arrays(n - 1, None)
        assert np.array_equal(full[n].reshape(n, n), D), n
        H = n // 2
        P = 0.5 * (D[:H, :H] - D[:H, n - 1:n - 1 - H:-1])
        Q = 0.5 * (D[:H, :H] + D[:H, n - 1:n - 1 - H:-1])
        assert np.array_equal(halves[n]["P"][:H * H].reshape(H, H), P), n
        assert np.array_equal(halves[n]["Q"][:H * H].reshape(H, H), Q), n
        if n % 2:
            assert np.array_equal(halves[n]["cc"], D[:H, H]), n
            assert np.array_equal(halves[n]["rr"], D[H, :H]), n
        if n >= 10:  # transposed copies (DEOData<N>::TR)
            assert np.array_equal(halves[n]["PT"].reshape(H, H), P.T), n
            assert np.array_equal(halves[n]["QT"].reshape(H, H), Q.T), n
