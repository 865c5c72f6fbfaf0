"""spectralelementmethod_amd -- MI355X-native spectral-element operator engine.

Drop-in for the tensor-product hot path of nchisholm/SpectralElementMethod
(sem/discrete.py operator apply/assembly, sem/basis_functions.py tensor
product evaluation, sem/mapping.py + sem/quadratures.py geometry, sem/linalg.py
det/inverse, sem/bary_interp.c).  Host API mirrors the reference's module and
class names; the arithmetic runs in hand-written HIP kernels for gfx950
(libsem_hip.so, C ABI in include/sem_hip.h).
"""
__version__ = "0.1.0"


def lib():
    from . import _lib
    return _lib.load()
