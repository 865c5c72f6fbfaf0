"""Element mappings (mirror of sem/mapping.py: ``Mapping`` :79-181).

In the reference each ``Mapping`` computes x_phys, J, J^-1 and detJ for one
cell on the host when it is constructed (sem/mapping.py:86-119).  Here the
fields of ALL cells come from one device launch (``sem_geom_fields``,
k_geometry in csrc/sem_kernels.h) and a ``Mapping`` is a view of cell i.

Out of scope: the Newton inverse map ``Mapping.inv``
(point location) and face ``SubMapping``s (boundary-condition surface
terms); they raise NotImplementedError.
"""
import numpy as np


class OutsideDomain(Exception):
    """Physical point outside an element (sem/mapping.py:12-16)."""


class Mapping(object):
    def __init__(self, basis, fields, index, compute_flags):
        self._basis = basis
        self._fields = fields
        self._i = index
        self._cmpflags = dict(compute_flags)

    @property
    def ndim(self):
        return self._basis.ndim

    def _get(self, key, flag):
        if not self._cmpflags.get(flag, False):
            raise AttributeError("'%s' was not requested (compute flag %r)" % (key, flag))
        return self._fields[key][self._i]

    @property
    def x_phys(self):
        return self._get("x_phys", "x_phys")

    @property
    def J(self):
        return self._get("J", "Jacobian")

    @property
    def invJ(self):
        return self._get("invJ", "Jacobian")

    @property
    def detJ(self):
        return self._get("detJ", "Jacobian")

    def __call__(self, x_param):
        """Parametric -> physical coordinates (sem/mapping.py:138-141)."""
        return np.moveaxis(self._basis.interpolate(self.x_phys, x_param), -1, 0)

    def inv(self, x_phys, x_param_guess=None):
        raise NotImplementedError("point location (Mapping.inv, sem/mapping.py:143-178) is out "
                                  "of scope for the operator engine")

    def get_submapping(self, face):
        raise NotImplementedError("face sub-mappings (sem/mapping.py:184-272) are out of scope")
