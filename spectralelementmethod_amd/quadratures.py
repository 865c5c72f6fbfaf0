"""Quadrature rules on the GLL nodes (host-side setup data).

Mirrors sem/quadratures.py: ``Quadrature1D`` (:14-118) and
``TensorQuadratureRule`` (:203-275).  These carry n <= 17 weights; the
per-node weighting on the hot path (detJ * w_m * w_n) happens inside the
device geometry kernel (csrc/sem_device.hip, k_geometry).
"""
import numpy as np


class Quadrature1D(object):
    """An n-point rule on [-1, 1] (sem/quadratures.py:14-118)."""

    @property
    def ndim(self):
        return 1

    @property
    def n_points(self):
        return len(self._abscissa)

    def __init__(self, abscissa, weights):
        self._abscissa = np.asarray(abscissa, dtype=np.float64)
        self._weights = np.asarray(weights, dtype=np.float64)

    def __call__(self, f):
        try:
            return np.dot(self._weights, f)
        except TypeError:
            return np.dot(self._weights, f(self._abscissa))

    @property
    def abscissa(self):
        return self._abscissa

    @property
    def weights(self):
        return self._weights

    def get_abscissa(self):
        return self._abscissa

    def get_weights(self):
        return self._weights

    def integrate(self, values):
        values = np.asarray(values)
        assert values.shape[0] == self._weights.size
        rank_shape = values.shape[1:]
        out = np.dot(self._weights, values.reshape(self._weights.size, -1))
        return out.reshape(rank_shape)

    def xweight(self, f_vals):
        """values times weights, not summed (sem/quadratures.py:111-115)."""
        return f_vals * self._weights

    def __repr__(self):
        return "{}(n={})".format(self.__class__.__name__, self.n_points)


class TensorQuadratureRule(object):
    """Tensor product of 1-D rules (sem/quadratures.py:203-275)."""

    @property
    def ndim(self):
        return self._ndim

    @property
    def n_points(self):
        return self._n_points

    @property
    def n_subquads(self):
        return len(self._weights)

    @property
    def shape(self):
        return tuple(len(a) for a in self._abscissa)

    @property
    def abscissa(self):
        return self._abscissa[:]

    @property
    def weights(self):
        return self._weights[:]

    def __init__(self, *quad_rules):
        self._ndim = 0
        self._n_points = 1
        self._abscissa = []
        self._weights = []
        for rule in quad_rules:
            self._ndim += rule.ndim
            self._n_points *= rule.abscissa.size
            self._abscissa.append(rule.abscissa)
            self._weights.append(rule.weights)

    def get_abscissa(self, sparse=False):
        return np.meshgrid(*self.abscissa, indexing="ij", sparse=sparse)

    def get_weights(self, sparse=False):
        grid = np.meshgrid(*self._weights, indexing="ij", sparse=sparse)
        return grid if sparse else np.prod(grid, axis=0)

    def __call__(self, f):
        try:
            return self.integrate(f)
        except TypeError:
            return self.integrate(f(self._abscissa))

    def integrate(self, f_vals):
        out = f_vals
        for wt in reversed(self._weights):
            out = np.inner(out, wt)
        return out

    def xweight(self, f_vals):
        """values times the tensor weights, not summed (:268-275)."""
        out = np.array(f_vals, dtype=np.float64, copy=True)
        for wt in self.get_weights(sparse=True):
            out *= wt
        return out
