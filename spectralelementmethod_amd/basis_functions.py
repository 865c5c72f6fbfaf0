"""Lagrange / tensor-product GLL bases (mirror of sem/basis_functions.py).

Same class names, properties and argument meaning as the reference:
``BarycentricLagrange`` (:185-341), ``LagrangeGaussLobatto`` (:344-393),
``TensorProduct`` (:396-659), ``NodalTensorProduct`` (:662-680) and
``TensorProductQS`` (:683-697).

Where the numbers come from:
* GLL nodes / barycentric / quadrature weights: ``sem_gll_table`` in
  libsem_hip.so (the reference's HDF5 values for orders 1..10, its mpmath
  generator's values for 11..16; the reference itself stops at 10 with
  NotImplementedError, sem/basis_functions.py:366-369 -- here the limit is 16).
* D1, basis evaluation and V_eq: the library's C twins of
  sem/basis_functions.py:213-255.
* Array-valued tensor operations (``deriv``, ``gradient``,
  ``compute_coeffs_grid_eq``, ``interpolate_on_grid_eq``) run on the GPU
  through ``sem_tensor_apply``; numpy inputs are staged to the device and the
  result is returned as numpy.  There is no host implementation of them.
"""
import itertools as it

import numpy as np

from . import _lib
from .quadratures import Quadrature1D, TensorQuadratureRule

MAX_ORDER = 16


def _as_f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _tensor_apply(n, A0, A1, coeffs):
    """out[..., m, q] = sum A0[m, r] A1[q, s] in[..., r, s] on the device."""
    import torch
    lib = _lib.load()
    is_np = not isinstance(coeffs, torch.Tensor)
    if is_np:
        t = torch.as_tensor(_as_f64(coeffs)).cuda()
    else:
        t = coeffs.to(dtype=torch.float64).contiguous()
        if not t.is_cuda:
            t = t.cuda()
    if t.shape[-2:] != (n, n):
        raise ValueError("trailing shape must be (%d, %d)" % (n, n))
    out = torch.empty_like(t)
    batch = t.numel() // (n * n)
    a0 = None if A0 is None else _lib.dptr(_as_f64(A0))
    a1 = None if A1 is None else _lib.dptr(_as_f64(A1))
    with torch.cuda.device(t.device):
        _lib.check(lib.sem_tensor_apply(n, batch, a0, a1, _lib.tptr(t), _lib.tptr(out),
                                        _lib.stream_ptr()))
    if is_np:
        return out.cpu().numpy()
    return out


class _Basis(object):
    def get_coeff_rank(self, coeffs):
        return coeffs.ndim - self.ndim


class _Nodal(object):
    @property
    def nodes(self):
        return self._nodes

    @property
    def n_nodes(self):
        return self._nodes.size

    @property
    def n_coeffs(self):
        return self._nodes.size


class _QuadSupported(object):
    @property
    def quad_rule(self):
        return self._quad_rule

    def __init__(self, quad_wts):
        self._quad_rule = Quadrature1D(self._nodes, quad_wts)

    def integrate(self, coeffs):
        return self._quad_rule.integrate(coeffs)


class _Basis1D(_Basis):
    @property
    def ndim(self):
        return 1

    @property
    def coeff_shape(self):
        return (self.n_coeffs,)

    @property
    def D1(self):
        return self._D1

    def get_D1_matrix(self, dim=0):
        return self._D1

    def get_D1_matrices(self):
        return [self._D1]

    def deriv(self, coeffs):
        return np.einsum("mr,...r->...m", self._D1, coeffs)

    def gradient(self, coeffs):
        return self.deriv(coeffs)


class BarycentricLagrange(_Basis1D, _Nodal):
    """Lagrange basis through given nodes in barycentric form
    (sem/basis_functions.py:185-341)."""

    @property
    def deg(self):
        return self._nodes.size - 1

    @property
    def bary_wts(self):
        return self._bary_wts

    def __init__(self, nodes, bary_wts):
        lib = _lib.load()
        self._nodes = _as_f64(nodes)
        self._bary_wts = _as_f64(bary_wts)
        n = self._nodes.size
        D1 = np.empty((n, n))
        _lib.check(lib.sem_diff_matrix(n, _lib.dptr(self._nodes), _lib.dptr(self._bary_wts),
                                       _lib.dptr(D1)))
        self._D1 = D1
        Veq = np.empty((n, n))
        Vinv = np.empty((n, n))
        _lib.check(lib.sem_interp_eq_matrix(n, _lib.dptr(self._nodes), _lib.dptr(self._bary_wts),
                                            _lib.dptr(Veq), _lib.dptr(Vinv)))
        self._interp_eq_mat = Veq
        self._interp_eq_inv = Vinv

    def __call__(self, x):
        """B[..., j] = l_j(x[...]) (sem/basis_functions.py:226-255)."""
        lib = _lib.load()
        x = _as_f64(x)
        n = self._nodes.size
        out = np.empty(x.shape + (n,))
        _lib.check(lib.sem_lagrange_eval(n, _lib.dptr(self._nodes), _lib.dptr(self._bary_wts),
                                         x.size, _lib.dptr(x.reshape(-1)),
                                         _lib.dptr(out.reshape(-1, n))))
        return out

    def interpolate(self, f, x, broadcast=False):
        """Lagrange interpolant of nodal values ``f`` at ``x``
        (sem/basis_functions.py:260-341)."""
        B = self(np.asarray(x, dtype=np.float64))
        f = np.asarray(f, dtype=np.float64)
        if broadcast:
            xnd = np.ndim(x)
            n_free = f.ndim - 1 - xnd
            f_ax = [Ellipsis] + list(range(n_free)) + [n_free]
            return np.einsum(B, [Ellipsis, n_free], f, f_ax,
                             [Ellipsis] + list(range(n_free)))[()]
        return np.inner(B, f)[()]

    def __repr__(self):
        return "{}(deg={})".format(self.__class__.__name__, self.deg)


class LagrangeGaussLobatto(BarycentricLagrange, _QuadSupported):
    """Lagrange basis through the GLL nodes (sem/basis_functions.py:344-393)."""

    def __init__(self, order):
        if order < 1:
            raise ValueError("Must specify an order of 1 or greater.")
        if order > MAX_ORDER:
            raise NotImplementedError("Basis only available up to order {}.".format(MAX_ORDER))
        lib = _lib.load()
        n = order + 1
        nodes, bary, quad = np.empty(n), np.empty(n), np.empty(n)
        _lib.check(lib.sem_gll_table(order, _lib.dptr(nodes), _lib.dptr(bary), _lib.dptr(quad)))
        self._n_coeffs = n
        BarycentricLagrange.__init__(self, nodes, bary)
        _QuadSupported.__init__(self, quad)


class TensorProduct(_Basis):
    """Tensor product of 1-D bases (sem/basis_functions.py:396-659)."""

    @property
    def ndim(self):
        return self._ndim

    @property
    def coeff_shape(self):
        return self._coeff_shape

    @property
    def n_subbases(self):
        return len(self._subbases)

    @property
    def n_coeffs(self):
        return self._n_coeffs

    @property
    def D1(self):
        return self._D1_mats

    def __init__(self, *subbases):
        if len(subbases) < 1:
            raise ValueError("Tensor product basis must comprise at "
                             "least two lower dimensional bases.")
        self._subbases = subbases
        self._ndim = sum(b.ndim for b in subbases)
        self._coeff_shape = tuple(it.chain.from_iterable(b.coeff_shape for b in subbases))
        self._subbasis_dims = []
        self._D1_mats = []
        self._n_coeffs = 1
        dim_first = 0
        for b in subbases:
            self._n_coeffs *= b.n_coeffs
            if isinstance(b, _Basis1D):
                self._subbasis_dims.append(dim_first)
                dim_first += 1
                self._D1_mats.append(b.D1)
            else:
                self._subbasis_dims.append(slice(dim_first, dim_first + b.ndim))
                dim_first += b.ndim
                self._D1_mats.extend(b._D1_mats)

    def get_D1_matrix(self, dim):
        return self._D1_mats[dim]

    def get_D1_matrices(self):
        return self._D1_mats[:]

    def get_subbasis(self, dim):
        if self.ndim == 2:
            return self._subbases[dim]
        subbases = self._subbases[dim + 1:] + self._subbases[:dim]
        return type(self)(*subbases)

    def iter_subbases(self, reverse=False):
        if not reverse:
            return zip(self._subbasis_dims, self._subbases)
        return zip(reversed(self._subbasis_dims), reversed(self._subbases))

    def _square(self):
        if self.ndim != 2 or self._coeff_shape[0] != self._coeff_shape[1]:
            raise NotImplementedError("device tensor ops support 2-D bases with n0 == n1")
        return self._coeff_shape[0]

    def __call__(self, x):
        if len(x) != self.ndim:
            raise ValueError("Cannot evaluate {}-dimensional basis at a {}-dimensional set of "
                             "points".format(self.ndim, len(x)))
        args = []
        for i, (dim, b) in enumerate(self.iter_subbases()):
            args.append(b(x[dim]))
            args.append([Ellipsis, i])
        args.append([Ellipsis] + list(range(self.n_subbases)))
        return np.einsum(*args)

    def interpolate(self, coeffs, x):
        out = coeffs
        for dim, b in self.iter_subbases(reverse=True):
            out = b.interpolate(out, x[dim], broadcast=dim < self.ndim - 1)
        return out

    def deriv(self, coeffs, dim):
        """D along ``dim`` (D(x)I for dim 0, I(x)D for dim 1) on the GPU
        (sem/basis_functions.py:626-639)."""
        n = self._square()
        D = self._D1_mats[dim]
        return _tensor_apply(n, D if dim == 0 else None, D if dim == 1 else None, coeffs)

    def gradient(self, coeffs):
        """[ndim, ..., n, n] (sem/basis_functions.py:641-650)."""
        g0 = self.deriv(coeffs, 0)
        g1 = self.deriv(coeffs, 1)
        if isinstance(g0, np.ndarray):
            return np.stack([g0, g1])
        import torch
        return torch.stack([g0, g1])

    def compute_coeffs_grid_eq(self, values):
        """Coefficients from values on the equispaced grid: solve V_eq along
        each dimension (sem/basis_functions.py:599-624), on the GPU."""
        n = self._square()
        Vinv0 = self._subbases[0]._interp_eq_inv
        Vinv1 = self._subbases[1]._interp_eq_inv
        return _tensor_apply(n, Vinv0, Vinv1, values)

    def interpolate_on_grid_eq(self, coeffs):
        """Values on the equispaced grid (sem/basis_functions.py:539-569)."""
        n = self._square()
        return _tensor_apply(n, self._subbases[0]._interp_eq_mat,
                             self._subbases[1]._interp_eq_mat, coeffs)

    def __repr__(self):
        return "{}({})".format(self.__class__.__name__,
                               ", ".join(repr(b) for b in self._subbases))


class NodalTensorProduct(TensorProduct):
    @property
    def nodes(self):
        return tuple(sb.nodes for sb in self._subbases)

    def __init__(self, *subbases):
        for sb in subbases:
            if not isinstance(sb, _Nodal):
                raise ValueError("All subbases must be nodal.")
        TensorProduct.__init__(self, *subbases)

    def nodegrid(self, sparse=False):
        return np.meshgrid(*self.nodes, indexing="ij", sparse=sparse)


class TensorProductQS(NodalTensorProduct, _QuadSupported):
    """Nodal tensor-product basis with its quadrature rule
    (sem/basis_functions.py:683-697)."""

    def __init__(self, *subbases):
        if not all(isinstance(b, _QuadSupported) for b in subbases):
            raise ValueError("All subbases must be supported by a quadrature rule.")
        NodalTensorProduct.__init__(self, *subbases)
        self._quad_rule = TensorQuadratureRule(*(b._quad_rule for b in self._subbases))


def gll_basis_2d(p):
    """Convenience: TensorProductQS(LagrangeGaussLobatto(p), same)."""
    b = LagrangeGaussLobatto(p)
    return TensorProductQS(b, b)
