"""Device operator context: the batched replacement of the reference's
per-element Python loop.

The reference applies an operator by iterating ``DOFManager.finite_elements``
(sem/discrete.py:189-209), building each element's dense operator with
einsums (examples/poisson.py:168-193; examples/squirmer-axisymmetric.py:
193-254), multiplying it into the element's slice of the global vector
(``np.einsum('pqrs,rs', Op, u[loc])``, squirmer:286,293) and adding the
result back through ``FiniteElement.node_ind`` (sem/discrete.py:658-663).

``SEMOperator`` owns one ``sem_ctx`` of libsem_hip.so on one GPU and does the
same computation for all elements in one kernel launch, matrix-free by sum
factorisation.  There is no CPU path: constructing it without the built
library or without a GPU raises.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib
from .basis_functions import LagrangeGaussLobatto, TensorProductQS

POISSON = _lib.OP_POISSON
AXISYM_STOKES = _lib.OP_AXISYM_STOKES
AXISYM_NS = _lib.OP_AXISYM_NS
AXISYM_NS_JVP = _lib.OP_AXISYM_NS_JVP
_KIND_NAMES = {"poisson": POISSON, "laplace": POISSON, "stiffness": POISSON,
               "axisym_stokes": AXISYM_STOKES, "stokes_axisym": AXISYM_STOKES,
               "axisym_ns": AXISYM_NS, "axisym_ns_jvp": AXISYM_NS_JVP}


def op_kind(kind):
    if isinstance(kind, str):
        try:
            return _KIND_NAMES[kind.lower()]
        except KeyError:
            raise ValueError("unknown operator kind %r" % kind)
    if kind not in (POISSON, AXISYM_STOKES, AXISYM_NS, AXISYM_NS_JVP):
        raise ValueError("unknown operator kind %r" % kind)
    return int(kind)


def _geom_key(kind):
    """The two Navier-Stokes kinds share one set of geometric factors."""
    return AXISYM_NS if kind == AXISYM_NS_JVP else kind


def _device_index(device):
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError("SEMOperator needs a GPU (no HIP device visible)")
        return torch.cuda.current_device()
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError("SEMOperator runs on a HIP device, got %s" % device)
    return device.index if device.index is not None else torch.cuda.current_device()


def _basis_arrays(p, basis, ndim=2):
    if basis is None:
        b1 = LagrangeGaussLobatto(p)
        basis = TensorProductQS(*([b1] * ndim))
    mats = basis.get_D1_matrices()
    if len(mats) != ndim:
        raise ValueError("basis spans %d dimensions, the mesh %d" % (len(mats), ndim))
    D = np.ascontiguousarray(mats[0], dtype=np.float64)
    if not all(np.array_equal(D, Dk) for Dk in mats[1:]):
        raise NotImplementedError("anisotropic tensor bases are not supported by the kernels")
    w = np.ascontiguousarray(basis.quad_rule.weights[0], dtype=np.float64)
    sub = basis._subbases[0]
    Vinv = np.ascontiguousarray(sub._interp_eq_inv, dtype=np.float64)
    return basis, D, w, Vinv


def reference_x_phys(nodes, e2n, basis):
    """x_phys [E, 2, n, n] of every element as the reference computes it:
    Mapping._compute_x_phys (sem/mapping.py:98-103) calls
    TensorProduct.compute_coeffs_grid_eq (sem/basis_functions.py:599-624) on
    the element's equispaced nodes [2, n, n]: LAPACK LU solves with V_eq's
    factors (sem/basis_functions.py:221-224), first with
    the n x 2n right-hand side of columns (xi1 index, component), then with
    the one of columns (xi0 index, component).  The calls are made element by
    element with exactly those right-hand sides, because the LAPACK/BLAS
    triangular solves round differently for other batchings (5e-11 at p = 16
    when all elements go to one call).  Each call is LAPACK dgetrs on the
    factors of lu_factor, as lu_solve makes it, here issued directly on an
    in-place Fortran-ordered view of the element's right-hand side (no
    per-call checks or copies: 17-30 against 50-85 us per element at p = 8 /
    16, bitwise the same; tests/test_oracle_golden.py)."""
    import scipy.linalg as spla
    from scipy.linalg import lapack
    sub = basis._subbases[0]
    # V_eq with the reference's own float64 expression (the barycentric
    # second form of BarycentricLagrange.__call__, sem/basis_functions.py:
    # 226-255; the library's C twin can differ in the last bit above p = 10)
    xn, bw = np.asarray(sub.nodes, dtype=np.float64), np.asarray(sub.bary_wts, dtype=np.float64)
    x_eq = np.linspace(-1, 1, xn.size)
    with np.errstate(divide="ignore", invalid="ignore"):
        kern = bw / (x_eq[:, None] - xn)
        veq = kern / kern.sum(axis=-1)[:, None]
    veq[np.isnan(veq)] = 1.0
    lu, piv = spla.lu_factor(veq)
    X = np.asarray(nodes)[:, np.asarray(e2n).astype(np.int64)]  # [2, E, n, n] = [c, e, i, j]
    E, n = X.shape[1], X.shape[2]
    getrs = lapack.dgetrs
    # solve along xi0: the element's n x 2n right-hand side [i, (j, c)],
    # Fortran order = the C block [(j, c), i]
    B = np.ascontiguousarray(X.transpose(1, 3, 0, 2)).reshape(E, 2 * n, n)
    for e in range(E):
        _, info = getrs(lu, piv, B[e].T, overwrite_b=1)
        assert info == 0
    # along xi1: right-hand side [j, (i, c)], Fortran order = C [(i, c), j]
    B = np.ascontiguousarray(B.reshape(E, n, 2, n).transpose(0, 3, 2, 1)).reshape(E, 2 * n, n)
    for e in range(E):
        _, info = getrs(lu, piv, B[e].T, overwrite_b=1)
        assert info == 0
    return np.ascontiguousarray(B.reshape(E, n, 2, n).transpose(0, 2, 1, 3))  # [e, c, i, j]


class SEMOperator(object):
    """Matrix-free spectral-element operators on one GPU.

    Parameters
    ----------
    p : int
        Polynomial order (1..16 on quadrilaterals and on hexahedra).
    e2n : array-like uint32 [n_elem, p+1, p+1] or [n_elem, p+1, p+1, p+1]
        Element -> global node map (lexicographic, sem/discrete.py:1044); a
        4-D map makes a hexahedral operator (include/sem_hip.h
        sem_ctx_create_nd: Poisson, stored geometry).
    nodes : array-like float64 [ndim, n_node]
        Mesh node coordinates (equispaced within each element).
    dofs_per_node : int
        1 for the Poisson operator, 2 (interleaved psi, omega) for the
        axisymmetric Stokes block.
    basis : TensorProductQS, optional
    device : torch.device or str, optional
    geometry : {"auto", "nodal", "stored"}
        How the Poisson action gets its geometric factors: re-derived per
        quadrature node from x_phys per global node ("nodal", least HBM
        traffic) or streamed from precomputed per-element factors ("stored");
        "auto" (default) picks per order (nodal at p = 1, 2, 4, 5, 8: the
        library's measured table).  See include/sem_hip.h
        sem_set_geom_mode.  "reference": stored factors from x_phys computed
        on the host exactly as the reference does it (LU solves of V_eq,
        Mapping._compute_x_phys, sem/mapping.py:98-103), so that above p = 10
        the action carries the reference's own float64 rounding of that
        ill-conditioned transform; setup only, quadrilaterals.
    kernel : {"auto", "column", "mfma"}
        Kernel family of the Poisson action: the LDS column kernel or the
        fp64 matrix-core element kernel (p <= 15); "auto" (default) resolves
        to the library's measured choice (the column kernel: on its seam
        plan it is ahead of mfma at every order).  See include/sem_hip.h
        sem_set_kernel.
    node_state : array-like uint8 [n_node], optional
        For operators that share the output vector with others applied
        before / after it in stream order: NODE_PRIOR marks nodes whose y
        entry already holds a value (added to, never zeroed), NODE_OTHER
        nodes another operator writes (left alone).  See
        include/sem_hip.h sem_set_map_shared.
    """

    GEOMETRY_MODES = {"stored": _lib.GEOM_STORED, "nodal": _lib.GEOM_NODAL,
                      "auto": _lib.GEOM_AUTO, "reference": _lib.GEOM_STORED}
    KERNELS = {"column": _lib.KERNEL_COLUMN, "mfma": _lib.KERNEL_MFMA, "auto": _lib.KERNEL_AUTO}

    def __init__(self, p, e2n, nodes, dofs_per_node=1, basis=None, device=None,
                 geometry="auto", node_state=None, kernel="auto"):
        if geometry not in self.GEOMETRY_MODES:
            raise ValueError("geometry must be one of %s" % sorted(self.GEOMETRY_MODES))
        if kernel not in self.KERNELS:
            raise ValueError("kernel must be one of %s" % sorted(self.KERNELS))
        self.geometry = geometry
        self.kernel = kernel
        self._shared = node_state is not None
        self._user_geom = False
        self._solver = None  # (operator in the solver numbering | None, order, inverse)
        self._lib = _lib.load()
        self.p = int(p)
        self.n = self.p + 1
        self.dpn = int(dofs_per_node)
        dev = _device_index(device)
        self.device = torch.device("cuda", dev)
        e2n_t = self._to_map(e2n)
        self.ndim = e2n_t.dim() - 1
        if self.ndim not in (2, 3) or tuple(e2n_t.shape[1:]) != (self.n,) * self.ndim:
            raise ValueError("e2n must have shape [E, %d, %d] or [E, %d, %d, %d]"
                             % ((self.n,) * 5))
        if self.ndim == 3 and (self.dpn != 1 or node_state is not None or
                               geometry in ("nodal", "reference") or kernel == "mfma"):
            raise NotImplementedError("hexahedral operators: Poisson (dofs_per_node = 1), "
                                      "stored geometry, column kernel, no node states")
        self.basis, self.D, self.w, self.Vinv = _basis_arrays(self.p, basis, self.ndim)
        nodes_t = torch.as_tensor(nodes, dtype=torch.float64)
        if nodes_t.dim() != 2 or nodes_t.shape[0] != self.ndim:
            raise ValueError("nodes must have shape [%d, n_node]" % self.ndim)
        self.n_elem = int(e2n_t.shape[0])
        self.n_node = int(nodes_t.shape[1])
        self.ndof = self.dpn * self.n_node
        with torch.cuda.device(self.device):
            self.e2n = e2n_t.to(self.device).contiguous()
            self.nodes = nodes_t.to(self.device).contiguous()
            ctx = C.c_void_p()
            _lib.check(self._lib.sem_ctx_create_nd(C.byref(ctx), self.ndim, self.p, self.n_elem,
                                                   self.n_node, self.dpn, dev))
            self._ctx = ctx
            _lib.check(self._lib.sem_set_geom_mode(ctx, self.GEOMETRY_MODES[geometry]))
            if kernel != "auto":
                _lib.check(self._lib.sem_set_kernel(ctx, self.KERNELS[kernel]))
            _lib.check(self._lib.sem_set_basis(ctx, _lib.dptr(self.D), _lib.dptr(self.w)))
            if node_state is None:
                _lib.check(self._lib.sem_set_map(ctx, _lib.tptr(self.e2n), _lib.stream_ptr()))
            else:
                st = torch.as_tensor(np.asarray(node_state, dtype=np.uint8))
                if st.shape != (self.n_node,):
                    raise ValueError("node_state must have shape [n_node]")
                st = st.to(self.device)
                _lib.check(self._lib.sem_set_map_shared(ctx, _lib.tptr(self.e2n), _lib.tptr(st),
                                                        _lib.stream_ptr()))
        self._geom_ready = set()

    @staticmethod
    def _to_map(e2n):
        if isinstance(e2n, torch.Tensor):
            if e2n.dtype == torch.int32:
                return e2n
            if e2n.dtype == torch.uint32:
                return e2n.view(torch.int32)
            e2n = e2n.cpu().numpy()
        a = np.ascontiguousarray(e2n)
        if a.dtype != np.uint32:
            if a.size and (a.min() < 0 or a.max() >= 2 ** 32):
                raise ValueError("element map entries must fit uint32")
            a = a.astype(np.uint32)
        return torch.from_numpy(a.view(np.int32))

    # ------------------------------------------------------------------
    def close(self):
        if getattr(self, "_solver", None) and self._solver[0] is not None:
            self._solver[0].close()
        self._solver = None
        if getattr(self, "_ctx", None):
            self._lib.sem_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, stream):
        return _lib.stream_ptr(stream)

    def plan_info(self):
        """Setup plan of the scatter (see include/sem_hip.h sem_plan_info)."""
        info = (C.c_int64 * 27)()
        _lib.check(self._lib.sem_plan_info(self._ctx, info, 27))
        v = list(info)
        if self.ndim == 3:
            return dict(ndim=3, workgroups=v[0], zero_list=v[1], conforming=bool(v[3]),
                        slots_per_workgroup=v[4], chains=v[5], chain_length_cap=v[6],
                        positions=v[7], subchains=v[8], seam_nodes=v[9], slotted_writes=v[10],
                        plain_stores=v[11], threads=v[12], geometry="stored",
                        kernel="column", plan="chains-seams",
                        hex_kernel="rows" if v[15] else "three_block", zmerge=bool(v[16]),
                        ymerge=bool(v[17]), template_map=bool(v[18]),
                        slot_grid=(v[4] // v[17], v[17]) if v[17] else (1, v[4]))
        counts = [x for x in v[8:8 + v[5]]]
        while counts and counts[-1] == 0:
            counts.pop()
        return dict(groups=v[0], zero_list=v[1], atomic_groups=v[2], conforming=bool(v[3]),
                    elements_per_group=v[4], colours=len(counts), rounds=v[6], slots=v[7],
                    chains_per_colour=counts,
                    kernel="mfma" if v[17] == _lib.KERNEL_MFMA else "column",
                    map_entry_bytes=v[18],
                    geometry="nodal" if v[19] == _lib.GEOM_NODAL else "stored",
                    plan={0: "chains", 1: "element-coloured", 2: "element",
                          4: "chains-seams", 5: "element-seams"}[v[20]],
                    geometry_axisym=(None if self.dpn != 2 else
                                     "nodal" if v[21] == _lib.GEOM_NODAL else "stored"),
                    seam_nodes=v[22] if v[20] in (4, 5) else 0, blocks=bool(v[23]),
                    row_carries=v[24], const_d=bool(v[25]), map_patterns=v[26])

    # ------------------------------------------------------------------
    def compute_geometry(self, kind=POISSON, stream=None):
        """Per-node geometric factors for ``kind`` from the mesh nodes
        (Mapping: sem/mapping.py:98-119; detJxW: sem/discrete.py:594-597).
        Raises AssertionError when detJ <= 0 anywhere (sem/mapping.py:117)."""
        kind = op_kind(kind)
        bad = C.c_int64(0)
        with torch.cuda.device(self.device):
            if self.geometry == "reference":
                xp = torch.from_numpy(reference_x_phys(self.nodes.cpu().numpy(),
                                                       self.e2n.cpu().numpy().view(np.uint32),
                                                       self.basis)).to(self.device)
                _lib.check(self._lib.sem_geom_from_xphys(self._ctx, _lib.tptr(xp), kind,
                                                         C.byref(bad), self._stream(stream)))
                torch.cuda.current_stream().synchronize()
            else:
                _lib.check(self._lib.sem_geom_from_nodes(self._ctx, _lib.tptr(self.nodes),
                                                         _lib.dptr(self.Vinv), kind, C.byref(bad),
                                                         self._stream(stream)))
        self._geom_ready.add(_geom_key(kind))
        return self

    def set_geometry(self, G, kind=POISSON, stream=None):
        """Install user factors [E, ncomp, n, n] (hexahedra: [E, 6, n, n, n],
        components 00, 01, 02, 11, 12, 22) (device or host)."""
        kind = op_kind(kind)
        ncomp = self._lib.sem_op_ncomp(kind) if self.ndim == 2 else 6
        G = torch.as_tensor(G, dtype=torch.float64).to(self.device).contiguous()
        shape = (self.n_elem, ncomp) + (self.n,) * self.ndim
        if tuple(G.shape) != shape:
            raise ValueError("G must have shape %s" % (list(shape),))
        with torch.cuda.device(self.device):
            _lib.check(self._lib.sem_set_geom(self._ctx, _lib.tptr(G), kind, self._stream(stream)))
            torch.cuda.current_stream().synchronize()
        self._geom_ready.add(_geom_key(kind))
        self._user_geom = True
        if self._solver is not None and self._solver[0] is not None:
            self._solver[0].close()
        self._solver = None
        return self

    def geometry_fields(self, stream=None):
        """Reference-layout x_phys [E,2,n,n], J/invJ [E,2,2,n,n],
        detJ/detJxW [E,n,n] as device tensors (FiniteElement properties,
        sem/discrete.py:582-597)."""
        E, d = self.n_elem, self.ndim
        loc = (self.n,) * d
        kw = dict(dtype=torch.float64, device=self.device)
        out = dict(x_phys=torch.empty(E, d, *loc, **kw), J=torch.empty(E, d, d, *loc, **kw),
                   invJ=torch.empty(E, d, d, *loc, **kw), detJ=torch.empty(E, *loc, **kw),
                   detJxW=torch.empty(E, *loc, **kw))
        with torch.cuda.device(self.device):
            _lib.check(self._lib.sem_geom_fields(
                self._ctx, _lib.tptr(self.nodes), _lib.dptr(self.Vinv), _lib.tptr(out["x_phys"]),
                _lib.tptr(out["J"]), _lib.tptr(out["invJ"]), _lib.tptr(out["detJ"]),
                _lib.tptr(out["detJxW"]), self._stream(stream)))
        return out

    # ------------------------------------------------------------------
    def _vec(self, v, name):
        if not isinstance(v, torch.Tensor):
            v = torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64))
        if v.dtype != torch.float64:
            raise TypeError("%s must be float64" % name)
        if v.device != self.device:
            v = v.to(self.device)
        if not v.is_contiguous():
            v = v.contiguous()
        if v.numel() != self.ndof:
            raise ValueError("%s has %d entries, expected ndof = %d" % (name, v.numel(), self.ndof))
        return v

    def set_reynolds(self, re):
        """Reynolds number of the Navier-Stokes kinds (squirmer n_rey)."""
        _lib.check(self._lib.sem_set_reynolds(self._ctx, float(re)))
        return self

    def apply(self, u, out=None, kind=POISSON, accumulate=False, stream=None, linearize=False,
              renumber=False):
        """out (=|+=) K u for all elements in one launch (device tensors).
        kind "axisym_ns": the Re > 0 residual at the state u = (psi, omega);
        with linearize=True the Newton linearisation at u is recorded for
        kind "axisym_ns_jvp" (Jacobian times the direction u).  renumber
        (Poisson, "auto" / True): run the action on the solver numbering's
        context, u gathered in and out gathered back (sem_gather, 2 x 20 B
        per DOF; see row_lines)."""
        kind = op_kind(kind)
        solver = self._solver_numbering(renumber) if (renumber and kind == POISSON) else None
        if solver is not None:
            if accumulate or linearize:
                raise NotImplementedError("apply(renumber=...) with accumulate / linearize")
            op, order, inv = solver
            is_np = not isinstance(u, torch.Tensor)
            u = self._vec(u, "u")
            out = torch.empty_like(u) if out is None else out
            if getattr(self, "_rn_buf", None) is None:
                self._rn_buf = (torch.empty_like(u), torch.empty_like(u))
            ui, yi = self._rn_buf
            with torch.cuda.device(self.device):
                self._gather(u, order, stream, out=ui)
                op.apply(ui, out=yi, stream=stream)
                self._gather(yi, inv, stream, out=out)
            return out.cpu().numpy() if is_np else out
        if _geom_key(kind) not in self._geom_ready:
            self.compute_geometry(kind, stream=stream)
        is_np = not isinstance(u, torch.Tensor)
        u = self._vec(u, "u")
        if out is None:
            out = torch.empty_like(u)
            accumulate = False
        elif not (isinstance(out, torch.Tensor) and out.dtype == torch.float64
                  and out.device == self.device and out.is_contiguous()
                  and out.numel() == self.ndof):
            raise TypeError("out must be a contiguous float64 tensor of %d entries on %s"
                            % (self.ndof, self.device))
        if out.data_ptr() == u.data_ptr():
            raise ValueError("apply: out must not alias u (the kernels read u while writing out)")
        with torch.cuda.device(self.device):
            flags = (_lib.APPLY_ACCUMULATE if accumulate else 0) | \
                (_lib.APPLY_LINEARIZE if linearize else 0)
            _lib.check(self._lib.sem_apply(self._ctx, kind, _lib.tptr(u), _lib.tptr(out), flags,
                                           self._stream(stream)))
        if is_np:
            return out.cpu().numpy()
        return out

    def apply_dot(self, u, out=None, stream=None):
        """(K u, u . K u) for the Poisson operator (sem_apply_dot): on the
        seam plan the dot is summed inside the action's own launches (what
        the device PCG uses for p . q).  Returns (out, 0-d device tensor)."""
        if _geom_key(POISSON) not in self._geom_ready:
            self.compute_geometry(POISSON, stream=stream)
        u = self._vec(u, "u")
        if out is None:
            out = torch.empty_like(u)
        dot = torch.empty((), dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self._lib.sem_apply_dot(self._ctx, POISSON, _lib.tptr(u), _lib.tptr(out),
                                               _lib.tptr(dot), self._stream(stream)))
        return out, dot

    def assemble(self, elem_vals, out=None, accumulate=False, stream=None):
        """Sum element-local nodal values [E, n, n] through the element map
        into a global vector (sem_assemble): the reference's RHS assembly
        grhs[inds] += lrhs (examples/poisson.py:219-243), e.g. the f = 1 load
        vector from geometry_fields()["detJxW"]."""
        if self.dpn != 1:
            raise NotImplementedError("assemble: dofs_per_node == 1")
        v = torch.as_tensor(elem_vals, dtype=torch.float64).to(self.device).contiguous()
        shape = (self.n_elem,) + (self.n,) * self.ndim
        if tuple(v.shape) != shape:
            raise ValueError("element values must have shape %s" % (list(shape),))
        if out is None:
            out = torch.empty(self.ndof, dtype=torch.float64, device=self.device)
            accumulate = False
        with torch.cuda.device(self.device):
            _lib.check(self._lib.sem_assemble(self._ctx, _lib.tptr(v), _lib.tptr(out),
                                              1 if accumulate else 0, self._stream(stream)))
        return out

    def diag(self, kind=POISSON, stream=None):
        kind = op_kind(kind)
        if _geom_key(kind) not in self._geom_ready:
            self.compute_geometry(kind, stream=stream)
        d = torch.empty(self.ndof, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self._lib.sem_diag(self._ctx, kind, _lib.tptr(d), self._stream(stream)))
        return d

    # ------------------------------------------------------------------
    # Solver numbering.  The column kernel's gathers and stores are fast when
    # the 7-9 elements of a wavefront read each node row from a few 64-byte
    # lines (57 consecutive ids at p = 8 on a lexicographic mesh).  The
    # reference's default numbering (DOFManager rcm_order=True) spreads a row
    # over ~17 lines and the action runs at 0.64x (profiles/r05/rcm/).  A
    # solve keeps its vectors for hundreds of actions, so pcg_solve may run on
    # a second context whose nodes are numbered in the kernel's own traversal
    # order, permuting rhs / x / mask once on entry and x once on exit
    # (sem_gather).  A single apply() would pay two permutations (2 x 20 B
    # per DOF) for a 0.36x gain and stays on the caller's numbering.
    def row_lines(self, e2n=None):
        """Mean count of 64-byte lines one wavefront row gather touches (the
        plan's groups of consecutive elements, lanes = (element, column))."""
        m = (self.e2n.cpu().numpy().view(np.uint32) if e2n is None else e2n).astype(np.int64)
        epw = max(1, self.plan_info().get("elements_per_group", 1))
        E = m.shape[0] // epw * epw
        if E == 0:
            return 0.0
        g = m[:E].reshape(-1, epw, self.n, self.n)
        tot = 0
        for r in range(self.n):
            x = np.sort(g[:, :, r, :].reshape(g.shape[0], -1) * self.dpn // 8, axis=1)
            tot += int((np.diff(x, axis=1) != 0).sum()) + x.shape[0]
        return tot / (g.shape[0] * self.n)

    def traversal_order(self):
        """Node numbering in the column kernel's traversal order: first touch
        over (group of consecutive elements, row, lane).  Returns order
        (order[k] = caller node of solver node k) and its inverse."""
        m = self.e2n.cpu().numpy().view(np.uint32).astype(np.int64)
        epw = max(1, self.plan_info().get("elements_per_group", 1))
        E = m.shape[0]
        G = -(-E // epw)
        g = np.full((G * epw, self.n, self.n), -1, dtype=np.int64)
        g[:E] = m
        seq = g.reshape(G, epw, self.n, self.n).transpose(0, 2, 1, 3).reshape(-1)
        seq = seq[seq >= 0]
        _, first = np.unique(seq, return_index=True)
        touched = seq[np.sort(first)]
        rest = np.setdiff1d(np.arange(self.n_node), touched, assume_unique=True)
        order = np.concatenate([touched, rest])
        inv = np.empty(self.n_node, dtype=np.int64)
        inv[order] = np.arange(self.n_node)
        return order, inv

    def _solver_numbering(self, renumber):
        """(operator in the traversal numbering, order, inverse) as device
        uint32 index tensors, or None when the caller's numbering is kept."""
        force = renumber is True or renumber == "on"
        if renumber is False or renumber == "off":
            return None
        if not (self.ndim == 2 and self.dpn == 1 and not self._shared and not self._user_geom):
            if force:
                raise NotImplementedError("solver renumbering: 2-D Poisson operators with "
                                          "library geometry and no node states")
            return None
        if self._solver is None:
            order, inv = self.traversal_order()
            m = self.e2n.cpu().numpy().view(np.uint32).astype(np.int64)
            self.solver_gain = self.row_lines(m) / max(self.row_lines(inv[m]), 1e-9)
            self._solver = (None, order, inv)
        op, order, inv = self._solver
        if op is None:
            if self.solver_gain < 1.3 and not force:
                return None
            m = self.e2n.cpu().numpy().view(np.uint32).astype(np.int64)
            op = SEMOperator(self.p, inv[m].astype(np.uint32), self.nodes.cpu().numpy()[:, order],
                             basis=self.basis, device=self.device, geometry=self.geometry,
                             kernel=self.kernel)
            self._solver = (op, torch.from_numpy(order.astype(np.uint32)).to(self.device),
                            torch.from_numpy(inv.astype(np.uint32)).to(self.device))
        return self._solver

    def _gather(self, src, idx, stream, out=None):
        """out[k] = src[idx[k]] (sem_gather)."""
        out = torch.empty_like(src) if out is None else out
        _lib.check(self._lib.sem_gather(_lib.tptr(src), _lib.tptr(idx), src.numel(),
                                        _lib.tptr(out), self._stream(stream)))
        return out

    def pcg_solve(self, rhs, x, dirichlet, rtol=1e-13, max_iter=20000, kind=POISSON,
                  stream=None, renumber="auto"):
        """Solve K x = rhs on the free DOFs (``dirichlet`` True => x fixed)
        with Jacobi-preconditioned CG on the device (sem_pcg_solve: every
        scalar stays on the device, convergence read every 16 iterations;
        rtol = 0 runs exactly max_iter iterations).  ``x`` (device tensor) is
        updated in place and returned with (iterations executed, relative
        residual).  Raises ValueError when not converged.  renumber: "auto"
        solves in the kernel's traversal numbering when the caller's
        numbering reads >= 1.3x the 64-byte lines per row (row_lines; e.g.
        the reference's RCM default), True forces it, False never."""
        kind = op_kind(kind)
        solver = self._solver_numbering(renumber) if kind == POISSON else None
        if solver is not None:
            op, order, inv = solver
            rhs = self._vec(rhs, "rhs")
            if not isinstance(x, torch.Tensor) or x.device != self.device:
                raise TypeError("x must be a device tensor on %s" % self.device)
            x = self._vec(x, "x")
            mask = torch.as_tensor(dirichlet, dtype=torch.float64).to(self.device)
            if mask.numel() != self.ndof:
                raise ValueError("dirichlet mask must have ndof entries")
            with torch.cuda.device(self.device):
                xi = self._gather(x, order, stream)
                _, its, rel = op.pcg_solve(self._gather(rhs, order, stream), xi,
                                           self._gather(mask, order, stream) != 0, rtol=rtol,
                                           max_iter=max_iter, kind=kind, stream=stream,
                                           renumber=False)
                self._gather(xi, inv, stream, out=x)
            return x, its, rel
        if _geom_key(kind) not in self._geom_ready:
            self.compute_geometry(kind, stream=stream)
        rhs = self._vec(rhs, "rhs")
        if not isinstance(x, torch.Tensor) or x.device != self.device:
            raise TypeError("x must be a device tensor on %s" % self.device)
        x = self._vec(x, "x")
        mask = torch.as_tensor(dirichlet, dtype=torch.bool).to(self.device).to(torch.uint8)
        if mask.numel() != self.ndof:
            raise ValueError("dirichlet mask must have ndof entries")
        its = C.c_int(0)
        rel = C.c_double(0.0)
        with torch.cuda.device(self.device):
            _lib.check(self._lib.sem_pcg_solve(self._ctx, kind, _lib.tptr(rhs), _lib.tptr(x),
                                               _lib.tptr(mask), float(rtol), int(max_iter),
                                               C.byref(its), C.byref(rel), self._stream(stream)))
        return x, its.value, rel.value
