"""ctypes binding of libsem_hip.so (the C ABI declared in include/sem_hip.h).

The library must be built in-tree (``__graft_entry__.build()`` or
``python -m spectralelementmethod_amd._build``).  There is no fallback: if the
library is missing, every operator raises.  ``torch`` is imported first so
that the HIP runtime PyTorch already loaded (soname libamdhip64.so.7) is the
one the library binds to: device pointers and streams are then shared.
"""
import ctypes as C
import os

import torch  # noqa: F401  (must precede the library: shares the HIP runtime)

from ._build import LIB_PATH

SEM_OK = 0
SEM_E_INVALID = -1
SEM_E_NOTIMPL = -2
SEM_E_DETJ = -3
SEM_E_HIP = -4
SEM_E_STATE = -5

OP_POISSON = 0
OP_AXISYM_STOKES = 1
OP_AXISYM_NS = 2
OP_AXISYM_NS_JVP = 3

APPLY_ACCUMULATE = 1
APPLY_SKIP_ZERO = 2
APPLY_LINEARIZE = 4
GEOM_STORED = 0
GEOM_NODAL = 1
GEOM_AUTO = 2
KERNEL_COLUMN = 0
KERNEL_MFMA = 1
KERNEL_AUTO = 2
NODE_PRIOR = 1
NODE_OTHER = 2

# every symbol include/sem_hip.h declares, with (restype, argtypes)
_i64 = C.c_int64
_dp = C.POINTER(C.c_double)
_vp = C.c_void_p
SIGNATURES = {
    "sem_op_ncomp": (C.c_int, [C.c_int]),
    "sem_last_error": (C.c_char_p, []),
    "sem_version": (C.c_char_p, []),
    "sem_gll_table": (C.c_int, [C.c_int, _dp, _dp, _dp]),
    "sem_diff_matrix": (C.c_int, [C.c_int, _dp, _dp, _dp]),
    "sem_lagrange_eval": (C.c_int, [C.c_int, _dp, _dp, _i64, _dp, _dp]),
    "sem_interp_eq_matrix": (C.c_int, [C.c_int, _dp, _dp, _dp, _dp]),
    "sem_legeval": (C.c_double, [C.c_double, C.c_uint]),
    "sem_barycentric_lagrange": (C.c_double, [_dp, C.c_uint, C.c_double]),
    "sem_node_degrees": (C.c_int, [_vp, _i64, C.c_int, _i64, _vp]),
    "sem_cuthill_mckee": (C.c_int, [_vp, _i64, C.c_int, _i64, _vp, _vp, _vp]),
    "sem_ctx_create": (C.c_int, [C.POINTER(_vp), C.c_int, _i64, _i64, C.c_int, C.c_int]),
    "sem_ctx_create_nd": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_int, _i64, _i64, C.c_int,
                                    C.c_int]),
    "sem_ctx_destroy": (None, [_vp]),
    "sem_set_basis": (C.c_int, [_vp, _dp, _dp]),
    "sem_set_map": (C.c_int, [_vp, _vp, _vp]),
    "sem_plan_info": (C.c_int, [_vp, C.POINTER(_i64), C.c_int]),
    "sem_geom_from_nodes": (C.c_int, [_vp, _vp, _dp, C.c_int, C.POINTER(_i64), _vp]),
    "sem_geom_fields": (C.c_int, [_vp, _vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sem_geom_from_xphys": (C.c_int, [_vp, _vp, C.c_int, C.POINTER(_i64), _vp]),
    "sem_set_geom": (C.c_int, [_vp, _vp, C.c_int, _vp]),
    "sem_set_geom_mode": (C.c_int, [_vp, C.c_int]),
    "sem_set_kernel": (C.c_int, [_vp, C.c_int]),
    "sem_set_reynolds": (C.c_int, [_vp, C.c_double]),
    "sem_set_map_shared": (C.c_int, [_vp, _vp, _vp, _vp]),
    "sem_apply": (C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int, _vp]),
    "sem_apply_dot": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp]),
    "sem_zero_shared": (C.c_int, [_vp, _vp, _vp]),
    "sem_vec_add": (C.c_int, [_vp, _vp, _i64, _vp]),
    "sem_diag": (C.c_int, [_vp, C.c_int, _vp, _vp]),
    "sem_assemble": (C.c_int, [_vp, _vp, _vp, C.c_int, _vp]),
    "sem_tensor_apply": (C.c_int, [C.c_int, _i64, _dp, _dp, _vp, _vp, _vp]),
    "sem_det_inv_2x2": (C.c_int, [_i64, _vp, _vp, _vp, _vp]),
    "sem_gather": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "sem_scatter_add": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "sem_pcg_solve": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double, C.c_int,
                                C.POINTER(C.c_int), C.POINTER(C.c_double), _vp]),
    "sem_schur_batched": (C.c_int, [_i64, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp,
                                    C.POINTER(_i64), _vp]),
    "sem_schur_backsolve": (C.c_int, [_i64, C.c_int, C.c_int, _vp, _vp, _vp, _vp]),
    "sem_csr_pcg_solve": (C.c_int, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, C.c_double, C.c_int,
                                    C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_int, _vp]),
    "sem_band_lu_solve": (C.c_int, [_i64, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp,
                                    C.POINTER(C.c_int), _vp]),
    "sem_rccl_unique_id": (C.c_int, [_vp, C.c_int]),
    "sem_copy_async": (C.c_int, [_vp, _vp, _i64, _vp]),
    "sem_dd_create": (C.c_int, [C.POINTER(_vp), _vp, _vp, _i64, _vp, _i64, C.c_int,
                                C.POINTER(C.c_int), C.POINTER(_i64), _vp, _vp, C.c_int]),
    "sem_dd_destroy": (None, [_vp]),
    "sem_dd_init_rccl": (C.c_int, [_vp, _vp, C.c_int, C.c_int]),
    "sem_dd_set_transport": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int, C.c_int]),
    "sem_dd_set_loopback": (C.c_int, [_vp]),
    "sem_dd_set_rccl_self": (C.c_int, [_vp]),
    "sem_dd_info": (C.c_int, [_vp, C.POINTER(_i64), C.c_int]),
    "sem_dd_set_graphs": (C.c_int, [_vp, C.c_int]),
    "sem_dd_apply": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp]),
    "sem_dd_diag": (C.c_int, [_vp, C.c_int, _vp, _vp]),
    "sem_dd_pcg_solve": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double, C.c_int, C.c_int,
                                   C.POINTER(C.c_int), C.POINTER(C.c_double), _vp]),
}

# sem_exchange_fn / sem_allreduce_fn (include/sem_hip.h)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, _vp, C.c_int, C.POINTER(C.c_int), C.POINTER(_i64), _vp, _vp,
                          _vp)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, _vp, _vp, C.c_int, _vp)
RCCL_ID_BYTES = 128
PCG_CHECK_EVERY = 16

_LIB = None


class SemError(RuntimeError):
    """HIP runtime or call-order failure inside libsem_hip.so."""


def load():
    """Load (once) and return the ctypes handle; raises if the .so is absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libsem_hip.so is not built (%s). Run `python -c 'import __graft_entry__ as g; "
            "g.build()'` or `python -m spectralelementmethod_amd._build`." % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def last_error():
    msg = load().sem_last_error()
    return msg.decode() if msg else ""


def check(rc):
    """Map a SEM_E_* code onto the exception type the reference raises."""
    if rc == SEM_OK:
        return
    msg = last_error()
    if rc == SEM_E_INVALID:
        raise ValueError(msg)
    if rc == SEM_E_NOTIMPL:
        raise NotImplementedError(msg)
    if rc == SEM_E_DETJ:
        raise AssertionError(msg)
    raise SemError("sem_hip error %d: %s" % (rc, msg))


def dptr(arr):
    """ctypes double* for a C-contiguous float64 numpy array."""
    return arr.ctypes.data_as(_dp)


def tptr(t):
    """raw device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    """hipStream_t of a torch stream (default: the current stream)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)
