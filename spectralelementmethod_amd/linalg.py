"""Small dense linear algebra (mirror of sem/linalg.py).

``det_inv_2x2`` (sem/linalg.py:105-115) runs on the GPU through
``sem_det_inv_2x2``; numpy inputs are staged to the device and returned as
numpy.  The stale Schur-complement assembler ``sp_schur_solve``
(sem/linalg.py:9-102) uses attributes that no longer exist in the reference
(SURVEY.md §2 row 4); its live counterpart is DOFManagerSC.solve_poisson.
"""
import numpy as np

from . import _lib


def det_inv_2x2(mat):
    """Determinant and inverse of 2x2 matrices stored as mat[2, 2, ...]."""
    import torch
    is_np = not isinstance(mat, torch.Tensor)
    t = torch.as_tensor(np.asarray(mat, dtype=np.float64) if is_np else mat,
                        dtype=torch.float64)
    if t.shape[:2] != (2, 2):
        raise ValueError("expected an array of shape (2, 2, ...)")
    t = t.cuda().contiguous() if not t.is_cuda else t.contiguous()
    rest = t.shape[2:]
    n = int(np.prod(rest)) if len(rest) else 1
    det = torch.empty(rest, dtype=torch.float64, device=t.device)
    inv = torch.empty_like(t)
    with torch.cuda.device(t.device):
        _lib.check(_lib.load().sem_det_inv_2x2(n, _lib.tptr(t), _lib.tptr(det), _lib.tptr(inv),
                                               _lib.stream_ptr()))
    if is_np:
        return det.cpu().numpy(), inv.cpu().numpy()
    return det, inv


def sp_schur_solve(global_system, local_systems):
    raise NotImplementedError("sem.linalg.sp_schur_solve targets a removed element API; use "
                              "DOFManagerSC.solve_poisson")
