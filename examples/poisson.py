#!/usr/bin/env python
r"""Poisson's equation on a square, restated on this package's facade.

Restates examples/poisson.py of the reference (:62-259) with the current
API names: Dirichlet u = 0.2((x+1) + (y+1)) on the left and bottom edges,
homogeneous Neumann on the top and right, right-hand side f = 1:

    -lap u = 1    (weak form: K u = M 1, K_e = Lse, f_e = JxW)

The driver is the reference's own sequence -- per-element operators from
FiniteElement geometry (Lse, fe = JxW; :143-203), local systems reordered
to the hierarchical DOF order, the static-condensation assembly and solve of
DOFManagerSC (:205-256, sem/discrete.py:404-528) -- so it exercises the
reference-shaped API; the element Schur complements, the condensed solve
and the interior back-solve run on the GPU.  ``solve_matrix_free`` gets the
same solution from the matrix-free device operator alone (no element
matrices), the engine's fast path.

    python examples/poisson.py [--msh meshes/square.msh] [--p 4 --nex 8 --ney 8 --warp 0]

(the reference's meshes/square.geo needs Gmsh, absent here: without --msh a
structured square of the same kind is generated, as in the golden fixtures)
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from spectralelementmethod_amd import meshgen  # noqa: E402
from spectralelementmethod_amd.basis_functions import gll_basis_2d  # noqa: E402
from spectralelementmethod_amd.discrete import DOFManagerSC, Mesh  # noqa: E402


class SolverFailure(Exception):
    """Failure to converge to a solution (examples/poisson.py:38-41)."""


def element_laplacian(fe):
    """Lse and fe = JxW of one element (examples/poisson.py:152-203)."""
    D = fe.basis.get_D1_matrices()
    invJ = fe.invJ
    gradh_xi0 = np.einsum("mp,imn->imnp", D[0], invJ[0, ...])
    gradh_xi1 = np.einsum("nq,imn->imnq", D[1], invJ[1, ...])
    JxW = fe.detJxW
    n = JxW.shape[0]
    Lse = np.zeros((n, n, n, n))
    p, q, r = np.ogrid[[slice(n)] * 3]
    Lse[p, q, r, q] += np.einsum("mn,imnp,imnr->pnr", JxW, gradh_xi0, gradh_xi0)
    Lse += np.einsum("mn,imnp,imns->pnms", JxW, gradh_xi0, gradh_xi1)
    Lse += np.einsum("mn,imnq,imnr->mqrn", JxW, gradh_xi1, gradh_xi0)
    Lse[p, q, p, r] += np.einsum("mn,imnq,imns->mqs", JxW, gradh_xi1, gradh_xi1)
    return Lse, JxW


class PoissonPlate(object):
    """Poisson's equation on a 2D plate (examples/poisson.py:62-259)."""

    def __init__(self, mesh, p):
        self.mesh = mesh
        self.dm = DOFManagerSC(mesh, 1, gll_basis_2d(p))   # RCM + SC node order
        self.soln_vec = np.zeros(self.dm.ndof)
        self.operators = None

    def run(self):
        self.set_boundary_conditions()
        self.compute_operators()
        self.solve()
        return self.soln_vec

    def set_boundary_conditions(self):
        """Essential BCs on the left and bottom edges (:124-141)."""
        x, y = self.mesh.nodes
        on = (np.abs(x + 1) < 1e-12) | (np.abs(y + 1) < 1e-12)
        self.on_ebc_node = on
        self.soln_vec[on] = 0.2 * ((x[on] + 1) + (y[on] + 1))
        # EBC nodes lie on element boundaries, i.e. among the exterior DOFs
        assert not on[self.dm.ndof_exterior:].any()
        self.gdof_mask = ~on[:self.dm.ndof_exterior]

    def compute_operators(self):
        """Local operators of every element (:143-203)."""
        self.operators = [element_laplacian(fe)
                          for fe in self.dm.finite_elements(x_phys=True, Jacobian=True)]

    def solve(self):
        """Static-condensation solve (:205-256)."""
        dm = self.dm
        local_systems = []
        for fe, (Lse, fe_rhs) in zip(dm.finite_elements(), self.operators):
            n_ldof = fe.n_nodes
            loc = (Lse.reshape(n_ldof, n_ldof), fe_rhs.reshape(n_ldof).copy())
            local_systems.append(dm.reorder_local_system_hier(fe, loc))
        gsys = dm.init_global_linear_system()
        dm.assemble_global_sc_system(gsys, local_systems)
        dm.solve(gsys, local_systems, self.soln_vec, ~self.gdof_mask)
        if not np.all(np.isfinite(self.soln_vec)):
            raise SolverFailure("non-finite solution")
        return self.soln_vec

    def solve_matrix_free(self, rtol=1e-13):
        """The same solution from the matrix-free device operator: rhs =
        assembled JxW (f = 1), Jacobi-PCG (DOFManagerSC.solve_poisson)."""
        op = self.dm.operator()
        rhs = op.assemble(op.geometry_fields()["detJxW"]).cpu().numpy()
        dof = np.where(self.on_ebc_node, self.soln_vec, 0.0)
        dof, its, rel = self.dm.solve_poisson(rhs, dof, self.on_ebc_node, rtol=rtol)
        return dof


def square_mesh(p, nex, ney, warp=0.0):
    nodes, e2n = meshgen.structured_square(nex, ney, p, warp)
    return Mesh.from_arrays(nodes, e2n)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--msh", default=None, help="Gmsh 2.2 mesh (region 'interior')")
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--nex", type=int, default=8)
    ap.add_argument("--ney", type=int, default=8)
    ap.add_argument("--warp", type=float, default=0.0)
    args = ap.parse_args(argv)
    if args.msh:
        from spectralelementmethod_amd import grid_importers
        mesh = grid_importers.load_msh(args.msh, 2)
        p = mesh.element_map().shape[1] - 1
    else:
        mesh, p = square_mesh(args.p, args.nex, args.ney, args.warp), args.p
    plate = PoissonPlate(mesh, p)
    u = plate.run()
    u_mf = plate.solve_matrix_free()
    print("ndof %d (exterior %d): |u| = %.16g, max u = %.16g; matrix-free PCG rel. diff %.2e" % (
        u.size, plate.dm.ndof_exterior, np.linalg.norm(u), u.max(),
        np.linalg.norm(u - u_mf) / np.linalg.norm(u)))
    return u


if __name__ == "__main__":
    main()
