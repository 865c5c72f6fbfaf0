/*
 * sem_hip.h -- C ABI of the MI355X spectral-element operator engine
 * (libsem_hip.so, built from spectralelementmethod_amd/csrc/).
 *
 * The reference (nchisholm/SpectralElementMethod) has no FFI: its hot path is
 * Python/NumPy classes.  Each entry point below replaces one piece of that
 * path; the reference interface it stands in for is cited per function
 * (paths relative to the reference checkout).  INTEGRATION.md shows the
 * ctypes binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - n = p + 1 GLL nodes per direction; element-local nodal arrays are
 *     [n][n] in lexicographic (xi0, xi1) order, C-contiguous, float64
 *     (sem/basis_functions.py:647, sem/mapping.py:113).
 *   - element->node map: uint32 [n_elem][n][n] (sem/discrete.py:1044).
 *   - DOF index = dpn * node + comp (sem/discrete.py:567-574).
 *   - Pointers named d_* are DEVICE pointers (caller-owned, e.g. PyTorch
 *     tensors); pointers named h_* are host pointers.
 *   - Every int-returning call returns SEM_OK (0) or a negative SEM_E_* code;
 *     sem_last_error() gives a thread-local message.
 *   - Work is enqueued on the caller's stream (hipStream_t passed as void*;
 *     NULL = the legacy default stream).  sem_apply and the vector kernels
 *     allocate nothing and do not synchronise (graph-capturable).
 */
#ifndef SEM_HIP_H
#define SEM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (mapped to the reference's Python exceptions) ---- */
#define SEM_OK 0
#define SEM_E_INVALID (-1)      /* ValueError      (sem/discrete.py:134, sem/basis_functions.py:358) */
#define SEM_E_NOTIMPL (-2)      /* NotImplementedError (sem/basis_functions.py:366-369, sem/mapping.py:110-111) */
#define SEM_E_DETJ (-3)         /* AssertionError detJ > 0 (sem/mapping.py:117) */
#define SEM_E_HIP (-4)          /* HIP runtime failure */
#define SEM_E_STATE (-5)        /* call order violated (e.g. apply before geometry) */

/* ---- operator kinds ---- */
#define SEM_OP_POISSON 0        /* scalar Laplacian Lse, examples/poisson.py:168-193 */
#define SEM_OP_AXISYM_STOKES 1  /* [Lve.w ; E2e.psi - Me.w], squirmer-axisymmetric.py:193-254,278-295 (Re=0) */
#define SEM_OP_AXISYM_NS 2      /* Re > 0 residual [Ae.w.psi + Lve.w ; E2e.psi - Me.w], squirmer:229-297 */
#define SEM_OP_AXISYM_NS_JVP 3  /* its Newton Jacobian (jac_l, squirmer:272-291) times a direction */

/* number of geometric factors per local node for an operator kind (3, 7 or 9) */
int sem_op_ncomp(int op_kind);

const char* sem_last_error(void);
const char* sem_version(void);

/* ------------------------------------------------------------------ */
/* Host-side basis data (C twins of the reference's 1-D basis layer)   */
/* ------------------------------------------------------------------ */

/* GLL nodes, barycentric and quadrature weights for 1 <= p <= 16, unfolded
 * from the stored non-negative half exactly as LagrangeGaussLobatto.__init__
 * (sem/basis_functions.py:349-393).  Orders 1..10 are the reference's
 * basis-data.hdf5 values; 11..16 come from its generator
 * sem/basis_data.py:19-109.  Each output has p+1 entries. */
int sem_gll_table(int p, double* h_nodes, double* h_bary, double* h_quad);

/* First-derivative matrix D1 (n*n, row-major) from nodes and barycentric
 * weights: BarycentricLagrange.__init__ (sem/basis_functions.py:213-219). */
int sem_diff_matrix(int n, const double* h_nodes, const double* h_bary, double* h_D);

/* Lagrange basis evaluated at points: B[i][j] = l_j(x_i) (n_x*n, row-major),
 * BarycentricLagrange.__call__ (sem/basis_functions.py:226-255). */
int sem_lagrange_eval(int n, const double* h_nodes, const double* h_bary,
                      int64_t n_x, const double* h_x, double* h_B);

/* Equispaced interpolation matrix V_eq (= B at linspace(-1,1,n),
 * sem/basis_functions.py:221-224) and its inverse (the lu_solve of
 * TensorProduct.compute_coeffs_grid_eq, sem/basis_functions.py:599-624). */
int sem_interp_eq_matrix(int n, const double* h_nodes, const double* h_bary,
                         double* h_Veq, double* h_Veq_inv);

/* C twins of sem/bary_interp.c:10-36 (legeval) and :39-90
 * (barycentric_lagrange, 2 <= n <= 17 here; the reference's table stops at
 * n = 9).  Interpolating exactly at a node returns the nodal value. */
double sem_legeval(double x, unsigned n);
double sem_barycentric_lagrange(const double* h_f, unsigned n, double x);

/* Node orderings of a cell-node map (host, no device): the reverse
 * Cuthill-McKee renumbering of DOFManager(mesh, rcm_order=True)
 * (sem/discrete.py:169-178 -> scipy.sparse.csgraph.reverse_cuthill_mckee on
 * the graph joining every two nodes of a cell, sem/discrete.py:142-167), run
 * on the cell map itself instead of materialising that graph (5.5e9 entries
 * at 1024^2 cells, p = 8).  h_cells: [n_cells][nloc] node ids.
 *   sem_node_degrees: scipy's degree of each node (row length + 1 for the
 *     diagonal; 0 for a node no cell references);
 *   sem_cuthill_mckee: Cuthill-McKee order (h_order[k] = k-th node) from
 *     h_seeds = argsort(degree) (the caller's sort, so ties follow numpy);
 *     RCM is h_order reversed.  Equal to scipy's on the same graph
 *     (tests/test_order.py). */
int sem_node_degrees(const uint32_t* h_cells, int64_t n_cells, int nloc, int64_t n_node,
                     int32_t* h_degree);
int sem_cuthill_mckee(const uint32_t* h_cells, int64_t n_cells, int nloc, int64_t n_node,
                      const int32_t* h_degree, const int64_t* h_seeds, int64_t* h_order);

/* ------------------------------------------------------------------ */
/* Operator context (one per GPU)                                      */
/* ------------------------------------------------------------------ */
typedef struct sem_ctx sem_ctx;

/* Replaces DOFManager(mesh, dofs_per_node, basis) bookkeeping
 * (sem/discrete.py:81-124) for the batched operator path. */
int sem_ctx_create(sem_ctx** out, int p, int64_t n_elem, int64_t n_node, int dpn, int device);
void sem_ctx_destroy(sem_ctx* ctx);

/* The same for a mesh of dimension ndim: 2 = quadrilaterals (sem_ctx_create),
 * 3 = hexahedra.  The reference's basis layer is N-dimensional
 * (TensorProduct.deriv / gradient, compute_coeffs_grid_eq,
 * sem/basis_functions.py:599-650; TensorQuadratureRule.xweight,
 * sem/quadratures.py:268-275; NCube, sem/geometry.py:32-216); only its 2x2
 * Jacobian inverse stops at 2-D (sem/mapping.py:110-111).  On a hexahedral
 * context (1 <= p <= 16, dpn = 1, Poisson; above p = 10 the equispaced ->
 * GLL transform runs as compensated passes, above p = 12 the action runs the
 * row form of the kernel by default):
 *   - element-local arrays are [n][n][n] in lexicographic (xi0, xi1, xi2)
 *     order, xi2 fastest; the map is uint32 [n_elem][n][n][n];
 *   - sem_geom_from_nodes takes nodes float64 [3][n_node] and stores the 6
 *     factors G_kl = detJxW sum_j invJ[k][j] invJ[l][j] per node;
 *     sem_geom_fields writes x_phys [E][3][n][n][n], J / invJ
 *     [E][3][3][n][n][n] (J[c][d] = d x_c / d xi_d, invJ = J^-1), detJ and
 *     detJxW [E][n][n][n]; sem_set_geom takes [E][6][n][n][n] in the order
 *     (00, 01, 02, 11, 12, 22);
 *   - sem_apply / sem_apply_dot / sem_diag / sem_assemble / sem_zero_shared /
 *     sem_pcg_solve work as on quadrilaterals (stored geometry, column kernel;
 *     SEM_GEOM_NODAL, SEM_KERNEL_MFMA, node states and the axisymmetric kinds
 *     return SEM_E_NOTIMPL);
 *   - sem_plan_info: [0] workgroups, [1] zero list, [2] 0, [3] 1, [4]
 *     element slots per workgroup, [5] chains along xi0, [6] sub-chain length
 *     cap, [7] launch positions, [8] sub-chains, [9] seam nodes, [10] slotted
 *     writes, [11] plain stores, [12] threads per workgroup, [13] 3, [14]
 *     geometry ready, [15] action kernel (1 row form, 0 three-block),
 *     [16] xi2 faces merged in LDS (z-merge), [17] xi1 faces merged in LDS
 *     too (y-merge): slots per row of the workgroup's slot grid, 0 = off,
 *     [18] template map: every element's node ids are its first node's id +
 *     one shared offset block, read as one base per element
 *     (SEM_HEX_TMAP=0 turns it off). */
int sem_ctx_create_nd(sem_ctx** out, int ndim, int p, int64_t n_elem, int64_t n_node, int dpn,
                      int device);

/* Basis of the operator: D (n*n, host) and 1-D quadrature weights w (n,
 * host): TensorProductQS.get_D1_matrices() / quad_rule.weights
 * (sem/basis_functions.py:156-162, sem/quadratures.py:246-252). */
int sem_set_basis(sem_ctx* ctx, const double* h_D, const double* h_w);

/* Element->node map (device, uint32 [n_elem][n][n]): the per-element
 * FiniteElement.node_ind gather/scatter index (sem/discrete.py:658-663,
 * 810-812).  The library keeps a repacked copy (coalesced per wavefront)
 * plus the list of element-boundary nodes; synchronises `stream`. */
int sem_set_map(sem_ctx* ctx, const uint32_t* d_e2n, void* stream);

/* sem_set_map for an operator that shares y with other operators applied in
 * stream order (e.g. partition-interface elements first, interior elements
 * second, so the interface sum can start early -- SURVEY.md §8(e)).
 * d_node_state (device uint8 [n_node], may be NULL):
 *   SEM_NODE_PRIOR  y[node] already holds the earlier operators' sum when this
 *                   one runs: its first touch adds (read-modify-write) and the
 *                   node is never zeroed;
 *   SEM_NODE_OTHER  a later operator writes y[node]: not zeroed here when this
 *                   operator does not reference it. */
#define SEM_NODE_PRIOR 1
#define SEM_NODE_OTHER 2
int sem_set_map_shared(sem_ctx* ctx, const uint32_t* d_e2n, const uint8_t* d_node_state,
                       void* stream);

/* Setup plan of the last sem_set_map (diagnostics): info[0] groups (one
 * wavefront of elements each), [1] zero-list length, [2] groups in
 * atomic-fallback chains, [3] mesh conforming (0/1), [4] elements per group,
 * [5] colour classes, [6] rounds of 4 groups per chain (one workgroup per
 * chain), [7] packed group slots, [8..16] chains per colour class (one launch
 * each; elements for the MFMA kernel), [17] kernel family (SEM_KERNEL_COLUMN
 * or SEM_KERNEL_MFMA), [18] bytes per packed map entry the Poisson column
 * kernel streams (2: 16-bit row offsets, used when every group row spans
 * < 4096 node ids; 4 otherwise; SEM_MAP16=0 in the environment forces 4).
 * [19] the Poisson geometry mode the action uses (SEM_GEOM_NODAL or
 * SEM_GEOM_STORED, AUTO resolved; nodal only once x_phys per node exists).
 * [20] scatter plan: 0 chains of consecutive elements (carry / merge codes),
 * 1 element-coloured chains (chosen when the element order defeats the chain
 * patterns: more than half of the groups would need atomics; SEM_PLAN=1 / 0
 * in the environment forces / forbids it), 2 one element per wavefront
 * (MFMA kernel), 4 the seam plan (Poisson, dofs_per_node == 1; AUTO where a
 * colour launch would be about one generation of resident workgroups or
 * less -- p >= 10, or few chains per colour; SEM_SEAM=1 / 0
 * forces / forbids): all chains in one launch in element order, nodes
 * written by several chains stored per writer colour and summed in colour
 * order by a second launch, bitwise equal to the colour launches; [5] is
 * then 1 and [8] the chain count.  (3 was a retired one-launch plan.)
 * 5: the n = 17 MFMA kernel's seam form (SEM_SEAM=1; measured slower than
 * its colour launches, which stay the default): every element in one launch in breadth-first
 * order, a node of several elements stored per element colour and summed
 * by the seam launch.
 * [21] the axisymmetric Stokes geometry mode (as [19]; 0 when
 * dofs_per_node != 2).  [22] seam nodes of the seam plan.  [23] 1 when the
 * chains use the block layout (structured numberings: a chain is [6]
 * stacked lines of elements, and the node row between two rounds is carried
 * in registers; SEM_BLOCK_ROUNDS=R in the environment forces R rounds, 0
 * turns it off), [24] the packed map entries so carried.
 * [25] 1 when the Poisson column kernels take D as compile-time constants:
 * sem_set_basis found the context's D equal to the baked standard GLL D
 * bit for bit (csrc/deo_const.h; 16-bit maps) at an order where that is
 * measured faster; SEM_CONST_D=0 / 1 in the environment
 * turns it off / on at every order.
 * [26] patterns of the 16-bit map's pattern table (0: one block of entries
 * per group): groups whose entries repeat share one copy and the map stream
 * shrinks to the per-row bases (SEM_MAP_PATTERNS=0 in the environment turns
 * it off; built for p >= 2).
 * Writes min(n_info, 27) values. */
int sem_plan_info(sem_ctx* ctx, int64_t* info, int n_info);

/* How the Poisson action obtains its geometric factors.
 *  SEM_GEOM_AUTO (default): NODAL for p = 1, 2, 4, 5, 8, STORED otherwise
 *    (per-order MI355X sweep at ~10^7 DOF, DESIGN.md §7: STORED wins at
 *    p = 3, 6, 7 and above 8, where the nodal kernel's register demand
 *    halves occupancy).
 *  SEM_GEOM_NODAL: sem_geom_from_nodes keeps x_phys per global node
 *    (16 B/node) and the action re-derives J, det, invJ and detJxW at every
 *    quadrature node from it -- the reference's own order of work, which
 *    recomputes the geometry inside the element loop (sem/discrete.py:189-209,
 *    582-597) -- trading ~600 FLOP for ~1.9 KB of HBM per element at p = 8.
 *  SEM_GEOM_STORED: the 3 factors per quadrature node are precomputed and
 *    streamed (24 B per element node).
 * Takes effect at the next sem_geom_from_nodes; sem_set_geom always installs
 * stored factors.  The axisymmetric Stokes block (SEM_OP_AXISYM_STOKES) reads
 * the same modes: NODAL re-derives its 7 factors per node from x_phys, with
 * rho = x (16 B/node instead of 56 B per element node; AUTO: NODAL,
 * DESIGN.md §4.2); the Navier-Stokes kinds always use stored factors.
 * x_phys per node is one array per context: sem_geom_from_nodes of either
 * kind recomputes it from the nodes it is given. */
#define SEM_GEOM_STORED 0
#define SEM_GEOM_NODAL 1
#define SEM_GEOM_AUTO 2
int sem_set_geom_mode(sem_ctx* ctx, int mode);

/* Kernel family of the Poisson action; takes effect at the next sem_set_map,
 * which plans the scatter for it.
 *  SEM_KERNEL_COLUMN: k_poisson_apply -- a wavefront holds floor(64/n)
 *    elements, each lane one element column; contractions along the lane in
 *    registers (D in even-odd form), transposes through LDS; chains of 4
 *    groups hand shared columns over through LDS; NODAL or STORED geometry.
 *  SEM_KERNEL_MFMA: k_poisson_mfma -- one element per wavefront as 16 x 16
 *    tiles on the fp64 matrix cores (v_mfma_f64_16x16x4_f64, four products
 *    per element with two transposes through a wave-private LDS tile;
 *    block-diagonal packing of 16/n x 16/n elements per tile for n <= 8);
 *    element-level colouring; stored factors, or x_phys per node when
 *    SEM_GEOM_NODAL is requested; n = p + 1 <= 16 and dpn = 1, else
 *    SEM_E_NOTIMPL.
 *  SEM_KERNEL_AUTO (default): COLUMN -- on its seam plan it measured ahead
 *    of MFMA at every order on MI355X; the build knob
 *    SEM_MFMA_MIN_N (default 17: never) restores an MFMA range.
 * The environment variable SEM_KERNEL (0/1/2) sets the initial value. */
#define SEM_KERNEL_COLUMN 0
#define SEM_KERNEL_MFMA 1
#define SEM_KERNEL_AUTO 2
int sem_set_kernel(sem_ctx* ctx, int kernel);

/* Geometry from mesh nodes (device, float64 [2][n_node]) for op_kind:
 * x_phys = V_eq^-1 X V_eq^-T (Mapping._compute_x_phys, sem/mapping.py:98-103),
 * J = gradient(x_phys) (sem/mapping.py:105-114), det/inverse
 * (sem/linalg.py:105-115), detJxW (sem/discrete.py:594-597) and the operator's
 * per-node factors (Poisson 3, axisymmetric 7).  h_Veq_inv is n*n host.
 * Returns SEM_E_DETJ if any detJ <= 0 (count in *n_bad_nodes if non-NULL). */
int sem_geom_from_nodes(sem_ctx* ctx, const double* d_nodes, const double* h_Veq_inv,
                        int op_kind, int64_t* n_bad_nodes, void* stream);

/* Stored factors for op_kind from x_phys given per element (device, float64
 * [n_elem][2][n][n], the FiniteElement.x_phys of each element,
 * sem/discrete.py:582-585): J, det/inverse and detJxW as sem_geom_from_nodes
 * computes them, without the equispaced->GLL transform.  With x_phys from the
 * reference's own LU path (Mapping._compute_x_phys, sem/mapping.py:98-103),
 * the factors carry the reference's float64 rounding of that transform --
 * which dominates the action's error above p = 10.
 * Quadrilaterals; SEM_E_DETJ as sem_geom_from_nodes. */
int sem_geom_from_xphys(sem_ctx* ctx, const double* d_x_phys, int op_kind, int64_t* n_bad_nodes,
                        void* stream);

/* Reference-layout geometry fields for FiniteElement properties
 * (x_phys [E][2][n][n], J and invJ [E][2][2][n][n], detJ and detJxW
 * [E][n][n]; any output may be NULL).  sem/discrete.py:582-597. */
int sem_geom_fields(sem_ctx* ctx, const double* d_nodes, const double* h_Veq_inv,
                    double* d_x_phys, double* d_J, double* d_invJ, double* d_detJ,
                    double* d_detJxW, void* stream);

/* Install precomputed per-node factors (device, [n_elem][ncomp][n][n]). */
int sem_set_geom(sem_ctx* ctx, const double* d_G, int op_kind, void* stream);

/* Global operator action y (=|+=) K u over all elements: the element loop
 * finite_elements() -> einsum('pqrs,rs', Op, u[loc]) -> y[loc] +=
 * (sem/discrete.py:189-209; examples/squirmer-axisymmetric.py:286,293;
 * examples/poisson.py:168-193), matrix-free by sum factorisation.
 * u, y: device float64 of length dpn*n_node.
 * flags: 0 overwrites y (shared entries are zeroed first by a small list
 * kernel); SEM_APPLY_ACCUMULATE adds into y; SEM_APPLY_SKIP_ZERO (overwrite
 * mode only) states that the caller already ran sem_zero_shared on y. */
#define SEM_APPLY_ACCUMULATE 1
#define SEM_APPLY_SKIP_ZERO 2
#define SEM_APPLY_LINEARIZE 4  /* SEM_OP_AXISYM_NS: also record the Newton
                                * linearisation at u for SEM_OP_AXISYM_NS_JVP */
int sem_apply(sem_ctx* ctx, int op_kind, const double* d_u, double* d_y, int flags,
              void* stream);

/* y = K u (overwrite) and *d_dot = u . y (a device double), for the
 * preconditioned CG's p . Kp: on the seam plan of a single-rank Poisson
 * context the dot is summed inside the action's own two launches (each
 * node's final value is stored exactly once: u[gid] * value at that store,
 * per-workgroup partials, one fixed-order sum -- deterministic); on any other
 * plan the action is followed by a separate dot pass.  Same y as sem_apply. */
int sem_apply_dot(sem_ctx* ctx, int op_kind, const double* d_u, double* d_y, double* d_dot,
                  void* stream);

/* Reynolds number N_Re of the SEM_OP_AXISYM_NS residual and its Jacobian
 * (the n_rey scaling of the advection operator Ae, squirmer:230-250).
 * SEM_OP_AXISYM_NS with u = (psi, omega) interleaved gives
 *   y[2k]   = Ae.omega.psi + Lve.omega,   y[2k+1] = E2e.psi - Me.omega
 * (compute_local_system res_l, squirmer:259-297; Ae at quadrature node
 * (m, n) = Re [w_m w_n (d0 psi d1 w - d1 psi d0 w) + (W/rho) w dpsi/dz]).
 * With SEM_APPLY_LINEARIZE it also stores 5 coefficients per element node so
 * that SEM_OP_AXISYM_NS_JVP applies the Jacobian at that state to any
 * direction u -- the matrix-free form of jac_l (squirmer:272-291). */
int sem_set_reynolds(sem_ctx* ctx, double re);

/* Zero the entries of y that the overwrite-mode kernel does not store
 * (element-boundary and unreferenced nodes; all dpn components). */
int sem_zero_shared(sem_ctx* ctx, double* d_y, void* stream);

/* Assembly of element-local nodal values through the element map:
 * out[map[e][i][j]] (+)= vals[e][i][j] (vals device float64 [n_elem][n][n],
 * dpn = 1) -- the reference's global RHS assembly grhs[inds] += lrhs
 * (examples/poisson.py:219-243, sem/discrete.py:478-500), e.g. the load
 * vector of f = 1 from detJxW (sem_geom_fields). */
int sem_assemble(sem_ctx* ctx, const double* d_vals, double* d_out, int accumulate, void* stream);

/* Diagonal of the assembled operator (Jacobi preconditioner for the
 * assembled Poisson solve; diag(Lse) summed through the map). */
int sem_diag(sem_ctx* ctx, int op_kind, double* d_diag, void* stream);

/* Batched tensor-product operator on device arrays [batch][n][n]:
 * out[b][m][q] = sum_{r,s} A0[m][r] A1[q][s] in[b][r][s]; A0/A1 are n*n host
 * matrices, NULL meaning identity.  TensorProduct.deriv / gradient
 * (D(x)I, I(x)D; sem/basis_functions.py:626-650), compute_coeffs_grid_eq
 * (V_eq^-1 (x) V_eq^-1; :599-624), interpolate_on_grid_eq (:539-569). */
int sem_tensor_apply(int n, int64_t batch, const double* h_A0, const double* h_A1,
                     const double* d_in, double* d_out, void* stream);

/* det_inv_2x2 (sem/linalg.py:105-115) over n points: d_mat [2][2][n] ->
 * d_det [n], d_inv [2][2][n]. */
int sem_det_inv_2x2(int64_t n, const double* d_mat, double* d_det, double* d_inv, void* stream);

/* ------------------------------------------------------------------ */
/* Device vector helpers (multi-GPU interface exchange, CG)            */
/* ------------------------------------------------------------------ */
/* dst[i] = src[idx[i]] */
int sem_gather(const double* d_src, const uint32_t* d_idx, int64_t n, double* d_dst, void* stream);
/* dst[i] += src[i] */
int sem_vec_add(double* d_dst, const double* d_src, int64_t n, void* stream);
/* dst[idx[i]] += src[i]  (idx entries unique) */
int sem_scatter_add(double* d_dst, const uint32_t* d_idx, int64_t n, const double* d_src,
                    void* stream);

/* Matrix-free preconditioned CG for K x = b on the free DOFs
 * (mask[i] != 0 => Dirichlet DOF: x[i] fixed, row/col removed), Jacobi
 * preconditioner.  Replaces the assembled solve of DOFManagerSC.solve
 * (sem/discrete.py:502-528; spsolve of the condensed system).  x holds the
 * Dirichlet values and the initial guess on entry.  Device-resident: alpha,
 * beta and the dot products never leave the device; the host reads the
 * residual history once every SEM_PCG_CHECK_EVERY iterations (one small copy
 * + one stream synchronisation), so up to SEM_PCG_CHECK_EVERY - 1 iterations
 * run past the converged one (they only refine x).  *iters = iterations
 * executed, *final_relres = ||r|| / ||r0|| after the last one.
 * SEM_E_INVALID if not converged within max_iter; rtol = 0 runs exactly
 * max_iter iterations (benchmarking) and returns SEM_OK. */
#define SEM_PCG_CHECK_EVERY 16
int sem_pcg_solve(sem_ctx* ctx, int op_kind, const double* d_b, double* d_x,
                  const uint8_t* d_dirichlet, double rtol, int max_iter,
                  int* iters, double* final_relres, void* stream);

/* ------------------------------------------------------------------ */
/* Static condensation (DOFManagerSC, sem/discrete.py:283-528)         */
/* ------------------------------------------------------------------ */
/* Element Schur complements of local systems in hierarchical order
 * (exterior DOFs first; DOFManagerSC.reorder_local_system_hier), all
 * elements in one launch: compute_local_sc_system (sem/discrete.py:428-466)
 *   S_e = A_ee - A_ei A_ii^-1 A_ie,  s_e = b_e - A_ei A_ii^-1 b_i.
 * d_mat [n_elem][nl][nl], d_rhs [n_elem][nl] -> d_sc_mat [n_elem][ne][ne],
 * d_sc_rhs [n_elem][ne]; d_work [n_elem][nl-ne][nl+1] keeps
 * A_ii^-1 [A_ie | b_i] for sem_schur_backsolve.  Gauss-Jordan with partial
 * pivoting, one workgroup per element (nl - ne <= 512).  SEM_E_INVALID
 * (count in *n_singular) when an interior block is singular (a pivot column
 * exactly zero) or holds a NaN or an off-diagonal inf, where the reference's
 * linalg.solve(..., check_finite=False) raises too; non-finite couplings
 * A_ie, A_ei, b_i and infinite diagonal entries of A_ii propagate as they
 * do there (sem/discrete.py:465-468). */
int sem_schur_batched(int64_t n_elem, int nl, int ne, const double* d_mat, const double* d_rhs,
                      double* d_work, double* d_sc_mat, double* d_sc_rhs, int64_t* n_singular,
                      void* stream);
/* Interior DOFs from the exterior ones, x_i = A_ii^-1 (b_i - A_ie x_e)
 * (_solve_interior_dofs, sem/discrete.py:512-524): d_xe [n_elem][ne] ->
 * d_xi [n_elem][nl-ne], from the d_work of sem_schur_batched. */
int sem_schur_backsolve(int64_t n_elem, int nl, int ne, const double* d_work, const double* d_xe,
                        double* d_xi, void* stream);
/* Jacobi-PCG (as sem_pcg_solve) on an assembled symmetric positive definite
 * CSR matrix (device int64 row pointers, int32 columns, float64 values):
 * the condensed exterior system of _solve_boundary_dofs
 * (sem/discrete.py:502-510, a scipy spsolve in the reference). */
int sem_csr_pcg_solve(int64_t n, const int64_t* d_rowptr, const int32_t* d_colind,
                      const double* d_val, const double* d_b, double* d_x,
                      const uint8_t* d_dirichlet, double rtol, int max_iter, int* iters,
                      double* final_relres, int device, void* stream);
/* Direct solve of a general (non-symmetric) square CSR system A x = b by
 * banded LU with partial pivoting: the condensed exterior system of
 * _solve_boundary_dofs when it is not symmetric (the axisymmetric Stokes /
 * Navier-Stokes block; scipy.sparse.linalg.spsolve in the reference,
 * sem/discrete.py:502-511).  kl / ku: lower / upper bandwidth of A as
 * ordered by the caller (reverse Cuthill-McKee, as the reference orders its
 * nodes); any kl (the multipliers are kept in the band, LAPACK's
 * in-place L).  Duplicate entries are summed.  Band storage
 * n (2 kl + ku + 1) doubles, allocated on the stream.  *info = 0 on
 * success, j + 1 when column j has an exactly zero pivot (A singular; x is
 * then not written), as LAPACK gbsv.  Synchronises the stream. */
int sem_band_lu_solve(int64_t n, int kl, int ku, const int64_t* d_rowptr, const int32_t* d_colind,
                      const double* d_val, const double* d_b, double* d_x, int* info,
                      void* stream);

/* ------------------------------------------------------------------ */
/* Domain decomposition across GPUs (one process per GPU)              */
/* ------------------------------------------------------------------ */
/* The reference's element loop (sem/discrete.py:189-209) is serial; its
 * elements are independent except for the scatter-add, so a rank owns a set
 * of elements and sums only the DOFs it shares with other ranks
 * (SURVEY.md §8(e)).  A sem_dd holds two operator contexts of one rank:
 *   iface     the elements touching a shared node, either over the rank's
 *             own numbering (the context holds ndof_local DOFs: it reads u
 *             directly and writes a private rank-sized vector) or over a
 *             COMPACT numbering of their n_iface_dofs DOFs; in both cases
 *             d_iface_dofs[i] = local DOF of compact DOF i (device uint32,
 *             the DOFs interface elements touch);
 *   interior  every other element, over the local numbering (ndof_local
 *             DOFs); NULL when the rank has no interior element.
 * iface is NULL (n_iface_dofs = 0, no peers) on a rank that shares no node;
 * it still takes part in the global dot products.
 * sem_dd_apply enqueues the interface elements on an internal side stream,
 * packs their shared entries and exchanges them with the peers while the
 * interior elements run on the caller's stream; the caller's stream then
 * adds the interface result into y.  Peer k receives/sends
 * h_peer_counts[k] values: d_peer_dofs (device uint32, concatenated over
 * peers) lists the COMPACT DOFs shared with each peer, in an order both
 * sides agree on (e.g. ascending global id).  d_not_owned (device uint8
 * [ndof_local], may be NULL) marks DOFs whose owner is another rank (left out
 * of the global dot products of sem_dd_pcg_solve). */
typedef struct sem_dd sem_dd;
int sem_dd_create(sem_dd** out, sem_ctx* iface, sem_ctx* interior, int64_t ndof_local,
                  const uint32_t* d_iface_dofs, int64_t n_iface_dofs, int n_peers,
                  const int* h_peers, const int64_t* h_peer_counts, const uint32_t* d_peer_dofs,
                  const uint8_t* d_not_owned, int device);
void sem_dd_destroy(sem_dd* dd);

/* Transport, native: an RCCL communicator over all ranks (ncclSend/ncclRecv
 * with each peer inside one group, ncclAllReduce for the dot products, all
 * on the library's streams; xGMI between the GPUs of one node).  Rank 0
 * creates the id with sem_rccl_unique_id and the caller broadcasts its
 * SEM_RCCL_ID_BYTES bytes (e.g. through torch.distributed). */
#define SEM_RCCL_ID_BYTES 128
int sem_rccl_unique_id(void* h_id, int nbytes);
int sem_dd_init_rccl(sem_dd* dd, const void* h_id, int world, int rank);

/* Transport, caller-supplied (tests, other communication libraries): the
 * exchange callback must leave in d_recv[off[k]..off[k+1]) the values peer
 * peers[k] sent from its d_send range, ordered after the work already on
 * `side_stream` and before anything enqueued on it later; the all-reduce
 * callback sums `count` doubles of d_buf over all ranks in place, ordered on
 * `stream`.  Both return 0 on success. */
typedef int (*sem_exchange_fn)(void* user, int n_peers, const int* peers, const int64_t* off,
                               double* d_send, double* d_recv, void* side_stream);
typedef int (*sem_allreduce_fn)(void* user, double* d_buf, int count, void* stream);
int sem_dd_set_transport(sem_dd* dd, sem_exchange_fn exchange, sem_allreduce_fn allreduce,
                         void* user, int world, int rank);

/* Transport, diagnostic loopback: every exchange copies this rank's own send
 * buffer into its receive buffer (one kernel on the side stream, the bytes
 * RCCL's send/recv would move), every all-reduce is the identity, world 1.
 * Times ONE rank of a decomposition alone on one GPU (bench.py --time-rank):
 * the kernels, streams and host enqueue of the real step, values NOT the
 * global action. */
int sem_dd_set_loopback(sem_dd* dd);

/* Transport, timing: RCCL on a one-rank communicator of this process, every
 * exchange a ncclSend / ncclRecv pair per peer addressed to this rank itself
 * inside one group on the side stream (RCCL's own host enqueue, proxy and
 * copy kernels in place of the loopback kernel), all-reduces over one rank.
 * Like sem_dd_set_loopback it times ONE rank of a decomposition alone
 * (bench.py --time-rank --time-rank-transport rccl_self); values NOT the
 * global action.  sem_dd_info [4] = 4. */
int sem_dd_set_rccl_self(sem_dd* dd);

/* hipMemcpyAsync(dst, src, nbytes, hipMemcpyDefault, stream): lets a
 * caller-supplied transport stage the library's device buffers. */
int sem_copy_async(void* dst, const void* src, int64_t nbytes, void* stream);

/* info[0] ndof_local, [1] n_iface_dofs, [2] peers, [3] exchanged values per
 * direction, [4] transport (0 none, 1 RCCL, 2 callbacks, 3 loopback),
 * [5] has interior, [6] captured step on (sem_dd_set_graphs), [7] captures,
 * [8] replays, [9] sem_dd_apply calls, [10] host nanoseconds spent in them,
 * [11] of which inside the transport call (a caller transport that
 * synchronises with the device makes [11] the device time up to the
 * exchange), eager steps only: [12] enqueueing the side-stream part (gather,
 * interface elements, pack), [13] the interior elements, [14] the finish;
 * [15] bit 0: the interior's zero list folded into the finish, bit 1: the
 * interior's seam sum fused with the finish (one launch), bit 2: the
 * interface seam sum fused with the pack, bit 3: the finish split around the
 * join, bit 4: the stream-join events are recorded without the system-scope
 * fence (only the one-device transports, loopback and RCCL to self, unless
 * SEM_DD_EVENT_FENCE=system|device forces a scope).
 * Hexahedral contexts (sem_ctx_create_nd, ndim 3) are accepted for both
 * iface and interior (interface context over the local numbering). */
int sem_dd_info(sem_dd* dd, int64_t* info, int n_info);

/* Captured step (default off; SEM_DD_GRAPH=1 in the environment turns it
 * on): sem_dd_apply and the PCG operator action replay the step's launches
 * as four HIP graphs around the transport call (side stream: gather,
 * interface elements, pack | unpack; caller's stream: interior elements |
 * final add), re-captured when the operator kind or the u / y pointers
 * change.  Same kernels, same order, same results as the eager path; the
 * host enqueues 4 graph launches instead of ~15 kernel launches, which on
 * ROCm 7 costs more host time, not less. */
int sem_dd_set_graphs(sem_dd* dd, int enable);

/* y = K u on this rank's DOFs, shared DOFs summed over all ranks (u, y local
 * device vectors, must not alias). */
int sem_dd_apply(sem_dd* dd, int op_kind, const double* d_u, double* d_y, void* stream);
/* diagonal of the globally assembled operator on this rank's DOFs */
int sem_dd_diag(sem_dd* dd, int op_kind, double* d_diag, void* stream);
/* sem_pcg_solve over the decomposition: global dot products over owned DOFs
 * (one all-reduce per dot), convergence read every check_every iterations. */
int sem_dd_pcg_solve(sem_dd* dd, int op_kind, const double* d_b, double* d_x,
                     const uint8_t* d_dirichlet, double rtol, int max_iter, int check_every,
                     int* iters, double* final_relres, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SEM_HIP_H */
