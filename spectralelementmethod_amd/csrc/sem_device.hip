// Device half of libsem_hip.so: the setup planner (map packing, group
// colouring, write codes), the small kernels and the C ABI.  The operator
// kernels are instantiated per order in sem_launch.hip.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "sem_ctx.h"

using sem::fail;
using namespace semk;
using namespace semd;

namespace {

inline int epw_of(int n) { return WAVE / n; }

// user-supplied factors [E][ncomp][n][n] -> packed (element positions epos)
__global__ void k_pack_geom(const double* __restrict__ G, int64_t n_elem, int n, int ncomp,
                            int epw, const int* __restrict__ epos, double* __restrict__ GP) {
  const int64_t nn = (int64_t)n * n;
  const int64_t total = n_elem * ncomp * nn;
  const int lw = epw * n;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / (ncomp * nn);
    const int64_t rem = t - e * ncomp * nn;
    const int c = (int)(rem / nn);
    const int node = (int)(rem - c * nn);
    const int r = node / n, jj = node - r * n;
    const int64_t pos = epos[e];  // packed position slot * epw + lane element
    const int64_t gg = pos / epw;
    const int kk = (int)(pos - gg * epw);
    GP[((gg * ncomp + c) * n + r) * lw + kk * n + jj] = G[t];
  }
}

// u.y over all nodes (the fallback of sem_apply_dot on plans without seams)
__global__ void __launch_bounds__(BLOCK)
    k_dot_plain(const double* __restrict__ u, const double* __restrict__ y, int64_t n,
                double* __restrict__ part) {
  double v = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK)
    v = fma(u[i], y[i], v);
  __shared__ double sh[BLOCK / WAVE];
  const double t = semk::block_sum_fixed<BLOCK / WAVE>(v, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void k_zero_list(double* __restrict__ y, const uint32_t* __restrict__ idx, int64_t n,
                            int dpn) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t base = (int64_t)idx[t] * dpn;
    for (int c = 0; c < dpn; ++c) y[base + c] = 0.0;
  }
}

// diag of the Poisson element operator, summed through the map:
// K_e[pq,pq] = sum_m D[m][p]^2 G00[m][q] + sum_n D[n][q]^2 G11[p][n] + 2 D[p][p] D[q][q] G01[p][q]
__global__ void k_poisson_diag(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                               const int* __restrict__ epos, const double* __restrict__ gD, int n,
                               int epw, int64_t n_elem, double* __restrict__ diag) {
  __shared__ double sD[MAXN * MAXN];
  for (int i = threadIdx.x; i < n * n; i += blockDim.x) sD[i] = gD[i];
  __syncthreads();
  const int lw = epw * n;
  const int64_t total = n_elem * n * n;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / (n * n);
    const int node = (int)(t - e * n * n);
    const int p = node / n, q = node - p * n;
    const int64_t pos = epos[e];  // packed position slot * epw + lane element
    const int64_t gg = pos / epw;
    const int kk = (int)(pos - gg * epw);
    const double* G = GP + gg * (int64_t)(3 * n * lw) + kk * n;
    double s = 0.0;
    for (int m = 0; m < n; ++m) s += sD[m * n + p] * sD[m * n + p] * G[(0 * n + m) * lw + q];
    for (int nn = 0; nn < n; ++nn) s += sD[nn * n + q] * sD[nn * n + q] * G[(2 * n + p) * lw + nn];
    s += 2.0 * sD[p * n + p] * sD[q * n + q] * G[(1 * n + p) * lw + q];
    const uint32_t gi = mapP[(gg * n + p) * lw + kk * n + q] & GID_MASK;
    atomic_add_f64(diag + gi, s);
  }
}

// out[map[e][i][j]] += vals[e][i][j] through the caller's map (setup-time assembly)
__global__ void k_assemble(const uint32_t* __restrict__ e2n, const double* __restrict__ vals,
                           int64_t total, double* __restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x)
    atomic_add_f64(out + e2n[t], vals[t]);
}

__global__ void k_gather(const double* __restrict__ src, const uint32_t* __restrict__ idx,
                         int64_t n, double* __restrict__ dst) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    dst[t] = src[idx[t]];
}

__global__ void k_vec_add(double* __restrict__ dst, const double* __restrict__ src, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    dst[t] += src[t];
}

__global__ void k_scatter_add(double* __restrict__ dst, const uint32_t* __restrict__ idx,
                              int64_t n, const double* __restrict__ src) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    dst[idx[t]] += src[t];
}

// out[b][m][q] = sum_{r,s} A0[m][r] A1[q][s] in[b][r][s]  (A = NULL -> identity)
// TensorProduct.deriv / gradient (D(x)I, I(x)D; sem/basis_functions.py:626-650),
// compute_coeffs_grid_eq (Vinv(x)Vinv; :599-624), interpolate_on_grid_eq (:539-569).
__global__ void k_tensor_apply(int n, int64_t batch, const double* __restrict__ gA0,
                               const double* __restrict__ gA1, const double* __restrict__ in,
                               double* __restrict__ out) {
  __shared__ double sA0[MAXN * MAXN], sA1[MAXN * MAXN];
  __shared__ double tile[MAXN * MAXN];
  const int nn = n * n;
  for (int i = threadIdx.x; i < nn; i += blockDim.x) {
    const int r = i / n, c = i - r * n;
    sA0[i] = gA0 ? gA0[i] : (r == c ? 1.0 : 0.0);
    sA1[i] = gA1 ? gA1[i] : (r == c ? 1.0 : 0.0);
  }
  for (int64_t b = blockIdx.x; b < batch; b += gridDim.x) {
    __syncthreads();
    for (int i = threadIdx.x; i < nn; i += blockDim.x) tile[i] = in[b * nn + i];
    __syncthreads();
    for (int i = threadIdx.x; i < nn; i += blockDim.x) {
      const int m = i / n, q = i - m * n;
      double a = 0.0;
      for (int r = 0; r < n; ++r) {
        double t = 0.0;
        for (int s = 0; s < n; ++s) t = fma(sA1[q * n + s], tile[r * n + s], t);
        a = fma(sA0[m * n + r], t, a);
      }
      out[b * nn + i] = a;
    }
  }
}

// det_inv_2x2 (sem/linalg.py:105-115) over n points: mat [2][2][n] -> det [n], inv [2][2][n]
__global__ void k_det_inv_2x2(int64_t n, const double* __restrict__ M, double* __restrict__ det,
                              double* __restrict__ inv) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const double a = M[t], b = M[n + t], c = M[2 * n + t], d = M[3 * n + t];
    const double dt = a * d - b * c;
    const double r = 1.0 / dt;
    det[t] = dt;
    inv[t] = d * r;
    inv[n + t] = -b * r;
    inv[2 * n + t] = -c * r;
    inv[3 * n + t] = a * r;
  }
}


}  // namespace
namespace sem {
int64_t ctx_ndof(const sem_ctx* c) { return c->n_node * c->dpn; }
int ctx_device(const sem_ctx* c) { return c->device; }
uint64_t ctx_epoch(const sem_ctx* c) { return c->epoch; }
int ctx_dpn(const sem_ctx* c) { return c->dpn; }
uint64_t ctx_map_epoch(const sem_ctx* c) { return c->map_epoch; }
bool ctx_seam_fusable(const sem_ctx* c) {
  // the n = 17 MFMA seam form sums its own seams (launch_apply_n ignores
  // defer_seam_sum there), so it is never fused with the finish
  return c->seam && !c->mfma && c->n_seam > 0 && c->dpn == 1 && c->seam_ns >= 1 &&
         c->seam_ns <= 8;
}
int ctx_seam_gids(const sem_ctx* c, std::vector<uint32_t>* gids) {
  gids->assign((size_t)c->n_seam, 0u);
  if (c->n_seam)
    HIP_TRY(hipMemcpy(gids->data(), c->d_seam_gid, c->n_seam * sizeof(uint32_t),
                      hipMemcpyDeviceToHost));
  return SEM_OK;
}
void ctx_set_defer_seam_sum(sem_ctx* c, bool defer) { c->defer_seam_sum = defer; }
bool ctx_seam_has_prior(const sem_ctx* c) {
  if (!c->n_seam) return false;
  std::vector<uint16_t> m((size_t)c->n_seam);
  if (hipMemcpy(m.data(), c->d_seam_mask, c->n_seam * sizeof(uint16_t), hipMemcpyDeviceToHost) !=
      hipSuccess) {
    (void)hipGetLastError();
    return true;  // unknown: treated as not fusable
  }
  for (uint16_t v : m)
    if (v & 0x100u) return true;
  return false;
}
int ctx_zero_list(const sem_ctx* c, std::vector<uint32_t>* nodes, bool* only_unreferenced) {
  if (c->ndim == 3) return semh::zero_list(c, nodes, only_unreferenced);
  nodes->assign((size_t)c->n_zero, 0u);
  *only_unreferenced = c->n_atomic_groups == 0;
  if (c->n_zero) {
    HIP_TRY(hipMemcpy(nodes->data(), c->d_zero, c->n_zero * sizeof(uint32_t),
                      hipMemcpyDeviceToHost));
  }
  return SEM_OK;
}
}  // namespace sem

namespace semd {
// second launch of the seam plan (k_seam_sum / k_seam_sum2 over the seam
// nodes, one instantiation per colour count)
int seam_ilp_of(const sem_ctx* c) { return c->n == 17 ? SEAM_ILP_17 : SEAM_ILP; }

int64_t seam_sum_blocks(const sem_ctx* c) {
  return c->n_seam ? grid_for(c->n_seam, BLOCK * seam_ilp_of(c)) : 0;
}

int launch_seam_sum(sem_ctx* c, double* y, int acc, hipStream_t st, const double* du,
                    double* dot) {
  if (!c->n_seam) return SEM_OK;
  const dim3 g(c->dpn == 2 ? grid_for(c->n_seam) : (int)seam_sum_blocks(c)), b(BLOCK);
  const bool ilp2 = seam_ilp_of(c) == 2;
  static_assert(SEAM_ILP == 1 || SEAM_ILP == 2, "seam-sum ILP 1 or 2");
  switch (c->seam_ns) {
#define SEAM_NS(K)                                                                           \
  case K:                                                                                  \
    if (c->dpn == 2)                                                                       \
      hipLaunchKernelGGL(k_seam_sum2<K>, g, b, 0, st, y, c->d_seam_gid, c->d_seam_mask,    \
                         c->n_seam, c->d_seam_buf, c->n_node, acc);                        \
    else if (dot && ilp2)                                                                  \
      hipLaunchKernelGGL((k_seam_sum<K, true, 2>), g, b, 0, st, y, c->d_seam_gid,          \
                         c->d_seam_mask, c->n_seam, c->d_seam_buf, c->n_node, acc, du, dot);\
    else if (dot)                                                                          \
      hipLaunchKernelGGL((k_seam_sum<K, true, 1>), g, b, 0, st, y, c->d_seam_gid,          \
                         c->d_seam_mask, c->n_seam, c->d_seam_buf, c->n_node, acc, du, dot);\
    else if (ilp2)                                                                         \
      hipLaunchKernelGGL((k_seam_sum<K, false, 2>), g, b, 0, st, y, c->d_seam_gid,         \
                         c->d_seam_mask, c->n_seam, c->d_seam_buf, c->n_node, acc, nullptr, \
                         nullptr);                                                         \
    else                                                                                   \
      hipLaunchKernelGGL((k_seam_sum<K, false, 1>), g, b, 0, st, y, c->d_seam_gid,         \
                         c->d_seam_mask, c->n_seam, c->d_seam_buf, c->n_node, acc, nullptr, \
                         nullptr);                                                         \
    break;
    SEAM_NS(1) SEAM_NS(2) SEAM_NS(3) SEAM_NS(4) SEAM_NS(5) SEAM_NS(6) SEAM_NS(7) SEAM_NS(8)
#undef SEAM_NS
    default:
      return sem::fail(SEM_E_STATE, "seam plan with more than 8 colours");
  }
  return SEM_OK;
}
}  // namespace semd

namespace {

int check_op(sem_ctx* c, int op_kind) {
  if (op_kind == SEM_OP_POISSON) {
    if (c->dpn != 1) return fail(SEM_E_INVALID, "Poisson operator needs dofs_per_node == 1");
    return SEM_OK;
  }
  if (op_kind == SEM_OP_AXISYM_STOKES || op_kind == SEM_OP_AXISYM_NS ||
      op_kind == SEM_OP_AXISYM_NS_JVP) {
    if (c->dpn != 2)
      return fail(SEM_E_INVALID, "axisymmetric Stokes block needs dofs_per_node == 2");
    return SEM_OK;
  }
  return fail(SEM_E_INVALID, "unknown op_kind " + std::to_string(op_kind));
}

// factor slot of an operator kind: the two Navier-Stokes kinds share one
int gp_slot(int op_kind) {
  return op_kind == SEM_OP_POISSON ? 0 : (op_kind == SEM_OP_AXISYM_STOKES ? 1 : 2);
}

// partial-sum buffer of sem_apply_dot (grown on demand, never shrunk)
int ensure_dot(sem_ctx* c, int64_t n) {
  if (c->d_dot && c->n_dot >= n) return SEM_OK;
  (void)hipFree(c->d_dot);
  c->d_dot = nullptr;
  HIP_TRY(hipMalloc(&c->d_dot, std::max<int64_t>(n, 1) * sizeof(double)));
  c->n_dot = std::max<int64_t>(n, 1);
  return SEM_OK;
}

// The zero fill is ordered on the stream of the kernels that fill the
// buffer: a plain hipMemset of device memory may still be in flight on the
// legacy default stream when a kernel on a non-blocking stream (the
// multi-GPU side stream) writes the factors.
int ensure_gp(sem_ctx* c, int op_kind, hipStream_t st) {
  const int slot = gp_slot(op_kind);
  if (!c->d_GP[slot]) {
    const int ncomp = sem_op_ncomp(op_kind);
    const size_t bytes = (size_t)c->n_slots * ncomp * c->n * c->lw * sizeof(double);
    HIP_TRY(hipMalloc(&c->d_GP[slot], bytes));
    HIP_TRY(hipMemsetAsync(c->d_GP[slot], 0, bytes, st));
  }
  return SEM_OK;
}

// ---------------------------------------------------------------------------
// Setup planner (host, once per map).
//   1. groups = EPW element slots (one wavefront each), chains = CH = 4 *
//      rounds consecutive groups (one workgroup each), from a group table
//      (groups_consecutive / groups_blocks below);
//   2. greedy colouring of chains: chains of one colour share no node
//      (per-node colour bitmask; chains needing > MAX_COLOURS colours, and
//      every chain of a non-conforming mesh, go to a final all-atomic class);
//   3. launch order = colour-major; epos[e] = packed position of element e;
//   4. inside a chain the 4 groups of a round run concurrently, rounds run in
//      order.  A node may be shared inside a round only by (a) the elements on
//      two neighbouring lanes of one group (row r, lanes L, L+1: MERGE on L,
//      SKIP on L+1) or (b) the last lane of group i-1 and lane 0 of group i
//      (row r: SKIP on the former, CARRY on the latter); anything else makes
//      the chain atomic.  Across rounds, (c) row n-1 of a lane's element and
//      row 0 of the same lane's element in the next round (the block layout)
//      is carried in registers: SKIP | CARRY on the former, which is then no
//      writer at all; any other node a chain touches again in a later round
//      is a read-modify-write of its own earlier store;
//   5. write codes in launch order: first writer of a node -> STORE, later
//      writers -> RMW (atomic chains -> ATOMIC);
//   6. zero list = unreferenced nodes + nodes whose first writer is atomic.
// ---------------------------------------------------------------------------
constexpr uint32_t W_ROWCARRY = W_SKIP | W_CARRY;  // sem_kernels.h k_poisson_apply

struct Plan {
  std::vector<uint32_t> owner;  // first element referencing each node
  std::vector<uint32_t> mapP;
  std::vector<int> epos;             // element -> packed position slot * epw + k
  std::vector<uint8_t> slot_fill;    // real elements in each slot (first lanes)
  std::vector<int64_t> colour_start;  // in chains
  std::vector<uint32_t> zero;
  int64_t n_atomic_groups = 0;
  int64_t n_slots = 0;
  bool conforming = true;
  int64_t n_rmw = 0;       // read-modify-write entries (a node's final value elsewhere)
  bool blocks = false;     // block layout (groups_blocks)
  int block_rounds = 0;
  int64_t row_carries = 0;  // entries carried to the next round in registers
  bool round_rmw = true;  // some chain read-modify-writes a node it stored in an earlier round
  // seam plan: chains in element order, one launch; nodes written by several
  // chains go through per-colour slots summed by k_seam_sum
  bool seam = false;
  std::vector<uint8_t> chain_colour;  // [chain] in launch order
  std::vector<uint32_t> seam_gid;
  std::vector<uint16_t> seam_mask;  // colours | 0x100 prior
  int seam_ns = 0;
  bool seam_failed = false;
};

// Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one L2).  For a seam-plan launch of at most SEM_CHAIN_SWIZZLE_MAX chains
// (default 2,400) the planner reorders the chains so that workgroup b runs
// chain q(b) = x * (nch / 8) + min(x, nch % 8) + b / 8 (x = b % 8): each XCD
// then works on one contiguous run of chains, which share node columns of u
// and x_phys and the partial lines of y at their ends.  A permutation of the
// chain blocks of the packed arrays (slots, element positions, chain
// colours); node-indexed data and the seam sums are untouched, so results
// are bitwise those of the unpermuted plan.  Measured as a kernel-side
// remap (profiles/r04/xcd/, kernel median ms per action): cfg2 256^2 (2,341
// chains) 0.042 against 0.044; on the larger launches (4,993 - 9,472 chains)
// neutral to 6 % slower, hence the bound.  (Done in the kernel, as a
// run-time choice, it cost the headline kernel a scratch spill per round.)
int64_t chain_swizzle_max() {
  const char* e = std::getenv("SEM_CHAIN_SWIZZLE_MAX");
  return e ? (int64_t)std::atoll(e) : (int64_t)2400;
}

void chain_swizzle(Plan& P, int n, int rounds) {
  if (P.colour_start.size() != 2) return;
  const int64_t nch = P.colour_start[1] - P.colour_start[0];
  if (nch < 16 || nch > chain_swizzle_max()) return;
  const int64_t spc = (int64_t)rounds * chain_waves_of(n);  // slots per chain
  if (P.n_slots != nch * spc) return;
  constexpr int64_t NX = 8;
  const int64_t q = nch / NX, r = nch % NX;
  std::vector<int64_t> perm(nch), inv(nch);  // new position b <- old chain perm[b]
  for (int64_t b = 0; b < nch; ++b) {
    const int64_t x = b % NX, k = b / NX;
    perm[b] = x * q + (x < r ? x : r) + k;
    inv[perm[b]] = b;
  }
  const size_t per_slot = P.mapP.size() / (size_t)P.n_slots;
  std::vector<uint32_t> mp(P.mapP.size());
  std::vector<uint8_t> fill(P.slot_fill.size());
  for (int64_t b = 0; b < nch; ++b) {
    std::copy(P.mapP.begin() + perm[b] * spc * per_slot,
              P.mapP.begin() + (perm[b] + 1) * spc * per_slot, mp.begin() + b * spc * per_slot);
    std::copy(P.slot_fill.begin() + perm[b] * spc, P.slot_fill.begin() + (perm[b] + 1) * spc,
              fill.begin() + b * spc);
  }
  P.mapP.swap(mp);
  P.slot_fill.swap(fill);
  const int epw = epw_of(n);
  for (int& ep : P.epos) {
    if (ep < 0) continue;
    const int64_t slot = ep / epw, k = ep % epw;
    const int64_t ch = slot / spc, within = slot % spc;
    ep = (int)((inv[ch] * spc + within) * epw + k);
  }
  if ((int64_t)P.chain_colour.size() == nch) {
    std::vector<uint8_t> cc(nch);
    for (int64_t b = 0; b < nch; ++b) cc[b] = P.chain_colour[perm[b]];
    P.chain_colour.swap(cc);
  }
}

// groups of EPW consecutive elements, chains of CH consecutive groups
void groups_consecutive(int64_t n_elem, int epw, int CH, std::vector<int64_t>& gel) {
  const int64_t n_groups = (n_elem + epw - 1) / epw;
  const int64_t n_chains = (n_groups + CH - 1) / CH;
  gel.assign((size_t)(n_chains * CH * epw), -1);
  for (int64_t e = 0; e < n_elem; ++e) gel[e] = e;
}

// Block layout for structured numberings: the elements form
// "lines" -- runs of consecutive ids in which each element's last node column
// is the next one's first -- of equal length L, and line l + 1 sits on line l
// (element e + L has e's node row n-1 as its row 0).  A chain is a block of
// R stacked lines x CW * EPW elements; round rd of the chain is line rd of the
// block, so the node row between consecutive rounds is carried from one round
// to the next in registers (same wave, same lane) instead of being written by
// two chains.  Returns false (gel untouched) when the numbering is not of
// that form; the caller then uses groups_consecutive.
bool groups_blocks(const std::vector<uint32_t>& e2n, int64_t n_elem, int n, int epw, int CW,
                   int R, std::vector<int64_t>& gel) {
  const int nn = n * n;
  auto at = [&](int64_t e, int r, int jj) { return e2n[e * nn + r * n + jj]; };
  std::vector<int64_t> ls{0};
  for (int64_t e = 0; e + 1 < n_elem; ++e) {
    bool cont = true;
    for (int r = 0; r < n && cont; ++r) cont = at(e, r, n - 1) == at(e + 1, r, 0);
    if (!cont) ls.push_back(e + 1);
  }
  ls.push_back(n_elem);
  const int64_t nl = (int64_t)ls.size() - 1;
  if (nl < 2 || R < 2) return false;
  const int64_t len = ls[1] - ls[0];
  for (int64_t l = 0; l < nl; ++l)
    if (ls[l + 1] - ls[l] != len) return false;
  std::vector<uint8_t> on(nl, 0);  // line l + 1 sits on line l
  int64_t n_on = 0;
  for (int64_t l = 0; l + 1 < nl; ++l) {
    bool ok = true;
    for (int64_t i = 0; i < len && ok; ++i)
      for (int jj = 0; jj < n && ok; ++jj) ok = at(ls[l] + i + len, 0, jj) == at(ls[l] + i, n - 1, jj);
    on[l] = ok ? 1 : 0;
    n_on += ok ? 1 : 0;
  }
  if (n_on * 2 < nl - 1) return false;
  const int64_t seg = (int64_t)CW * epw;
  const int64_t nseg = (len + seg - 1) / seg;
  std::vector<int64_t> out;
  out.reserve((size_t)((nl + R - 1) / R * nseg * R * seg));
  for (int64_t l = 0; l < nl;) {
    int r = 1;  // stacked lines of this block
    while (r < R && l + r < nl && on[l + r - 1]) ++r;
    for (int64_t sg = 0; sg < nseg; ++sg)
      for (int rd = 0; rd < R; ++rd)
        for (int w = 0; w < CW; ++w)
          for (int k = 0; k < epw; ++k) {
            const int64_t i = sg * seg + (int64_t)w * epw + k;
            out.push_back(rd < r && i < len ? ls[l + rd] + i : -1);
          }
    l += r;
  }
  gel.swap(out);
  return true;
}

// node_state (may be empty): SEM_NODE_PRIOR = y already holds a value when
// this operator runs (first touches become read-modify-write, never zeroed);
// SEM_NODE_OTHER = another operator writes it (not zeroed when unreferenced).
// block_rounds >= 2: try the block layout with that many rounds (P.blocks
// tells whether it applied; rounds is then block_rounds).
int build_plan(const std::vector<uint32_t>& e2n, int64_t n_elem, int64_t n_node, int n,
               int rounds, const std::vector<uint8_t>& node_state, Plan& P, int seam = 0,
               int seam_dpn = 1, int block_rounds = 0) {
  const int epw = WAVE / n, lw = epw * n, nn = n * n;
  const int CW = chain_waves_of(n);  // groups of a chain that run concurrently
  std::vector<int64_t> gel;          // [group][lane element] -> element or -1
  // block_rounds < 0: AUTO -- 4 rounds when the mesh then still has enough
  // chains to fill the chip many times over (block_min_chains); fewer chains
  // leave a tail of lone workgroups that costs more than the carried rows save
  const bool block_auto = block_rounds < 0;
  if (block_auto) block_rounds = 4;
  P.blocks = block_rounds >= 2 && groups_blocks(e2n, n_elem, n, epw, CW, block_rounds, gel);
  if (P.blocks && block_auto &&
      (int64_t)gel.size() / ((int64_t)epw * CW * block_rounds) < block_min_chains(n, seam_dpn)) {
    P.blocks = false;
    gel.clear();
  }
  if (P.blocks) rounds = P.block_rounds = block_rounds;
  const int CH = CW * rounds;
  if (!P.blocks) groups_consecutive(n_elem, epw, CH, gel);
  const int64_t n_groups = (int64_t)gel.size() / epw;
  const int64_t n_chains = n_groups / CH;
  auto is_bnd = [n](int r, int jj) { return r == 0 || r == n - 1 || jj == 0 || jj == n - 1; };
  // references and conformity (interior local nodes must be unique)
  std::vector<uint32_t> cnt(n_node, 0);
  P.owner.assign(n_node, 0xFFFFFFFFu);
  for (int64_t t = 0; t < n_elem * nn; ++t) {
    if (e2n[t] >= n_node) return fail(SEM_E_INVALID, "element map references node >= n_node");
    if (!cnt[e2n[t]]++) P.owner[e2n[t]] = (uint32_t)(t / nn);
  }
  bool conforming = true;
  for (int64_t e = 0; e < n_elem && conforming; ++e)
    for (int r = 1; r < n - 1 && conforming; ++r)
      for (int jj = 1; jj < n - 1; ++jj)
        if (cnt[e2n[e * nn + r * n + jj]] != 1) {
          conforming = false;
          break;
        }
  P.conforming = conforming;
  auto shared_local = [&](int r, int jj) { return !conforming || is_bnd(r, jj); };
  // the elements of chain ch, lane order
  auto chain_elem = [&](int64_t ch, int64_t t) { return gel[(size_t)(ch * CH * epw + t)]; };
  const int64_t chain_len = (int64_t)CH * epw;
  // 2. chain colouring
  std::vector<uint8_t> cmask(n_node, 0);
  std::vector<int> colour(n_chains);
  {
    std::vector<int64_t> stamp(n_node, -1);
    std::vector<uint32_t> cn;
    for (int64_t ch = 0; ch < n_chains; ++ch) {
      int c = MAX_COLOURS;
      if (conforming) {
        cn.clear();
        uint32_t forb = 0;
        for (int64_t t = 0; t < chain_len; ++t) {
          const int64_t e = chain_elem(ch, t);
          if (e < 0) continue;
          for (int r = 0; r < n; ++r)
            for (int jj = 0; jj < n; ++jj)
              if (is_bnd(r, jj)) {
                const uint32_t gid = e2n[e * nn + r * n + jj];
                if (stamp[gid] != ch) {
                  stamp[gid] = ch;
                  cn.push_back(gid);
                  forb |= cmask[gid];
                }
              }
        }
        for (int q = 0; q < MAX_COLOURS; ++q)
          if (!(forb & (1u << q))) {
            c = q;
            break;
          }
        if (c < MAX_COLOURS)
          for (uint32_t gid : cn) cmask[gid] |= (uint8_t)(1u << c);
      }
      colour[ch] = c;
    }
  }
  std::vector<uint8_t>().swap(cmask);
  // 3. launch order: colour-major (one launch per colour), or for the seam
  // plan element order in one launch
  std::vector<int64_t> order(n_chains);
  if (seam == 2) {  // AUTO (seam_auto): high orders, or colour classes below ~1 generation
    std::vector<int64_t> per(MAX_COLOURS + 1, 0);
    for (int64_t ch = 0; ch < n_chains; ++ch) per[colour[ch]]++;
    seam = seam_auto(n, *std::max_element(per.begin(), per.end()), seam_dpn, P.blocks) ? 1 : 0;
  }
  P.seam = seam == 1 && conforming;
  for (int64_t ch = 0; ch < n_chains && P.seam; ++ch)
    if (colour[ch] >= MAX_COLOURS) P.seam = false;
  std::vector<uint8_t> nw;      // seam plan: chains writing each node (saturating)
  std::vector<uint16_t> smask;  // and their colours
  if (P.seam) {
    for (int64_t ch = 0; ch < n_chains; ++ch) order[ch] = ch;
    P.colour_start = {0, n_chains};
    nw.assign(n_node, 0);
    smask.assign(n_node, 0);
    std::vector<int32_t> lastc2(n_node, -1);
    int maxc = 0;
    for (int64_t ch = 0; ch < n_chains; ++ch) {
      maxc = std::max(maxc, colour[ch]);
      for (int64_t t = 0; t < chain_len; ++t) {
        const int64_t e = chain_elem(ch, t);
        if (e < 0) continue;
        for (int r = 0; r < n; ++r)
          for (int jj = 0; jj < n; ++jj)
            if (is_bnd(r, jj)) {
              const uint32_t gid = e2n[e * nn + r * n + jj];
              if (lastc2[gid] != (int32_t)ch) {
                lastc2[gid] = (int32_t)ch;
                if (nw[gid] < 255) nw[gid]++;
                smask[gid] |= (uint16_t)(1u << colour[ch]);
              }
            }
      }
    }
    P.seam_ns = maxc + 1;
    P.chain_colour.resize(n_chains);
    for (int64_t ch = 0; ch < n_chains; ++ch) P.chain_colour[ch] = (uint8_t)colour[ch];
  } else {
    std::vector<int64_t> count(MAX_COLOURS + 2, 0);
    for (int64_t ch = 0; ch < n_chains; ++ch) count[colour[ch] + 1]++;
    P.colour_start.assign(MAX_COLOURS + 2, 0);
    for (int q = 0; q <= MAX_COLOURS; ++q) P.colour_start[q + 1] = P.colour_start[q] + count[q + 1];
    std::vector<int64_t> fill(P.colour_start.begin(), P.colour_start.end() - 1);
    for (int64_t ch = 0; ch < n_chains; ++ch) order[fill[colour[ch]]++] = ch;
  }
  P.n_slots = n_chains * CH;
  P.epos.assign(n_elem, 0);
  P.slot_fill.assign(P.n_slots, 0);
  for (int64_t q = 0; q < n_chains; ++q)
    for (int i = 0; i < CH; ++i) {
      const int64_t g = order[q] * CH + i;
      const int64_t slot = q * CH + i;
      int fill = 0;
      for (int k = 0; k < epw; ++k) {
        const int64_t e = gel[g * epw + k];
        if (e < 0) break;  // real elements first
        P.epos[e] = (int)(slot * epw + k);
        fill = k + 1;
      }
      P.slot_fill[slot] = (uint8_t)fill;
    }
  // 4./5. validation and write codes, chain by chain in launch order
  P.mapP.assign((size_t)P.n_slots * n * lw, W_SKIP << CODE_SHIFT);
  std::vector<uint8_t> written(n_node, 0);
  if (!node_state.empty())
    for (int64_t i = 0; i < n_node; ++i) written[i] = (node_state[i] & SEM_NODE_PRIOR) ? 1 : 0;
  std::vector<int64_t> lastc(n_node, -1);  // chain of the last touch
  std::vector<int> lastt(n_node, -1);      // (group in chain) * n * lw + pos of the last touch
  // per entry: 0 normal, 1 merge-skip, 2 carry-skip, 3 carry-in, 4 row carry-out
  std::vector<uint8_t> act((size_t)CH * n * lw);
  P.n_atomic_groups = 0;
  P.row_carries = 0;
  P.round_rmw = false;
  bool seam_conflict = false;
  auto lane_elem = [&](int64_t g, int lane) -> int64_t {
    const int k = lane / n;
    return k < epw ? gel[g * epw + k] : -1;
  };
  for (int64_t q = 0; q < n_chains; ++q) {
    const int64_t ch = order[q];
    bool atomic_chain = colour[ch] >= MAX_COLOURS;
    std::fill(act.begin(), act.end(), (uint8_t)0);
    if (!atomic_chain) {
      // (c) row carries between consecutive rounds of a wave
      for (int i = 0; i + CW < CH; ++i) {
        const int64_t g = ch * CH + i;
        for (int lane = 0; lane < lw; ++lane) {
          const int jj = lane % n;
          const int64_t e = lane_elem(g, lane), f = lane_elem(g + CW, lane);
          if (e < 0 || f < 0) continue;
          if (e2n[f * nn + jj] == e2n[e * nn + (n - 1) * n + jj])
            act[(size_t)i * n * lw + (n - 1) * lw + lane] = 4;
        }
      }
      for (int i = 0; i < CH && !atomic_chain; ++i) {
        const int64_t g = ch * CH + i;
        for (int r = 0; r < n && !atomic_chain; ++r)
          for (int lane = 0; lane < lw; ++lane) {
            const int jj = lane % n;
            const int64_t e = lane_elem(g, lane);
            if (e < 0) continue;
            if (!shared_local(r, jj)) continue;
            const int pos = r * lw + lane;
            const int tag = i * n * lw + pos;
            if (act[tag] == 4) continue;  // carried to the next round: not a writer
            const uint32_t gid = e2n[e * nn + r * n + jj];
            if (lastc[gid] == ch) {
              const int pi = lastt[gid] / (n * lw), ppos = lastt[gid] % (n * lw);
              const bool same_round = (pi / CW) == (i / CW);
              if (pi == i && lane > 0 && ppos == pos - 1 && jj == 0 && (ppos % lw) % n == n - 1) {
                act[tag] = 1;  // merge into lane L (pos-1)
              } else if (pi == i - 1 && lane == 0 && ppos == r * lw + lw - 1) {
                act[tag] = 3;  // carry-in
                act[pi * n * lw + ppos] = 2;  // carry-out skip
              } else if (same_round) {
                atomic_chain = true;
                break;
              } else if (P.seam && nw[gid] >= 2) {
                // an earlier round of this chain stored the node into its
                // seam slot: a second plain slot store would drop it
                seam_conflict = true;
              } else {
                P.round_rmw = true;  // an earlier round of this chain: sequential, RMW
              }
            }
            lastc[gid] = ch;
            lastt[gid] = tag;
          }
      }
    }
    if (atomic_chain) {
      for (int i = 0; i < CH; ++i)
        if (gel[(ch * CH + i) * epw] >= 0) P.n_atomic_groups++;
    }
    for (int i = 0; i < CH; ++i) {
      const int64_t g = ch * CH + i;
      uint32_t* out = P.mapP.data() + (q * CH + i) * (int64_t)n * lw;
      for (int r = 0; r < n; ++r)
        for (int lane = 0; lane < lw; ++lane) {
          const int pos = r * lw + lane;
          const int jj = lane % n;
          const int64_t e = lane_elem(g, lane);
          if (e < 0) continue;  // padding stays SKIP
          const uint32_t gid = e2n[e * nn + r * n + jj];
          const uint8_t a = act[i * n * lw + pos];
          uint32_t code;
          if (!shared_local(r, jj)) {
            code = written[gid] ? W_RMW : W_STORE;  // conforming interior node: sole writer
          } else if (atomic_chain) {
            code = W_ATOMIC;
            if (!written[gid]) {
              P.zero.push_back(gid);
              written[gid] = 1;
            }
          } else if (a == 4) {
            code = W_ROWCARRY;
            P.row_carries++;
          } else if (a == 1) {
            code = W_SKIP;
            out[pos - 1] |= W_MERGE << CODE_SHIFT;
          } else if (a == 2) {
            code = W_SKIP;
          } else if (P.seam && nw[gid] >= 2) {
            code = W_ATOMIC;  // seam slot of this chain's colour (k_seam_sum)
            if (a == 3) code |= W_CARRY;
          } else {
            code = written[gid] ? W_RMW : W_STORE;
            written[gid] = 1;
            if (a == 3) code |= W_CARRY;
          }
          out[pos] = gid | (code << CODE_SHIFT);
        }
    }
  }
  for (int64_t i = 0; i < n_node; ++i)
    if (cnt[i] == 0 && (node_state.empty() || !node_state[i])) P.zero.push_back((uint32_t)i);
  std::sort(P.zero.begin(), P.zero.end());
  P.n_rmw = 0;
  for (const uint32_t e : P.mapP) P.n_rmw += ((e >> CODE_SHIFT) & 3u) == W_RMW ? 1 : 0;
  if (P.seam) {
    if (P.n_atomic_groups || seam_conflict) {  // sharing the seam slots cannot express
      P.seam = false;
      P.seam_failed = true;  // the caller plans again without seams
      return SEM_OK;
    }
    for (int64_t i = 0; i < n_node; ++i)
      if (nw[i] >= 2) {
        P.seam_gid.push_back((uint32_t)i);
        const bool prior = !node_state.empty() && (node_state[i] & SEM_NODE_PRIOR);
        P.seam_mask.push_back((uint16_t)(smask[i] | (prior ? 0x100u : 0u)));
      }
  }
  return SEM_OK;
}


// 16-bit form of a column-kernel plan's packed map: one 32-bit
// base per (slot, row) = the smallest node id of the row's real elements,
// entries (gid - base) | code << 12, for rows spanning fewer than 4096 ids
// (locality-ordered meshes; 57 consecutive ids per row at p = 8 on the
// structured mesh); padding entries keep offset 0.  A group with a wider row
// is flagged (base[slot][0] = M16_WIDE) and reads the 32-bit map; the form is
// used only when at most 1 / 16 of the groups are flagged.
static bool build_map16(const Plan& P, int64_t n_elem, int n, int epw, int64_t n_groups,
                        std::vector<uint16_t>& m16, std::vector<uint32_t>& base) {
  const int lw = epw * n;
  m16.assign((size_t)P.n_slots * n * lw, (uint16_t)(W_SKIP << M16_CODE_SHIFT));
  base.assign((size_t)P.n_slots * n, 0u);
  int64_t wide = 0;
  for (int64_t sl = 0; sl < P.n_slots; ++sl) {
    if (!P.slot_fill[sl]) continue;
    const int lanes = P.slot_fill[sl] * n;
    bool fits = true;
    for (int r = 0; r < n && fits; ++r) {
      const uint32_t* row = &P.mapP[((size_t)sl * n + r) * lw];
      uint32_t lo = 0xFFFFFFFFu, hi = 0;
      for (int l = 0; l < lanes; ++l) {
        lo = std::min(lo, row[l] & GID_MASK);
        hi = std::max(hi, row[l] & GID_MASK);
      }
      base[(size_t)sl * n + r] = lo;
      fits = hi - lo <= M16_OFF_MASK;
    }
    if (!fits) {
      base[(size_t)sl * n] = M16_WIDE;
      ++wide;
      continue;
    }
    for (int r = 0; r < n; ++r) {
      const uint32_t* row = &P.mapP[((size_t)sl * n + r) * lw];
      const uint32_t lo = base[(size_t)sl * n + r];
      uint16_t* out = &m16[((size_t)sl * n + r) * lw];
      for (int l = 0; l < lanes; ++l)
        out[l] = (uint16_t)(((row[l] & GID_MASK) - lo) | ((row[l] >> CODE_SHIFT) << M16_CODE_SHIFT));
    }
  }
  int64_t filled = 0;
  for (uint8_t f : P.slot_fill) filled += f ? 1 : 0;
  (void)n_groups;
  return wide * 16 <= filled;
}

// Pattern table of a 16-bit map (the PAT kernels, csrc/sem_kernels.h): every
// group's block of n x lw entries (offsets and codes) deduplicated; the
// table replaces m16 and each group's pattern id goes into bits 28-31 of its
// bases 1..min(4, n - 1).  Declined when an order has no PAT kernels, when
// more than 1 / 8 of the groups are distinct, or past 16^min(4, n - 1)
// patterns.  On the
// structured block layout a handful of layouts (which rows are carried,
// slotted or merged) cover every group.
static bool build_map_patterns(std::vector<uint16_t>& m16, std::vector<uint32_t>& mb, int n,
                               int lw, int64_t n_slots, int64_t* n_pat) {
  *n_pat = 0;
  if (n < 3 || n > 31 || !((SEM_MAP_PATTERN_N >> n) & 1u) || SEM_MAP_TOUCH) return false;
  const int Q = std::min(4, n - 1);  // bases carrying the id (PatternMap::id_rows)
  const uint32_t max_pat = 1u << (4 * Q);
  const size_t blk = (size_t)n * lw;
  std::unordered_map<uint64_t, std::vector<uint32_t>> seen;
  std::vector<uint16_t> table;
  std::vector<uint32_t> pid((size_t)n_slots, 0);
  for (int64_t sl = 0; sl < n_slots; ++sl) {
    if (mb[(size_t)sl * n] == M16_WIDE) continue;  // reads the 32-bit map
    const uint16_t* e = &m16[(size_t)sl * blk];
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < blk; ++i) h = (h ^ e[i]) * 1099511628211ull;
    auto& cand = seen[h];
    uint32_t id = 0xFFFFFFFFu;
    for (uint32_t c : cand)
      if (std::memcmp(&table[(size_t)c * blk], e, blk * sizeof(uint16_t)) == 0) {
        id = c;
        break;
      }
    if (id == 0xFFFFFFFFu) {
      id = (uint32_t)(table.size() / blk);
      if (id >= max_pat || (int64_t)id * 8 > n_slots) return false;
      table.insert(table.end(), e, e + blk);
      cand.push_back(id);
    }
    pid[(size_t)sl] = id;
  }
  // bases 1..Q must have their top 4 bits free (node ids < 2^28: packed maps)
  for (int64_t sl = 0; sl < n_slots; ++sl) {
    if (mb[(size_t)sl * n] == M16_WIDE) continue;
    for (int q = 1; q <= Q; ++q)
      if (mb[(size_t)sl * n + q] & ~GID_MASK) return false;
  }
  for (int64_t sl = 0; sl < n_slots; ++sl) {
    if (mb[(size_t)sl * n] == M16_WIDE) continue;
    for (int q = 0; q < Q; ++q)
      mb[(size_t)sl * n + 1 + q] |= ((pid[(size_t)sl] >> (4 * q)) & 15u) << 28;
  }
  *n_pat = (int64_t)(table.size() / blk);
  m16.swap(table);
  return true;
}

// ---------------------------------------------------------------------------
// Element-level plan for the MFMA kernel (one element per wavefront, no
// chains): elements are greedily coloured so that elements of one colour
// share no node (a per-node colour bitmask over their element-boundary nodes,
// all nodes on a non-conforming map); one launch per colour, natural element
// order inside a colour; STORE for the first writer of a node in launch
// order, RMW after it.  Elements that would need more than MAX_COLOURS
// colours, or that reference one node twice, go to a final class whose
// shareable nodes are written with atomics.  Group = slot = one element, so
// the packed map and factors are compact per element ([slot][r][j]).
// ---------------------------------------------------------------------------
// seam = 1 (n = 17 kernel): one launch over all elements in breadth-first
// order instead of one per colour; a node of several elements is stored by
// each into the slot of its element's colour and summed by k_seam_sum (the
// column kernel's seam plan with one element per chain).
// seams for the n = 17 MFMA kernel under AUTO (SEM_SEAM=0 / 1 forces): off.
// p = 16, 198^2 on MI355X (profiles/r03/mfma17): one launch 0.161 ms + seam
// sums 0.052 ms (the seam slots of horizontal element edges are scattered
// 8-byte accesses) against 4 colour launches of 0.049 ms
#ifndef MFMA_SEAM_AUTO
#define MFMA_SEAM_AUTO 0
#endif
int build_plan_elem(const std::vector<uint32_t>& e2n, int64_t n_elem, int64_t n_node, int n,
                    const std::vector<uint8_t>& node_state, Plan& P, int seam = 0) {
  const int nn = n * n;
  auto is_bnd = [n](int r, int jj) { return r == 0 || r == n - 1 || jj == 0 || jj == n - 1; };
  std::vector<uint32_t> cnt(n_node, 0);
  P.owner.assign(n_node, 0xFFFFFFFFu);
  for (int64_t t = 0; t < n_elem * nn; ++t) {
    if (e2n[t] >= n_node) return fail(SEM_E_INVALID, "element map references node >= n_node");
    if (!cnt[e2n[t]]++) P.owner[e2n[t]] = (uint32_t)(t / nn);
  }
  bool conforming = true;
  for (int64_t e = 0; e < n_elem && conforming; ++e)
    for (int r = 1; r < n - 1 && conforming; ++r)
      for (int jj = 1; jj < n - 1; ++jj)
        if (cnt[e2n[e * nn + r * n + jj]] != 1) {
          conforming = false;
          break;
        }
  P.conforming = conforming;
  auto shared_local = [&](int r, int jj) { return !conforming || is_bnd(r, jj); };
  // breadth-first element order over shared nodes: greedy colouring along it
  // needs far fewer colours than along a random element order (split
  // triangles, shuffled: 8 instead of 11), and packing classes in it keeps
  // neighbouring elements in neighbouring groups
  std::vector<int64_t> bfs;
  bfs.reserve(n_elem);
  {
    std::vector<int64_t> start(n_node + 1, 0);
    for (int64_t e = 0; e < n_elem; ++e)
      for (int r = 0; r < n; ++r)
        for (int jj = 0; jj < n; ++jj)
          if (shared_local(r, jj)) start[e2n[e * nn + r * n + jj] + 1]++;
    for (int64_t i = 0; i < n_node; ++i) start[i + 1] += start[i];
    std::vector<int64_t> inc(start[n_node]), fill(start.begin(), start.end() - 1);
    for (int64_t e = 0; e < n_elem; ++e)
      for (int r = 0; r < n; ++r)
        for (int jj = 0; jj < n; ++jj)
          if (shared_local(r, jj)) inc[fill[e2n[e * nn + r * n + jj]]++] = e;
    std::vector<uint8_t> seen(n_elem, 0);
    for (int64_t s0 = 0; s0 < n_elem; ++s0) {
      if (seen[s0]) continue;
      seen[s0] = 1;
      size_t head = bfs.size();
      bfs.push_back(s0);
      while (head < bfs.size()) {
        const int64_t e = bfs[head++];
        for (int r = 0; r < n; ++r)
          for (int jj = 0; jj < n; ++jj) {
            if (!shared_local(r, jj)) continue;
            const uint32_t gid = e2n[e * nn + r * n + jj];
            for (int64_t t = start[gid]; t < start[gid + 1]; ++t)
              if (!seen[inc[t]]) {
                seen[inc[t]] = 1;
                bfs.push_back(inc[t]);
              }
          }
      }
    }
  }
  std::vector<uint8_t> cmask(n_node, 0);
  std::vector<int64_t> stamp(n_node, -1);
  std::vector<int> colour(n_elem);
  std::vector<uint32_t> cn;
  for (const int64_t e : bfs) {
    cn.clear();
    uint32_t forb = 0;
    bool dup = false;
    for (int r = 0; r < n; ++r)
      for (int jj = 0; jj < n; ++jj)
        if (shared_local(r, jj)) {
          const uint32_t gid = e2n[e * nn + r * n + jj];
          if (stamp[gid] == e) {
            dup = true;
            continue;
          }
          stamp[gid] = e;
          cn.push_back(gid);
          forb |= cmask[gid];
        }
    int c = MAX_COLOURS;
    if (!dup)
      for (int q = 0; q < MAX_COLOURS; ++q)
        if (!(forb & (1u << q))) {
          c = q;
          break;
        }
    if (c < MAX_COLOURS)
      for (uint32_t gid : cn) cmask[gid] |= (uint8_t)(1u << c);
    colour[e] = c;
  }
  std::vector<uint8_t>().swap(cmask);
  std::vector<int64_t> order(n_elem);
  int maxc = 0;
  for (int64_t e = 0; e < n_elem; ++e) maxc = std::max(maxc, colour[e]);
  P.seam = seam == 1 && conforming && maxc < MAX_COLOURS;
  if (P.seam) {
    order = bfs;
    P.colour_start = {0, n_elem};
    P.seam_ns = maxc + 1;
    P.chain_colour.resize(n_elem);
    for (int64_t q = 0; q < n_elem; ++q) P.chain_colour[q] = (uint8_t)colour[order[q]];
  } else {
    std::vector<int64_t> count(MAX_COLOURS + 2, 0);
    for (int64_t e = 0; e < n_elem; ++e) count[colour[e] + 1]++;
    P.colour_start.assign(MAX_COLOURS + 2, 0);
    for (int q = 0; q <= MAX_COLOURS; ++q)
      P.colour_start[q + 1] = P.colour_start[q] + count[q + 1];
    std::vector<int64_t> fill(P.colour_start.begin(), P.colour_start.end() - 1);
    for (int64_t e = 0; e < n_elem; ++e) order[fill[colour[e]]++] = e;
  }
  P.n_slots = n_elem;
  P.epos.assign(n_elem, 0);
  for (int64_t q = 0; q < n_elem; ++q) P.epos[order[q]] = (int)q;
  P.slot_fill.assign(n_elem, 1);
  P.mapP.assign((size_t)n_elem * nn, W_SKIP << CODE_SHIFT);
  std::vector<uint8_t> written(n_node, 0);
  if (!node_state.empty())
    for (int64_t i = 0; i < n_node; ++i) written[i] = (node_state[i] & SEM_NODE_PRIOR) ? 1 : 0;
  P.n_atomic_groups = 0;
  for (int64_t q = 0; q < n_elem; ++q) {
    const int64_t e = order[q];
    const bool atomic = colour[e] >= MAX_COLOURS;
    if (atomic) P.n_atomic_groups++;
    uint32_t* out = P.mapP.data() + q * nn;
    for (int r = 0; r < n; ++r)
      for (int jj = 0; jj < n; ++jj) {
        const uint32_t gid = e2n[e * nn + r * n + jj];
        uint32_t code;
        if (P.seam && cnt[gid] >= 2) {
          code = W_ATOMIC;  // seam slot of this element's colour (k_seam_sum)
        } else if (atomic && shared_local(r, jj)) {
          code = W_ATOMIC;
          if (!written[gid]) P.zero.push_back(gid);
        } else {
          code = written[gid] ? W_RMW : W_STORE;
        }
        written[gid] = 1;
        out[r * n + jj] = gid | (code << CODE_SHIFT);
      }
  }
  for (int64_t i = 0; i < n_node; ++i)
    if (cnt[i] == 0 && (node_state.empty() || !node_state[i])) P.zero.push_back((uint32_t)i);
  std::sort(P.zero.begin(), P.zero.end());
  P.n_rmw = 0;
  for (const uint32_t e : P.mapP) P.n_rmw += ((e >> CODE_SHIFT) & 3u) == W_RMW ? 1 : 0;
  if (P.seam) {
    std::vector<uint16_t> smask(n_node, 0);
    for (int64_t e = 0; e < n_elem; ++e)
      for (int t = 0; t < nn; ++t) smask[e2n[e * nn + t]] |= (uint16_t)(1u << colour[e]);
    for (int64_t i = 0; i < n_node; ++i)
      if (cnt[i] >= 2) {
        P.seam_gid.push_back((uint32_t)i);
        const bool prior = !node_state.empty() && (node_state[i] & SEM_NODE_PRIOR);
        P.seam_mask.push_back((uint16_t)(smask[i] | (prior ? 0x100u : 0u)));
      }
  }
  return SEM_OK;
}

// ---------------------------------------------------------------------------
// Element-coloured plan for the column kernel (meshes whose element order
// defeats the chain patterns: irregular valence, random element order).
// Elements are greedily coloured, in breadth-first order over shared nodes,
// so that elements of one colour share no node, then packed colour class by
// colour class, in that order inside a class, into groups of EPW elements and
// chains of chain_waves_of(n) * rounds groups (a class's last group / chain may
// be partly empty).  Nothing inside a launch shares a node, so the codes
// are plain STORE (first writer in launch order) / RMW with no merge or
// carry; elements needing more than MAX_COLOURS colours go to a final
// all-atomic class.  Chosen by sem_set_map when the chain plan would send
// more than half of its groups to the atomic fallback and this plan sends
// fewer.
// ---------------------------------------------------------------------------
int build_plan_ecol(const std::vector<uint32_t>& e2n, int64_t n_elem, int64_t n_node, int n,
                    int rounds, const std::vector<uint8_t>& node_state, Plan& P) {
  const int epw = WAVE / n, lw = epw * n, nn = n * n;
  const int CH = chain_waves_of(n) * rounds;
  auto is_bnd = [n](int r, int jj) { return r == 0 || r == n - 1 || jj == 0 || jj == n - 1; };
  std::vector<uint32_t> cnt(n_node, 0);
  P.owner.assign(n_node, 0xFFFFFFFFu);
  for (int64_t t = 0; t < n_elem * nn; ++t) {
    if (e2n[t] >= n_node) return fail(SEM_E_INVALID, "element map references node >= n_node");
    if (!cnt[e2n[t]]++) P.owner[e2n[t]] = (uint32_t)(t / nn);
  }
  bool conforming = true;
  for (int64_t e = 0; e < n_elem && conforming; ++e)
    for (int r = 1; r < n - 1 && conforming; ++r)
      for (int jj = 1; jj < n - 1; ++jj)
        if (cnt[e2n[e * nn + r * n + jj]] != 1) {
          conforming = false;
          break;
        }
  P.conforming = conforming;
  auto shared_local = [&](int r, int jj) { return !conforming || is_bnd(r, jj); };
  // breadth-first element order over shared nodes: greedy colouring along it
  // needs far fewer colours than along a random element order (split
  // triangles, shuffled: 8 instead of 11), and packing classes in it keeps
  // neighbouring elements in neighbouring groups
  std::vector<int64_t> bfs;
  bfs.reserve(n_elem);
  {
    std::vector<int64_t> start(n_node + 1, 0);
    for (int64_t e = 0; e < n_elem; ++e)
      for (int r = 0; r < n; ++r)
        for (int jj = 0; jj < n; ++jj)
          if (shared_local(r, jj)) start[e2n[e * nn + r * n + jj] + 1]++;
    for (int64_t i = 0; i < n_node; ++i) start[i + 1] += start[i];
    std::vector<int64_t> inc(start[n_node]), fill(start.begin(), start.end() - 1);
    for (int64_t e = 0; e < n_elem; ++e)
      for (int r = 0; r < n; ++r)
        for (int jj = 0; jj < n; ++jj)
          if (shared_local(r, jj)) inc[fill[e2n[e * nn + r * n + jj]]++] = e;
    std::vector<uint8_t> seen(n_elem, 0);
    for (int64_t s0 = 0; s0 < n_elem; ++s0) {
      if (seen[s0]) continue;
      seen[s0] = 1;
      size_t head = bfs.size();
      bfs.push_back(s0);
      while (head < bfs.size()) {
        const int64_t e = bfs[head++];
        for (int r = 0; r < n; ++r)
          for (int jj = 0; jj < n; ++jj) {
            if (!shared_local(r, jj)) continue;
            const uint32_t gid = e2n[e * nn + r * n + jj];
            for (int64_t t = start[gid]; t < start[gid + 1]; ++t)
              if (!seen[inc[t]]) {
                seen[inc[t]] = 1;
                bfs.push_back(inc[t]);
              }
          }
      }
    }
  }
  std::vector<uint8_t> cmask(n_node, 0);
  std::vector<int64_t> stamp(n_node, -1);
  std::vector<int> colour(n_elem);
  std::vector<uint32_t> cn;
  for (const int64_t e : bfs) {
    cn.clear();
    uint32_t forb = 0;
    bool dup = false;
    for (int r = 0; r < n; ++r)
      for (int jj = 0; jj < n; ++jj)
        if (shared_local(r, jj)) {
          const uint32_t gid = e2n[e * nn + r * n + jj];
          if (stamp[gid] == e) {
            dup = true;
            continue;
          }
          stamp[gid] = e;
          cn.push_back(gid);
          forb |= cmask[gid];
        }
    int c = MAX_COLOURS;
    if (!dup)
      for (int q = 0; q < MAX_COLOURS; ++q)
        if (!(forb & (1u << q))) {
          c = q;
          break;
        }
    if (c < MAX_COLOURS)
      for (uint32_t gid : cn) cmask[gid] |= (uint8_t)(1u << c);
    colour[e] = c;
  }
  std::vector<uint8_t>().swap(cmask);
  // pack each class into groups and chains
  std::vector<std::vector<int64_t>> cls(MAX_COLOURS + 1);
  for (const int64_t e : bfs) cls[colour[e]].push_back(e);
  P.colour_start.assign(MAX_COLOURS + 2, 0);
  int64_t n_chains = 0;
  for (int q = 0; q <= MAX_COLOURS; ++q) {
    const int64_t groups = ((int64_t)cls[q].size() + epw - 1) / epw;
    n_chains += (groups + CH - 1) / CH;
    P.colour_start[q + 1] = n_chains;
  }
  P.n_slots = n_chains * CH;
  P.epos.assign(n_elem, 0);
  P.slot_fill.assign(P.n_slots, 0);
  P.mapP.assign((size_t)P.n_slots * n * lw, W_SKIP << CODE_SHIFT);
  std::vector<uint8_t> written(n_node, 0);
  if (!node_state.empty())
    for (int64_t i = 0; i < n_node; ++i) written[i] = (node_state[i] & SEM_NODE_PRIOR) ? 1 : 0;
  P.n_atomic_groups = 0;
  for (int q = 0; q <= MAX_COLOURS; ++q) {
    const bool atomic = q == MAX_COLOURS;
    const int64_t slot0 = P.colour_start[q] * CH;
    const auto& L = cls[q];
    for (size_t idx = 0; idx < L.size(); ++idx) {
      const int64_t e = L[idx];
      const int64_t slot = slot0 + (int64_t)(idx / epw);
      const int k = (int)(idx % epw);
      P.epos[e] = (int)(slot * epw + k);
      P.slot_fill[slot] = (uint8_t)(k + 1);
      uint32_t* out = P.mapP.data() + slot * (int64_t)n * lw;
      for (int r = 0; r < n; ++r)
        for (int jj = 0; jj < n; ++jj) {
          const uint32_t gid = e2n[e * nn + r * n + jj];
          uint32_t code;
          if (atomic && shared_local(r, jj)) {
            code = W_ATOMIC;
            if (!written[gid]) P.zero.push_back(gid);
          } else {
            code = written[gid] ? W_RMW : W_STORE;
          }
          written[gid] = 1;
          out[r * lw + k * n + jj] = gid | (code << CODE_SHIFT);
        }
    }
    if (atomic) P.n_atomic_groups += ((int64_t)L.size() + epw - 1) / epw;
  }
  for (int64_t i = 0; i < n_node; ++i)
    if (cnt[i] == 0 && (node_state.empty() || !node_state[i])) P.zero.push_back((uint32_t)i);
  std::sort(P.zero.begin(), P.zero.end());
  return SEM_OK;
}

}  // namespace
extern "C" {

int sem_ctx_create(sem_ctx** out, int p, int64_t n_elem, int64_t n_node, int dpn, int device) {
  return sem_ctx_create_nd(out, 2, p, n_elem, n_node, dpn, device);
}

int sem_ctx_create_nd(sem_ctx** out, int ndim, int p, int64_t n_elem, int64_t n_node, int dpn,
                      int device) {
  if (!out) return fail(SEM_E_INVALID, "null ctx pointer");
  *out = nullptr;
  if (ndim != 2 && ndim != 3)
    return fail(SEM_E_NOTIMPL, "operators on quadrilaterals (ndim 2) and hexahedra (ndim 3) only");
  if (p < 1) return fail(SEM_E_INVALID, "Must specify an order of 1 or greater.");
  if (p > SEM_MAX_ORDER)
    return fail(SEM_E_NOTIMPL, "operator kernels built for orders 1.." +
                                   std::to_string(SEM_MAX_ORDER));
  if (n_elem < 1 || n_node < 1 || dpn < 1 || dpn > 2)
    return fail(SEM_E_INVALID, "bad sizes (n_elem, n_node >= 1, dpn in {1,2})");
  if (ndim == 2 && n_node > (int64_t)GID_MASK)
    return fail(SEM_E_INVALID, "n_node exceeds the per-GPU limit of 2^28 - 1 nodes");
  if (n_node > (int64_t)0xFFFFFFFFll)
    return fail(SEM_E_INVALID, "n_node exceeds the uint32 element map");
  DeviceGuard g(device);
  sem_ctx* c = new sem_ctx();
  c->p = p;
  c->n = p + 1;
  c->dpn = dpn;
  c->device = device;
  c->n_elem = n_elem;
  c->n_node = n_node;
  c->epw = epw_of(c->n);
  c->lw = c->epw * c->n;
  c->n_groups = (n_elem + c->epw - 1) / c->epw;
  if (const char* s = std::getenv("SEM_GEOM_MODE")) c->geom_mode = std::atoi(s);
  if (const char* s = std::getenv("SEM_KERNEL")) c->kernel = std::atoi(s);
  if (c->n_groups > 0x7FFFFFFFll) {
    delete c;
    return fail(SEM_E_INVALID, "too many elements");
  }
  hipError_t e1 = hipMalloc(&c->d_D, SEM_MAXN * SEM_MAXN * sizeof(double));
  hipError_t e2 = hipMalloc(&c->d_w, SEM_MAXN * sizeof(double));
  hipError_t e3 = hipMalloc(&c->d_Vinv, SEM_MAXN * SEM_MAXN * sizeof(double));
  hipError_t e4 = hipMalloc(&c->d_bad, sizeof(unsigned long long));
  if (!e4) e4 = hipMalloc(&c->d_deo, sizeof(DEOData<SEM_MAXN>));
  if (e1 || e2 || e3 || e4) {
    sem_ctx_destroy(c);
    return fail(SEM_E_HIP, "hipMalloc failed in sem_ctx_create");
  }
  if (ndim == 3) {
    c->ndim = 3;
    if (const int rc = semh::ctx_init(c)) {
      sem_ctx_destroy(c);
      return rc;
    }
  }
  *out = c;
  return SEM_OK;
}

void sem_ctx_destroy(sem_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  semh::ctx_free(c);
  (void)hipFree(c->d_D);
  (void)hipFree(c->d_w);
  (void)hipFree(c->d_Vinv);
  (void)hipFree(c->d_deo);
  (void)hipFree(c->d_mapP);
  (void)hipFree(c->d_map16);
  (void)hipFree(c->d_mbase);
  (void)hipFree(c->d_epos);
  (void)hipFree(c->d_zero);
  for (double* g : c->d_GP) (void)hipFree(g);
  (void)hipFree(c->d_lin);
  (void)hipFree(c->d_XG);
  (void)hipFree(c->d_owner);
  (void)hipFree(c->d_bad);
  (void)hipFree(c->d_ccol);
  (void)hipFree(c->d_seam_gid);
  (void)hipFree(c->d_seam_mask);
  (void)hipFree(c->d_seam_buf);
  (void)hipFree(c->d_dot);
  delete c;
}

int sem_set_basis(sem_ctx* c, const double* hD, const double* hw) {
  if (!c || !hD || !hw) return fail(SEM_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  const int n = c->n;
  // the kernels use D in even-odd form and half of w: a node set symmetric
  // about 0 (GLL), D[n-1-i][n-1-j] = -D[i][j] and w[n-1-i] = w[i]
  double dmax = 0.0, wmax = 0.0, dasym = 0.0, wasym = 0.0;
  for (int i = 0; i < n; ++i) {
    wmax = std::max(wmax, std::fabs(hw[i]));
    wasym = std::max(wasym, std::fabs(hw[i] - hw[n - 1 - i]));
    for (int j = 0; j < n; ++j) {
      dmax = std::max(dmax, std::fabs(hD[i * n + j]));
      dasym = std::max(dasym, std::fabs(hD[i * n + j] + hD[(n - 1 - i) * n + (n - 1 - j)]));
    }
  }
  if (!(dasym <= 1e-12 * dmax) || !(wasym <= 1e-14 * wmax))
    return fail(SEM_E_INVALID,
                "sem_set_basis: D and w must come from a node set symmetric about 0 (GLL)");
  c->epoch++;
  std::memcpy(c->hD, hD, sizeof(double) * n * n);
  std::memcpy(c->hw, hw, sizeof(double) * n);
  {
    const double* kd = sem_deo_const_d(n);
    // SEM_CONST_D: unset = the per-order choice (const_d_order), 0 = never,
    // 1 = wherever D matches
    const char* e = std::getenv("SEM_CONST_D");
    const bool want = e ? e[0] == '1' : const_d_order(n);
    c->const_d = want && kd && std::memcmp(kd, hD, sizeof(double) * n * n) == 0;
  }
  HIP_TRY(hipMemcpy(c->d_D, hD, sizeof(double) * n * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_w, hw, sizeof(double) * n, hipMemcpyHostToDevice));
  int rc = SEM_OK;
  SEM_DISPATCH_N(rc, n, upload_deo, c);
  if (rc) return rc;
  c->have_basis = true;
  return SEM_OK;
}

int sem_set_map(sem_ctx* c, const uint32_t* d_e2n, void* stream) {
  return sem_set_map_shared(c, d_e2n, nullptr, stream);
}

int sem_set_map_shared(sem_ctx* c, const uint32_t* d_e2n, const uint8_t* d_node_state,
                       void* stream) {
  if (!c || !d_e2n) return fail(SEM_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  if (c->ndim == 3) {
    if (d_node_state)
      return fail(SEM_E_NOTIMPL, "sem_set_map_shared: node states on hexahedra are not supported");
    return semh::set_map(c, d_e2n, S(stream));
  }
  c->epoch++;
  c->map_epoch++;
  hipStream_t st = S(stream);
  const int n = c->n;
  std::vector<uint32_t> h((size_t)c->n_elem * n * n);
  std::vector<uint8_t> state;
  HIP_TRY(hipMemcpyAsync(h.data(), d_e2n, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (d_node_state) {
    state.resize(c->n_node);
    HIP_TRY(hipMemcpyAsync(state.data(), d_node_state, state.size(), hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  Plan P;
  // measured on MI355X at p = 8, 10^6 elements: 1 round 0.79-0.81 ms,
  // 2: 0.85, 4: 0.88, 8: 0.97 (longer chains: fewer workgroups, lockstep).
  // Single-wave chains (no workgroup barrier, register carry, next-group
  // prefetch) measured 0.90-0.95 ms (nodal) and 0.89-0.92 (stored): the
  // prefetch registers halve occupancy.  Not kept.
  int rounds = 1;
  if (const char* s = std::getenv("SEM_CHAIN_ROUNDS")) rounds = std::max(1, std::atoi(s));
  const bool mfma = want_mfma(c);
  // block layout (groups_blocks): rounds stacked along the lines, the node
  // row between rounds carried in registers; SEM_BLOCK_ROUNDS=R forces R
  // (0 or 1: off), default AUTO (build_plan, block_min_chains)
  int brounds = -1;  // AUTO (build_plan)
  if (const char* s = std::getenv("SEM_BLOCK_ROUNDS")) brounds = std::atoi(s);
  // seam plan: one launch + seam sums; SEM_SEAM=1 / 0 forces / forbids it;
  // default AUTO (seam_auto, per dofs per node)
  int seam = 0;
  {
    const char* e = std::getenv("SEM_SEAM");
    seam = e ? (std::atoi(e) == 1 ? 1 : 0) : 2;
  }
  // the n = 17 MFMA kernel takes seams by default (MFMA_SEAM_AUTO); the
  // n <= 16 MFMA kernel has no seam form
  const int eseam = (mfma && n == 17) ? (seam == 2 ? MFMA_SEAM_AUTO : seam) : 0;
  int rc = mfma ? build_plan_elem(h, c->n_elem, c->n_node, n, state, P, eseam)
                : build_plan(h, c->n_elem, c->n_node, n, rounds, state, P, seam, c->dpn, brounds);
  if (!rc && P.seam_failed) {
    P = Plan();
    rc = build_plan(h, c->n_elem, c->n_node, n, rounds, state, P, 0, c->dpn, brounds);
  }
  if (rc) return rc;
  if (P.blocks) rounds = P.block_rounds;
  // XCD-contiguous chain order for small seam-plan launches (chain_swizzle)
  if (!mfma && P.seam) chain_swizzle(P, n, rounds);
  // element-coloured fallback for orders that defeat the chain patterns
  // (SEM_PLAN=1 forces it, SEM_PLAN=0 forbids it)
  const char* penv = std::getenv("SEM_PLAN");
  const int pmode = penv ? std::atoi(penv) : -1;
  c->ecol = false;
  const int64_t ng_col = (c->n_elem + epw_of(n) - 1) / epw_of(n);
  // element colouring gives up the chains' gather locality: on a structured
  // mesh whose element order breaks a quarter of the chains it measured 2.4x
  // slower than the chains with their atomics, so it is tried only when most
  // groups would be atomic
  if (!mfma && pmode != 0 && (pmode == 1 || P.n_atomic_groups * 2 > ng_col)) {
    Plan Q;
    if ((rc = build_plan_ecol(h, c->n_elem, c->n_node, n, rounds, state, Q))) return rc;
    if (pmode == 1 || Q.n_atomic_groups < P.n_atomic_groups) {
      P = std::move(Q);
      c->ecol = true;
    }
  }
  c->mfma = mfma;
  c->epw = mfma ? 1 : epw_of(n);
  c->lw = c->epw * n;
  c->n_groups = (c->n_elem + c->epw - 1) / c->epw;
  c->rounds = mfma ? 1 : rounds;
  c->blocks = !mfma && !c->ecol && P.blocks;
  c->row_carries = c->blocks ? P.row_carries : 0;
  c->round_sync = c->ecol || P.round_rmw;
  c->n_slots = P.n_slots;
  std::vector<uint32_t>().swap(h);
  c->d_e2n = d_e2n;
  (void)hipFree(c->d_mapP);
  (void)hipFree(c->d_epos);
  (void)hipFree(c->d_zero);
  c->d_mapP = nullptr;
  c->d_epos = nullptr;
  c->d_zero = nullptr;
  HIP_TRY(hipMalloc(&c->d_mapP, P.mapP.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(c->d_mapP, P.mapP.data(), P.mapP.size() * sizeof(uint32_t),
                    hipMemcpyHostToDevice));
  // 16-bit map for the column kernel (SEM_MAP16=0 keeps the 32-bit stream):
  // measured at p = 8, 10^6 elements: see DESIGN.md §4.1
  (void)hipFree(c->d_map16);
  (void)hipFree(c->d_mbase);
  c->d_map16 = nullptr;
  c->d_mbase = nullptr;
  c->map16 = false;
  c->map_pat = false;
  c->n_map_pat = 0;
  const char* m16env = std::getenv("SEM_MAP16");
  if (!mfma && !(m16env && std::atoi(m16env) == 0)) {
    std::vector<uint16_t> m16;
    std::vector<uint32_t> mb;
    if (build_map16(P, c->n_elem, n, c->epw, c->n_groups, m16, mb)) {
      const char* pe = std::getenv("SEM_MAP_PATTERNS");
      c->map_pat = !(pe && std::atoi(pe) == 0) &&
                   build_map_patterns(m16, mb, n, c->epw * n, P.n_slots, &c->n_map_pat);
      HIP_TRY(hipMalloc(&c->d_map16, m16.size() * sizeof(uint16_t)));
      HIP_TRY(hipMemcpy(c->d_map16, m16.data(), m16.size() * sizeof(uint16_t),
                        hipMemcpyHostToDevice));
      HIP_TRY(hipMalloc(&c->d_mbase, mb.size() * sizeof(uint32_t)));
      HIP_TRY(hipMemcpy(c->d_mbase, mb.data(), mb.size() * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
      c->map16 = true;
    }
  }
  HIP_TRY(hipMalloc(&c->d_epos, P.epos.size() * sizeof(int)));
  HIP_TRY(hipMemcpy(c->d_epos, P.epos.data(), P.epos.size() * sizeof(int), hipMemcpyHostToDevice));
  c->n_zero = (int64_t)P.zero.size();
  if (c->n_zero) {
    HIP_TRY(hipMalloc(&c->d_zero, P.zero.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(c->d_zero, P.zero.data(), P.zero.size() * sizeof(uint32_t),
                      hipMemcpyHostToDevice));
  }
  c->colour_start = P.colour_start;
  c->seam = P.seam;
  // sem_apply_dot's fused form: every node's final value is one STORE (or a
  // seam sum): no read-modify-write, nothing zeroed separately
  c->seam_dot = !mfma && P.seam && P.n_rmw == 0 && P.zero.empty() && state.empty();
  c->seam_ns = P.seam_ns;
  c->n_seam = (int64_t)P.seam_gid.size();
  (void)hipFree(c->d_ccol);
  (void)hipFree(c->d_seam_gid);
  (void)hipFree(c->d_seam_mask);
  (void)hipFree(c->d_seam_buf);
  c->d_ccol = nullptr;
  c->d_seam_gid = nullptr;
  c->d_seam_mask = nullptr;
  c->d_seam_buf = nullptr;
  if (P.seam) {
    HIP_TRY(hipMalloc(&c->d_ccol, P.chain_colour.size()));
    HIP_TRY(hipMemcpy(c->d_ccol, P.chain_colour.data(), P.chain_colour.size(),
                      hipMemcpyHostToDevice));
    if (c->n_seam) {
      HIP_TRY(hipMalloc(&c->d_seam_gid, c->n_seam * sizeof(uint32_t)));
      HIP_TRY(hipMemcpy(c->d_seam_gid, P.seam_gid.data(), c->n_seam * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
      HIP_TRY(hipMalloc(&c->d_seam_mask, c->n_seam * sizeof(uint16_t)));
      HIP_TRY(hipMemcpy(c->d_seam_mask, P.seam_mask.data(), c->n_seam * sizeof(uint16_t),
                        hipMemcpyHostToDevice));
      // slots addressed by node id (only seam nodes' slots are touched)
      HIP_TRY(hipMalloc(&c->d_seam_buf,
                        (size_t)c->n_node * c->seam_ns * c->dpn * sizeof(double)));
    }
  }
  c->n_atomic_groups = P.n_atomic_groups;
  c->conforming = P.conforming;
  (void)hipFree(c->d_owner);
  c->d_owner = nullptr;
  HIP_TRY(hipMalloc(&c->d_owner, P.owner.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(c->d_owner, P.owner.data(), P.owner.size() * sizeof(uint32_t),
                    hipMemcpyHostToDevice));
  // geometry was derived for the previous map
  for (double*& g : c->d_GP) {
    (void)hipFree(g);
    g = nullptr;
  }
  (void)hipFree(c->d_lin);
  c->d_lin = nullptr;
  c->lin_valid = false;
  c->xg_valid = false;
  c->xg_axi = false;
  return SEM_OK;
}

int sem_plan_info(sem_ctx* c, int64_t* info, int n_info) {
  if (!c || !info || n_info < 1) return fail(SEM_E_INVALID, "bad arguments");
  if (c->ndim == 3) return semh::plan_info(c, info, n_info);
  const int64_t nc = c->colour_start.empty() ? 0 : (int64_t)c->colour_start.size() - 1;
  constexpr int NV = 8 + MAX_COLOURS + 1 + 1 + 1 + 1 + 1 + 1 + 1 + 2 + 1 + 1;
  int64_t vals[NV] = {c->n_groups, c->n_zero, c->n_atomic_groups, c->conforming ? 1 : 0,
                      c->epw,      nc,        c->rounds,          c->n_slots};
  for (int64_t q = 0; q < nc && q <= MAX_COLOURS; ++q)
    vals[8 + q] = c->colour_start[q + 1] - c->colour_start[q];
  vals[NV - 10] = c->mfma ? SEM_KERNEL_MFMA : SEM_KERNEL_COLUMN;
  vals[NV - 9] = c->map16 ? 2 : 4;  // bytes per packed map entry
  // the geometry the Poisson action actually uses: nodal only once x_phys
  // per node exists (sem_set_geom installs stored factors); before any
  // geometry, the mode sem_geom_from_nodes will resolve to
  const bool eff_nodal = c->xg_valid ? true : (c->d_GP[0] ? false : nodal_mode(c));
  vals[NV - 8] = eff_nodal ? SEM_GEOM_NODAL : SEM_GEOM_STORED;
  // plan: 0 chains (colour launches), 1 element-coloured chains, 2 elements
  // (MFMA kernel), 4 chains + seam sums (3 was the retired one-launch plan),
  // 5 elements + seam sums (n = 17 MFMA kernel)
  vals[NV - 7] = c->mfma ? (c->seam ? 5 : 2) : (c->ecol ? 1 : (c->seam ? 4 : 0));
  // the same for the axisymmetric Stokes block (dofs_per_node = 2)
  const bool axi_nodal =
      c->xg_axi ? true : (c->d_GP[1] ? false : nodal_mode_op(c, SEM_OP_AXISYM_STOKES));
  vals[NV - 6] = c->dpn == 2 ? (axi_nodal ? SEM_GEOM_NODAL : SEM_GEOM_STORED) : 0;
  vals[NV - 5] = c->seam ? c->n_seam : 0;  // seam nodes
  vals[NV - 4] = c->blocks ? 1 : 0;          // block layout
  vals[NV - 3] = c->row_carries;             // entries carried between rounds
  vals[NV - 2] = c->const_d && c->map16 && !c->mfma ? 1 : 0;  // Poisson: D as constants
  vals[NV - 1] = c->map_pat ? c->n_map_pat : 0;  // map pattern table: patterns (0: off)
  for (int i = 0; i < n_info && i < NV; ++i) info[i] = vals[i];
  return SEM_OK;
}

static int geom_common(sem_ctx* c, const double* d_nodes, const double* h_Vinv) {
  if (!c || !d_nodes || !h_Vinv) return fail(SEM_E_INVALID, "null argument");
  if (!c->have_basis) return fail(SEM_E_STATE, "sem_set_basis must precede geometry");
  if (!c->d_e2n) return fail(SEM_E_STATE, "sem_set_map must precede geometry");
  HIP_TRY(hipMemcpy(c->d_Vinv, h_Vinv, sizeof(double) * c->n * c->n, hipMemcpyHostToDevice));
  return SEM_OK;
}

int sem_set_geom_mode(sem_ctx* c, int mode) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  if (mode != SEM_GEOM_STORED && mode != SEM_GEOM_NODAL && mode != SEM_GEOM_AUTO)
    return fail(SEM_E_INVALID, "unknown geometry mode " + std::to_string(mode));
  if (c->ndim == 3 && mode == SEM_GEOM_NODAL)
    return fail(SEM_E_NOTIMPL, "hexahedra: stored geometric factors only");
  c->geom_mode = mode;
  c->epoch++;
  return SEM_OK;
}

int sem_set_reynolds(sem_ctx* c, double re) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  if (!std::isfinite(re)) return fail(SEM_E_INVALID, "Reynolds number must be finite");
  c->reynolds = re;
  c->epoch++;
  c->lin_valid = false;  // a recorded linearisation belongs to the old Re
  return SEM_OK;
}

int sem_set_kernel(sem_ctx* c, int kernel) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  if (kernel != SEM_KERNEL_COLUMN && kernel != SEM_KERNEL_MFMA && kernel != SEM_KERNEL_AUTO)
    return fail(SEM_E_INVALID, "unknown kernel " + std::to_string(kernel));
  if (kernel == SEM_KERNEL_MFMA && c->ndim == 3)
    return fail(SEM_E_NOTIMPL, "hexahedra: column kernel only");
  if (kernel == SEM_KERNEL_MFMA && (c->dpn != 1 || c->n > 17))
    return fail(SEM_E_NOTIMPL, "the MFMA kernel needs dofs_per_node == 1 and p <= 16");
  c->kernel = kernel;
  c->epoch++;
  return SEM_OK;
}

int sem_geom_from_nodes(sem_ctx* c, const double* d_nodes, const double* h_Vinv, int op_kind,
                        int64_t* n_bad_nodes, void* stream) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  DeviceGuard g(c->device);
  int rc = geom_common(c, d_nodes, h_Vinv);
  if (rc) return rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if (c->ndim == 3) return semh::geom_from_nodes(c, d_nodes, op_kind, n_bad_nodes, S(stream));
  const bool nodal = nodal_mode_op(c, op_kind);
  c->epoch++;
  double* GP = nullptr;
  if (nodal) {
    if (!c->d_XG) HIP_TRY(hipMalloc(&c->d_XG, c->n_node * sizeof(double2)));
    // stale stored factors would otherwise survive for sem_diag
    (void)hipFree(c->d_GP[gp_slot(op_kind)]);
    c->d_GP[gp_slot(op_kind)] = nullptr;
  } else {
    if ((rc = ensure_gp(c, op_kind, S(stream)))) return rc;
    GP = c->d_GP[gp_slot(op_kind)];
  }
  hipStream_t st = S(stream);
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  if (nodal) HIP_TRY(hipMemsetAsync(c->d_XG, 0, c->n_node * sizeof(double2), st));
  SEM_DISPATCH_N(rc, c->n, launch_geom_n, c, d_nodes, op_kind, GP, nullptr, nullptr, nullptr,
                 nullptr, nullptr, nodal ? c->d_XG : nullptr, nullptr, st);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, c->d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (n_bad_nodes) *n_bad_nodes = (int64_t)bad;
  if (bad) return fail(SEM_E_DETJ, "detJ <= 0 at " + std::to_string(bad) + " quadrature nodes");
  // x_phys per node is one array for the mesh: recomputed here, from these
  // nodes, for every operator that reads it
  if (op_kind == SEM_OP_POISSON) c->xg_valid = nodal;
  if (op_kind == SEM_OP_AXISYM_STOKES) c->xg_axi = nodal;
  if (gp_slot(op_kind) == 2) c->lin_valid = false;  // linearisation used the old factors
  return SEM_OK;
}

int sem_geom_from_xphys(sem_ctx* c, const double* d_xphys, int op_kind, int64_t* n_bad_nodes,
                        void* stream) {
  if (!c || !d_xphys) return fail(SEM_E_INVALID, "null argument");
  if (c->ndim == 3) return fail(SEM_E_NOTIMPL, "sem_geom_from_xphys: quadrilaterals only");
  if (!c->have_basis) return fail(SEM_E_STATE, "sem_set_basis must precede geometry");
  if (!c->d_e2n) return fail(SEM_E_STATE, "sem_set_map must precede geometry");
  DeviceGuard g(c->device);
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  hipStream_t st = S(stream);
  c->epoch++;
  if ((rc = ensure_gp(c, op_kind, st))) return rc;
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  SEM_DISPATCH_N(rc, c->n, launch_geom_n, c, nullptr, op_kind, c->d_GP[gp_slot(op_kind)], nullptr,
                 nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, st, d_xphys);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, c->d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (n_bad_nodes) *n_bad_nodes = (int64_t)bad;
  if (bad) return fail(SEM_E_DETJ, "detJ <= 0 at " + std::to_string(bad) + " quadrature nodes");
  // the stored factors take over from any x_phys per node
  if (op_kind == SEM_OP_POISSON) c->xg_valid = false;
  if (op_kind == SEM_OP_AXISYM_STOKES) c->xg_axi = false;
  if (gp_slot(op_kind) == 2) c->lin_valid = false;
  return SEM_OK;
}

int sem_geom_fields(sem_ctx* c, const double* d_nodes, const double* h_Vinv, double* x_phys,
                    double* J, double* invJ, double* detJ, double* detJxW, void* stream) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  DeviceGuard g(c->device);
  int rc = geom_common(c, d_nodes, h_Vinv);
  if (rc) return rc;
  hipStream_t st = S(stream);
  if (c->ndim == 3) return semh::geom_fields(c, d_nodes, x_phys, J, invJ, detJ, detJxW, st);
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  SEM_DISPATCH_N(rc, c->n, launch_geom_n, c, d_nodes, SEM_OP_POISSON, nullptr, x_phys, J, invJ,
                 detJ, detJxW, nullptr, nullptr, st);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  return SEM_OK;
}

int sem_set_geom(sem_ctx* c, const double* d_G, int op_kind, void* stream) {
  if (!c || !d_G) return fail(SEM_E_INVALID, "null argument");
  if (c->ndim == 3) {
    DeviceGuard g(c->device);
    return semh::set_geom(c, d_G, op_kind, S(stream));
  }
  if (!c->d_epos) return fail(SEM_E_STATE, "sem_set_map must precede sem_set_geom");
  DeviceGuard g(c->device);
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if ((rc = ensure_gp(c, op_kind, S(stream)))) return rc;
  const int ncomp = sem_op_ncomp(op_kind);
  c->epoch++;
  if (op_kind == SEM_OP_POISSON) c->xg_valid = false;  // caller's factors take over
  if (op_kind == SEM_OP_AXISYM_STOKES) c->xg_axi = false;
  hipLaunchKernelGGL(k_pack_geom, dim3(grid_for(c->n_elem * ncomp * c->n * c->n)), dim3(BLOCK), 0,
                     S(stream), d_G, c->n_elem, c->n, ncomp, c->epw, c->d_epos,
                     c->d_GP[gp_slot(op_kind)]);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_zero_shared(sem_ctx* c, double* y, void* stream) {
  if (!c || !y) return fail(SEM_E_INVALID, "null argument");
  if (c->ndim == 3) {
    DeviceGuard g(c->device);
    return semh::zero_shared(c, y, S(stream));
  }
  if (!c->d_mapP) return fail(SEM_E_STATE, "map must be set");
  DeviceGuard g(c->device);
  if (c->n_zero)
    hipLaunchKernelGGL(k_zero_list, dim3(grid_for(c->n_zero, BLOCK, 4096)), dim3(BLOCK), 0,
                       S(stream), y, c->d_zero, c->n_zero, c->dpn);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_apply(sem_ctx* c, int op_kind, const double* u, double* y, int flags, void* stream) {
  if (!c || !u || !y) return fail(SEM_E_INVALID, "null argument");
  {  // the kernels read u while other workgroups write y (both __restrict__)
    const size_t nb = (size_t)c->n_node * c->dpn * sizeof(double);
    const char *a = reinterpret_cast<const char*>(u), *b = reinterpret_cast<const char*>(y);
    if (a < b + nb && b < a + nb) return fail(SEM_E_INVALID, "sem_apply: u and y overlap");
  }
  if (flags & ~(SEM_APPLY_ACCUMULATE | SEM_APPLY_SKIP_ZERO | SEM_APPLY_LINEARIZE))
    return fail(SEM_E_INVALID, "unknown sem_apply flags");
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if (c->ndim == 3) {
    DeviceGuard g(c->device);
    return semh::apply(c, op_kind, u, y, flags, S(stream));
  }
  if (!c->have_basis || !c->d_mapP) return fail(SEM_E_STATE, "basis and map must be set");
  if (!use_nodal(c, op_kind) && !c->d_GP[gp_slot(op_kind)])
    return fail(SEM_E_STATE, "geometry for this operator has not been computed");
  const bool lin = flags & SEM_APPLY_LINEARIZE;
  if (lin && op_kind != SEM_OP_AXISYM_NS)
    return fail(SEM_E_INVALID, "SEM_APPLY_LINEARIZE applies to SEM_OP_AXISYM_NS only");
  if (op_kind == SEM_OP_AXISYM_NS_JVP && !c->lin_valid)
    return fail(SEM_E_STATE, "no linearisation: apply SEM_OP_AXISYM_NS with SEM_APPLY_LINEARIZE first");
  if (lin && !c->d_lin) {
    HIP_TRY(hipMalloc(&c->d_lin, (size_t)c->n_slots * 5 * c->n * c->lw * sizeof(double)));
    c->epoch++;
  }
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  const int accumulate = flags & SEM_APPLY_ACCUMULATE;
  if (!accumulate && !(flags & SEM_APPLY_SKIP_ZERO) && c->n_zero)
    hipLaunchKernelGGL(k_zero_list, dim3(grid_for(c->n_zero, BLOCK, 4096)), dim3(BLOCK), 0, st, y,
                       c->d_zero, c->n_zero, c->dpn);
  SEM_DISPATCH_N(rc, c->n, launch_apply_n, c, op_kind, u, y, accumulate, lin, st, nullptr);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  if (lin) c->lin_valid = true;
  return SEM_OK;
}

int sem_apply_dot(sem_ctx* c, int op_kind, const double* u, double* y, double* d_dot,
                  void* stream) {
  if (!c || !d_dot) return fail(SEM_E_INVALID, "null argument");
  if (!(c->seam_dot && op_kind == SEM_OP_POISSON && c->dpn == 1)) {
    // no fused form on this plan: the action, then a separate u.y pass
    int rc = sem_apply(c, op_kind, u, y, 0, stream);
    if (rc) return rc;
    DeviceGuard g(c->device);
    hipStream_t st = S(stream);
    const int64_t n = c->n_node * c->dpn;
    const int nb = grid_for(n, BLOCK, 2048);
    if ((rc = ensure_dot(c, nb))) return rc;
    hipLaunchKernelGGL(k_dot_plain, dim3(nb), dim3(BLOCK), 0, st, u, y, n, c->d_dot);
    hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(DOT_FIN_THREADS), 0, st, c->d_dot, (int64_t)nb,
                       c->d_dot, (int64_t)0, d_dot);
    HIP_TRY(hipGetLastError());
    return SEM_OK;
  }
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if (!c->have_basis || !c->d_mapP) return fail(SEM_E_STATE, "basis and map must be set");
  if (!use_nodal(c, op_kind) && !c->d_GP[gp_slot(op_kind)])
    return fail(SEM_E_STATE, "geometry for this operator has not been computed");
  {
    const size_t nb = (size_t)c->n_node * sizeof(double);
    const char *a = reinterpret_cast<const char*>(u), *b = reinterpret_cast<const char*>(y);
    if (a < b + nb && b < a + nb) return fail(SEM_E_INVALID, "sem_apply_dot: u and y overlap");
  }
  DeviceGuard g(c->device);
  const int64_t nch = c->colour_start.back() - c->colour_start.front();
  if ((rc = ensure_dot(c, nch + seam_sum_blocks(c)))) return rc;
  SEM_DISPATCH_N(rc, c->n, launch_apply_n, c, op_kind, u, y, 0, false, S(stream), d_dot);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_vec_add(double* dst, const double* src, int64_t n, void* stream) {
  if (n < 0 || (n && (!dst || !src))) return fail(SEM_E_INVALID, "bad arguments");
  if (!n) return SEM_OK;
  hipLaunchKernelGGL(k_vec_add, dim3(grid_for(n)), dim3(BLOCK), 0, S(stream), dst, src, n);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_diag(sem_ctx* c, int op_kind, double* d_diag, void* stream) {
  if (!c || !d_diag) return fail(SEM_E_INVALID, "null argument");
  if (op_kind != SEM_OP_POISSON) return fail(SEM_E_NOTIMPL, "sem_diag: Poisson only");
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if (c->ndim == 3) {
    DeviceGuard g(c->device);
    return semh::diag(c, op_kind, d_diag, S(stream));
  }
  if (!c->d_mapP || !(c->d_GP[0] || use_nodal(c, op_kind)))
    return fail(SEM_E_STATE, "geometry/map not set");
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  if (!c->d_GP[0]) {  // NODAL mode: derive the stored factors once from x_phys per node
    if ((rc = ensure_gp(c, op_kind, st))) return rc;
    SEM_DISPATCH_N(rc, c->n, launch_geom_n, c, nullptr, SEM_OP_POISSON, c->d_GP[0], nullptr,
                   nullptr, nullptr, nullptr, nullptr, nullptr, c->d_XG, st);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemsetAsync(d_diag, 0, c->n_node * sizeof(double), st));
  hipLaunchKernelGGL(k_poisson_diag, dim3(grid_for(c->n_elem * c->n * c->n)), dim3(BLOCK), 0, st,
                     c->d_mapP, c->d_GP[0], c->d_epos, c->d_D, c->n, c->epw, c->n_elem, d_diag);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_assemble(sem_ctx* c, const double* vals, double* out, int accumulate, void* stream) {
  if (!c || !vals || !out) return fail(SEM_E_INVALID, "null argument");
  if (c->ndim == 3) {
    DeviceGuard g(c->device);
    return semh::assemble(c, vals, out, accumulate, S(stream));
  }
  if (!c->d_e2n) return fail(SEM_E_STATE, "sem_set_map must precede sem_assemble");
  if (c->dpn != 1) return fail(SEM_E_INVALID, "sem_assemble: dofs_per_node == 1 only");
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  if (!accumulate) HIP_TRY(hipMemsetAsync(out, 0, c->n_node * sizeof(double), st));
  const int64_t total = c->n_elem * c->n * c->n;
  hipLaunchKernelGGL(k_assemble, dim3(grid_for(total)), dim3(BLOCK), 0, st, c->d_e2n, vals, total,
                     out);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_gather(const double* src, const uint32_t* idx, int64_t n, double* dst, void* stream) {
  if (n < 0 || (n && (!src || !idx || !dst))) return fail(SEM_E_INVALID, "bad arguments");
  if (!n) return SEM_OK;
  hipLaunchKernelGGL(k_gather, dim3(grid_for(n)), dim3(BLOCK), 0, S(stream), src, idx, n, dst);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_scatter_add(double* dst, const uint32_t* idx, int64_t n, const double* src, void* stream) {
  if (n < 0 || (n && (!src || !idx || !dst))) return fail(SEM_E_INVALID, "bad arguments");
  if (!n) return SEM_OK;
  hipLaunchKernelGGL(k_scatter_add, dim3(grid_for(n)), dim3(BLOCK), 0, S(stream), dst, idx, n, src);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_tensor_apply(int n, int64_t batch, const double* h_A0, const double* h_A1,
                     const double* d_in, double* d_out, void* stream) {
  if (n < 1 || n > SEM_MAXN || batch < 0 || (batch && (!d_in || !d_out)))
    return fail(SEM_E_INVALID, "sem_tensor_apply: bad arguments");
  if (!batch) return SEM_OK;
  hipStream_t st = S(stream);
  double* dA = nullptr;
  HIP_TRY(hipMallocAsync((void**)&dA, 2 * n * n * sizeof(double), st));
  if (h_A0) HIP_TRY(hipMemcpyAsync(dA, h_A0, n * n * sizeof(double), hipMemcpyHostToDevice, st));
  if (h_A1)
    HIP_TRY(hipMemcpyAsync(dA + n * n, h_A1, n * n * sizeof(double), hipMemcpyHostToDevice, st));
  const int grid = (int)std::min<int64_t>(batch, 4096);
  hipLaunchKernelGGL(k_tensor_apply, dim3(grid), dim3(BLOCK), 0, st, n, batch,
                     h_A0 ? dA : nullptr, h_A1 ? dA + n * n : nullptr, d_in, d_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipFreeAsync(dA, st));
  return SEM_OK;
}

int sem_det_inv_2x2(int64_t n, const double* d_mat, double* d_det, double* d_inv, void* stream) {
  if (n < 0 || (n && (!d_mat || !d_det || !d_inv))) return fail(SEM_E_INVALID, "bad arguments");
  if (!n) return SEM_OK;
  hipLaunchKernelGGL(k_det_inv_2x2, dim3(grid_for(n)), dim3(BLOCK), 0, S(stream), n, d_mat, d_det,
                     d_inv);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

}  // extern "C"

namespace sem {
int ctx_seam_pack(sem_ctx* c, double* y, double* send, const uint32_t* sidx, const int32_t* sj,
                  int64_t ne, hipStream_t st) {
  const int64_t tot = c->n_seam + ne;
  if (!tot) return SEM_OK;
  const dim3 g(semd::grid_for(tot)), b(BLOCK);
  switch (c->seam_ns) {
#define SEAM_PACK(K)                                                                        \
  case K:                                                                                 \
    hipLaunchKernelGGL(k_seam_pack<K>, g, b, 0, st, y, c->d_seam_gid, c->d_seam_mask,      \
                       c->n_seam, c->d_seam_buf, c->n_node, send, sidx, sj, ne);          \
    break;
    SEAM_PACK(1) SEAM_PACK(2) SEAM_PACK(3) SEAM_PACK(4) SEAM_PACK(5) SEAM_PACK(6) SEAM_PACK(7)
    SEAM_PACK(8)
#undef SEAM_PACK
    default:
      return fail(SEM_E_STATE, "seam plan with more than 8 colours");
  }
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int ctx_seam_finish(sem_ctx* c, double* y, const DDFinish& f, hipStream_t st) {
  const int64_t tot = (f.sel ? f.n_sel : c->n_seam) + (f.skip_rest ? 0 : f.n_rest) +
                      (f.skip_zero ? 0 : f.nz);
  if (!tot) return SEM_OK;
  const dim3 g(semd::grid_for(tot)), b(BLOCK);
  switch (c->seam_ns) {
#define SEAM_FIN(K)                                                                         \
  case K:                                                                                 \
    hipLaunchKernelGGL(k_seam_dd_finish<K>, g, b, 0, st, y, c->d_seam_gid, c->d_seam_mask, \
                       c->n_seam, c->d_seam_buf, c->n_node, f);                           \
    break;
    SEAM_FIN(1) SEAM_FIN(2) SEAM_FIN(3) SEAM_FIN(4) SEAM_FIN(5) SEAM_FIN(6) SEAM_FIN(7)
    SEAM_FIN(8)
#undef SEAM_FIN
    default:
      return fail(SEM_E_STATE, "seam plan with more than 8 colours");
  }
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}
}  // namespace sem
