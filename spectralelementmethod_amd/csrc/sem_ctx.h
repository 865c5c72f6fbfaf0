// Operator context of libsem_hip.so and the helpers shared by the C ABI
// (sem_device.hip) and the per-order launch units (sem_launch.hip, compiled
// once per range of orders so the kernel instantiations build in parallel).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "sem_internal.h"
#include "sem_kernels.h"

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return sem::fail(SEM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));  \
  } while (0)

using semk::BLOCK;

constexpr int MAX_COLOURS = 8;  // + one trailing all-atomic class
// AUTO choice of the seam plan (Poisson column kernel), from the MI355X A/B
// of profiles/r02/seams2 (ms per action, colour launches -> seams; cpc =
// chains per colour): it wins where a colour launch is a few generations of
// resident workgroups or less -- p = 16 198^2 (cpc 1,633) 0.164 -> 0.134,
// p = 12 263^2 0.139 -> 0.114, p = 10 316^2 (1,296) 0.158 -> 0.128, p = 9
// 351^2 (1,297) 0.120 -> 0.113, p = 8 512^2 (2,342) 0.185 -> 0.179, 384^2
// (1,372) 0.107 -> 0.095, 128 x 1024 (1,171; one rank's strip of the
// 8-GPU split) 0.098 -> 0.089, 256^2 (585) 0.0635 -> 0.0477, p = 6 256^2
// (488) 0.040 -> 0.030, p = 4 395^2 (815) 0.045 -> 0.036 -- and loses where
// the colour launches stream many generations and the seams are a large
// share of the nodes: p = 8 1024^2 (9,365) 0.640 -> 0.668, p = 6 527^2
// (1,928) 0.118 -> 0.122, p = 4 790^2 (3,250) 0.113 -> 0.129, p = 2 1581^2
// 0.132 -> 0.161.
// Two DOFs per node (axisymmetric block, p = 6, profiles/r02/final/
// axisym_seams): 128^2 (cpc 114) 0.0441 -> 0.0236, 512^2 (cpc 1,820) 0.227
// -> 0.274 (the nodal kernel's seam instantiation runs 1 wave per SIMD
// instead of 2).
// AUTO of the block layout (sem_device.hip groups_blocks, 4 rounds): only
// where the mesh still has this many chains with it.  Measured on MI355X,
// ms per action, consecutive groups -> blocks (profiles/r03/sweep): the
// axisymmetric Stokes block at 512^2, p = 6 (1,920 block chains) 0.302 ->
// 0.257; Poisson p = 8 1024^2 (9,472) 0.684 -> 0.671, 395^2 (1,481) 0.106
// -> 0.107, p = 6 527^2 (1,980) 0.118 -> 0.122, p = 12 263^2 0.132 ->
// 0.151, p = 16 198^2 0.139 -> 0.188, 256^2 p = 8 0.046 -> 0.056.
inline int64_t block_min_chains(int n, int dpn) {
  (void)n;
  return dpn == 2 ? 1024 : 4096;
}
inline bool seam_auto(int n, int64_t chains_per_colour, int dpn = 1, bool blocks = false) {
  // block layout: the seams are a few % of the nodes (every R-th node row and
  // every 4*EPW-th column) -- 1024^2 p = 8: R = 4 seams 0.671, colours 0.692,
  // consecutive groups 0.684 ms (profiles/r03/blocks_ab.txt)
  if (blocks && dpn == 1) return true;
  if (dpn == 2) return chains_per_colour <= 512;
  // n = 7 (p = 6 at 527^2, 1,929 chains per colour; profiles/r04/p6/):
  // nodal seams 0.099-0.100 against nodal colours 0.106-0.111 and stored
  // colours 0.118-0.120 ms per action; stored seams 0.116-0.118
  return n >= 11 || chains_per_colour <= 1024 || ((n >= 9 || n == 7) && chains_per_colour <= 2400);
}

struct HexState;  // the 3-D (hexahedral) path, sem_hex.hip

struct sem_ctx {
  int p = 0, n = 0, dpn = 1, device = 0;
  int ndim = 2;              // 3: hexahedra, every entry point forwards to semh::
  HexState* hex = nullptr;
  int64_t n_elem = 0, n_node = 0;
  int epw = 0, lw = 0;
  int64_t n_groups = 0;
  double hD[SEM_MAXN * SEM_MAXN];
  double hw[SEM_MAXN];
  bool have_basis = false;
  double* d_D = nullptr;
  double* d_w = nullptr;
  double* d_Vinv = nullptr;
  double* d_deo = nullptr;  // even-odd D for n >= SEM_D_SCALAR_LOAD_N (scalar loads)
  uint32_t* d_mapP = nullptr;   // packed coded map, launch (colour) order
  uint16_t* d_map16 = nullptr;  // the same map as 16-bit row offsets (column kernel)
  uint32_t* d_mbase = nullptr;  // their per-(slot, row) 32-bit bases
  bool map16 = false;
  bool map_pat = false;   // d_map16 is a pattern table (MapRef::pat)
  int64_t n_map_pat = 0;
  int* d_epos = nullptr;         // element -> packed position slot * epw + k
  const uint32_t* d_e2n = nullptr;
  uint32_t* d_zero = nullptr;    // y entries no kernel stores first (unreferenced / first-atomic)
  int64_t n_zero = 0;
  int rounds = 1;                     // rounds of 4 groups per chain (workgroup)
  int64_t n_slots = 0;                // packed group slots = chains * 4 * rounds
  std::vector<int64_t> colour_start;  // chain ranges, one launch each
  int64_t n_atomic_groups = 0;        // groups in atomic-fallback chains
  bool conforming = true;
  double* d_GP[3] = {nullptr, nullptr, nullptr};  // Poisson, axisym. Stokes, Navier-Stokes
  double reynolds = 0.0;
  double* d_lin = nullptr;  // Navier-Stokes linearisation, 5 per element node
  bool lin_valid = false;
  // NODAL geometry (Poisson): x_phys per global node + the node's first element
  int geom_mode = SEM_GEOM_AUTO;
  // kernel family of the Poisson action (sem_set_kernel), fixed by
  // sem_set_map: the LDS column kernel or the fp64-MFMA element kernel (they
  // need different plans and packed layouts)
  int kernel = SEM_KERNEL_AUTO;
  bool mfma = false;
  // D is the standard GLL D of deo_const.h bit for bit: the Poisson column
  // kernels take it as compile-time constants (SEM_CONST_D=0 disables)
  bool const_d = false;
  bool ecol = false;  // column kernel on the element-coloured plan
  double2* d_XG = nullptr;
  uint32_t* d_owner = nullptr;
  bool xg_valid = false;  // the Poisson action reads d_XG
  bool xg_axi = false;    // the axisymmetric Stokes action reads d_XG
  unsigned long long* d_bad = nullptr;
  // seam plan of the Poisson column kernel (SeamPlan, sem_kernels.h)
  bool blocks = false;       // block layout of the chains (groups_blocks)
  int64_t row_carries = 0;
  bool round_sync = true;  // a chain writes some node in two rounds (Plan::round_rmw)
  bool seam = false;
  bool seam_dot = false;    // sem_apply_dot fuses u.y into the seam plan's launches
  bool defer_seam_sum = false;  // sem_apply leaves the seam sum to the caller (sem_dd's fused finish)
  double* d_dot = nullptr;  // u.y partials of sem_apply_dot (chains + seam-sum blocks)
  int64_t n_dot = 0;
  int seam_ns = 0;
  int64_t n_seam = 0;
  uint8_t* d_ccol = nullptr;
  uint32_t* d_seam_gid = nullptr;
  uint16_t* d_seam_mask = nullptr;
  double* d_seam_buf = nullptr;
  uint64_t epoch = 0;      // sem::ctx_epoch
  uint64_t map_epoch = 0;  // sem::ctx_map_epoch (sem_set_map_shared only)
  int n_cu = 0;        // compute units of `device` (persistent launches), 0 = not queried
};

namespace semd {
using namespace semk;

inline int grid_for(int64_t n, int per_block = BLOCK, int cap = 8192) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}


struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// even-odd halves of D (row-major h[m*N + r]); see DEO in sem_kernels.h
template <int N>
DEOData<N> make_deo_data(const double* h) {
  DEOData<N> d;
  constexpr int H = N / 2;
  for (int m = 0; m < H; ++m)
    for (int r = 0; r < H; ++r) {
      d.P[m * H + r] = 0.5 * (h[m * N + r] - h[m * N + N - 1 - r]);
      d.Q[m * H + r] = 0.5 * (h[m * N + r] + h[m * N + N - 1 - r]);
    }
  if (DEOData<N>::C)
    for (int m = 0; m < H; ++m) {
      d.cc[m] = h[m * N + H];
      d.rr[m] = h[H * N + m];
    }
  if (DEOData<N>::TR)
    for (int m = 0; m < H; ++m)
      for (int q = 0; q < H; ++q) {
        d.PT[q * H + m] = d.P[m * H + q];
        d.QT[q * H + m] = d.Q[m * H + q];
      }
  return d;
}

template <int N>
DEO<N> make_deo(const sem_ctx* c) {
  DEO<N> a;
  if constexpr (N >= SEM_D_SCALAR_LOAD_N)
    a.p = reinterpret_cast<const DEOData<N>*>(c->d_deo);
  else
    a.d = make_deo_data<N>(c->hD);
  return a;
}


// AUTO geometry of the column kernel, per order from the MI355X sweep at
// ~1e7 DOF (profiles/r01c/geosweep): NODAL (factors
// re-derived from x_phys per node) at p = 1, 2, 4, 5, 8, STORED at p = 3, 6,
// 7 and above 8.  The p = 3, 5, 6 picks are within 2-3 % (one run each);
// the clear wins are p = 2, 4, 8 (nodal) and p >= 9 (stored).
// Round 4: p = 6 (n = 7) nodal -- on the seam plan 0.099-0.100 against 0.116-0.118
// ms stored (527^2, profiles/r04/p6/).
inline bool auto_nodal_order(int n) {
  return n == 2 || n == 3 || n == 5 || n == 6 || n == 7 || n == 9;
}

// Orders whose Poisson column kernels run with D as compile-time constants
// when the basis is the standard GLL one (sem_set_basis):
// measured per order on MI355X at ~1e7 DOF (profiles/r04/const_d/, kernel
// median ms per action, argument form -> constants): p = 10 0.119 -> 0.108,
// 12 0.126 -> 0.123, 14 0.131 -> 0.123, 16 0.140 -> 0.122 (machine LICM
// off for that unit), every order from p = 10 2-13 % faster; p = 6 (LICM
// off) 0.102-0.105 -> 0.099; p = 9 with a 5-wave request 0.114 -> 0.112;
// p = 4 and p = 8 (nodal) 17-19 % slower (the hoisted constants spill), the
// other low orders within 1-2 %.
inline bool const_d_order(int n) { return n == 7 || n >= 10; }

inline bool nodal_mode(const sem_ctx* c) {
  if (c->mfma) return c->geom_mode == SEM_GEOM_NODAL;  // AUTO: stored factors
  return c->geom_mode == SEM_GEOM_NODAL ||
         (c->geom_mode == SEM_GEOM_AUTO && auto_nodal_order(c->n));
}

// AUTO: the MFMA element kernel from SEM_MFMA_MIN_N nodes per line up,
// Poisson only (dpn = 1), one 16 x 16 tile (n <= 16), and not when nodal
// geometry was requested explicitly.  Round 1 measured it ahead of the
// column kernel on colour launches at p = 13..15 (profiles/r01c/geosweep);
// the column kernel on the seam plan is ahead at every order (MI355X, ~1e7
// DOF, ms per action, MFMA / column: p = 10 0.160 / 0.126, p = 13 0.147 /
// 0.129, p = 14 0.143 / 0.141, p = 15 0.142 / 0.112; profiles/r02/final),
// so AUTO no longer picks it (SEM_KERNEL_MFMA still does).
#ifndef SEM_MFMA_MIN_N
#define SEM_MFMA_MIN_N 18
#endif
inline bool want_mfma(const sem_ctx* c) {
  if (c->dpn != 1 || c->n > 17) return false;
  if (c->kernel == SEM_KERNEL_MFMA) return true;
  if (c->kernel == SEM_KERNEL_COLUMN) return false;
  return c->n >= SEM_MFMA_MIN_N && c->geom_mode != SEM_GEOM_NODAL;
}

// axisymmetric Stokes block (dpn = 2, column kernel only): AUTO picks NODAL
// where it measured faster at ~9.4e6 nodes (DESIGN.md §4.2,
// profiles/r02/axisym): p = 2 / 4 / 6 0.226 / 0.192 / 0.214 ms against
// 0.367 / 0.306 / 0.305 stored, p = 16 0.428 vs 0.481; STORED at p = 8..12
// (0.275 vs 0.286 at p = 8, 0.286 vs 0.421 at p = 10: the nodal kernel's
// register demand drops it to one wave per SIMD).  Unmeasured orders follow
// their neighbours.
inline bool auto_nodal_axi_order(int n) { return n <= 7 || n == 17; }

inline bool nodal_mode_op(const sem_ctx* c, int op_kind) {
  if (op_kind == SEM_OP_POISSON) return nodal_mode(c);
  if (op_kind == SEM_OP_AXISYM_STOKES)
    return c->geom_mode == SEM_GEOM_NODAL ||
           (c->geom_mode == SEM_GEOM_AUTO && auto_nodal_axi_order(c->n));
  return false;  // Navier-Stokes: stored factors
}

inline bool use_nodal(const sem_ctx* c, int op_kind) {
  if (op_kind == SEM_OP_POISSON) return nodal_mode(c) && c->xg_valid;
  if (op_kind == SEM_OP_AXISYM_STOKES) return nodal_mode_op(c, op_kind) && c->xg_axi;
  return false;
}

// per-order entry points (sem_launch.hip)
// dot_out (device scalar, may be null): also u.y, fused into the seam plan's
// launches (the caller guarantees: seam plan, Poisson, overwrite)
template <int N>
int launch_apply_n(sem_ctx* c, int op_kind, const double* u, double* y, int acc, bool lin,
                   hipStream_t st, double* dot_out);
template <int N>
int launch_geom_n(sem_ctx* c, const double* nodes, int op_kind, double* GP, double* xph,
                  double* J, double* iJ, double* dJ, double* dJW, double2* XG,
                  const double2* XGin, hipStream_t st, const double* XEin = nullptr);
template <int N>
int upload_deo(sem_ctx* c);
// one launch of the Poisson column kernel with D as compile-time constants
// (16-bit map; sem_launch_cd.hip, a translation unit of its own so that its
// compiler flags are chosen per order, csrc/../_build.py)
struct PoissonLaunch {
  dim3 g, b;
  hipStream_t st;
  MapRef mr;
  const double* GP;
  const double2* XG;
  const double* u;
  double* y;
  int64_t c0, c1;
  int rounds, acc;
  SeamPlan sp;
};
template <int N>
void launch_poisson_const_d(const PoissonLaunch& L, bool nodal, bool seam, bool dot,
                            const WVec<N>& w, bool pat = false);
// the seam sums of the seam plan (sem_device.hip); du / dot: also the u.y
// partials of the seam nodes, one per block of seam_sum_blocks(c)
int launch_seam_sum(sem_ctx* c, double* y, int acc, hipStream_t st, const double* du = nullptr,
                    double* dot = nullptr);
int64_t seam_sum_blocks(const sem_ctx* c);

#define SEM_DISPATCH_N(rc, n, FN, ...)          \
  switch (n) {                                  \
    case 2: rc = FN<2>(__VA_ARGS__); break;     \
    case 3: rc = FN<3>(__VA_ARGS__); break;     \
    case 4: rc = FN<4>(__VA_ARGS__); break;     \
    case 5: rc = FN<5>(__VA_ARGS__); break;     \
    case 6: rc = FN<6>(__VA_ARGS__); break;     \
    case 7: rc = FN<7>(__VA_ARGS__); break;     \
    case 8: rc = FN<8>(__VA_ARGS__); break;     \
    case 9: rc = FN<9>(__VA_ARGS__); break;     \
    case 10: rc = FN<10>(__VA_ARGS__); break;   \
    case 11: rc = FN<11>(__VA_ARGS__); break;   \
    case 12: rc = FN<12>(__VA_ARGS__); break;   \
    case 13: rc = FN<13>(__VA_ARGS__); break;   \
    case 14: rc = FN<14>(__VA_ARGS__); break;   \
    case 15: rc = FN<15>(__VA_ARGS__); break;   \
    case 16: rc = FN<16>(__VA_ARGS__); break;   \
    case 17: rc = FN<17>(__VA_ARGS__); break;   \
    default: rc = sem::fail(SEM_E_NOTIMPL, "order out of range"); break; \
  }

}  // namespace semd

// the hexahedral (ndim = 3) halves of the C ABI entry points (sem_hex.hip)
namespace semh {
int ctx_init(sem_ctx* c);
void ctx_free(sem_ctx* c);
int set_map(sem_ctx* c, const uint32_t* d_e2n, hipStream_t st);
int geom_from_nodes(sem_ctx* c, const double* d_nodes, int op_kind, int64_t* n_bad,
                    hipStream_t st);
int geom_fields(sem_ctx* c, const double* d_nodes, double* x_phys, double* J, double* invJ,
                double* detJ, double* detJxW, hipStream_t st);
int set_geom(sem_ctx* c, const double* d_G, int op_kind, hipStream_t st);
int apply(sem_ctx* c, int op_kind, const double* u, double* y, int flags, hipStream_t st);
int diag(sem_ctx* c, int op_kind, double* d, hipStream_t st);
int zero_shared(sem_ctx* c, double* y, hipStream_t st);
int plan_info(const sem_ctx* c, int64_t* info, int n_info);
int zero_list(const sem_ctx* c, std::vector<uint32_t>* nodes, bool* only_unreferenced);
int assemble(sem_ctx* c, const double* vals, double* out, int accumulate, hipStream_t st);
}  // namespace semh
