// Domain decomposition of the operator across GPUs (one process per GPU) and
// the device-resident preconditioned CG that runs on one or many of them.
//
// The reference has no parallelism (sem/discrete.py:208-209: one Python loop
// over all elements).  Its element loop is independent per element except
// for the final scatter-add y[loc] += y_e: a node on the boundary between two
// ranks' elements receives contributions from both.  SURVEY.md §8(e).
//
// One rank owns a set of elements and the nodes they touch (local numbering).
// Its elements are split into
//   * interface elements: the ones touching a node shared with another rank,
//     applied by a context (`iface`) over a COMPACT renumbering of just their
//     nodes, into a small private vector y_c, on a side stream;
//   * interior elements: all others, applied by `interior` over the local
//     numbering straight into y, on the caller's stream, concurrently.
// The side stream then sums the shared entries of y_c with the neighbours
// (RCCL send/recv over xGMI, or a caller-supplied transport), and the
// caller's stream finally adds y_c into y.  The interface sum is therefore
// hidden behind the interior elements, and no kernel ever waits for the
// small interface launches.  Only shared entries travel: 8 B per shared DOF
// and direction, never the full vector.
//
//   main:  ev0 ------------- interior apply (u -> y) ------------- wait ev1, finish
//   side:  wait ev0, iface apply (u -> y_c), pack, exchange, ev1
//
// The interface context may number its nodes like the rank (local
// numbering, what distributed.py builds: it reads u directly and writes a
// rank-sized private y_c of which only its own nodes are ever read) or
// compactly (its own n_iface_dofs; u_c = u[cidx] is gathered first).
//
// finish (k_dd_finish, one launch): y[cidx[j]] += y_c[j] + the neighbours'
// values for compact DOF j, in peer order -- the unpack and the final add of
// one step in one kernel; it also takes over the interior operator's zero
// list (nodes only interface elements touch are overwritten instead of
// zeroed first), so the step enqueues no zero-fill and no unpack launches.
#include <hip/hip_runtime.h>

#include <limits>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sem_internal.h"

using sem::fail;

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(SEM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
  } while (0)

#define NCCL_TRY(expr)                                                                  \
  do {                                                                                  \
    ncclResult_t _r = (expr);                                                           \
    if (_r != ncclSuccess)                                                              \
      return fail(SEM_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r));       \
  } while (0)

#define SEM_TRY(expr)        \
  do {                       \
    int _rc = (expr);        \
    if (_rc) return _rc;     \
  } while (0)

namespace {

constexpr int BLK = 256;
constexpr int WV = 64;
// 512 workgroups (2 per CU, 8 waves per CU) stream the vectors fastest: at
// 1024^2 p = 8 the PCG iteration takes 1.42 ms against 1.46 / 1.50 / 1.54 /
// 1.57-1.66 with 384 / 768 / 1024 / 2048 workgroups and 1.53-1.59 with 256
// (profiles/r05/pcg/grid_ab/): fewer concurrent streams per array
#ifndef SEM_PCG_RED_BLOCKS
#define SEM_PCG_RED_BLOCKS 512
#endif
constexpr int RED_BLOCKS = SEM_PCG_RED_BLOCKS;  // partial sums per dot (fixed: deterministic order)
// The PCG vector kernels stream 5-9 vectors of n doubles per iteration: each
// thread walks the grid-stride sequence UNR entries at a time with all their
// loads issued before any use (memory-level parallelism: one load per array
// in flight per thread measured ~4 TB/s at 67M DOF, round 2).
#ifndef SEM_PCG_UNR
#define SEM_PCG_UNR 4
#endif
constexpr int UNR = SEM_PCG_UNR;

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int grid_for(int64_t n, int cap = 8192) {
  int64_t g = (n + BLK - 1) / BLK;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
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

// ---------------------------------------------------------------- PCG kernels
// DOF flags: bit 0 Dirichlet (row/column removed, x fixed), bit 1 the DOF is
// a copy owned by another rank (left out of the global dot products).
constexpr uint8_t F_DIR = 1, F_NOTOWN = 2;

__device__ double block_sum(double v) {
  __shared__ double sh[BLK / WV];
  for (int o = WV / 2; o > 0; o >>= 1) v += __shfl_down(v, o, WV);
  if ((threadIdx.x & (WV - 1)) == 0) sh[threadIdx.x / WV] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < BLK / WV; ++w) s += sh[w];
  __syncthreads();
  return s;
}

__device__ __forceinline__ void write_partials(double s0, double s1, double* partial) {
  s0 = block_sum(s0);
  s1 = block_sum(s1);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = s0;
    partial[RED_BLOCKS + blockIdx.x] = s1;
  }
}

// flags = dirichlet | (not owned) << 1
__global__ void k_cg_flags(const uint8_t* __restrict__ dir, const uint8_t* __restrict__ notown,
                           int64_t n, uint8_t* __restrict__ f) {
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK)
    f[t] = (dir[t] ? F_DIR : 0) | ((notown && notown[t]) ? F_NOTOWN : 0);
}

// diag -> 1 / diag in place (once per solve: the Jacobi preconditioner is
// then a multiply in the update pass, not an fp64 division per DOF); 0 on
// Dirichlet DOFs, so that z = r * dinv is 0 there without a flag
__global__ void k_cg_invert(double* __restrict__ d, const uint8_t* __restrict__ f, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK)
    d[t] = (f[t] & F_DIR) ? 0.0 : 1.0 / d[t];
}

// The Jacobi preconditioner as the vector passes read it (SEM_PCG_DINV32,
// default): 1 / diag rounded to float, with the DOF flags folded in -- 0 on
// Dirichlet DOFs, negative on DOFs another rank owns (left out of the dots):
// 4 bytes per DOF and pass instead of 8 + 1.  M = diag(float(1 / diag)) is
// still symmetric positive definite, so CG converges to the same solution;
// the iterates are those of that M.
#ifndef SEM_PCG_DINV32
#define SEM_PCG_DINV32 1
#endif
#if SEM_PCG_DINV32
typedef float dinv_t;
#else
typedef double dinv_t;
#endif
__device__ __forceinline__ bool pc_dir(dinv_t d) { return d == (dinv_t)0; }
__device__ __forceinline__ bool pc_own(dinv_t d) { return d >= (dinv_t)0; }
__device__ __forceinline__ double pc_z(double r, dinv_t d) { return r * (double)fabs(d); }

__global__ void k_cg_pack(const double* __restrict__ dinv, const uint8_t* __restrict__ f,
                          int64_t n, dinv_t* __restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK) {
    // |1/diag| outside the float range saturates (a free DOF is never 0, never
    // inf); a NaN diagonal stays NaN, so the solve reports a non-finite
    // residual instead of running on a made-up preconditioner
    dinv_t v = (dinv_t)fabs(dinv[t]);
    if (v == (dinv_t)0 && dinv[t] == dinv[t]) v = std::numeric_limits<dinv_t>::min();
    if (v > std::numeric_limits<dinv_t>::max()) v = std::numeric_limits<dinv_t>::max();
    if (f[t] & F_DIR) v = (dinv_t)0;
    else if (f[t] & F_NOTOWN) v = -v;
    out[t] = v;
  }
}

// r = b - K x on free DOFs (r holds K x on entry), p = z = M r;
// partial sums of r.z and r.r over owned DOFs
__global__ void __launch_bounds__(BLK)
    k_cg_start(const double* __restrict__ b, double* __restrict__ r, const dinv_t* __restrict__ dinv,
               int64_t n, double* __restrict__ p, double* __restrict__ partial) {
  double s0 = 0.0, s1 = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK) {
    const dinv_t dt = dinv[t];
    const double rt = pc_dir(dt) ? 0.0 : b[t] - r[t];
    const double zt = pc_z(rt, dt);
    r[t] = rt;
    p[t] = zt;
    if (pc_own(dt)) {
      s0 = fma(rt, zt, s0);
      s1 = fma(rt, rt, s1);
    }
  }
  write_partials(s0, s1, partial);
}

// V consecutive doubles (V = 2: one 16-byte access) of item i, nontemporal:
// every vector entry is touched once per pass (tools/r03/stream_bench.cpp on
// one MI355X: the residual pass 4.28 -> 4.78 TB/s, the step pass 4.46 ->
// 4.66, against 5.0 TB/s for a plain double2 copy on that box)
template <int V>
__device__ __forceinline__ void ldv(const double* __restrict__ a, int64_t i, double (&o)[V]) {
#pragma unroll
  for (int e = 0; e < V; ++e) o[e] = __builtin_nontemporal_load(a + i * V + e);
}
template <int V>
__device__ __forceinline__ void stv(double* __restrict__ a, int64_t i, const double (&o)[V]) {
#pragma unroll
  for (int e = 0; e < V; ++e) __builtin_nontemporal_store(o[e], a + i * V + e);
}
template <int V>
__device__ __forceinline__ void ldv(const float* __restrict__ a, int64_t i, float (&o)[V]) {
#pragma unroll
  for (int e = 0; e < V; ++e) o[e] = __builtin_nontemporal_load(a + i * V + e);
}
template <int V>
__device__ __forceinline__ void ldf(const uint8_t* __restrict__ f, int64_t i, uint8_t (&o)[V]) {
  if constexpr (V == 2) {
    const uchar2 t = reinterpret_cast<const uchar2*>(f)[i];
    o[0] = t.x;
    o[1] = t.y;
  } else {
    o[0] = f[i];
  }
}

// The vector kernels walk n / V items of V DOFs (16-byte accesses when
// V = 2) in a grid-stride sequence, UNR / V items at a time with every load
// issued before any use; the n % V last DOFs go to thread 0 of block 0.
// partial sums of p.q over owned DOFs (p = 0 on Dirichlet DOFs)
template <int V>
__global__ void __launch_bounds__(BLK)
    k_cg_pq(const double* __restrict__ p, const double* __restrict__ q,
            const uint8_t* __restrict__ f, int64_t n, double* __restrict__ partial) {
  constexpr int U = UNR / V;
  double s0 = 0.0;
  const int64_t nv = n / V, st = (int64_t)gridDim.x * BLK;
  for (int64_t i0 = blockIdx.x * (int64_t)BLK + threadIdx.x; i0 < nv; i0 += U * st) {
    double pv[U][V], qv[U][V];
    uint8_t fv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * st < nv ? i0 + u * st : 0;
      ldv<V>(p, i, pv[u]);
      ldv<V>(q, i, qv[u]);
      ldf<V>(f, i, fv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * st < nv)
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (!(fv[u][e] & F_NOTOWN)) s0 = fma(pv[u][e], qv[u][e], s0);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t t = nv * V; t < n; ++t)
      if (!(f[t] & F_NOTOWN)) s0 = fma(p[t], q[t], s0);
  write_partials(s0, 0.0, partial);
}

__device__ __forceinline__ double cg_alpha(const double* rz_old, const double* pq) {
  const double den = *pq;
  return den != 0.0 ? *rz_old / den : 0.0;
}

// alpha = rz / pq (on the device); r -= alpha q on free DOFs; partial sums of
// r.z and r.r with z = r / diag formed on the fly (not stored: the step
// kernel forms it again from r)
template <int V>
__global__ void __launch_bounds__(BLK)
    k_cg_residual(double* __restrict__ r, const double* __restrict__ q,
                  const dinv_t* __restrict__ dinv, const double* __restrict__ rz_old,
                  const double* __restrict__ pq, int64_t n, double* __restrict__ partial) {
  constexpr int U = UNR / V;
  const double alpha = cg_alpha(rz_old, pq);
  double s0 = 0.0, s1 = 0.0;
  auto one = [&](double qt, double rt, dinv_t dt) {
    rt = pc_dir(dt) ? 0.0 : fma(-alpha, qt, rt);
    if (pc_own(dt)) {
      s0 = fma(rt, pc_z(rt, dt), s0);
      s1 = fma(rt, rt, s1);
    }
    return rt;
  };
  const int64_t nv = n / V, st = (int64_t)gridDim.x * BLK;
  for (int64_t i0 = blockIdx.x * (int64_t)BLK + threadIdx.x; i0 < nv; i0 += U * st) {
    double qv[U][V], rv[U][V];
    dinv_t dv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * st < nv ? i0 + u * st : 0;
      ldv<V>(q, i, qv[u]);
      ldv<V>(r, i, rv[u]);
      ldv<V>(dinv, i, dv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u * st >= nv) continue;
#pragma unroll
      for (int e = 0; e < V; ++e) rv[u][e] = one(qv[u][e], rv[u][e], dv[u][e]);
      stv<V>(r, i0 + u * st, rv[u]);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t t = nv * V; t < n; ++t) r[t] = one(q[t], r[t], dinv[t]);
  write_partials(s0, s1, partial);
}

// the rest of the iteration in one pass, with z = r / diag (0 on Dirichlet
// DOFs: dinv is 0 there) and beta = rz_new / rz_old on the device.
//   STEP_NOW:   x += alpha p, then p = z + beta p (in place);
//   STEP_DEFER: pout = z + beta p, x untouched; alpha saved to *alpha_io;
//   STEP_PAIR:  x += alpha' pout + alpha p (alpha' = *alpha_io, pout = the
//               previous iteration's p), then pout = z + beta p.
// DEFER / PAIR alternate (SEM_PCG_X_PAIRS, default): x is read and written
// every second iteration, 40 instead of 44 bytes per DOF and iteration over
// the two, and x = fma(alpha, p, fma(alpha', p', x)) is bitwise the two
// single updates in order.
enum { STEP_NOW = 0, STEP_DEFER = 1, STEP_PAIR = 2 };
template <int V, int MODE>
__global__ void __launch_bounds__(BLK)
    k_cg_step(double* __restrict__ x, double* __restrict__ p, double* __restrict__ pout,
              const double* __restrict__ r, const dinv_t* __restrict__ dinv,
              const double* __restrict__ rz_new, const double* __restrict__ rz_old,
              const double* __restrict__ pq, double* __restrict__ alpha_io, int64_t n) {
  constexpr int U = UNR / V;
  const double alpha = cg_alpha(rz_old, pq);
  const double alpha_prev = MODE == STEP_PAIR ? *alpha_io : 0.0;
  const double den = *rz_old;
  const double beta = den != 0.0 ? *rz_new / den : 0.0;
  if (MODE == STEP_DEFER && blockIdx.x == 0 && threadIdx.x == 0) *alpha_io = alpha;
  double* dst = MODE == STEP_NOW ? p : pout;
  const int64_t nv = n / V, st = (int64_t)gridDim.x * BLK;
  for (int64_t i0 = blockIdx.x * (int64_t)BLK + threadIdx.x; i0 < nv; i0 += U * st) {
    double xv[U][V], pv[U][V], rv[U][V], av[U][V];
    dinv_t dv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * st < nv ? i0 + u * st : 0;
      if (MODE != STEP_DEFER) ldv<V>(x, i, xv[u]);
      if (MODE == STEP_PAIR) ldv<V>(pout, i, av[u]);
      ldv<V>(p, i, pv[u]);
      ldv<V>(r, i, rv[u]);
      ldv<V>(dinv, i, dv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u * st >= nv) continue;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        if (MODE == STEP_PAIR) xv[u][e] = fma(alpha_prev, av[u][e], xv[u][e]);
        if (MODE != STEP_DEFER) xv[u][e] = fma(alpha, pv[u][e], xv[u][e]);
        pv[u][e] = fma(beta, pv[u][e], pc_z(rv[u][e], dv[u][e]));
      }
      if (MODE != STEP_DEFER) stv<V>(x, i0 + u * st, xv[u]);
      stv<V>(dst, i0 + u * st, pv[u]);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t t = nv * V; t < n; ++t) {
      double xt = MODE != STEP_DEFER ? x[t] : 0.0;
      if (MODE == STEP_PAIR) xt = fma(alpha_prev, pout[t], xt);
      if (MODE != STEP_DEFER) x[t] = fma(alpha, p[t], xt);
      dst[t] = fma(beta, p[t], pc_z(r[t], dinv[t]));
    }
}

// the update of x still owed after a STEP_DEFER iteration: x += alpha' p'
__global__ void __launch_bounds__(BLK)
    k_cg_flush_x(double* __restrict__ x, const double* __restrict__ pp,
                 const double* __restrict__ alpha_io, int64_t n) {
  const double a = *alpha_io;
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK)
    x[t] = fma(a, pp[t], x[t]);
}

// fixed-order sum of the partials: out[0..nd) (deterministic run to run);
// hist (may be null): also record out[1] (the r.r history of a single-GPU
// solve, whose dots need no all-reduce)
__global__ void __launch_bounds__(BLK)
    k_cg_finish(const double* __restrict__ partial, int nb, int nd, double* __restrict__ out,
                double* __restrict__ hist) {
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < nb; i += BLK) {
    s0 += partial[i];
    s1 += partial[RED_BLOCKS + i];
  }
  s0 = block_sum(s0);
  s1 = block_sum(s1);
  if (threadIdx.x == 0) {
    out[0] = s0;
    if (nd > 1) out[1] = s1;
    if (hist) *hist = s1;
  }
}

// history of the (globally reduced) r.r, for the lagged convergence test
__global__ void k_cg_record(const double* __restrict__ rr, double* __restrict__ hist) {
  if (threadIdx.x == 0) *hist = *rr;
}

// y = A x for a CSR matrix (one thread per row; the condensed exterior
// systems of static condensation have a few tens of entries per row)
__global__ void k_csr_spmv(int64_t n, const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                           const double* __restrict__ v, const double* __restrict__ x,
                           double* __restrict__ y) {
  for (int64_t r = blockIdx.x * (int64_t)BLK + threadIdx.x; r < n; r += (int64_t)gridDim.x * BLK) {
    double acc = 0.0;
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) acc = fma(v[k], x[ci[k]], acc);
    y[r] = acc;
  }
}

__global__ void k_csr_diag(int64_t n, const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                           const double* __restrict__ v, double* __restrict__ d) {
  for (int64_t r = blockIdx.x * (int64_t)BLK + threadIdx.x; r < n; r += (int64_t)gridDim.x * BLK) {
    double acc = 0.0;
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
      if (ci[k] == r) acc += v[k];
    d[r] = acc;
  }
}

// the unpack and final add of one step (see the file header): compact DOF
// t < nc: v = y_c[t] + recv[rpos[rp[t]]] + ... (peer order, as the per-peer
// unpack launches added them), then y[i] = v (overwrite flag: a node no
// interior element touches) or y[i] + v, i = fidx[t] & 0x7fffffff; t >= nc:
// zero the interior's remaining zero-list DOFs (nodes no element touches)
// (yc_local: y_c is indexed like y, by local DOF)
__global__ void k_dd_finish(double* __restrict__ y, const uint32_t* __restrict__ fidx, int64_t nc,
                            const double* __restrict__ yc, int yc_local,
                            const int32_t* __restrict__ rp, const uint32_t* __restrict__ rpos,
                            const double* __restrict__ recv, const uint32_t* __restrict__ fzero,
                            int64_t nz) {
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < nc + nz;
       t += (int64_t)gridDim.x * BLK) {
    if (t < nc) {
      const uint32_t e = fidx[t];
      const uint32_t i = e & 0x7fffffffu;
      double v = yc[yc_local ? i : t];
      for (int32_t k = rp[t]; k < rp[t + 1]; ++k) v += recv[rpos[k]];
      y[i] = ((e >> 31) ? 0.0 : y[i]) + v;
    } else {
      y[fzero[t - nc]] = 0.0;
    }
  }
}

// the loopback transport's exchange (sem_dd_set_loopback): the send buffer
// back into the receive buffer, one kernel on the side stream as RCCL's
// send/recv would be
__global__ void k_dd_loopback(double* __restrict__ dst, const double* __restrict__ src, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK)
    dst[t] = src[t];
}

}  // namespace

// ---------------------------------------------------------------- context
struct sem_dd {
  int device = 0;
  sem_ctx* iface = nullptr;     // interface elements, compact numbering
  sem_ctx* interior = nullptr;  // interior elements, local numbering (may be null)
  int64_t ndof = 0;             // local DOFs
  int64_t nc = 0;               // compact (interface-element) DOFs
  uint32_t* d_cidx = nullptr;   // compact -> local DOF
  std::vector<int> peer;
  std::vector<int64_t> off;     // per-peer ranges of the exchange buffers
  uint32_t* d_pidx = nullptr;   // compact DOF of every exchanged entry
  uint8_t* d_notown = nullptr;  // local DOFs owned by another rank (global dots)
  double* d_uc = nullptr;
  double* d_yc = nullptr;
  bool iface_local = false;      // interface context over the local numbering
  bool iface_skip_zero = false;  // ... whose zero list it never needs (build_finish)
  uint32_t* d_sidx = nullptr;    // local mode: y_c entry of every exchanged value
  double* d_send = nullptr;
  double* d_recv = nullptr;
  // finish tables (k_dd_finish; built by build_finish for the interior
  // context's plan of map epoch fin_epoch)
  uint32_t* d_fidx = nullptr;   // cidx[j] | overwrite << 31
  int32_t* d_rp = nullptr;      // [nc + 1]: received values of compact DOF j at rpos[rp[j]..rp[j+1])
  uint32_t* d_rpos = nullptr;   // positions in d_recv, peer order
  uint32_t* d_fzero = nullptr;  // interior zero-list DOFs outside the interface
  int64_t n_fzero = 0;
  bool defer_zero = false;      // the interior's zero list is folded into k_dd_finish
  // the interior's seam sum fused into the finish (sem::ctx_seam_finish):
  // compact DOF of every interior seam node (or -1), the compact DOFs off
  // the seams; seam_deferred: this step's interior launch left its seam sum
  bool seam_fused = false, seam_deferred = false;
  int32_t* d_seam_cj = nullptr;
  uint32_t* d_rest = nullptr;
  int64_t n_rest = 0;
  // the interface context's seam sum fused with the pack (sem::ctx_seam_pack;
  // SEM_DD_FUSE_PACK=0 keeps the two launches): d_pack_sj[k] = seam index of
  // the k-th exchanged DOF in the interface plan, or -1
  bool pack_fused = false;
  int32_t* d_pack_sj = nullptr;
  // split finish (SEM_DD_SPLIT_FINISH, default on with the fused seam sum):
  // the interior's seam nodes no interface DOF touches, and the deferred
  // zero list, are finished on the caller's stream BEFORE the join with the
  // side stream (they do not need the exchange); the rest after it
  bool split_finish = false, split_pre_done = false;
  uint32_t* d_seam_pre = nullptr;
  uint32_t* d_seam_post = nullptr;
  int64_t n_seam_pre = 0, n_seam_post = 0;
  uint64_t fin_epoch = ~0ull;
  bool loopback = false;        // diagnostic transport (sem_dd_set_loopback)
  bool rccl_self = false;       // timing transport: RCCL send/recv to this rank itself
                                // on a one-rank communicator (sem_dd_set_rccl_self)
  hipStream_t side = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool ev_system = true;  // the events carry the system-scope fence (dd_fence_system)
  // transport: native RCCL communicator, or caller callbacks
  ncclComm_t comm = nullptr;
  sem_exchange_fn xfn = nullptr;
  sem_allreduce_fn rfn = nullptr;
  void* user = nullptr;
  int world = 1, rank = 0;
  // captured step (sem_dd_set_graphs): the launches of one action as three
  // HIP graphs around the transport call -- S: gather, interface elements,
  // pack (side stream); M: interior elements (caller's stream); G: the
  // finish (caller's) -- replayed while the kind, the u / y pointers and the
  // contexts' state stay the same.  Off by default: on ROCm 7
  // a graph launch costs more host time than the launches it replaces
  // (profiles/r03/multirank/: 2-rank rehearsal 0.787 ms per step eager,
  // 0.866 captured; tools/r03/stream_bench.cpp: 11.3 us per 2-kernel graph
  // replay against 4.7 us eager); SEM_DD_GRAPH=1 or sem_dd_set_graphs opt in
  bool graphs = false;
  hipStream_t cap = nullptr;  // capture stream of M and G
  hipGraphExec_t gS = nullptr, gM = nullptr, gG = nullptr;
  int g_kind = -1;
  const double* g_u = nullptr;
  double* g_y = nullptr;
  uint64_t g_ep_iface = 0, g_ep_interior = 0;  // the contexts' epochs at capture
  int64_t n_captures = 0, n_replays = 0;
  // host time spent enqueueing sem_dd_apply, and inside the transport call;
  // the rest split into the side-stream part (gather, interface elements,
  // pack), the interior elements and the finish (event + k_dd_finish)
  int64_t host_steps = 0, host_ns = 0, host_ns_transport = 0;
  int64_t host_ns_side = 0, host_ns_main = 0, host_ns_finish = 0;
};

namespace {

int64_t n_exchanged(const sem_dd* d) { return d->off.empty() ? 0 : d->off.back(); }

// changes whenever either context changes anything its captured launches
// read (map, geometry, modes, Reynolds number, linearisation buffer):
// a graph captured before such a call would replay stale arguments or freed
// pointers (sem::ctx_epoch)
uint64_t ep_iface(const sem_dd* d) { return d->iface ? sem::ctx_epoch(d->iface) : 0; }
uint64_t ep_interior(const sem_dd* d) { return d->interior ? sem::ctx_epoch(d->interior) : 0; }

using Clock = std::chrono::steady_clock;
inline int64_t ns_since(Clock::time_point t0) {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
}

// the finish tables for the interior context's current plan (see the file
// header): rebuilt when its map changes (synchronises the device then)
int build_finish(sem_dd* d) {
  const uint64_t ep = (d->interior ? sem::ctx_map_epoch(d->interior) : 0) * 1000003u +
                     (d->iface ? sem::ctx_map_epoch(d->iface) : 0);
  if (ep == d->fin_epoch && d->d_fidx) return SEM_OK;
  HIP_TRY(hipDeviceSynchronize());  // nothing in flight reads the old tables
  const int64_t nc = d->nc, ne = n_exchanged(d);
  std::vector<uint32_t> cidx((size_t)nc), pidx((size_t)ne);
  if (nc) HIP_TRY(hipMemcpy(cidx.data(), d->d_cidx, nc * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (ne) HIP_TRY(hipMemcpy(pidx.data(), d->d_pidx, ne * sizeof(uint32_t), hipMemcpyDeviceToHost));
  // received values per compact DOF, in peer order (the order of d_recv)
  std::vector<int32_t> rp((size_t)nc + 1, 0);
  for (int64_t t = 0; t < ne; ++t) {
    if (pidx[t] >= (uint64_t)nc) return fail(SEM_E_INVALID, "peer DOF outside the interface");
    rp[pidx[t] + 1]++;
  }
  for (int64_t j = 0; j < nc; ++j) rp[j + 1] += rp[j];
  std::vector<uint32_t> rpos((size_t)std::max<int64_t>(ne, 1));
  {
    std::vector<int32_t> fill(rp.begin(), rp.end() - 1);
    for (int64_t t = 0; t < ne; ++t) rpos[fill[pidx[t]]++] = (uint32_t)t;
  }
  // the interior's zero list: interface DOFs among it are overwritten by the
  // finish, the others zeroed by it -- only when the list holds nodes no
  // interior element touches (no atomic first writers: those must be zero
  // before the interior kernel runs)
  std::vector<uint32_t> fidx(cidx), fzero;
  std::vector<int32_t> compact((size_t)d->ndof, -1);
  for (int64_t j = 0; j < nc; ++j) compact[cidx[j]] = (int32_t)j;
  bool defer = false;
  if (d->interior) {
    std::vector<uint32_t> z;
    bool only_unref = false;
    SEM_TRY(sem::ctx_zero_list(d->interior, &z, &only_unref));
    defer = only_unref;
    if (defer && !z.empty()) {
      const int dpn = sem::ctx_dpn(d->interior);
      for (const uint32_t node : z)
        for (int c = 0; c < dpn; ++c) {
          const uint32_t dof = node * dpn + c;
          if (compact[dof] >= 0) fidx[compact[dof]] |= 0x80000000u;
          else fzero.push_back(dof);
        }
    }
  }
  // every finish table is freed (and nulled) exactly once, before any new
  // allocation: a rebuild after a map change may be handed the same addresses
  for (void** pp : {(void**)&d->d_sidx, (void**)&d->d_seam_cj, (void**)&d->d_rest,
                    (void**)&d->d_fidx, (void**)&d->d_rp, (void**)&d->d_rpos,
                    (void**)&d->d_fzero, (void**)&d->d_pack_sj, (void**)&d->d_seam_pre,
                    (void**)&d->d_seam_post}) {
    (void)hipFree(*pp);
    *pp = nullptr;
  }
  d->n_rest = 0;
  d->pack_fused = false;
  d->split_finish = false;
  d->n_seam_pre = d->n_seam_post = 0;
  HIP_TRY(hipMalloc(&d->d_fidx, std::max<int64_t>(nc, 1) * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&d->d_rp, rp.size() * sizeof(int32_t)));
  HIP_TRY(hipMalloc(&d->d_rpos, rpos.size() * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&d->d_fzero, std::max<size_t>(fzero.size(), 1) * sizeof(uint32_t)));
  if (nc) HIP_TRY(hipMemcpy(d->d_fidx, fidx.data(), nc * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d->d_rp, rp.data(), rp.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  if (ne) HIP_TRY(hipMemcpy(d->d_rpos, rpos.data(), ne * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (!fzero.empty())
    HIP_TRY(hipMemcpy(d->d_fzero, fzero.data(), fzero.size() * sizeof(uint32_t),
                      hipMemcpyHostToDevice));
  d->n_fzero = (int64_t)fzero.size();
  d->defer_zero = defer;
  // the interior's seam nodes (one DOF per node: DOF = node id) and the
  // interface DOFs the fused finish handles outside them
  // SEM_DD_FUSE_SEAM=0: the interior's own seam-sum launch, then k_dd_finish
  // (A/B and the bitwise test of the fused form)
  const char* fe = std::getenv("SEM_DD_FUSE_SEAM");
  d->seam_fused = d->interior && defer && sem::ctx_seam_fusable(d->interior) &&
                  !(fe && std::atoi(fe) == 0);
  if (d->seam_fused) {
    std::vector<uint32_t> sg;
    SEM_TRY(sem::ctx_seam_gids(d->interior, &sg));
    std::vector<int32_t> cj(sg.size());
    std::vector<uint8_t> covered((size_t)std::max<int64_t>(nc, 1), 0);
    for (size_t t = 0; t < sg.size(); ++t) {
      cj[t] = compact[sg[t]];
      if (cj[t] >= 0) covered[cj[t]] = 1;
    }
    std::vector<uint32_t> rest;
    for (int64_t j = 0; j < nc; ++j)
      if (!covered[j]) rest.push_back((uint32_t)j);
    HIP_TRY(hipMalloc(&d->d_seam_cj, std::max<size_t>(cj.size(), 1) * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&d->d_rest, std::max<size_t>(rest.size(), 1) * sizeof(uint32_t)));
    if (!cj.empty())
      HIP_TRY(hipMemcpy(d->d_seam_cj, cj.data(), cj.size() * sizeof(int32_t),
                        hipMemcpyHostToDevice));
    if (!rest.empty())
      HIP_TRY(hipMemcpy(d->d_rest, rest.data(), rest.size() * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
    d->n_rest = (int64_t)rest.size();
    const char* fs = std::getenv("SEM_DD_SPLIT_FINISH");
    if (!(fs && std::atoi(fs) == 0)) {
      std::vector<uint32_t> pre, post;
      for (size_t t = 0; t < cj.size(); ++t) (cj[t] >= 0 ? post : pre).push_back((uint32_t)t);
      HIP_TRY(hipMalloc(&d->d_seam_pre, std::max<size_t>(pre.size(), 1) * sizeof(uint32_t)));
      HIP_TRY(hipMalloc(&d->d_seam_post, std::max<size_t>(post.size(), 1) * sizeof(uint32_t)));
      if (!pre.empty())
        HIP_TRY(hipMemcpy(d->d_seam_pre, pre.data(), pre.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice));
      if (!post.empty())
        HIP_TRY(hipMemcpy(d->d_seam_post, post.data(), post.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice));
      d->n_seam_pre = (int64_t)pre.size();
      d->n_seam_post = (int64_t)post.size();
      d->split_finish = true;
    }
  }
  if (d->iface_local) {
    // pack reads y_c at the local DOF of every exchanged compact DOF; the
    // interface context's zero list (every node no interface element
    // touches) is never needed unless it holds atomic first writers
    std::vector<uint32_t> sidx((size_t)std::max<int64_t>(ne, 1), 0u);
    for (int64_t t = 0; t < ne; ++t) sidx[t] = cidx[pidx[t]];
    HIP_TRY(hipMalloc(&d->d_sidx, sidx.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(d->d_sidx, sidx.data(), sidx.size() * sizeof(uint32_t),
                      hipMemcpyHostToDevice));
    std::vector<uint32_t> zi;
    bool unref = false;
    SEM_TRY(sem::ctx_zero_list(d->iface, &zi, &unref));
    d->iface_skip_zero = unref;
    const char* fp = std::getenv("SEM_DD_FUSE_PACK");
    if (ne && sem::ctx_seam_fusable(d->iface) && !sem::ctx_seam_has_prior(d->iface) &&
        !(fp && std::atoi(fp) == 0)) {
      std::vector<uint32_t> sg;
      SEM_TRY(sem::ctx_seam_gids(d->iface, &sg));
      std::vector<int32_t> seam_of((size_t)d->ndof, -1);
      for (size_t t = 0; t < sg.size(); ++t) seam_of[sg[t]] = (int32_t)t;
      std::vector<int32_t> sj((size_t)ne);
      for (int64_t t = 0; t < ne; ++t) sj[t] = seam_of[sidx[t]];
      HIP_TRY(hipMalloc(&d->d_pack_sj, sj.size() * sizeof(int32_t)));
      HIP_TRY(hipMemcpy(d->d_pack_sj, sj.data(), sj.size() * sizeof(int32_t),
                        hipMemcpyHostToDevice));
      d->pack_fused = true;
    }
  }
  d->fin_epoch = ep;
  return SEM_OK;
}

// side-stream part of one step: interface elements into y_c (DIAG: the
// operator diagonal instead of the action), packed into the send buffer
int dd_side(sem_dd* d, int op_kind, bool diag, const double* u, hipStream_t sd) {
  if (!d->iface) return SEM_OK;
  if (diag) {
    SEM_TRY(sem_diag(d->iface, op_kind, d->d_yc, sd));
  } else if (d->iface_local && d->pack_fused) {
    // interface elements, then their seam sum and the pack in one launch
    sem::ctx_set_defer_seam_sum(d->iface, true);
    const int rc = sem_apply(d->iface, op_kind, u, d->d_yc,
                             d->iface_skip_zero ? SEM_APPLY_SKIP_ZERO : 0, sd);
    sem::ctx_set_defer_seam_sum(d->iface, false);
    SEM_TRY(rc);
    return sem::ctx_seam_pack(d->iface, d->d_yc, d->d_send, d->d_sidx, d->d_pack_sj,
                              n_exchanged(d), sd);
  } else if (d->iface_local) {
    SEM_TRY(sem_apply(d->iface, op_kind, u, d->d_yc, d->iface_skip_zero ? SEM_APPLY_SKIP_ZERO : 0,
                      sd));
  } else {
    SEM_TRY(sem_gather(u, d->d_cidx, d->nc, d->d_uc, sd));
    SEM_TRY(sem_apply(d->iface, op_kind, d->d_uc, d->d_yc, 0, sd));
  }
  return sem_gather(d->d_yc, d->iface_local ? d->d_sidx : d->d_pidx, n_exchanged(d), d->d_send,
                    sd);
}

// main-stream part: interior elements into y (their zero list deferred to
// the finish when build_finish allowed it)
int dd_main(sem_dd* d, int op_kind, bool diag, const double* u, double* y, hipStream_t st) {
  d->seam_deferred = false;
  if (d->interior) {
    if (diag) return sem_diag(d->interior, op_kind, y, st);
    const int flags = d->defer_zero ? SEM_APPLY_SKIP_ZERO : 0;
    if (!d->seam_fused) return sem_apply(d->interior, op_kind, u, y, flags, st);
    sem::ctx_set_defer_seam_sum(d->interior, true);  // summed by the fused finish
    const int rc = sem_apply(d->interior, op_kind, u, y, flags, st);
    sem::ctx_set_defer_seam_sum(d->interior, false);
    d->seam_deferred = rc == SEM_OK;
    return rc;
  }
  HIP_TRY(hipMemsetAsync(y, 0, d->ndof * sizeof(double), st));
  return SEM_OK;
}

int dd_begin(sem_dd* d, int op_kind, bool diag, const double* u, double* y, hipStream_t st) {
  SEM_TRY(build_finish(d));
  auto t0 = Clock::now();
  HIP_TRY(hipEventRecord(d->ev0, st));
  HIP_TRY(hipStreamWaitEvent(d->side, d->ev0, 0));
  SEM_TRY(dd_side(d, op_kind, diag, u, d->side));
  d->host_ns_side += ns_since(t0);
  t0 = Clock::now();
  const int rc = dd_main(d, op_kind, diag, u, y, st);
  d->host_ns_main += ns_since(t0);
  return rc;
}

int dd_exchange_impl(sem_dd* d);

// the transport call, timed on the host (sem_dd_info [11])
int dd_exchange(sem_dd* d) {
  const auto t0 = Clock::now();
  const int rc = dd_exchange_impl(d);
  d->host_ns_transport += ns_since(t0);
  return rc;
}

int dd_exchange_impl(sem_dd* d) {
  const int np = (int)d->peer.size();
  if (!np) return SEM_OK;
  if (d->loopback) {
    const int64_t ne = n_exchanged(d);
    if (ne)
      hipLaunchKernelGGL(k_dd_loopback, dim3(grid_for(ne)), dim3(BLK), 0, d->side, d->d_recv,
                         d->d_send, ne);
    HIP_TRY(hipGetLastError());
    return SEM_OK;
  }
  if (d->comm) {
    NCCL_TRY(ncclGroupStart());
    for (int k = 0; k < np; ++k) {
      const size_t cnt = (size_t)(d->off[k + 1] - d->off[k]);
      const int peer = d->rccl_self ? 0 : d->peer[k];
      NCCL_TRY(ncclSend(d->d_send + d->off[k], cnt, ncclFloat64, peer, d->comm, d->side));
      NCCL_TRY(ncclRecv(d->d_recv + d->off[k], cnt, ncclFloat64, peer, d->comm, d->side));
    }
    NCCL_TRY(ncclGroupEnd());
    return SEM_OK;
  }
  if (d->xfn) {
    const int rc = d->xfn(d->user, np, d->peer.data(), d->off.data(), d->d_send, d->d_recv,
                          d->side);
    return rc ? fail(SEM_E_HIP, "interface exchange callback failed (" + std::to_string(rc) + ")")
              : SEM_OK;
  }
  return fail(SEM_E_STATE, "no transport: call sem_dd_init_rccl or sem_dd_set_transport");
}

// unpack + final add + deferred zero list in one launch on `st` (with the
// interior's seam sum when it was deferred)
sem::DDFinish dd_finish_args(const sem_dd* d) {
  sem::DDFinish f{};
  f.fidx = d->d_fidx;
  f.nc = d->nc;
  f.yc = d->d_yc;
  f.yc_local = d->iface_local ? 1 : 0;
  f.rp = d->d_rp;
  f.rpos = d->d_rpos;
  f.recv = d->d_recv;
  f.fzero = d->d_fzero;
  f.nz = d->defer_zero ? d->n_fzero : 0;
  f.seam_cj = d->d_seam_cj;
  f.rest = d->d_rest;
  f.n_rest = d->n_rest;
  return f;
}

// split finish, before the join: the interior's seam nodes off the
// interface and the deferred zero list (no received value needed)
int dd_finish_pre(sem_dd* d, double* y, hipStream_t st) {
  d->split_pre_done = false;
  if (!(d->seam_deferred && d->split_finish)) return SEM_OK;
  sem::DDFinish f = dd_finish_args(d);
  f.sel = d->d_seam_pre;
  f.n_sel = d->n_seam_pre;
  f.skip_rest = 1;
  SEM_TRY(sem::ctx_seam_finish(d->interior, y, f, st));
  d->split_pre_done = true;
  return SEM_OK;
}

int dd_add(sem_dd* d, double* y, hipStream_t st) {
  if (d->seam_deferred && d->split_finish && d->split_pre_done) {
    // the part that needs the exchange (the pre part ran before the join)
    sem::DDFinish f = dd_finish_args(d);
    f.sel = d->d_seam_post;
    f.n_sel = d->n_seam_post;
    f.skip_zero = 1;
    return sem::ctx_seam_finish(d->interior, y, f, st);
  }
  if (d->seam_deferred) return sem::ctx_seam_finish(d->interior, y, dd_finish_args(d), st);
  const int64_t tot = d->nc + (d->defer_zero ? d->n_fzero : 0);
  if (!tot) return SEM_OK;
  hipLaunchKernelGGL(k_dd_finish, dim3(grid_for(tot)), dim3(BLK), 0, st, y, d->d_fidx, d->nc,
                     d->d_yc, d->iface_local ? 1 : 0, d->d_rp, d->d_rpos, d->d_recv, d->d_fzero,
                     d->defer_zero ? d->n_fzero : 0);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

// the caller's stream waits for everything enqueued so far on the side stream
// (a stream-memory-operation join, hipStreamWriteValue64 on the side stream +
// hipStreamWaitValue64 on the caller's, hung the step on the MI355X box in
// round 4 and was removed; the event join stays)
int dd_join(sem_dd* d, hipStream_t st) {
  HIP_TRY(hipEventRecord(d->ev1, d->side));
  HIP_TRY(hipStreamWaitEvent(st, d->ev1, 0));
  return SEM_OK;
}

int dd_finish(sem_dd* d, double* y, hipStream_t st) {
  const auto t0 = Clock::now();
  int rc = dd_finish_pre(d, y, st);
  if (!rc) rc = dd_join(d, st);
  if (!rc) rc = dd_add(d, y, st);
  // cleared on every exit: a flag left set by a failed
  // join would make the next captured finish run only its post part
  d->split_pre_done = false;
  d->host_ns_finish += ns_since(t0);
  return rc;
}

// ---------------------------------------------------------------- captured step
void drop_graphs(sem_dd* d) {
  for (hipGraphExec_t* g : {&d->gS, &d->gM, &d->gG})
    if (*g) {
      (void)hipGraphExecDestroy(*g);
      *g = nullptr;
    }
  d->g_kind = -1;
}

// body() enqueues onto `s` (a capturable, non-default stream) -> *out
template <class F>
int capture(hipStream_t s, F body, hipGraphExec_t* out) {
  HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  const int rc = body();
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(s, &g);
  if (rc || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    if (rc) return rc;
    HIP_TRY(e);
  }
  const hipError_t ei = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  HIP_TRY(ei);
  return SEM_OK;
}

int dd_capture(sem_dd* d, int op_kind, const double* u, double* y) {
  drop_graphs(d);
  d->split_pre_done = false;  // the captured finish is the whole finish
  if (!d->cap) HIP_TRY(hipStreamCreateWithFlags(&d->cap, hipStreamNonBlocking));
  if (d->iface) SEM_TRY(capture(d->side, [&] { return dd_side(d, op_kind, false, u, d->side); }, &d->gS));
  SEM_TRY(capture(d->cap, [&] { return dd_main(d, op_kind, false, u, y, d->cap); }, &d->gM));
  SEM_TRY(capture(d->cap, [&] { return dd_add(d, y, d->cap); }, &d->gG));
  d->g_kind = op_kind;
  d->g_u = u;
  d->g_y = y;
  d->g_ep_iface = ep_iface(d);
  d->g_ep_interior = ep_interior(d);
  d->n_captures++;
  return SEM_OK;
}

// one action through the captured graphs: the same dependency structure as
// dd_begin / dd_exchange / dd_finish, three graph launches instead of ~10
// kernel launches
int dd_apply_graphs(sem_dd* d, int op_kind, const double* u, double* y, hipStream_t st) {
  SEM_TRY(build_finish(d));
  if (d->g_kind != op_kind || d->g_u != u || d->g_y != y ||
      d->g_ep_iface != ep_iface(d) || d->g_ep_interior != ep_interior(d)) {
    // the previous replay may still be running on the side stream
    HIP_TRY(hipStreamSynchronize(d->side));
    SEM_TRY(dd_capture(d, op_kind, u, y));
  }
  HIP_TRY(hipEventRecord(d->ev0, st));
  HIP_TRY(hipStreamWaitEvent(d->side, d->ev0, 0));
  if (d->gS) HIP_TRY(hipGraphLaunch(d->gS, d->side));
  HIP_TRY(hipGraphLaunch(d->gM, st));
  SEM_TRY(dd_exchange(d));
  SEM_TRY(dd_join(d, st));
  if (d->gG) HIP_TRY(hipGraphLaunch(d->gG, st));
  d->n_replays++;
  return SEM_OK;
}

int dd_allreduce(sem_dd* d, double* buf, int count, hipStream_t st) {
  if (!d || d->world == 1) return SEM_OK;
  if (d->comm) {
    NCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, d->comm, st));
    return SEM_OK;
  }
  if (d->rfn) {
    const int rc = d->rfn(d->user, buf, count, st);
    return rc ? fail(SEM_E_HIP, "all-reduce callback failed (" + std::to_string(rc) + ")") : SEM_OK;
  }
  return fail(SEM_E_STATE, "no transport for the global dot products");
}

// ---------------------------------------------------------------- PCG loop
// Jacobi-preconditioned CG on the free DOFs with every scalar on the device:
// alpha and beta are formed inside the update kernels from the reduced dot
// products, so an iteration enqueues its work without waiting for the host.
// The host reads the r.r history every `check` iterations (one small copy
// and one stream synchronisation) and stops at the first block that reached
// the tolerance; the iterations past the converged one only refine x.
struct PcgOp {
  sem_ctx* ctx = nullptr;  // single GPU
  sem_dd* dd = nullptr;    // or a rank of a decomposition
  const int64_t* rp = nullptr;  // or an assembled CSR matrix
  const int32_t* ci = nullptr;
  const double* v = nullptr;
  int64_t n = 0;
  int device = 0;
  int apply(int kind, const double* p, double* q, hipStream_t st) const {
    if (rp) {
      hipLaunchKernelGGL(k_csr_spmv, dim3(grid_for(n)), dim3(BLK), 0, st, n, rp, ci, v, p, q);
      HIP_TRY(hipGetLastError());
      return SEM_OK;
    }
    if (dd) {
      if (dd->graphs) return dd_apply_graphs(dd, kind, p, q, st);
      SEM_TRY(dd_begin(dd, kind, false, p, q, st));
      SEM_TRY(dd_exchange(dd));
      return dd_finish(dd, q, st);
    }
    return sem_apply(ctx, kind, p, q, 0, st);
  }
  int diag(int kind, double* out, hipStream_t st) const {
    if (rp) {
      hipLaunchKernelGGL(k_csr_diag, dim3(grid_for(n)), dim3(BLK), 0, st, n, rp, ci, v, out);
      HIP_TRY(hipGetLastError());
      return SEM_OK;
    }
    if (dd) {
      SEM_TRY(dd_begin(dd, kind, true, nullptr, out, st));
      SEM_TRY(dd_exchange(dd));
      return dd_finish(dd, out, st);
    }
    return sem_diag(ctx, kind, out, st);
  }
};

struct PcgScratch {
  double* base = nullptr;
  dinv_t* pc = nullptr;  // the packed preconditioner (k_cg_pack)
  uint8_t* flags = nullptr;
  double* red = nullptr;
  double* hist = nullptr;
  double* h_hist = nullptr;  // pinned
  ~PcgScratch() {
    (void)hipFree(base);
    (void)hipFree(pc);
    (void)hipFree(flags);
    (void)hipFree(red);
    (void)hipFree(hist);
    (void)hipHostFree(h_hist);
  }
};

const bool g_sync_each = std::getenv("SEM_PCG_SYNC_EACH") != nullptr;  // diagnostic
// SEM_PCG_SEPARATE_PQ=1: the p.q pass after the action even on one GPU (A/B)
const bool g_separate_pq = std::getenv("SEM_PCG_SEPARATE_PQ") != nullptr;
// SEM_PCG_X_EVERY=1: x updated every iteration (STEP_NOW; A/B against the
// default pairs, bitwise the same x)
// (read per solve)
bool pcg_x_pairs() {
  const char* e = std::getenv("SEM_PCG_X_EVERY");
  return !(e && std::atoi(e) == 1);
}

int pcg_run(const PcgOp& op, int kind, const double* b, double* x, const uint8_t* dir,
            const uint8_t* notown, double rtol, int max_iter, int check, int* iters,
            double* relres, hipStream_t st) {
  if (!b || !x || !dir) return fail(SEM_E_INVALID, "null argument");
  if (kind != SEM_OP_POISSON && !op.rp) return fail(SEM_E_NOTIMPL, "PCG: Poisson only");
  // rtol = 0: run exactly max_iter iterations (benchmarking)
  if (max_iter < 0 || !(rtol >= 0.0)) return fail(SEM_E_INVALID, "need rtol >= 0, max_iter >= 0");
  if (check < 1) check = 1;
  DeviceGuard g(op.device);
  const int64_t n = op.n;
  PcgScratch s;
  const bool g_x_pairs = pcg_x_pairs();
  // r, p, q, 1/diag, the second p buffer (x updated every second iteration);
  // rows padded to 32 doubles (16-byte vector accesses)
  const int64_t nn = (n + 31) / 32 * 32;
  HIP_TRY(hipMalloc(&s.base, (g_x_pairs ? 5 : 4) * nn * sizeof(double)));
  HIP_TRY(hipMalloc(&s.flags, n));
  HIP_TRY(hipMalloc(&s.pc, nn * sizeof(dinv_t)));
  // partials [2][RED_BLOCKS], then scalars: T0 = (rz, rr), T1 = (rz, rr), pq
  HIP_TRY(hipMalloc(&s.red, (2 * RED_BLOCKS + 8) * sizeof(double)));
  HIP_TRY(hipMalloc(&s.hist, ((size_t)max_iter + 1) * sizeof(double)));
  HIP_TRY(hipHostMalloc(&s.h_hist, ((size_t)check + 1) * sizeof(double)));
  double* r = s.base;
  double* p = r + nn;
  double* q = p + nn;
  double* dg = q + nn;
  double* p_alt = g_x_pairs ? dg + nn : nullptr;  // the other p buffer
  // x is the caller's: 16-byte aligned -> the paired kernels
  const bool v2 = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  double* partial = s.red;
  double* T[2] = {s.red + 2 * RED_BLOCKS, s.red + 2 * RED_BLOCKS + 2};
  double* pq = s.red + 2 * RED_BLOCKS + 4;
  double* alpha_saved = s.red + 2 * RED_BLOCKS + 5;  // alpha of a STEP_DEFER iteration
  bool x_owed = false;  // x += alpha_saved * p_alt still to do
  const int gb = grid_for(n, RED_BLOCKS);
  const bool multi = op.dd && op.dd->world > 1;  // dots need an all-reduce
  hipLaunchKernelGGL(k_cg_flags, dim3(grid_for(n)), dim3(BLK), 0, st, dir, notown, n, s.flags);
  SEM_TRY(op.diag(kind, dg, st));
  hipLaunchKernelGGL(k_cg_invert, dim3(grid_for(n)), dim3(BLK), 0, st, dg, s.flags, n);
  hipLaunchKernelGGL(k_cg_pack, dim3(grid_for(n)), dim3(BLK), 0, st, dg, s.flags, n, s.pc);
  SEM_TRY(op.apply(kind, x, r, st));
  hipLaunchKernelGGL(k_cg_start, dim3(gb), dim3(BLK), 0, st, b, r, s.pc, n, p, partial);
  hipLaunchKernelGGL(k_cg_finish, dim3(1), dim3(BLK), 0, st, partial, gb, 2, T[0], nullptr);
  HIP_TRY(hipGetLastError());
  SEM_TRY(dd_allreduce(op.dd, T[0], 2, st));
  HIP_TRY(hipMemcpyAsync(s.h_hist, T[0] + 1, sizeof(double), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const double rr0 = s.h_hist[0];
  if (!std::isfinite(rr0)) return fail(SEM_E_INVALID, "PCG: non-finite initial residual");
  const double tol2 = rtol * rtol * rr0;
  double rr_last = rr0;
  int it = 0;
  bool done = rr0 == 0.0;
  while (!done && it < max_iter) {
    const int blk = std::min(check, max_iter - it);
    for (int k = 0; k < blk; ++k) {
      const int o = it & 1, nw = o ^ 1;
      if (op.ctx && !g_separate_pq) {
        // single GPU: p.q summed inside the action (sem_apply_dot; p = 0 on
        // Dirichlet DOFs, every DOF owned)
        SEM_TRY(sem_apply_dot(op.ctx, kind, p, q, pq, st));
      } else {
        SEM_TRY(op.apply(kind, p, q, st));
        hipLaunchKernelGGL(k_cg_pq<2>, dim3(gb), dim3(BLK), 0, st, p, q, s.flags, n, partial);
        hipLaunchKernelGGL(k_cg_finish, dim3(1), dim3(BLK), 0, st, partial, gb, 1, pq, nullptr);
        SEM_TRY(dd_allreduce(op.dd, pq, 1, st));
      }
      hipLaunchKernelGGL(k_cg_residual<2>, dim3(gb), dim3(BLK), 0, st, r, q, s.pc, T[o], pq, n,
                         partial);
      hipLaunchKernelGGL(k_cg_finish, dim3(1), dim3(BLK), 0, st, partial, gb, 2, T[nw],
                         multi ? nullptr : s.hist + it + 1);
      if (multi) {
        SEM_TRY(dd_allreduce(op.dd, T[nw], 2, st));
        hipLaunchKernelGGL(k_cg_record, dim3(1), dim3(WV), 0, st, T[nw] + 1, s.hist + it + 1);
      }
      if (!g_x_pairs) {
        if (v2)
          hipLaunchKernelGGL((k_cg_step<2, STEP_NOW>), dim3(gb), dim3(BLK), 0, st, x, p, nullptr, r,
                             s.pc, T[nw], T[o], pq, nullptr, n);
        else
          hipLaunchKernelGGL((k_cg_step<1, STEP_NOW>), dim3(gb), dim3(BLK), 0, st, x, p, nullptr, r,
                             s.pc, T[nw], T[o], pq, nullptr, n);
      } else if (!x_owed) {  // p_alt = z + beta p; x waits for the next iteration
        hipLaunchKernelGGL((k_cg_step<2, STEP_DEFER>), dim3(gb), dim3(BLK), 0, st, x, p, p_alt, r,
                           s.pc, T[nw], T[o], pq, alpha_saved, n);
      } else if (v2) {  // x += alpha' p_alt + alpha p; p_alt = z + beta p
        hipLaunchKernelGGL((k_cg_step<2, STEP_PAIR>), dim3(gb), dim3(BLK), 0, st, x, p, p_alt, r,
                           s.pc, T[nw], T[o], pq, alpha_saved, n);
      } else {
        hipLaunchKernelGGL((k_cg_step<1, STEP_PAIR>), dim3(gb), dim3(BLK), 0, st, x, p, p_alt, r,
                           s.pc, T[nw], T[o], pq, alpha_saved, n);
      }
      if (g_x_pairs) {  // the new p is in p_alt; the old one is the owed update's
        std::swap(p, p_alt);
        x_owed = !x_owed;
      }
      HIP_TRY(hipGetLastError());
      if (g_sync_each) HIP_TRY(hipDeviceSynchronize());  // diagnostic
      ++it;
    }
    HIP_TRY(hipMemcpyAsync(s.h_hist, s.hist + it - blk + 1, blk * sizeof(double),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int k = 0; k < blk; ++k) {
      rr_last = s.h_hist[k];
      if (!std::isfinite(rr_last)) return fail(SEM_E_INVALID, "PCG: non-finite residual");
      if (rr_last <= tol2) done = true;
    }
  }
  if (x_owed) {
    hipLaunchKernelGGL(k_cg_flush_x, dim3(grid_for(n)), dim3(BLK), 0, st, x, p_alt, alpha_saved, n);
    HIP_TRY(hipGetLastError());
  }
  if (iters) *iters = it;
  if (relres) *relres = rr0 > 0.0 ? std::sqrt(rr_last / rr0) : 0.0;
  if (!done && rtol > 0.0)
    return fail(SEM_E_INVALID, "PCG did not converge in " + std::to_string(max_iter) +
                                   " iterations");
  return SEM_OK;
}

}  // namespace

extern "C" {

int sem_pcg_solve(sem_ctx* c, int op_kind, const double* b, double* x, const uint8_t* mask,
                  double rtol, int max_iter, int* iters, double* relres, void* stream) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  PcgOp op;
  op.ctx = c;
  op.n = sem::ctx_ndof(c);
  op.device = sem::ctx_device(c);
  return pcg_run(op, op_kind, b, x, mask, nullptr, rtol, max_iter, SEM_PCG_CHECK_EVERY, iters,
                 relres, S(stream));
}

int sem_csr_pcg_solve(int64_t n, const int64_t* d_rowptr, const int32_t* d_colind,
                      const double* d_val, const double* d_b, double* d_x,
                      const uint8_t* d_dirichlet, double rtol, int max_iter, int* iters,
                      double* final_relres, int device, void* stream) {
  if (n < 1 || !d_rowptr || !d_colind || !d_val)
    return fail(SEM_E_INVALID, "sem_csr_pcg_solve: bad matrix");
  PcgOp op;
  op.rp = d_rowptr;
  op.ci = d_colind;
  op.v = d_val;
  op.n = n;
  op.device = device;
  return pcg_run(op, SEM_OP_POISSON, d_b, d_x, d_dirichlet, nullptr, rtol, max_iter,
                 SEM_PCG_CHECK_EVERY, iters, final_relres, S(stream));
}

int sem_copy_async(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (nbytes < 0 || (nbytes && (!dst || !src))) return fail(SEM_E_INVALID, "bad arguments");
  if (nbytes) HIP_TRY(hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDefault, S(stream)));
  return SEM_OK;
}

int sem_rccl_unique_id(void* h_id, int nbytes) {
  if (!h_id || nbytes < (int)sizeof(ncclUniqueId))
    return fail(SEM_E_INVALID, "need a buffer of SEM_RCCL_ID_BYTES bytes");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(h_id, &id, sizeof(id));
  return SEM_OK;
}

// Scope of the fence of the two events that order the side stream against
// the caller's stream.  Device scope (hipEventDisableSystemFence)
// only for the one-device transports -- the loopback copy and RCCL to this
// rank itself -- where every store into the buffers the events order is made
// by a kernel of this device and published device-wide by its own
// end-of-kernel release (one rank of the 8-strip split: 0.0924 against
// 0.0944-0.0961 ms per step, profiles/r05/dd/event_fence/).  A real peer
// exchange keeps the system-scope fence: with several ranks, RCCL's P2P
// transport may have the PEER's kernel or a copy engine write the receive
// side over xGMI, and the callback transport's host-staged copies land
// through the copy engines; what the device-scope release orders there is
// not established, so it is not assumed.  SEM_DD_EVENT_FENCE=system /
// device forces either scope for every transport (A/B and tests).
static bool dd_fence_system(const sem_dd* d) {
  const char* e = std::getenv("SEM_DD_EVENT_FENCE");
  if (e && std::string(e) == "system") return true;
  if (e && std::string(e) == "device") return false;
  return !(d->loopback || d->rccl_self);
}

static unsigned dd_event_flags(bool system) {
  return hipEventDisableTiming | (system ? 0u : hipEventDisableSystemFence);
}

// (re)creates ev0 / ev1 with the fence scope the current transport needs
// (transports are set up before the first step; nothing may be in flight)
static int dd_make_events(sem_dd* d) {
  const bool sys = dd_fence_system(d);
  if (d->ev0 && d->ev1 && d->ev_system == sys) return SEM_OK;
  HIP_TRY(hipDeviceSynchronize());
  if (d->ev0) (void)hipEventDestroy(d->ev0);
  if (d->ev1) (void)hipEventDestroy(d->ev1);
  d->ev0 = d->ev1 = nullptr;
  HIP_TRY(hipEventCreateWithFlags(&d->ev0, dd_event_flags(sys)));
  HIP_TRY(hipEventCreateWithFlags(&d->ev1, dd_event_flags(sys)));
  d->ev_system = sys;
  return SEM_OK;
}

int sem_dd_create(sem_dd** out, sem_ctx* iface, sem_ctx* interior, int64_t ndof_local,
                  const uint32_t* d_iface_dofs, int64_t n_iface_dofs, int n_peers,
                  const int* h_peers, const int64_t* h_peer_counts, const uint32_t* d_peer_dofs,
                  const uint8_t* d_not_owned, int device) {
  if (!out) return fail(SEM_E_INVALID, "null dd pointer");
  *out = nullptr;
  if (ndof_local < 1 || n_peers < 0 || n_iface_dofs < 0 ||
      (n_peers && (!h_peers || !h_peer_counts || !d_peer_dofs)))
    return fail(SEM_E_INVALID, "sem_dd_create: bad arguments");
  // a rank that shares no node still joins the global dot products
  if (!iface != (n_iface_dofs == 0) || (!iface && n_peers) || (iface && !d_iface_dofs))
    return fail(SEM_E_INVALID, "sem_dd_create: interface context, DOFs and peers disagree");
  if (!iface && !interior) return fail(SEM_E_INVALID, "sem_dd_create: no elements");
  if (iface && sem::ctx_ndof(iface) != n_iface_dofs && sem::ctx_ndof(iface) != ndof_local)
    return fail(SEM_E_INVALID,
                "interface context must hold n_iface_dofs (compact) or ndof_local (local) DOFs");
  if (interior && sem::ctx_ndof(interior) != ndof_local)
    return fail(SEM_E_INVALID, "interior context must hold ndof_local DOFs");
  if ((iface && sem::ctx_device(iface) != device) ||
      (interior && sem::ctx_device(interior) != device))
    return fail(SEM_E_INVALID, "contexts live on another device");
  DeviceGuard g(device);
  sem_dd* d = new sem_dd();
  d->device = device;
  d->iface = iface;
  d->interior = interior;
  d->ndof = ndof_local;
  d->nc = n_iface_dofs;
  d->iface_local = iface && sem::ctx_ndof(iface) == ndof_local && n_iface_dofs != ndof_local;
  d->off.assign(1, 0);
  for (int k = 0; k < n_peers; ++k) {
    if (h_peer_counts[k] < 0) {
      delete d;
      return fail(SEM_E_INVALID, "negative peer count");
    }
    d->peer.push_back(h_peers[k]);
    d->off.push_back(d->off.back() + h_peer_counts[k]);
  }
  const int64_t ne = d->off.back();
  auto bad = [&](hipError_t e) {
    if (e == hipSuccess) return false;
    sem_dd_destroy(d);
    return true;
  };
  const int64_t nc1 = std::max<int64_t>(n_iface_dofs, 1);
  const int64_t nyc = d->iface_local ? ndof_local : nc1;
  if (bad(hipMalloc(&d->d_cidx, nc1 * sizeof(uint32_t))) ||
      bad(hipMalloc(&d->d_uc, (d->iface_local ? 1 : nc1) * sizeof(double))) ||
      bad(hipMalloc(&d->d_yc, nyc * sizeof(double))) ||
      bad(hipMalloc(&d->d_pidx, std::max<int64_t>(ne, 1) * sizeof(uint32_t))) ||
      bad(hipMalloc(&d->d_send, std::max<int64_t>(ne, 1) * sizeof(double))) ||
      bad(hipMalloc(&d->d_recv, std::max<int64_t>(ne, 1) * sizeof(double))) ||
      bad(hipStreamCreateWithFlags(&d->side, hipStreamNonBlocking)) ||
      bad(hipEventCreateWithFlags(&d->ev0, dd_event_flags(true))) ||
      bad(hipEventCreateWithFlags(&d->ev1, dd_event_flags(true))))
    return fail(SEM_E_HIP, "sem_dd_create: HIP allocation failed");
  d->ev_system = true;  // no transport yet: the system scope
  if (n_iface_dofs && bad(hipMemcpy(d->d_cidx, d_iface_dofs, n_iface_dofs * sizeof(uint32_t),
                                    hipMemcpyDeviceToDevice)))
    return fail(SEM_E_HIP, "sem_dd_create: copy failed");
  if (ne && bad(hipMemcpy(d->d_pidx, d_peer_dofs, ne * sizeof(uint32_t), hipMemcpyDeviceToDevice)))
    return fail(SEM_E_HIP, "sem_dd_create: copy failed");
  if (d_not_owned) {
    if (bad(hipMalloc(&d->d_notown, ndof_local)) ||
        bad(hipMemcpy(d->d_notown, d_not_owned, ndof_local, hipMemcpyDeviceToDevice)))
      return fail(SEM_E_HIP, "sem_dd_create: copy failed");
  }
  // the device-to-device copies above may still run on the legacy stream
  if (bad(hipDeviceSynchronize())) return fail(SEM_E_HIP, "sem_dd_create: synchronize failed");
  if (const char* e = std::getenv("SEM_DD_GRAPH")) d->graphs = std::atoi(e) != 0;
  *out = d;
  return SEM_OK;
}

void sem_dd_destroy(sem_dd* d) {
  if (!d) return;
  DeviceGuard g(d->device);
  if (d->side) (void)hipStreamSynchronize(d->side);
  if (d->cap) (void)hipStreamSynchronize(d->cap);
  drop_graphs(d);
  if (d->cap) (void)hipStreamDestroy(d->cap);
  if (d->comm) (void)ncclCommDestroy(d->comm);
  (void)hipFree(d->d_cidx);
  (void)hipFree(d->d_pidx);
  (void)hipFree(d->d_notown);
  (void)hipFree(d->d_uc);
  (void)hipFree(d->d_yc);
  (void)hipFree(d->d_send);
  (void)hipFree(d->d_recv);
  (void)hipFree(d->d_fidx);
  (void)hipFree(d->d_rp);
  (void)hipFree(d->d_rpos);
  (void)hipFree(d->d_fzero);
  (void)hipFree(d->d_sidx);
  (void)hipFree(d->d_seam_cj);
  (void)hipFree(d->d_rest);
  (void)hipFree(d->d_pack_sj);
  (void)hipFree(d->d_seam_pre);
  (void)hipFree(d->d_seam_post);
  if (d->ev0) (void)hipEventDestroy(d->ev0);
  if (d->ev1) (void)hipEventDestroy(d->ev1);
  if (d->side) (void)hipStreamDestroy(d->side);
  delete d;
}

int sem_dd_init_rccl(sem_dd* d, const void* h_id, int world, int rank) {
  if (!d || !h_id || world < 1 || rank < 0 || rank >= world)
    return fail(SEM_E_INVALID, "sem_dd_init_rccl: bad arguments");
  for (int p : d->peer)
    if (p < 0 || p >= world || p == rank) return fail(SEM_E_INVALID, "peer rank out of range");
  DeviceGuard g(d->device);
  ncclUniqueId id;
  std::memcpy(&id, h_id, sizeof(id));
  ncclComm_t comm = nullptr;
  NCCL_TRY(ncclCommInitRank(&comm, world, id, rank));
  if (d->comm) (void)ncclCommDestroy(d->comm);
  d->comm = comm;
  d->loopback = false;
  d->rccl_self = false;
  d->world = world;
  d->rank = rank;
  return dd_make_events(d);
}

int sem_dd_set_rccl_self(sem_dd* d) {
  if (!d) return fail(SEM_E_INVALID, "null dd");
  DeviceGuard g(d->device);
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  ncclComm_t comm = nullptr;
  NCCL_TRY(ncclCommInitRank(&comm, 1, id, 0));
  if (d->comm) (void)ncclCommDestroy(d->comm);
  d->comm = comm;
  d->xfn = nullptr;
  d->rfn = nullptr;
  d->user = nullptr;
  d->world = 1;
  d->rank = 0;
  d->loopback = false;
  d->rccl_self = true;
  return dd_make_events(d);
}

int sem_dd_set_loopback(sem_dd* d) {
  if (!d) return fail(SEM_E_INVALID, "null dd");
  DeviceGuard g(d->device);
  if (d->comm) {
    (void)ncclCommDestroy(d->comm);
    d->comm = nullptr;
  }
  d->xfn = nullptr;
  d->rfn = nullptr;
  d->user = nullptr;
  d->world = 1;
  d->rank = 0;
  d->loopback = true;
  d->rccl_self = false;
  return dd_make_events(d);
}

int sem_dd_set_transport(sem_dd* d, sem_exchange_fn xfn, sem_allreduce_fn rfn, void* user,
                         int world, int rank) {
  if (!d || world < 1 || rank < 0 || rank >= world)
    return fail(SEM_E_INVALID, "sem_dd_set_transport: bad arguments");
  d->loopback = false;
  d->rccl_self = false;
  d->xfn = xfn;
  d->rfn = rfn;
  d->user = user;
  d->world = world;
  d->rank = rank;
  DeviceGuard g(d->device);
  if (d->comm) {
    (void)ncclCommDestroy(d->comm);
    d->comm = nullptr;
  }
  return dd_make_events(d);
}

int sem_dd_info(sem_dd* d, int64_t* info, int n_info) {
  if (!d || !info || n_info < 1) return fail(SEM_E_INVALID, "bad arguments");
  const int64_t v[16] = {d->ndof, d->nc, (int64_t)d->peer.size(), n_exchanged(d),
                         d->loopback ? 3 : d->rccl_self ? 4 : d->comm ? 1 : (d->xfn ? 2 : 0),
                         d->interior ? 1 : 0,
                         d->graphs ? 1 : 0, d->n_captures, d->n_replays,
                         d->host_steps, d->host_ns, d->host_ns_transport,
                         d->host_ns_side, d->host_ns_main, d->host_ns_finish,
                         (d->defer_zero ? 1 : 0) | (d->seam_fused ? 2 : 0) |
                             (d->pack_fused ? 4 : 0) |
                             (d->split_finish ? 8 : 0) | (d->ev_system ? 0 : 16)};
  for (int i = 0; i < n_info && i < 16; ++i) info[i] = v[i];
  return SEM_OK;
}

int sem_dd_set_graphs(sem_dd* d, int enable) {
  if (!d) return fail(SEM_E_INVALID, "null dd");
  DeviceGuard g(d->device);
  if (d->side) HIP_TRY(hipStreamSynchronize(d->side));
  drop_graphs(d);
  d->graphs = enable != 0;
  return SEM_OK;
}

int sem_dd_apply(sem_dd* d, int op_kind, const double* d_u, double* d_y, void* stream) {
  if (!d || !d_u || !d_y) return fail(SEM_E_INVALID, "null argument");
  if (d_u == d_y) return fail(SEM_E_INVALID, "sem_dd_apply: u and y must not alias");
  DeviceGuard g(d->device);
  const auto t0 = Clock::now();
  int rc;
  if (d->graphs) {
    rc = dd_apply_graphs(d, op_kind, d_u, d_y, S(stream));
  } else {
    SEM_TRY(dd_begin(d, op_kind, false, d_u, d_y, S(stream)));
    SEM_TRY(dd_exchange(d));
    rc = dd_finish(d, d_y, S(stream));
  }
  d->host_ns += ns_since(t0);
  d->host_steps++;
  return rc;
}

int sem_dd_diag(sem_dd* d, int op_kind, double* d_diag, void* stream) {
  if (!d || !d_diag) return fail(SEM_E_INVALID, "null argument");
  DeviceGuard g(d->device);
  SEM_TRY(dd_begin(d, op_kind, true, nullptr, d_diag, S(stream)));
  SEM_TRY(dd_exchange(d));
  return dd_finish(d, d_diag, S(stream));
}

int sem_dd_pcg_solve(sem_dd* d, int op_kind, const double* d_b, double* d_x,
                     const uint8_t* d_dirichlet, double rtol, int max_iter, int check_every,
                     int* iters, double* final_relres, void* stream) {
  if (!d) return fail(SEM_E_INVALID, "null dd");
  PcgOp op;
  op.dd = d;
  op.n = d->ndof;
  op.device = d->device;
  return pcg_run(op, op_kind, d_b, d_x, d_dirichlet, d->d_notown, rtol, max_iter, check_every,
                 iters, final_relres, S(stream));
}

}  // extern "C"
