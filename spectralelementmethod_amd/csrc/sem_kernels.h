// Device kernels of libsem_hip.so (included once, by sem_device.hip).
//
// Hot path (BASELINE.json north_star):
//   for every element e:  u_e = u[map[e]]                       (gather)
//                         d0 = D u_e,  d1 = u_e D^T              (D(x)I, I(x)D)
//                         w0 = G00 d0 + G01 d1, w1 = G01 d0 + G11 d1
//                         y_e = D^T w0 + w1 D                    (transposed pass)
//                         y[map[e]] += y_e                       (scatter-add)
// which equals the reference's per-element dense action
// einsum('pqrs,rs', Lse, u[loc]) (examples/poisson.py:168-193,
// examples/squirmer-axisymmetric.py:286) to rounding.
//
// CDNA4 mapping:
//  * GROUP = one wavefront's EPW = floor(64 / n) elements; lane = (element
//    slot k, line j).  Contractions along the lane's own column/row run in
//    registers with D as wave-uniform kernel arguments (SGPRs); the two
//    transposes go through a wave-private LDS tile.
//  * CHAIN = R rounds x 4 consecutive groups, processed by one 256-thread
//    workgroup (round by round, one group per wavefront).  Consecutive groups
//    of a chain usually share one column of nodes: the earlier group hands its
//    partial sums for that column to the later one through LDS ("carry"), so
//    every node has exactly one writer inside a chain and consecutive y rows
//    are completed by one workgroup (one XCD's L2), close in time.
//  * Chains are coloured at setup so that chains of one colour share no node;
//    one launch per colour.  Every packed map entry carries a 4-bit write code:
//    plain store for the first writer of a node in launch order,
//    read-modify-write for later writers, skip + register merge for a node
//    shared by the elements on two neighbouring lanes, carry-in for the node
//    handed over by the previous group, atomic only as a fallback.  No
//    atomics on structured (or any locality-ordered conforming) meshes.
//  * the map and the geometric factors are repacked at setup into
//    [group][row][lane] order: every wave-instruction streams one contiguous
//    run of HBM.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace semk {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
#ifndef SEM_CHAIN_WAVES
#define SEM_CHAIN_WAVES 4
#endif
constexpr int CHAIN_WAVES = SEM_CHAIN_WAVES;  // groups per round = wavefronts per workgroup
constexpr int CHAIN_BLOCK = CHAIN_WAVES * WAVE;
constexpr int MAXN = 17;

// packed map entry = gid | code << CODE_SHIFT
constexpr int CODE_SHIFT = 28;
constexpr uint32_t GID_MASK = (1u << CODE_SHIFT) - 1u;
constexpr uint32_t W_STORE = 0;   // first writer: y = v   (y += v in accumulate mode)
constexpr uint32_t W_RMW = 1;     // later writer: y += v (no concurrent writer)
constexpr uint32_t W_SKIP = 2;    // value merged into another lane / padding
constexpr uint32_t W_ATOMIC = 3;  // fallback
constexpr uint32_t W_MERGE = 4;   // add the next lane's value before writing
constexpr uint32_t W_CARRY = 8;   // add the value handed over by the previous group

#ifndef SEM_POISSON_MIN_WAVES
#define SEM_POISSON_MIN_WAVES 1
#endif

template <int N>
struct DMat {
  double v[N * N];
};

// Ordering point for LDS traffic between lanes of ONE wavefront (a wave's LDS
// operations complete in issue order; this only stops the compiler moving
// them across the exchange).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void atomic_add_f64(double* p, double v) {
  unsafeAtomicAdd(p, v);  // global_atomic_add_f64, no return
}

// Read-modify-write targets were written earlier by this workgroup or by an
// earlier launch: read them past the CU's vector L1 (nt) so a line cached
// before the workgroup's own store is never reused.
__device__ __forceinline__ double rmw_load(const double* p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ void emit1(double* __restrict__ y, uint32_t raw, double v,
                                      int accumulate) {
  const uint32_t a = (raw >> CODE_SHIFT) & 3u;
  double* dst = y + (raw & GID_MASK);
  if (a == W_STORE) {
    *dst = accumulate ? rmw_load(dst) + v : v;
  } else if (a == W_RMW) {
    *dst = rmw_load(dst) + v;
  } else if (a == W_ATOMIC) {
    atomic_add_f64(dst, v);
  }
}

__device__ __forceinline__ void emit2(double* __restrict__ y, uint32_t raw, double v0, double v1,
                                      int accumulate) {
  const uint32_t a = (raw >> CODE_SHIFT) & 3u;
  double* dst = y + 2 * (int64_t)(raw & GID_MASK);
  if ((a == W_STORE && !accumulate)) {
    *reinterpret_cast<double2*>(dst) = make_double2(v0, v1);
  } else if (a == W_STORE || a == W_RMW) {
    const double o0 = rmw_load(dst), o1 = rmw_load(dst + 1);
    *reinterpret_cast<double2*>(dst) = make_double2(o0 + v0, o1 + v1);
  } else if (a == W_ATOMIC) {
    atomic_add_f64(dst, v0);
    atomic_add_f64(dst + 1, v1);
  }
}

// row i of the tile (16-B aligned, RS doubles) -> registers
template <int N, int RS>
__device__ __forceinline__ void load_row(const double* L, int i, double (&r)[RS]) {
  const double2* row = reinterpret_cast<const double2*>(L + i * RS);
#pragma unroll
  for (int s = 0; s < RS / 2; ++s) {
    const double2 v = row[s];
    r[2 * s] = v.x;
    r[2 * s + 1] = v.y;
  }
}

template <int N, int RS>
__device__ __forceinline__ void store_row(double* L, int i, const double (&t)[N]) {
  double2* row = reinterpret_cast<double2*>(L + i * RS);
#pragma unroll
  for (int s = 0; s < N / 2; ++s) row[s] = make_double2(t[2 * s], t[2 * s + 1]);
  if (N % 2) L[i * RS + N - 1] = t[N - 1];
}

template <int N>
struct Tile {
  static constexpr int EPW = WAVE / N;
  static constexpr int LW = EPW * N;
  static constexpr int SLOTS = (WAVE + N - 1) / N;  // every lane owns a tile slot
  static constexpr int RS = (N % 2) ? N + 1 : N;    // 16-B aligned rows
  static constexpr int ES = N * RS;
};

// ---------------------------------------------------------------------------
// One group of the Poisson action: returns y_e[p][j] (p = 0..N-1) of the
// lane's column j in v[], and the raw coded map entries in raw[].
//   mapP[g][r][k*N + j] = map[e][r][j] | code,  GP[g][c][r][k*N + j] = G_c(e; r, j)
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void poisson_group(const uint32_t* __restrict__ mapP,
                                              const double* __restrict__ GP,
                                              const double* __restrict__ u, int64_t g, int lane,
                                              int j, bool in_wave, double* L, const DMat<N>& D,
                                              uint32_t (&raw)[N], double (&v)[N]) {
  using T = Tile<N>;
  constexpr int LW = T::LW;
  constexpr int RS = T::RS;
  const uint32_t* mp = mapP + g * (int64_t)(N * LW) + lane;
  const double* gp = GP + g * (int64_t)(3 * N * LW) + lane;
  double uc[N];
#pragma unroll
  for (int r = 0; r < N; ++r) raw[r] = in_wave ? mp[r * LW] : (W_SKIP << CODE_SHIFT);
#pragma unroll
  for (int r = 0; r < N; ++r) {
#ifdef SEM_DIAG_NO_U
    uc[r] = (double)(raw[r] & 7u);  // timing-only: no u gather
#else
    uc[r] = u[raw[r] & GID_MASK];
#endif
  }
  // column j: d0[m][j] = sum_r D[m][r] u[r][j]     (TensorProduct.deriv dim 0)
  double d0[N];
#pragma unroll
  for (int m = 0; m < N; ++m) {
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < N; ++r) a = fma(D.v[m * N + r], uc[r], a);
    d0[m] = a;
  }
#pragma unroll
  for (int r = 0; r < N; ++r) L[r * RS + j] = uc[r];
  wave_sync();
  // row i = j: d1[i][q] = sum_s D[q][s] u[i][s]     (TensorProduct.deriv dim 1)
  double t[N];
  {
    double ur[RS];
    load_row<N, RS>(L, j, ur);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < N; ++s) a = fma(D.v[q * N + s], ur[s], a);
      t[q] = a;
    }
  }
  wave_sync();
  store_row<N, RS>(L, j, t);
  wave_sync();
  // column j: geometric factors, w0/w1, and ya = D^T w0 along xi0 (kept in v)
  double w1[N];
  {
    double w0[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
      const double d1 = L[m * RS + j];
#ifdef SEM_DIAG_NO_G
      const double g00 = 1.0 + m, g01 = 0.25 * j, g11 = 2.0;  // timing-only
#else
      const double g00 = gp[(0 * N + m) * LW];
      const double g01 = gp[(1 * N + m) * LW];
      const double g11 = gp[(2 * N + m) * LW];
#endif
      w0[m] = fma(g00, d0[m], g01 * d1);
      w1[m] = fma(g01, d0[m], g11 * d1);
    }
#pragma unroll
    for (int p = 0; p < N; ++p) {
      double a = 0.0;
#pragma unroll
      for (int m = 0; m < N; ++m) a = fma(D.v[m * N + p], w0[m], a);
      v[p] = a;
    }
  }
  wave_sync();
#pragma unroll
  for (int m = 0; m < N; ++m) L[m * RS + j] = w1[m];
  wave_sync();
  // row i = j: yb[i][q] = sum_n D[n][q] w1[i][n]
  {
    double wr[RS];
    load_row<N, RS>(L, j, wr);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double a = 0.0;
#pragma unroll
      for (int nn = 0; nn < N; ++nn) a = fma(D.v[nn * N + q], wr[nn], a);
      t[q] = a;
    }
  }
  wave_sync();
  store_row<N, RS>(L, j, t);
  wave_sync();
#pragma unroll
  for (int p = 0; p < N; ++p) v[p] += L[p * RS + j];
  wave_sync();  // the tile is rewritten by the next group of this wave
}

// Scatter of one group's column values through the coded map, with the
// in-group merge (next lane) and the chain carry (previous group) applied.
// ncomp values per node (1: Poisson, 2: axisymmetric block).
template <int N, int NC>
__device__ __forceinline__ void chain_emit(double* __restrict__ y, const uint32_t (&raw)[N],
                                           double (&v)[NC][N], int lane, int wave, int rd,
                                           bool in_wave, double (*carry)[CHAIN_WAVES][NC][N],
                                           int accumulate) {
  constexpr int LW = Tile<N>::LW;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int p = 0; p < N; ++p) {
      const double vn = __shfl_down(v[c][p], 1, WAVE);
      if ((raw[p] >> CODE_SHIFT) & W_MERGE) v[c][p] += vn;
    }
  // hand the last lane's column to the next group of the chain
  if (lane == LW - 1) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int p = 0; p < N; ++p) carry[rd & 1][wave][c][p] = v[c][p];
  }
  __syncthreads();
  if (lane == 0) {
    const double* src = (wave > 0) ? &carry[rd & 1][wave - 1][0][0]
                                   : &carry[(rd + 1) & 1][CHAIN_WAVES - 1][0][0];
#pragma unroll
    for (int p = 0; p < N; ++p)
      if ((raw[p] >> CODE_SHIFT) & W_CARRY) {
#pragma unroll
        for (int c = 0; c < NC; ++c) v[c][p] += src[c * N + p];
      }
  }
  if (in_wave) {
#pragma unroll
    for (int p = 0; p < N; ++p) {
      if (NC == 1)
        emit1(y, raw[p], v[0][p], accumulate);
      else
        emit2(y, raw[p], v[0][p], v[NC - 1][p], accumulate);
    }
  }
  // this round's stores and carry reads complete before the next round
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Poisson stiffness action: one workgroup per chain, chains [c0, c1).
// ---------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(CHAIN_BLOCK, SEM_POISSON_MIN_WAVES)
    k_poisson_apply(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                    const double* __restrict__ u, double* __restrict__ y, int64_t c0, int64_t c1,
                    int rounds, int accumulate, const DMat<N> D) {
  using T = Tile<N>;
  __shared__ __attribute__((aligned(16))) double lds[CHAIN_WAVES * T::SLOTS * T::ES];
  __shared__ double carry[2][CHAIN_WAVES][1][N];
  const int64_t chain = c0 + blockIdx.x;
  if (chain >= c1) return;  // uniform over the workgroup
  const int wave = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < T::LW;
  double* L = lds + (wave * T::SLOTS + k) * T::ES;
  for (int rd = 0; rd < rounds; ++rd) {
    const int64_t g = (chain * rounds + rd) * CHAIN_WAVES + wave;
    uint32_t raw[N];
    double v[1][N];
    poisson_group<N>(mapP, GP, u, g, lane, j, in_wave, L, D, raw, v[0]);
#ifdef SEM_DIAG_NO_STORE
    if (in_wave && v[0][0] == 1234.5678) y[0] = v[0][1];  // timing-only
#else
    chain_emit<N, 1>(y, raw, v, lane, wave, rd, in_wave, carry, accumulate);
#endif
  }
}

// ---------------------------------------------------------------------------
// Axisymmetric Stokes block (Re = 0), dpn = 2 interleaved (psi, omega):
//   y[2k]   = Lve.omega          = stiff_rho(omega) + (W/rho) omega
//   y[2k+1] = E2e.psi - Me.omega = stiff_rho(psi) + 2W(iJ00 d0 + iJ10 d1)psi - rho^2 W omega
// (examples/squirmer-axisymmetric.py:193-227, 253-254, 278-295)
// factors: 0 G00rho 1 G01rho 2 G11rho 3 b0=2W iJ00 4 b1=2W iJ10 5 c=W/rho 6 m=rho^2 W
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void axisym_group(const uint32_t* __restrict__ mapP,
                                             const double* __restrict__ GP,
                                             const double* __restrict__ u, int64_t g, int lane,
                                             int j, bool in_wave, double* LP, double* LO,
                                             const DMat<N>& D, uint32_t (&raw)[N],
                                             double (&vo)[N], double (&vp)[N]) {
  using T = Tile<N>;
  constexpr int LW = T::LW;
  constexpr int RS = T::RS;
  const uint32_t* mp = mapP + g * (int64_t)(N * LW) + lane;
  const double* gp = GP + g * (int64_t)(7 * N * LW) + lane;
  const double2* u2 = reinterpret_cast<const double2*>(u);
  double ps[N], om[N];
#pragma unroll
  for (int r = 0; r < N; ++r) raw[r] = in_wave ? mp[r * LW] : (W_SKIP << CODE_SHIFT);
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const double2 val = u2[raw[r] & GID_MASK];
    ps[r] = val.x;
    om[r] = val.y;
  }
  double d0p[N], d0o[N];
#pragma unroll
  for (int m = 0; m < N; ++m) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int r = 0; r < N; ++r) {
      a = fma(D.v[m * N + r], ps[r], a);
      b = fma(D.v[m * N + r], om[r], b);
    }
    d0p[m] = a;
    d0o[m] = b;
  }
#pragma unroll
  for (int r = 0; r < N; ++r) {
    LP[r * RS + j] = ps[r];
    LO[r * RS + j] = om[r];
  }
  wave_sync();
  {
    double tp[N], to[N];
    double rp[RS], ro[RS];
    load_row<N, RS>(LP, j, rp);
    load_row<N, RS>(LO, j, ro);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int s = 0; s < N; ++s) {
        a = fma(D.v[q * N + s], rp[s], a);
        b = fma(D.v[q * N + s], ro[s], b);
      }
      tp[q] = a;
      to[q] = b;
    }
    wave_sync();
    store_row<N, RS>(LP, j, tp);
    store_row<N, RS>(LO, j, to);
  }
  wave_sync();
  double w1p[N], w1o[N];
  {
    double w0p[N], w0o[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
      const double d1p = LP[m * RS + j];
      const double d1o = LO[m * RS + j];
      const double g00 = gp[(0 * N + m) * LW];
      const double g01 = gp[(1 * N + m) * LW];
      const double g11 = gp[(2 * N + m) * LW];
      const double b0 = gp[(3 * N + m) * LW];
      const double b1 = gp[(4 * N + m) * LW];
      const double c = gp[(5 * N + m) * LW];
      const double mm = gp[(6 * N + m) * LW];
      w0p[m] = fma(g00, d0p[m], g01 * d1p);
      w1p[m] = fma(g01, d0p[m], g11 * d1p);
      w0o[m] = fma(g00, d0o[m], g01 * d1o);
      w1o[m] = fma(g01, d0o[m], g11 * d1o);
      // pointwise terms at test node (m, j): psi row 2W gx(psi) - rho^2 W omega,
      // omega row (W/rho) omega
      d0p[m] = fma(b0, d0p[m], fma(b1, d1p, -mm * om[m]));
      d0o[m] = c * om[m];
    }
#pragma unroll
    for (int p = 0; p < N; ++p) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int m = 0; m < N; ++m) {
        a = fma(D.v[m * N + p], w0p[m], a);
        b = fma(D.v[m * N + p], w0o[m], b);
      }
      vp[p] = a + d0p[p];
      vo[p] = b + d0o[p];
    }
  }
  wave_sync();
#pragma unroll
  for (int m = 0; m < N; ++m) {
    LP[m * RS + j] = w1p[m];
    LO[m * RS + j] = w1o[m];
  }
  wave_sync();
  {
    double tp[N], to[N];
    double rp[RS], ro[RS];
    load_row<N, RS>(LP, j, rp);
    load_row<N, RS>(LO, j, ro);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int nn = 0; nn < N; ++nn) {
        a = fma(D.v[nn * N + q], rp[nn], a);
        b = fma(D.v[nn * N + q], ro[nn], b);
      }
      tp[q] = a;
      to[q] = b;
    }
    wave_sync();
    store_row<N, RS>(LP, j, tp);
    store_row<N, RS>(LO, j, to);
  }
  wave_sync();
#pragma unroll
  for (int p = 0; p < N; ++p) {
    vo[p] += LO[p * RS + j];
    vp[p] += LP[p * RS + j];
  }
  wave_sync();
}

template <int N>
__global__ void __launch_bounds__(CHAIN_BLOCK)
    k_axisym_apply(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                   const double* __restrict__ u, double* __restrict__ y, int64_t c0, int64_t c1,
                   int rounds, int accumulate, const DMat<N> D) {
  using T = Tile<N>;
  __shared__ __attribute__((aligned(16))) double lds[CHAIN_WAVES * T::SLOTS * 2 * T::ES];
  __shared__ double carry[2][CHAIN_WAVES][2][N];
  const int64_t chain = c0 + blockIdx.x;
  if (chain >= c1) return;
  const int wave = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < T::LW;
  double* LP = lds + (wave * T::SLOTS + k) * 2 * T::ES;  // psi tile
  double* LO = LP + T::ES;                               // omega tile
  for (int rd = 0; rd < rounds; ++rd) {
    const int64_t g = (chain * rounds + rd) * CHAIN_WAVES + wave;
    uint32_t raw[N];
    double v[2][N];  // [0] omega row (y[2k]), [1] psi row (y[2k+1])
    axisym_group<N>(mapP, GP, u, g, lane, j, in_wave, LP, LO, D, raw, v[0], v[1]);
    chain_emit<N, 2>(y, raw, v, lane, wave, rd, in_wave, carry, accumulate);
  }
}

// ---------------------------------------------------------------------------
// Geometry: nodes -> x_phys -> J -> det/inv -> W -> operator factors.
// Thread per local node, EPB elements per block, LDS staging (setup path).
// ---------------------------------------------------------------------------
template <int N>
struct GeomShape {
  static constexpr int NN = N * N;
  static constexpr int EPB = (NN >= 256) ? 1 : 256 / NN;
  static constexpr int THREADS = ((EPB * NN + 63) / 64) * 64;
};

template <int N>
__global__ void __launch_bounds__(GeomShape<N>::THREADS)
    k_geometry(const double* __restrict__ nodes, int64_t n_node, const uint32_t* __restrict__ e2n,
               int64_t n_elem, const double* __restrict__ gVinv, const double* __restrict__ gD,
               const double* __restrict__ gw, int op_kind, const int* __restrict__ gpos,
               double* __restrict__ GP, double* __restrict__ xph, double* __restrict__ Jo,
               double* __restrict__ iJo, double* __restrict__ dJo, double* __restrict__ dJW,
               unsigned long long* __restrict__ n_bad) {
  using S = GeomShape<N>;
  constexpr int NN = S::NN;
  constexpr int EPB = S::EPB;
  constexpr int EPW = WAVE / N;
  constexpr int LW = EPW * N;
  __shared__ double sV[NN], sD[NN], sw[N];
  __shared__ double sx[EPB][2][NN], st[EPB][2][NN];
  const int tid = threadIdx.x;
  for (int i = tid; i < NN; i += blockDim.x) {
    sV[i] = gVinv[i];
    sD[i] = gD[i];
  }
  if (tid < N) sw[tid] = gw[tid];
  const int el = tid / NN;
  const int node = tid - el * NN;
  const int m = node / N;
  const int nq = node - m * N;
  const int64_t e = (int64_t)blockIdx.x * EPB + el;
  const bool act = (el < EPB) && (e < n_elem);
  if (act) {
    const uint32_t gi = e2n[e * NN + node];
    sx[el][0][node] = nodes[gi];
    sx[el][1][node] = nodes[n_node + gi];
  }
  __syncthreads();
  // x_phys = Vinv X Vinv^T   (compute_coeffs_grid_eq: dim 0 then dim 1),
  // evaluated on coordinates relative to the element's node (0,0): the map
  // is translation invariant (V_eq reproduces constants) and J = D x_phys
  // then no longer cancels the O(1) offset against O(h) variations.
  double x0[2] = {0.0, 0.0};
  if (act) {
    x0[0] = sx[el][0][0];
    x0[1] = sx[el][1][0];
    for (int c = 0; c < 2; ++c) {
      double a = 0.0;
      for (int i = 0; i < N; ++i) a = fma(sV[m * N + i], sx[el][c][i * N + nq] - x0[c], a);
      st[el][c][node] = a;
    }
  }
  __syncthreads();
  double xp[2] = {0.0, 0.0};
  if (act) {
    for (int c = 0; c < 2; ++c) {
      double a = 0.0;
      for (int jj = 0; jj < N; ++jj) a = fma(sV[nq * N + jj], st[el][c][m * N + jj], a);
      xp[c] = a;
    }
  }
  __syncthreads();
  if (act) {
    sx[el][0][node] = xp[0];
    sx[el][1][node] = xp[1];
  }
  __syncthreads();
  if (!act) return;
  // J[c][d] = d x_c / d xi_d (TensorProduct.gradient, swapaxes(0,1))
  double J[2][2];
  for (int c = 0; c < 2; ++c) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < N; ++r) {
      a = fma(sD[m * N + r], sx[el][c][r * N + nq], a);
      b = fma(sD[nq * N + r], sx[el][c][m * N + r], b);
    }
    J[c][0] = a;
    J[c][1] = b;
  }
  // det_inv_2x2 (sem/linalg.py:105-115)
  const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
  const double rdet = 1.0 / det;
  const double iJ00 = J[1][1] * rdet, iJ01 = -J[0][1] * rdet;
  const double iJ10 = -J[1][0] * rdet, iJ11 = J[0][0] * rdet;
  // detJxW via TensorQuadratureRule.xweight (sem/quadratures.py:268-275)
  const double W = det * sw[m] * sw[nq];
  if (!(det > 0.0)) atomicAdd(n_bad, 1ull);
  const int64_t base = e * NN + node;
  const double xabs0 = xp[0] + x0[0];
  const double xabs1 = xp[1] + x0[1];
  if (xph) {
    xph[(e * 2 + 0) * NN + node] = xabs0;
    xph[(e * 2 + 1) * NN + node] = xabs1;
  }
  if (Jo) {
    Jo[(e * 4 + 0) * NN + node] = J[0][0];
    Jo[(e * 4 + 1) * NN + node] = J[0][1];
    Jo[(e * 4 + 2) * NN + node] = J[1][0];
    Jo[(e * 4 + 3) * NN + node] = J[1][1];
  }
  if (iJo) {
    iJo[(e * 4 + 0) * NN + node] = iJ00;
    iJo[(e * 4 + 1) * NN + node] = iJ01;
    iJo[(e * 4 + 2) * NN + node] = iJ10;
    iJo[(e * 4 + 3) * NN + node] = iJ11;
  }
  if (dJo) dJo[base] = det;
  if (dJW) dJW[base] = W;
  if (GP) {
    const int64_t grp = e / EPW;
    const int kk = (int)(e - grp * EPW);
    const int64_t gg = gpos[grp];
    const int ncomp = (op_kind == 0) ? 3 : 7;
    double* o = GP + gg * (int64_t)(ncomp * N * LW) + m * LW + kk * N + nq;
    const double A00 = iJ00 * iJ00 + iJ01 * iJ01;
    const double A01 = iJ00 * iJ10 + iJ01 * iJ11;
    const double A11 = iJ10 * iJ10 + iJ11 * iJ11;
    if (op_kind == 0) {
      o[0 * N * LW] = W * A00;
      o[1 * N * LW] = W * A01;
      o[2 * N * LW] = W * A11;
    } else {
      const double rho = xabs0;
      const double rW = rho * W;
      o[0 * N * LW] = rW * A00;
      o[1 * N * LW] = rW * A01;
      o[2 * N * LW] = rW * A11;
      o[3 * N * LW] = 2.0 * W * iJ00;
      o[4 * N * LW] = 2.0 * W * iJ10;
      o[5 * N * LW] = W / rho;
      o[6 * N * LW] = rW * rho;
    }
  }
}

}  // namespace semk
