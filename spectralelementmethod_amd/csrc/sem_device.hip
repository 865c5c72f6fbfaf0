// Device half of libsem_hip.so: the operator context, the geometry kernel,
// the matrix-free operator kernels and the C ABI that launches them.
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
// CDNA4 mapping: one wavefront owns EPW = floor(64 / n)
// elements, lane = (element slot, line j).  Contractions along the lane's own
// column/row run in registers with D read as wave-uniform scalars (kernel
// arguments -> SGPRs); the two transposes go through a wave-private LDS tile,
// so no workgroup barrier is ever needed.  The element map and the geometric
// factors are repacked at setup into [group][row][lane] order so that every
// wave-instruction streams one contiguous run of HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
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

namespace {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
constexpr int WAVES_PER_BLOCK = BLOCK / WAVE;

inline int epw_of(int n) { return WAVE / n; }

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

// ---------------------------------------------------------------------------
// Poisson stiffness action
// ---------------------------------------------------------------------------
// Packed layouts (built by k_pack_map / k_geometry):
//   mapP[g][r][k*N + j]        = map[g*EPW + k][r][j]
//   GP  [g][c][r][k*N + j]     = factor c at node (r, j) of element g*EPW + k
// with LW = EPW*N values per (g, r).  Padding elements map to node 0 with
// zero factors and are masked at the scatter.
template <int N, bool ALL_ATOMIC>
__global__ void __launch_bounds__(BLOCK)
    k_poisson_apply(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                    const double* __restrict__ u, double* __restrict__ y, int64_t n_groups,
                    int64_t n_elem, int accumulate, const DMat<N> D) {
  constexpr int EPW = WAVE / N;
  constexpr int LW = EPW * N;
  constexpr int SLOTS = (WAVE + N - 1) / N;   // every lane owns a tile slot
  constexpr int RS = (N % 2) ? N + 1 : N;     // 16-B aligned rows
  constexpr int ES = N * RS;
  __shared__ __attribute__((aligned(16))) double lds[WAVES_PER_BLOCK * SLOTS * ES];

  const int wave = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int64_t g = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wave;
  if (g >= n_groups) return;  // whole wavefront leaves; no block barriers below
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < LW;
  const bool active = in_wave && (g * EPW + k < n_elem);
  double* L = lds + (wave * SLOTS + k) * ES;

  const uint32_t* mp = mapP + g * (int64_t)(N * LW) + lane;
  const double* gp = GP + g * (int64_t)(3 * N * LW) + lane;

  uint32_t gid[N];
  double uc[N];
#pragma unroll
  for (int r = 0; r < N; ++r) gid[r] = in_wave ? mp[r * LW] : 0u;
#pragma unroll
  for (int r = 0; r < N; ++r) uc[r] = in_wave ? u[gid[r]] : 0.0;

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
    const double2* row = reinterpret_cast<const double2*>(L + j * RS);
#pragma unroll
    for (int s = 0; s < RS / 2; ++s) {
      const double2 v = row[s];
      ur[2 * s] = v.x;
      ur[2 * s + 1] = v.y;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < N; ++s) a = fma(D.v[q * N + s], ur[s], a);
      t[q] = a;
    }
  }
  wave_sync();
  {
    double2* row = reinterpret_cast<double2*>(L + j * RS);
#pragma unroll
    for (int s = 0; s < N / 2; ++s) row[s] = make_double2(t[2 * s], t[2 * s + 1]);
    if (N % 2) L[j * RS + N - 1] = t[N - 1];
  }
  wave_sync();

  // column j: geometric factors, w0/w1, and ya = D^T w0 along xi0
  double ya[N];
  double w1[N];
  {
    double w0[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
      const double d1 = L[m * RS + j];
      const double g00 = gp[(0 * N + m) * LW];
      const double g01 = gp[(1 * N + m) * LW];
      const double g11 = gp[(2 * N + m) * LW];
      w0[m] = fma(g00, d0[m], g01 * d1);
      w1[m] = fma(g01, d0[m], g11 * d1);
    }
#pragma unroll
    for (int p = 0; p < N; ++p) {
      double a = 0.0;
#pragma unroll
      for (int m = 0; m < N; ++m) a = fma(D.v[m * N + p], w0[m], a);
      ya[p] = a;
    }
  }
  wave_sync();
#pragma unroll
  for (int m = 0; m < N; ++m) L[m * RS + j] = w1[m];
  wave_sync();

  // row i = j: yb[i][q] = sum_n D[n][q] w1[i][n]
  {
    double wr[RS];
    const double2* row = reinterpret_cast<const double2*>(L + j * RS);
#pragma unroll
    for (int s = 0; s < RS / 2; ++s) {
      const double2 v = row[s];
      wr[2 * s] = v.x;
      wr[2 * s + 1] = v.y;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      double a = 0.0;
#pragma unroll
      for (int nn = 0; nn < N; ++nn) a = fma(D.v[nn * N + q], wr[nn], a);
      t[q] = a;
    }
  }
  wave_sync();
  {
    double2* row = reinterpret_cast<double2*>(L + j * RS);
#pragma unroll
    for (int s = 0; s < N / 2; ++s) row[s] = make_double2(t[2 * s], t[2 * s + 1]);
    if (N % 2) L[j * RS + N - 1] = t[N - 1];
  }
  wave_sync();

  // column j: y[p][j] = ya[p] + yb[p][j]; scatter-add through the map.
  // Element-boundary nodes may be shared -> atomic; interior nodes of a
  // conforming mesh belong to this element only -> plain store.
  if (active) {
    const bool edge_col = (j == 0) || (j == N - 1);
#pragma unroll
    for (int p = 0; p < N; ++p) {
      const double v = ya[p] + L[p * RS + j];
      double* dst = y + gid[p];
      if (ALL_ATOMIC || p == 0 || p == N - 1 || edge_col) {
        atomic_add_f64(dst, v);
      } else if (accumulate) {
        *dst += v;
      } else {
        *dst = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Axisymmetric Stokes block (Re = 0), dpn = 2 interleaved (psi, omega):
//   y[2k]   = Lve.omega      = stiff_rho(omega) + (W/rho) omega
//   y[2k+1] = E2e.psi - Me.omega = stiff_rho(psi) + 2W(iJ00 d0 + iJ10 d1)psi - rho^2 W omega
// (examples/squirmer-axisymmetric.py:193-227, 253-254, 278-295)
// factors per node: 0 G00rho 1 G01rho 2 G11rho 3 b0=2W iJ00 4 b1=2W iJ10 5 c=W/rho 6 m=rho^2 W
// ---------------------------------------------------------------------------
template <int N, bool ALL_ATOMIC>
__global__ void __launch_bounds__(BLOCK)
    k_axisym_apply(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                   const double* __restrict__ u, double* __restrict__ y, int64_t n_groups,
                   int64_t n_elem, int accumulate, const DMat<N> D) {
  constexpr int EPW = WAVE / N;
  constexpr int LW = EPW * N;
  constexpr int SLOTS = (WAVE + N - 1) / N;
  constexpr int RS = (N % 2) ? N + 1 : N;
  constexpr int ES = 2 * N * RS;  // two fields per tile
  __shared__ __attribute__((aligned(16))) double lds[WAVES_PER_BLOCK * SLOTS * ES];

  const int wave = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int64_t g = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wave;
  if (g >= n_groups) return;
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < LW;
  const bool active = in_wave && (g * EPW + k < n_elem);
  double* LP = lds + (wave * SLOTS + k) * ES;  // psi tile
  double* LO = LP + N * RS;                     // omega tile

  const uint32_t* mp = mapP + g * (int64_t)(N * LW) + lane;
  const double* gp = GP + g * (int64_t)(7 * N * LW) + lane;
  const double2* u2 = reinterpret_cast<const double2*>(u);

  uint32_t gid[N];
  double ps[N], om[N];
#pragma unroll
  for (int r = 0; r < N; ++r) gid[r] = in_wave ? mp[r * LW] : 0u;
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const double2 v = in_wave ? u2[gid[r]] : make_double2(0.0, 0.0);
    ps[r] = v.x;
    om[r] = v.y;
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
  // row phase: d1 for both fields
  {
    double tp[N], to[N];
    double rp[RS], ro[RS];
    const double2* rowp = reinterpret_cast<const double2*>(LP + j * RS);
    const double2* rowo = reinterpret_cast<const double2*>(LO + j * RS);
#pragma unroll
    for (int s = 0; s < RS / 2; ++s) {
      const double2 a = rowp[s], b = rowo[s];
      rp[2 * s] = a.x;
      rp[2 * s + 1] = a.y;
      ro[2 * s] = b.x;
      ro[2 * s + 1] = b.y;
    }
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
#pragma unroll
    for (int q = 0; q < N; ++q) {
      LP[j * RS + q] = tp[q];
      LO[j * RS + q] = to[q];
    }
  }
  wave_sync();
  // column phase: factors, pointwise terms, ya along xi0
  double yap[N], yao[N], w1p[N], w1o[N];
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
      // pointwise (test index = node (m, j)): psi row gets 2W gx(psi) - rho^2 W omega,
      // omega row gets (W/rho) omega
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
      yap[p] = a + d0p[p];
      yao[p] = b + d0o[p];
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
    const double2* rowp = reinterpret_cast<const double2*>(LP + j * RS);
    const double2* rowo = reinterpret_cast<const double2*>(LO + j * RS);
#pragma unroll
    for (int s = 0; s < RS / 2; ++s) {
      const double2 a = rowp[s], b = rowo[s];
      rp[2 * s] = a.x;
      rp[2 * s + 1] = a.y;
      ro[2 * s] = b.x;
      ro[2 * s + 1] = b.y;
    }
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
#pragma unroll
    for (int q = 0; q < N; ++q) {
      LP[j * RS + q] = tp[q];
      LO[j * RS + q] = to[q];
    }
  }
  wave_sync();
  if (active) {
    const bool edge_col = (j == 0) || (j == N - 1);
#pragma unroll
    for (int p = 0; p < N; ++p) {
      // row 2k <- omega equation (Lve.omega), row 2k+1 <- psi equation
      const double vo = yao[p] + LO[p * RS + j];
      const double vp = yap[p] + LP[p * RS + j];
      double* dst = y + 2 * (int64_t)gid[p];
      if (ALL_ATOMIC || p == 0 || p == N - 1 || edge_col) {
        atomic_add_f64(dst, vo);
        atomic_add_f64(dst + 1, vp);
      } else {
        double2* d2 = reinterpret_cast<double2*>(dst);
        if (accumulate) {
          double2 o = *d2;
          *d2 = make_double2(o.x + vo, o.y + vp);
        } else {
          *d2 = make_double2(vo, vp);
        }
      }
    }
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
               const double* __restrict__ gw, int op_kind, double* __restrict__ GP,
               double* __restrict__ xph, double* __restrict__ Jo, double* __restrict__ iJo,
               double* __restrict__ dJo, double* __restrict__ dJW,
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
    const int64_t gg = e / EPW;
    const int kk = (int)(e - gg * EPW);
    const int ncomp = (op_kind == SEM_OP_POISSON) ? 3 : 7;
    double* o = GP + gg * (int64_t)(ncomp * N * LW) + m * LW + kk * N + nq;
    const double A00 = iJ00 * iJ00 + iJ01 * iJ01;
    const double A01 = iJ00 * iJ10 + iJ01 * iJ11;
    const double A11 = iJ10 * iJ10 + iJ11 * iJ11;
    if (op_kind == SEM_OP_POISSON) {
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

// user-supplied factors [E][ncomp][n][n] -> packed
__global__ void k_pack_geom(const double* __restrict__ G, int64_t n_elem, int n, int ncomp,
                            int epw, double* __restrict__ GP) {
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
    const int64_t gg = e / epw;
    const int kk = (int)(e - gg * epw);
    GP[((gg * ncomp + c) * n + r) * lw + kk * n + jj] = G[t];
  }
}

__global__ void k_pack_map(const uint32_t* __restrict__ e2n, int64_t n_elem, int n, int epw,
                           int64_t n_groups, uint32_t* __restrict__ mapP) {
  const int lw = epw * n;
  const int64_t total = n_groups * n * lw;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t gg = t / (n * lw);
    const int rem = (int)(t - gg * n * lw);
    const int r = rem / lw;
    const int lane = rem - r * lw;
    const int kk = lane / n, jj = lane - kk * n;
    const int64_t e = gg * epw + kk;
    mapP[t] = (e < n_elem) ? e2n[(e * n + r) * n + jj] : 0u;
  }
}

// reference counts: cnt[node] = total references, bnd[node] = 1 if referenced
// as an element-boundary local node
__global__ void k_node_refs(const uint32_t* __restrict__ e2n, int64_t n_elem, int n,
                            int64_t n_node, unsigned* __restrict__ cnt,
                            unsigned char* __restrict__ bnd, unsigned* __restrict__ n_oob) {
  const int64_t nn = (int64_t)n * n;
  const int64_t total = n_elem * nn;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t gi = e2n[t];
    if ((int64_t)gi >= n_node) {
      atomicAdd(n_oob, 1u);
      continue;
    }
    const int node = (int)(t % nn);
    const int r = node / n, jj = node - r * n;
    atomicAdd(cnt + gi, 1u);
    if (r == 0 || r == n - 1 || jj == 0 || jj == n - 1) bnd[gi] = 1;
  }
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
                               const double* __restrict__ gD, int n, int epw, int64_t n_elem,
                               double* __restrict__ diag) {
  __shared__ double sD[SEM_MAXN * SEM_MAXN];
  for (int i = threadIdx.x; i < n * n; i += blockDim.x) sD[i] = gD[i];
  __syncthreads();
  const int lw = epw * n;
  const int64_t total = n_elem * n * n;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / (n * n);
    const int node = (int)(t - e * n * n);
    const int p = node / n, q = node - p * n;
    const int64_t gg = e / epw;
    const int kk = (int)(e - gg * epw);
    const double* G = GP + gg * (int64_t)(3 * n * lw) + kk * n;
    double s = 0.0;
    for (int m = 0; m < n; ++m) s += sD[m * n + p] * sD[m * n + p] * G[(0 * n + m) * lw + q];
    for (int nn = 0; nn < n; ++nn) s += sD[nn * n + q] * sD[nn * n + q] * G[(2 * n + p) * lw + nn];
    s += 2.0 * sD[p * n + p] * sD[q * n + q] * G[(1 * n + p) * lw + q];
    const uint32_t gi = mapP[(gg * n + p) * lw + kk * n + q];
    atomic_add_f64(diag + gi, s);
  }
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

// ---- CG vector kernels (deterministic two-stage reductions) ----
constexpr int RED_BLOCKS = 1024;

__device__ double block_sum(double v) {
  __shared__ double sh[BLOCK / WAVE];
  for (int o = WAVE / 2; o > 0; o >>= 1) v += __shfl_down(v, o, WAVE);
  if ((threadIdx.x & (WAVE - 1)) == 0) sh[threadIdx.x / WAVE] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < BLOCK / WAVE; ++w) s += sh[w];
  __syncthreads();
  return s;
}

// partial[b] = sum a[i]*b[i] over the block's grid-stride slice (two dots at once)
__global__ void __launch_bounds__(BLOCK) k_dot2(const double* __restrict__ a,
                                                const double* __restrict__ b,
                                                const double* __restrict__ c,
                                                const double* __restrict__ d, int64_t n,
                                                double* __restrict__ partial) {
  double s0 = 0.0, s1 = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    s0 = fma(a[t], b[t], s0);
    if (c) s1 = fma(c[t], d[t], s1);
  }
  s0 = block_sum(s0);
  s1 = block_sum(s1);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = s0;
    partial[gridDim.x + blockIdx.x] = s1;
  }
}

__global__ void __launch_bounds__(BLOCK) k_finish2(const double* __restrict__ partial, int nb,
                                                   double* __restrict__ out) {
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    s0 += partial[i];
    s1 += partial[nb + i];
  }
  s0 = block_sum(s0);
  s1 = block_sum(s1);
  if (threadIdx.x == 0) {
    out[0] = s0;
    out[1] = s1;
  }
}

// r = mask ? 0 : b - r   (r holds K x on entry)
__global__ void k_residual(const double* __restrict__ b, double* __restrict__ r,
                           const uint8_t* __restrict__ mask, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    r[t] = mask[t] ? 0.0 : b[t] - r[t];
}

// z = r / diag on free DOFs, 0 on Dirichlet
__global__ void k_precond(const double* __restrict__ r, const double* __restrict__ diag,
                          const uint8_t* __restrict__ mask, int64_t n, double* __restrict__ z) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    z[t] = mask[t] ? 0.0 : r[t] / diag[t];
}

__global__ void k_mask(double* __restrict__ q, const uint8_t* __restrict__ mask, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    if (mask[t]) q[t] = 0.0;
}

// x += alpha p ; r -= alpha q
__global__ void k_update_xr(double* __restrict__ x, double* __restrict__ r,
                            const double* __restrict__ p, const double* __restrict__ q,
                            const double* __restrict__ scal, int64_t n) {
  const double alpha = scal[0];
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    x[t] = fma(alpha, p[t], x[t]);
    r[t] = fma(-alpha, q[t], r[t]);
  }
}

// p = z + beta p
__global__ void k_update_p(double* __restrict__ p, const double* __restrict__ z,
                           const double* __restrict__ scal, int64_t n) {
  const double beta = scal[1];
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    p[t] = fma(beta, p[t], z[t]);
}

// out[b][m][q] = sum_{r,s} A0[m][r] A1[q][s] in[b][r][s]  (A = NULL -> identity)
// TensorProduct.deriv / gradient (D(x)I, I(x)D; sem/basis_functions.py:626-650),
// compute_coeffs_grid_eq (Vinv(x)Vinv; :599-624), interpolate_on_grid_eq (:539-569).
__global__ void k_tensor_apply(int n, int64_t batch, const double* __restrict__ gA0,
                               const double* __restrict__ gA1, const double* __restrict__ in,
                               double* __restrict__ out) {
  __shared__ double sA0[SEM_MAXN * SEM_MAXN], sA1[SEM_MAXN * SEM_MAXN];
  __shared__ double tile[SEM_MAXN * SEM_MAXN];
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

inline int grid_for(int64_t n, int per_block = BLOCK, int cap = 8192) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct sem_ctx {
  int p = 0, n = 0, dpn = 1, device = 0;
  int64_t n_elem = 0, n_node = 0;
  int epw = 0, lw = 0;
  int64_t n_groups = 0;
  double hD[SEM_MAXN * SEM_MAXN];
  double hw[SEM_MAXN];
  bool have_basis = false;
  double* d_D = nullptr;
  double* d_w = nullptr;
  double* d_Vinv = nullptr;
  uint32_t* d_mapP = nullptr;
  const uint32_t* d_e2n = nullptr;
  uint32_t* d_zero = nullptr;  // nodes whose y entries are not fully overwritten
  int64_t n_zero = 0;
  bool interior_unique = true;
  double* d_GP[2] = {nullptr, nullptr};
  // CG scratch
  double* d_cg = nullptr;
  int64_t cg_len = 0;
  double* d_red = nullptr;
  unsigned long long* d_bad = nullptr;
};

namespace {

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

template <int N>
DMat<N> make_dmat(const double* h) {
  DMat<N> d;
  std::memcpy(d.v, h, sizeof(d.v));
  return d;
}

template <int N>
int launch_apply_n(sem_ctx* c, int op_kind, const double* u, double* y, int acc, hipStream_t st) {
  const DMat<N> D = make_dmat<N>(c->hD);
  const int grid = (int)((c->n_groups + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
  if (op_kind == SEM_OP_POISSON) {
    if (c->interior_unique)
      hipLaunchKernelGGL((k_poisson_apply<N, false>), dim3(grid), dim3(BLOCK), 0, st, c->d_mapP,
                         c->d_GP[0], u, y, c->n_groups, c->n_elem, acc, D);
    else
      hipLaunchKernelGGL((k_poisson_apply<N, true>), dim3(grid), dim3(BLOCK), 0, st, c->d_mapP,
                         c->d_GP[0], u, y, c->n_groups, c->n_elem, acc, D);
  } else {
    if (c->interior_unique)
      hipLaunchKernelGGL((k_axisym_apply<N, false>), dim3(grid), dim3(BLOCK), 0, st, c->d_mapP,
                         c->d_GP[1], u, y, c->n_groups, c->n_elem, acc, D);
    else
      hipLaunchKernelGGL((k_axisym_apply<N, true>), dim3(grid), dim3(BLOCK), 0, st, c->d_mapP,
                         c->d_GP[1], u, y, c->n_groups, c->n_elem, acc, D);
  }
  return SEM_OK;
}

template <int N>
void launch_geom_n(sem_ctx* c, const double* nodes, int op_kind, double* GP, double* xph,
                   double* J, double* iJ, double* dJ, double* dJW, hipStream_t st) {
  using Sh = GeomShape<N>;
  const int grid = (int)((c->n_elem + Sh::EPB - 1) / Sh::EPB);
  hipLaunchKernelGGL((k_geometry<N>), dim3(grid), dim3(Sh::THREADS), 0, st, nodes, c->n_node,
                     c->d_e2n, c->n_elem, c->d_Vinv, c->d_D, c->d_w, op_kind, GP, xph, J, iJ, dJ,
                     dJW, c->d_bad);
}

#define SEM_DISPATCH_N(n, FN, ...)                          \
  switch (n) {                                              \
    case 2: FN<2>(__VA_ARGS__); break;                      \
    case 3: FN<3>(__VA_ARGS__); break;                      \
    case 4: FN<4>(__VA_ARGS__); break;                      \
    case 5: FN<5>(__VA_ARGS__); break;                      \
    case 6: FN<6>(__VA_ARGS__); break;                      \
    case 7: FN<7>(__VA_ARGS__); break;                      \
    case 8: FN<8>(__VA_ARGS__); break;                      \
    case 9: FN<9>(__VA_ARGS__); break;                      \
    case 10: FN<10>(__VA_ARGS__); break;                    \
    case 11: FN<11>(__VA_ARGS__); break;                    \
    case 12: FN<12>(__VA_ARGS__); break;                    \
    case 13: FN<13>(__VA_ARGS__); break;                    \
    case 14: FN<14>(__VA_ARGS__); break;                    \
    case 15: FN<15>(__VA_ARGS__); break;                    \
    case 16: FN<16>(__VA_ARGS__); break;                    \
    case 17: FN<17>(__VA_ARGS__); break;                    \
    default: break;                                         \
  }

int check_op(sem_ctx* c, int op_kind) {
  if (op_kind == SEM_OP_POISSON) {
    if (c->dpn != 1) return fail(SEM_E_INVALID, "Poisson operator needs dofs_per_node == 1");
    return SEM_OK;
  }
  if (op_kind == SEM_OP_AXISYM_STOKES) {
    if (c->dpn != 2)
      return fail(SEM_E_INVALID, "axisymmetric Stokes block needs dofs_per_node == 2");
    return SEM_OK;
  }
  return fail(SEM_E_INVALID, "unknown op_kind " + std::to_string(op_kind));
}

int ensure_gp(sem_ctx* c, int op_kind) {
  const int slot = op_kind == SEM_OP_POISSON ? 0 : 1;
  if (!c->d_GP[slot]) {
    const int ncomp = sem_op_ncomp(op_kind);
    const size_t bytes = (size_t)c->n_groups * ncomp * c->n * c->lw * sizeof(double);
    HIP_TRY(hipMalloc(&c->d_GP[slot], bytes));
    HIP_TRY(hipMemset(c->d_GP[slot], 0, bytes));
  }
  return SEM_OK;
}

}  // namespace

extern "C" {

int sem_ctx_create(sem_ctx** out, int p, int64_t n_elem, int64_t n_node, int dpn, int device) {
  if (!out) return fail(SEM_E_INVALID, "null ctx pointer");
  *out = nullptr;
  if (p < 1) return fail(SEM_E_INVALID, "Must specify an order of 1 or greater.");
  if (p > SEM_MAX_ORDER)
    return fail(SEM_E_NOTIMPL, "operator kernels built for orders 1.." +
                                   std::to_string(SEM_MAX_ORDER));
  if (n_elem < 1 || n_node < 1 || dpn < 1 || dpn > 2)
    return fail(SEM_E_INVALID, "bad sizes (n_elem, n_node >= 1, dpn in {1,2})");
  if (n_node > 0xFFFFFFFFll) return fail(SEM_E_INVALID, "n_node exceeds uint32 map range");
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
  hipError_t e1 = hipMalloc(&c->d_D, SEM_MAXN * SEM_MAXN * sizeof(double));
  hipError_t e2 = hipMalloc(&c->d_w, SEM_MAXN * sizeof(double));
  hipError_t e3 = hipMalloc(&c->d_Vinv, SEM_MAXN * SEM_MAXN * sizeof(double));
  hipError_t e4 = hipMalloc(&c->d_bad, sizeof(unsigned long long));
  hipError_t e5 = hipMalloc(&c->d_red, (2 * RED_BLOCKS + 8) * sizeof(double));
  if (e1 || e2 || e3 || e4 || e5) {
    sem_ctx_destroy(c);
    return fail(SEM_E_HIP, "hipMalloc failed in sem_ctx_create");
  }
  *out = c;
  return SEM_OK;
}

void sem_ctx_destroy(sem_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  (void)hipFree(c->d_D);
  (void)hipFree(c->d_w);
  (void)hipFree(c->d_Vinv);
  (void)hipFree(c->d_mapP);
  (void)hipFree(c->d_zero);
  (void)hipFree(c->d_GP[0]);
  (void)hipFree(c->d_GP[1]);
  (void)hipFree(c->d_cg);
  (void)hipFree(c->d_red);
  (void)hipFree(c->d_bad);
  delete c;
}

int sem_set_basis(sem_ctx* c, const double* hD, const double* hw) {
  if (!c || !hD || !hw) return fail(SEM_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  const int n = c->n;
  std::memcpy(c->hD, hD, sizeof(double) * n * n);
  std::memcpy(c->hw, hw, sizeof(double) * n);
  HIP_TRY(hipMemcpy(c->d_D, hD, sizeof(double) * n * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_w, hw, sizeof(double) * n, hipMemcpyHostToDevice));
  c->have_basis = true;
  return SEM_OK;
}

int sem_set_map(sem_ctx* c, const uint32_t* d_e2n, void* stream) {
  if (!c || !d_e2n) return fail(SEM_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  const int n = c->n;
  c->d_e2n = d_e2n;
  if (!c->d_mapP) HIP_TRY(hipMalloc(&c->d_mapP, (size_t)c->n_groups * n * c->lw * sizeof(uint32_t)));
  hipLaunchKernelGGL(k_pack_map, dim3(grid_for(c->n_groups * n * c->lw)), dim3(BLOCK), 0, st,
                     d_e2n, c->n_elem, n, c->epw, c->n_groups, c->d_mapP);
  HIP_TRY(hipGetLastError());
  // node classification: which y entries are not overwritten by a unique
  // interior store (element-boundary nodes and unreferenced nodes).
  unsigned* d_cnt = nullptr;
  unsigned char* d_bnd = nullptr;
  unsigned* d_oob = nullptr;
  HIP_TRY(hipMalloc(&d_cnt, c->n_node * sizeof(unsigned)));
  HIP_TRY(hipMalloc(&d_bnd, c->n_node));
  HIP_TRY(hipMalloc(&d_oob, sizeof(unsigned)));
  HIP_TRY(hipMemsetAsync(d_cnt, 0, c->n_node * sizeof(unsigned), st));
  HIP_TRY(hipMemsetAsync(d_bnd, 0, c->n_node, st));
  HIP_TRY(hipMemsetAsync(d_oob, 0, sizeof(unsigned), st));
  hipLaunchKernelGGL(k_node_refs, dim3(grid_for(c->n_elem * n * n)), dim3(BLOCK), 0, st, d_e2n,
                     c->n_elem, n, c->n_node, d_cnt, d_bnd, d_oob);
  std::vector<unsigned> cnt(c->n_node);
  std::vector<unsigned char> bnd(c->n_node);
  unsigned oob = 0;
  HIP_TRY(hipMemcpyAsync(cnt.data(), d_cnt, c->n_node * sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(bnd.data(), d_bnd, c->n_node, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&oob, d_oob, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  (void)hipFree(d_cnt);
  (void)hipFree(d_bnd);
  (void)hipFree(d_oob);
  if (oob) return fail(SEM_E_INVALID, "element map references node >= n_node");
  std::vector<uint32_t> zero;
  bool unique = true;
  for (int64_t i = 0; i < c->n_node; ++i) {
    if (bnd[i] || cnt[i] == 0) {
      zero.push_back((uint32_t)i);
    } else if (cnt[i] != 1) {
      unique = false;  // an element-interior node referenced twice: non-conforming
    }
  }
  c->interior_unique = unique;
  if (!unique) {
    // every entry goes through atomics: zero all nodes
    zero.resize(c->n_node);
    for (int64_t i = 0; i < c->n_node; ++i) zero[i] = (uint32_t)i;
  }
  (void)hipFree(c->d_zero);
  c->d_zero = nullptr;
  c->n_zero = (int64_t)zero.size();
  if (c->n_zero) {
    HIP_TRY(hipMalloc(&c->d_zero, zero.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(c->d_zero, zero.data(), zero.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  return SEM_OK;
}

static int geom_common(sem_ctx* c, const double* d_nodes, const double* h_Vinv) {
  if (!c || !d_nodes || !h_Vinv) return fail(SEM_E_INVALID, "null argument");
  if (!c->have_basis) return fail(SEM_E_STATE, "sem_set_basis must precede geometry");
  if (!c->d_e2n) return fail(SEM_E_STATE, "sem_set_map must precede geometry");
  HIP_TRY(hipMemcpy(c->d_Vinv, h_Vinv, sizeof(double) * c->n * c->n, hipMemcpyHostToDevice));
  return SEM_OK;
}

int sem_geom_from_nodes(sem_ctx* c, const double* d_nodes, const double* h_Vinv, int op_kind,
                        int64_t* n_bad_nodes, void* stream) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  DeviceGuard g(c->device);
  int rc = geom_common(c, d_nodes, h_Vinv);
  if (rc) return rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if ((rc = ensure_gp(c, op_kind))) return rc;
  hipStream_t st = S(stream);
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  double* GP = c->d_GP[op_kind == SEM_OP_POISSON ? 0 : 1];
  SEM_DISPATCH_N(c->n, launch_geom_n, c, d_nodes, op_kind, GP, nullptr, nullptr, nullptr, nullptr,
                 nullptr, st);
  HIP_TRY(hipGetLastError());
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, c->d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (n_bad_nodes) *n_bad_nodes = (int64_t)bad;
  if (bad) return fail(SEM_E_DETJ, "detJ <= 0 at " + std::to_string(bad) + " quadrature nodes");
  return SEM_OK;
}

int sem_geom_fields(sem_ctx* c, const double* d_nodes, const double* h_Vinv, double* x_phys,
                    double* J, double* invJ, double* detJ, double* detJxW, void* stream) {
  if (!c) return fail(SEM_E_INVALID, "null ctx");
  DeviceGuard g(c->device);
  int rc = geom_common(c, d_nodes, h_Vinv);
  if (rc) return rc;
  hipStream_t st = S(stream);
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  SEM_DISPATCH_N(c->n, launch_geom_n, c, d_nodes, SEM_OP_POISSON, nullptr, x_phys, J, invJ, detJ,
                 detJxW, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  return SEM_OK;
}

int sem_set_geom(sem_ctx* c, const double* d_G, int op_kind, void* stream) {
  if (!c || !d_G) return fail(SEM_E_INVALID, "null argument");
  DeviceGuard g(c->device);
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if ((rc = ensure_gp(c, op_kind))) return rc;
  const int ncomp = sem_op_ncomp(op_kind);
  hipLaunchKernelGGL(k_pack_geom, dim3(grid_for(c->n_elem * ncomp * c->n * c->n)), dim3(BLOCK), 0,
                     S(stream), d_G, c->n_elem, c->n, ncomp, c->epw,
                     c->d_GP[op_kind == SEM_OP_POISSON ? 0 : 1]);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

int sem_zero_shared(sem_ctx* c, double* y, void* stream) {
  if (!c || !y) return fail(SEM_E_INVALID, "null argument");
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
  if (flags & ~(SEM_APPLY_ACCUMULATE | SEM_APPLY_SKIP_ZERO))
    return fail(SEM_E_INVALID, "unknown sem_apply flags");
  int rc;
  if ((rc = check_op(c, op_kind))) return rc;
  if (!c->have_basis || !c->d_mapP) return fail(SEM_E_STATE, "basis and map must be set");
  if (!c->d_GP[op_kind == SEM_OP_POISSON ? 0 : 1])
    return fail(SEM_E_STATE, "geometry for this operator has not been computed");
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  const int accumulate = flags & SEM_APPLY_ACCUMULATE;
  if (!accumulate && !(flags & SEM_APPLY_SKIP_ZERO) && c->n_zero)
    hipLaunchKernelGGL(k_zero_list, dim3(grid_for(c->n_zero, BLOCK, 4096)), dim3(BLOCK), 0, st, y,
                       c->d_zero, c->n_zero, c->dpn);
  SEM_DISPATCH_N(c->n, launch_apply_n, c, op_kind, u, y, accumulate, st);
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
  if (!c->d_GP[0] || !c->d_mapP) return fail(SEM_E_STATE, "geometry/map not set");
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  HIP_TRY(hipMemsetAsync(d_diag, 0, c->n_node * sizeof(double), st));
  hipLaunchKernelGGL(k_poisson_diag, dim3(grid_for(c->n_elem * c->n * c->n)), dim3(BLOCK), 0, st,
                     c->d_mapP, c->d_GP[0], c->d_D, c->n, c->epw, c->n_elem, d_diag);
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

int sem_pcg_solve(sem_ctx* c, int op_kind, const double* b, double* x, const uint8_t* mask,
                  double rtol, int max_iter, int* iters, double* relres, void* stream) {
  if (!c || !b || !x || !mask) return fail(SEM_E_INVALID, "null argument");
  if (op_kind != SEM_OP_POISSON) return fail(SEM_E_NOTIMPL, "sem_pcg_solve: Poisson only");
  DeviceGuard g(c->device);
  hipStream_t st = S(stream);
  const int64_t n = c->n_node;
  if (c->cg_len != n) {
    (void)hipFree(c->d_cg);
    HIP_TRY(hipMalloc(&c->d_cg, 4 * n * sizeof(double)));
    c->cg_len = n;
  }
  double* r = c->d_cg;
  double* z = r + n;
  double* p = z + n;
  double* q = p + n;
  // Jacobi diagonal (allocated per solve; setup cost)
  double* d_diag = nullptr;
  HIP_TRY(hipMalloc(&d_diag, n * sizeof(double)));
  int rc = sem_diag(c, op_kind, d_diag, stream);
  if (rc) {
    (void)hipFree(d_diag);
    return rc;
  }
  double* partial = c->d_red;
  double* scal = c->d_red + 2 * RED_BLOCKS;  // [alpha, beta, dot0, dot1]
  const int gb = grid_for(n, BLOCK, RED_BLOCKS);
  auto dot2 = [&](const double* a1, const double* b1, const double* a2, const double* b2,
                  double* out2) -> int {
    hipLaunchKernelGGL(k_dot2, dim3(gb), dim3(BLOCK), 0, st, a1, b1, a2, b2, n, partial);
    hipLaunchKernelGGL(k_finish2, dim3(1), dim3(BLOCK), 0, st, partial, gb, scal + 2);
    HIP_TRY(hipMemcpyAsync(out2, scal + 2, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SEM_OK;
  };
  // r = b - K x on free rows
  if ((rc = sem_apply(c, op_kind, x, r, 0, stream))) goto done;
  hipLaunchKernelGGL(k_residual, dim3(grid_for(n)), dim3(BLOCK), 0, st, b, r, mask, n);
  hipLaunchKernelGGL(k_precond, dim3(grid_for(n)), dim3(BLOCK), 0, st, r, d_diag, mask, n, z);
  HIP_TRY(hipMemcpyAsync(p, z, n * sizeof(double), hipMemcpyDeviceToDevice, st));
  {
    double h[2];
    if ((rc = dot2(r, z, r, r, h))) goto done;
    double rz = h[0];
    const double r0 = std::sqrt(h[1]);
    double res = r0;
    int it = 0;
    if (r0 == 0.0) {
      if (iters) *iters = 0;
      if (relres) *relres = 0.0;
      goto done;
    }
    while (it < max_iter && res > rtol * r0) {
      if ((rc = sem_apply(c, op_kind, p, q, 0, stream))) goto done;
      hipLaunchKernelGGL(k_mask, dim3(grid_for(n)), dim3(BLOCK), 0, st, q, mask, n);
      if ((rc = dot2(p, q, nullptr, nullptr, h))) goto done;
      const double alpha = rz / h[0];
      double hs[2] = {alpha, 0.0};
      HIP_TRY(hipMemcpyAsync(scal, hs, 2 * sizeof(double), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_update_xr, dim3(grid_for(n)), dim3(BLOCK), 0, st, x, r, p, q, scal, n);
      hipLaunchKernelGGL(k_precond, dim3(grid_for(n)), dim3(BLOCK), 0, st, r, d_diag, mask, n, z);
      if ((rc = dot2(r, z, r, r, h))) goto done;
      const double beta = h[0] / rz;
      rz = h[0];
      res = std::sqrt(h[1]);
      hs[0] = alpha;
      hs[1] = beta;
      HIP_TRY(hipMemcpyAsync(scal, hs, 2 * sizeof(double), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_update_p, dim3(grid_for(n)), dim3(BLOCK), 0, st, p, z, scal, n);
      ++it;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (iters) *iters = it;
    if (relres) *relres = res / r0;
    if (res > rtol * r0) rc = fail(SEM_E_INVALID, "PCG did not converge");
  }
done:
  (void)hipFree(d_diag);
  return rc;
}

}  // extern "C"
