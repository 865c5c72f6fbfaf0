// Static condensation on the device: the element Schur complements of
// DOFManagerSC.compute_local_sc_system / assemble_global_sc_system
// (sem/discrete.py:428-500) for every element in one launch, and the interior
// back-solve of DOFManagerSC._solve_interior_dofs (sem/discrete.py:512-524).
//
// A local system in hierarchical order (exterior DOFs first, ne of them,
// then ni interior DOFs) is
//        [A_ee A_ei] [x_e]   [b_e]
//        [A_ie A_ii] [x_i] = [b_i]
// and the reference forms, per element with LAPACK (scipy linalg.solve),
//   S = A_ee - A_ei A_ii^-1 A_ie,   s = b_e - A_ei A_ii^-1 b_i,
//   x_i = A_ii^-1 (b_i - A_ie x_e).
// Here one workgroup owns one element: Gauss-Jordan elimination with partial
// pivoting of [A_ii | A_ie | b_i] in a per-element workspace (row-major,
// W = ni + ne + 1 columns; L2-resident while the workgroup runs), leaving
// X = A_ii^-1 [A_ie | b_i] in its right columns, then S and s as dot
// products of A_ei rows with X columns.  X is kept for the back-solve, so
// the interior solve is one batched matrix-vector product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "sem_internal.h"

using sem::fail;

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(SEM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
  } while (0)

namespace {

constexpr int SCB = 256;  // threads per workgroup (one element)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

__global__ void __launch_bounds__(SCB)
    k_sc_condense(int64_t n_elem, int nl, int ne, const double* __restrict__ mat,
                  const double* __restrict__ rhs, double* __restrict__ work,
                  double* __restrict__ sc_mat, double* __restrict__ sc_rhs,
                  unsigned long long* __restrict__ n_singular) {
  const int ni = nl - ne;
  const int W = ni + ne + 1;
  __shared__ double s_val[SCB];
  __shared__ int s_idx[SCB];
  __shared__ int s_piv;
  __shared__ double s_fac[512];  // column k of the workspace (ni <= 512)
  for (int64_t e = blockIdx.x; e < n_elem; e += gridDim.x) {
    const double* A = mat + e * (int64_t)nl * nl;
    const double* b = rhs + e * (int64_t)nl;
    double* X = work + e * (int64_t)ni * W;
    // [A_ii | A_ie | b_i]
    for (int t = threadIdx.x; t < ni * W; t += SCB) {
      const int i = t / W, j = t - i * W;
      const int row = ne + i;
      X[t] = j < ni ? A[(int64_t)row * nl + ne + j]
                    : (j < ni + ne ? A[(int64_t)row * nl + (j - ni)] : b[row]);
    }
    // The reference (scipy linalg.solve, check_finite=False) raises when the
    // interior block holds a NaN or an off-diagonal inf (LAPACK reports the
    // block singular or an illegal value) but lets an infinite diagonal entry
    // through: that unknown decouples (1/inf = 0).  Same rule here; non-finite
    // couplings A_ie, A_ei, b propagate into S and s.
    bool bad_block = false;
    for (int t = threadIdx.x; t < ni * ni; t += SCB) {
      const int i = t / ni, j = t - i * ni;
      const double a = X[(int64_t)i * W + j];
      bad_block |= isnan(a) || (isinf(a) && i != j);
    }
    bool singular = __syncthreads_or(bad_block);
    for (int k = 0; k < ni && !singular; ++k) {
      // partial pivoting: largest |X[r][k]|, r >= k (first index on ties, like LAPACK)
      double best = -1.0;
      int bi = k;
      for (int r = k + threadIdx.x; r < ni; r += SCB) {
        const double a = fabs(X[(int64_t)r * W + k]);
        if (a > best) {
          best = a;
          bi = r;
        }
      }
      s_val[threadIdx.x] = best;
      s_idx[threadIdx.x] = bi;
      __syncthreads();
      for (int o = SCB / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
          const double v2 = s_val[threadIdx.x + o];
          const int i2 = s_idx[threadIdx.x + o];
          if (v2 > s_val[threadIdx.x] || (v2 == s_val[threadIdx.x] && i2 < s_idx[threadIdx.x])) {
            s_val[threadIdx.x] = v2;
            s_idx[threadIdx.x] = i2;
          }
        }
        __syncthreads();
      }
      if (threadIdx.x == 0) s_piv = s_idx[0];
      const double pv = s_val[0];
      __syncthreads();
      // an exactly zero pivot column is singular (LAPACK gesv info > 0)
      if (pv == 0.0) {
        singular = true;
        continue;
      }
      const int piv = s_piv;
      if (piv != k)
        for (int j = threadIdx.x; j < W; j += SCB) {
          const double t = X[(int64_t)k * W + j];
          X[(int64_t)k * W + j] = X[(int64_t)piv * W + j];
          X[(int64_t)piv * W + j] = t;
        }
      __syncthreads();
      const double inv = 1.0 / X[(int64_t)k * W + k];
      __syncthreads();
      for (int j = k + threadIdx.x; j < W; j += SCB) X[(int64_t)k * W + j] *= inv;
      for (int i = threadIdx.x; i < ni; i += SCB) s_fac[i] = X[(int64_t)i * W + k];
      __syncthreads();
      const int wk = W - k;
      for (int t = threadIdx.x; t < ni * wk; t += SCB) {
        const int i = t / wk, j = k + (t - i * wk);
        if (i != k) X[(int64_t)i * W + j] -= s_fac[i] * X[(int64_t)k * W + j];
      }
      __syncthreads();
    }
    if (singular && threadIdx.x == 0) atomicAdd(n_singular, 1ull);
    // S = A_ee - A_ei X[:, :ne],  s = b_e - A_ei X[:, ne]
    double* So = sc_mat + e * (int64_t)ne * ne;
    double* so = sc_rhs + e * (int64_t)ne;
    for (int t = threadIdx.x; t < ne * (ne + 1); t += SCB) {
      const int a = t / (ne + 1), c = t - a * (ne + 1);
      double acc = c < ne ? A[(int64_t)a * nl + c] : b[a];
      for (int i = 0; i < ni; ++i) acc = fma(-A[(int64_t)a * nl + ne + i], X[(int64_t)i * W + ni + c], acc);
      if (c < ne)
        So[(int64_t)a * ne + c] = acc;
      else
        so[a] = acc;
    }
    __syncthreads();  // the workspace of the next element of this workgroup
  }
}

// x_i = X[:, ne] - X[:, :ne] x_e  (the right columns of the workspace)
__global__ void k_sc_backsolve(int64_t n_elem, int ni, int ne, const double* __restrict__ work,
                               const double* __restrict__ xe, double* __restrict__ xi) {
  const int W = ni + ne + 1;
  const int64_t total = n_elem * ni;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / ni;
    const int i = (int)(t - e * ni);
    const double* X = work + (e * ni + i) * (int64_t)W + ni;
    const double* x = xe + e * ne;
    double acc = X[ne];
    for (int c = 0; c < ne; ++c) acc = fma(-X[c], x[c], acc);
    xi[t] = acc;
  }
}

// ---------------------------------------------------------------------------
// Banded LU with partial pivoting for the condensed exterior system when it
// is not symmetric (the axisymmetric Stokes / Navier-Stokes block that
// examples/squirmer-axisymmetric.py:299-387 condenses; the reference solves
// it with scipy.sparse.linalg.spsolve, sem/discrete.py:502-511).  The caller
// orders the unknowns by reverse Cuthill-McKee (as the reference orders its
// nodes, sem/discrete.py:169-178, 400), so the matrix is banded with lower /
// upper bandwidths kl / ku; row interchanges widen U to KU = kl + ku.
// Column-major band storage: entry (i, k) at AB[k * W + i - k + KU],
// W = KU + kl + 1 (LAPACK gbtrf's layout, without its separate kl rows).
// ---------------------------------------------------------------------------
constexpr int BLU = 1024;  // threads of the one factorising workgroup

__global__ void k_band_fill(int64_t n, int KU, int W, const int64_t* __restrict__ rowptr,
                            const int32_t* __restrict__ colind, const double* __restrict__ val,
                            double* __restrict__ AB) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    for (int64_t t = rowptr[i]; t < rowptr[i + 1]; ++t) {
      const int64_t k = colind[t];
      AB[k * W + (i - k + KU)] += val[t];  // duplicates summed (COO semantics)
    }
}

// The elimination is a chain of n dependent steps.  Step j: the pivot
// search over the kl + 1 entries of column j (fixed order: the largest
// |a|, the lowest row on ties), the row swap over KU + 1 columns, the
// multipliers (they replace column j below the diagonal, LAPACK's in-place
// L, so any kl fits) and b's update -- band_pivot, one workgroup -- then
// the rank-1 update of the kl x KU block below and right of the pivot --
// band_update.  b is eliminated alongside; then the column-oriented back
// substitution (U's column j above the diagonal is contiguous in this
// layout).  info = j + 1 for an exactly zero pivot in column j (LAPACK's
// convention), 0 otherwise.
//
// Two schedules, bitwise the same result (every entry gets the same fma in
// the same order of steps; tests/test_gpu_facade.py):
//  * narrow bands: the whole chain in one workgroup (k_band_lu_solve), the
//    update spread over its 1024 threads -- 2.8 us per step at kl = ku = 8
//    at any n, 6.6 at 64, but the update is one CU's work: 62 us per step at
//    kl = ku = 256, 452 us at 1024 (profiles/r06/band_lu_timing.json);
//  * wide bands (kl * (kl + ku) >= SEM_BAND_STEP_MIN, default 12288, or
//    SEM_BAND_LU_STEPS=1): two launches per step on the caller's stream,
//    band_pivot in one workgroup and band_update over the whole device,
//    then the back substitution in one workgroup -- 7.1-7.4 us per step
//    (launch-bound) from kl = ku = 8 to 256, 15.6 at 1024.
__device__ __forceinline__ bool band_pivot(int64_t n, int kl, int KU, int W,
                                           double* __restrict__ AB, double* __restrict__ b,
                                           int* __restrict__ info, int64_t j, double* s_val,
                                           int* s_idx) {
  const int tid = threadIdx.x;
  const int64_t ilast = min<int64_t>(n - 1, j + kl);
  const int nr = (int)(ilast - j);  // rows below the diagonal
  double best = -1.0;
  int bi = 0;
  for (int r = tid; r <= nr; r += BLU) {
    const double a = fabs(AB[j * W + r + KU]);
    if (a > best) {
      best = a;
      bi = r;
    }
  }
  s_val[tid] = best;
  s_idx[tid] = bi;
  __syncthreads();
  for (int o = BLU / 2; o > 0; o >>= 1) {
    if (tid < o) {
      const double v2 = s_val[tid + o];
      const int i2 = s_idx[tid + o];
      if (v2 > s_val[tid] || (v2 == s_val[tid] && i2 < s_idx[tid])) {
        s_val[tid] = v2;
        s_idx[tid] = i2;
      }
    }
    __syncthreads();
  }
  const double pv = s_val[0];
  const int p = s_idx[0];
  if (!(pv > 0.0)) {  // exactly zero (or NaN) pivot column
    if (tid == 0) *info = (int)(j + 1);
    return false;     // uniform: every thread read the same s_val[0]
  }
  const int64_t klast = min<int64_t>(n - 1, j + KU);
  if (p != 0) {
    for (int64_t k = j + tid; k <= klast; k += BLU) {
      double* a = AB + k * W + (j - k + KU);
      const double t = a[0];
      a[0] = a[p];
      a[p] = t;
    }
    if (tid == 0) {
      const double t = b[j];
      b[j] = b[j + p];
      b[j + p] = t;
    }
  }
  __syncthreads();
  const double inv = 1.0 / AB[j * W + KU];
  const double bj = b[j];
  double* lcol = AB + j * W + KU;  // (j + r, j) at lcol[r]
  for (int r = 1 + tid; r <= nr; r += BLU) {
    const double l = lcol[r] * inv;
    lcol[r] = l;
    b[j + r] = fma(-l, bj, b[j + r]);
  }
  return true;
}

// A(j + r, j + c) -= l_r A(j, j + c) for r in [1, nr], c in [1, nc]: entries
// t0, t0 + stride, ... of the nr x nc block, r fastest (a column of the
// block is contiguous in the band layout)
__device__ __forceinline__ void band_update(int64_t n, int kl, int KU, int W,
                                            double* __restrict__ AB, int64_t j, int64_t t0,
                                            int64_t stride) {
  const int nr = (int)(min<int64_t>(n - 1, j + kl) - j);
  const int nc = (int)(min<int64_t>(n - 1, j + KU) - j);
  const double* lcol = AB + j * W + KU;
  const int64_t tot = (int64_t)nr * nc;
  for (int64_t t = t0; t < tot; t += stride) {
    const int c = 1 + (int)(t / nr), r = 1 + (int)(t % nr);
    double* col = AB + (j + c) * W + (KU - c);  // (i, j + c) at col[i - j]
    col[r] = fma(-lcol[r], col[0], col[r]);
  }
}

__device__ __forceinline__ void band_backsub(int64_t n, int KU, int W,
                                             const double* __restrict__ AB,
                                             double* __restrict__ b, double* __restrict__ x) {
  const int tid = threadIdx.x;
  for (int64_t j = n - 1; j >= 0; --j) {
    const double xj = b[j] / AB[j * W + KU];
    __syncthreads();  // every thread read b[j] before it can change again
    if (tid == 0) x[j] = xj;
    const int64_t i0 = max<int64_t>(0, j - KU);
    for (int64_t i = i0 + tid; i < j; i += BLU) b[i] = fma(-AB[j * W + (i - j + KU)], xj, b[i]);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(BLU)
    k_band_lu_solve(int64_t n, int kl, int KU, int W, double* __restrict__ AB,
                    double* __restrict__ b, double* __restrict__ x, int* __restrict__ info) {
  __shared__ double s_val[BLU];
  __shared__ int s_idx[BLU];
  for (int64_t j = 0; j < n; ++j) {
    if (!band_pivot(n, kl, KU, W, AB, b, info, j, s_val, s_idx)) return;
    __syncthreads();
    band_update(n, kl, KU, W, AB, j, threadIdx.x, BLU);
    __syncthreads();
  }
  band_backsub(n, KU, W, AB, b, x);
  if (threadIdx.x == 0) *info = 0;
}

// the wide-band schedule: one launch of each per step, then k_band_backsub;
// a step after a zero pivot does nothing (info is set)
__global__ void __launch_bounds__(BLU)
    k_band_step_pivot(int64_t n, int kl, int KU, int W, double* __restrict__ AB,
                      double* __restrict__ b, int* __restrict__ info, int64_t j) {
  __shared__ double s_val[BLU];
  __shared__ int s_idx[BLU];
  if (*info) return;  // uniform
  band_pivot(n, kl, KU, W, AB, b, info, j, s_val, s_idx);
}

constexpr int BLU_UPD = 256;
__global__ void __launch_bounds__(BLU_UPD)
    k_band_step_update(int64_t n, int kl, int KU, int W, double* __restrict__ AB,
                       const int* __restrict__ info, int64_t j) {
  if (*info) return;  // uniform
  band_update(n, kl, KU, W, AB, j, (int64_t)blockIdx.x * BLU_UPD + threadIdx.x,
              (int64_t)gridDim.x * BLU_UPD);
}

__global__ void __launch_bounds__(BLU)
    k_band_backsub(int64_t n, int KU, int W, const double* __restrict__ AB,
                   double* __restrict__ b, double* __restrict__ x, const int* __restrict__ info) {
  if (*info) return;  // uniform
  band_backsub(n, KU, W, AB, b, x);
}

bool band_steps(int kl, int KU) {
  if (const char* e = getenv("SEM_BAND_LU_STEPS")) {
    if (e[0] == '0') return false;
    if (e[0] == '1') return true;
  }
  int64_t lim = 12288;
  if (const char* e = getenv("SEM_BAND_STEP_MIN")) lim = atoll(e);
  return (int64_t)kl * KU >= lim;
}

}  // namespace

extern "C" {

int sem_schur_batched(int64_t n_elem, int nl, int ne, const double* d_mat, const double* d_rhs,
                      double* d_work, double* d_sc_mat, double* d_sc_rhs, int64_t* n_singular,
                      void* stream) {
  if (n_elem < 0 || nl < 1 || ne < 0 || ne > nl || nl - ne > 512)
    return fail(SEM_E_INVALID, "sem_schur_batched: need 0 <= ne <= nl and nl - ne <= 512");
  if (n_elem && (!d_mat || !d_rhs || !d_sc_mat || !d_sc_rhs || (nl > ne && !d_work)))
    return fail(SEM_E_INVALID, "sem_schur_batched: null argument");
  if (!n_elem) return SEM_OK;
  hipStream_t st = S(stream);
  unsigned long long* d_bad = nullptr;
  HIP_TRY(hipMallocAsync((void**)&d_bad, sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(d_bad, 0, sizeof(unsigned long long), st));
  const int grid = (int)std::min<int64_t>(n_elem, 4096);
  hipLaunchKernelGGL(k_sc_condense, dim3(grid), dim3(SCB), 0, st, n_elem, nl, ne, d_mat, d_rhs,
                     d_work, d_sc_mat, d_sc_rhs, d_bad);
  HIP_TRY(hipGetLastError());
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipFreeAsync(d_bad, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (n_singular) *n_singular = (int64_t)bad;
  if (bad)
    return fail(SEM_E_INVALID, "singular interior block in " + std::to_string(bad) + " elements");
  return SEM_OK;
}

int sem_band_lu_solve(int64_t n, int kl, int ku, const int64_t* d_rowptr, const int32_t* d_colind,
                      const double* d_val, const double* d_b, double* d_x, int* info,
                      void* stream) {
  if (n < 0 || kl < 0 || ku < 0 || (int64_t)kl + ku > (1 << 28))
    return fail(SEM_E_INVALID, "sem_band_lu_solve: bad sizes");
  if (n && (!d_rowptr || !d_colind || !d_val || !d_b || !d_x || !info))
    return fail(SEM_E_INVALID, "sem_band_lu_solve: null argument");
  if (!n) {
    *info = 0;
    return SEM_OK;
  }
  const int KU = kl + ku;
  const int W = KU + kl + 1;
  hipStream_t st = S(stream);
  double *AB = nullptr, *b = nullptr;
  int* d_info = nullptr;
  HIP_TRY(hipMallocAsync((void**)&AB, (size_t)n * W * sizeof(double), st));
  HIP_TRY(hipMallocAsync((void**)&b, (size_t)n * sizeof(double), st));
  HIP_TRY(hipMallocAsync((void**)&d_info, sizeof(int), st));
  HIP_TRY(hipMemsetAsync(AB, 0, (size_t)n * W * sizeof(double), st));
  HIP_TRY(hipMemcpyAsync(b, d_b, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, st));
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_band_fill, dim3(grid), dim3(256), 0, st, n, KU, W, d_rowptr, d_colind, d_val,
                     AB);
  if (band_steps(kl, KU)) {
    HIP_TRY(hipMemsetAsync(d_info, 0, sizeof(int), st));
    for (int64_t j = 0; j < n; ++j) {
      const int64_t nr = std::min<int64_t>(n - 1, j + kl) - j;
      const int64_t nc = std::min<int64_t>(n - 1, j + KU) - j;
      hipLaunchKernelGGL(k_band_step_pivot, dim3(1), dim3(BLU), 0, st, n, kl, KU, W, AB, b, d_info,
                         j);
      const int64_t tot = nr * nc;
      if (tot > 0) {
        const int g = (int)std::min<int64_t>((tot + BLU_UPD - 1) / BLU_UPD, 2048);
        hipLaunchKernelGGL(k_band_step_update, dim3(g), dim3(BLU_UPD), 0, st, n, kl, KU, W, AB,
                           d_info, j);
      }
    }
    hipLaunchKernelGGL(k_band_backsub, dim3(1), dim3(BLU), 0, st, n, KU, W, AB, b, d_x, d_info);
  } else {
    hipLaunchKernelGGL(k_band_lu_solve, dim3(1), dim3(BLU), 0, st, n, kl, KU, W, AB, b, d_x,
                       d_info);
  }
  HIP_TRY(hipGetLastError());
  int h_info = 0;
  HIP_TRY(hipMemcpyAsync(&h_info, d_info, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipFreeAsync(AB, st));
  HIP_TRY(hipFreeAsync(b, st));
  HIP_TRY(hipFreeAsync(d_info, st));
  HIP_TRY(hipStreamSynchronize(st));
  *info = h_info;
  return SEM_OK;
}

int sem_schur_backsolve(int64_t n_elem, int nl, int ne, const double* d_work, const double* d_xe,
                        double* d_xi, void* stream) {
  if (n_elem < 0 || nl < 1 || ne < 0 || ne > nl) return fail(SEM_E_INVALID, "bad sizes");
  const int ni = nl - ne;
  if (!n_elem || !ni) return SEM_OK;
  if (!d_work || !d_xe || !d_xi) return fail(SEM_E_INVALID, "null argument");
  const int64_t total = n_elem * ni;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_sc_backsolve, dim3(grid), dim3(256), 0, S(stream), n_elem, ni, ne, d_work,
                     d_xe, d_xi);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

}  // extern "C"
