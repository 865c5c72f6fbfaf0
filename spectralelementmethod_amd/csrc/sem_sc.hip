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
