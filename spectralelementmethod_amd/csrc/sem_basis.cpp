// Host half of libsem_hip.so: GLL tables, 1-D Lagrange basis data and the C
// twins of the reference's sem/bary_interp.c.  Everything here is setup
// (n <= 17 numbers); the per-element hot path lives in sem_device.hip.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gll_table.h"
#include "sem_internal.h"

namespace sem {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Unfold the stored non-negative half exactly as LagrangeGaussLobatto.__init__
// (sem/basis_functions.py:372-388): the upper half is copied, the lower half
// mirrored with negated nodes; for an even node count the mirrored
// barycentric weights change sign.
int gll_table(int p, double* nodes, double* bary, double* quad) {
  if (p < 1) return fail(SEM_E_INVALID, "Must specify an order of 1 or greater.");
  if (p > SEM_GLL_MAX_ORDER)
    return fail(SEM_E_NOTIMPL, "Basis only available up to order " +
                                   std::to_string(SEM_GLL_MAX_ORDER) + ".");
  const int n = p + 1, m = n / 2, half = p / 2 + 1;
  const double(*h)[SEM_GLL_MAX_HALF] = sem_gll_half[p];
  for (int k = 0; k < half; ++k) {
    nodes[m + k] = h[0][k];
    bary[m + k] = h[1][k];
    quad[m + k] = h[2][k];
  }
  const double bsign = (n % 2 == 1) ? 1.0 : -1.0;
  for (int k = 0; k < m; ++k) {
    const int src = half - 1 - k;
    nodes[k] = -h[0][src];
    bary[k] = bsign * h[1][src];
    quad[k] = h[2][src];
  }
  return SEM_OK;
}

// BarycentricLagrange.__init__ (sem/basis_functions.py:213-219):
// D_ij = (b_j / b_i) / (x_i - x_j), D_ii = -sum_{j != i} D_ij.
void diff_matrix(int n, const double* x, const double* b, double* D) {
  for (int i = 0; i < n; ++i) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) {
      if (j == i) continue;
      const double v = (b[j] / b[i]) / (x[i] - x[j]);
      D[i * n + j] = v;
      s += v;
    }
    D[i * n + i] = -s;
  }
}

// BarycentricLagrange.__call__ (sem/basis_functions.py:226-255): kernel
// w_j/(x - x_j) normalised by its sum; an exact node gives the unit row.
void lagrange_eval(int n, const double* xn, const double* b, int64_t nx, const double* x,
                   double* B) {
  for (int64_t i = 0; i < nx; ++i) {
    double* row = B + i * n;
    int hit = -1;
    double s = 0.0;
    for (int j = 0; j < n; ++j) {
      const double d = x[i] - xn[j];
      if (d == 0.0) {
        hit = j;
        break;
      }
      row[j] = b[j] / d;
      s += row[j];
    }
    if (hit >= 0) {
      for (int j = 0; j < n; ++j) row[j] = (j == hit) ? 1.0 : 0.0;
    } else {
      for (int j = 0; j < n; ++j) row[j] /= s;
    }
  }
}

// Gauss-Jordan with partial pivoting in extended precision.
int invert(int n, const double* A, double* Ainv) {
  std::vector<long double> a(n * 2 * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 2 * n; ++j)
      a[i * 2 * n + j] = (j < n) ? A[i * n + j] : (j - n == i ? 1.0L : 0.0L);
  for (int c = 0; c < n; ++c) {
    int piv = c;
    for (int r = c + 1; r < n; ++r)
      if (fabsl(a[r * 2 * n + c]) > fabsl(a[piv * 2 * n + c])) piv = r;
    if (a[piv * 2 * n + c] == 0.0L) return fail(SEM_E_INVALID, "singular matrix");
    if (piv != c)
      for (int j = 0; j < 2 * n; ++j) std::swap(a[c * 2 * n + j], a[piv * 2 * n + j]);
    const long double d = a[c * 2 * n + c];
    for (int j = 0; j < 2 * n; ++j) a[c * 2 * n + j] /= d;
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      const long double f = a[r * 2 * n + c];
      if (f == 0.0L) continue;
      for (int j = 0; j < 2 * n; ++j) a[r * 2 * n + j] -= f * a[c * 2 * n + j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) Ainv[i * n + j] = (double)a[i * 2 * n + n + j];
  return SEM_OK;
}

}  // namespace sem

extern "C" {

const char* sem_last_error(void) { return sem::g_err.c_str(); }

const char* sem_version(void) { return "sem_hip 0.1.0 (gfx950)"; }

int sem_op_ncomp(int op_kind) {
  switch (op_kind) {
    case SEM_OP_POISSON:
      return 3;
    case SEM_OP_AXISYM_STOKES:
      return 7;
    case SEM_OP_AXISYM_NS:
    case SEM_OP_AXISYM_NS_JVP:
      return 9;
    default:
      return sem::fail(SEM_E_INVALID, "unknown op_kind " + std::to_string(op_kind));
  }
}

int sem_gll_table(int p, double* nodes, double* bary, double* quad) {
  if (!nodes || !bary || !quad) return sem::fail(SEM_E_INVALID, "null output pointer");
  return sem::gll_table(p, nodes, bary, quad);
}

int sem_diff_matrix(int n, const double* nodes, const double* bary, double* D) {
  if (n < 2 || n > SEM_MAXN || !nodes || !bary || !D)
    return sem::fail(SEM_E_INVALID, "sem_diff_matrix: bad arguments");
  sem::diff_matrix(n, nodes, bary, D);
  return SEM_OK;
}

int sem_lagrange_eval(int n, const double* nodes, const double* bary, int64_t nx, const double* x,
                      double* B) {
  if (n < 1 || nx < 0 || !nodes || !bary || (nx && (!x || !B)))
    return sem::fail(SEM_E_INVALID, "sem_lagrange_eval: bad arguments");
  sem::lagrange_eval(n, nodes, bary, nx, x, B);
  return SEM_OK;
}

int sem_interp_eq_matrix(int n, const double* nodes, const double* bary, double* Veq,
                         double* Veq_inv) {
  if (n < 2 || n > SEM_MAXN || !nodes || !bary || !Veq)
    return sem::fail(SEM_E_INVALID, "sem_interp_eq_matrix: bad arguments");
  // numpy.linspace(-1, 1, n): start + i*step with the last point exact
  std::vector<double> xe(n);
  const double step = 2.0 / (n - 1);
  for (int i = 0; i < n; ++i) xe[i] = -1.0 + i * step;
  xe[n - 1] = 1.0;
  sem::lagrange_eval(n, nodes, bary, n, xe.data(), Veq);
  if (Veq_inv) return sem::invert(n, Veq, Veq_inv);
  return SEM_OK;
}

// sem/bary_interp.c:10-36: three-term Legendre recursion.
double sem_legeval(double x, unsigned n) {
  double p0 = 1.0;
  if (n == 0) return p0;
  double p1 = x;
  for (unsigned i = 1; i < n; ++i) {
    const double p2 = ((2.0 * i + 1.0) * x * p1 - i * p0) / (i + 1.0);
    p0 = p1;
    p1 = p2;
  }
  return p1;
}

// sem/bary_interp.c:39-90: barycentric form over the GLL table of order n-1;
// a non-finite kernel (x on a node) returns the nodal value.
double sem_barycentric_lagrange(const double* f, unsigned n, double x) {
  if (!f || n < 2 || n > SEM_MAXN) {
    sem::set_error("sem_barycentric_lagrange: need 2 <= n <= 17");
    return NAN;
  }
  double nodes[SEM_MAXN], bary[SEM_MAXN], quad[SEM_MAXN];
  sem::gll_table((int)n - 1, nodes, bary, quad);
  double numer = 0.0, denom = 0.0;
  for (unsigned i = 0; i < n; ++i) {
    const double kern = bary[i] / (x - nodes[i]);
    if (!std::isfinite(kern)) return f[i];
    numer += kern * f[i];
    denom += kern;
  }
  return numer / denom;
}

}  // extern "C"
