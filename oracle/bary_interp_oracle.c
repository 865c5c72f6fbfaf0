/*
 * CPU ORACLE -- test infrastructure only (never linked into the product).
 *
 * Plain-C restatement of the reference's orphan native file
 * sem/bary_interp.c.  The reference file itself cannot be compiled here: it
 * #includes "glnodes.c" (sem/bary_interp.c:5), which the reference does not
 * contain, so there is no oracle/_ref build of it.  The missing tables are
 * therefore passed in as arguments (the stored non-negative halves of the
 * GLL nodes and barycentric weights, as in sem/data/basis-data.hdf5), and the
 * known answer of the reference's main() (sem/bary_interp.c:93-100,
 * f(0.654) = 0.653996, value 0.6539963274676562 from the reference's Python
 * twin) pins it in tests/test_oracle_golden.py.
 */
#include <math.h>

/* sem/bary_interp.c:10-36 */
double oracle_legeval(double x, unsigned n) {
  double p0 = 1.0, p1, p2;
  unsigned i;
  if (n == 0) return p0;
  p1 = x;
  if (n == 1) return p1;
  for (i = 1;; ++i) {
    p2 = ((2 * i + 1) * x * p1 - i * p0) / (i + 1);
    if (i == n - 1) return p2;
    p0 = p1;
    p1 = p2;
  }
}

/* sem/bary_interp.c:39-90 with the table rows passed explicitly:
 * half_nodes / half_bary hold n/2 + (n odd) values in ascending order. */
double oracle_barycentric_lagrange(const double* f, unsigned n, double x,
                                   const double* half_nodes, const double* half_bary) {
  double nodes[64], bary[64];
  double numer = 0.0, denom = 0.0, kern;
  unsigned i1, i2, j, i;
  if (n < 2 || n > 64) return NAN;
  if (n % 2 == 1) {
    nodes[n / 2] = 0.0;
    bary[n / 2] = half_bary[0];
    i1 = n / 2 + 1;
    i2 = n / 2 - 1;
    j = 1;
  } else {
    i1 = n / 2;
    i2 = n / 2 - 1;
    j = 0;
  }
  while (i1 < n) {
    nodes[i1] = half_nodes[j];
    nodes[i2] = -half_nodes[j];
    bary[i1] = half_bary[j];
    bary[i2] = (n % 2 == 0) ? -half_bary[j] : half_bary[j];
    i1 += 1;
    i2 -= 1;
    j += 1;
  }
  for (i = 0; i < n; ++i) {
    kern = bary[i] / (x - nodes[i]);
    if (!isfinite(kern)) return f[i];
    numer += kern * f[i];
    denom += kern;
  }
  return numer / denom;
}
