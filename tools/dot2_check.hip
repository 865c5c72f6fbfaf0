// Diagnostic: the compensated equispaced->GLL passes (sem_hex.h
// k_hex_eq2gll_pass) against a long double evaluation on the host, for one
// order.  Prints the max relative error of each pass chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I spectralelementmethod_amd/csrc \
//         tools/dot2_check.hip -o tools/dot2_check
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "sem_ctx.h"
#include "sem_hex.h"

constexpr int N = 15;

int main() {
  constexpr int N2 = N * N, N3 = N2 * N;
  const int64_t blocks = 64;
  std::mt19937_64 rng(5);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  // a well-conditioned random V and its hi/lo split (any matrix exercises the arithmetic)
  std::vector<long double> Vl((size_t)N2);
  std::vector<double> vh(N2), vlo(N2);
  for (int i = 0; i < N2; ++i) {
    Vl[i] = (long double)U(rng) * 100.0L + (long double)U(rng) * 1e-17L;
    vh[i] = (double)Vl[i];
    vlo[i] = (double)(Vl[i] - (long double)vh[i]);
  }
  std::vector<double> x((size_t)blocks * N3);
  for (auto& v : x) v = U(rng);
  // host long double reference: three passes
  std::vector<long double> a(x.begin(), x.end()), b(a.size());
  for (int ax = 0; ax < 3; ++ax) {
    const int st = ax == 0 ? N2 : ax == 1 ? N : 1;
    for (int64_t blk = 0; blk < blocks; ++blk)
      for (int node = 0; node < N3; ++node) {
        const int m = ax == 0 ? node / N2 : ax == 1 ? (node / N) % N : node % N;
        const int64_t line = blk * N3 + node - m * st;
        long double s = 0.0L;
        for (int r = 0; r < N; ++r) s += Vl[m * N + r] * a[line + r * st];
        b[blk * N3 + node] = s;
      }
    a.swap(b);
  }
  double *dx, *d1, *d2, *d3, *d4, *dvh, *dvl;
  const size_t bytes = x.size() * sizeof(double);
  if (hipMalloc(&dx, bytes) || hipMalloc(&d1, bytes) || hipMalloc(&d2, bytes) ||
      hipMalloc(&d3, bytes) || hipMalloc(&d4, bytes) || hipMalloc(&dvh, N2 * 8) ||
      hipMalloc(&dvl, N2 * 8)) {
    std::printf("hipMalloc failed\n");
    return 1;
  }
  (void)hipMemcpy(dx, x.data(), bytes, hipMemcpyHostToDevice);
  (void)hipMemcpy(dvh, vh.data(), N2 * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dvl, vlo.data(), N2 * 8, hipMemcpyHostToDevice);
  const dim3 g(256), bl(256);
  hipLaunchKernelGGL((semh::k_hex_eq2gll_pass<N, 0>), g, bl, 0, nullptr, dx, nullptr, d1, d2, dvh,
                     dvl, blocks);
  hipLaunchKernelGGL((semh::k_hex_eq2gll_pass<N, 1>), g, bl, 0, nullptr, d1, d2, d3, d4, dvh, dvl,
                     blocks);
  hipLaunchKernelGGL((semh::k_hex_eq2gll_pass<N, 2>), g, bl, 0, nullptr, d3, d4, d1, nullptr, dvh,
                     dvl, blocks);
  std::vector<double> out(x.size());
  if (hipMemcpy(out.data(), d1, bytes, hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("kernel failed\n");
    return 1;
  }
  // plain float64 evaluation on the host for comparison
  std::vector<double> p(x), q(x.size());
  for (int ax = 0; ax < 3; ++ax) {
    const int st = ax == 0 ? N2 : ax == 1 ? N : 1;
    for (int64_t blk = 0; blk < blocks; ++blk)
      for (int node = 0; node < N3; ++node) {
        const int m = ax == 0 ? node / N2 : ax == 1 ? (node / N) % N : node % N;
        const int64_t line = blk * N3 + node - m * st;
        double s = 0.0;
        for (int r = 0; r < N; ++r) s += vh[m * N + r] * p[line + r * st];
        q[blk * N3 + node] = s;
      }
    p.swap(q);
  }
  long double emax = 0, pmax = 0, amax = 0;
  for (size_t i = 0; i < out.size(); ++i) {
    emax = std::max(emax, fabsl((long double)out[i] - a[i]));
    pmax = std::max(pmax, fabsl((long double)p[i] - a[i]));
    amax = std::max(amax, fabsl(a[i]));
  }
  std::printf("n=%d three passes: device compensated %.3Le, host plain float64 %.3Le (max rel)\n",
              N, emax / amax, pmax / amax);
  return 0;
}
