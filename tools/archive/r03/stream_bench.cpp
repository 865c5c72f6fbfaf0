// Round 3 micro-benchmark (not part of the library): the PCG vector passes
// at 67.1M DOF in several forms, a double2 copy for calibration, and the host
// cost of replaying one hipGraphExec back to back (does a launch wait for the
// previous replay of the same executable?).
//   hipcc --offload-arch=gfx950 -O3 -x hip tools/r03/stream_bench.cpp -o gpurun_out/stream_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);      \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int BLK = 256;

template <bool NT>
__device__ __forceinline__ double2 ld(const double2* p) {
  if constexpr (NT) {
    double2 v;
    v.x = __builtin_nontemporal_load(&p->x);
    v.y = __builtin_nontemporal_load(&p->y);
    return v;
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st(double2* p, double2 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
  } else {
    *p = v;
  }
}

__global__ void k_copy(const double2* __restrict__ a, double2* __restrict__ b, int64_t nv) {
  for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < nv; i += (int64_t)gridDim.x * BLK)
    b[i] = a[i];
}

// residual-like: r = r - a q (3 reads + flags, 1 write), two dots
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(BLK)
    k_res(double2* __restrict__ r, const double2* __restrict__ q, const double2* __restrict__ d,
          const uchar2* __restrict__ f, int64_t nv, double a, double* __restrict__ out) {
  double s0 = 0, s1 = 0;
  const int64_t stp = (int64_t)gridDim.x * BLK;
  for (int64_t i0 = blockIdx.x * (int64_t)BLK + threadIdx.x; i0 < nv; i0 += U * stp) {
    double2 qv[U], rv[U], dv[U];
    uchar2 fv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stp < nv ? i0 + u * stp : 0;
      qv[u] = ld<NTL>(q + i);
      rv[u] = ld<NTL>(r + i);
      dv[u] = ld<NTL>(d + i);
      fv[u] = f[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u * stp >= nv) continue;
      double2 o;
      o.x = (fv[u].x & 1) ? 0.0 : fma(-a, qv[u].x, rv[u].x);
      o.y = (fv[u].y & 1) ? 0.0 : fma(-a, qv[u].y, rv[u].y);
      s0 = fma(o.x, o.x * dv[u].x, fma(o.y, o.y * dv[u].y, s0));
      s1 = fma(o.x, o.x, fma(o.y, o.y, s1));
      st<NTS>(r + i0 + u * stp, o);
    }
  }
  if (s0 == 12345.0 && s1 == 1.0) out[0] = s0;  // keep the sums live
}

// step-like: x += a p; p = r d + b p (4 reads, 2 writes)
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(BLK)
    k_step(double2* __restrict__ x, double2* __restrict__ p, const double2* __restrict__ r,
           const double2* __restrict__ d, int64_t nv, double a, double b) {
  const int64_t stp = (int64_t)gridDim.x * BLK;
  for (int64_t i0 = blockIdx.x * (int64_t)BLK + threadIdx.x; i0 < nv; i0 += U * stp) {
    double2 xv[U], pv[U], rv[U], dv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stp < nv ? i0 + u * stp : 0;
      xv[u] = ld<NTL>(x + i);
      pv[u] = ld<NTL>(p + i);
      rv[u] = ld<NTL>(r + i);
      dv[u] = ld<NTL>(d + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u * stp >= nv) continue;
      double2 xo, po;
      xo.x = fma(a, pv[u].x, xv[u].x);
      xo.y = fma(a, pv[u].y, xv[u].y);
      po.x = fma(b, pv[u].x, rv[u].x * dv[u].x);
      po.y = fma(b, pv[u].y, rv[u].y * dv[u].y);
      st<NTS>(x + i0 + u * stp, xo);
      st<NTS>(p + i0 + u * stp, po);
    }
  }
}

__global__ void k_spin(double* y, int iters) {
  double v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = fma(v, 1.0000001, 1e-9);
  if (v == 12345.0) y[0] = v;
}

template <class F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int64_t n = 67125249 + 1, nv = n / 2;
  double2 *x, *p, *r, *q, *d;
  uchar2* f;
  double* out;
  for (double2** a : {&x, &p, &r, &q, &d}) {
    CK(hipMalloc(a, nv * sizeof(double2)));
    CK(hipMemset(*a, 0, nv * sizeof(double2)));
  }
  CK(hipMalloc(&f, nv * sizeof(uchar2)));
  CK(hipMemset(f, 0, nv * sizeof(uchar2)));
  CK(hipMalloc(&out, 64));
  const double gb = 1e-9 * n;
  const int reps = 20;
  auto rate = [&](const char* name, double bytes_per_dof, float ms) {
    std::printf("%-34s %8.4f ms  %6.2f TB/s\n", name, ms, bytes_per_dof * gb / ms);
  };
  rate("copy double2 (grid 8192)", 16, time_ms([&] { k_copy<<<8192, BLK>>>(q, r, nv); }, reps));
  rate("copy double2 (grid 2048)", 16, time_ms([&] { k_copy<<<2048, BLK>>>(q, r, nv); }, reps));
#define RES(G, U, L, S)                                                                     \
  rate("residual g" #G " U" #U " ntl" #L " nts" #S, 33,                                     \
       time_ms([&] { k_res<U, L, S><<<G, BLK>>>(r, q, d, f, nv, 0.5, out); }, reps));
#define STEP(G, U, L, S)                                                                    \
  rate("step g" #G " U" #U " ntl" #L " nts" #S, 48,                                         \
       time_ms([&] { k_step<U, L, S><<<G, BLK>>>(x, p, r, d, nv, 0.5, 0.25); }, reps));
  RES(2048, 2, false, false)
  RES(2048, 2, false, true)
  RES(2048, 2, true, true)
  RES(2048, 4, false, false)
  RES(2048, 4, false, true)
  RES(4096, 2, false, false)
  RES(4096, 2, false, true)
  RES(8192, 1, false, true)
  RES(1024, 4, false, true)
  STEP(2048, 2, false, false)
  STEP(2048, 2, false, true)
  STEP(2048, 2, true, true)
  STEP(2048, 4, false, false)
  STEP(2048, 4, false, true)
  STEP(4096, 2, false, false)
  STEP(4096, 2, false, true)
  STEP(8192, 1, false, true)
  STEP(1024, 4, false, true)

  // graph replay: one ~0.3 ms kernel captured; host time of 20 back-to-back
  // hipGraphLaunch calls of the same executable vs 20 eager launches
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int iters = 20000;
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    k_spin<<<1024, BLK, 0, s>>>(out, iters);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("spin kernel %.3f ms\n", ms);
  }
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  k_spin<<<1024, BLK, 0, s>>>(out, iters);
  k_spin<<<1024, BLK, 0, s>>>(out, iters);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  for (int mode = 0; mode < 2; ++mode) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 20; ++i) {
      if (mode)
        CK(hipGraphLaunch(ge, s));
      else {
        k_spin<<<1024, BLK, 0, s>>>(out, iters);
        k_spin<<<1024, BLK, 0, s>>>(out, iters);
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    const auto t2 = std::chrono::steady_clock::now();
    std::printf("%s: host enqueue %.1f us per step, total %.3f ms per step\n",
                mode ? "graph" : "eager",
                std::chrono::duration<double, std::micro>(t1 - t0).count() / 20,
                std::chrono::duration<double, std::milli>(t2 - t0).count() / 20);
  }
  return 0;
}
