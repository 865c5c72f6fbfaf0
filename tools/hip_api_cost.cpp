// Host cost of the HIP calls one decomposition step (sem_dd_apply) makes:
// kernel launches with small and large argument blocks, hipExtLaunchKernel
// carrying a stop event, event records with each fence flag, cross-stream
// waits.  Prints microseconds per call (median of 5 batches of 200 calls,
// the device kept busy so that nothing drains).
//   hipcc --offload-arch=gfx950 -O2 tools/hip_api_cost.cpp -o tools/hip_api_cost
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                            \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

struct Big {
  double d[80];  // an argument block the size of k_poisson_apply's (even-odd D by value)
};

__global__ void k_small(double* p, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = 1.0;
}
__global__ void k_big(double* p, Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.d[3] < -1e300) p[0] = b.d[0];
}
__global__ void k_spin(double* p, long long cycles) {  // keeps the device busy
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && cycles < 0) p[0] = 0.0;
}

using Clock = std::chrono::steady_clock;

template <class F>
double per_call_us(hipStream_t busy, double* p, F f) {
  std::vector<double> t;
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, busy, p, 400000000LL);
    const auto t0 = Clock::now();
    for (int i = 0; i < 200; ++i) f();
    t.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / 200);
    if (hipDeviceSynchronize() != hipSuccess) return -1.0;
  }
  std::sort(t.begin(), t.end());
  return t[2];
}

int main() {
  double* p = nullptr;
  CK(hipMalloc(&p, 64));
  hipStream_t a, b, busy;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&busy, hipStreamNonBlocking));
  hipEvent_t ev_t, ev_nt, ev_nf;
  CK(hipEventCreate(&ev_t));
  CK(hipEventCreateWithFlags(&ev_nt, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev_nf, hipEventDisableTiming | hipEventDisableSystemFence));
  Big big{};
  // warm up every path once
  hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, a, p, 1);
  hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, a, p, big);
  CK(hipDeviceSynchronize());
  struct Row {
    const char* name;
    double us;
  };
  std::vector<Row> rows;
  // the device is kept busy by k_spin on its own stream; the streams timed
  // here wait on it so that their queues fill as in a real step
  CK(hipEventRecord(ev_nt, busy));
  rows.push_back({"hipLaunchKernelGGL, 12-byte arguments",
                  per_call_us(busy, p, [&] { hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, a, p, 1); })});
  rows.push_back({"hipLaunchKernelGGL, 648-byte arguments",
                  per_call_us(busy, p, [&] { hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, a, p, big); })});
  rows.push_back({"hipExtLaunchKernelGGL + stop event",
                  per_call_us(busy, p, [&] {
                    hipExtLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, a, nullptr, ev_nf, 0, p, 1);
                  })});
  rows.push_back({"hipEventRecord (timing)", per_call_us(busy, p, [&] { (void)hipEventRecord(ev_t, a); })});
  rows.push_back({"hipEventRecord (DisableTiming)",
                  per_call_us(busy, p, [&] { (void)hipEventRecord(ev_nt, a); })});
  rows.push_back({"hipEventRecord (DisableTiming|DisableSystemFence)",
                  per_call_us(busy, p, [&] { (void)hipEventRecord(ev_nf, a); })});
  rows.push_back({"hipEventRecord + hipStreamWaitEvent (other stream)",
                  per_call_us(busy, p, [&] {
                    (void)hipEventRecord(ev_nt, a);
                    (void)hipStreamWaitEvent(b, ev_nt, 0);
                  })});
  rows.push_back({"same, DisableSystemFence event", per_call_us(busy, p, [&] {
                    (void)hipEventRecord(ev_nf, a);
                    (void)hipStreamWaitEvent(b, ev_nf, 0);
                  })});
  rows.push_back({"launch + record + wait + launch (one join)", per_call_us(busy, p, [&] {
                    hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, a, p, 1);
                    (void)hipEventRecord(ev_nf, a);
                    (void)hipStreamWaitEvent(b, ev_nf, 0);
                    hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, b, p, 1);
                  })});
  rows.push_back({"hipGetLastError", per_call_us(busy, p, [&] { (void)hipGetLastError(); })});
  rows.push_back({"hipGetDevice + hipSetDevice(same)", per_call_us(busy, p, [&] {
                    int d = 0;
                    (void)hipGetDevice(&d);
                    (void)hipSetDevice(d);
                  })});
  for (const Row& r : rows) std::printf("%-55s %8.2f us\n", r.name, r.us);
  CK(hipDeviceSynchronize());
  return 0;
}
