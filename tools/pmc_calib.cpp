// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths and shapes of the operator kernels (MI355X_MICROARCH.md §HBM: the
// counters read exactly half of a 16-B-per-lane streaming read and exactly
// the bytes of a 16-B-per-lane streaming store; other widths are
// uncalibrated).  Every kernel below touches a KNOWN number of distinct bytes
// of a 1 GiB array (4x the 256 MiB Infinity Cache), each byte once; the
// counter divided by that number is the correction factor for that shape.
//
//   hipcc --offload-arch=gfx950 -O3 -x hip tools/pmc_calib.cpp -o tools/pmc_calib.bin
//   rocprofv3 --pmc FETCH_SIZE -- tools/pmc_calib.bin      (one counter per pass)
//   rocprofv3 --pmc WRITE_SIZE -- tools/pmc_calib.bin
//   python tools/pmc_calib_summary.py <fetch csv> <write csv> tools/pmc_calib.log
//
// Shapes (the operator's, csrc/sem_kernels.h, p = 8, 7 elements per wave):
//   stream16 / stream8 / stream4 / stream2: lane-linear reads of double2 /
//       double / uint32 / uint16 (the packed and 16-bit map streams are 2- and
//       4-byte lane-linear reads);
//   gather_rows: the u / x_phys gather -- lane (k, j) of a wave reads node
//       k*8 + j of 8 consecutive node rows of a 57-node window; every node of
//       the array read once overall (8 B per lane, L2-line sharing between
//       neighbouring waves as in the kernel);
//   gather_rows16: the same with double2 (x_phys is 16 B per node);
//   strided8: one 8-B read per lane at a stride of 8193 doubles (a column
//       seam node per element row) covering every word once over many passes;
//   wstream16 / wstream8 / wstream8_nt: lane-linear stores (plain; nontemporal
//       as the first-writer stores);
//   wscatter_rows / wscatter_rows_nt: the y scatter -- the gather_rows shape
//       as stores;
//   wrows_aligned: the scatter's rows as whole, 512-B aligned 64-double runs
//       (what a line-aligned chain layout would store);
//   wstrided8: one 8-B store per lane at a stride of 8193 doubles.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

constexpr int BLK = 256;
constexpr int64_t STRIDE = 8193;  // node column length of the 1024^2 p = 8 mesh

template <class T>
__device__ __forceinline__ double val(T v) {
  return (double)v;
}
template <>
__device__ __forceinline__ double val<double2>(double2 v) {
  return v.x + v.y;
}

template <class T>
__global__ void k_stream(const T* __restrict__ a, int64_t n, double* __restrict__ out) {
  double s = 0;
  for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK)
    s += val(a[i]);
  if (s == 1234.5) out[0] = s;
}

template <class T, bool NT>
__global__ void k_wstream(T* __restrict__ a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    if constexpr (NT)
      __builtin_nontemporal_store((T)i, a + i);
    else
      a[i] = T{};
  }
}

// rows x row_len array of T; a wave takes 8 consecutive rows of a 56-node
// segment (lanes k*9 + j, j < 9: node seg*56 + k*8 + j, the j = 8 lane
// overlapping the next element's j = 0 as the shared column does)
template <class T, int MODE>  // 0 read, 1 write, 2 write nontemporal
__global__ void k_rows(T* __restrict__ a, int64_t rows, int64_t row_len, double* __restrict__ out) {
  const int lane = threadIdx.x % 64;
  const int k = lane / 9, j = lane % 9;
  const int64_t wave = (blockIdx.x * (int64_t)BLK + threadIdx.x) / 64;
  const int64_t nwave = (int64_t)gridDim.x * BLK / 64;
  const int64_t segs = row_len / 56;
  double s = 0;
  if (lane < 63)
    for (int64_t w = wave; w < (rows / 8) * segs; w += nwave) {
      const int64_t band = w / segs, seg = w % segs;
      for (int r = 0; r < 8; ++r) {
        const int64_t idx = (band * 8 + r) * row_len + seg * 56 + k * 8 + j;
        if constexpr (MODE == 0) {
          s += val(a[idx]);
        } else if constexpr (MODE == 1) {
          if (j < 8) a[idx] = T{};  // one writer per node
        } else {
          if (j < 8) __builtin_nontemporal_store(T{}, a + idx);
        }
      }
    }
  if (s == 1234.5) out[0] = s;
}

// the aligned reference of the scatter shape: a wave writes 8 rows of 64
// consecutive doubles starting on a 512-B boundary (whole 128-B lines)
__global__ void k_wrows_aligned(double* __restrict__ a, int64_t rows, int64_t row_len) {
  const int lane = threadIdx.x % 64;
  const int64_t wave = (blockIdx.x * (int64_t)BLK + threadIdx.x) / 64;
  const int64_t nwave = (int64_t)gridDim.x * BLK / 64;
  const int64_t segs = row_len / 64;
  for (int64_t w = wave; w < (rows / 8) * segs; w += nwave) {
    const int64_t band = w / segs, seg = w % segs;
    for (int r = 0; r < 8; ++r) a[(band * 8 + r) * row_len + seg * 64 + lane] = 0.0;
  }
}

// n words covered at a stride: item i -> word (i * STRIDE) mod n (STRIDE odd
// and n a power of two: a permutation), every word once
template <bool WRITE>
__global__ void k_strided(double* __restrict__ a, int64_t n, double* __restrict__ out) {
  double s = 0;
  for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const int64_t idx = (i * STRIDE) & (n - 1);
    if constexpr (WRITE)
      a[idx] = 0.0;
    else
      s += a[idx];
  }
  if (s == 1234.5) out[0] = s;
}

int main() {
  const size_t bytes = size_t(1) << 30;
  void* a;
  double* out;
  CK(hipMalloc(&a, bytes + 4096));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, bytes + 4096));
  CK(hipDeviceSynchronize());
  const int grid = 8192;
  // each kernel is timed with HIP events (the second run of two: the first
  // warms the TLB); the bytes the counters see are those of both runs
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0.f;
#define TIMED(launch)                      \
  do {                                     \
    launch;                                \
    CK(hipEventRecord(e0));                \
    launch;                                \
    CK(hipEventRecord(e1));                \
    CK(hipEventSynchronize(e1));           \
    CK(hipEventElapsedTime(&ms, e0, e1));  \
  } while (0)
  // rows of the row kernels: row_len a multiple of 56 (full segments), every
  // element of rows x row_len touched once
  const int64_t row_len = 56 * 146;  // 8176 nodes (one 1024^2 column is 8193)
  std::printf("# name bytes_touched ms (each kernel launched twice in a row, this order; bytes are per launch)\n");
  auto rows_of = [&](size_t elt) { return (int64_t)(bytes / elt / row_len) / 8 * 8; };
  TIMED((k_stream<double2><<<grid, BLK>>>((const double2*)a, bytes / 16, out)));
  std::printf("stream16 %zu %.4f\n", bytes, ms);
  TIMED((k_stream<double><<<grid, BLK>>>((const double*)a, bytes / 8, out)));
  std::printf("stream8 %zu %.4f\n", bytes, ms);
  TIMED((k_stream<uint32_t><<<grid, BLK>>>((const uint32_t*)a, bytes / 4, out)));
  std::printf("stream4 %zu %.4f\n", bytes, ms);
  TIMED((k_stream<uint16_t><<<grid, BLK>>>((const uint16_t*)a, bytes / 2, out)));
  std::printf("stream2 %zu %.4f\n", bytes, ms);
  {
    const int64_t r = rows_of(8);
    TIMED((k_rows<double, 0><<<grid, BLK>>>((double*)a, r, row_len, out)));
    std::printf("gather_rows %lld %.4f\n", (long long)(r * row_len * 8), ms);
  }
  {
    const int64_t r = rows_of(16);
    TIMED((k_rows<double2, 0><<<grid, BLK>>>((double2*)a, r, row_len, out)));
    std::printf("gather_rows16 %lld %.4f\n", (long long)(r * row_len * 16), ms);
  }
  TIMED((k_strided<false><<<grid, BLK>>>((double*)a, bytes / 8, out)));
  std::printf("strided8 %zu %.4f\n", bytes, ms);
  TIMED((k_wstream<double2, false><<<grid, BLK>>>((double2*)a, bytes / 16)));
  std::printf("wstream16 %zu %.4f\n", bytes, ms);
  TIMED((k_wstream<double, false><<<grid, BLK>>>((double*)a, bytes / 8)));
  std::printf("wstream8 %zu %.4f\n", bytes, ms);
  TIMED((k_wstream<double, true><<<grid, BLK>>>((double*)a, bytes / 8)));
  std::printf("wstream8_nt %zu %.4f\n", bytes, ms);
  {
    const int64_t r = rows_of(8);
    TIMED((k_rows<double, 1><<<grid, BLK>>>((double*)a, r, row_len, out)));
    std::printf("wscatter_rows %lld %.4f\n", (long long)(r * row_len * 8), ms);
    TIMED((k_rows<double, 2><<<grid, BLK>>>((double*)a, r, row_len, out)));
    std::printf("wscatter_rows_nt %lld %.4f\n", (long long)(r * row_len * 8), ms);
  }
  {
    const int64_t rl = 8192, r = (int64_t)(bytes / 8 / rl) / 8 * 8;
    TIMED((k_wrows_aligned<<<grid, BLK>>>((double*)a, r, rl)));
    std::printf("wrows_aligned %lld %.4f\n", (long long)(r * rl * 8), ms);
  }
  TIMED((k_strided<true><<<grid, BLK>>>((double*)a, bytes / 8, out)));
  std::printf("wstrided8 %zu %.4f\n", bytes, ms);
  CK(hipDeviceSynchronize());
  return 0;
}
