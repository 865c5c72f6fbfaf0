// Round 3: calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access widths of the operator kernels (MI355X_MICROARCH.md §HBM: the
// counters read exactly half of a 16-B-per-lane streaming read; other
// widths are uncalibrated).  Each kernel touches a known number of bytes of
// a 1 GiB array (far past the 256 MiB Infinity Cache), once.
//   hipcc --offload-arch=gfx950 -O3 -x hip tools/r03/pmc_calib.cpp -o tools/r03/pmc_calib.bin
//   rocprofv3 --pmc FETCH_SIZE -- tools/r03/pmc_calib.bin   (then WRITE_SIZE)
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

template <class T>
__device__ __forceinline__ double val(T v) {
  return (double)v;
}
template <>
__device__ __forceinline__ double val<double2>(double2 v) {
  return v.x + v.y;
}

// every element of a[0, n) read once, 1 element per lane per step
template <class T>
__global__ void k_read(const T* __restrict__ a, int64_t n, double* __restrict__ out) {
  double s = 0;
  for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK)
    s += val(a[i]);
  if (s == 1234.5) out[0] = s;
}

// every element of a[0, n) written once
template <class T>
__global__ void k_write(T* __restrict__ a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK)
    a[i] = T{};
}

// the operator's gather shape: lane (k, j) of a wave reads 9 rows r of a
// 7-element group, node (k*8 + j) + r * row_stride -- 57 consecutive
// doubles per row, each row of the array read once overall
__global__ void k_gather_rows(const double* __restrict__ u, int64_t rows, int64_t row_len,
                              double* __restrict__ out) {
  const int lane = threadIdx.x % 64;
  const int k = lane / 9, j = lane % 9;
  const int64_t wave = (blockIdx.x * (int64_t)BLK + threadIdx.x) / 64;
  const int64_t nwave = (int64_t)gridDim.x * BLK / 64;
  const int64_t segs = row_len / 56;  // 7 elements x 8 new nodes per group row
  double s = 0;
  if (lane < 63)
    for (int64_t w = wave; w < (rows / 8) * segs; w += nwave) {
      const int64_t band = w / segs, seg = w % segs;
      for (int r = 0; r < 8; ++r)  // 8 new node rows per element row
        s += u[(band * 8 + r) * row_len + seg * 56 + k * 8 + j];
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
  const int grid = 8192;
  std::printf("array %zu bytes; per kernel below: bytes touched\n", bytes);
  k_read<double2><<<grid, BLK>>>((const double2*)a, bytes / 16, out);
  std::printf("k_read<double2>  read %zu\n", bytes);
  k_read<double><<<grid, BLK>>>((const double*)a, bytes / 8, out);
  std::printf("k_read<double>   read %zu\n", bytes);
  k_read<uint32_t><<<grid, BLK>>>((const uint32_t*)a, bytes / 4, out);
  std::printf("k_read<uint32>   read %zu\n", bytes);
  k_read<uint16_t><<<grid, BLK>>>((const uint16_t*)a, bytes / 2, out);
  std::printf("k_read<uint16>   read %zu\n", bytes);
  const int64_t row_len = 8192, rows = bytes / 8 / row_len;  // 16384 rows
  k_gather_rows<<<grid, BLK>>>((const double*)a, rows, row_len, out);
  std::printf("k_gather_rows    read %lld (every node of the used columns once)\n",
              (long long)((rows / 8) * 8 * (row_len / 56) * 56 * 8));
  k_write<double2><<<grid, BLK>>>((double2*)a, bytes / 16);
  std::printf("k_write<double2> write %zu\n", bytes);
  k_write<double><<<grid, BLK>>>((double*)a, bytes / 8);
  std::printf("k_write<double>  write %zu\n", bytes);
  CK(hipDeviceSynchronize());
  return 0;
}
