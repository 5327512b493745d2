// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access patterns of
// this repository's kernels (measurement tool, not product).  Each kernel
// touches a known number of bytes of a 2 GiB buffer (8x the 256 MiB
// Infinity Cache, so nothing is served on-die); the rocprofv3 counters of
// each dispatch divided into the known count give the correction factor
// per pattern (MI355X_MICROARCH.md calibrates only 16-B-per-lane streams).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d out -o run -- ./tools/fetch_calib
//
// Kernels (one dispatch each, in this order; printed with their byte counts):
//   read16   16 B per lane, coalesced (the guide's calibrated case)
//   read8    8 B per lane, coalesced (a wave reads 512 contiguous bytes)
//   gather8  8 B per lane, one element per 256-B stride (each element its
//            own line: the [line][S] gathers of one scenario at stride S)
//   gather8x8  8 B per lane, stride 64 B (two elements per 128-B line)
//   write8   8 B per lane, coalesced stores
//   write8s  8 B per lane, stores at a 256-B stride
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

__global__ void __launch_bounds__(256) read16(const double2 *__restrict__ a, long n, double *out) {
  double acc = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const double2 v = a[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;  // keeps the loads, never true
}
__global__ void __launch_bounds__(256) read8(const double *__restrict__ a, long n, double *out) {
  double acc = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc += a[i];
  if (acc == 12345.678) out[0] = acc;
}
__global__ void __launch_bounds__(256) gather8(const double *__restrict__ a, long n, long stride, double *out) {
  double acc = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc += a[i * stride];
  if (acc == 12345.678) out[0] = acc;
}
__global__ void __launch_bounds__(256) write8(double *__restrict__ a, long n, long stride) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) a[i * stride] = 1.0;
}

int main() {
  const long bytes = 2L << 30;  // 2 GiB
  double *a, *out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 8;
  const long n8 = bytes / 8;
  hipLaunchKernelGGL(read16, dim3(grid), dim3(256), 0, 0, (const double2 *)a, bytes / 16, out);
  std::printf("CALIB read16 %ld 0\n", bytes);
  hipLaunchKernelGGL(read8, dim3(grid), dim3(256), 0, 0, a, n8, out);
  std::printf("CALIB read8 %ld 0\n", bytes);
  hipLaunchKernelGGL(gather8, dim3(grid), dim3(256), 0, 0, a, n8 / 32, 32L, out);
  std::printf("CALIB gather8_stride256 %ld %ld\n", n8 / 32 * 8, n8 / 32 * 128);
  hipLaunchKernelGGL(gather8, dim3(grid), dim3(256), 0, 0, a, n8 / 8, 8L, out);
  std::printf("CALIB gather8_stride64 %ld %ld\n", n8 / 8 * 8, n8 / 16 * 128);
  hipLaunchKernelGGL(write8, dim3(grid), dim3(256), 0, 0, a, n8, 1L);
  std::printf("CALIB write8 %ld 0\n", bytes);
  hipLaunchKernelGGL(write8, dim3(grid), dim3(256), 0, 0, a, n8 / 32, 32L);
  std::printf("CALIB write8_stride256 %ld 0\n", n8 / 32 * 8);
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
