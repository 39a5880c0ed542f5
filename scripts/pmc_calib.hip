// Calibration for the PMC byte counters (MI355X_MICROARCH.md: FETCH_SIZE is
// calibrated only for 16-B/lane streaming reads; other widths must be
// calibrated on a known byte count). k_calib_copy8 streams N doubles with
// 8 B per lane, the access width of the hot-path kernels: it reads exactly
// 8N bytes and writes 8N bytes. scripts/pmc_summary.py divides the counters
// of the hot kernel by the measured/known ratio of this kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_calib_copy8(const double *__restrict__ a,
                              double *__restrict__ b, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] + 1.0;
}

int main() {
  const size_t n = (size_t)1 << 28;  // 2 GiB per array: beyond the 256 MB L3
  double *a, *b;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess)
    return 1;
  (void)hipMemset(a, 0, n * 8);
  (void)hipMemset(b, 0, n * 8);
  for (int r = 0; r < 3; r++)
    hipLaunchKernelGGL(k_calib_copy8, dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, 0, a, b, n);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("k_calib_copy8 bytes_read %zu bytes_written %zu\n", n * 8, n * 8);
  (void)hipFree(a);
  (void)hipFree(b);
  return 0;
}
