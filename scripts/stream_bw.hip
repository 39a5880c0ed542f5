// Streaming bandwidth calibration for FP64 kernels on MI355X: copy (1 read
// + 1 write) and triad (2 reads + 1 write) with 8-byte and 16-byte lanes.
// Prints achieved TB/s (bytes moved / kernel time), median of 20 launches.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void copy8(const double *__restrict__ a, double *__restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}
__global__ void triad8(const double *__restrict__ a, const double *__restrict__ c,
                       double *__restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] + 1.5 * c[i];
}
__global__ void triad16(const double2 *__restrict__ a, const double2 *__restrict__ c,
                        double2 *__restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    double2 x = a[i], y = c[i];
    b[i] = make_double2(x.x + 1.5 * y.x, x.y + 1.5 * y.y);
  }
}
__global__ void read8(const double *__restrict__ a, double *__restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double v = i < n ? a[i] : 0.0;
  if (v == 12345.678) out[0] = v;
}
__global__ void write8(double *__restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = 1.0;
}

template <class F>
double timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<float> t;
  for (int r = 0; r < 22; r++) {
    hipEventRecord(e0);
    f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (r >= 2) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2] * 1e-3;
}

// STREAM_CONTIG=1: the three arrays in one hipDeviceMallocContiguous
// allocation; STREAM_GAP (bytes): extra bytes between them
int main() {
  const size_t n = (size_t)1 << 27;  // 1 GiB per array of doubles
  double *a, *b, *c;
  const char *ce = getenv("STREAM_CONTIG");
  if (ce && atoi(ce)) {
    const size_t gap = getenv("STREAM_GAP") ? (size_t)atoll(getenv("STREAM_GAP")) / 8 : 0;
    double *base = nullptr;
    if (hipExtMallocWithFlags((void **)&base, (3 * (n + gap)) * 8, hipDeviceMallocContiguous) !=
        hipSuccess) {
      printf("contiguous allocation refused\n");
      return 1;
    }
    a = base, b = base + n + gap, c = base + 2 * (n + gap);
    printf("contiguous, gap %zu B\n", gap * 8);
  } else {
    hipMalloc(&a, n * 8);
    hipMalloc(&b, n * 8);
    hipMalloc(&c, n * 8);
  }
  hipMemset(a, 0, n * 8);
  hipMemset(b, 0, n * 8);
  hipMemset(c, 0, n * 8);
  const int bs = 256;
  const unsigned g8 = (unsigned)((n + bs - 1) / bs), g16 = (unsigned)((n / 2 + bs - 1) / bs);
  double t;
  t = timeit([&] { hipLaunchKernelGGL(read8, dim3(g8), dim3(bs), 0, 0, a, b, n); });
  printf("read8   %.3f TB/s\n", n * 8.0 / t / 1e12);
  t = timeit([&] { hipLaunchKernelGGL(write8, dim3(g8), dim3(bs), 0, 0, b, n); });
  printf("write8  %.3f TB/s\n", n * 8.0 / t / 1e12);
  t = timeit([&] { hipLaunchKernelGGL(copy8, dim3(g8), dim3(bs), 0, 0, a, b, n); });
  printf("copy8   %.3f TB/s\n", n * 16.0 / t / 1e12);
  t = timeit([&] { hipLaunchKernelGGL(triad8, dim3(g8), dim3(bs), 0, 0, a, c, b, n); });
  printf("triad8  %.3f TB/s\n", n * 24.0 / t / 1e12);
  t = timeit([&] {
    hipLaunchKernelGGL(triad16, dim3(g16), dim3(bs), 0, 0, (const double2 *)a,
                       (const double2 *)c, (double2 *)b, n / 2);
  });
  printf("triad16 %.3f TB/s\n", n * 24.0 / t / 1e12);
  return 0;
}
