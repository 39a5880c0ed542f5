// Ceiling probe for k_gsrb_pair2's access pattern on MI355X: one 1024-thread
// workgroup per 64^3 box (66^3 with ghosts) marches over the k planes like
// the pair kernel -- phi plane (66x66) and the rhs rows of the plane in,
// the previous plane's rows out -- with the same LDS ring and barriers but
// no stencil arithmetic. Reports algorithmic GB/s (24 B per interior cell).
//   hipcc --offload-arch=gfx950 -O3 scripts/plane_bw.hip -o scripts/plane_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int NC = 64, NG = NC + 2, PL = NG * NG, NT = 1024;
constexpr int EPT = (PL + NT - 1) / NT;
constexpr size_t SK = (size_t)NG * NG, BSZ = (size_t)NG * NG * NG;

__device__ __forceinline__ int xcd_swizzle(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7, slot = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}

template <int MODE>  // 0: LDS ring + barriers (pair-like), 1: direct copy
__global__ void __launch_bounds__(NT) k_plane(const double *__restrict__ src,
                                              const double *__restrict__ rhs,
                                              double *__restrict__ dst) {
  __shared__ double P[4][PL];
  const int tid = threadIdx.x;
  const int box = xcd_swizzle(blockIdx.x, gridDim.x);
  const double *x = src + box * BSZ, *r = rhs + box * BSZ;
  double *y = dst + box * BSZ;
  double acc = 0;
  if (MODE == 0) {
    for (int e = tid; e < 3 * PL; e += NT) P[e / PL][e % PL] = x[e];
    __syncthreads();
    for (int s = 1; s <= NC + 1; s++) {
      double nx[EPT], rr[4];
#pragma unroll
      for (int e = 0; e < EPT; e++) {
        const int xx = tid + NT * e;
        nx[e] = x[(size_t)(s + 2 <= NC + 1 ? s + 2 : NC + 1) * SK + (xx < PL ? xx : PL - 1)];
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int c = tid + NT * q, j = c / NC + 1, i = c % NC + 1;
        rr[q] = r[(size_t)(s <= NC ? s : NC) * SK + j * NG + i];
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 4; q++) acc += rr[q] * P[s & 3][(tid + NT * q) % PL];
      __syncthreads();
      if (s >= 2) {
        const double *Pm = P[(s - 1) & 3];
#pragma unroll
        for (int q = 0; q < (NG * NC + NT - 1) / NT; q++) {
          const int e = tid + NT * q;
          if (e < NG * NC) y[(size_t)(s - 1) * SK + NG + e] = Pm[NG + e];
        }
      }
      __syncthreads();
      if (s + 2 <= NC + 1) {
#pragma unroll
        for (int e = 0; e < EPT; e++) {
          const int xx = tid + NT * e;
          if (xx < PL) P[(s + 2) & 3][xx] = nx[e];
        }
      }
      __syncthreads();
    }
  } else {
    for (int s = 1; s <= NC; s++) {
#pragma unroll
      for (int q = 0; q < (NG * NC + NT - 1) / NT; q++) {
        const int e = tid + NT * q;
        if (e < NG * NC) {
          const size_t g = (size_t)s * SK + NG + e;
          y[g] = x[g] + r[g];
        }
      }
    }
  }
  if (acc == 12345.678) y[0] = acc;
}

int main() {
  const int nbox = 512;
  double *a, *b, *c;
  const size_t n = BSZ * (nbox + 73);
  hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&c, n * 8);
  hipMemset(a, 0, n * 8); hipMemset(b, 0, n * 8); hipMemset(c, 0, n * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 24.0 * NC * NC * NC * nbox;
  for (int mode = 0; mode < 2; mode++) {
    std::vector<float> ts;
    for (int it = 0; it < 12; it++) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k_plane<0>, dim3(nbox), dim3(NT), 0, 0, a, b, c);
      else hipLaunchKernelGGL(k_plane<1>, dim3(nbox), dim3(NT), 0, 0, a, b, c);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (it >= 2) ts.push_back(ms);
    }
    float best = 1e9, sum = 0;
    for (float t : ts) best = t < best ? t : best, sum += t;
    printf("mode %d (%s): avg %.1f us  best %.1f us  %.3f TB/s algorithmic (avg)\n", mode,
           mode ? "direct copy" : "pair-like LDS ring", 1e3 * sum / ts.size(), 1e3 * best,
           bytes / (sum / ts.size() * 1e-3) / 1e12);
  }
  return 0;
}
