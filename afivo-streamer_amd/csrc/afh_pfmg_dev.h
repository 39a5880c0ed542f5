// The PFMG level-1 solve on the device (AFH_COARSE_PFMG): the reference's
// HYPRE StructPFMG restated (afh_pfmg.h has the algorithm, its sources and
// the host setup). Shared by the 3-D (afh_mg.hip k_cs_pfmg) and 2-D
// (afh2d.hip k2_cs_pfmg) libraries: each kernel gathers its level-1 boxes
// into x, b of level 0, runs pf_solve_block and scatters x back.
//
// The whole solve is one workgroup. Each operation is oracle/c/afo.c's pf_*
// in the same order of arithmetic, so the two agree bitwise (the liberties
// change at most the sign of a zero: stencil entries zero on a whole level
// are skipped, and a skipped level's x = P x_c is stored, not 0 + P x_c).
// What makes it fast is the number of workgroup barriers per V-cycle, since
// every level operation is a few hundred points of latency-bound work:
//  - the Jacobi sweep writes the other of two x images (one pass, one
//    barrier: x' = (1 - w) x + w (b - sum a x) / a_c from the old x);
//  - a skipped level costs only its restriction (from b, since r = b there)
//    and its interpolation (x = P x_c, since x = 0 there);
//  - the levels of at most 64 points run in wave 0 alone, down and up,
//    with wave-level synchronisation only (the other waves wait at one
//    barrier), their operators staged in LDS at the start;
//  - dot products: 64 strided partial sums, then a shuffle tree in wave 0.
#ifndef AFH_PFMG_DEV_H
#define AFH_PFMG_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "afh_pfmg.h"

namespace afh_pf {

struct PfLvl {
  int n[3];
  int cdir;
  int active;
  int off;        // first point of the level
  int np;         // points
  uint32_t mask;  // stencil entries nonzero somewhere on the level
  int lgx, lgy;   // log2 n[0], log2 n[1] (-1: not a power of 2)
  double w;       // Jacobi weight
};

constexpr int PF_NPART = 64;      // = AFH_PFMG_NPART of the oracle's dot product
constexpr int PF_WAVE_PTS = 64;   // levels of at most this many points run in wave 0

__device__ __forceinline__ void pf_decode(const PfLvl &L, int p, int &i, int &j, int &k) {
  if (L.lgx >= 0 && L.lgy >= 0) {
    i = (p & (L.n[0] - 1)) + 1;
    j = ((p >> L.lgx) & (L.n[1] - 1)) + 1;
    k = (p >> (L.lgx + L.lgy)) + 1;
  } else {
    i = p % L.n[0] + 1;
    j = (p / L.n[0]) % L.n[1] + 1;
    k = p / (L.n[0] * L.n[1]) + 1;
  }
}

__device__ __forceinline__ int pf_pt(const PfLvl &L, int i, int j, int k) {
  return ((k - 1) * L.n[1] + (j - 1)) * L.n[0] + (i - 1);
}

// barrier of the operation's participants: the workgroup, or wave 0 alone
template <bool WAVE>
__device__ __forceinline__ void pf_sync() {
  if (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    __syncthreads();
  }
}

// -DAFH_PFMG_TIMING (an experiment build, never the product): thread 0
// accumulates the shader clock spent per operation kind (each including
// its barrier) and prints the sums at the end of the kernel
#ifdef AFH_PFMG_TIMING
__device__ __forceinline__ unsigned long long *pf_tacc() {
  __shared__ unsigned long long acc[24];
  return acc;
}
#define PF_T(slot)                                        \
  do {                                                    \
    if (threadIdx.x == 0) {                               \
      unsigned long long *a_ = afh_pf::pf_tacc();         \
      const unsigned long long now_ = clock64();          \
      a_[slot] += now_ - a_[23];                          \
      a_[12 + (slot)] += 1;                               \
      a_[23] = now_;                                      \
    }                                                     \
  } while (0)
#else
#define PF_T(slot) \
  do {             \
  } while (0)
#endif

template <bool WAVE>
__device__ __forceinline__ int pf_nthr() {
  return WAVE ? 64 : (int)blockDim.x;
}

// sum over the level's stencil entries s (mask) of a_s x(p + s), from start
// value v0, subtracted (sub) or added -- pf_relax / pf_residual's loops.
// (Round 6 measured and left: all operand loads first, branch-free; the
// solve was no faster)
template <bool SUB>
__device__ __forceinline__ double pf_stencil(const PfLvl &L, const double *__restrict__ Al,
                                             const double *x, int p, double v0, bool center) {
  int i, j, k;
  pf_decode(L, p, i, j, k);
  double v = v0;
#pragma unroll
  for (int s = 0; s < 27; s++) {
    if (!((L.mask >> s) & 1) || (s == 13 && !center)) continue;
    const int ii = i + s % 3 - 1, jj = j + (s / 3) % 3 - 1, kk = k + s / 9 - 1;
    if (ii < 1 || ii > L.n[0] || jj < 1 || jj > L.n[1] || kk < 1 || kk > L.n[2]) continue;
    const double t = Al[(size_t)s * L.np + p] * x[pf_pt(L, ii, jj, kk)];
    v = SUB ? v - t : v + t;
  }
  return v;
}

// weighted Jacobi (pf_relax), level l: zero guess x = w b / a_c into xo;
// else from xi into xo (the other image): x' = (1 - w) x + w t
template <bool WAVE>
__device__ __forceinline__ void pf_relax(const PfLvl &L, const double *__restrict__ Al,
                                         const double *xi, double *xo, const double *b,
                                         bool zero) {
  for (int p = threadIdx.x; p < L.np; p += pf_nthr<WAVE>()) {
    const double ac = Al[(size_t)13 * L.np + p];
    if (zero) {
      double v = b[L.off + p] / ac;
      if (L.w != 1.0) v = L.w * v;
      xo[L.off + p] = v;
    } else {
      const double t = pf_stencil<true>(L, Al, xi + L.off, p, b[L.off + p], false) / ac;
      const double xv = xi[L.off + p];
      xo[L.off + p] = L.w == 1.0 ? t : (1.0 - L.w) * xv + L.w * t;
    }
  }
  pf_sync<WAVE>();
  PF_T(WAVE ? 6 : 0);
}

// r = b - A x (pf_residual)
template <bool WAVE>
__device__ __forceinline__ void pf_residual(const PfLvl &L, const double *__restrict__ Al,
                                            const double *x, const double *b, double *r) {
  for (int p = threadIdx.x; p < L.np; p += pf_nthr<WAVE>())
    r[L.off + p] = b[L.off + p] - pf_stencil<false>(L, Al, x + L.off, p, 0.0, true);
  pf_sync<WAVE>();
  PF_T(WAVE ? 7 : 1);
}

// the level's stride and size along its coarsening direction (no indexing
// of a per-lane array by cdir: that would live in scratch memory)
__device__ __forceinline__ int pf_cstride(const PfLvl &F) {
  return F.cdir == 0 ? 1 : F.cdir == 1 ? F.n[0] : F.n[0] * F.n[1];
}
__device__ __forceinline__ int pf_csize(const PfLvl &F) {
  return F.cdir == 0 ? F.n[0] : F.cdir == 1 ? F.n[1] : F.n[2];
}

// b_{l+1} = R src_l (pf_restrict; src = r, or b on a skipped level)
template <bool WAVE>
__device__ __forceinline__ void pf_restrict(const PfLvl &F, const PfLvl &C,
                                            const double *__restrict__ Pw, const double *src,
                                            double *b) {
  const int cd = F.cdir, st = pf_cstride(F), nf = pf_csize(F);
  const double *Pl = Pw + (size_t)2 * F.off;
  for (int p = threadIdx.x; p < C.np; p += pf_nthr<WAVE>()) {
    int c0, c1, c2;
    pf_decode(C, p, c0, c1, c2);
    const int cc = cd == 0 ? c0 : cd == 1 ? c1 : c2;
    // the fine point 2 c along cdir, then its two neighbours along it
    const int q0 = pf_pt(F, cd == 0 ? 2 * c0 : c0, cd == 1 ? 2 * c1 : c1, cd == 2 ? 2 * c2 : c2);
    double v = src[F.off + q0];
    {
      const int q = q0 - st;
      v = v + Pl[(size_t)F.np + q] * src[F.off + q];
    }
    if (2 * cc + 1 <= nf) {
      const int q = q0 + st;
      v = v + Pl[q] * src[F.off + q];
    }
    b[C.off + p] = v;
  }
  pf_sync<WAVE>();
  PF_T(WAVE ? 8 : 2);
}

// x_l += P x_{l+1} (pf_interp_add); assign: x_l = P x_{l+1} (a skipped level)
template <bool WAVE>
__device__ __forceinline__ void pf_interp(const PfLvl &F, const PfLvl &C,
                                          const double *__restrict__ Pw, const double *xc,
                                          double *x, bool assign) {
  const int cd = F.cdir, nf = pf_csize(F);
  const int cst = cd == 0 ? 1 : cd == 1 ? C.n[0] : C.n[0] * C.n[1];
  const double *Pl = Pw + (size_t)2 * F.off;
  for (int p = threadIdx.x; p < F.np; p += pf_nthr<WAVE>()) {
    int f0, f1, f2;
    pf_decode(F, p, f0, f1, f2);
    const int fc = cd == 0 ? f0 : cd == 1 ? f1 : f2;
    // the coarse point with cdir coordinate 1 (then + (m - 1) cst for m)
    const int pc1 = pf_pt(C, cd == 0 ? 1 : f0, cd == 1 ? 1 : f1, cd == 2 ? 1 : f2);
    double e;
    if (!(fc & 1)) {
      e = xc[C.off + pc1 + (fc / 2 - 1) * cst];
    } else {
      e = 0.0;
      if (fc >= 3) e = Pl[p] * xc[C.off + pc1 + ((fc - 1) / 2 - 1) * cst];
      if (fc + 1 <= nf) e = e + Pl[(size_t)F.np + p] * xc[C.off + pc1 + ((fc + 1) / 2 - 1) * cst];
    }
    x[F.off + p] = assign ? e : x[F.off + p] + e;
  }
  pf_sync<WAVE>();
  PF_T(WAVE ? 9 : 3);
}

// v.v on level 0 (pf_dot: 64 strided partial sums, pairwise tree); every
// lane gets the value. Needs v complete (a barrier before).
__device__ __forceinline__ double pf_dot(const PfLvl &L, const double *v, double *slot) {
  if (threadIdx.x < 64) {
    double s = 0.0;
    for (int p = threadIdx.x; p < L.np; p += PF_NPART) s = s + v[p] * v[p];
    for (int st = 32; st > 0; st >>= 1) s = s + __shfl_down(s, st, 64);
    if (threadIdx.x == 0) *slot = s;
  }
  __syncthreads();
  const double out = *slot;
  __syncthreads();
  PF_T(4);
  return out;
}

// The device tables of a hierarchy: per level its PfLvl, the operators as
// 27 arrays of the level's points (SoA) and the two interpolation weights
// likewise.
inline void pf_device_tables(const afh_pfmg &h, std::vector<PfLvl> &lv, std::vector<double> &A,
                             std::vector<double> &P) {
  const size_t np = h.off[h.nl];
  lv.assign(h.nl, PfLvl());
  A.assign(27 * np, 0.0);
  P.assign(2 * np, 0.0);
  auto lg = [](int n) {
    int e = 0;
    while ((1 << e) < n) e++;
    return (1 << e) == n ? e : -1;
  };
  for (int l = 0; l < h.nl; l++) {
    PfLvl &L = lv[l];
    for (int d = 0; d < 3; d++) L.n[d] = h.n[l][d];
    L.cdir = l + 1 < h.nl ? h.cdir[l] : -1;
    L.active = h.active[l];
    L.off = (int)h.off[l];
    L.np = (int)(h.off[l + 1] - h.off[l]);
    L.w = h.w[l];
    L.lgx = lg(L.n[0]);
    L.lgy = lg(L.n[1]);
    L.mask = 0;
    for (int p = 0; p < L.np; p++)
      for (int s = 0; s < 27; s++) {
        const double a = h.A[27 * ((size_t)L.off + p) + s];
        A[(size_t)27 * L.off + (size_t)s * L.np + p] = a;
        if (a != 0.0) L.mask |= 1u << s;
      }
    for (int p = 0; p < L.np; p++)
      for (int c = 0; c < 2; c++)
        P[(size_t)2 * L.off + (size_t)c * L.np + p] = h.P[2 * ((size_t)L.off + p) + c];
  }
}

// First level of at most PF_WAVE_PTS points below level 0 (nl: none; 1 at
// the least, level 0 always runs on the workgroup)
inline int pf_wave_from(const std::vector<PfLvl> &lv, int wave_pts = PF_WAVE_PTS) {
  int ls = (int)lv.size();
  for (int l = (int)lv.size() - 1; l >= 1 && lv[l].np <= wave_pts; l--) ls = l;
  return ls;
}

// LDS bytes of pf_solve_block: two x images, b, r (np each), the staged
// operators of the wave levels, the dot product's slot
inline size_t pf_lds_bytes(const std::vector<PfLvl> &lv, bool stage,
                           int wave_pts = PF_WAVE_PTS) {
  const size_t np = lv.back().off + lv.back().np;
  const int ls = pf_wave_from(lv, wave_pts);
  const size_t nsm = ls < (int)lv.size() ? np - lv[ls].off : 0;
  return sizeof(double) * (4 * np + (stage ? 27 * nsm : 0) + 1);
}

// The down leg below `from` .. the bottom .. the up leg back to `from`, on
// the participants WAVE says (the wave part of a cycle, or all of it)
// (Aw: the operators of levels from.. (SoA per level as in A), first
// point soff)
template <bool WAVE>
__device__ __forceinline__ void pf_legs(const PfLvl *__restrict__ Lg, int nl, int from,
                                        const double *Aw, int soff,
                                        const double *__restrict__ Pw, double *X0, double *X1,
                                        uint64_t &cur, double *b, double *r) {
  auto X = [&](int c) { return c ? X1 : X0; };
  auto Al = [&](const PfLvl &L) { return Aw + (size_t)27 * (L.off - soff); };
  int l;
  for (l = from; l <= nl - 2; l++) {
    const PfLvl L = Lg[l];
    const int c = (cur >> l) & 1;
    if (L.active) {
      pf_relax<WAVE>(L, Al(L), X(c), X(c), b, true);
      pf_residual<WAVE>(L, Al(L), X(c), b, r);
      pf_restrict<WAVE>(L, Lg[l + 1], Pw, r, b);
    } else {
      pf_restrict<WAVE>(L, Lg[l + 1], Pw, b, b);
    }
  }
  {
    const PfLvl L = Lg[nl - 1];  // the bottom (always relaxed)
    const int c = (cur >> (nl - 1)) & 1;
    pf_relax<WAVE>(L, Al(L), X(c), X(c), b, true);
  }
  for (l = nl - 2; l >= from; l--) {
    const PfLvl L = Lg[l];
    const int c = (cur >> l) & 1, cc = (cur >> (l + 1)) & 1;
    pf_interp<WAVE>(L, Lg[l + 1], Pw, X(cc), X(c), !L.active);
    if (L.active) {
      pf_relax<WAVE>(L, Al(L), X(c), X(c ^ 1), b, false);
      cur ^= 1ull << l;
    }
  }
}

// pfmg_solve.c on one workgroup (at least 64 lanes): X0 and b of level 0
// hold the guess and the folded rhs; the rest is work space. A: the
// operators of every level (SoA per level); Aw: those of the wave levels
// wave_from.. (staged in LDS, or A's), first point soff. Returns the
// iteration count (HYPRE_StructPFMGGetNumIterations); *cur_out: the image
// (0: X0, 1: X1) holding x of level 0.
__device__ inline int pf_solve_block(const PfLvl *__restrict__ Lg, int nl, int wave_from,
                                     const double *__restrict__ A, const double *Aw, int soff,
                                     const double *__restrict__ Pw, double *X0, double *X1,
                                     double *b, double *r, double *slot, double tol,
                                     int max_iter, int *cur_out) {
  const PfLvl L0 = Lg[0];
  auto X = [&](int c) { return c ? X1 : X0; };
  auto Al = [&](const PfLvl &L) { return A + (size_t)27 * L.off; };
  uint64_t cur = 0;  // per level: the image holding its x
  int iters = 0;
  const double bb = pf_dot(L0, b, slot);
  *cur_out = 0;
  if (bb == 0.0) {
    for (int p = threadIdx.x; p < L0.np; p += blockDim.x) X0[p] = 0.0;
    __syncthreads();
    return 0;
  }
  const double eps = tol * tol;
  for (int it = 0; it < max_iter; it++) {
    pf_relax<false>(L0, Al(L0), X(cur & 1), X((cur & 1) ^ 1), b, false);
    cur ^= 1;
    pf_residual<false>(L0, Al(L0), X(cur & 1), b, r);
    if (tol > 0.0) {
      const double rr = pf_dot(L0, r, slot);
      if (rr / bb < eps && it > 0) break;
    }
    if (nl > 1) {
      pf_restrict<false>(L0, Lg[1], Pw, r, b);
      // levels 1 .. wave_from - 1 on the workgroup, down
      const int top = wave_from < nl - 1 ? wave_from : nl - 1;
      int l;
      for (l = 1; l < top; l++) {
        const PfLvl L = Lg[l];
        const int c = (cur >> l) & 1;
        if (L.active) {
          pf_relax<false>(L, Al(L), X(c), X(c), b, true);
          pf_residual<false>(L, Al(L), X(c), b, r);
          pf_restrict<false>(L, Lg[l + 1], Pw, r, b);
        } else {
          pf_restrict<false>(L, Lg[l + 1], Pw, b, b);
        }
      }
      if (wave_from >= nl) {
        // no wave part: the bottom on the workgroup
        const PfLvl L = Lg[nl - 1];
        const int c = (cur >> (nl - 1)) & 1;
        pf_relax<false>(L, Al(L), X(c), X(c), b, true);
      } else {
        if (threadIdx.x < 64) pf_legs<true>(Lg, nl, wave_from, Aw, soff, Pw, X0, X1, cur, b, r);
        // wave 0's images of the wave levels, to every lane
        __shared__ unsigned long long pf_cur;
        __syncthreads();
        PF_T(5);
        if (threadIdx.x == 0) pf_cur = cur;
        __syncthreads();
        cur = pf_cur;
      }
      // the up leg on the workgroup
      for (l = top - 1; l >= 1; l--) {
        const PfLvl L = Lg[l];
        const int c = (cur >> l) & 1, cc = (cur >> (l + 1)) & 1;
        pf_interp<false>(L, Lg[l + 1], Pw, X(cc), X(c), !L.active);
        if (L.active) {
          pf_relax<false>(L, Al(L), X(c), X(c ^ 1), b, false);
          cur ^= 1ull << l;
        }
      }
      pf_interp<false>(L0, Lg[1], Pw, X((cur >> 1) & 1), X(cur & 1), false);
    }
    pf_relax<false>(L0, Al(L0), X(cur & 1), X((cur & 1) ^ 1), b, false);
    cur ^= 1;
    iters = it + 1;
  }
  *cur_out = (int)(cur & 1);
  return iters;
}

}  // namespace afh_pf

#endif
