// FAS multigrid V-cycle over the box tree (afivo/src/m_af_multigrid.f90).
//
// Kernels, one launch per pass over one level (all boxes of the level):
//   k_gsrb          stencil_gsrb_357, constant 7-point stencil (m_af_stencil.f90:938-955)
//   k_residual      residual_box = rhs - stencil_apply_357 (m_af_multigrid.f90:801-810)
//   k_rstr_fas      update_coarse part 1: residual of the 8 fine cells of
//                   each parent cell + 8-cell means of residual and phi
//                   (m_af_multigrid.f90:704-717, af_restrict_box); the child's
//                   tmp is never written (the reference restores it)
//   k_parent_rhs    update_coarse part 2: rhs = L phi + tmp, tmp = phi (726-736)
//   k_corr_tmp      correct_children part 1: tmp = phi - tmp (636-637)
//   k_prolong       stencil_prolong_248 add (m_af_stencil.f90:749-771)
//   k_gradient      mg_box_lpl_gradient + mg_box_field_norm (1882-2025)
// plus the level-1 coarse solver (ours; the reference calls HYPRE PFMG).
#include <hip/hip_ext.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <map>

#include "afh_internal.h"
#include "afh_cs_direct.h"
#include "afh_pfmg_dev.h"

#include <mutex>

namespace afh {

struct Coef {
  double c[7];
};

constexpr int MAXMG = 16;
constexpr int CS_BOTTOM_SWEEPS = 16;   // same constant as oracle/c/afo.c
constexpr int CS_SMALL_CELLS = 4096;   // MG levels <= 16^3 run in one workgroup
constexpr int CS_DS_N = 16;            // k_cs_direct_small: LDS matrices up to 16 x 16
// k_cs_direct_small serves level-1 grids up to 1024 cells (S3's 8^3: 15 us,
// against ~25 us for the eight launches of k_cs_gather / k_cs_transform /
// k_cs_scatter); S1's 16^3 runs those: one workgroup is latency-bound there
// (one wave per SIMD), 0.573 against 0.551 ms per step with one thread per
// grid line (profiles/r03_ab_cs_direct_lines.txt; AFH_CS_DS_CELLS=4096 for A/B)
constexpr int CS_DS_CELLS = 1024;

struct CsParams {
  int n_mg;
  int dims[MAXMG][3];
  double hc[MAXMG][3];
  double cdiag[MAXMG];
  int bctype[6];
  int halo[MAXMG];  // 1: global arrays with a ghost layer, 0: compact (LDS)
  int lg[MAXMG];    // log2(nx) | log2(ny) << 8 when both are powers of 2, else -1
  double *u[MAXMG], *f[MAXMG];
  const double *dtab;  // [MAXMG][64][2] folded (diag, 1/diag) per class
};


// ------------------------------------------------------------ box kernels
// Gauss-Seidel update of cell c from its six neighbours (stencil_gsrb_357).
__device__ __forceinline__ double gs_cell(const double *__restrict__ x,
                                          const double *__restrict__ r,
                                          size_t c, size_t sj, size_t sk,
                                          const Coef &cf, double inv_c1) {
  return (r[c] - cf.c[1] * x[c - 1] - cf.c[2] * x[c + 1] - cf.c[3] * x[c - sj] -
          cf.c[4] * x[c + sj] - cf.c[5] * x[c - sk] - cf.c[6] * x[c + sk]) *
         inv_c1;
}

__global__ void k_gsrb(double *__restrict__ phi, const double *__restrict__ rhs,
                       const int32_t *__restrict__ ids, int nc, size_t bsz,
                       Coef cf, double inv_c1, int redblack) {
  const int hn = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hn * nc * nc) return;
  const int id = ids[blockIdx.y];
  int ih, j, k;
  if ((nc & (nc - 1)) == 0) {
    const int ln = __builtin_ctz(nc);
    ih = t & (hn - 1);
    j = ((t >> (ln - 1)) & (nc - 1)) + 1;
    k = (t >> (2 * ln - 1)) + 1;
  } else {
    ih = t % hn;
    j = (t / hn) % nc + 1;
    k = t / (hn * nc) + 1;
  }
  const int i = 2 - ((redblack ^ (k + j)) & 1) + 2 * ih;
  const int ng = nc + 2;
  double *x = phi + (size_t)(id - 1) * bsz;
  const double *r = rhs + (size_t)(id - 1) * bsz;
  x[ix3(ng, i, j, k)] =
      gs_cell(x, r, ix3(ng, i, j, k), ng, (size_t)ng * ng, cf, inv_c1);
}

// ------------------------------------------------------------ fused GSRB pair
// Half-sweeps n (odd, "red": i+j+k odd) and n+1 ("black") of gsrb_boxes
// (m_af_multigrid.f90:741-760) in ONE pass, without the level ghost fill
// between them; bitwise the same result as the two half-sweeps with
// af_gc_lvl in between.
//
// The pair reads `src` and writes the interior of `dst` (ping-pong between
// phi and a spare image), so every input is an old value and workgroups
// never race. One workgroup per tile of TJ rows (j) of a box marches over
// the k planes, holding four planes P[s-2..s+1] of its rows plus one halo
// row on each side (and the i ghosts) in LDS. Step s:
//   A  red cells of plane s (in-plane and k neighbours: old black values)
//   B  the red values next to the tile that af_gc_lvl / the neighbouring
//      tile would provide after the red half-sweep: x ghosts of the tile's
//      rows; the halo rows (ghost row of the box, or the red cells of the
//      adjacent tile recomputed from `src`); the z ghost planes at s = 2 and
//      s = NC+1. A same-level neighbour's red boundary cell is recomputed
//      from that neighbour's `src` (bitwise what its workgroup computes);
//      physical / refinement faces use gc_face_nocopy with the box's current
//      red and black values (coarse data from `coarse`, i.e. phi).
//   C  black cells of plane s-1 (new red neighbours); plane s-1 of the tile
//      is complete and written once, in full rows
//   D  plane s+2 (prefetched into registers during the step) -> LDS
// Each plane of phi and rhs is read once and phi is written once per pair
// (24 B/cell algorithmic).
template <int NC, int TJ_ = NC>
struct RbGeom {
  static constexpr int NG = NC + 2;
  // rows per tile: whole boxes on levels with a box per CU (measured on
  // MI355X, S1-64 leaf level: 16-row tiles of 1024 threads 1.06 ms per pair,
  // whole boxes 0.87 ms -- the tiles' halo rows cost more than the extra
  // occupancy gains); NC/4-row tiles on levels with 64..255 boxes
  static constexpr int TJ = TJ_;
  static constexpr int NTILE = NC / TJ;
  static constexpr int PLT = (TJ + 2) * NG;            // LDS plane (rows j0-1..j1+1)
  static constexpr int NT = NC * TJ >= 1024 ? 1024 : (NC * TJ < 64 ? 64 : NC * TJ);
  static constexpr int CPT = (NC * TJ + NT - 1) / NT;  // columns per thread
  static constexpr int EPT = (PLT + NT - 1) / NT;      // plane entries per thread
};

// One red ghost cell p of face nb for k_gsrb_pair. x1v / x2v: this box's
// current values next to the face (x1 black, old; x2 red, new).
template <int NC>
__device__ __forceinline__ double pair_ghost_k(
    const double *__restrict__ src, const double *__restrict__ coarse,
    const double *__restrict__ rhs,
    const afh_box_meta *__restrict__ meta, const afh_box_meta &m, int nb,
    int nb_id, double drd, int p0, int p1, int p2, int a, int b, size_t bsz,
    const Coef &cf, double inv_c1, afh_bc bc, int rb, double x1v, double x2v) {
  constexpr int NG = NC + 2;
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int p[3] = {p0, p1, p2};
  if (nb_id > 0) {
    // the neighbour's red boundary cell, from its (old) black values; its
    // ghost cell on our side is a copy of our x1 cell, taken from here (a
    // sharded neighbour replica need not hold that ghost)
    int q[3] = {p0, p1, p2};
    q[d] = low ? NC : 1;
    const size_t o = (size_t)(nb_id - 1) * bsz;
    const double *xn = src + o;
    const size_t c = ix3(NG, q[0], q[1], q[2]);
    const size_t st[3] = {1, (size_t)NG, (size_t)NG * NG};
    double v[6] = {xn[c - 1],  xn[c + 1],  xn[c - st[1]],
                   xn[c + st[1]], xn[c - st[2]], xn[c + st[2]]};
    v[2 * d + (low ? 1 : 0)] = x1v;
    return (rhs[o + c] - cf.c[1] * v[0] - cf.c[2] * v[1] - cf.c[3] * v[2] -
            cf.c[4] * v[3] - cf.c[5] * v[4] - cf.c[6] * v[5]) *
           inv_c1;
  }
  const int x1 = low ? 1 : NC;
  return gc_face_nocopy_k(coarse, meta, m, nb, nb_id, drd, p, a, b, NC, bsz, bc, rb,
                          [&](const int *q) { return q[d] == x1 ? x1v : x2v; });
}

template <int NC>
__device__ __forceinline__ double pair_ghost(
    const double *__restrict__ src, const double *__restrict__ coarse,
    const double *__restrict__ rhs,
    const afh_box_meta *__restrict__ meta, const afh_box_meta &m, int nb,
    int p0, int p1, int p2, int a, int b, size_t bsz, const Coef &cf,
    double inv_c1, afh_bc bc, int rb, double x1v, double x2v) {
  return pair_ghost_k<NC>(src, coarse, rhs, meta, m, nb, m.neighbors[nb - 1],
                          m.dr[(nb - 1) >> 1], p0, p1, p2, a, b, bsz, cf, inv_c1, bc,
                          rb, x1v, x2v);
}

template <int NC, int TJ>
__global__ void __launch_bounds__((RbGeom<NC, TJ>::NT)) __attribute__((amdgpu_waves_per_eu(4)))
    k_gsrb_pair(const double *__restrict__ src, double *__restrict__ dst,
                const double *__restrict__ rhs,
                const double *__restrict__ coarse,
                const afh_box_meta *__restrict__ meta,
                const int32_t *__restrict__ ids, size_t bsz, Coef cf,
                double inv_c1, GcArgs ga) {
  using G = RbGeom<NC, TJ>;
  constexpr int NG = G::NG, HN = NC / 2, NT = G::NT, CPT = G::CPT,
                EPT = G::EPT, PLT = G::PLT;
  constexpr size_t SK = (size_t)NG * NG;
  __shared__ double P[4][PLT];  // planes s-2 .. s+1 at slot (plane & 3)
  const int tid = threadIdx.x;
  const int id = ids[blockIdx.x / G::NTILE];
  const int j0 = (blockIdx.x % G::NTILE) * TJ + 1, j1 = j0 + TJ - 1;
  const afh_box_meta &m = meta[id - 1];
  const double *x = src + (size_t)(id - 1) * bsz;
  double *y = dst + (size_t)(id - 1) * bsz;
  const double *r = rhs + (size_t)(id - 1) * bsz;
  const size_t t0 = (size_t)(j0 - 1) * NG;  // first LDS row in a plane
  // tile column q of this thread: (i, j), LDS index c (row j - j0 + 1)
  auto colof = [&](int q, int &i, int &j, int &c) {
    const int col = tid + NT * q;
    i = col % NC + 1;
    j = j0 + col / NC;
    c = (col / NC + 1) * NG + i;
    return col < NC * TJ;
  };

  // planes 0..2 -> LDS; rhs of plane 1 -> registers
  for (int e = tid; e < 3 * PLT; e += NT)
    P[e / PLT][e % PLT] = x[(size_t)(e / PLT) * SK + t0 + e % PLT];
  double r1[CPT], r2[CPT];
#pragma unroll
  for (int q = 0; q < CPT; q++) {
    int i, j, c;
    colof(q, i, j, c);
    r1[q] = 0;
    r2[q] = colof(q, i, j, c) ? r[SK + j * NG + i] : 0.0;
  }
  __syncthreads();

  for (int s = 1; s <= NC + 1; s++) {
    // prefetch plane s+2 of phi and the tile of plane s+1 of rhs
    double nx[EPT], nr[CPT];
#pragma unroll
    for (int q = 0; q < EPT; q++) {
      const int e = tid + NT * q;
      nx[q] = (s + 2 <= NC + 1 && e < PLT) ? x[(size_t)(s + 2) * SK + t0 + e]
                                            : 0.0;
    }
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      int i, j, c;
      const bool ok = colof(q, i, j, c);
      nr[q] = (ok && s + 1 <= NC) ? r[(size_t)(s + 1) * SK + j * NG + i] : 0.0;
    }
    double *Pm = P[(s - 1) & 3], *P0 = P[s & 3], *Pp = P[(s + 1) & 3];
    double *Pmm = P[(s - 2) & 3];
    // A: red cells of plane s
    if (s <= NC) {
#pragma unroll
      for (int q = 0; q < CPT; q++) {
        int i, j, c;
        if (colof(q, i, j, c) && ((i + j + s) & 1))
          P0[c] = (r2[q] - cf.c[1] * P0[c - 1] - cf.c[2] * P0[c + 1] -
                   cf.c[3] * P0[c - NG] - cf.c[4] * P0[c + NG] -
                   cf.c[5] * Pm[c] - cf.c[6] * Pp[c]) *
                  inv_c1;
      }
    }
    __syncthreads();
    // B: red values around the tile
    if (s <= NC) {
      for (int u = tid; u < TJ + NC; u += NT) {
        int i, j, jl;
        double v;
        if (u < TJ) {
          // x ghosts of the tile's rows
          j = j0 + u;
          jl = u + 1;
          i = ((j + s) & 1) ? 0 : NC + 1;
          const int nb = i == 0 ? 1 : 2;
          v = pair_ghost<NC>(src, coarse, rhs, meta, m, nb, i, j, s, j, s, bsz,
                             cf, inv_c1, ga.bc[nb - 1], ga.rb,
                             P0[jl * NG + (i == 0 ? 1 : NC)],
                             P0[jl * NG + (i == 0 ? 2 : NC - 1)]);
        } else {
          // halo rows j0-1 and j1+1
          const bool lo = u - TJ < HN;
          j = lo ? j0 - 1 : j1 + 1;
          jl = lo ? 0 : TJ + 1;
          i = 2 - ((1 ^ (s + j)) & 1) + 2 * ((u - TJ) % HN);
          if (j == 0 || j == NC + 1) {
            const int nb = j == 0 ? 3 : 4;
            const int l1 = j == 0 ? 1 : TJ, l2 = j == 0 ? 2 : TJ - 1;
            v = pair_ghost<NC>(src, coarse, rhs, meta, m, nb, i, j, s, i, s,
                               bsz, cf, inv_c1, ga.bc[nb - 1], ga.rb,
                               P0[l1 * NG + i], P0[l2 * NG + i]);
          } else {
            // red cell of the adjacent tile of this box
            v = gs_cell(x, r, ix3(NG, i, j, s), NG, SK, cf, inv_c1);
          }
        }
        P0[jl * NG + i] = v;
      }
    }
    if (s == 2 || s == NC + 1) {
      // z ghost plane 0 (NC+1): x1 = plane 1 (NC), black, old;
      // x2 = plane 2 (NC-1), red, new
      const int nb = s == 2 ? 5 : 6, k = s == 2 ? 0 : NC + 1;
      double *Pg = s == 2 ? Pmm : P0;
      const double *X2 = s == 2 ? P0 : Pmm;
#pragma unroll
      for (int q = 0; q < CPT; q++) {
        int i, j, c;
        if (colof(q, i, j, c) && ((i + j + k) & 1))
          Pg[c] = pair_ghost<NC>(src, coarse, rhs, meta, m, nb, i, j, k, i, j,
                                 bsz, cf, inv_c1, ga.bc[nb - 1], ga.rb, Pm[c],
                                 X2[c]);
      }
    }
    __syncthreads();
    // C: black cells of plane s-1; write the tile of plane s-1
    if (s >= 2) {
      const int k = s - 1;
#pragma unroll
      for (int q = 0; q < CPT; q++) {
        int i, j, c;
        if (!colof(q, i, j, c)) continue;
        const size_t g = (size_t)k * SK + (size_t)j * NG + i;
        if (!((i + j + k) & 1)) {
          const double v =
              (r1[q] - cf.c[1] * Pm[c - 1] - cf.c[2] * Pm[c + 1] -
               cf.c[3] * Pm[c - NG] - cf.c[4] * Pm[c + NG] - cf.c[5] * Pmm[c] -
               cf.c[6] * P0[c]) *
              inv_c1;
          y[g] = v;
        } else {
          y[g] = Pm[c];
        }
      }
    }
    __syncthreads();
    // D: plane s+2 into the slot of plane s-2
    if (s + 2 <= NC + 1) {
#pragma unroll
      for (int q = 0; q < EPT; q++) {
        const int e = tid + NT * q;
        if (e < PLT) P[(s + 2) & 3][e] = nx[q];
      }
    }
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      r1[q] = r2[q];
      r2[q] = nr[q];
    }
    __syncthreads();
  }
}

// Whole-box form of k_gsrb_pair with a parity mapping: in step s thread t
// owns the same RPT (i, j) columns for the red cells of plane s (phase A)
// and the black cells of plane s-1 (phase C) -- i = 2 ih + 1 + ((j + s) & 1)
// -- so every lane works in both phases (the column mapping of k_gsrb_pair
// idles half the lanes in each). Black cells are updated in place in LDS and
// plane s-1 is then written in full rows (phase E). Same arithmetic in the
// same order as k_gsrb_pair: bitwise identical results.
#ifndef AFH_PAIR_NB_LOADS  // 1: every neighbour value of phase B from global
#define AFH_PAIR_NB_LOADS 0
#endif
template <int NC, int TJ = NC, int NTM = 0>
struct RbPar {
  static constexpr int NG = NC + 2, HN = NC / 2;
  static constexpr int NTILE = NC / TJ;
  static constexpr int NRED = TJ * HN;                      // red cells per tile plane
  // tiles: 2 workgroups per CU
  static constexpr int NTMAX = NTM ? NTM : (TJ == NC ? 1024 : 512);
  static constexpr int NT = NRED >= NTMAX ? NTMAX : NRED;
  static constexpr int RPT = NRED / NT;                     // red cells per thread
  static constexpr int PL = (TJ + 2) * NG;                  // LDS plane (rows j0-1..j1+1)
  static constexpr int EPT = (PL + NT - 1) / NT;            // plane entries per thread
  static constexpr int OPT = (NC * TJ + NT - 1) / NT;       // stored cells per thread
  static constexpr int OPTF = (NG * TJ + NT - 1) / NT;      // same, rows with x ghosts
};

// Parity-mapped form of k_gsrb_pair: in step s thread t owns the same RPT
// (i, j) columns for the red cells of plane s (phase A) and the black cells
// of plane s-1 (phase C) -- i = 2 ih + 1 + ((j + s) & 1) -- so every lane
// works in both phases (the column mapping of k_gsrb_pair idles half the
// lanes in each). Black cells are updated in place in LDS and plane s-1 is
// then written in full rows (phase E). A workgroup holds TJ rows of a box
// (TJ < NC: 512-thread workgroups, two per CU, halo rows recomputed as in
// k_gsrb_pair). Same arithmetic in the same order as k_gsrb_pair: bitwise
// identical results.
// DEPTH: planes of phi / rhs in flight per workgroup (1: loaded and stored
// in the same step; 2: loaded one step earlier). Plane rows are stored
// whole, x ghost cells included (one contiguous run per tile plane, no
// partially written cache lines; the level fill after the pair rewrites
// every ghost cell of dst).
// KS: the k planes split into KS chunks, one workgroup each (levels with
// too few boxes to fill the chip): a chunk recomputes the red cells of the
// plane below it (as tiles recompute halo rows) and stores its own planes.
// (Measured and removed in round 5: non-temporal plane loads, interior-only
// row stores, four barriers per plane, natural LDS row order, 512-thread
// whole boxes, the x ghost cells of the fill formed in the pair --
// profiles/r03_ab_*, r04_ab_*.)
template <int NC, int TJ, int DEPTH = 2, int KS = 1>
__global__ void __launch_bounds__((RbPar<NC, TJ>::NT))
    k_gsrb_pair2(const double *__restrict__ src, double *__restrict__ dst,
                 const double *__restrict__ rhs, const double *__restrict__ coarse,
                 const afh_box_meta *__restrict__ meta,
                 const int32_t *__restrict__ ids, size_t bsz, Coef cf,
                 double inv_c1, GcArgs ga) {
  using G = RbPar<NC, TJ>;
  constexpr int NG = G::NG, HN = G::HN, NT = G::NT, RPT = G::RPT, PL = G::PL,
                EPT = G::EPT;
  constexpr size_t SK = (size_t)NG * NG;
  __shared__ double P[4][PL];  // planes s-2 .. s+1 at slot (plane & 3)
  // LDS row layout (split parity): each row holds its even-i cells, then
  // its odd-i cells, so the red (black) cells the lanes of a row update and
  // all their neighbours are unit-stride in LDS (no bank conflicts); the
  // plane image is permuted on its way in (D) and out (E).
  constexpr int HG = NG / 2;
  auto L = [](int jl, int i) { return jl * NG + ((i & 1) ? HG + (i >> 1) : (i >> 1)); };
  auto perm = [&](int e) { return L(e / NG, e % NG); };  // plane entry -> LDS
  const int tid = threadIdx.x;
  const int wgs = xcd_swizzle(blockIdx.x, gridDim.x);
  const int chunk = wgs % KS, wg = wgs / KS;
  const int id = ids[wg / G::NTILE];
  const int j0 = (wg % G::NTILE) * TJ + 1, j1 = j0 + TJ - 1;
  constexpr int KC = NC / KS;
  const int k0 = chunk * KC + 1, k1 = k0 + KC - 1;  // planes this workgroup stores
  const int s0 = chunk == 0 ? 1 : k0 - 1;            // first step
  const afh_box_meta &m = meta[id - 1];
  // the box's neighbour ids and spacings, wave-uniform, read once: per-lane
  // metadata loads in the loop would wait for the plane prefetch (vmcnt(0))
  // (separate scalars, not an array: a selected array element becomes a
  // scratch load)
  const int nb1 = m.neighbors[0], nb2 = m.neighbors[1], nb3 = m.neighbors[2],
            nb4 = m.neighbors[3], nb5 = m.neighbors[4], nb6 = m.neighbors[5];
  const double dr0 = m.dr[0], dr1 = m.dr[1], dr2 = m.dr[2];
  auto nbid = [&](int nb) {
    return nb == 1 ? nb1 : nb == 2 ? nb2 : nb == 3 ? nb3 : nb == 4 ? nb4 : nb == 5 ? nb5 : nb6;
  };
  auto drof = [&](int nb) {
    const int d = (nb - 1) >> 1;
    return d == 0 ? dr0 : d == 1 ? dr1 : dr2;
  };
  // the face's boundary condition, selected the same way (a per-lane index
  // into the kernel-argument array would be a scratch copy)
  auto bcof = [&](int nb) {
    afh_bc b;
    b.type = nb == 1 ? ga.bc[0].type : nb == 2 ? ga.bc[1].type : nb == 3 ? ga.bc[2].type
           : nb == 4 ? ga.bc[3].type : nb == 5 ? ga.bc[4].type : ga.bc[5].type;
    b.value = nb == 1 ? ga.bc[0].value : nb == 2 ? ga.bc[1].value : nb == 3 ? ga.bc[2].value
            : nb == 4 ? ga.bc[3].value : nb == 5 ? ga.bc[4].value : ga.bc[5].value;
    return b;
  };
  const double *x = src + (size_t)(id - 1) * bsz;
  double *y = dst + (size_t)(id - 1) * bsz;
  const double *r = rhs + (size_t)(id - 1) * bsz;
  const size_t t0 = (size_t)(j0 - 1) * NG;  // first LDS row in a plane
  // owned column q in step s: (i, j), LDS index (j - j0 + 1) * NG + i
  auto col = [&](int q, int s, int &i, int &j) {
    const int rr = tid + NT * q;
    j = j0 + rr / HN;
    i = 2 * (rr % HN) + 1 + ((j + s) & 1);
    return L(j - j0 + 1, i);
  };

  // planes s0-1 .. s0+1 -> LDS; rhs of the red cells of plane s0
  for (int e = tid; e < 3 * PL; e += NT) {
    const int pl = s0 - 1 + e / PL;
    P[pl & 3][perm(e % PL)] = x[(size_t)pl * SK + t0 + e % PL];
  }
  // rhs in registers: rR red cells of plane s, rB black cells of plane s-1,
  // rBn black cells of plane s (step s+1). Both parities of a plane are
  // loaded in the same step (adjacent cells 2 ih + 1, 2 ih + 2 of a row), so
  // each rhs line is fetched once.
  double rR[RPT], rB[RPT], rBn[RPT];
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    const int rr = tid + NT * q;
    const int j = j0 + rr / HN, i1 = 2 * (rr % HN) + 1;
    const double lo = r[(size_t)s0 * SK + (size_t)j * NG + i1],
                 hi = r[(size_t)s0 * SK + (size_t)j * NG + i1 + 1];
    const bool odd = (j + s0) & 1;  // red cell of plane s0 is i1 + 1
    rR[q] = odd ? hi : lo;
    rBn[q] = odd ? lo : hi;
    rB[q] = 0.0;
  }
  __syncthreads();

  // B inputs (one step ahead, so phase B never waits on them): thread
  // u < TJ + NC owns one red ghost value of plane s. A same-level
  // neighbour's red boundary cell (or, for tiles, the adjacent tile's red
  // cell) is 6 neighbour values and an rhs value; physical / refinement
  // faces are evaluated in B (gc_face_nocopy).
  // x faces: the neighbour's boundary column is a copy in this box's ghost
  // column (the last level fill), so its rows j+-1 and planes s+-1 are read
  // from LDS where they are interior cells of the neighbour (unchanged
  // black values); only phi next to it and rhs come from the neighbour
  constexpr int NBL = TJ + NC;
  struct BDesc {
    int i, j, jl, nb, rep;  // nb 0: none
    bool pre, lm, lp, zm, zp;
    const double *xs, *rs;
    size_t c;
  };
  auto bdesc = [&](int s) {
    BDesc b;
    b.i = b.j = b.jl = b.nb = 0;
    b.rep = -1;
    b.pre = b.lm = b.lp = b.zm = b.zp = false;
    b.xs = b.rs = nullptr;
    b.c = 0;
    if (s >= k0 && s <= k1 && tid < TJ + NC) {
      const int u = tid;
      if (u < TJ) {
        b.j = j0 + u;
        b.jl = u + 1;
        b.i = ((b.j + s) & 1) ? 0 : NC + 1;
        b.nb = b.i == 0 ? 1 : 2;
      } else {
        const bool lo = u - TJ < HN;
        b.j = lo ? j0 - 1 : j1 + 1;
        b.jl = lo ? 0 : TJ + 1;
        b.i = 2 - ((1 ^ (s + b.j)) & 1) + 2 * ((u - TJ) % HN);
        b.nb = (b.j == 0 || b.j == NC + 1) ? (b.j == 0 ? 3 : 4) : 7;
      }
      int q[3] = {b.i, b.j, s};
      if (b.nb == 7) {
        b.xs = x;
        b.rs = r;
      } else {
        const int nb_id = nbid(b.nb);
        if (nb_id > 0) {
          const int d = (b.nb - 1) >> 1;
          const bool low = ((b.nb - 1) & 1) == 0;
          q[d] = low ? NC : 1;
          b.xs = src + (size_t)(nb_id - 1) * bsz;
          b.rs = rhs + (size_t)(nb_id - 1) * bsz;
          b.rep = 2 * d + (low ? 1 : 0);
        }
      }
      if (b.xs) {
        b.pre = true;
        b.c = ix3(NG, q[0], q[1], q[2]);
#if !AFH_PAIR_NB_LOADS
        const bool xg = b.rep == 0 || b.rep == 1;
        b.lm = xg && b.j >= 2;
        b.lp = xg && b.j <= NC - 1;
        b.zm = xg && s >= 2;
        b.zp = xg && s <= NC - 1;
#endif
      }
    }
    return b;
  };
  struct BIn {
    double bl[7];
  };
  // unconditional loads (lanes without a B value read a valid dummy cell):
  // a per-lane select around a load makes hipcc wait for each one
  auto load_b = [&](int s) {
    const BDesc d = bdesc(s);
    BIn b;
#pragma unroll
    for (int q = 0; q < 7; q++) b.bl[q] = 0.0;
    if (s >= k0 && s <= k1 && tid < NBL) {
      // values taken from LDS or replaced later re-read cell c (no extra
      // cache line)
      const double *xs = d.pre ? d.xs : x, *rs = d.pre ? d.rs : r;
      const size_t c = d.pre ? d.c : ix3(NG, 1, j0, 1);
      const long o2 = (d.rep == 2 || d.lm) ? 0 : -(long)NG;
      const long o3 = (d.rep == 3 || d.lp) ? 0 : (long)NG;
      const long o4 = (d.rep == 4 || d.zm) ? 0 : -(long)SK;
      const long o5 = (d.rep == 5 || d.zp) ? 0 : (long)SK;
      b.bl[0] = xs[c - 1];
      b.bl[1] = xs[c + 1];
      b.bl[2] = xs[c + o2];
      b.bl[3] = xs[c + o3];
      b.bl[4] = xs[c + o4];
      b.bl[5] = xs[c + o5];
      b.bl[6] = rs[c];
    }
    return b;
  };
  BIn bc = load_b(s0);
  // phi planes and rhs rows in flight: loaded in step s, consumed (LDS /
  // rotation) in step s+1 -- two planes of each per workgroup in flight
  struct Pf {
    double nx[EPT], nlo[RPT], nhi[RPT];
  };
  auto load_pf = [&](Pf &f, int kp) {  // phi plane kp, rhs plane kp - 1
    // (clamped indices instead of per-lane guards; a plane beyond NC + 1 is
    // never stored)
    const int kx = kp <= NC + 1 ? kp : NC + 1, kr = kp - 1 <= NC ? kp - 1 : NC;
#pragma unroll
    for (int e = 0; e < EPT; e++) {
      const int xx = tid + NT * e;
      f.nx[e] = x[(size_t)kx * SK + t0 + (xx < PL ? xx : PL - 1)];
    }
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const int rr = tid + NT * q;
      const int j = j0 + rr / HN, i1 = 2 * (rr % HN) + 1;
      const size_t g = (size_t)kr * SK + (size_t)j * NG + i1;
      f.nlo[q] = r[g];
      f.nhi[q] = r[g + 1];
    }
  };
  Pf X0, X1;
  if (DEPTH == 2) load_pf(X0, s0 + 2);

  // E: plane k of the tile to dst, in full rows
  auto store_plane = [&](const int k, const double *Pk) {
#pragma unroll
    for (int q = 0; q < G::OPTF; q++) {
      const int e = tid + NT * q;
      if (e < NG * TJ) st_nt<AFH_NT_PAIR>(y + ((size_t)k * SK + t0 + NG + e), Pk[perm(NG + e)]);
    }
  };
  // Step s, three barriers: A (red cells of plane s) with E of plane s-2 |
  // B (red ghosts of plane s: they are first read by C of step s+1) with C
  // (black cells of plane s-1) | D. At s = 2 and NC+1 the z ghost plane is
  // written between B and C (C reads it; it reads the black cells C
  // updates).
  auto step = [&](const int s, Pf &ld, const Pf &cn) {
    const BIn bn = load_b(s + 1);
    load_pf(ld, s + 1 + DEPTH);
    double *bl = bc.bl;
    const BDesc bd = bdesc(s);
    const int b_i = bd.i, b_j = bd.j, b_jl = bd.jl, b_nb = bd.nb, b_rep = bd.rep;
    const bool b_pre = bd.pre, b_lm = bd.lm, b_lp = bd.lp, b_zm = bd.zm, b_zp = bd.zp;
    double *Pm = P[(s - 1) & 3], *P0 = P[s & 3], *Pp = P[(s + 1) & 3];
    double *Pmm = P[(s - 2) & 3];
    // A: red cells of plane s
    if (s <= NC) {
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        int i, j;
        const int c = col(q, s, i, j);
        const int cm = L(j - j0 + 1, i - 1), cp = L(j - j0 + 1, i + 1);
        P0[c] = (rR[q] - cf.c[1] * P0[cm] - cf.c[2] * P0[cp] -
                 cf.c[3] * P0[c - NG] - cf.c[4] * P0[c + NG] - cf.c[5] * Pm[c] -
                 cf.c[6] * Pp[c]) *
                inv_c1;
      }
    }
    if (s - 2 >= k0 && s - 2 < k1) store_plane(s - 2, Pmm);
    __syncthreads();
    // B: red values around the tile: x ghost cells of its rows; the halo
    // rows (ghost row of the box, or the red cells of the adjacent tile
    // recomputed from src) -- same arithmetic as pair_ghost / gs_cell
    if (b_nb) {
      double v;
      if (b_pre) {
        if (b_rep >= 0) {
          // x1v: this box's cell next to the face (black, old)
          const int d = b_rep >> 1;
          int p1[3] = {b_i, b_jl, 0};
          p1[d] = (b_rep & 1) ? (d == 0 ? 1 : 1) : (d == 0 ? NC : TJ);
          const double x1v = P0[L(p1[1], p1[0])];
#pragma unroll
          for (int q = 0; q < 6; q++)
            if (q == b_rep) bl[q] = x1v;
        }
        if (b_lm) bl[2] = P0[L(b_jl - 1, b_i)];
        if (b_lp) bl[3] = P0[L(b_jl + 1, b_i)];
        if (b_zm) bl[4] = Pm[L(b_jl, b_i)];
        if (b_zp) bl[5] = Pp[L(b_jl, b_i)];
        v = (bl[6] - cf.c[1] * bl[0] - cf.c[2] * bl[1] - cf.c[3] * bl[2] -
             cf.c[4] * bl[3] - cf.c[5] * bl[4] - cf.c[6] * bl[5]) *
            inv_c1;
      } else if (b_nb <= 2) {
        v = pair_ghost_k<NC>(src, coarse, rhs, meta, m, b_nb, nbid(b_nb), drof(b_nb),
                             b_i, b_j, s, b_j, s, bsz, cf, inv_c1, bcof(b_nb), ga.rb,
                             P0[L(b_jl, b_i == 0 ? 1 : NC)],
                             P0[L(b_jl, b_i == 0 ? 2 : NC - 1)]);
      } else {
        const int l1 = b_j == 0 ? 1 : TJ, l2 = b_j == 0 ? 2 : TJ - 1;
        v = pair_ghost_k<NC>(src, coarse, rhs, meta, m, b_nb, nbid(b_nb), drof(b_nb),
                             b_i, b_j, s, b_i, s, bsz, cf, inv_c1, bcof(b_nb), ga.rb,
                             P0[L(l1, b_i)], P0[L(l2, b_i)]);
      }
      P0[L(b_jl, b_i)] = v;
    }
    if (s == 2 || s == NC + 1) {
      // z ghost plane 0 (NC+1): red cells; x1 = plane 1 (NC), black, old;
      // x2 = plane 2 (NC-1), red, new
      const int nb = s == 2 ? 5 : 6, k = s == 2 ? 0 : NC + 1;
      double *Pg = s == 2 ? Pmm : P0;
      const double *X2 = s == 2 ? P0 : Pmm;
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        int i, j;
        const int c = col(q, k, i, j);
        Pg[c] = pair_ghost_k<NC>(src, coarse, rhs, meta, m, nb, s == 2 ? nb5 : nb6, dr2,
                                 i, j, k, i, j, bsz, cf, inv_c1,
                                 s == 2 ? ga.bc[4] : ga.bc[5], ga.rb, Pm[c], X2[c]);
      }
      __syncthreads();
    }
    // C: black cells of plane s-1, in place
    if (s - 1 >= k0 && s - 1 <= k1) {
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        int i, j;
        const int c = col(q, s, i, j);
        const int cm = L(j - j0 + 1, i - 1), cp = L(j - j0 + 1, i + 1);
        Pm[c] = (rB[q] - cf.c[1] * Pm[cm] - cf.c[2] * Pm[cp] -
                 cf.c[3] * Pm[c - NG] - cf.c[4] * Pm[c + NG] - cf.c[5] * Pmm[c] -
                 cf.c[6] * P0[c]) *
                inv_c1;
      }
    }
    __syncthreads();
    // D: plane s+2 into the slot of plane s-2
    if (s + 2 <= NC + 1 && s + 2 <= k1 + 2) {
#pragma unroll
      for (int e = 0; e < EPT; e++) {
        const int xx = tid + NT * e;
        if (xx < PL) Pmm[perm(xx)] = cn.nx[e];
      }
    }
#pragma unroll
    for (int q = 0; q < RPT; q++) {
      const int j = j0 + (tid + NT * q) / HN;
      const bool odd = (j + s + 1) & 1;  // red cell of plane s+1 is i1 + 1
      rB[q] = rBn[q];
      rR[q] = odd ? cn.nhi[q] : cn.nlo[q];
      rBn[q] = odd ? cn.nlo[q] : cn.nhi[q];
    }
    bc = bn;
    __syncthreads();
  };
  if (DEPTH == 1) {
    for (int s = s0; s <= k1 + 1; s++) step(s, X0, X0);
  } else {
    for (int s = s0; s <= k1 + 1; s += 2) {
      step(s, X1, X0);
      if (s + 1 <= k1 + 1) step(s + 1, X0, X1);
    }
  }
  store_plane(k1, P[k1 & 3]);
}

// Whole-box form of the fused pair for small boxes (NC <= 16): the box, its
// ghost layer included, sits in LDS ((NC+2)^3 doubles, 47 KB at NC = 16), so
// the pair is four phases over the whole box -- A all red cells | B the red
// face ghosts the level fill would produce after the red sweep (same
// arithmetic as k_gsrb_pair2's B: a same-level neighbour's boundary cell
// recomputed from its old values, its loads issued at the start; physical
// and refinement faces through gc_face_nocopy) | C all black cells | the
// whole block stored contiguously -- instead of a plane march of NC+1 steps
// with three barriers each, which leaves small boxes latency-bound. The
// stored ghost cells are rewritten by the level fill after the pair; edge
// and corner ghosts are src's, unchanged by the pair. Bitwise the split
// half-sweeps.
template <int NC>
struct RbBox {
  static constexpr int NG = NC + 2, HN = NC / 2;
  static constexpr int NRED = NC * NC * HN;                  // red cells per box
#ifndef AFH_RBBOX_DIV  // (A/B builds: fewer threads per box, more boxes per CU)
#define AFH_RBBOX_DIV 1
#endif
  static constexpr int NT0 = NRED >= 512 ? 512 : (NRED < 64 ? 64 : NRED);
  static constexpr int NT = NT0 / AFH_RBBOX_DIV >= 64 ? NT0 / AFH_RBBOX_DIV : 64;
  static constexpr int RPT = (NRED + NT - 1) / NT;           // red cells per thread
  static constexpr int NGH = 3 * NC * NC;                    // red face ghosts
  static constexpr int GPT = (NGH + NT - 1) / NT;            // ghosts per thread
};

//
// PUSH: the level fill after the pair is done by the pair itself. The box
// stores its interior, edges and corners, and the face ghosts the fill
// would give: a same-level neighbour's ghost layer facing this box gets this
// box's new boundary cells (copy_from_nb seen from the other side), a
// physical / refinement face of this box its gc_face_nocopy value from the
// new interior and the coarse data. Nobody else writes those cells (each
// face ghost of dst has exactly one writer: the box, or its same-level
// neighbour), and every box of the level is in the launch; so dst ends as
// pair + k_gc_faces would leave it (edges and corners: src's, as without
// corners; k_gc_corners follows when the fill wants them).
//
// VAR (round 5): levels with electrode boxes, whose variable 7-point
// stencils v(7, nc^3) and bc_correction come per box id from vp / bp (null:
// the level's constant stencil). stencil_gsrb_357's variable branch
// (m_af_stencil.f90:836-841, 958-978) on those boxes: rhs + bc_correction,
// the sum over the neighbours divided by c(1), rhs - bc_correction -- the
// red cells with rhs (r + b), the black cells with ((r + b) - b) + b, the
// first half-sweep's round trip; phase B recomputes a variable neighbour's
// red boundary cell with its own stencil the same way. The pair leaves rhs
// alone (a neighbour's workgroup reads it); k_rhs_roundtrip applies the two
// round trips after the launch. Bitwise k_gsrb_v + k_gsrb + fills.
template <int NC, bool PUSH = false, bool VAR = false>
__global__ void __launch_bounds__(RbBox<NC>::NT)
    k_gsrb_pair_box(const double *__restrict__ src, double *__restrict__ dst,
                    const double *__restrict__ rhs, const double *__restrict__ coarse,
                    const afh_box_meta *__restrict__ meta,
                    const int32_t *__restrict__ ids, size_t bsz, Coef cf,
                    double inv_c1, GcArgs ga, const double *const *__restrict__ vp = nullptr,
                    const double *const *__restrict__ bp = nullptr, int pend = 0) {
  using G = RbBox<NC>;
  constexpr int NG = G::NG, HN = G::HN, NT = G::NT, RPT = G::RPT, GPT = G::GPT;
  constexpr int SK = NG * NG, NB = NG * NG * NG;
  __shared__ double P[NB];
  const int tid = threadIdx.x;
  const int id = ids[xcd_swizzle(blockIdx.x, gridDim.x)];
  const afh_box_meta &m = meta[id - 1];
  const int nb1 = m.neighbors[0], nb2 = m.neighbors[1], nb3 = m.neighbors[2],
            nb4 = m.neighbors[3], nb5 = m.neighbors[4], nb6 = m.neighbors[5];
  const double dr0 = m.dr[0], dr1 = m.dr[1], dr2 = m.dr[2];
  auto nbid = [&](int nb) {
    return nb == 1 ? nb1 : nb == 2 ? nb2 : nb == 3 ? nb3 : nb == 4 ? nb4 : nb == 5 ? nb5 : nb6;
  };
  auto bcof = [&](int nb) {
    afh_bc b;
    b.type = nb == 1 ? ga.bc[0].type : nb == 2 ? ga.bc[1].type : nb == 3 ? ga.bc[2].type
           : nb == 4 ? ga.bc[3].type : nb == 5 ? ga.bc[4].type : ga.bc[5].type;
    b.value = nb == 1 ? ga.bc[0].value : nb == 2 ? ga.bc[1].value : nb == 3 ? ga.bc[2].value
            : nb == 4 ? ga.bc[3].value : nb == 5 ? ga.bc[4].value : ga.bc[5].value;
    return b;
  };
  const double *x = src + (size_t)(id - 1) * bsz;
  double *y = dst + (size_t)(id - 1) * bsz;
  const double *r = rhs + (size_t)(id - 1) * bsz;
  // VAR: this box's stencil and correction (null: constant)
  const double *bv = VAR ? vp[id - 1] : nullptr, *bb = VAR ? bp[id - 1] : nullptr;
  // VAR, pend: the rhs round trips of the level's earlier pairs of this leg
  // not yet stored (k_rhs_roundtrip runs once, after the leg's last pair):
  // an electrode box's rhs is read through them, in k_rhs_roundtrip's order
  auto rtp = [&](double v, double c) {
    for (int q = 0; q < pend; q++) v = (v + c) - c;
    return v;
  };

  // red cell q of this thread: row (j, k), i = 2 ih + 1 + ((j + k) & 1);
  // the black cell of the same pair of columns is the other parity
  auto cell = [&](int q, bool red, int &i, int &j, int &k) {
    const int rr = tid + NT * q;
    const int ih = rr % HN, row = rr / HN;
    j = row % NC + 1;
    k = row / NC + 1;
    i = 2 * ih + 1 + (((j + k) & 1) ^ (red ? 0 : 1));
    return rr < G::NRED;
  };
  // face ghost u: face nb = u / (NC^2 / 2) + 1, (a, b) its in-face indices,
  // red parity
  auto ghost = [&](int u, int &nb, int p[3]) {
    const int per = NC * HN;
    nb = u / per + 1;
    const int w = u % per, d = (nb - 1) >> 1;
    const int ta = d == 0 ? 1 : 0, tb = d == 2 ? 1 : 2;
    const int bb = w / HN + 1, ah = w % HN;
    p[d] = ((nb - 1) & 1) ? NC + 1 : 0;
    p[tb] = bb;
    // red: p[0] + p[1] + p[2] odd
    p[ta] = 2 * ah + 1 + ((p[d] + bb) & 1);
  };

  // global loads first: the box image, rhs of the thread's cells, and the
  // neighbour values of the same-level face ghosts
  for (int e = tid; e < NB; e += NT) P[e] = x[e];
  double rR[RPT], rB[RPT];
  // VAR: the red / black cells' stencils (c(1) first, as v stores them)
  double vR[VAR ? RPT : 1][7], vB[VAR ? RPT : 1][7];
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    int i, j, k;
    const bool ok = cell(q, true, i, j, k);
    rR[q] = ok ? r[(size_t)(k * NG + j) * NG + i] : 0.0;
    int i2, j2, k2;
    cell(q, false, i2, j2, k2);
    rB[q] = ok ? r[(size_t)(k2 * NG + j2) * NG + i2] : 0.0;
    if constexpr (VAR) {
      if (ok && bv) {
        const int eR = ((k - 1) * NC + (j - 1)) * NC + (i - 1);
        const int eB = ((k2 - 1) * NC + (j2 - 1)) * NC + (i2 - 1);
#pragma unroll
        for (int s = 0; s < 7; s++) vR[q][s] = bv[7 * eR + s], vB[q][s] = bv[7 * eB + s];
        if (bb) {
          // rhs + bc_correction of the red sweep; the black sweep's after
          // the red sweep's round trip
          rR[q] = rtp(rR[q], bb[eR]) + bb[eR];
          rB[q] = ((rtp(rB[q], bb[eB]) + bb[eB]) - bb[eB]) + bb[eB];
        }
      }
    }
  }
  double bl[GPT][7];
  // VAR: a variable neighbour's stencil at its boundary cell (vn[g][0] = 0:
  // constant) and its rhs + bc_correction in bl[g][6]
  double vn[VAR ? GPT : 1][7];
  int brep[GPT];
  bool bpre[GPT];
#pragma unroll
  for (int g = 0; g < GPT; g++) {
    const int u = tid + NT * g;
    brep[g] = -1;
    bpre[g] = false;
    if constexpr (VAR) vn[g][0] = 0.0;
#pragma unroll
    for (int q = 0; q < 7; q++) bl[g][q] = 0.0;
    if (u < G::NGH) {
      int nb, p[3];
      ghost(u, nb, p);
      const int nid = nbid(nb);
      if (nid > 0) {
        const int d = (nb - 1) >> 1;
        const bool low = ((nb - 1) & 1) == 0;
        int q3[3] = {p[0], p[1], p[2]};
        q3[d] = low ? NC : 1;
        const double *xs = src + (size_t)(nid - 1) * bsz;
        const size_t c = ix3(NG, q3[0], q3[1], q3[2]);
        bpre[g] = true;
        brep[g] = 2 * d + (low ? 1 : 0);
        bl[g][0] = xs[c - 1];
        bl[g][1] = xs[c + 1];
        bl[g][2] = xs[c - NG];
        bl[g][3] = xs[c + NG];
        bl[g][4] = xs[c - SK];
        bl[g][5] = xs[c + SK];
        bl[g][6] = rhs[(size_t)(nid - 1) * bsz + c];
        if constexpr (VAR) {
          vn[g][0] = 0.0;
          const double *nv = vp[nid - 1];
          if (nv) {
            const int en = ((q3[2] - 1) * NC + (q3[1] - 1)) * NC + (q3[0] - 1);
#pragma unroll
            for (int s = 0; s < 7; s++) vn[g][s] = nv[7 * en + s];
            const double *nbc = bp[nid - 1];
            if (nbc) bl[g][6] = rtp(bl[g][6], nbc[en]) + nbc[en];
          }
        }
      }
    }
  }
  __syncthreads();
  // A: red cells
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    int i, j, k;
    if (!cell(q, true, i, j, k)) continue;
    const int c = (k * NG + j) * NG + i;
    if (VAR && bv) {
      const double *v = vR[VAR ? q : 0];
      P[c] = (rR[q] - v[1] * P[c - 1] - v[2] * P[c + 1] - v[3] * P[c - NG] -
              v[4] * P[c + NG] - v[5] * P[c - SK] - v[6] * P[c + SK]) /
             v[0];
    } else {
      P[c] = (rR[q] - cf.c[1] * P[c - 1] - cf.c[2] * P[c + 1] - cf.c[3] * P[c - NG] -
              cf.c[4] * P[c + NG] - cf.c[5] * P[c - SK] - cf.c[6] * P[c + SK]) *
             inv_c1;
    }
  }
  __syncthreads();
  // B: red face ghosts
#pragma unroll
  for (int g = 0; g < GPT; g++) {
    const int u = tid + NT * g;
    if (u >= G::NGH) continue;
    int nb, p[3];
    ghost(u, nb, p);
    const int d = (nb - 1) >> 1;
    const bool low = ((nb - 1) & 1) == 0;
    int q1[3] = {p[0], p[1], p[2]}, q2[3] = {p[0], p[1], p[2]};
    q1[d] = low ? 1 : NC;
    q2[d] = low ? 2 : NC - 1;
    const double x1v = P[ix3(NG, q1[0], q1[1], q1[2])];  // black, old
    double v;
    if (bpre[g]) {
      double b[7];
#pragma unroll
      for (int q = 0; q < 7; q++) b[q] = bl[g][q];
#pragma unroll
      for (int q = 0; q < 6; q++)
        if (q == brep[g]) b[q] = x1v;
      if (VAR && vn[VAR ? g : 0][0] != 0.0) {
        const double *w = vn[VAR ? g : 0];
        v = (b[6] - w[1] * b[0] - w[2] * b[1] - w[3] * b[2] - w[4] * b[3] - w[5] * b[4] -
             w[6] * b[5]) /
            w[0];
      } else {
        v = (b[6] - cf.c[1] * b[0] - cf.c[2] * b[1] - cf.c[3] * b[2] - cf.c[4] * b[3] -
             cf.c[5] * b[4] - cf.c[6] * b[5]) *
            inv_c1;
      }
    } else {
      const double x2v = P[ix3(NG, q2[0], q2[1], q2[2])];  // red, new
      const int ta = d == 0 ? 1 : 0, tb = d == 2 ? 1 : 2;
      v = pair_ghost_k<NC>(src, coarse, rhs, meta, m, nb, nbid(nb),
                           d == 0 ? dr0 : d == 1 ? dr1 : dr2, p[0], p[1], p[2], p[ta],
                           p[tb], bsz, cf, inv_c1, bcof(nb), ga.rb, x1v, x2v);
    }
    P[ix3(NG, p[0], p[1], p[2])] = v;
  }
  __syncthreads();
  // C: black cells
#pragma unroll
  for (int q = 0; q < RPT; q++) {
    int i, j, k;
    if (!cell(q, false, i, j, k)) continue;
    const int c = (k * NG + j) * NG + i;
    if (VAR && bv) {
      const double *v = vB[VAR ? q : 0];
      P[c] = (rB[q] - v[1] * P[c - 1] - v[2] * P[c + 1] - v[3] * P[c - NG] -
              v[4] * P[c + NG] - v[5] * P[c - SK] - v[6] * P[c + SK]) /
             v[0];
    } else {
      P[c] = (rB[q] - cf.c[1] * P[c - 1] - cf.c[2] * P[c + 1] - cf.c[3] * P[c - NG] -
              cf.c[4] * P[c + NG] - cf.c[5] * P[c - SK] - cf.c[6] * P[c + SK]) *
             inv_c1;
    }
  }
  __syncthreads();
  if constexpr (!PUSH) {
    for (int e = tid; e < NB; e += NT) y[e] = P[e];
  } else {
    // interior, edges and corners (not the six face ghost layers)
    for (int e = tid; e < NB; e += NT) {
      const int i = e % NG, j = (e / NG) % NG, k = e / SK;
      const int nout = (i == 0 || i == NG - 1) + (j == 0 || j == NG - 1) + (k == 0 || k == NG - 1);
      if (nout != 1) y[e] = P[e];
    }
    // face ghosts: pushed into the same-level neighbour, or this box's own
    for (int u = tid; u < 6 * NC * NC; u += NT) {
      const int nb = u / (NC * NC) + 1, w = u % (NC * NC);
      const int a = w % NC + 1, b = w / NC + 1;
      const int d = (nb - 1) >> 1;
      const bool low = ((nb - 1) & 1) == 0;
      const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
      int p[3];
      p[ta] = a;
      p[tb] = b;
      p[d] = low ? 0 : NC + 1;
      int q1[3] = {p[0], p[1], p[2]};
      q1[d] = low ? 1 : NC;
      const double x1v = P[ix3(NG, q1[0], q1[1], q1[2])];
      const int nid = nbid(nb);
      if (nid > 0) {
        int q[3] = {p[0], p[1], p[2]};
        q[d] = low ? NC + 1 : 0;  // the neighbour's ghost facing this box
        dst[(size_t)(nid - 1) * bsz + ix3(NG, q[0], q[1], q[2])] = x1v;
      } else {
        y[ix3(NG, p[0], p[1], p[2])] = gc_face_nocopy_k(
            coarse, meta, m, nb, nid, d == 0 ? dr0 : d == 1 ? dr1 : dr2, p, a, b, NC, bsz,
            bcof(nb), ga.rb, [&](const int *q) { return P[ix3(NG, q[0], q[1], q[2])]; });
      }
    }
  }
}

// correct_children's prolongation (stencil_prolong_248 add, k_prolong's
// expressions) for a small box in one workgroup, followed by the face fill
// the level's ghost fill would do, pushed like k_gsrb_pair_box<PUSH>: a
// same-level neighbour's ghost layer facing this box gets the corrected
// boundary cells, a physical / refinement face of this box its
// gc_face_nocopy value from the corrected interior and the coarse data.
// Edges and corners are left as they were: the up leg's pairs do not read
// them, and its last pair is followed by k_gc_corners. Replaces k_prolong +
// k_gc_box on levels smoothed by pushing pairs (one launch instead of two;
// the fill no longer re-reads the box). Same values.
template <int NC>
__global__ void __launch_bounds__(RbBox<NC>::NT)
    k_prolong_box(double *__restrict__ phi, const double *__restrict__ tmp,
                  const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids,
                  size_t bsz, GcArgs ga) {
  constexpr int NG = NC + 2, NT = RbBox<NC>::NT, HN = NC / 2;
  __shared__ double P[NG * NG * NG];
  const int tid = threadIdx.x;
  const int id = ids[xcd_swizzle(blockIdx.x, gridDim.x)];
  const afh_box_meta &m = meta[id - 1];
  double *y = phi + (size_t)(id - 1) * bsz;
  const double *pp = tmp + (size_t)(m.parent - 1) * bsz;
  const int o0 = ((m.ix[0] - 1) & 1) * HN, o1 = ((m.ix[1] - 1) & 1) * HN,
            o2 = ((m.ix[2] - 1) & 1) * HN;
  for (int e = tid; e < NC * NC * NC; e += NT) {
    const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
    const int i1 = o0 + ((i + 1) >> 1), i2 = i1 + 1 - 2 * (i & 1);
    const int j1 = o1 + ((j + 1) >> 1), j2 = j1 + 1 - 2 * (j & 1);
    const int k1 = o2 + ((k + 1) >> 1), k2 = k1 + 1 - 2 * (k & 1);
    const int c = ix3(NG, i, j, k);
    const double *a = pp + ix3(NG, 0, 0, k1), *b = pp + ix3(NG, 0, 0, k2);
    const double v = y[c] + (27 / 64.0) * a[j1 * NG + i1] + (9 / 64.0) * a[j1 * NG + i2] +
                     (9 / 64.0) * a[j2 * NG + i1] + (3 / 64.0) * a[j2 * NG + i2] +
                     (9 / 64.0) * b[j1 * NG + i1] + (3 / 64.0) * b[j1 * NG + i2] +
                     (3 / 64.0) * b[j2 * NG + i1] + (1 / 64.0) * b[j2 * NG + i2];
    P[c] = v;
    y[c] = v;
  }
  __syncthreads();
  for (int u = tid; u < 6 * NC * NC; u += NT) {
    const int nb = u / (NC * NC) + 1, w = u % (NC * NC);
    const int a = w % NC + 1, b = w / NC + 1;
    const int d = (nb - 1) >> 1;
    const bool low = ((nb - 1) & 1) == 0;
    const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
    int p[3];
    p[ta] = a;
    p[tb] = b;
    p[d] = low ? 0 : NC + 1;
    const int nid = m.neighbors[nb - 1];
    if (nid > 0) {
      int q1[3] = {p[0], p[1], p[2]}, q[3] = {p[0], p[1], p[2]};
      q1[d] = low ? 1 : NC;
      q[d] = low ? NC + 1 : 0;  // the neighbour's ghost facing this box
      phi[(size_t)(nid - 1) * bsz + ix3(NG, q[0], q[1], q[2])] = P[ix3(NG, q1[0], q1[1], q1[2])];
    } else {
      y[ix3(NG, p[0], p[1], p[2])] = gc_face_nocopy_k(
          phi, meta, m, nb, nid, m.dr[d], p, a, b, NC, bsz, ga.bc[nb - 1], ga.rb,
          [&](const int *q) { return P[ix3(NG, q[0], q[1], q[2])]; });
    }
  }
}

__device__ __forceinline__ double apply7(const double *x, size_t c, size_t sj, size_t sk,
                                         const Coef &cf);

// update_coarse's restriction (k_rstr_fas's expressions) of one small fine
// box into its octant of the parent, followed by the parent's face ghosts
// that octant determines, pushed like k_prolong_box: the parent's
// same-level neighbour's ghost layer facing it gets the new boundary values,
// a physical / refinement face of the parent its gc_face_nocopy value (from
// x1, x2 of the octant and the coarser level's data, which this launch does
// not change). Each octant covers three of the parent's faces; every face
// ghost the level fill would rewrite after the restriction has exactly one
// writer. Ghosts facing unchanged boxes keep their values: only valid when
// the level's ghosts were filled since phi last changed (the caller checks).
template <int NC>
__global__ void __launch_bounds__(NC >= 16 ? 512 : 64)
    k_rstr_box(double *__restrict__ phi, const double *__restrict__ rhs,
               double *__restrict__ tmp, const afh_box_meta *__restrict__ meta,
               const int32_t *__restrict__ ids, size_t bsz, Coef cf, GcArgs ga) {
  constexpr int NG = NC + 2, HN = NC / 2, NT = NC >= 16 ? 512 : 64;
  constexpr int SJ = NG, SK = NG * NG;
  __shared__ double Q[HN * HN * HN];
  const int tid = threadIdx.x;
  const int id = ids[xcd_swizzle(blockIdx.x, gridDim.x)];
  const afh_box_meta &m = meta[id - 1];
  const afh_box_meta &pm = meta[m.parent - 1];
  const double *x = phi + (size_t)(id - 1) * bsz, *r = rhs + (size_t)(id - 1) * bsz;
  const int o[3] = {((m.ix[0] - 1) & 1) * HN, ((m.ix[1] - 1) & 1) * HN,
                    ((m.ix[2] - 1) & 1) * HN};
  const size_t pb = (size_t)(m.parent - 1) * bsz;
  for (int e = tid; e < HN * HN * HN; e += NT) {
    const int i = e % HN + 1, j = (e / HN) % HN + 1, k = e / (HN * HN) + 1;
    const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
    const size_t cs[8] = {ix3(NG, fi, fj, fk),         ix3(NG, fi + 1, fj, fk),
                          ix3(NG, fi, fj + 1, fk),     ix3(NG, fi + 1, fj + 1, fk),
                          ix3(NG, fi, fj, fk + 1),     ix3(NG, fi + 1, fj, fk + 1),
                          ix3(NG, fi, fj + 1, fk + 1), ix3(NG, fi + 1, fj + 1, fk + 1)};
    double sr = r[cs[0]] - apply7(x, cs[0], SJ, SK, cf);
    double sp = x[cs[0]];
#pragma unroll
    for (int q = 1; q < 8; q++) {
      sr += r[cs[q]] - apply7(x, cs[q], SJ, SK, cf);
      sp += x[cs[q]];
    }
    const size_t po = pb + ix3(NG, o[0] + i, o[1] + j, o[2] + k);
    tmp[po] = 0.125 * sr;
    phi[po] = 0.125 * sp;
    Q[e] = 0.125 * sp;
  }
  __syncthreads();
  auto own = [&](const int *q) {
    return Q[((q[2] - o[2] - 1) * HN + (q[1] - o[1] - 1)) * HN + (q[0] - o[0] - 1)];
  };
  for (int u = tid; u < 3 * HN * HN; u += NT) {
    const int d = u / (HN * HN), w = u % (HN * HN);
    const bool low = o[d] == 0;
    const int nb = 2 * d + (low ? 1 : 2);
    const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
    int p[3];
    p[ta] = o[ta] + w % HN + 1;
    p[tb] = o[tb] + w / HN + 1;
    p[d] = low ? 0 : NC + 1;
    const int nid = pm.neighbors[nb - 1];
    if (nid > 0) {
      int q1[3] = {p[0], p[1], p[2]}, q[3] = {p[0], p[1], p[2]};
      q1[d] = low ? 1 : NC;
      q[d] = low ? NC + 1 : 0;  // the neighbour's ghost facing the parent
      phi[(size_t)(nid - 1) * bsz + ix3(NG, q[0], q[1], q[2])] = own(q1);
    } else {
      phi[pb + ix3(NG, p[0], p[1], p[2])] =
          gc_face_nocopy_k(phi, meta, pm, nb, nid, pm.dr[d], p, p[ta], p[tb], NC, bsz,
                           ga.bc[nb - 1], ga.rb, own);
    }
  }
}

// the edges and corners of a box from its face ghosts and its diagonal
// neighbours (k_gc_corners' loops, for the calling workgroup's box; the
// edge table arithmetically: edge n runs along n / 4, its sign bits r = n % 4
// over the two other dimensions in increasing order)
__device__ __forceinline__ void box_edges_corners(double *__restrict__ v,
                                                  const afh_box_meta &m, int id, int nc,
                                                  size_t bsz, int tid, int nt) {
  const int ng = nc + 2;
  double *c = v + (size_t)(id - 1) * bsz;
  for (int e = tid; e < 12 * nc; e += nt) {
    const int n = e / nc, pos = e % nc + 1;
    const int dim = n >> 2, r = n & 3;
    const int oa = dim == 0 ? 1 : 0, ob = dim == 2 ? 1 : 2;
    int dir[3] = {0, 0, 0}, x[3];
    dir[oa] = (r & 1) ? 1 : -1;
    dir[ob] = (r & 2) ? 1 : -1;
    x[dim] = pos;
    x[oa] = (r & 1) ? nc + 1 : 0;
    x[ob] = (r & 2) ? nc + 1 : 0;
    const int nb_id = m.neighbor_mat[(dir[0] + 1) + 3 * (dir[1] + 1) + 9 * (dir[2] + 1)];
    if (nb_id > 0) {
      c[ix3(ng, x[0], x[1], x[2])] =
          v[(size_t)(nb_id - 1) * bsz +
            ix3(ng, x[0] - dir[0] * nc, x[1] - dir[1] * nc, x[2] - dir[2] * nc)];
    } else {
      const int o1 = (dim + 1) % 3, o2 = (dim + 2) % 3;
      int di[3];
      for (int q = 0; q < 3; q++) di[q] = 1 - 2 * (x[q] & 1);
      di[dim] = 0;
      int ia[3] = {x[0], x[1], x[2]}, ib[3] = {x[0], x[1], x[2]};
      ia[o1] += di[o1];
      ib[o2] += di[o2];
      c[ix3(ng, x[0], x[1], x[2])] = c[ix3(ng, ia[0], ia[1], ia[2])] +
                                     c[ix3(ng, ib[0], ib[1], ib[2])] -
                                     c[ix3(ng, x[0] + di[0], x[1] + di[1], x[2] + di[2])];
    }
  }
  __syncthreads();
  if (tid < 8) {
    int dnb[3], x[3];
    for (int q = 0; q < 3; q++) {
      const int b = (tid >> q) & 1;
      dnb[q] = 2 * b - 1;
      x[q] = b * (nc + 1);
    }
    const int nb_id = m.neighbor_mat[(dnb[0] + 1) + 3 * (dnb[1] + 1) + 9 * (dnb[2] + 1)];
    if (nb_id > 0) {
      c[ix3(ng, x[0], x[1], x[2])] =
          v[(size_t)(nb_id - 1) * bsz +
            ix3(ng, x[0] - dnb[0] * nc, x[1] - dnb[1] * nc, x[2] - dnb[2] * nc)];
    } else {
      int di[3];
      for (int q = 0; q < 3; q++) di[q] = 1 - 2 * (x[q] & 1);
      c[ix3(ng, x[0], x[1], x[2])] = c[ix3(ng, x[0], x[1] + di[1], x[2] + di[2])] +
                                     c[ix3(ng, x[0] + di[0], x[1], x[2] + di[2])] +
                                     c[ix3(ng, x[0] + di[0], x[1] + di[1], x[2])] -
                                     2 * c[ix3(ng, x[0] + di[0], x[1] + di[1], x[2] + di[2])];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ double apply7(const double *x, size_t c, size_t sj,
                                         size_t sk, const Coef &cf) {
  return cf.c[0] * x[c] + cf.c[1] * x[c - 1] + cf.c[2] * x[c + 1] +
         cf.c[3] * x[c - sj] + cf.c[4] * x[c + sj] + cf.c[5] * x[c - sk] +
         cf.c[6] * x[c + sk];
}

// residual_box; with MAX (leaf boxes) the max |residual| is folded into
// shard slots (af_tree_maxabs_cc(i_tmp) of field_compute). Each thread
// takes a column of K cells along k: the z neighbours are shared and all
// loads are issued before the arithmetic (more bytes in flight per wave).
// GRAD (afh_mg_set_gradient_output): the same phi values also give |E| of
// field_from_potential's gradient (k_gradient_t's expressions, fac / dr of
// the box), stored in nrm -- one read of phi for both.
template <bool MAX, int K, bool GRAD = false>
__global__ void __launch_bounds__(256)
    k_residual(const double *__restrict__ phi, const double *__restrict__ rhs,
               double *__restrict__ tmp, const int32_t *__restrict__ ids,
               int nc, size_t bsz, Coef cf0, unsigned long long *red,
               const Coef *__restrict__ cft = nullptr,
               const afh_box_meta *__restrict__ meta = nullptr,
               double *__restrict__ nrm = nullptr, double gfac = 0.0) {
  // cft: boxes of several levels, the level's coefficients from the table
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double mx = 0.0;
  if (t < nc * nc * (nc / K)) {
    const int id = ids[blockIdx.y];
    const Coef cf = cft ? cft[meta[id - 1].lvl - 1] : cf0;
    int i, j, kq;
    cell3(t, nc, i, j, kq);
    const int ng = nc + 2;
    const size_t sj = ng, sk = (size_t)ng * ng;
    const size_t o = (size_t)(id - 1) * bsz, c0 = ix3(ng, i, j, (kq - 1) * K + 1);
    const double *x = phi + o;
    double z[K + 2], xm[K], xp[K], ym[K], yp[K], r[K];
#pragma unroll
    for (int q = 0; q < K + 2; q++) z[q] = x[c0 + (q - 1) * sk];
#pragma unroll
    for (int q = 0; q < K; q++) {
      const size_t c = c0 + q * sk;
      xm[q] = x[c - 1];
      xp[q] = x[c + 1];
      ym[q] = x[c - sj];
      yp[q] = x[c + sj];
      r[q] = rhs[o + c];
    }
#pragma unroll
    for (int q = 0; q < K; q++) {
      // apply7 operand order
      const double a = cf.c[0] * z[q + 1] + cf.c[1] * xm[q] + cf.c[2] * xp[q] +
                       cf.c[3] * ym[q] + cf.c[4] * yp[q] + cf.c[5] * z[q] +
                       cf.c[6] * z[q + 2];
      const double v = r[q] - a;
      st_nt<AFH_NT_MG>(tmp + (o + c0 + q * sk), v);
      mx = fmax(mx, fabs(v));
    }
    if constexpr (GRAD) {
      const afh_box_meta &mb = meta[id - 1];
      const double gx = gfac / mb.dr[0], gy = gfac / mb.dr[1], gz = gfac / mb.dr[2];
#pragma unroll
      for (int q = 0; q < K; q++) {
        const double pv = z[q + 1];
        const double fxl = gx * (pv - xm[q]), fxh = gx * (xp[q] - pv);
        const double fyl = gy * (pv - ym[q]), fyh = gy * (yp[q] - pv);
        const double fzl = gz * (pv - z[q]), fzh = gz * (z[q + 2] - pv);
        const double a = fxl + fxh, b = fyl + fyh, c = fzl + fzh;
        st_nt<AFH_NT_MG>(nrm + (o + c0 + q * sk), 0.5 * sqrt(a * a + b * b + c * c));
      }
    }
  }
  if (MAX) block_max_to_shard(mx, red);
}

__global__ void k_rstr_fas(double *__restrict__ phi,
                           const double *__restrict__ rhs,
                           double *__restrict__ tmp,
                           const afh_box_meta *__restrict__ meta,
                           const int32_t *__restrict__ ids, int nc, size_t bsz,
                           Coef cf) {
  const int hn = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hn * hn * hn) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  int i, j, k;
  cell3(t, hn, i, j, k);
  const int ng = nc + 2;
  const size_t sj = ng, sk = (size_t)ng * ng;
  const size_t o = (size_t)(id - 1) * bsz;
  const double *x = phi + o, *r = rhs + o;
  const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
  size_t cs[8] = {ix3(ng, fi, fj, fk),         ix3(ng, fi + 1, fj, fk),
                  ix3(ng, fi, fj + 1, fk),     ix3(ng, fi + 1, fj + 1, fk),
                  ix3(ng, fi, fj, fk + 1),     ix3(ng, fi + 1, fj, fk + 1),
                  ix3(ng, fi, fj + 1, fk + 1), ix3(ng, fi + 1, fj + 1, fk + 1)};
  double sr = r[cs[0]] - apply7(x, cs[0], sj, sk, cf);
  double sp = x[cs[0]];
#pragma unroll
  for (int q = 1; q < 8; q++) {
    sr += r[cs[q]] - apply7(x, cs[q], sj, sk, cf);
    sp += x[cs[q]];
  }
  const size_t po = (size_t)(m.parent - 1) * bsz +
                    ix3(ng, ((m.ix[0] - 1) & 1) * hn + i,
                        ((m.ix[1] - 1) & 1) * hn + j,
                        ((m.ix[2] - 1) & 1) * hn + k);
  tmp[po] = 0.125 * sr;
  phi[po] = 0.125 * sp;
}

// k_rstr_fas with each thread marching a column of K coarse cells (2K fine
// planes) along k: the 2x2 fine centre values of each plane are loaded once
// and serve as the z neighbours of the planes above and below (the one-cell
// form re-read the fine planes around every coarse plane from other blocks,
// 1.67x the algorithmic bytes in the PMC counters). Same operand order as
// k_rstr_fas / apply7: bitwise the same parent values.
template <int K>
__global__ void __launch_bounds__(256)
    k_rstr_fas_col(double *__restrict__ phi, const double *__restrict__ rhs,
                   double *__restrict__ tmp, const afh_box_meta *__restrict__ meta,
                   const int32_t *__restrict__ ids, int nc, size_t bsz, Coef cf,
                   const double *__restrict__ fine) {
  const int hn = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hn * hn * (hn / K)) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  int i, j, kq;
  cell3(t, hn, i, j, kq);
  const int k0 = (kq - 1) * K + 1;  // first coarse plane of the column
  const int ng = nc + 2;
  const size_t sj = ng;
  const size_t o = (size_t)(id - 1) * bsz;
  const double *x = fine + o, *r = rhs + o;  // (fine: phi, or its image in alt)
  const int fi = 2 * i - 1, fj = 2 * j - 1, f0 = 2 * k0 - 1;
  // centre values c[p][a + 2 b] of fine plane f0 - 1 + p at (fi + a, fj + b)
  double c[2 * K + 2][4];
#pragma unroll
  for (int p = 0; p < 2 * K + 2; p++) {
    const size_t b = ix3(ng, fi, fj, f0 - 1 + p);
    c[p][0] = x[b];
    c[p][1] = x[b + 1];
    c[p][2] = x[b + sj];
    c[p][3] = x[b + sj + 1];
  }
  const size_t pb = (size_t)(m.parent - 1) * bsz;
  const int pi = ((m.ix[0] - 1) & 1) * hn + i, pj = ((m.ix[1] - 1) & 1) * hn + j,
            pk = ((m.ix[2] - 1) & 1) * hn;
#pragma unroll
  for (int q = 0; q < K; q++) {
    double sr = 0.0, sp = 0.0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int p = 2 * q + 1 + h;  // fine plane f0 - 1 + p
      const size_t b = ix3(ng, fi, fj, f0 - 1 + p);
      // x neighbours (fi - 1, fi + 2) and y neighbours (fj - 1, fj + 2)
      const double xm0 = x[b - 1], xp0 = x[b + 2];
      const double xm1 = x[b + sj - 1], xp1 = x[b + sj + 2];
      const double ym0 = x[b - sj], ym1 = x[b - sj + 1];
      const double yp0 = x[b + 2 * sj], yp1 = x[b + 2 * sj + 1];
      const double r0 = r[b], r1 = r[b + 1], r2 = r[b + sj], r3 = r[b + sj + 1];
      const double *z = c[p], *zm = c[p - 1], *zp = c[p + 1];
      // cells (fi, fj), (fi+1, fj), (fi, fj+1), (fi+1, fj+1) of this plane
      const double a0 = cf.c[0] * z[0] + cf.c[1] * xm0 + cf.c[2] * z[1] + cf.c[3] * ym0 +
                        cf.c[4] * z[2] + cf.c[5] * zm[0] + cf.c[6] * zp[0];
      const double a1 = cf.c[0] * z[1] + cf.c[1] * z[0] + cf.c[2] * xp0 + cf.c[3] * ym1 +
                        cf.c[4] * z[3] + cf.c[5] * zm[1] + cf.c[6] * zp[1];
      const double a2 = cf.c[0] * z[2] + cf.c[1] * xm1 + cf.c[2] * z[3] + cf.c[3] * z[0] +
                        cf.c[4] * yp0 + cf.c[5] * zm[2] + cf.c[6] * zp[2];
      const double a3 = cf.c[0] * z[3] + cf.c[1] * z[2] + cf.c[2] * xp1 + cf.c[3] * z[1] +
                        cf.c[4] * yp1 + cf.c[5] * zm[3] + cf.c[6] * zp[3];
      if (h == 0) {
        sr = r0 - a0;
        sp = z[0];
      } else {
        sr += r0 - a0;
        sp += z[0];
      }
      sr += r1 - a1;
      sp += z[1];
      sr += r2 - a2;
      sp += z[2];
      sr += r3 - a3;
      sp += z[3];
    }
    const size_t po = pb + ix3(ng, pi, pj, pk + k0 + q);
    tmp[po] = 0.125 * sr;
    phi[po] = 0.125 * sp;
  }
}

__global__ void k_parent_rhs(const double *__restrict__ phi,
                             double *__restrict__ rhs, double *__restrict__ tmp,
                             const int32_t *__restrict__ ids, int nc,
                             size_t bsz, Coef cf) {
  const int ng = nc + 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ng * ng * ng) return;
  const int id = ids[blockIdx.y];
  int i, j, k;
  cell3g(t, ng, i, j, k);
  const size_t o = (size_t)(id - 1) * bsz, c = ix3(ng, i, j, k);
  // (the old rhs is read on the ghost layer only: 8 B per interior cell less)
  const double rv = (i >= 1 && i <= nc && j >= 1 && j <= nc && k >= 1 && k <= nc)
                        ? apply7(phi + o, c, ng, (size_t)ng * ng, cf)
                        : rhs[o + c];
  rhs[o + c] = rv + tmp[o + c];
  tmp[o + c] = phi[o + c];
}

// After k_rstr_box (faces pushed): a parent box's edges and corners, then
// its k_parent_rhs, in one workgroup per parent. The level's leaves keep
// their edges and corners until the up leg's k_gc_corners: nothing reads
// them before (the 7-point operators, the restriction and the pushing pairs
// read faces only; the prolongation reads parents' edges, set here).
template <int NT>
__global__ void __launch_bounds__(NT)
    k_parent_rhs_box(double *__restrict__ phi, double *__restrict__ rhs,
                     double *__restrict__ tmp, const afh_box_meta *__restrict__ meta,
                     const int32_t *__restrict__ ids, int nc, size_t bsz, Coef cf) {
  const int id = ids[xcd_swizzle(blockIdx.x, gridDim.x)];
  box_edges_corners(phi, meta[id - 1], id, nc, bsz, threadIdx.x, NT);
  const int ng = nc + 2;
  const size_t o = (size_t)(id - 1) * bsz;
  for (int t = threadIdx.x; t < ng * ng * ng; t += NT) {
    int i, j, k;
    cell3g(t, ng, i, j, k);
    const size_t c = ix3(ng, i, j, k);
    const double rv = (i >= 1 && i <= nc && j >= 1 && j <= nc && k >= 1 && k <= nc)
                          ? apply7(phi + o, c, ng, (size_t)ng * ng, cf)
                          : rhs[o + c];
    rhs[o + c] = rv + tmp[o + c];
    tmp[o + c] = phi[o + c];
  }
}

// ------------------------------------------------------------ electrode boxes
// Boxes the electrode surface crosses carry a variable 7-point stencil
// (mg_box_lsf_stencil, m_af_multigrid.f90:1762-1834): v(7, nc^3),
// coefficients fastest as afivo stores them, and bc_correction(nc^3) (f times
// the electrode potential, mg_set_operators_lvl 1156-1160); vp / bp index
// them by box id (bp null: no correction). These kernels run on the lists of
// such boxes only (one thread per cell; the boxes are few), the constant
// kernels on the rest of each level.
__device__ __forceinline__ double apply7v(const double *x, size_t c, size_t sj,
                                          size_t sk, const double *v) {
  return v[0] * x[c] + v[1] * x[c - 1] + v[2] * x[c + 1] + v[3] * x[c - sj] +
         v[4] * x[c + sj] + v[5] * x[c - sk] + v[6] * x[c + sk];
}

// stencil_gsrb_357, variable branch (m_af_stencil.f90:836-841, 958-978):
// rhs + bc_correction on every cell, the (i+j+k+redblack) even cells
// divided by c(1), rhs - bc_correction
__global__ void k_gsrb_v(double *__restrict__ phi, double *__restrict__ rhs,
                         const int32_t *__restrict__ ids, int nc, size_t bsz,
                         const double *const *__restrict__ vp,
                         const double *const *__restrict__ bp, int redblack) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  const int id = ids[blockIdx.y];
  int i, j, k;
  cell3(t, nc, i, j, k);
  const int ng = nc + 2;
  const size_t sj = ng, sk = (size_t)ng * ng, c = ix3(ng, i, j, k);
  double *x = phi + (size_t)(id - 1) * bsz, *r = rhs + (size_t)(id - 1) * bsz;
  const double *v = vp[id - 1] + 7 * (size_t)t, *b = bp[id - 1];
  double r1 = r[c];
  if (b) r1 = r1 + b[t];
  if (((i + j + k + redblack) & 1) == 0)
    x[c] = (r1 - v[1] * x[c - 1] - v[2] * x[c + 1] - v[3] * x[c - sj] -
            v[4] * x[c + sj] - v[5] * x[c - sk] - v[6] * x[c + sk]) /
           v[0];
  if (b) r[c] = r1 - b[t];
}

// The rhs round trips (rhs + bc_correction - bc_correction) of the n
// half-sweeps a fused variable pair did (k_gsrb_pair_box<.., VAR>), in the
// order k_gsrb_v applies them
__global__ void k_rhs_roundtrip(double *__restrict__ rhs, const int32_t *__restrict__ ids,
                                int nc, size_t bsz, const double *const *__restrict__ bp,
                                int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  const int id = ids[blockIdx.y];
  const double *b = bp[id - 1];
  if (!b) return;
  int i, j, k;
  cell3(t, nc, i, j, k);
  double *r = rhs + (size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k);
  double v = *r;
  for (int q = 0; q < n; q++) v = (v + b[t]) - b[t];
  *r = v;
}

// residual_box with the variable stencil: tmp = rhs - (L phi - bc_correction)
template <bool MAX>
__global__ void k_residual_v(const double *__restrict__ phi,
                             const double *__restrict__ rhs,
                             double *__restrict__ tmp,
                             const int32_t *__restrict__ ids, int nc, size_t bsz,
                             const double *const *__restrict__ vp,
                             const double *const *__restrict__ bp,
                             unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double mx = 0.0;
  if (t < nc * nc * nc) {
    const int id = ids[blockIdx.y];
    int i, j, k;
    cell3(t, nc, i, j, k);
    const int ng = nc + 2;
    const size_t o = (size_t)(id - 1) * bsz, c = ix3(ng, i, j, k);
    double a = apply7v(phi + o, c, ng, (size_t)ng * ng, vp[id - 1] + 7 * (size_t)t);
    if (bp[id - 1]) a = a - bp[id - 1][t];
    const double v = rhs[o + c] - a;
    tmp[o + c] = v;
    mx = fmax(mx, fabs(v));
  }
  if (MAX) block_max_to_shard(mx, red);
}

// k_rstr_fas for children with a variable stencil
__global__ void k_rstr_fas_v(double *__restrict__ phi,
                             const double *__restrict__ rhs,
                             double *__restrict__ tmp,
                             const afh_box_meta *__restrict__ meta,
                             const int32_t *__restrict__ ids, int nc, size_t bsz,
                             const double *const *__restrict__ vp,
                             const double *const *__restrict__ bp) {
  const int hn = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hn * hn * hn) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  int i, j, k;
  cell3(t, hn, i, j, k);
  const int ng = nc + 2;
  const size_t sj = ng, sk = (size_t)ng * ng;
  const size_t o = (size_t)(id - 1) * bsz;
  const double *x = phi + o, *r = rhs + o, *v = vp[id - 1], *b = bp[id - 1];
  const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
  double sr = 0.0, sp = 0.0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int ci = fi + (q & 1), cj = fj + ((q >> 1) & 1), ck = fk + (q >> 2);
    const size_t c = ix3(ng, ci, cj, ck);
    const size_t cv = ((size_t)(ck - 1) * nc + (cj - 1)) * nc + (ci - 1);
    double a = apply7v(x, c, sj, sk, v + 7 * cv);
    if (b) a = a - b[cv];
    const double res = r[c] - a;
    if (q == 0) {
      sr = res;
      sp = x[c];
    } else {
      sr += res;
      sp += x[c];
    }
  }
  const size_t po = (size_t)(m.parent - 1) * bsz +
                    ix3(ng, ((m.ix[0] - 1) & 1) * hn + i,
                        ((m.ix[1] - 1) & 1) * hn + j,
                        ((m.ix[2] - 1) & 1) * hn + k);
  tmp[po] = 0.125 * sr;
  phi[po] = 0.125 * sp;
}

// k_parent_rhs for parents with a variable stencil
__global__ void k_parent_rhs_v(const double *__restrict__ phi,
                               double *__restrict__ rhs, double *__restrict__ tmp,
                               const int32_t *__restrict__ ids, int nc, size_t bsz,
                               const double *const *__restrict__ vp,
                               const double *const *__restrict__ bp) {
  const int ng = nc + 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ng * ng * ng) return;
  const int id = ids[blockIdx.y];
  int i, j, k;
  cell3g(t, ng, i, j, k);
  const size_t o = (size_t)(id - 1) * bsz, c = ix3(ng, i, j, k);
  double rv = rhs[o + c];
  if (i >= 1 && i <= nc && j >= 1 && j <= nc && k >= 1 && k <= nc) {
    const size_t cv = ((size_t)(k - 1) * nc + (j - 1)) * nc + (i - 1);
    rv = apply7v(phi + o, c, ng, (size_t)ng * ng, vp[id - 1] + 7 * cv);
    if (bp[id - 1]) rv = rv - bp[id - 1][cv];
  }
  rhs[o + c] = rv + tmp[o + c];
  tmp[o + c] = phi[o + c];
}

// Level-1 electrode solve: copy of phi (compact, one slot per level-1 box),
// and max |phi - old|, max |phi| over the interiors (slots 0 and 1)
__global__ void k_copy_compact(const double *__restrict__ phi,
                               double *__restrict__ old,
                               const int32_t *__restrict__ ids, size_t bsz) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bsz) return;
  old[(size_t)blockIdx.y * bsz + t] = phi[(size_t)(ids[blockIdx.y] - 1) * bsz + t];
}

__global__ void k_change_max(const double *__restrict__ phi,
                             const double *__restrict__ old,
                             const int32_t *__restrict__ ids, int nc, size_t bsz,
                             unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double d = 0.0, m = 0.0;
  if (t < nc * nc * nc) {
    int i, j, k;
    cell3(t, nc, i, j, k);
    const size_t c = ix3(nc + 2, i, j, k);
    const double p = phi[(size_t)(ids[blockIdx.y] - 1) * bsz + c];
    d = fabs(p - old[(size_t)blockIdx.y * bsz + c]);
    m = fabs(p);
  }
  block_max_to_shard(d, red);
  __syncthreads();
  block_max_to_shard(m, red + RED_SHARDS);
}

// mg_box_lpllsf_gradient (m_af_multigrid.f90:2030-2120) on electrode leaf
// boxes: the faces next to the boundary from the electrode potential, in the
// order of the distance list (one thread per box: entries may share a face)
__global__ void k_lsf_gradient(const double *__restrict__ phi,
                               const double *__restrict__ lsf,
                               double *__restrict__ fcv,
                               const int32_t *__restrict__ ids, int nc, size_t bsz,
                               size_t fsz, const int *__restrict__ cnt,
                               const int32_t *const *__restrict__ ixp,
                               const double *const *__restrict__ ddp,
                               const double *const *__restrict__ bvp, double ix_,
                               double iy, double iz) {
  if (threadIdx.x != 0) return;
  const int id = ids[blockIdx.x];
  const int n = cnt[id - 1];
  const int ng = nc + 2, nf = nc + 1;
  const size_t d3 = (size_t)nf * nf * nf;
  const double *p = phi + (size_t)(id - 1) * bsz, *l = lsf + (size_t)(id - 1) * bsz;
  double *f = fcv + (size_t)(id - 1) * fsz;
  const int32_t *X = ixp[id - 1];
  const double *D = ddp[id - 1], *bv = bvp[id - 1];
  auto fx = [&](int d, int a, int b, int c) {
    return (size_t)d * d3 + ((size_t)(c - 1) * nf + (b - 1)) * nf + (a - 1);
  };
  for (int e = 0; e < n; e++) {
    const int i = X[3 * e], j = X[3 * e + 1], k = X[3 * e + 2];
    const double *dd = D + 6 * e;
    const size_t c = ix3(ng, i, j, k);
    if (l[c] < 0) continue;
    const double pc = p[c], bc = bv[((size_t)(k - 1) * nc + (j - 1)) * nc + (i - 1)];
    if (dd[0] < 1) f[fx(0, i, j, k)] = ix_ * (pc - bc) / dd[0];
    if (dd[1] < 1) f[fx(0, i + 1, j, k)] = ix_ * (bc - pc) / dd[1];
    if (dd[2] < 1) f[fx(1, i, j, k)] = iy * (pc - bc) / dd[2];
    if (dd[3] < 1) f[fx(1, i, j + 1, k)] = iy * (bc - pc) / dd[3];
    if (dd[4] < 1) f[fx(2, i, j, k)] = iz * (pc - bc) / dd[4];
    if (dd[5] < 1) f[fx(2, i, j, k + 1)] = iz * (bc - pc) / dd[5];
  }
}

// The same with one thread per entry (boxes of at most 16^3 cells): a face
// two entries write (an entry's low face is its low neighbour cell's high
// face) keeps the value of the later entry in the list, as the serial loop
// leaves it -- each entry skips the faces a later entry rewrites (the
// entry of each cell in LDS)
template <int NC>
__global__ void __launch_bounds__(256)
    k_lsf_gradient_par(const double *__restrict__ phi, const double *__restrict__ lsf,
                       double *__restrict__ fcv, const int32_t *__restrict__ ids,
                       size_t bsz, size_t fsz, const int *__restrict__ cnt,
                       const int32_t *const *__restrict__ ixp,
                       const double *const *__restrict__ ddp,
                       const double *const *__restrict__ bvp, double ix_, double iy,
                       double iz) {
  constexpr int NG = NC + 2, NF = NC + 1, N3 = NC * NC * NC;
  constexpr size_t D3 = (size_t)NF * NF * NF;
  __shared__ int emap[N3];
  const int id = ids[blockIdx.x];
  const int n = cnt[id - 1];
  for (int c = threadIdx.x; c < N3; c += blockDim.x) emap[c] = -1;
  __syncthreads();
  const int32_t *X = ixp[id - 1];
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int c = ((X[3 * e + 2] - 1) * NC + (X[3 * e + 1] - 1)) * NC + (X[3 * e] - 1);
    atomicMax(&emap[c], e);
  }
  __syncthreads();
  const double *p = phi + (size_t)(id - 1) * bsz, *l = lsf + (size_t)(id - 1) * bsz;
  double *f = fcv + (size_t)(id - 1) * fsz;
  const double *D = ddp[id - 1], *bv = bvp[id - 1];
  auto fx = [&](int d, int a, int b, int c) {
    return (size_t)d * D3 + ((size_t)(c - 1) * NF + (b - 1)) * NF + (a - 1);
  };
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int i = X[3 * e], j = X[3 * e + 1], k = X[3 * e + 2];
    const int ce = ((k - 1) * NC + (j - 1)) * NC + (i - 1);
    if (emap[ce] > e) continue;  // a later entry of the same cell
    const size_t c = ix3(NG, i, j, k);
    if (l[c] < 0) continue;
    const double *dd = D + 6 * e;
    const double pc = p[c], bc = bv[ce];
    // the face of direction q is also written by the entry of the cell
    // across it (direction q ^ 1) if that entry is later and writes it
    auto later = [&](int q) {
      const int d = q >> 1, sgn = (q & 1) ? 1 : -1;
      int a[3] = {i, j, k};
      a[d] += sgn;
      if (a[d] < 1 || a[d] > NC) return false;
      const int cn = ((a[2] - 1) * NC + (a[1] - 1)) * NC + (a[0] - 1);
      const int e2 = emap[cn];
      return e2 > e && !(l[ix3(NG, a[0], a[1], a[2])] < 0) && D[6 * e2 + (q ^ 1)] < 1;
    };
    if (dd[0] < 1 && !later(0)) f[fx(0, i, j, k)] = ix_ * (pc - bc) / dd[0];
    if (dd[1] < 1 && !later(1)) f[fx(0, i + 1, j, k)] = ix_ * (bc - pc) / dd[1];
    if (dd[2] < 1 && !later(2)) f[fx(1, i, j, k)] = iy * (pc - bc) / dd[2];
    if (dd[3] < 1 && !later(3)) f[fx(1, i, j + 1, k)] = iy * (bc - pc) / dd[3];
    if (dd[4] < 1 && !later(4)) f[fx(2, i, j, k)] = iz * (pc - bc) / dd[4];
    if (dd[5] < 1 && !later(5)) f[fx(2, i, j, k + 1)] = iz * (bc - pc) / dd[5];
  }
}

// mg_box_field_norm (m_af_multigrid.f90:1995-2025) from the stored faces
__global__ void k_field_norm(const double *__restrict__ fcv,
                             double *__restrict__ nrm,
                             const int32_t *__restrict__ ids, int nc, size_t bsz,
                             size_t fsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  const int id = ids[blockIdx.y];
  int i, j, k;
  cell3(t, nc, i, j, k);
  const int nf = nc + 1;
  const size_t d3 = (size_t)nf * nf * nf;
  const double *f = fcv + (size_t)(id - 1) * fsz;
  const size_t fb = ((size_t)(k - 1) * nf + (j - 1)) * nf + (i - 1);
  const double a = f[fb] + f[fb + 1], b = f[d3 + fb] + f[d3 + fb + nf],
               cc = f[2 * d3 + fb] + f[2 * d3 + fb + (size_t)nf * nf];
  nrm[(size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k)] = 0.5 * sqrt(a * a + b * b + cc * cc);
}

__global__ void k_corr_tmp(const double *__restrict__ phi,
                           double *__restrict__ tmp,
                           const int32_t *__restrict__ ids, size_t bsz) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bsz) return;
  const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz + t;
  tmp[o] = phi[o] - tmp[o];
}

// FMG box operations over whole (nc+2)^3 arrays: af_box_clear_cc (src null)
// and af_boxes_copy_cc (m_af_utils.f90)
__global__ void k_box_copy(const double *__restrict__ src,
                           double *__restrict__ dst,
                           const int32_t *__restrict__ ids, size_t bsz) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bsz) return;
  const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz + t;
  dst[o] = src ? src[o] : 0.0;
}

// stencil_prolong_248 add, a column of K cells along k per thread: the
// K/2 + 2 parent planes the column touches are loaded once (4 values each)
template <int K>
__global__ void __launch_bounds__(256)
    k_prolong(double *__restrict__ phi, const double *__restrict__ tmp,
              const afh_box_meta *__restrict__ meta,
              const int32_t *__restrict__ ids, int nc, size_t bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * (nc / K)) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  int i, j, kq;
  cell3(t, nc, i, j, kq);
  const int k0 = (kq - 1) * K + 1;  // odd
  const int ng = nc + 2, hn = nc >> 1;
  const size_t sk = (size_t)ng * ng;
  const int o0 = ((m.ix[0] - 1) & 1) * hn, o1 = ((m.ix[1] - 1) & 1) * hn,
            o2 = ((m.ix[2] - 1) & 1) * hn;
  const int i1 = o0 + ((i + 1) >> 1), i2 = i1 + 1 - 2 * (i & 1);
  const int j1 = o1 + ((j + 1) >> 1), j2 = j1 + 1 - 2 * (j & 1);
  const int P = o2 + ((k0 + 1) >> 1);  // k1 of the first (odd) cell
  const double *p = tmp + (size_t)(m.parent - 1) * bsz;
  const size_t c = (size_t)(id - 1) * bsz + ix3(ng, i, j, k0);
  // parent planes P-1 .. P+K/2, values at (i1,j1), (i2,j1), (i1,j2), (i2,j2)
  double pv[K / 2 + 2][4], ph[K];
#pragma unroll
  for (int q = 0; q < K / 2 + 2; q++) {
    const size_t b = ix3(ng, 0, 0, P - 1 + q);
    pv[q][0] = p[b + (size_t)j1 * ng + i1];
    pv[q][1] = p[b + (size_t)j1 * ng + i2];
    pv[q][2] = p[b + (size_t)j2 * ng + i1];
    pv[q][3] = p[b + (size_t)j2 * ng + i2];
  }
#pragma unroll
  for (int q = 0; q < K; q++) ph[q] = phi[c + q * sk];
#pragma unroll
  for (int q = 0; q < K; q++) {
    // cell k0+q: odd q -> (k1, k2) = planes (P+(q-1)/2, P+(q+1)/2);
    // even q -> (P+q/2, P+q/2-1); a, b index pv from plane P-1
    const int a = (q & 1) ? (q + 1) / 2 : q / 2 + 1;
    const int b = (q & 1) ? (q + 3) / 2 : q / 2;
    st_nt<AFH_NT_MG>(phi + (c + q * sk),
                     ph[q] + (27 / 64.0) * pv[a][0] + (9 / 64.0) * pv[a][1] +
                         (9 / 64.0) * pv[a][2] + (3 / 64.0) * pv[a][3] +
                         (9 / 64.0) * pv[b][0] + (3 / 64.0) * pv[b][1] +
                         (3 / 64.0) * pv[b][2] + (1 / 64.0) * pv[b][3]);
  }
}

// mg_box_lpl_gradient (fc = fac/dr * (phi_i - phi_i-1)) + mg_box_field_norm
__global__ void k_gradient(const double *__restrict__ phi,
                           double *__restrict__ fcv, double *__restrict__ nrm,
                           const afh_box_meta *__restrict__ meta,
                           const int32_t *__restrict__ ids, int nc, size_t bsz,
                           size_t fsz, double fac) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int i = t % nc + 1, j = (t / nc) % nc + 1, k = t / (nc * nc) + 1;
  const int ng = nc + 2, nf = nc + 1;
  const double *p = phi + (size_t)(id - 1) * bsz;
  double *f = fcv + (size_t)(id - 1) * fsz;
  const size_t c = ix3(ng, i, j, k), sj = ng, sk = (size_t)ng * ng;
  const double ix_ = fac / m.dr[0], iy = fac / m.dr[1], iz = fac / m.dr[2];
  const double fxl = ix_ * (p[c] - p[c - 1]), fxh = ix_ * (p[c + 1] - p[c]);
  const double fyl = iy * (p[c] - p[c - sj]), fyh = iy * (p[c + sj] - p[c]);
  const double fzl = iz * (p[c] - p[c - sk]), fzh = iz * (p[c + sk] - p[c]);
  const size_t d3 = (size_t)nf * nf * nf;
  auto fx = [&](int d, int a, int b, int cc) {
    return (size_t)d * d3 + ((size_t)(cc - 1) * nf + (b - 1)) * nf + (a - 1);
  };
  f[fx(0, i, j, k)] = fxl;
  if (i == nc) f[fx(0, nc + 1, j, k)] = fxh;
  f[fx(1, i, j, k)] = fyl;
  if (j == nc) f[fx(1, i, nc + 1, k)] = fyh;
  f[fx(2, i, j, k)] = fzl;
  if (k == nc) f[fx(2, i, j, nc + 1)] = fzh;
  if (nrm) {
    const double a = fxl + fxh, b = fyl + fyh, cc = fzl + fzh;
    nrm[(size_t)(id - 1) * bsz + c] = 0.5 * sqrt(a * a + b * b + cc * cc);
  }
}

// k_gradient for a compile-time box size, one level per launch: 2-D thread
// blocks (NC x R rows) so no index divisions, and fac/dr precomputed on the
// host (every box of a level has the same dr, so the quotient is bitwise the
// one mg_box_lpl_gradient computes per box).
// Each thread owns a column of K cells in k: the K + 2 phi values of the
// column are loaded once (the z differences of neighbouring cells share them),
// and every load of the column is issued before the first store.
template <int NC, int K, bool NT = false, bool FC = true>
__global__ void __launch_bounds__(256)
    k_gradient_t(const double *__restrict__ phi, double *__restrict__ fcv,
                 double *__restrict__ nrm, const int32_t *__restrict__ ids,
                 size_t bsz, size_t fsz, const afh_box_meta *__restrict__ meta,
                 double fac) {
  constexpr int R = 256 / NC < NC ? 256 / NC : NC;  // rows per block
  constexpr int NG = NC + 2, NF = NC + 1;
  constexpr size_t SJ = NG, SK = (size_t)NG * NG, D3 = (size_t)NF * NF * NF;
  const Blk B = xcd_block();
  const int i = threadIdx.x % NC + 1;
  const int j = (B.x % (NC / R)) * R + threadIdx.x / NC + 1;
  const int k0 = (B.x / (NC / R)) * K + 1;
  const int id = ids[B.y];
  // fac / dr per dimension (every box of a level has its level's dr bits):
  // all levels in one launch
  const double ix_ = fac / meta[id - 1].dr[0], iy = fac / meta[id - 1].dr[1],
               iz = fac / meta[id - 1].dr[2];
  const double *p = phi + (size_t)(id - 1) * bsz;
  double *f = fcv + (size_t)(id - 1) * fsz;
  double *nb = nrm ? nrm + (size_t)(id - 1) * bsz : nullptr;
  const size_t c0 = ((size_t)k0 * NG + j) * NG + i;
  double pc[K + 2], xm[K], xp[K], ym[K], yp[K];
#pragma unroll
  for (int q = 0; q < K + 2; q++) pc[q] = p[c0 + (q - 1) * SK];
#pragma unroll
  for (int q = 0; q < K; q++) {
    const size_t c = c0 + q * SK;
    xm[q] = p[c - 1];
    xp[q] = p[c + 1];
    ym[q] = p[c - SJ];
    yp[q] = p[c + SJ];
  }
#pragma unroll
  for (int q = 0; q < K; q++) {
    const int k = k0 + q;
    const double pv = pc[q + 1];
    const double fxl = ix_ * (pv - xm[q]), fxh = ix_ * (xp[q] - pv);
    const double fyl = iy * (pv - ym[q]), fyh = iy * (yp[q] - pv);
    const double fzl = iz * (pv - pc[q]), fzh = iz * (pc[q + 2] - pv);
    const size_t fb = ((size_t)(k - 1) * NF + (j - 1)) * NF + (i - 1);
    if (FC) {  // (without FC: the norm only, afh_fluid_set_field_source)
      st_nt<NT>(f + fb, fxl);
      if (i == NC) st_nt<NT>(f + fb + 1, fxh);
      st_nt<NT>(f + D3 + fb, fyl);
      if (j == NC) st_nt<NT>(f + D3 + fb + NF, fyh);
      st_nt<NT>(f + 2 * D3 + fb, fzl);
      if (k == NC) st_nt<NT>(f + 2 * D3 + fb + (size_t)NF * NF, fzh);
    }
    if (nb) {
      const double a = fxl + fxh, b = fyl + fyh, cc = fzl + fzh;
      st_nt<NT>(nb + c0 + q * SK, 0.5 * sqrt(a * a + b * b + cc * cc));
    }
  }
}

#ifndef AFH_GRAD_K  // cells per thread column of k_gradient_t
#define AFH_GRAD_K 4
#endif
template <int NC>
static void launch_gradient(afh_tree *t, const double *phi, double *fcv,
                            double *nrm, double fac, bool nt) {
  constexpr int R = 256 / NC < NC ? 256 / NC : NC;
  constexpr int K = NC >= AFH_GRAD_K ? AFH_GRAD_K : 1;
  const int ntot = t->ids.off[t->nlvl];  // every box of every level
  for (int o = 0; o < ntot; o += 65535) {  // grid.y limit
    const int n = std::min(65535, ntot - o);
    auto kern = fcv ? (nt ? k_gradient_t<NC, K, true> : k_gradient_t<NC, K>)
                    : (nt ? k_gradient_t<NC, K, true, false> : k_gradient_t<NC, K, false, false>);
    hipLaunchKernelGGL(kern, dim3((NC / R) * (NC / K), n), dim3(NC * R), 0, t->stream, phi,
                       fcv, nrm, t->ids.d + o, t->bsz, t->fsz, t->d_boxes, fac);
  }
}

// ------------------------------------------------------------ coarse solver
// Same arithmetic as oracle/c/afo.c (cs_*): BCs folded into the operator as
// in stencil_handle_boundaries (m_coarse_solver.f90:442-491).
__device__ __forceinline__ size_t gix(const CsParams &P, int m, int i, int j,
                                      int k) {
  const int h = P.halo[m];
  return ((size_t)(k - 1 + h) * (P.dims[m][1] + 2 * h) + (j - 1 + h)) *
             (P.dims[m][0] + 2 * h) +
         (i - 1 + h);
}

// boundary class of a cell (2 bits per dimension), index into P.dtab
__device__ __forceinline__ int cs_class(const CsParams &P, int m, int i, int j,
                                        int k) {
  return (i == 1) | ((i == P.dims[m][0]) << 1) | ((j == 1) << 2) |
         ((j == P.dims[m][1]) << 3) | ((k == 1) << 4) |
         ((k == P.dims[m][2]) << 5);
}
__device__ __forceinline__ double cs_diag(const CsParams &P, int m, int i,
                                          int j, int k) {
  return P.dtab[(m * 64 + cs_class(P, m, i, j, k)) * 2];
}
__device__ __forceinline__ double cs_inv_diag(const CsParams &P, int m, int i,
                                              int j, int k) {
  return P.dtab[(m * 64 + cs_class(P, m, i, j, k)) * 2 + 1];
}

__device__ __forceinline__ void cs_gs_cell(const CsParams &P, int m, int i,
                                           int j, int k) {
  const int nx = P.dims[m][0], ny = P.dims[m][1], nz = P.dims[m][2];
  double *u = P.u[m];
  const double *h = P.hc[m];
  double s = P.f[m][gix(P, m, i, j, k)];
  if (i > 1) s = s - h[0] * u[gix(P, m, i - 1, j, k)];
  if (i < nx) s = s - h[0] * u[gix(P, m, i + 1, j, k)];
  if (j > 1) s = s - h[1] * u[gix(P, m, i, j - 1, k)];
  if (j < ny) s = s - h[1] * u[gix(P, m, i, j + 1, k)];
  if (k > 1) s = s - h[2] * u[gix(P, m, i, j, k - 1)];
  if (k < nz) s = s - h[2] * u[gix(P, m, i, j, k + 1)];
  u[gix(P, m, i, j, k)] = s * cs_inv_diag(P, m, i, j, k);
}

// residual f - A u of one cell (the expression of residual_box on the folded
// operator, same operand order as oracle/c/afo.c cs_residual_restrict)
__device__ __forceinline__ double cs_res(const CsParams &P, int m, int i, int j,
                                         int k) {
  const int nx = P.dims[m][0], ny = P.dims[m][1], nz = P.dims[m][2];
  const double *u = P.u[m];
  const double *h = P.hc[m];
  double a = cs_diag(P, m, i, j, k) * u[gix(P, m, i, j, k)];
  if (i > 1) a = a + h[0] * u[gix(P, m, i - 1, j, k)];
  if (i < nx) a = a + h[0] * u[gix(P, m, i + 1, j, k)];
  if (j > 1) a = a + h[1] * u[gix(P, m, i, j - 1, k)];
  if (j < ny) a = a + h[1] * u[gix(P, m, i, j + 1, k)];
  if (k > 1) a = a + h[2] * u[gix(P, m, i, j, k - 1)];
  if (k < nz) a = a + h[2] * u[gix(P, m, i, j, k + 1)];
  return P.f[m][gix(P, m, i, j, k)] - a;
}

// per-workgroup partial sums of r^2 (res) or f^2 over MG level 0 (the
// stopping rule of the multi-launch coarse cycles; summed on the host in
// workgroup order)
__global__ void k_cs_norm2(CsParams P, int res, double *__restrict__ part) {
  __shared__ double s_part[4];
  const int nx = P.dims[0][0], ny = P.dims[0][1], nz = P.dims[0][2];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double v = 0.0;
  if (t < nx * ny * nz) {
    const int i = t % nx + 1, j = (t / nx) % ny + 1, k = t / (nx * ny) + 1;
    const double x = res ? cs_res(P, 0, i, j, k) : P.f[0][gix(P, 0, i, j, k)];
    v = x * x;
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((s_part[0] + s_part[1]) + s_part[2]) + s_part[3];
}

// u = 0 on MG level 0 (PFMG with a zero rhs)
__global__ void k_cs_zero(CsParams P) {
  const int nx = P.dims[0][0], ny = P.dims[0][1], nz = P.dims[0][2];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nx * ny * nz) return;
  P.u[0][gix(P, 0, t % nx + 1, (t / nx) % ny + 1, t / (nx * ny) + 1)] = 0.0;
}

// coarse cell (i, j, k) of level c = m + 1: mean of the 8 fine residuals
// (computed here, never stored), u = 0
__device__ __forceinline__ void cs_rstr_cell(const CsParams &P, int c, int i,
                                             int j, int k) {
  const int m = c - 1;
  const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
  double s = cs_res(P, m, fi, fj, fk);
  s += cs_res(P, m, fi + 1, fj, fk);
  s += cs_res(P, m, fi, fj + 1, fk);
  s += cs_res(P, m, fi + 1, fj + 1, fk);
  s += cs_res(P, m, fi, fj, fk + 1);
  s += cs_res(P, m, fi + 1, fj, fk + 1);
  s += cs_res(P, m, fi, fj + 1, fk + 1);
  s += cs_res(P, m, fi + 1, fj + 1, fk + 1);
  P.f[c][gix(P, c, i, j, k)] = 0.125 * s;
  P.u[c][gix(P, c, i, j, k)] = 0.0;
}

__device__ __forceinline__ double cs_refl(const CsParams &P, int c, int i,
                                          int j, int k) {
  double s = 1.0;
  int idx[3] = {i, j, k};
  for (int d = 0; d < 3; d++) {
    if (idx[d] < 1) {
      idx[d] = 1;
      if (P.bctype[2 * d] == AFH_BC_DIRICHLET) s = -s;
    } else if (idx[d] > P.dims[c][d]) {
      idx[d] = P.dims[c][d];
      if (P.bctype[2 * d + 1] == AFH_BC_DIRICHLET) s = -s;
    }
  }
  return s * P.u[c][gix(P, c, idx[0], idx[1], idx[2])];
}

__device__ __forceinline__ void cs_prol_cell(const CsParams &P, int m, int i,
                                             int j, int k) {
  const int c = m + 1;
  const int i1 = (i + 1) >> 1, i2 = i1 + 1 - 2 * (i & 1);
  const int j1 = (j + 1) >> 1, j2 = j1 + 1 - 2 * (j & 1);
  const int k1 = (k + 1) >> 1, k2 = k1 + 1 - 2 * (k & 1);
  double *u = P.u[m];
  const size_t g = gix(P, m, i, j, k);
  u[g] = u[g] + (27 / 64.0) * cs_refl(P, c, i1, j1, k1) +
         (9 / 64.0) * cs_refl(P, c, i2, j1, k1) +
         (9 / 64.0) * cs_refl(P, c, i1, j2, k1) +
         (3 / 64.0) * cs_refl(P, c, i2, j2, k1) +
         (9 / 64.0) * cs_refl(P, c, i1, j1, k2) +
         (3 / 64.0) * cs_refl(P, c, i2, j1, k2) +
         (3 / 64.0) * cs_refl(P, c, i1, j2, k2) +
         (1 / 64.0) * cs_refl(P, c, i2, j2, k2);
}

// multi-block passes over one (large, even-sized) MG level
__global__ void k_cs_gsrb(CsParams P, int m, int n) {
  const int nx = P.dims[m][0], ny = P.dims[m][1], nz = P.dims[m][2];
  const int hx = nx >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hx * ny * nz) return;
  const int ih = t % hx, j = (t / hx) % ny + 1, k = t / (hx * ny) + 1;
  cs_gs_cell(P, m, 2 - ((n ^ (k + j)) & 1) + 2 * ih, j, k);
}
// residual + restriction into level c (one launch)
__global__ void k_cs_rstr(CsParams P, int c) {
  const int nx = P.dims[c][0], ny = P.dims[c][1], nz = P.dims[c][2];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nx * ny * nz) return;
  cs_rstr_cell(P, c, t % nx + 1, (t / nx) % ny + 1, t / (nx * ny) + 1);
}
__global__ void k_cs_prol(CsParams P, int m) {
  const int nx = P.dims[m][0], ny = P.dims[m][1], nz = P.dims[m][2];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nx * ny * nz) return;
  cs_prol_cell(P, m, t % nx + 1, (t / nx) % ny + 1, t / (nx * ny) + 1);
}

// The small MG levels m0..bottom run inside ONE workgroup with u and f in
// LDS (compact layout, no ghost layer: the folded operator never reads
// outside the grid). Levels of more than WAVE_CELLS cells are swept by the
// whole workgroup with a barrier after every pass; from the first level of
// at most WAVE_CELLS cells down to the bottom and back, wave 0 works alone
// (no workgroup barriers: a wave's LDS operations complete in order, so a
// compiler fence is all a pass needs). Cell indices are decoded with
// shifts when the level's nx, ny are powers of two.
constexpr int CS_WAVE_CELLS = 512;

// One small level as the LDS kernel sees it: dims, log2 dims (-1 if not
// powers of two), stencil weights, offsets of u and f in the LDS pool.
// Every access goes through the __shared__ pool array itself, so the
// compiler emits LDS instructions (pointers stored in a struct would be
// generic / flat accesses).
struct SmLvl {
  int nx, ny, nz, lg;
  int uo, fo;
  double h0, h1, h2;
};

template <bool WAVE>
struct CsExec {
  __device__ static int tid() { return WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x; }
  __device__ static int nth() { return WAVE ? 64 : (int)blockDim.x; }
  __device__ static void sync() {
    if (WAVE) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    } else {
      __syncthreads();
    }
  }
};

__device__ __forceinline__ int sm_cls(const SmLvl &L, int i, int j, int k) {
  return (i == 1) | ((i == L.nx) << 1) | ((j == 1) << 2) | ((j == L.ny) << 3) |
         ((k == 1) << 4) | ((k == L.nz) << 5);
}

// cs_gs_cell on a compact LDS level (same operand order)
__device__ __forceinline__ void sm_gs_cell(double *lds, const double *dt,
                                           const SmLvl &L, int i, int j, int k) {
  const int c = ((k - 1) * L.ny + (j - 1)) * L.nx + (i - 1);
  const int sy = L.nx, sz = L.nx * L.ny;
  const double *u = lds + L.uo;
  double s = lds[L.fo + c];
  if (i > 1) s = s - L.h0 * u[c - 1];
  if (i < L.nx) s = s - L.h0 * u[c + 1];
  if (j > 1) s = s - L.h1 * u[c - sy];
  if (j < L.ny) s = s - L.h1 * u[c + sy];
  if (k > 1) s = s - L.h2 * u[c - sz];
  if (k < L.nz) s = s - L.h2 * u[c + sz];
  lds[L.uo + c] = s * dt[sm_cls(L, i, j, k) * 2 + 1];
}

// cs_res on a compact LDS level
__device__ __forceinline__ double sm_res(const double *lds, const double *dt,
                                         const SmLvl &L, int i, int j, int k) {
  const int c = ((k - 1) * L.ny + (j - 1)) * L.nx + (i - 1);
  const int sy = L.nx, sz = L.nx * L.ny;
  const double *u = lds + L.uo;
  double a = dt[sm_cls(L, i, j, k) * 2] * u[c];
  if (i > 1) a = a + L.h0 * u[c - 1];
  if (i < L.nx) a = a + L.h0 * u[c + 1];
  if (j > 1) a = a + L.h1 * u[c - sy];
  if (j < L.ny) a = a + L.h1 * u[c + sy];
  if (k > 1) a = a + L.h2 * u[c - sz];
  if (k < L.nz) a = a + L.h2 * u[c + sz];
  return lds[L.fo + c] - a;
}

// cs_refl on a compact LDS level
__device__ __forceinline__ double sm_refl(const double *lds, const SmLvl &C,
                                          const int *bct, int i, int j, int k) {
  double s = 1.0;
  int idx[3] = {i, j, k};
  const int dims[3] = {C.nx, C.ny, C.nz};
#pragma unroll
  for (int d = 0; d < 3; d++) {
    if (idx[d] < 1) {
      idx[d] = 1;
      if (bct[2 * d] == AFH_BC_DIRICHLET) s = -s;
    } else if (idx[d] > dims[d]) {
      idx[d] = dims[d];
      if (bct[2 * d + 1] == AFH_BC_DIRICHLET) s = -s;
    }
  }
  return s * lds[C.uo + ((idx[2] - 1) * C.ny + (idx[1] - 1)) * C.nx + (idx[0] - 1)];
}

// cell t (0-based, i fastest) -> (i, j, k), 1-based
__device__ __forceinline__ void sm_decode(const SmLvl &L, int t, int &i, int &j,
                                          int &k) {
  if (L.lg >= 0) {
    const int lx = L.lg & 0xff, ly = L.lg >> 8;
    i = (t & (L.nx - 1)) + 1;
    j = ((t >> lx) & (L.ny - 1)) + 1;
    k = (t >> (lx + ly)) + 1;
  } else {
    i = t % L.nx + 1;
    j = (t / L.nx) % L.ny + 1;
    k = t / (L.nx * L.ny) + 1;
  }
}

template <bool WAVE>
__device__ void sm_gs(double *lds, const SmLvl *lv, const double *dtab, int m,
                      int n) {
  using X = CsExec<WAVE>;
  const SmLvl L = lv[m];
  const double *dt = dtab + m * 128;
  if ((L.nx & 1) == 0) {
    // the cells of parity n only: nx/2 per row
    const int hx = L.nx >> 1, N = hx * L.ny * L.nz;
    for (int t = X::tid(); t < N; t += X::nth()) {
      int ih, j, k;
      if (L.lg >= 0) {
        const int lx = (L.lg & 0xff) - 1, ly = L.lg >> 8;
        ih = t & (hx - 1);
        j = ((t >> lx) & (L.ny - 1)) + 1;
        k = (t >> (lx + ly)) + 1;
      } else {
        ih = t % hx;
        j = (t / hx) % L.ny + 1;
        k = t / (hx * L.ny) + 1;
      }
      sm_gs_cell(lds, dt, L, 2 - ((n ^ (k + j)) & 1) + 2 * ih, j, k);
    }
  } else {
    const int N = L.nx * L.ny * L.nz;
    for (int t = X::tid(); t < N; t += X::nth()) {
      int i, j, k;
      sm_decode(L, t, i, j, k);
      const int i0 = 2 - ((n ^ (k + j)) & 1);
      if (((i - i0) & 1) == 0) sm_gs_cell(lds, dt, L, i, j, k);
    }
  }
  X::sync();
}

// residual of level m restricted into level m + 1 (cs_rstr_cell order)
template <bool WAVE>
__device__ void sm_rstr(double *lds, const SmLvl *lv, const double *dtab, int m) {
  using X = CsExec<WAVE>;
  const SmLvl L = lv[m], C = lv[m + 1];
  const double *dt = dtab + m * 128;
  const int N = C.nx * C.ny * C.nz;
  for (int t = X::tid(); t < N; t += X::nth()) {
    int i, j, k;
    sm_decode(C, t, i, j, k);
    const int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
    double s = sm_res(lds, dt, L, fi, fj, fk);
    s += sm_res(lds, dt, L, fi + 1, fj, fk);
    s += sm_res(lds, dt, L, fi, fj + 1, fk);
    s += sm_res(lds, dt, L, fi + 1, fj + 1, fk);
    s += sm_res(lds, dt, L, fi, fj, fk + 1);
    s += sm_res(lds, dt, L, fi + 1, fj, fk + 1);
    s += sm_res(lds, dt, L, fi, fj + 1, fk + 1);
    s += sm_res(lds, dt, L, fi + 1, fj + 1, fk + 1);
    lds[C.fo + t] = 0.125 * s;
    lds[C.uo + t] = 0.0;
  }
  X::sync();
}

// prolongation of level m + 1 added to level m (cs_prol_cell order)
template <bool WAVE>
__device__ void sm_prol(double *lds, const SmLvl *lv, const int *bct, int m) {
  using X = CsExec<WAVE>;
  const SmLvl L = lv[m], C = lv[m + 1];
  const int N = L.nx * L.ny * L.nz;
  for (int t = X::tid(); t < N; t += X::nth()) {
    int i, j, k;
    sm_decode(L, t, i, j, k);
    const int i1 = (i + 1) >> 1, i2 = i1 + 1 - 2 * (i & 1);
    const int j1 = (j + 1) >> 1, j2 = j1 + 1 - 2 * (j & 1);
    const int k1 = (k + 1) >> 1, k2 = k1 + 1 - 2 * (k & 1);
    lds[L.uo + t] = lds[L.uo + t] + (27 / 64.0) * sm_refl(lds, C, bct, i1, j1, k1) +
                    (9 / 64.0) * sm_refl(lds, C, bct, i2, j1, k1) +
                    (9 / 64.0) * sm_refl(lds, C, bct, i1, j2, k1) +
                    (3 / 64.0) * sm_refl(lds, C, bct, i2, j2, k1) +
                    (9 / 64.0) * sm_refl(lds, C, bct, i1, j1, k2) +
                    (3 / 64.0) * sm_refl(lds, C, bct, i2, j1, k2) +
                    (3 / 64.0) * sm_refl(lds, C, bct, i1, j2, k2) +
                    (1 / 64.0) * sm_refl(lds, C, bct, i2, j2, k2);
  }
  X::sync();
}

template <bool WAVE>
__device__ void sm_smooth(double *lds, const SmLvl *lv, const double *dtab,
                          int m, int pairs) {
  for (int s = 0; s < pairs; s++) {
    sm_gs<WAVE>(lds, lv, dtab, m, 1);
    sm_gs<WAVE>(lds, lv, dtab, m, 2);
  }
}

// The small MG levels m0..bottom run inside ONE workgroup with u and f in
// LDS (compact layout, no ghost layer: the folded operator never reads
// outside the grid). Levels of more than CS_WAVE_CELLS cells are swept by
// the whole workgroup with a barrier after every pass; from the first level
// of at most CS_WAVE_CELLS cells down to the bottom and back, wave 0 works
// alone (no workgroup barriers: a wave's LDS operations complete in order,
// so a compiler fence is all a pass needs).
// sum of v over the workgroup, the same value in every thread (wave
// shuffles, then the waves' partials in order)
__device__ double cs_block_sum(double v, double *part) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int q = 0; q < (int)(blockDim.x >> 6); q++) s += part[q];
  return s;
}

// tol2 > 0: HYPRE PFMG's stopping rule on level m0 = 0 (|r|^2 < tol2 |b|^2
// after a cycle, at most n_cycles; b = 0 gives u = 0); the cycles run go to
// *cycles_out (when set)
__global__ void __launch_bounds__(1024) k_cs_small(CsParams G, int m0,
                                                   int n_cycles, int wave_cells,
                                                   double tol2, int *cycles_out) {
  extern __shared__ double lds[];
  __shared__ double s_part[16];
  __shared__ SmLvl s_lv[MAXMG];
  __shared__ double s_dtab[MAXMG * 64 * 2];  // (diag, 1/diag) per class
  __shared__ int s_bct[6];
  const int bot = G.n_mg - 1;
  for (int q = threadIdx.x; q < (bot + 1) * 128; q += blockDim.x)
    s_dtab[q] = G.dtab[q];
  if (threadIdx.x == 0) {
    int off = 0;
    for (int m = m0; m <= bot; m++) {
      SmLvl &L = s_lv[m];
      L.nx = G.dims[m][0], L.ny = G.dims[m][1], L.nz = G.dims[m][2];
      L.lg = G.lg[m];
      L.h0 = G.hc[m][0], L.h1 = G.hc[m][1], L.h2 = G.hc[m][2];
      const int n = L.nx * L.ny * L.nz;
      L.uo = off;
      L.fo = off + n;
      off += 2 * n;
    }
    for (int q = 0; q < 6; q++) s_bct[q] = G.bctype[q];
  }
  __syncthreads();
  {
    const SmLvl L = s_lv[m0];
    const int N = L.nx * L.ny * L.nz;
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
      int i, j, k;
      sm_decode(L, t, i, j, k);
      lds[L.uo + t] = G.u[m0][gix(G, m0, i, j, k)];
      lds[L.fo + t] = G.f[m0][gix(G, m0, i, j, k)];
    }
    __syncthreads();
  }
  // first level handled by wave 0 alone
  int mw = m0;
  while (mw < bot && s_lv[mw].nx * s_lv[mw].ny * s_lv[mw].nz > wave_cells) mw++;
  const bool wave_tail = s_lv[mw].nx * s_lv[mw].ny * s_lv[mw].nz <= wave_cells;
  double bb = 0.0;
  if (tol2 > 0) {
    const SmLvl L = s_lv[m0];
    const int N = L.nx * L.ny * L.nz;
    double p = 0.0;
    for (int t = threadIdx.x; t < N; t += blockDim.x) p += lds[L.fo + t] * lds[L.fo + t];
    bb = cs_block_sum(p, s_part);
    if (bb == 0.0) {
      for (int t = threadIdx.x; t < N; t += blockDim.x) lds[L.uo + t] = 0.0;
      __syncthreads();
      n_cycles = 0;
    }
  }
  int cyc = 0;
  while (cyc < n_cycles) {
    for (int m = m0; m < mw; m++) {
      sm_smooth<false>(lds, s_lv, s_dtab, m, 2);
      sm_rstr<false>(lds, s_lv, s_dtab, m);
    }
    if (wave_tail) {
      if (threadIdx.x < 64) {
        for (int m = mw; m < bot; m++) {
          sm_smooth<true>(lds, s_lv, s_dtab, m, 2);
          sm_rstr<true>(lds, s_lv, s_dtab, m);
        }
        sm_smooth<true>(lds, s_lv, s_dtab, bot, CS_BOTTOM_SWEEPS);
        for (int m = bot - 1; m >= mw; m--) {
          sm_prol<true>(lds, s_lv, s_bct, m);
          sm_smooth<true>(lds, s_lv, s_dtab, m, 2);
        }
      }
      __syncthreads();
    } else {
      sm_smooth<false>(lds, s_lv, s_dtab, bot, CS_BOTTOM_SWEEPS);  // mw == bot
    }
    for (int m = mw - 1; m >= m0; m--) {
      sm_prol<false>(lds, s_lv, s_bct, m);
      sm_smooth<false>(lds, s_lv, s_dtab, m, 2);
    }
    cyc++;
    if (tol2 > 0) {
      const SmLvl L = s_lv[m0];
      const double *dt = s_dtab + m0 * 128;
      double p = 0.0;
      for (int t = threadIdx.x; t < L.nx * L.ny * L.nz; t += blockDim.x) {
        int i, j, k;
        sm_decode(L, t, i, j, k);
        const double r = sm_res(lds, dt, L, i, j, k);
        p += r * r;
      }
      if (cs_block_sum(p, s_part) / bb < tol2) break;  // the same in every thread
    }
  }
  if (cycles_out && threadIdx.x == 0) *cycles_out = cyc;
  {
    const SmLvl L = s_lv[m0];
    const int N = L.nx * L.ny * L.nz;
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
      int i, j, k;
      sm_decode(L, t, i, j, k);
      G.u[m0][gix(G, m0, i, j, k)] = lds[L.uo + t];
    }
  }
}

// coarse_solver_set_rhs_phi: gather rhs (+ folded BC values) and phi
__global__ void k_cs_gather(CsParams P, const double *__restrict__ phi,
                            const double *__restrict__ rhs,
                            const afh_box_meta *__restrict__ meta,
                            const int32_t *__restrict__ ids, int nc,
                            size_t bsz, afh_bc b0, afh_bc b1, afh_bc b2,
                            afh_bc b3, afh_bc b4, afh_bc b5) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int i = t % nc + 1, j = (t / nc) % nc + 1, k = t / (nc * nc) + 1;
  const int gi[3] = {(m.ix[0] - 1) * nc + i, (m.ix[1] - 1) * nc + j,
                     (m.ix[2] - 1) * nc + k};
  const afh_bc bc[6] = {b0, b1, b2, b3, b4, b5};
  const size_t c = (size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k);
  double rv = rhs[c];
  for (int nb = 1; nb <= 6; nb++) {
    const int dd = (nb - 1) >> 1;
    const bool low = ((nb - 1) & 1) == 0;
    const bool at = low ? (gi[dd] == 1) : (gi[dd] == P.dims[0][dd]);
    if (!at) continue;
    const double cnb = P.hc[0][dd];
    double b2r;
    if (bc[nb - 1].type == AFH_BC_DIRICHLET) b2r = -2 * cnb;
    else b2r = -(cnb * m.dr[dd]) * (low ? -1 : 1);
    rv = rv + b2r * bc[nb - 1].value;
  }
  const size_t g = gix(P, 0, gi[0], gi[1], gi[2]);
  P.f[0][g] = rv;
  P.u[0][g] = phi[c];
}

__global__ void k_cs_scatter(CsParams P, double *__restrict__ phi,
                             const afh_box_meta *__restrict__ meta,
                             const int32_t *__restrict__ ids, int nc,
                             size_t bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int i = t % nc + 1, j = (t / nc) % nc + 1, k = t / (nc * nc) + 1;
  phi[(size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k)] =
      P.u[0][gix(P, 0, (m.ix[0] - 1) * nc + i, (m.ix[1] - 1) * nc + j,
                 (m.ix[2] - 1) * nc + k)];
}

// AFH_COARSE_DIRECT: one 1-D transform of the level-1 grid along dim d,
// out(c) = sum_p M[p][c_d] in(.., p, ..) with M = Q (forward, Q^T f) or Q^T
// (inverse, Q u^); summed in p order as oracle/c/afo.c cs_transform. With
// `div` the forward result is divided by the eigenvalue sum (zero modes 0).
__global__ void __launch_bounds__(256)
    k_cs_transform(const double *__restrict__ in, int in_halo,
                   double *__restrict__ out, int out_halo,
                   const double *__restrict__ M, const double *__restrict__ e0,
                   const double *__restrict__ e1, const double *__restrict__ e2,
                   int nx, int ny, int nz, int d, int div, double lam) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nx * ny * nz) return;
  const int i = t % nx, j = (t / nx) % ny, k = t / (nx * ny);
  const int n = d == 0 ? nx : (d == 1 ? ny : nz);
  const int co = d == 0 ? i : (d == 1 ? j : k);
  // stride of dim d and the address of p = 0 in `in`
  const int hx = nx + 2 * in_halo, hy = ny + 2 * in_halo;
  const size_t st = d == 0 ? 1 : (d == 1 ? (size_t)hx : (size_t)hx * hy);
  int c[3] = {i + in_halo, j + in_halo, k + in_halo};
  c[d] = in_halo;
  const double *src = in + ((size_t)c[2] * hy + c[1]) * hx + c[0];
  double s = 0.0;
  // (unrolled: the loads of 16 terms in flight together; the sum keeps the
  // p order)
#pragma unroll 16
  for (int p = 0; p < n; p++) s = s + M[(size_t)p * n + co] * src[p * st];
  if (div) {
    const double den = ((e0[i] + e1[j]) + e2[k]) - lam;
    s = den != 0.0 ? s / den : 0.0;
  }
  const size_t o = out_halo
                       ? (((size_t)k + 1) * (ny + 2) + j + 1) * (nx + 2) + i + 1
                       : ((size_t)k * ny + j) * nx + i;
  out[o] = s;
}

// AFH_COARSE_DIRECT on a level-1 grid of at most CS_DS_CELLS cells (the 8^3
// of streamer_3d.cfg) in ONE workgroup: k_cs_gather's folded
// rhs, the six k_cs_transform passes and k_cs_scatter, the grid held in LDS
// (compact, i fastest) -- the same sums in the same order, one launch
// instead of eight.
__global__ void __launch_bounds__(1024)
    k_cs_direct_small(CsParams P, double *__restrict__ phi, const double *__restrict__ rhs,
                      const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids,
                      int nid, int nc, size_t bsz, afh_bc b0, afh_bc b1, afh_bc b2,
                      afh_bc b3, afh_bc b4, afh_bc b5, const double *__restrict__ q0,
                      const double *__restrict__ q1, const double *__restrict__ q2,
                      const double *__restrict__ qt0, const double *__restrict__ qt1,
                      const double *__restrict__ qt2, const double *__restrict__ e0,
                      const double *__restrict__ e1, const double *__restrict__ e2,
                      double lam) {
  __shared__ double A[CS_SMALL_CELLS], B[CS_SMALL_CELLS];
  __shared__ double Ml[6][CS_DS_N * CS_DS_N];
  const int nx = P.dims[0][0], ny = P.dims[0][1], nz = P.dims[0][2];
  const int N = nx * ny * nz, n3 = nc * nc * nc;
  const afh_bc bc[6] = {b0, b1, b2, b3, b4, b5};
  for (int u = threadIdx.x; u < nid * n3; u += blockDim.x) {
    const int id = ids[u / n3], t = u % n3;
    const afh_box_meta &m = meta[id - 1];
    const int i = t % nc + 1, j = (t / nc) % nc + 1, k = t / (nc * nc) + 1;
    const int gi[3] = {(m.ix[0] - 1) * nc + i, (m.ix[1] - 1) * nc + j,
                       (m.ix[2] - 1) * nc + k};
    double rv = rhs[(size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k)];
    for (int nb = 1; nb <= 6; nb++) {
      const int dd = (nb - 1) >> 1;
      const bool low = ((nb - 1) & 1) == 0;
      const bool at = low ? (gi[dd] == 1) : (gi[dd] == P.dims[0][dd]);
      if (!at) continue;
      const double cnb = P.hc[0][dd];
      double b2r;
      if (bc[nb - 1].type == AFH_BC_DIRICHLET) b2r = -2 * cnb;
      else b2r = -(cnb * m.dr[dd]) * (low ? -1 : 1);
      rv = rv + b2r * bc[nb - 1].value;
    }
    A[((gi[2] - 1) * ny + (gi[1] - 1)) * nx + (gi[0] - 1)] = rv;
  }
  // Q^T along x, y, z (divide), then Q along z, y, x: A -> B -> A -> B -> A -> B -> A
  const double *Ms[6] = {q0, q1, q2, qt2, qt1, qt0};
  const int ds[6] = {0, 1, 2, 2, 1, 0};
  const bool small = nx <= CS_DS_N && ny <= CS_DS_N && nz <= CS_DS_N;
  if (small)
    for (int ps = 0; ps < 6; ps++) {
      const int d = ds[ps], n = d == 0 ? nx : (d == 1 ? ny : nz);
      for (int u = threadIdx.x; u < n * n; u += blockDim.x) Ml[ps][u] = Ms[ps][u];
    }
  __syncthreads();
  if (small) {
    // grids of at most 16 cells per dimension: one thread per grid line
    // holds the line's n values in registers and forms its n outputs, each
    // the ordered sum over p of M[p][c] x[p] with the matrix entries
    // wave-uniform (scalar loads): per output no LDS traffic but the store,
    // instead of 2 n LDS reads (the LDS throughput bound this pass before)
    for (int ps = 0; ps < 6; ps++) {
      const double *in = (ps & 1) ? B : A;
      double *out = (ps & 1) ? A : B;
      const int d = ds[ps], n = d == 0 ? nx : (d == 1 ? ny : nz);
      const int st = d == 0 ? 1 : (d == 1 ? nx : nx * ny);
      const double *M = Ml[ps];  // uniform addresses: LDS broadcast reads
      const int nl = N / n;
      for (int l = threadIdx.x; l < nl; l += blockDim.x) {
        // the line's cell 0 along d
        const int base = d == 0 ? l * nx : d == 1 ? (l / nx) * nx * ny + l % nx : l;
        double x[CS_DS_N];
#pragma unroll
        for (int p = 0; p < CS_DS_N; p++) x[p] = p < n ? in[base + p * st] : 0.0;
#pragma unroll
        for (int c = 0; c < CS_DS_N; c++) {
          if (c < n) {
            double sum = 0.0;
#pragma unroll
            for (int p = 0; p < CS_DS_N; p++)
              if (p < n) sum = sum + M[p * n + c] * x[p];
            const int o = base + c * st;
            if (ps == 2) {
              const int i = o % nx, j = (o / nx) % ny, k = o / (nx * ny);
              const double den = ((e0[i] + e1[j]) + e2[k]) - lam;
              sum = den != 0.0 ? sum / den : 0.0;
            }
            out[o] = sum;
          }
        }
      }
      __syncthreads();
    }
  } else {
    for (int ps = 0; ps < 6; ps++) {
      const double *in = (ps & 1) ? B : A;
      double *out = (ps & 1) ? A : B;
      const int d = ds[ps], n = d == 0 ? nx : (d == 1 ? ny : nz);
      const int st = d == 0 ? 1 : (d == 1 ? nx : nx * ny);
      const double *M = Ms[ps];
      for (int t = threadIdx.x; t < N; t += blockDim.x) {
        const int i = t % nx, j = (t / nx) % ny, k = t / (nx * ny);
        const int co = d == 0 ? i : (d == 1 ? j : k);
        const double *src = in + (t - co * st);
        double sum = 0.0;
        for (int p = 0; p < n; p++) sum = sum + M[p * n + co] * src[p * st];
        if (ps == 2) {
          const double den = ((e0[i] + e1[j]) + e2[k]) - lam;
          sum = den != 0.0 ? sum / den : 0.0;
        }
        out[t] = sum;
      }
      __syncthreads();
    }
  }
  // the sixth pass wrote A
  for (int u = threadIdx.x; u < nid * n3; u += blockDim.x) {
    const int id = ids[u / n3], t = u % n3;
    const afh_box_meta &m = meta[id - 1];
    const int i = t % nc + 1, j = (t / nc) % nc + 1, k = t / (nc * nc) + 1;
    phi[(size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k)] =
        A[(((m.ix[2] - 1) * nc + k - 1) * ny + (m.ix[1] - 1) * nc + j - 1) * nx +
          (m.ix[0] - 1) * nc + i - 1];
  }
}

// ---- AFH_COARSE_PFMG (afh_pfmg_dev.h): the level-1 boxes gathered with
// the boundary fold and the level-set term, the solve, the scatter
using afh_pf::PfLvl;
using afh_pf::PF_NPART;

struct PfBc {
  afh_bc bc[6];
};

// LDS: x images, b, r in LDS (else the global scratch gx, 4 np doubles);
// STAGE: the wave levels' operators too (else read from A)
template <bool LDS, bool STAGE>
__global__ void __launch_bounds__(1024)
    k_cs_pfmg(const PfLvl *__restrict__ Lg, int nl, int wave_from, const double *__restrict__ A,
              const double *__restrict__ Pw, const double *__restrict__ b2r,
              const uint8_t *__restrict__ fmask, const double *const *__restrict__ vbc,
              double *__restrict__ gx, double *__restrict__ phi,
              const double *__restrict__ rhs, const afh_box_meta *__restrict__ meta,
              const int32_t *__restrict__ ids, int nid, int nc, size_t bsz, PfBc B,
              double tol, int max_iter, int *__restrict__ iters_out) {
  extern __shared__ double pf_sm[];
  __shared__ double slot;
#ifdef AFH_PFMG_TIMING
  if (threadIdx.x == 0) {
    for (int q = 0; q < 23; q++) afh_pf::pf_tacc()[q] = 0;
    afh_pf::pf_tacc()[23] = clock64();
  }
  const unsigned long long w0 = wall_clock64();
#endif
  const PfLvl L0 = Lg[0];
  const int np = Lg[nl - 1].off + Lg[nl - 1].np;
  const int soff = wave_from < nl ? Lg[wave_from].off : np;
  double *X0 = LDS ? pf_sm : gx;
  double *X1 = X0 + np, *b = X0 + 2 * np, *r = X0 + 3 * np;
  const double *Aw = A + (size_t)27 * soff;
  if (LDS && STAGE) {
    double *As = pf_sm + 4 * np;
    for (int u = threadIdx.x; u < 27 * (np - soff); u += blockDim.x) As[u] = Aw[u];
    Aw = As;
  }
  const int n3 = nc * nc * nc, nx = L0.n[0], ny = L0.n[1];
  // coarse_solver_set_rhs_phi: rhs + boundary values (+ level-set term), phi
  for (int u = threadIdx.x; u < nid * n3; u += blockDim.x) {
    const int q = u / n3, e = u % n3, id = ids[q];
    const afh_box_meta &m = meta[id - 1];
    const int i = e % nc + 1, j = (e / nc) % nc + 1, k = e / (nc * nc) + 1;
    const int gi = (m.ix[0] - 1) * nc + i, gj = (m.ix[1] - 1) * nc + j,
              gk = (m.ix[2] - 1) * nc + k;
    const int p = ((gk - 1) * ny + (gj - 1)) * nx + (gi - 1);
    const size_t c = (size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k);
    double rv = rhs[c];
    const int fm = fmask[p];
#pragma unroll
    for (int nb = 0; nb < 6; nb++)
      if ((fm >> nb) & 1) rv = rv + b2r[(size_t)nb * L0.np + p] * B.bc[nb].value;
    if (vbc[q]) rv = rv + vbc[q][e];
    b[p] = rv;
    X0[p] = phi[c];
  }
  __syncthreads();
  PF_T(10);
  int cur = 0;
  const int iters = afh_pf::pf_solve_block(Lg, nl, wave_from, A, Aw, soff, Pw, X0, X1, b, r,
                                           &slot, tol, max_iter, &cur);
  const double *x = cur ? X1 : X0;
  // coarse_solver_get_phi
  for (int u = threadIdx.x; u < nid * n3; u += blockDim.x) {
    const int q = u / n3, e = u % n3, id = ids[q];
    const afh_box_meta &m = meta[id - 1];
    const int i = e % nc + 1, j = (e / nc) % nc + 1, k = e / (nc * nc) + 1;
    (void)q;
    const int p = (((m.ix[2] - 1) * nc + k - 1) * ny + (m.ix[1] - 1) * nc + j - 1) * nx +
                  (m.ix[0] - 1) * nc + i - 1;
    phi[(size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k)] = x[p];
  }
  if (threadIdx.x == 0 && iters_out) *iters_out = iters;
#ifdef AFH_PFMG_TIMING
  PF_T(11);
  if (threadIdx.x == 0) {
    const unsigned long long *a = afh_pf::pf_tacc();
    printf("PFTIME nt %d np %d nl %d wave %d iters %d wall10ns %llu | relax %llu/%llu res %llu/%llu "
           "rstr %llu/%llu interp %llu/%llu dot %llu/%llu handoff %llu | wave relax %llu/%llu "
           "res %llu/%llu rstr %llu/%llu interp %llu/%llu | gather %llu scatter %llu\n",
           (int)blockDim.x, np, nl, wave_from, iters, wall_clock64() - w0, a[0], a[12], a[1],
           a[13], a[2], a[14], a[3], a[15], a[4], a[16], a[5], a[6], a[18], a[7], a[19], a[8],
           a[20], a[9], a[21], a[10], a[11]);
  }
#endif
}

}  // namespace afh

using namespace afh;

#ifndef AFH_RES_K  // cells per thread column of k_residual (8, 4 or 2; 0: 8 on
#define AFH_RES_K 0  // boxes of 32^3 and up, 4 below)
#endif
#ifndef AFH_RSTR_K  // coarse cells per thread column of k_rstr_fas_col
#define AFH_RSTR_K 4
#endif
struct afh_mg {
  afh_tree *t = nullptr;
  afh_mg_desc d;
  std::vector<Coef> lvl_c;  // per tree level
  CsParams P;
  int small_from = 0;       // first MG level run by k_cs_small
  size_t small_lds = 0;     // LDS bytes of the levels k_cs_small holds
  double *d_dtab = nullptr; // device copy of h_dtab
  std::vector<double> h_dtab;
  int tab_bc[6] = {0, 0, 0, 0, 0, 0};
  // fused GSRB pairs (k_gsrb_pair) on levels with at least fused_min boxes
  // (default: enough boxes for one workgroup per CU, 256 tiles)
  int fused_min = 0;
  bool force_tiles = false;  // AFH_GSRB_TILES
  bool pair_box = true;      // false: plane-marching pair for NC <= 16
  // AFH_RCCL_CAPTURE=1: a V-cycle of a tree sharded over RCCL is captured as
  // ONE graph with its exchanges (pack, grouped send / recv, unpack) inside,
  // instead of segments between host-driven exchanges. Off until measured on
  // more than one GPU (a capture failure falls back to the eager cycle)
  bool rccl_capture = false;
  // per level: the rhs replicas exchanged by this V-cycle's down leg
  std::vector<char> rhs_halo;
  int vc_max_lvl = 0;  // the highest level of the V-cycle being issued
  bool grad_nt = true;       // the gradient's face fields and |E| stored
                             // nontemporal (streaming): -9 % on S1-64 (scripts/grad_ab.py)
  // t->gen[i_phi] when this multigrid last left phi's ghost cells current
  // (a V-cycle over all levels, or an FMG fill); anything else that writes
  // phi bumps the generation. The fused pair needs current ghost cells on
  // entry (phase B takes a same-level neighbour's boundary column from this
  // box's ghost column), so a V-cycle that finds them stale (after a regrid,
  // an upload, a copy) smooths its top level with split half-sweeps first
  uint64_t phi_gc_gen = UINT64_MAX;
  uint64_t phi_gc_meth = UINT64_MAX;  // t->meth_gen of that fill (boundary values)
  int *cs_iters = nullptr;     // pairs the last k_cs_electrode took
  // level-1 cycles of the last coarse solve (afh_mg_coarse_iterations): on
  // the device when k_cs_small applied the stopping rule, else on the host
  // AFH_CS_DIRECT_SMALL: the direct solve of a level-1 grid of at most
  // CS_DS_CELLS cells in one workgroup (k_cs_direct_small), default on
  bool cs_direct_small = true;
  int cs_ds_cells = CS_DS_CELLS;  // its size limit (at most CS_SMALL_CELLS)
  bool pair_push = true;  // AFH_PAIR_PUSH: the small-box pair fills the faces
  // (round 4: S3 1.71 -> 1.57 ms per step, profiles/r04_push_ab.txt)
  bool prolong_push = true;  // AFH_PROLONG_PUSH: so does the small-box correction
  bool rstr_push = true;     // AFH_RSTR_PUSH: and the small-box restriction
  // inside afh_mg_fas_fmg's V-cycles: the levels below the cycle's top had
  // their ghost cells filled by the previous (one level lower) V-cycle's up
  // leg or the level-1 solve, so the restriction may push faces there too
  bool in_fmg = false;
  int tiles_min = 256;  // levels of fewer boxes run tiles (NC >= 32)
  int *d_cycles = nullptr;
  int cycles_host = 0;
  bool cycles_on_dev = false;
  double *d_norm = nullptr;   // k_cs_norm2 partial sums
  Coef *d_lvl_c = nullptr;    // lvl_c on the device (residual of every level in one launch)
  std::vector<double> h_norm;
  bool rstr_col = true;       // AFH_RSTR_COL=0: one coarse cell per thread (k_rstr_fas)
  int rstr_k = AFH_RSTR_K;     // coarse cells per column (AFH_RSTR_K=2|4|8 at run time)
  int res_k = AFH_RES_K;       // residual cells per column (AFH_RES_K=2|4|8 at run time)
  int prolong_k = 4;           // prolongation cells per column (AFH_PROLONG_K=2|4|8)
  int rstr_bs = 256;           // k_rstr_fas_col workgroup size
  int wave_cells = CS_WAVE_CELLS;
  // AFH_COARSE_DIRECT: eigenvectors Q and Q^T per dim, eigenvalues, work
  double *d_q[3] = {nullptr, nullptr, nullptr}, *d_qt[3] = {nullptr, nullptr, nullptr};
  double *d_e[3] = {nullptr, nullptr, nullptr};
  double *w1 = nullptr, *w2 = nullptr;
  int q_bc[6] = {0, 0, 0, 0, 0, 0};
  double *alt = nullptr;  // spare image of phi (all boxes) for the ping-pong
  // a spare image of its own (afh_photoi_helmh_compute's concurrent modes):
  // t->alt and alt point to it while this multigrid's work is issued
  double *alt_priv = nullptr;
  // electrode boxes (afh_mg_set_box_stencil / afh_mg_set_box_lsf): device
  // arrays per box id (null: none), their device pointer tables, and the
  // level lists split into constant- and variable-stencil boxes
  std::vector<double *> h_vp, h_bp, h_dd, h_bv;
  std::vector<int32_t *> h_ix;
  std::vector<int> h_lsf_n;
  double **d_vp = nullptr, **d_bp = nullptr, **d_dd = nullptr, **d_bv = nullptr;
  int32_t **d_ix = nullptr;
  int *d_lsf_n = nullptr;
  int i_lsf = 0;
  bool var_dirty = false, any_var = false, any_lsf = false;
  // V-cycles captured as hipGraphs (launch amortisation), one per (highest
  // level, set_residual, max|res|) variant; AFH_GRAPHS=0 disables them
  struct Graph {
    hipGraphExec_t exec = nullptr;
    uint64_t meth_gen = 0;
    bool warm = false;  // one eager call done (tables built, spare image allocated)
    // sharded (a hook): the V-cycle as segments between its exchanges, each
    // replayed as a graph, the exchange (ops[k]) run after segs[k]
    std::vector<hipGraphExec_t> segs;
    std::vector<std::array<int32_t, 4>> ops;
    bool eager_only = false;  // the recording met a reduction
    void release() {
      if (exec) hipGraphExecDestroy(exec);
      for (hipGraphExec_t s : segs)
        if (s) hipGraphExecDestroy(s);
      exec = nullptr;
      segs.clear();
      ops.clear();
    }
  };
  std::map<int, Graph> graphs;
  bool use_graphs = true;
  bool seg_graphs = true;  // sharded V-cycles as segment graphs (false: eager)
  int64_t n_replays = 0, n_seg_replays = 0;  // afh_mg_graph_stats
  std::vector<char> lvl_var;  // level has variable-stencil boxes
  LevelList ids_c, ids_v, leaves_c, leaves_v, parents_c, parents_v, lsf_leaves;
  double *cs_old = nullptr;   // level-1 electrode solve: previous phi
  // AFH_CS_ELEC_DIRECT (default on): the one-box electrode level-1 solve as
  // x = A^-1 ((rhs + bcc) - g) (afh_cs_direct.h); host copy of the level-1
  // box's stencil, the device inverse and g, and what they were built from
  bool csd_on = true, csd_ok = false;
  std::vector<double> h_v1;
  int h_v1_id = 0;
  uint64_t v1_gen = 1, csd_v_gen = 0, csd_meth_gen = UINT64_MAX;
  double *d_csd_ainv = nullptr, *d_csd_g = nullptr;
  // afh_mg_set_gradient_output: |E| (cc variable grad_iv, factor grad_fac)
  // from the final residual pass; the generations of phi and |E| it left
  // them at (afh_mg_compute_phi_gradient then skips its own pass)
  int grad_iv = 0;
  double grad_fac = -1.0;
  uint64_t grad_phi_gen = UINT64_MAX, grad_norm_gen = UINT64_MAX;
  // AFH_COARSE_PFMG (afh_pfmg.h, k_cs_pfmg): host copies of the level-1
  // boxes' electrode stencils; the folded level-1 operator the hierarchy was
  // built from and the (v1_gen, meth_gen) it was checked at; device levels,
  // operators (SoA per level), weights, boundary fold, level-set terms
  std::map<int, std::vector<double>> h_vl1;
  std::vector<double> pf_a7;
  uint64_t pf_v1_gen = 0, pf_meth_gen = UINT64_MAX;
  int pf_nl = 0, pf_np = 0, pf_lds = 0, pf_wave = 0;
  bool pf_stage = false;
  PfLvl *d_pf_lvl = nullptr;
  double *d_pf_A = nullptr, *d_pf_P = nullptr, *d_pf_b2r = nullptr, *d_pf_x = nullptr;
  uint8_t *d_pf_fmask = nullptr;
  const double **d_pf_vbc = nullptr;
};

// (diag, 1/diag) of the folded operator per MG level and boundary class, in
// the order of oracle/c/afo.c cs_build_table.
static int32_t build_table(afh_mg *mg) {
  const afh_bc *bc = mg->t->meth[mg->d.i_phi].bc;
  CsParams &P = mg->P;
  mg->h_dtab.assign((size_t)MAXMG * 64 * 2, 0.0);
  for (int m = 0; m < P.n_mg; m++)
    for (int c = 0; c < 64; c++) {
      double d = P.cdiag[m];
      for (int nb = 1; nb <= 6; nb++) {
        const int dd = (nb - 1) >> 1;
        const bool low = ((nb - 1) & 1) == 0;
        const int at = low ? (c >> (2 * dd)) & 1 : (c >> (2 * dd + 1)) & 1;
        if (!at) continue;
        if (bc[nb - 1].type == AFH_BC_DIRICHLET) d = d - P.hc[m][dd];
        else d = d + P.hc[m][dd];
      }
      mg->h_dtab[(m * 64 + c) * 2] = d;
      mg->h_dtab[(m * 64 + c) * 2 + 1] = 1 / d;
    }
  for (int q = 0; q < 6; q++) mg->tab_bc[q] = bc[q].type;
  AFH_HIP(hipStreamSynchronize(mg->t->stream));
  AFH_HIP(hipMemcpy(mg->d_dtab, mg->h_dtab.data(),
                    mg->h_dtab.size() * sizeof(double), hipMemcpyHostToDevice));
  P.dtab = mg->d_dtab;
  return AFH_OK;
}

// AFH_COARSE_DIRECT tables: the folded 1-D operator of each dimension is
// h tridiag(1, -2, 1) with end diagonals -h (Neumann) / -3h (Dirichlet),
// diagonalised by a cosine / sine basis; same formula and operation order
// as oracle/c/afo.c afo_cs_direct_tables.
static void cs_direct_tables(int n, int bc_lo, int bc_hi, double h, double *q,
                             double *e) {
  const int dlo = bc_lo == AFH_BC_DIRICHLET, dhi = bc_hi == AFH_BC_DIRICHLET;
  const double pi = 3.14159265358979323846;
  for (int p = 0; p < n; p++) {
    double th;
    if (dlo == dhi) th = pi * (p + dlo) / n;
    else th = pi * (p + 0.5) / n;
    double nrm2 = 0.0;
    for (int i = 0; i < n; i++) {
      double v = dlo ? sin(th * (i + 0.5)) : cos(th * (i + 0.5));
      q[i * n + p] = v;
      nrm2 = nrm2 + v * v;
    }
    const double inv = 1 / sqrt(nrm2);
    for (int i = 0; i < n; i++) q[i * n + p] = q[i * n + p] * inv;
    e[p] = h * (2 * cos(th) - 2);
  }
}

static int32_t build_direct(afh_mg *mg) {
  const afh_bc *bc = mg->t->meth[mg->d.i_phi].bc;
  AFH_HIP(hipStreamSynchronize(mg->t->stream));
  for (int d = 0; d < 3; d++) {
    const int n = mg->P.dims[0][d];
    std::vector<double> q((size_t)n * n), qt((size_t)n * n), e(n);
    cs_direct_tables(n, bc[2 * d].type, bc[2 * d + 1].type, mg->P.hc[0][d],
                     q.data(), e.data());
    for (int a = 0; a < n; a++)
      for (int b = 0; b < n; b++) qt[(size_t)a * n + b] = q[(size_t)b * n + a];
    AFH_HIP(hipMemcpy(mg->d_q[d], q.data(), sizeof(double) * n * n,
                      hipMemcpyHostToDevice));
    AFH_HIP(hipMemcpy(mg->d_qt[d], qt.data(), sizeof(double) * n * n,
                      hipMemcpyHostToDevice));
    AFH_HIP(hipMemcpy(mg->d_e[d], e.data(), sizeof(double) * n,
                      hipMemcpyHostToDevice));
  }
  for (int q = 0; q < 6; q++) mg->q_bc[q] = bc[q].type;
  return AFH_OK;
}

static bool fused_nc_ok(int nc) {
  return nc == 4 || nc == 8 || nc == 16 || nc == 32 || nc == 64;
}

static inline dim3 blocks1(size_t n, int bs = 256) {
  return dim3((unsigned)((n + bs - 1) / bs));
}

extern "C" {

int32_t afh_mg_create(afh_tree *t, const afh_mg_desc *d, afh_mg **out) {
  if (!d || !out) return set_error(AFH_ERR_ARG, "afh_mg_create: null");
  AFH_LIVE(t, "afh_mg_create");
  if (d->i_phi < 1 || d->i_phi > t->nvc || d->i_rhs < 1 || d->i_rhs > t->nvc ||
      d->i_tmp < 1 || d->i_tmp > t->nvc)
    return set_error(AFH_ERR_ARG, "afh_mg_create: bad variable index");
  if (!t->meth[d->i_phi].set)
    return set_error(AFH_ERR_STATE, "set cc methods (bc) for phi first");
  if (!(d->coarse_mode == AFH_COARSE_DIRECT ||
        ((d->coarse_mode == AFH_COARSE_CYCLES || d->coarse_mode == AFH_COARSE_PFMG) &&
         d->coarse_cycles >= 1)))
    return set_error(AFH_ERR_UNSUPPORTED, "coarse solver mode");
  if (!(d->coarse_tol >= 0.0))
    return set_error(AFH_ERR_ARG, "afh_mg_create: coarse_tol %g", d->coarse_tol);
  afh_mg *mg = new afh_mg();
  mg->t = t;
  mg->d = *d;
  mg->h_vp.assign(t->nb, nullptr), mg->h_bp.assign(t->nb, nullptr);
  mg->h_dd.assign(t->nb, nullptr), mg->h_bv.assign(t->nb, nullptr);
  mg->h_ix.assign(t->nb, nullptr), mg->h_lsf_n.assign(t->nb, 0);
  // mg_box_lpl_stencil: c(2:7) = 1/dr^2, c(1) = -sum(c(2:)) - lambda
  mg->lvl_c.resize(t->nlvl);
  for (int l = 1; l <= t->nlvl; l++) {
    // the level's spacing over the whole topology (a rank of a sharded tree
    // may compute no box of a level)
    const double *dr = &t->lvl_dr[3 * (l - 1)];
    Coef &c = mg->lvl_c[l - 1];
    for (int q = 0; q < 3; q++) {
      double inv = 1 / (dr[q] * dr[q]);
      c.c[1 + 2 * q] = inv;
      c.c[2 + 2 * q] = inv;
    }
    double s = c.c[1];
    for (int q = 2; q < 7; q++) s = s + c.c[q];
    c.c[0] = -s - d->helmholtz_lambda;
  }
  AFH_HIP(hipMalloc(&mg->d_lvl_c, sizeof(Coef) * t->nlvl));
  AFH_HIP(hipMemcpy(mg->d_lvl_c, mg->lvl_c.data(), sizeof(Coef) * t->nlvl,
                    hipMemcpyHostToDevice));
  // coarse hierarchy (same rule as oracle/c/afo.c afo_mg_create)
  CsParams &P = mg->P;
  memset(&P, 0, sizeof P);
  int m = 0;
  for (int q = 0; q < 3; q++) {
    P.dims[0][q] = t->cgs[q];
    P.hc[0][q] = mg->lvl_c[0].c[1 + 2 * q];
  }
  P.cdiag[0] = mg->lvl_c[0].c[0];
  for (;;) {
    int *n = P.dims[m];
    bool ok = (n[0] % 2 == 0) && (n[1] % 2 == 0) && (n[2] % 2 == 0) &&
              n[0] >= 4 && n[1] >= 4 && n[2] >= 4 && m < MAXMG - 1;
    if (!ok) break;
    for (int q = 0; q < 3; q++) {
      P.dims[m + 1][q] = n[q] / 2;
      P.hc[m + 1][q] = 0.25 * P.hc[m][q];
    }
    const double *h = P.hc[m + 1];
    P.cdiag[m + 1] = -(h[0] + h[0] + h[1] + h[1] + h[2] + h[2]) -
                     d->helmholtz_lambda;
    m++;
  }
  P.n_mg = m + 1;
  mg->small_from = P.n_mg - 1;
  while (mg->small_from > 0) {
    const int *n = P.dims[mg->small_from - 1];
    if ((long)n[0] * n[1] * n[2] > CS_SMALL_CELLS) break;
    mg->small_from--;
  }
  mg->small_lds = 0;
  for (int q = 0; q < P.n_mg; q++) {
    P.halo[q] = 1;
    const int nx = P.dims[q][0], ny = P.dims[q][1];
    const bool p2 = nx > 0 && ny > 0 && (nx & (nx - 1)) == 0 && (ny & (ny - 1)) == 0;
    P.lg[q] = p2 ? (__builtin_ctz(nx) | (__builtin_ctz(ny) << 8)) : -1;
    if (q >= mg->small_from)
      mg->small_lds += 2 * sizeof(double) * (size_t)P.dims[q][0] * P.dims[q][1] *
                       P.dims[q][2];
  }
  if (mg->small_lds + sizeof(CsParams) + MAXMG * 128 * sizeof(double) > 160 * 1024)
    return set_error(AFH_ERR_UNSUPPORTED, "coarse-solver LDS levels too large");
  AFH_HIP(raise_dyn_lds((const void *)k_cs_small, (int)mg->small_lds));
  AFH_HIP(hipMalloc(&mg->d_dtab, (size_t)MAXMG * 64 * 2 * sizeof(double)));
  if (int32_t e = build_table(mg)) return e;
  // AFH_GSRB_FUSED_MIN_BOXES: smallest level (in boxes) smoothed with the
  // fused red-black kernel; 0 disables it
  if (const char *env = getenv("AFH_RCCL_CAPTURE")) mg->rccl_capture = atoi(env) != 0;
  if (const char *env = getenv("AFH_GSRB_FUSED_MIN_BOXES"))
    mg->fused_min = atoi(env);
  else if (fused_nc_ok(t->nc))
    // whole boxes from 256 boxes (a workgroup per CU), NC/4-row tiles from
    // 64 boxes (NC >= 32). Boxes up to 16^3 (k_gsrb_pair_box) fuse on every
    // level: the small levels are launch-bound (S1 0.768 -> 0.737 ms/step,
    // S3 2.57 -> 2.54, scripts/env_bench_ab.sh); bitwise the split form
    // (test_3d every row, scripts/rtest_determinism.py)
    mg->fused_min = t->nc >= 32 ? 64 : (t->nc <= 16 && mg->pair_box ? 1 : 256);
  if (const char *env = getenv("AFH_GSRB_TILES")) mg->force_tiles = atoi(env) != 0;
  if (const char *env = getenv("AFH_GRAPHS")) mg->use_graphs = atoi(env) != 0;
  if (const char *env = getenv("AFH_RSTR_COL")) mg->rstr_col = atoi(env) != 0;
  if (const char *env = getenv("AFH_RSTR_K")) {
    const int k = atoi(env);
    mg->rstr_k = k == 8 ? 8 : k == 4 ? 4 : 2;
  }
  if (const char *env = getenv("AFH_RES_K"))
    mg->res_k = atoi(env) == 8 ? 8 : atoi(env) == 2 ? 2 : 4;
  if (const char *env = getenv("AFH_PROLONG_K"))
    mg->prolong_k = atoi(env) == 8 ? 8 : atoi(env) == 2 ? 2 : 4;
  if (const char *env = getenv("AFH_CS_ELEC_DIRECT")) mg->csd_on = atoi(env) != 0;
  if (const char *env = getenv("AFH_CS_DIRECT_SMALL")) mg->cs_direct_small = atoi(env) != 0;
  if (const char *env = getenv("AFH_PAIR_PUSH")) mg->pair_push = atoi(env) != 0;
  if (const char *env = getenv("AFH_PROLONG_PUSH")) mg->prolong_push = atoi(env) != 0;
  if (const char *env = getenv("AFH_RSTR_PUSH")) mg->rstr_push = atoi(env) != 0;
  AFH_HIP(hipMalloc(&mg->cs_iters, sizeof(int)));
  AFH_HIP(hipMalloc(&mg->d_cycles, sizeof(int)));
  if (fused_nc_ok(t->nc) && mg->fused_min > 0) {
    bool any = false;
    for (int l = 2; l <= t->nlvl; l++) any |= t->lvl_total[l - 1] >= mg->fused_min;
    if (any) {
      // one spare image per tree: the level fills after a pair fill t->alt
      if (!t->alt) {
        if (int32_t e2 = pool_alloc((void **)&t->alt_base,
                                    (size_t)t->nb * t->bsz * sizeof(double), "alt"))
          return e2;
        t->alt = t->alt_base;
        AFH_HIP(hipMemsetAsync(t->alt, 0, (size_t)t->nb * t->bsz * sizeof(double),
                               t->stream));
      }
      t->alt_refs++;
      mg->alt = t->alt;
    }
  }
  for (int q = 0; q < P.n_mg; q++) {
    size_t n = (size_t)(P.dims[q][0] + 2) * (P.dims[q][1] + 2) * (P.dims[q][2] + 2);
    AFH_HIP(hipMalloc(&P.u[q], n * sizeof(double)));
    AFH_HIP(hipMalloc(&P.f[q], n * sizeof(double)));
    AFH_HIP(hipMemsetAsync(P.u[q], 0, n * sizeof(double), t->stream));
    AFH_HIP(hipMemsetAsync(P.f[q], 0, n * sizeof(double), t->stream));
  }
  if (d->coarse_mode == AFH_COARSE_DIRECT) {
    const size_t n = (size_t)P.dims[0][0] * P.dims[0][1] * P.dims[0][2];
    for (int q = 0; q < 3; q++) {
      const size_t nd = P.dims[0][q];
      AFH_HIP(hipMalloc(&mg->d_q[q], nd * nd * sizeof(double)));
      AFH_HIP(hipMalloc(&mg->d_qt[q], nd * nd * sizeof(double)));
      AFH_HIP(hipMalloc(&mg->d_e[q], nd * sizeof(double)));
    }
    AFH_HIP(hipMalloc(&mg->w1, n * sizeof(double)));
    AFH_HIP(hipMalloc(&mg->w2, n * sizeof(double)));
    if (int32_t e = build_direct(mg)) return e;
  }
  AFH_HIP(hipStreamSynchronize(t->stream));
  *out = mg;
  return AFH_OK;
}

int32_t afh_mg_destroy(afh_mg *mg) {
  if (!mg) return AFH_OK;
  hipStreamSynchronize(mg->t->stream);
  for (auto &g : mg->graphs) g.second.release();
  for (int q = 0; q < mg->P.n_mg; q++) {
    hipFree(mg->P.u[q]);
    hipFree(mg->P.f[q]);
  }
  hipFree(mg->d_dtab);
  for (int q = 0; q < 3; q++) hipFree(mg->d_q[q]), hipFree(mg->d_qt[q]), hipFree(mg->d_e[q]);
  hipFree(mg->w1);
  hipFree(mg->w2);
  hipFree(mg->d_csd_ainv), hipFree(mg->d_csd_g);
  hipFree(mg->d_pf_lvl), hipFree(mg->d_pf_A), hipFree(mg->d_pf_P), hipFree(mg->d_pf_b2r);
  hipFree(mg->d_pf_x), hipFree(mg->d_pf_fmask), hipFree((void *)mg->d_pf_vbc);
  hipFree(mg->alt_priv);
  if (mg->alt && --mg->t->alt_refs == 0) {
    hipFree(mg->t->alt_base);
    mg->t->alt = mg->t->alt_base = nullptr;
  }
  for (auto *v : {&mg->h_vp, &mg->h_bp, &mg->h_dd, &mg->h_bv})
    for (double *q : *v) hipFree(q);
  for (int32_t *q : mg->h_ix) hipFree(q);
  hipFree(mg->d_vp), hipFree(mg->d_bp), hipFree(mg->d_dd), hipFree(mg->d_bv);
  hipFree(mg->d_ix), hipFree(mg->d_lsf_n), hipFree(mg->cs_old);
  hipFree(mg->cs_iters);
  hipFree(mg->d_cycles);
  hipFree(mg->d_norm);
  hipFree(mg->d_lvl_c);
  for (LevelList *L : {&mg->ids_c, &mg->ids_v, &mg->leaves_c, &mg->leaves_v,
                       &mg->parents_c, &mg->parents_v, &mg->lsf_leaves})
    hipFree(L->d);
  delete mg;
  return AFH_OK;
}

}  // extern "C"

// A launch whose start / end events are written by the dispatch itself
// (hipExtLaunchKernelGGL: the clock of rocprofv3's kernel trace, no barrier
// packets around the kernel) when e0 is set; a plain launch otherwise.
template <typename K, typename... A>
static void launch_ev(K k, hipEvent_t e0, hipEvent_t e1, dim3 g, dim3 b,
                      hipStream_t st, A... a) {
  if (e0)
    hipExtLaunchKernelGGL(k, g, b, 0, st, e0, e1, 0, a...);
  else
    hipLaunchKernelGGL(k, g, b, 0, st, a...);
}

template <int NC, int TJ>
static void launch_pair_t(afh_mg *mg, int lvl, const double *src, double *dst,
                          const Coef &cf, double inv_c1, hipEvent_t e0, hipEvent_t e1) {
  afh_tree *t = mg->t;
  launch_ev((k_gsrb_pair<NC, TJ>), e0, e1,
                     dim3(t->ids.n(lvl) * RbGeom<NC, TJ>::NTILE),
                     dim3(RbGeom<NC, TJ>::NT), t->stream, src, dst,
                     t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_phi), t->d_boxes,
                     t->ids.at(lvl), t->bsz, cf, inv_c1,
                     t->gc_args(mg->d.i_phi));
}

// whole boxes per workgroup, or NC/4-row tiles (NC >= 32) on levels of
// 64..255 boxes, which fill the CUs with 4 tiles per box
// (AFH_GSRB_TILES=1: tiles on every level, for tests)
// The geometry follows the boxes THIS rank smooths (the variants are bitwise
// alike and exchange the same data, so ranks need not agree on it): a rank
// of a sharded tree with fewer than 256 boxes of a level (S1-64 on 8 GPUs:
// 64 leaf boxes each) splits them, instead of leaving most CUs idle.
static bool pair_tiles(const afh_mg *mg, int lvl) {
  const int n = mg->t->ids.n(lvl);
  return mg->t->nc >= 32 && (mg->force_tiles || n < mg->tiles_min);
}

template <int NC, int TJ, int DEPTH, int KS = 1>
static void launch_pair2(afh_mg *mg, int lvl, const double *src, double *dst,
                         const Coef &cf, double inv_c1, hipEvent_t e0, hipEvent_t e1) {
  afh_tree *t = mg->t;
  launch_ev((k_gsrb_pair2<NC, TJ, DEPTH, KS>), e0, e1,
            dim3(t->ids.n(lvl) * RbPar<NC, TJ>::NTILE * KS), dim3(RbPar<NC, TJ>::NT),
            t->stream, src, dst, t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_phi), t->d_boxes,
            t->ids.at(lvl), t->bsz, cf, inv_c1, t->gc_args(mg->d.i_phi));
}

// the small-box pair fills the level's faces itself (k_gsrb_pair_box PUSH)
// unless the tree is sharded (a replica's ghosts are its owner's to fill,
// through the exchange hooks) or AFH_PAIR_PUSH=0
static bool pair_push(const afh_mg *mg) {
  return mg->pair_push && mg->pair_box && mg->t->nc <= 16 && !mg->t->hook;
}

// pend: rhs round trips of earlier pairs of the leg not yet stored (read
// through by the variable small-box pair); last: the leg's last pair, after
// which they are stored with its own (the other pair forms store their own)
template <int NC>
static void launch_pair(afh_mg *mg, int lvl, const double *src, double *dst,
                        const Coef &cf, double inv_c1, hipEvent_t e0, hipEvent_t e1,
                        int pend = 0, bool last = true) {
  afh_tree *t = mg->t;
  if (t->ids.n(lvl) == 0) return;
  if constexpr (NC <= 16) {
    if (mg->pair_box) {
      const bool var = mg->any_var && mg->lvl_var[lvl - 1];
      auto go = [&](auto kern) {
        launch_ev(kern, e0, e1, dim3(t->ids.n(lvl)), dim3(RbBox<NC>::NT), t->stream, src, dst,
                  t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_phi), t->d_boxes, t->ids.at(lvl),
                  t->bsz, cf, inv_c1, t->gc_args(mg->d.i_phi),
                  (const double *const *)mg->d_vp, (const double *const *)mg->d_bp,
                  var ? pend : 0);
      };
      if (pair_push(mg))
        var ? go(k_gsrb_pair_box<NC, true, true>) : go(k_gsrb_pair_box<NC, true>);
      else
        var ? go(k_gsrb_pair_box<NC, false, true>) : go(k_gsrb_pair_box<NC>);
      if (var && mg->ids_v.n(lvl) && last) {
        // the half-sweeps' rhs round trips on the electrode boxes: two per
        // pair, this pair's and the pending ones, in one launch (round 6)
        const int nc = t->nc;
        hipLaunchKernelGGL(k_rhs_roundtrip, dim3((nc * nc * nc + 255) / 256, mg->ids_v.n(lvl)),
                           dim3(256), 0, t->stream, t->ccv(mg->d.i_rhs), mg->ids_v.at(lvl),
                           nc, t->bsz, (const double *const *)mg->d_bp, pend + 2);
        // (the caller's launch check covers it)
      }
      return;
    }
  }
  if constexpr (NC >= 32) {
    if (pair_tiles(mg, lvl)) {
      // too few boxes for the chip: 64^3 splits the march over k, 32^3 runs
      // quarter-box tiles. A rank's share of a sharded level can be a few
      // boxes (S1-64's level 3 on 8 ranks: 8): 16 chunks of 4 planes then
      // (round 6; bitwise any split)
      if constexpr (NC == 64) {
        if (t->ids.n(lvl) <= 16)
          return launch_pair2<NC, NC, 1, 16>(mg, lvl, src, dst, cf, inv_c1, e0, e1);
        return launch_pair2<NC, NC, 1, 4>(mg, lvl, src, dst, cf, inv_c1, e0, e1);
      }
      return launch_pair2<NC, NC / 4, 2>(mg, lvl, src, dst, cf, inv_c1, e0, e1);
    }
  }
  if constexpr (NC >= 16) {
    if constexpr (NC == 64) return launch_pair2<NC, NC, 1>(mg, lvl, src, dst, cf, inv_c1, e0, e1);
    return launch_pair2<NC, NC, 2>(mg, lvl, src, dst, cf, inv_c1, e0, e1);
  }
  launch_pair_t<NC, NC>(mg, lvl, src, dst, cf, inv_c1, e0, e1);
}

extern "C" {

// gsrb_boxes smooths level lvl with the fused pair kernel (same answer on
// every rank of a sharded tree: decided on the level's total box count)
static bool fused_level(const afh_mg *mg, int lvl) {
  // electrode stencils: the small-box pair has a variable form (VAR)
  if (mg->any_var && mg->lvl_var[lvl - 1] && !(mg->pair_box && mg->t->nc <= 16))
    return false;
  return mg->alt && mg->t->lvl_total[lvl - 1] >= mg->fused_min;
}

// Device tables and split level lists after afh_mg_set_box_stencil /
// afh_mg_set_box_lsf changed them
static int32_t prepare_var(afh_mg *mg) {
  if (!mg->var_dirty) return AFH_OK;
  mg->var_dirty = false;
  for (auto &g : mg->graphs) g.second.release();
  mg->graphs.clear();
  afh_tree *t = mg->t;
  const int nb = t->nb, nl = t->nlvl;
  auto table = [&](auto **d, const auto &h) -> int32_t {
    if (!*d) AFH_HIP(hipMalloc(d, sizeof(h[0]) * nb));
    AFH_HIP(hipMemcpy(*d, h.data(), sizeof(h[0]) * nb, hipMemcpyHostToDevice));
    return AFH_OK;
  };
  int32_t e;
  if ((e = table(&mg->d_vp, mg->h_vp)) || (e = table(&mg->d_bp, mg->h_bp)) ||
      (e = table(&mg->d_dd, mg->h_dd)) || (e = table(&mg->d_bv, mg->h_bv)) ||
      (e = table(&mg->d_ix, mg->h_ix)) || (e = table(&mg->d_lsf_n, mg->h_lsf_n)))
    return e;
  mg->any_var = mg->any_lsf = false;
  mg->lvl_var.assign(nl, 0);
  for (int q = 0; q < nb; q++) {
    if (mg->h_vp[q]) mg->any_var = true, mg->lvl_var[t->boxes[q].lvl - 1] = 1;
    if (mg->h_lsf_n[q]) mg->any_lsf = true;
  }
  auto split = [&](const std::vector<std::vector<int32_t>> &src, LevelList &c,
                   LevelList &v) -> int32_t {
    std::vector<std::vector<int32_t>> lc(nl), lv(nl);
    for (int l = 0; l < nl; l++)
      for (int32_t id : src[l]) (mg->h_vp[id - 1] ? lv : lc)[l].push_back(id);
    int32_t e2;
    if ((e2 = upload_list(t, c, lc)) || (e2 = upload_list(t, v, lv))) return e2;
    return AFH_OK;
  };
  if ((e = split(t->h_ids, mg->ids_c, mg->ids_v)) ||
      (e = split(t->h_leaves, mg->leaves_c, mg->leaves_v)) ||
      (e = split(t->h_parents, mg->parents_c, mg->parents_v)))
    return e;
  std::vector<std::vector<int32_t>> ll(nl);
  for (int l = 0; l < nl; l++)
    for (int32_t id : t->h_leaves[l])
      if (mg->h_lsf_n[id - 1]) ll[l].push_back(id);
  return upload_list(t, mg->lsf_leaves, ll);
}

// the constant-stencil part of a level list (the whole list without
// electrode boxes)
static const LevelList &cst(const afh_mg *mg, const LevelList &all,
                            const LevelList &c) {
  return mg->any_var ? c : all;
}

static int32_t gsrb_half(afh_mg *mg, int lvl, int n, bool corners) {
  afh_tree *t = mg->t;
  const LevelList &L = cst(mg, t->ids, mg->ids_c);
  const int nid = L.n(lvl), nc = t->nc;
  const Coef cf = mg->lvl_c[lvl - 1];
  const int cells = nc * nc * nc / 2;
  if (nid) {
    prof_begin(t, AFH_PROF_GSRB);
    hipLaunchKernelGGL(k_gsrb, dim3((cells + 255) / 256, nid), dim3(256), 0,
                       t->stream, t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs),
                       L.at(lvl), nc, t->bsz, cf, 1 / cf.c[0], n);
    // read phi (all), rhs (half), write phi (half) = 16 B/cell
    prof_end(t, AFH_PROF_GSRB, 16.0 * nc * nc * nc * nid);
    AFH_LAUNCH_CHECK("k_gsrb");
  }
  const int nv = mg->any_var ? mg->ids_v.n(lvl) : 0;
  if (nv) {
    hipLaunchKernelGGL(k_gsrb_v, dim3((nc * nc * nc + 255) / 256, nv), dim3(256),
                       0, t->stream, t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs),
                       mg->ids_v.at(lvl), nc, t->bsz, mg->d_vp, mg->d_bp, n);
    AFH_LAUNCH_CHECK("k_gsrb_v");
  }
  // (a split half-sweep reads ghost cells only; a fused level's pair may
  // follow)
  return gc_lvl(t, lvl, mg->d.i_phi, corners, fused_level(mg, lvl), fused_level(mg, lvl) ? 2 : 1);
}

// gsrb_boxes (m_af_multigrid.f90:741-760): 2 n_cycle half-sweeps, each
// followed by a ghost fill of the level. On levels with enough boxes the
// pairs run fused (k_gsrb_pair), alternating phi -> alt -> phi; an odd
// number of pairs starts with one split pair.
static int32_t gsrb_boxes(afh_mg *mg, int lvl, bool up, bool stale_ghosts = false) {
  afh_tree *t = mg->t;
  const int n_cycle = up ? mg->d.n_cycle_up : mg->d.n_cycle_down;
  const int nid = t->ids.n(lvl), nc = t->nc;
  const Coef cf = mg->lvl_c[lvl - 1];
  const double inv_c1 = 1 / cf.c[0];
  // stale ghost cells on entry: the split half-sweeps, as the reference
  const bool fused = fused_level(mg, lvl) && !stale_ghosts;
  int n0 = 1;
  if (fused && (n_cycle & 1)) {
    if (int32_t e = gsrb_half(mg, lvl, 1, false)) return e;
    if (int32_t e = gsrb_half(mg, lvl, 2, up && n_cycle == 1)) return e;
    n0 = 2;
  }
  if (!fused) {
    for (int n = 1; n <= 2 * n_cycle; n++)
      if (int32_t e = gsrb_half(mg, lvl, n, up && n == 2 * n_cycle)) return e;
    return AFH_OK;
  }
  double *phi = t->ccv(mg->d.i_phi);
  const afh::GcArgs ga = t->gc_args(mg->d.i_phi);
  t->alt_of = mg->d.i_phi;
  // the pair recomputes neighbours' red boundary cells from their rhs; the
  // up leg's pairs read the rhs the down leg's exchange brought (nothing
  // writes a level's rhs between its two legs)
  if ((int)mg->rhs_halo.size() < t->nlvl) mg->rhs_halo.assign(t->nlvl, 0);
  // (one layer: the pair recomputes the neighbours' cells next to the box,
  // whose rhs is all it reads of theirs)
  if (!(up && mg->rhs_halo[lvl - 1]))
    if (int32_t e = call_hook(t, AFH_HOOK_HALO, lvl, mg->d.i_rhs, nullptr, 1)) return e;
  mg->rhs_halo[lvl - 1] = !up;
  for (int n = n0; n <= n_cycle; n++) {
    const bool to_alt = ((n - n0) & 1) == 0;
    const double *src = to_alt ? phi : mg->alt;
    double *dst = to_alt ? mg->alt : phi;
    const int dst_iv = to_alt ? 0 : mg->d.i_phi;
    // the bench's roofline times the big levels (>= 256 boxes, or tiles);
    // small-level pairs of small boxes are launch-bound and not timed
    const int pclass = (nc >= 32 && pair_tiles(mg, lvl)) ? AFH_PROF_GSRB_PAIR_TILED
                       : (nc >= 32 || t->lvl_total[lvl - 1] >= 256) ? AFH_PROF_GSRB_PAIR
                                                                     : -1;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = prof_ext(t, pclass, e0, e1);
    // (the variable small-box pair: the leg's rhs round trips stored once,
    // after its last pair; nothing else reads the rhs in between)
    const int pend = 2 * (n - n0);
    const bool last = n == n_cycle;
    switch (nc) {
    case 4: launch_pair<4>(mg, lvl, src, dst, cf, inv_c1, e0, e1, pend, last); break;
    case 8: launch_pair<8>(mg, lvl, src, dst, cf, inv_c1, e0, e1, pend, last); break;
    case 16: launch_pair<16>(mg, lvl, src, dst, cf, inv_c1, e0, e1, pend, last); break;
    case 32: launch_pair<32>(mg, lvl, src, dst, cf, inv_c1, e0, e1); break;
    default: launch_pair<64>(mg, lvl, src, dst, cf, inv_c1, e0, e1); break;
    }
    // a red+black pair reads phi and rhs and writes phi
    // once = 24 B/cell
    if (timed) prof_count(t, 24.0 * nc * nc * nc * nid);
    AFH_LAUNCH_CHECK("k_gsrb_pair");
    (void)dst;
    if (pair_push(mg)) {
      // the pair filled the faces; edges and corners on the leg's last pair
      if (up && n == n_cycle)
        if (int32_t e = gc_lvl_corners(t, lvl, dst_iv)) return e;
    } else if (int32_t e = gc_lvl_var(t, lvl, dst_iv, phi, ga, up && n == n_cycle, true,
                                      // another pair reads the replicas'
                                      // second layer: the leg's next pair, or
                                      // the next V-cycle's first on the
                                      // highest level (no fill between)
                                      n < n_cycle || (up && lvl == mg->vc_max_lvl) ? 2 : 1)) {
      return e;
    }
  }
  return AFH_OK;
}


// The restriction into level lvl-1 pushes that level's faces (k_rstr_box)
// and the parents' edges and corners come with their rhs (k_parent_rhs_box),
// instead of a full level fill between the two: small boxes smoothed by the
// pushing pair, no electrode stencils, and ghost cells valid on entry (the
// fill keeps the ghosts facing boxes the restriction does not change).
// AFH_RSTR_PUSH=0: off.
static bool rstr_push(const afh_mg *mg, int lvl, bool ghosts_valid) {
  const int nc = mg->t->nc;
  return ghosts_valid && mg->rstr_push && pair_push(mg) && !mg->any_var &&
         (nc == 4 || nc == 8 || nc == 16) && fused_level(mg, lvl - 1);
}

static int32_t update_coarse(afh_mg *mg, int lvl, bool ghosts_valid = false) {
  afh_tree *t = mg->t;
  const int nc = t->nc, hn = nc / 2;
  const LevelList &L = cst(mg, t->ids, mg->ids_c);
  const int nid = L.n(lvl);
  if (rstr_push(mg, lvl, ghosts_valid)) {
    const GcArgs ga = t->gc_args(mg->d.i_phi);
    const Coef cf = mg->lvl_c[lvl - 1];
    double *phi = t->ccv(mg->d.i_phi), *rhs = t->ccv(mg->d.i_rhs), *tmp = t->ccv(mg->d.i_tmp);
    if (nid) {
      if (nc == 4)
        hipLaunchKernelGGL(k_rstr_box<4>, dim3(nid), dim3(64), 0, t->stream, phi, rhs, tmp,
                           t->d_boxes, L.at(lvl), t->bsz, cf, ga);
      else if (nc == 8)
        hipLaunchKernelGGL(k_rstr_box<8>, dim3(nid), dim3(64), 0, t->stream, phi, rhs, tmp,
                           t->d_boxes, L.at(lvl), t->bsz, cf, ga);
      else
        hipLaunchKernelGGL(k_rstr_box<16>, dim3(nid), dim3(512), 0, t->stream, phi, rhs, tmp,
                           t->d_boxes, L.at(lvl), t->bsz, cf, ga);
      AFH_LAUNCH_CHECK("k_rstr_box");
    }
    const int np = t->parents.n(lvl - 1);
    if (np) {
      if (nc == 16)
        hipLaunchKernelGGL(k_parent_rhs_box<512>, dim3(np), dim3(512), 0, t->stream, phi, rhs,
                           tmp, t->d_boxes, t->parents.at(lvl - 1), nc, t->bsz,
                           mg->lvl_c[lvl - 2]);
      else
        hipLaunchKernelGGL(k_parent_rhs_box<256>, dim3(np), dim3(256), 0, t->stream, phi,
                           rhs, tmp, t->d_boxes, t->parents.at(lvl - 1), nc, t->bsz,
                           mg->lvl_c[lvl - 2]);
      AFH_LAUNCH_CHECK("k_parent_rhs_box");
    }
    return AFH_OK;
  }
  const double *fine = t->ccv(mg->d.i_phi);
  if (nid) {
    // column length (AFH_RSTR_K = 2, 4 or 8): a column reads 2K + 2 fine
    // planes for 2K; each doubling of K halves that excess at twice the
    // centre registers
    // (workgroup size AFH_RSTR_BS: with 128 the blocks of neighbouring
    // columns along k are 8 apart in dispatch order, i.e. on the same XCD,
    // whose L2 then holds the fine plane both read)
    const int RK = mg->rstr_k, BS = mg->rstr_bs;
    if (mg->rstr_col && RK == 8 && hn % 8 == 0)
      hipLaunchKernelGGL(k_rstr_fas_col<8>, dim3((hn * hn * (hn / 8) + BS - 1) / BS, nid),
                         dim3(BS), 0, t->stream, t->ccv(mg->d.i_phi),
                         t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), t->d_boxes,
                         L.at(lvl), nc, t->bsz, mg->lvl_c[lvl - 1], fine);
    else if (mg->rstr_col && RK >= 4 && hn % 4 == 0)
      hipLaunchKernelGGL(k_rstr_fas_col<4>, dim3((hn * hn * (hn / 4) + BS - 1) / BS, nid),
                         dim3(BS), 0, t->stream, t->ccv(mg->d.i_phi),
                         t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), t->d_boxes,
                         L.at(lvl), nc, t->bsz, mg->lvl_c[lvl - 1], fine);
    else if (mg->rstr_col && hn % 2 == 0)
      hipLaunchKernelGGL(k_rstr_fas_col<2>, dim3((hn * hn * (hn / 2) + BS - 1) / BS, nid),
                         dim3(BS), 0, t->stream, t->ccv(mg->d.i_phi),
                         t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), t->d_boxes,
                         L.at(lvl), nc, t->bsz, mg->lvl_c[lvl - 1], fine);
    else
      hipLaunchKernelGGL(k_rstr_fas, dim3((hn * hn * hn + 255) / 256, nid),
                         dim3(256), 0, t->stream, t->ccv(mg->d.i_phi),
                         t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), t->d_boxes,
                         L.at(lvl), nc, t->bsz, mg->lvl_c[lvl - 1]);
    AFH_LAUNCH_CHECK("k_rstr_fas");
  }
  const int nv = mg->any_var ? mg->ids_v.n(lvl) : 0;
  if (nv) {
    hipLaunchKernelGGL(k_rstr_fas_v, dim3((hn * hn * hn + 255) / 256, nv),
                       dim3(256), 0, t->stream, t->ccv(mg->d.i_phi),
                       t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), t->d_boxes,
                       mg->ids_v.at(lvl), nc, t->bsz, mg->d_vp, mg->d_bp);
    AFH_LAUNCH_CHECK("k_rstr_fas_v");
  }
  int32_t e;
  if ((e = call_hook(t, AFH_HOOK_RESTRICT, lvl, mg->d.i_phi)) ||
      (e = call_hook(t, AFH_HOOK_RESTRICT, lvl, mg->d.i_tmp)))
    return e;
  if ((e = gc_lvl(t, lvl - 1, mg->d.i_phi, 1, fused_level(mg, lvl - 1),
                  fused_level(mg, lvl - 1) ? 2 : 1)))
    return e;
  const LevelList &P = cst(mg, t->parents, mg->parents_c);
  const int np = P.n(lvl - 1);
  if (np) {
    hipLaunchKernelGGL(k_parent_rhs, dim3((unsigned)((t->bsz + 255) / 256), np),
                       dim3(256), 0, t->stream, t->ccv(mg->d.i_phi),
                       t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp),
                       P.at(lvl - 1), nc, t->bsz, mg->lvl_c[lvl - 2]);
    AFH_LAUNCH_CHECK("k_parent_rhs");
  }
  const int npv = mg->any_var ? mg->parents_v.n(lvl - 1) : 0;
  if (npv) {
    hipLaunchKernelGGL(k_parent_rhs_v, dim3((unsigned)((t->bsz + 255) / 256), npv),
                       dim3(256), 0, t->stream, t->ccv(mg->d.i_phi),
                       t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp),
                       mg->parents_v.at(lvl - 1), nc, t->bsz, mg->d_vp, mg->d_bp);
    AFH_LAUNCH_CHECK("k_parent_rhs_v");
  }
  return AFH_OK;
}

// the correction of level lvl also fills its faces (k_prolong_box): small
// boxes whose level the pushing pair smooths next (AFH_PROLONG_PUSH=0: off)
static bool prolong_push(const afh_mg *mg, int lvl) {
  const int nc = mg->t->nc;
  return mg->prolong_push && pair_push(mg) && (nc == 4 || nc == 8 || nc == 16) &&
         fused_level(mg, lvl);
}

static int32_t correct_children(afh_mg *mg, int lvl) {
  afh_tree *t = mg->t;
  const int np = t->parents.n(lvl - 1), nc = t->nc;
  if (np) {
    hipLaunchKernelGGL(k_corr_tmp, dim3((unsigned)((t->bsz + 255) / 256), np),
                       dim3(256), 0, t->stream, t->ccv(mg->d.i_phi),
                       t->ccv(mg->d.i_tmp), t->parents.at(lvl - 1), t->bsz);
    AFH_LAUNCH_CHECK("k_corr_tmp");
  }
  const int nid = t->ids.n(lvl);
  if (nid && prolong_push(mg, lvl)) {
    const GcArgs ga = t->gc_args(mg->d.i_phi);
    if (nc == 4)
      hipLaunchKernelGGL(k_prolong_box<4>, dim3(nid), dim3(RbBox<4>::NT), 0, t->stream,
                         t->ccv(mg->d.i_phi), t->ccv(mg->d.i_tmp), t->d_boxes, t->ids.at(lvl),
                         t->bsz, ga);
    else if (nc == 8)
      hipLaunchKernelGGL(k_prolong_box<8>, dim3(nid), dim3(RbBox<8>::NT), 0, t->stream,
                         t->ccv(mg->d.i_phi), t->ccv(mg->d.i_tmp), t->d_boxes, t->ids.at(lvl),
                         t->bsz, ga);
    else
      hipLaunchKernelGGL(k_prolong_box<16>, dim3(nid), dim3(RbBox<16>::NT), 0, t->stream,
                         t->ccv(mg->d.i_phi), t->ccv(mg->d.i_tmp), t->d_boxes, t->ids.at(lvl),
                         t->bsz, ga);
    AFH_LAUNCH_CHECK("k_prolong_box");
  } else if (nid) {
    double *fphi = t->ccv(mg->d.i_phi);
    // column length 4; AFH_PROLONG_K=8 where nc allows: the launch is
    // faster (195 against 223 us on S1-64) but the pair after it slower,
    // 13.32 against 12.57-12.60 ms per step (profiles/r03_ab_prolong_k.txt)
    const int want = mg->prolong_k;
    const int K = want == 8 && nc % 8 == 0 ? 8 : want >= 4 && nc % 4 == 0 ? 4 : 2;
    const dim3 grid((nc * nc * (nc / K) + 255) / 256, nid);
    if (K == 8)
      hipLaunchKernelGGL(k_prolong<8>, grid, dim3(256), 0, t->stream,
                         fphi, t->ccv(mg->d.i_tmp), t->d_boxes,
                         t->ids.at(lvl), nc, t->bsz);
    else if (K == 4)
      hipLaunchKernelGGL(k_prolong<4>, grid, dim3(256), 0, t->stream,
                         fphi, t->ccv(mg->d.i_tmp), t->d_boxes,
                         t->ids.at(lvl), nc, t->bsz);
    else
      hipLaunchKernelGGL(k_prolong<2>, grid, dim3(256), 0, t->stream,
                         fphi, t->ccv(mg->d.i_tmp), t->d_boxes,
                         t->ids.at(lvl), nc, t->bsz);
    AFH_LAUNCH_CHECK("k_prolong");
  }
  return AFH_OK;
}

// Level-1 solve with electrode stencils (the C oracle's solve_coarse_gs,
// OUR algorithm; the reference hands the LSF stencils to HYPRE,
// m_coarse_solver.f90:286-338): red-black Gauss-Seidel pairs with each box's
// own stencil and a level ghost fill after each half-sweep until phi is
// stationary (max change <= 4 spacing(max |phi|), after at least 11 pairs),
// then the level's ghost cells with corners. One host check per pair: meant
// for the small coarse grids electrode runs use.
// The same iteration for a level 1 of one box with six physical faces (the
// usual electrode case: coarse grid = one box) in one workgroup: the box and
// its rhs in LDS, each pair = two k_gsrb_v half sweeps (rhs + bc_correction,
// parity update, rhs = (rhs + bc) - bc), each followed by the face fill of
// gc_face_nocopy's physical branch (no corners), then max |change| and
// max |phi| over the interior and the same stopping test -- all on the
// device, no host round trip per pair. Every wave leaves the loop at the
// same test (block-uniform), bounded by the host loop's 200000 pairs.
// Bitwise the launch-per-pair form.
extern "C++" {
template <int NC>
__global__ void __launch_bounds__(1024)
    k_cs_electrode(double *__restrict__ x, double *__restrict__ r,
                   const double *__restrict__ v, const double *__restrict__ b,
                   GcArgs ga, double dr0, double dr1, double dr2,
                   int *__restrict__ iters) {
  constexpr int NG = NC + 2, N3 = NC * NC * NC, G3 = NG * NG * NG;
  constexpr int SJ = NG, SK = NG * NG;
  __shared__ double X[G3], R[N3];
  __shared__ double s_d[16], s_m[16];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < G3; e += nt) X[e] = x[e];
  for (int e = tid; e < N3; e += nt) {
    const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
    R[e] = r[ix3(NG, i, j, k)];
  }
  __syncthreads();
  constexpr int CPT = (N3 + 1023) / 1024;  // cells per thread (<= 4 at NC 16)
  double old[CPT];
  int it;
  for (it = 1; it <= 200000; it++) {
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      const int e = tid + q * nt;
      if (e < N3) {
        const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
        old[q] = X[ix3(NG, i, j, k)];
      }
    }
    for (int n = 1; n <= 2; n++) {
      for (int e = tid; e < N3; e += nt) {
        const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
        const int c = ix3(NG, i, j, k);
        const double *w = v + 7 * (size_t)e;
        double r1 = R[e];
        if (b) r1 = r1 + b[e];
        if (((i + j + k + n) & 1) == 0)
          X[c] = (r1 - w[1] * X[c - 1] - w[2] * X[c + 1] - w[3] * X[c - SJ] -
                  w[4] * X[c + SJ] - w[5] * X[c - SK] - w[6] * X[c + SK]) /
                 w[0];
        if (b) R[e] = r1 - b[e];
      }
      __syncthreads();
      // face ghosts (physical boundaries; gc_face_nocopy_k, nb_id < 0)
      for (int e = tid; e < 6 * NC * NC; e += nt) {
        const int nb = e / (NC * NC) + 1, ab = e % (NC * NC);
        const int d = (nb - 1) >> 1;
        const bool low = ((nb - 1) & 1) == 0;
        const int ta = d == 0 ? 1 : 0, tb = d == 2 ? 1 : 2;
        int p[3], q1[3];
        p[ta] = ab % NC + 1;
        p[tb] = ab / NC + 1;
        p[d] = low ? 0 : NC + 1;
        q1[0] = p[0], q1[1] = p[1], q1[2] = p[2];
        q1[d] = low ? 1 : NC;
        const afh_bc bc = ga.bc[nb - 1];
        const double drd = d == 0 ? dr0 : d == 1 ? dr1 : dr2;
        double c0, c1;
        switch (bc.type) {
        case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; break;
        case AFH_BC_NEUMANN: c0 = drd * (low ? -1 : 1); c1 = 1; break;
        default: c0 = 1; c1 = 0; break;
        }
        X[ix3(NG, p[0], p[1], p[2])] = c0 * bc.value + c1 * X[ix3(NG, q1[0], q1[1], q1[2])];
      }
      __syncthreads();
    }
    double dm = 0.0, mm = 0.0;
#pragma unroll
    for (int q = 0; q < CPT; q++) {
      const int e = tid + q * nt;
      if (e < N3) {
        const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
        const double pv = X[ix3(NG, i, j, k)];
        dm = fmax(dm, fabs(pv - old[q]));
        mm = fmax(mm, fabs(pv));
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      dm = fmax(dm, __shfl_xor(dm, o, 64));
      mm = fmax(mm, __shfl_xor(mm, o, 64));
    }
    if ((tid & 63) == 0) s_d[tid >> 6] = dm, s_m[tid >> 6] = mm;
    __syncthreads();
    dm = s_d[0], mm = s_m[0];
    for (int w = 1; w < (nt >> 6); w++) dm = fmax(dm, s_d[w]), mm = fmax(mm, s_m[w]);
    __syncthreads();  // s_d / s_m reused by the next pair
    double sp = 2.2250738585072014e-308;  // Fortran spacing(max |phi|)
    if (mm > 0) {
      int ex;
      frexp(mm, &ex);
      sp = ldexp(1.0, ex - 53);
    }
    if (dm <= 4 * sp && it > 10) break;
  }
  for (int e = tid; e < G3; e += nt) x[e] = X[e];
  for (int e = tid; e < N3; e += nt) {
    const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
    r[ix3(NG, i, j, k)] = R[e];
  }
  if (tid == 0) iters[0] = it;
}
}  // extern "C++"

// whether the electrode coarse solve runs as k_cs_electrode (one level-1 box
// with an electrode stencil and six physical faces, no sharding hook)
static bool cs_electrode_fused(const afh_mg *mg) {
  const afh_tree *t = mg->t;
  if (t->ids.n(1) != 1 || t->hook || (t->nc != 8 && t->nc != 16))
    return false;
  const int id = t->h_ids[0][0];
  bool phys = mg->h_vp[id - 1] != nullptr;
  for (int q = 0; q < 6; q++) phys = phys && t->boxes[id - 1].neighbors[q] < 0;
  return phys;
}

// The one-box electrode level-1 solve as a dense product (afh_cs_direct.h):
// x = A^-1 ((rhs + bcc) - g), one thread per row of A^-1, the columns in
// order; A^-1 stored column-major, so a wave's loads of one column are
// contiguous. Bitwise the C oracle's loop.
__global__ void __launch_bounds__(64)
    k_cs_elec_direct(double *__restrict__ x, const double *__restrict__ r,
                     const double *__restrict__ bcc, const double *__restrict__ ainv_t,
                     const double *__restrict__ g) {
  constexpr int NC = AFH_CSD_NC, NG = NC + 2, N = AFH_CSD_N;
  __shared__ double B[N];
  for (int e = threadIdx.x; e < N; e += blockDim.x) {
    const int i = e % NC + 1, j = (e / NC) % NC + 1, k = e / (NC * NC) + 1;
    double rv = r[ix3(NG, i, j, k)];
    if (bcc) rv = rv + bcc[e];
    B[e] = rv - g[e];
  }
  __syncthreads();
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  double acc = 0.0;
  for (int c = 0; c < N; c++) acc = acc + ainv_t[(size_t)c * N + row] * B[c];
  const int i = row % NC + 1, j = (row / NC) % NC + 1, k = row / (NC * NC) + 1;
  x[ix3(NG, i, j, k)] = acc;
}

namespace {
// A^-1 and g of the recent level-1 operators (a regrid creates new
// multigrids with the same level-1 stencil): keyed by the stencil, the
// boundary conditions and the spacing; shared by the thread ranks
struct CsdEntry {
  std::vector<double> v, ainv, g;
  afh_bc bc[6];
  double dr[3];
  bool singular;
};
std::mutex csd_mu;
std::vector<CsdEntry> csd_cache;
}  // namespace

// Before a V-cycle / FMG (outside any graph capture): whether the level-1
// solve is the direct one, and its device tables current
static int32_t prepare_cs_direct(afh_mg *mg) {
  afh_tree *t = mg->t;
  mg->csd_ok = false;
  // a level 1 of one 8^3 box with an electrode stencil and six physical
  // faces (the oracle's solve_coarse_direct: the same test); a sharded tree
  // too -- level 1 is replicated, every rank solves it alike, no collective
  if (!mg->csd_on || t->nc != AFH_CSD_NC || !(mg->any_var && mg->lvl_var[0]) ||
      t->ids.n(1) != 1 || mg->h_v1_id != t->h_ids[0][0] ||
      !mg->h_vp[mg->h_v1_id - 1])
    return AFH_OK;
  for (int q = 0; q < 6; q++)
    if (t->boxes[mg->h_v1_id - 1].neighbors[q] >= 0) return AFH_OK;
  if (mg->csd_v_gen == mg->v1_gen && mg->csd_meth_gen == t->meth_gen && mg->d_csd_ainv) {
    mg->csd_ok = true;
    return AFH_OK;
  }
  const afh_box_meta &m = t->boxes[mg->h_v1_id - 1];
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  const CsdEntry *hit = nullptr;
  std::lock_guard<std::mutex> lk(csd_mu);
  for (const CsdEntry &c : csd_cache)
    if (c.v == mg->h_v1 && !memcmp(c.bc, bc, sizeof c.bc) && !memcmp(c.dr, m.dr, sizeof c.dr))
      hit = &c;
  if (!hit) {
    CsdEntry c;
    c.v = mg->h_v1;
    memcpy(c.bc, bc, sizeof c.bc);
    memcpy(c.dr, m.dr, sizeof c.dr);
    c.ainv.assign((size_t)AFH_CSD_N * AFH_CSD_N, 0.0);
    c.g.assign(AFH_CSD_N, 0.0);
    std::vector<double> work((size_t)2 * AFH_CSD_N * AFH_CSD_N);
    c.singular = afh_csd_build(c.v.data(), c.bc, c.dr, c.ainv.data(), c.g.data(), work.data()) != 0;
    if (csd_cache.size() >= 4) csd_cache.erase(csd_cache.begin());
    csd_cache.push_back(std::move(c));
    hit = &csd_cache.back();
  }
  if (hit->singular) return AFH_OK;  // the iteration stays
  if (!mg->d_csd_ainv) {
    AFH_HIP(hipMalloc(&mg->d_csd_ainv, sizeof(double) * AFH_CSD_N * AFH_CSD_N));
    AFH_HIP(hipMalloc(&mg->d_csd_g, sizeof(double) * AFH_CSD_N));
  }
  AFH_HIP(hipStreamSynchronize(t->stream));
  AFH_HIP(hipMemcpy(mg->d_csd_ainv, hit->ainv.data(), sizeof(double) * hit->ainv.size(),
                    hipMemcpyHostToDevice));
  AFH_HIP(hipMemcpy(mg->d_csd_g, hit->g.data(), sizeof(double) * AFH_CSD_N,
                    hipMemcpyHostToDevice));
  mg->csd_v_gen = mg->v1_gen;
  mg->csd_meth_gen = t->meth_gen;
  mg->csd_ok = true;
  return AFH_OK;
}

static int32_t prepare_all(afh_mg *mg) {
  if (int32_t e = prepare_var(mg)) return e;
  return prepare_cs_direct(mg);
}

static int32_t solve_coarse_gs(afh_mg *mg) {
  afh_tree *t = mg->t;
  const int nid = t->ids.n(1), nc = t->nc, n3 = nc * nc * nc;
  if (mg->csd_ok) {
    const int id = t->h_ids[0][0];
    hipLaunchKernelGGL(k_cs_elec_direct, dim3(AFH_CSD_N / 64), dim3(64), 0, t->stream,
                       t->ccv(mg->d.i_phi) + (size_t)(id - 1) * t->bsz,
                       t->ccv(mg->d.i_rhs) + (size_t)(id - 1) * t->bsz, mg->h_bp[id - 1],
                       mg->d_csd_ainv, mg->d_csd_g);
    AFH_LAUNCH_CHECK("k_cs_elec_direct");
    mg->cycles_host = 1, mg->cycles_on_dev = false;
    return gc_lvl(t, 1, mg->d.i_phi, 1);
  }
  if (cs_electrode_fused(mg)) {
    const int id = t->h_ids[0][0];
    const afh_box_meta &m = t->boxes[id - 1];
    {
      double *phi = t->ccv(mg->d.i_phi) + (size_t)(id - 1) * t->bsz;
      double *rhs = t->ccv(mg->d.i_rhs) + (size_t)(id - 1) * t->bsz;
      int *iters = mg->cs_iters;
      const int nt = n3 >= 1024 ? 1024 : n3;
      if (nc == 8)
        hipLaunchKernelGGL(k_cs_electrode<8>, dim3(1), dim3(nt), 0, t->stream, phi, rhs,
                           mg->h_vp[id - 1], mg->h_bp[id - 1], t->gc_args(mg->d.i_phi),
                           m.dr[0], m.dr[1], m.dr[2], iters);
      else
        hipLaunchKernelGGL(k_cs_electrode<16>, dim3(1), dim3(nt), 0, t->stream, phi, rhs,
                           mg->h_vp[id - 1], mg->h_bp[id - 1], t->gc_args(mg->d.i_phi),
                           m.dr[0], m.dr[1], m.dr[2], iters);
      AFH_LAUNCH_CHECK("k_cs_electrode");
      return gc_lvl(t, 1, mg->d.i_phi, 1);
    }
  }
  if (!mg->cs_old) AFH_HIP(hipMalloc(&mg->cs_old, sizeof(double) * t->bsz * nid));
  // slots 6, 7: the step's deferred limits (0..2) stay as they are
  auto *red = reinterpret_cast<unsigned long long *>(t->scratch) + 6 * RED_SHARDS;
  double *phi = t->ccv(mg->d.i_phi);
  int32_t e;
  for (int it = 1; it <= 200000; it++) {
    hipLaunchKernelGGL(k_copy_compact, dim3((unsigned)((t->bsz + 255) / 256), nid),
                       dim3(256), 0, t->stream, phi, mg->cs_old, t->ids.at(1), t->bsz);
    AFH_LAUNCH_CHECK("k_copy_compact");
    for (int n = 1; n <= 2; n++)
      if ((e = gsrb_half(mg, 1, n, false))) return e;
    if ((e = red_init(t, 6, 0.0)) || (e = red_init(t, 7, 0.0))) return e;
    hipLaunchKernelGGL(k_change_max, dim3((n3 + 255) / 256, nid), dim3(256), 0,
                       t->stream, phi, mg->cs_old, t->ids.at(1), nc, t->bsz, red);
    AFH_LAUNCH_CHECK("k_change_max");
    double r[2];
    const int slots[2] = {6, 7};
    const bool mx[2] = {true, true};
    if ((e = red_finish_n(t, 2, slots, mx)) ||
        (e = red_reduce_fetch(t, 6, 2, 0, r, mg->d.i_phi, 1)))
      return e;
    double sp = 2.2250738585072014e-308;  // Fortran spacing(max |phi|)
    if (r[1] > 0) {
      int ex;
      frexp(r[1], &ex);
      sp = ldexp(1.0, ex - 53);
    }
    if (r[0] <= 4 * sp && it > 10) break;
  }
  return gc_lvl(t, 1, mg->d.i_phi, 1);
}

// AFH_COARSE_PFMG host side: the folded level-1 operator, boundary fold and
// level-set terms in oracle/c/afo.c solve_coarse_pfmg's order, the
// hierarchy (afh_pfmg_setup) when the operator changed, then k_cs_pfmg.
static int32_t pf_prepare(afh_mg *mg) {
  afh_tree *t = mg->t;
  if (mg->d_pf_lvl && mg->pf_v1_gen == mg->v1_gen && mg->pf_meth_gen == t->meth_gen)
    return AFH_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  AFH_HIP(hipStreamIsCapturing(t->stream, &cs));
  if (cs != hipStreamCaptureStatusNone)
    return set_error(AFH_ERR_STATE, "pfmg: setup changed during a graph capture");
  const int nc = t->nc, nid = t->ids.n(1);
  const int nx = t->cgs[0], ny = t->cgs[1], nz = t->cgs[2];
  const size_t n0 = (size_t)nx * ny * nz;
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  std::vector<double> a7(7 * n0, 0.0), b2r(6 * n0, 0.0);
  std::vector<uint8_t> fm(n0, 0);
  std::vector<const double *> vbc(std::max(nid, 1), nullptr);
  for (int q = 0; q < nid; q++) {
    const int id = t->h_ids[0][q];
    const afh_box_meta &m = t->boxes[id - 1];
    auto it = mg->h_vl1.find(id);
    const double *vst = it == mg->h_vl1.end() ? nullptr : it->second.data();
    vbc[q] = mg->h_bp[id - 1];
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          const int e = ((k - 1) * nc + (j - 1)) * nc + (i - 1);
          const int gi[3] = {(m.ix[0] - 1) * nc + i, (m.ix[1] - 1) * nc + j,
                             (m.ix[2] - 1) * nc + k};
          const size_t g = ((size_t)(gi[2] - 1) * ny + (gi[1] - 1)) * nx + (gi[0] - 1);
          double c[7];
          if (vst) memcpy(c, vst + 7 * (size_t)e, sizeof c);
          else memcpy(c, mg->lvl_c[0].c, sizeof c);
          for (int nb = 1; nb <= 6; nb++) {
            const int dd = (nb - 1) >> 1;
            const bool low = ((nb - 1) & 1) == 0;
            const int dims = t->cgs[dd];
            if (!(low ? gi[dd] == 1 : gi[dd] == dims)) continue;
            double k2;
            if (bc[nb - 1].type == AFH_BC_DIRICHLET) {
              c[0] = c[0] - c[nb];
              k2 = -2 * c[nb];
            } else {
              c[0] = c[0] + c[nb];
              k2 = -(c[nb] * m.dr[dd]) * (low ? -1 : 1);
            }
            b2r[(size_t)(nb - 1) * n0 + g] = k2;
            fm[g] |= (uint8_t)(1 << (nb - 1));
            c[nb] = 0.0;
          }
          memcpy(&a7[7 * g], c, sizeof c);
        }
  }
  AFH_HIP(hipStreamSynchronize(t->stream));
  if (!mg->d_pf_lvl || a7 != mg->pf_a7) {
    afh_pfmg h;
    if (afh_pfmg_setup(&h, nx, ny, nz, 3, a7.data()))
      return set_error(AFH_ERR_DEVICE, "pfmg: host setup allocation");
    const int np = (int)h.off[h.nl];
    std::vector<PfLvl> lv;
    std::vector<double> A, P;
    afh_pf::pf_device_tables(h, lv, A, P);
    afh_pfmg_free(&h);
    hipFree(mg->d_pf_lvl), hipFree(mg->d_pf_A), hipFree(mg->d_pf_P), hipFree(mg->d_pf_x);
    mg->d_pf_x = nullptr;
    AFH_HIP(hipMalloc(&mg->d_pf_lvl, sizeof(PfLvl) * lv.size()));
    AFH_HIP(hipMalloc(&mg->d_pf_A, sizeof(double) * A.size()));
    AFH_HIP(hipMalloc(&mg->d_pf_P, sizeof(double) * P.size()));
    AFH_HIP(hipMemcpy(mg->d_pf_lvl, lv.data(), sizeof(PfLvl) * lv.size(), hipMemcpyHostToDevice));
    AFH_HIP(hipMemcpy(mg->d_pf_A, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
    AFH_HIP(hipMemcpy(mg->d_pf_P, P.data(), sizeof(double) * P.size(), hipMemcpyHostToDevice));
    mg->pf_nl = (int)lv.size();
    mg->pf_np = np;
    // the vectors and the wave levels' operators in LDS when they fit, else
    // the vectors alone (round 6: levels of up to 128 or 256 points on wave
    // 0 measured slower, scripts/pfmg_probe.py)
    mg->pf_wave = afh_pf::pf_wave_from(lv);
    const size_t lds = afh_pf::pf_lds_bytes(lv, true);
    const size_t lds_x = afh_pf::pf_lds_bytes(lv, false);
    mg->pf_stage = lds + 64 <= 160 * 1024;
    mg->pf_lds = mg->pf_stage ? (int)lds : lds_x + 64 <= 160 * 1024 ? (int)lds_x : 0;
    if (mg->pf_lds)
      AFH_HIP(raise_dyn_lds(mg->pf_stage ? (const void *)k_cs_pfmg<true, true>
                                         : (const void *)k_cs_pfmg<true, false>,
                            mg->pf_lds));
    else
      AFH_HIP(hipMalloc(&mg->d_pf_x, sizeof(double) * 4 * (size_t)np));
    mg->pf_a7.swap(a7);
  }
  if (!mg->d_pf_b2r) {
    AFH_HIP(hipMalloc(&mg->d_pf_b2r, sizeof(double) * 6 * n0));
    AFH_HIP(hipMalloc(&mg->d_pf_fmask, n0));
  }
  hipFree((void *)mg->d_pf_vbc);
  AFH_HIP(hipMalloc((void **)&mg->d_pf_vbc, sizeof(double *) * vbc.size()));
  AFH_HIP(hipMemcpy(mg->d_pf_b2r, b2r.data(), sizeof(double) * 6 * n0, hipMemcpyHostToDevice));
  AFH_HIP(hipMemcpy(mg->d_pf_fmask, fm.data(), n0, hipMemcpyHostToDevice));
  AFH_HIP(hipMemcpy((void *)mg->d_pf_vbc, vbc.data(), sizeof(double *) * vbc.size(),
                    hipMemcpyHostToDevice));
  mg->pf_v1_gen = mg->v1_gen;
  mg->pf_meth_gen = t->meth_gen;
  return AFH_OK;
}

static int32_t solve_coarse_pfmg(afh_mg *mg) {
  afh_tree *t = mg->t;
  if (int32_t e = pf_prepare(mg)) return e;
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  PfBc B;
  for (int q = 0; q < 6; q++) B.bc[q] = bc[q];
  const int nid = t->ids.n(1);
  // workgroup: the level-0 points over whole waves, 256 .. 1024 lanes
  const int n0 = (int)(mg->pf_a7.size() / 7);
  // (256 or 512 lanes on S4 / S5's 512 / 2048 points measured slower)
  const int nt = std::min(1024, std::max(256, (n0 + 63) / 64 * 64));
  auto *kern = !mg->pf_lds ? k_cs_pfmg<false, false>
               : mg->pf_stage ? k_cs_pfmg<true, true> : k_cs_pfmg<true, false>;
  prof_begin(t, AFH_PROF_CS);
  hipLaunchKernelGGL(kern, dim3(1), dim3(nt),
                     mg->pf_lds, t->stream, mg->d_pf_lvl, mg->pf_nl, mg->pf_wave, mg->d_pf_A,
                     mg->d_pf_P, mg->d_pf_b2r, mg->d_pf_fmask, mg->d_pf_vbc, mg->d_pf_x,
                     t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->d_boxes, t->ids.at(1), nid,
                     t->nc, t->bsz, B, mg->d.coarse_tol, mg->d.coarse_cycles, mg->d_cycles);
  AFH_LAUNCH_CHECK("k_cs_pfmg");
  prof_end(t, AFH_PROF_CS, 0.0);
  mg->cycles_host = 0, mg->cycles_on_dev = true;
  return gc_lvl(t, 1, mg->d.i_phi, 1);
}

static int32_t solve_coarse(afh_mg *mg) {
  afh_tree *t = mg->t;
  if (mg->d.coarse_mode == AFH_COARSE_PFMG) return solve_coarse_pfmg(mg);
  if (mg->any_var && mg->lvl_var[0]) return solve_coarse_gs(mg);
  CsParams &P = mg->P;
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  for (int q = 0; q < 6; q++) P.bctype[q] = bc[q].type;
  for (int q = 0; q < 6; q++)
    if (mg->tab_bc[q] != bc[q].type) {
      if (int32_t e = build_table(mg)) return e;
      break;
    }
  const int nc = t->nc, nid = t->ids.n(1), n3 = nc * nc * nc;
  if (mg->d.coarse_mode == AFH_COARSE_DIRECT && mg->cs_direct_small &&
      (long)P.dims[0][0] * P.dims[0][1] * P.dims[0][2] <= mg->cs_ds_cells) {
    for (int q = 0; q < 6; q++)
      if (mg->q_bc[q] != bc[q].type) {
        if (int32_t e = build_direct(mg)) return e;
        break;
      }
    if (nid)
      hipLaunchKernelGGL(k_cs_direct_small, dim3(1), dim3(1024), 0, t->stream, P,
                         t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->d_boxes, t->ids.at(1),
                         nid, nc, t->bsz, bc[0], bc[1], bc[2], bc[3], bc[4], bc[5],
                         mg->d_q[0], mg->d_q[1], mg->d_q[2], mg->d_qt[0], mg->d_qt[1],
                         mg->d_qt[2], mg->d_e[0], mg->d_e[1], mg->d_e[2],
                         mg->d.helmholtz_lambda);
    AFH_LAUNCH_CHECK("k_cs_direct_small");
    mg->cycles_host = 0, mg->cycles_on_dev = false;
    return gc_lvl(t, 1, mg->d.i_phi, 1);
  }
  hipLaunchKernelGGL(k_cs_gather, dim3((n3 + 255) / 256, nid), dim3(256), 0,
                     t->stream, P, t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs),
                     t->d_boxes, t->ids.at(1), nc, t->bsz, bc[0], bc[1], bc[2],
                     bc[3], bc[4], bc[5]);
  AFH_LAUNCH_CHECK("k_cs_gather");
  const int s = mg->small_from;
  if (mg->d.coarse_mode == AFH_COARSE_DIRECT) {
    for (int q = 0; q < 6; q++)
      if (mg->q_bc[q] != bc[q].type) {
        if (int32_t e = build_direct(mg)) return e;
        break;
      }
    const int nx = P.dims[0][0], ny = P.dims[0][1], nz = P.dims[0][2];
    const dim3 g = blocks1((size_t)nx * ny * nz);
    const double lam = mg->d.helmholtz_lambda;
    // Q^T along x, y, z (divide), then Q along z, y, x
    struct Pass { const double *in; int ih; double *out; int oh; int d; bool fwd; int div; };
    const Pass ps[6] = {{P.f[0], 1, mg->w1, 0, 0, true, 0}, {mg->w1, 0, mg->w2, 0, 1, true, 0},
                        {mg->w2, 0, mg->w1, 0, 2, true, 1}, {mg->w1, 0, mg->w2, 0, 2, false, 0},
                        {mg->w2, 0, mg->w1, 0, 1, false, 0}, {mg->w1, 0, P.u[0], 1, 0, false, 0}};
    for (const Pass &q : ps)
      hipLaunchKernelGGL(k_cs_transform, g, dim3(256), 0, t->stream, q.in, q.ih,
                         q.out, q.oh, q.fwd ? mg->d_q[q.d] : mg->d_qt[q.d],
                         mg->d_e[0], mg->d_e[1], mg->d_e[2], nx, ny, nz, q.d,
                         q.div, lam);
    AFH_LAUNCH_CHECK("k_cs_transform");
    mg->cycles_host = 0, mg->cycles_on_dev = false;
  } else if (s == 0) {
    const double tol2 = mg->d.coarse_tol > 0 ? mg->d.coarse_tol * mg->d.coarse_tol : 0.0;
    hipLaunchKernelGGL(k_cs_small, dim3(1), dim3(1024), mg->small_lds, t->stream, P, 0,
                       mg->d.coarse_cycles, mg->wave_cells, tol2, mg->d_cycles);
    AFH_LAUNCH_CHECK("k_cs_small");
    mg->cycles_host = mg->d.coarse_cycles, mg->cycles_on_dev = tol2 > 0;
  } else {
    // with the stopping rule: |b|^2 first, |r|^2 after every cycle, read on
    // the host (no graph capture then, vcycle_graph)
    const bool tol = mg->d.coarse_tol > 0;
    const int n0 = P.dims[0][0] * P.dims[0][1] * P.dims[0][2], nblk = (n0 + 255) / 256;
    auto norm2 = [&](int res, double &out) -> int32_t {
      if (!mg->d_norm) AFH_HIP(hipMalloc(&mg->d_norm, sizeof(double) * nblk));
      mg->h_norm.resize(nblk);
      hipLaunchKernelGGL(k_cs_norm2, dim3(nblk), dim3(256), 0, t->stream, P, res, mg->d_norm);
      AFH_LAUNCH_CHECK("k_cs_norm2");
      AFH_HIP(hipMemcpyAsync(mg->h_norm.data(), mg->d_norm, sizeof(double) * nblk,
                             hipMemcpyDeviceToHost, t->stream));
      AFH_HIP(hipStreamSynchronize(t->stream));
      out = 0.0;
      for (double v : mg->h_norm) out += v;
      return AFH_OK;
    };
    double bb = 0.0;
    int n_cyc = mg->d.coarse_cycles;
    if (tol) {
      if (int32_t e = norm2(0, bb)) return e;
      if (bb == 0.0) {
        hipLaunchKernelGGL(k_cs_zero, dim3(nblk), dim3(256), 0, t->stream, P);
        AFH_LAUNCH_CHECK("k_cs_zero");
        n_cyc = 0;
      }
    }
    const double eps = tol ? mg->d.coarse_tol * mg->d.coarse_tol : 0.0;
    int done = 0;
    for (int cyc = 0; cyc < n_cyc; cyc++) {
      for (int m = 0; m < s; m++) {
        const size_t N = (size_t)P.dims[m][0] * P.dims[m][1] * P.dims[m][2];
        for (int sw = 0; sw < 2; sw++)
          for (int n = 1; n <= 2; n++)
            hipLaunchKernelGGL(k_cs_gsrb, blocks1(N / 2), dim3(256), 0,
                               t->stream, P, m, n);
        hipLaunchKernelGGL(k_cs_rstr, blocks1(N / 8), dim3(256), 0, t->stream, P,
                           m + 1);
      }
      hipLaunchKernelGGL(k_cs_small, dim3(1), dim3(1024), mg->small_lds,
                         t->stream, P, s, 1, mg->wave_cells, 0.0, (int *)nullptr);
      for (int m = s - 1; m >= 0; m--) {
        const size_t N = (size_t)P.dims[m][0] * P.dims[m][1] * P.dims[m][2];
        hipLaunchKernelGGL(k_cs_prol, blocks1(N), dim3(256), 0, t->stream, P, m);
        for (int sw = 0; sw < 2; sw++)
          for (int n = 1; n <= 2; n++)
            hipLaunchKernelGGL(k_cs_gsrb, blocks1(N / 2), dim3(256), 0,
                               t->stream, P, m, n);
      }
      done = cyc + 1;
      if (tol) {
        double rr;
        if (int32_t e = norm2(1, rr)) return e;
        if (rr / bb < eps) break;
      }
    }
    AFH_LAUNCH_CHECK("coarse solver cycle");
    mg->cycles_host = done, mg->cycles_on_dev = false;
  }
  hipLaunchKernelGGL(k_cs_scatter, dim3((n3 + 255) / 256, nid), dim3(256), 0,
                     t->stream, P, t->ccv(mg->d.i_phi), t->d_boxes,
                     t->ids.at(1), nc, t->bsz);
  AFH_LAUNCH_CHECK("k_cs_scatter");
  return gc_lvl(t, 1, mg->d.i_phi, 1);
}

static int32_t box_copy(afh_tree *t, int lvl, const double *src, double *dst) {
  const int n = t->ids.n(lvl);
  if (!n) return AFH_OK;
  hipLaunchKernelGGL(k_box_copy, dim3((unsigned)((t->bsz + 255) / 256), n),
                     dim3(256), 0, t->stream, src, dst, t->ids.at(lvl), t->bsz);
  AFH_LAUNCH_CHECK("k_box_copy");
  return AFH_OK;
}

// mg_fas_fmg (m_af_multigrid.f90:137-180) with set_coarse_phi_rhs (742-776)
// and init_phi_rhs (779-799). set_coarse_phi_rhs is update_coarse without
// restoring tmp; update_coarse's extra tmp = phi on the parents is
// overwritten by the phi -> tmp copies below before tmp is read again.
int32_t afh_mg_fas_fmg(afh_mg *mg, int32_t set_residual, int32_t have_guess) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  afh_tree *t = mg->t;
  AFH_LIVE(t, "afh_mg_fas_fmg");
  t->touch(mg->d.i_phi), t->touch(mg->d.i_rhs), t->touch(mg->d.i_tmp);
  const int nl = t->nlvl, i_phi = mg->d.i_phi;
  double *phi = t->ccv(i_phi), *tmp = t->ccv(mg->d.i_tmp);
  int32_t e;
  if ((e = prepare_all(mg))) return e;
  if (have_guess) {
    for (int lvl = nl; lvl >= 2; lvl--) {
      if (lvl == nl && (e = gc_lvl(t, lvl, i_phi, 1, fused_level(mg, lvl)))) return e;
      if ((e = update_coarse(mg, lvl))) return e;
    }
  } else {
    for (int lvl = nl; lvl >= 2; lvl--) {
      if ((e = box_copy(t, lvl, nullptr, phi)) ||
          (e = restrict_boxes(t, t->ids.at(lvl), t->ids.n(lvl), mg->d.i_rhs)) ||
          (e = call_hook(t, AFH_HOOK_RESTRICT, lvl, mg->d.i_rhs)))
        return e;
    }
  }
  if ((e = box_copy(t, 1, phi, tmp)) ||
      (e = afh_mg_fas_vcycle(mg, set_residual && nl == 1, 1)))
    return e;
  for (int lvl = 2; lvl <= nl; lvl++) {
    if ((e = box_copy(t, lvl, phi, tmp)) || (e = correct_children(mg, lvl)) ||
        (e = gc_lvl(t, lvl, i_phi, 1, fused_level(mg, lvl))))
      return e;
    mg->phi_gc_gen = t->gen[i_phi];  // the cycle's top level was just filled
    mg->phi_gc_meth = t->meth_gen;
    mg->in_fmg = true;
    e = afh_mg_fas_vcycle(mg, set_residual && lvl == nl, lvl);
    mg->in_fmg = false;
    if (e) return e;
  }
  return AFH_OK;
}

}  // extern "C"

// residual on every box of levels 1..max_lvl; with max_out also the leaf
// max|residual| (reduction slot 3, as afh_tree_maxabs_cc), in the same pass
// (device work only; residual_fetch reads the maximum)
// the final residual pass of a V-cycle also writes |E| (afh_mg_set_gradient_
// output): V-cycles over the whole tree, constant stencils only
static bool grad_fused(const afh_mg *mg, int max_lvl) {
  return mg->grad_iv > 0 && !mg->any_var && max_lvl == mg->t->nlvl;
}

static int32_t residual_levels(afh_mg *mg, int max_lvl, bool max_out) {
  afh_tree *t = mg->t;
  const int nc = t->nc, n3 = nc * nc * nc;
  auto *red = reinterpret_cast<unsigned long long *>(t->scratch) + 3 * RED_SHARDS;
  int32_t e;
  if (max_out && (e = red_init(t, 3, 0.0))) return e;
  // the constant-coefficient boxes of every level in one launch per part
  // (the level's coefficients from d_lvl_c): levels do not interact here
  const bool all_lvls = t->all_lvl_launch;
  for (int lvl = 1; lvl <= max_lvl; lvl++) {
    const Coef &cf = mg->lvl_c[lvl - 1];
    for (int part = 0; part < 2; part++) {
      // part 0: leaves (max folded), part 1: parents; without max_out the
      // level's whole id list in one launch
      if (!max_out && part) break;
      const LevelList &A = max_out ? (part ? t->parents : t->leaves) : t->ids;
      const LevelList &Lc = max_out ? (part ? mg->parents_c : mg->leaves_c) : mg->ids_c;
      const LevelList &Lv = max_out ? (part ? mg->parents_v : mg->leaves_v) : mg->ids_v;
      const LevelList &L = cst(mg, A, Lc);
      const int n_all = L.off[max_lvl] - L.off[0];
      const bool one = all_lvls && n_all <= 65535;
      const int n = one ? (lvl == 1 ? n_all : 0) : L.n(lvl);
      const bool mx = max_out && !part;
      if (n) {
        // columns of 8 on the large boxes: 693 against 728 us per 64^3 leaf
        // launch (profiles/r03_ab_res_k.txt); small boxes keep their threads
        const int rk = mg->res_k ? mg->res_k : nc >= 32 ? 8 : 4;
        const int kc = nc % rk == 0 ? rk : nc % 4 == 0 ? 4 : 2;
        const dim3 grid((n3 / kc + 255) / 256, n);
        const bool gr = grad_fused(mg, max_lvl);
        auto kern = gr ? (mx ? (kc == 8 ? k_residual<true, 8, true>
                                        : kc == 4 ? k_residual<true, 4, true>
                                                  : k_residual<true, 2, true>)
                             : (kc == 8 ? k_residual<false, 8, true>
                                        : kc == 4 ? k_residual<false, 4, true>
                                                  : k_residual<false, 2, true>))
                  : mx ? (kc == 8 ? k_residual<true, 8> : kc == 4 ? k_residual<true, 4>
                                                                  : k_residual<true, 2>)
                       : (kc == 8 ? k_residual<false, 8> : kc == 4 ? k_residual<false, 4>
                                                                   : k_residual<false, 2>);
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, t->stream,
                           t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs),
                           t->ccv(mg->d.i_tmp), L.at(lvl), nc, t->bsz, cf, red,
                           one ? mg->d_lvl_c : nullptr, (one || gr) ? t->d_boxes : nullptr,
                           gr ? t->ccv(mg->grad_iv) : nullptr, mg->grad_fac);
        AFH_LAUNCH_CHECK("k_residual");
      }
      const int nv = mg->any_var ? Lv.n(lvl) : 0;
      if (nv) {
        hipLaunchKernelGGL(mx ? k_residual_v<true> : k_residual_v<false>,
                           dim3((n3 + 255) / 256, nv), dim3(256), 0, t->stream,
                           t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs),
                           t->ccv(mg->d.i_tmp), Lv.at(lvl), nc, t->bsz, mg->d_vp,
                           mg->d_bp, red);
        AFH_LAUNCH_CHECK("k_residual_v");
      }
    }
  }
  if (!max_out) return AFH_OK;
  return red_finish(t, 3, true);
}

static int32_t residual_fetch(afh_mg *mg, double *max_out) {
  return red_reduce_fetch(mg->t, 3, 1, 0, max_out, mg->d.i_tmp);
}

// the device work of one V-cycle (everything but reading max|res|)
static int32_t vcycle_body(afh_mg *mg, int32_t set_residual, int max_lvl, bool max_out,
                           bool top_stale) {
  afh_tree *t = mg->t;
  int32_t e;
  mg->rhs_halo.assign(t->nlvl, 0);
  mg->vc_max_lvl = max_lvl;
  for (int lvl = max_lvl; lvl >= 2; lvl--) {
    if ((e = gsrb_boxes(mg, lvl, false, top_stale && lvl == max_lvl))) return e;
    // (ghosts of the levels below valid: phi and the boundary conditions
    // unchanged since a V-cycle over the whole tree filled them, or the
    // previous V-cycle of an FMG)
    if ((e = update_coarse(mg, lvl, !top_stale && (max_lvl == t->nlvl || mg->in_fmg) &&
                                        mg->phi_gc_meth == t->meth_gen)))
      return e;
  }
  if ((e = solve_coarse(mg))) return e;
  for (int lvl = 2; lvl <= max_lvl; lvl++) {
    if ((e = correct_children(mg, lvl))) return e;
    // (a pushing correction filled the faces, and the pushing pairs read no
    // edges or corners: k_gc_corners follows the leg's last pair)
    if (!prolong_push(mg, lvl) &&
        (e = gc_lvl_var(t, lvl, mg->d.i_phi, t->ccv(mg->d.i_phi),
                        t->gc_args(mg->d.i_phi), 1, fused_level(mg, lvl),
                        fused_level(mg, lvl) ? 2 : 1)))
      return e;
    if ((e = gsrb_boxes(mg, lvl, true))) return e;
  }
  if (set_residual) return residual_levels(mg, max_lvl, max_out);
  return AFH_OK;
}

// A sharded V-cycle (a hook) as segments: the device work between two
// exchanges is captured as one graph, the exchange itself (host-driven:
// pack, the transport, unpack) is recorded and run between the replays of
// its neighbouring segments. Every rank records and replays the same
// sequence of exchanges, in the eager order.
static int32_t vcycle_segments(afh_mg *mg, afh_mg::Graph &g, int32_t set_residual,
                               int max_lvl, bool max_out, bool top_stale, bool &done) {
  afh_tree *t = mg->t;
  if (g.segs.empty()) {
    afh_tree::SegRec rec;
    AFH_HIP(hipStreamBeginCapture(t->stream, hipStreamCaptureModeThreadLocal));
    t->seg_rec = &rec;
    int32_t e = vcycle_body(mg, set_residual, max_lvl, max_out, top_stale);
    t->seg_rec = nullptr;
    hipGraph_t last = nullptr;
    const hipError_t ce = hipStreamEndCapture(t->stream, &last);
    if (ce == hipSuccess) rec.graphs.push_back(last);
    if (!e && ce != hipSuccess) e = set_error(AFH_ERR_DEVICE, "segment capture failed");
    for (size_t k = 0; k < rec.graphs.size() && !e; k++) {
      size_t nn = 0;
      hipGraphExec_t x = nullptr;
      if (hipGraphGetNodes(rec.graphs[k], nullptr, &nn) != hipSuccess ||
          (nn && hipGraphInstantiate(&x, rec.graphs[k], nullptr, nullptr, 0) != hipSuccess))
        e = set_error(AFH_ERR_DEVICE, "segment instantiation failed");
      g.segs.push_back(x);  // (an empty segment replays as nothing)
    }
    for (hipGraph_t gr : rec.graphs)
      if (gr) hipGraphDestroy(gr);
    if (rec.bad) {
      // (a reduction on the way: this variant stays eager)
      g.release();
      g.eager_only = true;
      return AFH_OK;
    }
    if (e) {
      g.release();
      return e;
    }
    g.ops = rec.ops;
  }
  for (size_t k = 0; k < g.segs.size(); k++) {
    if (g.segs[k]) AFH_HIP(hipGraphLaunch(g.segs[k], t->stream));
    if (k < g.ops.size())
      if (int32_t e = call_hook(t, g.ops[k][0], g.ops[k][1], g.ops[k][2], nullptr, g.ops[k][3]))
        return e;
  }
  mg->n_replays++, mg->n_seg_replays++;
  done = true;
  return AFH_OK;
}

// Replays a captured V-cycle when it can: no kernel timing, no electrode
// coarse solve that reads the device every pair; sharded, as segments
// between the exchanges (vcycle_segments). The first call of a variant runs
// eagerly (tables, spare image); a change of boundary conditions drops the
// graph.
static int32_t vcycle_graph(afh_mg *mg, int32_t set_residual, int max_lvl, bool max_out,
                            bool top_stale, bool &done) {
  afh_tree *t = mg->t;
  done = false;
  // (the multi-launch coarse cycles with a stopping rule read the device
  // every cycle too)
  if (!mg->use_graphs || (t->hook && !mg->seg_graphs) || t->prof_class ||
      (mg->d.coarse_mode != AFH_COARSE_PFMG && mg->any_var && mg->lvl_var[0] &&
       !cs_electrode_fused(mg) && !mg->csd_ok) ||
      (mg->d.coarse_mode == AFH_COARSE_CYCLES && mg->d.coarse_tol > 0 && mg->small_from > 0))
    return AFH_OK;
  const int key = (max_lvl << 4) | (mg->in_fmg ? 8 : 0) | (top_stale ? 4 : 0) |
                  (set_residual ? 2 : 0) | (max_out ? 1 : 0);
  afh_mg::Graph &g = mg->graphs[key];
  if (g.meth_gen != t->meth_gen) {
    // new boundary values or types since the warm call / capture: run
    // eagerly once more (rebuilds the coarse-solve tables outside capture)
    g.release();
    g = afh_mg::Graph();
    g.meth_gen = t->meth_gen;
  }
  if (!g.warm) {
    g.warm = true;
    return AFH_OK;  // this call runs eagerly
  }
  if (g.eager_only) return AFH_OK;
  const bool whole = !t->hook || (mg->rccl_capture && t->hook_capturable);
  if (!whole) return vcycle_segments(mg, g, set_residual, max_lvl, max_out, top_stale, done);
  if (!g.exec) {
    hipGraph_t graph;
    AFH_HIP(hipStreamBeginCapture(t->stream, hipStreamCaptureModeThreadLocal));
    const int32_t e = vcycle_body(mg, set_residual, max_lvl, max_out, top_stale);
    const hipError_t ce = hipStreamEndCapture(t->stream, &graph);
    if (t->hook && (e || ce != hipSuccess)) {
      // (the exchanges would not capture: this variant stays eager)
      if (ce == hipSuccess) hipGraphDestroy(graph);
      (void)hipGetLastError();
      g.eager_only = true;
      return AFH_OK;
    }
    if (e) {
      if (ce == hipSuccess) hipGraphDestroy(graph);
      return e;
    }
    AFH_HIP(ce);
    const hipError_t ie = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    hipGraphDestroy(graph);
    AFH_HIP(ie);
  }
  AFH_HIP(hipGraphLaunch(g.exec, t->stream));
  mg->n_replays++;
  done = true;
  return AFH_OK;
}

// max_out: the leaf max|residual| folded into AFH_SLOT_MAXRES, read into
// max_res when given
static int32_t vcycle_impl(afh_mg *mg, int32_t set_residual, int32_t hl, bool max_out,
                           double *max_res) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  afh_tree *t = mg->t;
  AFH_LIVE(t, "afh_mg_fas_vcycle");
  const bool top_stale = mg->phi_gc_gen != t->gen[mg->d.i_phi];
  t->touch(mg->d.i_phi), t->touch(mg->d.i_rhs), t->touch(mg->d.i_tmp);
  const int max_lvl = (hl > 0 && hl <= t->nlvl) ? hl : t->nlvl;
  int32_t e;
  if ((e = prepare_all(mg))) return e;
  bool done;
  max_out = max_out && set_residual;
  if ((e = vcycle_graph(mg, set_residual, max_lvl, max_out, top_stale, done))) return e;
  if (!done && (e = vcycle_body(mg, set_residual, max_lvl, max_out, top_stale))) return e;
  // the up leg filled every level's ghost cells (corners on the last fill)
  if (max_lvl == t->nlvl) mg->phi_gc_gen = t->gen[mg->d.i_phi], mg->phi_gc_meth = t->meth_gen;
  if (set_residual && grad_fused(mg, max_lvl)) {  // |E| of this phi is stored
    t->touch(mg->grad_iv);
    mg->grad_phi_gen = t->gen[mg->d.i_phi];
    mg->grad_norm_gen = t->gen[mg->grad_iv];
  }
  return max_out && max_res ? residual_fetch(mg, max_res) : AFH_OK;
}

extern "C" {

int32_t afh_mg_fas_vcycle(afh_mg *mg, int32_t set_residual, int32_t hl) {
  return vcycle_impl(mg, set_residual, hl, false, nullptr);
}

int32_t afh_mg_fas_vcycle_maxres(afh_mg *mg, int32_t hl, double *max_res) {
  if (!max_res) return set_error(AFH_ERR_ARG, "null max_res");
  return vcycle_impl(mg, 1, hl, true, max_res);
}

int32_t afh_mg_fas_vcycle_fold(afh_mg *mg, int32_t hl) {
  return vcycle_impl(mg, 1, hl, true, nullptr);
}

int32_t afh_mg_set_gradient_output(afh_mg *mg, int32_t i_norm, double fac) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  AFH_LIVE(mg->t, "afh_mg_set_gradient_output");
  if (i_norm < 0 || i_norm > mg->t->nvc) return set_error(AFH_ERR_ARG, "bad variable index");
  mg->grad_iv = i_norm;
  mg->grad_fac = fac;
  mg->grad_phi_gen = mg->grad_norm_gen = UINT64_MAX;
  mg->t->meth_gen++;  // captured V-cycles baked the residual kernel in
  return AFH_OK;
}

int32_t afh_mg_graph_stats(afh_mg *mg, int64_t *replays, int64_t *segmented) {
  if (!mg || !replays || !segmented) return set_error(AFH_ERR_ARG, "afh_mg_graph_stats: null");
  *replays = mg->n_replays;
  *segmented = mg->n_seg_replays;
  return AFH_OK;
}

int32_t afh_mg_coarse_iterations(afh_mg *mg, int32_t *n) {
  if (!mg || !n) return set_error(AFH_ERR_ARG, "afh_mg_coarse_iterations: null");
  AFH_LIVE(mg->t, "afh_mg_coarse_iterations");
  *n = mg->cycles_host;
  if (mg->cycles_on_dev) {
    int v = 0;
    AFH_HIP(hipMemcpyAsync(&v, mg->d_cycles, sizeof(int), hipMemcpyDeviceToHost,
                           mg->t->stream));
    AFH_HIP(hipStreamSynchronize(mg->t->stream));
    *n = v;
  }
  return AFH_OK;
}

int32_t afh_mg_compute_phi_gradient(afh_mg *mg, int32_t i_fc, double fac,
                                    int32_t i_norm) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  afh_tree *t = mg->t;
  AFH_LIVE(t, "afh_mg_compute_phi_gradient");
  if (i_fc < 0 || i_fc > t->nvf || i_norm < 0 || i_norm > t->nvc)
    return set_error(AFH_ERR_ARG, "bad variable index");
  int32_t e;
  if ((e = prepare_all(mg))) return e;
  // i_fc = 0: the norm only (the flux evaluates the face field from phi,
  // afh_fluid_set_field_source); electrode boxes need the face field
  if (i_fc == 0 && (i_norm == 0 || mg->any_lsf))
    return set_error(AFH_ERR_ARG, "i_fc = 0 needs i_norm and no electrode boxes");
  // the last V-cycle's residual pass stored this |E| of this phi already
  // (afh_mg_set_gradient_output; neither changed since)
  if (i_fc == 0 && i_norm == mg->grad_iv && fac == mg->grad_fac && !mg->any_var &&
      mg->grad_phi_gen == t->gen[mg->d.i_phi] && mg->grad_norm_gen == t->gen[i_norm])
    return AFH_OK;
  const int nc = t->nc, n3 = nc * nc * nc;
  const int ntot = t->ids.off[t->nlvl];
  double *nrm = i_norm > 0 ? t->ccv(i_norm) : nullptr;
  double *fcv = i_fc > 0 ? t->fcv(i_fc) : nullptr;
  switch (nc) {
  case 4: launch_gradient<4>(t, t->ccv(mg->d.i_phi), fcv, nrm, fac, mg->grad_nt); break;
  case 8: launch_gradient<8>(t, t->ccv(mg->d.i_phi), fcv, nrm, fac, mg->grad_nt); break;
  case 16: launch_gradient<16>(t, t->ccv(mg->d.i_phi), fcv, nrm, fac, mg->grad_nt); break;
  case 32: launch_gradient<32>(t, t->ccv(mg->d.i_phi), fcv, nrm, fac, mg->grad_nt); break;
  case 64: launch_gradient<64>(t, t->ccv(mg->d.i_phi), fcv, nrm, fac, mg->grad_nt); break;
  default:
  if (!fcv) return set_error(AFH_ERR_UNSUPPORTED, "i_fc = 0: box size %d", nc);
  hipLaunchKernelGGL(k_gradient, dim3((n3 + 255) / 256, ntot), dim3(256), 0,
                     t->stream, t->ccv(mg->d.i_phi), t->fcv(i_fc),
                     i_norm > 0 ? t->ccv(i_norm) : nullptr, t->d_boxes,
                     t->ids.d, nc, t->bsz, t->fsz, fac);
  }
  AFH_LAUNCH_CHECK("k_gradient");
  if (!mg->any_lsf) return AFH_OK;
  // electrode leaf boxes: mg_box_lpllsf_gradient, then their |E| again
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = mg->lsf_leaves.n(l);
    if (!n) continue;
    const double *dr = &t->lvl_dr[3 * (l - 1)];
    auto par = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(n), dim3(256), 0, t->stream, t->ccv(mg->d.i_phi),
                         t->ccv(mg->i_lsf), t->fcv(i_fc), mg->lsf_leaves.at(l), t->bsz,
                         t->fsz, mg->d_lsf_n, mg->d_ix, mg->d_dd, mg->d_bv, fac / dr[0],
                         fac / dr[1], fac / dr[2]);
    };
    if (nc == 4) par(k_lsf_gradient_par<4>);
    else if (nc == 8) par(k_lsf_gradient_par<8>);
    else if (nc == 16) par(k_lsf_gradient_par<16>);
    else
      hipLaunchKernelGGL(k_lsf_gradient, dim3(n), dim3(64), 0, t->stream,
                         t->ccv(mg->d.i_phi), t->ccv(mg->i_lsf), t->fcv(i_fc),
                         mg->lsf_leaves.at(l), nc, t->bsz, t->fsz, mg->d_lsf_n,
                         mg->d_ix, mg->d_dd, mg->d_bv, fac / dr[0], fac / dr[1],
                         fac / dr[2]);
    AFH_LAUNCH_CHECK("k_lsf_gradient");
    if (nrm) {
      hipLaunchKernelGGL(k_field_norm, dim3((n3 + 255) / 256, n), dim3(256), 0,
                         t->stream, t->fcv(i_fc), nrm, mg->lsf_leaves.at(l), nc,
                         t->bsz, t->fsz);
      AFH_LAUNCH_CHECK("k_field_norm");
    }
  }
  return AFH_OK;
}

int32_t afh_mg_set_box_stencil(afh_mg *mg, int32_t id, const double *v,
                               const double *bc_correction) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  AFH_LIVE(mg->t, "afh_mg_set_box_stencil");
  if (id < 1 || id > mg->t->nb) return set_error(AFH_ERR_ARG, "bad box id");
  afh_tree *t = mg->t;
  const size_t n3 = (size_t)t->nc * t->nc * t->nc;
  AFH_HIP(hipStreamSynchronize(t->stream));
  hipFree(mg->h_vp[id - 1]), hipFree(mg->h_bp[id - 1]);
  mg->h_vp[id - 1] = mg->h_bp[id - 1] = nullptr;
  mg->var_dirty = true;
  if (t->boxes[id - 1].lvl == 1) {  // the level-1 solve's host copy
    mg->v1_gen++;
    if (v) mg->h_v1.assign(v, v + 7 * n3), mg->h_v1_id = id;
    else if (mg->h_v1_id == id) mg->h_v1.clear(), mg->h_v1_id = 0;
    if (v) mg->h_vl1[id].assign(v, v + 7 * n3);
    else mg->h_vl1.erase(id);
  }
  if (!v) return AFH_OK;
  AFH_HIP(hipMalloc(&mg->h_vp[id - 1], sizeof(double) * 7 * n3));
  AFH_HIP(hipMemcpy(mg->h_vp[id - 1], v, sizeof(double) * 7 * n3,
                    hipMemcpyHostToDevice));
  if (bc_correction) {
    AFH_HIP(hipMalloc(&mg->h_bp[id - 1], sizeof(double) * n3));
    AFH_HIP(hipMemcpy(mg->h_bp[id - 1], bc_correction, sizeof(double) * n3,
                      hipMemcpyHostToDevice));
  }
  return AFH_OK;
}

int32_t afh_mg_set_box_lsf(afh_mg *mg, int32_t id, int32_t n, const int32_t *ix,
                           const double *dd, const double *bval, int32_t i_lsf) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  AFH_LIVE(mg->t, "afh_mg_set_box_lsf");
  if (id < 1 || id > mg->t->nb || n < 0)
    return set_error(AFH_ERR_ARG, "bad box id / count");
  afh_tree *t = mg->t;
  const size_t n3 = (size_t)t->nc * t->nc * t->nc;
  AFH_HIP(hipStreamSynchronize(t->stream));
  hipFree(mg->h_ix[id - 1]), hipFree(mg->h_dd[id - 1]), hipFree(mg->h_bv[id - 1]);
  mg->h_ix[id - 1] = nullptr, mg->h_dd[id - 1] = mg->h_bv[id - 1] = nullptr;
  mg->h_lsf_n[id - 1] = 0;
  mg->var_dirty = true;
  if (n == 0) return AFH_OK;
  if (!ix || !dd || !bval || i_lsf < 1 || i_lsf > t->nvc)
    return set_error(AFH_ERR_ARG, "afh_mg_set_box_lsf: bad argument");
  for (int q = 0; q < 3 * n; q++)
    if (ix[q] < 1 || ix[q] > t->nc)
      return set_error(AFH_ERR_ARG, "cell index out of box");
  AFH_HIP(hipMalloc(&mg->h_ix[id - 1], sizeof(int32_t) * 3 * n));
  AFH_HIP(hipMemcpy(mg->h_ix[id - 1], ix, sizeof(int32_t) * 3 * n,
                    hipMemcpyHostToDevice));
  AFH_HIP(hipMalloc(&mg->h_dd[id - 1], sizeof(double) * 6 * n));
  AFH_HIP(hipMemcpy(mg->h_dd[id - 1], dd, sizeof(double) * 6 * n,
                    hipMemcpyHostToDevice));
  AFH_HIP(hipMalloc(&mg->h_bv[id - 1], sizeof(double) * n3));
  AFH_HIP(hipMemcpy(mg->h_bv[id - 1], bval, sizeof(double) * n3,
                    hipMemcpyHostToDevice));
  mg->h_lsf_n[id - 1] = n;
  mg->i_lsf = i_lsf;
  return AFH_OK;
}

}  // extern "C"

// photoi_helmh_compute (src/m_photoi_helmh.f90:162-204): the mode loop of
// Helmholtz FAS-FMG solves and the sum of the modes into the
// photoionization rate
namespace afh {
// y -= c * x over whole boxes (ghost cells included) of the listed boxes
__global__ void k_box_axpy(double *__restrict__ y, const double *__restrict__ x,
                           double c, const int32_t *__restrict__ ids, size_t bsz) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bsz) return;
  const size_t q = (size_t)(ids[blockIdx.y] - 1) * bsz + t;
  y[q] = y[q] - c * x[q];
}
}  // namespace afh

extern "C" {

// one FMG of mode mg issued on stream st with its own spare image (the
// tree's stream and spare image swapped in for the issue, restored after)
static int32_t fmg_on(afh_mg *mg, hipStream_t st) {
  afh_tree *t = mg->t;
  hipStream_t s0 = t->stream;
  double *a0 = t->alt, *m0 = mg->alt;
  t->stream = st;
  if (mg->alt_priv) t->alt = mg->alt = mg->alt_priv;
  const int32_t e = afh_mg_fas_fmg(mg, 1, 1);
  t->stream = s0;
  t->alt = a0, mg->alt = m0;
  return e;
}

int32_t afh_photoi_helmh_compute(afh_mg *const *modes, int32_t n_modes,
                                 const double *coeffs, int32_t i_photo,
                                 double max_rel_res, int32_t max_fmg,
                                 int32_t *n_fmg) {
  if (!modes || n_modes < 1 || !coeffs || max_fmg < 1)
    return set_error(AFH_ERR_ARG, "afh_photoi_helmh_compute: bad argument");
  afh_tree *t = modes[0] ? modes[0]->t : nullptr;
  AFH_LIVE(t, "afh_photoi_helmh_compute");
  for (int n = 0; n < n_modes; n++)
    if (!modes[n] || modes[n]->t != t)
      return set_error(AFH_ERR_ARG, "helmholtz modes must share one tree");
  if (i_photo < 1 || i_photo > t->nvc) return set_error(AFH_ERR_ARG, "bad i_photo");
  t->touch(i_photo);
  // af_tree_clear_cc(tree, i_photo)
  AFH_HIP(hipMemsetAsync(t->ccv(i_photo), 0, sizeof(double) * t->bsz * t->nb, t->stream));
  // the source is the last mode's rhs (photoi_set_src's i_rhs); modes with
  // an rhs and a tmp variable of their own get a copy of it and run
  // concurrently, one side stream each (unsharded trees, at most 4 modes):
  // every mode's solve is the same as alone, the sum below keeps the mode
  // order, and the shared variables end as the last mode leaves them
  const int src = modes[n_modes - 1]->d.i_rhs;
  bool conc = !t->hook && n_modes > 1 && n_modes <= 4;
  for (int n = 0; n < n_modes && conc; n++)
    for (int m = n + 1; m < n_modes; m++)
      if (modes[n]->d.i_rhs == modes[m]->d.i_rhs || modes[n]->d.i_tmp == modes[m]->d.i_tmp)
        conc = false;
  int32_t e;
  for (int n = 0; n + 1 < n_modes; n++)
    if (modes[n]->d.i_rhs != src) {
      t->touch(modes[n]->d.i_rhs);
      AFH_HIP(hipMemcpyAsync(t->ccv(modes[n]->d.i_rhs), t->ccv(src),
                             sizeof(double) * t->bsz * t->nb, hipMemcpyDeviceToDevice,
                             t->stream));
    }
  double max_rhs;
  if ((e = afh_tree_maxabs_cc(t, src, &max_rhs))) return e;
  max_rhs = std::max(max_rhs, std::sqrt(DBL_EPSILON));
  std::vector<int> done(n_modes, 0);
  if (conc) {
    for (int n = 0; n < n_modes; n++)
      if (!t->side[n]) AFH_HIP(hipStreamCreateWithFlags(&t->side[n], hipStreamNonBlocking));
    for (int n = 0; n <= n_modes; n++)
      if (!t->side_ev[n]) AFH_HIP(hipEventCreateWithFlags(&t->side_ev[n], hipEventDisableTiming));
    for (int n = 0; n + 1 < n_modes; n++)
      if (!modes[n]->alt_priv && modes[n]->alt) {
        const size_t bytes = (size_t)t->nb * t->bsz * sizeof(double);
        AFH_HIP(hipMalloc(&modes[n]->alt_priv, bytes));
        AFH_HIP(hipMemsetAsync(modes[n]->alt_priv, 0, bytes, t->stream));
      }
    // fork: every side stream after the work so far; join: the tree's
    // stream after every side stream
    AFH_HIP(hipEventRecord(t->side_ev[n_modes], t->stream));
    for (int n = 0; n < n_modes; n++) {
      AFH_HIP(hipStreamWaitEvent(t->side[n], t->side_ev[n_modes], 0));
      if ((e = fmg_on(modes[n], t->side[n]))) return e;
      AFH_HIP(hipEventRecord(t->side_ev[n], t->side[n]));
    }
    for (int n = 0; n < n_modes; n++) AFH_HIP(hipStreamWaitEvent(t->stream, t->side_ev[n], 0));
    for (int n = 0; n < n_modes; n++) {
      double residu;
      if ((e = afh_tree_maxabs_cc(t, modes[n]->d.i_tmp, &residu))) return e;
      done[n] = residu / max_rhs < max_rel_res ? 1 : 0;
    }
  }
  for (int n = 0; n < n_modes; n++) {
    afh_mg *mg = modes[n];
    int i;
    for (i = conc ? 2 : 1; i <= max_fmg; i++) {
      if (conc && i == 2 && done[n]) {
        i = 1;
        break;
      }
      double residu;
      if ((e = fmg_on(mg, t->stream)) || (e = afh_tree_maxabs_cc(t, mg->d.i_tmp, &residu)))
        return e;
      if (residu / max_rhs < max_rel_res) break;
    }
    if (n_fmg) n_fmg[n] = std::min(i, max_fmg);
    for (int l = 1; l <= t->nlvl; l++) {
      const int nl = t->leaves.n(l);
      if (!nl) continue;
      hipLaunchKernelGGL(k_box_axpy, dim3((unsigned)((t->bsz + 255) / 256), nl),
                         dim3(256), 0, t->stream, t->ccv(i_photo),
                         t->ccv(mg->d.i_phi), coeffs[n], t->leaves.at(l), t->bsz);
      AFH_LAUNCH_CHECK("k_box_axpy");
    }
  }
  return AFH_OK;
}

}  // extern "C"
