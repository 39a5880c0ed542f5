// libafivo_hip_2d.so -- the NDIM = 2 build of the hot path (BASELINE config
// 1: programs/standard_2d; the reference builds afivo/lib_2d from the same
// sources with NDIM=2, afivo/lib_2d/Makefile). Same C ABI as the 3-D library
// (include/afivo_hip.h, the subset include/afivo_hip_2d.h lists), with the
// 2-D conventions there: a box holds box%cc(0:nc+1, 0:nc+1, iv) (i fastest),
// box%fc(1:nc+1, 1:nc+1, 1:2, ivf), the first 4 / 4 / 9 / 2 entries of
// afh_box_meta's children / neighbors / neighbor_mat / ix, r_min, dr.
//
// Device layout (HBM): cc pool [iv][box][j][i], (nc+2)^2 doubles per box;
// fc pool [ivf][box][dim][j][i], (nc+1)^2 per dim; gc2 (second ghost layer
// of the flux species) [box][4][nc]. Boxes of 2-D configs are small (8^2 in
// every standard_2d cfg): one thread per cell (or per ghost cell / face
// cell), a grid of (cells / 256, boxes of the level list). Expressions are
// evaluated in the order the Fortran writes them; built with
// -ffp-contract=off, so results are bitwise those of the reference's 2-D
// box routines (tests/test_2d.py against the golden vectors of
// oracle/harness/golden_gen2d.f90), the coarse solve aside.
//
//   k2_gc         af_gc_box sides (m_af_ghostcell.f90:64-120): neighbour copy,
//                 bc_to_gc (173-245), af_gc_interp / af_gc_interp_lim
//                 (394-451, 503-558), mg_sides_rb (m_af_multigrid.f90:294-417)
//   k2_corners    af_gc_box_corner + af_corner_gc_extrap (125-170, 860-871)
//   k2_gsrb       stencil_gsrb_357, 2-D constant branch (m_af_stencil.f90:909-922)
//   k2_residual   residual_box = rhs - stencil_apply_357 (m_af_multigrid.f90:801-810,
//                 m_af_stencil.f90:421-431), optional leaf max|res|
//   k2_rstr_fas   update_coarse's residual + af_restrict_box of tmp and phi
//                 (m_af_multigrid.f90:691-727, m_af_restrict.f90:62-103)
//   k2_parent_rhs rhs = L phi + tmp, tmp = phi on the parents (728-737)
//   k2_corr       correct_children: tmp = phi - tmp, phi += prolong_248
//                 (624-646, m_af_stencil.f90:716-731, [9, 3, 3, 1] / 16)
//   k2_cs_direct  level-1 solve (replaces HYPRE; exact separable transforms,
//                 as the 3-D AFH_COARSE_DIRECT) in one workgroup
//   k2_gradient   mg_box_lpl_gradient + mg_box_field_norm (1882-1900, 1995-2010)
//   k2_set_rhs    field_set_rhs (src/m_field.f90:363-401)
//   k2_gc2        af_gc2_box (m_af_ghostcell.f90:672-744), bc_to_gc2 (329-341),
//                 gc2_prolong_rb (798-818)
//   k2_flux       flux_upwind_box (m_af_flux_schemes.f90:715-848) with the
//                 m_fluid callbacks (src/m_fluid.f90:102-227), Koren
//   k2_consistent af_consistent_fluxes / flux_from_children (m_af_core.f90:1257-1357)
//   k2_update     flux_update_densities (m_af_flux_schemes.f90:320-394) +
//                 add_source_terms / get_rates / get_derivatives (field forms)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/afivo_hip_2d.h"
#include "afh_pfmg_dev.h"

namespace afh2 {

static thread_local std::string g_err;

int32_t set_error(int32_t code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int32_t check_hip(hipError_t e, const char *what) {
  return set_error(AFH_ERR_DEVICE, "%s: %s", what, hipGetErrorString(e));
}

#define H2(call)                                                              \
  do {                                                                        \
    hipError_t _e = (call);                                                   \
    if (_e != hipSuccess) return ::afh2::check_hip(_e, #call);                \
  } while (0)
#define H2_LAUNCH(what)                                                       \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) return ::afh2::check_hip(_e, what);                 \
  } while (0)

constexpr int NT = 256;          // threads per workgroup
constexpr int RED_SHARDS = 256;  // shards of one reduction slot
constexpr int RED_SLOTS = 4;     // 0 cfl max, 1 sigma max, 2 chem min, 3 |x| max
constexpr int MAXS = AFH_MAX_SPECIES;
constexpr int MAXPREV = 4;
constexpr int CS2_CELLS = 4096;  // level-1 grids the one-workgroup solve holds

// ------------------------------------------------------------ device helpers
__device__ __forceinline__ int red_shard() {
  return (int)((blockIdx.x + gridDim.x * blockIdx.y) & (RED_SHARDS - 1));
}
__device__ __forceinline__ unsigned long long dbl_to_ord(double x) {
  unsigned long long u = __double_as_longlong(x);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
inline double ord_to_dbl(unsigned long long o) {
  unsigned long long u = (o & 0x8000000000000000ull) ? (o & ~0x8000000000000000ull) : ~o;
  double d;
  memcpy(&d, &u, sizeof d);
  return d;
}
inline unsigned long long host_ord(double x) {
  unsigned long long u;
  memcpy(&u, &x, sizeof u);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
// fold a per-thread max (MAXV) or min into shard red_shard() of `red`; every
// thread of the (NT-thread) workgroup calls
template <bool MAXV>
__device__ __forceinline__ void block_fold(double v, unsigned long long *red) {
  // (a kernel may fold twice: the partials of the first fold are read by
  // thread 0 before any wave writes the second's)
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    const double w = __shfl_xor(v, o, 64);
    v = MAXV ? fmax(v, w) : fmin(v, w);
  }
  __shared__ double s_red[NT / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s_red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < (int)(blockDim.x >> 6); q++)
      v = MAXV ? fmax(v, s_red[q]) : fmin(v, s_red[q]);
    if (MAXV) atomicMax(&red[red_shard()], dbl_to_ord(v));
    else atomicMin(&red[red_shard()], dbl_to_ord(v));
  }
}

__device__ __forceinline__ int ix2(int ng, int i, int j) { return j * ng + i; }

// af_limiter_apply (m_af_limiters.f90:41-149)
__device__ __forceinline__ double limiter(int lim, double a, double b) {
  const double third = 1 / 3.0;
  switch (lim) {
  case AFH_LIM_KOREN: {
    const double aa = a * a, ab = a * b;
    if (ab <= 0) return 0;
    if (aa <= 0.25 * ab) return 2 * a;
    if (aa <= 2.5 * ab) return third * (b + 2 * a);
    return 2 * b;
  }
  case AFH_LIM_VANLEER: {
    const double ab = a * b;
    return ab > 0 ? 2 * ab / (a + b) : 0;
  }
  case AFH_LIM_NONE: return 0.5 * (a + b);
  case AFH_LIM_ZERO: return 0.0;
  default: {
    const double th = lim == AFH_LIM_MINMOD ? 1.0 : lim == AFH_LIM_MC ? 2.0 : 4 / 3.0;
    if (a * b > 0) {
      double m = fabs(th * a);
      const double y = fabs(th * b), z = fabs(0.5 * (a + b));
      if (y < m) m = y;
      if (z < m) m = z;
      return copysign(m, a);
    }
    return 0.0;
  }
  }
}

struct Bc4 {
  afh_bc bc[4];
  int rb, lim;
};

// ------------------------------------------------------------ ghost cells
// One thread per side ghost cell (4 nc per box). Every read is an interior
// cell (of this box, a neighbour, or the parent's neighbour), so the boxes of
// a level fill in parallel as the reference's OpenMP loop does.
__device__ __forceinline__ void gc2_side(double *__restrict__ v,
                                         const afh_box_meta *__restrict__ meta, int id, int t,
                                         int nc, int bsz, const Bc4 &g) {
  const int nb = t / nc + 1, a = t % nc + 1;
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ng = nc + 2, hnc = nc >> 1;
  const afh_box_meta &m = meta[id - 1];
  double *c = v + (size_t)(id - 1) * bsz;
  // cell index along the face normal: ghost, first and second interior
  const int gi = low ? 0 : nc + 1, i1 = low ? 1 : nc, i2 = low ? 2 : nc - 1;
  auto at = [&](int n, int tg) { return d == 0 ? ix2(ng, n, tg) : ix2(ng, tg, n); };
  const int nb_id = m.neighbors[nb - 1];
  double val;
  if (nb_id > 0) {
    val = v[(size_t)(nb_id - 1) * bsz + at(low ? nc : 1, a)];
  } else if (nb_id < 0) {
    double c0, c1, c2;
    const afh_bc bc = g.bc[nb - 1];
    switch (bc.type) {
    case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = 0; break;
    case AFH_BC_NEUMANN: c0 = m.dr[d] * (low ? -1 : 1); c1 = 1; c2 = 0; break;
    case AFH_BC_CONTINUOUS: c0 = 0; c1 = 2; c2 = -1; break;
    default: c0 = 1; c1 = 0; c2 = 0; break;  // AFH_BC_DIRICHLET_COPY
    }
    val = c0 * bc.value + c1 * c[at(i1, a)] + c2 * c[at(i2, a)];
  } else {
    const int p_nb = meta[m.parent - 1].neighbors[nb - 1];
    const double *cp = v + (size_t)(p_nb - 1) * bsz;
    const int ix_c = low ? nc : 1;
    // the tangential offset of this child in its parent (af_get_child_offset)
    const int td = 1 - d;
    const int off = ((m.ix[td] - 1) & 1) * hnc;
    if (g.rb == AFH_RB_MG_SIDES) {
      // mg_sides_rb: tmp(q) = coarse(ix_c, off + q), slope 0.125 (tmp(q+1) - tmp(q-1))
      const int q = (a + 1) >> 1;
      const double tq = cp[at(ix_c, off + q)];
      const double grad = 0.125 * (cp[at(ix_c, off + q + 1)] - cp[at(ix_c, off + q - 1)]);
      const double gcv = (a & 1) ? tq - grad : tq + grad;
      val = 0.5 * gcv + 0.75 * c[at(i1, a)] - 0.25 * c[at(i2, a)];
    } else {
      const double sixth = 1 / 6.0, third = 1 / 3.0;
      const int c1i = off + ((a + 1) >> 1), c2i = c1i + 1 - 2 * (a & 1);
      const double a1 = cp[at(ix_c, c1i)], a2 = cp[at(ix_c, c2i)];
      val = 0.5 * a1 + sixth * a2 + third * c[at(i1, a)];
      if (g.rb == AFH_RB_GC_INTERP_LIM && val > 2 * a1) val = 2 * a1;
    }
  }
  c[at(gi, a)] = val;
}

__global__ void __launch_bounds__(NT)
    k2_gc(double *__restrict__ v, const afh_box_meta *__restrict__ meta,
          const int32_t *__restrict__ ids, int nc, int bsz, Bc4 g) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 4 * nc) return;
  gc2_side(v, meta, ids[blockIdx.y], t, nc, bsz, g);
}

// af_gc_box_corner (2-D): copy from the diagonal neighbour, or extrapolate
// from the side ghost cells (af_corner_gc_extrap); one thread per corner
__device__ __forceinline__ double gc2_corner_val(const double *__restrict__ v,
                                                 const afh_box_meta *__restrict__ meta, int id,
                                                 int cn, int nc, int bsz) {
  const int dx = cn & 1, dy = cn >> 1;  // af_child_dix of corner cn + 1
  const int ng = nc + 2;
  const int ix = dx * (nc + 1), iy = dy * (nc + 1);
  const int nb_id = meta[id - 1].neighbor_mat[(2 * dx) + 3 * (2 * dy)];
  const double *c = v + (size_t)(id - 1) * bsz;
  if (nb_id > 0) {
    const int sx = 2 * dx - 1, sy = 2 * dy - 1;
    return v[(size_t)(nb_id - 1) * bsz + ix2(ng, ix - sx * nc, iy - sy * nc)];
  }
  const int di = 1 - 2 * (ix & 1), dj = 1 - 2 * (iy & 1);
  return c[ix2(ng, ix + di, iy)] + c[ix2(ng, ix, iy + dj)] - c[ix2(ng, ix + di, iy + dj)];
}

__device__ __forceinline__ void gc2_corner(double *__restrict__ v,
                                           const afh_box_meta *__restrict__ meta, int id,
                                           int cn, int nc, int bsz) {
  const int ng = nc + 2, ix = (cn & 1) * (nc + 1), iy = (cn >> 1) * (nc + 1);
  const double val = gc2_corner_val(v, meta, id, cn, nc, bsz);
  v[(size_t)(id - 1) * bsz + ix2(ng, ix, iy)] = val;
}

__global__ void k2_corners(double *__restrict__ v, const afh_box_meta *__restrict__ meta,
                           const int32_t *__restrict__ ids, int n, int nc, int bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 4 * n) return;
  gc2_corner(v, meta, ids[t >> 2], t & 3, nc, bsz);
}

// A level fill with corners in one launch: one workgroup per box, its side
// ghosts (k2_gc), a barrier, its corners (k2_corners: a diagonal
// neighbour's interior cell, or extrapolated from this box's side ghosts).
// The side ghosts read interior cells only, so boxes need not wait for each
// other; the same values as the two launches (AFH2_GC_BOX=0). per > 1: per
// boxes in one workgroup, 4 nc lanes each (8^2 boxes: 8 per 256 lanes, all
// lanes busy and a quarter of the waves of one 64-lane workgroup per box)
__global__ void __launch_bounds__(256)
    k2_gc_box(double *__restrict__ v, const afh_box_meta *__restrict__ meta,
              const int32_t *__restrict__ ids, int n, int per, int nc, int bsz, Bc4 g) {
  const int L = 4 * nc;
  if (per > 1) {
    const int sub = threadIdx.x / L, b = blockIdx.x * per + sub;
    if (sub < per && b < n) gc2_side(v, meta, ids[b], threadIdx.x % L, nc, bsz, g);
  } else {
    const int id = ids[blockIdx.x];
    for (int t = threadIdx.x; t < L; t += blockDim.x) gc2_side(v, meta, id, t, nc, bsz, g);
  }
  __syncthreads();
  const int b = blockIdx.x * per + (threadIdx.x >> 2);
  if ((int)threadIdx.x < 4 * per && b < n) gc2_corner(v, meta, ids[b], threadIdx.x & 3, nc, bsz);
}

// ------------------------------------------------------------ multigrid
struct Coef2 {
  double c[5];  // (i,j), (i-1,j), (i+1,j), (i,j-1), (i,j+1)
  double inv_c1;
};

__global__ void __launch_bounds__(NT)
    k2_gsrb(double *__restrict__ phi, const double *__restrict__ rhs,
            const int32_t *__restrict__ ids, int nc, int bsz, Coef2 cf, int redblack) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int half = nc >> 1;
  if (t >= nc * half) return;
  const int j = t / half + 1, q = t % half;
  const int i0 = 2 - ((redblack ^ j) & 1);  // i0 = 2 - iand(ieor(redblack, j), 1)
  const int i = i0 + 2 * q;
  const int ng = nc + 2;
  const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz;
  double *p = phi + o;
  const int x = ix2(ng, i, j);
  p[x] = (rhs[o + x] - cf.c[1] * p[x - 1] - cf.c[2] * p[x + 1] - cf.c[3] * p[x - ng] -
          cf.c[4] * p[x + ng]) *
         cf.inv_c1;
}

// A face ghost of box m the level fill would write (k2_gc's physical and
// refinement branches), from the box's cells x1, x2 next to the face
__device__ __forceinline__ double gc2_face(const double *__restrict__ coarse,
                                          const afh_box_meta *__restrict__ meta,
                                          const afh_box_meta &m, int nb, int nb_id, int a,
                                          double x1, double x2, int nc, int bsz,
                                          const Bc4 &g) {
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ng = nc + 2, hnc = nc >> 1;
  auto at = [&](int n, int tg) { return d == 0 ? ix2(ng, n, tg) : ix2(ng, tg, n); };
  if (nb_id < 0) {
    double c0, c1, c2;
    const afh_bc bc = g.bc[nb - 1];
    switch (bc.type) {
    case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = 0; break;
    case AFH_BC_NEUMANN: c0 = m.dr[d] * (low ? -1 : 1); c1 = 1; c2 = 0; break;
    case AFH_BC_CONTINUOUS: c0 = 0; c1 = 2; c2 = -1; break;
    default: c0 = 1; c1 = 0; c2 = 0; break;  // AFH_BC_DIRICHLET_COPY
    }
    return c0 * bc.value + c1 * x1 + c2 * x2;
  }
  const int p_nb = meta[m.parent - 1].neighbors[nb - 1];
  const double *cp = coarse + (size_t)(p_nb - 1) * bsz;
  const int ix_c = low ? nc : 1;
  const int td = 1 - d;
  const int off = ((m.ix[td] - 1) & 1) * hnc;
  if (g.rb == AFH_RB_MG_SIDES) {
    const int q = (a + 1) >> 1;
    const double tq = cp[at(ix_c, off + q)];
    const double grad = 0.125 * (cp[at(ix_c, off + q + 1)] - cp[at(ix_c, off + q - 1)]);
    const double gcv = (a & 1) ? tq - grad : tq + grad;
    return 0.5 * gcv + 0.75 * x1 - 0.25 * x2;
  }
  const double sixth = 1 / 6.0, third = 1 / 3.0;
  const int c1i = off + ((a + 1) >> 1), c2i = c1i + 1 - 2 * (a & 1);
  const double a1 = cp[at(ix_c, c1i)], a2 = cp[at(ix_c, c2i)];
  double val = 0.5 * a1 + sixth * a2 + third * x1;
  if (g.rb == AFH_RB_GC_INTERP_LIM && val > 2 * a1) val = 2 * a1;
  return val;
}

// Two half-sweeps of a small box (odd cells i + j odd, then even) and the
// level fills after each, in one workgroup, the box image in LDS: A the odd
// cells | B the odd face ghosts the fill after A would give -- a same-level
// neighbour's odd boundary cell recomputed from its own image in src (its
// ghost facing this box included, so stale ghost cells give the split
// half-sweeps' numbers too), physical / refinement faces from x1 (even,
// old), x2 (odd, new) | C the even cells | store: the interior and the
// corners to dst, and the face ghosts the fill after C would write --
// pushed into the same-level neighbour's ghost layer, or this box's own
// physical / refinement value. Every box of the level is in the launch and
// every face ghost has one writer. src -> dst (phi / spare image, alternating
// per pair); the coarse data of refinement faces are read from phi (the
// coarser level, not written here). Bitwise k2_gsrb + k2_gc twice.
// LPB lanes per box, 64 / LPB boxes per one-wave workgroup (8^2 boxes: 32
// lanes, one per cell of a half-sweep, two boxes per wave; the lanes of a
// missing last box load a copy of box n and store nothing)
template <int NC, int LPB = 64>
__global__ void __launch_bounds__(64)
    k2_pair_box(const double *__restrict__ src, double *__restrict__ dst,
                const double *__restrict__ rhs, const double *__restrict__ coarse,
                const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids,
                int n, int bsz, Coef2 cf, Bc4 g) {
  constexpr int NG = NC + 2, NB = NG * NG, NT = LPB, H = NC / 2, PW = 64 / LPB;
  __shared__ double P_[PW][NB];
  const int sub = threadIdx.x / LPB, tid = threadIdx.x % LPB;
  const int bidx = blockIdx.x * PW + sub;
  const bool valid = bidx < n;
  double *P = P_[sub];
  const int id = ids[valid ? bidx : n - 1];
  const afh_box_meta &m = meta[id - 1];
  const double *x = src + (size_t)(id - 1) * bsz, *r = rhs + (size_t)(id - 1) * bsz;
  double *y = dst + (size_t)(id - 1) * bsz;
  for (int e = tid; e < NB; e += NT) P[e] = x[e];
  // B inputs: the odd ghost u < 2 NC (face u / H + 1, its odd positions) of
  // a same-level neighbour -- the neighbour's boundary cell, its four
  // neighbours and rhs, loaded before A
  constexpr int NGH = 2 * NC, GPT = (NGH + NT - 1) / NT;
  double bl[GPT][5];
  for (int q = 0; q < GPT; q++) {
    const int u = tid + NT * q;
    for (int k = 0; k < 5; k++) bl[q][k] = 0.0;
    if (u >= NGH) continue;
    const int nb = u / H + 1, d = (nb - 1) >> 1;
    const bool low = ((nb - 1) & 1) == 0;
    const int gi = low ? 0 : NC + 1;
    const int a = 2 * (u % H) + 1 + ((gi & 1) ? 1 : 0);  // gi + a odd
    const int nid = m.neighbors[nb - 1];
    if (nid > 0) {
      auto at = [&](int n, int tg) { return d == 0 ? ix2(NG, n, tg) : ix2(NG, tg, n); };
      const double *xs = src + (size_t)(nid - 1) * bsz;
      const int c = at(low ? NC : 1, a);
      bl[q][0] = xs[c - 1];
      bl[q][1] = xs[c + 1];
      bl[q][2] = xs[c - NG];
      bl[q][3] = xs[c + NG];
      bl[q][4] = rhs[(size_t)(nid - 1) * bsz + c];
    }
  }
  __syncthreads();
  // A: odd cells (k2_gsrb with an odd red-black counter)
  for (int q = tid; q < NC * H; q += NT) {
    const int j = q / H + 1, i = 2 - ((1 ^ j) & 1) + 2 * (q % H);
    const int c = ix2(NG, i, j);
    P[c] = (r[c] - cf.c[1] * P[c - 1] - cf.c[2] * P[c + 1] - cf.c[3] * P[c - NG] -
            cf.c[4] * P[c + NG]) *
           cf.inv_c1;
  }
  __syncthreads();
  // B: odd face ghosts
  for (int q = 0; q < GPT; q++) {
    const int u = tid + NT * q;
    if (u >= NGH) continue;
    const int nb = u / H + 1, d = (nb - 1) >> 1;
    const bool low = ((nb - 1) & 1) == 0;
    const int gi = low ? 0 : NC + 1, i1 = low ? 1 : NC, i2 = low ? 2 : NC - 1;
    const int a = 2 * (u % H) + 1 + ((gi & 1) ? 1 : 0);
    auto at = [&](int n, int tg) { return d == 0 ? ix2(NG, n, tg) : ix2(NG, tg, n); };
    const int nid = m.neighbors[nb - 1];
    double v;
    if (nid > 0)
      v = (bl[q][4] - cf.c[1] * bl[q][0] - cf.c[2] * bl[q][1] - cf.c[3] * bl[q][2] -
           cf.c[4] * bl[q][3]) *
          cf.inv_c1;
    else
      v = gc2_face(coarse, meta, m, nb, nid, a, P[at(i1, a)], P[at(i2, a)], NC, bsz, g);
    P[at(gi, a)] = v;
  }
  __syncthreads();
  // C: even cells
  for (int q = tid; q < NC * H; q += NT) {
    const int j = q / H + 1, i = 2 - ((0 ^ j) & 1) + 2 * (q % H);
    const int c = ix2(NG, i, j);
    P[c] = (r[c] - cf.c[1] * P[c - 1] - cf.c[2] * P[c + 1] - cf.c[3] * P[c - NG] -
            cf.c[4] * P[c + NG]) *
           cf.inv_c1;
  }
  __syncthreads();
  // store: interior and corners; the four faces' ghosts pushed
  for (int e = tid; e < NB; e += NT) {
    const int i = e % NG, j = e / NG;
    const int nout = (i == 0 || i == NG - 1) + (j == 0 || j == NG - 1);
    if (valid && nout != 1) y[e] = P[e];
  }
  for (int u = valid ? tid : 4 * NC; u < 4 * NC; u += NT) {
    const int nb = u / NC + 1, a = u % NC + 1, d = (nb - 1) >> 1;
    const bool low = ((nb - 1) & 1) == 0;
    const int gi = low ? 0 : NC + 1, i1 = low ? 1 : NC, i2 = low ? 2 : NC - 1;
    auto at = [&](int n, int tg) { return d == 0 ? ix2(NG, n, tg) : ix2(NG, tg, n); };
    const int nid = m.neighbors[nb - 1];
    if (nid > 0)
      dst[(size_t)(nid - 1) * bsz + at(low ? NC + 1 : 0, a)] = P[at(i1, a)];
    else
      y[at(gi, a)] = gc2_face(coarse, meta, m, nb, nid, a, P[at(i1, a)], P[at(i2, a)], NC,
                              bsz, g);
  }
}

__device__ __forceinline__ double apply5(const double *p, int x, int ng, const Coef2 &cf) {
  return cf.c[0] * p[x] + cf.c[1] * p[x - 1] + cf.c[2] * p[x + 1] + cf.c[3] * p[x - ng] +
         cf.c[4] * p[x + ng];
}

// tmp = rhs - L phi on the interior; with `red` the max |tmp| is folded.
// lvl_c (with meta): the box's coefficients by its level -- boxes of every
// level in one launch (they do not interact here)
__global__ void __launch_bounds__(NT)
    k2_residual(const double *__restrict__ phi, const double *__restrict__ rhs,
                double *__restrict__ tmp, const int32_t *__restrict__ ids, int nc, int bsz,
                Coef2 cf, unsigned long long *red, const Coef2 *__restrict__ lvl_c,
                const afh_box_meta *__restrict__ meta) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double mx = 0.0;
  if (t < nc * nc) {
    const int i = t % nc + 1, j = t / nc + 1, ng = nc + 2;
    const int id = ids[blockIdx.y];
    const size_t o = (size_t)(id - 1) * bsz;
    const int x = ix2(ng, i, j);
    const double r = rhs[o + x] - apply5(phi + o, x, ng, lvl_c ? lvl_c[meta[id - 1].lvl - 1] : cf);
    tmp[o + x] = r;
    mx = fabs(r);
  }
  if (red) block_fold<true>(mx, red);
}

// update_coarse per child: the child's residual (not stored: the reference
// restores the child's tmp) restricted into the parent's tmp, phi restricted
// into the parent's phi; one thread per parent cell the child covers
__global__ void __launch_bounds__(NT)
    k2_rstr_fas(double *__restrict__ phi, const double *__restrict__ rhs,
                double *__restrict__ tmp, const afh_box_meta *__restrict__ meta,
                const int32_t *__restrict__ ids, int nc, int bsz, Coef2 cf) {
  const int hnc = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hnc * hnc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int ii = t % hnc + 1, jj = t / hnc + 1, ng = nc + 2;
  const int ic = ((m.ix[0] - 1) & 1) * hnc + ii, jc = ((m.ix[1] - 1) & 1) * hnc + jj;
  const int i_f = 2 * ii - 1, j_f = 2 * jj - 1;
  const size_t o = (size_t)(id - 1) * bsz, po = (size_t)(m.parent - 1) * bsz;
  const double *p = phi + o, *r = rhs + o;
  const int x00 = ix2(ng, i_f, j_f), x10 = x00 + 1, x01 = x00 + ng, x11 = x01 + 1;
  const double r00 = r[x00] - apply5(p, x00, ng, cf), r10 = r[x10] - apply5(p, x10, ng, cf),
               r01 = r[x01] - apply5(p, x01, ng, cf), r11 = r[x11] - apply5(p, x11, ng, cf);
  // 0.25 * sum(cc(i_f:i_f+1, j_f:j_f+1)): column-major section order
  tmp[po + ix2(ng, ic, jc)] = 0.25 * (r00 + r10 + r01 + r11);
  phi[po + ix2(ng, ic, jc)] = 0.25 * (p[x00] + p[x10] + p[x01] + p[x11]);
}

// af_restrict_box of variable v (children -> parent), one thread per parent
// cell of one child; ids = the children
__global__ void __launch_bounds__(NT)
    k2_restrict(double *__restrict__ v, const afh_box_meta *__restrict__ meta,
                const int32_t *__restrict__ ids, int nc, int bsz) {
  const int hnc = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hnc * hnc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int ii = t % hnc + 1, jj = t / hnc + 1, ng = nc + 2;
  const int ic = ((m.ix[0] - 1) & 1) * hnc + ii, jc = ((m.ix[1] - 1) & 1) * hnc + jj;
  const double *c = v + (size_t)(id - 1) * bsz;
  const int x00 = ix2(ng, 2 * ii - 1, 2 * jj - 1);
  v[(size_t)(m.parent - 1) * bsz + ix2(ng, ic, jc)] =
      0.25 * (c[x00] + c[x00 + 1] + c[x00 + ng] + c[x00 + ng + 1]);
}

// parents of the coarse level: rhs = L phi (interior), then rhs = rhs + tmp
// and (with `copy`) tmp = phi over the whole block (af_box_add_cc /
// af_box_copy_cc use DTIMES(:))
__global__ void __launch_bounds__(NT)
    k2_parent_rhs(const double *__restrict__ phi, double *__restrict__ rhs,
                  double *__restrict__ tmp, const int32_t *__restrict__ ids, int nc, int bsz,
                  Coef2 cf, int copy) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int ng = nc + 2;
  if (t >= ng * ng) return;
  const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz;
  const int i = t % ng, j = t / ng;
  double r = rhs[o + t];
  if (i >= 1 && i <= nc && j >= 1 && j <= nc) r = apply5(phi + o, t, ng, cf);
  rhs[o + t] = r + tmp[o + t];
  if (copy) tmp[o + t] = phi[o + t];
}

// whole-block copies (DTIMES(:)): mode 0 dst = a - b (correct_children's
// tmp = phi - tmp), 1 dst = a, 2 dst = 0
__global__ void __launch_bounds__(NT)
    k2_block(double *__restrict__ dst, const double *__restrict__ a,
             const double *__restrict__ b, const int32_t *__restrict__ ids, int bsz,
             int mode) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bsz) return;
  const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz + t;
  dst[o] = mode == 0 ? a[o] - b[o] : (mode == 1 ? a[o] : 0.0);
}

// correct_children's tmp = phi - tmp over parent boxes whose corner ghosts
// of phi are still to be filled (the up leg's corner pass after the fused
// pair, folded in): a corner thread forms the corner as k2_corners does --
// from the diagonal neighbour's interior or this box's side ghosts, neither
// written here -- stores it and uses it
__global__ void __launch_bounds__(NT)
    k2_block_corners(double *__restrict__ tmp, double *__restrict__ phi,
                     const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids,
                     int nc, int bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bsz) return;
  const int id = ids[blockIdx.y], ng = nc + 2, i = t % ng, j = t / ng;
  const size_t o = (size_t)(id - 1) * bsz + t;
  double p;
  if ((i == 0 || i == ng - 1) && (j == 0 || j == ng - 1)) {
    p = gc2_corner_val(phi, meta, id, (i ? 1 : 0) + (j ? 2 : 0), nc, bsz);
    phi[o] = p;
  } else {
    p = phi[o];
  }
  tmp[o] = p - tmp[o];
}

// max |x| over the interiors of a level's leaves (af_tree_maxabs_cc)
__global__ void __launch_bounds__(NT)
    k2_maxabs(const double *__restrict__ v, const int32_t *__restrict__ ids, int nc, int bsz,
              unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double mx = 0.0;
  if (t < nc * nc)
    mx = fabs(v[(size_t)(ids[blockIdx.y] - 1) * bsz + ix2(nc + 2, t % nc + 1, t / nc + 1)]);
  block_fold<true>(mx, red);
}

// phi(child) += prolong_248(tmp(parent)); ids = the children
__global__ void __launch_bounds__(NT)
    k2_prolong(double *__restrict__ phi, const double *__restrict__ tmp,
               const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids, int nc,
               int bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int i = t % nc + 1, j = t / nc + 1, ng = nc + 2, hnc = nc >> 1;
  const int i_c1 = ((m.ix[0] - 1) & 1) * hnc + ((i + 1) >> 1), i_c2 = i_c1 + 1 - 2 * (i & 1);
  const int j_c1 = ((m.ix[1] - 1) & 1) * hnc + ((j + 1) >> 1), j_c2 = j_c1 + 1 - 2 * (j & 1);
  const double *p = tmp + (size_t)(m.parent - 1) * bsz;
  const double c1 = 9 / 16.0, c2 = 3 / 16.0, c3 = 3 / 16.0, c4 = 1 / 16.0;
  double *c = phi + (size_t)(id - 1) * bsz + ix2(ng, i, j);
  *c = *c + c1 * p[ix2(ng, i_c1, j_c1)] + c2 * p[ix2(ng, i_c2, j_c1)] +
       c3 * p[ix2(ng, i_c1, j_c2)] + c4 * p[ix2(ng, i_c2, j_c2)];
}

// Level-1 solve of the folded operator, h_x T_x + h_y T_y - lambda (T the
// 1-D Laplacian with the boundary conditions folded in, as
// stencil_handle_boundaries does for HYPRE, m_coarse_solver.f90:442-491):
// gather rhs + boundary terms, Q_x^T, Q_y^T, divide by the eigenvalue sums,
// Q_y, Q_x, scatter -- in one workgroup, the grid in LDS
__global__ void __launch_bounds__(1024)
    k2_cs_direct(double *__restrict__ phi, const double *__restrict__ rhs,
                 const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids,
                 int nid, int nc, int bsz, int nx, int ny, double hx, double hy, Bc4 g,
                 const double *__restrict__ qx, const double *__restrict__ qy,
                 const double *__restrict__ ex, const double *__restrict__ ey, double lam) {
  __shared__ double A[CS2_CELLS], B[CS2_CELLS];
  const int n2 = nc * nc, ng = nc + 2;
  for (int u = threadIdx.x; u < nid * n2; u += blockDim.x) {
    const int id = ids[u / n2], t = u % n2;
    const afh_box_meta &m = meta[id - 1];
    const int i = t % nc + 1, j = t / nc + 1;
    const int gi[2] = {(m.ix[0] - 1) * nc + i, (m.ix[1] - 1) * nc + j};
    const int dims[2] = {nx, ny};
    const double hc[2] = {hx, hy};
    double rv = rhs[(size_t)(id - 1) * bsz + ix2(ng, i, j)];
    for (int nb = 1; nb <= 4; nb++) {
      const int dd = (nb - 1) >> 1;
      const bool low = ((nb - 1) & 1) == 0;
      const bool on = low ? (gi[dd] == 1) : (gi[dd] == dims[dd]);
      if (!on) continue;
      double b2r;
      if (g.bc[nb - 1].type == AFH_BC_DIRICHLET) b2r = -2 * hc[dd];
      else b2r = -(hc[dd] * m.dr[dd]) * (low ? -1 : 1);
      rv = rv + b2r * g.bc[nb - 1].value;
    }
    A[(gi[1] - 1) * nx + gi[0] - 1] = rv;
  }
  __syncthreads();
  const int N = nx * ny;
  // pass 0: x forward (A -> B), 1: y forward + divide (B -> A), 2: y inverse
  // (A -> B), 3: x inverse (B -> A); M[p][c] in q (forward: Q, out = sum_p
  // Q[p][c] in[p]; inverse: Q^T)
  for (int ps = 0; ps < 4; ps++) {
    const double *in = (ps & 1) ? B : A;
    double *out = (ps & 1) ? A : B;
    const bool xd = ps == 0 || ps == 3;
    const int n = xd ? nx : ny, st = xd ? 1 : nx;
    const double *M = xd ? qx : qy;
    const bool inv = ps >= 2;
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
      const int i = t % nx, j = t / nx;
      const int co = xd ? i : j;
      const double *src = in + (t - co * st);
      double s = 0.0;
      for (int p = 0; p < n; p++)
        s = s + (inv ? M[(size_t)co * n + p] : M[(size_t)p * n + co]) * src[p * st];
      if (ps == 1) {
        const double den = (ex[i] + ey[j]) - lam;
        s = den != 0.0 ? s / den : 0.0;
      }
      out[t] = s;
    }
    __syncthreads();
  }
  for (int u = threadIdx.x; u < nid * n2; u += blockDim.x) {
    const int id = ids[u / n2], t = u % n2;
    const afh_box_meta &m = meta[id - 1];
    const int i = t % nc + 1, j = t / nc + 1;
    phi[(size_t)(id - 1) * bsz + ix2(ng, i, j)] =
        A[((m.ix[1] - 1) * nc + j - 1) * nx + (m.ix[0] - 1) * nc + i - 1];
  }
}

// AFH_COARSE_PFMG: the reference's HYPRE StructPFMG restated
// (afh_pfmg_dev.h), the NDIM = 2 grid: gather rhs + boundary terms (the
// folded operator's coefficients, b2r per face) and phi, solve, scatter;
// the vectors and the wave levels' operators in LDS
__global__ void __launch_bounds__(1024)
    k2_cs_pfmg(const afh_pf::PfLvl *__restrict__ Lg, int nl, int wave_from,
               const double *__restrict__ A, const double *__restrict__ Pw,
               const double *__restrict__ b2r, const uint8_t *__restrict__ fmask,
               double *__restrict__ phi, const double *__restrict__ rhs,
               const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids, int nid,
               int nc, int bsz, Bc4 g, double tol, int max_iter, int *__restrict__ iters_out) {
  extern __shared__ double pf_sm[];
  __shared__ double slot;
  const afh_pf::PfLvl L0 = Lg[0];
  const int np = Lg[nl - 1].off + Lg[nl - 1].np;
  const int soff = wave_from < nl ? Lg[wave_from].off : np;
  double *X0 = pf_sm, *X1 = X0 + np, *b = X0 + 2 * np, *r = X0 + 3 * np;
  double *As = pf_sm + 4 * np;
  for (int u = threadIdx.x; u < 27 * (np - soff); u += blockDim.x)
    As[u] = A[(size_t)27 * soff + u];
  const int n2 = nc * nc, ng = nc + 2, nx = L0.n[0];
  for (int u = threadIdx.x; u < nid * n2; u += blockDim.x) {
    const int id = ids[u / n2], t = u % n2;
    const afh_box_meta &m = meta[id - 1];
    const int i = t % nc + 1, j = t / nc + 1;
    const int p = ((m.ix[1] - 1) * nc + j - 1) * nx + (m.ix[0] - 1) * nc + i - 1;
    const size_t c = (size_t)(id - 1) * bsz + ix2(ng, i, j);
    double rv = rhs[c];
    const int fm = fmask[p];
    for (int nb = 0; nb < 4; nb++)
      if ((fm >> nb) & 1) rv = rv + b2r[(size_t)nb * L0.np + p] * g.bc[nb].value;
    b[p] = rv;
    X0[p] = phi[c];
  }
  __syncthreads();
  int cur = 0;
  const int iters = afh_pf::pf_solve_block(Lg, nl, wave_from, A, As, soff, Pw, X0, X1, b, r,
                                           &slot, tol, max_iter, &cur);
  const double *x = cur ? X1 : X0;
  for (int u = threadIdx.x; u < nid * n2; u += blockDim.x) {
    const int id = ids[u / n2], t = u % n2;
    const afh_box_meta &m = meta[id - 1];
    const int i = t % nc + 1, j = t / nc + 1;
    phi[(size_t)(id - 1) * bsz + ix2(ng, i, j)] =
        x[((m.ix[1] - 1) * nc + j - 1) * nx + (m.ix[0] - 1) * nc + i - 1];
  }
  if (threadIdx.x == 0 && iters_out) *iters_out = iters;
}

// mg_box_lpl_gradient (fc = fac / dr * (phi_i - phi_{i-1})) + mg_box_field_norm
__global__ void __launch_bounds__(NT)
    k2_gradient(const double *__restrict__ phi, double *__restrict__ fc,
                double *__restrict__ norm, const afh_box_meta *__restrict__ meta,
                const int32_t *__restrict__ ids, int nc, int bsz, int fsz, double fac) {
  const int nf = nc + 1, ng = nc + 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nf * nf) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int i = t % nf + 1, j = t / nf + 1;
  const double *p = phi + (size_t)(id - 1) * bsz;
  double *f = fc + (size_t)(id - 1) * fsz;
  const double ix = fac / m.dr[0], iy = fac / m.dr[1];
  if (j <= nc) f[t] = ix * (p[ix2(ng, i, j)] - p[ix2(ng, i - 1, j)]);
  if (i <= nc) f[nf * nf + t] = iy * (p[ix2(ng, i, j)] - p[ix2(ng, i, j - 1)]);
  if (norm && i <= nc && j <= nc) {
    // the four faces of the cell, recomputed (bitwise the stored values)
    const double fx0 = ix * (p[ix2(ng, i, j)] - p[ix2(ng, i - 1, j)]);
    const double fx1 = ix * (p[ix2(ng, i + 1, j)] - p[ix2(ng, i, j)]);
    const double fy0 = iy * (p[ix2(ng, i, j)] - p[ix2(ng, i, j - 1)]);
    const double fy1 = iy * (p[ix2(ng, i, j + 1)] - p[ix2(ng, i, j)]);
    const double sx = fx0 + fx1, sy = fy0 + fy1;
    norm[(size_t)(id - 1) * bsz + ix2(ng, i, j)] = 0.5 * sqrt(sx * sx + sy * sy);
  }
}

// ------------------------------------------------------------ fluid
struct RhsArgs {
  int n;
  const double *sp[MAXS];
  double q[MAXS];
};

// field_set_rhs over the whole block (DTIMES(:)); max |rhs| of the interior
__global__ void __launch_bounds__(NT)
    k2_set_rhs(double *__restrict__ rhs, RhsArgs A, const int32_t *__restrict__ ids, int nc,
               int bsz, unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double mx = 0.0;
  if (t < bsz) {
    const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz + t;
    double r = 0.0;
    for (int s = 0; s < A.n; s++) r = r + A.q[s] * A.sp[s][o];
    rhs[o] = r;
    const int ng = nc + 2, i = t % ng, j = t / ng;
    if (i >= 1 && i <= nc && j >= 1 && j <= nc) mx = fabs(r);
  }
  if (red) block_fold<true>(mx, red);
}

// af_gc2_box: layer 1 written back into the box, layer 2 into gc2[box][nb][a]
__global__ void __launch_bounds__(NT)
    k2_gc2(double *__restrict__ v, double *__restrict__ gc2,
           const afh_box_meta *__restrict__ meta, const int32_t *__restrict__ ids, int nc,
           int bsz, Bc4 g) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 4 * nc) return;
  const int id = ids[blockIdx.y];
  const int nb = t / nc + 1, a = t % nc + 1;
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ng = nc + 2;
  const afh_box_meta &m = meta[id - 1];
  double *c = v + (size_t)(id - 1) * bsz;
  auto at = [&](int n, int tg) { return d == 0 ? ix2(ng, n, tg) : ix2(ng, tg, n); };
  const int nb_id = m.neighbors[nb - 1];
  double l1, l2;
  if (nb_id > 0) {
    const double *cn = v + (size_t)(nb_id - 1) * bsz;
    l1 = cn[at(low ? nc : 1, a)];
    l2 = cn[at(low ? nc - 1 : 2, a)];
  } else if (nb_id < 0) {
    double c0, c1, c2;
    const afh_bc bc = g.bc[nb - 1];
    switch (bc.type) {
    case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = c0; break;
    case AFH_BC_NEUMANN: c0 = m.dr[d] * (low ? -1 : 1); c1 = 1; c2 = 3 * c0; break;
    default: c0 = 1; c1 = 0; c2 = c0; break;
    }
    l1 = c0 * bc.value + c1 * c[at(low ? 1 : nc, a)];
    l2 = c2 * bc.value + c1 * c[at(low ? 2 : nc - 1, a)];
  } else {
    // gc2_prolong_rb: limited-slope prolongation from the parent's neighbour
    const int hnc = nc >> 1, td = 1 - d;
    const int p_nb = meta[m.parent - 1].neighbors[nb - 1];
    const double *cp = v + (size_t)(p_nb - 1) * bsz;
    const int tc = ((m.ix[td] - 1) & 1) * hnc + ((a + 1) >> 1);
    const int nc_ = low ? nc : 1;
    const int ci = d == 0 ? nc_ : tc, cj = d == 0 ? tc : nc_;
    const int q = ix2(ng, ci, cj);
    const double f0 = cp[q];
    const double fx = 0.25 * limiter(g.lim, cp[q] - cp[q - 1], cp[q + 1] - cp[q]);
    const double fy = 0.25 * limiter(g.lim, cp[q] - cp[q - ng], cp[q + ng] - cp[q]);
    // signs: - for the first fine cell of a pair, + for the second; along the
    // normal the layers are (-1, 0) low and (nc+1, nc+2) high
    const double st = (a & 1) ? -1.0 : 1.0;
    auto val = [&](double sn) {
      const double sx = d == 0 ? sn : st, sy = d == 0 ? st : sn;
      double r = f0;
      r = sx < 0 ? r - fx : r + fx;
      r = sy < 0 ? r - fy : r + fy;
      return r;
    };
    l1 = val(low ? 1.0 : -1.0);
    l2 = val(low ? -1.0 : 1.0);
  }
  c[at(low ? 0 : nc + 1, a)] = l1;
  gc2[((size_t)(id - 1) * 4 + (nb - 1)) * nc + (a - 1)] = l2;
}

struct DevLT {
  int n_points, n_cols;
  double x_min, inv_fac;
  const double *rc;
};

// LT_get_loc + LT_get_col_at_loc (m_lookup_table.f90:330-406)
__device__ __forceinline__ double lt_col(const DevLT &lt, int col, double x) {
  const double frac = (x - lt.x_min) * lt.inv_fac;
  int low;
  double lf;
  if (frac <= 0) {
    low = 1;
    lf = 1;
  } else if (frac >= lt.n_points - 1) {
    low = lt.n_points - 1;
    lf = 0;
  } else {
    low = (int)ceil(frac);
    lf = low - frac;
  }
  const double *r = lt.rc + (size_t)(col - 1) * lt.n_points;
  return lf * r[low - 1] + (1 - lf) * r[low];
}

struct FluxArgs {
  const double *ne, *E, *Ef;
  double *F;
  const double *gc2;
  DevLT td;
  double N_inv;
  int lim;
};

// mobility and diffusion at a face between cells with |E| Elo, Ehi
__device__ __forceinline__ void face_vd(const FluxArgs &A, double Elo, double Ehi, double ex,
                                        double &v, double &dc, double &mu) {
  const double tfc = 0.5 * (Elo + Ehi) * 1e21 * A.N_inv;
  mu = lt_col(A.td, 1, tfc) * A.N_inv;
  dc = lt_col(A.td, 2, tfc) * A.N_inv;
  v = -mu * ex;
}

// One thread per cell: the low face of the cell in x and y (and the high
// face on the last cell of a line), reconstruct_upwind_1d + the m_fluid
// flux_upwind callback; the CFL sum of the cell over both dimensions
// (cfl_sum = 0 + x term + y term) and the conductivity maximum are folded.
// (Round 4 measured taking the high face's velocity and diffusion from the
// next cell's lane: neutral, profiles/r04_ab_2d_flux_shfl.txt; removed.)
__global__ void __launch_bounds__(NT)
    k2_flux(FluxArgs A, const int32_t *__restrict__ ids, const afh_box_meta *__restrict__ meta,
            int nc, int bsz, int fsz, unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double cfl = -HUGE_VAL, smax = -HUGE_VAL;
  if (t < nc * nc) {
    const int id = ids[blockIdx.y];
    const int i = t % nc + 1, j = t / nc + 1, ng = nc + 2, nf = nc + 1;
    const size_t o = (size_t)(id - 1) * bsz;
    const double *ne = A.ne + o, *E = A.E + o;
    const double *Ef = A.Ef + (size_t)(id - 1) * fsz;
    double *F = A.F + (size_t)(id - 1) * fsz;
    const double *g2 = A.gc2 + (size_t)(id - 1) * 4 * nc;
    const double idx[2] = {1 / meta[id - 1].dr[0], 1 / meta[id - 1].dr[1]};
    const int c0 = ix2(ng, i, j);
    const int cc[2] = {i, j}, st[2] = {1, ng};
    // line position along d, the other index (1-based), face of the cell
    const int other[2] = {j, i};
    const int face[2] = {(j - 1) * nf + (i - 1), nf * nf + (j - 1) * nf + (i - 1)};
    const int fst[2] = {1, nf};
    cfl = 0.0;
    for (int d = 0; d < 2; d++) {
      const int c = cc[d];
      const double Lm2 = (c == 1) ? g2[(2 * d) * nc + other[d] - 1] : ne[c0 - 2 * st[d]];
      const double Lm1 = ne[c0 - st[d]], L0 = ne[c0], Lp1 = ne[c0 + st[d]];
      const double Lp2 = (c == nc) ? g2[(2 * d + 1) * nc + other[d] - 1] : ne[c0 + 2 * st[d]];
      // low face
      const double ex_lo = Ef[face[d]];
      double vl, dl, mul;
      face_vd(A, E[c0 - st[d]], E[c0], ex_lo, vl, dl, mul);
      double u;
      if (-1 * ex_lo > 0) u = Lm1 + 0.5 * limiter(A.lim, L0 - Lm1, Lm1 - Lm2);
      else u = L0 - 0.5 * limiter(A.lim, L0 - Lm1, Lp1 - L0);
      F[face[d]] = vl * u - dl * idx[d] * (L0 - Lm1);
      smax = fmax(smax, mul * u);
      // high face (evaluated by every cell for its CFL term; stored on the
      // last cell of the line)
      const double ex_hi = Ef[face[d] + fst[d]];
      double vh = 0.0, dh = 0.0, muh = 0.0;
      face_vd(A, E[c0], E[c0 + st[d]], ex_hi, vh, dh, muh);
      if (c == nc) {
        double uh;
        if (-1 * ex_hi > 0) uh = L0 + 0.5 * limiter(A.lim, Lp1 - L0, L0 - Lm1);
        else uh = Lp1 - 0.5 * limiter(A.lim, Lp1 - L0, Lp2 - Lp1);
        F[face[d] + fst[d]] = vh * uh - dh * idx[d] * (Lp1 - L0);
        smax = fmax(smax, muh * uh);
      }
      const double mv = fmax(fabs(vh), fabs(vl)), md = fmax(dh, dl);
      cfl = cfl + (1.0 * mv * idx[d] + 2 * md * (idx[d] * idx[d]));
    }
  }
  block_fold<true>(cfl, red);
  block_fold<true>(smax, red + RED_SHARDS);
}

// flux_from_children: the face fluxes of a leaf next to refined boxes are
// the mean of the two fine faces; task = (parent id << 3) | nb
__global__ void k2_consistent(double *__restrict__ F, const afh_box_meta *__restrict__ meta,
                              const int32_t *__restrict__ tasks, int ntask, int nc, int fsz) {
  const int nch = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask * 2 * nch) return;
  const int task = tasks[t / (2 * nch)], r = t % (2 * nch);
  const int id = task >> 3, nb = task & 7;
  const afh_box_meta &m = meta[id - 1];
  const int nb_id = m.neighbors[nb - 1];
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  // af_child_adj_nb(:, nb) (m_af_types.f90:136), af_child_dix (134)
  const int adj[4][2] = {{1, 3}, {2, 4}, {1, 2}, {3, 4}};
  const int cdix[4][2] = {{0, 0}, {1, 0}, {0, 1}, {1, 1}};
  const int ic = r / nch, n = r % nch + 1;
  const int i_ch = adj[nb - 1][ic];
  const int c_id = m.children[i_ch - 1];
  const int i = low ? 1 : nc + 1, i_nb = low ? nc + 1 : 1;
  const int nf = nc + 1;
  const double *fc = F + (size_t)(c_id - 1) * fsz + (size_t)d * nf * nf;
  double *fn = F + (size_t)(nb_id - 1) * fsz + (size_t)d * nf * nf;
  if (d == 0) {
    const int jn = nch * cdix[i_ch - 1][1] + n;
    fn[(jn - 1) * nf + (i_nb - 1)] =
        0.5 * (fc[(2 * n - 2) * nf + (i - 1)] + fc[(2 * n - 1) * nf + (i - 1)]);
  } else {
    const int in = nch * cdix[i_ch - 1][0] + n;
    fn[(i_nb - 1) * nf + (in - 1)] =
        0.5 * (fc[(i - 1) * nf + (2 * n - 2)] + fc[(i - 1) * nf + (2 * n - 1)]);
  }
}

struct DevReaction {
  int rate_type, table_col, n_in, n_out;
  double rate_factor, c[4];
  int ix_in[4], ix_out[4], mult_out[4];
};

struct UpdArgs {
  int ns, nr, n_prev, last_step, e_index;
  double w_prev[MAXPREV];
  const double *prev[MAXS][MAXPREV];
  const double *der[MAXS];
  double *out[MAXS];
  const double *E, *F;
  const DevReaction *reac;
  DevLT chem;
  double inv_N, dt, dt_chemistry_nmin;
};

// get_rates for the field forms (src/m_chemistry.f90:565-620)
__device__ __forceinline__ double rate_of(const UpdArgs &A, const DevReaction &R,
                                          double field) {
  const double c0 = R.rate_factor;
  const double *c = R.c;
  switch (R.rate_type) {
  case AFH_RATE_TABULATED_FIELD: return c0 * lt_col(A.chem, R.table_col, field);
  case AFH_RATE_CONSTANT: return c0 * c[0];
  case AFH_RATE_LINEAR: return c0 * c[0] * (field - c[1]);
  case AFH_RATE_EXP_V1: {
    const double z = c[1] / (c[2] + field);
    return c0 * c[0] * exp(-(z * z));
  }
  default: {  // AFH_RATE_EXP_V2
    const double z = field / c[1];
    return c0 * c[0] * exp(-(z * z));
  }
  }
}

// flux_update_densities + add_source_terms of one leaf cell: y = sum_m w_m
// y_prev_m, chemistry source dt * derivs (+ the chemistry limit on the last
// step), then the flux divergence of the electrons (flux species). NS: the
// species count when it is a compile-time case (the per-cell arrays then stay
// in registers; wave-uniform indices use VGPR index mode), MAXS for any count
// (A.ns; the arrays in scratch)
template <int NS>
__global__ void __launch_bounds__(NT)
    k2_update(UpdArgs A, const int32_t *__restrict__ ids, const afh_box_meta *__restrict__ meta,
              int nc, int bsz, int fsz, unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double cmin = 1e100;
  const int ns = NS == MAXS ? A.ns : NS;
  if (t < nc * nc) {
    const int id = ids[blockIdx.y];
    const int i = t % nc + 1, j = t / nc + 1, ng = nc + 2, nf = nc + 1;
    const size_t x = (size_t)(id - 1) * bsz + ix2(ng, i, j);
    double y[NS], dens[NS], der[NS];
#pragma unroll
    for (int s = 0; s < ns; s++) {
      double tmp = 0.0;
      for (int q = 0; q < A.n_prev; q++) tmp = tmp + A.w_prev[q] * A.prev[s][q][x];
      y[s] = tmp;
      const double v = A.der[s][x];
      dens[s] = v > 0.0 ? v : 0.0;
      der[s] = 0.0;
    }
    const double field = 1e21 * A.inv_N * A.E[x];
    for (int r = 0; r < A.nr; r++) {
      const DevReaction &R = A.reac[r];
      double rate = rate_of(A, R, field);
      double prod = 1.0;
      for (int q = 0; q < R.n_in; q++) prod = prod * dens[R.ix_in[q] - 1];
      rate = rate * prod;
      for (int q = 0; q < R.n_in; q++) der[R.ix_in[q] - 1] = der[R.ix_in[q] - 1] - rate;
      for (int q = 0; q < R.n_out; q++)
        der[R.ix_out[q] - 1] = der[R.ix_out[q] - 1] + rate * R.mult_out[q];
    }
    if (A.last_step) {
      const double eps = 1e-100;
#pragma unroll
      for (int s = 0; s < ns; s++) {
        double a, b;
        if (A.dt_chemistry_nmin > 0) {
          a = dens[s] + A.dt_chemistry_nmin;
          b = fabs(der[s]);
          b = b > eps ? b : eps;
        } else {
          a = dens[s] > eps ? dens[s] : eps;
          b = -der[s] > eps ? -der[s] : eps;
        }
        cmin = fmin(cmin, a / b);
      }
    }
#pragma unroll
    for (int s = 0; s < ns; s++) y[s] = y[s] + A.dt * der[s];
    const double *F = A.F + (size_t)(id - 1) * fsz;
    const int f0 = (j - 1) * nf + (i - 1), d2 = nf * nf;
    const double dtx = A.dt / meta[id - 1].dr[0], dty = A.dt / meta[id - 1].dr[1];
    const int e = A.e_index;
    y[e] = y[e] + dtx * (F[f0] - F[f0 + 1]) + dty * (F[d2 + f0] - F[d2 + f0 + nf]);
#pragma unroll
    for (int s = 0; s < ns; s++) A.out[s][x] = y[s];
  }
  if (A.last_step) block_fold<false>(cmin, red);
}

__global__ void k2_red_fill(unsigned long long *red, unsigned long long v) {
  red[threadIdx.x + blockIdx.x * blockDim.x] = v;
}

// fold the shards of n consecutive slots into red_out[slot]
__global__ void k2_red_fold(unsigned long long *red, int slot0, int n, int is_max,
                            unsigned long long *out) {
  __shared__ unsigned long long s[RED_SHARDS];
  for (int q = 0; q < n; q++) {
    const unsigned long long *r = red + (size_t)(slot0 + q) * RED_SHARDS;
    s[threadIdx.x] = r[threadIdx.x];
    __syncthreads();
    for (int h = RED_SHARDS / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) {
        const unsigned long long a = s[threadIdx.x], b = s[threadIdx.x + h];
        s[threadIdx.x] = (is_max >> q) & 1 ? (a > b ? a : b) : (a < b ? a : b);
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) out[q] = s[0];
    __syncthreads();
  }
}

struct LevelList {
  std::vector<int32_t> off;
  int32_t *d = nullptr;
  int n(int lvl) const { return off[lvl] - off[lvl - 1]; }
  const int32_t *at(int lvl) const { return d + off[lvl - 1]; }
};

struct Meth {
  int set = 0;
  afh_bc bc[4];
  int rb = AFH_RB_GC_INTERP;
  int lim = AFH_LIM_MC;  // af_set_cc_methods default in 2-D (m_af_core.f90:401-402)
  int prolong = AFH_PROLONG_NONE;  // afh_set_cc_prolong
  int prolong_lim = AFH_LIM_MC;
};

}  // namespace afh2

using namespace afh2;

struct afh_tree {
  int device = 0;
  hipStream_t stream = nullptr;
  bool gc_box = true;  // level fills with corners in one launch (k2_gc_box; AFH2_GC_BOX=0)
  bool gc_pack = true;  // several small boxes per k2_gc_box workgroup
  // a box has a refinement boundary (a side ghost then reads the parent
  // neighbour's tangential ghost, so levels fill in order)
  bool any_refb = false;
  // afh_gc_tree of a tree without refinement boundaries in one launch (every
  // read an interior cell or, for corners, the box's own side ghosts;
  // AFH2_GC_TREE_ONE=0 level by level)
  bool gc_tree_one = true;
  // bumped by afh_set_cc_methods / afh_set_bc: boundary values and types are
  // kernel arguments, so captured V-cycles of older generations are dropped
  uint64_t meth_gen = 0;
  int nc = 0, ng = 0, nb = 0, nlvl = 0, nvc = 0, nvf = 0;
  int bsz = 0, fsz = 0;
  int cgs[2] = {0, 0};
  std::vector<afh_box_meta> boxes;
  afh_box_meta *d_boxes = nullptr;
  LevelList ids, leaves, parents, refb, children_of, cflux;
  std::vector<std::vector<int32_t>> h_ids, h_leaves, h_parents;
  double *cc = nullptr, *fc = nullptr, *gc2 = nullptr;
  unsigned long long *red = nullptr, *red_out = nullptr, *h_red = nullptr;
  std::vector<Meth> meth;
  std::vector<int> auto_vars;  // tree%cc_auto_vars (afh_set_cc_prolong order)
  std::vector<double> lvl_dr;  // 2 per level
  double *d_boxred = nullptr;  // per-leaf (value, cell) of afh_tree_sum_cc / reduce_loc
  // kernel timing (afh_profile_enable/read, as in libafivo_hip): HIP events
  // around every launch of one kernel class on the tree's stream
  int prof_class = 0;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double prof_bytes = 0;
  int64_t prof_launches = 0;
  double *ccv(int iv) const { return cc + (size_t)(iv - 1) * nb * bsz; }
  double *fcv(int ivf) const { return fc + (size_t)(ivf - 1) * nb * fsz; }
  Bc4 bc4(int iv) const {
    Bc4 g;
    for (int q = 0; q < 4; q++) g.bc[q] = meth[iv].bc[q];
    g.rb = meth[iv].rb;
    g.lim = meth[iv].lim;
    return g;
  }
};

struct afh_mg {
  afh_tree *t = nullptr;
  afh_mg_desc d;
  std::vector<Coef2> lvl_c;
  Coef2 *d_lvl_c = nullptr;  // lvl_c on the device (residual of every level in one launch)
  bool all_lvl = true;       // AFH2_ALL_LVL=0: one residual / gradient launch per level
  // V-cycles replayed as hipGraphs (launch gaps of the ~70 small launches of
  // a config-1 V-cycle), one per (highest level, residual, max) variant;
  // AFH2_GRAPHS=0: eager. The first call of a variant runs eagerly (the
  // coarse-solve tables are built outside capture); a boundary-condition
  // change drops the graphs
  struct Graph {
    hipGraphExec_t exec = nullptr;
    bool warm = false;
    uint64_t gen = 0;
  };
  std::map<int, Graph> graphs;
  bool use_graphs = true;
  // the up leg's corner pass folded into the next level's correction
  // (k2_block_corners; AFH2_CORNER_FOLD=0 for k2_corners)
  bool corner_fold = true;
  int nx = 0, ny = 0;
  double *d_q[2] = {nullptr, nullptr}, *d_e[2] = {nullptr, nullptr};
  int q_bc[4] = {0, 0, 0, 0};
  // the fused pair (k2_pair_box; AFH_PAIR2D=0: the split half-sweeps) and
  // its spare phi image (config 1: 1.08-1.14 -> 0.85-0.87 ms per step,
  // profiles/r04_push_ab.txt)
  bool pair = true;
  double *alt = nullptr;
  // AFH_COARSE_PFMG (afh_pfmg_dev.h, k2_cs_pfmg): the hierarchy's device
  // tables, built for the boundary types pf_bc (b2r: the boundary values'
  // factors per face, fmask: the faces a point touches); iterations
  int pf_nl = 0, pf_lds = 0, pf_wave = 0, pf_bc[4] = {-1, -1, -1, -1};
  afh_pf::PfLvl *d_pf_lvl = nullptr;
  double *d_pf_A = nullptr, *d_pf_P = nullptr, *d_pf_b2r = nullptr;
  uint8_t *d_pf_fmask = nullptr;
  int *d_pf_iters = nullptr;
};

struct afh_fluid {
  afh_tree *t = nullptr;
  afh_fluid_desc d;
  double *d_td = nullptr, *d_chem = nullptr;
  DevReaction *d_reac = nullptr;
  // (k2_update is compiled for the species count, 1..12)
};

namespace afh2 {

// per-box launches: a workgroup of the work rounded up to whole waves (at
// most NT lanes), so a small box does not dispatch idle waves (8^2 boxes:
// one wave per box instead of four)
static inline int blk2n(int work) { return work >= NT ? NT : ((work + 63) / 64) * 64; }
static inline dim3 blk2(int work) { return dim3((unsigned)blk2n(work)); }
static inline dim3 grid2(int work, int nbox) {
  const int b = blk2n(work);
  return dim3((unsigned)((work + b - 1) / b), (unsigned)nbox);
}

static int32_t upload_list(LevelList &L, const std::vector<std::vector<int32_t>> &lists) {
  L.off.assign(lists.size() + 1, 0);
  std::vector<int32_t> flat;
  for (size_t l = 0; l < lists.size(); l++) {
    flat.insert(flat.end(), lists[l].begin(), lists[l].end());
    L.off[l + 1] = (int)flat.size();
  }
  if (L.d) hipFree(L.d);
  L.d = nullptr;
  if (!flat.empty()) {
    H2(hipMalloc(&L.d, flat.size() * sizeof(int32_t)));
    H2(hipMemcpy(L.d, flat.data(), flat.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  return AFH_OK;
}

static void prof_mark(afh_tree *t, int kc) {
  if (t->prof_class != kc) return;
  if (t->ev_used == t->ev_pool.size()) {
    hipEvent_t e;
    hipEventCreate(&e);
    t->ev_pool.push_back(e);
  }
  hipEventRecord(t->ev_pool[t->ev_used++], t->stream);
}

static void prof_end(afh_tree *t, int kc, double bytes) {
  if (t->prof_class != kc) return;
  prof_mark(t, kc);
  t->prof_bytes += bytes;
  t->prof_launches++;
}

static void free_list(LevelList &L) {
  if (L.d) hipFree(L.d);
  L.d = nullptr;
}

// lvl = 0: every level in one launch (afh_gc_tree without refinement
// boundaries)
static int32_t gc_lvl(afh_tree *t, int lvl, int iv, bool corners) {
  const int n = lvl ? t->ids.n(lvl) : t->ids.off[t->nlvl] - t->ids.off[0];
  if (!n) return AFH_OK;
  if (!lvl) lvl = 1;  // ids.at(1): the list of every level from level 1
  if (corners && t->gc_box) {
    const int L = 4 * t->nc, per = t->gc_pack && L <= 128 ? 256 / L : 1;
    hipLaunchKernelGGL(k2_gc_box, dim3((n + per - 1) / per), dim3(per > 1 ? per * L : 64), 0,
                       t->stream, t->ccv(iv), t->d_boxes, t->ids.at(lvl), n, per, t->nc,
                       t->bsz, t->bc4(iv));
    H2_LAUNCH("k2_gc_box");
    return AFH_OK;
  }
  hipLaunchKernelGGL(k2_gc, grid2(4 * t->nc, n), blk2(4 * t->nc), 0, t->stream, t->ccv(iv),
                     t->d_boxes, t->ids.at(lvl), t->nc, t->bsz, t->bc4(iv));
  H2_LAUNCH("k2_gc");
  if (corners) {
    hipLaunchKernelGGL(k2_corners, dim3((4 * n + NT - 1) / NT), dim3(NT), 0, t->stream,
                       t->ccv(iv), t->d_boxes, t->ids.at(lvl), n, t->nc, t->bsz);
    H2_LAUNCH("k2_corners");
  }
  return AFH_OK;
}

// nslot consecutive slots from slot to v, one launch
static int32_t red_init(afh_tree *t, int slot, double v, int nslot = 1) {
  hipLaunchKernelGGL(k2_red_fill, dim3(nslot), dim3(RED_SHARDS), 0, t->stream,
                     t->red + (size_t)slot * RED_SHARDS, host_ord(v));
  H2_LAUNCH("k2_red_fill");
  return AFH_OK;
}

// fold slots slot0 .. slot0+n-1 (bit q of is_max: slot q is a maximum) and
// read them
static int32_t red_read(afh_tree *t, int slot0, int n, int is_max, double *out) {
  hipLaunchKernelGGL(k2_red_fold, dim3(1), dim3(RED_SHARDS), 0, t->stream, t->red, slot0, n,
                     is_max, t->red_out);
  H2_LAUNCH("k2_red_fold");
  H2(hipMemcpyAsync(t->h_red, t->red_out, n * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost, t->stream));
  H2(hipStreamSynchronize(t->stream));
  for (int q = 0; q < n; q++) out[q] = ord_to_dbl(t->h_red[q]);
  return AFH_OK;
}

static int32_t check_iv(afh_tree *t, int iv, const char *what) {
  if (!t) return set_error(AFH_ERR_ARG, "%s: null tree", what);
  if (iv < 1 || iv > t->nvc) return set_error(AFH_ERR_ARG, "%s: bad variable %d", what, iv);
  return AFH_OK;
}

}  // namespace afh2

// ============================================================ C ABI
extern "C" {

const char *afh_last_error(void) { return afh2::g_err.c_str(); }

int32_t afh_tree_create(const afh_tree_desc *desc, int32_t device, afh_tree **out) {
  if (!desc || !out || !desc->boxes) return set_error(AFH_ERR_ARG, "afh_tree_create: null");
  const int nc = desc->n_cell;
  if (nc < 2 || nc % 2 || desc->n_boxes < 1 || desc->highest_lvl < 1 ||
      desc->n_var_cell < 1 || desc->n_var_face < 0)
    return set_error(AFH_ERR_ARG, "afh_tree_create: bad sizes");
  // box_capacity (the 3-D in-place regrid) is accepted and not used: a 2-D
  // regrid copies the persisting boxes into the new tree's pools
  if (device >= 0) H2(hipSetDevice(device));
  afh_tree *t = new afh_tree();
  H2(hipGetDevice(&t->device));
  if (const char *env = getenv("AFH2_GC_BOX")) t->gc_box = atoi(env) != 0;
  if (const char *env = getenv("AFH2_GC_TREE_ONE")) t->gc_tree_one = atoi(env) != 0;
  t->nc = nc, t->ng = nc + 2, t->nb = desc->n_boxes, t->nlvl = desc->highest_lvl;
  t->nvc = desc->n_var_cell, t->nvf = desc->n_var_face;
  t->bsz = t->ng * t->ng, t->fsz = 2 * (nc + 1) * (nc + 1);
  t->cgs[0] = desc->coarse_grid_size[0], t->cgs[1] = desc->coarse_grid_size[1];
  t->boxes.assign(desc->boxes, desc->boxes + t->nb);
  t->meth.assign(t->nvc + 1, Meth());
  auto lists = [&](const int32_t *a, const int32_t *off) {
    std::vector<std::vector<int32_t>> r(t->nlvl);
    for (int l = 0; l < t->nlvl; l++) r[l].assign(a + off[l], a + off[l + 1]);
    return r;
  };
  t->h_ids = lists(desc->lvl_ids, desc->lvl_ids_off);
  t->h_leaves = lists(desc->lvl_leaves, desc->lvl_leaves_off);
  t->h_parents = lists(desc->lvl_parents, desc->lvl_parents_off);
  // per level: leaves next to a refinement boundary (af_restrict_ref_boundary),
  // children of the level's parents, consistent-flux tasks; grid spacing
  std::vector<std::vector<int32_t>> refb(t->nlvl), kids(t->nlvl), cfl(t->nlvl);
  t->lvl_dr.assign(2 * t->nlvl, 0.0);
  for (int l = 1; l <= t->nlvl; l++) {
    for (int id : t->h_ids[l - 1]) {
      if (id < 1 || id > t->nb) {
        delete t;
        return set_error(AFH_ERR_ARG, "afh_tree_create: box id %d", id);
      }
      const afh_box_meta &m = t->boxes[id - 1];
      t->lvl_dr[2 * (l - 1)] = m.dr[0], t->lvl_dr[2 * (l - 1) + 1] = m.dr[1];
    }
    for (int id : t->h_ids[l - 1])
      for (int nb = 0; nb < 4; nb++) t->any_refb = t->any_refb || t->boxes[id - 1].neighbors[nb] == 0;
    for (int id : t->h_leaves[l - 1]) {
      const afh_box_meta &m = t->boxes[id - 1];
      bool rb = false;
      for (int nb = 0; nb < 4; nb++) rb = rb || m.neighbors[nb] == 0;
      if (m.parent > 0 && rb) refb[l - 1].push_back(id);
    }
    for (int id : t->h_parents[l - 1]) {
      const afh_box_meta &m = t->boxes[id - 1];
      for (int c = 0; c < 4; c++)
        if (m.children[c] > 0) kids[l - 1].push_back(m.children[c]);
      for (int nb = 1; nb <= 4; nb++) {
        const int nid = m.neighbors[nb - 1];
        if (nid > 0) {
          const afh_box_meta &q = t->boxes[nid - 1];
          bool has = false;
          for (int c = 0; c < 4; c++) has = has || q.children[c] > 0;
          if (!has) cfl[l - 1].push_back((id << 3) | nb);
        }
      }
    }
  }
  int32_t e;
  if ((e = upload_list(t->ids, t->h_ids)) || (e = upload_list(t->leaves, t->h_leaves)) ||
      (e = upload_list(t->parents, t->h_parents)) || (e = upload_list(t->refb, refb)) ||
      (e = upload_list(t->children_of, kids)) || (e = upload_list(t->cflux, cfl)))
    return e;
  H2(hipMalloc(&t->d_boxes, sizeof(afh_box_meta) * t->nb));
  H2(hipMemcpy(t->d_boxes, t->boxes.data(), sizeof(afh_box_meta) * t->nb,
               hipMemcpyHostToDevice));
  H2(hipMalloc(&t->cc, sizeof(double) * (size_t)t->nvc * t->nb * t->bsz));
  H2(hipMemset(t->cc, 0, sizeof(double) * (size_t)t->nvc * t->nb * t->bsz));
  if (t->nvf) {
    H2(hipMalloc(&t->fc, sizeof(double) * (size_t)t->nvf * t->nb * t->fsz));
    H2(hipMemset(t->fc, 0, sizeof(double) * (size_t)t->nvf * t->nb * t->fsz));
  }
  H2(hipMalloc(&t->gc2, sizeof(double) * (size_t)t->nb * 4 * nc));
  H2(hipMalloc(&t->red, sizeof(unsigned long long) * RED_SLOTS * RED_SHARDS));
  H2(hipMalloc(&t->red_out, sizeof(unsigned long long) * RED_SLOTS));
  H2(hipHostMalloc(&t->h_red, sizeof(unsigned long long) * RED_SLOTS));
  H2(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
  *out = t;
  return AFH_OK;
}

int32_t afh_tree_destroy(afh_tree *t) {
  if (!t) return AFH_OK;
  hipStreamSynchronize(t->stream);
  for (LevelList *L : {&t->ids, &t->leaves, &t->parents, &t->refb, &t->children_of, &t->cflux})
    free_list(*L);
  hipFree(t->d_boxes), hipFree(t->cc), hipFree(t->fc), hipFree(t->gc2);
  hipFree(t->red), hipFree(t->red_out), hipHostFree(t->h_red), hipFree(t->d_boxred);
  for (hipEvent_t e : t->ev_pool) hipEventDestroy(e);
  hipStreamDestroy(t->stream);
  delete t;
  return AFH_OK;
}

int32_t afh_tree_sync(afh_tree *t) {
  if (!t) return set_error(AFH_ERR_ARG, "afh_tree_sync: null");
  H2(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

int32_t afh_profile_enable(afh_tree *t, int32_t kclass) {
  if (!t) return set_error(AFH_ERR_ARG, "afh_profile_enable: null");
  if (kclass != 0 && kclass != AFH_PROF_GSRB && kclass != AFH_PROF_FLUX &&
      kclass != AFH_PROF_CS)
    return set_error(AFH_ERR_UNSUPPORTED, "afh_profile_enable: class %d (2-D: GSRB, FLUX, CS)",
                     kclass);
  H2(hipStreamSynchronize(t->stream));
  t->prof_class = kclass;
  t->ev_used = 0;
  t->prof_bytes = 0;
  t->prof_launches = 0;
  return AFH_OK;
}

int32_t afh_profile_read(afh_tree *t, double *total_ms, int64_t *launches, double *bytes) {
  if (!t || !total_ms || !launches || !bytes)
    return set_error(AFH_ERR_ARG, "afh_profile_read: null argument");
  H2(hipStreamSynchronize(t->stream));
  double ms = 0;
  for (size_t q = 0; q + 1 < t->ev_used; q += 2) {
    float e = 0;
    H2(hipEventElapsedTime(&e, t->ev_pool[q], t->ev_pool[q + 1]));
    ms += e;
  }
  *total_ms = ms;
  *launches = t->prof_launches;
  *bytes = t->prof_bytes;
  t->ev_used = 0;
  t->prof_bytes = 0;
  t->prof_launches = 0;
  return AFH_OK;
}

int32_t afh_set_cc_methods(afh_tree *t, int32_t iv, const afh_bc *bc, int32_t rb,
                           int32_t lim) {
  if (int32_t e = check_iv(t, iv, "afh_set_cc_methods")) return e;
  if (!bc) return set_error(AFH_ERR_ARG, "afh_set_cc_methods: null bc");
  if (rb != AFH_RB_GC_INTERP && rb != AFH_RB_GC_INTERP_LIM && rb != AFH_RB_MG_SIDES)
    return set_error(AFH_ERR_ARG, "afh_set_cc_methods: rb %d", rb);
  for (int q = 0; q < 4; q++) {
    const int ty = bc[q].type;
    if (ty != AFH_BC_DIRICHLET && ty != AFH_BC_NEUMANN && ty != AFH_BC_CONTINUOUS &&
        ty != AFH_BC_DIRICHLET_COPY)
      return set_error(AFH_ERR_ARG, "afh_set_cc_methods: bc type %d", ty);
  }
  Meth &m = t->meth[iv];
  m.set = 1;
  for (int q = 0; q < 4; q++) m.bc[q] = bc[q];
  m.rb = rb;
  m.lim = lim;
  t->meth_gen++;
  return AFH_OK;
}

int32_t afh_set_bc(afh_tree *t, int32_t iv, int32_t nb, int32_t type, double value) {
  if (int32_t e = check_iv(t, iv, "afh_set_bc")) return e;
  if (nb < 1 || nb > 4) return set_error(AFH_ERR_ARG, "afh_set_bc: 2-D face %d", nb);
  if (type != AFH_BC_DIRICHLET && type != AFH_BC_NEUMANN && type != AFH_BC_CONTINUOUS &&
      type != AFH_BC_DIRICHLET_COPY)
    return set_error(AFH_ERR_ARG, "afh_set_bc: type %d", type);
  t->meth[iv].bc[nb - 1].type = type;
  t->meth[iv].bc[nb - 1].value = value;
  t->meth_gen++;
  return AFH_OK;
}

int32_t afh_cc_put(afh_tree *t, int32_t iv, const double *host) {
  if (int32_t e = check_iv(t, iv, "afh_cc_put")) return e;
  H2(hipMemcpyAsync(t->ccv(iv), host, sizeof(double) * (size_t)t->nb * t->bsz,
                    hipMemcpyHostToDevice, t->stream));
  H2(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

int32_t afh_cc_get(afh_tree *t, int32_t iv, double *host) {
  if (int32_t e = check_iv(t, iv, "afh_cc_get")) return e;
  H2(hipMemcpyAsync(host, t->ccv(iv), sizeof(double) * (size_t)t->nb * t->bsz,
                    hipMemcpyDeviceToHost, t->stream));
  H2(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

int32_t afh_fc_put(afh_tree *t, int32_t ivf, const double *host) {
  if (!t || ivf < 1 || ivf > t->nvf) return set_error(AFH_ERR_ARG, "afh_fc_put: bad variable");
  H2(hipMemcpyAsync(t->fcv(ivf), host, sizeof(double) * (size_t)t->nb * t->fsz,
                    hipMemcpyHostToDevice, t->stream));
  H2(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

int32_t afh_fc_get(afh_tree *t, int32_t ivf, double *host) {
  if (!t || ivf < 1 || ivf > t->nvf) return set_error(AFH_ERR_ARG, "afh_fc_get: bad variable");
  H2(hipMemcpyAsync(host, t->fcv(ivf), sizeof(double) * (size_t)t->nb * t->fsz,
                    hipMemcpyDeviceToHost, t->stream));
  H2(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

int32_t afh_gc_lvl(afh_tree *t, int32_t lvl, int32_t iv, int32_t corners) {
  if (int32_t e = check_iv(t, iv, "afh_gc_lvl")) return e;
  if (lvl < 1 || lvl > t->nlvl) return set_error(AFH_ERR_ARG, "afh_gc_lvl: level %d", lvl);
  if (!t->meth[iv].set) return set_error(AFH_ERR_STATE, "afh_gc_lvl: no methods for %d", iv);
  return gc_lvl(t, lvl, iv, corners != 0);
}

int32_t afh_gc_tree(afh_tree *t, int32_t iv, int32_t corners) {
  if (int32_t e = check_iv(t, iv, "afh_gc_tree")) return e;
  if (!t->meth[iv].set) return set_error(AFH_ERR_STATE, "afh_gc_tree: no methods for %d", iv);
  if (t->gc_tree_one && !t->any_refb && corners && t->gc_box) return gc_lvl(t, 0, iv, true);
  for (int l = 1; l <= t->nlvl; l++)
    if (int32_t e = gc_lvl(t, l, iv, corners != 0)) return e;
  return AFH_OK;
}

int32_t afh_restrict_tree(afh_tree *t, int32_t iv) {
  if (int32_t e = check_iv(t, iv, "afh_restrict_tree")) return e;
  // af_restrict_tree: levels highest-1 .. 1, the children of each parent
  for (int l = t->nlvl - 1; l >= 1; l--) {
    const int n = t->children_of.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k2_restrict, grid2(t->nc * t->nc / 4, n), blk2(t->nc * t->nc / 4), 0, t->stream,
                       t->ccv(iv), t->d_boxes, t->children_of.at(l), t->nc, t->bsz);
    H2_LAUNCH("k2_restrict");
  }
  return AFH_OK;
}

int32_t afh_tree_copy_cc(afh_tree *t, int32_t iv_from, int32_t iv_to) {
  if (int32_t e = check_iv(t, iv_from, "afh_tree_copy_cc")) return e;
  if (int32_t e = check_iv(t, iv_to, "afh_tree_copy_cc")) return e;
  H2(hipMemcpyAsync(t->ccv(iv_to), t->ccv(iv_from), sizeof(double) * (size_t)t->nb * t->bsz,
                    hipMemcpyDeviceToDevice, t->stream));
  return AFH_OK;
}

int32_t afh_tree_maxabs_cc(afh_tree *t, int32_t iv, double *out) {
  if (int32_t e = check_iv(t, iv, "afh_tree_maxabs_cc")) return e;
  if (!out) return set_error(AFH_ERR_ARG, "afh_tree_maxabs_cc: null out");
  if (int32_t e = red_init(t, 3, 0.0)) return e;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k2_maxabs, grid2(t->nc * t->nc, n), blk2(t->nc * t->nc), 0, t->stream, t->ccv(iv),
                       t->leaves.at(l), t->nc, t->bsz, t->red + 3 * RED_SHARDS);
    H2_LAUNCH("k2_maxabs");
  }
  return red_read(t, 3, 1, 1, out);
}

// ------------------------------------------------------------ multigrid
int32_t afh_mg_create(afh_tree *t, const afh_mg_desc *d, afh_mg **out) {
  if (!t || !d || !out) return set_error(AFH_ERR_ARG, "afh_mg_create: null");
  if (d->i_phi < 1 || d->i_phi > t->nvc || d->i_rhs < 1 || d->i_rhs > t->nvc ||
      d->i_tmp < 1 || d->i_tmp > t->nvc)
    return set_error(AFH_ERR_ARG, "afh_mg_create: bad variable index");
  if (!t->meth[d->i_phi].set) return set_error(AFH_ERR_STATE, "set cc methods for phi first");
  if (d->coarse_mode != AFH_COARSE_DIRECT &&
      !(d->coarse_mode == AFH_COARSE_PFMG && d->coarse_cycles >= 1 && d->coarse_tol >= 0))
    return set_error(AFH_ERR_UNSUPPORTED, "2-D: AFH_COARSE_DIRECT or AFH_COARSE_PFMG");
  if (d->n_cycle_down < 1 || d->n_cycle_up < 1)
    return set_error(AFH_ERR_ARG, "afh_mg_create: cycles");
  const int nx = t->cgs[0], ny = t->cgs[1];
  if (nx * ny > CS2_CELLS || t->ids.n(1) * t->nc * t->nc != nx * ny)
    return set_error(AFH_ERR_UNSUPPORTED, "2-D: level-1 grid %d x %d", nx, ny);
  afh_mg *mg = new afh_mg();
  mg->t = t;
  mg->d = *d;
  mg->nx = nx, mg->ny = ny;
  // mg_box_lpl_stencil: c(2:5) = 1/dr^2, c(1) = -sum(c(2:)) - lambda
  mg->lvl_c.resize(t->nlvl);
  for (int l = 1; l <= t->nlvl; l++) {
    const double *dr = &t->lvl_dr[2 * (l - 1)];
    Coef2 &c = mg->lvl_c[l - 1];
    for (int q = 0; q < 2; q++) {
      const double inv = 1 / (dr[q] * dr[q]);
      c.c[1 + 2 * q] = inv;
      c.c[2 + 2 * q] = inv;
    }
    double s = c.c[1];
    for (int q = 2; q < 5; q++) s = s + c.c[q];
    c.c[0] = -s - d->helmholtz_lambda;
    c.inv_c1 = 1 / c.c[0];
  }
  H2(hipMalloc(&mg->d_lvl_c, sizeof(Coef2) * t->nlvl));
  H2(hipMemcpy(mg->d_lvl_c, mg->lvl_c.data(), sizeof(Coef2) * t->nlvl, hipMemcpyHostToDevice));
  if (const char *env = getenv("AFH2_ALL_LVL")) mg->all_lvl = atoi(env) != 0;
  if (const char *env = getenv("AFH2_GRAPHS")) mg->use_graphs = atoi(env) != 0;
  if (const char *env = getenv("AFH2_CORNER_FOLD")) mg->corner_fold = atoi(env) != 0;
  H2(hipMalloc(&mg->d_q[0], sizeof(double) * nx * nx));
  H2(hipMalloc(&mg->d_q[1], sizeof(double) * ny * ny));
  H2(hipMalloc(&mg->d_e[0], sizeof(double) * nx));
  H2(hipMalloc(&mg->d_e[1], sizeof(double) * ny));
  if (const char *env = getenv("AFH_PAIR2D")) mg->pair = atoi(env) != 0;
  mg->pair = mg->pair && (t->nc == 4 || t->nc == 8 || t->nc == 16) &&
             d->n_cycle_down % 2 == 0 && d->n_cycle_up % 2 == 0;
  if (mg->pair) H2(hipMalloc(&mg->alt, sizeof(double) * (size_t)t->nb * t->bsz));
  *out = mg;
  return AFH_OK;
}

int32_t afh_mg_destroy(afh_mg *mg) {
  if (!mg) return AFH_OK;
  hipStreamSynchronize(mg->t->stream);
  for (int q = 0; q < 2; q++) hipFree(mg->d_q[q]), hipFree(mg->d_e[q]);
  hipFree(mg->alt);
  hipFree(mg->d_lvl_c);
  hipFree(mg->d_pf_lvl), hipFree(mg->d_pf_A), hipFree(mg->d_pf_P), hipFree(mg->d_pf_b2r);
  hipFree(mg->d_pf_fmask), hipFree(mg->d_pf_iters);
  for (auto &g : mg->graphs)
    if (g.second.exec) hipGraphExecDestroy(g.second.exec);
  delete mg;
  return AFH_OK;
}

}  // extern "C"

namespace afh2 {

// the folded 1-D operator h tridiag(1, -2, 1) with end diagonals -h
// (Neumann) / -3h (Dirichlet): cosine / sine eigenbasis (same as the 3-D
// AFH_COARSE_DIRECT tables)
static void cs_tables(int n, int bc_lo, int bc_hi, double h, double *q, double *e) {
  const int dlo = bc_lo == AFH_BC_DIRICHLET, dhi = bc_hi == AFH_BC_DIRICHLET;
  const double pi = 3.14159265358979323846;
  for (int p = 0; p < n; p++) {
    double th;
    if (dlo == dhi) th = pi * (p + dlo) / n;
    else th = pi * (p + 0.5) / n;
    double nrm2 = 0.0;
    for (int i = 0; i < n; i++) {
      const double v = dlo ? sin(th * (i + 0.5)) : cos(th * (i + 0.5));
      q[i * n + p] = v;
      nrm2 = nrm2 + v * v;
    }
    const double inv = 1 / sqrt(nrm2);
    for (int i = 0; i < n; i++) q[i * n + p] = q[i * n + p] * inv;
    e[p] = h * (2 * cos(th) - 2);
  }
}

// AFH_COARSE_PFMG: the folded level-1 operator (stencil_handle_boundaries,
// the 3-D library's pf_prepare with NDIM = 2), the hierarchy when the
// boundary types change, then k2_cs_pfmg
static int32_t solve_coarse_pfmg(afh_mg *mg) {
  afh_tree *t = mg->t;
  const Meth &M = t->meth[mg->d.i_phi];
  const int nc = t->nc, nid = t->ids.n(1), nx = mg->nx, ny = mg->ny;
  const size_t n0 = (size_t)nx * ny;
  bool fresh = !mg->d_pf_lvl;
  for (int q = 0; q < 4; q++) fresh = fresh || mg->pf_bc[q] != M.bc[q].type;
  if (fresh) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    H2(hipStreamIsCapturing(t->stream, &cs));
    if (cs != hipStreamCaptureStatusNone)
      return set_error(AFH_ERR_STATE, "pfmg: setup changed during a graph capture");
    std::vector<double> a7(7 * n0, 0.0), b2r(4 * n0, 0.0);
    std::vector<uint8_t> fm(n0, 0);
    const int dims[2] = {nx, ny};
    for (int q = 0; q < nid; q++) {
      const int id = t->h_ids[0][q];
      const afh_box_meta &m = t->boxes[id - 1];
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          const int gi[2] = {(m.ix[0] - 1) * nc + i, (m.ix[1] - 1) * nc + j};
          const size_t g = (size_t)(gi[1] - 1) * nx + (gi[0] - 1);
          double c[7] = {mg->lvl_c[0].c[0], mg->lvl_c[0].c[1], mg->lvl_c[0].c[2],
                         mg->lvl_c[0].c[3], mg->lvl_c[0].c[4], 0.0, 0.0};
          for (int nb = 1; nb <= 4; nb++) {
            const int dd = (nb - 1) >> 1;
            const bool low = ((nb - 1) & 1) == 0;
            if (!(low ? gi[dd] == 1 : gi[dd] == dims[dd])) continue;
            double k2;
            if (M.bc[nb - 1].type == AFH_BC_DIRICHLET) {
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
    afh_pfmg h;
    if (afh_pfmg_setup(&h, nx, ny, 1, 2, a7.data()))
      return set_error(AFH_ERR_DEVICE, "pfmg: host setup allocation");
    std::vector<afh_pf::PfLvl> lv;
    std::vector<double> A, P;
    afh_pf::pf_device_tables(h, lv, A, P);
    const size_t np = h.off[h.nl];
    afh_pfmg_free(&h);
    H2(hipStreamSynchronize(t->stream));
    hipFree(mg->d_pf_lvl), hipFree(mg->d_pf_A), hipFree(mg->d_pf_P);
    H2(hipMalloc(&mg->d_pf_lvl, sizeof(afh_pf::PfLvl) * lv.size()));
    H2(hipMalloc(&mg->d_pf_A, sizeof(double) * A.size()));
    H2(hipMalloc(&mg->d_pf_P, sizeof(double) * P.size()));
    if (!mg->d_pf_b2r) {
      H2(hipMalloc(&mg->d_pf_b2r, sizeof(double) * 4 * n0));
      H2(hipMalloc(&mg->d_pf_fmask, n0));
      H2(hipMalloc(&mg->d_pf_iters, sizeof(int)));
    }
    H2(hipMemcpy(mg->d_pf_lvl, lv.data(), sizeof(afh_pf::PfLvl) * lv.size(),
                 hipMemcpyHostToDevice));
    H2(hipMemcpy(mg->d_pf_A, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
    H2(hipMemcpy(mg->d_pf_P, P.data(), sizeof(double) * P.size(), hipMemcpyHostToDevice));
    H2(hipMemcpy(mg->d_pf_b2r, b2r.data(), sizeof(double) * b2r.size(), hipMemcpyHostToDevice));
    H2(hipMemcpy(mg->d_pf_fmask, fm.data(), n0, hipMemcpyHostToDevice));
    (void)np;
    mg->pf_nl = (int)lv.size();
    mg->pf_wave = afh_pf::pf_wave_from(lv);
    const size_t lds = afh_pf::pf_lds_bytes(lv, true);
    if (lds + 64 > 160 * 1024)
      return set_error(AFH_ERR_UNSUPPORTED, "2-D pfmg: level-1 grid %d x %d", nx, ny);
    mg->pf_lds = (int)lds;
    {
      // the attribute is per kernel, not per multigrid: only ever raised
      static std::mutex m;
      static std::map<int, int> top;
      int dev = 0;
      H2(hipGetDevice(&dev));
      std::lock_guard<std::mutex> g(m);
      if (mg->pf_lds > top[dev]) {
        H2(hipFuncSetAttribute((const void *)k2_cs_pfmg,
                               hipFuncAttributeMaxDynamicSharedMemorySize, mg->pf_lds));
        top[dev] = mg->pf_lds;
      }
    }
    for (int q = 0; q < 4; q++) mg->pf_bc[q] = M.bc[q].type;
  }
  const int nt = std::min(1024, std::max(256, (int)((n0 + 63) / 64 * 64)));
  prof_mark(t, AFH_PROF_CS);
  hipLaunchKernelGGL(k2_cs_pfmg, dim3(1), dim3(nt), mg->pf_lds, t->stream, mg->d_pf_lvl,
                     mg->pf_nl, mg->pf_wave, mg->d_pf_A, mg->d_pf_P, mg->d_pf_b2r, mg->d_pf_fmask,
                     t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->d_boxes, t->ids.at(1), nid,
                     t->nc, t->bsz, t->bc4(mg->d.i_phi), mg->d.coarse_tol, mg->d.coarse_cycles,
                     mg->d_pf_iters);
  H2_LAUNCH("k2_cs_pfmg");
  prof_end(t, AFH_PROF_CS, 0.0);
  return gc_lvl(t, 1, mg->d.i_phi, true);
}

static int32_t solve_coarse(afh_mg *mg) {
  afh_tree *t = mg->t;
  const Meth &M = t->meth[mg->d.i_phi];
  for (int q = 0; q < 4; q++) {
    if (M.bc[q].type != AFH_BC_DIRICHLET && M.bc[q].type != AFH_BC_NEUMANN)
      return set_error(AFH_ERR_UNSUPPORTED, "2-D coarse solve: bc type %d", M.bc[q].type);
  }
  if (mg->d.coarse_mode == AFH_COARSE_PFMG) return solve_coarse_pfmg(mg);
  bool fresh = false;
  for (int q = 0; q < 4; q++) fresh = fresh || mg->q_bc[q] != M.bc[q].type;
  const double hx = mg->lvl_c[0].c[1], hy = mg->lvl_c[0].c[3];
  if (fresh) {
    H2(hipStreamSynchronize(t->stream));
    const int n[2] = {mg->nx, mg->ny};
    const double h[2] = {hx, hy};
    for (int d = 0; d < 2; d++) {
      std::vector<double> q((size_t)n[d] * n[d]), e(n[d]);
      cs_tables(n[d], M.bc[2 * d].type, M.bc[2 * d + 1].type, h[d], q.data(), e.data());
      H2(hipMemcpy(mg->d_q[d], q.data(), sizeof(double) * q.size(), hipMemcpyHostToDevice));
      H2(hipMemcpy(mg->d_e[d], e.data(), sizeof(double) * e.size(), hipMemcpyHostToDevice));
    }
    for (int q = 0; q < 4; q++) mg->q_bc[q] = M.bc[q].type;
  }
  hipLaunchKernelGGL(k2_cs_direct, dim3(1), dim3(1024), 0, t->stream, t->ccv(mg->d.i_phi),
                     t->ccv(mg->d.i_rhs), t->d_boxes, t->ids.at(1), t->ids.n(1), t->nc, t->bsz,
                     mg->nx, mg->ny, hx, hy, t->bc4(mg->d.i_phi), mg->d_q[0], mg->d_q[1],
                     mg->d_e[0], mg->d_e[1], mg->d.helmholtz_lambda);
  H2_LAUNCH("k2_cs_direct");
  return gc_lvl(t, 1, mg->d.i_phi, true);
}

// gsrb_boxes (m_af_multigrid.f90:648-687): 2 n_cycle half sweeps, each
// followed by the level fill (corners after the last sweep of the up leg)
// skip_corners: the up leg's corner pass is left to correct_children of the
// next level (every box of lvl a parent; k2_block_corners)
static int32_t gsrb_boxes(afh_mg *mg, int lvl, bool up, bool skip_corners = false) {
  afh_tree *t = mg->t;
  const int n = t->ids.n(lvl);
  const int nc_ = up ? mg->d.n_cycle_up : mg->d.n_cycle_down;
  if (mg->pair && n) {
    // n_cycle fused pairs, phi -> alt -> phi (n_cycle even); the corners of
    // the up leg's last fill after them
    double *phi = t->ccv(mg->d.i_phi);
    for (int p = 0; p < nc_; p++) {
      const double *src = (p & 1) ? mg->alt : phi;
      double *dst = (p & 1) ? phi : mg->alt;
      const Coef2 cf = mg->lvl_c[lvl - 1];
      const Bc4 g = t->bc4(mg->d.i_phi);
      // timed on levels of >= 256 boxes, as the split half-sweeps
      const int pc = n >= 256 ? AFH_PROF_GSRB : -1;
      prof_mark(t, pc);
      const double *rh = t->ccv(mg->d.i_rhs);
      const int32_t *ids = t->ids.at(lvl);
      // several boxes per wave: four 4^2, two 8^2
      if (t->nc == 4)
        hipLaunchKernelGGL((k2_pair_box<4, 16>), dim3((n + 3) / 4), dim3(64), 0, t->stream, src,
                           dst, rh, phi, t->d_boxes, ids, n, t->bsz, cf, g);
      else if (t->nc == 8)
        hipLaunchKernelGGL((k2_pair_box<8, 32>), dim3((n + 1) / 2), dim3(64), 0, t->stream, src,
                           dst, rh, phi, t->d_boxes, ids, n, t->bsz, cf, g);
      else
        hipLaunchKernelGGL(k2_pair_box<16>, dim3(n), dim3(64), 0, t->stream, src, dst, rh, phi,
                           t->d_boxes, ids, n, t->bsz, cf, g);
      H2_LAUNCH("k2_pair_box");
      // a red+black pair reads phi and rhs and writes phi once = 24 B/cell
      prof_end(t, pc, 24.0 * t->nc * t->nc * n);
    }
    if (up && !skip_corners) {
      hipLaunchKernelGGL(k2_corners, dim3((4 * n + NT - 1) / NT), dim3(NT), 0, t->stream,
                         phi, t->d_boxes, t->ids.at(lvl), n, t->nc, t->bsz);
      H2_LAUNCH("k2_corners");
    }
    return AFH_OK;
  }
  for (int s = 1; s <= 2 * nc_; s++) {
    if (n) {
      // timed on levels of >= 256 boxes, as libafivo_hip's pair: the small
      // levels' launches are launch-bound, another regime
      const int pc = n >= 256 ? AFH_PROF_GSRB : -1;
      prof_mark(t, pc);
      hipLaunchKernelGGL(k2_gsrb, grid2(t->nc * t->nc / 2, n), blk2(t->nc * t->nc / 2), 0, t->stream,
                         t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->ids.at(lvl), t->nc,
                         t->bsz, mg->lvl_c[lvl - 1], s);
      H2_LAUNCH("k2_gsrb");
      prof_end(t, pc, 16.0 * t->nc * t->nc * n);
    }
    if (int32_t e = gc_lvl(t, lvl, mg->d.i_phi, up && s == 2 * nc_)) return e;
  }
  return AFH_OK;
}

// update_coarse (691-738)
static int32_t update_coarse(afh_mg *mg, int lvl) {
  afh_tree *t = mg->t;
  const int n = t->ids.n(lvl);
  if (n) {
    hipLaunchKernelGGL(k2_rstr_fas, grid2(t->nc * t->nc / 4, n), blk2(t->nc * t->nc / 4), 0, t->stream,
                       t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp),
                       t->d_boxes, t->ids.at(lvl), t->nc, t->bsz, mg->lvl_c[lvl - 1]);
    H2_LAUNCH("k2_rstr_fas");
  }
  if (int32_t e = gc_lvl(t, lvl - 1, mg->d.i_phi, true)) return e;
  const int np = t->parents.n(lvl - 1);
  if (np) {
    hipLaunchKernelGGL(k2_parent_rhs, grid2(t->bsz, np), blk2(t->bsz), 0, t->stream,
                       t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp),
                       t->parents.at(lvl - 1), t->nc, t->bsz, mg->lvl_c[lvl - 2], 1);
    H2_LAUNCH("k2_parent_rhs");
  }
  return AFH_OK;
}

// correct_children of the parents of level lvl-1 (624-646)
static int32_t correct_children(afh_mg *mg, int lvl, bool corners = false) {
  afh_tree *t = mg->t;
  const int np = t->parents.n(lvl - 1);
  if (!np) return AFH_OK;
  double *phi = t->ccv(mg->d.i_phi), *tmp = t->ccv(mg->d.i_tmp);
  if (corners) {
    hipLaunchKernelGGL(k2_block_corners, grid2(t->bsz, np), blk2(t->bsz), 0, t->stream, tmp,
                       phi, t->d_boxes, t->parents.at(lvl - 1), t->nc, t->bsz);
    H2_LAUNCH("k2_block_corners");
  } else {
    hipLaunchKernelGGL(k2_block, grid2(t->bsz, np), blk2(t->bsz), 0, t->stream, tmp, phi, tmp,
                       t->parents.at(lvl - 1), t->bsz, 0);
    H2_LAUNCH("k2_block");
  }
  const int nk = t->children_of.n(lvl - 1);
  hipLaunchKernelGGL(k2_prolong, grid2(t->nc * t->nc, nk), blk2(t->nc * t->nc), 0, t->stream, phi, tmp,
                     t->d_boxes, t->children_of.at(lvl - 1), t->nc, t->bsz);
  H2_LAUNCH("k2_prolong");
  return AFH_OK;
}

static int32_t residual_lvl(afh_mg *mg, int lvl, const LevelList &L, bool fold) {
  afh_tree *t = mg->t;
  const int n = L.n(lvl);
  if (!n) return AFH_OK;
  hipLaunchKernelGGL(k2_residual, grid2(t->nc * t->nc, n), blk2(t->nc * t->nc), 0, t->stream,
                     t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), L.at(lvl),
                     t->nc, t->bsz, mg->lvl_c[lvl - 1],
                     fold ? t->red + 3 * RED_SHARDS : nullptr, nullptr, nullptr);
  H2_LAUNCH("k2_residual");
  return AFH_OK;
}

// the residual of levels 1 .. max_lvl of list L in one launch (each box's
// coefficients by its level; false: max_lvl boxes exceed the grid's y limit)
static bool residual_all(afh_mg *mg, int max_lvl, const LevelList &L, bool fold) {
  afh_tree *t = mg->t;
  const int n = L.off[max_lvl] - L.off[0];
  if (!mg->all_lvl || n > 65535) return false;
  if (n)
    hipLaunchKernelGGL(k2_residual, grid2(t->nc * t->nc, n), blk2(t->nc * t->nc), 0, t->stream,
                       t->ccv(mg->d.i_phi), t->ccv(mg->d.i_rhs), t->ccv(mg->d.i_tmp), L.at(1),
                       t->nc, t->bsz, mg->lvl_c[0], fold ? t->red + 3 * RED_SHARDS : nullptr,
                       mg->d_lvl_c, t->d_boxes);
  return true;
}

// mg_fas_vcycle (185-264); with max_out the leaf max|tmp| is folded into
// slot 3 by the residual pass
static int32_t vcycle(afh_mg *mg, bool set_residual, int max_lvl, bool max_out) {
  int32_t e;
  for (int l = max_lvl; l >= 2; l--) {
    if ((e = gsrb_boxes(mg, l, false)) || (e = update_coarse(mg, l))) return e;
  }
  if ((e = solve_coarse(mg))) return e;
  afh_tree *tt = mg->t;
  bool pend = false;  // level l-1's corners left to correct_children(l)
  for (int l = 2; l <= max_lvl; l++) {
    const bool defer = mg->corner_fold && mg->pair && l < max_lvl && tt->ids.n(l) > 0 &&
                       tt->parents.n(l) == tt->ids.n(l);
    if ((e = correct_children(mg, l, pend)) || (e = gc_lvl(tt, l, mg->d.i_phi, true)) ||
        (e = gsrb_boxes(mg, l, true, defer)))
      return e;
    pend = defer;
  }
  if (!set_residual) return AFH_OK;
  afh_tree *t = mg->t;
  if (max_out && (e = red_init(t, 3, 0.0))) return e;
  if (max_out ? residual_all(mg, max_lvl, t->leaves, true) &&
                    residual_all(mg, max_lvl, t->parents, false)
              : residual_all(mg, max_lvl, t->ids, false))
    return AFH_OK;
  for (int l = 1; l <= max_lvl; l++) {
    if (max_out) {
      // leaves fold, parents do not (the same tmp values)
      if ((e = residual_lvl(mg, l, t->leaves, true)) ||
          (e = residual_lvl(mg, l, t->parents, false)))
        return e;
    } else if ((e = residual_lvl(mg, l, t->ids, false))) {
      return e;
    }
  }
  return AFH_OK;
}

// vcycle, replayed from a captured graph once a variant has run eagerly
// (not while kernels are being timed: the events are host calls)
static int32_t vcycle_run(afh_mg *mg, bool set_residual, int max_lvl, bool max_out) {
  afh_tree *t = mg->t;
  if (!mg->use_graphs || t->prof_class) return vcycle(mg, set_residual, max_lvl, max_out);
  const int key = (max_lvl << 2) | (set_residual ? 2 : 0) | (max_out ? 1 : 0);
  afh_mg::Graph &g = mg->graphs[key];
  if (g.gen != t->meth_gen) {
    if (g.exec) hipGraphExecDestroy(g.exec);
    g = afh_mg::Graph();
    g.gen = t->meth_gen;
  }
  if (!g.warm) {
    g.warm = true;
    return vcycle(mg, set_residual, max_lvl, max_out);
  }
  if (!g.exec) {
    hipGraph_t graph;
    H2(hipStreamBeginCapture(t->stream, hipStreamCaptureModeThreadLocal));
    const int32_t e = vcycle(mg, set_residual, max_lvl, max_out);
    const hipError_t ce = hipStreamEndCapture(t->stream, &graph);
    if (e) {
      if (ce == hipSuccess) hipGraphDestroy(graph);
      return e;
    }
    H2(ce);
    const hipError_t ie = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    hipGraphDestroy(graph);
    H2(ie);
  }
  H2(hipGraphLaunch(g.exec, t->stream));
  return AFH_OK;
}

}  // namespace afh2

extern "C" {

int32_t afh_mg_fas_vcycle(afh_mg *mg, int32_t set_residual, int32_t hl) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  const int max_lvl = (hl > 0 && hl <= mg->t->nlvl) ? hl : mg->t->nlvl;
  return vcycle_run(mg, set_residual != 0, max_lvl, false);
}

int32_t afh_mg_fas_vcycle_fold(afh_mg *mg, int32_t hl) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  const int max_lvl = (hl > 0 && hl <= mg->t->nlvl) ? hl : mg->t->nlvl;
  return vcycle_run(mg, true, max_lvl, true);
}

int32_t afh_mg_fas_vcycle_maxres(afh_mg *mg, int32_t hl, double *max_res) {
  if (!mg || !max_res) return set_error(AFH_ERR_ARG, "afh_mg_fas_vcycle_maxres: null");
  const int max_lvl = (hl > 0 && hl <= mg->t->nlvl) ? hl : mg->t->nlvl;
  if (int32_t e = vcycle_run(mg, true, max_lvl, true)) return e;
  return red_read(mg->t, 3, 1, 1, max_res);
}

// mg_fas_fmg (m_af_multigrid.f90:137-180)
int32_t afh_mg_fas_fmg(afh_mg *mg, int32_t set_residual, int32_t have_guess) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  afh_tree *t = mg->t;
  double *phi = t->ccv(mg->d.i_phi), *rhs = t->ccv(mg->d.i_rhs), *tmp = t->ccv(mg->d.i_tmp);
  const int nc = t->nc;
  int32_t e;
  if (have_guess) {
    for (int l = t->nlvl; l >= 2; l--) {
      // set_coarse_phi_rhs (742-776)
      if (l == t->nlvl && (e = gc_lvl(t, l, mg->d.i_phi, true))) return e;
      if ((e = residual_lvl(mg, l, t->ids, false))) return e;
      const int n = t->ids.n(l);
      if (n) {
        hipLaunchKernelGGL(k2_restrict, grid2(nc * nc / 4, n), blk2(nc * nc / 4), 0, t->stream, tmp,
                           t->d_boxes, t->ids.at(l), nc, t->bsz);
        hipLaunchKernelGGL(k2_restrict, grid2(nc * nc / 4, n), blk2(nc * nc / 4), 0, t->stream, phi,
                           t->d_boxes, t->ids.at(l), nc, t->bsz);
        H2_LAUNCH("k2_restrict");
      }
      if ((e = gc_lvl(t, l - 1, mg->d.i_phi, true))) return e;
      const int np = t->parents.n(l - 1);
      if (np) {
        hipLaunchKernelGGL(k2_parent_rhs, grid2(t->bsz, np), blk2(t->bsz), 0, t->stream, phi, rhs,
                           tmp, t->parents.at(l - 1), nc, t->bsz, mg->lvl_c[l - 2], 0);
        H2_LAUNCH("k2_parent_rhs");
      }
    }
  } else {
    // init_phi_rhs (779-799)
    for (int l = t->nlvl; l >= 2; l--) {
      const int n = t->ids.n(l);
      if (!n) continue;
      hipLaunchKernelGGL(k2_block, grid2(t->bsz, n), blk2(t->bsz), 0, t->stream, phi,
                         (const double *)nullptr, (const double *)nullptr, t->ids.at(l),
                         t->bsz, 2);
      hipLaunchKernelGGL(k2_restrict, grid2(nc * nc / 4, n), blk2(nc * nc / 4), 0, t->stream, rhs,
                         t->d_boxes, t->ids.at(l), nc, t->bsz);
      H2_LAUNCH("k2_restrict");
    }
  }
  const int n1 = t->ids.n(1);
  hipLaunchKernelGGL(k2_block, grid2(t->bsz, n1), blk2(t->bsz), 0, t->stream, tmp, phi,
                     (const double *)nullptr, t->ids.at(1), t->bsz, 1);
  H2_LAUNCH("k2_block");
  if ((e = vcycle(mg, set_residual && t->nlvl == 1, 1, false))) return e;
  for (int l = 2; l <= t->nlvl; l++) {
    const int n = t->ids.n(l);
    if (n) {
      hipLaunchKernelGGL(k2_block, grid2(t->bsz, n), blk2(t->bsz), 0, t->stream, tmp, phi,
                         (const double *)nullptr, t->ids.at(l), t->bsz, 1);
      H2_LAUNCH("k2_block");
    }
    if ((e = correct_children(mg, l)) || (e = gc_lvl(t, l, mg->d.i_phi, true)) ||
        (e = vcycle(mg, set_residual && l == t->nlvl, l, false)))
      return e;
  }
  return AFH_OK;
}

int32_t afh_mg_compute_phi_gradient(afh_mg *mg, int32_t i_fc, double fac, int32_t i_norm) {
  if (!mg) return set_error(AFH_ERR_ARG, "null mg");
  afh_tree *t = mg->t;
  if (i_fc < 1 || i_fc > t->nvf || i_norm < 0 || i_norm > t->nvc)
    return set_error(AFH_ERR_ARG, "bad variable index");
  // every level in one launch (the box's spacing comes from its meta)
  const int n_all = t->ids.off[t->nlvl] - t->ids.off[0];
  if (mg->all_lvl && n_all <= 65535) {
    if (n_all) {
      hipLaunchKernelGGL(k2_gradient, grid2((t->nc + 1) * (t->nc + 1), n_all), blk2((t->nc + 1) * (t->nc + 1)), 0,
                         t->stream, t->ccv(mg->d.i_phi), t->fcv(i_fc),
                         i_norm ? t->ccv(i_norm) : nullptr, t->d_boxes, t->ids.at(1), t->nc,
                         t->bsz, t->fsz, fac);
      H2_LAUNCH("k2_gradient");
    }
    return AFH_OK;
  }
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->ids.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k2_gradient, grid2((t->nc + 1) * (t->nc + 1), n), blk2((t->nc + 1) * (t->nc + 1)), 0,
                       t->stream, t->ccv(mg->d.i_phi), t->fcv(i_fc),
                       i_norm ? t->ccv(i_norm) : nullptr, t->d_boxes, t->ids.at(l), t->nc,
                       t->bsz, t->fsz, fac);
    H2_LAUNCH("k2_gradient");
  }
  return AFH_OK;
}

// ------------------------------------------------------------ fluid
int32_t afh_fluid_create(afh_tree *t, const afh_fluid_desc *d, afh_fluid **out) {
  if (!t || !d || !out) return set_error(AFH_ERR_ARG, "afh_fluid_create: null");
  if (d->n_species < 1 || d->n_species > AFH_MAX_SPECIES)
    return set_error(AFH_ERR_ARG, "afh_fluid_create: n_species");
  if (d->i_gas_dens || d->i_photo || d->n_ions)
    return set_error(AFH_ERR_UNSUPPORTED,
                     "2-D: variable gas density / photoionization / mobile ions");
  for (int r = 0; r < d->n_reactions; r++) {
    const int ty = d->reactions[r].rate_type;
    if (ty != AFH_RATE_TABULATED_FIELD && ty != AFH_RATE_CONSTANT && ty != AFH_RATE_LINEAR &&
        ty != AFH_RATE_EXP_V1 && ty != AFH_RATE_EXP_V2)
      return set_error(AFH_ERR_UNSUPPORTED, "2-D: rate type %d", ty);
  }
  afh_fluid *f = new afh_fluid();
  f->t = t;
  f->d = *d;
  f->d.reactions = nullptr;
  const size_t ntd = (size_t)d->td.n_points * d->td.n_cols;
  const size_t nch = (size_t)d->chem.n_points * d->chem.n_cols;
  H2(hipMalloc(&f->d_td, sizeof(double) * ntd));
  H2(hipMemcpy(f->d_td, d->td.rows_cols, sizeof(double) * ntd, hipMemcpyHostToDevice));
  if (nch) {
    H2(hipMalloc(&f->d_chem, sizeof(double) * nch));
    H2(hipMemcpy(f->d_chem, d->chem.rows_cols, sizeof(double) * nch, hipMemcpyHostToDevice));
  }
  std::vector<DevReaction> R(std::max(1, d->n_reactions));
  for (int r = 0; r < d->n_reactions; r++) {
    const afh_reaction &a = d->reactions[r];
    DevReaction &b = R[r];
    b.rate_type = a.rate_type, b.table_col = a.table_col, b.n_in = a.n_in, b.n_out = a.n_out;
    b.rate_factor = a.rate_factor;
    for (int q = 0; q < 4; q++) {
      b.c[q] = a.c[q], b.ix_in[q] = a.ix_in[q], b.ix_out[q] = a.ix_out[q];
      b.mult_out[q] = a.mult_out[q];
    }
  }
  H2(hipMalloc(&f->d_reac, sizeof(DevReaction) * R.size()));
  H2(hipMemcpy(f->d_reac, R.data(), sizeof(DevReaction) * R.size(), hipMemcpyHostToDevice));
  *out = f;
  return AFH_OK;
}

int32_t afh_fluid_destroy(afh_fluid *f) {
  if (!f) return AFH_OK;
  hipStreamSynchronize(f->t->stream);
  hipFree(f->d_td), hipFree(f->d_chem), hipFree(f->d_reac);
  delete f;
  return AFH_OK;
}

}  // extern "C"

namespace afh2 {

static constexpr double RHS_FAC = -1.6022e-19 / 8.8541878176e-12;  // -e / eps0

static int32_t set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in, double *max_rhs) {
  afh_tree *t = f->t;
  if (int32_t e = check_iv(t, i_rhs, "afh_field_set_rhs")) return e;
  RhsArgs A;
  A.n = 0;
  for (int s = 0; s < f->d.n_species; s++) {
    if (f->d.species_charge[s] == 0) continue;
    A.sp[A.n] = t->ccv(f->d.species_iv[s] + s_in);
    A.q[A.n] = f->d.species_charge[s] * RHS_FAC;
    A.n++;
  }
  if (max_rhs)
    if (int32_t e = red_init(t, 3, 0.0)) return e;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k2_set_rhs, grid2(t->bsz, n), blk2(t->bsz), 0, t->stream, t->ccv(i_rhs), A,
                       t->leaves.at(l), t->nc, t->bsz,
                       max_rhs ? t->red + 3 * RED_SHARDS : nullptr);
    H2_LAUNCH("k2_set_rhs");
  }
  return max_rhs ? red_read(t, 3, 1, 1, max_rhs) : AFH_OK;
}

static DevLT dev_lt(const afh_lt &lt, const double *d) {
  DevLT r;
  r.n_points = lt.n_points, r.n_cols = lt.n_cols, r.x_min = lt.x_min, r.inv_fac = lt.inv_fac;
  r.rc = d;
  return r;
}

// flux_upwind_tree (m_af_flux_schemes.f90:666-712); dt_lim = (1 / max CFL
// sum, dielectric relaxation time)
// the CFL and dielectric relaxation limits from the folded maxima
static void flux_limits(const double *r, double *dt_lim) {
  const double eps0 = 8.8541878176e-12, ec = 1.6022e-19;
  dt_lim[0] = 1 / r[0];
  dt_lim[1] = eps0 / (ec * std::max(r[1], 1e-100));
}

// fetch = false: the CFL and dielectric maxima stay in slots 0, 1 for
// afh_fluid_fetch_step
static int32_t flux_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim, bool fetch = true) {
  afh_tree *t = f->t;
  const int iv = f->d.i_electron + s_deriv;
  if (int32_t e = check_iv(t, iv, "afh_flux_upwind_tree")) return e;
  if (!t->meth[iv].set) return set_error(AFH_ERR_STATE, "flux: no methods for %d", iv);
  const int nc = t->nc;
  // af_restrict_ref_boundary
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->refb.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k2_restrict, grid2(nc * nc / 4, n), blk2(nc * nc / 4), 0, t->stream,
                       t->ccv(iv), t->d_boxes, t->refb.at(l), nc, t->bsz);
    H2_LAUNCH("k2_restrict");
  }
  int32_t e;
  if ((e = red_init(t, 0, -HUGE_VAL, 2))) return e;  // CFL and conductivity maxima
  FluxArgs A;
  A.ne = t->ccv(iv), A.E = t->ccv(f->d.i_efld), A.Ef = t->fcv(f->d.f_field);
  A.F = t->fcv(f->d.f_flux), A.gc2 = t->gc2;
  A.td = dev_lt(f->d.td, f->d_td);
  A.N_inv = 1 / f->d.gas_number_density;
  A.lim = f->d.limiter;
  // level by level: a level's refinement-boundary ghost cells read the
  // coarser leaves' ghost cells, which their own gc2 wrote (the reference's
  // level loop)
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k2_gc2, grid2(4 * nc, n), blk2(4 * nc), 0, t->stream, t->ccv(iv), t->gc2,
                       t->d_boxes, t->leaves.at(l), nc, t->bsz, t->bc4(iv));
    H2_LAUNCH("k2_gc2");
    prof_mark(t, AFH_PROF_FLUX);
    hipLaunchKernelGGL(k2_flux, grid2(nc * nc, n), blk2(nc * nc), 0, t->stream, A,
                       t->leaves.at(l), t->d_boxes, nc, t->bsz, t->fsz, t->red);
    H2_LAUNCH("k2_flux");
    // ne and |E| read, two face fields read and two fluxes written per cell
    prof_end(t, AFH_PROF_FLUX, 48.0 * nc * nc * n);
  }
  // af_consistent_fluxes
  const int ntask = t->cflux.off.back();
  if (ntask) {
    hipLaunchKernelGGL(k2_consistent, dim3((ntask * nc + NT - 1) / NT), dim3(NT), 0, t->stream,
                       t->fcv(f->d.f_flux), t->d_boxes, t->cflux.d, ntask, nc, t->fsz);
    H2_LAUNCH("k2_consistent");
  }
  if (!fetch) return AFH_OK;
  double r[2];
  if ((e = red_read(t, 0, 2, 3, r))) return e;
  flux_limits(r, dt_lim);
  return AFH_OK;
}

// fetch = false: the chemistry minimum stays in slot 2 (last step)
static int32_t update(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                      const int32_t *s_prev, const double *w_prev, int32_t s_out,
                      int32_t last_step, double *dt_lim, bool fetch = true) {
  afh_tree *t = f->t;
  if (n_prev < 1 || n_prev > MAXPREV || !s_prev || !w_prev)
    return set_error(AFH_ERR_ARG, "afh_flux_update_densities: previous states");
  UpdArgs A;
  A.ns = f->d.n_species, A.nr = f->d.n_reactions, A.n_prev = n_prev;
  A.last_step = last_step != 0;
  A.e_index = -1;
  for (int s = 0; s < A.ns; s++) {
    const int iv = f->d.species_iv[s];
    if (iv == f->d.i_electron) A.e_index = s;
    for (int q = 0; q < n_prev; q++) A.prev[s][q] = t->ccv(iv + s_prev[q]);
    A.der[s] = t->ccv(iv + s_deriv);
    A.out[s] = t->ccv(iv + s_out);
  }
  if (A.e_index < 0) return set_error(AFH_ERR_ARG, "flux species is no species");
  for (int q = 0; q < n_prev; q++) A.w_prev[q] = w_prev[q];
  A.E = t->ccv(f->d.i_efld), A.F = t->fcv(f->d.f_flux), A.reac = f->d_reac;
  A.chem = dev_lt(f->d.chem, f->d_chem);
  A.inv_N = 1 / f->d.gas_number_density;
  A.dt = dt, A.dt_chemistry_nmin = f->d.dt_chemistry_nmin;
  if (A.last_step)
    if (int32_t e = red_init(t, 2, 1e100)) return e;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    const dim3 g = grid2(t->nc * t->nc, n);
    const dim3 bk = blk2(t->nc * t->nc);
    const int32_t *ids = t->leaves.at(l);
    unsigned long long *red = t->red + 2 * RED_SHARDS;
    switch (A.ns) {
#define AFH2_UPD(N) \
  case N: hipLaunchKernelGGL(k2_update<N>, g, bk, 0, t->stream, A, ids, t->d_boxes, t->nc, t->bsz, t->fsz, red); break;
      AFH2_UPD(1) AFH2_UPD(2) AFH2_UPD(3) AFH2_UPD(4) AFH2_UPD(5) AFH2_UPD(6) AFH2_UPD(7)
      AFH2_UPD(8) AFH2_UPD(9) AFH2_UPD(10) AFH2_UPD(11) AFH2_UPD(12)
#undef AFH2_UPD
    default:
      hipLaunchKernelGGL(k2_update<MAXS>, g, bk, 0, t->stream, A, ids, t->d_boxes,
                         t->nc, t->bsz, t->fsz, red);
    }
    H2_LAUNCH("k2_update");
  }
  dt_lim[0] = 1e100, dt_lim[1] = 1e100;
  if (A.last_step && fetch) return red_read(t, 2, 1, 0, dt_lim);
  return AFH_OK;
}

}  // namespace afh2

extern "C" {

int32_t afh_field_set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in) {
  if (!f) return set_error(AFH_ERR_ARG, "null fluid");
  return set_rhs(f, i_rhs, s_in, nullptr);
}

int32_t afh_field_set_rhs_maxabs(afh_fluid *f, int32_t i_rhs, int32_t s_in, double *max_rhs) {
  if (!f || !max_rhs) return set_error(AFH_ERR_ARG, "afh_field_set_rhs_maxabs: null");
  return set_rhs(f, i_rhs, s_in, max_rhs);
}

int32_t afh_flux_upwind_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim) {
  if (!f || !dt_lim) return set_error(AFH_ERR_ARG, "afh_flux_upwind_tree: null");
  return flux_tree(f, s_deriv, dt_lim);
}

int32_t afh_flux_update_densities(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                                  const int32_t *s_prev, const double *w_prev, int32_t s_out,
                                  int32_t last_step, double *dt_lim) {
  if (!f || !dt_lim) return set_error(AFH_ERR_ARG, "afh_flux_update_densities: null");
  return update(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, dt_lim);
}

int32_t afh_fluid_forward_euler(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                                const int32_t *s_prev, const double *w_prev, int32_t s_out,
                                int32_t last_step, int32_t store_flux, double *dt_lim) {
  (void)store_flux;  // the 2-D step always stores the face fluxes
  if (!f || !dt_lim) return set_error(AFH_ERR_ARG, "afh_fluid_forward_euler: null");
  int32_t e;
  if ((e = flux_tree(f, s_deriv, dt_lim))) return e;
  return update(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, dt_lim + 2);
}

// Deferred reductions, as libafivo_hip: the step's limits stay in slots 0..2
// and afh_fluid_fetch_step reads them -- with the V-cycle residual of
// afh_mg_fas_vcycle_fold (slot 3) -- in one transfer
int32_t afh_fluid_forward_euler_fold(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                                     const int32_t *s_prev, const double *w_prev, int32_t s_out,
                                     int32_t last_step, int32_t store_flux) {
  (void)store_flux;
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_forward_euler_fold: null");
  double lim[4];
  int32_t e;
  if ((e = flux_tree(f, s_deriv, lim, false))) return e;
  return update(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, lim + 2, false);
}

int32_t afh_fluid_fetch_step(afh_fluid *f, int32_t last_step, int32_t n_extra,
                             const int32_t *extra_slots, double *dt_lim, double *extra) {
  if (!f || !dt_lim || (n_extra > 0 && (!extra_slots || !extra)))
    return set_error(AFH_ERR_ARG, "afh_fluid_fetch_step: null");
  if (n_extra < 0 || n_extra > 1) return set_error(AFH_ERR_ARG, "%d extra slots", n_extra);
  if (n_extra && extra_slots[0] != 3)
    return set_error(AFH_ERR_ARG, "extra slot %d (the 2-D build: 3 only)", extra_slots[0]);
  // slots 0, 1 maxima (CFL, sigma), 2 the chemistry minimum, 3 max |res|
  double r[4];
  if (int32_t e = red_read(f->t, 0, n_extra ? 4 : 3, 0xB, r)) return e;
  flux_limits(r, dt_lim);
  dt_lim[2] = last_step ? r[2] : 1e100;
  dt_lim[3] = 1e100;
  if (n_extra) extra[0] = r[3];
  return AFH_OK;
}

}  // extern "C"

// ============================================================ regrid, refinement, sums
namespace afh2 {

// af_prolong_limit / af_prolong_linear, NDIM = 2 (m_af_prolong.f90:311-420,
// 531-679) with add = .false.: one thread per parent cell of the child's
// quadrant writes its 4 child cells (value + 0: the child interior is zeroed
// first, so -0 becomes +0 as in the reference)
template <int METHOD>
__global__ void __launch_bounds__(NT)
    k2_prolong_new(double *__restrict__ v, const afh_box_meta *__restrict__ meta,
                   const int32_t *__restrict__ ids, int nc, int bsz, int lim) {
  const int hn = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hn * hn) return;
  const int id = ids[blockIdx.y];
  const afh_box_meta &m = meta[id - 1];
  const int i = t % hn + 1, j = t / hn + 1, ng = nc + 2;
  const int ic = i + ((m.ix[0] - 1) & 1) * hn, jc = j + ((m.ix[1] - 1) & 1) * hn;
  const double *p = v + (size_t)(m.parent - 1) * bsz;
  double *c = v + (size_t)(id - 1) * bsz;
  const int fi = 2 * i - 1, fj = 2 * j - 1;
  auto P = [&](int a, int b) { return p[ix2(ng, ic + a, jc + b)]; };
  if (METHOD == AFH_PROLONG_LIMIT) {
    const double f0 = P(0, 0);
    const double f1 = 0.25 * limiter(lim, P(0, 0) - P(-1, 0), P(1, 0) - P(0, 0));
    const double f2 = 0.25 * limiter(lim, P(0, 0) - P(0, -1), P(0, 1) - P(0, 0));
    c[ix2(ng, fi, fj)] = f0 - f1 - f2 + 0.0;
    c[ix2(ng, fi + 1, fj)] = f0 + f1 - f2 + 0.0;
    c[ix2(ng, fi, fj + 1)] = f0 - f1 + f2 + 0.0;
    c[ix2(ng, fi + 1, fj + 1)] = f0 + f1 + f2 + 0.0;
  } else {
    const double f1 = 1 / 16.0, f3 = 3 / 16.0, f9 = 9 / 16.0;
    const double f0 = f9 * P(0, 0);
    const double flx = f3 * P(-1, 0), fhx = f3 * P(1, 0);
    const double fly = f3 * P(0, -1), fhy = f3 * P(0, 1);
    const double fll = f1 * P(-1, -1), fhl = f1 * P(1, -1);
    const double flh = f1 * P(-1, 1), fhh = f1 * P(1, 1);
    c[ix2(ng, fi, fj)] = f0 + flx + fly + fll + 0.0;
    c[ix2(ng, fi + 1, fj)] = f0 + fhx + fly + fhl + 0.0;
    c[ix2(ng, fi, fj + 1)] = f0 + flx + fhy + flh + 0.0;
    c[ix2(ng, fi + 1, fj + 1)] = f0 + fhx + fhy + fhh + 0.0;
  }
}

// boxes ids[blockIdx.y] of variable blockIdx.z from one pool to another (the
// pools of a regrid hold different box counts: different variable strides)
__global__ void __launch_bounds__(NT)
    k2_copy_boxes(const double *__restrict__ src, double *__restrict__ dst,
                  const int32_t *__restrict__ ids, int per_box, size_t src_var,
                  size_t dst_var) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per_box) return;
  const size_t b = (size_t)(ids[blockIdx.y] - 1) * per_box + t;
  dst[blockIdx.z * dst_var + b] = src[blockIdx.z * src_var + b];
}

// NORM2 as the Fortran runtime the reference is built with evaluates it
// (afh.electrode.norm2): the largest |x| so far m, s = sum (x / m)^2 without
// m's own term, element by element; m sqrt(s + 1)
__device__ __forceinline__ double norm2_rt(const double *x, int n) {
  double m = 0.0, s = 0.0;
  for (int q = 0; q < n; q++) {
    const double a = fabs(x[q]);
    if (m == 0.0) {
      m = a;
    } else if (a > m) {
      double u = m / a;
      u = u * u;
      s = s * u + u;
      m = a;
    } else {
      const double u = a / m;
      s = s + u * u;
    }
  }
  return m * sqrt(s + 1.0);
}

// GM_dist_line (src/m_geometry.f90:21-51), n_dim = 2
__device__ __forceinline__ double dist_line2(const double r[2], const double *r0,
                                             const double *r1) {
  const double d0 = r1[0] - r0[0], d1 = r1[1] - r0[1];
  const double len2 = d0 * d0 + d1 * d1;
  const double frac = (r[0] - r0[0]) * d0 + (r[1] - r0[1]) * d1;
  double dv[2];
  if (frac <= 0.0) {
    dv[0] = r[0] - r0[0], dv[1] = r[1] - r0[1];
  } else if (frac >= len2) {
    dv[0] = r[0] - r1[0], dv[1] = r[1] - r1[1];
  } else {
    dv[0] = r[0] - (r0[0] + frac / len2 * d0);
    dv[1] = r[1] - (r0[1] + frac / len2 * d1);
  }
  return norm2_rt(dv, 2);
}

struct RefineArgs2 {
  afh_refine_desc d;
  DevLT td;
  double N;
  const double *ne, *E;
};

// default_refinement (src/m_refine.f90:198-298), NDIM = 2, per cell, reduced
// per box as cell_to_ref_flags does (m_af_core.f90:1095-1148): flag = do if
// any cell asks for refinement, else keep if any keeps, else remove; mask bit
// (dj+1)*3 + (di+1) when a cell within buffer_width of the side towards the
// neighbour (di, dj) asks for refinement. One workgroup per box.
__global__ void __launch_bounds__(NT)
    k2_refine_flags(RefineArgs2 A, const afh_box_meta *__restrict__ meta,
                    const int32_t *__restrict__ ids, int nc, int bsz,
                    int32_t *__restrict__ flags, uint32_t *__restrict__ masks) {
  const afh_refine_desc &p = A.d;
  const int id = ids[blockIdx.x];
  const afh_box_meta &b = meta[id - 1];
  __shared__ int s_do, s_keep;
  __shared__ unsigned s_mask;
  if (threadIdx.x == 0) s_do = 0, s_keep = 0, s_mask = 0;
  __syncthreads();
  const double min_dx = b.dr[0] < b.dr[1] ? b.dr[0] : b.dr[1];
  const double max_dx = b.dr[0] > b.dr[1] ? b.dr[0] : b.dr[1];
  const int bw = p.buffer_width;
  double rmin[2], rmax[2];
  for (int d = 0; d < 2; d++) rmin[d] = b.r_min[d], rmax[d] = b.r_min[d] + b.dr[d] * nc;
  int any_do = 0, any_keep = 0;
  unsigned msk = 0;
  for (int t = threadIdx.x; t < nc * nc; t += blockDim.x) {
    const int i = t % nc + 1, j = t / nc + 1;
    const size_t x = (size_t)(id - 1) * bsz + ix2(nc + 2, i, j);
    const double gas_dens = A.N;
    const double fld = A.E[x] * 1e21 / gas_dens;
    double alpha;
    if (p.use_alpha_effective) {
      alpha = (lt_col(A.td, p.td_alpha_col, p.adx_fac * fld) -
               lt_col(A.td, p.td_eta_col, p.adx_fac * fld)) *
              gas_dens / p.adx_fac;
      alpha = alpha > 0.0 ? alpha : 0.0;
    } else {
      alpha = lt_col(A.td, p.td_alpha_col, p.adx_fac * fld) * gas_dens / p.adx_fac;
    }
    const double adx = max_dx * alpha, ne = A.ne[x];
    int f;
    if (adx > p.adx && ne > p.min_dens) f = AFH_DO_REF;
    else if (adx < 0.125 * p.adx && max_dx < p.derefine_dx) f = AFH_RM_REF;
    else f = AFH_KEEP_REF;
    // af_r_cc: r_min + (i - 0.5) dr
    const double r[2] = {b.r_min[0] + (i - 0.5) * b.dr[0], b.r_min[1] + (j - 0.5) * b.dr[1]};
    for (int n = 0; n < p.n_seeds; n++) {
      const double dist = dist_line2(r, p.seed_r0[n], p.seed_r1[n]);
      if (dist - p.seed_width[n] < 2 * max_dx && max_dx > p.init_fac * p.seed_width[n])
        f = AFH_DO_REF;
    }
    for (int n = 0; n < p.n_regions; n++) {
      bool in = max_dx > p.region_dr[n];
      for (int d = 0; d < 2; d++)
        in = in && rmax[d] >= p.region_rmin[n][d] && rmin[d] <= p.region_rmax[n][d];
      if (in && i == nc / 2 && j == nc / 2) f = AFH_DO_REF;
    }
    for (int n = 0; n < p.n_limits; n++) {
      bool in = max_dx < 2 * p.limit_dr[n];
      for (int d = 0; d < 2; d++)
        in = in && rmin[d] >= p.limit_rmin[n][d] && rmax[d] <= p.limit_rmax[n][d];
      if (in && f == AFH_DO_REF) f = AFH_KEEP_REF;
    }
    if (max_dx > p.max_dx) f = AFH_DO_REF;
    else if (min_dx < 2 * p.min_dx && f == AFH_DO_REF) f = AFH_KEEP_REF;
    if (f == AFH_DO_REF) {
      any_do = 1;
      if (bw > 0) {
        const bool lo[2] = {i <= bw, j <= bw}, hi[2] = {i > nc - bw, j > nc - bw};
        for (int dj = -1; dj <= 1; dj++)
          for (int di = -1; di <= 1; di++) {
            if (!di && !dj) continue;
            const int dd[2] = {di, dj};
            bool in = true;
            for (int d = 0; d < 2; d++) in = in && (dd[d] == 0 || (dd[d] < 0 ? lo[d] : hi[d]));
            if (in) msk |= 1u << ((dj + 1) * 3 + (di + 1));
          }
      }
    } else if (f == AFH_KEEP_REF) {
      any_keep = 1;
    }
  }
  if (any_do) atomicOr(&s_do, 1);
  if (any_keep) atomicOr(&s_keep, 1);
  if (msk) atomicOr(&s_mask, msk);
  __syncthreads();
  if (threadIdx.x == 0) {
    flags[id - 1] = s_do ? AFH_DO_REF : s_keep ? AFH_KEEP_REF : AFH_RM_REF;
    masks[id - 1] = s_mask;
  }
}

// gfortran's real ** integer (_gfortran_pow_r8_i4): binary powering
__device__ __forceinline__ double ipow2(double x, int n) {
  double p = 1.0;
  for (;;) {
    if (n & 1) p *= x;
    n >>= 1;
    if (!n) break;
    x *= x;
  }
  return p;
}

// Per leaf box (one thread each; 2-D boxes are small): OP 0 the sum of
// cc(1:nc, 1:nc)**power in the Fortran element order (j outer, i inner);
// AFH_RED_MAX / MIN / MAXABS the extremum and its first cell (i fastest)
template <int OP>
__global__ void __launch_bounds__(NT)
    k2_box_reduce(const double *__restrict__ v, const int32_t *__restrict__ ids, int nl,
                  int nc, int bsz, int power, double *__restrict__ out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nl) return;
  const double *c = v + (size_t)(ids[q] - 1) * bsz;
  const int ng = nc + 2;
  double best = OP == 0 ? 0.0 : (OP == AFH_RED_MIN ? HUGE_VAL : -HUGE_VAL);
  int bix = -1;
  for (int j = 1; j <= nc; j++)
    for (int i = 1; i <= nc; i++) {
      double x = c[ix2(ng, i, j)];
      if (OP == 0) {
        best = best + ipow2(x, power);
      } else {
        if (OP == AFH_RED_MAXABS) x = fabs(x);
        if (bix < 0 || (OP == AFH_RED_MIN ? x < best : x > best))
          best = x, bix = (j - 1) * nc + (i - 1);
      }
    }
  out[2 * q] = best;
  out[2 * q + 1] = (double)bix;
}

static int32_t device_list(const std::vector<int32_t> &h, int32_t **d) {
  H2(hipMalloc(d, sizeof(int32_t) * std::max<size_t>(1, h.size())));
  if (!h.empty())
    H2(hipMemcpy(*d, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice));
  return AFH_OK;
}

static int32_t box_reduce(afh_tree *t, int iv, int op, int power, std::vector<double> &res) {
  const int nl = t->leaves.off[t->nlvl];
  res.assign(2 * (size_t)nl, 0.0);
  if (!nl) return AFH_OK;
  if (!t->d_boxred) H2(hipMalloc(&t->d_boxred, sizeof(double) * 2 * t->nb));
  const dim3 grid((nl + NT - 1) / NT), blk(NT);
  const double *v = t->ccv(iv);
  switch (op) {
  case 0:
    hipLaunchKernelGGL(k2_box_reduce<0>, grid, blk, 0, t->stream, v, t->leaves.d, nl, t->nc,
                       t->bsz, power, t->d_boxred);
    break;
  case AFH_RED_MAX:
    hipLaunchKernelGGL(k2_box_reduce<AFH_RED_MAX>, grid, blk, 0, t->stream, v, t->leaves.d, nl,
                       t->nc, t->bsz, power, t->d_boxred);
    break;
  case AFH_RED_MIN:
    hipLaunchKernelGGL(k2_box_reduce<AFH_RED_MIN>, grid, blk, 0, t->stream, v, t->leaves.d, nl,
                       t->nc, t->bsz, power, t->d_boxred);
    break;
  default:
    hipLaunchKernelGGL(k2_box_reduce<AFH_RED_MAXABS>, grid, blk, 0, t->stream, v, t->leaves.d,
                       nl, t->nc, t->bsz, power, t->d_boxred);
  }
  H2_LAUNCH("k2_box_reduce");
  H2(hipMemcpyAsync(res.data(), t->d_boxred, sizeof(double) * 2 * nl, hipMemcpyDeviceToHost,
                    t->stream));
  H2(hipStreamSynchronize(t->stream));
  return AFH_OK;
}

}  // namespace afh2

extern "C" {

int32_t afh_set_cc_prolong(afh_tree *t, int32_t iv, int32_t method, int32_t limiter) {
  if (int32_t e = check_iv(t, iv, "afh_set_cc_prolong")) return e;
  if (method < AFH_PROLONG_NONE || method > AFH_PROLONG_LIMIT)
    return set_error(AFH_ERR_UNSUPPORTED, "prolongation method %d", method);
  if (!t->meth[iv].set) return set_error(AFH_ERR_STATE, "set cc methods first");
  if (method != AFH_PROLONG_NONE &&
      std::find(t->auto_vars.begin(), t->auto_vars.end(), iv) == t->auto_vars.end())
    t->auto_vars.push_back(iv);
  t->meth[iv].prolong = method;
  t->meth[iv].prolong_lim = limiter;
  return AFH_OK;
}

// af_adjust_refinement's data movement (m_af_core.f90:697-881) onto the new
// topology: auto_restrict into boxes whose children go, the data of the
// boxes that persist (same id, level and index), then auto_prolong level by
// level (every automatic variable of the new boxes from their parents, then
// their ghost cells, corners included). The old tree stays valid.
int32_t afh_tree_regrid(afh_tree *o, const afh_tree_desc *d, afh_tree **out) {
  if (!o || !d || !out) return set_error(AFH_ERR_ARG, "afh_tree_regrid: null");
  if (d->n_cell != o->nc || d->n_var_cell != o->nvc || d->n_var_face != o->nvf)
    return set_error(AFH_ERR_ARG, "afh_tree_regrid: box size / variables differ");
  std::vector<char> in_old(o->nb + 1, 0), keep(d->n_boxes + 1, 0);
  for (const auto &L : o->h_ids)
    for (int32_t id : L) in_old[id] = 1;
  std::vector<int32_t> kept, rchild;
  for (int q = 0; q < d->lvl_ids_off[d->highest_lvl]; q++) {
    const int32_t id = d->lvl_ids[q];
    if (id < 1 || id > d->n_boxes) return set_error(AFH_ERR_ARG, "bad box id %d", id);
    if (id > o->nb || !in_old[id]) continue;
    const afh_box_meta &a = o->boxes[id - 1], &b = d->boxes[id - 1];
    if (a.lvl != b.lvl || a.ix[0] != b.ix[0] || a.ix[1] != b.ix[1]) continue;
    keep[id] = 1;
    kept.push_back(id);
    // auto_restrict (m_af_core.f90:826-840): the box lost its children
    if (a.children[0] > 0 && b.children[0] == 0)
      for (int c = 0; c < 4; c++) rchild.push_back(a.children[c]);
  }
  int32_t *d_list = nullptr;
  int32_t e;
  const int nc = o->nc;
  if (!rchild.empty()) {
    if ((e = device_list(rchild, &d_list))) return e;
    for (int iv : o->auto_vars) {
      hipLaunchKernelGGL(k2_restrict, grid2(nc * nc / 4, (int)rchild.size()), blk2(nc * nc / 4), 0,
                         o->stream, o->ccv(iv), o->d_boxes, d_list, nc, o->bsz);
      H2_LAUNCH("k2_restrict");
    }
    H2(hipStreamSynchronize(o->stream));
    hipFree(d_list);
    d_list = nullptr;
  }
  afh_tree *t = nullptr;
  if ((e = afh_tree_create(d, o->device, &t))) return e;
  t->meth = o->meth;
  t->auto_vars = o->auto_vars;
  if (!kept.empty()) {
    if ((e = device_list(kept, &d_list))) return e;
    const unsigned n = (unsigned)kept.size();
    hipLaunchKernelGGL(k2_copy_boxes, dim3((unsigned)((t->bsz + NT - 1) / NT), n, t->nvc),
                       dim3(NT), 0, t->stream, o->cc, t->cc, d_list, t->bsz,
                       (size_t)o->nb * o->bsz, (size_t)t->nb * t->bsz);
    H2_LAUNCH("k2_copy_boxes");
    if (t->nvf > 0) {
      hipLaunchKernelGGL(k2_copy_boxes, dim3((unsigned)((t->fsz + NT - 1) / NT), n, t->nvf),
                         dim3(NT), 0, t->stream, o->fc, t->fc, d_list, t->fsz,
                         (size_t)o->nb * o->fsz, (size_t)t->nb * t->fsz);
      H2_LAUNCH("k2_copy_boxes");
    }
    H2(hipStreamSynchronize(t->stream));
    hipFree(d_list);
    d_list = nullptr;
  }
  const int hn = nc / 2;
  for (int l = 2; l <= t->nlvl; l++) {
    std::vector<int32_t> add;
    for (int32_t id : t->h_ids[l - 1])
      if (!keep[id]) add.push_back(id);
    if (add.empty()) continue;
    if ((e = device_list(add, &d_list))) return e;
    const int n = (int)add.size();
    for (int iv : t->auto_vars) {
      const Meth &m = t->meth[iv];
      auto kern = m.prolong == AFH_PROLONG_LIMIT ? k2_prolong_new<AFH_PROLONG_LIMIT>
                                                 : k2_prolong_new<AFH_PROLONG_LINEAR>;
      hipLaunchKernelGGL(kern, grid2(hn * hn, n), blk2(hn * hn), 0, t->stream, t->ccv(iv),
                         t->d_boxes, d_list, nc, t->bsz, m.prolong_lim);
      H2_LAUNCH("k2_prolong_new");
    }
    // af_gc_box of every new box (sides, then corners) once all are prolonged
    for (int iv : t->auto_vars) {
      hipLaunchKernelGGL(k2_gc, grid2(4 * nc, n), blk2(4 * nc), 0, t->stream, t->ccv(iv),
                         t->d_boxes, d_list, nc, t->bsz, t->bc4(iv));
      H2_LAUNCH("k2_gc");
      hipLaunchKernelGGL(k2_corners, dim3((4 * n + NT - 1) / NT), dim3(NT), 0, t->stream,
                         t->ccv(iv), t->d_boxes, d_list, n, nc, t->bsz);
      H2_LAUNCH("k2_corners");
    }
    H2(hipStreamSynchronize(t->stream));
    hipFree(d_list);
    d_list = nullptr;
  }
  *out = t;
  return AFH_OK;
}

int32_t afh_refine_flags(afh_fluid *f, const afh_refine_desc *d, const uint8_t *electrode_box,
                         int32_t *flags, uint32_t *masks) {
  if (!f || !d || !flags || !masks) return set_error(AFH_ERR_ARG, "afh_refine_flags: null");
  afh_tree *t = f->t;
  if (electrode_box) return set_error(AFH_ERR_UNSUPPORTED, "2-D: electrodes");
  if (d->n_seeds > AFH_MAX_REFINE_REGIONS || d->n_regions > AFH_MAX_REFINE_REGIONS ||
      d->n_limits > AFH_MAX_REFINE_REGIONS || d->buffer_width < 0 ||
      d->buffer_width > t->nc || d->i_electron < 1 || d->i_electron > t->nvc ||
      d->i_efld < 1 || d->i_efld > t->nvc || d->td_alpha_col < 1 ||
      d->td_alpha_col > f->d.td.n_cols || d->td_eta_col < 1 || d->td_eta_col > f->d.td.n_cols)
    return set_error(AFH_ERR_ARG, "afh_refine_flags: bad descriptor");
  const int nb = t->nb, nids = t->ids.off[t->nlvl];
  int32_t *d_flags = nullptr;
  uint32_t *d_masks = nullptr;
  H2(hipMalloc(&d_flags, sizeof(int32_t) * nb));
  H2(hipMalloc(&d_masks, sizeof(uint32_t) * nb));
  H2(hipMemsetAsync(d_flags, 0, sizeof(int32_t) * nb, t->stream));
  H2(hipMemsetAsync(d_masks, 0, sizeof(uint32_t) * nb, t->stream));
  RefineArgs2 A;
  A.d = *d;
  A.td = dev_lt(f->d.td, f->d_td);
  A.N = f->d.gas_number_density;
  A.ne = t->ccv(d->i_electron);
  A.E = t->ccv(d->i_efld);
  if (nids > 0) {
    hipLaunchKernelGGL(k2_refine_flags, dim3(nids), dim3(NT), 0, t->stream, A, t->d_boxes,
                       t->ids.d, t->nc, t->bsz, d_flags, d_masks);
    H2_LAUNCH("k2_refine_flags");
  }
  H2(hipMemcpyAsync(flags, d_flags, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, t->stream));
  H2(hipMemcpyAsync(masks, d_masks, sizeof(uint32_t) * nb, hipMemcpyDeviceToHost, t->stream));
  H2(hipStreamSynchronize(t->stream));
  hipFree(d_flags), hipFree(d_masks);
  return AFH_OK;
}

// af_tree_sum_cc (m_af_utils.f90:966-1026), Cartesian: per leaf the sum of
// cc**power, then my_sum = my_sum + fac * tmp in the reference's loop order
// (levels, then leaves), fac = product(af_lvl_dr)
int32_t afh_tree_sum_cc(afh_tree *t, int32_t iv, int32_t power, double *out) {
  if (int32_t e = check_iv(t, iv, "afh_tree_sum_cc")) return e;
  if (power < 1 || !out) return set_error(AFH_ERR_ARG, "afh_tree_sum_cc: bad argument");
  std::vector<double> res;
  if (int32_t e = box_reduce(t, iv, 0, power, res)) return e;
  double sum = 0.0;
  size_t q = 0;
  for (int l = 1; l <= t->nlvl; l++) {
    const double fac = t->lvl_dr[2 * (l - 1)] * t->lvl_dr[2 * (l - 1) + 1];
    for (int b = 0; b < t->leaves.n(l); b++, q++) sum = sum + fac * res[2 * q];
  }
  *out = sum;
  return AFH_OK;
}

// af_tree_max_cc / min_cc / maxabs_cc with af_reduction_loc (m_af_utils.f90:
// 694-874): loc = (box id, i, j, 0), the first cell of the first box in loop
// order holding the extremum
int32_t afh_tree_reduce_loc(afh_tree *t, int32_t iv, int32_t op, double *out, int32_t *loc) {
  if (int32_t e = check_iv(t, iv, "afh_tree_reduce_loc")) return e;
  if (!out || op < AFH_RED_MAX || op > AFH_RED_MAXABS)
    return set_error(AFH_ERR_ARG, "afh_tree_reduce_loc: bad argument");
  std::vector<double> res;
  if (int32_t e = box_reduce(t, iv, op, 1, res)) return e;
  const bool is_min = op == AFH_RED_MIN;
  double val = (is_min ? 1 : -1) * (1.7976931348623157e308 / 10);
  int32_t lid = -1, lix = -1;
  size_t q = 0;
  for (int l = 1; l <= t->nlvl; l++)
    for (int b = 0; b < t->leaves.n(l); b++, q++) {
      const double tmp = res[2 * q];
      const double nv = is_min ? std::min(tmp, val) : std::max(tmp, val);
      if (std::fabs(nv - val) > 0) {
        val = tmp;
        lid = t->h_leaves[l - 1][b];
        lix = (int32_t)res[2 * q + 1];
      }
    }
  *out = val;
  if (loc) {
    const int nc = t->nc;
    loc[0] = lid;
    loc[1] = lix < 0 ? -1 : lix % nc + 1;
    loc[2] = lix < 0 ? -1 : lix / nc + 1;
    loc[3] = 0;
  }
  return AFH_OK;
}

}  // extern "C"
