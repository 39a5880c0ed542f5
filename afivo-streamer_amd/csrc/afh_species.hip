// Drift-diffusion-reaction fluid model on the device (src/m_fluid.f90 over
// afivo/src/m_af_flux_schemes.f90), electrons + immobile ions, LFA, constant
// gas density.
//
//   k_set_rhs       field_set_rhs (src/m_field.f90:363-401)
//   k_gc2           af_gc2_box (m_af_ghostcell.f90:672-744): 2 ghost layers of
//                   the flux species; layer 1 is written back into the box as
//                   the reference does, layer 2 goes to a per-box face buffer
//   k_flux          flux_upwind_box + reconstruct_upwind_1d + Koren limiter +
//                   the m_fluid flux_upwind / flux_direction callbacks; one
//                   thread per cell computes the low face of each dimension
//                   (and the high face on the last cell), plus the cell's CFL
//                   sum; max-reductions of CFL sum and conductivity
//   k_consistent    af_consistent_fluxes (m_af_core.f90:1257-1402)
//   k_update        flux_update_densities + add_source_terms + get_rates +
//                   get_derivatives (m_af_flux_schemes.f90:320-436,
//                   src/m_fluid.f90:298-466, src/m_chemistry.f90:565-688)
#include <algorithm>
#include <type_traits>
#include <utility>

#include "afh_internal.h"
#include "afh_networks.h"

namespace afh {

constexpr int MAXS = AFH_MAX_SPECIES;
constexpr int MAXPREV = 4;

__device__ __forceinline__ size_t fidx(int nf, int d, int i, int j, int k) {
  return (size_t)d * nf * nf * nf + ((size_t)(k - 1) * nf + (j - 1)) * nf +
         (i - 1);
}

struct DevLT {
  int n_points, n_cols;
  double x_min, inv_fac;
  const double *rc;
  const double *rm = nullptr;  // row-major copy [row][col] (chemistry table)
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

// limiter with a compile-time choice (LIM = AFH_LIM_KOREN, the reference's
// flux limiter) or the runtime switch (LIM = 0)
template <int LIM>
__device__ __forceinline__ double limiter_t(int lim, double a, double b) {
  if (LIM == AFH_LIM_KOREN) {
    const double third = 1 / 3.0;
    const double aa = a * a, ab = a * b;
    if (ab <= 0) return 0;
    if (aa <= 0.25 * ab) return 2 * a;
    if (aa <= 2.5 * ab) return third * (b + 2 * a);
    return 2 * b;
  }
  return limiter(lim, a, b);
}

// ------------------------------------------------------------ rhs
struct RhsArgs {
  int n;
  const double *sp[MAXS];
  double q[MAXS];
};

// rhs over the whole (nc+2)^3 block (ghosts included, as DTIMES(:) in the
// reference); with `red`, max|rhs| over the interior is folded into shard
// slots (af_tree_maxabs_cc over leaves: set_rhs runs on leaves only).
template <bool MAX>
__global__ void __launch_bounds__(256)
    k_set_rhs(double *__restrict__ rhs, RhsArgs A,
              const int32_t *__restrict__ ids, size_t bsz, int ng,
              unsigned long long *red) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double mx = 0.0;
  if (t < bsz) {
    const size_t o = (size_t)(ids[blockIdx.y] - 1) * bsz + t;
    double r = 0.0;
    for (int s = 0; s < A.n; s++) r = r + A.q[s] * A.sp[s][o];
    rhs[o] = r;
    if (MAX) {
      int i, j, k;
      cell3g((int)t, ng, i, j, k);
      if (i >= 1 && i < ng - 1 && j >= 1 && j < ng - 1 && k >= 1 && k < ng - 1)
        mx = fabs(r);
    }
  }
  if (MAX) block_max_to_shard(mx, red);
}

// k_set_rhs on the ghost shell of a box only (the interior is written by
// k_update with an rhs output): face blockIdx.y, one thread per cell of an
// ng x ng face; z faces whole, y faces without the z ghost rows, x faces
// without the y and z ghost rows, so every shell cell is written once.
__global__ void __launch_bounds__(256)
    k_rhs_shell(double *__restrict__ rhs, RhsArgs A,
                const int32_t *__restrict__ ids, size_t bsz, int ng) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ng * ng) return;
  const int a = t % ng, b = t / ng, f = blockIdx.y, d = f >> 1;
  const int side = (f & 1) ? ng - 1 : 0;
  int i, j, k;
  if (d == 2) {
    i = a, j = b, k = side;
  } else if (d == 1) {
    if (b == 0 || b == ng - 1) return;
    i = a, j = side, k = b;
  } else {
    if (a == 0 || a == ng - 1 || b == 0 || b == ng - 1) return;
    i = side, j = a, k = b;
  }
  const size_t o = (size_t)(ids[blockIdx.z] - 1) * bsz + ((size_t)k * ng + j) * ng + i;
  double r = 0.0;
  for (int s = 0; s < A.n; s++) r = r + A.q[s] * A.sp[s][o];
  rhs[o] = r;
}

// ------------------------------------------------------------ gc2
__global__ void k_gc2(double *__restrict__ v, double *__restrict__ gc2,
                      const afh_box_meta *__restrict__ meta,
                      const int32_t *__restrict__ ids, int nc, size_t bsz,
                      GcArgs ga) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc) return;
  const int id = ids[blockIdx.z];
  const int nb = blockIdx.y + 1;
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
  int a, b;
  if ((nc & (nc - 1)) == 0) {
    a = (t & (nc - 1)) + 1;
    b = (t >> __builtin_ctz(nc)) + 1;
  } else {
    a = t % nc + 1;
    b = t / nc + 1;
  }
  const int ng = nc + 2;
  const afh_box_meta &m = meta[id - 1];
  double *c = v + (size_t)(id - 1) * bsz;
  double *g2 = gc2 + ((size_t)(id - 1) * 6 + (nb - 1)) * nc * nc + t;
  const int nb_id = m.neighbors[nb - 1];
  int p[3];
  p[ta] = a;
  p[tb] = b;
  p[d] = low ? 0 : nc + 1;
  const size_t dst1 = ix3(ng, p[0], p[1], p[2]);
  double l1, l2;
  if (nb_id > 0) {
    const double *cn = v + (size_t)(nb_id - 1) * bsz;
    int q[3] = {p[0], p[1], p[2]};
    q[d] = low ? nc : 1;
    l1 = cn[ix3(ng, q[0], q[1], q[2])];
    q[d] = low ? nc - 1 : 2;
    l2 = cn[ix3(ng, q[0], q[1], q[2])];
  } else if (nb_id < 0) {
    // bc_to_gc2, incl. the c0 on layer 2 for highy (m_af_ghostcell.f90:361)
    double c0, c1, c2;
    const afh_bc bc = ga.bc[nb - 1];
    switch (bc.type) {
    case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = c0; break;
    case AFH_BC_NEUMANN: c0 = m.dr[d] * (low ? -1 : 1); c1 = 1; c2 = 3 * c0; break;
    default: c0 = 1; c1 = 0; c2 = c0; break;
    }
    if (nb == 4) c2 = c0;
    int q[3] = {p[0], p[1], p[2]};
    q[d] = low ? 1 : nc;
    l1 = c0 * bc.value + c1 * c[ix3(ng, q[0], q[1], q[2])];
    q[d] = low ? 2 : nc - 1;
    l2 = c2 * bc.value + c1 * c[ix3(ng, q[0], q[1], q[2])];
  } else {
    // gc2_prolong_rb: limited-slope prolongation from the parent's neighbour
    const int hnc = nc >> 1;
    const int p_nb_id = meta[m.parent - 1].neighbors[nb - 1];
    const double *cp = v + (size_t)(p_nb_id - 1) * bsz;
    int cc3[3];
    cc3[ta] = ((m.ix[ta] - 1) & 1) * hnc + ((a + 1) >> 1);
    cc3[tb] = ((m.ix[tb] - 1) & 1) * hnc + ((b + 1) >> 1);
    cc3[d] = low ? nc : 1;
    const size_t cq = ix3(ng, cc3[0], cc3[1], cc3[2]);
    const size_t st[3] = {1, (size_t)ng, (size_t)ng * ng};
    const double f0 = cp[cq];
    double f[3];
    for (int q = 0; q < 3; q++)
      f[q] = 0.25 * limiter(ga.lim, cp[cq] - cp[cq - st[q]],
                            cp[cq + st[q]] - cp[cq]);
    // sign per dim: - for the first fine cell of the pair, + for the second;
    // normal dim: layer order (-1, 0) low / (nc+1, nc+2) high
    double s[3];
    s[ta] = (a & 1) ? -1.0 : 1.0;
    s[tb] = (b & 1) ? -1.0 : 1.0;
    auto val = [&](double sn) {
      double sg[3] = {s[0], s[1], s[2]};
      sg[d] = sn;
      double r = f0;
      r = sg[0] < 0 ? r - f[0] : r + f[0];
      r = sg[1] < 0 ? r - f[1] : r + f[1];
      r = sg[2] < 0 ? r - f[2] : r + f[2];
      return r;
    };
    // low face: layer 2 (-1) is the first cell, layer 1 (0) the second
    l1 = val(low ? 1.0 : -1.0);
    l2 = val(low ? -1.0 : 1.0);
  }
  c[dst1] = l1;
  *g2 = l2;
}

// ------------------------------------------------------------ flux
struct FluxArgs {
  const double *ne;   // flux species, state s_deriv
  const double *E;    // |E| cell centred
  const double *Ef;   // face field
  // face field from the potential (afh_fluid_set_field_source): with phi
  // set, the kernels evaluate mg_box_lpl_gradient's face value
  // fac / dr * (phi_f - phi_{f-1}) themselves instead of reading Ef
  // (m_af_multigrid.f90:1882-1900): the same expression, bitwise
  const double *phi;
  double fac;
  double gfac[3];     // fac / dr per dimension of this level
  double *F;          // face flux
  // with mobile ions: the electrons' mu u per face (their share of the
  // dielectric relaxation sum, m_fluid.f90:196, 207-214) is stored here for
  // k_flux_ion, which folds the maximum of the sum (null: folded here)
  double *sig;
  const double *gc2;
  DevLT td;
  double N_inv;
  // variable gas density (cc variable, ghost cells filled) or null: then
  // N_inv = 2 / (N_{f-1} + N_f) per face (src/m_fluid.f90:146-154);
  // only k_flux_staged reads it
  const double *Ng;
  double inv_dx[3];   // 1/dr per dimension of this level
  int lim;
  // all leaf levels in one launch (k_flux_staged): the box's 1/dr from its
  // meta record (the same doubles as the level's, afh_tree_create checks)
  const afh_box_meta *meta;
};

// LT_get_col(td_tbl, td_mobility/td_diffusion, x): both columns at the same
// location (src/m_fluid.f90:168-174, m_lookup_table.f90:330-406)
__device__ __forceinline__ void lt_mu_dc(const DevLT &lt, double x, double &mu,
                                         double &dc) {
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
  const double *r = lt.rc + (low - 1);
  mu = lf * r[0] + (1 - lf) * r[1];
  dc = lf * r[lt.n_points] + (1 - lf) * r[lt.n_points + 1];
}

// One cell face between cells f-1 and f: upwind reconstruction with the
// limiter (reconstruct_upwind_1d, m_af_flux_schemes.f90:282-303) and the
// m_fluid flux_upwind callback (src/m_fluid.f90:160-205).
__device__ __forceinline__ void face_eval(const FluxArgs &A, double Lm2,
                                          double Lm1, double L0, double Lp1,
                                          double Elo, double Ehi, double ex,
                                          double inv_dx, double &v, double &dc,
                                          double &flux, double &sigma) {
  double u;
  if (-1 * ex > 0)
    u = Lm1 + 0.5 * limiter(A.lim, L0 - Lm1, Lm1 - Lm2);
  else
    u = L0 - 0.5 * limiter(A.lim, L0 - Lm1, Lp1 - L0);
  const double tfc = 0.5 * (Elo + Ehi) * 1e21 * A.N_inv;
  double mu, d;
  lt_mu_dc(A.td, tfc, mu, d);
  mu = mu * A.N_inv;
  dc = d * A.N_inv;
  v = -mu * ex;
  flux = v * u - dc * inv_dx * (L0 - Lm1);
  sigma = mu * u;
}

// transport only (for the CFL term of a face owned by another thread)
__device__ __forceinline__ void face_vd(const FluxArgs &A, double Elo,
                                        double Ehi, double ex, double &v,
                                        double &dc) {
  const double tfc = 0.5 * (Elo + Ehi) * 1e21 * A.N_inv;
  double mu, d;
  lt_mu_dc(A.td, tfc, mu, d);
  mu = mu * A.N_inv;
  dc = d * A.N_inv;
  v = -mu * ex;
}

// One thread per cell. Each thread owns the low face of its cell in every
// dimension (and the high face on the last cell of a line). The CFL sum needs
// the velocity / diffusion of the high face too: in x it comes from the next
// lane (__shfl_down, SHFL = lines of nc cells never straddle a wave); in y and
// z it is recomputed (transport only, bitwise identical expression).
// Table location of LT_get_loc (m_lookup_table.f90:330-363): row `low`
// (1-based) and weight `lf` of that row.
__device__ __forceinline__ void lt_loc(const DevLT &lt, double x, int &low,
                                       double &lf) {
  const double frac = (x - lt.x_min) * lt.inv_fac;
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
}

// Staged form of k_flux: (1) every neighbour value the thread needs is
// loaded up front (restrict-qualified, so the loads are issued together);
// (2) the table rows of all faces are fetched together; (3) limiter, flux,
// CFL. Same expressions in the same order as face_eval / face_vd, so the
// results are bitwise those of k_flux (which issued one memory round trip per
// face and table lookup). The CFL sum of a cell needs the transport of its
// high faces: x from the next lane (SHFL), y from the next row of the
// workgroup through LDS (the workgroup's last row and the box's last row
// evaluate it), z evaluated here.
// minimum waves per SIMD the flux kernel is compiled for (register budget)
#ifndef AFH_FLUX_MINW
#define AFH_FLUX_MINW 4
#endif
template <bool SHFL, int LIM, bool PHI = false>
__global__ void __launch_bounds__(256, AFH_FLUX_MINW)
    k_flux_staged(FluxArgs A, const int32_t *__restrict__ ids, int nc, size_t bsz,
                  size_t fsz, unsigned long long *red) {
  __shared__ double s_v[256], s_d[256];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = t < nc * nc * nc;
  const int tt = active ? t : 0;
  const int id = ids[blockIdx.y];
  int i, j, k;
  cell3(tt, nc, i, j, k);
  const int ng = nc + 2, nf = nc + 1;
  const double *__restrict__ ne = A.ne + (size_t)(id - 1) * bsz;
  const double *__restrict__ E = A.E + (size_t)(id - 1) * bsz;
  const double *__restrict__ Ef = A.Ef + (size_t)(id - 1) * fsz;
  double *__restrict__ F = A.F + (size_t)(id - 1) * fsz;
  const double *__restrict__ g2 = A.gc2 + (size_t)(id - 1) * 6 * nc * nc;
  const double *__restrict__ Ng = A.Ng ? A.Ng + (size_t)(id - 1) * bsz : nullptr;
  const int c0 = (k * ng + j) * ng + i;
  const int fcell = ((k - 1) * nf + (j - 1)) * nf + (i - 1);
  const int fd = nf * nf * nf;
  double idx[3], gf[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    idx[d] = A.meta ? 1 / A.meta[id - 1].dr[d] : A.inv_dx[d];
    // fac / dr; for fac = -1 (field_from_potential) that is -(1 / dr)
    // bitwise (IEEE division rounds symmetrically): no second division
    if (PHI)
      gf[d] = !A.meta ? A.gfac[d] : A.fac == -1.0 ? -idx[d] : A.fac / A.meta[id - 1].dr[d];
  }
  const double *__restrict__ ph = PHI ? A.phi + (size_t)(id - 1) * bsz : nullptr;
  const double P0 = PHI ? ph[c0] : 0.0;
  const int cc[3] = {i, j, k};
  const int st[3] = {1, ng, ng * ng};
  const int fst[3] = {1, nf, nf * nf};
  const int gq[3] = {(k - 1) * nc + (j - 1), (k - 1) * nc + (i - 1),
                     (j - 1) * nc + (i - 1)};
  // y partner: the cell of the next row is in this workgroup
  const bool y_lds = j < nc && (int)threadIdx.x + nc < (int)blockDim.x;
  // a high face is evaluated here: box edge, or no partner to take it from
  bool need_hi[3];
  need_hi[0] = i == nc || !SHFL;
  need_hi[1] = !y_lds;
  need_hi[2] = true;

  // (1) loads
  double L[3][5], Em[3], Ep[3], ex_lo[3], ex_hi[3];
  const double L0 = ne[c0], E0 = E[c0];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const int c = cc[d];
    L[d][0] = (c == 1) ? g2[(2 * d) * nc * nc + gq[d]] : ne[c0 - 2 * st[d]];
    L[d][1] = ne[c0 - st[d]];
    L[d][2] = L0;
    L[d][3] = ne[c0 + st[d]];
    L[d][4] = (c == nc) ? g2[(2 * d + 1) * nc * nc + gq[d]] : 0.0;
    Em[d] = E[c0 - st[d]];
    Ep[d] = need_hi[d] ? E[c0 + st[d]] : 0.0;
    if (PHI) {
      ex_lo[d] = gf[d] * (P0 - ph[c0 - st[d]]);
      ex_hi[d] = need_hi[d] ? gf[d] * (ph[c0 + st[d]] - P0) : 0.0;
    } else {
      ex_lo[d] = Ef[d * fd + fcell];
      ex_hi[d] = need_hi[d] ? Ef[d * fd + fcell + fst[d]] : 0.0;
    }
  }
  // 1/N at the low and high face of every dimension
  double ni_lo[3], ni_hi[3];
  if (Ng) {
    const double N0 = Ng[c0];
#pragma unroll
    for (int d = 0; d < 3; d++) {
      ni_lo[d] = 2 / (Ng[c0 - st[d]] + N0);
      ni_hi[d] = need_hi[d] ? 2 / (N0 + Ng[c0 + st[d]]) : A.N_inv;
    }
  } else {
#pragma unroll
    for (int d = 0; d < 3; d++) ni_lo[d] = ni_hi[d] = A.N_inv;
  }
  // (2) table rows: low face of every dimension, high face where needed
  int lo_row[3], hi_row[3];
  double lo_lf[3], hi_lf[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    lt_loc(A.td, 0.5 * (Em[d] + E0) * 1e21 * ni_lo[d], lo_row[d], lo_lf[d]);
    if (need_hi[d])
      lt_loc(A.td, 0.5 * (E0 + Ep[d]) * 1e21 * ni_hi[d], hi_row[d], hi_lf[d]);
    else
      hi_row[d] = 1, hi_lf[d] = 0.0;
  }
  const int np = A.td.n_points;
  double lo_r[3][4], hi_r[3][4];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const double *r = A.td.rc + (lo_row[d] - 1);
    lo_r[d][0] = r[0], lo_r[d][1] = r[1], lo_r[d][2] = r[np], lo_r[d][3] = r[np + 1];
    if (need_hi[d]) {
      const double *h = A.td.rc + (hi_row[d] - 1);
      hi_r[d][0] = h[0], hi_r[d][1] = h[1], hi_r[d][2] = h[np], hi_r[d][3] = h[np + 1];
    } else {
      hi_r[d][0] = hi_r[d][1] = hi_r[d][2] = hi_r[d][3] = 0.0;
    }
  }
  // (3) fluxes and CFL (face_eval / face_vd arithmetic)
  double cfl = 0.0, smax = -HUGE_VAL;
  auto finish = [&](const double rr[4], double lf, double ex, double ni,
                    double &v, double &dc) {
    double mu = lf * rr[0] + (1 - lf) * rr[1];
    const double dd = lf * rr[2] + (1 - lf) * rr[3];
    mu = mu * ni;
    dc = dd * ni;
    v = -mu * ex;
    return mu;
  };
  auto upwind = [&](double Lm2, double Lm1, double Lc, double Lp1, double ex) {
    if (-1 * ex > 0) return Lm1 + 0.5 * limiter_t<LIM>(A.lim, Lc - Lm1, Lm1 - Lm2);
    return Lc - 0.5 * limiter_t<LIM>(A.lim, Lc - Lm1, Lp1 - Lc);
  };
  double vl[3], dl[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const double u = upwind(L[d][0], L[d][1], L[d][2], L[d][3], ex_lo[d]);
    const double mu = finish(lo_r[d], lo_lf[d], ex_lo[d], ni_lo[d], vl[d], dl[d]);
    const double flux = vl[d] * u - dl[d] * idx[d] * (L[d][2] - L[d][1]);
    if (active) F[d * fd + fcell] = flux;
    smax = fmax(smax, mu * u);
    if (A.sig && active) A.sig[(size_t)(id - 1) * fsz + d * fd + fcell] = mu * u;
  }
  // x partner by lane shuffle: executed by every lane (a shuffle reading an
  // inactive lane returns 0, so never inside the divergent branch below)
  double vsh = 0, dsh = 0;
  if (SHFL) {
    vsh = __shfl_down(vl[0], 1, 64);
    dsh = __shfl_down(dl[0], 1, 64);
  }
  s_v[threadIdx.x] = vl[1];
  s_d[threadIdx.x] = dl[1];
  __syncthreads();
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const double inv_dx = idx[d];
    double vh, dh;
    if (cc[d] == nc) {
      const double u = upwind(L[d][1], L[d][2], L[d][3], L[d][4], ex_hi[d]);
      const double mu = finish(hi_r[d], hi_lf[d], ex_hi[d], ni_hi[d], vh, dh);
      const double flux = vh * u - dh * inv_dx * (L[d][3] - L[d][2]);
      if (active) F[d * fd + fcell + fst[d]] = flux;
      smax = fmax(smax, mu * u);
      if (A.sig && active) A.sig[(size_t)(id - 1) * fsz + d * fd + fcell + fst[d]] = mu * u;
    } else if (d == 0 && SHFL) {
      vh = vsh;
      dh = dsh;
    } else if (d == 1 && y_lds) {
      vh = s_v[threadIdx.x + nc];
      dh = s_d[threadIdx.x + nc];
    } else {
      finish(hi_r[d], hi_lf[d], ex_hi[d], ni_hi[d], vh, dh);
    }
    const double mv = fmax(fabs(vh), fabs(vl[d]));
    const double md = fmax(dh, dl[d]);
    cfl = cfl + (1.0 * mv * inv_dx + 2 * md * (inv_dx * inv_dx));
  }
  if (!active) cfl = smax = -HUGE_VAL;
  if (A.sig) smax = -HUGE_VAL;  // k_flux_ion folds the sum
  for (int o = 32; o > 0; o >>= 1) {
    cfl = fmax(cfl, __shfl_xor(cfl, o, 64));
    smax = fmax(smax, __shfl_xor(smax, o, 64));
  }
  __shared__ double r1[4], r2[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) r1[w] = cfl, r2[w] = smax;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < (int)(blockDim.x >> 6); q++)
      cfl = fmax(cfl, r1[q]), smax = fmax(smax, r2[q]);
    atomicMax(&red[red_shard()], dbl_to_ord(cfl));
    atomicMax(&red[RED_SHARDS + red_shard()], dbl_to_ord(smax));
  }
}

// ------------------------------------------------------------ mobile ions
// The ion part of the m_fluid flux_upwind callback (src/m_fluid.f90:207-214)
// for every face of a leaf: mu = mobility N_inv, v = sign(q) mu E_f, flux =
// v u_f with u_f reconstruct_upwind_1d's Koren-limited upwind value along
// sign(q) E_f (flux_direction, m_fluid.f90:216-232; the second ghost layer
// of each ion from its own gc2 buffer); sigma = the electrons' mu u_f (from
// k_flux_staged) + mu u_f of each ion in flux-species order, its maximum
// folded into slot 1 (the dielectric relaxation limit). One thread per
// cell: the low face of each dimension, the high face on the box's last
// cell. Same expressions as the reference's array statements, bitwise.
struct IonArgs {
  int n;
  const double *ni[AFH_MAX_IONS];   // ion densities, state s_deriv
  double *F[AFH_MAX_IONS];          // their face fluxes
  const double *gc2[AFH_MAX_IONS];  // their second ghost layers [box][6][nc][nc]
  double mob[AFH_MAX_IONS];         // mobility x N (the reference's scaled value)
  double sgn[AFH_MAX_IONS];         // flux_species_charge_sign
};

template <int LIM, bool PHI>
__global__ void __launch_bounds__(256)
    k_flux_ion(FluxArgs A, IonArgs I, const int32_t *__restrict__ ids, int nc, size_t bsz,
               size_t fsz, unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = t < nc * nc * nc;
  const int tt = active ? t : 0;
  const int id = ids[blockIdx.y];
  int i, j, k;
  cell3(tt, nc, i, j, k);
  const int ng = nc + 2, nf = nc + 1;
  const size_t ob = (size_t)(id - 1) * bsz, of = (size_t)(id - 1) * fsz;
  const double *__restrict__ Ef = A.Ef + of;
  const double *__restrict__ ph = PHI ? A.phi + ob : nullptr;
  const double *__restrict__ Ng = A.Ng ? A.Ng + ob : nullptr;
  const int c0 = (k * ng + j) * ng + i;
  const int fcell = ((k - 1) * nf + (j - 1)) * nf + (i - 1);
  const int fd = nf * nf * nf, nn = nc * nc;
  const int cc[3] = {i, j, k};
  const int st[3] = {1, ng, ng * ng};
  const int fst[3] = {1, nf, nf * nf};
  const int gq[3] = {(k - 1) * nc + (j - 1), (k - 1) * nc + (i - 1), (j - 1) * nc + (i - 1)};
  double smax = -HUGE_VAL;
  for (int d = 0; d < 3; d++) {
    const double gf = !PHI ? 0.0 : !A.meta ? A.gfac[d]
                    : A.fac == -1.0 ? -(1 / A.meta[id - 1].dr[d]) : A.fac / A.meta[id - 1].dr[d];
    for (int hi = 0; hi < 2; hi++) {
      if (hi && cc[d] != nc) continue;
      const int fi = d * fd + fcell + (hi ? fst[d] : 0);
      const int cl = c0 - st[d] + (hi ? st[d] : 0);  // cell f-1; cl + st[d] is cell f
      const double ex = PHI ? gf * (ph[cl + st[d]] - ph[cl]) : Ef[fi];
      const double ni = Ng ? 2 / (Ng[cl] + Ng[cl + st[d]]) : A.N_inv;
      double sigma = A.sig[of + fi];
      for (int n = 0; n < I.n; n++) {
        const double *L = I.ni[n] + ob;
        const double *g2 = I.gc2[n] + (size_t)(id - 1) * 6 * nn;
        const double Lm1 = L[cl], L0 = L[cl + st[d]];
        // L(f-2): second ghost layer below the box's first cell
        const double Lm2 = (!hi && cc[d] == 1) ? g2[(2 * d) * nn + gq[d]] : L[cl - st[d]];
        // L(f+1): second ghost layer above the box's last cell
        const double Lp1 = hi ? g2[(2 * d + 1) * nn + gq[d]] : L[cl + 2 * st[d]];
        double u;
        if (I.sgn[n] * ex > 0)
          u = Lm1 + 0.5 * limiter_t<LIM>(A.lim, L0 - Lm1, Lm1 - Lm2);
        else
          u = L0 - 0.5 * limiter_t<LIM>(A.lim, L0 - Lm1, Lp1 - L0);
        const double mu = I.mob[n] * ni;
        const double v = I.sgn[n] * mu * ex;
        if (active) I.F[n][of + fi] = v * u;
        sigma = sigma + mu * u;
      }
      smax = fmax(smax, sigma);
    }
  }
  if (!active) smax = -HUGE_VAL;
  for (int o = 32; o > 0; o >>= 1) smax = fmax(smax, __shfl_xor(smax, o, 64));
  __shared__ double r2[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) r2[w] = smax;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < (int)(blockDim.x >> 6); q++) smax = fmax(smax, r2[q]);
    atomicMax(&red[RED_SHARDS + red_shard()], dbl_to_ord(smax));
  }
}

// ------------------------------------------------------------ update
struct DevReaction {
  int rate_type, table_col, n_in, n_out;
  double rate_factor, c[4];
  int ix_in[4], ix_out[4], mult_out[4];
};

struct UpdArgs {
  int ns, nr, n_prev, last_step, e_index;  // e_index: species slot of the flux species
  int der_q;  // s_deriv == s_prev[der_q] (the derivative state is read once), or -1
  double w_prev[MAXPREV];
  const double *prev[MAXS][MAXPREV];
  const double *der[MAXS];
  double *out[MAXS];
  const double *E;
  const double *F;
  const DevReaction *reac;
  DevLT chem;
  DevLT td;        // transport table (mean-energy column for Te)
  int te_col;      // td_energy_eV column (1-based), 0 if absent
  double Tg;       // gas temperature
  double inv_N;
  double dt;
  double dt_dr[3];  // dt / dr per dimension of this level
  // all leaf levels in one launch: dt / dr from the box's meta record
  const afh_box_meta *meta;
  double dt_chemistry_nmin;
  // variable gas density (m_fluid.f90:339-348): N per cell, the gas species
  // densities gas_frac * N occupy species slots ns .. ns+ng-1 (the host
  // remaps the reactions' species indices, gas first in the reference)
  const double *Ng;
  int ng;
  double gas_frac[AFH_MAX_GAS_SPECIES];
  // field_set_rhs of the output state folded into the update (or null):
  // rhs = sum over charged species of rq[s] * n_out[s], in species order
  // (src/m_field.f90:363-401), max|rhs| into rhs_red
  double *rhs;
  double rq[MAXS];
  unsigned long long *rhs_red;
  // photoionization rate (or null), added to the electron and species
  // slot photo_s after the chemistry limit (m_fluid.f90:435-440)
  const double *photo;
  int photo_s;
  // mobile ions: species slot and face flux of each (their flux divergence
  // is added as the electrons', flux_update_densities over i_cc_flux)
  int n_ion;
  int ion_s[AFH_MAX_IONS];
  const double *Fion[AFH_MAX_IONS];
  // set_box_mask's electrode part (src/m_fluid.f90:469-483), or null: a cell
  // with mlsf <= 0 keeps the weighted sum of the previous states (no source,
  // no photoionization, no flux divergence); mstat[id - 1] = 0 for a box
  // with no other cell, which adds no chemistry limit either
  // (add_source_terms returns early, m_fluid.f90:332)
  const double *mlsf;
  const uint8_t *mstat;
};

// Register-resident species arrays indexed by runtime reaction data (the
// index is wave-uniform): direct indexing (VGPR index mode,
// s_set_gpr_idx_on), or with AFH_UPD_SELECT=1 a select over every species.
#ifndef AFH_UPD_SELECT
#define AFH_UPD_SELECT 0
#endif
template <int NS>
__device__ __forceinline__ double sel(const double (&a)[NS], int idx) {
#if AFH_UPD_SELECT
  double r = a[0];
#pragma unroll
  for (int s = 1; s < NS; s++) r = (s == idx) ? a[s] : r;
  return r;
#else
  return a[idx];
#endif
}
template <int NS>
__device__ __forceinline__ void add_at(double (&a)[NS], int idx, double v) {
#if AFH_UPD_SELECT
#pragma unroll
  for (int s = 0; s < NS; s++)
    if (s == idx) a[s] = a[s] + v;
#else
  a[idx] = a[idx] + v;
#endif
}

// get_rates for one cell and one reaction, src/m_chemistry.f90:565-650
// (operand order as there; `**2` as a product, real powers pow). Te < 0 on
// the first call of a cell: Te = electron_eV_to_K * LT_get_col(td_tbl,
// td_energy_eV, Td) is looked up once.
// the temperature-dependent forms (only compiled into the update kernels of
// reaction sets that use them: their pow / exp code raises the register
// count)
__device__ __forceinline__ double rate_slow(const UpdArgs &A, const DevReaction &R,
                                         double field, double &Te) {
  const double c0 = R.rate_factor;
  const double *c = R.c;
  const double Tg = A.Tg;
  const double kB = 1.3806503e-23, eV = 1.6022e-19;  // UC_boltzmann_const, UC_elec_volt
  const double electron_eV_to_K = 2 * eV / (3 * kB);
  if ((R.rate_type == AFH_RATE_K1 || R.rate_type == AFH_RATE_K3) && Te < 0)
    Te = electron_eV_to_K * lt_col(A.td, A.te_col, field);
  switch (R.rate_type) {
  case AFH_RATE_K1: return c0 * c[0] * pow(300 / Te, c[1]);
  case AFH_RATE_K3: {
    const double z = (kB / eV) * Te + c[1];
    return c0 * (c[0] * (z * z) - c[2]) * c[3];
  }
  case AFH_RATE_K4: return c0 * c[0] * pow(Tg / 300, c[1]) * exp(-c[2] / Tg);
  case AFH_RATE_K5: return c0 * c[0] * exp(-c[1] / Tg);
  case AFH_RATE_K6: return c0 * c[0] * pow(Tg, c[1]);
  case AFH_RATE_K7: return c0 * c[0] * pow(Tg / c[1], c[2]);
  case AFH_RATE_K8: return c0 * c[0] * pow(300 / Tg, c[1]);
  case AFH_RATE_K9: return c0 * c[0] * exp(-c[1] * Tg);
  case AFH_RATE_K10: return c0 * pow(10.0, c[0] + c[1] * (Tg - 300));
  case AFH_RATE_K11: return c0 * c[0] * pow(300 / Tg, c[1]) * exp(-c[2] / Tg);
  case AFH_RATE_K12: return c0 * c[0] * pow(Tg, c[1]) * exp(-c[2] / Tg);
  case AFH_RATE_K13: return c0 * c[0] * exp(-pow(c[1] / (c[2] + field), c[3]));
  case AFH_RATE_K14: return c0 * c[0] * exp(-pow(field / c[1], c[2]));
  default:  // AFH_RATE_K15
    return c0 * c[0] * exp(-pow(c[1] / (kB * (Tg + field / c[2])), c[3]));
  }
}

// Tabulated rates of one cell: the table location (low, lf) depends only on
// the field, so it is found once per cell (lt_loc) and every tabulated
// reaction reads its column from the two rows of a row-major copy of the
// table (one or two cache lines per cell instead of two per reaction); same
// expression as LT_get_col_at_loc, bitwise.
__device__ __forceinline__ double lt_at_rm(const DevLT &lt, int col, int low, double lf) {
  const double *r = lt.rm + (size_t)(low - 1) * lt.n_cols + (col - 1);
  return lf * r[0] + (1 - lf) * r[lt.n_cols];
}

template <bool SLOW>
__device__ __forceinline__ double rate_of(const UpdArgs &A, const DevReaction &R,
                                          double field, double &Te, int low = -1,
                                          double lf = 0.0) {
  const double c0 = R.rate_factor;
  const double *c = R.c;
  switch (R.rate_type) {
  case AFH_RATE_TABULATED_FIELD:
    return c0 * (low > 0 ? lt_at_rm(A.chem, R.table_col, low, lf)
                         : lt_col(A.chem, R.table_col, field));
  case AFH_RATE_CONSTANT: return c0 * c[0];
  case AFH_RATE_LINEAR: return c0 * c[0] * (field - c[1]);
  case AFH_RATE_EXP_V1: {
    const double z = c[1] / (c[2] + field);
    return c0 * c[0] * exp(-(z * z));
  }
  case AFH_RATE_EXP_V2: {
    const double z = field / c[1];
    return c0 * c[0] * exp(-(z * z));
  }
  default: return SLOW ? rate_slow(A, R, field, Te) : 0.0;
  }
}

// Compiled reaction networks (afh_networks.h, scripts/gen_networks.py): the
// reaction loop of get_rates / get_derivatives unrolled at compile time, so
// the rate form is a constant, not a per-reaction switch, and every species
// index is a register number, not a run-time index into the state arrays
// (the generic loop pays both per reaction and cell). The coefficients are
// still read from A.reac. Same expressions in the same order as rate_of and
// the generic loop: bitwise the same derivatives.
template <int T, bool SLOW>
__device__ __forceinline__ double rate_t(const UpdArgs &A, const DevReaction &R, double field,
                                         double &Te, int low, double lf) {
  const double c0 = R.rate_factor;
  const double *c = R.c;
  if constexpr (T == AFH_RATE_TABULATED_FIELD) {
    return c0 * (low > 0 ? lt_at_rm(A.chem, R.table_col, low, lf)
                         : lt_col(A.chem, R.table_col, field));
  } else if constexpr (T == AFH_RATE_CONSTANT) {
    return c0 * c[0];
  } else if constexpr (T == AFH_RATE_LINEAR) {
    return c0 * c[0] * (field - c[1]);
  } else if constexpr (T == AFH_RATE_EXP_V1) {
    const double z = c[1] / (c[2] + field);
    return c0 * c[0] * exp(-(z * z));
  } else if constexpr (T == AFH_RATE_EXP_V2) {
    const double z = field / c[1];
    return c0 * c[0] * exp(-(z * z));
  } else {
    static_assert(SLOW, "temperature-dependent rate form in a fast update");
    return rate_slow(A, R, field, Te);
  }
}

// a temperature-dependent rate form in network NET (afh_fluid::slow_rates)
template <class NET>
constexpr bool net_slow() {
  for (int r = 0; r < NET::NR; r++)
    if (NET::type[r] > AFH_RATE_EXP_V2) return true;
  return false;
}

// dens / der slot of 1-based reference species index ix (afh_fluid_create's
// remap: gas species after the plasma species)
template <class NET>
constexpr int net_slot(int ix) {
  return ix <= NET::NG ? NET::NS + ix - 1 : ix - NET::NG - 1;
}

template <class NET, bool SLOW, int R, int NT>
__device__ __forceinline__ void net_one(const UpdArgs &A, double field, double &Te, int clow,
                                        double clf, const double (&dens)[NT], double (&der)[NT]) {
  constexpr int NI = NET::n_in[R], NO = NET::n_out[R];
  const DevReaction &X = A.reac[R];
  double rate = rate_t<NET::type[R], SLOW>(A, X, field, Te, clow, clf);
  double prod = 1.0;
  if constexpr (NI > 0) prod = prod * dens[net_slot<NET>(NET::ix_in[R][0])];
  if constexpr (NI > 1) prod = prod * dens[net_slot<NET>(NET::ix_in[R][1])];
  if constexpr (NI > 2) prod = prod * dens[net_slot<NET>(NET::ix_in[R][2])];
  if constexpr (NI > 3) prod = prod * dens[net_slot<NET>(NET::ix_in[R][3])];
  rate = rate * prod;
  if constexpr (NI > 0) der[net_slot<NET>(NET::ix_in[R][0])] += -rate;
  if constexpr (NI > 1) der[net_slot<NET>(NET::ix_in[R][1])] += -rate;
  if constexpr (NI > 2) der[net_slot<NET>(NET::ix_in[R][2])] += -rate;
  if constexpr (NI > 3) der[net_slot<NET>(NET::ix_in[R][3])] += -rate;
  if constexpr (NO > 0) der[net_slot<NET>(NET::ix_out[R][0])] += rate * NET::mult[R][0];
  if constexpr (NO > 1) der[net_slot<NET>(NET::ix_out[R][1])] += rate * NET::mult[R][1];
  if constexpr (NO > 2) der[net_slot<NET>(NET::ix_out[R][2])] += rate * NET::mult[R][2];
  if constexpr (NO > 3) der[net_slot<NET>(NET::ix_out[R][3])] += rate * NET::mult[R][3];
}

template <class NET, bool SLOW, int NT, size_t... R>
__device__ __forceinline__ void net_all(const UpdArgs &A, double field, double &Te, int clow,
                                        double clf, const double (&dens)[NT], double (&der)[NT],
                                        std::index_sequence<R...>) {
  (net_one<NET, SLOW, (int)R, NT>(A, field, Te, clow, clf, dens, der), ...);
}

template <class NET>
struct net_nr {
  static constexpr int v = NET::NR;
};
template <>
struct net_nr<void> {
  static constexpr int v = 1;
};

// does the fluid's reaction list have network NET's structure?
template <class NET>
static bool net_matches(const afh_fluid_desc *d) {
  const bool gas = d->i_gas_dens > 0;
  if (d->n_species != NET::NS || d->n_reactions != NET::NR || gas != (NET::GAS != 0) ||
      (gas && d->n_gas_species != NET::NG))
    return false;
  for (int r = 0; r < NET::NR; r++) {
    const afh_reaction &a = d->reactions[r];
    if (a.rate_type != NET::type[r] || a.n_in != NET::n_in[r] || a.n_out != NET::n_out[r])
      return false;
    for (int q = 0; q < a.n_in; q++)
      if (a.ix_in[q] != NET::ix_in[r][q]) return false;
    for (int q = 0; q < a.n_out; q++)
      if (a.ix_out[q] != NET::ix_out[r][q] || a.mult_out[q] != NET::mult[r][q]) return false;
  }
  return true;
}

// LDS-staged plane-marching flux (NC in {16, 32, 64}): a workgroup owns TJ
// rows of a box and marches over k. Each step stages plane k of n_e (rows
// j0-2 .. j0+TJ+1, columns -1 .. NC+2, second ghost layers from gc2) and of
// |E| (rows j0-1 .. j0+TJ) in LDS, double-buffered and prefetched one plane
// ahead; the transport table (mobility, diffusion interleaved per row) lives
// in LDS for the whole march. The z stencil comes from a register window of
// the thread's own column. Every face is evaluated once (low faces; high
// faces on the box boundary); the CFL sum takes the high-face transport from
// the next lane (x), the next row through LDS (y; the tile's last row looks
// it up) and the next plane (z: the x+y part is carried one step). The
// per-cell global loads of k_flux_staged (~40 vector-memory instructions per
// cell, the texture addresser ~80 % busy) become ~12. Same expressions in the
// same operand order: bitwise identical fluxes and limits.
#ifndef AFH_FLUX_LDS_NT  // threads of a k_flux_lds workgroup (NC * rows)
#define AFH_FLUX_LDS_NT 512
#endif
template <int NC, int NTT = AFH_FLUX_LDS_NT>
struct FluxLds {
  static constexpr int TJ = NTT / NC < NC ? NTT / NC : NC;  // rows per tile
  static constexpr int NT = NC * TJ;                       // NTT
  static constexpr int NTILE = NC / TJ;
  static constexpr int RW = NC + 4;                        // n_e row: i = -1 .. NC+2
  static constexpr int NR = TJ + 4;                        // rows j0-2 .. j0+TJ+1
  static constexpr int EW = NC + 2;                        // |E| row: i = 0 .. NC+1
  static constexpr int ER = TJ + 2;                        // rows j0-1 .. j0+TJ
  static constexpr int NPE = (NR * RW + NT - 1) / NT;      // staged n_e per thread
  static constexpr int EPE = (ER * EW + NT - 1) / NT;      // staged |E| per thread
};
constexpr int FLUX_LDS_MAX_POINTS = 2048;  // transport table rows held in LDS

template <int LIM>
__device__ __forceinline__ double upwind_t(int lim, double Lm2, double Lm1,
                                           double L0, double Lp1, double ex) {
  if (-1 * ex > 0) return Lm1 + 0.5 * limiter_t<LIM>(lim, L0 - Lm1, Lm1 - Lm2);
  return L0 - 0.5 * limiter_t<LIM>(lim, L0 - Lm1, Lp1 - L0);
}

// LT_get_loc + LT_get_col for mobility and diffusion from the interleaved LDS
// table T[2 r] = mu N (row r+1), T[2 r + 1] = D N (lt_mu_dc order)
__device__ __forceinline__ void lds_mu_dc(const double *T, const DevLT &lt,
                                          double x, double &mu, double &dc) {
  int low;
  double lf;
  lt_loc(lt, x, low, lf);
  const double *r = T + 2 * (low - 1);
  mu = lf * r[0] + (1 - lf) * r[2];
  dc = lf * r[1] + (1 - lf) * r[3];
}

#ifndef AFH_FLUX_LDS_MINW
#define AFH_FLUX_LDS_MINW 4
#endif
template <int NC, int LIM, bool PHI = false>
__global__ void __launch_bounds__(AFH_FLUX_LDS_NT, AFH_FLUX_LDS_MINW)
    k_flux_lds(FluxArgs A, const double *__restrict__ tdi,
               const int32_t *__restrict__ ids, size_t bsz, size_t fsz,
               unsigned long long *red) {
  using G = FluxLds<NC>;
  constexpr int NG = NC + 2, NF = NC + 1, TJ = G::TJ, NT = G::NT, RW = G::RW,
                NR = G::NR, EW = G::EW, ER = G::ER, NPE = G::NPE, EPE = G::EPE;
  constexpr size_t SK = (size_t)NG * NG, FSK = (size_t)NF * NF;
  constexpr size_t FD = (size_t)NF * NF * NF;
  constexpr int NN = NC * NC;
  extern __shared__ double T[];  // 2 n_points (dynamic)
  __shared__ double SN[2][NR * RW], SE[2][ER * EW];
  __shared__ double sv[NT], sd[NT];
  __shared__ double r1[NT / 64], r2[NT / 64];
  const int tid = threadIdx.x;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int id = ids[wg / G::NTILE];
  const int i = tid % NC + 1;
  const int jr = tid / NC;
  const int j0 = (wg % G::NTILE) * TJ + 1, j = j0 + jr;
  const double *ne = A.ne + (size_t)(id - 1) * bsz;
  const double *E = A.E + (size_t)(id - 1) * bsz;
  const double *Ef = A.Ef + (size_t)(id - 1) * fsz;
  double *F = A.F + (size_t)(id - 1) * fsz;
  const double *g2 = A.gc2 + (size_t)(id - 1) * 6 * NN;
  const double ix = A.inv_dx[0], iy = A.inv_dx[1], iz = A.inv_dx[2];
  const double N_inv = A.N_inv;
  const int np = A.td.n_points;
  for (int e = tid; e < 2 * np; e += NT) T[e] = tdi[e];

  // staged value e of plane k: n_e (rows j0-2 .. j0+TJ+1, cols -1 .. NC+2)
  auto ne_at = [&](int k, int e) -> double {
    if (e >= NR * RW) return 0.0;
    const int jj = j0 - 2 + e / RW, ii = e % RW - 1;
    const bool jin = jj >= 0 && jj <= NC + 1, iin = ii >= 0 && ii <= NC + 1;
    if (jin && iin) return ne[((size_t)k * NG + jj) * NG + ii];
    if (jin && jj >= 1 && jj <= NC) {  // x second ghost layer
      if (ii == -1) return g2[0 * NN + (k - 1) * NC + (jj - 1)];
      if (ii == NC + 2) return g2[1 * NN + (k - 1) * NC + (jj - 1)];
    }
    if (iin && ii >= 1 && ii <= NC) {  // y second ghost layer
      if (jj == -1) return g2[2 * NN + (k - 1) * NC + (ii - 1)];
      if (jj == NC + 2) return g2[3 * NN + (k - 1) * NC + (ii - 1)];
    }
    return 0.0;
  };
  auto e_at = [&](int k, int e) -> double {
    if (e >= ER * EW) return 0.0;
    return E[((size_t)k * NG + (j0 - 1 + e / EW)) * NG + e % EW];
  };
  // own column (i, j): n_e window k-2 .. k+1 and |E| at k-1, k+1
  const size_t cc = (size_t)j * NG + i;
  const size_t fcol = (size_t)(j - 1) * NF + (i - 1);
  const int gz = (j - 1) * NC + (i - 1);
  double zm2 = g2[4 * NN + gz], zm1 = ne[cc], zp1 = ne[2 * SK + cc];
  double em1 = E[cc];
  // plane 1 into LDS buffer 1
#pragma unroll
  for (int q = 0; q < NPE; q++) {
    const int e = tid + NT * q;
    if (e < NR * RW) SN[1][e] = ne_at(1, e);
  }
#pragma unroll
  for (int q = 0; q < EPE; q++) {
    const int e = tid + NT * q;
    if (e < ER * EW) SE[1][e] = e_at(1, e);
  }
  // face fields of plane 1 (PHI: from the potential, k_gradient_t's
  // expressions; pk = phi of the own cell in the current plane)
  const double *ph = PHI ? A.phi + (size_t)(id - 1) * bsz : nullptr;
  const double gfx = A.gfac[0], gfy = A.gfac[1], gfz = A.gfac[2];
  double exl, eyl, ezl, exh, eyh, pk = 0.0;
  if (PHI) {
    const size_t c1 = SK + cc;
    pk = ph[c1];
    exl = gfx * (pk - ph[c1 - 1]);
    eyl = gfy * (pk - ph[c1 - NG]);
    ezl = gfz * (pk - ph[cc]);
    exh = i == NC ? gfx * (ph[c1 + 1] - pk) : 0.0;
    eyh = (jr == TJ - 1) ? gfy * (ph[c1 + NG] - pk) : 0.0;
  } else {
    exl = Ef[fcol], eyl = Ef[FD + fcol], ezl = Ef[2 * FD + fcol];
    exh = i == NC ? Ef[fcol + 1] : 0.0;
    eyh = (jr == TJ - 1) ? Ef[FD + fcol + NF] : 0.0;
  }
  __syncthreads();

  // LDS indices of the own cell in the staged planes
  const int cn = (jr + 2) * RW + (i + 1);  // n_e
  const int ce = (jr + 1) * EW + i;        // |E|
  double cfl_xy = 0, vz_lo = 0, dz_lo = 0;
  double cmax = -HUGE_VAL, smax = -HUGE_VAL;

  for (int k = 1; k <= NC; k++) {
    const double *N0 = SN[k & 1], *E0p = SE[k & 1];
    // prefetch plane k+1 (staging) and the own column / faces of step k+1
    double pn[NPE], pe[EPE];
    const bool more = k < NC;
#pragma unroll
    for (int q = 0; q < NPE; q++) pn[q] = more ? ne_at(k + 1, tid + NT * q) : 0.0;
#pragma unroll
    for (int q = 0; q < EPE; q++) pe[q] = more ? e_at(k + 1, tid + NT * q) : 0.0;
    const size_t fbn = (size_t)k * FSK + fcol;  // faces of plane k+1
    const double zp2 = k + 2 <= NC + 1 ? ne[(size_t)(k + 2) * SK + cc]
                                       : g2[5 * NN + gz];  // k = NC: 2nd layer
    const double ep1 = E[(size_t)(k + 1) * SK + cc];
    // (PHI: the potential of plane k+1 is prefetched raw -- own cell, x-1,
    // y-1, and x+1 / y+1 on the last column / row -- and the face fields
    // are formed where the window advances, below)
    double nexl = 0, neyl = 0, nezl = 0, nexh = 0, neyh = 0, npk = 0;
    double ezh;
    if (PHI) {
      const size_t cn1 = (size_t)(k + 1) * SK + cc;  // own cell, plane k+1
      ezh = k == NC ? gfz * (ph[cn1] - pk) : 0.0;
      if (more) {
        npk = ph[cn1];
        nexl = ph[cn1 - 1];
        neyl = ph[cn1 - NG];
        if (i == NC) nexh = ph[cn1 + 1];
        if (jr == TJ - 1) neyh = ph[cn1 + NG];
      }
    } else {
      ezh = k == NC ? Ef[2 * FD + (size_t)NC * FSK + fcol] : 0.0;
      if (more) {
        nexl = Ef[fbn];
        neyl = Ef[FD + fbn];
        nezl = Ef[2 * FD + fbn];
        if (i == NC) nexh = Ef[fbn + 1];
        if (jr == TJ - 1) neyh = Ef[FD + fbn + NF];
      }
    }
    const size_t fb = (size_t)(k - 1) * FSK + fcol;
    const double z0 = N0[cn], e0 = E0p[ce];
    double mu, dcv;
    // z low face of cell k
    double vz, dz;
    {
      const double u = upwind_t<LIM>(A.lim, zm2, zm1, z0, zp1, ezl);
      lds_mu_dc(T, A.td, 0.5 * (em1 + e0) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dz = dcv * N_inv;
      vz = -mu * ezl;
      st_nt<AFH_NT_FLUX>(F + (2 * FD + fb), vz * u - dz * iz * (z0 - zm1));
      smax = fmax(smax, mu * u);
    }
    if (k > 1) {
      const double mv = fmax(fabs(vz), fabs(vz_lo));
      const double md = fmax(dz, dz_lo);
      cmax = fmax(cmax, cfl_xy + (1.0 * mv * iz + 2 * md * (iz * iz)));
    }
    vz_lo = vz;
    dz_lo = dz;
    // x low face
    double vx, dx;
    {
      const double u = upwind_t<LIM>(A.lim, N0[cn - 2], N0[cn - 1], z0, N0[cn + 1], exl);
      lds_mu_dc(T, A.td, 0.5 * (E0p[ce - 1] + e0) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dx = dcv * N_inv;
      vx = -mu * exl;
      st_nt<AFH_NT_FLUX>(F + (fb), vx * u - dx * ix * (z0 - N0[cn - 1]));
      smax = fmax(smax, mu * u);
    }
    double vxh = __shfl_down(vx, 1, 64), dxh = __shfl_down(dx, 1, 64);
    if (i == NC) {
      const double u = upwind_t<LIM>(A.lim, N0[cn - 1], z0, N0[cn + 1], N0[cn + 2], exh);
      lds_mu_dc(T, A.td, 0.5 * (e0 + E0p[ce + 1]) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dxh = dcv * N_inv;
      vxh = -mu * exh;
      st_nt<AFH_NT_FLUX>(F + (fb + 1), vxh * u - dxh * ix * (N0[cn + 1] - z0));
      smax = fmax(smax, mu * u);
    }
    // y low face
    double vy, dy;
    {
      const double u = upwind_t<LIM>(A.lim, N0[cn - 2 * RW], N0[cn - RW], z0,
                                     N0[cn + RW], eyl);
      lds_mu_dc(T, A.td, 0.5 * (E0p[ce - EW] + e0) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dy = dcv * N_inv;
      vy = -mu * eyl;
      st_nt<AFH_NT_FLUX>(F + (FD + fb), vy * u - dy * iy * (z0 - N0[cn - RW]));
      smax = fmax(smax, mu * u);
    }
    sv[tid] = vy;
    sd[tid] = dy;
    __syncthreads();
    double vyh, dyh;
    if (jr + 1 < TJ) {
      vyh = sv[tid + NC];
      dyh = sd[tid + NC];
    } else if (j == NC) {
      const double u = upwind_t<LIM>(A.lim, N0[cn - RW], z0, N0[cn + RW],
                                     N0[cn + 2 * RW], eyh);
      lds_mu_dc(T, A.td, 0.5 * (e0 + E0p[ce + EW]) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dyh = dcv * N_inv;
      vyh = -mu * eyh;
      st_nt<AFH_NT_FLUX>(F + (FD + fb + NF), vyh * u - dyh * iy * (N0[cn + RW] - z0));
      smax = fmax(smax, mu * u);
    } else {
      lds_mu_dc(T, A.td, 0.5 * (e0 + E0p[ce + EW]) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dyh = dcv * N_inv;
      vyh = -mu * eyh;
    }
    {
      const double mvx = fmax(fabs(vxh), fabs(vx)), mdx = fmax(dxh, dx);
      const double mvy = fmax(fabs(vyh), fabs(vy)), mdy = fmax(dyh, dy);
      double c = 0.0;
      c = c + (1.0 * mvx * ix + 2 * mdx * (ix * ix));
      c = c + (1.0 * mvy * iy + 2 * mdy * (iy * iy));
      cfl_xy = c;
    }
    if (k == NC) {
      // z high face of the box (between NC and NC+1)
      const double u = upwind_t<LIM>(A.lim, zm1, z0, zp1, zp2, ezh);
      lds_mu_dc(T, A.td, 0.5 * (e0 + ep1) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      const double dh = dcv * N_inv, vh = -mu * ezh;
      st_nt<AFH_NT_FLUX>(F + (2 * FD + fb + FSK), vh * u - dh * iz * (zp1 - z0));
      smax = fmax(smax, mu * u);
      const double mv = fmax(fabs(vh), fabs(vz_lo));
      const double md = fmax(dh, dz_lo);
      cmax = fmax(cmax, cfl_xy + (1.0 * mv * iz + 2 * md * (iz * iz)));
    }
    // plane k+1 into the other buffer; advance the windows
    if (more) {
#pragma unroll
      for (int q = 0; q < NPE; q++) {
        const int e = tid + NT * q;
        if (e < NR * RW) SN[(k + 1) & 1][e] = pn[q];
      }
#pragma unroll
      for (int q = 0; q < EPE; q++) {
        const int e = tid + NT * q;
        if (e < ER * EW) SE[(k + 1) & 1][e] = pe[q];
      }
    }
    zm2 = zm1;
    zm1 = z0;
    zp1 = zp2;
    em1 = e0;
    if (PHI) {
      if (more) {
        exl = gfx * (npk - nexl);
        eyl = gfy * (npk - neyl);
        ezl = gfz * (npk - pk);
        exh = i == NC ? gfx * (nexh - npk) : 0.0;
        eyh = (jr == TJ - 1) ? gfy * (neyh - npk) : 0.0;
      }
      pk = npk;
    } else {
      exl = nexl, eyl = neyl, ezl = nezl, exh = nexh, eyh = neyh;
    }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) {
    cmax = fmax(cmax, __shfl_xor(cmax, o, 64));
    smax = fmax(smax, __shfl_xor(smax, o, 64));
  }
  const int lane = tid & 63, w = tid >> 6;
  if (lane == 0) r1[w] = cmax, r2[w] = smax;
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < NT / 64; q++) cmax = fmax(cmax, r1[q]), smax = fmax(smax, r2[q]);
    atomicMax(&red[red_shard()], dbl_to_ord(cmax));
    atomicMax(&red[RED_SHARDS + red_shard()], dbl_to_ord(smax));
  }
}

__constant__ int c_child_adj_nb[6][4] = {{1, 3, 5, 7}, {2, 4, 6, 8},
                                         {1, 2, 5, 6}, {3, 4, 7, 8},
                                         {1, 2, 3, 4}, {5, 6, 7, 8}};
__constant__ int c_cdix[8][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0},
                                 {0, 0, 1}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1}};

__global__ void k_consistent(double *__restrict__ F,
                             const afh_box_meta *__restrict__ meta,
                             const int32_t *__restrict__ tasks, int nc,
                             size_t fsz) {
  const int nch = nc >> 1;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 4 * nch * nch) return;
  const int task = tasks[blockIdx.y];
  const int id = task >> 3, nb = task & 7;
  const afh_box_meta &m = meta[id - 1];
  const int nb_id = m.neighbors[nb - 1];
  const int d = (nb - 1) >> 1;
  const bool low = ((nb - 1) & 1) == 0;
  const int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
  const int ic = t / (nch * nch), aa = t % nch + 1, bb = (t / nch) % nch + 1;
  const int i_ch = c_child_adj_nb[nb - 1][ic];
  const int c_id = m.children[i_ch - 1];
  const int i = low ? 1 : nc + 1, i_nb = low ? nc + 1 : 1;
  const int nf = nc + 1;
  int pc[3], p1[3], p2[3], p3[3], p4[3];
  pc[d] = i_nb;
  pc[ta] = nch * c_cdix[i_ch - 1][ta] + aa;
  pc[tb] = nch * c_cdix[i_ch - 1][tb] + bb;
  p1[d] = p2[d] = p3[d] = p4[d] = i;
  p1[ta] = 2 * aa - 1, p1[tb] = 2 * bb - 1;
  p2[ta] = 2 * aa, p2[tb] = 2 * bb - 1;
  p3[ta] = 2 * aa - 1, p3[tb] = 2 * bb;
  p4[ta] = 2 * aa, p4[tb] = 2 * bb;
  const double *fc = F + (size_t)(c_id - 1) * fsz;
  F[(size_t)(nb_id - 1) * fsz + fidx(nf, d, pc[0], pc[1], pc[2])] =
      0.25 * (fc[fidx(nf, d, p1[0], p1[1], p1[2])] +
              fc[fidx(nf, d, p2[0], p2[1], p2[2])] +
              fc[fidx(nf, d, p3[0], p3[1], p3[2])] +
              fc[fidx(nf, d, p4[0], p4[1], p4[2])]);
}

// NP: the number of previous states when known at compile time (1, 2), or
// MAXPREV (any, A.n_prev); SD: the derivative state is no previous state
// (A.der_q < 0) -- both only trim registers and dead loads
#ifndef AFH_UPD_KC  // cells per thread column of k_update (1, 2, 4)
#define AFH_UPD_KC 1
#endif
#ifndef AFH_UPD_MINW  // minimum waves per SIMD of the update kernel
#define AFH_UPD_MINW 1
#endif
template <int NS, bool SLOW, int NP = MAXPREV, bool SD = true, bool GAS = false,
          class NET = void>
__global__ void __launch_bounds__(256, AFH_UPD_MINW)
    k_update(UpdArgs A, const int32_t *__restrict__ ids, int nc, size_t bsz,
             size_t fsz, unsigned long long *red) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int id = ids[blockIdx.y];
  double cmin = 1e100, rmax = 0.0;
  // KC cells along k per thread: the z flux between two of them is loaded
  // once (the high face of cell k is the low face of cell k + 1)
  constexpr int KC = AFH_UPD_KC;
  double fz_carry = 0.0;
#pragma unroll 1
  for (int kc = 0; kc < KC; kc++)
  if (t < nc * nc * (nc / KC)) {
    int i, j, kq;
    cell3(t, nc, i, j, kq);
    const int k = (kq - 1) * KC + 1 + kc;
    const int ng = nc + 2, nf = nc + 1;
    const size_t x = (size_t)(id - 1) * bsz + (size_t)((k * ng + j) * ng + i);
    // every load first (fluxes, |E|, states), then the arithmetic
    const double *F = A.F + (size_t)(id - 1) * fsz;
    const int f0 = ((k - 1) * nf + (j - 1)) * nf + (i - 1);
    const int d3 = nf * nf * nf;
    const double fx0 = F[f0], fx1 = F[f0 + 1], fy0 = F[d3 + f0], fy1 = F[d3 + f0 + nf],
                 fz0 = kc ? fz_carry : F[2 * d3 + f0], fz1 = F[2 * d3 + f0 + nf * nf];
    fz_carry = fz1;
    const double ev = A.E[x];
    const double pho = A.photo ? A.photo[x] : 0.0;
    // set_box_mask: `where (lsf <= 0) mask = .false.` (a NaN stays true)
    const bool upd = !A.mlsf || !(A.mlsf[x] <= 0.0);
    const bool src = !A.mlsf || A.mstat[id - 1] != 0;
    const int n_prev = NP == MAXPREV ? A.n_prev : NP;
    const int der_q = (NP == MAXPREV || SD) ? A.der_q : -2;  // -2: see below
    double pv[NS][NP], dv[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
#pragma unroll
      for (int q = 0; q < NP; q++) pv[s][q] = q < n_prev ? A.prev[s][q][x] : 0.0;
      dv[s] = (NP != MAXPREV && !SD) || A.der_q >= 0 ? 0.0 : A.der[s][x];
    }
    (void)der_q;
    // GAS: slots NS .. NS+ng-1 hold the gas species
    constexpr int NT = GAS ? NS + AFH_MAX_GAS_SPECIES : NS;
    double y[NS], der[NT], dens[NT];
    double field;
    if (GAS) {
      const double Nc = A.Ng[x];
      field = 1e21 * (ev / Nc);
#pragma unroll
      for (int g = 0; g < NT - NS; g++) {
        const double v = g < A.ng ? A.gas_frac[g] * Nc : 0.0;
        dens[NS + g] = v > 0.0 ? v : 0.0;
        der[NS + g] = 0.0;
      }
    } else {
      field = 1e21 * A.inv_N * ev;
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
      double tmp = 0.0;
#pragma unroll
      for (int q = 0; q < NP; q++)
        if (q < n_prev) tmp = tmp + A.w_prev[q] * pv[s][q];
      y[s] = tmp;
      double v = dv[s];
#pragma unroll
      for (int q = 0; q < NP; q++)
        if (q == A.der_q) v = pv[s][q];
      dens[s] = v > 0.0 ? v : 0.0;  // max(dens, 0.0_dp)
      der[s] = 0.0;
    }
    double Te = -1.0;  // electron temperature, looked up once per cell
    int clow = -1;
    double clf = 0.0;
    if (A.chem.rm) lt_loc(A.chem, field, clow, clf);
    if constexpr (!std::is_void<NET>::value) {
      net_all<NET, SLOW>(A, field, Te, clow, clf, dens, der,
                         std::make_index_sequence<NET::NR>{});
    } else {
      for (int r = 0; r < A.nr; r++) {
        const DevReaction &R = A.reac[r];
        double rate = rate_of<SLOW>(A, R, field, Te, clow, clf);
        double prod = 1.0;
        for (int q = 0; q < R.n_in; q++) prod = prod * sel(dens, R.ix_in[q] - 1);
        rate = rate * prod;
        for (int q = 0; q < R.n_in; q++) add_at(der, R.ix_in[q] - 1, -rate);
        for (int q = 0; q < R.n_out; q++)
          add_at(der, R.ix_out[q] - 1, rate * R.mult_out[q]);
      }
    }
    if (A.last_step && src) {
      const double eps = 1e-100;
#pragma unroll
      for (int s = 0; s < NT; s++) {
        if (s >= NS + (GAS ? A.ng : 0)) continue;
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
    if (A.photo) {
      add_at(der, A.e_index, pho);
      add_at(der, A.photo_s, pho);
    }
    if (upd) {
#pragma unroll
      for (int s = 0; s < NS; s++) y[s] = y[s] + A.dt * der[s];
    }
    double dtr[3];
#pragma unroll
    for (int d = 0; d < 3; d++) dtr[d] = A.meta ? A.dt / A.meta[id - 1].dr[d] : A.dt_dr[d];
    const double div = dtr[0] * (fx0 - fx1);
    const double dvy = dtr[1] * (fy0 - fy1);
    const double dvz = dtr[2] * (fz0 - fz1);
#pragma unroll
    for (int s = 0; s < NS; s++)
      if (s == A.e_index && upd) y[s] = y[s] + div + dvy + dvz;
    for (int n = 0; n < A.n_ion && upd; n++) {
      const double *G = A.Fion[n] + (size_t)(id - 1) * fsz;
      const double gx0 = G[f0], gx1 = G[f0 + 1], gy0 = G[d3 + f0], gy1 = G[d3 + f0 + nf],
                   gz0 = G[2 * d3 + f0], gz1 = G[2 * d3 + f0 + nf * nf];
      const double ix_ = dtr[0] * (gx0 - gx1), iy_ = dtr[1] * (gy0 - gy1),
                   iz_ = dtr[2] * (gz0 - gz1);
#pragma unroll
      for (int s = 0; s < NS; s++)
        if (s == A.ion_s[n]) y[s] = y[s] + ix_ + iy_ + iz_;
    }
#pragma unroll
    for (int s = 0; s < NS; s++) st_nt<AFH_NT_UPD>(A.out[s] + x, y[s]);
    if (A.rhs) {
      double r = 0.0;
#pragma unroll
      for (int s = 0; s < NS; s++)
        if (A.rq[s] != 0.0) r = r + A.rq[s] * y[s];
      st_nt<AFH_NT_UPD>(A.rhs + x, r);
      rmax = fmax(rmax, fabs(r));
    }
  }
  if (A.rhs) block_max_to_shard(rmax, A.rhs_red);
  if (A.last_step) {
    for (int o = 32; o > 0; o >>= 1) cmin = fmin(cmin, __shfl_xor(cmin, o, 64));
    __shared__ double r1[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) r1[w] = cmin;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int q = 1; q < (int)(blockDim.x >> 6); q++) cmin = fmin(cmin, r1[q]);
      atomicMin(&red[red_shard()], dbl_to_ord(cmin));
    }
  }
}

// the update of a compiled network (NET::NS == NS): the variants of
// launch_update's generic dispatch
template <int NS, class NET>
static bool launch_update_net(const UpdArgs &A, afh_tree *t, const dim3 &grid,
                              const int32_t *ids, unsigned long long *red, bool slow) {
  if constexpr (NET::NS != NS) {
    return false;
  } else {
    constexpr bool SL = net_slow<NET>();
    const int nc = t->nc;
    const bool sd = A.der_q < 0;
    if (NET::GAS != (A.Ng != nullptr) || slow != SL) return false;
    if constexpr (NET::GAS) {
      hipLaunchKernelGGL((k_update<NS, SL, MAXPREV, true, true, NET>), grid, dim3(256), 0,
                         t->stream, A, ids, nc, t->bsz, t->fsz, red);
    } else {
      if (A.n_prev == 1 && !sd)
        hipLaunchKernelGGL((k_update<NS, SL, 1, false, false, NET>), grid, dim3(256), 0,
                           t->stream, A, ids, nc, t->bsz, t->fsz, red);
      else if (A.n_prev == 2 && !sd)
        hipLaunchKernelGGL((k_update<NS, SL, 2, false, false, NET>), grid, dim3(256), 0,
                           t->stream, A, ids, nc, t->bsz, t->fsz, red);
      else
        hipLaunchKernelGGL((k_update<NS, SL, MAXPREV, true, false, NET>), grid, dim3(256),
                           0, t->stream, A, ids, nc, t->bsz, t->fsz, red);
    }
    return true;
  }
}

template <int NS>
void launch_update(const UpdArgs &A, afh_tree *t, int l, int n_boxes,
                   unsigned long long *red, bool slow, int net = 0) {
  // boxes leaves.at(l) .. + n_boxes (one level, or every level from 1)
  const int nc = t->nc, n3 = nc * nc * nc;
  const dim3 grid((n3 / AFH_UPD_KC + 255) / 256, n_boxes);
  const auto *ids = t->leaves.at(l);
  const bool sd = A.der_q < 0;
  switch (net) {
#define AFH_NET_CASE(K, NET) \
  case K:                   \
    if (launch_update_net<NS, net::NET>(A, t, grid, ids, red, slow)) return; \
    break;
    AFH_NETWORKS(AFH_NET_CASE)
#undef AFH_NET_CASE
  default: break;
  }
  if (A.Ng)
    hipLaunchKernelGGL((k_update<NS, true, MAXPREV, true, true>), grid, dim3(256), 0,
                       t->stream, A, ids, nc, t->bsz, t->fsz, red);
  else if (slow && A.n_prev == 1 && !sd)
    hipLaunchKernelGGL((k_update<NS, true, 1, false>), grid, dim3(256), 0, t->stream, A,
                       ids, nc, t->bsz, t->fsz, red);
  else if (slow && A.n_prev == 2 && !sd)
    hipLaunchKernelGGL((k_update<NS, true, 2, false>), grid, dim3(256), 0, t->stream, A,
                       ids, nc, t->bsz, t->fsz, red);
  else if (slow)
    hipLaunchKernelGGL((k_update<NS, true>), grid, dim3(256), 0, t->stream, A,
                       ids, nc, t->bsz, t->fsz, red);
  else if (A.n_prev == 1 && !sd)
    hipLaunchKernelGGL((k_update<NS, false, 1, false>), grid, dim3(256), 0,
                       t->stream, A, ids, nc, t->bsz, t->fsz, red);
  else if (A.n_prev == 2 && !sd)
    hipLaunchKernelGGL((k_update<NS, false, 2, false>), grid, dim3(256), 0,
                       t->stream, A, ids, nc, t->bsz, t->fsz, red);
  else
    hipLaunchKernelGGL((k_update<NS, false>), grid, dim3(256), 0, t->stream, A,
                       ids, nc, t->bsz, t->fsz, red);
}

// Fused forward-Euler species step: flux_upwind_tree + flux_update_densities
// of forward_euler (src/m_fluid.f90:56-70) when no face needs a coarse-fine
// correction (af_consistent_fluxes has no task). k_flux_lds's plane march,
// and at step k the six face fluxes of cell (i, j, k) are all in hand: x-hi
// from the next lane, y-hi from the next row through LDS (the tile's last
// row evaluates the whole face), z-hi evaluated from the register window and
// carried as z-lo of step k + 1. The cell is then advanced with k_update's
// expressions (states and |E| of the cell; the flux species' s_deriv value is
// the staged n_e), the chemistry of a compiled network (NET) or the generic
// reaction loop, and with an rhs output field_set_rhs of the new state
// (k_update's). PHI: the face fields from the potential (k_flux_lds<PHI>'s
// expressions). Face fluxes leave the kernel only with wf; the reductions are
// k_flux_lds's (CFL, sigma) and k_update's (chemistry on the last step,
// max|rhs|). Bitwise the results of k_flux_lds + k_update: same expressions,
// same operand order. The n_e and |E| of the cell's own plane stay in LDS /
// registers and the face fluxes never go through HBM: 64 B per cell fewer
// than the two kernels.
// NS: species slots (>= ns; NET::NS with a network); NP: previous states;
// SD: the derivative state is not one of them (der_q < 0); NTT: threads
#ifndef AFH_FE_NT  // threads of a k_fe_lds workgroup (NC * rows)
#define AFH_FE_NT 256
#endif
#ifndef AFH_FE_MINW  // 3 waves per SIMD: every variant fits 168 VGPRs unspilled
#define AFH_FE_MINW 3
#endif
constexpr int FE_CHEM_LDS = 2048;  // rate-table doubles staged in LDS (16 KB)
template <int NC, int LIM, int NS, int NP, bool SD, bool PHI = false, class NET = void,
          bool WF = false, int NTT = AFH_FE_NT>
__global__ void __launch_bounds__(NTT, AFH_FE_MINW)
    k_fe_lds(FluxArgs A, UpdArgs U, const double *__restrict__ tdi,
             const int32_t *__restrict__ ids, size_t bsz, size_t fsz,
             unsigned long long *red) {
  // WF: the face fluxes are stored too (store_flux); a compile-time switch,
  // so that no conditional store sits between a load and its wait
  constexpr bool wf = WF;
  using G = FluxLds<NC, NTT>;
  constexpr int NG = NC + 2, NF = NC + 1, TJ = G::TJ, NT = G::NT, RW = G::RW,
                NR = G::NR, EW = G::EW, ER = G::ER, NPE = G::NPE, EPE = G::EPE;
  // box-local offsets as 32-bit ints: scalar base + vector offset loads
  constexpr int SK = NG * NG, FSK = NF * NF, FD = NF * NF * NF;
  constexpr int NN = NC * NC;
  constexpr bool HAS_NET = !std::is_void<NET>::value;
  extern __shared__ double T[];  // 2 n_points (dynamic)
  __shared__ double SN[2][NR * RW], SE[2][ER * EW];
  __shared__ double sv[NT], sd[NT], sf[NT];
  __shared__ double r1[NT / 64], r2[NT / 64], r3[NT / 64], r4[NT / 64];
  const int tid = threadIdx.x;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int id = ids[wg / G::NTILE];
  const int i = tid % NC + 1;
  const int jr = tid / NC;
  const int j0 = (wg % G::NTILE) * TJ + 1, j = j0 + jr;
  const size_t boff = (size_t)(id - 1) * bsz;
  const double *ne = A.ne + boff;
  const double *E = A.E + boff;
  const double *Ef = A.Ef + (size_t)(id - 1) * fsz;
  const double *ph = PHI ? A.phi + boff : nullptr;
  double *F = A.F + (size_t)(id - 1) * fsz;
  const double *g2 = A.gc2 + (size_t)(id - 1) * 6 * NN;
  const double ix = A.inv_dx[0], iy = A.inv_dx[1], iz = A.inv_dx[2];
  const double gfx = A.gfac[0], gfy = A.gfac[1], gfz = A.gfac[2];
  const double N_inv = A.N_inv;
  const int np = A.td.n_points;
  const int eix = U.e_index, dq = U.der_q, ns = HAS_NET ? NS : U.ns;
  for (int e = tid; e < 2 * np; e += NT) T[e] = tdi[e];
  // the network's reaction records in LDS: per-cell reads of them from
  // global memory wait on the vector-memory counter, which drains the next
  // plane's prefetch
  constexpr int NRS = net_nr<NET>::v;
  __shared__ DevReaction sreac[NRS];
  if (HAS_NET) {
    const int nw = (int)(sizeof(DevReaction) / sizeof(int)) * NRS;
    for (int e = tid; e < nw; e += NT)
      reinterpret_cast<int *>(sreac)[e] = reinterpret_cast<const int *>(U.reac)[e];
  }
  UpdArgs Ul = U;
  if (HAS_NET) Ul.reac = sreac;
  // with a network, its row-major rate table too, after the transport
  // table in the dynamic LDS (the host runs the fused step with a network
  // only when the table fits FE_CHEM_LDS doubles): the per-cell table rows
  // come from LDS (unconditionally, so that the compiler addresses them as
  // LDS)
  if constexpr (HAS_NET) {
    double *Tc = T + 2 * np;
    const int nch = U.chem.n_points * U.chem.n_cols;
    for (int e = tid; e < nch; e += NT) Tc[e] = U.chem.rm[e];
    Ul.chem.rm = Tc;
  }

  auto ne_at = [&](int k, int e) -> double {
    if (e >= NR * RW) return 0.0;
    const int jj = j0 - 2 + e / RW, ii = e % RW - 1;
    const bool jin = jj >= 0 && jj <= NC + 1, iin = ii >= 0 && ii <= NC + 1;
    if (jin && iin) return ne[(k * NG + jj) * NG + ii];
    if (jin && jj >= 1 && jj <= NC) {
      if (ii == -1) return g2[0 * NN + (k - 1) * NC + (jj - 1)];
      if (ii == NC + 2) return g2[1 * NN + (k - 1) * NC + (jj - 1)];
    }
    if (iin && ii >= 1 && ii <= NC) {
      if (jj == -1) return g2[2 * NN + (k - 1) * NC + (ii - 1)];
      if (jj == NC + 2) return g2[3 * NN + (k - 1) * NC + (ii - 1)];
    }
    return 0.0;
  };
  auto e_at = [&](int k, int e) -> double {
    if (e >= ER * EW) return 0.0;
    return E[(k * NG + (j0 - 1 + e / EW)) * NG + e % EW];
  };
  const int cc = j * NG + i;
  const int fcol = (j - 1) * NF + (i - 1);
  const int gz = (j - 1) * NC + (i - 1);
  // own column: n_e window k-1 .. k+1 (k = 1 here)
  double zm1 = ne[cc], z0 = ne[SK + cc], zp1 = ne[2 * SK + cc];
  const double zm2 = g2[4 * NN + gz];
#pragma unroll
  for (int q = 0; q < NPE; q++) {
    const int e = tid + NT * q;
    if (e < NR * RW) SN[1][e] = ne_at(1, e);
  }
#pragma unroll
  for (int q = 0; q < EPE; q++) {
    const int e = tid + NT * q;
    if (e < ER * EW) SE[1][e] = e_at(1, e);
  }
  // face fields of plane 1 (PHI: k_flux_lds<PHI>'s expressions; pk = phi of
  // the own cell in the current plane)
  double exl, eyl, exh, eyh, pk = 0.0;
  if (PHI) {
    const int c1 = SK + cc;
    pk = ph[c1];
    exl = gfx * (pk - ph[c1 - 1]);
    eyl = gfy * (pk - ph[c1 - NG]);
    exh = i == NC ? gfx * (ph[c1 + 1] - pk) : 0.0;
    eyh = (jr == TJ - 1) ? gfy * (ph[c1 + NG] - pk) : 0.0;
  } else {
    exl = Ef[fcol], eyl = Ef[FD + fcol];
    exh = i == NC ? Ef[fcol + 1] : 0.0;
    eyh = (jr == TJ - 1) ? Ef[FD + fcol + NF] : 0.0;
  }
  double mu, dcv;
  double cmax = -HUGE_VAL, smax = -HUGE_VAL, cmin = 1e100, rmax = 0.0;
  // z low face of the box (between planes 0 and 1)
  double vz_lo, dz_lo, fz_lo;
  {
    const double ezl = PHI ? gfz * (pk - ph[cc]) : Ef[2 * FD + fcol];
    const double u = upwind_t<LIM>(A.lim, zm2, zm1, z0, zp1, ezl);
    lds_mu_dc(tdi, A.td, 0.5 * (E[cc] + E[SK + cc]) * 1e21 * N_inv, mu, dcv);
    mu = mu * N_inv;
    dz_lo = dcv * N_inv;
    vz_lo = -mu * ezl;
    fz_lo = vz_lo * u - dz_lo * iz * (z0 - zm1);
    if (wf) F[2 * FD + fcol] = fz_lo;
    smax = fmax(smax, mu * u);
  }
  __syncthreads();

  const int cn = (jr + 2) * RW + (i + 1);
  const int ce = (jr + 1) * EW + i;

  for (int k = 1; k <= NC; k++) {
    const double *N0 = SN[k & 1], *E0p = SE[k & 1];
    const bool more = k < NC;
    // z-high face inputs, then the cell's states, then next step's faces and
    // the staging of plane k+1 (vmcnt retires in issue order)
    const double zp2 = k + 2 <= NC + 1 ? ne[(k + 2) * SK + cc]
                                       : g2[5 * NN + gz];
    const double ep1 = E[(k + 1) * SK + cc];
    const int fbn = k * FSK + fcol;
    const int x = k * SK + cc;
    // the next plane's face fields (PHI: the potential of plane k+1, raw --
    // own cell, x-1, y-1, and x+1 / y+1 on the last column / row -- formed
    // where the window advances, below)
    double ezh, nexl = 0, neyl = 0, nexh = 0, neyh = 0, npk = 0;
    if (PHI) {
      const int cn1 = (k + 1) * SK + cc;  // own cell, plane k+1
      npk = ph[cn1];
      if (more) {
        nexl = ph[cn1 - 1];
        neyl = ph[cn1 - NG];
        if (i == NC) nexh = ph[cn1 + 1];
        if (jr == TJ - 1) neyh = ph[cn1 + NG];
      }
      ezh = gfz * (npk - pk);
    } else {
      ezh = Ef[2 * FD + fbn];
      if (more) {
        nexl = Ef[fbn];
        neyl = Ef[FD + fbn];
        if (i == NC) nexh = Ef[fbn + 1];
        if (jr == TJ - 1) neyh = Ef[FD + fbn + NF];
      }
    }
    // the cell's states (used at the end of the step: issued after the
    // loads the step's z-high face waits for)
    double pv[NS][NP], dv[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
#pragma unroll
      for (int q = 0; q < NP; q++)
        pv[s][q] = (s >= ns || (!SD && s == eix && q == dq)) ? 0.0
                                                              : (U.prev[s][q] + boff)[x];
      dv[s] = (!SD || s >= ns || s == eix) ? 0.0 : (U.der[s] + boff)[x];
    }
    double pn[NPE], pe[EPE];
#pragma unroll
    for (int q = 0; q < NPE; q++) pn[q] = more ? ne_at(k + 1, tid + NT * q) : 0.0;
#pragma unroll
    for (int q = 0; q < EPE; q++) pe[q] = more ? e_at(k + 1, tid + NT * q) : 0.0;

    const int fb = (k - 1) * FSK + fcol;
    const double e0 = E0p[ce];
    // x low face
    double vx, dx, fx;
    {
      const double u = upwind_t<LIM>(A.lim, N0[cn - 2], N0[cn - 1], z0, N0[cn + 1], exl);
      lds_mu_dc(T, A.td, 0.5 * (E0p[ce - 1] + e0) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dx = dcv * N_inv;
      vx = -mu * exl;
      fx = vx * u - dx * ix * (z0 - N0[cn - 1]);
      if (wf) F[fb] = fx;
      smax = fmax(smax, mu * u);
    }
    double vxh = __shfl_down(vx, 1, 64), dxh = __shfl_down(dx, 1, 64);
    double fxh = __shfl_down(fx, 1, 64);
    if (i == NC) {
      const double u = upwind_t<LIM>(A.lim, N0[cn - 1], z0, N0[cn + 1], N0[cn + 2], exh);
      lds_mu_dc(T, A.td, 0.5 * (e0 + E0p[ce + 1]) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dxh = dcv * N_inv;
      vxh = -mu * exh;
      fxh = vxh * u - dxh * ix * (N0[cn + 1] - z0);
      if (wf) F[fb + 1] = fxh;
      smax = fmax(smax, mu * u);
    }
    // y low face
    double vy, dy, fy;
    {
      const double u = upwind_t<LIM>(A.lim, N0[cn - 2 * RW], N0[cn - RW], z0,
                                     N0[cn + RW], eyl);
      lds_mu_dc(T, A.td, 0.5 * (E0p[ce - EW] + e0) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dy = dcv * N_inv;
      vy = -mu * eyl;
      fy = vy * u - dy * iy * (z0 - N0[cn - RW]);
      if (wf) F[FD + fb] = fy;
      smax = fmax(smax, mu * u);
    }
    sv[tid] = vy;
    sd[tid] = dy;
    sf[tid] = fy;
    __syncthreads();
    double vyh, dyh, fyh;
    if (jr + 1 < TJ) {
      vyh = sv[tid + NC];
      dyh = sd[tid + NC];
      fyh = sf[tid + NC];
    } else {
      // the tile's last row: the whole high face (the next tile, or the box
      // boundary, owns it; the sigma term is counted by its owner too)
      const double u = upwind_t<LIM>(A.lim, N0[cn - RW], z0, N0[cn + RW],
                                     N0[cn + 2 * RW], eyh);
      lds_mu_dc(T, A.td, 0.5 * (e0 + E0p[ce + EW]) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dyh = dcv * N_inv;
      vyh = -mu * eyh;
      fyh = vyh * u - dyh * iy * (N0[cn + RW] - z0);
      if (j == NC) {
        if (wf) F[FD + fb + NF] = fyh;
        smax = fmax(smax, mu * u);
      }
    }
    // z high face (low face of cell k+1)
    double vzh, dzh, fzh;
    {
      const double u = upwind_t<LIM>(A.lim, zm1, z0, zp1, zp2, ezh);
      lds_mu_dc(T, A.td, 0.5 * (e0 + ep1) * 1e21 * N_inv, mu, dcv);
      mu = mu * N_inv;
      dzh = dcv * N_inv;
      vzh = -mu * ezh;
      fzh = vzh * u - dzh * iz * (zp1 - z0);
      if (wf) F[2 * FD + fb + FSK] = fzh;
      smax = fmax(smax, mu * u);
    }
    {
      const double mvx = fmax(fabs(vxh), fabs(vx)), mdx = fmax(dxh, dx);
      const double mvy = fmax(fabs(vyh), fabs(vy)), mdy = fmax(dyh, dy);
      double c = 0.0;
      c = c + (1.0 * mvx * ix + 2 * mdx * (ix * ix));
      c = c + (1.0 * mvy * iy + 2 * mdy * (iy * iy));
      const double mv = fmax(fabs(vzh), fabs(vz_lo));
      const double md = fmax(dzh, dz_lo);
      cmax = fmax(cmax, c + (1.0 * mv * iz + 2 * md * (iz * iz)));
    }
    // density update of cell (i, j, k): k_update
    {
      double y[NS], der[NS], dens[NS];
#pragma unroll
      for (int s = 0; s < NS; s++) {
#pragma unroll
        for (int q = 0; q < NP; q++)
          if (!SD && s == eix && q == dq) pv[s][q] = z0;
        if (SD && s == eix) dv[s] = z0;
        double tmp = 0.0;
#pragma unroll
        for (int q = 0; q < NP; q++) tmp = tmp + U.w_prev[q] * pv[s][q];
        y[s] = tmp;
        double v = dv[s];
#pragma unroll
        for (int q = 0; q < NP; q++)
          if (!SD && q == dq) v = pv[s][q];
        dens[s] = v > 0.0 ? v : 0.0;
        der[s] = 0.0;
      }
      const double field = 1e21 * U.inv_N * e0;
      double Te = -1.0;
      int clow = -1;
      double clf = 0.0;
      if (U.chem.rm) lt_loc(U.chem, field, clow, clf);
      if constexpr (HAS_NET) {
        net_all<NET, false>(Ul, field, Te, clow, clf, dens, der,
                            std::make_index_sequence<NET::NR>{});
      } else {
        for (int r = 0; r < U.nr; r++) {
          const DevReaction &R = U.reac[r];
          double rate = rate_of<false>(U, R, field, Te, clow, clf);
          double prod = 1.0;
          for (int q = 0; q < R.n_in; q++) prod = prod * sel(dens, R.ix_in[q] - 1);
          rate = rate * prod;
          for (int q = 0; q < R.n_in; q++) add_at(der, R.ix_in[q] - 1, -rate);
          for (int q = 0; q < R.n_out; q++)
            add_at(der, R.ix_out[q] - 1, rate * R.mult_out[q]);
        }
      }
      if (U.last_step) {
        const double eps = 1e-100;
#pragma unroll
        for (int s = 0; s < NS; s++) {
          if (s >= ns) break;
          double a, b;
          if (U.dt_chemistry_nmin > 0) {
            a = dens[s] + U.dt_chemistry_nmin;
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
      for (int s = 0; s < NS; s++) y[s] = y[s] + U.dt * der[s];
      const double div = U.dt_dr[0] * (fx - fxh);
      const double dvy = U.dt_dr[1] * (fy - fyh);
      const double dvz = U.dt_dr[2] * (fz_lo - fzh);
#pragma unroll
      for (int s = 0; s < NS; s++)
        if (s == eix) y[s] = y[s] + div + dvy + dvz;
#pragma unroll
      for (int s = 0; s < NS; s++)
        if (s < ns) st_nt<AFH_NT_UPD>(U.out[s] + boff + x, y[s]);
      if (U.rhs) {
        double r = 0.0;
#pragma unroll
        for (int s = 0; s < NS; s++)
          if (s < ns && U.rq[s] != 0.0) r = r + U.rq[s] * y[s];
        st_nt<AFH_NT_UPD>(U.rhs + boff + x, r);
        rmax = fmax(rmax, fabs(r));
      }
    }
    if (more) {
#pragma unroll
      for (int q = 0; q < NPE; q++) {
        const int e = tid + NT * q;
        if (e < NR * RW) SN[(k + 1) & 1][e] = pn[q];
      }
#pragma unroll
      for (int q = 0; q < EPE; q++) {
        const int e = tid + NT * q;
        if (e < ER * EW) SE[(k + 1) & 1][e] = pe[q];
      }
    }
    zm1 = z0;
    z0 = zp1;
    zp1 = zp2;
    vz_lo = vzh, dz_lo = dzh, fz_lo = fzh;
    if (PHI) {
      if (more) {
        exl = gfx * (npk - nexl);
        eyl = gfy * (npk - neyl);
        exh = i == NC ? gfx * (nexh - npk) : 0.0;
        eyh = (jr == TJ - 1) ? gfy * (neyh - npk) : 0.0;
      }
      pk = npk;
    } else {
      exl = nexl, eyl = neyl, exh = nexh, eyh = neyh;
    }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) {
    cmax = fmax(cmax, __shfl_xor(cmax, o, 64));
    smax = fmax(smax, __shfl_xor(smax, o, 64));
    cmin = fmin(cmin, __shfl_xor(cmin, o, 64));
    rmax = fmax(rmax, __shfl_xor(rmax, o, 64));
  }
  const int lane = tid & 63, w = tid >> 6;
  if (lane == 0) r1[w] = cmax, r2[w] = smax, r3[w] = cmin, r4[w] = rmax;
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < NT / 64; q++)
      cmax = fmax(cmax, r1[q]), smax = fmax(smax, r2[q]), cmin = fmin(cmin, r3[q]),
      rmax = fmax(rmax, r4[q]);
    atomicMax(&red[red_shard()], dbl_to_ord(cmax));
    atomicMax(&red[RED_SHARDS + red_shard()], dbl_to_ord(smax));
    if (U.last_step) atomicMin(&red[2 * RED_SHARDS + red_shard()], dbl_to_ord(cmin));
    if (U.rhs) atomicMax(&U.rhs_red[red_shard()], dbl_to_ord(rmax));
  }
}


// ------------------------------------------------------------ refinement
// default_refinement (src/m_refine.f90:198-298; N per cell with a variable gas density) per
// cell, reduced per box as cell_to_ref_flags (m_af_core.f90:1095-1148):
// one workgroup per box; the box-level rules are applied per cell in the
// reference's order. Same expressions as oracle/c/afo.c refine_cell.
struct RefineArgs {
  afh_refine_desc d;
  DevLT td;
  double N;
  const double *ne, *E;
  const double *Ng;     // gas density per cell (variable N), or null
  const uint8_t *elec;  // per box, or null
};

__device__ __forceinline__ double dist_line(const double r[3], const double *r0,
                                            const double *r1) {
  double len2 = 0, frac = 0, dv[3];
#pragma unroll
  for (int d = 0; d < 3; d++) len2 = len2 + (r1[d] - r0[d]) * (r1[d] - r0[d]);
#pragma unroll
  for (int d = 0; d < 3; d++) frac = frac + (r[d] - r0[d]) * (r1[d] - r0[d]);
  if (frac <= 0.0) {
#pragma unroll
    for (int d = 0; d < 3; d++) dv[d] = r[d] - r0[d];
  } else if (frac >= len2) {
#pragma unroll
    for (int d = 0; d < 3; d++) dv[d] = r[d] - r1[d];
  } else {
#pragma unroll
    for (int d = 0; d < 3; d++) dv[d] = r[d] - (r0[d] + frac / len2 * (r1[d] - r0[d]));
  }
  return sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
}

__global__ void __launch_bounds__(256)
    k_refine_flags(RefineArgs A, const afh_box_meta *__restrict__ meta,
                   const int32_t *__restrict__ ids, int nc, size_t bsz,
                   int32_t *__restrict__ flags, uint32_t *__restrict__ masks) {
  const afh_refine_desc &p = A.d;
  const int id = ids[blockIdx.x];
  const afh_box_meta &b = meta[id - 1];
  __shared__ int s_do, s_keep;
  __shared__ unsigned s_mask;
  if (threadIdx.x == 0) s_do = 0, s_keep = 0, s_mask = 0;
  __syncthreads();
  double min_dx = b.dr[0], max_dx = b.dr[0];
  for (int d = 1; d < 3; d++) {
    if (b.dr[d] < min_dx) min_dx = b.dr[d];
    if (b.dr[d] > max_dx) max_dx = b.dr[d];
  }
  const int elec = A.elec ? A.elec[id - 1] : 0;
  const int bw = p.buffer_width, n3 = nc * nc * nc;
  double rmin[3], rmax[3];
  for (int d = 0; d < 3; d++) rmin[d] = b.r_min[d], rmax[d] = b.r_min[d] + b.dr[d] * nc;
  int any_do = 0, any_keep = 0;
  unsigned m = 0;
  for (int t = threadIdx.x; t < n3; t += blockDim.x) {
    int i, j, k;
    cell3(t, nc, i, j, k);
    const size_t x = (size_t)(id - 1) * bsz + ix3(nc + 2, i, j, k);
    const double gas_dens = A.Ng ? A.Ng[x] : A.N;  // m_refine.f90:219-223
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
    const double r[3] = {b.r_min[0] + (i - 0.5) * b.dr[0], b.r_min[1] + (j - 0.5) * b.dr[1],
                         b.r_min[2] + (k - 0.5) * b.dr[2]};
    for (int n = 0; n < p.n_seeds; n++) {
      const double dist = dist_line(r, p.seed_r0[n], p.seed_r1[n]);
      if (dist - p.seed_width[n] < 2 * max_dx && max_dx > p.init_fac * p.seed_width[n])
        f = AFH_DO_REF;
    }
    if (elec && max_dx > p.electrode_dx) f = AFH_DO_REF;
    for (int n = 0; n < p.n_regions; n++) {
      bool in = max_dx > p.region_dr[n];
      for (int d = 0; d < 3; d++)
        in = in && rmax[d] >= p.region_rmin[n][d] && rmin[d] <= p.region_rmax[n][d];
      if (in && i == nc / 2 && j == nc / 2 && k == nc / 2) f = AFH_DO_REF;
    }
    for (int n = 0; n < p.n_limits; n++) {
      bool in = max_dx < 2 * p.limit_dr[n];
      for (int d = 0; d < 3; d++)
        in = in && rmin[d] >= p.limit_rmin[n][d] && rmax[d] <= p.limit_rmax[n][d];
      if (in && f == AFH_DO_REF) f = AFH_KEEP_REF;
    }
    if (max_dx > p.max_dx) f = AFH_DO_REF;
    else if (min_dx < 2 * p.min_dx && f == AFH_DO_REF) f = AFH_KEEP_REF;
    if (f == AFH_DO_REF) {
      any_do = 1;
      if (bw > 0) {
        const bool lo[3] = {i <= bw, j <= bw, k <= bw};
        const bool hi[3] = {i > nc - bw, j > nc - bw, k > nc - bw};
        for (int dk = -1; dk <= 1; dk++)
          for (int dj = -1; dj <= 1; dj++)
            for (int di = -1; di <= 1; di++) {
              if (!di && !dj && !dk) continue;
              const int dd[3] = {di, dj, dk};
              bool in = true;
              for (int d = 0; d < 3; d++)
                in = in && (dd[d] == 0 || (dd[d] < 0 ? lo[d] : hi[d]));
              if (in) m |= 1u << ((dk + 1) * 9 + (dj + 1) * 3 + (di + 1));
            }
      }
    } else if (f == AFH_KEEP_REF) {
      any_keep = 1;
    }
  }
  if (any_do) atomicOr(&s_do, 1);
  if (any_keep) atomicOr(&s_keep, 1);
  if (m) atomicOr(&s_mask, m);
  __syncthreads();
  if (threadIdx.x == 0) {
    flags[id - 1] = s_do ? AFH_DO_REF : s_keep ? AFH_KEEP_REF : AFH_RM_REF;
    masks[id - 1] = s_mask;
  }
}
// electrode_species_bc (src/streamer.f90:578-636): one thread per interior
// cell of an electrode box. A cell with lsf < 0 is written only by its own
// thread and its electron density is read only by cells with lsf < 0 next to
// it -- which never use it (they average neighbours with lsf > 0) -- so the
// in-place update is race-free and order-independent, as in the reference.
struct ElecBcArgs {
  double *sp[MAXS];
  int ns;
  const double *lsf;
  double *ne, *ion;
  int neumann_zero;
};
__global__ void __launch_bounds__(256)
    k_electrode_bc(ElecBcArgs A, const int32_t *__restrict__ ids, int nc, size_t bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  int i, j, k;
  cell3(t, nc, i, j, k);
  const int ng = nc + 2;
  const size_t b0 = (size_t)(ids[blockIdx.y] - 1) * bsz;
  const int c = (k * ng + j) * ng + i;
  const double *lsf = A.lsf + b0;
  if (!(lsf[c] < 0)) return;
  for (int s = 0; s < A.ns; s++) A.sp[s][b0 + c] = 0.0;
  if (!A.neumann_zero) return;
  const int nb[6] = {c - 1, c + 1, c - ng, c + ng, c - ng * ng, c + ng * ng};
  int cnt = 0;
  double sum = 0.0;  // sum(dens_nb, mask=(lsf_nb > 0)), in array order
#pragma unroll
  for (int m = 0; m < 6; m++)
    if (lsf[nb[m]] > 0) {
      cnt++;
      sum = sum + A.ne[b0 + nb[m]];
    }
  if (cnt > 0) {
    const double v = sum / cnt;
    A.ne[b0 + c] = v;
    A.ion[b0 + c] = v;
  }
}
}  // namespace afh

using namespace afh;

struct afh_fluid {
  afh_tree *t = nullptr;
  afh_fluid_desc d;
  double *d_td = nullptr, *d_chem = nullptr, *d_chem_rm = nullptr;
  DevReaction *d_reac = nullptr;
  int e_index = -1;
  DevLT td, chem;
  // k_flux_lds: transport table interleaved per row (mu N, D N); unset when
  // the table does not fit LDS: k_flux_staged
  double *d_tdi = nullptr;
  bool slow_rates = false;  // a reaction with a temperature-dependent form
  // compiled network of the reaction list (afh_networks.h, 1-based; 0: the
  // generic loop); AFH_UPD_NET=0 forces the generic loop, =2 requires a match
  int net = 0;
  int32_t *d_ids = nullptr;  // box list of afh_electrode_species_bc
  int ids_cap = 0;
  // afh_fluid_set_update_mask: the level set whose cells <= 0 the update
  // leaves alone (0: none); per box whether any cell is updated
  int mask_iv = 0;
  uint8_t *d_mstat = nullptr;
  int mstat_cap = 0;
  // afh_fluid_set_rhs_output: the update also writes field_set_rhs(rhs_iv,
  // s_out); rhs_state = the state it was written for (-1: none)
  int rhs_iv = 0, rhs_state = -1;
  bool rhs_ghosts = false;
  // afh_fluid_set_field_source: the flux evaluates the face field from the
  // potential phi_iv (fac / dr * (phi_f - phi_{f-1})) instead of reading
  // f_field (0: read f_field)
  int phi_iv = 0;
  double phi_fac = -1.0;
  double ion_se_yield = 0.0;  // afh_fluid_set_ion_se_yield
  // mobile ions: second ghost layers of each ion [ion][box][6][nc][nc] and
  // the electrons' mu u per face (k_flux_staged -> k_flux_ion)
  double *d_gc2_ion = nullptr, *d_sig = nullptr;
  // write generations (afh_tree::gen) of rhs_iv and of the densities of
  // rhs_state right after the update wrote the rhs: still equal = current
  std::vector<uint64_t> rhs_snap;
  std::vector<int> rhs_vars(int s_out) const {
    std::vector<int> v{rhs_iv};
    for (int s = 0; s < d.n_species; s++) v.push_back(d.species_iv[s] + s_out);
    return v;
  }
  bool rhs_current(int s_out) const {
    if (rhs_iv <= 0 || rhs_state < 0 || rhs_state != s_out) return false;
    const std::vector<int> v = rhs_vars(s_out);
    for (size_t q = 0; q < v.size(); q++)
      if (q >= rhs_snap.size() || t->gen[v[q]] != rhs_snap[q]) return false;
    return true;
  }
  void touch_state(int s_) {
    for (int s = 0; s < d.n_species; s++) t->touch(d.species_iv[s] + s_);
  }
};

extern "C" {

int32_t afh_fluid_create(afh_tree *t, const afh_fluid_desc *d, afh_fluid **out) {
  if (!d || !out) return set_error(AFH_ERR_ARG, "afh_fluid_create: null");
  AFH_LIVE(t, "afh_fluid_create");
  if (d->n_species < 1 || d->n_species > MAXS || d->n_reactions < 0 ||
      d->n_reactions > AFH_MAX_REACTIONS)
    return set_error(AFH_ERR_ARG, "bad species/reaction count");
  if (d->td.n_points < 2 || d->td.n_cols < 2 || !d->td.rows_cols)
    return set_error(AFH_ERR_ARG, "transport table needs mobility + diffusion");
  afh_fluid *f = new afh_fluid();
  f->t = t;
  f->d = *d;
  for (int s = 0; s < d->n_species; s++) {
    if (d->species_iv[s] < 1 || d->species_iv[s] > t->nvc)
      return set_error(AFH_ERR_ARG, "bad species index");
    if (d->species_iv[s] == d->i_electron) f->e_index = s;
  }
  if (f->e_index < 0) return set_error(AFH_ERR_ARG, "electron not in species list");
  const bool gas = d->i_gas_dens > 0;
  const int ng = gas ? d->n_gas_species : 0;
  if (gas && (d->i_gas_dens > t->nvc || ng < 0 || ng > AFH_MAX_GAS_SPECIES))
    return set_error(AFH_ERR_ARG, "bad gas density variable / gas species count");
  if (!t->meth[d->i_electron].set)
    return set_error(AFH_ERR_STATE, "set cc methods for the electrons first");
  if (d->i_photo < 0 || d->i_photo > t->nvc ||
      (d->i_photo > 0 && (d->photo_species < 1 || d->photo_species > d->n_species)))
    return set_error(AFH_ERR_ARG, "bad photoionization variable / species");
  size_t ntd = (size_t)d->td.n_points * d->td.n_cols;
  size_t nch = (size_t)d->chem.n_points * d->chem.n_cols;
  AFH_HIP(hipMalloc(&f->d_td, ntd * sizeof(double)));
  AFH_HIP(hipMemcpy(f->d_td, d->td.rows_cols, ntd * sizeof(double),
                    hipMemcpyHostToDevice));
  AFH_HIP(hipMalloc(&f->d_chem, std::max<size_t>(1, nch) * sizeof(double)));
  if (nch) {
    AFH_HIP(hipMemcpy(f->d_chem, d->chem.rows_cols, nch * sizeof(double),
                      hipMemcpyHostToDevice));
    const int np = d->chem.n_points, ncol = d->chem.n_cols;
    std::vector<double> rm(nch);
    for (int c = 0; c < ncol; c++)
      for (int r = 0; r < np; r++) rm[(size_t)r * ncol + c] = d->chem.rows_cols[(size_t)c * np + r];
    AFH_HIP(hipMalloc(&f->d_chem_rm, nch * sizeof(double)));
    AFH_HIP(hipMemcpy(f->d_chem_rm, rm.data(), nch * sizeof(double), hipMemcpyHostToDevice));
  }
  if (d->n_ions < 0 || d->n_ions > AFH_MAX_IONS)
    return set_error(AFH_ERR_ARG, "bad mobile ion count");
  for (int q = 0; q < d->n_ions; q++) {
    const int sp = d->ion_species[q];
    if (sp < 1 || sp > d->n_species || sp - 1 == f->e_index || d->species_charge[sp - 1] == 0)
      return set_error(AFH_ERR_ARG, "mobile ion %d: bad species", q + 1);
    if (d->f_ion_flux[q] < 1 || d->f_ion_flux[q] > t->nvf || d->f_ion_flux[q] == d->f_flux)
      return set_error(AFH_ERR_ARG, "mobile ion %d: bad flux variable", q + 1);
    if (!t->meth[d->species_iv[sp - 1]].set)
      return set_error(AFH_ERR_STATE, "set cc methods for mobile ion %d first", q + 1);
  }
  if (d->n_ions > 0) {
    AFH_HIP(hipMalloc(&f->d_gc2_ion,
                      sizeof(double) * d->n_ions * (size_t)t->cap * 6 * t->nc * t->nc));
    AFH_HIP(hipMalloc(&f->d_sig, sizeof(double) * (size_t)t->cap * t->fsz));
  }
  // a variable gas density takes k_flux_staged (per-face 1/N); so do mobile
  // ions (k_flux_staged hands the electrons' mu u to k_flux_ion)
  if (!gas && d->n_ions == 0 && d->td.n_points <= FLUX_LDS_MAX_POINTS) {
    const int n = d->td.n_points;
    std::vector<double> ti(2 * (size_t)n);
    for (int r = 0; r < n; r++) {
      ti[2 * r] = d->td.rows_cols[r];
      ti[2 * r + 1] = d->td.rows_cols[n + r];
    }
    AFH_HIP(hipMalloc(&f->d_tdi, ti.size() * sizeof(double)));
    AFH_HIP(hipMemcpy(f->d_tdi, ti.data(), ti.size() * sizeof(double),
                      hipMemcpyHostToDevice));
  }
  std::vector<DevReaction> R(std::max(1, d->n_reactions));
  for (int r = 0; r < d->n_reactions; r++) {
    const afh_reaction &a = d->reactions[r];
    DevReaction &b = R[r];
    if (a.rate_type < AFH_RATE_TABULATED_FIELD || a.rate_type > AFH_RATE_K15 ||
        a.rate_type == 7)
      return set_error(AFH_ERR_UNSUPPORTED, "reaction rate type %d", a.rate_type);
    if (a.rate_type > AFH_RATE_EXP_V2) f->slow_rates = true;
    if ((a.rate_type == AFH_RATE_K1 || a.rate_type == AFH_RATE_K3) &&
        (d->td_energy_col < 1 || d->td_energy_col > d->td.n_cols))
      return set_error(AFH_ERR_ARG, "rate type %d needs the td mean-energy column",
                       a.rate_type);
    if (a.n_in < 0 || a.n_in > 4 || a.n_out < 0 || a.n_out > 4)
      return set_error(AFH_ERR_ARG, "reaction species count");
    b.rate_type = a.rate_type;
    b.table_col = a.table_col;
    b.n_in = a.n_in;
    b.n_out = a.n_out;
    b.rate_factor = a.rate_factor;
    // species indices: 1..ng gas, then the plasma species (the reference's
    // order); the kernels keep the plasma species first, the gas after them
    auto remap = [&](int ix) { return ix <= ng ? d->n_species + ix : ix - ng; };
    for (int q = 0; q < 4; q++) {
      b.c[q] = a.c[q];
      b.ix_in[q] = q < a.n_in ? remap(a.ix_in[q]) : a.ix_in[q];
      b.ix_out[q] = q < a.n_out ? remap(a.ix_out[q]) : a.ix_out[q];
      b.mult_out[q] = a.mult_out[q];
    }
    for (int q = 0; q < a.n_in; q++)
      if (a.ix_in[q] < 1 || a.ix_in[q] > ng + d->n_species)
        return set_error(AFH_ERR_ARG, "reaction species index");
    for (int q = 0; q < a.n_out; q++)
      if (a.ix_out[q] < 1 || a.ix_out[q] > ng + d->n_species)
        return set_error(AFH_ERR_ARG, "reaction species index");
  }
  {
    const char *env = getenv("AFH_UPD_NET");
    if (!(env && atoi(env) == 0)) {
#define AFH_NET_MATCH(K, NET) \
  if (!f->net && net_matches<net::NET>(d)) f->net = K;
      AFH_NETWORKS(AFH_NET_MATCH)
#undef AFH_NET_MATCH
    }
    // AFH_UPD_NET=2 (tests): a compiled network must match
    if (env && atoi(env) == 2 && !f->net)
      return set_error(AFH_ERR_UNSUPPORTED, "no compiled reaction network matches");
  }
  AFH_HIP(hipMalloc(&f->d_reac, sizeof(DevReaction) * R.size()));
  AFH_HIP(hipMemcpy(f->d_reac, R.data(), sizeof(DevReaction) * R.size(),
                    hipMemcpyHostToDevice));
  f->td = DevLT{d->td.n_points, d->td.n_cols, d->td.x_min, d->td.inv_fac, f->d_td};
  f->chem = DevLT{d->chem.n_points, d->chem.n_cols, d->chem.x_min,
                  d->chem.inv_fac, f->d_chem, f->d_chem_rm};
  *out = f;
  return AFH_OK;
}

int32_t afh_fluid_destroy(afh_fluid *f) {
  if (!f) return AFH_OK;
  hipStreamSynchronize(f->t->stream);
  hipFree(f->d_td);
  hipFree(f->d_chem);
  hipFree(f->d_chem_rm);
  hipFree(f->d_reac);
  hipFree(f->d_tdi);
  hipFree(f->d_ids);
  hipFree(f->d_gc2_ion);
  hipFree(f->d_sig);
  hipFree(f->d_mstat);
  delete f;
  return AFH_OK;
}

int32_t afh_electrode_species_bc(afh_fluid *f, int32_t i_lsf, int32_t i_1pos_ion,
                                 int32_t neumann_zero, int32_t n_ids,
                                 const int32_t *ids) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_electrode_species_bc: null");
  afh_tree *t = f->t;
  AFH_LIVE(t, "afh_electrode_species_bc");
  if (i_lsf < 1 || i_lsf > t->nvc || i_1pos_ion < 1 || i_1pos_ion > t->nvc ||
      n_ids < 0 || (n_ids && !ids))
    return set_error(AFH_ERR_ARG, "electrode_species_bc: bad argument");
  for (int q = 0; q < n_ids; q++)
    if (ids[q] < 1 || ids[q] > t->nb) return set_error(AFH_ERR_ARG, "bad box id");
  if (!n_ids) return AFH_OK;
  f->touch_state(0);
  t->touch(i_1pos_ion);
  if (n_ids > f->ids_cap) {
    // the previous list may still be read by a queued launch
    AFH_HIP(hipStreamSynchronize(t->stream));
    hipFree(f->d_ids);
    f->d_ids = nullptr;
    AFH_HIP(hipMalloc(&f->d_ids, sizeof(int32_t) * n_ids));
    f->ids_cap = n_ids;
  }
  // pageable source: the copy is staged before the call returns
  AFH_HIP(hipMemcpyAsync(f->d_ids, ids, sizeof(int32_t) * n_ids,
                         hipMemcpyHostToDevice, t->stream));
  ElecBcArgs A;
  A.ns = f->d.n_species;
  for (int s = 0; s < A.ns; s++) A.sp[s] = t->ccv(f->d.species_iv[s]);
  A.lsf = t->ccv(i_lsf);
  A.ne = t->ccv(f->d.i_electron);
  A.ion = t->ccv(i_1pos_ion);
  A.neumann_zero = neumann_zero ? 1 : 0;
  const int n3 = t->nc * t->nc * t->nc;
  hipLaunchKernelGGL(k_electrode_bc, dim3((n3 + 255) / 256, n_ids), dim3(256), 0,
                     t->stream, A, f->d_ids, t->nc, t->bsz);
  AFH_LAUNCH_CHECK("k_electrode_bc");
  return AFH_OK;
}

int32_t afh_fluid_set_update_mask(afh_fluid *f, int32_t i_lsf) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_set_update_mask: null");
  AFH_LIVE(f->t, "afh_fluid_set_update_mask");
  if (i_lsf < 0 || i_lsf > f->t->nvc) return set_error(AFH_ERR_ARG, "bad i_lsf");
  f->mask_iv = i_lsf;
  return AFH_OK;
}

int32_t afh_fluid_set_rhs_output(afh_fluid *f, int32_t i_rhs, int32_t ghosts) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_set_rhs_output: null");
  AFH_LIVE(f->t, "afh_fluid_set_rhs_output");
  if (i_rhs < 0 || i_rhs > f->t->nvc) return set_error(AFH_ERR_ARG, "bad i_rhs");
  f->rhs_iv = i_rhs;
  f->rhs_ghosts = ghosts != 0;
  f->rhs_state = -1;
  return AFH_OK;
}

int32_t afh_fluid_set_field_source(afh_fluid *f, int32_t i_phi, double fac) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_set_field_source: null");
  AFH_LIVE(f->t, "afh_fluid_set_field_source");
  if (i_phi < 0 || i_phi > f->t->nvc) return set_error(AFH_ERR_ARG, "bad i_phi");
  f->phi_iv = i_phi;
  f->phi_fac = fac;
  return AFH_OK;
}

int32_t afh_fluid_rhs_maxabs(afh_fluid *f, int32_t s_out, double *max_rhs) {
  if (!f || !max_rhs) return set_error(AFH_ERR_ARG, "afh_fluid_rhs_maxabs: null");
  AFH_LIVE(f->t, "afh_fluid_rhs_maxabs");
  if (!f->rhs_current(s_out))
    return set_error(AFH_ERR_STATE, "no current rhs output of state %d", s_out);
  return red_reduce_fetch(f->t, 4, 1, 0, max_rhs, f->rhs_iv);
}

int32_t afh_fluid_rhs_valid(afh_fluid *f, int32_t s_out, int32_t *valid) {
  if (!f || !valid) return set_error(AFH_ERR_ARG, "afh_fluid_rhs_valid: null");
  AFH_LIVE(f->t, "afh_fluid_rhs_valid");
  *valid = f->rhs_current(s_out) ? 1 : 0;
  return AFH_OK;
}

}  // extern "C"

// field_set_rhs; with max_out, also af_tree_maxabs_cc(i_rhs) (reduction
// slot 3, the one afh_tree_maxabs_cc uses), folded into the same pass
// -UC_elem_charge / UC_eps0 (src/m_field.f90:377-380)
static constexpr double RHS_FAC = -1.6022e-19 / 8.8541878176e-12;

static RhsArgs rhs_args(afh_fluid *f, int32_t s_in) {
  afh_tree *t = f->t;
  RhsArgs A;
  A.n = 0;
  for (int s = 0; s < f->d.n_species; s++) {
    if (f->d.species_charge[s] == 0) continue;
    A.sp[A.n] = t->ccv(f->d.species_iv[s] + s_in);
    A.q[A.n] = f->d.species_charge[s] * RHS_FAC;
    A.n++;
  }
  return A;
}

static int32_t set_rhs_impl(afh_fluid *f, int32_t i_rhs, int32_t s_in,
                            double *max_out) {
  if (!f) return set_error(AFH_ERR_ARG, "null fluid");
  afh_tree *t = f->t;
  AFH_LIVE(t, "afh_field_set_rhs");
  if (i_rhs < 1 || i_rhs > t->nvc) return set_error(AFH_ERR_ARG, "bad i_rhs");
  t->touch(i_rhs);
  const RhsArgs A = rhs_args(f, s_in);
  int32_t e;
  auto *red = reinterpret_cast<unsigned long long *>(t->scratch) + 3 * RED_SHARDS;
  if (max_out && (e = red_init(t, 3, 0.0))) return e;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    const dim3 grid((unsigned)((t->bsz + 255) / 256), n);
    if (max_out)
      hipLaunchKernelGGL(k_set_rhs<true>, grid, dim3(256), 0, t->stream,
                         t->ccv(i_rhs), A, t->leaves.at(l), t->bsz, t->ng, red);
    else
      hipLaunchKernelGGL(k_set_rhs<false>, grid, dim3(256), 0, t->stream,
                         t->ccv(i_rhs), A, t->leaves.at(l), t->bsz, t->ng, red);
    AFH_LAUNCH_CHECK("k_set_rhs");
  }
  if (!max_out) return AFH_OK;
  if ((e = red_finish(t, 3, true))) return e;
  return red_reduce_fetch(t, 3, 1, 0, max_out, i_rhs);
}

extern "C" {

int32_t afh_field_set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in) {
  return set_rhs_impl(f, i_rhs, s_in, nullptr);
}

int32_t afh_field_set_rhs_maxabs(afh_fluid *f, int32_t i_rhs, int32_t s_in,
                                 double *max_rhs) {
  if (!max_rhs) return set_error(AFH_ERR_ARG, "null max_rhs");
  return set_rhs_impl(f, i_rhs, s_in, max_rhs);
}

}  // extern "C"

template <int NC>
static void launch_flux_lds(afh_tree *t, const FluxArgs &A, const double *tdi,
                            int l, unsigned long long *red) {
  const dim3 grid(t->leaves.n(l) * FluxLds<NC>::NTILE);
  const size_t lds = 2 * sizeof(double) * A.td.n_points;
  const bool koren = A.lim == AFH_LIM_KOREN;
  auto kern = A.phi ? (koren ? k_flux_lds<NC, AFH_LIM_KOREN, true> : k_flux_lds<NC, 0, true>)
                    : (koren ? k_flux_lds<NC, AFH_LIM_KOREN> : k_flux_lds<NC, 0>);
  hipLaunchKernelGGL(kern, grid, dim3(FluxLds<NC>::NT), lds, t->stream, A, tdi,
                     t->leaves.at(l), t->bsz, t->fsz, red);
}

// flux_upwind_tree before the face loop (m_af_flux_schemes.f90:666-720):
// af_restrict_ref_boundary, then two ghost layers of the flux species
static int32_t flux_prelude(afh_fluid *f, int iv, double *gc2) {
  afh_tree *t = f->t;
  const int nc = t->nc;
  int32_t e;
  // af_restrict_ref_boundary: only leaves are restricted and their parents
  // are no leaves, so the levels are independent -- one launch over the
  // refinement-boundary leaves of levels 2.. (contiguous in the level list);
  // per level with the sharding hook, which exchanges after each
  if (!t->hook && t->nlvl >= 2) {
    if ((e = restrict_boxes(t, t->refb.at(2), t->refb.off[t->nlvl] - t->refb.off[1], iv)))
      return e;
  } else {
    for (int l = t->nlvl; l >= 2; l--) {
      if ((e = restrict_boxes(t, t->refb.at(l), t->refb.n(l), iv)) ||
          (t->hook && (e = call_hook(t, AFH_HOOK_RESTRICT, l, iv))))
        return e;
    }
  }
  // two ghost layers, level by level (coarse write-back before fine reads)
  for (int l = 1; l <= t->nlvl; l++) {
    // (a level without leaves anywhere is read only as the coarse side of
    // the next level's refinement boundaries: no exchange when there are
    // none)
    if ((t->lvl_leaves_total[l - 1] > 0 || t->lvl_rb_coarse[l - 1]) &&
        (e = call_hook(t, AFH_HOOK_HALO, l, iv)))
      return e;
    const int n = t->leaves.n(l);
    if (n) {
      const int b2 = fit_blk(nc * nc);
      hipLaunchKernelGGL(k_gc2, dim3((nc * nc + b2 - 1) / b2, 6, n), dim3(b2),
                         0, t->stream, t->ccv(iv), gc2, t->d_boxes,
                         t->leaves.at(l), nc, t->bsz, t->gc_args(iv));
      AFH_LAUNCH_CHECK("k_gc2");
    }
    // k_gc2 wrote the first ghost layer back into the boxes (coarse data of
    // the next level's refinement boundaries)
    if (t->lvl_rb_coarse[l - 1] && (e = call_hook(t, AFH_HOOK_RIMS, l, iv)))
      return e;
  }
  return AFH_OK;
}

static FluxArgs flux_args(afh_fluid *f, int iv) {
  afh_tree *t = f->t;
  FluxArgs A;
  A.ne = t->ccv(iv);
  A.E = t->ccv(f->d.i_efld);
  A.Ef = t->fcv(f->d.f_field);
  A.phi = f->phi_iv > 0 ? t->ccv(f->phi_iv) : nullptr;
  A.fac = f->phi_fac;
  A.sig = f->d.n_ions > 0 ? f->d_sig : nullptr;
  A.F = t->fcv(f->d.f_flux);
  A.gc2 = t->gc2;
  A.td = f->td;
  A.N_inv = 1 / f->d.gas_number_density;
  A.Ng = f->d.i_gas_dens > 0 ? t->ccv(f->d.i_gas_dens) : nullptr;
  A.lim = f->d.limiter;
  A.meta = nullptr;
  return A;
}

// flux_update_densities arguments (m_af_flux_schemes.f90:320-436); bytes =
// algorithmic HBM bytes per cell of k_update
static int32_t upd_args(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                        const int32_t *s_prev, const double *w_prev, int32_t s_out,
                        int32_t last_step, UpdArgs &A, double &upd_bytes) {
  if (n_prev < 1 || n_prev > MAXPREV || !s_prev || !w_prev)
    return set_error(AFH_ERR_ARG, "flux_update_densities: bad previous states");
  afh_tree *t = f->t;
  if (f->d.n_species > 16)
    return set_error(AFH_ERR_UNSUPPORTED, "more than 16 plasma species");
  auto bad = [&](int s_) {
    for (int s = 0; s < f->d.n_species; s++) {
      const int iv = f->d.species_iv[s] + s_;
      if (iv < 1 || iv > t->nvc) return true;
    }
    return false;
  };
  for (int q = 0; q < n_prev; q++)
    if (bad(s_prev[q])) return set_error(AFH_ERR_ARG, "bad previous state");
  if (bad(s_deriv) || bad(s_out)) return set_error(AFH_ERR_ARG, "bad s_deriv / s_out");
  A.ns = f->d.n_species;
  A.nr = f->d.n_reactions;
  A.n_prev = n_prev;
  A.last_step = last_step ? 1 : 0;
  A.e_index = f->e_index;
  A.der_q = -1;
  for (int q = 0; q < n_prev; q++)
    if (s_prev[q] == s_deriv && A.der_q < 0) A.der_q = q;
  for (int q = 0; q < n_prev; q++) A.w_prev[q] = w_prev[q];
  for (int s = 0; s < A.ns; s++) {
    const int iv = f->d.species_iv[s];
    for (int q = 0; q < n_prev; q++) A.prev[s][q] = t->ccv(iv + s_prev[q]);
    A.der[s] = t->ccv(iv + s_deriv);
    A.out[s] = t->ccv(iv + s_out);
  }
  A.E = t->ccv(f->d.i_efld);
  A.F = t->fcv(f->d.f_flux);
  A.reac = f->d_reac;
  A.chem = f->chem;
  A.td = f->td;
  A.te_col = f->d.td_energy_col;
  A.Tg = f->d.gas_temperature;
  A.inv_N = 1 / f->d.gas_number_density;
  A.Ng = f->d.i_gas_dens > 0 ? t->ccv(f->d.i_gas_dens) : nullptr;
  A.ng = f->d.i_gas_dens > 0 ? f->d.n_gas_species : 0;
  for (int g = 0; g < AFH_MAX_GAS_SPECIES; g++) A.gas_frac[g] = f->d.gas_fractions[g];
  A.rhs = f->rhs_iv > 0 ? t->ccv(f->rhs_iv) : nullptr;
  for (int s = 0; s < A.ns; s++) A.rq[s] = f->d.species_charge[s] * RHS_FAC;
  A.rhs_red = reinterpret_cast<unsigned long long *>(t->scratch) + 4 * RED_SHARDS;
  A.dt = dt;
  A.dt_chemistry_nmin = f->d.dt_chemistry_nmin;
  A.photo = f->d.i_photo > 0 ? t->ccv(f->d.i_photo) : nullptr;
  A.photo_s = f->d.photo_species - 1;
  A.n_ion = f->d.n_ions;
  for (int q = 0; q < AFH_MAX_IONS; q++) {
    A.ion_s[q] = q < A.n_ion ? f->d.ion_species[q] - 1 : -1;
    A.Fion[q] = q < A.n_ion ? t->fcv(f->d.f_ion_flux[q]) : nullptr;
  }
  A.meta = nullptr;
  A.mlsf = f->mask_iv > 0 ? t->ccv(f->mask_iv) : nullptr;
  A.mstat = f->d_mstat;
  // algorithmic bytes per cell: each distinct species state read once, the
  // output written once, |E| and 3 fluxes read
  int distinct = n_prev;
  for (int q = 0; q < n_prev; q++) distinct -= (s_prev[q] == s_deriv) ? 1 : 0;
  distinct += 1;
  upd_bytes = 8.0 * (A.ns * (distinct + 1) + 4 + (A.rhs ? 1 : 0) + (A.photo ? 1 : 0));
  return AFH_OK;
}

extern "C" {

}  // extern "C"

// flux_upwind_tree's device work up to the folded CFL / sigma maxima
// (reduction slots 0, 1); the caller fetches them
static int32_t flux_tree_dev(afh_fluid *f, int32_t s_deriv) {
  afh_tree *t = f->t;
  const int nc = t->nc, n3 = nc * nc * nc;
  const int iv = f->d.i_electron + s_deriv;
  if (iv < 1 || iv > t->nvc) return set_error(AFH_ERR_ARG, "bad s_deriv");
  t->touch(iv);  // ghost layers written back
  int32_t e;
  if ((e = flux_prelude(f, iv, t->gc2))) return e;
  // every flux species (af_restrict_ref_boundary and af_gc2_box over i_cc)
  const size_t g2sz = (size_t)t->cap * 6 * nc * nc;
  for (int n = 0; n < f->d.n_ions; n++) {
    const int ivn = f->d.species_iv[f->d.ion_species[n] - 1] + s_deriv;
    t->touch(ivn);
    if ((e = flux_prelude(f, ivn, f->d_gc2_ion + n * g2sz))) return e;
  }
  if ((e = red_init(t, 0, -HUGE_VAL)) || (e = red_init(t, 1, -HUGE_VAL))) return e;
  auto *red = reinterpret_cast<unsigned long long *>(t->scratch);
  FluxArgs A = flux_args(f, iv);
  const bool shfl = (64 % nc) == 0;
  const bool lds = f->d_tdi && (nc == 64 || nc == 32 || nc == 16);
  // the staged kernel takes each box's 1/dr from its meta record: every leaf
  // level in one launch (small boxes: one launch instead of one per level)
  const bool all_lvls = !lds && t->all_lvl_launch && t->leaves.off[t->nlvl] <= 65535;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = all_lvls ? (l == 1 ? t->leaves.off[t->nlvl] : 0) : t->leaves.n(l);
    if (!n) continue;
    for (int q = 0; q < 3; q++) {
      A.inv_dx[q] = 1 / t->lvl_dr[3 * (l - 1) + q];
      A.gfac[q] = A.fac / t->lvl_dr[3 * (l - 1) + q];  // fac / box%dr, bitwise
    }
    if (all_lvls) A.meta = t->d_boxes;
    prof_begin(t, AFH_PROF_FLUX);
    if (lds) {
      switch (nc) {
      case 16: launch_flux_lds<16>(t, A, f->d_tdi, l, red); break;
      case 32: launch_flux_lds<32>(t, A, f->d_tdi, l, red); break;
      default: launch_flux_lds<64>(t, A, f->d_tdi, l, red); break;
      }
    } else {
      const bool koren = A.lim == AFH_LIM_KOREN;
      auto kern =
          A.phi ? (shfl ? (koren ? k_flux_staged<true, AFH_LIM_KOREN, true>
                                 : k_flux_staged<true, 0, true>)
                        : (koren ? k_flux_staged<false, AFH_LIM_KOREN, true>
                                 : k_flux_staged<false, 0, true>))
                : (shfl ? (koren ? k_flux_staged<true, AFH_LIM_KOREN> : k_flux_staged<true, 0>)
                        : (koren ? k_flux_staged<false, AFH_LIM_KOREN> : k_flux_staged<false, 0>));
      hipLaunchKernelGGL(kern, dim3((n3 + 255) / 256, n), dim3(256), 0,
                         t->stream, A, t->leaves.at(l), nc, t->bsz, t->fsz, red);
    }
    // read n_e, |E|, 3 face fields; write 3 fluxes = 64 B/cell
    prof_end(t, AFH_PROF_FLUX, 64.0 * n3 * n);
    AFH_LAUNCH_CHECK("k_flux");
    if (f->d.n_ions > 0) {
      IonArgs I;
      I.n = f->d.n_ions;
      for (int q = 0; q < I.n; q++) {
        const int sp = f->d.ion_species[q] - 1;
        I.ni[q] = t->ccv(f->d.species_iv[sp] + s_deriv);
        I.F[q] = t->fcv(f->d.f_ion_flux[q]);
        I.gc2[q] = f->d_gc2_ion + q * g2sz;
        I.mob[q] = f->d.ion_mobility[q];
        I.sgn[q] = f->d.species_charge[sp] > 0 ? 1.0 : -1.0;
      }
      const bool koren = A.lim == AFH_LIM_KOREN;
      auto kern = A.phi ? (koren ? k_flux_ion<AFH_LIM_KOREN, true> : k_flux_ion<0, true>)
                        : (koren ? k_flux_ion<AFH_LIM_KOREN, false> : k_flux_ion<0, false>);
      hipLaunchKernelGGL(kern, dim3((n3 + 255) / 256, n), dim3(256), 0, t->stream, A, I,
                         t->leaves.at(l), nc, t->bsz, t->fsz, red);
      AFH_LAUNCH_CHECK("k_flux_ion");
    }
  }
  // af_consistent_fluxes over every flux variable (i_flux)
  const int ntask = t->cflux.off[t->nlvl];
  for (int q = -1; q < f->d.n_ions; q++) {
    const int fv = q < 0 ? f->d.f_flux : f->d.f_ion_flux[q];
    if (ntask) {
      hipLaunchKernelGGL(k_consistent, dim3((nc * nc + 255) / 256, ntask),
                         dim3(256), 0, t->stream, t->fcv(fv), t->d_boxes,
                         t->cflux.d, nc, t->fsz);
      AFH_LAUNCH_CHECK("k_consistent");
    }
    if ((e = call_hook(t, AFH_HOOK_CFLUX, 0, fv))) return e;
  }
  {
    const int slots[2] = {0, 1};
    const bool mx[2] = {true, true};
    return red_finish_n(t, 2, slots, mx);
  }
}

// dt_lim(1:2) of flux_upwind_tree from the folded maxima
static void flux_dt_limits(const double r[2], double *dt_lim) {
  const double cfl_max = r[0], sig_max = r[1];
  dt_lim[0] = 1 / cfl_max;
  dt_lim[1] = 8.8541878176e-12 / (1.6022e-19 * std::max(sig_max, 1e-100));
}

// handle_ion_se_flux (src/m_fluid.f90:584-663): one thread per face cell
// (a, b) of face blockIdx.y of leaf box ids[blockIdx.z]; physical faces only;
// the positive mobile ions in order (the host lists only those). The 3-D
// low-y case is the reference's fc(1:nc, 1:nc, 1, 2) (m_fluid.f90:639-642:
// the y faces j = 1..nc of the first z plane), as the oracle
struct IonSeArgs {
  double *fe;
  const double *fi[AFH_MAX_IONS];
  int n;
  double y;
};
__global__ void k_ion_se(IonSeArgs A, const afh_box_meta *__restrict__ meta,
                         const int32_t *__restrict__ ids, int nc, size_t fsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc) return;
  const int id = ids[blockIdx.z], nb = blockIdx.y;
  if (meta[id - 1].neighbors[nb] >= 0) return;  // not a physical boundary
  const int d = nb >> 1;
  const bool hi = nb & 1;
  const int a = t % nc + 1, b = t / nc + 1, f = hi ? nc + 1 : 1;
  int i = d == 0 ? f : a, j = d == 1 ? f : (d == 0 ? a : b), k = d == 2 ? f : b;
  if (nb == 2) j = b, k = 1;  // af_neighb_lowy as the reference indexes it
  const size_t nf = nc + 1;
  const size_t c = (size_t)(id - 1) * fsz + (size_t)d * nf * nf * nf +
                   ((size_t)(k - 1) * nf + (j - 1)) * nf + (i - 1);
  double fe = A.fe[c];
  for (int n = 0; n < A.n; n++) {
    const double v = A.fi[n][c];
    fe = fe - A.y * (hi ? (v > 0.0 ? v : 0.0) : (v < 0.0 ? v : 0.0));
  }
  A.fe[c] = fe;
}

static int32_t ion_se_dev(afh_fluid *f) {
  afh_tree *t = f->t;
  IonSeArgs A{};
  A.fe = t->fcv(f->d.f_flux);
  A.y = f->ion_se_yield;
  for (int q = 0; q < f->d.n_ions; q++)
    if (f->d.species_charge[f->d.ion_species[q] - 1] > 0) A.fi[A.n++] = t->fcv(f->d.f_ion_flux[q]);
  const int n = t->leaves.off[t->nlvl] - t->leaves.off[0], nc = t->nc;
  if (!A.n || !n) return AFH_OK;
  // every leaf of every level, at most 65535 per launch (the grid's z limit)
  const int blk = fit_blk(nc * nc);
  for (int q0 = 0; q0 < n; q0 += 65535) {
    const int nq = std::min(65535, n - q0);
    hipLaunchKernelGGL(k_ion_se, dim3((nc * nc + blk - 1) / blk, 6, nq), dim3(blk), 0,
                       t->stream, A, t->d_boxes, t->leaves.at(1) + q0, nc, t->fsz);
    AFH_LAUNCH_CHECK("k_ion_se");
  }
  return AFH_OK;
}

extern "C" {

int32_t afh_fluid_set_ion_se_yield(afh_fluid *f, double yield) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_set_ion_se_yield: null");
  AFH_LIVE(f->t, "afh_fluid_set_ion_se_yield");
  if (!(yield >= 0)) return set_error(AFH_ERR_ARG, "ion_se_yield %g", yield);
  f->ion_se_yield = yield;
  return AFH_OK;
}

int32_t afh_fluid_ion_se_flux(afh_fluid *f) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_ion_se_flux: null");
  AFH_LIVE(f->t, "afh_fluid_ion_se_flux");
  return ion_se_dev(f);
}

int32_t afh_flux_upwind_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim) {
  if (!f || !dt_lim) return set_error(AFH_ERR_ARG, "null argument");
  afh_tree *t = f->t;
  AFH_LIVE(t, "afh_flux_upwind_tree");
  const int iv = f->d.i_electron + s_deriv;
  if (iv < 1 || iv > t->nvc) return set_error(AFH_ERR_ARG, "bad s_deriv");
  int32_t e;
  double r[2];
  if ((e = flux_tree_dev(f, s_deriv)) || (e = red_reduce_fetch(t, 0, 2, 0, r))) return e;
  flux_dt_limits(r, dt_lim);
  return AFH_OK;
}

}  // extern "C"

// set_box_mask's box summary: stat[id - 1] = 1 when some interior cell of
// leaf box ids[blockIdx.x] has lsf > 0 (or NaN: `.not. (lsf <= 0)`), else 0
__global__ void k_mask_status(const double *__restrict__ lsf, const int32_t *__restrict__ ids,
                              int nc, size_t bsz, uint8_t *__restrict__ stat) {
  const int id = ids[blockIdx.x];
  const double *c = lsf + (size_t)(id - 1) * bsz;
  const int ng = nc + 2, n3 = nc * nc * nc;
  int any = 0;
  for (int q = threadIdx.x; q < n3 && !any; q += blockDim.x) {
    const int i = q % nc + 1, j = (q / nc) % nc + 1, k = q / (nc * nc) + 1;
    any = !(c[(k * ng + j) * ng + i] <= 0.0);
  }
  any = __syncthreads_or(any);
  if (threadIdx.x == 0) stat[id - 1] = any ? 1 : 0;
}

// flux_update_densities' device work; on the last step the chemistry dt
// minimum folded into reduction slot 2 for the caller to fetch
static int32_t update_dev(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                          const int32_t *s_prev, const double *w_prev, int32_t s_out,
                          int32_t last_step) {
  afh_tree *t = f->t;
  const int nc = t->nc, n3 = nc * nc * nc;
  UpdArgs A;
  double upd_bytes;
  int32_t e;
  if ((e = upd_args(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, A,
                    upd_bytes)))
    return e;
  if ((e = red_init(t, 2, 1e100))) return e;
  f->rhs_state = -1;
  if (A.rhs && (e = red_init(t, 4, 0.0))) return e;
  if (A.mlsf) {
    // the boxes' mask summary from the level set as it is now
    if (f->mstat_cap < t->cap) {
      // (a queued update may still read the old summary)
      AFH_HIP(hipStreamSynchronize(t->stream));
      hipFree(f->d_mstat);
      f->d_mstat = nullptr;
      AFH_HIP(hipMalloc(&f->d_mstat, (size_t)t->cap));
      f->mstat_cap = t->cap;
    }
    A.mstat = f->d_mstat;
    const int nl = t->leaves.off[t->nlvl];
    for (int c0 = 0; c0 < nl; c0 += 65535) {
      hipLaunchKernelGGL(k_mask_status, dim3(std::min(65535, nl - c0)), dim3(256), 0,
                         t->stream, A.mlsf, t->leaves.at(1) + c0, nc, t->bsz, f->d_mstat);
      AFH_LAUNCH_CHECK("k_mask_status");
    }
  }
  auto *red = reinterpret_cast<unsigned long long *>(t->scratch) + 2 * RED_SHARDS;
  // dt / dr from each box's meta record: every leaf level in one launch
  const bool all_lvls = t->all_lvl_launch && t->leaves.off[t->nlvl] <= 65535;
  if (all_lvls) A.meta = t->d_boxes;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = all_lvls ? (l == 1 ? t->leaves.off[t->nlvl] : 0) : t->leaves.n(l);
    if (!n) continue;
    for (int q = 0; q < 3; q++) A.dt_dr[q] = dt / t->lvl_dr[3 * (l - 1) + q];
    prof_begin(t, AFH_PROF_UPDATE);
    switch (A.ns) {
#define AFH_CASE(N) case N: launch_update<N>(A, t, l, n, red, f->slow_rates, f->net); break;
      AFH_CASE(1) AFH_CASE(2) AFH_CASE(3) AFH_CASE(4) AFH_CASE(5) AFH_CASE(6)
      AFH_CASE(7) AFH_CASE(8) AFH_CASE(9) AFH_CASE(10) AFH_CASE(11)
      AFH_CASE(12) AFH_CASE(13) AFH_CASE(14) AFH_CASE(15) AFH_CASE(16)
#undef AFH_CASE
    }
    prof_end(t, AFH_PROF_UPDATE, upd_bytes * n3 * n);
    AFH_LAUNCH_CHECK("k_update");
  }
  if (A.rhs) {
    // the ghost shell of rhs from the ghost cells of the new state (the
    // update leaves them as they are), then max|rhs| folded
    const RhsArgs R = rhs_args(f, s_out);
    for (int l = 1; l <= t->nlvl && f->rhs_ghosts; l++) {
      const int n = t->leaves.n(l);
      if (!n) continue;
      hipLaunchKernelGGL(k_rhs_shell, dim3((t->ng * t->ng + 255) / 256, 6, n),
                         dim3(256), 0, t->stream, A.rhs, R, t->leaves.at(l),
                         t->bsz, t->ng);
      AFH_LAUNCH_CHECK("k_rhs_shell");
    }
  }
  f->touch_state(s_out);
  if (A.rhs) {
    t->touch(f->rhs_iv);
    f->rhs_state = s_out;
    f->rhs_snap.clear();
    for (int v : f->rhs_vars(s_out)) f->rhs_snap.push_back(t->gen[v]);
  }
  // max|rhs| (slot 4) and the chemistry limit (slot 2) in one fold launch
  int slots[2], n_fold = 0;
  bool mx[2];
  if (A.rhs) slots[n_fold] = 4, mx[n_fold++] = true;
  if (last_step) slots[n_fold] = 2, mx[n_fold++] = false;
  return n_fold ? red_finish_n(t, n_fold, slots, mx) : AFH_OK;
}

extern "C" {

int32_t afh_flux_update_densities(afh_fluid *f, double dt, int32_t s_deriv,
                                  int32_t n_prev, const int32_t *s_prev,
                                  const double *w_prev, int32_t s_out,
                                  int32_t last_step, double *dt_lim) {
  if (!f || !dt_lim) return set_error(AFH_ERR_ARG, "afh_flux_update_densities: null");
  afh_tree *t = f->t;
  AFH_LIVE(t, "afh_flux_update_densities");
  int32_t e;
  if ((e = update_dev(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step))) return e;
  double r = 1e100;
  if (last_step) {
    if ((e = red_reduce_fetch(t, 2, 0, 1, &r))) return e;
  } else {
    AFH_HIP(hipStreamSynchronize(t->stream));
  }
  dt_lim[0] = r;
  dt_lim[1] = 1e100;
  return AFH_OK;
}

}  // extern "C"

// species slots of the fused kernel (runtime ns <= FE_MAX_SPECIES)
constexpr int FE_MAX_SPECIES = 4;

template <int NC, int NS, int NP, bool SD, bool PHI, class NET>
static void launch_fe(afh_tree *t, const FluxArgs &A, const UpdArgs &U,
                      const double *tdi, int l, unsigned long long *red, int wf) {
  using G = FluxLds<NC, AFH_FE_NT>;
  const dim3 grid(t->leaves.n(l) * G::NTILE);
  size_t lds = 2 * sizeof(double) * A.td.n_points;
  if (!std::is_void<NET>::value) lds += sizeof(double) * U.chem.n_points * U.chem.n_cols;
  if (wf)
    hipLaunchKernelGGL((k_fe_lds<NC, AFH_LIM_KOREN, NS, NP, SD, PHI, NET, true>), grid,
                       dim3(G::NT), lds, t->stream, A, U, tdi, t->leaves.at(l), t->bsz,
                       t->fsz, red);
  else
    hipLaunchKernelGGL((k_fe_lds<NC, AFH_LIM_KOREN, NS, NP, SD, PHI, NET, false>), grid,
                       dim3(G::NT), lds, t->stream, A, U, tdi, t->leaves.at(l), t->bsz,
                       t->fsz, red);
}

// the fused kernel's variants: previous states (1, 2), derivative state among
// them or not, face field from phi or stored, the compiled network of the
// 3-species air chemistry (net 1) or the generic reaction loop
template <int NC>
static void launch_fe_nc(afh_tree *t, const FluxArgs &A, const UpdArgs &U,
                         const double *tdi, int l, unsigned long long *red, int wf,
                         int net) {
  const bool sd = U.der_q < 0, phi = A.phi != nullptr;
  const int v = (U.n_prev == 2 ? 1 : 0) | (sd ? 2 : 0) | (phi ? 4 : 0);
#define AFH_FE_CASES(NSX, NETX)                                                    \
  switch (v) {                                                                     \
  case 0: launch_fe<NC, NSX, 1, false, false, NETX>(t, A, U, tdi, l, red, wf); break; \
  case 1: launch_fe<NC, NSX, 2, false, false, NETX>(t, A, U, tdi, l, red, wf); break; \
  case 2: launch_fe<NC, NSX, 1, true, false, NETX>(t, A, U, tdi, l, red, wf); break;  \
  case 3: launch_fe<NC, NSX, 2, true, false, NETX>(t, A, U, tdi, l, red, wf); break;  \
  case 4: launch_fe<NC, NSX, 1, false, true, NETX>(t, A, U, tdi, l, red, wf); break;  \
  case 5: launch_fe<NC, NSX, 2, false, true, NETX>(t, A, U, tdi, l, red, wf); break;  \
  case 6: launch_fe<NC, NSX, 1, true, true, NETX>(t, A, U, tdi, l, red, wf); break;   \
  default: launch_fe<NC, NSX, 2, true, true, NETX>(t, A, U, tdi, l, red, wf); break;  \
  }
  if (net == 1) {
    AFH_FE_CASES(net::Airsiglo::NS, net::Airsiglo)
  } else {
    AFH_FE_CASES(FE_MAX_SPECIES, void)
  }
#undef AFH_FE_CASES
}

extern "C" {

}  // extern "C"

// forward_euler's limits from the folded slots (CFL, sigma; the chemistry
// minimum on the last step) plus `n_extra` more slots, one transfer
static int32_t fetch_step(afh_fluid *f, int32_t last_step, int n_extra, const int32_t *extra,
                          double *dt_lim, double *extra_out) {
  int32_t slots[RED_SLOTS];
  double r[RED_SLOTS];
  int n = 0;
  slots[n++] = AFH_SLOT_CFL;
  slots[n++] = AFH_SLOT_SIGMA;
  if (last_step) slots[n++] = AFH_SLOT_CHEM;
  if (n_extra < 0 || n_extra > 2)
    return set_error(AFH_ERR_ARG, "afh_fluid_fetch_step: %d extra slots", n_extra);
  for (int q = 0; q < n_extra; q++) {
    if (extra[q] != AFH_SLOT_MAXRES && extra[q] != AFH_SLOT_RHS)
      return set_error(AFH_ERR_ARG, "afh_fluid_fetch_step: slot %d", extra[q]);
    slots[n++] = extra[q];
  }
  int32_t e;
  if ((e = red_fetch_slots(f->t, n, slots, r))) return e;
  flux_dt_limits(r, dt_lim);
  dt_lim[2] = last_step ? r[2] : 1e100;
  dt_lim[3] = 1e100;
  for (int q = 0; q < n_extra; q++) extra_out[q] = r[n - n_extra + q];
  return AFH_OK;
}

// forward_euler's device work: flux_upwind_tree + flux_update_densities (or
// the fused kernel), the limits folded into slots 0..2 for fetch_step
static int32_t fe_dev(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                      const int32_t *s_prev, const double *w_prev, int32_t s_out,
                      int32_t last_step, int32_t store_flux) {
  afh_tree *t = f->t;
  const int nc = t->nc, n3 = nc * nc * nc;
  const int iv = f->d.i_electron + s_deriv;
  if (iv < 1 || iv > t->nvc) return set_error(AFH_ERR_ARG, "bad s_deriv");
  UpdArgs U;
  double upd_bytes;
  int32_t e;
  if ((e = upd_args(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, U,
                    upd_bytes)))
    return e;
  // the fused kernel reads n_e(s_deriv) of neighbouring rows of the same box
  // while other workgroups write the outputs: no output may alias it or |E|
  bool alias = false;
  for (int s = 0; s < f->d.n_species; s++) {
    const int ivo = f->d.species_iv[s] + s_out;
    alias |= ivo == iv || ivo == f->d.i_efld;
  }
  // k_fe_lds moves 64 B/cell less than the two kernels (the face fluxes, n_e
  // and |E| are not written and read back). S1-64 unit steps, alternating
  // on one box (profiles/r05_fe_ab.txt): 13.03 ms with the two
  // kernels, 12.59 fused for Heun's first stage only, 12.00 fused for both
  // -- the default (AFH_FE_FUSED unset or 1) on 64^3 boxes; 2: also on
  // 16^3 / 32^3 boxes (S1: no faster); 0: never
  const char *fused_env = getenv("AFH_FE_FUSED");
  const int fe_mode = fused_env ? atoi(fused_env) : 1;
  // (a network's rate table is staged in the kernel's LDS)
  const bool net_ok =
      (f->net == 1 && f->chem.rm && f->chem.n_points * f->chem.n_cols <= FE_CHEM_LDS) ||
      (f->net == 0 && f->d.n_species <= FE_MAX_SPECIES);
  const bool policy = fe_mode == 2 || (fe_mode == 1 && nc == 64);
  const bool fused = policy && f->d_tdi &&
                     (nc == 16 || nc == 32 || nc == 64) && !t->any_cflux &&
                     !f->slow_rates && net_ok && f->d.i_gas_dens <= 0 &&
                     f->d.i_photo <= 0 && n_prev <= 2 && !alias &&
                     f->d.limiter == AFH_LIM_KOREN && f->d.n_ions == 0 && !f->mask_iv;
  if (!fused) {
    // flux and update back to back on the stream (the flux maxima are not
    // needed before the update); secondary emission from ions at the walls
    // between them (m_fluid.f90:63-67)
    if ((e = flux_tree_dev(f, s_deriv))) return e;
    if (f->d.n_ions > 0 && f->ion_se_yield > 0 && (e = ion_se_dev(f))) return e;
    return update_dev(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step);
  }
  t->touch(iv);
  f->rhs_state = -1;
  if ((e = flux_prelude(f, iv, t->gc2))) return e;
  if ((e = red_init(t, 0, -HUGE_VAL)) || (e = red_init(t, 1, -HUGE_VAL)) ||
      (e = red_init(t, 2, 1e100)) || (U.rhs && (e = red_init(t, 4, 0.0))))
    return e;
  auto *red = reinterpret_cast<unsigned long long *>(t->scratch);
  const FluxArgs A0 = flux_args(f, iv);
  // algorithmic bytes per cell: the update's states and outputs (n_e of
  // s_deriv among them, read once for flux and update) + |E| + the face
  // field's input -- the 3 stored components, or phi (PHI) -- + the 3 face
  // fluxes with store_flux. upd_bytes counts |E| + 3 fluxes (32 B): the same
  // as |E| + 3 face-field components, 16 B more than |E| + phi. S1-64:
  // 72 B/cell with one previous state, 96 with two.
  const double fe_bytes =
      upd_bytes - (f->phi_iv > 0 ? 16.0 : 0.0) + (store_flux ? 24.0 : 0.0);
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    FluxArgs A = A0;
    for (int q = 0; q < 3; q++) {
      A.inv_dx[q] = 1 / t->lvl_dr[3 * (l - 1) + q];
      A.gfac[q] = A.fac / t->lvl_dr[3 * (l - 1) + q];  // fac / box%dr, as the flux
      U.dt_dr[q] = dt / t->lvl_dr[3 * (l - 1) + q];
    }
    prof_begin(t, AFH_PROF_FE);
    switch (nc) {
    case 16: launch_fe_nc<16>(t, A, U, f->d_tdi, l, red, store_flux != 0, f->net); break;
    case 32: launch_fe_nc<32>(t, A, U, f->d_tdi, l, red, store_flux != 0, f->net); break;
    default: launch_fe_nc<64>(t, A, U, f->d_tdi, l, red, store_flux != 0, f->net); break;
    }
    prof_end(t, AFH_PROF_FE, fe_bytes * n3 * n);
    AFH_LAUNCH_CHECK("k_fe_lds");
  }
  if (U.rhs) {
    // update_dev's rhs epilogue: the ghost shell from the new state's ghost
    // cells, then the bookkeeping of the folded rhs
    const RhsArgs R = rhs_args(f, s_out);
    for (int l = 1; l <= t->nlvl && f->rhs_ghosts; l++) {
      const int n = t->leaves.n(l);
      if (!n) continue;
      hipLaunchKernelGGL(k_rhs_shell, dim3((t->ng * t->ng + 255) / 256, 6, n),
                         dim3(256), 0, t->stream, U.rhs, R, t->leaves.at(l),
                         t->bsz, t->ng);
      AFH_LAUNCH_CHECK("k_rhs_shell");
    }
  }
  f->touch_state(s_out);
  if (U.rhs) {
    t->touch(f->rhs_iv);
    f->rhs_state = s_out;
    f->rhs_snap.clear();
    for (int v : f->rhs_vars(s_out)) f->rhs_snap.push_back(t->gen[v]);
  }
  int slots[4] = {0, 1}, n_fold = 2;
  bool mx[4] = {true, true};
  if (last_step) slots[n_fold] = 2, mx[n_fold++] = false;
  if (U.rhs) slots[n_fold] = 4, mx[n_fold++] = true;
  return red_finish_n(t, n_fold, slots, mx);
}

extern "C" {

int32_t afh_fluid_forward_euler(afh_fluid *f, double dt, int32_t s_deriv,
                                int32_t n_prev, const int32_t *s_prev,
                                const double *w_prev, int32_t s_out,
                                int32_t last_step, int32_t store_flux,
                                double *dt_lim) {
  if (!f || !dt_lim) return set_error(AFH_ERR_ARG, "afh_fluid_forward_euler: null");
  AFH_LIVE(f->t, "afh_fluid_forward_euler");
  int32_t e;
  if ((e = fe_dev(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, store_flux)))
    return e;
  return fetch_step(f, last_step, 0, nullptr, dt_lim, nullptr);
}

int32_t afh_fluid_forward_euler_fold(afh_fluid *f, double dt, int32_t s_deriv,
                                     int32_t n_prev, const int32_t *s_prev,
                                     const double *w_prev, int32_t s_out,
                                     int32_t last_step, int32_t store_flux) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_fluid_forward_euler_fold: null");
  AFH_LIVE(f->t, "afh_fluid_forward_euler_fold");
  return fe_dev(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out, last_step, store_flux);
}

int32_t afh_fluid_fetch_step(afh_fluid *f, int32_t last_step, int32_t n_extra,
                             const int32_t *extra_slots, double *dt_lim, double *extra) {
  if (!f || !dt_lim || (n_extra > 0 && (!extra_slots || !extra)))
    return set_error(AFH_ERR_ARG, "afh_fluid_fetch_step: null");
  AFH_LIVE(f->t, "afh_fluid_fetch_step");
  return fetch_step(f, last_step, n_extra, extra_slots, dt_lim, extra);
}

}  // extern "C"

extern "C" {

int32_t afh_refine_flags(afh_fluid *f, const afh_refine_desc *d,
                         const uint8_t *electrode_box, int32_t *flags,
                         uint32_t *masks) {
  if (!f || !d || !flags || !masks) return set_error(AFH_ERR_ARG, "afh_refine_flags: null");
  afh_tree *t = f->t;
  AFH_LIVE(t, "afh_refine_flags");
  if (d->n_seeds > AFH_MAX_REFINE_REGIONS || d->n_regions > AFH_MAX_REFINE_REGIONS ||
      d->n_limits > AFH_MAX_REFINE_REGIONS || d->buffer_width < 0 ||
      d->buffer_width > t->nc || d->i_electron < 1 || d->i_electron > t->nvc ||
      d->i_efld < 1 || d->i_efld > t->nvc || d->td_alpha_col < 1 ||
      d->td_alpha_col > f->td.n_cols || d->td_eta_col < 1 || d->td_eta_col > f->td.n_cols)
    return set_error(AFH_ERR_ARG, "afh_refine_flags: bad descriptor");
  const int nb = t->nb, nids = t->ids.off[t->nlvl];
  int32_t *d_flags = nullptr;
  uint32_t *d_masks = nullptr;
  uint8_t *d_elec = nullptr;
  AFH_HIP(hipMalloc(&d_flags, sizeof(int32_t) * nb));
  AFH_HIP(hipMalloc(&d_masks, sizeof(uint32_t) * nb));
  AFH_HIP(hipMemsetAsync(d_flags, 0, sizeof(int32_t) * nb, t->stream));
  AFH_HIP(hipMemsetAsync(d_masks, 0, sizeof(uint32_t) * nb, t->stream));
  if (electrode_box) {
    AFH_HIP(hipMalloc(&d_elec, nb));
    AFH_HIP(hipMemcpyAsync(d_elec, electrode_box, nb, hipMemcpyHostToDevice, t->stream));
  }
  RefineArgs A;
  A.d = *d;
  A.td = f->td;
  A.N = f->d.gas_number_density;
  A.Ng = f->d.i_gas_dens > 0 ? t->ccv(f->d.i_gas_dens) : nullptr;
  A.ne = t->ccv(d->i_electron);
  A.E = t->ccv(d->i_efld);
  A.elec = d_elec;
  if (nids > 0) {
    hipLaunchKernelGGL(k_refine_flags, dim3(nids), dim3(256), 0, t->stream, A,
                       t->d_boxes, t->ids.d, t->nc, t->bsz, d_flags, d_masks);
    AFH_LAUNCH_CHECK("k_refine_flags");
  }
  AFH_HIP(hipMemcpyAsync(flags, d_flags, sizeof(int32_t) * nb, hipMemcpyDeviceToHost,
                         t->stream));
  AFH_HIP(hipMemcpyAsync(masks, d_masks, sizeof(uint32_t) * nb, hipMemcpyDeviceToHost,
                         t->stream));
  AFH_HIP(hipStreamSynchronize(t->stream));
  hipFree(d_flags), hipFree(d_masks), hipFree(d_elec);
  return AFH_OK;
}

}  // extern "C"


// photoionization_rate_from_alpha (src/m_photoi.f90:217-253): one thread per
// leaf interior cell, operand order as there
namespace afh {
__global__ void k_photoi_src(double *__restrict__ rhs, const double *__restrict__ E,
                             const double *__restrict__ ne,
                             const double *__restrict__ Ng, double N,
                             DevLT td, int alpha_col, double coeff,
                             const int32_t *__restrict__ ids, int nc, size_t bsz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc * nc * nc) return;
  int i, j, k;
  cell3(t, nc, i, j, k);
  const int ng = nc + 2;
  const size_t x = (size_t)(ids[blockIdx.y] - 1) * bsz + (size_t)((k * ng + j) * ng + i);
  const double fld = E[x];
  const double gas_dens = Ng ? Ng[x] : N;
  const double Td = fld * 1e21 / gas_dens;
  int low;
  double lf;
  lt_loc(td, Td, low, lf);
  const int np = td.n_points;
  const double *ra = td.rc + (size_t)(alpha_col - 1) * np + (low - 1);
  const double *rm = td.rc + (low - 1);
  const double alpha = lf * ra[0] + (1 - lf) * ra[1];
  const double mobility = lf * rm[0] + (1 - lf) * rm[1];
  double tmp = fld * mobility * alpha * ne[x] * coeff;
  if (tmp < 0) tmp = 0;
  rhs[x] = tmp;
}
}  // namespace afh

extern "C" {

int32_t afh_photoi_set_src(afh_fluid *f, int32_t i_rhs, int32_t alpha_col, double coeff) {
  if (!f) return set_error(AFH_ERR_ARG, "afh_photoi_set_src: null");
  afh_tree *t = f->t;
  AFH_LIVE(t, "afh_photoi_set_src");
  if (i_rhs < 1 || i_rhs > t->nvc || alpha_col < 1 || alpha_col > f->td.n_cols)
    return set_error(AFH_ERR_ARG, "afh_photoi_set_src: bad argument");
  t->touch(i_rhs);
  const int nc = t->nc, n3 = nc * nc * nc;
  const double *Ng = f->d.i_gas_dens > 0 ? t->ccv(f->d.i_gas_dens) : nullptr;
  for (int l = 1; l <= t->nlvl; l++) {
    const int n = t->leaves.n(l);
    if (!n) continue;
    hipLaunchKernelGGL(k_photoi_src, dim3((n3 + 255) / 256, n), dim3(256), 0, t->stream,
                       t->ccv(i_rhs), t->ccv(f->d.i_efld), t->ccv(f->d.i_electron), Ng,
                       f->d.gas_number_density, f->td, alpha_col, coeff,
                       t->leaves.at(l), nc, t->bsz);
    AFH_LAUNCH_CHECK("k_photoi_src");
  }
  return AFH_OK;
}

}  // extern "C"
