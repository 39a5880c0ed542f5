/* The reference's level-1 solve, HYPRE StructPFMG, restated (round 5).
 *
 * afivo hands its level-1 grid to HYPRE 2.31.0's StructPFMG
 * (afivo/src/m_coarse_solver.f90:71-100, 404-414, 427-439): one box
 * ilower = 1 .. coarse_grid_size, the 7-point stencil of the level with the
 * physical boundaries folded in (stencil_handle_boundaries, 442-491),
 * symmetric storage unless a level set is present, tolerance 1e-6, at most
 * 50 iterations, one pre- and one post-relaxation, every other setting
 * HYPRE's default: weighted Jacobi relaxation, Galerkin coarse operators,
 * relaxation skipped on the levels an isotropic problem does not need, and
 * the current phi as the initial guess (solve_coarse_grid,
 * m_af_multigrid.f90:266-291). HYPRE is not in the snapshot,
 * so this is its published algorithm (struct_ls/pfmg_setup.c,
 * pfmg_setup_interp.c, pfmg_setup_rap*.c, pfmg_solve.c, point_relax.c,
 * semi_interp.c, semi_restrict.c of HYPRE 2.31.0) written down from its
 * definition; the iterates equal HYPRE's to rounding, not bitwise.
 *
 *  Setup (this header, host code of both the HIP library and the C oracle):
 *  - per direction d the mean over the grid of -sign(a_c) (a_-d + a_+d);
 *    dxyz_d = sqrt(max_mean / mean_d) (PFMGComputeDxyz, summed in HYPRE's
 *    loop order so that exact ties stay ties);
 *  - semicoarsening, level by level, along the direction of smallest dxyz
 *    that still has more than one point (first such on a tie), dxyz of that
 *    direction doubled, down to one point; the coarse points are the even
 *    indices 2, 4, ... of the 1-based level grid (cindex 0, stride 2);
 *  - a level is relaxed when its direction was coarsened before since the
 *    last relaxed level (skip_relax = 1), the finest and the coarsest
 *    always; Jacobi weight 2 / (3 - beta / alpha), alpha = sum_d dxyz_d^-2,
 *    beta the same without the coarsening direction (2/3 when the
 *    coefficients vary by more than 10 % squared, 1 on the coarsest);
 *  - interpolation at the odd points f of the coarsening direction:
 *    w_lo = -(sum of A's entries of offset -1 there) / (sum of those of
 *    offset 0), w_hi alike, each set to 0 where A's pure -1 (+1) entry is 0;
 *    restriction its transpose; coarse operator R A P (27 points).
 *  Solve (afo.c afo_pfmg_solve, afh_mg.hip k_cs_pfmg):
 *    b.b = 0 gives x = 0; else for i = 0 .. max_iter - 1: relax level 0
 *    once; r = b - A x; stop if i > 0 and r.r / b.b < tol^2; restrict r;
 *    down the levels (relaxed: x = w b / a_c, r = b - A x; skipped: x = 0,
 *    r = b), the coarsest x = b / a_c; up: x += P x_c, relax once where
 *    relaxed; x_0 += P x_1; relax level 0 once.
 *
 * Layout: level l's points (1-based i, j, k) at off[l] + ((k-1) ny + (j-1))
 * nx + (i-1); A: 27 coefficients per point, offset (dx, dy, dz) at
 * (dz+1) 9 + (dy+1) 3 + (dx+1) (13 = the centre); P: 2 per point of level l
 * (toward the lower, the upper coarse neighbour along cdir[l]; 0 at even
 * points). C99 and C++.
 */
#ifndef AFH_PFMG_H
#define AFH_PFMG_H

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define AFH_PFMG_MAXL 64
#define AFH_PFMG_S 27
#define AFH_PFMG_C 13

typedef struct afh_pfmg {
  int nl;                         /* levels */
  int n[AFH_PFMG_MAXL][3];        /* points per direction */
  int cdir[AFH_PFMG_MAXL];        /* level l -> l + 1 (l < nl - 1) */
  int active[AFH_PFMG_MAXL];      /* relaxed on level l */
  double w[AFH_PFMG_MAXL];        /* Jacobi weight of level l */
  size_t off[AFH_PFMG_MAXL + 1];  /* first point of level l; off[nl] = all */
  double *A;                      /* 27 per point */
  double *P;                      /* 2 per point */
  double dxyz[3];                 /* as computed for level 0 */
  int dxyz_flag;
} afh_pfmg;

static inline int afh_pfmg_s(int dx, int dy, int dz) {
  return (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1);
}

static inline size_t afh_pfmg_ix(const afh_pfmg *h, int l, int i, int j, int k) {
  return h->off[l] + ((size_t)(k - 1) * h->n[l][1] + (size_t)(j - 1)) * h->n[l][0] +
         (size_t)(i - 1);
}

static inline void afh_pfmg_free(afh_pfmg *h) {
  free(h->A);
  free(h->P);
  h->A = h->P = NULL;
  h->nl = 0;
}

/* floor(log2(n)) (hypre_Log2) */
static inline int afh_pfmg_log2(int n) {
  int e = -1;
  while (n > 0) n >>= 1, e++;
  return e;
}

/* Builds the hierarchy from the folded level-1 operator a7 (per point, in
 * the level's point order: centre, -x, +x, -y, +y, -z, +z, the entries
 * toward the outside 0). ndim 2 or 3 (ndim = 2: nz = 1 and no z entries).
 * Returns 0, -1 on allocation failure. */
static inline int afh_pfmg_setup(afh_pfmg *h, int nx, int ny, int nz, int ndim,
                                 const double *a7) {
  memset(h, 0, sizeof *h);
  const size_t n0 = (size_t)nx * ny * nz;
  /* PFMGComputeDxyz (SS7 / SS5): the box loop in HYPRE's order, i fastest */
  double cx[3] = {0, 0, 0}, sq[3] = {0, 0, 0};
  for (size_t p = 0; p < n0; p++) {
    const double *a = a7 + 7 * p;
    const double dg = a[0] < 0.0 ? -1.0 : 1.0;
    for (int d = 0; d < ndim; d++) {
      const double t = -dg * (a[1 + 2 * d] + a[2 + 2 * d]);
      cx[d] = cx[d] + t;
      sq[d] = sq[d] + t * t;
    }
  }
  double mean[3], dev[3], cmax = 0.0;
  for (int d = 0; d < 3; d++) {
    cx[d] = cx[d] / (double)n0;
    sq[d] = sq[d] / (double)n0;
    mean[d] = cx[d];
    dev[d] = sq[d];
  }
  for (int d = 0; d < 3; d++) cmax = cx[d] > cmax ? cx[d] : cmax;
  if (cmax == 0.0) cmax = 1.0;
  for (int d = 0; d < 3; d++) {
    if (cx[d] > 0) {
      const double c = cx[d] / cmax;
      h->dxyz[d] = sqrt(1.0 / c);
    } else {
      h->dxyz[d] = 1.0e+123;
    }
  }
  for (int d = 0; d < ndim; d++) {
    dev[d] = dev[d] - mean[d] * mean[d];
    /* square of the coefficient of variation */
    if (dev[d] / (mean[d] * mean[d]) > .1) {
      h->dxyz_flag = 1;
      break;
    }
  }
  /* max_levels from the grid (pfmg_setup.c) */
  const int dims[3] = {nx, ny, nz};
  int max_levels = 1;
  for (int d = 0; d < ndim; d++) max_levels += afh_pfmg_log2(dims[d]) + 2;
  if (max_levels > AFH_PFMG_MAXL) max_levels = AFH_PFMG_MAXL;
  double dxyz[3] = {h->dxyz[0], h->dxyz[1], h->dxyz[2]};
  int coarsen[3] = {1, 1, 1}; /* forces relaxation on the finest grid */
  h->n[0][0] = nx, h->n[0][1] = ny, h->n[0][2] = nz;
  for (int l = 0;; l++) {
    double min_dxyz = dxyz[0] + dxyz[1] + dxyz[2] + 1, alpha = 0.0, beta = 0.0;
    int cdir = -1;
    for (int d = 0; d < ndim; d++) {
      if (h->n[l][d] > 1 && dxyz[d] < min_dxyz) {
        min_dxyz = dxyz[d];
        cdir = d;
      }
      alpha += 1.0 / (dxyz[d] * dxyz[d]);
    }
    h->w[l] = 1.0;
    if (cdir != -1) {
      if (h->dxyz_flag || ndim == 1) {
        h->w[l] = 2.0 / 3.0;
      } else {
        for (int d = 0; d < ndim; d++)
          if (d != cdir) beta += 1.0 / (dxyz[d] * dxyz[d]);
        if (beta == alpha) alpha = 0.0;
        else alpha = beta / alpha;
        h->w[l] = 2.0 / (3.0 - alpha);
      }
      if (l == max_levels - 1) cdir = -1;
    }
    if (cdir == -1) {
      h->active[l] = 1; /* forces relaxation on the coarsest grid */
      h->nl = l + 1;
      break;
    }
    h->cdir[l] = cdir;
    if (coarsen[cdir]) {
      /* coarsened in this direction before: relax level l */
      h->active[l] = 1;
      coarsen[0] = coarsen[1] = coarsen[2] = 0;
      coarsen[cdir] = 1;
    } else {
      h->active[l] = 0;
      coarsen[cdir] = 1;
    }
    dxyz[cdir] *= 2;
    for (int d = 0; d < 3; d++) h->n[l + 1][d] = h->n[l][d];
    h->n[l + 1][cdir] = h->n[l][cdir] / 2; /* even indices 2, 4, .. */
  }
  h->off[0] = 0;
  for (int l = 0; l < h->nl; l++)
    h->off[l + 1] = h->off[l] + (size_t)h->n[l][0] * h->n[l][1] * h->n[l][2];
  const size_t np = h->off[h->nl];
  h->A = (double *)calloc(np * AFH_PFMG_S, sizeof(double));
  h->P = (double *)calloc(np * 2, sizeof(double));
  if (!h->A || !h->P) {
    afh_pfmg_free(h);
    return -1;
  }
  for (size_t p = 0; p < n0; p++) {
    const double *a = a7 + 7 * p;
    double *A = h->A + AFH_PFMG_S * p;
    A[AFH_PFMG_C] = a[0];
    A[afh_pfmg_s(-1, 0, 0)] = a[1];
    A[afh_pfmg_s(1, 0, 0)] = a[2];
    A[afh_pfmg_s(0, -1, 0)] = a[3];
    A[afh_pfmg_s(0, 1, 0)] = a[4];
    if (ndim > 2) {
      A[afh_pfmg_s(0, 0, -1)] = a[5];
      A[afh_pfmg_s(0, 0, 1)] = a[6];
    }
  }
  for (int l = 0; l + 1 < h->nl; l++) {
    const int cd = h->cdir[l];
    const int *nf = h->n[l];
    /* PFMGSetupInterpOp: the odd points of direction cd */
    for (int k = 1; k <= nf[2]; k++)
      for (int j = 1; j <= nf[1]; j++)
        for (int i = 1; i <= nf[0]; i++) {
          const int q[3] = {i, j, k};
          if (!(q[cd] & 1)) continue;
          const size_t p = afh_pfmg_ix(h, l, i, j, k);
          const double *A = h->A + AFH_PFMG_S * p;
          double center = 0.0, p0 = 0.0, p1 = 0.0;
          for (int s = 0; s < AFH_PFMG_S; s++) {
            const int o[3] = {s % 3 - 1, (s / 3) % 3 - 1, s / 9 - 1};
            if (o[cd] == 0) center += A[s];
            else if (o[cd] == -1) p0 -= A[s];
            else p1 -= A[s];
          }
          if (center == 0.0) {
            p0 = 0.0;
            p1 = 0.0;
          } else {
            p0 /= center;
            p1 /= center;
          }
          int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
          lo[cd] = -1, hi[cd] = 1;
          /* zero where the operator has no entry in that direction: keeps
             the interpolation and the coarse operator inside the domain */
          if (A[afh_pfmg_s(lo[0], lo[1], lo[2])] == 0.0) p0 = 0.0;
          if (A[afh_pfmg_s(hi[0], hi[1], hi[2])] == 0.0) p1 = 0.0;
          h->P[2 * p] = p0;
          h->P[2 * p + 1] = p1;
        }
    /* Galerkin coarse operator R A P, R = P^T */
    const int *nc = h->n[l + 1];
    for (int k = 1; k <= nc[2]; k++)
      for (int j = 1; j <= nc[1]; j++)
        for (int i = 1; i <= nc[0]; i++) {
          double *Ac = h->A + AFH_PFMG_S * afh_pfmg_ix(h, l + 1, i, j, k);
          const int c[3] = {i, j, k};
          for (int df = -1; df <= 1; df++) {
            int f[3] = {c[0], c[1], c[2]};
            f[cd] = 2 * c[cd] + df;
            if (f[cd] < 1 || f[cd] > nf[cd]) continue;
            const size_t fp = afh_pfmg_ix(h, l, f[0], f[1], f[2]);
            const double rw = df == 0 ? 1.0 : (df < 0 ? h->P[2 * fp + 1] : h->P[2 * fp]);
            if (rw == 0.0) continue;
            const double *A = h->A + AFH_PFMG_S * fp;
            for (int s = 0; s < AFH_PFMG_S; s++) {
              const double a = A[s];
              if (a == 0.0) continue;
              const int o[3] = {s % 3 - 1, (s / 3) % 3 - 1, s / 9 - 1};
              int g[3];
              int inside = 1;
              for (int d = 0; d < 3; d++) {
                g[d] = f[d] + o[d];
                if (g[d] < 1 || g[d] > nf[d]) inside = 0;
              }
              if (!inside) continue;
              int oc[3] = {o[0], o[1], o[2]};
              if (!(g[cd] & 1)) {
                oc[cd] = g[cd] / 2 - c[cd];
                Ac[afh_pfmg_s(oc[0], oc[1], oc[2])] += rw * a;
              } else {
                const size_t gp = afh_pfmg_ix(h, l, g[0], g[1], g[2]);
                if (g[cd] - 1 >= 2) {
                  oc[cd] = (g[cd] - 1) / 2 - c[cd];
                  Ac[afh_pfmg_s(oc[0], oc[1], oc[2])] += rw * a * h->P[2 * gp];
                }
                if (g[cd] + 1 <= nf[cd]) {
                  oc[cd] = (g[cd] + 1) / 2 - c[cd];
                  Ac[afh_pfmg_s(oc[0], oc[1], oc[2])] += rw * a * h->P[2 * gp + 1];
                }
              }
            }
          }
        }
  }
  return 0;
}

#endif
