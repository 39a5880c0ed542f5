/* Exact level-1 solve of a one-box electrode grid (round 4; our algorithm,
 * like the Gauss-Seidel iteration it replaces -- the reference hands the
 * level-set stencils to HYPRE, afivo/src/m_coarse_solver.f90:286-338).
 *
 * The red-black Gauss-Seidel iteration with the box's variable stencil
 * (stencil_gsrb_357, m_af_stencil.f90:958-978: rhs + bc_correction, cell =
 * (rhs - sum of the neighbour terms) / c(1)) and the physical face fill
 * after each half sweep (bc_to_gc: Dirichlet g = 2 bv - x, Neumann
 * g = x -+ dr bv) converges to the x with
 *
 *   (c1 + sum_out c_q a_q) x_e + sum_in c_q x_q = (rhs_e + bcc_e) - g_e,
 *   g_e = sum_out c_q (b_q bv_q)
 *
 * (a_q, b_q the face fill's coefficients of the interior cell and the
 * boundary value; "out": the neighbours across a physical face). For a box
 * of up to AFH_CSD_N cells that system is inverted once on the host when the
 * stencil or the boundary conditions change (Gauss-Jordan with partial
 * pivoting) and each coarse solve is x = A^-1 ((rhs + bcc) - g), a dense
 * product in a fixed order: the device (k_cs_elec_direct) and the C oracle
 * (oracle/c/afo.c) evaluate the same expressions in the same order, so they
 * agree bitwise; the inverse itself is this header's arithmetic on the host
 * of both. C99 and C++.
 */
#ifndef AFH_CS_DIRECT_H
#define AFH_CS_DIRECT_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../../include/afivo_hip.h"

#define AFH_CSD_NC 8
#define AFH_CSD_N (AFH_CSD_NC * AFH_CSD_NC * AFH_CSD_NC)

/* The face fill's coefficients (gc_face_nocopy's physical branch):
 * ghost = b * value + a * interior */
static inline void afh_csd_face(const afh_bc *bc, int nb, const double *dr, double *a,
                                double *b) {
  const int d = (nb - 1) >> 1, low = ((nb - 1) & 1) == 0;
  switch (bc[nb - 1].type) {
  case AFH_BC_DIRICHLET: *b = 2; *a = -1; break;
  case AFH_BC_NEUMANN: *b = dr[d] * (low ? -1 : 1); *a = 1; break;
  default: *b = 1; *a = 0; break;
  }
}

/* A^-1 (column-major: ainv_t[c * n + r] = (A^-1)_{r c}) and g of the box's
 * stencil v (7 per cell, cell index ((k-1) nc + (j-1)) nc + (i-1)), the six
 * faces' boundary conditions and the box's spacing. work: 2 n^2 doubles.
 * Returns 0, or 1 when A is singular (the caller keeps the iteration). */
static inline int afh_csd_build(const double *v, const afh_bc *bc, const double *dr,
                                double *ainv_t, double *g, double *work) {
  const int nc = AFH_CSD_NC, n = AFH_CSD_N, w2 = 2 * AFH_CSD_N;
  double *m = work; /* [A | I], row-major, n x 2n */
  memset(m, 0, sizeof(double) * (size_t)n * w2);
  for (int r = 0; r < n; r++) m[(size_t)r * w2 + n + r] = 1.0;
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++) {
        const int e = ((k - 1) * nc + (j - 1)) * nc + (i - 1);
        const double *c = v + 7 * (size_t)e;
        const int p[3] = {i, j, k};
        double diag = c[0], ge = 0.0;
        for (int q = 1; q <= 6; q++) {
          const int d = (q - 1) >> 1, low = ((q - 1) & 1) == 0;
          int pq[3] = {p[0], p[1], p[2]};
          pq[d] += low ? -1 : 1;
          if (pq[d] < 1 || pq[d] > nc) {
            double a, b;
            afh_csd_face(bc, q, dr, &a, &b);
            diag = diag + c[q] * a;
            ge = ge + c[q] * (b * bc[q - 1].value);
          } else {
            const int f = ((pq[2] - 1) * nc + (pq[1] - 1)) * nc + (pq[0] - 1);
            m[(size_t)e * w2 + f] = c[q];
          }
        }
        m[(size_t)e * w2 + e] = diag;
        g[e] = ge;
      }
  /* Gauss-Jordan with partial pivoting */
  for (int col = 0; col < n; col++) {
    int piv = col;
    double best = fabs(m[(size_t)col * w2 + col]);
    for (int r = col + 1; r < n; r++) {
      const double x = fabs(m[(size_t)r * w2 + col]);
      if (x > best) best = x, piv = r;
    }
    if (!(best > 0.0)) return 1;
    /* (columns left of col are zero in rows col and piv, unit vectors of
       the earlier pivots elsewhere: the row operations start at col) */
    if (piv != col)
      for (int c = col; c < w2; c++) {
        const double t = m[(size_t)col * w2 + c];
        m[(size_t)col * w2 + c] = m[(size_t)piv * w2 + c];
        m[(size_t)piv * w2 + c] = t;
      }
    const double inv = 1.0 / m[(size_t)col * w2 + col];
    for (int c = col; c < w2; c++) m[(size_t)col * w2 + c] = m[(size_t)col * w2 + c] * inv;
    for (int r = 0; r < n; r++) {
      if (r == col) continue;
      const double f = m[(size_t)r * w2 + col];
      if (f == 0.0) continue;
      for (int c = col; c < w2; c++)
        m[(size_t)r * w2 + c] = m[(size_t)r * w2 + c] - f * m[(size_t)col * w2 + c];
    }
  }
  for (int r = 0; r < n; r++)
    for (int c = 0; c < n; c++) ainv_t[(size_t)c * n + r] = m[(size_t)r * w2 + n + c];
  return 0;
}

#endif
