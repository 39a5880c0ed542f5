/*
 * ORACLE TEST INFRASTRUCTURE -- not product code. See afo.h.
 *
 * CPU restatement of the afivo-streamer hot path (NDIM = 3), mirroring the
 * reference's per-box Fortran routines statement by statement, with the same
 * floating-point evaluation order (compile with -ffp-contract=off). Paths in
 * citations are relative to the reference root.
 */
#define _POSIX_C_SOURCE 200809L
#include "afo.h"
#include "../../afivo-streamer_amd/csrc/afh_cs_direct.h"
#include "../../afivo-streamer_amd/csrc/afh_pfmg.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char g_err[512];
static int32_t fail(int32_t code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
const char *afo_last_error(void) { return g_err; }
/* error setter for the C++ part of the oracle (c/afo_dist.cpp) */
__attribute__((visibility("hidden"))) int32_t afo_fail_msg(int32_t code, const char *msg) {
  return fail(code, "%s", msg);
}

typedef struct {
  int set;
  afh_bc bc[6];
  int rb;
  int lim;
  int prolong, prolong_lim; /* afo_set_cc_prolong (0: not an auto variable) */
} cc_method;

struct afh_tree {
  int nc, ng, nb, nlvl, nvc, nvf;
  size_t bsz, fsz; /* doubles per box per cc var / per fc var (3 dims) */
  afh_box_meta *boxes;
  int *ids, *ids_off, *leaves, *leaves_off, *parents, *parents_off;
  int cgs[3];
  double *cc, *fc;
  cc_method *meth; /* n_var_cell entries */
  int n_auto, *auto_vars; /* tree%cc_auto_vars: prolonged / restricted on regrid */
  /* box sharding (afo_tree_set_hook, afo_plan_*) */
  afh_hook_fn hook;
  void *hook_ctx;
  /* write generation per cc variable (afo_fluid_rhs_valid), as the device */
  unsigned long long *gen;
  /* box capacity of the pools (afh_tree_desc.box_capacity) and the in-place
   * regrid contract of the device library: a regrid whose topology fits the
   * capacity retires the old handle (its entry points fail) */
  int cap, retired;
  int nplans;
  struct afo_plan {
    int n, fc;
    int32_t *reg;
    int64_t *off;
  } *plans;
  /* sharded tree: leaves another rank sums (replicated levels count on rank
   * 0 only, as the device library); NULL on an unsharded tree */
  unsigned char *sum_skip;
  /* the deferred reductions (afo_*_fold): the last value of each slot --
   * the limits (0..2) already reduced over ranks, the |x| maxima (3, 4) this
   * rank's, reduced when they are read */
  double slot[8];
};

#define LIVE(t)                                                               \
  do {                                                                        \
    if (!(t)) return fail(AFH_ERR_ARG, "null tree");                          \
    if ((t)->retired)                                                         \
      return fail(AFH_ERR_STATE, "tree handle retired by an in-place regrid"); \
  } while (0)

static inline void touch(afh_tree *t, int iv) {
  if (iv >= 0 && iv <= t->nvc) t->gen[iv]++;
}

static int32_t hook(afh_tree *t, int kind, int lvl, int iv, double *vals, int n) {
  if (!t->hook) return AFH_OK;
  return t->hook(t->hook_ctx, kind, lvl, iv, vals, n) ? AFH_ERR_STATE : AFH_OK;
}

struct afh_mg {
  afh_tree *t;
  afh_mg_desc d;
  double *lvl_c; /* per level: 7 stencil coefficients (mg_box_lpl_stencil) */
  /* coarse solver hierarchy */
  int n_mg;
  int dims[16][3];
  double *u[16], *f[16], *r[16];
  double hc[16][3]; /* 1/h^2 per dim per MG level */
  double cdiag[16];  /* unfolded diagonal per MG level */
  double dtab[16][64][2]; /* folded (diag, 1/diag) per boundary class */
  /* AFH_COARSE_DIRECT: per dimension the orthonormal eigenvectors q[d]
   * (n x n, q[i*n + p] = v_p(i)) and eigenvalues e[d] of the 1-D folded
   * operator, two work grids, and the BC types the tables were built for */
  double *q[3], *e[3], *w1, *w2;
  int q_bc[6];
  /* electrode (level-set) boxes, per box id - 1 (NULL / 0 = none): the
   * variable operator stencil v(7, nc^3) and its bc_correction
   * (mg_box_lsf_stencil + mg_set_operators_lvl), and the boundary distances
   * of mg_box_lpllsf_gradient (n cells: ix(3, n), dd(6, n), boundary value
   * per cell) */
  double **vst, **vbc;
  int *lsf_n;
  int32_t **lsf_ix;
  double **lsf_dd, **lsf_bv;
  int i_lsf;
  int cs_iters; /* level-1 cycles of the last coarse solve */
  /* AFH_COARSE_PFMG: the hierarchy (afh_pfmg.h), the folded level-1
   * operator it was built from, and the level vectors */
  afh_pfmg pf;
  double *pf_a7, *pf_x, *pf_b, *pf_r, *pf_e;
};

#define AFH_CS_BOTTOM_SWEEPS 16

struct afh_fluid {
  afh_tree *t;
  afh_fluid_desc d;
  double *td, *chem;
  afh_reaction reac[AFH_MAX_REACTIONS];
  int rhs_iv, rhs_state, rhs_ghosts; /* afo_fluid_set_rhs_output */
  int phi_iv;     /* afo_fluid_set_field_source (0: read f_field) */
  double phi_fac;
  double ion_se_yield; /* afo_fluid_set_ion_se_yield (input_data%ion_se_yield) */
  double rhs_max;
  int mask_iv; /* afo_fluid_set_update_mask: set_box_mask's level set (0: none) */
  /* generations of rhs_iv and the densities of rhs_state after the update */
  unsigned long long rhs_snap[AFH_MAX_SPECIES + 1];
};

/* ---------------------------------------------------------------- tables
 * afivo/src/m_af_types.f90:167-236 (NDIM = 3) */
static const int child_dix[8][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0},
                                    {1, 1, 0}, {0, 0, 1}, {1, 0, 1},
                                    {0, 1, 1}, {1, 1, 1}};
static const int child_adj_nb[6][4] = {{1, 3, 5, 7}, {2, 4, 6, 8},
                                       {1, 2, 5, 6}, {3, 4, 7, 8},
                                       {1, 2, 3, 4}, {5, 6, 7, 8}};
static const int edge_dim[12] = {1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3};
static const int edge_dir[12][3] = {
    {0, -1, -1}, {0, 1, -1}, {0, -1, 1}, {0, 1, 1}, {-1, 0, -1}, {1, 0, -1},
    {-1, 0, 1},  {1, 0, 1},  {-1, -1, 0}, {1, -1, 0}, {-1, 1, 0}, {1, 1, 0}};
static const int nb_adj_edge[12][2] = {{3, 5}, {4, 5}, {3, 6}, {4, 6},
                                       {1, 5}, {2, 5}, {1, 6}, {2, 6},
                                       {1, 3}, {2, 3}, {1, 4}, {2, 4}};
static const int edge_min_ix[12][3] = {
    {0, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 1, 1}, {0, 0, 0}, {1, 0, 0},
    {0, 0, 1}, {1, 0, 1}, {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0}};

static inline int nb_dim(int nb) { return (nb - 1) / 2; } /* 0-based dim */
static inline int nb_low(int nb) { return (nb - 1) % 2 == 0; }
static inline int nb_pm(int nb) { return nb_low(nb) ? -1 : 1; }

/* ---------------------------------------------------------------- access */
static inline double *ccb(afh_tree *t, int iv, int id) {
  return t->cc + ((size_t)(iv - 1) * t->nb + (size_t)(id - 1)) * t->bsz;
}
#define IX(t, i, j, k) ((((size_t)(k)) * (t)->ng + (size_t)(j)) * (t)->ng + (size_t)(i))
/* fc(i,j,k,dim) with Fortran indices 1..nc+1 */
static inline double *fcb(afh_tree *t, int ivf, int id) {
  return t->fc + ((size_t)(ivf - 1) * t->nb + (size_t)(id - 1)) * t->fsz;
}
#define FX(t, d, i, j, k)                                                     \
  ((size_t)(d) * (size_t)((t)->nc + 1) * ((t)->nc + 1) * ((t)->nc + 1) +      \
   (((size_t)(k)-1) * ((t)->nc + 1) + ((size_t)(j)-1)) * ((t)->nc + 1) +      \
   ((size_t)(i)-1))

static inline afh_box_meta *B(afh_tree *t, int id) { return &t->boxes[id - 1]; }
static inline int nmat(afh_tree *t, int id, int dx, int dy, int dz) {
  return B(t, id)->neighbor_mat[(dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
}
/* af_get_child_offset, m_af_types.f90:903-910 */
static inline void child_offset(afh_tree *t, int id, int nb, int off[3]) {
  for (int d = 0; d < 3; d++) {
    off[d] = ((B(t, id)->ix[d] - 1) & 1) * (t->nc >> 1);
    if (nb > 0 && nb_dim(nb) == d) off[d] -= nb_pm(nb) * t->nc;
  }
}

/* ---------------------------------------------------------------- tree */
int32_t afo_tree_create(const afh_tree_desc *d, int32_t device,
                        afh_tree **out) {
  (void)device;
  if (!d || !out || d->n_cell < 2 || (d->n_cell & 1) || d->n_boxes < 1)
    return fail(AFH_ERR_ARG, "afo_tree_create: bad descriptor");
  if (d->periodic[0] || d->periodic[1] || d->periodic[2])
    return fail(AFH_ERR_UNSUPPORTED, "periodic domains not supported");
  afh_tree *t = calloc(1, sizeof *t);
  t->nc = d->n_cell;
  t->ng = d->n_cell + 2;
  t->nb = d->n_boxes;
  t->nlvl = d->highest_lvl;
  t->nvc = d->n_var_cell;
  t->nvf = d->n_var_face;
  t->bsz = (size_t)t->ng * t->ng * t->ng;
  t->fsz = 3 * (size_t)(t->nc + 1) * (t->nc + 1) * (t->nc + 1);
  for (int i = 0; i < 3; i++) t->cgs[i] = d->coarse_grid_size[i];
  t->boxes = malloc(sizeof(afh_box_meta) * t->nb);
  memcpy(t->boxes, d->boxes, sizeof(afh_box_meta) * t->nb);
  int n = t->nlvl + 1;
#define CPYL(dst, dsto, src, srco)                                            \
  t->dsto = malloc(sizeof(int) * n);                                          \
  memcpy(t->dsto, d->srco, sizeof(int) * n);                                  \
  t->dst = malloc(sizeof(int) * (t->dsto[t->nlvl] + 1));                      \
  memcpy(t->dst, d->src, sizeof(int) * t->dsto[t->nlvl]);
  CPYL(ids, ids_off, lvl_ids, lvl_ids_off)
  CPYL(leaves, leaves_off, lvl_leaves, lvl_leaves_off)
  CPYL(parents, parents_off, lvl_parents, lvl_parents_off)
#undef CPYL
  t->cc = calloc((size_t)t->nvc * t->nb * t->bsz, sizeof(double));
  t->fc = calloc((size_t)(t->nvf > 0 ? t->nvf : 1) * t->nb * t->fsz,
                 sizeof(double));
  t->meth = calloc(t->nvc + 1, sizeof(cc_method));
  t->auto_vars = calloc(t->nvc + 1, sizeof(int));
  t->gen = calloc(t->nvc + 1, sizeof(unsigned long long));
  t->cap = d->box_capacity > t->nb ? d->box_capacity : t->nb;
  if (!t->cc || !t->fc) return fail(AFH_ERR_ARG, "out of memory");
  *out = t;
  return AFH_OK;
}

/* sharded trees (c/afo_dist.cpp): box id's data read as NaN in every
 * variable (the unused id standing for boxes a rank does not store) */
__attribute__((visibility("hidden"))) void afo_set_sum_skip(afh_tree *t,
                                                           const unsigned char *skip) {
  free(t->sum_skip);
  t->sum_skip = (unsigned char *)malloc((size_t)t->nb);
  memcpy(t->sum_skip, skip, (size_t)t->nb);
}

__attribute__((visibility("hidden"))) void afo_poison_box(afh_tree *t, int id) {
  for (int iv = 1; iv <= t->nvc; iv++) memset(ccb(t, iv, id), 0xff, sizeof(double) * t->bsz);
  for (int iv = 1; iv <= t->nvf; iv++) memset(fcb(t, iv, id), 0xff, sizeof(double) * t->fsz);
}

int32_t afo_tree_destroy(afh_tree *t) {
  if (!t) return AFH_OK;
  free(t->boxes);
  free(t->ids), free(t->ids_off), free(t->leaves), free(t->leaves_off);
  free(t->parents), free(t->parents_off);
  free(t->cc), free(t->fc), free(t->meth), free(t->auto_vars), free(t->gen);
  free(t->sum_skip);
  for (int q = 0; q < t->nplans; q++) free(t->plans[q].reg), free(t->plans[q].off);
  free(t->plans);
  free(t);
  return AFH_OK;
}
int32_t afo_tree_sync(afh_tree *t) {
  (void)t;
  return AFH_OK;
}

#define LVL_N(t, arr, l) ((t)->arr##_off[(l)] - (t)->arr##_off[(l)-1])
#define LVL_AT(t, arr, l, i) ((t)->arr[(t)->arr##_off[(l)-1] + (i)])

int32_t afo_set_cc_methods(afh_tree *t, int32_t iv, const afh_bc *bc6,
                           int32_t rb, int32_t lim) {
  if (iv < 1 || iv > t->nvc) return fail(AFH_ERR_ARG, "bad iv");
  cc_method *m = &t->meth[iv];
  m->set = 1;
  memcpy(m->bc, bc6, sizeof m->bc);
  m->rb = rb;
  m->lim = lim;
  return AFH_OK;
}
int32_t afo_set_bc(afh_tree *t, int32_t iv, int32_t nb, int32_t type,
                   double value) {
  if (iv < 1 || iv > t->nvc || nb < 1 || nb > 6) return fail(AFH_ERR_ARG, "bad arg");
  t->meth[iv].bc[nb - 1].type = type;
  t->meth[iv].bc[nb - 1].value = value;
  return AFH_OK;
}

int32_t afo_cc_put(afh_tree *t, int32_t iv, const double *h) {
  LIVE(t);
  if (iv < 1 || iv > t->nvc) return fail(AFH_ERR_ARG, "bad iv");
  touch(t, iv);
  memcpy(ccb(t, iv, 1), h, sizeof(double) * t->bsz * t->nb);
  return AFH_OK;
}
int32_t afo_cc_get(afh_tree *t, int32_t iv, double *h) {
  LIVE(t);
  if (iv < 1 || iv > t->nvc) return fail(AFH_ERR_ARG, "bad iv");
  memcpy(h, ccb(t, iv, 1), sizeof(double) * t->bsz * t->nb);
  return AFH_OK;
}
int32_t afo_fc_put(afh_tree *t, int32_t ivf, const double *h) {
  LIVE(t);
  if (ivf < 1 || ivf > t->nvf) return fail(AFH_ERR_ARG, "bad ivf");
  memcpy(fcb(t, ivf, 1), h, sizeof(double) * t->fsz * t->nb);
  return AFH_OK;
}
int32_t afo_fc_get(afh_tree *t, int32_t ivf, double *h) {
  LIVE(t);
  if (ivf < 1 || ivf > t->nvf) return fail(AFH_ERR_ARG, "bad ivf");
  memcpy(h, fcb(t, ivf, 1), sizeof(double) * t->fsz * t->nb);
  return AFH_OK;
}

/* afh_tree_pack_boxes / afh_tree_unpack_boxes (include/afivo_hip.h): the
 * boxes' rows in caller memory (host memory here), same row layout */
static int32_t box_rows(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                        int32_t n_fc, double *buf, int unpack) {
  LIVE(t);
  if (n < 0 || (n && (!ids || !buf)) || n_cc < 0 || n_cc > t->nvc || n_fc < 0 ||
      n_fc > t->nvf)
    return fail(AFH_ERR_ARG, "bad box rows");
  const size_t w = (size_t)n_cc * t->bsz + (size_t)n_fc * t->fsz;
  for (int r = 0; r < n; r++) {
    if (ids[r] < 1 || ids[r] > t->nb) return fail(AFH_ERR_ARG, "bad box id");
    double *b = buf + (size_t)r * w;
    for (int q = 0; q < n_cc + n_fc; q++) {
      const size_t blk = q < n_cc ? t->bsz : t->fsz;
      double *c = q < n_cc ? ccb(t, q + 1, ids[r]) : fcb(t, q - n_cc + 1, ids[r]);
      if (unpack) memcpy(c, b, sizeof(double) * blk);
      else memcpy(b, c, sizeof(double) * blk);
      b += blk;
    }
  }
  return AFH_OK;
}
int32_t afo_tree_pack_boxes(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                            int32_t n_fc, double *buf) {
  return box_rows(t, ids, n, n_cc, n_fc, buf, 0);
}
int32_t afo_tree_unpack_boxes(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                              int32_t n_fc, const double *buf) {
  return box_rows(t, ids, n, n_cc, n_fc, (double *)buf, 1);
}
int32_t afo_device_alloc(int32_t device, int64_t n_bytes, void **out) {
  (void)device;
  if (!out || n_bytes < 0) return fail(AFH_ERR_ARG, "bad allocation");
  *out = malloc(n_bytes > 0 ? (size_t)n_bytes : 8);
  return *out ? AFH_OK : fail(AFH_ERR_DEVICE, "out of memory");
}
int32_t afo_device_free(void *p) {
  free(p);
  return AFH_OK;
}

/* ------------------------------------------------------------ ghost cells */

/* copy_from_nb, m_af_ghostcell.f90:654-669 */
static void copy_from_nb(afh_tree *t, int id, int nb_id, const int dnb[3],
                         const int lo[3], const int hi[3], int iv) {
  double *c = ccb(t, iv, id), *cn = ccb(t, iv, nb_id);
  int nc = t->nc;
  for (int k = lo[2]; k <= hi[2]; k++)
    for (int j = lo[1]; j <= hi[1]; j++)
      for (int i = lo[0]; i <= hi[0]; i++)
        c[IX(t, i, j, k)] =
            cn[IX(t, i - dnb[0] * nc, j - dnb[1] * nc, k - dnb[2] * nc)];
}

/* bc_to_gc, m_af_ghostcell.f90:173-279 */
static void bc_to_gc(afh_tree *t, int id, int nb, int iv, const afh_bc *bc) {
  double c0, c1, c2;
  int nc = t->nc, d = nb_dim(nb);
  switch (bc->type) {
  case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = 0; break;
  case AFH_BC_NEUMANN: c0 = B(t, id)->dr[d] * nb_pm(nb); c1 = 1; c2 = 0; break;
  case AFH_BC_CONTINUOUS: c0 = 0; c1 = 2; c2 = -1; break;
  default: c0 = 1; c1 = 0; c2 = 0; break; /* dirichlet_copy */
  }
  double *c = ccb(t, iv, id);
  int g = nb_low(nb) ? 0 : nc + 1, x1 = nb_low(nb) ? 1 : nc,
      x2 = nb_low(nb) ? 2 : nc - 1;
  for (int b = 1; b <= nc; b++)
    for (int a = 1; a <= nc; a++) {
      int p0[3], p1[3], p2[3];
      /* (a, b) run over the two tangential dims in index order */
      int td0 = (d == 0) ? 1 : 0, td1 = (d == 2) ? 1 : 2;
      p0[d] = g, p1[d] = x1, p2[d] = x2;
      p0[td0] = p1[td0] = p2[td0] = a;
      p0[td1] = p1[td1] = p2[td1] = b;
      c[IX(t, p0[0], p0[1], p0[2])] =
          c0 * bc->value + c1 * c[IX(t, p1[0], p1[1], p1[2])] +
          c2 * c[IX(t, p2[0], p2[1], p2[2])];
    }
}

/* mg_sides_rb, m_af_multigrid.f90:294-461 (3D) */
static void mg_sides_rb(afh_tree *t, int id, int nb, int iv) {
  int nc = t->nc, hnc = nc / 2, co[3];
  int p_id = B(t, id)->parent, p_nb_id = B(t, p_id)->neighbors[nb - 1];
  child_offset(t, id, 0, co);
  double *cp = ccb(t, iv, p_nb_id), *c = ccb(t, iv, id);
  int tw = hnc + 2;
  double tmp[(64 / 2 + 2) * (64 / 2 + 2) * 4];
  double gc[64 * 64 * 4];
#define TMP(a, b) tmp[(b) * tw + (a)]
#define GC(a, b) gc[((b)-1) * nc + ((a)-1)]
  for (int b = 0; b <= hnc + 1; b++)
    for (int a = 0; a <= hnc + 1; a++) {
      double v = 0;
      switch (nb) {
      case 1: v = cp[IX(t, nc, co[1] + a, co[2] + b)]; break;
      case 2: v = cp[IX(t, 1, co[1] + a, co[2] + b)]; break;
      case 3: v = cp[IX(t, co[0] + a, nc, co[2] + b)]; break;
      case 4: v = cp[IX(t, co[0] + a, 1, co[2] + b)]; break;
      case 5: v = cp[IX(t, co[0] + a, co[1] + b, nc)]; break;
      case 6: v = cp[IX(t, co[0] + a, co[1] + b, 1)]; break;
      }
      TMP(a, b) = v;
    }
  for (int j = 1; j <= hnc; j++)
    for (int i = 1; i <= hnc; i++) {
      double g1 = 0.125 * (TMP(i + 1, j) - TMP(i - 1, j));
      double g2 = 0.125 * (TMP(i, j + 1) - TMP(i, j - 1));
      GC(2 * i - 1, 2 * j - 1) = TMP(i, j) - g1 - g2;
      GC(2 * i, 2 * j - 1) = TMP(i, j) + g1 - g2;
      GC(2 * i - 1, 2 * j) = TMP(i, j) - g1 + g2;
      GC(2 * i, 2 * j) = TMP(i, j) + g1 + g2;
    }
  int ix = nb_low(nb) ? 1 : nc, di = nb_low(nb) ? 1 : -1;
  switch (nb_dim(nb)) {
  case 0:
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        c[IX(t, ix - di, j, k)] = 0.5 * GC(j, k) + 0.75 * c[IX(t, ix, j, k)] -
                                  0.25 * c[IX(t, ix + di, j, k)];
    break;
  case 1:
    for (int k = 1; k <= nc; k++)
      for (int i = 1; i <= nc; i++)
        c[IX(t, i, ix - di, k)] = 0.5 * GC(i, k) + 0.75 * c[IX(t, i, ix, k)] -
                                  0.25 * c[IX(t, i, ix + di, k)];
    break;
  case 2:
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++)
        c[IX(t, i, j, ix - di)] = 0.5 * GC(i, j) + 0.75 * c[IX(t, i, j, ix)] -
                                  0.25 * c[IX(t, i, j, ix + di)];
    break;
  }
#undef TMP
#undef GC
}

/* af_gc_interp / af_gc_interp_lim, m_af_ghostcell.f90:394-612 (3D) */
static void gc_interp(afh_tree *t, int id, int nb, int iv, int lim) {
  const double third = 1 / 3.0, sixth = 1 / 6.0;
  int nc = t->nc, off[3];
  int p_id = B(t, id)->parent, p_nb_id = B(t, p_id)->neighbors[nb - 1];
  child_offset(t, id, nb, off);
  double *cp = ccb(t, iv, p_nb_id), *c = ccb(t, iv, id);
  int ix, ix_f, ix_c;
  if (nb_low(nb)) ix = 0, ix_f = 1, ix_c = nc;
  else ix = nc + 1, ix_f = nc, ix_c = 1;
  for (int b = 1; b <= nc; b++) {
    for (int a = 1; a <= nc; a++) {
      double c1, c2, c3, cf;
      size_t dst;
      int a1, a2, b1, b2;
      /* a runs over the first tangential dim, b over the second */
      int d = nb_dim(nb);
      int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
      a1 = off[ta] + ((a + 1) >> 1);
      a2 = a1 + 1 - 2 * (a & 1);
      b1 = off[tb] + ((b + 1) >> 1);
      b2 = b1 + 1 - 2 * (b & 1);
      if (d == 0) {
        c1 = cp[IX(t, ix_c, a1, b1)];
        c2 = cp[IX(t, ix_c, a2, b1)];
        c3 = cp[IX(t, ix_c, a1, b2)];
        cf = c[IX(t, ix_f, a, b)];
        dst = IX(t, ix, a, b);
      } else if (d == 1) {
        c1 = cp[IX(t, a1, ix_c, b1)];
        c2 = cp[IX(t, a2, ix_c, b1)];
        c3 = cp[IX(t, a1, ix_c, b2)];
        cf = c[IX(t, a, ix_f, b)];
        dst = IX(t, a, ix, b);
      } else {
        /* case (3): c(2) uses j_c2, c(3) uses i_c2 (m_af_ghostcell.f90:479-482) */
        c1 = cp[IX(t, a1, b1, ix_c)];
        c2 = cp[IX(t, a1, b2, ix_c)];
        c3 = cp[IX(t, a2, b1, ix_c)];
        cf = c[IX(t, a, b, ix_f)];
        dst = IX(t, a, b, ix);
      }
      double v = third * c1 + sixth * c2 + sixth * c3 + third * cf;
      if (lim && v > 2 * c1) v = 2 * c1;
      c[dst] = v;
    }
  }
}

/* af_edge_gc_extrap, m_af_ghostcell.f90:895-924 */
static void edge_extrap(afh_tree *t, int id, const int lo[3], int dim, int iv) {
  double *c = ccb(t, iv, id);
  int o1 = dim % 3, o2 = (dim + 1) % 3; /* 1 + mod(dim, 3) with 1-based dim */
  /* dim here is 0-based: o_dims = [1+mod(dim1,3), 1+mod(dim1+1,3)] with
   * dim1 = dim+1 gives 0-based (dim+1)%3 and (dim+2)%3 */
  o1 = (dim + 1) % 3;
  o2 = (dim + 2) % 3;
  int di[3];
  for (int d = 0; d < 3; d++) di[d] = 1 - 2 * (lo[d] & 1);
  di[dim] = 0;
  int ia[3] = {lo[0], lo[1], lo[2]}, ib[3] = {lo[0], lo[1], lo[2]}, ic[3],
      x[3] = {lo[0], lo[1], lo[2]};
  ia[o1] += di[o1];
  ib[o2] += di[o2];
  for (int d = 0; d < 3; d++) ic[d] = lo[d] + di[d];
  for (int n = 1; n <= t->nc; n++) {
    ia[dim] = ib[dim] = ic[dim] = x[dim] = n;
    c[IX(t, x[0], x[1], x[2])] = c[IX(t, ia[0], ia[1], ia[2])] +
                                 c[IX(t, ib[0], ib[1], ib[2])] -
                                 c[IX(t, ic[0], ic[1], ic[2])];
  }
}

/* af_corner_gc_extrap, m_af_ghostcell.f90:860-889 (3D) */
static void corner_extrap(afh_tree *t, int id, const int x[3], int iv) {
  double *c = ccb(t, iv, id);
  int di[3];
  for (int d = 0; d < 3; d++) di[d] = 1 - 2 * (x[d] & 1);
  c[IX(t, x[0], x[1], x[2])] =
      c[IX(t, x[0], x[1] + di[1], x[2] + di[2])] +
      c[IX(t, x[0] + di[0], x[1], x[2] + di[2])] +
      c[IX(t, x[0] + di[0], x[1] + di[1], x[2])] -
      2 * c[IX(t, x[0] + di[0], x[1] + di[1], x[2] + di[2])];
}

/* af_gc_box_corner, m_af_ghostcell.f90:125-170 */
static void gc_box_corner(afh_tree *t, int id, int iv) {
  int nc = t->nc;
  for (int n = 0; n < 12; n++) {
    int dim = edge_dim[n] - 1, lo[3], hi[3], dnb[3] = {0, 0, 0};
    int nb_id = nmat(t, id, edge_dir[n][0], edge_dir[n][1], edge_dir[n][2]);
    for (int d = 0; d < 3; d++) lo[d] = edge_min_ix[n][d] * (nc + 1);
    lo[dim] = 1;
    if (nb_id > 0) {
      for (int d = 0; d < 3; d++) hi[d] = lo[d];
      hi[dim] = nc;
      for (int q = 0; q < 2; q++) {
        int nb = nb_adj_edge[n][q];
        dnb[nb_dim(nb)] += nb_pm(nb);
      }
      copy_from_nb(t, id, nb_id, dnb, lo, hi, iv);
    } else {
      edge_extrap(t, id, lo, dim, iv);
    }
  }
  for (int n = 0; n < 8; n++) {
    int dnb[3], lo[3];
    for (int d = 0; d < 3; d++) {
      dnb[d] = 2 * child_dix[n][d] - 1;
      lo[d] = child_dix[n][d] * (nc + 1);
    }
    int nb_id = nmat(t, id, dnb[0], dnb[1], dnb[2]);
    if (nb_id > 0) copy_from_nb(t, id, nb_id, dnb, lo, lo, iv);
    else corner_extrap(t, id, lo, iv);
  }
}

/* af_gc_box, m_af_ghostcell.f90:64-120 */
static void gc_box(afh_tree *t, int id, int iv, int corners) {
  int nc = t->nc;
  cc_method *m = &t->meth[iv];
  for (int nb = 1; nb <= 6; nb++) {
    int nb_id = B(t, id)->neighbors[nb - 1];
    if (nb_id > 0) {
      int lo[3] = {1, 1, 1}, hi[3] = {nc, nc, nc}, dnb[3] = {0, 0, 0};
      int d = nb_dim(nb);
      lo[d] = hi[d] = nb_low(nb) ? 0 : nc + 1;
      dnb[d] = nb_pm(nb);
      copy_from_nb(t, id, nb_id, dnb, lo, hi, iv);
    } else if (nb_id == 0) {
      if (m->rb == AFH_RB_MG_SIDES) mg_sides_rb(t, id, nb, iv);
      else gc_interp(t, id, nb, iv, m->rb == AFH_RB_GC_INTERP_LIM);
    } else {
      bc_to_gc(t, id, nb, iv, &m->bc[nb - 1]);
    }
  }
  if (corners) gc_box_corner(t, id, iv);
}

/* af_gc_lvl; with sharding hooks (replicas refreshed before, their ghost
 * cells after) */
static int32_t gc_lvl(afh_tree *t, int lvl, int iv, int corners) {
  int n = LVL_N(t, ids, lvl);
  if (hook(t, AFH_HOOK_HALO, lvl, iv, NULL, 0)) return AFH_ERR_STATE;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; i++) gc_box(t, LVL_AT(t, ids, lvl, i), iv, corners);
  return hook(t, AFH_HOOK_RIMS, lvl, iv, NULL, 0);
}

int32_t afo_gc_lvl(afh_tree *t, int32_t lvl, int32_t iv, int32_t corners) {
  LIVE(t);
  if (lvl < 1 || lvl > t->nlvl || iv < 1 || iv > t->nvc || !t->meth[iv].set)
    return fail(AFH_ERR_ARG, "afo_gc_lvl: bad argument / no methods");
  touch(t, iv);
  return gc_lvl(t, lvl, iv, corners);
}
int32_t afo_gc_tree(afh_tree *t, int32_t iv, int32_t corners) {
  for (int l = 1; l <= t->nlvl; l++) {
    int32_t e = afo_gc_lvl(t, l, iv, corners);
    if (e) return e;
  }
  return AFH_OK;
}

/* -------------------------------------------------------- restriction */

/* af_restrict_box, m_af_restrict.f90:62-136 (3D): 0.125 * sum over the 2^3
 * children in column-major element order */
static void restrict_box(afh_tree *t, int c_id, int p_id, int iv) {
  int hnc = t->nc / 2, off[3];
  child_offset(t, c_id, 0, off);
  double *c = ccb(t, iv, c_id), *p = ccb(t, iv, p_id);
  for (int k = 1; k <= hnc; k++)
    for (int j = 1; j <= hnc; j++)
      for (int i = 1; i <= hnc; i++) {
        int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
        double s = c[IX(t, fi, fj, fk)];
        s += c[IX(t, fi + 1, fj, fk)];
        s += c[IX(t, fi, fj + 1, fk)];
        s += c[IX(t, fi + 1, fj + 1, fk)];
        s += c[IX(t, fi, fj, fk + 1)];
        s += c[IX(t, fi + 1, fj, fk + 1)];
        s += c[IX(t, fi, fj + 1, fk + 1)];
        s += c[IX(t, fi + 1, fj + 1, fk + 1)];
        p[IX(t, off[0] + i, off[1] + j, off[2] + k)] = 0.125 * s;
      }
}

int32_t afo_restrict_tree(afh_tree *t, int32_t iv) {
  LIVE(t);
  touch(t, iv);
  /* af_restrict_tree -> af_restrict_to_boxes over parents per level */
  for (int l = t->nlvl - 1; l >= 1; l--) {
    int n = LVL_N(t, parents, l);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) {
      int id = LVL_AT(t, parents, l, i);
      for (int c = 0; c < 8; c++) {
        int cid = B(t, id)->children[c];
        if (cid > 0) restrict_box(t, cid, id, iv);
      }
    }
    if (hook(t, AFH_HOOK_RESTRICT, l + 1, iv, NULL, 0)) return AFH_ERR_STATE;
  }
  return AFH_OK;
}

int32_t afo_tree_copy_cc(afh_tree *t, int32_t a, int32_t b) {
  LIVE(t);
  touch(t, b);
  memcpy(ccb(t, b, 1), ccb(t, a, 1), sizeof(double) * t->bsz * t->nb);
  return AFH_OK;
}

/* af_tree_maxabs_cc over leaf interiors, m_af_utils.f90:773-784, 852-862 */
static double maxabs_local(afh_tree *t, int32_t iv);
int32_t afo_tree_maxabs_cc(afh_tree *t, int32_t iv, double *out) {
  LIVE(t);
  *out = maxabs_local(t, iv);
  return hook(t, AFH_HOOK_MAX, 0, iv, out, 1);
}

static double maxabs_local(afh_tree *t, int32_t iv) {
  double mx = -HUGE_VAL;
  int nc = t->nc;
  for (int l = 1; l <= t->nlvl; l++)
    for (int i = 0; i < LVL_N(t, leaves, l); i++) {
      double *c = ccb(t, iv, LVL_AT(t, leaves, l, i));
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int ii = 1; ii <= nc; ii++) {
            double v = fabs(c[IX(t, ii, j, k)]);
            if (v > mx) mx = v;
          }
    }
  return mx;
}

/* gfortran's real ** integer (_gfortran_pow_r8_i4): binary powering */
static double ipow(double x, int n) {
  double p = 1.0;
  for (;;) {
    if (n & 1) p *= x;
    n >>= 1;
    if (!n) break;
    x *= x;
  }
  return p;
}

/* af_tree_sum_cc, m_af_utils.f90:966-1026 (leaves in loop order; the per-box
 * sum is sequential here, a fixed tree on the device: equal to rounding) */
int32_t afo_tree_sum_cc(afh_tree *t, int32_t iv, int32_t power, double *out) {
  LIVE(t);
  if (iv < 1 || iv > t->nvc || power < 1) return fail(AFH_ERR_ARG, "bad argument");
  const int nc = t->nc;
  double my_sum = 0.0;
  for (int l = 1; l <= t->nlvl; l++) {
    if (LVL_N(t, ids, l) == 0) continue;
    const afh_box_meta *m = B(t, LVL_AT(t, ids, l, 0));
    const double fac = m->dr[0] * m->dr[1] * m->dr[2];
    for (int q = 0; q < LVL_N(t, leaves, l); q++) {
      if (t->sum_skip && t->sum_skip[LVL_AT(t, leaves, l, q) - 1]) continue;
      const double *c = ccb(t, iv, LVL_AT(t, leaves, l, q));
      double tmp = 0.0;
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc; i++) tmp += ipow(c[IX(t, i, j, k)], power);
      my_sum = my_sum + fac * tmp;
    }
  }
  *out = my_sum;
  return hook(t, AFH_HOOK_SUM, 0, iv, out, 1);
}

/* af_reduction_loc with box_max_cc / box_min_cc / box_maxabs_cc,
 * m_af_utils.f90:694-754, 840-874 (one thread: boxes in loop order) */
int32_t afo_tree_reduce_loc(afh_tree *t, int32_t iv, int32_t op, double *out,
                            int32_t *loc) {
  LIVE(t);
  if (iv < 1 || iv > t->nvc || op < AFH_RED_MAX || op > AFH_RED_MAXABS)
    return fail(AFH_ERR_ARG, "bad argument");
  if (t->hook && loc) return fail(AFH_ERR_UNSUPPORTED, "location of a sharded reduction");
  const int nc = t->nc, is_min = op == AFH_RED_MIN;
  double val = (is_min ? 1 : -1) * (DBL_MAX / 10);
  int lid = -1, li = -1, lj = -1, lk = -1;
  for (int l = 1; l <= t->nlvl; l++)
    for (int q = 0; q < LVL_N(t, leaves, l); q++) {
      const int id = LVL_AT(t, leaves, l, q);
      const double *c = ccb(t, iv, id);
      /* maxloc / minloc: the first extremum, i fastest */
      double bv = 0;
      int bi = 0, bj = 0, bk = 0, first = 1;
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc; i++) {
            double x = c[IX(t, i, j, k)];
            if (op == AFH_RED_MAXABS) x = fabs(x);
            if (first || (is_min ? x < bv : x > bv)) bv = x, bi = i, bj = j, bk = k, first = 0;
          }
      const double nv = is_min ? fmin(bv, val) : fmax(bv, val);
      if (fabs(nv - val) > 0) val = bv, lid = id, li = bi, lj = bj, lk = bk;
    }
  *out = val;
  if (loc) loc[0] = lid, loc[1] = li, loc[2] = lj, loc[3] = lk;
  return hook(t, is_min ? AFH_HOOK_MIN : AFH_HOOK_MAX, 0, iv, out, 1);
}

/* ------------------------------------------------------------ multigrid */

/* stencil_apply_357, m_af_stencil.f90:445-457 (constant stencil) */
static void apply_357(afh_tree *t, int id, const double *cf, int iv,
                      int i_out) {
  double *x = ccb(t, iv, id), *o = ccb(t, i_out, id);
  int nc = t->nc;
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++)
        o[IX(t, i, j, k)] =
            cf[0] * x[IX(t, i, j, k)] + cf[1] * x[IX(t, i - 1, j, k)] +
            cf[2] * x[IX(t, i + 1, j, k)] + cf[3] * x[IX(t, i, j - 1, k)] +
            cf[4] * x[IX(t, i, j + 1, k)] + cf[5] * x[IX(t, i, j, k - 1)] +
            cf[6] * x[IX(t, i, j, k + 1)];
}

/* stencil_gsrb_357, m_af_stencil.f90:938-955 (constant stencil) */
static void gsrb_357(afh_tree *t, int id, const double *cf, int redblack,
                     int iv, int i_rhs) {
  double *x = ccb(t, iv, id), *r = ccb(t, i_rhs, id);
  double inv_c1 = 1 / cf[0];
  int nc = t->nc;
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++) {
      int i0 = 2 - ((redblack ^ (k + j)) & 1);
      for (int i = i0; i <= nc; i += 2)
        x[IX(t, i, j, k)] =
            (r[IX(t, i, j, k)] - cf[1] * x[IX(t, i - 1, j, k)] -
             cf[2] * x[IX(t, i + 1, j, k)] - cf[3] * x[IX(t, i, j - 1, k)] -
             cf[4] * x[IX(t, i, j + 1, k)] - cf[5] * x[IX(t, i, j, k - 1)] -
             cf[6] * x[IX(t, i, j, k + 1)]) *
            inv_c1;
    }
}

/* Cell (i, j, k) of a variable stencil v(7, nc, nc, nc) / bc_correction(nc^3) */
static inline size_t vix(int nc, int i, int j, int k) {
  return ((size_t)(k - 1) * nc + (size_t)(j - 1)) * nc + (size_t)(i - 1);
}

/* stencil_apply_357 with a variable stencil, then - bc_correction
 * (m_af_stencil.f90:459-475) */
static void apply_357_var(afh_tree *t, int id, const double *v, const double *bcc,
                          int iv, int i_out) {
  double *x = ccb(t, iv, id), *o = ccb(t, i_out, id);
  int nc = t->nc;
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++) {
        const double *c = v + 7 * vix(nc, i, j, k);
        o[IX(t, i, j, k)] =
            c[0] * x[IX(t, i, j, k)] + c[1] * x[IX(t, i - 1, j, k)] +
            c[2] * x[IX(t, i + 1, j, k)] + c[3] * x[IX(t, i, j - 1, k)] +
            c[4] * x[IX(t, i, j + 1, k)] + c[5] * x[IX(t, i, j, k - 1)] +
            c[6] * x[IX(t, i, j, k + 1)];
      }
  if (bcc)
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++)
          o[IX(t, i, j, k)] = o[IX(t, i, j, k)] - bcc[vix(nc, i, j, k)];
}

/* stencil_gsrb_357 with a variable stencil (m_af_stencil.f90:836-841,
 * 958-978): rhs + bc_correction, the red or black cells divided by c(1),
 * then rhs - bc_correction */
static void gsrb_357_var(afh_tree *t, int id, const double *v, const double *bcc,
                         int redblack, int iv, int i_rhs) {
  double *x = ccb(t, iv, id), *r = ccb(t, i_rhs, id);
  int nc = t->nc;
  if (bcc)
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++)
          r[IX(t, i, j, k)] = r[IX(t, i, j, k)] + bcc[vix(nc, i, j, k)];
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++) {
      int i0 = 2 - ((redblack ^ (k + j)) & 1);
      for (int i = i0; i <= nc; i += 2) {
        const double *c = v + 7 * vix(nc, i, j, k);
        x[IX(t, i, j, k)] =
            (r[IX(t, i, j, k)] - c[1] * x[IX(t, i - 1, j, k)] -
             c[2] * x[IX(t, i + 1, j, k)] - c[3] * x[IX(t, i, j - 1, k)] -
             c[4] * x[IX(t, i, j + 1, k)] - c[5] * x[IX(t, i, j, k - 1)] -
             c[6] * x[IX(t, i, j, k + 1)]) /
            c[0];
      }
    }
  if (bcc)
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++)
          r[IX(t, i, j, k)] = r[IX(t, i, j, k)] - bcc[vix(nc, i, j, k)];
}

/* stencil_prolong_248 with add = .true., m_af_stencil.f90:749-771 */
static void prolong_248_add(afh_tree *t, int p_id, int c_id, int iv,
                            int iv_to) {
  static const double w[8] = {27 / 64.0, 9 / 64.0, 9 / 64.0, 3 / 64.0,
                              9 / 64.0,  3 / 64.0, 3 / 64.0, 1 / 64.0};
  int nc = t->nc, off[3];
  child_offset(t, c_id, 0, off);
  double *p = ccb(t, iv, p_id), *c = ccb(t, iv_to, c_id);
  for (int k = 1; k <= nc; k++) {
    int k1 = off[2] + ((k + 1) >> 1), k2 = k1 + 1 - 2 * (k & 1);
    for (int j = 1; j <= nc; j++) {
      int j1 = off[1] + ((j + 1) >> 1), j2 = j1 + 1 - 2 * (j & 1);
      for (int i = 1; i <= nc; i++) {
        int i1 = off[0] + ((i + 1) >> 1), i2 = i1 + 1 - 2 * (i & 1);
        c[IX(t, i, j, k)] =
            c[IX(t, i, j, k)] + w[0] * p[IX(t, i1, j1, k1)] +
            w[1] * p[IX(t, i2, j1, k1)] + w[2] * p[IX(t, i1, j2, k1)] +
            w[3] * p[IX(t, i2, j2, k1)] + w[4] * p[IX(t, i1, j1, k2)] +
            w[5] * p[IX(t, i2, j1, k2)] + w[6] * p[IX(t, i1, j2, k2)] +
            w[7] * p[IX(t, i2, j2, k2)];
      }
    }
  }
}

static double *lvl_coeffs(afh_mg *mg, int lvl) { return mg->lvl_c + 7 * (lvl - 1); }

/* mg_auto_op (af_stencil_apply_box with the operator key): the box's
 * electrode stencil if it has one, else the level's constant stencil */
static void apply_box(afh_mg *mg, int id, int iv, int i_out) {
  afh_tree *t = mg->t;
  if (mg->vst[id - 1])
    apply_357_var(t, id, mg->vst[id - 1], mg->vbc[id - 1], iv, i_out);
  else
    apply_357(t, id, lvl_coeffs(mg, B(t, id)->lvl), iv, i_out);
}

/* mg_auto_gsrb (af_stencil_gsrb_box with the operator key) */
static void gsrb_box(afh_mg *mg, int id, int redblack) {
  afh_tree *t = mg->t;
  if (mg->vst[id - 1])
    gsrb_357_var(t, id, mg->vst[id - 1], mg->vbc[id - 1], redblack, mg->d.i_phi,
                 mg->d.i_rhs);
  else
    gsrb_357(t, id, lvl_coeffs(mg, B(t, id)->lvl), redblack, mg->d.i_phi,
             mg->d.i_rhs);
}

/* residual_box, m_af_multigrid.f90:801-810 */
static void residual_box(afh_mg *mg, int id) {
  afh_tree *t = mg->t;
  int nc = t->nc;
  apply_box(mg, id, mg->d.i_phi, mg->d.i_tmp);
  double *o = ccb(t, mg->d.i_tmp, id), *r = ccb(t, mg->d.i_rhs, id);
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++)
        o[IX(t, i, j, k)] = r[IX(t, i, j, k)] - o[IX(t, i, j, k)];
}

/* gsrb_boxes, m_af_multigrid.f90:648-687 */
int32_t afo_mg_gsrb_boxes(afh_mg *mg, int32_t lvl, int32_t up) {
  afh_tree *t = mg->t;
  int n_cycle = up ? mg->d.n_cycle_up : mg->d.n_cycle_down;
  int nid = LVL_N(t, ids, lvl);
  for (int n = 1; n <= 2 * n_cycle; n++) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nid; i++) gsrb_box(mg, LVL_AT(t, ids, lvl, i), n);
    int use_corners = up && n == 2 * n_cycle;
    if (gc_lvl(t, lvl, mg->d.i_phi, use_corners)) return AFH_ERR_STATE;
  }
  return AFH_OK;
}

/* update_coarse, m_af_multigrid.f90:691-738 */
int32_t afo_mg_update_coarse(afh_mg *mg, int32_t lvl) {
  afh_tree *t = mg->t;
  int nc = t->nc, nid = LVL_N(t, ids, lvl);
  size_t bsz = t->bsz;
  int i_phi = mg->d.i_phi, i_tmp = mg->d.i_tmp, i_rhs = mg->d.i_rhs;
#pragma omp parallel
  {
    double *save = malloc(sizeof(double) * bsz);
#pragma omp for schedule(static)
    for (int i = 0; i < nid; i++) {
      int id = LVL_AT(t, ids, lvl, i), p_id = B(t, id)->parent;
      memcpy(save, ccb(t, i_tmp, id), sizeof(double) * bsz);
      residual_box(mg, id);
      restrict_box(t, id, p_id, i_tmp);
      restrict_box(t, id, p_id, i_phi);
      /* restore interior of tmp (ghosts were untouched) */
      memcpy(ccb(t, i_tmp, id), save, sizeof(double) * bsz);
    }
    free(save);
  }
  (void)nc;
  if (hook(t, AFH_HOOK_RESTRICT, lvl, i_phi, NULL, 0) ||
      hook(t, AFH_HOOK_RESTRICT, lvl, i_tmp, NULL, 0) ||
      gc_lvl(t, lvl - 1, i_phi, 1))
    return AFH_ERR_STATE;
  int np = LVL_N(t, parents, lvl - 1);
#pragma omp parallel for schedule(static)
  for (int i = 0; i < np; i++) {
    int id = LVL_AT(t, parents, lvl - 1, i);
    apply_box(mg, id, i_phi, i_rhs);
    double *r = ccb(t, i_rhs, id), *tm = ccb(t, i_tmp, id), *p = ccb(t, i_phi, id);
    for (size_t q = 0; q < bsz; q++) r[q] = r[q] + tm[q];
    for (size_t q = 0; q < bsz; q++) tm[q] = p[q];
  }
  return AFH_OK;
}

/* correct_children, m_af_multigrid.f90:624-646 (correct children of the
 * parents of level lvl-1, i.e. boxes of level lvl) */
int32_t afo_mg_correct_children(afh_mg *mg, int32_t lvl) {
  afh_tree *t = mg->t;
  int np = LVL_N(t, parents, lvl - 1);
  size_t bsz = t->bsz;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < np; i++) {
    int id = LVL_AT(t, parents, lvl - 1, i);
    double *tm = ccb(t, mg->d.i_tmp, id), *p = ccb(t, mg->d.i_phi, id);
    for (size_t q = 0; q < bsz; q++) tm[q] = p[q] - tm[q];
    for (int c = 0; c < 8; c++) {
      int cid = B(t, id)->children[c];
      if (cid == 0) continue;
      prolong_248_add(t, id, cid, mg->d.i_tmp, mg->d.i_phi);
    }
  }
  return AFH_OK;
}


/* ---- coarse-grid solver (OUR algorithm; the reference calls HYPRE PFMG,
 * absent from the snapshot). The level-1 grid (coarse_grid_size cells) is
 * solved by V(2,2) multigrid cycles with red-black Gauss-Seidel, boundary
 * conditions folded into the operator exactly as stencil_handle_boundaries /
 * coarse_solver_set_rhs_phi do (m_coarse_solver.f90:286-338, 442-491),
 * 8-cell average restriction and trilinear (27,9,9,3,9,3,3,1)/64
 * prolongation with ghost values reflected through the homogeneous BCs.
 * The HIP library implements the same arithmetic in the same order. */
#define GIX(mg, m, i, j, k)                                                   \
  ((((size_t)(k)) * ((mg)->dims[m][1] + 2) + (size_t)(j)) *                   \
       ((mg)->dims[m][0] + 2) +                                               \
   (size_t)(i))

/* Folded diagonal of a cell: depends only on which grid faces the cell
 * touches (class = 2 bits per dimension: at low face, at high face). The
 * table (diag, 1/diag) per class is built once per solve. */
static inline int cs_class(afh_mg *mg, int m, int i, int j, int k) {
  int idx[3] = {i, j, k}, c = 0;
  for (int d = 0; d < 3; d++) {
    c |= (idx[d] == 1) << (2 * d);
    c |= (idx[d] == mg->dims[m][d]) << (2 * d + 1);
  }
  return c;
}

static void cs_build_table(afh_mg *mg) {
  const afh_bc *bc = mg->t->meth[mg->d.i_phi].bc;
  for (int m = 0; m < mg->n_mg; m++)
    for (int c = 0; c < 64; c++) {
      double d = mg->cdiag[m];
      for (int nb = 1; nb <= 6; nb++) {
        int dd = nb_dim(nb);
        int at = nb_low(nb) ? (c >> (2 * dd)) & 1 : (c >> (2 * dd + 1)) & 1;
        if (!at) continue;
        if (bc[nb - 1].type == AFH_BC_DIRICHLET) d = d - mg->hc[m][dd];
        else d = d + mg->hc[m][dd];
      }
      mg->dtab[m][c][0] = d;
      mg->dtab[m][c][1] = 1 / d;
    }
}

static inline double cs_diag(afh_mg *mg, int m, int i, int j, int k) {
  return mg->dtab[m][cs_class(mg, m, i, j, k)][0];
}
static inline double cs_inv_diag(afh_mg *mg, int m, int i, int j, int k) {
  return mg->dtab[m][cs_class(mg, m, i, j, k)][1];
}

/* one red-black half sweep on MG level m */
static void cs_gsrb(afh_mg *mg, int m, int n) {
  double *u = mg->u[m], *f = mg->f[m];
  int nx = mg->dims[m][0], ny = mg->dims[m][1], nz = mg->dims[m][2];
  const double *h = mg->hc[m];
  for (int k = 1; k <= nz; k++)
    for (int j = 1; j <= ny; j++) {
      int i0 = 2 - ((n ^ (k + j)) & 1);
      for (int i = i0; i <= nx; i += 2) {
        double s = f[GIX(mg, m, i, j, k)];
        if (i > 1) s = s - h[0] * u[GIX(mg, m, i - 1, j, k)];
        if (i < nx) s = s - h[0] * u[GIX(mg, m, i + 1, j, k)];
        if (j > 1) s = s - h[1] * u[GIX(mg, m, i, j - 1, k)];
        if (j < ny) s = s - h[1] * u[GIX(mg, m, i, j + 1, k)];
        if (k > 1) s = s - h[2] * u[GIX(mg, m, i, j, k - 1)];
        if (k < nz) s = s - h[2] * u[GIX(mg, m, i, j, k + 1)];
        u[GIX(mg, m, i, j, k)] = s * cs_inv_diag(mg, m, i, j, k);
      }
    }
}

/* f - A u at cell (i, j, k) of MG level m (cs_residual_restrict's order) */
static double cs_res_cell(afh_mg *mg, int m, int i, int j, int k) {
  const double *u = mg->u[m];
  int nx = mg->dims[m][0], ny = mg->dims[m][1], nz = mg->dims[m][2];
  const double *h = mg->hc[m];
  double a = cs_diag(mg, m, i, j, k) * u[GIX(mg, m, i, j, k)];
  if (i > 1) a = a + h[0] * u[GIX(mg, m, i - 1, j, k)];
  if (i < nx) a = a + h[0] * u[GIX(mg, m, i + 1, j, k)];
  if (j > 1) a = a + h[1] * u[GIX(mg, m, i, j - 1, k)];
  if (j < ny) a = a + h[1] * u[GIX(mg, m, i, j + 1, k)];
  if (k > 1) a = a + h[2] * u[GIX(mg, m, i, j, k - 1)];
  if (k < nz) a = a + h[2] * u[GIX(mg, m, i, j, k + 1)];
  return mg->f[m][GIX(mg, m, i, j, k)] - a;
}

/* HYPRE's hypre_StructInnerProd of the residual (res = 1) or of the rhs
 * with itself on the level-1 grid, cells i fastest (the device sums in
 * another order: equal to rounding, which only matters for a stopping test
 * that falls within rounding of the tolerance) */
static double cs_norm2(afh_mg *mg, int res) {
  double s = 0.0;
  for (int k = 1; k <= mg->dims[0][2]; k++)
    for (int j = 1; j <= mg->dims[0][1]; j++)
      for (int i = 1; i <= mg->dims[0][0]; i++) {
        const double v = res ? cs_res_cell(mg, 0, i, j, k) : mg->f[0][GIX(mg, 0, i, j, k)];
        s = s + v * v;
      }
  return s;
}

/* residual on level m restricted (8-cell mean) into f[m+1]; u[m+1] = 0 */
static void cs_residual_restrict(afh_mg *mg, int m) {
  double *u = mg->u[m], *f = mg->f[m], *r = mg->r[m];
  int nx = mg->dims[m][0], ny = mg->dims[m][1], nz = mg->dims[m][2];
  const double *h = mg->hc[m];
  for (int k = 1; k <= nz; k++)
    for (int j = 1; j <= ny; j++)
      for (int i = 1; i <= nx; i++) {
        double a = cs_diag(mg, m, i, j, k) * u[GIX(mg, m, i, j, k)];
        if (i > 1) a = a + h[0] * u[GIX(mg, m, i - 1, j, k)];
        if (i < nx) a = a + h[0] * u[GIX(mg, m, i + 1, j, k)];
        if (j > 1) a = a + h[1] * u[GIX(mg, m, i, j - 1, k)];
        if (j < ny) a = a + h[1] * u[GIX(mg, m, i, j + 1, k)];
        if (k > 1) a = a + h[2] * u[GIX(mg, m, i, j, k - 1)];
        if (k < nz) a = a + h[2] * u[GIX(mg, m, i, j, k + 1)];
        r[GIX(mg, m, i, j, k)] = f[GIX(mg, m, i, j, k)] - a;
      }
  int c = m + 1;
  double *fc = mg->f[c], *uc = mg->u[c];
  for (int k = 1; k <= mg->dims[c][2]; k++)
    for (int j = 1; j <= mg->dims[c][1]; j++)
      for (int i = 1; i <= mg->dims[c][0]; i++) {
        int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
        double s = r[GIX(mg, m, fi, fj, fk)];
        s += r[GIX(mg, m, fi + 1, fj, fk)];
        s += r[GIX(mg, m, fi, fj + 1, fk)];
        s += r[GIX(mg, m, fi + 1, fj + 1, fk)];
        s += r[GIX(mg, m, fi, fj, fk + 1)];
        s += r[GIX(mg, m, fi + 1, fj, fk + 1)];
        s += r[GIX(mg, m, fi, fj + 1, fk + 1)];
        s += r[GIX(mg, m, fi + 1, fj + 1, fk + 1)];
        fc[GIX(mg, c, i, j, k)] = 0.125 * s;
        uc[GIX(mg, c, i, j, k)] = 0.0;
      }
}

/* value of u[c] at (i,j,k), reflecting through homogeneous BCs outside */
static inline double cs_refl(afh_mg *mg, int c, int i, int j, int k) {
  const afh_bc *bc = mg->t->meth[mg->d.i_phi].bc;
  double s = 1.0;
  int idx[3] = {i, j, k};
  for (int d = 0; d < 3; d++) {
    if (idx[d] < 1) {
      idx[d] = 1;
      if (bc[2 * d].type == AFH_BC_DIRICHLET) s = -s;
    } else if (idx[d] > mg->dims[c][d]) {
      idx[d] = mg->dims[c][d];
      if (bc[2 * d + 1].type == AFH_BC_DIRICHLET) s = -s;
    }
  }
  return s * mg->u[c][GIX(mg, c, idx[0], idx[1], idx[2])];
}

static void cs_prolong_add(afh_mg *mg, int m) {
  static const double w[8] = {27 / 64.0, 9 / 64.0, 9 / 64.0, 3 / 64.0,
                              9 / 64.0,  3 / 64.0, 3 / 64.0, 1 / 64.0};
  int c = m + 1;
  double *u = mg->u[m];
  for (int k = 1; k <= mg->dims[m][2]; k++) {
    int k1 = (k + 1) >> 1, k2 = k1 + 1 - 2 * (k & 1);
    for (int j = 1; j <= mg->dims[m][1]; j++) {
      int j1 = (j + 1) >> 1, j2 = j1 + 1 - 2 * (j & 1);
      for (int i = 1; i <= mg->dims[m][0]; i++) {
        int i1 = (i + 1) >> 1, i2 = i1 + 1 - 2 * (i & 1);
        u[GIX(mg, m, i, j, k)] =
            u[GIX(mg, m, i, j, k)] + w[0] * cs_refl(mg, c, i1, j1, k1) +
            w[1] * cs_refl(mg, c, i2, j1, k1) + w[2] * cs_refl(mg, c, i1, j2, k1) +
            w[3] * cs_refl(mg, c, i2, j2, k1) + w[4] * cs_refl(mg, c, i1, j1, k2) +
            w[5] * cs_refl(mg, c, i2, j1, k2) + w[6] * cs_refl(mg, c, i1, j2, k2) +
            w[7] * cs_refl(mg, c, i2, j2, k2);
      }
    }
  }
}

static void cs_cycle(afh_mg *mg, int m) {
  if (m == mg->n_mg - 1) {
    for (int it = 0; it < AFH_CS_BOTTOM_SWEEPS; it++) {
      cs_gsrb(mg, m, 1);
      cs_gsrb(mg, m, 2);
    }
    return;
  }
  for (int s = 0; s < 2; s++) {
    cs_gsrb(mg, m, 1);
    cs_gsrb(mg, m, 2);
  }
  cs_residual_restrict(mg, m);
  cs_cycle(mg, m + 1);
  cs_prolong_add(mg, m);
  for (int s = 0; s < 2; s++) {
    cs_gsrb(mg, m, 1);
    cs_gsrb(mg, m, 2);
  }
}

/* ---- AFH_COARSE_DIRECT: exact solve of the folded level-1 problem.
 * The folded operator is separable, A = Tx (x) I (x) I + I (x) Ty (x) I +
 * I (x) I (x) Tz - lambda, with T_d = h_d tridiag(1, -2, 1) whose end
 * diagonals are -h_d (Neumann face) or -3 h_d (Dirichlet face), exactly the
 * folding of stencil_handle_boundaries. Each T_d is diagonalised by a
 * cosine / sine basis (DCT-II for Neumann-Neumann, DST-II for
 * Dirichlet-Dirichlet, DCT-IV / DST-IV for mixed ends):
 *   v_p(i) = cos|sin(theta_p (i + 1/2)) / norm,  eig_p = h (2 cos theta_p - 2)
 * so u = Q (Lambda^-1 (Q^T f)), with Q^T and Q applied one dimension at a
 * time as dense n x n products in a fixed summation order (the HIP library
 * evaluates the same sums in the same order). */
void afo_cs_direct_tables(int n, int bc_lo, int bc_hi, double h, double *q,
                          double *e) {
  const int dlo = bc_lo == AFH_BC_DIRICHLET, dhi = bc_hi == AFH_BC_DIRICHLET;
  const double pi = 3.14159265358979323846;
  for (int p = 0; p < n; p++) {
    double th;
    if (dlo == dhi) th = pi * (p + dlo) / n;   /* NN: p, DD: p + 1 */
    else th = pi * (p + 0.5) / n;              /* mixed */
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

static void cs_direct_build(afh_mg *mg) {
  const afh_bc *bc = mg->t->meth[mg->d.i_phi].bc;
  for (int d = 0; d < 3; d++) {
    int n = mg->dims[0][d];
    afo_cs_direct_tables(n, bc[2 * d].type, bc[2 * d + 1].type, mg->hc[0][d],
                         mg->q[d], mg->e[d]);
  }
  for (int q = 0; q < 6; q++) mg->q_bc[q] = bc[q].type;
}

/* one 1-D transform along dim d: out(c) = sum_p coef(c, p) in(.. p ..),
 * coef = Q[p][c] (forward, Q^T) or Q[c][p] (inverse); in/out with a ghost
 * layer when *_halo. With `div`, the forward result is divided by the
 * eigenvalue sum (zero modes set to 0). */
static void cs_transform(afh_mg *mg, const double *in, int in_halo, double *out,
                         int out_halo, int d, int fwd, int div) {
  const int nx = mg->dims[0][0], ny = mg->dims[0][1], nz = mg->dims[0][2];
  const int n = mg->dims[0][d];
  const double *q = mg->q[d];
  const double lam = mg->d.helmholtz_lambda;
#pragma omp parallel for schedule(static)
  for (int k = 0; k < nz; k++)
    for (int j = 0; j < ny; j++)
      for (int i = 0; i < nx; i++) {
        int c[3] = {i, j, k};
        const int co = c[d];
        double s = 0.0;
        for (int p = 0; p < n; p++) {
          c[d] = p;
          size_t x = in_halo ? (((size_t)c[2] + 1) * (ny + 2) + c[1] + 1) * (nx + 2) + c[0] + 1
                             : ((size_t)c[2] * ny + c[1]) * nx + c[0];
          const double cf = fwd ? q[p * n + co] : q[co * n + p];
          s = s + cf * in[x];
        }
        if (div) {
          const double den = ((mg->e[0][i] + mg->e[1][j]) + mg->e[2][k]) - lam;
          s = den != 0.0 ? s / den : 0.0;
        }
        size_t o = out_halo ? (((size_t)k + 1) * (ny + 2) + j + 1) * (nx + 2) + i + 1
                            : ((size_t)k * ny + j) * nx + i;
        out[o] = s;
      }
}

static void cs_direct_solve(afh_mg *mg) {
  const afh_bc *bc = mg->t->meth[mg->d.i_phi].bc;
  for (int q = 0; q < 6; q++)
    if (mg->q_bc[q] != bc[q].type) {
      cs_direct_build(mg);
      break;
    }
  cs_transform(mg, mg->f[0], 1, mg->w1, 0, 0, 1, 0);
  cs_transform(mg, mg->w1, 0, mg->w2, 0, 1, 1, 0);
  cs_transform(mg, mg->w2, 0, mg->w1, 0, 2, 1, 1);
  cs_transform(mg, mg->w1, 0, mg->w2, 0, 2, 0, 0);
  cs_transform(mg, mg->w2, 0, mg->w1, 0, 1, 0, 0);
  cs_transform(mg, mg->w1, 0, mg->u[0], 1, 0, 0, 0);
}

/* Fortran spacing(x): the distance from |x| to the next larger double */
static double f_spacing(double x) {
  x = fabs(x);
  if (x == 0) return 2.2250738585072014e-308; /* tiny(1.0_dp) */
  int e;
  frexp(x, &e);
  return ldexp(1.0, e - 53);
}

/* Level-1 solve with electrode stencils (OUR algorithm; HYPRE is given the
 * LSF stencils in the reference, m_coarse_solver.f90:286-338): red-black
 * Gauss-Seidel pairs with the boxes' own stencils and a level ghost fill
 * after each half-sweep, until phi is stationary (max change <= 4 spacing
 * of max |phi|, after at least 11 pairs) -- the golden harness' exact
 * solve -- then the level's ghost cells with corners. */
/* The one-box electrode level-1 solve as a dense product (afh_cs_direct.h,
 * the library's AFH_CS_ELEC_DIRECT, default on): a level 1 of one box of
 * 8^3 with an electrode stencil and six physical faces. The inverse of the
 * last operator is kept (a regrid makes new multigrids with the same
 * level-1 stencil). Returns 1 when it does not apply (the iteration runs). */
static struct {
  double *v, *ainv, *g;
  afh_bc bc[6];
  double dr[3];
  int valid, singular;
} csd_last;
/* thread ranks (tests/test_dist_driver.py) solve level 1 concurrently
 * through ctypes, which releases the GIL: the cache's lookup, build and use
 * are one critical section (the device library's csd_mu) */
static pthread_mutex_t csd_mu = PTHREAD_MUTEX_INITIALIZER;

static int solve_coarse_direct(afh_mg *mg) {
  afh_tree *t = mg->t;
  const char *env = getenv("AFH_CS_ELEC_DIRECT");
  /* (a sharded tree too: level 1 is replicated, every rank solves it alike
     without a collective) */
  if ((env && !atoi(env)) || t->nc != AFH_CSD_NC || LVL_N(t, ids, 1) != 1) return 1;
  const int id = LVL_AT(t, ids, 1, 0);
  const afh_box_meta *m = B(t, id);
  if (!mg->vst[id - 1]) return 1;
  for (int q = 0; q < 6; q++)
    if (m->neighbors[q] >= 0) return 1;
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  const size_t n = AFH_CSD_N;
  pthread_mutex_lock(&csd_mu);
  if (!csd_last.valid || memcmp(csd_last.v, mg->vst[id - 1], sizeof(double) * 7 * n) ||
      memcmp(csd_last.bc, bc, sizeof csd_last.bc) ||
      memcmp(csd_last.dr, m->dr, sizeof csd_last.dr)) {
    if (!csd_last.v) {
      csd_last.v = malloc(sizeof(double) * 7 * n);
      csd_last.ainv = malloc(sizeof(double) * n * n);
      csd_last.g = malloc(sizeof(double) * n);
    }
    memcpy(csd_last.v, mg->vst[id - 1], sizeof(double) * 7 * n);
    memcpy(csd_last.bc, bc, sizeof csd_last.bc);
    memcpy(csd_last.dr, m->dr, sizeof csd_last.dr);
    double *work = malloc(sizeof(double) * 2 * n * n);
    csd_last.singular = afh_csd_build(csd_last.v, csd_last.bc, csd_last.dr, csd_last.ainv,
                                      csd_last.g, work);
    free(work);
    csd_last.valid = 1;
  }
  if (csd_last.singular) {
    pthread_mutex_unlock(&csd_mu);
    return 1;
  }
  double b[AFH_CSD_N];
  const double *r = ccb(t, mg->d.i_rhs, id), *bcc = mg->vbc[id - 1];
  double *x = ccb(t, mg->d.i_phi, id);
  const int nc = AFH_CSD_NC;
  for (int e = 0; e < (int)n; e++) {
    const int i = e % nc + 1, j = (e / nc) % nc + 1, k = e / (nc * nc) + 1;
    double rv = r[IX(t, i, j, k)];
    if (bcc) rv = rv + bcc[e];
    b[e] = rv - csd_last.g[e];
  }
#pragma omp parallel for schedule(static)
  for (int row = 0; row < (int)n; row++) {
    double acc = 0.0;
    for (size_t c = 0; c < n; c++) acc = acc + csd_last.ainv[c * n + row] * b[c];
    const int i = row % nc + 1, j = (row / nc) % nc + 1, k = row / (nc * nc) + 1;
    x[IX(t, i, j, k)] = acc;
  }
  pthread_mutex_unlock(&csd_mu);
  mg->cs_iters = 1;
  return gc_lvl(t, 1, mg->d.i_phi, 1) ? -1 : 0;
}

static int32_t solve_coarse_gs(afh_mg *mg) {
  afh_tree *t = mg->t;
  int nc = t->nc, nid = LVL_N(t, ids, 1);
  size_t bsz = t->bsz;
  {
    const int rc = solve_coarse_direct(mg);
    if (rc == 0) return AFH_OK;
    if (rc < 0) return AFH_ERR_STATE;
  }
  double *old = malloc(sizeof(double) * bsz * (nid > 0 ? nid : 1));
  for (int it = 1; it <= 200000; it++) {
    for (int q = 0; q < nid; q++)
      memcpy(old + q * bsz, ccb(t, mg->d.i_phi, LVL_AT(t, ids, 1, q)),
             sizeof(double) * bsz);
    for (int n = 1; n <= 2; n++) {
      for (int q = 0; q < nid; q++) gsrb_box(mg, LVL_AT(t, ids, 1, q), n);
      if (gc_lvl(t, 1, mg->d.i_phi, 0)) return free(old), AFH_ERR_STATE;
    }
    double diff = 0, vmax = 0;
    for (int q = 0; q < nid; q++) {
      const double *p = ccb(t, mg->d.i_phi, LVL_AT(t, ids, 1, q)), *o = old + q * bsz;
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc; i++) {
            size_t c = IX(t, i, j, k);
            diff = fmax(diff, fabs(p[c] - o[c]));
            vmax = fmax(vmax, fabs(p[c]));
          }
    }
    if (hook(t, AFH_HOOK_MAX, 1, mg->d.i_phi, &diff, 1) ||
        hook(t, AFH_HOOK_MAX, 1, mg->d.i_phi, &vmax, 1))
      return free(old), AFH_ERR_STATE;
    if (diff <= 4 * f_spacing(vmax) && it > 10) break;
  }
  free(old);
  return gc_lvl(t, 1, mg->d.i_phi, 1) ? AFH_ERR_STATE : AFH_OK;
}

/* ---- AFH_COARSE_PFMG: the reference's HYPRE StructPFMG, restated
 * (afh_pfmg.h has the algorithm and its sources; the hierarchy is built
 * there). The level operations below fix one evaluation order, which the
 * device kernel (afh_mg.hip k_cs_pfmg) repeats, so the two agree bitwise. */

/* weighted Jacobi on level l (point_relax.c): zero guess x = w b / a_c;
 * else t = (b - sum_{s != c} a_s x_s) / a_c, x = (1 - w) x + w t */
static void pf_relax(afh_mg *mg, int l, int zero) {
  const afh_pfmg *h = &mg->pf;
  const int nx = h->n[l][0], ny = h->n[l][1], nz = h->n[l][2];
  const double w = h->w[l];
  double *x = mg->pf_x, *t = mg->pf_r;
  const double *b = mg->pf_b;
  for (int k = 1; k <= nz; k++)
    for (int j = 1; j <= ny; j++)
      for (int i = 1; i <= nx; i++) {
        const size_t p = afh_pfmg_ix(h, l, i, j, k);
        const double *A = h->A + AFH_PFMG_S * p;
        if (zero) {
          double v = b[p] / A[AFH_PFMG_C];
          if (w != 1.0) v = w * v;
          t[p] = v;
          continue;
        }
        double v = b[p];
        for (int s = 0; s < AFH_PFMG_S; s++) {
          if (s == AFH_PFMG_C) continue;
          const int ii = i + s % 3 - 1, jj = j + (s / 3) % 3 - 1, kk = k + s / 9 - 1;
          if (ii < 1 || ii > nx || jj < 1 || jj > ny || kk < 1 || kk > nz) continue;
          v = v - A[s] * x[afh_pfmg_ix(h, l, ii, jj, kk)];
        }
        t[p] = v / A[AFH_PFMG_C];
      }
  for (size_t p = h->off[l]; p < h->off[l + 1]; p++) {
    if (zero || w == 1.0) x[p] = t[p];
    else x[p] = (1.0 - w) * x[p] + w * t[p];
  }
}

/* r = b - A x on level l */
static void pf_residual(afh_mg *mg, int l) {
  const afh_pfmg *h = &mg->pf;
  const int nx = h->n[l][0], ny = h->n[l][1], nz = h->n[l][2];
  for (int k = 1; k <= nz; k++)
    for (int j = 1; j <= ny; j++)
      for (int i = 1; i <= nx; i++) {
        const size_t p = afh_pfmg_ix(h, l, i, j, k);
        const double *A = h->A + AFH_PFMG_S * p;
        double a = 0.0;
        for (int s = 0; s < AFH_PFMG_S; s++) {
          const int ii = i + s % 3 - 1, jj = j + (s / 3) % 3 - 1, kk = k + s / 9 - 1;
          if (ii < 1 || ii > nx || jj < 1 || jj > ny || kk < 1 || kk > nz) continue;
          a = a + A[s] * mg->pf_x[afh_pfmg_ix(h, l, ii, jj, kk)];
        }
        mg->pf_r[p] = mg->pf_b[p] - a;
      }
}

/* r.r (or b.b) on level 0: AFH_PFMG_NPART strided partial sums, then a
 * pairwise tree (the device's wave reduction, afh_pfmg_dev.h pf_dot) */
#define AFH_PFMG_NPART 64
static double pf_dot(afh_mg *mg, const double *v) {
  double part[AFH_PFMG_NPART];
  const size_t n = mg->pf.off[1];
  for (int q = 0; q < AFH_PFMG_NPART; q++) {
    double s = 0.0;
    for (size_t p = q; p < n; p += AFH_PFMG_NPART) s = s + v[p] * v[p];
    part[q] = s;
  }
  for (int st = AFH_PFMG_NPART / 2; st > 0; st >>= 1)
    for (int q = 0; q < st; q++) part[q] = part[q] + part[q + st];
  return part[0];
}

/* b_{l+1} = R r_l (semi_restrict.c; R = P^T) */
static void pf_restrict(afh_mg *mg, int l) {
  const afh_pfmg *h = &mg->pf;
  const int cd = h->cdir[l], *nf = h->n[l], *nc = h->n[l + 1];
  for (int k = 1; k <= nc[2]; k++)
    for (int j = 1; j <= nc[1]; j++)
      for (int i = 1; i <= nc[0]; i++) {
        int f[3] = {i, j, k};
        f[cd] = 2 * f[cd];
        const size_t fp = afh_pfmg_ix(h, l, f[0], f[1], f[2]);
        double v = mg->pf_r[fp];
        f[cd] -= 1;
        {
          const size_t q = afh_pfmg_ix(h, l, f[0], f[1], f[2]);
          v = v + h->P[2 * q + 1] * mg->pf_r[q];
        }
        f[cd] += 2;
        if (f[cd] <= nf[cd]) {
          const size_t q = afh_pfmg_ix(h, l, f[0], f[1], f[2]);
          v = v + h->P[2 * q] * mg->pf_r[q];
        }
        mg->pf_b[afh_pfmg_ix(h, l + 1, i, j, k)] = v;
      }
}

/* x_l += P x_{l+1} (semi_interp.c) */
static void pf_interp_add(afh_mg *mg, int l) {
  const afh_pfmg *h = &mg->pf;
  const int cd = h->cdir[l], *nf = h->n[l];
  for (int k = 1; k <= nf[2]; k++)
    for (int j = 1; j <= nf[1]; j++)
      for (int i = 1; i <= nf[0]; i++) {
        const int f[3] = {i, j, k};
        const size_t p = afh_pfmg_ix(h, l, i, j, k);
        int c[3] = {i, j, k};
        double e;
        if (!(f[cd] & 1)) {
          c[cd] = f[cd] / 2;
          e = mg->pf_x[afh_pfmg_ix(h, l + 1, c[0], c[1], c[2])];
        } else {
          e = 0.0;
          if (f[cd] >= 3) {
            c[cd] = (f[cd] - 1) / 2;
            e = h->P[2 * p] * mg->pf_x[afh_pfmg_ix(h, l + 1, c[0], c[1], c[2])];
          }
          if (f[cd] + 1 <= nf[cd]) {
            c[cd] = (f[cd] + 1) / 2;
            e = e + h->P[2 * p + 1] * mg->pf_x[afh_pfmg_ix(h, l + 1, c[0], c[1], c[2])];
          }
        }
        mg->pf_x[p] = mg->pf_x[p] + e;
      }
}

/* pfmg_solve.c: returns the iteration count */
static int pf_solve(afh_mg *mg, double tol, int max_iter) {
  const afh_pfmg *h = &mg->pf;
  const int nl = h->nl;
  const double bb = pf_dot(mg, mg->pf_b);
  if (bb == 0.0) {
    for (size_t p = 0; p < h->off[1]; p++) mg->pf_x[p] = 0.0;
    return 0;
  }
  const double eps = tol * tol;
  int iters = 0;
  for (int i = 0; i < max_iter; i++) {
    pf_relax(mg, 0, 0);
    pf_residual(mg, 0);
    if (tol > 0.0) {
      const double rr = pf_dot(mg, mg->pf_r);
      if (rr / bb < eps && i > 0) break;
    }
    if (nl > 1) {
      pf_restrict(mg, 0);
      int l;
      for (l = 1; l <= nl - 2; l++) {
        if (h->active[l]) {
          pf_relax(mg, l, 1);
          pf_residual(mg, l);
        } else {
          for (size_t p = h->off[l]; p < h->off[l + 1]; p++) {
            mg->pf_x[p] = 0.0;
            mg->pf_r[p] = mg->pf_b[p];
          }
        }
        pf_restrict(mg, l);
      }
      if (h->active[l]) pf_relax(mg, l, 1);
      else
        for (size_t p = h->off[l]; p < h->off[l + 1]; p++) mg->pf_x[p] = 0.0;
      for (l = nl - 2; l >= 1; l--) {
        pf_interp_add(mg, l);
        if (h->active[l]) pf_relax(mg, l, 0);
      }
      pf_interp_add(mg, 0);
    }
    pf_relax(mg, 0, 0);
    iters = i + 1;
  }
  return iters;
}

/* coarse_solver_set_rhs_phi + hypre_set_matrix / stencil_handle_boundaries
 * (m_coarse_solver.f90:163-194, 247-284, 442-491): the folded operator of
 * every level-1 cell (the boxes' electrode stencils where present), the rhs
 * with the boundary values and the level-set term, phi as the guess; then
 * PFMG, and phi back (coarse_solver_get_phi). The hierarchy is rebuilt when
 * the folded operator changes. */
static int32_t solve_coarse_pfmg(afh_mg *mg) {
  afh_tree *t = mg->t;
  const int nc = t->nc, nid = LVL_N(t, ids, 1);
  const int nx = mg->dims[0][0], ny = mg->dims[0][1], nz = mg->dims[0][2];
  const size_t n0 = (size_t)nx * ny * nz;
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  double *a7 = malloc(sizeof(double) * 7 * n0);
  if (!a7) return fail(AFH_ERR_STATE, "pfmg: a7");
  double *b0 = malloc(sizeof(double) * n0), *x0 = malloc(sizeof(double) * n0);
  if (!b0 || !x0) return free(a7), free(b0), free(x0), fail(AFH_ERR_STATE, "pfmg: b");
  for (int q = 0; q < nid; q++) {
    const int id = LVL_AT(t, ids, 1, q);
    const afh_box_meta *m = B(t, id);
    const double *vst = mg->vst[id - 1], *vbc = mg->vbc[id - 1];
    const double *pr = ccb(t, mg->d.i_rhs, id), *pp = ccb(t, mg->d.i_phi, id);
    int o[3];
    for (int d = 0; d < 3; d++) o[d] = (m->ix[d] - 1) * nc;
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          const int e = ((k - 1) * nc + (j - 1)) * nc + (i - 1);
          const int gi[3] = {o[0] + i, o[1] + j, o[2] + k};
          const size_t g = ((size_t)(gi[2] - 1) * ny + (gi[1] - 1)) * nx + (gi[0] - 1);
          double c[7];
          if (vst) memcpy(c, vst + 7 * (size_t)e, sizeof c);
          else memcpy(c, mg->lvl_c, sizeof c);
          double rv = pr[IX(t, i, j, k)];
          for (int nb = 1; nb <= 6; nb++) {
            const int dd = nb_dim(nb);
            const int at = nb_low(nb) ? (gi[dd] == 1) : (gi[dd] == mg->dims[0][dd]);
            if (!at) continue;
            double b2r;
            if (bc[nb - 1].type == AFH_BC_DIRICHLET) {
              c[0] = c[0] - c[nb];
              b2r = -2 * c[nb];
            } else {
              c[0] = c[0] + c[nb];
              b2r = -(c[nb] * m->dr[dd]) * nb_pm(nb);
            }
            rv = rv + b2r * bc[nb - 1].value;
            c[nb] = 0.0;
          }
          if (vbc) rv = rv + vbc[e];
          memcpy(a7 + 7 * g, c, sizeof c);
          b0[g] = rv;
          x0[g] = pp[IX(t, i, j, k)];
        }
  }
  if (!mg->pf_a7 || memcmp(mg->pf_a7, a7, sizeof(double) * 7 * n0)) {
    afh_pfmg_free(&mg->pf);
    free(mg->pf_x), free(mg->pf_b), free(mg->pf_r), free(mg->pf_e);
    free(mg->pf_a7);
    mg->pf_a7 = a7;
    a7 = NULL;
    if (afh_pfmg_setup(&mg->pf, nx, ny, nz, 3, mg->pf_a7))
      return free(b0), free(x0), fail(AFH_ERR_STATE, "pfmg: setup");
    const size_t np = mg->pf.off[mg->pf.nl];
    mg->pf_x = calloc(np, sizeof(double));
    mg->pf_b = calloc(np, sizeof(double));
    mg->pf_r = calloc(np, sizeof(double));
    mg->pf_e = calloc(np, sizeof(double));
  }
  free(a7);
  memcpy(mg->pf_b, b0, sizeof(double) * n0);
  memcpy(mg->pf_x, x0, sizeof(double) * n0);
  free(b0), free(x0);
  mg->cs_iters = pf_solve(mg, mg->d.coarse_tol, mg->d.coarse_cycles);
  for (int q = 0; q < nid; q++) {
    const int id = LVL_AT(t, ids, 1, q);
    double *p = ccb(t, mg->d.i_phi, id);
    int o[3];
    for (int d = 0; d < 3; d++) o[d] = (B(t, id)->ix[d] - 1) * nc;
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          const size_t g = ((size_t)(o[2] + k - 1) * ny + (o[1] + j - 1)) * nx + (o[0] + i - 1);
          p[IX(t, i, j, k)] = mg->pf_x[g];
        }
  }
  return gc_lvl(t, 1, mg->d.i_phi, 1) ? AFH_ERR_STATE : AFH_OK;
}

int32_t afo_pfmg_probe(int32_t nx, int32_t ny, int32_t nz, const double *a7, int32_t maxl,
                       int32_t *nl, int32_t *cdir, int32_t *active, double *w) {
  afh_pfmg h;
  if (!a7 || !nl || !cdir || !active || !w || nx < 1 || ny < 1 || nz < 1)
    return fail(AFH_ERR_ARG, "afo_pfmg_probe: bad argument");
  if (afh_pfmg_setup(&h, nx, ny, nz, nz > 1 ? 3 : 2, a7)) return fail(AFH_ERR_STATE, "setup");
  *nl = h.nl;
  for (int l = 0; l < h.nl && l < maxl; l++) {
    cdir[l] = l + 1 < h.nl ? h.cdir[l] : -1;
    active[l] = h.active[l];
    w[l] = h.w[l];
  }
  afh_pfmg_free(&h);
  return AFH_OK;
}

/* The whole hierarchy of afh_pfmg_setup (tests/test_pfmg.py checks it
 * against an independent numpy statement): per level dims (3), cdir, active,
 * w; the point offsets (nl + 1); A (27 per point) and P (2 per point) of all
 * levels. Call with A = P = NULL to get *nl and *np first. */
int32_t afo_pfmg_probe_full(int32_t nx, int32_t ny, int32_t nz, const double *a7, int32_t maxl,
                            int32_t *nl, int64_t *np, int32_t *dims, int32_t *cdir,
                            int32_t *active, double *w, int64_t *off, double *A, double *P) {
  afh_pfmg h;
  if (!a7 || !nl || !np || nx < 1 || ny < 1 || nz < 1)
    return fail(AFH_ERR_ARG, "afo_pfmg_probe_full: bad argument");
  if (afh_pfmg_setup(&h, nx, ny, nz, nz > 1 ? 3 : 2, a7)) return fail(AFH_ERR_STATE, "setup");
  *nl = h.nl;
  *np = (int64_t)h.off[h.nl];
  if (h.nl > maxl) return afh_pfmg_free(&h), fail(AFH_ERR_ARG, "afo_pfmg_probe_full: maxl");
  for (int l = 0; l < h.nl; l++) {
    if (dims)
      for (int d = 0; d < 3; d++) dims[3 * l + d] = h.n[l][d];
    if (cdir) cdir[l] = l + 1 < h.nl ? h.cdir[l] : -1;
    if (active) active[l] = h.active[l];
    if (w) w[l] = h.w[l];
  }
  if (off)
    for (int l = 0; l <= h.nl; l++) off[l] = (int64_t)h.off[l];
  if (A) memcpy(A, h.A, sizeof(double) * AFH_PFMG_S * h.off[h.nl]);
  if (P) memcpy(P, h.P, sizeof(double) * 2 * h.off[h.nl]);
  afh_pfmg_free(&h);
  return AFH_OK;
}

/* The folded level-1 operator of the last PFMG solve of mg (a7: 7 per point
 * of the level-1 grid, dims nx ny nz), for the probes above */
int32_t afo_mg_pfmg_operator(afh_mg *mg, int32_t *dims, double *a7) {
  if (!mg || !dims) return fail(AFH_ERR_ARG, "afo_mg_pfmg_operator: null");
  for (int d = 0; d < 3; d++) dims[d] = mg->dims[0][d];
  if (!mg->pf_a7) return fail(AFH_ERR_STATE, "afo_mg_pfmg_operator: no PFMG solve yet");
  const size_t n0 = (size_t)mg->dims[0][0] * mg->dims[0][1] * mg->dims[0][2];
  if (a7) memcpy(a7, mg->pf_a7, sizeof(double) * 7 * n0);
  return AFH_OK;
}

/* solve_coarse_grid, m_af_multigrid.f90:266-291 */
int32_t afo_mg_solve_coarse(afh_mg *mg) {
  afh_tree *t = mg->t;
  int nc = t->nc, nid = LVL_N(t, ids, 1);
  if (mg->d.coarse_mode == AFH_COARSE_PFMG) return solve_coarse_pfmg(mg);
  for (int q = 0; q < t->nb; q++)
    if (mg->vst[q] && B(t, q + 1)->lvl == 1) return solve_coarse_gs(mg);
  const afh_bc *bc = t->meth[mg->d.i_phi].bc;
  /* coarse_solver_set_rhs_phi: gather rhs (+ BC contributions) and phi */
  for (int q = 0; q < nid; q++) {
    int id = LVL_AT(t, ids, 1, q);
    double *p = ccb(t, mg->d.i_phi, id), *r = ccb(t, mg->d.i_rhs, id);
    int o[3];
    for (int d = 0; d < 3; d++) o[d] = (B(t, id)->ix[d] - 1) * nc;
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          size_t g = GIX(mg, 0, o[0] + i, o[1] + j, o[2] + k);
          double rv = r[IX(t, i, j, k)];
          int gi[3] = {o[0] + i, o[1] + j, o[2] + k};
          for (int nb = 1; nb <= 6; nb++) {
            int dd = nb_dim(nb);
            int at = nb_low(nb) ? (gi[dd] == 1) : (gi[dd] == mg->dims[0][dd]);
            if (!at) continue;
            double cnb = mg->hc[0][dd], b2r;
            if (bc[nb - 1].type == AFH_BC_DIRICHLET) b2r = -2 * cnb;
            else b2r = -(cnb * B(t, id)->dr[dd]) * nb_pm(nb);
            rv = rv + b2r * bc[nb - 1].value;
          }
          mg->f[0][g] = rv;
          mg->u[0][g] = p[IX(t, i, j, k)];
        }
  }
  if (mg->d.coarse_mode == AFH_COARSE_DIRECT) {
    cs_direct_solve(mg);
    mg->cs_iters = 0;
  } else if (mg->d.coarse_tol > 0) {
    /* HYPRE PFMG's stopping rule (pfmg_solve: r.r / b.b < tol^2, at most
     * max_iter cycles; b = 0 gives x = 0), with our V(2,2) cycles */
    cs_build_table(mg);
    const double bb = cs_norm2(mg, 0), eps = mg->d.coarse_tol * mg->d.coarse_tol;
    int c = 0;
    if (bb == 0.0) {
      for (int k = 1; k <= mg->dims[0][2]; k++)
        for (int j = 1; j <= mg->dims[0][1]; j++)
          for (int i = 1; i <= mg->dims[0][0]; i++) mg->u[0][GIX(mg, 0, i, j, k)] = 0.0;
    } else {
      while (c < mg->d.coarse_cycles) {
        cs_cycle(mg, 0);
        c++;
        if (cs_norm2(mg, 1) / bb < eps) break;
      }
    }
    mg->cs_iters = c;
  } else {
    cs_build_table(mg);
    for (int c = 0; c < mg->d.coarse_cycles; c++) cs_cycle(mg, 0);
    mg->cs_iters = mg->d.coarse_cycles;
  }
  /* coarse_solver_get_phi */
  for (int q = 0; q < nid; q++) {
    int id = LVL_AT(t, ids, 1, q);
    double *p = ccb(t, mg->d.i_phi, id);
    int o[3];
    for (int d = 0; d < 3; d++) o[d] = (B(t, id)->ix[d] - 1) * nc;
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++)
          p[IX(t, i, j, k)] = mg->u[0][GIX(mg, 0, o[0] + i, o[1] + j, o[2] + k)];
  }
  if (gc_lvl(t, 1, mg->d.i_phi, 1)) return AFH_ERR_STATE;
  return AFH_OK;
}

/* mg_init minus HYPRE (m_af_multigrid.f90:43-109); mg_box_lpl_stencil
 * (1227-1245): c(2:7) = 1/dr^2, c(1) = -sum(c(2:)) - lambda */
int32_t afo_mg_create(afh_tree *t, const afh_mg_desc *d, afh_mg **out) {
  if (!t->meth[d->i_phi].set)
    return fail(AFH_ERR_STATE, "set cc methods (bc) for phi first");
  afh_mg *mg = calloc(1, sizeof *mg);
  mg->t = t;
  mg->d = *d;
  mg->lvl_c = malloc(sizeof(double) * 7 * t->nlvl);
  mg->vst = calloc(t->nb, sizeof(double *));
  mg->vbc = calloc(t->nb, sizeof(double *));
  mg->lsf_n = calloc(t->nb, sizeof(int));
  mg->lsf_ix = calloc(t->nb, sizeof(int32_t *));
  mg->lsf_dd = calloc(t->nb, sizeof(double *));
  mg->lsf_bv = calloc(t->nb, sizeof(double *));
  for (int l = 1; l <= t->nlvl; l++) {
    /* a box of the level (a rank of a sharded tree may compute none of its
     * boxes, but stores one) */
    int id = 0;
    for (int b = 1; b <= t->nb && !id; b++)
      if (B(t, b)->lvl == l) id = b;
    if (!id) return fail(AFH_ERR_ARG, "no box on level %d", l);
    double *c = mg->lvl_c + 7 * (l - 1);
    for (int dd = 0; dd < 3; dd++) {
      double dr = B(t, id)->dr[dd];
      double inv = 1 / (dr * dr);
      c[1 + 2 * dd] = inv;
      c[2 + 2 * dd] = inv;
    }
    double s = c[1];
    for (int q = 2; q < 7; q++) s = s + c[q];
    c[0] = -s - d->helmholtz_lambda;
  }
  /* coarse hierarchy */
  int m = 0;
  for (int dd = 0; dd < 3; dd++) mg->dims[0][dd] = t->cgs[dd];
  mg->cdiag[0] = mg->lvl_c[0];
  for (int dd = 0; dd < 3; dd++) mg->hc[0][dd] = mg->lvl_c[1 + 2 * dd];
  for (;;) {
    int *n = mg->dims[m];
    int ok = (n[0] % 2 == 0) && (n[1] % 2 == 0) && (n[2] % 2 == 0) &&
             n[0] >= 4 && n[1] >= 4 && n[2] >= 4 && m < 15;
    if (!ok) break;
    for (int dd = 0; dd < 3; dd++) {
      mg->dims[m + 1][dd] = n[dd] / 2;
      mg->hc[m + 1][dd] = 0.25 * mg->hc[m][dd];
    }
    const double *h = mg->hc[m + 1];
    mg->cdiag[m + 1] = -(h[0] + h[0] + h[1] + h[1] + h[2] + h[2]) -
                       d->helmholtz_lambda;
    m++;
  }
  mg->n_mg = m + 1;
  for (int q = 0; q < mg->n_mg; q++) {
    size_t n = (size_t)(mg->dims[q][0] + 2) * (mg->dims[q][1] + 2) *
               (mg->dims[q][2] + 2);
    mg->u[q] = calloc(n, sizeof(double));
    mg->f[q] = calloc(n, sizeof(double));
    mg->r[q] = calloc(n, sizeof(double));
  }
  if (d->coarse_mode == AFH_COARSE_DIRECT) {
    size_t n = (size_t)mg->dims[0][0] * mg->dims[0][1] * mg->dims[0][2];
    for (int dd = 0; dd < 3; dd++) {
      int nd = mg->dims[0][dd];
      mg->q[dd] = malloc(sizeof(double) * nd * nd);
      mg->e[dd] = malloc(sizeof(double) * nd);
    }
    mg->w1 = malloc(sizeof(double) * n);
    mg->w2 = malloc(sizeof(double) * n);
    cs_direct_build(mg);
  } else if (d->coarse_mode == AFH_COARSE_PFMG) {
    if (d->coarse_cycles < 1 || !(d->coarse_tol >= 0))
      return fail(AFH_ERR_ARG, "pfmg: coarse_cycles >= 1 and coarse_tol >= 0");
  } else if (d->coarse_mode != AFH_COARSE_CYCLES || d->coarse_cycles < 1) {
    return fail(AFH_ERR_UNSUPPORTED, "coarse solver mode");
  }
  *out = mg;
  return AFH_OK;
}

/* afh_mg_set_gradient_output: the library folds |E| into the V-cycle's
 * residual pass; the values are those of mg_compute_phi_gradient, which the
 * oracle computes in full every time */
int32_t afo_mg_set_gradient_output(afh_mg *mg, int32_t i_norm, double fac) {
  (void)fac;
  if (!mg || i_norm < 0 || i_norm > mg->t->nvc)
    return fail(AFH_ERR_ARG, "afo_mg_set_gradient_output: bad argument");
  return AFH_OK;
}

int32_t afo_mg_graph_stats(afh_mg *mg, int64_t *replays, int64_t *segmented) {
  if (!mg || !replays || !segmented) return fail(AFH_ERR_ARG, "afo_mg_graph_stats: null");
  *replays = *segmented = 0;
  return AFH_OK;
}

int32_t afo_mg_coarse_iterations(afh_mg *mg, int32_t *n) {
  if (!mg || !n) return fail(AFH_ERR_ARG, "afo_mg_coarse_iterations: null");
  *n = mg->cs_iters;
  return AFH_OK;
}

int32_t afo_mg_destroy(afh_mg *mg) {
  if (!mg) return AFH_OK;
  for (int q = 0; q < mg->n_mg; q++) free(mg->u[q]), free(mg->f[q]), free(mg->r[q]);
  for (int d = 0; d < 3; d++) free(mg->q[d]), free(mg->e[d]);
  free(mg->w1), free(mg->w2);
  afh_pfmg_free(&mg->pf);
  free(mg->pf_a7), free(mg->pf_x), free(mg->pf_b), free(mg->pf_r), free(mg->pf_e);
  free(mg->lvl_c);
  for (int q = 0; q < mg->t->nb; q++) {
    free(mg->vst[q]), free(mg->vbc[q]);
    free(mg->lsf_ix[q]), free(mg->lsf_dd[q]), free(mg->lsf_bv[q]);
  }
  free(mg->vst), free(mg->vbc), free(mg->lsf_n);
  free(mg->lsf_ix), free(mg->lsf_dd), free(mg->lsf_bv);
  free(mg);
  return AFH_OK;
}

/* The electrode operator stencil of box id as mg_set_operators_lvl stored it
 * (m_af_multigrid.f90:1133-1171): v = stencils(ix)%v(7, nc, nc, nc),
 * bc_correction = stencils(ix)%bc_correction (NULL: none); v = NULL removes
 * it (the level's constant stencil applies again). */
int32_t afo_mg_set_box_stencil(afh_mg *mg, int32_t id, const double *v,
                               const double *bc_correction) {
  if (!mg || id < 1 || id > mg->t->nb) return fail(AFH_ERR_ARG, "bad box id");
  size_t n3 = (size_t)mg->t->nc * mg->t->nc * mg->t->nc;
  free(mg->vst[id - 1]), free(mg->vbc[id - 1]);
  mg->vst[id - 1] = mg->vbc[id - 1] = NULL;
  if (!v) return AFH_OK;
  mg->vst[id - 1] = malloc(sizeof(double) * 7 * n3);
  memcpy(mg->vst[id - 1], v, sizeof(double) * 7 * n3);
  if (bc_correction) {
    mg->vbc[id - 1] = malloc(sizeof(double) * n3);
    memcpy(mg->vbc[id - 1], bc_correction, sizeof(double) * n3);
  }
  return AFH_OK;
}

/* The boundary distances of box id (mg_lsf_distance_key, sparse: ix(3, n)
 * 1-based cell indices, dd(6, n)) and mg_lsf_boundary_value(box) (nc^3), for
 * mg_box_lpllsf_gradient; i_lsf = the level-set cc variable. n = 0 removes. */
int32_t afo_mg_set_box_lsf(afh_mg *mg, int32_t id, int32_t n, const int32_t *ix,
                           const double *dd, const double *bval, int32_t i_lsf) {
  if (!mg || id < 1 || id > mg->t->nb || n < 0)
    return fail(AFH_ERR_ARG, "bad box id / count");
  afh_tree *t = mg->t;
  size_t n3 = (size_t)t->nc * t->nc * t->nc;
  free(mg->lsf_ix[id - 1]), free(mg->lsf_dd[id - 1]), free(mg->lsf_bv[id - 1]);
  mg->lsf_ix[id - 1] = NULL, mg->lsf_dd[id - 1] = mg->lsf_bv[id - 1] = NULL;
  mg->lsf_n[id - 1] = 0;
  if (n == 0) return AFH_OK;
  if (!ix || !dd || !bval || i_lsf < 1 || i_lsf > t->nvc)
    return fail(AFH_ERR_ARG, "afo_mg_set_box_lsf: bad argument");
  for (int e = 0; e < 3 * n; e++)
    if (ix[e] < 1 || ix[e] > t->nc) return fail(AFH_ERR_ARG, "cell index out of box");
  mg->lsf_n[id - 1] = n;
  mg->lsf_ix[id - 1] = malloc(sizeof(int32_t) * 3 * n);
  memcpy(mg->lsf_ix[id - 1], ix, sizeof(int32_t) * 3 * n);
  mg->lsf_dd[id - 1] = malloc(sizeof(double) * 6 * n);
  memcpy(mg->lsf_dd[id - 1], dd, sizeof(double) * 6 * n);
  mg->lsf_bv[id - 1] = malloc(sizeof(double) * n3);
  memcpy(mg->lsf_bv[id - 1], bval, sizeof(double) * n3);
  mg->i_lsf = i_lsf;
  return AFH_OK;
}

/* mg_fas_vcycle, m_af_multigrid.f90:185-264 (subtract_mean = .false.) */
int32_t afo_mg_fas_vcycle(afh_mg *mg, int32_t set_residual, int32_t hl) {
  LIVE(mg->t);
  afh_tree *t = mg->t;
  touch(t, mg->d.i_phi), touch(t, mg->d.i_rhs), touch(t, mg->d.i_tmp);
  int max_lvl = (hl > 0) ? hl : t->nlvl;
  for (int lvl = max_lvl; lvl >= 2; lvl--) {
    if (afo_mg_gsrb_boxes(mg, lvl, 0) || afo_mg_update_coarse(mg, lvl))
      return AFH_ERR_STATE;
  }
  if (afo_mg_solve_coarse(mg)) return AFH_ERR_STATE;
  for (int lvl = 2; lvl <= max_lvl; lvl++) {
    afo_mg_correct_children(mg, lvl);
    if (gc_lvl(t, lvl, mg->d.i_phi, 1) || afo_mg_gsrb_boxes(mg, lvl, 1))
      return AFH_ERR_STATE;
  }
  if (set_residual) {
    for (int lvl = 1; lvl <= max_lvl; lvl++) {
      int n = LVL_N(t, ids, lvl);
#pragma omp parallel for schedule(static)
      for (int i = 0; i < n; i++) residual_box(mg, LVL_AT(t, ids, lvl, i));
    }
  }
  return AFH_OK;
}

/* mg_fas_vcycle(set_residual) + af_tree_maxabs_cc(i_tmp)
 * (src/m_field.f90:455-465) */
int32_t afo_mg_fas_vcycle_maxres(afh_mg *mg, int32_t hl, double *max_res) {
  int32_t e = afo_mg_fas_vcycle(mg, 1, hl);
  return e ? e : afo_tree_maxabs_cc(mg->t, mg->d.i_tmp, max_res);
}

/* afh_mg_fas_vcycle_fold: the maximum kept for afo_tree_fetch_reduced */
int32_t afo_mg_fas_vcycle_fold(afh_mg *mg, int32_t hl) {
  int32_t e = afo_mg_fas_vcycle(mg, 1, hl);
  if (!e) mg->t->slot[AFH_SLOT_MAXRES] = maxabs_local(mg->t, mg->d.i_tmp);
  return e;
}

/* the |x| maxima only (the limits are read by afo_fluid_fetch_step) */
int32_t afo_tree_fetch_reduced(afh_tree *t, int32_t n, const int32_t *slots, double *out) {
  LIVE(t);
  if (n < 1 || n > 2) return fail(AFH_ERR_ARG, "fetch of %d slots", n);
  for (int q = 0; q < n; q++) {
    if (slots[q] != AFH_SLOT_MAXRES && slots[q] != AFH_SLOT_RHS)
      return fail(AFH_ERR_ARG, "bad reduction slot %d", slots[q]);
    out[q] = t->slot[slots[q]];
  }
  return hook(t, AFH_HOOK_MAX, 0, 0, out, n);
}

/* mg_fas_fmg, m_af_multigrid.f90:137-180; set_coarse_phi_rhs (742-776) is
 * update_coarse without restoring tmp -- the extra tmp = phi on the parents
 * is overwritten by the phi -> tmp copies below before tmp is read again;
 * init_phi_rhs (779-799) clears phi on levels >= 2 and restricts rhs. */
int32_t afo_mg_fas_fmg(afh_mg *mg, int32_t set_residual, int32_t have_guess) {
  LIVE(mg->t);
  afh_tree *t = mg->t;
  touch(t, mg->d.i_phi), touch(t, mg->d.i_rhs), touch(t, mg->d.i_tmp);
  int nl = t->nlvl, i_phi = mg->d.i_phi, i_tmp = mg->d.i_tmp;
  size_t bsz = t->bsz;
  if (have_guess) {
    for (int lvl = nl; lvl >= 2; lvl--) {
      if (lvl == nl && gc_lvl(t, lvl, i_phi, 1)) return AFH_ERR_STATE;
      if (afo_mg_update_coarse(mg, lvl)) return AFH_ERR_STATE;
    }
  } else {
    for (int lvl = nl; lvl >= 2; lvl--) {
      int n = LVL_N(t, ids, lvl);
      for (int i = 0; i < n; i++) {
        int id = LVL_AT(t, ids, lvl, i);
        memset(ccb(t, i_phi, id), 0, sizeof(double) * bsz);
        restrict_box(t, id, B(t, id)->parent, mg->d.i_rhs);
      }
      if (hook(t, AFH_HOOK_RESTRICT, lvl, mg->d.i_rhs, NULL, 0)) return AFH_ERR_STATE;
    }
  }
  for (int lvl = 1; lvl <= nl; lvl++) {
    int n = LVL_N(t, ids, lvl);
    for (int i = 0; i < n; i++) {
      int id = LVL_AT(t, ids, lvl, i);
      memcpy(ccb(t, i_tmp, id), ccb(t, i_phi, id), sizeof(double) * bsz);
    }
    if (lvl > 1) {
      afo_mg_correct_children(mg, lvl);
      if (gc_lvl(t, lvl, i_phi, 1)) return AFH_ERR_STATE;
    }
    if (afo_mg_fas_vcycle(mg, set_residual && lvl == nl, lvl)) return AFH_ERR_STATE;
  }
  return AFH_OK;
}

/* mg_box_lpl_gradient + mg_box_field_norm, m_af_multigrid.f90:1882-2025 */
int32_t afo_mg_compute_phi_gradient(afh_mg *mg, int32_t i_fc, double fac,
                                    int32_t i_norm) {
  afh_tree *t = mg->t;
  int nc = t->nc;
  if (i_fc < 0 || i_fc > t->nvf || i_norm < 0 || i_norm > t->nvc)
    return fail(AFH_ERR_ARG, "bad variable index");
  /* i_fc = 0: the norm only (afo_fluid_set_field_source); the face values
   * go through a per-box scratch array */
  if (i_fc == 0) {
    int lsf = 0;
    for (int q = 0; q < t->nb; q++) lsf |= mg->lsf_n && mg->lsf_n[q] != 0;
    if (i_norm == 0 || lsf)
      return fail(AFH_ERR_ARG, "i_fc = 0 needs i_norm and no electrode boxes");
  }
  for (int lvl = 1; lvl <= t->nlvl; lvl++) {
    int n = LVL_N(t, ids, lvl);
#pragma omp parallel for schedule(static)
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, ids, lvl, q);
      double *scratch = i_fc == 0 ? malloc(sizeof(double) * t->fsz) : NULL;
      double *p = ccb(t, mg->d.i_phi, id), *f = i_fc ? fcb(t, i_fc, id) : scratch;
      double inv[3];
      for (int d = 0; d < 3; d++) inv[d] = fac / B(t, id)->dr[d];
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc + 1; i++)
            f[FX(t, 0, i, j, k)] =
                inv[0] * (p[IX(t, i, j, k)] - p[IX(t, i - 1, j, k)]);
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc + 1; j++)
          for (int i = 1; i <= nc; i++)
            f[FX(t, 1, i, j, k)] =
                inv[1] * (p[IX(t, i, j, k)] - p[IX(t, i, j - 1, k)]);
      for (int k = 1; k <= nc + 1; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc; i++)
            f[FX(t, 2, i, j, k)] =
                inv[2] * (p[IX(t, i, j, k)] - p[IX(t, i, j, k - 1)]);
      /* mg_box_lpllsf_gradient (m_af_multigrid.f90:2030-2120): electrode
       * leaf boxes replace the faces next to the boundary, in order */
      if (mg->lsf_n[id - 1] && B(t, id)->children[0] == 0) {
        const double *lsf = ccb(t, mg->i_lsf, id), *bv = mg->lsf_bv[id - 1];
        for (int e = 0; e < mg->lsf_n[id - 1]; e++) {
          const int32_t *x = mg->lsf_ix[id - 1] + 3 * e;
          const double *dd = mg->lsf_dd[id - 1] + 6 * e;
          int i = x[0], j = x[1], k = x[2];
          double pc = p[IX(t, i, j, k)], bc = bv[vix(nc, i, j, k)];
          if (lsf[IX(t, i, j, k)] < 0) continue;
          if (dd[0] < 1) f[FX(t, 0, i, j, k)] = inv[0] * (pc - bc) / dd[0];
          if (dd[1] < 1) f[FX(t, 0, i + 1, j, k)] = inv[0] * (bc - pc) / dd[1];
          if (dd[2] < 1) f[FX(t, 1, i, j, k)] = inv[1] * (pc - bc) / dd[2];
          if (dd[3] < 1) f[FX(t, 1, i, j + 1, k)] = inv[1] * (bc - pc) / dd[3];
          if (dd[4] < 1) f[FX(t, 2, i, j, k)] = inv[2] * (pc - bc) / dd[4];
          if (dd[5] < 1) f[FX(t, 2, i, j, k + 1)] = inv[2] * (bc - pc) / dd[5];
        }
      }
      if (i_norm > 0) {
        double *o = ccb(t, i_norm, id);
        for (int k = 1; k <= nc; k++)
          for (int j = 1; j <= nc; j++)
            for (int i = 1; i <= nc; i++) {
              double a = f[FX(t, 0, i, j, k)] + f[FX(t, 0, i + 1, j, k)];
              double b = f[FX(t, 1, i, j, k)] + f[FX(t, 1, i, j + 1, k)];
              double c = f[FX(t, 2, i, j, k)] + f[FX(t, 2, i, j, k + 1)];
              o[IX(t, i, j, k)] = 0.5 * sqrt(a * a + b * b + c * c);
            }
      }
      free(scratch);
    }
  }
  return AFH_OK;
}

/* ------------------------------------------------------------ fluid */

int32_t afo_fluid_create(afh_tree *t, const afh_fluid_desc *d,
                         afh_fluid **out) {
  if (d->n_species < 1 || d->n_species > AFH_MAX_SPECIES ||
      d->n_reactions > AFH_MAX_REACTIONS)
    return fail(AFH_ERR_ARG, "bad species/reaction count");
  if (d->i_gas_dens > 0 &&
      (d->i_gas_dens > t->nvc || d->n_gas_species < 0 ||
       d->n_gas_species > AFH_MAX_GAS_SPECIES))
    return fail(AFH_ERR_ARG, "bad gas density variable / gas species count");
  if (d->n_ions < 0 || d->n_ions > AFH_MAX_IONS)
    return fail(AFH_ERR_ARG, "bad mobile ion count");
  for (int q = 0; q < d->n_ions; q++) {
    const int sp = d->ion_species[q];
    if (sp < 1 || sp > d->n_species || d->species_iv[sp - 1] == d->i_electron ||
        d->species_charge[sp - 1] == 0)
      return fail(AFH_ERR_ARG, "mobile ion: bad species");
    if (d->f_ion_flux[q] < 1 || d->f_ion_flux[q] > t->nvf || d->f_ion_flux[q] == d->f_flux)
      return fail(AFH_ERR_ARG, "mobile ion: bad flux variable");
  }
  const int ng = d->i_gas_dens > 0 ? d->n_gas_species : 0;
  for (int r = 0; r < d->n_reactions; r++) {
    const afh_reaction *R = &d->reactions[r];
    for (int q = 0; q < R->n_in; q++)
      if (R->ix_in[q] < 1 || R->ix_in[q] > ng + d->n_species)
        return fail(AFH_ERR_ARG, "reaction species index");
    for (int q = 0; q < R->n_out; q++)
      if (R->ix_out[q] < 1 || R->ix_out[q] > ng + d->n_species)
        return fail(AFH_ERR_ARG, "reaction species index");
  }
  afh_fluid *f = calloc(1, sizeof *f);
  f->t = t;
  f->d = *d;
  if (d->i_gas_dens <= 0) f->d.n_gas_species = 0;
  size_t ntd = (size_t)d->td.n_points * d->td.n_cols;
  size_t nch = (size_t)d->chem.n_points * d->chem.n_cols;
  f->td = malloc(sizeof(double) * (ntd ? ntd : 1));
  f->chem = malloc(sizeof(double) * (nch ? nch : 1));
  memcpy(f->td, d->td.rows_cols, sizeof(double) * ntd);
  if (nch) memcpy(f->chem, d->chem.rows_cols, sizeof(double) * nch);
  f->d.td.rows_cols = f->td;
  f->d.chem.rows_cols = f->chem;
  for (int r = 0; r < d->n_reactions; r++) {
    f->reac[r] = d->reactions[r];
    int rt = d->reactions[r].rate_type;
    if (rt < AFH_RATE_TABULATED_FIELD || rt > AFH_RATE_K15 || rt == 7)
      return fail(AFH_ERR_UNSUPPORTED, "reaction rate type %d", rt);
    if ((rt == AFH_RATE_K1 || rt == AFH_RATE_K3) &&
        (d->td_energy_col < 1 || d->td_energy_col > d->td.n_cols))
      return fail(AFH_ERR_ARG, "rate type %d needs the td mean-energy column", rt);
  }
  f->d.reactions = f->reac;
  *out = f;
  return AFH_OK;
}
int32_t afo_fluid_destroy(afh_fluid *f) {
  if (!f) return AFH_OK;
  free(f->td), free(f->chem), free(f);
  return AFH_OK;
}

int32_t afo_fluid_set_field_source(afh_fluid *f, int32_t i_phi, double fac) {
  if (i_phi < 0 || i_phi > f->t->nvc) return fail(AFH_ERR_ARG, "bad i_phi");
  f->phi_iv = i_phi;
  f->phi_fac = fac;
  return AFH_OK;
}

int32_t afo_fluid_set_ion_se_yield(afh_fluid *f, double yield) {
  if (!(yield >= 0)) return fail(AFH_ERR_ARG, "ion_se_yield %g", yield);
  f->ion_se_yield = yield;
  return AFH_OK;
}

/* handle_ion_se_flux (src/m_fluid.f90:584-663) over the leaves
 * (af_loop_box(tree, handle_ion_se_flux, .true.), m_fluid.f90:63-67): on
 * every physical face of a leaf box (neighbors < af_no_box), for each mobile
 * ion of positive charge in order, the electrons' face flux loses
 * ion_se_yield times the ion flux out of the domain: min(0, F_ion) on the
 * low faces, max(0, F_ion) on the high ones. The reference's 3-D low-y case
 * (m_fluid.f90:639-642) indexes fc(1:nc, 1:nc, 1, 2): the y faces j = 1..nc
 * of the first z plane, not the wall's fc(1:nc, 1, 1:nc, 2); reproduced as
 * written (its results are the parity target). */
int32_t afo_fluid_ion_se_flux(afh_fluid *f) {
  afh_tree *t = f->t;
  LIVE(t);
  const int nc = t->nc;
  const double y = f->ion_se_yield;
  for (int l = 1; l <= t->nlvl; l++)
    for (int q = 0; q < LVL_N(t, leaves, l); q++) {
      const int id = LVL_AT(t, leaves, l, q);
      const afh_box_meta *m = B(t, id);
      double *Fe = fcb(t, f->d.f_flux, id);
      for (int nb = 0; nb < 6; nb++) {
        if (m->neighbors[nb] >= 0) continue;
        const int d = nb >> 1, hi = nb & 1, fi = hi ? nc + 1 : 1;
        for (int n = 0; n < f->d.n_ions; n++) {
          if (f->d.species_charge[f->d.ion_species[n] - 1] <= 0) continue;
          const double *Fi = fcb(t, f->d.f_ion_flux[n], id);
          for (int b = 1; b <= nc; b++)
            for (int a = 1; a <= nc; a++) {
              int p[3];
              if (nb == 2) { /* af_neighb_lowy as the reference indexes it */
                p[0] = a, p[1] = b, p[2] = 1;
              } else {
                p[d] = fi;
                p[d == 0 ? 1 : 0] = a;
                p[d == 2 ? 1 : 2] = b;
              }
              const size_t c = FX(t, d, p[0], p[1], p[2]);
              const double v = Fi[c];
              Fe[c] = Fe[c] - y * (hi ? (v > 0.0 ? v : 0.0) : (v < 0.0 ? v : 0.0));
            }
        }
      }
    }
  return AFH_OK;
}

/* set_box_mask's electrode part (src/m_fluid.f90:469-483) */
int32_t afo_fluid_set_update_mask(afh_fluid *f, int32_t i_lsf) {
  if (!f || i_lsf < 0 || i_lsf > f->t->nvc) return fail(AFH_ERR_ARG, "bad i_lsf");
  f->mask_iv = i_lsf;
  return AFH_OK;
}

int32_t afo_fluid_set_rhs_output(afh_fluid *f, int32_t i_rhs, int32_t ghosts) {
  if (i_rhs < 0 || i_rhs > f->t->nvc) return fail(AFH_ERR_ARG, "bad i_rhs");
  f->rhs_iv = i_rhs;
  f->rhs_ghosts = ghosts != 0;
  f->rhs_state = -1;
  return AFH_OK;
}
static int rhs_current(afh_fluid *f, int s_out) {
  if (f->rhs_iv <= 0 || f->rhs_state < 0 || f->rhs_state != s_out) return 0;
  if (f->t->gen[f->rhs_iv] != f->rhs_snap[0]) return 0;
  for (int s = 0; s < f->d.n_species; s++)
    if (f->t->gen[f->d.species_iv[s] + s_out] != f->rhs_snap[s + 1]) return 0;
  return 1;
}
int32_t afo_fluid_rhs_valid(afh_fluid *f, int32_t s_out, int32_t *valid) {
  *valid = rhs_current(f, s_out);
  return AFH_OK;
}
int32_t afo_fluid_rhs_maxabs(afh_fluid *f, int32_t s_out, double *max_rhs) {
  if (!rhs_current(f, s_out))
    return fail(AFH_ERR_STATE, "no current rhs output of state %d", s_out);
  *max_rhs = f->rhs_max;
  return hook(f->t, AFH_HOOK_MAX, 0, f->rhs_iv, max_rhs, 1);
}

/* electrode_species_bc, src/streamer.f90:578-636 (3D branch) */
int32_t afo_electrode_species_bc(afh_fluid *f, int32_t i_lsf, int32_t i_1pos_ion,
                                 int32_t neumann_zero, int32_t n_ids,
                                 const int32_t *ids) {
  afh_tree *t = f->t;
  if (i_lsf < 1 || i_lsf > t->nvc || i_1pos_ion < 1 || i_1pos_ion > t->nvc ||
      n_ids < 0 || (n_ids && !ids))
    return fail(AFH_ERR_ARG, "electrode_species_bc: bad argument");
  for (int s = 0; s < f->d.n_species; s++) touch(t, f->d.species_iv[s]);
  touch(t, i_1pos_ion);
  for (int q = 0; q < n_ids; q++)
    if (ids[q] < 1 || ids[q] > t->nb) return fail(AFH_ERR_ARG, "bad box id");
  const int nc = t->nc;
  for (int q = 0; q < n_ids; q++) {
    const int id = ids[q];
    const double *lsf = ccb(t, i_lsf, id);
    double *ne = ccb(t, f->d.i_electron, id), *ion = ccb(t, i_1pos_ion, id);
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          const size_t x = IX(t, i, j, k);
          if (!(lsf[x] < 0)) continue;
          for (int s = 0; s < f->d.n_species; s++) ccb(t, f->d.species_iv[s], id)[x] = 0.0;
          const size_t nb[6] = {IX(t, i - 1, j, k), IX(t, i + 1, j, k), IX(t, i, j - 1, k),
                                IX(t, i, j + 1, k), IX(t, i, j, k - 1), IX(t, i, j, k + 1)};
          int cnt = 0;
          for (int m = 0; m < 6; m++) cnt += lsf[nb[m]] > 0;
          if (cnt > 0 && neumann_zero) {
            double sum = 0.0; /* sum(dens_nb, mask=(lsf_nb > 0)) */
            for (int m = 0; m < 6; m++)
              if (lsf[nb[m]] > 0) sum = sum + ne[nb[m]];
            ne[x] = sum / cnt;
            ion[x] = ne[x];
          }
        }
  }
  return AFH_OK;
}

/* LT_get_loc + LT_get_col_at_loc (linear spacing, no extrapolation),
 * src/lookup_table_fortran/m_lookup_table.f90:330-406 */
static inline double lt_col(const afh_lt *lt, int col, double x) {
  double frac = (x - lt->x_min) * lt->inv_fac;
  int low;
  double lf;
  if (frac <= 0) {
    low = 1;
    lf = 1;
  } else if (frac >= lt->n_points - 1) {
    low = lt->n_points - 1;
    lf = 0;
  } else {
    low = (int)ceil(frac);
    lf = low - frac;
  }
  const double *rc = lt->rows_cols + (size_t)(col - 1) * lt->n_points;
  return lf * rc[low - 1] + (1 - lf) * rc[low];
}

/* get_rates for one cell and one reaction, src/m_chemistry.f90:565-650
 * (operand order as written there; `**2` as a product, real powers pow).
 * *Te < 0 on the first call of a cell: Te = electron_eV_to_K *
 * LT_get_col(td_tbl, td_energy_eV, Td) is looked up once. */
static double rate_of(const afh_fluid *fl, const afh_reaction *R, double field,
                      double *Te) {
  const double c0 = R->rate_factor;
  const double *c = R->c;
  const double Tg = fl->d.gas_temperature;
  const double kB = 1.3806503e-23, eV = 1.6022e-19;  /* UC_boltzmann_const, UC_elec_volt */
  const double electron_eV_to_K = 2 * eV / (3 * kB);
  if ((R->rate_type == AFH_RATE_K1 || R->rate_type == AFH_RATE_K3) && *Te < 0)
    *Te = electron_eV_to_K * lt_col(&fl->d.td, fl->d.td_energy_col, field);
  switch (R->rate_type) {
  case AFH_RATE_TABULATED_FIELD: return c0 * lt_col(&fl->d.chem, R->table_col, field);
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
  case AFH_RATE_K1: return c0 * c[0] * pow(300 / *Te, c[1]);
  case AFH_RATE_K3: {
    const double z = (kB / eV) * *Te + c[1];
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
  default: /* AFH_RATE_K15 */
    return c0 * c[0] * exp(-pow(c[1] / (kB * (Tg + field / c[2])), c[3]));
  }
}

/* field_set_rhs, src/m_field.f90:363-401 */
int32_t afo_field_set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in) {
  LIVE(f->t);
  afh_tree *t = f->t;
  touch(t, i_rhs);
  const double fac = -1.6022e-19 / 8.8541878176e-12;
  for (int l = 1; l <= t->nlvl; l++) {
    int n = LVL_N(t, leaves, l);
#pragma omp parallel for schedule(static)
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, leaves, l, q);
      double *r = ccb(t, i_rhs, id);
      for (size_t x = 0; x < t->bsz; x++) r[x] = 0.0;
      for (int s = 0; s < f->d.n_species; s++) {
        if (f->d.species_charge[s] == 0) continue;
        double qq = f->d.species_charge[s] * fac;
        double *c = ccb(t, f->d.species_iv[s] + s_in, id);
        for (size_t x = 0; x < t->bsz; x++) r[x] = r[x] + qq * c[x];
      }
    }
  }
  return AFH_OK;
}

/* field_set_rhs + af_tree_maxabs_cc(i_rhs) (src/m_field.f90:363-401, 419) */
int32_t afo_field_set_rhs_maxabs(afh_fluid *f, int32_t i_rhs, int32_t s_in,
                                 double *max_rhs) {
  int32_t e = afo_field_set_rhs(f, i_rhs, s_in);
  return e ? e : afo_tree_maxabs_cc(f->t, i_rhs, max_rhs);
}

/* af_limiter_koren, m_af_limiters.f90:72-95; af_limiter_gminmod
 * (120-149); vanleer (97-110); none/zero */
static inline double limiter(int lim, double a, double b) {
  const double third = 1 / 3.0;
  switch (lim) {
  case AFH_LIM_KOREN: {
    double aa = a * a, ab = a * b;
    if (ab <= 0) return 0;
    if (aa <= 0.25 * ab) return 2 * a;
    if (aa <= 2.5 * ab) return third * (b + 2 * a);
    return 2 * b;
  }
  case AFH_LIM_VANLEER: {
    double ab = a * b;
    return ab > 0 ? 2 * ab / (a + b) : 0;
  }
  case AFH_LIM_NONE: return 0.5 * (a + b);
  case AFH_LIM_ZERO: return 0.0;
  default: {
    double th = lim == AFH_LIM_MINMOD ? 1.0 : lim == AFH_LIM_MC ? 2.0 : 4 / 3.0;
    if (a * b > 0) {
      double x = fabs(th * a), y = fabs(th * b), z = fabs(0.5 * (a + b));
      double m = x;
      if (y < m) m = y;
      if (z < m) m = z;
      return copysign(m, a);
    }
    return 0.0;
  }
  }
}

/* cc2 index for the (nc+4)^3 array with indices -1..nc+2 */
#define I2(n4, i, j, k) ((((size_t)(k) + 1) * (n4) + (size_t)(j) + 1) * (n4) + (size_t)(i) + 1)

/* bc_to_gc2, m_af_ghostcell.f90:282-375 (incl. the c0 quirk for highy) */
static void bc_to_gc2(afh_tree *t, int id, double *cc, int nb, const afh_bc *bc) {
  int nc = t->nc, n4 = nc + 4, d = nb_dim(nb);
  double c0, c1, c2;
  switch (bc->type) {
  case AFH_BC_DIRICHLET: c0 = 2; c1 = -1; c2 = c0; break;
  case AFH_BC_NEUMANN: c0 = B(t, id)->dr[d] * nb_pm(nb); c1 = 1; c2 = 3 * c0; break;
  default: c0 = 1; c1 = 0; c2 = c0; break;
  }
  if (nb == 4) c2 = c0; /* m_af_ghostcell.f90:361 uses c0 on layer 2 */
  int g1 = nb_low(nb) ? 0 : nc + 1, g2 = nb_low(nb) ? -1 : nc + 2;
  int x1 = nb_low(nb) ? 1 : nc, x2 = nb_low(nb) ? 2 : nc - 1;
  int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
  for (int b = 1; b <= nc; b++)
    for (int a = 1; a <= nc; a++) {
      int p[3];
      p[ta] = a, p[tb] = b;
      p[d] = g1; size_t G1 = I2(n4, p[0], p[1], p[2]);
      p[d] = g2; size_t G2 = I2(n4, p[0], p[1], p[2]);
      p[d] = x1; size_t X1 = I2(n4, p[0], p[1], p[2]);
      p[d] = x2; size_t X2 = I2(n4, p[0], p[1], p[2]);
      cc[G1] = c0 * bc->value + c1 * cc[X1];
      cc[G2] = c2 * bc->value + c1 * cc[X2];
    }
}

/* gc2_prolong_rb, m_af_ghostcell.f90:753-856 (3D) */
static void gc2_prolong_rb(afh_tree *t, int id, int nb, int iv, double *cc) {
  int nc = t->nc, n4 = nc + 4, d = nb_dim(nb);
  int lo[3] = {1, 1, 1}, hi[3] = {nc, nc, nc}, lo_c[3], hi_c[3], off[3];
  lo[d] = nb_low(nb) ? -1 : nc + 1;
  hi[d] = nb_low(nb) ? 0 : nc + 2;
  child_offset(t, id, 0, off);
  for (int q = 0; q < 3; q++) {
    /* (lo+1)/2 with Fortran integer division (truncation toward zero) */
    lo_c[q] = off[q] + (lo[q] + 1) / 2;
    hi_c[q] = off[q] + (hi[q] + 1) / 2;
    if (q == d) {
      lo_c[q] -= nb_pm(nb) * nc;
      hi_c[q] -= nb_pm(nb) * nc;
    }
  }
  int p_nb_id = B(t, B(t, id)->parent)->neighbors[nb - 1];
  double *cp = ccb(t, iv, p_nb_id);
  int lim = t->meth[iv].lim;
  for (int k = lo_c[2]; k <= hi_c[2]; k++) {
    int kf = lo[2] + 2 * (k - lo_c[2]);
    for (int j = lo_c[1]; j <= hi_c[1]; j++) {
      int jf = lo[1] + 2 * (j - lo_c[1]);
      for (int i = lo_c[0]; i <= hi_c[0]; i++) {
        int fi = lo[0] + 2 * (i - lo_c[0]);
        double f0 = cp[IX(t, i, j, k)];
        double sa0 = cp[IX(t, i, j, k)] - cp[IX(t, i - 1, j, k)];
        double sa1 = cp[IX(t, i, j, k)] - cp[IX(t, i, j - 1, k)];
        double sa2 = cp[IX(t, i, j, k)] - cp[IX(t, i, j, k - 1)];
        double sb0 = cp[IX(t, i + 1, j, k)] - cp[IX(t, i, j, k)];
        double sb1 = cp[IX(t, i, j + 1, k)] - cp[IX(t, i, j, k)];
        double sb2 = cp[IX(t, i, j, k + 1)] - cp[IX(t, i, j, k)];
        double f1 = 0.25 * limiter(lim, sa0, sb0);
        double f2 = 0.25 * limiter(lim, sa1, sb1);
        double f3 = 0.25 * limiter(lim, sa2, sb2);
        cc[I2(n4, fi, jf, kf)] = f0 - f1 - f2 - f3;
        cc[I2(n4, fi, jf, kf + 1)] = f0 - f1 - f2 + f3;
        cc[I2(n4, fi, jf + 1, kf)] = f0 - f1 + f2 - f3;
        cc[I2(n4, fi, jf + 1, kf + 1)] = f0 - f1 + f2 + f3;
        cc[I2(n4, fi + 1, jf, kf)] = f0 + f1 - f2 - f3;
        cc[I2(n4, fi + 1, jf, kf + 1)] = f0 + f1 - f2 + f3;
        cc[I2(n4, fi + 1, jf + 1, kf)] = f0 + f1 + f2 - f3;
        cc[I2(n4, fi + 1, jf + 1, kf + 1)] = f0 + f1 + f2 + f3;
      }
    }
  }
}

/* af_gc2_box, m_af_ghostcell.f90:672-744 */
static void gc2_box(afh_tree *t, int id, int iv, double *cc) {
  int nc = t->nc, n4 = nc + 4;
  double *c = ccb(t, iv, id);
  for (int k = 0; k <= nc + 1; k++)
    for (int j = 0; j <= nc + 1; j++)
      for (int i = 0; i <= nc + 1; i++) cc[I2(n4, i, j, k)] = c[IX(t, i, j, k)];
  for (int nb = 1; nb <= 6; nb++) {
    int nb_id = B(t, id)->neighbors[nb - 1], d = nb_dim(nb);
    if (nb_id > 0) {
      int lo[3] = {1, 1, 1}, hi[3] = {nc, nc, nc};
      lo[d] = nb_low(nb) ? -1 : nc + 1;
      hi[d] = nb_low(nb) ? 0 : nc + 2;
      double *cn = ccb(t, iv, nb_id);
      int sh = -nb_pm(nb) * nc;
      for (int k = lo[2]; k <= hi[2]; k++)
        for (int j = lo[1]; j <= hi[1]; j++)
          for (int i = lo[0]; i <= hi[0]; i++) {
            int p[3] = {i, j, k};
            p[d] += sh;
            cc[I2(n4, i, j, k)] = cn[IX(t, p[0], p[1], p[2])];
          }
    } else if (nb_id == 0) {
      gc2_prolong_rb(t, id, nb, iv, cc);
    } else {
      bc_to_gc2(t, id, cc, nb, &t->meth[iv].bc[nb - 1]);
    }
  }
  for (int k = 0; k <= nc + 1; k++)
    for (int j = 0; j <= nc + 1; j++)
      for (int i = 0; i <= nc + 1; i++) c[IX(t, i, j, k)] = cc[I2(n4, i, j, k)];
}

/* flux_upwind_box (m_af_flux_schemes.f90:715-848) with reconstruct_upwind_1d
 * (282-303) and the m_fluid callbacks flux_direction / flux_upwind
 * (src/m_fluid.f90:102-227) for electrons, constant N, LFA. Returns the box
 * maxima of cfl_sum and sigma. */
/* value m (-1 .. nc+2) of the line along dim d at (a, b) of an enlarged box */
static double line_at(const double *cc2, int n4, int d, int a, int b, int m) {
  int p[3];
  if (d == 0) p[0] = m, p[1] = a, p[2] = b;
  else if (d == 1) p[0] = a, p[1] = m, p[2] = b;
  else p[0] = a, p[1] = b, p[2] = m;
  return cc2[I2(n4, p[0], p[1], p[2])];
}

static void flux_box(afh_fluid *fl, int id, int s_deriv, double *cfl_max,
                     double *sig_max, double *cc2, double *cfl, double *cc2i) {
  afh_tree *t = fl->t;
  int nc = t->nc, n4 = nc + 4;
  int i_e = fl->d.i_electron + s_deriv;
  const double N_inv = 1 / fl->d.gas_number_density;
  const double SI_to_Td = 1e21;
  gc2_box(t, id, i_e, cc2);
  /* mobile ions (flux species 2.., m_streamer.f90:253-282): their own two
   * ghost layers (af_gc2_box over every flux species) */
  const size_t n4c = (size_t)n4 * n4 * n4;
  for (int q = 0; q < fl->d.n_ions; q++)
    gc2_box(t, id, fl->d.species_iv[fl->d.ion_species[q] - 1] + s_deriv, cc2i + q * n4c);
  double *ne = ccb(t, i_e, id), *E = ccb(t, fl->d.i_efld, id);
  double *F = fcb(t, fl->d.f_flux, id);
  /* the face field: stored (f_field), or mg_box_lpl_gradient's value from
   * the potential (afo_fluid_set_field_source) */
  const double *Ef = fl->phi_iv ? NULL : fcb(t, fl->d.f_field, id);
  const double *Pp = fl->phi_iv ? ccb(t, fl->phi_iv, id) : NULL;
  /* variable gas density: N_inv = 2 / (N_{f-1} + N_f) per face (m_fluid.f90:146-154) */
  const double *Ng = fl->d.i_gas_dens > 0 ? ccb(t, fl->d.i_gas_dens, id) : NULL;
  size_t ncell = (size_t)nc * nc * nc;
  for (size_t q = 0; q < ncell; q++) cfl[q] = 0.0;
  double smax = -HUGE_VAL;
  for (int d = 0; d < 3; d++) {
    double inv_dx = 1 / B(t, id)->dr[d];
    for (int b = 1; b <= nc; b++)
      for (int a = 1; a <= nc; a++) {
        /* line along dim d; (a, b) = (i, j) of the other two dims */
        double line[64 + 4], Ecc[64 + 2], necc[64 + 2], Ex[64 + 1], Nl[64 + 2];
        double v[64 + 1], dc[64 + 1], u[64 + 1];
        for (int m = -1; m <= nc + 2; m++) {
          int p[3];
          if (d == 0) p[0] = m, p[1] = a, p[2] = b;
          else if (d == 1) p[0] = a, p[1] = m, p[2] = b;
          else p[0] = a, p[1] = b, p[2] = m;
          line[m + 1] = cc2[I2(n4, p[0], p[1], p[2])];
          if (m >= 0 && m <= nc + 1) {
            Ecc[m] = E[IX(t, p[0], p[1], p[2])];
            necc[m] = ne[IX(t, p[0], p[1], p[2])];
            Nl[m] = Ng ? Ng[IX(t, p[0], p[1], p[2])] : 0.0;
          }
          if (m >= 1 && m <= nc + 1) {
            if (Pp) {
              int pm[3] = {p[0], p[1], p[2]};
              pm[d] -= 1;
              Ex[m - 1] = (fl->phi_fac / B(t, id)->dr[d]) *
                          (Pp[IX(t, p[0], p[1], p[2])] - Pp[IX(t, pm[0], pm[1], pm[2])]);
            } else {
              Ex[m - 1] = Ef[FX(t, d, p[0], p[1], p[2])];
            }
          }
        }
#define L(m) line[(m) + 1]
        for (int fidx = 1; fidx <= nc + 1; fidx++) {
          int pos = (-1 * Ex[fidx - 1] > 0);
          if (pos)
            u[fidx - 1] = L(fidx - 1) + 0.5 * limiter(fl->d.limiter,
                                                      L(fidx) - L(fidx - 1),
                                                      L(fidx - 1) - L(fidx - 2));
          else
            u[fidx - 1] = L(fidx) - 0.5 * limiter(fl->d.limiter,
                                                  L(fidx) - L(fidx - 1),
                                                  L(fidx + 1) - L(fidx));
        }
#undef L
        for (int fidx = 1; fidx <= nc + 1; fidx++) {
          const double ni = Ng ? 2 / (Nl[fidx - 1] + Nl[fidx]) : N_inv;
          double tfc = 0.5 * (Ecc[fidx - 1] + Ecc[fidx]) * SI_to_Td * ni;
          double mu = lt_col(&fl->d.td, 1, tfc) * ni;
          double dcf = lt_col(&fl->d.td, 2, tfc) * ni;
          v[fidx - 1] = -mu * Ex[fidx - 1];
          dc[fidx - 1] = dcf;
          double flux = v[fidx - 1] * u[fidx - 1] -
                        dcf * inv_dx * (necc[fidx] - necc[fidx - 1]);
          double sigma = mu * u[fidx - 1];
          int p[3];
          if (d == 0) p[0] = fidx, p[1] = a, p[2] = b;
          else if (d == 1) p[0] = a, p[1] = fidx, p[2] = b;
          else p[0] = a, p[1] = b, p[2] = fidx;
          /* ion fluxes (m_fluid.f90:207-214): mu = mobility N_inv,
           * v = sign mu E_x, flux = v u; sigma = sigma + mu u */
          for (int q = 0; q < fl->d.n_ions; q++) {
            const double *c2 = cc2i + q * n4c;
            const double sg = fl->d.species_charge[fl->d.ion_species[q] - 1] > 0 ? 1.0 : -1.0;
            const double Lm2 = line_at(c2, n4, d, a, b, fidx - 2);
            const double Lm1 = line_at(c2, n4, d, a, b, fidx - 1);
            const double L0 = line_at(c2, n4, d, a, b, fidx);
            const double Lp1 = line_at(c2, n4, d, a, b, fidx + 1);
            double ui;
            if (sg * Ex[fidx - 1] > 0)
              ui = Lm1 + 0.5 * limiter(fl->d.limiter, L0 - Lm1, Lm1 - Lm2);
            else
              ui = L0 - 0.5 * limiter(fl->d.limiter, L0 - Lm1, Lp1 - L0);
            const double mui = fl->d.ion_mobility[q] * ni;
            const double vi = sg * mui * Ex[fidx - 1];
            fcb(t, fl->d.f_ion_flux[q], id)[FX(t, d, p[0], p[1], p[2])] = vi * ui;
            sigma = sigma + mui * ui;
          }
          if (sigma > smax) smax = sigma;
          F[FX(t, d, p[0], p[1], p[2])] = flux;
        }
        for (int c = 1; c <= nc; c++) {
          double mv = fmax(fabs(v[c]), fabs(v[c - 1]));
          double md = fmax(dc[c], dc[c - 1]);
          double term = 1.0 * mv * inv_dx + 2 * md * (inv_dx * inv_dx);
          int p[3];
          if (d == 0) p[0] = c, p[1] = a, p[2] = b;
          else if (d == 1) p[0] = a, p[1] = c, p[2] = b;
          else p[0] = a, p[1] = b, p[2] = c;
          size_t ci = ((size_t)(p[2] - 1) * nc + (p[1] - 1)) * nc + (p[0] - 1);
          cfl[ci] = cfl[ci] + term;
        }
      }
  }
  double cm = -HUGE_VAL;
  for (size_t q = 0; q < ncell; q++)
    if (cfl[q] > cm) cm = cfl[q];
  *cfl_max = cm;
  *sig_max = smax;
}

/* af_restrict_ref_boundary, m_af_restrict.f90:140-161 */
static int32_t restrict_ref_boundary(afh_tree *t, int iv) {
  for (int l = t->nlvl; l >= 2; l--) {
    int n = LVL_N(t, leaves, l);
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, leaves, l, q), p_id = B(t, id)->parent;
      int any = 0;
      for (int nb = 0; nb < 6; nb++) any |= (B(t, id)->neighbors[nb] == 0);
      if (p_id > 0 && any) restrict_box(t, id, p_id, iv);
    }
    if (hook(t, AFH_HOOK_RESTRICT, l, iv, NULL, 0)) return AFH_ERR_STATE;
  }
  return AFH_OK;
}

/* af_consistent_fluxes / flux_from_children, m_af_core.f90:1257-1402 */
static void consistent_fluxes(afh_tree *t, int f_ix) {
  int nc = t->nc, nch = nc / 2;
  for (int l = 1; l <= t->nlvl - 1; l++) {
    int n = LVL_N(t, parents, l);
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, parents, l, q);
      for (int nb = 1; nb <= 6; nb++) {
        int nb_id = B(t, id)->neighbors[nb - 1];
        if (nb_id <= 0 || B(t, nb_id)->children[0] != 0) continue;
        int d = nb_dim(nb);
        int i = nb_low(nb) ? 1 : nc + 1, i_nb = nb_low(nb) ? nc + 1 : 1;
        double *fn = fcb(t, f_ix, nb_id);
        for (int ic = 0; ic < 4; ic++) {
          int i_ch = child_adj_nb[nb - 1][ic];
          int c_id = B(t, id)->children[i_ch - 1];
          double *fcc = fcb(t, f_ix, c_id);
          int ioff[3];
          for (int x = 0; x < 3; x++) ioff[x] = nch * child_dix[i_ch - 1][x];
          int ta = (d == 0) ? 1 : 0, tb = (d == 2) ? 1 : 2;
          for (int bb = 1; bb <= nch; bb++)
            for (int aa = 1; aa <= nch; aa++) {
              int pc[3], p1[3], p2[3], p3[3], p4[3];
              pc[d] = i_nb, pc[ta] = ioff[ta] + aa, pc[tb] = ioff[tb] + bb;
              p1[d] = p2[d] = p3[d] = p4[d] = i;
              p1[ta] = 2 * aa - 1, p1[tb] = 2 * bb - 1;
              p2[ta] = 2 * aa, p2[tb] = 2 * bb - 1;
              p3[ta] = 2 * aa - 1, p3[tb] = 2 * bb;
              p4[ta] = 2 * aa, p4[tb] = 2 * bb;
              fn[FX(t, d, pc[0], pc[1], pc[2])] =
                  0.25 * (fcc[FX(t, d, p1[0], p1[1], p1[2])] +
                          fcc[FX(t, d, p2[0], p2[1], p2[2])] +
                          fcc[FX(t, d, p3[0], p3[1], p3[2])] +
                          fcc[FX(t, d, p4[0], p4[1], p4[2])]);
            }
        }
      }
    }
  }
}

/* flux_upwind_tree, m_af_flux_schemes.f90:666-712 */
int32_t afo_flux_upwind_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim) {
  LIVE(f->t);
  afh_tree *t = f->t;
  int nc = t->nc;
  touch(t, f->d.i_electron + s_deriv); /* ghost layers written back */
  if (restrict_ref_boundary(t, f->d.i_electron + s_deriv)) return AFH_ERR_STATE;
  for (int q = 0; q < f->d.n_ions; q++) {
    const int iv = f->d.species_iv[f->d.ion_species[q] - 1] + s_deriv;
    touch(t, iv);
    if (restrict_ref_boundary(t, iv)) return AFH_ERR_STATE;
  }
  double cfl_max = -HUGE_VAL, sig_max = -HUGE_VAL;
  for (int l = 1; l <= t->nlvl; l++) {
    int n = LVL_N(t, leaves, l);
    if (hook(t, AFH_HOOK_HALO, l, f->d.i_electron + s_deriv, NULL, 0))
      return AFH_ERR_STATE;
    for (int q = 0; q < f->d.n_ions; q++)
      if (hook(t, AFH_HOOK_HALO, l, f->d.species_iv[f->d.ion_species[q] - 1] + s_deriv,
               NULL, 0))
        return AFH_ERR_STATE;
#pragma omp parallel
    {
      double *cc2 = malloc(sizeof(double) * (size_t)(nc + 4) * (nc + 4) * (nc + 4));
      double *cc2i = malloc(sizeof(double) * (size_t)(nc + 4) * (nc + 4) * (nc + 4) *
                            (f->d.n_ions > 0 ? f->d.n_ions : 1));
      double *cfl = malloc(sizeof(double) * (size_t)nc * nc * nc);
      double lc = -HUGE_VAL, ls = -HUGE_VAL;
#pragma omp for schedule(static)
      for (int q = 0; q < n; q++) {
        double c, s;
        flux_box(f, LVL_AT(t, leaves, l, q), s_deriv, &c, &s, cc2, cfl, cc2i);
        if (c > lc) lc = c;
        if (s > ls) ls = s;
      }
#pragma omp critical
      {
        if (lc > cfl_max) cfl_max = lc;
        if (ls > sig_max) sig_max = ls;
      }
      free(cc2), free(cfl), free(cc2i);
    }
    /* the boxes' first ghost layer was written back (gc2) */
    if (hook(t, AFH_HOOK_RIMS, l, f->d.i_electron + s_deriv, NULL, 0))
      return AFH_ERR_STATE;
    for (int q = 0; q < f->d.n_ions; q++)
      if (hook(t, AFH_HOOK_RIMS, l, f->d.species_iv[f->d.ion_species[q] - 1] + s_deriv,
               NULL, 0))
        return AFH_ERR_STATE;
  }
  /* af_consistent_fluxes over every flux variable */
  consistent_fluxes(t, f->d.f_flux);
  if (hook(t, AFH_HOOK_CFLUX, 0, f->d.f_flux, NULL, 0)) return AFH_ERR_STATE;
  for (int q = 0; q < f->d.n_ions; q++) {
    consistent_fluxes(t, f->d.f_ion_flux[q]);
    if (hook(t, AFH_HOOK_CFLUX, 0, f->d.f_ion_flux[q], NULL, 0)) return AFH_ERR_STATE;
  }
  {
    double r[2] = {cfl_max, sig_max};
    if (hook(t, AFH_HOOK_MAX, 0, 0, r, 2)) return AFH_ERR_STATE;
    cfl_max = r[0];
    sig_max = r[1];
  }
  /* dt_lim(1) = min over boxes of 1/maxval(cfl_sum) = 1/max(cfl_sum);
   * other_dt(1) = eps0/(e*max(maxval(sigma),1e-100)) minimised over lines */
  dt_lim[0] = 1 / cfl_max;
  dt_lim[1] = 8.8541878176e-12 / (1.6022e-19 * fmax(sig_max, 1e-100));
  return AFH_OK;
}

/* flux_update_densities (m_af_flux_schemes.f90:320-436) with
 * add_source_terms, get_rates, get_derivatives (src/m_fluid.f90:298-466,
 * src/m_chemistry.f90:565-688) and set_box_mask (469-515): with an electrode
 * (afo_fluid_set_update_mask) a cell with lsf <= 0 keeps the weighted sum of
 * the previous states -- its rates still count for the chemistry limit --
 * and a box without another cell is skipped by add_source_terms altogether
 * (m_fluid.f90:332); no dielectric or plasma region. */
int32_t afo_flux_update_densities(afh_fluid *fl, double dt, int32_t s_deriv,
                                  int32_t n_prev, const int32_t *s_prev,
                                  const double *w_prev, int32_t s_out,
                                  int32_t last_step, double *dt_lim) {
  LIVE(fl->t);
  afh_tree *t = fl->t;
  int nc = t->nc, ns = fl->d.n_species, nr = fl->d.n_reactions;
  double chem_min = 1e100;
  const double eps = 1e-100;
  for (int l = 1; l <= t->nlvl; l++) {
    int n = LVL_N(t, leaves, l);
#pragma omp parallel for schedule(static) reduction(min : chem_min)
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, leaves, l, q);
      double dt_dr[3];
      for (int d = 0; d < 3; d++) dt_dr[d] = dt / B(t, id)->dr[d];
      double *E = ccb(t, fl->d.i_efld, id);
      double *F = fcb(t, fl->d.f_flux, id);
      const double *lsf = fl->mask_iv > 0 ? ccb(t, fl->mask_iv, id) : NULL;
      /* if (.not. any(mask)) return (m_fluid.f90:332) */
      int any_mask = 1;
      if (lsf) {
        any_mask = 0;
        for (int k = 1; k <= nc && !any_mask; k++)
          for (int j = 1; j <= nc && !any_mask; j++)
            for (int i = 1; i <= nc && !any_mask; i++)
              if (!(lsf[IX(t, i, j, k)] <= 0.0)) any_mask = 1;
      }
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc; i++) {
            size_t x = IX(t, i, j, k);
            /* where (lsf <= 0) mask = .false. */
            const int upd = !lsf || !(lsf[x] <= 0.0);
            /* weighted sum of previous states */
            for (int s = 0; s < ns; s++) {
              int iv = fl->d.species_iv[s];
              double tmp = 0.0;
              for (int m = 0; m < n_prev; m++)
                tmp = tmp + w_prev[m] * ccb(t, iv + s_prev[m], id)[x];
              ccb(t, iv + s_out, id)[x] = tmp;
            }
            /* source terms; with a variable gas density the gas species
             * come first (densities gas_fractions * N) and the field is E/N
             * per cell (m_fluid.f90:339-348) */
            const int ng = fl->d.n_gas_species;
            double field;
            double dens[AFH_MAX_SPECIES + AFH_MAX_GAS_SPECIES];
            double der[AFH_MAX_SPECIES + AFH_MAX_GAS_SPECIES];
            if (fl->d.i_gas_dens > 0) {
              const double Nc = ccb(t, fl->d.i_gas_dens, id)[x];
              field = 1e21 * (E[x] / Nc);
              for (int g = 0; g < ng; g++) {
                double v = fl->d.gas_fractions[g] * Nc;
                dens[g] = v > 0.0 ? v : 0.0;
                der[g] = 0.0;
              }
            } else {
              double tmpN = 1 / fl->d.gas_number_density;
              field = 1e21 * tmpN * E[x];
            }
            for (int s = 0; s < ns; s++) {
              double v = ccb(t, fl->d.species_iv[s] + s_deriv, id)[x];
              dens[ng + s] = v > 0.0 ? v : 0.0; /* max(dens, 0.0_dp) */
              der[ng + s] = 0.0;
            }
            double Te = -1.0; /* electron temperature, looked up once */
            for (int r = 0; r < nr; r++) {
              const afh_reaction *R = &fl->reac[r];
              double rate = rate_of(fl, R, field, &Te);
              double prod = 1.0;
              for (int m = 0; m < R->n_in; m++) prod = prod * dens[R->ix_in[m] - 1];
              rate = rate * prod;
              for (int m = 0; m < R->n_in; m++)
                der[R->ix_in[m] - 1] = der[R->ix_in[m] - 1] - rate;
              for (int m = 0; m < R->n_out; m++)
                der[R->ix_out[m] - 1] =
                    der[R->ix_out[m] - 1] + rate * R->mult_out[m];
            }
            if (last_step && any_mask) {
              for (int s = 0; s < ng + ns; s++) {
                double a, b;
                if (fl->d.dt_chemistry_nmin > 0) {
                  a = dens[s] + fl->d.dt_chemistry_nmin;
                  b = fabs(der[s]);
                  b = b > eps ? b : eps;
                } else {
                  a = dens[s] > eps ? dens[s] : eps;
                  b = -der[s] > eps ? -der[s] : eps;
                }
                double r = a / b;
                if (r < chem_min) chem_min = r;
              }
            }
            if (!upd) continue; /* masked: the weighted sum only */
            /* photoionization (m_fluid.f90:435-440) */
            if (fl->d.i_photo > 0) {
              const double pho = ccb(t, fl->d.i_photo, id)[x];
              for (int s = 0; s < ns; s++)
                if (fl->d.species_iv[s] == fl->d.i_electron) der[ng + s] = der[ng + s] + pho;
              der[ng + fl->d.photo_species - 1] = der[ng + fl->d.photo_species - 1] + pho;
            }
            for (int s = 0; s < ns; s++) {
              double *o = ccb(t, fl->d.species_iv[s] + s_out, id);
              o[x] = o[x] + dt * der[ng + s];
            }
            /* flux divergence for the electrons */
            double *o = ccb(t, fl->d.i_electron + s_out, id);
            o[x] = o[x] +
                   dt_dr[0] * (F[FX(t, 0, i, j, k)] - F[FX(t, 0, i + 1, j, k)]) +
                   dt_dr[1] * (F[FX(t, 1, i, j, k)] - F[FX(t, 1, i, j + 1, k)]) +
                   dt_dr[2] * (F[FX(t, 2, i, j, k)] - F[FX(t, 2, i, j, k + 1)]);
            /* and for the mobile ions (i_cc_flux 2..) */
            for (int q = 0; q < fl->d.n_ions; q++) {
              const double *G = fcb(t, fl->d.f_ion_flux[q], id);
              double *oi = ccb(t, fl->d.species_iv[fl->d.ion_species[q] - 1] + s_out, id);
              oi[x] = oi[x] +
                      dt_dr[0] * (G[FX(t, 0, i, j, k)] - G[FX(t, 0, i + 1, j, k)]) +
                      dt_dr[1] * (G[FX(t, 1, i, j, k)] - G[FX(t, 1, i, j + 1, k)]) +
                      dt_dr[2] * (G[FX(t, 2, i, j, k)] - G[FX(t, 2, i, j, k + 1)]);
            }
          }
    }
  }
  /* field_set_rhs of the new state folded into the update (the device does
   * it in the same pass); max|rhs| over the leaf interiors, hook deferred to
   * afo_fluid_rhs_maxabs as on the device */
  fl->rhs_state = -1;
  if (fl->rhs_iv > 0 && fl->rhs_ghosts) {
    int32_t e = afo_field_set_rhs(fl, fl->rhs_iv, s_out);
    if (e) return e;
  } else if (fl->rhs_iv > 0) {
    /* interiors only, the arithmetic of afo_field_set_rhs */
    const double fac = -1.6022e-19 / 8.8541878176e-12;
    for (int l = 1; l <= t->nlvl; l++)
      for (int q = 0; q < LVL_N(t, leaves, l); q++) {
        const int id = LVL_AT(t, leaves, l, q);
        double *r = ccb(t, fl->rhs_iv, id);
        for (int k = 1; k <= nc; k++)
          for (int j = 1; j <= nc; j++)
            for (int i = 1; i <= nc; i++) {
              const size_t x = IX(t, i, j, k);
              double v = 0.0;
              for (int s = 0; s < fl->d.n_species; s++) {
                if (fl->d.species_charge[s] == 0) continue;
                v = v + fl->d.species_charge[s] * fac *
                            ccb(t, fl->d.species_iv[s] + s_out, id)[x];
              }
              r[x] = v;
            }
      }
  }
  if (fl->rhs_iv > 0) {
    double mx = 0.0;
    for (int l = 1; l <= t->nlvl; l++)
      for (int q = 0; q < LVL_N(t, leaves, l); q++) {
        const double *c = ccb(t, fl->rhs_iv, LVL_AT(t, leaves, l, q));
        for (int k = 1; k <= nc; k++)
          for (int j = 1; j <= nc; j++)
            for (int i = 1; i <= nc; i++) {
              const double v = fabs(c[IX(t, i, j, k)]);
              if (v > mx) mx = v;
            }
      }
    fl->rhs_max = mx;
    t->slot[AFH_SLOT_RHS] = mx;
  }
  for (int s = 0; s < fl->d.n_species; s++) touch(t, fl->d.species_iv[s] + s_out);
  if (fl->rhs_iv > 0) {
    touch(t, fl->rhs_iv);
    fl->rhs_state = s_out;
    fl->rhs_snap[0] = t->gen[fl->rhs_iv];
    for (int s = 0; s < fl->d.n_species; s++)
      fl->rhs_snap[s + 1] = t->gen[fl->d.species_iv[s] + s_out];
  }
  if (last_step && hook(t, AFH_HOOK_MIN, 0, 0, &chem_min, 1)) return AFH_ERR_STATE;
  dt_lim[0] = last_step ? chem_min : 1e100;
  dt_lim[1] = 1e100;
  return AFH_OK;
}

/* The species part of forward_euler (src/m_fluid.f90:56-70):
 * flux_upwind_tree then flux_update_densities. store_flux is a device
 * option (the face fluxes are always stored here). */
int32_t afo_fluid_forward_euler(afh_fluid *f, double dt, int32_t s_deriv,
                                int32_t n_prev, const int32_t *s_prev,
                                const double *w_prev, int32_t s_out,
                                int32_t last_step, int32_t store_flux,
                                double *dt_lim) {
  (void)store_flux;
  double a[2], b[2];
  int32_t e;
  if ((e = afo_flux_upwind_tree(f, s_deriv, a))) return e;
  /* secondary emission from ions at the walls (m_fluid.f90:63-67) */
  if (f->d.n_ions > 0 && f->ion_se_yield > 0 && (e = afo_fluid_ion_se_flux(f))) return e;
  if ((e = afo_flux_update_densities(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out,
                                     last_step, b)))
    return e;
  dt_lim[0] = a[0], dt_lim[1] = a[1], dt_lim[2] = b[0], dt_lim[3] = b[1];
  return AFH_OK;
}

/* afh_fluid_forward_euler_fold / afh_fluid_fetch_step: the limits kept on
 * the tree until they are read (slots 0..2 hold dt_lim(1:3)) */
int32_t afo_fluid_forward_euler_fold(afh_fluid *f, double dt, int32_t s_deriv,
                                     int32_t n_prev, const int32_t *s_prev,
                                     const double *w_prev, int32_t s_out,
                                     int32_t last_step, int32_t store_flux) {
  double lim[4];
  int32_t e = afo_fluid_forward_euler(f, dt, s_deriv, n_prev, s_prev, w_prev, s_out,
                                      last_step, store_flux, lim);
  if (e) return e;
  for (int q = 0; q < 3; q++) f->t->slot[q] = lim[q];
  return AFH_OK;
}

int32_t afo_fluid_fetch_step(afh_fluid *f, int32_t last_step, int32_t n_extra,
                             const int32_t *extra_slots, double *dt_lim, double *extra) {
  afh_tree *t = f->t;
  LIVE(t);
  if (n_extra < 0 || n_extra > 2) return fail(AFH_ERR_ARG, "%d extra slots", n_extra);
  dt_lim[0] = t->slot[0], dt_lim[1] = t->slot[1];
  dt_lim[2] = last_step ? t->slot[2] : 1e100;
  dt_lim[3] = 1e100;
  return n_extra ? afo_tree_fetch_reduced(t, n_extra, extra_slots, extra) : AFH_OK;
}

/* Kernel timing is a device concept; the oracle accepts and ignores it. */
int32_t afo_profile_enable(afh_tree *t, int32_t kclass) {
  (void)t, (void)kclass;
  return AFH_OK;
}
int32_t afo_profile_read(afh_tree *t, double *ms, int64_t *n, double *bytes) {
  (void)t;
  *ms = 0, *n = 0, *bytes = 0;
  return AFH_OK;
}

/* ---------------------------------------------------------------- sharding
 * Host-side plans: copy the cells of box regions (id, lo[3], hi[3]) between
 * a variable and a packed buffer, i fastest, regions in order. */
int32_t afo_tree_set_stream(afh_tree *t, void *stream) {
  (void)t, (void)stream; /* host library: nothing to order */
  return AFH_OK;
}

int32_t afo_tree_set_hook(afh_tree *t, afh_hook_fn fn, void *ctx) {
  t->hook = fn;
  t->hook_ctx = ctx;
  return AFH_OK;
}

static int32_t plan_create(afh_tree *t, const int32_t *reg, int32_t n,
                           int32_t *plan, int64_t *n_values, int fc) {
  if (n < 0 || (n > 0 && !reg) || !plan || !n_values)
    return fail(AFH_ERR_ARG, "afo_plan_create: bad argument");
  int w = fc ? 8 : 7, lo = fc ? 2 : 1, vmin = fc ? 1 : 0;
  struct afo_plan p;
  p.n = n;
  p.fc = fc;
  p.reg = malloc(sizeof(int32_t) * w * (n > 0 ? n : 1));
  p.off = malloc(sizeof(int64_t) * (n + 1));
  p.off[0] = 0;
  for (int r = 0; r < n; r++) {
    const int32_t *q = reg + w * r;
    if (q[0] < 1 || q[0] > t->nb) return fail(AFH_ERR_ARG, "plan: bad box id");
    if (fc && (q[1] < 0 || q[1] > 2)) return fail(AFH_ERR_ARG, "plan: bad dim");
    int64_t cells = 1;
    for (int d = 0; d < 3; d++) {
      if (q[lo + d] < vmin || q[lo + 3 + d] > t->nc + 1 || q[lo + 3 + d] < q[lo + d])
        return fail(AFH_ERR_ARG, "plan: bad region");
      cells *= q[lo + 3 + d] - q[lo + d] + 1;
    }
    p.off[r + 1] = p.off[r] + cells;
  }
  if (n > 0) memcpy(p.reg, reg, sizeof(int32_t) * w * n);
  t->plans = realloc(t->plans, sizeof(struct afo_plan) * (t->nplans + 1));
  t->plans[t->nplans] = p;
  *plan = t->nplans++;
  *n_values = p.off[n];
  return AFH_OK;
}

int32_t afo_plan_create(afh_tree *t, const int32_t *reg, int32_t n,
                        int32_t *plan, int64_t *n_values) {
  return plan_create(t, reg, n, plan, n_values, 0);
}

int32_t afo_plan_create_fc(afh_tree *t, const int32_t *reg, int32_t n,
                           int32_t *plan, int64_t *n_values) {
  return plan_create(t, reg, n, plan, n_values, 1);
}

static int32_t plan_copy(afh_tree *t, int32_t plan, int32_t iv, double *buf,
                         int unpack) {
  if (plan < 0 || plan >= t->nplans)
    return fail(AFH_ERR_ARG, "afo_plan_pack/unpack: bad plan");
  struct afo_plan *p = &t->plans[plan];
  if (p->fc) {
    if (iv < 1 || iv > t->nvf) return fail(AFH_ERR_ARG, "plan: bad variable");
    for (int r = 0; r < p->n; r++) {
      const int32_t *q = p->reg + 8 * r;
      double *c = fcb(t, iv, q[0]), *b = buf + p->off[r];
      for (int k = q[4]; k <= q[7]; k++)
        for (int j = q[3]; j <= q[6]; j++)
          for (int i = q[2]; i <= q[5]; i++) {
            if (unpack) c[FX(t, q[1], i, j, k)] = *b;
            else *b = c[FX(t, q[1], i, j, k)];
            b++;
          }
    }
    return AFH_OK;
  }
  if (iv < 1 || iv > t->nvc) return fail(AFH_ERR_ARG, "plan: bad variable");
  for (int r = 0; r < p->n; r++) {
    const int32_t *q = p->reg + 7 * r;
    double *c = ccb(t, iv, q[0]), *b = buf + p->off[r];
    for (int k = q[3]; k <= q[6]; k++)
      for (int j = q[2]; j <= q[5]; j++)
        for (int i = q[1]; i <= q[4]; i++) {
          if (unpack) c[IX(t, i, j, k)] = *b;
          else *b = c[IX(t, i, j, k)];
          b++;
        }
  }
  return AFH_OK;
}

int32_t afo_plan_pack(afh_tree *t, int32_t plan, int32_t iv, double *buf) {
  return plan_copy(t, plan, iv, buf, 0);
}

int32_t afo_plan_unpack(afh_tree *t, int32_t plan, int32_t iv,
                        const double *buf) {
  if (t && plan >= 0 && plan < t->nplans && !t->plans[plan].fc && iv > 0) touch(t, iv);
  return plan_copy(t, plan, iv, (double *)buf, 1);
}

/* ------------------------------------------------------------ regrid */

/* The prolongation of variable iv used when boxes are added
 * (tree%cc_methods(iv)%prolong / prolong_limiter, af_set_cc_methods,
 * m_af_core.f90:343-420); registering it makes iv an automatic variable
 * (tree%cc_auto_vars, in registration order) that af_adjust_refinement
 * restricts into derefined parents and prolongs into new boxes. */
int32_t afo_set_cc_prolong(afh_tree *t, int32_t iv, int32_t method, int32_t lim) {
  if (!t || iv < 1 || iv > t->nvc) return fail(AFH_ERR_ARG, "bad variable index");
  if (method < AFH_PROLONG_NONE || method > AFH_PROLONG_LIMIT)
    return fail(AFH_ERR_UNSUPPORTED, "prolongation method %d", method);
  if (!t->meth[iv].set) return fail(AFH_ERR_STATE, "set cc methods first");
  int known = 0;
  for (int q = 0; q < t->n_auto; q++) known |= t->auto_vars[q] == iv;
  if (!known && method != AFH_PROLONG_NONE) t->auto_vars[t->n_auto++] = iv;
  t->meth[iv].prolong = method;
  t->meth[iv].prolong_lim = lim;
  return AFH_OK;
}

/* af_prolong_limit, m_af_prolong.f90:311-420 (3D, add = .false.: the child
 * interior starts at 0 and each value is f0 +- f1 +- f2 +- f3 + 0) */
static void prolong_limit(afh_tree *t, int p_id, int c_id, int iv, int lim) {
  int nc = t->nc, hnc = nc / 2, off[3];
  child_offset(t, c_id, 0, off);
  const double *p = ccb(t, iv, p_id);
  double *c = ccb(t, iv, c_id);
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++) c[IX(t, i, j, k)] = 0;
  for (int k = 1; k <= hnc; k++)
    for (int j = 1; j <= hnc; j++)
      for (int i = 1; i <= hnc; i++) {
        int ic = i + off[0], jc = j + off[1], kc = k + off[2];
        int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
        double f0 = p[IX(t, ic, jc, kc)];
        double a[3] = {f0 - p[IX(t, ic - 1, jc, kc)], f0 - p[IX(t, ic, jc - 1, kc)],
                       f0 - p[IX(t, ic, jc, kc - 1)]};
        double b[3] = {p[IX(t, ic + 1, jc, kc)] - f0, p[IX(t, ic, jc + 1, kc)] - f0,
                       p[IX(t, ic, jc, kc + 1)] - f0};
        double f[3];
        for (int d = 0; d < 3; d++) f[d] = 0.25 * limiter(lim, a[d], b[d]);
        for (int q = 0; q < 8; q++) {
          double sx = (q & 1) ? f[0] : -f[0];
          size_t x = IX(t, fi + (q & 1), fj + ((q >> 1) & 1), fk + (q >> 2));
          double v = f0 + sx;
          v = ((q >> 1) & 1) ? v + f[1] : v - f[1];
          v = (q >> 2) ? v + f[2] : v - f[2];
          c[x] = v + c[x];
        }
      }
}

/* af_prolong_linear, m_af_prolong.f90:531-679 (3D, add = .false.) */
static void prolong_linear(afh_tree *t, int p_id, int c_id, int iv) {
  const double f1 = 1 / 64.0, f3 = 3 / 64.0, f9 = 9 / 64.0, f27 = 27 / 64.0;
  int nc = t->nc, hnc = nc / 2, off[3];
  child_offset(t, c_id, 0, off);
  const double *p = ccb(t, iv, p_id);
  double *c = ccb(t, iv, c_id);
  for (int k = 1; k <= nc; k++)
    for (int j = 1; j <= nc; j++)
      for (int i = 1; i <= nc; i++) c[IX(t, i, j, k)] = 0;
#define P(a, b, d) p[IX(t, ic + (a), jc + (b), kc + (d))]
  for (int k = 1; k <= hnc; k++)
    for (int j = 1; j <= hnc; j++)
      for (int i = 1; i <= hnc; i++) {
        int ic = i + off[0], jc = j + off[1], kc = k + off[2];
        int fi = 2 * i - 1, fj = 2 * j - 1, fk = 2 * k - 1;
        double f000 = f27 * P(0, 0, 0);
        double f00l = f9 * P(0, 0, -1), f0l0 = f9 * P(0, -1, 0), f0ll = f3 * P(0, -1, -1);
        double fl00 = f9 * P(-1, 0, 0), fl0l = f3 * P(-1, 0, -1), fll0 = f3 * P(-1, -1, 0);
        double flll = f1 * P(-1, -1, -1);
        double f00h = f9 * P(0, 0, 1), f0h0 = f9 * P(0, 1, 0), f0hh = f3 * P(0, 1, 1);
        double fh00 = f9 * P(1, 0, 0), fh0h = f3 * P(1, 0, 1), fhh0 = f3 * P(1, 1, 0);
        double fhhh = f1 * P(1, 1, 1);
        double fl0h = f3 * P(-1, 0, 1), fh0l = f3 * P(1, 0, -1), flh0 = f3 * P(-1, 1, 0);
        double fhl0 = f3 * P(1, -1, 0), f0lh = f3 * P(0, -1, 1), f0hl = f3 * P(0, 1, -1);
        double fllh = f1 * P(-1, -1, 1), flhl = f1 * P(-1, 1, -1), fhll = f1 * P(1, -1, -1);
        double fhhl = f1 * P(1, 1, -1), fhlh = f1 * P(1, -1, 1), flhh = f1 * P(-1, 1, 1);
        double *o;
#define W(di, dj, dk, expr) o = &c[IX(t, fi + di, fj + dj, fk + dk)]; *o = expr + *o;
        W(0, 0, 0, f000 + fl00 + f0l0 + f00l + fll0 + fl0l + f0ll + flll)
        W(1, 0, 0, f000 + fh00 + f0l0 + f00l + fhl0 + fh0l + f0ll + fhll)
        W(0, 1, 0, f000 + fl00 + f0h0 + f00l + flh0 + fl0l + f0hl + flhl)
        W(1, 1, 0, f000 + fh00 + f0h0 + f00l + fhh0 + fh0l + f0hl + fhhl)
        W(0, 0, 1, f000 + fl00 + f0l0 + f00h + fll0 + fl0h + f0lh + fllh)
        W(1, 0, 1, f000 + fh00 + f0l0 + f00h + fhl0 + fh0h + f0lh + fhlh)
        W(0, 1, 1, f000 + fl00 + f0h0 + f00h + flh0 + fl0h + f0hh + flhh)
        W(1, 1, 1, f000 + fh00 + f0h0 + f00h + fhh0 + fh0h + f0hh + fhhh)
#undef W
      }
#undef P
}

/* af_adjust_refinement's data movement (m_af_core.f90:697-822) given the new
 * topology in `d` (box ids as afivo keeps them: a box of the old tree that
 * is in the new level lists with the same level and index persists):
 * auto_restrict (826-840) of every automatic variable into boxes whose
 * children were removed, the old data of persisting boxes, then
 * auto_prolong (843-881): level by level, each new box's automatic
 * variables prolonged from its parent and their ghost cells filled
 * (af_gc_box with corners). Variables without a prolongation method start at
 * 0 in new boxes. Returns the new tree (the old one is left as it was, apart
 * from the restricted parents). */
int32_t afo_tree_regrid(afh_tree *o, const afh_tree_desc *d, afh_tree **out) {
  if (!o || !d || !out) return fail(AFH_ERR_ARG, "afo_tree_regrid: null");
  LIVE(o);
  const int in_place = (d->n_boxes > d->box_capacity ? d->n_boxes : d->box_capacity) <= o->cap;
  if (d->n_cell != o->nc || d->n_var_cell != o->nvc || d->n_var_face != o->nvf)
    return fail(AFH_ERR_ARG, "afo_tree_regrid: box size / variables differ");
  afh_tree *t;
  int32_t e;
  if ((e = afo_tree_create(d, -1, &t))) return e;
  memcpy(t->meth, o->meth, sizeof(cc_method) * (o->nvc + 1));
  t->n_auto = o->n_auto;
  memcpy(t->auto_vars, o->auto_vars, sizeof(int) * (o->nvc + 1));
  t->hook = o->hook, t->hook_ctx = o->hook_ctx;
  char *in_old = calloc(o->nb + 1, 1), *keep = calloc(t->nb + 1, 1);
  for (int q = 0; q < o->ids_off[o->nlvl]; q++) in_old[o->ids[q]] = 1;
  for (int q = 0; q < t->ids_off[t->nlvl]; q++) {
    int id = t->ids[q];
    if (id <= o->nb && in_old[id] && B(o, id)->lvl == B(t, id)->lvl &&
        B(o, id)->ix[0] == B(t, id)->ix[0] && B(o, id)->ix[1] == B(t, id)->ix[1] &&
        B(o, id)->ix[2] == B(t, id)->ix[2])
      keep[id] = 1;
  }
  /* auto_restrict: persisting boxes that lost their children */
  for (int id = 1; id <= t->nb; id++) {
    if (!keep[id] || B(o, id)->children[0] <= 0 || B(t, id)->children[0] != 0) continue;
    for (int c = 0; c < 8; c++)
      for (int q = 0; q < o->n_auto; q++)
        restrict_box(o, B(o, id)->children[c], id, o->auto_vars[q]);
  }
  for (int id = 1; id <= t->nb; id++) {
    if (!keep[id]) continue;
    for (int iv = 1; iv <= t->nvc; iv++)
      memcpy(ccb(t, iv, id), ccb(o, iv, id), sizeof(double) * t->bsz);
    for (int iv = 1; iv <= t->nvf; iv++)
      memcpy(fcb(t, iv, id), fcb(o, iv, id), sizeof(double) * t->fsz);
  }
  /* auto_prolong */
  for (int l = 2; l <= t->nlvl; l++) {
    int n = LVL_N(t, ids, l);
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, ids, l, q);
      if (keep[id]) continue;
      for (int a = 0; a < t->n_auto; a++) {
        int iv = t->auto_vars[a];
        if (t->meth[iv].prolong == AFH_PROLONG_LIMIT)
          prolong_limit(t, B(t, id)->parent, id, iv, t->meth[iv].prolong_lim);
        else
          prolong_linear(t, B(t, id)->parent, id, iv);
      }
    }
    for (int q = 0; q < n; q++) {
      int id = LVL_AT(t, ids, l, q);
      if (keep[id]) continue;
      for (int a = 0; a < t->n_auto; a++) gc_box(t, id, t->auto_vars[a], 1);
    }
  }
  free(in_old), free(keep);
  t->cap = in_place ? o->cap : t->cap;
  if (in_place) o->retired = 1;
  *out = t;
  return AFH_OK;
}

/* ------------------------------------------------------------ refinement */

/* GM_dist_line (src/m_geometry.f90:23-51): distance from r to the segment
 * r0-r1 (norm2 as sqrt of the sum of squares) */
static double dist_line(const double r[3], const double r0[3], const double r1[3]) {
  double len2 = 0, frac = 0, dv[3];
  for (int d = 0; d < 3; d++) len2 = len2 + (r1[d] - r0[d]) * (r1[d] - r0[d]);
  for (int d = 0; d < 3; d++) frac = frac + (r[d] - r0[d]) * (r1[d] - r0[d]);
  if (frac <= 0.0) {
    for (int d = 0; d < 3; d++) dv[d] = r[d] - r0[d];
  } else if (frac >= len2) {
    for (int d = 0; d < 3; d++) dv[d] = r[d] - r1[d];
  } else {
    for (int d = 0; d < 3; d++) dv[d] = r[d] - (r0[d] + frac / len2 * (r1[d] - r0[d]));
  }
  return sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
}

/* default_refinement for cell (i, j, k) of box id (src/m_refine.f90:198-298,
 * constant gas density), the box-level rules applied per cell in the order
 * the reference applies them to the whole array */
static int refine_cell(afh_fluid *fl, const afh_refine_desc *p, int id, int elec,
                       int i, int j, int k) {
  afh_tree *t = fl->t;
  const afh_box_meta *b = B(t, id);
  int nc = t->nc;
  double min_dx = b->dr[0], max_dx = b->dr[0];
  for (int d = 1; d < 3; d++) {
    if (b->dr[d] < min_dx) min_dx = b->dr[d];
    if (b->dr[d] > max_dx) max_dx = b->dr[d];
  }
  size_t x = IX(t, i, j, k);
  /* m_refine.f90:219-223: the cell's gas density when it varies */
  double gas_dens = fl->d.i_gas_dens > 0 ? ccb(t, fl->d.i_gas_dens, id)[x]
                                         : fl->d.gas_number_density;
  double fld = ccb(t, p->i_efld, id)[x] * 1e21 / gas_dens;  /* SI_to_Townsend */
  double alpha;
  if (p->use_alpha_effective) {
    alpha = (lt_col(&fl->d.td, p->td_alpha_col, p->adx_fac * fld) -
             lt_col(&fl->d.td, p->td_eta_col, p->adx_fac * fld)) *
            gas_dens / p->adx_fac;
    alpha = alpha > 0.0 ? alpha : 0.0;
  } else {
    alpha = lt_col(&fl->d.td, p->td_alpha_col, p->adx_fac * fld) * gas_dens / p->adx_fac;
  }
  double adx = max_dx * alpha, ne = ccb(t, p->i_electron, id)[x];
  int f;
  if (adx > p->adx && ne > p->min_dens) f = AFH_DO_REF;
  else if (adx < 0.125 * p->adx && max_dx < p->derefine_dx) f = AFH_RM_REF;
  else f = AFH_KEEP_REF;
  double r[3] = {b->r_min[0] + (i - 0.5) * b->dr[0], b->r_min[1] + (j - 0.5) * b->dr[1],
                 b->r_min[2] + (k - 0.5) * b->dr[2]};
  for (int n = 0; n < p->n_seeds; n++) {
    double dist = dist_line(r, p->seed_r0[n], p->seed_r1[n]);
    if (dist - p->seed_width[n] < 2 * max_dx && max_dx > p->init_fac * p->seed_width[n])
      f = AFH_DO_REF;
  }
  if (elec && max_dx > p->electrode_dx) f = AFH_DO_REF;
  double rmin[3], rmax[3];
  for (int d = 0; d < 3; d++) rmin[d] = b->r_min[d], rmax[d] = b->r_min[d] + b->dr[d] * nc;
  for (int n = 0; n < p->n_regions; n++) {
    int in = max_dx > p->region_dr[n];
    for (int d = 0; d < 3; d++)
      in = in && rmax[d] >= p->region_rmin[n][d] && rmin[d] <= p->region_rmax[n][d];
    if (in && i == nc / 2 && j == nc / 2 && k == nc / 2) f = AFH_DO_REF;
  }
  for (int n = 0; n < p->n_limits; n++) {
    int in = max_dx < 2 * p->limit_dr[n];
    for (int d = 0; d < 3; d++)
      in = in && rmin[d] >= p->limit_rmin[n][d] && rmax[d] <= p->limit_rmax[n][d];
    if (in && f == AFH_DO_REF) f = AFH_KEEP_REF;
  }
  if (max_dx > p->max_dx) f = AFH_DO_REF;
  else if (min_dx < 2 * p->min_dx && f == AFH_DO_REF) f = AFH_KEEP_REF;
  return f;
}

int32_t afo_refine_flags(afh_fluid *fl, const afh_refine_desc *p,
                         const uint8_t *electrode_box, int32_t *flags, uint32_t *masks) {
  if (!fl || !p || !flags || !masks) return fail(AFH_ERR_ARG, "afo_refine_flags: null");
  afh_tree *t = fl->t;
  if (p->n_seeds > AFH_MAX_REFINE_REGIONS || p->n_regions > AFH_MAX_REFINE_REGIONS ||
      p->n_limits > AFH_MAX_REFINE_REGIONS || p->buffer_width < 0 ||
      p->buffer_width > t->nc)
    return fail(AFH_ERR_ARG, "afo_refine_flags: bad descriptor");
  int nc = t->nc, bw = p->buffer_width;
  for (int q = 0; q < t->nb; q++) flags[q] = 0, masks[q] = 0;
#pragma omp parallel for schedule(dynamic)
  for (int q = 0; q < t->ids_off[t->nlvl]; q++) {
    int id = t->ids[q], any_do = 0, any_keep = 0;
    uint32_t m = 0;
    int elec = electrode_box ? electrode_box[id - 1] : 0;
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++)
        for (int i = 1; i <= nc; i++) {
          int f = refine_cell(fl, p, id, elec, i, j, k);
          if (f == AFH_DO_REF) {
            any_do = 1;
            if (bw > 0) {
              /* the neighbour slabs this cell lies in (cell_to_ref_flags) */
              int lo[3] = {i <= bw, j <= bw, k <= bw};
              int hi[3] = {i > nc - bw, j > nc - bw, k > nc - bw};
              for (int dk = -1; dk <= 1; dk++)
                for (int dj = -1; dj <= 1; dj++)
                  for (int di = -1; di <= 1; di++) {
                    if (!di && !dj && !dk) continue;
                    int dd[3] = {di, dj, dk}, in = 1;
                    for (int d = 0; d < 3; d++)
                      in = in && (dd[d] == 0 || (dd[d] < 0 ? lo[d] : hi[d]));
                    if (in) m |= 1u << ((dk + 1) * 9 + (dj + 1) * 3 + (di + 1));
                  }
            }
          } else if (f == AFH_KEEP_REF) {
            any_keep = 1;
          }
        }
    flags[id - 1] = any_do ? AFH_DO_REF : any_keep ? AFH_KEEP_REF : AFH_RM_REF;
    masks[id - 1] = m;
  }
  return AFH_OK;
}

/* Cell flags with the box summary (flag, mask) of afh_refine_flags, for the
 * driver's refinement routine (af_subr_ref) in af_adjust_refinement: a set
 * of cells asking for refinement whose cell_to_ref_flags result
 * (m_af_core.f90:1095-1148) is exactly (flag, mask); the other cells keep
 * (flag >= keep) or remove (flag = remove) the refinement. Per dimension a
 * cell index is in the low buffer slab, the high one, both or neither; one
 * representative cell per class combination whose neighbour slabs all lie in
 * the mask is marked when it adds a direction (or, for a box refining only
 * away from its sides, a cell in no slab). */
int32_t afo_refine_cell_flags(int32_t flag, uint32_t mask, int32_t nc, int32_t bw,
                               int32_t *cf) {
  if (nc < 1 || bw < 0 || bw > nc || !cf || flag < AFH_RM_REF || flag > AFH_DO_REF)
    return fail(AFH_ERR_ARG, "refine_cell_flags: bad argument");
  const size_t n3 = (size_t)nc * nc * nc;
  for (size_t q = 0; q < n3; q++) cf[q] = flag == AFH_RM_REF ? AFH_RM_REF : AFH_KEEP_REF;
  if (flag != AFH_DO_REF) return mask ? fail(AFH_ERR_ARG, "mask without refinement") : AFH_OK;
  int rep[4]; /* class -> first index (1-based) or 0; class = lo | hi << 1 */
  for (int c = 0; c < 4; c++) rep[c] = 0;
  for (int i = nc; i >= 1; i--) rep[(i <= bw) | ((i > nc - bw) << 1)] = i;
  uint32_t need = mask;
  int placed = 0;
  for (int pass = 0; pass < 2; pass++)
    for (int cz = 0; cz < 4; cz++)
      for (int cy = 0; cy < 4; cy++)
        for (int cx = 0; cx < 4; cx++) {
          if (!rep[cx] || !rep[cy] || !rep[cz]) continue;
          const int cl[3] = {cx, cy, cz};
          uint32_t mem = 0;
          for (int dk = -1; dk <= 1; dk++)
            for (int dj = -1; dj <= 1; dj++)
              for (int di = -1; di <= 1; di++) {
                if (!di && !dj && !dk) continue;
                const int dd[3] = {di, dj, dk};
                int in = 1;
                for (int d = 0; d < 3; d++)
                  in = in && (dd[d] == 0 || (cl[d] & (dd[d] < 0 ? 1 : 2)));
                if (in) mem |= 1u << ((dk + 1) * 9 + (dj + 1) * 3 + (di + 1));
              }
          if ((mem & ~mask) != 0) continue;
          /* pass 0: cells that add a direction; pass 1: any cell if none yet */
          if (pass == 0 ? (mem & need) == 0 : placed) continue;
          cf[((size_t)(rep[cz] - 1) * nc + (rep[cy] - 1)) * nc + (rep[cx] - 1)] = AFH_DO_REF;
          need &= ~mem;
          placed = 1;
        }
  if (need || !placed) return fail(AFH_ERR_ARG, "refine_cell_flags: inconsistent mask");
  return AFH_OK;
}

/* photoionization_rate_from_alpha, src/m_photoi.f90:217-253 (leaf interiors) */
int32_t afo_photoi_set_src(afh_fluid *f, int32_t i_rhs, int32_t alpha_col, double coeff) {
  afh_tree *t = f->t;
  LIVE(t);
  if (i_rhs < 1 || i_rhs > t->nvc || alpha_col < 1 || alpha_col > f->d.td.n_cols)
    return fail(AFH_ERR_ARG, "afo_photoi_set_src: bad argument");
  touch(t, i_rhs);
  const int nc = t->nc;
  const afh_lt *td = &f->d.td;
  for (int l = 1; l <= t->nlvl; l++)
    for (int q = 0; q < LVL_N(t, leaves, l); q++) {
      const int id = LVL_AT(t, leaves, l, q);
      const double *E = ccb(t, f->d.i_efld, id), *ne = ccb(t, f->d.i_electron, id);
      const double *Ng = f->d.i_gas_dens > 0 ? ccb(t, f->d.i_gas_dens, id) : NULL;
      double *r = ccb(t, i_rhs, id);
      for (int k = 1; k <= nc; k++)
        for (int j = 1; j <= nc; j++)
          for (int i = 1; i <= nc; i++) {
            const size_t x = IX(t, i, j, k);
            const double fld = E[x];
            const double gas_dens = Ng ? Ng[x] : f->d.gas_number_density;
            const double Td = fld * 1e21 / gas_dens;
            const double alpha = lt_col(td, alpha_col, Td);
            const double mobility = lt_col(td, 1, Td);
            double tmp = fld * mobility * alpha * ne[x] * coeff;
            if (tmp < 0) tmp = 0;
            r[x] = tmp;
          }
    }
  return AFH_OK;
}

/* photoi_helmh_compute, src/m_photoi_helmh.f90:162-204 */
int32_t afo_photoi_helmh_compute(afh_mg *const *modes, int32_t n_modes,
                                 const double *coeffs, int32_t i_photo,
                                 double max_rel_res, int32_t max_fmg,
                                 int32_t *n_fmg) {
  if (!modes || n_modes < 1 || !coeffs || max_fmg < 1)
    return fail(AFH_ERR_ARG, "afo_photoi_helmh_compute: bad argument");
  afh_tree *t = modes[0]->t;
  LIVE(t);
  if (i_photo < 1 || i_photo > t->nvc) return fail(AFH_ERR_ARG, "bad i_photo");
  touch(t, i_photo);
  memset(ccb(t, i_photo, 1), 0, sizeof(double) * t->bsz * t->nb);
  /* the source is the last mode's rhs; a mode with an rhs variable of its
     own solves with a copy of it (the library's concurrent modes; here one
     after another) */
  const int src = modes[n_modes - 1]->d.i_rhs;
  for (int n = 0; n + 1 < n_modes; n++)
    if (modes[n]->d.i_rhs != src) {
      touch(t, modes[n]->d.i_rhs);
      memcpy(ccb(t, modes[n]->d.i_rhs, 1), ccb(t, src, 1), sizeof(double) * t->bsz * t->nb);
    }
  double max_rhs;
  int32_t e;
  if ((e = afo_tree_maxabs_cc(t, src, &max_rhs))) return e;
  if (max_rhs < sqrt(DBL_EPSILON)) max_rhs = sqrt(DBL_EPSILON);
  for (int n = 0; n < n_modes; n++) {
    afh_mg *mg = modes[n];
    int i;
    for (i = 1; i <= max_fmg; i++) {
      double residu;
      if ((e = afo_mg_fas_fmg(mg, 1, 1)) ||
          (e = afo_tree_maxabs_cc(t, mg->d.i_tmp, &residu)))
        return e;
      if (residu / max_rhs < max_rel_res) break;
    }
    if (n_fmg) n_fmg[n] = i < max_fmg ? i : max_fmg;
    for (int l = 1; l <= t->nlvl; l++)
      for (int q = 0; q < LVL_N(t, leaves, l); q++) {
        const int id = LVL_AT(t, leaves, l, q);
        double *y = ccb(t, i_photo, id);
        const double *x = ccb(t, mg->d.i_phi, id);
        for (size_t c = 0; c < t->bsz; c++) y[c] = y[c] - coeffs[n] * x[c];
      }
  }
  return AFH_OK;
}
