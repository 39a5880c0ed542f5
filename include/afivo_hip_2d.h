/*
 * afivo_hip_2d.h -- the NDIM = 2 build of the C ABI (BASELINE config 1,
 * programs/standard_2d): libafivo_hip_2d.so.
 *
 * The reference builds its 2-D library from the same sources as the 3-D one
 * with NDIM=2 (afivo/lib_2d/Makefile); a program links one of the two. In the
 * same way libafivo_hip_2d.so exports the entry points below under the names
 * and with the argument meaning of include/afivo_hip.h (a 2-D Fortran driver
 * binds the same ISO_C_BINDING interfaces, afivo-streamer_amd/fortran/
 * m_afivo_hip.F90, against this library). Types are those of afivo_hip.h, read
 * with the 2-D conventions:
 *
 *   - afh_box_meta: ix[0..1], children[0..3] (af_child_dix order (0,0), (1,0),
 *     (0,1), (1,1)), neighbors[0..3] (lowx, highx, lowy, highy),
 *     neighbor_mat[0..8] = neighbor_mat(-1:1, -1:1) (i fastest), r_min[0..1],
 *     dr[0..1]; the remaining entries are ignored;
 *   - afh_tree_desc: coarse_grid_size[0..1], r_base / dr_base [0..1];
 *   - bc arrays of afh_set_cc_methods: bc[0..3]; afh_set_bc: nb = 1..4;
 *   - host arrays of afh_cc_put/get hold, per box, box%cc(0:nc+1, 0:nc+1, iv)
 *     (i fastest), boxes in id order; afh_fc_put/get box%fc(1:nc+1, 1:nc+1,
 *     1:2, ivf).
 *
 * Built: the tree with its ghost cells (af_gc_box with neighbour copy,
 * bc_to_gc, af_gc_interp / af_gc_interp_lim / mg_sides_rb, corners),
 * restriction, the FAS V-cycle and FMG of a Poisson / Helmholtz operator with
 * the exact level-1 solve (AFH_COARSE_DIRECT) or the reference's HYPRE PFMG
 * restated (AFH_COARSE_PFMG, round 5), the field gradient and
 * |E|, field_set_rhs, the species step (af_restrict_ref_boundary, af_gc2_box,
 * flux_upwind_box with the m_fluid callbacks, af_consistent_fluxes,
 * flux_update_densities with the field-dependent rate forms). Not built in
 * 2-D (AFH_ERR_UNSUPPORTED or not exported): cylindrical coordinates
 * (af_cyl), electrodes / level sets, variable gas density, photoionization,
 * the temperature rate forms, sharding, ion secondary emission. Built in
 * round 4 for the 2-D time loop (afh.driver over this library,
 * programs/standard_2d/tests/test_2d_rtest.log): the device regrid with the
 * prolongation of the automatic variables, default_refinement's flags, the
 * regression-log sums and extrema, and the deferred reductions
 * (afh_mg_fas_vcycle_fold, afh_fluid_forward_euler_fold,
 * afh_fluid_fetch_step, below).
 */
#ifndef AFIVO_HIP_2D_H
#define AFIVO_HIP_2D_H

#include "afivo_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

const char *afh_last_error(void);
int32_t afh_tree_create(const afh_tree_desc *desc, int32_t device, afh_tree **out);
int32_t afh_tree_destroy(afh_tree *t);
int32_t afh_tree_sync(afh_tree *t);
int32_t afh_set_cc_methods(afh_tree *t, int32_t iv, const afh_bc *bc6, int32_t rb,
                           int32_t prolong_limiter);
int32_t afh_set_bc(afh_tree *t, int32_t iv, int32_t nb, int32_t type, double value);
int32_t afh_cc_put(afh_tree *t, int32_t iv, const double *host);
int32_t afh_cc_get(afh_tree *t, int32_t iv, double *host);
int32_t afh_fc_put(afh_tree *t, int32_t ivf, const double *host);
int32_t afh_fc_get(afh_tree *t, int32_t ivf, double *host);
int32_t afh_gc_lvl(afh_tree *t, int32_t lvl, int32_t iv, int32_t corners);
int32_t afh_gc_tree(afh_tree *t, int32_t iv, int32_t corners);
int32_t afh_restrict_tree(afh_tree *t, int32_t iv);
int32_t afh_tree_copy_cc(afh_tree *t, int32_t iv_from, int32_t iv_to);
int32_t afh_tree_maxabs_cc(afh_tree *t, int32_t iv, double *out);
int32_t afh_mg_create(afh_tree *t, const afh_mg_desc *desc, afh_mg **out);
int32_t afh_mg_destroy(afh_mg *mg);
int32_t afh_mg_fas_vcycle(afh_mg *mg, int32_t set_residual, int32_t highest_lvl);
int32_t afh_mg_fas_vcycle_maxres(afh_mg *mg, int32_t highest_lvl, double *max_res);
/* deferred form: max|res| stays on the device for afh_fluid_fetch_step */
int32_t afh_mg_fas_vcycle_fold(afh_mg *mg, int32_t highest_lvl);
int32_t afh_mg_fas_fmg(afh_mg *mg, int32_t set_residual, int32_t have_guess);
int32_t afh_mg_compute_phi_gradient(afh_mg *mg, int32_t i_fc, double fac, int32_t i_norm);
int32_t afh_fluid_create(afh_tree *t, const afh_fluid_desc *desc, afh_fluid **out);
int32_t afh_fluid_destroy(afh_fluid *f);
int32_t afh_field_set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in);
int32_t afh_field_set_rhs_maxabs(afh_fluid *f, int32_t i_rhs, int32_t s_in,
                                 double *max_rhs);
int32_t afh_flux_upwind_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim);
int32_t afh_flux_update_densities(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                                  const int32_t *s_prev, const double *w_prev,
                                  int32_t s_out, int32_t last_step, double *dt_lim);
/* the device regrid (af_adjust_refinement's data movement, round 4): the
 * persisting boxes are copied into the new tree's pools (box_capacity is not
 * used in 2-D) */
int32_t afh_set_cc_prolong(afh_tree *t, int32_t iv, int32_t method, int32_t limiter);
int32_t afh_tree_regrid(afh_tree *old, const afh_tree_desc *desc, afh_tree **out);
/* default_refinement reduced per box; masks use the 2-D bit (dj+1)*3 + (di+1);
 * the seeds' / regions' first two coordinates; electrode_box must be NULL */
int32_t afh_refine_flags(afh_fluid *f, const afh_refine_desc *d,
                         const uint8_t *electrode_box, int32_t *flags,
                         uint32_t *masks);
/* kernel timing, as in afivo_hip.h: classes AFH_PROF_GSRB (k2_gsrb on
 * levels of >= 256 boxes, 16 B per cell of a half sweep), AFH_PROF_FLUX
 * (k2_flux, 48 B per leaf cell) and AFH_PROF_CS (the PFMG level-1 solve,
 * k2_cs_pfmg; 0 bytes) */
int32_t afh_profile_enable(afh_tree *t, int32_t kclass);
int32_t afh_profile_read(afh_tree *t, double *total_ms, int64_t *launches, double *bytes);
/* the output_regression_log reductions; loc = (id, i, j, 0) */
int32_t afh_tree_sum_cc(afh_tree *t, int32_t iv, int32_t power, double *out);
int32_t afh_tree_reduce_loc(afh_tree *t, int32_t iv, int32_t op, double *out,
                            int32_t *loc);
/* store_flux is ignored: the 2-D species step always stores the face fluxes */
int32_t afh_fluid_forward_euler(afh_fluid *f, double dt, int32_t s_deriv, int32_t n_prev,
                                const int32_t *s_prev, const double *w_prev, int32_t s_out,
                                int32_t last_step, int32_t store_flux, double *dt_lim);
/* Deferred reductions, as afivo_hip.h: the step's limits stay on the device
 * and afh_fluid_fetch_step reads them with at most one extra slot
 * (AFH_SLOT_MAXRES, the V-cycle residual of afh_mg_fas_vcycle_fold) in one
 * transfer. */
int32_t afh_fluid_forward_euler_fold(afh_fluid *f, double dt, int32_t s_deriv,
                                     int32_t n_prev, const int32_t *s_prev,
                                     const double *w_prev, int32_t s_out,
                                     int32_t last_step, int32_t store_flux);
int32_t afh_fluid_fetch_step(afh_fluid *f, int32_t last_step, int32_t n_extra,
                             const int32_t *extra_slots, double *dt_lim, double *extra);

#ifdef __cplusplus
}
#endif
#endif
