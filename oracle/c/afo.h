/*
 * ORACLE TEST INFRASTRUCTURE -- not product code.
 *
 * libafo.so: a plain-C CPU restatement of the afivo-streamer hot path, used as
 * the parity checker for the HIP library (tests/, __graft_entry__.smoke(),
 * bench.py cpu_baseline). Same signatures as include/afivo_hip.h with the
 * `afo_` prefix, so one Python wrapper drives either library. Each routine
 * cites the reference routine it restates. Pinned against the golden vectors
 * in tests/golden/ (generated from the reference's own afivo numerics, see
 * oracle/Makefile and oracle/make_golden.py).
 *
 * The level-1 solve: AFH_COARSE_PFMG restates the reference's own solver,
 * HYPRE 2.31.0 StructPFMG (absent here; afivo-streamer_amd/csrc/afh_pfmg.h
 * has the algorithm), pinned by the reference's regression logs (rows within
 * 5e-8, tests/test_rtest.py); AFH_COARSE_DIRECT / _CYCLES are our exact
 * solve and V(2,2) cycles. The boundary conditions are folded into the
 * operator as stencil_handle_boundaries does (m_coarse_solver.f90:442-491).
 */
#ifndef AFO_H
#define AFO_H
#include "../../include/afivo_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

const char *afo_last_error(void);
/* Test probe of the PFMG setup (afh_pfmg.h) on a folded 7-point operator a7
 * (7 per point): level count, coarsening direction, relaxed flag and Jacobi
 * weight per level (at most maxl). */
int32_t afo_pfmg_probe_full(int32_t nx, int32_t ny, int32_t nz, const double *a7, int32_t maxl,
                            int32_t *nl, int64_t *np, int32_t *dims, int32_t *cdir,
                            int32_t *active, double *w, int64_t *off, double *A, double *P);
int32_t afo_mg_pfmg_operator(afh_mg *mg, int32_t *dims, double *a7);
int32_t afo_pfmg_probe(int32_t nx, int32_t ny, int32_t nz, const double *a7, int32_t maxl,
                       int32_t *nl, int32_t *cdir, int32_t *active, double *w);
int32_t afo_tree_create(const afh_tree_desc *desc, int32_t device,
                        afh_tree **out);
int32_t afo_tree_destroy(afh_tree *t);
int32_t afo_tree_sync(afh_tree *t);
int32_t afo_set_cc_methods(afh_tree *t, int32_t iv, const afh_bc *bc6,
                           int32_t rb, int32_t prolong_limiter);
int32_t afo_set_bc(afh_tree *t, int32_t iv, int32_t nb, int32_t type,
                   double value);
int32_t afo_cc_put(afh_tree *t, int32_t iv, const double *host);
int32_t afo_cc_get(afh_tree *t, int32_t iv, double *host);
int32_t afo_fc_put(afh_tree *t, int32_t ivf, const double *host);
int32_t afo_fc_get(afh_tree *t, int32_t ivf, double *host);
int32_t afo_gc_lvl(afh_tree *t, int32_t lvl, int32_t iv, int32_t corners);
int32_t afo_gc_tree(afh_tree *t, int32_t iv, int32_t corners);
int32_t afo_restrict_tree(afh_tree *t, int32_t iv);
int32_t afo_tree_copy_cc(afh_tree *t, int32_t iv_from, int32_t iv_to);
int32_t afo_fluid_set_rhs_output(afh_fluid *f, int32_t i_rhs, int32_t ghosts);
int32_t afo_fluid_set_update_mask(afh_fluid *f, int32_t i_lsf);
int32_t afo_fluid_set_field_source(afh_fluid *f, int32_t i_phi, double fac);
int32_t afo_fluid_set_ion_se_yield(afh_fluid *f, double yield);
int32_t afo_fluid_ion_se_flux(afh_fluid *f);
int32_t afo_fluid_rhs_maxabs(afh_fluid *f, int32_t s_out, double *max_rhs);
int32_t afo_electrode_species_bc(afh_fluid *f, int32_t i_lsf, int32_t i_1pos_ion,
                                 int32_t neumann_zero, int32_t n_ids,
                                 const int32_t *ids);
int32_t afo_tree_maxabs_cc(afh_tree *t, int32_t iv, double *out);
int32_t afo_tree_sum_cc(afh_tree *t, int32_t iv, int32_t power, double *out);
int32_t afo_tree_reduce_loc(afh_tree *t, int32_t iv, int32_t op, double *out,
                            int32_t *loc);
int32_t afo_fluid_rhs_valid(afh_fluid *f, int32_t s_out, int32_t *valid);
int32_t afo_photoi_set_src(afh_fluid *f, int32_t i_rhs, int32_t alpha_col, double coeff);
int32_t afo_photoi_helmh_compute(afh_mg *const *modes, int32_t n_modes,
                                 const double *coeffs, int32_t i_photo,
                                 double max_rel_res, int32_t max_fmg,
                                 int32_t *n_fmg);
int32_t afo_mg_create(afh_tree *t, const afh_mg_desc *desc, afh_mg **out);
int32_t afo_mg_destroy(afh_mg *mg);
int32_t afo_mg_fas_vcycle(afh_mg *mg, int32_t set_residual,
                          int32_t highest_lvl);
int32_t afo_mg_fas_vcycle_maxres(afh_mg *mg, int32_t highest_lvl,
                                 double *max_res);
int32_t afo_mg_fas_vcycle_fold(afh_mg *mg, int32_t highest_lvl);
int32_t afo_tree_fetch_reduced(afh_tree *t, int32_t n, const int32_t *slots, double *out);
int32_t afo_mg_fas_fmg(afh_mg *mg, int32_t set_residual, int32_t have_guess);
int32_t afo_mg_coarse_iterations(afh_mg *mg, int32_t *n);
int32_t afo_mg_graph_stats(afh_mg *mg, int64_t *replays, int64_t *segmented);
int32_t afo_mg_set_gradient_output(afh_mg *mg, int32_t i_norm, double fac);
int32_t afo_mg_compute_phi_gradient(afh_mg *mg, int32_t i_fc, double fac,
                                    int32_t i_norm);
int32_t afo_mg_set_box_stencil(afh_mg *mg, int32_t id, const double *v,
                               const double *bc_correction);
int32_t afo_mg_set_box_lsf(afh_mg *mg, int32_t id, int32_t n, const int32_t *ix,
                           const double *dd, const double *bval, int32_t i_lsf);
int32_t afo_set_cc_prolong(afh_tree *t, int32_t iv, int32_t method, int32_t limiter);
int32_t afo_tree_regrid(afh_tree *old, const afh_tree_desc *desc, afh_tree **out);
int32_t afo_refine_flags(afh_fluid *f, const afh_refine_desc *d,
                         const uint8_t *electrode_box, int32_t *flags, uint32_t *masks);
int32_t afo_refine_cell_flags(int32_t flag, uint32_t mask, int32_t nc, int32_t bw,
                              int32_t *cell_flags);
int32_t afo_fluid_create(afh_tree *t, const afh_fluid_desc *desc,
                         afh_fluid **out);
int32_t afo_fluid_destroy(afh_fluid *f);
int32_t afo_field_set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in);
int32_t afo_field_set_rhs_maxabs(afh_fluid *f, int32_t i_rhs, int32_t s_in,
                                 double *max_rhs);
int32_t afo_flux_upwind_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim);
int32_t afo_flux_update_densities(afh_fluid *f, double dt, int32_t s_deriv,
                                  int32_t n_prev, const int32_t *s_prev,
                                  const double *w_prev, int32_t s_out,
                                  int32_t last_step, double *dt_lim);
int32_t afo_fluid_forward_euler(afh_fluid *f, double dt, int32_t s_deriv,
                                int32_t n_prev, const int32_t *s_prev,
                                const double *w_prev, int32_t s_out,
                                int32_t last_step, int32_t store_flux,
                                double *dt_lim);
int32_t afo_fluid_forward_euler_fold(afh_fluid *f, double dt, int32_t s_deriv,
                                     int32_t n_prev, const int32_t *s_prev,
                                     const double *w_prev, int32_t s_out,
                                     int32_t last_step, int32_t store_flux);
int32_t afo_fluid_fetch_step(afh_fluid *f, int32_t last_step, int32_t n_extra,
                             const int32_t *extra_slots, double *dt_lim, double *extra);
int32_t afo_profile_enable(afh_tree *t, int32_t kclass);
int32_t afo_profile_read(afh_tree *t, double *total_ms, int64_t *launches,
                         double *bytes);
int32_t afo_tree_set_hook(afh_tree *t, afh_hook_fn fn, void *ctx);
int32_t afo_tree_set_stream(afh_tree *t, void *hip_stream);
int32_t afo_plan_create(afh_tree *t, const int32_t *regions, int32_t n,
                        int32_t *plan, int64_t *n_values);
int32_t afo_plan_create_fc(afh_tree *t, const int32_t *regions, int32_t n,
                           int32_t *plan, int64_t *n_values);
int32_t afo_plan_pack(afh_tree *t, int32_t plan, int32_t iv, double *buf);
int32_t afo_plan_unpack(afh_tree *t, int32_t plan, int32_t iv,
                        const double *buf);
/* Debug hooks: the individual V-cycle stages (for golden trace tests). */
int32_t afo_mg_gsrb_boxes(afh_mg *mg, int32_t lvl, int32_t up);
int32_t afo_mg_update_coarse(afh_mg *mg, int32_t lvl);
int32_t afo_mg_solve_coarse(afh_mg *mg);
int32_t afo_mg_correct_children(afh_mg *mg, int32_t lvl);

/* native box sharding: the CPU twin of afh_dist_* (c/afo_dist.cpp);
 * AFH_DIST_LOCAL only (ranks are threads), the RCCL entry points refuse */
int32_t afo_dist_partition(const afh_tree_desc *desc, int32_t n_ranks, int32_t *owner,
                           int32_t *lp);
int32_t afo_dist_plan(const afh_tree_desc *desc, const int32_t *owner, int32_t kind,
                      int32_t level, int32_t recv_rank, int32_t send_rank, int32_t *regions,
                      int32_t cap, int32_t *n);
int32_t afo_dist_local_ids(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                          int32_t *ids, int32_t cap, int32_t *n);
int32_t afo_tree_create_sharded(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                                int32_t device, afh_tree **out);
int32_t afo_dist_group_create(int32_t n_ranks, afh_dist_group **out);
int32_t afo_dist_group_destroy(afh_dist_group *g);
int32_t afo_dist_rccl_unique_id(void *id128);
int32_t afo_dist_rccl_comm(const void *id128, int32_t rank, int32_t n_ranks, int32_t device,
                           void **comm);
int32_t afo_dist_rccl_comm_destroy(void *comm);
int32_t afo_dist_create(afh_tree *t, const afh_tree_desc *desc, const int32_t *owner,
                        int32_t rank, int32_t n_ranks, int32_t transport, void *group_or_comm,
                        afh_dist **out);
int32_t afo_dist_destroy(afh_dist *d);
int32_t afo_dist_stats(afh_dist *d, int64_t *n_exchanges, int64_t *bytes);

#ifdef __cplusplus
}
#endif
#endif
