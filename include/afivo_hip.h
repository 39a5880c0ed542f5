/*
 * afivo_hip.h -- C ABI of the MI355X-native afivo-streamer hot path.
 *
 * The symbols below are what an ISO_C_BINDING layer under the reference's
 * Fortran driver binds to (see INTEGRATION.md for the bind(C) stubs). Each
 * entry point replaces one reference interface on the per-timestep path; the
 * replaced routine is cited (file:line, paths relative to the reference root).
 *
 * Conventions (all mirror afivo so a Fortran caller passes its own numbers):
 *   - box ids are 1-based; 0 = af_no_box, -1 = af_phys_boundary
 *     (afivo/src/m_af_types.f90:37-40);
 *   - variable indices (iv for cell-centred, ivf for face-centred) are 1-based,
 *     state copies are consecutive indices (iv + s), as af_add_cc_variable
 *     with n_copies lays them out;
 *   - host arrays exchanged with afh_cc_put/get hold, per box, the Fortran
 *     array box%cc(0:nc+1,0:nc+1,0:nc+1,iv) (i fastest), boxes in id order;
 *     afh_fc_put/get hold box%fc(1:nc+1,1:nc+1,1:nc+1,1:3,ivf);
 *   - every call returns AFH_OK (0) or a negative AFH_ERR_* code;
 *     afh_last_error() gives a message (the Fortran shim turns it into
 *     `error stop`, as the reference does on failure);
 *   - all device work of one tree is ordered on one HIP stream; calls are
 *     asynchronous unless they return host data (maxabs, dt limits, get).
 *
 * No torch types, no C++ types: plain pointers and sizes.
 */
#ifndef AFIVO_HIP_H
#define AFIVO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AFH_OK 0
#define AFH_ERR_ARG -1
#define AFH_ERR_UNSUPPORTED -2
#define AFH_ERR_DEVICE -3
#define AFH_ERR_STATE -4

/* Boundary-condition types, afivo/src/m_af_types.f90:51-64 */
#define AFH_BC_DIRICHLET -10
#define AFH_BC_NEUMANN -11
#define AFH_BC_CONTINUOUS -12
#define AFH_BC_DIRICHLET_COPY -13

/* Refinement-boundary ghost-cell methods (tree%cc_methods(iv)%rb) */
#define AFH_RB_GC_INTERP 1     /* af_gc_interp, m_af_ghostcell.f90:394-498 */
#define AFH_RB_GC_INTERP_LIM 2 /* af_gc_interp_lim, m_af_ghostcell.f90:503-612 */
#define AFH_RB_MG_SIDES 3      /* mg_sides_rb, m_af_multigrid.f90:294-461 */

/* Limiters, afivo/src/m_af_limiters.f90:12-25 */
#define AFH_LIM_NONE 1
#define AFH_LIM_VANLEER 2
#define AFH_LIM_KOREN 3
#define AFH_LIM_MINMOD 4
#define AFH_LIM_MC 5
#define AFH_LIM_GMINMOD43 6
#define AFH_LIM_ZERO 7

/* Reaction rate types, src/m_chemistry.f90:58-115 (numbers as there; Td =
 * reduced field, Te from the transport table's mean-energy column, Tg =
 * gas temperature). rate_tabulated_energy (0) needs the energy equation
 * (LEA) and is not on the LFA path: rejected. */
#define AFH_RATE_TABULATED_FIELD 1 /* c0 * table(Td) */
#define AFH_RATE_CONSTANT 2        /* c0 c1 */
#define AFH_RATE_LINEAR 3          /* c0 c1 (Td - c2) */
#define AFH_RATE_EXP_V1 4          /* c0 c1 exp(-(c2 / (c3 + Td))^2) */
#define AFH_RATE_EXP_V2 5          /* c0 c1 exp(-(Td / c2)^2) */
#define AFH_RATE_K1 6              /* c0 c1 (300 / Te)^c2 */
#define AFH_RATE_K3 8              /* c0 (c1 (kB/eV Te + c2)^2 - c3) c4 */
#define AFH_RATE_K4 9              /* c0 c1 (Tg / 300)^c2 exp(-c3 / Tg) */
#define AFH_RATE_K5 10             /* c0 c1 exp(-c2 / Tg) */
#define AFH_RATE_K6 11             /* c0 c1 Tg^c2 */
#define AFH_RATE_K7 12             /* c0 c1 (Tg / c2)^c3 */
#define AFH_RATE_K8 13             /* c0 c1 (300 / Tg)^c2 */
#define AFH_RATE_K9 14             /* c0 c1 exp(-c2 Tg) */
#define AFH_RATE_K10 15            /* c0 10^(c1 + c2 (Tg - 300)) */
#define AFH_RATE_K11 16            /* c0 c1 (300 / Tg)^c2 exp(-c3 / Tg) */
#define AFH_RATE_K12 17            /* c0 c1 Tg^c2 exp(-c3 / Tg) */
#define AFH_RATE_K13 18            /* c0 c1 exp(-(c2 / (c3 + Td))^c4) */
#define AFH_RATE_K14 19            /* c0 c1 exp(-(Td / c2)^c3) */
#define AFH_RATE_K15 20            /* c0 c1 exp(-(c2 / (kB (Tg + Td / c3)))^c4) */

/* Coarse-grid solver modes (replaces HYPRE PFMG, m_coarse_solver.f90) */
#define AFH_COARSE_CYCLES 1 /* fixed number of device MG cycles */
#define AFH_COARSE_DIRECT 2 /* exact solve: the folded operator is separable;
                               cosine / sine eigenbases per dimension */
#define AFH_COARSE_PFMG 3   /* the reference's solver, HYPRE StructPFMG, restated
                               (csrc/afh_pfmg.h): at most coarse_cycles
                               iterations, tolerance coarse_tol (50, 1e-6 in
                               the reference, m_af_types.f90:560-565) */

#define AFH_MAX_SPECIES 32
#define AFH_MAX_GAS_SPECIES 8
#define AFH_MAX_IONS 8
#define AFH_MAX_REACTIONS 128

/* Topology of one box: the box_t fields the hot path reads
 * (afivo/src/m_af_types.f90:286-322). */
typedef struct afh_box_meta {
  int32_t lvl;
  int32_t ix[3];
  int32_t parent;
  int32_t children[8];
  int32_t neighbors[6];
  int32_t neighbor_mat[27]; /* neighbor_mat(-1:1,-1:1,-1:1), i fastest */
  double r_min[3];
  double dr[3];
} afh_box_meta;

/* The af_t tree (m_af_types.f90:326-393): boxes plus per-level id lists. */
typedef struct afh_tree_desc {
  int32_t n_cell;
  int32_t n_boxes; /* highest_id; boxes[0..n_boxes-1] have ids 1..n_boxes */
  int32_t highest_lvl;
  int32_t n_var_cell;
  int32_t n_var_face;
  int32_t coarse_grid_size[3];
  int32_t periodic[3];
  double r_base[3];
  double dr_base[3];
  const afh_box_meta *boxes;
  /* lvl l (1-based) list = arr[off[l-1] .. off[l]-1]; off has highest_lvl+1 */
  const int32_t *lvl_ids, *lvl_ids_off;
  const int32_t *lvl_leaves, *lvl_leaves_off;
  const int32_t *lvl_parents, *lvl_parents_off;
  /* boxes the device data pools hold (>= n_boxes; 0: n_boxes) -- afivo's
   * box_limit: afh_tree_regrid keeps the data in place when the new tree
   * fits, instead of copying it into new pools */
  int32_t box_capacity;
} afh_tree_desc;

/* One face of a physical boundary: replaces an af_subr_bc callback whose
 * value is uniform over the face (af_bc_neumann_zero, field_bc_homogeneous,
 * ..., m_af_ghostcell.f90:614-652, src/m_field.f90:547-605). */
typedef struct afh_bc {
  int32_t type;  /* AFH_BC_* */
  double value;  /* bc_val */
} afh_bc;

/* Lookup table with linear x-spacing, src/lookup_table_fortran/
 * m_lookup_table.f90 LT_t (rows_cols is column-major: (n_points, n_cols)). */
typedef struct afh_lt {
  int32_t n_points;
  int32_t n_cols;
  double x_min;
  double inv_fac;
  const double *rows_cols;
} afh_lt;

/* One reaction, src/m_chemistry.f90 reaction_t / tiny_react_t (23-48). */
typedef struct afh_reaction {
  int32_t rate_type;  /* AFH_RATE_* */
  int32_t table_col;  /* lookup_table_index for tabulated rates (1-based) */
  double rate_factor; /* c0 */
  double c[4];        /* rate_data */
  int32_t n_in;
  int32_t ix_in[4];   /* 1-based species index into afh_fluid_desc lists */
  int32_t n_out;
  int32_t ix_out[4];
  int32_t mult_out[4];
} afh_reaction;

/* The fluid model state the m_fluid callbacks read (LFA, constant gas
 * density): species registry (m_chemistry.f90:262-300), flux species
 * (m_streamer.f90:237-260), transport + chemistry tables. */
typedef struct afh_fluid_desc {
  int32_t n_species;
  int32_t species_iv[AFH_MAX_SPECIES];     /* cc index of state 0 */
  int32_t species_charge[AFH_MAX_SPECIES];
  int32_t i_electron;   /* flux species (state 0 index) */
  int32_t i_efld;       /* |E| cell-centred (i_electric_fld) */
  int32_t f_flux;       /* flux_elec face variable */
  int32_t f_field;      /* electric field face variable */
  int32_t limiter;      /* AFH_LIM_KOREN in the reference */
  double gas_number_density;
  afh_lt td;            /* transport table: col 1 mobility*N, col 2 D*N */
  afh_lt chem;          /* chemtbl_fld */
  int32_t n_reactions;
  const afh_reaction *reactions;
  double dt_chemistry_nmin; /* < 0: limit loss (m_dt.f90:34-37 default) */
  double gas_temperature;   /* Tg (m_gas.f90:21, 300 K by default) */
  int32_t td_energy_col;    /* mean-energy column of td (td_energy_eV,
                               m_transport_data.f90:158), 0 if absent */
  /* Variable gas density (gas_constant_density = .false.): cc variable of
   * N (0: the constant gas_number_density). The flux then uses
   * N_inv = 2 / (N_{f-1} + N_f) per face (m_fluid.f90:146-154) and the
   * chemistry E/N per cell with gas species densities gas_fractions * N
   * (m_fluid.f90:339-348): reactions index the gas species 1..n_gas_species
   * first, then the plasma species (m_chemistry.f90:193-197). */
  int32_t i_gas_dens;
  int32_t n_gas_species;
  double gas_fractions[AFH_MAX_GAS_SPECIES];
  /* Photoionization source (photoi_enabled, m_fluid.f90:435-440): cc
   * variable of the photoionization rate i_photo (0: none); it is added to
   * the electron and to species photo_species (1-based index into
   * species_iv, photoi_species_index) after the chemistry time step limit. */
  int32_t i_photo;
  int32_t photo_species;
  /* Mobile ions (input_data%mobile_ions / ion_mobilities,
   * m_transport_data.f90:195-215; flux species 2.. of m_streamer.f90:
   * 253-282): n_ions plasma species (1-based index into species_iv) that
   * move with the field. Each has the face flux variable f_ion_flux and the
   * mobility times the gas density the reference scales it to
   * (ion_mobilities * 1e5 / (k_B 300 K)); its flux is
   * sign(q) mu N_inv E_f u_f with the Koren-limited upwind value u_f
   * (upwind along sign(q) E_f, no diffusion), its mu u_f adds to the
   * electrons' in the dielectric relaxation limit, and its CFL is ignored
   * (m_fluid.f90:207-214). 0: electrons only. */
  int32_t n_ions;
  int32_t ion_species[AFH_MAX_IONS];
  int32_t f_ion_flux[AFH_MAX_IONS];
  double ion_mobility[AFH_MAX_IONS];
} afh_fluid_desc;

/* Multigrid options, mg_t (m_af_types.f90:572-665) + coarse solver. */
typedef struct afh_mg_desc {
  int32_t i_phi, i_rhs, i_tmp;
  int32_t n_cycle_down, n_cycle_up; /* 2, 2 */
  double helmholtz_lambda;
  int32_t coarse_mode;   /* AFH_COARSE_CYCLES, _DIRECT or _PFMG */
  int32_t coarse_cycles; /* AFH_COARSE_CYCLES: MG V(2,2) cycles on the
                            level-1 grid (at most, with coarse_tol) */
  /* AFH_COARSE_CYCLES: stop once the level-1 residual's 2-norm is below
   * coarse_tol times the (boundary-folded) rhs's, as HYPRE PFMG's
   * SetTol does (m_coarse_solver.f90:408-414, 433-435; tolerance 1e-6 and
   * at most 50 iterations by default, m_af_types.f90:560-565); a zero rhs
   * gives phi = 0 there. 0: always coarse_cycles cycles. */
  double coarse_tol;
} afh_mg_desc;

typedef struct afh_tree afh_tree;
typedef struct afh_mg afh_mg;
typedef struct afh_fluid afh_fluid;

const char *afh_last_error(void);

/* af_init + af_adjust_refinement result (m_af_core.f90:138-822): create the
 * device box pool (all variables, zeroed) for this topology. device < 0
 * keeps the current device. */
int32_t afh_tree_create(const afh_tree_desc *desc, int32_t device,
                        afh_tree **out);
int32_t afh_tree_destroy(afh_tree *t);
int32_t afh_tree_sync(afh_tree *t);

/* af_set_cc_methods (m_af_core.f90:343-427): bc[6] per face, rb method,
 * prolongation limiter used for 2-layer ghost cells (gc2_prolong_rb). */
int32_t afh_set_cc_methods(afh_tree *t, int32_t iv, const afh_bc *bc6,
                           int32_t rb, int32_t prolong_limiter);
/* Update one face of the b.c. (e.g. a new voltage, field_set_voltage). */
int32_t afh_set_bc(afh_tree *t, int32_t iv, int32_t nb, int32_t type,
                   double value);

/* Host <-> device transfers of tree%boxes(:)%cc(..., iv) / %fc(..., ivf). */
int32_t afh_cc_put(afh_tree *t, int32_t iv, const double *host);
int32_t afh_cc_get(afh_tree *t, int32_t iv, double *host);
int32_t afh_fc_put(afh_tree *t, int32_t ivf, const double *host);
int32_t afh_fc_get(afh_tree *t, int32_t ivf, double *host);
/* Whole boxes in device memory, for moving boxes between trees and ranks
 * without a host round trip (the rank-local regrid's box exchange,
 * afivo-streamer_amd/afh/driver.py _regrid_rank_local, which replaces the
 * whole-tree gather of af_adjust_refinement's data movement,
 * m_af_core.f90:842-881). Row r of `buf` (n_cc * (nc+2)^3 + n_fc * 3 (nc+1)^3
 * doubles) holds box ids[r] (local ids, 1-based, host array): its cell-centred
 * variables 1..n_cc, then its face variables 1..n_fc, ghost cells included --
 * the per-box layout of the afh_cc_get / afh_fc_get host arrays. `buf` is
 * device memory on the tree's device; the call returns when the copies are
 * done. */
int32_t afh_tree_pack_boxes(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                            int32_t n_fc, double *buf);
int32_t afh_tree_unpack_boxes(afh_tree *t, const int32_t *ids, int32_t n, int32_t n_cc,
                              int32_t n_fc, const double *buf);
/* Device memory for such rows when the caller has no device allocator of
 * its own (the thread ranks of AFH_DIST_LOCAL): n_bytes on `device`
 * (the calling thread's current device is left as it was). */
int32_t afh_device_alloc(int32_t device, int64_t n_bytes, void **out);
int32_t afh_device_free(void *p);

/* af_gc_lvl / af_gc_tree (m_af_ghostcell.f90:25-61) */
int32_t afh_gc_lvl(afh_tree *t, int32_t lvl, int32_t iv, int32_t corners);
int32_t afh_gc_tree(afh_tree *t, int32_t iv, int32_t corners);
/* af_restrict_tree (m_af_restrict.f90:50-59) */
int32_t afh_restrict_tree(afh_tree *t, int32_t iv);
/* af_tree_copy_cc (m_af_utils.f90) / copy_current_state (streamer.f90:639) */
int32_t afh_tree_copy_cc(afh_tree *t, int32_t iv_from, int32_t iv_to);
/* Deferred reductions. The device work of a step folds its maxima and
 * minima into reduction slots on the device; the *_fold entry points leave
 * them there and return without waiting, and afh_tree_fetch_reduced reads
 * any of them in one transfer -- one host synchronisation per step instead
 * of one per reduction. A slot holds its last fold until the next operation
 * that uses it. Sharded trees reduce over ranks in the fetch. */
#define AFH_SLOT_CFL 0    /* flux_upwind_tree: max CFL sum (dt_lim(1) = 1 / v) */
#define AFH_SLOT_SIGMA 1  /* flux_upwind_tree: max conductivity */
#define AFH_SLOT_CHEM 2   /* density update, last step: min chemistry dt (a minimum) */
#define AFH_SLOT_MAXRES 3 /* V-cycle with residual: leaf max|residual| */
#define AFH_SLOT_RHS 4    /* density update with the rhs output: max|rhs| */
/* the |x| maxima AFH_SLOT_MAXRES and AFH_SLOT_RHS (n <= 2); the limits are
 * read by afh_fluid_fetch_step */
int32_t afh_tree_fetch_reduced(afh_tree *t, int32_t n, const int32_t *slots, double *out);
/* af_tree_maxabs_cc over leaf interiors (m_af_utils.f90:773-784) */
int32_t afh_tree_maxabs_cc(afh_tree *t, int32_t iv, double *out);
/* af_tree_sum_cc (m_af_utils.f90:966-1026): sum over the leaf interiors of
 * cc(iv)**power (power >= 1, evaluated as gfortran's integer power), each
 * box weighted by the cell volume of its level, product(af_lvl_dr); boxes
 * are folded in the reference's loop order (levels, then leaves). The
 * output_regression_log sums (src/m_output.f90:783-837). */
int32_t afh_tree_sum_cc(afh_tree *t, int32_t iv, int32_t power, double *out);
/* af_tree_max_cc / af_tree_min_cc / af_tree_maxabs_cc with the location of
 * the extremum (af_reduction_loc + box_max_cc / box_min_cc / box_maxabs_cc,
 * m_af_utils.f90:694-874): the first cell (i fastest) of the first box in
 * loop order holding it; loc = (box id, i, j, k), 1-based (af_loc_t), or
 * NULL. A sharded tree reduces the value over the ranks and returns no
 * location (loc must be NULL). */
#define AFH_RED_MAX 1
#define AFH_RED_MIN 2
#define AFH_RED_MAXABS 3
int32_t afh_tree_reduce_loc(afh_tree *t, int32_t iv, int32_t op, double *out,
                            int32_t *loc);

/* mg_init (m_af_multigrid.f90:43-109) + stencils; mg_fas_vcycle (185-264) */
int32_t afh_mg_create(afh_tree *t, const afh_mg_desc *desc, afh_mg **out);
int32_t afh_mg_destroy(afh_mg *mg);
int32_t afh_mg_fas_vcycle(afh_mg *mg, int32_t set_residual,
                          int32_t highest_lvl);
/* mg_fas_vcycle(set_residual = .true.) followed by af_tree_maxabs_cc(i_tmp):
 * the V-cycle + convergence test of field_compute (src/m_field.f90:455-465),
 * with the leaf max|residual| folded into the residual pass (no second read
 * of tmp). Same results as the two calls. */
int32_t afh_mg_fas_vcycle_maxres(afh_mg *mg, int32_t highest_lvl,
                                 double *max_res);
/* afh_mg_fas_vcycle_maxres without reading the maximum: it stays folded in
 * reduction slot AFH_SLOT_MAXRES (afh_tree_fetch_reduced,
 * afh_fluid_fetch_step) and the call returns without waiting for the device.
 * field_compute with one V-cycle (multigrid_num_vcycles = 1) needs the
 * residual only after the step. */
int32_t afh_mg_fas_vcycle_fold(afh_mg *mg, int32_t highest_lvl);
/* mg_fas_fmg (m_af_multigrid.f90:137-180): full multigrid; have_guess = 0
 * starts from phi = 0 on levels >= 2 (field_compute at start-up,
 * src/m_field.f90:447-470) */
int32_t afh_mg_fas_fmg(afh_mg *mg, int32_t set_residual, int32_t have_guess);
/* HYPRE_StructPFMGGetNumIteration (m_coarse_solver.f90:433-435): level-1
 * cycles of the last coarse solve (AFH_COARSE_CYCLES; 0 for the direct
 * solve); synchronises the tree's stream. */
int32_t afh_mg_coarse_iterations(afh_mg *mg, int32_t *n);
/* Diagnostics (no reference counterpart): V-cycles replayed from captured
 * hipGraphs so far, and of those the sharded ones replayed as segments
 * between their exchanges (AFH_GRAPHS, AFH_SEG_GRAPHS). The oracle replays
 * nothing and returns 0, 0. */
int32_t afh_mg_graph_stats(afh_mg *mg, int64_t *replays, int64_t *segmented);
/* mg_compute_phi_gradient (m_af_multigrid.f90:1837-1879) incl. the norm.
 * i_fc = 0 computes the norm i_norm only, on trees without electrode boxes:
 * for a fluid whose flux takes the face field from the potential
 * (afh_fluid_set_field_source), which never reads a stored face field. */
int32_t afh_mg_compute_phi_gradient(afh_mg *mg, int32_t i_fc, double fac,
                                    int32_t i_norm);
/* field_from_potential's |E| folded into the V-cycle: from now on the final
 * residual pass of a V-cycle over the whole tree (set_residual) also stores
 * |E| = afh_mg_compute_phi_gradient's norm with factor fac into cc variable
 * i_norm (0: off), from the same reads of phi; a following
 * afh_mg_compute_phi_gradient(mg, 0, fac, i_norm) then finds it current (phi
 * and |E| unchanged since) and launches nothing. Same values bitwise.
 * Constant-stencil trees only (with electrode stencils it stays off). */
int32_t afh_mg_set_gradient_output(afh_mg *mg, int32_t i_norm, double fac);

/* Electrode (level-set) boxes: the stencils mg_set_operators_tree stores on
 * the boxes an electrode surface crosses (mg_set_operators_lvl,
 * m_af_multigrid.f90:1133-1171), handed over per box after every operator
 * (re)build. afh_mg_set_box_stencil: v = box%stencils(ix)%v(7, nc, nc, nc)
 * of the operator key (mg_box_lsf_stencil, 1762-1834), bc_correction =
 * box%stencils(ix)%bc_correction (nc^3, or NULL); v = NULL removes the
 * box's stencil. Smoothing, residuals and the FAS restriction of such boxes
 * use it (stencil_gsrb_357 / stencil_apply_357 variable branch,
 * m_af_stencil.f90:459-475, 836-841, 958-978); a level-1 grid with electrode
 * boxes is solved by Gauss-Seidel to stationarity (HYPRE gets the same
 * stencils in the reference). afh_mg_set_box_lsf: the boundary distances
 * (mg_lsf_distance_key: n cells, ix(3, n) 1-based, dd(6, n)) and
 * mg_lsf_boundary_value(box) (nc^3) for mg_box_lpllsf_gradient
 * (2030-2120) on leaf boxes; i_lsf = the level-set cc variable; n = 0
 * removes. */
int32_t afh_mg_set_box_stencil(afh_mg *mg, int32_t id, const double *v,
                               const double *bc_correction);
int32_t afh_mg_set_box_lsf(afh_mg *mg, int32_t id, int32_t n, const int32_t *ix,
                           const double *dd, const double *bval, int32_t i_lsf);

/* Fluid model bound to a tree (the m_fluid / m_chemistry module state). */
int32_t afh_fluid_create(afh_tree *t, const afh_fluid_desc *desc,
                         afh_fluid **out);
int32_t afh_fluid_destroy(afh_fluid *f);
/* field_set_rhs folded into the density update: with i_rhs > 0, every
 * afh_flux_update_densities / afh_fluid_forward_euler also writes
 * rhs = field_set_rhs(i_rhs, s_out) (src/m_field.f90:363-401) -- the interior
 * from the new densities in registers; with `ghosts` also the ghost shell,
 * from the ghost cells of state s_out -- and folds max|rhs| over the leaf
 * interiors. Without `ghosts` the rhs ghost cells keep their old values: no
 * routine on the path reads them (the multigrid reads rhs on interiors
 * only: gsrb, residual, restriction, coarse gather), and on 64^3 boxes the
 * strided x-face shell costs as much as a third of a full rhs pass. This is the
 * rhs the field_compute that follows the update in the reference
 * (m_fluid.f90:51-53, streamer.f90 after af_advance) computes, provided no
 * density of state s_out changes in between; afh_fluid_rhs_maxabs(s_out)
 * then returns what afh_field_set_rhs_maxabs(i_rhs, s_out) would (an error
 * if the last update did not write state s_out's rhs). i_rhs = 0 disables.
 * The library tracks whether that rhs is still current: any call that may
 * change a density of the state or the rhs variable itself (another update,
 * afh_electrode_species_bc, afh_tree_copy_cc into a density or rhs,
 * afh_cc_put, a multigrid call with i_rhs = that variable, a regrid)
 * invalidates it; afh_fluid_rhs_valid(s) returns 1 when the rhs of state s
 * from the last update is current (field_compute may skip field_set_rhs). */
int32_t afh_fluid_set_rhs_output(afh_fluid *f, int32_t i_rhs, int32_t ghosts);
int32_t afh_fluid_rhs_maxabs(afh_fluid *f, int32_t s_out, double *max_rhs);
/* Face field from the potential: with i_phi > 0 the flux
 * (afh_flux_upwind_tree, afh_fluid_forward_euler) evaluates the face field of
 * every face as mg_box_lpl_gradient does, fac / dr * (phi_f - phi_{f-1})
 * (m_af_multigrid.f90:1882-1900; fac = -1 in field_from_potential,
 * src/m_field.f90:488-505), from phi's interior and ghost cells, instead of
 * reading f_field -- the same expression on the same values, so the fluxes
 * are bitwise those from the stored face field, as long as phi and its
 * ghost cells are the ones the gradient saw (field_from_potential is followed
 * by the flux with phi untouched in m_fluid.f90 / af_advance). The stored
 * face field is then neither written (afh_mg_compute_phi_gradient with
 * i_fc = 0) nor read: 24 B per cell less in each of the gradient and the
 * flux pass. Not for electrode boxes (mg_box_lpllsf_gradient) or dielectric
 * surface corrections of the face field. i_phi = 0 (the default): read
 * f_field. */
int32_t afh_fluid_set_field_source(afh_fluid *f, int32_t i_phi, double fac);
int32_t afh_fluid_rhs_valid(afh_fluid *f, int32_t s_out, int32_t *valid);
/* Secondary emission from ions at the domain walls: input_data%ion_se_yield
 * (m_transport_data.f90:217, 0 by default; >= 0). afh_fluid_ion_se_flux is
 * handle_ion_se_flux over the leaves (src/m_fluid.f90:584-663, called by
 * forward_euler between flux_upwind_tree and flux_update_densities,
 * m_fluid.f90:63-67): on every physical face of a leaf box, for each mobile
 * ion of positive charge in order, the electrons' face flux loses the yield
 * times the ion flux out of the domain (min(0, F) on low faces, max(0, F) on
 * high faces); the 3-D low-y face as the reference indexes it,
 * fc(1:nc, 1:nc, 1, 2) (m_fluid.f90:639-642: the y faces j = 1..nc of the
 * first z plane). afh_fluid_forward_euler[_fold] call it when the yield is
 * positive and the fluid has mobile ions; a caller of afh_flux_upwind_tree /
 * afh_flux_update_densities calls it between the two. */
int32_t afh_fluid_set_ion_se_yield(afh_fluid *f, double yield);
int32_t afh_fluid_ion_se_flux(afh_fluid *f);
/* electrode_species_bc over the boxes tagged mg_lsf_box (src/streamer.f90:
 * 578-636, called per step by set_electrode_densities, 569-574): in every
 * cell with lsf < 0 all plasma species (state 0, m_streamer.f90:242) are set
 * to 0; with neumann_zero (bc_species => af_bc_neumann_zero), a cell next to
 * a cell with lsf > 0 gets the mean electron density of those neighbours,
 * copied to the first positive ion (i_1pos_ion). Reads the ghost cells of
 * i_lsf and the electrons (the caller fills them, as in the reference). */
int32_t afh_electrode_species_bc(afh_fluid *f, int32_t i_lsf, int32_t i_1pos_ion,
                                 int32_t neumann_zero, int32_t n_ids,
                                 const int32_t *ids);
/* field_set_rhs (src/m_field.f90:363-401) */
int32_t afh_field_set_rhs(afh_fluid *f, int32_t i_rhs, int32_t s_in);
/* field_set_rhs followed by af_tree_maxabs_cc(i_rhs) (src/m_field.f90:
 * 363-401, 419-421): the leaf max|rhs| is folded into the rhs pass. */
int32_t afh_field_set_rhs_maxabs(afh_fluid *f, int32_t i_rhs, int32_t s_in,
                                 double *max_rhs);
/* Photoionization (config 5; src/m_photoi.f90:140-255, m_photoi_helmh.f90:
 * 162-204). afh_photoi_set_src: photoi_set_src's Zheleznyak source,
 * photoionization_rate_from_alpha on the leaf interiors:
 * rhs = max(0, |E| mu(Td) alpha(Td) n_e coeff), Td = 1e21 |E| / N, mu and
 * alpha from the transport table (td_mobility = col 1, td_alpha = alpha_col),
 * coeff = photoi_eta * quench_fac. */
int32_t afh_photoi_set_src(afh_fluid *f, int32_t i_rhs, int32_t alpha_col,
                           double coeff);
/* photoi_helmh_compute: i_photo = 0 everywhere; max_rhs = max(max|rhs| over
 * the leaves, sqrt(epsilon)); for each mode n (multigrid modes[n], its own
 * phi variable, helmholtz_lambda = lambda_n^2, the source in its i_rhs) up to
 * max_fmg FAS-FMG cycles (have_guess) until max|tmp| / max_rhs < max_rel_res;
 * then i_photo -= coeffs[n] * phi_n on the leaves, ghost cells included.
 * n_fmg[n] (or NULL) returns the cycles each mode took. */
int32_t afh_photoi_helmh_compute(afh_mg *const *modes, int32_t n_modes,
                                 const double *coeffs, int32_t i_photo,
                                 double max_rel_res, int32_t max_fmg,
                                 int32_t *n_fmg);
/* flux_upwind_tree with the m_fluid flux_upwind / flux_direction callbacks
 * (m_af_flux_schemes.f90:666-848, src/m_fluid.f90:102-227); dt_lim[2] =
 * (CFL limit for CFL number 1, dielectric relaxation time). */
int32_t afh_flux_upwind_tree(afh_fluid *f, int32_t s_deriv, double *dt_lim);
/* set_box_mask's electrode part (src/m_fluid.f90:469-483) for
 * afh_flux_update_densities / afh_fluid_forward_euler: a cell whose level set
 * cc(i_lsf) is <= 0 keeps the weighted sum of the previous states -- no
 * chemistry source, no photoionization, no flux divergence
 * (m_af_flux_schemes.f90:371-429 with the mask) -- and a leaf box with no
 * other cell adds no chemistry time-step limit (add_source_terms returns
 * before it, m_fluid.f90:332). i_lsf = 0: no mask (the default). */
int32_t afh_fluid_set_update_mask(afh_fluid *f, int32_t i_lsf);
/* flux_update_densities with add_source_terms / set_box_mask
 * (m_af_flux_schemes.f90:320-436, src/m_fluid.f90:298-515); dt_lim[2] =
 * (chemistry limit on the last step, 1e100 otherwise; energy limit). */
int32_t afh_flux_update_densities(afh_fluid *f, double dt, int32_t s_deriv,
                                  int32_t n_prev, const int32_t *s_prev,
                                  const double *w_prev, int32_t s_out,
                                  int32_t last_step, double *dt_lim);

/* The species part of forward_euler (src/m_fluid.f90:56-70):
 * flux_upwind_tree(s_deriv) followed by flux_update_densities. When no face
 * needs a coarse-fine correction anywhere in the topology (no
 * af_consistent_fluxes task), the limiter is Koren, all reaction rates are
 * field forms, n_species <= 4, n_prev <= 2 and no output state aliases
 * n_e(s_deriv) or |E|, both can run as one fused kernel per level (opt-in,
 * environment AFH_FE_FUSED=1; the face fluxes stay on chip and are written
 * to f_flux only with store_flux); otherwise the two calls above run. Results are bitwise those of the two
 * calls. dt_lim[4] = (CFL limit, dielectric relaxation limit, chemistry
 * limit on the last step / 1e100, 1e100) -- the reference's dt_limits(1:4)
 * before dt_cfl_number. */
int32_t afh_fluid_forward_euler(afh_fluid *f, double dt, int32_t s_deriv,
                                int32_t n_prev, const int32_t *s_prev,
                                const double *w_prev, int32_t s_out,
                                int32_t last_step, int32_t store_flux,
                                double *dt_lim);
/* afh_fluid_forward_euler without reading the limits (slots AFH_SLOT_CFL,
 * _SIGMA and, on the last step, _CHEM); returns without waiting. */
int32_t afh_fluid_forward_euler_fold(afh_fluid *f, double dt, int32_t s_deriv,
                                     int32_t n_prev, const int32_t *s_prev,
                                     const double *w_prev, int32_t s_out,
                                     int32_t last_step, int32_t store_flux);
/* dt_lim[4] of the last afh_fluid_forward_euler_fold, as
 * afh_fluid_forward_euler returns them, plus n_extra more slots
 * (AFH_SLOT_MAXRES, AFH_SLOT_RHS; n_extra <= 2) into extra -- one transfer. */
int32_t afh_fluid_fetch_step(afh_fluid *f, int32_t last_step, int32_t n_extra,
                             const int32_t *extra_slots, double *dt_lim, double *extra);

/* Regrid (af_adjust_refinement's data movement, m_af_core.f90:697-881).
 * afh_set_cc_prolong registers the prolongation of variable iv
 * (tree%cc_methods(iv)%prolong / prolong_limiter, af_set_cc_methods
 * m_af_core.f90:343-420: AFH_PROLONG_LINEAR = af_prolong_linear,
 * AFH_PROLONG_LIMIT = af_prolong_limit with `limiter`, m_af_prolong.f90)
 * and makes iv an automatic variable (tree%cc_auto_vars, registration
 * order). afh_tree_regrid builds the tree of the new topology `desc` (as
 * afivo left it after af_adjust_refinement: persisting boxes keep their ids)
 * on the device: auto_restrict into boxes whose children were removed, the
 * data of persisting boxes, then auto_prolong level by level (each new box
 * prolonged from its parent, then its ghost cells, corners included). The
 * old tree is left valid (destroy it when done). Single-rank trees. */
#define AFH_PROLONG_NONE 0
#define AFH_PROLONG_LINEAR 1
#define AFH_PROLONG_LIMIT 2
int32_t afh_set_cc_prolong(afh_tree *t, int32_t iv, int32_t method, int32_t limiter);
int32_t afh_tree_regrid(afh_tree *old, const afh_tree_desc *desc, afh_tree **out);

/* Refinement flags (default_refinement, src/m_refine.f90:198-298, reduced
 * per box as cell_to_ref_flags does, afivo/src/m_af_core.f90:1095-1148): for
 * every box of the tree, flags[id-1] = AFH_DO_REF if a cell asks for
 * refinement, AFH_KEEP_REF if one asks to keep it, AFH_RM_REF if all ask for
 * removal; masks[id-1] bit (dk+1)*9 + (dj+1)*3 + (di+1) is set when a cell
 * within buffer_width cells of the box side towards neighbour (di,dj,dk)
 * asks for refinement (cell_to_ref_flags' neighbour rule). The driver's
 * refinement routine for af_adjust_refinement rebuilds the same box flags
 * from these without the field data leaving the device. Time-dependent
 * switches (refine_init_time, refine_regions_tstop) are the caller's: pass
 * only the seeds / regions active now. electrode_box: per box 1 when the box
 * is tagged mg_lsf_box (NULL: none). */
#define AFH_RM_REF -1
#define AFH_KEEP_REF 0
#define AFH_DO_REF 1
#define AFH_MAX_REFINE_REGIONS 8
typedef struct afh_refine_desc {
  int32_t i_electron, i_efld;        /* cc variables */
  int32_t td_alpha_col, td_eta_col;  /* transport-table columns (td_alpha 3, td_eta 4) */
  int32_t use_alpha_effective;       /* refine_use_alpha_effective */
  int32_t buffer_width;              /* refine_buffer_width (cells) */
  double adx_fac, adx, min_dens;     /* refine_adx_fac, refine_adx, refine_min_dens */
  double derefine_dx, max_dx, min_dx; /* derefine_dx, refine_max_dx, refine_min_dx */
  double electrode_dx;               /* current_electrode_dx */
  int32_t n_seeds;                   /* init_conds (while global_time < refine_init_time) */
  double init_fac;                   /* refine_init_fac */
  double seed_r0[AFH_MAX_REFINE_REGIONS][3], seed_r1[AFH_MAX_REFINE_REGIONS][3];
  double seed_width[AFH_MAX_REFINE_REGIONS];
  int32_t n_regions;                 /* refine_regions_* (active ones) */
  double region_dr[AFH_MAX_REFINE_REGIONS];
  double region_rmin[AFH_MAX_REFINE_REGIONS][3], region_rmax[AFH_MAX_REFINE_REGIONS][3];
  int32_t n_limits;                  /* refine_limits_* */
  double limit_dr[AFH_MAX_REFINE_REGIONS];
  double limit_rmin[AFH_MAX_REFINE_REGIONS][3], limit_rmax[AFH_MAX_REFINE_REGIONS][3];
} afh_refine_desc;
int32_t afh_refine_flags(afh_fluid *f, const afh_refine_desc *d,
                         const uint8_t *electrode_box, int32_t *flags,
                         uint32_t *masks);

/* The cell flags a driver's refinement routine hands af_adjust_refinement
 * for a box with summary (flag, mask) of afh_refine_flags: cell_to_ref_flags
 * gives back exactly (flag, mask) (buffer_width bw). cell_flags: nc^3, i
 * fastest (afivo's cell_flags(nc, nc, nc)). */
int32_t afh_refine_cell_flags(int32_t flag, uint32_t mask, int32_t nc, int32_t bw,
                              int32_t *cell_flags);

/* Kernel timing (replaces the reference's omp_get_wtime cost buckets,
 * src/m_streamer.f90:181-187): while enabled, every launch of the selected
 * kernel class is bracketed by HIP events on the tree's stream;
 * afh_profile_read returns the summed device time, the number of launches
 * and the algorithmic HBM bytes those launches move, then resets. */
#define AFH_PROF_GSRB 1      /* red-black Gauss-Seidel half sweep */
#define AFH_PROF_GHOST 2     /* ghost-cell fill (faces) */
#define AFH_PROF_FLUX 3      /* flux kernel */
#define AFH_PROF_UPDATE 4    /* density update */
#define AFH_PROF_GSRB_PAIR 5 /* fused red+black Gauss-Seidel pair (whole boxes) */
#define AFH_PROF_GSRB_PAIR_TILED 6 /* the same with NC/4-row tiles */
#define AFH_PROF_FE 7        /* fused flux + density update (afh_fluid_forward_euler) */
#define AFH_PROF_CS 8        /* the level-1 solve (2-D build: k2_cs_pfmg; no bytes) */
int32_t afh_profile_enable(afh_tree *t, int32_t kclass);
int32_t afh_profile_read(afh_tree *t, double *total_ms, int64_t *launches,
                         double *bytes);

/* ---------------------------------------------------------------------------
 * Box sharding. A sharded run creates on every rank a tree
 * whose afh_tree_desc holds the WHOLE topology in `boxes` but only the boxes
 * this rank computes in the level lists (lvl_ids / lvl_leaves /
 * lvl_parents); storage is allocated for every box, and the boxes of other
 * ranks are replicas that are valid only where an exchange refreshed them.
 * The library calls the hook below at every point where a replica is read
 * after its owner wrote it; the host side performs the exchange with
 * afh_plan_pack / afh_plan_unpack and its collective library (RCCL via
 * torch.distributed on the GPU, gloo in the CPU tests).
 *
 * Hook kinds (level = tree level, iv = cc variable, 0 = the smoother's spare
 * image of phi):
 *   AFH_HOOK_HALO      owned boxes of `level` wrote iv: refresh the replicas
 *                      other ranks read (interior cells next to owned boxes);
 *                      called before every ghost-cell fill of the level
 *   AFH_HOOK_RIMS      after the ghost-cell fill: refresh replicas' ghost
 *                      cells read by the neighbour recomputation of the fused
 *                      smoother and by refinement-boundary interpolation
 *   AFH_HOOK_RESTRICT  owned boxes of `level` restricted iv into their
 *                      parents (level-1)
 *   AFH_HOOK_MAX/MIN   reduce vals[0..n-1] over all ranks, in place
 * A hook returns 0 on success. With no hook set (single rank) no call is
 * made. */
#define AFH_HOOK_HALO 1
#define AFH_HOOK_RIMS 2
#define AFH_HOOK_RESTRICT 3
#define AFH_HOOK_MAX 4
#define AFH_HOOK_MIN 5
#define AFH_HOOK_CFLUX 6 /* af_consistent_fluxes wrote face fluxes of
                            neighbouring leaves (iv = face variable) */
#define AFH_HOOK_SUM 7   /* sum vals[0..n-1] over all ranks, in place */
typedef int32_t (*afh_hook_fn)(void *ctx, int32_t kind, int32_t level,
                               int32_t iv, double *vals, int32_t n);
int32_t afh_tree_set_hook(afh_tree *t, afh_hook_fn fn, void *ctx);
/* Order the tree's device work on a caller-owned HIP stream (e.g. the
 * stream the collective library uses), so that exchanges need no host
 * synchronisation. The library no longer destroys the stream. */
int32_t afh_tree_set_stream(afh_tree *t, void *hip_stream);

/* A plan is a list of box regions: n x 7 int32 (box id, lo[3], hi[3]; cell
 * indices 0..nc+1, inclusive). afh_plan_pack copies variable iv of the
 * regions, in order, i fastest, into buf (device memory for libafivo_hip);
 * afh_plan_unpack copies back. Both are ordered on the tree's stream. */
int32_t afh_plan_create(afh_tree *t, const int32_t *regions, int32_t n,
                        int32_t *plan, int64_t *n_values);
/* Face-variable plan: n x 8 int32 (box id, dim 0..2, lo[3], hi[3]; face
 * indices 1..nc+1 of box%fc(:,:,:,dim+1,ivf)); pack/unpack take ivf. */
int32_t afh_plan_create_fc(afh_tree *t, const int32_t *regions, int32_t n,
                           int32_t *plan, int64_t *n_values);
int32_t afh_plan_pack(afh_tree *t, int32_t plan, int32_t iv, double *buf);
int32_t afh_plan_unpack(afh_tree *t, int32_t plan, int32_t iv,
                        const double *buf);

/* ---- Native box sharding -------------------------------
 * The partition, the exchange plans and the exchange hook inside the library
 * (the Python hook of afh/dist.py is the reference these restate; the tests
 * compare them), so a driver in any language shards a tree:
 *   owner <- afh_dist_partition(full desc, n_ranks)  (box id b: owner[b-1],
 *            -1 = replicated coarse level, *lp = the partition level)
 *   afh_tree_create_sharded(full desc, owner, rank, device, &t)  (storage
 *            only for the boxes this rank reads: its own, the replicated
 *            levels and the replicas its exchanges name; renumbered 1..n in
 *            ascending global id, afh_dist_local_ids gives the global ids,
 *            plus one unused id n+1 standing for every box not stored;
 *            cc/fc arrays and box ids in calls on t are local)
 *   afh_dist_create(t, full desc, owner, rank, n_ranks, transport, x, &d)
 * Transports: AFH_DIST_LOCAL -- the ranks are threads of one process (one
 * tree each, on one GPU or several; x = an afh_dist_group shared by the
 * ranks): pack, group barrier, peer copies, unpack; AFH_DIST_RCCL -- one
 * rank per process (x = an RCCL communicator, afh_dist_rccl_comm): grouped
 * ncclSend / ncclRecv on the tree's stream, ncclAllReduce for reductions.
 * afh_dist_plan returns the regions one exchange moves from send_rank to
 * recv_rank (n x 7 int32, n x 8 for AFH_HOOK_CFLUX; regions may be null to
 * query n). */
#define AFH_DIST_LOCAL 1
#define AFH_DIST_RCCL 2
typedef struct afh_dist afh_dist;
typedef struct afh_dist_group afh_dist_group;
int32_t afh_dist_partition(const afh_tree_desc *desc, int32_t n_ranks, int32_t *owner,
                           int32_t *lp);
/* The same with a size floor (round 6): the partition frontier starts at the
 * first level >= 2 whose boxes hold at least min_level_cells cells (and at
 * least n_ranks boxes); the levels below it are replicated -- every rank
 * computes them, no exchange. No such level: the whole tree is replicated
 * (*lp = 0). min_level_cells = 0 is afh_dist_partition. */
int32_t afh_dist_partition_levels(const afh_tree_desc *desc, int32_t n_ranks,
                                  int64_t min_level_cells, int32_t *owner, int32_t *lp);
int32_t afh_dist_plan(const afh_tree_desc *desc, const int32_t *owner, int32_t kind,
                      int32_t level, int32_t recv_rank, int32_t send_rank, int32_t *regions,
                      int32_t cap, int32_t *n);
int32_t afh_dist_local_ids(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                          int32_t *ids, int32_t cap, int32_t *n);
int32_t afh_tree_create_sharded(const afh_tree_desc *desc, const int32_t *owner, int32_t rank,
                                int32_t device, afh_tree **out);
int32_t afh_dist_group_create(int32_t n_ranks, afh_dist_group **out);
int32_t afh_dist_group_destroy(afh_dist_group *g);
int32_t afh_dist_rccl_unique_id(void *id128);
int32_t afh_dist_rccl_comm(const void *id128, int32_t rank, int32_t n_ranks, int32_t device,
                           void **comm);
int32_t afh_dist_rccl_comm_destroy(void *comm);
int32_t afh_dist_create(afh_tree *t, const afh_tree_desc *desc, const int32_t *owner,
                        int32_t rank, int32_t n_ranks, int32_t transport, void *group_or_comm,
                        afh_dist **out);
int32_t afh_dist_destroy(afh_dist *d);
int32_t afh_dist_stats(afh_dist *d, int64_t *n_exchanges, int64_t *bytes);
/* The bytes this rank sent to / received from each peer so far (n_ranks
 * entries each; null to skip): the per-link input of the scaling model. */
int32_t afh_dist_peer_bytes(afh_dist *d, int64_t *sent, int64_t *received);

#ifdef __cplusplus
}
#endif
#endif
