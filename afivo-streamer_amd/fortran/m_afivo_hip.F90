!> ISO_C_BINDING interface to libafivo_hip (include/afivo_hip.h).
!>
!> This is the layer a Fortran afivo-streamer driver uses to hand its
!> per-timestep hot path to the MI355X library: the bind(C) types mirror the
!> C structs field by field (same order, same padding) and every entry point
!> keeps the C name. Nothing here depends on afivo; m_afivo_hip_tree packs an
!> afivo tree into these types.
!>
!> The symbol prefix is AFH_PFX ("afh_" by default). Building with
!> -DAFH_PFX='"afo_"' binds the same interface to the C oracle
!> (oracle/lib/libafo.so), which the CPU tests use.
#ifndef AFH_PFX
#define AFH_PFX "afh_"
#endif
module m_afivo_hip
  use iso_c_binding
  implicit none
  public

  character(len=*), parameter :: afh_pfx = AFH_PFX

  integer(c_int32_t), parameter :: AFH_OK = 0
  integer(c_int32_t), parameter :: AFH_ERR_ARG = -1
  integer(c_int32_t), parameter :: AFH_ERR_UNSUPPORTED = -2
  integer(c_int32_t), parameter :: AFH_ERR_DEVICE = -3
  integer(c_int32_t), parameter :: AFH_ERR_STATE = -4

  ! afivo/src/m_af_types.f90:51-64
  integer(c_int32_t), parameter :: AFH_BC_DIRICHLET = -10
  integer(c_int32_t), parameter :: AFH_BC_NEUMANN = -11
  integer(c_int32_t), parameter :: AFH_BC_CONTINUOUS = -12
  integer(c_int32_t), parameter :: AFH_BC_DIRICHLET_COPY = -13

  integer(c_int32_t), parameter :: AFH_RB_GC_INTERP = 1
  integer(c_int32_t), parameter :: AFH_RB_GC_INTERP_LIM = 2
  integer(c_int32_t), parameter :: AFH_RB_MG_SIDES = 3

  integer(c_int32_t), parameter :: AFH_LIM_NONE = 1
  integer(c_int32_t), parameter :: AFH_LIM_VANLEER = 2
  integer(c_int32_t), parameter :: AFH_LIM_KOREN = 3
  integer(c_int32_t), parameter :: AFH_LIM_MINMOD = 4
  integer(c_int32_t), parameter :: AFH_LIM_MC = 5
  integer(c_int32_t), parameter :: AFH_LIM_GMINMOD43 = 6
  integer(c_int32_t), parameter :: AFH_LIM_ZERO = 7

  integer(c_int32_t), parameter :: AFH_RATE_TABULATED_FIELD = 1
  integer(c_int32_t), parameter :: AFH_RATE_CONSTANT = 2
  integer(c_int32_t), parameter :: AFH_RATE_LINEAR = 3
  integer(c_int32_t), parameter :: AFH_RATE_EXP_V1 = 4
  integer(c_int32_t), parameter :: AFH_RATE_EXP_V2 = 5
  integer(c_int32_t), parameter :: AFH_RATE_K1 = 6, AFH_RATE_K3 = 8, &
       AFH_RATE_K4 = 9, AFH_RATE_K5 = 10, AFH_RATE_K6 = 11, AFH_RATE_K7 = 12, &
       AFH_RATE_K8 = 13, AFH_RATE_K9 = 14, AFH_RATE_K10 = 15, AFH_RATE_K11 = 16, &
       AFH_RATE_K12 = 17, AFH_RATE_K13 = 18, AFH_RATE_K14 = 19, AFH_RATE_K15 = 20

  integer(c_int32_t), parameter :: AFH_COARSE_CYCLES = 1
  integer(c_int32_t), parameter :: AFH_COARSE_DIRECT = 2
  integer(c_int32_t), parameter :: AFH_COARSE_PFMG = 3
  integer, parameter :: AFH_MAX_SPECIES = 32
  integer, parameter :: AFH_MAX_REACTIONS = 128

  integer(c_int32_t), parameter :: AFH_PROF_GSRB = 1
  integer(c_int32_t), parameter :: AFH_PROF_GHOST = 2
  integer(c_int32_t), parameter :: AFH_PROF_FLUX = 3
  integer(c_int32_t), parameter :: AFH_PROF_UPDATE = 4
  integer(c_int32_t), parameter :: AFH_PROF_GSRB_PAIR = 5
  integer(c_int32_t), parameter :: AFH_PROF_GSRB_PAIR_TILED = 6
  integer(c_int32_t), parameter :: AFH_PROF_FE = 7

  type, bind(C) :: afh_box_meta
     integer(c_int32_t) :: lvl
     integer(c_int32_t) :: ix(3)
     integer(c_int32_t) :: parent
     integer(c_int32_t) :: children(8)
     integer(c_int32_t) :: neighbors(6)
     integer(c_int32_t) :: neighbor_mat(27)
     real(c_double)     :: r_min(3)
     real(c_double)     :: dr(3)
  end type afh_box_meta

  type, bind(C) :: afh_tree_desc
     integer(c_int32_t) :: n_cell
     integer(c_int32_t) :: n_boxes
     integer(c_int32_t) :: highest_lvl
     integer(c_int32_t) :: n_var_cell
     integer(c_int32_t) :: n_var_face
     integer(c_int32_t) :: coarse_grid_size(3)
     integer(c_int32_t) :: periodic(3)
     real(c_double)     :: r_base(3)
     real(c_double)     :: dr_base(3)
     type(c_ptr)        :: boxes = c_null_ptr
     type(c_ptr)        :: lvl_ids = c_null_ptr, lvl_ids_off = c_null_ptr
     type(c_ptr)        :: lvl_leaves = c_null_ptr, lvl_leaves_off = c_null_ptr
     type(c_ptr)        :: lvl_parents = c_null_ptr, lvl_parents_off = c_null_ptr
     integer(c_int32_t) :: box_capacity = 0
  end type afh_tree_desc

  type, bind(C) :: afh_bc
     integer(c_int32_t) :: type
     real(c_double)     :: value
  end type afh_bc

  type, bind(C) :: afh_lt
     integer(c_int32_t) :: n_points
     integer(c_int32_t) :: n_cols
     real(c_double)     :: x_min
     real(c_double)     :: inv_fac
     type(c_ptr)        :: rows_cols = c_null_ptr
  end type afh_lt

  type, bind(C) :: afh_reaction
     integer(c_int32_t) :: rate_type
     integer(c_int32_t) :: table_col
     real(c_double)     :: rate_factor
     real(c_double)     :: c(4)
     integer(c_int32_t) :: n_in
     integer(c_int32_t) :: ix_in(4)
     integer(c_int32_t) :: n_out
     integer(c_int32_t) :: ix_out(4)
     integer(c_int32_t) :: mult_out(4)
  end type afh_reaction

  ! regrid (afh_set_cc_prolong / afh_tree_regrid / afh_refine_flags)
  integer(c_int32_t), parameter :: AFH_PROLONG_NONE = 0, AFH_PROLONG_LINEAR = 1
  integer(c_int32_t), parameter :: AFH_PROLONG_LIMIT = 2
  ! afh_tree_reduce_loc operations
  integer(c_int32_t), parameter :: AFH_RED_MAX = 1, AFH_RED_MIN = 2, AFH_RED_MAXABS = 3
  ! deferred reduction slots (afh_tree_fetch_reduced, afh_fluid_fetch_step)
  integer(c_int32_t), parameter :: AFH_SLOT_CFL = 0, AFH_SLOT_SIGMA = 1, &
       AFH_SLOT_CHEM = 2, AFH_SLOT_MAXRES = 3, AFH_SLOT_RHS = 4
  ! exchange hook kinds (afh_tree_set_hook)
  integer(c_int32_t), parameter :: AFH_HOOK_HALO = 1, AFH_HOOK_RIMS = 2, &
       AFH_HOOK_RESTRICT = 3, AFH_HOOK_MAX = 4, AFH_HOOK_MIN = 5, AFH_HOOK_CFLUX = 6, &
       AFH_HOOK_SUM = 7
  ! afh_dist_create transports
  integer(c_int32_t), parameter :: AFH_DIST_LOCAL = 1, AFH_DIST_RCCL = 2
  integer(c_int32_t), parameter :: AFH_RM_REF = -1, AFH_KEEP_REF = 0, AFH_DO_REF = 1
  integer, parameter :: AFH_MAX_REFINE_REGIONS = 8
  integer, parameter :: AFH_MAX_GAS_SPECIES = 8
  integer, parameter :: AFH_MAX_IONS = 8

  !> default_refinement's parameters (src/m_refine.f90:10-60)
  type, bind(C) :: afh_refine_desc
     integer(c_int32_t) :: i_electron = 0, i_efld = 0
     integer(c_int32_t) :: td_alpha_col = 3, td_eta_col = 4
     integer(c_int32_t) :: use_alpha_effective = 0
     integer(c_int32_t) :: buffer_width = 4
     real(c_double)     :: adx_fac = 1, adx = 1, min_dens = -1e99_c_double
     real(c_double)     :: derefine_dx = 1e-4_c_double, max_dx = 1e-3_c_double
     real(c_double)     :: min_dx = 1e-7_c_double
     real(c_double)     :: electrode_dx = 1e99_c_double
     integer(c_int32_t) :: n_seeds = 0
     real(c_double)     :: init_fac = 0.25_c_double
     real(c_double)     :: seed_r0(3, AFH_MAX_REFINE_REGIONS) = 0
     real(c_double)     :: seed_r1(3, AFH_MAX_REFINE_REGIONS) = 0
     real(c_double)     :: seed_width(AFH_MAX_REFINE_REGIONS) = 0
     integer(c_int32_t) :: n_regions = 0
     real(c_double)     :: region_dr(AFH_MAX_REFINE_REGIONS) = 0
     real(c_double)     :: region_rmin(3, AFH_MAX_REFINE_REGIONS) = 0
     real(c_double)     :: region_rmax(3, AFH_MAX_REFINE_REGIONS) = 0
     integer(c_int32_t) :: n_limits = 0
     real(c_double)     :: limit_dr(AFH_MAX_REFINE_REGIONS) = 0
     real(c_double)     :: limit_rmin(3, AFH_MAX_REFINE_REGIONS) = 0
     real(c_double)     :: limit_rmax(3, AFH_MAX_REFINE_REGIONS) = 0
  end type afh_refine_desc

  type, bind(C) :: afh_fluid_desc
     integer(c_int32_t) :: n_species
     integer(c_int32_t) :: species_iv(AFH_MAX_SPECIES)
     integer(c_int32_t) :: species_charge(AFH_MAX_SPECIES)
     integer(c_int32_t) :: i_electron
     integer(c_int32_t) :: i_efld
     integer(c_int32_t) :: f_flux
     integer(c_int32_t) :: f_field
     integer(c_int32_t) :: limiter
     real(c_double)     :: gas_number_density
     type(afh_lt)       :: td
     type(afh_lt)       :: chem
     integer(c_int32_t) :: n_reactions
     type(c_ptr)        :: reactions = c_null_ptr
     real(c_double)     :: dt_chemistry_nmin
     real(c_double)     :: gas_temperature = 300.0_c_double
     integer(c_int32_t) :: td_energy_col = 0
     integer(c_int32_t) :: i_gas_dens = 0        ! variable gas density (0: constant)
     integer(c_int32_t) :: n_gas_species = 0
     real(c_double)     :: gas_fractions(AFH_MAX_GAS_SPECIES) = 0
     integer(c_int32_t) :: i_photo = 0          ! photoionization rate (0: none)
     integer(c_int32_t) :: photo_species = 0
     integer(c_int32_t) :: n_ions = 0              ! mobile ions (0: electrons only)
     integer(c_int32_t) :: ion_species(AFH_MAX_IONS) = 0
     integer(c_int32_t) :: f_ion_flux(AFH_MAX_IONS) = 0
     real(c_double)     :: ion_mobility(AFH_MAX_IONS) = 0
  end type afh_fluid_desc

  type, bind(C) :: afh_mg_desc
     integer(c_int32_t) :: i_phi, i_rhs, i_tmp
     integer(c_int32_t) :: n_cycle_down, n_cycle_up
     real(c_double)     :: helmholtz_lambda
     integer(c_int32_t) :: coarse_mode
     integer(c_int32_t) :: coarse_cycles
     real(c_double)     :: coarse_tol = 0   ! PFMG's stopping rule (0: fixed cycles)
  end type afh_mg_desc

  interface
     function afh_last_error() bind(C, name=afh_pfx//"last_error")
       import
       type(c_ptr) :: afh_last_error
     end function afh_last_error

     function afh_tree_create(desc, device, out) bind(C, name=afh_pfx//"tree_create")
       import
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), value       :: device
       type(c_ptr), intent(out)        :: out
       integer(c_int32_t)              :: afh_tree_create
     end function afh_tree_create

     function afh_tree_destroy(t) bind(C, name=afh_pfx//"tree_destroy")
       import
       type(c_ptr), value :: t
       integer(c_int32_t) :: afh_tree_destroy
     end function afh_tree_destroy

     function afh_tree_sync(t) bind(C, name=afh_pfx//"tree_sync")
       import
       type(c_ptr), value :: t
       integer(c_int32_t) :: afh_tree_sync
     end function afh_tree_sync

     function afh_set_cc_methods(t, iv, bc6, rb, prolong_limiter) &
          bind(C, name=afh_pfx//"set_cc_methods")
       import
       type(c_ptr), value              :: t
       integer(c_int32_t), value       :: iv
       type(afh_bc), intent(in)        :: bc6(6)
       integer(c_int32_t), value       :: rb, prolong_limiter
       integer(c_int32_t)              :: afh_set_cc_methods
     end function afh_set_cc_methods

     function afh_set_bc(t, iv, nb, bc_type, bc_value) bind(C, name=afh_pfx//"set_bc")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv, nb, bc_type
       real(c_double), value     :: bc_value
       integer(c_int32_t)        :: afh_set_bc
     end function afh_set_bc

     function afh_cc_put(t, iv, host) bind(C, name=afh_pfx//"cc_put")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv
       real(c_double), intent(in) :: host(*)
       integer(c_int32_t)        :: afh_cc_put
     end function afh_cc_put

     function afh_cc_get(t, iv, host) bind(C, name=afh_pfx//"cc_get")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv
       real(c_double), intent(inout) :: host(*)
       integer(c_int32_t)        :: afh_cc_get
     end function afh_cc_get

     function afh_fc_put(t, ivf, host) bind(C, name=afh_pfx//"fc_put")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: ivf
       real(c_double), intent(in) :: host(*)
       integer(c_int32_t)        :: afh_fc_put
     end function afh_fc_put

     function afh_fc_get(t, ivf, host) bind(C, name=afh_pfx//"fc_get")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: ivf
       real(c_double), intent(inout) :: host(*)
       integer(c_int32_t)        :: afh_fc_get
     end function afh_fc_get

     ! whole boxes as device rows (the rank-local regrid's box exchange):
     ! buf is device memory on the tree's device (c_ptr by value)
     function afh_tree_pack_boxes(t, ids, n, n_cc, n_fc, buf) &
          bind(C, name=afh_pfx//"tree_pack_boxes")
       import
       type(c_ptr), value              :: t
       integer(c_int32_t), intent(in)  :: ids(*)
       integer(c_int32_t), value       :: n, n_cc, n_fc
       type(c_ptr), value              :: buf
       integer(c_int32_t)              :: afh_tree_pack_boxes
     end function afh_tree_pack_boxes

     function afh_tree_unpack_boxes(t, ids, n, n_cc, n_fc, buf) &
          bind(C, name=afh_pfx//"tree_unpack_boxes")
       import
       type(c_ptr), value              :: t
       integer(c_int32_t), intent(in)  :: ids(*)
       integer(c_int32_t), value       :: n, n_cc, n_fc
       type(c_ptr), value              :: buf
       integer(c_int32_t)              :: afh_tree_unpack_boxes
     end function afh_tree_unpack_boxes

     ! device memory for such rows (n_bytes on `device`)
     function afh_device_alloc(device, n_bytes, out) bind(C, name=afh_pfx//"device_alloc")
       import
       integer(c_int32_t), value       :: device
       integer(c_int64_t), value       :: n_bytes
       type(c_ptr), intent(out)        :: out
       integer(c_int32_t)              :: afh_device_alloc
     end function afh_device_alloc

     function afh_device_free(p) bind(C, name=afh_pfx//"device_free")
       import
       type(c_ptr), value              :: p
       integer(c_int32_t)              :: afh_device_free
     end function afh_device_free

     function afh_gc_lvl(t, lvl, iv, corners) bind(C, name=afh_pfx//"gc_lvl")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: lvl, iv, corners
       integer(c_int32_t)        :: afh_gc_lvl
     end function afh_gc_lvl

     function afh_gc_tree(t, iv, corners) bind(C, name=afh_pfx//"gc_tree")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv, corners
       integer(c_int32_t)        :: afh_gc_tree
     end function afh_gc_tree

     function afh_restrict_tree(t, iv) bind(C, name=afh_pfx//"restrict_tree")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv
       integer(c_int32_t)        :: afh_restrict_tree
     end function afh_restrict_tree

     function afh_tree_copy_cc(t, iv_from, iv_to) bind(C, name=afh_pfx//"tree_copy_cc")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv_from, iv_to
       integer(c_int32_t)        :: afh_tree_copy_cc
     end function afh_tree_copy_cc

     function afh_tree_maxabs_cc(t, iv, out) bind(C, name=afh_pfx//"tree_maxabs_cc")
       import
       type(c_ptr), value         :: t
       integer(c_int32_t), value  :: iv
       real(c_double), intent(out) :: out
       integer(c_int32_t)         :: afh_tree_maxabs_cc
     end function afh_tree_maxabs_cc

     function afh_mg_create(t, desc, out) bind(C, name=afh_pfx//"mg_create")
       import
       type(c_ptr), value            :: t
       type(afh_mg_desc), intent(in) :: desc
       type(c_ptr), intent(out)      :: out
       integer(c_int32_t)            :: afh_mg_create
     end function afh_mg_create

     function afh_mg_destroy(mg) bind(C, name=afh_pfx//"mg_destroy")
       import
       type(c_ptr), value :: mg
       integer(c_int32_t) :: afh_mg_destroy
     end function afh_mg_destroy

     function afh_mg_fas_vcycle(mg, set_residual, highest_lvl) &
          bind(C, name=afh_pfx//"mg_fas_vcycle")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: set_residual, highest_lvl
       integer(c_int32_t)        :: afh_mg_fas_vcycle
     end function afh_mg_fas_vcycle

     !> mg_fas_fmg (m_af_multigrid.f90:137-180)
     function afh_mg_fas_fmg(mg, set_residual, have_guess) &
          bind(C, name=afh_pfx//"mg_fas_fmg")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: set_residual, have_guess
       integer(c_int32_t)        :: afh_mg_fas_fmg
     end function afh_mg_fas_fmg

     !> HYPRE_StructPFMGGetNumIteration (m_coarse_solver.f90:433-435)
     function afh_mg_coarse_iterations(mg, n) bind(C, name=afh_pfx//"mg_coarse_iterations")
       import
       type(c_ptr), value              :: mg
       integer(c_int32_t), intent(out) :: n
       integer(c_int32_t)              :: afh_mg_coarse_iterations
     end function afh_mg_coarse_iterations

     !> diagnostics: V-cycles replayed from graphs (of them, segmented)
     function afh_mg_graph_stats(mg, replays, segmented) &
          bind(C, name=afh_pfx//"mg_graph_stats")
       import
       type(c_ptr), value              :: mg
       integer(c_int64_t), intent(out) :: replays, segmented
       integer(c_int32_t)              :: afh_mg_graph_stats
     end function afh_mg_graph_stats

     !> field_from_potential's |E| folded into the V-cycle's residual pass
     function afh_mg_set_gradient_output(mg, i_norm, fac) &
          bind(C, name=afh_pfx//"mg_set_gradient_output")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: i_norm
       real(c_double), value     :: fac
       integer(c_int32_t)        :: afh_mg_set_gradient_output
     end function afh_mg_set_gradient_output

     !> af_tree_sum_cc (m_af_utils.f90:966-1026)
     function afh_tree_sum_cc(t, iv, power, out) bind(C, name=afh_pfx//"tree_sum_cc")
       import
       type(c_ptr), value          :: t
       integer(c_int32_t), value   :: iv, power
       real(c_double), intent(out) :: out
       integer(c_int32_t)          :: afh_tree_sum_cc
     end function afh_tree_sum_cc

     !> af_tree_max_cc / min_cc / maxabs_cc with location (af_reduction_loc,
     !> m_af_utils.f90:694-874); loc = [id, i, j, k]
     function afh_tree_reduce_loc(t, iv, op, out, loc) &
          bind(C, name=afh_pfx//"tree_reduce_loc")
       import
       type(c_ptr), value              :: t
       integer(c_int32_t), value       :: iv, op
       real(c_double), intent(out)     :: out
       integer(c_int32_t), intent(out) :: loc(4)
       integer(c_int32_t)              :: afh_tree_reduce_loc
     end function afh_tree_reduce_loc

     !> mg_fas_vcycle(set_residual) + af_tree_maxabs_cc(i_tmp), fused
     function afh_mg_fas_vcycle_maxres(mg, highest_lvl, max_res) &
          bind(C, name=afh_pfx//"mg_fas_vcycle_maxres")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: highest_lvl
       real(c_double), intent(out) :: max_res
       integer(c_int32_t)        :: afh_mg_fas_vcycle_maxres
     end function afh_mg_fas_vcycle_maxres

     ! the same with max|residual| left folded in AFH_SLOT_MAXRES
     function afh_mg_fas_vcycle_fold(mg, highest_lvl) &
          bind(C, name=afh_pfx//"mg_fas_vcycle_fold")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: highest_lvl
       integer(c_int32_t)        :: afh_mg_fas_vcycle_fold
     end function afh_mg_fas_vcycle_fold

     function afh_tree_fetch_reduced(t, n, slots, vals) &
          bind(C, name=afh_pfx//"tree_fetch_reduced")
       import
       type(c_ptr), value             :: t
       integer(c_int32_t), value      :: n
       integer(c_int32_t), intent(in) :: slots(*)
       real(c_double), intent(out)    :: vals(*)
       integer(c_int32_t)             :: afh_tree_fetch_reduced
     end function afh_tree_fetch_reduced

     function afh_mg_compute_phi_gradient(mg, i_fc, fac, i_norm) &
          bind(C, name=afh_pfx//"mg_compute_phi_gradient")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: i_fc
       real(c_double), value     :: fac
       integer(c_int32_t), value :: i_norm
       integer(c_int32_t)        :: afh_mg_compute_phi_gradient
     end function afh_mg_compute_phi_gradient

     ! electrode (level-set) boxes: stencils stored by mg_set_operators_tree
     function afh_mg_set_box_stencil(mg, id, v, bc_correction) &
          bind(C, name=afh_pfx//"mg_set_box_stencil")
       import
       type(c_ptr), value        :: mg
       integer(c_int32_t), value :: id
       type(c_ptr), value        :: v, bc_correction   ! c_loc(...) or c_null_ptr
       integer(c_int32_t)        :: afh_mg_set_box_stencil
     end function afh_mg_set_box_stencil

     function afh_mg_set_box_lsf(mg, id, n, ix, dd, bval, i_lsf) &
          bind(C, name=afh_pfx//"mg_set_box_lsf")
       import
       type(c_ptr), value             :: mg
       integer(c_int32_t), value      :: id, n
       integer(c_int32_t), intent(in) :: ix(*)
       real(c_double), intent(in)     :: dd(*), bval(*)
       integer(c_int32_t), value      :: i_lsf
       integer(c_int32_t)             :: afh_mg_set_box_lsf
     end function afh_mg_set_box_lsf

     function afh_set_cc_prolong(t, iv, method, limiter) &
          bind(C, name=afh_pfx//"set_cc_prolong")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: iv, method, limiter
       integer(c_int32_t)        :: afh_set_cc_prolong
     end function afh_set_cc_prolong

     ! af_adjust_refinement's data movement onto the new topology
     function afh_tree_regrid(t, desc, out) bind(C, name=afh_pfx//"tree_regrid")
       import
       type(c_ptr), value             :: t
       type(afh_tree_desc), intent(in) :: desc
       type(c_ptr), intent(out)       :: out
       integer(c_int32_t)             :: afh_tree_regrid
     end function afh_tree_regrid

     ! default_refinement + cell_to_ref_flags per box, on the device
     function afh_refine_flags(f, desc, electrode_box, flags, masks) &
          bind(C, name=afh_pfx//"refine_flags")
       import
       type(c_ptr), value                :: f
       type(afh_refine_desc), intent(in) :: desc
       type(c_ptr), value                :: electrode_box  ! c_loc(int8 array) or c_null_ptr
       integer(c_int32_t), intent(out)   :: flags(*), masks(*)
       integer(c_int32_t)                :: afh_refine_flags
     end function afh_refine_flags

     ! cell flags for af_adjust_refinement's ref_subr from a box summary
     function afh_refine_cell_flags(flag, mask, nc, bw, cell_flags) &
          bind(C, name=afh_pfx//"refine_cell_flags")
       import
       integer(c_int32_t), value       :: flag, mask, nc, bw
       integer(c_int32_t), intent(out) :: cell_flags(*)
       integer(c_int32_t)              :: afh_refine_cell_flags
     end function afh_refine_cell_flags

     function afh_fluid_create(t, desc, out) bind(C, name=afh_pfx//"fluid_create")
       import
       type(c_ptr), value               :: t
       type(afh_fluid_desc), intent(in) :: desc
       type(c_ptr), intent(out)         :: out
       integer(c_int32_t)               :: afh_fluid_create
     end function afh_fluid_create

     function afh_fluid_destroy(f) bind(C, name=afh_pfx//"fluid_destroy")
       import
       type(c_ptr), value :: f
       integer(c_int32_t) :: afh_fluid_destroy
     end function afh_fluid_destroy

     !> field_set_rhs folded into the density update (0 disables)
     function afh_fluid_set_rhs_output(f, i_rhs, ghosts) bind(C, name=afh_pfx//"fluid_set_rhs_output")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_rhs, ghosts
       integer(c_int32_t)        :: afh_fluid_set_rhs_output
     end function afh_fluid_set_rhs_output

     !> face field of the flux from the potential i_phi (0: read f_field)
     function afh_fluid_set_field_source(f, i_phi, fac) bind(C, name=afh_pfx//"fluid_set_field_source")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_phi
       real(c_double), value     :: fac
       integer(c_int32_t)        :: afh_fluid_set_field_source
     end function afh_fluid_set_field_source

     !> input_data%ion_se_yield: handle_ion_se_flux inside forward_euler
     function afh_fluid_set_ion_se_yield(f, yield) bind(C, name=afh_pfx//"fluid_set_ion_se_yield")
       import
       type(c_ptr), value    :: f
       real(c_double), value :: yield
       integer(c_int32_t)    :: afh_fluid_set_ion_se_yield
     end function afh_fluid_set_ion_se_yield

     !> handle_ion_se_flux over the leaves (src/m_fluid.f90:584-663)
     function afh_fluid_ion_se_flux(f) bind(C, name=afh_pfx//"fluid_ion_se_flux")
       import
       type(c_ptr), value :: f
       integer(c_int32_t) :: afh_fluid_ion_se_flux
     end function afh_fluid_ion_se_flux

     !> max|rhs| of the rhs the last update wrote for state s_out
     function afh_fluid_rhs_maxabs(f, s_out, max_rhs) bind(C, name=afh_pfx//"fluid_rhs_maxabs")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: s_out
       real(c_double), intent(out) :: max_rhs
       integer(c_int32_t)        :: afh_fluid_rhs_maxabs
     end function afh_fluid_rhs_maxabs

     !> 1 when the rhs of state s_out from the last update is current
     function afh_fluid_rhs_valid(f, s_out, valid) bind(C, name=afh_pfx//"fluid_rhs_valid")
       import
       type(c_ptr), value              :: f
       integer(c_int32_t), value       :: s_out
       integer(c_int32_t), intent(out) :: valid
       integer(c_int32_t)              :: afh_fluid_rhs_valid
     end function afh_fluid_rhs_valid

     !> photoi_set_src, Zheleznyak source (src/m_photoi.f90:140-186)
     function afh_photoi_set_src(f, i_rhs, alpha_col, coeff) &
          bind(C, name=afh_pfx//"photoi_set_src")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_rhs, alpha_col
       real(c_double), value     :: coeff
       integer(c_int32_t)        :: afh_photoi_set_src
     end function afh_photoi_set_src

     !> photoi_helmh_compute (src/m_photoi_helmh.f90:162-204); modes: the
     !> Helmholtz multigrid handles, one per mode
     function afh_photoi_helmh_compute(modes, n_modes, coeffs, i_photo, max_rel_res, &
          max_fmg, n_fmg) bind(C, name=afh_pfx//"photoi_helmh_compute")
       import
       type(c_ptr), intent(in)         :: modes(*)
       integer(c_int32_t), value       :: n_modes, i_photo, max_fmg
       real(c_double), intent(in)      :: coeffs(*)
       real(c_double), value           :: max_rel_res
       integer(c_int32_t), intent(out) :: n_fmg
       integer(c_int32_t)              :: afh_photoi_helmh_compute
     end function afh_photoi_helmh_compute

     !> order the tree's device work on a caller-owned HIP stream
     function afh_tree_set_stream(t, stream) bind(C, name=afh_pfx//"tree_set_stream")
       import
       type(c_ptr), value :: t, stream
       integer(c_int32_t) :: afh_tree_set_stream
     end function afh_tree_set_stream

     !> exchange hook of a sharded tree (afh_hook_fn: a bind(C) function
     !> (ctx, kind, level, iv, vals, n) -> int32)
     function afh_tree_set_hook(t, fn, ctx) bind(C, name=afh_pfx//"tree_set_hook")
       import
       type(c_ptr), value    :: t, ctx
       type(c_funptr), value :: fn
       integer(c_int32_t)    :: afh_tree_set_hook
     end function afh_tree_set_hook

     !> region plans for exchanges: n x 7 (cc) / n x 8 (fc) int32 regions
     function afh_plan_create(t, regions, n, plan, n_values) &
          bind(C, name=afh_pfx//"plan_create")
       import
       type(c_ptr), value              :: t
       integer(c_int32_t), intent(in)  :: regions(*)
       integer(c_int32_t), value       :: n
       integer(c_int32_t), intent(out) :: plan
       integer(c_int64_t), intent(out) :: n_values
       integer(c_int32_t)              :: afh_plan_create
     end function afh_plan_create

     function afh_plan_create_fc(t, regions, n, plan, n_values) &
          bind(C, name=afh_pfx//"plan_create_fc")
       import
       type(c_ptr), value              :: t
       integer(c_int32_t), intent(in)  :: regions(*)
       integer(c_int32_t), value       :: n
       integer(c_int32_t), intent(out) :: plan
       integer(c_int64_t), intent(out) :: n_values
       integer(c_int32_t)              :: afh_plan_create_fc
     end function afh_plan_create_fc

     function afh_plan_pack(t, plan, iv, buf) bind(C, name=afh_pfx//"plan_pack")
       import
       type(c_ptr), value        :: t, buf
       integer(c_int32_t), value :: plan, iv
       integer(c_int32_t)        :: afh_plan_pack
     end function afh_plan_pack

     function afh_plan_unpack(t, plan, iv, buf) bind(C, name=afh_pfx//"plan_unpack")
       import
       type(c_ptr), value        :: t, buf
       integer(c_int32_t), value :: plan, iv
       integer(c_int32_t)        :: afh_plan_unpack
     end function afh_plan_unpack

     !> native box sharding (include/afivo_hip.h, afh_dist_*): the library
     !> partitions the tree, stores a rank's boxes and runs the exchanges.
     !> With MPI, rank 0 calls afh_dist_rccl_unique_id, broadcasts the 128
     !> bytes (MPI_Bcast), every rank calls afh_dist_rccl_comm and then
     !> afh_dist_create(..., AFH_DIST_RCCL, comm, d).
     function afh_dist_partition(desc, n_ranks, owner, lp) &
          bind(C, name=afh_pfx//"dist_partition")
       import
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), value       :: n_ranks
       integer(c_int32_t), intent(out) :: owner(*), lp
       integer(c_int32_t)              :: afh_dist_partition
     end function afh_dist_partition

     function afh_dist_partition_levels(desc, n_ranks, min_level_cells, owner, lp) &
          bind(C, name=afh_pfx//"dist_partition_levels")
       import
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), value       :: n_ranks
       integer(c_int64_t), value       :: min_level_cells
       integer(c_int32_t), intent(out) :: owner(*), lp
       integer(c_int32_t)              :: afh_dist_partition_levels
     end function afh_dist_partition_levels

     function afh_dist_plan(desc, owner, kind, level, recv_rank, send_rank, regions, cap, n) &
          bind(C, name=afh_pfx//"dist_plan")
       import
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), intent(in)  :: owner(*)
       integer(c_int32_t), value       :: kind, level, recv_rank, send_rank, cap
       type(c_ptr), value              :: regions
       integer(c_int32_t), intent(out) :: n
       integer(c_int32_t)              :: afh_dist_plan
     end function afh_dist_plan

     !> the global ids of the boxes rank stores (local id k = ids(k))
     function afh_dist_local_ids(desc, owner, rank, ids, cap, n) &
          bind(C, name=afh_pfx//"dist_local_ids")
       import
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), intent(in)  :: owner(*)
       integer(c_int32_t), value       :: rank, cap
       type(c_ptr), value              :: ids
       integer(c_int32_t), intent(out) :: n
       integer(c_int32_t)              :: afh_dist_local_ids
     end function afh_dist_local_ids

     function afh_tree_create_sharded(desc, owner, rank, device, out) &
          bind(C, name=afh_pfx//"tree_create_sharded")
       import
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), intent(in)  :: owner(*)
       integer(c_int32_t), value       :: rank, device
       type(c_ptr), intent(out)        :: out
       integer(c_int32_t)              :: afh_tree_create_sharded
     end function afh_tree_create_sharded

     function afh_dist_group_create(n_ranks, out) bind(C, name=afh_pfx//"dist_group_create")
       import
       integer(c_int32_t), value :: n_ranks
       type(c_ptr), intent(out)  :: out
       integer(c_int32_t)        :: afh_dist_group_create
     end function afh_dist_group_create

     function afh_dist_group_destroy(g) bind(C, name=afh_pfx//"dist_group_destroy")
       import
       type(c_ptr), value :: g
       integer(c_int32_t) :: afh_dist_group_destroy
     end function afh_dist_group_destroy

     function afh_dist_rccl_unique_id(id128) bind(C, name=afh_pfx//"dist_rccl_unique_id")
       import
       type(c_ptr), value :: id128
       integer(c_int32_t) :: afh_dist_rccl_unique_id
     end function afh_dist_rccl_unique_id

     function afh_dist_rccl_comm(id128, rank, n_ranks, device, comm) &
          bind(C, name=afh_pfx//"dist_rccl_comm")
       import
       type(c_ptr), value        :: id128
       integer(c_int32_t), value :: rank, n_ranks, device
       type(c_ptr), intent(out)  :: comm
       integer(c_int32_t)        :: afh_dist_rccl_comm
     end function afh_dist_rccl_comm

     function afh_dist_rccl_comm_destroy(comm) bind(C, name=afh_pfx//"dist_rccl_comm_destroy")
       import
       type(c_ptr), value :: comm
       integer(c_int32_t) :: afh_dist_rccl_comm_destroy
     end function afh_dist_rccl_comm_destroy

     function afh_dist_create(t, desc, owner, rank, n_ranks, transport, group_or_comm, out) &
          bind(C, name=afh_pfx//"dist_create")
       import
       type(c_ptr), value              :: t, group_or_comm
       type(afh_tree_desc), intent(in) :: desc
       integer(c_int32_t), intent(in)  :: owner(*)
       integer(c_int32_t), value       :: rank, n_ranks, transport
       type(c_ptr), intent(out)        :: out
       integer(c_int32_t)              :: afh_dist_create
     end function afh_dist_create

     function afh_dist_destroy(d) bind(C, name=afh_pfx//"dist_destroy")
       import
       type(c_ptr), value :: d
       integer(c_int32_t) :: afh_dist_destroy
     end function afh_dist_destroy

     function afh_dist_stats(d, n_exchanges, bytes) bind(C, name=afh_pfx//"dist_stats")
       import
       type(c_ptr), value              :: d
       integer(c_int64_t), intent(out) :: n_exchanges, bytes
       integer(c_int32_t)              :: afh_dist_stats
     end function afh_dist_stats

     function afh_dist_peer_bytes(d, sent, received) bind(C, name=afh_pfx//"dist_peer_bytes")
       import
       type(c_ptr), value              :: d
       integer(c_int64_t), intent(out) :: sent(*), received(*)
       integer(c_int32_t)              :: afh_dist_peer_bytes
     end function afh_dist_peer_bytes

     !> electrode_species_bc (src/streamer.f90:578-636) over the mg_lsf_box boxes
     function afh_electrode_species_bc(f, i_lsf, i_1pos_ion, neumann_zero, n_ids, ids) &
          bind(C, name=afh_pfx//"electrode_species_bc")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_lsf, i_1pos_ion, neumann_zero, n_ids
       integer(c_int32_t), intent(in) :: ids(*)
       integer(c_int32_t)        :: afh_electrode_species_bc
     end function afh_electrode_species_bc

     function afh_field_set_rhs(f, i_rhs, s_in) bind(C, name=afh_pfx//"field_set_rhs")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_rhs, s_in
       integer(c_int32_t)        :: afh_field_set_rhs
     end function afh_field_set_rhs

     !> field_set_rhs + af_tree_maxabs_cc(i_rhs), fused
     function afh_field_set_rhs_maxabs(f, i_rhs, s_in, max_rhs) &
          bind(C, name=afh_pfx//"field_set_rhs_maxabs")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_rhs, s_in
       real(c_double), intent(out) :: max_rhs
       integer(c_int32_t)        :: afh_field_set_rhs_maxabs
     end function afh_field_set_rhs_maxabs

     function afh_flux_upwind_tree(f, s_deriv, dt_lim) &
          bind(C, name=afh_pfx//"flux_upwind_tree")
       import
       type(c_ptr), value          :: f
       integer(c_int32_t), value   :: s_deriv
       real(c_double), intent(out) :: dt_lim(2)
       integer(c_int32_t)          :: afh_flux_upwind_tree
     end function afh_flux_upwind_tree

     ! set_box_mask's electrode part (src/m_fluid.f90:469-483): cells with
     ! cc(i_lsf) <= 0 are not updated; 0: no mask
     function afh_fluid_set_update_mask(f, i_lsf) bind(C, name=afh_pfx//"fluid_set_update_mask")
       import
       type(c_ptr), value        :: f
       integer(c_int32_t), value :: i_lsf
       integer(c_int32_t)        :: afh_fluid_set_update_mask
     end function afh_fluid_set_update_mask

     function afh_flux_update_densities(f, dt, s_deriv, n_prev, s_prev, w_prev, &
          s_out, last_step, dt_lim) bind(C, name=afh_pfx//"flux_update_densities")
       import
       type(c_ptr), value             :: f
       real(c_double), value          :: dt
       integer(c_int32_t), value      :: s_deriv, n_prev
       integer(c_int32_t), intent(in) :: s_prev(*)
       real(c_double), intent(in)     :: w_prev(*)
       integer(c_int32_t), value      :: s_out, last_step
       real(c_double), intent(out)    :: dt_lim(2)
       integer(c_int32_t)             :: afh_flux_update_densities
     end function afh_flux_update_densities

     ! forward_euler's species part (m_fluid.f90:56-70): fused on the device
     function afh_fluid_forward_euler(f, dt, s_deriv, n_prev, s_prev, w_prev, &
          s_out, last_step, store_flux, dt_lim) &
          bind(C, name=afh_pfx//"fluid_forward_euler")
       import
       type(c_ptr), value             :: f
       real(c_double), value          :: dt
       integer(c_int32_t), value      :: s_deriv, n_prev
       integer(c_int32_t), intent(in) :: s_prev(*)
       real(c_double), intent(in)     :: w_prev(*)
       integer(c_int32_t), value      :: s_out, last_step, store_flux
       real(c_double), intent(out)    :: dt_lim(4)
       integer(c_int32_t)             :: afh_fluid_forward_euler
     end function afh_fluid_forward_euler

     function afh_fluid_forward_euler_fold(f, dt, s_deriv, n_prev, s_prev, w_prev, &
          s_out, last_step, store_flux) &
          bind(C, name=afh_pfx//"fluid_forward_euler_fold")
       import
       type(c_ptr), value             :: f
       real(c_double), value          :: dt
       integer(c_int32_t), value      :: s_deriv, n_prev
       integer(c_int32_t), intent(in) :: s_prev(*)
       real(c_double), intent(in)     :: w_prev(*)
       integer(c_int32_t), value      :: s_out, last_step, store_flux
       integer(c_int32_t)             :: afh_fluid_forward_euler_fold
     end function afh_fluid_forward_euler_fold

     function afh_fluid_fetch_step(f, last_step, n_extra, extra_slots, dt_lim, extra) &
          bind(C, name=afh_pfx//"fluid_fetch_step")
       import
       type(c_ptr), value             :: f
       integer(c_int32_t), value      :: last_step, n_extra
       integer(c_int32_t), intent(in) :: extra_slots(*)
       real(c_double), intent(out)    :: dt_lim(4), extra(*)
       integer(c_int32_t)             :: afh_fluid_fetch_step
     end function afh_fluid_fetch_step

     function afh_profile_enable(t, kclass) bind(C, name=afh_pfx//"profile_enable")
       import
       type(c_ptr), value        :: t
       integer(c_int32_t), value :: kclass
       integer(c_int32_t)        :: afh_profile_enable
     end function afh_profile_enable

     function afh_profile_read(t, total_ms, launches, bytes) &
          bind(C, name=afh_pfx//"profile_read")
       import
       type(c_ptr), value            :: t
       real(c_double), intent(out)   :: total_ms
       integer(c_int64_t), intent(out) :: launches
       real(c_double), intent(out)   :: bytes
       integer(c_int32_t)            :: afh_profile_read
     end function afh_profile_read

     function c_strlen(s) bind(C, name="strlen")
       import
       type(c_ptr), value :: s
       integer(c_size_t)  :: c_strlen
     end function c_strlen
  end interface

contains

  !> Turn a non-zero return code into `error stop`, as the reference does on
  !> failure (e.g. m_af_stencil.f90:338), with the library's message.
  subroutine afh_check(ierr, what)
    integer(c_int32_t), intent(in) :: ierr
    character(len=*), intent(in), optional :: what
    character(kind=c_char), pointer :: msg(:)
    type(c_ptr)                     :: p
    integer                         :: n
    character(len=:), allocatable   :: text
    if (ierr == AFH_OK) return
    p = afh_last_error()
    n = int(c_strlen(p))
    call c_f_pointer(p, msg, [n])
    allocate(character(len=n) :: text)
    text = transfer(msg(1:n), text)
    if (present(what)) then
      write(*, '(A,A,A,I0,A,A)') "afivo_hip: ", what, " failed (", ierr, "): ", text
    else
      write(*, '(A,I0,A,A)') "afivo_hip: call failed (", ierr, "): ", text
    end if
    error stop "afivo_hip call failed"
  end subroutine afh_check

end module m_afivo_hip
