!> ORACLE TEST INFRASTRUCTURE -- golden-vector generator (build container only).
!>
!> Drives the afivo numerics compiled from the reference sources
!> (/root/reference/afivo/src, NDIM=3) through one Heun time step of the
!> streamer hot path and dumps every intermediate state as raw binary:
!>
!>   field_compute (rhs, FAS V-cycles, field_from_potential)
!>   -> flux_upwind_tree (sub-step 1) -> flux_update_densities
!>   -> field_compute -> flux_upwind_tree (sub-step 2) -> flux_update_densities
!>
!> The FAS V-cycle driver below re-sequences the reference's public box-level
!> routines exactly as mg_fas_vcycle does (afivo/src/m_af_multigrid.f90:185-264,
!> gsrb_boxes 648-687, update_coarse 691-738, correct_children 624-646,
!> residual_box 801-810), because mg_init / solve_coarse_grid call HYPRE
!> (afivo/src/m_coarse_solver.f90), which is absent from the reference snapshot.
!> The level-1 problem is instead solved to machine precision by Gauss-Seidel
!> red-black sweeps with the reference's own af_stencil_gsrb_box and af_gc_box,
!> which converge to the same linear system HYPRE is given (boundary conditions
!> folded as in stencil_handle_boundaries, m_coarse_solver.f90:442-491).
!>
!> Case rod8 adds a rod electrode as a level-set function (the electrode
!> operators of m_field.f90:255-346 with field_electrode_type = rod): the
!> reference stores its LSF stencils (mg_set_operators_tree ->
!> store_lsf_distance_matrix / mg_box_lsf_stencil), which are dumped to lsf.bin,
!> and the field solve (V-cycles, FMG, gradient with mg_box_lpllsf_gradient)
!> runs through them.
!>
!> Case regrid8 runs af_adjust_refinement (m_af_core.f90:697-822) once on
!> an AMR tree whose densities are prolonged with af_prolong_limit (the
!> streamer's default, m_streamer.f90:395-410): boxes near a moving point
!> are refined, boxes far from it derefined; the topology and every variable
!> are dumped before and after (auto_restrict / auto_prolong / af_gc_box).
!>
!> Usage: golden_gen <case> <td_file> <out_dir>
!>   case = uni4 | amr4 | uni8 | rod8 | regrid8
program golden_gen
#include "cpp_macros.h"
  use m_af_types
  use m_af_core
  use m_af_utils
  use m_af_ghostcell
  use m_af_stencil
  use m_af_restrict
  use m_af_prolong, only: af_prolong_limit
  use m_af_multigrid
  use m_af_flux_schemes
  use m_af_limiters
  use m_coarse_solver, only: mg_lsf_boundary_value
  use m_geometry, only: GM_dist_line
  use m_lookup_table, only: LT_get_col
  use hx_physics

  implicit none

  type(af_t)         :: tree
  type(mg_t)         :: mg
  character(len=256) :: case_name, td_file, out_dir
  integer            :: nc, grid(3), max_lvl, amr_lvl, n_dump, i
  real(dp)           :: dom(3), r0(3), width, dt, dtl(4), residuals(2)
  real(dp)           :: max_rhs, threshold
  ! photoionization Helmholtz mode: Bourdon's second lambda at 1 bar
  ! (src/m_photoi_helmh.f90:100), 1/m
  real(dp), parameter :: helm_lambda = 44081.25_dp
  logical            :: trace, use_lsf, do_regrid
  integer            :: u_log, i_lsf
  type(ref_info_t)   :: regrid_info
  ! default_refinement parameters of the regrid8 case (src/m_refine.f90:10-60
  ! names), dumped with the flags
  real(dp) :: rf_adx = 0.3_dp, rf_adx_fac = 1.0_dp, rf_min_dens = 1.0e16_dp
  real(dp) :: rf_derefine_dx = 1.0e-4_dp, rf_max_dx = 1.0e-3_dp
  real(dp) :: rf_min_dx = 1.0e-7_dp, rf_init_fac = 0.25_dp
  real(dp) :: rf_seed_r0(3), rf_seed_r1(3), rf_seed_width
  real(dp) :: rf_region_dr, rf_region_rmin(3), rf_region_rmax(3)
  real(dp) :: rf_limit_dr, rf_limit_rmin(3), rf_limit_rmax(3)
  integer  :: rf_buffer = 2
  ! rod electrode (field_rod_r0/r1/radius as fractions of the domain)
  real(dp)           :: rod_r0(3), rod_r1(3), rod_radius

  call get_command_argument(1, case_name)
  call get_command_argument(2, td_file)
  call get_command_argument(3, out_dir)

  use_lsf = .false.
  do_regrid = .false.
  select case (trim(case_name))
  case ("regrid8")
     nc = 8; grid = [8, 8, 8]; max_lvl = 2; amr_lvl = 3; trace = .false.
     do_regrid = .true.
  case ("rod8")
     nc = 8; grid = [8, 8, 8]; max_lvl = 2; amr_lvl = 3; trace = .false.
     use_lsf = .true.
  case ("uni4")
     nc = 4; grid = [4, 4, 4]; max_lvl = 3; amr_lvl = 0; trace = .true.
  case ("amr4")
     nc = 4; grid = [8, 4, 4]; max_lvl = 2; amr_lvl = 4; trace = .false.
  case ("uni8")
     nc = 8; grid = [8, 8, 8]; max_lvl = 2; amr_lvl = 0; trace = .false.
  case default
     error stop "unknown case"
  end select

  ! Domain: cells are cubic at every level
  dom = 1.0e-3_dp * grid / 4
  r0  = 0.5_dp * dom
  r0(1) = 0.4_dp * dom(1)
  width = 0.15_dp * dom(3)

  call hx_init_gas(1.0_dp, 300.0_dp)
  call hx_init_transport(trim(td_file))
  ! Background field -2.5 MV/m: current_voltage = -L_z * E (m_field.f90:516)
  current_voltage = -dom(3) * (-2.5e6_dp)

  ! Variables, in the order the streamer registers them
  call af_add_cc_variable(tree, "e", n_copies=3)
  call af_add_cc_variable(tree, "M+", n_copies=3)
  call af_add_cc_variable(tree, "M-", n_copies=3)
  call af_add_cc_variable(tree, "phi", n_copies=2)
  call af_add_cc_variable(tree, "electric_fld")
  call af_add_cc_variable(tree, "rhs")
  call af_add_cc_variable(tree, "tmp")
  call af_add_fc_variable(tree, "flux_elec")
  call af_add_fc_variable(tree, "field")
  if (tree%n_var_cell /= n_cc_vars) error stop "variable layout"
  if (use_lsf) then
     ! the electrode's level-set variable (m_streamer.f90 adds "lsf" when
     ! ST_use_electrode), appended after the standard layout
     call af_add_cc_variable(tree, "lsf", ix=i_lsf)
     tree%mg_i_lsf = i_lsf
     rod_r0 = [0.5_dp, 0.5_dp, 1.0_dp] * dom
     rod_r1 = [0.5_dp, 0.5_dp, 0.6_dp] * dom
     rod_radius = 0.1_dp * dom(3)
  end if

  ! Ghost-cell methods as set by streamer.f90:81-84 and m_field.f90:349-350;
  ! phi gets (sides_bc, mg_auto_rb) as in mg_init (m_af_multigrid.f90:102-105)
  if (do_regrid) then
     ! streamer.f90:81-84 with prolong_density = limit (the default)
     call af_set_cc_methods(tree, i_e, af_bc_neumann_zero, af_gc_interp_lim, &
          af_prolong_limit)
     call af_set_cc_methods(tree, i_pos, af_bc_neumann_zero, af_gc_interp_lim, &
          af_prolong_limit)
     call af_set_cc_methods(tree, i_neg, af_bc_neumann_zero, af_gc_interp_lim, &
          af_prolong_limit)
  else
     call af_set_cc_methods(tree, i_e, af_bc_neumann_zero, af_gc_interp_lim)
     call af_set_cc_methods(tree, i_pos, af_bc_neumann_zero, af_gc_interp_lim)
     call af_set_cc_methods(tree, i_neg, af_bc_neumann_zero, af_gc_interp_lim)
  end if
  call af_set_cc_methods(tree, i_efld, af_bc_neumann_zero, af_gc_interp)
  call af_set_cc_methods(tree, i_phi, hx_bc_phi, hx_rb_phi)

  call af_init(tree, nc, dom, grid)
  call af_refine_up_to_lvl(tree, max_lvl)
  do i = max_lvl+1, amr_lvl
     call refine_amr()
  end do

  ! Multigrid options and stencils: mg_init minus the HYPRE set-up
  ! (m_af_multigrid.f90:43-109), then mg_use (118-126)
  mg%i_phi = i_phi
  mg%i_tmp = i_tmp
  mg%i_rhs = i_rhs
  mg%sides_bc => hx_bc_phi
  tree%n_stencil_keys_stored = tree%n_stencil_keys_stored + 1
  mg%operator_key = tree%n_stencil_keys_stored
  tree%n_stencil_keys_stored = tree%n_stencil_keys_stored + 1
  mg%prolongation_key = tree%n_stencil_keys_stored
  mg%initialized = .true.
  tree%mg_current_operator_mask = mg%operator_mask
  if (use_lsf) then
     ! field_initialize with an electrode (m_field.f90:255-346, 439-443):
     ! rod level-set function, golden-section distances, electrode at the
     ! applied voltage; mg_init copies tree%mg_i_lsf (m_af_multigrid.f90:77-82)
     call af_loop_box(tree, set_lsf_box)
     mg%i_lsf = tree%mg_i_lsf
     mg%lsf => rod_lsf
     mg%lsf_dist => mg_lsf_dist_gss
     mg%lsf_length_scale = rod_radius
     mg%lsf_boundary_value = current_voltage
  end if
  call mg_set_operators_tree(tree, mg)

  call af_loop_box(tree, set_init)
  call af_restrict_tree(tree, [i_e, i_pos, i_neg])
  call af_gc_tree(tree, [i_e, i_pos, i_neg])
  call af_gc_tree(tree, [i_phi])

  n_dump = 0
  open(newunit=u_log, file=trim(out_dir)//"/log.txt", status="replace")
  call dump_topology("topology.bin")
  call dump_tables()
  call dump_state("init")
  if (use_lsf) call dump_lsf()

  if (do_regrid) then
     ! the field of the initial state (field_compute + field_from_potential)
     call hx_field_set_rhs(tree, 0)
     call vcycle(.true., .false.)
     call vcycle(.true., .false.)
     call field_from_potential()
     call dump_state("regrid_in")
     call dump_refine_flags()
     call af_adjust_refinement(tree, ref_regrid, regrid_info)
     call dump_topology("topology_after.bin")
     call dump_in_use("in_use_after.bin")
     call dump_state("regrid")
     close(u_log)
     stop
  end if

  ! ------------------------------------------------------------------
  ! field_compute(tree, mg, 0, time, .true.), m_field.f90:405-485
  call hx_field_set_rhs(tree, 0)
  call dump_state("rhs")
  call af_tree_maxabs_cc(tree, i_rhs, max_rhs)
  threshold = max(1e-6_dp, max_rhs * 1e-4_dp, &
       1e-10_dp * abs(current_voltage) / (dom(3) * af_min_dr(tree)))
  write(u_log, *) "field0_threshold", threshold
  call vcycle(.true., trace)
  call dump_state("vcycle1")
  call af_tree_maxabs_cc(tree, i_tmp, residuals(1))
  write(u_log, *) "vcycle1_residual", residuals(1)
  call vcycle(.true., .false.)
  call dump_state("vcycle2")
  call af_tree_maxabs_cc(tree, i_tmp, residuals(2))
  write(u_log, *) "vcycle2_residual", residuals(2)
  call field_from_potential()
  call dump_state("field0")

  if (use_lsf) then
     ! FAS-FMG through the electrode stencils, from the potential above
     call dump_state("fmg_in")
     call fmg(.false.)
     call dump_state("fmg0")
     call fmg(.true.)
     call dump_state("fmg1")
     close(u_log)
     stop
  end if

  ! ------------------------------------------------------------------
  ! Heun sub-step 1: forward_euler(dt, s_deriv=0, [0], [1], s_out=1, 1, 2)
  dt = 2.0e-12_dp
  last_step = .false.
  call flux_upwind_tree(tree, 1, [i_e], 0, [f_flux], 2, dtl(1:2), &
       hx_flux_upwind, hx_flux_direction, flux_dummy_line_modify, &
       af_limiter_koren_t)
  write(u_log, *) "flux1_dt", dtl(1:2)
  call dump_state("flux1")
  call flux_update_densities(tree, dt, 3, [i_e, i_pos, i_neg], 1, [i_e], &
       [f_flux], 0, 1, [0], [1.0_dp], 1, hx_add_source_terms, 2, dtl(3:4), &
       hx_set_box_mask)
  write(u_log, *) "update1_dt", dtl(3:4)
  call dump_state("update1")

  ! Heun sub-step 2: field_compute(s=1), then
  ! forward_euler(dt/2, s_deriv=1, [0,1], [.5,.5], s_out=0, 2, 2)
  call hx_field_set_rhs(tree, 1)
  call af_tree_maxabs_cc(tree, i_rhs, max_rhs)
  threshold = max(1e-6_dp, max_rhs * 1e-4_dp, &
       1e-10_dp * abs(current_voltage) / (dom(3) * af_min_dr(tree)))
  write(u_log, *) "field1_threshold", threshold
  do i = 1, 2
     call vcycle(.true., .false.)
     call af_tree_maxabs_cc(tree, i_tmp, residuals(i))
     write(u_log, *) "field1_residual", i, residuals(i)
     if (residuals(i) < threshold) exit
  end do
  call field_from_potential()
  call dump_state("field1")

  last_step = .true.
  call flux_upwind_tree(tree, 1, [i_e], 1, [f_flux], 2, dtl(1:2), &
       hx_flux_upwind, hx_flux_direction, flux_dummy_line_modify, &
       af_limiter_koren_t)
  write(u_log, *) "flux2_dt", dtl(1:2)
  call dump_state("flux2")
  call flux_update_densities(tree, 0.5_dp * dt, 3, [i_e, i_pos, i_neg], 1, &
       [i_e], [f_flux], 1, 2, [0, 1], [0.5_dp, 0.5_dp], 0, &
       hx_add_source_terms, 2, dtl(3:4), hx_set_box_mask)
  write(u_log, *) "update2_dt", dtl(3:4)
  call dump_state("update2")

  ! ------------------------------------------------------------------
  ! FAS-FMG (m_af_multigrid.f90:137-180): the start-up solve without a guess
  ! (field_compute with have_guess = .false., m_field.f90:447-470), then with
  ! the result as guess
  call dump_state("fmg_in")
  call hx_field_set_rhs(tree, 0)
  call fmg(.false.)
  call dump_state("fmg0")
  call fmg(.true.)
  call dump_state("fmg1")

  ! ------------------------------------------------------------------
  ! Helmholtz FMG of a photoionization mode (photoi_helmh_compute,
  ! src/m_photoi_helmh.f90:162-204): helmholtz_lambda = lambda^2 in the
  ! operator (mg_box_lpl_stencil, m_af_multigrid.f90:1243), photoi_helmh_bc
  ! (Dirichlet 0 on the z faces, Neumann 0 elsewhere = hx_bc_phi with zero
  ! voltage), the mode starting from zero; FMG without and with guess
  current_voltage = 0.0_dp
  mg%helmholtz_lambda = helm_lambda**2
  ! a new operator stencil key, as mg_init gives every mg_t of a mode
  ! (stencils are stored once per key, m_af_multigrid.f90:1150-1154)
  tree%n_stencil_keys_stored = tree%n_stencil_keys_stored + 1
  mg%operator_key = tree%n_stencil_keys_stored
  call mg_set_operators_tree(tree, mg)
  call af_tree_clear_cc(tree, i_phi)
  call dump_state("helm_in")
  call fmg(.false.)
  call dump_state("helm0")
  call fmg(.true.)
  call dump_state("helm1")

  close(u_log)

contains

  !> Initial condition: Gaussian seed on a background (cf. init_cond_set_box,
  !> src/m_init_cond.f90:217-291), and a smooth initial potential guess.
  subroutine set_init(box)
    type(box_t), intent(inout) :: box
    integer                    :: IJK
    real(dp)                   :: r(3), d2

    do k = 0, box%n_cell+1
       do j = 0, box%n_cell+1
          do i = 0, box%n_cell+1
             r = af_r_cc(box, [IJK])
             d2 = sum((r - r0)**2)
             box%cc(IJK, i_e) = 1e15_dp + 5e18_dp * exp(-d2/width**2)
             box%cc(IJK, i_pos) = box%cc(IJK, i_e) + &
                  1e17_dp * exp(-d2/(2*width)**2)
             box%cc(IJK, i_neg) = 1e14_dp * (1 + r(1)/dom(1))
             box%cc(IJK, i_phi) = current_voltage * r(3) / dom(3) + &
                  50.0_dp * sin(6.2831853_dp * r(1) / dom(1)) * &
                  cos(3.1415926_dp * r(2) / dom(2))
          end do
       end do
    end do
  end subroutine set_init

  !> rod_lsf, src/m_field.f90:626-630
  real(dp) function rod_lsf(r)
    real(dp), intent(in) :: r(3)
    rod_lsf = GM_dist_line(r, rod_r0, rod_r1, 3) - rod_radius
  end function rod_lsf

  !> set_lsf_box, src/m_field.f90:608-619 (all cells, ghost cells included)
  subroutine set_lsf_box(box)
    type(box_t), intent(inout) :: box
    integer                    :: IJK
    do k = 0, box%n_cell+1
       do j = 0, box%n_cell+1
          do i = 0, box%n_cell+1
             box%cc(IJK, i_lsf) = rod_lsf(af_r_cc(box, [IJK]))
          end do
       end do
    end do
  end subroutine set_lsf_box

  !> The electrode stencils the reference stored (mg_set_operators_lvl,
  !> m_af_multigrid.f90:1133-1171) per box: the variable operator stencil
  !> v(7, nc^3) and its bc_correction (mg_box_lsf_stencil 1762-1834, f times
  !> mg_lsf_boundary_value), and the sparse boundary distances
  !> (store_lsf_distance_matrix 977-1097) with the boundary values, as used
  !> by mg_box_lpllsf_gradient (2030-2120).
  subroutine dump_lsf()
    integer :: u, id, ix, n, has
    open(newunit=u, file=trim(out_dir)//"/lsf.bin", &
         access="stream", form="unformatted", status="replace")
    do id = 1, tree%highest_id
       associate (box => tree%boxes(id))
         ix = af_stencil_index(box, mg%operator_key)
         has = 0
         if (ix > af_stencil_none) then
            if (box%stencils(ix)%stype == stencil_variable) has = 1
         end if
         write(u) has
         if (has == 1) then
            write(u) box%stencils(ix)%v
            has = 0
            if (allocated(box%stencils(ix)%bc_correction)) has = 1
            write(u) has
            if (has == 1) write(u) box%stencils(ix)%bc_correction
         end if
         ix = af_stencil_index(box, mg_lsf_distance_key)
         n = 0
         if (ix > af_stencil_none) n = size(box%stencils(ix)%sparse_ix, 2)
         write(u) n
         if (n > 0) then
            write(u) box%stencils(ix)%sparse_ix
            write(u) box%stencils(ix)%sparse_v
            write(u) mg_lsf_boundary_value(box, mg)
         end if
       end associate
    end do
    close(u)
  end subroutine dump_lsf

  subroutine ref_amr(box, cell_flags)
    type(box_t), intent(in) :: box
    integer, intent(out)    :: cell_flags(DTIMES(box%n_cell))
    real(dp)                :: rc(3), half(3)
    half = 0.5_dp * box%n_cell * box%dr
    rc = box%r_min + half
    if (box%lvl < amr_lvl .and. &
         all(abs(rc - r0) < half + 0.25_dp * width)) then
       cell_flags = af_do_ref
    else
       cell_flags = af_keep_ref
    end if
  end subroutine ref_amr

  !> Regrid rule: refine (up to level 4) where cells are near r1, remove
  !> refinement where all cells are far from it
  subroutine ref_regrid(box, cell_flags)
    type(box_t), intent(in) :: box
    integer, intent(out)    :: cell_flags(DTIMES(box%n_cell))
    integer                 :: IJK
    real(dp)                :: r1(3), d
    r1 = r0 + [0.35_dp, 0.0_dp, 0.0_dp] * dom
    do k = 1, box%n_cell
       do j = 1, box%n_cell
          do i = 1, box%n_cell
             d = norm2(af_r_cc(box, [IJK]) - r1)
             if (d < 1.0_dp * width .and. box%lvl < 4) then
                cell_flags(IJK) = af_do_ref
             else if (d > 1.6_dp * width) then
                cell_flags(IJK) = af_rm_ref
             else
                cell_flags(IJK) = af_keep_ref
             end if
          end do
       end do
    end do
  end subroutine ref_regrid

  !> default_refinement (src/m_refine.f90:198-298) with constant gas density,
  !> alpha without attachment, one initial seed, one refine region and one
  !> refine limit
  subroutine ref_default(box, cell_flags)
    type(box_t), intent(in) :: box
    integer, intent(out)    :: cell_flags(DTIMES(box%n_cell))
    integer                 :: IJK, nc
    real(dp)                :: min_dx, max_dx, alpha, adx, fld, dist
    real(dp)                :: rmin(3), rmax(3)
    nc = box%n_cell
    min_dx = minval(box%dr)
    max_dx = maxval(box%dr)
    do k = 1, nc
       do j = 1, nc
          do i = 1, nc
             fld = box%cc(IJK, i_efld) * SI_to_Townsend / gas_number_density
             alpha = LT_get_col(td_tbl, td_alpha, rf_adx_fac * fld) * &
                  gas_number_density / rf_adx_fac
             adx = max_dx * alpha
             if (adx > rf_adx .and. box%cc(IJK, i_e) > rf_min_dens) then
                cell_flags(IJK) = af_do_ref
             else if (adx < 0.125_dp * rf_adx .and. max_dx < rf_derefine_dx) then
                cell_flags(IJK) = af_rm_ref
             else
                cell_flags(IJK) = af_keep_ref
             end if
             dist = GM_dist_line(af_r_cc(box, [IJK]), rf_seed_r0, rf_seed_r1, 3)
             if (dist - rf_seed_width < 2 * max_dx .and. &
                  max_dx > rf_init_fac * rf_seed_width) cell_flags(IJK) = af_do_ref
          end do
       end do
    end do
    rmin = box%r_min
    rmax = box%r_min + box%dr * box%n_cell
    if (max_dx > rf_region_dr .and. all(rmax >= rf_region_rmin .and. &
         rmin <= rf_region_rmax)) cell_flags(DTIMES(nc/2)) = af_do_ref
    if (max_dx < 2 * rf_limit_dr .and. all(rmin >= rf_limit_rmin .and. &
         rmax <= rf_limit_rmax)) where (cell_flags == af_do_ref) cell_flags = af_keep_ref
    if (max_dx > rf_max_dx) then
       cell_flags = af_do_ref
    else if (min_dx < 2 * rf_min_dx) then
       where (cell_flags == af_do_ref) cell_flags = af_keep_ref
    end if
  end subroutine ref_default

  !> Per box: the flag cell_to_ref_flags gives the box itself
  !> (m_af_core.f90:1111-1118) and the neighbour directions whose buffer
  !> slab holds a refining cell (1124-1146), bit (dk+1)*9+(dj+1)*3+(di+1)
  subroutine dump_refine_flags()
    integer :: u, id, lvl, n, nc, IJK, di, dj, dk, ix0(3), ix1(3), f, m
    integer :: cf(tree%n_cell, tree%n_cell, tree%n_cell)
    integer, allocatable :: flags(:), masks(:)
    nc = tree%n_cell
    rf_seed_r0 = r0
    rf_seed_r1 = r0 + [0.0_dp, 0.0_dp, 0.3_dp] * dom
    rf_seed_width = 0.05_dp * dom(3)
    rf_region_dr = 1.0e-4_dp
    rf_region_rmin = [0.0_dp, 0.0_dp, 0.75_dp] * dom
    rf_region_rmax = [0.3_dp, 0.3_dp, 1.0_dp] * dom
    rf_limit_dr = 1.0e-4_dp
    rf_limit_rmin = [0.5_dp, 0.5_dp, 0.0_dp] * dom
    rf_limit_rmax = [1.0_dp, 1.0_dp, 0.5_dp] * dom
    allocate(flags(tree%highest_id), masks(tree%highest_id))
    flags = 0
    masks = 0
    do lvl = 1, tree%highest_lvl
       do n = 1, size(tree%lvls(lvl)%ids)
          id = tree%lvls(lvl)%ids(n)
          call ref_default(tree%boxes(id), cf)
          if (any(cf == af_do_ref)) then
             f = af_do_ref
          else if (any(cf == af_keep_ref)) then
             f = af_keep_ref
          else
             f = af_rm_ref
          end if
          m = 0
          do dk = -1, 1
             do dj = -1, 1
                do di = -1, 1
                   if (di == 0 .and. dj == 0 .and. dk == 0) cycle
                   ix0 = 1
                   ix1 = nc
                   where ([di, dj, dk] == 1)
                      ix0 = nc - rf_buffer + 1
                      ix1 = nc
                   elsewhere ([di, dj, dk] == -1)
                      ix0 = 1
                      ix1 = rf_buffer
                   end where
                   if (any(cf(ix0(1):ix1(1), ix0(2):ix1(2), ix0(3):ix1(3)) &
                        == af_do_ref)) m = ibset(m, (dk+1)*9 + (dj+1)*3 + (di+1))
                end do
             end do
          end do
          flags(id) = f
          masks(id) = m
       end do
    end do
    open(newunit=u, file=trim(out_dir)//"/refine.bin", &
         access="stream", form="unformatted", status="replace")
    write(u) tree%highest_id, flags, masks
    write(u) rf_adx, rf_adx_fac, rf_min_dens, rf_derefine_dx, rf_max_dx, &
         rf_min_dx, rf_init_fac, rf_seed_r0, rf_seed_r1, rf_seed_width, &
         rf_region_dr, rf_region_rmin, rf_region_rmax, rf_limit_dr, &
         rf_limit_rmin, rf_limit_rmax
    write(u) rf_buffer
    close(u)
  end subroutine dump_refine_flags

  subroutine dump_in_use(fname)
    character(len=*), intent(in) :: fname
    integer :: u, id
    open(newunit=u, file=trim(out_dir)//"/"//fname, &
         access="stream", form="unformatted", status="replace")
    write(u) tree%highest_id
    write(u) [(merge(1, 0, tree%boxes(id)%in_use), id = 1, tree%highest_id)]
    close(u)
  end subroutine dump_in_use

  subroutine refine_amr()
    type(ref_info_t) :: ref_info
    call af_adjust_refinement(tree, ref_amr, ref_info)
  end subroutine refine_amr

  ! ---------------- FAS V-cycle (m_af_multigrid.f90:185-264) ----------------
  !> mg_fas_fmg, m_af_multigrid.f90:137-180, with set_residual = .true.
  subroutine fmg(have_guess)
    logical, intent(in) :: have_guess
    integer             :: lvl, i, id, p_id

    if (have_guess) then
       do lvl = tree%highest_lvl, 2, -1
          ! set_coarse_phi_rhs, m_af_multigrid.f90:742-776
          if (lvl == tree%highest_lvl) call af_gc_lvl(tree, lvl, [mg%i_phi])
          do i = 1, size(tree%lvls(lvl)%ids)
             id = tree%lvls(lvl)%ids(i)
             p_id = tree%boxes(id)%parent
             call residual_box(tree%boxes(id))
             call af_restrict_box(tree%boxes(id), tree%boxes(p_id), [mg%i_tmp], &
                  use_geometry=.true.)
             call af_restrict_box(tree%boxes(id), tree%boxes(p_id), [mg%i_phi], &
                  use_geometry=.false.)
          end do
          call af_gc_lvl(tree, lvl-1, [mg%i_phi])
          do i = 1, size(tree%lvls(lvl-1)%parents)
             id = tree%lvls(lvl-1)%parents(i)
             call af_stencil_apply_box(tree%boxes(id), mg%operator_key, &
                  mg%i_phi, mg%i_rhs)
             call af_box_add_cc(tree%boxes(id), mg%i_tmp, mg%i_rhs)
          end do
       end do
    else
       ! init_phi_rhs, m_af_multigrid.f90:779-799
       do lvl = tree%highest_lvl, 2, -1
          do i = 1, size(tree%lvls(lvl)%ids)
             id = tree%lvls(lvl)%ids(i)
             tree%boxes(id)%cc(:, :, :, mg%i_phi) = 0.0_dp
             p_id = tree%boxes(id)%parent
             call af_restrict_box(tree%boxes(id), tree%boxes(p_id), [mg%i_rhs], &
                  use_geometry=.true.)
          end do
       end do
    end if

    do i = 1, size(tree%lvls(1)%ids)
       id = tree%lvls(1)%ids(i)
       tree%boxes(id)%cc(:, :, :, mg%i_tmp) = tree%boxes(id)%cc(:, :, :, mg%i_phi)
    end do
    call vcycle(1 == tree%highest_lvl, .false., 1)

    do lvl = 2, tree%highest_lvl
       do i = 1, size(tree%lvls(lvl)%ids)
          id = tree%lvls(lvl)%ids(i)
          tree%boxes(id)%cc(:, :, :, mg%i_tmp) = tree%boxes(id)%cc(:, :, :, mg%i_phi)
       end do
       call correct_children(tree%lvls(lvl-1)%parents)
       call af_gc_lvl(tree, lvl, [mg%i_phi])
       call vcycle(lvl == tree%highest_lvl, .false., lvl)
    end do
  end subroutine fmg

  subroutine vcycle(set_residual, do_trace, highest)
    logical, intent(in) :: set_residual, do_trace
    integer, intent(in), optional :: highest
    integer             :: lvl, i, id, max_lvl
    character(len=40)   :: tag

    max_lvl = tree%highest_lvl
    if (present(highest)) max_lvl = highest

    do lvl = max_lvl, 2, -1
       call gsrb_boxes(lvl, mg_cycle_down)
       if (do_trace) then
          write(tag, "(A,I0)") "tr_gsrb_down_", lvl
          call dump_state(trim(tag))
       end if
       call update_coarse(lvl)
       if (do_trace) then
          write(tag, "(A,I0)") "tr_update_coarse_", lvl
          call dump_state(trim(tag))
       end if
    end do

    call solve_coarse_exact()
    if (do_trace) call dump_state("tr_coarse")

    do lvl = 2, max_lvl
       call correct_children(tree%lvls(lvl-1)%parents)
       call af_gc_lvl(tree, lvl, [mg%i_phi])
       if (do_trace) then
          write(tag, "(A,I0)") "tr_correct_", lvl
          call dump_state(trim(tag))
       end if
       call gsrb_boxes(lvl, mg_cycle_up)
       if (do_trace) then
          write(tag, "(A,I0)") "tr_gsrb_up_", lvl
          call dump_state(trim(tag))
       end if
    end do

    if (set_residual) then
       do lvl = 1, max_lvl
          do i = 1, size(tree%lvls(lvl)%ids)
             id = tree%lvls(lvl)%ids(i)
             call residual_box(tree%boxes(id))
          end do
       end do
    end if
  end subroutine vcycle

  !> gsrb_boxes, m_af_multigrid.f90:648-687 (box_gsrb = mg_auto_gsrb)
  subroutine gsrb_boxes(lvl, type_cycle)
    integer, intent(in) :: lvl, type_cycle
    integer             :: n, i, n_cycle
    logical             :: use_corners

    if (type_cycle == mg_cycle_down) then
       n_cycle = mg%n_cycle_down
    else
       n_cycle = mg%n_cycle_up
    end if

    associate (ids => tree%lvls(lvl)%ids)
      do n = 1, 2 * n_cycle
         do i = 1, size(ids)
            call af_stencil_gsrb_box(tree%boxes(ids(i)), mg%operator_key, &
                 n, mg%i_phi, mg%i_rhs)
         end do
         use_corners = mg%use_corners .or. &
              (type_cycle /= mg_cycle_down .and. n == 2 * n_cycle)
         do i = 1, size(ids)
            call af_gc_box(tree, ids(i), [mg%i_phi], use_corners)
         end do
      end do
    end associate
  end subroutine gsrb_boxes

  !> residual_box, m_af_multigrid.f90:801-810 (box_op = mg_auto_op)
  subroutine residual_box(box)
    type(box_t), intent(inout) :: box
    integer                    :: nc
    call af_stencil_apply_box(box, mg%operator_key, mg%i_phi, mg%i_tmp)
    nc = box%n_cell
    box%cc(DTIMES(1:nc), mg%i_tmp) = box%cc(DTIMES(1:nc), mg%i_rhs) &
         - box%cc(DTIMES(1:nc), mg%i_tmp)
  end subroutine residual_box

  !> update_coarse, m_af_multigrid.f90:691-738 (box_rstr = mg_box_rstr_lpl)
  subroutine update_coarse(lvl)
    integer, intent(in)   :: lvl
    integer               :: i, id, p_id, nc
    real(dp), allocatable :: tmp(DTIMES(:))

    nc = tree%n_cell
    allocate(tmp(DTIMES(1:nc)))

    do i = 1, size(tree%lvls(lvl)%ids)
       id = tree%lvls(lvl)%ids(i)
       p_id = tree%boxes(id)%parent
       tmp = tree%boxes(id)%cc(DTIMES(1:nc), mg%i_tmp)
       call residual_box(tree%boxes(id))
       call af_restrict_box(tree%boxes(id), tree%boxes(p_id), [mg%i_tmp], &
            use_geometry=.true.)
       call af_restrict_box(tree%boxes(id), tree%boxes(p_id), [mg%i_phi], &
            use_geometry=.false.)
       tree%boxes(id)%cc(DTIMES(1:nc), mg%i_tmp) = tmp
    end do

    call af_gc_lvl(tree, lvl-1, [mg%i_phi])

    do i = 1, size(tree%lvls(lvl-1)%parents)
       id = tree%lvls(lvl-1)%parents(i)
       call af_stencil_apply_box(tree%boxes(id), mg%operator_key, mg%i_phi, &
            mg%i_rhs)
       call af_box_add_cc(tree%boxes(id), mg%i_tmp, mg%i_rhs)
       call af_box_copy_cc(tree%boxes(id), mg%i_phi, mg%i_tmp)
    end do
  end subroutine update_coarse

  !> correct_children, m_af_multigrid.f90:624-646 (box_corr = mg_auto_corr)
  subroutine correct_children(ids)
    integer, intent(in) :: ids(:)
    integer             :: i, id, i_c, c_id

    do i = 1, size(ids)
       id = ids(i)
       tree%boxes(id)%cc(DTIMES(:), mg%i_tmp) = &
            tree%boxes(id)%cc(DTIMES(:), mg%i_phi) - &
            tree%boxes(id)%cc(DTIMES(:), mg%i_tmp)
       do i_c = 1, af_num_children
          c_id = tree%boxes(id)%children(i_c)
          if (c_id == af_no_box) cycle
          call af_stencil_prolong_box(tree%boxes(id), tree%boxes(c_id), &
               mg%prolongation_key, mg%i_tmp, mg%i_phi, .true.)
       end do
    end do
  end subroutine correct_children

  !> Exact level-1 solve (stands in for the HYPRE call in solve_coarse_grid,
  !> m_af_multigrid.f90:266-291): GSRB sweeps until phi is stationary, then
  !> af_gc_lvl(tree, 1, [i_phi]) as the reference does after HYPRE.
  subroutine solve_coarse_exact()
    integer  :: it, n, i, id, nc
    real(dp) :: diff, vmax
    real(dp), allocatable :: old(:, :, :, :)

    nc = tree%n_cell
    allocate(old(0:nc+1, 0:nc+1, 0:nc+1, size(tree%lvls(1)%ids)))
    do it = 1, 200000
       do i = 1, size(tree%lvls(1)%ids)
          old(:, :, :, i) = tree%boxes(tree%lvls(1)%ids(i))%cc(:, :, :, i_phi)
       end do
       do n = 1, 2
          do i = 1, size(tree%lvls(1)%ids)
             call af_stencil_gsrb_box(tree%boxes(tree%lvls(1)%ids(i)), &
                  mg%operator_key, n, mg%i_phi, mg%i_rhs)
          end do
          do i = 1, size(tree%lvls(1)%ids)
             call af_gc_box(tree, tree%lvls(1)%ids(i), [mg%i_phi], .false.)
          end do
       end do
       diff = 0; vmax = 0
       do i = 1, size(tree%lvls(1)%ids)
          id = tree%lvls(1)%ids(i)
          diff = max(diff, maxval(abs(tree%boxes(id)%cc(1:nc, 1:nc, 1:nc, &
               i_phi) - old(1:nc, 1:nc, 1:nc, i))))
          vmax = max(vmax, maxval(abs(tree%boxes(id)%cc(1:nc, 1:nc, 1:nc, &
               i_phi))))
       end do
       if (diff <= 4 * spacing(vmax) .and. it > 10) exit
    end do
    write(u_log, *) "coarse_iterations", it, diff, vmax
    call af_gc_lvl(tree, 1, [mg%i_phi])
  end subroutine solve_coarse_exact

  !> field_from_potential, m_field.f90:488-505 (no dielectric)
  subroutine field_from_potential()
    call mg_compute_phi_gradient(tree, mg, f_field, -1.0_dp, i_efld)
    call af_gc_tree(tree, [i_efld])
  end subroutine field_from_potential

  ! ---------------- raw binary dumps ----------------
  subroutine dump_state(name)
    character(len=*), intent(in) :: name
    integer                      :: u, id
    n_dump = n_dump + 1
    open(newunit=u, file=trim(out_dir)//"/state_"//name//".bin", &
         access="stream", form="unformatted", status="replace")
    do id = 1, tree%highest_id
       write(u) tree%boxes(id)%cc
    end do
    do id = 1, tree%highest_id
       write(u) tree%boxes(id)%fc
    end do
    close(u)
    write(u_log, *) "state ", name
  end subroutine dump_state

  subroutine dump_topology(fname)
    character(len=*), intent(in) :: fname
    integer :: u, id, lvl
    open(newunit=u, file=trim(out_dir)//"/"//fname, &
         access="stream", form="unformatted", status="replace")
    write(u) tree%n_cell, tree%highest_id, tree%highest_lvl, &
         tree%n_var_cell, tree%n_var_face
    write(u) tree%coarse_grid_size(1:3)
    write(u) tree%r_base, tree%dr_base
    do id = 1, tree%highest_id
       associate (b => tree%boxes(id))
         write(u) b%lvl, b%ix, b%parent, b%children, b%neighbors, &
              b%neighbor_mat, b%r_min, b%dr
       end associate
    end do
    do lvl = 1, tree%highest_lvl
       write(u) size(tree%lvls(lvl)%ids), size(tree%lvls(lvl)%leaves), &
            size(tree%lvls(lvl)%parents)
       write(u) tree%lvls(lvl)%ids, tree%lvls(lvl)%leaves, &
            tree%lvls(lvl)%parents
    end do
    write(u) current_voltage, gas_number_density, dom
    close(u)
  end subroutine dump_topology

  subroutine dump_tables()
    integer :: u
    open(newunit=u, file=trim(out_dir)//"/tables.bin", &
         access="stream", form="unformatted", status="replace")
    write(u) td_tbl%n_points, td_tbl%n_cols, td_tbl%x_min, td_tbl%inv_fac
    write(u) td_tbl%rows_cols
    write(u) chemtbl_fld%n_points, chemtbl_fld%n_cols, chemtbl_fld%x_min, &
         chemtbl_fld%inv_fac
    write(u) chemtbl_fld%rows_cols
    close(u)
  end subroutine dump_tables

end program golden_gen
