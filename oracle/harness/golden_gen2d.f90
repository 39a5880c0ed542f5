!> ORACLE TEST INFRASTRUCTURE -- 2-D golden-vector generator (build container only).
!>
!> The NDIM = 2 twin of golden_gen.f90 for BASELINE config 1 (the reference's
!> 2-D build, afivo/lib_2d/Makefile: the same afivo sources compiled with
!> NDIM=2). Drives those numerics, compiled from /root/reference with
!> -DNDIM=2 by oracle/Makefile (target ref2d), through one Heun time step of
!> the streamer hot path and dumps every intermediate state as raw binary:
!>
!>   field_compute (rhs, FAS V-cycles, field_from_potential)
!>   -> flux_upwind_tree (sub-step 1) -> flux_update_densities
!>   -> field_compute -> flux_upwind_tree (sub-step 2) -> flux_update_densities
!>   -> FAS-FMG without / with a guess -> a Helmholtz FMG
!>
!> As in golden_gen.f90 the V-cycle re-sequences the reference's public box
!> routines exactly as mg_fas_vcycle does (m_af_multigrid.f90:185-264, 624-738,
!> 801-810), and the level-1 problem is solved to stationarity with the
!> reference's own af_stencil_gsrb_box + af_gc_box (HYPRE, which mg_init and
!> solve_coarse_grid call, is absent). The physics callbacks are hx_physics,
!> compiled with NDIM=2 (its flux line extraction, boundary conditions and
!> chemistry are written for any NDIM).
!>
!> Usage: golden_gen2d <case> <td_file> <out_dir>
!>   case = uni2d (uniform, 2 x 2 level-1 boxes of 8^2, 3 levels)
!>        | amr2d (16 x 8 coarse cells, refined around a point to level 5)
program golden_gen2d
#include "cpp_macros.h"
  use m_af_types
  use m_af_core
  use m_af_utils
  use m_af_ghostcell
  use m_af_stencil
  use m_af_restrict
  use m_af_multigrid
  use m_af_flux_schemes
  use m_af_limiters
  use hx_physics

  implicit none

  type(af_t)         :: tree
  type(mg_t)         :: mg
  character(len=256) :: case_name, td_file, out_dir
  integer            :: nc, grid(NDIM), max_lvl, amr_lvl, i
  real(dp)           :: dom(NDIM), r0(NDIM), width, dt, dtl(4), residuals(2)
  real(dp)           :: max_rhs, threshold
  ! photoionization Helmholtz mode: Bourdon's second lambda at 1 bar
  ! (src/m_photoi_helmh.f90:100), 1/m
  real(dp), parameter :: helm_lambda = 44081.25_dp
  integer            :: u_log

  call get_command_argument(1, case_name)
  call get_command_argument(2, td_file)
  call get_command_argument(3, out_dir)

  select case (trim(case_name))
  case ("uni2d")
     nc = 8; grid = [16, 16]; max_lvl = 3; amr_lvl = 0
  case ("amr2d")
     nc = 8; grid = [16, 8]; max_lvl = 2; amr_lvl = 5
  case default
     error stop "unknown case"
  end select

  ! Domain: cells are square at every level
  dom = 1.0e-3_dp * grid / 4
  r0  = 0.5_dp * dom
  r0(1) = 0.4_dp * dom(1)
  width = 0.15_dp * dom(NDIM)

  call hx_init_gas(1.0_dp, 300.0_dp)
  call hx_init_transport(trim(td_file))
  ! Background field -2.5 MV/m along the last dimension:
  ! current_voltage = -L * E (m_field.f90:516)
  current_voltage = -dom(NDIM) * (-2.5e6_dp)

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

  ! Ghost-cell methods as set by streamer.f90:81-84 and m_field.f90:349-350;
  ! phi gets (sides_bc, mg_auto_rb) as in mg_init (m_af_multigrid.f90:102-105)
  call af_set_cc_methods(tree, i_e, af_bc_neumann_zero, af_gc_interp_lim)
  call af_set_cc_methods(tree, i_pos, af_bc_neumann_zero, af_gc_interp_lim)
  call af_set_cc_methods(tree, i_neg, af_bc_neumann_zero, af_gc_interp_lim)
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
  call mg_set_operators_tree(tree, mg)

  call af_loop_box(tree, set_init)
  call af_restrict_tree(tree, [i_e, i_pos, i_neg])
  call af_gc_tree(tree, [i_e, i_pos, i_neg])
  call af_gc_tree(tree, [i_phi])

  open(newunit=u_log, file=trim(out_dir)//"/log.txt", status="replace")
  call dump_topology("topology.bin")
  call dump_tables()
  call dump_state("init")

  ! ------------------------------------------------------------------
  ! field_compute(tree, mg, 0, time, .true.), m_field.f90:405-485
  call hx_field_set_rhs(tree, 0)
  call dump_state("rhs")
  call af_tree_maxabs_cc(tree, i_rhs, max_rhs)
  threshold = max(1e-6_dp, max_rhs * 1e-4_dp, &
       1e-10_dp * abs(current_voltage) / (dom(NDIM) * af_min_dr(tree)))
  write(u_log, *) "field0_threshold", threshold
  call vcycle(.true.)
  call dump_state("vcycle1")
  call af_tree_maxabs_cc(tree, i_tmp, residuals(1))
  write(u_log, *) "vcycle1_residual", residuals(1)
  call vcycle(.true.)
  call dump_state("vcycle2")
  call af_tree_maxabs_cc(tree, i_tmp, residuals(2))
  write(u_log, *) "vcycle2_residual", residuals(2)
  call field_from_potential()
  call dump_state("field0")

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
       1e-10_dp * abs(current_voltage) / (dom(NDIM) * af_min_dr(tree)))
  write(u_log, *) "field1_threshold", threshold
  do i = 1, 2
     call vcycle(.true.)
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
  ! FAS-FMG (m_af_multigrid.f90:137-180) without and with a guess
  call dump_state("fmg_in")
  call hx_field_set_rhs(tree, 0)
  call fmg(.false.)
  call dump_state("fmg0")
  call fmg(.true.)
  call dump_state("fmg1")

  ! ------------------------------------------------------------------
  ! Helmholtz FMG of a photoionization mode (m_photoi_helmh.f90:162-204):
  ! lambda^2 in the operator, Dirichlet 0 on the last dimension's faces
  current_voltage = 0.0_dp
  mg%helmholtz_lambda = helm_lambda**2
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
    real(dp)                   :: r(NDIM), d2

    do KJI_DO(0, box%n_cell+1)
       r = af_r_cc(box, [IJK])
       d2 = sum((r - r0)**2)
       box%cc(IJK, i_e) = 1e15_dp + 5e18_dp * exp(-d2/width**2)
       box%cc(IJK, i_pos) = box%cc(IJK, i_e) + &
            1e17_dp * exp(-d2/(2*width)**2)
       box%cc(IJK, i_neg) = 1e14_dp * (1 + r(1)/dom(1))
       box%cc(IJK, i_phi) = current_voltage * r(NDIM) / dom(NDIM) + &
            50.0_dp * sin(6.2831853_dp * r(1) / dom(1))
    end do; CLOSE_DO
  end subroutine set_init

  subroutine ref_amr(box, cell_flags)
    type(box_t), intent(in) :: box
    integer, intent(out)    :: cell_flags(DTIMES(box%n_cell))
    real(dp)                :: rc(NDIM), half(NDIM)
    half = 0.5_dp * box%n_cell * box%dr
    rc = box%r_min + half
    if (box%lvl < amr_lvl .and. &
         all(abs(rc - r0) < half + 0.25_dp * width)) then
       cell_flags = af_do_ref
    else
       cell_flags = af_keep_ref
    end if
  end subroutine ref_amr

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
             tree%boxes(id)%cc(DTIMES(:), mg%i_phi) = 0.0_dp
             p_id = tree%boxes(id)%parent
             call af_restrict_box(tree%boxes(id), tree%boxes(p_id), [mg%i_rhs], &
                  use_geometry=.true.)
          end do
       end do
    end if

    do i = 1, size(tree%lvls(1)%ids)
       id = tree%lvls(1)%ids(i)
       tree%boxes(id)%cc(DTIMES(:), mg%i_tmp) = tree%boxes(id)%cc(DTIMES(:), mg%i_phi)
    end do
    call vcycle(1 == tree%highest_lvl, 1)

    do lvl = 2, tree%highest_lvl
       do i = 1, size(tree%lvls(lvl)%ids)
          id = tree%lvls(lvl)%ids(i)
          tree%boxes(id)%cc(DTIMES(:), mg%i_tmp) = tree%boxes(id)%cc(DTIMES(:), mg%i_phi)
       end do
       call correct_children(tree%lvls(lvl-1)%parents)
       call af_gc_lvl(tree, lvl, [mg%i_phi])
       call vcycle(lvl == tree%highest_lvl, lvl)
    end do
  end subroutine fmg

  subroutine vcycle(set_residual, highest)
    logical, intent(in) :: set_residual
    integer, intent(in), optional :: highest
    integer             :: lvl, i, id, max_lvl

    max_lvl = tree%highest_lvl
    if (present(highest)) max_lvl = highest

    do lvl = max_lvl, 2, -1
       call gsrb_boxes(lvl, mg_cycle_down)
       call update_coarse(lvl)
    end do

    call solve_coarse_exact()

    do lvl = 2, max_lvl
       call correct_children(tree%lvls(lvl-1)%parents)
       call af_gc_lvl(tree, lvl, [mg%i_phi])
       call gsrb_boxes(lvl, mg_cycle_up)
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
    real(dp), allocatable :: old(:, :, :)

    nc = tree%n_cell
    allocate(old(0:nc+1, 0:nc+1, size(tree%lvls(1)%ids)))
    do it = 1, 2000000
       do i = 1, size(tree%lvls(1)%ids)
          old(:, :, i) = tree%boxes(tree%lvls(1)%ids(i))%cc(:, :, i_phi)
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
          diff = max(diff, maxval(abs(tree%boxes(id)%cc(1:nc, 1:nc, &
               i_phi) - old(1:nc, 1:nc, i))))
          vmax = max(vmax, maxval(abs(tree%boxes(id)%cc(1:nc, 1:nc, i_phi))))
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
    write(u) tree%coarse_grid_size(1:NDIM)
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

end program golden_gen2d
