!> ORACLE TEST INFRASTRUCTURE (build container only) -- CPU timing of the
!> reference's own code on the bench workloads (BASELINE.md).
!>
!> The modules are set up from a .cfg as the streamer does (as replay_step);
!> a uniform tree of `levels` levels is built with af_init +
!> af_refine_up_to_lvl, the densities set by init_cond_set_box, phi by the
!> applied field (field_bc_homogeneous's linear potential) and E by
!> field_from_potential (m_field.f90:488-505). Timed, with the OpenMP thread
!> count of the environment:
!>  * species: forward_euler (src/m_fluid.f90:21-99, flux_upwind_tree +
!>    flux_update_densities with the chemistry) with i_step = n_steps = 1, so
!>    it never reaches field_compute, Heun stages 1 and 2 alternating;
!>  * V-cycle: mg_fas_vcycle (m_af_multigrid.f90:185-264) re-sequenced from
!>    the reference's public box routines (af_stencil_gsrb_box,
!>    af_stencil_apply_box, af_gc_box / af_gc_lvl, af_restrict_box,
!>    af_stencil_prolong_box) with the reference's OpenMP loops; the level-1
!>    solve (HYPRE in the reference, absent here) is not timed.
!> mg_init is replaced by its stencil set-up (mg_set_operators_tree), as in
!> golden_gen, since its coarse-solver set-up needs HYPRE.
!>
!> Record mode (round 6): instead of <levels>, a record file of
!> replay_step's format (the topology and every variable of a state the
!> device driver reached, e.g. streamer_2d.cfg's own set-up tree): the tree
!> is rebuilt with af_adjust_refinement box for box and loaded, so the
!> reference is timed on the very tree the GPU bench line runs.
!>
!> Usage: ref_timing <levels|record> <repeats> <cfg> [-key=value ...]
!> Prints "TIMING species_s <s per step> vcycle_s <s per V-cycle> cells <n>".
#include "cpp_macros.h"
program ref_timing
  use m_config
  use m_af_all
  use m_streamer
  use m_field
  use m_init_cond
  use m_refine
  use m_photoi
  use m_chemistry
  use m_gas
  use m_dt
  use m_transport_data
  use m_table_data
  use m_model
  use m_fluid
  use omp_lib
  implicit none

  type(CFG_t)        :: cfg
  type(af_t)         :: tree
  type(ref_info_t)   :: ref_info
  character(len=512) :: arg, rec_file
  integer            :: n, levels, reps, k, lvl, ios, ur, hid, nvc, nvf, nc_rec, id, iv
  integer, allocatable :: parent(:), blvl(:), bix(:, :), in_use(:), rid(:)
  real(dp)           :: t0, t_species, t_vcycle, dt_lim, dt, time
  logical            :: from_record

  call get_command_argument(1, arg)
  ! (a path is not read as a number: list-directed input ends at its '/')
  from_record = verify(trim(arg), "0123456789") /= 0
  if (from_record) then
     rec_file = arg
  else
     read(arg, *, iostat=ios) levels
  end if
  call get_command_argument(2, arg)
  read(arg, *) reps
  do n = 3, command_argument_count()
     call get_command_argument(n, arg)
     if (arg(1:1) == '-') then
        call CFG_update_from_line(cfg, trim(arg(2:)))
     else
        call CFG_read_file(cfg, trim(arg))
     end if
  end do

  call model_initialize(cfg)
  call dt_initialize(cfg)
  call table_data_initialize(cfg)
  call gas_initialize(tree, cfg)
  call transport_data_initialize(cfg)
  call chemistry_initialize(tree, cfg)
  call ST_initialize(tree, cfg, NDIM)
  call photoi_initialize(tree, cfg)
  call refine_initialize(cfg)
  call field_initialize(tree, cfg, mg)
  call init_cond_initialize(tree, cfg)
  do n = 1, size(all_densities)
     call af_set_cc_methods(tree, all_densities(n), bc_species, af_gc_interp_lim, &
          ST_prolongation_method)
  end do
  do n = 1, tree%n_var_cell
     if (tree%cc_write_output(n) .and. .not. (tree%has_cc_method(n) .or. n == i_phi)) &
          call af_set_cc_methods(tree, n, af_bc_neumann_zero, af_gc_interp, &
          ST_prolongation_method)
  end do

  call af_init(tree, ST_box_size, ST_domain_origin + ST_domain_len, &
       ST_coarse_grid_size, periodic=ST_periodic, coord=af_xyz, &
       r_min=ST_domain_origin, mem_limit_gb=200.0_dp)
  if (from_record) then
     ! the recorded topology (replay_step.f90's record layout)
     open(newunit=ur, file=trim(rec_file), access="stream", form="unformatted", &
          action="read")
     read(ur) hid, nvc, nvf, nc_rec
     if (nvc /= tree%n_var_cell .or. nvf /= tree%n_var_face) &
          error stop "record: variable registry differs"
     allocate(parent(hid), blvl(hid), bix(3, hid), in_use(hid), rid(hid))
     do id = 1, hid
        read(ur) parent(id), blvl(id), bix(:, id), in_use(id)
     end do
     do lvl = 1, 29
        call af_adjust_refinement(tree, refine_as_recorded, ref_info)
        if (ref_info%n_add == 0) exit
     end do
     rid = 0
     do id = 1, hid
        if (in_use(id) == 0) cycle
        do n = 1, tree%highest_id
           if (tree%boxes(n)%in_use .and. tree%boxes(n)%lvl == blvl(id)) then
              if (all(tree%boxes(n)%ix == bix(1:NDIM, id))) then
                 rid(id) = n
                 exit
              end if
           end if
        end do
        if (rid(id) == 0) error stop "recorded box missing in the rebuilt tree"
     end do
  else
     call af_refine_up_to_lvl(tree, levels)
  end if

  ! mg_init (m_af_multigrid.f90:43-109) without the HYPRE set-up
  tree%n_stencil_keys_stored = tree%n_stencil_keys_stored + 1
  mg%operator_key = tree%n_stencil_keys_stored
  tree%n_stencil_keys_stored = tree%n_stencil_keys_stored + 1
  mg%prolongation_key = tree%n_stencil_keys_stored
  mg%initialized = .true.
  tree%mg_current_operator_mask = mg%operator_mask
  if (.not. associated(mg%sides_rb)) mg%sides_rb => auto_rb
  if (.not. tree%has_cc_method(mg%i_phi)) &
       call af_set_cc_methods(tree, mg%i_phi, mg%sides_bc, mg%sides_rb)
  call mg_set_operators_tree(tree, mg)

  if (from_record) then
     ! the recorded state (skipping dt .. s_out), every variable of every box
     read(ur) dt, time, k, k
     do n = 1, k
        read(ur) lvl
     end do
     do n = 1, k
        read(ur) t0
     end do
     read(ur) lvl
     do iv = 1, nvc
        do id = 1, hid
           if (in_use(id) /= 0) read(ur) tree%boxes(rid(id))%cc(DTIMES(:), iv)
        end do
     end do
     do iv = 1, nvf
        do id = 1, hid
           if (in_use(id) /= 0) read(ur) tree%boxes(rid(id))%fc(DTIMES(:), :, iv)
        end do
     end do
     close(ur)
  else
     call af_loop_box(tree, init_cond_set_box)
     call af_loop_box(tree, set_phi)
     call af_gc_tree(tree, all_densities)
     call af_gc_tree(tree, [i_phi])
     call field_from_potential(tree, mg)
     call af_loop_box(tree, set_rhs)
  end if

  ! species: forward_euler, Heun stages alternating (one warm-up pair)
  dt = 1e-13_dp
  time = 0
  do k = 0, 2 * reps + 1
     if (k == 2) t0 = omp_get_wtime()
     dt_lim = 1e100_dp
     if (mod(k, 2) == 0) then
        call forward_euler(tree, dt, dt, dt_lim, time, 0, 1, [0], [1.0_dp], 1, 1, 1)
     else
        call forward_euler(tree, 0.5_dp * dt, 0.5_dp * dt, dt_lim, time, 1, 2, [0, 1], &
             [0.5_dp, 0.5_dp], 0, 1, 1)
     end if
  end do
  t_species = (omp_get_wtime() - t0) / (2 * reps)

  ! V-cycle without the level-1 solve (one warm-up cycle)
  t_vcycle = 0
  do k = 0, reps
     t0 = omp_get_wtime()
     do lvl = tree%highest_lvl, 2, -1
        call gsrb_boxes(lvl, mg_cycle_down)
        call update_coarse(lvl)
     end do
     do lvl = 2, tree%highest_lvl
        call correct_children(lvl - 1)
        call af_gc_lvl(tree, lvl, [mg%i_phi])
        call gsrb_boxes(lvl, mg_cycle_up)
     end do
     call residual_tree()
     if (k > 0) t_vcycle = t_vcycle + (omp_get_wtime() - t0)
  end do
  t_vcycle = t_vcycle / reps

  write(*, '(A,ES12.4,A,ES12.4,A,I0,A,I0,A,I0)') "TIMING species_s ", t_species, &
       " vcycle_s ", t_vcycle, " cells ", af_num_leaves_used(tree) * ST_box_size**NDIM, &
       " threads ", omp_get_max_threads(), " boxes ", af_num_boxes_used(tree)

contains

  !> Refine the boxes the record lists as parents (replay_step.f90)
  subroutine refine_as_recorded(box, cell_flags)
    type(box_t), intent(in) :: box
    integer, intent(out)    :: cell_flags(DTIMES(box%n_cell))
    integer                 :: c
    logical                 :: has_child
    has_child = .false.
    do c = 1, hid
       if (in_use(c) /= 0 .and. blvl(c) == box%lvl + 1) then
          if (all((bix(1:NDIM, c) + 1) / 2 == box%ix)) then
             has_child = .true.
             exit
          end if
       end if
    end do
    if (has_child) then
       cell_flags = af_do_ref
    else
       cell_flags = af_keep_ref
    end if
  end subroutine refine_as_recorded

  !> mg_auto_rb (m_af_multigrid.f90:926-940) for a constant-coefficient box
  subroutine auto_rb(boxes, id, nb, iv, op_mask)
    type(box_t), intent(inout) :: boxes(:)
    integer, intent(in)        :: id, nb, iv, op_mask
    call mg_sides_rb(boxes, id, nb, iv)
  end subroutine auto_rb

  subroutine set_phi(box)
    type(box_t), intent(inout) :: box
    integer :: IJK, nc
    real(dp) :: r(NDIM)
    nc = box%n_cell
    do KJI_DO(0, nc+1)
       r = af_r_cc(box, [IJK])
       box%cc(IJK, i_phi) = current_voltage * (r(NDIM) - ST_domain_origin(NDIM)) / &
            ST_domain_len(NDIM)
    end do; CLOSE_DO
  end subroutine set_phi

  subroutine set_rhs(box)
    type(box_t), intent(inout) :: box
    box%cc(DTIMES(:), i_rhs) = 1e-3_dp * box%cc(DTIMES(:), i_electron)
  end subroutine set_rhs

  !> gsrb_boxes (m_af_multigrid.f90:648-687) with its OpenMP loops
  subroutine gsrb_boxes(lvl, type_cycle)
    integer, intent(in) :: lvl, type_cycle
    integer             :: n, i, n_cycle
    logical             :: use_corners
    n_cycle = merge(mg%n_cycle_down, mg%n_cycle_up, type_cycle == mg_cycle_down)
    !$omp parallel private(n, i, use_corners)
    do n = 1, 2 * n_cycle
       !$omp do
       do i = 1, size(tree%lvls(lvl)%ids)
          call af_stencil_gsrb_box(tree%boxes(tree%lvls(lvl)%ids(i)), mg%operator_key, &
               n, mg%i_phi, mg%i_rhs)
       end do
       !$omp end do
       use_corners = mg%use_corners .or. &
            (type_cycle /= mg_cycle_down .and. n == 2 * n_cycle)
       !$omp do
       do i = 1, size(tree%lvls(lvl)%ids)
          call af_gc_box(tree, tree%lvls(lvl)%ids(i), [mg%i_phi], use_corners)
       end do
       !$omp end do
    end do
    !$omp end parallel
  end subroutine gsrb_boxes

  subroutine residual_box(box)
    type(box_t), intent(inout) :: box
    integer                    :: nc
    call af_stencil_apply_box(box, mg%operator_key, mg%i_phi, mg%i_tmp)
    nc = box%n_cell
    box%cc(DTIMES(1:nc), mg%i_tmp) = box%cc(DTIMES(1:nc), mg%i_rhs) &
         - box%cc(DTIMES(1:nc), mg%i_tmp)
  end subroutine residual_box

  subroutine residual_tree()
    integer :: lvl, i
    do lvl = 1, tree%highest_lvl
       !$omp parallel do
       do i = 1, size(tree%lvls(lvl)%ids)
          call residual_box(tree%boxes(tree%lvls(lvl)%ids(i)))
       end do
       !$omp end parallel do
    end do
  end subroutine residual_tree

  !> update_coarse (m_af_multigrid.f90:691-738)
  subroutine update_coarse(lvl)
    integer, intent(in)   :: lvl
    integer               :: i, id, p_id, nc
    real(dp), allocatable :: tmp(DTIMES(:))
    nc = tree%n_cell
    !$omp parallel private(i, id, p_id, tmp)
    allocate(tmp(DTIMES(1:nc)))
    !$omp do
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
    !$omp end do
    !$omp end parallel
    call af_gc_lvl(tree, lvl-1, [mg%i_phi])
    !$omp parallel do private(id)
    do i = 1, size(tree%lvls(lvl-1)%parents)
       id = tree%lvls(lvl-1)%parents(i)
       call af_stencil_apply_box(tree%boxes(id), mg%operator_key, mg%i_phi, mg%i_rhs)
       call af_box_add_cc(tree%boxes(id), mg%i_tmp, mg%i_rhs)
       call af_box_copy_cc(tree%boxes(id), mg%i_phi, mg%i_tmp)
    end do
    !$omp end parallel do
  end subroutine update_coarse

  !> correct_children (m_af_multigrid.f90:624-646)
  subroutine correct_children(plvl)
    integer, intent(in) :: plvl
    integer             :: i, id, i_c, c_id
    !$omp parallel do private(id, i_c, c_id)
    do i = 1, size(tree%lvls(plvl)%parents)
       id = tree%lvls(plvl)%parents(i)
       tree%boxes(id)%cc(DTIMES(:), mg%i_tmp) = tree%boxes(id)%cc(DTIMES(:), mg%i_phi) - &
            tree%boxes(id)%cc(DTIMES(:), mg%i_tmp)
       do i_c = 1, af_num_children
          c_id = tree%boxes(id)%children(i_c)
          if (c_id == af_no_box) cycle
          call af_stencil_prolong_box(tree%boxes(id), tree%boxes(c_id), &
               mg%prolongation_key, mg%i_tmp, mg%i_phi, .true.)
       end do
    end do
    !$omp end parallel do
  end subroutine correct_children

end program ref_timing
