!> ORACLE TEST INFRASTRUCTURE (build container only).
!>
!> replay_step: one forward-Euler species step of the reference's own fluid
!> model (forward_euler, src/m_fluid.f90:21-99: flux_upwind_tree with its
!> flux_upwind / flux_direction callbacks, flux_update_densities with
!> add_source_terms, get_rates, get_derivatives, photoionization source) on a
!> tree state recorded from the device driver (afh.driver), to compare the
!> two on identical inputs.
!>
!> The modules are set up from the .cfg as the streamer does
!> (initialize_modules, streamer.f90:429-458) and the tree is rebuilt from the
!> recorded topology with afivo's own routines: af_init, then
!> af_adjust_refinement with a routine that refines exactly the boxes the
!> record lists as parents, level by level (box ids therefore follow afivo's
!> allocation order; recorded boxes are matched to the reference boxes by level
!> and index, box%ix). forward_euler is called with
!> i_step = n_steps = 1, so it never reaches field_compute: the field and the
!> state come from the record. The coarse-grid solver (HYPRE, absent from the
!> reference snapshot) is therefore never called; the link leaves its symbols
!> unresolved (--unresolved-symbols=ignore-in-object-files) instead of
!> providing anything in their place.
!>
!> Usage: replay_step <record_file> <out_file> <cfg> [-key=value ...] [--user-gas=sprite]
!> Record (stream, little endian): int32 highest_id, n_var_cell, n_var_face,
!> nc; per id: int32 parent, lvl, ix(3), in_use; float64 dt, time; int32
!> s_deriv, n_prev, s_prev(n_prev); float64 w_prev(n_prev); int32 s_out;
!> then every cc variable of every box in use ((nc+2)^3, i fastest) and every
!> fc variable ((nc+1)^3 x 3).
!> Output: float64 dt_lim, then every cc variable of every box in use.
!> NDIM = 2 (oracle/Makefile _ref/2d/replay_step): the same record with the
!> 2-D box shapes ((nc+2)^2 per cc variable, (nc+1)^2 x 2 per fc variable);
!> ix keeps three entries, the third unused.
#include "cpp_macros.h"
program replay_step
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
  use m_user_methods
  implicit none

  type(CFG_t)        :: cfg
  type(af_t)         :: tree
  type(ref_info_t)   :: ref_info
  character(len=512) :: rec_file, out_file, arg
  integer            :: ur, uo, n, hid, nvc, nvf, nc, id, iv, lvl
  integer            :: s_deriv, n_prev, s_out
  integer, allocatable :: parent(:), blvl(:), bix(:, :), in_use(:), s_prev(:)
  integer, allocatable :: rid(:)
  real(dp), allocatable :: w_prev(:)
  real(dp)           :: dt, time, dt_lim

  call get_command_argument(1, rec_file)
  call get_command_argument(2, out_file)
  do n = 3, command_argument_count()
     call get_command_argument(n, arg)
     if (arg(1:11) == "--user-gas=") then
        ! programs/3d_sprite's user_initialize (m_user.f90:24-30): the gas
        ! density "M" is a cc variable (m_gas.f90:146-148); its values come
        ! from the record
        if (trim(arg(12:)) == "sprite") user_gas_density => sprite_gas_density
     else if (arg(1:1) == '-') then
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
  ! default methods of the densities and output variables (streamer.f90:81-104)
  do n = 1, size(all_densities)
     call af_set_cc_methods(tree, all_densities(n), bc_species, af_gc_interp_lim, &
          ST_prolongation_method)
  end do
  do n = 1, tree%n_var_cell
     if (tree%cc_write_output(n) .and. .not. (tree%has_cc_method(n) .or. n == i_phi)) &
          call af_set_cc_methods(tree, n, af_bc_neumann_zero, af_gc_interp, &
          ST_prolongation_method)
  end do

  open(newunit=ur, file=trim(rec_file), access="stream", form="unformatted", &
       action="read")
  read(ur) hid, nvc, nvf, nc
  if (nvc /= tree%n_var_cell .or. nvf /= tree%n_var_face) &
       error stop "record: variable registry differs"
  allocate(parent(hid), blvl(hid), bix(3, hid), in_use(hid))
  ! (bix(1:NDIM, :) is the box index; a 2-D record leaves bix(3, :) at 0)
  do id = 1, hid
     read(ur) parent(id), blvl(id), bix(:, id), in_use(id)
  end do

  call af_init(tree, ST_box_size, ST_domain_origin + ST_domain_len, &
       ST_coarse_grid_size, periodic=ST_periodic, coord=af_xyz, &
       r_min=ST_domain_origin, mem_limit_gb=8.0_dp)
  do lvl = 1, 29
     call af_adjust_refinement(tree, refine_as_recorded, ref_info)
     if (ref_info%n_add == 0) exit
  end do
  ! recorded box -> reference box with the same level and index
  allocate(rid(hid))
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
  if (count(in_use /= 0) /= count(tree%boxes(1:tree%highest_id)%in_use)) &
       error stop "rebuilt tree has extra boxes"

  read(ur) dt, time, s_deriv, n_prev
  allocate(s_prev(n_prev), w_prev(n_prev))
  read(ur) s_prev, w_prev, s_out
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

  global_time = time
  dt_lim = 1e100_dp
  call forward_euler(tree, dt, dt, dt_lim, time, s_deriv, n_prev, s_prev, &
       w_prev, s_out, 1, 1)

  open(newunit=uo, file=trim(out_file), access="stream", form="unformatted", &
       action="write", status="replace")
  write(uo) dt_lim
  do iv = 1, nvc
     do id = 1, hid
        if (in_use(id) /= 0) write(uo) tree%boxes(rid(id))%cc(DTIMES(:), iv)
     end do
  end do
  close(uo)

contains

  !> gas_density of programs/3d_sprite/m_user.f90:34-40
  pure real(dp) function sprite_gas_density(box, IJK)
    type(box_t), intent(in) :: box
    integer, intent(in)     :: IJK
    real(dp)                :: rr(NDIM)
    rr = af_r_cc(box, [IJK])
    sprite_gas_density = 2.5e25_dp * exp(-rr(NDIM) / 7.2e3_dp)
  end function sprite_gas_density

  !> Refine the boxes the record lists as parents
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

end program replay_step
