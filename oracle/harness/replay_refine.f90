!> ORACLE TEST INFRASTRUCTURE (build container only).
!>
!> replay_refine: the reference's own refinement (af_adjust_refinement,
!> afivo/src/m_af_core.f90:697-822, with refine_routine => default_refinement,
!> src/m_refine.f90:198-298) replayed on field data recorded from the device
!> driver (afh.driver.Simulation.record_refinement). The modules are set up
!> from the .cfg as the streamer does (initialize_modules, streamer.f90:429-458),
!> the tree as af_init + af_refine_up_to_lvl (streamer.f90:151, 466-469). For
!> each recorded call the electron density and |E| of every box are loaded into
!> the reference tree (same ids: the two topologies evolve together as long as
!> every call agrees), global_time is set, af_adjust_refinement runs with
!> refine_buffer_width, and the resulting topology is written out.
!> Usage: replay_refine <record_file> <out_file> <cfg> [-key=value ...]
!> Record: int32 n_calls, then per call: int32 n_boxes, float64 global_time,
!> int32 full, then per box id 1..n_boxes: int32 in_use, and (in use) either
!> float64 e(nc^3), E(nc^3), i fastest (full = 0), or every cc variable of
!> the box with its ghost cells, cc(0:nc+1, 0:nc+1, 0:nc+1, n_var_cell)
!> (full = 1: the whole state af_adjust_refinement moves). Output per call:
!> int32 highest_id, highest_lvl, then per id 1..highest_id: in_use, lvl,
!> ix(3), parent, children(8), neighbors(6); after a full call also the
!> auto variables (int32 n, iv(n)), the number of added boxes, and per
!> added box its id and every cc variable with ghost cells (the data
!> auto_prolong / auto_restrict left, m_af_core.f90:825-881).
#include "cpp_macros.h"
program replay_refine
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
  implicit none

  type(CFG_t)        :: cfg
  type(af_t)         :: tree
  type(ref_info_t)   :: ref_info
  character(len=512) :: rec_file, out_file, arg
  integer            :: ur, uo, n_calls, call_ix, nb, id, in_use, nc, lvl, n, full
  integer            :: n_add, i
  real(dp)           :: t_glob
  real(dp), allocatable :: buf(:), fbuf(:, :, :, :)

  call get_command_argument(1, rec_file)
  call get_command_argument(2, out_file)
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
  ! mg_init's methods for phi (m_af_multigrid.f90:61, 102-105; mg_init
  ! itself needs HYPRE): no prolongation argument, so af_prolong_linear and
  ! phi an auto variable; mg_auto_rb (private there) is mg_sides_rb for
  ! boxes without a variable-epsilon tag (926-940), phi_rb below
  if (.not. tree%has_cc_method(mg%i_phi)) &
       call af_set_cc_methods(tree, mg%i_phi, mg%sides_bc, phi_rb)

  call af_init(tree, ST_box_size, ST_domain_origin + ST_domain_len, &
       ST_coarse_grid_size, periodic=ST_periodic, coord=af_xyz, &
       r_min=ST_domain_origin, mem_limit_gb=4.0_dp)
  do lvl = 1, af_max_lvl-1
     if (all(af_lvl_dr(tree, lvl) <= refine_max_dx)) exit
  end do
  call af_refine_up_to_lvl(tree, lvl)

  nc = tree%n_cell
  allocate(buf(nc**3))
  allocate(fbuf(0:nc+1, 0:nc+1, 0:nc+1, tree%n_var_cell))
  open(newunit=ur, file=trim(rec_file), access="stream", form="unformatted", &
       action="read")
  open(newunit=uo, file=trim(out_file), access="stream", form="unformatted", &
       action="write", status="replace")
  read(ur) n_calls
  do call_ix = 1, n_calls
     read(ur) nb, t_glob, full
     global_time = t_glob
     do id = 1, nb
        read(ur) in_use
        if (in_use /= 0 .and. full /= 0) then
           read(ur) fbuf
           if (id <= tree%highest_id) tree%boxes(id)%cc = fbuf
        else if (in_use /= 0) then
           read(ur) buf
           ! a box the reference tree does not have (after a disagreement)
           if (id <= tree%highest_id) &
                tree%boxes(id)%cc(1:nc, 1:nc, 1:nc, i_electron) = reshape(buf, [nc, nc, nc])
           read(ur) buf
           if (id <= tree%highest_id) &
                tree%boxes(id)%cc(1:nc, 1:nc, 1:nc, i_electric_fld) = reshape(buf, [nc, nc, nc])
        end if
     end do
     ! the applied voltage field_compute last set (phi's boundary values)
     call field_set_voltage(tree, global_time)
     call af_adjust_refinement(tree, refine_routine, ref_info, refine_buffer_width)
     write(uo) tree%highest_id, tree%highest_lvl
     do id = 1, tree%highest_id
        associate (b => tree%boxes(id))
          write(uo) merge(1, 0, b%in_use), b%lvl, b%ix, b%parent, b%children, b%neighbors
        end associate
     end do
     if (full /= 0) then
        write(uo) size(tree%cc_auto_vars), tree%cc_auto_vars
        n_add = 0
        do lvl = 1, size(ref_info%lvls)
           n_add = n_add + size(ref_info%lvls(lvl)%add)
        end do
        write(uo) n_add
        do lvl = 1, size(ref_info%lvls)
           do i = 1, size(ref_info%lvls(lvl)%add)
              id = ref_info%lvls(lvl)%add(i)
              write(uo) id, tree%boxes(id)%cc
           end do
        end do
     end if
  end do
  close(ur)
  close(uo)
contains
  subroutine phi_rb(boxes, id, nb, iv, op_mask)
    type(box_t), intent(inout) :: boxes(:)
    integer, intent(in)        :: id, nb, iv, op_mask
    call mg_sides_rb(boxes, id, nb, iv)
  end subroutine phi_rb
end program replay_refine
