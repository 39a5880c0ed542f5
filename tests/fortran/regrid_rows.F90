!> INTEGRATION.md's sharded-regrid snippet as a compilable unit: whole boxes
!> packed into device rows, handed to a peer (the send / receive itself is
!> the driver's: GPU-aware MPI or RCCL) and unpacked into another tree.
!> tests/test_fortran_boundary.py compiles it against m_afivo_hip.
subroutine move_box_rows(gpu, t_old, lids, t_small, lids_small, n, n_var_cell, n_var_face, &
     row_width)
  use iso_c_binding
  use m_afivo_hip
  implicit none
  integer(c_int32_t), intent(in) :: gpu, n, n_var_cell, n_var_face
  type(c_ptr), intent(in)        :: t_old, t_small
  integer(c_int32_t), intent(in) :: lids(n), lids_small(n)
  integer(c_int64_t), intent(in) :: row_width
  type(c_ptr)                    :: buf

  call afh_check(afh_device_alloc(gpu, int(8, c_int64_t) * n * row_width, buf))
  call afh_check(afh_tree_pack_boxes(t_old, lids, n, n_var_cell, n_var_face, buf))
  ! ncclSend(buf, n * row_width, ncclFloat64, peer, comm, stream) ... ncclRecv
  call afh_check(afh_tree_unpack_boxes(t_small, lids_small, n, n_var_cell, n_var_face, buf))
  call afh_check(afh_device_free(buf))
end subroutine move_box_rows
