!> ORACLE TEST INFRASTRUCTURE (build container only).
!>
!> dat_roundtrip: the reference's own af_read_tree followed by af_write_tree
!> (afivo/src/m_af_output.f90:41-374) on a .dat file written by
!> afivo-streamer_amd/afh/datfile.py, so the test can require the two files
!> to be byte-identical (the format is then the reference's in both
!> directions). The data after the tree (the streamer's write_sim_data
!> record) is carried through unchanged by the read/write callbacks.
!>
!> Usage: dat_roundtrip <in.dat> <out> <1|0: other data present>
!>        (writes <out>.dat)
program dat_roundtrip
  use m_af_all
  implicit none
  type(af_t)              :: tree
  character(len=512)      :: fin, fout, flag
  integer(1), allocatable :: other(:)
  logical                 :: have_other

  call get_command_argument(1, fin)
  call get_command_argument(2, fout)
  call get_command_argument(3, flag)
  have_other = .false.
  if (trim(flag) == "1") then
     call af_read_tree(tree, trim(fin), read_other)
  else
     call af_read_tree(tree, trim(fin))
  end if
  if (have_other) then
     call af_write_tree(tree, trim(fout), write_other)
  else
     call af_write_tree(tree, trim(fout))
  end if

contains

  subroutine read_other(my_unit)
    integer, intent(in) :: my_unit
    integer             :: p, sz
    inquire(unit=my_unit, pos=p, size=sz)
    allocate(other(sz - p + 1))
    if (size(other) > 0) read(my_unit) other
    have_other = .true.
  end subroutine read_other

  subroutine write_other(my_unit)
    integer, intent(in) :: my_unit
    if (size(other) > 0) write(my_unit) other
  end subroutine write_other

end program dat_roundtrip
