!> Glue between an afivo tree (type af_t, afivo/src/m_af_types.f90:326-393)
!> and libafivo_hip: packs the topology into afh_tree_desc and moves
!> tree%boxes(:)%cc / %fc variables to and from the device pool.
!>
!> Compiled inside an afivo-streamer build (it uses m_af_types); see
!> INTEGRATION.md for where the calls go in the streamer driver.
module m_afivo_hip_tree
  use iso_c_binding
  use m_af_types
  use m_afivo_hip
  implicit none
  private

  !> Host arrays a descriptor points into; keep it alive while the descriptor
  !> is used (afh_tree_create copies everything it needs).
  type, public :: afh_tree_store_t
     type(afh_tree_desc)             :: desc
     type(afh_box_meta), allocatable :: meta(:)
     integer(c_int32_t), allocatable :: ids(:), ids_off(:)
     integer(c_int32_t), allocatable :: leaves(:), leaves_off(:)
     integer(c_int32_t), allocatable :: parents(:), parents_off(:)
  end type afh_tree_store_t

  public :: afh_tree_from_af
  public :: afh_put_cc_tree, afh_get_cc_tree
  public :: afh_put_fc_tree, afh_get_fc_tree
  public :: afh_bc_from_type
  public :: afh_mg_stencils_from_af

contains

  !> Hand the electrode stencils mg_set_operators_tree stored on the boxes
  !> (m_af_multigrid.f90:1133-1171) to the device multigrid `mg_h`: per box
  !> the variable operator stencil of mg%operator_key with its bc_correction,
  !> and the boundary distances (mg_lsf_distance_key) with
  !> mg_lsf_boundary_value for the gradient. Call after every operator
  !> (re)build (mg_init / mg_use / regrid) and when the electrode voltage
  !> changes.
  subroutine afh_mg_stencils_from_af(mg_h, tree, mg)
    use m_af_stencil, only: af_stencil_index, stencil_variable
    use m_coarse_solver, only: mg_lsf_boundary_value
    type(c_ptr), intent(in)   :: mg_h
    type(af_t), intent(in), target :: tree
    type(mg_t), intent(in)    :: mg
    integer                   :: id, ix, n
    real(c_double), allocatable, target :: bval(:, :, :)
    type(c_ptr)               :: vp, bp
    do id = 1, tree%highest_id
       if (.not. tree%boxes(id)%in_use) cycle
       associate (box => tree%boxes(id))
         vp = c_null_ptr
         bp = c_null_ptr
         ix = af_stencil_index(box, mg%operator_key)
         if (ix > af_stencil_none) then
            if (box%stencils(ix)%stype == stencil_variable) then
               vp = c_loc(tree%boxes(id)%stencils(ix)%v)
               if (allocated(box%stencils(ix)%bc_correction)) &
                    bp = c_loc(tree%boxes(id)%stencils(ix)%bc_correction)
            end if
         end if
         call afh_check(afh_mg_set_box_stencil(mg_h, int(id, c_int32_t), vp, bp), &
              "mg_set_box_stencil")
         n = 0
         ix = af_stencil_index(box, mg_lsf_distance_key)
         if (ix > af_stencil_none) n = size(box%stencils(ix)%sparse_ix, 2)
         if (n > 0) then
            bval = mg_lsf_boundary_value(box, mg)
            call afh_check(afh_mg_set_box_lsf(mg_h, int(id, c_int32_t), &
                 int(n, c_int32_t), int(box%stencils(ix)%sparse_ix, c_int32_t), &
                 box%stencils(ix)%sparse_v, bval, int(mg%i_lsf, c_int32_t)), &
                 "mg_set_box_lsf")
         else
            call afh_check(afh_mg_set_box_lsf(mg_h, int(id, c_int32_t), 0_c_int32_t, &
                 [0_c_int32_t], [0.0_c_double], [0.0_c_double], 0_c_int32_t), &
                 "mg_set_box_lsf")
         end if
       end associate
    end do
  end subroutine afh_mg_stencils_from_af

  !> Pack tree%boxes(1:highest_id) and tree%lvls(1:highest_lvl) into st%desc.
  subroutine afh_tree_from_af(tree, st)
    type(af_t), intent(in)                      :: tree
    type(afh_tree_store_t), intent(inout), target :: st
    integer :: id, l, nl, nb

    nb = tree%highest_id
    nl = tree%highest_lvl
    if (allocated(st%meta)) deallocate(st%meta, st%ids, st%ids_off, &
         st%leaves, st%leaves_off, st%parents, st%parents_off)
    allocate(st%meta(max(nb, 1)))

    do id = 1, nb
       st%meta(id) = afh_box_meta(0, 0, 0, 0, 0, 0, 0.0_c_double, 0.0_c_double)
       if (tree%boxes(id)%in_use) st%meta(id) = box_meta(tree%boxes(id))
    end do

    allocate(st%ids_off(nl+1), st%leaves_off(nl+1), st%parents_off(nl+1))
    st%ids_off(1) = 0
    st%leaves_off(1) = 0
    st%parents_off(1) = 0
    do l = 1, nl
       st%ids_off(l+1) = st%ids_off(l) + size(tree%lvls(l)%ids)
       st%leaves_off(l+1) = st%leaves_off(l) + size(tree%lvls(l)%leaves)
       st%parents_off(l+1) = st%parents_off(l) + size(tree%lvls(l)%parents)
    end do
    allocate(st%ids(max(st%ids_off(nl+1), 1)))
    allocate(st%leaves(max(st%leaves_off(nl+1), 1)))
    allocate(st%parents(max(st%parents_off(nl+1), 1)))
    do l = 1, nl
       st%ids(st%ids_off(l)+1:st%ids_off(l+1)) = tree%lvls(l)%ids
       st%leaves(st%leaves_off(l)+1:st%leaves_off(l+1)) = tree%lvls(l)%leaves
       st%parents(st%parents_off(l)+1:st%parents_off(l+1)) = tree%lvls(l)%parents
    end do

    st%desc%n_cell = tree%n_cell
    st%desc%n_boxes = nb
    st%desc%highest_lvl = nl
    st%desc%n_var_cell = tree%n_var_cell
    st%desc%n_var_face = tree%n_var_face
    st%desc%coarse_grid_size = tree%coarse_grid_size
    st%desc%periodic = merge(1, 0, tree%periodic)
    st%desc%r_base = tree%r_base
    st%desc%dr_base = tree%dr_base
    st%desc%boxes = c_loc(st%meta)
    st%desc%lvl_ids = c_loc(st%ids)
    st%desc%lvl_ids_off = c_loc(st%ids_off)
    st%desc%lvl_leaves = c_loc(st%leaves)
    st%desc%lvl_leaves_off = c_loc(st%leaves_off)
    st%desc%lvl_parents = c_loc(st%parents)
    st%desc%lvl_parents_off = c_loc(st%parents_off)
  end subroutine afh_tree_from_af

  !> The box_t fields the device reads (m_af_types.f90:286-322)
  function box_meta(b) result(m)
    type(box_t), intent(in) :: b
    type(afh_box_meta)      :: m
    integer                 :: dx, dy, dz
    m%lvl = b%lvl
    m%ix = b%ix
    m%parent = b%parent
    m%children = b%children
    m%neighbors = b%neighbors
    ! element by element: reshape() of this (-1:1)^3 component returned zeros
    ! with amdflang -O2
    do dz = -1, 1
       do dy = -1, 1
          do dx = -1, 1
             m%neighbor_mat(1 + (dx+1) + 3*(dy+1) + 9*(dz+1)) = &
                  b%neighbor_mat(dx, dy, dz)
          end do
       end do
    end do
    m%r_min = b%r_min
    m%dr = b%dr
  end function box_meta

  !> tree%boxes(:)%cc(..., iv) -> device (boxes in id order)
  subroutine afh_put_cc_tree(t, tree, iv)
    type(c_ptr), intent(in) :: t
    type(af_t), intent(in)  :: tree
    integer, intent(in)     :: iv
    real(c_double), allocatable :: buf(:, :, :, :)
    integer :: id, ng
    ng = tree%n_cell + 2
    allocate(buf(ng, ng, ng, tree%highest_id))
    buf = 0
    do id = 1, tree%highest_id
       if (tree%boxes(id)%in_use) buf(:, :, :, id) = tree%boxes(id)%cc(:, :, :, iv)
    end do
    call afh_check(afh_cc_put(t, int(iv, c_int32_t), buf), "cc_put")
  end subroutine afh_put_cc_tree

  !> device -> tree%boxes(:)%cc(..., iv)
  subroutine afh_get_cc_tree(t, tree, iv)
    type(c_ptr), intent(in)  :: t
    type(af_t), intent(inout) :: tree
    integer, intent(in)      :: iv
    real(c_double), allocatable :: buf(:, :, :, :)
    integer :: id, ng
    ng = tree%n_cell + 2
    allocate(buf(ng, ng, ng, tree%highest_id))
    call afh_check(afh_cc_get(t, int(iv, c_int32_t), buf), "cc_get")
    do id = 1, tree%highest_id
       if (tree%boxes(id)%in_use) tree%boxes(id)%cc(:, :, :, iv) = buf(:, :, :, id)
    end do
  end subroutine afh_get_cc_tree

  !> tree%boxes(:)%fc(..., ivf) -> device
  subroutine afh_put_fc_tree(t, tree, ivf)
    type(c_ptr), intent(in) :: t
    type(af_t), intent(in)  :: tree
    integer, intent(in)     :: ivf
    real(c_double), allocatable :: buf(:, :, :, :, :)
    integer :: id, nf
    nf = tree%n_cell + 1
    allocate(buf(nf, nf, nf, 3, tree%highest_id))
    buf = 0
    do id = 1, tree%highest_id
       if (tree%boxes(id)%in_use) buf(:, :, :, :, id) = tree%boxes(id)%fc(:, :, :, :, ivf)
    end do
    call afh_check(afh_fc_put(t, int(ivf, c_int32_t), buf), "fc_put")
  end subroutine afh_put_fc_tree

  !> device -> tree%boxes(:)%fc(..., ivf)
  subroutine afh_get_fc_tree(t, tree, ivf)
    type(c_ptr), intent(in)  :: t
    type(af_t), intent(inout) :: tree
    integer, intent(in)      :: ivf
    real(c_double), allocatable :: buf(:, :, :, :, :)
    integer :: id, nf
    nf = tree%n_cell + 1
    allocate(buf(nf, nf, nf, 3, tree%highest_id))
    call afh_check(afh_fc_get(t, int(ivf, c_int32_t), buf), "fc_get")
    do id = 1, tree%highest_id
       if (tree%boxes(id)%in_use) tree%boxes(id)%fc(:, :, :, :, ivf) = buf(:, :, :, :, id)
    end do
  end subroutine afh_get_fc_tree

  !> afivo boundary-condition type (af_bc_dirichlet, ..., m_af_types.f90:51-64)
  !> and a face-uniform value -> afh_bc
  function afh_bc_from_type(bc_type, bc_value) result(bc)
    integer, intent(in)  :: bc_type
    real(dp), intent(in) :: bc_value
    type(afh_bc)         :: bc
    select case (bc_type)
    case (af_bc_dirichlet)
       bc%type = AFH_BC_DIRICHLET
    case (af_bc_neumann)
       bc%type = AFH_BC_NEUMANN
    case (af_bc_continuous)
       bc%type = AFH_BC_CONTINUOUS
    case (af_bc_dirichlet_copy)
       bc%type = AFH_BC_DIRICHLET_COPY
    case default
       error stop "afh_bc_from_type: unknown boundary condition type"
    end select
    bc%value = bc_value
  end function afh_bc_from_type

end module m_afivo_hip_tree
