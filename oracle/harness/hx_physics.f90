!> ORACLE TEST INFRASTRUCTURE -- golden-vector harness, physics callbacks.
!>
!> This module is NOT part of the product. It is compiled only in the build
!> container, linked against afivo modules compiled from the reference sources
!> (/root/reference/afivo/src, see oracle/Makefile), and used to generate the
!> fixtures in tests/golden/.
!>
!> The golden-vector harnesses (golden_gen.f90, golden_gen2d.f90) link only the
!> afivo numerics compiled from the reference, not the streamer modules: they
!> re-sequence mg_fas_vcycle around a level-1 solve of their own, because the
!> reference's solve_coarse_grid calls HYPRE, which is absent. The physics
!> callbacks below are restatements of the reference callbacks for that
!> harness, restricted to the branches the hot path takes in configs 1-3 (LFA
!> model, constant gas density, no energy equation, no dielectric, no photoi,
!> no ion mobility, old-style transport data), each citing the lines it
!> follows. (The streamer modules themselves DO compile here since round 2 --
!> oracle/Makefile _ref/full and _ref/full2d, with silo_f9x.inc taken from the
!> bundled Silo tarball -- and pin these restatements: replay_step runs the
!> reference's own forward_euler on recorded states, tests/
!> test_reference_replay.py and tests/test_2d_replay.py.)
module hx_physics
#include "cpp_macros.h"
  use m_af_types
  use m_lookup_table
  use m_units_constants

  implicit none
  public

  ! Variable layout mirrors chemistry_initialize + ST_initialize ordering
  ! (src/m_chemistry.f90:262-270, src/m_streamer.f90:237-302):
  ! species e, M+, M- with 3 copies each (Heun needs num_steps+1 = 3).
  integer, parameter :: i_e = 1, i_pos = 4, i_neg = 7
  integer, parameter :: i_phi = 10, i_efld = 12, i_rhs = 13, i_tmp = 14
  integer, parameter :: n_cc_vars = 14
  integer, parameter :: f_flux = 1, f_field = 2

  ! src/m_gas.f90:39
  real(dp), parameter :: SI_to_Townsend = 1e21_dp
  real(dp), parameter :: Townsend_to_SI = 1e-21_dp

  real(dp) :: gas_number_density, gas_inverse_number_density
  real(dp) :: current_voltage = 0.0_dp

  ! src/m_transport_data.f90:10-13
  integer, parameter :: td_mobility = 1, td_diffusion = 2
  integer, parameter :: td_alpha = 3, td_eta = 4
  type(LT_t) :: td_tbl
  type(LT_t) :: chemtbl_fld

  ! Standard 2-reaction model, src/m_chemistry.f90:205-239
  integer, parameter :: n_species = 3, n_reactions = 2
  ! Species charges: e -1, M+ +1, M- -1
  integer, parameter :: species_charge(3) = [-1, 1, -1]
  integer, parameter :: species_itree(3) = [i_e, i_pos, i_neg]

  logical :: last_step = .false.

contains

  !> Gas number density from the ideal gas law, src/m_gas.f90:174-176
  subroutine hx_init_gas(pressure_bar, temperature)
    real(dp), intent(in) :: pressure_bar, temperature
    gas_number_density = 1e5_dp * pressure_bar / &
         (UC_boltzmann_const * temperature)
    gas_inverse_number_density = 1/gas_number_density
  end subroutine hx_init_gas

  !> Old-style transport table, src/m_transport_data.f90:68-107, using the
  !> reference's own table_from_file / LT_create / table_set_column. Then the
  !> chemistry field table, src/m_chemistry.f90:205-239 + 326-358.
  subroutine hx_init_transport(td_file)
    use m_config
    use m_table_data
    character(len=*), intent(in) :: td_file
    type(CFG_t)                  :: cfg
    real(dp), allocatable        :: xx(:), yy(:), x_data(:), y1(:), y2(:)
    real(dp)                     :: max_Td

    call table_data_initialize(cfg)

    call table_from_file(td_file, "efield[V/m]_vs_mu[m2/Vs]", xx, yy)
    xx = xx * SI_to_Townsend / gas_number_density
    yy = yy * gas_number_density
    max_Td = xx(size(xx))
    td_tbl = LT_create(table_min_townsend, max_Td, table_size, &
         4, table_xspacing)
    call table_set_column(td_tbl, td_mobility, xx, yy)

    call table_from_file(td_file, "efield[V/m]_vs_dif[m2/s]", xx, yy)
    xx = xx * SI_to_Townsend / gas_number_density
    yy = yy * gas_number_density
    call table_set_column(td_tbl, td_diffusion, xx, yy)

    call table_from_file(td_file, "efield[V/m]_vs_alpha[1/m]", xx, yy)
    xx = xx * SI_to_Townsend / gas_number_density
    yy = yy / gas_number_density
    call table_set_column(td_tbl, td_alpha, xx, yy)

    call table_from_file(td_file, "efield[V/m]_vs_eta[1/m]", xx, yy)
    xx = xx * SI_to_Townsend / gas_number_density
    yy = yy / gas_number_density
    call table_set_column(td_tbl, td_eta, xx, yy)

    ! m_chemistry.f90:214-233: y_data = alpha * mu * x * Td_to_SI * N
    x_data = td_tbl%x
    y1 = td_tbl%rows_cols(:, td_alpha) * td_tbl%rows_cols(:, td_mobility) * &
         x_data * Townsend_to_SI * gas_number_density
    y2 = td_tbl%rows_cols(:, td_eta) * td_tbl%rows_cols(:, td_mobility) * &
         x_data * Townsend_to_SI * gas_number_density

    ! m_chemistry.f90:330-331, 351-354
    chemtbl_fld = LT_create(td_tbl%x(1), td_tbl%x(td_tbl%n_points), &
         table_size, 2, table_xspacing)
    call table_set_column(chemtbl_fld, 1, x_data, y1)
    call table_set_column(chemtbl_fld, 2, x_data, y2)
  end subroutine hx_init_transport

  !> Load td_tbl and chemtbl_fld from a tables.bin fixture (the layout
  !> golden_gen's dump_tables writes: per table n_points, n_cols, x_min,
  !> inv_fac, rows_cols), instead of rebuilding them from the transport-data
  !> file with hx_init_transport.
  subroutine hx_load_tables(path)
    character(len=*), intent(in) :: path
    integer                      :: u
    open(newunit=u, file=path, access="stream", form="unformatted", &
         status="old", action="read")
    call read_lt(u, td_tbl)
    call read_lt(u, chemtbl_fld)
    close(u)
  contains
    subroutine read_lt(u, lt)
      integer, intent(in)       :: u
      type(LT_t), intent(inout) :: lt
      integer(4)                :: np, ncol
      integer                   :: i
      read(u) np, ncol, lt%x_min, lt%inv_fac
      lt%n_points = np
      lt%n_cols = ncol
      lt%xspacing = LT_xspacing_linear
      lt%extrapolate_above = .false.
      if (allocated(lt%rows_cols)) deallocate(lt%rows_cols, lt%cols_rows, lt%x)
      allocate(lt%rows_cols(np, ncol), lt%cols_rows(ncol, np), lt%x(np))
      read(u) lt%rows_cols
      lt%cols_rows = transpose(lt%rows_cols)
      lt%x = [(lt%x_min + (i - 1) / lt%inv_fac, i = 1, np)]
    end subroutine read_lt
  end subroutine hx_load_tables

  !> field_bc_homogeneous, src/m_field.f90:547-567
  subroutine hx_bc_phi(box, nb, iv, coords, bc_val, bc_type)
    type(box_t), intent(in) :: box
    integer, intent(in)     :: nb
    integer, intent(in)     :: iv
    real(dp), intent(in)    :: coords(NDIM, box%n_cell**(NDIM-1))
    real(dp), intent(out)   :: bc_val(box%n_cell**(NDIM-1))
    integer, intent(out)    :: bc_type

    if (af_neighb_dim(nb) == NDIM) then
       if (af_neighb_low(nb)) then
          bc_type = af_bc_dirichlet
          bc_val = 0.0_dp
       else
          bc_type = af_bc_dirichlet
          bc_val  = current_voltage
       end if
    else
       bc_type = af_bc_neumann
       bc_val = 0.0_dp
    end if
  end subroutine hx_bc_phi

  !> mg_auto_rb for a normal box (afivo/src/m_af_multigrid.f90:926-940)
  subroutine hx_rb_phi(boxes, id, nb, iv, op_mask)
    use m_af_multigrid, only: mg_sides_rb
    type(box_t), intent(inout) :: boxes(:)
    integer, intent(in)        :: id, nb, iv, op_mask
    call mg_sides_rb(boxes, id, nb, iv)
  end subroutine hx_rb_phi

  !> field_set_rhs, src/m_field.f90:363-401 (leaves, including ghost cells)
  subroutine hx_field_set_rhs(tree, s_in)
    type(af_t), intent(inout) :: tree
    integer, intent(in)       :: s_in
    real(dp), parameter       :: fac = -UC_elem_charge / UC_eps0
    real(dp)                  :: q
    integer                   :: lvl, i, id, n, ix

    do lvl = 1, tree%highest_lvl
       do i = 1, size(tree%lvls(lvl)%leaves)
          id = tree%lvls(lvl)%leaves(i)
          tree%boxes(id)%cc(DTIMES(:), i_rhs) = 0.0_dp
          do n = 1, n_species
             if (species_charge(n) == 0) cycle
             ix = species_itree(n) + s_in
             q = species_charge(n) * fac
             tree%boxes(id)%cc(DTIMES(:), i_rhs) = &
                  tree%boxes(id)%cc(DTIMES(:), i_rhs) + &
                  q * tree%boxes(id)%cc(DTIMES(:), ix)
          end do
       end do
    end do
  end subroutine hx_field_set_rhs

  !> flux_upwind, src/m_fluid.f90:102-209 (constant N, LFA, no ions)
  subroutine hx_flux_upwind(nf, n_var, flux_dim, u, flux, cfl_sum, &
       n_other_dt, other_dt, box, line_ix, s_deriv)
    use m_af_flux_schemes
    integer, intent(in)     :: nf, n_var, flux_dim
    real(dp), intent(in)    :: u(nf, n_var)
    real(dp), intent(out)   :: flux(nf, n_var)
    real(dp), intent(out)   :: cfl_sum(nf-1)
    integer, intent(in)     :: n_other_dt
    real(dp), intent(inout) :: other_dt(n_other_dt)
    type(box_t), intent(in) :: box
    integer, intent(in)     :: line_ix(NDIM-1)
    integer, intent(in)     :: s_deriv
    real(dp) :: E_cc(0:nf), E_x(nf), ne_cc(0:nf), v(nf), dc(nf)
    real(dp) :: tmp_fc(nf), N_inv(nf), mu(nf), sigma(nf), inv_dx, cfl_factor
    integer  :: nc

    nc = box%n_cell
    inv_dx = 1/box%dr(flux_dim)
    N_inv = 1/gas_number_density

    call flux_get_line_1fc(box, f_field, flux_dim, line_ix, E_x)
    call flux_get_line_1cc(box, i_e+s_deriv, flux_dim, line_ix, ne_cc)
    call flux_get_line_1cc(box, i_efld, flux_dim, line_ix, E_cc)

    tmp_fc = 0.5_dp * (E_cc(0:nc) + E_cc(1:nc+1)) * SI_to_Townsend * N_inv
    mu = LT_get_col(td_tbl, td_mobility, tmp_fc) * N_inv
    dc = LT_get_col(td_tbl, td_diffusion, tmp_fc) * N_inv

    v = -mu * E_x
    flux(:, 1) = v * u(:, 1) - dc * inv_dx * (ne_cc(1:nc+1) - ne_cc(0:nc))
    sigma = mu * u(:, 1)
    cfl_factor = 1.0_dp
    cfl_sum = cfl_factor * max(abs(v(2:)), abs(v(:nf-1))) * inv_dx + &
         2 * max(dc(2:), dc(:nf-1))  * inv_dx**2
    other_dt(1) = UC_eps0 / (UC_elem_charge * max(maxval(sigma), 1e-100_dp))
  end subroutine hx_flux_upwind

  !> flux_direction, src/m_fluid.f90:212-227 (electrons: charge sign -1)
  subroutine hx_flux_direction(box, line_ix, s_deriv, n_var, flux_dim, &
       direction_positive)
    use m_af_flux_schemes
    type(box_t), intent(in) :: box
    integer, intent(in)     :: line_ix(NDIM-1)
    integer, intent(in)     :: s_deriv, flux_dim, n_var
    logical, intent(out)    :: direction_positive(box%n_cell+1, n_var)
    real(dp)                :: E_x(box%n_cell+1)
    integer                 :: n

    call flux_get_line_1fc(box, f_field, flux_dim, line_ix, E_x)
    do n = 1, n_var
       direction_positive(:, n) = (-1 * E_x > 0)
    end do
  end subroutine hx_flux_direction

  !> set_box_mask, src/m_fluid.f90:469-515 (no electrode/dielectric/region)
  subroutine hx_set_box_mask(box, mask)
    type(box_t), intent(in) :: box
    logical, intent(out)    :: mask(DTIMES(box%n_cell))
    mask = .true.
  end subroutine hx_set_box_mask

  !> add_source_terms, src/m_fluid.f90:298-466 with get_rates /
  !> get_derivatives (src/m_chemistry.f90:565-688) for the 2-reaction model.
  subroutine hx_add_source_terms(box, dt, n_vars, i_cc, s_deriv, s_out, &
       n_dt, dt_lim, mask)
    type(box_t), intent(inout) :: box
    real(dp), intent(in)       :: dt
    integer, intent(in)        :: n_vars
    integer, intent(in)        :: i_cc(n_vars)
    integer, intent(in)        :: s_deriv, s_out, n_dt
    real(dp), intent(inout)    :: dt_lim(n_dt)
    logical, intent(in)        :: mask(DTIMES(box%n_cell))
    real(dp) :: tmp
    real(dp) :: rates(box%n_cell**NDIM, n_reactions)
    real(dp) :: derivs(box%n_cell**NDIM, n_species)
    real(dp) :: dens(box%n_cell**NDIM, n_species)
    real(dp) :: fields(box%n_cell**NDIM)
    integer  :: IJK, ix, nc, n_cells, n, iv
    real(dp), parameter :: eps = 1e-100_dp

    nc      = box%n_cell
    n_cells = box%n_cell**NDIM
    if (.not. any(mask)) return

    tmp = 1 / gas_number_density
    fields = SI_to_Townsend * tmp * &
         pack(box%cc(DTIMES(1:nc), i_efld), .true.)

    dens(:, 1:n_species) = reshape(box%cc(DTIMES(1:nc), &
         species_itree(1:n_species)+s_deriv), [n_cells, n_species])
    dens = max(dens, 0.0_dp)

    ! get_rates: rate_tabulated_field with rate_factor 1
    rates(:, 1) = 1.0_dp * LT_get_col(chemtbl_fld, 1, fields)
    rates(:, 2) = 1.0_dp * LT_get_col(chemtbl_fld, 2, fields)

    ! get_derivatives
    derivs(:, :) = 0.0_dp
    ! e + M -> e + e + M+
    rates(:, 1) = rates(:, 1) * dens(:, 1)
    derivs(:, 1) = derivs(:, 1) - rates(:, 1)
    derivs(:, 1) = derivs(:, 1) + rates(:, 1) * 2
    derivs(:, 2) = derivs(:, 2) + rates(:, 1) * 1
    ! e + M -> M-
    rates(:, 2) = rates(:, 2) * dens(:, 1)
    derivs(:, 1) = derivs(:, 1) - rates(:, 2)
    derivs(:, 3) = derivs(:, 3) + rates(:, 2) * 1

    if (last_step) then
       ! m_fluid.f90:402-413 with the m_dt defaults dt_chemistry_nmin = -1,
       ! dt_chemistry_limit_loss = .true. (src/m_dt.f90:34-37)
       tmp = minval(max(dens, eps) / max(-derivs, eps))
       dt_lim(1) = tmp
    end if

    do n = 1, n_species
       ix = 0
       iv = species_itree(n)
       do KJI_DO(1,nc)
          ix = ix + 1
          if (.not. mask(IJK)) cycle
          box%cc(IJK, iv+s_out) = box%cc(IJK, iv+s_out) + dt * derivs(ix, n)
       end do; CLOSE_DO
    end do
  end subroutine hx_add_source_terms

end module hx_physics
