#include "cpp_macros.h"
!> ORACLE TEST INFRASTRUCTURE (build container only).
!>
!> export_case: set up the reference's streamer modules from a .cfg file exactly
!> as its driver does (src/streamer.f90:429-458, initialize_modules, in that
!> order; the user, output and dielectric modules are not needed), then write
!> what the device driver needs in plain text, one named array per line
!> ("name n v1 ... vn", reals in ES25.17E3 = exact round trip):
!>   * every configuration value the modules registered (CFG_get on the
!>     keys listed below, defaults included),
!>   * the variable registry the modules created (cc / fc names, indices),
!>   * the transport table td_tbl (m_transport_data.f90:128-163),
!>   * the species and reactions as the chemistry parser left them
!>     (m_chemistry.f90:180-387, 741-1160: rate types, folded rate factors,
!>     coefficients, species indices, multiplicities),
!>   * the field-rate lookup table chemtbl_fld, rebuilt with the reference's own
!>     LT_create / table_set_column from the reactions' x_data / y_data exactly
!>     as chemistry_initialize does (m_chemistry.f90:330-355; the module keeps
!>     it private),
!>   * get_rates (m_chemistry.f90:565-653) of every reaction on a field grid
!>     (a known answer for the device rate forms),
!>   * current_voltage at t = 0 (field_set_voltage, m_field.f90:508-543).
!> Usage (from the directory of the cfg, as run_test.sh runs the streamer):
!>   export_case <out_file> <cfg> [-key=value ...]
program export_case
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
  use m_lookup_table
  use m_user_methods
  implicit none

  type(CFG_t) :: cfg
  type(af_t)  :: tree
  character(len=512) :: out_file
  integer :: u, n, i, n_fld
  type(LT_t) :: chemtbl
  real(dp), allocatable :: flds(:), rates(:, :)
  real(dp) :: out_dt = 1.0e-10_dp
  logical  :: out_rtest = .false.
  character(len=32) :: user_gas = ""

  call get_command_argument(1, out_file)
  ! CFG_update_from_arguments skips nothing: shift the output file away by
  ! reading the remaining arguments ourselves
  call read_cfg_args(cfg)
  ! --user-gas=sprite: programs/3d_sprite's user_initialize sets
  ! user_gas_density (3d_sprite/m_user.f90:24-30), which makes gas_initialize
  ! register the gas density variable "M" (m_gas.f90:146-148)
  if (user_gas == "sprite") user_gas_density => sprite_gas_density

  ! initialize_modules (src/streamer.f90:429-458)
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
  call field_set_voltage(tree, 0.0_dp)

  open(newunit=u, file=trim(out_file), action="write")

  ! configuration values (defaults included)
  call put_r("end_time"); call put_i("box_size"); call put_ia("coarse_grid_size")
  call put_ra("domain_len"); call put_ra("domain_origin")
  call put_r("dt_max"); call put_r("dt_min"); call put_r("dt_safety_factor")
  call put_r("dt_cfl_number"); call put_r("dt_chemistry_nmin")
  call put_l("dt_chemistry_limit_loss"); call put_r("dt_max_growth_factor")
  call put_s("time_integrator")
  call put_i("multigrid_num_vcycles"); call put_r("multigrid_max_rel_residual")
  call put_i("refine_buffer_width"); call put_i("refine_per_steps")
  call put_r("refine_min_dx"); call put_r("refine_max_dx"); call put_r("refine_adx")
  call put_r("derefine_dx"); call put_r("refine_init_time"); call put_r("refine_init_fac")
  call put_r("refine_electrode_dx"); call put_r("refine_adx_fac")
  call put_r("refine_min_dens"); call put_l("refine_use_alpha_effective")
  call put_ra("refine_regions_dr"); call put_ra("refine_regions_tstop")
  call put_ra("refine_regions_rmin"); call put_ra("refine_regions_rmax")
  call put_ra("refine_limits_dr"); call put_ra("refine_limits_rmin")
  call put_ra("refine_limits_rmax")
  ! m_output is not initialized (it writes files); its two keys with the
  ! defaults of m_output.f90:22, 25
  call CFG_add_get(cfg, "output%dt", out_dt, "output time step")
  call CFG_add_get(cfg, "output%regression_test", out_rtest, "regression log")
  call put_r("output%dt"); call put_l("output%regression_test")
  call put_l("photoi%enabled"); call put_i("photoi%per_steps"); call put_r("photoi%eta")
  call put_r("photoi%quenching_pressure"); call put_s("photoi%method")
  call put_s("photoi%source_type"); call put_s("photoi%species")
  call put_s("photoi_helmh%author"); call put_r("photoi_helmh%max_rel_residual")
  call put_r("gas%pressure"); call put_r("gas%temperature")
  call put_r("background_density"); call put_r("stochastic_density")
  call put_ra("seed_density"); call put_ra("seed_density2"); call put_ra("seed_rel_r0")
  call put_ra("seed_rel_r1"); call put_ia("seed_charge_type"); call put_ra("seed_width")
  call put_sa("seed_falloff")
  call put_s("field_given_by"); call put_s("field_bc_type")
  call put_l("use_electrode"); call put_l("use_dielectric"); call put_l("cylindrical")
  call put_s("prolong_density"); call put_s("species_boundary_condition")
  call put_l("input_data%old_style")
  ! electrode (m_field.f90:196-230; relative coordinates, as in the cfg)
  call put_s("field_electrode_type"); call put_l("field_electrode_grounded")
  call put_ra("field_rod_r0"); call put_ra("field_rod_r1"); call put_r("field_rod_radius")

  ! derived module state
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:dt_cfl_number_value", 1, dt_cfl_number
  write(u, "(A,1X,I0,*(1X,I0))") "i:coarse_grid_size_value", NDIM, ST_coarse_grid_size
  write(u, "(A,1X,I0,*(1X,I0))") "i:time_integrator_value", 1, time_integrator
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:current_voltage", 1, current_voltage
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:gas_number_density", 1, gas_number_density
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:gas_temperature_value", 1, gas_temperature
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:gas_pressure_value", 1, gas_pressure
  call put_lv("gas_constant_density", gas_constant_density)
  if (allocated(gas_fractions)) then
     write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:gas_fractions", size(gas_fractions), gas_fractions
     write(u, "(A,1X,I0,*(1X,A))") "s:gas_components", size(gas_components), &
          (trim(gas_components(i)), i = 1, size(gas_components))
  end if
  call put_lv("td_old_style", td_old_style)
  write(u, "(A,1X,I0,*(1X,I0))") "i:td_cols", 5, td_mobility, td_diffusion, &
       td_alpha, td_eta, td_energy_eV
  write(u, "(A,1X,I0,*(1X,I0))") "i:n_mobile_ions", 1, transport_data_ions%n_mobile_ions
  ! flux species (m_streamer.f90:253-282): the electrons, then the mobile
  ! ions with their scaled mobilities (m_transport_data.f90:195-215)
  write(u, "(A,1X,I0,*(1X,I0))") "i:flux_species", flux_num_species, flux_species
  write(u, "(A,1X,I0,*(1X,I0))") "i:flux_variables", flux_num_species, flux_variables
  write(u, "(A,1X,I0,*(1X,I0))") "i:flux_species_charge_sign", flux_num_species, &
       flux_species_charge_sign
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:ion_mobilities", &
       transport_data_ions%n_mobile_ions, transport_data_ions%mobilities
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:ion_se_yield", 1, ion_se_yield

  ! variable registry (af_add_cc_variable order)
  write(u, "(A,1X,I0,*(1X,A))") "s:cc_names", tree%n_var_cell, &
       (trim(tree%cc_names(i)), i = 1, tree%n_var_cell)
  write(u, "(A,1X,I0,*(1X,I0))") "i:cc_num_copies", tree%n_var_cell, &
       tree%cc_num_copies(1:tree%n_var_cell)
  write(u, "(A,1X,I0,*(1X,A))") "s:fc_names", tree%n_var_face, &
       (trim(tree%fc_names(i)), i = 1, tree%n_var_face)
  write(u, "(A,1X,I0,*(1X,I0))") "i:ivars", 10, i_phi, i_electron, i_1pos_ion, &
       i_electric_fld, i_rhs, i_tmp, i_photo, flux_elec, electric_fld, i_lsf
  write(u, "(A,1X,I0,*(1X,I0))") "i:all_densities", size(all_densities), all_densities
  write(u, "(A,1X,I0,*(1X,I0))") "i:photoi_species_index", 1, photoi_species_index

  ! transport table
  call put_lt("td", td_tbl)

  ! species and reactions
  write(u, "(A,1X,I0,*(1X,I0))") "i:n_species", 3, n_species, n_gas_species, n_reactions
  write(u, "(A,1X,I0,*(1X,A))") "s:species_list", n_species, &
       (trim(species_list(i)), i = 1, n_species)
  write(u, "(A,1X,I0,*(1X,I0))") "i:species_charge", n_species, species_charge(1:n_species)
  write(u, "(A,1X,I0,*(1X,I0))") "i:species_itree", n_species, species_itree(1:n_species)
  do n = 1, n_reactions
     associate (r => reactions(n))
       write(u, "(A,I0,1X,I0,*(1X,I0))") "i:reaction_", n, 5, r%rate_type, &
            r%reaction_type, r%n_coeff, r%lookup_table_index, r%n_species_in
       write(u, "(A,I0,A,1X,I0,*(1X,ES25.17E3))") "r:reaction_", n, "_factor", 1, r%rate_factor
       write(u, "(A,I0,A,1X,I0,*(1X,ES25.17E3))") "r:reaction_", n, "_data", &
            r%n_coeff, r%rate_data(1:r%n_coeff)
       write(u, "(A,I0,A,1X,I0,*(1X,I0))") "i:reaction_", n, "_in", size(r%ix_in), r%ix_in
       write(u, "(A,I0,A,1X,I0,*(1X,I0))") "i:reaction_", n, "_out", size(r%ix_out), r%ix_out
       write(u, "(A,I0,A,1X,I0,*(1X,I0))") "i:reaction_", n, "_mult", &
            size(r%multiplicity_out), r%multiplicity_out
       write(u, "(A,I0,A,1X,I0,1X,A)") "s:reaction_", n, "_desc", 1, &
            '"' // trim(r%description) // '"'
     end associate
  end do

  ! chemtbl_fld rebuilt as chemistry_initialize builds it (330-355)
  i = count(reactions(1:n_reactions)%rate_type == 1)
  chemtbl = LT_create(td_tbl%x(1), td_tbl%x(td_tbl%n_points), &
       table_size, max(i, 1), table_xspacing)
  do n = 1, n_reactions
     if (reactions(n)%rate_type == 1) then
        call table_set_column(chemtbl, reactions(n)%lookup_table_index, &
             reactions(n)%x_data, reactions(n)%y_data)
     end if
  end do
  call put_lt("chem", chemtbl)

  ! get_rates on a field grid (0 .. 1.2 x the table range, incl. clamping)
  n_fld = 257
  allocate(flds(n_fld), rates(n_fld, max(n_reactions, 1)))
  do i = 1, n_fld
     flds(i) = (i - 1) * 1.2_dp * td_tbl%x(td_tbl%n_points) / (n_fld - 1)
  end do
  if (n_reactions > 0) call get_rates(flds, rates, n_fld)
  write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:rate_fields", n_fld, flds
  do n = 1, n_reactions
     write(u, "(A,I0,1X,I0,*(1X,ES25.17E3))") "r:rates_", n, n_fld, rates(:, n)
  end do
  close(u)

contains

  !> gas_density of programs/3d_sprite/m_user.f90:34-40 (exponential
  !> atmosphere, scale height 7.2 km)
  pure real(dp) function sprite_gas_density(box, IJK)
    type(box_t), intent(in) :: box
    integer, intent(in)     :: IJK
    real(dp)                :: rr(NDIM)
    rr = af_r_cc(box, [IJK])
    sprite_gas_density = 2.5e25_dp * exp(-rr(NDIM) / 7.2e3_dp)
  end function sprite_gas_density

  subroutine read_cfg_args(cfg)
    type(CFG_t), intent(inout) :: cfg
    integer :: n, ix
    character(len=1024) :: arg
    do n = 2, command_argument_count()
       call get_command_argument(n, arg)
       if (arg(1:11) == "--user-gas=") then
          user_gas = trim(arg(12:))
       else if (arg(1:1) == '-') then
          ix = index(arg, '=')
          call CFG_update_from_line(cfg, trim(arg(2:)))
       else
          call CFG_read_file(cfg, trim(arg))
       end if
    end do
  end subroutine read_cfg_args

  subroutine put_lt(name, lt)
    character(len=*), intent(in) :: name
    type(LT_t), intent(in) :: lt
    write(u, "(A,1X,I0,*(1X,I0))") "i:" // name // "_shape", 2, lt%n_points, lt%n_cols
    write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:" // name // "_xmin", 1, lt%x_min
    write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:" // name // "_inv_fac", 1, lt%inv_fac
    write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:" // name // "_x", lt%n_points, lt%x
    write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:" // name // "_rows_cols", &
         lt%n_points * lt%n_cols, lt%rows_cols
  end subroutine put_lt

  subroutine put_r(key)
    character(len=*), intent(in) :: key
    real(dp) :: x
    call CFG_get(cfg, key, x)
    write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:" // key, 1, x
  end subroutine put_r

  subroutine put_ra(key)
    character(len=*), intent(in) :: key
    real(dp), allocatable :: x(:)
    integer :: n
    call CFG_get_size(cfg, key, n)
    allocate(x(n))
    call CFG_get(cfg, key, x)
    write(u, "(A,1X,I0,*(1X,ES25.17E3))") "r:" // key, n, x
  end subroutine put_ra

  subroutine put_i(key)
    character(len=*), intent(in) :: key
    integer :: x
    call CFG_get(cfg, key, x)
    write(u, "(A,1X,I0,*(1X,I0))") "i:" // key, 1, x
  end subroutine put_i

  subroutine put_ia(key)
    character(len=*), intent(in) :: key
    integer, allocatable :: x(:)
    integer :: n
    call CFG_get_size(cfg, key, n)
    allocate(x(n))
    call CFG_get(cfg, key, x)
    write(u, "(A,1X,I0,*(1X,I0))") "i:" // key, n, x
  end subroutine put_ia

  subroutine put_l(key)
    character(len=*), intent(in) :: key
    logical :: x
    call CFG_get(cfg, key, x)
    call put_lv(key, x)
  end subroutine put_l

  subroutine put_lv(key, x)
    character(len=*), intent(in) :: key
    logical, intent(in) :: x
    write(u, "(A,1X,I0,1X,I0)") "i:" // key, 1, merge(1, 0, x)
  end subroutine put_lv

  subroutine put_s(key)
    character(len=*), intent(in) :: key
    character(len=512) :: x
    call CFG_get(cfg, key, x)
    write(u, "(A,1X,I0,1X,A)") "s:" // key, 1, '"' // trim(x) // '"'
  end subroutine put_s

  subroutine put_sa(key)
    character(len=*), intent(in) :: key
    character(len=64), allocatable :: x(:)
    integer :: n, i
    call CFG_get_size(cfg, key, n)
    allocate(x(n))
    call CFG_get(cfg, key, x)
    write(u, "(A,1X,I0,*(1X,A))") "s:" // key, n, ('"' // trim(x(i)) // '"', i = 1, n)
  end subroutine put_sa

end program export_case
