! TEST INFRASTRUCTURE ONLY.  Interface of the physics package's driver_microphysics
! (core_atmosphere/physics/mpas_atmphys_driver_microphysics.F), which the DO_PHYSICS dycore calls
! after the step when config_microp_scheme /= 'off' (mpas_atm_time_integration.F:1650-1660).  The
! physics-coupling oracle runs with config_microp_scheme = 'off', so reaching this is an error.
module mpas_atmphys_driver_microphysics
   use mpas_kind_types
   use mpas_derived_types
   implicit none
contains
   subroutine driver_microphysics(configs, mesh, state, time_lev, diag, diag_physics, tend, itimestep, its, ite)
      type(mpas_pool_type), intent(in) :: configs, mesh
      type(mpas_pool_type), intent(inout) :: state, diag, diag_physics, tend
      integer, intent(in) :: time_lev, itimestep, its, ite
      write(0, *) 'oracle: driver_microphysics is not available (config_microp_scheme must be off)'
      stop 3
   end subroutine driver_microphysics
end module mpas_atmphys_driver_microphysics
