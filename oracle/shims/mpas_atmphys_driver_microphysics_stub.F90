! TEST INFRASTRUCTURE ONLY.  Interface of the physics package's driver_microphysics
! (core_atmosphere/physics/mpas_atmphys_driver_microphysics.F), which the DO_PHYSICS dycore calls
! after the step when config_microp_scheme /= 'off' (mpas_atm_time_integration.F:1650-1660).
! The WRF schemes are out of scope; config_microp_scheme = 'mp_test_double' selects this test
! double instead, so that the reference and the drop-in can be compared with a microphysics step
! between the dynamics and the end of atm_srk3 (the regional specified-zone reset, 1672-1790, and
! summarize_timestep, 1794, follow it).  It changes what a scheme changes on the owned cells
! its..ite: theta_m and the moist scalars of time level time_lev, by smooth deterministic amounts
! (condensation-like: qv down by 0.5 %, theta_m up by L/cp-like heating of that vapour).
module mpas_atmphys_driver_microphysics
   use mpas_kind_types
   use mpas_derived_types
   use mpas_pool_routines
   implicit none
contains
   subroutine driver_microphysics(configs, mesh, state, time_lev, diag, diag_physics, tend, itimestep, its, ite)
      type(mpas_pool_type), intent(in) :: configs, mesh
      type(mpas_pool_type), intent(inout) :: state, diag, diag_physics, tend
      integer, intent(in) :: time_lev, itimestep, its, ite
      character(len=StrKIND), pointer :: scheme
      real(kind=RKIND), dimension(:,:), pointer :: theta_m
      real(kind=RKIND), dimension(:,:,:), pointer :: scalars
      integer, pointer :: index_qv
      integer :: i, k
      real(kind=RKIND) :: dq
      call mpas_pool_get_config(configs, 'config_microp_scheme', scheme)
      if (trim(scheme) /= 'mp_test_double') then
         write(0, *) 'oracle: driver_microphysics test double: config_microp_scheme must be mp_test_double'
         stop 3
      end if
      call mpas_pool_get_array(state, 'theta_m', theta_m, time_lev)
      call mpas_pool_get_array(state, 'scalars', scalars, time_lev)
      call mpas_pool_get_dimension(state, 'index_qv', index_qv)
      do i = its, ite
         do k = 1, size(theta_m, 1)
            dq = 0.005_RKIND * scalars(index_qv, k, i)
            scalars(index_qv, k, i) = scalars(index_qv, k, i) - dq
            theta_m(k, i) = theta_m(k, i) * (1.0_RKIND + 2.5_RKIND * dq)
         end do
      end do
   end subroutine driver_microphysics
end module mpas_atmphys_driver_microphysics
