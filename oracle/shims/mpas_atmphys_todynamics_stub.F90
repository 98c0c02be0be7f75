! TEST INFRASTRUCTURE ONLY (oracle of the physics-coupling path; never part of the product).
!
! Test double of the physics package's module mpas_atmphys_todynamics: physics_get_tend
! (core_atmosphere/physics/mpas_atmphys_todynamics.F:59) normally turns the PBL / convection /
! radiation tendencies into the dycore's tend_ru_physics, tend_rtheta_physics, tend_rho_physics and
! the tend pool's scalars_tend.  Here it hands over PRESCRIBED tendencies, which the harness reads
! into the tend_physics pool (tend_ru_physics_in, tend_rtheta_physics_in, tend_rho_physics_in,
! scalars_tend_in), so that the unmodified dycore compiled with -DDO_PHYSICS can be run as the
! oracle of its own physics-coupling code (mpas_atm_time_integration.F:424-449, 1610-1648, 3437,
! 3743).  Same interface as the real routine.
module mpas_atmphys_todynamics
   use mpas_kind_types
   use mpas_derived_types
   use mpas_pool_routines
   implicit none
contains
   subroutine physics_get_tend(block, mesh, state, diag, tend, tend_physics, configs, rk_step, dynamics_substep, &
                               tend_ru_physics, tend_rtheta_physics, tend_rho_physics)
      type(block_type), intent(in), target :: block
      type(mpas_pool_type), intent(in) :: mesh
      type(mpas_pool_type), intent(in) :: state
      type(mpas_pool_type), intent(in) :: configs
      integer, intent(in) :: rk_step
      integer, intent(in) :: dynamics_substep
      type(mpas_pool_type), intent(inout) :: diag
      type(mpas_pool_type), intent(inout) :: tend
      type(mpas_pool_type), intent(inout) :: tend_physics
      real(kind=RKIND), dimension(:,:) :: tend_ru_physics, tend_rtheta_physics, tend_rho_physics
      real(kind=RKIND), dimension(:,:), pointer :: a
      real(kind=RKIND), dimension(:,:,:), pointer :: s_in, s_tend

      call mpas_pool_get_array(tend_physics, 'tend_ru_physics_in', a)
      tend_ru_physics(:,:) = a(:,:)
      call mpas_pool_get_array(tend_physics, 'tend_rtheta_physics_in', a)
      tend_rtheta_physics(:,:) = a(:,:)
      call mpas_pool_get_array(tend_physics, 'tend_rho_physics_in', a)
      tend_rho_physics(:,:) = a(:,:)
      call mpas_pool_get_array(tend_physics, 'scalars_tend_in', s_in)
      call mpas_pool_get_array(tend, 'scalars_tend', s_tend)
      s_tend(:,:,:) = s_in(:,:,:)
   end subroutine physics_get_tend
end module mpas_atmphys_todynamics
