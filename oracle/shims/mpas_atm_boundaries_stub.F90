! Test-infrastructure shim (not reference source).  The real
! core_atmosphere/dynamics/mpas_atm_boundaries.F needs the PIO stream manager;
! the dycore only uses its zone constants (mpas_atm_boundaries.F:10-12) and,
! when config_apply_lbcs=.true. (never in our configs), the two getters below.
module mpas_atm_boundaries
   use mpas_derived_types, only : mpas_clock_type, block_type
   use mpas_kind_types, only : RKIND
   implicit none
   integer, parameter :: nSpecZone = 2
   integer, parameter :: nRelaxZone = 5
   integer, parameter :: nBdyZone = nSpecZone + nRelaxZone
contains
   function mpas_atm_get_bdy_tend(clock, block, vertDim, horizDim, field, delta_t) result(return_tend)
      type (mpas_clock_type), intent(in) :: clock
      type (block_type), intent(inout) :: block
      integer, intent(in) :: vertDim, horizDim
      character(len=*), intent(in) :: field
      real (kind=RKIND), intent(in) :: delta_t
      real (kind=RKIND), dimension(vertDim,horizDim+1) :: return_tend
      return_tend(:,:) = 0.0_RKIND
   end function mpas_atm_get_bdy_tend

   function mpas_atm_get_bdy_state(clock, block, vertDim, horizDim, field, delta_t) result(return_state)
      type (mpas_clock_type), intent(in) :: clock
      type (block_type), intent(inout) :: block
      integer, intent(in) :: vertDim, horizDim
      character(len=*), intent(in) :: field
      real (kind=RKIND), intent(in) :: delta_t
      real (kind=RKIND), dimension(vertDim,horizDim+1) :: return_state
      return_state(:,:) = 0.0_RKIND
   end function mpas_atm_get_bdy_state
end module mpas_atm_boundaries
