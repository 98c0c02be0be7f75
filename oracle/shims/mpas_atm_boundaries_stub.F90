! Test-infrastructure shim (not reference source).  The real
! core_atmosphere/dynamics/mpas_atm_boundaries.F needs the PIO stream manager;
! the dycore uses its zone constants (mpas_atm_boundaries.F:10-12) and, when
! config_apply_lbcs = .true., the two getters below.  They read the block's 'lbc'
! pool as the real ones do (lbc_<field> time level 1 = tendency over the LBC
! interval, time level 2 = the interval-end state; scalars from lbc_scalars via
! the pool's index_<field> dimension) and evaluate the same expression
! (state - (seconds to the interval end - delta_t) * tendency, :366-407).  The
! seconds from the step start to the interval end come from the harness
! (harness_seconds_to_interval_end), standing in for LBC_intv_end - the clock time.
module mpas_atm_boundaries
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types, only : RKIND
   implicit none
   integer, parameter :: nSpecZone = 2
   integer, parameter :: nRelaxZone = 5
   integer, parameter :: nBdyZone = nSpecZone + nRelaxZone
   real (kind=RKIND) :: harness_seconds_to_interval_end = 0.0_RKIND
contains
   subroutine lbc_arrays(block, field, tl, a2, a3, idx)
      type (block_type), intent(inout) :: block
      character(len=*), intent(in) :: field
      integer, intent(in) :: tl
      real (kind=RKIND), dimension(:,:), pointer :: a2
      real (kind=RKIND), dimension(:,:,:), pointer :: a3
      integer, pointer :: idx
      type (mpas_pool_type), pointer :: lbc
      integer :: lev
      call mpas_pool_get_subpool(block % structs, 'lbc', lbc)
      lev = mpas_pool_get_error_level()
      call mpas_pool_set_error_level(MPAS_POOL_SILENT)
      nullify(a2, a3, idx)
      call mpas_pool_get_array(lbc, 'lbc_'//trim(field), a2, tl)
      if (.not. associated(a2)) then
         call mpas_pool_get_array(lbc, 'lbc_scalars', a3, tl)
         call mpas_pool_get_dimension(lbc, 'index_'//trim(field), idx)
      end if
      call mpas_pool_set_error_level(lev)
   end subroutine lbc_arrays

   function mpas_atm_get_bdy_tend(clock, block, vertDim, horizDim, field, delta_t) result(return_tend)
      type (mpas_clock_type), intent(in) :: clock
      type (block_type), intent(inout) :: block
      integer, intent(in) :: vertDim, horizDim
      character(len=*), intent(in) :: field
      real (kind=RKIND), intent(in) :: delta_t
      real (kind=RKIND), dimension(vertDim,horizDim+1) :: return_tend
      real (kind=RKIND), dimension(:,:), pointer :: t2
      real (kind=RKIND), dimension(:,:,:), pointer :: t3
      integer, pointer :: idx
      call lbc_arrays(block, field, 1, t2, t3, idx)
      if (associated(t2)) then
         return_tend(:,:) = t2(:,:)
      else
         return_tend(:,:) = t3(idx,:,:)
      end if
   end function mpas_atm_get_bdy_tend

   function mpas_atm_get_bdy_state(clock, block, vertDim, horizDim, field, delta_t) result(return_state)
      type (mpas_clock_type), intent(in) :: clock
      type (block_type), intent(inout) :: block
      integer, intent(in) :: vertDim, horizDim
      character(len=*), intent(in) :: field
      real (kind=RKIND), intent(in) :: delta_t
      real (kind=RKIND), dimension(vertDim,horizDim+1) :: return_state
      real (kind=RKIND), dimension(:,:), pointer :: t2, s2
      real (kind=RKIND), dimension(:,:,:), pointer :: t3, s3
      integer, pointer :: idx
      real (kind=RKIND) :: dt
      dt = harness_seconds_to_interval_end
      dt = dt - delta_t
      call lbc_arrays(block, field, 1, t2, t3, idx)
      call lbc_arrays(block, field, 2, s2, s3, idx)
      if (associated(t2) .and. associated(s2)) then
         return_state(:,:) = s2(:,:) - dt * t2(:,:)
      else
         return_state(:,:) = s3(idx,:,:) - dt * t3(idx,:,:)
      end if
   end function mpas_atm_get_bdy_state
end module mpas_atm_boundaries
