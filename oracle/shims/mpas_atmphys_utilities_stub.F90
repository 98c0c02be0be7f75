! TEST INFRASTRUCTURE ONLY.  The DO_PHYSICS dycore uses module mpas_atmphys_utilities
! (mpas_atm_time_integration.F:25) but calls nothing from it.
module mpas_atmphys_utilities
   implicit none
end module mpas_atmphys_utilities
