! Test-infrastructure shim (not reference source): the opaque PIO types that
! mpas_derived_types.F / mpas_io_types.inc name.  PIO itself is absent from this
! image and the dycore never touches I/O, so four empty types and the offset
! kind are all the framework needs to compile (SURVEY.md Appendix B step 2).
module pio_types
   implicit none
   integer, parameter :: PIO_OFFSET_KIND = selected_int_kind(18)
   integer, parameter :: PIO_OFFSET = PIO_OFFSET_KIND
   type file_desc_t
      integer :: dummy = 0
   end type file_desc_t
   type io_desc_t
      integer :: dummy = 0
   end type io_desc_t
   type iosystem_desc_t
      integer :: dummy = 0
   end type iosystem_desc_t
   type var_desc_t
      integer :: dummy = 0
   end type var_desc_t
end module pio_types

module pio
   use pio_types
end module pio
