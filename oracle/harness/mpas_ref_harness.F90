! =============================================================================
! mpas_ref_harness -- TEST INFRASTRUCTURE ONLY (the "oracle", never the product)
!
! Drives the UNMODIFIED reference dycore (module atm_time_integration, compiled
! from /root/reference by oracle/Makefile) on synthetic inputs written by
! mpas-model_amd/mpas_dycore/io_oracle.py.  It plays the role of
! core_atmosphere/mpas_atm_core.F for a single block on one MPI rank:
!
!   * builds block%structs pools 'mesh','state'(2 time levels),'diag','tend',
!     'tend_physics' plus block%dimensions and the configs pool in memory
!     (what the Registry-generated code does in the real model);
!   * runs the model-init diagnostics exactly as atm_mpas_init_block does
!     (mpas_atm_core.F:365-424): atm_init_coupled_diagnostics,
!     atm_compute_solve_diagnostics, mpas_rbf_interp_initialize,
!     mpas_init_reconstruct;
!   * steps atm_srk3 (mpas_atm_time_integration.F:142) nsteps times, shifting
!     time levels after each step (mpas_atm_core.F:671);
!   * dumps every real field of every pool (raw little-endian, Fortran order,
!     including the n+1 garbage slot) and the wall time of each step.
!
! Usage:  mpas_ref_harness <input_dir> <output_dir>
!   <input_dir>/harness.nml   namelist /harness/ (dims, configs, nsteps, dump_steps)
!   <input_dir>/<field>.bin   input arrays (missing files -> zero)
! =============================================================================
module harness_fields
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types
   implicit none

   character(len=256) :: indir, outdir
   ! comma-separated 'pool.name' list; when not blank only these fields are dumped (full-size runs)
   character(len=1024) :: dump_only = ''
   logical :: dump_ints = .false.   ! mode 'init' also dumps integer fields (index arrays it builds)
   ! multi-block runs: fields are registered (for dumping) from the first block only, are active
   ! (so mpas_dmpar exchanges them), and carry their decomposed dimension's name (for
   ! mpas_pool_link_parinfo), inferred from the current block's element counts
   logical :: registering = .true., fields_active = .false.
   integer :: cur_nC1 = -1, cur_nE1 = -1, cur_nV1 = -1
   type (block_type), pointer :: hblock => null()

   integer, parameter :: MAXF = 400
   integer :: nf = 0
   character(len=64), dimension(MAXF) :: fname, fpool
   integer, dimension(MAXF) :: frank, fntl
   logical, dimension(MAXF) :: fisint

contains

   logical function file_exists(name)
      character(len=*), intent(in) :: name
      inquire(file=trim(indir)//'/'//trim(name)//'.bin', exist=file_exists)
   end function file_exists

   character(len=StrKIND) function dimname_of(n)
      integer, intent(in) :: n
      dimname_of = 'nVertLevels'
      if (n == cur_nC1) dimname_of = 'nCells'
      if (n == cur_nE1) dimname_of = 'nEdges'
      if (n == cur_nV1) dimname_of = 'nVertices'
   end function dimname_of

   subroutine register(pname, name, rnk, ntl, isint)
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: rnk, ntl
      logical, intent(in) :: isint
      if (.not. registering) return
      nf = nf + 1
      fname(nf) = name
      fpool(nf) = pname
      frank(nf) = rnk
      fntl(nf) = ntl
      fisint(nf) = isint
   end subroutine register

   subroutine read_r(name, a, n)
      character(len=*), intent(in) :: name
      integer, intent(in) :: n
      real(kind=RKIND), intent(inout) :: a(n)
      integer :: u
      if (.not. file_exists(name)) return
      open(newunit=u, file=trim(indir)//'/'//trim(name)//'.bin', access='stream', form='unformatted', status='old')
      read(u) a
      close(u)
   end subroutine read_r

   subroutine read_i(name, a, n)
      character(len=*), intent(in) :: name
      integer, intent(in) :: n
      integer, intent(inout) :: a(n)
      integer :: u
      if (.not. file_exists(name)) return
      open(newunit=u, file=trim(indir)//'/'//trim(name)//'.bin', access='stream', form='unformatted', status='old')
      read(u) a
      close(u)
   end subroutine read_i

   ! restore a field from a previous dump (pool.name[.tlN].bin), used by the kernel modes
   subroutine read_dump_r(pname, name, t, ntl, a, n)
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: t, ntl, n
      real(kind=RKIND), intent(inout) :: a(n)
      character(len=8) :: tl
      character(len=320) :: fn
      logical :: ex
      integer :: u
      tl = ''
      if (ntl > 1) write(tl, '(a,i1)') '.tl', t
      fn = trim(indir)//'/'//trim(pname)//'.'//trim(name)//trim(tl)//'.bin'
      inquire(file=trim(fn), exist=ex)
      if (.not. ex) return
      open(newunit=u, file=trim(fn), access='stream', form='unformatted', status='old')
      read(u) a
      close(u)
   end subroutine read_dump_r

   subroutine add_r0(pool, pname, name)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name
      type (field0DReal), pointer :: f
      real(kind=RKIND) :: tmp(1)
      allocate(f)
      f % block => hblock
      f % fieldName = name
      f % isActive = .false.
      tmp(1) = 0.0_RKIND
      call read_r(name, tmp, 1)
      f % scalar = tmp(1)
      call mpas_pool_add_field(pool, name, f)
      call register(pname, name, 0, 1, .false.)
   end subroutine add_r0

   subroutine add_r1(pool, pname, name, d1)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: d1
      type (field1DReal), pointer :: f
      allocate(f)
      f % block => hblock
      f % fieldName = name
      f % isActive = .false.
      f % dimSizes(1) = d1
      f % isActive = fields_active
      f % dimNames(1) = dimname_of(d1)
      allocate(f % array(d1))
      f % array = 0.0_RKIND
      call read_r(name, f % array, d1)
      call read_dump_r(pname, name, 1, 1, f % array, d1)
      call mpas_pool_add_field(pool, name, f)
      call register(pname, name, 1, 1, .false.)
   end subroutine add_r1

   subroutine add_r2(pool, pname, name, d1, d2, ntl)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: d1, d2, ntl
      type (field2DReal), dimension(:), pointer :: fa
      integer :: t
      allocate(fa(ntl))
      do t = 1, ntl
         fa(t) % block => hblock
         fa(t) % fieldName = name
         fa(t) % isActive = .false.
         fa(t) % dimSizes(1) = d1
         fa(t) % dimSizes(2) = d2
         fa(t) % isActive = fields_active
         fa(t) % dimNames(2) = dimname_of(d2)
         allocate(fa(t) % array(d1, d2))
         fa(t) % array = 0.0_RKIND
      end do
      call read_r(name, fa(1) % array, d1*d2)
      do t = 1, ntl
         call read_dump_r(pname, name, t, ntl, fa(t) % array, d1*d2)
      end do
      call mpas_pool_add_field(pool, name, fa)
      call register(pname, name, 2, ntl, .false.)
   end subroutine add_r2

   subroutine add_r3(pool, pname, name, d1, d2, d3, ntl)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: d1, d2, d3, ntl
      type (field3DReal), dimension(:), pointer :: fa
      integer :: t
      allocate(fa(ntl))
      do t = 1, ntl
         fa(t) % block => hblock
         fa(t) % fieldName = name
         fa(t) % isActive = .false.
         fa(t) % dimSizes(1) = d1
         fa(t) % dimSizes(2) = d2
         fa(t) % dimSizes(3) = d3
         fa(t) % isActive = fields_active
         fa(t) % dimNames(3) = dimname_of(d3)
         allocate(fa(t) % array(d1, d2, d3))
         fa(t) % array = 0.0_RKIND
      end do
      call read_r(name, fa(1) % array, d1*d2*d3)
      do t = 1, ntl
         call read_dump_r(pname, name, t, ntl, fa(t) % array, d1*d2*d3)
      end do
      call mpas_pool_add_field(pool, name, fa)
      call register(pname, name, 3, ntl, .false.)
   end subroutine add_r3

   ! a character field of ntl time levels (state xtime, Registry.xml), initialised to `init`
   subroutine add_c0(pool, pname, name, ntl, init)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name, init
      integer, intent(in) :: ntl
      type (field0DChar), dimension(:), pointer :: fa
      integer :: t
      allocate(fa(ntl))
      do t = 1, ntl
         fa(t) % block => hblock
         fa(t) % fieldName = name
         fa(t) % isActive = .false.
         fa(t) % scalar = init
      end do
      call mpas_pool_add_field(pool, name, fa)
      call register(pname, name, -1, ntl, .false.)
   end subroutine add_c0

   subroutine add_i1(pool, pname, name, d1)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: d1
      type (field1DInteger), pointer :: f
      allocate(f)
      f % block => hblock
      f % fieldName = name
      f % isActive = .false.
      f % dimSizes(1) = d1
      allocate(f % array(d1))
      f % array = 0
      call read_i(name, f % array, d1)
      call mpas_pool_add_field(pool, name, f)
      call register(pname, name, 1, 1, .true.)
   end subroutine add_i1

   subroutine add_i2(pool, pname, name, d1, d2)
      type (mpas_pool_type), pointer :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: d1, d2
      type (field2DInteger), pointer :: f
      allocate(f)
      f % block => hblock
      f % fieldName = name
      f % isActive = .false.
      f % dimSizes(1) = d1
      f % dimSizes(2) = d2
      allocate(f % array(d1, d2))
      f % array = 0
      call read_i(name, f % array, d1*d2)
      call mpas_pool_add_field(pool, name, f)
      call register(pname, name, 2, 1, .true.)
   end subroutine add_i2

   subroutine dump_all(dir, pools)
      character(len=*), intent(in) :: dir
      type (mpas_pool_type), pointer, dimension(:) :: pools
      integer :: i, u, ip, t
      character(len=8) :: tl
      type (mpas_pool_type), pointer :: p
      type (field0DReal), pointer :: f0
      type (field1DReal), pointer :: f1
      type (field2DReal), pointer :: f2
      type (field3DReal), pointer :: f3
      type (field1DInteger), pointer :: i1
      type (field2DInteger), pointer :: i2
      type (field0DChar), pointer :: c0
      call execute_command_line('mkdir -p '//trim(dir))
      do i = 1, nf
         if (frank(i) < 0) then   ! character scalar (state xtime), one text file per time level
            call mpas_pool_get_subpool(hblock % structs, trim(fpool(i)), p)
            do t = 1, fntl(i)
               write(tl, '(a,i1)') '.tl', t
               call mpas_pool_get_field(p, trim(fname(i)), c0, t)
               open(newunit=u, file=trim(dir)//'/'//trim(fpool(i))//'.'//trim(fname(i))//trim(tl)//'.txt', &
                    status='replace')
               write(u, '(a)') trim(c0 % scalar)
               close(u)
            end do
            cycle
         end if
         if (fisint(i)) then
            if (.not. dump_ints) cycle
            call mpas_pool_get_subpool(hblock % structs, trim(fpool(i)), p)
            open(newunit=u, file=trim(dir)//'/'//trim(fpool(i))//'.'//trim(fname(i))//'.bin', &
                 access='stream', form='unformatted', status='replace')
            if (frank(i) == 1) then
               call mpas_pool_get_field(p, trim(fname(i)), i1)
               write(u) i1 % array
            else
               call mpas_pool_get_field(p, trim(fname(i)), i2)
               write(u) i2 % array
            end if
            close(u)
            cycle
         end if
         if (len_trim(dump_only) > 0) then
            if (index(','//trim(dump_only)//',', ','//trim(fpool(i))//'.'//trim(fname(i))//',') == 0) cycle
         end if
         call mpas_pool_get_subpool(hblock % structs, trim(fpool(i)), p)
         do t = 1, fntl(i)
            tl = ''
            if (fntl(i) > 1) write(tl, '(a,i1)') '.tl', t
            open(newunit=u, file=trim(dir)//'/'//trim(fpool(i))//'.'//trim(fname(i))//trim(tl)//'.bin', &
                 access='stream', form='unformatted', status='replace')
            select case (frank(i))
            case (0)
               call mpas_pool_get_field(p, trim(fname(i)), f0)
               write(u) f0 % scalar
            case (1)
               call mpas_pool_get_field(p, trim(fname(i)), f1)
               write(u) f1 % array
            case (2)
               call mpas_pool_get_field(p, trim(fname(i)), f2, t)
               write(u) f2 % array
            case (3)
               call mpas_pool_get_field(p, trim(fname(i)), f3, t)
               write(u) f3 % array
            end select
            close(u)
         end do
      end do
   end subroutine dump_all

end module harness_fields


program mpas_ref_harness
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types
   use mpas_dmpar
   use mpas_log
   use mpas_atm_dimensions
   use atm_time_integration
   use mpas_rbf_interpolation
   use mpas_vector_reconstruction
   use mpas_timekeeping
   use harness_fields
   use mpas_atm_boundaries, only : harness_seconds_to_interval_end
#ifdef HARNESS_INIT
   use atm_advection, only : atm_initialize_advection_rk, atm_initialize_deformation_weights
   use atm_jw_ref, only : init_atm_case_jw
   use atm_core_init_ref, only : atm_compute_mesh_scaling, atm_compute_signs, atm_compute_damping_coefs, &
                                 atm_adv_coef_compression, atm_couple_coef_3rd_order
#endif
   use omp_lib
   implicit none

   ! ---- namelist inputs (written by io_oracle.py) ----
   integer :: nCells, nEdges, nVertices, nVertLevels_in, maxEdges_in, maxEdges2_in, num_scalars_in
   integer :: nsteps, moist_end, nthreads_req
   integer :: dump_steps(16)
   real(kind=RKIND) :: dt, sphere_radius
   integer :: config_time_integration_order, config_number_of_sub_steps, config_dynamics_split_steps
   integer :: config_number_rayleigh_damp_u_levels
   logical :: config_split_dynamics_transport, config_scalar_advection, config_positive_definite
   logical :: config_monotonic, config_mix_full, config_rayleigh_damp_u
   real(kind=RKIND) :: config_h_mom_eddy_visc2, config_h_mom_eddy_visc4, config_v_mom_eddy_visc2
   real(kind=RKIND) :: config_h_theta_eddy_visc2, config_h_theta_eddy_visc4, config_v_theta_eddy_visc2
   real(kind=RKIND) :: config_len_disp, config_visc4_2dsmag, config_del4u_div_factor, config_coef_3rd_order
   real(kind=RKIND) :: config_smagorinsky_coef, config_epssm, config_smdiv, config_apvm_upwinding
   real(kind=RKIND) :: config_mpas_cam_coef, config_rayleigh_damp_u_timescale_days
   character(len=64) :: config_horiz_mixing, config_convection_scheme, config_microp_scheme
   real(kind=RKIND) :: config_zd, config_xnutr
   logical :: config_h_ScaleWithMesh
   character(len=32) :: mode
   logical :: config_apply_lbcs_in          ! regional LBCs: lbc pool + masks from the inputs
   real(kind=RKIND) :: lbc_interval_end     ! seconds from the first step's start to the LBC interval end
   integer :: kernel_small_step, kernel_rk_step
   real(kind=RKIND) :: kernel_dts
   integer :: print_minmax   ! summarize_timestep switches: 1 global_minmax_vel, 2 detailed_minmax_vel, 4 global_minmax_sca
   integer :: nblocks, ib, nhalo_ev
   integer :: nCellsSolve_in, nEdgesSolve_in, nVerticesSolve_in
   character(len=256) :: rootdir
   type (block_type), pointer :: blk
   type (field2DReal), pointer :: f2_u, f2_pv, f2_ru, f2_rw
   namelist /block/ nCells, nEdges, nVertices, nCellsSolve_in, nEdgesSolve_in, nVerticesSolve_in
   namelist /harness/ mode, nblocks, print_minmax, dump_only, kernel_small_step, kernel_rk_step, kernel_dts, nCells, nEdges, nVertices, nVertLevels_in, maxEdges_in, maxEdges2_in, num_scalars_in, &
      nsteps, moist_end, nthreads_req, dump_steps, dt, sphere_radius, &
      config_time_integration_order, config_number_of_sub_steps, config_dynamics_split_steps, &
      config_number_rayleigh_damp_u_levels, config_split_dynamics_transport, config_scalar_advection, &
      config_positive_definite, config_monotonic, config_mix_full, config_rayleigh_damp_u, &
      config_h_mom_eddy_visc2, config_h_mom_eddy_visc4, config_v_mom_eddy_visc2, &
      config_h_theta_eddy_visc2, config_h_theta_eddy_visc4, config_v_theta_eddy_visc2, &
      config_len_disp, config_visc4_2dsmag, config_del4u_div_factor, config_coef_3rd_order, &
      config_smagorinsky_coef, config_epssm, config_smdiv, config_apvm_upwinding, &
      config_mpas_cam_coef, config_rayleigh_damp_u_timescale_days, config_horiz_mixing, config_convection_scheme, &
      config_microp_scheme, config_zd, config_xnutr, config_h_ScaleWithMesh, config_apply_lbcs_in, lbc_interval_end

   type (domain_type), pointer :: domain
   type (mpas_pool_type), pointer :: configs, dimpool, mesh, state, diag, tend, tend_physics, diag_physics
   type (mpas_pool_type), pointer, dimension(:) :: plist
   integer :: K, nC1, nE1, nV1, ns, step, i, u, nthr, t
   integer, dimension(:), pointer :: cts, cte, csts, cste, ets, ete, ests, este, vts, vte, vsts, vste
   real(kind=RKIND), dimension(:,:), pointer :: uu, uReconstructX, uReconstructY, uReconstructZ, &
                                                uReconstructZonal, uReconstructMeridional
   real(kind=RKIND) :: t0, t1, t2, tloop, twarm
   real(kind=RKIND) :: tdumps = 0.0_RKIND, tdumps2 = 0.0_RKIND
   real(kind=RKIND), allocatable :: steptime(:)
   character(len=16) :: sdir
   type (MPAS_Time_type) :: nowTime
   type (MPAS_TimeInterval_type) :: dtInterval
   character(len=*), parameter :: start_time = '2000-01-01_00:00:00'

   call get_command_argument(1, indir)
   call get_command_argument(2, outdir)
   dump_steps = -1
   nthreads_req = 0
   moist_end = 1
   config_horiz_mixing = '2d_smagorinsky'
   config_convection_scheme = 'off'
   config_microp_scheme = 'off'
   mode = 'run'
   kernel_small_step = 2
   kernel_rk_step = 1
   kernel_dts = 0.0_RKIND
   print_minmax = 0
   nblocks = 1
   config_apply_lbcs_in = .false.
   lbc_interval_end = 0.0_RKIND
   config_zd = 22000.0_RKIND       ! Registry.xml defaults
   config_xnutr = 0.2_RKIND
   config_h_ScaleWithMesh = .true.
   open(newunit=u, file=trim(indir)//'/harness.nml', status='old')
   read(u, nml=harness)
   close(u)
   if (nthreads_req > 0) call omp_set_num_threads(nthreads_req)
   nthr = omp_get_max_threads()
   nCellsSolve_in = nCells
   nEdgesSolve_in = nEdges
   nVerticesSolve_in = nVertices
   ! halo layers of the exchange lists: cells 2, edges / vertices 3 (mpas_block_creator.F:734);
   ! a single block keeps 2 everywhere (its lists are empty and its fields inactive)
   nhalo_ev = 2
   if (nblocks > 1) nhalo_ev = 3
   fields_active = nblocks > 1

   K = nVertLevels_in
   ns = num_scalars_in
   nC1 = nCells + 1
   nE1 = nEdges + 1
   nV1 = nVertices + 1

   ! ---- domain / block / log / MPI (mpas_subdriver.F equivalent, one rank) ----
   allocate(domain)
   allocate(domain % dminfo)
   call mpas_dmpar_init(domain % dminfo)
   allocate(domain % core)
   domain % core % coreName = 'atmosphere'
   call mpas_log_init(domain % logInfo, domain)
   call mpas_log_open()
   call mpas_pool_create_pool(configs)
   domain % configs => configs
   nullify(domain % clock)
   ! the time loop passes atm_timestep its nowTime as mpas_atm_core.F does (atm_do_timestep)
   call mpas_timekeeping_init('gregorian')
   call mpas_set_time(nowTime, dateTimeString=start_time)

   call mpas_atm_set_dims(K, maxEdges_in, maxEdges2_in, ns)

   ! ---- configs (Registry.xml:56-290 names) ----
   call mpas_pool_add_config_char(configs, 'config_time_integration', 'SRK3')
   call mpas_pool_add_config_int(configs, 'config_time_integration_order', config_time_integration_order)
   call mpas_pool_add_config_real(configs, 'config_dt', dt)
   call mpas_pool_add_config_logical(configs, 'config_split_dynamics_transport', config_split_dynamics_transport)
   call mpas_pool_add_config_int(configs, 'config_number_of_sub_steps', config_number_of_sub_steps)
   call mpas_pool_add_config_int(configs, 'config_dynamics_split_steps', config_dynamics_split_steps)
   call mpas_pool_add_config_real(configs, 'config_h_mom_eddy_visc2', config_h_mom_eddy_visc2)
   call mpas_pool_add_config_real(configs, 'config_h_mom_eddy_visc4', config_h_mom_eddy_visc4)
   call mpas_pool_add_config_real(configs, 'config_v_mom_eddy_visc2', config_v_mom_eddy_visc2)
   call mpas_pool_add_config_real(configs, 'config_h_theta_eddy_visc2', config_h_theta_eddy_visc2)
   call mpas_pool_add_config_real(configs, 'config_h_theta_eddy_visc4', config_h_theta_eddy_visc4)
   call mpas_pool_add_config_real(configs, 'config_v_theta_eddy_visc2', config_v_theta_eddy_visc2)
   call mpas_pool_add_config_char(configs, 'config_horiz_mixing', trim(config_horiz_mixing))
   call mpas_pool_add_config_real(configs, 'config_len_disp', config_len_disp)
   call mpas_pool_add_config_real(configs, 'config_visc4_2dsmag', config_visc4_2dsmag)
   call mpas_pool_add_config_real(configs, 'config_del4u_div_factor', config_del4u_div_factor)
   call mpas_pool_add_config_logical(configs, 'config_scalar_advection', config_scalar_advection)
   call mpas_pool_add_config_logical(configs, 'config_positive_definite', config_positive_definite)
   call mpas_pool_add_config_logical(configs, 'config_monotonic', config_monotonic)
   call mpas_pool_add_config_real(configs, 'config_coef_3rd_order', config_coef_3rd_order)
   ! init_atmosphere namelist keys the JW case reads (mode 'jw'): Registry defaults of core_init_atmosphere
   call mpas_pool_add_config_int(configs, 'config_init_case', 2)
   call mpas_pool_add_config_int(configs, 'config_theta_adv_order', 3)
   call mpas_pool_add_config_real(configs, 'config_smagorinsky_coef', config_smagorinsky_coef)
   call mpas_pool_add_config_logical(configs, 'config_mix_full', config_mix_full)
   call mpas_pool_add_config_real(configs, 'config_epssm', config_epssm)
   call mpas_pool_add_config_real(configs, 'config_smdiv', config_smdiv)
   call mpas_pool_add_config_real(configs, 'config_apvm_upwinding', config_apvm_upwinding)
   call mpas_pool_add_config_real(configs, 'config_mpas_cam_coef', config_mpas_cam_coef)
   call mpas_pool_add_config_logical(configs, 'config_rayleigh_damp_u', config_rayleigh_damp_u)
   call mpas_pool_add_config_real(configs, 'config_rayleigh_damp_u_timescale_days', config_rayleigh_damp_u_timescale_days)
   call mpas_pool_add_config_int(configs, 'config_number_rayleigh_damp_u_levels', config_number_rayleigh_damp_u_levels)
   call mpas_pool_add_config_logical(configs, 'config_apply_lbcs', config_apply_lbcs_in)
   call mpas_pool_add_config_char(configs, 'config_IAU_option', 'off')
   call mpas_pool_add_config_char(configs, 'config_microp_scheme', trim(config_microp_scheme))
   call mpas_pool_add_config_char(configs, 'config_convection_scheme', trim(config_convection_scheme))
   call mpas_pool_add_config_logical(configs, 'config_print_global_minmax_vel', iand(print_minmax, 1) /= 0)
   call mpas_pool_add_config_logical(configs, 'config_print_detailed_minmax_vel', iand(print_minmax, 2) /= 0)
   call mpas_pool_add_config_logical(configs, 'config_print_global_minmax_sca', iand(print_minmax, 4) /= 0)
   call mpas_pool_add_config_real(configs, 'config_zd', config_zd)
   call mpas_pool_add_config_real(configs, 'config_xnutr', config_xnutr)
   call mpas_pool_add_config_logical(configs, 'config_h_ScaleWithMesh', config_h_ScaleWithMesh)


   ! ---- blocks (one, or nblocks with local-copy halo exchanges between them) ----
   rootdir = indir
   nullify(hblock)
   do ib = 0, nblocks - 1
      call build_block(ib)
   end do
   if (nblocks > 1) call link_blocks()

   allocate(plist(1))
   write(0, '(a)') 'harness: pools built'

   if (nblocks > 1) then
      ! model init (mpas_atm_core.F:143-186): u exchange, per-block diagnostics, then the
      ! pv_edge / ru / rw exchanges; then the time loop (atm_srk3 exchanges between the blocks)
      call mpas_pool_get_subpool(domain % blocklist % structs, 'state', state)
      call mpas_pool_get_field(state, 'u', f2_u, 1)
      call mpas_dmpar_exch_halo_field(f2_u)
      blk => domain % blocklist
      do while (associated(blk))
         call init_block(blk)
         blk => blk % next
      end do
      call mpas_pool_get_subpool(domain % blocklist % structs, 'diag', diag)
      call mpas_pool_get_field(diag, 'pv_edge', f2_pv)
      call mpas_dmpar_exch_halo_field(f2_pv)
      call mpas_pool_get_field(diag, 'ru', f2_ru)
      call mpas_dmpar_exch_halo_field(f2_ru)
      call mpas_pool_get_field(diag, 'rw', f2_rw)
      call mpas_dmpar_exch_halo_field(f2_rw)
      write(0, '(a)') 'harness: init diagnostics done'
      if (any(dump_steps == 0)) call dump_blocks(trim(outdir)//'/step_0000')
      call mpas_pool_get_config(configs, 'config_apply_lbcs', config_apply_lbcs)
      allocate(steptime(max(nsteps,1)))
      call mpas_set_timeInterval(dtInterval, dt=dt)
      tloop = omp_get_wtime()
      do step = 1, nsteps
         t0 = omp_get_wtime()
         call atm_timestep(domain, dt, nowTime, step)
         nowTime = nowTime + dtInterval
         t1 = omp_get_wtime()
         steptime(step) = t1 - t0
         if (step == 2) then   ! steady state: both time-level parities have run once
#ifdef MPAS_DYCORE_DROPIN
            call atm_dycore_wait()
#endif
            twarm = omp_get_wtime()
         end if
         write(0, '(a,i6,f10.3)') 'harness: step', step, steptime(step)
         ! once, on the first block: the state fields of all blocks are linked (mpas_atm_core.F:670-671)
         call mpas_pool_get_subpool(domain % blocklist % structs, 'state', state)
         call mpas_pool_shift_time_levels(state)
#ifdef MPAS_DYCORE_DROPIN
         if (any(dump_steps == step)) call atm_dycore_wait()   ! device time stays in the loop's time
#endif
   #ifdef MPAS_DYCORE_DROPIN
      if (any(dump_steps == step)) call atm_dycore_wait()   ! device time stays in the loop's time
#endif
      t2 = omp_get_wtime()   ! dumps are not part of the loop's time
         if (any(dump_steps == step)) then
            write(sdir, '(a,i4.4)') 'step_', step
#ifdef MPAS_DYCORE_DROPIN
            call atm_dycore_to_host(domain)   ! the HBM state into the pools before they are read
#endif
            call dump_blocks(trim(outdir)//'/'//trim(sdir))
         end if
         tdumps = tdumps + (omp_get_wtime() - t2)
         if (step > 2) tdumps2 = tdumps2 + (omp_get_wtime() - t2)
      end do
#ifdef MPAS_DYCORE_DROPIN
      call atm_dycore_wait()   ! the steps run asynchronously: the loop ends when the device is done
#endif
      twarm = omp_get_wtime() - twarm - tdumps2
      tloop = omp_get_wtime() - tloop - tdumps
#ifdef MPAS_DYCORE_DROPIN
      call atm_dycore_to_host(domain)
#endif
      call execute_command_line('mkdir -p '//trim(outdir))
      open(newunit=u, file=trim(outdir)//'/timing.txt', status='replace')
      write(u, '(a,i6)') 'threads ', nthr
      do step = 1, nsteps
         write(u, '(a,i6,es24.16)') 'step ', step, steptime(step)
      end do
      write(u, '(a,es24.16)') 'total ', tloop
      if (nsteps > 2) write(u, '(a,es24.16)') 'after2 ', twarm   ! steps 3..nsteps
      close(u)
      call mpas_dmpar_finalize(domain % dminfo)
      stop
   end if

#ifdef HARNESS_INIT
   if (trim(mode) == 'init') then
      ! the reference's mesh-dependent precompute, in model order: deriv_two / defc_a / defc_b as
      ! init_atmosphere computes them for the init file (mpas_init_atm_cases.F:190-191 via
      ! mpas_atm_advection.F), then atm_mpas_init_block's own (mpas_atm_core.F:311, 358, 360, 456, 458)
      dump_ints = .true.
      call atm_initialize_advection_rk(mesh, nCells, nEdges, maxEdges_in, .true., sphere_radius)
      call atm_initialize_deformation_weights(mesh, nCells, .true., sphere_radius)
      call atm_compute_signs(mesh)
      call atm_adv_coef_compression(mesh)
      call atm_couple_coef_3rd_order(mesh, configs)
      call atm_compute_mesh_scaling(mesh, configs)
      call atm_compute_damping_coefs(mesh, configs)
      call dump_all(trim(outdir)//'/step_0000', plist)
      call mpas_dmpar_finalize(domain % dminfo)
      stop
   end if
   if (trim(mode) == 'jw') then
      ! the reference's Jablonowski-Williamson initial state (init_atmosphere, config_init_case = 2,
      ! mpas_init_atm_cases.F:367-1160) on the case's mesh given on the unit sphere: it scales the
      ! mesh, computes deriv_two / defc, the vertical grid and metrics, the state, zb / zb3, rw / w
      call init_atm_case_jw(mesh, nCells, K, state, diag, configs, 2)
      call dump_all(trim(outdir)//'/step_0000', plist)
      call mpas_dmpar_finalize(domain % dminfo)
      stop
   end if
#endif

   if (trim(mode) == 'acoustic') then
      ! kernel mode: one acoustic sub-step on a state restored from a dump
      ! (atm_advance_acoustic_step 2312 + atm_divergence_damping_3d 2726), as srk3 calls them (794-869)
!$OMP PARALLEL DO
      do t = 1, nthr
         call atm_advance_acoustic_step(state, diag, tend, mesh, configs, nCells, K, kernel_dts, kernel_small_step, &
                                        cts(t), cte(t), vts(t), vte(t), ets(t), ete(t), &
                                        csts(t), cste(t), vsts(t), vste(t), ests(t), este(t))
      end do
!$OMP END PARALLEL DO
!$OMP PARALLEL DO
      do t = 1, nthr
         call atm_divergence_damping_3d(state, diag, mesh, configs, kernel_dts, ets(t), ete(t))
      end do
!$OMP END PARALLEL DO
      call dump_all(trim(outdir)//'/step_0000', plist)
      call mpas_dmpar_finalize(domain % dminfo)
      stop
   end if

   ! ---- model init (mpas_atm_core.F:365-424) ----
   allocate(ke_vertex(K, nV1))
   ke_vertex(:, nV1) = 0.0_RKIND
   allocate(ke_edge(K, nE1))
   ke_edge(:, nE1) = 0.0_RKIND
!$OMP PARALLEL DO
   do t = 1, nthr
      call atm_init_coupled_diagnostics(state, 1, diag, mesh, configs, cts(t), cte(t), vts(t), vte(t), &
                                        ets(t), ete(t), csts(t), cste(t), vsts(t), vste(t), ests(t), este(t))
      call atm_compute_solve_diagnostics(dt, state, 1, diag, mesh, configs, cts(t), cte(t), vts(t), vte(t), &
                                         ets(t), ete(t))
   end do
!$OMP END PARALLEL DO
   deallocate(ke_vertex)
   deallocate(ke_edge)
   write(0, '(a)') 'harness: init diagnostics done'
   call mpas_rbf_interp_initialize(mesh)
   write(0, '(a)') 'harness: rbf init done'
   call mpas_init_reconstruct(mesh)
   write(0, '(a)') 'harness: reconstruct init done'
   call mpas_pool_get_array(state, 'u', uu, 1)
   call mpas_pool_get_array(diag, 'uReconstructX', uReconstructX)
   call mpas_pool_get_array(diag, 'uReconstructY', uReconstructY)
   call mpas_pool_get_array(diag, 'uReconstructZ', uReconstructZ)
   call mpas_pool_get_array(diag, 'uReconstructZonal', uReconstructZonal)
   call mpas_pool_get_array(diag, 'uReconstructMeridional', uReconstructMeridional)
   call mpas_reconstruct(mesh, uu, uReconstructX, uReconstructY, uReconstructZ, uReconstructZonal, uReconstructMeridional)

   write(0, '(a)') 'harness: reconstruct done'
   if (any(dump_steps == 0)) call dump_all(trim(outdir)//'/step_0000', plist)

   call mpas_pool_get_config(configs, 'config_apply_lbcs', config_apply_lbcs)

   ! ---- time loop (mpas_atm_core.F:604-748 -> atm_do_timestep -> atm_timestep -> atm_srk3) ----
   allocate(steptime(max(nsteps,1)))
   call mpas_set_timeInterval(dtInterval, dt=dt)
   tloop = omp_get_wtime()
   do step = 1, nsteps
      t0 = omp_get_wtime()
      ! LBC_intv_end - the clock time at the step's start, as mpas_atm_get_bdy_state computes it
      harness_seconds_to_interval_end = lbc_interval_end - real(step - 1, RKIND) * dt
      call atm_timestep(domain, dt, nowTime, step)
      nowTime = nowTime + dtInterval
      t1 = omp_get_wtime()
      steptime(step) = t1 - t0
      if (step == 2) then   ! steady state: both time-level parities have run once
#ifdef MPAS_DYCORE_DROPIN
         call atm_dycore_wait()
#endif
         twarm = omp_get_wtime()
      end if
      write(0, '(a,i6,f10.3)') 'harness: step', step, steptime(step)
      call mpas_pool_shift_time_levels(state)
#ifdef MPAS_DYCORE_DROPIN
      if (any(dump_steps == step)) call atm_dycore_wait()   ! device time stays in the loop's time
#endif
      t2 = omp_get_wtime()   ! dumps are not part of the loop's time
      if (any(dump_steps == step)) then
         write(sdir, '(a,i4.4)') 'step_', step
#ifdef MPAS_DYCORE_DROPIN
         call atm_dycore_to_host(domain)   ! the HBM state into the pools before they are read
#endif
         call dump_all(trim(outdir)//'/'//trim(sdir), plist)
      end if
      tdumps = tdumps + (omp_get_wtime() - t2)
      if (step > 2) tdumps2 = tdumps2 + (omp_get_wtime() - t2)
   end do

#ifdef MPAS_DYCORE_DROPIN
   call atm_dycore_wait()   ! the steps run asynchronously: the loop ends when the device is done
#endif
   twarm = omp_get_wtime() - twarm - tdumps2
   tloop = omp_get_wtime() - tloop - tdumps
#ifdef MPAS_DYCORE_DROPIN
   call atm_dycore_to_host(domain)
#endif
   call execute_command_line('mkdir -p '//trim(outdir))
   open(newunit=u, file=trim(outdir)//'/timing.txt', status='replace')
   write(u, '(a,i6)') 'threads ', nthr
   do step = 1, nsteps
      write(u, '(a,i6,es24.16)') 'step ', step, steptime(step)
   end do
   write(u, '(a,es24.16)') 'total ', tloop
   if (nsteps > 2) write(u, '(a,es24.16)') 'after2 ', twarm   ! steps 3..nsteps
   close(u)

   call mpas_dmpar_finalize(domain % dminfo)

contains

   ! One block of the domain (mpas_block_creator.F does this for the real model): its dims,
   ! parinfo exchange lists, pools and fields.  nblocks > 1: inputs from <indir>/block<ib>/, whose
   ! block.nml holds the block dims and copy_<loc>_<layer>_<peer>.bin its local-copy lists.
   subroutine build_block(ib)
      integer, intent(in) :: ib
      character(len=16) :: bname
      type (block_type), pointer :: prevblk
      if (nblocks > 1) then
         write(bname, '(a,i0)') '/block', ib
         indir = trim(rootdir)//trim(bname)
         open(newunit=u, file=trim(indir)//'/block.nml', status='old')
         read(u, nml=block)
         close(u)
         nC1 = nCells + 1
         nE1 = nEdges + 1
         nV1 = nVertices + 1
      end if
      cur_nC1 = nC1
      cur_nE1 = nE1
      cur_nV1 = nV1
      prevblk => hblock
      allocate(hblock)
      hblock % blockID = ib
      hblock % localBlockID = ib
      hblock % domain => domain
      ! single block on one rank: every exchange list is empty (2 halo layers, no neighbours),
      ! so mpas_dmpar exchanges (incl. the explicit scale_arr exchange of
      ! atm_advance_scalars_mono_work, mpas_atm_time_integration.F:4084-4098) are no-ops.
      allocate(hblock % parinfo)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % cellsToSend, 2)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % cellsToRecv, 2)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % cellsToCopy, 2)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % edgesToSend, nhalo_ev)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % edgesToRecv, nhalo_ev)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % edgesToCopy, nhalo_ev)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % verticesToSend, nhalo_ev)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % verticesToRecv, nhalo_ev)
      call mpas_dmpar_init_multihalo_exchange_list(hblock % parinfo % verticesToCopy, nhalo_ev)
      if (ib == 0) then
         domain % blocklist => hblock
      else
         prevblk % next => hblock
         hblock % prev => prevblk
      end if
      call mpas_pool_create_pool(hblock % structs)
      call mpas_pool_create_pool(hblock % dimensions)
      hblock % configs => configs
      ! ---- subpools ----
      call mpas_pool_create_pool(mesh)
      call mpas_pool_create_pool(state)
      call mpas_pool_create_pool(diag)
      call mpas_pool_create_pool(tend)
      call mpas_pool_create_pool(tend_physics)
      call mpas_pool_create_pool(diag_physics)
      call mpas_pool_add_subpool(hblock % structs, 'mesh', mesh)
      call mpas_pool_add_subpool(hblock % structs, 'state', state)
      call mpas_pool_add_subpool(hblock % structs, 'diag', diag)
      call mpas_pool_add_subpool(hblock % structs, 'tend', tend)
      call mpas_pool_add_subpool(hblock % structs, 'tend_physics', tend_physics)
      ! empty: only the DO_PHYSICS build looks it up, for driver_microphysics (scheme 'off' -> unused)
      call mpas_pool_add_subpool(hblock % structs, 'diag_physics', diag_physics)
   
      call add_dims(hblock % dimensions)
      call add_dims(mesh)
      call add_dims(state)
      call add_dims(diag)
      call add_dims(tend)
      call add_dims(tend_physics)
      call mpas_pool_add_dimension(state, 'moist_start', 1)
      call mpas_pool_add_dimension(state, 'moist_end', moist_end)
      call mpas_pool_add_dimension(state, 'index_qv', 1)
      call mpas_pool_add_config_real(mesh, 'sphere_radius', sphere_radius)
      call mpas_pool_add_config_logical(mesh, 'on_a_sphere', .true.)
      call mpas_pool_add_config_logical(mesh, 'is_periodic', .false.)
      call mpas_pool_add_config_real(mesh, 'x_period', 0.0_RKIND)
      call mpas_pool_add_config_real(mesh, 'y_period', 0.0_RKIND)
   
      ! ---- thread ranges (replaces mpas_atm_threading.F; static contiguous blocks) ----
      call thread_ranges(nCells, cts, cte)
      call thread_ranges(nCells, csts, cste)
      call thread_ranges(nEdges, ets, ete)
      call thread_ranges(nEdges, ests, este)
      call thread_ranges(nVertices, vts, vte)
      call thread_ranges(nVertices, vsts, vste)
      call mpas_pool_add_dimension(hblock % dimensions, 'nThreads', nthr)
      call mpas_pool_add_dimension(hblock % dimensions, 'cellThreadStart', cts)
      call mpas_pool_add_dimension(hblock % dimensions, 'cellThreadEnd', cte)
      call mpas_pool_add_dimension(hblock % dimensions, 'cellSolveThreadStart', csts)
      call mpas_pool_add_dimension(hblock % dimensions, 'cellSolveThreadEnd', cste)
      call mpas_pool_add_dimension(hblock % dimensions, 'edgeThreadStart', ets)
      call mpas_pool_add_dimension(hblock % dimensions, 'edgeThreadEnd', ete)
      call mpas_pool_add_dimension(hblock % dimensions, 'edgeSolveThreadStart', ests)
      call mpas_pool_add_dimension(hblock % dimensions, 'edgeSolveThreadEnd', este)
      call mpas_pool_add_dimension(hblock % dimensions, 'vertexThreadStart', vts)
      call mpas_pool_add_dimension(hblock % dimensions, 'vertexThreadEnd', vte)
      call mpas_pool_add_dimension(hblock % dimensions, 'vertexSolveThreadStart', vsts)
      call mpas_pool_add_dimension(hblock % dimensions, 'vertexSolveThreadEnd', vste)
   
      ! ---- mesh pool (Registry.xml var_struct "mesh") ----
      call add_r1(mesh, 'mesh', 'latCell', nC1);  call add_r1(mesh, 'mesh', 'lonCell', nC1)
      call add_r1(mesh, 'mesh', 'xCell', nC1);    call add_r1(mesh, 'mesh', 'yCell', nC1)
      call add_r1(mesh, 'mesh', 'zCell', nC1);    call add_r1(mesh, 'mesh', 'areaCell', nC1)
      call add_r1(mesh, 'mesh', 'invAreaCell', nC1); call add_r1(mesh, 'mesh', 'meshDensity', nC1)
      call add_r1(mesh, 'mesh', 'meshScalingRegionalCell', nC1); call add_r1(mesh, 'mesh', 'specZoneMaskCell', nC1)
      call add_r1(mesh, 'mesh', 'latEdge', nE1);  call add_r1(mesh, 'mesh', 'lonEdge', nE1)
      call add_r1(mesh, 'mesh', 'xEdge', nE1);    call add_r1(mesh, 'mesh', 'yEdge', nE1)
      call add_r1(mesh, 'mesh', 'zEdge', nE1);    call add_r1(mesh, 'mesh', 'dcEdge', nE1)
      call add_r1(mesh, 'mesh', 'dvEdge', nE1);   call add_r1(mesh, 'mesh', 'invDcEdge', nE1)
      call add_r1(mesh, 'mesh', 'invDvEdge', nE1); call add_r1(mesh, 'mesh', 'angleEdge', nE1)
      call add_r1(mesh, 'mesh', 'fEdge', nE1);    call add_r1(mesh, 'mesh', 'meshScalingDel2', nE1)
      call add_r1(mesh, 'mesh', 'meshScalingDel4', nE1); call add_r1(mesh, 'mesh', 'meshScalingRegionalEdge', nE1)
      call add_r1(mesh, 'mesh', 'specZoneMaskEdge', nE1)
      call add_r1(mesh, 'mesh', 'latVertex', nV1); call add_r1(mesh, 'mesh', 'lonVertex', nV1)
      call add_r1(mesh, 'mesh', 'xVertex', nV1);  call add_r1(mesh, 'mesh', 'yVertex', nV1)
      call add_r1(mesh, 'mesh', 'zVertex', nV1);  call add_r1(mesh, 'mesh', 'areaTriangle', nV1)
      call add_r1(mesh, 'mesh', 'invAreaTriangle', nV1); call add_r1(mesh, 'mesh', 'fVertex', nV1)
      call add_r1(mesh, 'mesh', 'fzm', K);  call add_r1(mesh, 'mesh', 'fzp', K)
      call add_r1(mesh, 'mesh', 'rdzw', K); call add_r1(mesh, 'mesh', 'rdzu', K)
      call add_r1(mesh, 'mesh', 'u_init', K); call add_r1(mesh, 'mesh', 'v_init', K)
      call add_r1(mesh, 'mesh', 'qv_init', K)
      call add_r0(mesh, 'mesh', 'cf1'); call add_r0(mesh, 'mesh', 'cf2'); call add_r0(mesh, 'mesh', 'cf3')
      call add_i1(mesh, 'mesh', 'nEdgesOnCell', nC1); call add_i1(mesh, 'mesh', 'indexToCellID', nC1)
      call add_i1(mesh, 'mesh', 'bdyMaskCell', nC1);  call add_i1(mesh, 'mesh', 'nearestRelaxationCell', nC1)
      call add_i1(mesh, 'mesh', 'nEdgesOnEdge', nE1); call add_i1(mesh, 'mesh', 'nAdvCellsForEdge', nE1)
      call add_i1(mesh, 'mesh', 'bdyMaskEdge', nE1)
      call add_i2(mesh, 'mesh', 'edgesOnCell', maxEdges_in, nC1)
      call add_i2(mesh, 'mesh', 'cellsOnCell', maxEdges_in, nC1)
      call add_i2(mesh, 'mesh', 'verticesOnCell', maxEdges_in, nC1)
      call add_i2(mesh, 'mesh', 'kiteForCell', maxEdges_in, nC1)
      call add_i2(mesh, 'mesh', 'cellsOnEdge', 2, nE1)
      call add_i2(mesh, 'mesh', 'verticesOnEdge', 2, nE1)
      call add_i2(mesh, 'mesh', 'edgesOnEdge', maxEdges2_in, nE1)
      call add_i2(mesh, 'mesh', 'advCellsForEdge', 15, nE1)
      call add_i2(mesh, 'mesh', 'cellsOnVertex', 3, nV1)
      call add_i2(mesh, 'mesh', 'edgesOnVertex', 3, nV1)
      call add_r2(mesh, 'mesh', 'edgesOnCell_sign', maxEdges_in, nC1, 1)
      call add_r2(mesh, 'mesh', 'edgesOnVertex_sign', 3, nV1, 1)
      call add_r2(mesh, 'mesh', 'kiteAreasOnVertex', 3, nV1, 1)
      call add_r2(mesh, 'mesh', 'weightsOnEdge', maxEdges2_in, nE1, 1)
      call add_r2(mesh, 'mesh', 'adv_coefs', 15, nE1, 1)
      call add_r2(mesh, 'mesh', 'adv_coefs_3rd', 15, nE1, 1)
      call add_r2(mesh, 'mesh', 'defc_a', maxEdges_in, nC1, 1)
      call add_r2(mesh, 'mesh', 'defc_b', maxEdges_in, nC1, 1)
      call add_r2(mesh, 'mesh', 'zgrid', K+1, nC1, 1)
      call add_r2(mesh, 'mesh', 'hx', K+1, nC1, 1)       ! terrain height (the JW init's own use)
      call add_r1(mesh, 'mesh', 'dzu', K)
      call add_r2(mesh, 'mesh', 'zz', K, nC1, 1)
      call add_r2(mesh, 'mesh', 'zxu', K, nE1, 1)
      call add_r2(mesh, 'mesh', 'dss', K, nC1, 1)
      call add_r2(mesh, 'mesh', 't_init', K, nC1, 1)
      call add_r2(mesh, 'mesh', 'localVerticalUnitVectors', 3, nC1, 1)
      call add_r2(mesh, 'mesh', 'edgeNormalVectors', 3, nE1, 1)
      call add_r3(mesh, 'mesh', 'cellTangentPlane', 3, 2, nC1, 1)
      call add_r3(mesh, 'mesh', 'coeffs_reconstruct', 3, maxEdges_in, nC1, 1)
      call add_r3(mesh, 'mesh', 'deriv_two', 15, 2, nE1, 1)
      call add_r3(mesh, 'mesh', 'zb', K+1, 2, nE1, 1)
      call add_r3(mesh, 'mesh', 'zb3', K+1, 2, nE1, 1)
      call add_r3(mesh, 'mesh', 'zb_cell', K+1, maxEdges_in, nC1, 1)
      call add_r3(mesh, 'mesh', 'zb3_cell', K+1, maxEdges_in, nC1, 1)
      call add_i2(mesh, 'mesh', 'advCells', 21, nC1)   ! core_init_atmosphere Registry (TWENTYONE nCells)
   
      write(0, '(a)') 'harness: mesh pool read'
      ! ---- state pool: 2 time levels (Registry.xml var_struct "state" time_levs="2") ----
      call add_r2(state, 'state', 'u', K, nE1, 2)
      call add_r2(state, 'state', 'w', K+1, nC1, 2)
      call add_r2(state, 'state', 'theta_m', K, nC1, 2)
      call add_r2(state, 'state', 'rho_zz', K, nC1, 2)
      call add_r3(state, 'state', 'scalars', ns, K, nC1, 2)
      call add_c0(state, 'state', 'xtime', 2, start_time)
      if (config_apply_lbcs_in) call add_lbc_pool()
   
      ! ---- diag pool ----
      call add_r2(diag, 'diag', 'theta', K, nC1, 1);        call add_r2(diag, 'diag', 'rho', K, nC1, 1)
      call add_r2(diag, 'diag', 'rho_base', K, nC1, 1);     call add_r2(diag, 'diag', 'theta_base', K, nC1, 1)
      call add_r2(diag, 'diag', 'rho_p', K, nC1, 1);        call add_r2(diag, 'diag', 'rho_p_save', K, nC1, 1)
      call add_r2(diag, 'diag', 'rho_pp', K, nC1, 1);       call add_r2(diag, 'diag', 'rho_zz_old_split', K, nC1, 1)
      call add_r2(diag, 'diag', 'rtheta_base', K, nC1, 1);  call add_r2(diag, 'diag', 'rtheta_p', K, nC1, 1)
      call add_r2(diag, 'diag', 'rtheta_p_save', K, nC1, 1); call add_r2(diag, 'diag', 'rtheta_pp', K, nC1, 1)
      call add_r2(diag, 'diag', 'rtheta_pp_old', K, nC1, 1); call add_r2(diag, 'diag', 'exner', K, nC1, 1)
      call add_r2(diag, 'diag', 'exner_base', K, nC1, 1);   call add_r2(diag, 'diag', 'pressure_base', K, nC1, 1)
      call add_r2(diag, 'diag', 'pressure_p', K, nC1, 1);   call add_r2(diag, 'diag', 'h_divergence', K, nC1, 1)
      call add_r2(diag, 'diag', 'kdiff', K, nC1, 1);        call add_r2(diag, 'diag', 'ke', K, nC1, 1)
      call add_r2(diag, 'diag', 'divergence', K, nC1, 1);   call add_r2(diag, 'diag', 'pv_cell', K, nC1, 1)
      call add_r2(diag, 'diag', 'tend_rtheta_adv', K, nC1, 1); call add_r2(diag, 'diag', 'cqw', K, nC1, 1)
      call add_r2(diag, 'diag', 'cofwr', K, nC1, 1);        call add_r2(diag, 'diag', 'cofwz', K, nC1, 1)
      call add_r2(diag, 'diag', 'cofwt', K, nC1, 1);        call add_r2(diag, 'diag', 'coftz', K+1, nC1, 1)
      call add_r2(diag, 'diag', 'a_tri', K, nC1, 1);        call add_r2(diag, 'diag', 'alpha_tri', K, nC1, 1)
      call add_r2(diag, 'diag', 'gamma_tri', K, nC1, 1);    call add_r1(diag, 'diag', 'cofrz', K)
      call add_r2(diag, 'diag', 'uReconstructX', K, nC1, 1); call add_r2(diag, 'diag', 'uReconstructY', K, nC1, 1)
      call add_r2(diag, 'diag', 'uReconstructZ', K, nC1, 1); call add_r2(diag, 'diag', 'uReconstructZonal', K, nC1, 1)
      call add_r2(diag, 'diag', 'uReconstructMeridional', K, nC1, 1)
      call add_r2(diag, 'diag', 'rw', K+1, nC1, 1);         call add_r2(diag, 'diag', 'rw_p', K+1, nC1, 1)
      call add_r2(diag, 'diag', 'rw_save', K+1, nC1, 1);    call add_r2(diag, 'diag', 'wwAvg', K+1, nC1, 1)
      call add_r2(diag, 'diag', 'wwAvg_split', K+1, nC1, 1)
      call add_r2(diag, 'diag', 'ru', K, nE1, 1);           call add_r2(diag, 'diag', 'ruAvg', K, nE1, 1)
      call add_r2(diag, 'diag', 'ruAvg_split', K, nE1, 1);  call add_r2(diag, 'diag', 'ru_p', K, nE1, 1)
      call add_r2(diag, 'diag', 'ru_save', K, nE1, 1);      call add_r2(diag, 'diag', 'cqu', K, nE1, 1)
      call add_r2(diag, 'diag', 'rho_edge', K, nE1, 1);     call add_r2(diag, 'diag', 'v', K, nE1, 1)
      call add_r2(diag, 'diag', 'pv_edge', K, nE1, 1);      call add_r2(diag, 'diag', 'gradPVn', K, nE1, 1)
      call add_r2(diag, 'diag', 'gradPVt', K, nE1, 1)
      call add_r2(diag, 'diag', 'vorticity', K, nV1, 1);    call add_r2(diag, 'diag', 'pv_vertex', K, nV1, 1)
      call add_r1(diag, 'diag', 'surface_pressure', nC1)
   
      ! ---- tend / tend_physics pools ----
      call add_r2(tend, 'tend', 'u', K, nE1, 1);            call add_r2(tend, 'tend', 'u_euler', K, nE1, 1)
      call add_r2(tend, 'tend', 'w', K+1, nC1, 1);          call add_r2(tend, 'tend', 'w_euler', K+1, nC1, 1)
      call add_r2(tend, 'tend', 'w_pgf', K+1, nC1, 1);      call add_r2(tend, 'tend', 'w_buoy', K+1, nC1, 1)
      call add_r2(tend, 'tend', 'theta_m', K, nC1, 1);      call add_r2(tend, 'tend', 'theta_euler', K, nC1, 1)
      call add_r2(tend, 'tend', 'rho_zz', K, nC1, 1);       call add_r2(tend, 'tend', 'rt_diabatic_tend', K, nC1, 1)
      call add_r3(tend, 'tend', 'scalars_tend', ns, K, nC1, 1)
      call add_r2(tend_physics, 'tend_physics', 'rthdynten', K, nC1, 1)
      call add_r2(tend_physics, 'tend_physics', 'rqvdynten', K, nC1, 1)
      ! prescribed physics tendencies, handed to the DO_PHYSICS dycore by the physics_get_tend test
      ! double (shims/mpas_atmphys_todynamics_stub.F90); shapes as allocated in atm_srk3
      if (file_exists('tend_ru_physics_in')) then
         call add_r2(tend_physics, 'tend_physics', 'tend_ru_physics_in', K, nE1, 1)
         call add_r2(tend_physics, 'tend_physics', 'tend_rtheta_physics_in', K, nC1, 1)
         call add_r2(tend_physics, 'tend_physics', 'tend_rho_physics_in', K, nC1, 1)
         call add_r3(tend_physics, 'tend_physics', 'scalars_tend_in', ns, K, nC1, 1)
      end if
      if (nblocks > 1) call read_copy_lists()
      registering = .false.
   end subroutine build_block

   ! the local-copy exchange lists of this block (mpas_dmpar exchList: endPointID = destination
   ! localBlockID, srcList = owned local indices here, destList = halo local indices there)
   subroutine read_copy_lists()
      character(len=8), dimension(3), parameter :: locs = [character(len=8) :: 'cell', 'edge', 'vertex']
      integer :: il, layer, peer, nb, uu2
      logical :: ex
      character(len=320) :: fn
      type (mpas_multihalo_exchange_list), pointer :: ml
      type (mpas_exchange_list), pointer :: node, tail
      do il = 1, 3
         if (il == 1) ml => hblock % parinfo % cellsToCopy
         if (il == 2) ml => hblock % parinfo % edgesToCopy
         if (il == 3) ml => hblock % parinfo % verticesToCopy
         do layer = 1, size(ml % halos)
            do peer = 0, nblocks - 1
               write(fn, '(a,a,i0,a,i0,a)') trim(indir)//'/copy_'//trim(locs(il)), '_', layer, '_', peer, '.bin'
               inquire(file=trim(fn), exist=ex, size=nb)
               if (.not. ex) cycle
               allocate(node)
               node % endPointID = peer
               node % nlist = nb / 8
               allocate(node % srcList(node % nlist), node % destList(node % nlist))
               nullify(node % next)
               open(newunit=uu2, file=trim(fn), access='stream', form='unformatted', status='old')
               read(uu2) node % srcList, node % destList
               close(uu2)
               if (.not. associated(ml % halos(layer) % exchList)) then
                  ml % halos(layer) % exchList => node
               else
                  tail => ml % halos(layer) % exchList
                  do while (associated(tail % next))
                     tail => tail % next
                  end do
                  tail % next => node
               end if
            end do
         end do
      end do
   end subroutine read_copy_lists

   ! the block list as mpas_block_creator_finalize_block_phase1 leaves it: every field linked to the
   ! same field of the neighbouring blocks, and to its block's exchange lists
   subroutine link_blocks()
      type (block_type), pointer :: b
      b => domain % blocklist
      do while (associated(b))
         if (associated(b % prev) .and. associated(b % next)) then
            call mpas_pool_link_pools(b % structs, b % prev % structs, b % next % structs)
         else if (associated(b % prev)) then
            call mpas_pool_link_pools(b % structs, b % prev % structs)
         else if (associated(b % next)) then
            call mpas_pool_link_pools(b % structs, nextPool=b % next % structs)
         else
            call mpas_pool_link_pools(b % structs)
         end if
         call mpas_pool_link_parinfo(b, b % structs)
         b => b % next
      end do
   end subroutine link_blocks

   ! atm_mpas_init_block's diagnostics (mpas_atm_core.F:365-421) on one block of a multi-block run
   subroutine init_block(b)
      type (block_type), pointer :: b
      type (mpas_pool_type), pointer :: bm, bs, bd
      integer, pointer :: nC, nE, nV, bnthr
      integer, dimension(:), pointer :: a_cts, a_cte, a_csts, a_cste, a_ets, a_ete, a_ests, a_este, &
                                        a_vts, a_vte, a_vsts, a_vste
      call mpas_pool_get_subpool(b % structs, 'mesh', bm)
      call mpas_pool_get_subpool(b % structs, 'state', bs)
      call mpas_pool_get_subpool(b % structs, 'diag', bd)
      call mpas_pool_get_dimension(bm, 'nCells', nC)
      call mpas_pool_get_dimension(bm, 'nEdges', nE)
      call mpas_pool_get_dimension(bm, 'nVertices', nV)
      call mpas_pool_get_dimension(b % dimensions, 'nThreads', bnthr)
      call mpas_pool_get_dimension(b % dimensions, 'cellThreadStart', a_cts)
      call mpas_pool_get_dimension(b % dimensions, 'cellThreadEnd', a_cte)
      call mpas_pool_get_dimension(b % dimensions, 'cellSolveThreadStart', a_csts)
      call mpas_pool_get_dimension(b % dimensions, 'cellSolveThreadEnd', a_cste)
      call mpas_pool_get_dimension(b % dimensions, 'edgeThreadStart', a_ets)
      call mpas_pool_get_dimension(b % dimensions, 'edgeThreadEnd', a_ete)
      call mpas_pool_get_dimension(b % dimensions, 'edgeSolveThreadStart', a_ests)
      call mpas_pool_get_dimension(b % dimensions, 'edgeSolveThreadEnd', a_este)
      call mpas_pool_get_dimension(b % dimensions, 'vertexThreadStart', a_vts)
      call mpas_pool_get_dimension(b % dimensions, 'vertexThreadEnd', a_vte)
      call mpas_pool_get_dimension(b % dimensions, 'vertexSolveThreadStart', a_vsts)
      call mpas_pool_get_dimension(b % dimensions, 'vertexSolveThreadEnd', a_vste)
      allocate(ke_vertex(K, nV + 1))
      ke_vertex(:, nV + 1) = 0.0_RKIND
      allocate(ke_edge(K, nE + 1))
      ke_edge(:, nE + 1) = 0.0_RKIND
!$OMP PARALLEL DO
      do t = 1, bnthr
         call atm_init_coupled_diagnostics(bs, 1, bd, bm, configs, a_cts(t), a_cte(t), a_vts(t), a_vte(t), &
                                           a_ets(t), a_ete(t), a_csts(t), a_cste(t), a_vsts(t), a_vste(t), &
                                           a_ests(t), a_este(t))
         call atm_compute_solve_diagnostics(dt, bs, 1, bd, bm, configs, a_cts(t), a_cte(t), a_vts(t), a_vte(t), &
                                            a_ets(t), a_ete(t))
      end do
!$OMP END PARALLEL DO
      deallocate(ke_vertex)
      deallocate(ke_edge)
      call mpas_rbf_interp_initialize(bm)
      call mpas_init_reconstruct(bm)
      call mpas_pool_get_array(bs, 'u', uu, 1)
      call mpas_pool_get_array(bd, 'uReconstructX', uReconstructX)
      call mpas_pool_get_array(bd, 'uReconstructY', uReconstructY)
      call mpas_pool_get_array(bd, 'uReconstructZ', uReconstructZ)
      call mpas_pool_get_array(bd, 'uReconstructZonal', uReconstructZonal)
      call mpas_pool_get_array(bd, 'uReconstructMeridional', uReconstructMeridional)
      call mpas_reconstruct(bm, uu, uReconstructX, uReconstructY, uReconstructZ, uReconstructZonal, &
                            uReconstructMeridional)
   end subroutine init_block

   ! every block's pools into <dir>/block<i>
   subroutine dump_blocks(dir)
      character(len=*), intent(in) :: dir
      character(len=16) :: bname
      type (block_type), pointer :: b
      b => domain % blocklist
      do while (associated(b))
         hblock => b
         write(bname, '(a,i0)') '/block', b % localBlockID
         call dump_all(trim(dir)//trim(bname), plist)
         b => b % next
      end do
   end subroutine dump_blocks

   ! regional runs: the lbc pool the reference's mpas_atm_boundaries reads (lbc_<field>, time level
   ! 1 = tendency, 2 = interval-end state; lbc.lbc_<field>.tl<N>.bin inputs) and the moist species
   ! indices srk3 looks up (state and lbc pools; 0 = absent species)
   subroutine add_lbc_pool()
      type (mpas_pool_type), pointer :: lbc
      character(len=8), dimension(8), parameter :: sp = ['qv', 'qc', 'qr', 'qi', 'qs', 'qg', 'nr', 'ni']
      integer :: j
      call mpas_pool_create_pool(lbc)
      call mpas_pool_add_subpool(hblock % structs, 'lbc', lbc)
      call add_r2(lbc, 'lbc', 'lbc_u', K, nE1, 2)
      call add_r2(lbc, 'lbc', 'lbc_ru', K, nE1, 2)
      call add_r2(lbc, 'lbc', 'lbc_rho_zz', K, nC1, 2)
      call add_r2(lbc, 'lbc', 'lbc_rtheta_m', K, nC1, 2)
      call add_r3(lbc, 'lbc', 'lbc_scalars', ns, K, nC1, 2)
      do j = 1, size(sp)
         call mpas_pool_add_dimension(lbc, 'index_'//trim(sp(j)), merge(j, 0, j <= moist_end))
         if (j > 1) call mpas_pool_add_dimension(state, 'index_'//trim(sp(j)), merge(j, 0, j <= moist_end))
      end do
   end subroutine add_lbc_pool

   subroutine add_dims(p)
      type (mpas_pool_type), pointer :: p
      call mpas_pool_add_dimension(p, 'nCells', nCells)
      call mpas_pool_add_dimension(p, 'nEdges', nEdges)
      call mpas_pool_add_dimension(p, 'nVertices', nVertices)
      call mpas_pool_add_dimension(p, 'nCellsSolve', nCellsSolve_in)
      call mpas_pool_add_dimension(p, 'nEdgesSolve', nEdgesSolve_in)
      call mpas_pool_add_dimension(p, 'nVerticesSolve', nVerticesSolve_in)
      call mpas_pool_add_dimension(p, 'nVertLevels', K)
      call mpas_pool_add_dimension(p, 'nVertLevelsP1', K+1)
      call mpas_pool_add_dimension(p, 'maxEdges', maxEdges_in)
      call mpas_pool_add_dimension(p, 'maxEdges2', maxEdges2_in)
      call mpas_pool_add_dimension(p, 'vertexDegree', 3)
      call mpas_pool_add_dimension(p, 'num_scalars', ns)
   end subroutine add_dims

   subroutine thread_ranges(n, s, e)
      integer, intent(in) :: n
      integer, dimension(:), pointer :: s, e
      integer :: i
      allocate(s(nthr), e(nthr))
      do i = 1, nthr
         s(i) = (i-1) * n / nthr + 1
         e(i) = i * n / nthr
      end do
   end subroutine thread_ranges

end program mpas_ref_harness
