! atm_time_integration_mi355x.F90 -- drop-in replacement of the MPAS-Atmosphere
! dycore module `atm_time_integration`
! (src/core_atmosphere/dynamics/mpas_atm_time_integration.F) that runs the time
! step on an MI355X through the C ABI of libmpas_dycore.so (include/mpas_dycore.h).
!
! The module keeps the reference's module name, its public routines and its
! public module variables, so callers compile unchanged:
!   * the routines are atm_timestep, atm_srk3, atm_init_coupled_diagnostics and
!     atm_compute_solve_diagnostics;
!   * the variables are ke_vertex, ke_edge and config_apply_lbcs;
!   * the callers are mpas_atm_core.F and the oracle harness.
! Build it against the MPAS framework modules instead of mpas_atm_time_integration.F
! and link -lmpas_dycore (INTEGRATION.md).
!
! Data flow follows mpas_atm_core.F:
!   * The first atm_compute_solve_diagnostics call (model init, :399) creates the
!     device context. It uploads the mesh / state / diag pool arrays, which are
!     the pools' own (K, n+1) memory images, and runs init diagnostics on the GPU.
!   * atm_srk3 / atm_timestep advance the HBM-resident state. They then copy the
!     prognostics and the cell-centre velocity back into time level 2 of the host
!     pools, where the caller's mpas_pool_shift_time_levels (mpas_atm_core.F:671)
!     expects them.
module atm_time_integration

   use iso_c_binding
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types

   implicit none

   ! module variables the reference exports (mpas_atm_time_integration.F:66-69)
   real (kind=RKIND), allocatable, dimension(:,:) :: ke_vertex
   real (kind=RKIND), allocatable, dimension(:,:) :: ke_edge
   logical, pointer :: config_apply_lbcs

   type, bind(C) :: dyc_dims
      integer(c_int32_t) :: nCells, nEdges, nVertices, nVertLevels, maxEdges, maxEdges2, num_scalars
      integer(c_int32_t) :: nCellsSolve, nEdgesSolve, nVerticesSolve, moist_start, moist_end, index_qv
   end type dyc_dims

   type, bind(C) :: dyc_config   ! field order == mpas_dyc_config in include/mpas_dycore.h
      integer(c_int32_t) :: time_integration_order, number_of_sub_steps, dynamics_split_steps
      integer(c_int32_t) :: number_rayleigh_damp_u_levels, split_dynamics_transport, scalar_advection
      integer(c_int32_t) :: positive_definite, monotonic, mix_full, rayleigh_damp_u, horiz_mixing
      real(c_double) :: h_mom_eddy_visc2, h_mom_eddy_visc4, v_mom_eddy_visc2
      real(c_double) :: h_theta_eddy_visc2, h_theta_eddy_visc4, v_theta_eddy_visc2
      real(c_double) :: len_disp, visc4_2dsmag, del4u_div_factor, coef_3rd_order
      real(c_double) :: smagorinsky_coef, epssm, smdiv, apvm_upwinding
      real(c_double) :: mpas_cam_coef, rayleigh_damp_u_timescale_days
   end type dyc_config

   interface
      integer(c_int) function mpas_dyc_create(dims, cfg, device, ctx) bind(C, name='mpas_dyc_create')
         import :: c_int, c_ptr, dyc_dims, dyc_config
         type(dyc_dims), intent(in) :: dims
         type(dyc_config), intent(in) :: cfg
         integer(c_int), value :: device
         type(c_ptr), intent(out) :: ctx
      end function
      integer(c_int) function mpas_dyc_set_field(ctx, pool, name, tl, host, nbytes) bind(C, name='mpas_dyc_set_field')
         import :: c_int, c_ptr, c_char, c_int32_t, c_int64_t
         type(c_ptr), value :: ctx
         character(kind=c_char), dimension(*), intent(in) :: pool, name
         integer(c_int32_t), value :: tl
         type(c_ptr), value :: host
         integer(c_int64_t), value :: nbytes
      end function
      integer(c_int) function mpas_dyc_get_field(ctx, pool, name, tl, host, nbytes) bind(C, name='mpas_dyc_get_field')
         import :: c_int, c_ptr, c_char, c_int32_t, c_int64_t
         type(c_ptr), value :: ctx
         character(kind=c_char), dimension(*), intent(in) :: pool, name
         integer(c_int32_t), value :: tl
         type(c_ptr), value :: host
         integer(c_int64_t), value :: nbytes
      end function
      integer(c_int) function mpas_dyc_init_diagnostics(ctx, dt) bind(C, name='mpas_dyc_init_diagnostics')
         import :: c_int, c_ptr, c_double
         type(c_ptr), value :: ctx
         real(c_double), value :: dt
      end function
      integer(c_int) function mpas_dyc_timestep(ctx, dt, itimestep) bind(C, name='mpas_dyc_timestep')
         import :: c_int, c_ptr, c_double, c_int32_t
         type(c_ptr), value :: ctx
         real(c_double), value :: dt
         integer(c_int32_t), value :: itimestep
      end function
      integer(c_int) function mpas_dyc_shift_time_levels(ctx) bind(C, name='mpas_dyc_shift_time_levels')
         import :: c_int, c_ptr
         type(c_ptr), value :: ctx
      end function
      integer(c_int) function mpas_dyc_use_graph(ctx, on) bind(C, name='mpas_dyc_use_graph')
         import :: c_int, c_ptr, c_int32_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: on
      end function
      type(c_ptr) function mpas_dyc_last_error(ctx) bind(C, name='mpas_dyc_last_error')
         import :: c_ptr
         type(c_ptr), value :: ctx
      end function
   end interface

   type(c_ptr), save, private :: dyc = c_null_ptr
   logical, save, private :: coeffs_ready = .false.

   private :: check, up_r0, up_r1, up_r2, up_r3, up_i1, up_i2, down_r2, down_r3, create_context

   contains

   ! atm_timestep (mpas_atm_time_integration.F:87-139): the reference only dispatches to
   ! atm_srk3 (and stamps xtime, which lives in the host pools untouched here)
   subroutine atm_timestep(domain, dt, nowTime, itimestep)
      type (domain_type), intent(inout) :: domain
      real (kind=RKIND), intent(in) :: dt
      type (MPAS_Time_type), intent(in) :: nowTime
      integer, intent(in) :: itimestep
      call atm_srk3(domain, dt, itimestep)
   end subroutine atm_timestep

   ! atm_srk3 (:142-1796) on the GPU; time level 2 of the host state pool receives the result
   subroutine atm_srk3(domain, dt, itimestep)
      type (domain_type), intent(inout) :: domain
      real (kind=RKIND), intent(in) :: dt
      integer, intent(in) :: itimestep
      type (mpas_pool_type), pointer :: mesh, state, diag
      call mpas_pool_get_subpool(domain % blocklist % structs, 'mesh', mesh)
      call mpas_pool_get_subpool(domain % blocklist % structs, 'state', state)
      call mpas_pool_get_subpool(domain % blocklist % structs, 'diag', diag)
      if (.not. c_associated(dyc)) call create_context(mesh, state, diag, domain % blocklist % configs)
      if (.not. coeffs_ready) then
         ! mpas_init_reconstruct runs on the host after the init diagnostics (mpas_atm_core.F:409)
         call up_r3(mesh, 'mesh', 'coeffs_reconstruct')
         coeffs_ready = .true.
      end if
      call check(mpas_dyc_timestep(dyc, real(dt, c_double), int(itimestep, c_int32_t)), 'mpas_dyc_timestep')
      ! the device swaps now; the caller swaps the host pools right after (mpas_atm_core.F:671),
      ! so the new state goes to host time level 2
      call check(mpas_dyc_shift_time_levels(dyc), 'mpas_dyc_shift_time_levels')
      call down_r2(state, 'state', 'u', 2, 1)
      call down_r2(state, 'state', 'w', 2, 1)
      call down_r2(state, 'state', 'theta_m', 2, 1)
      call down_r2(state, 'state', 'rho_zz', 2, 1)
      call down_r3(state, 'state', 'scalars', 2, 1)
      call down_r2(diag, 'diag', 'uReconstructX', 1, 1)
      call down_r2(diag, 'diag', 'uReconstructY', 1, 1)
      call down_r2(diag, 'diag', 'uReconstructZ', 1, 1)
      call down_r2(diag, 'diag', 'uReconstructZonal', 1, 1)
      call down_r2(diag, 'diag', 'uReconstructMeridional', 1, 1)
      call down_r2(diag, 'diag', 'pressure_p', 1, 1)
      call down_r2(diag, 'diag', 'exner', 1, 1)
   end subroutine atm_srk3

   ! atm_init_coupled_diagnostics (:5825): the core always calls it together with
   ! atm_compute_solve_diagnostics (mpas_atm_core.F:390-399); both run in one device call there
   subroutine atm_init_coupled_diagnostics(state, time_lev, diag, mesh, configs, &
                                           cellStart, cellEnd, vertexStart, vertexEnd, edgeStart, edgeEnd, &
                                           cellSolveStart, cellSolveEnd, vertexSolveStart, vertexSolveEnd, &
                                           edgeSolveStart, edgeSolveEnd)
      type (mpas_pool_type), intent(inout) :: state
      integer, intent(in) :: time_lev
      type (mpas_pool_type), intent(inout) :: diag
      type (mpas_pool_type), intent(inout) :: mesh
      type (mpas_pool_type), intent(in) :: configs
      integer, intent(in) :: cellStart, cellEnd, vertexStart, vertexEnd, edgeStart, edgeEnd
      integer, intent(in) :: cellSolveStart, cellSolveEnd, vertexSolveStart, vertexSolveEnd, edgeSolveStart, edgeSolveEnd
   end subroutine atm_init_coupled_diagnostics

   ! atm_compute_solve_diagnostics (:5419) at model init: create the context, upload the pools,
   ! run atm_init_coupled_diagnostics + atm_compute_solve_diagnostics on the device and copy the
   ! coupled state and diagnostics back
   subroutine atm_compute_solve_diagnostics(dt, state, time_lev, diag, mesh, configs, &
                                            cellStart, cellEnd, vertexStart, vertexEnd, edgeStart, edgeEnd, &
                                            rk_step)
      real (kind=RKIND), intent(in) :: dt
      type (mpas_pool_type), intent(inout) :: state
      integer, intent(in) :: time_lev
      type (mpas_pool_type), intent(inout) :: diag
      type (mpas_pool_type), intent(in) :: mesh
      type (mpas_pool_type), intent(in) :: configs
      integer, intent(in) :: cellStart, cellEnd, vertexStart, vertexEnd, edgeStart, edgeEnd
      integer, intent(in), optional :: rk_step
      if (c_associated(dyc)) return
      call create_context(mesh, state, diag, configs)
      call check(mpas_dyc_init_diagnostics(dyc, real(dt, c_double)), 'mpas_dyc_init_diagnostics')
      call down_r2(state, 'state', 'theta_m', 1, 1)
      call down_r2(state, 'state', 'rho_zz', 1, 1)
      call down_r2(diag, 'diag', 'ru', 1, 1)
      call down_r2(diag, 'diag', 'rw', 1, 1)
      call down_r2(diag, 'diag', 'pv_edge', 1, 1)
      call down_r2(diag, 'diag', 'exner', 1, 1)
      call down_r2(diag, 'diag', 'pressure_p', 1, 1)
   end subroutine atm_compute_solve_diagnostics

   ! The harness's single-sub-step kernel mode calls these two srk3 internals directly
   ! (:2312, :2726).  On the device they are fused into the time step, and no caller of the
   ! module's public API (mpas_atm_core.F) calls them, so the drop-in stops here.
   ! Acoustic-kernel parity is covered by tests/test_gpu_kernels.py through the C ABI.
   subroutine atm_advance_acoustic_step(state, diag, tend, mesh, configs, nCells, nVertLevels, dts, small_step, &
                                        cellStart, cellEnd, vertexStart, vertexEnd, edgeStart, edgeEnd, &
                                        cellSolveStart, cellSolveEnd, vertexSolveStart, vertexSolveEnd, &
                                        edgeSolveStart, edgeSolveEnd)
      type (mpas_pool_type), intent(inout) :: state, diag, tend, mesh
      type (mpas_pool_type), intent(in) :: configs
      integer, intent(in) :: nCells, nVertLevels, small_step
      real (kind=RKIND), intent(in) :: dts
      integer, intent(in) :: cellStart, cellEnd, vertexStart, vertexEnd, edgeStart, edgeEnd
      integer, intent(in) :: cellSolveStart, cellSolveEnd, vertexSolveStart, vertexSolveEnd, edgeSolveStart, edgeSolveEnd
      write(0, '(a)') 'MI355X dycore: atm_advance_acoustic_step is internal to mpas_dyc_timestep'
      error stop 1
   end subroutine atm_advance_acoustic_step

   subroutine atm_divergence_damping_3d(state, diag, mesh, configs, dts, edgeStart, edgeEnd)
      type (mpas_pool_type), intent(inout) :: state, diag, mesh
      type (mpas_pool_type), intent(in) :: configs
      real (kind=RKIND), intent(in) :: dts
      integer, intent(in) :: edgeStart, edgeEnd
      write(0, '(a)') 'MI355X dycore: atm_divergence_damping_3d is internal to mpas_dyc_timestep'
      error stop 1
   end subroutine atm_divergence_damping_3d

   subroutine create_context(mesh, state, diag, configs)
      type (mpas_pool_type), intent(in) :: mesh, state, diag
      type (mpas_pool_type), intent(in) :: configs
      type(dyc_dims) :: d
      type(dyc_config) :: c
      integer, pointer :: ip
      real (kind=RKIND), pointer :: rp
      logical, pointer :: lp
      character(len=StrKIND), pointer :: sp
      integer :: i
      character(len=32), dimension(3), parameter :: i1_names = [character(len=32) :: &
         'nEdgesOnCell', 'nEdgesOnEdge', 'nAdvCellsForEdge']
      character(len=32), dimension(10), parameter :: i2_names = [character(len=32) :: &
         'edgesOnCell', 'cellsOnCell', 'verticesOnCell', 'kiteForCell', 'cellsOnEdge', 'verticesOnEdge', &
         'edgesOnEdge', 'advCellsForEdge', 'cellsOnVertex', 'edgesOnVertex']
      character(len=32), dimension(17), parameter :: r1_names = [character(len=32) :: &
         'dcEdge', 'dvEdge', 'invDcEdge', 'invDvEdge', 'fEdge', 'meshScalingDel2', 'meshScalingDel4', &
         'specZoneMaskEdge', 'angleEdge', 'invAreaCell', 'specZoneMaskCell', 'latCell', 'lonCell', &
         'invAreaTriangle', 'fVertex', 'u_init', 'v_init']
      character(len=32), dimension(4), parameter :: v_names = [character(len=32) :: 'fzm', 'fzp', 'rdzw', 'rdzu']
      character(len=32), dimension(13), parameter :: r2_names = [character(len=32) :: &
         'edgesOnCell_sign', 'edgesOnVertex_sign', 'kiteAreasOnVertex', 'weightsOnEdge', 'adv_coefs', &
         'adv_coefs_3rd', 'defc_a', 'defc_b', 'zgrid', 'zz', 'zxu', 'dss', 't_init']

      call mpas_pool_get_dimension(mesh, 'nCells', ip);         d % nCells = ip
      call mpas_pool_get_dimension(mesh, 'nEdges', ip);         d % nEdges = ip
      call mpas_pool_get_dimension(mesh, 'nVertices', ip);      d % nVertices = ip
      call mpas_pool_get_dimension(mesh, 'nVertLevels', ip);    d % nVertLevels = ip
      call mpas_pool_get_dimension(mesh, 'maxEdges', ip);       d % maxEdges = ip
      call mpas_pool_get_dimension(mesh, 'maxEdges2', ip);      d % maxEdges2 = ip
      call mpas_pool_get_dimension(state, 'num_scalars', ip);   d % num_scalars = ip
      call mpas_pool_get_dimension(mesh, 'nCellsSolve', ip);    d % nCellsSolve = ip
      call mpas_pool_get_dimension(mesh, 'nEdgesSolve', ip);    d % nEdgesSolve = ip
      call mpas_pool_get_dimension(mesh, 'nVerticesSolve', ip); d % nVerticesSolve = ip
      call mpas_pool_get_dimension(state, 'moist_start', ip);   d % moist_start = ip
      call mpas_pool_get_dimension(state, 'moist_end', ip);     d % moist_end = ip
      call mpas_pool_get_dimension(state, 'index_qv', ip);      d % index_qv = ip

      call mpas_pool_get_config(configs, 'config_time_integration_order', ip);     c % time_integration_order = ip
      call mpas_pool_get_config(configs, 'config_number_of_sub_steps', ip);        c % number_of_sub_steps = ip
      call mpas_pool_get_config(configs, 'config_dynamics_split_steps', ip);       c % dynamics_split_steps = ip
      call mpas_pool_get_config(configs, 'config_number_rayleigh_damp_u_levels', ip)
      c % number_rayleigh_damp_u_levels = ip
      call mpas_pool_get_config(configs, 'config_split_dynamics_transport', lp);   c % split_dynamics_transport = merge(1, 0, lp)
      call mpas_pool_get_config(configs, 'config_scalar_advection', lp);           c % scalar_advection = merge(1, 0, lp)
      call mpas_pool_get_config(configs, 'config_positive_definite', lp);          c % positive_definite = merge(1, 0, lp)
      call mpas_pool_get_config(configs, 'config_monotonic', lp);                  c % monotonic = merge(1, 0, lp)
      call mpas_pool_get_config(configs, 'config_mix_full', lp);                   c % mix_full = merge(1, 0, lp)
      call mpas_pool_get_config(configs, 'config_rayleigh_damp_u', lp);            c % rayleigh_damp_u = merge(1, 0, lp)
      call mpas_pool_get_config(configs, 'config_horiz_mixing', sp)
      c % horiz_mixing = merge(1, 0, trim(sp) == '2d_smagorinsky')
      call mpas_pool_get_config(configs, 'config_h_mom_eddy_visc2', rp);   c % h_mom_eddy_visc2 = rp
      call mpas_pool_get_config(configs, 'config_h_mom_eddy_visc4', rp);   c % h_mom_eddy_visc4 = rp
      call mpas_pool_get_config(configs, 'config_v_mom_eddy_visc2', rp);   c % v_mom_eddy_visc2 = rp
      call mpas_pool_get_config(configs, 'config_h_theta_eddy_visc2', rp); c % h_theta_eddy_visc2 = rp
      call mpas_pool_get_config(configs, 'config_h_theta_eddy_visc4', rp); c % h_theta_eddy_visc4 = rp
      call mpas_pool_get_config(configs, 'config_v_theta_eddy_visc2', rp); c % v_theta_eddy_visc2 = rp
      call mpas_pool_get_config(configs, 'config_len_disp', rp);           c % len_disp = rp
      call mpas_pool_get_config(configs, 'config_visc4_2dsmag', rp);       c % visc4_2dsmag = rp
      call mpas_pool_get_config(configs, 'config_del4u_div_factor', rp);   c % del4u_div_factor = rp
      call mpas_pool_get_config(configs, 'config_coef_3rd_order', rp);     c % coef_3rd_order = rp
      call mpas_pool_get_config(configs, 'config_smagorinsky_coef', rp);   c % smagorinsky_coef = rp
      call mpas_pool_get_config(configs, 'config_epssm', rp);              c % epssm = rp
      call mpas_pool_get_config(configs, 'config_smdiv', rp);              c % smdiv = rp
      call mpas_pool_get_config(configs, 'config_apvm_upwinding', rp);     c % apvm_upwinding = rp
      call mpas_pool_get_config(configs, 'config_mpas_cam_coef', rp);      c % mpas_cam_coef = rp
      call mpas_pool_get_config(configs, 'config_rayleigh_damp_u_timescale_days', rp)
      c % rayleigh_damp_u_timescale_days = rp

      call check(mpas_dyc_create(d, c, -1_c_int, dyc), 'mpas_dyc_create')
      call check(mpas_dyc_use_graph(dyc, 1_c_int32_t), 'mpas_dyc_use_graph')

      do i = 1, size(i1_names)
         call up_i1(mesh, 'mesh', trim(i1_names(i)))
      end do
      do i = 1, size(i2_names)
         call up_i2(mesh, 'mesh', trim(i2_names(i)))
      end do
      do i = 1, size(r1_names)
         call up_r1(mesh, 'mesh', trim(r1_names(i)))
      end do
      do i = 1, size(v_names)
         call up_r1(mesh, 'mesh', trim(v_names(i)))
      end do
      call up_r0(mesh, 'mesh', 'cf1'); call up_r0(mesh, 'mesh', 'cf2'); call up_r0(mesh, 'mesh', 'cf3')
      do i = 1, size(r2_names)
         call up_r2(mesh, 'mesh', trim(r2_names(i)), 1)
      end do
      call up_r3(mesh, 'mesh', 'zb_cell')
      call up_r3(mesh, 'mesh', 'zb3_cell')
      call up_r2(state, 'state', 'u', 1)
      call up_r2(state, 'state', 'w', 1)
      call up_r3(state, 'state', 'scalars', 1)
      call up_r2(diag, 'diag', 'theta', 1)
      call up_r2(diag, 'diag', 'rho', 1)
      call up_r2(diag, 'diag', 'rho_base', 1)
      call up_r2(diag, 'diag', 'theta_base', 1)
   end subroutine create_context

   ! ---- pool array <-> device field (the pools' own memory images, no repacking)
   subroutine up_r0(pool, pname, name)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      real (kind=RKIND), pointer :: a
      call mpas_pool_get_array(pool, name, a)
      if (.not. associated(a)) return
      call check(mpas_dyc_set_field(dyc, pname//c_null_char, name//c_null_char, 1_c_int32_t, c_loc(a), &
                                    int(8, c_int64_t)), 'set '//name)
   end subroutine up_r0

   subroutine up_r1(pool, pname, name)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      real (kind=RKIND), dimension(:), pointer :: a
      call mpas_pool_get_array(pool, name, a)
      if (.not. associated(a)) return
      call check(mpas_dyc_set_field(dyc, pname//c_null_char, name//c_null_char, 1_c_int32_t, c_loc(a(1)), &
                                    int(8, c_int64_t) * size(a, kind=c_int64_t)), 'set '//name)
   end subroutine up_r1

   subroutine up_r2(pool, pname, name, tl)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: tl
      real (kind=RKIND), dimension(:,:), pointer :: a
      call mpas_pool_get_array(pool, name, a, tl)
      if (.not. associated(a)) return
      call check(mpas_dyc_set_field(dyc, pname//c_null_char, name//c_null_char, int(tl, c_int32_t), c_loc(a(1,1)), &
                                    int(8, c_int64_t) * size(a, kind=c_int64_t)), 'set '//name)
   end subroutine up_r2

   subroutine up_r3(pool, pname, name, tl)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in), optional :: tl
      real (kind=RKIND), dimension(:,:,:), pointer :: a
      integer :: t
      t = 1
      if (present(tl)) t = tl
      call mpas_pool_get_array(pool, name, a, t)
      if (.not. associated(a)) return
      call check(mpas_dyc_set_field(dyc, pname//c_null_char, name//c_null_char, int(t, c_int32_t), c_loc(a(1,1,1)), &
                                    int(8, c_int64_t) * size(a, kind=c_int64_t)), 'set '//name)
   end subroutine up_r3

   subroutine up_i1(pool, pname, name)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      integer, dimension(:), pointer :: a
      call mpas_pool_get_array(pool, name, a)
      if (.not. associated(a)) return
      call check(mpas_dyc_set_field(dyc, pname//c_null_char, name//c_null_char, 1_c_int32_t, c_loc(a(1)), &
                                    int(4, c_int64_t) * size(a, kind=c_int64_t)), 'set '//name)
   end subroutine up_i1

   subroutine up_i2(pool, pname, name)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      integer, dimension(:,:), pointer :: a
      call mpas_pool_get_array(pool, name, a)
      if (.not. associated(a)) return
      call check(mpas_dyc_set_field(dyc, pname//c_null_char, name//c_null_char, 1_c_int32_t, c_loc(a(1,1)), &
                                    int(4, c_int64_t) * size(a, kind=c_int64_t)), 'set '//name)
   end subroutine up_i2

   subroutine down_r2(pool, pname, name, host_tl, dev_tl)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: host_tl, dev_tl
      real (kind=RKIND), dimension(:,:), pointer :: a
      call mpas_pool_get_array(pool, name, a, host_tl)
      if (.not. associated(a)) return
      call check(mpas_dyc_get_field(dyc, pname//c_null_char, name//c_null_char, int(dev_tl, c_int32_t), c_loc(a(1,1)), &
                                    int(8, c_int64_t) * size(a, kind=c_int64_t)), 'get '//name)
   end subroutine down_r2

   subroutine down_r3(pool, pname, name, host_tl, dev_tl)
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      integer, intent(in) :: host_tl, dev_tl
      real (kind=RKIND), dimension(:,:,:), pointer :: a
      call mpas_pool_get_array(pool, name, a, host_tl)
      if (.not. associated(a)) return
      call check(mpas_dyc_get_field(dyc, pname//c_null_char, name//c_null_char, int(dev_tl, c_int32_t), &
                                    c_loc(a(1,1,1)), int(8, c_int64_t) * size(a, kind=c_int64_t)), 'get '//name)
   end subroutine down_r3

   ! non-zero C ABI status -> fatal, as the reference's MPAS_LOG_CRIT path (mpas_log.F:612)
   subroutine check(ierr, what)
      integer(c_int), intent(in) :: ierr
      character(len=*), intent(in) :: what
      character(kind=c_char), pointer :: msg(:)
      character(len=512) :: text
      integer :: i
      if (ierr == 0) return
      text = ''
      call c_f_pointer(mpas_dyc_last_error(dyc), msg, [512])
      do i = 1, 512
         if (msg(i) == c_null_char) exit
         text(i:i) = msg(i)
      end do
      write(0, '(a,i0,a)') 'MI355X dycore: '//what//' failed (', ierr, '): '//trim(text)
      error stop 1
   end subroutine check

end module atm_time_integration
