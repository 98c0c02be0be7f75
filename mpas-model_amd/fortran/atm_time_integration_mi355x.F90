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
! and link -lmpas_dycore (INTEGRATION.md).  Built with -DDO_PHYSICS it also does the
! reference's physics hand-off around the step (physics_get_tend before, the
! rqvdynten / clip / microphysics tail after).
!
! Data flow follows mpas_atm_core.F:
!   * Model init (atm_mpas_init_block, mpas_atm_core.F:387-404) calls
!     atm_compute_solve_diagnostics once per block (per thread; the thread whose
!     range starts at cell 1 does the block's work).  A one-block device context
!     uploads the block's pools -- their own (K, n+1) memory images -- runs the init
!     diagnostics on the GPU and copies the results back, so the host's init-time
!     exchanges, mpas_reconstruct and initial output see them.
!   * The first atm_srk3 builds the context of the whole domain: every block of
!     domain%blocklist, its parinfo exchange lists (local copies between blocks of
!     this task, RCCL messages to other tasks), the RCCL communicator when there
!     are several MPI tasks, and the same model init on the device.
!   * atm_srk3 / atm_timestep then advance the HBM-resident state.  The host pools
!     are refreshed by atm_dycore_to_host(domain) -- before output and restart
!     writes -- or after every step when atm_dycore_sync_every_step is set (or
!     MPAS_DYCORE_SYNC_EVERY_STEP=1), and always in the DO_PHYSICS build, whose
!     host physics reads the state every step.
module atm_time_integration

   use iso_c_binding
   use mpas_derived_types
   use mpas_pool_routines
   use mpas_kind_types
   use mpas_dmpar
   use mpas_log
   use mpas_timekeeping
   use mpas_atm_boundaries, only : mpas_atm_get_bdy_state
#ifdef DO_PHYSICS
   use mpas_atmphys_todynamics, only : physics_get_tend
   use mpas_atmphys_driver_microphysics, only : driver_microphysics
#endif

   implicit none

   ! module variables the reference exports (mpas_atm_time_integration.F:66-69)
   real (kind=RKIND), allocatable, dimension(:,:) :: ke_vertex
   real (kind=RKIND), allocatable, dimension(:,:) :: ke_edge
   logical, pointer :: config_apply_lbcs

   ! .true.: atm_srk3 copies the new state into host time level 2 after every step, where the
   ! caller's mpas_pool_shift_time_levels (mpas_atm_core.F:671) expects it.  .false. (default):
   ! the state stays in HBM and atm_dycore_to_host copies it when the host reads the pools.
   logical, save :: atm_dycore_sync_every_step = .false.

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

   type, bind(C) :: dyc_extreme
      real(c_double) :: value, lat, lon
      integer(c_int32_t) :: k, index
   end type dyc_extreme

   type, bind(C) :: dyc_plan_msg   ! mpas_dyc_plan_msg
      integer(c_int32_t) :: point, direction, block, peer_rank, peer_block
      integer(c_int64_t) :: count
   end type dyc_plan_msg

   type, bind(C) :: dyc_summary
      integer(c_int32_t) :: flags
      real(c_double) :: w_min, w_max, u_min, u_max
      type(dyc_extreme) :: w_min_at, w_max_at, u_min_at, u_max_at, wsp_max_at
      integer(c_int64_t) :: nan_w, nan_u
   end type dyc_summary

   integer(c_int32_t), parameter, private :: DYC_CELL = 0, DYC_EDGE = 1, DYC_VERTEX = 2, DYC_SEND = 0, DYC_RECV = 1
   integer(c_int32_t), parameter, private :: PHYS_TENDENCIES = 1, PHYS_RQVDYNTEN = 2, PHYS_MICROPHYSICS = 4
   integer(c_int32_t), parameter, private :: SUM_VEL = 1, SUM_DETAILED = 2, SUM_SCA = 4
   integer, parameter, private :: UP = 1, DOWN = 2
   integer(c_int), parameter, private :: DYC_HOST_ONLY = -2   ! MPAS_DYC_HOST_ONLY

   interface
      integer(c_int) function mpas_dyc_create(dims, cfg, device, ctx) bind(C, name='mpas_dyc_create')
         import :: c_int, c_ptr, dyc_dims, dyc_config
         type(dyc_dims), intent(in) :: dims
         type(dyc_config), intent(in) :: cfg
         integer(c_int), value :: device
         type(c_ptr), intent(out) :: ctx
      end function
      integer(c_int) function mpas_dyc_create_blocks(nblocks, dims, cfg, device, ctx) &
            bind(C, name='mpas_dyc_create_blocks')
         import :: c_int, c_int32_t, c_ptr, dyc_dims, dyc_config
         integer(c_int32_t), value :: nblocks
         type(dyc_dims), dimension(*), intent(in) :: dims
         type(dyc_config), intent(in) :: cfg
         integer(c_int), value :: device
         type(c_ptr), intent(out) :: ctx
      end function
      subroutine mpas_dyc_destroy(ctx) bind(C, name='mpas_dyc_destroy')
         import :: c_ptr
         type(c_ptr), value :: ctx
      end subroutine
      integer(c_int) function mpas_dyc_set_block_field(ctx, block, pool, name, tl, host, nbytes) &
            bind(C, name='mpas_dyc_set_block_field')
         import :: c_int, c_ptr, c_char, c_int32_t, c_int64_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: block
         character(kind=c_char), dimension(*), intent(in) :: pool, name
         integer(c_int32_t), value :: tl
         type(c_ptr), value :: host
         integer(c_int64_t), value :: nbytes
      end function
      integer(c_int) function mpas_dyc_get_block_field(ctx, block, pool, name, tl, host, nbytes) &
            bind(C, name='mpas_dyc_get_block_field')
         import :: c_int, c_ptr, c_char, c_int32_t, c_int64_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: block
         character(kind=c_char), dimension(*), intent(in) :: pool, name
         integer(c_int32_t), value :: tl
         type(c_ptr), value :: host
         integer(c_int64_t), value :: nbytes
      end function
      integer(c_int64_t) function mpas_dyc_block_field_bytes(ctx, block, pool, name) &
            bind(C, name='mpas_dyc_block_field_bytes')
         import :: c_ptr, c_char, c_int32_t, c_int64_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: block
         character(kind=c_char), dimension(*), intent(in) :: pool, name
      end function
      integer(c_int) function mpas_dyc_set_exchange_list(ctx, block, location, halo_layer, direction, peer_rank, &
            peer_block, local_index, n) bind(C, name='mpas_dyc_set_exchange_list')
         import :: c_int, c_ptr, c_int32_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: block, location, halo_layer, direction, peer_rank, peer_block
         integer(c_int32_t), dimension(*), intent(in) :: local_index
         integer(c_int32_t), value :: n
      end function
      integer(c_int) function mpas_dyc_set_exchange_positions(ctx, block, location, halo_layer, direction, &
            peer_rank, local_index, position, n) bind(C, name='mpas_dyc_set_exchange_positions')
         import :: c_int, c_ptr, c_int32_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: block, location, halo_layer, direction, peer_rank
         integer(c_int32_t), dimension(*), intent(in) :: local_index, position
         integer(c_int32_t), value :: n
      end function
      integer(c_int64_t) function mpas_dyc_comm_unique_id_bytes() bind(C, name='mpas_dyc_comm_unique_id_bytes')
         import :: c_int64_t
      end function
      integer(c_int) function mpas_dyc_comm_unique_id(id, nbytes) bind(C, name='mpas_dyc_comm_unique_id')
         import :: c_int, c_ptr, c_int64_t
         type(c_ptr), value :: id
         integer(c_int64_t), value :: nbytes
      end function
      integer(c_int) function mpas_dyc_comm_init(ctx, id, nbytes, nranks, rank) bind(C, name='mpas_dyc_comm_init')
         import :: c_int, c_ptr, c_int64_t, c_int32_t
         type(c_ptr), value :: ctx, id
         integer(c_int64_t), value :: nbytes
         integer(c_int32_t), value :: nranks, rank
      end function
      integer(c_int) function mpas_dyc_init_diagnostics(ctx, dt) bind(C, name='mpas_dyc_init_diagnostics')
         import :: c_int, c_ptr, c_double
         type(c_ptr), value :: ctx
         real(c_double), value :: dt
      end function
      integer(c_int) function mpas_dyc_solve_diagnostics(ctx, dt) bind(C, name='mpas_dyc_solve_diagnostics')
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
      integer(c_int) function mpas_dyc_synchronize(ctx) bind(C, name='mpas_dyc_synchronize')
         import :: c_int, c_ptr
         type(c_ptr), value :: ctx
      end function
      integer(c_int) function mpas_dyc_use_graph(ctx, on) bind(C, name='mpas_dyc_use_graph')
         import :: c_int, c_ptr, c_int32_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: on
      end function
      integer(c_int) function mpas_dyc_set_physics(ctx, flags) bind(C, name='mpas_dyc_set_physics')
         import :: c_int, c_ptr, c_int32_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: flags
      end function
      integer(c_int) function mpas_dyc_set_summary(ctx, flags) bind(C, name='mpas_dyc_set_summary')
         import :: c_int, c_ptr, c_int32_t
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: flags
      end function
      integer(c_int) function mpas_dyc_get_summary(ctx, out, scalar_minmax, n) bind(C, name='mpas_dyc_get_summary')
         import :: c_int, c_ptr, c_int32_t, dyc_summary
         type(c_ptr), value :: ctx
         type(dyc_summary), intent(out) :: out
         type(c_ptr), value :: scalar_minmax
         integer(c_int32_t), value :: n
      end function
      integer(c_int) function mpas_dyc_get_block_summary(ctx, block, out, scalar_minmax, n) &
            bind(C, name='mpas_dyc_get_block_summary')
         import :: c_int, c_ptr, c_int32_t, dyc_summary
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: block
         type(dyc_summary), intent(out) :: out
         type(c_ptr), value :: scalar_minmax
         integer(c_int32_t), value :: n
      end function
      integer(c_int) function mpas_dyc_finish_step(ctx, dt) bind(C, name='mpas_dyc_finish_step')
         import :: c_int, c_ptr, c_double
         type(c_ptr), value :: ctx
         real(c_double), value :: dt
      end function
      integer(c_int) function mpas_dyc_set_lbc(ctx, apply, seconds_to_interval_end) bind(C, name='mpas_dyc_set_lbc')
         import :: c_int, c_ptr, c_int32_t, c_double
         type(c_ptr), value :: ctx
         integer(c_int32_t), value :: apply
         real(c_double), value :: seconds_to_interval_end
      end function
      integer(c_int) function mpas_dyc_plan_exchanges(ctx, nranks, rank, dt, msgs, cap, n_msgs, keys, keys_bytes, &
            keys_len) bind(C, name='mpas_dyc_plan_exchanges')
         import :: c_int, c_ptr, c_int32_t, c_int64_t, c_double
         type(c_ptr), value :: ctx, msgs, keys
         integer(c_int32_t), value :: nranks, rank
         real(c_double), value :: dt
         integer(c_int64_t), value :: cap, keys_bytes
         integer(c_int64_t), intent(out) :: n_msgs, keys_len
      end function
      type(c_ptr) function mpas_dyc_last_error(ctx) bind(C, name='mpas_dyc_last_error')
         import :: c_ptr
         type(c_ptr), value :: ctx
      end function
   end interface

   type(c_ptr), save, private :: dyc = c_null_ptr        ! every block of this task (the time loop)
   type(c_ptr), save, private :: dyc_init = c_null_ptr   ! one block, model init
   logical, save, private :: coupled_init = .false.      ! atm_init_coupled_diagnostics was called
   logical, save, private :: host_stale = .false.        ! the host pools lag the device state
   logical, save, private :: wait_every_step = .false.   ! MPAS_DYCORE_WAIT_EVERY_STEP=1 (diagnostics)
   integer(c_int32_t), save, private :: summary_flags = 0, physics_flags = 0
   real (kind=RKIND), save, private :: dt_init = 0.0_RKIND
   ! atm_dycore_plan_exchanges: the domain context as host-only contexts (no GPU, no uploads)
   logical, save, private :: plan_only = .false.
   integer(c_int64_t), save, private :: plan_id_sum = 0
   ! regional runs: the host lbc pool's interval-end arrays last uploaded (mpas_atm_update_bdy_tend
   ! shifts the pool's time levels and reads new ones each time the lbc_in alarm rings), and a
   ! one-column probe block through which mpas_atm_get_bdy_state reports LBC_intv_end - now
   type(c_ptr), save, private :: lbc_uploaded = c_null_ptr
   type (block_type), pointer, save, private :: lbc_probe => null()

   ! ---- fields moved between the pools and HBM (Registry.xml var_struct names) ----
   character(len=32), dimension(3), parameter, private :: mesh_i1 = [character(len=32) :: &
      'nEdgesOnCell', 'nEdgesOnEdge', 'nAdvCellsForEdge']
   character(len=32), dimension(10), parameter, private :: mesh_i2 = [character(len=32) :: &
      'edgesOnCell', 'cellsOnCell', 'verticesOnCell', 'kiteForCell', 'cellsOnEdge', 'verticesOnEdge', &
      'edgesOnEdge', 'advCellsForEdge', 'cellsOnVertex', 'edgesOnVertex']
   character(len=32), dimension(42), parameter, private :: mesh_r = [character(len=32) :: &
      'dcEdge', 'dvEdge', 'invDcEdge', 'invDvEdge', 'fEdge', 'meshScalingDel2', 'meshScalingDel4', &
      'specZoneMaskEdge', 'angleEdge', 'latEdge', 'lonEdge', 'invAreaCell', 'specZoneMaskCell', 'latCell', &
      'lonCell', 'invAreaTriangle', 'fVertex', 'u_init', 'v_init', 'fzm', 'fzp', 'rdzw', 'rdzu', 'cf1', 'cf2', &
      'cf3', 'edgesOnCell_sign', 'edgesOnVertex_sign', 'kiteAreasOnVertex', 'weightsOnEdge', 'adv_coefs', &
      'adv_coefs_3rd', 'defc_a', 'defc_b', 'zgrid', 'zz', 'zxu', 'dss', 't_init', 'zb_cell', 'zb3_cell', &
      'coeffs_reconstruct']
   character(len=32), dimension(5), parameter, private :: state_names = [character(len=32) :: &
      'u', 'w', 'theta_m', 'rho_zz', 'scalars']
   ! diag: the model-init inputs first (never copied back), uReconstruct* last (the host computes
   ! them at init with mpas_reconstruct, mpas_atm_core.F:411-421)
   integer, parameter, private :: N_DIAG_IN = 4, N_RECON = 5
   character(len=32), dimension(56), parameter, private :: diag_names = [character(len=32) :: &
      'theta', 'rho', 'rho_base', 'theta_base', &
      'rho_p', 'rho_p_save', 'rho_pp', 'rho_zz_old_split', 'rtheta_base', 'rtheta_p', 'rtheta_p_save', &
      'rtheta_pp', 'rtheta_pp_old', 'exner', 'exner_base', 'pressure_base', 'pressure_p', 'pressure', &
      'h_divergence', 'kdiff', 'ke', 'divergence', 'pv_cell', 'tend_rtheta_adv', 'cqw', 'cofwr', 'cofwz', &
      'cofwt', 'coftz', 'a_tri', 'alpha_tri', 'gamma_tri', 'cofrz', 'rw', 'rw_p', 'rw_save', 'wwAvg', &
      'wwAvg_split', 'ru', 'ruAvg', 'ruAvg_split', 'ru_p', 'ru_save', 'cqu', 'rho_edge', 'v', 'pv_edge', &
      'gradPVn', 'gradPVt', 'vorticity', 'pv_vertex', &
      'uReconstructX', 'uReconstructY', 'uReconstructZ', 'uReconstructZonal', 'uReconstructMeridional']

   private :: check, fatal, xfer, block_dims, read_config, create_domain_context, set_block_lists, &
              upload_block, pools_to_host, count_blocks, device_index, summarize_timestep, sorted_by

   contains

   ! atm_timestep (mpas_atm_time_integration.F:87-139): the 'SRK3' check, atm_srk3, and the
   ! xtime stamp of time level 2 on every block
   subroutine atm_timestep(domain, dt, nowTime, itimestep)
      type (domain_type), intent(inout) :: domain
      real (kind=RKIND), intent(in) :: dt
      type (MPAS_Time_type), intent(in) :: nowTime
      integer, intent(in) :: itimestep
      type (block_type), pointer :: block
      type (MPAS_Time_type) :: currTime
      type (MPAS_TimeInterval_type) :: dtInterval
      character (len=StrKIND), pointer :: xtime
      character (len=StrKIND) :: xtime_new
      character (len=StrKIND), pointer :: config_time_integration
      type (mpas_pool_type), pointer :: state

      call mpas_pool_get_config(domain % blocklist % configs, 'config_time_integration', config_time_integration)
      call mpas_pool_get_config(domain % blocklist % configs, 'config_apply_lbcs', config_apply_lbcs)
      if (trim(config_time_integration) == 'SRK3') then
         call atm_srk3(domain, dt, itimestep)
      else
         call mpas_log_write('Unknown time integration option '//trim(config_time_integration), messageType=MPAS_LOG_ERR)
         call mpas_log_write('Currently, only ''SRK3'' is supported.', messageType=MPAS_LOG_CRIT)
      end if

      call mpas_set_timeInterval(dtInterval, dt=dt)
      currTime = nowTime + dtInterval
      call mpas_get_time(currTime, dateTimeString=xtime_new)
      block => domain % blocklist
      do while (associated(block))
         call mpas_pool_get_subpool(block % structs, 'state', state)
         call mpas_pool_get_array(state, 'xtime', xtime, 2)
         if (associated(xtime)) xtime = xtime_new
         block => block % next
      end do
   end subroutine atm_timestep

   ! atm_srk3 (:142-1796) on the GPU
   subroutine atm_srk3(domain, dt, itimestep)
      type (domain_type), intent(inout) :: domain
      real (kind=RKIND), intent(in) :: dt
      integer, intent(in) :: itimestep

      if (.not. c_associated(dyc)) call create_domain_context(domain)
      call mpas_pool_get_config(domain % blocklist % configs, 'config_apply_lbcs', config_apply_lbcs)
      if (config_apply_lbcs) call lbc_to_device(domain)
#ifdef DO_PHYSICS
      call physics_to_device(domain)
#endif
      call check(dyc, mpas_dyc_timestep(dyc, real(dt, c_double), int(itimestep, c_int32_t)), 'mpas_dyc_timestep')
#ifdef DO_PHYSICS
      if (iand(physics_flags, PHYS_MICROPHYSICS) /= 0) then
         ! the microphysics on time level 2 of the step (1650-1660), then the rest of atm_srk3: the
         ! specified-zone reset (1672-1790) and summarize_timestep's reductions (1794)
         call pools_to_host(domain, 2, 2)
         call physics_after_step(domain, dt, itimestep)
         call check(dyc, mpas_dyc_finish_step(dyc, real(dt, c_double)), 'mpas_dyc_finish_step')
      end if
#endif
      ! the device swaps now; the caller swaps the host pools right after (mpas_atm_core.F:671)
      call check(dyc, mpas_dyc_shift_time_levels(dyc), 'mpas_dyc_shift_time_levels')
#ifdef DO_PHYSICS
      ! the host physics reads the new state every step
      if (iand(physics_flags, PHYS_MICROPHYSICS) == 0 .or. config_apply_lbcs) call pools_to_host(domain, 2, 1)
#else
      if (atm_dycore_sync_every_step) then
         call pools_to_host(domain, 2, 1)
      else
         host_stale = .true.
      end if
#endif
      if (summary_flags /= 0) call summarize_timestep(domain)
      if (wait_every_step) call check(dyc, mpas_dyc_synchronize(dyc), 'mpas_dyc_synchronize')
   end subroutine atm_srk3

   ! Copy the device state into the host pools' time level 1 (the current one once the caller
   ! has shifted time levels after the step): prognostics, diagnostics, rthdynten / rqvdynten.
   ! Call it wherever the host reads the pools -- before history / restart writes
   ! (mpas_stream_mgr_write in atm_core_run, mpas_atm_core.F:690-760) -- and at the end of the run.
   subroutine atm_dycore_to_host(domain)
      type (domain_type), intent(inout) :: domain
      if (.not. c_associated(dyc) .or. .not. host_stale) return
      call pools_to_host(domain, 1, 1)
      host_stale = .false.
   end subroutine atm_dycore_to_host

   ! Wait until the device has finished every step issued so far (the steps are asynchronous)
   subroutine atm_dycore_wait()
      if (c_associated(dyc)) call check(dyc, mpas_dyc_synchronize(dyc), 'mpas_dyc_synchronize')
   end subroutine atm_dycore_wait

   ! This task's RCCL exchange plan, without a GPU: the domain context is built as the first
   ! atm_srk3 builds it (create_domain_context: every block of domain%blocklist, the id broadcast
   ! over dminfo%comm, set_block_lists with parinfo's lists), but as host-only contexts, with no
   ! uploads and no model init; then mpas_dyc_plan_exchanges runs the planner over one model run's
   ! exchange calls.  `path` gets one line 'id <n>' (a checksum of the broadcast id words), then
   ! 'msg <point> <direction> <block> <peer_rank> <peer_block> <count>' per RCCL message and
   ! 'key <plan key>' per exchange call, in issue order.  The context is destroyed afterwards.
   subroutine atm_dycore_plan_exchanges(domain, dt, path)
      type (domain_type), intent(inout) :: domain
      real (kind=RKIND), intent(in) :: dt
      character(len=*), intent(in) :: path
      type(dyc_plan_msg), allocatable, target :: msgs(:)
      character(kind=c_char), allocatable, target :: keys(:)
      integer(c_int64_t) :: nm, kl
      integer(c_int) :: ierr
      integer :: u, i, j, nprocs, myrank
      if (c_associated(dyc)) call fatal(dyc, 'atm_dycore_plan_exchanges after the domain context exists')
      nprocs = domain % dminfo % nprocs
      myrank = domain % dminfo % my_proc_id
      plan_only = .true.
      call create_domain_context(domain)
      ierr = mpas_dyc_plan_exchanges(dyc, int(nprocs, c_int32_t), int(myrank, c_int32_t), real(dt, c_double), &
                                     c_null_ptr, 0_c_int64_t, nm, c_null_ptr, 0_c_int64_t, kl)
      allocate(msgs(max(nm, 1_c_int64_t)), keys(max(kl, 1_c_int64_t)))
      call check(dyc, mpas_dyc_plan_exchanges(dyc, int(nprocs, c_int32_t), int(myrank, c_int32_t), real(dt, c_double), &
                                              c_loc(msgs), nm, nm, c_loc(keys), kl, kl), 'mpas_dyc_plan_exchanges')
      open(newunit=u, file=path, status='replace', action='write', recl=65536)
      write(u, '(a,i0)') 'id ', plan_id_sum
      do i = 1, int(nm)
         write(u, '(a,5(1x,i0),1x,i0)') 'msg', msgs(i) % point, msgs(i) % direction, msgs(i) % block, &
            msgs(i) % peer_rank, msgs(i) % peer_block, msgs(i) % count
      end do
      j = 1   ! keys: NUL-terminated text, one key per line
      do i = 1, int(kl)
         if (keys(i) == c_null_char .or. keys(i) == achar(10)) then
            if (i > j) write(u, '(a,a)') 'key ', transfer(keys(j:i - 1), repeat(' ', i - j))
            j = i + 1
            if (keys(i) == c_null_char) exit
         end if
      end do
      close(u)
      call mpas_dyc_destroy(dyc)
      dyc = c_null_ptr
      plan_only = .false.
   end subroutine atm_dycore_plan_exchanges

   ! Copy the host pools' current state (time level 1) and diagnostics into HBM, after the host
   ! changed them between steps (e.g. an analysis increment or a state read from a file).
   subroutine atm_dycore_from_host(domain)
      type (domain_type), intent(inout) :: domain
      type (block_type), pointer :: block
      type (mpas_pool_type), pointer :: state, diag
      integer :: ib, i
      if (.not. c_associated(dyc)) return
      block => domain % blocklist
      ib = 0
      do while (associated(block))
         call mpas_pool_get_subpool(block % structs, 'state', state)
         call mpas_pool_get_subpool(block % structs, 'diag', diag)
         do i = 1, size(state_names)
            call xfer(dyc, ib, state, 'state', trim(state_names(i)), 1, 1, UP, .true.)
         end do
         do i = 1, size(diag_names)
            call xfer(dyc, ib, diag, 'diag', trim(diag_names(i)), 1, 1, UP, .false.)
         end do
         ib = ib + 1
         block => block % next
      end do
   end subroutine atm_dycore_from_host

   ! atm_init_coupled_diagnostics (:5825): the core calls it together with
   ! atm_compute_solve_diagnostics (mpas_atm_core.F:387-404), except on a restart; the device
   ! runs both in the call below, so this only records that the coupled init is wanted
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
      coupled_init = .true.
   end subroutine atm_init_coupled_diagnostics

   ! atm_compute_solve_diagnostics (:5419) at model init, once per block: a one-block context
   ! runs the init diagnostics (with atm_init_coupled_diagnostics unless this is a restart) and
   ! the results go back into the block's pools
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
      type(dyc_dims) :: d(1)
      type(dyc_config) :: c
      integer :: i

      if (cellStart /= 1) return   ! one thread per block does the block's work
      if (c_associated(dyc)) call fatal(dyc, 'atm_compute_solve_diagnostics after the first time step')
      if (c_associated(dyc_init)) call mpas_dyc_destroy(dyc_init)
      dyc_init = c_null_ptr
      dt_init = dt
      call block_dims(mesh, state, d(1))
      call read_config(configs, c)
      call check(dyc_init, mpas_dyc_create_blocks(1_c_int32_t, d, c, device_index(), dyc_init), 'mpas_dyc_create_blocks')
      call upload_block(dyc_init, 0, mesh, state, diag)
      if (coupled_init) then
         call check(dyc_init, mpas_dyc_init_diagnostics(dyc_init, real(dt, c_double)), 'mpas_dyc_init_diagnostics')
      else
         call check(dyc_init, mpas_dyc_solve_diagnostics(dyc_init, real(dt, c_double)), 'mpas_dyc_solve_diagnostics')
      end if
      call xfer(dyc_init, 0, state, 'state', 'theta_m', 1, 1, DOWN, .true.)
      call xfer(dyc_init, 0, state, 'state', 'rho_zz', 1, 1, DOWN, .true.)
      do i = N_DIAG_IN + 1, size(diag_names) - N_RECON
         call xfer(dyc_init, 0, diag, 'diag', trim(diag_names(i)), 1, 1, DOWN, .false.)
      end do
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
      call fatal(c_null_ptr, 'atm_advance_acoustic_step is internal to mpas_dyc_timestep')
   end subroutine atm_advance_acoustic_step

   subroutine atm_divergence_damping_3d(state, diag, mesh, configs, dts, edgeStart, edgeEnd)
      type (mpas_pool_type), intent(inout) :: state, diag, mesh
      type (mpas_pool_type), intent(in) :: configs
      real (kind=RKIND), intent(in) :: dts
      integer, intent(in) :: edgeStart, edgeEnd
      call fatal(c_null_ptr, 'atm_divergence_damping_3d is internal to mpas_dyc_timestep')
   end subroutine atm_divergence_damping_3d

   ! ------------------------------------------------------------------ the domain context
   ! Every block of this task (mpas_dyc_create_blocks, block order = domain%blocklist order), the
   ! parinfo exchange lists, the RCCL communicator of the MPI tasks, and the model init.  A
   ! single block on a single task keeps its model-init context, which already holds that state.
   subroutine create_domain_context(domain)
      type (domain_type), intent(inout) :: domain
      type (block_type), pointer :: block
      type (mpas_pool_type), pointer :: mesh, state, diag
      type(dyc_dims), allocatable :: d(:)
      type(dyc_config) :: c
      integer :: nb, ib, nprocs, myrank
      integer(c_int64_t) :: idbytes
      integer, allocatable, target :: idwords(:)
      logical, pointer :: lp
      character (len=StrKIND), pointer :: microp

      nb = count_blocks(domain)
      nprocs = domain % dminfo % nprocs
      myrank = domain % dminfo % my_proc_id
      if (nb == 1 .and. nprocs == 1 .and. c_associated(dyc_init) .and. .not. plan_only) then
         dyc = dyc_init
         dyc_init = c_null_ptr
      else
         if (c_associated(dyc_init)) call mpas_dyc_destroy(dyc_init)
         dyc_init = c_null_ptr
         allocate(d(nb))
         block => domain % blocklist
         ib = 0
         do while (associated(block))
            call mpas_pool_get_subpool(block % structs, 'mesh', mesh)
            call mpas_pool_get_subpool(block % structs, 'state', state)
            call block_dims(mesh, state, d(ib + 1))
            ib = ib + 1
            block => block % next
         end do
         call read_config(domain % blocklist % configs, c)
         if (plan_only) then
            call check(dyc, mpas_dyc_create_blocks(int(nb, c_int32_t), d, c, DYC_HOST_ONLY, dyc), 'mpas_dyc_create_blocks')
         else
            call check(dyc, mpas_dyc_create_blocks(int(nb, c_int32_t), d, c, device_index(), dyc), 'mpas_dyc_create_blocks')
         end if
         if (nprocs > 1) then
            ! RCCL id from task 0 to every task over the model's communicator (dminfo % comm)
            idbytes = mpas_dyc_comm_unique_id_bytes()
            allocate(idwords((idbytes + 3) / 4))
            idwords = 0
            if (myrank == 0) then
               if (plan_only) then   ! no GPU: a known pattern stands for the id (RCCL's needs a device)
                  idwords = [(7919 * ib + 13, ib = 1, size(idwords))]
               else
                  call check(dyc, mpas_dyc_comm_unique_id(c_loc(idwords), idbytes), 'mpas_dyc_comm_unique_id')
               end if
            end if
            call mpas_dmpar_bcast_ints(domain % dminfo, size(idwords), idwords)
            if (plan_only) then
               plan_id_sum = sum(int(idwords, c_int64_t) * [(int(ib, c_int64_t), ib = 1, size(idwords))])
            else
               call check(dyc, mpas_dyc_comm_init(dyc, c_loc(idwords), idbytes, int(nprocs, c_int32_t), &
                                                  int(myrank, c_int32_t)), 'mpas_dyc_comm_init')
            end if
         end if
         block => domain % blocklist
         ib = 0
         do while (associated(block))
            call mpas_pool_get_subpool(block % structs, 'mesh', mesh)
            call mpas_pool_get_subpool(block % structs, 'state', state)
            call mpas_pool_get_subpool(block % structs, 'diag', diag)
            call set_block_lists(block, ib, myrank, nprocs > 1, nb > 1)
            if (.not. plan_only) call upload_block(dyc, ib, mesh, state, diag)
            ib = ib + 1
            block => block % next
         end do
         if (plan_only) return   ! atm_dycore_plan_exchanges: the lists are in, nothing runs
         if (coupled_init) then
            call check(dyc, mpas_dyc_init_diagnostics(dyc, real(dt_init, c_double)), 'mpas_dyc_init_diagnostics')
         else
            call check(dyc, mpas_dyc_solve_diagnostics(dyc, real(dt_init, c_double)), 'mpas_dyc_solve_diagnostics')
         end if
      end if
      ! mpas_init_reconstruct ran on the host after the init diagnostics (mpas_atm_core.F:409)
      block => domain % blocklist
      ib = 0
      do while (associated(block))
         call mpas_pool_get_subpool(block % structs, 'mesh', mesh)
         call xfer(dyc, ib, mesh, 'mesh', 'coeffs_reconstruct', 1, 1, UP, .true.)
         ib = ib + 1
         block => block % next
      end do
      call check(dyc, mpas_dyc_use_graph(dyc, 1_c_int32_t), 'mpas_dyc_use_graph')
      ! regional runs (config_apply_lbcs): the boundary-zone masks and relaxation scaling of the mesh
      ! pool (mpas_atm_setup_bdy_masks, atm_compute_mesh_scaling); the lbc pool follows every step
      call mpas_pool_get_config(domain % blocklist % configs, 'config_apply_lbcs', lp)
      if (associated(lp)) then
         if (lp) then
            block => domain % blocklist
            ib = 0
            do while (associated(block))
               call mpas_pool_get_subpool(block % structs, 'mesh', mesh)
               call xfer(dyc, ib, mesh, 'mesh', 'bdyMaskCell', 1, 1, UP, .true.)
               call xfer(dyc, ib, mesh, 'mesh', 'bdyMaskEdge', 1, 1, UP, .true.)
               call xfer(dyc, ib, mesh, 'mesh', 'nearestRelaxationCell', 1, 1, UP, .true.)
               call xfer(dyc, ib, mesh, 'mesh', 'meshScalingRegionalCell', 1, 1, UP, .true.)
               call xfer(dyc, ib, mesh, 'mesh', 'meshScalingRegionalEdge', 1, 1, UP, .true.)
               ib = ib + 1
               block => block % next
            end do
         end if
      end if
#ifdef DO_PHYSICS
      physics_flags = PHYS_TENDENCIES
      block => domain % blocklist
      if (rqvdynten_wanted(block % configs)) physics_flags = ior(physics_flags, PHYS_RQVDYNTEN)
      call mpas_pool_get_config(block % configs, 'config_microp_scheme', microp)
      if (trim(microp) /= 'off') physics_flags = ior(physics_flags, PHYS_MICROPHYSICS)
      call check(dyc, mpas_dyc_set_physics(dyc, physics_flags), 'mpas_dyc_set_physics')
#endif
      ! summarize_timestep's namelist switches (Registry.xml defaults when a core lacks them)
      summary_flags = SUM_VEL
      call mpas_pool_get_config(domain % blocklist % configs, 'config_print_global_minmax_vel', lp)
      if (associated(lp)) then
         if (.not. lp) summary_flags = 0
      end if
      call mpas_pool_get_config(domain % blocklist % configs, 'config_print_detailed_minmax_vel', lp)
      if (associated(lp)) then
         if (lp) summary_flags = ior(summary_flags, SUM_DETAILED)
      end if
      call mpas_pool_get_config(domain % blocklist % configs, 'config_print_global_minmax_sca', lp)
      if (associated(lp)) then
         if (lp) summary_flags = ior(summary_flags, SUM_SCA)
      end if
      call check(dyc, mpas_dyc_set_summary(dyc, summary_flags), 'mpas_dyc_set_summary')
      call env_sync_switch()
   end subroutine create_domain_context

   ! The block's parinfo lists (mpas_multihalo_exchange_list, built by mpas_block_creator):
   !  * xToCopy: endPointID = the local block receiving, srcList = owned elements here, destList
   !    = its halo elements, element i of one to element i of the other (mpas_dmpar.F:5480-5502);
   !  * xToSend / xToRecv (other tasks): endPointID = the task, and the other list holds buffer
   !    positions (mpas_dmpar.F:5440-5470, 5510-5540).  One block per task: sorted by position they
   !    give the order the two sides exchange (a block-pair list with the peer's block 0).  Several
   !    blocks per task (positional): the lists go in as they are, element and position, and the
   !    library lays the message out as mpas_dmpar lays out its buffer, which the task's blocks fill
   !    together (mpas_dyc_set_exchange_positions).
   subroutine set_block_lists(block, ib, myrank, remote, positional)
      type (block_type), pointer :: block
      integer, intent(in) :: ib, myrank
      logical, intent(in) :: remote, positional
      type (mpas_multihalo_exchange_list), pointer :: ml
      type (mpas_exchange_list), pointer :: node
      integer :: il, kind, layer
      integer(c_int32_t) :: loc
      integer(c_int32_t), allocatable :: idx(:)
      do il = 1, 3
         loc = int(il - 1, c_int32_t)
         do kind = 1, 3
            nullify(ml)
            select case (il * 10 + kind)
            case (11); ml => block % parinfo % cellsToCopy
            case (12); if (remote) ml => block % parinfo % cellsToSend
            case (13); if (remote) ml => block % parinfo % cellsToRecv
            case (21); ml => block % parinfo % edgesToCopy
            case (22); if (remote) ml => block % parinfo % edgesToSend
            case (23); if (remote) ml => block % parinfo % edgesToRecv
            case (31); ml => block % parinfo % verticesToCopy
            case (32); if (remote) ml => block % parinfo % verticesToSend
            case (33); if (remote) ml => block % parinfo % verticesToRecv
            end select
            if (.not. associated(ml)) cycle
            if (.not. associated(ml % halos)) cycle
            do layer = 1, size(ml % halos)
               node => ml % halos(layer) % exchList
               do while (associated(node))
                  if (node % nList > 0) then
                     if (kind == 1) then
                        call check(dyc, mpas_dyc_set_exchange_list(dyc, int(ib, c_int32_t), loc, int(layer, c_int32_t), &
                                   DYC_SEND, int(myrank, c_int32_t), int(node % endPointID, c_int32_t), &
                                   int(node % srcList(1:node % nList), c_int32_t), int(node % nList, c_int32_t)), &
                                   'mpas_dyc_set_exchange_list')
                        call check(dyc, mpas_dyc_set_exchange_list(dyc, int(node % endPointID, c_int32_t), loc, &
                                   int(layer, c_int32_t), DYC_RECV, int(myrank, c_int32_t), int(ib, c_int32_t), &
                                   int(node % destList(1:node % nList), c_int32_t), int(node % nList, c_int32_t)), &
                                   'mpas_dyc_set_exchange_list')
                     else if (positional .and. kind == 2) then
                        call check(dyc, mpas_dyc_set_exchange_positions(dyc, int(ib, c_int32_t), loc, &
                                   int(layer, c_int32_t), DYC_SEND, int(node % endPointID, c_int32_t), &
                                   int(node % srcList(1:node % nList), c_int32_t), &
                                   int(node % destList(1:node % nList), c_int32_t), int(node % nList, c_int32_t)), &
                                   'mpas_dyc_set_exchange_positions')
                     else if (positional) then
                        call check(dyc, mpas_dyc_set_exchange_positions(dyc, int(ib, c_int32_t), loc, &
                                   int(layer, c_int32_t), DYC_RECV, int(node % endPointID, c_int32_t), &
                                   int(node % destList(1:node % nList), c_int32_t), &
                                   int(node % srcList(1:node % nList), c_int32_t), int(node % nList, c_int32_t)), &
                                   'mpas_dyc_set_exchange_positions')
                     else if (kind == 2) then
                        idx = sorted_by(node % srcList(1:node % nList), node % destList(1:node % nList))
                        call check(dyc, mpas_dyc_set_exchange_list(dyc, int(ib, c_int32_t), loc, int(layer, c_int32_t), &
                                   DYC_SEND, int(node % endPointID, c_int32_t), 0_c_int32_t, idx, &
                                   int(node % nList, c_int32_t)), 'mpas_dyc_set_exchange_list')
                     else
                        idx = sorted_by(node % destList(1:node % nList), node % srcList(1:node % nList))
                        call check(dyc, mpas_dyc_set_exchange_list(dyc, int(ib, c_int32_t), loc, int(layer, c_int32_t), &
                                   DYC_RECV, int(node % endPointID, c_int32_t), 0_c_int32_t, idx, &
                                   int(node % nList, c_int32_t)), 'mpas_dyc_set_exchange_list')
                     end if
                  end if
                  node => node % next
               end do
            end do
         end do
      end do
   end subroutine set_block_lists

   ! values(:) reordered by ascending key(:) (buffer positions are distinct)
   function sorted_by(values, key) result(out)
      integer, dimension(:), intent(in) :: values, key
      integer(c_int32_t), allocatable :: out(:)
      integer, allocatable :: perm(:)
      integer :: i, j, t
      allocate(perm(size(key)), out(size(key)))
      perm = [(i, i = 1, size(key))]
      do i = 2, size(key)   ! insertion sort: lists arrive (nearly) in position order
         t = perm(i)
         j = i - 1
         do while (j >= 1)
            if (key(perm(j)) <= key(t)) exit
            perm(j + 1) = perm(j)
            j = j - 1
         end do
         perm(j + 1) = t
      end do
      out = int(values(perm), c_int32_t)
   end function sorted_by

   ! the model-init inputs of one block: mesh, state time level 1 (a restart also has the coupled
   ! state and its diagnostics), diag theta / rho / base state
   subroutine upload_block(ctx, ib, mesh, state, diag)
      type(c_ptr), intent(in) :: ctx
      integer, intent(in) :: ib
      type (mpas_pool_type), intent(in) :: mesh, state, diag
      integer :: i
      do i = 1, size(mesh_i1)
         call xfer(ctx, ib, mesh, 'mesh', trim(mesh_i1(i)), 1, 1, UP, .true.)
      end do
      do i = 1, size(mesh_i2)
         call xfer(ctx, ib, mesh, 'mesh', trim(mesh_i2(i)), 1, 1, UP, .true.)
      end do
      do i = 1, size(mesh_r)
         call xfer(ctx, ib, mesh, 'mesh', trim(mesh_r(i)), 1, 1, UP, .false.)
      end do
      do i = 1, size(state_names)
         call xfer(ctx, ib, state, 'state', trim(state_names(i)), 1, 1, UP, .true.)
      end do
      if (coupled_init) then
         do i = 1, N_DIAG_IN
            call xfer(ctx, ib, diag, 'diag', trim(diag_names(i)), 1, 1, UP, .true.)
         end do
      else
         do i = 1, size(diag_names)
            call xfer(ctx, ib, diag, 'diag', trim(diag_names(i)), 1, 1, UP, .false.)
         end do
      end if
   end subroutine upload_block

   ! the device state of time level dev_tl into host time level host_tl of every block
   subroutine pools_to_host(domain, host_tl, dev_tl)
      type (domain_type), intent(inout) :: domain
      integer, intent(in) :: host_tl, dev_tl
      type (block_type), pointer :: block
      type (mpas_pool_type), pointer :: state, diag, tend_physics
      integer :: ib, i
      block => domain % blocklist
      ib = 0
      do while (associated(block))
         call mpas_pool_get_subpool(block % structs, 'state', state)
         call mpas_pool_get_subpool(block % structs, 'diag', diag)
         do i = 1, size(state_names)
            call xfer(dyc, ib, state, 'state', trim(state_names(i)), host_tl, dev_tl, DOWN, .true.)
         end do
         do i = N_DIAG_IN + 1, size(diag_names)
            call xfer(dyc, ib, diag, 'diag', trim(diag_names(i)), 1, 1, DOWN, .false.)
         end do
         call mpas_pool_get_subpool(block % structs, 'tend_physics', tend_physics)
         if (associated(tend_physics)) then
            call xfer(dyc, ib, tend_physics, 'tend_physics', 'rthdynten', 1, 1, DOWN, .false.)
            if (iand(physics_flags, PHYS_RQVDYNTEN) /= 0) &
               call xfer(dyc, ib, tend_physics, 'tend_physics', 'rqvdynten', 1, 1, DOWN, .false.)
         end if
         ib = ib + 1
         block => block % next
      end do
   end subroutine pools_to_host

#ifdef DO_PHYSICS
   ! physics_get_tend (mpas_atm_time_integration.F:424-449) on the host, its tendencies into HBM
   subroutine physics_to_device(domain)
      type (domain_type), intent(inout) :: domain
      type (block_type), pointer :: block
      type (mpas_pool_type), pointer :: mesh, state, diag, tend, tend_physics
      real (kind=RKIND), allocatable, dimension(:,:), target :: tru, trt, trho
      integer, pointer :: nCells, nEdges, nVertLevels
      integer :: ib
      block => domain % blocklist
      ib = 0
      do while (associated(block))
         call mpas_pool_get_subpool(block % structs, 'mesh', mesh)
         call mpas_pool_get_subpool(block % structs, 'state', state)
         call mpas_pool_get_subpool(block % structs, 'diag', diag)
         call mpas_pool_get_subpool(block % structs, 'tend', tend)
         call mpas_pool_get_subpool(block % structs, 'tend_physics', tend_physics)
         call mpas_pool_get_dimension(mesh, 'nCells', nCells)
         call mpas_pool_get_dimension(mesh, 'nEdges', nEdges)
         call mpas_pool_get_dimension(mesh, 'nVertLevels', nVertLevels)
         allocate(tru(nVertLevels, nEdges + 1), trt(nVertLevels, nCells + 1), trho(nVertLevels, nCells + 1))
         tru = 0.0_RKIND
         trt = 0.0_RKIND
         trho = 0.0_RKIND
         call physics_get_tend(block, mesh, state, diag, tend, tend_physics, block % configs, 1, 1, tru, trt, trho)
         call check(dyc, mpas_dyc_set_block_field(dyc, int(ib, c_int32_t), 'tend_physics'//c_null_char, &
                    'tend_ru_physics'//c_null_char, 1_c_int32_t, c_loc(tru), 8_c_int64_t * size(tru, kind=c_int64_t)), &
                    'set tend_ru_physics')
         call check(dyc, mpas_dyc_set_block_field(dyc, int(ib, c_int32_t), 'tend_physics'//c_null_char, &
                    'tend_rtheta_physics'//c_null_char, 1_c_int32_t, c_loc(trt), 8_c_int64_t * size(trt, kind=c_int64_t)), &
                    'set tend_rtheta_physics')
         call check(dyc, mpas_dyc_set_block_field(dyc, int(ib, c_int32_t), 'tend_physics'//c_null_char, &
                    'tend_rho_physics'//c_null_char, 1_c_int32_t, c_loc(trho), 8_c_int64_t * size(trho, kind=c_int64_t)), &
                    'set tend_rho_physics')
         call xfer(dyc, ib, tend, 'tend', 'scalars_tend', 1, 1, UP, .true.)
         deallocate(tru, trt, trho)
         ib = ib + 1
         block => block % next
      end do
   end subroutine physics_to_device

   ! the microphysics call of 1650-1660 on the host, on time level 2 of the step before the shift
   ! (rqvdynten and the clip ran on the device); what it changes -- theta_m, scalars, rtheta_p,
   ! exner, pressure_p, rt_diabatic_tend -- goes back to the device before mpas_dyc_finish_step
   subroutine physics_after_step(domain, dt, itimestep)
      type (domain_type), intent(inout) :: domain
      real (kind=RKIND), intent(in) :: dt
      integer, intent(in) :: itimestep
      type (block_type), pointer :: block
      type (mpas_pool_type), pointer :: mesh, state, diag, diag_physics, tend
      character (len=StrKIND), pointer :: config_microp_scheme
      integer, pointer :: nThreads
      integer, dimension(:), pointer :: cellSolveThreadStart, cellSolveThreadEnd
      integer :: ib, thread
      call mpas_pool_get_config(domain % blocklist % configs, 'config_microp_scheme', config_microp_scheme)
      if (trim(config_microp_scheme) == 'off') return
      block => domain % blocklist
      ib = 0
      do while (associated(block))
         call mpas_pool_get_subpool(block % structs, 'mesh', mesh)
         call mpas_pool_get_subpool(block % structs, 'state', state)
         call mpas_pool_get_subpool(block % structs, 'diag', diag)
         call mpas_pool_get_subpool(block % structs, 'diag_physics', diag_physics)
         call mpas_pool_get_subpool(block % structs, 'tend', tend)
         call mpas_pool_get_dimension(block % dimensions, 'nThreads', nThreads)
         call mpas_pool_get_dimension(block % dimensions, 'cellSolveThreadStart', cellSolveThreadStart)
         call mpas_pool_get_dimension(block % dimensions, 'cellSolveThreadEnd', cellSolveThreadEnd)
!$OMP PARALLEL DO
         do thread = 1, nThreads
            call driver_microphysics(block % configs, mesh, state, 2, diag, diag_physics, tend, itimestep, &
                                     cellSolveThreadStart(thread), cellSolveThreadEnd(thread))
         end do
!$OMP END PARALLEL DO
         call xfer(dyc, ib, state, 'state', 'theta_m', 2, 2, UP, .true.)
         call xfer(dyc, ib, state, 'state', 'scalars', 2, 2, UP, .true.)
         call xfer(dyc, ib, diag, 'diag', 'rtheta_p', 1, 1, UP, .true.)
         call xfer(dyc, ib, diag, 'diag', 'exner', 1, 1, UP, .true.)
         call xfer(dyc, ib, diag, 'diag', 'pressure_p', 1, 1, UP, .true.)
         call xfer(dyc, ib, tend, 'tend', 'rt_diabatic_tend', 1, 1, UP, .true.)
         ib = ib + 1
         block => block % next
      end do
   end subroutine physics_after_step

   ! rqvdynten is computed for the convection schemes that read it (1629-1643)
   logical function rqvdynten_wanted(configs)
      type (mpas_pool_type), intent(in) :: configs
      character (len=StrKIND), pointer :: scheme
      call mpas_pool_get_config(configs, 'config_convection_scheme', scheme)
      rqvdynten_wanted = trim(scheme) == 'cu_grell_freitas' .or. trim(scheme) == 'cu_tiedtke' .or. &
                         trim(scheme) == 'cu_ntiedtke'
   end function rqvdynten_wanted
#endif

   ! summarize_timestep (:6675-7018): the device reduced the extrema over the owned elements of
   ! each block, each over all tasks (mpas_dyc_get_block_summary); the host writes the reference's
   ! log lines, one set per block as the reference's block loops do
   subroutine summarize_timestep(domain)
      type (domain_type), intent(inout) :: domain
      type(dyc_summary), allocatable :: s(:)
      integer, pointer :: num_scalars
      type (mpas_pool_type), pointer :: state
      real(c_double), allocatable, target :: sca(:,:)
      integer :: i, ib, nb
      call mpas_pool_get_subpool(domain % blocklist % structs, 'state', state)
      call mpas_pool_get_dimension(state, 'num_scalars', num_scalars)
      nb = count_blocks(domain)
      allocate(s(nb), sca(2 * num_scalars, nb))
      do ib = 1, nb
         call check(dyc, mpas_dyc_get_block_summary(dyc, int(ib - 1, c_int32_t), s(ib), c_loc(sca(1, ib)), &
                    int(2 * num_scalars, c_int32_t)), 'mpas_dyc_get_block_summary')
      end do
      if (iand(summary_flags, SUM_DETAILED) /= 0) then
         call mpas_log_write('')
         do ib = 1, nb
            call located(' global min w: ', s(ib) % w_min_at)
            call located(' global max w: ', s(ib) % w_max_at)
            call located(' global min u: ', s(ib) % u_min_at)
            call located(' global max u: ', s(ib) % u_max_at)
            call located(' global max wsp: ', s(ib) % wsp_max_at)
            if (s(ib) % nan_w > 0) call mpas_log_write('NaN detected in ''w'' field.', messageType=MPAS_LOG_CRIT)
            if (s(ib) % nan_u > 0) call mpas_log_write('NaN detected in ''u'' field.', messageType=MPAS_LOG_CRIT)
         end do
      else if (iand(summary_flags, SUM_VEL) /= 0) then
         call mpas_log_write('')
         do ib = 1, nb
            call mpas_log_write('global min, max w $r $r', realArgs=(/s(ib) % w_min, s(ib) % w_max/))
            call mpas_log_write('global min, max u $r $r', realArgs=(/s(ib) % u_min, s(ib) % u_max/))
         end do
      end if
      if (iand(summary_flags, SUM_SCA) /= 0) then
         if (iand(summary_flags, SUM_VEL + SUM_DETAILED) == 0) call mpas_log_write('')
         do ib = 1, nb
            do i = 1, num_scalars
               call mpas_log_write(' global min, max scalar $i $r $r', intArgs=(/i/), &
                                   realArgs=(/sca(2 * i - 1, ib), sca(2 * i, ib)/))
            end do
         end do
      end if
   contains
      subroutine located(what, e)
         character(len=*), intent(in) :: what
         type(dyc_extreme), intent(in) :: e
         call mpas_log_write(what//'$r k=$i, $r lat, $r lon', intArgs=(/int(e % k)/), &
                             realArgs=(/real(e % value, RKIND), real(e % lat, RKIND), real(e % lon, RKIND)/))
      end subroutine located
   end subroutine summarize_timestep

   ! Regional runs (config_apply_lbcs), before every step: the lbc pool into HBM whenever the host
   ! read new boundary data (mpas_atm_update_bdy_tend, called by atm_core_run on the lbc_in alarm,
   ! mpas_atm_core.F:584-627, shifts the pool's time levels and reads the interval-end state into
   ! time level 2, so its array moves), and the seconds from the step's start to the LBC interval
   ! end.  The module keeps that interval end private (LBC_intv_end); its public getter reports it:
   ! mpas_atm_get_bdy_state(clock, block, ..., delta_t = 0) returns state - (LBC_intv_end - now) *
   ! tendency (mpas_atm_boundaries.F:337-409), and a probe block whose lbc pool holds state 0 and
   ! tendency -1 gets back exactly LBC_intv_end - now.
   subroutine lbc_to_device(domain)
      type (domain_type), intent(inout) :: domain
      type (block_type), pointer :: block
      type (mpas_pool_type), pointer :: lbc
      real (kind=RKIND), dimension(:,:), pointer :: u2
      real (kind=RKIND), dimension(1, 2) :: probe
      character(len=32), dimension(4), parameter :: lbc2 = [character(len=32) :: &
         'lbc_u', 'lbc_ru', 'lbc_rho_zz', 'lbc_rtheta_m']
      integer :: ib, i, tl
      block => domain % blocklist
      call mpas_pool_get_subpool(block % structs, 'lbc', lbc)
      if (.not. associated(lbc)) call fatal(dyc, 'config_apply_lbcs: the block has no lbc pool')
      call mpas_pool_get_array(lbc, 'lbc_u', u2, 2)
      if (.not. c_associated(lbc_uploaded, c_loc(u2(1,1)))) then
         ib = 0
         do while (associated(block))
            call mpas_pool_get_subpool(block % structs, 'lbc', lbc)
            do tl = 1, 2
               do i = 1, size(lbc2)
                  call xfer(dyc, ib, lbc, 'lbc', trim(lbc2(i)), tl, tl, UP, .true.)
               end do
               call xfer(dyc, ib, lbc, 'lbc', 'lbc_scalars', tl, tl, UP, .true.)
            end do
            ib = ib + 1
            block => block % next
         end do
         lbc_uploaded = c_loc(u2(1,1))
      end if
      if (.not. associated(lbc_probe)) call make_lbc_probe()
      probe = mpas_atm_get_bdy_state(domain % clock, lbc_probe, 1, 1, 'dyc_probe', 0.0_RKIND)
      call check(dyc, mpas_dyc_set_lbc(dyc, 1_c_int32_t, real(probe(1, 1), c_double)), 'mpas_dyc_set_lbc')
   end subroutine lbc_to_device

   ! the probe block of lbc_to_device: an lbc pool with one field lbc_dyc_probe(1, 1+1) of two time
   ! levels, tendency (time level 1) -1, state (time level 2) 0
   subroutine make_lbc_probe()
      type (mpas_pool_type), pointer :: lbc
      type (field2DReal), dimension(:), pointer :: fa
      integer :: t
      allocate(lbc_probe)
      call mpas_pool_create_pool(lbc_probe % structs)
      call mpas_pool_create_pool(lbc)
      call mpas_pool_add_subpool(lbc_probe % structs, 'lbc', lbc)
      allocate(fa(2))
      do t = 1, 2
         fa(t) % block => lbc_probe
         fa(t) % fieldName = 'lbc_dyc_probe'
         fa(t) % isActive = .true.
         fa(t) % dimSizes(1) = 1
         fa(t) % dimSizes(2) = 2
         allocate(fa(t) % array(1, 2))
      end do
      fa(1) % array = -1.0_RKIND
      fa(2) % array = 0.0_RKIND
      call mpas_pool_add_field(lbc, 'lbc_dyc_probe', fa)
   end subroutine make_lbc_probe

   ! ------------------------------------------------------------------ helpers
   integer function count_blocks(domain)
      type (domain_type), intent(in) :: domain
      type (block_type), pointer :: block
      count_blocks = 0
      block => domain % blocklist
      do while (associated(block))
         count_blocks = count_blocks + 1
         block => block % next
      end do
   end function count_blocks

   ! the HIP device of this task: MPAS_DYCORE_DEVICE, else the launcher's node-local rank (one task
   ! per GPU), else the current device
   integer(c_int) function device_index()
      character(len=32) :: v
      integer :: st, i, n
      character(len=32), dimension(5), parameter :: names = [character(len=32) :: 'MPAS_DYCORE_DEVICE', &
         'OMPI_COMM_WORLD_LOCAL_RANK', 'MPI_LOCALRANKID', 'SLURM_LOCALID', 'LOCAL_RANK']
      device_index = -1
      do i = 1, size(names)
         call get_environment_variable(trim(names(i)), v, status=st)
         if (st /= 0) cycle
         read(v, *, iostat=st) n
         if (st == 0) then
            device_index = int(n, c_int)
            return
         end if
      end do
   end function device_index

   subroutine env_sync_switch()
      character(len=8) :: v
      integer :: st
      call get_environment_variable('MPAS_DYCORE_SYNC_EVERY_STEP', v, status=st)
      if (st == 0) atm_dycore_sync_every_step = trim(v) == '1'
      call get_environment_variable('MPAS_DYCORE_WAIT_EVERY_STEP', v, status=st)
      if (st == 0) wait_every_step = trim(v) == '1'
   end subroutine env_sync_switch

   subroutine block_dims(mesh, state, d)
      type (mpas_pool_type), intent(in) :: mesh, state
      type(dyc_dims), intent(out) :: d
      integer, pointer :: ip
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
   end subroutine block_dims

   subroutine read_config(configs, c)
      type (mpas_pool_type), intent(in) :: configs
      type(dyc_config), intent(out) :: c
      integer, pointer :: ip
      real (kind=RKIND), pointer :: rp
      logical, pointer :: lp
      character(len=StrKIND), pointer :: sp
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
   end subroutine read_config

   ! One pool field <-> its device field on block ib, as the pool's own memory image (no
   ! repacking).  dir = UP (host -> HBM) or DOWN.  A field the pool lacks, or holds at another
   ! size than the device (e.g. an inactive physics field), is skipped unless `required`.
   subroutine xfer(ctx, ib, pool, pname, name, host_tl, dev_tl, dir, required)
      type(c_ptr), intent(in) :: ctx
      integer, intent(in) :: ib, host_tl, dev_tl, dir
      type (mpas_pool_type), intent(in) :: pool
      character(len=*), intent(in) :: pname, name
      logical, intent(in) :: required
      type (mpas_pool_field_info_type) :: info
      real (kind=RKIND), pointer :: r0
      real (kind=RKIND), dimension(:), pointer :: r1
      real (kind=RKIND), dimension(:,:), pointer :: r2
      real (kind=RKIND), dimension(:,:,:), pointer :: r3
      integer, dimension(:), pointer :: i1
      integer, dimension(:,:), pointer :: i2
      type(c_ptr) :: host
      integer(c_int64_t) :: nb
      integer :: tl
      host = c_null_ptr
      nb = 0
      call mpas_pool_get_field_info(pool, name, info)
      tl = 1
      if (info % nTimeLevels > 1) tl = host_tl
      if (info % fieldType == MPAS_POOL_REAL) then
         select case (info % nDims)
         case (0)
            call mpas_pool_get_array(pool, name, r0, tl)
            if (associated(r0)) then
               host = c_loc(r0)
               nb = 8
            end if
         case (1)
            call mpas_pool_get_array(pool, name, r1, tl)
            if (associated(r1)) then
               host = c_loc(r1(1))
               nb = 8_c_int64_t * size(r1, kind=c_int64_t)
            end if
         case (2)
            call mpas_pool_get_array(pool, name, r2, tl)
            if (associated(r2)) then
               host = c_loc(r2(1,1))
               nb = 8_c_int64_t * size(r2, kind=c_int64_t)
            end if
         case (3)
            call mpas_pool_get_array(pool, name, r3, tl)
            if (associated(r3)) then
               host = c_loc(r3(1,1,1))
               nb = 8_c_int64_t * size(r3, kind=c_int64_t)
            end if
         end select
      else if (info % fieldType == MPAS_POOL_INTEGER) then
         select case (info % nDims)
         case (1)
            call mpas_pool_get_array(pool, name, i1, tl)
            if (associated(i1)) then
               host = c_loc(i1(1))
               nb = 4_c_int64_t * size(i1, kind=c_int64_t)
            end if
         case (2)
            call mpas_pool_get_array(pool, name, i2, tl)
            if (associated(i2)) then
               host = c_loc(i2(1,1))
               nb = 4_c_int64_t * size(i2, kind=c_int64_t)
            end if
         end select
      end if
      if (.not. c_associated(host) .or. nb /= mpas_dyc_block_field_bytes(ctx, int(ib, c_int32_t), &
                                                                         pname//c_null_char, name//c_null_char)) then
         if (required) call fatal(ctx, 'pool field '//pname//'.'//name//' missing or not the device size')
         return
      end if
      if (dir == UP) then
         call check(ctx, mpas_dyc_set_block_field(ctx, int(ib, c_int32_t), pname//c_null_char, name//c_null_char, &
                                                  int(dev_tl, c_int32_t), host, nb), 'set '//pname//'.'//name)
      else
         call check(ctx, mpas_dyc_get_block_field(ctx, int(ib, c_int32_t), pname//c_null_char, name//c_null_char, &
                                                  int(dev_tl, c_int32_t), host, nb), 'get '//pname//'.'//name)
      end if
   end subroutine xfer

   ! non-zero C ABI status -> fatal, as the reference's MPAS_LOG_CRIT path (mpas_log.F:612)
   subroutine check(ctx, ierr, what)
      type(c_ptr), intent(in) :: ctx
      integer(c_int), intent(in) :: ierr
      character(len=*), intent(in) :: what
      character(kind=c_char), pointer :: msg(:)
      character(len=512) :: text, line
      integer :: i
      if (ierr == 0) return
      text = ''
      if (c_associated(ctx)) then
         call c_f_pointer(mpas_dyc_last_error(ctx), msg, [512])
         do i = 1, 512
            if (msg(i) == c_null_char) exit
            text(i:i) = msg(i)
         end do
      end if
      write(line, '(a,a,i0,a,a)') what, ' failed (', ierr, '): ', trim(text)
      call fatal(c_null_ptr, trim(line))
   end subroutine check

   subroutine fatal(ctx, what)
      type(c_ptr), intent(in) :: ctx
      character(len=*), intent(in) :: what
      write(0, '(a)') 'MI355X dycore: '//what
      call mpas_log_write('MI355X dycore: '//what, messageType=MPAS_LOG_CRIT)
      error stop 1
   end subroutine fatal

end module atm_time_integration
