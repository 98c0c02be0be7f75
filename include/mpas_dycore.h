/*
 * mpas_dycore.h -- C ABI of the MI355X-native MPAS-Atmosphere dycore.
 *
 * This is the drop-in boundary behind the reference's Fortran operator API
 * (module atm_time_integration, src/core_atmosphere/dynamics/
 * mpas_atm_time_integration.F).  A Fortran shim module named
 * atm_time_integration keeps the reference's public
 * routines and binds these entry points with iso_c_binding:
 *
 *   atm_timestep(domain, dt, nowTime, itimestep)      mpas_atm_time_integration.F:87
 *       -> mpas_dyc_timestep                          (atm_srk3, :142-1796)
 *   atm_init_coupled_diagnostics(state, 1, diag, ...) mpas_atm_time_integration.F:5825
 *   atm_compute_solve_diagnostics(dt, state, 1, ...)  mpas_atm_time_integration.F:5419
 *       -> mpas_dyc_init_diagnostics                  (called at mpas_atm_core.F:390,399)
 *   mpas_pool_shift_time_levels(state)                mpas_pool_routines.F:5541
 *       -> mpas_dyc_shift_time_levels                 (called at mpas_atm_core.F:671)
 *   mpas_pool_get_array(pool, name, ptr[, timeLevel])  mpas_pool_routines.F:4282
 *       -> mpas_dyc_set_field / mpas_dyc_get_field    (pool-owned host memory <-> HBM)
 *
 * Conventions (match what the Fortran pools hold, so the shim passes pool
 * pointers unchanged):
 *   - real fields are fp64 Fortran memory images including the garbage slot:
 *     u(nVertLevels, nEdges+1), w(nVertLevels+1, nCells+1),
 *     scalars(num_scalars, nVertLevels, nCells+1), zb_cell(nVertLevels+1, maxEdges, nCells+1) ...
 *   - integer fields are int32 with MPAS 1-based indices (n+1 = garbage slot);
 *   - time_level is 1 or 2 for the state pool (ignored otherwise).
 * All functions return 0 on success and a negative MPAS_DYC_E* code on error
 * (the shim maps non-zero to mpas_log_write(..., MPAS_LOG_CRIT), which is how
 * the reference reports fatal errors, mpas_log.F:612).  No torch types, no
 * C++ types: plain pointers and sizes.
 */
#ifndef MPAS_DYCORE_H
#define MPAS_DYCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPAS_DYC_OK 0
#define MPAS_DYC_EINVAL -1    /* bad argument / unknown field / size mismatch */
#define MPAS_DYC_EHIP -2      /* HIP runtime error */
#define MPAS_DYC_ESTATE -3    /* call out of sequence */
#define MPAS_DYC_ECOMM -4     /* halo exchange failure */

/* nVertLevels: 4..MPAS_DYC_MAX_LEVELS.  Up to MPAS_DYC_MAX_LEVELS_WAVE a column is one 64-lane
 * wavefront (lane = level), or half of one in the pair layout (two levels per lane); up to
 * MPAS_DYC_MAX_LEVELS_WIDE the pair-layout kernels give a whole wavefront to one column (two levels
 * per lane) and the per-cell kernels one 128-lane workgroup, whose cross-level moves go through LDS;
 * above, every kernel runs one column per 256-lane workgroup up to MPAS_DYC_MAX_LEVELS_256, and per
 * 512-lane workgroup above (the batched per-cell and one-column edge kernels; no pair layout, so no
 * regional LBCs there).  Every kernel family and regional LBCs run at any nVertLevels up to
 * MPAS_DYC_MAX_LEVELS_WIDE. */
#define MPAS_DYC_MAX_LEVELS_WAVE 63
#define MPAS_DYC_MAX_LEVELS_WIDE 127
#define MPAS_DYC_MAX_LEVELS_256 255
#define MPAS_DYC_MAX_LEVELS 511

typedef struct mpas_dyc_ctx mpas_dyc_ctx;

/* Registry.xml dims (8-46) for one block; *Solve = owned counts (mpas_block_creator.F). */
typedef struct {
  int32_t nCells, nEdges, nVertices, nVertLevels, maxEdges, maxEdges2, num_scalars;
  int32_t nCellsSolve, nEdgesSolve, nVerticesSolve;
  int32_t moist_start, moist_end; /* 1-based, as in the state pool */
  int32_t index_qv;               /* 1-based */
} mpas_dyc_dims;

/* nhyd_model namelist (Registry.xml:56-290).  Logicals as int 0/1;
 * config_horiz_mixing: 1 = "2d_smagorinsky", 0 = "2d_fixed". */
typedef struct {
  int32_t config_time_integration_order, config_number_of_sub_steps, config_dynamics_split_steps;
  int32_t config_number_rayleigh_damp_u_levels;
  int32_t config_split_dynamics_transport, config_scalar_advection, config_positive_definite;
  int32_t config_monotonic, config_mix_full, config_rayleigh_damp_u, config_horiz_mixing;
  double config_h_mom_eddy_visc2, config_h_mom_eddy_visc4, config_v_mom_eddy_visc2;
  double config_h_theta_eddy_visc2, config_h_theta_eddy_visc4, config_v_theta_eddy_visc2;
  double config_len_disp, config_visc4_2dsmag, config_del4u_div_factor, config_coef_3rd_order;
  double config_smagorinsky_coef, config_epssm, config_smdiv, config_apvm_upwinding;
  double config_mpas_cam_coef, config_rayleigh_damp_u_timescale_days;
} mpas_dyc_config;

/* Create a dycore context on HIP device `device` (-1 = current); allocates all
 * device fields (mesh, state x2 time levels, diag, tend, module scratch).
 * device = MPAS_DYC_HOST_ONLY: a planner-only context (see mpas_dyc_plan_exchanges). */
int mpas_dyc_create(const mpas_dyc_dims* dims, const mpas_dyc_config* cfg, int device, mpas_dyc_ctx** out);
void mpas_dyc_destroy(mpas_dyc_ctx* ctx);
const char* mpas_dyc_last_error(const mpas_dyc_ctx* ctx);

/* Host <-> device copy of one named pool field (pool: "mesh","state","diag","tend",
 * "tend_physics"; scalars 0-d fields cf1/cf2/cf3 take 8 bytes). nbytes must match. */
int mpas_dyc_set_field(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level,
                       const void* host, int64_t nbytes);
int mpas_dyc_get_field(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level,
                       void* host, int64_t nbytes);
/* Size in bytes of a field's Fortran memory image (0 if unknown). */
int64_t mpas_dyc_field_bytes(const mpas_dyc_ctx* ctx, const char* pool, const char* name);
/* Raw device pointer of a field (for zero-copy use from torch / RCCL); NULL if unknown.
 * Device layout = the Fortran image, except scalars / scalars_tend, which are
 * scalar-major [num_scalars][n+1][nVertLevels] in HBM (set/get transpose them).
 * A pointer is valid until the next mpas_dyc_timestep / mpas_dyc_shift_time_levels: the step
 * rotates buffers instead of copying them, so re-query it after every step for
 *   - diag.ru, ru_save, rw, rw_save, rtheta_p, rtheta_p_save, rho_p, rho_p_save (the _save
 *     copies of atm_rk_integration_setup / atm_rk_dynamics_substep_finish, 1847-1850, 6051-6054,
 *     are buffer trades),
 *   - state.theta_m (theta_m_1 = theta_m_2 at every substep end, 6058, is a trade of its two
 *     time levels), and every state field's time levels across mpas_dyc_shift_time_levels.
 * The maxEdges / maxEdges2-strided mesh fields (edgesOnCell, cellsOnCell, verticesOnCell,
 * kiteForCell, edgesOnCell_sign, defc_a, defc_b, coeffs_reconstruct, zb_cell, zb3_cell,
 * edgesOnEdge, weightsOnEdge) return their image at the declared maxEdges; the kernels read a
 * copy at the mesh's actual cell degree (mpas_dyc_block_layout), so change them through
 * mpas_dyc_set_field, not through this pointer. */
void* mpas_dyc_field_device_ptr(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level);

/* atm_init_coupled_diagnostics + atm_compute_solve_diagnostics on time level 1
 * (model init, mpas_atm_core.F:387-404). */
int mpas_dyc_init_diagnostics(mpas_dyc_ctx* ctx, double dt);
/* The same model init for a restart (config_do_restart, mpas_atm_core.F:387-404): only
 * atm_compute_solve_diagnostics (with the init exchanges), on a state whose coupled fields
 * (theta_m, rho_zz, rho_p, rtheta_p, exner, pressure_p, ru, rw, ...) the host has set. */
int mpas_dyc_solve_diagnostics(mpas_dyc_ctx* ctx, double dt);
/* atm_timestep -> atm_srk3: advance time level 1 to time level 2 by dt. Asynchronous. */
int mpas_dyc_timestep(mpas_dyc_ctx* ctx, double dt, int32_t itimestep);
/* mpas_pool_shift_time_levels(state): swap time levels 1 and 2 (pointer swap).  Between steps, only
 * time level 1 (the state the last step produced) is defined for u and w: the step does not copy
 * u_2 / w_2 into time level 1 at its substep ends (6060-6061), because nothing reads them before
 * the next step's atm_rk_integration_setup overwrites that buffer (1852-1853).  Read u and w at
 * time level 1 after the shift. */
int mpas_dyc_shift_time_levels(mpas_dyc_ctx* ctx);
/* Block until all queued device work of the context is complete. */
int mpas_dyc_synchronize(mpas_dyc_ctx* ctx);
/* Physics coupling (the reference built with -DDO_PHYSICS, mpas_atm_time_integration.F:424-449,
 * 1610-1648, 3437, 3743).  With MPAS_DYC_PHYSICS_TENDENCIES the host (the physics package's
 * physics_get_tend, mpas_atmphys_todynamics.F:59) supplies, before each mpas_dyc_timestep,
 *   tend_physics.tend_ru_physics (K, nEdges+1), tend_physics.tend_rtheta_physics and
 *   tend_physics.tend_rho_physics (K, nCells+1), and tend.scalars_tend (ns, K, nCells+1);
 * the step adds them where the reference does (tend_u, tend_theta, tend_rho; the scalar
 * transport's scalar_tend_save / scalar_tend), and at its end sets negative scalars of time
 * level 2 to zero (1645-1646).  MPAS_DYC_PHYSICS_RQVDYNTEN also computes tend_physics.rqvdynten
 * (1629-1643; config_convection_scheme cu_grell_freitas, cu_tiedtke or cu_ntiedtke).  The
 * microphysics driver (1650-1660) stays with the host, after the step. */
#define MPAS_DYC_PHYSICS_TENDENCIES 1
#define MPAS_DYC_PHYSICS_RQVDYNTEN 2
/* MPAS_DYC_PHYSICS_MICROPHYSICS: the host runs driver_microphysics (1650-1660) after each
 * mpas_dyc_timestep, on time level 2 of the step (uploading what it changes: theta_m and scalars of
 * time level 2, rtheta_p, exner, pressure_p, rt_diabatic_tend), and then calls mpas_dyc_finish_step,
 * which runs what follows the microphysics in atm_srk3: the regional reset of the specified zone
 * (1672-1790, config_apply_lbcs) and summarize_timestep's reductions (1794).  Without this flag
 * mpas_dyc_timestep runs them itself and mpas_dyc_finish_step does nothing. */
#define MPAS_DYC_PHYSICS_MICROPHYSICS 4
int mpas_dyc_set_physics(mpas_dyc_ctx* ctx, int32_t flags);
/* The end of atm_srk3 after the host's microphysics (see MPAS_DYC_PHYSICS_MICROPHYSICS); call it
 * before mpas_dyc_shift_time_levels.  Asynchronous. */
int mpas_dyc_finish_step(mpas_dyc_ctx* ctx, double dt);
/* Regional lateral boundary conditions, config_apply_lbcs (mpas_atm_time_integration.F:683-778,
 * 934-987, 1109-1180, 1253-1270, 1491-1560, 1672-1790; the routines at 6088-6671).  apply = 1 turns
 * them on (the pair kernel layout is required).  The host sets, as in the reference's lbc pool
 * (mpas_atm_boundaries.F): lbc.lbc_u / lbc_ru (K, nEdges+1), lbc.lbc_rho_zz / lbc_rtheta_m
 * (K, nCells+1) and lbc.lbc_scalars (ns, K, nCells+1), each with time level 1 = the tendency over
 * the current LBC interval and time level 2 = the interval-end state; the mesh's bdyMaskCell,
 * bdyMaskEdge, nearestRelaxationCell, meshScalingRegionalCell / Edge; and, before every step,
 * seconds_to_interval_end = LBC interval end - the step's start time.  A driving value delta
 * seconds into the step is then state - (seconds_to_interval_end - delta) * tendency, as
 * mpas_atm_get_bdy_state (:337-409) computes it.  All scalars are driven. */
int mpas_dyc_set_lbc(mpas_dyc_ctx* ctx, int32_t apply, double seconds_to_interval_end);
/* The model-init precompute of atm_mpas_init_block (mpas_atm_core.F:311-358, 456-458; the routines at
 * 927-1288), on the device, for every block: invAreaCell, invDvEdge, invDcEdge, invAreaTriangle;
 * atm_compute_signs (edgesOnVertex_sign, edgesOnCell_sign, zb_cell, zb3_cell, kiteForCell);
 * atm_adv_coef_compression (nAdvCellsForEdge, advCellsForEdge, adv_coefs, adv_coefs_3rd);
 * atm_couple_coef_3rd_order (config_coef_3rd_order of the context's config);
 * atm_compute_mesh_scaling (meshScalingDel2 / Del4, meshScalingRegionalCell / Edge,
 * config_h_ScaleWithMesh) and atm_compute_damping_coefs (dss, config_zd, config_xnutr).
 * It reads what the init file holds, set beforehand with mpas_dyc_set_field: the connectivity,
 * dcEdge, dvEdge, zgrid and mesh.deriv_two (15, 2, nEdges+1), mesh.zb / zb3 (nVertLevels+1, 2,
 * nEdges+1), mesh.meshDensity, mesh.areaCell (nCells+1), mesh.areaTriangle (nVertices+1).
 * Every + - * / in the reference's order.  Two values are transcendental: meshDensity**0.25 and the
 * damping layer's sin.  Set them too -- mesh.meshDensity_root4 (nCells+1: meshDensity**0.25),
 * mesh.meshDensityEdge_root4 (nEdges+1: ((meshDensity(c1) + meshDensity(c2)) / 2)**0.25) and
 * mesh.dss_sin (nVertLevels, nCells+1: sin(0.5 pi (z - config_zd) / (zt - config_zd)) where z >
 * config_zd), from the C library as the compiled reference calls it -- and the outputs are the
 * reference's bits.  Unset, they are computed on the device correctly rounded; the reference's C library
 * is 1 ulp away for ~0.1 % of arguments, and meshScaling* then differ by up to 2 ulp there, dss by up to
 * 4.  Cells of more than 10 edges are refused (MPAS_DYC_EINVAL).  Synchronous. */
int mpas_dyc_model_init(mpas_dyc_ctx* ctx, int32_t h_scale_with_mesh, double config_zd, double config_xnutr);
/* deriv_two as core_init_atmosphere computes it (mpas_atm_advection.F:21-394,
 * atm_initialize_advection_rk, polynomial_order = 2, on a sphere), into mesh.deriv_two (15, 2, nEdges+1)
 * of one block (allocated if not yet set), on the device.  The transcendental half comes from the
 * caller, per cell and edgesOnCell slot (nCells x maxEdges at the declared stride, slots beyond
 * nEdgesOnCell ignored): xp / yp, the tangent-plane coordinates of cellsOnCell(i) (132-181: cos / sin
 * of thetat(i) times the arc length), and sin_the / cos_the of edgesOnCell(i)'s normal angle thetae
 * (303-315, 334-335 / 347-348).  The least-squares fit -- amatrix, poly_fit_2 with MIGS / ELGS
 * (215-226, 567-741) -- and the weights 2 cos^2 b(4,j) + 2 cos sin b(5,j) + 2 sin^2 b(6,j) (327-358)
 * run here, one thread per cell, in the Fortran's operand order: bit for bit the reference's deriv_two
 * when the inputs are its values (they are the C library's sin / cos / asin, which no device library
 * reproduces; init_atm.deriv_two_inputs computes them that way).  Uses the block's nEdgesOnCell,
 * edgesOnCell and cellsOnEdge.  Cells with more than 14 edges: MPAS_DYC_EINVAL.  Synchronous. */
int mpas_dyc_init_deriv_two(mpas_dyc_ctx* ctx, int32_t block, const double* xp, const double* yp,
                            const double* sin_the, const double* cos_the);
/* zb / zb3, the z-metric terms of the omega equation, as core_init_atmosphere computes them
 * (mpas_init_atm_cases.F:1045-1093) for config_theta_adv_order 2, 3 or 4, into mesh.zb / mesh.zb3
 * (nVertLevels+1, 2, nEdges+1) of one block (allocated if not yet set), on the device, from the block's
 * mesh.deriv_two, zgrid, dcEdge, dvEdge, areaCell and connectivity.  Edges with no owned cell and
 * level nVertLevels+1 are 0.  Bit for bit the reference's arithmetic.  Synchronous. */
int mpas_dyc_init_zb(mpas_dyc_ctx* ctx, int32_t block, int32_t theta_adv_order);
/* The reconstruction coefficients of every block on the device: mpas_rbf_interp_initialize's vectors
 * (operators/mpas_vector_operations.F:697-769: edge normals, each cell's tangent plane) and
 * mpas_init_reconstruct (operators/mpas_vector_reconstruction.F:112-177: the inverse-multiquadric RBF
 * system of each cell's edges with a constant vector in the plane, solved by elgs + mpas_legs), what
 * mpas_atm_core.F:408-409 runs at model init, into mesh.coeffs_reconstruct.  Reads mesh.xCell, yCell,
 * zCell (nCells+1), xEdge, yEdge, zEdge (nEdges+1), set beforehand, and the connectivity.  + - * / sqrt
 * only, in the Fortran's order: bit for bit the reference's coefficients.  Cells with more than 14
 * edges: MPAS_DYC_EINVAL.  Synchronous. */
int mpas_dyc_init_reconstruct(mpas_dyc_ctx* ctx);
/* atm_compute_output_diagnostics(state, time_level, diag, mesh) (mpas_atm_core.F:753, called
 * before history writes at :544 and :694): diag theta, rho and pressure from theta_m, rho_zz,
 * scalars(index_qv) of the time level, zz, pressure_base and pressure_p.  Asynchronous. */
int mpas_dyc_output_diagnostics(mpas_dyc_ctx* ctx, int32_t time_level);

/* ---- summarize_timestep (mpas_atm_time_integration.F:6675-7018, called at the end of atm_srk3, 1794) ----
 * The modes are the namelist switches of the reference; each step reduces the enabled ones on
 * the device (part of mpas_dyc_timestep, captured with the step), and mpas_dyc_get_summary
 * folds the blocks of this process and, over RCCL, all ranks. */
#define MPAS_DYC_PRINT_GLOBAL_MINMAX_VEL 1   /* config_print_global_minmax_vel (default .true.), 6945-6983 */
#define MPAS_DYC_PRINT_DETAILED_MINMAX_VEL 2 /* config_print_detailed_minmax_vel, 6721-6943 */
#define MPAS_DYC_PRINT_GLOBAL_MINMAX_SCA 4   /* config_print_global_minmax_sca, 6986-7016 */

/* One located extreme of the detailed mode: the value, the level and the lat/lon in degrees of
 * the first owned element (cell-major, level-minor) holding it, as the reference's loops find it,
 * reduced over ranks as mpas_dmpar_min/maxattributes_real does (MPI_MINLOC / MPI_MAXLOC per
 * attribute, mpas_dmpar.F:1090-1160).  lon is shifted to (-180, 180] as at 6771-6773. */
typedef struct {
  double value, lat, lon;
  int32_t k;      /* 1-based level (kMax_global); -1 if no element */
  int32_t index;  /* 1-based local index on its block (indexMax); -1 if no element */
} mpas_dyc_extreme;

typedef struct {
  int32_t flags;                     /* the modes the values below were reduced for */
  double w_min, w_max, u_min, u_max; /* global_minmax_vel: min/max over owned w, u starting from 0.0 */
  mpas_dyc_extreme w_min_at, w_max_at, u_min_at, u_max_at, wsp_max_at; /* detailed_minmax_vel */
  int64_t nan_w, nan_u;              /* NaNs in the owned w, u (the detailed mode aborts on any, 6926-6940) */
} mpas_dyc_summary;

/* Modes reduced by every following step (default MPAS_DYC_PRINT_GLOBAL_MINMAX_VEL; 0 = none). */
int mpas_dyc_set_summary(mpas_dyc_ctx* ctx, int32_t flags);
/* The last step's summary over all blocks and ranks (collective when ranks share a communicator:
 * every rank calls it after the same step).  Waits for the step.  scalar_minmax (may be NULL)
 * receives num_scalars (min, max) pairs of the global_minmax_sca mode; n = its length in doubles. */
int mpas_dyc_get_summary(mpas_dyc_ctx* ctx, mpas_dyc_summary* out, double* scalar_minmax, int32_t n);
/* The same for one block of this process, reduced over ranks: the reference writes one set of log
 * lines per block of a task, each reduced over tasks (6945-6983, 6991-7015).  Collective like
 * mpas_dyc_get_summary: every rank calls it for the same block index after the same step. */
int mpas_dyc_get_block_summary(mpas_dyc_ctx* ctx, int32_t block, mpas_dyc_summary* out, double* scalar_minmax,
                               int32_t n);

/* ---- domain decomposition: several blocks per process, halo exchange ----
 *
 * A context holds the blocks this process owns (MPAS domain%blocklist; one per
 * GPU in production, several per GPU in tests).  Each block has its own dims
 * (owned-first element order, nCellsSolve etc. = owned counts, as built by
 * mpas_block_creator.F) and its own fields, addressed with the *_block_field
 * variants (the functions above act on block 0).  Halo exchanges happen inside
 * mpas_dyc_timestep at the reference's mpas_dmpar_exch_halo_field points
 * (mpas_atm_time_integration.F:329-1717, 3757, 4098): block-to-block copies
 * inside the process, RCCL ncclSend/ncclRecv between processes. */
#define MPAS_DYC_CELL 0
#define MPAS_DYC_EDGE 1
#define MPAS_DYC_VERTEX 2
#define MPAS_DYC_SEND 0
#define MPAS_DYC_RECV 1

int mpas_dyc_create_blocks(int32_t nblocks, const mpas_dyc_dims* dims /* [nblocks] */, const mpas_dyc_config* cfg,
                           int device, mpas_dyc_ctx** out);
int32_t mpas_dyc_num_blocks(const mpas_dyc_ctx* ctx);
int mpas_dyc_set_block_field(mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name,
                             int32_t time_level, const void* host, int64_t nbytes);
int mpas_dyc_get_block_field(mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name,
                             int32_t time_level, void* host, int64_t nbytes);
int64_t mpas_dyc_block_field_bytes(const mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name);
void* mpas_dyc_block_field_device_ptr(mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name,
                                      int32_t time_level);
/* One entry of a block's multihalo exchange list (mpas_dmpar.F mpas_multihalo_exchange_list:
 * procID/blockID/nList/srcList|destList): the elements of `location` in halo layer
 * `halo_layer` (cells 1..2, edges/vertices 1..3) that this block sends to (owned elements)
 * or receives from (halo elements) block `peer_block` of rank `peer_rank`, as 1-based local
 * indices in message order.  Both sides must list the same elements in the same order. */
int mpas_dyc_set_exchange_list(mpas_dyc_ctx* ctx, int32_t block, int32_t location, int32_t halo_layer,
                               int32_t direction, int32_t peer_rank, int32_t peer_block, const int32_t* local_index,
                               int32_t n);
/* A list of another task as mpas_dmpar keeps it when tasks hold several blocks (parinfo xToSend /
 * xToRecv: endPointID = the task, the other list = buffer positions; mpas_dmpar.F:5448-5535): this
 * block's elements local_index[i] (1-based; owned to send, halo to receive) take 1-based slot
 * position[i] of the (location, halo_layer) region of the one message between this task and task
 * peer_rank, whose slots all blocks of this task fill together.  The message is laid out as
 * mpas_dmpar lays out its buffer -- per field of the exchange, per halo layer a region as long as its
 * largest position -- so a task need not know which block of the peer receives an element.  A peer
 * rank takes either positional lists or block-pair lists (mpas_dyc_set_exchange_list), not both. */
int mpas_dyc_set_exchange_positions(mpas_dyc_ctx* ctx, int32_t block, int32_t location, int32_t halo_layer,
                                    int32_t direction, int32_t peer_rank, const int32_t* local_index,
                                    const int32_t* position, int32_t n);
/* RCCL communicator for exchanges between processes (one rank per GPU): rank 0 creates the
 * id (ncclGetUniqueId), every rank passes it to mpas_dyc_comm_init (ncclCommInitRank). */
int64_t mpas_dyc_comm_unique_id_bytes(void);
int mpas_dyc_comm_unique_id(void* id, int64_t nbytes);
int mpas_dyc_comm_init(mpas_dyc_ctx* ctx, const void* id, int64_t nbytes, int32_t nranks, int32_t rank);
/* Ranks without RCCL: the host's own all-gather (MPI_Allgather, a torch.distributed gloo group, ...)
 * for the few set-up collectives, and the one-sided transfer (mpas_dyc_set_p2p, switched on here) for
 * every halo message -- all ranks on one node.  fn(send, recv, nbytes, user) must place every rank's
 * nbytes in recv in rank order and return 0; it is called from mpas_dyc_timestep /
 * mpas_dyc_init_diagnostics / mpas_dyc_halo_exchange (set-up of new exchange points, on every rank at
 * the same call) and from mpas_dyc_get_summary, never during graph capture.  Instead of
 * mpas_dyc_comm_init; a context has one or the other. */
typedef int (*mpas_dyc_allgather_fn)(const void* send, void* recv, int64_t nbytes, void* user);
int mpas_dyc_comm_init_host(mpas_dyc_ctx* ctx, int32_t nranks, int32_t rank, mpas_dyc_allgather_fn fn, void* user);
/* Test hook: route block-to-block exchanges inside this process through RCCL (send to self). */
int mpas_dyc_set_transport(mpas_dyc_ctx* ctx, int32_t rccl_for_local_blocks);
/* One-sided transfer between the ranks of one node (on = 1; 0 = RCCL groups; -1 = the environment
 * variable MPAS_DYCORE_P2P, read at context creation, default 0).  Replaces the ncclSend / ncclRecv
 * groups of every exchange point by kernels that move the halo themselves (halo.hip), with flags in
 * each rank's arena (ready / consumed counters, IPC-mapped by the peers at set-up).  Blocking
 * exchanges with block-pair lists (the default) are pulls: k_p2p_pull copies the peer's owned
 * columns from its fields (IPC-mapped) straight into this rank's halo columns.  Positional lists and
 * split-phase exchanges (MPAS_DYCORE_P2P_PULL=0 for all) keep the send / receive buffers: the pack
 * fills this rank's send buffer (device memory the peers map), k_p2p_post raises ready, and
 * k_p2p_get pulls each peer's message and waits until this rank's own buffer has been pulled.  Same
 * messages and order as the RCCL path (the plans are the ones mpas_dyc_plan_exchanges reports).
 * Set-up runs once per exchange-plan build, over the communicator of mpas_dyc_comm_init (or the host
 * all-gather of mpas_dyc_comm_init_host); if IPC is refused or the ranks span several nodes, every
 * rank drops the transfer together and plans for RCCL (mpas_dyc_get_p2p then returns 0).  A message
 * that does not arrive within 30 s makes mpas_dyc_synchronize return MPAS_DYC_ECOMM.  Collective:
 * every rank calls it with the same value. */
int mpas_dyc_set_p2p(mpas_dyc_ctx* ctx, int32_t on);
/* 1 while the one-sided transfer is on (0 after the set-up found it unavailable on some rank -- IPC
 * refused, ranks on several nodes -- and every rank went back to RCCL, with a line on stderr). */
int mpas_dyc_get_p2p(const mpas_dyc_ctx* ctx);
/* Split-phase exchanges: at the tend_u, rho_pp and rtheta_pp exchanges the interior
 * elements are computed while the halo traffic runs on a second stream.  on = 1 / 0;
 * -1 (default) = automatic: on when exchanges go through RCCL (more than one rank). */
int mpas_dyc_set_overlap(mpas_dyc_ctx* ctx, int32_t on);
/* mpas_dmpar_exch_halo_field(field, haloLayers) for one field; layer_mask bit l-1 = layer l. */
int mpas_dyc_halo_exchange(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level,
                           int32_t layer_mask);

/* ---- exchange-plan dry run (no device) ----
 * `device` = MPAS_DYC_HOST_ONLY in mpas_dyc_create(_blocks) makes a context that holds dims,
 * config and exchange lists but no device memory, stream or communicator.  Only
 * mpas_dyc_set_exchange_list, mpas_dyc_set_overlap / _set_transport and
 * mpas_dyc_plan_exchanges work on it (field calls return MPAS_DYC_ESTATE).  It lets a host
 * check, before any GPU is touched, that the RCCL messages every rank will post match: rank r's
 * sends to rank p at an exchange point must be rank p's receives from r there, in the same
 * order and of the same sizes (what ncclGroupStart/End requires, mpas_dmpar.F:5386-5552). */
#define MPAS_DYC_HOST_ONLY (-2)

/* One RCCL message of an exchange point, as the step posts it. */
typedef struct {
  int32_t point;      /* 0-based index of the exchange call in issue order (see below) */
  int32_t direction;  /* MPAS_DYC_SEND (ncclSend) / MPAS_DYC_RECV (ncclRecv) */
  int32_t block;      /* local block that packs / unpacks it */
  int32_t peer_rank, peer_block;
  int64_t count;      /* doubles */
} mpas_dyc_plan_msg;

/* Run the exchange planner as rank `rank` of `nranks` over the calls one model run issues, in
 * order: the model-init exchanges (mpas_dyc_init_diagnostics), then one atm_srk3 on each
 * time-level parity (a step, mpas_dyc_shift_time_levels, a step).  Writes up to `cap` messages
 * (each point's sends, then its receives, in posting order) and sets *n_msgs to the number
 * needed; writes the calls' plan keys, one per line in issue order, into keys[keys_bytes]
 * (NUL-terminated) and sets *keys_len to the bytes needed.  Returns MPAS_DYC_EINVAL when
 * either buffer was too small (the counts are still set). */
int mpas_dyc_plan_exchanges(mpas_dyc_ctx* ctx, int32_t nranks, int32_t rank, double dt, mpas_dyc_plan_msg* msgs,
                            int64_t cap, int64_t* n_msgs, char* keys, int64_t keys_bytes, int64_t* keys_len);

/* 1 if the last mpas_dyc_timestep replayed a captured hipGraph, 0 if it ran eagerly.  With more
 * than one rank a failed capture is an error (MPAS_DYC_EHIP), never a per-rank eager fallback:
 * one eager rank would add ~280 launches per dt to every exchange wait of the others. */
int mpas_dyc_graph_active(const mpas_dyc_ctx* ctx);

/* ---- measurement hooks (bench.py / tests) ---- */
/* A `reps`-sub-step acoustic loop (atm_advance_acoustic_step + atm_divergence_damping_3d per
 * sub-step, srk3 :788-870) of block 0 on the current state, all sub-steps numbered
 * `small_step`, timed with HIP events on the compute stream.  The launches are the ones srk3
 * issues: the edge phase, the cell phase, and for every further sub-step the edge phase with
 * the previous sub-step's damping fused in.  The last sub-step's damping is its own kernel.
 * reps = 1 is exactly one sub-step followed by its damping.
 * Returns the average time per sub-step in *ms_out.  ms_kernels[3] (may be NULL) gets
 * {edge phases, cell phases, the standalone damping}, each summed and divided by reps. */
int mpas_dyc_time_acoustic_step(mpas_dyc_ctx* ctx, double dts, int32_t small_step, int32_t reps,
                                double* ms_out, double* ms_kernels);
/* Capture one full timestep in a hipGraph and replay it for subsequent
 * mpas_dyc_timestep calls (1 = on, 0 = off). */
int mpas_dyc_use_graph(mpas_dyc_ctx* ctx, int32_t on);
/* Algorithmic HBM bytes of one acoustic sub-step of block 0 (B_ac). */
double mpas_dyc_acoustic_bytes(const mpas_dyc_ctx* ctx);
/* Exchange profile of a multi-rank run (bench.py --gpus N): with on = 1 every following
 * mpas_dyc_timestep runs eagerly (no hipGraph) with HIP events around the exposed part of each
 * halo exchange -- a blocking exchange whole, a split-phase one from the moment the compute stream
 * reaches the join until the exchange stream's work has completed -- and around each RCCL group.
 * mpas_dyc_get_profile then returns, for the last such step: out[0] = exchanges waited on,
 * out[1] = ms of the step (events on the compute stream), out[2] = ms of exposed exchange time,
 * out[3] = RCCL groups issued, out[4] = ms inside them (mostly overlapped with compute). */
int mpas_dyc_set_profile(mpas_dyc_ctx* ctx, int32_t on);
int mpas_dyc_get_profile(mpas_dyc_ctx* ctx, double* out, int32_t n);
/* The plan key of the exchange whose RCCL group was enqueued last ("warm_rccl <key>" while the
 * connections are set up before graph capture, which synchronises after every group): what a
 * watchdog reports when a rank hangs in RCCL.  Safe to read from another thread (a fixed buffer). */
const char* mpas_dyc_last_exchange(const mpas_dyc_ctx* ctx);
/* ncclGetVersion of the RCCL the library links (e.g. 22703 = 2.27.3), -1 on error. */
int32_t mpas_dyc_rccl_version(void);
/* How the kernels see a block, once its mesh is set (computed on the first call that needs it):
 * out[0] = maxEdges the kernels index with (max(nEdgesOnCell), at least 6 -- mesh files may
 * declare more, e.g. 10, Registry.xml:13-16), out[1] = maxEdges2 likewise, out[2] = kernel
 * family (0 one column per element, 1 batched stencil records, 2 pair layout: two elements per
 * wavefront, two levels per lane -- one element per wavefront above MPAS_DYC_MAX_LEVELS_WAVE),
 * out[3] = column shape (0 one wavefront, 1 nVertLevels > MPAS_DYC_MAX_LEVELS_WAVE: one 128-lane
 * workgroup per column in the per-cell kernels, one wavefront per column in the pair layout; 2
 * nVertLevels > MPAS_DYC_MAX_LEVELS_WIDE: one 256-lane workgroup per column in every kernel; 3
 * nVertLevels > MPAS_DYC_MAX_LEVELS_256: one 512-lane workgroup per column). */
int mpas_dyc_block_layout(mpas_dyc_ctx* ctx, int32_t block, int32_t* out /* [4] */);

#ifdef __cplusplus
}
#endif
#endif /* MPAS_DYCORE_H */
