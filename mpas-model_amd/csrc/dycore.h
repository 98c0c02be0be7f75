// MI355X-native MPAS split-explicit dycore: device data model shared by the
// kernels (kernels.hip) and the host sequencer (dycore.hip).
//
// Layout in HBM: every MPAS array keeps its Fortran memory
// image (K, n+1) == element-major [n+1][K] -- one contiguous column of K (or
// K+1) fp64 levels per cell/edge/vertex, k the fast axis -- including the
// garbage slot n+1 (device index n).  Index arrays are converted once to
// 0-based int32 with "missing" -> n (the garbage slot).  A 64-lane wavefront
// owns one column (lane = k), so every column read is a 448 B (K=56)
// coalesced segment and neighbour gathers fetch whole columns.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpas {

// core_atmosphere constants: src/framework/mpas_constants.F:25-36 (promoted to double)
constexpr double GRAVITY = 9.80616;
constexpr double RGAS = 287.0;
constexpr double RV = 461.6;
constexpr double CP = 7.0 * RGAS / 2.0;
constexpr double CV = CP - RGAS;
constexpr double RVORD = RV / RGAS;
constexpr double PRANDTL = 1.0;
constexpr double P0 = 1.0e5;   // mpas_atm_time_integration.F:2985, 5907
constexpr double SECONDS_PER_DAY = 86400.0;
// regional boundary zones (core_atmosphere/dynamics/mpas_atm_boundaries.F:10-12): bdyMask 1..5
// relaxation, > 5 specified
constexpr int N_SPEC_ZONE = 2, N_RELAX_ZONE = 5;

struct Dims {
  int nCells, nEdges, nVertices, K, maxEdges, maxEdges2, ns;
  int nCellsSolve, nEdgesSolve, nVerticesSolve;
  int moist_start, moist_end;  // 0-based inclusive range of moist scalars
  int diabatic;                // rt_diabatic_tend holds nonzero data (else it is read as 0)
  int physics;                 // DO_PHYSICS coupling: tend_*_physics and scalars_tend come from the host
  int lbc;                     // config_apply_lbcs: regional lateral boundary conditions (lbc.hip)
  // lengths of the compact phase-2 lists of the split-phase kernels (compute_bnd; Ptrs::bnd_*)
  int n_bnd_edges, n_bnd_pairs, n_bnd_cells;
};

struct Config {
  int time_integration_order, number_of_sub_steps, dynamics_split_steps;
  int number_rayleigh_damp_u_levels;
  int split_dynamics_transport, scalar_advection, positive_definite, monotonic, mix_full;
  int rayleigh_damp_u, horiz_mixing_smag;  // horiz_mixing: 1 = 2d_smagorinsky, 0 = 2d_fixed
  double h_mom_eddy_visc2, h_mom_eddy_visc4, v_mom_eddy_visc2;
  double h_theta_eddy_visc2, h_theta_eddy_visc4, v_theta_eddy_visc2;
  double len_disp, visc4_2dsmag, del4u_div_factor, coef_3rd_order, smagorinsky_coef;
  double epssm, smdiv, apvm_upwinding, mpas_cam_coef, rayleigh_damp_u_timescale_days;
};

// Device pointers handed to every kernel (by value, in kernarg memory).
// Time-level fields are resolved to tl1/tl2 on the host before each launch.
constexpr int CELL_HALO_EDGE = 1, CELL_BND_EDGE = 2;

struct Ptrs {
  // ---- mesh: connectivity (0-based, missing -> n)
  const int *nEdgesOnCell, *edgesOnCell, *cellsOnCell, *verticesOnCell, *kiteForCell;
  const int *cellsOnEdge, *verticesOnEdge, *nEdgesOnEdge, *edgesOnEdge;
  const int *nAdvCellsForEdge, *advCellsForEdge, *cellsOnVertex, *edgesOnVertex;
  // ---- mesh: geometry / coefficients
  const double *dcEdge, *dvEdge, *invDcEdge, *invDvEdge, *invAreaCell, *invAreaTriangle;
  const double *fEdge, *fVertex, *meshScalingDel2, *meshScalingDel4, *specZoneMaskEdge, *specZoneMaskCell;
  const double *fzm, *fzp, *rdzw, *rdzu;
  const double *edgesOnCell_sign, *edgesOnVertex_sign, *kiteAreasOnVertex, *weightsOnEdge;
  const double *adv_coefs, *adv_coefs_3rd, *defc_a, *defc_b;
  const double *zgrid, *zz, *zxu, *dss, *zb_cell, *zb3_cell;
  const double *zb_p, *zb_m;  // scratch: zb_cell + zb3_cell and zb_cell - zb3_cell (k_build_zb)
  const double *u_init, *v_init, *t_init, *angleEdge;
  const double *latCell, *lonCell, *coeffs_reconstruct;
  double cf1, cf2, cf3;
  // ---- state, two time levels resolved per launch
  double *u1, *u2, *w1, *w2, *theta_m1, *theta_m2, *rho_zz1, *rho_zz2, *scalars1, *scalars2;
  // ---- diag
  double *theta, *rho, *rho_base, *theta_base, *rho_p, *rho_p_save, *rho_pp, *rho_zz_old_split;
  double *rtheta_base, *rtheta_p, *rtheta_p_save, *rtheta_pp, *rtheta_pp_old;
  double *exner, *exner_base, *pressure_base, *pressure_p, *pressure, *h_divergence, *kdiff, *ke, *divergence;
  double *pv_cell, *tend_rtheta_adv, *cqw, *cofwr, *cofwz, *cofwt, *coftz, *a_tri, *alpha_tri, *gamma_tri, *cofrz;
  double *rw, *rw_p, *rw_save, *wwAvg, *wwAvg_split;
  // what the acoustic cell phase reads for rw, w (tl2) and rho_zz (tl2): the fields themselves,
  // except in a dynamics substep's first stage (srk3 stage_fin), whose recovery writes the fields
  const double *rw_rd, *w2_rd, *rho_zz2_rd;
  double *ru, *ruAvg, *ruAvg_split, *ru_p, *ru_save, *cqu, *rho_edge, *v, *pv_edge, *gradPVn, *gradPVt;
  double *vorticity, *pv_vertex;
  double *uReconstructX, *uReconstructY, *uReconstructZ, *uReconstructZonal, *uReconstructMeridional;
  // ---- tend / tend_physics
  double *tend_u, *tend_u_euler, *tend_w, *tend_w_euler, *tend_theta, *tend_theta_euler;
  double *tend_rho, *rt_diabatic_tend, *scalars_tend, *rthdynten, *rqvdynten;
  // ---- module scratch (mpas_atm_time_integration.F:35-71)
  double *qtot, *tend_ru_physics, *tend_rtheta_physics, *tend_rho_physics;
  double *delsq_theta, *delsq_w, *delsq_divergence, *delsq_u, *delsq_vorticity, *dpdz;
  double *ke_vertex, *ke_edge, *horiz_flux_array;
  double *s_max, *s_min, *scale_arr, *flux_arr, *flux_upwind_tmp, *flux_tmp, *wdtn, *rho_zz_int;
  double *scalar_old_copy;
  double *advflux_w, *advflux_th;  // edge values of w / theta_m for horizontal advection
  // split-phase flags.  edge_bnd: 1 = a cell of the edge is a halo cell.  cell_bnd bits:
  // CELL_HALO_EDGE = an edge of the cell is a halo edge, CELL_BND_EDGE = an edge of the cell has
  // edge_bnd set; halo cells have both bits.
  const int *edge_bnd, *cell_bnd;
  // phase 2 (halo-boundary elements) of a split kernel walks a compact list instead of testing
  // the flag on every element: bnd_edges = edges with edge_bnd set (k_recover_edges), bnd_pairs =
  // those of them with an owned cell (the pair-layout acoustic edge phase and damping),
  // bnd_cells = owned cells with CELL_HALO_EDGE (k_smlstep_pert_b); ascending element order
  const int *bnd_edges, *bnd_pairs, *bnd_cells;
  // per-cell stencil records (built on the device from edgesOnCell / cellsOnEdge / dvEdge,
  // k_build_cell_rec): cell_rec = 16 int32 per cell, [0, 7) edgesOnCell, [7, 14) the cell across
  // each of those edges, [14] nEdgesOnCell, unused slots -> garbage element; cell_sdv =
  // edgesOnCell_sign * dvEdge (maxEdges doubles per cell).  A cell reads its whole stencil with
  // one scalar load.
  const int* cell_rec;
  const double* cell_sdv;
  // ---- regional LBCs (lbc.hip): zone masks, relaxation scaling, the driving data of the lbc pool
  // (_t = tendency, lbc_<field> time level 1; _s = interval-end state, time level 2), the seconds
  // from the step start to the interval end, and the scalar filter's scratch
  const int *bdyMaskCell, *bdyMaskEdge, *nearestRelaxationCell;
  const double *meshScalingRegionalCell, *meshScalingRegionalEdge;
  const double *lbc_u_t, *lbc_u_s, *lbc_ru_t, *lbc_ru_s, *lbc_rho_zz_t, *lbc_rho_zz_s;
  const double *lbc_rtheta_m_t, *lbc_rtheta_m_s, *lbc_scalars_t, *lbc_scalars_s;
  const double* lbc_dtr;
  double* lbc_tmp;
};
constexpr int CELL_REC = 16, CELL_REC_ME = 7;

// Halo pack fused into a producer (the acoustic cell phase, k_acoustic_cells_r): owned cell c of the
// block writes its new rtheta_pp (and rho_pp) column also to rt[s] (rho[s]) for s in
// [start[c], start[c+1]) -- its slots in the RCCL send buffer of the per-sub-step exchange
// (mpas_atm_time_integration.F:845, 792).  start == nullptr: nothing to pack.
struct PackMap {
  const int* start;      // nCellsSolve + 1 offsets
  double* const* rt;     // send-buffer column of rtheta_pp per slot
  double* const* rho;    // send-buffer column of rho_pp per slot, or nullptr
};

// Halo unpack fused into the consumer (the next acoustic edge phase, or the stage's last divergence
// damping, k_acoustic_edges_p / k_divdamp_p): a halo cell h with rt[h - nCellsSolve] >= 0 has its
// exchanged rtheta_pp column at recv + rt[..] (rho_pp: recv + rho[..]); the consumer reads it there
// and writes it into the field for the later readers.  recv == nullptr: the fields hold the values.
struct UnpackMap {
  const double* recv;
  const int* rt;
  const int* rho;  // nullptr: rho_pp not in this exchange
};

// The same for the exchange before the large-step recovery (mpas_atm_time_integration.F:876-887:
// rw_p, ru_p, rho_pp all halo layers, rtheta_pp layer 2), whose producers are the stage's last
// acoustic cell phase (cells) and last damping (edges) and whose consumers are the recovery of the
// halo cells and halo edges (k_recover_cells1 / k_recover_edges), so the exchange launches no
// k_halo_copy.  Fields by index: cells 0 = rw_p (K+1 levels), 1 = rho_pp, 2 = rtheta_pp; edges
// 0 = ru_p.
// XPack: owned element i writes field fid[s] of its new column also to dst[s], s in
// [start[i], start[i+1]).  start == nullptr: nothing to pack.
struct XPack {
  const int* start;
  const int* fid;
  double* const* dst;
};
// XUnpack: halo element i (i >= nSolve) has field f's received column at recv + off[f * nh + i -
// nSolve] (-1: not in this exchange); the consumer reads it there and writes it into the field.
// The u exchange after the recovery (988) is the third such point: packed where the recovery
// computes u (k_divdamp_p<REC>, k_recover_edges), unpacked by the diagnostics' vertex kernel
// (k_diag_vertices_p), the first reader of u's halo.
// recv == nullptr: the fields hold the values.
struct XUnpack {
  const double* recv;
  const int* off;
  int nh;
  // wb (optional): the consumer element that writes halo element i's column back into the field
  // (wb[i - nSolve]), when several of the consumer's elements read it
  const int* wb;
};

}  // namespace mpas
