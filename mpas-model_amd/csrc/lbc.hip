// Regional (limited-area) lateral boundary conditions, config_apply_lbcs = .true.
// (mpas_atm_time_integration.F:683-778, 934-987, 1109-1180, 1253-1270, 1491-1560, 1672-1790 call
// sites; the routines at 6088-6671).
//
// Zones (mesh bdyMaskCell / bdyMaskEdge, mpas_atm_boundaries.F:10-12): 0 interior, 1..nRelaxZone
// relaxation (1 unused by the filters), > nRelaxZone specified.  Driving values follow
// mpas_atm_get_bdy_state (mpas_atm_boundaries.F:337-409): the host keeps the LBC interval's end
// state (lbc_<field> time level 2) and its tendency (time level 1); a value delta seconds into the
// step is  state - (dtr - delta) * tend,  dtr = seconds from the step start to the interval end
// (*p.lbc_dtr, set by the host before every step).  One wave per column, lane = level.
#pragma once
#include "dycore.h"

namespace mpas {

__global__ void k_set_f64(double* p, double v) { *p = v; }

// mpas_atm_get_bdy_state's expression: dt = dtr - delta_t; state - dt * tend
__device__ __forceinline__ double lbc_drive(const double* st, const double* tn, size_t o, double dtl) {
  return st[o] - dtl * tn[o];
}

// atm_bdy_adjust_dynamics_speczone_tend (6147-6200): owned specified-zone cells / edges take the
// driving tendencies (mpas_atm_get_bdy_tend, the time-level-1 arrays); tend_rw and
// rt_diabatic_tend are zeroed on levels 1..nVertLevels
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_spec_tend_cells(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve || p.bdyMaskCell[c] <= N_RELAX_ZONE) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)c * K + k;
  p.tend_rho[o] = p.lbc_rho_zz_t[o];
  p.tend_theta[o] = p.lbc_rtheta_m_t[o];
  p.tend_w[(size_t)c * (K + 1) + k] = 0.0;
  p.rt_diabatic_tend[o] = 0.0;
}
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_spec_tend_edges(Dims d, Ptrs p) {
  const int e = wave_elem(0);
  if (e >= d.nEdgesSolve || p.bdyMaskEdge[e] <= N_RELAX_ZONE) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)e * K + k;
  p.tend_u[o] = p.lbc_ru_t[o];
}

// atm_bdy_adjust_dynamics_relaxzone_tend (6204-6391), cells: Rayleigh damping of rho_zz and
// rho_zz*theta_m (state time level 2) toward the driving values, then the Laplacian filter of
// their departures over the cell's edges.  Owned cells with 1 < mask <= nRelaxZone.
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_relax_cells(Dims d, Ptrs p, double dt, double delta) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int m = p.bdyMaskCell[c];
  if (!(m > 1 && m <= N_RELAX_ZONE)) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const double dtl = *p.lbc_dtr - delta;
  const size_t o = (size_t)c * K + k;
  const double msr = p.meshScalingRegionalCell[c];
  const double rdc = ((double)m - 1.) / (double)N_RELAX_ZONE / (50. * dt * msr);
  double trho = p.tend_rho[o], trt = p.tend_theta[o];
  trho = trho - rdc * (p.rho_zz2[o] - lbc_drive(p.lbc_rho_zz_s, p.lbc_rho_zz_t, o, dtl));
  trt = trt - rdc * (p.rho_zz2[o] * p.theta_m2[o] - lbc_drive(p.lbc_rtheta_m_s, p.lbc_rtheta_m_t, o, dtl));
  const double lfc = ((double)m - 1.) / (double)N_RELAX_ZONE / (10. * dt * msr);
  const int ne = p.nEdgesOnCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = p.edgesOnCell[(size_t)c * d.maxEdges + i];
    const double es = p.edgesOnCell_sign[(size_t)c * d.maxEdges + i] * p.dvEdge[e] * p.invDcEdge[e] * lfc;
    const size_t o1 = (size_t)p.cellsOnEdge[2 * e] * K + k, o2 = (size_t)p.cellsOnEdge[2 * e + 1] * K + k;
    trt = trt + es * ((p.rho_zz2[o2] * p.theta_m2[o2] - lbc_drive(p.lbc_rtheta_m_s, p.lbc_rtheta_m_t, o2, dtl)) -
                      (p.rho_zz2[o1] * p.theta_m2[o1] - lbc_drive(p.lbc_rtheta_m_s, p.lbc_rtheta_m_t, o1, dtl)));
    trho = trho + es * ((p.rho_zz2[o2] - lbc_drive(p.lbc_rho_zz_s, p.lbc_rho_zz_t, o2, dtl)) -
                        (p.rho_zz2[o1] - lbc_drive(p.lbc_rho_zz_s, p.lbc_rho_zz_t, o1, dtl)));
  }
  p.tend_rho[o] = trho;
  p.tend_theta[o] = trt;
}

// the same routine, edges (every edge of the block, edgeStart..edgeEnd): Rayleigh damping of ru
// (diag) toward the driving ru, then the filter built from the divergence of (ru - ru_driving)
// at the edge's two cells and its vorticity at the edge's two vertices
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_relax_edges(Dims d, Ptrs p, double dt, double delta) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int m = p.bdyMaskEdge[e];
  if (!(m > 1 && m <= N_RELAX_ZONE)) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const double dtl = *p.lbc_dtr - delta;
  const size_t o = (size_t)e * K + k;
  const double msr = p.meshScalingRegionalEdge[e];
  auto dru = [&](int ee) {
    const size_t oo = (size_t)ee * K + k;
    return p.ru[oo] - lbc_drive(p.lbc_ru_s, p.lbc_ru_t, oo, dtl);
  };
  const double rdc = ((double)m - 1.) / (double)N_RELAX_ZONE / (50. * dt * msr);
  double tu = p.tend_u[o] - rdc * dru(e);
  const double dc = p.dcEdge[e];
  const double lfc = dc * dc * ((double)m - 1.) / (double)N_RELAX_ZONE / (10. * dt * msr);
  const double r_dc = p.invDcEdge[e], r_dv = fmin(p.invDvEdge[e], 4. * p.invDcEdge[e]);
  double div[2], vor[2];
  for (int s = 0; s < 2; ++s) {
    const int c = p.cellsOnEdge[2 * e + s];
    const double invA = p.invAreaCell[c];
    double dv = 0.0;
    const int ne = p.nEdgesOnCell[c];
    for (int i = 0; i < ne; ++i) {
      const int ed = p.edgesOnCell[(size_t)c * d.maxEdges + i];
      const double es = invA * p.dvEdge[ed] * p.edgesOnCell_sign[(size_t)c * d.maxEdges + i];
      dv = dv + es * dru(ed);
    }
    div[s] = dv;
    const int v = p.verticesOnEdge[2 * e + s];
    double vo = 0.0;
    for (int i = 0; i < 3; ++i) {  // vertexDegree
      const int ev = p.edgesOnVertex[(size_t)v * 3 + i];
      const double es = p.invAreaTriangle[v] * p.dcEdge[ev] * p.edgesOnVertex_sign[(size_t)v * 3 + i];
      vo = vo + es * dru(ev);
    }
    vor[s] = vo;
  }
  tu = tu + lfc * ((div[1] - div[0]) * r_dc - (vor[1] - vor[0]) * r_dv);
  p.tend_u[o] = tu;
}

// 934-987: after the large-step recovery, specified-zone edges take the driving u (owned edges,
// state time level 2) and ru (every edge)
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_u(Dims d, Ptrs p, double delta) {
  const int e = wave_elem(0);
  if (e >= d.nEdges || p.bdyMaskEdge[e] <= N_RELAX_ZONE) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const double dtl = *p.lbc_dtr - delta;
  const size_t o = (size_t)e * K + k;
  if (e < d.nEdgesSolve) p.u2[o] = lbc_drive(p.lbc_u_s, p.lbc_u_t, o, dtl);
  p.ru[o] = lbc_drive(p.lbc_ru_s, p.lbc_ru_t, o, dtl);
}

// atm_bdy_adjust_scalars_work (6494-6586), first loop: owned cells, relaxation zone -> filtered
// and damped toward the driving scalars, specified zone -> the driving scalars; into lbc_tmp
// (every read sees the scalars before the update, as the reference's scalars_tmp arranges)
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_scalars_tmp(Dims d, Ptrs p, double dt, double dt_rk,
                                                                    double delta) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int m = p.bdyMaskCell[c];
  if (m <= 1) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const double dtl = *p.lbc_dtr - delta;
  if (m > N_RELAX_ZONE) {
    for (int is = 0; is < d.ns; ++is)
      p.lbc_tmp[SIX(c, k, is)] = lbc_drive(p.lbc_scalars_s, p.lbc_scalars_t, SIX(c, k, is), dtl);
    return;
  }
  const double lfc = dt_rk * ((double)m - 1.) / (double)N_RELAX_ZONE / (10. * dt * p.meshScalingRegionalCell[c]);
  const double rdc = lfc / 5.0;
  const int ne = p.nEdgesOnCell[c];
  for (int is = 0; is < d.ns; ++is) {
    auto dep = [&](int cc) {
      return p.scalars2[SIX(cc, k, is)] - lbc_drive(p.lbc_scalars_s, p.lbc_scalars_t, SIX(cc, k, is), dtl);
    };
    double t = p.scalars2[SIX(c, k, is)];
    for (int i = 0; i < ne; ++i) {
      const int e = p.edgesOnCell[(size_t)c * d.maxEdges + i];
      const double es = p.edgesOnCell_sign[(size_t)c * d.maxEdges + i] * p.dvEdge[e] * p.invDcEdge[e] * lfc;
      const double ff = es * (dep(p.cellsOnEdge[2 * e + 1]) - dep(p.cellsOnEdge[2 * e]));
      t = t + ff;
    }
    t = t - rdc * dep(c);
    p.lbc_tmp[SIX(c, k, is)] = t;
  }
}
// second loop: the new values into scalars (time level 2), owned cells with mask > 1
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_scalars_copy(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve || p.bdyMaskCell[c] <= 1) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  for (int is = 0; is < d.ns; ++is) p.scalars2[SIX(c, k, is)] = p.lbc_tmp[SIX(c, k, is)];
}

// atm_zero_gradient_w_bdy_work (6117-6143): owned specified-zone cells copy w (time level 2,
// levels 2..nVertLevels) from their nearest relaxation-zone cell
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_zero_grad_w(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve || p.bdyMaskCell[c] <= N_RELAX_ZONE) return;
  const int k = lane_id(), K = d.K;
  if (k < 1 || k >= K) return;
  const size_t K1 = K + 1;
  p.w2[(size_t)c * K1 + k] = p.w2[(size_t)p.nearestRelaxationCell[c] * K1 + k];
}

// atm_bdy_reset_speczone_values (6394-6433): owned specified-zone cells, theta_m (time level 2)
// and rtheta_p from the driving rtheta_m and rho_zz at the end of the step
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_reset_spec(Dims d, Ptrs p, double delta) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve || p.bdyMaskCell[c] <= N_RELAX_ZONE) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const double dtl = *p.lbc_dtr - delta;
  const size_t o = (size_t)c * K + k;
  const double rt = lbc_drive(p.lbc_rtheta_m_s, p.lbc_rtheta_m_t, o, dtl);
  const double rho = lbc_drive(p.lbc_rho_zz_s, p.lbc_rho_zz_t, o, dtl);
  p.theta_m2[o] = rt / rho;
  p.rtheta_p[o] = rt - p.rtheta_base[o];
}

// atm_bdy_set_scalars_work (6632-6671): owned specified-zone cells take the driving scalars
__global__ __launch_bounds__(BLOCK_THREADS) void k_lbc_set_scalars(Dims d, Ptrs p, double delta) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve || p.bdyMaskCell[c] <= N_RELAX_ZONE) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const double dtl = *p.lbc_dtr - delta;
  for (int is = 0; is < d.ns; ++is)
    p.scalars2[SIX(c, k, is)] = lbc_drive(p.lbc_scalars_s, p.lbc_scalars_t, SIX(c, k, is), dtl);
}

}  // namespace mpas
