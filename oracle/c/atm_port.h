/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement ("port") of the reference acoustic
 * sub-step, used by tests/ as a per-kernel oracle and by bench.py's cpu_baseline
 * leg.  Never linked into the product.
 *
 * Layout: the Fortran memory images of the pool arrays (k fastest, garbage slot
 * included), 0-based indices (missing -> n).  See atm_port.c for the line-by-line
 * citations of src/core_atmosphere/dynamics/mpas_atm_time_integration.F.
 */
#ifndef ATM_PORT_H
#define ATM_PORT_H
#include <stdint.h>

typedef struct {
  int32_t nCells, nEdges, nCellsSolve, K, maxEdges;
  /* connectivity (0-based) */
  const int32_t *cellsOnEdge, *edgesOnCell, *nEdgesOnCell;
  /* mesh */
  const double *edgesOnCell_sign, *invDcEdge, *dvEdge, *invAreaCell, *specZoneMaskEdge, *specZoneMaskCell;
  const double *zz, *zxu, *dss, *fzm, *fzp, *rdzw;
  /* state / diag (read) */
  const double *theta_m, *rho_zz, *w, *exner, *cqu;
  const double *cofwr, *cofwz, *cofwt, *coftz, *cofrz, *a_tri, *alpha_tri, *gamma_tri;
  const double *tend_ru, *tend_rho, *tend_rt, *tend_rw, *rw, *rw_save;
  /* updated */
  double *ru_p, *ruAvg, *rho_pp, *rtheta_pp, *rtheta_pp_old, *rw_p, *wwAvg;
} atm_port_acoustic_args;

/* atm_advance_acoustic_step_work (2447-2723) followed by atm_divergence_damping_3d
 * (2726-2795); nthreads <= 0 uses the OpenMP default. */
void atm_port_acoustic_substep(const atm_port_acoustic_args* a, double dts, int small_step, double epssm,
                               double smdiv, double len_disp, int nthreads);

#endif
