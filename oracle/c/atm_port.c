/*
 * TEST INFRASTRUCTURE ONLY -- scalar C restatement of the reference acoustic
 * sub-step (src/core_atmosphere/dynamics/mpas_atm_time_integration.F), the
 * per-kernel oracle for the graded kernel and the cpu_baseline "port".
 * Compiled with -ffp-contract=off: every expression keeps the Fortran
 * left-to-right evaluation order, so results are bit-identical to the
 * reference's x86 build (which has no FMA).  Pinned against the compiled
 * reference's fixture by tests/test_oracle.py.
 */
#include "atm_port.h"

#include <stdlib.h>
#include <string.h>

#define RGAS 287.0
#define CP (7.0 * RGAS / 2.0)
#define GRAVITY 9.80616

static void acoustic_work(const atm_port_acoustic_args* a, double dts, int small_step, double epssm, int nthreads) {
  const int K = a->K, K1 = a->K + 1, ME = a->maxEdges;
  const double rcv = RGAS / (CP - RGAS);  /* 2535 */
  const double c2 = CP * rcv;              /* 2536 */
  const double resm = (1.0 - epssm) / (1.0 + epssm);
  (void)nthreads;

  /* edge phase: 2540-2601 */
#pragma omp parallel for schedule(static)
  for (int iEdge = 0; iEdge < a->nEdges; ++iEdge) {
    const int cell1 = a->cellsOnEdge[2 * iEdge], cell2 = a->cellsOnEdge[2 * iEdge + 1];
    if (!(cell1 < a->nCellsSolve || cell2 < a->nCellsSolve)) continue;
    for (int k = 0; k < K; ++k) {
      const size_t o = (size_t)iEdge * K + k, o1 = (size_t)cell1 * K + k, o2 = (size_t)cell2 * K + k;
      if (small_step != 1) {
        double pgrad = ((a->rtheta_pp[o2] - a->rtheta_pp[o1]) * a->invDcEdge[iEdge]) / (.5 * (a->zz[o2] + a->zz[o1]));
        pgrad = a->cqu[o] * 0.5 * c2 * (a->exner[o1] + a->exner[o2]) * pgrad;
        pgrad = pgrad + 0.5 * a->zxu[o] * GRAVITY * (a->rho_pp[o1] + a->rho_pp[o2]);
        a->ru_p[o] = a->ru_p[o] + dts * (a->tend_ru[o] - (1.0 - a->specZoneMaskEdge[iEdge]) * pgrad);
        a->ruAvg[o] = a->ruAvg[o] + a->ru_p[o];
      } else {
        a->ru_p[o] = dts * a->tend_ru[o];
        a->ruAvg[o] = a->ru_p[o];
      }
    }
  }

  /* rtheta_pp_old: 2603-2611 */
#pragma omp parallel for schedule(static)
  for (int iCell = 0; iCell < a->nCells; ++iCell)
    for (int k = 0; k < K; ++k)
      a->rtheta_pp_old[(size_t)iCell * K + k] = (small_step == 1) ? 0.0 : a->rtheta_pp[(size_t)iCell * K + k];

  /* cell phase: 2615-2721 */
#pragma omp parallel
  {
    double* rs = (double*)malloc(sizeof(double) * K);
    double* ts = (double*)malloc(sizeof(double) * K);
#pragma omp for schedule(static)
    for (int iCell = 0; iCell < a->nCellsSolve; ++iCell) {
      double* rho_pp = a->rho_pp + (size_t)iCell * K;
      double* rtheta_pp = a->rtheta_pp + (size_t)iCell * K;
      double* rw_p = a->rw_p + (size_t)iCell * K1;
      double* wwAvg = a->wwAvg + (size_t)iCell * K1;
      const double* zz = a->zz + (size_t)iCell * K;
      if (small_step == 1) {
        for (int k = 0; k < K1; ++k) wwAvg[k] = 0.0;
        for (int k = 0; k < K; ++k) rho_pp[k] = 0.0;
        for (int k = 0; k < K; ++k) rtheta_pp[k] = 0.0;
        for (int k = 0; k < K1; ++k) rw_p[k] = 0.0;
      }
      if (a->specZoneMaskCell[iCell] == 0.0) {
        for (int k = 0; k < K; ++k) { ts[k] = 0.0; rs[k] = 0.0; }
        for (int i = 0; i < a->nEdgesOnCell[iCell]; ++i) {
          const int iEdge = a->edgesOnCell[iCell * ME + i];
          const int cell1 = a->cellsOnEdge[2 * iEdge], cell2 = a->cellsOnEdge[2 * iEdge + 1];
          for (int k = 0; k < K; ++k) {
            const double flux = a->edgesOnCell_sign[iCell * ME + i] * dts * a->dvEdge[iEdge] *
                                a->ru_p[(size_t)iEdge * K + k] * a->invAreaCell[iCell];
            rs[k] = rs[k] - flux;
            ts[k] = ts[k] - flux * 0.5 * (a->theta_m[(size_t)cell2 * K + k] + a->theta_m[(size_t)cell1 * K + k]);
          }
        }
        const double* coftz = a->coftz + (size_t)iCell * K1;
        for (int k = 0; k < K; ++k) { /* 2646-2652 */
          rs[k] = rho_pp[k] + dts * a->tend_rho[(size_t)iCell * K + k] + rs[k] - a->cofrz[k] * resm * (rw_p[k + 1] - rw_p[k]);
          ts[k] = rtheta_pp[k] + dts * a->tend_rt[(size_t)iCell * K + k] + ts[k] -
                  resm * a->rdzw[k] * (coftz[k + 1] * rw_p[k + 1] - coftz[k] * rw_p[k]);
        }
        for (int k = 1; k < K; ++k) wwAvg[k] = wwAvg[k] + 0.5 * (1.0 - epssm) * rw_p[k]; /* 2655-2657 */
        for (int k = 1; k < K; ++k) { /* 2660-2670 */
          const size_t o = (size_t)iCell * K + k;
          rw_p[k] = rw_p[k] + dts * a->tend_rw[(size_t)iCell * K1 + k] -
                    a->cofwz[o] * ((zz[k] * ts[k] - zz[k - 1] * ts[k - 1]) + resm * (zz[k] * rtheta_pp[k] - zz[k - 1] * rtheta_pp[k - 1])) -
                    a->cofwr[o] * ((rs[k] + rs[k - 1]) + resm * (rho_pp[k] + rho_pp[k - 1])) +
                    a->cofwt[o] * (ts[k] + resm * rtheta_pp[k]) + a->cofwt[o - 1] * (ts[k - 1] + resm * rtheta_pp[k - 1]);
        }
        for (int k = 1; k < K; ++k) /* 2675-2677 */
          rw_p[k] = (rw_p[k] - a->a_tri[(size_t)iCell * K + k] * rw_p[k - 1]) * a->alpha_tri[(size_t)iCell * K + k];
        for (int k = K - 1; k >= 0; --k) /* 2680-2682 */
          rw_p[k] = rw_p[k] - a->gamma_tri[(size_t)iCell * K + k] * rw_p[k + 1];
        for (int k = 1; k < K; ++k) { /* 2687-2693 */
          const size_t o = (size_t)iCell * K + k, ow = (size_t)iCell * K1 + k;
          const double dd = a->rw_save[ow] - a->rw[ow];
          rw_p[k] = (rw_p[k] + dd - dts * a->dss[o] * (a->fzm[k] * zz[k] + a->fzp[k] * zz[k - 1]) *
                                         (a->fzm[k] * a->rho_zz[o] + a->fzp[k] * a->rho_zz[o - 1]) * a->w[ow]) /
                        (1.0 + dts * a->dss[o]) - dd;
        }
        for (int k = 1; k < K; ++k) wwAvg[k] = wwAvg[k] + 0.5 * (1.0 + epssm) * rw_p[k]; /* 2697-2699 */
        for (int k = 0; k < K; ++k) { /* 2704-2708 */
          rho_pp[k] = rs[k] - a->cofrz[k] * (rw_p[k + 1] - rw_p[k]);
          rtheta_pp[k] = ts[k] - a->rdzw[k] * (coftz[k + 1] * rw_p[k + 1] - coftz[k] * rw_p[k]);
        }
      } else { /* 2710-2719 */
        for (int k = 0; k < K; ++k) {
          rho_pp[k] = rho_pp[k] + dts * a->tend_rho[(size_t)iCell * K + k];
          rtheta_pp[k] = rtheta_pp[k] + dts * a->tend_rt[(size_t)iCell * K + k];
          rw_p[k] = rw_p[k] + dts * a->tend_rw[(size_t)iCell * K1 + k];
          wwAvg[k] = wwAvg[k] + 0.5 * (1.0 + epssm) * rw_p[k];
        }
      }
    }
    free(rs);
    free(ts);
  }
}

/* atm_divergence_damping_3d: 2765-2793 */
static void divergence_damping(const atm_port_acoustic_args* a, double dts, double smdiv, double len_disp) {
  const int K = a->K;
  const double rdts = 1.0 / dts;
  const double coef_divdamp = 2.0 * smdiv * len_disp * rdts;
#pragma omp parallel for schedule(static)
  for (int iEdge = 0; iEdge < a->nEdges; ++iEdge) {
    const int cell1 = a->cellsOnEdge[2 * iEdge], cell2 = a->cellsOnEdge[2 * iEdge + 1];
    if (!(cell1 < a->nCellsSolve || cell2 < a->nCellsSolve)) continue;
    for (int k = 0; k < K; ++k) {
      const size_t o = (size_t)iEdge * K + k, o1 = (size_t)cell1 * K + k, o2 = (size_t)cell2 * K + k;
      const double divCell1 = -(a->rtheta_pp[o1] - a->rtheta_pp_old[o1]);
      const double divCell2 = -(a->rtheta_pp[o2] - a->rtheta_pp_old[o2]);
      a->ru_p[o] = a->ru_p[o] + coef_divdamp * (divCell2 - divCell1) * (1.0 - a->specZoneMaskEdge[iEdge]) /
                                    (a->theta_m[o1] + a->theta_m[o2]);
    }
  }
}

void atm_port_acoustic_substep(const atm_port_acoustic_args* a, double dts, int small_step, double epssm,
                               double smdiv, double len_disp, int nthreads) {
  acoustic_work(a, dts, small_step, epssm, nthreads);
  divergence_damping(a, dts, smdiv, len_disp);
}
