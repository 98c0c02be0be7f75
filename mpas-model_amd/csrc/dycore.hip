// Host side of the MI355X-native dycore: field registry in HBM, the atm_srk3
// sequencer (mpas_atm_time_integration.F:142-1796) and the C ABI declared in
// include/mpas_dycore.h.  One translation unit with the kernels.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/mpas_dycore.h"
#include "kernels.hip"

using namespace mpas;

namespace {

enum Loc { L_CELL, L_EDGE, L_VERTEX, L_NONE };
enum Target { T_NONE, T_CELL, T_EDGE, T_VERTEX, T_SMALL };  // int index semantics

struct Field {
  std::string pool, name;
  Loc loc;
  int64_t inner;      // doubles/ints per element (Fortran leading dims product)
  bool is_int;
  Target target;
  int ntl;
  void* buf[2] = {nullptr, nullptr};
  int64_t count() const { return inner; }
};

}  // namespace

struct mpas_dyc_ctx {
  Dims d{};
  Config cf{};
  int index_qv = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  std::vector<Field> fields;
  std::map<std::string, int> by_name;  // "pool.name"
  int cur = 0;                          // time level 1 -> buf[cur], 2 -> buf[1-cur]
  std::string err;
  hipEvent_t ev[8] = {};
  bool use_graph = false;
  hipGraphExec_t graph_exec[2] = {nullptr, nullptr};
  double graph_dt[2] = {0, 0};
};

namespace {

#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                      \
      return MPAS_DYC_EHIP;                                                           \
    }                                                                                 \
  } while (0)

int64_t nloc(const mpas_dyc_ctx* c, Loc l) {
  switch (l) {
    case L_CELL: return c->d.nCells + 1;
    case L_EDGE: return c->d.nEdges + 1;
    case L_VERTEX: return c->d.nVertices + 1;
    default: return 1;
  }
}

int64_t field_elems(const mpas_dyc_ctx* c, const Field& f) { return nloc(c, f.loc) * f.inner; }
int64_t field_bytes(const mpas_dyc_ctx* c, const Field& f) {
  return field_elems(c, f) * (f.is_int ? 4 : 8);
}

void add(mpas_dyc_ctx* c, const char* pool, const char* name, Loc loc, int64_t inner, int ntl = 1,
         bool is_int = false, Target t = T_NONE) {
  Field f;
  f.pool = pool;
  f.name = name;
  f.loc = loc;
  f.inner = inner;
  f.is_int = is_int;
  f.target = t;
  f.ntl = ntl;
  c->by_name[f.pool + "." + f.name] = (int)c->fields.size();
  c->fields.push_back(f);
}

// The Registry.xml var_structs the dycore touches (same list the oracle harness builds).
void build_registry(mpas_dyc_ctx* c) {
  const int K = c->d.K, ME = c->d.maxEdges, ME2 = c->d.maxEdges2, ns = c->d.ns;
  // mesh: connectivity
  add(c, "mesh", "nEdgesOnCell", L_CELL, 1, 1, true);
  add(c, "mesh", "edgesOnCell", L_CELL, ME, 1, true, T_EDGE);
  add(c, "mesh", "cellsOnCell", L_CELL, ME, 1, true, T_CELL);
  add(c, "mesh", "verticesOnCell", L_CELL, ME, 1, true, T_VERTEX);
  add(c, "mesh", "kiteForCell", L_CELL, ME, 1, true, T_SMALL);
  add(c, "mesh", "cellsOnEdge", L_EDGE, 2, 1, true, T_CELL);
  add(c, "mesh", "verticesOnEdge", L_EDGE, 2, 1, true, T_VERTEX);
  add(c, "mesh", "nEdgesOnEdge", L_EDGE, 1, 1, true);
  add(c, "mesh", "edgesOnEdge", L_EDGE, ME2, 1, true, T_EDGE);
  add(c, "mesh", "nAdvCellsForEdge", L_EDGE, 1, 1, true);
  add(c, "mesh", "advCellsForEdge", L_EDGE, 15, 1, true, T_CELL);
  add(c, "mesh", "cellsOnVertex", L_VERTEX, 3, 1, true, T_CELL);
  add(c, "mesh", "edgesOnVertex", L_VERTEX, 3, 1, true, T_EDGE);
  // mesh: geometry
  for (const char* n : {"dcEdge", "dvEdge", "invDcEdge", "invDvEdge", "fEdge", "meshScalingDel2",
                        "meshScalingDel4", "specZoneMaskEdge", "angleEdge"})
    add(c, "mesh", n, L_EDGE, 1);
  for (const char* n : {"invAreaCell", "specZoneMaskCell"}) add(c, "mesh", n, L_CELL, 1);
  for (const char* n : {"invAreaTriangle", "fVertex"}) add(c, "mesh", n, L_VERTEX, 1);
  for (const char* n : {"fzm", "fzp", "rdzw", "rdzu", "u_init", "v_init"}) add(c, "mesh", n, L_NONE, K);
  for (const char* n : {"cf1", "cf2", "cf3"}) add(c, "mesh", n, L_NONE, 1);
  add(c, "mesh", "edgesOnCell_sign", L_CELL, ME);
  add(c, "mesh", "edgesOnVertex_sign", L_VERTEX, 3);
  add(c, "mesh", "kiteAreasOnVertex", L_VERTEX, 3);
  add(c, "mesh", "weightsOnEdge", L_EDGE, ME2);
  add(c, "mesh", "adv_coefs", L_EDGE, 15);
  add(c, "mesh", "adv_coefs_3rd", L_EDGE, 15);
  add(c, "mesh", "defc_a", L_CELL, ME);
  add(c, "mesh", "defc_b", L_CELL, ME);
  add(c, "mesh", "zgrid", L_CELL, K + 1);
  add(c, "mesh", "zz", L_CELL, K);
  add(c, "mesh", "zxu", L_EDGE, K);
  add(c, "mesh", "dss", L_CELL, K);
  add(c, "mesh", "t_init", L_CELL, K);
  add(c, "mesh", "zb_cell", L_CELL, (int64_t)ME * (K + 1));
  add(c, "mesh", "zb3_cell", L_CELL, (int64_t)ME * (K + 1));
  // state (2 time levels)
  add(c, "state", "u", L_EDGE, K, 2);
  add(c, "state", "w", L_CELL, K + 1, 2);
  add(c, "state", "theta_m", L_CELL, K, 2);
  add(c, "state", "rho_zz", L_CELL, K, 2);
  add(c, "state", "scalars", L_CELL, (int64_t)ns * K, 2);
  // diag
  for (const char* n : {"theta", "rho", "rho_base", "theta_base", "rho_p", "rho_p_save", "rho_pp",
                        "rho_zz_old_split", "rtheta_base", "rtheta_p", "rtheta_p_save", "rtheta_pp",
                        "rtheta_pp_old", "exner", "exner_base", "pressure_base", "pressure_p", "h_divergence",
                        "kdiff", "ke", "divergence", "pv_cell", "tend_rtheta_adv", "cqw", "cofwr", "cofwz",
                        "cofwt", "a_tri", "alpha_tri", "gamma_tri"})
    add(c, "diag", n, L_CELL, K);
  add(c, "diag", "coftz", L_CELL, K + 1);
  add(c, "diag", "cofrz", L_NONE, K);
  for (const char* n : {"rw", "rw_p", "rw_save", "wwAvg", "wwAvg_split"}) add(c, "diag", n, L_CELL, K + 1);
  for (const char* n : {"ru", "ruAvg", "ruAvg_split", "ru_p", "ru_save", "cqu", "rho_edge", "v", "pv_edge",
                        "gradPVn", "gradPVt"})
    add(c, "diag", n, L_EDGE, K);
  for (const char* n : {"vorticity", "pv_vertex"}) add(c, "diag", n, L_VERTEX, K);
  // tend / tend_physics
  add(c, "tend", "u", L_EDGE, K);
  add(c, "tend", "u_euler", L_EDGE, K);
  add(c, "tend", "w", L_CELL, K + 1);
  add(c, "tend", "w_euler", L_CELL, K + 1);
  add(c, "tend", "theta_m", L_CELL, K);
  add(c, "tend", "theta_euler", L_CELL, K);
  add(c, "tend", "rho_zz", L_CELL, K);
  add(c, "tend", "rt_diabatic_tend", L_CELL, K);
  add(c, "tend", "scalars_tend", L_CELL, (int64_t)ns * K);
  add(c, "tend_physics", "rthdynten", L_CELL, K);
  // module scratch (mpas_atm_time_integration.F:35-71)
  for (const char* n : {"qtot", "tend_rtheta_physics", "tend_rho_physics", "delsq_theta", "delsq_w",
                        "delsq_divergence", "dpdz", "s_max", "s_min", "rho_zz_int", "scalar_old_copy"})
    add(c, "scratch", n, L_CELL, K);
  for (const char* n : {"tend_ru_physics", "delsq_u", "ke_edge", "flux_arr", "flux_upwind_tmp", "flux_tmp",
                        "advflux_w", "advflux_th"})
    add(c, "scratch", n, L_EDGE, K);
  for (const char* n : {"delsq_vorticity", "ke_vertex"}) add(c, "scratch", n, L_VERTEX, K);
  add(c, "scratch", "horiz_flux_array", L_EDGE, (int64_t)ns * K);
  add(c, "scratch", "scale_arr", L_CELL, 2 * (int64_t)K);
  add(c, "scratch", "wdtn", L_CELL, K + 1);
}

Field* find(mpas_dyc_ctx* c, const char* pool, const char* name) {
  auto it = c->by_name.find(std::string(pool) + "." + name);
  if (it == c->by_name.end()) return nullptr;
  return &c->fields[it->second];
}

template <class T>
T* P(mpas_dyc_ctx* c, const char* pool, const char* name, int tl = 1) {
  Field* f = find(c, pool, name);
  if (!f) {
    fprintf(stderr, "mpas_dycore: internal: missing field %s.%s\n", pool, name);
    abort();
  }
  int slot = (f->ntl == 2) ? ((tl == 1) ? c->cur : 1 - c->cur) : 0;
  return (T*)f->buf[slot];
}

Ptrs make_ptrs(mpas_dyc_ctx* c) {
  Ptrs p{};
#define MI(x) p.x = P<const int>(c, "mesh", #x)
#define MR(x) p.x = P<const double>(c, "mesh", #x)
#define DG(x) p.x = P<double>(c, "diag", #x)
#define SC(x) p.x = P<double>(c, "scratch", #x)
  MI(nEdgesOnCell); MI(edgesOnCell); MI(cellsOnCell); MI(verticesOnCell); MI(kiteForCell);
  MI(cellsOnEdge); MI(verticesOnEdge); MI(nEdgesOnEdge); MI(edgesOnEdge); MI(nAdvCellsForEdge);
  MI(advCellsForEdge); MI(cellsOnVertex); MI(edgesOnVertex);
  MR(dcEdge); MR(dvEdge); MR(invDcEdge); MR(invDvEdge); MR(invAreaCell); MR(invAreaTriangle);
  MR(fEdge); MR(fVertex); MR(meshScalingDel2); MR(meshScalingDel4); MR(specZoneMaskEdge); MR(specZoneMaskCell);
  MR(fzm); MR(fzp); MR(rdzw); MR(rdzu);
  MR(edgesOnCell_sign); MR(edgesOnVertex_sign); MR(kiteAreasOnVertex); MR(weightsOnEdge);
  MR(adv_coefs); MR(adv_coefs_3rd); MR(defc_a); MR(defc_b);
  MR(zgrid); MR(zz); MR(zxu); MR(dss); MR(zb_cell); MR(zb3_cell);
  MR(u_init); MR(v_init); MR(t_init); MR(angleEdge);
  p.u1 = P<double>(c, "state", "u", 1); p.u2 = P<double>(c, "state", "u", 2);
  p.w1 = P<double>(c, "state", "w", 1); p.w2 = P<double>(c, "state", "w", 2);
  p.theta_m1 = P<double>(c, "state", "theta_m", 1); p.theta_m2 = P<double>(c, "state", "theta_m", 2);
  p.rho_zz1 = P<double>(c, "state", "rho_zz", 1); p.rho_zz2 = P<double>(c, "state", "rho_zz", 2);
  p.scalars1 = P<double>(c, "state", "scalars", 1); p.scalars2 = P<double>(c, "state", "scalars", 2);
  DG(theta); DG(rho); DG(rho_base); DG(theta_base); DG(rho_p); DG(rho_p_save); DG(rho_pp); DG(rho_zz_old_split);
  DG(rtheta_base); DG(rtheta_p); DG(rtheta_p_save); DG(rtheta_pp); DG(rtheta_pp_old);
  DG(exner); DG(exner_base); DG(pressure_base); DG(pressure_p); DG(h_divergence); DG(kdiff); DG(ke); DG(divergence);
  DG(pv_cell); DG(tend_rtheta_adv); DG(cqw); DG(cofwr); DG(cofwz); DG(cofwt); DG(coftz); DG(a_tri); DG(alpha_tri);
  DG(gamma_tri); DG(cofrz);
  DG(rw); DG(rw_p); DG(rw_save); DG(wwAvg); DG(wwAvg_split);
  DG(ru); DG(ruAvg); DG(ruAvg_split); DG(ru_p); DG(ru_save); DG(cqu); DG(rho_edge); DG(v); DG(pv_edge);
  DG(gradPVn); DG(gradPVt); DG(vorticity); DG(pv_vertex);
  p.tend_u = P<double>(c, "tend", "u"); p.tend_u_euler = P<double>(c, "tend", "u_euler");
  p.tend_w = P<double>(c, "tend", "w"); p.tend_w_euler = P<double>(c, "tend", "w_euler");
  p.tend_theta = P<double>(c, "tend", "theta_m"); p.tend_theta_euler = P<double>(c, "tend", "theta_euler");
  p.tend_rho = P<double>(c, "tend", "rho_zz"); p.rt_diabatic_tend = P<double>(c, "tend", "rt_diabatic_tend");
  p.scalars_tend = P<double>(c, "tend", "scalars_tend"); p.rthdynten = P<double>(c, "tend_physics", "rthdynten");
  SC(qtot); SC(tend_ru_physics); SC(tend_rtheta_physics); SC(tend_rho_physics);
  SC(delsq_theta); SC(delsq_w); SC(delsq_divergence); SC(delsq_u); SC(delsq_vorticity); SC(dpdz);
  SC(ke_vertex); SC(ke_edge); SC(horiz_flux_array);
  SC(s_max); SC(s_min); SC(scale_arr); SC(flux_arr); SC(flux_upwind_tmp); SC(flux_tmp); SC(wdtn); SC(rho_zz_int);
  SC(scalar_old_copy);
  SC(advflux_w); SC(advflux_th);
  // 0-d mesh fields are mirrored on the host
  p.cf1 = c->fields[c->by_name["mesh.cf1"]].buf[1] ? *(double*)c->fields[c->by_name["mesh.cf1"]].buf[1] : 0.0;
  p.cf2 = c->fields[c->by_name["mesh.cf2"]].buf[1] ? *(double*)c->fields[c->by_name["mesh.cf2"]].buf[1] : 0.0;
  p.cf3 = c->fields[c->by_name["mesh.cf3"]].buf[1] ? *(double*)c->fields[c->by_name["mesh.cf3"]].buf[1] : 0.0;
#undef MI
#undef MR
#undef DG
#undef SC
  return p;
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK)); }

#define LAUNCH(kern, n, ...)                                                                  \
  do {                                                                                        \
    if ((n) > 0) hipLaunchKernelGGL(kern, grid_for(n), dim3(BLOCK_THREADS), 0, ctx->stream, __VA_ARGS__); \
  } while (0)

// ---------------------------------------------------------------------------
// reference routines, one host function each
// ---------------------------------------------------------------------------
void copy_n(mpas_dyc_ctx* ctx, double* dst, const double* src, int64_t n) {
  (void)hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream);
}

// atm_rk_integration_setup (1847-1857): copies over owned+halo elements (not the garbage slot)
void rk_integration_setup(mpas_dyc_ctx* ctx, const Ptrs& p) {
  const Dims& d = ctx->d;
  const int64_t K = d.K, K1 = d.K + 1;
  copy_n(ctx, p.ru_save, p.ru, (int64_t)d.nEdges * K);
  copy_n(ctx, p.rw_save, p.rw, (int64_t)d.nCells * K1);
  copy_n(ctx, p.rtheta_p_save, p.rtheta_p, (int64_t)d.nCells * K);
  copy_n(ctx, p.rho_p_save, p.rho_p, (int64_t)d.nCells * K);
  copy_n(ctx, p.u2, p.u1, (int64_t)d.nEdges * K);
  copy_n(ctx, p.w2, p.w1, (int64_t)d.nCells * K1);
  copy_n(ctx, p.theta_m2, p.theta_m1, (int64_t)d.nCells * K);
  copy_n(ctx, p.rho_zz2, p.rho_zz1, (int64_t)d.nCells * K);
  copy_n(ctx, p.rho_zz_old_split, p.rho_zz1, (int64_t)d.nCells * K);
  copy_n(ctx, p.scalars2, p.scalars1, (int64_t)d.nCells * K * d.ns);
}

void vert_imp_coefs(mpas_dyc_ctx* ctx, const Ptrs& p, double dts) {
  LAUNCH(k_vert_imp_coefs, std::max(ctx->d.nCellsSolve, 1), ctx->d, p, dts, ctx->cf.epssm);
}

void dyn_tend(mpas_dyc_ctx* ctx, const Ptrs& p, int rk_step, double dt) {
  const Dims& d = ctx->d;
  const Config& cf = ctx->cf;
  DynTendScal s{};
  s.rk_step = rk_step;
  s.dt = dt;
  s.invDt = 1.0 / dt;
  s.coef_3rd_order = cf.coef_3rd_order;
  s.c_s = cf.smagorinsky_coef;
  if (cf.horiz_mixing_smag) {
    s.h_mom_eddy_visc4 = cf.visc4_2dsmag * (cf.len_disp * cf.len_disp * cf.len_disp);
    s.h_theta_eddy_visc4 = s.h_mom_eddy_visc4;
  } else {
    s.h_mom_eddy_visc4 = cf.h_mom_eddy_visc4;
    s.h_theta_eddy_visc4 = cf.h_theta_eddy_visc4;
  }
  if (cf.rayleigh_damp_u)
    s.rayleigh_coef_inverse = 1.0 / ((double)cf.number_rayleigh_damp_u_levels *
                                     (cf.rayleigh_damp_u_timescale_days * SECONDS_PER_DAY));
  LAUNCH(k_dyn_cells1, d.nCells, d, p, cf, s);
  LAUNCH(k_dyn_edges, d.nEdges, d, p, cf, s, rk_step > 1 ? 1 : 0);
  if (rk_step == 1) {
    if (s.h_mom_eddy_visc4 > 0.0) LAUNCH(k_dyn_delsq_vc, d.nVertices + d.nCells, d, p);
    LAUNCH(k_dyn_edges_rk1b, d.nEdgesSolve, d, p, cf, s);
    LAUNCH(k_dyn_cells2, d.nCells, d, p);
  }
  LAUNCH(k_dyn_advflux, d.nEdges, d, p);
  LAUNCH(k_dyn_cells3, d.nCellsSolve, d, p, cf, s);
}

void acoustic_step(mpas_dyc_ctx* ctx, const Ptrs& p, double dts, int small_step) {
  const Dims& d = ctx->d;
  LAUNCH(k_acoustic_edges, d.nEdges, d, p, dts, small_step);
  LAUNCH(k_acoustic_cells, d.nCells, d, p, dts, small_step, ctx->cf.epssm);
}

void divergence_damping(mpas_dyc_ctx* ctx, const Ptrs& p, double dts) {
  const double rdts = 1.0 / dts;
  const double coef_divdamp = 2.0 * ctx->cf.smdiv * ctx->cf.len_disp * rdts;
  LAUNCH(k_divdamp, ctx->d.nEdges, ctx->d, p, coef_divdamp);
}

void solve_diagnostics(mpas_dyc_ctx* ctx, const Ptrs& p, double dt, int tl, int rk_step /*0 = absent*/) {
  const Dims& d = ctx->d;
  const double* u = (tl == 1) ? p.u1 : p.u2;
  const double* h = (tl == 1) ? p.rho_zz1 : p.rho_zz2;
  const int reconstruct_v = (rk_step == 0 || rk_step == 3) ? 1 : 0;
  LAUNCH(k_diag_vertices, d.nVertices, d, p, u);
  LAUNCH(k_diag_cells, d.nCells, d, p, u, ctx->cf.apvm_upwinding);
  LAUNCH(k_diag_edges, d.nEdges, d, p, u, h, reconstruct_v, ctx->cf.apvm_upwinding, dt);
}

void advance_scalars(mpas_dyc_ctx* ctx, const Ptrs& p, double dt, int rk_step, bool advance_density) {
  const Dims& d = ctx->d;
  double wt_new = 1.0;
  if (advance_density) {
    if (rk_step == 1 && ctx->cf.time_integration_order == 3) wt_new = 1. / 3;
    if (rk_step == 1 && ctx->cf.time_integration_order == 2) wt_new = 1. / 2;
    if (rk_step == 2) wt_new = 1. / 2;
    if (rk_step == 3) wt_new = 1.;
  }
  LAUNCH(k_scalars_edges, d.nEdges, d, p);
  LAUNCH(k_scalars_cells, d.nCellsSolve, d, p, dt, wt_new, ctx->cf.coef_3rd_order);
}

void advance_scalars_mono(mpas_dyc_ctx* ctx, const Ptrs& p, double dt, bool advance_density) {
  const Dims& d = ctx->d;
  LAUNCH(k_mono_prep, d.nCells, d, p, dt, advance_density ? 1 : 0);
  for (int is = 0; is < d.ns; ++is) {
    LAUNCH(k_mono_bounds, d.nCellsSolve, d, p, is, ctx->cf.coef_3rd_order);
    LAUNCH(k_mono_edges1, d.nEdges, d, p, is, dt);
    LAUNCH(k_mono_cells1, d.nCellsSolve, d, p, is, dt, advance_density ? 1 : 0);
    LAUNCH(k_mono_edges2, d.nEdges, d, p, dt);
    LAUNCH(k_mono_cells2, d.nCells, d, p, is, advance_density ? 1 : 0);
  }
}

// atm_srk3 (mpas_atm_time_integration.F:142-1796), single block: halo exchanges are no-ops
int srk3(mpas_dyc_ctx* ctx, double dt) {
  const Dims& d = ctx->d;
  const Config& cf = ctx->cf;
  Ptrs p = make_ptrs(ctx);
  int dynamics_split = cf.dynamics_split_steps;
  double dt_dynamics;
  if (cf.split_dynamics_transport) {
    dt_dynamics = dt / (double)dynamics_split;
  } else {
    dynamics_split = 1;
    dt_dynamics = dt;
  }
  const int nss = cf.number_of_sub_steps;
  double rk_timestep[3], rk_sub_timestep[3];
  int number_sub_steps[3];
  if (cf.time_integration_order == 3) {
    rk_timestep[0] = dt_dynamics / 3.;
    rk_timestep[1] = dt_dynamics / 2.;
    rk_timestep[2] = dt_dynamics;
    rk_sub_timestep[0] = dt_dynamics / 3.;
    rk_sub_timestep[1] = dt_dynamics / (double)nss;
    rk_sub_timestep[2] = dt_dynamics / (double)nss;
    number_sub_steps[0] = 1;
    number_sub_steps[1] = std::max(1, nss / 2);
    number_sub_steps[2] = nss;
  } else {
    rk_timestep[0] = dt_dynamics / 2.;
    rk_timestep[1] = dt_dynamics / 2.;
    rk_timestep[2] = dt_dynamics;
    rk_sub_timestep[0] = dt_dynamics / (double)nss;
    rk_sub_timestep[1] = dt_dynamics / (double)nss;
    rk_sub_timestep[2] = dt_dynamics / (double)nss;
    number_sub_steps[0] = std::max(1, nss / 2);
    number_sub_steps[1] = std::max(1, nss / 2);
    number_sub_steps[2] = nss;
  }
  // halo: theta_m, scalars, pressure_p, rtheta_p (329-338)
  rk_integration_setup(ctx, p);                                   // 341-381
  LAUNCH(k_moist_cells, d.nCells, d, p);                          // 383-422
  LAUNCH(k_moist_edges, d.nEdges, d, p);
  // physics tendencies are zero without DO_PHYSICS (450-457): scratch arrays stay zero.

  for (int dynamics_substep = 1; dynamics_substep <= dynamics_split; ++dynamics_substep) {
    vert_imp_coefs(ctx, p, rk_sub_timestep[0]);                   // 476-510
    // halo: exner (513)
    for (int rk_step = 1; rk_step <= 3; ++rk_step) {
      if (cf.time_integration_order == 3 && rk_step == 2) vert_imp_coefs(ctx, p, rk_sub_timestep[1]);
      dyn_tend(ctx, p, rk_step, dt);                              // 561-630
      // halo: tend_u layer 1 (642)
      LAUNCH(k_smlstep_pert, d.nCellsSolve, d, p);                // 644-678
      for (int small_step = 1; small_step <= number_sub_steps[rk_step - 1]; ++small_step) {
        // halo: rho_pp layer 1 (792)
        acoustic_step(ctx, p, rk_sub_timestep[rk_step - 1], small_step);  // 794-837
        // halo: rtheta_pp layer 1 (845)
        divergence_damping(ctx, p, rk_sub_timestep[rk_step - 1]);          // 849-869
      }
      // halo: rw_p, ru_p, rho_pp (all), rtheta_pp layer 2 (876-887)
      const double invNs = 1 / (double)number_sub_steps[rk_step - 1];
      LAUNCH(k_recover_edges, d.nEdges, d, p, invNs);             // 889-930
      LAUNCH(k_recover_cells, d.nCells + 1, d, p, rk_timestep[rk_step - 1], invNs, rk_step);
      // halo: u (988)
      if (cf.scalar_advection && !cf.split_dynamics_transport) {  // 993-1185
        if (rk_step < 3 || (!cf.monotonic && !cf.positive_definite))
          advance_scalars(ctx, p, rk_timestep[rk_step - 1], rk_step, false);
        else
          advance_scalars_mono(ctx, p, rk_timestep[rk_step - 1], false);
      }
      solve_diagnostics(ctx, p, dt, 2, rk_step);                  // 1187-1228
      // halo: w, pv_edge, rho_edge (+ scalars) (1234-1249)
    }
    // halo: theta_m, pressure_p, rtheta_p between dynamics substeps (1282-1297)
    LAUNCH(k_substep_finish, d.nEdges + d.nCells, d, p, dynamics_substep, dynamics_split,
           1.0 / (double)dynamics_split);                          // 1304-1341
  }

  if (cf.scalar_advection && cf.split_dynamics_transport) {       // 1355-1576
    double rk_ts[3] = {dt / 3., dt / 2., dt};
    if (cf.time_integration_order == 2) rk_ts[0] = dt / 2.;
    for (int rk_step = 1; rk_step <= 3; ++rk_step) {
      if (rk_step < 3 || (!cf.monotonic && !cf.positive_definite))
        advance_scalars(ctx, p, rk_ts[rk_step - 1], rk_step, true);
      else
        advance_scalars_mono(ctx, p, rk_ts[rk_step - 1], true);
      // halo: scalars (1571)
    }
  }
  // mpas_reconstruct (1581-1603) produces output-only diagnostics (uReconstruct*);
  // summarize_timestep (1794) only logs: both outside the hot path.
  return MPAS_DYC_OK;
}

int init_diagnostics(mpas_dyc_ctx* ctx, double dt) {
  const Dims& d = ctx->d;
  Ptrs p = make_ptrs(ctx);
  LAUNCH(k_init_coupled_a, d.nCells, d, p, ctx->index_qv);
  LAUNCH(k_init_coupled_b, d.nEdges, d, p);
  LAUNCH(k_init_coupled_c, d.nCells, d, p);
  solve_diagnostics(ctx, p, dt, 1, 0);
  return MPAS_DYC_OK;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int mpas_dyc_create(const mpas_dyc_dims* dims, const mpas_dyc_config* cfg, int device, mpas_dyc_ctx** out) {
  if (!dims || !cfg || !out) return MPAS_DYC_EINVAL;
  *out = nullptr;
  if (dims->nVertLevels < 4 || dims->nVertLevels > 63) return MPAS_DYC_EINVAL;  // column = one wavefront
  if (dims->maxEdges < 3 || dims->maxEdges2 < dims->maxEdges || dims->num_scalars < 1) return MPAS_DYC_EINVAL;
  mpas_dyc_ctx* ctx = new mpas_dyc_ctx();
  Dims& d = ctx->d;
  d.nCells = dims->nCells;
  d.nEdges = dims->nEdges;
  d.nVertices = dims->nVertices;
  d.K = dims->nVertLevels;
  d.maxEdges = dims->maxEdges;
  d.maxEdges2 = dims->maxEdges2;
  d.ns = dims->num_scalars;
  d.nCellsSolve = dims->nCellsSolve;
  d.nEdgesSolve = dims->nEdgesSolve;
  d.nVerticesSolve = dims->nVerticesSolve;
  d.moist_start = dims->moist_start - 1;
  d.moist_end = dims->moist_end - 1;
  ctx->index_qv = dims->index_qv - 1;
  Config& c = ctx->cf;
  c.time_integration_order = cfg->config_time_integration_order;
  c.number_of_sub_steps = cfg->config_number_of_sub_steps;
  c.dynamics_split_steps = cfg->config_dynamics_split_steps;
  c.number_rayleigh_damp_u_levels = cfg->config_number_rayleigh_damp_u_levels;
  c.split_dynamics_transport = cfg->config_split_dynamics_transport;
  c.scalar_advection = cfg->config_scalar_advection;
  c.positive_definite = cfg->config_positive_definite;
  c.monotonic = cfg->config_monotonic;
  c.mix_full = cfg->config_mix_full;
  c.rayleigh_damp_u = cfg->config_rayleigh_damp_u;
  c.horiz_mixing_smag = cfg->config_horiz_mixing;
  c.h_mom_eddy_visc2 = cfg->config_h_mom_eddy_visc2;
  c.h_mom_eddy_visc4 = cfg->config_h_mom_eddy_visc4;
  c.v_mom_eddy_visc2 = cfg->config_v_mom_eddy_visc2;
  c.h_theta_eddy_visc2 = cfg->config_h_theta_eddy_visc2;
  c.h_theta_eddy_visc4 = cfg->config_h_theta_eddy_visc4;
  c.v_theta_eddy_visc2 = cfg->config_v_theta_eddy_visc2;
  c.len_disp = cfg->config_len_disp;
  c.visc4_2dsmag = cfg->config_visc4_2dsmag;
  c.del4u_div_factor = cfg->config_del4u_div_factor;
  c.coef_3rd_order = cfg->config_coef_3rd_order;
  c.smagorinsky_coef = cfg->config_smagorinsky_coef;
  c.epssm = cfg->config_epssm;
  c.smdiv = cfg->config_smdiv;
  c.apvm_upwinding = cfg->config_apvm_upwinding;
  c.mpas_cam_coef = cfg->config_mpas_cam_coef;
  c.rayleigh_damp_u_timescale_days = cfg->config_rayleigh_damp_u_timescale_days;
  if (c.time_integration_order != 2 && c.time_integration_order != 3) {
    delete ctx;
    return MPAS_DYC_EINVAL;
  }

  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess) {
      delete ctx;
      return MPAS_DYC_EHIP;
    }
  }
  hipGetDevice(&ctx->device);
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return MPAS_DYC_EHIP;
  }
  for (auto& e : ctx->ev) hipEventCreate(&e);
  build_registry(ctx);
  for (auto& f : ctx->fields) {
    const int64_t nb = field_bytes(ctx, f);
    for (int t = 0; t < f.ntl; ++t) {
      if (hipMalloc(&f.buf[t], nb) != hipSuccess || hipMemset(f.buf[t], 0, nb) != hipSuccess) {
        mpas_dyc_destroy(ctx);
        return MPAS_DYC_EHIP;
      }
    }
    if (f.pool == "mesh" && (f.name == "cf1" || f.name == "cf2" || f.name == "cf3")) {
      f.buf[1] = new double(0.0);  // host mirror of the 0-d field
    }
  }
  *out = ctx;
  return MPAS_DYC_OK;
}

void mpas_dyc_destroy(mpas_dyc_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  for (auto& g : ctx->graph_exec)
    if (g) hipGraphExecDestroy(g);
  for (auto& f : ctx->fields) {
    for (int t = 0; t < f.ntl; ++t)
      if (f.buf[t]) hipFree(f.buf[t]);
    if (f.pool == "mesh" && (f.name == "cf1" || f.name == "cf2" || f.name == "cf3")) delete (double*)f.buf[1];
  }
  for (auto& e : ctx->ev)
    if (e) hipEventDestroy(e);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* mpas_dyc_last_error(const mpas_dyc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int64_t mpas_dyc_field_bytes(const mpas_dyc_ctx* ctx, const char* pool, const char* name) {
  if (!ctx || !pool || !name) return 0;
  auto it = ctx->by_name.find(std::string(pool) + "." + name);
  if (it == ctx->by_name.end()) return 0;
  return field_bytes(ctx, ctx->fields[it->second]);
}

void* mpas_dyc_field_device_ptr(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level) {
  if (!ctx || !pool || !name) return nullptr;
  Field* f = find(ctx, pool, name);
  if (!f) return nullptr;
  int slot = (f->ntl == 2) ? ((time_level == 2) ? 1 - ctx->cur : ctx->cur) : 0;
  return f->buf[slot];
}

static int64_t target_n(const mpas_dyc_ctx* c, Target t) {
  switch (t) {
    case T_CELL: return c->d.nCells;
    case T_EDGE: return c->d.nEdges;
    case T_VERTEX: return c->d.nVertices;
    default: return 0;
  }
}

int mpas_dyc_set_field(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level,
                       const void* host, int64_t nbytes) {
  if (!ctx || !pool || !name || !host) return MPAS_DYC_EINVAL;
  Field* f = find(ctx, pool, name);
  if (!f) {
    ctx->err = std::string("unknown field ") + pool + "." + name;
    return MPAS_DYC_EINVAL;
  }
  if (f->pool == "mesh" && (f->name == "cf1" || f->name == "cf2" || f->name == "cf3")) {
    if (nbytes != 8) return MPAS_DYC_EINVAL;
    *(double*)f->buf[1] = *(const double*)host;
    HIPCHK(hipMemcpy(f->buf[0], host, 8, hipMemcpyHostToDevice));
    return MPAS_DYC_OK;
  }
  const int64_t nb = field_bytes(ctx, *f);
  if (nbytes != nb) {
    ctx->err = "size mismatch for " + f->pool + "." + f->name + ": got " + std::to_string(nbytes) +
               " expected " + std::to_string(nb);
    return MPAS_DYC_EINVAL;
  }
  const int slot = (f->ntl == 2) ? ((time_level == 2) ? 1 - ctx->cur : ctx->cur) : 0;
  HIPCHK(hipSetDevice(ctx->device));
  if (f->is_int && f->target != T_NONE) {
    // MPAS 1-based -> device 0-based; out-of-range / 0 -> garbage slot
    const int64_t n = field_elems(ctx, *f);
    std::vector<int32_t> tmp(n);
    const int32_t* src = (const int32_t*)host;
    const int64_t nt = target_n(ctx, f->target);
    for (int64_t i = 0; i < n; ++i) {
      int32_t v = src[i] - 1;
      if (f->target == T_SMALL) v = v < 0 ? 0 : v;
      else if (v < 0 || v > nt) v = (int32_t)nt;
      tmp[i] = v;
    }
    HIPCHK(hipMemcpyAsync(f->buf[slot], tmp.data(), nb, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  } else {
    HIPCHK(hipMemcpyAsync(f->buf[slot], host, nb, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_get_field(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level, void* host,
                       int64_t nbytes) {
  if (!ctx || !pool || !name || !host) return MPAS_DYC_EINVAL;
  Field* f = find(ctx, pool, name);
  if (!f) {
    ctx->err = std::string("unknown field ") + pool + "." + name;
    return MPAS_DYC_EINVAL;
  }
  if (f->pool == "mesh" && (f->name == "cf1" || f->name == "cf2" || f->name == "cf3")) {
    if (nbytes != 8) return MPAS_DYC_EINVAL;
    *(double*)host = *(double*)f->buf[1];
    return MPAS_DYC_OK;
  }
  const int64_t nb = field_bytes(ctx, *f);
  if (nbytes != nb) {
    ctx->err = "size mismatch for " + f->pool + "." + f->name;
    return MPAS_DYC_EINVAL;
  }
  const int slot = (f->ntl == 2) ? ((time_level == 2) ? 1 - ctx->cur : ctx->cur) : 0;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(host, f->buf[slot], nb, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (f->is_int && f->target != T_NONE) {
    int32_t* h = (int32_t*)host;
    const int64_t n = field_elems(ctx, *f);
    for (int64_t i = 0; i < n; ++i) h[i] += 1;
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_init_diagnostics(mpas_dyc_ctx* ctx, double dt) {
  if (!ctx) return MPAS_DYC_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  int r = init_diagnostics(ctx, dt);
  HIPCHK(hipGetLastError());
  return r;
}

int mpas_dyc_timestep(mpas_dyc_ctx* ctx, double dt, int32_t itimestep) {
  (void)itimestep;
  if (!ctx || !(dt > 0.0)) return MPAS_DYC_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->use_graph) {
    const int parity = ctx->cur;
    if (!ctx->graph_exec[parity] || ctx->graph_dt[parity] != dt) {
      if (ctx->graph_exec[parity]) hipGraphExecDestroy(ctx->graph_exec[parity]);
      hipGraph_t g;
      HIPCHK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
      int r = srk3(ctx, dt);
      HIPCHK(hipStreamEndCapture(ctx->stream, &g));
      if (r) return r;
      HIPCHK(hipGraphInstantiate(&ctx->graph_exec[parity], g, nullptr, nullptr, 0));
      hipGraphDestroy(g);
      ctx->graph_dt[parity] = dt;
    }
    HIPCHK(hipGraphLaunch(ctx->graph_exec[parity], ctx->stream));
    return MPAS_DYC_OK;
  }
  int r = srk3(ctx, dt);
  HIPCHK(hipGetLastError());
  return r;
}

int mpas_dyc_shift_time_levels(mpas_dyc_ctx* ctx) {
  if (!ctx) return MPAS_DYC_EINVAL;
  ctx->cur ^= 1;
  return MPAS_DYC_OK;
}

int mpas_dyc_synchronize(mpas_dyc_ctx* ctx) {
  if (!ctx) return MPAS_DYC_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return MPAS_DYC_OK;
}

int mpas_dyc_use_graph(mpas_dyc_ctx* ctx, int32_t on) {
  if (!ctx) return MPAS_DYC_EINVAL;
  ctx->use_graph = on != 0;
  return MPAS_DYC_OK;
}

double mpas_dyc_acoustic_bytes(const mpas_dyc_ctx* ctx) {
  if (!ctx) return 0.0;
  const Dims& d = ctx->d;
  // B_ac = 8 [K (7 nE_act + 18 nC_own) + 9 (K+1) nC_own]   (SURVEY.md §8d);
  // single block: every edge has an owned cell.
  const double K = d.K;
  const double nEact = d.nEdges, nC = d.nCellsSolve;
  return 8.0 * (K * (7.0 * nEact + 18.0 * nC) + 9.0 * (K + 1.0) * nC);
}

int mpas_dyc_time_acoustic_step(mpas_dyc_ctx* ctx, double dts, int32_t small_step, int32_t reps, double* ms_out,
                                double* ms_kernels) {
  if (!ctx || reps < 1) return MPAS_DYC_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  Ptrs p = make_ptrs(ctx);
  const Dims& d = ctx->d;
  double acc[3] = {0, 0, 0};
  HIPCHK(hipEventRecord(ctx->ev[0], ctx->stream));
  for (int r = 0; r < reps; ++r) {
    HIPCHK(hipEventRecord(ctx->ev[1], ctx->stream));
    LAUNCH(k_acoustic_edges, d.nEdges, d, p, dts, small_step);
    HIPCHK(hipEventRecord(ctx->ev[2], ctx->stream));
    LAUNCH(k_acoustic_cells, d.nCells, d, p, dts, small_step, ctx->cf.epssm);
    HIPCHK(hipEventRecord(ctx->ev[3], ctx->stream));
    divergence_damping(ctx, p, dts);
    HIPCHK(hipEventRecord(ctx->ev[4], ctx->stream));
    if (ms_kernels) {
      HIPCHK(hipEventSynchronize(ctx->ev[4]));
      float t;
      hipEventElapsedTime(&t, ctx->ev[1], ctx->ev[2]);
      acc[0] += t;
      hipEventElapsedTime(&t, ctx->ev[2], ctx->ev[3]);
      acc[1] += t;
      hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[4]);
      acc[2] += t;
    }
  }
  HIPCHK(hipEventRecord(ctx->ev[5], ctx->stream));
  HIPCHK(hipEventSynchronize(ctx->ev[5]));
  float tot;
  HIPCHK(hipEventElapsedTime(&tot, ctx->ev[0], ctx->ev[5]));
  if (ms_out) *ms_out = tot / reps;
  if (ms_kernels)
    for (int i = 0; i < 3; ++i) ms_kernels[i] = acc[i] / reps;
  return MPAS_DYC_OK;
}

}  // extern "C"
