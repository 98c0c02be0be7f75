// The floor of the gather kernels' access patterns on MI355X (VERDICT r03 "Next 2").
//
// Replays the real index streams of the x1.163842 mesh (dumped by tools/gather_floor.py) through
// three of the library's own kernels, on the same device data layout:
//   advflux   k_dyn_advflux_p<10>           10 stencil cells x (w, theta_m) per edge
//   scalars   k_scalars_edges_p<10>         10 stencil cells x scalars per edge
//   dynedges  k_dyn_edges_p<false, 10>      10 TRiSK edges x (u, pv_edge) + 2 cells x 4 fields
// next to a "floor" twin of each: the same wave -> edge mapping (pair layout, XCD slabs), the same
// index loads, the same 16-byte column gathers and own-column loads, the same stores, but a plain sum
// instead of the flux arithmetic -- what that access pattern costs with nothing else in the way.  A
// "stream" twin moves the same number of bytes per edge from contiguous per-edge columns (no index
// indirection): the cost of the bytes alone.  Each variant is timed with HIP events over REPS
// launches, in interleaved rounds; the median per launch is printed.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/gather_floor.hip -o tools/gather_floor
//   tools/gather_floor DUMPDIR [reps] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../mpas-model_amd/csrc/kernels.hip"

using namespace mpas;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

template <class T>
std::vector<T> load(const std::string& dir, const char* name, size_t n) {
  std::vector<T> v(n);
  FILE* f = fopen((dir + "/" + name).c_str(), "rb");
  if (!f || fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "cannot read %zu values from %s/%s\n", n, dir.c_str(), name);
    exit(1);
  }
  fclose(f);
  return v;
}

template <class T>
T* dev(const std::vector<T>& h) {
  T* d = nullptr;
  CK(hipMalloc(&d, h.size() * sizeof(T) + 256));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

double* dev_field(size_t n, unsigned seed) {  // smooth positive values, 256 B of slack
  std::vector<double> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = 1.0 + 1e-3 * (double)((i * 2654435761u + seed) % 1000);
  return dev(h);
}

// ---- floor twins: the real kernel's loads and stores, a plain sum for the arithmetic --------------
__global__ __launch_bounds__(EDGE_THREADS) void f_advflux(Dims d, Ptrs p) {
  const int eA = 2 * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = threadIdx.x & 31;
  const int lc = min(l, K / 2 - 1), lw = min(l, K / 2);
  const size_t K1 = K + 1;
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  int ic[10];
  double a[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    ic[j] = sel(h, p.advCellsForEdge[(size_t)eA * 15 + j], p.advCellsForEdge[(size_t)eB * 15 + j]);
    a[j] = sel(h, ld_uniform_f64(p.adv_coefs + (size_t)eA * 15 + j), ld_uniform_f64(p.adv_coefs + (size_t)eB * 15 + j)) +
           sel(h, ld_uniform_f64(p.adv_coefs_3rd + (size_t)eA * 15 + j),
               ld_uniform_f64(p.adv_coefs_3rd + (size_t)eB * 15 + j));
  }
  const d2 rue = ld2(p.ru + o);
  const bool onA = ceA.x < d.nCellsSolve || ceA.y < d.nCellsSolve;
  const bool onB = hasB && (ceB.x < d.nCellsSolve || ceB.y < d.nCellsSolve);
  if (!onA && !onB) return;
  d2 fw = rue, ft = rue;
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const d2 w_ = ld2(p.w2 + (size_t)ic[j] * K1 + 2 * lw), t_ = ld2(p.theta_m2 + (size_t)ic[j] * K + 2 * lc);
    fw.x += a[j] * w_.x;
    fw.y += a[j] * w_.y;
    ft.x += a[j] * t_.x;
    ft.y += a[j] * t_.y;
  }
  if ((h ? onB : onA) && 2 * l < K) {
    st2(p.advflux_w + o, fw);
    st2(p.advflux_th + o, ft);
  }
}

// the same bytes per edge from contiguous columns: edge e reads columns 10 e .. 10 e + 9 of two
// (10 nE)-column arrays
__global__ __launch_bounds__(EDGE_THREADS) void s_advflux(Dims d, Ptrs p, const double* __restrict__ W,
                                                          const double* __restrict__ T) {
  const int eA = 2 * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = threadIdx.x & 31;
  const int lc = min(l, K / 2 - 1), lw = min(l, K / 2);
  const size_t K1 = K + 1;
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const d2 rue = ld2(p.ru + o);
  d2 fw = rue, ft = rue;
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const size_t c = (size_t)e * 10 + j;
    const d2 w_ = ld2(W + c * K1 + 2 * lw), t_ = ld2(T + c * K + 2 * lc);
    fw.x += w_.x;
    fw.y += w_.y;
    ft.x += t_.x;
    ft.y += t_.y;
  }
  if ((h == 0 || hasB) && 2 * l < K) {
    st2(p.advflux_w + o, fw);
    st2(p.advflux_th + o, ft);
  }
}

__global__ __launch_bounds__(EDGE_THREADS) void f_scalars(Dims d, Ptrs p) {
  const int eA = 2 * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = threadIdx.x & 31, ns = d.ns;
  const int lc = min(l, K / 2 - 1);
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  int ic[10];
  double a[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    ic[j] = sel(h, p.advCellsForEdge[(size_t)eA * 15 + j], p.advCellsForEdge[(size_t)eB * 15 + j]);
    a[j] = sel(h, ld_uniform_f64(p.adv_coefs + (size_t)eA * 15 + j), ld_uniform_f64(p.adv_coefs + (size_t)eB * 15 + j)) +
           sel(h, ld_uniform_f64(p.adv_coefs_3rd + (size_t)eA * 15 + j),
               ld_uniform_f64(p.adv_coefs_3rd + (size_t)eB * 15 + j));
  }
  const d2 uh = ld2(p.ruAvg + o);
  const bool st = (h == 0 || hasB) && 2 * l < K;
  for (int is = 0; is < ns; ++is) {
    d2 acc = uh;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const d2 sv = ld2(p.scalars2 + SIX(ic[j], 2 * lc, is));
      acc.x += a[j] * sv.x;
      acc.y += a[j] * sv.y;
    }
    if (st) st2(p.horiz_flux_array + HIX(e, 2 * lc, is), acc);
  }
}

__global__ __launch_bounds__(EDGE_THREADS) void f_dynedges(Dims d, Ptrs p) {
  const int eA = 2 * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = threadIdx.x & 31;
  const int lc = min(l, K / 2 - 1), lw = min(l, K / 2);
  const int e = sel(h, eA, eB);
  const size_t K1 = K + 1;
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const double invDc = sel(h, ld_uniform_f64(p.invDcEdge + eA), ld_uniform_f64(p.invDcEdge + eB));
  const d2 re = ld2(p.rho_edge + o);
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const size_t o1 = (size_t)c1 * K + 2 * lc, o2 = (size_t)c2 * K + 2 * lc;
  int eoe[10];
  double wgt[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    eoe[j] = sel(h, p.edgesOnEdge[(size_t)eA * d.maxEdges2 + j], p.edgesOnEdge[(size_t)eB * d.maxEdges2 + j]);
    wgt[j] = sel(h, ld_uniform_f64(p.weightsOnEdge + (size_t)eA * d.maxEdges2 + j),
                 ld_uniform_f64(p.weightsOnEdge + (size_t)eB * d.maxEdges2 + j));
  }
  const d2 uk = ld2(p.u2 + o), pve = ld2(p.pv_edge + o), tue = ld2(p.tend_u_euler + o);
  const d2 rw1 = ld2(p.rw + (size_t)c1 * K1 + 2 * lw), rw2 = ld2(p.rw + (size_t)c2 * K1 + 2 * lw);
  const d2 ke1 = ld2(p.ke + o1), ke2 = ld2(p.ke + o2), hd1 = ld2(p.h_divergence + o1), hd2 = ld2(p.h_divergence + o2);
  d2 q{invDc * re.x + uk.x + pve.x + tue.x + rw1.x + rw2.x + ke1.x + ke2.x + hd1.x + hd2.x,
       re.y + uk.y + pve.y + tue.y + rw1.y + rw2.y + ke1.y + ke2.y + hd1.y + hd2.y};
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const size_t oj = (size_t)eoe[j] * K + 2 * lc;
    const d2 pv = ld2(p.pv_edge + oj), uu = ld2(p.u2 + oj);
    q.x += wgt[j] * uu.x * pv.x;
    q.y += wgt[j] * uu.y * pv.y;
  }
  const bool solve = h ? (hasB && eB < d.nEdgesSolve) : (eA < d.nEdgesSolve);
  if (solve && 2 * l < K) st2(p.tend_u + o, q);
}

// ---- cell-centric advflux (VERDICT r04 Next 3) ---------------------------------------------------
// One wavefront per cell that is cellsOnEdge(1) of an edge (c1): lanes 0-31 form w's edge values,
// lanes 32-63 theta_m's, two levels per lane.  advCellsForEdge lists c1, c2, c1's other neighbours in
// c1's cellsOnCell order, then c2's neighbours not yet listed (atm_adv_coef_compression,
// mpas_atm_core.F:1154-1191): slots 0 .. ne(c1) are c1's ring, which the wave loads once for all of
// its c1-edges; only the last slots (c2's far neighbours) are gathered per edge.  The sum runs over
// the slots in the same order with the same expression as k_dyn_advflux_p: the same bits.
// list[i] = (cell, bit mask of its edge positions whose edge has it as c1).
// one c1-edge of the cell (its position IE among the cell's NE edges, both compile-time constants, so
// every slot's ring column and coefficient offset is static)
template <int ME, int NE, int IE>
__device__ __forceinline__ void advflux_c_edge(const Dims& d, const Ptrs& p, const d2 (&col)[ME + 1], int e, int c,
                                               const double* F, size_t stride, int off, d2 fzm, d2 fzp, int h, int l,
                                               int lc) {
  constexpr int NF = ME - 3;
  const int K = d.K, kx = 2 * l, ky = 2 * l + 1;
  const size_t o = (size_t)e * K + 2 * lc;
  const int na = __builtin_amdgcn_readfirstlane(p.nAdvCellsForEdge[e]);
  const int* ac = p.advCellsForEdge + (size_t)e * 15;
  const double* A = p.adv_coefs + (size_t)e * 15;
  const double* B = p.adv_coefs_3rd + (size_t)e * 15;
  double a[NE + 1 + NF], b[NE + 1 + NF];
#pragma unroll
  for (int j = 0; j < NE + 1 + NF; ++j) {
    a[j] = ld_uniform_f64(A + j);
    b[j] = ld_uniform_f64(B + j);
  }
  d2 far[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int cf = NE + 1 + f < na ? ac[NE + 1 + f] : c;
    far[f] = ld2(F + (size_t)cf * stride + off);
  }
  const d2 rue = ld2(p.ru + o);
  const d2 rue_m = km1(rue, l);
  const double rewx = kx < K ? fzm.x * rue.x + fzp.x * rue_m.x : 0.0;
  const double rewy = ky < K ? fzm.y * rue.y + fzp.y * rue_m.y : 0.0;
  const double sx = h ? sgn1(rue.x) : sgn1(rewx), sy = h ? sgn1(rue.y) : sgn1(rewy);
  d2 fl{0.0, 0.0};
  auto add = [&](int j, d2 v) {
    fl.x = fl.x + (a[j] + sx * b[j]) * v.x;
    fl.y = fl.y + (a[j] + sy * b[j]) * v.y;
  };
  add(0, col[0]);
  add(1, col[1 + IE]);
#pragma unroll
  for (int m = 0; m < NE; ++m)
    if (m != IE) add(2 + m - (m > IE ? 1 : 0), col[1 + m]);
#pragma unroll
  for (int f = 0; f < NF; ++f)
    if (NE + 1 + f < na) add(NE + 1 + f, far[f]);
  if (2 * l < K) st2((h ? p.advflux_th : p.advflux_w) + o, fl);
}

template <int ME, int NE>
__device__ __forceinline__ void advflux_c_cell(const Dims& d, const Ptrs& p, const d2 (&col)[ME + 1], const int (&eo)[ME],
                                               int mask, int c, const double* F, size_t stride, int off, d2 fzm,
                                               d2 fzp, int h, int l, int lc) {
#define ADVF_E(IE) \
  if (IE < NE && ((mask >> IE) & 1)) advflux_c_edge<ME, NE, (IE < NE ? IE : 0)>(d, p, col, eo[IE < ME ? IE : 0], c, F, stride, off, fzm, fzp, h, l, lc)
  ADVF_E(0);
  ADVF_E(1);
  ADVF_E(2);
  ADVF_E(3);
  ADVF_E(4);
  ADVF_E(5);
  ADVF_E(6);
#undef ADVF_E
}

template <int ME>
__global__ __launch_bounds__(EDGE_THREADS) void k_advflux_c(Dims d, Ptrs p, const int2* __restrict__ list, int n) {
  const int iw = pair_wave();
  if (iw >= n) return;
  const int c = __builtin_amdgcn_readfirstlane(list[iw].x), mask = __builtin_amdgcn_readfirstlane(list[iw].y);
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, K / 2 - 1), lw = min(l, K / 2);
  const size_t stride = h ? (size_t)K : (size_t)K + 1;
  const int off = 2 * (h ? lc : lw);
  const double* F = h ? p.theta_m2 : p.w2;
  const int* rec = p.cell_rec + (size_t)c * CELL_REC;
  const int ne = rec[14];
  int eo[ME];
  d2 col[ME + 1];
  col[0] = ld2(F + (size_t)c * stride + off);
#pragma unroll
  for (int m = 0; m < ME; ++m) {
    eo[m] = rec[m];
    col[1 + m] = ld2(F + (size_t)rec[7 + m] * stride + off);
  }
  const d2 fzm = ld2(p.fzm + 2 * lc), fzp = ld2(p.fzp + 2 * lc);
  if (ne == 6) advflux_c_cell<ME, 6>(d, p, col, eo, mask, c, F, stride, off, fzm, fzp, h, l, lc);
  else if (ne == 5) advflux_c_cell<ME, 5>(d, p, col, eo, mask, c, F, stride, off, fzm, fzp, h, l, lc);
  else if (ME >= 7 && ne == 7) advflux_c_cell<ME, ME>(d, p, col, eo, mask, c, F, stride, off, fzm, fzp, h, l, lc);
}

// the same loads and stores, a plain sum for the arithmetic
template <int ME>
__global__ __launch_bounds__(EDGE_THREADS) void f_advflux_c(Dims d, Ptrs p, const int2* __restrict__ list, int n) {
  constexpr int NF = ME - 3;
  const int iw = pair_wave();
  if (iw >= n) return;
  const int c = __builtin_amdgcn_readfirstlane(list[iw].x), mask = __builtin_amdgcn_readfirstlane(list[iw].y);
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, K / 2 - 1), lw = min(l, K / 2);
  const size_t stride = h ? (size_t)K : (size_t)K + 1;
  const int off = 2 * (h ? lc : lw);
  const double* F = h ? p.theta_m2 : p.w2;
  const int* rec = p.cell_rec + (size_t)c * CELL_REC;
  const int ne = rec[14];
  d2 acc = ld2(F + (size_t)c * stride + off);
#pragma unroll
  for (int m = 0; m < ME; ++m) {
    const d2 v = ld2(F + (size_t)rec[7 + m] * stride + off);
    acc.x += v.x;
    acc.y += v.y;
  }
#pragma unroll
  for (int ie = 0; ie < ME; ++ie) {
    if (!((mask >> ie) & 1)) continue;
    const int e = rec[ie];
    const size_t o = (size_t)e * K + 2 * lc;
    d2 fl = ld2(p.ru + o);
    const int* ac = p.advCellsForEdge + (size_t)e * 15;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const d2 v = ld2(F + (size_t)__builtin_amdgcn_readfirstlane(ac[ne + 1 + f]) * stride + off);
      fl.x += v.x + acc.x;
      fl.y += v.y + acc.y;
    }
    if (2 * l < K) st2((h ? p.advflux_th : p.advflux_w) + o, fl);
  }
}

// the acoustic edge phase with the previous sub-step's damping (k_acoustic_edges_p<true>): 5 columns of
// the edge and 6 fields at both of its cells, two stores -- a plain sum for the arithmetic
__global__ __launch_bounds__(EDGE_THREADS) void f_acoustic_edges(Dims d, Ptrs p) {
  int eA, eB;
  bool hasB;
  if (!pair_edges(d, p, 0, eA, eB, hasB)) return;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, K / 2 - 1);
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const bool onA = ceA.x < d.nCellsSolve || ceA.y < d.nCellsSolve;
  const bool onB = hasB && (ceB.x < d.nCellsSolve || ceB.y < d.nCellsSolve);
  if (!onA && !onB) return;
  const d2 tu = ld2(p.tend_u + o), rp = ld2(p.ru_p + o), ra = ld2(p.ruAvg + o), cq = ld2(p.cqu + o),
           zx = ld2(p.zxu + o);
  const double mask = sel(h, ld_uniform_f64(p.specZoneMaskEdge + eA), ld_uniform_f64(p.specZoneMaskEdge + eB));
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const size_t o1 = (size_t)c1 * K + 2 * lc, o2 = (size_t)c2 * K + 2 * lc;
  d2 acc{tu.x + rp.x + cq.x + zx.x + mask, tu.y + rp.y + cq.y + zx.y};
  const double* fs[6] = {p.rtheta_pp, p.zz, p.exner, p.rho_pp, p.rtheta_pp_old, p.theta_m1};
  for (const double* f : fs) {
    const d2 v1 = ld2(f + o1), v2 = ld2(f + o2);
    acc.x += v1.x + v2.x;
    acc.y += v1.y + v2.y;
  }
  if (2 * l < K && (h ? onB : onA)) {
    st2(p.ru_p + o, acc);
    st2(p.ruAvg + o, d2{ra.x + acc.x, ra.y + acc.y});
  }
}

// k_mono_edges1_p's loads and stores for a pair of scalars (nq = 2): the stencil rows once, per scalar
// 10 stencil columns of the new scalar and the edge's two cells of the old one, three flux arrays
// stored (round 5: two), a plain sum for the arithmetic
__global__ __launch_bounds__(EDGE_THREADS) void f_mono_edges1(Dims d, Ptrs p, int is, int nq, MonoFlux2 f2) {
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, K / 2 - 1);
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  int ic[10];
  double a[10], b[10];
  ld_row(p.advCellsForEdge + (size_t)e * 15, ic);
  ld_row(p.adv_coefs + (size_t)e * 15, a);
  ld_row(p.adv_coefs_3rd + (size_t)e * 15, b);
  const d2 uh = ld2(p.ruAvg + o);
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const int ns = d.ns;
#pragma unroll 1
  for (int q = 0; q < nq; ++q) {
    const int iq = is + q;
    d2 acc = uh;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const d2 v = ld2(p.scalars2 + SIX(ic[j], 2 * lc, iq));
      acc.x += (a[j] + b[j]) * v.x;
      acc.y += (a[j] - b[j]) * v.y;
    }
    const d2 s1 = ld2(p.scalars1 + SIX(c1, 2 * lc, iq)), s2 = ld2(p.scalars1 + SIX(c2, 2 * lc, iq));
    if ((h == 0 || hasB) && 2 * l < K) {
      st2((q ? f2.flux_arr : p.flux_arr) + o, acc);
      st2((q ? f2.flux_upwind_tmp : p.flux_upwind_tmp) + o, d2{s1.x + s2.x, s1.y + s2.y});
    }
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s DUMPDIR [reps] [rounds]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int reps = argc > 2 ? atoi(argv[2]) : 20, rounds = argc > 3 ? atoi(argv[3]) : 5;
  int nC, nE, nV, K, ns;
  {
    FILE* f = fopen((dir + "/meta.txt").c_str(), "r");
    if (!f || fscanf(f, "%d %d %d %d %d", &nC, &nE, &nV, &K, &ns) != 5) {
      fprintf(stderr, "bad %s/meta.txt\n", dir.c_str());
      return 1;
    }
    fclose(f);
  }
  if (K % 2 || K > 64) {
    fprintf(stderr, "even K <= 64 only\n");
    return 1;
  }
  Dims d{};
  d.nCells = nC;
  d.nEdges = nE;
  d.nVertices = nV;
  d.K = K;
  d.maxEdges = 6;
  d.maxEdges2 = 10;
  d.ns = ns;
  d.nCellsSolve = nC;
  d.nEdgesSolve = nE;
  d.nVerticesSolve = nV;
  Ptrs p{};
  p.advCellsForEdge = dev(load<int>(dir, "advCellsForEdge.i32", (size_t)(nE + 1) * 15));
  p.nAdvCellsForEdge = dev(load<int>(dir, "nAdvCellsForEdge.i32", (size_t)nE + 1));
  p.cellsOnEdge = dev(load<int>(dir, "cellsOnEdge.i32", (size_t)(nE + 1) * 2));
  p.edgesOnEdge = dev(load<int>(dir, "edgesOnEdge.i32", (size_t)(nE + 1) * 10));
  p.nEdgesOnEdge = dev(load<int>(dir, "nEdgesOnEdge.i32", (size_t)nE + 1));
  p.adv_coefs = dev(load<double>(dir, "adv_coefs.f64", (size_t)(nE + 1) * 15));
  p.adv_coefs_3rd = dev(load<double>(dir, "adv_coefs_3rd.f64", (size_t)(nE + 1) * 15));
  p.weightsOnEdge = dev(load<double>(dir, "weightsOnEdge.f64", (size_t)(nE + 1) * 10));
  // cell records (k_build_cell_rec's layout) and the c1 list of the cell-centric advflux
  std::vector<int> crec = load<int>(dir, "cell_rec.i32", (size_t)(nC + 1) * CELL_REC);
  p.cell_rec = dev(crec);
  std::vector<int2> c1list;
  {
    std::vector<int> coe = load<int>(dir, "cellsOnEdge.i32", (size_t)(nE + 1) * 2);
    std::vector<int> ace = load<int>(dir, "advCellsForEdge.i32", (size_t)(nE + 1) * 15);
    std::vector<int> nae = load<int>(dir, "nAdvCellsForEdge.i32", (size_t)nE + 1);
    std::vector<int> mask(nC, 0);
    int bad = 0;
    for (int e = 0; e < nE; ++e) {
      const int c = coe[2 * e];
      const int* r = &crec[(size_t)c * CELL_REC];
      const int ne = r[14];
      int ie = -1;
      for (int m = 0; m < ne; ++m)
        if (r[m] == e) ie = m;
      // slots 0 .. ne: c, the cell across e, c's other neighbours in order; then at most ne(c2) - 3 more
      bool ok = ie >= 0 && ace[(size_t)e * 15] == c && ace[(size_t)e * 15 + 1] == r[7 + ie] &&
                nae[e] - (ne + 1) <= 3 && nae[e] >= ne + 1;
      for (int m = 0, j = 2; ok && m < ne; ++m)
        if (m != ie) ok = ace[(size_t)e * 15 + j++] == r[7 + m];
      if (!ok) {
        ++bad;
        continue;
      }
      mask[c] |= 1 << ie;
    }
    for (int c = 0; c < nC; ++c)
      if (mask[c]) c1list.push_back(int2{c, mask[c]});
    printf("cell-centric advflux: %zu c1 cells for %d edges, %d edges off the ring pattern\n", c1list.size(), nE, bad);
  }
  int2* d_c1list = dev(c1list);
  const int n_c1 = (int)c1list.size();
  const size_t cK = (size_t)(nC + 1) * K, cK1 = (size_t)(nC + 1) * (K + 1), eK = (size_t)(nE + 1) * K;
  unsigned seed = 1;
  p.invDcEdge = dev_field(nE + 1, seed++);
  p.fzm = dev_field(K, seed++);
  p.fzp = dev_field(K, seed++);
  p.rdzw = dev_field(K, seed++);
  p.w2 = dev_field(cK1, seed++);
  p.rw = dev_field(cK1, seed++);
  p.theta_m2 = dev_field(cK, seed++);
  p.ke = dev_field(cK, seed++);
  p.h_divergence = dev_field(cK, seed++);
  p.scalars2 = dev_field(cK * ns, seed++);
  p.scalars1 = dev_field(cK * ns, seed++);
  double* fl2[3];
  for (double*& f : fl2) f = dev_field(eK, seed++);
  const MonoFlux2 mf2{fl2[0], fl2[1], fl2[2]};
  p.flux_arr = dev_field(eK, seed++);
  p.flux_upwind_tmp = dev_field(eK, seed++);
  p.flux_tmp = dev_field(eK, seed++);
  p.bdyMaskEdge = dev(std::vector<int>(nE + 1, 0));
  p.dvEdge = dev_field(nE + 1, seed++);  // k_mono_edges1_p's upwind flux
  for (double** f : {&p.ru, &p.ruAvg, &p.advflux_w, &p.advflux_th, &p.rho_edge, &p.u2, &p.pv_edge, &p.tend_u_euler,
                     &p.tend_u, &p.ru_p, &p.cqu})
    *f = dev_field(eK, seed++);
  p.zxu = dev_field(eK, seed++);
  for (double** f : {&p.rtheta_pp, &p.exner, &p.rho_pp, &p.rtheta_pp_old, &p.theta_m1}) *f = dev_field(cK, seed++);
  p.zz = dev_field(cK, seed++);
  {
    std::vector<double> zmask(nE + 1, 0.0);
    p.specZoneMaskEdge = dev(zmask);
  }
  p.horiz_flux_array = dev_field(eK * ns, seed++);
  double* W10 = dev_field((size_t)nE * 10 * (K + 1), seed++);
  double* T10 = dev_field((size_t)nE * 10 * K, seed++);
  Config cf{};
  DynTendScal s{};
  s.rk_step = 2;
  const dim3 blk(EDGE_THREADS), grid((unsigned)(((nE + 1) / 2 + EDGE_WPB - 1) / EDGE_WPB));
  const dim3 gridc((unsigned)((n_c1 + EDGE_WPB - 1) / EDGE_WPB));
  {  // the cell-centric kernel gives the pair kernel's bits
    const size_t eKb = (size_t)(nE + 1) * K * sizeof(double);
    std::vector<double> w0(eKb / 8), t0(eKb / 8), w1(eKb / 8), t1(eKb / 8);
    CK(hipMemset(p.advflux_w, 0, eKb));
    CK(hipMemset(p.advflux_th, 0, eKb));
    hipLaunchKernelGGL((k_dyn_advflux_p<10, false>), grid, blk, 0, 0, d, p);
    CK(hipMemcpy(w0.data(), p.advflux_w, eKb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(t0.data(), p.advflux_th, eKb, hipMemcpyDeviceToHost));
    CK(hipMemset(p.advflux_w, 0, eKb));
    CK(hipMemset(p.advflux_th, 0, eKb));
    hipLaunchKernelGGL(k_advflux_c<6>, gridc, blk, 0, 0, d, p, d_c1list, n_c1);
    CK(hipMemcpy(w1.data(), p.advflux_w, eKb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(t1.data(), p.advflux_th, eKb, hipMemcpyDeviceToHost));
    size_t dw = 0, dtt = 0;
    for (size_t i = 0; i < (size_t)nE * K; ++i) {
      dw += memcmp(&w0[i], &w1[i], 8) != 0;
      dtt += memcmp(&t0[i], &t1[i], 8) != 0;
    }
    printf("cell-centric vs pair kernel: %zu / %zu w values and %zu theta values differ in any bit\n", dw,
           (size_t)nE * K, dtt);
  }
  struct V {
    const char* name;
    std::function<void()> run;
    std::vector<double> us;
  };
  std::vector<V> vs = {
      {"advflux kernel", [&] { hipLaunchKernelGGL((k_dyn_advflux_p<10, false>), grid, blk, 0, 0, d, p); }, {}},
      {"advflux floor", [&] { hipLaunchKernelGGL(f_advflux, grid, blk, 0, 0, d, p); }, {}},
      {"advflux stream", [&] { hipLaunchKernelGGL(s_advflux, grid, blk, 0, 0, d, p, W10, T10); }, {}},
      {"advflux cell", [&] { hipLaunchKernelGGL(k_advflux_c<6>, gridc, blk, 0, 0, d, p, d_c1list, n_c1); }, {}},
      {"advflux cell fl", [&] { hipLaunchKernelGGL(f_advflux_c<6>, gridc, blk, 0, 0, d, p, d_c1list, n_c1); }, {}},
      {"scalars kernel", [&] { hipLaunchKernelGGL((k_scalars_edges_p<10, false>), grid, blk, 0, 0, d, p); }, {}},
      {"scalars floor", [&] { hipLaunchKernelGGL(f_scalars, grid, blk, 0, 0, d, p); }, {}},
      {"dynedges kernel",
       [&] { hipLaunchKernelGGL((k_dyn_edges_p<false, 10, false, false>), grid, blk, 0, 0, d, p, cf, s, 0, XPack{}); },
       {}},
      {"dynedges floor", [&] { hipLaunchKernelGGL(f_dynedges, grid, blk, 0, 0, d, p); }, {}},
      {"acoustic edges",
       [&] { hipLaunchKernelGGL((k_acoustic_edges_p<true, false, false>), grid, blk, 0, 0, d, p, 30.0, 2, 0.1, 0, 0,
                                UnpackMap{}); },
       {}},
      {"acoustic edges fl", [&] { hipLaunchKernelGGL(f_acoustic_edges, grid, blk, 0, 0, d, p); }, {}},
      {"mono edges1 x2", [&] { hipLaunchKernelGGL((k_mono_edges1_p<10, false>), grid, blk, 0, 0, d, p, 0, 30.0,
                                                  ns >= 2 ? 2 : 1, mf2); }, {}},
      {"mono edges1 x2 fl", [&] { hipLaunchKernelGGL(f_mono_edges1, grid, blk, 0, 0, d, p, 0, ns >= 2 ? 2 : 1, mf2); },
       {}},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) v.run();  // warm
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(1e3 * ms / reps);
    }
  CK(hipGetLastError());
  printf("x1.%d, K = %d, ns = %d, %d launches x %d rounds, median us per launch\n", nC, K, ns, reps, rounds);
  for (auto& v : vs) {
    std::sort(v.us.begin(), v.us.end());
    printf("%-16s %8.1f   (min %.1f max %.1f)\n", v.name, v.us[v.us.size() / 2], v.us.front(), v.us.back());
  }
  return 0;
}
