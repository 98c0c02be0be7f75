// The model-init precompute core_atmosphere runs on every start, on the device
// (mpas_atm_core.F:311-358 and 927-1288, called from atm_mpas_init_block): the inverses of the cell /
// triangle areas and edge lengths, atm_compute_signs (edge signs, zb_cell / zb3_cell, kiteForCell),
// atm_adv_coef_compression, atm_couple_coef_3rd_order, atm_compute_mesh_scaling and
// atm_compute_damping_coefs.  Inputs are the init file's fields (deriv_two, zb, zb3, meshDensity,
// areaCell, areaTriangle, zgrid and the connectivity), as the reference reads them from its input
// stream; outputs go to the mesh pool at the declared strides (maxEdges = the block's declared value).
//
// Arithmetic follows the Fortran statement by statement (same operands, same order, fp64, no
// contraction).  Two functions go beyond + - * / sqrt: x**0.25 (a runtime pow in the compiled
// reference) and sin.  The caller may hand in the C library's values (mesh.meshDensity_root4,
// meshDensityEdge_root4, dss_sin: what the compiled reference gets, so the outputs are its bits --
// Dycore(model_init="device") does); without them they are computed here correctly rounded (cr_root4,
// cr_sin below, both proved against a 60-digit evaluation in tests/test_gpu_model_init.py), and the
// reference's C library, which rounds them correctly for all but ~0.1 % of arguments, is 1 ulp away
// there: meshScalingDel2 / RegionalCell / RegionalEdge then differ by up to 2 ulp, dss by up to 4.
// x**0.75 is sqrt(x) * sqrt(sqrt(x)), as the reference build lowers it (init_atm._pow).
// Included by dycore.hip.
#pragma once
#include "dycore.h"

namespace mpas {

// ---- double-double helpers (exact products with fma; fp-contract is off for the library) ----
struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return dd{s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd two_prod(double a, double b) {
  const double p = a * b;
  return dd{p, fma(a, b, -p)};
}
__device__ __forceinline__ dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  const double lo = s.lo + (a.lo + b.lo);
  const double hi = s.hi + lo;
  return dd{hi, lo - (hi - s.hi)};
}
__device__ __forceinline__ dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  const double lo = p.lo + (a.hi * b.lo + a.lo * b.hi);
  const double hi = p.hi + lo;
  return dd{hi, lo - (hi - p.hi)};
}
// sign of (a - b) for double-doubles
__device__ __forceinline__ int dd_cmp(dd a, dd b) {
  const dd d = dd_add(a, dd{-b.hi, -b.lo});
  return (d.hi > 0.0) - (d.hi < 0.0);
}

// x**0.25 correctly rounded, x > 0 finite: y = sqrt(sqrt(x)) is within an ulp or so; the correctly
// rounded root is the double whose rounding interval [y - u/2, y + u/2] holds x**0.25, i.e. whose two
// midpoints m satisfy m_lo**4 <= x < m_hi**4, decided exactly enough in double-double.
__device__ double cr_root4(double x) {
  double y = sqrt(sqrt(x));
  for (int it = 0; it < 4; ++it) {
    const double up = nextafter(y, INFINITY), dn = nextafter(y, 0.0);
    // midpoints as double-doubles: y + (up - y) / 2 (the halves are exact)
    const dd mh = two_sum(y, 0.5 * (up - y)), ml = two_sum(y, -0.5 * (y - dn));
    const dd mh2 = dd_mul(mh, mh), ml2 = dd_mul(ml, ml);
    const dd mh4 = dd_mul(mh2, mh2), ml4 = dd_mul(ml2, ml2);
    const dd xx{x, 0.0};
    if (dd_cmp(xx, mh4) >= 0) y = up;       // the root lies above the upper midpoint
    else if (dd_cmp(xx, ml4) < 0) y = dn;   // below the lower one
    else break;
  }
  return y;
}

// sin(x) correctly rounded for 0 <= x <= pi/2 (the damping layer's argument): the Taylor series in
// double-double, Horner form, 1/(2k+1)! as (hi, lo) pairs.
__constant__ double SIN_C[16][2] = {
    {1.0, 0.0},
    {-0.16666666666666666, -9.25185853854297e-18},
    {0.008333333333333333, 1.1564823173178714e-19},
    {-0.0001984126984126984, -1.7209558293420705e-22},
    {2.7557319223985893e-06, -1.858393274046472e-22},
    {-2.505210838544172e-08, 1.448814070935912e-24},
    {1.6059043836821613e-10, 1.2585294588752098e-26},
    {-7.647163731819816e-13, -7.03872877733453e-30},
    {2.8114572543455206e-15, 1.6508842730861433e-31},
    {-8.22063524662433e-18, -2.2141894119604265e-34},
    {1.9572941063391263e-20, -1.3643503830087908e-36},
    {-3.868170170630684e-23, 8.843177655482344e-40},
    {6.446950284384474e-26, -1.9330404233703465e-42},
    {-9.183689863795546e-29, -1.4303150396787322e-45},
    {1.1309962886447716e-31, 1.0498015412959506e-47},
    {-1.216125041553518e-34, -5.586290567888806e-51},
};
__device__ double cr_sin(double x) {
  const dd x2 = two_prod(x, x);
  dd s{SIN_C[15][0], SIN_C[15][1]};
  for (int k = 14; k >= 0; --k) s = dd_add(dd_mul(s, x2), dd{SIN_C[k][0], SIN_C[k][1]});
  s = dd_mul(s, dd{x, 0.0});
  return s.hi + s.lo;
}

struct MInit {
  // inputs (device, 0-based indices, missing -> the garbage element)
  const int *nEdgesOnCell, *edgesOnCell, *cellsOnCell, *verticesOnCell, *cellsOnEdge, *verticesOnEdge;
  const int *cellsOnVertex, *edgesOnVertex;
  const double *deriv_two, *zb, *zb3, *meshDensity, *areaCell, *areaTriangle, *dcEdge, *dvEdge, *zgrid;
  // outputs
  double *invAreaCell, *invDvEdge, *invDcEdge, *invAreaTriangle;
  double *edgesOnVertex_sign, *edgesOnCell_sign, *zb_cell, *zb3_cell;
  int *kiteForCell, *nAdvCellsForEdge, *advCellsForEdge;
  double *adv_coefs, *adv_coefs_3rd;
  double *meshScalingDel2, *meshScalingDel4, *meshScalingRegionalCell, *meshScalingRegionalEdge, *dss;
  // the caller's C-library values (mesh.meshDensity_root4, meshDensityEdge_root4, dss_sin), or nullptr:
  // correctly rounded ones are computed here
  const double *root4_cell, *root4_edge, *dss_sin;
  int nCells, nEdges, nVertices, K, maxEdges;  // maxEdges: the declared stride
};

__device__ __forceinline__ int gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }

// 339-353
__global__ void k_mi_inverses(MInit m) {
  const int i = gtid();
  if (i < m.nCells) m.invAreaCell[i] = 1.0 / m.areaCell[i];
  if (i < m.nEdges) {
    m.invDvEdge[i] = 1.0 / m.dvEdge[i];
    m.invDcEdge[i] = 1.0 / m.dcEdge[i];
  }
  if (i < m.nVertices) m.invAreaTriangle[i] = 1.0 / m.areaTriangle[i];
}

// atm_compute_signs, 1023-1035 (vertexDegree 3)
__global__ void k_mi_vertex_signs(MInit m) {
  const int v = gtid();
  if (v >= m.nVertices) return;
  for (int i = 0; i < 3; ++i) {
    const int e = m.edgesOnVertex[3 * v + i];
    m.edgesOnVertex_sign[3 * v + i] = e < m.nEdges ? (v == m.verticesOnEdge[2 * e + 1] ? 1.0 : -1.0) : 0.0;
  }
}

// 1037-1053: one thread per (cell, slot); the zb / zb3 column of the slot's edge side is copied
__global__ void k_mi_cell_signs(MInit m) {
  const int t = gtid();
  if (t >= m.nCells * m.maxEdges) return;
  const int c = t / m.maxEdges, i = t - c * m.maxEdges;
  if (i >= m.nEdgesOnCell[c]) return;
  const int e = m.edgesOnCell[(size_t)c * m.maxEdges + i];
  const size_t K1 = m.K + 1, slot = (size_t)c * m.maxEdges + i;
  if (e < m.nEdges) {
    const int side = c == m.cellsOnEdge[2 * e] ? 0 : 1;
    m.edgesOnCell_sign[slot] = side == 0 ? 1.0 : -1.0;
    for (size_t k = 0; k < K1; ++k) {
      m.zb_cell[slot * K1 + k] = m.zb[((size_t)e * 2 + side) * K1 + k];
      m.zb3_cell[slot * K1 + k] = m.zb3[((size_t)e * 2 + side) * K1 + k];
    }
  } else {
    m.edgesOnCell_sign[slot] = 0.0;
  }
  // 1055-1072: kiteForCell, the 1-based position of the cell among its vertex's cells (0-based here)
  const int v = m.verticesOnCell[slot];
  if (v < m.nVertices) {
    for (int j = 0; j < 3; ++j)
      if (c == m.cellsOnVertex[3 * v + j]) {
        m.kiteForCell[slot] = j;
        break;
      }
  } else {
    m.kiteForCell[slot] = 0;
  }
}

// atm_adv_coef_compression, 1154-1264, one thread per edge; the list and the sums in the reference's
// order (j_in = the last list position holding the cell)
__global__ void k_mi_adv_compression(MInit m) {
  const int e = gtid();
  if (e >= m.nEdges) return;
  m.nAdvCellsForEdge[e] = 0;
  const int c1 = m.cellsOnEdge[2 * e], c2 = m.cellsOnEdge[2 * e + 1];
  if (!(c1 < m.nCells || c2 < m.nCells)) return;
  int lst[20];
  lst[0] = c1;
  lst[1] = c2;
  int n = 2;
  const int ne1 = m.nEdgesOnCell[c1], ne2 = m.nEdgesOnCell[c2];
  for (int i = 0; i < ne1; ++i) {
    const int cc = m.cellsOnCell[(size_t)c1 * m.maxEdges + i];
    if (cc != c2) lst[n++] = cc;
  }
  for (int i = 0; i < ne2; ++i) {
    const int cc = m.cellsOnCell[(size_t)c2 * m.maxEdges + i];
    bool add = true;
    for (int j = 0; j < n; ++j)
      if (lst[j] == cc) add = false;
    if (add) lst[n++] = cc;
  }
  m.nAdvCellsForEdge[e] = n;
  for (int j = 0; j < 15; ++j) m.advCellsForEdge[(size_t)e * 15 + j] = j < n ? lst[j] : m.nCells;  // unused: none
  double a[20], b[20];
  for (int j = 0; j < 20; ++j) a[j] = b[j] = 0.0;
  auto jin = [&](int cell) {
    int r = -1;
    for (int j = 0; j < n; ++j)
      if (lst[j] == cell) r = j;
    return r;
  };
  const double* d2 = m.deriv_two + (size_t)e * 30;  // deriv_two(15, 2, nEdges+1)
  // every cell looked up is in the list by construction (j >= 0)
  int j = jin(c1);
  a[j] = a[j] + d2[0];
  b[j] = b[j] + d2[0];
  for (int i = 0; i < ne1; ++i) {
    j = jin(m.cellsOnCell[(size_t)c1 * m.maxEdges + i]);
    a[j] = a[j] + d2[i + 1];
    b[j] = b[j] + d2[i + 1];
  }
  j = jin(c2);
  a[j] = a[j] + d2[15];
  b[j] = b[j] - d2[15];
  for (int i = 0; i < ne2; ++i) {
    j = jin(m.cellsOnCell[(size_t)c2 * m.maxEdges + i]);
    a[j] = a[j] + d2[15 + i + 1];
    b[j] = b[j] - d2[15 + i + 1];
  }
  const double dc = m.dcEdge[e], dv = m.dvEdge[e];
  for (j = 0; j < n; ++j) {
    a[j] = -(dc * dc) * a[j] / 12.;
    b[j] = -(dc * dc) * b[j] / 12.;
  }
  j = jin(c1);
  a[j] = a[j] + 0.5;
  j = jin(c2);
  a[j] = a[j] + 0.5;
  for (j = 0; j < 15; ++j) {  // adv_coefs(:, iEdge) = 0 first (1195-1196); 15 = the array's FIFTEEN
    m.adv_coefs[(size_t)e * 15 + j] = j < n ? dv * a[j] : 0.0;
    m.adv_coefs_3rd[(size_t)e * 15 + j] = j < n ? dv * b[j] : 0.0;
  }
}

// atm_couple_coef_3rd_order, 1285-1286: every element of both arrays, garbage slot included
__global__ void k_mi_couple(double* a, int64_t n, double coef) {
  for (int64_t i = gtid(); i < n; i += (int64_t)gridDim.x * blockDim.x) a[i] = coef * a[i];
}

// atm_compute_mesh_scaling, 956-982 (config_h_ScaleWithMesh = scale)
__global__ void k_mi_mesh_scaling(MInit m, int scale) {
  const int i = gtid();
  if (i < m.nEdges) {
    double s2 = 1.0, s4 = 1.0, sr = 1.0;
    if (scale) {
      const int c1 = m.cellsOnEdge[2 * i], c2 = m.cellsOnEdge[2 * i + 1];
      const double x = (m.meshDensity[c1] + m.meshDensity[c2]) / 2.0;
      s2 = 1.0 / (m.root4_edge ? m.root4_edge[i] : cr_root4(x));
      s4 = 1.0 / (sqrt(x) * sqrt(sqrt(x)));
      sr = s2;
    }
    m.meshScalingDel2[i] = s2;
    m.meshScalingDel4[i] = s4;
    m.meshScalingRegionalEdge[i] = sr;
  }
  if (i < m.nCells)
    m.meshScalingRegionalCell[i] = scale ? 1.0 / (m.root4_cell ? m.root4_cell[i] : cr_root4(m.meshDensity[i])) : 1.0;
}

// atm_compute_damping_coefs, 1105-1116: one thread per (cell, level)
__global__ void k_mi_damping(MInit m, double zd, double xnutr) {
  const int t = gtid();
  if (t >= m.nCells * m.K) return;
  const int c = t / m.K, k = t - c * m.K;
  const size_t K1 = m.K + 1;
  const double pii = 3.141592653589793;  // acos(-1.0)
  const double zt = m.zgrid[(size_t)c * K1 + m.K];
  const double z = 0.5 * (m.zgrid[(size_t)c * K1 + k] + m.zgrid[(size_t)c * K1 + k + 1]);
  double v = 0.0;
  if (z > zd) {
    const double s = m.dss_sin ? m.dss_sin[(size_t)c * m.K + k] : cr_sin(0.5 * pii * (z - zd) / (zt - zd));
    v = xnutr * (s * s);
    v = v / (m.root4_cell ? m.root4_cell[c] : cr_root4(m.meshDensity[c]));
  }
  m.dss[(size_t)c * m.K + k] = v;
}

// ---- deriv_two (core_init_atmosphere/mpas_atm_advection.F:21-394, atm_initialize_advection_rk,
// polynomial_order = 2, on a sphere): the arithmetic half, one thread per cell.  The caller hands in
// the transcendental half per cell and edgesOnCell slot (stride maxEdges): xp / yp of the neighbour
// cellsOnCell(i) in the cell's tangent plane (132-181) and sin / cos of the edge's normal angle thetae
// (303-315, 334-335 / 347-348).  Here: amatrix (215-226), poly_fit_2 (567-614) with h = wt w the
// identity, MIGS / ELGS (633-741) and the weights 2 cos^2 b(4,j) + 2 cos sin b(5,j) + 2 sin^2 b(6,j)
// (336-357) for each edge, on the side the cell takes in cellsOnEdge.  Matrix products sum their inner
// index from the first term up, starting from 0.0, as the compiled matmul does (init_atm._matmul_seq).
struct D2Fit {
  const int *nEdgesOnCell, *edgesOnCell, *cellsOnEdge;  // device, 0-based
  const double *xp, *yp, *sin_the, *cos_the;              // (nCells, maxEdges)
  double* deriv_two;                                      // (nEdges + 1, 2, 15)
  int* bad;                                               // set when a cell has more than 14 edges
  int nCells, nEdges, maxEdges;
};
constexpr int D2_MAXM = 15;  // the cell and up to 14 neighbours (deriv_two holds 15 weights per side)

__global__ void k_mi_deriv_two(D2Fit q) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= q.nCells) return;
  const int ne = q.nEdgesOnCell[c];
  if (ne < 1 || ne > q.maxEdges || ne + 1 > D2_MAXM) {
    if (ne + 1 > D2_MAXM) *q.bad = 1;
    return;
  }
  const int m = ne + 1;  // ma
  double a[D2_MAXM][6];
  a[0][0] = 1.;
  for (int j = 1; j < 6; ++j) a[0][j] = 0.;
  for (int i = 1; i < m; ++i) {
    const double x = q.xp[(size_t)c * q.maxEdges + i - 1], y = q.yp[(size_t)c * q.maxEdges + i - 1];
    a[i][0] = 1.;
    a[i][1] = x;
    a[i][2] = y;
    a[i][3] = x * x;
    a[i][4] = x * y;
    a[i][5] = y * y;
  }
  // ath = matmul(transpose(a), h), h the m x m identity
  double ath[6][D2_MAXM];
  for (int r = 0; r < 6; ++r)
    for (int col = 0; col < m; ++col) {
      double s = 0.0;
      for (int k = 0; k < m; ++k) s = s + a[k][r] * (k == col ? 1.0 : 0.0);
      ath[r][col] = s;
    }
  // atha = matmul(ath, a)
  double A[6][6];
  for (int r = 0; r < 6; ++r)
    for (int col = 0; col < 6; ++col) {
      double s = 0.0;
      for (int k = 0; k < m; ++k) s = s + ath[r][k] * a[k][col];
      A[r][col] = s;
    }
  // ELGS (678-741): partial-pivoting elimination, pivot order in indx
  int indx[6];
  double cs[6];
  for (int i = 0; i < 6; ++i) {
    indx[i] = i;
    double c1 = 0.0;
    for (int j = 0; j < 6; ++j) c1 = fmax(c1, fabs(A[i][j]));
    cs[i] = c1;
  }
  for (int j = 0; j < 5; ++j) {
    double pi1 = 0.0;
    int k = j;
    for (int i = j; i < 6; ++i) {
      const double pi = fabs(A[indx[i]][j]) / cs[indx[i]];
      if (pi > pi1) {
        pi1 = pi;
        k = i;
      }
    }
    const int t = indx[j];
    indx[j] = indx[k];
    indx[k] = t;
    for (int i = j + 1; i < 6; ++i) {
      const double pj = A[indx[i]][j] / A[indx[j]][j];
      A[indx[i]][j] = pj;
      for (int kk = j + 1; kk < 6; ++kk) A[indx[i]][kk] = A[indx[i]][kk] - pj * A[indx[j]][kk];
    }
  }
  // MIGS (633-675)
  double B[6][6], X[6][6];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) B[i][j] = i == j ? 1.0 : 0.0;
  for (int i = 0; i < 5; ++i)
    for (int j = i + 1; j < 6; ++j)
      for (int k = 0; k < 6; ++k) B[indx[j]][k] = B[indx[j]][k] - A[indx[j]][i] * B[indx[i]][k];
  for (int i = 0; i < 6; ++i) {
    X[5][i] = B[indx[5]][i] / A[indx[5]][5];
    for (int j = 4; j >= 0; --j) {
      double v = B[indx[j]][i];
      for (int k = j + 1; k < 6; ++k) v = v - A[indx[j]][k] * X[k][i];
      X[j][i] = v / A[indx[j]][j];
    }
  }
  // b = matmul(atha_inv, ath): only rows 4..6 (the second-derivative terms) are used
  double b[3][D2_MAXM];
  for (int r = 3; r < 6; ++r)
    for (int col = 0; col < m; ++col) {
      double s = 0.0;
      for (int k = 0; k < 6; ++k) s = s + X[r][k] * ath[k][col];
      b[r - 3][col] = s;
    }
  for (int i = 0; i < ne; ++i) {
    const int e = q.edgesOnCell[(size_t)c * q.maxEdges + i];
    if (e < 0 || e >= q.nEdges) continue;
    const double cs_ = q.cos_the[(size_t)c * q.maxEdges + i], sn_ = q.sin_the[(size_t)c * q.maxEdges + i];
    const double costsint = cs_ * sn_, cos2t = cs_ * cs_, sin2t = sn_ * sn_;
    const int side = q.cellsOnEdge[2 * e] == c ? 0 : 1;
    double* out = q.deriv_two + ((size_t)e * 2 + side) * 15;
    for (int j = 0; j < m; ++j) out[j] = 2. * cos2t * b[0][j] + 2. * costsint * b[1][j] + 2. * sin2t * b[2][j];
  }
}

// ---- zb / zb3, the z-metric terms of the omega equation (core_init_atmosphere/
// mpas_init_atm_cases.F:1045-1093), one thread per edge and level: the second derivative of zgrid
// across the edge from deriv_two (each side's sum from the cell itself, then cellsOnCell in order),
// z_edge and z_edge3 for config_theta_adv_order 2 / 3 / 4, over dvEdge / areaCell of each side.
// Edges without an owned cell keep 0, as does level nVertLevels+1.
struct ZbFit {
  const int *nEdgesOnCell, *cellsOnCell, *cellsOnEdge;
  const double *deriv_two, *zgrid, *dcEdge, *dvEdge, *areaCell;
  double *zb, *zb3;
  int nCells, nCellsSolve, nEdges, K, maxEdges, order;
};

__global__ void k_mi_zb(ZbFit q) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)q.nEdges * q.K) return;
  const int e = (int)(t / q.K), k = (int)(t % q.K);
  const int c1 = q.cellsOnEdge[2 * e], c2 = q.cellsOnEdge[2 * e + 1];
  if (!(c1 < q.nCellsSolve || c2 < q.nCellsSolve)) return;
  const size_t K1 = (size_t)q.K + 1;
  const double z1 = q.zgrid[(size_t)c1 * K1 + k], z2 = q.zgrid[(size_t)c2 * K1 + k];
  double z_edge, z_edge3 = 0.;
  if (q.order == 2) {
    z_edge = (z1 + z2) / 2.;
  } else {
    const double* d1 = q.deriv_two + ((size_t)e * 2 + 0) * 15;
    const double* d2 = q.deriv_two + ((size_t)e * 2 + 1) * 15;
    double f1 = d1[0] * z1, f2 = d2[0] * z2;
    const int n1 = q.nEdgesOnCell[c1], n2 = q.nEdgesOnCell[c2];
    for (int i = 0; i < n1 && i < q.maxEdges; ++i)
      f1 = f1 + d1[i + 1] * q.zgrid[(size_t)q.cellsOnCell[(size_t)c1 * q.maxEdges + i] * K1 + k];
    for (int i = 0; i < n2 && i < q.maxEdges; ++i)
      f2 = f2 + d2[i + 1] * q.zgrid[(size_t)q.cellsOnCell[(size_t)c2 * q.maxEdges + i] * K1 + k];
    const double dc = q.dcEdge[e];
    z_edge = 0.5 * (z1 + z2) - (dc * dc) * (f1 + f2) / 12.;
    if (q.order == 3) z_edge3 = -((dc * dc) * (f1 - f2) / 12.);
  }
  const double dv = q.dvEdge[e];
  q.zb[((size_t)e * 2 + 0) * K1 + k] = (z_edge - z1) * dv / q.areaCell[c1];
  q.zb[((size_t)e * 2 + 1) * K1 + k] = (z_edge - z2) * dv / q.areaCell[c2];
  q.zb3[((size_t)e * 2 + 0) * K1 + k] = z_edge3 * dv / q.areaCell[c1];
  q.zb3[((size_t)e * 2 + 1) * K1 + k] = z_edge3 * dv / q.areaCell[c2];
}

// ---- coeffs_reconstruct (mpas_rbf_interp_initialize -> mpas_initialize_vectors,
// operators/mpas_vector_operations.F:697-769, then mpas_init_reconstruct,
// operators/mpas_vector_reconstruction.F:112-177 with mpas_rbf_interp_func_3D_plane_vec_const_dir_comp_coeffs,
// mpas_rbf_interpolation.F:1079-1145), what mpas_atm_core.F:408-409 runs at model init, one thread per
// cell: the edge normals (unit(x(cell2) - x(cell1))), the cell's tangent plane, and the RBF system of
// its edges (inverse multiquadric, a constant vector in the plane) solved by elgs + mpas_legs
// (:1670-1846).  + - * / sqrt only, each in the Fortran's order (sum() over R3 as (a1 + a2) + a3, **2 as
// x * x): bit for bit the reference's coefficients (reconstruct.py is the host restatement).
struct RecInit {
  const int *nEdgesOnCell, *edgesOnCell, *cellsOnEdge;
  const double *xCell, *yCell, *zCell, *xEdge, *yEdge, *zEdge;
  double* coeffs;  // (nCells + 1, maxEdges, 3)
  int* bad;
  int nCells, maxEdges;
};
constexpr int REC_MAXE = 14, REC_MAXN = REC_MAXE + 2;

struct v3 {
  double x, y, z;
};
__device__ __forceinline__ double sum3(v3 a) { return (a.x + a.y) + a.z; }
__device__ __forceinline__ v3 unit3(v3 v) {
  const double mag = sqrt((v.x * v.x + v.y * v.y) + v.z * v.z);
  return v3{v.x / mag, v.y / mag, v.z / mag};
}
__device__ __forceinline__ double rbf_imq(double r2) { return 1 / sqrt(1 + r2); }

__global__ void k_mi_reconstruct(RecInit q) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= q.nCells) return;
  const int pc = q.nEdgesOnCell[c];
  if (pc < 1 || pc > q.maxEdges || pc > REC_MAXE) {
    if (pc > REC_MAXE) *q.bad = 1;
    return;
  }
  auto xc = [&](int i) { return v3{q.xCell[i], q.yCell[i], q.zCell[i]}; };
  auto normal = [&](int e) {  // edgeNormalVectors(:, e)
    const v3 a = xc(q.cellsOnEdge[2 * e]), b = xc(q.cellsOnEdge[2 * e + 1]);
    return unit3(v3{b.x - a.x, b.y - a.y, b.z - a.z});
  };
  const v3 center = xc(c);
  const v3 rhat = unit3(center);  // localVerticalUnitVectors
  // cellTangentPlane: the first edge's normal with its radial part removed, and rhat x xhat
  const v3 n1 = normal(q.edgesOnCell[(size_t)c * q.maxEdges]);
  const double ndr = sum3(v3{n1.x * rhat.x, n1.y * rhat.y, n1.z * rhat.z});
  const v3 b1 = unit3(v3{n1.x - ndr * rhat.x, n1.y - ndr * rhat.y, n1.z - ndr * rhat.z});
  const v3 b2 = unit3(v3{rhat.y * b1.z - rhat.z * b1.y, rhat.z * b1.x - rhat.x * b1.z, rhat.x * b1.y - rhat.y * b1.x});
  double ps[REC_MAXE][2], pu[REC_MAXE][2];
  double alpha = 0.0;
  for (int i = 0; i < pc; ++i) {
    const int e = q.edgesOnCell[(size_t)c * q.maxEdges + i];
    const v3 loc{q.xEdge[e], q.yEdge[e], q.zEdge[e]};
    const v3 d{center.x - loc.x, center.y - loc.y, center.z - loc.z};
    alpha = alpha + sqrt(sum3(v3{d.x * d.x, d.y * d.y, d.z * d.z}));
    const v3 nor = normal(e);
    ps[i][0] = sum3(v3{loc.x * b1.x, loc.y * b1.y, loc.z * b1.z});
    ps[i][1] = sum3(v3{loc.x * b2.x, loc.y * b2.y, loc.z * b2.z});
    pu[i][0] = sum3(v3{nor.x * b1.x, nor.y * b1.y, nor.z * b1.z});
    pu[i][1] = sum3(v3{nor.x * b2.x, nor.y * b2.y, nor.z * b2.z});
  }
  alpha = alpha / pc;
  const double pd0 = sum3(v3{center.x * b1.x, center.y * b1.y, center.z * b1.z});
  const double pd1 = sum3(v3{center.x * b2.x, center.y * b2.y, center.z * b2.z});
  const double a2 = alpha * alpha;
  const int N = pc + 2;
  double M[REC_MAXN][REC_MAXN], R[REC_MAXN][2];
  for (int i = 0; i < N; ++i) {
    for (int j = 0; j < N; ++j) M[i][j] = 0.0;
    R[i][0] = R[i][1] = 0.0;
  }
  for (int j = 0; j < pc; ++j)
    for (int i = j; i < pc; ++i) {
      const double d0 = ps[i][0] - ps[j][0], d1 = ps[i][1] - ps[j][1];
      const double r2 = (d0 * d0 + d1 * d1) / a2;
      const double dot = pu[i][0] * pu[j][0] + pu[i][1] * pu[j][1];
      M[i][j] = rbf_imq(r2) * dot;
      M[j][i] = M[i][j];
    }
  for (int j = 0; j < pc; ++j) {
    const double d0 = pd0 - ps[j][0], d1 = pd1 - ps[j][1];
    const double f = rbf_imq((d0 * d0 + d1 * d1) / a2);
    R[j][0] = f * pu[j][0];
    R[j][1] = f * pu[j][1];
  }
  for (int i = 0; i < pc; ++i) {
    M[i][pc] = pu[i][0];
    M[i][pc + 1] = pu[i][1];
    M[pc][i] = pu[i][0];
    M[pc + 1][i] = pu[i][1];
  }
  R[pc][0] = 1.0;
  R[pc + 1][1] = 1.0;
  // elgs: scaled partial pivoting
  int indx[REC_MAXN];
  double C[REC_MAXN];
  for (int i = 0; i < N; ++i) {
    indx[i] = i;
    double c1 = 0.0;
    for (int j = 0; j < N; ++j) c1 = fmax(c1, fabs(M[i][j]));
    C[i] = c1;
  }
  for (int j = 0; j < N - 1; ++j) {
    double pi1 = 0.0;
    int k = j;
    for (int i = j; i < N; ++i) {
      const double pi = fabs(M[indx[i]][j]) / C[indx[i]];
      if (pi > pi1) {
        pi1 = pi;
        k = i;
      }
    }
    const int t = indx[j];
    indx[j] = indx[k];
    indx[k] = t;
    for (int i = j + 1; i < N; ++i) {
      const double pj = M[indx[i]][j] / M[indx[j]][j];
      M[indx[i]][j] = pj;
      for (int kk = j + 1; kk < N; ++kk) M[indx[i]][kk] = M[indx[i]][kk] - pj * M[indx[j]][kk];
    }
  }
  // mpas_legs: forward elimination of both right-hand sides, back substitution
  for (int i = 0; i < N - 1; ++i)
    for (int j = i + 1; j < N; ++j)
      for (int r = 0; r < 2; ++r) R[indx[j]][r] = R[indx[j]][r] - M[indx[j]][i] * R[indx[i]][r];
  double X[REC_MAXN][2];
  for (int r = 0; r < 2; ++r) X[N - 1][r] = R[indx[N - 1]][r] / M[indx[N - 1]][N - 1];
  for (int i = N - 2; i >= 0; --i)
    for (int r = 0; r < 2; ++r) {
      double xi = R[indx[i]][r];
      for (int j = i + 1; j < N; ++j) xi = xi - M[indx[i]][j] * X[j][r];
      X[i][r] = xi / M[indx[i]][i];
    }
  double* out = q.coeffs + (size_t)c * q.maxEdges * 3;
  for (int i = 0; i < q.maxEdges; ++i) {
    const bool on = i < pc;
    out[i * 3 + 0] = on ? b1.x * X[i][0] + b2.x * X[i][1] : 0.0;
    out[i * 3 + 1] = on ? b1.y * X[i][0] + b2.y * X[i][1] : 0.0;
    out[i * 3 + 2] = on ? b1.z * X[i][0] + b2.z * X[i][1] : 0.0;
  }
}

}  // namespace mpas
