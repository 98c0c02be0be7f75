// Hand-written CDNA4 (gfx950) HIP kernels for the MPAS-Atmosphere split-explicit
// dycore time step (src/core_atmosphere/dynamics/mpas_atm_time_integration.F).
//
// Execution model: one 64-lane wavefront per column, lane = k.
// Blocks are 256 threads = 4 columns.  Element indices are made wave-uniform
// with readfirstlane so connectivity/geometry loads go through the scalar unit,
// and every field access is a contiguous K*8-byte column segment.  Vertical
// neighbours (k-1, k+1, k-2) come from cross-lane shuffles; the sequential
// vertical recurrences (Thomas sweeps, alpha/gamma LU factors) are evaluated
// in the reference operation order with v_readlane, so results track the
// Fortran to rounding (parity bar: DESIGN.md §6).
//
// Each kernel cites the reference lines it implements.  Arithmetic keeps the
// Fortran left-to-right expression trees -- the build
// uses -ffp-contract=off so no FMA re-association happens either.
#include "dycore.h"

namespace mpas {

#ifdef MPAS_WIDE
// Wide columns (the library's second and third builds, nVertLevels 64..127 and 128..255; dycore.hip
// picks the build per context): one column per workgroup of WIDE_THREADS lanes (128 / 256), lane =
// level, and the cross-lane moves below go through LDS.  The kernel bodies are the same source.
#ifndef WIDE_THREADS
#define WIDE_THREADS 128
#endif
#define WAVES_PER_BLOCK 1
#define BLOCK_THREADS WIDE_THREADS
#else
#ifndef WAVES_PER_BLOCK
#define WAVES_PER_BLOCK 4  // at most 4 (summary.hip's per-wave partials)
#endif
#define BLOCK_THREADS (64 * WAVES_PER_BLOCK)
#endif

// XCD-aware block order.  Workgroups are dealt round-robin to the 8 XCDs, each with
// its own 4 MiB L2; remapping blockIdx so that XCD x runs one contiguous 1/8 of the
// (space-filling-curve ordered) elements keeps every neighbour gather of an edge or
// cell stencil inside the L2 that already holds its neighbours' columns.  The map is a
// bijection for any grid size, so correctness never depends on the actual placement.
__device__ __forceinline__ int xcd_block() {
#ifdef NO_XCD_REMAP
  return blockIdx.x;
#endif
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q = nb >> 3, r = nb & 7, x = bid & 7, i = bid >> 3;
  return x * q + min(x, r) + i;
}

// element of this wavefront, wave-uniform (scalar register)
#ifdef MPAS_WIDE
__device__ __forceinline__ int wave_elem(int start) { return __builtin_amdgcn_readfirstlane(start + xcd_block()); }
__device__ __forceinline__ int lane_id() { return threadIdx.x; }
#else
__device__ __forceinline__ int wave_elem(int start) {
  int e = start + xcd_block() * WAVES_PER_BLOCK + (threadIdx.x >> 6);
  return __builtin_amdgcn_readfirstlane(e);
}
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
#endif

// edge-stencil kernels (TRiSK / advection / acoustic edge phases) run EDGE_WPB waves per
// workgroup: consecutive (SFC-ordered) edges of one workgroup share neighbour columns in the CU's L1
#ifdef MPAS_WIDE
#define EDGE_WPB 1
#define EDGE_THREADS WIDE_THREADS
__device__ __forceinline__ int wave_elem_e() { return __builtin_amdgcn_readfirstlane(xcd_block()); }
#else
#ifndef EDGE_WPB
#define EDGE_WPB 4
#endif
#define EDGE_THREADS (64 * EDGE_WPB)
__device__ __forceinline__ int wave_elem_e() {
  int e = xcd_block() * EDGE_WPB + (threadIdx.x >> 6);
  return __builtin_amdgcn_readfirstlane(e);
}
#endif

// Scalar arrays are scalar-major in HBM: scalars / scalars_tend as [ns][nCells+1][K],
// horiz_flux_array as [ns][nEdges+1][K], so every per-scalar access is a contiguous
// column (the Fortran image (ns, K, n+1) is transposed at the C ABI).
#define SIX(c, k, is) (((size_t)(is) * (size_t)(d.nCells + 1) + (size_t)(c)) * (size_t)K + (size_t)(k))
#define HIX(e, k, is) (((size_t)(is) * (size_t)(d.nEdges + 1) + (size_t)(e)) * (size_t)K + (size_t)(k))

// per-cell edge terms kept in registers up to this many edges (hexagons and pentagons);
// larger cells take the plain loop
constexpr int MAX_EDGES_UNROLL = 6;
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// value held by lane-1 (k-1) / lane+1 (k+1); the end lanes keep their own value (as __shfl_up /
// __shfl_down do).  DPP wavefront shifts (wave_shr:1 / wave_shl:1, GFX9 DPP controls 0x138 /
// 0x130) move the two halves of a double through the VALU, without the LDS round trip of
// ds_bpermute.
#ifdef MPAS_WIDE
// the column spans several wavefronts: every move is a store to LDS, a barrier and a load.  Every
// call site is reached by all lanes of the workgroup (the kernels keep these moves out of
// lane-dependent branches, which the wavefront DPP forms need as well); the first barrier keeps a
// move from overwriting the previous one's values before every lane has read them -- which also
// lets every helper below use the same LDS rows.
#define WIDE_LDS_ROWS 8
__shared__ double wide_lds[WIDE_LDS_ROWS][WIDE_THREADS];
__device__ __forceinline__ double col_move(double x, int delta, bool zero_end) {
  __syncthreads();
  wide_lds[0][threadIdx.x] = x;
  __syncthreads();
  const int s = (int)threadIdx.x + delta;
  if (s < 0 || s >= WIDE_THREADS) return zero_end ? 0.0 : x;
  return wide_lds[0][s];
}
// N values moved by delta = -1 (up1: value of level k-1) or +1 (dn1: level k+1) in one LDS round
// trip; the end lanes keep their own value
template <int N>
__device__ __forceinline__ void col_shift(double (&v)[N], int delta) {
  static_assert(N <= WIDE_LDS_ROWS, "LDS rows");
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) wide_lds[i][threadIdx.x] = v[i];
  __syncthreads();
  const int s = (int)threadIdx.x + delta;
  if (s >= 0 && s < WIDE_THREADS) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = wide_lds[i][s];
  }
}
__device__ __forceinline__ double up1(double x) { return col_move(x, -1, false); }
__device__ __forceinline__ double dn1(double x) { return col_move(x, 1, false); }
__device__ __forceinline__ double up2(double x) { return col_move(x, -2, false); }
__device__ __forceinline__ double up1z(double x) { return col_move(x, -1, true); }
__device__ __forceinline__ double dn1z(double x) { return col_move(x, 1, true); }
#elif !defined(MPAS_SHFL_BPERMUTE)
__device__ __forceinline__ double up1(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false),
                          __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ double dn1(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false),
                          __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false));
}
#else
__device__ __forceinline__ double up1(double x) { return __shfl_up(x, 1, 64); }
__device__ __forceinline__ double dn1(double x) { return __shfl_down(x, 1, 64); }
#endif
#ifndef MPAS_WIDE
template <int N>
__device__ __forceinline__ void col_shift(double (&v)[N], int delta) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = delta < 0 ? up1(v[i]) : dn1(v[i]);
}
#endif
#ifndef MPAS_WIDE
__device__ __forceinline__ double up2(double x) { return __shfl_up(x, 2, 64); }
// lane-1 / lane+1 value with 0.0 shifted in at the end lane
// (bound_ctrl: the out-of-range lane reads 0)
__device__ __forceinline__ double up1z(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, 0x138, 0xf, 0xf, true),
                          __builtin_amdgcn_mov_dpp(lo, 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ double dn1z(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, 0x130, 0xf, 0xf, true),
                          __builtin_amdgcn_mov_dpp(lo, 0x130, 0xf, 0xf, true));
}
#endif

// The column's tridiagonal sweeps (mpas_atm_time_integration.F:2675-2682) with lane = level.
// Forward x(k) = (x(k) - a(k) x(k-1)) alpha(k), k = 2..K (lanes 1..K-1), then backward
// x(k) = x(k) - gamma(k) x(k+1), k = K..1 (lanes K-1..0).  Instead of one lane per iteration,
// every lane re-evaluates its update from its neighbour's current value each iteration: after
// iteration j lanes <= j (forward) / >= K-1-j (backward) hold their final values, and each is
// computed from exactly the operands the sequential recurrence uses, so the result is the same
// bit for bit.  Lanes outside the sweep take a = 0, alpha = 1 / gamma = 0 and keep their value.
__device__ __forceinline__ double thomas_column(double r, double a, double alpha, double gamma, int k, int K) {
  const bool fwd = k >= 1 && k < K, bwd = k < K;
  const double af = fwd ? a : 0.0, alf = fwd ? alpha : 1.0, gb = bwd ? gamma : 0.0;
  double x = r;
  for (int it = 1; it < K; ++it) x = (r - af * up1z(x)) * alf;
  const double xf = x;
  for (int it = 0; it < K; ++it) x = xf - gb * dn1z(x);
  return x;
}

// A wave-uniform fp64 mesh value read as two int32 halves: integer loads cannot alias the
// kernel's fp64 stores (TBAA), so the compiler proves them unclobbered and issues them on the
// scalar unit (SGPRs) instead of spending vector registers on a broadcast.
__device__ __forceinline__ double ld_uniform_f64(const double* a) {
  const int* q = reinterpret_cast<const int*>(a);
  return __hiloint2double(q[1], q[0]);
}

#ifdef MPAS_WIDE
// DPP wavefront shifts (as up1 / dn1 of the one-wavefront build): value of lane-1 / lane+1, own at
// the end lane
__device__ __forceinline__ double wave_shr1(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false),
                          __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ double wave_shl1(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false),
                          __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false));
}
// The column's tridiagonal sweeps (2675-2682) in the wide build: forward x(k) = (x(k) - a(k) x(k-1))
// alpha(k) for k = 1..K-1, then backward x(k) = x(k) - gamma(k) x(k+1) for k = K-1..0; x(K) is read,
// never written.  The column goes through LDS to the first wavefront, which holds levels
// NL l .. NL l + NL-1 on lane l (NL = WIDE_THREADS / 64: 2 or 4) and runs thomas_column's lane sweep
// over them: every iteration each lane re-evaluates its NL updates in level order, the first from its
// neighbour's current value, so after ceil(K / NL) iterations each level holds what the sequential
// loop computes, from the same operands, bit for bit.
__device__ __forceinline__ double column_solve(double x, double a, double alpha, double gamma, int k, int K) {
  constexpr int NL = WIDE_THREADS / 64;
  __syncthreads();
  wide_lds[0][threadIdx.x] = x;
  wide_lds[1][threadIdx.x] = a;
  wide_lds[2][threadIdx.x] = alpha;
  wide_lds[3][threadIdx.x] = gamma;
  __syncthreads();
  if (threadIdx.x < 64) {
    double r[NL], aa[NL], al[NL], g[NL], xv[NL], xf[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int kj = NL * threadIdx.x + j;
      r[j] = wide_lds[0][kj];
      aa[j] = wide_lds[1][kj];
      al[j] = wide_lds[2][kj];
      g[j] = wide_lds[3][kj];
      xv[j] = r[j];
    }
    const int nit = (K + NL - 1) / NL;
    for (int it = 0; it < nit; ++it) {
      double prev = wave_shr1(xv[NL - 1]);  // level NL l - 1
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const int kj = NL * threadIdx.x + j;
        if (kj >= 1 && kj < K) xv[j] = (r[j] - aa[j] * prev) * al[j];
        prev = xv[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) xf[j] = xv[j];
    for (int it = 0; it < nit; ++it) {
      double next = wave_shl1(xv[0]);  // level NL (l + 1)
#pragma unroll
      for (int j = NL - 1; j >= 0; --j) {
        const int kj = NL * threadIdx.x + j;
        if (kj < K) xv[j] = xf[j] - g[j] * next;
        next = xv[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) wide_lds[0][NL * threadIdx.x + j] = xv[j];
  }
  __syncthreads();
  return wide_lds[0][k];
}
// the LU factors of the implicit w solve (2124-2127): alpha(k) = 1 / (b(k) - a(k) gamma(k-1)),
// gamma(k) = c(k) alpha(k) for k = 1..K-1; lane 0 keeps alpha = gamma = 0
__device__ __forceinline__ void column_lu(double a, double b, double c, int k, int K, double& alpha, double& gamma) {
  __syncthreads();
  wide_lds[0][threadIdx.x] = a;
  wide_lds[1][threadIdx.x] = b;
  wide_lds[2][threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    double g = 0.0;
    wide_lds[3][0] = 0.0;
    wide_lds[4][0] = 0.0;
    for (int kk = 1; kk < K; ++kk) {
      const double al = 1. / (wide_lds[1][kk] - wide_lds[0][kk] * g);
      g = wide_lds[2][kk] * al;
      wide_lds[3][kk] = al;
      wide_lds[4][kk] = g;
    }
  }
  __syncthreads();
  alpha = k < K ? wide_lds[3][k] : 0.0;
  gamma = k < K ? wide_lds[4][k] : 0.0;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  __syncthreads();
  wide_lds[0][threadIdx.x] = v;
  __syncthreads();
  return wide_lds[0][l];
}
#else
__device__ __forceinline__ double readlane_d(double v, int l) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
#endif

// the value of lane-1 (own at lane 0) and of lanes 0, 1, 2 (the bottom-boundary extrapolation of
// the w recovery, 3077-3078): one LDS round trip in the wide build instead of four
#ifdef MPAS_WIDE
__device__ __forceinline__ void up1_first3(double x, double& m, double& f0, double& f1, double& f2) {
  __syncthreads();
  wide_lds[0][threadIdx.x] = x;
  __syncthreads();
  m = threadIdx.x ? wide_lds[0][threadIdx.x - 1] : x;
  f0 = wide_lds[0][0];
  f1 = wide_lds[0][1];
  f2 = wide_lds[0][2];
}
#else
__device__ __forceinline__ void up1_first3(double x, double& m, double& f0, double& f1, double& f2) {
  m = up1(x);
  f0 = readlane_d(x, 0);
  f1 = readlane_d(x, 1);
  f2 = readlane_d(x, 2);
}
#endif

// Fortran sign(1.0_RKIND, x): IEEE copysign semantics
__device__ __forceinline__ double sgn1(double x) { return copysign(1.0, x); }

// statement functions flux4/flux3, mpas_atm_time_integration.F:3326-3331 (same trees at 3717, 4655)
__device__ __forceinline__ double flux4(double q_im2, double q_im1, double q_i, double q_ip1, double ua) {
  return ua * (7.0 * (q_i + q_im1) - (q_ip1 + q_im2)) / 12.0;
}
__device__ __forceinline__ double flux3(double q_im2, double q_im1, double q_i, double q_ip1, double ua, double coef3) {
  return flux4(q_im2, q_im1, q_i, q_ip1, ua) + coef3 * fabs(ua) * ((q_ip1 - q_im2) - 3.0 * (q_i - q_im1)) / 12.0;
}

#define LD(p, i) (act ? (p)[(i)] : 0.0)

// Physics tendencies (tend_ru_physics, tend_rtheta_physics, tend_rho_physics) are zeroed
// by atm_srk3 when the model is built without DO_PHYSICS (mpas_atm_time_integration.F:
// 268-279, 450-457): the kernels add the same +0.0 without streaming the zero arrays.
#define PHYS_ZERO 0.0
// With physics coupling on (mpas_dyc_set_physics, the reference built with DO_PHYSICS), the
// tendencies physics_get_tend computed (mpas_atm_time_integration.F:424-449) are added in the
// same places instead of the zeros of 450-457.
#define PHYS(arr, i) (d.physics ? (arr)[(i)] : 0.0)
#define LDW(p, i) (actw ? (p)[(i)] : 0.0)

// zb_p = zb_cell + zb3_cell, zb_m = zb_cell - zb3_cell.  The reference forms
// zb_cell + sign(1,flux) * zb3_cell (2299, 3085) with sign(1,flux) = +-1, whose product is exact,
// so the sum is one of these two doubles bit for bit.  The w-flux kernels then load only the one
// their flux sign selects: the sign is mostly uniform down a column, so a wave touches the cache
// lines of one array instead of both (8 B instead of 16 B per cell-edge-level).
__global__ void k_build_zb(int64_t n, const double* __restrict__ zb, const double* __restrict__ zb3,
                           double* __restrict__ zp, double* __restrict__ zm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    zp[i] = zb[i] + 1.0 * zb3[i];
    zm[i] = zb[i] + -1.0 * zb3[i];
  }
}

// Per-cell stencil records (dycore.h, Ptrs::cell_rec / cell_sdv), one thread per cell.  The
// cell across edge i is the other entry of cellsOnEdge, exactly the operand the reference
// loops pick with their cellsOnEdge(1/2,iEdge) tests.  cell_sdv = edgesOnCell_sign * dvEdge:
// the sign is +-1, so edgesOnCell_sign * x * dvEdge == x * cell_sdv bit for bit for any x.
__global__ void k_build_cell_rec(Dims d, const int* __restrict__ noc, const int* __restrict__ eoc,
                                 const int* __restrict__ coe, const double* __restrict__ dvEdge,
                                 const double* __restrict__ sign, int* rec, double* cdv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > d.nCells) return;
  const int ne = (c < d.nCells) ? noc[c] : 0;
  for (int i = 0; i < CELL_REC_ME; ++i) {
    int e = d.nEdges, o = d.nCells;
    if (i < ne && i < d.maxEdges) {
      e = eoc[(size_t)c * d.maxEdges + i];
      if (e >= 0 && e < d.nEdges) {
        const int c1 = coe[2 * e], c2 = coe[2 * e + 1];
        o = (c1 == c) ? c2 : c1;
      } else {
        e = d.nEdges;
      }
    }
    rec[(size_t)c * CELL_REC + i] = e;
    rec[(size_t)c * CELL_REC + CELL_REC_ME + i] = o;
    if (i < d.maxEdges)
      cdv[(size_t)c * d.maxEdges + i] = (i < ne) ? sign[(size_t)c * d.maxEdges + i] * dvEdge[e] : 0.0;
  }
  // bits 2i..2i+1: edgesOnCell_sign code (0: +1, 1: -1, 2: 0, mpas_atm_core.F:1041-1050);
  // bit 16+i: this cell is cellsOnEdge(1) of edge i
  int bits = 0;
  for (int i = 0; i < CELL_REC_ME && i < d.maxEdges; ++i) {
    if (i >= ne) continue;
    const double sg = sign[(size_t)c * d.maxEdges + i];
    bits |= (sg > 0.0 ? 0 : (sg < 0.0 ? 1 : 2)) << (2 * i);
    const int e = rec[(size_t)c * CELL_REC + i];
    if (e < d.nEdges && coe[2 * e] == c) bits |= 1 << (16 + i);
  }
  rec[(size_t)c * CELL_REC + 14] = ne;
  rec[(size_t)c * CELL_REC + 15] = bits;
}

// A cell's stencil from its record: one scalar round trip (see k_build_cell_rec).
template <int ME>
struct CellSten {
  int e[ME], o[ME];
  int ne, bits;
  // edgesOnCell_sign(i): exactly +1, -1 or 0, as atm_compute_signs stores it
  __device__ __forceinline__ double sg(int i) const {
    const int s = (bits >> (2 * i)) & 3;
    return s == 0 ? 1.0 : (s == 1 ? -1.0 : 0.0);
  }
  __device__ __forceinline__ bool first(int i) const { return (bits >> (16 + i)) & 1; }
};
template <int ME>
__device__ __forceinline__ CellSten<ME> load_sten(const Ptrs& p, int c) {
  CellSten<ME> s;
  const int* r = p.cell_rec + (size_t)c * CELL_REC;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    s.e[i] = r[i];
    s.o[i] = r[CELL_REC_ME + i];
  }
  s.ne = r[14];
  s.bits = r[15];
  return s;
}

// receive-buffer offset of field f of element i in a fused unpack (XUnpack), -1: not received
__device__ __forceinline__ int rec_off(const XUnpack& u, int f, int i, int nsolve) {
  return (u.recv && i >= nsolve && i - nsolve < u.nh) ? u.off[(size_t)f * u.nh + (i - nsolve)] : -1;
}

// ============================================================================
// atm_compute_moist_coefficients  (mpas_atm_time_integration.F:1899-1931)
// ============================================================================
__global__ __launch_bounds__(BLOCK_THREADS) void k_moist_cells(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  double q = 0.0;
  if (act) {
    for (int iq = d.moist_start; iq <= d.moist_end; ++iq) q = q + p.scalars2[SIX(c, k, iq)];
    p.qtot[(size_t)c * K + k] = q;
  }
  double qm = up1(q);
  if (act && k >= 1) {
    double qtotal = 0.5 * (q + qm);
    p.cqw[(size_t)c * K + k] = 1.0 / (1.0 + qtotal);
  }
}

__global__ __launch_bounds__(BLOCK_THREADS) void k_moist_edges(Dims d, Ptrs p) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  if (!(c1 < d.nCellsSolve || c2 < d.nCellsSolve)) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  double qtotal = 0.0;
  for (int iq = d.moist_start; iq <= d.moist_end; ++iq)
    qtotal = qtotal + 0.5 * (p.scalars2[SIX(c1, k, iq)] + p.scalars2[SIX(c2, k, iq)]);
  p.cqu[(size_t)e * K + k] = 1.0 / (1.0 + qtotal);
}

// ============================================================================
// atm_compute_vert_imp_coefs_work  (mpas_atm_time_integration.F:2064-2129)
// ============================================================================
__global__ __launch_bounds__(BLOCK_THREADS) void k_vert_imp_coefs(Dims d, Ptrs p, double dts, double epssm) {
  const int c = wave_elem(0);
  const int k = lane_id(), K = d.K;
  const double dtseps = .5 * dts * (1. + epssm);
  const double rcv = RGAS / (CP - RGAS);
  const double c2 = CP * rcv;
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)K) p.cofrz[threadIdx.x] = dtseps * p.rdzw[threadIdx.x];
  if (c >= d.nCellsSolve) return;
  const bool act = k < K;
  const size_t o = (size_t)c * K + k;
  const double zz = LD(p.zz, o), pp = LD(p.exner, o), t = LD(p.theta_m2, o);
  const double rb = LD(p.rho_base, o), rtb = LD(p.rtheta_base, o), pb = LD(p.exner_base, o);
  const double rt = LD(p.rtheta_p, o), cqw = LD(p.cqw, o), qtot = LD(p.qtot, o);
  const double fzm = act ? p.fzm[k] : 0.0, fzp = act ? p.fzp[k] : 0.0;
  const double rdzu = act ? p.rdzu[k] : 0.0, rdzw = act ? p.rdzw[k] : 0.0;
  const double zzm = up1(zz), pm = up1(pp), tm = up1(t);
  double cofwr = 0.0, cofwz = 0.0, coftz = 0.0;
  if (act && k >= 1) {
    cofwr = .5 * dtseps * GRAVITY * (fzm * zz + fzp * zzm);
    cofwz = dtseps * c2 * (fzm * zz + fzp * zzm) * rdzu * cqw * (fzm * pp + fzp * pm);
    coftz = dtseps * (fzm * t + fzp * tm);
  }
  double cofwt = 0.0;
  if (act) cofwt = .5 * dtseps * rcv * zz * GRAVITY * rb / (1. + qtot) * pp / ((rtb + rt) * pb);
  // k+1 / k-1 neighbours
  const double coftz_p = dn1(coftz), coftz_m = up1(coftz);
  const double cofwt_m = up1(cofwt), rdzw_m = up1(rdzw);
  const double cofrz = dtseps * rdzw, cofrz_m = up1(cofrz);
  double a = 0.0, b = 1.0, cc = 0.0;
  if (act && k >= 1) {
    a = -cofwz * coftz_m * rdzw_m * zzm + cofwr * cofrz_m - cofwt_m * coftz_m * rdzw_m;
    b = 1. + cofwz * (coftz * rdzw * zz + coftz * rdzw_m * zzm) - coftz * (cofwt * rdzw - cofwt_m * rdzw_m) +
        cofwr * (cofrz - cofrz_m);
    cc = -cofwz * coftz_p * rdzw * zz - cofwr * cofrz + cofwt * coftz_p * rdzw;
  }
  // sequential LU recurrence in the reference order (2124-2127)
  double alpha = 0.0, gamma = 0.0;
#ifdef MPAS_WIDE
  column_lu(a, b, cc, k, K, alpha, gamma);
#else
  for (int kk = 1; kk < K; ++kk) {
    const double gp = readlane_d(gamma, kk - 1);
    if (k == kk) {
      alpha = 1. / (b - a * gp);
      gamma = cc * alpha;
    }
  }
#endif
  if (act) {
    if (k >= 1) {
      p.cofwr[o] = cofwr;
      p.cofwz[o] = cofwz;
    }
    p.cofwt[o] = cofwt;
    p.a_tri[o] = a;
    p.alpha_tri[o] = alpha;
    p.gamma_tri[o] = gamma;
  }
  if (k <= K) p.coftz[(size_t)c * (K + 1) + k] = coftz;  // coftz(1) = coftz(K+1) = 0
}

// ============================================================================
// atm_compute_dyn_tend_work  (mpas_atm_time_integration.F:4663-5414)
// ============================================================================
struct DynTendScal {
  int rk_step;
  // tend_rtheta_adv / rthdynten (5350-5351) are read only by the physics, after the step: every
  // dyn_tend overwrites them, so only the last one of a dt stores them (store_phys_diag = 1)
  int store_phys_diag;
  double dt, invDt, h_mom_eddy_visc4, h_theta_eddy_visc4, coef_3rd_order, c_s;
  double rayleigh_coef_inverse;
};

// cells (all): 2d Smagorinsky kdiff + cam filter (rk1, 4677-4720); h_divergence (4729-4748);
// tend_rho and dpdz (rk1, 4755-4766)
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_cells1(Dims d, Ptrs p, Config cf, DynTendScal s) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t o = (size_t)c * K + k;
  const int ne = p.nEdgesOnCell[c];
  if (s.rk_step == 1 && act) {
    double kd;
    if (cf.horiz_mixing_smag) {
      double d_diag = 0.0, d_off = 0.0;
      for (int i = 0; i < ne; ++i) {
        const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
        const double a = p.defc_a[c * d.maxEdges + i], bb = p.defc_b[c * d.maxEdges + i];
        const double ue = p.u2[(size_t)e * K + k], ve = p.v[(size_t)e * K + k];
        d_diag = d_diag + a * ue - bb * ve;
        d_off = d_off + bb * ue + a * ve;
      }
      const double csl = s.c_s * cf.len_disp;
      kd = fmin((csl * csl) * sqrt(d_diag * d_diag + d_off * d_off), (0.01 * (cf.len_disp * cf.len_disp)) * s.invDt);
    } else {
      kd = cf.h_theta_eddy_visc2;
    }
    if (cf.mpas_cam_coef > 0.0) {
      if (k == K - 3) kd = fmax(kd, 2.0833 * cf.len_disp * cf.mpas_cam_coef);
      if (k == K - 2) kd = fmax(kd, 2.0 * 2.0833 * cf.len_disp * cf.mpas_cam_coef);
      if (k == K - 1) kd = fmax(kd, 4.0 * 2.0833 * cf.len_disp * cf.mpas_cam_coef);
    }
    p.kdiff[o] = kd;
  }
  double hd = 0.0;
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double edge_sign = p.edgesOnCell_sign[c * d.maxEdges + i] * p.dvEdge[e];
    hd = hd + edge_sign * LD(p.ru, (size_t)e * K + k);
  }
  hd = hd * p.invAreaCell[c];
  if (act) p.h_divergence[o] = hd;
  if (s.rk_step == 1) {
    const size_t ow = (size_t)c * (K + 1) + k;
    const double rwk = (k <= K) ? p.rw[ow] : 0.0;
    const double rwp = dn1(rwk);
    if (act) {
      p.tend_rho[o] = -hd - p.rdzw[k] * (rwp - rwk) + PHYS(p.tend_rho_physics, o);
      const double qt = p.qtot[o];
      p.dpdz[o] = -GRAVITY * (p.rho_base[o] * (qt) + p.rho_p_save[o] * (1. + qt));
    }
  }
}

template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_cells1_b(Dims d, Ptrs p, Config cf, DynTendScal s) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t o = (size_t)c * K + kc;
  const bool rk1 = s.rk_step == 1, smag = rk1 && cf.horiz_mixing_smag;
  const CellSten<ME> st = load_sten<ME>(p, c);
  double sdv[ME], da[ME], db[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    sdv[i] = ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i);
    da[i] = smag ? ld_uniform_f64(p.defc_a + (size_t)c * ME + i) : 0.0;
    db[i] = smag ? ld_uniform_f64(p.defc_b + (size_t)c * ME + i) : 0.0;
  }
  const double invA = ld_uniform_f64(p.invAreaCell + c);
  double rwk = 0.0, qt = 0.0, rb = 0.0, rps = 0.0;
  if (rk1) {
    rwk = p.rw[(size_t)c * (K + 1) + kw];
    qt = p.qtot[o];
    rb = p.rho_base[o];
    rps = p.rho_p_save[o];
  }
  double rue[ME], ue[ME], ve[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const size_t oe = (size_t)uni(st.e[i]) * K + kc;
    rue[i] = p.ru[oe];
    ue[i] = smag ? p.u2[oe] : 0.0;
    ve[i] = smag ? p.v[oe] : 0.0;
  }
  // 2d Smagorinsky kdiff + cam filter (rk1, 4677-4720)
  if (rk1 && act) {
    double kd;
    if (smag) {
      double d_diag = 0.0, d_off = 0.0;
#pragma unroll
      for (int i = 0; i < ME; ++i) {
        if (i < st.ne) {
          d_diag = d_diag + da[i] * ue[i] - db[i] * ve[i];
          d_off = d_off + db[i] * ue[i] + da[i] * ve[i];
        }
      }
      const double csl = s.c_s * cf.len_disp;
      kd = fmin((csl * csl) * sqrt(d_diag * d_diag + d_off * d_off), (0.01 * (cf.len_disp * cf.len_disp)) * s.invDt);
    } else {
      kd = cf.h_theta_eddy_visc2;
    }
    if (cf.mpas_cam_coef > 0.0) {
      if (k == K - 3) kd = fmax(kd, 2.0833 * cf.len_disp * cf.mpas_cam_coef);
      if (k == K - 2) kd = fmax(kd, 2.0 * 2.0833 * cf.len_disp * cf.mpas_cam_coef);
      if (k == K - 1) kd = fmax(kd, 4.0 * 2.0833 * cf.len_disp * cf.mpas_cam_coef);
    }
    p.kdiff[o] = kd;
  }
  // h_divergence (4729-4748)
  double hd = 0.0;
#pragma unroll
  for (int i = 0; i < ME; ++i)
    if (i < st.ne) hd = hd + sdv[i] * rue[i];  // edgesOnCell_sign * dvEdge * ru
  hd = hd * invA;
  if (act) p.h_divergence[o] = hd;
  // tend_rho and dpdz (rk1, 4755-4766)
  if (rk1) {
    const double rwp = dn1(rwk);
    if (act) {
      p.tend_rho[o] = -hd - p.rdzw[k] * (rwp - rwk) + PHYS(p.tend_rho_physics, o);
      p.dpdz[o] = -GRAVITY * (rb * (qt) + rps * (1. + qt));
    }
  }
}

// edges: tend_u (edge-solve: PGF rk1 4781-4788, vertical transport 4792-4807, Coriolis/KE 4811-4838)
// + rk1 del2 on all edges (4856-4883); finalize (Rayleigh + euler + physics, 5015-5036) when rk>1.
// Like k_dyn_advflux this is latency bound: every column the edge reads is loaded before the
// first use (RK1 adds the PGF and del2 operands), then the reference expressions are evaluated.
template <bool RK1>
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_edges(Dims d, Ptrs p, Config cf, DynTendScal s, int finalize) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)e * K + k;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  const size_t o1 = (size_t)c1 * K + k, o2 = (size_t)c2 * K + k;
  const bool solve = e < d.nEdgesSolve;
  const int neoe = solve ? p.nEdgesOnEdge[e] : 0;
  const bool hex = neoe == 10;  // hexagon-hexagon edge: the 20 TRiSK gathers go out together
  // ---- loads
  const double uk = LD(p.u2, o);
  double tue = (act && !(RK1 && solve)) ? p.tend_u_euler[o] : 0.0;  // rk1 recomputes it on solve edges
  double rw1 = 0.0, rw2 = 0.0, pve = 0.0, re = 0.0, ke1 = 0.0, ke2 = 0.0, hd1 = 0.0, hd2 = 0.0;
  double pv[10], uu[10];
  if (solve && k <= K) {
    rw1 = p.rw[(size_t)c1 * K1 + k];
    rw2 = p.rw[(size_t)c2 * K1 + k];
  }
  if (act && (solve || RK1)) re = p.rho_edge[o];
  if (solve && act) {
    pve = p.pv_edge[o];
    if (hex) {
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int eoe = uni(p.edgesOnEdge[e * d.maxEdges2 + j]);
        pv[j] = p.pv_edge[(size_t)eoe * K + k];
        uu[j] = p.u2[(size_t)eoe * K + k];
      }
    }
    ke1 = p.ke[o1];
    ke2 = p.ke[o2];
    hd1 = p.h_divergence[o1];
    hd2 = p.h_divergence[o2];
  }
  double cqu = 0.0, pp1 = 0.0, pp2 = 0.0, zz1 = 0.0, zz2 = 0.0, zxu = 0.0, dpz1 = 0.0, dpz2 = 0.0;
  double dv1 = 0.0, dv2 = 0.0, vo1 = 0.0, vo2 = 0.0, kd1 = 0.0, kd2 = 0.0;
  if (RK1 && act) {
    if (solve) {
      cqu = p.cqu[o];
      pp1 = p.pressure_p[o1];
      pp2 = p.pressure_p[o2];
      zz1 = p.zz[o1];
      zz2 = p.zz[o2];
      zxu = p.zxu[o];
      dpz1 = p.dpdz[o1];
      dpz2 = p.dpdz[o2];
    }
    const int v1 = p.verticesOnEdge[2 * e], v2 = p.verticesOnEdge[2 * e + 1];
    dv1 = p.divergence[o1];
    dv2 = p.divergence[o2];
    vo1 = p.vorticity[(size_t)v1 * K + k];
    vo2 = p.vorticity[(size_t)v2 * K + k];
    kd1 = p.kdiff[o1];
    kd2 = p.kdiff[o2];
  }
  // ---- tend_u
  if (solve) {
    if (RK1 && act)
      tue = -cqu * ((pp2 - pp1) * p.invDcEdge[e] / (.5 * (zz2 + zz1)) - 0.5 * zxu * (dpz1 + dpz2));
    // vertical transport of u: wduz(k), k = 1..K+1 on lanes 0..K
    const double um1 = up1(uk), um2 = up2(uk), up1v = dn1(uk);
    const double rwa = (k <= K) ? 0.5 * (rw1 + rw2) : 0.0;
    double wduz = 0.0;
    if (k == 1 || k == K - 1) {
      wduz = 0.5 * (rw1 + rw2) * (p.fzm[k] * uk + p.fzp[k] * um1);
    } else if (k >= 2 && k <= K - 2) {
      wduz = flux3(um2, um1, uk, up1v, rwa, 1.0);
    }
    const double wduz_p = dn1(wduz);
    double tu = act ? -p.rdzw[k] * (wduz_p - wduz) : 0.0;
    // nonlinear Coriolis term (Ringler et al. 2009)
    double q = 0.0;
    if (hex && act) {
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const double workpv = 0.5 * (pve + pv[j]);
        q = q + p.weightsOnEdge[e * d.maxEdges2 + j] * uu[j] * workpv;
      }
    } else {
      for (int j = 0; j < neoe; ++j) {
        const int eoe = uni(p.edgesOnEdge[e * d.maxEdges2 + j]);
        const double workpv = 0.5 * (pve + LD(p.pv_edge, (size_t)eoe * K + k));
        q = q + p.weightsOnEdge[e * d.maxEdges2 + j] * LD(p.u2, (size_t)eoe * K + k) * workpv;
      }
    }
    if (act) tu = tu + re * (q - (ke2 - ke1) * p.invDcEdge[e]) - uk * 0.5 * (hd1 + hd2);
    if (finalize && act) {
      if (cf.rayleigh_damp_u && k >= K - cf.number_rayleigh_damp_u_levels) {
        const double coef = (double)(k + 1 - (K - cf.number_rayleigh_damp_u_levels)) * s.rayleigh_coef_inverse;
        tu = tu - re * uk * coef;
      }
      tu = tu + tue + PHYS(p.tend_ru_physics, o);
    }
    if (act) p.tend_u[o] = tu;
  }
  if (RK1 && act) {
    // del^2 part of the del^4 filter, all edges (4858-4883)
    const double r_dc = p.invDcEdge[e];
    const double r_dv = fmin(p.invDvEdge[e], 4 * p.invDcEdge[e]);
    const double u_diffusion = (dv2 - dv1) * r_dc - (vo2 - vo1) * r_dv;
    p.delsq_u[o] = 0.0 + u_diffusion;
    const double kdiffu = 0.5 * (kd1 + kd2);
    tue = tue + re * kdiffu * u_diffusion * p.meshScalingDel2[e];
    p.tend_u_euler[o] = tue;
  }
}

// k_dyn_edges with batched loads (NE2 = 2*maxEdges-2 >= nEdgesOnEdge): the edge's metadata
// (cellsOnEdge, verticesOnEdge, edgesOnEdge, weightsOnEdge) and own columns go out first, then
// every gather at once, so a wave waits for two memory round trips.  Same expressions and order
// as k_dyn_edges; solve edges (tend_u and, at rk1, del2) and halo edges (rk1 del2 only) are
// separate paths so that neither issues the other's loads.
template <bool RK1, int NE2>
__global__ __launch_bounds__(EDGE_THREADS) void k_dyn_edges_b(Dims d, Ptrs p, Config cf, DynTendScal s,
                                                               int finalize) {
  const int e = wave_elem_e();
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)e * K + kc;
  const bool solve = e < d.nEdgesSolve;
  const int2 ce = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * e);
  const double invDc = ld_uniform_f64(p.invDcEdge + e);
  const double re = p.rho_edge[o];
  // rk1 del^2 of u (4856-4883), all edges
  auto del2 = [&](double tue, double dv1, double dv2, double vo1, double vo2, double kd1, double kd2, double invDv,
                  double msd2) {
    const double r_dc = invDc;
    const double r_dv = fmin(invDv, 4 * invDc);
    const double u_diffusion = (dv2 - dv1) * r_dc - (vo2 - vo1) * r_dv;
    if (act) p.delsq_u[o] = 0.0 + u_diffusion;
    const double kdiffu = 0.5 * (kd1 + kd2);
    tue = tue + re * kdiffu * u_diffusion * msd2;
    if (act) p.tend_u_euler[o] = tue;
  };
  if (!solve) {
    if (!RK1) return;
    const int2 ve = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * e);
    const double invDv = ld_uniform_f64(p.invDvEdge + e), msd2 = ld_uniform_f64(p.meshScalingDel2 + e);
    const double tue = p.tend_u_euler[o];
    const int c1 = uni(ce.x), c2 = uni(ce.y), v1 = uni(ve.x), v2 = uni(ve.y);
    const size_t o1 = (size_t)c1 * K + kc, o2 = (size_t)c2 * K + kc;
    del2(tue, p.divergence[o1], p.divergence[o2], p.vorticity[(size_t)v1 * K + kc],
         p.vorticity[(size_t)v2 * K + kc], p.kdiff[o1], p.kdiff[o2], invDv, msd2);
    return;
  }
  // ---- solve edges: batch 1
  const int neoe = p.nEdgesOnEdge[e];
  int eoe[NE2];
  double wgt[NE2];
#pragma unroll
  for (int j = 0; j < NE2; ++j) {
    eoe[j] = p.edgesOnEdge[(size_t)e * d.maxEdges2 + j];
    wgt[j] = ld_uniform_f64(p.weightsOnEdge + (size_t)e * d.maxEdges2 + j);
  }
  int2 ve = make_int2(0, 0);
  double invDv = 0.0, msd2 = 0.0, cqu = 0.0, zxu = 0.0;
  if (RK1) {
    ve = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * e);
    invDv = ld_uniform_f64(p.invDvEdge + e);
    msd2 = ld_uniform_f64(p.meshScalingDel2 + e);
    cqu = p.cqu[o];
    zxu = p.zxu[o];
  }
  const double uk = p.u2[o], pve = p.pv_edge[o];
  double tue = RK1 ? 0.0 : p.tend_u_euler[o];  // rk1 recomputes it on solve edges
  // ---- batch 2: gathers
  const int c1 = uni(ce.x), c2 = uni(ce.y);
  const size_t o1 = (size_t)c1 * K + kc, o2 = (size_t)c2 * K + kc;
  const double rw1 = p.rw[(size_t)c1 * K1 + kw], rw2 = p.rw[(size_t)c2 * K1 + kw];
  const double ke1 = p.ke[o1], ke2 = p.ke[o2], hd1 = p.h_divergence[o1], hd2 = p.h_divergence[o2];
  double pv[NE2], uu[NE2];
#pragma unroll
  for (int j = 0; j < NE2; ++j) {
    const size_t oj = (size_t)uni(eoe[j]) * K + kc;
    pv[j] = p.pv_edge[oj];
    uu[j] = p.u2[oj];
  }
  double pp1 = 0.0, pp2 = 0.0, zz1 = 0.0, zz2 = 0.0, dpz1 = 0.0, dpz2 = 0.0;
  double dv1 = 0.0, dv2 = 0.0, vo1 = 0.0, vo2 = 0.0, kd1 = 0.0, kd2 = 0.0;
  if (RK1) {
    const int v1 = uni(ve.x), v2 = uni(ve.y);
    pp1 = p.pressure_p[o1];
    pp2 = p.pressure_p[o2];
    zz1 = p.zz[o1];
    zz2 = p.zz[o2];
    dpz1 = p.dpdz[o1];
    dpz2 = p.dpdz[o2];
    dv1 = p.divergence[o1];
    dv2 = p.divergence[o2];
    vo1 = p.vorticity[(size_t)v1 * K + kc];
    vo2 = p.vorticity[(size_t)v2 * K + kc];
    kd1 = p.kdiff[o1];
    kd2 = p.kdiff[o2];
  }
  const double fzm = p.fzm[kc], fzp = p.fzp[kc], rdzw = p.rdzw[kc];
  // ---- tend_u (PGF rk1 4781-4788, vertical transport 4792-4807, Coriolis/KE 4811-4838)
  if (RK1) tue = -cqu * ((pp2 - pp1) * invDc / (.5 * (zz2 + zz1)) - 0.5 * zxu * (dpz1 + dpz2));
  const double um1 = up1(uk), um2 = up2(uk), up1v = dn1(uk);
  const double rwa = 0.5 * (rw1 + rw2);
  double wduz = 0.0;
  if (k == 1 || k == K - 1) {
    wduz = 0.5 * (rw1 + rw2) * (fzm * uk + fzp * um1);
  } else if (k >= 2 && k <= K - 2) {
    wduz = flux3(um2, um1, uk, up1v, rwa, 1.0);
  }
  const double wduz_p = dn1(wduz);
  double tu = -rdzw * (wduz_p - wduz);
  double q = 0.0;
#pragma unroll
  for (int j = 0; j < NE2; ++j) {
    if (j < neoe) {
      const double workpv = 0.5 * (pve + pv[j]);
      q = q + wgt[j] * uu[j] * workpv;
    }
  }
  tu = tu + re * (q - (ke2 - ke1) * invDc) - uk * 0.5 * (hd1 + hd2);
  if (finalize) {
    if (cf.rayleigh_damp_u && k >= K - cf.number_rayleigh_damp_u_levels) {
      const double coef = (double)(k + 1 - (K - cf.number_rayleigh_damp_u_levels)) * s.rayleigh_coef_inverse;
      tu = tu - re * uk * coef;
    }
    tu = tu + tue + PHYS(p.tend_ru_physics, o);
  }
  if (act) p.tend_u[o] = tu;
  if (RK1) del2(tue, dv1, dv2, vo1, vo2, kd1, kd2, invDv, msd2);
}

// vertices: delsq_vorticity (4889-4898); cells: delsq_divergence (4900-4910)   [rk1, visc4>0]
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_delsq_vc(Dims d, Ptrs p) {
  const int idx = wave_elem(0);
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  if (idx < d.nVertices) {
    const int v = idx;
    double dv = 0.0;
    for (int i = 0; i < 3; ++i) {
      const int e = uni(p.edgesOnVertex[3 * v + i]);
      const double edge_sign = p.invAreaTriangle[v] * p.dcEdge[e] * p.edgesOnVertex_sign[3 * v + i];
      dv = dv + edge_sign * LD(p.delsq_u, (size_t)e * K + k);
    }
    if (act) p.delsq_vorticity[(size_t)v * K + k] = dv;
  } else {
    const int c = idx - d.nVertices;
    if (c >= d.nCells) return;
    double dd = 0.0;
    const double r = p.invAreaCell[c];
    const int ne = p.nEdgesOnCell[c];
    for (int i = 0; i < ne; ++i) {
      const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
      const double edge_sign = r * p.dvEdge[e] * p.edgesOnCell_sign[c * d.maxEdges + i];
      dd = dd + edge_sign * LD(p.delsq_u, (size_t)e * K + k);
    }
    if (act) p.delsq_divergence[(size_t)c * K + k] = dd;
  }
}

// edge-solve, rk1: del^4 (4917-4942), vertical mixing of u (4949-5006), then finalize (5015-5036)
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_edges_rk1b(Dims d, Ptrs p, Config cf, DynTendScal s) {
  const int e = wave_elem(0);
  if (e >= d.nEdgesSolve) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t o = (size_t)e * K + k;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  double tue = LD(p.tend_u_euler, o);
  const double uk = LD(p.u2, o);
  if (s.h_mom_eddy_visc4 > 0.0 && act) {
    const int v1 = p.verticesOnEdge[2 * e], v2 = p.verticesOnEdge[2 * e + 1];
    const double u_mix_scale = p.meshScalingDel4[e] * s.h_mom_eddy_visc4;
    const double r_dc = u_mix_scale * cf.del4u_div_factor * p.invDcEdge[e];
    const double r_dv = u_mix_scale * fmin(p.invDvEdge[e], 4 * p.invDcEdge[e]);
    const double u_diffusion =
        p.rho_edge[o] * ((p.delsq_divergence[(size_t)c2 * K + k] - p.delsq_divergence[(size_t)c1 * K + k]) * r_dc -
                         (p.delsq_vorticity[(size_t)v2 * K + k] - p.delsq_vorticity[(size_t)v1 * K + k]) * r_dv);
    tue = tue - u_diffusion;
  }
  if (cf.v_mom_eddy_visc2 > 0.0) {
    // lanes 1..K-2 (Fortran k = 2..K-1)
    double um = up1(uk), upv = dn1(uk);
    double mixm = 0.0, mix0 = 0.0, mixp = 0.0;
    if (!cf.mix_full) {
      const double ca = cos(p.angleEdge[e]), sa = sin(p.angleEdge[e]);
      mix0 = act ? uk - p.u_init[k] * ca - p.v_init[k] * sa : 0.0;
      mixm = up1(mix0);
      mixp = dn1(mix0);
    }
    if (k >= 1 && k <= K - 2) {
      const size_t K1 = K + 1;
      const double z1 = 0.5 * (p.zgrid[c1 * K1 + k - 1] + p.zgrid[c2 * K1 + k - 1]);
      const double z2 = 0.5 * (p.zgrid[c1 * K1 + k] + p.zgrid[c2 * K1 + k]);
      const double z3 = 0.5 * (p.zgrid[c1 * K1 + k + 1] + p.zgrid[c2 * K1 + k + 1]);
      const double z4 = 0.5 * (p.zgrid[c1 * K1 + k + 2] + p.zgrid[c2 * K1 + k + 2]);
      const double zm = 0.5 * (z1 + z2), z0 = 0.5 * (z2 + z3), zp = 0.5 * (z3 + z4);
      if (cf.mix_full)
        tue = tue + p.rho_edge[o] * cf.v_mom_eddy_visc2 * ((upv - uk) / (zp - z0) - (uk - um) / (z0 - zm)) / (0.5 * (zp - zm));
      else
        tue = tue + p.rho_edge[o] * cf.v_mom_eddy_visc2 * ((mixp - mix0) / (zp - z0) - (mix0 - mixm) / (z0 - zm)) / (0.5 * (zp - zm));
    }
  }
  if (!act) return;
  p.tend_u_euler[o] = tue;
  double tu = p.tend_u[o];
  if (cf.rayleigh_damp_u && k >= K - cf.number_rayleigh_damp_u_levels) {
    const double coef = (double)(k + 1 - (K - cf.number_rayleigh_damp_u_levels)) * s.rayleigh_coef_inverse;
    tu = tu - p.rho_edge[o] * uk * coef;
  }
  p.tend_u[o] = tu + tue + PHYS(p.tend_ru_physics, o);
}

// cells (all), rk1: del^2 for w (5107-5130) and theta (5278-5301)
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_cells2(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const double r_areaCell = p.invAreaCell[c];
  const int ne = p.nEdgesOnCell[c];
  double dw = 0.0, tw = 0.0, dth = 0.0, tth = 0.0;
  const double prandtl_inv = 1.0 / PRANDTL;
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
    const double sg = p.edgesOnCell_sign[c * d.maxEdges + i];
    const double re = LD(p.rho_edge, (size_t)e * K + k);
    const double re_m = up1(re);
    const double kd1 = LD(p.kdiff, (size_t)c1 * K + k), kd2 = LD(p.kdiff, (size_t)c2 * K + k);
    const double kd1m = up1(kd1), kd2m = up1(kd2);
    if (act && k >= 1) {
      const double edge_sign = 0.5 * r_areaCell * sg * p.dvEdge[e] * p.invDcEdge[e];
      double w_turb_flux = edge_sign * (re + re_m) * (p.w2[(size_t)c2 * (K + 1) + k] - p.w2[(size_t)c1 * (K + 1) + k]);
      dw = dw + w_turb_flux;
      w_turb_flux = w_turb_flux * p.meshScalingDel2[e] * 0.25 * (kd1 + kd2 + kd1m + kd2m);
      tw = tw + w_turb_flux;
    }
    if (act) {
      const double edge_sign = r_areaCell * sg * p.dvEdge[e] * p.invDcEdge[e];
      const double pr_scale = prandtl_inv * p.meshScalingDel2[e];
      double ttf = edge_sign * (p.theta_m2[(size_t)c2 * K + k] - p.theta_m2[(size_t)c1 * K + k]) * re;
      dth = dth + ttf;
      ttf = ttf * 0.5 * (kd1 + kd2) * pr_scale;
      tth = tth + ttf;
    }
  }
  if (act) {
    p.delsq_w[(size_t)c * K + k] = dw;
    p.delsq_theta[(size_t)c * K + k] = dth;
    p.tend_theta_euler[(size_t)c * K + k] = tth;
  }
  if (k <= K) p.tend_w_euler[(size_t)c * (K + 1) + k] = (act && k >= 1) ? tw : 0.0;
}

// Vertices and cells interleaved, two vertices then one cell per three waves: vertex 2j, 2j+1 and cell
// j lie at the same place of the space-filling curve (vertices are numbered in cell order, nVertices
// ~ 2 nCells), so one XCD's slab of waves reads delsq_u of one region once for both halves instead of
// the vertex and cell halves each streaming all of delsq_u through different L2s.  Launch
// 3 * max(ceil(nVertices / 2), nCells) waves.
template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_delsq_vc_b(Dims d, Ptrs p) {
  const int idx = wave_elem(0);
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const int j3 = idx / 3, t3 = idx - 3 * j3;
  if (t3 < 2) {
    const int v = 2 * j3 + t3;
    if (v >= d.nVertices) return;
    int ei[3];
    double sg[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ei[i] = p.edgesOnVertex[3 * v + i];
      sg[i] = ld_uniform_f64(p.edgesOnVertex_sign + 3 * v + i);
    }
    const double iat = ld_uniform_f64(p.invAreaTriangle + v);
    double dc[3], du[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = uni(ei[i]);
      dc[i] = ld_uniform_f64(p.dcEdge + e);
      du[i] = p.delsq_u[(size_t)e * K + k];
    }
    double dv = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) dv = dv + (iat * dc[i] * sg[i]) * du[i];
    p.delsq_vorticity[(size_t)v * K + k] = dv;
  } else {
    const int c = j3;
    if (c >= d.nCells) return;
    const CellSten<ME> st = load_sten<ME>(p, c);
    double sdv[ME], du[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) sdv[i] = ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i);
    const double r = ld_uniform_f64(p.invAreaCell + c);
#pragma unroll
    for (int i = 0; i < ME; ++i) du[i] = p.delsq_u[(size_t)uni(st.e[i]) * K + k];
    double dd = 0.0;
#pragma unroll
    for (int i = 0; i < ME; ++i)
      if (i < st.ne) dd = dd + (r * sdv[i]) * du[i];  // r * dvEdge * edgesOnCell_sign
    p.delsq_divergence[(size_t)c * K + k] = dd;
  }
}

// tp: the final tend_u also goes to the 642 exchange's send buffer (XPack), or nothing
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_edges_rk1b_b(Dims d, Ptrs p, Config cf, DynTendScal s,
                                                                    XPack tp = XPack{}) {
  const int e = wave_elem(0);
  if (e >= d.nEdgesSolve) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const int kc = min(k, K - 1);
  const size_t K1 = K + 1;
  const size_t o = (size_t)e * K + kc;
  const int2 ce = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * e);
  const int2 ve = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * e);
  const bool del4 = s.h_mom_eddy_visc4 > 0.0, vmix = cf.v_mom_eddy_visc2 > 0.0;
  const double msd4 = ld_uniform_f64(p.meshScalingDel4 + e), invDc = ld_uniform_f64(p.invDcEdge + e);
  const double invDv = ld_uniform_f64(p.invDvEdge + e);
  const double ang = (vmix && !cf.mix_full) ? ld_uniform_f64(p.angleEdge + e) : 0.0;
  double tue = p.tend_u_euler[o];
  const double uk = p.u2[o], re = p.rho_edge[o], tu0 = p.tend_u[o];
  const int c1 = uni(ce.x), c2 = uni(ce.y), v1 = uni(ve.x), v2 = uni(ve.y);
  double dd1 = 0.0, dd2 = 0.0, dv1 = 0.0, dv2 = 0.0;
  if (del4) {
    dd1 = p.delsq_divergence[(size_t)c1 * K + kc];
    dd2 = p.delsq_divergence[(size_t)c2 * K + kc];
    dv1 = p.delsq_vorticity[(size_t)v1 * K + kc];
    dv2 = p.delsq_vorticity[(size_t)v2 * K + kc];
  }
  // zgrid levels k-1 .. k+2 of both cells, lanes 1..K-2 (Fortran k = 2..K-1)
  const int kz = max(1, min(k, K - 2));
  double zg1[4], zg2[4];
  if (vmix) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      zg1[j] = p.zgrid[(size_t)c1 * K1 + kz - 1 + j];
      zg2[j] = p.zgrid[(size_t)c2 * K1 + kz - 1 + j];
    }
  }
  if (del4 && act) {
    const double u_mix_scale = msd4 * s.h_mom_eddy_visc4;
    const double r_dc = u_mix_scale * cf.del4u_div_factor * invDc;
    const double r_dv = u_mix_scale * fmin(invDv, 4 * invDc);
    const double u_diffusion = re * ((dd2 - dd1) * r_dc - (dv2 - dv1) * r_dv);
    tue = tue - u_diffusion;
  }
  if (vmix) {
    const double um = up1(uk), upv = dn1(uk);
    double mixm = 0.0, mix0 = 0.0, mixp = 0.0;
    if (!cf.mix_full) {
      const double ca = cos(ang), sa = sin(ang);
      mix0 = act ? uk - p.u_init[kc] * ca - p.v_init[kc] * sa : 0.0;
      mixm = up1(mix0);
      mixp = dn1(mix0);
    }
    if (k >= 1 && k <= K - 2) {
      const double z1 = 0.5 * (zg1[0] + zg2[0]);
      const double z2 = 0.5 * (zg1[1] + zg2[1]);
      const double z3 = 0.5 * (zg1[2] + zg2[2]);
      const double z4 = 0.5 * (zg1[3] + zg2[3]);
      const double zm = 0.5 * (z1 + z2), z0 = 0.5 * (z2 + z3), zp = 0.5 * (z3 + z4);
      if (cf.mix_full)
        tue = tue + re * cf.v_mom_eddy_visc2 * ((upv - uk) / (zp - z0) - (uk - um) / (z0 - zm)) / (0.5 * (zp - zm));
      else
        tue = tue + re * cf.v_mom_eddy_visc2 * ((mixp - mix0) / (zp - z0) - (mix0 - mixm) / (z0 - zm)) / (0.5 * (zp - zm));
    }
  }
  if (!act) return;
  p.tend_u_euler[o] = tue;
  double tu = tu0;
  if (cf.rayleigh_damp_u && k >= K - cf.number_rayleigh_damp_u_levels) {
    const double coef = (double)(k + 1 - (K - cf.number_rayleigh_damp_u_levels)) * s.rayleigh_coef_inverse;
    tu = tu - re * uk * coef;
  }
  const double tuf = tu + tue + PHYS(p.tend_ru_physics, o);
  p.tend_u[o] = tuf;
  if (tp.start) {
    const int s0 = __builtin_amdgcn_readfirstlane(tp.start[e]), s1 = __builtin_amdgcn_readfirstlane(tp.start[e + 1]);
    for (int sl = s0; sl < s1; ++sl) tp.dst[sl][k] = tuf;
  }
}

template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_cells2_b(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const int kc = min(k, K - 1);
  const size_t K1 = K + 1;
  const CellSten<ME> st = load_sten<ME>(p, c);
  double sdv[ME], idc[ME], msd2[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) sdv[i] = ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i);
  const double r_areaCell = ld_uniform_f64(p.invAreaCell + c);
  const double kds = p.kdiff[(size_t)c * K + kc], ws = p.w2[(size_t)c * K1 + kc], ths = p.theta_m2[(size_t)c * K + kc];
  double re[ME], kdo[ME], wo[ME], tho[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const int e = uni(st.e[i]), co = uni(st.o[i]);
    idc[i] = ld_uniform_f64(p.invDcEdge + e);
    msd2[i] = ld_uniform_f64(p.meshScalingDel2 + e);
    re[i] = p.rho_edge[(size_t)e * K + kc];
    kdo[i] = p.kdiff[(size_t)co * K + kc];
    wo[i] = p.w2[(size_t)co * K1 + kc];
    tho[i] = p.theta_m2[(size_t)co * K + kc];
  }
  double dw = 0.0, tw = 0.0, dth = 0.0, tth = 0.0;
  const double prandtl_inv = 1.0 / PRANDTL;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    // cellsOnEdge(1/2) of edge i: this cell and the one across, in the edge's order
    const bool f = st.first(i);
    const double kd1 = f ? kds : kdo[i], kd2 = f ? kdo[i] : kds;
    const double w1 = f ? ws : wo[i], w2 = f ? wo[i] : ws;
    const double t1 = f ? ths : tho[i], t2 = f ? tho[i] : ths;
    const double re_m = up1(re[i]);
    const double kd1m = up1(kd1), kd2m = up1(kd2);
    if (i < st.ne) {
      if (act && k >= 1) {
        const double edge_sign = 0.5 * r_areaCell * sdv[i] * idc[i];  // 0.5*r_areaCell*sign*dvEdge*invDcEdge
        double w_turb_flux = edge_sign * (re[i] + re_m) * (w2 - w1);
        dw = dw + w_turb_flux;
        w_turb_flux = w_turb_flux * msd2[i] * 0.25 * (kd1 + kd2 + kd1m + kd2m);
        tw = tw + w_turb_flux;
      }
      if (act) {
        const double edge_sign = r_areaCell * sdv[i] * idc[i];
        const double pr_scale = prandtl_inv * msd2[i];
        double ttf = edge_sign * (t2 - t1) * re[i];
        dth = dth + ttf;
        ttf = ttf * 0.5 * (kd1 + kd2) * pr_scale;
        tth = tth + ttf;
      }
    }
  }
  if (act) {
    p.delsq_w[(size_t)c * K + k] = dw;
    p.delsq_theta[(size_t)c * K + k] = dth;
    p.tend_theta_euler[(size_t)c * K + k] = tth;
  }
  if (k <= K) p.tend_w_euler[(size_t)c * K1 + k] = (act && k >= 1) ? tw : 0.0;
}

// edges of owned cells: the 3rd/4th-order edge values of w and theta_m used by the
// horizontal advection in atm_compute_dyn_tend_work (flux_arr at 5056-5066 and 5236-5244).
// The reference recomputes them inside the cell loop for both cells of an edge; here each
// edge is evaluated once (same expression, same order) and the cell kernel reads it back.
// Latency, not bandwidth, bounds these gathers (one wave per edge, 20 neighbour columns
// mostly from L2): every load the edge needs is issued before the first wait, index loads
// first, then the 20 gathers, then the edge's own ru, so one memory round trip covers them.
template <int NA>
__device__ __forceinline__ void adv_edge_sums(const Ptrs& p, int e, int K, int k, size_t o, bool act, double& fw,
                                              double& ft) {
  const size_t K1 = K + 1;
  int ic[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) ic[j] = uni(p.advCellsForEdge[e * 15 + j]);
  double wv[NA], tv[NA];
  if (k <= K) {
#pragma unroll
    for (int j = 0; j < NA; ++j) wv[j] = p.w2[(size_t)ic[j] * K1 + k];
  } else {
#pragma unroll
    for (int j = 0; j < NA; ++j) wv[j] = 0.0;
  }
  if (act) {
#pragma unroll
    for (int j = 0; j < NA; ++j) tv[j] = p.theta_m2[(size_t)ic[j] * K + k];
  } else {
#pragma unroll
    for (int j = 0; j < NA; ++j) tv[j] = 0.0;
  }
  const double rue = LD(p.ru, o), rue_m = up1(rue);
  const double ru_edge_w = act ? p.fzm[k] * rue + p.fzp[k] * rue_m : 0.0;
  const double sgn_w = sgn1(ru_edge_w), sgn_t = sgn1(rue);
  fw = 0.0;
  ft = 0.0;
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const double a = p.adv_coefs[e * 15 + j], b = p.adv_coefs_3rd[e * 15 + j];
    fw = fw + (a + sgn_w * b) * wv[j];
    ft = ft + (a + sgn_t * b) * tv[j];
  }
}

__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_advflux(Dims d, Ptrs p) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  if (!(c1 < d.nCellsSolve || c2 < d.nCellsSolve)) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t o = (size_t)e * K + k;
  const int na = p.nAdvCellsForEdge[e];
  double fw = 0.0, ft = 0.0;
  if (na == 10) {
    adv_edge_sums<10>(p, e, K, k, o, act, fw, ft);
  } else {
    const double rue = LD(p.ru, o), rue_m = up1(rue);
    const double ru_edge_w = act ? p.fzm[k] * rue + p.fzp[k] * rue_m : 0.0;
    const double sgn_w = sgn1(ru_edge_w), sgn_t = sgn1(rue);
    if (k <= K) {
      for (int j = 0; j < na; ++j) {
        const int ic = uni(p.advCellsForEdge[e * 15 + j]);
        const double a = p.adv_coefs[e * 15 + j], b = p.adv_coefs_3rd[e * 15 + j];
        fw = fw + (a + sgn_w * b) * p.w2[(size_t)ic * (K + 1) + k];
        ft = ft + (a + sgn_t * b) * ((k < K) ? p.theta_m2[(size_t)ic * K + k] : 0.0);
      }
    }
  }
  if (act) {
    p.advflux_w[o] = fw;
    p.advflux_th[o] = ft;
  }
}

// k_dyn_cells3 on the per-cell stencil record (ME = maxEdges <= 7, RK1 = rk_step == 1): the
// edge columns of every edge of the cell (and the cells across them) are loaded in one batch
// after a single scalar round trip; the sums keep the reference order edge by edge.
template <int ME, bool RK1, bool SML = false>
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_cells3_r(Dims d, Ptrs p, Config cf, DynTendScal s) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const bool actw = k <= K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + kc, ow = (size_t)c * K1 + kw;
  const CellSten<ME> st = load_sten<ME>(p, c);
  const bool del4w = RK1 && s.h_mom_eddy_visc4 > 0.0, del4t = RK1 && s.h_theta_eddy_visc4 > 0.0;
  // ---- every load up front
  double rue[ME], afw[ME], aft[ME], x1[ME], x2[ME];  // x1/x2: rk>1 ru_save, theta_m across; rk1 delsq_w / delsq_theta across
  double sdv[ME], msi[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const size_t oe = (size_t)st.e[i] * K + kc, oc = (size_t)st.o[i] * K + kc;
    rue[i] = p.ru[oe];
    afw[i] = p.advflux_w[oe];
    aft[i] = p.advflux_th[oe];
    if (RK1) {
      x1[i] = del4w ? p.delsq_w[oc] : 0.0;
      x2[i] = del4t ? p.delsq_theta[oc] : 0.0;
      sdv[i] = ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i);
      msi[i] = 0.0;
      if (del4w || del4t) msi[i] = ld_uniform_f64(p.meshScalingDel4 + st.e[i]);
    } else {
      x1[i] = p.ru_save[oe];
      x2[i] = p.theta_m1[oc];
      sdv[i] = ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i);
    }
  }
  double idc[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) idc[i] = RK1 && (del4w || del4t) ? ld_uniform_f64(p.invDcEdge + st.e[i]) : 0.0;
  const double invA = ld_uniform_f64(p.invAreaCell + c);
  const double fzm = p.fzm[kc], fzp = p.fzp[kc], rdzu = p.rdzu[kc], rdzw_k = p.rdzw[kc];
  const double thc1 = p.theta_m1[o];
  const double twe0 = p.tend_w_euler[ow];
  const double wk = p.w2[ow], rwk = p.rw[ow];
  const double ppk = p.pressure_p[o], dpk = p.dpdz[o], cqw = p.cqw[o];
  const double rz = p.rho_zz2[o];
  const double dsw = del4w ? p.delsq_w[o] : 0.0, dst = del4t ? p.delsq_theta[o] : 0.0;
  const double tte0 = p.tend_theta_euler[o];
  const double th = p.theta_m2[o], rws = p.rw_save[ow];
  const double rtd = d.diabatic ? p.rt_diabatic_tend[o] : 0.0;
  // SML: the fused smlstep's tend_u of the cell's edges, issued with the rest (the zb column its
  // sign selects is loaded at the end: early, it would cost a wave per SIMD)
  const bool sml = SML && !(p.cell_bnd[c] & CELL_HALO_EDGE) && p.bdyMaskCell[c] <= N_RELAX_ZONE;
  double ut[ME], zz = 0.0;
  if (sml) {
#pragma unroll
    for (int i = 0; i < ME; ++i) ut[i] = p.tend_u[(size_t)uni(st.e[i]) * K + kc];
    zz = p.zz[o];
  }
  // ---- horizontal advection of w (5046-5074) and theta (5231-5252)
  double tw = 0.0, tt = 0.0;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const double rue_m = up1(rue[i]);
    if (i < st.ne) {
      const double sg = st.sg(i);
      const double ru_edge_w = fzm * rue[i] + fzp * rue_m;
      tw = tw - sg * ru_edge_w * afw[i];
      tt = tt - sg * rue[i] * aft[i];
    }
  }
  // ---- w euler tendency: del4 (rk1, 5134-5152)
  double twe = twe0;
  if (del4w) {
    const double r_areaCell = s.h_mom_eddy_visc4 * invA;
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      if (i < st.ne) {
        const double edge_sign = msi[i] * r_areaCell * sdv[i] * idc[i];
        const double dd = st.first(i) ? (x1[i] - dsw) : (dsw - x1[i]);  // delsq_w(cell2) - delsq_w(cell1)
        if (act && k >= 1) twe = twe - edge_sign * dd;
      }
    }
  }
  // ---- w: vertical advection, PGF/buoyancy (5167-5197)
  const double wm1 = up1(wk), wm2 = up2(wk), wp1 = dn1(wk), rwm1 = up1(rwk);
  double wdwz = 0.0;
  if (k == 1 || k == K - 1) wdwz = 0.25 * (rwk + rwm1) * (wk + wm1);
  else if (k >= 2 && k <= K - 2) wdwz = flux3(wm2, wm1, wk, wp1, 0.5 * (rwk + rwm1), 1.0);
  const double wdwz_p = dn1(wdwz);
  if (act && k >= 1) tw = tw * invA - rdzu * (wdwz_p - wdwz);
  const double ppm = up1(ppk), dpm = up1(dpk);
  if (RK1 && act && k >= 1) twe = twe - cqw * (rdzu * (ppk - ppm) - (fzm * dpk + fzp * dpm));
  const double rzm = up1(rz), rdzw_m = up1(rdzw_k);
  if (RK1 && cf.v_mom_eddy_visc2 > 0.0) {
    if (act && k >= 1)
      twe = twe + cf.v_mom_eddy_visc2 * 0.5 * (rz + rzm) * ((wp1 - wk) * rdzw_k - (wk - wm1) * rdzw_m) * rdzu;
  }
  if (act && k >= 1) tw = tw + twe;
  // ---- perturbation flux for rtheta_pp (rk > 1, 5256-5269), after all advection terms
  if (!RK1) {
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      if (i < st.ne) {
        const double flux = sdv[i] * (x1[i] - rue[i]) * 0.5 * (x2[i] + thc1);  // sign*dvEdge*(ru_save-ru)*0.5*(th2+th1)
        if (act) tt = tt - flux;
      }
    }
  }
  // ---- theta euler tendency: del4 (rk1, 5305-5323)
  double tte = tte0;
  if (del4t) {
    const double r_areaCell = s.h_theta_eddy_visc4 * (1.0 / PRANDTL) * invA;
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      if (i < st.ne) {
        const double edge_sign = msi[i] * r_areaCell * sdv[i] * idc[i];
        const double dd = st.first(i) ? (x2[i] - dst) : (dst - x2[i]);
        if (act) tte = tte - edge_sign * dd;
      }
    }
  }
  // ---- theta: vertical advection (5331-5354)
  const double thm1 = up1(th), thm2 = up2(th), thp1 = dn1(th);
  const double ths = thc1, thsm1 = up1(ths);
  double wdtz = 0.0;
  if (k == 1) {
    wdtz = rwk * (fzm * th + fzp * thm1);
    wdtz = wdtz + (rws - rwk) * (fzm * ths + fzp * thsm1);
  } else if (k >= 2 && k <= K - 2) {
    wdtz = flux3(thm2, thm1, th, thp1, rwk, s.coef_3rd_order);
    wdtz = wdtz + (rws - rwk) * (fzm * ths + fzp * thsm1);
  } else if (k == K - 1) {
    wdtz = rws * (fzm * th + fzp * thm1);
  }
  const double wdtz_p = dn1(wdtz);
  if (RK1 && cf.v_theta_eddy_visc2 > 0.0) {
    if (act && k >= 1 && k <= K - 2) {
      const size_t zo = (size_t)c * K1;
      const double z1 = p.zgrid[zo + k - 1], z2 = p.zgrid[zo + k], z3 = p.zgrid[zo + k + 1], z4 = p.zgrid[zo + k + 2];
      const double zm = 0.5 * (z1 + z2), z0 = 0.5 * (z2 + z3), zp = 0.5 * (z3 + z4);
      if (cf.mix_full) {
        tte = tte + cf.v_theta_eddy_visc2 * (1.0 / PRANDTL) * rz *
                        ((thp1 - th) / (zp - z0) - (th - thm1) / (z0 - zm)) / (0.5 * (zp - zm));
      } else {
        const double ti = p.t_init[o], tim = p.t_init[o - 1], tip = p.t_init[o + 1];
        tte = tte + cf.v_theta_eddy_visc2 * (1.0 / PRANDTL) * rz *
                        (((thp1 - tip) - (th - ti)) / (zp - z0) - ((th - ti) - (thm1 - tim)) / (z0 - zm)) / (0.5 * (zp - zm));
      }
    }
  }
  double twf = (act && k >= 1) ? tw : 0.0;
  // SML: atm_set_smlstep_pert_variables (2290-2307) of this cell, fused: the cell's edges are all
  // owned (no halo edge), so their tend_u is final here and needs no exchange (the cells with a
  // halo edge run k_smlstep_pert_b after the 642 exchange); same expressions as k_smlstep_pert_b
  if (sml) {
    double zs[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) zs[i] = (sgn1(ut[i]) > 0.0 ? p.zb_p : p.zb_m)[((size_t)c * ME + i) * K1 + kw];
    double wt = twf;
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      const double utm = up1(ut[i]);
      if (i < st.ne && act && k >= 1) {
        const double flux = st.sg(i) * (fzm * ut[i] + fzp * utm);
        wt = wt - zs[i] * flux;
      }
    }
    const double zzm = up1(zz);
    if (act && k >= 1) twf = (fzm * zz + fzp * zzm) * wt;
  }
  if (actw) {
    p.tend_w[ow] = twf;
    if (RK1) p.tend_w_euler[ow] = twe;
  }
  if (act) {
    tt = tt * invA - rdzw_k * (wdtz_p - wdtz);
    if (s.store_phys_diag) {
      p.tend_rtheta_adv[o] = tt;
      p.rthdynten[o] = tt / rz;
    }
    tt = tt + rz * rtd;
    if (RK1) p.tend_theta_euler[o] = tte;
    p.tend_theta[o] = tt + tte + PHYS(p.tend_rtheta_physics, o);
  }
}

// k_dyn_advflux with batched loads (NA = 2*maxEdges-2 >= nAdvCellsForEdge): the edge's index
// and coefficient rows and its ru column go out together, then the 2*NA neighbour columns.
template <int NA>
__global__ __launch_bounds__(EDGE_THREADS) void k_dyn_advflux_b(Dims d, Ptrs p) {
  const int e = wave_elem_e();
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)e * K + kc;
  const int2 ce = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * e);
  const int na = p.nAdvCellsForEdge[e];
  int ic[NA];
  double a[NA], b[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    ic[j] = p.advCellsForEdge[(size_t)e * 15 + j];
    a[j] = ld_uniform_f64(p.adv_coefs + (size_t)e * 15 + j);
    b[j] = ld_uniform_f64(p.adv_coefs_3rd + (size_t)e * 15 + j);
  }
  const double rue = p.ru[o];
  if (!(ce.x < d.nCellsSolve || ce.y < d.nCellsSolve)) return;
  double wv[NA], tv[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int cj = uni(ic[j]);
    wv[j] = p.w2[(size_t)cj * K1 + kw];
    tv[j] = p.theta_m2[(size_t)cj * K + kc];
  }
  const double fzm = p.fzm[kc], fzp = p.fzp[kc];
  const double rue_m = up1(rue);
  const double ru_edge_w = act ? fzm * rue + fzp * rue_m : 0.0;
  const double sgn_w = sgn1(ru_edge_w), sgn_t = sgn1(rue);
  double fw = 0.0, ft = 0.0;
  if (na <= NA) {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      if (j < na) {
        fw = fw + (a[j] + sgn_w * b[j]) * wv[j];
        ft = ft + (a[j] + sgn_t * b[j]) * tv[j];
      }
    }
  } else {  // not produced by meshes with maxEdges <= 7; kept for completeness
    for (int j = 0; j < na; ++j) {
      const int cj = uni(p.advCellsForEdge[(size_t)e * 15 + j]);
      const double aj = p.adv_coefs[(size_t)e * 15 + j], bj = p.adv_coefs_3rd[(size_t)e * 15 + j];
      fw = fw + (aj + sgn_w * bj) * p.w2[(size_t)cj * K1 + kw];
      ft = ft + (aj + sgn_t * bj) * p.theta_m2[(size_t)cj * K + kc];
    }
  }
  if (act) {
    p.advflux_w[o] = fw;
    p.advflux_th[o] = ft;
  }
}

// cells (solve): w tendency (5046-5074, del4 5134-5152, 5167-5223) and theta tendency
// (5231-5269, del4 5305-5323, 5331-5414)
__global__ __launch_bounds__(BLOCK_THREADS) void k_dyn_cells3(Dims d, Ptrs p, Config cf, DynTendScal s) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const bool actw = k <= K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k, ow = (size_t)c * K1 + k;
  const int ne = p.nEdgesOnCell[c];
  const double fzm = act ? p.fzm[k] : 0.0, fzp = act ? p.fzp[k] : 0.0;
  const bool rk1 = s.rk_step == 1;
  // ---------------- horizontal advection of w (5046-5074) and theta (5231-5252) from the
  // edge fluxes of k_dyn_advflux, plus the rk>1 perturbation flux terms (5256-5269): one
  // pass over the edges loads each edge column once.  The two theta sums keep the
  // reference order (all advection terms, then all perturbation terms).
  const double thc1 = LD(p.theta_m1, o);
  double tw = 0.0, tt = 0.0;
  double tpert[MAX_EDGES_UNROLL];
  const bool pert = !rk1 && ne <= MAX_EDGES_UNROLL;
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double sg = p.edgesOnCell_sign[c * d.maxEdges + i];
    const double rue = LD(p.ru, (size_t)e * K + k);
    const double rue_m = up1(rue);
    const double ru_edge_w = fzm * rue + fzp * rue_m;
    tw = tw - sg * ru_edge_w * LD(p.advflux_w, (size_t)e * K + k);
    tt = tt - sg * rue * LD(p.advflux_th, (size_t)e * K + k);
    if (pert && act) {
      const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
      const double th1 = (c1 == c) ? thc1 : p.theta_m1[(size_t)c1 * K + k];
      const double th2 = (c2 == c) ? thc1 : p.theta_m1[(size_t)c2 * K + k];
#pragma unroll
      for (int q = 0; q < MAX_EDGES_UNROLL; ++q)
        if (q == i) tpert[q] = sg * p.dvEdge[e] * (p.ru_save[(size_t)e * K + k] - rue) * 0.5 * (th2 + th1);
    }
  }
  // ---------------- w euler tendency: del4 (rk1)
  double twe = actw ? p.tend_w_euler[ow] : 0.0;
  if (rk1 && s.h_mom_eddy_visc4 > 0.0) {
    const double r_areaCell = s.h_mom_eddy_visc4 * p.invAreaCell[c];
    for (int i = 0; i < ne; ++i) {
      const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
      const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
      const double edge_sign = p.meshScalingDel4[e] * r_areaCell * p.dvEdge[e] *
                               p.edgesOnCell_sign[c * d.maxEdges + i] * p.invDcEdge[e];
      if (act && k >= 1) twe = twe - edge_sign * (p.delsq_w[(size_t)c2 * K + k] - p.delsq_w[(size_t)c1 * K + k]);
    }
  }
  // ---------------- w: vertical advection, PGF/buoyancy (5167-5197)
  const double wk = LDW(p.w2, ow), rwk = LDW(p.rw, ow);
  const double wm1 = up1(wk), wm2 = up2(wk), wp1 = dn1(wk), rwm1 = up1(rwk);
  double wdwz = 0.0;
  if (k == 1 || k == K - 1) wdwz = 0.25 * (rwk + rwm1) * (wk + wm1);
  else if (k >= 2 && k <= K - 2) wdwz = flux3(wm2, wm1, wk, wp1, 0.5 * (rwk + rwm1), 1.0);
  const double wdwz_p = dn1(wdwz);
  const double rdzu = act ? p.rdzu[k] : 0.0;
  if (act && k >= 1) tw = tw * p.invAreaCell[c] - rdzu * (wdwz_p - wdwz);
  const double ppk = LD(p.pressure_p, o), ppm = up1(ppk);
  const double dpk = LD(p.dpdz, o), dpm = up1(dpk);
  if (rk1 && act && k >= 1)
    twe = twe - p.cqw[o] * (rdzu * (ppk - ppm) - (fzm * dpk + fzp * dpm));
  if (rk1 && cf.v_mom_eddy_visc2 > 0.0) {
    const double rz = LD(p.rho_zz2, o), rzm = up1(rz);
    const double rdzw_k = act ? p.rdzw[k] : 0.0, rdzw_m = up1(rdzw_k);
    if (act && k >= 1)
      twe = twe + cf.v_mom_eddy_visc2 * 0.5 * (rz + rzm) * ((wp1 - wk) * rdzw_k - (wk - wm1) * rdzw_m) * rdzu;
  }
  if (act && k >= 1) tw = tw + twe;
  if (actw) {
    p.tend_w[ow] = (act && k >= 1) ? tw : 0.0;
    if (rk1) p.tend_w_euler[ow] = twe;
  }
  if (pert) {
    if (act) {
#pragma unroll
      for (int q = 0; q < MAX_EDGES_UNROLL; ++q)
        if (q < ne) tt = tt - tpert[q];
    }
  } else if (!rk1) {  // perturbation flux for rtheta_pp (5256-5269), cells with > MAX_EDGES_UNROLL edges
    for (int i = 0; i < ne; ++i) {
      const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
      const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
      if (act) {
        const double flux = p.edgesOnCell_sign[c * d.maxEdges + i] * p.dvEdge[e] *
                            (p.ru_save[(size_t)e * K + k] - p.ru[(size_t)e * K + k]) * 0.5 *
                            (p.theta_m1[(size_t)c2 * K + k] + p.theta_m1[(size_t)c1 * K + k]);
        tt = tt - flux;
      }
    }
  }
  double tte = LD(p.tend_theta_euler, o);
  if (rk1 && s.h_theta_eddy_visc4 > 0.0) {
    const double r_areaCell = s.h_theta_eddy_visc4 * (1.0 / PRANDTL) * p.invAreaCell[c];
    for (int i = 0; i < ne; ++i) {
      const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
      const double edge_sign = p.meshScalingDel4[e] * r_areaCell * p.dvEdge[e] *
                               p.edgesOnCell_sign[c * d.maxEdges + i] * p.invDcEdge[e];
      const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
      if (act) tte = tte - edge_sign * (p.delsq_theta[(size_t)c2 * K + k] - p.delsq_theta[(size_t)c1 * K + k]);
    }
  }
  // ---------------- theta: vertical advection (5331-5354)
  const double th = LD(p.theta_m2, o), thm1 = up1(th), thm2 = up2(th), thp1 = dn1(th);
  const double ths = LD(p.theta_m1, o), thsm1 = up1(ths);
  const double rws = LDW(p.rw_save, ow);
  double wdtz = 0.0;
  if (k == 1) {
    wdtz = rwk * (fzm * th + fzp * thm1);
    wdtz = wdtz + (rws - rwk) * (fzm * ths + fzp * thsm1);
  } else if (k >= 2 && k <= K - 2) {
    wdtz = flux3(thm2, thm1, th, thp1, rwk, s.coef_3rd_order);
    wdtz = wdtz + (rws - rwk) * (fzm * ths + fzp * thsm1);
  } else if (k == K - 1) {
    wdtz = rws * (fzm * th + fzp * thm1);
  }
  const double wdtz_p = dn1(wdtz);
  if (rk1 && cf.v_theta_eddy_visc2 > 0.0) {
    const double rz = LD(p.rho_zz2, o);
    if (act && k >= 1 && k <= K - 2) {
      const size_t zo = (size_t)c * K1;
      const double z1 = p.zgrid[zo + k - 1], z2 = p.zgrid[zo + k], z3 = p.zgrid[zo + k + 1], z4 = p.zgrid[zo + k + 2];
      const double zm = 0.5 * (z1 + z2), z0 = 0.5 * (z2 + z3), zp = 0.5 * (z3 + z4);
      if (cf.mix_full) {
        tte = tte + cf.v_theta_eddy_visc2 * (1.0 / PRANDTL) * rz *
                        ((thp1 - th) / (zp - z0) - (th - thm1) / (z0 - zm)) / (0.5 * (zp - zm));
      } else {
        const double ti = p.t_init[o], tim = p.t_init[o - 1], tip = p.t_init[o + 1];
        tte = tte + cf.v_theta_eddy_visc2 * (1.0 / PRANDTL) * rz *
                        (((thp1 - tip) - (th - ti)) / (zp - z0) - ((th - ti) - (thm1 - tim)) / (z0 - zm)) / (0.5 * (zp - zm));
      }
    }
  }
  if (act) {
    const double rz = p.rho_zz2[o];
    tt = tt * p.invAreaCell[c] - p.rdzw[k] * (wdtz_p - wdtz);
    if (s.store_phys_diag) {
      p.tend_rtheta_adv[o] = tt;
      p.rthdynten[o] = tt / rz;
    }
    tt = tt + rz * (d.diabatic ? p.rt_diabatic_tend[o] : 0.0);
    if (rk1) p.tend_theta_euler[o] = tte;
    p.tend_theta[o] = tt + tte + PHYS(p.tend_rtheta_physics, o);
  }
}

// ============================================================================
// atm_set_smlstep_pert_variables_work  (mpas_atm_time_integration.F:2290-2307)
// ============================================================================
// phase: 0 = every cell; 1 / 2 = only cells without / with a halo edge (split around the
// tend_u halo exchange, which then overlaps the interior cells)
__global__ __launch_bounds__(BLOCK_THREADS) void k_smlstep_pert(Dims d, Ptrs p, int phase) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  if (phase && (((p.cell_bnd[c] & CELL_HALO_EDGE) != 0) != (phase == 2))) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const double fzm = act ? p.fzm[k] : 0.0, fzp = act ? p.fzp[k] : 0.0;
  double wt = (k <= K) ? p.tend_w[(size_t)c * K1 + k] : 0.0;
  const int ne = p.nEdgesOnCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double ut = LD(p.tend_u, (size_t)e * K + k), utm = up1(ut);
    if (act && k >= 1) {
      const double flux = p.edgesOnCell_sign[c * d.maxEdges + i] * (fzm * ut + fzp * utm);
      const size_t zo = ((size_t)c * d.maxEdges + i) * K1 + k;
      wt = wt - (p.zb_cell[zo] + sgn1(ut) * p.zb3_cell[zo]) * flux;
    }
  }
  const double zz = LD(p.zz, (size_t)c * K + k), zzm = up1(zz);
  if (act && k >= 1) p.tend_w[(size_t)c * K1 + k] = (fzm * zz + fzp * zzm) * wt;
}

template <int ME>
// tu_up: the 642 exchange's fused unpack (XUnpack, edge field tend_u): the cell's halo edges read
// their received tend_u from the receive buffer and write it into tend_u for the later readers (every
// reader of a halo edge's tend_u reads an edge of an owned cell, and such an edge has exactly one)
__global__ __launch_bounds__(BLOCK_THREADS) void k_smlstep_pert_b(Dims d, Ptrs p, int phase,
                                                                  XUnpack tu_up = XUnpack{}) {
  int c = wave_elem(0);
  if (phase == 2) {  // the compact bnd_cells list (owned cells with CELL_HALO_EDGE)
    if (c >= d.n_bnd_cells) return;
    c = __builtin_amdgcn_readfirstlane(p.bnd_cells[c]);
  }
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const CellSten<ME> st = load_sten<ME>(p, c);
  int uoff[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    uoff[i] = rec_off(tu_up, 0, uni(st.e[i]), d.nEdgesSolve);
    if (uoff[i] >= 0 && act) p.tend_u[(size_t)uni(st.e[i]) * K + k] = tu_up.recv[uoff[i] + k];
  }
  if (p.bdyMaskCell[c] > N_RELAX_ZONE) return;  // no conversion in the specified zone (2292; any run)
  const int bnd = phase ? p.cell_bnd[c] : 0;
  double wt = p.tend_w[(size_t)c * K1 + kw];
  const double zz = p.zz[(size_t)c * K + kc];
  const double fzm = p.fzm[kc], fzp = p.fzp[kc];
  if (phase && (((bnd & CELL_HALO_EDGE) != 0) != (phase == 2))) return;
  double ut[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i)
    ut[i] = uoff[i] >= 0 ? tu_up.recv[uoff[i] + kc] : p.tend_u[(size_t)uni(st.e[i]) * K + kc];
  // zb_cell + sign(1,ut) * zb3_cell, loaded as the one of zb_p / zb_m the sign selects (k_build_zb)
  double zs[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) zs[i] = (sgn1(ut[i]) > 0.0 ? p.zb_p : p.zb_m)[((size_t)c * ME + i) * K1 + kw];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const double utm = up1(ut[i]);
    if (i < st.ne && act && k >= 1) {
      const double flux = st.sg(i) * (fzm * ut[i] + fzp * utm);
      wt = wt - zs[i] * flux;
    }
  }
  const double zzm = up1(zz);
  if (act && k >= 1) p.tend_w[(size_t)c * K1 + k] = (fzm * zz + fzp * zzm) * wt;
}

// ============================================================================
// atm_advance_acoustic_step_work  (mpas_atm_time_integration.F:2535-2721)
// ============================================================================
// edge phase (2540-2601): edges with >=1 owned cell.
// DD: first apply the divergence damping of the previous sub-step (atm_divergence_damping_3d,
// 2765-2793, same expression), then this sub-step's update.  srk3 calls damping and the next
// edge phase back to back on the same edges (849-869, then 794-837), with only the rtheta_pp /
// rho_pp halo exchange in between, so one pass over ru_p does both.  The sum is the same
// double either way: the damped ru_p is rounded before the update adds to it.
// phase: 0 = every edge; 1 / 2 = edges without / with a halo cell (split around that exchange).
// fresh = 1: the previous sub-step was sub-step 1, whose edge phase srk3 no longer launches:
// its ru_p and ruAvg are dts * tend_u (794-837 with small_step = 1), formed here from tend_u.
template <bool DD>
__global__ __launch_bounds__(EDGE_THREADS) void k_acoustic_edges(Dims d, Ptrs p, double dts, int small_step,
                                                                  double coef_divdamp, int phase, int fresh) {
  const int e = wave_elem_e();
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t o = (size_t)e * K + min(k, K - 1);  // lanes >= K load level K-1 and store nothing
  // one scalar round trip for the edge's metadata, with its own columns already in flight
  const int2 ce = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * e);
  const int bnd = phase ? p.edge_bnd[e] : 0;
  const double tu = p.tend_u[o];
  if (small_step == 1) {
    if (!(ce.x < d.nCellsSolve || ce.y < d.nCellsSolve) || (phase && ((bnd != 0) != (phase == 2)))) return;
    const double rup = dts * tu;
    if (act) {
      p.ru_p[o] = rup;
      p.ruAvg[o] = rup;
    }
    return;
  }
  double rup = fresh ? dts * tu : p.ru_p[o];
  const double rua = fresh ? rup : p.ruAvg[o], cqu = p.cqu[o], zxu = p.zxu[o];
  const double mask = p.specZoneMaskEdge[e], invDc = p.invDcEdge[e];
  if (!(ce.x < d.nCellsSolve || ce.y < d.nCellsSolve) || (phase && ((bnd != 0) != (phase == 2)))) return;
  const int c1 = uni(ce.x), c2 = uni(ce.y);
  const double rcv = RGAS / (CP - RGAS);
  const double c2v = CP * rcv;
  const size_t o1 = (size_t)c1 * K + min(k, K - 1), o2 = (size_t)c2 * K + min(k, K - 1);
  const double rt1 = p.rtheta_pp[o1], rt2 = p.rtheta_pp[o2];
  const double zz1 = p.zz[o1], zz2 = p.zz[o2], ex1 = p.exner[o1], ex2 = p.exner[o2];
  const double rp1 = p.rho_pp[o1], rp2 = p.rho_pp[o2];
  if (DD) {
    const double d1 = -(rt1 - p.rtheta_pp_old[o1]);
    const double d2 = -(rt2 - p.rtheta_pp_old[o2]);
    rup = rup + coef_divdamp * (d2 - d1) * (1.0 - mask) / (p.theta_m1[o1] + p.theta_m1[o2]);
  }
  double pgrad = ((rt2 - rt1) * invDc) / (.5 * (zz2 + zz1));
  pgrad = cqu * 0.5 * c2v * (ex1 + ex2) * pgrad;
  pgrad = pgrad + 0.5 * zxu * GRAVITY * (rp1 + rp2);
  rup = rup + dts * (tu - (1.0 - mask) * pgrad);
  if (act) {
    p.ru_p[o] = rup;
    p.ruAvg[o] = rua + rup;
  }
}

// ---------------------------------------------------------------------------------------------
// Pair layout for gather-heavy edge kernels: one wavefront carries TWO edges (lanes 0-31 edge
// 2w, lanes 32-63 edge 2w+1) and each lane TWO consecutive levels (2l, 2l+1), so every column
// access is one 16-byte load per lane.  On MI355X a scattered 64-lane vector load costs about
// the same ~14 CU cycles whether it moves 8 or 16 bytes per lane (exp microbenchmark, DESIGN.md
// §4), so this halves the instruction cost of the neighbour gathers.  Needs an even K.
struct d2 {
  double x, y;
};
__device__ __forceinline__ d2 ld2(const double* __restrict__ a) {
  d2 r;
  __builtin_memcpy(&r, a, 16);
  return r;
}
__device__ __forceinline__ void st2(double* a, d2 v) { __builtin_memcpy(a, &v, 16); }

// The first N entries of one edge's row of the 15-wide stencil tables (advCellsForEdge, adv_coefs,
// adv_coefs_3rd), each half-wave its own edge's row, as 16-byte vector loads: both halves' rows
// come in the same few instructions and one wait.  Through the scalar cache the two edges' rows
// need ~100 SGPRs, so they arrive in dependent batches, a memory round trip each, before the
// first gather can issue.
template <int N>
__device__ __forceinline__ void ld_row(const double* __restrict__ src, double (&dst)[N]) {
#pragma unroll
  for (int j = 0; j + 1 < N; j += 2) {
    const d2 v = ld2(src + j);
    dst[j] = v.x;
    dst[j + 1] = v.y;
  }
  if (N & 1) dst[N - 1] = src[N - 1];
}
template <int N>
__device__ __forceinline__ void ld_row(const int* __restrict__ src, int (&dst)[N]) {
#pragma unroll
  for (int j = 0; j + 3 < N; j += 4) {
    int4 v;
    __builtin_memcpy(&v, src + j, 16);
    dst[j] = v.x;
    dst[j + 1] = v.y;
    dst[j + 2] = v.z;
    dst[j + 3] = v.w;
  }
#pragma unroll
  for (int j = N & ~3; j < N; ++j) dst[j] = src[j];
}
// store of a lane's two levels; two = false (odd K, last pair): its second level is level K, past
// the column, so only the first is stored
__device__ __forceinline__ void pst(double* a, d2 v, bool two) {
  if (two) st2(a, v);
  else a[0] = v.x;
}
// PAIR_EPW elements per wavefront: 2 in the K <= 63 build (lanes 0..31 and 32..63, levels 2l, 2l+1
// of lane l of each half), 1 in the wide build (lanes 0..63 of one column: K <= 127 with the same
// two levels per lane, the same DPP moves and 16-byte accesses, no LDS).  PAIR_WPB wavefronts of
// consecutive elements per workgroup.
#ifdef MPAS_WIDE
#define PAIR_EPW 1
#define PAIR_WPB 4
#else
#define PAIR_EPW 2
#define PAIR_WPB EDGE_WPB
#endif
#define PAIR_THREADS (64 * PAIR_WPB)
__device__ __forceinline__ int pair_wave() {
  return __builtin_amdgcn_readfirstlane(xcd_block() * PAIR_WPB + (threadIdx.x >> 6));
}
__device__ __forceinline__ int pair_half() { return PAIR_EPW == 2 ? (threadIdx.x >> 5) & 1 : 0; }
__device__ __forceinline__ int pair_lane() { return PAIR_EPW == 2 ? threadIdx.x & 31 : threadIdx.x & 63; }
// the two edges of this wavefront: consecutive edges, or in phase 2 of a split kernel consecutive
// entries of the compact bnd_pairs list (halo-boundary edges with an owned cell); false: none
__device__ __forceinline__ bool pair_edges(const Dims& d, const Ptrs& p, int phase, int& eA, int& eB, bool& hasB) {
  const int i = PAIR_EPW * pair_wave();
  if (phase == 2) {
    if (i >= d.n_bnd_pairs) return false;
    hasB = PAIR_EPW == 2 && i + 1 < d.n_bnd_pairs;
    eA = __builtin_amdgcn_readfirstlane(p.bnd_pairs[i]);
    eB = hasB ? __builtin_amdgcn_readfirstlane(p.bnd_pairs[i + 1]) : eA;
    return true;
  }
  if (i >= d.nEdges) return false;
  hasB = PAIR_EPW == 2 && i + 1 < d.nEdges;
  eA = i;
  eB = hasB ? i + 1 : i;
  return true;
}
__device__ __forceinline__ int sel(int h, int a, int b) { return h ? b : a; }
__device__ __forceinline__ double sel(int h, double a, double b) { return h ? b : a; }

// vertical neighbours in the pair layout (levels 2l, 2l+1 on lane l of each half-wave), with the
// end-of-column behaviour of up1 / up2 / dn1 (a lane with no neighbour keeps its own value)
__device__ __forceinline__ double lane_shr1(double v) {  // value of lane-1 (own at lane 0)
  const int lo = __double2loint(v), hi = __double2hiint(v);
  return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false),
                          __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ double lane_shl1(double v) {  // value of lane+1 (own at lane 63)
  const int lo = __double2loint(v), hi = __double2hiint(v);
  return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false),
                          __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ d2 km1(d2 v, int l) {  // levels (k-1) of (2l, 2l+1)
  const double t = lane_shr1(v.y);
  return d2{l == 0 ? v.x : t, v.x};
}
__device__ __forceinline__ d2 km2(d2 v, int l) {  // levels (k-2)
  const double tx = lane_shr1(v.x), ty = lane_shr1(v.y);
  return d2{l == 0 ? v.x : tx, l == 0 ? v.y : ty};
}
__device__ __forceinline__ d2 kp1(d2 v) {  // levels (k+1)
  return d2{v.y, lane_shl1(v.x)};
}

// an edge field of the wavefront's two edges (pair layout) into their slots of a fused exchange's
// send buffer (XPack over owned edges: the damped ru_p of 876-887, the final tend_u of 642); st: this
// lane stores its edge's levels
__device__ __forceinline__ void pack_rec_edge(const XPack& pk, const Dims& d, int eA, int eB, bool hasB, int h,
                                              int lc, bool st, bool two, d2 v) {
  if (!pk.start) return;
  for (int half = 0; half < (hasB ? 2 : 1); ++half) {
    const int e = half ? eB : eA;
    if (e >= d.nEdgesSolve) continue;
    const int s0 = __builtin_amdgcn_readfirstlane(pk.start[e]), s1 = __builtin_amdgcn_readfirstlane(pk.start[e + 1]);
    for (int s = s0; s < s1; ++s) {
      double* dst = pk.dst[s];
      if (h == half && st) pst(dst + 2 * lc, v, two);
    }
  }
}

// k_dyn_edges_b in the pair layout (NE2 = 2*maxEdges-2 TRiSK neighbours).  SPLIT (rk1 only): this
// launch computes tend_u alone and k_dyn_edges_pgf_p the PGF part of tend_u_euler and del2 --
// at rk1 the two are independent (no finalize), and together they need 244 VGPRs (2 waves/SIMD).
// tp: with finalize, the final tend_u also goes to the 642 exchange's send buffer (XPack), or nothing
template <bool RK1, int NE2, bool SPLIT = false, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_dyn_edges_p(Dims d, Ptrs p, Config cf, DynTendScal s,
                                                              int finalize, XPack tp = XPack{}) {
  constexpr bool PGF = RK1 && !SPLIT;
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1), lw = min(l, K / 2);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t K1 = K + 1;
  const size_t o = (size_t)e * K + 2 * lc;
  const bool solveA = eA < d.nEdgesSolve, solveB = hasB && eB < d.nEdgesSolve;
  const bool solve = h ? solveB : solveA;
  const bool mine = h == 0 || hasB;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const double invDc = sel(h, ld_uniform_f64(p.invDcEdge + eA), ld_uniform_f64(p.invDcEdge + eB));
  const d2 re = ld2(p.rho_edge + o);
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const size_t o1 = (size_t)c1 * K + 2 * lc, o2 = (size_t)c2 * K + 2 * lc;
  const int kx = 2 * l, ky = 2 * l + 1;  // true levels of the two components
  const bool stx = mine && kx < K, sty = mine && ky < K;
  auto store = [&](double* a, d2 v) {
    if (ODD) {
      if (stx) pst(a + o, v, sty);
    } else if (stx && sty) {
      st2(a + o, v);
    }
  };
  // rk1 del^2 of u (4856-4883), all edges
  auto del2 = [&](d2 tue, d2 dv1, d2 dv2, d2 vo1, d2 vo2, d2 kd1, d2 kd2, double invDv, double msd2) {
    const double r_dc = invDc;
    const double r_dv = fmin(invDv, 4 * invDc);
    d2 ud, out;
    ud.x = (dv2.x - dv1.x) * r_dc - (vo2.x - vo1.x) * r_dv;
    ud.y = (dv2.y - dv1.y) * r_dc - (vo2.y - vo1.y) * r_dv;
    store(p.delsq_u, d2{0.0 + ud.x, 0.0 + ud.y});
    out.x = tue.x + re.x * (0.5 * (kd1.x + kd2.x)) * ud.x * msd2;
    out.y = tue.y + re.y * (0.5 * (kd1.y + kd2.y)) * ud.y * msd2;
    store(p.tend_u_euler, out);
  };
  if (!solveA && !solveB) {  // halo pair: rk1 del2 only
    if (!PGF) return;
    const int2 veA = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eA);
    const int2 veB = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eB);
    const double invDv = sel(h, ld_uniform_f64(p.invDvEdge + eA), ld_uniform_f64(p.invDvEdge + eB));
    const double msd2 = sel(h, ld_uniform_f64(p.meshScalingDel2 + eA), ld_uniform_f64(p.meshScalingDel2 + eB));
    const d2 tue = ld2(p.tend_u_euler + o);
    const int v1 = sel(h, veA.x, veB.x), v2 = sel(h, veA.y, veB.y);
    del2(tue, ld2(p.divergence + o1), ld2(p.divergence + o2), ld2(p.vorticity + (size_t)v1 * K + 2 * lc),
         ld2(p.vorticity + (size_t)v2 * K + 2 * lc), ld2(p.kdiff + o1), ld2(p.kdiff + o2), invDv, msd2);
    return;
  }
  // ---- batch 1: metadata of both edges, own columns
  const int neoe = sel(h, p.nEdgesOnEdge[eA], p.nEdgesOnEdge[eB]);
  int eoe[NE2];
  double wgt[NE2];
  // (through the scalar cache: as vector loads, ld_row, 413 -> 426 us per call)
  ld_row(p.edgesOnEdge + (size_t)e * d.maxEdges2, eoe);
#pragma unroll
  for (int j = 0; j < NE2; ++j) {
    wgt[j] = sel(h, ld_uniform_f64(p.weightsOnEdge + (size_t)eA * d.maxEdges2 + j),
                 ld_uniform_f64(p.weightsOnEdge + (size_t)eB * d.maxEdges2 + j));
  }
  int v1 = 0, v2 = 0;
  double invDv = 0.0, msd2 = 0.0;
  d2 cqu{}, zxu{};
  if (PGF) {
    const int2 veA = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eA);
    const int2 veB = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eB);
    v1 = sel(h, veA.x, veB.x);
    v2 = sel(h, veA.y, veB.y);
    invDv = sel(h, ld_uniform_f64(p.invDvEdge + eA), ld_uniform_f64(p.invDvEdge + eB));
    msd2 = sel(h, ld_uniform_f64(p.meshScalingDel2 + eA), ld_uniform_f64(p.meshScalingDel2 + eB));
    cqu = ld2(p.cqu + o);
    zxu = ld2(p.zxu + o);
  }
  const d2 uk = ld2(p.u2 + o), pve = ld2(p.pv_edge + o);
  d2 tue = RK1 ? d2{0.0, 0.0} : ld2(p.tend_u_euler + o);
  if (PGF && !solve) tue = ld2(p.tend_u_euler + o);  // the halo edge of a mixed pair
  // ---- batch 2: gathers
  const d2 rw1 = ld2(p.rw + (size_t)c1 * K1 + 2 * lw), rw2 = ld2(p.rw + (size_t)c2 * K1 + 2 * lw);
  const d2 ke1 = ld2(p.ke + o1), ke2 = ld2(p.ke + o2), hd1 = ld2(p.h_divergence + o1), hd2 = ld2(p.h_divergence + o2);
  d2 pv[NE2], uu[NE2];
#pragma unroll
  for (int j = 0; j < NE2; ++j) {
    const size_t oj = (size_t)eoe[j] * K + 2 * lc;
    pv[j] = ld2(p.pv_edge + oj);
    uu[j] = ld2(p.u2 + oj);
  }
  d2 pp1{}, pp2{}, zz1{}, zz2{}, dpz1{}, dpz2{}, dv1{}, dv2{}, vo1{}, vo2{}, kd1{}, kd2{};
  if (PGF) {
    pp1 = ld2(p.pressure_p + o1);
    pp2 = ld2(p.pressure_p + o2);
    zz1 = ld2(p.zz + o1);
    zz2 = ld2(p.zz + o2);
    dpz1 = ld2(p.dpdz + o1);
    dpz2 = ld2(p.dpdz + o2);
    dv1 = ld2(p.divergence + o1);
    dv2 = ld2(p.divergence + o2);
    vo1 = ld2(p.vorticity + (size_t)v1 * K + 2 * lc);
    vo2 = ld2(p.vorticity + (size_t)v2 * K + 2 * lc);
    kd1 = ld2(p.kdiff + o1);
    kd2 = ld2(p.kdiff + o2);
  }
  const d2 fzm = ld2(p.fzm + 2 * lc), fzp = ld2(p.fzp + 2 * lc), rdzw = ld2(p.rdzw + 2 * lc);
  // ---- tend_u (PGF rk1 4781-4788, vertical transport 4792-4807, Coriolis/KE 4811-4838)
  if (PGF && solve) {
    tue.x = -cqu.x * ((pp2.x - pp1.x) * invDc / (.5 * (zz2.x + zz1.x)) - 0.5 * zxu.x * (dpz1.x + dpz2.x));
    tue.y = -cqu.y * ((pp2.y - pp1.y) * invDc / (.5 * (zz2.y + zz1.y)) - 0.5 * zxu.y * (dpz1.y + dpz2.y));
  }
  const d2 um1 = km1(uk, l), um2 = km2(uk, l), up1v = kp1(uk);
  auto wduz_at = [&](int k, double rw1_, double rw2_, double fzm_, double fzp_, double u0, double um1_, double um2_,
                     double up1_) {
    const double rwa = 0.5 * (rw1_ + rw2_);
    if (k == 1 || k == K - 1) return 0.5 * (rw1_ + rw2_) * (fzm_ * u0 + fzp_ * um1_);
    if (k >= 2 && k <= K - 2) return flux3(um2_, um1_, u0, up1_, rwa, 1.0);
    return 0.0;
  };
  d2 wduz;
  wduz.x = wduz_at(kx, rw1.x, rw2.x, fzm.x, fzp.x, uk.x, um1.x, um2.x, up1v.x);
  wduz.y = wduz_at(ky, rw1.y, rw2.y, fzm.y, fzp.y, uk.y, um1.y, um2.y, up1v.y);
  const d2 wduz_p = kp1(wduz);
  d2 tu;
  tu.x = -rdzw.x * (wduz_p.x - wduz.x);
  tu.y = -rdzw.y * (wduz_p.y - wduz.y);
  d2 q{0.0, 0.0};
#pragma unroll
  for (int j = 0; j < NE2; ++j) {
    if (j < neoe) {
      q.x = q.x + wgt[j] * uu[j].x * (0.5 * (pve.x + pv[j].x));
      q.y = q.y + wgt[j] * uu[j].y * (0.5 * (pve.y + pv[j].y));
    }
  }
  tu.x = tu.x + re.x * (q.x - (ke2.x - ke1.x) * invDc) - uk.x * 0.5 * (hd1.x + hd2.x);
  tu.y = tu.y + re.y * (q.y - (ke2.y - ke1.y) * invDc) - uk.y * 0.5 * (hd1.y + hd2.y);
  if (finalize) {
    if (cf.rayleigh_damp_u) {
      const int k0 = K - cf.number_rayleigh_damp_u_levels;
      if (kx >= k0) tu.x = tu.x - re.x * uk.x * ((double)(kx + 1 - k0) * s.rayleigh_coef_inverse);
      if (ky >= k0) tu.y = tu.y - re.y * uk.y * ((double)(ky + 1 - k0) * s.rayleigh_coef_inverse);
    }
    const d2 tph = d.physics ? ld2(p.tend_ru_physics + o) : d2{0.0, 0.0};  // tend_ru_physics
    tu.x = tu.x + tue.x + tph.x;
    tu.y = tu.y + tue.y + tph.y;
  }
  if (solve) store(p.tend_u, tu);
  if (finalize) pack_rec_edge(tp, d, eA, eB, hasB, h, lc, solve && stx, ODD ? sty : true, tu);
  if (PGF) del2(tue, dv1, dv2, vo1, vo2, kd1, kd2, invDv, msd2);
}

// rk1, all edges: the PGF part of tend_u_euler (4781-4788, edges 1..nEdgesSolve) and the del2 of u
// (4856-4883) -- the half of k_dyn_edges_p<true> that SPLIT leaves out
template <bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_dyn_edges_pgf_p(Dims d, Ptrs p) {
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const bool solve = h ? (hasB && eB < d.nEdgesSolve) : (eA < d.nEdgesSolve);
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int2 veA = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eA);
  const int2 veB = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eB);
  const double invDc = sel(h, ld_uniform_f64(p.invDcEdge + eA), ld_uniform_f64(p.invDcEdge + eB));
  const double invDv = sel(h, ld_uniform_f64(p.invDvEdge + eA), ld_uniform_f64(p.invDvEdge + eB));
  const double msd2 = sel(h, ld_uniform_f64(p.meshScalingDel2 + eA), ld_uniform_f64(p.meshScalingDel2 + eB));
  const d2 re = ld2(p.rho_edge + o), cqu = ld2(p.cqu + o), zxu = ld2(p.zxu + o);
  d2 tue0{};
  if (!solve) tue0 = ld2(p.tend_u_euler + o);  // an owned edge overwrites it below: not read there
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y), v1 = sel(h, veA.x, veB.x), v2 = sel(h, veA.y, veB.y);
  const size_t o1 = (size_t)c1 * K + 2 * lc, o2 = (size_t)c2 * K + 2 * lc;
  const d2 pp1 = ld2(p.pressure_p + o1), pp2 = ld2(p.pressure_p + o2), zz1 = ld2(p.zz + o1), zz2 = ld2(p.zz + o2);
  const d2 dpz1 = ld2(p.dpdz + o1), dpz2 = ld2(p.dpdz + o2), dv1 = ld2(p.divergence + o1), dv2 = ld2(p.divergence + o2);
  const d2 vo1 = ld2(p.vorticity + (size_t)v1 * K + 2 * lc), vo2 = ld2(p.vorticity + (size_t)v2 * K + 2 * lc);
  const d2 kd1 = ld2(p.kdiff + o1), kd2 = ld2(p.kdiff + o2);
  d2 tue = tue0;
  if (solve) {
    tue.x = -cqu.x * ((pp2.x - pp1.x) * invDc / (.5 * (zz2.x + zz1.x)) - 0.5 * zxu.x * (dpz1.x + dpz2.x));
    tue.y = -cqu.y * ((pp2.y - pp1.y) * invDc / (.5 * (zz2.y + zz1.y)) - 0.5 * zxu.y * (dpz1.y + dpz2.y));
  }
  const double r_dc = invDc;
  const double r_dv = fmin(invDv, 4 * invDc);
  d2 ud, out;
  ud.x = (dv2.x - dv1.x) * r_dc - (vo2.x - vo1.x) * r_dv;
  ud.y = (dv2.y - dv1.y) * r_dc - (vo2.y - vo1.y) * r_dv;
  out.x = tue.x + re.x * (0.5 * (kd1.x + kd2.x)) * ud.x * msd2;
  out.y = tue.y + re.y * (0.5 * (kd1.y + kd2.y)) * ud.y * msd2;
  if ((h == 0 || hasB) && 2 * l < K) {
    pst(p.delsq_u + o, d2{0.0 + ud.x, 0.0 + ud.y}, two);
    pst(p.tend_u_euler + o, out, two);
  }
}

// k_dyn_advflux_b in the pair layout
template <int NA, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_dyn_advflux_p(Dims d, Ptrs p) {
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1), lw = min(l, K / 2);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const size_t K1 = K + 1;
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int naA = p.nAdvCellsForEdge[eA], naB = p.nAdvCellsForEdge[eB];
  int ic[NA];
  double a[NA], b[NA];
  // (the rows through the scalar cache: as vector loads, ld_row, this kernel measured 368 -> 407 us
  // per call -- its 20 gathers per wave already fill the vector memory pipe)
  ld_row(p.advCellsForEdge + (size_t)e * 15, ic);
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    a[j] = sel(h, ld_uniform_f64(p.adv_coefs + (size_t)eA * 15 + j), ld_uniform_f64(p.adv_coefs + (size_t)eB * 15 + j));
    b[j] = sel(h, ld_uniform_f64(p.adv_coefs_3rd + (size_t)eA * 15 + j),
               ld_uniform_f64(p.adv_coefs_3rd + (size_t)eB * 15 + j));
  }
  const d2 rue = ld2(p.ru + o);
  const bool onA = ceA.x < d.nCellsSolve || ceA.y < d.nCellsSolve;
  const bool onB = hasB && (ceB.x < d.nCellsSolve || ceB.y < d.nCellsSolve);
  if (!onA && !onB) return;
  const bool wide = naA > NA || naB > NA;  // not produced by meshes with maxEdges <= 7
  d2 wv[NA], tv[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    wv[j] = ld2(p.w2 + (size_t)ic[j] * K1 + 2 * lw);
    tv[j] = ld2(p.theta_m2 + (size_t)ic[j] * K + 2 * lc);
  }
  const d2 fzm = ld2(p.fzm + 2 * lc), fzp = ld2(p.fzp + 2 * lc);
  const d2 rue_m = km1(rue, l);
  const int kx = 2 * l, ky = 2 * l + 1;
  const double rewx = kx < K ? fzm.x * rue.x + fzp.x * rue_m.x : 0.0;
  const double rewy = ky < K ? fzm.y * rue.y + fzp.y * rue_m.y : 0.0;
  const double swx = sgn1(rewx), swy = sgn1(rewy), stx_ = sgn1(rue.x), sty_ = sgn1(rue.y);
  const int na = sel(h, naA, naB);
  d2 fw{0.0, 0.0}, ft{0.0, 0.0};
  if (wide) {  // general path: every coefficient and neighbour read in the loop
    for (int j = 0; j < max(naA, naB); ++j) {
      if (j < na) {
        const int cj = p.advCellsForEdge[(size_t)e * 15 + j];
        const double aj = p.adv_coefs[(size_t)e * 15 + j], bj = p.adv_coefs_3rd[(size_t)e * 15 + j];
        const d2 w_ = ld2(p.w2 + (size_t)cj * K1 + 2 * lw), t_ = ld2(p.theta_m2 + (size_t)cj * K + 2 * lc);
        fw.x = fw.x + (aj + swx * bj) * w_.x;
        fw.y = fw.y + (aj + swy * bj) * w_.y;
        ft.x = ft.x + (aj + stx_ * bj) * t_.x;
        ft.y = ft.y + (aj + sty_ * bj) * t_.y;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    if (j < na && !wide) {
      fw.x = fw.x + (a[j] + swx * b[j]) * wv[j].x;
      fw.y = fw.y + (a[j] + swy * b[j]) * wv[j].y;
      ft.x = ft.x + (a[j] + stx_ * b[j]) * tv[j].x;
      ft.y = ft.y + (a[j] + sty_ * b[j]) * tv[j].y;
    }
  }
  if ((h ? onB : onA) && 2 * l < K) {
    pst(p.advflux_w + o, fw, two);
    pst(p.advflux_th + o, ft, two);
  }
}

// k_diag_vertices in the pair layout: two vertices per wavefront, two levels per lane (16-byte
// gathers of u at the three edges); same expressions in the same order
// uu_up: the u exchange's fused unpack (988, XUnpack with write-back vertices): a received halo edge's u
// comes from the receive buffer for every vertex that reads it, and its write-back vertex (uu_up.wb)
// stores it into uw (the field u names) for the later readers
template <bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_diag_vertices_p(Dims d, Ptrs p, const double* __restrict__ u,
                                                                  int store_dv, XUnpack uu_up = XUnpack{},
                                                                  double* uw = nullptr) {
  const int vA = PAIR_EPW * pair_wave();
  if (vA >= d.nVertices) return;
  const bool hasB = PAIR_EPW == 2 && vA + 1 < d.nVertices;
  const int vB = hasB ? vA + 1 : vA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int v = sel(h, vA, vB);
  int ei[3];
  double sd[3], ef[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int eA = p.edgesOnVertex[3 * vA + i], eB = p.edgesOnVertex[3 * vB + i];
    const double dcA = ld_uniform_f64(p.dcEdge + eA), dcB = ld_uniform_f64(p.dcEdge + eB);
    sd[i] = sel(h, ld_uniform_f64(p.edgesOnVertex_sign + 3 * vA + i) * dcA,
                ld_uniform_f64(p.edgesOnVertex_sign + 3 * vB + i) * dcB);
    ef[i] = sel(h, dcA * ld_uniform_f64(p.dvEdge + eA), dcB * ld_uniform_f64(p.dvEdge + eB));  // ke_edge_of
    ei[i] = sel(h, eA, eB);
  }
  d2 uu[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int of = rec_off(uu_up, 0, ei[i], d.nEdgesSolve);
    if (of >= 0) {
      uu[i] = ld2(uu_up.recv + of + 2 * lc);
      if (uu_up.wb[ei[i] - d.nEdgesSolve] == v && (h == 0 || hasB) && 2 * l < K)
        pst(uw + (size_t)ei[i] * K + 2 * lc, uu[i], two);
    } else {
      uu[i] = ld2(u + (size_t)ei[i] * K + 2 * lc);
    }
  }
  const double iat = sel(h, ld_uniform_f64(p.invAreaTriangle + vA), ld_uniform_f64(p.invAreaTriangle + vB));
  const double fv = sel(h, ld_uniform_f64(p.fVertex + vA), ld_uniform_f64(p.fVertex + vB));
  d2 vort{0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    vort.x = vort.x + sd[i] * uu[i].x;
    vort.y = vort.y + sd[i] * uu[i].y;
  }
  vort.x = vort.x * iat;
  vort.y = vort.y * iat;
  const double r = 0.25 * iat;
  d2 kev;
  kev.x = (ef[0] * (uu[0].x * uu[0].x) + ef[1] * (uu[1].x * uu[1].x) + ef[2] * (uu[2].x * uu[2].x)) * r;
  kev.y = (ef[0] * (uu[0].y * uu[0].y) + ef[1] * (uu[1].y * uu[1].y) + ef[2] * (uu[2].y * uu[2].y)) * r;
  if ((h == 0 || hasB) && 2 * l < K) {
    const size_t o = (size_t)v * K + 2 * lc;
    if (store_dv) pst(p.vorticity + o, vort, two);
    pst(p.ke_vertex + o, kev, two);
    pst(p.pv_vertex + o, d2{fv + vort.x, fv + vort.y}, two);
  }
}

// k_dyn_cells1_b in the pair layout: two cells per wavefront, two levels per lane (16-byte gathers
// of ru, and for the Smagorinsky kdiff of u and v, at the cell's edges); same expressions in the
// same order.  rw has K+1 levels: with an even K its lanes run one further than the K-level fields'
// (level K, which the top level's rw(k+1) reads).
template <int ME, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_dyn_cells1_p(Dims d, Ptrs p, Config cf, DynTendScal s) {
  const int cA = PAIR_EPW * pair_wave();
  if (cA >= d.nCells) return;
  const bool hasB = PAIR_EPW == 2 && cA + 1 < d.nCells;
  const int cB = hasB ? cA + 1 : cA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const int lw = ODD ? lc : min(l, K / 2);  // rw: levels 0..K
  const bool two = !ODD || 2 * l + 1 < K;   // odd K: the last pair holds level K-1 only
  const int c = sel(h, cA, cB);
  const size_t o = (size_t)c * K + 2 * lc;
  const bool rk1 = s.rk_step == 1, smag = rk1 && cf.horiz_mixing_smag;
  const CellSten<ME> sA = load_sten<ME>(p, cA), sB = load_sten<ME>(p, cB);
  const int ne = sel(h, sA.ne, sB.ne);
  double sdv[ME], da[ME], db[ME];
  int ei[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    sdv[i] = sel(h, ld_uniform_f64(p.cell_sdv + (size_t)cA * ME + i), ld_uniform_f64(p.cell_sdv + (size_t)cB * ME + i));
    da[i] = smag ? sel(h, ld_uniform_f64(p.defc_a + (size_t)cA * ME + i), ld_uniform_f64(p.defc_a + (size_t)cB * ME + i)) : 0.0;
    db[i] = smag ? sel(h, ld_uniform_f64(p.defc_b + (size_t)cA * ME + i), ld_uniform_f64(p.defc_b + (size_t)cB * ME + i)) : 0.0;
    ei[i] = sel(h, sA.e[i], sB.e[i]);
  }
  const double invA = sel(h, ld_uniform_f64(p.invAreaCell + cA), ld_uniform_f64(p.invAreaCell + cB));
  d2 rwk{0.0, 0.0}, qt{0.0, 0.0}, rb{0.0, 0.0}, rps{0.0, 0.0};
  if (rk1) {
    rwk = ld2(p.rw + (size_t)c * (K + 1) + 2 * lw);
    qt = ld2(p.qtot + o);
    rb = ld2(p.rho_base + o);
    rps = ld2(p.rho_p_save + o);
  }
  d2 rue[ME], ue[ME], ve[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const size_t oe = (size_t)ei[i] * K + 2 * lc;
    rue[i] = ld2(p.ru + oe);
    ue[i] = smag ? ld2(p.u2 + oe) : d2{0.0, 0.0};
    ve[i] = smag ? ld2(p.v + oe) : d2{0.0, 0.0};
  }
  const bool st = (h == 0 || hasB) && 2 * l < K;
  // 2d Smagorinsky kdiff + cam filter (rk1, 4677-4720)
  if (rk1) {
    d2 kd;
    if (smag) {
      d2 dd{0.0, 0.0}, df{0.0, 0.0};
#pragma unroll
      for (int i = 0; i < ME; ++i) {
        if (i < ne) {
          dd.x = dd.x + da[i] * ue[i].x - db[i] * ve[i].x;
          df.x = df.x + db[i] * ue[i].x + da[i] * ve[i].x;
          dd.y = dd.y + da[i] * ue[i].y - db[i] * ve[i].y;
          df.y = df.y + db[i] * ue[i].y + da[i] * ve[i].y;
        }
      }
      const double csl = s.c_s * cf.len_disp;
      const double cap = (0.01 * (cf.len_disp * cf.len_disp)) * s.invDt;
      kd.x = fmin((csl * csl) * sqrt(dd.x * dd.x + df.x * df.x), cap);
      kd.y = fmin((csl * csl) * sqrt(dd.y * dd.y + df.y * df.y), cap);
    } else {
      kd = d2{cf.h_theta_eddy_visc2, cf.h_theta_eddy_visc2};
    }
    if (cf.mpas_cam_coef > 0.0) {
      const int k0 = 2 * l, k1 = 2 * l + 1;
      const double c3 = 2.0833 * cf.len_disp * cf.mpas_cam_coef, c2 = 2.0 * 2.0833 * cf.len_disp * cf.mpas_cam_coef,
                   c1 = 4.0 * 2.0833 * cf.len_disp * cf.mpas_cam_coef;
      if (k0 == K - 3) kd.x = fmax(kd.x, c3);
      if (k0 == K - 2) kd.x = fmax(kd.x, c2);
      if (k0 == K - 1) kd.x = fmax(kd.x, c1);
      if (k1 == K - 3) kd.y = fmax(kd.y, c3);
      if (k1 == K - 2) kd.y = fmax(kd.y, c2);
      if (k1 == K - 1) kd.y = fmax(kd.y, c1);
    }
    if (st) pst(p.kdiff + o, kd, two);
  }
  // h_divergence (4729-4748)
  d2 hd{0.0, 0.0};
#pragma unroll
  for (int i = 0; i < ME; ++i)
    if (i < ne) {  // edgesOnCell_sign * dvEdge * ru
      hd.x = hd.x + sdv[i] * rue[i].x;
      hd.y = hd.y + sdv[i] * rue[i].y;
    }
  hd.x = hd.x * invA;
  hd.y = hd.y * invA;
  if (st) pst(p.h_divergence + o, hd, two);
  // tend_rho and dpdz (rk1, 4755-4766)
  if (rk1) {
    const d2 rwp = kp1(rwk);
    const d2 rz = ld2(p.rdzw + 2 * lc);
    d2 tr, dz;
    tr.x = -hd.x - rz.x * (rwp.x - rwk.x) + PHYS(p.tend_rho_physics, o);
    tr.y = -hd.y - rz.y * (rwp.y - rwk.y) + PHYS(p.tend_rho_physics, o + 1);
    dz.x = -GRAVITY * (rb.x * (qt.x) + rps.x * (1. + qt.x));
    dz.y = -GRAVITY * (rb.y * (qt.y) + rps.y * (1. + qt.y));
    if (st) {
      pst(p.tend_rho + o, tr, two);
      pst(p.dpdz + o, dz, two);
    }
  }
}

// k_dyn_cells2_b in the pair layout: two cells per wavefront, two levels per lane (16-byte gathers
// of rho_edge at the cell's edges and of kdiff, w, theta_m at its neighbours); same expressions in the
// same order.  Level 0 of delsq_w / tend_w_euler is 0 (the w fluxes start at level 1) and level K of
// tend_w_euler is 0, as there.
template <int ME, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_dyn_cells2_p(Dims d, Ptrs p) {
  const int cA = PAIR_EPW * pair_wave();
  if (cA >= d.nCells) return;
  const bool hasB = PAIR_EPW == 2 && cA + 1 < d.nCells;
  const int cB = hasB ? cA + 1 : cA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int c = sel(h, cA, cB);
  const size_t K1 = K + 1;
  const CellSten<ME> sA = load_sten<ME>(p, cA), sB = load_sten<ME>(p, cB);
  const double rA = ld_uniform_f64(p.invAreaCell + cA), rB = ld_uniform_f64(p.invAreaCell + cB);
  const double prandtl_inv = 1.0 / PRANDTL;
  const int ne = sel(h, sA.ne, sB.ne);
  double est[ME], msd[ME];
  int eo[ME], co[ME];
  bool fi[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const int eA = sA.e[i], eB = sB.e[i];
    const double sdA = ld_uniform_f64(p.cell_sdv + (size_t)cA * ME + i), sdB = ld_uniform_f64(p.cell_sdv + (size_t)cB * ME + i);
    const double idA = ld_uniform_f64(p.invDcEdge + eA), idB = ld_uniform_f64(p.invDcEdge + eB);
    const double mA = ld_uniform_f64(p.meshScalingDel2 + eA), mB = ld_uniform_f64(p.meshScalingDel2 + eB);
    // r_areaCell*sign*dvEdge*invDcEdge; the w fluxes' 0.5*r_areaCell*... is 0.5 times it exactly (a
    // power-of-two factor: ((0.5 r) s) i and 0.5 ((r s) i) round alike)
    est[i] = sel(h, rA * sdA * idA, rB * sdB * idB);
    msd[i] = sel(h, mA, mB);
    eo[i] = sel(h, eA, eB);
    co[i] = sel(h, sA.o[i], sB.o[i]);
    fi[i] = h ? sB.first(i) : sA.first(i);
  }
  const d2 kds = ld2(p.kdiff + (size_t)c * K + 2 * lc), ws = ld2(p.w2 + (size_t)c * K1 + 2 * lc),
           ths = ld2(p.theta_m2 + (size_t)c * K + 2 * lc);
  // two passes (the w fluxes, then the theta fluxes, each summed in edge order as there): theta_m's
  // gathers are issued after the w pass (fewer live registers: 138 VGPRs against 160 in one pass)
  d2 re[ME], kdo[ME], wo[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    re[i] = ld2(p.rho_edge + (size_t)eo[i] * K + 2 * lc);
    kdo[i] = ld2(p.kdiff + (size_t)co[i] * K + 2 * lc);
    wo[i] = ld2(p.w2 + (size_t)co[i] * K1 + 2 * lc);
  }
  d2 dw{0.0, 0.0}, tw{0.0, 0.0}, dth{0.0, 0.0}, tth{0.0, 0.0};
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    // cellsOnEdge(1/2) of edge i: this cell and the one across, in the edge's order
    const bool f = fi[i];
    const d2 kd1 = f ? kds : kdo[i], kd2 = f ? kdo[i] : kds;
    const d2 w1 = f ? ws : wo[i], w2 = f ? wo[i] : ws;
    const d2 re_m = km1(re[i], l), kd1m = km1(kd1, l), kd2m = km1(kd2, l);
    if (i < ne) {
      const double esw = 0.5 * est[i];
      double wtf = esw * (re[i].x + re_m.x) * (w2.x - w1.x);
      dw.x = dw.x + wtf;
      wtf = wtf * msd[i] * 0.25 * (kd1.x + kd2.x + kd1m.x + kd2m.x);
      tw.x = tw.x + wtf;
      wtf = esw * (re[i].y + re_m.y) * (w2.y - w1.y);
      dw.y = dw.y + wtf;
      wtf = wtf * msd[i] * 0.25 * (kd1.y + kd2.y + kd1m.y + kd2m.y);
      tw.y = tw.y + wtf;
    }
  }
  d2 tho[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) tho[i] = ld2(p.theta_m2 + (size_t)co[i] * K + 2 * lc);
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const bool f = fi[i];
    const d2 kd1 = f ? kds : kdo[i], kd2 = f ? kdo[i] : kds;
    const d2 t1 = f ? ths : tho[i], t2 = f ? tho[i] : ths;
    if (i < ne) {
      const double prs = prandtl_inv * msd[i];
      double ttf = est[i] * (t2.x - t1.x) * re[i].x;
      dth.x = dth.x + ttf;
      ttf = ttf * 0.5 * (kd1.x + kd2.x) * prs;
      tth.x = tth.x + ttf;
      ttf = est[i] * (t2.y - t1.y) * re[i].y;
      dth.y = dth.y + ttf;
      ttf = ttf * 0.5 * (kd1.y + kd2.y) * prs;
      tth.y = tth.y + ttf;
    }
  }
  if (!(h == 0 || hasB)) return;
  if (l == 0) {  // level 0: no w flux
    dw.x = 0.0;
    tw.x = 0.0;
  }
  if (2 * l < K) {
    const size_t o = (size_t)c * K + 2 * lc;
    pst(p.delsq_w + o, dw, two);
    pst(p.delsq_theta + o, dth, two);
    pst(p.tend_theta_euler + o, tth, two);
  }
  if (2 * l <= K) {  // tend_w_euler, levels 0..K (level K: 0)
    double* tw_out = p.tend_w_euler + (size_t)c * K1 + 2 * l;
    const double x = 2 * l < K ? tw.x : 0.0;
    if (2 * l + 1 <= K) st2(tw_out, d2{x, 2 * l + 1 < K ? tw.y : 0.0});
    else tw_out[0] = x;
  }
}

// k_dyn_delsq_vc_b in the pair layout: each group of three wavefronts holds 2 PAIR_EPW vertices
// (two wavefronts) and PAIR_EPW cells (one), the vertices 2c, 2c+1 next to cell c as there; two
// levels per lane, 16-byte gathers of delsq_u; same expressions in the same order.  Launch over
// PAIR_EPW * 3 * max(ceil(nVertices / (2 PAIR_EPW)), ceil(nCells / PAIR_EPW)) elements.
template <int ME, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_dyn_delsq_vc_p(Dims d, Ptrs p) {
  const int wv = pair_wave();
  const int j3 = wv / 3, t3 = wv - 3 * j3;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  if (t3 < 2) {
    const int vA = PAIR_EPW * (2 * j3 + t3);
    if (vA >= d.nVertices) return;
    const bool hasB = PAIR_EPW == 2 && vA + 1 < d.nVertices;
    const int vB = hasB ? vA + 1 : vA;
    const int v = sel(h, vA, vB);
    int ei[3];
    double cf[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int eA = p.edgesOnVertex[3 * vA + i], eB = p.edgesOnVertex[3 * vB + i];
      // iat * dc * sg, left to right as k_dyn_delsq_vc_b
      const double cA = ld_uniform_f64(p.invAreaTriangle + vA) * ld_uniform_f64(p.dcEdge + eA) *
                        ld_uniform_f64(p.edgesOnVertex_sign + 3 * vA + i);
      const double cB = ld_uniform_f64(p.invAreaTriangle + vB) * ld_uniform_f64(p.dcEdge + eB) *
                        ld_uniform_f64(p.edgesOnVertex_sign + 3 * vB + i);
      cf[i] = sel(h, cA, cB);
      ei[i] = sel(h, eA, eB);
    }
    d2 du[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) du[i] = ld2(p.delsq_u + (size_t)ei[i] * K + 2 * lc);
    d2 dv{0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      dv.x = dv.x + cf[i] * du[i].x;
      dv.y = dv.y + cf[i] * du[i].y;
    }
    if ((h == 0 || hasB) && 2 * l < K) pst(p.delsq_vorticity + (size_t)v * K + 2 * lc, dv, two);
  } else {
    const int cA = PAIR_EPW * j3;
    if (cA >= d.nCells) return;
    const bool hasB = PAIR_EPW == 2 && cA + 1 < d.nCells;
    const int cB = hasB ? cA + 1 : cA;
    const int c = sel(h, cA, cB);
    const CellSten<ME> sA = load_sten<ME>(p, cA), sB = load_sten<ME>(p, cB);
    const double rA = ld_uniform_f64(p.invAreaCell + cA), rB = ld_uniform_f64(p.invAreaCell + cB);
    const int ne = sel(h, sA.ne, sB.ne);
    double cf[ME];
    int ei[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      // r * dvEdge * edgesOnCell_sign (cell_sdv), as k_dyn_delsq_vc_b
      cf[i] = sel(h, rA * ld_uniform_f64(p.cell_sdv + (size_t)cA * ME + i), rB * ld_uniform_f64(p.cell_sdv + (size_t)cB * ME + i));
      ei[i] = sel(h, sA.e[i], sB.e[i]);
    }
    d2 du[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) du[i] = ld2(p.delsq_u + (size_t)ei[i] * K + 2 * lc);
    d2 dd{0.0, 0.0};
#pragma unroll
    for (int i = 0; i < ME; ++i)
      if (i < ne) {
        dd.x = dd.x + cf[i] * du[i].x;
        dd.y = dd.y + cf[i] * du[i].y;
      }
    if ((h == 0 || hasB) && 2 * l < K) pst(p.delsq_divergence + (size_t)c * K + 2 * lc, dd, two);
  }
}

// k_diag_edges_b in the pair layout
template <int NE2, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_diag_edges_p(Dims d, Ptrs p, const double* __restrict__ u,
                                                               const double* __restrict__ hh, int reconstruct_v,
                                                               double apvm, double dt, int store_grad) {
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int2 veA = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eA);
  const int2 veB = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * eB);
  int neoe = 0;
  int eoe[NE2];
  double wgt[NE2];
  if (reconstruct_v) {
    neoe = sel(h, p.nEdgesOnEdge[eA], p.nEdgesOnEdge[eB]);
    // (through the scalar cache: as vector loads, ld_row, 285 -> 288-294 us per call)
#pragma unroll
    for (int j = 0; j < NE2; ++j) {
      eoe[j] = sel(h, p.edgesOnEdge[(size_t)eA * d.maxEdges2 + j], p.edgesOnEdge[(size_t)eB * d.maxEdges2 + j]);
      wgt[j] = sel(h, ld_uniform_f64(p.weightsOnEdge + (size_t)eA * d.maxEdges2 + j),
                   ld_uniform_f64(p.weightsOnEdge + (size_t)eB * d.maxEdges2 + j));
    }
  }
  double invDv = 0.0, invDc = 0.0;
  d2 ue{};
  if (apvm > 0.0) {
    invDv = sel(h, ld_uniform_f64(p.invDvEdge + eA), ld_uniform_f64(p.invDvEdge + eB));
    invDc = sel(h, ld_uniform_f64(p.invDcEdge + eA), ld_uniform_f64(p.invDcEdge + eB));
    ue = ld2(u + o);
  }
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y), v1 = sel(h, veA.x, veB.x), v2 = sel(h, veA.y, veB.y);
  const d2 h1 = ld2(hh + (size_t)c1 * K + 2 * lc), h2 = ld2(hh + (size_t)c2 * K + 2 * lc);
  const d2 pv1 = ld2(p.pv_vertex + (size_t)v1 * K + 2 * lc), pv2 = ld2(p.pv_vertex + (size_t)v2 * K + 2 * lc);
  d2 pc1{}, pc2{};
  if (apvm > 0.0) {
    pc1 = ld2(p.pv_cell + (size_t)c1 * K + 2 * lc);
    pc2 = ld2(p.pv_cell + (size_t)c2 * K + 2 * lc);
  }
  const bool st = (h == 0 || hasB) && 2 * l < K;
  d2 vv;
  if (reconstruct_v) {
    d2 uu[NE2];
#pragma unroll
    for (int j = 0; j < NE2; ++j) uu[j] = ld2(u + (size_t)eoe[j] * K + 2 * lc);
    vv = d2{0.0, 0.0};
#pragma unroll
    for (int j = 0; j < NE2; ++j) {
      if (j < neoe) {
        vv.x = vv.x + wgt[j] * uu[j].x;
        vv.y = vv.y + wgt[j] * uu[j].y;
      }
    }
    if (st) pst(p.v + o, vv, two);
  } else {
    vv = ld2(p.v + o);
  }
  if (st) pst(p.rho_edge + o, d2{0.5 * (h1.x + h2.x), 0.5 * (h1.y + h2.y)}, two);
  d2 pve{0.5 * (pv1.x + pv2.x), 0.5 * (pv1.y + pv2.y)};
  if (apvm > 0.0) {
    const double r = apvm * dt;
    const double r1 = 1.0 * invDv;
    const double r2 = 1.0 * invDc;
    const d2 gt{(pv2.x - pv1.x) * r1, (pv2.y - pv1.y) * r1};
    const d2 gn{(pc2.x - pc1.x) * r2, (pc2.y - pc1.y) * r2};
    if (st && store_grad) {
      pst(p.gradPVt + o, gt, two);
      pst(p.gradPVn + o, gn, two);
    }
    pve.x = pve.x - r * (vv.x * gt.x + ue.x * gn.x);
    pve.y = pve.y - r * (vv.y * gt.y + ue.y * gn.y);
  }
  if (st) pst(p.pv_edge + o, pve, two);
}

// k_divdamp in the pair layout
// fresh = 1: the stage has one sub-step, whose edge phase srk3 does not launch, so ru_p enters as
// dts * tend_u and ruAvg (= the same value, 794-837 with small_step = 1) is stored here.
// REC: the stage's last damping also recovers the edges with two owned cells (recover_edges,
// 3048-3059): their rho_zz at both cells was recovered by the last cell phase
// (k_acoustic_cells_r<ME, true>), and nothing between here and k_recover_edges -- the 876-887
// exchange, k_recover_cells1 on halo cells -- touches ru_save, ruAvg, ru or u there.
// k_recover_edges then runs on the other edges (phase 2).
// two levels (2*lc, 2*lc+1) of cell c's rtheta_pp (which = 0) or rho_pp (1) column: from the
// exchange's receive buffer for a halo cell the fused unpack covers -- written back into the field,
// lanes `st` only, for the later readers -- else from the field
template <bool ODD>
__device__ __forceinline__ d2 ld_pp(const Dims& d, const Ptrs& p, const UnpackMap& um, int which, int c, int lc,
                                    bool st) {
  double* fld = which ? p.rho_pp : p.rtheta_pp;
  const size_t o = (size_t)c * d.K + 2 * lc;
  const int* map = which ? um.rho : um.rt;
  if (map && c >= d.nCellsSolve && c < d.nCells) {
    const int off = map[c - d.nCellsSolve];
    if (off >= 0) {
      const d2 v = ld2(um.recv + off + 2 * lc);
      if (st) pst(fld + o, v, !ODD || 2 * lc + 1 < d.K);
      return v;
    }
  }
  return ld2(fld + o);
}

// dl = 1: rtheta_pp_old holds rtheta_pp - rtheta_pp_old (k_acoustic_cells_r<ME, true> with dl)
// rp: the stage's last damping also packs ru_p of the 876-887 exchange (XPack), or nothing
template <bool REC = false, bool UP = false, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_divdamp_p(Dims d, Ptrs p, double coef_divdamp, int phase, double dts,
                                                            int fresh, double invNs = 0.0, UnpackMap um = UnpackMap{},
                                                            int dl = 0, XPack rp = XPack{}, XPack upk = XPack{}) {
  int eA, eB;
  bool hasB;
  if (!pair_edges(d, p, phase, eA, eB, hasB)) return;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int bA = phase ? p.edge_bnd[eA] : 0, bB = phase ? p.edge_bnd[eB] : 0;
  d2 ru;
  if (fresh) {
    const d2 tu = ld2(p.tend_u + o);
    ru = d2{dts * tu.x, dts * tu.y};
  } else {
    ru = ld2(p.ru_p + o);
  }
  const double mask = sel(h, ld_uniform_f64(p.specZoneMaskEdge + eA), ld_uniform_f64(p.specZoneMaskEdge + eB));
  auto active = [&](int2 ce, int bnd) {
    return (ce.x < d.nCellsSolve || ce.y < d.nCellsSolve) && (phase == 0 || ((bnd != 0) == (phase == 2)));
  };
  const bool onA = active(ceA, bA), onB = hasB && active(ceB, bB);
  if (!onA && !onB) return;
  const size_t o1 = (size_t)sel(h, ceA.x, ceB.x) * K + 2 * lc, o2 = (size_t)sel(h, ceA.y, ceB.y) * K + 2 * lc;
  const bool lv = 2 * l < K && (h ? onB : onA);
  d2 dd1, dd2;  // rtheta_pp - rtheta_pp_old at the two cells
  if (dl) {
    dd1 = ld2(p.rtheta_pp_old + o1);
    dd2 = ld2(p.rtheta_pp_old + o2);
  } else {
    const d2 r1 = UP ? ld_pp<ODD>(d, p, um, 0, sel(h, ceA.x, ceB.x), lc, lv) : ld2(p.rtheta_pp + o1);
    const d2 r2 = UP ? ld_pp<ODD>(d, p, um, 0, sel(h, ceA.y, ceB.y), lc, lv) : ld2(p.rtheta_pp + o2);
    const d2 q1 = ld2(p.rtheta_pp_old + o1), q2 = ld2(p.rtheta_pp_old + o2);
    dd1 = d2{r1.x - q1.x, r1.y - q1.y};
    dd2 = d2{r2.x - q2.x, r2.y - q2.y};
  }
  const d2 t1 = ld2(p.theta_m1 + o1), t2 = ld2(p.theta_m1 + o2);
  d2 out;
  out.x = ru.x + coef_divdamp * (-(dd2.x) - -(dd1.x)) * (1.0 - mask) / (t1.x + t2.x);
  out.y = ru.y + coef_divdamp * (-(dd2.y) - -(dd1.y)) * (1.0 - mask) / (t1.y + t2.y);
  pack_rec_edge(rp, d, eA, eB, hasB, h, lc, (h ? onB : onA) && 2 * l < K, two, out);
  if (!REC) {
    if ((h ? onB : onA) && 2 * l < K) {
      pst(p.ru_p + o, out, two);
      if (fresh) pst(p.ruAvg + o, ru, two);
    }
    return;
  }
  const bool rA = onA && (phase ? bA : p.edge_bnd[eA]) == 0;  // edges with two owned cells
  const bool rB = onB && (phase ? bB : p.edge_bnd[eB]) == 0;
  const d2 rs = ld2(p.ru_save + o);
  const d2 ra = fresh ? ru : ld2(p.ruAvg + o);  // fresh: sub-step 1 left ruAvg = dts * tend_u
  const d2 z1 = ld2(p.rho_zz2 + o1), z2 = ld2(p.rho_zz2 + o2);
  const d2 rr{rs.x + out.x, rs.y + out.y};
  const d2 un{2. * rr.x / (z1.x + z2.x), 2. * rr.y / (z1.y + z2.y)};
  if ((h ? onB : onA) && 2 * l < K) {
    // dl (one block, not the dt's last stage, see damping_delta): nothing reads ru_p of a
    // recovered edge before the next stage's sub-step 1 forms it again from tend_u, so only the
    // edges k_recover_edges still recovers from it get it stored
    if (!(dl && (h ? rB : rA))) pst(p.ru_p + o, out, two);
    if (h ? rB : rA) {  // recover_edges (3048-3059), same expressions
      pst(p.ruAvg + o, d2{rs.x + (ra.x * invNs), rs.y + (ra.y * invNs)}, two);
      pst(p.ru + o, rr, two);
      pst(p.u2 + o, un, two);
    } else if (fresh) {
      pst(p.ruAvg + o, ru, two);
    }
  }
  // the recovered u of an owned edge into its slots of the u exchange (988) when fused
  pack_rec_edge(upk, d, eA, eB, hasB, h, lc, (h ? onB : onA) && (h ? rB : rA) && 2 * l < K, two, un);
}

// k_scalars_edges in the pair layout (atm_advance_scalars_work, 3357-3426)
// VROW: the stencil rows as vector loads (ld_row) -- one scalar: 338 -> 278 us per call; with the
// six moist species in the scalar loop the scalar-cache rows are faster (854 vs 944 us)
template <int NA, bool ODD = false, bool VROW = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_scalars_edges_p(Dims d, Ptrs p) {
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane(), ns = d.ns;
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int na = sel(h, p.nAdvCellsForEdge[eA], p.nAdvCellsForEdge[eB]);
  // VROW (one scalar): the weights a + b and a - b of the wave's two edges in LDS, one row per
  // half-wave (the two values a + sgn(u) b takes: sgn is +-1, so the sum is the same either way), read
  // as half-wave broadcasts in the sums, as in k_mono_edges1_p: the two rows no longer take 40 VGPRs
  // (108 -> 84), 35.86-36.03 -> 35.68-35.88 ms per dt.  With six scalars the scalar-cache rows stay
  // (the LDS rows measured no faster there, 42.23-42.26 against 42.26-42.37 ms per dt).
  __shared__ d2 wts[PAIR_WPB][PAIR_EPW][NA];
  d2 (&w)[NA] = wts[threadIdx.x >> 6][h];
  int ic[NA];
  double a[NA], b[NA];
  if constexpr (VROW) {
    if (l < NA) {
      const double aa = p.adv_coefs[(size_t)e * 15 + l], bb = p.adv_coefs_3rd[(size_t)e * 15 + l];
      w[l] = d2{aa + bb, aa - bb};
    }
    ld_row(p.advCellsForEdge + (size_t)e * 15, ic);
  } else {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      ic[j] = sel(h, p.advCellsForEdge[(size_t)eA * 15 + j], p.advCellsForEdge[(size_t)eB * 15 + j]);
      a[j] = sel(h, ld_uniform_f64(p.adv_coefs + (size_t)eA * 15 + j), ld_uniform_f64(p.adv_coefs + (size_t)eB * 15 + j));
      b[j] = sel(h, ld_uniform_f64(p.adv_coefs_3rd + (size_t)eA * 15 + j),
                 ld_uniform_f64(p.adv_coefs_3rd + (size_t)eB * 15 + j));
    }
  }
  // the weight of stencil cell j at the lane's two levels: w[j] picked by the sign, or a + sgn b
  auto wt = [&](int j, double sg, bool pos) -> double {
    if constexpr (VROW) {
      const d2 wj = w[j];
      return pos ? wj.x : wj.y;
    } else {
      return a[j] + sg * b[j];
    }
  };
  const d2 uh = ld2(p.ruAvg + o);
  const double sgx = sgn1(uh.x), sgy = sgn1(uh.y);
  const bool px = sgx > 0.0, py = sgy > 0.0;
  if constexpr (VROW) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const bool hex = na == 10;  // the reference's unrolled hexagon form (3363-3390)
  bool st = (h == 0 || hasB) && 2 * l < K;
  // regional: edges of the two outer relaxation rows take a first-order upwind flux, and
  // specified-zone edges keep the array's previous values (3359, 3409-3420)
  const int bm = d.lbc ? sel(h, p.bdyMaskEdge[eA], p.bdyMaskEdge[eB]) : 0;
  if (bm >= N_RELAX_ZONE - 1) {
    if (bm > N_RELAX_ZONE) return;
    const double dv = sel(h, ld_uniform_f64(p.dvEdge + eA), ld_uniform_f64(p.dvEdge + eB));
    const int c1 = sel(h, p.cellsOnEdge[2 * eA], p.cellsOnEdge[2 * eB]);
    const int c2 = sel(h, p.cellsOnEdge[2 * eA + 1], p.cellsOnEdge[2 * eB + 1]);
    const double udx = copysign(0.5, uh.x), udy = copysign(0.5, uh.y);
    const d2 upos{dv * fabs(udx + 0.5), dv * fabs(udy + 0.5)}, uneg{dv * fabs(udx - 0.5), dv * fabs(udy - 0.5)};
    for (int is = 0; is < ns; ++is) {
      const d2 s1 = ld2(p.scalars2 + SIX(c1, 2 * lc, is)), s2 = ld2(p.scalars2 + SIX(c2, 2 * lc, is));
      if (st) pst(p.horiz_flux_array + HIX(e, 2 * lc, is), d2{upos.x * s1.x + uneg.x * s2.x, upos.y * s1.y + uneg.y * s2.y}, two);
    }
    return;
  }
  for (int is = 0; is < ns; ++is) {
    d2 sv[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) sv[j] = ld2(p.scalars2 + SIX(ic[j], 2 * lc, is));
    d2 acc{0.0, 0.0};
    if (hex) {
      acc.x = wt(0, sgx, px) * sv[0].x;
      acc.y = wt(0, sgy, py) * sv[0].y;
#pragma unroll
      for (int j = 1; j < 10 && j < NA; ++j) {
        acc.x = acc.x + wt(j, sgx, px) * sv[j].x;
        acc.y = acc.y + wt(j, sgy, py) * sv[j].y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        if (j < na) {
          acc.x = acc.x + wt(j, sgx, px) * sv[j].x;
          acc.y = acc.y + wt(j, sgy, py) * sv[j].y;
        }
      }
    }
    if (st) pst(p.horiz_flux_array + HIX(e, 2 * lc, is), acc, two);
  }
}

// k_moist_edges in the pair layout (two edges per wave, two levels per lane): the 2 x (moist species)
// column gathers as 16-byte loads, the sum over the species in the same order (1920-1926)
template <bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_moist_edges_p(Dims d, Ptrs p) {
  int eA, eB;
  bool hasB;
  if (!pair_edges(d, p, 0, eA, eB, hasB)) return;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const bool on = (c1 < d.nCellsSolve || c2 < d.nCellsSolve) && (h == 0 || hasB);
  d2 q{0.0, 0.0};
  for (int iq = d.moist_start; iq <= d.moist_end; ++iq) {
    const d2 s1 = ld2(p.scalars2 + SIX(c1, 2 * lc, iq)), s2 = ld2(p.scalars2 + SIX(c2, 2 * lc, iq));
    q.x = q.x + 0.5 * (s1.x + s2.x);
    q.y = q.y + 0.5 * (s1.y + s2.y);
  }
  if (on && 2 * l < K) pst(p.cqu + (size_t)e * K + 2 * lc, d2{1.0 / (1.0 + q.x), 1.0 / (1.0 + q.y)}, two);
}

// (a two-scalar variant -- both scalars' gathers from one pass over the stencil indices and
// coefficients -- needs 197 VGPRs, runs 2 waves per SIMD instead of 4 and took exactly the time
// of two launches: the in-flight gathers per SIMD, not the index loads, bound this kernel)
// k_mono_edges1 in the pair layout (atm_advance_scalars_mono_work, 3916-3961, 4007-4022)
// the second scratch set's edge fluxes (mono_slot1) for the pair's second scalar
struct MonoFlux2 {
  double *flux_arr, *flux_upwind_tmp, *flux_tmp;
};
template <int NA, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_mono_edges1_p(Dims d, Ptrs p, int is, double dt, int nq = 1,
                                                                MonoFlux2 f2 = MonoFlux2{}) {
  // the stencil weights of the wave's two edges, a + b and a - b (the two values a + sgn(u) b takes),
  // in LDS: one row per half-wave, written by its first NA lanes and read as half-wave broadcasts
  // where the sums use them.  Held in registers, the two rows took 40 VGPRs for the whole kernel
  // (146 VGPRs, 3 waves per SIMD).
  __shared__ d2 wts[PAIR_WPB][PAIR_EPW][NA];
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane(), ns = d.ns;
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int na = sel(h, p.nAdvCellsForEdge[eA], p.nAdvCellsForEdge[eB]);
  d2 (&w)[NA] = wts[threadIdx.x >> 6][h];
  if (l < NA) {
    const double a = p.adv_coefs[(size_t)e * 15 + l], b = p.adv_coefs_3rd[(size_t)e * 15 + l];
    w[l] = d2{a + b, a - b};
  }
  int ic[NA];
  ld_row(p.advCellsForEdge + (size_t)e * 15, ic);
  const double dv = sel(h, ld_uniform_f64(p.dvEdge + eA), ld_uniform_f64(p.dvEdge + eB));
  const d2 uh = ld2(p.ruAvg + o);
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const bool on = c1 < d.nCellsSolve || c2 < d.nCellsSolve;
  // 4017-4020 (operator precedence as written: (apply_lbcs .and. mask == 5) .or. mask == 4): the
  // two outer relaxation rows keep only the upwind flux
  const int bm = sel(h, p.bdyMaskEdge[eA], p.bdyMaskEdge[eB]);
  const bool upw = (d.lbc && bm == N_RELAX_ZONE) || bm == N_RELAX_ZONE - 1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // nq = 2: the pair's second scalar (is + 1) from the same rows, into the second scratch set
  // (f2), one after the other -- each scalar's operations as in its own launch
#pragma unroll 1
  for (int q = 0; q < nq; ++q) {
    const int iq = is + q;
    // scalars outside the block (the garbage slot) read as 0, as the reference's halo loops see them
    auto val = [&](const double* arr, int cc) {
      const d2 v = ld2(arr + SIX(cc, 2 * lc, iq));
      return cc < d.nCells ? v : d2{0.0, 0.0};
    };
    d2 sv[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) sv[j] = val(p.scalars2, ic[j]);
    const d2 so1 = val(p.scalars1, c1), so2 = val(p.scalars1, c2);
    d2 fa{0.0, 0.0};
    if (on) {
      if (na == 10) {
        // sum_j (a_j +- b_j) q_j, then times u (the reference's 10-cell tree)
        const bool upx = uh.x > 0, upy = uh.y > 0;
        double ax = 0.0, ay = 0.0;
#pragma unroll
        for (int j = 0; j < 10 && j < NA; ++j) {
          const d2 wj = w[j];
          const double tx = (upx ? wj.x : wj.y) * sv[j].x, ty = (upy ? wj.x : wj.y) * sv[j].y;
          ax = (j == 0) ? tx : ax + tx;
          ay = (j == 0) ? ty : ay + ty;
        }
        fa = d2{uh.x * ax, uh.y * ay};
      } else {
        // sum_j u (a_j + sgn(u) b_j) q_j over the edge's na cells
        const bool px = sgn1(uh.x) > 0.0, py = sgn1(uh.y) > 0.0;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          if (j < na) {
            const d2 wj = w[j];
            fa.x = fa.x + (uh.x * (px ? wj.x : wj.y)) * sv[j].x;
            fa.y = fa.y + (uh.y * (py ? wj.x : wj.y)) * sv[j].y;
          }
        }
      }
    }
    d2 fu;
    fu.x = dv * dt * (fmax(0.0, uh.x) * so1.x + fmin(0.0, uh.x) * so2.x);
    fu.y = dv * dt * (fmax(0.0, uh.y) * so1.y + fmin(0.0, uh.y) * so2.y);
    if ((h == 0 || hasB) && 2 * l < K) {
      pst((q ? f2.flux_arr : p.flux_arr) + o, upw ? fu : fa, two);
      pst((q ? f2.flux_upwind_tmp : p.flux_upwind_tmp) + o, fu, two);
      // flux_tmp (upw ? 0 : dt fa - fu) is not stored: k_mono_cells1_b, its only reader, forms it from
      // flux_arr and flux_upwind_tmp with the same operations (one edge array less written per scalar)
    }
  }
}

// atm_compute_vert_imp_coefs_work (2064-2129) in the pair layout: two owned cells per wave, two
// levels per lane.  The LU recurrence alpha(k) = 1/(b(k) - a(k) gamma(k-1)), gamma(k) = c(k) alpha(k)
// runs as a lane-shift sweep: each iteration finalizes one more lane (two levels, the second from
// the first in registers), K/2 iterations instead of K-1, each from exactly the operands of the
// sequential recurrence -- and a wave now carries two columns, halving the DP work per column.
template <bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_vert_imp_coefs_p(Dims d, Ptrs p, double dts, double epssm) {
  const int K = d.K, h = pair_half(), l = pair_lane();
  const double dtseps = .5 * dts * (1. + epssm);
  const double rcv = RGAS / (CP - RGAS);
  const double c2 = CP * rcv;
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)K) p.cofrz[threadIdx.x] = dtseps * p.rdzw[threadIdx.x];
  const int cA = PAIR_EPW * pair_wave();
  if (cA >= d.nCellsSolve) return;
  const bool hasB = PAIR_EPW == 2 && cA + 1 < d.nCellsSolve;
  const int c = sel(h, cA, hasB ? cA + 1 : cA);
  const bool mine = h == 0 || hasB;
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int kx = 2 * l, ky = 2 * l + 1;
  const bool ax = kx < K, ay = ky < K;  // "act" of the two levels
  const size_t o = (size_t)c * K + 2 * lc;
  auto LDP = [&](const double* a) {
    d2 v = ld2(a + o);
    return d2{ax ? v.x : 0.0, ay ? v.y : 0.0};
  };
  auto LD1 = [&](const double* a) {
    d2 v = ld2(a + 2 * lc);
    return d2{ax ? v.x : 0.0, ay ? v.y : 0.0};
  };
  const d2 zz = LDP(p.zz), pp = LDP(p.exner), t = LDP(p.theta_m2), rb = LDP(p.rho_base), rtb = LDP(p.rtheta_base);
  const d2 pb = LDP(p.exner_base), rt = LDP(p.rtheta_p), cqw = LDP(p.cqw), qtot = LDP(p.qtot);
  const d2 fzm = LD1(p.fzm), fzp = LD1(p.fzp), rdzu = LD1(p.rdzu), rdzw = LD1(p.rdzw);
  const d2 zzm = km1(zz, l), pm = km1(pp, l), tm = km1(t, l);
  d2 cofwr{0.0, 0.0}, cofwz{0.0, 0.0}, coftz{0.0, 0.0}, cofwt{0.0, 0.0};
  auto lev1 = [&](bool act, int k, double zz_, double zzm_, double pp_, double pm_, double t_, double tm_,
                  double fzm_, double fzp_, double rdzu_, double cqw_, double& wr, double& wz, double& tz) {
    if (act && k >= 1) {
      wr = .5 * dtseps * GRAVITY * (fzm_ * zz_ + fzp_ * zzm_);
      wz = dtseps * c2 * (fzm_ * zz_ + fzp_ * zzm_) * rdzu_ * cqw_ * (fzm_ * pp_ + fzp_ * pm_);
      tz = dtseps * (fzm_ * t_ + fzp_ * tm_);
    }
  };
  lev1(ax, kx, zz.x, zzm.x, pp.x, pm.x, t.x, tm.x, fzm.x, fzp.x, rdzu.x, cqw.x, cofwr.x, cofwz.x, coftz.x);
  lev1(ay, ky, zz.y, zzm.y, pp.y, pm.y, t.y, tm.y, fzm.y, fzp.y, rdzu.y, cqw.y, cofwr.y, cofwz.y, coftz.y);
  if (ax) cofwt.x = .5 * dtseps * rcv * zz.x * GRAVITY * rb.x / (1. + qtot.x) * pp.x / ((rtb.x + rt.x) * pb.x);
  if (ay) cofwt.y = .5 * dtseps * rcv * zz.y * GRAVITY * rb.y / (1. + qtot.y) * pp.y / ((rtb.y + rt.y) * pb.y);
  const d2 coftz_p = kp1(coftz), coftz_m = km1(coftz, l), cofwt_m = km1(cofwt, l), rdzw_m = km1(rdzw, l);
  const d2 cofrz{dtseps * rdzw.x, dtseps * rdzw.y};
  const d2 cofrz_m = km1(cofrz, l);
  d2 a{0.0, 0.0}, b{1.0, 1.0}, cc{0.0, 0.0};
  auto lev2 = [&](bool act, int k, double& a_, double& b_, double& c_, double wz, double wr, double wt, double tz,
                  double tzm, double tzp, double wtm, double rw, double rwm, double z, double zm, double rz,
                  double rzm) {
    if (act && k >= 1) {
      a_ = -wz * tzm * rwm * zm + wr * rzm - wtm * tzm * rwm;
      b_ = 1. + wz * (tz * rw * z + tz * rwm * zm) - tz * (wt * rw - wtm * rwm) + wr * (rz - rzm);
      c_ = -wz * tzp * rw * z - wr * rz + wt * tzp * rw;
    }
  };
  lev2(ax, kx, a.x, b.x, cc.x, cofwz.x, cofwr.x, cofwt.x, coftz.x, coftz_m.x, coftz_p.x, cofwt_m.x, rdzw.x,
       rdzw_m.x, zz.x, zzm.x, cofrz.x, cofrz_m.x);
  lev2(ay, ky, a.y, b.y, cc.y, cofwz.y, cofwr.y, cofwt.y, coftz.y, coftz_m.y, coftz_p.y, cofwt_m.y, rdzw.y,
       rdzw_m.y, zz.y, zzm.y, cofrz.y, cofrz_m.y);
  // sequential LU recurrence (2124-2127) as a lane-shift sweep
  const bool fx = kx >= 1 && ax, fy = ay;
  d2 alpha{0.0, 0.0}, gamma{0.0, 0.0};
  for (int it = 0; it < (ODD ? K + 1 : K) / 2; ++it) {
    const double gpx = lane_shr1(gamma.y);
    if (fx) {
      alpha.x = 1. / (b.x - a.x * (l == 0 ? 0.0 : gpx));
      gamma.x = cc.x * alpha.x;
    }
    if (fy) {
      alpha.y = 1. / (b.y - a.y * gamma.x);
      gamma.y = cc.y * alpha.y;
    }
  }
  if (mine && ax) {
    if (l == 0) {  // level 1 only: cofwr(1) / cofwz(1) are not written (2077-2081)
      p.cofwr[o + 1] = cofwr.y;
      p.cofwz[o + 1] = cofwz.y;
    } else {
      pst(p.cofwr + o, cofwr, two);
      pst(p.cofwz + o, cofwz, two);
    }
    pst(p.cofwt + o, cofwt, two);
    pst(p.a_tri + o, a, two);
    pst(p.alpha_tri + o, alpha, two);
    pst(p.gamma_tri + o, gamma, two);
  }
  // coftz(1) = coftz(K+1) = 0: levels 0..K, the lane holding level K stores that one level
  if (mine && kx <= K) {
    double* ct = p.coftz + (size_t)c * (K + 1) + kx;
    if (ky <= K) {
      ct[0] = coftz.x;
      ct[1] = coftz.y;
    } else {
      ct[0] = coftz.x;
    }
  }
}

// k_acoustic_edges in the pair layout (same expressions, per level)
// UP: the Theta''/rho'' halo comes from the exchange's receive buffer (fused unpack, UnpackMap)
template <bool DD, bool UP = false, bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_acoustic_edges_p(Dims d, Ptrs p, double dts, int small_step,
                                                                   double coef_divdamp, int phase, int fresh,
                                                                   UnpackMap um = UnpackMap{}) {
  int eA, eB;
  bool hasB;
  if (!pair_edges(d, p, phase, eA, eB, hasB)) return;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const bool lev = 2 * l < K;                     // this lane holds levels 2l, 2l+1
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const int bA = phase ? p.edge_bnd[eA] : 0, bB = phase ? p.edge_bnd[eB] : 0;
  const d2 tu = ld2(p.tend_u + o);
  auto active = [&](int2 ce, int bnd) {
    return (ce.x < d.nCellsSolve || ce.y < d.nCellsSolve) && !(phase && ((bnd != 0) != (phase == 2)));
  };
  const bool onA = active(ceA, bA), onB = hasB && active(ceB, bB);
  if (!onA && !onB) return;
  const bool st = lev && (h ? onB : onA);
  if (small_step == 1) {
    const d2 rup = {dts * tu.x, dts * tu.y};
    if (st) {
      pst(p.ru_p + o, rup, two);
      pst(p.ruAvg + o, rup, two);
    }
    return;
  }
  d2 rup, rua;
  if (fresh) {  // sub-step 1 left ru_p = ruAvg = dts * tend_u (see k_acoustic_edges)
    rup = d2{dts * tu.x, dts * tu.y};
    rua = rup;
  } else {
    rup = ld2(p.ru_p + o);
    rua = ld2(p.ruAvg + o);
  }
  const d2 cqu = ld2(p.cqu + o), zxu = ld2(p.zxu + o);
  const double mask = sel(h, ld_uniform_f64(p.specZoneMaskEdge + eA), ld_uniform_f64(p.specZoneMaskEdge + eB));
  const double invDc = sel(h, ld_uniform_f64(p.invDcEdge + eA), ld_uniform_f64(p.invDcEdge + eB));
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  const size_t o1 = (size_t)c1 * K + 2 * lc, o2 = (size_t)c2 * K + 2 * lc;
  const d2 rt1 = UP ? ld_pp<ODD>(d, p, um, 0, c1, lc, st) : ld2(p.rtheta_pp + o1);
  const d2 rt2 = UP ? ld_pp<ODD>(d, p, um, 0, c2, lc, st) : ld2(p.rtheta_pp + o2);
  const d2 zz1 = ld2(p.zz + o1), zz2 = ld2(p.zz + o2), ex1 = ld2(p.exner + o1), ex2 = ld2(p.exner + o2);
  const d2 rp1 = UP ? ld_pp<ODD>(d, p, um, 1, c1, lc, st) : ld2(p.rho_pp + o1);
  const d2 rp2 = UP ? ld_pp<ODD>(d, p, um, 1, c2, lc, st) : ld2(p.rho_pp + o2);
  d2 ro1{}, ro2{}, th1{}, th2{};
  if (DD) {
    ro1 = ld2(p.rtheta_pp_old + o1);
    ro2 = ld2(p.rtheta_pp_old + o2);
    th1 = ld2(p.theta_m1 + o1);
    th2 = ld2(p.theta_m1 + o2);
  }
  const double rcv = RGAS / (CP - RGAS);
  const double c2v = CP * rcv;
  auto level = [&](double r, double tu_, double cq, double zx, double a1, double a2, double z1, double z2,
                   double x1, double x2, double p1, double p2, double o1_, double o2_, double t1, double t2) {
    if (DD) {
      const double dd1 = -(a1 - o1_);
      const double dd2 = -(a2 - o2_);
      r = r + coef_divdamp * (dd2 - dd1) * (1.0 - mask) / (t1 + t2);
    }
    double pgrad = ((a2 - a1) * invDc) / (.5 * (z2 + z1));
    pgrad = cq * 0.5 * c2v * (x1 + x2) * pgrad;
    pgrad = pgrad + 0.5 * zx * GRAVITY * (p1 + p2);
    return r + dts * (tu_ - (1.0 - mask) * pgrad);
  };
  rup.x = level(rup.x, tu.x, cqu.x, zxu.x, rt1.x, rt2.x, zz1.x, zz2.x, ex1.x, ex2.x, rp1.x, rp2.x, ro1.x, ro2.x,
                th1.x, th2.x);
  rup.y = level(rup.y, tu.y, cqu.y, zxu.y, rt1.y, rt2.y, zz1.y, zz2.y, ex1.y, ex2.y, rp1.y, rp2.y, ro1.y, ro2.y,
                th1.y, th2.y);
  if (st) {
    pst(p.ru_p + o, rup, two);
    pst(p.ruAvg + o, d2{rua.x + rup.x, rua.y + rup.y}, two);
  }
}

// cell phase (2603-2721) on the per-cell stencil record (ME = maxEdges <= 7): every load the
// column needs -- the record, its own 22 columns, the ru_p of its edges and theta_m of the cells
// across them -- is issued before the first use, so one wave waits for two memory round trips
// (record, then gathers) instead of a chain per edge.  Same expressions, same order as below.
// recover_cells1 (2998-3040) of owned cell c from the final sub-step's new rho_pp / rtheta_pp /
// rw_p / wwAvg, still in registers (k_acoustic_cells_r<ME, true>): the same expressions as
// k_recover_cells1, lane for lane (inactive lanes see zz = fzm = fzp = 0 there too).
// The recovery's own operands (RecIn) are loaded after the tridiagonal solve: loaded with the
// sub-step's operands they held 12 more VGPRs across it (134 -> 122 VGPRs, 3 -> 4 waves/SIMD;
// -0.1 ms per dt same box, profiles/r02_ab_recin_late.log).
struct RecIn {
  double rps, rb, rtps, rtb, exb, rtd;
};
__device__ __forceinline__ RecIn load_rec_in(const Dims& d, const Ptrs& p, size_t o, int rk_step) {
  RecIn r;
  r.rps = p.rho_p_save[o];
  r.rb = p.rho_base[o];
  r.rtps = p.rtheta_p_save[o];
  r.rtb = p.rtheta_base[o];
  r.exb = rk_step == 3 ? p.exner_base[o] : 0.0;
  r.rtd = (rk_step == 3 && d.diabatic) ? p.rt_diabatic_tend[o] : 0.0;
  return r;
}
__device__ __forceinline__ void recover_cell_fused(const Dims& d, const Ptrs& p, int c, int k, double zz_k, double rws,
                                                   double fzm_k, double fzp_k, const RecIn& ri, double rhopp,
                                                   double rtpp, double rwp, double wwa, double dt, double invNs,
                                                   int rk_step) {
  const int K = d.K;
  const size_t K1 = K + 1;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t o = (size_t)c * K + kc, ow = (size_t)c * K1 + kw;
  const double rcv = RGAS / (CP - RGAS);
  const double rps = ri.rps, rb = ri.rb, rtps = ri.rtps, rtb = ri.rtb;
  const double fzm = act ? fzm_k : 0.0, fzp = act ? fzp_k : 0.0;
  const double zz = act ? zz_k : 0.0, zzm = up1(zz);
  double rz = 0.0;
  if (act) {
    const double rho_p = rps + rhopp;
    // rho_p is read only as rho_p_save, after the rotation at the next substep start, and by
    // the pool after the dt: the stage-3 value; stages 1-2 do not store it
    if (rk_step == 3) p.rho_p[o] = rho_p;
    rz = rho_p + rb;
    p.rho_zz2[o] = rz;
  }
  double w = 0.0;  // w(1) = w(nVertLevels+1) = 0
  if (act && k >= 1) {
    p.wwAvg[ow] = rws + (wwa * invNs);
    const double rw = rws + rwp;
    p.rw[ow] = rw;
    w = rw / (fzm * zz + fzp * zzm);  // divided by density in k_recover_cells3
  }
  if (k <= K) p.w2[ow] = w;
  if (act) {
    if (rk_step == 3) {
      const double rtp = rtps + rtpp - dt * rz * ri.rtd;  // rtd = 0.0 without diabatic forcing, as in k_recover_cells1
      p.rtheta_p[o] = rtp;
      p.theta_m2[o] = (rtp + rtb) / rz;
      const double ex = pow(zz * (RGAS / P0) * (rtp + rtb), rcv);
      p.exner[o] = ex;
      p.pressure_p[o] = zz * RGAS * (ex * rtp + rtb * (ex - ri.exb));
    } else {
      const double rtp = rtps + rtpp;
      p.rtheta_p[o] = rtp;
      p.theta_m2[o] = (rtp + rtb) / rz;
    }
  }
}

// FIN: the stage's last sub-step also recovers its owned cells (recover_cell_fused): nothing
// between this launch and k_recover_cells1 -- the Theta''/rho'' exchange, the damping (ru_p,
// ruAvg) and the 876-887 exchange -- reads or writes what the recovery reads or writes for an
// owned cell, so k_recover_cells1 then runs on the halo cells and the garbage slot only.
// keep_pp = 0 (FIN only): rho_pp and rw_p are not stored.  After a stage's last sub-step nothing
// reads them but the 876-887 exchange and the halo-cell recovery; srk3 passes 0 only for a block
// without exchanges and a stage that is not the dt's last (whose values the pool keeps).
// dl = 1 (FIN, keep_pp = 0, pair layout): the stage's last damping is the only reader of this
// sub-step's rtheta_pp and rtheta_pp_old, and it needs only their difference (2771-2772), so the
// column stores dtheta = rtheta_pp - rtheta_pp_old into rtheta_pp_old (the same subtraction the
// damping would do) and no rtheta_pp: one stream fewer here and one fewer gather there
// (k_divdamp_p with dl = 1)
// the column's new rtheta_pp / rho_pp into its send-buffer slots (PackMap), lane k = level k
__device__ __forceinline__ void pack_column(const PackMap& pk, int c, int k, bool act, double rt, double rho) {
  if (!pk.start) return;
  const int s0 = __builtin_amdgcn_readfirstlane(pk.start[c]), s1 = __builtin_amdgcn_readfirstlane(pk.start[c + 1]);
  for (int s = s0; s < s1; ++s) {
    if (act) pk.rt[s][k] = rt;
    if (act && pk.rho) pk.rho[s][k] = rho;
  }
}

// the column's new rw_p / rho_pp / rtheta_pp into its slots of the 876-887 exchange's send buffer
// (XPack, fields 0 / 1 / 2), lane k = level k (rw_p: levels 0..K)
__device__ __forceinline__ void pack_rec_cell(const XPack& pk, int c, int k, bool act, bool actw, double rw,
                                              double rho, double rt) {
  if (!pk.start) return;
  const int s0 = __builtin_amdgcn_readfirstlane(pk.start[c]), s1 = __builtin_amdgcn_readfirstlane(pk.start[c + 1]);
  for (int s = s0; s < s1; ++s) {
    const int f = __builtin_amdgcn_readfirstlane(pk.fid[s]);
    double* dst = pk.dst[s];
    if (f == 0) {
      if (actw) dst[k] = rw;
    } else if (act) {
      dst[k] = f == 1 ? rho : rt;
    }
  }
}

// rp: the stage's last sub-step (FIN) also packs the 876-887 exchange (XPack), or nothing
template <int ME, bool FIN = false>
__global__ __launch_bounds__(BLOCK_THREADS) void k_acoustic_cells_r(Dims d, Ptrs p, double dts, int small_step,
                                                                    double epssm, double rdt = 0.0,
                                                                    double invNs = 0.0, int rk_step = 0,
                                                                    int keep_pp = 1, PackMap pk = PackMap{}, int dl = 0,
                                                                    XPack rp = XPack{}) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K, actw = k <= K;
  const int kc = min(k, K - 1), kw = min(k, K);  // clamped lanes load in bounds and store nothing
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + kc, ow = (size_t)c * K1 + kw;
  // sub-step 1 starts from zero perturbations (2617-2622): rtheta_pp, rho_pp, rw_p and wwAvg are
  // not read then (the values would be replaced by 0 below), which saves four streams
  const bool first = small_step == 1;
  double rtpp = first ? 0.0 : p.rtheta_pp[o];
  if (c >= d.nCellsSolve) {
    if (act) p.rtheta_pp_old[o] = (FIN && dl) ? rtpp - (first ? 0.0 : rtpp) : (first ? 0.0 : rtpp);
    return;
  }
  int re[ME], rc[ME];
  double sdv[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    re[i] = p.cell_rec[(size_t)c * CELL_REC + i];
    rc[i] = p.cell_rec[(size_t)c * CELL_REC + CELL_REC_ME + i];
    sdv[i] = ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i);
  }
  const int ne = p.cell_rec[(size_t)c * CELL_REC + 14];
  const double invA = p.invAreaCell[c], spec = p.specZoneMaskCell[c];
  double rhopp = first ? 0.0 : p.rho_pp[o], rwp = first ? 0.0 : p.rw_p[ow], wwa = first ? 0.0 : p.wwAvg[ow];
  const double thc = p.theta_m1[o], trho = p.tend_rho[o], tth = p.tend_theta[o], tw = p.tend_w[ow];
  double ru[ME], th[ME];
  // sub-step 1: ru_p = dts * tend_u (794-837), formed here; srk3 launches no edge phase for it
  const double* __restrict__ rusrc = small_step == 1 ? p.tend_u : p.ru_p;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    ru[i] = rusrc[(size_t)re[i] * K + kc];
    th[i] = p.theta_m1[(size_t)rc[i] * K + kc];
  }
  if (small_step == 1) {
#pragma unroll
    for (int i = 0; i < ME; ++i) ru[i] = dts * ru[i];
  }
  const double coftz = p.coftz[ow], zz = p.zz[o], cofwt = p.cofwt[o], cofwz = p.cofwz[o], cofwr = p.cofwr[o];
  const double a_tri = p.a_tri[o], alpha_tri = p.alpha_tri[o], gamma_tri = p.gamma_tri[o];
  // rho_zz (tl2), rw and w (tl2) through the *_rd pointers: in a dynamics substep's first stage
  // they name the buffers that hold these values until the recovery (srk3, stage_fin)
  const double rz = p.rho_zz2_rd[o], dss = p.dss[o], rws = p.rw_save[ow], rw = p.rw_rd[ow], w2 = p.w2_rd[ow];
  const double cofrz = p.cofrz[kc], rdzw = p.rdzw[kc], fzm = p.fzm[kc], fzp = p.fzp[kc];
  RecIn ri{};
  const double rtpp_old = (small_step == 1) ? 0.0 : rtpp;
  const double resm = (1.0 - epssm) / (1.0 + epssm);
  if (small_step == 1) { wwa = 0.0; rhopp = 0.0; rtpp = 0.0; rwp = 0.0; }
  if (!act) { rhopp = 0.0; rtpp = 0.0; }  // the column's k = K+1 lane: zero, as a masked load gives
  if (spec == 0.0) {
    double ts = 0.0, rs = 0.0;
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      if (i < ne) {
        const double flux = dts * sdv[i] * ru[i] * invA;  // == sign * dts * dvEdge * ru_p * invAreaCell
        rs = rs - flux;
        ts = ts - flux * 0.5 * (th[i] + thc);  // (th2 + th1): the sum commutes exactly
      }
    }
    double dn2[2] = {coftz, rwp};  // levels k+1 (one LDS round trip in the wide build)
    col_shift(dn2, 1);
    const double coftz_p = dn2[0], rwp_p = dn2[1];
    if (act) {
      rs = rhopp + dts * trho + rs - cofrz * resm * (rwp_p - rwp);
      ts = rtpp + dts * tth + ts - resm * rdzw * (coftz_p * rwp_p - coftz * rwp);
    }
    if (act && k >= 1) wwa = wwa + 0.5 * (1.0 - epssm) * rwp;
    // rw_p right-hand side (2660-2670)
    double up7[7] = {zz, ts, rs, rtpp, rhopp, cofwt, rz};  // levels k-1
    col_shift(up7, -1);
    const double zzm = up7[0], tsm = up7[1], rsm = up7[2], rtppm = up7[3], rhoppm = up7[4], cofwtm = up7[5];
    if (act && k >= 1) {
      rwp = rwp + dts * tw - cofwz * ((zz * ts - zzm * tsm) + resm * (zz * rtpp - zzm * rtppm)) -
            cofwr * ((rs + rsm) + resm * (rhopp + rhoppm)) + cofwt * (ts + resm * rtpp) +
            cofwtm * (tsm + resm * rtppm);
    }
    // tridiagonal solve sweeping up and then down the column (2675-2682), reference order
#ifdef MPAS_WIDE
    rwp = column_solve(rwp, a_tri, alpha_tri, gamma_tri, k, K);
#else
    rwp = thomas_column(rwp, a_tri, alpha_tri, gamma_tri, k, K);
#endif
    // implicit Rayleigh damping of w (2687-2693)
    const double rzm = up7[6];
    if (act && k >= 1) {
      const double dd = rws - rw;
      rwp = (rwp + dd - dts * dss * (fzm * zz + fzp * zzm) * (fzm * rz + fzp * rzm) * w2) / (1.0 + dts * dss) - dd;
      wwa = wwa + 0.5 * (1.0 + epssm) * rwp;
    }
    const double rwp_p2 = dn1(rwp);
    const double rho_new = rs - cofrz * (rwp_p2 - rwp);
    const double rt_new = ts - rdzw * (coftz_p * rwp_p2 - coftz * rwp);
    if (act) {
      if (FIN && dl) {
        p.rtheta_pp_old[o] = rt_new - rtpp_old;
      } else {
        p.rtheta_pp_old[o] = rtpp_old;  // stored last: no store precedes the loads above
        p.rtheta_pp[o] = rt_new;
      }
      if (!FIN || keep_pp) p.rho_pp[o] = rho_new;
    }
    if (actw) {
      if (!FIN || keep_pp) p.rw_p[ow] = rwp;
      if (!FIN) p.wwAvg[ow] = wwa;
      else if (k == 0 || k == K) p.wwAvg[ow] = wwa;  // levels 2..K: recover_cell_fused
    }
    pack_column(pk, c, k, act, rt_new, rho_new);
    if (FIN) pack_rec_cell(rp, c, k, act, actw, rwp, rho_new, rt_new);
    if (FIN) ri = load_rec_in(d, p, o, rk_step);
    if (FIN) recover_cell_fused(d, p, c, k, zz, rws, fzm, fzp, ri, rho_new, rt_new, rwp, wwa, rdt, invNs, rk_step);
  } else {
    // specified zone (2710-2719): regional only, masks are 0 for global meshes
    if (act) {
      rhopp = rhopp + dts * trho;
      rtpp = rtpp + dts * tth;
      rwp = rwp + dts * tw;
      wwa = wwa + 0.5 * (1.0 + epssm) * rwp;
      if (FIN && dl) {
        p.rtheta_pp_old[o] = rtpp - rtpp_old;
      } else {
        p.rtheta_pp_old[o] = rtpp_old;
        p.rtheta_pp[o] = rtpp;
      }
      p.rho_pp[o] = rhopp;
    }
    if (actw) {
      p.rw_p[ow] = rwp;
      if (!FIN) p.wwAvg[ow] = wwa;
      else if (k == 0 || k == K) p.wwAvg[ow] = wwa;
    }
    pack_column(pk, c, k, act, rtpp, rhopp);
    if (FIN) pack_rec_cell(rp, c, k, act, actw, rwp, rhopp, rtpp);
    if (FIN) ri = load_rec_in(d, p, o, rk_step);
    if (FIN) recover_cell_fused(d, p, c, k, zz, rws, fzm, fzp, ri, rhopp, rtpp, rwp, wwa, rdt, invNs, rk_step);
  }
}

// cell phase (2603-2721): rtheta_pp_old for all cells, column solve for owned cells
__global__ __launch_bounds__(BLOCK_THREADS) void k_acoustic_cells(Dims d, Ptrs p, double dts, int small_step, double epssm) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K, actw = k <= K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k, ow = (size_t)c * K1 + k;
  double rtpp = LD(p.rtheta_pp, o);
  if (act) p.rtheta_pp_old[o] = (small_step == 1) ? 0.0 : rtpp;
  if (c >= d.nCellsSolve) return;
  const double resm = (1.0 - epssm) / (1.0 + epssm);
  double rhopp = LD(p.rho_pp, o), rwp = LDW(p.rw_p, ow), wwa = LDW(p.wwAvg, ow);
  if (small_step == 1) { wwa = 0.0; rhopp = 0.0; rtpp = 0.0; rwp = 0.0; }
  if (p.specZoneMaskCell[c] == 0.0) {
    double ts = 0.0, rs = 0.0;
    const int ne = p.nEdgesOnCell[c];
    const double invA = p.invAreaCell[c];
    // theta_m of this cell is loaded once; the edge's other cell supplies the second
    // operand, in the reference's (cell2 + cell1) order
    const double thc = LD(p.theta_m1, o);
    for (int i = 0; i < ne; ++i) {
      const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
      const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
      if (act) {
        // sub-step 1: ru_p = dts * tend_u (794-837), formed here (no edge phase is launched for it)
        const double rue = small_step == 1 ? dts * p.tend_u[(size_t)e * K + k] : p.ru_p[(size_t)e * K + k];
        const double flux = p.edgesOnCell_sign[c * d.maxEdges + i] * dts * p.dvEdge[e] * rue * invA;
        rs = rs - flux;
        const double th1 = (c1 == c) ? thc : p.theta_m1[(size_t)c1 * K + k];
        const double th2 = (c2 == c) ? thc : p.theta_m1[(size_t)c2 * K + k];
        ts = ts - flux * 0.5 * (th2 + th1);
      }
    }
    const double cofrz = act ? p.cofrz[k] : 0.0, rdzw = act ? p.rdzw[k] : 0.0;
    const double coftz = LDW(p.coftz, ow), coftz_p = dn1(coftz);
    const double rwp_p = dn1(rwp);
    if (act) {
      rs = rhopp + dts * p.tend_rho[o] + rs - cofrz * resm * (rwp_p - rwp);
      ts = rtpp + dts * p.tend_theta[o] + ts - resm * rdzw * (coftz_p * rwp_p - coftz * rwp);
    }
    if (act && k >= 1) wwa = wwa + 0.5 * (1.0 - epssm) * rwp;
    // rw_p right-hand side (2660-2670)
    const double zz = LD(p.zz, o), zzm = up1(zz);
    const double tsm = up1(ts), rsm = up1(rs), rtppm = up1(rtpp), rhoppm = up1(rhopp);
    const double cofwt = LD(p.cofwt, o), cofwtm = up1(cofwt);
    if (act && k >= 1) {
      rwp = rwp + dts * p.tend_w[ow] -
            p.cofwz[o] * ((zz * ts - zzm * tsm) + resm * (zz * rtpp - zzm * rtppm)) -
            p.cofwr[o] * ((rs + rsm) + resm * (rhopp + rhoppm)) + cofwt * (ts + resm * rtpp) +
            cofwtm * (tsm + resm * rtppm);
    }
    // tridiagonal solve sweeping up and then down the column (2675-2682), reference order
    const double a_tri = LD(p.a_tri, o), alpha_tri = LD(p.alpha_tri, o), gamma_tri = LD(p.gamma_tri, o);
#ifdef MPAS_WIDE
    rwp = column_solve(rwp, a_tri, alpha_tri, gamma_tri, k, K);
#else
    for (int kk = 1; kk < K; ++kk) {
      const double xm = readlane_d(rwp, kk - 1);
      if (k == kk) rwp = (rwp - a_tri * xm) * alpha_tri;
    }
    for (int kk = K - 1; kk >= 0; --kk) {
      const double xp = readlane_d(rwp, kk + 1);
      if (k == kk) rwp = rwp - gamma_tri * xp;
    }
#endif
    // implicit Rayleigh damping of w (2687-2693)
    if (act && k >= 1) {
      const double fzm = p.fzm[k], fzp = p.fzp[k];
      const double rz = p.rho_zz2_rd[o], rzm = p.rho_zz2_rd[o - 1];
      const double dss = p.dss[o];
      const double dd = p.rw_save[ow] - p.rw_rd[ow];
      rwp = (rwp + dd - dts * dss * (fzm * zz + fzp * zzm) * (fzm * rz + fzp * rzm) * p.w2_rd[ow]) / (1.0 + dts * dss) - dd;
      wwa = wwa + 0.5 * (1.0 + epssm) * rwp;
    }
    const double rwp_p2 = dn1(rwp);
    if (act) {
      p.rho_pp[o] = rs - cofrz * (rwp_p2 - rwp);
      p.rtheta_pp[o] = ts - rdzw * (coftz_p * rwp_p2 - coftz * rwp);
    }
    if (actw) {
      p.rw_p[ow] = rwp;
      p.wwAvg[ow] = wwa;
    }
  } else {
    // specified zone (2710-2719): regional only, masks are 0 for global meshes
    if (act) {
      rhopp = rhopp + dts * p.tend_rho[o];
      rtpp = rtpp + dts * p.tend_theta[o];
      rwp = rwp + dts * p.tend_w[ow];
      wwa = wwa + 0.5 * (1.0 + epssm) * rwp;
      p.rho_pp[o] = rhopp;
      p.rtheta_pp[o] = rtpp;
    }
    if (actw) {
      p.rw_p[ow] = rwp;
      p.wwAvg[ow] = wwa;
    }
  }
}

// atm_divergence_damping_3d (2765-2793).  EPW edges per wavefront: every load of all
// EPW edges is issued before the first store, so each wave keeps EPW x 7 column loads
// in flight (the kernel is latency x occupancy bound with one edge per wave).
template <int EPW>
__global__ __launch_bounds__(BLOCK_THREADS) void k_divdamp(Dims d, Ptrs p, double coef_divdamp, int phase, double dts,
                                                           int fresh) {  // fresh: see k_divdamp_p
  const int e0 = wave_elem(0) * EPW;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  double ru[EPW], d1[EPW], d2[EPW], th[EPW], mask[EPW];
  bool on[EPW];
#pragma unroll
  for (int j = 0; j < EPW; ++j) {
    const int e = e0 + j;
    on[j] = false;
    if (e < d.nEdges) {
      const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
      on[j] = (c1 < d.nCellsSolve || c2 < d.nCellsSolve) &&
              (phase == 0 || ((p.edge_bnd[e] != 0) == (phase == 2)));  // 1 / 2: edges without / with a halo cell
      if (on[j] && act) {
        const size_t o = (size_t)e * K + k, o1 = (size_t)c1 * K + k, o2 = (size_t)c2 * K + k;
        ru[j] = fresh ? dts * p.tend_u[o] : p.ru_p[o];
        d1[j] = -(p.rtheta_pp[o1] - p.rtheta_pp_old[o1]);
        d2[j] = -(p.rtheta_pp[o2] - p.rtheta_pp_old[o2]);
        th[j] = p.theta_m1[o1] + p.theta_m1[o2];
        mask[j] = p.specZoneMaskEdge[e];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < EPW; ++j) {
    if (on[j] && act) {
      p.ru_p[(size_t)(e0 + j) * K + k] = ru[j] + coef_divdamp * (d2[j] - d1[j]) * (1.0 - mask[j]) / th[j];
      if (fresh) p.ruAvg[(size_t)(e0 + j) * K + k] = ru[j];
    }
  }
}

// ============================================================================
// atm_recover_large_step_variables_work  (mpas_atm_time_integration.F:2984-3097)
// Three launches for the three barrier-separated phases.  phase 0 = every element; around the
// 876-887 exchange, phase 1 takes the elements that read no halo data (owned cells; edges with
// two owned cells; owned cells whose edges all have two owned cells) and phase 2 the rest.
// ============================================================================
// cells (all, and the garbage slot): 2998-3040
// ru: the 876-887 exchange's fused unpack (XUnpack, cell fields rw_p / rho_pp / rtheta_pp): a halo
// cell reads its received columns from the receive buffer and writes them into the fields
__global__ __launch_bounds__(BLOCK_THREADS) void k_recover_cells1(Dims d, Ptrs p, double dt, double invNs, int rk_step,
                                                                  int phase, int c0, XUnpack ru = XUnpack{}) {
  const int c = wave_elem(c0);
  if (phase && ((c >= d.nCellsSolve) != (phase == 2))) return;
  const int k = lane_id(), K = d.K;
  const size_t K1 = K + 1;
  if (c == d.nCells) {  // rho_zz(:, nCells+1) = 1 (2989-2991)
    if (k < K) p.rho_zz2[(size_t)c * K + k] = 1.0;
    return;
  }
  if (c > d.nCells) return;
  const bool act = k < K;
  const size_t o = (size_t)c * K + k, ow = (size_t)c * K1 + k;
  const int orw = rec_off(ru, 0, c, d.nCellsSolve), orho = rec_off(ru, 1, c, d.nCellsSolve),
            ort = rec_off(ru, 2, c, d.nCellsSolve);
  if (orw >= 0 && k <= K) p.rw_p[ow] = ru.recv[orw + k];
  if (orho >= 0 && act) p.rho_pp[o] = ru.recv[orho + k];
  if (ort >= 0 && act) p.rtheta_pp[o] = ru.recv[ort + k];
  const double rcv = RGAS / (CP - RGAS);
  double rz = 0.0;
  if (act) {
    const double rho_p = p.rho_p_save[o] + (orho >= 0 ? ru.recv[orho + k] : p.rho_pp[o]);
    if (rk_step == 3) p.rho_p[o] = rho_p;  // stored at stage 3 only (recover_cell_fused)
    rz = rho_p + p.rho_base[o];
    p.rho_zz2[o] = rz;
  }
  const double fzm = act ? p.fzm[k] : 0.0, fzp = act ? p.fzp[k] : 0.0;
  const double zz = LD(p.zz, o), zzm = up1(zz);
  double w = 0.0;  // w(1) = w(nVertLevels+1) = 0
  if (act && k >= 1) {
    p.wwAvg[ow] = p.rw_save[ow] + (p.wwAvg[ow] * invNs);
    const double rw = p.rw_save[ow] + (orw >= 0 ? ru.recv[orw + k] : p.rw_p[ow]);
    p.rw[ow] = rw;
    w = rw / (fzm * zz + fzp * zzm);  // divided by density in k_recover_cells3
  }
  if (k <= K) p.w2[ow] = w;
  if (act) {
    if (rk_step == 3) {
      const double rtpp = ort >= 0 ? ru.recv[ort + k] : p.rtheta_pp[o];
      const double rtp = p.rtheta_p_save[o] + rtpp - dt * rz * (d.diabatic ? p.rt_diabatic_tend[o] : 0.0);
      p.rtheta_p[o] = rtp;
      p.theta_m2[o] = (rtp + p.rtheta_base[o]) / rz;
      const double ex = pow(zz * (RGAS / P0) * (rtp + p.rtheta_base[o]), rcv);
      p.exner[o] = ex;
      p.pressure_p[o] = zz * RGAS * (ex * rtp + p.rtheta_base[o] * (ex - p.exner_base[o]));
    } else {
      const double rtp = p.rtheta_p_save[o] + (ort >= 0 ? ru.recv[ort + k] : p.rtheta_pp[o]);
      p.rtheta_p[o] = rtp;
      p.theta_m2[o] = (rtp + p.rtheta_base[o]) / rz;
    }
  }
}

// edges (all): 3048-3059
// phase 2 walks the compact bnd_edges list (the edges with edge_bnd set)
// ru: the 876-887 exchange's fused unpack (XUnpack, edge field ru_p), as in k_recover_cells1
// upk: the recovered u of an owned edge also goes to the u exchange's send buffer (988, XPack)
__global__ __launch_bounds__(BLOCK_THREADS) void k_recover_edges(Dims d, Ptrs p, double invNs, int phase,
                                                                 XUnpack ru = XUnpack{}, XPack upk = XPack{}) {
  int e = wave_elem(0);
  if (phase == 2) {
    if (e >= d.n_bnd_edges) return;
    e = __builtin_amdgcn_readfirstlane(p.bnd_edges[e]);
  }
  if (e >= d.nEdges) return;
  if (phase && ((p.edge_bnd[e] != 0) != (phase == 2))) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)e * K + k;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  const int oru = rec_off(ru, 0, e, d.nEdgesSolve);
  double rup;
  if (oru >= 0) {
    rup = ru.recv[oru + k];
    p.ru_p[o] = rup;
  } else {
    rup = p.ru_p[o];
  }
  p.ruAvg[o] = p.ru_save[o] + (p.ruAvg[o] * invNs);
  const double ruv = p.ru_save[o] + rup;
  p.ru[o] = ruv;
  const double un = 2. * ruv / (p.rho_zz2[(size_t)c1 * K + k] + p.rho_zz2[(size_t)c2 * K + k]);
  p.u2[o] = un;
  if (upk.start && e < d.nEdgesSolve) {
    const int s0 = __builtin_amdgcn_readfirstlane(upk.start[e]), s1 = __builtin_amdgcn_readfirstlane(upk.start[e + 1]);
    for (int sl = s0; sl < s1; ++sl) upk.dst[sl][k] = un;
  }
}

// cells (all): w from the flux-divergence operator, then divided by density (3063-3097)
__global__ __launch_bounds__(BLOCK_THREADS) void k_recover_cells3(Dims d, Ptrs p, int phase) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  if (phase && (((p.cell_bnd[c] & CELL_BND_EDGE) != 0) != (phase == 2))) return;
  const int k = lane_id(), K = d.K;
  const size_t K1 = K + 1;
  const bool act = k < K;
  const size_t o = (size_t)c * K + k, ow = (size_t)c * K1 + k;
  const double fzm = act ? p.fzm[k] : 0.0, fzp = act ? p.fzp[k] : 0.0;
  double w = act ? p.w2[ow] : 0.0;
  const int ne = p.nEdgesOnCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double sg = p.edgesOnCell_sign[c * d.maxEdges + i];
    const double ruk = act ? p.ru[(size_t)e * K + k] : 0.0;
    double rum, ru1, ru2, ru3;
    up1_first3(ruk, rum, ru1, ru2, ru3);
    const size_t zo = ((size_t)c * d.maxEdges + i) * K1 + k;
    if (k == 0) {
      const double flux = (p.cf1 * ru1 + p.cf2 * ru2 + p.cf3 * ru3);
      w = w + sg * (p.zb_cell[zo] + sgn1(flux) * p.zb3_cell[zo]) * flux;
    } else if (act) {
      const double flux = (fzm * ruk + fzp * rum);
      w = w + sg * (p.zb_cell[zo] + sgn1(flux) * p.zb3_cell[zo]) * flux;
    }
  }
  const double rz = act ? p.rho_zz2[o] : 0.0;
  double rzm, r1, r2, r3;
  up1_first3(rz, rzm, r1, r2, r3);
  if (k == 0) w = w / (p.cf1 * r1 + p.cf2 * r2 + p.cf3 * r3);
  else if (act) w = w / (fzm * rz + fzp * rzm);
  if (act) p.w2[ow] = w;  // w(K+1) stays 0
}

// ============================================================================
// atm_compute_solve_diagnostics_work  (mpas_atm_time_integration.F:5585-5820)
// ke_edge is recomputed where it is consumed with the reference expression
// efac*u**2 (bit-identical), collapsing the four barrier phases into three launches.
// ============================================================================
__device__ __forceinline__ double ke_edge_of(const Ptrs& p, const double* u, int e, int K, int k) {
  const double efac = p.dcEdge[e] * p.dvEdge[e];
  const double uu = u[(size_t)e * K + k];
  return efac * (uu * uu);
}

__global__ __launch_bounds__(BLOCK_THREADS) void k_diag_vertices(Dims d, Ptrs p, const double* __restrict__ u,
                                                                 int store_dv = 1) {
  const int v = wave_elem(0);
  if (v >= d.nVertices) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  double vort = 0.0, kev = 0.0;
  for (int i = 0; i < 3; ++i) {
    const int e = uni(p.edgesOnVertex[3 * v + i]);
    const double s = p.edgesOnVertex_sign[3 * v + i] * p.dcEdge[e];
    vort = vort + s * u[(size_t)e * K + k];
  }
  vort = vort * p.invAreaTriangle[v];
  const int e1 = uni(p.edgesOnVertex[3 * v]), e2 = uni(p.edgesOnVertex[3 * v + 1]), e3 = uni(p.edgesOnVertex[3 * v + 2]);
  const double r = 0.25 * p.invAreaTriangle[v];
  kev = (ke_edge_of(p, u, e1, K, k) + ke_edge_of(p, u, e2, K, k) + ke_edge_of(p, u, e3, K, k)) * r;
  const size_t o = (size_t)v * K + k;
  if (store_dv) p.vorticity[o] = vort;
  p.ke_vertex[o] = kev;
  p.pv_vertex[o] = (p.fVertex[v] + vort);
}

__global__ __launch_bounds__(BLOCK_THREADS) void k_diag_cells(Dims d, Ptrs p, const double* __restrict__ u, double apvm,
                                                              int store_dv = 1) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const int ne = p.nEdgesOnCell[c];
  const double r = p.invAreaCell[c];
  double div = 0.0, ke = 0.0;
  // divergence (5626-5640) and the edge part of ke (5650-5660): independent sums, one pass
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double s = p.edgesOnCell_sign[c * d.maxEdges + i] * p.dvEdge[e];
    const double ue = u[(size_t)e * K + k];
    div = div + s * ue;
    ke = ke + 0.25 * (p.dcEdge[e] * p.dvEdge[e] * (ue * ue));  // ke_edge (5600)
  }
  div = div * r;
  ke = ke * p.invAreaCell[c];
  const double ke_fact = 1.0 - .375;
  ke = ke_fact * ke;
  double pvc = 0.0;
  for (int i = 0; i < ne; ++i) {
    const int iv = uni(p.verticesOnCell[c * d.maxEdges + i]);
    const int j = p.kiteForCell[c * d.maxEdges + i];
    const double kite = p.kiteAreasOnVertex[3 * iv + j];
    ke = ke + (1. - ke_fact) * kite * p.ke_vertex[(size_t)iv * K + k] * r;
    pvc = pvc + kite * p.pv_vertex[(size_t)iv * K + k] * r;
  }
  const size_t o = (size_t)c * K + k;
  if (store_dv) p.divergence[o] = div;
  p.ke[o] = ke;
  if (apvm > 0.0) p.pv_cell[o] = pvc;
}

__global__ __launch_bounds__(BLOCK_THREADS) void k_diag_edges(Dims d, Ptrs p, const double* __restrict__ u,
                                                               const double* __restrict__ h, int reconstruct_v,
                                                               double apvm, double dt, int store_grad) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)e * K + k;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  const int v1 = p.verticesOnEdge[2 * e], v2 = p.verticesOnEdge[2 * e + 1];
  p.rho_edge[o] = 0.5 * (h[(size_t)c1 * K + k] + h[(size_t)c2 * K + k]);
  // ke_edge (5600) is module scratch: it is recomputed where consumed, never stored
  double vv;
  if (reconstruct_v) {
    vv = 0.0;
    const int neoe = p.nEdgesOnEdge[e];
    if (neoe == 10) {
      double uu[10];
#pragma unroll
      for (int i = 0; i < 10; ++i) uu[i] = u[(size_t)uni(p.edgesOnEdge[e * d.maxEdges2 + i]) * K + k];
#pragma unroll
      for (int i = 0; i < 10; ++i) vv = vv + p.weightsOnEdge[e * d.maxEdges2 + i] * uu[i];
    } else {
      for (int i = 0; i < neoe; ++i) {
        const int eoe = uni(p.edgesOnEdge[e * d.maxEdges2 + i]);
        vv = vv + p.weightsOnEdge[e * d.maxEdges2 + i] * u[(size_t)eoe * K + k];
      }
    }
    p.v[o] = vv;
  } else {
    vv = p.v[o];
  }
  const double pv1 = p.pv_vertex[(size_t)v1 * K + k], pv2 = p.pv_vertex[(size_t)v2 * K + k];
  double pve = 0.5 * (pv1 + pv2);
  if (apvm > 0.0) {
    const double r = apvm * dt;
    const double r1 = 1.0 * p.invDvEdge[e];
    const double r2 = 1.0 * p.invDcEdge[e];
    const double gt = (pv2 - pv1) * r1;
    const double gn = (p.pv_cell[(size_t)c2 * K + k] - p.pv_cell[(size_t)c1 * K + k]) * r2;
    if (store_grad) {  // see solve_diagnostics: only the last call of a dt stores them
      p.gradPVt[o] = gt;
      p.gradPVn[o] = gn;
    }
    pve = pve - r * (vv * gt + u[o] * gn);
  }
  p.pv_edge[o] = pve;
}

// batched variants of the recover / diagnostics kernels (maxEdges <= 7, see k_acoustic_cells_r)
// hdiv = 1: also the next stage's h_divergence (4729-4748) from the ru just recovered, which
// this kernel already gathers -- k_dyn_cells1 at rk_step 2 / 3 computes nothing else, and no
// kernel in between reads or writes ru or h_divergence; srk3 then skips that launch.
template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_recover_cells3_b(Dims d, Ptrs p, int phase, int hdiv) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  if (p.bdyMaskCell[c] > N_RELAX_ZONE) return;  // no specified-zone update (3069; any run)
  const int k = lane_id(), K = d.K;
  const size_t K1 = K + 1;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t o = (size_t)c * K + kc, ow = (size_t)c * K1 + kw;
  const int bnd = phase ? p.cell_bnd[c] : 0;
  const int ne = p.nEdgesOnCell[c];
  int ei[ME];
  double sg[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    ei[i] = p.edgesOnCell[(size_t)c * ME + i];
    sg[i] = ld_uniform_f64(p.edgesOnCell_sign + (size_t)c * ME + i);
  }
  double w = p.w2[ow];
  const double rz = p.rho_zz2[o];
  const double fzm = p.fzm[kc], fzp = p.fzp[kc];
  if (phase && (((bnd & CELL_BND_EDGE) != 0) != (phase == 2))) return;
  double ru[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) ru[i] = p.ru[(size_t)uni(ei[i]) * K + kc];
  if (!act) w = 0.0;
  // the vertical flux of each edge, then zb_cell + sign(1,flux) * zb3_cell as the one of
  // zb_p / zb_m the sign selects (k_build_zb)
  double fl[ME], zs[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const double ruk = ru[i];
    double rum, ru1, ru2, ru3;
    up1_first3(ruk, rum, ru1, ru2, ru3);
    fl[i] = (k == 0) ? (p.cf1 * ru1 + p.cf2 * ru2 + p.cf3 * ru3) : (fzm * ruk + fzp * rum);
  }
#pragma unroll
  for (int i = 0; i < ME; ++i) zs[i] = (sgn1(fl[i]) > 0.0 ? p.zb_p : p.zb_m)[((size_t)c * ME + i) * K1 + kw];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    if (i < ne && (k == 0 || act)) w = w + sg[i] * zs[i] * fl[i];
  }
  if (hdiv) {  // as k_dyn_cells1_b: edgesOnCell_sign * dvEdge * ru summed in edge order, times 1/area
    double hd = 0.0;
#pragma unroll
    for (int i = 0; i < ME; ++i)
      if (i < ne) hd = hd + ld_uniform_f64(p.cell_sdv + (size_t)c * ME + i) * ru[i];
    hd = hd * ld_uniform_f64(p.invAreaCell + c);
    if (act) p.h_divergence[o] = hd;
  }
  double rzm, r1, r2, r3;
  up1_first3(rz, rzm, r1, r2, r3);
  if (k == 0) w = w / (p.cf1 * r1 + p.cf2 * r2 + p.cf3 * r3);
  else if (act) w = w / (fzm * rz + fzp * rzm);
  if (act) p.w2[ow] = w;  // w(K+1) stays 0
}

template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_diag_cells_b(Dims d, Ptrs p, const double* __restrict__ u,
                                                                double apvm, int store_dv = 1) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const int ne = p.nEdgesOnCell[c];
  int ei[ME], vi[ME], kj[ME];
  double sg[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    ei[i] = p.edgesOnCell[(size_t)c * ME + i];
    vi[i] = p.verticesOnCell[(size_t)c * ME + i];
    kj[i] = p.kiteForCell[(size_t)c * ME + i];
    sg[i] = ld_uniform_f64(p.edgesOnCell_sign + (size_t)c * ME + i);
  }
  const double r = ld_uniform_f64(p.invAreaCell + c);
  double dc[ME], dv[ME], kite[ME], ue[ME], kv[ME], pvv[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    const int e = uni(ei[i]), iv = uni(vi[i]);
    dc[i] = ld_uniform_f64(p.dcEdge + e);
    dv[i] = ld_uniform_f64(p.dvEdge + e);
    kite[i] = ld_uniform_f64(p.kiteAreasOnVertex + 3 * iv + kj[i]);
    ue[i] = u[(size_t)e * K + k];
    kv[i] = p.ke_vertex[(size_t)iv * K + k];
    pvv[i] = apvm > 0.0 ? p.pv_vertex[(size_t)iv * K + k] : 0.0;
  }
  double div = 0.0, ke = 0.0;
  // divergence (5626-5640) and the edge part of ke (5650-5660)
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    if (i < ne) {
      div = div + (sg[i] * dv[i]) * ue[i];
      ke = ke + 0.25 * (dc[i] * dv[i] * (ue[i] * ue[i]));  // ke_edge (5600)
    }
  }
  div = div * r;
  ke = ke * r;
  const double ke_fact = 1.0 - .375;
  ke = ke_fact * ke;
  double pvc = 0.0;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    if (i < ne) {
      ke = ke + (1. - ke_fact) * kite[i] * kv[i] * r;
      pvc = pvc + kite[i] * pvv[i] * r;
    }
  }
  const size_t o = (size_t)c * K + k;
  if (store_dv) p.divergence[o] = div;
  p.ke[o] = ke;
  if (apvm > 0.0) p.pv_cell[o] = pvc;
}

template <int NE2>
__global__ __launch_bounds__(EDGE_THREADS) void k_diag_edges_b(Dims d, Ptrs p, const double* __restrict__ u,
                                                                const double* __restrict__ h, int reconstruct_v,
                                                                double apvm, double dt, int store_grad) {
  const int e = wave_elem_e();
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)e * K + k;
  const int2 ce = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * e);
  const int2 ve = *reinterpret_cast<const int2*>(p.verticesOnEdge + 2 * e);
  int neoe = 0;
  int eoe[NE2];
  double wgt[NE2];
  if (reconstruct_v) {
    neoe = p.nEdgesOnEdge[e];
#pragma unroll
    for (int j = 0; j < NE2; ++j) {
      eoe[j] = p.edgesOnEdge[(size_t)e * d.maxEdges2 + j];
      wgt[j] = ld_uniform_f64(p.weightsOnEdge + (size_t)e * d.maxEdges2 + j);
    }
  }
  double invDv = 0.0, invDc = 0.0, ue = 0.0;
  if (apvm > 0.0) {
    invDv = ld_uniform_f64(p.invDvEdge + e);
    invDc = ld_uniform_f64(p.invDcEdge + e);
    ue = u[o];
  }
  const int c1 = uni(ce.x), c2 = uni(ce.y), v1 = uni(ve.x), v2 = uni(ve.y);
  const double h1 = h[(size_t)c1 * K + k], h2 = h[(size_t)c2 * K + k];
  const double pv1 = p.pv_vertex[(size_t)v1 * K + k], pv2 = p.pv_vertex[(size_t)v2 * K + k];
  double pc1 = 0.0, pc2 = 0.0;
  if (apvm > 0.0) {
    pc1 = p.pv_cell[(size_t)c1 * K + k];
    pc2 = p.pv_cell[(size_t)c2 * K + k];
  }
  double vv;
  if (reconstruct_v) {
    double uu[NE2];
#pragma unroll
    for (int j = 0; j < NE2; ++j) uu[j] = u[(size_t)uni(eoe[j]) * K + k];
    vv = 0.0;
#pragma unroll
    for (int j = 0; j < NE2; ++j)
      if (j < neoe) vv = vv + wgt[j] * uu[j];
    p.v[o] = vv;
  } else {
    vv = p.v[o];
  }
  p.rho_edge[o] = 0.5 * (h1 + h2);
  double pve = 0.5 * (pv1 + pv2);
  if (apvm > 0.0) {
    const double r = apvm * dt;
    const double r1 = 1.0 * invDv;
    const double r2 = 1.0 * invDc;
    const double gt = (pv2 - pv1) * r1;
    const double gn = (pc2 - pc1) * r2;
    if (store_grad) {  // see solve_diagnostics: only the last call of a dt stores them
      p.gradPVt[o] = gt;
      p.gradPVn[o] = gn;
    }
    pve = pve - r * (vv * gt + ue * gn);
  }
  p.pv_edge[o] = pve;
}

// ============================================================================
// end of atm_srk3 with physics (DO_PHYSICS block, mpas_atm_time_integration.F:1610-1648):
// rqvdynten for the convection schemes that need it, then negative mixing ratios set to zero
// ============================================================================
__global__ __launch_bounds__(BLOCK_THREADS) void k_physics_rqvdynten(Dims d, Ptrs p, int index_qv, int monotonic,
                                                                      double config_dt) {
  const int c = wave_elem(0);
  if (c > d.nCells) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  p.rqvdynten[(size_t)c * K + k] =
      monotonic ? (p.scalars2[SIX(c, k, index_qv)] - p.scalars1[SIX(c, k, index_qv)]) / config_dt : 0.0;
}
__global__ void k_physics_clip_scalars(double* s, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (s[i] < 0.0) s[i] = 0.0;  // where (scalars_2 < 0.0) scalars_2 = 0.0
}

// ============================================================================
// atm_compute_output_diagnostics  (core_atmosphere/mpas_atm_core.F:753-800): theta, rho and
// pressure of the history output from the prognostic state of time level `tl`
// ============================================================================
__global__ __launch_bounds__(BLOCK_THREADS) void k_output_diagnostics(Dims d, Ptrs p, int tl, int index_qv) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)c * K + k;
  const double* theta_m = tl == 1 ? p.theta_m1 : p.theta_m2;
  const double* rho_zz = tl == 1 ? p.rho_zz1 : p.rho_zz2;
  const double* scalars = tl == 1 ? p.scalars1 : p.scalars2;
  p.theta[o] = theta_m[o] / (1.0 + RVORD * scalars[SIX(c, k, index_qv)]);
  p.rho[o] = rho_zz[o] * p.zz[o];
  p.pressure[o] = p.pressure_base[o] + p.pressure_p[o];
}

// ============================================================================
// atm_init_coupled_diagnostics  (mpas_atm_time_integration.F:5906-5988)
// ============================================================================
// cells: theta_m, rho_zz (5909-5914)
__global__ __launch_bounds__(BLOCK_THREADS) void k_init_coupled_a(Dims d, Ptrs p, int index_qv) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)c * K + k;
  p.theta_m1[o] = p.theta[o] * (1. + RVORD * p.scalars1[SIX(c, k, index_qv)]);
  p.rho_zz1[o] = p.rho[o] / p.zz[o];
}
// edges: ru (5918-5924)
__global__ __launch_bounds__(BLOCK_THREADS) void k_init_coupled_b(Dims d, Ptrs p) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  const size_t o = (size_t)e * K + k;
  p.ru[o] = 0.5 * p.u1[o] * (p.rho_zz1[(size_t)c1 * K + k] + p.rho_zz1[(size_t)c2 * K + k]);
}
// cells: rw, rho_p, rtheta_base, rtheta_p, exner, exner_base, pressure_p, pressure_base (5931-5988)
__global__ __launch_bounds__(BLOCK_THREADS) void k_init_coupled_c(Dims d, Ptrs p) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k;
  const double fzm = act ? p.fzm[k] : 0.0, fzp = act ? p.fzp[k] : 0.0;
  const double rz = LD(p.rho_zz1, o), rzm = up1(rz);
  const double zz = LD(p.zz, o), zzm = up1(zz);
  double rw = 0.0;
  if (act && k >= 1) rw = p.w1[(size_t)c * K1 + k] * (fzp * rzm + fzm * rz) * (fzp * zzm + fzm * zz);
  const int ne = p.nEdgesOnCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double ruk = LD(p.ru, (size_t)e * K + k), rum = up1(ruk);
    if (act && k >= 1) {
      const double flux = (fzm * ruk + fzp * rum);
      const size_t zo = ((size_t)c * d.maxEdges + i) * K1 + k;
      rw = rw - p.edgesOnCell_sign[c * d.maxEdges + i] * (p.zb_cell[zo] + sgn1(flux) * p.zb3_cell[zo]) * flux *
                    (fzp * zzm + fzm * zz);
    }
  }
  if (k <= K) p.rw[(size_t)c * K1 + k] = rw;
  if (!act) return;
  const double rcv = RGAS / (CP - RGAS);
  const double rho_p = rz - p.rho_base[o];
  p.rho_p[o] = rho_p;
  const double rtb = p.theta_base[o] * p.rho_base[o];
  p.rtheta_base[o] = rtb;
  const double th = p.theta_m1[o];
  const double rtp = th * rho_p + p.rho_base[o] * (th - p.theta_base[o]);
  p.rtheta_p[o] = rtp;
  const double ex = pow(zz * (RGAS / P0) * (rtp + rtb), rcv);
  const double exb = pow(zz * (RGAS / P0) * (rtb), rcv);
  p.exner[o] = ex;
  p.exner_base[o] = exb;
  p.pressure_p[o] = zz * RGAS * (ex * rtp + rtb * (ex - exb));
  p.pressure_base[o] = zz * RGAS * exb * rtb;
}

// ============================================================================
// atm_rk_dynamics_substep_finish  (mpas_atm_time_integration.F:6051-6079)
// ============================================================================
// Called at 1304-1341; flat 16-byte streams: each (K, n) / (K+1, n) array is contiguous over its
// owned+halo columns, so every lane moves two doubles.  Same ranges (garbage slot excluded), same
// expressions.  Only the averaging of ruAvg / wwAvg over the dynamics substeps (6064-6078) is
// stored here.  The copies of 6051-6061 are not:
//  * ru_save = ru, rw_save = rw, rtheta_p_save = rtheta_p, rho_p_save = rho_p: srk3 rotates each
//    pair's buffers instead (rotate_saves), see stage_pre;
//  * theta_m_1 = theta_m_2: srk3 swaps the two time-level buffers (swap_theta);
//  * u_1 = u_2, w_1 = w_2, rho_zz_1 = rho_zz_2 and, at the last substep, rho_zz_1 =
//    rho_zz_old_split: nothing in the dynamics reads time level 1 of u, w or rho_zz (the substeps
//    read time level 2, the acoustic step and dyn_tend theta_m of time level 1), so rho_zz_1 keeps
//    the step's starting value, which is what the last substep restores (1824, 6079) and the
//    split transport reads; u_1 / w_1 are overwritten by the next atm_rk_integration_setup after
//    mpas_pool_shift_time_levels before anything reads them.
__device__ __forceinline__ void fin_avg(double* avg, double* split, int64_t j, int n, int first, int last, double inv) {
  for (int q = 0; q < n; ++q) {  // n = 2, or 1 for an odd tail
    const int64_t i = j + q;
    const double a = first ? avg[i] : avg[i] + split[i];
    split[i] = a;
    if (last) avg[i] = a * inv;
  }
}
__global__ __launch_bounds__(BLOCK_THREADS) void k_substep_finish_v(Dims d, Ptrs p, int dynamics_substep,
                                                                     int dynamics_split, double inv_dynamics_split) {
  const int64_t nE = (int64_t)d.nEdges * d.K, nW = (int64_t)d.nCells * (d.K + 1);
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  const int first = dynamics_substep == 1, last = dynamics_substep == dynamics_split;
  const double inv = inv_dynamics_split;
  for (int w = 0; w < 2; ++w) {
    double* avg = w ? p.wwAvg : p.ruAvg;
    double* split = w ? p.wwAvg_split : p.ruAvg_split;
    const int64_t n = w ? nW : nE;
    for (int64_t j = 2 * t0; j < n; j += 2 * st) {
      if (j + 1 < n) {
        const d2 a = ld2(avg + j);
        d2 s2 = a;
        if (!first) {
          const d2 b = ld2(split + j);
          s2 = d2{a.x + b.x, a.y + b.y};
        }
        st2(split + j, s2);
        if (last) st2(avg + j, d2{s2.x * inv, s2.y * inv});
      } else {
        fin_avg(avg, split, j, 1, first, last, inv);
      }
    }
  }
}

// ============================================================================
// atm_advance_scalars_work  (mpas_atm_time_integration.F:3346-3504)
// ============================================================================
// edges (all): scalar value at the edge, horiz_flux_arr(ns, K, nEdges+1)  (3357-3426)
__global__ __launch_bounds__(BLOCK_THREADS) void k_scalars_edges(Dims d, Ptrs p) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  if (k >= K) return;
  const double uh = p.ruAvg[(size_t)e * K + k];
  const double sg = sgn1(uh);
  const int na = p.nAdvCellsForEdge[e];
  if (na == 10) {
    // unrolled hexagon form (3363-3390): sum of ten products, left to right
    double w[10];
    int ica[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      w[j] = p.adv_coefs[e * 15 + j] + sg * p.adv_coefs_3rd[e * 15 + j];
      ica[j] = uni(p.advCellsForEdge[e * 15 + j]);
    }
    for (int is = 0; is < ns; ++is) {
      double acc = w[0] * p.scalars2[SIX(ica[0], k, is)];
#pragma unroll
      for (int j = 1; j < 10; ++j) acc = acc + w[j] * p.scalars2[SIX(ica[j], k, is)];
      p.horiz_flux_array[HIX(e, k, is)] = acc;
    }
  } else {
    for (int is = 0; is < ns; ++is) {
      double acc = 0.0;
      for (int j = 0; j < na; ++j) {
        const int ic = uni(p.advCellsForEdge[e * 15 + j]);
        const double scalar_weight = p.adv_coefs[e * 15 + j] + sg * p.adv_coefs_3rd[e * 15 + j];
        acc = acc + scalar_weight * p.scalars2[SIX(ic, k, is)];
      }
      p.horiz_flux_array[HIX(e, k, is)] = acc;
    }
  }
}

// cells (solve): flux divergence, vertical flux3 transport and update (3433-3504)
__global__ __launch_bounds__(BLOCK_THREADS) void k_scalars_cells(Dims d, Ptrs p, double dt, double wt_new,
                                                                  double coef_3rd_order) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k;
  const double wt_old = 1. - wt_new;
  const int ne = p.nEdgesOnCell[c];
  const double invA = p.invAreaCell[c];
  const double fnm = act ? p.fzm[k] : 0.0, fnp = act ? p.fzp[k] : 0.0;
  const double wwa = (k <= K) ? p.wwAvg[(size_t)c * K1 + k] : 0.0;
  const double rdnw = act ? p.rdzw[k] : 0.0;
  const double rzo = LD(p.rho_zz1, o), rzn = LD(p.rho_zz2, o);
  const double rho_zz_new_inv = act ? 1.0 / (wt_old * rzo + wt_new * rzn) : 0.0;
  // edgesOnCell_sign * uhAvg of every edge, loaded once for all scalars
  double sru[MAX_EDGES_UNROLL];
  int eid[MAX_EDGES_UNROLL];
  const bool reg = ne <= MAX_EDGES_UNROLL;
  if (reg) {
#pragma unroll
    for (int i = 0; i < MAX_EDGES_UNROLL; ++i) {
      eid[i] = 0;
      sru[i] = 0.0;
      if (i < ne) {
        eid[i] = uni(p.edgesOnCell[c * d.maxEdges + i]);
        if (act) sru[i] = p.edgesOnCell_sign[c * d.maxEdges + i] * p.ruAvg[(size_t)eid[i] * K + k];
      }
    }
  }
  for (int is = 0; is < ns; ++is) {
    double stc = 0.0;
    if (reg) {
#pragma unroll
      for (int i = 0; i < MAX_EDGES_UNROLL; ++i)
        if (i < ne && act) stc = stc - sru[i] * p.horiz_flux_array[HIX(eid[i], k, is)];
    } else {
      for (int i = 0; i < ne; ++i) {
        const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
        if (act)
          stc = stc - p.edgesOnCell_sign[c * d.maxEdges + i] * p.ruAvg[(size_t)e * K + k] *
                          p.horiz_flux_array[HIX(e, k, is)];
      }
    }
    if (act) {
      double sts = 0.0;
      if (d.physics) sts = p.scalars_tend[SIX(c, k, is)];  // scalar_tend_save from physics
      else p.scalars_tend[SIX(c, k, is)] = 0.0;           // no physics: zeroed (3437-3439)
      stc = stc * invA + sts;
    }
    const double sn = LD(p.scalars2, SIX(c, k, is));
    const double snm1 = up1(sn), snm2 = up2(sn), snp1 = dn1(sn);
    double wdtn = 0.0;
    if (k == 1 || k == K - 1) wdtn = wwa * (fnm * sn + fnp * snm1);
    else if (k >= 2 && k <= K - 2) wdtn = flux3(snm2, snm1, sn, snp1, wwa, coef_3rd_order);
    const double wdtn_p = dn1(wdtn);
    if (act) {
      const double so = p.scalars1[SIX(c, k, is)];
      p.scalars2[SIX(c, k, is)] = (so * rzo + dt * (stc - rdnw * (wdtn_p - wdtn))) * rho_zz_new_inv;
    }
  }
}

// ============================================================================
// atm_advance_scalars_mono_work  (mpas_atm_time_integration.F:3737-4210)
// ============================================================================
// cells (solve): source update of scalars_old (3737-3752) and rho_zz_int (3766-3792)
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_prep(Dims d, Ptrs p, double dt, int advance_density) {
  const int c = wave_elem(0);
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const size_t K1 = K + 1;
  if (c >= d.nCells) return;
  const size_t o = (size_t)c * K + k;
  if (c >= d.nCellsSolve) {  // rho_zz_int(:,iCell) = 0 on all cells (3772-3774)
    if (advance_density && act) p.rho_zz_int[o] = 0.0;
    return;
  }
  if (act) {
    const double rzo = p.rho_zz1[o];
    for (int is = 0; is < ns; ++is) {
      const size_t so = SIX(c, k, is);
      if (!d.physics) p.scalars_tend[so] = 0.0;  // 3743-3747: zeroed only without physics
      p.scalars1[so] = p.scalars1[so] + dt * p.scalars_tend[so] / rzo;
      p.scalars_tend[so] = 0.0;
    }
  }
  if (advance_density) {
    double rzi = 0.0;
    const int ne = p.nEdgesOnCell[c];
    for (int i = 0; i < ne; ++i) {
      const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
      if (act)
        rzi = rzi - p.edgesOnCell_sign[c * d.maxEdges + i] * p.ruAvg[(size_t)e * K + k] * p.dvEdge[e] * p.invAreaCell[c];
    }
    const double wwa = (k <= K) ? p.wwAvg[(size_t)c * K1 + k] : 0.0, wwap = dn1(wwa);
    if (act) p.rho_zz_int[o] = p.rho_zz1[o] + dt * (rzi - p.rdzw[k] * (wwap - wwa));
  }
}

// k_mono_prep for the batched families: the cell's edge record and every gather of ruAvg issued
// before the sums (the general kernel's edge loop waits on each edge in turn), and without physics
// the zeroed scalars_tend is not read back (its value there is 0.0 either way); same expressions in
// the same order.
template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_prep_b(Dims d, Ptrs p, double dt, int advance_density) {
  const int c = wave_elem(0);
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const int kc = min(k, K - 1);
  const size_t K1 = K + 1;
  if (c >= d.nCells) return;
  const size_t o = (size_t)c * K + k;
  if (c >= d.nCellsSolve) {  // rho_zz_int(:,iCell) = 0 on all cells (3772-3774)
    if (advance_density && act) p.rho_zz_int[o] = 0.0;
    return;
  }
  const CellSten<ME> st = load_sten<ME>(p, c);
  double ra[ME], dv[ME];
  if (advance_density) {
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      const int e = uni(st.e[i]);
      ra[i] = p.ruAvg[(size_t)e * K + kc];
      dv[i] = ld_uniform_f64(p.dvEdge + e);
    }
  }
  if (act) {
    const double rzo = p.rho_zz1[o];
    for (int is = 0; is < ns; ++is) {
      const size_t so = SIX(c, k, is);
      const double tend = d.physics ? p.scalars_tend[so] : 0.0;  // 3743-3747: zeroed only without physics
      p.scalars1[so] = p.scalars1[so] + dt * tend / rzo;
      p.scalars_tend[so] = 0.0;
    }
  }
  if (advance_density) {
    double rzi = 0.0;
    const double ia = ld_uniform_f64(p.invAreaCell + c);
#pragma unroll
    for (int i = 0; i < ME; ++i)
      if (i < st.ne) rzi = rzi - st.sg(i) * ra[i] * dv[i] * ia;
    const double wwa = (k <= K) ? p.wwAvg[(size_t)c * K1 + k] : 0.0, wwap = dn1(wwa);
    if (act) p.rho_zz_int[o] = p.rho_zz1[o] + dt * (rzi - p.rdzw[k] * (wwap - wwa));
  }
}

// per scalar iScalar, cells (solve): vertical flux and min/max bounds (3843-3908)
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_bounds(Dims d, Ptrs p, int is, double coef_3rd_order) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k;
  auto sold = [&](int cc) -> double { return (cc < d.nCells) ? p.scalars1[SIX(cc, k, is)] : 0.0; };
  const double so = act ? sold(c) : 0.0;
  const double sn = LD(p.scalars2, SIX(c, k, is));
  const double som = up1(so), sop = dn1(so);
  const double snm1 = up1(sn), snm2 = up2(sn), snp1 = dn1(sn);
  const double wwa = (k <= K) ? p.wwAvg[(size_t)c * K1 + k] : 0.0;
  const double fnm = act ? p.fzm[k] : 0.0, fnp = act ? p.fzp[k] : 0.0;
  double wdtn = 0.0;
  if (k == 1 || k == K - 1) wdtn = wwa * (fnm * sn + fnp * snm1);
  else if (k >= 2 && k <= K - 2) wdtn = flux3(snm2, snm1, sn, snp1, wwa, coef_3rd_order);
  if (k <= K) p.wdtn[(size_t)c * K1 + k] = wdtn;
  if (!act) return;
  double smax, smin;
  if (k == 0) {
    smax = fmax(so, sop);
    smin = fmin(so, sop);
  } else if (k == K - 1) {
    smax = fmax(so, som);
    smin = fmin(so, som);
  } else {
    smax = fmax(fmax(som, so), sop);
    smin = fmin(fmin(som, so), sop);
  }
  const int ne = p.nEdgesOnCell[c];
  for (int i = 0; i < ne; ++i) {
    const int cc = uni(p.cellsOnCell[c * d.maxEdges + i]);
    const double v = sold(cc);
    smax = fmax(smax, v);
    smin = fmin(smin, v);
  }
  p.s_max[o] = smax;
  p.s_min[o] = smin;
}

// per scalar, edges: high-order flux (3916-3961), upwind flux and flux difference (4007-4022)
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_edges1(Dims d, Ptrs p, int is, double dt) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  if (k >= K) return;
  const size_t o = (size_t)e * K + k;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  auto snew = [&](int cc) -> double { return (cc < d.nCells) ? p.scalars2[SIX(cc, k, is)] : 0.0; };
  auto sold = [&](int cc) -> double { return (cc < d.nCells) ? p.scalars1[SIX(cc, k, is)] : 0.0; };
  const double uh = p.ruAvg[o];
  double fa = 0.0;
  if (c1 < d.nCellsSolve || c2 < d.nCellsSolve) {
    const int na = p.nAdvCellsForEdge[e];
    if (na == 10) {
      const int ii = (uh > 0) ? 0 : 1;
      double acc = 0.0;
#pragma unroll
      for (int jj = 0; jj < 10; ++jj) {
        const double a = p.adv_coefs[e * 15 + jj], b = p.adv_coefs_3rd[e * 15 + jj];
        const double swa = (ii == 0) ? (a + b) : (a - b);
        const double term = swa * snew(uni(p.advCellsForEdge[e * 15 + jj]));
        acc = (jj == 0) ? term : acc + term;
      }
      fa = uh * (acc);
    } else {
      for (int i = 0; i < na; ++i) {
        const int ic = uni(p.advCellsForEdge[e * 15 + i]);
        const double scalar_weight = uh * (p.adv_coefs[e * 15 + i] + sgn1(uh) * p.adv_coefs_3rd[e * 15 + i]);
        fa = fa + scalar_weight * snew(ic);
      }
    }
  }
  p.flux_arr[o] = fa;
  const double fu = p.dvEdge[e] * dt * (fmax(0.0, uh) * sold(c1) + fmin(0.0, uh) * sold(c2));
  p.flux_upwind_tmp[o] = fu;
  p.flux_tmp[o] = dt * fa - fu;
}

// per scalar, cells (solve): upwind update, in/out flux sums and limiter factors (3969-4076)
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_cells1(Dims d, Ptrs p, int is, double dt, int advance_density) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k, ow = (size_t)c * K1 + k;
  const double eps = 1.e-20;
  const double so = LD(p.scalars1, SIX(c, k, is)), som = up1(so);
  const double rzo = LD(p.rho_zz1, o);
  const double wwa = (k <= K) ? p.wwAvg[ow] : 0.0;
  const double rdnw = act ? p.rdzw[k] : 0.0;
  double snew = so * rzo;
  double fua = 0.0;  // flux_upwind_arr(k), k >= 2
  if (act && k >= 1) fua = dt * (fmax(0.0, wwa) * som + fmin(0.0, wwa) * so);
  const double fua_p = dn1(fua);
  if (act && k <= K - 2) snew = snew - fua_p * rdnw;
  double wd = (k <= K) ? p.wdtn[ow] : 0.0;
  if (act && k >= 1) {
    snew = snew + fua * rdnw;
    wd = dt * wd - fua;
  }
  if (k <= K) p.wdtn[ow] = wd;
  const double wdp = dn1(wd);
  double sin_ = 0.0, sout = 0.0;
  if (act) {
    sin_ = -rdnw * (fmin(0.0, wdp) - fmax(0.0, wd));
    sout = -rdnw * (fmax(0.0, wdp) - fmin(0.0, wd));
  }
  const int ne = p.nEdgesOnCell[c];
  const double invA = p.invAreaCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double sg = p.edgesOnCell_sign[c * d.maxEdges + i];
    if (act) {
      const double ft = p.flux_tmp[(size_t)e * K + k];
      snew = snew - sg * p.flux_upwind_tmp[(size_t)e * K + k] * invA;
      sout = sout - fmax(0.0, sg * ft) * invA;
      sin_ = sin_ - fmin(0.0, sg * ft) * invA;
    }
  }
  if (!act) return;
  const double rhoref = advance_density ? p.rho_zz_int[o] : p.rho_zz2[o];
  double scale_factor = (p.s_max[o] * rhoref - snew) / (sin_ + eps);
  const double scale_in = fmin(1.0, fmax(0.0, scale_factor));
  scale_factor = (p.s_min[o] * rhoref - snew) / (sout - eps);
  const double scale_out = fmin(1.0, fmax(0.0, scale_factor));
  p.scalar_old_copy[o] = snew;  // upwind solution (the reference's scratch scalar_new)
  p.scale_arr[((size_t)c * 2 + 0) * K + k] = scale_in;
  p.scale_arr[((size_t)c * 2 + 1) * K + k] = scale_out;
}

// per scalar, edges with an owned cell: flux correction and rescale (4102-4138)
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_edges2(Dims d, Ptrs p, double dt) {
  const int e = wave_elem(0);
  if (e >= d.nEdges) return;
  const int c1 = p.cellsOnEdge[2 * e], c2 = p.cellsOnEdge[2 * e + 1];
  if (!(c1 < d.nCellsSolve || c2 < d.nCellsSolve)) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  const size_t o = (size_t)e * K + k;
  double flux = dt * p.flux_arr[o] - p.flux_upwind_tmp[o];
  auto sc = [&](int cc, int io) -> double { return (cc < d.nCells) ? p.scale_arr[((size_t)cc * 2 + io) * K + k] : 0.0; };
  flux = fmax(0.0, flux) * fmin(sc(c1, 1), sc(c2, 0)) + fmin(0.0, flux) * fmin(sc(c1, 0), sc(c2, 1));
  p.flux_arr[o] = flux;
}

// per scalar, cells: vertical flux rescale, update and positive-definite copy-back (4145-4210)
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_cells2(Dims d, Ptrs p, int is, int advance_density) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + k, ow = (size_t)c * K1 + k;
  if (c >= d.nCellsSolve) {  // halo cells: scalars_new = max(0, scalar_new) with scalar_new = input copy
    if (act) p.scalars2[SIX(c, k, is)] = fmax(0.0, p.scalars2[SIX(c, k, is)]);
    return;
  }
  const double si = act ? p.scale_arr[((size_t)c * 2 + 0) * K + k] : 0.0;
  const double so_ = act ? p.scale_arr[((size_t)c * 2 + 1) * K + k] : 0.0;
  const double sim = up1(si), som = up1(so_);
  double wd = (k <= K) ? p.wdtn[ow] : 0.0;
  if (act && k >= 1) {
    const double f = wd;
    wd = fmax(0.0, f) * fmin(som, si) + fmin(0.0, f) * fmin(so_, sim);
  }
  const double wdp = dn1(wd);
  if (!act) return;
  double snew = p.scalar_old_copy[o];
  const int ne = p.nEdgesOnCell[c];
  const double invA = p.invAreaCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    snew = snew - p.edgesOnCell_sign[c * d.maxEdges + i] * p.flux_arr[(size_t)e * K + k] * invA;
  }
  const double rhoref = advance_density ? p.rho_zz_int[o] : p.rho_zz2[o];
  snew = (snew + (-p.rdzw[k] * (wdp - wd))) / rhoref;
  p.scalars2[SIX(c, k, is)] = fmax(0.0, snew);
}

// ---- batched-load variants of the transport cell kernels (maxEdges 6 / 7, per-cell records) and
// the pair-layout flux correction; same expressions and order as the kernels above
template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_scalars_cells_b(Dims d, Ptrs p, double dt, double wt_new,
                                                                    double coef_3rd_order) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  if (p.bdyMaskCell[c] > N_RELAX_ZONE) return;  // specified zone not updated here (3435; any run)
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + kc;
  const double wt_old = 1. - wt_new;
  const CellSten<ME> st = load_sten<ME>(p, c);
  const double invA = ld_uniform_f64(p.invAreaCell + c);
  const double fnm = p.fzm[kc], fnp = p.fzp[kc], rdnw = p.rdzw[kc];
  const double wwa = p.wwAvg[(size_t)c * K1 + kw];
  const double rzo = p.rho_zz1[o], rzn = p.rho_zz2[o];
  double ra[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) ra[i] = p.ruAvg[(size_t)st.e[i] * K + kc];
  const double rho_zz_new_inv = act ? 1.0 / (wt_old * rzo + wt_new * rzn) : 0.0;
  double sru[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) sru[i] = st.sg(i) * ra[i];  // edgesOnCell_sign * uhAvg
  for (int is = 0; is < ns; ++is) {
    double hf[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) hf[i] = p.horiz_flux_array[HIX(st.e[i], kc, is)];
    double sn = p.scalars2[SIX(c, kc, is)];
    const double so = p.scalars1[SIX(c, kc, is)];
    if (!act) sn = 0.0;
    double stc = 0.0;
#pragma unroll
    for (int i = 0; i < ME; ++i)
      if (i < st.ne) stc = stc - sru[i] * hf[i];
    if (act) {
      double sts = 0.0;
      if (d.physics) sts = p.scalars_tend[SIX(c, k, is)];  // scalar_tend_save from physics
      else p.scalars_tend[SIX(c, k, is)] = 0.0;           // no physics: zeroed (3437-3439)
      stc = stc * invA + sts;
    }
    const double snm1 = up1(sn), snm2 = up2(sn), snp1 = dn1(sn);
    double wdtn = 0.0;
    if (k == 1 || k == K - 1) wdtn = wwa * (fnm * sn + fnp * snm1);
    else if (k >= 2 && k <= K - 2) wdtn = flux3(snm2, snm1, sn, snp1, wwa, coef_3rd_order);
    const double wdtn_p = dn1(wdtn);
    if (act) p.scalars2[SIX(c, k, is)] = (so * rzo + dt * (stc - rdnw * (wdtn_p - wdtn))) * rho_zz_new_inv;
  }
}

// the second scratch set (mono_slot1) of k_mono_bounds_b / k_mono_cells1_b / k_mono_cells2_b for the pair's second scalar
struct MonoCell2 {
  double *wdtn, *s_max, *s_min, *flux_arr, *flux_upwind_tmp, *scalar_old_copy, *scale_arr;
};
template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_bounds_b(Dims d, Ptrs p, int is, double coef_3rd_order,
                                                                  int nq = 1, MonoCell2 s2 = MonoCell2{}) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + kc;
  const int ne = p.nEdgesOnCell[c];
  int cc[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) cc[i] = p.cellsOnCell[(size_t)c * ME + i];
  const double wwa = p.wwAvg[(size_t)c * K1 + kw];
  const double fnm = p.fzm[kc], fnp = p.fzp[kc];
  // nq = 2: the pair's second scalar (is + 1) into the second scratch set (s2), after the first
#pragma unroll 1
  for (int q = 0; q < nq; ++q) {
    const int iq = is + q;
    double so = p.scalars1[SIX(c, kc, iq)], sn = p.scalars2[SIX(c, kc, iq)];
    double sv[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      const double v = p.scalars1[SIX(cc[i], kc, iq)];
      sv[i] = cc[i] < d.nCells ? v : 0.0;  // sold() of the reference's halo loop
    }
    if (!act) {
      so = 0.0;
      sn = 0.0;
    }
    const double som = up1(so), sop = dn1(so);
    const double snm1 = up1(sn), snm2 = up2(sn), snp1 = dn1(sn);
    double wdtn = 0.0;
    if (k == 1 || k == K - 1) wdtn = wwa * (fnm * sn + fnp * snm1);
    else if (k >= 2 && k <= K - 2) wdtn = flux3(snm2, snm1, sn, snp1, wwa, coef_3rd_order);
    if (k <= K) (q ? s2.wdtn : p.wdtn)[(size_t)c * K1 + k] = wdtn;
    if (!act) continue;
    double smax, smin;
    if (k == 0) {
      smax = fmax(so, sop);
      smin = fmin(so, sop);
    } else if (k == K - 1) {
      smax = fmax(so, som);
      smin = fmin(so, som);
    } else {
      smax = fmax(fmax(som, so), sop);
      smin = fmin(fmin(som, so), sop);
    }
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      if (i < ne) {
        smax = fmax(smax, sv[i]);
        smin = fmin(smin, sv[i]);
      }
    }
    (q ? s2.s_max : p.s_max)[o] = smax;
    (q ? s2.s_min : p.s_min)[o] = smin;
  }
}

// pair_rule: the edge fluxes come from k_mono_edges1_p, whose flux_arr holds the upwind flux on the
// outer relaxation rows (upw, 4017-4020) -- flux_tmp is 0 there; else from k_mono_edges1 (no such rows)
// FB: k_mono_bounds_b fused in (3798-3850 + 3857-3907 before 3969-4076): the cell forms its own s_max /
// s_min from the old scalar of its column and ring and its vertical flux wdtn from the new scalar, with
// k_mono_bounds_b's expressions, instead of reading them back (nothing else reads s_max / s_min, and the
// edge pass in between touches none of the inputs); coef_3rd_order only for FB
template <int ME, bool FB = false>
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_cells1_b(Dims d, Ptrs p, int is, double dt, int advance_density,
                                                                  int nq = 1, MonoCell2 s2 = MonoCell2{},
                                                                  int pair_rule = 1, double coef_3rd_order = 0.0) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + kc, ow = (size_t)c * K1 + kw;
  const double eps = 1.e-20;
  const CellSten<ME> st = load_sten<ME>(p, c);
  const double invA = ld_uniform_f64(p.invAreaCell + c);
  const double rzo_l = p.rho_zz1[o];
  const double wwa = p.wwAvg[ow], rdnw = p.rdzw[kc];
  const double rhoref = advance_density ? p.rho_zz_int[o] : p.rho_zz2[o];
  int cc[ME];  // FB: cellsOnCell, as k_mono_bounds_b reads it
  double fnm = 0.0, fnp = 0.0;
  if (FB) {
#pragma unroll
    for (int i = 0; i < ME; ++i) cc[i] = p.cellsOnCell[(size_t)c * ME + i];
    fnm = p.fzm[kc];
    fnp = p.fzp[kc];
  }
  // nq = 2: the pair's second scalar (is + 1) with the second scratch set (s2), after the first --
  // the cell's own columns and stencil read once
#pragma unroll 1
  for (int q = 0; q < nq; ++q) {
    const int iq = is + q;
    double* wdtn = q ? s2.wdtn : p.wdtn;
    const double* farr = q ? s2.flux_arr : p.flux_arr;
    const double* fup = q ? s2.flux_upwind_tmp : p.flux_upwind_tmp;
    double so = p.scalars1[SIX(c, kc, iq)];
    double rzo = rzo_l;
    double wd, smx, smn;
    if (FB) {  // k_mono_bounds_b
      double sn = p.scalars2[SIX(c, kc, iq)], sb = so;
      double sv[ME];
#pragma unroll
      for (int i = 0; i < ME; ++i) {
        const double v = p.scalars1[SIX(cc[i], kc, iq)];
        sv[i] = cc[i] < d.nCells ? v : 0.0;  // sold() of the reference's halo loop
      }
      if (!act) {
        sb = 0.0;
        sn = 0.0;
      }
      const double som = up1(sb), sop = dn1(sb);
      const double snm1 = up1(sn), snm2 = up2(sn), snp1 = dn1(sn);
      wd = 0.0;
      if (k == 1 || k == K - 1) wd = wwa * (fnm * sn + fnp * snm1);
      else if (k >= 2 && k <= K - 2) wd = flux3(snm2, snm1, sn, snp1, wwa, coef_3rd_order);
      if (k == 0) {
        smx = fmax(sb, sop);
        smn = fmin(sb, sop);
      } else if (k == K - 1) {
        smx = fmax(sb, som);
        smn = fmin(sb, som);
      } else {
        smx = fmax(fmax(som, sb), sop);
        smn = fmin(fmin(som, sb), sop);
      }
#pragma unroll
      for (int i = 0; i < ME; ++i) {
        if (i < st.ne) {
          smx = fmax(smx, sv[i]);
          smn = fmin(smn, sv[i]);
        }
      }
    } else {
      wd = wdtn[ow];
      smx = (q ? s2.s_max : p.s_max)[o];
      smn = (q ? s2.s_min : p.s_min)[o];
    }
    double ft[ME], fu[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      const double fa = farr[(size_t)st.e[i] * K + kc];
      fu[i] = fup[(size_t)st.e[i] * K + kc];
      // flux_tmp of k_mono_edges1(_p) (4014, 4017-4020): dt flux_arr - flux_upwind, 0 on the upwind-only rows
      const int bm = pair_rule ? p.bdyMaskEdge[st.e[i]] : 0;
      const bool upw = (d.lbc && bm == N_RELAX_ZONE) || bm == N_RELAX_ZONE - 1;
      ft[i] = upw ? 0.0 : dt * fa - fu[i];
    }
    if (!act) {
      so = 0.0;
      rzo = 0.0;
    }
    const double som = up1(so);
    double snew = so * rzo;
    double fua = 0.0;  // flux_upwind_arr(k), k >= 2
    if (act && k >= 1) fua = dt * (fmax(0.0, wwa) * som + fmin(0.0, wwa) * so);
    const double fua_p = dn1(fua);
    if (act && k <= K - 2) snew = snew - fua_p * rdnw;
    if (k > K) wd = 0.0;
    if (act && k >= 1) {
      snew = snew + fua * rdnw;
      wd = dt * wd - fua;
    }
    if (k <= K) wdtn[ow] = wd;
    const double wdp = dn1(wd);
    double sin_ = 0.0, sout = 0.0;
    if (act) {
      sin_ = -rdnw * (fmin(0.0, wdp) - fmax(0.0, wd));
      sout = -rdnw * (fmax(0.0, wdp) - fmin(0.0, wd));
    }
#pragma unroll
    for (int i = 0; i < ME; ++i) {
      if (i < st.ne && act) {
        const double sg = st.sg(i);
        snew = snew - sg * fu[i] * invA;
        sout = sout - fmax(0.0, sg * ft[i]) * invA;
        sin_ = sin_ - fmin(0.0, sg * ft[i]) * invA;
      }
    }
    if (act) {
      double scale_factor = (smx * rhoref - snew) / (sin_ + eps);
      const double scale_in = fmin(1.0, fmax(0.0, scale_factor));
      scale_factor = (smn * rhoref - snew) / (sout - eps);
      const double scale_out = fmin(1.0, fmax(0.0, scale_factor));
      double* sa = q ? s2.scale_arr : p.scale_arr;
      (q ? s2.scalar_old_copy : p.scalar_old_copy)[o] = snew;  // upwind solution (the reference's scalar_new)
      sa[((size_t)c * 2 + 0) * K + k] = scale_in;
      sa[((size_t)c * 2 + 1) * K + k] = scale_out;
    }
  }
}

template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_mono_cells2_b(Dims d, Ptrs p, int is, int advance_density,
                                                                  int nq = 1, MonoCell2 s2 = MonoCell2{},
                                                                  double* flux_arr2 = nullptr) {
  const int c = wave_elem(0);
  if (c >= d.nCells) return;
  const int k = lane_id(), K = d.K, ns = d.ns;
  const bool act = k < K;
  const int kc = min(k, K - 1), kw = min(k, K);
  const size_t K1 = K + 1;
  const size_t o = (size_t)c * K + kc, ow = (size_t)c * K1 + kw;
  // only cells with bdyMaskCell <= nSpecZone get the update copied back (4205; the reference tests
  // the mask whether or not config_apply_lbcs is set, as at 2292, 3069 and 3435)
  if (p.bdyMaskCell[c] > N_SPEC_ZONE) return;
  if (c >= d.nCellsSolve) {  // halo cells: scalars_new = max(0, scalar_new) with scalar_new = input copy
    for (int q = 0; q < nq; ++q)
      if (act) p.scalars2[SIX(c, k, is + q)] = fmax(0.0, p.scalars2[SIX(c, k, is + q)]);
    return;
  }
  const CellSten<ME> st = load_sten<ME>(p, c);
  const double invA = ld_uniform_f64(p.invAreaCell + c);
  const double rhoref = advance_density ? p.rho_zz_int[o] : p.rho_zz2[o];
  const double rdzw = p.rdzw[kc];
  // nq = 2: the pair's second scalar (is + 1) from the second scratch set (s2, flux_arr2), after the first
#pragma unroll 1
  for (int q = 0; q < nq; ++q) {
    const double* sa = q ? s2.scale_arr : p.scale_arr;
    const double* far = q ? flux_arr2 : p.flux_arr;
    double si = sa[((size_t)c * 2 + 0) * K + kc], so_ = sa[((size_t)c * 2 + 1) * K + kc];
    double wd = (q ? s2.wdtn : p.wdtn)[ow];
    const double sold_copy = (q ? s2.scalar_old_copy : p.scalar_old_copy)[o];
    double fa[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) fa[i] = far[(size_t)st.e[i] * K + kc];
    if (!act) {
      si = 0.0;
      so_ = 0.0;
    }
    if (k > K) wd = 0.0;
    const double sim = up1(si), som = up1(so_);
    if (act && k >= 1) {
      const double f = wd;
      wd = fmax(0.0, f) * fmin(som, si) + fmin(0.0, f) * fmin(so_, sim);
    }
    const double wdp = dn1(wd);
    if (!act) continue;
    double snew = sold_copy;
#pragma unroll
    for (int i = 0; i < ME; ++i)
      if (i < st.ne) snew = snew - st.sg(i) * fa[i] * invA;
    snew = (snew + (-rdzw * (wdp - wd))) / rhoref;
    p.scalars2[SIX(c, k, is + q)] = fmax(0.0, snew);
  }
}

template <bool ODD = false>
__global__ __launch_bounds__(PAIR_THREADS) void k_mono_edges2_p(Dims d, Ptrs p, double dt) {
  const int eA = PAIR_EPW * pair_wave();
  if (eA >= d.nEdges) return;
  const bool hasB = PAIR_EPW == 2 && eA + 1 < d.nEdges;
  const int eB = hasB ? eA + 1 : eA;
  const int K = d.K, h = pair_half(), l = pair_lane();
  const int lc = min(l, (ODD ? K + 1 : K) / 2 - 1);
  const bool two = !ODD || 2 * l + 1 < K;  // odd K: the last pair holds level K-1 only
  const int e = sel(h, eA, eB);
  const size_t o = (size_t)e * K + 2 * lc;
  const int2 ceA = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eA);
  const int2 ceB = *reinterpret_cast<const int2*>(p.cellsOnEdge + 2 * eB);
  const d2 fa = ld2(p.flux_arr + o), fu = ld2(p.flux_upwind_tmp + o);
  const bool onA = ceA.x < d.nCellsSolve || ceA.y < d.nCellsSolve;
  const bool onB = hasB && (ceB.x < d.nCellsSolve || ceB.y < d.nCellsSolve);
  if (!onA && !onB) return;
  const int c1 = sel(h, ceA.x, ceB.x), c2 = sel(h, ceA.y, ceB.y);
  auto sc = [&](int cc, int io) {
    const d2 v = ld2(p.scale_arr + ((size_t)cc * 2 + io) * K + 2 * lc);
    return cc < d.nCells ? v : d2{0.0, 0.0};
  };
  const d2 a10 = sc(c1, 0), a11 = sc(c1, 1), a20 = sc(c2, 0), a21 = sc(c2, 1);
  d2 f{dt * fa.x - fu.x, dt * fa.y - fu.y};
  const int bm = sel(h, p.bdyMaskEdge[eA], p.bdyMaskEdge[eB]);
  if ((d.lbc && bm == N_RELAX_ZONE) || bm == N_RELAX_ZONE - 1) f = d2{0.0, 0.0};  // 4113-4115
  f.x = fmax(0.0, f.x) * fmin(a11.x, a20.x) + fmin(0.0, f.x) * fmin(a10.x, a21.x);
  f.y = fmax(0.0, f.y) * fmin(a11.y, a20.y) + fmin(0.0, f.y) * fmin(a10.y, a21.y);
  if ((h ? onB : onA) && 2 * l < K) pst(p.flux_arr + o, f, two);
}

// ============================================================================
// mpas_reconstruct_2d  (operators/mpas_vector_reconstruction.F:245-294), owned cells:
// cell-centre velocity from the edge normals with the precomputed RBF weights
// coeffs_reconstruct(R3, maxEdges, nCells), then its zonal / meridional components.
// ============================================================================
__global__ __launch_bounds__(BLOCK_THREADS) void k_reconstruct(Dims d, Ptrs p, const double* __restrict__ u) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K;
  if (k >= K) return;
  double x = 0.0, y = 0.0, z = 0.0;
  const int ne = p.nEdgesOnCell[c];
  for (int i = 0; i < ne; ++i) {
    const int e = uni(p.edgesOnCell[c * d.maxEdges + i]);
    const double* cf = p.coeffs_reconstruct + ((size_t)c * d.maxEdges + i) * 3;
    const double ue = u[(size_t)e * K + k];
    x = x + cf[0] * ue;
    y = y + cf[1] * ue;
    z = z + cf[2] * ue;
  }
  const size_t o = (size_t)c * K + k;
  p.uReconstructX[o] = x;
  p.uReconstructY[o] = y;
  p.uReconstructZ[o] = z;
  const double clat = cos(p.latCell[c]), slat = sin(p.latCell[c]);
  const double clon = cos(p.lonCell[c]), slon = sin(p.lonCell[c]);
  p.uReconstructZonal[o] = -x * slon + y * clon;
  p.uReconstructMeridional[o] = -(x * clon + y * slon) * slat + z * clat;
}


// k_reconstruct on the per-cell stencil record (ME = maxEdges, 6 or 7): the edge indices come from
// the record in one scalar round trip, the ME columns of u and the coefficient rows are issued
// together (slots beyond nEdgesOnCell name the garbage edge and are not summed), then the sums in
// the reference order (mpas_vector_reconstruction.F:245-294)
template <int ME>
__global__ __launch_bounds__(BLOCK_THREADS) void k_reconstruct_b(Dims d, Ptrs p, const double* __restrict__ u) {
  const int c = wave_elem(0);
  if (c >= d.nCellsSolve) return;
  const int k = lane_id(), K = d.K;
  const int kc = min(k, K - 1);
  const CellSten<ME> st = load_sten<ME>(p, c);
  double ue[ME], cx[ME], cy[ME], cz[ME];
#pragma unroll
  for (int i = 0; i < ME; ++i) ue[i] = u[(size_t)st.e[i] * K + kc];
  const double* cf = p.coeffs_reconstruct + (size_t)c * ME * 3;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    cx[i] = ld_uniform_f64(cf + 3 * i);
    cy[i] = ld_uniform_f64(cf + 3 * i + 1);
    cz[i] = ld_uniform_f64(cf + 3 * i + 2);
  }
  const double lat = ld_uniform_f64(p.latCell + c), lon = ld_uniform_f64(p.lonCell + c);
  double x = 0.0, y = 0.0, z = 0.0;
#pragma unroll
  for (int i = 0; i < ME; ++i) {
    if (i < st.ne) {
      x = x + cx[i] * ue[i];
      y = y + cy[i] * ue[i];
      z = z + cz[i] * ue[i];
    }
  }
  if (k >= K) return;
  const size_t o = (size_t)c * K + k;
  p.uReconstructX[o] = x;
  p.uReconstructY[o] = y;
  p.uReconstructZ[o] = z;
  const double clat = cos(lat), slat = sin(lat);
  const double clon = cos(lon), slon = sin(lon);
  p.uReconstructZonal[o] = -x * slon + y * clon;
  p.uReconstructMeridional[o] = -(x * clon + y * slon) * slat + z * clat;
}

}  // namespace mpas
