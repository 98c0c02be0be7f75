// summarize_timestep (mpas_atm_time_integration.F:6675-7018) on the device.
//
// The reference ends every atm_srk3 (1794) with global extrema of the new state:
//   * config_print_global_minmax_vel (default true, 6945-6983): min/max of w and u over the
//     owned elements, both starting from 0.0, reduced over ranks (mpas_dmpar_min/max_real);
//   * config_print_detailed_minmax_vel (6721-6943): the first (cell, level) in loop order that
//     holds the extreme of w, u and the wind speed sqrt(u^2 + v^2), with its level and lat/lon,
//     reduced over ranks with MPI_MINLOC / MPI_MAXLOC (mpas_dmpar_min/maxattributes_real,
//     mpas_dmpar.F:1090-1160), and a NaN check on w and u that aborts (MPAS_LOG_CRIT);
//   * config_print_global_minmax_sca (6986-7016): per scalar min/max, starting from 0.0.
//
// Here one launch reduces all of a block's fields (blockIdx.y = field) into per-workgroup
// partial records, and a second launch folds the partials of each field.  The located extrema
// are ordered by (value, linear index c*K + k): the reference's loop keeps the first element of
// its cell-major / level-minor order that beats the running value by a strict comparison, i.e.
// the smallest linear index among the elements equal to the extreme, so any reduction tree
// gives the reference's element.  A value has to beat the start value (1e20 / -1e20) to count,
// as with the strict comparison there.
#pragma once
#include "dycore.h"

namespace mpas {

constexpr int SUM_REC = 16;         // doubles per field record
constexpr int SUM_MAX_FIELDS = 40;  // fields per launch
constexpr int SUM_PARTS = 1024;     // workgroups per field in the first pass
constexpr int SUM_UNROLL = 4;       // columns whose loads a wavefront issues together

// record slots
enum {
  SR_MIN = 0, SR_IMIN, SR_MAX, SR_IMAX,  // located extrema and their linear index (-1: none)
  SR_MIN0, SR_MAX0,                        // min / max starting from 0.0
  SR_NAN,                                  // NaN count
  SR_SPD, SR_ISPD,                         // max sqrt(u^2 + v^2) and its index (fields with v)
  SR_LAT_MIN, SR_LON_MIN, SR_LAT_MAX, SR_LON_MAX, SR_LAT_SPD, SR_LON_SPD,  // at the extrema
  SR_COUNT                                 // elements reduced
};

struct SumField {
  const double* a;    // column-major field, column stride `stride` doubles
  const double* v;    // optional second field for the wind speed (same layout), or null
  const double* lat;  // per-column latitude / longitude, or null
  const double* lon;
  long long ncol;     // owned columns
  int K;              // levels reduced per column (k = 0..K-1)
  int stride;
};
struct SumFields {
  SumField f[SUM_MAX_FIELDS];
};

struct SumAcc {
  double mn, mx, m0, M0, spd, nan, cnt;
  long long imn, imx, ispd;
  __device__ void init() {
    mn = 1.0e20; mx = -1.0e20; m0 = 0.0; M0 = 0.0; spd = -1.0e20; nan = 0.0; cnt = 0.0;
    imn = imx = ispd = -1;
  }
  // (value, index) orders: the smaller index wins a tie; index -1 = nothing found yet
  __device__ static bool better_min(double v, long long i, double bv, long long bi) {
    return bi < 0 || v < bv || (v == bv && i < bi);
  }
  __device__ static bool better_max(double v, long long i, double bv, long long bi) {
    return bi < 0 || v > bv || (v == bv && i < bi);
  }
  __device__ void add(double x, double spd_x, long long i) {
    if (x < 1.0e20 && better_min(x, i, mn, imn)) { mn = x; imn = i; }
    if (x > -1.0e20 && better_max(x, i, mx, imx)) { mx = x; imx = i; }
    if (x < m0) m0 = x;  // scalar_min = min(scalar_min, x), scalar_max = max(scalar_max, x) (6962-6963)
    if (x > M0) M0 = x;
    if (spd_x > -1.0e20 && better_max(spd_x, i, spd, ispd)) { spd = spd_x; ispd = i; }
    if (x != x) nan += 1.0;
    cnt += 1.0;
  }
  __device__ void merge(const SumAcc& o) {
    if (o.imn >= 0 && better_min(o.mn, o.imn, mn, imn)) { mn = o.mn; imn = o.imn; }
    if (o.imx >= 0 && better_max(o.mx, o.imx, mx, imx)) { mx = o.mx; imx = o.imx; }
    if (o.m0 < m0) m0 = o.m0;
    if (o.M0 > M0) M0 = o.M0;
    if (o.ispd >= 0 && better_max(o.spd, o.ispd, spd, ispd)) { spd = o.spd; ispd = o.ispd; }
    nan += o.nan;
    cnt += o.cnt;
  }
};

__device__ void sum_block_reduce(SumAcc& a) {
  __shared__ double sd[4][7];
  __shared__ long long sl[4][3];
  for (int off = 32; off >= 1; off >>= 1) {  // wavefront butterfly
    const int src = (threadIdx.x & 63) ^ off;
    SumAcc o;
    o.mn = __shfl(a.mn, src, 64); o.mx = __shfl(a.mx, src, 64); o.m0 = __shfl(a.m0, src, 64);
    o.M0 = __shfl(a.M0, src, 64); o.spd = __shfl(a.spd, src, 64); o.nan = __shfl(a.nan, src, 64);
    o.cnt = __shfl(a.cnt, src, 64);
    o.imn = __shfl(a.imn, src, 64); o.imx = __shfl(a.imx, src, 64); o.ispd = __shfl(a.ispd, src, 64);
    a.merge(o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sd[w][0] = a.mn; sd[w][1] = a.mx; sd[w][2] = a.m0; sd[w][3] = a.M0; sd[w][4] = a.spd; sd[w][5] = a.nan;
    sd[w][6] = a.cnt;
    sl[w][0] = a.imn; sl[w][1] = a.imx; sl[w][2] = a.ispd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      SumAcc o;
      o.mn = sd[i][0]; o.mx = sd[i][1]; o.m0 = sd[i][2]; o.M0 = sd[i][3]; o.spd = sd[i][4]; o.nan = sd[i][5];
      o.cnt = sd[i][6];
      o.imn = sl[i][0]; o.imx = sl[i][1]; o.ispd = sl[i][2];
      a.merge(o);
    }
  }
}

__device__ void sum_store(double* r, const SumAcc& a) {
  r[SR_MIN] = a.mn; r[SR_IMIN] = (double)a.imn; r[SR_MAX] = a.mx; r[SR_IMAX] = (double)a.imx;
  r[SR_MIN0] = a.m0; r[SR_MAX0] = a.M0; r[SR_NAN] = a.nan; r[SR_SPD] = a.spd; r[SR_ISPD] = (double)a.ispd;
  r[SR_COUNT] = a.cnt;
}
__device__ SumAcc sum_load(const double* r) {
  SumAcc a;
  a.mn = r[SR_MIN]; a.imn = (long long)r[SR_IMIN]; a.mx = r[SR_MAX]; a.imx = (long long)r[SR_IMAX];
  a.m0 = r[SR_MIN0]; a.M0 = r[SR_MAX0]; a.nan = r[SR_NAN]; a.spd = r[SR_SPD]; a.ispd = (long long)r[SR_ISPD];
  a.cnt = r[SR_COUNT];
  return a;
}

// pass 1: grid (SUM_PARTS, nfields); a wavefront walks whole columns, lane = level, and issues
// the loads of SUM_UNROLL columns before reducing them (the reduction is order-free: extrema with
// index tie-breaks, integer counts)
__global__ __launch_bounds__(256) void k_summary_partial(SumFields fs, double* __restrict__ part) {
  const SumField& f = fs.f[blockIdx.y];
  SumAcc a;
  a.init();
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  for (int k0 = 0; k0 < f.K; k0 += 64) {
    const int k = k0 + lane;
    const bool lv = k < f.K;
    for (long long c0 = wave; c0 < f.ncol; c0 += nw * SUM_UNROLL) {
      double x[SUM_UNROLL], y[SUM_UNROLL];
#pragma unroll
      for (int u = 0; u < SUM_UNROLL; ++u) {
        const long long c = c0 + u * nw;
        const bool ok = lv && c < f.ncol;
        x[u] = ok ? f.a[c * f.stride + k] : 0.0;
        y[u] = (ok && f.v) ? f.v[c * f.stride + k] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < SUM_UNROLL; ++u) {
        const long long c = c0 + u * nw;
        if (!lv || c >= f.ncol) continue;
        double s = -1.0e30;  // below the start value: no wind-speed candidate
        if (f.v) s = sqrt(x[u] * x[u] + y[u] * y[u]);  // spd = sqrt(u*u + v*v) (6893)
        a.add(x[u], s, c * f.K + k);
      }
    }
  }
  sum_block_reduce(a);
  if (threadIdx.x == 0) sum_store(part + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * SUM_REC, a);
}

// pass 2: one workgroup per field folds its partial records and picks up the lat/lon of each
// located extreme (column = index / K)
__global__ __launch_bounds__(256) void k_summary_final(SumFields fs, const double* __restrict__ part, int nparts,
                                                       double* __restrict__ out) {
  const SumField& f = fs.f[blockIdx.x];
  SumAcc a;
  a.init();
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) a.merge(sum_load(part + ((size_t)blockIdx.x * nparts + i) * SUM_REC));
  sum_block_reduce(a);
  if (threadIdx.x == 0) {
    double* r = out + (size_t)blockIdx.x * SUM_REC;
    sum_store(r, a);
    auto at = [&](long long idx, int slat, int slon) {
      r[slat] = 0.0;  // latMax = lonMax = 0.0 when nothing was found (6745-6746)
      r[slon] = 0.0;
      if (idx >= 0 && f.lat) {
        r[slat] = f.lat[idx / f.K];
        r[slon] = f.lon[idx / f.K];
      }
    };
    at(a.imn, SR_LAT_MIN, SR_LON_MIN);
    at(a.imx, SR_LAT_MAX, SR_LON_MAX);
    at(a.ispd, SR_LAT_SPD, SR_LON_SPD);
  }
}

}  // namespace mpas
