// Halo exchange kernel (mpas_dmpar_exch_halo_field, framework/mpas_dmpar.F).
//
// An exchange point is a list of segments. One segment = one field x one halo
// layer x one peer block, and it comes in three kinds:
//   * pack: owned columns -> an RCCL send buffer;
//   * unpack: an RCCL receive buffer -> halo columns;
//   * direct: owned columns of one block -> halo columns of another block of
//     the same process.
// blockIdx.y selects the segment. Each wavefront moves one element column
// (inner = K, K+1, 2K or num_scalars*K doubles) with contiguous lane accesses
// on both sides. Reads only touch owned columns and writes only halo columns,
// so all segments of a launch are independent.
#pragma once
#include "dycore.h"

namespace mpas {

struct XSeg {
  const double* src;  // field (sidx != null) or contiguous buffer
  double* dst;        // field (didx != null) or contiguous buffer
  const int* sidx;    // 0-based source element per message slot, or null (slot i = column i)
  const int* didx;    // 0-based destination element per message slot, or null
  int n;              // elements
  int inner;          // doubles per element
};

__global__ __launch_bounds__(256) void k_halo_copy(const XSeg* __restrict__ segs) {
  const XSeg* s = segs + blockIdx.y;
  const int i = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (i >= s->n) return;
  const int inner = s->inner;
  const int si = s->sidx ? __builtin_amdgcn_readfirstlane(s->sidx[i]) : i;
  const int di = s->didx ? __builtin_amdgcn_readfirstlane(s->didx[i]) : i;
  const double* src = s->src + (size_t)si * inner;
  double* dst = s->dst + (size_t)di * inner;
  for (int j = threadIdx.x & 63; j < inner; j += 64) dst[j] = src[j];
}

// atm_rk_integration_setup (mpas_atm_time_integration.F:1847-1857): the ten state/diag
// copies of one block in a single launch; blockIdx.y selects the copy.
struct CopyList {
  const double* src[10];
  double* dst[10];
  long long n[10];
};

__global__ __launch_bounds__(256) void k_copy_many(CopyList c) {
  const int j = blockIdx.y;
  const long long n = c.n[j];
  const double* __restrict__ src = c.src[j];
  double* __restrict__ dst = c.dst[j];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) dst[i] = src[i];
}

}  // namespace mpas
