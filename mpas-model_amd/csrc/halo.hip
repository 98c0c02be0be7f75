// Halo exchange pack / unpack kernels (mpas_dmpar_exch_halo_field, framework/mpas_dmpar.F).
//
// An exchange point moves, for every peer block, the halo columns of one or
// more fields.  The host builds a segment table per block (one segment = one
// field x one halo layer x one peer); blockIdx.y selects the segment and each
// wavefront moves one element column (inner = K, K+1, 2K or num_scalars*K
// doubles) with contiguous, coalesced lane accesses on both sides.
#pragma once
#include "dycore.h"

namespace mpas {

struct XSeg {
  double* base;       // field buffer (element-major, `inner` doubles per element)
  const int* idx;     // 0-based local element index, message order
  int n;              // elements
  int inner;          // doubles per element
  long long off;      // offset of this segment in the message buffer (doubles)
};

__global__ __launch_bounds__(256) void k_halo_pack(const XSeg* __restrict__ segs, double* __restrict__ buf) {
  const XSeg* s = segs + blockIdx.y;
  const int n = s->n;
  const int i = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (i >= n) return;
  const int inner = s->inner;
  const int e = __builtin_amdgcn_readfirstlane(s->idx[i]);
  const double* src = s->base + (size_t)e * inner;
  double* dst = buf + s->off + (size_t)i * inner;
  for (int j = threadIdx.x & 63; j < inner; j += 64) dst[j] = src[j];
}

__global__ __launch_bounds__(256) void k_halo_unpack(const XSeg* __restrict__ segs, const double* __restrict__ buf) {
  const XSeg* s = segs + blockIdx.y;
  const int n = s->n;
  const int i = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (i >= n) return;
  const int inner = s->inner;
  const int e = __builtin_amdgcn_readfirstlane(s->idx[i]);
  double* dst = s->base + (size_t)e * inner;
  const double* src = buf + s->off + (size_t)i * inner;
  for (int j = threadIdx.x & 63; j < inner; j += 64) dst[j] = src[j];
}

}  // namespace mpas
