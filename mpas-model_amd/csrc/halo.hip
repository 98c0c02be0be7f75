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

// ---------------------------------------------------------------------------
// One-sided halo transfer between the ranks of one node (MPAS_DYCORE_P2P): the messages of an
// exchange point are pulled over xGMI by the receiving rank's kernel, with no RCCL group, no second
// stream and no host involvement, so a step stays one captured graph of kernels.
//
// Per exchange point and rank: a send buffer in ordinary device memory (the producer's stores are in
// memory once its kernel has ended: the L2 write-back that makes them visible to the other XCDs),
// mapped into every peer that reads it (IPC); and a flag arena in uncached memory per rank,
// [plan][sender rank][ready, consumed].  A use n
// of an exchange point (the n-th time the step runs it; every rank runs the same sequence):
//   k_p2p_post (after the pack or the fused producer): n = ++use counter; ready[plan][me] = n in the
//     arena of every rank this rank sends to;
//   k_p2p_get (where the halo is needed): per peer, wait for ready[plan][peer] >= n in this rank's
//     arena, copy the peer's message from its send buffer into this rank's receive buffer (ordinary
//     device memory: the unpack or the fused consumer reads it as before), and when the last chunk
//     of that peer is in, set consumed[plan][me] = n in the peer's arena; one more workgroup waits
//     for consumed[plan][r] >= n from every rank r this rank sends to, so the kernel ends only when
//     this rank's send buffer may be written again (the next use's producer comes after it).
// Every rank raises its flags before it waits on its peers', and all ranks run the exchange points
// in one order, so the waits resolve.  A wait that has not resolved after 30 s (P2P_TIMEOUT_TICKS) sets
// the context's status word and gives up (and so does every later wait): the host reports the error
// (mpas_dyc_synchronize) instead of a hung GPU.
constexpr unsigned long long P2P_TIMEOUT_TICKS = 30ull * 100000000ull;  // wall_clock64 runs at 100 MHz
constexpr int P2P_CHUNK = 4096;                                          // doubles per workgroup

struct P2PGet {
  const double* src;                  // the peer's send buffer: its message to this rank
  double* dst;                        // this rank's receive buffer: the message from that peer
  long long count;                    // doubles
  const unsigned long long* ready;    // raised by the peer's post (this rank's arena)
  unsigned long long* consumed;       // raised here once the message is copied (the peer's arena)
  unsigned long long* done;           // chunks copied so far, over all uses (local)
  int nchunk;
};

// The flags are uncached memory: the waits poll with relaxed system-scope loads and the signals are
// relaxed system-scope stores, with no release fence (a write-back of the whole L2: 4.7 us per post
// with one).  The data a post announces was stored by earlier kernels on the stream (in memory when
// they end); after its poll has seen the flag, a copy workgroup runs one system-scope acquire and
// reads the peer's buffer with system-scope loads, so no cache of this GPU serves a stale copy of
// it; and a consumed flag is raised after every copy load of the message has returned its value.
// (Send buffers in uncached memory gave a peer process stale halo values in about one run in four
// with two ranks on one GPU, whatever the reading side did: the producers' stores into them were not
// all in memory when the next kernel raised the ready flag -- a release fence at the end of the pack
// cured it, and so does ordinary memory; tools/p2p_repeat.sh.)
__device__ inline bool p2p_wait_geq(const unsigned long long* f, unsigned long long n, int* status) {
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < n) {
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (wall_clock64() - t0 > P2P_TIMEOUT_TICKS) {
      atomicOr(status, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  return true;
}

// a system-scope load of a double: the peer's data as it is in memory, whatever a cache of this GPU
// holds from an earlier exchange (an IPC mapping of another process's memory need not be uncached)
__device__ inline double sys_load(const double* a) {
  const unsigned long long v = __hip_atomic_load((const unsigned long long*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return __longlong_as_double((long long)v);
}

// use[0]: this exchange point's use counter (read by the get of the same use, later on the stream)
__global__ __launch_bounds__(64) void k_p2p_post(unsigned long long* use, unsigned long long* const* ready, int npeer) {
  const unsigned long long n = use[0] + 1;
  __syncthreads();
  if (threadIdx.x == 0) use[0] = n;
  for (int i = threadIdx.x; i < npeer; i += 64) __hip_atomic_store(ready[i], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// grid (max chunks, nget + 1): row y < nget pulls chunk x of peer y; row nget waits for the peers
// that pull from this rank (one lane per peer)
__global__ __launch_bounds__(256) void k_p2p_get(const P2PGet* __restrict__ g, int nget,
                                                 const unsigned long long* const* consumed, int ncons,
                                                 const unsigned long long* use, int* status) {
  const unsigned long long n = use[0];
  if ((int)blockIdx.y == nget) {
    if (blockIdx.x == 0 && (int)threadIdx.x < ncons) (void)p2p_wait_geq(consumed[threadIdx.x], n, status);
    return;
  }
  const P2PGet& p = g[blockIdx.y];
  if ((int)blockIdx.x >= p.nchunk) return;
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = p2p_wait_geq(p.ready, n, status);
    // as in k_p2p_pull: one system-scope acquire after the poll, then system-scope loads of the
    // peer's buffer (another process's memory, mapped here over IPC)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (!ok) return;
  const long long c0 = (long long)blockIdx.x * P2P_CHUNK;
  const long long c1 = min(p.count, c0 + P2P_CHUNK);
  // four loads in flight per lane before the stores (the source is another GPU's memory)
  for (long long i = c0 + threadIdx.x; i < c1; i += 4 * 256) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < c1 ? sys_load(p.src + i + u * 256) : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < c1) p.dst[i + u * 256] = v[u];
  }
  __syncthreads();  // every lane's loads have returned (their values are stored)
  if (threadIdx.x == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(p.done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old + 1 == n * (unsigned long long)p.nchunk)
      __hip_atomic_store(p.consumed, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A blocking exchange (post then get, nothing between them): both in one launch.  Every row's first
// workgroup raises the ready flags before it waits for anything (the send buffer was completed by the
// kernels before this one), so no workgroup depends on another being scheduled first; the use
// counter is read by every workgroup at its start and advanced by the last one to finish
// (use[1 + nget] counts finished workgroups over all uses).
__global__ __launch_bounds__(256) void k_p2p_exchange(const P2PGet* __restrict__ g, int nget,
                                                      unsigned long long* const* ready, int nready,
                                                      const unsigned long long* const* consumed, int ncons,
                                                      unsigned long long* use, int* status) {
  const unsigned long long n = use[0] + 1;
  if (blockIdx.x == 0 && (int)threadIdx.x < nready)
    __hip_atomic_store(ready[threadIdx.x], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if ((int)blockIdx.y == nget) {
    if (blockIdx.x == 0 && (int)threadIdx.x < ncons) (void)p2p_wait_geq(consumed[threadIdx.x], n, status);
  } else {
    const P2PGet& p = g[blockIdx.y];
    if ((int)blockIdx.x < p.nchunk) {
      __shared__ int ok;
      if (threadIdx.x == 0) {
        ok = p2p_wait_geq(p.ready, n, status);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // as in k_p2p_get
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (ok) {
        const long long c0 = (long long)blockIdx.x * P2P_CHUNK;
        const long long c1 = min(p.count, c0 + P2P_CHUNK);
        for (long long i = c0 + threadIdx.x; i < c1; i += 4 * 256) {
          double v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < c1 ? sys_load(p.src + i + u * 256) : 0.0;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (i + u * 256 < c1) p.dst[i + u * 256] = v[u];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          const unsigned long long old = __hip_atomic_fetch_add(p.done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (old + 1 == n * (unsigned long long)p.nchunk)
            __hip_atomic_store(p.consumed, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long total = (unsigned long long)gridDim.x * gridDim.y;
    const unsigned long long old = __hip_atomic_fetch_add(use + 1 + nget, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old + 1 == n * total) __hip_atomic_store(use, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Pull exchange (blocking one-sided exchanges with block-pair lists): the receiving rank copies each
// peer's owned columns straight from the peer's field (IPC-mapped) into its own halo columns -- the
// peer's pack segment and this rank's unpack segment of one message slot, fused -- so an exchange is
// this one launch: no pack, no send or receive buffer, no unpack.  The protocol is k_p2p_exchange's:
// ready raised at the start (the peer's field is final: its producer has ended), per peer the last
// workgroup raises consumed, and the kernel ends only when every rank that reads this rank's fields
// has finished (the next kernel may overwrite them).  The peer's field is ordinary device memory:
// its producer's stores reach memory when that kernel ends (the L2 write-back that makes them
// visible to the other XCDs), and the loads here are system-scope so that no cache of this GPU
// holds a stale copy from the previous exchange.
struct P2PSeg {
  const double* src;  // the peer's field (mapped), sub-field base
  double* dst;        // this rank's field
  const int* sidx;    // the peer's send list (0-based owned elements), a copy in this rank's memory
  const int* didx;    // this rank's receive list (halo elements)
  int n, inner, peer;
};
struct P2PPeer {
  const unsigned long long* ready;  // raised by the peer (this rank's arena)
  unsigned long long* consumed;     // raised here when all of the peer's segments are copied (its arena)
  unsigned long long* done;         // workgroups done, over all uses (local)
  unsigned long long nwg;           // workgroups per use with work for this peer
};


constexpr int P2P_PULL_COLS = 16;  // element columns per workgroup (4 per wave)

// grid (nchunk + 1): workgroup x < nchunk copies columns chunk[x].y .. +15 of segment chunk[x].x (a
// chunk never spans two segments, so one peer); workgroup nchunk waits for the ranks that read this
// rank's fields.  Completion is counted per peer (one atomic per workgroup) and, by the last
// workgroup of each peer and the waiting one, per launch: the last of those advances the use
// counter, after every workgroup has read it.
__global__ __launch_bounds__(256) void k_p2p_pull(const P2PSeg* __restrict__ segs, const int2* __restrict__ chunk,
                                                  int nchunk, const P2PPeer* __restrict__ peers, int npeer_work,
                                                  unsigned long long* const* ready, int nready,
                                                  const unsigned long long* const* consumed, int ncons,
                                                  unsigned long long* use, int* status) {
  const unsigned long long n = use[0] + 1;
  bool last = false;  // this workgroup closes a peer (or is the waiting one)
  if ((blockIdx.x == 0 || (int)blockIdx.x == nchunk) && (int)threadIdx.x < nready)
    __hip_atomic_store(ready[threadIdx.x], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if ((int)blockIdx.x == nchunk) {
    if ((int)threadIdx.x < ncons) (void)p2p_wait_geq(consumed[threadIdx.x], n, status);
    last = true;
  } else {
    const int2 ch = chunk[blockIdx.x];
    const P2PSeg& sg = segs[ch.x];
    const P2PPeer& pr = peers[sg.peer];
    __shared__ int ok;
    if (threadIdx.x == 0) {
      ok = p2p_wait_geq(pr.ready, n, status);
      // the peer's field is ordinary (cacheable) memory: one system-scope acquire per workgroup after
      // the poll, so that no line of it this GPU cached at an earlier exchange is read again
      // (MI355X_MICROARCH.md, consumer: one relaxed poll, one acquire, vmcnt(0), barrier)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (ok) {
      // the wave's four columns: every load issued before the first store (over xGMI each is a
      // round trip of a microsecond or more); columns of up to 64 levels in one load per lane,
      // taller ones (the wide builds) in a loop
      const int inner = sg.inner, lane = threadIdx.x & 63;
      constexpr int NC = P2P_PULL_COLS / 4;
      int di[NC];
      const double* src[NC];
      double v[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = __builtin_amdgcn_readfirstlane(ch.y + c * 4 + (int)(threadIdx.x >> 6));
        const bool in = i < sg.n;
        const int si = in ? __builtin_amdgcn_readfirstlane(sg.sidx[i]) : 0;
        di[c] = in ? __builtin_amdgcn_readfirstlane(sg.didx[i]) : -1;
        src[c] = sg.src + (size_t)si * inner;
        v[c] = (in && lane < inner) ? sys_load(src[c] + lane) : 0.0;
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (di[c] < 0) continue;
        double* dst = sg.dst + (size_t)di[c] * inner;
        if (lane < inner) dst[lane] = v[c];
        for (int j = lane + 64; j < inner; j += 64) dst[j] = sys_load(src[c] + j);
      }
    }
    __syncthreads();  // every lane's loads have returned
    if (threadIdx.x == 0) {
      const unsigned long long old = __hip_atomic_fetch_add(pr.done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (old + 1 == n * pr.nwg) {
        __hip_atomic_store(pr.consumed, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        last = true;
      }
    }
  }
  if (threadIdx.x == 0 && last) {
    const unsigned long long old = __hip_atomic_fetch_add(use + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old + 1 == n * (unsigned long long)(npeer_work + 1))
      __hip_atomic_store(use, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
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
