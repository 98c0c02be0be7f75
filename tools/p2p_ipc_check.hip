// Two processes on one GPU run the library's one-sided halo protocol (halo.hip: k_p2p_post /
// k_p2p_get) against each other through IPC mappings of uncached memory, as two ranks of a node do
// over xGMI.  Each iteration: a fill kernel writes this rank's send buffer with a pattern of (iteration,
// rank), the post raises the ready flag in the peer's arena, the get pulls the peer's buffer into
// ordinary device memory (raising the peer's consumed flag and waiting for its own), and a check kernel
// counts the received doubles that are not the peer's pattern of that iteration.  No host
// synchronisation between iterations: the next fill overwrites the send buffer right after the get,
// which is safe only if the consumed flags work.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpas-model_amd/csrc -I include tools/p2p_ipc_check.hip -o tools/p2p_ipc_check
//   python tools/p2p_ipc_check.py         (starts the two processes with a rendezvous directory)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "halo.hip"

using namespace mpas;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "rank %d: %s: %s\n", rank, #x, hipGetErrorString(e_));                  \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

__device__ inline double pattern(long long it, int rank, long long i) {
  return (double)(it * 1000003 + rank * 7919) + (double)i * 0.5;
}

__global__ void k_fill(double* b, long long n, long long it, int rank) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = pattern(it, rank, i);
}

__global__ void k_check(const double* b, long long n, long long it, int peer, unsigned long long* bad) {
  unsigned long long nb = 0;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) nb += b[i] != pattern(it, peer, i);
  if (nb) atomicAdd(bad, nb);
}

static bool write_file(const std::string& path, const void* p, size_t n) {
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;
  const bool ok = fwrite(p, 1, n, f) == n;
  fclose(f);
  return ok && rename(tmp.c_str(), path.c_str()) == 0;
}

static bool read_file(const std::string& path, void* p, size_t n, int timeout_s) {
  for (int t = 0; t < timeout_s * 100; ++t) {
    if (FILE* f = fopen(path.c_str(), "rb")) {
      const bool ok = fread(p, 1, n, f) == n;
      fclose(f);
      if (ok) return true;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return false;
}

int run_pull(int rank, const std::string& dir, long long n, long long iters);

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s RANK(0|1) DIR [doubles] [iterations] [buffers|pull]\n", argv[0]);
    return 2;
  }
  const int rank = atoi(argv[1]), peer = 1 - rank;
  const std::string dir = argv[2];
  const long long n = argc > 3 ? atoll(argv[3]) : 100000;
  const long long iters = argc > 4 ? atoll(argv[4]) : 2000;
  if (argc > 5 && std::string(argv[5]) == "pull") return run_pull(rank, dir, n, iters);
  double *send = nullptr, *recv = nullptr;
  unsigned long long *flags = nullptr, *cnt = nullptr, *bad = nullptr;
  int* status = nullptr;
  CK(hipMalloc(&send, n * sizeof(double)));  // ordinary device memory, as the library's send buffers
  CK(hipExtMallocWithFlags((void**)&flags, 4 * sizeof(unsigned long long), hipDeviceMallocUncached));
  CK(hipMemset(flags, 0, 4 * sizeof(unsigned long long)));
  CK(hipMalloc(&recv, n * sizeof(double)));
  CK(hipMalloc(&cnt, 2 * sizeof(unsigned long long)));
  CK(hipMemset(cnt, 0, 2 * sizeof(unsigned long long)));
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  CK(hipMemset(bad, 0, sizeof(unsigned long long)));
  CK(hipMalloc(&status, sizeof(int)));
  CK(hipMemset(status, 0, sizeof(int)));
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t mine[2], theirs[2];
  CK(hipIpcGetMemHandle(&mine[0], send));
  CK(hipIpcGetMemHandle(&mine[1], flags));
  if (!write_file(dir + "/h" + std::to_string(rank), mine, sizeof(mine)) ||
      !read_file(dir + "/h" + std::to_string(peer), theirs, sizeof(theirs), 60)) {
    fprintf(stderr, "rank %d: handle rendezvous failed\n", rank);
    return 1;
  }
  void *psend = nullptr, *pflags = nullptr;
  CK(hipIpcOpenMemHandle(&psend, theirs[0], hipIpcMemLazyEnablePeerAccess));
  CK(hipIpcOpenMemHandle(&pflags, theirs[1], hipIpcMemLazyEnablePeerAccess));
  // flags in each arena: [0] ready raised by the peer, [1] consumed raised by the peer
  unsigned long long* peer_flags = (unsigned long long*)pflags;
  P2PGet g{(const double*)psend, recv, n, flags + 0, peer_flags + 1, cnt + 1, (int)((n + P2P_CHUNK - 1) / P2P_CHUNK)};
  P2PGet* dg = nullptr;
  unsigned long long** dready = nullptr;
  const unsigned long long** dcons = nullptr;
  unsigned long long* ready_ptr = peer_flags + 0;
  const unsigned long long* cons_ptr = flags + 1;
  CK(hipMalloc(&dg, sizeof(g)));
  CK(hipMemcpy(dg, &g, sizeof(g), hipMemcpyHostToDevice));
  CK(hipMalloc(&dready, sizeof(void*)));
  CK(hipMemcpy(dready, &ready_ptr, sizeof(void*), hipMemcpyHostToDevice));
  CK(hipMalloc(&dcons, sizeof(void*)));
  CK(hipMemcpy(dcons, &cons_ptr, sizeof(void*), hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // both processes start together (a second rendezvous) so that the timing is of the exchange
  const char go = 1;
  char other = 0;
  if (!write_file(dir + "/go" + std::to_string(rank), &go, 1) || !read_file(dir + "/go" + std::to_string(peer), &other, 1, 60)) {
    fprintf(stderr, "rank %d: start rendezvous failed\n", rank);
    return 1;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int fill_blocks = (int)std::min<long long>(1024, (n + 255) / 256);
  CK(hipEventRecord(e0, s));
  for (long long it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(k_fill, dim3(fill_blocks), dim3(256), 0, s, send, n, it, rank);
    hipLaunchKernelGGL(k_p2p_post, dim3(1), dim3(64), 0, s, cnt, dready, 1);
    hipLaunchKernelGGL(k_p2p_get, dim3(g.nchunk, 2), dim3(256), 0, s, (const P2PGet*)dg, 1,
                       (const unsigned long long* const*)dcons, 1, (const unsigned long long*)cnt, status);
    hipLaunchKernelGGL(k_check, dim3(fill_blocks), dim3(256), 0, s, recv, n, it, peer, bad);
  }
  CK(hipEventRecord(e1, s));
  CK(hipStreamSynchronize(s));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long nbad = 0;
  int st = 0;
  CK(hipMemcpy(&nbad, bad, sizeof(nbad), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&st, status, sizeof(st), hipMemcpyDeviceToHost));
  printf("{\"rank\": %d, \"doubles\": %lld, \"iterations\": %lld, \"bad\": %llu, \"timed_out\": %d, \"us_per_iteration\": %.2f}\n",
         rank, n, iters, nbad, st, 1000.0 * ms / iters);
  // both ends keep their mappings until the peer is done with them
  (void)write_file(dir + "/done" + std::to_string(rank), &go, 1);
  (void)read_file(dir + "/done" + std::to_string(peer), &other, 1, 60);
  CK(hipIpcCloseMemHandle(psend));
  CK(hipIpcCloseMemHandle(pflags));
  return (nbad == 0 && st == 0) ? 0 : 1;
}

// Pull mode (k_p2p_pull): the "field" is ordinary device memory (hipMalloc) of `cols` columns of 64
// doubles; the first half are this rank's owned columns (written by the fill kernel each iteration),
// the second half its halo, which k_p2p_pull fills from the peer's owned columns through the peer's
// send list (every other owned column, reversed) into this rank's receive list.
__global__ void k_fill_cols(double* f, int cols, long long it, int rank) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), j = threadIdx.x & 63;
  if (c < cols / 2) f[(size_t)c * 64 + j] = pattern(it, rank, (long long)c * 64 + j);
}

__global__ void k_check_cols(const double* f, const int* sidx, const int* didx, int m, long long it, int peer,
                             unsigned long long* bad) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), j = threadIdx.x & 63;
  if (i < m && f[(size_t)didx[i] * 64 + j] != pattern(it, peer, (long long)sidx[i] * 64 + j)) atomicAdd(bad, 1ull);
}

int run_pull(int rank, const std::string& dir, long long n, long long iters) {
  const int peer = 1 - rank;
  const int cols = (int)std::max<long long>(8, 2 * (n / 64 / 2));  // n doubles of owned + halo columns
  const int own = cols / 2, m = own / 2;                            // m columns move each way
  double* field = nullptr;
  unsigned long long *flags = nullptr, *cnt = nullptr, *bad = nullptr;
  int *status = nullptr, *sidx = nullptr, *didx = nullptr;
  CK(hipMalloc(&field, (size_t)cols * 64 * sizeof(double)));
  CK(hipMemset(field, 0, (size_t)cols * 64 * sizeof(double)));
  CK(hipExtMallocWithFlags((void**)&flags, 4 * sizeof(unsigned long long), hipDeviceMallocUncached));
  CK(hipMemset(flags, 0, 4 * sizeof(unsigned long long)));
  CK(hipMalloc(&cnt, 3 * sizeof(unsigned long long)));
  CK(hipMemset(cnt, 0, 3 * sizeof(unsigned long long)));
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  CK(hipMemset(bad, 0, sizeof(unsigned long long)));
  CK(hipMalloc(&status, sizeof(int)));
  CK(hipMemset(status, 0, sizeof(int)));
  std::vector<int> hs(m), hd(m);
  for (int i = 0; i < m; ++i) {
    hs[i] = own - 1 - 2 * i;  // the peer's send list: every other owned column, reversed
    hd[i] = own + i;          // this rank's receive list: its halo columns in order
  }
  CK(hipMalloc(&sidx, m * sizeof(int)));
  CK(hipMemcpy(sidx, hs.data(), m * sizeof(int), hipMemcpyHostToDevice));
  CK(hipMalloc(&didx, m * sizeof(int)));
  CK(hipMemcpy(didx, hd.data(), m * sizeof(int), hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t mine[2], theirs[2];
  CK(hipIpcGetMemHandle(&mine[0], field));
  CK(hipIpcGetMemHandle(&mine[1], flags));
  if (!write_file(dir + "/h" + std::to_string(rank), mine, sizeof(mine)) ||
      !read_file(dir + "/h" + std::to_string(peer), theirs, sizeof(theirs), 60)) {
    fprintf(stderr, "rank %d: handle rendezvous failed\n", rank);
    return 1;
  }
  void *pfield = nullptr, *pflags = nullptr;
  CK(hipIpcOpenMemHandle(&pfield, theirs[0], hipIpcMemLazyEnablePeerAccess));
  CK(hipIpcOpenMemHandle(&pflags, theirs[1], hipIpcMemLazyEnablePeerAccess));
  unsigned long long* peer_flags = (unsigned long long*)pflags;
  // one segment, one peer; chunks of P2P_PULL_COLS columns
  P2PSeg sg{(const double*)pfield, field, sidx, didx, m, 64, 0};
  std::vector<int2> chunks;
  for (int c = 0; c < m; c += P2P_PULL_COLS) chunks.push_back(make_int2(0, c));
  P2PPeer pr{flags + 0, peer_flags + 1, cnt + 2, (unsigned long long)chunks.size()};
  unsigned long long* ready_ptr = peer_flags + 0;
  const unsigned long long* cons_ptr = flags + 1;
  P2PSeg* dsg = nullptr;
  P2PPeer* dpr = nullptr;
  int2* dch = nullptr;
  unsigned long long** dready = nullptr;
  const unsigned long long** dcons = nullptr;
  CK(hipMalloc(&dsg, sizeof(sg)));
  CK(hipMemcpy(dsg, &sg, sizeof(sg), hipMemcpyHostToDevice));
  CK(hipMalloc(&dpr, sizeof(pr)));
  CK(hipMemcpy(dpr, &pr, sizeof(pr), hipMemcpyHostToDevice));
  CK(hipMalloc(&dch, chunks.size() * sizeof(int2)));
  CK(hipMemcpy(dch, chunks.data(), chunks.size() * sizeof(int2), hipMemcpyHostToDevice));
  CK(hipMalloc(&dready, sizeof(void*)));
  CK(hipMemcpy(dready, &ready_ptr, sizeof(void*), hipMemcpyHostToDevice));
  CK(hipMalloc(&dcons, sizeof(void*)));
  CK(hipMemcpy(dcons, &cons_ptr, sizeof(void*), hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char go = 1;
  char other = 0;
  if (!write_file(dir + "/go" + std::to_string(rank), &go, 1) || !read_file(dir + "/go" + std::to_string(peer), &other, 1, 60)) {
    fprintf(stderr, "rank %d: start rendezvous failed\n", rank);
    return 1;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (long long it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(k_fill_cols, dim3((own + 3) / 4), dim3(256), 0, s, field, cols, it, rank);
    hipLaunchKernelGGL(k_p2p_pull, dim3((int)chunks.size() + 1), dim3(256), 0, s, (const P2PSeg*)dsg, (const int2*)dch,
                       (int)chunks.size(), (const P2PPeer*)dpr, 1, (unsigned long long* const*)dready, 1,
                       (const unsigned long long* const*)dcons, 1, cnt, status);
    hipLaunchKernelGGL(k_check_cols, dim3((m + 3) / 4), dim3(256), 0, s, field, sidx, didx, m, it, peer, bad);
  }
  CK(hipEventRecord(e1, s));
  CK(hipStreamSynchronize(s));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long nbad = 0;
  int st = 0;
  CK(hipMemcpy(&nbad, bad, sizeof(nbad), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&st, status, sizeof(st), hipMemcpyDeviceToHost));
  printf("{\"mode\": \"pull\", \"rank\": %d, \"columns_moved\": %d, \"iterations\": %lld, \"bad\": %llu, \"timed_out\": %d, "
         "\"us_per_iteration\": %.2f}\n", rank, m, iters, nbad, st, 1000.0 * ms / iters);
  (void)write_file(dir + "/done" + std::to_string(rank), &go, 1);
  (void)read_file(dir + "/done" + std::to_string(peer), &other, 1, 60);
  CK(hipIpcCloseMemHandle(pfield));
  CK(hipIpcCloseMemHandle(pflags));
  return (nbad == 0 && st == 0) ? 0 : 1;
}
