// Microbenchmark: 20 column gathers per element from a 163842-column array (K=56 doubles per
// column), neighbours = SFC-local random offsets.  (a) one element per wave, lane = level,
// 8-byte loads; (b) two elements per wave, lane = 2 levels, 16-byte loads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#define K 56
#ifndef NG
#define NG 20
#endif
__global__ __launch_bounds__(256) void ga(const double* __restrict__ a, const int* __restrict__ nb, double* out, int n) {
  int e = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (e >= n) return;
  int k = min((int)(threadIdx.x & 63), K - 1);
  int ic[NG];
#pragma unroll
  for (int j = 0; j < NG; ++j) ic[j] = nb[e * NG + j];
  double v[NG];
#pragma unroll
  for (int j = 0; j < NG; ++j) v[j] = a[(size_t)__builtin_amdgcn_readfirstlane(ic[j]) * K + k];
  double s = 0;
#pragma unroll
  for (int j = 0; j < NG; ++j) s += v[j] * (j + 1);
  if ((threadIdx.x & 63) < K) out[(size_t)e * K + k] = s;
}
__global__ __launch_bounds__(256) void gb(const double* __restrict__ a, const int* __restrict__ nb, double* out, int n) {
  int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  int h = (threadIdx.x >> 5) & 1, l = min((int)(threadIdx.x & 31), K / 2 - 1);
  int e = 2 * w + h;
  if (2 * w >= n) return;
  e = min(e, n - 1);
  int icA[NG], icB[NG];
#pragma unroll
  for (int j = 0; j < NG; ++j) { icA[j] = nb[(2 * w) * NG + j]; icB[j] = nb[min(2 * w + 1, n - 1) * NG + j]; }
  double2 v[NG];
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    int c = h ? icB[j] : icA[j];
    v[j] = *reinterpret_cast<const double2*>(a + (size_t)c * K + 2 * l);
  }
  double2 s = {0, 0};
#pragma unroll
  for (int j = 0; j < NG; ++j) { s.x += v[j].x * (j + 1); s.y += v[j].y * (j + 1); }
  if ((threadIdx.x & 31) < K / 2) *reinterpret_cast<double2*>(out + (size_t)e * K + 2 * l) = s;
}
// streaming: out[e] = a[e] * 2 (+ 5 more own columns), 1 col/wave dwordx2 vs 2 cols/wave dwordx4
#define NS 6
__global__ __launch_bounds__(256) void sa(const double* __restrict__ a, double* out, int n) {
  int e = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (e >= n) return;
  int k = min((int)(threadIdx.x & 63), K - 1);
  double s = 0;
#pragma unroll
  for (int j = 0; j < NS; ++j) s += a[(size_t)j * n * K + (size_t)e * K + k] * (j + 1);
  if ((threadIdx.x & 63) < K) out[(size_t)e * K + k] = s;
}
__global__ __launch_bounds__(256) void sb(const double* __restrict__ a, double* out, int n) {
  int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  int h = (threadIdx.x >> 5) & 1, l = min((int)(threadIdx.x & 31), K / 2 - 1);
  int e = min(2 * w + h, n - 1);
  if (2 * w >= n) return;
  double2 s = {0, 0};
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    double2 v = *reinterpret_cast<const double2*>(a + (size_t)j * n * K + (size_t)e * K + 2 * l);
    s.x += v.x * (j + 1); s.y += v.y * (j + 1);
  }
  if ((threadIdx.x & 31) < K / 2) *reinterpret_cast<double2*>(out + (size_t)e * K + 2 * l) = s;
}
// (c) streaming reference: each wave reads its own 20 consecutive columns (no gather reuse)
int main() {
  const int nC = 163842, nE = 491520;
  std::vector<int> nb((size_t)nE * NG);
  std::mt19937 rng(1);
  for (int e = 0; e < nE; ++e) {
    int c0 = (int)((long)e * nC / nE);
    for (int j = 0; j < NG; ++j) { int c = c0 + (int)(rng() % 41) - 20; nb[(size_t)e * NG + j] = std::min(std::max(c, 0), nC - 1); }
  }
  double *a, *out; int* dnb;
  double* big; hipMalloc(&big, (size_t)NS * nE * K * 8); hipMemset(big, 0, (size_t)NS * nE * K * 8);
  hipMalloc(&a, (size_t)(nC + 1) * K * 8); hipMalloc(&out, (size_t)nE * K * 8); hipMalloc(&dnb, nb.size() * 4);
  hipMemset(a, 0, (size_t)(nC + 1) * K * 8);
  hipMemcpy(dnb, nb.data(), nb.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t t0, t1; hipEventCreate(&t0); hipEventCreate(&t1);
  for (int variant = 0; variant < 4; ++variant) {
    for (int it = 0; it < 3; ++it) {
      hipEventRecord(t0);
      for (int r = 0; r < 20; ++r) {
        if (variant == 0) hipLaunchKernelGGL(ga, dim3((nE + 3) / 4), dim3(256), 0, 0, a, dnb, out, nE);
        else if (variant == 1) hipLaunchKernelGGL(gb, dim3((nE / 2 + 3) / 4), dim3(256), 0, 0, a, dnb, out, nE);
        else if (variant == 2) hipLaunchKernelGGL(sa, dim3((nE + 3) / 4), dim3(256), 0, 0, big, out, nE);
        else hipLaunchKernelGGL(sb, dim3((nE / 2 + 3) / 4), dim3(256), 0, 0, big, out, nE);
      }
      hipEventRecord(t1); hipEventSynchronize(t1);
      float ms; hipEventElapsedTime(&ms, t0, t1);
      if (it == 2) printf("NG=%d variant %c: %.1f us per launch\n", NG, "abcd"[variant], ms * 1000 / 20);
    }
  }
  return 0;
}
