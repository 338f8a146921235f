// Diagnostic: does instruction fetch slow the in-kernel 16x16 inversions?
// k_cr_inv<4> runs four distinct unrolled copies of wave_inv16_dpp (one per
// pivot step, ~5.6 KB of code each) once per workgroup, one workgroup per CU
// at the coarse levels, so every copy may run from a cold instruction cache.
// k_copies: C inlined copies in sequence (each executed once), cycles per copy;
// k_loop: one copy run C times in a loop (warm after the first pass).
// Launched with NB single-wave workgroups (one per CU at NB <= 256).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 inv16_icache.hip -o inv16_icache
#include "../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc/dwhmc_device.h"
#include <cstdio>
#include <vector>
using namespace dwh;

constexpr int C = 4;

template <int K>
__device__ __forceinline__ void copies(double2 (&a)[4], double& pp, long long* t) {
  if constexpr (K < C) {
    pp *= wave_inv16_dpp<true>(a);
    t[K + 1] = clock64();
    copies<K + 1>(a, pp, t);
  }
}

__global__ __launch_bounds__(64) void k_copies(const double2* in, double2* out, long long* cyc) {
  double2 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = in[(blockIdx.x * 4 + j) * 64 + threadIdx.x];
  double pp = 1.0;
  __builtin_amdgcn_s_waitcnt(0);
  long long t[C + 1];
  t[0] = clock64();
  copies<0>(a, pp, t);
#pragma unroll
  for (int j = 0; j < 4; ++j) out[(blockIdx.x * 4 + j) * 64 + threadIdx.x] = make_double2(a[j].x + pp, a[j].y);
  if (threadIdx.x == 0)
    for (int k = 0; k < C; ++k) cyc[blockIdx.x * C + k] = t[k + 1] - t[k];
}

__global__ __launch_bounds__(64) void k_loop(const double2* in, double2* out, long long* cyc) {
  double2 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = in[(blockIdx.x * 4 + j) * 64 + threadIdx.x];
  double pp = 1.0;
  __builtin_amdgcn_s_waitcnt(0);
  long long t[C + 1];
  t[0] = clock64();
#pragma unroll 1
  for (int k = 0; k < C; ++k) {
    pp *= wave_inv16_dpp<true>(a);
    const long long x = clock64();
    // store through a select chain, so the loop stays rolled
#pragma unroll
    for (int m = 0; m < C; ++m)
      if (m == k) t[m + 1] = x;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) out[(blockIdx.x * 4 + j) * 64 + threadIdx.x] = make_double2(a[j].x + pp, a[j].y);
  if (threadIdx.x == 0)
    for (int k = 0; k < C; ++k) cyc[blockIdx.x * C + k] = t[k + 1] - t[k];
}

int main() {
  for (int nb : {96, 256}) {
    std::vector<double2> h((size_t)nb * 4 * 64);
    for (size_t i = 0; i < h.size(); ++i)   // diagonally dominant tiles
      h[i] = make_double2(((i * 2654435761u) % 1000) * 1e-4, ((i * 40503u) % 1000) * 1e-4);
    for (int b = 0; b < nb; ++b)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 4; ++j) {
          const int r = l & 15, c = (l >> 4) + 4 * j;   // strided layout
          if (r == c) h[((size_t)b * 4 + j) * 64 + l].x += 4.0;
        }
    double2 *in, *out;
    long long* cyc;
    (void)hipMalloc(&in, h.size() * sizeof(double2));
    (void)hipMalloc(&out, h.size() * sizeof(double2));
    (void)hipMalloc(&cyc, (size_t)nb * C * sizeof(long long));
    (void)hipMemcpy(in, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice);
    std::vector<long long> hc((size_t)nb * C);
    for (int kind = 0; kind < 2; ++kind)
      for (int launch = 0; launch < 3; ++launch) {
        if (kind == 0) hipLaunchKernelGGL(k_copies, dim3(nb), dim3(64), 0, 0, in, out, cyc);
        else hipLaunchKernelGGL(k_loop, dim3(nb), dim3(64), 0, 0, in, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hc.data(), cyc, hc.size() * sizeof(long long), hipMemcpyDeviceToHost);
        std::printf("nb=%3d %-8s launch %d  cycles per inversion (mean over WGs):", nb, kind ? "loop" : "copies",
                    launch);
        for (int k = 0; k < C; ++k) {
          double s = 0;
          for (int b = 0; b < nb; ++b) s += hc[(size_t)b * C + k];
          std::printf(" %7.0f", s / nb);
        }
        std::printf("\n");
      }
    (void)hipFree(in);
    (void)hipFree(out);
    (void)hipFree(cyc);
  }
  return 0;
}
