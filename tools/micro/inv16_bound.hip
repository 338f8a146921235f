// Diagnostic: what bounds the 16x16 register inversion (wave_inv16_dpp's
// pivot step)?  One wave per workgroup runs REP inversions of a 16x16 complex
// tile in the strided layout; each variant removes one piece of the pivot step
// (results are garbage for the ablated variants; only the cycle count matters):
//   V=0 full step           V=1 column from the own lane (no ds_bpermute)
//   V=2 no reciprocal chain V=3 row from the own lane (no DPP broadcast)
//   V=4 pivot from the own lane (no v_readlane)   V=5 = 1+2+3+4 (update only)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include inv16_bound.hip -o inv16_bound
#include "../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc/dwhmc_device.h"
#include <cstdio>
#include <vector>
using namespace dwh;

template <int V, int P>
__device__ __forceinline__ void step(double2 (&a)[4], double& pprod) {
  constexpr int PS = P & 3, PE = P >> 2;   // strided layout
  const int l = threadIdx.x & 63, r = l & 15, q = l >> 4;
  constexpr bool nob = V == 1 || V == 5, norcp = V == 2 || V == 5, nodpp = V == 3 || V == 5,
                 norl = V == 4 || V == 5;
  double2 rowp[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj)
    rowp[jj] = nodpp ? a[jj] : make_double2(dpp_rowbcast<P>(a[jj].x), dpp_rowbcast<P>(a[jj].y));
  const double2 colp = nob ? a[PE] : make_double2(bcast_quarter<PS>(a[PE].x), bcast_quarter<PS>(a[PE].y));
  const double2 piv = norl ? a[(PE + 1) & 3]
                           : make_double2(readlane_f64(a[PE].x, PS * 16 + P), readlane_f64(a[PE].y, PS * 16 + P));
  const double m2 = fma(piv.x, piv.x, piv.y * piv.y);
  const double s = norcp ? m2 : rcp_nr(m2);
  const double2 inv = make_double2(piv.x * s, -piv.y * s);
  pprod *= m2;
  const bool prow = (r == P);
  const double2 fi = cmul(make_double2(colp.x - (prow ? 1.0 : 0.0), colp.y), inv);
  rowp[PE].x += (q == PS) ? 1.0 : 0.0;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const double2 x = rowp[jj];
    double2 v;
    v.x = fma(-fi.x, x.x, fma(fi.y, x.y, a[jj].x));
    v.y = fma(-fi.x, x.y, fma(-fi.y, x.x, a[jj].y));
    a[jj] = v;
  }
}
template <int V, int... Ps>
__device__ __forceinline__ void all(double2 (&a)[4], double& pp, std::integer_sequence<int, Ps...>) {
  (step<V, Ps>(a, pp), ...);
}

template <int V>
__global__ __launch_bounds__(64) void k_bound(const double2* in, double2* out, long long* cyc, int rep) {
  double2 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = in[(blockIdx.x * 4 + j) * 64 + threadIdx.x];
  double pp = 1.0;
  __builtin_amdgcn_s_waitcnt(0);
  const long long t0 = clock64();
  for (int it = 0; it < rep; ++it) all<V>(a, pp, std::make_integer_sequence<int, 16>{});
  const long long t1 = clock64();
#pragma unroll
  for (int j = 0; j < 4; ++j) out[(blockIdx.x * 4 + j) * 64 + threadIdx.x] = make_double2(a[j].x + pp, a[j].y);
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
void run(const double2* in, double2* out, long long* cyc, int nblk, int rep) {
  hipLaunchKernelGGL(k_bound<V>, dim3(nblk), dim3(64), 0, 0, in, out, cyc, rep);   // warm
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_bound<V>, dim3(nblk), dim3(64), 0, 0, in, out, cyc, rep);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(nblk);
  hipMemcpy(c.data(), cyc, nblk * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (long long x : c) m += (double)x;
  m /= nblk;
  printf("V=%d  clock64 cycles per pivot %.1f   wall ns per pivot %.1f\n", V, m / (16.0 * rep),
         ms * 1e6 / (16.0 * rep));
}

int main() {
  const int nblk = 240, rep = 256;
  std::vector<double2> h((size_t)nblk * 4 * 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = make_double2(0.01 * (double)(i % 7), 1.0 + 0.001 * (double)(i % 5));
  double2 *in, *out;
  long long* cyc;
  hipMalloc(&in, h.size() * 16);
  hipMalloc(&out, h.size() * 16);
  hipMalloc(&cyc, nblk * 8);
  hipMemcpy(in, h.data(), h.size() * 16, hipMemcpyHostToDevice);
  run<0>(in, out, cyc, nblk, rep);
  run<1>(in, out, cyc, nblk, rep);
  run<2>(in, out, cyc, nblk, rep);
  run<3>(in, out, cyc, nblk, rep);
  run<4>(in, out, cyc, nblk, rep);
  run<5>(in, out, cyc, nblk, rep);
  return 0;
}
