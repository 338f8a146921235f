// Producer / consumer latency between dependent launches (tools/micro, A/B
// only): a 1-workgroup consumer reading data the previous kernel wrote vs
// data nobody wrote since.
#include <hip/hip_runtime.h>
#include <cstdio>

// 272 workgroups, each writes 64 x 4 doubles into 2 slots of part
__global__ __launch_bounds__(256) void k_prod(double* part, int M, int j) {
  const int b = blockIdx.x, t = threadIdx.x;
  part[((int64_t)(b % 32) * M + (b / 32) * 64 + (t >> 2)) * 4 + (t & 3)] = 1e-300 * j + t;
}
// one thread per (site, entry): sum 32 slots (16 in flight)
__global__ __launch_bounds__(256) void k_cons(const double* part, int M, double* P) {
  const int idx = blockIdx.x * 256 + threadIdx.x, site = idx >> 2, e = idx & 3;
  if (site >= M) return;
  double s = 0.0;
  for (int b0 = 0; b0 < 32; b0 += 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = part[((int64_t)(b0 + u) * M + site) * 4 + e];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  P[(int64_t)site * 4 + e] = s;
}

int main() {
  const int M = 1024;
  double *part, *part2, *P;
  hipMalloc(&part, (size_t)32 * M * 4 * 8);
  hipMalloc(&part2, (size_t)32 * M * 4 * 8);
  hipMalloc(&P, (size_t)M * 4 * 8);
  hipMemset(part, 0, (size_t)32 * M * 4 * 8);
  hipMemset(part2, 0, (size_t)32 * M * 4 * 8);
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int K = 2000;
  auto run = [&](const char* name, auto fn) {
    for (int i = 0; i < 50; ++i) fn(i);
    hipEventRecord(e0, s);
    for (int i = 0; i < K; ++i) fn(i);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-52s %8.2f us per iteration\n", name, 1e3 * ms / K);
  };
  for (int nwg : {1, 16}) {
    const int sites = nwg * 64;
    char nm[128];
    snprintf(nm, sizeof nm, "prod only (272 WG)");
    if (nwg == 1) run(nm, [&](int j) { hipLaunchKernelGGL(k_prod, dim3(272), dim3(256), 0, s, part, M, j); });
    snprintf(nm, sizeof nm, "cons only, %d WG", nwg);
    run(nm, [&](int) { hipLaunchKernelGGL(k_cons, dim3(nwg), dim3(256), 0, s, part2, sites, P); });
    snprintf(nm, sizeof nm, "prod + cons of the produced data, %d WG", nwg);
    run(nm, [&](int j) {
      hipLaunchKernelGGL(k_prod, dim3(272), dim3(256), 0, s, part, M, j);
      hipLaunchKernelGGL(k_cons, dim3(nwg), dim3(256), 0, s, part, M, P);
    });
    snprintf(nm, sizeof nm, "prod + cons of other data, %d WG", nwg);
    run(nm, [&](int j) {
      hipLaunchKernelGGL(k_prod, dim3(272), dim3(256), 0, s, part, M, j);
      hipLaunchKernelGGL(k_cons, dim3(nwg), dim3(256), 0, s, part2, M, P);
    });
  }
  return 0;
}
