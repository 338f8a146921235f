// Dependent-launch floor on this box: K back-to-back launches of small
// kernels on one stream, timed with HIP events (tools/micro, A/B only).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(double* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345.0) p[1] = 1.0;
}
__global__ __launch_bounds__(1024) void k_red1024(double* p, int n) {
  __shared__ double sh[16];
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) a += p[i];
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < 16; ++k) s += sh[k];
  if (threadIdx.x < n) p[n + threadIdx.x] = s * 1e-30 + p[threadIdx.x];
}
__global__ __launch_bounds__(256) void k_tile(double2* A, int n, int j) {
  // 64 x 64 tiles touched by one read-modify-write each (like a pass)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double2* t = A + (int64_t)blockIdx.x * 64 * 64;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    double2 x = t[lane + (16 * w + u) * 64];
    x.x += 1e-300 * j;
    t[lane + (16 * w + u) * 64] = x;
  }
}

int main() {
  double* p;
  double2* A;
  hipMalloc(&p, 1 << 24);
  hipMalloc(&A, (size_t)64 << 20);
  hipMemset(p, 0, 1 << 24);
  hipMemset(A, 0, (size_t)64 << 20);
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
    printf("%-40s %8.2f us per launch\n", name, 1e3 * ms / K);
  };
  run("empty 1x64", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, p); });
  run("empty 256x256", [&](int) { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, p); });
  run("red1024 n=1024", [&](int) { hipLaunchKernelGGL(k_red1024, dim3(1), dim3(1024), 0, s, p, 1024); });
  run("red1024 n=4096", [&](int) { hipLaunchKernelGGL(k_red1024, dim3(1), dim3(1024), 0, s, p, 4096); });
  run("tile x2", [&](int j) { hipLaunchKernelGGL(k_tile, dim3(2), dim3(256), 0, s, A, 64, j); });
  run("tile x272", [&](int j) { hipLaunchKernelGGL(k_tile, dim3(272), dim3(256), 0, s, A, 64, j); });
  run("red1024 + tile x272", [&](int j) {
    hipLaunchKernelGGL(k_red1024, dim3(1), dim3(1024), 0, s, p, 1024);
    hipLaunchKernelGGL(k_tile, dim3(272), dim3(256), 0, s, A, 64, j);
  });
  // the same chains captured in a graph (100 pairs per graph)
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; ++i) {
    hipLaunchKernelGGL(k_red1024, dim3(1), dim3(1024), 0, s, p, 1024);
    hipLaunchKernelGGL(k_tile, dim3(272), dim3(256), 0, s, A, 64, i);
  }
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEventRecord(e0, s);
  for (int i = 0; i < 20; ++i) hipGraphLaunch(ge, s);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-40s %8.2f us per launch\n", "graph: red1024 + tile x272", 1e3 * ms / (20 * 200));
  return 0;
}
