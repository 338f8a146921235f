// Microbenchmark: sustained v_mfma_f64_16x16x4_f64 throughput on MI355X.
// Every wave runs ITER iterations of 8 independent accumulator chains on
// random operands; reports TFLOP/s over the whole chip and the implied
// cycles per MFMA at the measured clock.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;
__global__ __launch_bounds__(256) void k_peak(const double* a, const double* b, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double x = a[t & 1023], y = b[t & 1023];
  d4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
  long long t0 = clock64();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
  }
  long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[t] = s;
  if (threadIdx.x == 0) out[gridDim.x * blockDim.x + blockIdx.x] = (double)(t1 - t0);
}
int main() {
  int ncu = 0;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  ncu = prop.multiProcessorCount;
  std::vector<double> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + 1e-3 * ((i * 7919) % 1000);
  double *a, *b, *o;
  hipMalloc(&a, 8192);
  hipMalloc(&b, 8192);
  hipMemcpy(a, h.data(), 8192, hipMemcpyHostToDevice);
  hipMemcpy(b, h.data(), 8192, hipMemcpyHostToDevice);
  for (int bpc : {1, 2, 4}) {
    const int blocks = ncu * bpc;
    hipMalloc(&o, (size_t)(blocks * 256 + blocks) * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_peak, dim3(blocks), dim3(256), 0, 0, a, b, o);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_peak, dim3(blocks), dim3(256), 0, 0, a, b, o);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<double> cyc(blocks);
    hipMemcpy(cyc.data(), o + blocks * 256, blocks * 8, hipMemcpyDeviceToHost);
    double mc = 0;
    for (double c : cyc) mc += c;
    mc /= blocks;
    const double flops = (double)reps * blocks * 4 /*waves*/ * ITER * 8 * 2048.0;
    const double sec = ms * 1e-3;
    const double per_launch = sec / reps;
    printf("blocks/CU=%d  %.2f TFLOP/s  launch %.3f ms  in-kernel %.0f cycles/wave -> %.1f cycles/MFMA/wave, clock %.2f GHz\n",
           bpc, flops / sec / 1e12, per_launch * 1e3, mc, mc / (ITER * 8.0), mc / per_launch / 1e9);
    hipFree(o);
  }
  return 0;
}
