// Microbenchmark: do fp64 VALU FMAs (v_fma_f64) and fp64 MFMAs
// (v_mfma_f64_16x16x4_f64) of one wave execute concurrently on MI355X?
// Per loop iteration a wave issues NM MFMAs on 8 independent accumulators
// and NF FMAs on 16 independent scalar chains.  If the two pipes overlap, the
// mixed loop takes max(MFMA, VALU) cycles per iteration, else their sum.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_valu_coexec.hip -o tools/micro/mfma_valu_coexec
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 2048;

template <int NM, int NF>
__global__ __launch_bounds__(256) void k_mix(const double* a, const double* b, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double x = a[t & 1023], y = b[t & 1023];
  d4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
  double f[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) f[i] = x + i;
  const long long t0 = clock64();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int r = 0; r < (NM > NF / 16 ? NM : NF / 16); ++r) {
      if (r < NM) acc[r & 7] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[r & 7], 0, 0, 0);
      if (r < NF / 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) f[i] = __builtin_fma(f[i], y, x);
      }
    }
    // interleave: one MFMA, then a sixteenth of the iteration's FMAs
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (NM > r) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (NF > 0) __builtin_amdgcn_sched_group_barrier(0x002, NF / 8, 0);
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += f[i];
  out[t] = s;
  if (threadIdx.x == 0) out[gridDim.x * blockDim.x + blockIdx.x] = (double)(t1 - t0);
}

template <int NM, int NF>
void run(const char* name, const double* a, const double* b, int ncu) {
  const int blocks = ncu;   // one 4-wave block per CU = one wave per SIMD
  double* o;
  (void)hipMalloc(&o, (size_t)(blocks * 256 + blocks) * 8);
  hipLaunchKernelGGL((k_mix<NM, NF>), dim3(blocks), dim3(256), 0, 0, a, b, o);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 5;
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_mix<NM, NF>), dim3(blocks), dim3(256), 0, 0, a, b, o);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<double> cyc(blocks);
  (void)hipMemcpy(cyc.data(), o + blocks * 256, blocks * 8, hipMemcpyDeviceToHost);
  double mc = 0;
  for (double c : cyc) mc += c;
  mc /= blocks;
  const double fl = (double)reps * blocks * 4 * ITER * (NM * 2048.0 + NF * 128.0);
  printf("%-28s NM=%2d NF=%3d  %.1f cycles/iter  %.2f TFLOP/s (MFMA %.2f + VALU %.2f)\n", name, NM, NF,
         mc / ITER, fl / (ms * 1e-3) / 1e12,
         (double)reps * blocks * 4 * ITER * NM * 2048.0 / (ms * 1e-3) / 1e12,
         (double)reps * blocks * 4 * ITER * NF * 128.0 / (ms * 1e-3) / 1e12);
  (void)hipFree(o);
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  std::vector<double> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + 1e-3 * ((i * 7919) % 1000);
  double *a, *b;
  (void)hipMalloc(&a, 8192);
  (void)hipMalloc(&b, 8192);
  (void)hipMemcpy(a, h.data(), 8192, hipMemcpyHostToDevice);
  (void)hipMemcpy(b, h.data(), 8192, hipMemcpyHostToDevice);
  printf("CUs %d\n", ncu);
  run<8, 0>("MFMA only", a, b, ncu);
  run<0, 128>("VALU only", a, b, ncu);
  run<8, 128>("MFMA + VALU (balanced)", a, b, ncu);
  run<8, 64>("MFMA + VALU (half)", a, b, ncu);
  run<8, 32>("MFMA + VALU (quarter)", a, b, ncu);
  run<4, 128>("MFMA half + VALU", a, b, ncu);
  return 0;
}
