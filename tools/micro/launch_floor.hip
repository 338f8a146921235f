// Diagnostic: the floor of a chain of dependent launches on one stream, the
// structure of a CR step (every stage reads what the previous one wrote).
//   A: empty kernel, 1 workgroup                        (launch + dispatch)
//   B: 64 workgroups x 256 threads, each loads 16 B per thread of a block
//      the previous launch stored and stores its own    (one memory round trip)
//   C: as B with 1024 workgroups
// N launches back to back, timed with events around the whole chain; the
// average per launch is what a stage costs at least.
// Build: hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty() {}

__global__ __launch_bounds__(256) void k_copy(const double2* __restrict__ in, double2* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    double2 v = in[i];
    v.x += 1.0;
    out[i] = v;
  }
}

int main() {
  const int N = 2000;
  double2 *a, *b;
  const int n = 1024 * 256;
  (void)hipMalloc(&a, n * sizeof(double2));
  (void)hipMalloc(&b, n * sizeof(double2));
  (void)hipMemset(a, 0, n * sizeof(double2));
  (void)hipMemset(b, 0, n * sizeof(double2));
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    const int wg = mode == 0 ? 1 : mode == 1 ? 64 : 1024;
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0, s);
      for (int k = 0; k < N; ++k) {
        if (mode == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        else hipLaunchKernelGGL(k_copy, dim3(wg), dim3(256), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, wg * 256);
      }
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1)
        printf("%s: %d dependent launches, %.2f us per launch\n",
               mode == 0 ? "empty kernel (1 workgroup)" : mode == 1 ? "load+store, 64 workgroups" : "load+store, 1024 workgroups",
               N, 1000.0 * ms / N);
    }
  }
  return 0;
}
