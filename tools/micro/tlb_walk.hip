// Single-workgroup dependent launches reading a fresh 32 KiB column of a
// 64 MiB matrix every launch (as the reduction's k_q_rs does) vs the same
// column every launch (tools/micro, A/B only).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_col(const double2* A, int64_t off, double2* out) {
  const double2 a = A[off + threadIdx.x];
  __shared__ double sh[16];
  double s = a.x + a.y;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < 16; ++k) t += sh[k];
  out[threadIdx.x] = make_double2(t, a.x);
}
// the same, but the whole 64 MiB also touched by a 256-workgroup kernel in between
__global__ __launch_bounds__(256) void k_touch(double2* A, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256 * 64) A[i].y += 1e-300;
}

int main() {
  const int n = 2048;
  double2 *A, *out;
  hipMalloc(&A, (size_t)n * n * sizeof(double2));
  hipMalloc(&out, 1 << 20);
  hipMemset(A, 0, (size_t)n * n * sizeof(double2));
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int K = 2000;
  auto run = [&](const char* name, auto fn) {
    for (int i = 0; i < 20; ++i) fn(i);
    hipEventRecord(e0, s);
    for (int i = 0; i < K; ++i) fn(i);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-52s %8.2f us per iteration\n", name, 1e3 * ms / K);
  };
  run("same column", [&](int) { hipLaunchKernelGGL(k_col, dim3(1), dim3(1024), 0, s, A, (int64_t)0, out); });
  run("fresh column (stride n)", [&](int j) {
    hipLaunchKernelGGL(k_col, dim3(1), dim3(1024), 0, s, A, (int64_t)(j % n) * n, out);
  });
  run("fresh column, stride 7n (other pages)", [&](int j) {
    hipLaunchKernelGGL(k_col, dim3(1), dim3(1024), 0, s, A, (int64_t)((7 * j) % n) * n, out);
  });
  run("touch-all (256 WG, 1/64 of lines)", [&](int) {
    hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, s, A, (int64_t)n * n);
  });
  run("touch-all + same column", [&](int) {
    hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, s, A, (int64_t)n * n);
    hipLaunchKernelGGL(k_col, dim3(1), dim3(1024), 0, s, A, (int64_t)0, out);
  });
  run("touch-all + fresh column", [&](int j) {
    hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, s, A, (int64_t)n * n);
    hipLaunchKernelGGL(k_col, dim3(1), dim3(1024), 0, s, A, (int64_t)((7 * j) % n) * n, out);
  });
  return 0;
}
