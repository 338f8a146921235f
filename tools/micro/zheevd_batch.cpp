// Micro-benchmark: rocSOLVER zheevd one matrix at a time vs strided_batched,
// n = 2048 (the L = 32 BdG size).  Decides whether the transport measurement
// of a multi-chain context batches its eigensolves.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2048;
  const int batch = argc > 2 ? std::atoi(argv[2]) : 4;
  std::vector<rocblas_double_complex> h((size_t)n * n * batch);
  std::mt19937_64 g(1);
  std::normal_distribution<double> nd;
  for (int b = 0; b < batch; ++b)
    for (int j = 0; j < n; ++j)
      for (int i = 0; i <= j; ++i) {
        const double re = nd(g), im = i == j ? 0.0 : nd(g);
        h[(size_t)b * n * n + i + (size_t)j * n] = rocblas_double_complex(re, im);
        h[(size_t)b * n * n + j + (size_t)i * n] = rocblas_double_complex(re, -im);
      }
  rocblas_double_complex* A;
  double *D, *E;
  int* info;
  const size_t sA = (size_t)n * n;
  (void)hipMalloc(&A, sA * batch * sizeof(*A));
  (void)hipMalloc(&D, (size_t)n * batch * sizeof(double));
  (void)hipMalloc(&E, (size_t)n * batch * sizeof(double));
  (void)hipMalloc(&info, batch * sizeof(int));
  rocblas_handle hd;
  rocblas_create_handle(&hd);
  auto reset = [&] { (void)hipMemcpy(A, h.data(), sA * batch * sizeof(*A), hipMemcpyHostToDevice); };
  auto time_it = [&](auto fn) {
    reset();
    fn();
    (void)hipDeviceSynchronize();
    reset();
    (void)hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    fn();
    (void)hipDeviceSynchronize();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  const double t_loop = time_it([&] {
    for (int b = 0; b < batch; ++b)
      rocsolver_zheevd(hd, rocblas_evect_original, rocblas_fill_upper, n, A + b * sA, n, D + (size_t)b * n,
                       E + (size_t)b * n, info + b);
  });
  const double t_bat = time_it([&] {
    rocsolver_zheevd_strided_batched(hd, rocblas_evect_original, rocblas_fill_upper, n, A, n, sA, D, n, E, n,
                                     info, batch);
  });
  std::printf("{\"n\": %d, \"batch\": %d, \"ms_loop\": %.2f, \"ms_batched\": %.2f, \"ms_per_matrix_loop\": %.2f, "
              "\"ms_per_matrix_batched\": %.2f}\n",
              n, batch, t_loop, t_bat, t_loop / batch, t_bat / batch);
  rocblas_destroy_handle(hd);
  return 0;
}
