// Micro-benchmark of rocSOLVER's Hermitian eigensolvers at the BdG size of
// L = 32 (n = 2048), on a BdG-structured matrix [[h, D], [conj D, -h]]
// (h real symmetric, D complex symmetric): zheevd (the transport / eigen
// path's solver), zheevdj, zheevj, zheevdx over the positive half of the
// spectrum (the negative half follows from particle-hole symmetry), and
// zhetrd alone.  Decides whether the measurement path changes solver.
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/eig_variants.cpp -lrocsolver -lrocblas -o tools/micro/eig_variants
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 1024, n = 2 * N;
  std::vector<rocblas_double_complex> h((size_t)n * n, rocblas_double_complex(0, 0));
  std::mt19937_64 g(1);
  std::normal_distribution<double> nd;
  auto at = [&](int i, int j) -> rocblas_double_complex& { return h[i + (size_t)j * n]; };
  for (int j = 0; j < N; ++j)
    for (int i = 0; i <= j; ++i) {
      const double hv = (std::abs(i - j) <= 2 || std::abs(i - j) == 32) ? nd(g) : 0.0;   // banded-ish hopping
      at(i, j) = at(j, i) = rocblas_double_complex(hv, 0);
      at(i + N, j + N) = at(j + N, i + N) = rocblas_double_complex(-hv, 0);
      const double dr = (std::abs(i - j) == 1 || std::abs(i - j) == 32) ? 0.3 * nd(g) : 0.0;
      const double di = dr != 0.0 ? 0.3 * nd(g) : 0.0;
      at(i, j + N) = at(j, i + N) = rocblas_double_complex(dr, di);
      at(j + N, i) = at(i + N, j) = rocblas_double_complex(dr, -di);
    }
  const size_t sA = (size_t)n * n;
  rocblas_double_complex *A, *Z, *tau;
  double *W, *E, *res;
  int *info, *nev, *sweeps;
  (void)hipMalloc(&A, sA * sizeof(*A));
  (void)hipMalloc(&Z, sA * sizeof(*Z));
  (void)hipMalloc(&tau, n * sizeof(*tau));
  (void)hipMalloc(&W, n * sizeof(double));
  (void)hipMalloc(&E, n * sizeof(double));
  (void)hipMalloc(&res, sizeof(double));
  (void)hipMalloc(&info, sizeof(int));
  (void)hipMalloc(&nev, sizeof(int));
  (void)hipMalloc(&sweeps, sizeof(int));
  rocblas_handle hd;
  rocblas_create_handle(&hd);
  auto reset = [&] { (void)hipMemcpy(A, h.data(), sA * sizeof(*A), hipMemcpyHostToDevice); };
  auto time_it = [&](const char* name, auto fn) {
    reset();
    fn();
    (void)hipDeviceSynchronize();
    reset();
    (void)hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    const rocblas_status st = fn();
    (void)hipDeviceSynchronize();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    int inf = -1, ne = -1;
    (void)hipMemcpy(&inf, info, sizeof(int), hipMemcpyDeviceToHost);
    (void)hipMemcpy(&ne, nev, sizeof(int), hipMemcpyDeviceToHost);
    std::printf("%-28s n=%d  %9.2f ms  status=%d info=%d nev=%d\n", name, n, ms, (int)st, inf, ne);
    std::fflush(stdout);
  };
  time_it("zheevd", [&] {
    return rocsolver_zheevd(hd, rocblas_evect_original, rocblas_fill_upper, n, A, n, W, E, info);
  });
  time_it("zhetrd (tridiagonal only)", [&] { return rocsolver_zhetrd(hd, rocblas_fill_upper, n, A, n, W, E, tau); });
  time_it("zheevdx (E > 0 half)", [&] {
    return rocsolver_zheevdx(hd, rocblas_evect_original, rocblas_erange_value, rocblas_fill_upper, n, A, n, 0.0,
                             1e300, 0, 0, nev, W, Z, n, info);
  });
  time_it("zheevdj", [&] { return rocsolver_zheevdj(hd, rocblas_evect_original, rocblas_fill_upper, n, A, n, W, info); });
  time_it("zheevj (1e-13, 20 sweeps)", [&] {
    return rocsolver_zheevj(hd, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_upper, n, A, n, 1e-13,
                            res, 20, sweeps, W, info);
  });
  rocblas_destroy_handle(hd);
  return 0;
}
