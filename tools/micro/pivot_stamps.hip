// Diagnostic: phase timing of k_gj_pivot / k_gj_update2 via s_memtime stamps.
// Build: hipcc --offload-arch=gfx950 -O3 -DDWH_STAMPS -I../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc \
//        pivot_stamps.hip -o pivot_stamps
#include "../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc/dwhmc_kernels.hip"
#include <cstdio>
#include <random>
#include <vector>
using namespace dwh;
int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 1024, nbatch = argc > 2 ? atoi(argv[2]) : 15;
  Dims d{};
  d.N = N; d.Np = (N + 63) / 64 * 64; d.nb = d.Np / 64; d.nc = 1; d.P = nbatch; d.nbatch = nbatch;
  d.mat = (int64_t)d.Np * d.Np;
  std::vector<double2> h((size_t)nbatch * d.mat);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (int b = 0; b < nbatch; ++b)
    for (int i = 0; i < d.Np; ++i)
      for (int j = 0; j < d.Np; ++j)
        h[(size_t)b * d.mat + (size_t)i * d.Np + j] = make_double2(0.05 * U(g), (i == j ? -3.0 : 0.0) + 0.05 * U(g));
  double2 *M, *P, *C; double* ld;
  hipMalloc(&M, h.size() * 16); hipMalloc(&P, 2 * (size_t)nbatch * 4096 * 16);
  hipMalloc(&C, 2 * (size_t)nbatch * d.Np * 64 * 16); hipMalloc(&ld, nbatch * d.nb * 8);
  hipMemcpy(M, h.data(), h.size() * 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1, e2; hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    launch_gj_pivot(d, M, 0, P, C, C, nullptr, ld, 0);
    hipEventRecord(e1);
    { GJPanelPtrs pp{C, nullptr, C, nullptr, P, nullptr, nullptr, nullptr}; launch_gj_update(d, M, 0, 0, pp, 0); }
    hipEventRecord(e2);
    hipEventSynchronize(e2);
    float t1, t2; hipEventElapsedTime(&t1, e0, e1); hipEventElapsedTime(&t2, e1, e2);
    printf("rep %d: pivot %.1f us  update %.1f us\n", rep, t1 * 1e3, t2 * 1e3);
  }
  static unsigned long long st[4096][8];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof st);
  int nblk = d.nb * nbatch;
  double acc[8] = {0};
  int cnt = 0;
  for (int b = 0; b < nblk; ++b) {
    if (st[b][7] <= st[b][5]) continue;   // block k returns before the panel phases
    ++cnt;
    for (int i = 1; i < 8; ++i) acc[i] += (double)(st[b][i] - st[b][i - 1]);
  }
  nblk = cnt;
  const char* nm[8] = {"", "load S_kk", "inv16 (kb0)", "Xpanel (kb0)", "update (kb0)", "kb1..3", "col copy", "panel GEMM"};
  printf("mean cycles per phase over %d blocks (s_memtime ticks, 100 MHz?):\n", nblk);
  for (int i = 1; i < 8; ++i) printf("  %-14s %10.0f\n", nm[i], acc[i] / nblk);
  return 0;
}
