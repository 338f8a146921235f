// Diagnostic: phase timing of k_cr_inv via s_memtime stamps (shader clock).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCR_STAMPS cr_inv_stamps.hip -o cr_inv_stamps
// Run:   ./cr_inv_stamps [BP=64] [nbatch=15] [nblocks=1]
#include "../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc/dwhmc_cr.hip"
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
using namespace dwh;
int main(int argc, char** argv) {
  const int BP = argc > 1 ? atoi(argv[1]) : 64, nbatch = argc > 2 ? atoi(argv[2]) : 15;
  const int nblk = argc > 3 ? atoi(argv[3]) : 1;
  CrDims c{};
  c.Lx = BP / 2; c.Ly = nblk; c.N = c.Lx * c.Ly; c.BP = BP; c.P = nbatch; c.nbatch = nbatch; c.nblk = nblk;
  c.item = (int64_t)nblk * BP * BP;
  std::vector<double2> h((size_t)nbatch * c.item);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (size_t e = 0; e < h.size(); ++e) {
    const int i = (e / BP) % BP, j = e % BP;
    h[e] = make_double2(0.1 * U(g), (i == j ? -1.0 : 0.0) + 0.1 * U(g));
  }
  double2* M; double* ld; int *blk, *slot;
  hipMalloc(&M, h.size() * 16); hipMalloc(&ld, nbatch * nblk * 8);
  std::vector<int> hb(nblk), hs(nblk);
  for (int i = 0; i < nblk; ++i) hb[i] = hs[i] = i;
  hipMalloc(&blk, nblk * 4); hipMalloc(&slot, nblk * 4);
  hipMemcpy(blk, hb.data(), nblk * 4, hipMemcpyHostToDevice);
  hipMemcpy(slot, hs.data(), nblk * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 4; ++rep) {
    hipMemcpy(M, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    hipEventRecord(e0);
    launch_cr_inv(c, M, blk, blk, slot, nblk, ld, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t; hipEventElapsedTime(&t, e0, e1);
    printf("rep %d: k_cr_inv<%d> %d x %d blocks: %.1f us\n", rep, BP / 16, nblk, nbatch, t * 1e3);
  }
  static unsigned long long st[1024][16];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_cr_stamps), sizeof st);
  const int nb = nblk * nbatch;
  double acc[6] = {0};
  for (int b = 0; b < nb; ++b)
    for (int i = 1; i < 6; ++i) acc[i] += (double)(st[b][i] - st[b][i - 1]);
  const char* nm[6] = {"", "load block", "pivot 0 inverse", "step kb=0 (wave 0)", "steps kb=1..",
                       "store+ld"};
  printf("mean s_memtime ticks per phase over %d blocks (wave 0's view):\n", nb);
  for (int i = 1; i < 6; ++i) printf("  %-20s %10.0f\n", nm[i], acc[i] / nb);
  return 0;
}
