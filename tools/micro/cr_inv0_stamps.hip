// Diagnostic: phase timing of k_cr_inv0 (level-0 inversions from the static
// R = A^-1, BP = 64) and of k_cr_inv<4> via s_memtime stamps (shader clock).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCR_STAMPS cr_inv0_stamps.hip -o cr_inv0_stamps
// Run:   ./cr_inv0_stamps [nbatch=12] [nblocks=16]
#include "../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc/dwhmc_cr.hip"
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
using namespace dwh;

static void report(const char* what, int nb, const char* const* nm, int nph) {
  static unsigned long long st[1024][16];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_cr_stamps), sizeof st);
  std::vector<double> acc(nph, 0.0);
  double tot = 0;
  for (int b = 0; b < nb; ++b) {
    for (int i = 1; i < nph; ++i) acc[i] += (double)(st[b][i] - st[b][i - 1]);
    tot += (double)(st[b][nph - 1] - st[b][0]);
  }
  printf("%s: mean s_memtime ticks per phase over %d workgroups (wave 0's view), total %.0f\n", what, nb, tot / nb);
  for (int i = 1; i < nph; ++i) printf("  %-34s %8.0f\n", nm[i], acc[i] / nb);
}

int main(int argc, char** argv) {
  const int nbatch = argc > 1 ? atoi(argv[1]) : 12, nblk = argc > 2 ? atoi(argv[2]) : 16;
  const int BP = 64, HP = 32;
  CrDims c{};
  c.Lx = HP; c.Ly = nblk; c.N = c.Lx * c.Ly; c.BP = BP; c.P = nbatch; c.nbatch = nbatch;
  c.nblk = 3 * nblk;              // D blocks, R blocks, outputs
  c.item = (int64_t)c.nblk * HP * BP;
  std::vector<double2> h((size_t)nbatch * c.item);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (size_t e = 0; e < h.size(); ++e) {
    const int i = (e / BP) % HP, j = e % BP;
    const bool diag = (i == j);
    h[e] = make_double2(0.05 * U(g) + (diag ? 1.0 : 0.0), (diag ? -0.7 : 0.0) + 0.05 * U(g));
  }
  double2* M; double *ld, *ldA; int *blk, *rblk, *dst, *slot;
  hipMalloc(&M, h.size() * 16); hipMalloc(&ld, nbatch * nblk * 8); hipMalloc(&ldA, nbatch * nblk * 8);
  hipMemset(ldA, 0, nbatch * nblk * 8);
  std::vector<int> hb(nblk), hr(nblk), hd(nblk), hs(nblk);
  for (int i = 0; i < nblk; ++i) { hb[i] = i; hr[i] = nblk + i; hd[i] = 2 * nblk + i; hs[i] = i; }
  hipMalloc(&blk, nblk * 4); hipMalloc(&rblk, nblk * 4); hipMalloc(&dst, nblk * 4); hipMalloc(&slot, nblk * 4);
  hipMemcpy(blk, hb.data(), nblk * 4, hipMemcpyHostToDevice);
  hipMemcpy(rblk, hr.data(), nblk * 4, hipMemcpyHostToDevice);
  hipMemcpy(dst, hd.data(), nblk * 4, hipMemcpyHostToDevice);
  hipMemcpy(slot, hs.data(), nblk * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 4; ++rep) {
    hipMemcpy(M, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    hipEventRecord(e0);
    launch_cr_inv0(c, M, blk, rblk, dst, slot, nblk, ld, ldA, 0, nullptr, nullptr, 0.0, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t; hipEventElapsedTime(&t, e0, e1);
    printf("rep %d: k_cr_inv0 %d x %d blocks: %.1f us\n", rep, nblk, nbatch, t * 1e3);
  }
  const char* nm0[10] = {"", "load A/B/R + barrier", "Z = R B + barrier", "S = A + B conj Z, S00^-1 (w0) + barrier",
                         "P, Q; P, T, T^-1 (w3) + barrier", "(merged into the previous)",
                         "X01, X10, X00 = S00^-1 + P T^-1 Q + barrier", "(merged into the previous)",
                         "Y = Z conj X", "store + ln|det|"};
  report("k_cr_inv0", nblk * nbatch, nm0, 10);
  for (int rep = 0; rep < 4; ++rep) {
    hipMemcpy(M, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    hipEventRecord(e0);
    launch_cr_inv(c, M, blk, dst, slot, nblk, ld, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t; hipEventElapsedTime(&t, e0, e1);
    printf("rep %d: k_cr_inv<4> %d x %d blocks: %.1f us\n", rep, nblk, nbatch, t * 1e3);
  }
  const char* nm1[6] = {"", "load block", "pivot 0 inverse", "step kb=0 (wave 0)", "steps kb=1..", "store+ld"};
  report("k_cr_inv<4>", nblk * nbatch, nm1, 6);
  return 0;
}
