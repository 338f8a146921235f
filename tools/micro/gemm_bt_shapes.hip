// Timing of the eigensolver back-transform products at L = 32 (n = 2048,
// M = 1024 computed columns, 16 matrices): W = V^H U (K = n - 1, split in ks
// chunks) as 'C','N' on V in place, and as 'N','N' on a transposed copy of V;
// U -= V W2 ('N','N', K = 64).  Build: see tools/micro/README or
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc gemm_bt_shapes.hip
#include "dwhmc_gemm.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int n = 2048, M = 1024, NB = 64, batch = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t sA = (int64_t)n * n;
  double2 *A, *U, *Vt, *W;
  CK(hipMalloc(&A, sA * batch * sizeof(double2)));
  CK(hipMalloc(&U, sA * batch * sizeof(double2)));
  CK(hipMalloc(&Vt, (int64_t)NB * n * batch * sizeof(double2)));
  CK(hipMalloc(&W, (int64_t)8 * NB * n * batch * sizeof(double2)));
  CK(hipMemset(A, 0, sA * batch * sizeof(double2)));
  CK(hipMemset(U, 0, sA * batch * sizeof(double2)));
  CK(hipMemset(Vt, 0, (int64_t)NB * n * batch * sizeof(double2)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double2 one = make_double2(1, 0), zero = make_double2(0, 0), mone = make_double2(-1, 0);
  for (int ms : {2047, 1023, 511}) {
    for (int ks : {1, 4, 8}) {
      const int c = ks == 1 ? ms : std::max(16, ((ms + ks - 1) / ks + 15) / 16 * 16);
      const int nfull = ms / c, rem = ms - nfull * c, S = nfull + (rem > 0);
      const int64_t sW = (int64_t)NB * n, sWs = ks * sW;
      float tc = 0, tn = 0;
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(e0, 0));
        dwh::gemm_z_chunked('C', 'N', NB, M, c, rem > 0 ? rem : c, S, one, A + 1, n, c, sA, U + 1, n, c, sA, zero, W,
                            ks * NB, NB, sWs, batch, 0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (rep) tc += t / 3;
        CK(hipEventRecord(e0, 0));
        dwh::gemm_z_chunked('N', 'N', NB, M, c, rem > 0 ? rem : c, S, one, Vt, NB, (int64_t)c * NB, (int64_t)NB * n,
                            U + 1, n, c, sA, zero, W, ks * NB, NB, sWs, batch, 0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&t, e0, e1));
        if (rep) tn += t / 3;
      }
      const double fl = 6.0 * NB * M * (double)ms * batch;
      printf("W = V^H U  ms %4d ks %d: C,N %8.1f us (%5.1f TF)   N,N on V^T %8.1f us (%5.1f TF)\n", ms, ks, 1e3 * tc,
             fl / (tc * 1e-3) * 1e-12, 1e3 * tn, fl / (tn * 1e-3) * 1e-12);
    }
    float tu = 0;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(e0, 0));
      dwh::gemm_z('N', 'N', ms, M, NB, mone, A + 1, n, sA, W, NB, (int64_t)NB * n, one, U + 1, n, sA, batch, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (rep) tu += t / 3;
    }
    printf("U -= V W2  ms %4d     : N,N %8.1f us (%5.1f TF)\n", ms, 1e3 * tu, 6.0 * NB * M * (double)ms * batch / (tu * 1e-3) * 1e-12);
  }
  // J_mn = U^H (J U): M = n, N = n / 2, K = n, 'C','N' vs 'N','N' on U^H (A as scratch)
  for (int b2 : {batch}) {
    float tcn = 0, tnn = 0;
    for (int rep = 0; rep < 4; ++rep) {
      float t;
      CK(hipEventRecord(e0, 0));
      dwh::gemm_z('C', 'N', n, M, n, one, U, n, sA, A, n, sA, zero, W, n, (int64_t)n * M, b2 > 8 ? 8 : b2, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      if (rep) tcn += t / 3;
      CK(hipEventRecord(e0, 0));
      dwh::gemm_z('N', 'N', n, M, n, one, U, n, sA, A, n, sA, zero, W, n, (int64_t)n * M, b2 > 8 ? 8 : b2, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      if (rep) tnn += t / 3;
    }
    const double fl = 6.0 * n * M * (double)n * (b2 > 8 ? 8 : b2);
    printf("J_mn shape %d x %d x %d, batch %d: C,N %8.1f us (%5.1f TF)   N,N %8.1f us (%5.1f TF)\n", n, M, n,
           b2 > 8 ? 8 : b2, 1e3 * tcn, fl / (tcn * 1e-3) * 1e-12, 1e3 * tnn, fl / (tnn * 1e-3) * 1e-12);
  }
  return 0;
}
