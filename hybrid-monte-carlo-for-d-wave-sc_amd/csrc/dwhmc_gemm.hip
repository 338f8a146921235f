// The library's own batched fp64 matrix products on the MFMA
// (v_mfma_f64_16x16x4_f64), replacing rocBLAS zgemm / dgemm on the
// measurement path and the eig fallback:
//   * J_mn = U^H (J U)                [src/Observables.jl:334-335]
//   * rho = (U f(E)) U^H              [eig path: ρ = U f(E) U† of compute_forces!]
//   * the eigensolver's back-transform (W = V^H U, U -= V W2) and Löwdin step
//     (G = Z Z^T, Y = 3/2 Y - 1/2 G Z), dwhmc_eig.hip / dwhmc_api.cpp
// C = alpha op(A) op(B) + beta C, column-major, op in {N, C} (C: conjugate
// transpose; transpose for real), complex (3 real MFMAs per complex MAC:
// t1 = Ar Br, t2 = Ai Bi, t3 = (Ar + Ai)(Br + Bi); re = t1 - t2,
// im = t3 - t1 - t2) or real.  Two-level batching: z = outer * S + s, operand
// offsets outer * s2 + s * s1 (the back-transform's K chunks), the last
// chunk of each outer batch with K = Klast.
//
// Tiling: one 256-thread workgroup per 64 x 64 output tile, four waves of
// 32 x 32 (2 x 2 MFMA tiles); K in chunks of 16 staged through LDS (k-major:
// the MFMA A / B fragments of one k-step are 16 consecutive m (n) per lane
// group, conflict-free ds_read_b128), double-buffered, the next chunk's
// global loads issued before the current chunk's MFMAs.  Epilogue through
// LDS: every thread stores whole 64-row column segments (1 KB coalesced per
// four columns), alpha / beta applied there.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {
namespace {

constexpr int GM = 64, GN = 64, GK = 16, GP = 1;   // tile, K chunk, LDS row padding (elements)

template <bool CPLX>
struct Elem;
template <>
struct Elem<true> {
  using T = double2;
  static __device__ __forceinline__ T zero() { return make_double2(0.0, 0.0); }
  static __device__ __forceinline__ T conj(T x) { return make_double2(x.x, -x.y); }
};
template <>
struct Elem<false> {
  using T = double;
  static __device__ __forceinline__ T zero() { return 0.0; }
  static __device__ __forceinline__ T conj(T x) { return x; }
};

struct GemmArgs {
  int M, N, K, Klast;
  const void* A;
  int lda;
  int64_t a1, a2;   // inner (chunk) / outer (batch) offsets, elements
  const void* B;
  int ldb;
  int64_t b1, b2;
  void* C;
  int ldc;
  int64_t c1, c2;
  double2 alpha, beta;
  int S;            // inner batch count
  int tiles_m;      // ceil(M / 64)
};

// one K chunk of op(A) (64 x 16) and op(B) (16 x 64) into registers: element
// e of thread t; OPA/OPB: 0 = N, 1 = C
template <bool CPLX, int OPA, int OPB>
struct Chunk {
  using T = typename Elem<CPLX>::T;
  T a[4], b[4];
  __device__ __forceinline__ void load(const T* A, int lda, const T* B, int ldb, int m0, int n0, int k0, int M,
                                       int N, int K) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (OPA == 0) {   // A[m + k lda], m contiguous
        const int m = m0 + (t & 63), k = k0 + (t >> 6) + 4 * j;
        a[j] = (m < M && k < K) ? A[m + (int64_t)k * lda] : Elem<CPLX>::zero();
      } else {                    // op(A)[m][k] = conj(A[k + m lda]), k contiguous
        const int k = k0 + (t & 15), m = m0 + (t >> 4) + 16 * j;
        a[j] = (m < M && k < K) ? Elem<CPLX>::conj(A[k + (int64_t)m * lda]) : Elem<CPLX>::zero();
      }
      if constexpr (OPB == 0) {   // B[k + n ldb], k contiguous
        const int k = k0 + (t & 15), n = n0 + (t >> 4) + 16 * j;
        b[j] = (n < N && k < K) ? B[k + (int64_t)n * ldb] : Elem<CPLX>::zero();
      } else {                    // op(B)[k][n] = conj(B[n + k ldb]), n contiguous
        const int n = n0 + (t & 63), k = k0 + (t >> 6) + 4 * j;
        b[j] = (n < N && k < K) ? Elem<CPLX>::conj(B[n + (int64_t)k * ldb]) : Elem<CPLX>::zero();
      }
    }
  }
  // LDS images As[k][m], Bs[k][n] (row stride GM + GP)
  __device__ __forceinline__ void store(T* As, T* Bs) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (OPA == 0) As[((t >> 6) + 4 * j) * (GM + GP) + (t & 63)] = a[j];
      else As[(t & 15) * (GM + GP) + (t >> 4) + 16 * j] = a[j];
      if constexpr (OPB == 0) Bs[(t & 15) * (GN + GP) + (t >> 4) + 16 * j] = b[j];
      else Bs[((t >> 6) + 4 * j) * (GN + GP) + (t & 63)] = b[j];
    }
  }
};

template <bool CPLX, int OPA, int OPB>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  using E = Elem<CPLX>;
  using T = typename E::T;
  constexpr int NACC = CPLX ? 3 : 1;
  constexpr int IMG = GK * (GM + GP);   // one K-chunk image (GM == GN)
  __shared__ T smem[4 * IMG];           // As[2], Bs[2]; the epilogue tile 64 x (64 + GP) reuses all of it
  static_assert(GM == GN && 4 * IMG >= GN * (GM + GP), "epilogue tile fits the LDS images");
  // K-chunk images: As[b] = smem + b IMG, Bs[b] = smem + (2 + b) IMG
  const int z = blockIdx.y, outer = z / g.S, s = z - outer * g.S;
  const int tm = blockIdx.x % g.tiles_m, tn = blockIdx.x / g.tiles_m;
  const int m0 = tm * GM, n0 = tn * GN;
  const int K = s == g.S - 1 ? g.Klast : g.K;
  const T* A = static_cast<const T*>(g.A) + outer * g.a2 + s * g.a1;
  const T* B = static_cast<const T*>(g.B) + outer * g.b2 + s * g.b1;
  T* C = static_cast<T*>(g.C) + outer * g.c2 + s * g.c1;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  d4 acc[NACC][2][2];
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = d4{0.0, 0.0, 0.0, 0.0};
  Chunk<CPLX, OPA, OPB> ch;
  const int nk = (K + GK - 1) / GK;
  if (nk > 0) {
    ch.load(A, g.lda, B, g.ldb, m0, n0, 0, g.M, g.N, K);
    ch.store(smem, smem + 2 * IMG);
  }
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) ch.load(A, g.lda, B, g.ldb, m0, n0, (kc + 1) * GK, g.M, g.N, K);
    const T* as = smem + cur * IMG;
    const T* bs = smem + (2 + cur) * IMG;
#pragma unroll
    for (int ks = 0; ks < GK / 4; ++ks) {
      const int k = 4 * ks + lk;
      T av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = as[k * (GM + GP) + wm + 16 * i + lr];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = bs[k * (GN + GP) + wn + 16 * j + lr];
      if constexpr (CPLX) {
        double as_[2], bs_[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) as_[i] = av[i].x + av[i].y;
#pragma unroll
        for (int j = 0; j < 2; ++j) bs_[j] = bv[j].x + bv[j].y;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[0][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i].x, bv[j].x, acc[0][i][j], 0, 0, 0);
            acc[1][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i].y, bv[j].y, acc[1][i][j], 0, 0, 0);
            acc[2][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(as_[i], bs_[j], acc[2][i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[0][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[0][i][j], 0, 0, 0);
      }
    }
    if (kc + 1 < nk) ch.store(smem + (cur ^ 1) * IMG, smem + (2 + (cur ^ 1)) * IMG);
    __syncthreads();
  }
  // epilogue: the 64 x 64 tile column-major in LDS (reusing the A / B images),
  // then whole column segments per thread
  T* Cs = smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = wm + 16 * i + lk + 4 * rr, col = wn + 16 * j + lr;
        T v;
        if constexpr (CPLX) {
          const double t1 = acc[0][i][j][rr], t2 = acc[1][i][j][rr], t3 = acc[2][i][j][rr];
          v = make_double2(t1 - t2, t3 - t1 - t2);
        } else {
          v = acc[0][i][j][rr];
        }
        Cs[col * (GM + GP) + row] = v;
      }
  __syncthreads();
  const int row = threadIdx.x & 63, gr = m0 + row;
  if (gr >= g.M) return;
  const bool beta0 = g.beta.x == 0.0 && g.beta.y == 0.0;
#pragma unroll 4
  for (int c = threadIdx.x >> 6; c < GN; c += 4) {
    const int gc = n0 + c;
    if (gc >= g.N) break;
    const T v = Cs[c * (GM + GP) + row];
    T* dst = C + gr + (int64_t)gc * g.ldc;
    if constexpr (CPLX) {
      double2 o = make_double2(g.alpha.x * v.x - g.alpha.y * v.y, g.alpha.x * v.y + g.alpha.y * v.x);
      if (!beta0) {
        const double2 cv = *dst;
        o.x += g.beta.x * cv.x - g.beta.y * cv.y;
        o.y += g.beta.x * cv.y + g.beta.y * cv.x;
      }
      *dst = o;
    } else {
      double o = g.alpha.x * v;
      if (!beta0) o += g.beta.x * *dst;
      *dst = o;
    }
  }
}

template <bool CPLX>
void launch(char opa, char opb, const GemmArgs& g, int nz, hipStream_t s) {
  const dim3 grid(g.tiles_m * ((g.N + GN - 1) / GN), nz), block(256);
  const bool ca = opa != 'N', cb = opb != 'N';
  if (!ca && !cb) hipLaunchKernelGGL((k_gemm<CPLX, 0, 0>), grid, block, 0, s, g);
  else if (ca && !cb) hipLaunchKernelGGL((k_gemm<CPLX, 1, 0>), grid, block, 0, s, g);
  else if (!ca && cb) hipLaunchKernelGGL((k_gemm<CPLX, 0, 1>), grid, block, 0, s, g);
  else hipLaunchKernelGGL((k_gemm<CPLX, 1, 1>), grid, block, 0, s, g);
}

}  // namespace

void gemm_z(char opa, char opb, int M, int N, int K, double2 alpha, const double2* A, int lda, int64_t sA,
            const double2* B, int ldb, int64_t sB, double2 beta, double2* C, int ldc, int64_t sC, int batch,
            hipStream_t s) {
  gemm_z_chunked(opa, opb, M, N, K, K, 1, alpha, A, lda, 0, sA, B, ldb, 0, sB, beta, C, ldc, 0, sC, batch, s);
}

void gemm_z_chunked(char opa, char opb, int M, int N, int K, int Klast, int S, double2 alpha, const double2* A,
                    int lda, int64_t a1, int64_t a2, const double2* B, int ldb, int64_t b1, int64_t b2,
                    double2 beta, double2* C, int ldc, int64_t c1, int64_t c2, int batch, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0 || S <= 0) return;
  GemmArgs g{M, N, K, Klast, A, lda, a1, a2, B, ldb, b1, b2, C, ldc, c1, c2, alpha, beta, S, (M + GM - 1) / GM};
  launch<true>(opa, opb, g, batch * S, s);
}

void gemm_d(char opa, char opb, int M, int N, int K, double alpha, const double* A, int lda, int64_t sA,
            const double* B, int ldb, int64_t sB, double beta, double* C, int ldc, int64_t sC, int batch,
            hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return;
  GemmArgs g{M, N, K, K, A, lda, 0, sA, B, ldb, 0, sB, C, ldc, 0, sC, make_double2(alpha, 0.0),
             make_double2(beta, 0.0), 1, (M + GM - 1) / GM};
  launch<false>(opa, opb, g, batch, s);
}

}  // namespace dwh
