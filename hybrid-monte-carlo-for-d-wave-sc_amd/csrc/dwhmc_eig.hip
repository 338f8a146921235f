// Hermitian eigensolver of the measurement path and of the eig fallback:
// every eigenpair of m dense n x n H_BdG matrices (column-major, lower
// triangle referenced), replacing LAPACK's eigen!(Hermitian(H)) of
// diagonalize_H_BdG! [src/Hamiltonian.jl:96-114] as measure_transport_and_spectra
// [src/Observables.jl:314-526] and the eig path use it.  No vendor solver:
//
//  1. Householder tridiagonalisation, LAPACK zhetd2 'L' algebra (reflectors
//     H_i = I - tau_i v_i v_i^H, v_i[i+1] = 1, beta_i real so T is real
//     symmetric).  Per column, batched over the m matrices:
//       k_eig_reduce (one thread per row): the previous pass's hemv partials
//                   summed per row into p = A v_{i-1} and column i, both with
//                   the rank-2 pairs the trailing triangle still lacks;
//       k_eig_step  (one workgroup per matrix): w_{i-1} = tau p - 1/2 tau
//                   (tau p)^H v v, pair i-1 on column i, the reflector of
//                   column i (zlarfg); column i of A becomes v_i (zeros above
//                   i+1), so A ends as the dense V the back-transform uses;
//       k_eig_pass  (one workgroup per 64 x 64 lower-triangle tile of the
//                   trailing matrix): every K-th pass applies the pending
//                   pairs to the tile and writes it back, the others only
//                   read it (K = 8 for batches: HBM-bound, 9/16 of the
//                   read + write traffic; K = 1 for one matrix); each
//                   accumulates the tile's share of A v_i, partials written
//                   once per slot and summed in a fixed order
//                   (bit-reproducible).
//  2. k_eig_bisect: every eigenvalue of T on Sturm counts, 64 (one matrix)
//     down to 4 (batches) lanes per eigenvalue index, a multisection per
//     round down to the last bit.
//  3. k_eig_invit: inverse iteration, T - lambda I = LU with partial pivoting
//     streamed per thread (two solves from a fixed pseudo-random start,
//     one thread per eigenvalue); k_eig_orth: the vectors of eigenvalue
//     clusters (consecutive gaps <= kEigClusterTol = 1e-6 ||T||, up to
//     kEigMaxCluster long; longer ones by the same Cholesky QR on the
//     library's products, driven from the host) orthonormalised by Cholesky
//     QR, twice (exact degeneracies of clean lattices included).  Every other pair is orthogonal only to
//     ~eps ||T|| / gap <= ~2e-10 after inverse iteration; one symmetric
//     (Löwdin) orthogonalisation step over all vectors (the library's real
//     products, dwhmc_gemm.hip, driven by dwhmc_api.cpp) takes those overlaps
//     to rounding.  (kEigZeroTol = 2.5e-4 ||T|| is a different tolerance: the
//     particle-hole split point c0 below.)
//     For H_BdG (the only matrices the library decomposes) steps 3-4 run on
//     the upper half of the spectrum only: from c0 (n/2, or lower when the
//     levels around zero are closer than kEigZeroTol, found on the host from
//     the eigenvalues), and k_eig_theta
//     fills the columns below c0 with the particle-hole partners
//     (u; v) -> (-conj v; conj u) of the columns above n - c0.
//  4. U = H_0 H_1 ... H_{n-2} Z: reflectors in blocks of kEigNB as
//     I - V T V^H (k_eig_tfac: compact-WY T per block), applied last block
//     first: W = V^H U (the library's complex product, split over K into
//     chunks when few matrices are batched, its output being only kEigNB x
//     n), W2 = T sum of the chunks (k_eig_tw), U -= V W2.
//
// The numpy prototype with the same operation order: tools/eig_proto.py.
#include <cfloat>
#include <cstdlib>
#include <algorithm>

#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {
namespace {

constexpr int kStepT = 1024;   // threads of k_eig_step

// sums over the workgroup (fixed order: xor-shuffle tree per wave, then the
// waves in index order); every thread returns the totals.  sh: one slot per
// wave and value, not shared with another reduction of the same phase.
__device__ __forceinline__ double group_sum(double v, double* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < nw; ++k) s += sh[k];
  return s;
}
__device__ __forceinline__ double2 group_sum2(double2 v, double2* sh) {
  v.x = wave_sum(v.x);
  v.y = wave_sum(v.y);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double2 s = make_double2(0.0, 0.0);
  for (int k = 0; k < nw; ++k) {
    s.x += sh[k].x;
    s.y += sh[k].y;
  }
  return s;
}

__device__ __forceinline__ double2 cz() { return make_double2(0.0, 0.0); }

// Deferred rank-2 pairs (pair j = (v_j, w_j), the update zhetd2 applies after
// column j).  Pass i (trailing rows / columns >= i+1) writes A only when
// eig_write_pass(i, K): it applies every pending pair j in
// [eig_pend_first(i, K), i-1] (at most K) to its tile before the hemv.  The
// other passes read A as it stands, stale by those pairs, and their diagonal
// tiles add the dots w_j^H v_i, v_j^H v_i over their rows, with which
// k_eig_reduce corrects the hemv: A v = A_stale v - sum_j v_j (w_j^H v) +
// w_j (v_j^H v).  K = 1: every pass writes, pending = {pair i-1}.  Batches of
// kEigDeferMin+ matrices use K = kEigDefer (HBM-bound passes: (K-1)/K of the
// column sweeps only read); one matrix K = 1 (latency-bound).  Same algebra:
// tools/eig_proto.py tridiagonalize_deferred.
__host__ __device__ __forceinline__ bool eig_write_pass(int i, int K) { return i % K == K - 1; }
__host__ __device__ __forceinline__ int eig_pend_first(int i, int K) { return i >= K ? (i / K) * K - 1 : 0; }
constexpr int KD = kEigDeferMax;

// k_eig_reduce (before step i >= 1): the pass i-1 partials of every row summed
// (ascending tile index), less the pairs pass i-1 left out (read pass), into
// pfin = A^{(i-1)} v_{i-1}; column i of A with those pairs applied into colfin
// (the step applies pair i-1 itself).  One thread per row, many workgroups,
// so the single-workgroup step reads 2 n values.
// gpart (one matrix, k_eig_pass1f follows): this workgroup's share of
// g = sum_r conj(tau_{i-1} p_r) v_{i-1}[r], summed in a fixed order.
__global__ __launch_bounds__(256) void k_eig_reduce(const double2* __restrict__ part, int64_t sP, int n, int i,
                                                    double2* __restrict__ pfin, const double2* __restrict__ A,
                                                    int64_t sA, double2* __restrict__ colfin,
                                                    const double2* __restrict__ vv, const double2* __restrict__ ww,
                                                    const double2* __restrict__ dpart, int K,
                                                    const double2* __restrict__ tau, double2* __restrict__ gpart) {
  const int k = blockIdx.y, tid = threadIdx.x, r = i + blockIdx.x * 256 + tid;
  const int t0 = i / kEigTB, T = (n + kEigTB - 1) / kEigTB;
  const bool rd = !eig_write_pass(i - 1, K);
  const int f = eig_pend_first(i - 1, K), np = rd ? i - 1 - f : 0;
  __shared__ double2 dots[2 * KD];
  if (tid < 2 * np) {   // ascending tile order, 16 loads in flight
    double2 s = cz();
    for (int Y0 = t0; Y0 < T; Y0 += 16) {
      double2 q[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) q[u] = Y0 + u < T ? dpart[((int64_t)k * T + Y0 + u) * 2 * KD + tid] : cz();
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (Y0 + u < T) s = cadd(s, q[u]);
    }
    dots[tid] = s;
  }
  __syncthreads();
  const bool ok = r < n;
  part += k * sP;
  vv += (int64_t)k * kEigRing * n;
  ww += (int64_t)k * kEigRing * n;
  double2 s = cz();
  if (ok) {
    constexpr int YB = 16;   // partial rows in flight per thread
    for (int Y0 = t0; Y0 < T; Y0 += YB) {
      double2 q[YB];
#pragma unroll
      for (int u = 0; u < YB; ++u) q[u] = Y0 + u < T ? part[(int64_t)(Y0 + u) * n + r] : cz();
#pragma unroll
      for (int u = 0; u < YB; ++u)
        if (Y0 + u < T) s = cadd(s, q[u]);
    }
    double2 c = A[k * sA + r + (int64_t)i * n];
    // the pending pairs' entries all loaded before the corrections (np < KD)
    double2 vj[KD], wj[KD], vji[KD], wji[KD];
#pragma unroll
    for (int q = 0; q < KD; ++q) {
      if (q < np) {
        const int sl = (f + q) % kEigRing;
        vj[q] = vv[(int64_t)sl * n + r];
        wj[q] = ww[(int64_t)sl * n + r];
        vji[q] = vv[(int64_t)sl * n + i];
        wji[q] = ww[(int64_t)sl * n + i];
      }
    }
#pragma unroll
    for (int q = 0; q < KD; ++q) {
      if (q < np) {
        s = csub(csub(s, cmul(vj[q], dots[2 * q])), cmul(wj[q], dots[2 * q + 1]));
        c = csub(csub(c, cmulc(vj[q], wji[q])), cmulc(wj[q], vji[q]));
      }
    }
    pfin[(int64_t)k * n + r] = s;
    colfin[(int64_t)k * n + r] = c;
  }
  if (gpart) {
    // g = sum conj(x_r) v_r (x = tau p, rows >= i), and for the norm of the
    // updated column c = a - bu v (a = c0 - x) over the rows >= i+2:
    // S1 = sum |a|^2, S2 = sum conj(v) a, S3 = sum |v|^2
    __shared__ double2 sg[3][kStepT / 64];
    const double2 tp = tau[(int64_t)k * n + i - 1];
    const double2 x = cmul(tp, s);
    const double2 v = ok ? vv[(int64_t)((i + kEigRing - 1) % kEigRing) * n + r] : cz();
    double2 gq = make_double2(x.x * v.x + x.y * v.y, x.x * v.y - x.y * v.x);   // conj(x) v
    double2 s1 = cz(), s2 = cz();
    if (ok && r >= i + 2) {
      const double2 av = csub(colfin[(int64_t)k * n + r], x);
      s1 = make_double2(av.x * av.x + av.y * av.y, v.x * v.x + v.y * v.y);      // (S1, S3)
      s2 = make_double2(v.x * av.x + v.y * av.y, v.x * av.y - v.y * av.x);      // conj(v) a
    }
    // the three sums in one workgroup reduction (wave trees, then the waves
    // in index order: one barrier)
    gq.x = wave_sum(gq.x);
    gq.y = wave_sum(gq.y);
    s1.x = wave_sum(s1.x);
    s1.y = wave_sum(s1.y);
    s2.x = wave_sum(s2.x);
    s2.y = wave_sum(s2.y);
    const int wv = tid >> 6, nw = blockDim.x >> 6;
    if ((tid & 63) == 0) {
      sg[0][wv] = gq;
      sg[1][wv] = s1;
      sg[2][wv] = s2;
    }
    __syncthreads();
    if (tid == 0) {
      gq = s1 = s2 = cz();
      for (int q = 0; q < nw; ++q) {
        gq = cadd(gq, sg[0][q]);
        s1 = cadd(s1, sg[1][q]);
        s2 = cadd(s2, sg[2][q]);
      }
      double2* gp = gpart + ((int64_t)k * kEigGP + blockIdx.x) * 3;
      gp[0] = gq;
      gp[1] = s1;
      gp[2] = s2;
    }
  }
}

// Step i: w_{i-1} from p = pfin (w = x - 1/2 tau (x^H v) v, x = tau p, zhetd2
// 'L'), pair i-1 applied to column i (colfin, or A for i = 0), the reflector
// of column i (zlarfg) into v_i and column i of A.  Every load is issued up
// front; two workgroup reductions are its only barriers.
// Step i: see k_eig_reduce; every load is issued up front.
template <int kMaxR>   // row slots per thread: ceil(n / kStepT)
__global__ __launch_bounds__(kStepT) void k_eig_step(double2* __restrict__ A, int n, int i, int64_t sA,
                                                     const double2* __restrict__ pfin,
                                                     const double2* __restrict__ colfin,
                                                     double2* __restrict__ vv, double2* __restrict__ ww,
                                                     double* __restrict__ d, double* __restrict__ e,
                                                     double2* __restrict__ tau) {
  const int k = blockIdx.x, tid = threadIdx.x;
  A += k * sA;
  pfin += (int64_t)k * n;
  colfin += (int64_t)k * n;
  vv += (int64_t)k * kEigRing * n;
  ww += (int64_t)k * kEigRing * n;
  d += (int64_t)k * n;
  e += (int64_t)k * n;
  tau += (int64_t)k * n;
  __shared__ double2 sh1[kStepT / 64];
  __shared__ double sh2[kStepT / 64];
  __shared__ double2 bc;
  double2* vcur = vv + (int64_t)(i % kEigRing) * n;
  const double2* vprv = vv + (int64_t)((i + kEigRing - 1) % kEigRing) * n;   // v_{i-1}
  double2* wout = ww + (int64_t)((i + kEigRing - 1) % kEigRing) * n;        // w_{i-1}
  double2 cr[kMaxR], vp[kMaxR], wr[kMaxR];
#pragma unroll
  for (int s = 0; s < kMaxR; ++s) {
    const int r = i + tid + s * kStepT;
    cr[s] = vp[s] = wr[s] = cz();
    if (r < n) {
      cr[s] = i > 0 ? colfin[r] : A[r];
      if (i > 0) {
        vp[s] = vprv[r];
        wr[s] = pfin[r];
      }
    }
  }
  const double2 pi = i > 0 ? pfin[i] : cz();   // p[i] (v_{i-1}[i] = 1: w[i] = x[i] + alpha)
  double2 wi = cz();
  if (i > 0) {
    const double2 tp = tau[i - 1];
    double2 g = cz();
#pragma unroll
    for (int s = 0; s < kMaxR; ++s) {
      wr[s] = cmul(tp, wr[s]);
      g.x += wr[s].x * vp[s].x + wr[s].y * vp[s].y;
      g.y += wr[s].x * vp[s].y - wr[s].y * vp[s].x;
    }
    g = group_sum2(g, sh1);
    const double2 al = cmul(tp, make_double2(-0.5 * g.x, -0.5 * g.y));
    wi = cadd(cmul(tp, pi), al);
#pragma unroll
    for (int s = 0; s < kMaxR; ++s) {
      const int r = i + tid + s * kStepT;
      wr[s] = cadd(wr[s], cmul(al, vp[s]));
      if (r < n) wout[r] = wr[s];
    }
  }
  // column i with pair i-1 (v_{i-1}[i] = 1)
  double xn = 0.0;
#pragma unroll
  for (int s = 0; s < kMaxR; ++s) {
    const int r = i + tid + s * kStepT;
    if (r < n) {
      double2 c = cr[s];
      if (i > 0) c = csub(csub(c, cmulc(vp[s], wi)), wr[s]);
      cr[s] = c;
      if (r >= i + 2) xn += c.x * c.x + c.y * c.y;
      if (r == i) d[i] = c.x;
      if (r == i + 1) bc = c;
    }
  }
  if (i == n - 1) return;
  xn = group_sum(xn, sh2);   // its barrier publishes bc
  const double2 al = bc;
  // zlarfg: beta = -sign(Re alpha) ||(alpha, x)||, tau = (beta - alpha) / beta, v = x / (alpha - beta)
  double2 t = cz(), sc = cz();
  double beta = al.x;
  if (!(xn == 0.0 && al.y == 0.0)) {
    beta = -copysign(sqrt(al.x * al.x + al.y * al.y + xn), al.x);
    t = make_double2((beta - al.x) / beta, -al.y / beta);
    sc = cinv(make_double2(al.x - beta, al.y));
  }
#pragma unroll
  for (int s = 0; s < kMaxR; ++s) {
    const int r = i + tid + s * kStepT;
    if (r >= i + 1 && r < n) {
      const double2 v = r == i + 1 ? make_double2(1.0, 0.0) : cmul(cr[s], sc);
      vcur[r] = v;
      A[r + (int64_t)i * n] = v;
    }
  }
  for (int r = tid; r <= i; r += kStepT) A[r + (int64_t)i * n] = cz();
  if (tid == 0) {
    e[i] = beta;
    tau[i] = t;
  }
}

// tile (R, C), R >= C, of the trailing lower triangle [t0, T)^2 from a linear index
__device__ __forceinline__ void tri_decode(int b, int& R, int& C) {
  int r = (int)((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= b) ++r;
  while (r * (r + 1) / 2 > b) --r;
  R = r;
  C = b - r * (r + 1) / 2;
}

// Pass i over the trailing lower triangle (rows / cols >= i+1), one
// workgroup per 64 x 64 tile: a write pass applies the pending pairs to the
// tile and writes it back; every pass accumulates the tile's share of A v_i
// into fixed partial slots, and a read pass's diagonal tiles the dots of the
// pending pairs with v_i.
// The scalars of column i that k_eig_step forms, from k_eig_reduce's
// per-workgroup partials (g, S1/S3, S2; fixed order): al = -1/2 tau g,
// w_{i-1}[i], bu = conj(w_{i-1}[i]) + al (column c = c0 - tau p - bu v_{i-1}),
// ||c_{i+2:}||^2 = S1 - 2 Re(conj(bu) S2) + |bu|^2 S3 (a sweep over the rows
// where that cancels), and the reflector (zlarfg).  Every thread of every
// workgroup gets the same bits; sx: 4 doubles of LDS.
struct ColScal {
  double2 tp, al, bu, sc, t;
  double beta, di;
};
__device__ __forceinline__ ColScal col_scalars(int n, int i, const double2* __restrict__ pfin,
                                               const double2* __restrict__ colfin, const double2* __restrict__ vp,
                                               const double2* __restrict__ gpart, int ngp, double2 tp, double* sx) {
  ColScal q;
  q.tp = tp;
  double2 g = cz(), s13 = cz(), s2 = cz();
  for (int b = 0; b < ngp; ++b) {
    g = cadd(g, gpart[3 * b]);
    s13 = cadd(s13, gpart[3 * b + 1]);
    s2 = cadd(s2, gpart[3 * b + 2]);
  }
  q.al = cmul(tp, make_double2(-0.5 * g.x, -0.5 * g.y));
  const double2 wi = cadd(cmul(tp, pfin[i]), q.al);
  q.bu = make_double2(wi.x + q.al.x, q.al.y - wi.y);   // conj(wi) + al
  const double b2 = q.bu.x * q.bu.x + q.bu.y * q.bu.y;
  double xn = s13.x - 2.0 * (q.bu.x * s2.x + q.bu.y * s2.y) + b2 * s13.y;
  if (!(xn >= 1e-3 * (s13.x + b2 * s13.y))) {
    xn = 0.0;
    for (int r = i + 2 + (int)threadIdx.x; r < n; r += blockDim.x) {
      const double2 c = csub(csub(colfin[r], cmul(tp, pfin[r])), cmul(q.bu, vp[r]));
      xn += c.x * c.x + c.y * c.y;
    }
    xn = group_sum(xn, sx);
  }
  const double2 ci = csub(csub(colfin[i], cmul(tp, pfin[i])), q.bu);   // v_{i-1}[i] = 1
  q.di = ci.x;
  const double2 alpha = csub(csub(colfin[i + 1], cmul(tp, pfin[i + 1])), cmul(q.bu, vp[i + 1]));
  // zlarfg: beta = -sign(Re alpha) ||(alpha, x)||, tau = (beta - alpha) / beta, v = x / (alpha - beta)
  q.t = cz();
  q.sc = cz();
  q.beta = alpha.x;
  if (!(xn == 0.0 && alpha.y == 0.0)) {
    q.beta = -copysign(sqrt(alpha.x * alpha.x + alpha.y * alpha.y + xn), alpha.x);
    q.t = make_double2((q.beta - alpha.x) / q.beta, -alpha.y / q.beta);
    q.sc = cinv(make_double2(alpha.x - q.beta, alpha.y));
  }
  return q;
}
// v_i and w_{i-1} at an index x >= i+1 from (p, c0, v_{i-1}) there
__device__ __forceinline__ double2 col_vnew(const ColScal& q, int x, int i, double2 px, double2 cx, double2 vx) {
  return x == i + 1 ? make_double2(1.0, 0.0) : cmul(csub(csub(cx, cmul(q.tp, px)), cmul(q.bu, vx)), q.sc);
}

template <int KM>   // most pending pairs (kEigDeferMax; K = 1 runs k_eig_pass1 / 1f)
__global__ __launch_bounds__(256) void k_eig_pass(double2* __restrict__ A, int n, int i, int64_t sA,
                                                  double2* __restrict__ part, int64_t sP,
                                                  const double2* __restrict__ vv, const double2* __restrict__ ww,
                                                  int t0, double2* __restrict__ dpart, int T, int K) {
  const int k = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  A += k * sA;
  part += k * sP;
  vv += (int64_t)k * kEigRing * n;
  ww += (int64_t)k * kEigRing * n;
  const double2* v = vv + (int64_t)(i % kEigRing) * n;
  const bool wp = eig_write_pass(i, K);
  const int f = eig_pend_first(i, K), np = i - f;   // pending pairs f .. i-1 (<= KM)
  int R, C;
  tri_decode(blockIdx.x, R, C);
  R += t0;
  C += t0;
  __shared__ double2 cv[64], csum[64];
  __shared__ double2 rowp[4][64];
  // the pending pairs' column values (write pass) and the column-sum
  // transpose; for KM > 2 one LDS region, the two phases split by a barrier
  constexpr bool kAlias = KM > 2;   // (KM <= 2: a separate region)
  __shared__ double2 lds[64 * 65 + (kAlias ? 0 : 2 * KM * 64)];
  double2(*colc)[65] = reinterpret_cast<double2(*)[65]>(lds);
  double2* cpv = kAlias ? lds : lds + 64 * 65;   // [KM][64]: v_j of the tile's columns
  double2* cpw = cpv + KM * 64;                  // [KM][64]: w_j
  const int gr = R * kEigTB + lane;
  const bool rok = gr >= i + 1 && gr < n;
  if (tid < 64) {
    const int gc = C * kEigTB + tid;
    cv[tid] = gc >= i + 1 && gc < n ? v[gc] : cz();
  }
  if (wp) {
    for (int q = w; q < np; q += 4) {   // wave w stages pairs w, w+4
      const int sl = (f + q) % kEigRing, gc = C * kEigTB + lane;
      const bool ok = gc >= i + 1 && gc < n;
      cpv[q * 64 + lane] = ok ? vv[(int64_t)sl * n + gc] : cz();
      cpw[q * 64 + lane] = ok ? ww[(int64_t)sl * n + gc] : cz();
    }
  }
  const double2 vr = rok ? v[gr] : cz();
  // the pending pairs at this lane's row: the write pass's update, or a read
  // pass's dots (diagonal tiles), loaded with the tile
  const bool rowpairs = wp || R == C;
  double2 rv[KM], rw[KM];
#pragma unroll
  for (int q = 0; q < KM; ++q) {
    const int sl = (f + q) % kEigRing;
    const bool ok = rowpairs && rok && q < np;
    rv[q] = ok ? vv[(int64_t)sl * n + gr] : cz();
    rw[q] = ok ? ww[(int64_t)sl * n + gr] : cz();
  }
  __syncthreads();
  constexpr int NCW = kEigTB / 4;   // columns per wave
  double2 a[NCW];
  unsigned act = 0;
#pragma unroll
  for (int u = 0; u < NCW; ++u) {
    const int gc = C * kEigTB + w + 4 * u;
    const bool ok = rok && gc >= i + 1 && gr >= gc;
    act |= (unsigned)ok << u;
    a[u] = ok ? A[gr + (int64_t)gc * n] : cz();
  }
  if (wp && np > 0) {
#pragma unroll
    for (int u = 0; u < NCW; ++u) {
      const int cc = w + 4 * u, gc = C * kEigTB + cc;
      if ((act >> u) & 1) {
        double2 x = a[u];
#pragma unroll
        for (int q = 0; q < KM; ++q)
          if (q < np) x = csub(csub(x, cmulc(rv[q], cpw[q * 64 + cc])), cmulc(rw[q], cpv[q * 64 + cc]));
        a[u] = x;
        A[gr + (int64_t)gc * n] = x;
      }
    }
    if (kAlias) __syncthreads();   // the pair values are dead: the region becomes colc
  }
  double2 pr = cz();
#pragma unroll
  for (int u = 0; u < NCW; ++u) {
    const int cc = w + 4 * u, gc = C * kEigTB + cc;
    double2 t = cz();
    if ((act >> u) & 1) {
      pr = cadd(pr, cmul(a[u], cv[cc]));
      if (gr > gc) t = make_double2(a[u].x * vr.x + a[u].y * vr.y, a[u].x * vr.y - a[u].y * vr.x);   // conj(a) v_r
    }
    colc[cc][lane] = t;
  }
  rowp[w][lane] = pr;
  if (!wp && np > 0 && R == C && w == 0) {
    // dots of the pending pairs with v_i over this tile's rows
#pragma unroll
    for (int q = 0; q < KM; ++q) {
      if (q >= np) break;
      double2 dw = make_double2(rw[q].x * vr.x + rw[q].y * vr.y, rw[q].x * vr.y - rw[q].y * vr.x);
      double2 dv = make_double2(rv[q].x * vr.x + rv[q].y * vr.y, rv[q].x * vr.y - rv[q].y * vr.x);
      dw.x = wave_sum(dw.x);
      dw.y = wave_sum(dw.y);
      dv.x = wave_sum(dv.x);
      dv.y = wave_sum(dv.y);
      if (lane == 0) {
        dpart[((int64_t)k * T + R) * 2 * KD + 2 * q] = dw;
        dpart[((int64_t)k * T + R) * 2 * KD + 2 * q + 1] = dv;
      }
    }
  }
  __syncthreads();
  {
    const int cc = tid >> 2, q = tid & 3;
    double2 s = cz();
#pragma unroll
    for (int r = 0; r < 16; ++r) s = cadd(s, colc[cc][q * 16 + r]);
    s.x += __shfl_xor(s.x, 1, 64);
    s.y += __shfl_xor(s.y, 1, 64);
    s.x += __shfl_xor(s.x, 2, 64);
    s.y += __shfl_xor(s.y, 2, 64);
    if (q == 0) csum[cc] = s;
  }
  __syncthreads();
  if (tid < 64) {
    const double2 rs = cadd(cadd(rowp[0][tid], rowp[1][tid]), cadd(rowp[2][tid], rowp[3][tid]));
    const double2 cs = csum[tid];
    const int r = R * kEigTB + tid, c = C * kEigTB + tid;
    if (R == C) {
      if (r < n) part[(int64_t)R * n + r] = cadd(rs, cs);
    } else {
      if (r < n) part[(int64_t)C * n + r] = rs;
      if (c < n) part[(int64_t)R * n + c] = cs;
    }
  }
}

// K = 1 pass in one sweep over the tile (round-3 form: the pending pair i-1
// applied, written back, and the hemv accumulated per column in one loop;
// tile loads after the staging barrier)
__global__ __launch_bounds__(256) void k_eig_pass1(double2* __restrict__ A, int n, int i, int64_t sA,
                                                   double2* __restrict__ part, int64_t sP,
                                                   const double2* __restrict__ vv, const double2* __restrict__ ww,
                                                   int t0) {
  const int k = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  A += k * sA;
  part += k * sP;
  vv += (int64_t)k * kEigRing * n;
  ww += (int64_t)k * kEigRing * n;
  const double2* v = vv + (int64_t)(i % kEigRing) * n;
  const double2* va = vv + (int64_t)((i + kEigRing - 1) % kEigRing) * n;   // pair i-1
  const double2* wa = ww + (int64_t)((i + kEigRing - 1) % kEigRing) * n;
  const int np = i == 0 ? 0 : 1;
  int R, C;
  tri_decode(blockIdx.x, R, C);
  R += t0;
  C += t0;
  __shared__ double2 cv[64], cva[64], cwa[64], csum[64];
  __shared__ double2 colc[64][65];
  __shared__ double2 rowp[4][64];
  if (tid < 64) {
    const int gc = C * kEigTB + tid;
    const bool ok = gc >= i + 1 && gc < n;
    cv[tid] = ok ? v[gc] : cz();
    cva[tid] = ok && np ? va[gc] : cz();
    cwa[tid] = ok && np ? wa[gc] : cz();
  }
  const int gr = R * kEigTB + lane;
  const bool rok = gr >= i + 1 && gr < n;
  const double2 vr = rok ? v[gr] : cz();
  const double2 var = rok && np ? va[gr] : cz();
  const double2 war = rok && np ? wa[gr] : cz();
  __syncthreads();
  double2 pr = cz();
  constexpr int NCW = kEigTB / 4;   // columns per wave
  double2 a[NCW];
  unsigned act = 0;
#pragma unroll
  for (int u = 0; u < NCW; ++u) {
    const int gc = C * kEigTB + w + 4 * u;
    const bool ok = rok && gc >= i + 1 && gr >= gc;
    act |= (unsigned)ok << u;
    a[u] = ok ? A[gr + (int64_t)gc * n] : cz();
  }
#pragma unroll
  for (int u = 0; u < NCW; ++u) {
    const int cc = w + 4 * u, gc = C * kEigTB + cc;
    double2 t = cz();
    if ((act >> u) & 1) {
      if (np) {
        a[u] = csub(csub(a[u], cmulc(var, cwa[cc])), cmulc(war, cva[cc]));
        A[gr + (int64_t)gc * n] = a[u];
      }
      pr = cadd(pr, cmul(a[u], cv[cc]));
      if (gr > gc) t = make_double2(a[u].x * vr.x + a[u].y * vr.y, a[u].x * vr.y - a[u].y * vr.x);   // conj(a) v_r
    }
    colc[cc][lane] = t;
  }
  rowp[w][lane] = pr;
  __syncthreads();
  {
    const int cc = tid >> 2, q = tid & 3;
    double2 s = cz();
#pragma unroll
    for (int r = 0; r < 16; ++r) s = cadd(s, colc[cc][q * 16 + r]);
    s.x += __shfl_xor(s.x, 1, 64);
    s.y += __shfl_xor(s.y, 1, 64);
    s.x += __shfl_xor(s.x, 2, 64);
    s.y += __shfl_xor(s.y, 2, 64);
    if (q == 0) csum[cc] = s;
  }
  __syncthreads();
  if (tid < 64) {
    const double2 rs = cadd(cadd(rowp[0][tid], rowp[1][tid]), cadd(rowp[2][tid], rowp[3][tid]));
    const double2 cs = csum[tid];
    const int r = R * kEigTB + tid, c = C * kEigTB + tid;
    if (R == C) {
      if (r < n) part[(int64_t)R * n + r] = cadd(rs, cs);
    } else {
      if (r < n) part[(int64_t)C * n + r] = rs;
      if (c < n) part[(int64_t)R * n + c] = cs;
    }
  }
}

// One matrix (K = 1), 1 <= i <= n-2: step i folded into pass i.  Every
// workgroup forms the scalars of column i itself from k_eig_reduce's
// outputs — g (the reduce workgroups' partials, fixed order), w_{i-1}[i] and
// bu = conj(w_{i-1}[i]) + al of the updated column c = c0 - tau p - bu v_{i-1},
// the norm of c over the rows >= i+2 (a sweep over p, c0, v_{i-1} in a fixed
// order: the same bits in every workgroup), the reflector (zlarfg) — and
// then v_i and w_{i-1} on its tile's rows and columns.  The diagonal tiles
// write v_i and column i of A (tile t0 also the rows above and d, e, tau).
// Saves the single-workgroup step launch of every column.
__global__ __launch_bounds__(256) void k_eig_pass1f(double2* __restrict__ A, int n, int i, int64_t sA,
                                                    double2* __restrict__ part, int64_t sP,
                                                    double2* __restrict__ vv, const double2* __restrict__ pfin,
                                                    const double2* __restrict__ colfin,
                                                    const double2* __restrict__ gpart, int ngp,
                                                    double* __restrict__ d, double* __restrict__ e,
                                                    double2* __restrict__ tau, int t0) {
  const int k = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  A += k * sA;
  part += k * sP;
  vv += (int64_t)k * kEigRing * n;
  pfin += (int64_t)k * n;
  colfin += (int64_t)k * n;
  gpart += (int64_t)k * kEigGP * 3;
  const double2* vp = vv + (int64_t)((i + kEigRing - 1) % kEigRing) * n;   // v_{i-1}
  double2* vcur = vv + (int64_t)(i % kEigRing) * n;
  int R, C;
  tri_decode(blockIdx.x, R, C);
  R += t0;
  C += t0;
  const int gr = R * kEigTB + lane;
  const bool rok = gr >= i + 1 && gr < n;
  // the tile, in flight while the scalars are formed
  constexpr int NCW = kEigTB / 4;   // columns per wave
  double2 a[NCW];
  unsigned act = 0;
#pragma unroll
  for (int u = 0; u < NCW; ++u) {
    const int gc = C * kEigTB + w + 4 * u;
    const bool ok = rok && gc >= i + 1 && gr >= gc;
    act |= (unsigned)ok << u;
    a[u] = ok ? A[gr + (int64_t)gc * n] : cz();
  }
  // this workgroup's column / row inputs, loaded before the scalars they
  // combine with (independent loads: one round trip)
  const int gcs = C * kEigTB + (tid & 63);
  const bool cok = tid < 64 && gcs >= i + 1 && gcs < n;
  double2 pc = cz(), cc0 = cz(), vc = cz(), pr0 = cz(), cr0 = cz(), var = cz();
  if (cok) {
    pc = pfin[gcs];
    cc0 = colfin[gcs];
    vc = vp[gcs];
  }
  if (rok) {
    pr0 = pfin[gr];
    cr0 = colfin[gr];
    var = vp[gr];
  }
  // scalars of column i (zhetd2 'L': x = tau p, w = x - 1/2 tau (x^H v) v)
  __shared__ double sx[4];
  const ColScal cs = col_scalars(n, i, pfin, colfin, vp, gpart, ngp, tau[(int64_t)k * n + i - 1], sx);
  const double2 tp = cs.tp, al = cs.al;
  __shared__ double2 cv[64], cva[64], cwa[64], csum[64];
  __shared__ double2 colc[64][65];
  __shared__ double2 rowp[4][64];
  if (tid < 64) {
    cv[tid] = cok ? col_vnew(cs, gcs, i, pc, cc0, vc) : cz();
    cva[tid] = vc;
    cwa[tid] = cok ? cadd(cmul(tp, pc), cmul(al, vc)) : cz();
  }
  double2 vr = cz(), war = cz();
  if (rok) {
    vr = col_vnew(cs, gr, i, pr0, cr0, var);
    war = cadd(cmul(tp, pr0), cmul(al, var));
  }
  if (R == C) {   // column i of A and v_i on this tile's rows
    if (rok) {
      vcur[gr] = vr;
      A[gr + (int64_t)i * n] = vr;
    } else if (gr < n && gr <= i) {
      A[gr + (int64_t)i * n] = cz();
    }
    if (R == t0) {
      for (int r = tid; r < t0 * kEigTB && r <= i; r += 256) A[r + (int64_t)i * n] = cz();
      if (tid == 0) {
        d[(int64_t)k * n + i] = cs.di;
        e[(int64_t)k * n + i] = cs.beta;
        tau[(int64_t)k * n + i] = cs.t;
      }
    }
  }
  __syncthreads();
  double2 pr = cz();
#pragma unroll
  for (int u = 0; u < NCW; ++u) {
    const int cc = w + 4 * u, gc = C * kEigTB + cc;
    double2 tt = cz();
    if ((act >> u) & 1) {
      a[u] = csub(csub(a[u], cmulc(var, cwa[cc])), cmulc(war, cva[cc]));
      A[gr + (int64_t)gc * n] = a[u];
      pr = cadd(pr, cmul(a[u], cv[cc]));
      if (gr > gc) tt = make_double2(a[u].x * vr.x + a[u].y * vr.y, a[u].x * vr.y - a[u].y * vr.x);   // conj(a) v_r
    }
    colc[cc][lane] = tt;
  }
  rowp[w][lane] = pr;
  __syncthreads();
  {
    const int cc = tid >> 2, q = tid & 3;
    double2 s = cz();
#pragma unroll
    for (int r = 0; r < 16; ++r) s = cadd(s, colc[cc][q * 16 + r]);
    s.x += __shfl_xor(s.x, 1, 64);
    s.y += __shfl_xor(s.y, 1, 64);
    s.x += __shfl_xor(s.x, 2, 64);
    s.y += __shfl_xor(s.y, 2, 64);
    if (q == 0) csum[cc] = s;
  }
  __syncthreads();
  if (tid < 64) {
    const double2 rs = cadd(cadd(rowp[0][tid], rowp[1][tid]), cadd(rowp[2][tid], rowp[3][tid]));
    const double2 cs = csum[tid];
    const int r = R * kEigTB + tid, c = C * kEigTB + tid;
    if (R == C) {
      if (r < n) part[(int64_t)R * n + r] = cadd(rs, cs);
    } else {
      if (r < n) part[(int64_t)C * n + r] = rs;
      if (c < n) part[(int64_t)R * n + c] = cs;
    }
  }
}

// Gershgorin interval of T (lo, hi), ||T|| bound and max e^2 over the workgroup
__device__ void gersh(const double* __restrict__ d, const double* __restrict__ e, int n, double* sh, double& lo,
                      double& hi, double& emax) {
  double a = DBL_MAX, b = -DBL_MAX, c = 0.0;
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    const double er = r < n - 1 ? e[r] : 0.0, el = r > 0 ? e[r - 1] : 0.0;
    const double rad = fabs(er) + fabs(el);
    a = fmin(a, d[r] - rad);
    b = fmax(b, d[r] + rad);
    c = fmax(c, er * er);
  }
  for (int off = 32; off > 0; off >>= 1) {
    a = fmin(a, __shfl_xor(a, off, 64));
    b = fmax(b, __shfl_xor(b, off, 64));
    c = fmax(c, __shfl_xor(c, off, 64));
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sh[3 * w] = a;
    sh[3 * w + 1] = b;
    sh[3 * w + 2] = c;
  }
  __syncthreads();
  lo = DBL_MAX;
  hi = -DBL_MAX;
  emax = 0.0;
  for (int k = 0; k < nw; ++k) {
    lo = fmin(lo, sh[3 * k]);
    hi = fmax(hi, sh[3 * k + 1]);
    emax = fmax(emax, sh[3 * k + 2]);
  }
}

// G lanes per eigenvalue index j (G | 64, 64 / G eigenvalues per wave): a
// G-section of [lo, hi] per round (lane l of the group counts at
// lo + (l+1)(hi-lo)/(G+1); the counts are monotone in l, so the group's bits
// of a ballot find the sub-interval holding eigenvalue j), rounds to the last
// bit.  G = 64 (~9 rounds) when few eigenvalues are asked for (the rounds are
// the latency); batches use smaller groups, the same bits from fewer Sturm
// counts (G x rounds per eigenvalue: 64 x 9 = 576, 4 x 23 = 92).  Sturm count:
// the dstebz recurrence with d and e^2 broadcast from LDS and 1/q by
// v_rcp_f64 + one Newton step.
constexpr int kBisW = 8;   // waves per workgroup
__global__ __launch_bounds__(64 * kBisW) void k_eig_bisect(const double* __restrict__ d,
                                                           const double* __restrict__ e, int n, int lgG,
                                                           double* __restrict__ E, double* __restrict__ tnorm) {
  extern __shared__ double lds[];   // d[0, n), e^2[n, 2n)
  const int k = blockIdx.y, lane = threadIdx.x & 63;
  d += (int64_t)k * n;
  e += (int64_t)k * n;
  E += (int64_t)k * n;
  __shared__ double sh[3 * kBisW];
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    lds[r] = d[r];
    const double er = r < n - 1 ? e[r] : 0.0;
    lds[n + r] = er * er;
  }
  double gl, gu, emax;
  gersh(d, e, n, sh, gl, gu, emax);   // its barriers publish the LDS copies
  const double tn = fmax(fabs(gl), fabs(gu));
  if (blockIdx.x == 0 && threadIdx.x == 0) tnorm[k] = tn;
  gl -= 2.0 * DBL_EPSILON * tn * n + 1e-300;
  gu += 2.0 * DBL_EPSILON * tn * n + 1e-300;
  const double pivmin = DBL_MIN * fmax(1.0, emax);
  const int G = 1 << lgG, g0 = lane & ~(G - 1), gi = lane & (G - 1);
  const int j = ((blockIdx.x * kBisW + (threadIdx.x >> 6)) << (6 - lgG)) + (lane >> lgG);
  if (((blockIdx.x * kBisW + (threadIdx.x >> 6)) << (6 - lgG)) >= n) return;   // whole wave idle
  const unsigned long long gmask = G == 64 ? ~0ull : ((1ull << G) - 1);
  const double* ld = lds;
  const double* le2 = lds + n;
  const double step = 1.0 / (G + 1);
  double lo = gl, hi = gu;
  bool done = j >= n;
  for (int it = 0; it < 256; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (mid <= lo || mid >= hi) done = true;
    if (__ballot(!done) == 0) break;
    const double x = fmin(lo + (gi + 1) * ((hi - lo) * step), hi);
    double q = ld[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    int c = q < 0.0;
#pragma unroll 8
    for (int r = 1; r < n; ++r) {
      // 1/q: v_rcp_f64 + one Newton step (<= 11 ulp; a relative error of 1/q is a
      // relative perturbation of e^2_{r-1}, far below the count's resolution)
      const double r0 = __builtin_amdgcn_rcp(q);
      const double rq = fma(r0, fma(-q, r0, 1.0), r0);
      q = (ld[r] - x) - le2[r - 1] * rq;
      if (fabs(q) < pivmin) q = -pivmin;
      c += q < 0.0;
    }
    // first lane of the group whose count exceeds j: eigenvalue j lies in (x_{f-1}, x_f]
    const unsigned long long above = (__ballot(c > j) >> g0) & gmask;
    const int f = above ? __builtin_ctzll(above) : G;
    const double xf = __shfl(x, g0 + (f < G ? f : G - 1), 64), xp = __shfl(x, g0 + (f > 0 ? f - 1 : 0), 64);
    const double nlo = f > 0 ? xp : lo, nhi = f < G ? xf : hi;
    if (nlo == lo && nhi == hi) done = true;
    if (!done) {
      lo = nlo;
      hi = nhi;
    }
  }
  if (gi == 0 && j < n) E[j] = 0.5 * (lo + hi);
}

// start vector entry r of eigenvalue m: splitmix64 of (m, r) in [-1/2, 1/2)
// (independent-looking starts: the vectors of a degenerate level are the
// starts' projections onto its eigenspace, so correlated starts would leave
// them nearly dependent)
__device__ __forceinline__ double start_entry(int m, int r) {
  unsigned long long z = ((unsigned long long)(unsigned)m << 32 | (unsigned)r) + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * 0x1.0p-53 - 0.5;
}

__device__ __forceinline__ double clamp_small(double x, double small) {
  return fabs(x) < small ? (x != 0.0 ? copysign(small, x) : small) : x;
}

// inverse iteration for eigenvalue m (vector: column m of Zt, Zt[r n + m];
// LU scratch: columns m of U0/U1/U2, U0 holding the reciprocal pivots): two
// solves with T - lam I from a fixed pseudo-random start (lam is accurate to
// a few ulps of ||T||, so one solve already leaves neighbours at ~ulp / gap),
// normalised
__device__ void invit_one(const double* d, const double* e, int n, double lam, int m,
                          double small, double* __restrict__ Zt, double* __restrict__ U0, double* __restrict__ U1,
                          double* __restrict__ U2) {
  double* __restrict__ x = Zt + m;
  double* __restrict__ u0 = U0 + m;
  double* __restrict__ u1 = U1 + m;
  double* __restrict__ u2 = U2 + m;
  const int64_t ld = n;
  constexpr int PB = 16;   // rows per prefetch block
  double scale = 1.0;
  for (int it = 0; it < 2; ++it) {
    const bool first = it == 0;
    // forward: factor T - lam I (row interchanges) and eliminate y in one sweep
    double cu0 = d[0] - lam, cu1 = n > 1 ? e[0] : 0.0;
    double yk = first ? start_entry(m, 0) : x[0] * scale;
    for (int r0 = 0; r0 < n - 1; r0 += PB) {
      double yb[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int r = r0 + u;
        yb[u] = r < n - 1 ? (first ? start_entry(m, r + 1) : x[(r + 1) * ld] * scale) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int r = r0 + u;
        if (r >= n - 1) break;
        const double b = e[r], nd = d[r + 1] - lam, ne = r + 1 < n - 1 ? e[r + 1] : 0.0;
        const double yk1 = yb[u];
        // branch-free (lanes hold different shifts): keep = no row interchange
        const bool keep = fabs(cu0) >= fabs(b);
        const double c0 = (keep && cu0 == 0.0) ? small : cu0;
        const double piv = keep ? c0 : b;
        const double rp = rcp_nr(piv);
        const double mu = (keep ? b : c0) * rp;
        u0[r * ld] = rcp_nr(clamp_small(piv, small));
        u1[r * ld] = keep ? cu1 : nd;
        u2[r * ld] = keep ? 0.0 : ne;
        x[r * ld] = keep ? yk : yk1;
        const double ncu0 = keep ? nd - mu * cu1 : cu1 - mu * nd;
        const double ncu1 = keep ? ne : -mu * ne;
        const double nyk = keep ? yk1 - mu * yk : yk - mu * yk1;
        cu0 = ncu0;
        cu1 = ncu1;
        yk = nyk;
      }
    }
    u0[(n - 1) * ld] = 1.0 / clamp_small(cu0, small);
    u1[(n - 1) * ld] = 0.0;
    u2[(n - 1) * ld] = 0.0;
    x[(n - 1) * ld] = yk;
    // backward substitution, PB rows loaded ahead of their use
    double x1 = 0.0, x2 = 0.0, nrm = 0.0;
    for (int rt = n - 1; rt >= 0; rt -= PB) {
      double yb[PB], a0[PB], a1[PB], a2[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int r = rt - u;
        const bool ok = r >= 0;
        yb[u] = ok ? x[r * ld] : 0.0;
        a0[u] = ok ? u0[r * ld] : 0.0;
        a1[u] = ok ? u1[r * ld] : 0.0;
        a2[u] = ok ? u2[r * ld] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int r = rt - u;
        if (r < 0) break;
        const double xr = (yb[u] - a1[u] * x1 - a2[u] * x2) * a0[u];
        x[r * ld] = xr;
        x2 = x1;
        x1 = xr;
        nrm += xr * xr;
      }
    }
    scale = 1.0 / sqrt(nrm);
  }
  for (int r0 = 0; r0 < n; r0 += 16) {
    double t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) t[u] = r0 + u < n ? x[(r0 + u) * ld] : 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (r0 + u < n) x[(r0 + u) * ld] = t[u] * scale;
  }
}

__global__ __launch_bounds__(64) void k_eig_invit(const double* __restrict__ d, const double* __restrict__ e,
                                                  int n, const double* __restrict__ E,
                                                  const double* __restrict__ tnorm, double* __restrict__ Zt,
                                                  double* __restrict__ U0, double* __restrict__ U1,
                                                  double* __restrict__ U2, int64_t sZ, int j0,
                                                  const int* __restrict__ c0) {
  extern __shared__ double lds[];   // d[0, n), e[n, 2n)
  const int k = blockIdx.y;
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    lds[r] = d[(int64_t)k * n + r];
    lds[n + r] = r < n - 1 ? e[(int64_t)k * n + r] : 0.0;
  }
  __syncthreads();
  const int j = j0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  if (c0 && j < c0[k]) {   // a particle-hole partner column: zero (the Löwdin step reads it)
    double* z = Zt + k * sZ + j;
    for (int r = 0; r < n; ++r) z[(int64_t)r * n] = 0.0;
    return;
  }
  const double tn = tnorm[k];
  const double small = tn > 0.0 ? DBL_EPSILON * tn : DBL_EPSILON;
  invit_one(lds, lds + n, n, E[(int64_t)k * n + j], j, small, Zt + k * sZ, U0 + k * sZ, U1 + k * sZ,
            U2 + k * sZ);
}

// Clusters (runs of eigenvalues with consecutive gaps <= ctol ||T||, up to
// kEigMaxCluster long) get their inverse-iteration vectors orthonormalised:
// two rounds of Cholesky QR on the cluster's columns of Zt (G = Z^T Z = L L^T,
// Z <- Z L^-T; the rows of a cluster are contiguous in Zt).  Vectors of
// separated eigenvalues are orthogonal to ~2 eps ||T|| / gap already; inside a
// cluster the rotation is O(that) for distinct eigenvalues, and an orthonormal
// basis of the eigenspace for exactly degenerate ones.  One workgroup per
// candidate first index; clusters longer than maxc are left to the host-driven
// Cholesky QR (long_clusters in dwhmc_api.cpp); *bad = 1 when G is not
// positive definite (the caller then re-solves with rocSOLVER's zheev).
__global__ __launch_bounds__(256) void k_eig_orth(const double* __restrict__ E, const double* __restrict__ tnorm,
                                                  int n, double* __restrict__ Zt, int64_t sZ, double ctol,
                                                  int* __restrict__ bad, int maxc, int j0,
                                                  const int* __restrict__ c0) {
  constexpr int MC = kEigMaxCluster;
  const int k = blockIdx.y, j = j0 + blockIdx.x, tid = threadIdx.x;
  if (c0 && j < c0[k]) return;
  E += (int64_t)k * n;
  Zt += k * sZ;
  const double tol = ctol * tnorm[k];
  if (j > 0 && E[j] - E[j - 1] <= tol) return;
  int end = j + 1;
  while (end < n && end - j <= MC && E[end] - E[end - 1] <= tol) ++end;
  const int kc = end - j;
  // a cluster longer than maxc is orthonormalised by the host-driven Cholesky
  // QR over several workgroups (own_heev_enqueue, dwhmc_api.cpp)
  if (kc == 1 || kc > maxc) return;
  constexpr int RC = 64;   // rows per LDS chunk (Gram sums, substitution)
  __shared__ double G[MC][MC + 1];
  __shared__ double Zs[RC][MC + 1];
  __shared__ int fail;
  for (int round = 0; round < 2; ++round) {
    // G = Z_c^T Z_c (lower triangle): rows staged RC at a time in LDS, each
    // thread accumulating its pairs over the rows in order
    constexpr int NPT = (MC * (MC + 1) / 2 + 255) / 256;
    const int npair = kc * (kc + 1) / 2;
    double acc[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) acc[u] = 0.0;
    for (int r0 = 0; r0 < n; r0 += RC) {
      for (int q = tid; q < RC * kc; q += 256) {
        const int rr = q / kc, c = q % kc, r = r0 + rr;
        Zs[rr][c] = r < n ? Zt[(int64_t)r * n + j + c] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int pq = tid + 256 * u;
        if (pq < npair) {
          int p = (int)((sqrt(8.0 * pq + 1.0) - 1.0) * 0.5);
          while ((p + 1) * (p + 2) / 2 <= pq) ++p;
          while (p * (p + 1) / 2 > pq) --p;
          const int q = pq - p * (p + 1) / 2;
          double a = acc[u];
          for (int rr = 0; rr < RC; ++rr) a += Zs[rr][p] * Zs[rr][q];
          acc[u] = a;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int pq = tid + 256 * u;
      if (pq < npair) {
        int p = (int)((sqrt(8.0 * pq + 1.0) - 1.0) * 0.5);
        while ((p + 1) * (p + 2) / 2 <= pq) ++p;
        while (p * (p + 1) / 2 > pq) --p;
        G[p][pq - p * (p + 1) / 2] = acc[u];
      }
    }
    if (tid == 0) fail = 0;
    __syncthreads();
    // Cholesky, right-looking, in place (lower)
    for (int c = 0; c < kc; ++c) {
      if (tid == 0) {
        // the columns are normalised: a pivot this small means cond(Z) > ~1e7,
        // beyond what two rounds of Cholesky QR repair
        const double g = G[c][c];
        if (!(g > 1e-14)) fail = 1;
        G[c][c] = sqrt(fmax(g, DBL_MIN));
      }
      __syncthreads();
      for (int r = c + 1 + tid; r < kc; r += 256) G[r][c] /= G[c][c];
      __syncthreads();
      for (int pq = tid; pq < kc * kc; pq += 256) {
        const int p = pq / kc, q = pq % kc;
        if (q > c && p >= q) G[p][q] -= G[p][c] * G[q][c];
      }
      __syncthreads();
    }
    if (fail) {
      if (tid == 0) *bad = 1;
      return;
    }
    // each row z (1 x kc) <- z L^-T: forward substitution L x = z^T, on RC-row
    // chunks staged in LDS (one row per thread)
    for (int r0 = 0; r0 < n; r0 += RC) {
      for (int q = tid; q < RC * kc; q += 256) {
        const int rr = q / kc, c = q % kc, r = r0 + rr;
        Zs[rr][c] = r < n ? Zt[(int64_t)r * n + j + c] : 0.0;
      }
      __syncthreads();
      if (tid < RC) {
        for (int p = 0; p < kc; ++p) {
          double v = Zs[tid][p];
          for (int q = 0; q < p; ++q) v -= G[p][q] * Zs[tid][q];
          Zs[tid][p] = v / G[p][p];
        }
      }
      __syncthreads();
      for (int q = tid; q < RC * kc; q += 256) {
        const int rr = q / kc, c = q % kc, r = r0 + rr;
        if (r < n) Zt[(int64_t)r * n + j + c] = Zs[rr][c];
      }
      __syncthreads();
    }
  }
}

// U[r + c n] = (Zt[r n + c], 0), through a 64 x 64 LDS tile
__global__ __launch_bounds__(256) void k_eig_zt_to_u(const double* __restrict__ Zt, double2* __restrict__ U, int n,
                                                     int64_t sZ, int64_t sA, int j0) {
  const int k = blockIdx.z;
  Zt += k * sZ;
  U += k * sA;
  __shared__ double t[64][65];
  const int r0 = blockIdx.y * 64, c0 = j0 + blockIdx.x * 64;
  for (int q = threadIdx.x; q < 64 * 64; q += 256) {
    const int rr = q >> 6, cc = q & 63;   // read row r0+rr of Zt: columns c0+cc contiguous
    const int r = r0 + rr, c = c0 + cc;
    t[rr][cc] = (r < n && c < n) ? Zt[(int64_t)r * n + c] : 0.0;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 64 * 64; q += 256) {
    const int cc = q >> 6, rr = q & 63;   // write column c0+cc of U: rows r0+rr contiguous
    const int r = r0 + rr, c = c0 + cc;
    if (r < n && c < n) U[r + (int64_t)c * n] = make_double2(t[rr][cc], 0.0);
  }
}

// U[:, j] = Θ U[:, n-1-j] for j < c0[k]: Θ (u; v) = (-conj v; conj u), one
// thread per row
__global__ __launch_bounds__(256) void k_eig_theta(double2* __restrict__ U, int n, int64_t sA,
                                                   const int* __restrict__ c0) {
  const int k = blockIdx.z, j = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
  if (j >= c0[k] || r >= n) return;
  U += k * sA;
  const int N = n / 2;
  const double2* src = U + (int64_t)(n - 1 - j) * n;
  const double2 v = r < N ? src[r + N] : src[r - N];
  U[r + (int64_t)j * n] = r < N ? make_double2(-v.x, v.y) : make_double2(v.x, -v.y);
}

// compact-WY T of reflector block b (columns j0 .. j0+kb-1 of V, rows j0+1 ..):
// G = V^H V, T[j][j] = tau_j, T[0:j, j] = -tau_j T[0:j, 0:j] G[0:j, j].
// k_eig_tgram: partial G of row slice g (kEigGS slices per block, so the
// blocks' Gram sums fill the chip); k_eig_tfac: the slices summed in order,
// then the recurrence.
__global__ __launch_bounds__(256) void k_eig_tgram(const double2* __restrict__ V, int n, int64_t sA,
                                                   double2* __restrict__ Gp) {
  constexpr int NB = kEigNB;
  const int blk = blockIdx.x, g = blockIdx.y, k = blockIdx.z, tid = threadIdx.x;
  const int nblk = gridDim.x;
  const int j0 = blk * NB, kb = min(NB, n - 1 - j0), ms = n - 1 - j0;
  const int rc = ((ms + kEigGS - 1) / kEigGS + NB - 1) / NB * NB;
  const int rb = j0 + 1 + g * rc, re = min(n, rb + rc);
  V += k * sA;
  Gp += (((int64_t)k * nblk + blk) * kEigGS + g) * NB * NB;
  __shared__ double2 S[NB][NB + 1];
  double2 acc[NB * NB / 256];
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) acc[u] = cz();
  for (int r0 = rb; r0 < re; r0 += NB) {
    for (int q = tid; q < NB * NB; q += 256) {
      const int cc = q / NB, rr = q % NB, r = r0 + rr;
      S[rr][cc] = (r < re && cc < kb) ? V[r + (int64_t)(j0 + cc) * n] : cz();
    }
    __syncthreads();
    // thread: column q = tid % NB, rows p = tid / NB + 4 u of G
#pragma unroll 2
    for (int rr = 0; rr < NB; ++rr) {
      const double2 y = S[rr][tid % NB];
#pragma unroll
      for (int u = 0; u < NB * NB / 256; ++u) {
        const double2 x = S[rr][(tid + 256 * u) / NB];   // conj(x) y
        acc[u].x += x.x * y.x + x.y * y.y;
        acc[u].y += x.x * y.y - x.y * y.x;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) Gp[tid + 256 * u] = acc[u];
}

__global__ __launch_bounds__(256) void k_eig_tfac(const double2* __restrict__ Gp, int n,
                                                  const double2* __restrict__ tau, double2* __restrict__ Tb,
                                                  int64_t sT) {
  constexpr int NB = kEigNB;
  const int blk = blockIdx.x, k = blockIdx.y, tid = threadIdx.x, nblk = gridDim.x;
  const int j0 = blk * NB, kb = min(NB, n - 1 - j0);
  tau += (int64_t)k * n;
  Tb += k * sT + (int64_t)blk * NB * NB;
  Gp += ((int64_t)k * nblk + blk) * kEigGS * NB * NB;
  __shared__ double2 G[NB][NB + 1];
  __shared__ double2 S[NB][NB + 1];   // T
  for (int pq = tid; pq < NB * NB; pq += 256) {
    double2 a = cz();
    for (int g = 0; g < kEigGS; ++g) a = cadd(a, Gp[(int64_t)g * NB * NB + pq]);
    G[pq / NB][pq % NB] = a;
  }
  for (int q = tid; q < NB * NB; q += 256) S[q / NB][q % NB] = cz();
  __syncthreads();
  for (int j = 0; j < kb; ++j) {
    const double2 tj = tau[j0 + j];
    double2 s = cz();
    if (tid < j) {
      for (int q = tid; q < j; ++q) s = cadd(s, cmul(S[tid][q], G[q][j]));
    }
    __syncthreads();
    if (tid < j) S[tid][j] = cmul(make_double2(-tj.x, -tj.y), s);
    if (tid == j) S[j][j] = tj;
    __syncthreads();
  }
  for (int q = tid; q < NB * NB; q += 256) {
    const int p = q % NB, c = q / NB;
    Tb[p + (int64_t)c * NB] = S[p][c];
  }
}

// Vt: the reflector blocks conjugate-transposed, block b (columns b NB ..
// b NB + kb - 1 of V, rows from b NB + 1) at Vt + b NB n as kb x (n - b NB - 1),
// leading dimension ldv = min(NB, n - 1) (fits the n x n slot), so the
// back-transform's W = V^H U is an 'N','N' product (1.7x faster than 'C','N'
// on V in place: profiles/r05_exp_backtransform_vt.txt).  Block (x, b, k):
// 32 rows of block b.
__global__ __launch_bounds__(256) void k_eig_vt(const double2* __restrict__ A, int n, int64_t sA,
                                                double2* __restrict__ Vt) {
  __shared__ double2 tile[kEigNB][33];
  const int b = blockIdx.y, k = blockIdx.z, r0 = b * kEigNB, rr0 = blockIdx.x * 32;
  const int ms = n - r0 - 1, kb = min(kEigNB, n - 1 - r0), ldv = min(kEigNB, n - 1);
  if (rr0 >= ms) return;
  A += k * sA;
  Vt += k * sA + (int64_t)r0 * n;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int idx = threadIdx.x + 256 * q, j = idx >> 5, r = idx & 31;
    tile[j][r] = (j < kb && rr0 + r < ms) ? A[(r0 + 1 + rr0 + r) + (int64_t)(r0 + j) * n] : cz();
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int idx = threadIdx.x + 256 * q, r = idx >> 6, j = idx & 63;
    if (rr0 + r < ms) {
      const double2 v = tile[j][r];
      if (j < ldv) Vt[j + (int64_t)(rr0 + r) * ldv] = make_double2(v.x, -v.y);
    }
  }
}

// W2 = T (sum over the S K-chunks of W): T kb x kb (ld kEigNB), chunk s of W
// at rows s kb (ld ldw).  One workgroup per 16 columns: the chunk sums of its
// columns (coalesced over the rows) and T staged in LDS, then 64 MACs per output.
__global__ __launch_bounds__(256) void k_eig_tw(const double2* __restrict__ Tb, int64_t sT,
                                                const double2* __restrict__ W, int ldw, int64_t sW, int S, int kb,
                                                int n, double2* __restrict__ W2, int64_t sW2) {
  constexpr int NB = kEigNB, CW = 16;
  __shared__ double2 Ts[NB][NB + 1];
  __shared__ double2 Ws[CW][NB + 1];
  const int k = blockIdx.y, tid = threadIdx.x, c0 = blockIdx.x * CW;
  Tb += k * sT;
  W += k * sW;
  for (int q = tid; q < NB * NB; q += 256) Ts[q % NB][q / NB] = Tb[q];
  for (int q = tid; q < NB * CW; q += 256) {
    const int p = q % NB, cj = q / NB, col = c0 + cj;
    double2 a = cz();
    if (p < kb && col < n)
      for (int s = 0; s < S; ++s) a = cadd(a, W[(int64_t)col * ldw + s * kb + p]);
    Ws[cj][p] = a;
  }
  __syncthreads();
  for (int q = tid; q < NB * CW; q += 256) {
    const int p = q % NB, cj = q / NB, col = c0 + cj;
    if (p >= kb || col >= n) continue;
    double2 a = cz();
#pragma unroll 8
    for (int r = 0; r < kb; ++r) a = cadd(a, cmul(Ts[p][r], Ws[cj][r]));
    W2[k * sW2 + p + (int64_t)col * NB] = a;
  }
}

}  // namespace

// the deferral depth K of a batch of m matrices: kEigDefer from kEigDeferMin
// matrices on (HBM-bound passes), 1 below (latency-bound;
// profiles/r04_exp_eig_defer_*.json)
int eig_defer_k(int m) { return m < kEigDeferMin ? 1 : kEigDefer; }
// first column of a batch's one-matrix-scheme tail: n - M rounded up to a
// multiple of kEigDefer (column s-1 a write pass), M = DWHMC_EIG_SWITCH_M
// (A/B; 0: no tail)
int eig_switch_col(int n) {
  const char* v = std::getenv("DWHMC_EIG_SWITCH_M");   // read per solve (tests switch it)
  const int M = v ? std::atoi(v) : kEigSwitchM;
  if (M <= 0) return n + 1;
  const int s0 = std::max(kEigDefer, n - M);
  return (s0 + kEigDefer - 1) / kEigDefer * kEigDefer;
}

void launch_eig_step(double2* A, int n, int i, int64_t sA, const double2* part, int64_t sP, double2* pfin,
                     double2* colfin, double2* vv, double2* ww, double* d, double* e, double2* tau,
                     const double2* dpart, int m, int K, hipStream_t s) {
  if (i > 0)
    hipLaunchKernelGGL(k_eig_reduce, dim3((n - i + 255) / 256, m), dim3(256), 0, s, part, sP, n, i, pfin, A, sA,
                       colfin, vv, ww, dpart, K, (const double2*)tau, (double2*)nullptr);
  const int rs = (n - i + kStepT - 1) / kStepT;   // row slots the rows i..n-1 need
  static_assert(kEigMaxN <= 5 * kStepT, "k_eig_step instantiations");
#define DWH_EIG_STEP(R) \
  hipLaunchKernelGGL((k_eig_step<R>), dim3(m), dim3(kStepT), 0, s, A, n, i, sA, pfin, colfin, vv, ww, d, e, tau)
  switch (rs) {
    case 1: DWH_EIG_STEP(1); break;
    case 2: DWH_EIG_STEP(2); break;
    case 3: DWH_EIG_STEP(3); break;
    case 4: DWH_EIG_STEP(4); break;
    default: DWH_EIG_STEP(5); break;
  }
#undef DWH_EIG_STEP
}

void launch_eig_pass(double2* A, int n, int i, int64_t sA, double2* part, int64_t sP, const double2* vv,
                     const double2* ww, double2* dpart, int m, int K, hipStream_t s) {
  const int T = (n + kEigTB - 1) / kEigTB, t0 = (i + 1) / kEigTB, nT = T - t0;
  if (nT <= 0) return;
  if (K == 1)
    hipLaunchKernelGGL(k_eig_pass1, dim3(nT * (nT + 1) / 2, m), dim3(256), 0, s, A, n, i, sA, part, sP, vv, ww, t0);
  else
    hipLaunchKernelGGL(k_eig_pass<KD>, dim3(nT * (nT + 1) / 2, m), dim3(256), 0, s, A, n, i, sA, part, sP, vv, ww,
                       t0, dpart, T, K);
}

// Column i of the reduction: one matrix (K = 1) folds step i into pass i for
// 1 <= i <= n-2 (k_eig_reduce with the g partials, then k_eig_pass1f); else
// step i, then pass i.
void launch_eig_column(double2* A, int n, int i, int64_t sA, double2* part, int64_t sP, double2* pfin,
                       double2* colfin, double2* vv, double2* ww, double* d, double* e, double2* tau,
                       double2* dpart, double2* gpart, int m, hipStream_t s, int sw) {
  // Batches keep the step: folding it into the deferred pass measured slower,
  // every pass workgroup re-reading the column's vectors: 14.1 vs 13.2 ms per
  // measurement at 16 snapshots (profiles/r04_exp_eig_fused_step.txt) -- over
  // the HBM-bound columns.  The last kEigSwitchM columns (small trailing
  // triangles: the launches are the cost) run the one-matrix scheme instead
  // (K = 1: reduce + the pass with the step folded in, two launches per column
  // instead of three), switching after a write pass so no pair is pending.
  int K = eig_defer_k(m);
  if (K > 1 && i >= sw) K = 1;
  if (K == 1 && i >= 1 && i <= n - 2) {
    const int ngp = (n - i + 255) / 256;
    hipLaunchKernelGGL(k_eig_reduce, dim3(ngp, m), dim3(256), 0, s, part, sP, n, i, pfin, A, sA, colfin, vv, ww,
                       dpart, K, (const double2*)tau, gpart);
    const int T = (n + kEigTB - 1) / kEigTB, t0 = (i + 1) / kEigTB, nT = T - t0;
    hipLaunchKernelGGL(k_eig_pass1f, dim3(nT * (nT + 1) / 2, m), dim3(256), 0, s, A, n, i, sA, part, sP, vv, pfin,
                       colfin, gpart, ngp, d, e, tau, t0);
    return;
  }
  launch_eig_step(A, n, i, sA, part, sP, pfin, colfin, vv, ww, d, e, tau, dpart, m, K, s);
  if (i < n - 1) launch_eig_pass(A, n, i, sA, part, sP, vv, ww, dpart, m, K, s);
}

void launch_eig_bisect(const double* d, const double* e, int n, double* E, double* tnorm, int m, hipStream_t s) {
  // lanes per eigenvalue: 64 down to 4 as the batch grows, keeping >= ~2048
  // waves (two per SIMD) in flight
  int lgG = 6;
  while (lgG > 2 && ((int64_t)m * n << (lgG - 1)) >= (int64_t)2048 * 64) --lgG;
  const int per_wg = kBisW << (6 - lgG);
  hipLaunchKernelGGL(k_eig_bisect, dim3((n + per_wg - 1) / per_wg, m), dim3(64 * kBisW), 2 * n * sizeof(double), s, d,
                     e, n, lgG, E, tnorm);
}

void launch_eig_invit(const double* d, const double* e, int n, const double* E, const double* tnorm, double* Zt,
                      double* U0, double* U1, double* U2, int64_t sZ, int* bad, int m, hipStream_t s, int maxc, int j0,
                      const int* c0) {
  const int nj = n - j0;
  if (nj <= 0) return;
  hipLaunchKernelGGL(k_eig_invit, dim3((nj + 63) / 64, m), dim3(64), 2 * n * sizeof(double), s, d, e, n, E, tnorm,
                     Zt, U0, U1, U2, sZ, j0, c0);
  hipLaunchKernelGGL(k_eig_orth, dim3(nj, m), dim3(256), 0, s, E, tnorm, n, Zt, sZ, kEigClusterTol, bad,
                     maxc < 1 || maxc > kEigMaxCluster ? kEigMaxCluster : maxc, j0, c0);
}

void launch_eig_theta(double2* U, int n, int64_t sA, const int* c0, int m, hipStream_t s) {
  if (n < 2) return;
  hipLaunchKernelGGL(k_eig_theta, dim3((n + 255) / 256, n / 2, m), dim3(256), 0, s, U, n, sA, c0);
}

void launch_eig_zt_to_u(const double* Zt, double2* U, int n, int64_t sZ, int64_t sA, int m, hipStream_t s, int j0) {
  const int T = (n + 63) / 64, TC = (n - j0 + 63) / 64;
  if (TC <= 0) return;
  hipLaunchKernelGGL(k_eig_zt_to_u, dim3(TC, T, m), dim3(256), 0, s, Zt, U, n, sZ, sA, j0);
}

void launch_eig_tfac(const double2* V, int n, int64_t sA, const double2* tau, double2* Gp, double2* Tb, int64_t sT,
                     int m, hipStream_t s) {
  const int nblk = (n - 1 + kEigNB - 1) / kEigNB;
  if (nblk <= 0) return;
  hipLaunchKernelGGL(k_eig_tgram, dim3(nblk, kEigGS, m), dim3(256), 0, s, V, n, sA, Gp);
  hipLaunchKernelGGL(k_eig_tfac, dim3(nblk, m), dim3(256), 0, s, Gp, n, tau, Tb, sT);
}

void launch_eig_vt(const double2* A, int n, int64_t sA, double2* Vt, int m, hipStream_t s) {
  const int nblk = (n - 1 + kEigNB - 1) / kEigNB;
  if (nblk < 1) return;
  hipLaunchKernelGGL(k_eig_vt, dim3((n - 1 + 31) / 32, nblk, m), dim3(256), 0, s, A, n, sA, Vt);
}

void launch_eig_tw(const double2* Tb, int64_t sT, const double2* W, int ldw, int64_t sW, int S, int kb, int n,
                   double2* W2, int64_t sW2, int m, hipStream_t s) {
  hipLaunchKernelGGL(k_eig_tw, dim3((n + 15) / 16, m), dim3(256), 0, s, Tb, sT, W, ldw, sW, S, kb, n, W2, sW2);
}

}  // namespace dwh
