// Structure-preserving (quaternion) Hermitian eigensolver for the BdG matrix
// of the transport / spectra measurement (src/Observables.jl:314-526, the
// eigen!(Hermitian(H)) of src/Hamiltonian.jl:96-114); numpy prototype with the
// same algebra: tools/qeig_proto.py.
//
// H_BdG = [[h, D], [conj D, -conj h]] (h Hermitian, D symmetric) anticommutes
// with Theta (u; v) = (-conj v; conj u), Theta^2 = -1.
// Unitaries that commute with Theta keep that form, so the matrix is reduced
// site by site (M = N sites, n = 2M) on its particle rows only:
//
//   step j        x = column j below site j+1 (particle and hole entries of
//                 the sites j+1 ..), v = x + s x1 (x1: site j+1's two entries,
//                 s = |x| / |x1|), U = I - tau (v v^H + Theta v (Theta v)^H),
//                 tau = 2 / |v|^2, U x = y = -s x1.  Since H Theta = -Theta H,
//                 one matrix-vector product p = H v per site; w1 = tau p -
//                 tau^2 / 2 (r v - conj(c) Theta v), r = v^H p, c = v^H Theta p,
//                 and H <- H - v w1^H - w1 v^H + Theta v (Theta w1)^H +
//                 Theta w1 (Theta v)^H on the particle rows of the sites > j+1.
//   launches      k_q_rs (one workgroup per matrix): p = H v_j read from P,
//                 w1_j, site j+1's two columns updated, its diagonal block and
//                 the reflector v_{j+1}; k_q_pass (one workgroup per 64 x 64
//                 lower-triangle tile of h and of D on the remaining sites):
//                 update j applied and written back, p = H v_{j+1} from the
//                 same tiles (both triangles by symmetry) into P by 64-bit
//                 fixed-point integer atomics (exact: bit-reproducible in any
//                 order).  Two launches per SITE (the one-stage reduction
//                 needs two per column, i.e. twice as many), each pass over
//                 m^2 stored elements (m active sites; the one-stage pass
//                 reads (2m)^2 / 2).  L = 32: 16.1 ms against 29.5 ms for the
//                 one-stage tridiagonalisation (profiles/r06_qeig_reduction_L32.txt:
//                 latency-bound, ~14-20 us per site for two dependent launches).
//   rotations     k_q_rot: unit quaternions g_j per site make the
//                 off-diagonal site blocks b_j sigma_z: T = [[A, C], [conj C,
//                 -A]] with A = tridiag(a'; b) real and C = diag(d') complex.
//   eigenvalues   k_q_bisect: G-lane multisection on block Sturm counts
//                 (S_{j+1} = D_{j+1} - x - b_j^2 sigma_z S_j^-1 sigma_z, the
//                 negative eigenvalues of each 2 x 2 S_j).
//
// Storage (one matrix; A column-major n x n, ld n): the particle rows of A
// (rows < M) hold the reducing matrix; the reflector v_j is kept in the
// bottom rows of columns 2j (particle entries, row M + site) and 2j + 1 (hole
// entries), which the reduction never reads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cfloat>
#include <cstdlib>
#include <type_traits>

#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {
namespace {

constexpr int kQTB = 64;     // pass tile: rows x columns
#ifndef QINVIT_ITERS
#define QINVIT_ITERS 2   // inverse-iteration solves per eigenvector (at most)
#endif
#ifndef QINVIT_SHARE
#define QINVIT_SHARE 1e-6
#endif
constexpr double kQInvitShare = QINVIT_SHARE;   // bound on the other eigenvectors' share after one solve
constexpr int kQMaxCluster = 32;   // longest eigenvalue cluster the structure-preserving solver orthonormalises
constexpr double kQClusterShift = 1e-12;   // a cluster member's inverse-iteration shift below its level, x ||T||
constexpr int kQRS = 1024;   // k_q_rs threads
constexpr int kQMaxR = 3;    // rows per k_q_rs thread: M <= kQMaxM
}  // namespace
constexpr int kQMaxM = kQRS * kQMaxR;
namespace {

__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 cneg(double2 a) { return make_double2(-a.x, -a.y); }
__device__ __forceinline__ double2 cscale(double s, double2 a) { return make_double2(s * a.x, s * a.y); }
// a * conj(b) accumulated: acc + a conj(b)
__device__ __forceinline__ double2 cmac_c(double2 acc, double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, fma(a.y, b.y, acc.x)), fma(a.y, b.x, fma(-a.x, b.y, acc.y)));
}
// acc + a b
__device__ __forceinline__ double2 cmac(double2 acc, double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, fma(-a.y, b.y, acc.x)), fma(a.x, b.y, fma(a.y, b.x, acc.y)));
}

// Sum over a 16-lane DPP row, in every lane of the row (quad swaps, then the
// half-row and row mirrors: no LDS traffic; a + b = b + a, so all 16 lanes
// hold the same bits)
__device__ __forceinline__ double dpp_sum16(double x) {
  x += __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xf, 0xf, true);    // quad_perm [1,0,3,2]
  x += __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xf, 0xf, true);    // quad_perm [2,3,0,1]
  x += __builtin_amdgcn_update_dpp(x, x, 0x141, 0xf, 0xf, true);   // row_half_mirror
  x += __builtin_amdgcn_update_dpp(x, x, 0x140, 0xf, 0xf, true);   // row_mirror
  return x;
}
// wave total (uniform): the four row sums in a fixed order
__device__ __forceinline__ double dpp_wave_sum(double x) {
  x = dpp_sum16(x);
  return (readlane_f64(x, 0) + readlane_f64(x, 16)) + (readlane_f64(x, 32) + readlane_f64(x, 48));
}
// v_permlane32_swap (W = 32: lanes 32-63 of a <-> lanes 0-31 of b) or
// v_permlane16_swap (W = 16: the odd 16-lane rows of a <-> the even rows of
// b) on both dwords of a pair of doubles: afterwards a + b holds, in the
// lanes whose bit log2(W) is clear, a summed with its partner lane and, in
// the others, b summed with its partner
template <int W>
__device__ __forceinline__ void perm_swap(double& a, double& b) {
  uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  if constexpr (W == 32) {
    const auto r0 = __builtin_amdgcn_permlane32_swap(ua.x, ub.x, false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap(ua.y, ub.y, false, false);
    ua = make_uint2(r0[0], r1[0]);
    ub = make_uint2(r0[1], r1[1]);
  } else {
    const auto r0 = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
    ua = make_uint2(r0[0], r1[0]);
    ub = make_uint2(r0[1], r1[1]);
  }
  a = __builtin_bit_cast(double, ua);
  b = __builtin_bit_cast(double, ub);
}

// workgroup totals of three values (fixed order; every thread returns them).
// One barrier: sh must not be reused by the previous reduction of the kernel.
__device__ __forceinline__ void block_sum3(double& a, double& b, double& c, double (*sh)[3]) {
  a = dpp_wave_sum(a);
  b = dpp_wave_sum(b);
  c = dpp_wave_sum(c);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w][0] = a;
    sh[w][1] = b;
    sh[w][2] = c;
  }
  __syncthreads();
  a = b = c = 0.0;
  for (int k = 0; k < nw; ++k) {
    a += sh[k][0];
    b += sh[k][1];
    c += sh[k][2];
  }
}

// Per-matrix scratch q of the reduction (doubles): P [M][4] as 64-bit fixed
// point (p_p re, im, p_h re, im of p = H v, accumulated by k_q_pass with
// integer atomics: exact, so the sum is the same bits in any order), the
// dots r = v^H p and c' = sum (v_h p_p - v_p p_h) (c = v^H Theta p = conj c')
// accumulated the same way in kQDotSlots slots [slot][4] (a pass workgroup
// adds into slot blockIdx % kQDotSlots: one hot address would serialise the
// atomics, +12 ms at L = 32), the fixed-point scales of p and of the dots
// per reflector [M] each, the Frobenius partials [256] and ||H||_F.
constexpr int kQDotSlots = 64;   // dot accumulators (spread over the pass workgroups: no hot address)
__host__ __device__ __forceinline__ int64_t q_racc_off(int M) { return 4 * (int64_t)M; }
__host__ __device__ __forceinline__ int64_t q_scale_off(int M) { return 4 * (int64_t)M + 4 * kQDotSlots; }
__host__ __device__ __forceinline__ int64_t q_scale2_off(int M) { return 5 * (int64_t)M + 4 * kQDotSlots; }
__host__ __device__ __forceinline__ int64_t q_fro_off(int M) { return 6 * (int64_t)M + 4 * kQDotSlots; }
constexpr int kQFro = 256;   // k_q_fro workgroups

// Diagnostic build only (-DQSTAMPS, tools/q_ab.sh): s_memrealtime (100 MHz)
// of wave 0 at the phases of k_q_rs ([j][0..7]) and of k_q_pass's
// workgroup 0 ([j][8..14]), the shader clock at k_q_rs's end ([j][15]);
// read back by dwh_debug_qeig into $QSTAMPS_FILE.
#ifdef QSTAMPS
__device__ unsigned long long g_qst[4096][16];
#define QSTAMP(cond, i)                                                    \
  do {                                                                     \
    unsigned long long t_ = __builtin_amdgcn_s_memrealtime();              \
    asm volatile("" ::"s"(t_));                                            \
    if ((cond) && threadIdx.x == 0 && j >= 0 && j < 4096) g_qst[j][i] = t_; \
  } while (0)
#else
#define QSTAMP(cond, i) \
  do {                  \
  } while (0)
#endif
#define QST(i) QSTAMP(true, i)
#define QSTP(i) QSTAMP(blockIdx.x == 0, 8 + (i))

// Partial sums of |H_ij|^2 over the particle rows (all 2M columns): ||H||_F
// bounds |(H v)_i| / |v| for every trailing block the reduction meets (the
// similarity transforms keep the Frobenius norm), hence the fixed-point
// scale of p.
__global__ __launch_bounds__(256) void k_q_fro(const double2* __restrict__ A, int M, int64_t sA,
                                               double* __restrict__ q, int64_t sQ) {
  const int k = blockIdx.y, n = 2 * M;
  A += k * sA;
  double s = 0.0;
  for (int c = blockIdx.x; c < n; c += kQFro)
    for (int r = threadIdx.x; r < M; r += 256) {
      const double2 a = A[r + (int64_t)c * n];
      s += a.x * a.x + a.y * a.y;
    }
  __shared__ double sh[4][3];
  double d1 = 0.0, d2 = 0.0;
  block_sum3(s, d1, d2, sh);
  if (threadIdx.x == 0) q[k * sQ + q_fro_off(M) + blockIdx.x] = s;
}

// Step j of the reduction for one matrix (blockIdx.x), j = -1 .. M-2:
// (j >= 0) p = H v_j (P, from k_q_pass), r, c, w1_j (to W by site: W[s]
// particle, W[M + s] hole); site j+1's columns updated with pair j; its
// diagonal block (qa, qd); (j + 1 <= M - 2) the reflector v_{j+1}, tau, y and
// its fixed-point scale.  j = -1 also forms ||H||_F from k_q_fro's partials.
// Every load is issued first and every global store comes after the last
// barrier (a barrier waits for the stores in flight).
__global__ __launch_bounds__(kQRS) void k_q_rs(double2* __restrict__ A, int M, int j, int64_t sA,
                                               double* __restrict__ q, int64_t sQ,
                                               double2* __restrict__ W, double* __restrict__ tau,
                                               double2* __restrict__ Y, double* __restrict__ qa,
                                               double2* __restrict__ qd) {
  const int k = blockIdx.x, n = 2 * M, t = threadIdx.x;
  A += k * sA;
  q += k * sQ;
  long long* P = reinterpret_cast<long long*>(q);
  W += (int64_t)k * n;
  tau += (int64_t)k * M;
  Y += (int64_t)k * 2 * M;
  qa += (int64_t)k * M;
  qd += (int64_t)k * M;
  __shared__ double sh2[kQRS / 64][3];
  __shared__ double2 bc[8];
  const int s0 = j + 1;            // site j+1: the column pair reduced next
  const int m = M - s0;            // active sites of step j (j >= 0), rows i <-> site s0 + i
  const bool upd = j >= 0;
  QST(0);
  const double2 z = make_double2(0.0, 0.0);
  double2 cp[kQMaxR], ch[kQMaxR];  // site s0's particle / hole column at row s0 + i (updated)
  double2 vp[kQMaxR], vh[kQMaxR], wp[kQMaxR], wh[kQMaxR];
  const double2* vpj = A + M + (int64_t)(2 * j) * n;       // v_j by site: particle
  const double2* vhj = A + M + (int64_t)(2 * j + 1) * n;   // hole
  // uniform values as vector loads (a scalar load is sunk to its use, after
  // the first reduction: a second memory round trip)
  int zv;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
  const double tj = upd ? tau[j + zv] : 0.0;
  const double isc = upd ? 1.0 / q[q_scale_off(M) + j + zv] : 0.0;
  const double isc2 = upd ? 1.0 / q[q_scale2_off(M) + j + zv] : 0.0;
  long long* Racc = reinterpret_cast<long long*>(q + q_racc_off(M));
  // wave 0: one dot slot per lane
  long long ra0 = 0, ra1 = 0, ra2 = 0;
  if (upd && t < kQDotSlots) {
    ra0 = Racc[4 * t];
    ra1 = Racc[4 * t + 1];
    ra2 = Racc[4 * t + 2];
  }
  const double fro = upd ? q[q_fro_off(M) + kQFro + zv] : (t < kQFro ? q[q_fro_off(M) + t] : 0.0);
  double2 pp[kQMaxR], ph[kQMaxR];
#pragma unroll
  for (int u = 0; u < kQMaxR; ++u) {
    const int i = t + u * kQRS;
    cp[u] = ch[u] = vp[u] = vh[u] = wp[u] = wh[u] = pp[u] = ph[u] = z;
    if (i < m) {
      cp[u] = A[(int64_t)(s0 + i) + (int64_t)s0 * n];
      ch[u] = A[(int64_t)(s0 + i) + (int64_t)(M + s0) * n];
      if (upd) {
        const long long* ps = P + 4 * (int64_t)(s0 + i);
        pp[u] = make_double2((double)ps[0] * isc, (double)ps[1] * isc);
        ph[u] = make_double2((double)ps[2] * isc, (double)ps[3] * isc);
        vp[u] = vpj[s0 + i];
        vh[u] = vhj[s0 + i];
      }
    }
  }
  double hf = fro;
  if (upd) {
    QST(1);
    // r = v^H p and c = v^H Theta p = conj(sum v_h p_p - v_p p_h), accumulated
    // by k_q_pass tile by tile (fixed point, exact): wave 0 sums the slots;
    // published with the row-0 entries (thread 0) through one barrier
    if (t < 64) {
      const double s0r = dpp_wave_sum((double)ra0 * isc2), s1r = dpp_wave_sum((double)ra1 * isc2),
                   s2r = dpp_wave_sum((double)ra2 * isc2);
      if (t == 0) {
        bc[6] = make_double2(s0r, s1r);
        bc[7] = make_double2(-s2r, 0.0);
        bc[0] = vp[0];
        bc[1] = vh[0];
        bc[2] = pp[0];
        bc[3] = ph[0];
      }
    }
    __syncthreads();
    QST(2);
    const double r = bc[6].x, cr = bc[6].y, ci = bc[7].x;
    // w1 = tau p - tau^2 / 2 (r v - conj(c) Theta v), (Theta v)_p = -conj v_h, (Theta v)_h = conj v_p
    const double h2 = 0.5 * tj * tj;
    const double2 cc = make_double2(cr, -ci);
    auto w1 = [&](double2 a_p, double2 a_h, double2 b_p, double2 b_h, double2& o_p, double2& o_h) {
      // (a: v, b: p) -> (o_p, o_h) = w1
      const double2 tvp = cneg(cconj(a_h)), tvh = cconj(a_p);
      const double2 ap = cmac(cscale(r, a_p), cneg(cc), tvp), ah = cmac(cscale(r, a_h), cneg(cc), tvh);
      o_p = make_double2(tj * b_p.x - h2 * ap.x, tj * b_p.y - h2 * ap.y);
      o_h = make_double2(tj * b_h.x - h2 * ah.x, tj * b_h.y - h2 * ah.y);
    };
#pragma unroll
    for (int u = 0; u < kQMaxR; ++u) w1(vp[u], vh[u], pp[u], ph[u], wp[u], wh[u]);
    const double2 v0p = bc[0], v0h = bc[1];
    double2 w0p, w0h;
    w1(bc[0], bc[1], bc[2], bc[3], w0p, w0h);
    QST(3);
    // column s0 (particle, l = 0): v_l = v0p, w_l = w0p, tv_l = -conj v0h, tw_l = -conj w0h;
    // column M + s0 (hole, l = m): v_l = v0h, w_l = w0h, tv_l = conj v0p, tw_l = conj w0p
    const double2 Lv[2] = {v0p, v0h}, Lw[2] = {w0p, w0h};
    const double2 Ltv[2] = {cneg(cconj(v0h)), cconj(v0p)}, Ltw[2] = {cneg(cconj(w0h)), cconj(w0p)};
#pragma unroll
    for (int u = 0; u < kQMaxR; ++u) {
      const double2 tvr = cneg(cconj(vh[u])), twr = cneg(cconj(wh[u]));
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        double2 d = z;
        d = cmac_c(d, vp[u], Lw[hh]);
        d = cmac_c(d, wp[u], Lv[hh]);
        d = cmac_c(d, cneg(tvr), Ltw[hh]);
        d = cmac_c(d, cneg(twr), Ltv[hh]);
        if (hh == 0) {
          cp[u].x -= d.x;
          cp[u].y -= d.y;
        } else {
          ch[u].x -= d.x;
          ch[u].y -= d.y;
        }
      }
    }
  }
  const bool refl = s0 <= M - 2;
  // the reflector of site s0: x = rows i >= 1 (sites s0 + 1 ..): x_p = cp, x_h = conj ch
  double nx = 0.0, sc = 0.0, tq = 0.0;
  double2 yp = z, yh = z;
  bool e1only = false;   // x1 = 0: v = x + |x| e_p (site s0 + 1)
  if (refl || !upd) {
    double nx2 = 0.0, d1 = 0.0;
#pragma unroll
    for (int u = 0; u < kQMaxR; ++u) {
      const int i = t + u * kQRS;
      if (i >= 1 && i < m) nx2 += cp[u].x * cp[u].x + cp[u].y * cp[u].y + ch[u].x * ch[u].x + ch[u].y * ch[u].y;
    }
    // x1: row i = 1 (thread 1), published with the norm's barrier
    if (t == 1) {
      bc[4] = cp[0];
      bc[5] = cconj(ch[0]);
    }
    QST(4);
    // j = -1: the Frobenius partials (k_q_fro) in the same reduction
    double fsum = !upd && t < kQFro ? fro : 0.0;
    block_sum3(nx2, fsum, d1, sh2);
    if (!upd) hf = sqrt(fsum);
    QST(5);
    const double2 x1p = bc[4], x1h = bc[5];
    nx = sqrt(nx2);
    const double n1 = sqrt(x1p.x * x1p.x + x1p.y * x1p.y + x1h.x * x1h.x + x1h.y * x1h.y);
    if (refl && nx > 0.0) {
      if (n1 > 0.0) {
        sc = nx / n1;
        tq = 1.0 / (nx * (nx + n1));   // 2 / |v|^2, |v|^2 = 2 |x| (|x| + |x1|)
        yp = cscale(-sc, x1p);
        yh = cscale(-sc, x1h);
      } else {
        e1only = true;
        tq = 1.0 / (nx * nx);
        yp = make_double2(-nx, 0.0);
      }
    }
  }
  QST(6);
  // the stores
  if (upd && t < kQDotSlots) Racc[4 * t] = Racc[4 * t + 1] = Racc[4 * t + 2] = 0;   // for the next pass
  if (t == 0) {   // site s0's diagonal block (row i = 0 of its columns)
    qa[s0] = cp[0].x;
    qd[s0] = ch[0];
  }
  double2* vpn = A + M + (int64_t)(2 * s0) * n;       // v_{s0} by site
  double2* vhn = A + M + (int64_t)(2 * s0 + 1) * n;
#pragma unroll
  for (int u = 0; u < kQMaxR; ++u) {
    const int i = t + u * kQRS;
    if (i >= m) continue;
    if (upd) {
      W[s0 + i] = wp[u];
      W[M + s0 + i] = wh[u];
      long long* ps = P + 4 * (int64_t)(s0 + i);   // zeroed for the next pass's atomics
      ps[0] = ps[1] = ps[2] = ps[3] = 0;
    }
    if (refl && i >= 1) {
      // row 1 (site s0 + 1): x1 (1 + s), or x1 + |x| e_p when x1 = 0 (branch-free)
      const bool first = i == 1;
      const double fac = first && !e1only ? 1.0 + sc : 1.0, add = first && e1only ? nx : 0.0;
      const double keep = nx > 0.0 ? 1.0 : 0.0;
      const double2 xp = make_double2(keep * (fac * cp[u].x + add), keep * fac * cp[u].y);
      const double2 xh = make_double2(keep * fac * ch[u].x, -keep * fac * ch[u].y);
      vpn[s0 + i] = xp;
      vhn[s0 + i] = xh;
    }
  }
  if (t == 0) {
    if (!upd) q[q_fro_off(M) + kQFro] = hf;

    if (refl) {
      tau[s0] = tq;
      Y[2 * s0] = yp;
      Y[2 * s0 + 1] = yh;
      // fixed-point scale of p = H v_{s0}: |p_i| <= ||H||_F |v| = ||H||_F sqrt(2 / tau) < 2^60 / scale
      const double bnd = tq > 0.0 ? hf * sqrt(2.0 / tq) : 0.0;
      q[q_scale_off(M) + s0] = bnd > 0.0 ? ldexp(1.0, 59 - ilogb(bnd)) : 1.0;
      // and of the dots: |r|, |c| <= ||H||_F |v|^2
      const double bnd2 = tq > 0.0 ? hf * (2.0 / tq) : 0.0;
      q[q_scale2_off(M) + s0] = bnd2 > 0.0 ? ldexp(1.0, 59 - ilogb(bnd2)) : 1.0;
    }
  }
  QST(7);
#ifdef QSTAMPS
  {
    unsigned long long c_ = __builtin_amdgcn_s_memtime();   // shader clock: the clock rate from [7] / [15]
    asm volatile("" ::"s"(c_));
    if (threadIdx.x == 0 && j >= 0 && j < 4096) g_qst[j][15] = c_;
  }
#endif
}

__device__ __forceinline__ void q_tri_decode(int b, int& R, int& C) {
  int r = (int)((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= b) ++r;
  while (r * (r + 1) / 2 > b) --r;
  R = r;
  C = b - r * (r + 1) / 2;
}

// Pass of step j (j = -1 .. M-3) over the sites s >= s1 = j+2: pair j applied
// (j >= 0) to the lower triangles of h (particle rows x particle columns) and
// of D (particle rows x hole columns, D = D^T) and written back, and p = H
// v_{j+1} from the same tiles (the upper triangles by symmetry: h^H = h, D^T
// = D):
//   p_p = h v'_p + D v'_h,  p_h = conj(D) v'_p - conj(h) v'_h.
// One workgroup of 16 waves per lower 64 x 64 tile (R, C) of h or of D (tiles
// at fixed 64-site boundaries); lane = row, wave w the columns 4 w .. 4 w + 3
// (four elements per thread: the waves hide each other's FP64 and LDS
// latency).  Row sums through LDS; column sums by a lane transpose-reduce
// (17 shuffles for 4 columns x 4 doubles).  Both go to P as 64-bit fixed
// point (scale from k_q_rs) by integer atomics: exact in any order, so
// bit-reproducible, and no separate partial-sum launch.
constexpr int kQPW = 16;   // waves per pass workgroup
__global__ __launch_bounds__(64 * kQPW) void k_q_pass(double2* __restrict__ A, int M, int j, int64_t sA,
                                                      const double2* __restrict__ W, double* __restrict__ q,
                                                      int64_t sQ) {
  const int k = blockIdx.y, n = 2 * M, s1 = j + 2;
  const int nT = (M + kQTB - 1) / kQTB, t0 = s1 / kQTB, nt = nT - t0, ntri = nt * (nt + 1) / 2;
  const int type = (int)blockIdx.x >= ntri ? 1 : 0;   // 0: h, 1: D
  int R, C;
  q_tri_decode(blockIdx.x - type * ntri, R, C);
  R += t0;
  C += t0;
  A += k * sA;
  W += (int64_t)k * n;
  q += k * sQ;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  QSTP(0);
  const int sr = R * kQTB + lane;
  const bool rok = sr >= s1 && sr < M;
  const int64_t cb = type ? (int64_t)M * n : 0;   // D: columns M + s
  // the tile (lower triangle), in flight while the vectors are staged
  double2 a[4];
  unsigned act = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int sc = C * kQTB + 4 * w + u;
    const bool ok = rok && sc >= s1 && sc <= sr;
    act |= (unsigned)ok << u;
    a[u] = ok ? A[cb + sr + (int64_t)sc * n] : make_double2(0.0, 0.0);
  }
  int zv;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
  const double scale = q[q_scale_off(M) + j + 1 + zv];
  // per column: v_l, w_l, tv_l, tw_l (pair j, by block type), v'_p, v'_h (v_{j+1})
  __shared__ double2 cv[kQTB][6];
  __shared__ double2 rowv[kQTB][2];   // v_{j+1} at the tile's rows (particle, hole)
  __shared__ double rowp[kQPW][kQTB][4];
  __shared__ double colsum[kQTB][4];
  const double2* vpj = A + M + (int64_t)(2 * j) * n;
  const double2* vhj = A + M + (int64_t)(2 * j + 1) * n;
  const double2* vpn = A + M + (int64_t)(2 * (j + 1)) * n;
  const double2* vhn = A + M + (int64_t)(2 * (j + 1) + 1) * n;
  const double2 z = make_double2(0.0, 0.0);
  if (tid < kQTB) {
    const int sc = C * kQTB + tid;
    double2 v = z, wv = z, tv = z, tw = z, np = z, nh = z;
    if (sc >= s1 && sc < M) {
      if (j >= 0) {
        const double2 vp = vpj[sc], vh = vhj[sc], wp = W[sc], wh = W[M + sc];
        v = type ? vh : vp;
        wv = type ? wh : wp;
        tv = type ? cconj(vp) : cneg(cconj(vh));
        tw = type ? cconj(wp) : cneg(cconj(wh));
      }
      np = vpn[sc];
      nh = vhn[sc];
    }
    cv[tid][0] = v;
    cv[tid][1] = wv;
    cv[tid][2] = tv;
    cv[tid][3] = tw;
    cv[tid][4] = np;
    cv[tid][5] = nh;
  }
  double2 vr = z, wr = z, tvr = z, twr = z, npr = z, nhr = z;
  if (rok) {
    if (j >= 0) {
      vr = vpj[sr];
      wr = W[sr];
      tvr = cneg(cconj(vhj[sr]));
      twr = cneg(cconj(W[M + sr]));
    }
    npr = vpn[sr];
    nhr = vhn[sr];
  }
  if (tid < kQTB) {
    rowv[tid][0] = npr;
    rowv[tid][1] = nhr;
  }
  __syncthreads();
  QSTP(1);
  double2 rp = z, rh = z;
  double cs[16];   // column sums: [u][p_p re, im, p_h re, im]
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int cl = 4 * w + u;
    double2 x = a[u];
    const bool on = (act >> u) & 1;
    if (on && j >= 0) {
      double2 d = z;
      d = cmac_c(d, vr, cv[cl][1]);
      d = cmac_c(d, wr, cv[cl][0]);
      d = cmac_c(d, cneg(tvr), cv[cl][3]);
      d = cmac_c(d, cneg(twr), cv[cl][2]);
      x.x -= d.x;
      x.y -= d.y;
      a[u] = x;   // stored after the barrier below (a barrier waits for stores in flight)
    }
    const double2 cnp = cv[cl][4], cnh = cv[cl][5];
    const bool off = on && C * kQTB + cl < sr;   // strictly below the diagonal: also the transpose
    double2 cpp, cph;
    if (type == 0) {   // h: p_p += h v'_p, p_h -= conj(h) v'_h; transposed: conj(h) v'_p, -h v'_h
      rp = cmac(rp, x, cnp);
      rh = cmac(rh, cneg(cconj(x)), cnh);
      cpp = cmac(z, cconj(x), npr);
      cph = cmac(z, cneg(x), nhr);
    } else {           // D: p_p += D v'_h, p_h += conj(D) v'_p; transposed: the same
      rp = cmac(rp, x, cnh);
      rh = cmac(rh, cconj(x), cnp);
      cpp = cmac(z, x, nhr);
      cph = cmac(z, cconj(x), npr);
    }
    cs[4 * u] = off ? cpp.x : 0.0;
    cs[4 * u + 1] = off ? cpp.y : 0.0;
    cs[4 * u + 2] = off ? cph.x : 0.0;
    cs[4 * u + 3] = off ? cph.y : 0.0;
  }
  QSTP(2);
  // column sums over the 64 lanes, transpose-reduce without LDS: each stage
  // pairs lanes that differ in one index bit (v_permlane32 / 16_swap for
  // bits 5 / 4, DPP row_mirror / row_half_mirror for bits 3 / 2) and halves
  // the values a lane holds; lane l ends with value (l >> 2) & 15, summed
  // over a quarter of the lanes, then the quad sums
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    perm_swap<32>(cs[i], cs[i + 8]);
    cs[i] += cs[i + 8];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    perm_swap<16>(cs[i], cs[i + 4]);
    cs[i] += cs[i + 4];
  }
  {
    const bool up3 = lane & 8, up2 = lane & 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double send = up3 ? cs[i] : cs[i + 2], keep = up3 ? cs[i + 2] : cs[i];
      cs[i] = keep + __builtin_amdgcn_update_dpp(send, send, 0x140, 0xf, 0xf, true);   // row_mirror
    }
    const double send = up2 ? cs[0] : cs[1], keep = up2 ? cs[1] : cs[0];
    cs[0] = keep + __builtin_amdgcn_update_dpp(send, send, 0x141, 0xf, 0xf, true);     // row_half_mirror
  }
  cs[0] += __builtin_amdgcn_update_dpp(cs[0], cs[0], 0xB1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
  cs[0] += __builtin_amdgcn_update_dpp(cs[0], cs[0], 0x4E, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
  QSTP(3);
  if ((lane & 3) == 0) {
    const int vi = (lane >> 2) & 15;
    colsum[4 * w + (vi >> 2)][vi & 3] = cs[0];
  }
  rowp[w][lane][0] = rp.x;
  rowp[w][lane][1] = rp.y;
  rowp[w][lane][2] = rh.x;
  rowp[w][lane][3] = rh.y;
  __syncthreads();
  QSTP(4);
  if (j >= 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((act >> u) & 1) A[cb + sr + (int64_t)(C * kQTB + 4 * w + u) * n] = a[u];
  }
  QSTP(5);
  if (tid < 4 * kQTB) {
    const int so = tid >> 2, e = tid & 3;
    double rv = 0.0;
#pragma unroll
    for (int ww = 0; ww < kQPW; ++ww) rv += rowp[ww][so][e];
    const double cvs = colsum[so][e];
    unsigned long long* P = reinterpret_cast<unsigned long long*>(q);
    const int srs = R * kQTB + so, scs = C * kQTB + so;
    auto fx = [&](double x) { return (unsigned long long)__double2ll_rn(x * scale); };
    // this entry's share of r = v^H p and c' = sum (v_h p_p - v_p p_h)
    double dr = 0.0, dcr = 0.0, dci = 0.0;
    auto dots = [&](double val, double2 vp, double2 vh) {
      if (e == 0) {        // Re p_p
        dr += vp.x * val;
        dcr += vh.x * val;
        dci += vh.y * val;
      } else if (e == 1) { // Im p_p
        dr += vp.y * val;
        dcr -= vh.y * val;
        dci += vh.x * val;
      } else if (e == 2) { // Re p_h
        dr += vh.x * val;
        dcr -= vp.x * val;
        dci -= vp.y * val;
      } else {             // Im p_h
        dr += vh.y * val;
        dcr += vp.y * val;
        dci -= vp.x * val;
      }
    };
    if (R == C) {
      if (srs < M && srs >= s1) {
        atomicAdd(&P[(int64_t)srs * 4 + e], fx(rv + cvs));
        dots(rv + cvs, rowv[so][0], rowv[so][1]);
      }
    } else {
      if (srs < M && srs >= s1) {
        atomicAdd(&P[(int64_t)srs * 4 + e], fx(rv));
        dots(rv, rowv[so][0], rowv[so][1]);
      }
      if (scs < M && scs >= s1) {
        atomicAdd(&P[(int64_t)scs * 4 + e], fx(cvs));
        dots(cvs, cv[so][4], cv[so][5]);
      }
    }
    // per wave (no barrier: the tile's stores are in flight), three fixed-point atomics
    dr = dpp_wave_sum(dr);
    dcr = dpp_wave_sum(dcr);
    dci = dpp_wave_sum(dci);
    if (lane == 0) {
      const double sc2 = q[q_scale2_off(M) + j + 1];
      unsigned long long* Ra = reinterpret_cast<unsigned long long*>(q + q_racc_off(M)) + 4 * (blockIdx.x % kQDotSlots);
      atomicAdd(&Ra[0], (unsigned long long)__double2ll_rn(dr * sc2));
      atomicAdd(&Ra[1], (unsigned long long)__double2ll_rn(dcr * sc2));
      atomicAdd(&Ra[2], (unsigned long long)__double2ll_rn(dci * sc2));
    }
  }
  QSTP(6);
}

// quaternion product of unit quaternions (al, be) <-> [[al, -conj be], [be, conj al]]
__device__ __forceinline__ void qmul(double2 a1, double2 b1, double2 a2, double2 b2, double2& a, double2& b) {
  // al = a1 a2 - conj(b1) b2, be = b1 a2 + conj(a1) b2
  a = make_double2(a1.x * a2.x - a1.y * a2.y - (b1.x * b2.x + b1.y * b2.y),
                   a1.x * a2.y + a1.y * a2.x - (b1.x * b2.y - b1.y * b2.x));
  b = make_double2(b1.x * a2.x - b1.y * a2.y + (a1.x * b2.x + a1.y * b2.y),
                   b1.x * a2.y + b1.y * a2.x + (a1.x * b2.y - a1.y * b2.x));
}

// Site rotations (one workgroup per matrix): g_0 = 1, g_{j+1} = q^_j
// tau(g_j), q^_j = quat(y_p, y_h) / |q_j| (1 when q_j = 0), tau(quat(al, be))
// = quat(al, -be) = k g k^-1 with k = i sigma_z = quat(i, 0).  Hence g_j =
// x_{j-1} .. x_1 x_0 k^-j with x_i = q^_i k: a prefix product of unit
// quaternions (per-thread chunks, then a Hillis-Steele scan of the chunk
// totals in LDS, later factors on the left), k^-j = quat((-i)^j, 0).  The
// rotated diagonal blocks g^H [[a, d], [conj d, -a]] g -> (ra, rd), b_j =
// |q_j|; g as (al, be) per site in G[2 s], G[2 s + 1].
constexpr int kQRotT = 1024;
__global__ __launch_bounds__(kQRotT) void k_q_rot(const double* __restrict__ qa, const double2* __restrict__ qd,
                                                  const double2* __restrict__ Y, int M, double* __restrict__ ra,
                                                  double2* __restrict__ rd, double* __restrict__ rb,
                                                  double2* __restrict__ G) {
  const int k = blockIdx.x, t = threadIdx.x;
  qa += (int64_t)k * M;
  qd += (int64_t)k * M;
  Y += (int64_t)k * 2 * M;
  ra += (int64_t)k * M;
  rd += (int64_t)k * M;
  rb += (int64_t)k * M;
  G += (int64_t)k * 2 * M;
  __shared__ double2 sa[2][kQRotT], sb[2][kQRotT];
  const int ne = M - 1, per = (ne + kQRotT - 1) / kQRotT, i0 = t * per;
  double2 la[kQMaxR], lb[kQMaxR];
  double nq[kQMaxR];
  double2 ta = make_double2(1.0, 0.0), tb = make_double2(0.0, 0.0);   // the chunk's product
#pragma unroll
  for (int u = 0; u < kQMaxR; ++u) {
    const int i = i0 + u;
    nq[u] = 0.0;
    if (u < per && i < ne) {
      const double2 yp = Y[2 * i], yh = Y[2 * i + 1];
      const double q2 = yp.x * yp.x + yp.y * yp.y + yh.x * yh.x + yh.y * yh.y;
      nq[u] = sqrt(q2);
      double2 xa = make_double2(1.0, 0.0), xb = make_double2(0.0, 0.0);
      if (nq[u] > 0.0) {
        const double iv = 1.0 / nq[u];
        xa = make_double2(yp.x * iv, yp.y * iv);
        xb = make_double2(yh.x * iv, yh.y * iv);
      }
      // x = q^ k = quat(i al, i be)
      xa = make_double2(-xa.y, xa.x);
      xb = make_double2(-xb.y, xb.x);
      double2 na, nb;
      qmul(xa, xb, ta, tb, na, nb);   // later factor on the left
      ta = na;
      tb = nb;
    }
    la[u] = ta;
    lb[u] = tb;
  }
  // inclusive scan of the chunk totals over the threads (ping-pong buffers)
  int cur = 0;
  sa[0][t] = ta;
  sb[0][t] = tb;
  __syncthreads();
  for (int d = 1; d < kQRotT; d <<= 1) {
    double2 va = sa[cur][t], vb = sb[cur][t];
    if (t >= d) {
      double2 na, nb;
      qmul(va, vb, sa[cur][t - d], sb[cur][t - d], na, nb);
      va = na;
      vb = nb;
    }
    sa[cur ^ 1][t] = va;
    sb[cur ^ 1][t] = vb;
    cur ^= 1;
    __syncthreads();
  }
  const double2 ea = t > 0 ? sa[cur][t - 1] : make_double2(1.0, 0.0);   // product of the earlier chunks
  const double2 eb = t > 0 ? sb[cur][t - 1] : make_double2(0.0, 0.0);
  auto site = [&](int s, double2 al, double2 be, double b) {
    // renormalise, then D' = g^H D g, g = [[al, -conj be], [be, conj al]], D = [[a, d], [conj d, -a]]
    const double nn = 1.0 / sqrt(al.x * al.x + al.y * al.y + be.x * be.x + be.y * be.y);
    al = make_double2(al.x * nn, al.y * nn);
    be = make_double2(be.x * nn, be.y * nn);
    G[2 * s] = al;
    G[2 * s + 1] = be;
    const double a = qa[s];
    const double2 d = qd[s];
    const double2 c00 = make_double2(a * al.x + (d.x * be.x - d.y * be.y), a * al.y + (d.x * be.y + d.y * be.x));
    const double2 c10 = make_double2((d.x * al.x + d.y * al.y) - a * be.x, (d.x * al.y - d.y * al.x) - a * be.y);
    const double2 nbe = make_double2(-be.x, be.y), cal = make_double2(al.x, -al.y);   // -conj be, conj al
    const double2 c01 = make_double2(a * nbe.x + (d.x * cal.x - d.y * cal.y), a * nbe.y + (d.x * cal.y + d.y * cal.x));
    const double2 c11 = make_double2((d.x * nbe.x + d.y * nbe.y) - a * cal.x, (d.x * nbe.y - d.y * nbe.x) - a * cal.y);
    ra[s] = (al.x * c00.x + al.y * c00.y) + (be.x * c10.x + be.y * c10.y);
    rd[s] = make_double2((al.x * c01.x + al.y * c01.y) + (be.x * c11.x + be.y * c11.y),
                         (al.x * c01.y - al.y * c01.x) + (be.x * c11.y - be.y * c11.x));
    rb[s] = b;
  };
  if (t == 0) site(0, make_double2(1.0, 0.0), make_double2(0.0, 0.0), ne > 0 ? nq[0] : 0.0);
#pragma unroll
  for (int u = 0; u < kQMaxR; ++u) {
    const int i = i0 + u;
    if (u < per && i < ne) {
      double2 pa, pb;
      qmul(la[u], lb[u], ea, eb, pa, pb);   // P_{i+1} = x_i .. x_0
      // g_{i+1} = P_{i+1} k^-(i+1) = quat(pa c, pb c), c = (-i)^(i+1)
      const int j = (i + 1) & 3;
      const double2 c = j == 0 ? make_double2(1.0, 0.0)
                        : j == 1 ? make_double2(0.0, -1.0)
                        : j == 2 ? make_double2(-1.0, 0.0) : make_double2(0.0, 1.0);
      const double2 al = make_double2(pa.x * c.x - pa.y * c.y, pa.x * c.y + pa.y * c.x);
      const double2 be = make_double2(pb.x * c.x - pb.y * c.y, pb.x * c.y + pb.y * c.x);
      const double bn = i + 1 < ne ? (u + 1 < per ? nq[u + 1] : 0.0) : 0.0;
      site(i + 1, al, be, bn);
    }
  }
  // b of the sites whose q lives in the next thread's chunk
  if (per > 0 && i0 + per - 1 < ne && i0 + per < ne) {
    const double2 yp = Y[2 * (i0 + per)], yh = Y[2 * (i0 + per) + 1];
    rb[i0 + per] = sqrt(yp.x * yp.x + yp.y * yp.y + yh.x * yh.x + yh.y * yh.y);
  }
}

// Eigenvalues of T by G-lane multisection on block Sturm counts (as
// k_eig_bisect): S_0 = D_0 - x, S_{s+1} = D_{s+1} - x - b_s^2 sigma_z S_s^-1
// sigma_z; S = [[p, q], [conj q, r]] contributes 1 negative eigenvalue when
// det < 0, 2 when det > 0 and p < 0.  A determinant below pivmin = (eps
// ||T||)^2 is replaced by -pivmin (keeps b^2 / det and the next determinant
// finite).  LDS: one record (a', d' re, d' im, b^2) per site.
#ifndef QBIS_W
#define QBIS_W 4
#endif
constexpr int kQBisW = QBIS_W;   // waves per bisection workgroup
constexpr int kQBisPad = 8;   // Sturm sweep block (sites); zero records past M
__global__ __launch_bounds__(64 * kQBisW) void k_q_bisect(const double* __restrict__ ra, const double2* __restrict__ rd,
                                                          const double* __restrict__ rb, int M, int lgG, int jofs,
                                                          double* __restrict__ E, double* __restrict__ tnorm) {
  extern __shared__ double lds[];
  const int k = blockIdx.y, lane = threadIdx.x & 63, n = 2 * M;
  ra += (int64_t)k * M;
  rd += (int64_t)k * M;
  rb += (int64_t)k * M;
  E += (int64_t)k * n;
  __shared__ double shn[kQBisW];
  double tl = 0.0;
  // one 32-byte record per site: a, d (re, im), b^2 (b_{M-1} = 0); zero
  // records past M (kQBisPad) so the blocked sweep reads without bounds checks
  double4* rec = reinterpret_cast<double4*>(lds);
  for (int s = threadIdx.x; s < M + kQBisPad; s += blockDim.x) {
    if (s >= M) {
      rec[s] = make_double4(0.0, 0.0, 0.0, 0.0);
      continue;
    }
    const double a = ra[s];
    const double2 d = rd[s];
    const double bl = s > 0 ? rb[s - 1] : 0.0, br = s + 1 < M ? rb[s] : 0.0;
    rec[s] = make_double4(a, d.x, d.y, br * br);
    tl = fmax(tl, fabs(a) + sqrt(d.x * d.x + d.y * d.y) + fabs(bl) + fabs(br));
  }
  for (int off = 32; off > 0; off >>= 1) tl = fmax(tl, __shfl_xor(tl, off, 64));
  if (lane == 0) shn[threadIdx.x >> 6] = tl;
  __syncthreads();
  double tn = 0.0;
  for (int w = 0; w < kQBisW; ++w) tn = fmax(tn, shn[w]);
  if (blockIdx.x == 0 && threadIdx.x == 0) tnorm[k] = tn;
  // (jofs > 0: the upper half of a spectrum symmetric about 0 lies in [0, ||T||])
  const double gl = jofs > 0 ? -1e-300 : -tn * (1.0 + 4.0 * DBL_EPSILON) - 1e-300,
               gu = tn * (1.0 + 4.0 * DBL_EPSILON) + 1e-300;
  const double pivmin = (DBL_EPSILON * tn) * (DBL_EPSILON * tn) + DBL_MIN;
  const int G = 1 << lgG, g0 = lane & ~(G - 1), gi = lane & (G - 1);
  // indices jofs .. n-1; (jofs > 0) the lower half mirrored: the spectrum of
  // T is symmetric (particle-hole), E_{n-1-j} = -E_j
  const int j = jofs + ((blockIdx.x * kQBisW + (threadIdx.x >> 6)) << (6 - lgG)) + (lane >> lgG);
  if (jofs + ((blockIdx.x * kQBisW + (threadIdx.x >> 6)) << (6 - lgG)) >= n) return;
  const unsigned long long gmask = G == 64 ? ~0ull : ((1ull << G) - 1);
  const double step = 1.0 / (G + 1);
  double lo = gl, hi = gu;
  bool done = j >= n;
  for (int it = 0; it < 256; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (mid <= lo || mid >= hi) done = true;
    if (__ballot(!done) == 0) break;
    const double x = fmin(lo + (gi + 1) * ((hi - lo) * step), hi);
    const double4 r0s = rec[0];
    double p = r0s.x - x, qr = r0s.y, qi = r0s.z, r = -r0s.x - x;
    int c = 0;
    // blocks of kQBisPad sites, the block's records read up front (one LDS
    // wait per block, not one per site on the chain); past M the records are
    // zero (b^2 = 0: no coupling) and the counts are masked
    for (int s0 = 0; s0 < M; s0 += kQBisPad) {
      double4 rr[kQBisPad + 1];
#pragma unroll
      for (int u = 0; u <= kQBisPad; ++u) rr[u] = rec[s0 + u];
#pragma unroll
      for (int u = 0; u < kQBisPad; ++u) {
        double det = p * r - (qr * qr + qi * qi);
        if (fabs(det) < pivmin) det = -pivmin;
        c += s0 + u < M ? (det < 0.0 ? 1 : (p < 0.0 ? 2 : 0)) : 0;
        const double q0 = __builtin_amdgcn_rcp(det);
        const double rq = fma(q0, fma(-det, q0, 1.0), q0);
        const double f = rr[u].w * rq;
        const double a1 = rr[u + 1].x;
        const double np = (a1 - x) - f * r, nr = (-a1 - x) - f * p;
        qr = rr[u + 1].y - f * qr;
        qi = rr[u + 1].z - f * qi;
        p = np;
        r = nr;
      }
    }
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
  if (gi == 0 && j < n) {
    const double e = 0.5 * (lo + hi);
    E[j] = e;
    if (jofs > 0) E[n - 1 - j] = -e;
  }
}

// ---------------------------------------------------------------------------
// Eigenvectors of the particle-hole half (indices j0 .. n-1 of E, nv = n - j0)
// ---------------------------------------------------------------------------

// entry (r, c) of T - lam in the interleaved site order (row 2s: particle of
// site s, 2s+1: hole): row 2s = b_{s-1} @ 2s-2, a_s - lam @ 2s, d_s @ 2s+1,
// b_s @ 2s+2; row 2s+1 = -b_{s-1} @ 2s-1, conj d_s @ 2s, -a_s - lam @ 2s+1,
// -b_s @ 2s+3.  T's arrays in LDS: a [0, M), b [M, 2M), d [2M, 4M) (re, im).
__device__ __forceinline__ double2 q_tent(const double* L, int M, double lam, int r, int c) {
  const int n = 2 * M;
  if (r >= n || c < 0 || c >= n) return make_double2(0.0, 0.0);
  const int s = r >> 1, dc = c - r;
  const bool hole = r & 1;
  if (dc == 0) return make_double2(hole ? -L[s] - lam : L[s] - lam, 0.0);
  if (dc == 2 && s + 1 < M) return make_double2(hole ? -L[M + s] : L[M + s], 0.0);
  if (dc == -2 && s > 0) return make_double2(hole ? -L[M + s - 1] : L[M + s - 1], 0.0);
  if (!hole && dc == 1) return make_double2(L[2 * M + 2 * s], L[2 * M + 2 * s + 1]);
  if (hole && dc == -1) return make_double2(L[2 * M + 2 * s], -L[2 * M + 2 * s + 1]);
  return make_double2(0.0, 0.0);
}

// start vector entry (a fixed pseudo-random value in [-1/2, 1/2) per
// (eigenvalue index, component): a 32-bit integer hash, cheap inside the sweep)
__device__ __forceinline__ double q_start(int j, int r) {
  unsigned h = (unsigned)r * 0x9E3779B1u ^ (unsigned)j * 0x85EBCA6Bu;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return (double)h * 0x1.0p-32 - 0.5;
}

__device__ __forceinline__ double2 cmul2(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 csub2(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// Inverse iteration, one eigenvalue per thread (tools/qeig_proto.py
// band_solve_pivoted): T - lam = P L U with partial pivoting over the three
// rows that reach column k (lower bandwidth 2, so U's rows carry columns
// k .. k+4; a pivot below eps ||T|| is clamped), the eliminated right-hand
// side in the same sweep; per step six complex (1/u_kk, u_k,k+1..k+4, y_k)
// into the scratch S[(k 6 + e) nv + jj] (coalesced over the threads), then the
// back substitution.  Two solves from a fixed pseudo-random start (lam is
// bisected to the last bit), normalised: vector jj in Zt[r nv + jj] (row r
// in the interleaved order).
__global__ __launch_bounds__(64) void k_q_invit(const double* __restrict__ ra, const double2* __restrict__ rd,
                                                const double* __restrict__ rb, int M, const double* __restrict__ E,
                                                const double* __restrict__ tnorm, int j0, double2* __restrict__ Zt,
                                                int64_t sZ, double2* __restrict__ S, int64_t sS) {
  extern __shared__ double lds[];
  const int k = blockIdx.y, n = 2 * M, nv = n - j0;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    lds[i] = ra[(int64_t)k * M + i];
    lds[M + i] = rb[(int64_t)k * M + i];
    const double2 dv = rd[(int64_t)k * M + i];
    lds[2 * M + 2 * i] = dv.x;
    lds[2 * M + 2 * i + 1] = dv.y;
  }
  __syncthreads();
  const int jj = blockIdx.x * blockDim.x + threadIdx.x;
  if (jj >= nv) return;
  const double tn = tnorm[k];
  // A member of a cluster (a neighbour within kEigClusterTol ||T||) is solved
  // at e - kQClusterShift ||T||: for an exactly degenerate level the members'
  // bisected values differ by ulps, and solving at them weights the
  // eigenspace's directions by 1 / (E_i - e) — ratios of 10..1000, so the
  // vectors turn nearly parallel and k_q_orth's Cholesky QR amplifies their
  // out-of-cluster rounding by as much (clean 10 x 10: residual 3e-13,
  // 1.5e-12 against the Theta partners).  A shift far above the ulp spread
  // and far below the gap to the next level weights the eigenspace evenly.
  const double* Ek = E + (int64_t)k * n;
  const double e = Ek[j0 + jj];
  const double ctol = kEigClusterTol * tn;
  const bool member = (jj > 0 && e - Ek[j0 + jj - 1] <= ctol) || (j0 + jj + 1 < n && Ek[j0 + jj + 1] - e <= ctol);
  const double lam = member ? e - kQClusterShift * tn : e;
  const double small = tn > 0.0 ? DBL_EPSILON * tn : DBL_EPSILON;
  double2* z = Zt + k * sZ + jj;
  double2* sc = S + k * sS + jj;
  const double2 zero = make_double2(0.0, 0.0);
  double scale = 1.0;
  for (int it = 0; it < QINVIT_ITERS; ++it) {
    auto rhs = [&](int r) -> double2 {
      if (r >= n) return zero;
      if (it == 0) return make_double2(q_start(j0 + jj, 2 * r), q_start(j0 + jj, 2 * r + 1));
      const double2 v = z[(int64_t)r * nv];
      return make_double2(v.x * scale, v.y * scale);
    };
    double2 w0[5], w1[5], w2[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      w0[c] = q_tent(lds, M, lam, 0, c);
      w1[c] = q_tent(lds, M, lam, 1, c);
      w2[c] = q_tent(lds, M, lam, 2, c);
    }
    double2 y0 = rhs(0), y1 = rhs(1), y2 = rhs(2);
    double nb2 = (y0.x * y0.x + y0.y * y0.y) + (y1.x * y1.x + y1.y * y1.y) + (y2.x * y2.x + y2.y * y2.y);
    // one elimination step (row kk leaves the window into the scratch)
    // hole: the parity of row kk+3 (a compile-time constant in the unrolled sweep)
    auto step = [&](int kk, bool hole, double2 ny) {
      // the next window row: row r = kk+3 at columns r-2 .. r+2, branch-free
      //   particle (s = r/2): [ b_{s-1}, 0, a_s - lam, d_s, b_s ]
      //   hole:               [ -b_{s-1}, conj d_s, -a_s - lam, 0, -b_s ]
      // (b_{M-1} = 0 from k_q_rot; rows past n are zero)
      double2 nr[5];
      {
        const int r = kk + 3, sr = min(r >> 1, M - 1);
        const double on = r < n ? 1.0 : 0.0, sg = hole ? -on : on;
        const double as = lds[sr], bs = lds[M + sr], bm = lds[M + sr - 1];
        const double dr = lds[2 * M + 2 * sr], di = lds[2 * M + 2 * sr + 1];
        nr[0] = make_double2(sg * bm, 0.0);
        nr[1] = hole ? make_double2(on * dr, -on * di) : zero;
        nr[2] = make_double2(sg * as - on * lam, 0.0);
        nr[3] = hole ? zero : make_double2(on * dr, on * di);
        nr[4] = make_double2(sg * bs, 0.0);
      }
      const double m0 = w0[0].x * w0[0].x + w0[0].y * w0[0].y;
      const double m1 = w1[0].x * w1[0].x + w1[0].y * w1[0].y;
      const double m2 = w2[0].x * w2[0].x + w2[0].y * w2[0].y;
      const int sel = m1 > m0 ? (m2 > m1 ? 2 : 1) : (m2 > m0 ? 2 : 0);
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        const double2 p0 = w0[c], p1 = w1[c], p2 = w2[c];
        w0[c] = sel == 0 ? p0 : (sel == 1 ? p1 : p2);
        w1[c] = sel == 1 ? p0 : p1;
        w2[c] = sel == 2 ? p0 : p2;
      }
      {
        const double2 q0 = y0, q1 = y1, q2 = y2;
        y0 = sel == 0 ? q0 : (sel == 1 ? q1 : q2);
        y1 = sel == 1 ? q0 : q1;
        y2 = sel == 2 ? q0 : q2;
      }
      double pm = w0[0].x * w0[0].x + w0[0].y * w0[0].y;
      if (pm < small * small) {
        w0[0] = make_double2(small, 0.0);
        pm = small * small;
      }
      const double ip = rcp_nr(pm);
      const double2 r = make_double2(w0[0].x * ip, -w0[0].y * ip);   // 1 / u_kk
      const double2 f1 = cmul2(w1[0], r), f2 = cmul2(w2[0], r);
#pragma unroll
      for (int c = 1; c < 5; ++c) {
        w1[c] = csub2(w1[c], cmul2(f1, w0[c]));
        w2[c] = csub2(w2[c], cmul2(f2, w0[c]));
      }
      y1 = csub2(y1, cmul2(f1, y0));
      y2 = csub2(y2, cmul2(f2, y0));
      double2* st = sc + (int64_t)kk * 6 * nv;
      st[0] = r;
#pragma unroll
      for (int c = 1; c < 5; ++c) st[(int64_t)c * nv] = w0[c];
      st[(int64_t)5 * nv] = y0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        w0[c] = w1[c + 1];
        w1[c] = w2[c + 1];
      }
      w0[4] = w1[4] = zero;
#pragma unroll
      for (int c = 0; c < 5; ++c) w2[c] = nr[c];
      y0 = y1;
      y1 = y2;
      y2 = ny;
      nb2 += ny.x * ny.x + ny.y * ny.y;
    };
    // forward sweep in blocks of FB steps, the next block's right-hand side
    // rows loaded one block ahead (a load's wait then only covers loads and
    // stores issued before it, not this block's scratch stores)
    constexpr int FB = 4;
    double2 ra_[FB], rb_[FB];
#pragma unroll
    for (int u = 0; u < FB; ++u) ra_[u] = rhs(3 + u);
    for (int k0 = 0; k0 < n; k0 += 2 * FB) {
#pragma unroll
      for (int u = 0; u < FB; ++u) rb_[u] = rhs(k0 + FB + 3 + u);
#pragma unroll
      for (int u = 0; u < FB; ++u)
        if (k0 + u < n) step(k0 + u, (u + 1) & 1, ra_[u]);
#pragma unroll
      for (int u = 0; u < FB; ++u) ra_[u] = rhs(k0 + 2 * FB + 3 + u);
#pragma unroll
      for (int u = 0; u < FB; ++u)
        if (k0 + FB + u < n) step(k0 + FB + u, (FB + u + 1) & 1, rb_[u]);
    }
    // back substitution: x_k = (y_k - sum_t u_k,k+t x_{k+t}) / u_kk, the next
    // block's factors loaded one block ahead
    double2 x1 = zero, x2 = zero, x3 = zero, x4 = zero;
    double nrm = 0.0;
    constexpr int PB = 4;
    double2 fa[PB][6], fb[PB][6];
    auto load_blk = [&](int k0, double2 (&f)[PB][6]) {
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int kk = k0 - u;
#pragma unroll
        for (int e = 0; e < 6; ++e) f[u][e] = kk >= 0 ? sc[((int64_t)kk * 6 + e) * nv] : zero;
      }
    };
    auto solve_blk = [&](int k0, const double2 (&f)[PB][6]) {
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int kk = k0 - u;
        if (kk >= 0) {
          double2 t = f[u][5];
          t = csub2(t, cmul2(f[u][1], x1));
          t = csub2(t, cmul2(f[u][2], x2));
          t = csub2(t, cmul2(f[u][3], x3));
          t = csub2(t, cmul2(f[u][4], x4));
          const double2 x = cmul2(t, f[u][0]);
          z[(int64_t)kk * nv] = x;
          nrm += x.x * x.x + x.y * x.y;
          x4 = x3;
          x3 = x2;
          x2 = x1;
          x1 = x;
        }
      }
    };
    load_blk(n - 1, fa);
    for (int k0 = n - 1; k0 >= 0; k0 -= 2 * PB) {
      load_blk(k0 - PB, fb);
      solve_blk(k0, fa);
      load_blk(k0 - 2 * PB, fa);
      solve_blk(k0 - PB, fb);
    }
    scale = 1.0 / sqrt(nrm);
    // a second solve only where the first may not have converged: the growth
    // g = |x| / |b| bounds the other eigenvectors' share of x by 1 / (g gap)
    // (gap: to the nearest other eigenvalue); above kQInvitShare (a start
    // vector nearly orthogonal to the eigenvector, or a small gap) the wave
    // solves again from x.  Below it the Löwdin step leaves O(share^2): L = 32
    // disordered, one solve everywhere, residual 5e-15 ||H||, orthogonality
    // 4e-14 (two solves: 7e-16, 3e-15; profiles/r06_qeig_eigensystem.txt)
    if (it == 0 && QINVIT_ITERS > 1) {
      const int jg = j0 + jj;
      double gap = DBL_MAX;
      // (the lowest computed vector's lower neighbour -lam is its own
      // partner's eigenvalue: a share of Theta u in x only rotates the pair
      // x, Theta x inside their exactly orthogonal plane, by ~1 / (g 2 lam),
      // which moves the residual by ~1 / g)
      if (jg > j0) gap = fmin(gap, e - Ek[jg - 1]);
      if (jg + 1 < n) gap = fmin(gap, Ek[jg + 1] - e);
      const double g = sqrt(nrm / nb2);
      const bool need = !(g * gap * kQInvitShare > 1.0);
      if (__ballot(need) == 0) break;
    }
  }
  for (int r = 0; r < n; ++r) {
    const double2 v = z[(int64_t)r * nv];
    z[(int64_t)r * nv] = make_double2(v.x * scale, v.y * scale);
  }
}

// The same inverse iteration with one 16-lane DPP row per eigenvalue (four
// per one-wave workgroup, which leaves the back substitution's prefetch its
// 512 registers): lanes 0..4 hold column c = lane of the three window
// rows, lane 12 the right-hand side's three window entries, the others zeros
// (lane 5: what column 4 shifts in; lane 8: what lane 7 shifts in, so no
// right-hand side value walks down into the columns).  Per step lane 0 picks the pivot row (row_newbcast),
// forms 1 / u_kk and the two multipliers (row_newbcast to the row), every
// lane eliminates its own entries, one store per lane writes the step's six
// complex (lane 0: 1 / u_kk, lanes 1..4: u_k,k+c, lane 12: y_k; the scratch
// layout of k_q_invit), and the window moves one column by row_shl:1 with the
// banks of lanes 8..15 masked (the right-hand side lane shifts its own
// entries).  The thread-per-eigenvalue sweep issued ~385 instructions per
// step on one wave per SIMD; this one ~100, on 16x the waves.  The back
// substitution runs redundantly in all 16 lanes of a row (same addresses:
// one transaction), lane 0 storing.  Same operation order as k_q_invit per
// eigenvalue, so the same vectors up to the order of the pivot magnitudes'
// sums (identical).
// f(integral_constant<int, U>) for U = 0 .. 15 (compile-time DPP controls)
template <int U = 0, class F>
__device__ __forceinline__ void q_unroll16(F&& f) {
  if constexpr (U < 16) {
    f(std::integral_constant<int, U>{});
    q_unroll16<U + 1>(f);
  }
}
__device__ __forceinline__ double2 dpp_bcast0(double2 v) {
  return make_double2(__builtin_amdgcn_update_dpp(v.x, v.x, 0x150, 0xf, 0xf, true),
                      __builtin_amdgcn_update_dpp(v.y, v.y, 0x150, 0xf, 0xf, true));
}
// lanes 0..7 of each row take lane + 1's value (lane 7: lane 8's, unused);
// lanes 8..15 keep their own (bank mask 0b0011)
__device__ __forceinline__ double2 dpp_shl1_lo(double2 v) {
  return make_double2(__builtin_amdgcn_update_dpp(v.x, v.x, 0x101, 0xf, 0x3, true),
                      __builtin_amdgcn_update_dpp(v.y, v.y, 0x101, 0xf, 0x3, true));
}

__global__ __launch_bounds__(64) void k_q_invit16(const double* __restrict__ ra, const double2* __restrict__ rd,
                                                   const double* __restrict__ rb, int M, const double* __restrict__ E,
                                                   const double* __restrict__ tnorm, int j0, double2* __restrict__ Zt,
                                                   int64_t sZ, double2* __restrict__ S, int64_t sS) {
  extern __shared__ double lds[];
  const int k = blockIdx.y, n = 2 * M, nv = n - j0;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    lds[i] = ra[(int64_t)k * M + i];
    lds[M + i] = rb[(int64_t)k * M + i];
    const double2 dv = rd[(int64_t)k * M + i];
    lds[2 * M + 2 * i] = dv.x;
    lds[2 * M + 2 * i + 1] = dv.y;
  }
  __syncthreads();
  const int l = threadIdx.x & 15;
  const int jj = blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);
  if (jj >= nv) return;   // whole 16-lane rows (DPP rows) leave together
  const double tn = tnorm[k];
  const double* Ek = E + (int64_t)k * n;
  const double e = Ek[j0 + jj];
  const double ctol = kEigClusterTol * tn;
  const bool member = (jj > 0 && e - Ek[j0 + jj - 1] <= ctol) || (j0 + jj + 1 < n && Ek[j0 + jj + 1] - e <= ctol);
  const double lam = member ? e - kQClusterShift * tn : e;   // (k_q_invit)
  const double small = tn > 0.0 ? DBL_EPSILON * tn : DBL_EPSILON;
  double2* z = Zt + k * sZ + jj;
  double2* sc = S + k * sS + jj;
  const double2 zero = make_double2(0.0, 0.0);
  const bool ylane = l == 12;
  // this lane's share of a new row [b_{s-1}, (hole) conj d, a - lam, (particle) d, b_s]
  const double c0 = l == 0 ? 1.0 : 0.0, c1 = l == 1 ? 1.0 : 0.0, c2 = l == 2 ? 1.0 : 0.0, c3 = l == 3 ? 1.0 : 0.0,
               c4 = l == 4 ? 1.0 : 0.0;
  // scratch entry of this lane's store: 0 (1/u_kk), 1..4 (u), 5 (y); others none
  const int est = l < 5 ? l : 5;
  const bool stl = l < 5 || ylane;
  double scale = 1.0;
  for (int it = 0; it < QINVIT_ITERS; ++it) {
    auto rhs = [&](int r) -> double2 {
      if (r >= n) return zero;
      if (it == 0) return make_double2(q_start(j0 + jj, 2 * r), q_start(j0 + jj, 2 * r + 1));
      const double2 v = z[(int64_t)r * nv];
      return make_double2(v.x * scale, v.y * scale);
    };
    double2 w0, w1, w2;
    if (ylane) {
      w0 = rhs(0);
      w1 = rhs(1);
      w2 = rhs(2);
    } else {
      w0 = l < 5 ? q_tent(lds, M, lam, 0, l) : zero;
      w1 = l < 5 ? q_tent(lds, M, lam, 1, l) : zero;
      w2 = l < 5 ? q_tent(lds, M, lam, 2, l) : zero;
    }
    double nb2 = (w0.x * w0.x + w0.y * w0.y) + (w1.x * w1.x + w1.y * w1.y) + (w2.x * w2.x + w2.y * w2.y);
    auto step = [&](int kk, bool hole, double2 ny) {
      // pivot row: lane 0's magnitudes (ties resolved as in k_q_invit)
      const double m0 = w0.x * w0.x + w0.y * w0.y;
      const double m1 = w1.x * w1.x + w1.y * w1.y;
      const double m2 = w2.x * w2.x + w2.y * w2.y;
      const int sel0 = m1 > m0 ? (m2 > m1 ? 2 : 1) : (m2 > m0 ? 2 : 0);
      const int sel = __builtin_amdgcn_update_dpp(sel0, sel0, 0x150, 0xf, 0xf, true);
      {
        // the row swap by 0/1 weights (exact for finite entries): a select
        // chain on the broadcast index became a dynamically indexed stack
        // array (scratch round trips on the pivot chain)
        const double s1 = sel == 1 ? 1.0 : 0.0, s2 = sel == 2 ? 1.0 : 0.0, s0 = 1.0 - s1 - s2;
        const double2 p0 = w0, p1 = w1, p2 = w2;
        w0 = make_double2(fma(s2, p2.x, fma(s1, p1.x, s0 * p0.x)), fma(s2, p2.y, fma(s1, p1.y, s0 * p0.y)));
        w1 = make_double2(fma(s1, p0.x, (1.0 - s1) * p1.x), fma(s1, p0.y, (1.0 - s1) * p1.y));
        w2 = make_double2(fma(s2, p0.x, (1.0 - s2) * p2.x), fma(s2, p0.y, (1.0 - s2) * p2.y));
      }
      // lane 0: 1 / u_kk and the multipliers
      // (branch-free, component-wise: a branch or a select of whole double2
      // values here also became a stack array)
      double pm = w0.x * w0.x + w0.y * w0.y;
      const bool tiny = l == 0 && pm < small * small;   // the pivot only (lane 0)
      w0.x = tiny ? small : w0.x;
      w0.y = tiny ? 0.0 : w0.y;
      pm = tiny ? small * small : pm;
      const double ip = rcp_nr(pm);
      const double2 r = make_double2(w0.x * ip, -w0.y * ip);   // 1 / u_kk (lane 0)
      const double2 f1 = dpp_bcast0(cmul2(w1, r)), f2 = dpp_bcast0(cmul2(w2, r));
      // the step's row of U (and y_k) before the update (lane 0: 1 / u_kk)
      const double2 sv = make_double2(l == 0 ? r.x : w0.x, l == 0 ? r.y : w0.y);
      if (stl) sc[((int64_t)kk * 6 + est) * nv] = sv;
      w1 = csub2(w1, cmul2(f1, w0));
      w2 = csub2(w2, cmul2(f2, w0));
      // the window moves one column (the right-hand side lane: one row)
      w0 = dpp_shl1_lo(w1);
      w1 = dpp_shl1_lo(w2);
      // the next window row r = kk + 3 (k_q_invit's row formula, this lane's column)
      const int rr = kk + 3, sr = min(rr >> 1, M - 1);
      const double on = rr < n ? 1.0 : 0.0, sg = hole ? -on : on;
      const double as = lds[sr], bs = lds[M + sr], bm = lds[M + sr - 1];
      const double dr = lds[2 * M + 2 * sr], di = lds[2 * M + 2 * sr + 1];
      const double cd = hole ? c1 : c3;
      const double2 nr = make_double2(sg * (c0 * bm + c2 * as + c4 * bs) - c2 * on * lam + cd * on * dr,
                                      (hole ? -cd : cd) * on * di);
      w2 = make_double2(ylane ? ny.x : nr.x, ylane ? ny.y : nr.y);
      nb2 += ny.x * ny.x + ny.y * ny.y;
    };
    // the right-hand side's rows 16 at a time, one per lane (lane l: row
    // k0 + 3 + l, the next 16 loaded a block ahead), each step's row reaching
    // the row's lanes by row_newbcast: one hash or load per 16 steps and lane
    // instead of one per step in every lane
    double2 rv = rhs(3 + l);
    for (int k0 = 0; k0 < n; k0 += 16) {
      const double2 rn = rhs(k0 + 16 + 3 + l);
      q_unroll16([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const double2 ny = make_double2(__builtin_amdgcn_update_dpp(rv.x, rv.x, 0x150 + u, 0xf, 0xf, true),
                                        __builtin_amdgcn_update_dpp(rv.y, rv.y, 0x150 + u, 0xf, 0xf, true));
        if (k0 + u < n) step(k0 + u, (u + 1) & 1, ny);
      });
      rv = rn;
    }
    nb2 = __builtin_amdgcn_update_dpp(nb2, nb2, 0x15C, 0xf, 0xf, true);   // lane 12's (row_newbcast:12)
    // the scratch stores of the row's other lanes before its reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // back substitution (every lane of the row the same; lane 0 stores x)
    double2 x1 = zero, x2 = zero, x3 = zero, x4 = zero;
    double nrm = 0.0;
    constexpr int PB = 4;
    double2 fa[PB][6], fb[PB][6];
    auto load_blk = [&](int k0, double2 (&f)[PB][6]) {
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int kk = k0 - u;
#pragma unroll
        for (int q = 0; q < 6; ++q) f[u][q] = kk >= 0 ? sc[((int64_t)kk * 6 + q) * nv] : zero;
      }
    };
    auto solve_blk = [&](int k0, const double2 (&f)[PB][6]) {
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int kk = k0 - u;
        if (kk >= 0) {
          double2 t = f[u][5];
          t = csub2(t, cmul2(f[u][1], x1));
          t = csub2(t, cmul2(f[u][2], x2));
          t = csub2(t, cmul2(f[u][3], x3));
          t = csub2(t, cmul2(f[u][4], x4));
          const double2 x = cmul2(t, f[u][0]);
          if (l == 0) z[(int64_t)kk * nv] = x;
          nrm += x.x * x.x + x.y * x.y;
          x4 = x3;
          x3 = x2;
          x2 = x1;
          x1 = x;
        }
      }
    };
    load_blk(n - 1, fa);
    for (int k0 = n - 1; k0 >= 0; k0 -= 2 * PB) {
      load_blk(k0 - PB, fb);
      solve_blk(k0, fa);
      load_blk(k0 - 2 * PB, fa);
      solve_blk(k0 - PB, fb);
    }
    scale = 1.0 / sqrt(nrm);
    if (it == 0 && QINVIT_ITERS > 1) {   // (k_q_invit's test)
      const int jg = j0 + jj;
      double gap = DBL_MAX;
      if (jg > j0) gap = fmin(gap, e - Ek[jg - 1]);
      if (jg + 1 < n) gap = fmin(gap, Ek[jg + 1] - e);
      const double g = sqrt(nrm / nb2);
      const bool need = !(g * gap * kQInvitShare > 1.0);
      if (__ballot(need) == 0) break;
      // lane 0's z stores before the right-hand side lane reads them
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (l == 0)
    for (int r = 0; r < n; ++r) {
      const double2 v = z[(int64_t)r * nv];
      z[(int64_t)r * nv] = make_double2(v.x * scale, v.y * scale);
    }
}

// The crowd at zero: when E_N + E_{N+1} <= kEigZeroTol ||T|| (j0 = N), the
// levels j0 .. j0 + c - 1 with E_j + E_N within it (extended over cluster
// gaps): their vectors x_j overlap the partners Theta x_k of one another (by
// ~eps ||T|| / (E_j + E_k)), which the Löwdin step over the x's cannot see.
// 0 when there is none.  The same function on the host (q_zero_crowd) and in
// k_q_orth, so both see the same c.
__host__ __device__ inline int q_crowd(const double* E, int n, int j0, double tn) {
  const int nv = n - j0;
  const double zt = kEigZeroTol * tn, ct = kEigClusterTol * tn;
  if (nv < 2 || E[j0] + E[j0 + 1] > zt) return 0;
  int c = 2;
  while (c < nv && (E[j0 + c] + E[j0] <= zt || E[j0 + c] - E[j0 + c - 1] <= ct)) ++c;
  return c;
}

// Clusters of the computed eigenvalues (consecutive gaps <= ctol ||T||, at
// most kQMaxCluster long: longer ones are declined on the host) get their
// inverse-iteration vectors orthonormalised, as k_eig_orth does for the
// one-stage solver's real vectors: two rounds of Cholesky QR on the
// cluster's columns of Zt (G = Z^H Z = L L^H, Z <- Z L^-H; a cluster's
// columns are contiguous in each row of Zt).  One workgroup per candidate
// first index; *bad = 1 when G is not positive definite (the caller's
// re-solve).  The crowd at zero (q_crowd, c <= kQMaxCluster / 2 levels) is
// orthonormalised as the 2c columns x_0, Theta x_0, x_1, Theta x_1, ...
// (Theta in T's interleaved basis: (Theta z)_2s = -conj z_2s+1, (Theta
// z)_2s+1 = conj z_2s): Cholesky QR in that order keeps the pairs (the
// new Theta x_i is Theta of the new x_i, as Theta preserves the span of the
// earlier pairs), and only the x columns are written back.
__global__ __launch_bounds__(256) void k_q_orth(const double* __restrict__ E, const double* __restrict__ tnorm, int M,
                                                int j0, double2* __restrict__ Zt, int64_t sZ, double ctol,
                                                int* __restrict__ bad) {
  constexpr int MC = kQMaxCluster, RC = 64;   // rows staged per chunk (64: half the barriers of 32)
  const int k = blockIdx.y, n = 2 * M, nv = n - j0, jj = blockIdx.x, tid = threadIdx.x;
  E += (int64_t)k * n;
  Zt += k * sZ;
  const double tol = ctol * tnorm[k];
  const int ce = q_crowd(E, n, j0, tnorm[k]);
  const bool theta = jj == 0 && ce >= 2;
  if (jj > 0 && jj < ce) return;   // inside the crowd
  int kc = ce;
  if (!theta) {
    if (jj > 0 && E[j0 + jj] - E[j0 + jj - 1] <= tol) return;   // inside a cluster
    int end = jj + 1;
    while (end < nv && end - jj < MC && E[j0 + end] - E[j0 + end - 1] <= tol) ++end;
    kc = end - jj;
    if (kc == 1) return;
  }
  const int kw = theta ? 2 * kc : kc;   // working columns
  // working column c of row r (theta: x_{c/2}, and Theta x_{c/2} for odd c)
  auto zin = [&](int r, int c) -> double2 {
    if (r >= n) return make_double2(0.0, 0.0);
    if (!theta) return Zt[(int64_t)r * nv + jj + c];
    if (!(c & 1)) return Zt[(int64_t)r * nv + jj + (c >> 1)];
    const double2 p = Zt[(int64_t)(r ^ 1) * nv + jj + (c >> 1)];
    return (r & 1) ? make_double2(p.x, -p.y) : make_double2(-p.x, p.y);
  };
  __shared__ double2 G[MC][MC + 1];
  __shared__ double2 Zs[RC][MC + 1];
  __shared__ int fail;
  constexpr int NPT = (MC * (MC + 1) / 2 + 255) / 256;
  const int npair = kw * (kw + 1) / 2;
  auto pair_of = [&](int pq, int& pr, int& qc) {
    int r = (int)((sqrt(8.0 * pq + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= pq) ++r;
    while (r * (r + 1) / 2 > pq) --r;
    pr = r;
    qc = pq - r * (r + 1) / 2;
  };
  for (int round = 0; round < 2; ++round) {
    // G = Z_c^H Z_c (lower triangle), rows staged RC at a time
    double2 acc[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) acc[u] = make_double2(0.0, 0.0);
    for (int r0 = 0; r0 < n; r0 += RC) {
      for (int q = tid; q < RC * kw; q += 256) {
        const int rr = q / kw, c = q % kw;
        Zs[rr][c] = zin(r0 + rr, c);
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int pq = tid + 256 * u;
        if (pq < npair) {
          int pr, qc;
          pair_of(pq, pr, qc);
          double2 a = acc[u];
          for (int rr = 0; rr < RC; ++rr) {   // conj(z_p) z_q
            const double2 zp = Zs[rr][pr], zq = Zs[rr][qc];
            a.x += zp.x * zq.x + zp.y * zq.y;
            a.y += zp.x * zq.y - zp.y * zq.x;
          }
          acc[u] = a;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int pq = tid + 256 * u;
      if (pq < npair) {
        int pr, qc;
        pair_of(pq, pr, qc);
        G[pr][qc] = acc[u];
      }
    }
    if (tid == 0) fail = 0;
    __syncthreads();
    // Cholesky G = L L^H, right-looking, in place (lower)
    for (int c = 0; c < kw; ++c) {
      if (tid == 0) {
        const double g = G[c][c].x;   // the columns are normalised: a pivot this small means cond(Z) > ~1e7
        if (!(g > 1e-14)) fail = 1;
        G[c][c] = make_double2(sqrt(fmax(g, DBL_MIN)), 0.0);
      }
      __syncthreads();
      for (int r = c + 1 + tid; r < kw; r += 256) {
        const double d = G[c][c].x;
        G[r][c] = make_double2(G[r][c].x / d, G[r][c].y / d);
      }
      __syncthreads();
      for (int pq = tid; pq < kw * kw; pq += 256) {   // G[p][q] -= L[p][c] conj(L[q][c])
        const int pp = pq / kw, qq = pq % kw;
        if (qq > c && pp >= qq) {
          const double2 a = G[pp][c], b = G[qq][c];
          G[pp][qq].x -= a.x * b.x + a.y * b.y;
          G[pp][qq].y -= a.y * b.x - a.x * b.y;
        }
      }
      __syncthreads();
    }
    if (fail) {
      if (tid == 0) *bad = 1;
      return;
    }
    // each row z <- z L^-H: y = conj(z)^T, L y' = y, z <- conj(y')^T
    for (int r0 = 0; r0 < n; r0 += RC) {
      for (int q = tid; q < RC * kw; q += 256) {
        const int rr = q / kw, c = q % kw;
        Zs[rr][c] = zin(r0 + rr, c);
      }
      __syncthreads();
      if (tid < RC) {
        for (int pp = 0; pp < kw; ++pp) {
          double2 v = make_double2(Zs[tid][pp].x, -Zs[tid][pp].y);   // conj z_p
          for (int qq = 0; qq < pp; ++qq) {   // - L[p][q] y'_q, y'_q = conj(new z_q)
            const double2 l = G[pp][qq], y = make_double2(Zs[tid][qq].x, -Zs[tid][qq].y);
            v.x -= l.x * y.x - l.y * y.y;
            v.y -= l.x * y.y + l.y * y.x;
          }
          const double d = G[pp][pp].x;
          Zs[tid][pp] = make_double2(v.x / d, -v.y / d);   // conj back
        }
      }
      __syncthreads();
      for (int q = tid; q < RC * kc; q += 256) {   // the x columns back
        const int rr = q / kc, c = q % kc, r = r0 + rr;
        if (r < n) Zt[(int64_t)r * nv + jj + c] = Zs[rr][theta ? 2 * c : c];
      }
      __syncthreads();
    }
  }
}

// U' (column-major n x n, interleaved rows) columns j0 + jj from Yt (nv x n,
// ld nv: vector jj's entry r at Yt[jj + r nv]) with the site rotations g_s
// (G[2 s] = al, G[2 s + 1] = be; g = [[al, -conj be], [be, conj al]]) applied
// to each row pair (2 s, 2 s + 1): through a 32-row x 64-column LDS tile.
__global__ __launch_bounds__(256) void k_q_ztu(const double2* __restrict__ Yt, int64_t sY, const double2* __restrict__ G,
                                               int M, int j0, double2* __restrict__ U, int64_t sU) {
  const int k = blockIdx.z, n = 2 * M, nv = n - j0;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 64;
  Yt += k * sY;
  G += (int64_t)k * n;
  U += k * sU;
  __shared__ double2 t[32][65];
  for (int q = threadIdx.x; q < 32 * 64; q += 256) {
    const int rr = q >> 6, cc = q & 63, r = r0 + rr, c = c0 + cc;   // read: columns contiguous
    t[rr][cc] = (r < n && c < nv) ? Yt[c + (int64_t)r * nv] : make_double2(0.0, 0.0);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 32 * 64; q += 256) {
    const int cc = q >> 5, rr = q & 31, r = r0 + rr, c = c0 + cc;   // write: rows contiguous
    if (r >= n || c >= nv) continue;
    const int s = r >> 1, rp = rr & ~1;
    const double2 zp = t[rp][cc], zh = t[rp + 1][cc];
    const double2 al = G[2 * s], be = G[2 * s + 1];
    double2 o;
    if (!(r & 1))   // al zp - conj(be) zh
      o = make_double2(al.x * zp.x - al.y * zp.y - (be.x * zh.x + be.y * zh.y),
                       al.x * zp.y + al.y * zp.x - (be.x * zh.y - be.y * zh.x));
    else            // be zp + conj(al) zh
      o = make_double2(be.x * zp.x - be.y * zp.y + (al.x * zh.x + al.y * zh.y),
                       be.x * zp.y + be.y * zp.x + (al.x * zh.y - al.y * zh.x));
    U[r + (int64_t)(j0 + c) * n] = o;
  }
}

// V' (column-major n x n, interleaved rows) for the one-stage back-transform
// (dwhmc_eig.hip): column 2j = v_j, 2j+1 = Theta v_j (Theta (u; v) = (-conj
// v; conj u)) on the rows of the sites > j, zero elsewhere; columns 2M-2,
// 2M-1 zero; tau'[2j] = tau'[2j+1] = tau_j (real).  v_j from A's bottom rows
// (the reduction's storage: particle at row M + s of column 2j, hole of 2j+1).
__global__ __launch_bounds__(256) void k_q_vexpand(const double2* __restrict__ A, int64_t sA,
                                                   const double* __restrict__ tau, int M, double2* __restrict__ V,
                                                   double2* __restrict__ tauc) {
  const int k = blockIdx.z, n = 2 * M, c = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
  A += k * sA;
  V += k * sA;
  const int j = c >> 1, s = r >> 1;
  if (r == 0) tauc[(int64_t)k * n + c] = make_double2(j <= M - 2 ? tau[(int64_t)k * M + j] : 0.0, 0.0);
  if (r >= n) return;
  double2 o = make_double2(0.0, 0.0);
  if (j <= M - 2 && s >= j + 1) {
    const double2 vp = A[M + s + (int64_t)(2 * j) * n], vh = A[M + s + (int64_t)(2 * j + 1) * n];
    if (!(c & 1))
      o = (r & 1) ? vh : vp;
    else
      o = (r & 1) ? make_double2(vp.x, -vp.y) : make_double2(-vh.x, vh.y);
  }
  V[r + (int64_t)c * n] = o;
}

// The eigenvectors in the BdG order: column j >= j0 from U' (interleaved rows),
// column j < j0 the particle-hole partner Theta of column n - 1 - j.
__global__ __launch_bounds__(256) void k_q_final(const double2* __restrict__ Ui, int64_t sU, int M, int j0,
                                                 double2* __restrict__ U) {
  const int k = blockIdx.z, n = 2 * M, j = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  Ui += k * sU;
  U += k * sU;
  const bool hole = r >= M;
  const int s = hole ? r - M : r;
  double2 o;
  if (j >= j0) {
    o = Ui[2 * s + (hole ? 1 : 0) + (int64_t)j * n];
  } else {
    const int jp = n - 1 - j;
    const double2 v = Ui[2 * s + (hole ? 0 : 1) + (int64_t)jp * n];
    o = hole ? make_double2(v.x, -v.y) : make_double2(-v.x, v.y);
  }
  U[r + (int64_t)j * n] = o;
}

}  // namespace

#ifdef QSTAMPS
int q_stamps_read(unsigned long long* out, int nsteps) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qst), (size_t)nsteps * 16 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

bool q_supported(int M) { return M >= 1 && M <= kQMaxM; }

// the per-matrix scratch in double2 units
int q_part_elems(int M) { return (int)((q_fro_off(M) + kQFro + 2) / 2); }

void launch_q_reduce(double2* A, int M, int64_t sA, double2* part, int64_t sP, double2* W, double* tau, double2* Y,
                     double* qa, double2* qd, int m, hipStream_t s) {
  if (M < 1 || M > kQMaxM) return;   // callers check q_supported(M)
  double* q = reinterpret_cast<double*>(part);
  const int64_t sQ = 2 * sP;
  const int nT = (M + kQTB - 1) / kQTB;
  (void)hipMemset2DAsync(q, (size_t)sQ * sizeof(double), 0, (size_t)(4 * M + 4 * kQDotSlots) * sizeof(double), m,
                         s);   // P, dots
  hipLaunchKernelGGL(k_q_fro, dim3(kQFro, m), dim3(256), 0, s, A, M, sA, q, sQ);
  for (int j = -1; j <= M - 2; ++j) {
    hipLaunchKernelGGL(k_q_rs, dim3(m), dim3(kQRS), 0, s, A, M, j, sA, q, sQ, W, tau, Y, qa, qd);
    if (j <= M - 3) {
      const int nt = nT - (j + 2) / kQTB;
      hipLaunchKernelGGL(k_q_pass, dim3(nt * (nt + 1), m), dim3(64 * kQPW), 0, s, A, M, j, sA, W, q, sQ);
    }
  }
}

void launch_q_rot(const double* qa, const double2* qd, const double2* Y, int M, double* ra, double2* rd, double* rb,
                  double2* G, int m, hipStream_t s) {
  hipLaunchKernelGGL(k_q_rot, dim3(m), dim3(kQRotT), 0, s, qa, qd, Y, M, ra, rd, rb, G);
}

void launch_q_bisect(const double* ra, const double2* rd, const double* rb, int M, double* E, double* tnorm, int m,
                     hipStream_t s) {
  // the upper half only, the lower mirrored (E_{n-1-j} = -E_j)
  const int n = 2 * M, jofs = M, ni = n - jofs;
  int lgG = 6;
  while (lgG > 2 && ((int64_t)m * ni << (lgG - 1)) >= (int64_t)2048 * 64) --lgG;
  const int per_wg = kQBisW << (6 - lgG);
  hipLaunchKernelGGL(k_q_bisect, dim3((ni + per_wg - 1) / per_wg, m), dim3(64 * kQBisW),
                     (size_t)4 * (M + kQBisPad) * sizeof(double), s, ra, rd, rb, M, lgG, jofs, E, tnorm);
}

int64_t q_invit_scratch(int M, int j0) { return (int64_t)2 * M * 6 * (2 * M - j0); }

void launch_q_invit(const double* ra, const double2* rd, const double* rb, int M, const double* E, const double* tnorm,
                    int j0, double2* Zt, int64_t sZ, double2* S, int64_t sS, int m, hipStream_t s) {
  const int nv = 2 * M - j0;
  // 16-lane rows (k_q_invit16) while they fit one wave per SIMD (m nv <=
  // 4096): one L = 32 measurement 24.4 -> 23.8 ms; for larger batches the
  // thread per eigenvalue issues less in total (16 snapshots: 7.19 against
  // 7.59 ms per measurement; profiles/r06_exp_qinvit_lanes.txt).
  // DWHMC_QINVIT_THREAD=1 / 0 forces either (A/B).
  const char* env = std::getenv("DWHMC_QINVIT_THREAD");
  const bool thread = env && *env ? *env == '1' : (int64_t)m * nv > 4096;
  if (thread)
    hipLaunchKernelGGL(k_q_invit, dim3((nv + 63) / 64, m), dim3(64), (size_t)4 * M * sizeof(double), s, ra, rd, rb,
                       M, E, tnorm, j0, Zt, sZ, S, sS);
  else
    hipLaunchKernelGGL(k_q_invit16, dim3((nv + 3) / 4, m), dim3(64), (size_t)4 * M * sizeof(double), s, ra, rd, rb,
                       M, E, tnorm, j0, Zt, sZ, S, sS);
}

void launch_q_ztu(const double2* Yt, int64_t sY, const double2* G, int M, int j0, double2* U, int64_t sU, int m,
                  hipStream_t s) {
  const int n = 2 * M, nv = n - j0;
  hipLaunchKernelGGL(k_q_ztu, dim3((nv + 63) / 64, (n + 31) / 32, m), dim3(256), 0, s, Yt, sY, G, M, j0, U, sU);
}

void launch_q_vexpand(const double2* A, int64_t sA, const double* tau, int M, double2* V, double2* tauc, int m,
                      hipStream_t s) {
  const int n = 2 * M;
  hipLaunchKernelGGL(k_q_vexpand, dim3((n + 255) / 256, n, m), dim3(256), 0, s, A, sA, tau, M, V, tauc);
}

void launch_q_final(const double2* Ui, int64_t sU, int M, int j0, double2* U, int m, hipStream_t s) {
  const int n = 2 * M;
  hipLaunchKernelGGL(k_q_final, dim3((n + 255) / 256, n, m), dim3(256), 0, s, Ui, sU, M, j0, U);
}

int q_zero_crowd(const double* E, int n, int j0, double tn) { return q_crowd(E, n, j0, tn); }

int q_max_cluster() { return kQMaxCluster; }

void launch_q_orth(const double* E, const double* tnorm, int M, int j0, double2* Zt, int64_t sZ, double ctol, int* bad,
                   int m, hipStream_t s) {
  const int nv = 2 * M - j0;
  hipLaunchKernelGGL(k_q_orth, dim3(nv, m), dim3(256), 0, s, E, tnorm, M, j0, Zt, sZ, ctol, bad);
}

}  // namespace dwh
