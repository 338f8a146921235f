// Transport and spectra of measure_transport_and_spectra
// [src/Observables.jl:320-526] from the exact eigenpairs of one chain's H_BdG.
//
// This is the measurement path the reference runs every measure_transport_freq
// sweeps (src/Simulation.jl:170-186), not the leapfrog hot path: the
// eigenpairs come from the library's own Hermitian eigensolver
// (dwhmc_eig.hip) and J_mn = U^H (J ⊕ J) U from its own batched fp64 MFMA
// product (dwhmc_gemm.hip), both driven by dwhmc_api.cpp; the kernels here
// are everything around them.  All matrices are column-major with leading dimension n2 = 2N (the
// eigenvector of E_n is column n of U, as Julia's eigen! returns it).
//
// The O(n2^2 · n_ω) optical-conductivity sum is the only heavy kernel: every
// thread owns one ω and streams the (ΔE, c ΔE) pairs of a chunk of rows through
// LDS (one broadcast read per pair per wave), writing one partial per (chunk,
// ω); a second kernel adds the chunks in a fixed order, so results are
// deterministic run to run.
#include "dwhmc_internal.h"

namespace dwh {
namespace {

constexpr int kTB = 256;   // threads per block of every kernel here
constexpr double kInvPi = 0.31830988618379067154;
constexpr int kMaxDft = 1024;   // longest lattice side of the A(k, 0) DFT passes (twiddle table in LDS)

// LogExpFunctions.logistic, overflow-safe (the fermi factor f_n = logistic(-βE_n))
__device__ inline double logistic_d(double x) {
  if (x >= 0) return 1.0 / (1.0 + exp(-x));
  const double e = exp(x);
  return e / (1.0 + e);
}

// fixed-order tree sum of NV values per thread over the block; result in sh[v][0]
template <int NV>
__device__ inline void block_sum(double (&v)[NV], double (*sh)[kTB]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NV; ++k) sh[k][tid] = v[k];
  __syncthreads();
  for (int s = kTB / 2; s > 0; s >>= 1) {
    if (tid < s) {
#pragma unroll
      for (int k = 0; k < NV; ++k) sh[k][tid] += sh[k][tid + s];
    }
    __syncthreads();
  }
}

// Dense H_BdG = [[h, D], [conj(D), -h]] of one chain (init_static_H! +
// update_H_BdG!, src/Hamiltonian.jl:10-86); hcol/hval hold h with the
// reference's overwrite order already resolved, Dcol/Dsrc the pairing pattern
// (D[i, Dcol] = Δ[Dsrc] / 2).  Every entry is written at most once; the rest of
// A is zeroed beforehand.
__global__ void k_tr_assemble(double2* __restrict__ A, int n2, int N, const int* __restrict__ hcol,
                              const double* __restrict__ hval, const int* __restrict__ Dcol,
                              const int* __restrict__ Dsrc, const double2* __restrict__ Delta) {
  const int i = blockIdx.x * kTB + threadIdx.x;
  if (i >= N) return;
  for (int s = 0; s < kHSlots; ++s) {
    const int c = hcol[i * kHSlots + s];
    if (c < 0) continue;
    const double v = hval[i * kHSlots + s];
    A[i + (size_t)c * n2] = make_double2(v, 0.0);
    A[(i + N) + (size_t)(c + N) * n2] = make_double2(-v, 0.0);
  }
  for (int s = 0; s < kSlots; ++s) {
    const int c = Dcol[i * kSlots + s];
    if (c < 0) continue;
    const double2 d = Delta[Dsrc[i * kSlots + s]];
    A[i + (size_t)(c + N) * n2] = make_double2(0.5 * d.x, 0.5 * d.y);
    A[(i + N) + (size_t)c * n2] = make_double2(0.5 * d.x, -0.5 * d.y);
  }
}

// Per eigenstate n (one block per column of U):
//   f_n = logistic(-β E_n)                                   (compute_forces!, :50)
//   dia_n = [E_n > 0] w_n tanh(β E_n / 2), w_n the x-bond kinetic weight  (:345-362)
//   Wn_n = Σ_i |u_i|^2                                        (DOS weight, :452-456)
//   wan_n = (|Σ_i (-1)^x u_i|^2 + |Σ_i (-1)^y u_i|^2) / 2N     (antinodal, :465-488)
//   w0_n = L(-E_n) if > 1e-6 else 0                          (A(k, 0) weight, :497-503)
// nbr: jx (+x), jpy (+x+y), jmy (+x-y) per site, 0-based.
__global__ void k_tr_colstats(const double2* __restrict__ U, int n2, int N, int Lx,
                              const double* __restrict__ E, double beta, double eta, double t,
                              double tp, const int* __restrict__ nbr, double* __restrict__ f,
                              double* __restrict__ dia, double* __restrict__ Wn,
                              double* __restrict__ wan, double* __restrict__ w0) {
  __shared__ double sh[6][kTB];
  const int n = blockIdx.x;
  const double2* u = U + (size_t)n * n2;
  const double2* v = u + N;
  double acc[6] = {0, 0, 0, 0, 0, 0};   // w, W, Re ax, Im ax, Re ay, Im ay
  for (int i = threadIdx.x; i < N; i += kTB) {
    const double2 ui = u[i], vi = v[i];
    double w = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int j = nbr[b * N + i];
      const double2 uj = u[j], vj = v[j];
      // 2 Re(v_i conj(v_j) - conj(u_i) u_j)
      const double bond = 2.0 * ((vi.x * vj.x + vi.y * vj.y) - (ui.x * uj.x + ui.y * uj.y));
      w += (b == 0 ? t : tp) * bond;
    }
    acc[0] += w;
    acc[1] += ui.x * ui.x + ui.y * ui.y;
    const int x = i % Lx + 1, y = i / Lx + 1;
    const double sx = (x % 2 == 0) ? 1.0 : -1.0, sy = (y % 2 == 0) ? 1.0 : -1.0;
    acc[2] += sx * ui.x;
    acc[3] += sx * ui.y;
    acc[4] += sy * ui.x;
    acc[5] += sy * ui.y;
  }
  block_sum<6>(acc, sh);
  if (threadIdx.x == 0) {
    const double e = E[n];
    f[n] = logistic_d(-beta * e);
    dia[n] = e > 0 ? sh[0][0] * tanh(0.5 * beta * e) : 0.0;
    Wn[n] = sh[1][0];
    wan[n] = 0.5 * (sh[2][0] * sh[2][0] + sh[3][0] * sh[3][0] + sh[4][0] * sh[4][0] +
                    sh[5][0] * sh[5][0]) / N;
    const double l0 = kInvPi * (eta / (e * e + eta * eta));
    w0[n] = l0 > 1e-6 ? l0 : 0.0;
  }
}

// JU = (J ⊕ J) U with J the x-current operator in CSR form (duplicates summed,
// build_current_operator!, src/Observables.jl:237-283); J is purely imaginary,
// val holds Im J
__global__ void k_tr_current(const double2* __restrict__ U, double2* __restrict__ JU, int n2, int N,
                             const int* __restrict__ rowptr, const int* __restrict__ col,
                             const double* __restrict__ val) {
  const int r = blockIdx.x * kTB + threadIdx.x;
  if (r >= n2) return;
  const int n = blockIdx.y;
  const int rr = r < N ? r : r - N, off = r < N ? 0 : N;
  const double2* u = U + (size_t)n * n2 + off;
  double2 acc = make_double2(0.0, 0.0);
  for (int k = rowptr[rr]; k < rowptr[rr + 1]; ++k) {
    const double a = val[k];
    const double2 b = u[col[k]];
    acc.x -= a * b.y;
    acc.y += a * b.x;
  }
  JU[(size_t)n * n2 + r] = acc;
}

// Per column m of J_mn (threads over n): the paramagnetic sum Λ (:366-384)
// and the DC conductivity (:405-413), before the 1/N (and π·(1/π)) factors.
__global__ void k_tr_pairs(const double2* __restrict__ Jmn, int n2, const double* __restrict__ E,
                           const double* __restrict__ f, double beta, double eta,
                           double* __restrict__ lam_part, double* __restrict__ dc_part) {
  __shared__ double sh[2][kTB];
  const int m = blockIdx.x;
  const double Em = E[m], fm = f[m], eta2 = eta * eta;
  double acc[2] = {0, 0};
  for (int n = threadIdx.x; n < n2; n += kTB) {
    const double2 j = Jmn[(size_t)m * n2 + n];
    const double J2 = j.x * j.x + j.y * j.y;
    const double dE = Em - E[n], fn = f[n];
    const double bf = beta * fn * (1.0 - fn);
    const double ratio = fabs(dE) < 1e-8 ? bf : (fn - fm) / dE;
    acc[0] += ratio * J2;
    acc[1] += bf * J2 * (eta / (dE * dE + eta2));
  }
  block_sum<2>(acc, sh);
  if (threadIdx.x == 0) {
    lam_part[m] = sh[0][0];
    dc_part[m] = sh[1][0];
  }
}

__device__ inline double grid_point(double start, double step, int k) {
  return __dadd_rn(start, __dmul_rn(step, (double)k));
}

// σ(ω) partials (:415-423).  The reference sums c_nm L(ω - ΔE_nm) / ω over all
// ordered pairs with c_nm = (f_n - f_m) |J_nm|^2 (skipped where |f_n - f_m| <
// 1e-12) and ΔE_nm = E_m - E_n.  The pair (m, n) has c_mn = -c_nm and ΔE_mn =
// -ΔE_nm, so the two add up to
//     c_nm [1/a - 1/b] = c_nm · 4ω ΔE_nm / (a b),  a, b = (ω ∓ ΔE_nm)^2 + η^2,
// and σ(ω) = π/N · (1/π) η/ω · Σ_{ordered} = 4η/N · Σ_{n<m} c_nm ΔE_nm / (a b):
// half the pairs, one reciprocal per pair (v_rcp_f64 + one Newton step),
// and no 1/ω at small ω.  With E
// ascending, f_n - f_m vanishes (< 1e-12) for whole runs of m on either side
// of the Fermi level; a 256-pair tile whose c are all zero is skipped.
// Block (x, y): ω_k for k in the x tile, rows n in [y·rows, (y+1)·rows),
// m > n read down column n of J_mn (|J_nm| = |J_mn|, J_mn Hermitian).
// one Newton step (<= ~11 ulp, the bisection's Sturm count uses the same): the
// σ terms are positive-weighted sums, so a few-ulp relative error per term
// is a few-ulp relative error of σ
__device__ inline double rcp_nr1(double p) {
  const double r = __builtin_amdgcn_rcp(p);
  return fma(r, fma(-p, r, 1.0), r);
}

// ph (launch_tr_reduce): rows n < N only, m in (n, n2-1-n], the pairs
// strictly inside counted twice (each stands for its particle-hole partner
// (n2-1-m, n2-1-n)), the self-partnered m = n2-1-n once.
__global__ void __launch_bounds__(kTB)
k_tr_sigma(const double2* __restrict__ Jmn, int n2, const double* __restrict__ E,
           const double* __restrict__ f, double eta, double w_start, double w_step, int nw,
           int rows, int nrow, int ph, double* __restrict__ part) {
  __shared__ double sdE[kTB], scd[kTB];
  const int tid = threadIdx.x;
  const int k = blockIdx.x * kTB + tid;
  const double w = grid_point(w_start, w_step, k < nw ? k : nw - 1);
  const double eta2 = eta * eta, w4 = 4.0 * w;
  const int n0 = blockIdx.y * rows, n1 = min(n0 + rows, nrow);
  double acc0 = 0, acc1 = 0;
  for (int n = n0; n < n1; ++n) {
    const double En = E[n], fn = f[n];
    const double2* col = Jmn + (size_t)n * n2;
    const int mend = ph ? n2 - 1 - n : n2 - 1;   // last m of row n
    for (int m0 = ((n + 1) / kTB) * kTB; m0 <= mend; m0 += kTB) {
      const int m = m0 + tid;
      double cd = 0.0, dE = 0.0;
      if (m > n && m <= mend) {
        const double df = fn - f[m];
        if (fabs(df) >= 1e-12) {
          const double2 j = col[m];
          dE = E[m] - En;
          cd = df * (j.x * j.x + j.y * j.y) * dE;
          if (ph && m < mend) cd *= 2.0;
        }
      }
      if (!__syncthreads_or(cd != 0.0)) continue;
      scd[tid] = cd;
      sdE[tid] = dE;
      __syncthreads();
#pragma unroll 4
      for (int q = 0; q < kTB; q += 2) {
        // b = (ω+ΔE)^2 + η^2 = a + 4ωΔE (ΔE >= 0, ω > 0: no cancellation)
        const double d0 = sdE[q], d1 = sdE[q + 1];
        const double a0 = w - d0, a1 = w - d1;
        const double e0 = fma(a0, a0, eta2), e1 = fma(a1, a1, eta2);
        const double p0 = e0 * fma(w4, d0, e0);
        const double p1 = e1 * fma(w4, d1, e1);
        acc0 = fma(scd[q], rcp_nr1(p0), acc0);
        acc1 = fma(scd[q + 1], rcp_nr1(p1), acc1);
      }
      __syncthreads();
    }
  }
  if (k < nw) part[(size_t)blockIdx.y * nw + k] = acc0 + acc1;
}

// out = in^H per matrix k (in: R x C, ld lin; out: C x R, ld lout), 32 x 32
// tiles through LDS (both sides coalesced)
__global__ void __launch_bounds__(kTB)
k_tr_conj_transpose(const double2* __restrict__ in, int R, int C, int lin, int64_t sin,
                    double2* __restrict__ out, int lout, int64_t sout) {
  __shared__ double2 tile[32][33];
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32, k = blockIdx.z;
  in += k * sin;
  out += k * sout;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = threadIdx.x + kTB * q, c = idx >> 5, r = idx & 31;
    if (r0 + r < R && c0 + c < C) tile[c][r] = in[(r0 + r) + (int64_t)(c0 + c) * lin];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = threadIdx.x + kTB * q, r = idx >> 5, c = idx & 31;
    if (r0 + r < R && c0 + c < C) {
      const double2 v = tile[c][r];
      out[(c0 + c) + (int64_t)(r0 + r) * lout] = make_double2(v.x, -v.y);
    }
  }
}

// σ(ω_k) = 4η/N Σ_chunks part: 64 ω per block, wave q sums the chunks
// [q nchunk/4, (q+1) nchunk/4), the four in wave order
__global__ void k_tr_sigma_sum(const double* __restrict__ part, int nchunk, int nw, double eta, int N,
                               double* __restrict__ sigma) {
  __shared__ double sh[4][64];
  const int l = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + l;
  double s = 0;
  if (k < nw) {
    const int c0 = nchunk * q / 4, c1 = nchunk * (q + 1) / 4;
    for (int c = c0; c < c1; ++c) s += part[(size_t)c * nw + k];
  }
  sh[q][l] = s;
  __syncthreads();
  if (q == 0 && k < nw) sigma[k] = (((sh[0][l] + sh[1][l]) + sh[2][l]) + sh[3][l]) * (4.0 * eta / N);
}

// out[0] = stiffness = Σ dia / N - Σ lam / N; out[1] = dc = Σ dc / N
// (lam, dc over the npair columns k_tr_pairs computed, times pw: 2 when
// they are the half whose particle-hole partners carry the same sums)
__global__ void k_tr_scalars(const double* __restrict__ dia, const double* __restrict__ lam,
                             const double* __restrict__ dc, int n2, int N, int npair, double pw,
                             double* __restrict__ out) {
  __shared__ double sh[3][kTB];
  double acc[3] = {0, 0, 0};
  for (int n = threadIdx.x; n < n2; n += kTB) {
    acc[0] += dia[n];
    if (n < npair) {
      acc[1] += lam[n];
      acc[2] += dc[n];
    }
  }
  block_sum<3>(acc, sh);
  if (threadIdx.x == 0) {
    out[0] = sh[0][0] / N - pw * sh[1][0] / N;
    out[1] = pw * sh[2][0] / N;
  }
}

// DOS and antinodal DOS on the grid -ω_max:Δω:ω_max (:446-490): slice y of
// the eigenvalue range into part[y][k] (dos, dos_an interleaved), then the
// slices in a fixed order (k_tr_dos_sum)
__global__ void k_tr_dos(const double* __restrict__ E, const double* __restrict__ Wn,
                         const double* __restrict__ wan, int n2, double eta, double w_start,
                         double w_step, int nd, int per, double2* __restrict__ part) {
  const int k = blockIdx.x * kTB + threadIdx.x;
  if (k >= nd) return;
  const double w = grid_point(w_start, w_step, k), eta2 = eta * eta;
  const int n0 = blockIdx.y * per, n1 = min(n0 + per, n2);
  double a = 0, b = 0;
  for (int n = n0; n < n1; ++n) {
    const double d = w - E[n];
    const double l = kInvPi * (eta / (d * d + eta2));
    a += Wn[n] * l;
    b += wan[n] * l;
  }
  part[(size_t)blockIdx.y * nd + k] = make_double2(a, b);
}

__global__ void k_tr_dos_sum(const double2* __restrict__ part, int nsl, int nd, int N, double* __restrict__ dos,
                             double* __restrict__ dos_an) {
  const int k = blockIdx.x * kTB + threadIdx.x;
  if (k >= nd) return;
  double a = 0, b = 0;
  for (int c = 0; c < nsl; ++c) {
    const double2 p = part[(size_t)c * nd + k];
    a += p.x;
    b += p.y;
  }
  dos[k] = a / N;
  dos_an[k] = b;
}

// (cos, sin) of -2π q / L: the twiddle the LDS tables hold, for sides above kMaxDft
__device__ __forceinline__ double2 dft_twiddle(int q, int L) {
  double2 t;
  sincospi(-2.0 * (double)q / L, &t.y, &t.x);
  return t;
}

// A(k, ω=0) (:492-516): FFT2 of every particle column u_n as an Lx x Ly image
// (site i = x + Lx y), done as two direct DFT passes.  Pass x:
// T[kx + Lx y, n] = Σ_x u[x + Lx y, n] e^{-2πi kx x / Lx}
__global__ void k_tr_dft_x(const double2* __restrict__ U, int n2, int Lx, int Ly,
                           double2* __restrict__ T) {
  __shared__ double2 tw[kMaxDft];   // (cos, sin) of -2π q / Lx, computed once per block
  const bool tab = Lx <= kMaxDft;    // longer sides: each twiddle by sincospi (no table)
  if (tab)
    for (int q = threadIdx.x; q < Lx; q += kTB) sincospi(-2.0 * (double)q / Lx, &tw[q].y, &tw[q].x);
  __syncthreads();
  const int N = Lx * Ly;
  const int idx = blockIdx.x * kTB + threadIdx.x;
  if (idx >= N) return;
  const int n = blockIdx.y, kx = idx % Lx, y = idx / Lx;
  const double2* u = U + (size_t)n * n2 + (size_t)y * Lx;
  double2 acc = make_double2(0.0, 0.0);
  for (int x = 0; x < Lx; ++x) {
    const double2 t = tab ? tw[(kx * x) % Lx] : dft_twiddle((kx * x) % Lx, Lx);
    const double s = t.y, c = t.x;
    const double2 a = u[x];
    acc.x += a.x * c - a.y * s;
    acc.y += a.x * s + a.y * c;
  }
  T[(size_t)n * N + idx] = acc;
}

// Pass y and weight: Pw[kx + Lx ky, n] = w0_n |Σ_y T[kx + Lx y, n] e^{-2πi ky y / Ly}|^2
__global__ void k_tr_dft_y(const double2* __restrict__ T, const double* __restrict__ w0, int Lx,
                           int Ly, double* __restrict__ Pw) {
  __shared__ double2 tw[kMaxDft];
  const bool tab = Ly <= kMaxDft;
  if (tab)
    for (int q = threadIdx.x; q < Ly; q += kTB) sincospi(-2.0 * (double)q / Ly, &tw[q].y, &tw[q].x);
  __syncthreads();
  const int N = Lx * Ly;
  const int idx = blockIdx.x * kTB + threadIdx.x;
  if (idx >= N) return;
  const int n = blockIdx.y, kx = idx % Lx, ky = idx / Lx;
  const double2* tcol = T + (size_t)n * N + kx;
  double2 acc = make_double2(0.0, 0.0);
  for (int y = 0; y < Ly; ++y) {
    const double2 t = tab ? tw[(ky * y) % Ly] : dft_twiddle((ky * y) % Ly, Ly);
    const double s = t.y, c = t.x;
    const double2 a = tcol[(size_t)y * Lx];
    acc.x += a.x * c - a.y * s;
    acc.y += a.x * s + a.y * c;
  }
  Pw[(size_t)n * N + idx] = w0[n] * (acc.x * acc.x + acc.y * acc.y);
}

// A_k[kx + Lx ky] = Σ_n Pw[k, n] / N in two fixed-order stages: slice y of
// the n range into part[y][k], then the slices in order
__global__ void k_tr_ak_part(const double* __restrict__ Pw, int n2, int N, int per,
                             double* __restrict__ part) {
  const int k = blockIdx.x * kTB + threadIdx.x;
  if (k >= N) return;
  const int n0 = blockIdx.y * per, n1 = min(n0 + per, n2);
  double s = 0;
  for (int n = n0; n < n1; ++n) s += Pw[(size_t)n * N + k];
  part[(size_t)blockIdx.y * N + k] = s;
}

__global__ void k_tr_ak_sum(const double* __restrict__ part, int nsl, int N, double* __restrict__ ak) {
  const int k = blockIdx.x * kTB + threadIdx.x;
  if (k >= N) return;
  double s = 0;
  for (int c = 0; c < nsl; ++c) s += part[(size_t)c * N + k];
  ak[k] = s / N;
}

// ---------------------------------------------------------------------------
// Eigendecomposition leapfrog step (algo eig): the reference's own method —
// diagonalize_H_BdG! (src/Hamiltonian.jl:96-114), compute_forces!
// (src/Observables.jl:14-62) and the E_f of compute_total_energy
// (src/HMC.jl:21-27) — for β·E'/2 beyond the pole table.  zheevd gives E, U
// per chain; ρ = U diag(f) U^H is one zgemm of JU = U diag(f) with U^H; the
// kernels here form JU and gather P_ij = -ρ_{i,j+N} - ρ_{j,i+N}, Tr ρ_hh and E_f.
// ---------------------------------------------------------------------------
__global__ void k_eig_scale(const double2* __restrict__ U, double2* __restrict__ JU, const double* __restrict__ E,
                            int n2, double beta) {
  const int a = blockIdx.x * kTB + threadIdx.x;
  const int n = blockIdx.y, k = blockIdx.z;
  if (a >= n2) return;
  const double f = logistic_d(-beta * E[(int64_t)k * n2 + n]);
  const int64_t o = ((int64_t)k * n2 + n) * n2 + a;
  const double2 u = U[o];
  JU[o] = make_double2(u.x * f, u.y * f);
}

// one block per chain; bond b = i + N·dir with partner j = Dcol[bond_ij[b]]
__global__ void k_eig_gather(const double2* __restrict__ rho, const double* __restrict__ E, int N,
                             const int* __restrict__ Dcol, const int* __restrict__ bond_ij, double beta,
                             double2* __restrict__ Pair, double* __restrict__ Ef, double* __restrict__ Trhh) {
  __shared__ double sh[2][kTB];
  const int c = blockIdx.x, n2 = 2 * N;
  const double2* R = rho + (int64_t)c * n2 * n2;
  for (int b = threadIdx.x; b < n2; b += kTB) {
    const int i = b < N ? b : b - N;
    const int j = Dcol[bond_ij[b]];
    const double2 r1 = R[i + (int64_t)(j + N) * n2], r2 = R[j + (int64_t)(i + N) * n2];
    Pair[(int64_t)c * n2 + b] = make_double2(-(r1.x + r2.x), -(r1.y + r2.y));
  }
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < N; i += kTB) v[0] += R[(i + N) + (int64_t)(i + N) * n2].x;
  for (int n = threadIdx.x; n < n2; n += kTB) {
    const double e = E[(int64_t)c * n2 + n];
    if (e > 0) {
      const double x = beta * e;
      v[1] += x + 2.0 * log1p(exp(-x));
    }
  }
  block_sum<2>(v, sh);
  if (threadIdx.x == 0) {
    Trhh[c] = sh[0][0];
    Ef[c] = -sh[1][0];
  }
}

// any non-finite entry of U (nu complex) or E (ne real) -> *bad = 1
__global__ void k_nonfinite(const double2* __restrict__ U, int64_t nu, const double* __restrict__ E, int64_t ne,
                            int* __restrict__ bad) {
  bool nf = false;
  const int64_t stride = (int64_t)gridDim.x * kTB;
  for (int64_t k = (int64_t)blockIdx.x * kTB + threadIdx.x; k < nu; k += stride) {
    const double2 u = U[k];
    nf |= !isfinite(u.x) || !isfinite(u.y);
  }
  for (int64_t k = (int64_t)blockIdx.x * kTB + threadIdx.x; k < ne; k += stride) nf |= !isfinite(E[k]);
  if (nf) *bad = 1;
}

inline int cdiv(int64_t a, int b) { return (int)((a + b - 1) / b); }

}  // namespace

void launch_nonfinite(const double2* U, int64_t nu, const double* E, int64_t ne, int* bad, hipStream_t s) {
  const int64_t n = nu > ne ? nu : ne;
  const int grid = (int)std::min<int64_t>(std::max<int64_t>(cdiv(n, kTB), 1), 2048);
  hipLaunchKernelGGL(k_nonfinite, dim3(grid), dim3(kTB), 0, s, U, nu, E, ne, bad);
}

void launch_eig_scale(const double2* U, double2* JU, const double* E, int N, int nc, double beta, hipStream_t s) {
  hipLaunchKernelGGL(k_eig_scale, dim3(cdiv(2 * N, kTB), 2 * N, nc), dim3(kTB), 0, s, U, JU, E, 2 * N, beta);
}

void launch_eig_gather(const double2* rho, const double* E, int N, int nc, const int* Dcol, const int* bond_ij,
                       double beta, double2* Pair, double* Ef, double* Trhh, hipStream_t s) {
  hipLaunchKernelGGL(k_eig_gather, dim3(nc), dim3(kTB), 0, s, rho, E, N, Dcol, bond_ij, beta, Pair, Ef, Trhh);
}

void launch_tr_assemble(double2* A, int N, const int* hcol, const double* hval, const int* Dcol,
                        const int* Dsrc, const double2* Delta, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_assemble, dim3(cdiv(N, kTB)), dim3(kTB), 0, s, A, 2 * N, N, hcol, hval,
                     Dcol, Dsrc, Delta);
}

void launch_tr_colstats(const double2* U, int N, int Lx, const double* E, double beta, double eta,
                        double t, double tp, const int* nbr, double* f, double* dia, double* Wn,
                        double* wan, double* w0, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_colstats, dim3(2 * N), dim3(kTB), 0, s, U, 2 * N, N, Lx, E, beta, eta, t,
                     tp, nbr, f, dia, Wn, wan, w0);
}

void launch_tr_current(const double2* U, double2* JU, int N, const int* rowptr, const int* col,
                       const double* val, int ncol, hipStream_t s) {
  hipLaunchKernelGGL(k_tr_current, dim3(cdiv(2 * N, kTB), ncol), dim3(kTB), 0, s, U, JU, 2 * N,
                     N, rowptr, col, val);
}

void launch_tr_conj_transpose(const double2* in, int R, int C, int lin, int64_t sin, double2* out, int lout,
                              int64_t sout, int m, hipStream_t s) {
  if (R <= 0 || C <= 0 || m <= 0) return;
  hipLaunchKernelGGL(k_tr_conj_transpose, dim3(cdiv(R, 32), cdiv(C, 32), m), dim3(kTB), 0, s, in, R, C, lin, sin,
                     out, lout, sout);
}

int tr_sigma_chunks(int N) { return std::min(2 * N, 512); }
constexpr int kDosPer = 128;   // eigenvalues per DOS slice
int tr_dos_slices(int N) { return cdiv(2 * N, kDosPer); }

void launch_tr_reduce(const TrBufs& b, int N, int Lx, int Ly, double beta, double eta,
                      const TrGrid& g, bool ph, hipStream_t s) {
  const int n2 = 2 * N;
  const int npair = ph ? N : n2;   // columns of J_mn the pair sums read
  hipLaunchKernelGGL(k_tr_pairs, dim3(npair), dim3(kTB), 0, s, b.Jmn, n2, b.E, b.f, beta, eta, b.lam,
                     b.dc);
  if (g.nw > 0) {
    const int nchunk = std::min(tr_sigma_chunks(N), npair), rows = cdiv(npair, nchunk);
    const int used = cdiv(npair, rows);
    hipLaunchKernelGGL(k_tr_sigma, dim3(cdiv(g.nw, kTB), used), dim3(kTB), 0, s, b.Jmn, n2, b.E,
                       b.f, eta, g.w0, g.dw, g.nw, rows, npair, (int)ph, b.part);
    hipLaunchKernelGGL(k_tr_sigma_sum, dim3(cdiv(g.nw, 64)), dim3(256), 0, s, b.part, used, g.nw,
                       eta, N, b.sigma);
  }
  hipLaunchKernelGGL(k_tr_scalars, dim3(1), dim3(kTB), 0, s, b.dia, b.lam, b.dc, n2, N, npair, ph ? 2.0 : 1.0,
                     b.scalars);
  if (g.nd > 0) {
    // eigenvalue slices of kDosPer (partials in the σ partial buffer, free
    // again after k_tr_sigma_sum; sized for both)
    const int pr = kDosPer, ns = tr_dos_slices(N);
    double2* dp = reinterpret_cast<double2*>(b.part);
    hipLaunchKernelGGL(k_tr_dos, dim3(cdiv(g.nd, kTB), ns), dim3(kTB), 0, s, b.E, b.Wn, b.wan, n2, eta, g.d0, g.dw,
                       g.nd, pr, dp);
    hipLaunchKernelGGL(k_tr_dos_sum, dim3(cdiv(g.nd, kTB)), dim3(kTB), 0, s, dp, ns, g.nd, N, b.dos, b.dos_an);
  }
  // A(k, 0): T reuses JU, the weighted |FFT|^2 reuses J_mn (both no longer needed)
  hipLaunchKernelGGL(k_tr_dft_x, dim3(cdiv(N, kTB), n2), dim3(kTB), 0, s, b.U, n2, Lx, Ly, b.JU);
  double* Pw = reinterpret_cast<double*>(b.Jmn);
  hipLaunchKernelGGL(k_tr_dft_y, dim3(cdiv(N, kTB), n2), dim3(kTB), 0, s, b.JU, b.w0, Lx, Ly, Pw);
  // slices of the n sum: partials into JU (free again after k_tr_dft_y)
  const int per = 64, nsl = cdiv(n2, per);
  double* akp = reinterpret_cast<double*>(b.JU);
  hipLaunchKernelGGL(k_tr_ak_part, dim3(cdiv(N, kTB), nsl), dim3(kTB), 0, s, Pw, n2, N, per, akp);
  hipLaunchKernelGGL(k_tr_ak_sum, dim3(cdiv(N, kTB)), dim3(kTB), 0, s, akp, nsl, N, b.ak);
}

}  // namespace dwh
