// gfx950 kernels of the block cyclic-reduction (CR) path (DWHMC_ALGO=cr).
//
// Ordering the BdG basis by lattice row y (block y = [particles of row y |
// holes of row y], b = 2 Lx, padded to BP = 16*NT) makes H_BdG - i y_q block
// tridiagonal with periodic corners: hopping (src/Hamiltonian.jl:26-43) and
// pairing (src/Hamiltonian.jl:68-83) only couple row y to y-1, y, y+1
// (neighbour tables src/Types.jl:60-80).  Cyclic reduction eliminates every
// other block per level (Schur complements, no pivoting: i(H - i y) has
// Hermitian part y I > 0 and every Schur complement inherits it) and a
// backward pass recovers the block-tridiagonal part of G = (H - i y)^-1,
// which holds every entry the force (G12 at the pairing bonds), E_f (ln|det|
// from the block pivots) and Tr ρ_hh (diag G22) need.  The host planner
// (dwhmc_api.cpp, mirrored by tools/cr_model.py) turns the recursion into
// stages: block inversions (k_cr_inv) and task lists of block products
// (k_cr_gemm), all batched over (chain, pole).
//
// Particle-hole symmetry (S H* S^-1 = -H, S = [[0, I], [-I, 0]] per site)
// makes every CR block X either M-form [[A, B], [conj B, -conj A]] (H - i y,
// inverses, G) or Q-form [[A, B], [-conj B, conj A]] (products of two
// M-forms), with particle x at column x and hole x at column HP + x.  Blocks
// are stored as their top half T = [A | B] (HP x BP, BP = 2 HP): half the
// memory, and a product computes only the top half of its output with the
// bottom rows of the right operand synthesised from its top half:
//   Y[HP + i, j] = sgn * conj(T_Y[i, (j + HP) mod BP]),  sgn = -s_Y (j < HP), +s_Y (j >= HP)
// (s = -1 M-form, +1 Q-form; tools/cr_model.py top_product).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {

// Diagnostic build only (-DCR_STAMPS, tools/micro/cr_inv_stamps.hip): per-block
// s_memtime stamps of k_cr_inv's phases; never compiled into the library.
#ifdef CR_STAMPS
__device__ unsigned long long g_cr_stamps[1024][16];
#define CR_STAMP(i)                                                                  \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0)                                                            \
      g_cr_stamps[blockIdx.y * gridDim.x + blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)
#else
#define CR_STAMP(i) \
  do {              \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// Level-0 blocks D[y] (pool block y), U[y] = A[y, y+1] (Ly + y), L[y] =
// A[y+1, y] (2 Ly + y) of A = H_BdG - i y_q for every (chain, pole), top
// halves (particle rows): A part h - i y (columns 0..Lx-1), B part the pairing
// Δ/2 (columns HP..HP+Lx-1).  One wave per block row, lanes over columns
// (coalesced row writes), over the blocks of `list` (level-0 block ids).
// Ly == 2: the single off-diagonal block lives in U (L = 0); Ly == 1:
// everything in D.  Padded sites (Lx <= x < HP) are 1 on the diagonal of D
// (hole -1 implied by the M-form), zero elsewhere.  All blocks are written
// once at context creation; per factorisation only the blocks CR overwrites
// (the level-0 eliminated D blocks) are rewritten and k_cr_pair_scatter
// refreshes the pairing entries of the others.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 half_delta(const double2* __restrict__ Delta, const int* __restrict__ Dsrc,
                                              int N, int c, int i, int s) {
  const int src = Dsrc[i * kSlots + s];
  if (src < 0) return make_double2(0.0, 0.0);
  const double2 d = Delta[(int64_t)c * 2 * N + src];
  return make_double2(0.5 * d.x, 0.5 * d.y);
}

__global__ __launch_bounds__(256) void k_cr_fill(double2* __restrict__ pool, int64_t item, int Lx,
                                                 int Ly, int BP, int P, int nrows, int fill_blocks,
                                                 const int* __restrict__ list,
                                                 const int* __restrict__ hcol,
                                                 const double* __restrict__ hval,
                                                 const int* __restrict__ Dcol,
                                                 const int* __restrict__ Dsrc,
                                                 const double2* __restrict__ Delta,
                                                 const double* __restrict__ ypole,
                                                 const int64_t* __restrict__ off_ph) {
  const int bi = blockIdx.y, c = bi / P, q = bi - c * P;
  const int N = Lx * Ly, HP = BP / 2;
  if ((int)blockIdx.x >= fill_blocks) {
    // pairing scatter Δ/2 (particle row, hole column) into the level-0 blocks
    // CR does not overwrite (hole-row entries implied by the M-form)
    const int e = ((int)blockIdx.x - fill_blocks) * blockDim.x + threadIdx.x;
    if (e >= N * kSlots) return;
    const int64_t o = off_ph[e];
    if (o >= 0) pool[(int64_t)bi * item + o] = half_delta(Delta, Dsrc, N, c, e / kSlots, e % kSlots);
    return;
  }
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const int lb = list[row / HP], r = row - (row / HP) * HP;
  const int t = lb / Ly, y = lb - t * Ly;     // t: 0 D, 1 U, 2 L
  double2* out = pool + (int64_t)bi * item + ((int64_t)(t * Ly + y) * HP + r) * BP;
  const bool zero = (t == 1 && Ly < 2) || (t == 2 && Ly < 3);
  const int yr = (t == 2) ? (y + 1) % Ly : y;
  const int yc = (t == 1) ? (y + 1) % Ly : y;
  const bool rpad = r >= Lx;
  const int i = yr * Lx + r;
  int hc[kHSlots], dc[kSlots];
  double hv[kHSlots];
  double2 dv[kSlots];
#pragma unroll
  for (int s = 0; s < kHSlots; ++s) {
    hc[s] = (!rpad && !zero) ? hcol[i * kHSlots + s] : -1;
    hv[s] = (!rpad && !zero) ? hval[((int64_t)c * N + i) * kHSlots + s] : 0.0;
  }
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    dc[s] = (!rpad && !zero) ? Dcol[i * kSlots + s] : -1;
    dv[s] = (!rpad && !zero) ? half_delta(Delta, Dsrc, N, c, i, s) : make_double2(0.0, 0.0);
  }
  const double yq = ypole[q];
  for (int cc = lane; cc < BP; cc += 64) {
    double2 v = make_double2(0.0, 0.0);
    const int pc = cc >= HP ? 1 : 0, xc = cc - pc * HP;
    if (rpad || xc >= Lx) {
      if (t == 0 && cc == r) v.x = 1.0;
    } else if (!zero) {
      const int j = yc * Lx + xc;
      if (pc == 0) {          // particle-particle: h - i y
#pragma unroll
        for (int s = 0; s < kHSlots; ++s)
          if (hc[s] == j) v.x = hv[s];
        if (i == j) v.y = -yq;
      } else {                // particle-hole: Δ/2
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
          if (dc[s] == j) v = dv[s];
      }
    }
    out[cc] = v;
  }
}

// ---------------------------------------------------------------------------
// In-place no-pivot Gauss-Jordan inversion of M-form BP x BP blocks (BP = 16
// NT) stored as top halves: the bottom rows are synthesised on load
// (conj B | -conj A), only the top half of the (M-form) inverse is stored.
// Register resident: the 2x2 wave grid owns NT/2 x NT/2 MFMA tiles each (C
// layout).  Per 16-wide sub-step kb: the owners publish block row kb and
// block column kb to LDS, every wave inverts the 16x16 pivot tile (wave
// local), forms X_J = P^-1 A_kJ for its own columns, then updates its tiles:
//   A_IJ <- [J != kb] A_IJ - A_Ik X_J  (I != kb),   A_kJ <- X_J   (X_kb = P^-1).
// ln|det| (= Σ ln|pivots|) goes to ldpart[bi][slot].
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) void k_cr_inv(double2* __restrict__ pool, int64_t item,
                                                const int* __restrict__ blk,
                                                const int* __restrict__ slot,
                                                double* __restrict__ ldpart, int nslots) {
  constexpr int BP = 16 * NT, TH = NT / 2;
  constexpr int RS = BP + 1;        // LDS row stride of the row panel
  constexpr int XS = TH * 16 + 1;   // LDS row stride of a wave's X panel
  __shared__ double2 Rp[16 * RS];
  __shared__ double2 Cp[BP * 17];
  __shared__ double2 Dw[4][16 * 17];
  __shared__ double2 Xw[4][16 * XS];
  const int bi = blockIdx.y, li = blockIdx.x;
  double ld = 0.0;   // Σ ln|pivots| (identical in every wave)
  constexpr int HP = BP / 2;
  double2* M = pool + (int64_t)bi * item + (int64_t)blk[li] * HP * BP;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lr = l & 15, lk = l >> 4;
  const int I0 = (w >> 1) * TH, J0 = (w & 1) * TH;   // wave row 0: top half, 1: bottom half
  d4 ar[TH][TH], ai[TH][TH];
  CR_STAMP(0);
#pragma unroll
  for (int ti = 0; ti < TH; ++ti)
#pragma unroll
    for (int tj = 0; tj < TH; ++tj)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = (I0 + ti) * 16 + lk + 4 * rr, col = (J0 + tj) * 16 + lr;
        double2 v;
        if (row < HP) {
          v = M[(int64_t)row * BP + col];
        } else {   // M-form bottom half: [conj B | -conj A]
          const double2 u = M[(int64_t)(row - HP) * BP + (col < HP ? col + HP : col - HP)];
          v = col < HP ? make_double2(u.x, -u.y) : make_double2(-u.x, u.y);
        }
        ar[ti][tj][rr] = v.x;
        ai[ti][tj][rr] = v.y;
      }
  CR_STAMP(1);
#pragma unroll 1
  for (int kb = 0; kb < NT; ++kb) {
    // (1) publish block row kb and block column kb
#pragma unroll
    for (int ti = 0; ti < TH; ++ti)
      if (I0 + ti == kb) {
#pragma unroll
        for (int tj = 0; tj < TH; ++tj)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            Rp[(lk + 4 * rr) * RS + (J0 + tj) * 16 + lr] = make_double2(ar[ti][tj][rr], ai[ti][tj][rr]);
      }
#pragma unroll
    for (int tj = 0; tj < TH; ++tj)
      if (J0 + tj == kb) {
#pragma unroll
        for (int ti = 0; ti < TH; ++ti)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            Cp[((I0 + ti) * 16 + lk + 4 * rr) * 17 + lr] = make_double2(ar[ti][tj][rr], ai[ti][tj][rr]);
      }
    __syncthreads();
    if (kb == 0) CR_STAMP(2);
    // (2) every wave inverts the pivot tile in registers (lane: row l&15, cols 4(l>>4)..)
    double2 dv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dv[jj] = Rp[(l & 15) * RS + kb * 16 + (l >> 4) * 4 + jj];
    ld += 0.5 * log(wave_inv16_dpp(dv));
    if (kb == 0) CR_STAMP(3);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) Dw[w][(l & 15) * 17 + (l >> 4) * 4 + jj] = dv[jj];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (3) X_J = P^-1 A_kJ for this wave's columns
#pragma unroll
    for (int tj = 0; tj < TH; ++tj) {
      d4 xr = {0.0, 0.0, 0.0, 0.0}, xi = {0.0, 0.0, 0.0, 0.0};
      if (J0 + tj == kb) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double2 v = Dw[w][(lk + 4 * rr) * 17 + lr];
          xr[rr] = v.x;
          xi[rr] = v.y;
        }
      } else {
        mma16_lds<false>(xr, xi, Dw[w], 17, Rp + (J0 + tj) * 16, RS);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Xw[w][(lk + 4 * rr) * XS + tj * 16 + lr] = make_double2(xr[rr], xi[rr]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (kb == 0) CR_STAMP(4);
    // (4) tile updates
#pragma unroll
    for (int ti = 0; ti < TH; ++ti)
#pragma unroll
      for (int tj = 0; tj < TH; ++tj) {
        if (I0 + ti == kb) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const double2 v = Xw[w][(lk + 4 * rr) * XS + tj * 16 + lr];
            ar[ti][tj][rr] = v.x;
            ai[ti][tj][rr] = v.y;
          }
        } else {
          if (J0 + tj == kb) {
            ar[ti][tj] = d4{0.0, 0.0, 0.0, 0.0};
            ai[ti][tj] = d4{0.0, 0.0, 0.0, 0.0};
          }
          mma16_lds<true>(ar[ti][tj], ai[ti][tj], Cp + (I0 + ti) * 16 * 17, 17, Xw[w] + tj * 16, XS);
        }
      }
    __syncthreads();
    if (kb == 0) CR_STAMP(5);
  }
  CR_STAMP(6);
  if (I0 == 0) {   // top half of the inverse
#pragma unroll
    for (int ti = 0; ti < TH; ++ti)
#pragma unroll
      for (int tj = 0; tj < TH; ++tj)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          M[(int64_t)((I0 + ti) * 16 + lk + 4 * rr) * BP + (J0 + tj) * 16 + lr] =
              make_double2(ar[ti][tj][rr], ai[ti][tj][rr]);
  }
  if (tid == 0) ldpart[(int64_t)bi * nslots + slot[li]] = ld;
  CR_STAMP(7);
}

// ---------------------------------------------------------------------------
// Batched block products on top halves: task t of batch item bi writes
//   out = [cin] + sg Σ_{h < nt} A_h B_h      (top halves, HP x BP)
// K runs over all BP rows of B_h: rows 0..HP-1 are stored, rows HP..BP-1 are
// synthesised as sgn * conj(B_top[k - HP, (j + HP) mod BP]) with sgn from the
// term's form bit (CrTask::bq) and the column half of the output tile.
// One wave per TS x TS output tile (TS = 32: 2x2 MFMA tiles, operand reuse;
// TS = 16: one MFMA tile with two interleaved accumulator chains, 4x the
// waves for the small stages of the coarse levels, which are latency bound).
// MFMA fragments come straight from L2 with a register prefetch; 1D grid with
// the XCD-aware remap so one item's tasks share an XCD's L2.  out never
// aliases an operand (planner invariant); out == cin is allowed.
// ---------------------------------------------------------------------------
template <int BP>
__device__ __forceinline__ void cr_tile32(double2* base, const CrTask* tk, int cin, int nt, int tr,
                                          int tc, double sg) {
  constexpr int HP = BP / 2, KS = BP / 4, KH = HP / 4;
  constexpr int64_t BB = (int64_t)HP * BP;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int c0 = tc * 32, crot = c0 < HP ? c0 + HP : c0 - HP;
  d4 acr[2][2], aci[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      if (cin >= 0) {
        const double2* C = base + cin * BB + (int64_t)(tr * 32 + mi * 16 + lk) * BP + c0 + ni * 16 + lr;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double2 v = C[(int64_t)4 * rr * BP];
          acr[mi][ni][rr] = v.x;
          aci[mi][ni][rr] = v.y;
        }
      } else {
        acr[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
        aci[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
      }
    }
#pragma unroll 1
  for (int h = 0; h < nt; ++h) {
    const double2* A = base + tk->a[h] * BB + (int64_t)(tr * 32 + lr) * BP + lk;
    const double2* Bt = base + tk->b[h] * BB + (int64_t)lk * BP + lr;
    // synthesised rows: sgn * conj(.), sgn = -s (left column half) / +s (right), s = +1 Q, -1 M
    const double sb = ((tk->bq >> h) & 1) ? 1.0 : -1.0;
    const double sgn = c0 < HP ? -sb : sb;
    double2 fa[2][2], fb[2][2];
    auto load = [&](int s, double2 (&a)[2], double2 (&bb)[2]) {
      a[0] = A[s * 4];
      a[1] = A[(int64_t)16 * BP + s * 4];
      if (s < KH) {
        bb[0] = Bt[(int64_t)s * 4 * BP + c0];
        bb[1] = Bt[(int64_t)s * 4 * BP + c0 + 16];
      } else {
        const double2 u0 = Bt[(int64_t)(s - KH) * 4 * BP + crot];
        const double2 u1 = Bt[(int64_t)(s - KH) * 4 * BP + crot + 16];
        bb[0] = make_double2(sgn * u0.x, -sgn * u0.y);
        bb[1] = make_double2(sgn * u1.x, -sgn * u1.y);
      }
    };
    load(0, fa[0], fb[0]);
    load(1, fa[1], fb[1]);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int cs = s & 1;
      const double2 av[2] = {make_double2(sg * fa[cs][0].x, sg * fa[cs][0].y),
                             make_double2(sg * fa[cs][1].x, sg * fa[cs][1].y)};
      const double2 bv[2] = {fb[cs][0], fb[cs][1]};
      if (s + 2 < KS) load(s + 2, fa[cs], fb[cs]);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          acr[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mi].x, bv[ni].x, acr[mi][ni], 0, 0, 0);
          aci[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mi].x, bv[ni].y, aci[mi][ni], 0, 0, 0);
        }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          acr[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[mi].y, bv[ni].y, acr[mi][ni], 0, 0, 0);
          aci[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mi].y, bv[ni].x, aci[mi][ni], 0, 0, 0);
        }
    }
  }
  double2* O = base + tk->out * BB + (int64_t)(tr * 32 + lk) * BP + c0 + lr;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        O[(int64_t)(mi * 16 + 4 * rr) * BP + ni * 16] = make_double2(acr[mi][ni][rr], aci[mi][ni][rr]);
}

template <int BP>
__device__ __forceinline__ void cr_tile16(double2* base, const CrTask* tk, int cin, int nt, int tr,
                                          int tc, double sg) {
  constexpr int HP = BP / 2, KS = BP / 4, KH = HP / 4, PF = 4;
  constexpr int64_t BB = (int64_t)HP * BP;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int c0 = tc * 16, crot = c0 < HP ? c0 + HP : c0 - HP;
  d4 acr[2], aci[2];
  acr[1] = d4{0.0, 0.0, 0.0, 0.0};
  aci[1] = d4{0.0, 0.0, 0.0, 0.0};
  if (cin >= 0) {
    const double2* C = base + cin * BB + (int64_t)(tr * 16 + lk) * BP + c0 + lr;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const double2 v = C[(int64_t)4 * rr * BP];
      acr[0][rr] = v.x;
      aci[0][rr] = v.y;
    }
  } else {
    acr[0] = d4{0.0, 0.0, 0.0, 0.0};
    aci[0] = d4{0.0, 0.0, 0.0, 0.0};
  }
#pragma unroll 1
  for (int h = 0; h < nt; ++h) {
    const double2* A = base + tk->a[h] * BB + (int64_t)(tr * 16 + lr) * BP + lk;
    const double2* Bt = base + tk->b[h] * BB + (int64_t)lk * BP + lr;
    const double sb = ((tk->bq >> h) & 1) ? 1.0 : -1.0;
    const double sgn = c0 < HP ? -sb : sb;
    auto bload = [&](int s) {
      if (s < KH) return Bt[(int64_t)s * 4 * BP + c0];
      const double2 u = Bt[(int64_t)(s - KH) * 4 * BP + crot];
      return make_double2(sgn * u.x, -sgn * u.y);
    };
    double2 fa[PF], fb[PF];
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      fa[s] = A[s * 4];
      fb[s] = bload(s);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int cs = s % PF, p = s & 1;
      const double2 av = make_double2(sg * fa[cs].x, sg * fa[cs].y), bv = fb[cs];
      if (s + PF < KS) {
        fa[cs] = A[(s + PF) * 4];
        fb[cs] = bload(s + PF);
      }
      acr[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, acr[p], 0, 0, 0);
      aci[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, aci[p], 0, 0, 0);
      acr[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, bv.y, acr[p], 0, 0, 0);
      aci[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, aci[p], 0, 0, 0);
    }
  }
  double2* O = base + tk->out * BB + (int64_t)(tr * 16 + lk) * BP + c0 + lr;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
    O[(int64_t)4 * rr * BP] = make_double2(acr[0][rr] + acr[1][rr], aci[0][rr] + aci[1][rr]);
}

template <int BP, int TS>
__global__ __launch_bounds__(256) void k_cr_gemm(double2* __restrict__ pool, int64_t item,
                                                 const CrTask* __restrict__ tasks, int ntasks,
                                                 int maxt, int total, double sg) {
  const int gw = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (int)(threadIdx.x >> 6));
  if (gw >= total) return;
  const int per_item = ntasks * maxt;
  const int bi = gw / per_item;
  const int rmd = gw - bi * per_item;
  const int tsk = rmd / maxt, tile = rmd - tsk * maxt;
  const CrTask* tk = tasks + tsk;
  const int tr0 = tk->r0 / TS, tc0 = tk->c0 / TS;
  const int ct = (tk->c1 + TS - 1) / TS - tc0;
  const int rt = (tk->r1 + TS - 1) / TS - tr0;
  if (tile >= rt * ct) return;   // restricted task: fewer tiles than the stage maximum
  const int tr = tr0 + tile / ct, tc = tc0 + tile % ct;
  double2* base = pool + (int64_t)bi * item;
  if (TS == 32) cr_tile32<BP>(base, tk, tk->cin, tk->nt, tr, tc, sg);
  else cr_tile16<BP>(base, tk, tk->cin, tk->nt, tr, tc, sg);
}

// ---------------------------------------------------------------------------
// Force from the level-0 G blocks: P_ij = Σ_q c_q (G12[i,j] + G12[j,i]) with
// G12 read straight from the B parts of the pool (offsets goff per pairing
// slot), F = -β/2J (Δ - J P) (src/Observables.jl:14-62), then the leapfrog
// kick and the next step's drift (kick_drift).
// ---------------------------------------------------------------------------
__global__ void k_cr_pair_force(const double2* __restrict__ pool, int64_t item,
                                const int64_t* __restrict__ goff, const int* __restrict__ bond_ij,
                                const int* __restrict__ bond_ji, const double* __restrict__ cpole,
                                int N, int P, double2* __restrict__ Delta,
                                double2* __restrict__ Pair, double2* __restrict__ F,
                                double2* __restrict__ Pi, double kick, double drift, double cap2,
                                int* __restrict__ flag, double beta, double J) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (b >= 2 * N) return;
  const int64_t o1 = goff[bond_ij[b]], o2 = goff[bond_ji[b]];
  double2 Pv = make_double2(0.0, 0.0);
  for (int q = 0; q < P; ++q) {
    const double2* G = pool + (int64_t)(c * P + q) * item;
    const double2 g1 = G[o1], g2 = G[o2];
    const double cq = cpole[q];
    Pv.x += cq * (g1.x + g2.x);
    Pv.y += cq * (g1.y + g2.y);
  }
  const int64_t o = (int64_t)c * 2 * N + b;
  Pair[o] = Pv;
  const double2 d = Delta[o];
  const double f = -beta / (2.0 * J);
  const double2 Fv = make_double2(f * (d.x - J * Pv.x), f * (d.y - J * Pv.y));
  F[o] = Fv;
  kick_drift(Fv, o, Delta, Pi, kick, drift, cap2, flag);
}

// E_f = -2N C - β Σ_q c_q ln|det(H - i y_q)| (block pivots) and
// Tr ρ_hh = N/2 - Σ_q c_q Re Tr G22 (G22[x,x] = -conj(A[x,x]) of the M-form
// diagonal G blocks); one block per chain (src/HMC.jl:21-27, Observables.jl:120-145)
__global__ __launch_bounds__(256) void k_cr_fermion_energy(const double2* __restrict__ pool,
                                                           int64_t item,
                                                           const int64_t* __restrict__ doff,
                                                           const double* __restrict__ ldpart,
                                                           const double* __restrict__ cpole, int N,
                                                           int nld, int P, double Cx, double beta,
                                                           double* __restrict__ Ef,
                                                           double* __restrict__ Trhh) {
  const int c = blockIdx.x;
  __shared__ double red[2][4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double ef = 0.0, tr = 0.0;
  for (int q = 0; q < P; ++q) {
    const int bi = c * P + q;
    double ld = 0.0, t = 0.0;
    for (int k = threadIdx.x; k < nld; k += blockDim.x) ld += ldpart[(int64_t)bi * nld + k];
    for (int i = threadIdx.x; i < N; i += blockDim.x) t -= pool[(int64_t)bi * item + doff[i]].x;
    ef += cpole[q] * ld;
    tr += cpole[q] * t;
  }
  ef = wave_sum(ef);
  tr = wave_sum(tr);
  if (l == 0) {
    red[0][w] = ef;
    red[1][w] = tr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Ef[c] = -2.0 * N * Cx - beta * (red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    Trhh[c] = 0.5 * N - (red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
bool cr_supported_bp(int BP) { return BP == 32 || BP == 64 || BP == 96; }

void launch_cr_fill(const CrDims& c, double2* pool, const int* list, int nlist, const int* hcol,
                    const double* hval, const int* Dcol, const int* Dsrc, const double2* Delta,
                    const double* ypole, const int64_t* off_ph, hipStream_t s) {
  const int nrows = nlist * c.BP / 2;
  const int fill_blocks = (nrows + 3) / 4;
  const int scatter_blocks = off_ph ? (c.N * kSlots + 255) / 256 : 0;
  if (fill_blocks + scatter_blocks == 0) return;
  hipLaunchKernelGGL(k_cr_fill, dim3(fill_blocks + scatter_blocks, c.nbatch), dim3(256), 0, s, pool,
                     c.item, c.Lx, c.Ly, c.BP, c.P, nrows, fill_blocks, list, hcol, hval, Dcol, Dsrc,
                     Delta, ypole, off_ph);
}

void launch_cr_inv(const CrDims& c, double2* pool, const int* blk, const int* slot, int n,
                   double* ldpart, hipStream_t s) {
  if (n <= 0) return;
  const dim3 g(n, c.nbatch);
  switch (c.BP) {
    case 32: hipLaunchKernelGGL(k_cr_inv<2>, g, dim3(256), 0, s, pool, c.item, blk, slot, ldpart, c.Ly); break;
    case 64: hipLaunchKernelGGL(k_cr_inv<4>, g, dim3(256), 0, s, pool, c.item, blk, slot, ldpart, c.Ly); break;
    default: hipLaunchKernelGGL(k_cr_inv<6>, g, dim3(256), 0, s, pool, c.item, blk, slot, ldpart, c.Ly); break;
  }
}

void launch_cr_gemm(const CrDims& c, double2* pool, const CrTask* tasks, int ntasks, int maxt32,
                    int maxt16, double sg, hipStream_t s) {
  if (ntasks <= 0) return;
  // latency-bound small stages (fewer than ~2 waves per SIMD at 32x32 tiles)
  // run 16x16 wave tiles: 4x the waves, 4x shorter MFMA chains
  static const int small = [] {
    const char* e = std::getenv("DWHMC_CR_SMALL");
    return e ? std::atoi(e) : 1024;
  }();
  // 32-wide tiles must not straddle the A | B column halves
  const bool use16 = (c.BP / 2) % 32 != 0 || (int64_t)c.nbatch * ntasks * maxt32 < small;
  const int maxt = use16 ? maxt16 : maxt32;
  const int total = c.nbatch * ntasks * maxt;
  const dim3 g((total + 3) / 4), b(256);
#define CR_GEMM(BPV)                                                                             \
  if (use16)                                                                                     \
    hipLaunchKernelGGL((k_cr_gemm<BPV, 16>), g, b, 0, s, pool, c.item, tasks, ntasks, maxt, total, sg); \
  else                                                                                           \
    hipLaunchKernelGGL((k_cr_gemm<BPV, 32>), g, b, 0, s, pool, c.item, tasks, ntasks, maxt, total, sg);
  switch (c.BP) {
    case 32: CR_GEMM(32) break;
    case 64: CR_GEMM(64) break;
    default: CR_GEMM(96) break;
  }
#undef CR_GEMM
}

void launch_cr_pair_force(const CrDims& c, const double2* pool, const int64_t* goff,
                          const int* bond_ij, const int* bond_ji, const double* cpole,
                          double2* Delta, double2* Pair, double2* F, double2* Pi,
                          const KickDrift& kd, double beta, double J, hipStream_t s) {
  const int nc = c.nbatch / c.P;
  hipLaunchKernelGGL(k_cr_pair_force, dim3((2 * c.N + 255) / 256, nc), dim3(256), 0, s, pool, c.item,
                     goff, bond_ij, bond_ji, cpole, c.N, c.P, Delta, Pair, F, Pi, kd.kick, kd.drift,
                     kd.cap * kd.cap, kd.flag, beta, J);
}

void launch_cr_fermion_energy(const CrDims& c, const double2* pool, const int64_t* doff,
                              const double* ldpart, const double* cpole, double Cx, double beta,
                              double* Ef, double* Trhh, hipStream_t s) {
  const int nc = c.nbatch / c.P;
  hipLaunchKernelGGL(k_cr_fermion_energy, dim3(nc), dim3(256), 0, s, pool, c.item, doff, ldpart,
                     cpole, c.N, c.Ly, c.P, Cx, beta, Ef, Trhh);
}

}  // namespace dwh
