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
// A[y+1, y] (2 Ly + y) of A = H_BdG - i y_q for every (chain, pole); one wave
// per block row, lanes over columns (coalesced row writes), over the blocks of
// `list` (level-0 block ids).  Ly == 2: the single off-diagonal block lives in
// U (L = 0); Ly == 1: everything in D.  Padding rows/columns (b <= r < BP) are
// the identity in D, zero elsewhere.  All blocks are written once at context
// creation; per factorisation only the blocks CR overwrites (the level-0
// eliminated D blocks) are rewritten and k_cr_pair_scatter refreshes the
// pairing entries of the others.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_cr_fill(double2* __restrict__ pool, int64_t item, int Lx,
                                                 int Ly, int BP, int P, int nrows,
                                                 const int* __restrict__ list,
                                                 const int* __restrict__ hcol,
                                                 const double* __restrict__ hval,
                                                 const int* __restrict__ Dcol,
                                                 const double2* __restrict__ Dv,
                                                 const double* __restrict__ ypole) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const int bi = blockIdx.y, c = bi / P, q = bi - c * P;
  const int N = Lx * Ly, b = 2 * Lx;
  const int lb = list[row / BP], r = row - (row / BP) * BP;
  const int t = lb / Ly, y = lb - t * Ly;     // t: 0 D, 1 U, 2 L
  double2* out = pool + (int64_t)bi * item + ((int64_t)(t * Ly + y) * BP + r) * BP;
  const bool zero = (t == 1 && Ly < 2) || (t == 2 && Ly < 3);
  const int yr = (t == 2) ? (y + 1) % Ly : y;
  const int yc = (t == 1) ? (y + 1) % Ly : y;
  const bool rpad = r >= b;
  const int pr = r >= Lx ? 1 : 0;
  const int i = yr * Lx + (r - pr * Lx);
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
    dv[s] = (!rpad && !zero) ? Dv[(int64_t)c * N * kSlots + (int64_t)s * N + i] : make_double2(0.0, 0.0);
  }
  const double yq = ypole[q];
  for (int cc = lane; cc < BP; cc += 64) {
    double2 v = make_double2(0.0, 0.0);
    if (rpad || cc >= b) {
      if (t == 0 && cc == r) v.x = 1.0;
    } else if (!zero) {
      const int pc = cc >= Lx ? 1 : 0;
      const int j = yc * Lx + (cc - pc * Lx);
      if (pc == pr) {
#pragma unroll
        for (int s = 0; s < kHSlots; ++s)
          if (hc[s] == j) v.x = pr ? -hv[s] : hv[s];
        if (i == j) v.y = -yq;
      } else {
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
          if (dc[s] == j) v = pr ? make_double2(dv[s].x, -dv[s].y) : dv[s];
      }
    }
    out[cc] = v;
  }
}

// Pairing entries Δ/2 (particle row, hole column) and conj (hole row, particle
// column) into the level-0 blocks CR does not overwrite (offsets from the
// planner; -1 = entry lies in a rewritten block or the slot is empty).
__global__ void k_cr_pair_scatter(double2* __restrict__ pool, int64_t item, int N, int P,
                                  const int64_t* __restrict__ off_ph,
                                  const int64_t* __restrict__ off_hp,
                                  const double2* __restrict__ Dv) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int bi = blockIdx.y, c = bi / P;
  if (e >= N * kSlots) return;
  const int i = e / kSlots, sl = e - i * kSlots;
  const double2 v = Dv[(int64_t)c * N * kSlots + (int64_t)sl * N + i];
  double2* base = pool + (int64_t)bi * item;
  const int64_t o1 = off_ph[e], o2 = off_hp[e];
  if (o1 >= 0) base[o1] = v;
  if (o2 >= 0) base[o2] = make_double2(v.x, -v.y);
}

// ---------------------------------------------------------------------------
// In-place no-pivot Gauss-Jordan inversion of BP x BP blocks (BP = 16 NT),
// register resident: the 2x2 wave grid owns NT/2 x NT/2 MFMA tiles each (C
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
  double2* M = pool + (int64_t)bi * item + (int64_t)blk[li] * BP * BP;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lr = l & 15, lk = l >> 4;
  const int I0 = (w >> 1) * TH, J0 = (w & 1) * TH;
  d4 ar[TH][TH], ai[TH][TH];
  CR_STAMP(0);
#pragma unroll
  for (int ti = 0; ti < TH; ++ti)
#pragma unroll
    for (int tj = 0; tj < TH; ++tj)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const double2 v = M[(int64_t)((I0 + ti) * 16 + lk + 4 * rr) * BP + (J0 + tj) * 16 + lr];
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
#pragma unroll
  for (int ti = 0; ti < TH; ++ti)
#pragma unroll
    for (int tj = 0; tj < TH; ++tj)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        M[(int64_t)((I0 + ti) * 16 + lk + 4 * rr) * BP + (J0 + tj) * 16 + lr] =
            make_double2(ar[ti][tj][rr], ai[ti][tj][rr]);
  if (tid == 0) ldpart[(int64_t)bi * nslots + slot[li]] = ld;
  CR_STAMP(7);
}

// ---------------------------------------------------------------------------
// Batched block products: task t of batch item bi writes
//   out = [cin] + sg Σ_{h < nt} A_h B_h      (BP x BP blocks of the item's pool)
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
  constexpr int KS = BP / 4;
  constexpr int64_t BB = (int64_t)BP * BP;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 acr[2][2], aci[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      if (cin >= 0) {
        const double2* C = base + cin * BB + (int64_t)(tr * 32 + mi * 16 + lk) * BP + tc * 32 + ni * 16 + lr;
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
    const double2* B = base + tk->b[h] * BB + (int64_t)lk * BP + tc * 32 + lr;
    double2 fa[2][2], fb[2][2];
    auto load = [&](int s, double2 (&a)[2], double2 (&bb)[2]) {
      a[0] = A[s * 4];
      a[1] = A[(int64_t)16 * BP + s * 4];
      bb[0] = B[(int64_t)s * 4 * BP];
      bb[1] = B[(int64_t)s * 4 * BP + 16];
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
  double2* O = base + tk->out * BB + (int64_t)(tr * 32 + lk) * BP + tc * 32 + lr;
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
  constexpr int KS = BP / 4, PF = 4;
  constexpr int64_t BB = (int64_t)BP * BP;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 acr[2], aci[2];
  acr[1] = d4{0.0, 0.0, 0.0, 0.0};
  aci[1] = d4{0.0, 0.0, 0.0, 0.0};
  if (cin >= 0) {
    const double2* C = base + cin * BB + (int64_t)(tr * 16 + lk) * BP + tc * 16 + lr;
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
    const double2* B = base + tk->b[h] * BB + (int64_t)lk * BP + tc * 16 + lr;
    double2 fa[PF], fb[PF];
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      fa[s] = A[s * 4];
      fb[s] = B[(int64_t)s * 4 * BP];
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int cs = s % PF, p = s & 1;
      const double2 av = make_double2(sg * fa[cs].x, sg * fa[cs].y), bv = fb[cs];
      if (s + PF < KS) {
        fa[cs] = A[(s + PF) * 4];
        fb[cs] = B[(int64_t)(s + PF) * 4 * BP];
      }
      acr[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, acr[p], 0, 0, 0);
      aci[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, aci[p], 0, 0, 0);
      acr[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, bv.y, acr[p], 0, 0, 0);
      aci[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, aci[p], 0, 0, 0);
    }
  }
  double2* O = base + tk->out * BB + (int64_t)(tr * 16 + lk) * BP + tc * 16 + lr;
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
// G12 at the pairing pattern and diag(G22) from the level-0 blocks of G
// (element offsets precomputed by the planner; -1 = empty slot).
// ---------------------------------------------------------------------------
__global__ void k_cr_gather(const double2* __restrict__ pool, int64_t item, int N,
                            const int64_t* __restrict__ goff, const int64_t* __restrict__ doff,
                            double2* __restrict__ G12nn, double2* __restrict__ diagS) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int bi = blockIdx.y;
  if (i >= N) return;
  const double2* base = pool + (int64_t)bi * item;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const int64_t o = goff[i * kSlots + s];
    G12nn[((int64_t)bi * N + i) * kSlots + s] = o >= 0 ? base[o] : make_double2(0.0, 0.0);
  }
  diagS[(int64_t)bi * N + i] = base[doff[i]];
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
bool cr_supported_bp(int BP) { return BP == 32 || BP == 64 || BP == 96; }

void launch_cr_fill(const CrDims& c, double2* pool, const int* list, int nlist, const int* hcol,
                    const double* hval, const int* Dcol, const double2* Dv, const double* ypole,
                    hipStream_t s) {
  if (nlist <= 0) return;
  const int nrows = nlist * c.BP;
  hipLaunchKernelGGL(k_cr_fill, dim3((nrows + 3) / 4, c.nbatch), dim3(256), 0, s, pool, c.item, c.Lx,
                     c.Ly, c.BP, c.P, nrows, list, hcol, hval, Dcol, Dv, ypole);
}

void launch_cr_pair_scatter(const CrDims& c, double2* pool, const int64_t* off_ph,
                            const int64_t* off_hp, const double2* Dv, hipStream_t s) {
  hipLaunchKernelGGL(k_cr_pair_scatter, dim3((c.N * kSlots + 255) / 256, c.nbatch), dim3(256), 0, s,
                     pool, c.item, c.N, c.P, off_ph, off_hp, Dv);
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
    return e ? std::atoi(e) : 2048;
  }();
  const bool use16 = (int64_t)c.nbatch * ntasks * maxt32 < small;
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

void launch_cr_gather(const CrDims& c, const double2* pool, const int64_t* goff,
                      const int64_t* doff, double2* G12nn, double2* diagS, hipStream_t s) {
  hipLaunchKernelGGL(k_cr_gather, dim3((c.N + 255) / 256, c.nbatch), dim3(256), 0, s, pool, c.item,
                     c.N, goff, doff, G12nn, diagS);
}

}  // namespace dwh
