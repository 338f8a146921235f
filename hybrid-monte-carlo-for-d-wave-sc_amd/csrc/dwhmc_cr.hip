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

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {

// Diagnostic build only (-DCR_STAMPS: tools/cr_inv_sched_stamps.py through
// dwh_debug_cr_stamps, tools/micro/cr_inv_stamps.hip): per-workgroup stamps of
// the inversion launch whose first inverted block is g_cr_stamp_key, in the
// library's own schedule (side work and guard workgroups included).  Row of a
// workgroup (blockIdx.y * gridDim.x + blockIdx.x < kCrStampWG): [0] / [30]
// s_memrealtime (100 MHz, chip-wide) at entry / exit, [1..29] s_memtime
// (shader clock) at the phase boundaries of the kernel, [31] kind (1
// inversion, 2 side work, 3 guard).  Wave 0's view.  Never in the library.
#ifdef CR_STAMPS
__device__ unsigned long long g_cr_stamps[kCrStampWG][32];
__device__ int g_cr_stamp_key = -1;
#define CR_STAMP_INIT(blkp) const bool stamp_on = (blkp)[0] == g_cr_stamp_key
#define CR_STAMP_AT(i, v)                                                               \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    const int wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                \
    if (stamp_on && threadIdx.x == 0 && wg_ < kCrStampWG) g_cr_stamps[wg_][i] = (v);     \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#define CR_STAMP(i) CR_STAMP_AT(i, __builtin_amdgcn_s_memtime())
#define CR_RSTAMP(i) CR_STAMP_AT(i, __builtin_amdgcn_s_memrealtime())
#else
#define CR_STAMP_INIT(blkp) \
  do {                      \
  } while (0)
#define CR_STAMP_AT(i, v) \
  do {                    \
  } while (0)
#define CR_STAMP(i) \
  do {              \
  } while (0)
#define CR_RSTAMP(i) \
  do {               \
  } while (0)
#endif

// Diagnostic build only (-DCR_GEMM_STAMPS, tools/gemm_stamps.py): per-workgroup
// phase stamps of the k_cr_gemm launch whose total tile count equals
// g_gemm_sel (wave 0's view): [0] s_memrealtime at entry, [1..4] s_memtime at
// entry / descriptor loaded / partials in LDS / after the reduction barrier,
// [5] s_memtime at the end, [6] s_memrealtime at the end, [7] HW_ID.
#ifdef CR_GEMM_STAMPS
__device__ unsigned long long g_gemm_stamps[65536][8];
__device__ int g_gemm_sel;
#define GEMM_STAMP(i, sel)                                                             \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    if ((sel) && threadIdx.x == 0 && blockIdx.x < 65536)                               \
      g_gemm_stamps[blockIdx.x][i] = (i) == 0 || (i) == 6 ? __builtin_amdgcn_s_memrealtime() \
                                                          : __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#else
#define GEMM_STAMP(i, sel) \
  do {                     \
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
// once at context creation and CR never overwrites them (level-0 inverses go
// to other blocks), so a factorisation only scatters the pairing entries Δ/2
// (the trailing blocks of this launch) — and inside a trajectory not even
// that: k_cr_pair_force scatters the drifted Δ itself.
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
// In-place no-pivot block Gauss-Jordan inversion of M-form BP x BP blocks
// (BP = 16 NT) stored as top halves: the bottom rows are synthesised on load
// (conj B | -conj A), only the top half of the (M-form) inverse is stored.
// NT waves; wave w keeps block column w (NT 16 x 16 MFMA tiles, C layout) in
// registers.  Column kb (P^-1 = A_kk^-1 and the old A_Ik) sits in LDS panel
// kb & 1 at the start of pivot step kb.  Step kb:
//   phase 1   wave kb reads P^-1; every wave J != kb forms X_J = P^-1 A_kJ
//             from its tile kb (used in place as the MFMA B operand: the C
//             layout of row 4s + lk is the B layout of k-step s), A_kJ <- X_J;
//             the lookahead wave kb+1 copies X and its other column tiles
//             (not yet updated) into the next panel;
//   phase 2   wave kb: A_Ik <- -A_Ik P^-1 for its column;
//             wave kb+1 updates tile kb+1 only, inverts it (the next pivot) and
//             writes it to the next panel — its pivot chain carries no other
//             tile updates; other waves J: the lookahead column's tile J
//             inside the next panel, Q_J -= A_Jk X_{kb+1}, then their own
//             A_IJ <- A_IJ - A_Ik X_J.
// Two barriers per pivot step (double-buffered panel).  16 x 16 pivot tiles
// are inverted in registers (wave_inv16_dpp); complex MACs are 3 real MFMAs.
// ln|det| (= Σ ln|pivots|) goes to ldpart[bi][slot].
// ---------------------------------------------------------------------------
// acc(16x16, C layout) += (NEG ? -1 : 1) * A(16 x 16, LDS row-major, stride 17) * B
// with B given in the C layout (b_r, b_i: row 4 rr + lk, column lr).
template <bool NEG>
__device__ __forceinline__ void mma16_3m(d4& cr, d4& ci, const double2* A, const d4& br, const d4& bi) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 t1 = cr, t2 = {0.0, 0.0, 0.0, 0.0}, t3 = cr + ci;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const double2 av = A[lr * 17 + 4 * ks + lk];
    const double a_r = NEG ? -av.x : av.x, a_i = NEG ? -av.y : av.y;
    t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a_r, br[ks], t1, 0, 0, 0);
    t2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a_i, bi[ks], t2, 0, 0, 0);
    t3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a_r + a_i, br[ks] + bi[ks], t3, 0, 0, 0);
  }
  cr = t1 - t2;
  ci = t3 - t1 - t2;
}

// acc(16x16, C layout) += (NEG ? -1 : 1) * X^T * A^T: X given in the C layout
// (its register rr is the A-operand fragment of k-step rr of X^T), A a 16 x 16
// row-major LDS tile (stride 17) read transposed as the B operand.  Used for
// a tile kept transposed: (T - A X)^T = T^T - X^T A^T.
template <bool NEG>
__device__ __forceinline__ void mma16_3m_T(d4& cr, d4& ci, const double2* A, const d4& xr, const d4& xi) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 t1 = cr, t2 = {0.0, 0.0, 0.0, 0.0}, t3 = cr + ci;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const double2 bv = A[lr * 17 + 4 * ks + lk];
    const double a_r = NEG ? -xr[ks] : xr[ks], a_i = NEG ? -xi[ks] : xi[ks];
    t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a_r, bv.x, t1, 0, 0, 0);
    t2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a_i, bv.y, t2, 0, 0, 0);
    t3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a_r + a_i, bv.x + bv.y, t3, 0, 0, 0);
  }
  cr = t1 - t2;
  ci = t3 - t1 - t2;
}

// one workgroup (NT waves) inverts block blk[li] of batch item bi; pan / ldw:
// the caller's LDS (double-buffered panel, per-wave ln|det| partials)
template <int NT>
__device__ __forceinline__ void cr_inv_wg(double2* __restrict__ pool, int64_t item, int bi, int li,
                                          const int* __restrict__ blk, const int* __restrict__ dst,
                                          const int* __restrict__ slot, double* __restrict__ ldpart,
                                          int nslots, double2 (*pan)[NT][16 * 17], double* ldw) {
  constexpr int BP = 16 * NT, HP = BP / 2, TSZ = 16 * 17;
  const double2* M = pool + (int64_t)bi * item + (int64_t)blk[li] * HP * BP;
  double2* Mo = pool + (int64_t)bi * item + (int64_t)dst[li] * HP * BP;   // may equal M
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 ar[NT], ai[NT];
  CR_STAMP_INIT(blk);
  CR_RSTAMP(0);
  CR_STAMP(1);
  // Tiles in the MFMA C layout (lane: rows lk + 4 rr, column lr), except the
  // diagonal tile (w, w), which is kept TRANSPOSED until it becomes this
  // wave's pivot: its C layout is then the strided inversion layout (lane:
  // row lr, columns lk + 4 rr), so the pivot is inverted in registers with no
  // transpose, and its updates A_ww -= A_wk X_w run as
  // A_ww^T -= X_w^T A_wk^T (mma16_3m_T: X from registers, A_wk^T from LDS).
  // The diagonal tile is loaded transposed straight from memory (lane: row lr,
  // columns lk + 4 rr of the tile), so no LDS transpose precedes the first
  // pivot inversion.
#pragma unroll
  for (int I = 0; I < NT; ++I)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const bool diag = (I == w);
      const int row = I * 16 + (diag ? lr : lk + 4 * rr), col = w * 16 + (diag ? lk + 4 * rr : lr);
      double2 v;
      if (row < HP) {
        v = M[(int64_t)row * BP + col];
      } else {   // M-form bottom half: [conj B | -conj A]
        const double2 u = M[(int64_t)(row - HP) * BP + (col < HP ? col + HP : col - HP)];
        v = col < HP ? make_double2(u.x, -u.y) : make_double2(-u.x, u.y);
      }
      ar[I][rr] = v.x;
      ai[I][rr] = v.y;
    }
#ifdef CR_STAMPS
  if (stamp_on) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  CR_STAMP(2);
  // Π |pivot|^2 of this wave's pivot tile (each wave inverts exactly one);
  // its log is taken after the loop, off the pivot chain
  double pp = 1.0;
  // in-place inverse of the (transposed-stored) diagonal tile
  auto invert = [&](d4& tr, d4& ti) -> double {
    double2 dv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dv[jj] = make_double2(tr[jj], ti[jj]);
    const double r = wave_inv16_dpp<true>(dv);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      tr[jj] = dv[jj].x;
      ti[jj] = dv[jj].y;
    }
    return r;
  };
  if (w == 0) pp = invert(ar[0], ai[0]);
  CR_STAMP(3);
#pragma unroll
  for (int kb = 0; kb < NT; ++kb) {
    double2(*P)[TSZ] = pan[kb & 1];
    double2(*Q)[TSZ] = pan[(kb + 1) & 1];   // next step's panel, filled during this step
    const bool has_next = kb + 1 < NT;
    if (kb == 0 && w == 0) {   // publish column 0; tile 0 holds P^-1 in the strided layout
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int o = (I == 0) ? lr * 17 + lk + 4 * rr : (lk + 4 * rr) * 17 + lr;
          P[I][o] = make_double2(ar[I][rr], ai[I][rr]);
        }
    }
    __syncthreads();
    CR_STAMP(4 + 3 * kb);
    // phase 1: the publisher reads P^-1; every other wave forms X = P^-1 A_kJ
    // from its tile kb; the lookahead wave hands X and its not-yet-updated
    // column tiles to the next panel (the other waves update them there, off
    // the lookahead's pivot chain)
    d4 br = {0.0, 0.0, 0.0, 0.0}, bim = {0.0, 0.0, 0.0, 0.0};
    d4 xr = {0.0, 0.0, 0.0, 0.0}, xi = {0.0, 0.0, 0.0, 0.0};
    if (w == kb) {   // P^-1 in the C layout, read back from the panel
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const double2 v = P[kb][(lk + 4 * rr) * 17 + lr];
        br[rr] = v.x;
        bim[rr] = v.y;
      }
    } else {
      d4 tr = ar[0], ti = ai[0];   // this wave's tile kb (off-diagonal: C layout)
#pragma unroll
      for (int I = 1; I < NT; ++I)
        if (I == kb) {
          tr = ar[I];
          ti = ai[I];
        }
      mma16_3m<false>(xr, xi, P[kb], tr, ti);
#pragma unroll
      for (int I = 0; I < NT; ++I)
        if (I == kb) {
          ar[I] = xr;
          ai[I] = xi;
        }
      if (has_next && w == kb + 1) {
#pragma unroll
        for (int I = 0; I < NT; ++I)
          if (I != kb + 1) {   // X (= new tile kb) and the old tiles I != kb, kb + 1
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
              Q[I][(lk + 4 * rr) * 17 + lr] = make_double2(ar[I][rr], ai[I][rr]);
          }
      }
    }
    if (has_next) __syncthreads();
    CR_STAMP(5 + 3 * kb);
    // phase 2
    if (w == kb) {
      // this wave's column: A_Ik <- -A_Ik P^-1, tile kb <- P^-1
#pragma unroll
      for (int I = 0; I < NT; ++I) {
        if (I != kb) {
          ar[I] = d4{0.0, 0.0, 0.0, 0.0};
          ai[I] = d4{0.0, 0.0, 0.0, 0.0};
          mma16_3m<true>(ar[I], ai[I], P[I], br, bim);
        } else {
          ar[I] = br;
          ai[I] = bim;
        }
      }
    } else if (has_next && w == kb + 1) {
      // next pivot: update the (transposed) diagonal tile, invert it, publish
      // it to the next panel in the strided layout; this wave's other tiles are
      // rebuilt from the panel when it publishes at step kb + 1
#pragma unroll
      for (int I = 0; I < NT; ++I)
        if (I == kb + 1) {
          mma16_3m_T<true>(ar[I], ai[I], P[I], xr, xi);
          pp = invert(ar[I], ai[I]);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) Q[I][lr * 17 + lk + 4 * rr] = make_double2(ar[I][rr], ai[I][rr]);
        }
    } else {
      if (has_next) {   // the lookahead column's tile w: Q[w] -= A_wk X_{kb+1}
        d4 yr, yi, cr, ci;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double2 v = Q[kb][(lk + 4 * rr) * 17 + lr];
          const double2 u = Q[w][(lk + 4 * rr) * 17 + lr];
          yr[rr] = v.x;
          yi[rr] = v.y;
          cr[rr] = u.x;
          ci[rr] = u.y;
        }
        mma16_3m<true>(cr, ci, P[w], yr, yi);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) Q[w][(lk + 4 * rr) * 17 + lr] = make_double2(cr[rr], ci[rr]);
      }
#pragma unroll
      for (int I = 0; I < NT; ++I)
        if (I != kb) {
          if (I == w && kb < w) mma16_3m_T<true>(ar[I], ai[I], P[I], xr, xi);   // still transposed
          else mma16_3m<true>(ar[I], ai[I], P[I], xr, xi);
        }
    }
    CR_STAMP(6 + 3 * kb);
  }
  // top half of the inverse: tile rows I < NT / 2
#pragma unroll
  for (int I = 0; I < NT / 2; ++I)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      Mo[(int64_t)(I * 16 + lk + 4 * rr) * BP + w * 16 + lr] = make_double2(ar[I][rr], ai[I][rr]);
  if (l == 0) ldw[w] = 0.5 * log(pp);
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < NT; ++k) t += ldw[k];
    ldpart[(int64_t)bi * nslots + slot[li]] = t;
  }
#ifdef CR_STAMPS
  if (stamp_on) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  CR_STAMP(28);
  CR_RSTAMP(30);
  CR_STAMP_AT(31, 1ull);
}

// the site guard of chain c (SiteGuard, dwhmc_internal.h): one workgroup
__device__ __forceinline__ void site_guard_wg(const SiteGuard& sg, int N, int c) {
  const double2* D = sg.Delta + (int64_t)c * 2 * N;
  bool over = false;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    double sm = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 v = D[sg.site4[4 * i + k]];
      sm += sqrt(fma(v.x, v.x, v.y * v.y));
    }
    over = over || !(sm <= sg.cap4);
  }
  if (over) *sg.flag = 1;
}

// gcol: the guard column's x (-1: no guard); arguments in first-use order
template <int NT>
__global__ __launch_bounds__(64 * NT) void k_cr_inv(double2* __restrict__ pool, int64_t item,
                                                    const int* __restrict__ blk,
                                                    const int* __restrict__ dst, int gcol,
                                                    const int* __restrict__ slot,
                                                    double* __restrict__ ldpart, int nslots,
                                                    SiteGuard sg, int N, int P) {
  __shared__ double2 pan[2][NT][16 * 17];
  __shared__ double ldw[NT];
  const int2 xy = xcd_grid2d();
  if (xy.x == gcol) {   // the guard column, pole 0 of each chain
    if (xy.y % P == 0) site_guard_wg(sg, N, xy.y / P);
    return;
  }
  cr_inv_wg<NT>(pool, item, xy.y, xy.x, blk, dst, slot, ldpart, nslots, pan, ldw);
}

// ---------------------------------------------------------------------------
// Level-0 inversions from the static particle block.  A level-0 diagonal
// block is D = [[A, B], [conj B, -conj A]] with A = h_row - i y (hopping,
// disorder, mu: Δ-independent) and B = Δ/2 (in-row pairing).  Its M-form
// inverse [[X, Y], [conj Y, -conj X]] follows from R = A^-1, kept per (row,
// pole) since context creation (k_cr_inv on the Δ = 0 blocks, out of place:
// top half [R | 0], ln|det D0| = 2 ln|det A|):
//   Z = R B,  S = A + B conj(Z)  (the Schur complement of -conj A in D),
//   X = S^-1,  Y = Z conj(X),  ln|det D| = ln|det A| + ln|det S|.
// i S has Hermitian part >= y I like i D (a Schur complement), so S needs no
// pivoting either.  S^-1 by 2 x 2 tile blocks (HP = 32): S00^-1 in registers,
// P = S00^-1 S01, Q = S10 S00^-1, T = S11 - S10 P, T^-1 in registers,
// X01 = -P T^-1, X10 = -T^-1 Q, X11 = T^-1, X00 = S00^-1 + P (T^-1 Q).  The
// serial chain is two 16 x 16 register inversions and six 16 x 16 tile
// products in five barrier-separated phases (the wave that inverts T forms
// its own P; X00 is formed from T^-1 directly) instead of four inversions and
// their panel updates (k_cr_inv<4>).  Wave w
// owns tile (w >> 1, w & 1) of every 32 x 32 matrix; tiles meet in LDS
// (row-major, stride 17); MFMA operands in the C layout as in mma16_3m.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void tile_to_lds(double2* T, const d4& cr, const d4& ci) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) T[(lk + 4 * rr) * 17 + lr] = make_double2(cr[rr], ci[rr]);
}
// C-layout registers of an LDS tile; CONJ: of its complex conjugate
template <bool CONJ = false>
__device__ __forceinline__ void tile_from_lds(const double2* T, d4& cr, d4& ci) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const double2 v = T[(lk + 4 * rr) * 17 + lr];
    cr[rr] = v.x;
    ci[rr] = CONJ ? -v.y : v.y;
  }
}

// site guard of launch_cr_inv0 (Σ_k |Δ| over each site's four bonds <= cap4)
__device__ __forceinline__ void inv0_site_guard(const double2* __restrict__ D, const int* __restrict__ site4,
                                                int N, double cap4, int* __restrict__ flag) {
  bool over = false;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    double sm = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 v = D[site4[4 * i + k]];
      sm += sqrt(fma(v.x, v.x, v.y * v.y));
    }
    over = over || !(sm <= cap4);
  }
  if (over) *flag = 1;
}

// gcol: the guard column's x (-1: no guard); arguments in first-use order
__global__ __launch_bounds__(256) void k_cr_inv0(double2* __restrict__ pool, int64_t item,
                                                 const int* __restrict__ blk, const int* __restrict__ rblk,
                                                 const int* __restrict__ dst, int gcol,
                                                 const int* __restrict__ slot, double* __restrict__ ldpart,
                                                 const double* __restrict__ ldA, int nslots,
                                                 const double2* __restrict__ Delta,
                                                 const int* __restrict__ site4, int N, int P, double cap4,
                                                 int* __restrict__ flag) {
  constexpr int BP = 64, HP = 32, TSZ = 16 * 17;
  __shared__ double2 sR[4][TSZ], sB[4][TSZ], sZ[4][TSZ], sS[4][TSZ], sX[4][TSZ], sA[4][TSZ];
  __shared__ double ldw[2];
  const int2 xy = xcd_grid2d();
  const int bi = xy.y, li = xy.x;
  CR_STAMP_INIT(blk);
  CR_RSTAMP(0);
  // site guard (launch_cr_inv0 with Delta): the extra last workgroup column,
  // pole 0 of each chain, on a CU the inversions leave idle
  if (li == gcol) {
    if (bi % P == 0) inv0_site_guard(Delta + (int64_t)(bi / P) * 2 * N, site4, N, cap4, flag);
    CR_RSTAMP(30);
    CR_STAMP_AT(31, 3ull);
    return;
  }
  const double2* D = pool + (int64_t)bi * item + (int64_t)blk[li] * HP * BP;
  const double2* Rm = pool + (int64_t)bi * item + (int64_t)rblk[li] * HP * BP;
  double2* Mo = pool + (int64_t)bi * item + (int64_t)dst[li] * HP * BP;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int ti = w >> 1, tj = w & 1;
  CR_STAMP(1);
  // this wave's tiles: A (C layout, registers), R and B (LDS)
  d4 acr, aci;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = ti * 16 + lk + 4 * rr, col = tj * 16 + lr;
    const double2 a = D[(int64_t)row * BP + col];
    const double2 b = D[(int64_t)row * BP + HP + col];
    const double2 r = Rm[(int64_t)row * BP + col];
    acr[rr] = a.x;
    aci[rr] = a.y;
    sB[w][(lk + 4 * rr) * 17 + lr] = b;
    sR[w][(lk + 4 * rr) * 17 + lr] = r;
  }
  __syncthreads();
  CR_STAMP(2);
  // Z = R B
  d4 zr = {0.0, 0.0, 0.0, 0.0}, zi = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    d4 br, bim;
    tile_from_lds(sB[2 * k + tj], br, bim);
    mma16_3m<false>(zr, zi, sR[2 * ti + k], br, bim);
  }
  tile_to_lds(sZ[w], zr, zi);
  __syncthreads();
  CR_STAMP(3);
  // S = A + B conj(Z)
  d4 sr = acr, si = aci;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    d4 br, bim;
    tile_from_lds<true>(sZ[2 * k + tj], br, bim);
    mma16_3m<false>(sr, si, sB[2 * ti + k], br, bim);
  }
  double pp = 1.0;   // Π |pivot|^2 (waves 0, 3); the log after the chain
  if (w == 0) pp = wave_inv16_c(sr, si);   // S00^-1 (C layout in, C layout out)
  tile_to_lds(sS[w], sr, si);                           // S00^-1, S01, S10, S11
  __syncthreads();
  CR_STAMP(4);
  // P = S00^-1 S01 (wave 1, sA[1]); Q = S10 S00^-1 (wave 2, registers + sA[2]);
  // wave 3 forms P itself (no barrier in its chain), T = S11 - S10 P and T^-1
  d4 qr = {0.0, 0.0, 0.0, 0.0}, qi = {0.0, 0.0, 0.0, 0.0};
  if (w == 1) {
    d4 pr = {0.0, 0.0, 0.0, 0.0}, pi = {0.0, 0.0, 0.0, 0.0};
    mma16_3m<false>(pr, pi, sS[0], sr, si);
    tile_to_lds(sA[1], pr, pi);
  } else if (w == 2) {
    d4 br, bim;
    tile_from_lds(sS[0], br, bim);
    mma16_3m<false>(qr, qi, sS[2], br, bim);
    tile_to_lds(sA[2], qr, qi);
  } else if (w == 3) {
    d4 br, bim, pr = {0.0, 0.0, 0.0, 0.0}, pi = {0.0, 0.0, 0.0, 0.0};
    tile_from_lds(sS[1], br, bim);
    mma16_3m<false>(pr, pi, sS[0], br, bim);   // P
    mma16_3m<true>(sr, si, sS[2], pr, pi);     // T = S11 - S10 P
    pp = wave_inv16_c(sr, si);
    tile_to_lds(sX[3], sr, si);
  }
  __syncthreads();
  CR_STAMP(5);
  // X01 = -P T^-1 (wave 1), X10 = -T^-1 Q (wave 2), X00 = S00^-1 + P (T^-1 Q)
  // (wave 0; = S00^-1 - X01 Q), X11 = T^-1 (wave 3)
  d4 xr = sr, xi = si;   // wave 0: S00^-1; wave 3: T^-1 = X11
  if (w == 1) {
    d4 br, bim;
    tile_from_lds(sX[3], br, bim);
    xr = d4{0.0, 0.0, 0.0, 0.0};
    xi = d4{0.0, 0.0, 0.0, 0.0};
    mma16_3m<true>(xr, xi, sA[1], br, bim);
    tile_to_lds(sX[1], xr, xi);
  } else if (w == 2) {
    xr = d4{0.0, 0.0, 0.0, 0.0};
    xi = d4{0.0, 0.0, 0.0, 0.0};
    mma16_3m<true>(xr, xi, sX[3], qr, qi);
    tile_to_lds(sX[2], xr, xi);
  } else if (w == 0) {
    d4 br, bim, ur = {0.0, 0.0, 0.0, 0.0}, ui = {0.0, 0.0, 0.0, 0.0};
    tile_from_lds(sA[2], br, bim);
    mma16_3m<false>(ur, ui, sX[3], br, bim);   // U = T^-1 Q
    mma16_3m<false>(xr, xi, sA[1], ur, ui);    // X00 = S00^-1 + P U
    tile_to_lds(sX[0], xr, xi);
  }
  __syncthreads();
  CR_STAMP(6);
  // Y = Z conj(X)
  d4 yr = {0.0, 0.0, 0.0, 0.0}, yi = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    d4 br, bim;
    tile_from_lds<true>(sX[2 * k + tj], br, bim);
    mma16_3m<false>(yr, yi, sZ[2 * ti + k], br, bim);
  }
  CR_STAMP(7);
  // top half of D^-1 = [X | Y]
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = ti * 16 + lk + 4 * rr, col = tj * 16 + lr;
    Mo[(int64_t)row * BP + col] = make_double2(xr[rr], xi[rr]);
    Mo[(int64_t)row * BP + HP + col] = make_double2(yr[rr], yi[rr]);
  }
  if (l == 0 && (w == 0 || w == 3)) ldw[w == 3] = 0.5 * log(pp);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t o = (int64_t)bi * nslots + slot[li];
    ldpart[o] = 0.5 * ldA[o] + ldw[0] + ldw[1];
  }
#ifdef CR_STAMPS
  if (stamp_on) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  CR_STAMP(28);
  CR_RSTAMP(30);
  CR_STAMP_AT(31, 1ull);
}

// HP = 48 (BP = 96): 3 x 3 tiles, one wave per tile (9 waves).  Z = R B,
// S = A + B conj(Z) as tile products; S^-1 by block Gauss-Jordan over the
// three diagonal tiles (pivot p: its wave inverts S_pp in registers, row p
// <- S_pp^-1 S_pj, the rest S_ij -= S_ip S_pj, column p <- -S_ip S_pp^-1;
// tiles meet in two alternating LDS buffers); Y = Z conj(X).  Three 16 x 16
// register inversions on the chain instead of k_cr_inv<6>'s six, and a
// quarter of its flops.  The R and B tiles' LDS becomes the Gauss-Jordan
// buffers once S is formed.
__global__ __launch_bounds__(576) void k_cr_inv0_96(double2* __restrict__ pool, int64_t item,
                                                    const int* __restrict__ blk, const int* __restrict__ rblk,
                                                    const int* __restrict__ dst, int gcol,
                                                    const int* __restrict__ slot, double* __restrict__ ldpart,
                                                    const double* __restrict__ ldA, int nslots,
                                                    const double2* __restrict__ Delta,
                                                    const int* __restrict__ site4, int N, int P, double cap4,
                                                    int* __restrict__ flag) {
  constexpr int BP = 96, HP = 48, TSZ = 16 * 17;
  __shared__ double2 sZ[9][TSZ], s1[9][TSZ], s2[9][TSZ], sP[TSZ];
  __shared__ double ldw[3];
  const int2 xy = xcd_grid2d();
  const int bi = xy.y, li = xy.x;
  if (li == gcol) {
    if (bi % P == 0) inv0_site_guard(Delta + (int64_t)(bi / P) * 2 * N, site4, N, cap4, flag);
    return;
  }
  const double2* D = pool + (int64_t)bi * item + (int64_t)blk[li] * HP * BP;
  const double2* Rm = pool + (int64_t)bi * item + (int64_t)rblk[li] * HP * BP;
  double2* Mo = pool + (int64_t)bi * item + (int64_t)dst[li] * HP * BP;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int ti = w / 3, tj = w - 3 * (w / 3);
  d4 sr, si;   // A, then S, then (S^-1) tile (ti, tj)
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = ti * 16 + lk + 4 * rr, col = tj * 16 + lr;
    const double2 a = D[(int64_t)row * BP + col];
    s2[w][(lk + 4 * rr) * 17 + lr] = D[(int64_t)row * BP + HP + col];   // B
    s1[w][(lk + 4 * rr) * 17 + lr] = Rm[(int64_t)row * BP + col];       // R
    sr[rr] = a.x;
    si[rr] = a.y;
  }
  __syncthreads();
  d4 br, bim, zr = {0.0, 0.0, 0.0, 0.0}, zi = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {   // Z = R B
    tile_from_lds(s2[3 * k + tj], br, bim);
    mma16_3m<false>(zr, zi, s1[3 * ti + k], br, bim);
  }
  tile_to_lds(sZ[w], zr, zi);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 3; ++k) {   // S = A + B conj(Z)
    tile_from_lds<true>(sZ[3 * k + tj], br, bim);
    mma16_3m<false>(sr, si, s2[3 * ti + k], br, bim);
  }
  tile_to_lds(s1[w], sr, si);   // R is dead (read only before the last barrier)
  __syncthreads();
  double pp = 1.0;   // Π |pivot|^2 of the diagonal waves; the log after the chain
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    double2(*cur)[TSZ] = (p & 1) ? s2 : s1;
    double2(*nxt)[TSZ] = (p & 1) ? s1 : s2;
    if (ti == p && tj == p) {
      pp = wave_inv16_c(sr, si);
      tile_to_lds(sP, sr, si);
    }
    __syncthreads();
    if (ti == p && tj != p) {   // row p <- S_pp^-1 S_pj
      d4 nr = {0.0, 0.0, 0.0, 0.0}, ni = {0.0, 0.0, 0.0, 0.0};
      mma16_3m<false>(nr, ni, sP, sr, si);
      sr = nr;
      si = ni;
      tile_to_lds(cur[w], sr, si);
    }
    __syncthreads();
    if (ti != p && tj != p) {   // S_ij -= S_ip S_pj (old column p, new row p)
      tile_from_lds(cur[3 * p + tj], br, bim);
      mma16_3m<true>(sr, si, cur[3 * ti + p], br, bim);
    } else if (ti != p) {       // column p <- -S_ip S_pp^-1
      d4 nr = {0.0, 0.0, 0.0, 0.0}, ni = {0.0, 0.0, 0.0, 0.0};
      tile_from_lds(sP, br, bim);
      mma16_3m<true>(nr, ni, cur[w], br, bim);
      sr = nr;
      si = ni;
    }
    tile_to_lds(nxt[w], sr, si);
    __syncthreads();
  }
  // X = S^-1 in s2 (p = 2 wrote nxt = s2); Y = Z conj(X)
  d4 yr = {0.0, 0.0, 0.0, 0.0}, yi = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    tile_from_lds<true>(s2[3 * k + tj], br, bim);
    mma16_3m<false>(yr, yi, sZ[3 * ti + k], br, bim);
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = ti * 16 + lk + 4 * rr, col = tj * 16 + lr;
    Mo[(int64_t)row * BP + col] = make_double2(sr[rr], si[rr]);
    Mo[(int64_t)row * BP + HP + col] = make_double2(yr[rr], yi[rr]);
  }
  if (l == 0 && ti == tj) ldw[ti] = 0.5 * log(pp);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t o = (int64_t)bi * nslots + slot[li];
    ldpart[o] = 0.5 * ldA[o] + ldw[0] + ldw[1] + ldw[2];
  }
}

// HP = 16 (BP = 32): every matrix is one tile and one wave does the whole
// chain: Z = R B, S = A + B conj(Z), S^-1 (one register inversion), Y = Z
// conj(X) -- one 16 x 16 inversion and three tile products where k_cr_inv<2>
// runs two inversions and their panel updates.  LDS only carries tiles
// between the wave's own lanes (the barriers are wave-local).
// STATIC: R = A^-1 from the static block rblk (ln|det A| = ldA / 2); else R
// is A^-1 formed here (k_cr_inv32: any M-form block, the same Schur
// complement after one more register inversion; no pivoting, as i A is a
// principal block of i D).  In place when dst == blk: every read precedes
// the wave's first store.
template <bool STATIC>
__device__ __forceinline__ void cr_inv32_wave(double2* __restrict__ pool, int64_t item, int bi, int li,
                                              const int* __restrict__ blk, const int* __restrict__ rblk,
                                              const int* __restrict__ dst, const int* __restrict__ slot,
                                              double* __restrict__ ldpart, const double* __restrict__ ldA,
                                              int nslots) {
  constexpr int BP = 32, HP = 16, TSZ = 16 * 17;
  __shared__ double2 sR[TSZ], sB[TSZ], sZ[TSZ], sX[TSZ];
  const double2* D = pool + (int64_t)bi * item + (int64_t)blk[li] * HP * BP;
  double2* Mo = pool + (int64_t)bi * item + (int64_t)dst[li] * HP * BP;
  const int l = threadIdx.x, lr = l & 15, lk = l >> 4;
  d4 sr, si;   // A, then S, then X = S^-1
  double ld = 0.0, pa = 1.0;   // pa, ps: Π |pivot|^2 of A and S (their logs after the chain)
  if constexpr (STATIC) {
    const double2* Rm = pool + (int64_t)bi * item + (int64_t)rblk[li] * HP * BP;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = lk + 4 * rr;
      const double2 a = D[(int64_t)row * BP + lr];
      sB[row * 17 + lr] = D[(int64_t)row * BP + HP + lr];
      sR[row * 17 + lr] = Rm[(int64_t)row * BP + lr];
      sr[rr] = a.x;
      si[rr] = a.y;
    }
    ld = 0.5 * ldA[(int64_t)bi * nslots + slot[li]];
  } else {
    d4 rr_, ri_;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = lk + 4 * rr;
      const double2 a = D[(int64_t)row * BP + lr];
      sB[row * 17 + lr] = D[(int64_t)row * BP + HP + lr];
      sr[rr] = rr_[rr] = a.x;
      si[rr] = ri_[rr] = a.y;
    }
    pa = wave_inv16_c(rr_, ri_);   // R = A^-1
    tile_to_lds(sR, rr_, ri_);
  }
  __syncthreads();
  d4 br, bim, zr = {0.0, 0.0, 0.0, 0.0}, zi = {0.0, 0.0, 0.0, 0.0};
  tile_from_lds(sB, br, bim);
  mma16_3m<false>(zr, zi, sR, br, bim);   // Z = R B
  tile_to_lds(sZ, zr, zi);
  __syncthreads();
  tile_from_lds<true>(sZ, br, bim);
  mma16_3m<false>(sr, si, sB, br, bim);   // S = A + B conj(Z)
  const double ps = wave_inv16_c(sr, si);
  tile_to_lds(sX, sr, si);
  __syncthreads();
  d4 yr = {0.0, 0.0, 0.0, 0.0}, yi = {0.0, 0.0, 0.0, 0.0};
  tile_from_lds<true>(sX, br, bim);
  mma16_3m<false>(yr, yi, sZ, br, bim);   // Y = Z conj(X)
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = lk + 4 * rr;
    Mo[(int64_t)row * BP + lr] = make_double2(sr[rr], si[rr]);
    Mo[(int64_t)row * BP + HP + lr] = make_double2(yr[rr], yi[rr]);
  }
  if (l == 0) ldpart[(int64_t)bi * nslots + slot[li]] = ld + 0.5 * (log(pa) + log(ps));
}

__global__ __launch_bounds__(64) void k_cr_inv0_32(double2* __restrict__ pool, int64_t item,
                                                   const int* __restrict__ blk, const int* __restrict__ rblk,
                                                   const int* __restrict__ dst, int gcol,
                                                   const int* __restrict__ slot, double* __restrict__ ldpart,
                                                   const double* __restrict__ ldA, int nslots,
                                                   const double2* __restrict__ Delta,
                                                   const int* __restrict__ site4, int N, int P, double cap4,
                                                   int* __restrict__ flag) {
  const int2 xy = xcd_grid2d();
  const int bi = xy.y, li = xy.x;
  if (li == gcol) {
    if (bi % P == 0) inv0_site_guard(Delta + (int64_t)(bi / P) * 2 * N, site4, N, cap4, flag);
    return;
  }
  cr_inv32_wave<true>(pool, item, bi, li, blk, rblk, dst, slot, ldpart, ldA, nslots);
}

// gcol: the guard column's x (-1: no guard), as k_cr_inv
__global__ __launch_bounds__(64) void k_cr_inv32(double2* __restrict__ pool, int64_t item,
                                                 const int* __restrict__ blk, const int* __restrict__ dst,
                                                 int gcol, const int* __restrict__ slot,
                                                 double* __restrict__ ldpart, int nslots, SiteGuard sg, int N,
                                                 int P) {
  const int2 xy = xcd_grid2d();
  const int bi = xy.y, li = xy.x;
  if (li == gcol) {
    if (bi % P == 0) site_guard_wg(sg, N, bi / P);
    return;
  }
  cr_inv32_wave<false>(pool, item, bi, li, blk, nullptr, dst, slot, ldpart, nullptr, nslots);
}

// ---------------------------------------------------------------------------
// Batched block products on top halves: task t of batch item bi writes
//   out = [cin] + sg Σ_{h < nt} A_h B_h      (top halves, HP x BP)
// K runs over all BP rows of B_h: rows 0..HP-1 are stored, rows HP..BP-1 are
// synthesised as sgn * conj(B_top[k - HP, (j + HP) mod BP]) with sgn from the
// term's form bit (CrTask::bq) and the column half of the output tile.
// Complex MACs use three real MFMAs (v_mfma_f64_16x16x4_f64):
//   t1 += ar br,  t2 += ai bi,  t3 += (ar + ai)(br + bi);
//   re = t1 - t2,  im = t3 - t1 - t2
// Output tiles are TS x TS (TS = 16 MI).  KSPLIT waves of a workgroup share a
// tile, each running 1/KSPLIT of every term's K range (short serial MFMA
// chains for the latency-bound coarse stages); their partials are summed
// through LDS.  KSPLIT = 1: four independent tiles per workgroup, no LDS, no
// barriers.  MFMA fragments come straight from L2 with a register prefetch;
// 1D grid with the XCD-aware remap so one item's tasks share an XCD's L2.
// out never aliases an operand (planner invariant); out == cin is allowed.
// ---------------------------------------------------------------------------
// minimum waves per SIMD the 16 x 16 tile kernels are compiled for, and their
// operand prefetch depth in k-steps
#ifndef CR_GEMM_WAVES
#define CR_GEMM_WAVES 2
#endif
#ifndef CR_GEMM_PF
#define CR_GEMM_PF 4
#endif
constexpr int kGemmWaves = CR_GEMM_WAVES, kGemmPf = CR_GEMM_PF;
// -DCR_GEMM_4M=1 (A/B builds): complex MACs as four real MFMAs with no fp64
// VALU in the K loop, instead of 3M's three plus two fp64 adds per k-step
#ifndef CR_GEMM_4M
#define CR_GEMM_4M 0
#endif

__device__ __forceinline__ double flip_sign(double x, unsigned m) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  return __builtin_bit_cast(double, b ^ ((unsigned long long)m << 32));
}

// One term's K range of this wave: t1 += Ar Br, t2 += Ai Bi, t3 += (Ar + Ai)(Br + Bi).
// Synthesised B rows are sgn * conj(u): Br = sgn ux, Bi = -sgn uy,
// Br + Bi = sgn (ux - uy).  The signs are applied by flipping the sign bit
// with a 32-bit integer XOR (smask = 0x80000000 when sgn < 0), not by fp64
// multiplies: fp64 VALU ops share the DP pipe with the f64 MFMAs and stall
// it (tools/micro/mfma_valu_coexec.hip: ~10-15 cycles per interleaved
// v_mul/v_add_f64).  The products are the ones the explicit sign multiplies
// gave, bit for bit.
template <int BP, int MI, int KSPLIT, int KQ, int PFX = 0>
__device__ __forceinline__ void cr_term(const double2* A, const double2* Bt, int c0, int crot, unsigned smask,
                                        d4 (&t1)[MI][MI], d4 (&t2)[MI][MI], d4 (&t3)[MI][MI]) {
  constexpr int HP = BP / 2, KS = BP / 4, KH = HP / 4, KSS = KS / KSPLIT, S0 = KQ * KSS;
  constexpr int PFD = PFX > 0 ? PFX : (MI == 1 ? kGemmPf : 2);
  constexpr int PF = KSS < PFD ? KSS : PFD;
  auto load = [&](int s, double2 (&a)[MI], double2 (&b)[MI]) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) a[mi] = A[(int64_t)16 * mi * BP + s * 4];
#pragma unroll
    for (int ni = 0; ni < MI; ++ni)
      b[ni] = s < KH ? Bt[(int64_t)s * 4 * BP + c0 + 16 * ni] : Bt[(int64_t)(s - KH) * 4 * BP + crot + 16 * ni];
  };
  double2 fa[PF][MI], fb[PF][MI];
#pragma unroll
  for (int p = 0; p < PF; ++p) load(S0 + p, fa[p], fb[p]);
#pragma unroll
  for (int j = 0; j < KSS; ++j) {
    const int cs = j % PF;
    const bool syn = S0 + j >= KH;   // compile time
    double ar[MI], ai[MI], br[MI], bi[MI];
#if !CR_GEMM_4M
    double as[MI], bs[MI];
#endif
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      ar[mi] = fa[cs][mi].x;
      ai[mi] = fa[cs][mi].y;
      if (syn) {
        const double ux = fb[cs][mi].x, uy = fb[cs][mi].y;
        br[mi] = flip_sign(ux, smask);
        bi[mi] = flip_sign(uy, smask ^ 0x80000000u);
      } else {
        br[mi] = fb[cs][mi].x;
        bi[mi] = fb[cs][mi].y;
      }
#if !CR_GEMM_4M
      as[mi] = ar[mi] + ai[mi];
      bs[mi] = syn ? flip_sign(fb[cs][mi].x - fb[cs][mi].y, smask) : br[mi] + bi[mi];
#endif
    }
    if (j + PF < KSS) load(S0 + j + PF, fa[cs], fb[cs]);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < MI; ++ni) {
#if CR_GEMM_4M
        // four real products, no fp64 VALU: t3 collects both cross terms
        t1[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], t1[mi][ni], 0, 0, 0);
        t3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], bi[ni], t3[mi][ni], 0, 0, 0);
        t2[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], bi[ni], t2[mi][ni], 0, 0, 0);
        t3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], br[ni], t3[mi][ni], 0, 0, 0);
#else
        t1[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], t1[mi][ni], 0, 0, 0);
        t2[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], bi[ni], t2[mi][ni], 0, 0, 0);
        t3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(as[mi], bs[ni], t3[mi][ni], 0, 0, 0);
#endif
      }
  }
}

// This wave's share of a 32 x 32 output tile of task tk over all its terms
// (the stage sign sg is applied in the epilogue: negating every A fragment
// negates the sums exactly); operand fields read through the uniform pointer
template <int BP, int MI, int KSPLIT, int KQ, int PFX = 0>
__device__ __forceinline__ void cr_tile_part(const double2* base, const CrTask* __restrict__ tk, int tr, int tc,
                                             d4 (&t1)[MI][MI], d4 (&t2)[MI][MI], d4 (&t3)[MI][MI]) {
  constexpr int TS = 16 * MI, HP = BP / 2;
  constexpr int64_t BB = (int64_t)HP * BP;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int c0 = tc * TS, crot = c0 < HP ? c0 + HP : c0 - HP;
  const int nt = tk->nt, bq = tk->bq;
#pragma unroll 1
  for (int h = 0; h < nt; ++h) {
    const double2* A = base + tk->a[h] * BB + (int64_t)(tr * TS + lr) * BP + lk;
    const double2* Bt = base + tk->b[h] * BB + (int64_t)lk * BP + lr;
    // synthesised rows: sgn * conj(.), sgn = -s (left column half) / +s (right), s = +1 Q, -1 M
    const bool q = (bq >> h) & 1;
    const unsigned smask = ((c0 < HP) == q) ? 0x80000000u : 0u;   // sgn < 0
    cr_term<BP, MI, KSPLIT, KQ, PFX>(A, Bt, c0, crot, smask, t1, t2, t3);
  }
}

// register slot v = (mi MI + ni) 4 + rr of a wave's TS x TS output share <->
// element offset from the lane's own output element
template <int BP, int MI>
__device__ __forceinline__ int64_t cr_slot_off(int v) {
  const int mi = v / (MI * 4), ni = (v / 4) % MI, rr = v % 4;
  return (int64_t)(mi * 16 + 4 * rr) * BP + ni * 16;
}

// Epilogue of both descriptor forms: out = [C] + sg (t1 - t2, t3 - t1 - t2)
// at O (the lane's first output element; C likewise, cpf its values loaded at
// tile start).  KSPLIT > 1: the waves of a tile sum their partials through LDS
// (every wave of the workgroup reaches the barrier, valid or not).
template <int BP, int MI, int KSPLIT>
__device__ __forceinline__ void cr_tile_store(d4 (&t1)[MI][MI], d4 (&t2)[MI][MI], d4 (&t3)[MI][MI], double sg,
                                              double2* O, bool hasc, const double2 (&cpf)[MI * MI * 4 / KSPLIT],
                                              bool valid, [[maybe_unused]] bool stamp = false) {
  constexpr int NV = MI * MI * 4;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, kq = w % KSPLIT;
  auto put = [&](int v, double2 x) {
    if (hasc) {
      const double2 c = cpf[v / KSPLIT];
      x.x += c.x;
      x.y += c.y;
    }
    O[cr_slot_off<BP, MI>(v)] = x;
  };
  // complex partial of register slot v
  auto partial = [&](int v) {
    const int mi = v / (MI * 4), ni = (v / 4) % MI, rr = v % 4;
    const double a = t1[mi][ni][rr], b = t2[mi][ni][rr], c = t3[mi][ni][rr];
#if CR_GEMM_4M
    return make_double2(sg * (a - b), sg * c);
#else
    return make_double2(sg * (a - b), sg * (c - a - b));
#endif
  };
  if constexpr (KSPLIT == 1) {
    if (!valid) return;
#pragma unroll
    for (int v = 0; v < NV; ++v) put(v, partial(v));
  } else {
    __shared__ double2 red[4][NV][64];
#pragma unroll
    for (int v = 0; v < NV; ++v) red[w][v][l] = partial(v);
#ifdef CR_GEMM_STAMPS
    if (stamp) __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    GEMM_STAMP(3, stamp);
#endif
    __syncthreads();
#ifdef CR_GEMM_STAMPS
    GEMM_STAMP(4, stamp);
#endif
    if (!valid) return;
    const int g0 = w - kq;   // first wave of this tile's group
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (v % KSPLIT != kq) continue;
      double2 x = red[g0][v][l];
#pragma unroll
      for (int k = 1; k < KSPLIT; ++k) {
        const double2 y = red[g0 + k][v][l];
        x.x += y.x;
        x.y += y.y;
      }
      put(v, x);
    }
  }
}

// The accumulate input of the lane's slots (v % KSPLIT == kq), loaded at
// tile start so its latency overlaps the operand loads
template <int BP, int MI, int KSPLIT>
__device__ __forceinline__ void cr_tile_cin(const double2* C, double2 (&cpf)[MI * MI * 4 / KSPLIT]) {
  const int kq = (threadIdx.x >> 6) % KSPLIT;
#pragma unroll
  for (int i = 0; i < MI * MI * 4 / KSPLIT; ++i) cpf[i] = C[cr_slot_off<BP, MI>(i * KSPLIT + kq)];
}

// One workgroup's share of a 32 x 32 product stage (task list; side work of
// the inversion launches and the DWHMC_CR_GEMM=32 A/B configurations):
// workgroup slot g of the 1D grid (already XCD-remapped by the caller) covers
// tiles g * TPW .. + TPW - 1 of ntasks x maxt task slots per batch item.
// TILESIGN: each task's sign from its descriptor (kCrNegBit; side-work task
// lists mix stages of both signs) instead of sg.  PFX: operand prefetch depth
// in k-steps (0: the default).
template <int BP, int MI, int KSPLIT, int PFX = 0, bool TILESIGN = false>
__device__ __forceinline__ void cr_gemm_wg(double2* __restrict__ pool, int64_t item,
                                           const CrTask* __restrict__ tasks, int ntasks, int maxt, int total,
                                           double sg, int g) {
  static_assert(MI == 2, "16 x 16 stages run k_cr_gemm16 (dispatch-ordered slots)");
  constexpr int TS = 16 * MI, TPW = 4 / KSPLIT, HP = BP / 2, NV = MI * MI * 4;
  constexpr int64_t BB = (int64_t)HP * BP;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int kq = w % KSPLIT;
  const int gt = __builtin_amdgcn_readfirstlane(g * TPW + w / KSPLIT);
  const int per_item = ntasks * maxt;
  const int bi = gt / per_item;
  const int rmd = gt - bi * per_item;
  bool valid = gt < total;
  const int tsk = rmd / maxt, tile = rmd - tsk * maxt;
  const CrTask* tk = tasks + (valid ? tsk : 0);
  if constexpr (TILESIGN) sg = (tk->bq & kCrNegBit) ? -1.0 : 1.0;
  const int tr0 = tk->r0 / TS, tc0 = tk->c0 / TS;
  const int ct = (tk->c1 + TS - 1) / TS - tc0;
  const int rt = (tk->r1 + TS - 1) / TS - tr0;
  valid = valid && tile < rt * ct;   // restricted task: fewer tiles than the stage maximum
  const int tr = tr0 + (valid ? tile / ct : 0);
  const int tc = tc0 + (valid ? tile % ct : 0);
  const int cin = tk->cin, out = tk->out;
  double2* base = pool + (int64_t)(valid ? bi : 0) * item;
  d4 t1[MI][MI], t2[MI][MI], t3[MI][MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < MI; ++ni) {
      t1[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
      t2[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
      t3[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
    }
  double2* O = base + out * BB + (int64_t)(tr * TS + lk) * BP + tc * TS + lr;
  const bool hasc = cin >= 0;
  double2 cpf[NV / KSPLIT];
#pragma unroll
  for (int i = 0; i < NV / KSPLIT; ++i) cpf[i] = make_double2(0.0, 0.0);
  if (hasc && valid) cr_tile_cin<BP, MI, KSPLIT>(base + cin * BB + (int64_t)(tr * TS + lk) * BP + tc * TS + lr, cpf);
  auto run = [&](auto kqc) {
    constexpr int KQ = decltype(kqc)::value;
    cr_tile_part<BP, MI, KSPLIT, KQ, PFX>(base, tk, tr, tc, t1, t2, t3);
  };
  if (valid) {
    if (KSPLIT == 1 || kq == 0) run(std::integral_constant<int, 0>{});
    if constexpr (KSPLIT >= 2) {
      if (kq == 1) run(std::integral_constant<int, 1>{});
    }
  }
  cr_tile_store<BP, MI, KSPLIT>(t1, t2, t3, sg, O, hasc, cpf, valid);
}

// Argument order: what the first loads need leads (the build preloads the
// leading kernel-argument dwords into SGPRs, build.py), and the grid size is
// an argument (gridDim is a hidden argument, read by an s_load)
template <int BP, int MI, int KSPLIT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_cr_gemm(double2* __restrict__ pool, int64_t item,
                                                 int total, double sg, int nwg, int ntasks, int maxt,
                                                 const CrTask* __restrict__ tasks) {
  cr_gemm_wg<BP, MI, KSPLIT>(pool, item, tasks, ntasks, maxt, total, sg, xcd_remap(blockIdx.x, nwg));
}

// 16 x 16 output tiles from dispatch-ordered slots (CrSlot: the host did the
// XCD remap, the batch-item split and every block / tile address): wave w
// of workgroup b takes slot b * TPW + w / KSPLIT with one 64-byte scalar load
// and issues its operand loads right after it.  Empty slots (out == kCrNone)
// pad the last workgroup.
template <int BP, int KSPLIT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kGemmWaves))) void k_cr_gemm16(
    double2* __restrict__ pool, const CrSlot* __restrict__ slots, double sg) {
  constexpr int TPW = 4 / KSPLIT, NV = 4;
  // the wave index as a scalar: the K-quarter dispatch below branches on SCC
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int kq = w % KSPLIT;
#ifdef CR_GEMM_STAMPS
  const bool g_gemm_on = (int)(gridDim.x * TPW) == g_gemm_sel;
  GEMM_STAMP(0, g_gemm_on);
  GEMM_STAMP(1, g_gemm_on);
  if (g_gemm_on && threadIdx.x == 0 && blockIdx.x < 65536)
    g_gemm_stamps[blockIdx.x][7] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
#endif
  // the whole slot in one s_load_dwordx16 (CrSlot field order: base lo / hi,
  // out, cin, nt, smask, a[4], b[4], rot)
  typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
  const u32x16 d = *reinterpret_cast<const u32x16*>(slots + (blockIdx.x * TPW + w / KSPLIT));
  const uint32_t out = d[2], cin = d[3];
  const bool valid = out != kCrNone;
  double2* base = pool + (((uint64_t)d[1] << 32) | d[0]);
  d4 t1[1][1], t2[1][1], t3[1][1];
  t1[0][0] = d4{0.0, 0.0, 0.0, 0.0};
  t2[0][0] = d4{0.0, 0.0, 0.0, 0.0};
  t3[0][0] = d4{0.0, 0.0, 0.0, 0.0};
#ifdef CR_GEMM_STAMPS
  if (g_gemm_on) __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  GEMM_STAMP(2, g_gemm_on);
#endif
  const int lo = lk * BP + lr;   // the lane's first output element in a tile
  const bool hasc = cin != kCrNone;
  double2 cpf[NV / KSPLIT];
#pragma unroll
  for (int i = 0; i < NV / KSPLIT; ++i) cpf[i] = make_double2(0.0, 0.0);
  if (hasc && valid) cr_tile_cin<BP, 1, KSPLIT>(base + cin + lo, cpf);
  auto run = [&](auto kqc) {
    constexpr int KQ = decltype(kqc)::value;
    const int nt = (int)d[4], rot = (int)d[14];
    // the terms' operands rotate through scalar registers (a dynamic index
    // into the slot would be lowered to VGPR-indexed moves)
    uint32_t a0 = d[6], a1 = d[7], a2 = d[8], a3 = d[9], b0 = d[10], b1 = d[11], b2 = d[12], b3 = d[13];
    unsigned sm = d[5];
#pragma unroll 1
    for (int h = 0; h < nt; ++h) {
      cr_term<BP, 1, KSPLIT, KQ>(base + a0 + (lr * BP + lk), base + b0 + lo, 0, rot, (sm & 1u) << 31, t1, t2, t3);
      a0 = a1;
      a1 = a2;
      a2 = a3;
      b0 = b1;
      b1 = b2;
      b2 = b3;
      sm >>= 1;
    }
  };
  if (valid) {
    if (KSPLIT == 1 || kq == 0) run(std::integral_constant<int, 0>{});
    if constexpr (KSPLIT >= 2) {
      if (kq == 1) run(std::integral_constant<int, 1>{});
    }
    if constexpr (KSPLIT == 4) {
      if (kq == 2) run(std::integral_constant<int, 2>{});
      if (kq == 3) run(std::integral_constant<int, 3>{});
    }
  }
#ifdef CR_GEMM_STAMPS
  cr_tile_store<BP, 1, KSPLIT>(t1, t2, t3, sg, base + out + lo, hasc, cpf, valid, g_gemm_on);
#else
  cr_tile_store<BP, 1, KSPLIT>(t1, t2, t3, sg, base + out + lo, hasc, cpf, valid);
#endif
#ifdef CR_GEMM_STAMPS
  if (g_gemm_on) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GEMM_STAMP(5, g_gemm_on);
  GEMM_STAMP(6, g_gemm_on);
#endif
}

// ---------------------------------------------------------------------------
// An inversion stage with side work: the first ninv x nbatch workgroups
// invert (k_cr_inv), the rest run product tiles that are off the critical
// path (the previous level's W1/W2 and U'/L'): an inversion
// stage occupies only ninv x nbatch CUs (224 of 256 at the finest level of
// L = 32, 14 at the coarsest) for its whole ~16 us, and the side tiles fill
// the idle CUs instead of lengthening the product launches of the critical
// path.  The inversions have the lowest workgroup ids, so they are
// dispatched first and keep a CU each; the side workgroups run one per CU
// (the inversion's register budget), so each wave computes a 32 x 32 output
// tile over the full K (12 independent MFMA chains: a wave alone on its SIMD
// must hide its own MFMA and memory latency; one 16 x 16 tile per wave ran at
// a third of that rate).
// ---------------------------------------------------------------------------
// arguments in first-use order: the inversion workgroups (the first
// ninv x nbatch) need only the leading ones; nside: side-work workgroups
template <int NT>
__global__ __launch_bounds__(64 * NT) void k_cr_inv_side(double2* __restrict__ pool, int64_t item,
                                                         const int* __restrict__ blk,
                                                         const int* __restrict__ dst, int ninv, int nbatch,
                                                         const int* __restrict__ slot,
                                                         double* __restrict__ ldpart, int nslots,
                                                         int nside, const CrTask* __restrict__ stasks, int nst,
                                                         int maxt, int total, SiteGuard sg, int N) {
  static_assert(NT == 4, "side work runs 4-wave workgroups");
  __shared__ double2 pan[2][NT][16 * 17];
  __shared__ double ldw[NT];
  const int b = blockIdx.x, nall = ninv * nbatch;
  // inversions first: their branch needs only the leading (preloaded) arguments
  if (b < nall) {
    // the batch items grouped per XCD (xcd_remap over the inversion range)
    const int bl = CR_XCD_ITEMS ? xcd_remap(b, nall) : b;
    cr_inv_wg<NT>(pool, item, bl / ninv, bl - (bl / ninv) * ninv, blk, dst, slot, ldpart, nslots, pan, ldw);
    return;
  }
  CR_STAMP_INIT(blk);
  CR_RSTAMP(0);
  // the workgroups after the side work check the site guard (level-0 launches)
  if (b >= nall + nside) {
    site_guard_wg(sg, N, b - nall - nside);
    CR_RSTAMP(30);
    CR_STAMP_AT(31, 3ull);
    return;
  }
  cr_gemm_wg<16 * NT, 2, 1, 0, true>(pool, item, stasks, nst, maxt, total, 1.0, xcd_remap(b - nall, nside));
#ifdef CR_STAMPS
  if (stamp_on) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  CR_RSTAMP(30);
  CR_STAMP_AT(31, 2ull);
}

// ---------------------------------------------------------------------------
// Force from the level-0 G blocks: P_ij = Σ_q c_q (G12[i,j] + G12[j,i]) with
// G12 read straight from the B parts of the pool (offsets goff per pairing
// slot), F = -β/2J (Δ - J P) (src/Observables.jl:14-62), then the leapfrog
// kick and the next step's drift (kick_drift).
// ---------------------------------------------------------------------------
// 32 lanes per bond, one pole per lane (the G entries of the poles live in
// different batch items: independent loads), shuffle reduction.  With a
// drift (inside a trajectory) the drifted Δ/2 is scattered straight into the
// level-0 pairing entries of every pole, so the next factorisation needs no
// k_cr_fill launch.  bond4[4 b ..]: the pool offsets of G12[i, j], G12[j, i]
// and of the two pairing entries bond b writes (-1: written by another bond;
// small lattices map several bonds onto one entry), resolved at context
// creation so the G loads wait for one index load, not two.
// arguments in first-use order (kernel-argument preload)
constexpr int kPfLanes = 32;   // lanes per bond (poles strided over them)
__global__ __launch_bounds__(256) void k_cr_pair_force(
    double2* __restrict__ pool, int64_t item, const int64_t* __restrict__ bond4, int N, int P,
    const double* __restrict__ cpole, double2* __restrict__ Delta, double2* __restrict__ Pair,
    double2* __restrict__ F, double2* __restrict__ Pi, double kick, double drift, double cap2,
    int* __restrict__ flag, double beta, double J) {
  constexpr int LB = kPfLanes;
  const int b = blockIdx.x * (256 / LB) + (threadIdx.x / LB), sub = threadIdx.x % LB;
  const int c = blockIdx.y;
  if (b >= 2 * N) return;   // uniform per lane group
  const int64_t o1 = bond4[4 * b], o2 = bond4[4 * b + 1], p1 = bond4[4 * b + 2], p2 = bond4[4 * b + 3];
  // Δ and π of the bond, loaded beside the G entries (not after the reduction)
  const int64_t o = (int64_t)c * 2 * N + b;
  double2 d0 = make_double2(0.0, 0.0), p0 = make_double2(0.0, 0.0);
  if (sub == 0) {
    d0 = Delta[o];
    p0 = Pi[o];
  }
  double2 Pv = make_double2(0.0, 0.0);
  for (int q = sub; q < P; q += LB) {
    const double2* G = pool + (int64_t)(c * P + q) * item;
    const double2 g1 = G[o1], g2 = G[o2];
    const double cq = cpole[q];
    Pv.x += cq * (g1.x + g2.x);
    Pv.y += cq * (g1.y + g2.y);
  }
#pragma unroll
  for (int off = LB / 2; off > 0; off >>= 1) {
    Pv.x += __shfl_xor(Pv.x, off, LB);
    Pv.y += __shfl_xor(Pv.y, off, LB);
  }
  double2 dn = make_double2(0.0, 0.0);
  if (sub == 0) {
    Pair[o] = Pv;
    const double2 d = d0;
    const double f = -beta / (2.0 * J);
    const double2 Fv = make_double2(f * (d.x - J * Pv.x), f * (d.y - J * Pv.y));
    F[o] = Fv;
    dn = kick_drift_pre(Fv, o, p0, d0, Delta, Pi, kick, drift, cap2, flag);
  }
  if (drift != 0.0) {
    dn.x = 0.5 * __shfl(dn.x, 0, LB);
    dn.y = 0.5 * __shfl(dn.y, 0, LB);
    // an entry is written only by the bond k_cr_fill takes its value from
    // (Dsrc: the one the reference's overwrite order leaves, src/Hamiltonian.jl:68-83)
    for (int q = sub; q < P; q += LB) {
      double2* G = pool + (int64_t)(c * P + q) * item;
      if (p1 >= 0) G[p1] = dn;
      if (p2 >= 0) G[p2] = dn;
    }
  }
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
                                                           double* __restrict__ part,
                                                           double* __restrict__ Ef,
                                                           double* __restrict__ Trhh,
                                                           unsigned* __restrict__ done) {
  // one block per (pole, chain): its weighted Σ ln|pivots| and Re Tr G22
  const int q = blockIdx.x, c = blockIdx.y, bi = c * P + q;
  __shared__ double red[2][4];
  __shared__ bool last;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double ld = 0.0, t = 0.0;
  for (int k = threadIdx.x; k < nld; k += blockDim.x) ld += ldpart[(int64_t)bi * nld + k];
  for (int i = threadIdx.x; i < N; i += blockDim.x) t -= pool[(int64_t)bi * item + doff[i]].x;
  ld = wave_sum(ld);
  t = wave_sum(t);
  if (l == 0) {
    red[0][w] = ld;
    red[1][w] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * bi] = cpole[q] * (red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    part[2 * bi + 1] = cpole[q] * (red[1][0] + red[1][1] + red[1][2] + red[1][3]);
    // the last block of this chain sums the pole partials in pole order
    // (deterministic); release / acquire through the counter at agent scope
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const unsigned n = __hip_atomic_fetch_add(&done[c], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (n == (unsigned)P - 1);
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  double ef = 0.0, tr = 0.0;
  for (int k = 0; k < P; ++k) {
    ef += __hip_atomic_load(&part[2 * (c * P + k)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tr += __hip_atomic_load(&part[2 * (c * P + k) + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  Ef[c] = -2.0 * N * Cx - beta * ef;
  Trhh[c] = 0.5 * N - tr;
  done[c] = 0;   // ready for the next launch (stream order)
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
bool cr_supported_bp(int BP) { return BP == 32 || BP == 64 || BP == 96 || BP == 128; }
bool cr_supported_side(int BP) { return BP == 64; }
bool cr_supported_inv0(int BP) { return BP == 64 || BP == 32 || BP == 96; }

void launch_cr_inv0(const CrDims& c, double2* pool, const int* blk, const int* rblk, const int* dst,
                    const int* slot, int n, double* ldpart, const double* ldA, hipStream_t s,
                    const double2* Delta, const int* site4, double cap4, int* flag) {
  if (n <= 0) return;
  const bool guard = Delta != nullptr && site4 != nullptr && flag != nullptr;
  hipLaunchKernelGGL(c.BP == 32 ? k_cr_inv0_32 : c.BP == 96 ? k_cr_inv0_96 : k_cr_inv0,
                     dim3(n + (guard ? 1 : 0), c.nbatch), dim3(c.BP == 32 ? 64 : c.BP == 96 ? 576 : 256), 0, s, pool,
                     c.item, blk, rblk, dst, guard ? n : -1, slot, ldpart, ldA, c.Ly, guard ? Delta : nullptr, site4,
                     c.N, c.P, cap4, flag);
}

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

void launch_cr_inv(const CrDims& c, double2* pool, const int* blk, const int* dst, const int* slot,
                   int n, double* ldpart, hipStream_t s, const SiteGuard& sg) {
  if (n <= 0) return;
  const bool guard = sg.Delta != nullptr;
  const dim3 g(n + (guard ? 1 : 0), c.nbatch);
  const int gcol = guard ? n : -1;
  switch (c.BP) {
    case 32:
      if (c.inv32)
        hipLaunchKernelGGL(k_cr_inv32, g, dim3(64), 0, s, pool, c.item, blk, dst, gcol, slot, ldpart, c.Ly, sg, c.N,
                           c.P);
      else
        hipLaunchKernelGGL(k_cr_inv<2>, g, dim3(128), 0, s, pool, c.item, blk, dst, gcol, slot, ldpart, c.Ly, sg,
                           c.N, c.P);
      break;
    case 64:
      hipLaunchKernelGGL(k_cr_inv<4>, g, dim3(256), 0, s, pool, c.item, blk, dst, gcol, slot, ldpart, c.Ly, sg, c.N,
                         c.P);
      break;
    case 96:
      hipLaunchKernelGGL(k_cr_inv<6>, g, dim3(384), 0, s, pool, c.item, blk, dst, gcol, slot, ldpart, c.Ly, sg, c.N,
                         c.P);
      break;
    default:
      hipLaunchKernelGGL(k_cr_inv<8>, g, dim3(512), 0, s, pool, c.item, blk, dst, gcol, slot, ldpart, c.Ly, sg, c.N,
                         c.P);
      break;
  }
}

void launch_cr_inv_side(const CrDims& c, double2* pool, const int* blk, const int* dst, const int* slot,
                        int n, double* ldpart, const CrTask* stasks, int nst, int maxt32, hipStream_t s,
                        const SiteGuard& sg) {
  if (nst <= 0) {
    launch_cr_inv(c, pool, blk, dst, slot, n, ldpart, s, sg);
    return;
  }
  const int total = c.nbatch * nst * maxt32;
  const int side_wg = (total + 3) / 4;
  const int nc = c.nbatch / c.P;
  const dim3 g(n * c.nbatch + side_wg + (sg.Delta != nullptr ? nc : 0));
  hipLaunchKernelGGL(k_cr_inv_side<4>, g, dim3(256), 0, s, pool, c.item, blk, dst, n, c.nbatch, slot, ldpart,
                     c.Ly, side_wg, stasks, nst, maxt32, total, sg, c.N);
}

// Stage configuration (tile TS, K split).  16 x 16 tiles; the K split by the
// stage's size (ntiles16 16 x 16 output tiles per batch item x nbatch): a
// 4-way split (short serial MFMA chains on many waves) for the stages of a
// single L = 32 chain, whose stages are short and latency bound
// (profiles/r01_cr_gemm_config_sweep.txt: fastest on every stage there), no
// split once a stage has enough tiles to fill the chip by itself (batched
// chains, L = 48: no LDS reduction, one tile per wave;
// profiles/r03_exp_gemm_ksplit_by_size.txt: from 2048 tiles, C3 -0.9 %,
// C5 -5 %, 4 chains at L = 32 -3 %; C2's stages stay below it).
// DWHMC_CR_GEMM=TS:KSPLIT forces one
// configuration for every stage (A/B runs; tests/test_gpu_parity.py runs
// every compiled variant).
CrGemmCfg cr_gemm_config(const CrDims& c, int ntasks, int maxt32, int maxt16, int ntmax, int ntiles16) {
  (void)ntasks;
  (void)maxt32;
  (void)maxt16;
  (void)ntmax;
  // read at every context creation (tests switch it between contexts)
  const CrGemmCfg forced = [] {
    CrGemmCfg f{0, 1};
    if (const char* e = std::getenv("DWHMC_CR_GEMM")) {
      f.ts = std::atoi(e);
      if (const char* p = std::strchr(e, ':')) f.ksplit = std::atoi(p + 1);
    }
    if (f.ksplit != 1 && f.ksplit != 2 && f.ksplit != 4) f.ksplit = 1;
    if (f.ts == 32 && f.ksplit == 4) f.ksplit = 2;
    return f;
  }();
  const bool ts32_ok = (c.BP / 2) % 32 == 0;   // 32-wide tiles must not straddle A | B
  if (forced.ts == 16 || (forced.ts == 32 && ts32_ok)) return forced;
  const int64_t T = (int64_t)ntiles16 * c.nbatch;
  return CrGemmCfg{16, T >= 2048 ? 1 : 4};
}

// host twin of xcd_remap (dwhmc_device.h)
static int xcd_remap_host(int orig, int total) {
  const int q = total / 8, r = total % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

int cr_gemm_slot_wgs(const CrDims& c, int ntl16, const CrGemmCfg& cfg) {
  const int tpw = 4 / cfg.ksplit;
  return (c.nbatch * ntl16 + tpw - 1) / tpw;
}

// Slot b * TPW + j of the launch = tile (xcd_remap(b, nwg) * TPW + j) of the
// stage's nbatch x ntl16 tiles (batch item major): the order the round-5
// kernel derived on the device, so the work distribution over XCDs is kept.
void cr_gemm_slots(const CrDims& c, const CrTile* tl16, int ntl16, const CrGemmCfg& cfg, CrSlot* out) {
  const int tpw = 4 / cfg.ksplit, nwg = cr_gemm_slot_wgs(c, ntl16, cfg), HP = c.BP / 2;
  const int64_t total = (int64_t)c.nbatch * ntl16, BB = (int64_t)HP * c.BP;
  for (int b = 0; b < nwg; ++b)
    for (int j = 0; j < tpw; ++j) {
      CrSlot& sl = out[(size_t)b * tpw + j];
      sl = CrSlot{};
      const int64_t gt = (int64_t)xcd_remap_host(b, nwg) * tpw + j;
      if (gt >= total) {   // padding of the last workgroup
        sl.out = kCrNone;
        sl.cin = kCrNone;
        continue;
      }
      const int bi = (int)(gt / ntl16);
      const CrTile& t = tl16[gt - (int64_t)bi * ntl16];
      const int r0 = 16 * t.tr, c0 = 16 * t.tc;
      sl.base = (uint64_t)bi * (uint64_t)c.item;
      sl.out = (uint32_t)(t.out * BB + (int64_t)r0 * c.BP + c0);
      sl.cin = t.cin >= 0 ? (uint32_t)(t.cin * BB + (int64_t)r0 * c.BP + c0) : kCrNone;
      sl.nt = t.nt;
      for (int h = 0; h < t.nt; ++h) {
        sl.a[h] = (uint32_t)(t.a[h] * BB + (int64_t)r0 * c.BP);
        sl.b[h] = (uint32_t)(t.b[h] * BB + c0);
        const bool q = (t.bq >> h) & 1;
        if ((c0 < HP) == q) sl.smask |= 1u << h;   // synthesised rows: sgn < 0
      }
      sl.rot = (c0 < HP ? c0 + HP : c0 - HP) - c0;
    }
}

void launch_cr_gemm(const CrDims& c, double2* pool, const CrTask* tasks, int ntasks, int maxt32,
                    int maxt16, const CrSlot* slots, int nslot_wgs, const CrGemmCfg& cfg, double sg,
                    hipStream_t s) {
  (void)maxt16;
  if (ntasks <= 0) return;
  const dim3 b(256);
  if (cfg.ts == 16) {
    const dim3 g(nslot_wgs);
#define CR_GEMM16(BPV, KSV) hipLaunchKernelGGL((k_cr_gemm16<BPV, KSV>), g, b, 0, s, pool, slots, sg)
#define CR_GEMM16_BP(BPV)                        \
  if (cfg.ksplit == 4) CR_GEMM16(BPV, 4);        \
  else if (cfg.ksplit == 2) CR_GEMM16(BPV, 2);   \
  else CR_GEMM16(BPV, 1);
    switch (c.BP) {
      case 32: CR_GEMM16_BP(32) break;
      case 64: CR_GEMM16_BP(64) break;
      case 96: CR_GEMM16_BP(96) break;
      default: CR_GEMM16_BP(128) break;
    }
#undef CR_GEMM16_BP
#undef CR_GEMM16
    return;
  }
  const int total = c.nbatch * ntasks * maxt32;
  const int tpw = 4 / cfg.ksplit;
  const dim3 g((total + tpw - 1) / tpw);
#define CR_GEMM(BPV, KSV) \
  hipLaunchKernelGGL((k_cr_gemm<BPV, 2, KSV>), g, b, 0, s, pool, c.item, total, sg, (int)g.x, ntasks, maxt32, tasks)
#define CR_GEMM_BP(BPV)                      \
  if (cfg.ksplit == 2) CR_GEMM(BPV, 2);      \
  else CR_GEMM(BPV, 1);
  switch (c.BP) {
    case 32: CR_GEMM_BP(32) break;
    case 64: CR_GEMM_BP(64) break;
    case 96: CR_GEMM_BP(96) break;
    default: CR_GEMM_BP(128) break;
  }
#undef CR_GEMM_BP
#undef CR_GEMM
}

void launch_cr_pair_force(const CrDims& c, double2* pool, const int64_t* bond4, const double* cpole,
                          double2* Delta, double2* Pair, double2* F, double2* Pi,
                          const KickDrift& kd, double beta, double J, hipStream_t s) {
  const int nc = c.nbatch / c.P;
  constexpr int BPW = 256 / kPfLanes;   // bonds per workgroup
  hipLaunchKernelGGL(k_cr_pair_force, dim3((2 * c.N + BPW - 1) / BPW, nc), dim3(256), 0, s, pool, c.item, bond4, c.N,
                     c.P, cpole, Delta, Pair, F, Pi, kd.kick, kd.drift, kd.cap * kd.cap, kd.flag, beta, J);
}

void launch_cr_fermion_energy(const CrDims& c, const double2* pool, const int64_t* doff,
                              const double* ldpart, const double* cpole, double Cx, double beta,
                              double* part, unsigned* done, double* Ef, double* Trhh, hipStream_t s) {
  const int nc = c.nbatch / c.P;
  hipLaunchKernelGGL(k_cr_fermion_energy, dim3(c.P, nc), dim3(256), 0, s, pool, c.item, doff, ldpart,
                     cpole, c.N, c.Ly, c.P, Cx, beta, part, Ef, Trhh, done);
}

}  // namespace dwh

#ifdef CR_STAMPS
namespace dwh {
int cr_stamps_arm(int key) {
  static unsigned long long zero[kCrStampWG][32];
  if (key >= 0 && hipMemcpyToSymbol(HIP_SYMBOL(g_cr_stamps), zero, sizeof(zero)) != hipSuccess) return -2;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cr_stamp_key), &key, sizeof(int)) == hipSuccess ? 0 : -2;
}
int cr_stamps_read(unsigned long long* out, int nwg) {
  if (nwg > kCrStampWG) nwg = kCrStampWG;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cr_stamps), (size_t)nwg * 32 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
}  // namespace dwh
#endif

#ifdef CR_GEMM_STAMPS
extern "C" int dwh_debug_gemm_stamps_select(int total) {
  return hipMemcpyToSymbol(HIP_SYMBOL(dwh::g_gemm_sel), &total, sizeof(int)) == hipSuccess ? 0 : -2;
}
extern "C" int dwh_debug_gemm_stamps_read(unsigned long long* out, int nblocks) {
  if (nblocks > 65536) nblocks = 65536;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dwh::g_gemm_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif
