// gfx950 (MI355X, CDNA4) kernels of the DwaveHMC.jl fermionic action/force path.
//
// Per leapfrog step (src/HMC.jl:98-114) and per imaginary-axis pole z = i y_q:
//   S(z)    = -(h + z) - D† R(z) D          Schur complement of H_BdG - z over
//                                            its static particle block, R = (h - z)^-1
//   S^-1    : in-place blocked Gauss-Jordan, no pivoting (i·S has Hermitian part
//             y·I > 0, so every pivot is bounded away from 0), trailing updates on
//             v_mfma_f64_16x16x4_f64 tiles staged through LDS
//   G12     = -R D S^-1   only at the 4N nearest-neighbour entries
//   P_ij    = Σ_q c_q (G12[i,j] + G12[j,i])   (= -ρ_{i,j+N} - ρ_{j,i+N})
//   F_ij    = -β/2J (Δ_ij - J P_ij)          (src/Observables.jl:14-62)
//   E_f     = -2N C - β Σ_q c_q ln|det(H - i y_q)|  from the GJ pivots
// See DESIGN.md §2-§3 for the derivation and the roofline of each kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {

// ---------------------------------------------------------------------------
// dense M = h_c - i y_q, padded with identity (input of the R = (h - i y)^-1 GJ)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fill_hz(double2* __restrict__ M, int64_t mat, int N,
                                                 int Np, int P, const int* __restrict__ hcol,
                                                 const double* __restrict__ hval,
                                                 const double* __restrict__ ypole) {
  const int a = blockIdx.x, bi = blockIdx.y;
  const int c = bi / P, q = bi % P;
  double2* row = M + (int64_t)bi * mat + (int64_t)a * Np;
  __shared__ int hc[kHSlots];
  __shared__ double hv[kHSlots];
  if (threadIdx.x < kHSlots) {
    hc[threadIdx.x] = (a < N) ? hcol[a * kHSlots + threadIdx.x] : -1;
    hv[threadIdx.x] = (a < N) ? hval[((int64_t)c * N + a) * kHSlots + threadIdx.x] : 0.0;
  }
  __syncthreads();
  const double y = ypole[q];
  for (int b = threadIdx.x; b < Np; b += blockDim.x) {
    double2 v = make_double2(0.0, 0.0);
    if (a < N) {
#pragma unroll
      for (int s = 0; s < kHSlots; ++s)
        if (hc[s] == b) v.x = hv[s];
      if (b == a) v.y = -y;
    } else if (b == a) {
      v.x = 1.0;
    }
    row[b] = v;
  }
}

// ---------------------------------------------------------------------------
// Pivot step k of the blocked Gauss-Jordan (one launch per step, grid nb x nbatch):
// every block inverts the 64x64 pivot block S_kk in LDS (4 sub-steps of 16:
// a wave-local 16x16 inversion through lane shuffles, then MFMA rank-16
// updates), then block j != k forms its row-panel tile X_kj = S_kk^-1 S_kj in
// place (and into the row-panel buffer); block k stores
// S_kk^-1 to Pbuf and the pivots' ln|u_pp|.  The redundant inversions cost
// latency only (all blocks run concurrently) and remove the serial diag launch.
// ---------------------------------------------------------------------------

constexpr int kLdA = kGJ + 1;   // padded LDS row stride of the pivot block

// Diagnostic build only (-DDWH_STAMPS, tools/micro/pivot_stamps.hip): per-block
// s_memtime stamps of the pivot kernel's phases; never compiled into the library.
#ifdef DWH_STAMPS
__device__ unsigned long long g_stamps[4096][8];
#define DWH_STAMP(i)                                                          \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    if (threadIdx.x == 0)                                                     \
      g_stamps[blockIdx.y * gridDim.x + blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
#else
#define DWH_STAMP(i) \
  do {               \
  } while (0)
#endif

__global__ __launch_bounds__(256) void k_gj_pivot(double2* __restrict__ M, int64_t mat, int Np,
                                                  int nb, int k, double2* __restrict__ Pout,
                                                  double2* __restrict__ XRout,
                                                  double2* __restrict__ colcopy,
                                                  double2* __restrict__ nextcol,
                                                  double* __restrict__ ldpart) {
  __shared__ double2 A[kGJ * kLdA];        // the pivot block, inverted in place
  __shared__ double2 Xs[16 * kGJ];         // row sub-panel of the current sub-step
  __shared__ double2 Cs[kGJ * 17];         // column sub-panel copy (row stride 17: no bank conflicts)
  __shared__ double2 Dw[4][16 * 17];       // per-wave copy of the 16x16 sub-block inverse
  __shared__ double2 Bs[16][kGJ];          // staging of S_kj for the panel product
  __shared__ double2 xbw[4][32];           // per-wave row/column exchange of wave_inv16
  __shared__ double pm[kGJ];
  const int j = blockIdx.x, bi = blockIdx.y;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lr = l & 15, lk = l >> 4;
  double2* Mb = M + (int64_t)bi * mat;
  const double2* Skk = Mb + (int64_t)(k * kGJ) * Np + k * kGJ;
  DWH_STAMP(0);
  {
    double2 v[16];   // all 16 loads in flight before the LDS stores
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u;
      v[u] = Skk[(int64_t)(e >> 6) * Np + (e & 63)];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u;
      A[(e >> 6) * kLdA + (e & 63)] = v[u];
    }
  }
  __syncthreads();
  DWH_STAMP(1);

#pragma unroll 1
  for (int kb = 0; kb < 4; ++kb) {
    const int o = kb * 16;
    // (a) every wave inverts the 16x16 diagonal sub-block (redundantly)
    double2 dv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dv[jj] = A[(o + (l >> 2)) * kLdA + o + (l & 3) * 4 + jj];
    wave_inv16(dv, xbw[w], w == 0 ? pm : nullptr, o);
    if (kb == 0) DWH_STAMP(2);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) Dw[w][(l >> 2) * 17 + (l & 3) * 4 + jj] = dv[jj];
    // column sub-panel copy (old values)
    for (int e = tid; e < kGJ * 16; e += 256) Cs[(e >> 4) * 17 + (e & 15)] = A[(e >> 4) * kLdA + o + (e & 15)];
    // (b) X[:, block w] = Dinv * A[kb rows, block w]  (block kb: X = Dinv)
    {
      d4 xr = {0, 0, 0, 0}, xi = {0, 0, 0, 0};
      if (w == kb) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double2 v = Dw[w][(lk + 4 * rr) * 17 + lr];
          xr[rr] = v.x;
          xi[rr] = v.y;
        }
      } else {
        mma16_lds<false>(xr, xi, Dw[w], 17, A + o * kLdA + w * 16, kLdA);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Xs[(lk + 4 * rr) * kGJ + w * 16 + lr] = make_double2(xr[rr], xi[rr]);
    }
    __syncthreads();
    if (kb == 0) DWH_STAMP(3);
    // (c) rows kb <- X; other rows: A[ib, jb] = [jb != kb] A[ib, jb] - C[ib] X[jb]
    for (int e = tid; e < 16 * kGJ; e += 256) A[(o + (e >> 6)) * kLdA + (e & 63)] = Xs[e];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
      const int t = w + 4 * tt;
      const int ibx = t >> 2;
      const int ib = ibx < kb ? ibx : ibx + 1;
      const int jb = t & 3;
      d4 cr, ci;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const double2 v = (jb == kb) ? make_double2(0.0, 0.0)
                                     : A[(ib * 16 + lk + 4 * rr) * kLdA + jb * 16 + lr];
        cr[rr] = v.x;
        ci[rr] = v.y;
      }
      mma16_lds<true>(cr, ci, Cs + ib * 16 * 17, 17, Xs + jb * 16, kGJ);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) A[(ib * 16 + lk + 4 * rr) * kLdA + jb * 16 + lr] = make_double2(cr[rr], ci[rr]);
    }
    __syncthreads();
    if (kb == 0) DWH_STAMP(4);
  }
  DWH_STAMP(5);

  if (j == k) {
    double2* Pb = Pout + (int64_t)bi * kGJ * kGJ;
    for (int e = tid; e < kGJ * kGJ; e += 256) Pb[e] = A[(e >> 6) * kLdA + (e & 63)];
    if (nb == 1) {
      double2* Sk = Mb + (int64_t)(k * kGJ) * Np + k * kGJ;
      for (int e = tid; e < kGJ * kGJ; e += 256) Sk[(int64_t)(e >> 6) * Np + (e & 63)] = A[(e >> 6) * kLdA + (e & 63)];
    }
    if (tid < 64) {
      const double v = wave_sum(0.5 * log(pm[tid]));
      if (tid == 0) ldpart[(int64_t)bi * nb + k] = v;
    }
    return;
  }
  // column-panel copy S_jk -> colcopy[j] (first step only; later steps get
  // their column panel from the previous update)
  if (colcopy != nullptr) {
    const double2* Sjk = Mb + (int64_t)(j * kGJ) * Np + k * kGJ;
    double2* dst = colcopy + (int64_t)bi * Np * kGJ + (int64_t)j * kGJ * kGJ;
    double2 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u;
      v[u] = Sjk[(int64_t)(e >> 6) * Np + (e & 63)];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) dst[tid + 256 * u] = v[u];
  }
  DWH_STAMP(6);
  // row-panel tile X_kj = A * S_kj (in place): 4 waves x (32x32) outputs
  double2* Skj = Mb + (int64_t)(k * kGJ) * Np + j * kGJ;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  d4 acr[2][2], aci[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      acr[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
      aci[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
    }
#pragma unroll 1
  for (int kc = 0; kc < kGJ; kc += 16) {
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) Bs[tid >> 4][(tid & 15) * 4 + s4] = Skj[(int64_t)(kc + (tid >> 4)) * Np + (tid & 15) * 4 + s4];
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        mma16_lds<false>(acr[mi][ni], aci[mi][ni], A + (wr + mi * 16) * kLdA + kc, kLdA,
                         &Bs[0][wc + ni * 16], kGJ);
    __syncthreads();
  }
  // X_{k,k+1} is also row block k of the next column panel (nextcol)
  double2* CpN = (j == k + 1 && nextcol != nullptr)
                     ? nextcol + (int64_t)bi * Np * kGJ + (int64_t)k * kGJ * kGJ
                     : nullptr;
  double2* XRt = XRout ? XRout + (int64_t)bi * kGJ * Np + j * kGJ : nullptr;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr + mi * 16 + lk + 4 * r, col = wc + ni * 16 + lr;
        const double2 v = make_double2(acr[mi][ni][r], aci[mi][ni][r]);
        Skj[(int64_t)row * Np + col] = v;
        if (XRt) XRt[(int64_t)row * Np + col] = v;
        if (CpN) CpN[row * kGJ + col] = v;
      }
  DWH_STAMP(7);
}

// One wave's 32x32 share of  acc -= sum_h A_h B_h  (NT terms, K = 64 each).
// Per-lane fragment pointers; fully unrolled with a two-deep register
// prefetch that runs across the term boundary.
struct GemmTerm {
  const double2* a;   // &A[wr + lr][lk]
  const double2* b;   // &B[lk][wc + lr]
  int lda, ldb;
};

template <int NT>
__device__ __forceinline__ void tile_nt_gemm(d4 (&acr)[2][2], d4 (&aci)[2][2], const GemmTerm& t0,
                                             const GemmTerm& t1) {
  constexpr int NS = 16 * NT;
  double2 fa[2][2], fb[2][2];
  auto load = [&](int s, double2 (&a)[2], double2 (&b)[2]) {
    const GemmTerm& t = (s >= 16) ? t1 : t0;
    const int kk = (s & 15) * 4;
    a[0] = t.a[kk];
    a[1] = t.a[(int64_t)16 * t.lda + kk];
    b[0] = t.b[(int64_t)kk * t.ldb];
    b[1] = t.b[(int64_t)kk * t.ldb + 16];
  };
  load(0, fa[0], fb[0]);
  load(1, fa[1], fb[1]);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = s & 1;
    const double2 av[2] = {fa[c][0], fa[c][1]};
    const double2 bv[2] = {fb[c][0], fb[c][1]};
    if (s + 2 < NS) load(s + 2, fa[c], fb[c]);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        acr[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[mi].x, bv[ni].x, acr[mi][ni], 0, 0, 0);
        aci[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[mi].x, bv[ni].y, aci[mi][ni], 0, 0, 0);
      }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        acr[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mi].y, bv[ni].y, acr[mi][ni], 0, 0, 0);
        aci[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[mi].y, bv[ni].x, aci[mi][ni], 0, 0, 0);
      }
  }
}

// Trailing updates of the blocked Gauss-Jordan, one 64x64 tile per block:
//   out = init - sum_h A_h * B_h   (h = 1 or 2 terms of K = 64 each)
// Each wave owns a 32x32 sub-tile; MFMA fragments come straight from L2 into
// registers with a two-deep prefetch (no LDS, no barriers).  1D grid with an
// XCD-aware remap so one matrix's panels stay in one XCD's L2.
//
// Panels (per batch item): CpA = column panel of block column k (rows I != k),
// CpB = column k+1 after the edge update, XR1/XR2 = row panels of pivots k /
// k+1 (64 x Np, ld Np), Pb1/Pb2 = the pivot inverses.  Modes:
//  0 SINGLE  (step k):       I != k:  out = [J!=k]S_IJ - CpA_I*(J==k ? Pb1 : XR1_J)
//  1 EDGE    (pair k,k+1):   row k+1: S_{k+1,J} = [J!=k]S_{k+1,J} - CpA_{k+1}*(J==k ? Pb1 : XR1_J)
//                            col k+1: CpB_I = S_{I,k+1} - CpA_I*XR1_{k+1}   (I != k, k+1)
//  2 COMBINED (pair k,k+1):  rank-128 remainder of both steps, I != k+1:
//     I == k : out = init_k - XR1_{k+1} * (J==k+1 ? Pb2 : XR2_J),
//              init_k = J==k ? Pb1 : J==k+1 ? 0 : XR1_J
//     I != k : out = [J!=k,k+1]S_IJ - CpA_I*(J==k ? Pb1 : J==k+1 ? 0 : XR1_J)
//                                   - CpB_I*(J==k+1 ? Pb2 : XR2_J)
// In modes 0/2 tiles of block column `ncol` (k+1 resp. k+2) are also written
// to CpN, the next column panel; mode 0 stores S_kk = Pb1 and mode 2 stores
// S_{k+1,k+1} = Pb2 from one designated tile.
struct GJPanels {
  const double2 *CpA, *CpB, *XR1, *XR2, *Pb1, *Pb2;
  double2 *CpBw, *CpN;
};

#ifndef DWH_UPD_OCC
#define DWH_UPD_OCC 1
#endif
template <int mode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DWH_UPD_OCC))) void k_gj_update(double2* __restrict__ M, int64_t mat, int Np,
                                                   int nb, int k, int total, GJPanels pn) {
  const int tiles = mode == 1 ? 2 * nb - 2 : (nb - 1) * nb;
  const int item = xcd_remap(blockIdx.x, total);
  const int bi = item / tiles, t = item - bi * tiles;
  int I, J;
  if (mode == 1) {
    if (t < nb) {
      I = k + 1;
      J = t;
    } else {
      const int u = t - nb;
      I = u < k ? u : u + 2;
      J = k + 1;
    }
  } else {
    const int skip = mode == 0 ? k : k + 1;
    const int Ii = t / nb;
    J = t - Ii * nb;
    I = Ii < skip ? Ii : Ii + 1;
  }
  double2* Mb = M + (int64_t)bi * mat;
  const int64_t pnl = (int64_t)bi * Np * kGJ;     // column panel / row panel batch offset
  const int64_t pvb = (int64_t)bi * kGJ * kGJ;
  auto colp = [&](const double2* base, int row) { return base + pnl + (int64_t)row * kGJ * kGJ; };
  auto rowp = [&](const double2* base, int col) { return base + pnl + col * kGJ; };
  // terms: A (64 x 64, lda), B (64 x 64, ldb); init source
  const double2 *A0 = nullptr, *B0 = nullptr, *A1 = nullptr, *B1 = nullptr, *Cin = nullptr;
  int lda0 = kGJ, ldb0 = Np, lda1 = kGJ, ldb1 = Np, ldc_in = Np;
  double2* out = Mb + (int64_t)(I * kGJ) * Np + J * kGJ;
  int ldo = Np;
  double2* out2 = nullptr;
  if (mode == 0) {
    A0 = colp(pn.CpA, I);
    if (J == k) { B0 = pn.Pb1 + pvb; ldb0 = kGJ; } else { B0 = rowp(pn.XR1, J); }
    if (J != k) Cin = out;
    if (J == k + 1 && pn.CpN) out2 = const_cast<double2*>(colp(pn.CpN, I));
  } else if (mode == 1) {
    A0 = colp(pn.CpA, I);
    if (J == k) { B0 = pn.Pb1 + pvb; ldb0 = kGJ; } else { B0 = rowp(pn.XR1, J); }
    if (I == k + 1) {
      if (J != k) Cin = out;
    } else {            // column k+1: result goes to CpB only
      Cin = out;
      out = const_cast<double2*>(colp(pn.CpBw, I));
      ldo = kGJ;
    }
  } else {
    if (I == k) {
      A1 = rowp(pn.XR1, k + 1); lda1 = Np;
      if (J == k + 1) { B1 = pn.Pb2 + pvb; ldb1 = kGJ; } else { B1 = rowp(pn.XR2, J); }
      if (J == k) { Cin = pn.Pb1 + pvb; ldc_in = kGJ; }
      else if (J != k + 1) { Cin = rowp(pn.XR1, J); }
    } else {
      if (J != k + 1) {
        A0 = colp(pn.CpA, I);
        if (J == k) { B0 = pn.Pb1 + pvb; ldb0 = kGJ; } else { B0 = rowp(pn.XR1, J); }
      }
      A1 = colp(pn.CpB, I);
      if (J == k + 1) { B1 = pn.Pb2 + pvb; ldb1 = kGJ; } else { B1 = rowp(pn.XR2, J); }
      if (J != k && J != k + 1) Cin = out;
    }
    if (J == k + 2 && pn.CpN) out2 = const_cast<double2*>(colp(pn.CpN, I));
  }
  if (A0 == nullptr) {   // single term in slot 1 -> move to slot 0
    A0 = A1; B0 = B1; lda0 = lda1; ldb0 = ldb1;
    A1 = nullptr;
  }
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  const int lr = l & 15, lk = l >> 4;
  d4 acr[2][2], aci[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      if (Cin != nullptr) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double2 v = Cin[(int64_t)(wr + mi * 16 + lk + 4 * rr) * ldc_in + wc + ni * 16 + lr];
          acr[mi][ni][rr] = v.x;
          aci[mi][ni][rr] = v.y;
        }
      } else {
        acr[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
        aci[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
      }
    }
  const GemmTerm t0{A0 + (int64_t)(wr + lr) * lda0 + lk, B0 + (int64_t)lk * ldb0 + wc + lr, lda0, ldb0};
  if (A1 != nullptr) {
    const GemmTerm t1{A1 + (int64_t)(wr + lr) * lda1 + lk, B1 + (int64_t)lk * ldb1 + wc + lr, lda1, ldb1};
    tile_nt_gemm<2>(acr, aci, t0, t1);
  } else {
    tile_nt_gemm<1>(acr, aci, t0, t0);
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = wr + mi * 16 + lk + 4 * rr, col = wc + ni * 16 + lr;
        const double2 v = make_double2(acr[mi][ni][rr], aci[mi][ni][rr]);
        out[(int64_t)row * ldo + col] = v;
        if (out2) out2[row * kGJ + col] = v;
      }
  // designated tile stores the pivot inverse into the diagonal block
  const int dI = mode == 0 ? (k == 0 ? 1 : 0) : (k == 0 ? 0 : 0);
  const int pk = mode == 0 ? k : k + 1;
  if (mode != 1 && I == dI && J == pk) {
    const double2* Pb = (mode == 0 ? pn.Pb1 : pn.Pb2) + pvb;
    double2* Sk = Mb + (int64_t)(pk * kGJ) * Np + pk * kGJ;
    for (int e = tid; e < kGJ * kGJ; e += blockDim.x) Sk[(int64_t)(e >> 6) * Np + (e & 63)] = Pb[e];
  }
}

// ---------------------------------------------------------------------------
// Pairing values of D for every chain, slot-major so that lanes indexed by
// row load contiguously: Dv[c][s][r] = Δ_c[Dsrc[r][s]] / 2 (the reference's
// overwrite order is resolved on the host into Dsrc).
// ---------------------------------------------------------------------------
__global__ void k_dvals(const int* __restrict__ Dsrc, const double2* __restrict__ Delta,
                        double2* __restrict__ Dv, int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (e >= N * kSlots) return;
  const int src = Dsrc[e];
  const double2 d = src >= 0 ? Delta[(int64_t)c * 2 * N + src] : make_double2(0.0, 0.0);
  const int r = e / kSlots, sl = e - r * kSlots;
  Dv[(int64_t)c * N * kSlots + (int64_t)sl * N + r] = make_double2(0.5 * d.x, 0.5 * d.y);
}

// ---------------------------------------------------------------------------
// Assembly of S^T for one row a of one (chain, pole):
//   TT[a,k]  = Σ_{l ∈ Dcol(a)} D[a,l] R[l,k]               (rows of R, coalesced)
//   S^T[a,b] = -(h[a,b] + i y δ_ab) - Σ_{k ∈ Dcol(b)} TT[a,k] conj(D[b,k])
// T = R D is not stored: k_contract rebuilds its rows from rows of R.
// ---------------------------------------------------------------------------
static_assert(kSlots == 4, "k_assemble / k_contract load the pairing pattern as int4");
__global__ __launch_bounds__(256) void k_assemble(const double2* __restrict__ R,
                                                  double2* __restrict__ S, int64_t mat, int N,
                                                  int Np, int P, const int* __restrict__ Dcol,
                                                  const double2* __restrict__ Dv,
                                                  const int* __restrict__ hcol,
                                                  const double* __restrict__ hval,
                                                  const double* __restrict__ ypole) {
  extern __shared__ double2 smem[];
  double2* TTrow = smem;
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int bi = item / Np, a = item - bi * Np;
  const int c = bi / P, q = bi % P;
  double2* Srow = S + (int64_t)bi * mat + (int64_t)a * Np;
  if (a >= N) {  // padding rows: identity
    for (int b = threadIdx.x; b < Np; b += blockDim.x)
      Srow[b] = make_double2(b == a ? 1.0 : 0.0, 0.0);
    return;
  }
  const double2* Rb = R + (int64_t)bi * mat;
  const double2* Dvc = Dv + (int64_t)c * N * kSlots;
  int lcol[kSlots];
  double2 dval[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    lcol[s] = Dcol[a * kSlots + s];
    dval[s] = Dvc[s * N + a];
  }
  __shared__ int hc[kHSlots];
  __shared__ double hv[kHSlots];
  if (threadIdx.x < kHSlots) {
    hc[threadIdx.x] = hcol[a * kHSlots + threadIdx.x];
    hv[threadIdx.x] = hval[((int64_t)c * N + a) * kHSlots + threadIdx.x];
  }
  for (int kk = threadIdx.x; kk < N; kk += blockDim.x) {
    double2 tt = make_double2(0.0, 0.0);
#pragma unroll
    for (int s = 0; s < kSlots; ++s)
      if (lcol[s] >= 0) tt = cadd(tt, cmul(dval[s], Rb[(int64_t)lcol[s] * Np + kk]));
    TTrow[kk] = tt;
  }
  __syncthreads();
  const double y = ypole[q];
  for (int b = threadIdx.x; b < Np; b += blockDim.x) {
    double2 st = make_double2(0.0, 0.0);
    if (b < N) {
      const int4 kc4 = *reinterpret_cast<const int4*>(Dcol + b * kSlots);
      const int kc[4] = {kc4.x, kc4.y, kc4.z, kc4.w};
#pragma unroll
      for (int s = 0; s < kSlots; ++s)
        if (kc[s] >= 0) st = cadd(st, cmulc(TTrow[kc[s]], Dvc[s * N + b]));
#pragma unroll
      for (int s = 0; s < kHSlots; ++s)
        if (hc[s] == b) st.x += hv[s];
      if (b == a) st.y += y;
    }
    Srow[b] = make_double2(-st.x, -st.y);
  }
}

// ---------------------------------------------------------------------------
// Contraction: G12[i, j] = -Σ_k T[i,k] S^-1[k,j] = -Σ_k T[i,k] SinvT[j,k]
// for the ≤4 pairing columns j of row i; plus diag(S^-1) for Tr ρ_hh.
// T[i,k] = Σ_{l ∈ Dcol(k)} R[i,l] D[k,l] is rebuilt on the fly from row i of R
// (staged in LDS), so T never goes through HBM.
// ---------------------------------------------------------------------------
template <int NT, bool TWO_PASS>
__global__ __launch_bounds__(NT) void k_contract(const double2* __restrict__ R,
                                                 const double2* __restrict__ SinvT, int64_t mat,
                                                 int N, int Np, int P, const int* __restrict__ Dcol,
                                                 const double2* __restrict__ Dv,
                                                 double2* __restrict__ G12nn,
                                                 double2* __restrict__ diagS) {
  constexpr int NW = NT / 64;
  extern __shared__ double2 smem[];
  double2* Rrow = smem;
  double2* Trow = smem + Np;   // TWO_PASS only
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int bi = item / N, i = item - bi * N;
  const int c = bi / P;
  const double2* Ri = R + (int64_t)bi * mat + (int64_t)i * Np;
  const double2* Sb = SinvT + (int64_t)bi * mat;
  const double2* Dvc = Dv + (int64_t)c * N * kSlots;
  for (int kk = threadIdx.x; kk < N; kk += NT) Rrow[kk] = Ri[kk];
  int js[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) js[s] = Dcol[i * kSlots + s];
  __syncthreads();
  auto trow = [&](int kk) {
    const int4 lc = *reinterpret_cast<const int4*>(Dcol + kk * kSlots);
    const int ls[4] = {lc.x, lc.y, lc.z, lc.w};
    double2 t = make_double2(0.0, 0.0);
#pragma unroll
    for (int s = 0; s < kSlots; ++s)
      if (ls[s] >= 0) t = cadd(t, cmul(Rrow[ls[s]], Dvc[s * N + kk]));
    return t;
  };
  if (TWO_PASS) {
    for (int kk = threadIdx.x; kk < N; kk += NT) Trow[kk] = trow(kk);
    __syncthreads();
  }
  double acc[2 * kSlots];
#pragma unroll
  for (int s = 0; s < 2 * kSlots; ++s) acc[s] = 0.0;
#pragma unroll 4
  for (int kk = threadIdx.x; kk < N; kk += NT) {
    const double2 t = TWO_PASS ? Trow[kk] : trow(kk);
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      if (js[s] >= 0) {
        const double2 v = Sb[(int64_t)js[s] * Np + kk];
        acc[2 * s] += t.x * v.x - t.y * v.y;
        acc[2 * s + 1] += t.x * v.y + t.y * v.x;
      }
    }
  }
  __shared__ double red[NW][2 * kSlots];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < 2 * kSlots; ++s) {
    const double v = wave_sum(acc[s]);
    if (l == 0) red[w][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < 2 * kSlots) {
    const int s = threadIdx.x;
    double v = 0.0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][s];
    double* out = reinterpret_cast<double*>(G12nn + ((int64_t)bi * N + i) * kSlots);
    out[s] = js[s >> 1] >= 0 ? -v : 0.0;
  }
  if (threadIdx.x == 0) diagS[(int64_t)bi * N + i] = Sb[(int64_t)i * Np + i];
}

// ---------------------------------------------------------------------------
// Bond-level kernels (O(N)).  Bond b = i + N*dir, chain c: offset c*2N + b.
// ---------------------------------------------------------------------------
__global__ void k_pair_force(const double2* __restrict__ G12nn, const int* __restrict__ bond_ij,
                             const int* __restrict__ bond_ji, const double* __restrict__ cpole,
                             int N, int P, double2* __restrict__ Delta,
                             double2* __restrict__ Pair, double2* __restrict__ F,
                             double2* __restrict__ Pi, double kick, double drift, double cap2,
                             int* __restrict__ flag, double beta, double J) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (b >= 2 * N) return;
  const int ij = bond_ij[b], ji = bond_ji[b];
  double2 Pv = make_double2(0.0, 0.0);
  for (int q = 0; q < P; ++q) {
    const double2* G = G12nn + (int64_t)(c * P + q) * N * kSlots;
    const double2 g1 = G[ij], g2 = G[ji];
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

__global__ void k_force_from_pair(const double2* __restrict__ Pair, double2* __restrict__ Delta,
                                  double2* __restrict__ F, double2* __restrict__ Pi, int N,
                                  double kick, double drift, double cap2, int* __restrict__ flag,
                                  double beta, double J) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (b >= 2 * N) return;
  const int64_t o = (int64_t)c * 2 * N + b;
  const double2 Pv = Pair[o], d = Delta[o];
  const double f = -beta / (2.0 * J);
  const double2 Fv = make_double2(f * (d.x - J * Pv.x), f * (d.y - J * Pv.y));
  F[o] = Fv;
  kick_drift(Fv, o, Delta, Pi, kick, drift, cap2, flag);
}

__global__ __launch_bounds__(256) void k_fermion_energy(const double* __restrict__ ldstatic,
                                                        const double* __restrict__ ldpart,
                                                        const double2* __restrict__ diagS,
                                                        const double* __restrict__ cpole, int N,
                                                        int nb, int P, double Cx, double beta,
                                                        double* __restrict__ Ef,
                                                        double* __restrict__ Trhh) {
  const int c = blockIdx.x;
  __shared__ double red[4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double ef_acc = 0.0, tr_acc = 0.0;
  for (int q = 0; q < P; ++q) {
    const int bi = c * P + q;
    double ld = 0.0, tr = 0.0;
    for (int k = threadIdx.x; k < nb; k += blockDim.x) ld += ldpart[(int64_t)bi * nb + k];
    for (int i = threadIdx.x; i < N; i += blockDim.x) tr += diagS[(int64_t)bi * N + i].x;
    ld = wave_sum(ld);
    if (l == 0) red[w] = ld;
    __syncthreads();
    ld = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    tr = wave_sum(tr);
    if (l == 0) red[w] = tr;
    __syncthreads();
    tr = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    ef_acc += cpole[q] * (ldstatic[bi] + ld);
    tr_acc += cpole[q] * tr;
  }
  if (threadIdx.x == 0) {
    Ef[c] = -2.0 * N * Cx - beta * ef_acc;
    Trhh[c] = 0.5 * N - tr_acc;
  }
}

__global__ __launch_bounds__(256) void k_total_energy(const double2* __restrict__ Delta,
                                                      const double2* __restrict__ Pi,
                                                      const double* __restrict__ Ef, int N,
                                                      double beta, double J, double mass,
                                                      double* __restrict__ Hout) {
  const int c = blockIdx.x;
  __shared__ double red[2][4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double sd = 0.0, sp = 0.0;
  for (int b = threadIdx.x; b < 2 * N; b += blockDim.x) {
    const double2 d = Delta[(int64_t)c * 2 * N + b];
    const double2 p = Pi[(int64_t)c * 2 * N + b];
    sd += d.x * d.x + d.y * d.y;
    sp += p.x * p.x + p.y * p.y;
  }
  sd = wave_sum(sd);
  sp = wave_sum(sp);
  if (l == 0) {
    red[0][w] = sd;
    red[1][w] = sp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double SD = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const double SP = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    Hout[c] = (1.0 / (2.0 * mass)) * SP + (beta / (2.0 * J)) * SD + Ef[c];
  }
}

__global__ void k_refresh(const double2* __restrict__ noise, double2* __restrict__ Pi, int n,
                          double scale) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const double2 z = noise[o];
  Pi[o] = make_double2(z.x * scale, z.y * scale);
}

__global__ void k_backup(const double2* __restrict__ Delta, const double2* __restrict__ Pair,
                         const double* __restrict__ Ef, const double* __restrict__ Trhh,
                         double2* __restrict__ DeltaB, double2* __restrict__ PairB,
                         double* __restrict__ EfB, double* __restrict__ TrhhB, int n, int nc) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o < n) {
    DeltaB[o] = Delta[o];
    PairB[o] = Pair[o];
  }
  if (o < nc) {
    EfB[o] = Ef[o];
    TrhhB[o] = Trhh[o];
  }
}

__global__ void k_metropolis(const double* __restrict__ Hold, const double* __restrict__ Hnew,
                             const double* __restrict__ uniform, uint8_t* __restrict__ accepted,
                             double* __restrict__ dH, int nc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const double d = Hnew[c] - Hold[c];
  // src/HMC.jl:128 — accept if ΔH < 0 || rand() < exp(-ΔH)
  const bool acc = (d < 0.0) || (uniform[c] < exp(-d));
  accepted[c] = acc ? 1 : 0;
  dH[c] = d;
}

__global__ void k_restore(const uint8_t* __restrict__ accepted, const double2* __restrict__ DeltaB,
                          const double2* __restrict__ PairB, const double* __restrict__ EfB,
                          const double* __restrict__ TrhhB, double2* __restrict__ Delta,
                          double2* __restrict__ Pair, double* __restrict__ Ef,
                          double* __restrict__ Trhh, int N) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (accepted[c]) return;
  if (b < 2 * N) {
    const int64_t o = (int64_t)c * 2 * N + b;
    Delta[o] = DeltaB[o];
    Pair[o] = PairB[o];
  }
  if (b == 0) {
    Ef[c] = EfB[c];
    Trhh[c] = TrhhB[c];
  }
}

// ---------------------------------------------------------------------------
// Trajectory start and end of the throughput path, one workgroup per chain
// (src/HMC.jl:71-144); the energy sums keep k_total_energy's order (256
// threads, strided bonds, wave sums, 4 partials), so H_old / H_new are the
// same bits as the separate kernels give.
//   begin: π = noise·sqrt(2m) (:77), H_old (:80), backup of Δ, P, E_f, Tr ρ_hh
//          (:84-86), F from the cached P, the first half kick and (Nt > 0) the
//          first drift (:91-92, :101)
//   end:   H_new (:122), Metropolis (:124-129), restore on rejection (:130-141)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double block_sum256(double v, double* red) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  v = wave_sum(v);
  if (l == 0) red[w] = v;
  __syncthreads();
  const double t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(256) void k_traj_begin(const double2* __restrict__ noise, double scale,
                                                    double2* __restrict__ Pi, double2* __restrict__ Delta,
                                                    const double2* __restrict__ Pair, double2* __restrict__ F,
                                                    const double* __restrict__ Ef, const double* __restrict__ Trhh,
                                                    double2* __restrict__ DeltaB, double2* __restrict__ PairB,
                                                    double* __restrict__ EfB, double* __restrict__ TrhhB,
                                                    double* __restrict__ Hold, int N, double beta, double J,
                                                    double mass, double kick, double drift, double cap2,
                                                    int* __restrict__ flag, const int* __restrict__ halt) {
  const int c = blockIdx.x;
  // a guard trip earlier in this batch (SweepHalt): keep the backups
  if (halt != nullptr && halt[0] != 0) return;
  __shared__ double red[4];
  double sd = 0.0, sp = 0.0;
  const double f = -beta / (2.0 * J);
  for (int b = threadIdx.x; b < 2 * N; b += blockDim.x) {
    const int64_t o = (int64_t)c * 2 * N + b;
    const double2 z = noise[o], d = Delta[o], P = Pair[o];
    const double2 p = make_double2(z.x * scale, z.y * scale);
    sd += d.x * d.x + d.y * d.y;
    sp += p.x * p.x + p.y * p.y;
    DeltaB[o] = d;
    PairB[o] = P;
    Pi[o] = p;
    const double2 Fv = make_double2(f * (d.x - J * P.x), f * (d.y - J * P.y));
    F[o] = Fv;
    kick_drift(Fv, o, Delta, Pi, kick, drift, cap2, flag);
  }
  const double SD = block_sum256(sd, red), SP = block_sum256(sp, red);
  if (threadIdx.x == 0) {
    Hold[c] = (1.0 / (2.0 * mass)) * SP + (beta / (2.0 * J)) * SD + Ef[c];
    EfB[c] = Ef[c];
    TrhhB[c] = Trhh[c];
  }
}

__global__ __launch_bounds__(256) void k_traj_end(double2* __restrict__ Delta, const double2* __restrict__ Pi,
                                                  double2* __restrict__ Pair, double* __restrict__ Ef,
                                                  double* __restrict__ Trhh, const double2* __restrict__ DeltaB,
                                                  const double2* __restrict__ PairB, const double* __restrict__ EfB,
                                                  const double* __restrict__ TrhhB, const double* __restrict__ Hold,
                                                  double* __restrict__ Hnew, const double* __restrict__ uniform,
                                                  uint8_t* __restrict__ accepted, double* __restrict__ dH, int N,
                                                  double beta, double J, double mass, int* __restrict__ halt,
                                                  int seq, const int* __restrict__ flag) {
  const int c = blockIdx.x;
  if (halt != nullptr) {
    // *flag comes from earlier launches; halt[0] may also be set by chain 0's
    // workgroup of this launch, which only makes the others return as well
    if (halt[0] != 0) return;
    if (*flag != 0) {
      if (c == 0 && threadIdx.x == 0) {
        halt[1] = seq;
        halt[0] = 1;
      }
      return;
    }
  }
  __shared__ double red[4];
  __shared__ int acc_s;
  double sd = 0.0, sp = 0.0;
  for (int b = threadIdx.x; b < 2 * N; b += blockDim.x) {
    const double2 d = Delta[(int64_t)c * 2 * N + b];
    const double2 p = Pi[(int64_t)c * 2 * N + b];
    sd += d.x * d.x + d.y * d.y;
    sp += p.x * p.x + p.y * p.y;
  }
  const double SD = block_sum256(sd, red), SP = block_sum256(sp, red);
  if (threadIdx.x == 0) {
    const double h = (1.0 / (2.0 * mass)) * SP + (beta / (2.0 * J)) * SD + Ef[c];
    Hnew[c] = h;
    const double dd = h - Hold[c];
    const bool acc = (dd < 0.0) || (uniform[c] < exp(-dd));   // src/HMC.jl:128
    accepted[c] = acc ? 1 : 0;
    dH[c] = dd;
    acc_s = acc;
  }
  __syncthreads();
  if (acc_s) return;
  for (int b = threadIdx.x; b < 2 * N; b += blockDim.x) {
    const int64_t o = (int64_t)c * 2 * N + b;
    Delta[o] = DeltaB[o];
    Pair[o] = PairB[o];
  }
  if (threadIdx.x == 0) {
    Ef[c] = EfB[c];
    Trhh[c] = TrhhB[c];
  }
}

__global__ void k_sum_ld(const double* __restrict__ ldpart, double* __restrict__ ldsum, int nb,
                         int nbatch) {
  const int bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= nbatch) return;
  double s = 0.0;
  for (int k = 0; k < nb; ++k) s += ldpart[(int64_t)bi * nb + k];
  ldsum[bi] = s;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline dim3 bonds_grid(const Dims& d) { return dim3((2 * d.N + 255) / 256, d.nc); }

void launch_fill_hz(const Dims& d, double2* M, const int* hcol, const double* hval,
                    const double* ypole, hipStream_t s) {
  hipLaunchKernelGGL(k_fill_hz, dim3(d.Np, d.nbatch), dim3(256), 0, s, M, d.mat, d.N, d.Np, d.P,
                     hcol, hval, ypole);
}
void launch_gj_pivot(const Dims& d, double2* M, int k, double2* Pout, double2* XRout,
                     double2* colcopy, double2* nextcol, double* ldpart, hipStream_t s) {
  hipLaunchKernelGGL(k_gj_pivot, dim3(d.nb, d.nbatch), dim3(256), 0, s, M, d.mat, d.Np, d.nb, k,
                     Pout, XRout, colcopy, nextcol, ldpart);
}
int gj_update_tiles(const Dims& d, int mode) {
  if (d.nb < 2) return 0;
  return mode == 1 ? 2 * d.nb - 2 : (d.nb - 1) * d.nb;
}
void launch_gj_update(const Dims& d, double2* M, int k, int mode, const GJPanelPtrs& p,
                      hipStream_t s) {
  const int tiles = gj_update_tiles(d, mode);
  if (tiles <= 0) return;
  const int total = tiles * d.nbatch;
  GJPanels pn{p.CpA, p.CpB, p.XR1, p.XR2, p.Pb1, p.Pb2, p.CpBw, p.CpN};
  switch (mode) {
    case 0: hipLaunchKernelGGL(k_gj_update<0>, dim3(total), dim3(256), 0, s, M, d.mat, d.Np, d.nb, k, total, pn); break;
    case 1: hipLaunchKernelGGL(k_gj_update<1>, dim3(total), dim3(256), 0, s, M, d.mat, d.Np, d.nb, k, total, pn); break;
    default: hipLaunchKernelGGL(k_gj_update<2>, dim3(total), dim3(256), 0, s, M, d.mat, d.Np, d.nb, k, total, pn); break;
  }
}
void launch_dvals(const Dims& d, const int* Dsrc, const double2* Delta, double2* Dv,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_dvals, dim3((d.N * kSlots + 255) / 256, d.nc), dim3(256), 0, s, Dsrc, Delta,
                     Dv, d.N);
}
void launch_assemble(const Dims& d, const double2* R, double2* S, const int* Dcol,
                     const double2* Dv, const int* hcol, const double* hval, const double* ypole,
                     hipStream_t s) {
  const size_t shm = (size_t)d.Np * sizeof(double2);
#ifndef DWH_ASSEMBLE_NT
#define DWH_ASSEMBLE_NT 256
#endif
  hipLaunchKernelGGL(k_assemble, dim3(d.Np * d.nbatch), dim3(DWH_ASSEMBLE_NT), shm, s, R, S, d.mat,
                     d.N, d.Np, d.P, Dcol, Dv, hcol, hval, ypole);
}
void launch_contract(const Dims& d, const double2* R, const double2* SinvT, const int* Dcol,
                     const double2* Dv, double2* G12nn, double2* diagS, hipStream_t s) {
#ifndef DWH_CONTRACT_NT
#define DWH_CONTRACT_NT 256
#endif
#ifndef DWH_CONTRACT_2P
#define DWH_CONTRACT_2P false
#endif
  const size_t shm = (DWH_CONTRACT_2P ? 2 : 1) * (size_t)d.Np * sizeof(double2);
  hipLaunchKernelGGL((k_contract<DWH_CONTRACT_NT, DWH_CONTRACT_2P>), dim3(d.N * d.nbatch),
                     dim3(DWH_CONTRACT_NT), shm, s, R, SinvT, d.mat, d.N, d.Np, d.P, Dcol, Dv, G12nn,
                     diagS);
}
void launch_pair_force(const Dims& d, const double2* G12nn, const int* bond_ij,
                       const int* bond_ji, const double* cpole, double2* Delta, double2* Pair,
                       double2* F, double2* Pi, const KickDrift& kd, double beta, double J,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_pair_force, bonds_grid(d), dim3(256), 0, s, G12nn, bond_ij, bond_ji, cpole,
                     d.N, d.P, Delta, Pair, F, Pi, kd.kick, kd.drift, kd.cap * kd.cap, kd.flag, beta,
                     J);
}
void launch_force_from_pair(const Dims& d, const double2* Pair, double2* Delta, double2* F,
                            double2* Pi, const KickDrift& kd, double beta, double J, hipStream_t s) {
  hipLaunchKernelGGL(k_force_from_pair, bonds_grid(d), dim3(256), 0, s, Pair, Delta, F, Pi, d.N,
                     kd.kick, kd.drift, kd.cap * kd.cap, kd.flag, beta, J);
}
void launch_fermion_energy(const Dims& d, const double* ldstatic, const double* ldpart,
                           const double2* diagS, const double* cpole, double Cx, double beta,
                           double* Ef, double* Trhh, hipStream_t s) {
  hipLaunchKernelGGL(k_fermion_energy, dim3(d.nc), dim3(256), 0, s, ldstatic, ldpart, diagS, cpole,
                     d.N, d.nld, d.P, Cx, beta, Ef, Trhh);
}
void launch_total_energy(const Dims& d, const double2* Delta, const double2* Pi,
                         const double* Ef, double beta, double J, double mass, double* Hout,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_total_energy, dim3(d.nc), dim3(256), 0, s, Delta, Pi, Ef, d.N, beta, J,
                     mass, Hout);
}
void launch_refresh(const Dims& d, const double2* noise, double2* Pi, double scale, hipStream_t s) {
  const int n = 2 * d.N * d.nc;
  hipLaunchKernelGGL(k_refresh, dim3((n + 255) / 256), dim3(256), 0, s, noise, Pi, n, scale);
}
void launch_backup(const Dims& d, const double2* Delta, const double2* Pair, const double* Ef,
                   const double* Trhh, double2* DeltaB, double2* PairB, double* EfB,
                   double* TrhhB, hipStream_t s) {
  const int n = 2 * d.N * d.nc;
  const int m = n > d.nc ? n : d.nc;
  hipLaunchKernelGGL(k_backup, dim3((m + 255) / 256), dim3(256), 0, s, Delta, Pair, Ef, Trhh,
                     DeltaB, PairB, EfB, TrhhB, n, d.nc);
}
void launch_metropolis(const Dims& d, const double* Hold, const double* Hnew,
                       const double* uniform, uint8_t* accepted, double* dH, hipStream_t s) {
  hipLaunchKernelGGL(k_metropolis, dim3((d.nc + 63) / 64), dim3(64), 0, s, Hold, Hnew, uniform,
                     accepted, dH, d.nc);
}
void launch_restore(const Dims& d, const uint8_t* accepted, const double2* DeltaB,
                    const double2* PairB, const double* EfB, const double* TrhhB,
                    double2* Delta, double2* Pair, double* Ef, double* Trhh, hipStream_t s) {
  hipLaunchKernelGGL(k_restore, bonds_grid(d), dim3(256), 0, s, accepted, DeltaB, PairB, EfB,
                     TrhhB, Delta, Pair, Ef, Trhh, d.N);
}
void launch_traj_begin(const Dims& d, const double2* noise, double scale, double2* Pi, double2* Delta,
                       const double2* Pair, double2* F, const double* Ef, const double* Trhh, double2* DeltaB,
                       double2* PairB, double* EfB, double* TrhhB, double* Hold, double beta, double J,
                       double mass, const KickDrift& kd, const SweepHalt& sh, hipStream_t s) {
  hipLaunchKernelGGL(k_traj_begin, dim3(d.nc), dim3(256), 0, s, noise, scale, Pi, Delta, Pair, F, Ef, Trhh,
                     DeltaB, PairB, EfB, TrhhB, Hold, d.N, beta, J, mass, kd.kick, kd.drift, kd.cap * kd.cap,
                     kd.flag, (const int*)sh.halt);
}
void launch_traj_end(const Dims& d, double2* Delta, const double2* Pi, double2* Pair, double* Ef, double* Trhh,
                     const double2* DeltaB, const double2* PairB, const double* EfB, const double* TrhhB,
                     const double* Hold, double* Hnew, const double* uniform, uint8_t* accepted, double* dH,
                     double beta, double J, double mass, const SweepHalt& sh, hipStream_t s) {
  hipLaunchKernelGGL(k_traj_end, dim3(d.nc), dim3(256), 0, s, Delta, Pi, Pair, Ef, Trhh, DeltaB, PairB, EfB,
                     TrhhB, Hold, Hnew, uniform, accepted, dH, d.N, beta, J, mass, sh.halt, sh.seq, sh.flag);
}
void launch_sum_ld(const Dims& d, const double* ldpart, double* ldsum, hipStream_t s) {
  hipLaunchKernelGGL(k_sum_ld, dim3((d.nbatch + 63) / 64), dim3(64), 0, s, ldpart, ldsum, d.nb,
                     d.nbatch);
}

// ---------------------------------------------------------------------------
// MFMA f64 layout self-test (A = asymmetric integers, B asymmetric): exact.
// ---------------------------------------------------------------------------
__global__ void k_mfma_layout(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)],
                                            acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

int selftest_mfma_layout(int device) {
  if (hipSetDevice(device) != hipSuccess) return -2;
  double hA[64], hB[64], hD[256];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 4; ++k) hA[i * 4 + k] = (double)(i * 7 + k * 3 + 1);
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (double)(k * 11 - j * 2 + 5);
  double *dA, *dB, *dD;
  if (hipMalloc(&dA, sizeof hA) != hipSuccess) return -2;
  if (hipMalloc(&dB, sizeof hB) != hipSuccess) return -2;
  if (hipMalloc(&dD, sizeof hD) != hipSuccess) return -2;
  (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_mfma_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  (void)hipFree(dA);
  (void)hipFree(dB);
  (void)hipFree(dD);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double r = 0;
      for (int k = 0; k < 4; ++k) r += hA[i * 4 + k] * hB[k * 16 + j];
      if (r != hD[i * 16 + j]) ++bad;
    }
  return bad;
}

}  // namespace dwh
