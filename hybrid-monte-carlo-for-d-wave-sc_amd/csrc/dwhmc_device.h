// Device helpers shared by the dense Gauss-Jordan (dwhmc_kernels.hip) and the
// block cyclic-reduction (dwhmc_cr.hip) kernels: complex arithmetic, the
// XCD-aware grid remap, wave reductions, the wave-local 16x16 complex
// inversion and the LDS-operand complex MFMA step (v_mfma_f64_16x16x4_f64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

// CDNA4 only: LDS footprints above 64 KiB per workgroup, f64 MFMA layouts of gfx950
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libdwhmc device code targets gfx950 (MI355X) only"
#endif

namespace dwh {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a * conj(b)
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {
  return make_double2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cinv(double2 a) {
  const double s = 1.0 / (a.x * a.x + a.y * a.y);
  return make_double2(a.x * s, -a.y * s);
}
// 1/a with v_rcp_f64 + two Newton steps (error ~1 ulp; the IEEE division
// sequence has ~3x the latency and sits on the pivot dependency chain).
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}
__device__ __forceinline__ double2 cinv_fast(double2 a) {
  const double s = rcp_nr(fma(a.x, a.x, a.y * a.y));
  return make_double2(a.x * s, -a.y * s);
}

// Bijective XCD-aware remap of a 1D grid (cdna_hip_programming.md §5): blocks
// b and b+8 share an XCD, so item ranges [x*q, (x+1)*q) are given to one XCD
// and neighbouring rows of one matrix share that XCD's L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int total) {
  const int q = total / 8, r = total % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// The same grouping for a 2D grid (x: work within a batch item, y: batch
// item): this workgroup's (x, y) after remapping its linear index, so a
// batch item's workgroups share an XCD (and the XCD the block-product stages
// give it, up to rounding), and the blocks one stage writes are read by the
// next through that XCD's L2.  -DCR_XCD_ITEMS=0: hardware order (A/B).
#ifndef CR_XCD_ITEMS
#define CR_XCD_ITEMS 1
#endif
__device__ __forceinline__ int2 xcd_grid2d() {
#if CR_XCD_ITEMS
  const int nx = gridDim.x, g = xcd_remap(blockIdx.x + nx * blockIdx.y, nx * gridDim.y);
  return make_int2(g % nx, g / nx);
#else
  return make_int2(blockIdx.x, blockIdx.y);
#endif
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// 16x16 complex block in one wave: lane l holds row l>>2, columns (l&3)*4..+3.
// Row p and column p are exchanged through a per-wave LDS scratch (xb: 16
// row + 16 column entries) between wavefront-scope fences; the update is
// branch-free (selects instead of a divergent row-p path).  pm receives
// |pivot|^2 (lane 0) when non-null.
__device__ __forceinline__ void wave_inv16(double2 (&a)[4], double2* xb, double* pm, int pbase) {
  const int l = threadIdx.x & 63;
  const int r = l >> 2, cq = l & 3;
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int ps = p >> 2, pe = p & 3;
    const bool prow = (r == p);
    if (prow) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) xb[cq * 4 + jj] = a[jj];
    }
    if (cq == ps) xb[16 + r] = a[pe];
    // cross-lane hand-off: the fences are compiler ordering points (a plain
    // predicated store/load pair may legally be reordered for other lanes)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double2 piv = xb[p];
    const double2 colp = xb[16 + r];
    double2 rowp[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) rowp[jj] = xb[cq * 4 + jj];
    const double2 inv = cinv_fast(piv);
    if (pm != nullptr && l == 0) pm[pbase + p] = piv.x * piv.x + piv.y * piv.y;
    // row p: a <- rowp * inv ; other rows: a <- a - (colp*inv) * rowp
    const double2 fi = cmul(colp, inv);
    const double2 g = prow ? make_double2(-inv.x, -inv.y) : fi;
    const double2 pc = prow ? inv : make_double2(-fi.x, -fi.y);   // new value in column p
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const double2 base = prow ? make_double2(0.0, 0.0) : a[jj];
      const double2 v = csub(base, cmul(g, rowp[jj]));
      a[jj] = (cq * 4 + jj == p) ? pc : v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// acc(16x16, C layout) += sgn * Aop(16 x 16, k) * Bop(16 x 16), complex, 4 MFMA per k-step.
// Aop(m, k) = A[(m) * lda + k], Bop(k, n) = B[k * ldb + n]  (LDS pointers)
template <bool NEG>
__device__ __forceinline__ void mma16_lds(d4& acr, d4& aci, const double2* A, int lda,
                                          const double2* B, int ldb) {
  const int l = threadIdx.x & 63;
  const int lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int ks = 0; ks < 16; ks += 4) {
    const double2 av = A[lr * lda + ks + lk];
    const double2 bv = B[(ks + lk) * ldb + lr];
    const double ar = NEG ? -av.x : av.x, ai = NEG ? -av.y : av.y;
    acr = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, bv.x, acr, 0, 0, 0);
    aci = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, bv.y, aci, 0, 0, 0);
    acr = __builtin_amdgcn_mfma_f64_16x16x4f64(-ai, bv.y, acr, 0, 0, 0);
    aci = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, bv.x, aci, 0, 0, 0);
  }
}

// kick π += kick·F, then (drift != 0) the next leapfrog step's drift
// Δ += drift·π with the |Δ| guard (src/HMC.jl:101 fused with :111-113)
__device__ __forceinline__ void kick_drift(double2 Fv, int64_t o, double2* __restrict__ Delta,
                                           double2* __restrict__ Pi, double kick, double drift,
                                           double cap2, int* __restrict__ flag) {
  if (kick == 0.0 && drift == 0.0) return;
  double2 p = Pi[o];
  p.x += kick * Fv.x;
  p.y += kick * Fv.y;
  Pi[o] = p;
  if (drift != 0.0) {
    double2 d = Delta[o];
    d.x += drift * p.x;
    d.y += drift * p.y;
    Delta[o] = d;
    if (d.x * d.x + d.y * d.y > cap2) atomicOr(flag, 1);
  }
}

// kick_drift with Pi[o] and Delta[o] already loaded (p, d): the caller issues
// those loads before its own long-latency work; returns the drifted Δ
__device__ __forceinline__ double2 kick_drift_pre(double2 Fv, int64_t o, double2 p, double2 d,
                                                  double2* __restrict__ Delta, double2* __restrict__ Pi,
                                                  double kick, double drift, double cap2, int* __restrict__ flag) {
  if (kick == 0.0 && drift == 0.0) return d;
  p.x += kick * Fv.x;
  p.y += kick * Fv.y;
  Pi[o] = p;
  if (drift != 0.0) {
    d.x += drift * p.x;
    d.y += drift * p.y;
    Delta[o] = d;
    if (d.x * d.x + d.y * d.y > cap2) atomicOr(flag, 1);
  }
  return d;
}

// ---------------------------------------------------------------------------
// Register-only 16x16 complex no-pivot Gauss-Jordan inversion in one wave.
// Layout: lane l holds row r = l & 15, columns 4q .. 4q+3 with q = l >> 4.
// Pivot p (compile time): row p reaches every lane of its 16-lane row through
// DPP row_newbcast:p, column p reaches the other column quarters through
// ds_bpermute (LDS crossbar, no LDS storage), the pivot value through
// readlane.  No barriers.  pprod accumulates Π |pivot|^2 (uniform in the wave).
// ---------------------------------------------------------------------------
template <int P>
__device__ __forceinline__ double dpp_rowbcast(double x) {
  // full row/bank masks + bound_ctrl: every lane is written, the old value is dead
  return __builtin_amdgcn_update_dpp(x, x, 0x150 + P, 0xf, 0xf, true);
}

// value of quarter QS (lanes 16 QS .. 16 QS + 15) broadcast to all quarters, per row position
template <int QS>
__device__ __forceinline__ double bcast_quarter(double x) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  // one LDS-crossbar permute per dword (no LDS storage): lane l reads lane
  // 16 QS + (l & 15); 2 instructions per double instead of ~6 with the
  // v_permlane16/32_swap pair and their register copies (the inversion is
  // issue-bound)
  const int src = ((QS << 4) | (threadIdx.x & 15)) << 2;
  const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)(unsigned)b);
  const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)(unsigned)(b >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double readlane_f64(double x, int lane) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, lane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// STRIDED: lane l holds columns q, q + 4, q + 8, q + 12 (q = l >> 4) instead
// of 4q .. 4q + 3 — the MFMA C layout of the transposed tile, so a tile kept
// transposed in MFMA registers is inverted in place without an LDS transpose.
template <int P, bool STRIDED = false>
__device__ __forceinline__ void inv16_step(double2 (&a)[4], double& pprod) {
  constexpr int PS = STRIDED ? (P & 3) : (P >> 2), PE = STRIDED ? (P >> 2) : (P & 3);
  const int l = threadIdx.x & 63, r = l & 15, q = l >> 4;
  double2 rowp[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) rowp[jj] = make_double2(dpp_rowbcast<P>(a[jj].x), dpp_rowbcast<P>(a[jj].y));
  const double2 colp = make_double2(bcast_quarter<PS>(a[PE].x), bcast_quarter<PS>(a[PE].y));
  // the pivot straight from its owner lane, off the column broadcast's chain
  const double2 piv = make_double2(readlane_f64(a[PE].x, PS * 16 + P), readlane_f64(a[PE].y, PS * 16 + P));
  const double m2 = fma(piv.x, piv.x, piv.y * piv.y);
  const double s = rcp_nr(m2);
  const double2 inv = make_double2(piv.x * s, -piv.y * s);
  pprod *= m2;
  const bool prow = (r == P);
  // Select-free form: one update a <- a - f rowp' for every entry.  On the
  // pivot row colp' = piv - 1, so f = (piv - 1)/piv = 1 - 1/piv and the row
  // becomes a_p / piv; in column p rowp' = piv + 1, so the column becomes
  // colp - f (piv + 1) = -colp/piv (1/piv on the pivot row) up to one rounding
  // of colp - f piv.  Replaces ~12 per-lane selects by two adds.
  const double2 fi = cmul(make_double2(colp.x - (prow ? 1.0 : 0.0), colp.y), inv);
  rowp[PE].x += (q == PS) ? 1.0 : 0.0;
  const double2 f = fi;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const double2 x = rowp[jj];
    double2 v;
    v.x = fma(-f.x, x.x, fma(f.y, x.y, a[jj].x));
    v.y = fma(-f.x, x.y, fma(-f.y, x.x, a[jj].y));
    a[jj] = v;
  }
}

template <bool STRIDED, int... Ps>
__device__ __forceinline__ void inv16_all(double2 (&a)[4], double& pprod,
                                          std::integer_sequence<int, Ps...>) {
  (inv16_step<Ps, STRIDED>(a, pprod), ...);
}

// returns Π |pivot|^2 of the 16 pivots
template <bool STRIDED = false>
__device__ __forceinline__ double wave_inv16_dpp(double2 (&a)[4]) {
  double pprod = 1.0;
  inv16_all<STRIDED>(a, pprod, std::make_integer_sequence<int, 16>{});
  return pprod;
}

// In-place inverse of a 16 x 16 tile held in the MFMA C layout (lane: rows
// lk + 4 rr, column lr).  Those registers are the strided layout of the
// transposed tile, and inverting M^T in that layout leaves (M^T)^-1 =
// (M^-1)^T strided, i.e. M^-1 in the C layout.  Returns Π |pivot|^2.
__device__ __forceinline__ double wave_inv16_c(d4& cr, d4& ci) {
  double2 dv[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) dv[jj] = make_double2(cr[jj], ci[jj]);
  const double p = wave_inv16_dpp<true>(dv);
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    cr[jj] = dv[jj].x;
    ci[jj] = dv[jj].y;
  }
  return p;
}

}  // namespace dwh
