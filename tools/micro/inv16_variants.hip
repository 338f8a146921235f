// Diagnostic: variants of the 16x16 register inversion (wave_inv16_dpp, the
// pivot chain of every CR block inversion) — cycles per pivot and agreement
// with the library's form.  One wave per workgroup, REP back-to-back
// inversions of a 16x16 complex tile in the strided layout.
//   V=0 the library's pivot step (dwhmc_device.h inv16_step<P, true>)
//   V=1 column lookahead: column P+1 is broadcast (ds_bpermute) at the start
//       of step P from the pre-update tile and updated by the lanes
//       themselves (the same FMAs as its owner), so the LDS-crossbar round
//       trip leaves the pivot chain; the pivot reaches every lane by a DPP
//       row broadcast of the carried column instead of v_readlane
//   V=2 V=1 with one Newton step on v_rcp_f64 instead of two
//   V=3 panel-blocked: four 4-column panels, scalar steps on the panel only,
//       rank-4 MFMA update of the rest (inv16_panel)
//   V=4 V=1 with the DPP row broadcast fused into the update FMAs
//       (v_fmac_f64_dpp row_newbcast, la_step_fused)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 inv16_variants.hip -o inv16_variants
#include "../../hybrid-monte-carlo-for-d-wave-sc_amd/csrc/dwhmc_device.h"
#include <cmath>
#include <cstdio>
#include <vector>
using namespace dwh;

template <int NR>
__device__ __forceinline__ double rcp_n(double d) {
  double r = __builtin_amdgcn_rcp(d);
#pragma unroll
  for (int k = 0; k < NR; ++k) r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

// column-lookahead pivot step (strided layout: lane (r = l & 15, q = l >> 4),
// a[jj] = A[r][q + 4 jj]); cp: column P of the current tile in every lane of
// row r.  On return cp holds column P + 1 of the updated tile.
template <int P, int NR>
__device__ __forceinline__ void la_step(double2 (&a)[4], double2& cp, double& pprod) {
  constexpr int PS = P & 3, PE = P >> 2;
  constexpr int QN = (P + 1) & 3, EN = (P + 1) >> 2;
  const int l = threadIdx.x & 63, r = l & 15, q = l >> 4;
  // next column (pre-update) and its pivot-row entry A[P][P+1]: off the chain
  double2 cn = make_double2(0.0, 0.0), apn = make_double2(0.0, 0.0);
  if constexpr (P < 15) {
    cn = make_double2(bcast_quarter<QN>(a[EN].x), bcast_quarter<QN>(a[EN].y));
    apn = make_double2(readlane_f64(a[EN].x, QN * 16 + P), readlane_f64(a[EN].y, QN * 16 + P));
  }
  double2 rowp[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) rowp[jj] = make_double2(dpp_rowbcast<P>(a[jj].x), dpp_rowbcast<P>(a[jj].y));
  const double2 piv = make_double2(dpp_rowbcast<P>(cp.x), dpp_rowbcast<P>(cp.y));
  const double m2 = fma(piv.x, piv.x, piv.y * piv.y);
  const double s = rcp_n<NR>(m2);
  const double2 inv = make_double2(piv.x * s, -piv.y * s);
  pprod *= m2;
  const bool prow = (r == P);
  const double2 f = cmul(make_double2(cp.x - (prow ? 1.0 : 0.0), cp.y), inv);
  rowp[PE].x += (q == PS) ? 1.0 : 0.0;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const double2 x = rowp[jj];
    double2 v;
    v.x = fma(-f.x, x.x, fma(f.y, x.y, a[jj].x));
    v.y = fma(-f.x, x.y, fma(-f.y, x.x, a[jj].y));
    a[jj] = v;
  }
  if constexpr (P < 15) {   // the owner's update of column P + 1, replicated
    double2 v;
    v.x = fma(-f.x, apn.x, fma(f.y, apn.y, cn.x));
    v.y = fma(-f.x, apn.y, fma(-f.y, apn.x, cn.y));
    cp = v;
  }
}
// V=4: the column-lookahead step with the DPP row broadcast fused into the
// update FMAs (v_fmac_f64_dpp row_newbcast: src0 read from lane P of each
// 16-lane row), one v_mov_b64 copy per complex entry for the in-place hazard
// (the pivot row's own lanes need their unscaled value after the first FMA);
// the fold's +1 of column P goes onto the pivot element itself (and off again
// after: (a + 1)(1 - f_P) - 1 = 1/piv).
template <int P>
__device__ __forceinline__ void fused_upd(double& ax, double& ay, double nfx, double nfy, double fy) {
  double t;
  asm volatile(
      "s_nop 1\n\t"
      "v_mov_b64 %[t], %[ay]\n\t"
      "v_fmac_f64_dpp %[ay], %[ax], %[nfy] row_newbcast:%c[p] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[ax], %[ax], %[nfx] row_newbcast:%c[p] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[ax], %[t], %[fy] row_newbcast:%c[p] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[ay], %[t], %[nfx] row_newbcast:%c[p] row_mask:0xf bank_mask:0xf"
      : [ax] "+v"(ax), [ay] "+v"(ay), [t] "=&v"(t)
      : [nfx] "v"(nfx), [nfy] "v"(nfy), [fy] "v"(fy), [p] "i"(P));
}
template <int P>
__device__ __forceinline__ void la_step_fused(double2 (&a)[4], double2& cp, double& pprod) {
  constexpr int PS = P & 3, PE = P >> 2;
  constexpr int QN = (P + 1) & 3, EN = (P + 1) >> 2;
  const int l = threadIdx.x & 63, r = l & 15;
  double2 cn = make_double2(0.0, 0.0), apn = make_double2(0.0, 0.0);
  if constexpr (P < 15) {
    cn = make_double2(bcast_quarter<QN>(a[EN].x), bcast_quarter<QN>(a[EN].y));
    apn = make_double2(readlane_f64(a[EN].x, QN * 16 + P), readlane_f64(a[EN].y, QN * 16 + P));
  }
  const double2 piv = make_double2(dpp_rowbcast<P>(cp.x), dpp_rowbcast<P>(cp.y));
  const double m2 = fma(piv.x, piv.x, piv.y * piv.y);
  const double s = rcp_n<2>(m2);
  const double2 inv = make_double2(piv.x * s, -piv.y * s);
  pprod *= m2;
  const bool prow = (r == P);
  const double2 f = cmul(make_double2(cp.x - (prow ? 1.0 : 0.0), cp.y), inv);
  const bool pl = l == PS * 16 + P;   // the pivot element's lane
  a[PE].x += pl ? 1.0 : 0.0;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) fused_upd<P>(a[jj].x, a[jj].y, -f.x, -f.y, f.y);
  a[PE].x -= pl ? 1.0 : 0.0;
  if constexpr (P < 15) {
    double2 v;
    v.x = fma(-f.x, apn.x, fma(f.y, apn.y, cn.x));
    v.y = fma(-f.x, apn.y, fma(-f.y, apn.x, cn.y));
    cp = v;
  }
}
template <int... Ps>
__device__ __forceinline__ void la_fused_all(double2 (&a)[4], double& pprod, std::integer_sequence<int, Ps...>) {
  double2 cp = make_double2(bcast_quarter<0>(a[0].x), bcast_quarter<0>(a[0].y));
  (la_step_fused<Ps>(a, cp, pprod), ...);
}

template <int NR, int... Ps>
__device__ __forceinline__ void la_all(double2 (&a)[4], double& pprod, std::integer_sequence<int, Ps...>) {
  double2 cp = make_double2(bcast_quarter<0>(a[0].x), bcast_quarter<0>(a[0].y));
  (la_step<Ps, NR>(a, cp, pprod), ...);
}

// Panel-blocked form: four 4-column panels.  Panel j (pivots K = 4j..4j+3):
// the old pivot rows R = T[K, :] go to LDS (off the chain), the panel
// T[:, K] (register j of every lane: one complex per lane) takes its four
// Gauss-Jordan steps alone (2 DPP + 4 ds_bpermute + the reciprocal + 4 FMAs
// each, instead of 8 DPP + 16 FMAs on the whole tile), leaving C' = T'[:, K];
// with F = E - C' the other columns follow by one rank-4 update
// T[:, J] -= F R[:, J], run as T^T -= R^T F^T on the MFMA: the strided layout
// is the C layout of T^T, F^T is the B operand exactly as register j holds F,
// and R^T is the A operand read back from LDS (rows of K zeroed, so register
// j keeps C').  Complex MACs as 4 real MFMAs accumulating in place.
template <int J, int K, int NR>
__device__ __forceinline__ void panel_step(double2& c, double& pprod) {
  constexpr int P = 4 * J + K;
  const int l = threadIdx.x & 63, r = l & 15, q = l >> 4;
  const double2 rowp = make_double2(dpp_rowbcast<P>(c.x), dpp_rowbcast<P>(c.y));
  const double2 colp = make_double2(bcast_quarter<K>(c.x), bcast_quarter<K>(c.y));
  const double2 piv = make_double2(dpp_rowbcast<P>(colp.x), dpp_rowbcast<P>(colp.y));
  const double m2 = fma(piv.x, piv.x, piv.y * piv.y);
  const double s = rcp_n<NR>(m2);
  const double2 inv = make_double2(piv.x * s, -piv.y * s);
  pprod *= m2;
  const double2 f = cmul(make_double2(colp.x - (r == P ? 1.0 : 0.0), colp.y), inv);
  const double2 x = make_double2(rowp.x + (q == K ? 1.0 : 0.0), rowp.y);
  c.x = fma(-f.x, x.x, fma(f.y, x.y, c.x));
  c.y = fma(-f.x, x.y, fma(-f.y, x.x, c.y));
}

template <int J, int NR>
__device__ __forceinline__ void panel(d4& tr, d4& ti, double2* S, double& pprod) {
  const int l = threadIdx.x & 63, r = l & 15, q = l >> 4;
  // old pivot rows -> LDS S[k][m] = T[4J + k][m]
  if ((r >> 2) == J) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) S[(r & 3) * 16 + q + 4 * jj] = make_double2(tr[jj], ti[jj]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double2 rt = S[q * 16 + r];                 // A operand: R^T[m = r][k = q]
  if ((r >> 2) == J) rt = make_double2(0.0, 0.0);
  double2 c = make_double2(tr[J], ti[J]);
  panel_step<J, 0, NR>(c, pprod);
  panel_step<J, 1, NR>(c, pprod);
  panel_step<J, 2, NR>(c, pprod);
  panel_step<J, 3, NR>(c, pprod);
  tr[J] = c.x;
  ti[J] = c.y;
  // B operand F^T[k = q][n = r] = F[r][q] = delta - C'[r][q]
  const double fr = (r == 4 * J + q ? 1.0 : 0.0) - c.x, fi = -c.y;
  // T^T -= R^T F^T:  re -= ar br - ai bi,  im -= ar bi + ai br
  tr = __builtin_amdgcn_mfma_f64_16x16x4f64(-rt.x, fr, tr, 0, 0, 0);
  ti = __builtin_amdgcn_mfma_f64_16x16x4f64(-rt.x, fi, ti, 0, 0, 0);
  tr = __builtin_amdgcn_mfma_f64_16x16x4f64(rt.y, fi, tr, 0, 0, 0);
  ti = __builtin_amdgcn_mfma_f64_16x16x4f64(-rt.y, fr, ti, 0, 0, 0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // S is rewritten by the next panel
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NR>
__device__ __forceinline__ double inv16_panel(double2 (&a)[4], double2* S) {
  d4 tr, ti;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    tr[jj] = a[jj].x;
    ti[jj] = a[jj].y;
  }
  double pp = 1.0;
  panel<0, NR>(tr, ti, S, pp);
  panel<1, NR>(tr, ti, S, pp);
  panel<2, NR>(tr, ti, S, pp);
  panel<3, NR>(tr, ti, S, pp);
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) a[jj] = make_double2(tr[jj], ti[jj]);
  return pp;
}

template <int V>
__device__ __forceinline__ double inv16(double2 (&a)[4], double2* S) {
  if constexpr (V == 0) {
    return wave_inv16_dpp<true>(a);
  } else if constexpr (V == 3) {
    return inv16_panel<2>(a, S);
  } else if constexpr (V == 4) {
    double pp = 1.0;
    la_fused_all(a, pp, std::make_integer_sequence<int, 16>{});
    return pp;
  } else {
    double pp = 1.0;
    la_all<V == 2 ? 1 : 2>(a, pp, std::make_integer_sequence<int, 16>{});
    return pp;
  }
}

template <int V>
__global__ __launch_bounds__(64) void k_var(const double2* in, double2* out, double* pm, long long* cyc, int rep) {
  double2 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = in[(blockIdx.x * 4 + j) * 64 + threadIdx.x];
  __shared__ double2 S[64];
  double pp = 1.0;
  __builtin_amdgcn_s_waitcnt(0);
  const long long t0 = clock64();
  for (int it = 0; it < rep; ++it) pp *= inv16<V>(a, S);
  const long long t1 = clock64();
#pragma unroll
  for (int j = 0; j < 4; ++j) out[(blockIdx.x * 4 + j) * 64 + threadIdx.x] = a[j];
  if (threadIdx.x == 0) {
    cyc[blockIdx.x] = t1 - t0;
    pm[blockIdx.x] = pp;
  }
}

struct Res {
  double cyc_per_pivot, ns_per_pivot;
  std::vector<double2> out;
  std::vector<double> pm;
};

template <int V>
Res run(const double2* in, double2* out, double* pm, long long* cyc, int nblk, int rep) {
  hipLaunchKernelGGL(k_var<V>, dim3(nblk), dim3(64), 0, 0, in, out, pm, cyc, rep);   // warm
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_var<V>, dim3(nblk), dim3(64), 0, 0, in, out, pm, cyc, rep);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(nblk);
  hipMemcpy(c.data(), cyc, nblk * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (long long x : c) m += (double)x;
  m /= nblk;
  Res r{m / (16.0 * rep), ms * 1e6 / (16.0 * rep), {}, {}};
  // one inversion for the agreement check
  hipLaunchKernelGGL(k_var<V>, dim3(nblk), dim3(64), 0, 0, in, out, pm, cyc, 1);
  r.out.resize((size_t)nblk * 4 * 64);
  r.pm.resize(nblk);
  hipMemcpy(r.out.data(), out, r.out.size() * 16, hipMemcpyDeviceToHost);
  hipMemcpy(r.pm.data(), pm, nblk * 8, hipMemcpyDeviceToHost);
  return r;
}

int main() {
  const int nblk = 240, rep = 256;
  // well-conditioned tiles like the CR pivots: (h - i y) with |h| ~ 1, y ~ 0.5
  std::vector<double2> h((size_t)nblk * 4 * 64);
  unsigned s = 12345;
  auto rnd = [&] {
    s = s * 1664525u + 1013904223u;
    return (double)(s >> 8) / (double)(1u << 24) - 0.5;
  };
  for (int b = 0; b < nblk; ++b)
    for (int j = 0; j < 4; ++j)
      for (int l = 0; l < 64; ++l) {
        const int r = l & 15, c = (l >> 4) + 4 * j;   // strided layout
        double2 v = make_double2(0.3 * rnd(), 0.3 * rnd());
        if (r == c) v = make_double2(v.x + 2.0, v.y - 0.5);
        h[((size_t)b * 4 + j) * 64 + l] = v;
      }
  double2 *in, *out;
  double* pm;
  long long* cyc;
  hipMalloc(&in, h.size() * 16);
  hipMalloc(&out, h.size() * 16);
  hipMalloc(&pm, nblk * 8);
  hipMalloc(&cyc, nblk * 8);
  hipMemcpy(in, h.data(), h.size() * 16, hipMemcpyHostToDevice);
  Res r0 = run<0>(in, out, pm, cyc, nblk, rep);
  Res r1 = run<1>(in, out, pm, cyc, nblk, rep);
  Res r2 = run<2>(in, out, pm, cyc, nblk, rep);
  Res r3 = run<3>(in, out, pm, cyc, nblk, rep);
  Res r4 = run<4>(in, out, pm, cyc, nblk, rep);
  Res* rs[5] = {&r0, &r1, &r2, &r3, &r4};
  for (int v = 0; v < 5; ++v) {
    double d = 0, mx = 0, dp = 0;
    bool same = true;
    for (size_t i = 0; i < r0.out.size(); ++i) {
      const double2 x = rs[v]->out[i], y = r0.out[i];
      d = std::fmax(d, std::fmax(std::fabs(x.x - y.x), std::fabs(x.y - y.y)));
      mx = std::fmax(mx, std::fmax(std::fabs(y.x), std::fabs(y.y)));
      same = same && x.x == y.x && x.y == y.y;
    }
    for (int b = 0; b < nblk; ++b) dp = std::fmax(dp, std::fabs(rs[v]->pm[b] / r0.pm[b] - 1.0));
    printf("V=%d  cycles per pivot %.1f  wall ns per pivot %.1f  max|inv - inv_V0| %.2e (max|inv| %.2e)%s  "
           "pivot product rel %.1e\n",
           v, rs[v]->cyc_per_pivot, rs[v]->ns_per_pivot, d, mx, same ? " bitwise equal" : "", dp);
  }
  return 0;
}
