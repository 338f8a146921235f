// Sparse level-0 stages of the block cyclic reduction (round 5).
//
// The level-0 off-diagonal blocks U[y] = A[y, y+1] and L[y] = A[y+1, y] of
// A = H_BdG - i y_q couple neighbouring lattice rows only through the vertical
// hopping (-t at x, -t' at x ± 1: src/Hamiltonian.jl:26-43) and the vertical
// pairing entry Δ/2 (src/Hamiltonian.jl:68-83): at most 4 nonzeros in every
// row and column of the BP x BP block.  Level 0 is the largest level of the
// recursion, and every product there that has a U or L factor is a sparse one,
// so the level-0 forward pass after the inversions and the sparse half of the
// backward pass run here on the vector units, with no dense V1, V2, W1, W2
// (tools/cr_model.py cr_selected_inverse_top_sparse0 states the algebra and
// checks it against dense inverses):
//
//   forward (k_cr_sp_fwd, per kept row k, er = k+1, el = k-1):
//     V1r = -U_k Dinv_er,  V2r = -L_er Dinv_er,  V2l = -L_el Dinv_el   (one row at a time, in LDS)
//     D'_k = D_k + V1r L_k + V2l U_el,  U'_k = V1r U_er,  L'_k = V2r L_k
//   backward (k_cr_sp_bwd, per eliminated row e, a = e-1, c = e+1):
//     Z_a = G_aa U_a + G_ac L_e,  Z_c = G_ca U_a + G_cc L_e     (dense . sparse)
//     Y_a = L_a G_aa + U_e G_ca,  Y_c = L_a G_ac + U_e G_cc     (sparse . dense)
//     M   = L_a Z_a + U_e Z_c = Y_a U_a + Y_c L_e               (dense . sparse, Y rows in LDS)
//   after which one-term dense products (k_cr_gemm) finish the level:
//     G_ae = -Z_a Dinv, G_ce = -Z_c Dinv, G_ea = -Dinv Y_a, G_ec = -Dinv Y_c,
//     T = -Dinv M, then G_ee = Dinv - T Dinv.
//
// Blocks are top halves (HP x BP) of M-form [[A, B], [conj B, -conj A]] or
// Q-form [[A, B], [-conj B, conj A]] blocks (dwhmc_cr.hip); the sparse
// operands are read through per-block patterns of the FULL BP x BP matrix
// (rows and columns, kCrSpNZ entries each, built on the host from the hopping
// and pairing tables exactly as k_cr_fill writes the blocks): entry = offset
// of the stored top-half element | (column or row index) << 14 | op << 22,
// op 0: the element, 1: its conjugate, 2: minus its conjugate (the
// synthesised bottom half), 3: empty (reads element 0, weight zero, so every
// load is unconditional and issued up front).  Pattern layout
// [block][entry][BP] (lanes over the last index read contiguous words).
// One wave per output row: every row of every output depends only on rows of
// the inputs, and the backward M = L_a Z_a + U_e Z_c is formed as
// Y_a U_a + Y_c L_e (the same sum regrouped), from the wave's own Y rows.
#include "dwhmc_device.h"
#include "dwhmc_internal.h"

namespace dwh {
namespace {

// stored value of pattern entry e (op 3: zero), times -1 when NEG, for a
// wave-uniform entry: the op's signs and the zeroing act on the bit patterns
// (scalar ALU; the value comes through a scalar load)
template <bool NEG = false>
__device__ __forceinline__ double2 sp_sval(const double2* __restrict__ S, int e) {
  constexpr unsigned long long SB = 1ull << 63, N = NEG ? SB : 0ull;
  const int off = e & 0x3fff, op = (e >> 22) & 3;
  const double2 v = S[off];
  const unsigned long long keep = op == 3 ? 0ull : ~0ull;
  const unsigned long long bx = (__builtin_bit_cast(unsigned long long, v.x) ^ (op == 2 ? SB : 0ull) ^ N) & keep;
  const unsigned long long by = (__builtin_bit_cast(unsigned long long, v.y) ^ (op == 1 ? SB : 0ull) ^ N) & keep;
  return make_double2(__builtin_bit_cast(double, bx), __builtin_bit_cast(double, by));
}
__device__ __forceinline__ int sp_idx(int e) { return (e >> 14) & 0xff; }

// a += b c
__device__ __forceinline__ void cmac(double2& a, double2 b, double2 c) {
  a.x = fma(b.x, c.x, fma(-b.y, c.y, a.x));
  a.y = fma(b.x, c.y, fma(b.y, c.x, a.y));
}

__device__ __forceinline__ double sp_flip(double x, unsigned m) {
  return __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, x) ^ ((unsigned long long)m << 32));
}

// Column c of the full BP x BP M-form block whose top half X (row-major
// HP x BP) is stored, with its lane-constant parts precomputed: a row access
// is one select for the column and two sign-bit XORs.  Bottom row HP + k,
// column c: conj(X[k, c + HP]) (c < HP) or -conj(X[k, c - HP]) (c >= HP).
template <int BP>
struct FullCol {
  int c, crot;
  unsigned mx, my;   // sign-bit masks of a synthesised entry's real / imaginary part
  __device__ __forceinline__ explicit FullCol(int col) : c(col) {
    constexpr int HP = BP / 2;
    crot = c < HP ? c + HP : c - HP;
    mx = c >= HP ? 0x80000000u : 0u;
    my = c < HP ? 0x80000000u : 0u;
  }
  // element (kk, c), kk wave-uniform
  __device__ __forceinline__ double2 at(const double2* __restrict__ X, int kk) const {
    constexpr int HP = BP / 2;
    const bool top = kk < HP;
    const double2 u = X[(top ? kk : kk - HP) * BP + (top ? c : crot)];
    return make_double2(sp_flip(u.x, top ? 0u : mx), sp_flip(u.y, top ? 0u : my));
  }
};

// column entry: a static hopping value (v, op applied) or, for a pairing
// entry, op(Δ[src] / 2) (the value k_cr_fill keeps in the pool) — never both;
// meta word m: src + 1 (0: none) in bits 0-21, op in 22-23 (1 conj,
// 2 -conj), row in 24-31.  x: the entry's one load (tcv or Δ).
__device__ __forceinline__ double2 sp_cval(double2 x, int m) {
  if ((m & 0x3fffff) == 0) return x;
  const int op = (m >> 22) & 3;
  return make_double2(op == 2 ? -0.5 * x.x : 0.5 * x.x, op == 0 ? 0.5 * x.y : -0.5 * x.y);   // op 1: conj, 2: -conj
}

constexpr int kSpRowsWG = 4;   // one output row per wave, four waves per workgroup
constexpr int NZ = kCrSpNZ;
// waves per SIMD the register budget is sized for at BP <= 64 (forward,
// backward): six (<= 80 VGPRs, 79 used) and five (<= 96), the most without
// scratch spills, so the C3 forward stage (1536 workgroups of 25 KB LDS) is
// resident in one round (-DSP_WAVES_F / -DSP_WAVES_B for A/B builds)
#ifndef SP_WAVES_F
#define SP_WAVES_F 6
#endif
#ifndef SP_WAVES_B
#define SP_WAVES_B 5
#endif
template <int BP>
constexpr int kSpWavesF = BP <= 64 ? SP_WAVES_F : 2;
template <int BP>
constexpr int kSpWavesB = BP <= 64 ? SP_WAVES_B : 2;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Column data of the sparse right operands (dense . sparse products): every
// output row of a workgroup uses the same column patterns, so the workgroup
// stages them once in LDS — the value and the row index of each entry — from
// the task's own column arrays (tcm / tcv: [NB][kCrSpNZ][BP], coalesced, no
// dependence on the task descriptor), one load per entry behind the meta word.
template <int BP, int NB>
__device__ __forceinline__ void stage_columns(double2 (*cv)[kCrSpNZ][BP], unsigned char (*ci)[kCrSpNZ][BP],
                                              const double2* __restrict__ tcv, const int* __restrict__ tcm,
                                              const double2* __restrict__ Dc) {
  constexpr int TOT = NB * NZ * BP, IT = (TOT + 64 * kSpRowsWG - 1) / (64 * kSpRowsWG);
  int m[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) m[i] = tcm[min((int)threadIdx.x + 64 * kSpRowsWG * i, TOT - 1)];
  double2 x[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {   // one load per entry: the static value or Δ
    const int q = min((int)threadIdx.x + 64 * kSpRowsWG * i, TOT - 1), s = m[i] & 0x3fffff;
    x[i] = *(s ? Dc + (s - 1) : tcv + q);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int q = threadIdx.x + 64 * kSpRowsWG * i;
    if (q < TOT) {
      (&cv[0][0][0])[q] = sp_cval(x[i], m[i]);
      (&ci[0][0][0])[q] = (unsigned char)((unsigned)m[i] >> 24);
    }
  }
}

// forward: one wave per output row r of the kept row k's D', U', L'; the
// row's operands are loaded into registers up front (pattern words through
// lanes, then every value and dense element at once), the V rows meet in LDS.
template <int BP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kSpWavesF<BP>))) void k_cr_sp_fwd(double2* __restrict__ pool, int64_t item,
                                                   const CrSpFwd* __restrict__ tasks, const int* __restrict__ trow,
                                                   const double2* __restrict__ tcv, const int* __restrict__ tcm,
                                                   const double2* __restrict__ Delta, int twoN, int P, int nrb) {
  constexpr int HP = BP / 2, NCL = (BP + 63) / 64;
  constexpr int64_t BB = (int64_t)HP * BP;
  constexpr int TA = 3 * NZ * BP, TR = 3 * NZ * HP;   // per-task column / row array sizes
  __shared__ double2 cv[3][NZ][BP];
  __shared__ unsigned char ci[3][NZ][BP];
  __shared__ double2 sc[kSpRowsWG][3][BP];
  const double2* Dc = Delta + (int64_t)(__builtin_amdgcn_readfirstlane(xcd_grid2d().y) / P) * twoN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int2 xy = xcd_grid2d();   // batch items grouped per XCD
  const int ti = __builtin_amdgcn_readfirstlane(xy.x / nrb);
  const int r = __builtin_amdgcn_readfirstlane((xy.x - ti * nrb) * kSpRowsWG + w);
  const CrSpFwd t = tasks[ti];
  double2* base = pool + (int64_t)xy.y * item;
  const double2 *Dir = base + t.dir * BB, *Dil = base + t.dil * BB, *Dk = base + t.dk * BB;
  int cl[NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) cl[j] = min(l + 64 * j, BP - 1);
  // row r of U_k, L_er, L_el: pattern words and values are wave-uniform
  // (scalar loads), negated here so the V rows come out with their sign
  const int* rw = trow + (int64_t)ti * TR + r * 3 * NZ;
  int pu[NZ], pr[NZ], pl[NZ];
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    pu[e] = rw[e];
    pr[e] = rw[NZ + e];
    pl[e] = rw[2 * NZ + e];
  }
  double2 wu[NZ], wr[NZ], wl[NZ];
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    wu[e] = sp_sval<true>(base + t.uk * BB, pu[e]);
    wr[e] = sp_sval<true>(base + t.ler * BB, pr[e]);
    wl[e] = sp_sval<true>(base + t.lel * BB, pl[e]);
  }
  double2 dk[NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) dk[j] = Dk[r * BP + cl[j]];
  double2 xu[NZ][NCL], xr[NZ][NCL], xl[NZ][NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const FullCol<BP> fc(cl[j]);
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      xu[e][j] = fc.at(Dir, sp_idx(pu[e]));
      xr[e][j] = fc.at(Dir, sp_idx(pr[e]));
      xl[e][j] = fc.at(Dil, sp_idx(pl[e]));
    }
  }
  stage_columns<BP, 3>(cv, ci, tcv + (int64_t)ti * TA, tcm + (int64_t)ti * TA, Dc);
  // V1r = -U_k Dinv_er, V2r = -L_er Dinv_er, V2l = -L_el Dinv_el
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    double2 v1 = make_double2(0.0, 0.0), v2r = v1, v2l = v1;
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      cmac(v1, wu[e], xu[e][j]);
      cmac(v2r, wr[e], xr[e][j]);
      cmac(v2l, wl[e], xl[e][j]);
    }
    if (l + 64 * j < BP) {
      sc[w][0][cl[j]] = v1;
      sc[w][1][cl[j]] = v2r;
      sc[w][2][cl[j]] = v2l;
    }
  }
  __syncthreads();
  // D'_k = D_k + V1r L_k + V2l U_el, U'_k = V1r U_er, L'_k = V2r L_k
  double2 *On = base + t.od * BB, *Ou = base + t.ou * BB, *Ol = base + t.ol * BB;
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = cl[j];
    double2 d = dk[j], u = make_double2(0.0, 0.0), lo = make_double2(0.0, 0.0);
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      const double2 vl = cv[0][e][c], vu = cv[1][e][c], vr = cv[2][e][c];
      const int kl = ci[0][e][c], ku = ci[1][e][c], kr = ci[2][e][c];
      cmac(d, sc[w][0][kl], vl);
      cmac(lo, sc[w][1][kl], vl);
      cmac(d, sc[w][2][ku], vu);
      cmac(u, sc[w][0][kr], vr);
    }
    if (l + 64 * j < BP) {
      On[r * BP + c] = d;
      Ou[r * BP + c] = u;
      Ol[r * BP + c] = lo;
    }
  }
}

// backward: one wave per output row r of the eliminated row e's Z_a, Z_c,
// Y_a, Y_c and M = Y_a U_a + Y_c L_e.  Row r of each G block is staged in the
// wave's LDS (Z gathers from it), full rows of the G blocks feed Y.
template <int BP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kSpWavesB<BP>))) void k_cr_sp_bwd(double2* __restrict__ pool, int64_t item,
                                                   const CrSpBwd* __restrict__ tasks, const int* __restrict__ trow,
                                                   const double2* __restrict__ tcv, const int* __restrict__ tcm,
                                                   const double2* __restrict__ Delta, int twoN, int P, int nrb) {
  constexpr int HP = BP / 2, NCL = (BP + 63) / 64;
  constexpr int64_t BB = (int64_t)HP * BP;
  constexpr int TA = 2 * NZ * BP, TR = 2 * NZ * HP;   // per-task column / row array sizes
  __shared__ double2 cv[2][NZ][BP];
  __shared__ unsigned char ci[2][NZ][BP];
  __shared__ double2 gr[kSpRowsWG][4][BP];
  double2(*sc)[4][BP] = gr;   // the Y rows (sc[w][0 / 1]) reuse the wave's G rows once Z is formed
  const double2* Dc = Delta + (int64_t)(__builtin_amdgcn_readfirstlane(xcd_grid2d().y) / P) * twoN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int2 xy = xcd_grid2d();   // batch items grouped per XCD
  const int ti = __builtin_amdgcn_readfirstlane(xy.x / nrb);
  const int r = __builtin_amdgcn_readfirstlane((xy.x - ti * nrb) * kSpRowsWG + w);
  const CrSpBwd t = tasks[ti];
  double2* base = pool + (int64_t)xy.y * item;
  const double2 *Gaa = base + t.gaa * BB, *Gac = base + t.gac * BB, *Gca = base + t.gca * BB,
                *Gcc = base + t.gcc * BB;
  int cl[NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) cl[j] = min(l + 64 * j, BP - 1);
  // row r of L_a, U_e: wave-uniform pattern words and values (scalar loads)
  const int* rw = trow + (int64_t)ti * TR + r * 2 * NZ;
  int pa[NZ], pe[NZ];
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    pa[e] = rw[e];
    pe[e] = rw[NZ + e];
  }
  double2 va[NZ], ve[NZ];
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    va[e] = sp_sval(base + t.la * BB, pa[e]);
    ve[e] = sp_sval(base + t.ue * BB, pe[e]);
  }
  // rows r of the G blocks (for Z) into this wave's LDS
#pragma unroll
  for (int j = 0; j < NCL; ++j)
    if (l + 64 * j < BP) {
      gr[w][0][cl[j]] = Gaa[r * BP + cl[j]];
      gr[w][1][cl[j]] = Gca[r * BP + cl[j]];
      gr[w][2][cl[j]] = Gac[r * BP + cl[j]];
      gr[w][3][cl[j]] = Gcc[r * BP + cl[j]];
    }
  double2 gaa[NZ][NCL], gac[NZ][NCL], gca[NZ][NCL], gcc[NZ][NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const FullCol<BP> fc(cl[j]);
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      gaa[e][j] = fc.at(Gaa, sp_idx(pa[e]));
      gac[e][j] = fc.at(Gac, sp_idx(pa[e]));
      gca[e][j] = fc.at(Gca, sp_idx(pe[e]));
      gcc[e][j] = fc.at(Gcc, sp_idx(pe[e]));
    }
  }
  stage_columns<BP, 2>(cv, ci, tcv + (int64_t)ti * TA, tcm + (int64_t)ti * TA, Dc);
  __syncthreads();
  double2 *Oza = base + t.oza * BB, *Ozc = base + t.ozc * BB, *Oya = base + t.oya * BB,
          *Oyc = base + t.oyc * BB, *Omx = base + t.omx * BB;
  double2 yk[NCL][2];
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = cl[j];
    // Y_a[r, :] = L_a[r, :] G_aa + U_e[r, :] G_ca, Y_c[r, :] = L_a[r, :] G_ac + U_e[r, :] G_cc
    // Z_a[r, :] = G_aa[r, :] U_a + G_ac[r, :] L_e, Z_c[r, :] = G_ca[r, :] U_a + G_cc[r, :] L_e
    double2 ya = make_double2(0.0, 0.0), yc = ya, za = ya, zc = ya;
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      cmac(ya, va[e], gaa[e][j]);
      cmac(yc, va[e], gac[e][j]);
      cmac(ya, ve[e], gca[e][j]);
      cmac(yc, ve[e], gcc[e][j]);
      const double2 wa = cv[0][e][c], we = cv[1][e][c];
      const int ka = ci[0][e][c], ke = ci[1][e][c];
      cmac(za, gr[w][0][ka], wa);
      cmac(zc, gr[w][1][ka], wa);
      cmac(za, gr[w][2][ke], we);
      cmac(zc, gr[w][3][ke], we);
    }
    if (l + 64 * j < BP) {
      Oya[r * BP + c] = ya;
      Oyc[r * BP + c] = yc;
      Oza[r * BP + c] = za;
      Ozc[r * BP + c] = zc;
    }
    yk[j][0] = ya;
    yk[j][1] = yc;
  }
  wave_sync();   // every lane's Z gathers from gr[w] are done
#pragma unroll
  for (int j = 0; j < NCL; ++j)
    if (l + 64 * j < BP) {
      sc[w][0][cl[j]] = yk[j][0];
      sc[w][1][cl[j]] = yk[j][1];
    }
  wave_sync();
  // M[r, :] = Y_a[r, :] U_a + Y_c[r, :] L_e
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = cl[j];
    double2 mx = make_double2(0.0, 0.0);
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      cmac(mx, sc[w][0][ci[0][e][c]], cv[0][e][c]);
      cmac(mx, sc[w][1][ci[1][e][c]], cv[1][e][c]);
    }
    if (l + 64 * j < BP) Omx[r * BP + c] = mx;
  }
}

}  // namespace

bool cr_supported_sparse0(int BP) { return BP == 32 || BP == 64 || BP == 96; }

void launch_cr_sp_fwd(const CrDims& c, double2* pool, const CrSpFwd* tasks, int n, const int* trow,
                      const double2* tcv, const int* tcm, const double2* Delta, hipStream_t s) {
  if (n <= 0) return;
  const int nrb = c.BP / 2 / kSpRowsWG;
  const dim3 g(n * nrb, c.nbatch), b(64 * kSpRowsWG);
  switch (c.BP) {
    case 32: hipLaunchKernelGGL(k_cr_sp_fwd<32>, g, b, 0, s, pool, c.item, tasks, trow, tcv, tcm, Delta, 2 * c.N, c.P, nrb); break;
    case 64: hipLaunchKernelGGL(k_cr_sp_fwd<64>, g, b, 0, s, pool, c.item, tasks, trow, tcv, tcm, Delta, 2 * c.N, c.P, nrb); break;
    default: hipLaunchKernelGGL(k_cr_sp_fwd<96>, g, b, 0, s, pool, c.item, tasks, trow, tcv, tcm, Delta, 2 * c.N, c.P, nrb); break;
  }
}

void launch_cr_sp_bwd(const CrDims& c, double2* pool, const CrSpBwd* tasks, int n, const int* trow,
                      const double2* tcv, const int* tcm, const double2* Delta, hipStream_t s) {
  if (n <= 0) return;
  const int nrb = c.BP / 2 / kSpRowsWG;
  const dim3 g(n * nrb, c.nbatch), b(64 * kSpRowsWG);
  switch (c.BP) {
    case 32: hipLaunchKernelGGL(k_cr_sp_bwd<32>, g, b, 0, s, pool, c.item, tasks, trow, tcv, tcm, Delta, 2 * c.N, c.P, nrb); break;
    case 64: hipLaunchKernelGGL(k_cr_sp_bwd<64>, g, b, 0, s, pool, c.item, tasks, trow, tcv, tcm, Delta, 2 * c.N, c.P, nrb); break;
    default: hipLaunchKernelGGL(k_cr_sp_bwd<96>, g, b, 0, s, pool, c.item, tasks, trow, tcv, tcm, Delta, 2 * c.N, c.P, nrb); break;
  }
}

}  // namespace dwh
