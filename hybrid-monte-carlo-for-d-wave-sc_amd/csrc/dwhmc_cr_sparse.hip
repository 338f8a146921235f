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

// stored value of pattern entry e (op 3: zero)
__device__ __forceinline__ double2 sp_val(const double2* __restrict__ S, int e) {
  const int off = e & 0x3fff, op = (e >> 22) & 3;
  const double2 v = S[off];
  const double sr = op == 2 ? -1.0 : (op == 3 ? 0.0 : 1.0);
  const double si = op == 1 ? -1.0 : (op == 3 ? 0.0 : 1.0);
  return make_double2(sr * v.x, si * v.y);
}
__device__ __forceinline__ int sp_idx(int e) { return (e >> 14) & 0xff; }

// a += b c
__device__ __forceinline__ void cmac(double2& a, double2 b, double2 c) {
  a.x = fma(b.x, c.x, fma(-b.y, c.y, a.x));
  a.y = fma(b.x, c.y, fma(b.y, c.x, a.y));
}

// element (kk, c) of the full block whose top half is X (row-major HP x BP),
// form s = -1 (M) / +1 (Q): bottom rows synthesised from the top half
template <int BP>
__device__ __forceinline__ double2 full_at(const double2* __restrict__ X, double s, int kk, int c) {
  constexpr int HP = BP / 2;
  const bool top = kk < HP;
  const int cc = top ? c : (c < HP ? c + HP : c - HP);
  const double2 u = X[(top ? kk : kk - HP) * BP + cc];
  const double sg = top ? 1.0 : (c < HP ? -s : s);
  return top ? u : make_double2(sg * u.x, -sg * u.y);
}

constexpr int kSpRowsWG = 4;   // one output row per wave, four waves per workgroup
constexpr int NZ = kCrSpNZ;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// forward: one wave per output row r of the kept row k's D', U', L'
template <int BP>
__global__ __launch_bounds__(256) void k_cr_sp_fwd(double2* __restrict__ pool, int64_t item,
                                                   const CrSpFwd* __restrict__ tasks, const int* __restrict__ rowpat,
                                                   const int* __restrict__ colpat, int nrb) {
  constexpr int HP = BP / 2, NCL = (BP + 63) / 64;
  constexpr int64_t BB = (int64_t)HP * BP;
  __shared__ double2 sc[kSpRowsWG][3][BP];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int ti = __builtin_amdgcn_readfirstlane(blockIdx.x / nrb);
  const int r = __builtin_amdgcn_readfirstlane((blockIdx.x - ti * nrb) * kSpRowsWG + w);
  const CrSpFwd* t = tasks + ti;
  double2* base = pool + (int64_t)blockIdx.y * item;
  const double2 *Dir = base + t->dir * BB, *Dil = base + t->dil * BB;
  const double2 *Uk = base + t->uk * BB, *Ler = base + t->ler * BB, *Lel = base + t->lel * BB;
  const double2 *Lk = base + t->lk * BB, *Uel = base + t->uel * BB, *Uer = base + t->uer * BB;
  const double2* Dk = base + t->dk * BB;
  // row r of U_k, L_er, L_el (uniform) and the column patterns of this lane's
  // columns of L_k, U_el, U_er: every pattern load first, then every value
  int pu[NZ], pr[NZ], pl[NZ], ql[NCL][NZ], qu[NCL][NZ], qr[NCL][NZ];
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    pu[e] = rowpat[(t->uk * NZ + e) * BP + r];
    pr[e] = rowpat[(t->ler * NZ + e) * BP + r];
    pl[e] = rowpat[(t->lel * NZ + e) * BP + r];
#pragma unroll
    for (int j = 0; j < NCL; ++j) {
      const int c = min(l + 64 * j, BP - 1);
      ql[j][e] = colpat[(t->lk * NZ + e) * BP + c];
      qu[j][e] = colpat[(t->uel * NZ + e) * BP + c];
      qr[j][e] = colpat[(t->uer * NZ + e) * BP + c];
    }
  }
  double2 v1[NCL], v2r[NCL], v2l[NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) v1[j] = v2r[j] = v2l[j] = make_double2(0.0, 0.0);
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    const double2 vu = sp_val(Uk, pu[e]), vr = sp_val(Ler, pr[e]), vl = sp_val(Lel, pl[e]);
#pragma unroll
    for (int j = 0; j < NCL; ++j) {
      const int c = min(l + 64 * j, BP - 1);
      cmac(v1[j], vu, full_at<BP>(Dir, -1.0, sp_idx(pu[e]), c));
      cmac(v2r[j], vr, full_at<BP>(Dir, -1.0, sp_idx(pr[e]), c));
      cmac(v2l[j], vl, full_at<BP>(Dil, -1.0, sp_idx(pl[e]), c));
    }
  }
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = l + 64 * j;
    if (c >= BP) continue;
    sc[w][0][c] = make_double2(-v1[j].x, -v1[j].y);   // V1r = -U_k Dinv_er
    sc[w][1][c] = make_double2(-v2r[j].x, -v2r[j].y);  // V2r = -L_er Dinv_er
    sc[w][2][c] = make_double2(-v2l[j].x, -v2l[j].y);  // V2l = -L_el Dinv_el
  }
  wave_sync();
  double2 *On = base + t->od * BB, *Ou = base + t->ou * BB, *Ol = base + t->ol * BB;
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = l + 64 * j;
    if (c >= BP) continue;
    double2 d = Dk[r * BP + c], u = make_double2(0.0, 0.0), lo = make_double2(0.0, 0.0);
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      const double2 vl = sp_val(Lk, ql[j][e]), vu = sp_val(Uel, qu[j][e]), vr = sp_val(Uer, qr[j][e]);
      cmac(d, sc[w][0][sp_idx(ql[j][e])], vl);    // V1r L_k
      cmac(lo, sc[w][1][sp_idx(ql[j][e])], vl);   // V2r L_k
      cmac(d, sc[w][2][sp_idx(qu[j][e])], vu);    // V2l U_el
      cmac(u, sc[w][0][sp_idx(qr[j][e])], vr);    // V1r U_er
    }
    On[r * BP + c] = d;
    Ou[r * BP + c] = u;
    Ol[r * BP + c] = lo;
  }
}

// backward: one wave per output row r of the eliminated row e's Z_a, Z_c,
// Y_a, Y_c and M = Y_a U_a + Y_c L_e
template <int BP>
__global__ __launch_bounds__(256) void k_cr_sp_bwd(double2* __restrict__ pool, int64_t item,
                                                   const CrSpBwd* __restrict__ tasks, const int* __restrict__ rowpat,
                                                   const int* __restrict__ colpat, int nrb) {
  constexpr int HP = BP / 2, NCL = (BP + 63) / 64;
  constexpr int64_t BB = (int64_t)HP * BP;
  __shared__ double2 sc[kSpRowsWG][2][BP];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int ti = __builtin_amdgcn_readfirstlane(blockIdx.x / nrb);
  const int r = __builtin_amdgcn_readfirstlane((blockIdx.x - ti * nrb) * kSpRowsWG + w);
  const CrSpBwd* t = tasks + ti;
  double2* base = pool + (int64_t)blockIdx.y * item;
  const double2 *Gaa = base + t->gaa * BB, *Gac = base + t->gac * BB, *Gca = base + t->gca * BB,
                *Gcc = base + t->gcc * BB;
  const double2 *Ua = base + t->ua * BB, *Le = base + t->le * BB, *La = base + t->la * BB, *Ue = base + t->ue * BB;
  int pa[NZ], pe[NZ], qa[NCL][NZ], qe[NCL][NZ];
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    pa[e] = rowpat[(t->la * NZ + e) * BP + r];
    pe[e] = rowpat[(t->ue * NZ + e) * BP + r];
#pragma unroll
    for (int j = 0; j < NCL; ++j) {
      const int c = min(l + 64 * j, BP - 1);
      qa[j][e] = colpat[(t->ua * NZ + e) * BP + c];
      qe[j][e] = colpat[(t->le * NZ + e) * BP + c];
    }
  }
  // Y_a[r, :] = L_a[r, :] G_aa + U_e[r, :] G_ca, Y_c[r, :] = L_a[r, :] G_ac + U_e[r, :] G_cc
  double2 ya[NCL], yc[NCL], za[NCL], zc[NCL];
#pragma unroll
  for (int j = 0; j < NCL; ++j) ya[j] = yc[j] = za[j] = zc[j] = make_double2(0.0, 0.0);
#pragma unroll
  for (int e = 0; e < NZ; ++e) {
    const double2 va = sp_val(La, pa[e]), ve = sp_val(Ue, pe[e]);
#pragma unroll
    for (int j = 0; j < NCL; ++j) {
      const int c = min(l + 64 * j, BP - 1);
      cmac(ya[j], va, full_at<BP>(Gaa, -1.0, sp_idx(pa[e]), c));
      cmac(yc[j], va, full_at<BP>(Gac, -1.0, sp_idx(pa[e]), c));
      cmac(ya[j], ve, full_at<BP>(Gca, -1.0, sp_idx(pe[e]), c));
      cmac(yc[j], ve, full_at<BP>(Gcc, -1.0, sp_idx(pe[e]), c));
    }
  }
  // Z_a[r, :] = G_aa[r, :] U_a + G_ac[r, :] L_e, Z_c[r, :] = G_ca[r, :] U_a + G_cc[r, :] L_e
#pragma unroll
  for (int j = 0; j < NCL; ++j)
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      const double2 vua = sp_val(Ua, qa[j][e]), vle = sp_val(Le, qe[j][e]);
      const int ka = sp_idx(qa[j][e]), ke = sp_idx(qe[j][e]);
      cmac(za[j], Gaa[r * BP + ka], vua);
      cmac(zc[j], Gca[r * BP + ka], vua);
      cmac(za[j], Gac[r * BP + ke], vle);
      cmac(zc[j], Gcc[r * BP + ke], vle);
    }
  double2 *Oza = base + t->oza * BB, *Ozc = base + t->ozc * BB, *Oya = base + t->oya * BB,
          *Oyc = base + t->oyc * BB, *Omx = base + t->omx * BB;
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = l + 64 * j;
    if (c >= BP) continue;
    sc[w][0][c] = ya[j];
    sc[w][1][c] = yc[j];
    Oya[r * BP + c] = ya[j];
    Oyc[r * BP + c] = yc[j];
    Oza[r * BP + c] = za[j];
    Ozc[r * BP + c] = zc[j];
  }
  wave_sync();
  // M[r, :] = Y_a[r, :] U_a + Y_c[r, :] L_e
#pragma unroll
  for (int j = 0; j < NCL; ++j) {
    const int c = l + 64 * j;
    if (c >= BP) continue;
    double2 mx = make_double2(0.0, 0.0);
#pragma unroll
    for (int e = 0; e < NZ; ++e) {
      cmac(mx, sc[w][0][sp_idx(qa[j][e])], sp_val(Ua, qa[j][e]));
      cmac(mx, sc[w][1][sp_idx(qe[j][e])], sp_val(Le, qe[j][e]));
    }
    Omx[r * BP + c] = mx;
  }
}

}  // namespace

bool cr_supported_sparse0(int BP) { return BP == 32 || BP == 64 || BP == 96; }

void launch_cr_sp_fwd(const CrDims& c, double2* pool, const CrSpFwd* tasks, int n, const int* rowpat,
                      const int* colpat, hipStream_t s) {
  if (n <= 0) return;
  const int nrb = c.BP / 2 / kSpRowsWG;
  const dim3 g(n * nrb, c.nbatch), b(64 * kSpRowsWG);
  switch (c.BP) {
    case 32: hipLaunchKernelGGL(k_cr_sp_fwd<32>, g, b, 0, s, pool, c.item, tasks, rowpat, colpat, nrb); break;
    case 64: hipLaunchKernelGGL(k_cr_sp_fwd<64>, g, b, 0, s, pool, c.item, tasks, rowpat, colpat, nrb); break;
    default: hipLaunchKernelGGL(k_cr_sp_fwd<96>, g, b, 0, s, pool, c.item, tasks, rowpat, colpat, nrb); break;
  }
}

void launch_cr_sp_bwd(const CrDims& c, double2* pool, const CrSpBwd* tasks, int n, const int* rowpat,
                      const int* colpat, hipStream_t s) {
  if (n <= 0) return;
  const int nrb = c.BP / 2 / kSpRowsWG;
  const dim3 g(n * nrb, c.nbatch), b(64 * kSpRowsWG);
  switch (c.BP) {
    case 32: hipLaunchKernelGGL(k_cr_sp_bwd<32>, g, b, 0, s, pool, c.item, tasks, rowpat, colpat, nrb); break;
    case 64: hipLaunchKernelGGL(k_cr_sp_bwd<64>, g, b, 0, s, pool, c.item, tasks, rowpat, colpat, nrb); break;
    default: hipLaunchKernelGGL(k_cr_sp_bwd<96>, g, b, 0, s, pool, c.item, tasks, rowpat, colpat, nrb); break;
  }
}

}  // namespace dwh
