// Internal launch interface between the C-ABI context (dwhmc_api.cpp) and the
// gfx950 kernels (dwhmc_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace dwh {

constexpr int kGJ = 64;        // Gauss-Jordan block (rows/cols of one diagonal block)
constexpr int kSlots = 4;      // pairing entries per BdG row (NN bonds)
constexpr int kHSlots = 9;     // hopping entries per row (diag + 4 NN + 4 NNN)

struct Dims {
  int N;        // sites
  int Np;       // padded to kGJ
  int nb;       // Np / kGJ
  int nc;       // chains
  int P;        // poles per chain
  int nbatch;   // nc * P
  int64_t mat;  // elements per padded matrix (Np*Np)
  int nld;      // ln|det| partials per batch item (dense: nb pivot blocks; cr: Ly block inversions)
};

// after the force: π += kick·F, then (drift != 0) Δ += drift·π with the
// |Δ| <= cap guard setting *flag (the next leapfrog step's drift, fused)
struct KickDrift {
  double kick, drift, cap;
  int* flag;
};

// Block cyclic-reduction path (dwhmc_cr.hip): every batch item owns a pool of
// nblk blocks (level-0 D/U/L, Schur complements, products, G blocks), each the
// top half (HP x BP, BP = 2 HP, HP = Lx rounded up to 16) of a BP x BP block
// of particle-hole form (see dwhmc_cr.hip).
struct CrDims {
  int Lx, Ly, N, BP, P, nbatch, nblk;
  int64_t item;   // elements per batch item pool (nblk * HP * BP)
  int inv32 = 1;  // BP = 32 inversions by the one-wave Schur complement (k_cr_inv32; else k_cr_inv<2>)
};
// out = [cin] + sg * sum_{h<nt} A_h B_h over pool block indices (cin = -1: zero),
// computed only on the output rows [r0, r1) x columns [c0, c1) (rounded out to
// whole wave tiles; the rest of `out` is left untouched); bit h of bq: B_h is
// Q-form (else M-form)
struct CrTask {
  int out, cin, nt, bq;
  int a[4], b[4];
  int r0, r1, c0, c1;
};
// CrTask::bq bit of side-work tasks whose stage sign is negative (side-work
// task lists mix stages of both signs)
constexpr int kCrNegBit = 1 << 8;
// One 16 x 16 output tile of a product stage with its task's operands, so a
// workgroup reads its whole descriptor with one 64-byte scalar load (tr, tc:
// tile row / column in 16-tile units)
struct alignas(64) CrTile {
  int out, cin, nt, bq;
  int a[4], b[4];
  int tr, tc, neg, pad1;   // neg: 1 = negative sign
};
// One 16 x 16 output tile of ONE batch item of a product stage, stored in
// dispatch order (slot blockIdx.x * tiles-per-workgroup + tile: the host applies
// the XCD-aware remap and the batch-item split), with every operand resolved
// to an element offset: a wave reads its whole descriptor with one 64-byte
// scalar load and forms no block, batch-item or tile address itself.
// base: the batch item's first pool element; out / cin: the tile origin (row
// 16 tr, column 16 tc) of the output / accumulate input within the item
// (cin kCrNone: none; out kCrNone: an empty slot); a[h]: A_h at row 16 tr;
// b[h]: B_h at column 16 tc; rot: the column shift of the synthesised B rows'
// source ((c + HP) mod BP - c); bit h of smask: term h's synthesised rows carry
// a negative sign.
constexpr uint32_t kCrNone = 0xffffffffu;
struct alignas(64) CrSlot {
  uint64_t base;
  uint32_t out, cin;
  int nt;
  unsigned smask;
  uint32_t a[4], b[4];
  int rot, pad;
};
static_assert(sizeof(CrSlot) == 64 && offsetof(CrSlot, out) == 8 && offsetof(CrSlot, nt) == 16 &&
                  offsetof(CrSlot, a) == 24 && offsetof(CrSlot, b) == 40 && offsetof(CrSlot, rot) == 56,
              "k_cr_gemm16 reads a slot as 16 dwords in this order");
// wave tiles of a task at tile size ts
inline int cr_task_tiles(const CrTask& t, int ts) {
  return ((t.r1 + ts - 1) / ts - t.r0 / ts) * ((t.c1 + ts - 1) / ts - t.c0 / ts);
}
bool cr_supported_bp(int BP);
// diagnostic stamp builds (-DCR_STAMPS, dwh_debug_cr_stamps): workgroups recorded per launch
constexpr int kCrStampWG = 2048;
#ifdef CR_STAMPS
int cr_stamps_arm(int key);   // key >= 0: clears the stamps, records the launch whose first block is `key`; -1: off
int cr_stamps_read(unsigned long long* out, int nwg);
#endif
// level-0 blocks of `list` (ids t*Ly + y, t = 0 D / 1 U / 2 L) fully
// rewritten, plus (off_ph != nullptr) the pairing entries Δ[Dsrc]/2 of the
// level-0 blocks outside the list, in one launch
void launch_cr_fill(const CrDims& c, double2* pool, const int* list, int nlist, const int* hcol,
                    const double* hval, const int* Dcol, const int* Dsrc, const double2* Delta,
                    const double* ypole, const int64_t* off_ph, hipStream_t s);
// P from the level-0 G blocks (pole weights), F, kick / drift; per bond b,
// bond4[4 b ..] = pool offsets of G12[i, j], G12[j, i] and of the two
// pairing entries the bond writes (-1: none); with kd.drift != 0 the drifted
// Δ/2 is also scattered into those level-0 entries (k_cr_fill's scatter)
void launch_cr_pair_force(const CrDims& c, double2* pool, const int64_t* bond4, const double* cpole,
                          double2* Delta, double2* Pair, double2* F, double2* Pi,
                          const KickDrift& kd, double beta, double J, hipStream_t s);
// E_f and Tr ρ_hh from the CR block pivots and the G22 diagonal (pool offsets doff)
// part: 2 x nbatch scratch, done: nchains counters (zero at creation; the
// kernel leaves them zero)
void launch_cr_fermion_energy(const CrDims& c, const double2* pool, const int64_t* doff,
                              const double* ldpart, const double* cpole, double Cx, double beta,
                              double* part, unsigned* done, double* Ef, double* Trhh, hipStream_t s);
// inverts blocks blk[i] into dst[i] (dst == blk: in place); ln|det| into ldpart slots
// Site spectral guard, checked by one extra workgroup per chain of the level-0
// inversion launch: Σ of |Δ| over each site's 4 bonds (site4[4 i ..], indices
// into a chain's N x 2 Δ) <= cap4, else *flag = 1.  Delta == nullptr: off.
struct SiteGuard {
  const double2* Delta = nullptr;
  const int* site4 = nullptr;
  double cap4 = 0.0;
  int* flag = nullptr;
};
void launch_cr_inv(const CrDims& c, double2* pool, const int* blk, const int* dst, const int* slot,
                   int n, double* ldpart, hipStream_t s, const SiteGuard& sg = SiteGuard{});
// level-0 inversions of blocks blk[i] (BP = 32, 64, 96) from the static R = A^-1
// blocks rblk[i] (k_cr_inv0); ln|det| = ldA/2 + ln|det S| into ldpart slots
bool cr_supported_inv0(int BP);
// Delta != nullptr: one extra workgroup per chain checks the site guard
// (Σ of |Δ| over each site's 4 bonds site4[4 i ..] <= cap4, else *flag = 1)
void launch_cr_inv0(const CrDims& c, double2* pool, const int* blk, const int* rblk, const int* dst,
                    const int* slot, int n, double* ldpart, const double* ldA, hipStream_t s,
                    const double2* Delta = nullptr, const int* site4 = nullptr, double cap4 = 0.0,
                    int* flag = nullptr);
// the same inversions plus nst side-work product tasks per batch item
// (32 x 32 wave tiles, maxt32 per task, each task's sign in bq & kCrNegBit)
// on the CUs the inversions leave idle
bool cr_supported_side(int BP);
void launch_cr_inv_side(const CrDims& c, double2* pool, const int* blk, const int* dst, const int* slot,
                        int n, double* ldpart, const CrTask* stasks, int nst, int maxt32, hipStream_t s,
                        const SiteGuard& sg = SiteGuard{});
// Sparse level-0 stages (dwhmc_cr_sparse.hip): the level-0 U / L blocks have
// at most kCrSpNZ nonzeros per row and column (vertical hopping + one pairing
// entry); rowpat / colpat hold them per pool block ([block][entry][BP], entry
// = top-half offset | index << 14 | op << 22, op 3 empty; dwhmc_cr_sparse.hip)
constexpr int kCrSpNZ = 4;
bool cr_supported_sparse0(int BP);
// forward, per kept row k (er = k+1, el = k-1): D'_k = D_k + V1r L_k + V2l U_el,
// U'_k = V1r U_er, L'_k = V2r L_k with V1r = -U_k Dinv_er, V2r = -L_er Dinv_er,
// V2l = -L_el Dinv_el (pool block indices)
struct CrSpFwd {
  int dk, uk, lk, uel, lel, uer, ler, dir, dil, od, ou, ol;
};
// backward, per eliminated row e (a = e-1, c = e+1): Z_a = G_aa U_a + G_ac L_e,
// Z_c = G_ca U_a + G_cc L_e, Y_a = L_a G_aa + U_e G_ca, Y_c = L_a G_ac + U_e G_cc,
// M = L_a Z_a + U_e Z_c (= Y_a U_a + Y_c L_e, the form the kernel uses)
struct CrSpBwd {
  int gaa, gac, gca, gcc, ua, le, la, ue, oza, ozc, oya, oyc, omx, pad0, pad1, pad2;
};
// Per task (tasks[ti]), arrays of kCrSpNZ x BP entries for each of its sparse
// operands, so a workgroup reads its patterns without first reading the
// task: trow — the row-pattern words of the left sparse operands (forward:
// U_k, L_er, L_el; backward: L_a, U_e); tcv / tcm — the column entries of the
// right ones (forward: L_k, U_el, U_er; backward: U_a, L_e): static hopping
// value with op applied, and meta = (Δ index + 1, 0 none) | op << 22 |
// row << 24.  Delta: the chains' N x 2 Δ (batch item bi reads chain bi / P).
void launch_cr_sp_fwd(const CrDims& c, double2* pool, const CrSpFwd* tasks, int n, const int* trow,
                      const double2* tcv, const int* tcm, const double2* Delta, hipStream_t s);
void launch_cr_sp_bwd(const CrDims& c, double2* pool, const CrSpBwd* tasks, int n, const int* trow,
                      const double2* tcv, const int* tcm, const double2* Delta, hipStream_t s);
// block-product stage configuration: output tile TS x TS (16 or 32) and the
// number of waves splitting each tile's K range (1, 2, 4)
struct CrGemmCfg {
  int ts, ksplit;
};
// tile pairs of a stage (CrTile::pad1 = the second tile's column, -1 single), one per wave
// maxt32 / maxt16: the largest cr_task_tiles over the stage's tasks at ts = 32 / 16;
// ntmax: the largest term count
CrGemmCfg cr_gemm_config(const CrDims& c, int ntasks, int maxt32, int maxt16, int ntmax, int ntiles16);
// 16 x 16 stages (cfg.ts == 16): the dispatch-ordered slots of the stage's
// (task, tile) list tl16 (ntl16 entries per batch item) over every batch item,
// a whole number of workgroups (cr_gemm_slot_wgs of them)
int cr_gemm_slot_wgs(const CrDims& c, int ntl16, const CrGemmCfg& cfg);
void cr_gemm_slots(const CrDims& c, const CrTile* tl16, int ntl16, const CrGemmCfg& cfg, CrSlot* out);
// slots: the stage's cr_gemm_slots (16 x 16 stages); tasks: 32 x 32 stages
void launch_cr_gemm(const CrDims& c, double2* pool, const CrTask* tasks, int ntasks, int maxt32,
                    int maxt16, const CrSlot* slots, int nslot_wgs, const CrGemmCfg& cfg, double sg,
                    hipStream_t s);

// dense h - i y_q (padded with identity) for every (chain, pole): R init input
void launch_fill_hz(const Dims& d, double2* M, const int* hcol, const double* hval,
                    const double* ypole, hipStream_t s);
// Blocked Gauss-Jordan (no pivoting) on all nbatch matrices in M, in pairs of
// 64-wide block steps (see k_gj_update in dwhmc_kernels.hip for the modes).
// pivot: every block inverts S_kk; block j writes X_kj = S_kk^-1 S_kj in place
// and to XRout; block k writes S_kk^-1 to Pout; colcopy (nullable) receives the
// column panel of block column k; nextcol (nullable) receives X_{k,k+1} as row
// block k of the next column panel.
void launch_gj_pivot(const Dims& d, double2* M, int k, double2* Pout, double2* XRout,
                     double2* colcopy, double2* nextcol, double* ldpart, hipStream_t s);
struct GJPanelPtrs {
  const double2 *CpA, *CpB, *XR1, *XR2, *Pb1, *Pb2;
  double2 *CpBw, *CpN;
};
int gj_update_tiles(const Dims& d, int mode);
void launch_gj_update(const Dims& d, double2* M, int k, int mode, const GJPanelPtrs& p,
                      hipStream_t s);
// Dv[c][r][s] = Δ_c[Dsrc[r][s]] / 2: the pairing values of D for every chain
void launch_dvals(const Dims& d, const int* Dsrc, const double2* Delta, double2* Dv,
                  hipStream_t s);
// S^T = -(h + i y) - (D† R D)^T for every (chain, pole)
void launch_assemble(const Dims& d, const double2* R, double2* S, const int* Dcol,
                     const double2* Dv, const int* hcol, const double* hval, const double* ypole,
                     hipStream_t s);
// G12 at the pairing pattern: G12nn[bi][i][s] = -(R D S^{-1})[i, Dcol[i][s]]; diag of S^{-1}
void launch_contract(const Dims& d, const double2* R, const double2* SinvT, const int* Dcol,
                     const double2* Dv, double2* G12nn, double2* diagS, hipStream_t s);
// P = Σ_q c_q (G12[i,j] + G12[j,i]); F = -β/2J (Δ - J P); kick / drift
void launch_pair_force(const Dims& d, const double2* G12nn, const int* bond_ij,
                       const int* bond_ji, const double* cpole, double2* Delta, double2* Pair,
                       double2* F, double2* Pi, const KickDrift& kd, double beta, double J,
                       hipStream_t s);
// F from cached P; kick / drift
void launch_force_from_pair(const Dims& d, const double2* Pair, double2* Delta, double2* F,
                            double2* Pi, const KickDrift& kd, double beta, double J, hipStream_t s);
// E_f and Tr ρ_hh from the pivots of the last factorisation
void launch_fermion_energy(const Dims& d, const double* ldstatic, const double* ldpart,
                           const double2* diagS, const double* cpole, double Cx, double beta,
                           double* Ef, double* Trhh, hipStream_t s);
// H = Σ|π|²/2m + β/2J Σ|Δ|² + E_f into Hout[c]
// trajectory start / end of the throughput path in one launch each (k_traj_begin:
// refresh + H_old + backup + force from the cached P + kick/drift; k_traj_end:
// H_new + Metropolis + restore).
// Guard trips inside a batch of sweeps (SweepHalt): k_traj_end of the sweep
// whose kernels set *flag records its sequence number in halt[1] and sets
// halt[0]; every later k_traj_begin / k_traj_end of the batch then returns at
// once, so the backups (Δ, P, E_f, Tr ρ_hh) keep the tripped sweep's starting
// point for the host to resume from.  halt == nullptr: off.
struct SweepHalt {
  int* halt = nullptr;   // [0] halted, [1] sequence number of the tripped sweep
  int seq = 0;           // this sweep's sequence number in the batch
  const int* flag = nullptr;
};
void launch_traj_begin(const Dims& d, const double2* noise, double scale, double2* Pi, double2* Delta,
                       const double2* Pair, double2* F, const double* Ef, const double* Trhh, double2* DeltaB,
                       double2* PairB, double* EfB, double* TrhhB, double* Hold, double beta, double J,
                       double mass, const KickDrift& kd, const SweepHalt& sh, hipStream_t s);
void launch_traj_end(const Dims& d, double2* Delta, const double2* Pi, double2* Pair, double* Ef, double* Trhh,
                     const double2* DeltaB, const double2* PairB, const double* EfB, const double* TrhhB,
                     const double* Hold, double* Hnew, const double* uniform, uint8_t* accepted, double* dH,
                     double beta, double J, double mass, const SweepHalt& sh, hipStream_t s);
void launch_total_energy(const Dims& d, const double2* Delta, const double2* Pi,
                         const double* Ef, double beta, double J, double mass, double* Hout,
                         hipStream_t s);
void launch_refresh(const Dims& d, const double2* noise, double2* Pi, double scale, hipStream_t s);
void launch_backup(const Dims& d, const double2* Delta, const double2* Pair, const double* Ef,
                   const double* Trhh, double2* DeltaB, double2* PairB, double* EfB,
                   double* TrhhB, hipStream_t s);
void launch_metropolis(const Dims& d, const double* Hold, const double* Hnew,
                       const double* uniform, uint8_t* accepted, double* dH, hipStream_t s);
void launch_restore(const Dims& d, const uint8_t* accepted, const double2* DeltaB,
                    const double2* PairB, const double* EfB, const double* TrhhB,
                    double2* Delta, double2* Pair, double* Ef, double* Trhh, hipStream_t s);
void launch_sum_ld(const Dims& d, const double* ldpart, double* ldsum, hipStream_t s);

// Transport / spectra measurement (dwhmc_transport.hip): device buffers of one
// measurement (n2 = 2N; U, JU, Jmn: n2 x n2 column-major)
struct TrBufs {
  double2 *U, *JU, *Jmn;
  double *E, *f, *dia, *Wn, *wan, *w0, *lam, *dc;   // n2 each
  double *part, *sigma, *dos, *dos_an, *ak, *scalars;
};
// ω grid: w0 + k dw (k < nw); DOS grid: d0 + k dw (k < nd)
struct TrGrid {
  double w0, d0, dw;
  int nw, nd;
};
// DOS eigenvalue slices (k_tr_dos partials: 2 x slices x nd doubles in the
// σ partial buffer)
// out_k = in_k^H (in: R x C, ld lin; out: C x R, ld lout), k < m
void launch_tr_conj_transpose(const double2* in, int R, int C, int lin, int64_t sin, double2* out, int lout,
                              int64_t sout, int m, hipStream_t s);
int tr_dos_slices(int N);
int tr_sigma_chunks(int N);   // rows of TrBufs::part (each nw long)
// dense H_BdG of one chain into A (zeroed beforehand)
void launch_tr_assemble(double2* A, int N, const int* hcol, const double* hval, const int* Dcol,
                        const int* Dsrc, const double2* Delta, hipStream_t s);
// f, the diamagnetic / DOS / antinodal weights and the A(k,0) weight per eigenstate;
// nbr: 3 x N (+x, +x+y, +x-y neighbours, 0-based)
void launch_tr_colstats(const double2* U, int N, int Lx, const double* E, double beta, double eta,
                        double t, double tp, const int* nbr, double* f, double* dia, double* Wn,
                        double* wan, double* w0, hipStream_t s);
// JU = (J ⊕ J) U, J in CSR form (N rows, val = Im J)
// JU[:, :ncol] = (J ⊕ J) U[:, :ncol]
void launch_tr_current(const double2* U, double2* JU, int N, const int* rowptr, const int* col,
                       const double* val, int ncol, hipStream_t s);
// everything after J_mn: Λ, dc, σ(ω), stiffness, DOS, A(k,0) (overwrites JU and Jmn).
// ph: U is closed under the particle-hole map (column n2-1-j = Θ column j for
// every j, dwh eigensolver's half solve without a zero-straddling cluster), so
// J_mn is needed (and computed) only in its columns < N and every pair sum
// runs over half the pairs (the pair (n, m) and its partner (n2-1-m, n2-1-n)
// carry the same |J|², E differences and Fermi-factor differences)
void launch_tr_reduce(const TrBufs& b, int N, int Lx, int Ly, double beta, double eta,
                      const TrGrid& g, bool ph, hipStream_t s);

// Eigendecomposition leapfrog step (algo eig; U, JU, rho: nc chains of n2 x n2
// column-major, E: nc x n2): JU = U diag(logistic(-β E)); after rho = JU U^H,
// P at the bonds, Tr ρ_hh and E_f per chain
void launch_eig_scale(const double2* U, double2* JU, const double* E, int N, int nc, double beta, hipStream_t s);
void launch_eig_gather(const double2* rho, const double* E, int N, int nc, const int* Dcol, const int* bond_ij,
                       double beta, double2* Pair, double* Ef, double* Trhh, hipStream_t s);

// *bad = 1 when any entry of U (nu complex) or E (ne real) is not finite
void launch_nonfinite(const double2* U, int64_t nu, const double* E, int64_t ne, int* bad, hipStream_t s);

// Hermitian eigensolver (dwhmc_eig.hip): m matrices of order n <= kEigMaxN,
// column-major, per-matrix stride sA (complex) / sZ (double)
constexpr int kEigTB = 64;                  // trailing-update tile (one workgroup; hemv partial slots)
constexpr int kEigNB = 64;                  // reflectors per back-transform block
constexpr int kEigMaxN = 5120;              // rows k_eig_step holds in registers
// eigenvalue gap / ||T|| below which inverse-iteration vectors are
// orthonormalised together (Cholesky QR); wider gaps leave overlaps <= ~eps /
// 1e-6 that the symmetric orthogonalisation step squares away.  (2.5e-4 in
// round 3 made runs of >64 "clustered" levels from n ~ 3000 on; runs that
// long are now orthonormalised by the host-driven Cholesky QR.)
constexpr double kEigClusterTol = 1e-6;
// the particle-hole half solve computes the partners' vectors itself unless
// the gap below c0 exceeds this (the partner images are not orthogonalised
// against the computed vectors: their overlap is ~eps ||T|| / gap)
constexpr double kEigZeroTol = 2.5e-4;
constexpr int kEigMaxCluster = 64;          // longest such run (else *bad: vendor fallback)
// deferral of the tridiagonalisation's rank-2 pairs (dwhmc_eig.hip): batches
// of kEigDeferMin+ matrices apply them every kEigDefer-th pass (at most
// kEigDeferMax pending); v_j / w_j live in a ring of kEigRing slots per matrix
constexpr int kEigDefer = 8;
constexpr int kEigSwitchM = 512;   // trailing columns a batch runs in the one-matrix scheme (eig_switch_col)
constexpr int kEigDeferMax = 8;
constexpr int kEigRing = kEigDeferMax + 2;
constexpr int kEigGP = (kEigMaxN + 255) / 256;   // k_eig_reduce workgroups per matrix (g partials)
// column i of the tridiagonalisation (k_eig_reduce + k_eig_step): the pass
// partials (+ the read pass's pending-pair corrections) -> pfin, column i with
// the pending pairs -> colfin, then w_{i-1}, v_i (d, e, tau).
// vv, ww: kEigRing x n per matrix (v_j, w_j in slot j % kEigRing);
// dpart: ceil(n / kEigTB) x 2 kEigDeferMax per matrix (a read pass's dots);
// pfin, colfin: n per matrix
void launch_eig_step(double2* A, int n, int i, int64_t sA, const double2* part, int64_t sP, double2* pfin,
                     double2* colfin, double2* vv, double2* ww, double* d, double* e, double2* tau,
                     const double2* dpart, int m, int K, hipStream_t s);
// step i + pass i (one matrix: folded into one pass launch); gpart: 3 kEigGP per matrix
void launch_eig_column(double2* A, int n, int i, int64_t sA, double2* part, int64_t sP, double2* pfin,
                       double2* colfin, double2* vv, double2* ww, double* d, double* e, double2* tau,
                       double2* dpart, double2* gpart, int m, hipStream_t s, int sw);
// first column a batch runs in the one-matrix scheme (eig_switch_col: the last
// kEigSwitchM columns, DWHMC_EIG_SWITCH_M overrides, 0 = none), passed to
// launch_eig_column as sw
int eig_switch_col(int n);
// the pending pairs on the trailing triangle (write passes) + hemv partials of v_i
void launch_eig_pass(double2* A, int n, int i, int64_t sA, double2* part, int64_t sP, const double2* vv,
                     const double2* ww, double2* dpart, int m, int K, hipStream_t s);
// eigenvalues ascending into E, ||T|| bound per matrix into tnorm
void launch_eig_bisect(const double* d, const double* e, int n, double* E, double* tnorm, int m, hipStream_t s);
// eigenvectors of T into Zt (Zt[r n + j]: component r of vector j), clusters orthonormalised;
// a cluster longer than maxc (<= kEigMaxCluster) sets *bad (the caller's vendor fallback)
// Only the indices [j0, n), and with c0 (per matrix, device) only those >= c0
// (the columns j0 <= j < c0 of Zt are zeroed): the particle-hole half solve
void launch_eig_invit(const double* d, const double* e, int n, const double* E, const double* tnorm, double* Zt,
                      double* U0, double* U1, double* U2, int64_t sZ, int* bad, int m, hipStream_t s,
                      int maxc = kEigMaxCluster, int j0 = 0, const int* c0 = nullptr);
// columns j < c0[k] of U = the particle-hole partners of columns n-1-j:
// (u; v) -> (-conj v; conj u)
void launch_eig_theta(double2* U, int n, int64_t sA, const int* c0, int m, hipStream_t s);
// U[:, j0:] from Zt[:, j0:] (real -> complex, transposed through LDS)
void launch_eig_zt_to_u(const double* Zt, double2* U, int n, int64_t sZ, int64_t sA, int m, hipStream_t s,
                        int j0 = 0);
constexpr int kEigDeferMin = 4;             // batches from this many matrices defer their rank-2 pairs
int eig_defer_k(int m);                     // deferral depth for m matrices (1: none)
constexpr int kEigGS = 8;                   // row slices of each block's Gram sum
// compact-WY T of every reflector block; Gp: m x nblk x kEigGS x kEigNB^2 scratch
void launch_eig_tfac(const double2* V, int n, int64_t sA, const double2* tau, double2* Gp, double2* Tb, int64_t sT,
                     int m, hipStream_t s);
// W2 (kb x n, ld kEigNB) = T (sum of the S row chunks of W, chunk s at rows s kb, ld ldw)
// the reflector blocks of V conjugate-transposed (block b at Vt + b kEigNB n,
// leading dimension kEigNB), for the back-transform's W = V^H U
void launch_eig_vt(const double2* A, int n, int64_t sA, double2* Vt, int m, hipStream_t s);
void launch_eig_tw(const double2* Tb, int64_t sT, const double2* W, int ldw, int64_t sW, int S, int kb, int n,
                   double2* W2, int64_t sW2, int m, hipStream_t s);

// Structure-preserving (quaternion) eigensolver (dwhmc_qeig.hip): m matrices
// of order n = 2M, column-major at stride sA, reduced site by site on their
// particle rows (A's bottom rows then hold the reflectors); part: q_part_elems
// per matrix (stride sP); W: 2M per matrix; tau, qa: M; Y: 2M; qd: M
int q_part_elems(int M);
bool q_supported(int M);   // sites per matrix the reduction takes (1 .. 3072)
#ifdef QSTAMPS
int q_stamps_read(unsigned long long* out, int nsteps);   // diagnostic builds (-DQSTAMPS)
#endif
void launch_q_reduce(double2* A, int M, int64_t sA, double2* part, int64_t sP, double2* W, double* tau, double2* Y,
                     double* qa, double2* qd, int m, hipStream_t s);
// site rotations: (ra, rd, rb) = T's blocks (a', d', b), G: per site (al, be)
void launch_q_rot(const double* qa, const double2* qd, const double2* Y, int M, double* ra, double2* rd, double* rb,
                  double2* G, int m, hipStream_t s);
// the 2M eigenvalues of T ascending into E (stride 2M), ||T|| bound into tnorm
void launch_q_bisect(const double* ra, const double2* rd, const double* rb, int M, double* E, double* tnorm, int m,
                     hipStream_t s);
// eigenvectors of the particle-hole half (E indices j0 .. 2M-1, nv = 2M - j0):
// inverse iteration into Zt (row r of vector jj at Zt[r nv + jj], interleaved
// rows 2s / 2s+1 = particle / hole of site s; LU scratch S: q_invit_scratch
// double2 per matrix)
int64_t q_invit_scratch(int M, int j0);
void launch_q_invit(const double* ra, const double2* rd, const double* rb, int M, const double* E, const double* tnorm,
                    int j0, double2* Zt, int64_t sZ, double2* S, int64_t sS, int m, hipStream_t s);
// the vectors of eigenvalue clusters (gaps <= ctol ||T||, at most q_max_cluster()
// long) orthonormalised in Zt (two rounds of Cholesky QR); *bad = 1 on failure
int q_max_cluster();
// the crowd at zero of one matrix's eigenvalues E (n, computed from j0): the
// number of levels k_q_orth orthonormalises with their Theta partners, 0: none
int q_zero_crowd(const double* E, int n, int j0, double tn);
void launch_q_orth(const double* E, const double* tnorm, int M, int j0, double2* Zt, int64_t sZ, double ctol, int* bad,
                   int m, hipStream_t s);
// U' columns j0.. (n x n, interleaved rows) = site rotations G of Yt (nv x n, ld nv)
void launch_q_ztu(const double2* Yt, int64_t sY, const double2* G, int M, int j0, double2* U, int64_t sU, int m,
                  hipStream_t s);
// the reflector pairs as the one-stage back-transform's V (n x n, interleaved
// rows; columns 2j, 2j+1 = v_j, Theta v_j) and complex tau (n per matrix)
void launch_q_vexpand(const double2* A, int64_t sA, const double* tau, int M, double2* V, double2* tauc, int m,
                      hipStream_t s);
// U (BdG order) from U' (interleaved): columns >= j0 copied, below j0 the Theta partners
void launch_q_final(const double2* Ui, int64_t sU, int M, int j0, double2* U, int m, hipStream_t s);

// The library's own batched fp64 products (dwhmc_gemm.hip):
// C = alpha op(A) op(B) + beta C, column-major, op 'N' or 'C' (conjugate
// transpose; 'T' for real), per-matrix strides sA / sB / sC (elements)
void gemm_z(char opa, char opb, int M, int N, int K, double2 alpha, const double2* A, int lda, int64_t sA,
            const double2* B, int ldb, int64_t sB, double2 beta, double2* C, int ldc, int64_t sC, int batch,
            hipStream_t s);
// two-level batch: batch x S products, operands at outer * x2 + s * x1; the
// last inner one (s = S - 1) with K = Klast
void gemm_z_chunked(char opa, char opb, int M, int N, int K, int Klast, int S, double2 alpha, const double2* A,
                    int lda, int64_t a1, int64_t a2, const double2* B, int ldb, int64_t b1, int64_t b2,
                    double2 beta, double2* C, int ldc, int64_t c1, int64_t c2, int batch, hipStream_t s);
void gemm_d(char opa, char opb, int M, int N, int K, double alpha, const double* A, int lda, int64_t sA,
            const double* B, int ldb, int64_t sB, double beta, double* C, int ldc, int64_t sC, int batch,
            hipStream_t s);

int selftest_mfma_layout(int device);

}  // namespace dwh
