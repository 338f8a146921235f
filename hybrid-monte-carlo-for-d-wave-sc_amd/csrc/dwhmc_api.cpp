// C-ABI context of the MI355X fermionic action/force path (include/dwhmc.h).
//
// Host-side responsibilities, each restating a reference function:
//   * static hopping block h from the neighbour tables with the reference's
//     upper-triangle overwrite order        (src/Hamiltonian.jl:10-47)
//   * pairing pattern D[r, c] <- Δ[src]/2 with the reference's overwrite order
//                                            (src/Hamiltonian.jl:55-86)
//   * pole selection from the compiled table for κ = β E'/2; beyond the
//     table the eigendecomposition path (algo eig: the library's own
//     eigensolver per step, dwhmc_eig.hip — the reference's own diagonalize
//     + compute_forces!)
//   * the per-sweep launch sequence of hmc_sweep! (src/HMC.jl:71-144)
// All arithmetic runs in the HIP kernels (dwhmc_kernels.hip); there is no CPU
// fallback: a missing device is an error.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/dwhmc.h"
#include "dwhmc_internal.h"
// Two compiled pole tables (tools/gen_pole_table.py): "budget", sup|tanh
// error| <= 5e-12 — half the 1e-11 absolute budget the pairing tolerance
// leaves for the expansion (|δP_ij| <= ε; E_f and F budgets are looser,
// DESIGN.md §2) — and "strict" (<= 2e-14).  DWHMC_POLE_TABLE selects one;
// default "budget".
namespace tab_strict {
#include "pole_table.inc"
}
namespace tab_budget {
#include "pole_table_eps5e-12.inc"
}

using dwh::Dims;
using dwh::kGJ;
using dwh::kHSlots;
using dwh::kSlots;

namespace {

thread_local std::string g_create_error;

struct PoleView {
  double kappa;
  int m;
  double C_u, err_tanh;
  const double *t, *a;
};
template <typename E>
PoleView pole_view(const E& e, const double* T, const double* A) {
  return PoleView{e.kappa, e.m, e.C_u, e.err_tanh, T + e.off, A + e.off};
}
struct PoleTable {
  const char* name;
  int size;
  PoleView (*at)(int);
};
const PoleTable kPoleTables[2] = {
    {"budget", tab_budget::kPoleTableSize,
     [](int e) { return pole_view(tab_budget::kPoleEntries[e], tab_budget::kPoleT, tab_budget::kPoleA); }},
    {"strict", tab_strict::kPoleTableSize,
     [](int e) { return pole_view(tab_strict::kPoleEntries[e], tab_strict::kPoleT, tab_strict::kPoleA); }},
};
const PoleTable* pole_table(std::string* err) {
  const char* e = std::getenv("DWHMC_POLE_TABLE");
  if (!e || !*e || std::strcmp(e, "budget") == 0) return &kPoleTables[0];
  if (std::strcmp(e, "strict") == 0) return &kPoleTables[1];
  *err = "DWHMC_POLE_TABLE must be budget or strict";
  return nullptr;
}

enum TimerName {
  T_GJ_UPDATE = 0, T_GJ_PIVOT, T_ASSEMBLE, T_CONTRACT, T_STEP, T_GJ_EDGE, T_CR_GEMM, T_CR_INV, T_CR_INVSIDE,
  T_EIG_OWN, T_EIG_VENDOR, T_CR_SPARSE, T_COUNT
};
const char* kTimerNames[T_COUNT] = {"gj_update", "gj_pivot", "assemble", "contract",
                                    "step",      "gj_edge",  "cr_gemm",  "cr_inv",
                                    "cr_inv_side",
                                    "eig_own",   "eig_vendor",   // eigensolves (work: matrices)
                                    "cr_sparse"};

enum Algo { ALGO_DENSE = 0, ALGO_CR = 1, ALGO_EIG = 2 };

// One stage of the cyclic-reduction plan: a batch of block inversions or a
// task list of block products (all batch items at once).
struct CrStage {
  int kind;        // 0 inversion, 1 products
  int first, n;    // range in CrPlan::inv_blk / CrPlan::tasks
  double sg;       // products: sign of the sum
  double flops;    // products: algorithmic fp64 flops per batch item (restricted ranges)
  int maxt32, maxt16, ntmax;
  int tfirst, ntiles;   // products: range in CrPlan::tiles16 (the stage's (task, tile) pairs);
                        // inversions: their side-work tasks in CrPlan::tasks (launch_cr_inv_side,
                        // maxt32 tiles each), flops in `flops`
  dwh::CrGemmCfg cfg;   // products: tile / K-split chosen once per context
  int sfirst = 0, nswg = 0;   // 16 x 16 products: their dispatch-ordered slots (CrPlan::slots, nswg workgroups)
  int l0 = 0;           // inversions: level 0 from the static R = A^-1 blocks (k_cr_inv0)
  int sp = 0;           // kind 2 (sparse level-0 stage): 0 forward (CrPlan::sp_fwd), 1 backward (sp_bwd)
};

struct CrPlan {
  int nblk = 0;
  std::vector<CrStage> stages;
  std::vector<dwh::CrTask> tasks;
  std::vector<dwh::CrTile> tiles16;          // per product stage: its 16 x 16 tiles with their operands
  std::vector<dwh::CrSlot> slots;            // per 16 x 16 product stage: its tiles of every batch item,
                                             // dispatch order (dwh::cr_gemm_slots; built with the stage configs)
  std::vector<int> inv_blk, inv_dst, inv_slot;   // inversion source / destination block, ln|det| slot
  std::vector<int> inv0_r;                       // level-0 inversions (l0 stage): R = A^-1 block per entry
  std::vector<int64_t> goff, doff;
  std::vector<int> fill_all, fill_step;      // level-0 blocks written at create / every step
  std::vector<int64_t> off_ph;               // pairing entries outside fill_step (-1: none)
  int n_ph = 0;                              // entries of off_ph >= 0
  // sparse level 0 (dwhmc_cr_sparse.hip): the stages' tasks and the level-0
  // U / L patterns (CrPlan::rowpat / colpat: [3 Ly][kCrSpNZ][BP])
  std::vector<dwh::CrSpFwd> sp_fwd;
  std::vector<dwh::CrSpBwd> sp_bwd;
  std::vector<int> rowpat, colpat;
};

// The sparse stages' per-task operand arrays (launch_cr_sp_fwd / _bwd,
// dwhmc_internal.h).  Per task: the row-pattern words of its left sparse
// operands, laid out [row r < HP][operand][entry] so a wave reads its row's
// words (and then their values) with scalar loads (row); and the column
// entries of its right operands, [operand][entry][column], value (cv) and
// meta word (cm: Δ index + 1 | op << 22 | row << 24), read coalesced.
// Forward tasks first; the backward ones from row_bwd0 / col_bwd0.
struct SpTaskArrays {
  std::vector<int> row, cm;
  std::vector<double2> cv;
  size_t row_bwd0 = 0, col_bwd0 = 0;
};

SpTaskArrays cr_sparse_task_arrays(const CrPlan& pl, int BP, const std::vector<double2>& colval,
                                   const std::vector<int>& colsrc) {
  const int NZ = dwh::kCrSpNZ, E = NZ * BP, HP = BP / 2;
  SpTaskArrays a;
  auto rows = [&](std::initializer_list<int> rbs) {   // [r][operand][entry]
    for (int r = 0; r < HP; ++r)
      for (int rb : rbs)
        for (int e = 0; e < NZ; ++e) a.row.push_back(pl.rowpat[(size_t)rb * E + (size_t)e * BP + r]);
  };
  auto cols = [&](int cb) {
    for (int k = cb * E; k < (cb + 1) * E; ++k) {
      const int w = pl.colpat[k], op = (w >> 22) & 3, idx = (w >> 14) & 0xff, src = colsrc[k];
      a.cv.push_back(colval[k]);
      a.cm.push_back((src < 0 ? 0 : src + 1) | op << 22 | idx << 24);
    }
  };
  for (const dwh::CrSpFwd& t : pl.sp_fwd) {
    rows({t.uk, t.ler, t.lel});
    cols(t.lk);
    cols(t.uel);
    cols(t.uer);
  }
  a.row_bwd0 = a.row.size();
  a.col_bwd0 = a.cv.size();
  for (const dwh::CrSpBwd& t : pl.sp_bwd) {
    rows({t.la, t.ue});
    cols(t.ua);
    cols(t.le);
  }
  return a;
}

// Nonzero patterns of the level-0 U[y] = A[y, y+1] (pool block Ly + y) and
// L[y] = A[y+1, y] (2 Ly + y) blocks, from the hopping / pairing tables
// exactly as k_cr_fill writes them (top half: hopping at (x, x_j), pairing at
// (x, HP + x_j) for partners j in the other row), as entries of the FULL
// block: row x of the top half, and row HP + x synthesised from it (M-form:
// [conj B | -conj A]).  Entry = top-half offset | (column for rowpat, row for
// colpat) << 14 | op << 22 (op 0 as stored, 1 conj, 2 -conj, 3 empty).  False when a
// row or column holds more than kCrSpNZ entries (the dense level 0 then runs).
bool cr_sparse_patterns(int Lx, int Ly, int BP, const std::vector<int>& hcol, const std::vector<int>& Dcol,
                        std::vector<int>& rowpat, std::vector<int>& colpat) {
  const int HP = BP / 2, NZ = dwh::kCrSpNZ;
  const int empty = 3 << 22;   // op 3: weight zero (dwhmc_cr_sparse.hip sp_val)
  rowpat.assign((size_t)3 * Ly * NZ * BP, empty);
  colpat.assign((size_t)3 * Ly * NZ * BP, empty);
  for (int t = 1; t <= 2; ++t)
    for (int y = 0; y < Ly; ++y) {
      if ((t == 1 && Ly < 2) || (t == 2 && Ly < 3)) continue;   // k_cr_fill's zero blocks
      const int b = t * Ly + y;
      const int yr = (t == 2) ? (y + 1) % Ly : y, yc = (t == 1) ? (y + 1) % Ly : y;
      std::set<std::pair<int, int>> top;
      for (int x = 0; x < Lx; ++x) {
        const int i = yr * Lx + x;
        for (int s = 0; s < kHSlots; ++s) {
          const int j = hcol[(size_t)i * kHSlots + s];
          if (j >= 0 && j / Lx == yc) top.insert({x, j % Lx});
        }
        for (int s = 0; s < kSlots; ++s) {
          const int j = Dcol[(size_t)i * kSlots + s];
          if (j >= 0 && j / Lx == yc) top.insert({x, HP + j % Lx});
        }
      }
      std::vector<int> rn(BP, 0), cn(BP, 0);
      auto put = [&](int r, int c, int off, int op) {
        if (rn[r] >= NZ || cn[c] >= NZ) return false;
        rowpat[((size_t)b * NZ + rn[r]++) * BP + r] = off | (c << 14) | (op << 22);
        colpat[((size_t)b * NZ + cn[c]++) * BP + c] = off | (r << 14) | (op << 22);
        return true;
      };
      for (const auto& xc : top) {
        const int x = xc.first, c = xc.second, off = x * BP + c;
        if (!put(x, c, off, 0)) return false;
        if (!(c >= HP ? put(HP + x, c - HP, off, 1) : put(HP + x, c + HP, off, 2))) return false;
      }
    }
  return true;
}
// Column-pattern values of the level-0 U / L blocks in the kernels' own
// [block][entry][BP] order, so the dense . sparse products read them
// coalesced instead of gathering one pool row per lane: the static hopping
// entries as stored (op applied; chain-independent: U / L hold no diagonal),
// and for the pairing entries the Δ index whose Δ/2 k_cr_fill / the force
// scatter writes there (src, the kernel applies op), exactly as k_cr_fill
// resolves both (the last matching table slot).
void cr_sparse_colvals(const std::vector<int>& colpat, int Lx, int Ly, int BP, const std::vector<int>& hcol,
                       const std::vector<double>& hval, const std::vector<int>& Dcol, const std::vector<int>& Dsrc,
                       std::vector<double2>& colval, std::vector<int>& colsrc) {
  const int HP = BP / 2, NZ = dwh::kCrSpNZ;
  colval.assign(colpat.size(), make_double2(0.0, 0.0));
  colsrc.assign(colpat.size(), -1);
  for (int t = 1; t <= 2; ++t)
    for (int y = 0; y < Ly; ++y) {
      const int b = t * Ly + y;
      const int yr = (t == 2) ? (y + 1) % Ly : y, yc = (t == 1) ? (y + 1) % Ly : y;
      for (int e = 0; e < NZ; ++e)
        for (int c = 0; c < BP; ++c) {
          const size_t k = ((size_t)b * NZ + e) * BP + c;
          const int w = colpat[k], op = (w >> 22) & 3;
          if (op == 3) continue;
          const int off = w & 0x3fff, x = off / BP, ct = off % BP;
          const int i = yr * Lx + x;
          if (ct < HP) {
            const int j = yc * Lx + ct;
            double h = 0.0;
            for (int sl = 0; sl < kHSlots; ++sl)
              if (hcol[(size_t)i * kHSlots + sl] == j) h = hval[(size_t)i * kHSlots + sl];
            colval[k] = make_double2(op == 2 ? -h : h, 0.0);
          } else {
            const int j = yc * Lx + (ct - HP);
            int src = -1;
            for (int sl = 0; sl < kSlots; ++sl)
              if (Dcol[(size_t)i * kSlots + sl] == j) src = Dsrc[(size_t)i * kSlots + sl];
            colsrc[k] = src;
          }
        }
    }
}

// nonzeros of row r / column c of level-0 block b in the patterns
int sp_nrow(const std::vector<int>& pat, int b, int r, int BP) {
  int n = 0;
  for (int e = 0; e < dwh::kCrSpNZ; ++e) n += ((pat[((size_t)b * dwh::kCrSpNZ + e) * BP + r] >> 22) & 3) != 3;
  return n;
}

// Lattice rows per CR block.  Default: as many rows as fill the narrowest
// block half (16 sites) — R = 16 / Lx, lowered to a divisor of Ly — so a
// lattice with Lx <= 8 runs fewer, unpadded blocks at no extra cost per block
// (8 x 8: 4 blocks of two rows instead of 8 half-empty ones, one CR level
// less).  Wider lattices keep one row per block: more rows would widen the
// blocks, and at L = 16 two rows per block (BP 64) measured slower than one
// (profiles/r04_exp_cr_two_row_blocks_C2.txt).
int cr_rows_per_block(int64_t Lx, int64_t Ly) {
  auto ok = [&](int64_t r) { return r >= 1 && Ly % r == 0 && dwh::cr_supported_bp((int)(2 * ((r * Lx + 15) / 16 * 16))); };
  int64_t r = std::max<int64_t>(1, 16 / Lx);
  while (r > 1 && !ok(r)) --r;
  return (int)r;
}

// Block cyclic reduction of the periodic block-tridiagonal H_BdG - i y (blocks
// = lattice rows) into stages; restates tools/cr_model.py
// cr_selected_inverse_top (checked there against dense inverses for Ly = 1 ..
// 24, odd and even).  Blocks are top halves (HP x BP); V, W are Q-form, every
// other block M-form (the form of each right operand goes into CrTask::bq).  Pool blocks:
// level-0 D[y] = y, U[y] = Ly + y, L[y] = 2 Ly + y (filled by k_cr_fill).
// Forward level (m blocks, eliminate odd e < m - m%2, keep even k):
//   inv D_e;  V1 = -U_a D_e^-1, V2 = -L_e D_e^-1, W1 = -D_e^-1 L_a, W2 = -D_e^-1 U_e
//   D'_k = D_k + V1(k+1) L_k + V2(k-1) U_(k-1);  U'_k = V1(k+1) U_(k+1);  L'_k = V2(k+1) L_k
//   (m = 2 folds the self-couplings of the 1-block chain into D': 4 terms)
// Backward (G of the next level known at its kept blocks and adjacent pairs):
//   G_ea = W1 G_aa + W2 G_ca,  G_ec = W1 G_ac + W2 G_cc,
//   G_ae = G_aa V1 + G_ac V2,  G_ce = G_ca V1 + G_cc V2,  G_ee = D_e^-1 + W1 G_ae + W2 G_ce.
//
// side: products off the critical path (W1/W2: operands of the backward pass
// only; U'/L': operands of the next level's products, which follow its
// inversion) leave the product stages and run as side work of a later
// inversion stage, on the CUs its few inversion workgroups leave idle; the
// product stages on the critical path keep only V1/V2 and D'.  Levels down
// to m = 4 (below that the stages are pure latency) and only where the
// receiving inversion stage leaves a quarter of the ncu CUs idle (nbatch =
// chains x poles inversion workgroups per block).
// side_woff = 2: inversion stages between a level and the one that runs its
// W products; side_m = 4: smallest level size m whose products move
// (profiles/r02_exp_cr_side_work.txt, r04_exp_cr_side_knobs_C3.txt).
//
// inv0: the level-0 inversions use static R = A^-1 blocks (k_cr_inv0), one
// per eliminated row, computed at context creation.
//
// Lx, Ly: the CR lattice — a block holds Lx consecutive sites of the linear
// site index i = y * Lx + x, i.e. R = Lx / Lx_lattice lattice rows when the
// context groups rows (cr_rows_per_block): every coupling stays between
// neighbouring blocks (hopping and pairing span one lattice row), so the
// recursion is the same; only which entries of the level-0 G blocks the
// force reads changes (computed from Dcol below, not assumed diagonal).
CrPlan build_cr_plan(int Lx, int Ly, int BP, const std::vector<int>& Dcol, bool side, int nbatch,
                     int ncu, bool inv0, const std::vector<int>* hcol) {
  // W products two inversion stages after their level, side work from m = 4
  // (profiles/r02_exp_cr_side_work.txt, r04_exp_cr_side_knobs_C3.txt)
  constexpr int side_woff = 2, side_m = 4;
  CrPlan pl;
  const int HP = BP / 2;
  // sparse level 0 (dwhmc_cr_sparse.hip): even Ly >= 4, a supported block,
  // patterns within kCrSpNZ, and BP >= 64 — at BP = 32 the dense level-0
  // products are cheaper than the two sparse launches (C2 L = 16: 10.3k vs
  // 9.5k steps/s; C3 L = 32: 3.82k vs 3.74k; C5 L = 48: 1.27k vs 1.08k,
  // profiles/r05_exp_sparse_level0.txt).  DWHMC_CR_SPARSE0=1 / 0 forces it
  // on (any supported BP) / off.
  const bool sparse0 = [&] {
    const char* e = std::getenv("DWHMC_CR_SPARSE0");
    const bool force = e && *e == '1';
    if ((e && *e == '0') || !hcol || Ly % 2 != 0 || Ly < 4 || !dwh::cr_supported_sparse0(BP)) return false;
    if (!force && BP < 64) return false;
    return cr_sparse_patterns(Lx, Ly, BP, *hcol, Dcol, pl.rowpat, pl.colpat);
  }();
  if (!sparse0) {
    pl.rowpat.clear();
    pl.colpat.clear();
  }
  // Backward merge (round 6): the G_ee stage of a coarse level u runs inside
  // the first backward stage of the next finer level f (m_f <= merge_max_m,
  // not level 0), one launch less per merged pair.  f's products that would
  // read G_ee(u) = Dinv + W1 G_ae + W2 G_ce = Dinv + G_ea V1 + G_ec V2 (u's
  // quantities at that position) read its expansion instead:
  //   W G_ee = (W Dinv) + (W W1) G_ae + (W W2) G_ce,
  //   G_ee V = (Dinv V) + G_ea (V1 V) + G_ec (V2 V),
  // the three forward products of each (W Dinv as the accumulate input)
  // formed off the critical path: side work of the final inversion (BP = 64)
  // or inside the top level's D' stage (other BP), while their cost fits
  // (tools/cr_model.py cr_flop_count restates the policy).
  // Default: levels up to m_f = 4 with side work (BP = 64; C3 +0.4 %, m_f = 8
  // -0.3 %: its products lengthen the final inversion and the merged m = 8
  // stage runs several workgroup rounds), up to 8 without (C2 +3.2 %;
  // profiles/r06_exp_cr_merge.txt).  DWHMC_CR_MERGE=m: levels up to m_f = m
  // (0: every G_ee stage on its own; A/B, tests).
  const int merge_max_m = [&] {
    const char* e = std::getenv("DWHMC_CR_MERGE");
    return e ? std::max(0, std::atoi(e)) : side ? 4 : 8;
  }();
  const bool merge = merge_max_m >= 2;
  auto nr = [&](int b, int r) { return sp_nrow(pl.rowpat, b, r, BP); };
  auto nc = [&](int b, int c) { return sp_nrow(pl.colpat, b, c, BP); };
  int nblk = 3 * Ly;
  std::vector<char> qform(3 * Ly, 0);   // per pool block: Q-form (products V, W)
  auto nb = [&]() {
    qform.push_back(0);
    return nblk++;
  };
  auto nbq = [&]() {
    qform.push_back(1);
    return nblk++;
  };
  struct Level {
    int m;
    std::vector<int> D, U, L, E, K;
    std::vector<int> Dinv;             // block holding D_e^-1 (then G_ee), by position e
    std::vector<int> V1, V2, W1, W2;   // indexed by position e
    std::vector<char> elim;
    bool sparse = false;               // level 0 by the sparse stages (no V / W blocks)
    // backward merge: this level's first backward stage also runs the G_ee
    // stage of the level above; xa / xc[e]: the blocks of the expansion of
    // G_aa / G_cc (when G_ee of the level above): {Dinv V, V1 V, V2 V,
    // W Dinv, W W1, W W2} (-1: none)
    bool merged = false;
    std::vector<std::array<int, 6>> xa, xc;
    std::vector<int> Gea, Gec, Gae, Gce;   // backward outputs by eliminated position
  };
  // Level-0 blocks are inverted out of place (they are never overwritten, so
  // per step only their pairing entries change), coarser blocks in place.
  // Returns the blocks that hold the inverses.
  // pending side work per inversion stage (ordinal: 0 = level 0, ..., the
  // last = the final single-block inversion)
  int n_inv = 1;
  std::vector<int> inv_wgs;   // inversion workgroups of each inversion stage
  for (int m = Ly; m > 1; m = (m + 1) / 2) {
    ++n_inv;
    inv_wgs.push_back(nbatch * (m / 2));
  }
  inv_wgs.push_back(nbatch);
  auto idle_ok = [&](int ord) { return 4 * inv_wgs[ord] <= 3 * ncu; };
  std::vector<std::vector<dwh::CrTask>> side_tasks(n_inv);
  std::vector<double> side_flops(n_inv, 0.0);
  int inv_ord = 0;
  auto add_inv = [&](const std::vector<int>& blocks, int& slot) {
    std::vector<dwh::CrTask>& stk = side_tasks[inv_ord];
    CrStage st{};
    st.kind = 0;
    st.first = (int)pl.inv_blk.size();
    st.n = (int)blocks.size();
    st.sg = 1.0;                        // side tasks carry their own sign (kCrNegBit)
    st.flops = side_flops[inv_ord];     // the side products' flops per batch item
    st.tfirst = (int)pl.tasks.size();
    st.ntiles = (int)stk.size();
    st.cfg = {32, 1};
    for (const dwh::CrTask& t : stk) st.maxt32 = std::max(st.maxt32, dwh::cr_task_tiles(t, 32));
    pl.tasks.insert(pl.tasks.end(), stk.begin(), stk.end());
    ++inv_ord;
    std::vector<int> dst;
    // level-0 blocks (the first inversion stage): from their static R blocks
    if (inv0 && std::all_of(blocks.begin(), blocks.end(), [&](int b) { return b < 3 * Ly; })) {
      st.l0 = 1;
      for (size_t i = 0; i < blocks.size(); ++i) pl.inv0_r.push_back(nb());
    }
    for (int b : blocks) {
      const int d = b < 3 * Ly ? nb() : b;
      pl.inv_blk.push_back(b);
      pl.inv_dst.push_back(d);
      pl.inv_slot.push_back(slot++);
      dst.push_back(d);
    }
    pl.stages.push_back(st);
    return dst;
  };
  struct Term { int a, b; };
  std::vector<dwh::CrTask> cur_tasks;
  // output window of the next tasks (full block unless restricted)
  int w_r0 = 0, w_r1 = HP, w_c0 = 0, w_c1 = BP;
  // The level-0 G blocks are read only by the gathers: the force reads the
  // pairing (B-part) entries (p_i, HP + p_j) of every bond, E_f and Tr rho_hh
  // the diagonal (p, p) of G_D.  need[k][y]: the 16 x 16 top-half tiles
  // (tr * (BP / 16) + tc) of G_D[y] (k = 0), G_U[y] = G[y, y+1] (1),
  // G_L[y] = G[y+1, y] (2) that hold such entries — the block the gathers
  // below resolve each bond to.  The last backward level computes only those
  // tiles of its G_ea (= G_L), G_ec (= G_U) and G_ee (= G_D).  One lattice
  // row per block: the diagonal B tiles of G_U / G_L (vertical bonds at
  // (x, HP + x)); two rows: the off-diagonal ones.
  const int ntc = BP / 16;
  std::vector<std::vector<std::set<int>>> need(3, std::vector<std::set<int>>(Ly));
  {
    const int Ns = Lx * Ly;
    for (int i = 0; i < Ns; ++i) {
      const int pi = i % Lx, y = i / Lx;
      need[0][y].insert((pi / 16) * ntc + pi / 16);
      for (int s = 0; s < kSlots; ++s) {
        const int j = Dcol[(size_t)i * kSlots + s];
        if (j < 0) continue;
        const int pj = j % Lx, yj = j / Lx;
        const int tile = (pi / 16) * ntc + (HP + pj) / 16;
        if (Ly == 1 || yj == y) need[0][y].insert(tile);
        else if (yj == (y + 1) % Ly) need[1][y].insert(tile);
        else need[2][(y - 1 + Ly) % Ly].insert(tile);
      }
    }
  }
  // per task of cur_tasks: the tiles to compute (nullptr: every tile of the window)
  std::vector<const std::set<int>*> cur_keep;
  const std::set<int>* keep_next = nullptr;
  auto task = [&](int out, int cin, std::initializer_list<Term> terms) {
    cur_keep.push_back(keep_next);
    dwh::CrTask t{};
    t.out = out;
    t.cin = cin;
    t.r0 = w_r0;
    t.r1 = w_r1;
    t.c0 = w_c0;
    t.c1 = w_c1;
    t.nt = 0;
    t.bq = 0;
    for (const Term& x : terms) {
      t.a[t.nt] = x.a;
      t.b[t.nt] = x.b;
      if (qform[x.b]) t.bq |= 1 << t.nt;
      t.nt++;
    }
    cur_tasks.push_back(t);
  };
  // to_side: the tasks become side work of inversion stage `ord` (tiles
  // with their own sign) instead of a product stage
  auto flush = [&](double sg, bool to_side = false, int ord = 0) {
    if (cur_tasks.empty()) return;
    if (to_side) {
      for (dwh::CrTask t : cur_tasks) {
        if (sg < 0) t.bq |= dwh::kCrNegBit;
        side_tasks[ord].push_back(t);
        side_flops[ord] += 8.0 * t.nt * BP * (double)(t.r1 - t.r0) * (t.c1 - t.c0);
      }
      cur_tasks.clear();
      cur_keep.clear();
      return;
    }
    CrStage st{};
    st.kind = 1;
    st.first = (int)pl.tasks.size();
    st.n = (int)cur_tasks.size();
    st.sg = sg;
    st.flops = 0.0;                     // accumulated per task below
    st.tfirst = (int)pl.tiles16.size();
    st.ntiles = 0;
    st.cfg = {16, 1};
    for (size_t ti = 0; ti < cur_tasks.size(); ++ti) {
      const dwh::CrTask& t = cur_tasks[ti];
      const int nk = dwh::cr_task_tiles(t, 16), ct = (t.c1 + 15) / 16 - t.c0 / 16;
      int kept = 0;
      for (int k = 0; k < nk; ++k) {
        const int tr = t.r0 / 16 + k / ct, tc = t.c0 / 16 + k % ct;
        if (cur_keep[ti] && !cur_keep[ti]->count(tr * ntc + tc)) continue;
        dwh::CrTile d{};
        d.out = t.out;
        d.cin = t.cin;
        d.nt = t.nt;
        d.bq = t.bq;
        for (int h = 0; h < 4; ++h) {
          d.a[h] = t.a[h];
          d.b[h] = t.b[h];
        }
        d.tr = tr;
        d.tc = tc;
        pl.tiles16.push_back(d);
        kept++;
      }
      st.flops += 8.0 * t.nt * BP * (double)(t.r1 - t.r0) * (t.c1 - t.c0) * kept / nk;
      st.maxt32 = std::max(st.maxt32, dwh::cr_task_tiles(t, 32));
      st.maxt16 = std::max(st.maxt16, dwh::cr_task_tiles(t, 16));
      st.ntmax = std::max(st.ntmax, t.nt);
      pl.tasks.push_back(t);
    }
    st.ntiles = (int)pl.tiles16.size() - st.tfirst;
    pl.stages.push_back(st);
    cur_tasks.clear();
    cur_keep.clear();
  };

  Level cur;
  cur.m = Ly;
  for (int y = 0; y < Ly; ++y) {
    cur.D.push_back(y);
    cur.U.push_back(Ly + y);
    cur.L.push_back(2 * Ly + y);
  }
  std::vector<Level> levels;
  int slot = 0;
  while (cur.m > 1) {
    const int m = cur.m;
    // inv_ord: this level's inversion stage (added below)
    const bool side_ul = side && m >= side_m && idle_ok(inv_ord + 1);
    // with the backward merge the final inversion hosts the merge products,
    // which read W: the W products go at most to the stage before it
    const int w_ord = std::min(n_inv - (merge ? 2 : 1), inv_ord + side_woff);
    const bool side_w = side && m >= side_m && w_ord > inv_ord && idle_ok(w_ord);
    cur.elim.assign(m, 0);
    cur.E.clear();
    cur.K.clear();
    for (int e = 1; e < m - (m % 2); e += 2) {
      cur.E.push_back(e);
      cur.elim[e] = 1;
    }
    for (int k = 0; k < m; k += 2) cur.K.push_back(k);
    cur.V1.assign(m, -1);
    cur.V2.assign(m, -1);
    cur.W1.assign(m, -1);
    cur.W2.assign(m, -1);
    std::vector<int> inv;
    for (int e : cur.E) inv.push_back(cur.D[e]);
    const std::vector<int> dinv = add_inv(inv, slot);
    cur.Dinv.assign(m, -1);
    for (size_t i = 0; i < cur.E.size(); ++i) cur.Dinv[cur.E[i]] = dinv[i];
    if (sparse0 && levels.empty() && m % 2 == 0 && m >= 4) {
      // level 0: D', U', L' of every kept row in one sparse stage (no V / W)
      CrStage st{};
      st.kind = 2;
      st.sp = 0;
      st.first = (int)pl.sp_fwd.size();
      Level nxt;
      nxt.m = (int)cur.K.size();
      for (int k : cur.K) {
        const int er = k + 1, el = (k - 1 + m) % m;
        const int Dn = nb(), Un = nb(), Ln = nb();
        pl.sp_fwd.push_back(dwh::CrSpFwd{cur.D[k], cur.U[k], cur.L[k], cur.U[el], cur.L[el], cur.U[er], cur.L[er],
                                         cur.Dinv[er], cur.Dinv[el], Dn, Un, Ln});
        for (int r = 0; r < HP; ++r)   // V1r, V2r, V2l rows
          st.flops += 8.0 * BP * (nr(cur.U[k], r) + nr(cur.L[er], r) + nr(cur.L[el], r));
        for (int c = 0; c < BP; ++c)   // D' (2 terms), U', L'
          st.flops += 8.0 * HP * (2 * nc(cur.L[k], c) + nc(cur.U[el], c) + nc(cur.U[er], c));
        nxt.D.push_back(Dn);
        nxt.U.push_back(Un);
        nxt.L.push_back(Ln);
      }
      st.n = (int)pl.sp_fwd.size() - st.first;
      pl.stages.push_back(st);
      cur.sparse = true;
      levels.push_back(cur);
      cur = nxt;
      continue;
    }
    for (int e : cur.E) {
      const int a = e - 1;
      cur.V1[e] = nbq();
      task(cur.V1[e], -1, {{cur.U[a], cur.Dinv[e]}});
      cur.V2[e] = nbq();
      task(cur.V2[e], -1, {{cur.L[e], cur.Dinv[e]}});
    }
    if (side_w) flush(-1.0);
    for (int e : cur.E) {
      const int a = e - 1;
      cur.W1[e] = nbq();
      task(cur.W1[e], -1, {{cur.Dinv[e], cur.L[a]}});
      cur.W2[e] = nbq();
      task(cur.W2[e], -1, {{cur.Dinv[e], cur.U[e]}});
    }
    // W_l: first needed by the backward pass; placed three inversion stages
    // later (the coarse inversions leave ~240 of 256 CUs idle), the U'/L'
    // products of this level take the next one
    flush(-1.0, side_w, w_ord);
    Level nxt;
    nxt.m = (int)cur.K.size();
    std::vector<dwh::CrTask> ul_tasks;   // U'/L' (side work when `side`)
    for (int k : cur.K) {
      if (m == 2) {
        const int e = 1, Dn = nb();
        task(Dn, cur.D[0], {{cur.V1[e], cur.L[0]}, {cur.V2[e], cur.U[1]}, {cur.V1[e], cur.U[1]},
                            {cur.V2[e], cur.L[0]}});
        nxt.D.push_back(Dn);
        nxt.U.push_back(-1);
        nxt.L.push_back(-1);
        continue;
      }
      const int er = k + 1, el = (k - 1 + m) % m;
      const bool hr = er < m && cur.elim[er], hl = cur.elim[el];
      const int Dn = nb();
      if (hr && hl)
        task(Dn, cur.D[k], {{cur.V1[er], cur.L[k]}, {cur.V2[el], cur.U[el]}});
      else if (hr)
        task(Dn, cur.D[k], {{cur.V1[er], cur.L[k]}});
      else
        task(Dn, cur.D[k], {{cur.V2[el], cur.U[el]}});
      nxt.D.push_back(Dn);
      if (hr) {
        const int Un = nb(), Ln = nb();
        task(Un, -1, {{cur.V1[er], cur.U[er]}});
        task(Ln, -1, {{cur.V2[er], cur.L[k]}});
        if (side_ul) {   // move them behind the D' tasks of this stage
          ul_tasks.push_back(cur_tasks[cur_tasks.size() - 2]);
          ul_tasks.push_back(cur_tasks.back());
          cur_tasks.resize(cur_tasks.size() - 2);
          cur_keep.resize(cur_keep.size() - 2);
        }
        nxt.U.push_back(Un);
        nxt.L.push_back(Ln);
      } else {   // odd m: the kept pair (m-1, 0) keeps its direct coupling
        nxt.U.push_back(cur.U[k]);
        nxt.L.push_back(cur.L[k]);
      }
    }
    // the top level (its only kept block is the final one): plan the
    // backward merges now that every forward block exists; their products go
    // into this D' stage (no side work) or the final inversion (side work)
    std::vector<dwh::CrTask> merge_tasks;
    if (merge && nxt.m == 1) {
      std::vector<Level*> all;
      for (Level& lv : levels) all.push_back(&lv);
      all.push_back(&cur);
      // budget: side work of two workgroup rounds (4 wave tiles each) on the
      // CUs the final inversion leaves idle (a side workgroup takes ~6 us of
      // the inversion's ~16), or 16 x 16 tiles added to this (latency-bound)
      // D' stage
      const int64_t t32 = (int64_t)((HP + 31) / 32) * ((BP + 31) / 32), t16 = (int64_t)(HP / 16) * (BP / 16);
      int64_t side_t = 0;
      for (const dwh::CrTask& t : side_tasks[n_inv - 1]) side_t += dwh::cr_task_tiles(t, 32);
      const int64_t budget = side ? 8 * ((int64_t)ncu - nbatch) - side_t * nbatch : 1024;
      int64_t used = 0;
      for (int li = (int)all.size() - 2; li >= 1; --li) {
        Level& f = *all[li];
        const Level& u = *all[li + 1];
        if (f.sparse || f.m > merge_max_m) break;
        int nx = 0;
        for (int e : f.E) {
          const int a = e - 1, c = (e + 1) % f.m;
          nx += u.elim[a / 2] + u.elim[(c / 2) % u.m];
        }
        const int64_t cost = 6 * (int64_t)nx * nbatch * (side ? t32 : t16);
        if (used + cost > budget) break;
        used += cost;
        f.merged = true;
        f.xa.assign(f.m, {-1, -1, -1, -1, -1, -1});
        f.xc.assign(f.m, {-1, -1, -1, -1, -1, -1});
        for (int e : f.E) {
          const int a = e - 1, c = (e + 1) % f.m;
          // p: u's eliminated position next to e; V, W: the f products that meet G_ee(u)[p]
          auto expand = [&](int pu, int V, int W) {
            std::array<int, 6> x;
            x[0] = nb();    // Dinv V  (M Q -> M)
            x[1] = nbq();   // V1 V    (Q Q -> Q)
            x[2] = nbq();   // V2 V
            x[3] = nb();    // W Dinv  (Q M -> M)
            x[4] = nbq();   // W W1
            x[5] = nbq();   // W W2
            const int src[6][2] = {{u.Dinv[pu], V}, {u.V1[pu], V}, {u.V2[pu], V},
                                   {W, u.Dinv[pu]}, {W, u.W1[pu]}, {W, u.W2[pu]}};
            for (int k = 0; k < 6; ++k) {
              dwh::CrTask t{};
              t.out = x[k];
              t.cin = -1;
              t.r0 = 0;
              t.r1 = HP;
              t.c0 = 0;
              t.c1 = BP;
              t.nt = 1;
              t.a[0] = src[k][0];
              t.b[0] = src[k][1];
              t.bq = qform[src[k][1]] ? 1 : 0;
              merge_tasks.push_back(t);
            }
            return x;
          };
          if (u.elim[a / 2]) f.xa[e] = expand(a / 2, f.V1[e], f.W1[e]);
          if (u.elim[(c / 2) % u.m]) f.xc[e] = expand((c / 2) % u.m, f.V2[e], f.W2[e]);
        }
      }
      if (!side)
        for (const dwh::CrTask& t : merge_tasks) {
          cur_tasks.push_back(t);
          cur_keep.push_back(nullptr);
        }
    }
    flush(1.0);
    if (!ul_tasks.empty()) {
      cur_tasks = ul_tasks;
      cur_keep.assign(ul_tasks.size(), nullptr);
      flush(1.0, true, inv_ord);
    }
    if (side && !merge_tasks.empty()) {
      cur_tasks = merge_tasks;
      cur_keep.assign(merge_tasks.size(), nullptr);
      flush(1.0, true, n_inv - 1);
    }
    levels.push_back(cur);
    cur = nxt;
  }
  const int Dfin = add_inv({cur.D[0]}, slot)[0];
  std::vector<int> GD{Dfin}, GU{Dfin}, GL{Dfin};
  // the G_ee tasks of the level above when they run in this level's first stage
  struct GeeTask { int out, cin, a0, b0, a1, b1; };
  std::vector<GeeTask> pend;
  auto emit_pend = [&] {
    for (const GeeTask& t : pend) task(t.out, t.cin, {{t.a0, t.b0}, {t.a1, t.b1}});
    pend.clear();
  };
  for (int li = (int)levels.size() - 1; li >= 0; --li) {
    Level& lv = levels[li];
    // a pending G_ee stage whose finer level does not merge runs on its own
    if (!pend.empty() && !lv.merged) {
      emit_pend();
      flush(1.0);
    }
    const int m = lv.m, mn = (int)lv.K.size();
    std::vector<int> gd(m, -1), gu(m, -1), gl(m, -1);
    for (int kk = 0; kk < mn; ++kk) {
      const int k = lv.K[kk];
      gd[k] = GD[kk];
      if (!(k + 1 < m && lv.elim[k + 1])) {
        gu[k] = GU[kk];
        gl[k] = GL[kk];
      }
    }
    // Level 0 is the last backward level: G_ea, G_ec (cross-block bonds, not
    // operands of anything after them) are formed only on the B-part tiles
    // the vertical pairing bonds read (need); G_ae, G_ce (right operands of
    // G_ee in the dense level 0) need their whole top half there, and only
    // their need tiles in the sparse level 0 (G_ee from T = -Dinv M); G_ee
    // (in-block bonds, hole diagonal) its need tiles.
    const bool sel = (li == 0);
    const int H0 = sel ? HP : 0, H1 = sel ? HP + Lx : BP;
    if (lv.sparse) {
      // sparse level 0: Z_a, Z_c, Y_a, Y_c, M in one sparse stage, then
      // one-term products G_ae = -Z_a Dinv, G_ce = -Z_c Dinv, G_ea = -Dinv Y_a,
      // G_ec = -Dinv Y_c (need tiles), T = -Dinv M; then G_ee = Dinv - T Dinv
      CrStage st{};
      st.kind = 2;
      st.sp = 1;
      st.first = (int)pl.sp_bwd.size();
      struct Bw { int e, a, za, zc, ya, yc, mx; };
      std::vector<Bw> bw;
      for (int e : lv.E) {
        const int a = e - 1, c = (e + 1) % m;
        const int ia = a / 2, ic = (c / 2) % mn;
        const int Gaa = GD[ia], Gcc = GD[ic], Gac = GU[ia], Gca = GL[ia];
        const Bw x{e, a, nbq(), nbq(), nbq(), nbq(), nb()};
        bw.push_back(x);
        pl.sp_bwd.push_back(dwh::CrSpBwd{Gaa, Gac, Gca, Gcc, lv.U[a], lv.L[e], lv.L[a], lv.U[e], x.za, x.zc, x.ya,
                                         x.yc, x.mx, 0, 0, 0});
        for (int cc = 0; cc < BP; ++cc) st.flops += 8.0 * HP * 2 * (nc(lv.U[a], cc) + nc(lv.L[e], cc));   // Z_a, Z_c
        for (int r = 0; r < HP; ++r) st.flops += 8.0 * BP * 3 * (nr(lv.L[a], r) + nr(lv.U[e], r));       // Y_a, Y_c, M
      }
      st.n = (int)pl.sp_bwd.size() - st.first;
      pl.stages.push_back(st);
      std::vector<int> tn(m, -1);
      for (const Bw& x : bw) {
        const int e = x.e, a = x.a, D = lv.Dinv[e];
        const int gea = nb(), gec = nb(), gae = nb(), gce = nb();
        tn[e] = nbq();
        w_c0 = H0;
        w_c1 = H1;
        keep_next = &need[2][a];   // G_ea = G_L[a]
        task(gea, -1, {{D, x.ya}});
        keep_next = &need[1][e];   // G_ec = G_U[e]
        task(gec, -1, {{D, x.yc}});
        // G_ae = G_U[a] and G_ce = G_L[e] are read only by the gathers here
        // (G_ee comes from T, not from them): their need tiles only
        keep_next = &need[1][a];
        task(gae, -1, {{x.za, D}});
        keep_next = &need[2][e];
        task(gce, -1, {{x.zc, D}});
        keep_next = nullptr;
        w_c0 = 0;
        w_c1 = BP;
        task(tn[e], -1, {{D, x.mx}});
        gu[a] = gae;
        gl[a] = gea;
        gu[e] = gec;
        gl[e] = gce;
      }
      flush(-1.0);
      for (int e : lv.E) {
        const int gee = nb();
        keep_next = &need[0][e];
        task(gee, lv.Dinv[e], {{tn[e], lv.Dinv[e]}});
        gd[e] = gee;
      }
      keep_next = nullptr;
      flush(-1.0);
      GD = gd;
      GU = gu;
      GL = gl;
      continue;
    }
    // merged: this stage also runs the level above's G_ee (pend), and reads
    // G_ee(u) = Dinv + W1 G_ae + W2 G_ce = Dinv + G_ea V1 + G_ec V2 (u's
    // blocks at that position) through its expansion (xa / xc, formed in the
    // forward pass)
    const Level* up = lv.merged ? &levels[li + 1] : nullptr;
    emit_pend();
    lv.Gea.assign(m, -1);
    lv.Gec.assign(m, -1);
    lv.Gae.assign(m, -1);
    lv.Gce.assign(m, -1);
    for (int e : lv.E) {
      const int a = e - 1, c = (e + 1) % m;
      const int ia = a / 2, ic = (c / 2) % mn;
      const int Gaa = GD[ia], Gcc = GD[ic];
      const int Gac = mn == 1 ? GD[0] : GU[ia];
      const int Gca = mn == 1 ? GD[0] : GL[ia];
      const int gea = nb(), gec = nb(), gae = nb(), gce = nb();
      const bool xa = up && lv.xa[e][0] >= 0, xc = up && lv.xc[e][0] >= 0;
      w_c0 = H0;
      w_c1 = H1;
      keep_next = sel ? &need[2][a] : nullptr;   // G_ea = G[a + 1, a] = G_L[a]
      if (xa) {   // W1 G_aa = (W1 Dinv) + (W1 W1u) G_ae,u + (W1 W2u) G_ce,u
        const std::array<int, 6>& x = lv.xa[e];
        task(gea, x[3], {{x[4], up->Gae[ia]}, {x[5], up->Gce[ia]}, {lv.W2[e], Gca}});
      } else {
        task(gea, -1, {{lv.W1[e], Gaa}, {lv.W2[e], Gca}});
      }
      keep_next = sel ? &need[1][e] : nullptr;   // G_ec = G[e, e + 1] = G_U[e]
      if (xc) {   // W2 G_cc
        const std::array<int, 6>& x = lv.xc[e];
        task(gec, x[3], {{lv.W1[e], Gac}, {x[4], up->Gae[ic]}, {x[5], up->Gce[ic]}});
      } else {
        task(gec, -1, {{lv.W1[e], Gac}, {lv.W2[e], Gcc}});
      }
      keep_next = nullptr;
      w_c0 = 0;
      w_c1 = BP;
      if (xa) {   // G_aa V1 = (Dinv V1) + G_ea,u (V1u V1) + G_ec,u (V2u V1)
        const std::array<int, 6>& x = lv.xa[e];
        task(gae, x[0], {{up->Gea[ia], x[1]}, {up->Gec[ia], x[2]}, {Gac, lv.V2[e]}});
      } else {
        task(gae, -1, {{Gaa, lv.V1[e]}, {Gac, lv.V2[e]}});
      }
      if (xc) {   // G_cc V2
        const std::array<int, 6>& x = lv.xc[e];
        task(gce, x[0], {{Gca, lv.V1[e]}, {up->Gea[ic], x[1]}, {up->Gec[ic], x[2]}});
      } else {
        task(gce, -1, {{Gca, lv.V1[e]}, {Gcc, lv.V2[e]}});
      }
      gu[a] = gae;
      gl[a] = gea;
      gu[e] = gec;
      gl[e] = gce;
      lv.Gea[e] = gea;
      lv.Gec[e] = gec;
      lv.Gae[e] = gae;
      lv.Gce[e] = gce;
    }
    flush(1.0);
    // G_ee = Dinv + W1 G_ae + W2 G_ce, in place; deferred into the next finer
    // level's first stage when that one merges
    const bool defer = li >= 1 && levels[li - 1].merged;
    for (int e : lv.E) {
      if (defer) {
        pend.push_back(GeeTask{lv.Dinv[e], lv.Dinv[e], lv.W1[e], lv.Gae[e], lv.W2[e], lv.Gce[e]});
      } else {
        keep_next = sel ? &need[0][e] : nullptr;
        task(lv.Dinv[e], lv.Dinv[e], {{lv.W1[e], lv.Gae[e]}, {lv.W2[e], lv.Gce[e]}});
      }
      gd[e] = lv.Dinv[e];
    }
    keep_next = nullptr;
    if (!defer) flush(1.0);
    GD = gd;
    GU = gu;
    GL = gl;
  }
  // gather offsets of the level-0 G blocks
  const int N = Lx * Ly;
  const int64_t BB = (int64_t)HP * BP;
  pl.goff.assign((size_t)N * kSlots, -1);
  pl.doff.assign(N, 0);
  for (int i = 0; i < N; ++i) {
    const int x = i % Lx, y = i / Lx;
    for (int s = 0; s < kSlots; ++s) {
      const int j = Dcol[(size_t)i * kSlots + s];
      if (j < 0) continue;
      const int xj = j % Lx, yj = j / Lx;
      int blk;
      if (Ly == 1 || yj == y) blk = GD[y];
      else if (yj == (y + 1) % Ly) blk = GU[y];
      else blk = GL[(y - 1 + Ly) % Ly];
      pl.goff[(size_t)i * kSlots + s] = blk * BB + (int64_t)x * BP + (HP + xj);
    }
    pl.doff[i] = GD[y] * BB + (int64_t)x * BP + x;   // G22[x, x] = -conj(A[x, x])
  }
  // level-0 fill lists and pairing scatter offsets: CR never overwrites a
  // level-0 block (their inverses are formed out of place), so per step only
  // the pairing entries are scattered
  std::vector<char> rewrite(3 * Ly, 0);
  for (int b = 0; b < 3 * Ly; ++b) {
    pl.fill_all.push_back(b);
    if (rewrite[b]) pl.fill_step.push_back(b);
  }
  pl.off_ph.assign((size_t)N * kSlots, -1);
  auto blk_of = [&](int yr, int yc) {
    if (yc == yr) return yr;                              // D[yr]
    if (Ly >= 2 && yc == (yr + 1) % Ly) return Ly + yr;   // U[yr]
    return 2 * Ly + yc;                                   // L[yc] = A[yc+1, yc]
  };
  for (int i = 0; i < N; ++i)
    for (int s = 0; s < kSlots; ++s) {
      const int j = Dcol[(size_t)i * kSlots + s];
      if (j < 0) continue;
      const int yi = i / Lx, xi = i % Lx, yj = j / Lx, xj = j % Lx;
      const int b = blk_of(yi, yj);
      if (rewrite[b]) continue;
      pl.off_ph[(size_t)i * kSlots + s] = b * BB + (int64_t)xi * BP + (HP + xj);
      pl.n_ph++;
    }
  pl.nblk = nblk;
  return pl;
}

struct TimingRec {
  int name;
  hipEvent_t a, b;
  double work;
};

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
};

}  // namespace

struct dwh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  Dims d{};
  int64_t Lx = 0, Ly = 0;
  double t = 0, tp = 0, mu = 0, beta = 0, J = 0, delta_cap = 2.0;
  // guard: per site (mean |Δ| of its 4 bonds <= delta_cap, checked by the
  // level-0 inversion launch) or per bond (|Δ_ij| <= delta_cap, the drift kernels)
  bool site_guard = false;
  std::vector<int> site4_host;   // per site: the Delta indices of its 4 bonds
  int* site4 = nullptr;
  double kappa = 0, Ebound = 0, Cx = 0, err_tanh = 0, hmax = 0;
  std::vector<double> y, cq;
  // creation inputs kept for a pole re-selection (reselect_poles)
  std::vector<int64_t> nn_host, nnn_host;
  std::vector<double> dis_host;
  int reselections = 0;
  int64_t device_bytes = 0;
  bool factorized = false;
  std::string err;

  // device buffers
  double2 *R = nullptr, *S = nullptr;
  double2* Dv = nullptr;   // pairing values of D per chain (nc x N x kSlots)
  // Gauss-Jordan panels: column panels CpA[2] (parity), CpB; row panels XR1/XR2; pivots Pb1/Pb2
  double2 *CpA0 = nullptr, *CpA1 = nullptr, *CpB = nullptr, *XR1 = nullptr, *XR2 = nullptr,
          *Pb1 = nullptr, *Pb2 = nullptr;
  double2 *G12nn = nullptr, *diagS = nullptr;
  double *ldpart = nullptr, *ldstatic = nullptr, *d_y = nullptr, *d_c = nullptr;
  int *Dcol = nullptr, *Dsrc = nullptr, *hcol = nullptr, *bond_ij = nullptr, *bond_ji = nullptr;
  double* hval = nullptr;
  double2 *Delta = nullptr, *Pi = nullptr, *Pair = nullptr, *F = nullptr, *DeltaB = nullptr,
          *PairB = nullptr;
  double *Ef = nullptr, *EfB = nullptr, *Trhh = nullptr, *TrhhB = nullptr, *Hold = nullptr,
         *Hnew = nullptr;
  int* flag = nullptr;
  // guard trips inside a batch of throughput sweeps (dwh::SweepHalt): halt[0]
  // halted, halt[1] sequence number of the tripped sweep in `enq`
  int* halt = nullptr;
  struct EnqSweep {
    int64_t sweep, Nt;
    double dt, mass;
  };
  std::vector<EnqSweep> enq;   // throughput sweeps enqueued since the last settle()
  // draws / results: single-sweep scratch (s_*) and the throughput path
  double2* s_noise = nullptr;
  double* s_uniform = nullptr;
  uint8_t* s_acc = nullptr;
  double* s_dH = nullptr;
  int64_t ndraws = 0;
  double2* noise = nullptr;
  double* uniform = nullptr;
  uint8_t* acc = nullptr;
  double* dH = nullptr;
  std::vector<void*> allocations;

  // block cyclic-reduction path (algo == ALGO_CR)
  int algo = ALGO_DENSE;
  dwh::CrDims cr{};
  CrPlan plan;
  double2* bpool = nullptr;   // CR block pool (nbatch x nblk blocks)
  dwh::CrTask* d_tasks = nullptr;
  dwh::CrSlot* d_slots = nullptr;
  dwh::CrSpFwd* d_sp_fwd = nullptr;
  dwh::CrSpBwd* d_sp_bwd = nullptr;
  SpTaskArrays sp_arr;   // the sparse stages' per-task operand arrays
  int *d_sp_row = nullptr, *d_sp_cm = nullptr;
  double2* d_sp_cv = nullptr;
  double* efpart = nullptr;     // per (chain, pole) E_f / Tr G22 partials
  unsigned* efdone = nullptr;   // per chain: pole blocks done (k_cr_fermion_energy)
  int *d_inv_blk = nullptr, *d_inv_dst = nullptr, *d_inv_slot = nullptr, *d_inv0_r = nullptr;
  double* ldA = nullptr;   // static ln|det| of the Δ = 0 level-0 blocks (= 2 ln|det A|) per slot
  int64_t *d_doff = nullptr, *d_off_ph = nullptr;
  int64_t* d_bond4 = nullptr;   // k_cr_pair_force: per bond its G12 offsets and pairing-entry offsets
  int *d_fill_all = nullptr, *d_fill_step = nullptr;
  // the pool's level-0 pairing entries already hold the current Δ (set by a
  // drifting k_cr_pair_force, consumed by the next factorisation); every
  // other path that changes Δ leaves it false
  bool pairing_in_pool = false;
  bool pending = false;    // dwh_hmc_trajectory done, dwh_hmc_finish not yet
  int async_rc = 0;        // eig path: a rocSOLVER / rocBLAS call refused while enqueuing

  // transport / spectra measurement (device side allocated on first use): host
  // copies of the x-current operator J (CSR of its imaginary parts, duplicates
  // summed, src/Observables.jl:237-283) and of the +x, +x+y, +x-y neighbours;
  // the rocBLAS handle (rocSOLVER zheevd, zgemm) runs on ctx->stream
  std::vector<int> tr_nbr, tr_rowptr, tr_col;
  std::vector<double> tr_val;
  int tr_slots = 0;   // chains the per-chain transport buffers hold
  rocblas_handle blas = nullptr;
  dwh::TrBufs tr{};
  int *d_tr_nbr = nullptr, *d_tr_rowptr = nullptr, *d_tr_col = nullptr, *d_tr_info = nullptr;
  int* d_tr_bad = nullptr;   // eigen_solve: non-finite E / U after zheevd
  double* d_tr_val = nullptr;
  double* d_tr_offd = nullptr;   // zheevd off-diagonal workspace (2N)
  int64_t tr_nw = -1, tr_nd = -1;   // ω / DOS grid lengths the output buffers hold
  double2* d_tr_stage = nullptr;     // Δ snapshots of dwh_measure_transport_deltas
  int64_t tr_nstage = 0;
  // own eigensolver (dwhmc_eig.hip) workspace for eig_slots matrices: hemv
  // partials, v ping-pong, w, tridiagonal (d, e), tau, compact-WY T blocks and
  // the back-transform's two nb x n products; the n x n work lives in the
  // slots' JU (A -> V), Jmn and U (eigenvector / LU scratch) buffers
  int eig_slots = 0;
  double2 *d_eig_part = nullptr, *d_eig_vv = nullptr, *d_eig_ww = nullptr, *d_eig_tau = nullptr;
  double2 *d_eig_T = nullptr, *d_eig_W = nullptr, *d_eig_W2 = nullptr, *d_eig_dpart = nullptr;
  double2* d_eig_pfin = nullptr;   // the hemv partials reduced per row (k_eig_reduce)
  double2* d_eig_colfin = nullptr;   // column i with its pending pairs (k_eig_reduce)
  double2* d_eig_gpart = nullptr;    // k_eig_reduce's g partials (one matrix)
  int* d_eig_c0 = nullptr;         // particle-hole half solve: first computed eigenvector per matrix
  bool eig_half = false;           // the last own solve ran the particle-hole half solve
  std::vector<int> eig_c0h;        // its c0 per matrix (N: no zero crowding)
  // the last eigen_solve's U of every slot is closed under the particle-hole
  // map column by column (half solve, c0 = N everywhere, no fallback):
  // transport's pair sums then run over half the pairs
  bool eig_ph = false;
  int64_t eig_long_clusters = 0;   // clusters longer than k_eig_orth's limit, orthonormalised by long_clusters
  int eig_ph_last = -1;    // dwh_info_t::eig_half: eig_ph of the last eigensolve (-1: none yet)
  int eig_quat_last = 0;   // the last eigensolve took the structure-preserving solver
  double *d_eig_d = nullptr, *d_eig_e = nullptr, *d_eig_tn = nullptr;
  // structure-preserving solver (dwhmc_qeig.hip) workspace: q_slots matrices
  // (q_bufs), the eigenvector stage's for q_vec_slots (q_heev_enqueue)
  double* d_q = nullptr;
  int q_slots = 0, q_vec_slots = 0;
  double2 *d_qz = nullptr, *d_qs = nullptr, *d_qg = nullptr;
  // the reduction's launch sequence as a graph (its arguments: the slots, d_q, m)
  hipGraphExec_t q_graph = nullptr;
  const void* q_graph_key[2] = {};
  int q_graph_m = 0;
  hipStream_t eig_sx[3] = {};       // extra streams of the sub-batched tridiagonalisation
  hipEvent_t eig_ev[4] = {};

  // timing
  int timing = 0;   // bitmask over TimerName (bit i = kTimerNames[i])
  std::vector<TimingRec> recs;
  std::vector<hipEvent_t> pool;
  double t_ms[T_COUNT] = {0};
  int64_t t_n[T_COUNT] = {0};
  double t_work[T_COUNT] = {0};
};

namespace {

int fail(dwh_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  else g_create_error = msg;
  return code;
}

#define HIPCHECK(ctx, x)                                                                  \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      return fail((ctx), DWH_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

int settle(dwh_ctx* ctx);
// finish (and recover) pending throughput sweeps before the state is read or changed
#define SETTLE(ctx)                                 \
  do {                                              \
    if (!(ctx)->enq.empty())                        \
      if (int rc_ = settle(ctx)) return rc_;        \
  } while (0)

template <typename T>
int dalloc(dwh_ctx* ctx, T** p, size_t n) {
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess)
    return fail(ctx, DWH_ERR_HIP, "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
  ctx->allocations.push_back(q);
  ctx->device_bytes += (int64_t)bytes;
  *p = static_cast<T*>(q);
  return DWH_OK;
}

hipEvent_t take_event(dwh_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e;
  // no system-scope fence per record: the timers bracket device kernels only,
  // and the fence's L2 writeback would perturb the kernels being timed
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}

struct Scope {
  dwh_ctx* ctx;
  int name;
  double work;
  hipStream_t st;
  hipEvent_t a{};
  bool on;
  Scope(dwh_ctx* c, int n, double w)
      : ctx(c), name(n), work(w), st(c->stream), on(((c->timing >> n) & 1) != 0) {
    if (on) {
      a = take_event(ctx);
      (void)hipEventRecord(a, st);
    }
  }
  ~Scope() {
    if (on) {
      hipEvent_t b = take_event(ctx);
      (void)hipEventRecord(b, st);
      ctx->recs.push_back({name, a, b, work});
    }
  }
};

void drain_timing(dwh_ctx* ctx) {
  if (ctx->recs.empty()) return;
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& r : ctx->recs) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    ctx->t_ms[r.name] += ms;
    ctx->t_n[r.name] += 1;
    ctx->t_work[r.name] += r.work;
    ctx->pool.push_back(r.a);
    ctx->pool.push_back(r.b);
  }
  ctx->recs.clear();
}

double tile_flops() { return 8.0 * kGJ * kGJ * kGJ; }

void gj_pivot(dwh_ctx* ctx, double2* M, int k, double2* Pout, double2* XR, double2* colcopy,
              double2* nextcol) {
  const Dims& d = ctx->d;
  Scope s(ctx, T_GJ_PIVOT, (double)d.nbatch * d.nb * tile_flops());
  dwh::launch_gj_pivot(d, M, k, Pout, XR, colcopy, nextcol, ctx->ldpart, ctx->stream);
}

// complex K=64 terms of one update launch (per matrix), for the flop count
double gj_update_terms(const Dims& d, int mode) {
  const int nb = d.nb;
  if (nb < 2) return 0;
  if (mode == 0) return (double)(nb - 1) * nb;
  if (mode == 1) return 2.0 * nb - 2;
  return nb + (double)(nb - 2) * (1 + 2.0 * (nb - 1));
}

void gj_update(dwh_ctx* ctx, double2* M, int k, int mode, const dwh::GJPanelPtrs& p) {
  const Dims& d = ctx->d;
  Scope s(ctx, mode == 1 ? T_GJ_EDGE : T_GJ_UPDATE,
          (double)d.nbatch * gj_update_terms(d, mode) * tile_flops());
  dwh::launch_gj_update(d, M, k, mode, p, ctx->stream);
}

// Blocked no-pivot Gauss-Jordan inversion of all nbatch matrices in M, two
// 64-wide block steps at a time: pivot k, edge update (block row k+1 and the
// next column panel), pivot k+1, then ONE rank-128 update of the remaining
// tiles — every matrix tile is streamed through HBM once per two pivot steps.
// An odd last step uses the single rank-64 update.
void run_gj(dwh_ctx* ctx, double2* M) {
  const Dims& d = ctx->d;
  double2* CpA[2] = {ctx->CpA0, ctx->CpA1};
  if (d.nb == 1) {
    gj_pivot(ctx, M, 0, ctx->Pb1, ctx->XR1, nullptr, nullptr);
    return;
  }
  int cur = 0;
  for (int k = 0; k < d.nb;) {
    double2* colcopy = (k == 0) ? CpA[cur] : nullptr;
    if (k + 1 < d.nb) {
      gj_pivot(ctx, M, k, ctx->Pb1, ctx->XR1, colcopy, nullptr);
      dwh::GJPanelPtrs e{CpA[cur], nullptr, ctx->XR1, nullptr, ctx->Pb1, nullptr, ctx->CpB, nullptr};
      gj_update(ctx, M, k, 1, e);
      gj_pivot(ctx, M, k + 1, ctx->Pb2, ctx->XR2, nullptr, CpA[cur ^ 1]);
      dwh::GJPanelPtrs c{CpA[cur], ctx->CpB, ctx->XR1, ctx->XR2, ctx->Pb1, ctx->Pb2, nullptr,
                         k + 2 < d.nb ? CpA[cur ^ 1] : nullptr};
      gj_update(ctx, M, k, 2, c);
      cur ^= 1;
      k += 2;
    } else {
      gj_pivot(ctx, M, k, ctx->Pb1, ctx->XR1, colcopy, nullptr);
      dwh::GJPanelPtrs sg{CpA[cur], nullptr, ctx->XR1, nullptr, ctx->Pb1, nullptr, nullptr, nullptr};
      gj_update(ctx, M, k, 0, sg);
      k += 1;
    }
  }
}

// The per-factorisation assembly launch (timer "assemble"), with its
// algorithmic bytes.  CR: the pairing entries Δ/2 scattered into the level-0
// blocks of every batch item (16 B each; no level-0 block is rewritten, CR
// inverts them out of place); dense: S^T = -(h + z) - D^H R D written from R
// (read R once, write S^T).
void assembly_enqueue(dwh_ctx* ctx) {
  if (ctx->algo == ALGO_CR) {
    const dwh::CrDims& c = ctx->cr;
    const CrPlan& pl = ctx->plan;
    Scope s(ctx, T_ASSEMBLE,
            (double)pl.fill_step.size() * 8.0 * c.BP * (double)c.BP * c.nbatch + 16.0 * (double)pl.n_ph * c.nbatch);
    dwh::launch_cr_fill(c, ctx->bpool, ctx->d_fill_step, (int)pl.fill_step.size(), ctx->hcol, ctx->hval, ctx->Dcol,
                        ctx->Dsrc, ctx->Delta, ctx->d_y, ctx->d_off_ph, ctx->stream);
  } else {
    const Dims& d = ctx->d;
    Scope s(ctx, T_ASSEMBLE, (double)d.nbatch * 32.0 * d.N * (double)d.N);
    dwh::launch_assemble(d, ctx->R, ctx->S, ctx->Dcol, ctx->Dv, ctx->hcol, ctx->hval, ctx->d_y, ctx->stream);
  }
}

// level-0 blocks -> CR stages -> gather of the selected G entries
void cr_enqueue(dwh_ctx* ctx) {
  const dwh::CrDims& c = ctx->cr;
  const double bp3 = 8.0 * c.BP * (double)c.BP * c.BP * c.nbatch;
  {
    // algorithmic bytes: rewritten level-0 blocks (top halves, none with the
    // out-of-place level-0 inversions) + the pairing entries Δ/2 scattered
    // into the level-0 blocks of every batch item (16 B each)
    // inside a trajectory the previous step's force kernel already scattered
    // the drifted Δ into the pool (pairing_in_pool)
    if (!ctx->pairing_in_pool) assembly_enqueue(ctx);
    ctx->pairing_in_pool = false;
  }
  const CrPlan& plan = ctx->plan;
  // the site guard rides on the first (level-0) inversion launch: every
  // factorised Δ passes through it
  dwh::SiteGuard guard;
  if (ctx->site_guard) guard = dwh::SiteGuard{ctx->Delta, ctx->site4, 4.0 * ctx->delta_cap, ctx->flag};
  for (size_t si = 0; si < plan.stages.size(); ++si) {
    const CrStage& st = plan.stages[si];
    if (st.kind == 0 && st.ntiles > 0) {
      Scope s(ctx, T_CR_INVSIDE, st.n * bp3 + st.flops * c.nbatch);
      dwh::launch_cr_inv_side(c, ctx->bpool, ctx->d_inv_blk + st.first, ctx->d_inv_dst + st.first,
                              ctx->d_inv_slot + st.first, st.n, ctx->ldpart, ctx->d_tasks + st.tfirst,
                              st.ntiles, st.maxt32, ctx->stream, guard);
      guard = dwh::SiteGuard{};
    } else if (st.kind == 0 && st.l0) {
      Scope s(ctx, T_CR_INV, st.n * bp3);
      dwh::launch_cr_inv0(c, ctx->bpool, ctx->d_inv_blk + st.first, ctx->d_inv0_r, ctx->d_inv_dst + st.first,
                          ctx->d_inv_slot + st.first, st.n, ctx->ldpart, ctx->ldA, ctx->stream, guard.Delta,
                          guard.site4, guard.cap4, guard.flag);
      guard = dwh::SiteGuard{};
    } else if (st.kind == 0) {
      Scope s(ctx, T_CR_INV, st.n * bp3);
      dwh::launch_cr_inv(c, ctx->bpool, ctx->d_inv_blk + st.first, ctx->d_inv_dst + st.first,
                         ctx->d_inv_slot + st.first, st.n, ctx->ldpart, ctx->stream, guard);
      guard = dwh::SiteGuard{};
    } else if (st.kind == 2) {
      Scope s(ctx, T_CR_SPARSE, st.flops * c.nbatch);
      const size_t spE = (size_t)dwh::kCrSpNZ * c.BP, spR = (size_t)dwh::kCrSpNZ * (c.BP / 2);
      const SpTaskArrays& sa = ctx->sp_arr;
      if (st.sp == 0)
        dwh::launch_cr_sp_fwd(c, ctx->bpool, ctx->d_sp_fwd + st.first, st.n, ctx->d_sp_row + st.first * 3 * spR,
                              ctx->d_sp_cv + st.first * 3 * spE, ctx->d_sp_cm + st.first * 3 * spE, ctx->Delta,
                              ctx->stream);
      else
        dwh::launch_cr_sp_bwd(c, ctx->bpool, ctx->d_sp_bwd + st.first, st.n,
                              ctx->d_sp_row + sa.row_bwd0 + st.first * 2 * spR,
                              ctx->d_sp_cv + sa.col_bwd0 + st.first * 2 * spE,
                              ctx->d_sp_cm + sa.col_bwd0 + st.first * 2 * spE, ctx->Delta, ctx->stream);
    } else {
      Scope s(ctx, T_CR_GEMM, st.flops * c.nbatch);
      dwh::launch_cr_gemm(c, ctx->bpool, ctx->d_tasks + st.first, st.n, st.maxt32, st.maxt16,
                          ctx->d_slots + st.sfirst, st.nswg, st.cfg, st.sg, ctx->stream);
    }
  }
}

dwh::KickDrift kickdrift(dwh_ctx* ctx, double kick, double drift) {
  // the site guard is checked by k_cr_inv0, not per bond by the drift
  const double cap = ctx->site_guard ? std::numeric_limits<double>::infinity() : ctx->delta_cap;
  return dwh::KickDrift{kick, drift, cap, ctx->flag};
}

int transport_prepare(dwh_ctx* ctx, int64_t nw, int64_t nd, int slots);
// where the slots of a batched eigensolve take their H_BdG(Δ) from: slot k
// assembles Δ = Delta + k dstride with the hopping / disorder of chain
// chain0 + k cstep
struct TrSrc {
  const double2* Delta;
  int64_t dstride;
  int64_t chain0;
  int cstep;
};
TrSrc chains_src(const dwh_ctx* ctx, int64_t c0);
int eigen_solve(dwh_ctx* ctx, const TrSrc& src, int m);
int eigen_info_check(dwh_ctx* ctx, int m);

// algo eig: the library's eigensolver on every chain's H_BdG
// (src/Hamiltonian.jl:96-114), ρ = U diag(f) U^H by one batched product, then
// P, Tr ρ_hh and E_f (src/Observables.jl:14-62, src/HMC.jl:21-27) in
// k_eig_gather
void eig_enqueue(dwh_ctx* ctx) {
  const int N = ctx->d.N, n2 = 2 * N, nc = ctx->d.nc;
  if (int rc = eigen_solve(ctx, chains_src(ctx, 0), nc)) {
    ctx->async_rc = rc;
    return;
  }
  const dwh::TrBufs& b = ctx->tr;
  dwh::launch_eig_scale(b.U, b.JU, b.E, N, nc, ctx->beta, ctx->stream);
  const int64_t sA = (int64_t)n2 * n2;
  // rho = (U f) U^H, the library's own product
  dwh::gemm_z('N', 'C', n2, n2, n2, make_double2(1.0, 0.0), b.JU, n2, sA, b.U, n2, sA, make_double2(0.0, 0.0),
              b.Jmn, n2, sA, nc, ctx->stream);
  if (hipGetLastError() != hipSuccess) {   // a refused launch surfaces at the next eig_check
    ctx->err = "eig path: rho product launch failed";
    ctx->async_rc = DWH_ERR_HIP;
    return;
  }
  dwh::launch_eig_gather(b.Jmn, b.E, N, nc, ctx->Dcol, ctx->bond_ij, ctx->beta, ctx->Pair, ctx->Ef, ctx->Trhh,
                         ctx->stream);
}

// after a stream synchronisation (eig): an enqueue-time refusal, then the
// eigensolver's convergence flags
int eig_check(dwh_ctx* ctx) {
  if (ctx->algo != ALGO_EIG) return DWH_OK;
  if (ctx->async_rc != DWH_OK) {
    const int rc = ctx->async_rc;
    ctx->async_rc = DWH_OK;
    return rc;
  }
  return eigen_info_check(ctx, ctx->d.nc);
}

// assemble -> factorisation -> P -> F (+ kick / next drift); E_f separately
void factorize_enqueue(dwh_ctx* ctx, const dwh::KickDrift& kd) {
  const Dims& d = ctx->d;
  Scope step(ctx, T_STEP, (double)d.nbatch * 8.0 * (double)d.N * d.N * d.N);
  if (ctx->algo == ALGO_EIG) {
    // E_f and Tr ρ_hh come with every decomposition (k_eig_gather)
    eig_enqueue(ctx);
    dwh::launch_force_from_pair(d, ctx->Pair, ctx->Delta, ctx->F, ctx->Pi, kd, ctx->beta, ctx->J, ctx->stream);
    return;
  }
  if (ctx->algo == ALGO_CR) {
    cr_enqueue(ctx);
    // the kernel scatters the drifted Δ into the pool only when it drifts
    ctx->pairing_in_pool = kd.drift != 0.0;
    dwh::launch_cr_pair_force(ctx->cr, ctx->bpool, ctx->d_bond4, ctx->d_c, ctx->Delta, ctx->Pair, ctx->F, ctx->Pi,
                              kd, ctx->beta, ctx->J, ctx->stream);
    return;
  }
  dwh::launch_dvals(d, ctx->Dsrc, ctx->Delta, ctx->Dv, ctx->stream);
  assembly_enqueue(ctx);
  run_gj(ctx, ctx->S);
  {
    Scope s(ctx, T_CONTRACT, (double)d.nbatch * 32.0 * d.N * (double)d.N);
    dwh::launch_contract(d, ctx->R, ctx->S, ctx->Dcol, ctx->Dv, ctx->G12nn, ctx->diagS,
                         ctx->stream);
  }
  dwh::launch_pair_force(d, ctx->G12nn, ctx->bond_ij, ctx->bond_ji, ctx->d_c, ctx->Delta,
                         ctx->Pair, ctx->F, ctx->Pi, kd, ctx->beta, ctx->J, ctx->stream);
}

void fermion_energy_enqueue(dwh_ctx* ctx) {
  if (ctx->algo == ALGO_EIG) return;   // written by k_eig_gather with P
  if (ctx->algo == ALGO_CR)
    dwh::launch_cr_fermion_energy(ctx->cr, ctx->bpool, ctx->d_doff, ctx->ldpart, ctx->d_c, ctx->Cx,
                                  ctx->beta, ctx->efpart, ctx->efdone, ctx->Ef, ctx->Trhh, ctx->stream);
  else
    dwh::launch_fermion_energy(ctx->d, ctx->ldstatic, ctx->ldpart, ctx->diagS, ctx->d_c, ctx->Cx,
                               ctx->beta, ctx->Ef, ctx->Trhh, ctx->stream);
}

// One hmc_sweep! trajectory reading its draws from device pointers
// (src/HMC.jl:71-122): refresh, H_old, backup, leapfrog, H_new.
// with_hnew = false: the caller's k_traj_end forms H_new (with the Metropolis test)
void trajectory_enqueue(dwh_ctx* ctx, const double2* noise, int64_t Nt, double dt, double mass,
                        bool with_hnew = true, const dwh::SweepHalt& sh = dwh::SweepHalt{}) {
  const Dims& d = ctx->d;
  hipStream_t s = ctx->stream;
  const double coef_field = dt / (2.0 * mass);                                        // :95
  // :77 refresh, :80 H_old, :84-86 backup, :91-92 half kick fused with step
  // 1's drift (:101): one launch (k_traj_begin)
  dwh::launch_traj_begin(d, noise, std::sqrt(2.0 * mass), ctx->Pi, ctx->Delta, ctx->Pair, ctx->F, ctx->Ef,
                         ctx->Trhh, ctx->DeltaB, ctx->PairB, ctx->EfB, ctx->TrhhB, ctx->Hold, ctx->beta, ctx->J,
                         mass, kickdrift(ctx, 0.5 * dt, Nt > 0 ? coef_field : 0.0), sh, s);
  for (int64_t step = 1; step <= Nt; ++step) {                                        // :98
    // :105-107 update_H_BdG! + diagonalize + compute_forces!, then the kick of
    // :111-113 (dt) and the next step's drift (:101), or the final half kick
    // of :118 on the last step
    factorize_enqueue(ctx, step < Nt ? kickdrift(ctx, dt, coef_field) : kickdrift(ctx, 0.5 * dt, 0.0));
  }
  if (Nt <= 0)
    dwh::launch_force_from_pair(d, ctx->Pair, ctx->Delta, ctx->F, ctx->Pi, kickdrift(ctx, 0.5 * dt, 0.0),
                                ctx->beta, ctx->J, s);
  else
    fermion_energy_enqueue(ctx);
  if (with_hnew)
    dwh::launch_total_energy(d, ctx->Delta, ctx->Pi, ctx->Ef, ctx->beta, ctx->J, mass,  // :122
                             ctx->Hnew, s);
}

// One hmc_sweep! body (src/HMC.jl:71-144): trajectory, Metropolis, restore.
void sweep_enqueue(dwh_ctx* ctx, const double2* noise, const double* uniform, uint8_t* acc,
                   double* dH, int64_t Nt, double dt, double mass, const dwh::SweepHalt& sh = dwh::SweepHalt{}) {
  const Dims& d = ctx->d;
  hipStream_t s = ctx->stream;
  trajectory_enqueue(ctx, noise, Nt, dt, mass, false, sh);
  // :122 H_new, :124-129 Metropolis, :130-141 restore: one launch
  dwh::launch_traj_end(d, ctx->Delta, ctx->Pi, ctx->Pair, ctx->Ef, ctx->Trhh, ctx->DeltaB, ctx->PairB, ctx->EfB,
                       ctx->TrhhB, ctx->Hold, ctx->Hnew, uniform, acc, dH, ctx->beta, ctx->J, mass, sh, s);
}

// Spectral radius of the static particle block h of one chain (real
// symmetric, rows hrow + diagonal w_i - mu), by Lanczos with full
// reorthogonalisation from a fixed pseudo-random start: the extreme Ritz
// values converge first; the returned bound adds the residual |β s_m| of the
// extreme Ritz pairs and a 2 % margin.  For
// N <= the step count the Krylov space is all of R^N and the Ritz values are
// the spectrum.  The caller takes min(this, the Gershgorin bound).
double spectral_radius_bound(const std::vector<std::vector<std::pair<int, double>>>& hrow,
                             const double* diag, int N) {
  const int k = std::min(N, 160);
  std::vector<std::vector<double>> Q;
  std::vector<double> alpha, beta;
  std::vector<double> q(N), w(N);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  double nrm = 0;
  for (int i = 0; i < N; ++i) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    q[i] = (double)(st >> 11) * 0x1.0p-53 - 0.5;
    nrm += q[i] * q[i];
  }
  for (double& x : q) x /= std::sqrt(nrm);
  double bnext = 0;
  for (int j = 0; j < k; ++j) {
    Q.push_back(q);
    for (int i = 0; i < N; ++i) {
      double v = diag[i] * q[i];
      for (const auto& e : hrow[i]) v += e.second * q[e.first];
      w[i] = v;
    }
    double a = 0;
    for (int i = 0; i < N; ++i) a += w[i] * q[i];
    alpha.push_back(a);
    for (int pass = 0; pass < 2; ++pass)
      for (const auto& qq : Q) {
        double c = 0;
        for (int i = 0; i < N; ++i) c += w[i] * qq[i];
        for (int i = 0; i < N; ++i) w[i] -= c * qq[i];
      }
    double b = 0;
    for (int i = 0; i < N; ++i) b += w[i] * w[i];
    b = std::sqrt(b);
    bnext = b;
    if (j + 1 == k || b < 1e-12) break;
    beta.push_back(b);
    for (int i = 0; i < N; ++i) q[i] = w[i] / b;
  }
  // extreme eigenvalues of the tridiagonal T by bisection on Sturm counts
  const int m = (int)alpha.size();
  double lo = 0, hi = 0;
  for (int i = 0; i < m; ++i) {
    const double r = (i > 0 ? std::fabs(beta[i - 1]) : 0.0) + (i + 1 < m ? std::fabs(beta[i]) : 0.0);
    lo = std::min(lo, alpha[i] - r);
    hi = std::max(hi, alpha[i] + r);
  }
  auto count_below = [&](double x) {   // eigenvalues of T < x
    int c = 0;
    double d = 1.0;
    for (int i = 0; i < m; ++i) {
      d = alpha[i] - x - (i > 0 ? beta[i - 1] * beta[i - 1] / d : 0.0);
      if (d == 0.0) d = 1e-300;
      if (d < 0) ++c;
    }
    return c;
  };
  auto kth = [&](int idx) {   // idx-th smallest (0-based)
    double a = lo, b = hi;
    for (int it = 0; it < 200 && b - a > 1e-13 * std::max(1.0, std::fabs(b)); ++it) {
      const double mid = 0.5 * (a + b);
      if (count_below(mid) > idx) b = mid;
      else a = mid;
    }
    return b;
  };
  // residual of the Ritz pair (θ, Q s) is |β_m s_m|: last component of the
  // eigenvector s of T for θ, by inverse iteration on the tridiagonal system
  auto resid_of = [&](double th) {
    if (m == N) return 0.0;
    std::vector<double> x(m, 1.0), c(m), d(m), y(m);
    const double sh = th + 1e-10 * std::max(1.0, std::fabs(th));
    for (int it = 0; it < 3; ++it) {
      // Thomas solve (T - sh I) y = x
      for (int i = 0; i < m; ++i) {
        const double b = alpha[i] - sh - (i > 0 ? beta[i - 1] * c[i - 1] : 0.0);
        const double bb = (b == 0.0) ? 1e-300 : b;
        c[i] = (i + 1 < m) ? beta[i] / bb : 0.0;
        d[i] = (x[i] - (i > 0 ? beta[i - 1] * d[i - 1] : 0.0)) / bb;
      }
      y[m - 1] = d[m - 1];
      for (int i = m - 2; i >= 0; --i) y[i] = d[i] - c[i] * y[i + 1];
      double n2 = 0;
      for (double v : y) n2 += v * v;
      const double inv = 1.0 / std::sqrt(n2);
      for (int i = 0; i < m; ++i) x[i] = y[i] * inv;
    }
    return std::fabs(bnext * x[m - 1]);
  };
  const double tmin = kth(0), tmax = kth(m - 1);
  const double rho = std::max(std::fabs(tmin) + resid_of(tmin), std::fabs(tmax) + resid_of(tmax));
  return 1.02 * rho + 1e-12;
}

// Certifies rho >= ‖h‖ for the real symmetric h (off-diagonal hrow, diagonal
// diag): rho I - h and rho I + h are positive definite iff every pivot of
// their LDLᵀ factorisations is > 0 (Sylvester's law of inertia), so a
// Lanczos estimate that missed an eigenvalue fails here.  Band LDLᵀ in the
// folded row order (lattice rows 0, Ly-1, 1, Ly-2, ...: with the periodic
// corner folded in, the lattice couplings lie within 3 Lx - 1 of the
// diagonal), O(N b²); a bandwidth over 512 (a table that is not a lattice of
// rows) is not certified and the caller keeps the Gershgorin bound.
bool certify_spectral_bound(const std::vector<std::vector<std::pair<int, double>>>& hrow, const double* diag,
                            int N, int Lx, int Ly, double rho) {
  auto pos = [&](int i) {
    const int x = i % Lx, y = i / Lx;
    const int f = 2 * y < Ly ? 2 * y : 2 * (Ly - 1 - y) + 1;
    return f * Lx + x;
  };
  std::vector<int> p(N), inv(N);
  int b = 0;
  for (int i = 0; i < N; ++i) {
    p[i] = pos(i);
    inv[p[i]] = i;
  }
  for (int i = 0; i < N; ++i)
    for (const auto& e : hrow[i]) b = std::max(b, std::abs(p[i] - p[e.first]));
  if (b > 512) return false;
  const size_t W = (size_t)b + 1;
  std::vector<double> A((size_t)N * W), Lw((size_t)N * W), d(N);
  for (int sgn = -1; sgn <= 1; sgn += 2) {   // rho I + sgn h
    std::fill(A.begin(), A.end(), 0.0);
    for (int k = 0; k < N; ++k) {   // row k of the lower band: A[k][k - j] at k * W + j
      const int i = inv[k];
      A[(size_t)k * W] = rho + sgn * diag[i];
      for (const auto& e : hrow[i]) {
        const int c = p[e.first];
        if (c < k) A[(size_t)k * W + (k - c)] += sgn * e.second;
      }
    }
    // L[k][j] d[j] kept as Lw (the row's W entries), L[k][j] recovered on use
    for (int k = 0; k < N; ++k) {
      const int j0 = std::max(0, k - b);
      double dk = A[(size_t)k * W];
      for (int j = j0; j < k; ++j) {
        // s = A[k][j] - Σ_{i < j} L[k][i] d[i] L[j][i]
        double sacc = A[(size_t)k * W + (k - j)];
        const int i0 = std::max(j0, j - b);
        for (int i = i0; i < j; ++i)
          sacc -= Lw[(size_t)k * W + (k - i)] * (Lw[(size_t)j * W + (j - i)] / d[i]);
        Lw[(size_t)k * W + (k - j)] = sacc;   // = L[k][j] d[j]
        dk -= sacc * sacc / d[j];
      }
      if (!(dk > 0)) return false;
      d[k] = dk;
    }
  }
  return true;
}

// Default guard cap.  Bond guard (max|Δ_ij| <= cap): 2 (the ordered phase), or
// 6 standard deviations of the Gaussian boson fluctuations <|Δ|²> = 2J/β at
// high temperature.  Site guard (the mean of |Δ| over each site's four bonds
// <= cap, CR path: its level-0 inversion launch checks it): max(1.25, 4 sqrt(2J/β)) — the same ≈ 1.6x
// margin over the largest value thermalised L = 32 chains reach (site mean
// 0.79 / 1.08 / 1.49 at β = 16 / 8 / 4 over 300 sweeps against max|Δ_ij|
// 1.27 / 1.78 / 2.49, tools/delta_stats.py, profiles/r02_delta_stats.txt).
// Either way the pairing block's norm is at most its max row sum <= 2 cap.
double default_delta_cap(double beta, double J, bool site_guard) {
  const double s = std::sqrt(2.0 * std::fabs(J) / beta);
  return site_guard ? std::max(1.25, 4.0 * s) : std::max(2.0, 6.0 * s);
}

// ‖h‖ bound over the chains: min(Gershgorin, Lanczos) when every chain's
// h certifies the Lanczos value, else Gershgorin
double h_norm_bound(const std::vector<std::vector<std::pair<int, double>>>& hrow, const double* disorder, double mu,
                    int N, int Lx, int Ly, int64_t nchains, double gersh, double* lanczos = nullptr,
                    bool* certified = nullptr) {
  double rho = 0;
  std::vector<double> diag(N);
  for (int64_t c = 0; c < nchains; ++c) {
    for (int i = 0; i < N; ++i) diag[i] = disorder[c * (int64_t)N + i] - mu;
    rho = std::max(rho, spectral_radius_bound(hrow, diag.data(), N));
  }
  bool ok = rho < gersh;
  for (int64_t c = 0; c < nchains && ok; ++c) {
    for (int i = 0; i < N; ++i) diag[i] = disorder[c * (int64_t)N + i] - mu;
    ok = certify_spectral_bound(hrow, diag.data(), N, Lx, Ly, rho);
  }
  if (lanczos) *lanczos = rho;
  if (certified) *certified = ok;
  return ok ? rho : gersh;
}

// static h (off-diagonal rows): the reference's upper-triangle loop with
// overwrite (Hamiltonian.jl:26-44), nnn after nn
std::vector<std::vector<std::pair<int, double>>> build_hrow(int N, double t, double tp, const int64_t* nn,
                                                            const int64_t* nnn) {
  auto NN = [&](int i, int dir) { return (int)(nn[(int64_t)dir * N + i] - 1); };
  auto NNN = [&](int i, int dir) { return (int)(nnn[(int64_t)dir * N + i] - 1); };
  std::map<std::pair<int, int>, double> up;
  for (int i = 0; i < N; ++i) {
    for (int dir = 0; dir < 4; ++dir) {
      const int j = NN(i, dir);
      if (j > i) up[{i, j}] = -t;
    }
    for (int dir = 0; dir < 4; ++dir) {
      const int j = NNN(i, dir);
      if (j > i) up[{i, j}] = -tp;
    }
  }
  std::vector<std::vector<std::pair<int, double>>> hrow(N);
  for (auto& kv : up) {
    hrow[kv.first.first].push_back({kv.first.second, kv.second});
    hrow[kv.first.second].push_back({kv.first.first, kv.second});
  }
  return hrow;
}

int create_impl(dwh_ctx** out, int64_t Lx, int64_t Ly, double t, double tp, double mu, double beta,
                double J, const int64_t* nn, const int64_t* nnn, int64_t nchains,
                const double* disorder, double delta_cap, int32_t algo_req, int32_t device) {
  if (!out) return fail(nullptr, DWH_ERR_ARG, "ctx pointer is NULL");
  *out = nullptr;
  if (Lx < 1 || Ly < 1) return fail(nullptr, DWH_ERR_ARG, "Lx, Ly must be >= 1");
  if (!(beta > 0)) return fail(nullptr, DWH_ERR_ARG, "beta must be > 0");
  if (J == 0 || !std::isfinite(J)) return fail(nullptr, DWH_ERR_ARG, "J must be finite and nonzero");
  if (nchains < 1) return fail(nullptr, DWH_ERR_ARG, "nchains must be >= 1");
  if (!nn || !nnn || !disorder) return fail(nullptr, DWH_ERR_ARG, "NULL table or disorder");
  const int64_t N64 = Lx * Ly;
  if (N64 > 9216) return fail(nullptr, DWH_ERR_ARG, "N = Lx*Ly > 9216 not supported (LDS row staging)");
  const int N = (int)N64;
  for (int64_t e = 0; e < 4 * N64; ++e)
    if (nn[e] < 1 || nn[e] > N64 || nnn[e] < 1 || nnn[e] > N64)
      return fail(nullptr, DWH_ERR_ARG, "neighbour table entry out of [1, N]");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return fail(nullptr, DWH_ERR_HIP, "no HIP device available (the fermion path has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(nullptr, DWH_ERR_ARG, "device index out of range");

  auto NN = [&](int i, int dir) { return (int)(nn[(int64_t)dir * N + i] - 1); };
  auto NNN = [&](int i, int dir) { return (int)(nnn[(int64_t)dir * N + i] - 1); };

  // --- static h: reference upper-triangle loop with overwrite (Hamiltonian.jl:26-44)
  const std::vector<std::vector<std::pair<int, double>>> hrow = build_hrow(N, t, tp, nn, nnn);
  std::vector<int> hcol((size_t)N * kHSlots, -1);
  std::vector<double> hval((size_t)nchains * N * kHSlots, 0.0);
  double hmax = 0;
  for (int i = 0; i < N; ++i) {
    if ((int)hrow[i].size() + 1 > kHSlots)
      return fail(nullptr, DWH_ERR_ARG, "more than 8 hopping partners per site");
    hcol[(size_t)i * kHSlots] = i;
    double off = 0;
    for (size_t s = 0; s < hrow[i].size(); ++s) {
      hcol[(size_t)i * kHSlots + 1 + s] = hrow[i][s].first;
      off += std::fabs(hrow[i][s].second);
    }
    for (int64_t c = 0; c < nchains; ++c) {
      const double w = disorder[c * N64 + i];
      if (!std::isfinite(w)) return fail(nullptr, DWH_ERR_ARG, "non-finite disorder");
      hval[((size_t)c * N + i) * kHSlots] = w - mu;  // Hamiltonian.jl:18-22
      for (size_t s = 0; s < hrow[i].size(); ++s)
        hval[((size_t)c * N + i) * kHSlots + 1 + s] = hrow[i][s].second;
      hmax = std::max(hmax, std::fabs(w - mu) + off);
    }
  }
  // --- pairing pattern with the reference overwrite order (Hamiltonian.jl:68-83)
  std::map<std::pair<int, int>, int> dmap;
  for (int i = 0; i < N; ++i)
    for (int dir = 0; dir < 2; ++dir) {
      const int j = NN(i, dir);
      const int src = i + N * dir;
      dmap[{i, j}] = src;
      dmap[{j, i}] = src;
    }
  std::vector<int> Dcol((size_t)N * kSlots, -1), Dsrc((size_t)N * kSlots, -1);
  std::vector<int> dcount(N, 0);
  for (auto& kv : dmap) {
    const int r = kv.first.first;
    if (dcount[r] >= kSlots) return fail(nullptr, DWH_ERR_ARG, "more than 4 pairing partners per site");
    Dcol[(size_t)r * kSlots + dcount[r]] = kv.first.second;
    Dsrc[(size_t)r * kSlots + dcount[r]] = kv.second;
    dcount[r]++;
  }
  for (auto& kv : dmap) {
    auto it = dmap.find({kv.first.second, kv.first.first});
    if (it == dmap.end() || it->second != kv.second)
      return fail(nullptr, DWH_ERR_ARG, "pairing block not symmetric (unsupported table)");
  }
  auto slot_of = [&](int r, int c) {
    for (int s = 0; s < kSlots; ++s)
      if (Dcol[(size_t)r * kSlots + s] == c) return s;
    return -1;
  };
  std::vector<int> bij(2 * (size_t)N), bji(2 * (size_t)N);
  for (int dir = 0; dir < 2; ++dir)
    for (int i = 0; i < N; ++i) {
      const int j = NN(i, dir);
      const int sij = slot_of(i, j), sji = slot_of(j, i);
      if (sij < 0 || sji < 0) return fail(nullptr, DWH_ERR_ARG, "bond missing from the pairing pattern");
      bij[(size_t)dir * N + i] = i * kSlots + sij;
      bji[(size_t)dir * N + i] = j * kSlots + sji;
    }

  // --- pole selection: E' >= ‖H_BdG‖ <= ‖h‖ + ‖pairing block‖ with
  // ‖h‖ <= min(Gershgorin, Lanczos bound) and the pairing block's norm <= its
  // max row sum Σ_j |Δ_ij|/2 <= 2 delta_cap (bond guard: each of the 4 bonds
  // <= cap; site guard: their mean <= cap)
  // (the Lanczos bound only where certified, certify_spectral_bound)
  hmax = h_norm_bound(hrow, disorder, mu, N, (int)Lx, (int)Ly, nchains, hmax);
  // algorithm: explicit request, else DWHMC_ALGO = dense | cr | eig | auto
  // (auto: cr when the lattice-row block 2 Lx fits a supported padded size,
  // else dense; eig when κ = β E'/2 is beyond the pole table)
  std::string want = "auto";
  if (algo_req == DWH_ALGO_DENSE) want = "dense";
  else if (algo_req == DWH_ALGO_CR) want = "cr";
  else if (algo_req == DWH_ALGO_EIG) want = "eig";
  else if (const char* e = std::getenv("DWHMC_ALGO")) want = e;
  if (want != "auto" && want != "dense" && want != "cr" && want != "eig")
    return fail(nullptr, DWH_ERR_ARG, "DWHMC_ALGO must be auto, dense, cr or eig");
  // site guard on the CR path (checked by its level-0 inversion launch)
  const bool site_guard = [&] {
    const int BPc = (int)(2 * ((Lx + 15) / 16 * 16));
    return want == "cr" || (want == "auto" && dwh::cr_supported_bp(BPc));
  }();
  if (delta_cap <= 0) delta_cap = default_delta_cap(beta, J, site_guard);
  const double Eb = hmax + 2.0 * delta_cap;
  const double kneed = 0.5 * beta * Eb;
  std::string terr;
  const PoleTable* tab = pole_table(&terr);
  if (!tab) return fail(nullptr, DWH_ERR_ARG, terr);
  int sel = -1;
  for (int e = 0; e < tab->size; ++e)
    if (tab->at(e).kappa >= kneed * (1.0 - 1e-12)) {
      sel = e;
      break;
    }
  if (sel < 0 && want == "auto") want = "eig";
  if (sel < 0 && want != "eig") {
    char buf[256];
    std::snprintf(buf, sizeof buf, "beta*E_bound/2 = %g exceeds the pole table (max kappa %g)", kneed,
                  tab->at(tab->size - 1).kappa);
    return fail(nullptr, DWH_ERR_TABLE, buf);
  }
  const bool eig = want == "eig";
  // the eigen path is exact for any Δ: no pole set, no |Δ| guard
  if (eig) delta_cap = std::numeric_limits<double>::max();
  const PoleView pv = eig ? PoleView{} : tab->at(sel);
  const PoleView* pe = eig ? nullptr : &pv;
  const double kappa = eig ? kneed : pe->kappa;
  const double Ep = eig ? Eb : 2.0 * kappa / beta;
  const int npole = eig ? 1 : pe->m;   // eig: one dummy batch item per chain
  std::vector<double> y(npole, 0.0), cq(npole, 0.0);
  double suma = 0;
  for (int q = 0; q < (eig ? 0 : npole); ++q) {
    y[q] = Ep * std::sqrt(pe->t[q]);
    cq[q] = 0.5 * pe->a[q] * Ep;
    suma += pe->a[q];
  }

  dwh_ctx* ctx = new dwh_ctx();
  ctx->nn_host.assign(nn, nn + 4 * N64);
  ctx->nnn_host.assign(nnn, nnn + 4 * N64);
  ctx->dis_host.assign(disorder, disorder + nchains * N64);
  ctx->device = device;
  ctx->Lx = Lx;
  ctx->Ly = Ly;
  ctx->t = t;
  ctx->tp = tp;
  ctx->mu = mu;
  ctx->beta = beta;
  ctx->J = J;
  ctx->delta_cap = delta_cap;
  ctx->site_guard = site_guard && !eig;
  // x-current operator J [src/Observables.jl:237-283]: i t at (i, i+x), i t' at
  // (i, i+x+y) and (i, i+x-y), plus their conjugate transposes, summed into CSR
  // (SparseArrays.sparse adds duplicates); stored as imaginary parts
  {
    std::vector<std::map<int, double>> jrow(N);
    ctx->tr_nbr.assign(3 * (size_t)N, 0);
    for (int i = 0; i < N; ++i) {
      const int js[3] = {NN(i, 0), NNN(i, 0), NNN(i, 3)};
      const double ts[3] = {t, tp, tp};
      for (int b = 0; b < 3; ++b) {
        jrow[i][js[b]] += ts[b];
        jrow[js[b]][i] -= ts[b];
        ctx->tr_nbr[(size_t)b * N + i] = js[b];
      }
    }
    ctx->tr_rowptr.assign(N + 1, 0);
    for (int r = 0; r < N; ++r) {
      for (auto& kv : jrow[r]) {
        ctx->tr_col.push_back(kv.first);
        ctx->tr_val.push_back(kv.second);
      }
      ctx->tr_rowptr[r + 1] = (int)ctx->tr_col.size();
    }
  }
  ctx->kappa = kappa;
  ctx->Ebound = Ep;
  ctx->hmax = hmax;
  ctx->err_tanh = eig ? 0.0 : pe->err_tanh;
  ctx->Cx = eig ? 0.0 : pe->C_u - kappa * std::log(Ep) * suma;
  ctx->y = y;
  ctx->cq = cq;
  Dims& d = ctx->d;
  d.N = N;
  d.Np = ((N + kGJ - 1) / kGJ) * kGJ;
  d.nb = d.Np / kGJ;
  d.nc = (int)nchains;
  d.P = npole;
  d.nbatch = d.nc * d.P;
  d.mat = (int64_t)d.Np * d.Np;
  d.nld = d.nb;
  {
    const bool ok = dwh::cr_supported_bp((int)(2 * ((Lx + 15) / 16 * 16)));
    // the CR lattice: R lattice rows per block (cr_rows_per_block)
    const int rows = ok ? cr_rows_per_block(Lx, Ly) : 1;
    const int Lxc = (int)Lx * rows, Lyc = (int)Ly / rows;
    const int BP = 2 * ((Lxc + 15) / 16 * 16);   // top halves HP x BP, HP = Lxc rounded to 16
    if (want == "cr" && !ok) {
      ctx->err = "DWHMC_ALGO=cr needs 2*Lx <= 128";
      g_create_error = ctx->err;
      delete ctx;
      return DWH_ERR_ARG;
    }
    ctx->algo = eig ? ALGO_EIG : (want == "dense" || !ok) ? ALGO_DENSE : ALGO_CR;
    if (ctx->algo == ALGO_CR) {
      // DWHMC_CR_SIDE=0: every product on its own stage (A/B runs, tests)
      const char* es = std::getenv("DWHMC_CR_SIDE");
      const bool side = dwh::cr_supported_side(BP) && !(es && *es == '0');
      int ncu = 256;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
        ncu = 256;
      // DWHMC_CR_INV0=0: level-0 blocks inverted whole (k_cr_inv) like the rest
      const char* e0 = std::getenv("DWHMC_CR_INV0");
      const bool inv0 = dwh::cr_supported_inv0(BP) && !(e0 && *e0 == '0');
      ctx->plan = build_cr_plan(Lxc, Lyc, BP, Dcol, side, d.nbatch, ncu, inv0, &hcol);
      dwh::CrDims& c = ctx->cr;
      c.Lx = Lxc;
      c.Ly = Lyc;
      c.N = N;
      c.BP = BP;
      c.P = d.P;
      c.nbatch = d.nbatch;
      c.nblk = ctx->plan.nblk;
      c.item = (int64_t)c.nblk * (BP / 2) * BP;
      // DWHMC_CR_INV32=0: BP = 32 inversions by k_cr_inv<2> (A/B knob)
      const char* e32 = std::getenv("DWHMC_CR_INV32");
      c.inv32 = !(e32 && *e32 == '0');
      d.nld = Lyc;
      if ((uint64_t)c.item >= (uint64_t)dwh::kCrNone) {
        ctx->err = "CR pool: a batch item exceeds 2^32 elements (32-bit block-product offsets)";
        g_create_error = ctx->err;
        delete ctx;
        return DWH_ERR_ARG;
      }
      CrPlan& pl = ctx->plan;
      pl.slots.clear();
      for (CrStage& st : pl.stages) {
        if (st.kind != 1) continue;
        st.cfg = dwh::cr_gemm_config(c, st.n, st.maxt32, st.maxt16, st.ntmax, st.ntiles);
        if (st.cfg.ts != 16) continue;
        st.nswg = dwh::cr_gemm_slot_wgs(c, st.ntiles, st.cfg);
        st.sfirst = (int)pl.slots.size();
        pl.slots.resize(pl.slots.size() + (size_t)st.nswg * (4 / st.cfg.ksplit));
        dwh::cr_gemm_slots(c, pl.tiles16.data() + st.tfirst, st.ntiles, st.cfg, pl.slots.data() + st.sfirst);
      }
      if (const char* e = std::getenv("DWHMC_CR_PLAN_DUMP"); e && *e == '1') {
        int i = 0;
        for (const CrStage& st : ctx->plan.stages) {
          if (st.kind == 0)
            std::fprintf(stderr, "cr stage %2d: inv%s blocks=%d side_tasks=%d side_flops/item=%.3g\n", i,
                         st.l0 ? "0 " : "  ", st.n, st.ntiles, st.flops);
          else if (st.kind == 2)
            std::fprintf(stderr, "cr stage %2d: sparse %s tasks=%d flops/item=%.3g\n", i, st.sp ? "bwd" : "fwd", st.n,
                         st.flops);
          else
            std::fprintf(stderr, "cr stage %2d: gemm  tasks=%d maxt32=%d maxt16=%d ntmax=%d flops/item=%.3g cfg=%d:%d ntiles=%d\n",
                         i, st.n, st.maxt32, st.maxt16, st.ntmax, st.flops, st.cfg.ts, st.cfg.ksplit, st.ntiles);
          ++i;
        }
      }
    }
  }

  auto bail = [&](int code) {
    g_create_error = ctx->err;
    dwh_destroy(ctx);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) {
    ctx->err = "hipSetDevice failed";
    return bail(DWH_ERR_HIP);
  }
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    ctx->err = "hipStreamCreate failed";
    return bail(DWH_ERR_HIP);
  }
  const size_t nmat = (size_t)d.nbatch * d.mat;
  const size_t nbond = (size_t)d.nc * 2 * N;
  int rc = DWH_OK;
#define ALLOC(p, n) \
  if ((rc = dalloc(ctx, &ctx->p, (n))) != DWH_OK) return bail(rc)
  if (ctx->algo == ALGO_DENSE) {
    ALLOC(R, nmat);
    ALLOC(S, nmat);
    const size_t npanel = (size_t)d.nbatch * d.Np * kGJ;
    ALLOC(CpA0, npanel);
    ALLOC(CpA1, npanel);
    ALLOC(CpB, npanel);
    ALLOC(XR1, npanel);
    ALLOC(XR2, npanel);
    ALLOC(Pb1, (size_t)d.nbatch * kGJ * kGJ);
    ALLOC(Pb2, (size_t)d.nbatch * kGJ * kGJ);
  } else if (ctx->algo == ALGO_CR) {
    const CrPlan& pl = ctx->plan;
    ALLOC(bpool, (size_t)d.nbatch * ctx->cr.item);
    ALLOC(d_tasks, pl.tasks.size());
    ALLOC(d_slots, pl.slots.size());
    ALLOC(d_sp_fwd, pl.sp_fwd.size());
    ALLOC(d_sp_bwd, pl.sp_bwd.size());
    if (!pl.colpat.empty()) {
      std::vector<double2> colval;
      std::vector<int> colsrc;
      cr_sparse_colvals(pl.colpat, ctx->cr.Lx, ctx->cr.Ly, ctx->cr.BP, hcol, hval, Dcol, Dsrc, colval, colsrc);
      ctx->sp_arr = cr_sparse_task_arrays(pl, ctx->cr.BP, colval, colsrc);
    }
    ALLOC(d_sp_row, ctx->sp_arr.row.size());
    ALLOC(d_sp_cv, ctx->sp_arr.cv.size());
    ALLOC(d_sp_cm, ctx->sp_arr.cm.size());
    ALLOC(efpart, 2 * (size_t)d.nbatch);
    ALLOC(efdone, (size_t)d.nc);
    ALLOC(d_inv_blk, pl.inv_blk.size());
    ALLOC(d_inv_dst, pl.inv_dst.size());
    ALLOC(d_inv_slot, pl.inv_slot.size());
    ALLOC(d_inv0_r, pl.inv0_r.size());
    ALLOC(ldA, (size_t)d.nbatch * ctx->cr.Ly);
    ALLOC(d_doff, pl.doff.size());
    ALLOC(d_off_ph, pl.off_ph.size());
    ALLOC(d_bond4, 4 * bij.size());
    ALLOC(d_fill_all, pl.fill_all.size());
    ALLOC(d_fill_step, pl.fill_step.size());
  }
  if (ctx->algo == ALGO_DENSE) {
    ALLOC(Dv, (size_t)d.nc * N * kSlots);
    ALLOC(G12nn, (size_t)d.nbatch * N * kSlots);
    ALLOC(diagS, (size_t)d.nbatch * N);
  }
  ALLOC(ldpart, (size_t)d.nbatch * d.nld);
  ALLOC(ldstatic, (size_t)d.nbatch);
  ALLOC(d_y, (size_t)d.P);
  ALLOC(d_c, (size_t)d.P);
  ALLOC(Dcol, Dcol.size());
  ALLOC(Dsrc, Dsrc.size());
  ALLOC(hcol, hcol.size());
  ALLOC(hval, hval.size());
  ALLOC(bond_ij, bij.size());
  ALLOC(bond_ji, bji.size());
  ALLOC(Delta, nbond);
  ALLOC(Pi, nbond);
  ALLOC(Pair, nbond);
  ALLOC(F, nbond);
  ALLOC(DeltaB, nbond);
  ALLOC(PairB, nbond);
  ALLOC(Ef, (size_t)d.nc);
  ALLOC(EfB, (size_t)d.nc);
  ALLOC(Trhh, (size_t)d.nc);
  ALLOC(TrhhB, (size_t)d.nc);
  ALLOC(Hold, (size_t)d.nc);
  ALLOC(Hnew, (size_t)d.nc);
  ALLOC(flag, 1);
  ALLOC(halt, 2);
  if (ctx->site_guard) ALLOC(site4, 4 * (size_t)N);
  ALLOC(s_noise, nbond);
  ALLOC(s_uniform, (size_t)d.nc);
  ALLOC(s_acc, (size_t)d.nc);
  ALLOC(s_dH, (size_t)d.nc);
#undef ALLOC
  ctx->ndraws = 0;
  hipStream_t s = ctx->stream;
#define UP(dst, src, n)                                                                     \
  if ((n) > 0 && hipMemcpyAsync(ctx->dst, (src), (n) * sizeof(*ctx->dst), hipMemcpyHostToDevice, s) != \
      hipSuccess) {                                                                         \
    ctx->err = "upload " #dst;                                                              \
    return bail(DWH_ERR_HIP);                                                               \
  }
  UP(d_y, y.data(), y.size());
  UP(d_c, cq.data(), cq.size());
  UP(Dcol, Dcol.data(), Dcol.size());
  UP(Dsrc, Dsrc.data(), Dsrc.size());
  UP(hcol, hcol.data(), hcol.size());
  UP(hval, hval.data(), hval.size());
  UP(bond_ij, bij.data(), bij.size());
  UP(bond_ji, bji.data(), bji.size());
  if (ctx->site_guard) {
    // site i: bonds (i, +x), (i, +y), (i - x, +x), (i - y, +y) in the N x 2 Δ layout
    ctx->site4_host.resize(4 * (size_t)N);
    for (int i = 0; i < N; ++i) {
      ctx->site4_host[4 * i + 0] = i;
      ctx->site4_host[4 * i + 1] = N + i;
      ctx->site4_host[4 * i + 2] = (int)(nn[2 * N64 + i] - 1);
      ctx->site4_host[4 * i + 3] = N + (int)(nn[3 * N64 + i] - 1);
    }
    UP(site4, ctx->site4_host.data(), ctx->site4_host.size());
  }
  // per bond b (2N of them, CR path): G12[i, j], G12[j, i] and the pairing
  // entries it writes (Dsrc picks the bond whose value an entry holds); kept
  // alive until the uploads below have been synchronised
  std::vector<int64_t> bond4;
  if (ctx->algo == ALGO_CR) {
    const CrPlan& pl = ctx->plan;
    bond4.resize(4 * bij.size());
    for (size_t b = 0; b < bij.size(); ++b) {
      const int e1 = bij[b], e2 = bji[b];
      bond4[4 * b] = pl.goff[e1];
      bond4[4 * b + 1] = pl.goff[e2];
      bond4[4 * b + 2] = Dsrc[e1] == (int)b ? pl.off_ph[e1] : -1;
      bond4[4 * b + 3] = Dsrc[e2] == (int)b ? pl.off_ph[e2] : -1;
    }
  }
  if (ctx->algo == ALGO_CR) {
    const CrPlan& pl = ctx->plan;
    UP(d_tasks, pl.tasks.data(), pl.tasks.size());
    UP(d_slots, pl.slots.data(), pl.slots.size());
    UP(d_sp_fwd, pl.sp_fwd.data(), pl.sp_fwd.size());
    UP(d_sp_bwd, pl.sp_bwd.data(), pl.sp_bwd.size());
    UP(d_sp_row, ctx->sp_arr.row.data(), ctx->sp_arr.row.size());
    UP(d_sp_cv, ctx->sp_arr.cv.data(), ctx->sp_arr.cv.size());
    UP(d_sp_cm, ctx->sp_arr.cm.data(), ctx->sp_arr.cm.size());
    UP(d_inv_blk, pl.inv_blk.data(), pl.inv_blk.size());
    UP(d_inv_dst, pl.inv_dst.data(), pl.inv_dst.size());
    UP(d_inv_slot, pl.inv_slot.data(), pl.inv_slot.size());
    UP(d_inv0_r, pl.inv0_r.data(), pl.inv0_r.size());
    UP(d_doff, pl.doff.data(), pl.doff.size());
    UP(d_off_ph, pl.off_ph.data(), pl.off_ph.size());
    UP(d_bond4, bond4.data(), bond4.size());
    UP(d_fill_all, pl.fill_all.data(), pl.fill_all.size());
    UP(d_fill_step, pl.fill_step.data(), pl.fill_step.size());
  }
#undef UP
  // zeroed cache, like initialize_cache (src/Types.jl:182-212): P = 0, E_f = 0
  (void)hipMemsetAsync(ctx->Delta, 0, nbond * sizeof(double2), s);
  if (ctx->efdone) (void)hipMemsetAsync(ctx->efdone, 0, (size_t)d.nc * sizeof(unsigned), s);
  (void)hipMemsetAsync(ctx->Pi, 0, nbond * sizeof(double2), s);
  (void)hipMemsetAsync(ctx->Pair, 0, nbond * sizeof(double2), s);
  (void)hipMemsetAsync(ctx->F, 0, nbond * sizeof(double2), s);
  (void)hipMemsetAsync(ctx->Ef, 0, d.nc * sizeof(double), s);
  (void)hipMemsetAsync(ctx->Trhh, 0, d.nc * sizeof(double), s);
  (void)hipMemsetAsync(ctx->flag, 0, sizeof(int), s);
  (void)hipMemsetAsync(ctx->halt, 0, 2 * sizeof(int), s);
  if (ctx->diagS) (void)hipMemsetAsync(ctx->diagS, 0, (size_t)d.nbatch * N * sizeof(double2), s);
  if (ctx->algo == ALGO_DENSE) {
    // static R = (h - i y)^-1 and ln|det(h - i y)| for every (chain, pole)
    dwh::launch_fill_hz(d, ctx->R, ctx->hcol, ctx->hval, ctx->d_y, s);
    run_gj(ctx, ctx->R);
    dwh::launch_sum_ld(d, ctx->ldpart, ctx->ldstatic, s);
  } else if (ctx->algo == ALGO_CR) {
    // the CR path factorises the whole BdG matrix: no static part; every
    // level-0 block written once (pairing entries 0 until the first factorize)
    (void)hipMemsetAsync(ctx->ldstatic, 0, d.nbatch * sizeof(double), s);
    dwh::launch_cr_fill(ctx->cr, ctx->bpool, ctx->d_fill_all, (int)ctx->plan.fill_all.size(), ctx->hcol,
                        ctx->hval, ctx->Dcol, ctx->Dsrc, ctx->Delta, ctx->d_y, nullptr, s);
    // static R = A^-1 of the level-0 blocks k_cr_inv0 inverts: the Δ = 0
    // blocks [[A, 0], [0, -conj A]] inverted out of place give [R | 0] and
    // 2 ln|det A| (the pairing entries are still zero here)
    for (const CrStage& st : ctx->plan.stages)
      if (st.kind == 0 && st.l0)
        dwh::launch_cr_inv(ctx->cr, ctx->bpool, ctx->d_inv_blk + st.first, ctx->d_inv0_r, ctx->d_inv_slot + st.first,
                           st.n, ctx->ldA, s);
  }
  if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) {
    ctx->err = "static R initialisation failed on the device";
    return bail(DWH_ERR_HIP);
  }
  // eig: rocBLAS handle and the per-chain U, JU (= U diag f), ρ, E buffers
  if (ctx->algo == ALGO_EIG && (rc = transport_prepare(ctx, 0, 0, d.nc)) != DWH_OK) return bail(rc);
  *out = ctx;
  return DWH_OK;
}

// ---------------------------------------------------------------------------
// transport / spectra measurement (src/Observables.jl:314-526)
// ---------------------------------------------------------------------------

// length(start:step:stop) of the Julia float ranges of src/Observables.jl:395,430:
// the step count is rounded when (stop - start)/step is an integer up to
// rounding (Base.floatrange), else floored
int64_t julia_range_len(double start, double step, double stop) {
  const double r = (stop - start) / step;
  const double n = std::nearbyint(r);
  const double k = std::fabs(r - n) < 1e-8 * std::max(1.0, std::fabs(r)) ? n : std::floor(r);
  return k < 0 ? 0 : (int64_t)k + 1;
}

void drop_alloc(dwh_ctx* ctx, void* p) {
  if (!p) return;
  auto it = std::find(ctx->allocations.begin(), ctx->allocations.end(), p);
  if (it != ctx->allocations.end()) ctx->allocations.erase(it);
  (void)hipFree(p);
}

// device buffers + rocBLAS handle on first use.  Buffers hold `slots` chains
// (one slot per chain of a batched measurement), each slot laid out as
// TrBufs; the σ partials are shared (chains are reduced one after another).
int transport_prepare(dwh_ctx* ctx, int64_t nw, int64_t nd, int slots) {
  const int N = ctx->d.N;
  const size_t n2 = 2 * (size_t)N;
  dwh::TrBufs& b = ctx->tr;
  int rc = DWH_OK;
  if (!ctx->blas) {
    if (rocblas_create_handle(&ctx->blas) != rocblas_status_success)
      return fail(ctx, DWH_ERR_HIP, "rocblas_create_handle failed");
    if (rocblas_set_stream(ctx->blas, ctx->stream) != rocblas_status_success)
      return fail(ctx, DWH_ERR_HIP, "rocblas_set_stream failed");
    if ((rc = dalloc(ctx, &ctx->d_tr_nbr, ctx->tr_nbr.size())) ||
        (rc = dalloc(ctx, &ctx->d_tr_rowptr, ctx->tr_rowptr.size())) ||
        (rc = dalloc(ctx, &ctx->d_tr_col, ctx->tr_col.size())) ||
        (rc = dalloc(ctx, &ctx->d_tr_val, ctx->tr_val.size())) || (rc = dalloc(ctx, &ctx->d_tr_bad, 1)))
      return rc;
    auto up = [&](void* dst, const void* src, size_t bytes) {
      return bytes == 0 ? hipSuccess : hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream);
    };
    HIPCHECK(ctx, up(ctx->d_tr_nbr, ctx->tr_nbr.data(), ctx->tr_nbr.size() * sizeof(int)));
    HIPCHECK(ctx, up(ctx->d_tr_rowptr, ctx->tr_rowptr.data(), ctx->tr_rowptr.size() * sizeof(int)));
    HIPCHECK(ctx, up(ctx->d_tr_col, ctx->tr_col.data(), ctx->tr_col.size() * sizeof(int)));
    HIPCHECK(ctx, up(ctx->d_tr_val, ctx->tr_val.data(), ctx->tr_val.size() * sizeof(double)));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  }
  if (slots > ctx->tr_slots) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    for (void* q : {(void*)b.U, (void*)b.JU, (void*)b.Jmn, (void*)b.E, (void*)b.f, (void*)b.dia, (void*)b.Wn,
                    (void*)b.wan, (void*)b.w0, (void*)b.lam, (void*)b.dc, (void*)ctx->d_tr_offd, (void*)b.ak,
                    (void*)b.scalars, (void*)ctx->d_tr_info})
      drop_alloc(ctx, q);
    const size_t m = (size_t)slots;
    if ((rc = dalloc(ctx, &b.U, m * n2 * n2)) || (rc = dalloc(ctx, &b.JU, m * n2 * n2)) ||
        (rc = dalloc(ctx, &b.Jmn, m * n2 * n2)))
      return rc;
    for (double** q : {&b.E, &b.f, &b.dia, &b.Wn, &b.wan, &b.w0, &b.lam, &b.dc, &ctx->d_tr_offd})
      if ((rc = dalloc(ctx, q, m * n2))) return rc;
    if ((rc = dalloc(ctx, &b.ak, m * N)) || (rc = dalloc(ctx, &b.scalars, 2 * m)) ||
        (rc = dalloc(ctx, &ctx->d_tr_info, m)))
      return rc;
    ctx->tr_slots = slots;
    ctx->tr_nw = ctx->tr_nd = -1;   // per-slot outputs below are re-sized too
  }
  if (nw != ctx->tr_nw || nd != ctx->tr_nd) {
    // partials of the σ chunks and of the DOS slices (one after the other)
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    drop_alloc(ctx, b.part);
    drop_alloc(ctx, b.sigma);
    b.part = b.sigma = nullptr;
    const size_t np = std::max<size_t>((size_t)dwh::tr_sigma_chunks(N) * nw, (size_t)2 * dwh::tr_dos_slices(N) * nd);
    if ((rc = dalloc(ctx, &b.part, std::max<size_t>(np, 1))) ||
        (rc = dalloc(ctx, &b.sigma, (size_t)ctx->tr_slots * nw)))
      return rc;
    ctx->tr_nw = nw;
  }
  if (nd != ctx->tr_nd) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    drop_alloc(ctx, b.dos);
    drop_alloc(ctx, b.dos_an);
    b.dos = b.dos_an = nullptr;
    if ((rc = dalloc(ctx, &b.dos, (size_t)ctx->tr_slots * nd)) ||
        (rc = dalloc(ctx, &b.dos_an, (size_t)ctx->tr_slots * nd)))
      return rc;
    ctx->tr_nd = nd;
  }
  return DWH_OK;
}

// the buffers of slot k
dwh::TrBufs tr_slot(const dwh_ctx* ctx, int k) {
  const size_t n2 = 2 * (size_t)ctx->d.N, N = ctx->d.N;
  dwh::TrBufs b = ctx->tr;
  const size_t mat = n2 * n2 * k, vec = n2 * k;
  b.U += mat;
  b.JU += mat;
  b.Jmn += mat;
  for (double** q : {&b.E, &b.f, &b.dia, &b.Wn, &b.wan, &b.w0, &b.lam, &b.dc}) *q += vec;
  b.ak += N * k;
  b.scalars += 2 * k;
  b.sigma += (size_t)std::max<int64_t>(ctx->tr_nw, 0) * k;
  b.dos += (size_t)std::max<int64_t>(ctx->tr_nd, 0) * k;
  b.dos_an += (size_t)std::max<int64_t>(ctx->tr_nd, 0) * k;
  return b;
}

// dense H_BdG(Δ) of chains c0 .. c0+m-1 into slots 0 .. m-1 -> rocSOLVER zheevd
// (strided-batched for m > 1: its latency-bound panel kernels then cover every
// chain at once): eigenvalues ascending into E, eigenvectors into the columns
// of U (diagonalize_H_BdG!, src/Hamiltonian.jl:96-114; the reference's zheevr
// and zheevd agree to rounding)
TrSrc chains_src(const dwh_ctx* ctx, int64_t c0) {
  const int64_t n2 = 2 * (int64_t)ctx->d.N;
  return TrSrc{ctx->Delta + c0 * n2, n2, c0, 1};
}

// dense H_BdG(Δ) of the m slots' chains into A (m matrices at stride n2^2)
int assemble_slots(dwh_ctx* ctx, const TrSrc& src, int m, double2* A) {
  const int N = ctx->d.N;
  const int64_t sA = 4 * (int64_t)N * N;
  HIPCHECK(ctx, hipMemsetAsync(A, 0, (size_t)m * sA * sizeof(double2), ctx->stream));
  for (int k = 0; k < m; ++k)
    dwh::launch_tr_assemble(A + k * sA, N, ctx->hcol,
                            ctx->hval + (size_t)(src.chain0 + (int64_t)k * src.cstep) * N * kHSlots, ctx->Dcol,
                            ctx->Dsrc, src.Delta + (size_t)k * src.dstride, ctx->stream);
  HIPCHECK(ctx, hipGetLastError());
  return DWH_OK;
}

// The own eigensolver (dwhmc_eig.hip): H assembled into the slots' JU, reduced
// to tridiagonal form in place (JU becomes the reflectors V), eigenvalues by
// bisection into E, eigenvectors of T by inverse iteration (Jmn and U as
// scratch), then U = V-reflectors · Z by blocked compact-WY zgemms
// DWHMC_EIG_DEBUG=1: synchronise after each phase of the own solver and print
// its wall time to stderr (diagnosing a slow or stuck phase on the device)
struct EigPhase {
  bool on;
  hipStream_t s;
  std::chrono::steady_clock::time_point t;
  explicit EigPhase(hipStream_t st) : s(st), t(std::chrono::steady_clock::now()) {
    const char* e = std::getenv("DWHMC_EIG_DEBUG");
    on = e && *e == '1';
  }
  void mark(const char* what) {
    if (!on) return;
    const hipError_t err = hipStreamSynchronize(s);
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "eig phase %-14s %9.3f ms  %s\n", what,
                 std::chrono::duration<double, std::milli>(now - t).count(), hipGetErrorString(err));
    std::fflush(stderr);
    t = now;
  }
};

// Clusters longer than maxc (runs of eigenvalues with gaps <= kEigClusterTol
// ||T||, e.g. the degenerate shells of clean lattices, which k_eig_orth's one
// workgroup does not take): Cholesky QR, twice, on the library's own real
// products — G = Y Y^T of the cluster's rows Y of Zt (the vectors), G = R^T R
// on the host, Y <- R^-T Y — before the Löwdin step.  Replaces round 4's
// rocSOLVER zheev fallback (minutes at n = 4608).  Ud: scratch (the slots' U
// buffers, free between inverse iteration and the Löwdin step).  A
// non-positive pivot sets d_tr_bad (eigen_solve's vendor fallback, as for a
// non-finite result).  Synchronises the stream when a long cluster exists.
int long_clusters(dwh_ctx* ctx, const std::vector<double>& Eh, const std::vector<double>& tn, double* Zt, double* Ud,
                  int n, int64_t sZ, int m, int maxc, bool half) {
  hipStream_t s = ctx->stream;
  std::vector<double> G, W;
  for (int k = 0; k < m; ++k) {
    const double* E = Eh.data() + (size_t)k * n;
    const double tol = dwh::kEigClusterTol * tn[k];
    const int jstart = half ? ctx->eig_c0h[k] : 0;
    for (int j = jstart; j < n;) {
      int end = j + 1;
      while (end < n && E[end] - E[end - 1] <= tol) ++end;
      const int L = end - j;
      if (L > maxc) {
        double* Y = Zt + (int64_t)k * sZ + j;   // L x n, leading dimension n (column-major Zt)
        double* Gd = Ud + (int64_t)k * sZ;      // L x L
        double* Tmp = Gd + (int64_t)L * L;      // L x n
        G.resize((size_t)L * L);
        W.assign((size_t)L * L, 0.0);
        for (int round = 0; round < 2; ++round) {
          dwh::gemm_d('N', 'T', L, L, n, 1.0, Y, n, 0, Y, n, 0, 0.0, Gd, L, 0, 1, s);
          HIPCHECK(ctx, hipGetLastError());
          HIPCHECK(ctx, hipMemcpyAsync(G.data(), Gd, G.size() * sizeof(double), hipMemcpyDeviceToHost, s));
          HIPCHECK(ctx, hipStreamSynchronize(s));
          // G = R^T R (R upper, stored in G's upper triangle, column-major)
          bool ok = true;
          for (int c = 0; c < L && ok; ++c) {
            for (int r = 0; r <= c; ++r) {
              double x = G[(size_t)c * L + r];
              for (int q = 0; q < r; ++q) x -= G[(size_t)r * L + q] * G[(size_t)c * L + q];
              if (r < c) {
                G[(size_t)c * L + r] = x / G[(size_t)r * L + r];
              } else {
                if (!(x > 0.0)) ok = false;
                G[(size_t)c * L + c] = ok ? std::sqrt(x) : 0.0;
              }
            }
          }
          if (!ok) {
            const int one = 1;
            HIPCHECK(ctx, hipMemcpyAsync(ctx->d_tr_bad, &one, sizeof(int), hipMemcpyHostToDevice, s));
            HIPCHECK(ctx, hipStreamSynchronize(s));
            return DWH_OK;
          }
          // W = R^-T (lower triangular): R^T W = I, forward substitution per column
          // (R^T[i][q] = R[q][i] = G[i * L + q] for q <= i)
          std::fill(W.begin(), W.end(), 0.0);
          for (int c = 0; c < L; ++c)
            for (int i = c; i < L; ++i) {
              double x = i == c ? 1.0 : 0.0;
              for (int q = c; q < i; ++q) x -= G[(size_t)i * L + q] * W[(size_t)c * L + q];
              W[(size_t)c * L + i] = x / G[(size_t)i * L + i];
            }
          HIPCHECK(ctx, hipMemcpyAsync(Gd, W.data(), W.size() * sizeof(double), hipMemcpyHostToDevice, s));
          dwh::gemm_d('N', 'N', L, n, L, 1.0, Gd, L, 0, Y, n, 0, 0.0, Tmp, L, 0, 1, s);
          HIPCHECK(ctx, hipMemcpy2DAsync(Y, (size_t)n * sizeof(double), Tmp, (size_t)L * sizeof(double),
                                         (size_t)L * sizeof(double), n, hipMemcpyDeviceToDevice, s));
          HIPCHECK(ctx, hipGetLastError());
        }
        ctx->eig_long_clusters++;
      }
      j = end;
    }
  }
  return DWH_OK;
}

// sub-batch streams of own_heev_enqueue's tridiagonalisation (default / most)
constexpr int kEigStreams = 2, kEigStreamsMax = 4;

// back-transform: W = V^H U is only NB x n, so with fewer than 4 matrices its
// K range is split into up to kEigKS chunks (one batched zgemm per matrix)
#ifndef EIG_KS
#define EIG_KS 8   // (A/B builds)
#endif
constexpr int kEigKS = EIG_KS;

// the own eigensolver's per-matrix workspace for m matrices (both solvers)
int eig_scratch(dwh_ctx* ctx, int m) {
  const int N = ctx->d.N, n = 2 * N;
  const int T = (n + dwh::kEigTB - 1) / dwh::kEigTB, NB = dwh::kEigNB;
  const int nblk = std::max(1, (n - 1 + NB - 1) / NB);
  constexpr int KS = kEigKS;
  const int64_t sP = (int64_t)T * n, sT = (int64_t)nblk * NB * NB, sW = (int64_t)NB * n;
  int rc;
  if (m > ctx->eig_slots) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    for (void* q : {(void*)ctx->d_eig_part, (void*)ctx->d_eig_vv, (void*)ctx->d_eig_ww, (void*)ctx->d_eig_tau,
                    (void*)ctx->d_eig_dpart, (void*)ctx->d_eig_pfin, (void*)ctx->d_eig_c0, (void*)ctx->d_eig_colfin, (void*)ctx->d_eig_gpart,
                    (void*)ctx->d_eig_T, (void*)ctx->d_eig_W, (void*)ctx->d_eig_W2, (void*)ctx->d_eig_d,
                    (void*)ctx->d_eig_e, (void*)ctx->d_eig_tn})
      drop_alloc(ctx, q);
    const size_t mm = (size_t)m;
    if ((rc = dalloc(ctx, &ctx->d_eig_part, mm * sP)) || (rc = dalloc(ctx, &ctx->d_eig_vv, mm * dwh::kEigRing * n)) ||
        (rc = dalloc(ctx, &ctx->d_eig_ww, mm * dwh::kEigRing * n)) || (rc = dalloc(ctx, &ctx->d_eig_tau, mm * n)) ||
        (rc = dalloc(ctx, &ctx->d_eig_dpart, mm * 2 * dwh::kEigDeferMax * T)) ||
        (rc = dalloc(ctx, &ctx->d_eig_pfin, mm * n)) || (rc = dalloc(ctx, &ctx->d_eig_colfin, mm * n)) ||
        (rc = dalloc(ctx, &ctx->d_eig_gpart, mm * 3 * dwh::kEigGP)) ||
        (rc = dalloc(ctx, &ctx->d_eig_T, mm * sT)) || (rc = dalloc(ctx, &ctx->d_eig_W, mm * std::max<int64_t>(KS * sW, (int64_t)nblk * dwh::kEigGS * NB * NB))) ||
        (rc = dalloc(ctx, &ctx->d_eig_W2, mm * sW)) || (rc = dalloc(ctx, &ctx->d_eig_d, mm * n)) ||
        (rc = dalloc(ctx, &ctx->d_eig_e, mm * n)) || (rc = dalloc(ctx, &ctx->d_eig_tn, mm)) ||
        (rc = dalloc(ctx, &ctx->d_eig_c0, mm)))
      return rc;
    ctx->eig_slots = m;
  }
  return DWH_OK;
}

// U = (I - V_0 T_0 V_0^H) ... (I - V_last T_last V_last^H) U on the columns
// j0.. of the slots' U: the reflectors' V (n x n per matrix, column c = v_c
// on the rows > c, zeros above) and complex tau (ctx->d_eig_tau), V^H block
// by block into Vt (an n x n slot buffer); the library's own products
// (dwhmc_gemm.hip)
int eig_back_transform(dwh_ctx* ctx, const double2* V, double2* Vt, int j0, int m) {
  const int N = ctx->d.N, n = 2 * N, NB = dwh::kEigNB;
  const dwh::TrBufs& b = ctx->tr;
  const int64_t sA = (int64_t)n * n;
  const int nblk = std::max(1, (n - 1 + NB - 1) / NB);
  const int64_t sT = (int64_t)nblk * NB * NB, sW = (int64_t)NB * n;
  const int M = n - j0;
  hipStream_t s = ctx->stream;
  dwh::launch_eig_tfac(V, n, sA, ctx->d_eig_tau, ctx->d_eig_W, ctx->d_eig_T, sT, m, s);   // W as Gram scratch
  HIPCHECK(ctx, hipGetLastError());
  const double2 one = make_double2(1.0, 0.0), zero = make_double2(0.0, 0.0), mone = make_double2(-1.0, 0.0);
  const int ks = m >= 4 ? 1 : kEigKS;
  const int64_t sWs = ks * sW;
  const int ldv = std::min(NB, n - 1);   // as k_eig_vt lays the blocks out
  dwh::launch_eig_vt(V, n, sA, Vt, m, s);
  for (int blk = nblk - 1; blk >= 0; --blk) {
    const int r0 = blk * NB, kb = std::min(NB, n - 1 - r0), ms = n - r0 - 1;
    const double2* Vb = V + (r0 + 1) + (int64_t)r0 * n;
    double2* Us = b.U + (r0 + 1) + (int64_t)j0 * n;
    const int ldw = ks * NB;
    // W = V^H U in K chunks of c rows (a multiple of 16, the last one shorter),
    // chunk s at rows s kb of W: one launch for every (matrix, chunk)
    const int c = ks == 1 ? ms : std::max(16, ((ms + ks - 1) / ks + 15) / 16 * 16);
    const int nfull = ms / c, rem = ms - nfull * c, S = nfull + (rem > 0);
    dwh::gemm_z_chunked('N', 'N', kb, M, c, rem > 0 ? rem : c, S, one, Vt + (int64_t)r0 * n, ldv, (int64_t)c * ldv, sA,
                        Us, n, c, sA, zero, ctx->d_eig_W, ldw, kb, sWs, m, s);
    if (S == 1)   // W2 = T W on the MFMA (4x faster than k_eig_tw's LDS MACs at 16 matrices)
      dwh::gemm_z('N', 'N', kb, M, kb, one, ctx->d_eig_T + (int64_t)blk * NB * NB, NB, sT, ctx->d_eig_W, ldw, sWs,
                  zero, ctx->d_eig_W2, NB, sW, m, s);
    else
      dwh::launch_eig_tw(ctx->d_eig_T + (int64_t)blk * NB * NB, sT, ctx->d_eig_W, ldw, sWs, S, kb, M,
                         ctx->d_eig_W2, sW, m, s);
    dwh::gemm_z('N', 'N', ms, M, kb, mone, Vb, n, sA, ctx->d_eig_W2, NB, sW, one, Us, n, sA, m, s);
  }
  HIPCHECK(ctx, hipGetLastError());
  return DWH_OK;
}

int own_heev_enqueue(dwh_ctx* ctx, const TrSrc& src, int m) {
  const int N = ctx->d.N, n = 2 * N;
  const dwh::TrBufs& b = ctx->tr;
  const int64_t sA = (int64_t)n * n, sZ = 2 * sA;   // sZ in doubles
  const int T = (n + dwh::kEigTB - 1) / dwh::kEigTB;
  const int64_t sP = (int64_t)T * n;
  int rc;
  if ((rc = eig_scratch(ctx, m))) return rc;
  hipStream_t s = ctx->stream;
  double2* A = b.JU;
  EigPhase ph(s);
  if ((rc = assemble_slots(ctx, src, m, A))) return rc;
  ph.mark("assemble");
  // Batches of 8+ matrices run as sub-batches of 4+ on their own streams,
  // column by column: one sub-batch's HBM-bound pass overlaps another's
  // latency-bound reduce and step (DWHMC_EIG_STREAMS: the number of streams,
  // 1 = one stream, A/B)
  int ng = m >= 8 ? kEigStreams : 1;
  if (const char* es = std::getenv("DWHMC_EIG_STREAMS")) ng = std::max(1, std::min(std::atoi(es), kEigStreamsMax));
  ng = std::max(1, std::min(ng, m / dwh::kEigDeferMin));
  for (int g = 1; g < ng; ++g)
    if (!ctx->eig_sx[g - 1] &&
        hipStreamCreateWithFlags(&ctx->eig_sx[g - 1], hipStreamNonBlocking) != hipSuccess)
      return fail(ctx, DWH_ERR_HIP, "eigensolver stream creation failed");
  for (int g = 0; g < ng && ng > 1; ++g)
    if (!ctx->eig_ev[g] && hipEventCreateWithFlags(&ctx->eig_ev[g], hipEventDisableTiming) != hipSuccess)
      return fail(ctx, DWH_ERR_HIP, "eigensolver event creation failed");
  if (ng > 1) {
    HIPCHECK(ctx, hipEventRecord(ctx->eig_ev[0], s));
    for (int g = 1; g < ng; ++g) HIPCHECK(ctx, hipStreamWaitEvent(ctx->eig_sx[g - 1], ctx->eig_ev[0], 0));
  }
  const int64_t sDp = (int64_t)2 * dwh::kEigDeferMax * T, sGp = (int64_t)3 * dwh::kEigGP, sR = (int64_t)dwh::kEigRing * n;
  const int sw = dwh::eig_switch_col(n);
  for (int i = 0; i < n; ++i) {
    if (ph.on && i % 512 == 0 && i > 0) ph.mark("tridiag/512");
    for (int g = 0; g < ng; ++g) {
      const int64_t k0 = (int64_t)m * g / ng;
      const int mg = (int)((int64_t)m * (g + 1) / ng - k0);
      dwh::launch_eig_column(A + k0 * sA, n, i, sA, ctx->d_eig_part + k0 * sP, sP, ctx->d_eig_pfin + k0 * n,
                             ctx->d_eig_colfin + k0 * n, ctx->d_eig_vv + k0 * sR, ctx->d_eig_ww + k0 * sR,
                             ctx->d_eig_d + k0 * n, ctx->d_eig_e + k0 * n, ctx->d_eig_tau + k0 * n,
                             ctx->d_eig_dpart + k0 * sDp, ctx->d_eig_gpart + k0 * sGp, mg,
                             g ? ctx->eig_sx[g - 1] : s, sw);
    }
  }
  for (int g = 1; g < ng; ++g) {
    HIPCHECK(ctx, hipEventRecord(ctx->eig_ev[g], ctx->eig_sx[g - 1]));
    HIPCHECK(ctx, hipStreamWaitEvent(s, ctx->eig_ev[g], 0));
  }
  ph.mark("tridiag");
  dwh::launch_eig_bisect(ctx->d_eig_d, ctx->d_eig_e, n, b.E, ctx->d_eig_tn, m, s);
  ph.mark("bisect");
  double* Zt = reinterpret_cast<double*>(b.Jmn);
  double* Ud = reinterpret_cast<double*>(b.U);
  // DWHMC_EIG_MAX_CLUSTER (tests): a shorter limit for the single-workgroup
  // cluster orthonormalisation, to exercise the long-cluster path below
  int maxc = dwh::kEigMaxCluster;
  if (const char* e = std::getenv("DWHMC_EIG_MAX_CLUSTER")) maxc = std::max(1, std::min(maxc, std::atoi(e)));
  // Particle-hole half solve (H_BdG: E <-> -E with eigenvectors (u; v) <->
  // (-v*; u*)): eigenvectors of T only for the indices from
  // c0, the largest index <= n/2 below which the spectrum has a gap wider
  // than kEigZeroTol ||T|| (n/2 unless levels crowd around zero, e.g. the
  // exact zero modes of clean lattices, which are then computed whole; 0 for
  // a spectrum with degenerate levels anywhere); the
  // columns below c0 are the partners of the columns above n - c0
  // (k_eig_theta after the back-transform).  c0 comes from the eigenvalues
  // on the host (one synchronisation); every matrix computes the columns
  // [j0, n), j0 = min c0, the ones below its own c0 zeroed.  Inverse
  // iteration, the orthogonalisation and the back-transform run on ~half the
  // columns.  DWHMC_EIG_HALF=0: every column (A/B).
  const char* eh = std::getenv("DWHMC_EIG_HALF");
  const bool half = n % 2 == 0 && !(eh && *eh == '0');
  ctx->eig_half = half;
  ctx->eig_c0h.assign(half ? m : 0, N);
  int j0 = 0;
  // the eigenvalues on the host (one synchronisation): the half solve's c0
  // and the clusters longer than maxc
  std::vector<double> Eh((size_t)m * n), tn(m);
  HIPCHECK(ctx, hipMemcpyAsync(Eh.data(), b.E, Eh.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHECK(ctx, hipMemcpyAsync(tn.data(), ctx->d_eig_tn, m * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHECK(ctx, hipStreamSynchronize(s));
  if (half) {
    j0 = N;
    for (int k = 0; k < m; ++k) {
      const double* E = Eh.data() + (size_t)k * n;
      const double tol = dwh::kEigZeroTol * tn[k];
      int c = N;
      while (c > 0 && !(E[c] - E[c - 1] > tol)) --c;   // (NaN gaps: keep going, c -> 0)
      // degenerate levels (clean lattices: most levels in clusters) leave the
      // partner images' overlaps with the computed vectors at ~1e-13 and
      // above; such a matrix computes every vector (c0 = 0)
      const double ctol = dwh::kEigClusterTol * tn[k];
      for (int j = 1; j < n && c > 0; ++j)
        if (!(E[j] - E[j - 1] > ctol)) c = 0;
      ctx->eig_c0h[k] = c;
      j0 = std::min(j0, c);
    }
    HIPCHECK(ctx, hipMemcpyAsync(ctx->d_eig_c0, ctx->eig_c0h.data(), m * sizeof(int), hipMemcpyHostToDevice, s));
    ph.mark("c0");
  }
  const int M = n - j0;   // eigenvector columns computed
  dwh::launch_eig_invit(ctx->d_eig_d, ctx->d_eig_e, n, b.E, ctx->d_eig_tn, Zt, Zt + sA, Ud, Ud + sA, sZ,
                        ctx->d_tr_bad, m, s, maxc, j0, half ? ctx->d_eig_c0 : nullptr);
  ph.mark("invit+orth");
  if ((rc = long_clusters(ctx, Eh, tn, Zt, Ud, n, sZ, m, maxc, half))) return rc;
  ph.mark("long clusters");
  // One symmetric (Löwdin) orthogonalisation step over the computed vectors:
  // with Y = Z^T (column-major Zt, its rows j0.. the vectors) and G = Y Y^T =
  // I + F, Y <- (3/2 I - 1/2 G) Y leaves ||F|| -> O(||F||^2).  Outside clusters
  // F_jl ~ c eps ||T|| / |λ_j - λ_l| (inverse iteration's per-vector error), so
  // the mixing moves each residual by ~ F_jl |λ_j - λ_l| ~ c eps ||T||:
  // orthogonality to rounding, accuracy kept.  (Zeroed partner rows stay zero.)
  double* G = Ud;          // the slots' U buffers (LU scratch until now)
  double* Y2 = Zt + sA;    // second half of the slots' Jmn buffers
  dwh::gemm_d('N', 'T', M, M, n, 1.0, Zt + j0, n, sZ, Zt + j0, n, sZ, 0.0, G, M, sZ, m, s);
  HIPCHECK(ctx, hipMemcpy2DAsync(Y2, sZ * sizeof(double), Zt, sZ * sizeof(double), sA * sizeof(double), m,
                                 hipMemcpyDeviceToDevice, s));
  dwh::gemm_d('N', 'N', M, n, M, -0.5, G, M, sZ, Zt + j0, n, sZ, 1.5, Y2 + j0, n, sZ, m, s);
  dwh::launch_eig_zt_to_u(Y2, b.U, n, sZ, sA, m, s, j0);
  HIPCHECK(ctx, hipGetLastError());
  ph.mark("lowdin");
  if (n < 2) return DWH_OK;
  // V^H block by block into the slots' Jmn buffers (free after the Löwdin step)
  if ((rc = eig_back_transform(ctx, A, b.Jmn, j0, m))) return rc;
  if (half) dwh::launch_eig_theta(b.U, n, sA, ctx->d_eig_c0, m, s);
  ph.mark("backtransform");
  HIPCHECK(ctx, hipGetLastError());
  return DWH_OK;
}

int eigen_enqueue(dwh_ctx* ctx, const TrSrc& src, int m, bool qr) {
  const int N = ctx->d.N, n2 = 2 * N;
  const dwh::TrBufs& b = ctx->tr;
  const int64_t sA = (int64_t)n2 * n2;
  if (int rc = assemble_slots(ctx, src, m, b.U)) return rc;
  auto* A = reinterpret_cast<rocblas_double_complex*>(b.U);
  rocblas_status st;
  if (qr)
    st = m == 1 ? rocsolver_zheev(ctx->blas, rocblas_evect_original, rocblas_fill_upper, n2, A, n2, b.E,
                                  ctx->d_tr_offd, ctx->d_tr_info)
                : rocsolver_zheev_strided_batched(ctx->blas, rocblas_evect_original, rocblas_fill_upper, n2, A, n2,
                                                  sA, b.E, n2, ctx->d_tr_offd, n2, ctx->d_tr_info, m);
  else
    st = m == 1 ? rocsolver_zheevd(ctx->blas, rocblas_evect_original, rocblas_fill_upper, n2, A, n2, b.E,
                                   ctx->d_tr_offd, ctx->d_tr_info)
                : rocsolver_zheevd_strided_batched(ctx->blas, rocblas_evect_original, rocblas_fill_upper, n2, A,
                                                   n2, sA, b.E, n2, ctx->d_tr_offd, n2, ctx->d_tr_info, m);
  if (st != rocblas_status_success)
    return fail(ctx, DWH_ERR_HIP, std::string("rocsolver_zheevd: ") + rocblas_status_to_string(st));
  return DWH_OK;
}

int q_heev_enqueue(dwh_ctx* ctx, const TrSrc& src, int m, bool* done);

// The library's own eigensolver for every order up to kEigMaxN; rocSOLVER only
// beyond it (zheevd) and as the re-solve (QR-iteration zheev) of a solve that
// left a non-finite value: rocSOLVER's zheevd returns NaN eigenvectors for
// spectra with exactly degenerate eigenvalues (the clean lattice, W = 0).
// Synchronises the stream.
int eigen_solve(dwh_ctx* ctx, const TrSrc& src, int m) {
  int rc;
  const int64_t n2 = 2 * (int64_t)ctx->d.N;
  const bool own = n2 <= dwh::kEigMaxN;
  ctx->eig_ph = false;
  ctx->eig_ph_last = 0;   // dwh_info_t::eig_half describes this solve on every exit path
  HIPCHECK(ctx, hipMemsetAsync(ctx->d_tr_bad, 0, sizeof(int), ctx->stream));
  if (own) {
    // the own solver (k_eig_orth flags an over-long cluster in d_tr_bad);
    // rocSOLVER zheev only if it flagged or produced non-finite values
    HIPCHECK(ctx, hipMemsetAsync(ctx->d_tr_info, 0, m * sizeof(int), ctx->stream));
    Scope sc(ctx, T_EIG_OWN, m);
    // the structure-preserving solver first (DWHMC_EIG_QUAT=0: the one-stage
    // solver only, A/B); it declines spectra with over-long clusters or crowds
    bool done = false;
    const char* qe = std::getenv("DWHMC_EIG_QUAT");
    if (dwh::q_supported(ctx->d.N) && !(qe && *qe == '0')) rc = q_heev_enqueue(ctx, src, m, &done);
    else rc = DWH_OK;
    if (!rc && !done) rc = own_heev_enqueue(ctx, src, m);
    ctx->eig_quat_last = done ? 1 : 0;
  } else {
    Scope sc(ctx, T_EIG_VENDOR, m);
    rc = eigen_enqueue(ctx, src, m, false);
  }
  if (rc) return rc;
  dwh::launch_nonfinite(ctx->tr.U, m * n2 * n2, ctx->tr.E, m * n2, ctx->d_tr_bad, ctx->stream);
  int bad = 0;
  HIPCHECK(ctx, hipMemcpyAsync(&bad, ctx->d_tr_bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (!bad && own && ctx->eig_half && (int)ctx->eig_c0h.size() == m)
    ctx->eig_ph = std::all_of(ctx->eig_c0h.begin(), ctx->eig_c0h.end(), [&](int c) { return c == ctx->d.N; });
  ctx->eig_ph_last = ctx->eig_ph ? 1 : 0;
  if (bad) {
    Scope sc(ctx, T_EIG_VENDOR, m);
    rc = eigen_enqueue(ctx, src, m, true);
  }
  return rc;
}

int eigen_info_check(dwh_ctx* ctx, int m) {
  std::vector<int> info(m, 0);
  HIPCHECK(ctx, hipMemcpyAsync(info.data(), ctx->d_tr_info, m * sizeof(int), hipMemcpyDeviceToHost,
                               ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHECK(ctx, hipGetLastError());
  for (int k = 0; k < m; ++k)
    if (info[k] != 0)
      return fail(ctx, DWH_ERR_HIP, "the rocSOLVER eigensolver (zheevd / zheev fallback) did not converge (info = " +
                                        std::to_string(info[k]) + ")");
  return DWH_OK;
}

int transport_args(dwh_ctx* ctx, double eta, double domega, double omega_max, int64_t n_omega, int64_t n_dos,
                   int64_t* nw, int64_t* nd) {
  if (dwh_transport_grid(eta, domega, omega_max, nw, nd) != DWH_OK)
    return fail(ctx, DWH_ERR_ARG, g_create_error);
  if (n_omega != *nw || n_dos != *nd)
    return fail(ctx, DWH_ERR_ARG, "n_omega / n_dos differ from dwh_transport_grid (" + std::to_string(*nw) +
                                      ", " + std::to_string(*nd) + ")");
  return DWH_OK;
}

// measure_transport_and_spectra for chains c0 .. c0+m-1 (slots 0 .. m-1);
// outputs per chain at strides 1 / nw / nd / N
int transport_run(dwh_ctx* ctx, const TrSrc& src, int m, double eta, double domega, double omega_max, int64_t nw,
                  int64_t nd, double* stiffness, double* dc_cond, double* sigma, double* dos, double* dos_an,
                  double* ak0) {
  int rc;
  if ((rc = transport_prepare(ctx, nw, nd, m))) return rc;
  if ((rc = eigen_solve(ctx, src, m))) return rc;
  const int N = ctx->d.N, n2 = 2 * N;
  const int64_t sA = (int64_t)n2 * n2;
  hipStream_t s = ctx->stream;
  // particle-hole closed U (eig_ph): only the columns < N of J_mn are read
  const bool ph = ctx->eig_ph;
  const int ncol = ph ? N : n2;
  for (int k = 0; k < m; ++k) {
    const dwh::TrBufs b = tr_slot(ctx, k);
    dwh::launch_tr_colstats(b.U, N, (int)ctx->Lx, b.E, ctx->beta, eta, ctx->t, ctx->tp, ctx->d_tr_nbr, b.f,
                            b.dia, b.Wn, b.wan, b.w0, s);
    dwh::launch_tr_current(b.U, b.JU, N, ctx->d_tr_rowptr, ctx->d_tr_col, ctx->d_tr_val, ncol, s);
  }
  HIPCHECK(ctx, hipGetLastError());
  // J_mn = U^H (J ⊕ J) U  (src/Observables.jl:334-335), the library's own product
  const dwh::TrBufs& b0 = ctx->tr;
  const double2 one = make_double2(1.0, 0.0), zero = make_double2(0.0, 0.0);
  if (ph) {
    // only columns < N of J_mn: its columns [N, n2) hold U^H half by half
    // (N x n2, ld N), so both products are 'N','N' (1.6x faster than the
    // conjugate-transposed operand: profiles/r05_exp_backtransform_vt.txt)
    double2* Ut = b0.Jmn + (int64_t)N * n2;
    for (int h = 0; h < 2; ++h) {
      dwh::launch_tr_conj_transpose(b0.U + (int64_t)h * N * n2, n2, N, n2, sA, Ut, N, sA, m, s);
      dwh::gemm_z('N', 'N', N, ncol, n2, one, Ut, N, sA, b0.JU, n2, sA, zero, b0.Jmn + (int64_t)h * N, n2, sA, m, s);
    }
  } else {
    dwh::gemm_z('C', 'N', n2, ncol, n2, one, b0.U, n2, sA, b0.JU, n2, sA, zero, b0.Jmn, n2, sA, m, s);
  }
  HIPCHECK(ctx, hipGetLastError());
  const dwh::TrGrid g{eta, -omega_max, domega, (int)nw, (int)nd};
  for (int k = 0; k < m; ++k)
    dwh::launch_tr_reduce(tr_slot(ctx, k), N, (int)ctx->Lx, (int)ctx->Ly, ctx->beta, eta, g, ph, s);
  HIPCHECK(ctx, hipGetLastError());
  std::vector<double> sc(2 * (size_t)m);
  HIPCHECK(ctx, hipMemcpyAsync(sc.data(), b0.scalars, sc.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  if (nw > 0)
    HIPCHECK(ctx, hipMemcpyAsync(sigma, b0.sigma, m * nw * sizeof(double), hipMemcpyDeviceToHost, s));
  if (nd > 0) {
    HIPCHECK(ctx, hipMemcpyAsync(dos, b0.dos, m * nd * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(dos_an, b0.dos_an, m * nd * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  HIPCHECK(ctx, hipMemcpyAsync(ak0, b0.ak, (size_t)m * N * sizeof(double), hipMemcpyDeviceToHost, s));
  if ((rc = eigen_info_check(ctx, m))) return rc;
  for (int k = 0; k < m; ++k) {
    stiffness[k] = sc[2 * k];
    dc_cond[k] = sc[2 * k + 1];
  }
  return DWH_OK;
}

// Workspace of the structure-preserving solver (dwhmc_qeig.hip) for q_slots
// matrices, one array per quantity (the kernels' per-matrix strides):
// reduction scratch, w, y, the diagonal blocks before / after the site
// rotations, the rotations, tau, ||T||; for the eigenvectors (q_vec_slots
// matrices, nv = N columns): Zt (n x nv), the inverse iteration's LU
// scratch, the Löwdin Gram matrix (nv x nv).
struct QBufs {
  double2 *part, *W, *Y, *qd, *rd, *G;
  double *tau, *qa, *ra, *rb, *tn;
  int64_t sP;
};
QBufs q_bufs(dwh_ctx* ctx) {
  const int M = ctx->d.N, n = 2 * M, m = ctx->q_slots;
  const int64_t sP = dwh::q_part_elems(M);
  double* w = ctx->d_q;
  QBufs q;
  q.sP = sP;
  int64_t o = 0;   // doubles
  auto take2 = [&](int64_t per) { double2* p = reinterpret_cast<double2*>(w + o); o += 2 * per * m; return p; };
  auto take1 = [&](int64_t per) { double* p = w + o; o += per * m; return p; };
  q.part = take2(sP);
  q.W = take2(n);
  q.Y = take2(n);
  q.qd = take2(M);
  q.rd = take2(M);
  q.G = take2(n);
  q.tau = take1(M);
  q.qa = take1(M);
  q.ra = take1(M);
  q.rb = take1(M);
  q.tn = take1(2);
  return q;
}
int64_t q_bufs_doubles(int M, int m) {
  const int n = 2 * M;
  return m * (2 * (int64_t)dwh::q_part_elems(M) + 2 * (3 * (int64_t)n + 2 * M) + 4 * (int64_t)M + 2);
}

// Eigenvalues by the structure-preserving reduction: H_BdG of the m sources
// assembled into the slots' JU, reduced site by site on their particle rows
// (the reflectors left in JU's bottom rows), site rotations, block Sturm
// bisection; the 2N ascending eigenvalues of each into the slots' E (device).
// ms (optional, m = 1): the reduction's device time (HIP events; synchronises).
int qeig_values(dwh_ctx* ctx, const TrSrc& src, int m, float* ms) {
  const int M = ctx->d.N, n = 2 * M;
  if (!dwh::q_supported(M)) return fail(ctx, DWH_ERR_ARG, "structure-preserving solver: lattice too large");
  const int64_t sA = (int64_t)n * n;
  int rc;
  if (m > ctx->q_slots) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    drop_alloc(ctx, ctx->d_q);
    ctx->d_q = nullptr;
    ctx->q_slots = 0;
    if ((rc = dalloc(ctx, &ctx->d_q, (size_t)q_bufs_doubles(M, m)))) return rc;
    ctx->q_slots = m;
  }
  const QBufs q = q_bufs(ctx);
  hipStream_t s = ctx->stream;
  double2* A = ctx->tr.JU;
  if ((rc = assemble_slots(ctx, src, m, A))) return rc;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ms) {
    HIPCHECK(ctx, hipEventCreate(&e0));
    HIPCHECK(ctx, hipEventCreate(&e1));
    HIPCHECK(ctx, hipEventRecord(e0, s));
  }
  const char* qg = std::getenv("DWHMC_Q_GRAPH");
  if (qg && *qg == '1') {
    // opt-in: the 2 M launches captured once per (slots, workspace, m) and
    // replayed — one L = 32 measurement 24.4-24.7 -> 24.2-24.3 ms, but
    // tests/bench_transport.py under rocprofv3 --kernel-trace segfaulted with
    // it (recapture for a new batch size) and not without it
    // (profiles/r06_exp_qreduce_graph.txt), so stream launches stay the default
    if (!ctx->q_graph || ctx->q_graph_key[0] != A || ctx->q_graph_key[1] != ctx->d_q || ctx->q_graph_m != m) {
      if (ctx->q_graph) {
        HIPCHECK(ctx, hipStreamSynchronize(s));
        (void)hipGraphExecDestroy(ctx->q_graph);
        ctx->q_graph = nullptr;
      }
      hipGraph_t g = nullptr;
      HIPCHECK(ctx, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      dwh::launch_q_reduce(A, M, sA, q.part, q.sP, q.W, q.tau, q.Y, q.qa, q.qd, m, s);
      HIPCHECK(ctx, hipStreamEndCapture(s, &g));
      const hipError_t e = hipGraphInstantiate(&ctx->q_graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (e != hipSuccess) {
        ctx->q_graph = nullptr;
        return fail(ctx, DWH_ERR_HIP, std::string("reduction graph: ") + hipGetErrorString(e));
      }
      ctx->q_graph_key[0] = A;
      ctx->q_graph_key[1] = ctx->d_q;
      ctx->q_graph_m = m;
    }
    HIPCHECK(ctx, hipGraphLaunch(ctx->q_graph, s));
  } else {
    dwh::launch_q_reduce(A, M, sA, q.part, q.sP, q.W, q.tau, q.Y, q.qa, q.qd, m, s);
  }
  if (ms) HIPCHECK(ctx, hipEventRecord(e1, s));
  dwh::launch_q_rot(q.qa, q.qd, q.Y, M, q.ra, q.rd, q.rb, q.G, m, s);
  dwh::launch_q_bisect(q.ra, q.rd, q.rb, M, ctx->tr.E, q.tn, m, s);
  HIPCHECK(ctx, hipGetLastError());
  if (ms) {
    HIPCHECK(ctx, hipStreamSynchronize(s));
    HIPCHECK(ctx, hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  return DWH_OK;
}

// Every eigenpair by the structure-preserving solver (m matrices): qeig_values,
// then — when no matrix's spectrum has a cluster (consecutive gaps <=
// kEigClusterTol ||T||) longer than q_max_cluster() or a crowd at zero
// (q_zero_crowd) longer than half that, checked on the host from the
// eigenvalues (one synchronisation) — the particle-hole half: inverse
// iteration on T for the N upper eigenvalues (k_q_invit), the clusters and
// the crowd orthonormalised (k_q_orth), one Löwdin step (the library's complex
// products), the site rotations into U' (interleaved rows), the reflector
// pairs as a one-stage V and its back-transform, then the BdG row order and
// the Theta partners for the lower half (k_q_final).  *done = false: not
// taken (the caller runs the one-stage solver; the slots' JU / E are
// overwritten either way).
int q_heev_enqueue(dwh_ctx* ctx, const TrSrc& src, int m, bool* done) {
  *done = false;
  const int N = ctx->d.N, n = 2 * N, j0 = N, nv = n - j0;
  const dwh::TrBufs& b = ctx->tr;
  const int64_t sA = (int64_t)n * n;
  int rc;
  if ((rc = qeig_values(ctx, src, m, nullptr))) return rc;
  const QBufs q = q_bufs(ctx);
  hipStream_t s = ctx->stream;
  const char* eh = std::getenv("DWHMC_EIG_HALF");   // =0: every column solved (the one-stage solver)
  if (n % 2 || (eh && *eh == '0')) return DWH_OK;
  std::vector<double> Eh((size_t)m * n), tn((size_t)2 * m);
  HIPCHECK(ctx, hipMemcpyAsync(Eh.data(), b.E, Eh.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHECK(ctx, hipMemcpyAsync(tn.data(), q.tn, m * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHECK(ctx, hipStreamSynchronize(s));
  // Crowding at zero matters through E_j + E_k of two computed vectors j != k
  // (x_j against the partner Theta x_k, which the Löwdin step does not
  // see): E_N + E_{N+1} <= kEigZeroTol ||T||, the one-stage half solve's
  // bound on it.  A single level near zero is harmless: x_N and Theta x_N
  // are orthogonal exactly (<u, Theta u> = 0 for Theta^2 = -1).
  // Clusters (consecutive gaps <= kEigClusterTol ||T||) up to q_max_cluster()
  // long are orthonormalised in the structure-preserving path (k_q_orth);
  // longer ones are declined.
  // A crowd at zero (q_zero_crowd) of up to q_max_cluster() / 2 levels is
  // orthonormalised together with its Theta partners (k_q_orth).
  bool clusters = false;
  for (int k = 0; k < m; ++k) {
    const double* E = Eh.data() + (size_t)k * n;
    const int crowd = dwh::q_zero_crowd(E, n, j0, tn[k]);
    if (2 * crowd > dwh::q_max_cluster()) return DWH_OK;
    clusters = clusters || crowd > 0;
    int run = 1;
    for (int j = j0 + std::max(crowd, 1); j < n; ++j) {
      if (!(E[j] - E[j - 1] > dwh::kEigClusterTol * tn[k])) {
        clusters = true;
        if (++run > dwh::q_max_cluster()) return DWH_OK;
      } else {
        run = 1;
      }
    }
  }
  // vector workspace
  const int64_t sZ = (int64_t)n * nv, sS = dwh::q_invit_scratch(N, j0), sG = (int64_t)nv * nv;
  if (m > ctx->q_vec_slots) {
    HIPCHECK(ctx, hipStreamSynchronize(s));
    for (void* p : {(void*)ctx->d_qz, (void*)ctx->d_qs, (void*)ctx->d_qg}) drop_alloc(ctx, p);
    ctx->d_qz = ctx->d_qs = ctx->d_qg = nullptr;
    ctx->q_vec_slots = 0;
    if ((rc = dalloc(ctx, &ctx->d_qz, (size_t)m * sZ)) || (rc = dalloc(ctx, &ctx->d_qs, (size_t)m * sS)) ||
        (rc = dalloc(ctx, &ctx->d_qg, (size_t)m * sG)))
      return rc;
    ctx->q_vec_slots = m;
  }
  if ((rc = eig_scratch(ctx, m))) return rc;
  EigPhase ph(s);
  ph.mark("q values");
  dwh::launch_q_invit(q.ra, q.rd, q.rb, N, b.E, q.tn, j0, ctx->d_qz, sZ, ctx->d_qs, sS, m, s);
  if (clusters) dwh::launch_q_orth(b.E, q.tn, N, j0, ctx->d_qz, sZ, dwh::kEigClusterTol, ctx->d_tr_bad, m, s);
  ph.mark("q invit");
  // Löwdin on X = Zt (nv x n, ld nv): G' = X X^H (= conj(Z^H Z)), Y^T = 1.5 X - 0.5 G' X into the slots' Jmn
  const double2 one = make_double2(1.0, 0.0), zero = make_double2(0.0, 0.0);
  dwh::gemm_z('N', 'C', nv, nv, n, one, ctx->d_qz, nv, sZ, ctx->d_qz, nv, sZ, zero, ctx->d_qg, nv, sG, m, s);
  HIPCHECK(ctx, hipMemcpy2DAsync(b.Jmn, sA * sizeof(double2), ctx->d_qz, sZ * sizeof(double2), sZ * sizeof(double2), m,
                                 hipMemcpyDeviceToDevice, s));
  dwh::gemm_z('N', 'N', nv, n, nv, make_double2(-0.5, 0.0), ctx->d_qg, nv, sG, ctx->d_qz, nv, sZ,
              make_double2(1.5, 0.0), b.Jmn, nv, sA, m, s);
  // the site rotations, transposed into the slots' U columns j0.. (interleaved rows)
  dwh::launch_q_ztu(b.Jmn, sA, q.G, N, j0, b.U, sA, m, s);
  ph.mark("q lowdin");
  // the reflector pairs as V (slots' Jmn) and complex tau; V^H blocks into the slots' JU
  dwh::launch_q_vexpand(b.JU, sA, q.tau, N, b.Jmn, ctx->d_eig_tau, m, s);
  HIPCHECK(ctx, hipGetLastError());
  if ((rc = eig_back_transform(ctx, b.Jmn, b.JU, j0, m))) return rc;
  ph.mark("q backtransform");
  // BdG row order and the Theta partners, through the slots' JU
  dwh::launch_q_final(b.U, sA, N, j0, b.JU, m, s);
  HIPCHECK(ctx, hipMemcpyAsync(b.U, b.JU, (size_t)m * sA * sizeof(double2), hipMemcpyDeviceToDevice, s));
  HIPCHECK(ctx, hipGetLastError());
  ph.mark("q final");
  ctx->eig_half = true;
  ctx->eig_c0h.assign(m, N);
  *done = true;
  return DWH_OK;
}

}  // namespace

extern "C" {

int dwh_transport_grid(double eta, double domega, double omega_max, int64_t* n_omega, int64_t* n_dos) {
  if (!n_omega || !n_dos) return fail(nullptr, DWH_ERR_ARG, "NULL argument");
  if (!(eta > 0) || !(domega > 0) || !(omega_max > 0) || !std::isfinite(eta + domega + omega_max))
    return fail(nullptr, DWH_ERR_ARG, "eta, domega, omega_max must be finite and > 0");
  *n_omega = julia_range_len(eta, domega, omega_max);
  *n_dos = julia_range_len(-omega_max, domega, omega_max);
  if (*n_omega > (1 << 24) || *n_dos > (1 << 24))
    return fail(nullptr, DWH_ERR_ARG, "frequency grid longer than 2^24 points");
  return DWH_OK;
}

// Development entry (tools/qeig_check.py): qeig_values of `chain`, the
// eigenvalues into E and the reduction's device time into *ms.
int dwh_debug_qeig(dwh_ctx* ctx, int64_t chain, double* E, double* ms) {
  if (!ctx || !E) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (chain < 0 || chain >= ctx->d.nc) return fail(ctx, DWH_ERR_ARG, "chain index out of range");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  int rc;
  if ((rc = transport_prepare(ctx, std::max<int64_t>(ctx->tr_nw, 0), std::max<int64_t>(ctx->tr_nd, 0), 1)))
    return rc;
  float t = 0.0f;
  if ((rc = qeig_values(ctx, chains_src(ctx, chain), 1, &t))) return rc;
  const int M = ctx->d.N;
  HIPCHECK(ctx, hipMemcpyAsync(E, ctx->tr.E, 2 * (size_t)M * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (ms) *ms = t;
#ifdef QSTAMPS
  if (const char* f = std::getenv("QSTAMPS_FILE")) {   // diagnostic builds: the phase stamps
    std::vector<unsigned long long> st((size_t)std::min(M, 4096) * 16);
    if (dwh::q_stamps_read(st.data(), std::min(M, 4096)) == 0)
      if (FILE* fp = std::fopen(f, "wb")) {
        std::fwrite(st.data(), sizeof(unsigned long long), st.size(), fp);
        std::fclose(fp);
      }
  }
#endif
  return DWH_OK;
}

int dwh_eigensystem(dwh_ctx* ctx, int64_t chain, double* E, dwh_c128* U) {
  if (!ctx || !E) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (chain < 0 || chain >= ctx->d.nc) return fail(ctx, DWH_ERR_ARG, "chain index out of range");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  int rc;
  if ((rc = transport_prepare(ctx, std::max<int64_t>(ctx->tr_nw, 0), std::max<int64_t>(ctx->tr_nd, 0), 1)))
    return rc;
  const size_t n2 = 2 * (size_t)ctx->d.N;
  if (!U && dwh::q_supported(ctx->d.N) && (int64_t)n2 <= dwh::kEigMaxN) {
    // eigenvalues only: the structure-preserving reduction (half the
    // launches and a quarter of the pass traffic of the one-stage path)
    Scope sc(ctx, T_EIG_OWN, 1);
    ctx->eig_ph = false;
    ctx->eig_ph_last = 0;
    if ((rc = qeig_values(ctx, chains_src(ctx, chain), 1, nullptr))) return rc;
    HIPCHECK(ctx, hipMemsetAsync(ctx->d_tr_bad, 0, sizeof(int), ctx->stream));
    dwh::launch_nonfinite(ctx->tr.U, 0, ctx->tr.E, (int64_t)n2, ctx->d_tr_bad, ctx->stream);
    int bad = 0;
    HIPCHECK(ctx, hipMemcpyAsync(E, ctx->tr.E, n2 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(&bad, ctx->d_tr_bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    if (!bad) return DWH_OK;   // (non-finite eigenvalues: the full solve below)
  }
  if ((rc = eigen_solve(ctx, chains_src(ctx, chain), 1))) return rc;
  HIPCHECK(ctx, hipMemcpyAsync(E, ctx->tr.E, n2 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  if (U)
    HIPCHECK(ctx, hipMemcpyAsync(U, ctx->tr.U, n2 * n2 * sizeof(double2), hipMemcpyDeviceToHost,
                                 ctx->stream));
  return eigen_info_check(ctx, 1);
}

int dwh_measure_transport(dwh_ctx* ctx, int64_t chain, double eta, double domega, double omega_max,
                          double* stiffness, double* dc_cond, double* sigma, int64_t n_omega,
                          double* dos, double* dos_an, int64_t n_dos, double* ak0) {
  if (!ctx || !stiffness || !dc_cond || !ak0) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (chain < 0 || chain >= ctx->d.nc) return fail(ctx, DWH_ERR_ARG, "chain index out of range");
  int64_t nw = 0, nd = 0;
  int rc;
  if ((rc = transport_args(ctx, eta, domega, omega_max, n_omega, n_dos, &nw, &nd))) return rc;
  if ((nw > 0 && !sigma) || (nd > 0 && (!dos || !dos_an))) return fail(ctx, DWH_ERR_ARG, "NULL grid output");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  return transport_run(ctx, chains_src(ctx, chain), 1, eta, domega, omega_max, nw, nd, stiffness, dc_cond, sigma, dos, dos_an,
                       ak0);
}

int dwh_measure_transport_batched(dwh_ctx* ctx, double eta, double domega, double omega_max,
                                  double* stiffness, double* dc_cond, double* sigma, int64_t n_omega,
                                  double* dos, double* dos_an, int64_t n_dos, double* ak0) {
  if (!ctx || !stiffness || !dc_cond || !ak0) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  int64_t nw = 0, nd = 0;
  int rc;
  if ((rc = transport_args(ctx, eta, domega, omega_max, n_omega, n_dos, &nw, &nd))) return rc;
  if ((nw > 0 && !sigma) || (nd > 0 && (!dos || !dos_an))) return fail(ctx, DWH_ERR_ARG, "NULL grid output");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  // chains in groups whose three n2 x n2 work matrices fit in 16 GiB
  const int N = ctx->d.N, nc = ctx->d.nc;
  const double per = 3.0 * 16.0 * 4.0 * N * (double)N;
  const int group = std::max(1, std::min(nc, (int)(16.0 * (1 << 30) / per)));
  for (int c0 = 0; c0 < nc; c0 += group) {
    const int m = std::min(group, nc - c0);
    if ((rc = transport_run(ctx, chains_src(ctx, c0), m, eta, domega, omega_max, nw, nd, stiffness + c0, dc_cond + c0,
                            sigma ? sigma + (size_t)c0 * nw : nullptr, dos ? dos + (size_t)c0 * nd : nullptr,
                            dos_an ? dos_an + (size_t)c0 * nd : nullptr, ak0 + (size_t)c0 * N)))
      return rc;
  }
  return DWH_OK;
}

int dwh_measure_transport_deltas(dwh_ctx* ctx, int64_t chain, int64_t nstates, const dwh_c128* Delta,
                                 double eta, double domega, double omega_max, double* stiffness,
                                 double* dc_cond, double* sigma, int64_t n_omega, double* dos, double* dos_an,
                                 int64_t n_dos, double* ak0) {
  if (!ctx || !Delta || !stiffness || !dc_cond || !ak0) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (chain < 0 || chain >= ctx->d.nc) return fail(ctx, DWH_ERR_ARG, "chain index out of range");
  if (nstates < 1) return fail(ctx, DWH_ERR_ARG, "nstates must be >= 1");
  int64_t nw = 0, nd = 0;
  int rc;
  if ((rc = transport_args(ctx, eta, domega, omega_max, n_omega, n_dos, &nw, &nd))) return rc;
  if ((nw > 0 && !sigma) || (nd > 0 && (!dos || !dos_an))) return fail(ctx, DWH_ERR_ARG, "NULL grid output");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  const int N = ctx->d.N;
  const int64_t n2 = 2 * (int64_t)N;
  for (int64_t e = 0; e < nstates * n2; ++e)
    if (!std::isfinite(Delta[e].re) || !std::isfinite(Delta[e].im)) return fail(ctx, DWH_ERR_ARG, "non-finite Delta");
  // staging buffer for the snapshots (grown on demand)
  if (nstates > ctx->tr_nstage) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    drop_alloc(ctx, ctx->d_tr_stage);
    ctx->d_tr_stage = nullptr;
    ctx->tr_nstage = 0;
    if ((rc = dalloc(ctx, &ctx->d_tr_stage, (size_t)nstates * n2))) return rc;
    ctx->tr_nstage = nstates;
  }
  HIPCHECK(ctx, hipMemcpyAsync(ctx->d_tr_stage, Delta, (size_t)nstates * n2 * sizeof(double2),
                               hipMemcpyHostToDevice, ctx->stream));
  // groups whose three n2 x n2 work matrices fit in 16 GiB, as the batched call
  const double per = 3.0 * 16.0 * 4.0 * N * (double)N;
  const int group = std::max(1, std::min((int)nstates, (int)(16.0 * (1 << 30) / per)));
  for (int64_t s0 = 0; s0 < nstates; s0 += group) {
    const int m = (int)std::min<int64_t>(group, nstates - s0);
    const TrSrc src{ctx->d_tr_stage + s0 * n2, n2, chain, 0};
    if ((rc = transport_run(ctx, src, m, eta, domega, omega_max, nw, nd, stiffness + s0, dc_cond + s0,
                            sigma ? sigma + (size_t)s0 * nw : nullptr, dos ? dos + (size_t)s0 * nd : nullptr,
                            dos_an ? dos_an + (size_t)s0 * nd : nullptr, ak0 + (size_t)s0 * N)))
      return rc;
  }
  return DWH_OK;
}

int dwh_create(dwh_ctx** ctx, int64_t Lx, int64_t Ly, double t, double tp, double mu, double beta,
               double J, const int64_t* nn_table, const int64_t* nnn_table, const double* disorder,
               int32_t device) {
  return create_impl(ctx, Lx, Ly, t, tp, mu, beta, J, nn_table, nnn_table, 1, disorder, 0.0,
                     DWH_ALGO_AUTO, device);
}

int dwh_create_batched(dwh_ctx** ctx, int64_t Lx, int64_t Ly, double t, double tp, double mu,
                       double beta, double J, const int64_t* nn_table, const int64_t* nnn_table,
                       int64_t nchains, const double* disorder, double delta_cap, int32_t device) {
  return create_impl(ctx, Lx, Ly, t, tp, mu, beta, J, nn_table, nnn_table, nchains, disorder,
                     delta_cap, DWH_ALGO_AUTO, device);
}

int dwh_create_ex(dwh_ctx** ctx, int64_t Lx, int64_t Ly, double t, double tp, double mu, double beta,
                  double J, const int64_t* nn_table, const int64_t* nnn_table, int64_t nchains,
                  const double* disorder, double delta_cap, int32_t algo, int32_t device) {
  if (algo != DWH_ALGO_AUTO && algo != DWH_ALGO_DENSE && algo != DWH_ALGO_CR && algo != DWH_ALGO_EIG)
    return fail(nullptr, DWH_ERR_ARG, "algo must be DWH_ALGO_AUTO, DWH_ALGO_DENSE, DWH_ALGO_CR or DWH_ALGO_EIG");
  return create_impl(ctx, Lx, Ly, t, tp, mu, beta, J, nn_table, nnn_table, nchains, disorder,
                     delta_cap, algo, device);
}

void dwh_destroy(dwh_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto& r : ctx->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : ctx->pool) (void)hipEventDestroy(e);
  if (ctx->blas) (void)rocblas_destroy_handle(ctx->blas);
  if (ctx->q_graph) (void)hipGraphExecDestroy(ctx->q_graph);
  for (void* p : ctx->allocations) (void)hipFree(p);
  for (hipEvent_t ev : ctx->eig_ev)
    if (ev) (void)hipEventDestroy(ev);
  for (hipStream_t st : ctx->eig_sx)
    if (st) (void)hipStreamDestroy(st);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* dwh_last_error(const dwh_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int dwh_info(dwh_ctx* ctx, dwh_info_t* out) {
  if (!ctx || !out) return DWH_ERR_ARG;
  out->N = ctx->d.N;
  out->Np = ctx->d.Np;
  out->nchains = ctx->d.nc;
  out->npoles = ctx->algo == ALGO_EIG ? 0 : ctx->d.P;
  out->kappa = ctx->kappa;
  out->e_bound = ctx->Ebound;
  out->err_tanh = ctx->err_tanh;
  out->delta_cap = ctx->delta_cap;
  out->device_bytes = ctx->device_bytes;
  out->algo = ctx->algo;
  out->block = ctx->algo == ALGO_CR ? ctx->cr.BP : ctx->algo == ALGO_EIG ? 0 : kGJ;
  out->eig_half = ctx->eig_ph_last;
  out->eig_long_clusters = ctx->eig_long_clusters;
  out->eig_quat = ctx->eig_quat_last;
  return DWH_OK;
}

int dwh_debug_cr_stamps(dwh_ctx* ctx, int32_t inv_stage, uint64_t* out, int64_t nwg) {
  if (!ctx || !out || nwg < 1) return fail(ctx, DWH_ERR_ARG, "dwh_debug_cr_stamps: bad argument");
  if (ctx->algo != ALGO_CR) return fail(ctx, DWH_ERR_STATE, "dwh_debug_cr_stamps: CR path only");
#ifdef CR_STAMPS
  int key = -1, k = 0;
  for (const CrStage& st : ctx->plan.stages)
    if (st.kind == 0 && k++ == inv_stage) key = ctx->plan.inv_blk[st.first];
  if (key < 0) return fail(ctx, DWH_ERR_ARG, "dwh_debug_cr_stamps: no such inversion stage");
  if (int rc = settle(ctx)) return rc;
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (dwh::cr_stamps_arm(key) != 0) return fail(ctx, DWH_ERR_HIP, "dwh_debug_cr_stamps: arm");
  cr_enqueue(ctx);
  HIPCHECK(ctx, hipGetLastError());
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (dwh::cr_stamps_arm(-1) != 0 ||
      dwh::cr_stamps_read(reinterpret_cast<unsigned long long*>(out), (int)std::min<int64_t>(nwg, dwh::kCrStampWG)) != 0)
    return fail(ctx, DWH_ERR_HIP, "dwh_debug_cr_stamps: read");
  return DWH_OK;
#else
  (void)inv_stage;
  return fail(ctx, DWH_ERR_STATE, "dwh_debug_cr_stamps: not a -DCR_STAMPS build");
#endif
}

int dwh_bench_assembly(dwh_ctx* ctx, int64_t reps) {
  if (!ctx || reps < 0) return fail(ctx, DWH_ERR_ARG, "dwh_bench_assembly: bad argument");
  if (ctx->algo == ALGO_EIG) return fail(ctx, DWH_ERR_STATE, "dwh_bench_assembly: the eig path has no per-step assembly");
  if (int rc = settle(ctx)) return rc;
  for (int64_t r = 0; r < reps; ++r) assembly_enqueue(ctx);
  HIPCHECK(ctx, hipGetLastError());
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

namespace {

// Re-create the device side of `ctx` for |Δ_ij| <= new_cap: a new pole-table
// entry for the larger spectral bound E' = hmax + 2 new_cap, same lattice,
// disorder and algorithm; Δ, π, the throughput draws and the timing state
// carry over.  The context is left unfactorised.
int reselect_poles(dwh_ctx* ctx, double new_cap) {
  dwh_ctx* n = nullptr;
  const int32_t algo = ctx->algo == ALGO_CR ? DWH_ALGO_CR : ctx->algo == ALGO_EIG ? DWH_ALGO_EIG : DWH_ALGO_DENSE;
  int rc = create_impl(&n, ctx->Lx, ctx->Ly, ctx->t, ctx->tp, ctx->mu, ctx->beta, ctx->J,
                       ctx->nn_host.data(), ctx->nnn_host.data(), ctx->d.nc, ctx->dis_host.data(), new_cap,
                       algo, ctx->device);
  // a spectral bound beyond the pole table: the eigendecomposition path
  if (rc == DWH_ERR_TABLE)
    rc = create_impl(&n, ctx->Lx, ctx->Ly, ctx->t, ctx->tp, ctx->mu, ctx->beta, ctx->J, ctx->nn_host.data(),
                     ctx->nnn_host.data(), ctx->d.nc, ctx->dis_host.data(), new_cap, DWH_ALGO_EIG, ctx->device);
  if (rc != DWH_OK)
    return fail(ctx, rc, "pole re-selection for delta_cap=" + std::to_string(new_cap) + ": " + g_create_error);
  const size_t nb = (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2);
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(n->Delta, ctx->Delta, nb, hipMemcpyDeviceToDevice);
  if (e == hipSuccess) e = hipMemcpy(n->Pi, ctx->Pi, nb, hipMemcpyDeviceToDevice);
  if (e != hipSuccess) {
    dwh_destroy(n);
    return fail(ctx, DWH_ERR_HIP, std::string("pole re-selection: ") + hipGetErrorString(e));
  }
  // the throughput draws move with the context
  const size_t nbond = (size_t)ctx->d.nc * 2 * ctx->d.N, nc = ctx->d.nc, ns = (size_t)ctx->ndraws;
  auto move = [&](void* p, size_t bytes) {
    if (!p) return;
    auto it = std::find(ctx->allocations.begin(), ctx->allocations.end(), p);
    if (it != ctx->allocations.end()) ctx->allocations.erase(it);
    bytes = std::max<size_t>(bytes, 1);
    ctx->device_bytes -= (int64_t)bytes;
    n->allocations.push_back(p);
    n->device_bytes += (int64_t)bytes;
  };
  move(ctx->noise, nbond * ns * sizeof(double2));
  move(ctx->uniform, nc * ns * sizeof(double));
  move(ctx->acc, nc * ns);
  move(ctx->dH, nc * ns * sizeof(double));
  n->noise = ctx->noise;
  n->uniform = ctx->uniform;
  n->acc = ctx->acc;
  n->dH = ctx->dH;
  n->ndraws = ctx->ndraws;
  ctx->noise = nullptr;
  ctx->uniform = nullptr;
  ctx->acc = nullptr;
  ctx->dH = nullptr;
  ctx->ndraws = 0;
  n->timing = ctx->timing;
  std::copy(ctx->t_ms, ctx->t_ms + T_COUNT, n->t_ms);
  std::copy(ctx->t_n, ctx->t_n + T_COUNT, n->t_n);
  std::copy(ctx->t_work, ctx->t_work + T_COUNT, n->t_work);
  n->reselections = ctx->reselections + 1;
  // the context keeps its stream (a handle from dwh_stream stays valid); the
  // new device side's stream goes with the old one
  (void)hipStreamSynchronize(n->stream);
  std::swap(n->stream, ctx->stream);
  std::swap(*ctx, *n);
  if (ctx->blas) (void)rocblas_set_stream(ctx->blas, ctx->stream);
  dwh_destroy(n);
  return DWH_OK;
}

// Host-side guard for an uploaded Δ: re-select the poles when max|Δ_ij| (bond
// guard) or the largest mean |Δ| over a site's bonds (site guard) is above
// the cap (the reference accepts any Δ, src/HMC.jl:98-114).
int fit_cap(dwh_ctx* ctx, const dwh_c128* D, size_t n, bool* reselected = nullptr) {
  if (reselected) *reselected = false;
  double m = 0;
  for (size_t k = 0; k < n; ++k) {
    const double a = std::hypot(D[k].re, D[k].im);
    if (!std::isfinite(a)) return fail(ctx, DWH_ERR_ARG, "non-finite Delta");
    m = std::max(m, a);
  }
  if (ctx->site_guard) {
    const size_t N = (size_t)ctx->d.N, nc = n / (2 * N);
    m = 0;
    for (size_t c = 0; c < nc; ++c)
      for (size_t i = 0; i < N; ++i) {
        double sm = 0;
        for (int k = 0; k < 4; ++k) {
          const dwh_c128 v = D[c * 2 * N + ctx->site4_host[4 * i + k]];
          sm += std::hypot(v.re, v.im);
        }
        m = std::max(m, 0.25 * sm);
      }
  }
  if (m <= ctx->delta_cap) return DWH_OK;
  if (reselected) *reselected = true;
  return reselect_poles(ctx, std::max(2.0 * ctx->delta_cap, 1.5 * m));
}

// Reads and clears the device guard flag (set by the drift kernels when
// max|Δ_ij| > delta_cap).
int take_flag(dwh_ctx* ctx, int* f) {
  *f = 0;
  HIPCHECK(ctx, hipMemcpyAsync(f, ctx->flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (*f) HIPCHECK(ctx, hipMemsetAsync(ctx->flag, 0, sizeof(int), ctx->stream));
  return DWH_OK;
}

// A sweep drifted |Δ| past the cap, so its forces used poles not valid for
// its spectrum: back to the sweep's starting point (Δ backed up by k_backup,
// src/HMC.jl:84), re-select the poles for twice the cap and refactorise, so
// the caller can run the same sweep again.
constexpr int kMaxReselect = 12;
int redo_after_guard(dwh_ctx* ctx, int attempt) {
  if (attempt >= kMaxReselect)
    return fail(ctx, DWH_ERR_SPECTRUM, "|Delta_ij| kept exceeding the re-selected pole sets");
  const size_t nb = (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2);
  HIPCHECK(ctx, hipMemcpyAsync(ctx->Delta, ctx->DeltaB, nb, hipMemcpyDeviceToDevice, ctx->stream));
  int rc = reselect_poles(ctx, 2.0 * ctx->delta_cap);
  if (rc != DWH_OK) return rc;
  return dwh_factorize(ctx);
}

// one logged throughput sweep (sequence number = its index in ctx->enq)
void enqueue_logged(dwh_ctx* ctx, int64_t sw, int64_t Nt, double dt, double mass) {
  const Dims& d = ctx->d;
  const size_t nbond = (size_t)d.nc * 2 * d.N;
  const dwh::SweepHalt sh{ctx->halt, (int)ctx->enq.size(), ctx->flag};
  ctx->enq.push_back({sw, Nt, dt, mass});
  sweep_enqueue(ctx, ctx->noise + nbond * sw, ctx->uniform + (size_t)d.nc * sw, ctx->acc + (size_t)d.nc * sw,
                ctx->dH + (size_t)d.nc * sw, Nt, dt, mass, sh);
}

// Waits for the enqueued throughput sweeps.  A guard trip in one of them
// (k_traj_end recorded its sequence number t, every later sweep of the batch
// was a no-op that kept the backups): Δ back to sweep t's start, poles
// re-selected for twice the cap, refactorised — exactly what dwh_hmc_sweep
// does for a trip — and sweeps t.. enqueued again, until a pass ends without
// a trip.  The results then equal the single-sweep path's bit for bit.
int settle(dwh_ctx* ctx) {
  for (int attempt = 0;; ++attempt) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    if (int rc = eig_check(ctx)) return rc;
    int f = 0;
    if (int rc = take_flag(ctx, &f)) return rc;
    if (!f) {
      ctx->enq.clear();
      return DWH_OK;
    }
    int h[2] = {0, 0};
    HIPCHECK(ctx, hipMemcpy(h, ctx->halt, sizeof h, hipMemcpyDeviceToHost));
    if (!h[0] || h[1] < 0 || h[1] >= (int)ctx->enq.size()) {
      ctx->enq.clear();
      char buf[256];
      std::snprintf(buf, sizeof buf,
                    "%s exceeded delta_cap=%g outside a logged sweep (the pole set was built for spectra "
                    "within E'=%g)",
                    ctx->site_guard ? "the mean |Delta| of a site's bonds" : "|Delta_ij|", ctx->delta_cap,
                    ctx->Ebound);
      return fail(ctx, DWH_ERR_SPECTRUM, buf);
    }
    const std::vector<dwh_ctx::EnqSweep> rest(ctx->enq.begin() + h[1], ctx->enq.end());
    ctx->enq.clear();
    HIPCHECK(ctx, hipMemsetAsync(ctx->halt, 0, 2 * sizeof(int), ctx->stream));
    if (int rc = redo_after_guard(ctx, attempt)) return rc;
    for (const auto& e : rest) enqueue_logged(ctx, e.sweep, e.Nt, e.dt, e.mass);
    HIPCHECK(ctx, hipGetLastError());
  }
}

}  // namespace

int dwh_update_pairing(dwh_ctx* ctx, const dwh_c128* Delta) {
  if (!ctx || !Delta) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  if (int rc = fit_cap(ctx, Delta, (size_t)ctx->d.nc * 2 * ctx->d.N)) return rc;
  HIPCHECK(ctx, hipMemcpyAsync(ctx->Delta, Delta, (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2),
                               hipMemcpyHostToDevice, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_factorize(dwh_ctx* ctx) {
  if (!ctx) return DWH_ERR_ARG;
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  factorize_enqueue(ctx, kickdrift(ctx, 0.0, 0.0));
  fermion_energy_enqueue(ctx);
  HIPCHECK(ctx, hipGetLastError());
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (int rc = eig_check(ctx)) return rc;
  ctx->factorized = true;
  drain_timing(ctx);
  return DWH_OK;
}

int dwh_forces(dwh_ctx* ctx, const dwh_c128* Delta, dwh_c128* F_out) {
  if (!ctx || !F_out) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  const size_t nb = (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2);
  if (Delta)
    HIPCHECK(ctx, hipMemcpyAsync(ctx->DeltaB, Delta, nb, hipMemcpyHostToDevice, ctx->stream));
  dwh::launch_force_from_pair(ctx->d, ctx->Pair, Delta ? ctx->DeltaB : ctx->Delta, ctx->F, ctx->Pi,
                              kickdrift(ctx, 0.0, 0.0), ctx->beta, ctx->J, ctx->stream);
  HIPCHECK(ctx, hipMemcpyAsync(F_out, ctx->F, nb, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_pairing(dwh_ctx* ctx, dwh_c128* P_out) {
  if (!ctx || !P_out) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  HIPCHECK(ctx, hipMemcpyAsync(P_out, ctx->Pair, (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2),
                               hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_fermion_energy(dwh_ctx* ctx, double* Ef) {
  if (!ctx || !Ef) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  HIPCHECK(ctx, hipMemcpyAsync(Ef, ctx->Ef, ctx->d.nc * sizeof(double), hipMemcpyDeviceToHost,
                               ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_hole_trace(dwh_ctx* ctx, double* tr) {
  if (!ctx || !tr) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  HIPCHECK(ctx, hipMemcpyAsync(tr, ctx->Trhh, ctx->d.nc * sizeof(double), hipMemcpyDeviceToHost,
                               ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_total_energy(dwh_ctx* ctx, double mass, double* H) {
  if (!ctx || !H) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  dwh::launch_total_energy(ctx->d, ctx->Delta, ctx->Pi, ctx->Ef, ctx->beta, ctx->J, mass, ctx->Hnew,
                           ctx->stream);
  HIPCHECK(ctx, hipMemcpyAsync(H, ctx->Hnew, ctx->d.nc * sizeof(double), hipMemcpyDeviceToHost,
                               ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_set_state(dwh_ctx* ctx, const dwh_c128* Delta, const dwh_c128* pi) {
  if (!ctx) return DWH_ERR_ARG;
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  const size_t nb = (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2);
  bool reselected = false;
  if (Delta)
    if (int rc = fit_cap(ctx, Delta, (size_t)ctx->d.nc * 2 * ctx->d.N, &reselected)) return rc;
  if (Delta) HIPCHECK(ctx, hipMemcpyAsync(ctx->Delta, Delta, nb, hipMemcpyHostToDevice, ctx->stream));
  if (pi) HIPCHECK(ctx, hipMemcpyAsync(ctx->Pi, pi, nb, hipMemcpyHostToDevice, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  // a re-selected context has no factorisation yet: the cached P / E_f the next
  // sweep starts from must belong to this Δ
  if (reselected) return dwh_factorize(ctx);
  return DWH_OK;
}

int dwh_get_state(dwh_ctx* ctx, dwh_c128* Delta, dwh_c128* pi) {
  if (!ctx) return DWH_ERR_ARG;
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  SETTLE(ctx);
  const size_t nb = (size_t)ctx->d.nc * 2 * ctx->d.N * sizeof(double2);
  if (Delta) HIPCHECK(ctx, hipMemcpyAsync(Delta, ctx->Delta, nb, hipMemcpyDeviceToHost, ctx->stream));
  if (pi) HIPCHECK(ctx, hipMemcpyAsync(pi, ctx->Pi, nb, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_hmc_sweep(dwh_ctx* ctx, const dwh_c128* noise, const double* uniform, int64_t Nt, double dt,
                  double mass, uint8_t* accepted, double* dH) {
  if (!ctx || !noise || !uniform || !accepted || !dH) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (Nt < 0 || !(mass > 0) || !std::isfinite(dt)) return fail(ctx, DWH_ERR_ARG, "bad Nt/dt/mass");
  if (ctx->pending) return fail(ctx, DWH_ERR_STATE, "dwh_hmc_finish the pending trajectory first");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  if (!ctx->enq.empty())
    if (int rc = settle(ctx)) return rc;
  for (int attempt = 0;; ++attempt) {
    const Dims& d = ctx->d;
    HIPCHECK(ctx, hipMemcpyAsync(ctx->s_noise, noise, (size_t)d.nc * 2 * d.N * sizeof(double2),
                                 hipMemcpyHostToDevice, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(ctx->s_uniform, uniform, d.nc * sizeof(double), hipMemcpyHostToDevice,
                                 ctx->stream));
    sweep_enqueue(ctx, ctx->s_noise, ctx->s_uniform, ctx->s_acc, ctx->s_dH, Nt, dt, mass);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipMemcpyAsync(accepted, ctx->s_acc, d.nc, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(dH, ctx->s_dH, d.nc * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    if (int rc = eig_check(ctx)) return rc;
    if (Nt > 0) ctx->factorized = true;
    drain_timing(ctx);
    int f = 0;
    if (int rc = take_flag(ctx, &f)) return rc;
    if (!f) return DWH_OK;
    if (int rc = redo_after_guard(ctx, attempt)) return rc;
  }
}

int dwh_hmc_trajectory(dwh_ctx* ctx, const dwh_c128* noise, int64_t Nt, double dt, double mass,
                       double* dH) {
  if (!ctx || !noise || !dH) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (Nt < 0 || !(mass > 0) || !std::isfinite(dt)) return fail(ctx, DWH_ERR_ARG, "bad Nt/dt/mass");
  if (ctx->pending) return fail(ctx, DWH_ERR_STATE, "dwh_hmc_finish the pending trajectory first");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  if (!ctx->enq.empty())
    if (int rc = settle(ctx)) return rc;
  for (int attempt = 0;; ++attempt) {
    const Dims& d = ctx->d;
    HIPCHECK(ctx, hipMemcpyAsync(ctx->s_noise, noise, (size_t)d.nc * 2 * d.N * sizeof(double2),
                                 hipMemcpyHostToDevice, ctx->stream));
    // ΔH by the Metropolis kernel's own arithmetic (src/HMC.jl:124), with a
    // uniform of 2 > exp(-ΔH) for ΔH >= 0: its accept flags are not used
    std::vector<double> two((size_t)d.nc, 2.0);
    HIPCHECK(ctx, hipMemcpyAsync(ctx->s_uniform, two.data(), d.nc * sizeof(double), hipMemcpyHostToDevice,
                                 ctx->stream));
    trajectory_enqueue(ctx, ctx->s_noise, Nt, dt, mass);
    dwh::launch_metropolis(d, ctx->Hold, ctx->Hnew, ctx->s_uniform, ctx->s_acc, ctx->s_dH, ctx->stream);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipMemcpyAsync(dH, ctx->s_dH, d.nc * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    if (int rc = eig_check(ctx)) return rc;
    if (Nt > 0) ctx->factorized = true;
    drain_timing(ctx);
    int f = 0;
    if (int rc = take_flag(ctx, &f)) return rc;
    if (!f) {
      ctx->pending = true;
      return DWH_OK;
    }
    if (int rc = redo_after_guard(ctx, attempt)) return rc;
  }
}

int dwh_hmc_finish(dwh_ctx* ctx, const uint8_t* accepted) {
  if (!ctx || !accepted) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (!ctx->pending) return fail(ctx, DWH_ERR_STATE, "no pending trajectory (dwh_hmc_trajectory first)");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  const Dims& d = ctx->d;
  HIPCHECK(ctx, hipMemcpyAsync(ctx->s_acc, accepted, d.nc, hipMemcpyHostToDevice, ctx->stream));
  dwh::launch_restore(d, ctx->s_acc, ctx->DeltaB, ctx->PairB, ctx->EfB, ctx->TrhhB, ctx->Delta,  // :130-141
                      ctx->Pair, ctx->Ef, ctx->Trhh, ctx->stream);
  HIPCHECK(ctx, hipGetLastError());
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  ctx->pending = false;
  return DWH_OK;
}

int dwh_load_draws(dwh_ctx* ctx, int64_t nsweeps, const dwh_c128* noise, const double* uniform) {
  if (!ctx || nsweeps < 1 || !noise || !uniform) return fail(ctx, DWH_ERR_ARG, "bad argument");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  // pending throughput sweeps replay from the loaded draws after a guard trip
  // (settle): finish them before the draws are replaced
  SETTLE(ctx);
  const Dims& d = ctx->d;
  const size_t nbond = (size_t)d.nc * 2 * d.N;
  if (nsweeps > ctx->ndraws) {
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    auto drop = [&](void* p, size_t bytes) {
      if (!p) return;
      auto it = std::find(ctx->allocations.begin(), ctx->allocations.end(), p);
      if (it != ctx->allocations.end()) ctx->allocations.erase(it);
      ctx->device_bytes -= (int64_t)std::max<size_t>(bytes, 1);
      (void)hipFree(p);
    };
    // allocate the new buffers first and swap them in only when all of them
    // exist, so a failed allocation leaves the old draws (and ndraws) intact
    double2* nz = nullptr;
    double* un = nullptr;
    uint8_t* ac = nullptr;
    double* dh = nullptr;
    const size_t ns = (size_t)nsweeps, nc = (size_t)d.nc;
    int rc = dalloc(ctx, &nz, nbond * ns);
    if (rc == DWH_OK) rc = dalloc(ctx, &un, nc * ns);
    if (rc == DWH_OK) rc = dalloc(ctx, &ac, nc * ns);
    if (rc == DWH_OK) rc = dalloc(ctx, &dh, nc * ns);
    const size_t old = (size_t)ctx->ndraws;
    if (rc != DWH_OK) {
      drop(nz, nbond * ns * sizeof(double2));
      drop(un, nc * ns * sizeof(double));
      drop(ac, nc * ns);
      drop(dh, nc * ns * sizeof(double));
      return rc;
    }
    drop(ctx->noise, nbond * old * sizeof(double2));
    drop(ctx->uniform, nc * old * sizeof(double));
    drop(ctx->acc, nc * old);
    drop(ctx->dH, nc * old * sizeof(double));
    ctx->noise = nz;
    ctx->uniform = un;
    ctx->acc = ac;
    ctx->dH = dh;
  }
  ctx->ndraws = std::max<int64_t>(ctx->ndraws, nsweeps);
  HIPCHECK(ctx, hipMemcpyAsync(ctx->noise, noise, nbond * nsweeps * sizeof(double2),
                               hipMemcpyHostToDevice, ctx->stream));
  HIPCHECK(ctx, hipMemcpyAsync(ctx->uniform, uniform, (size_t)d.nc * nsweeps * sizeof(double),
                               hipMemcpyHostToDevice, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_run_sweeps(dwh_ctx* ctx, int64_t first, int64_t nsweeps, int64_t Nt, double dt, double mass) {
  if (!ctx) return DWH_ERR_ARG;
  if (first < 0 || nsweeps < 0 || first + nsweeps > ctx->ndraws)
    return fail(ctx, DWH_ERR_ARG, "sweep range outside the loaded draws");
  if (Nt < 0 || !(mass > 0)) return fail(ctx, DWH_ERR_ARG, "bad Nt/mass");
  if (ctx->pending) return fail(ctx, DWH_ERR_STATE, "dwh_hmc_finish the pending trajectory first");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  const Dims& d = ctx->d;
  const size_t nbond = (size_t)d.nc * 2 * d.N;
  (void)d;
  (void)nbond;
  for (int64_t sw = first; sw < first + nsweeps; ++sw) enqueue_logged(ctx, sw, Nt, dt, mass);
  HIPCHECK(ctx, hipGetLastError());
  if (Nt > 0 && nsweeps > 0) ctx->factorized = true;
  return DWH_OK;
}

int dwh_sweep_results(dwh_ctx* ctx, int64_t first, int64_t nsweeps, uint8_t* accepted, double* dH) {
  if (!ctx) return DWH_ERR_ARG;
  if (first < 0 || nsweeps < 0 || first + nsweeps > ctx->ndraws)
    return fail(ctx, DWH_ERR_ARG, "sweep range outside the loaded draws");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  if (int rc = settle(ctx)) return rc;
  const size_t nc = ctx->d.nc;
  if (accepted)
    HIPCHECK(ctx, hipMemcpyAsync(accepted, ctx->acc + nc * first, nc * nsweeps, hipMemcpyDeviceToHost,
                                 ctx->stream));
  if (dH)
    HIPCHECK(ctx, hipMemcpyAsync(dH, ctx->dH + nc * first, nc * nsweeps * sizeof(double),
                                 hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  return DWH_OK;
}

int dwh_synchronize(dwh_ctx* ctx) {
  if (!ctx) return DWH_ERR_ARG;
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  if (int rc = settle(ctx)) return rc;
  HIPCHECK(ctx, hipGetLastError());
  drain_timing(ctx);
  return DWH_OK;
}

int dwh_stream(dwh_ctx* ctx, void** stream) {
  if (!ctx || !stream) return DWH_ERR_ARG;
  *stream = (void*)ctx->stream;
  return DWH_OK;
}

int dwh_timing_enable(dwh_ctx* ctx, int32_t enable) {
  if (!ctx) return DWH_ERR_ARG;
  drain_timing(ctx);
  ctx->timing = enable;
  return DWH_OK;
}

int dwh_timing_read(dwh_ctx* ctx, const char* name, double* total_ms, int64_t* launches,
                    double* work) {
  if (!ctx || !name) return DWH_ERR_ARG;
  drain_timing(ctx);
  for (int i = 0; i < T_COUNT; ++i)
    if (std::strcmp(name, kTimerNames[i]) == 0) {
      if (total_ms) *total_ms = ctx->t_ms[i];
      if (launches) *launches = ctx->t_n[i];
      if (work) *work = ctx->t_work[i];
      return DWH_OK;
    }
  return fail(ctx, DWH_ERR_ARG, std::string("unknown timer ") + name);
}

int dwh_timing_reset(dwh_ctx* ctx) {
  if (!ctx) return DWH_ERR_ARG;
  drain_timing(ctx);
  for (int i = 0; i < T_COUNT; ++i) {
    ctx->t_ms[i] = 0;
    ctx->t_n[i] = 0;
    ctx->t_work[i] = 0;
  }
  return DWH_OK;
}

int dwh_selftest_mfma(int32_t device) { return dwh::selftest_mfma_layout(device); }

int dwh_debug_gemm(int32_t device, int32_t cplx, char opa, char opb, int64_t M, int64_t N, int64_t K,
                   const double* alpha, const void* A, int64_t lda, const void* B, int64_t ldb, const double* beta,
                   void* C, int64_t ldc, int64_t batch) {
  if (M < 1 || N < 1 || K < 0 || batch < 1 || !alpha || !beta || !A || !B || !C)
    return fail(nullptr, DWH_ERR_ARG, "bad gemm arguments");
  if ((opa != 'N' && opa != 'C') || (opb != 'N' && opb != 'C'))
    return fail(nullptr, DWH_ERR_ARG, "op must be 'N' or 'C'");
  const int64_t acols = opa == 'N' ? K : M, bcols = opb == 'N' ? N : K;
  const int64_t arows = opa == 'N' ? M : K, brows = opb == 'N' ? K : N;
  if (lda < std::max<int64_t>(1, arows) || ldb < std::max<int64_t>(1, brows) || ldc < M)
    return fail(nullptr, DWH_ERR_ARG, "leading dimension too small");
  const size_t es = cplx ? sizeof(double2) : sizeof(double);
  const int64_t sA = lda * std::max<int64_t>(acols, 1), sB = ldb * std::max<int64_t>(bcols, 1), sC = ldc * N;
  if (hipSetDevice(device) != hipSuccess) return fail(nullptr, DWH_ERR_HIP, "hipSetDevice failed");
  void *dA = nullptr, *dB = nullptr, *dC = nullptr;
  auto cleanup = [&]() {
    (void)hipFree(dA);
    (void)hipFree(dB);
    (void)hipFree(dC);
  };
  if (hipMalloc(&dA, es * sA * batch) != hipSuccess || hipMalloc(&dB, es * sB * batch) != hipSuccess ||
      hipMalloc(&dC, es * sC * batch) != hipSuccess) {
    cleanup();
    return fail(nullptr, DWH_ERR_HIP, "hipMalloc (gemm test buffers)");
  }
  hipError_t e = hipMemcpy(dA, A, es * sA * batch, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dB, B, es * sB * batch, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dC, C, es * sC * batch, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    if (cplx)
      dwh::gemm_z(opa, opb, (int)M, (int)N, (int)K, make_double2(alpha[0], alpha[1]), (const double2*)dA, (int)lda,
                  sA, (const double2*)dB, (int)ldb, sB, make_double2(beta[0], beta[1]), (double2*)dC, (int)ldc, sC,
                  (int)batch, nullptr);
    else
      dwh::gemm_d(opa == 'C' ? 'T' : 'N', opb == 'C' ? 'T' : 'N', (int)M, (int)N, (int)K, alpha[0],
                  (const double*)dA, (int)lda, sA, (const double*)dB, (int)ldb, sB, beta[0], (double*)dC, (int)ldc,
                  sC, (int)batch, nullptr);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(C, dC, es * sC * batch, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) return fail(nullptr, DWH_ERR_HIP, std::string("gemm test: ") + hipGetErrorString(e));
  return DWH_OK;
}

}  // extern "C"

namespace {
// hopping columns (kHSlots per site: the site, then its NN / NNN partners in
// build_hrow's order) of a periodic Lx x Ly lattice with the reference's
// tables (src/Types.jl:60-80): what dwh_create derives from ModelParameters
std::vector<int> standard_hcol(int Lx, int Ly) {
  const int N = Lx * Ly;
  std::vector<int64_t> nn((size_t)4 * N), nnn((size_t)4 * N);
  auto idx = [&](int x, int y) { return (int64_t)(((y % Ly + Ly) % Ly) * Lx + ((x % Lx + Lx) % Lx)) + 1; };
  for (int y = 0; y < Ly; ++y)
    for (int x = 0; x < Lx; ++x) {
      const int i = y * Lx + x;
      nn[0 * N + i] = idx(x + 1, y);
      nn[1 * N + i] = idx(x, y + 1);
      nn[2 * N + i] = idx(x - 1, y);
      nn[3 * N + i] = idx(x, y - 1);
      nnn[0 * N + i] = idx(x + 1, y + 1);
      nnn[1 * N + i] = idx(x - 1, y + 1);
      nnn[2 * N + i] = idx(x - 1, y - 1);
      nnn[3 * N + i] = idx(x + 1, y - 1);
    }
  const auto hrow = build_hrow(N, 1.0, -0.35, nn.data(), nnn.data());
  std::vector<int> hcol((size_t)N * kHSlots, -1);
  for (int i = 0; i < N; ++i) {
    hcol[(size_t)i * kHSlots] = i;
    for (size_t k = 0; k < hrow[i].size() && k + 1 < (size_t)kHSlots; ++k) hcol[(size_t)i * kHSlots + 1 + k] = hrow[i][k].first;
  }
  return hcol;
}

// pairing columns (+x, +y, -x, -y) of every site of a periodic Lx x Ly lattice
std::vector<int> nn_pairing_cols(int Lx, int Ly) {
  const int N = Lx * Ly;
  std::vector<int> Dcol((size_t)N * kSlots);
  for (int i = 0; i < N; ++i) {
    const int x = i % Lx, y = i / Lx;
    Dcol[(size_t)i * kSlots + 0] = y * Lx + (x + 1) % Lx;
    Dcol[(size_t)i * kSlots + 1] = ((y + 1) % Ly) * Lx + x;
    Dcol[(size_t)i * kSlots + 2] = y * Lx + (x - 1 + Lx) % Lx;
    Dcol[(size_t)i * kSlots + 3] = ((y - 1 + Ly) % Ly) * Lx + x;
  }
  return Dcol;
}
}  // namespace

extern "C" {

// ---- host-only check of the CR schedule (no device) -------------------------
// Builds the plan dwh_create would for an Lx x Ly periodic lattice (NN pairing
// bonds) and nbatch = chains x poles batch items, then checks its dataflow:
// every block a stage reads is a level-0 / static block or was written by an
// EARLIER stage (launches are stream ordered, workgroups of one launch are
// not), no block is read and written in one stage except a task's own
// accumulate input, no two tasks of a stage write the same block, and every
// block the force / E_f gather reads was written.
int dwh_debug_cr_plan_check(int64_t Lx, int64_t Ly, int64_t nbatch, int32_t side, int32_t inv0, int64_t* stats) {
  if (Lx < 1 || Ly < 1 || nbatch < 1) return fail(nullptr, DWH_ERR_ARG, "bad lattice / batch");
  std::vector<int> Dcol = nn_pairing_cols((int)Lx, (int)Ly);
  if (!dwh::cr_supported_bp((int)(2 * ((Lx + 15) / 16 * 16))))
    return fail(nullptr, DWH_ERR_ARG, "lattice row too wide for the CR path");
  const int rows = cr_rows_per_block(Lx, Ly), Lxc = (int)Lx * rows, Lyc = (int)Ly / rows;
  const int BP = 2 * ((Lxc + 15) / 16 * 16);
  const std::vector<int> hcol = standard_hcol((int)Lx, (int)Ly);
  const CrPlan pl = build_cr_plan(Lxc, Lyc, BP, Dcol, side && dwh::cr_supported_side(BP), (int)nbatch,
                                  256, inv0 && dwh::cr_supported_inv0(BP), &hcol);
  if (const char* e = std::getenv("DWHMC_CR_PLAN_DUMP"); e && *e == '1') {
    int i = 0;
    for (const CrStage& st : pl.stages) {
      if (st.kind == 0)
        std::fprintf(stderr, "cr stage %2d: inv%s blocks=%d (x%lld wg) side_tasks=%d maxt32=%d side_flops/item=%.3g\n", i,
                     st.l0 ? "0 " : "  ", st.n, (long long)nbatch, st.ntiles, st.maxt32, st.flops);
      else if (st.kind == 2)
        std::fprintf(stderr, "cr stage %2d: sparse %s tasks=%d flops/item=%.3g\n", i, st.sp ? "bwd" : "fwd", st.n,
                     st.flops);
      else
        std::fprintf(stderr, "cr stage %2d: gemm  tasks=%d maxt32=%d maxt16=%d ntmax=%d flops/item=%.3g ntiles=%d\n", i,
                     st.n, st.maxt32, st.maxt16, st.ntmax, st.flops, st.ntiles);
      ++i;
    }
  }
  std::vector<int> written(pl.nblk, -1);   // stage of the first write; -2: ready from the start
  for (int b = 0; b < 3 * Lyc && b < pl.nblk; ++b) written[b] = -2;
  for (int r : pl.inv0_r) written[r] = -2;
  int64_t nside = 0, ninv = 0, ngemm = 0, ntask = 0;
  char buf[256];
  // 16 x 16 tiles written so far (block, tile row, tile column): product
  // stages write only their tile lists (restricted level-0 G blocks);
  // inversions and side-work tasks whole blocks (whole[b])
  const int ntc = BP / 16;
  std::set<std::pair<int, int>> tiles_written;   // (block, tr * ntc + tc)
  std::vector<char> whole(pl.nblk, 0);
  for (int b = 0; b < pl.nblk; ++b) whole[b] = written[b] == -2;
  for (int si = 0; si < (int)pl.stages.size(); ++si) {
    const CrStage& st = pl.stages[si];
    if (st.kind == 0) {
      for (int k = 0; k < st.n; ++k) whole[pl.inv_dst[st.first + k]] = 1;
      for (int k = 0; k < st.ntiles; ++k) whole[pl.tasks[st.tfirst + k].out] = 1;
    } else if (st.kind == 2) {
      for (int k = 0; k < st.n; ++k) {
        if (st.sp == 0) {
          const dwh::CrSpFwd& t = pl.sp_fwd[st.first + k];
          whole[t.od] = whole[t.ou] = whole[t.ol] = 1;
        } else {
          const dwh::CrSpBwd& t = pl.sp_bwd[st.first + k];
          whole[t.oza] = whole[t.ozc] = whole[t.oya] = whole[t.oyc] = whole[t.omx] = 1;
        }
      }
    } else {
      for (int k = 0; k < st.ntiles; ++k) {
        const dwh::CrTile& t = pl.tiles16[st.tfirst + k];
        tiles_written.insert({t.out, t.tr * ntc + t.tc});
      }
    }
    std::vector<std::pair<int, int>> rd;   // (block, task id or -1)
    std::vector<std::pair<int, int>> wr;
    // ids: task k -> k (its accumulate input may be its output), its
    // operands -> k + 2^20 (never its output); inversion entry k -> -1 - k
    // (in place: reads and writes its own block)
    auto add_task = [&](const dwh::CrTask& t, int id) {
      for (int h = 0; h < t.nt; ++h) {
        rd.push_back({t.a[h], id + (1 << 20)});
        rd.push_back({t.b[h], id + (1 << 20)});
      }
      if (t.cin >= 0) rd.push_back({t.cin, id});
      wr.push_back({t.out, id});
    };
    if (st.kind == 0) {
      ++ninv;
      for (int k = 0; k < st.n; ++k) {
        rd.push_back({pl.inv_blk[st.first + k], -1 - k});
        wr.push_back({pl.inv_dst[st.first + k], -1 - k});
      }
      if (st.ntiles > 0) ++nside;
      for (int k = 0; k < st.ntiles; ++k) add_task(pl.tasks[st.tfirst + k], k);
    } else if (st.kind == 2) {
      ++ngemm;
      for (int k = 0; k < st.n; ++k) {
        const int id = k + (1 << 21);
        if (st.sp == 0) {
          const dwh::CrSpFwd& t = pl.sp_fwd[st.first + k];
          for (int b : {t.dk, t.uk, t.lk, t.uel, t.lel, t.uer, t.ler, t.dir, t.dil}) rd.push_back({b, id});
          for (int b : {t.od, t.ou, t.ol}) wr.push_back({b, id});
        } else {
          const dwh::CrSpBwd& t = pl.sp_bwd[st.first + k];
          for (int b : {t.gaa, t.gac, t.gca, t.gcc, t.ua, t.le, t.la, t.ue}) rd.push_back({b, id});
          for (int b : {t.oza, t.ozc, t.oya, t.oyc, t.omx}) wr.push_back({b, id});
        }
      }
    } else {
      ++ngemm;
      for (int k = 0; k < st.n; ++k) add_task(pl.tasks[st.first + k], k);
    }
    ntask += (int64_t)wr.size();
    for (const auto& r : rd) {
      if (r.first < 0 || r.first >= pl.nblk || written[r.first] == -1) {
        std::snprintf(buf, sizeof buf, "stage %d reads block %d before any stage writes it", si, r.first);
        return fail(nullptr, DWH_ERR_STATE, buf);
      }
      for (const auto& w : wr)
        if (w.first == r.first && w.second != r.second) {
          std::snprintf(buf, sizeof buf, "stage %d reads block %d that the same stage writes", si, r.first);
          return fail(nullptr, DWH_ERR_STATE, buf);
        }
    }
    for (size_t i = 0; i < wr.size(); ++i)
      for (size_t j = i + 1; j < wr.size(); ++j)
        if (wr[i].first == wr[j].first && wr[i].second != wr[j].second) {
          std::snprintf(buf, sizeof buf, "stage %d writes block %d from two tasks", si, wr[i].first);
          return fail(nullptr, DWH_ERR_STATE, buf);
        }
    for (const auto& w : wr) {
      // level-0 blocks (refilled only at their pairing entries) and the static
      // R = A^-1 blocks of k_cr_inv0 are read on every step: nothing may
      // overwrite them
      if (w.first >= 0 && w.first < pl.nblk && written[w.first] == -2) {
        std::snprintf(buf, sizeof buf, "stage %d overwrites static block %d", si, w.first);
        return fail(nullptr, DWH_ERR_STATE, buf);
      }
      if (w.first >= 0 && w.first < pl.nblk && written[w.first] == -1) written[w.first] = si;
    }
  }
  const int64_t BB = (int64_t)(BP / 2) * BP;
  // the gathers read entries of tiles some stage wrote (the level-0 backward
  // stages compute only the tiles of their need sets, build_cr_plan)
  auto tile_ok = [&](int64_t o) {
    const int b = (int)(o / BB), r = (int)((o % BB) / BP), col = (int)(o % BP);
    return whole[b] || tiles_written.count({b, (r / 16) * ntc + col / 16}) > 0;
  };
  for (int64_t o : pl.goff)
    if (o >= 0 && (written[o / BB] == -1 || !tile_ok(o)))
      return fail(nullptr, DWH_ERR_STATE, "force gather reads an unwritten block / tile");
  for (int64_t o : pl.doff)
    if (written[o / BB] == -1 || !tile_ok(o)) return fail(nullptr, DWH_ERR_STATE, "E_f gather reads an unwritten block / tile");
  if (stats) {
    stats[0] = (int64_t)pl.stages.size();
    stats[1] = ninv;
    stats[2] = nside;
    stats[3] = ngemm;
    stats[4] = ntask;
    stats[5] = pl.nblk;
  }
  return DWH_OK;
}

int dwh_debug_cr_plan_flops(int64_t Lx, int64_t Ly, int64_t nbatch, int32_t side, int32_t inv0, double* flops) {
  if (Lx < 1 || Ly < 1 || nbatch < 1 || !flops) return fail(nullptr, DWH_ERR_ARG, "bad lattice / batch / output");
  if (!dwh::cr_supported_bp((int)(2 * ((Lx + 15) / 16 * 16))))
    return fail(nullptr, DWH_ERR_ARG, "lattice row too wide for the CR path");
  const int rows = cr_rows_per_block(Lx, Ly), Lxc = (int)Lx * rows, Lyc = (int)Ly / rows;
  const int BP = 2 * ((Lxc + 15) / 16 * 16);
  std::vector<int> Dcol = nn_pairing_cols((int)Lx, (int)Ly);
  const std::vector<int> hcol = standard_hcol((int)Lx, (int)Ly);
  const CrPlan pl = build_cr_plan(Lxc, Lyc, BP, Dcol, side && dwh::cr_supported_side(BP), (int)nbatch,
                                  256, inv0 && dwh::cr_supported_inv0(BP), &hcol);
  const double bp3 = 8.0 * BP * (double)BP * BP;
  flops[0] = flops[1] = flops[2] = 0.0;
  for (const CrStage& st : pl.stages) {
    if (st.kind == 0) {
      flops[0] += st.n * bp3;
      flops[2] += st.flops;
    } else {
      flops[1] += st.flops;
    }
  }
  return DWH_OK;
}

int dwh_debug_h_bound(int64_t Lx, int64_t Ly, double t, double tp, double mu, const int64_t* nn_table,
                      const int64_t* nnn_table, int64_t nchains, const double* disorder, double* out) {
  if (Lx < 1 || Ly < 1 || nchains < 1 || !nn_table || !nnn_table || !disorder || !out)
    return fail(nullptr, DWH_ERR_ARG, "bad lattice / NULL argument");
  const int64_t N64 = Lx * Ly;
  if (N64 > 9216) return fail(nullptr, DWH_ERR_ARG, "N = Lx*Ly > 9216 not supported");
  for (int64_t e = 0; e < 4 * N64; ++e)
    if (nn_table[e] < 1 || nn_table[e] > N64 || nnn_table[e] < 1 || nnn_table[e] > N64)
      return fail(nullptr, DWH_ERR_ARG, "neighbour table entry out of [1, N]");
  const int N = (int)N64;
  const auto hrow = build_hrow(N, t, tp, nn_table, nnn_table);
  double gersh = 0;
  for (int64_t c = 0; c < nchains; ++c)
    for (int i = 0; i < N; ++i) {
      double off = 0;
      for (const auto& e : hrow[i]) off += std::fabs(e.second);
      gersh = std::max(gersh, std::fabs(disorder[c * N64 + i] - mu) + off);
    }
  double lz = 0;
  bool ok = false;
  out[3] = h_norm_bound(hrow, disorder, mu, N, (int)Lx, (int)Ly, nchains, gersh, &lz, &ok);
  out[0] = gersh;
  out[1] = lz;
  out[2] = ok ? 1.0 : 0.0;
  out[4] = certify_spectral_bound(hrow, std::vector<double>(N, -mu).data(), N, (int)Lx, (int)Ly, 0.0) ? 1.0 : 0.0;
  return DWH_OK;
}

// ---- assembly read-back (parity tests of init_static_H! / update_H_BdG!) ----

int dwh_debug_dense_H(dwh_ctx* ctx, int64_t chain, dwh_c128* H) {
  if (!ctx || !H) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (chain < 0 || chain >= ctx->d.nc) return fail(ctx, DWH_ERR_ARG, "chain index out of range");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  const int N = ctx->d.N;
  const size_t n2 = 2 * (size_t)N;
  double2* A = nullptr;
  HIPCHECK(ctx, hipMalloc(&A, n2 * n2 * sizeof(double2)));
  // the eigen path's assembly (eigen_enqueue): zero, then k_tr_assemble
  hipError_t e = hipMemsetAsync(A, 0, n2 * n2 * sizeof(double2), ctx->stream);
  if (e == hipSuccess) {
    dwh::launch_tr_assemble(A, N, ctx->hcol, ctx->hval + (size_t)chain * N * kHSlots, ctx->Dcol, ctx->Dsrc,
                            ctx->Delta + (size_t)chain * 2 * N, ctx->stream);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(H, A, n2 * n2 * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(A);
  if (e != hipSuccess) return fail(ctx, DWH_ERR_HIP, std::string("dense H read-back: ") + hipGetErrorString(e));
  return DWH_OK;
}

int dwh_debug_level0(dwh_ctx* ctx, int64_t chain, int64_t pole, int32_t refill, dwh_c128* M, double* y) {
  if (!ctx || !M) return fail(ctx, DWH_ERR_ARG, "NULL argument");
  if (ctx->algo != ALGO_CR) return fail(ctx, DWH_ERR_STATE, "level-0 blocks exist only on the CR path");
  const dwh::CrDims& c = ctx->cr;
  if (chain < 0 || chain >= ctx->d.nc || pole < 0 || pole >= c.P)
    return fail(ctx, DWH_ERR_ARG, "chain or pole index out of range");
  HIPCHECK(ctx, hipSetDevice(ctx->device));
  if (refill) {
    // exactly cr_enqueue's assembly launch (rewritten blocks + Δ/2 scatter)
    const CrPlan& pl = ctx->plan;
    dwh::launch_cr_fill(c, ctx->bpool, ctx->d_fill_step, (int)pl.fill_step.size(), ctx->hcol, ctx->hval,
                        ctx->Dcol, ctx->Dsrc, ctx->Delta, ctx->d_y, ctx->d_off_ph, ctx->stream);
    HIPCHECK(ctx, hipGetLastError());
  }
  const int Lx = c.Lx, Ly = c.Ly, N = c.N, BP = c.BP, HP = BP / 2;
  const size_t nblk0 = 3 * (size_t)Ly, bsz = (size_t)HP * BP;
  std::vector<double2> h(nblk0 * bsz);
  const int64_t bi = chain * c.P + pole;
  HIPCHECK(ctx, hipMemcpyAsync(h.data(), ctx->bpool + bi * c.item, h.size() * sizeof(double2),
                               hipMemcpyDeviceToHost, ctx->stream));
  HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
  // expand the M-form top halves [A | B] into the reference basis (particles
  // i = y Lx + x, holes i + N): rows i: [A | B], rows i + N: [conj B | -conj A]
  const size_t n2 = 2 * (size_t)N;
  std::vector<uint8_t> seen(n2 * n2, 0);
  for (size_t k = 0; k < n2 * n2; ++k) M[k] = dwh_c128{0.0, 0.0};
  auto put = [&](size_t r, size_t col, double re, double im) -> bool {
    const size_t o = r + col * n2;   // column-major
    if (seen[o]) return false;
    seen[o] = 1;
    M[o] = dwh_c128{re, im};
    return true;
  };
  for (int t = 0; t < 3; ++t) {
    if ((t == 1 && Ly < 2) || (t == 2 && Ly < 3)) continue;   // k_cr_fill's zero blocks
    for (int yb = 0; yb < Ly; ++yb) {
      const int yr = (t == 2) ? (yb + 1) % Ly : yb, yc = (t == 1) ? (yb + 1) % Ly : yb;
      const double2* blk = h.data() + (size_t)(t * Ly + yb) * bsz;
      for (int r = 0; r < Lx; ++r)
        for (int x = 0; x < Lx; ++x) {
          const size_t i = (size_t)yr * Lx + r, j = (size_t)yc * Lx + x;
          const double2 a = blk[(size_t)r * BP + x], b = blk[(size_t)r * BP + HP + x];
          if (!put(i, j, a.x, a.y) || !put(i, j + N, b.x, b.y) || !put(i + N, j, b.x, -b.y) ||
              !put(i + N, j + N, -a.x, a.y))
            return fail(ctx, DWH_ERR_STATE, "level-0 blocks overlap");
        }
    }
  }
  if (y) std::copy(ctx->y.begin(), ctx->y.end(), y);
  return DWH_OK;
}

}  // extern "C"
