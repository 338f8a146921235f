/*
 * dwhmc.h — C ABI of the MI355X-native fermionic action/force path of
 * DwaveHMC.jl (YinkaiYu/Hybrid-Monte-Carlo-for-d-wave-SC).
 *
 * The reference is pure Julia with no FFI; each entry point below replaces a
 * Julia function of the hot path (file:line of the reference in brackets) and
 * is what a Julia `ccall`, a C++ host or Python `ctypes` binds (see
 * INTEGRATION.md).  Conventions:
 *   - every array is borrowed for the duration of the call only;
 *   - complex numbers are interleaved fp64 pairs (Julia ComplexF64,
 *     numpy complex128, C99 double _Complex);
 *   - per-chain bond arrays (Δ, π, F, P) are Julia's column-major N×2 layout:
 *     element (i, dir) at offset i + N*dir, dir 0 = +x, dir 1 = +y
 *     (src/Types.jl:106-111); chain c starts at offset c*2N;
 *   - neighbour tables are Julia's column-major N×4 Int64 matrices, 1-based
 *     (src/Types.jl:53-80);
 *   - functions return DWH_OK (0) or a negative DWH_ERR_* code; the message is
 *     in dwh_last_error(ctx) (dwh_last_error(NULL) after a failed create);
 *   - a context is bound to one HIP device and one stream and is not
 *     thread-safe (one context per host thread).
 */
#ifndef DWHMC_H
#define DWHMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double re, im; } dwh_c128;
typedef struct dwh_ctx dwh_ctx;

enum {
  DWH_OK = 0,
  DWH_ERR_ARG = -1,       /* bad argument (Julia: ArgumentError / DimensionMismatch) */
  DWH_ERR_HIP = -2,       /* HIP runtime failure (no device, OOM, launch failure) */
  DWH_ERR_STATE = -3,     /* call out of order */
  DWH_ERR_SPECTRUM = -4,  /* |Δ| left the guarded range the pole set was built for */
  DWH_ERR_TABLE = -5      /* β·E_bound outside the pole table with DWH_ALGO_DENSE / _CR requested */
};

typedef struct {
  int64_t N;          /* sites Lx*Ly */
  int64_t Np;         /* N padded to the 64-row GJ block */
  int64_t nchains;
  int64_t npoles;     /* imaginary-axis pole pairs = no-pivot LUs per chain per step (eig: 0) */
  double kappa;       /* β·E'/2 of the pole table entry in use (eig: of the spectral bound) */
  double e_bound;     /* E' : spectral bound the poles are valid on */
  double err_tanh;    /* sup |tanh - rational| of the table entry (eig: 0) */
  double delta_cap;   /* guard cap: on max|Δ_ij| (bond guard), or on the mean |Δ| of each site's
                         4 bonds (site guard: the CR path, whose level-0
                         inversion launch checks it); eig: DBL_MAX, no guard */
  int64_t device_bytes;
  int64_t algo;       /* 0 = dense Schur-complement Gauss-Jordan, 1 = block cyclic reduction,
                         2 = eigendecomposition */
  int64_t block;      /* dense: GJ block (64); cr: padded lattice-row block BP >= 2 Lx; eig: 0 */
  int64_t eig_half;   /* last eigensolve (transport / eig path): 1 = particle-hole half solve,
                         J_mn and the pair sums over the columns < N; 0 = every column; -1 = none yet */
  int64_t eig_long_clusters; /* eigenvalue clusters so far too long for the one-workgroup
                                orthonormalisation, taken by the multi-workgroup Cholesky QR */
  int64_t eig_quat;   /* last eigensolve with vectors: 1 = the structure-preserving (quaternion)
                         solver, 0 = the one-stage tridiagonalisation (spectra with a cluster
                         longer than 32 levels or a crowd at zero longer than 16, or
                         DWHMC_EIG_QUAT=0) */
} dwh_info_t;

/* ModelParameters + initialize_cache + init_static_H!
 * [src/Types.jl:49-91, src/Types.jl:182-212, src/Hamiltonian.jl:10-47].
 * One chain, default delta_cap (bond guard max(2, 6 sqrt(2J/β)); site guard
 * max(1.25, 4 sqrt(2J/β))).  disorder: length N
 * (state.disorder_pot). */
int dwh_create(dwh_ctx** ctx, int64_t Lx, int64_t Ly, double t, double tp, double mu,
               double beta, double J, const int64_t* nn_table, const int64_t* nnn_table,
               const double* disorder, int32_t device);

/* Batched form: nchains independent Markov chains / disorder realisations on one
 * device (disorder: nchains*N).  delta_cap <= 0 selects the default
 * (bond guard max(2, 6 sqrt(2J/β)), site guard max(1.25, 4 sqrt(2J/β)));
 * either guard bounds the pairing block's norm by 2 delta_cap; the pole set
 * covers spectra within ‖h‖ + 2 delta_cap and is
 * re-selected for a larger cap when an uploaded Δ or a trajectory exceeds it. */
int dwh_create_batched(dwh_ctx** ctx, int64_t Lx, int64_t Ly, double t, double tp, double mu,
                       double beta, double J, const int64_t* nn_table, const int64_t* nnn_table,
                       int64_t nchains, const double* disorder, double delta_cap, int32_t device);

/* Factorisation algorithm of a context:
 *   DWH_ALGO_DENSE  Schur complement over the static particle block + blocked
 *                   Gauss-Jordan of the dense N x N complement per pole;
 *   DWH_ALGO_CR     block cyclic reduction of the block-tridiagonal (lattice-row
 *                   blocks, periodic) BdG matrix per pole; needs 2 Lx <= 128;
 *   DWH_ALGO_EIG    the reference's own method: the eigendecomposition of every chain's
 *                   2N x 2N H_BdG per step (dwh_eigensystem's solver), ρ = U diag(f) U^H by zgemm
 *                   [src/Hamiltonian.jl:96-114, src/Observables.jl:14-62]; any β,
 *                   no pole set, no |Δ| guard; O(N^3) with a large constant;
 *   DWH_ALGO_AUTO   DWHMC_ALGO from the environment (dense | cr | eig | auto),
 *                   else CR when supported, else dense; EIG when β·E'/2 is beyond
 *                   the pole table (β above a few hundred).  All give the same
 *                   results to fp64 rounding. */
enum { DWH_ALGO_AUTO = -1, DWH_ALGO_DENSE = 0, DWH_ALGO_CR = 1, DWH_ALGO_EIG = 2 };

/* dwh_create_batched with an explicit algorithm. */
int dwh_create_ex(dwh_ctx** ctx, int64_t Lx, int64_t Ly, double t, double tp, double mu,
                  double beta, double J, const int64_t* nn_table, const int64_t* nnn_table,
                  int64_t nchains, const double* disorder, double delta_cap, int32_t algo,
                  int32_t device);

void dwh_destroy(dwh_ctx* ctx);
const char* dwh_last_error(const dwh_ctx* ctx);
int dwh_info(dwh_ctx* ctx, dwh_info_t* out);

/* update_H_BdG! [src/Hamiltonian.jl:55-86]: set Δ (nchains*2N) on the device. */
int dwh_update_pairing(dwh_ctx* ctx, const dwh_c128* Delta);

/* diagonalize_H_BdG! replacement [src/Hamiltonian.jl:96-114]: pole-expanded
 * no-pivot LU of H_BdG(Δ) - i y_q for all poles; caches the pairing
 * amplitudes P_ij and the fermion energy E_f for the current Δ. */
int dwh_factorize(dwh_ctx* ctx);

/* compute_forces! [src/Observables.jl:14-62]: F = -β/2J (Δ - J P) with the
 * cached P.  Delta may be NULL (use the device Δ).  F_out: nchains*2N. */
int dwh_forces(dwh_ctx* ctx, const dwh_c128* Delta, dwh_c128* F_out);

/* P_ij = -ρ_{i,j+N} - ρ_{j,i+N} of the last factorisation [src/Observables.jl:37-53]. */
int dwh_pairing(dwh_ctx* ctx, dwh_c128* P_out);

/* Fermion part of compute_total_energy [src/HMC.jl:21-27], per chain. */
int dwh_fermion_energy(dwh_ctx* ctx, double* Ef);

/* Tr ρ_hh per chain (hole-block trace of the density matrix); with
 * Tr ρ_pp + Tr ρ_hh = N this gives hole_conc = 2 Tr ρ_hh / N - 1
 * [src/Observables.jl:120-145]. */
int dwh_hole_trace(dwh_ctx* ctx, double* tr_hh);

/* compute_total_energy [src/HMC.jl:12-41] for the device Δ, π and cached E_f. */
int dwh_total_energy(dwh_ctx* ctx, double mass, double* H);

/* Device state access (Δ, π: nchains*2N; either pointer may be NULL). */
int dwh_set_state(dwh_ctx* ctx, const dwh_c128* Delta, const dwh_c128* pi);
int dwh_get_state(dwh_ctx* ctx, dwh_c128* Delta, dwh_c128* pi);

/* hmc_sweep! [src/HMC.jl:71-144] with the RNG draws injected (the reference
 * is unseeded): noise = randn!(ComplexF64) draws (Var Re = Var Im = 1/2),
 * nchains*2N; uniform = the rand() of the Metropolis test, nchains.
 * Outputs accepted[nchains] (0/1) and dH[nchains]. */
int dwh_hmc_sweep(dwh_ctx* ctx, const dwh_c128* noise, const double* uniform, int64_t Nt,
                  double dt, double mass, uint8_t* accepted, double* dH);

/* hmc_sweep! split at its Metropolis test, so a host whose RNG must be
 * consumed exactly as the reference consumes it (src/HMC.jl:128 draws
 * rand() only when ΔH >= 0) decides acceptance itself:
 *   dwh_hmc_trajectory: momentum refresh from `noise`, H_old, backup,
 *     leapfrog, H_new [src/HMC.jl:76-122]; dH[nchains] = H_new - H_old.
 *   dwh_hmc_finish: accepted[nchains] (0/1) from the host; rejected chains are
 *     restored [src/HMC.jl:130-141].
 * Between the two calls the context refuses another sweep (DWH_ERR_STATE). */
int dwh_hmc_trajectory(dwh_ctx* ctx, const dwh_c128* noise, int64_t Nt, double dt, double mass,
                       double* dH);
int dwh_hmc_finish(dwh_ctx* ctx, const uint8_t* accepted);

/* Throughput path: upload the draws of nsweeps sweeps once (noise:
 * nsweeps*nchains*2N, uniform: nsweeps*nchains), then enqueue sweeps that
 * read them from HBM without host round trips.  A guard trip inside a batch
 * makes the batch's later sweeps no-ops on the device; the next
 * dwh_sweep_results / dwh_synchronize (or any call that reads or changes the
 * state) re-selects the pole set, resumes from the tripped sweep's starting Δ
 * and replays the remaining sweeps — the same steps dwh_hmc_sweep takes — so
 * the results equal the single-sweep path's bit for bit. */
int dwh_load_draws(dwh_ctx* ctx, int64_t nsweeps, const dwh_c128* noise, const double* uniform);
int dwh_run_sweeps(dwh_ctx* ctx, int64_t first_sweep, int64_t nsweeps, int64_t Nt, double dt,
                   double mass);
int dwh_sweep_results(dwh_ctx* ctx, int64_t first_sweep, int64_t nsweeps, uint8_t* accepted,
                      double* dH);
int dwh_synchronize(dwh_ctx* ctx);

/* hipStream_t the context launches on (for events / interop).  The handle
 * stays valid for the context's lifetime, pole re-selections included. */
int dwh_stream(dwh_ctx* ctx, void** stream);

/* Kernel timing with HIP events on the stream each kernel runs on
 * (bench/profiling).  enable is a bitmask over the timer names below
 * (bit 0 "gj_update", bit 1 "gj_pivot", bit 2 "assemble", bit 3 "contract",
 * bit 4 "step", bit 5 "gj_edge", bit 6 "cr_gemm", bit 7 "cr_inv", bit 8 "cr_inv_side",
 * bit 9 "eig_own", bit 10 "eig_vendor", bit 11 "cr_sparse");
 * 0 disables, -1 times everything. */
int dwh_timing_enable(dwh_ctx* ctx, int32_t enable);
/* name: "gj_update" (rank-128 paired / rank-64 trailing updates),
 * "gj_edge" (edge update between the two pivots of a pair), "gj_pivot",
 * "cr_gemm" (cyclic-reduction block products), "cr_inv" (its block
 * inversions), "cr_inv_side" (inversion stages that also run the products off
 * the critical path; work = inversion + side-product flops), "cr_sparse" (the
 * sparse level-0 stages: products with the level-0 U / L blocks, work = their
 * sparse flops), "eig_own" / "eig_vendor" (eigensolves by the library's solver /
 * by rocSOLVER, opt-in or fallback; work = matrices), "assemble",
 * "contract", "step"; returns total milliseconds, launches and the
 * algorithmic work summed over launches (fp64 flops; HBM bytes for
 * "assemble"). */
int dwh_timing_read(dwh_ctx* ctx, const char* name, double* total_ms, int64_t* launches,
                    double* work);
int dwh_timing_reset(dwh_ctx* ctx);
/* Enqueues the per-factorisation assembly launch (timer "assemble": CR, the
 * pairing entries Δ/2 scattered into the level-0 blocks, replacing
 * update_H_BdG! src/Hamiltonian.jl:55-86; dense, the Schur-complement
 * assembly) reps times back to back on the context's stream and waits, so a
 * bench reads a warm per-launch average with the timers instead of the one
 * launch a factorisation makes.  Idempotent: the pool keeps the current Δ.
 * eig path: DWH_ERR_STATE. */
int dwh_bench_assembly(dwh_ctx* ctx, int64_t reps);
/* Diagnostic: one CR factorisation at the context's Δ with per-workgroup phase
 * stamps of its inv_stage-th inversion launch (in the plan's own schedule,
 * side work included) into out (nwg rows of 32 uint64: [0]/[30]
 * s_memrealtime at entry/exit, [1..29] s_memtime phase stamps, [31] kind 1
 * inversion / 2 side work / 3 guard).  Only a library built with -DCR_STAMPS
 * records them (tools/cr_inv_sched_stamps.py); others return DWH_ERR_STATE. */
int dwh_debug_cr_stamps(dwh_ctx* ctx, int32_t inv_stage, uint64_t* out, int64_t nwg);

/* ---- measurement path (not the leapfrog step) ----------------------------
 * Eigen-decomposition of one chain's H_BdG(Δ) at the device Δ: what the
 * reference's diagonalize_H_BdG! [src/Hamiltonian.jl:96-114] leaves in
 * cache.E_n / cache.U, which the hot path replaces by the pole expansion but
 * transport and spectra need.  The library's own Hermitian eigensolver on
 * the context's stream (dwhmc_eig.hip: Householder tridiagonalisation,
 * multisection on Sturm counts, inverse iteration with cluster
 * orthonormalisation (clusters of any length), blocked back-transform; the
 * plain products on the library's own MFMA kernel, dwhmc_gemm.hip);
 * rocSOLVER runs only for an order above the own solver's 5120 (zheevd) and
 * as the re-solve (zheev) of a result with non-finite values.
 * E: 2N, ascending; U (nullable): 2N x 2N column-major, the eigenvector of
 * E[n] in column n (phases are the solver's). */
int dwh_eigensystem(dwh_ctx* ctx, int64_t chain, double* E, dwh_c128* U);

/* Lengths of the frequency grids of measure_transport_and_spectra
 * [src/Observables.jl:395,430]: ω = η:Δω:ω_max and -ω_max:Δω:ω_max, counted
 * as Julia's float ranges count them; point k of either grid is start + k·Δω. */
int dwh_transport_grid(double eta, double domega, double omega_max, int64_t* n_omega,
                       int64_t* n_dos);

/* measure_transport_and_spectra [src/Observables.jl:314-526] for one chain at
 * the device Δ, i.e. the SpectrumResult fields [:293-308]: superfluid
 * stiffness, DC conductivity, σ(ω) on the ω grid (n_omega values), DOS and
 * antinodal DOS on the DOS grid (n_dos values each) and A(k, ω=0) as the
 * column-major Lx x Ly map (element (kx, ky) at kx + Lx·ky, FFTW's forward
 * sign).  n_omega / n_dos must equal dwh_transport_grid's.  The current
 * operator J_x [:237-283] is built once per context; J_mn = U^H (J ⊕ J) U is
 * the library's own MFMA product (dwhmc_gemm.hip); the rest runs in
 * dwhmc_transport.hip. */
int dwh_measure_transport(dwh_ctx* ctx, int64_t chain, double eta, double domega, double omega_max,
                          double* stiffness, double* dc_cond, double* sigma, int64_t n_omega,
                          double* dos, double* dos_an, int64_t n_dos, double* ak0);

/* dwh_measure_transport for every chain of the context at once: the
 * eigensolves and J_mn products are batched over the chains (every kernel
 * of the eigensolver and the products take all chains per launch).
 * Outputs per chain c at stiffness[c], dc_cond[c], sigma[c*n_omega],
 * dos[c*n_dos], dos_an[c*n_dos], ak0[c*Lx*Ly]. */
int dwh_measure_transport_batched(dwh_ctx* ctx, double eta, double domega, double omega_max,
                                  double* stiffness, double* dc_cond, double* sigma, int64_t n_omega,
                                  double* dos, double* dos_an, int64_t n_dos, double* ak0);

/* measure_transport_and_spectra at nstates pairing fields of one chain's
 * lattice and disorder: Delta[k] (nstates x 2N, the Δ layout above), e.g. the
 * states of nstates consecutive measurement sweeps [src/Simulation.jl:169-171]
 * kept by the host and measured in one call.  The eigensolves and J_mn
 * products are batched over the snapshots as in
 * dwh_measure_transport_batched; outputs per snapshot k at stiffness[k],
 * dc_cond[k], sigma[k*n_omega], dos[k*n_dos], dos_an[k*n_dos], ak0[k*Lx*Ly].
 * The context's own Δ is not touched. */
int dwh_measure_transport_deltas(dwh_ctx* ctx, int64_t chain, int64_t nstates, const dwh_c128* Delta,
                                 double eta, double domega, double omega_max, double* stiffness,
                                 double* dc_cond, double* sigma, int64_t n_omega, double* dos, double* dos_an,
                                 int64_t n_dos, double* ak0);

/* ---- assembly read-back (parity tests; not on the hot path) -------------
 * The BdG matrix H_BdG(Δ) exactly as the device assembles it, so tests can
 * compare it bit-for-bit with init_static_H! + update_H_BdG!
 * [src/Hamiltonian.jl:10-47, 55-86] (Hermitian completion of the reference's
 * upper triangle, including its overwrite order on 1- and 2-site rings).
 *
 * dwh_debug_dense_H: the dense matrix the eigen/transport path builds
 * (k_tr_assemble) from the device Δ of `chain`; H: 2N x 2N column-major.
 *
 * dwh_debug_level0 (CR path only): the level-0 blocks of batch item
 * (chain, pole) — H_BdG(Δ) - i y_pole I as the factorisation consumes it —
 * expanded from the stored M-form top halves into the reference basis
 * (particles i = y Lx + x, holes i + N); M: 2N x 2N column-major, y (nullable):
 * the npoles pole heights y_q.  refill != 0 first runs the factorisation's
 * assembly launch on the device Δ; refill == 0 reads the pool as the last
 * trajectory step left it (Δ/2 scattered by the force kernel). */
int dwh_debug_dense_H(dwh_ctx* ctx, int64_t chain, dwh_c128* H);

/* Development entry of the structure-preserving (quaternion) eigensolver
 * (dwhmc_qeig.hip, tools/qeig_proto.py): the 2N eigenvalues of H_BdG(Δ of
 * `chain`) ascending into E, the site-by-site reduction's device time into
 * *ms (nullable). */
int dwh_debug_qeig(dwh_ctx* ctx, int64_t chain, double* E, double* ms);
int dwh_debug_level0(dwh_ctx* ctx, int64_t chain, int64_t pole, int32_t refill, dwh_c128* M, double* y);

/* Host-only check of the cyclic-reduction schedule dwh_create builds for an
 * Lx x Ly periodic lattice with nearest-neighbour pairing and nbatch = chains x
 * poles batch items (side / inv0: enable the side-work placement and the
 * static level-0 particle blocks, as dwh_create does where the block size
 * supports them): every block a stage reads was written by an earlier stage
 * (or is a level-0 / static block), no stage reads what it writes except a
 * task's own accumulate input, no block is written by two tasks of one stage,
 * and the force / E_f gathers read written blocks.  No device is touched.
 * stats (nullable, 6): stages, inversion stages, inversion stages with side
 * work, product stages, writes, pool blocks.  DWH_ERR_STATE with the first
 * violation in dwh_last_error(NULL). */
int dwh_debug_cr_plan_check(int64_t Lx, int64_t Ly, int64_t nbatch, int32_t side, int32_t inv0, int64_t* stats);

/* Algorithmic fp64 flops per batch item of the same plan (host only), as the
 * "cr_*" timers count them: flops[0] block inversions (8 BP^3 each), flops[1]
 * block products of the product stages, flops[2] block products run as side
 * work inside inversion stages (8 BP rows cols per term on the restricted
 * output windows).  flops[1] + flops[2] does not depend on `side`. */
int dwh_debug_cr_plan_flops(int64_t Lx, int64_t Ly, int64_t nbatch, int32_t side, int32_t inv0, double* flops);

/* The ‖h‖ bound pole selection uses (host only; h = the static particle block
 * of src/Hamiltonian.jl:10-44 with w_i - mu on the diagonal, per chain):
 * out[0] Gershgorin, out[1] the Lanczos estimate, out[2] 1 if every chain
 * certified it (rho I -/+ h positive definite by band LDLᵀ), out[3] the bound
 * used (the Lanczos value if certified, else Gershgorin), out[4] a negative
 * control (1 if rho = 0 "certified": must be 0). */
int dwh_debug_h_bound(int64_t Lx, int64_t Ly, double t, double tp, double mu, const int64_t* nn_table,
                      const int64_t* nnn_table, int64_t nchains, const double* disorder, double* out);

/* Self-test of the f64 MFMA fragment layout (A = I, asymmetric B); 0 = pass. */
int dwh_selftest_mfma(int32_t device);

/* The library's own batched fp64 MFMA product (the measurement path's
 * J_mn = U^H J U, the eigensolver's back-transform and orthogonalisation, the
 * eig path's rho), through host buffers for tests:
 * C_k = alpha op(A_k) op(B_k) + beta C_k, k < batch, column-major, op 'N' or
 * 'C' (conjugate transpose; transpose when real); cplx 1: dwh_c128 data and
 * alpha / beta as {re, im}, 0: double (alpha[0], beta[0]).  Batch strides:
 * lda * (columns of A), ldb * (columns of B), ldc * N elements. */
int dwh_debug_gemm(int32_t device, int32_t cplx, char opa, char opb, int64_t M, int64_t N, int64_t K,
                   const double* alpha, const void* A, int64_t lda, const void* B, int64_t ldb, const double* beta,
                   void* C, int64_t ldc, int64_t batch);

#ifdef __cplusplus
}
#endif
#endif /* DWHMC_H */
