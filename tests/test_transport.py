"""Transport and spectra (src/Observables.jl:225-526), SURVEY.md §8(f) row 4.

CPU (not gpu): the oracle restatement pinned three ways —
  * vectorised form vs the reference's literal (n, m) loops;
  * the reference's own consistency check scripts/debug_transport.jl:50-95:
    the diamagnetic term in its tanh form (the one measure_transport_and_spectra
    uses) equals its Fermi-factor form (particle-hole symmetry of H_BdG);
  * Julia's float-range lengths for the ω grids.
The reference ships no transport fixtures, so these plus the
loop form are the pins; the absolute values are otherwise "parity unpinned"
against a Julia run.

GPU: the device path (the hand-written eigensolver csrc/dwhmc_eig.hip, with
rocSOLVER zheev only where it flags a result, + the library's own MFMA
products csrc/dwhmc_gemm.hip + dwhmc_transport.hip)
through the C ABI vs the oracle on the same Δ.  Tolerances (fp64):
  * eigenvalues          |E_gpu - E_ref| ≤ 1e-12 (1 + max|E|)
  * stiffness, dc        |Δ| ≤ 1e-9 (1 + |ref|)
  * σ(ω), DOS, DOS_AN    max|Δ| ≤ 1e-9 (1 + max|ref|)
  * A(k, 0)              max|Δ| ≤ 1e-9 (1 + max|ref|)
Every quantity is a sum over eigenstates of functions of E_n only, weighted by
basis-invariant sums inside degenerate subspaces, so eigenvector phases and
the solver's basis choice inside degenerate levels do not enter.
"""
import numpy as np
import pytest

T, TP, MU = 1.0, -0.35, -1.08


def _case(O, Lx, Ly, beta, seed, W=1.0, nimp=0.1, amp=0.25, mu=MU):
    p = O.ModelParameters(Lx, Ly, T, TP, mu, W, nimp, beta, 0.8, 1.0)
    rng = np.random.default_rng(seed)
    st = O.initialize_state(p, rng)
    N = p.N
    D = st.Delta + amp * np.stack([np.ones(N), -np.ones(N)], 1) * np.exp(0.3j * rng.standard_normal((N, 1)))
    return p, st.disorder_pot, D


def _kinetic_weights(p, U):
    """Per-state x-bond weights of src/Observables.jl:350-359 split into the
    particle (u) and hole (v) parts."""
    N = p.N
    u, v = U[:N], U[N:]
    i = np.arange(N)
    wu = np.zeros(U.shape[1])
    wv = np.zeros(U.shape[1])
    for j, tt in ((p.nn_table[:, 0] - 1, p.t), (p.nnn_table[:, 0] - 1, p.tp), (p.nnn_table[:, 3] - 1, p.tp)):
        wu += tt * 2.0 * np.real(np.conj(u[i]) * u[j]).sum(axis=0)
        wv += tt * 2.0 * np.real(v[i] * np.conj(v[j])).sum(axis=0)
    return wu, wv


# --------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("Lx,Ly", [(4, 4), (3, 5), (2, 4)])
def test_oracle_vectorised_matches_loops(oracle, Lx, Ly):
    O = oracle
    p, dis, D = _case(O, Lx, Ly, 8.0, seed=Lx * 10 + Ly)
    cache, _, _ = O.evaluate(p, dis, D)
    r = O.measure_transport_and_spectra(cache, p)
    q = O.measure_transport_loops(cache, p)
    for k in ("superfluid_stiffness", "dc_conductivity"):
        assert abs(r[k] - q[k]) <= 1e-12 * (1 + abs(q[k])), k
    s, sq = r["optical_conductivity"], q["optical_conductivity"]
    assert np.max(np.abs(s - sq)) <= 1e-12 * (1 + np.max(np.abs(sq)))


def test_diamagnetic_forms_agree(oracle):
    """scripts/debug_transport.jl:9-95 (10x10 clean, β = 1000, μ = -1, uniform
    d-wave Δx = 0.2, Δy = -0.2): Σ_{E>0} w_n tanh(βE_n/2) (the form
    measure_transport_and_spectra uses) equals the Fermi-factor form
    Σ_n [w^u_n f_n + w^v_n (1 - f_n)]; the ordered state has ρ_s > 0."""
    O = oracle
    p = O.ModelParameters(10, 10, 1.0, -0.35, -1.0, 0.0, 0.0, 1000.0, 1.6, 0.1)
    N = p.N
    D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(np.complex128)
    cache, _, _ = O.evaluate(p, np.zeros(N), D)
    E, f = cache.E_n, cache.fermi_factors
    wu, wv = _kinetic_weights(p, cache.U)
    w = wv - wu
    dia1 = float(np.sum(np.where(E > 0, w * np.tanh(0.5 * p.beta * np.maximum(E, 0.0)), 0.0))) / N
    dia2 = float(np.sum(wu * f + wv * (1.0 - f))) / N
    assert abs(dia1 - dia2) <= 1e-10 * (1 + abs(dia1)), (dia1, dia2)
    r = O.measure_transport_and_spectra(cache, p)
    assert r["superfluid_stiffness"] > 0, r["superfluid_stiffness"]


def test_julia_range_lengths(oracle):
    O = oracle
    assert len(O.julia_range(0.01, 0.002, 4.0)) == 1996       # ω_min:Δω:ω_max (defaults)
    assert len(O.julia_range(-4.0, 0.002, 4.0)) == 4001       # DOS grid
    assert len(O.julia_range(0.0, 0.25, 1.0)) == 5
    assert len(O.julia_range(0.0, 0.3, 1.0)) == 4             # 0, .3, .6, .9
    assert len(O.julia_range(1.0, 0.5, 0.0)) == 0


def test_current_operator(oracle):
    """Hermitian, purely imaginary; duplicates summed (sparse()): on Lx = 2 the
    +x and -x neighbours coincide and the current cancels."""
    O = oracle
    p = O.ModelParameters(4, 3, T, TP, MU, 0.0, 0.0, 4.0, 1.0, 1.0)
    Jx = O.current_operator(p)
    assert np.allclose(Jx, Jx.conj().T) and np.allclose(Jx.real, 0)
    assert np.count_nonzero(Jx) == 6 * p.N
    p2 = O.ModelParameters(2, 3, T, TP, MU, 0.0, 0.0, 4.0, 1.0, 1.0)
    assert np.allclose(O.current_operator(p2), 0)


# --------------------------------------------------------------------------- GPU
def _ctx(dwhmc, p, dis, **kw):
    return dwhmc.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                                dis, **kw)


def test_transport_grid_matches_julia(dwhmc, oracle):
    """dwh_transport_grid is host arithmetic: no device needed."""
    for args in ((0.01, 0.002, 4.0), (0.05, 0.01, 2.0), (0.02, 0.3, 1.0)):
        nw, nd = dwhmc.transport_grid(*args)
        assert nw == len(oracle.julia_range(args[0], args[1], args[2]))
        assert nd == len(oracle.julia_range(-args[2], args[1], args[2]))


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly", [(4, 4), (6, 6), (5, 7), (2, 4)])
def test_eigensystem_matches_oracle(dwhmc, oracle, Lx, Ly):
    O = oracle
    p, dis, D = _case(O, Lx, Ly, 8.0, seed=Lx * 7 + Ly)
    cache, _, _ = O.evaluate(p, dis, D)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    E, U = ctx.eigensystem(0)
    ctx.close()
    Href = O.hermitian_from_upper(cache.H_base)
    scale = 1 + np.max(np.abs(cache.E_n))
    assert np.max(np.abs(E - cache.E_n)) <= 1e-12 * scale
    assert np.max(np.abs(Href @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N))) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,beta,clean,half", [(8, 8, 16.0, False, "1"), (16, 16, 8.0, False, "1"),
                                                   (32, 32, 16.0, False, "1"), (32, 32, 16.0, False, "0"),
                                                   (16, 16, 8.0, True, "1"), (12, 10, 4.0, True, "1"),
                                                   (16, 16, 8.0, "zero", "1"), (8, 12, 8.0, "zero", "1"),
                                                   (16, 16, 8.0, "zero", "0")])
def test_own_eigensolver_full_size(dwhmc, oracle, monkeypatch, Lx, Ly, beta, clean, half):
    """The hand-written eigensolver (csrc/dwhmc_eig.hip: Householder
    tridiagonalisation, bisection, inverse iteration + cluster Cholesky QR,
    blocked back-transform) at BASELINE sizes (n = 2N up to 2048) against
    LAPACK zheevr (the oracle, as eigen!(Hermitian(H)) in
    src/Hamiltonian.jl:96-114): eigenvalues within 1e-12 (1 + max|E|),
    ‖H U − U E‖ within 1e-11 (1 + max|E|), ‖UᴴU − I‖ ≤ 1e-12.  Clean lattices
    (W = 0, uniform d-wave Δ) have exactly degenerate levels: their vectors
    come out of the cluster orthonormalisation; at μ = 0 ("zero") with L % 4
    == 0 the d-wave nodes sit on the grid and give exact zero modes, a cluster
    across E = 0 that the particle-hole half solve (default; half = "0": every
    column, DWHMC_EIG_HALF=0) computes whole."""
    O = oracle
    monkeypatch.setenv("DWHMC_EIG_HALF", half)
    if clean:
        mu = 0.0 if clean == "zero" else -1.0
        p = O.ModelParameters(Lx, Ly, T, TP, mu, 0.0, 0.0, beta, 0.8, 1.0)
        dis = np.zeros(p.N)
        D = np.stack([np.full(p.N, 0.2), np.full(p.N, -0.2)], 1).astype(np.complex128)
    else:
        p, dis, D = _case(O, Lx, Ly, beta, seed=Lx * 31 + Ly)
    cache, _, _ = O.evaluate(p, dis, D)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    ctx.timing_enable(["eig_own", "eig_vendor"])
    E, U = ctx.eigensystem(0)
    own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
    ctx.close()
    assert (own, vendor) == (1, 0), "the own solver ran without the rocSOLVER fallback"
    H = O.hermitian_from_upper(cache.H_base)
    scale = 1 + np.max(np.abs(cache.E_n))
    assert np.all(np.isfinite(U))
    assert np.max(np.abs(E - cache.E_n)) <= 1e-12 * scale
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N))) <= 1e-12


@pytest.mark.gpu
def test_own_eigensolver_L48(dwhmc, oracle):
    """C5's lattice (48 x 48, n = 4608: the k_eig_step row slots beyond 2048,
    the 73.7 KiB of dynamic LDS of k_eig_bisect / k_eig_invit, the cluster
    density of 4608 levels) through the own solver with no rocSOLVER fallback,
    at the tolerances of test_own_eigensolver_full_size (kEigMaxN
    covers it).  Eigenvalues against LAPACK (zheevr, values only); the
    residual ‖H U − U E‖ and ‖UᴴU − I‖ by numpy products (seconds; LAPACK's
    eigenvectors at n = 4608 would take minutes)."""
    import scipy.linalg as sla
    O = oracle
    p, dis, D = _case(O, 48, 48, 32.0, seed=4848)
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, D)
    Eref = sla.eigh(cache.H_base, lower=False, eigvals_only=True, driver="evr", check_finite=False)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    ctx.timing_enable(["eig_own", "eig_vendor"])
    E, U = ctx.eigensystem(0)
    own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
    ctx.close()
    assert (own, vendor) == (1, 0)
    assert np.all(np.isfinite(U))
    scale = 1 + np.max(np.abs(Eref))
    assert np.max(np.abs(E - Eref)) <= 1e-12 * scale
    H = O.hermitian_from_upper(cache.H_base)
    res = np.max(np.abs(H @ U - U * E[None, :]))
    orth = np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N)))
    assert res <= 1e-11 * scale, res
    assert orth <= 1e-12, orth


@pytest.mark.gpu
def test_eigensystem_above_own_limit_vendor_route(dwhmc, oracle):
    """The one size where rocSOLVER is the only route:
    n = 2N = 5200 > kEigMaxN = 5120 (52 x 50) runs zheevd, counted by the
    eig_vendor timer, and dwh_info_t::eig_half reports 0 for it.
    Size-independent checks, no LAPACK solve of n = 5200 on the host: the
    eigenvalues ascend, Σ E = tr H = 0 and Σ E² = ‖H‖_F² (1e-10 relative),
    and for 96 eigenpairs spread over the spectrum ‖H u − E u‖ ≤ 1e-10
    (1 + max|E|) and their Gram matrix is I within 1e-12."""
    O, m = oracle, dwhmc
    p, dis, D = _case(O, 52, 50, 16.0, seed=5250)
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, D)
    H = O.hermitian_from_upper(cache.H_base)
    del cache
    ctx = _ctx(m, p, dis)
    ctx.set_pairing(D)
    ctx.timing_enable(["eig_own", "eig_vendor"])
    E, U = ctx.eigensystem(0)
    own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
    half = ctx.info["eig_half"]
    ctx.close()
    assert (own, vendor) == (0, 1) and half == 0
    assert np.all(np.isfinite(E)) and np.all(np.isfinite(U))
    assert np.all(np.diff(E) >= 0)
    fro2 = float(np.sum(np.abs(H) ** 2))
    assert abs(E.sum()) <= 1e-10 * np.sqrt(fro2) * len(E)
    assert abs(np.sum(E ** 2) - fro2) <= 1e-10 * fro2
    S = np.linspace(0, len(E) - 1, 96).astype(int)
    res = np.max(np.abs(H @ U[:, S] - U[:, S] * E[S][None, :]))
    assert res <= 1e-10 * (1 + np.max(np.abs(E))), res
    assert np.max(np.abs(U[:, S].conj().T @ U[:, S] - np.eye(len(S)))) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,maxc", [(12, 10, "1"), (24, 24, "4")])
def test_eigensolver_long_clusters(dwhmc, oracle, monkeypatch, Lx, Ly, maxc):
    """Clusters longer than k_eig_orth's one-workgroup limit are
    orthonormalised in the library (Cholesky QR twice on its own products,
    R from the host) instead of the round-4 rocSOLVER zheev fallback:
    DWHMC_EIG_MAX_CLUSTER lowers the limit so the degenerate shells of a clean
    lattice take that path (eig_long_clusters > 0, eig_vendor == 0), and the
    eigenpairs meet test_own_eigensolver_full_size's tolerances."""
    O = oracle
    monkeypatch.setenv("DWHMC_EIG_MAX_CLUSTER", maxc)
    monkeypatch.setenv("DWHMC_EIG_QUAT", "0")   # the one-stage solver's cluster paths
    p = O.ModelParameters(Lx, Ly, T, TP, -1.0, 0.0, 0.0, 4.0, 0.8, 1.0)
    dis = np.zeros(p.N)
    D = np.stack([np.full(p.N, 0.2), np.full(p.N, -0.2)], 1).astype(np.complex128)
    cache, _, _ = O.evaluate(p, dis, D)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    ctx.timing_enable(["eig_own", "eig_vendor"])
    E, U = ctx.eigensystem(0)
    own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
    nlong = ctx.info["eig_long_clusters"]
    ctx.close()
    assert (own, vendor) == (1, 0) and nlong > 0, (own, vendor, nlong)
    H = O.hermitian_from_upper(cache.H_base)
    scale = 1 + np.max(np.abs(cache.E_n))
    assert np.max(np.abs(E - cache.E_n)) <= 1e-12 * scale
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N))) <= 1e-12


@pytest.mark.gpu
def test_own_eigensolver_L48_low_cluster_limit(dwhmc, oracle, monkeypatch):
    """C5's lattice with the one-workgroup cluster limit at 2: every cluster of
    3+ levels takes the multi-workgroup path; no rocSOLVER solve (which took
    more than 400 s here in round 4), within 60 s, at the tolerances of
    test_own_eigensolver_L48."""
    import time
    import scipy.linalg as sla
    O = oracle
    monkeypatch.setenv("DWHMC_EIG_MAX_CLUSTER", "2")
    monkeypatch.setenv("DWHMC_EIG_QUAT", "0")
    p, dis, D = _case(O, 48, 48, 32.0, seed=4848)
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, D)
    Eref = sla.eigh(cache.H_base, lower=False, eigvals_only=True, driver="evr", check_finite=False)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    ctx.timing_enable(["eig_own", "eig_vendor"])
    t0 = time.perf_counter()
    E, U = ctx.eigensystem(0)
    el = time.perf_counter() - t0
    own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
    ctx.close()
    assert (own, vendor) == (1, 0) and el < 60.0, (own, vendor, el)
    scale = 1 + np.max(np.abs(Eref))
    assert np.max(np.abs(E - Eref)) <= 1e-12 * scale
    H = O.hermitian_from_upper(cache.H_base)
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N))) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,beta", [(12, 10, 4.0), (16, 16, 8.0), (32, 32, 16.0)])
def test_structure_preserving_solver_clusters(dwhmc, oracle, Lx, Ly, beta):
    """Clean lattices (W = 0, uniform d-wave Δ, μ = -1: degenerate shells of up
    to 8+ levels, no zero modes) through the structure-preserving eigensolver:
    its inverse-iteration vectors of each cluster are orthonormalised by
    Cholesky QR (k_q_orth) instead of the solver declining to the one-stage
    path.  eig_quat == 1, no rocSOLVER fallback, and the tolerances of
    test_own_eigensolver_full_size; the measurement against the oracle."""
    O = oracle
    p = O.ModelParameters(Lx, Ly, T, TP, -1.0, 0.0, 0.0, beta, 0.8, 1.0)
    dis = np.zeros(p.N)
    D = np.stack([np.full(p.N, 0.2), np.full(p.N, -0.2)], 1).astype(np.complex128)
    cache, _, _ = O.evaluate(p, dis, D)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    ctx.timing_enable(["eig_own", "eig_vendor"])
    E, U = ctx.eigensystem(0)
    own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
    quat, half = ctx.info["eig_quat"], ctx.info["eig_half"]
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max) if Lx < 32 else None
    ctx.close()
    assert (own, vendor, quat, half) == (1, 0, 1, 1), (own, vendor, quat, half)
    H = O.hermitian_from_upper(cache.H_base)
    scale = 1 + np.max(np.abs(cache.E_n))
    assert np.all(np.isfinite(U))
    assert np.max(np.abs(E - cache.E_n)) <= 1e-12 * scale
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N))) <= 1e-12
    if r is not None:
        _check_transport(r, O.measure_transport_and_spectra(cache, p))


def _check_transport(r, ref):
    for k in ("superfluid_stiffness", "dc_conductivity"):
        assert abs(r[k] - ref[k]) <= 1e-9 * (1 + abs(ref[k])), (k, r[k], ref[k])
    for k in ("optical_conductivity", "dos", "dos_AN", "A_k_omega0"):
        a, b = np.asarray(r[k]), np.asarray(ref[k])
        assert a.shape == b.shape, (k, a.shape, b.shape)
        err = np.max(np.abs(a - b)) if a.size else 0.0
        assert err <= 1e-9 * (1 + np.max(np.abs(b))), (k, err)
    for k in ("omega_grid", "dos_omega_grid"):
        assert np.array_equal(np.asarray(r[k]), ref[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,beta", [(4, 4, 8.0), (6, 6, 16.0), (5, 7, 4.0), (2, 4, 8.0), (8, 8, 16.0)])
def test_transport_matches_oracle(dwhmc, oracle, Lx, Ly, beta):
    O = oracle
    p, dis, D = _case(O, Lx, Ly, beta, seed=Lx * 13 + Ly)
    cache, _, _ = O.evaluate(p, dis, D)
    ref = O.measure_transport_and_spectra(cache, p)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max)
    ctx.close()
    _check_transport(r, ref)


@pytest.mark.gpu
def test_transport_clean_degenerate_spectrum(dwhmc, oracle):
    """scripts/debug_transport.jl:9-95's case (10x10 clean, β = 1000, uniform
    d-wave): exactly degenerate levels, on which rocSOLVER's zheevd returns NaN
    eigenvectors; eigen_solve detects them and re-solves with zheev."""
    O = oracle
    p = O.ModelParameters(10, 10, 1.0, -0.35, -1.0, 0.0, 0.0, 1000.0, 1.6, 0.1)
    N = p.N
    D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(np.complex128)
    cache, _, _ = O.evaluate(p, np.zeros(N), D)
    ref = O.measure_transport_and_spectra(cache, p)
    ctx = _ctx(dwhmc, p, np.zeros(N))
    ctx.set_pairing(D)
    E, U = ctx.eigensystem(0)
    assert np.all(np.isfinite(U))
    assert np.max(np.abs(E - cache.E_n)) <= 1e-12 * (1 + np.max(np.abs(E)))
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * N))) <= 1e-12
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max)
    ctx.close()
    _check_transport(r, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,mu,half,quat,ran_half", [(8, 8, 0.0, "1", "0", 0), (12, 8, 0.0, "1", "0", 0),
                                                          (8, 8, 0.0, "1", "1", 1), (12, 8, 0.0, "1", "1", 1),
                                                          (8, 8, -1.0, "1", "1", 1), (6, 6, -1.08, "0", "1", 0)])
def test_transport_particle_hole_half(dwhmc, oracle, monkeypatch, Lx, Ly, mu, half, quat, ran_half):
    """The particle-hole half measurement: with the eigensolver's half solve
    (columns j < N the partners Θ of columns n2-1-j) J_mn is formed in its
    columns < N only and Λ, the DC sum and σ(ω) run over half the pairs.  A
    clean lattice at μ = 0 with L % 4 == 0 has exact zero modes: the
    one-stage solver (quat = "0") solves that cluster across E = 0 whole, so
    U is not partner-closed there and every pair is summed; the
    structure-preserving solver orthonormalises the crowd together with its
    Θ partners (k_q_orth), so U stays partner-closed and the half sums run.
    half = "0" (DWHMC_EIG_HALF=0): the full solve and sums.  ran_half: which
    path the library reports it took (dwh_info_t::eig_half), so the half-sum
    code cannot pass silently on the full path."""
    O = oracle
    monkeypatch.setenv("DWHMC_EIG_HALF", half)
    monkeypatch.setenv("DWHMC_EIG_QUAT", quat)
    p = O.ModelParameters(Lx, Ly, 1.0, -0.35, mu, 0.0, 0.0, 16.0, 0.8, 1.0)
    N = p.N
    D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(np.complex128)
    D = D * np.exp(0.2j * np.random.default_rng(Lx + Ly).standard_normal((N, 1)))   # complex, non-uniform phases
    if mu == 0.0:
        D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(np.complex128)   # the clean nodes
    cache, _, _ = O.evaluate(p, np.zeros(N), D)
    ref = O.measure_transport_and_spectra(cache, p)
    ctx = _ctx(dwhmc, p, np.zeros(N))
    ctx.set_pairing(D)
    assert ctx.info["eig_half"] == -1
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max)
    assert ctx.info["eig_half"] == ran_half
    assert ctx.info["eig_quat"] == (1 if quat == "1" and half == "1" else 0)
    E, U = ctx.eigensystem(0)
    ctx.close()
    _check_transport(r, ref)
    H = O.hermitian_from_upper(cache.H_base)
    scale = 1 + np.max(np.abs(cache.E_n))
    assert np.max(np.abs(E - cache.E_n)) <= 1e-12 * scale
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * N))) <= 1e-12


@pytest.mark.gpu
def test_transport_coarse_grid_and_chain_select(dwhmc, oracle):
    """Non-default η, Δω, ω_max; chain 1 of a batched context."""
    O = oracle
    p, dis, D = _case(O, 6, 4, 8.0, seed=64)
    p.eta, p.domega, p.omega_max = 0.05, 0.01, 2.5
    _, dis2, D2 = _case(O, 6, 4, 8.0, seed=65)
    cache, _, _ = O.evaluate(p, dis2, D2)
    ref = O.measure_transport_and_spectra(cache, p)
    ctx = _ctx(dwhmc, p, np.stack([dis, dis2]))
    ctx.set_pairing(np.stack([D, D2]))
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max, chain=1)
    ctx.close()
    _check_transport(r, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,nc", [(6, 4, 3), (16, 16, 4)])
def test_transport_batched_matches_per_chain(dwhmc, oracle, Lx, Ly, nc):
    """dwh_measure_transport_batched (strided-batched eigensolves) = per-chain
    dwh_measure_transport = oracle, for every chain of a batched context."""
    O = oracle
    cases = [_case(O, Lx, Ly, 8.0, seed=500 + c) for c in range(nc)]
    p = cases[0][0]
    ctx = _ctx(dwhmc, p, np.stack([c[1] for c in cases]))
    ctx.set_pairing(np.stack([c[2] for c in cases]))
    allr = ctx.measure_transport_all(p.eta, p.domega, p.omega_max)
    one = ctx.measure_transport(p.eta, p.domega, p.omega_max, chain=nc - 1)
    ctx.close()
    _check_transport(allr[nc - 1], one)
    for c, (pc, dis, D) in enumerate(cases):
        cache, _, _ = O.evaluate(pc, dis, D)
        _check_transport(allr[c], O.measure_transport_and_spectra(cache, pc))


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,ns", [(6, 4, 5), (16, 16, 3)])
def test_transport_deltas_matches_per_state(dwhmc, oracle, Lx, Ly, ns):
    """dwh_measure_transport_deltas (Δ snapshots of chain 1, eigensolves
    batched over the snapshots) = the oracle at each snapshot on chain 1's
    disorder, and the device state is left as it was."""
    O = oracle
    p, dis0, D0 = _case(O, Lx, Ly, 8.0, seed=700)
    _, dis1, D1 = _case(O, Lx, Ly, 8.0, seed=701)
    snaps = [_case(O, Lx, Ly, 8.0, seed=710 + k)[2] for k in range(ns)]
    ctx = _ctx(dwhmc, p, np.stack([dis0, dis1]))
    ctx.set_pairing(np.stack([D0, D1]))
    rs = ctx.measure_transport_deltas(np.stack(snaps), p.eta, p.domega, p.omega_max, chain=1)
    Dnow, _ = ctx.get_state()
    one = ctx.measure_transport(p.eta, p.domega, p.omega_max, chain=1)
    with pytest.raises(ValueError):
        ctx.measure_transport_deltas(np.stack(snaps), p.eta, p.domega, p.omega_max, chain=2)
    ctx.close()
    assert np.array_equal(Dnow, np.stack([D0, D1]))
    cache, _, _ = O.evaluate(p, dis1, D1)
    _check_transport(one, O.measure_transport_and_spectra(cache, p))
    assert len(rs) == ns
    for k, D in enumerate(snaps):
        cache, _, _ = O.evaluate(p, dis1, D)
        _check_transport(rs[k], O.measure_transport_and_spectra(cache, p))


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,ns,streams", [(6, 4, 9, "1"), (8, 8, 12, "3")])
def test_transport_deltas_sub_batch_streams(dwhmc, oracle, monkeypatch, Lx, Ly, ns, streams):
    """Batches of 8+ matrices tridiagonalise as sub-batches on their own
    streams (two by default; DWHMC_EIG_STREAMS sets the count): every
    snapshot's result is bit-identical to the one-stream / three-stream run
    (each matrix sees the same kernels and deferral depth) and equals the
    oracle."""
    O = oracle
    p, dis, D0 = _case(O, Lx, Ly, 8.0, seed=900)
    snaps = [_case(O, Lx, Ly, 8.0, seed=910 + k)[2] for k in range(ns)]
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D0)
    monkeypatch.delenv("DWHMC_EIG_STREAMS", raising=False)
    rs = ctx.measure_transport_deltas(np.stack(snaps), p.eta, p.domega, p.omega_max)
    monkeypatch.setenv("DWHMC_EIG_STREAMS", streams)
    ro = ctx.measure_transport_deltas(np.stack(snaps), p.eta, p.domega, p.omega_max)
    ctx.close()
    assert len(rs) == len(ro) == ns
    for a, b in zip(rs, ro):
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    for k in (0, ns // 2, ns - 1):
        cache, _, _ = O.evaluate(p, dis, snaps[k])
        _check_transport(rs[k], O.measure_transport_and_spectra(cache, p))


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,mu", [(8, 8, 0.0), (12, 10, -1.0)])
def test_transport_deltas_clean_structure_preserving(dwhmc, oracle, Lx, Ly, mu):
    """A batch of clean-lattice snapshots through the structure-preserving
    eigensolver: uniform d-wave Δ under global phases (degenerate shells; at
    μ = 0 the nodal zero modes, a crowd at zero) mixed with non-uniform
    phases (no exact degeneracy), so one k_q_orth launch sees matrices with
    and without clusters.  eig_quat == 1 and every snapshot equals the
    oracle."""
    O = oracle
    p = O.ModelParameters(Lx, Ly, T, TP, mu, 0.0, 0.0, 16.0, 0.8, 1.0)
    N = p.N
    dis = np.zeros(N)
    base = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(np.complex128)
    rng = np.random.default_rng(Lx * 7 + Ly)
    snaps = [base * np.exp(1j * ph) for ph in (0.0, 0.7, -2.1)]
    snaps += [base * np.exp(0.2j * rng.standard_normal((N, 1))) for _ in range(2)]
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(snaps[0])
    rs = ctx.measure_transport_deltas(np.stack(snaps), p.eta, p.domega, p.omega_max)
    quat, half = ctx.info["eig_quat"], ctx.info["eig_half"]
    ctx.close()
    assert (quat, half) == (1, 1), (quat, half)
    for k, D in enumerate(snaps):
        cache, _, _ = O.evaluate(p, dis, D)
        _check_transport(rs[k], O.measure_transport_and_spectra(cache, p))


@pytest.mark.gpu
@pytest.mark.parametrize("switch_m", ["0", "64", "512"])
def test_transport_deferred_batch_switch(dwhmc, oracle, monkeypatch, switch_m):
    """Batches of 4+ matrices tridiagonalise with the 8-deep deferral and run
    their last DWHMC_EIG_SWITCH_M columns in the one-matrix scheme (0: the
    deferral to the end, 64: a long deferred run then the switch, 512: at
    n = 512 the switch after the first write pass) -- every setting equals the
    oracle per snapshot."""
    O = oracle
    p, dis, D0 = _case(O, 16, 16, 8.0, seed=950)
    snaps = [_case(O, 16, 16, 8.0, seed=960 + k)[2] for k in range(4)]
    monkeypatch.setenv("DWHMC_EIG_SWITCH_M", switch_m)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D0)
    rs = ctx.measure_transport_deltas(np.stack(snaps), p.eta, p.domega, p.omega_max)
    ctx.close()
    for k in (0, 3):
        cache, _, _ = O.evaluate(p, dis, snaps[k])
        _check_transport(rs[k], O.measure_transport_and_spectra(cache, p))


@pytest.mark.gpu
def test_transport_L32_properties(dwhmc, oracle):
    """BASELINE C3 size (N = 1024): device vs oracle at full size, plus the
    size-independent checks ∫DOS dω ≈ 1 on the grid and A(k,0) ≥ 0."""
    O = oracle
    p, dis, D = _case(O, 32, 32, 16.0, seed=3232)
    cache, _, _ = O.evaluate(p, dis, D)
    ref = O.measure_transport_and_spectra(cache, p)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max)
    ctx.close()
    _check_transport(r, ref)
    assert np.min(r["A_k_omega0"]) >= 0
    # sum rule: ∫ DOS dω over the grid = (1/N) Σ_n W_n ∫_{-ω_max}^{ω_max} L(ω - E_n) dω
    # (the band reaches past ω_max, so this is < 1)
    E, Wn = cache.E_n, np.sum(np.abs(cache.U[:p.N]) ** 2, axis=0)
    inside = (np.arctan((p.omega_max - E) / p.eta) - np.arctan((-p.omega_max - E) / p.eta)) / np.pi
    assert abs(np.sum(r["dos"]) * p.domega - np.sum(Wn * inside) / p.N) < 2e-3


@pytest.mark.gpu
def test_transport_argument_errors(dwhmc, oracle):
    O = oracle
    p, dis, D = _case(O, 4, 4, 8.0, seed=1)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    with pytest.raises(ValueError):
        ctx.measure_transport(-0.01, p.domega, p.omega_max)
    with pytest.raises(ValueError):
        ctx.measure_transport(p.eta, p.domega, p.omega_max, chain=3)
    ctx.close()


@pytest.mark.gpu
def test_host_mirror_measure_transport_and_spectra(dwhmc, oracle):
    """hmc.measure_transport_and_spectra(cache, p) mirrors the reference call
    (src/Simulation.jl:171) on the state the cache's context holds."""
    m, O = dwhmc, oracle
    p = m.ModelParameters(6, 6, T, TP, MU, 1.0, 0.1, 8.0, 0.8, 1.0)
    rng = np.random.default_rng(5)
    st = m.initialize_state(p, rng)
    cache = m.initialize_cache(p)
    m.init_static_H(cache, p, st)
    m.update_H_BdG(cache, p, st)
    m.diagonalize_H_BdG(cache, p)
    res = m.measure_transport_and_spectra(cache, p)
    cache.ctx.close()
    po = O.ModelParameters(6, 6, T, TP, MU, 1.0, 0.1, 8.0, 0.8, 1.0)
    oc, _, _ = O.evaluate(po, st.disorder_pot, st.Delta)
    ref = O.measure_transport_and_spectra(oc, po)
    _check_transport({k: getattr(res, k) for k in ref}, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("Lx,Ly,quat", [(6, 4, "1"), (8, 8, "1"), (12, 8, "1"), (12, 8, "0"), (16, 16, "1")])
def test_transport_structure_preserving_solver(dwhmc, oracle, monkeypatch, Lx, Ly, quat):
    """The measurement on the structure-preserving eigensolver (reduction site
    by site, inverse iteration on the 2 x 2-block tridiagonal T, site
    rotations, reflector-pair back-transform, Θ partners: csrc/dwhmc_qeig.hip)
    against the oracle at the same tolerances, and DWHMC_EIG_QUAT=0 (the
    one-stage solver); dwh_info_t::eig_quat reports which one ran."""
    O = oracle
    monkeypatch.setenv("DWHMC_EIG_QUAT", quat)
    p, dis, D = _case(O, Lx, Ly, 16.0, seed=700 + Lx + Ly)
    cache, _, _ = O.evaluate(p, dis, D)
    ref = O.measure_transport_and_spectra(cache, p)
    ctx = _ctx(dwhmc, p, dis)
    ctx.set_pairing(D)
    r = ctx.measure_transport(p.eta, p.domega, p.omega_max)
    assert ctx.info["eig_quat"] == (1 if quat == "1" else 0)
    assert ctx.info["eig_half"] == 1
    E, U = ctx.eigensystem(0)
    ctx.close()
    _check_transport(r, ref)
    n = 2 * p.N
    H = O.hermitian_from_upper(cache.H_base)
    scale = 1.0 + np.max(np.abs(E))
    assert np.max(np.abs(H @ U - U * E[None, :])) / scale < 1e-12
    assert np.max(np.abs(U.conj().T @ U - np.eye(n))) < 1e-12
