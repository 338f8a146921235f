"""GPU parity: the HIP path through the C ABI vs the CPU oracle.

Tolerances (fp64; the default pole set approximates tanh to <= 5e-12 on the
spectrum, the strict one to <= 2e-14):
  * forces          ‖F_gpu - F_ref‖∞ ≤ 1e-10 (1 + ‖F_ref‖∞)
  * pairing P_ij    ‖P_gpu - P_ref‖∞ ≤ 1e-11
  * E_f             |ΔE_f| ≤ 1e-11 |E_f|
  * hole density    |Δ hole_conc| ≤ 1e-11
  * HMC sweep       |ΔdH| ≤ 1e-8 (1 + |dH|), Δ after the sweep ≤ 1e-10, accept flag equal
The oracle restates the reference with LAPACK zheevr (oracle/dwhmc_oracle.py).
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T, TP, MU, J = 1.0, -0.35, -1.08, 0.8


def make_case(O, Lx, Ly, beta, seed, W=1.0, nimp=0.05, amp=0.3, mu=MU, tp=TP, Jc=J):
    p = O.ModelParameters(Lx, Ly, T, tp, mu, W, nimp, beta, Jc, 1.0)
    rng = np.random.default_rng(seed)
    st = O.initialize_state(p, rng)
    N = p.N
    dwave = np.stack([np.ones(N), -np.ones(N)], axis=1) * amp
    Delta = st.Delta + dwave * (1 + 0.3 * rng.standard_normal((N, 1))) * np.exp(1j * 0.2 * rng.standard_normal((N, 1)))
    return p, st.disorder_pot, Delta


@pytest.fixture(params=["cr", "dense"])
def algo(request):
    """Both factorisations (include/dwhmc.h DWH_ALGO_*) must meet the same bar."""
    return request.param


@pytest.fixture(params=["cr", "dense", "eig"])
def algo3(request):
    """The two pole factorisations and the eigendecomposition path (the one
    the context falls back to beyond the pole table)."""
    return request.param


def device_ctx(dwhmc, p, disorder, algo="auto", **kw):
    ctx = dwhmc.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                               disorder, algo=algo, **kw)
    if algo != "auto":
        assert ctx.info["algo"] == {"dense": 0, "cr": 1, "eig": 2}[algo]
    return ctx


def test_mfma_f64_layout(dwhmc):
    assert dwhmc.selftest_mfma(0) == 0


# (20, 6) and (36, 4): BP = 64 and 96 with even Ly >= 4, i.e. the default
# sparse level 0 (on from BP = 64) in the fast sweep, ahead of the full-size
# tests
@pytest.mark.parametrize("Lx,Ly,beta", [(4, 4, 4.0), (6, 6, 8.0), (5, 7, 16.0), (8, 8, 16.0),
                                        (16, 16, 8.0), (16, 8, 16.0), (3, 3, 4.0), (2, 2, 4.0),
                                        (2, 5, 8.0), (20, 6, 8.0), (36, 4, 16.0)])
def test_factorize_matches_oracle(dwhmc, oracle, Lx, Ly, beta, algo3):
    algo = algo3
    O = oracle
    p, dis, Delta = make_case(O, Lx, Ly, beta, seed=Lx * 100 + Ly)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, algo)
    if algo == "cr" and Lx in (20, 36):
        assert ctx.info["block"] == {20: 64, 36: 96}[Lx]
    ctx.set_pairing(Delta)
    ctx.factorize()
    P = ctx.pairing()[0]
    F = ctx.forces()[0]
    Ef = ctx.fermion_energy()[0]
    assert np.max(np.abs(P - P_ref)) <= 1e-11, np.max(np.abs(P - P_ref))
    assert np.max(np.abs(F - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(Ef - Ef_ref) <= 1e-11 * abs(Ef_ref), (Ef, Ef_ref)
    # hole density from Tr ρ_hh (src/Observables.jl:120-145)
    hole_ref = O.measure_observables(cache, p, Delta)["hole_conc"]
    hole = 2.0 * ctx.hole_trace()[0] / p.N - 1.0
    assert abs(hole - hole_ref) <= 1e-11, (hole, hole_ref)
    ctx.close()


def test_full_size_L32_beta16(dwhmc, oracle, algo3):
    algo = algo3
    """BASELINE config C3 size (N = 1024, n = 2048) against the eigen oracle."""
    O = oracle
    p, dis, Delta = make_case(O, 32, 32, 16.0, seed=3232)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    ctx = device_ctx(dwhmc, p, dis, algo)
    ctx.set_pairing(Delta)
    ctx.factorize()
    F = ctx.forces()[0]
    Ef = ctx.fermion_energy()[0]
    assert np.max(np.abs(F - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(Ef - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


def test_full_size_L48_beta32_batched(dwhmc, oracle, algo):
    """BASELINE config C5 (N = 2304, n = 4608, β = 32) at its real batch: four
    chains with different disorder in one context (nbatch = 4 x the poles,
    the side-work placement of the bench's schedule), against the eigen
    oracle."""
    O = oracle
    cases = [make_case(O, 48, 48, 32.0, seed=s) for s in (4848, 4849, 4850, 4851)]
    p = cases[0][0]
    ctx = device_ctx(dwhmc, p, np.stack([c[1] for c in cases]), algo)
    assert ctx.info["npoles"] >= 12 and ctx.info["nchains"] == 4
    ctx.set_pairing(np.stack([c[2] for c in cases]))
    ctx.factorize()
    F = ctx.forces()
    Ef = ctx.fermion_energy()
    for c, (pc, dc, Dc) in enumerate(cases):
        _, F_ref, Ef_ref = O.evaluate(pc, dc, Dc)
        assert np.max(np.abs(F[c] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
        assert abs(Ef[c] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


def test_batched_chains_independent(dwhmc, oracle, algo3):
    algo = algo3
    O = oracle
    cases = [make_case(O, 6, 6, 8.0, seed=s) for s in (1, 2, 3)]
    p = cases[0][0]
    dis = np.stack([c[1] for c in cases])
    Delta = np.stack([c[2] for c in cases])
    ctx = device_ctx(dwhmc, p, dis, algo)
    ctx.set_pairing(Delta)
    ctx.factorize()
    F = ctx.forces()
    Ef = ctx.fermion_energy()
    for c, (pc, dc, Dc) in enumerate(cases):
        _, F_ref, Ef_ref = O.evaluate(pc, dc, Dc)
        assert np.max(np.abs(F[c] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
        assert abs(Ef[c] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


def test_clean_dwave_closed_form_on_device(dwhmc, oracle, algo3):
    algo = algo3
    """I5 / scripts/benchmark_clean.jl:15-43 directly on the HIP path."""
    O = oracle
    L, beta, D0 = 8, 16.0, 0.25
    p = O.ModelParameters(L, L, T, TP, MU, 0.0, 0.0, beta, J, 1.0)
    Delta = np.stack([np.full(p.N, D0), np.full(p.N, -D0)], axis=1).astype(np.complex128)
    _, Px, Fx, Ef = O.clean_dwave_closed_form(D0, L, L, T, TP, MU, beta, J)
    ctx = device_ctx(dwhmc, p, np.zeros(p.N), algo)
    ctx.set_pairing(Delta)
    ctx.factorize()
    P = ctx.pairing()[0]
    F = ctx.forces()[0]
    assert np.max(np.abs(P[:, 0] - Px)) <= 1e-11
    assert np.max(np.abs(P[:, 1] + Px)) <= 1e-11
    assert np.max(np.abs(F[:, 0] - Fx)) <= 1e-10
    assert abs(ctx.fermion_energy()[0] - Ef) <= 1e-11 * abs(Ef)
    ctx.close()


def _oracle_after_sweeps(O, p, dis, Delta0, draws, Nt, dt, factorize_first=True):
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    st = O.SimulationState(dis, Delta0.copy(), np.zeros_like(Delta0))
    O.update_H_BdG(cache, p, st.Delta)
    if factorize_first:
        O.diagonalize_H_BdG(cache, p)
    out = []
    for noise, u in draws:
        acc, dH = O.hmc_sweep(cache, p, st, Nt, dt, noise, u)
        out.append((acc, dH, st.Delta.copy(), st.pi.copy()))
    return out


@pytest.mark.parametrize("factorize_first,Lx,Ly", [(True, 6, 6), (False, 6, 6), (True, 2, 4), (True, 3, 2)])
def test_hmc_sweep_matches_oracle(dwhmc, oracle, factorize_first, Lx, Ly, algo3):
    algo = algo3
    """hmc_sweep! (src/HMC.jl:71-144) with injected draws; factorize_first=False
    reproduces the zeroed-cache first sweep of scripts/benchmark_clean.jl:82-88.
    The 2x4 and 3x2 lattices map several bonds onto one pairing entry (the
    reference's overwrite order, src/Hamiltonian.jl:68-83) inside trajectories."""
    O = oracle
    p, dis, Delta0 = make_case(O, Lx, Ly, 8.0, seed=77 + Lx, amp=0.1)
    Nt = 6
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
    rng = np.random.default_rng(5)
    draws = [((rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5),
              float(rng.random())) for _ in range(4)]
    ref = _oracle_after_sweeps(O, p, dis, Delta0, draws, Nt, dt, factorize_first)
    ctx = device_ctx(dwhmc, p, dis, algo)
    ctx.set_pairing(Delta0)
    if factorize_first:
        ctx.factorize()
    for (noise, u), (acc_r, dH_r, D_r, pi_r) in zip(draws, ref):
        acc, dH = ctx.hmc_sweep(noise, np.array([u]), Nt, dt, p.mass)
        D, pi = ctx.get_state()
        assert abs(dH[0] - dH_r) <= 1e-8 * (1 + abs(dH_r)), (dH[0], dH_r)
        assert bool(acc[0]) == acc_r
        assert np.max(np.abs(D[0] - D_r)) <= 1e-10
        assert np.max(np.abs(pi[0] - pi_r)) <= 1e-9
    ctx.close()


def test_throughput_path_equals_single_sweeps(dwhmc, oracle, algo3):
    algo = algo3
    O = oracle
    p, dis, Delta0 = make_case(O, 8, 8, 8.0, seed=9, amp=0.1)
    Nt, ns = 4, 3
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
    rng = np.random.default_rng(11)
    noise = (rng.standard_normal((ns, 2, p.N, 2)) + 1j * rng.standard_normal((ns, 2, p.N, 2))) * math.sqrt(0.5)
    uni = rng.random((ns, 2))
    dis2 = np.stack([dis, dis[::-1].copy()])
    D2 = np.stack([Delta0, Delta0[::-1].copy()])
    a = device_ctx(dwhmc, p, dis2, algo)
    a.set_pairing(D2)
    a.factorize()
    res_single = [a.hmc_sweep(noise[s], uni[s], Nt, dt, p.mass) for s in range(ns)]
    Da, _ = a.get_state()
    b = device_ctx(dwhmc, p, dis2, algo)
    b.set_pairing(D2)
    b.factorize()
    b.load_draws(noise, uni)
    b.run_sweeps(0, ns, Nt, dt, p.mass)
    acc, dH = b.sweep_results(0, ns)
    Db, _ = b.get_state()
    for s in range(ns):
        assert np.array_equal(acc[s], res_single[s][0])
        assert np.array_equal(dH[s], res_single[s][1])
    assert np.array_equal(Da, Db)
    a.close()
    b.close()


def test_spectrum_guard_reselects_on_upload(dwhmc, oracle, algo):
    """An uploaded Δ above delta_cap re-selects the pole set for it (the
    reference accepts any Δ, src/HMC.jl:98-114) instead of silently using
    poles that do not cover the spectrum.  dense: bond guard (max|Δ_ij|);
    cr: site guard (the largest mean |Δ| over a site's bonds)."""
    O = oracle
    p, dis, Delta0 = make_case(O, 4, 4, 4.0, seed=1, amp=0.9)
    ctx = device_ctx(dwhmc, p, dis, algo, delta_cap=0.5)
    kap0 = ctx.info["kappa"]
    ctx.set_pairing(Delta0)
    inf = ctx.info
    m = np.max(np.abs(Delta0)) if algo == "dense" else _site_mean_max(Delta0, p)
    assert inf["delta_cap"] >= 1.5 * m * (1 - 1e-12) and inf["kappa"] > kap0
    ctx.factorize()
    _, F_ref, Ef_ref = O.evaluate(p, dis, Delta0)
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(ctx.fermion_energy()[0] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


def test_spectrum_guard_reselects_mid_sweep(dwhmc, oracle, algo):
    """A trajectory that drifts |Δ| past the cap is rerun from its start with a
    re-selected pole set; the result is that of a context built with the final
    cap from the outset, and matches the oracle."""
    O = oracle
    p, dis, Delta0 = make_case(O, 4, 4, 4.0, seed=2, amp=0.0)
    rng = np.random.default_rng(3)
    noise = 8.0 * (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
    Nt, dt = 4, 0.1
    a = device_ctx(dwhmc, p, dis, algo, delta_cap=0.2)
    a.set_pairing(Delta0)
    a.factorize()
    acc_a, dH_a = a.hmc_sweep(noise, np.array([0.3]), Nt, dt, p.mass)
    cap = a.info["delta_cap"]
    assert cap > 0.2
    b = device_ctx(dwhmc, p, dis, algo, delta_cap=cap)
    b.set_pairing(Delta0)
    b.factorize()
    acc_b, dH_b = b.hmc_sweep(noise, np.array([0.3]), Nt, dt, p.mass)
    assert acc_a[0] == acc_b[0] and dH_a[0] == dH_b[0]
    for x, y in zip(a.get_state(), b.get_state()):
        assert np.array_equal(x, y)
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, Delta0)
    O.diagonalize_H_BdG(cache, p)
    st = O.SimulationState(dis, Delta0.copy(), np.zeros_like(Delta0))
    acc_r, dH_r = O.hmc_sweep(cache, p, st, Nt, dt, noise, 0.3)
    assert acc_a[0] == acc_r and abs(dH_a[0] - dH_r) <= 1e-8 * (1 + abs(dH_r))
    a.close()
    b.close()


def test_default_delta_cap_follows_temperature(dwhmc, oracle):
    """delta_cap <= 0 selects max(2, 6 sqrt(2J/β)) for the bond guard (dense
    path) and max(1.25, 4 sqrt(2J/β)) for the site guard (CR path): wide enough
    for the boson fluctuations of the reference's high-temperature scans
    (scripts/batch_scan_T.jl:21-22 goes up to T = 1000)."""
    O = oracle
    for beta in (16.0, 0.5, 1e-3):
        p, dis, _ = make_case(O, 4, 4, beta, seed=4)
        ctx = device_ctx(dwhmc, p, dis, "dense", delta_cap=0.0)
        assert ctx.info["delta_cap"] == pytest.approx(max(2.0, 6.0 * math.sqrt(2 * J / beta)))
        ctx.close()
        ctx = device_ctx(dwhmc, p, dis, "auto", delta_cap=0.0)
        assert ctx.info["algo"] == 1
        assert ctx.info["delta_cap"] == pytest.approx(max(1.25, 4.0 * math.sqrt(2 * J / beta)))
        ctx.close()


def _site_mean_max(D, p):
    a = np.abs(D)
    nn = p.nn_table - 1
    return float(np.max(0.25 * (a[:, 0] + a[:, 1] + a[nn[:, 2], 0] + a[nn[:, 3], 1])))


def test_site_guard_default_cap(dwhmc, oracle):
    """CR contexts guard the mean |Δ| over each site's four bonds (checked by
    the level-0 inversion launch: k_cr_inv0 / k_cr_inv0_32, k_cr_inv or
    k_cr_inv_side),
    default max(1.25, 4 sqrt(2J/β)); E' = ‖h‖ + 2 cap bounds the spectrum
    either way.  At the C3 workload that is 13 pole pairs instead of 14."""
    O = oracle
    for (Lx, Ly), beta in (((20, 20), 16.0), ((20, 20), 2.0), ((12, 6), 8.0), ((40, 4), 8.0)):
        p, dis, _ = make_case(O, Lx, Ly, beta, seed=5)
        ctx = device_ctx(dwhmc, p, dis, "cr", delta_cap=0.0)
        assert ctx.info["delta_cap"] == pytest.approx(max(1.25, 4.0 * math.sqrt(2 * J / beta)))
        assert ctx.info["e_bound"] >= ctx.info["delta_cap"] * 2
        ctx.close()
    p, dis, _ = make_case(O, 32, 32, 16.0, seed=1000)
    ctx = device_ctx(dwhmc, p, dis, "cr", delta_cap=0.0)
    # κ = 73.7 takes the κ = 76.1 entry: 12 pole pairs in the default
    # (5e-12) table, 13 in the strict one
    assert ctx.info["npoles"] == (13 if os.environ.get("DWHMC_POLE_TABLE") == "strict" else 12)
    ctx.close()


def test_site_guard_reselects_on_upload(dwhmc, oracle):
    """Site guard: an uploaded Δ whose largest site mean exceeds the cap
    re-selects the poles for 1.5 x that mean; results match the oracle."""
    O = oracle
    p, dis, Delta = make_case(O, 20, 6, 8.0, seed=21, amp=0.9)
    ctx = device_ctx(dwhmc, p, dis, "cr", delta_cap=0.3)
    kap0 = ctx.info["kappa"]
    ctx.set_pairing(Delta)
    m = _site_mean_max(Delta, p)
    assert ctx.info["delta_cap"] >= 1.5 * m * (1 - 1e-12) and ctx.info["kappa"] > kap0
    ctx.factorize()
    _, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(ctx.fermion_energy()[0] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


@pytest.mark.parametrize("inv0", ["1", "0"])
@pytest.mark.parametrize("Lx,Ly", [(20, 4), (40, 3), (12, 5)])
def test_site_guard_reselects_mid_sweep(dwhmc, oracle, monkeypatch, Lx, Ly, inv0):
    """Site guard: a trajectory whose drift takes a site mean past the cap is
    rerun from its start with re-selected poles (the level-0 inversion launch
    sets the flag: k_cr_inv0 / k_cr_inv0_32, or with DWHMC_CR_INV0=0 k_cr_inv
    / k_cr_inv32); the result equals a context built with the final cap and
    matches the oracle."""
    monkeypatch.setenv("DWHMC_CR_INV0", inv0)
    O = oracle
    p, dis, Delta0 = make_case(O, Lx, Ly, 4.0, seed=22 + Lx, amp=0.0)
    rng = np.random.default_rng(23)
    noise = 8.0 * (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
    Nt, dt = 4, 0.1
    a = device_ctx(dwhmc, p, dis, "cr", delta_cap=0.2)
    a.set_pairing(Delta0)
    a.factorize()
    acc_a, dH_a = a.hmc_sweep(noise, np.array([0.3]), Nt, dt, p.mass)
    cap = a.info["delta_cap"]
    assert cap > 0.2
    b = device_ctx(dwhmc, p, dis, "cr", delta_cap=cap)
    b.set_pairing(Delta0)
    b.factorize()
    acc_b, dH_b = b.hmc_sweep(noise, np.array([0.3]), Nt, dt, p.mass)
    assert acc_a[0] == acc_b[0] and dH_a[0] == dH_b[0]
    for x, y in zip(a.get_state(), b.get_state()):
        assert np.array_equal(x, y)
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, Delta0)
    O.diagonalize_H_BdG(cache, p)
    st = O.SimulationState(dis, Delta0.copy(), np.zeros_like(Delta0))
    acc_r, dH_r = O.hmc_sweep(cache, p, st, Nt, dt, noise, 0.3)
    assert acc_a[0] == acc_r and abs(dH_a[0] - dH_r) <= 1e-8 * (1 + abs(dH_r))
    a.close()
    b.close()


@pytest.mark.parametrize("algo_g,Lx,Ly", [("cr", 20, 4), ("cr", 12, 5), ("dense", 6, 6)])
def test_guard_trip_recovers_in_throughput_path(dwhmc, oracle, algo_g, Lx, Ly):
    """A guard trip in the middle of a dwh_run_sweeps batch (sweep 2 of 5, in
    chain 1 of 2): the later sweeps of the batch become no-ops on the device,
    and dwh_sweep_results re-selects the poles, resumes from the tripped
    sweep's backed-up Δ and replays sweeps 2..4 — the same steps
    dwh_hmc_sweep takes for a trip (src/HMC.jl:98-114 accepts any Δ).  Every
    sweep's accept flag and ΔH, the final Δ, π and the re-selected pole set
    equal the single-sweep path bit for bit.  cr: site guard (level-0
    inversion launch); dense: bond guard (drift kernels)."""
    O = oracle
    p, dis, Delta0 = make_case(O, Lx, Ly, 4.0, seed=24 + Lx, amp=0.0)
    ns, Nt, dt = 5, 4, 0.1
    rng = np.random.default_rng(25)
    noise = (rng.standard_normal((ns, 2, p.N, 2)) + 1j * rng.standard_normal((ns, 2, p.N, 2))) * math.sqrt(0.5)
    scale = np.full((ns, 2), 0.05)
    scale[2, 1] = 8.0                                  # the trip: sweep 2, chain 1
    noise *= scale[:, :, None, None]
    uni = rng.random((ns, 2))
    dis2 = np.stack([dis, dis[::-1].copy()])
    D2 = np.stack([Delta0, Delta0[::-1].copy()])
    cap0 = 0.2
    a = device_ctx(dwhmc, p, dis2, algo_g, delta_cap=cap0)
    a.set_pairing(D2)
    a.factorize()
    ref = []
    for s in range(ns):
        ref.append(a.hmc_sweep(noise[s], uni[s], Nt, dt, p.mass))
        if s == 1:
            assert a.info["delta_cap"] == cap0          # no trip before sweep 2
    assert a.info["delta_cap"] > cap0                   # sweep 2 tripped
    b = device_ctx(dwhmc, p, dis2, algo_g, delta_cap=cap0)
    b.set_pairing(D2)
    b.factorize()
    b.load_draws(noise, uni)
    b.run_sweeps(0, ns, Nt, dt, p.mass)
    acc, dH = b.sweep_results(0, ns)
    for s in range(ns):
        assert np.array_equal(acc[s], ref[s][0]), s
        assert np.array_equal(dH[s], ref[s][1]), s
    for x, y in zip(a.get_state(), b.get_state()):
        assert np.array_equal(x, y)
    ia, ib = a.info, b.info
    assert (ia["delta_cap"], ia["kappa"], ia["npoles"]) == (ib["delta_cap"], ib["kappa"], ib["npoles"])
    # load_draws / run_sweeps / load_draws / sweep_results: the
    # second upload settles the pending batch first, so its replay after the
    # trip reads the draws it was enqueued with, not the new ones
    c = device_ctx(dwhmc, p, dis2, algo_g, delta_cap=cap0)
    c.set_pairing(D2)
    c.factorize()
    c.load_draws(noise, uni)
    c.run_sweeps(0, ns, Nt, dt, p.mass)
    c.load_draws(noise[::-1].copy() * 3.0, uni[::-1].copy())
    acc, dH = c.sweep_results(0, ns)
    for s in range(ns):
        assert np.array_equal(acc[s], ref[s][0]), s
        assert np.array_equal(dH[s], ref[s][1]), s
    for x, y in zip(a.get_state(), c.get_state()):
        assert np.array_equal(x, y)
    a.close()
    b.close()
    c.close()


def test_reselection_keeps_stream(dwhmc, oracle):
    """dwh_stream's handle stays valid across a guard re-selection."""
    O = oracle
    p, dis, Delta0 = make_case(O, 20, 4, 4.0, seed=31, amp=0.9)
    ctx = device_ctx(dwhmc, p, dis, "cr", delta_cap=0.3)
    s0 = ctx.stream()
    ctx.set_pairing(Delta0)                            # re-selects (site mean > 0.3)
    assert ctx.info["delta_cap"] > 0.3
    assert ctx.stream() == s0
    ctx.factorize()
    ctx.close()


def test_high_temperature_sweeps_match_oracle(dwhmc, oracle):
    """T = 2 (β = 0.5): |Δ| ~ sqrt(2J/β) ~ 1.8, beyond the old fixed cap of 2 in a
    few bonds; sweeps run without a guard failure and match the oracle."""
    O = oracle
    p, dis, _ = make_case(O, 6, 6, 0.5, seed=8)
    rng = np.random.default_rng(12)
    Delta = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(p.J / p.beta)
    ctx = device_ctx(dwhmc, p, dis, "auto", delta_cap=0.0)
    ctx.set_pairing(Delta)
    ctx.factorize()
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, Delta)
    O.diagonalize_H_BdG(cache, p)
    st = O.SimulationState(dis, Delta.copy(), np.zeros_like(Delta))
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, 10)
    for s in range(4):
        noise = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
        u = rng.random()
        acc, dH = ctx.hmc_sweep(noise, np.array([u]), 10, dt, p.mass)
        acc_r, dH_r = O.hmc_sweep(cache, p, st, 10, dt, noise, u)
        assert acc[0] == acc_r and abs(dH[0] - dH_r) <= 1e-8 * (1 + abs(dH_r)), (s, dH[0], dH_r)
    D, _ = ctx.get_state()
    assert np.max(np.abs(D[0] - st.Delta)) <= 1e-10
    ctx.close()


def test_host_mirror_api_roundtrip(dwhmc, oracle):
    """The reference-named API (init_static_H ... hmc_sweep) drives the device."""
    O = oracle
    m = dwhmc
    p = m.ModelParameters(6, 6, T, TP, MU, 1.0, 0.05, 8.0, J, 1.0)
    st = m.initialize_state(p, np.random.default_rng(4))
    cache = m.initialize_cache(p)
    m.init_static_H(cache, p, st)
    m.update_H_BdG(cache, p, st)
    m.diagonalize_H_BdG(cache, p)
    m.compute_forces(cache, p, st)
    po = O.ModelParameters(6, 6, T, TP, MU, 1.0, 0.05, 8.0, J, 1.0)
    oc, F_ref, Ef_ref = O.evaluate(po, st.disorder_pot, st.Delta)
    assert np.max(np.abs(cache.forces - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    obs = m.measure_observables(cache, p, st)
    obs_ref = O.measure_observables(oc, po, st.Delta)
    for k in O.OBS_FIELDS:
        a, b = getattr(obs, k), obs_ref[k]
        assert abs(a - b) <= 1e-10 * (1 + abs(b)), (k, a, b)
    acc, dH = m.hmc_sweep(cache, p, st, Nt=4, dt=m.calc_optimal_dt(p.beta, p.J, p.mass, 4),
                          rng=np.random.default_rng(0))
    assert np.isfinite(dH)


@pytest.mark.parametrize("L", [4, 8])
def test_golden_fixture_on_device(dwhmc, L, algo):
    """Committed oracle vectors (tests/golden/oracle_L*.npz, tests/make_golden.py)."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"oracle_L{L}.npz"), allow_pickle=False)
    beta = float(g["beta"])
    ctx = dwhmc.FermionContext(L, L, T, TP, MU, beta, J, g["nn"], g["nnn"], g["disorder"], algo=algo)
    ctx.set_pairing(g["Delta"])
    ctx.factorize()
    F = ctx.forces()[0]
    assert np.max(np.abs(F - g["F"])) <= 1e-10 * (1 + np.max(np.abs(g["F"])))
    assert abs(ctx.fermion_energy()[0] - float(g["Ef"])) <= 1e-11 * abs(float(g["Ef"]))
    acc, dH = ctx.hmc_sweep(g["sweep_noise"], np.array([float(g["sweep_uniform"])]), int(g["sweep_Nt"]),
                            float(g["sweep_dt"]), 1.0)
    assert abs(dH[0] - float(g["sweep_dH"])) <= 1e-8 * (1 + abs(float(g["sweep_dH"])))
    assert bool(acc[0]) == bool(g["sweep_accepted"])
    D, pi = ctx.get_state()
    assert np.max(np.abs(D[0] - g["sweep_Delta"])) <= 1e-10
    ctx.close()


def test_cr_block_limit(dwhmc, oracle):
    """DWH_ALGO_CR needs the padded lattice-row block 2 Lx <= 128; auto falls back to dense."""
    O = oracle
    p, dis, _ = make_case(O, 65, 2, 4.0, seed=1)
    with pytest.raises(ValueError):
        device_ctx(dwhmc, p, dis, "cr")
    ctx = device_ctx(dwhmc, p, dis)
    assert ctx.info["algo"] == 0
    ctx.close()


@pytest.mark.parametrize("Lx,Ly", [(4, 1), (6, 2), (5, 3), (3, 9), (7, 6), (48, 5), (16, 13), (64, 1), (64, 2),
                                   (64, 3), (50, 4), (57, 2), (24, 7), (32, 5), (17, 9), (20, 11), (32, 3),
                                   (29, 2), (32, 1)])
def test_cr_ragged_chains(dwhmc, oracle, Lx, Ly):
    """Cyclic-reduction chains of every shape: Ly = 1 (one block), 2 (single
    off-diagonal block), odd lengths at every level, padded blocks (2 Lx not a
    multiple of 32), against the eigen oracle.  Every case runs the
    static-particle-block level-0 inversions: k_cr_inv0_32 on the BP = 32
    chains (Lx <= 16, one-wave Schur complement), k_cr_inv0 on the BP = 64
    ones (17 <= Lx <= 32, which also run the side-work schedule,
    k_cr_inv_side), k_cr_inv0_96 on the BP = 96 ones (33 <= Lx <= 48) on odd
    and short chains."""
    O = oracle
    p, dis, Delta = make_case(O, Lx, Ly, 8.0, seed=Lx * 31 + Ly)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    Ef = ctx.fermion_energy()[0]
    assert abs(Ef - Ef_ref) <= 1e-11 * abs(Ef_ref), (Ef, Ef_ref)
    hole_ref = O.measure_observables(cache, p, Delta)["hole_conc"]
    assert abs(2.0 * ctx.hole_trace()[0] / p.N - 1.0 - hole_ref) <= 1e-11
    ctx.close()


@pytest.mark.parametrize("inv0,inv32", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")])
@pytest.mark.parametrize("Lx,Ly", [(12, 5), (16, 6), (8, 8), (20, 3)])
def test_cr_inversion_variants(dwhmc, oracle, monkeypatch, Lx, Ly, inv0, inv32):
    """The CR inversion kernels against the eigen oracle: level 0 from the
    static particle block (k_cr_inv0_32 / k_cr_inv0, DWHMC_CR_INV0) or whole;
    BP = 32 blocks by the one-wave Schur complement (k_cr_inv32,
    DWHMC_CR_INV32) or the two-wave panel inversion (k_cr_inv<2>).  8 x 8
    runs two-row BP = 32 blocks, 20 x 3 BP = 64 (k_cr_inv32 unused)."""
    O = oracle
    monkeypatch.setenv("DWHMC_CR_INV0", inv0)
    monkeypatch.setenv("DWHMC_CR_INV32", inv32)
    p, dis, Delta = make_case(O, Lx, Ly, 8.0, seed=Lx * 13 + Ly)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(ctx.fermion_energy()[0] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


@pytest.mark.parametrize("cfg", ["16:1", "16:2", "16:4", "32:1", "32:2"])
@pytest.mark.parametrize("Lx,Ly", [(20, 6), (40, 3), (12, 5), (16, 8)])
def test_cr_block_product_variants(dwhmc, oracle, monkeypatch, cfg, Lx, Ly):
    """Every compiled block-product kernel variant (16x16 / 32x32 wave tiles,
    K split 1/2/4; DWHMC_CR_GEMM, read at context creation) against the eigen
    oracle, on BP = 64 (Lx = 20), 96 (Lx = 40) and 32 (Lx = 12, 16) blocks
    (16 x 8: the sparse level 0 forced on, and its one-term restricted
    stages).  32-wide tiles need BP/2 % 32 == 0 and fall back to 16x16
    otherwise."""
    O = oracle
    monkeypatch.setenv("DWHMC_CR_GEMM", cfg)
    monkeypatch.setenv("DWHMC_CR_SPARSE0", "1")
    p, dis, Delta = make_case(O, Lx, Ly, 8.0, seed=Lx * 7 + Ly)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    Ef = ctx.fermion_energy()[0]
    assert abs(Ef - Ef_ref) <= 1e-11 * abs(Ef_ref), (Ef, Ef_ref)
    ctx.close()


def test_split_trajectory_matches_sweep(dwhmc, oracle):
    """dwh_hmc_trajectory + dwh_hmc_finish (the host decides acceptance, as the
    Julia binding does to consume its RNG like src/HMC.jl:128) reproduce
    dwh_hmc_sweep bit for bit, accepted and rejected sweeps alike."""
    O = oracle
    p, dis, Delta = make_case(O, 4, 4, 8.0, seed=3)
    a = device_ctx(dwhmc, p, dis)
    b = device_ctx(dwhmc, p, dis)
    for c in (a, b):
        c.set_pairing(Delta)
        c.factorize()
    rng = np.random.default_rng(9)
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, 1)      # coarse, and u near 1 on odd sweeps:
    seen = set()                                         # some trajectories are rejected
    for k in range(8):
        noise = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
        u = 0.9999 if k % 2 else rng.random()
        acc1, dH1 = a.hmc_sweep(noise, np.array([u]), 4, dt, p.mass)
        dH2 = b.hmc_trajectory(noise, 4, dt, p.mass)
        acc2 = bool(dH2[0] < 0 or u < math.exp(-dH2[0]))
        b.hmc_finish([acc2])
        assert acc1[0] == acc2 and dH1[0] == dH2[0]
        seen.add(acc2)
        for x, y in zip(a.get_state(), b.get_state()):
            assert np.array_equal(x, y)
        assert np.array_equal(a.pairing(), b.pairing())
        assert np.array_equal(a.fermion_energy(), b.fermion_energy())
    assert seen == {True, False}
    # call order is enforced
    noise = np.zeros((p.N, 2), dtype=np.complex128)
    b.hmc_trajectory(noise, 1, dt, p.mass)
    with pytest.raises(dwhmc.DwhError):
        b.hmc_sweep(noise, np.array([0.5]), 1, dt, p.mass)
    b.hmc_finish([False])
    with pytest.raises(dwhmc.DwhError):
        b.hmc_finish([True])
    a.close()
    b.close()


def test_cr_bp128_matches_dense_L64(dwhmc, oracle):
    """L = 64 (BP = 128 lattice-row blocks, k_cr_inv<8>): the CR path against the
    dense Schur-complement path of the same context parameters (both through
    the C ABI; the eigen oracle at n = 8192 is too slow for a unit test; the
    small-Ly BP = 128 lattices are checked against the oracle in
    test_cr_ragged_chains)."""
    O = oracle
    p, dis, Delta = make_case(O, 64, 64, 8.0, seed=64)
    res = {}
    for algo in ("cr", "dense"):
        ctx = device_ctx(dwhmc, p, dis, algo)
        assert ctx.info["block"] == (128 if algo == "cr" else 64)
        ctx.set_pairing(Delta)
        ctx.factorize()
        res[algo] = (ctx.forces()[0], ctx.fermion_energy()[0], ctx.pairing()[0], ctx.hole_trace()[0])
        ctx.close()
    Fc, Ec, Pc, Tc = res["cr"]
    Fd, Ed, Pd, Td = res["dense"]
    assert np.max(np.abs(Fc - Fd)) <= 1e-10 * (1 + np.max(np.abs(Fd)))
    assert np.max(np.abs(Pc - Pd)) <= 1e-11
    assert abs(Ec - Ed) <= 1e-11 * abs(Ed)
    assert abs(Tc - Td) <= 1e-11 * p.N


def test_c1_workload_matches_oracle(dwhmc, oracle, algo):
    """BASELINE configs[0] (C1): L = 8, β = 4, W = 1, n_imp = 0.05, 10
    trajectories of Nt = 10 from initialize_state's Δ₀ — the workload of the
    (stale) scripts/test_hmc.jl:26-29 — device vs oracle sweep by sweep with
    the same injected draws (dt = calc_optimal_dt(β, J, m, 10))."""
    O = oracle
    p = O.ModelParameters(8, 8, T, TP, MU, 1.0, 0.05, 4.0, J, 1.0)
    st = O.initialize_state(p, np.random.default_rng(1000))
    ctx = device_ctx(dwhmc, p, st.disorder_pot, algo)
    ctx.set_pairing(st.Delta)
    ctx.factorize()
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, st.disorder_pot)
    O.update_H_BdG(cache, p, st.Delta)
    O.diagonalize_H_BdG(cache, p)
    ref = O.SimulationState(st.disorder_pot, st.Delta.copy(), np.zeros_like(st.Delta))
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, 10)
    rng = np.random.default_rng(11)
    for s in range(10):
        noise = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
        u = rng.random()
        acc, dH = ctx.hmc_sweep(noise, np.array([u]), 10, dt, p.mass)
        acc_r, dH_r = O.hmc_sweep(cache, p, ref, 10, dt, noise, u)
        assert acc[0] == acc_r and abs(dH[0] - dH_r) <= 1e-8 * (1 + abs(dH_r)), (s, dH[0], dH_r)
    D, _ = ctx.get_state()
    assert np.max(np.abs(D[0] - ref.Delta)) <= 1e-10
    ctx.close()


@pytest.mark.parametrize("L,beta", [(10, 1000.0), (12, 5000.0), (10, 10000.0)])
def test_low_temperature_matches_oracle(dwhmc, oracle, L, beta, algo3):
    """The reference's production β range: scripts/batch_scan_T.jl:21-24 goes to
    T = 1e-4 (β = 10⁴), scripts/benchmark_beta_scan.jl:37-40 to β = 5000.
    The pole table reaches κ = 262144 (β·E'/2; 31-43 pole pairs here), so
    auto selects the CR path; the pole GJ path and the eigendecomposition path
    (algo eig) must meet the same tolerances as everywhere else."""
    O = oracle
    p, dis, Delta = make_case(O, L, L, beta, seed=L + int(beta))
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    if algo3 == "cr":
        assert device_ctx(dwhmc, p, dis).info["algo"] == 1   # auto: CR inside the table
    ctx = device_ctx(dwhmc, p, dis, algo3)
    assert (ctx.info["npoles"] == 0) == (algo3 == "eig")
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    Ef = ctx.fermion_energy()[0]
    assert abs(Ef - Ef_ref) <= 1e-11 * abs(Ef_ref), (Ef, Ef_ref)
    hole_ref = O.measure_observables(cache, p, Delta)["hole_conc"]
    assert abs(2.0 * ctx.hole_trace()[0] / p.N - 1.0 - hole_ref) <= 1e-11
    ctx.close()


@pytest.mark.parametrize("Lx,Ly,beta", [(32, 32, 1000.0), (24, 24, 10000.0), (64, 4, 1000.0), (48, 6, 5000.0),
                                        (13, 9, 20000.0)])
def test_low_temperature_large_lattice_cr(dwhmc, oracle, Lx, Ly, beta):
    """The CR path at the extended table's κ (29-43 pole pairs) on the C3
    lattice, a 24 x 24 one and the BP = 128 / 96 / 32 block sizes: the longest
    CR chains at the worst-conditioned resolvents (cond ≈ βE'/π), same
    tolerances."""
    O = oracle
    p, dis, Delta = make_case(O, Lx, Ly, beta, seed=7 * Lx + Ly + int(beta))
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, "cr")
    assert ctx.info["npoles"] >= 20
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(ctx.fermion_energy()[0] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    hole_ref = O.measure_observables(cache, p, Delta)["hole_conc"]
    assert abs(2.0 * ctx.hole_trace()[0] / p.N - 1.0 - hole_ref) <= 1e-11
    ctx.close()


def test_clean_closed_form_beta5000(dwhmc, oracle, algo3):
    """I5 (scripts/benchmark_clean.jl:15-43) at β = 5000 on 12 x 12, every
    algorithm (the degenerate clean spectrum is the hard case for the eigen
    path, the large κ for the pole paths)."""
    O = oracle
    L, beta, D0 = 12, 5000.0, 0.25
    p = O.ModelParameters(L, L, T, TP, MU, 0.0, 0.0, beta, J, 1.0)
    Delta = np.stack([np.full(p.N, D0), np.full(p.N, -D0)], axis=1).astype(np.complex128)
    _, Px, Fx, Ef = O.clean_dwave_closed_form(D0, L, L, T, TP, MU, beta, J)
    ctx = device_ctx(dwhmc, p, np.zeros(p.N), algo3)
    ctx.set_pairing(Delta)
    ctx.factorize()
    P = ctx.pairing()[0]
    F = ctx.forces()[0]
    assert np.max(np.abs(P[:, 0] - Px)) <= 1e-11
    assert np.max(np.abs(P[:, 1] + Px)) <= 1e-11
    assert np.max(np.abs(F[:, 0] - Fx)) <= 1e-10 * (1 + abs(Fx))
    assert abs(ctx.fermion_energy()[0] - Ef) <= 1e-11 * abs(Ef)
    ctx.close()


@pytest.mark.parametrize("algo_lt", ["cr", "eig"])
def test_low_temperature_sweeps_match_oracle(dwhmc, oracle, algo_lt):
    """hmc_sweep! at β = 1000 (T = 1e-3, scripts/batch_scan_T.jl:21-24) through
    the CR path (κ inside the extended table) and the eigendecomposition path,
    two chains batched, against the oracle."""
    O = oracle
    cases = [make_case(O, 6, 6, 1000.0, seed=s, amp=0.1) for s in (61, 62)]
    p = cases[0][0]
    Nt = 5
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
    rng = np.random.default_rng(21)
    draws = [((rng.standard_normal((2, p.N, 2)) + 1j * rng.standard_normal((2, p.N, 2))) * math.sqrt(0.5),
              rng.random(2)) for _ in range(3)]
    refs = [_oracle_after_sweeps(O, pc, dc, Dc, [(n[c], float(u[c])) for n, u in draws], Nt, dt)
            for c, (pc, dc, Dc) in enumerate(cases)]
    ctx = device_ctx(dwhmc, p, np.stack([c[1] for c in cases]), algo_lt)
    ctx.set_pairing(np.stack([c[2] for c in cases]))
    ctx.factorize()
    for s, (noise, u) in enumerate(draws):
        acc, dH = ctx.hmc_sweep(noise, u, Nt, dt, p.mass)
        D, _ = ctx.get_state()
        for c in range(2):
            acc_r, dH_r, D_r, _ = refs[c][s]
            assert bool(acc[c]) == acc_r
            assert abs(dH[c] - dH_r) <= 1e-8 * (1 + abs(dH_r)), (s, c, dH[c], dH_r)
            assert np.max(np.abs(D[c] - D_r)) <= 1e-10
    ctx.close()


def test_guard_falls_back_to_eig_beyond_table(dwhmc, oracle):
    """β = 40000 fits the pole table at the default cap (κ <= 2.3e5 of
    262144); an uploaded Δ whose re-selected cap would need κ beyond the table
    moves the context to the eigendecomposition path instead of failing."""
    O = oracle
    p, dis, Delta = make_case(O, 8, 8, 40000.0, seed=300)
    Delta = Delta * (3.0 / np.max(np.abs(Delta)))
    ctx = device_ctx(dwhmc, p, dis)
    assert ctx.info["algo"] in (0, 1)
    ctx.set_pairing(Delta)
    assert ctx.info["algo"] == 2
    ctx.factorize()
    _, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(ctx.fermion_energy()[0] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    ctx.close()


@pytest.mark.parametrize("sparse0", ["1", "0"])
@pytest.mark.parametrize("Lx,Ly,beta", [(16, 16, 8.0), (12, 10, 8.0), (20, 4, 16.0), (40, 6, 16.0), (8, 8, 4.0),
                                        (9, 12, 8.0), (32, 32, 16.0)])
def test_cr_sparse_level0(dwhmc, oracle, monkeypatch, Lx, Ly, beta, sparse0):
    """Level 0 by the sparse stages (k_cr_sp_fwd / k_cr_sp_bwd: every product
    with a level-0 U / L block on the vector units, one-term dense products for
    G_ae, G_ce, G_ea, G_ec, T = -Dinv M and G_ee = Dinv - T Dinv;
    tools/cr_model.py cr_selected_inverse_top_sparse0) or the dense level 0
    (DWHMC_CR_SPARSE0=0), against the eigen oracle: P, F, E_f, hole density
    and two HMC sweeps.  BP = 32 (Lx = 12, 16, 9, and 8 x 8 as two-row
    blocks: 4 blocks), 64 (20, 32) and 96 (40); Ly = 4 is the smallest level 0
    the sparse stages take."""
    O = oracle
    monkeypatch.setenv("DWHMC_CR_SPARSE0", sparse0)
    p, dis, Delta = make_case(O, Lx, Ly, beta, seed=Lx * 17 + Ly)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    assert abs(ctx.fermion_energy()[0] - Ef_ref) <= 1e-11 * abs(Ef_ref)
    hole_ref = O.measure_observables(cache, p, Delta)["hole_conc"]
    assert abs(2.0 * ctx.hole_trace()[0] / p.N - 1.0 - hole_ref) <= 1e-11
    if p.N <= 400:
        Nt = 3
        dt = O.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
        rng = np.random.default_rng(9)
        draws = [((rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5),
                  float(rng.random())) for _ in range(2)]
        ref = _oracle_after_sweeps(O, p, dis, Delta, draws, Nt, dt)
        for (noise, u), (acc_r, dH_r, D_r, _) in zip(draws, ref):
            acc, dH = ctx.hmc_sweep(noise, np.array([u]), Nt, dt, p.mass)
            assert bool(acc[0]) == acc_r and abs(dH[0] - dH_r) <= 1e-8 * (1 + abs(dH_r))
            assert np.max(np.abs(ctx.get_state()[0][0] - D_r)) <= 1e-10
    ctx.close()


@pytest.mark.parametrize("merge", ["0", "4", "8"])
@pytest.mark.parametrize("Lx,Ly,beta", [(20, 16, 8.0), (12, 16, 8.0), (20, 12, 16.0), (9, 24, 4.0)])
def test_cr_backward_merge(dwhmc, oracle, monkeypatch, merge, Lx, Ly, beta):
    """The backward merge (round 6, build_cr_plan): a coarse level's G_ee stage
    inside the next finer level's first stage, whose products read G_ee
    through its expansion (forward products as side work of the final
    inversion at BP = 64, inside the top level's D' stage at BP = 32).
    DWHMC_CR_MERGE = 0 / 4 / 8 (levels up to that size) against the eigen
    oracle at the factorisation tolerances, on BP = 64 (Lx = 20) and BP = 32
    (Lx = 12, 9) lattices with even and odd coarse levels (Ly = 16, 12, 24)."""
    O = oracle
    monkeypatch.setenv("DWHMC_CR_MERGE", merge)
    p, dis, Delta = make_case(O, Lx, Ly, beta, seed=Lx * 11 + Ly)
    cache, F_ref, Ef_ref = O.evaluate(p, dis, Delta)
    P_ref, _ = O.pairing_P(cache.U, cache.E_n, p)
    ctx = device_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    ctx.factorize()
    assert np.max(np.abs(ctx.pairing()[0] - P_ref)) <= 1e-11
    assert np.max(np.abs(ctx.forces()[0] - F_ref)) <= 1e-10 * (1 + np.max(np.abs(F_ref)))
    Ef = ctx.fermion_energy()[0]
    assert abs(Ef - Ef_ref) <= 1e-11 * abs(Ef_ref), (Ef, Ef_ref)
    hole_ref = O.measure_observables(cache, p, Delta)["hole_conc"]
    assert abs(2.0 * ctx.hole_trace()[0] / p.N - 1.0 - hole_ref) <= 1e-11
    ctx.close()
