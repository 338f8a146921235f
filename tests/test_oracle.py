"""Pin the CPU oracle (oracle/dwhmc_oracle.py) before trusting it.

The reference ships no golden vectors, so the oracle is pinned
by closed forms and identities that the reference's own scripts rely on:
  * scripts/benchmark_clean.jl:15-43     clean d-wave BCS closed form (I5)
  * scripts/test_forces.jl:31-55          mean-field fixed point drives F -> 0
  * scripts/bench_forces.jl:124-129       force invariant to loop order (≤1e-10)
  * SURVEY.md §8a I1-I4                  spectrum symmetry, E_f as a determinant,
                                         F = -∂H/∂Δ* (Wirtinger), ρ-block symmetry
  * src/HMC.jl leapfrog                   reversibility, O(dt²) energy error
plus the committed golden fixture (tests/golden/oracle_L4.npz, made by
tests/make_golden.py) as a regression vector.
"""
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T, TP, MU, J = 1.0, -0.35, -1.08, 0.8


def params(O, L, beta, W=1.0, nimp=0.05, Ly=None, mu=MU, tp=TP, Jc=J):
    return O.ModelParameters(L, Ly or L, T, tp, mu, W, nimp, beta, Jc, 1.0)


def random_case(O, L, beta, seed, amp=0.3, **kw):
    p = params(O, L, beta, **kw)
    rng = np.random.default_rng(seed)
    st = O.initialize_state(p, rng)
    D = st.Delta + amp * np.stack([np.ones(p.N), -np.ones(p.N)], 1) * (1 + 0.2 * rng.standard_normal((p.N, 1)))
    return p, st.disorder_pot, D


@pytest.mark.parametrize("L", [4, 6, 8])
@pytest.mark.parametrize("beta", [4.0, 16.0, 180.0])
def test_clean_dwave_closed_form(oracle, L, beta):
    """I5: uniform d-wave, W=0 — eigen oracle vs the 2x2 k-space solution."""
    O = oracle
    D0 = 0.2
    p = params(O, L, beta, W=0.0, nimp=0.0)
    Delta = np.stack([np.full(p.N, D0), np.full(p.N, -D0)], 1).astype(complex)
    cache, F, Ef = O.evaluate(p, np.zeros(p.N), Delta)
    spec, Px, Fx, Ef_cf = O.clean_dwave_closed_form(D0, L, L, T, TP, MU, beta, J)
    assert np.max(np.abs(np.sort(cache.E_n) - spec)) < 1e-12
    P, _ = O.pairing_P(cache.U, cache.E_n, p)
    assert np.max(np.abs(P[:, 0] - Px)) < 1e-12
    assert np.max(np.abs(P[:, 1] + Px)) < 1e-12
    assert np.max(np.abs(F[:, 0] - Fx)) < 1e-10
    assert abs(Ef - Ef_cf) < 1e-12 * abs(Ef_cf)
    # scripts/benchmark_clean.jl: Δ_pair = J (P_x - P_y)/2 equals calc_BCS_RHS(Δ0)
    obs = O.measure_observables(cache, p, Delta)
    assert abs(obs["Delta_pair"] - O.bcs_rhs(D0, L, L, T, TP, MU, beta, J)) < 1e-12


def test_identities_I1_I2_I4(oracle):
    O = oracle
    p, dis, D = random_case(O, 6, 8.0, seed=3)
    cache, F, Ef = O.evaluate(p, dis, D)
    E = cache.E_n
    # I1: ± pairs and tr H = 0
    assert np.max(np.abs(np.sort(E) + np.sort(E)[::-1])) < 1e-12
    Hf = O.hermitian_from_upper(cache.H_base)
    assert abs(np.trace(Hf)) < 1e-12
    # I2: E_f = -Σ ln(1+e^{-βE}) = -ln det(2cosh(βH/2))
    assert abs(Ef + np.sum(O.log1pexp(-p.beta * E))) < 1e-9
    assert abs(Ef + np.sum(np.logaddexp(p.beta * E / 2, -p.beta * E / 2))) < 1e-9
    # I4: ρ_{i,j+N} = ρ_{j,i+N}; Tr ρ_pp + Tr ρ_hh = N; hole_conc = 2Tr ρ_hh/N - 1
    f = O.logistic(-p.beta * E)
    rho = (cache.U * f) @ cache.U.conj().T
    N = p.N
    assert np.max(np.abs(rho[:N, N:] - rho[:N, N:].T)) < 1e-12
    assert abs(np.trace(rho[:N, :N]).real + np.trace(rho[N:, N:]).real - N) < 1e-10
    hole = O.measure_observables(cache, p, D)["hole_conc"]
    assert abs(hole - (2 * np.trace(rho[N:, N:]).real / N - 1)) < 1e-12


def test_I3_force_is_wirtinger_gradient(oracle):
    """F = -∂(E_boson + E_f)/∂Δ* by central finite differences (doc/algorithm.md:58)."""
    O = oracle
    p, dis, D = random_case(O, 4, 6.0, seed=5)
    _, F, _ = O.evaluate(p, dis, D)

    def action(Dx):
        _, _, Ef = O.evaluate(p, dis, Dx)
        return p.beta / (2 * p.J) * np.sum(np.abs(Dx) ** 2) + Ef

    h = 1e-5
    for (i, d) in [(0, 0), (5, 1), (11, 0)]:
        e = np.zeros_like(D)
        e[i, d] = h
        dre = (action(D + e) - action(D - e)) / (2 * h)
        dim = (action(D + 1j * e) - action(D - 1j * e)) / (2 * h)
        grad_conj = 0.5 * (dre + 1j * dim)        # ∂/∂Δ*
        assert abs(F[i, d] + grad_conj) < 1e-6 * (1 + abs(F[i, d]))


def test_loop_order_invariance(oracle):
    """scripts/bench_forces.jl:124-129: vectorised vs literal loop order ≤ 1e-10."""
    O = oracle
    p, dis, D = random_case(O, 4, 8.0, seed=8)
    cache, F, _ = O.evaluate(p, dis, D)
    F_loop = O.compute_forces_loops(cache.U, cache.E_n, D, p)
    assert np.max(np.abs(F - F_loop)) < 1e-10


def test_mean_field_iteration_drives_force_to_zero(oracle):
    """scripts/test_forces.jl:31-55 (4x4, β=20, J=1, t'=-0.35, μ=-0.5, W=0):
    Δ <- Δ + (2J/β) F ; the force norm must decrease towards 0."""
    O = oracle
    p = O.ModelParameters(4, 4, 1.0, -0.35, -0.5, 0.0, 0.0, 20.0, 1.0, 1.0)
    rng = np.random.default_rng(0)
    st = O.initialize_state(p, rng)
    D = st.Delta.copy()
    norms = []
    for _ in range(50):
        _, F, _ = O.evaluate(p, np.zeros(p.N), D)
        norms.append(np.linalg.norm(F))
        D = D + (2 * p.J / p.beta) * F
    assert norms[-1] < 1e-3 * norms[0]
    assert norms[-1] < 1e-4


def test_leapfrog_reversibility_and_dt2(oracle):
    O = oracle
    p, dis, D0 = random_case(O, 4, 4.0, seed=2, amp=0.1)
    rng = np.random.default_rng(1)
    noise = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
    dHs = []
    for Nt in (8, 16):
        dt = 0.4 / Nt
        cache = O.initialize_cache(p)
        O.init_static_H(cache, p, dis)
        st = O.SimulationState(dis, D0.copy(), np.zeros_like(D0))
        O.update_H_BdG(cache, p, st.Delta)
        O.diagonalize_H_BdG(cache, p)
        _, dH = O.hmc_sweep(cache, p, st, Nt, dt, noise, 0.0)
        dHs.append(abs(dH))
        if Nt == 16:
            # reverse: flip π and integrate back (π refreshed from the flipped value)
            back = O.SimulationState(dis, st.Delta.copy(), np.zeros_like(D0))
            c2 = O.initialize_cache(p)
            O.init_static_H(c2, p, dis)
            O.update_H_BdG(c2, p, back.Delta)
            O.diagonalize_H_BdG(c2, p)
            O.hmc_sweep(c2, p, back, Nt, dt, -st.pi / math.sqrt(2 * p.mass), 0.0)
            assert np.max(np.abs(back.Delta - D0)) < 1e-11
    ratio = dHs[0] / dHs[1]
    assert 2.5 < ratio < 6.0, ratio     # ~4 for O(dt²)


def test_golden_fixture_regression(oracle):
    path = os.path.join(ROOT, "tests", "golden", "oracle_L4.npz")
    g = np.load(path, allow_pickle=False)
    O = oracle
    p = O.ModelParameters(4, 4, T, TP, MU, 1.0, 0.05, float(g["beta"]), J, 1.0)
    cache, F, Ef = O.evaluate(p, g["disorder"], g["Delta"])
    assert np.array_equal(p.nn_table, g["nn"]) and np.array_equal(p.nnn_table, g["nnn"])
    assert np.array_equal(cache.H_base, g["H_upper"])
    assert np.max(np.abs(np.sort(cache.E_n) - g["E"])) < 1e-12
    assert np.max(np.abs(F - g["F"])) < 1e-12
    assert abs(Ef - float(g["Ef"])) < 1e-12 * abs(float(g["Ef"]))
