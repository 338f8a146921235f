"""The reference's own end-to-end physics checks, run through the GPU path.

* scripts/benchmark_clean.jl:49-119: clean 10x10 lattice at beta = 180, HMC
  (50 thermalisation sweeps at Nt = 20, 100 measurement sweeps at Nt = 5),
  then <|Delta_global|> must satisfy the BCS gap equation of
  calc_BCS_RHS (benchmark_clean.jl:15-43) to |<D> - RHS(<D>)| < 0.02 — the
  reference's pass criterion (:116).
  Measured on MI355X: <|Delta_global|> = 0.3534, RHS = 0.3584.
* HMC exactness: <exp(-dH)> = 1 over equilibrium trajectories (SURVEY.md §8c
  pin 6), checked to 4 standard errors.

Draws come from numpy (the reference's Julia RNG cannot be reproduced), so
these are statistical pins, not bitwise ones.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def calc_BCS_RHS(D, Lx, Ly, t, tp, mu, beta, J):
    """scripts/benchmark_clean.jl:15-43."""
    nx, ny = np.meshgrid(np.arange(Lx), np.arange(Ly), indexing="xy")
    kx, ky = 2 * np.pi * nx / Lx, 2 * np.pi * ny / Ly
    eps = -2 * t * (np.cos(kx) + np.cos(ky)) - 4 * tp * np.cos(kx) * np.cos(ky) - mu
    g = np.cos(kx) - np.cos(ky)
    E = np.sqrt(eps ** 2 + np.abs(D * g) ** 2)
    return J / (Lx * Ly) * np.sum(g ** 2 / (2 * E) * np.tanh(0.5 * beta * E)) * D


def test_benchmark_clean_gap_equation(dwhmc):
    m = dwhmc
    Lx = Ly = 10
    t, tp, mu, beta, J, mass = 1.0, -0.35, -1.08, 180.0, 1.6, 1.0
    p = m.ModelParameters(Lx, Ly, t, tp, mu, 0.0, 0.0, beta, J, mass)
    rng = np.random.default_rng(2024)
    st = m.initialize_state(p, rng)
    st.Delta[:, 0] = 0.2          # benchmark_clean.jl:77-80: uniform d-wave start
    st.Delta[:, 1] = -0.2
    cache = m.initialize_cache(p)
    m.init_static_H(cache, p, st)
    m.update_H_BdG(cache, p, st)
    m.diagonalize_H_BdG(cache, p)
    dt = m.calc_optimal_dt(beta, J, mass, 20)
    for _ in range(50):
        m.hmc_sweep(cache, p, st, Nt=20, dt=dt, rng=rng)
    dt = m.calc_optimal_dt(beta, J, mass, 5)
    hist = []
    for _ in range(100):
        m.hmc_sweep(cache, p, st, Nt=5, dt=dt, rng=rng)
        hist.append(m.measure_observables(cache, p, st).Delta_global)
    cache.ctx.close()
    Dm = float(np.mean(hist))
    rhs = calc_BCS_RHS(Dm, Lx, Ly, t, tp, mu, beta, J)
    print(f"<|Delta_global|> = {Dm:.6f} +/- {np.std(hist):.6f}, BCS RHS = {rhs:.6f}")
    assert Dm > 0.01, Dm                       # an ordered d-wave state
    assert abs(Dm - rhs) < 0.02, (Dm, rhs)     # benchmark_clean.jl:116


def test_exp_minus_dH_averages_to_one(dwhmc):
    """<e^{-dH}> = 1 (area preservation + reversibility of the leapfrog for
    the action the force is the exact gradient of), on a disordered 8x8
    lattice after thermalisation at calc_optimal_dt(Nt = 10) (acceptance
    ~0.97 there; measured <e^-dH> = 1.0000)."""
    m = dwhmc
    p = m.ModelParameters(8, 8, 1.0, -0.35, -1.08, 1.0, 0.1, 8.0, 0.8, 1.0)
    rng = np.random.default_rng(7)
    st = m.initialize_state(p, rng)
    cache = m.initialize_cache(p)
    m.init_static_H(cache, p, st)
    m.update_H_BdG(cache, p, st)
    m.diagonalize_H_BdG(cache, p)
    dt = m.calc_optimal_dt(p.beta, p.J, p.mass, 10)
    for _ in range(40):
        m.hmc_sweep(cache, p, st, Nt=10, dt=dt, rng=rng)
    w = []
    for _ in range(400):
        _, dH = m.hmc_sweep(cache, p, st, Nt=10, dt=dt, rng=rng)
        w.append(math.exp(-dH))
    cache.ctx.close()
    w = np.asarray(w)
    print(f"<exp(-dH)> = {w.mean():.4f}  acceptance ~ {np.mean(np.minimum(w, 1.0)):.3f}")
    # batch means over 20 blocks against autocorrelation
    b = w.reshape(20, -1).mean(axis=1)
    se = b.std(ddof=1) / math.sqrt(len(b))
    assert abs(w.mean() - 1.0) <= 4 * se + 1e-3, (w.mean(), se)
