"""Test infrastructure (CPU oracle): σ_DC of the reference's formula
(src/Observables.jl:404-425) at high temperature for i.i.d. Gaussian pairing
fields, where the fermion weight is negligible (E_f ≈ -2N ln 2 + O(β²)) and
the HMC ensemble is Gaussian with <|Δ_ij|²> = 2J/β, at several broadenings
η, plus the share of the diagonal (n = m) terms.  Pins the oracle to the
reference's published R(T = 1000) and backs the η inference of
tests/test_ref_tscan.py (tests/test_ref_tscan_oracle.py,
profiles/r03_ref_tscan_investigation.md).

Usage: python tests/ref_tscan_oracle_sigma.py [T] [samples]   (~0.5 s per sample)
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dwhmc_oracle as O  # noqa: E402

MULTS = (1.0, 1.1, 1.2, 1.25, 1.3)


def current_operator(p):
    """J_x ⊕ J_x (src/Observables.jl:237-283), dense."""
    N = p.N
    Jp = np.zeros((N, N), complex)
    for i in range(N):
        for j, t in ((p.nn_table[i, 0] - 1, p.t), (p.nnn_table[i, 0] - 1, p.tp), (p.nnn_table[i, 3] - 1, p.tp)):
            Jp[i, j] += 1j * t
            Jp[j, i] += np.conj(1j * t)
    Z = np.zeros((N, N))
    return np.block([[Jp, Z], [Z, Jp]])


def sigma_samples(T=1000.0, ns=40, L=24, J=0.8, mu=-1.4, mults=MULTS, seed=None):
    """σ_DC per sample (ns x len(mults)) at η = mult · 8/L² (batch_scan_T.jl:17)
    and the diagonal share of each sample at η = 8/L², for the published
    model (plot_stiffness.ipynb cell 1: W = 1, n_imp = 0)."""
    beta = 1.0 / T
    eta0 = 8.0 / (L * L)
    p = O.ModelParameters(L, L, 1.0, -0.35, mu, 1.0, 0.0, beta, J, 1.0, eta=eta0, domega=0.2 * eta0, omega_max=4.0)
    Jb = current_operator(p)
    rng = np.random.default_rng(int(T * 10) + 3 if seed is None else seed)
    sig, diag = [], []
    for _ in range(ns):
        D = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(J / beta)
        cache = O.initialize_cache(p)
        O.init_static_H(cache, p, np.zeros(p.N))
        O.update_H_BdG(cache, p, D)
        O.diagonalize_H_BdG(cache, p)
        E, U = cache.E_n, cache.U
        Jmn = U.conj().T @ Jb @ U
        f = 1.0 / (1.0 + np.exp(beta * E))
        A = (beta * f * (1 - f))[:, None] * np.abs(Jmn) ** 2
        dE = E[None, :] - E[:, None]
        row = []
        for m in mults:
            eta = eta0 * m
            terms = A * (eta / math.pi) / (dE ** 2 + eta ** 2)
            row.append(terms.sum() * math.pi / p.N)
            if m == 1.0:
                diag.append(np.trace(terms) / terms.sum())
        sig.append(row)
    return np.array(sig), np.array(diag)


def main(T=1000.0, ns=40):
    a, diag = sigma_samples(T, ns)
    for k, m in enumerate(MULTS):
        se = a[:, k].std(ddof=1) / math.sqrt(ns)
        print(f"T={T:g} eta={m:g} x 8/L^2: sigma_DC {a[:, k].mean():.4e} +- {se:.1e}  R {1 / a[:, k].mean():.1f}")
    print(f"diagonal (n = m) share of sigma_DC at eta = 8/L^2: {np.mean(diag):.3f}")


if __name__ == "__main__":
    main(*(float(x) for x in sys.argv[1:2]), *(int(x) for x in sys.argv[2:3]))
