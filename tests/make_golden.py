#!/usr/bin/env python3
"""Write tests/golden/oracle_*.npz: small regression vectors from the CPU
oracle (the reference itself cannot run here: no Julia in the image).
Contents: lattice tables, the upper-triangle H_BdG exactly as
src/Hamiltonian.jl builds it, spectrum, forces, E_f, and one injected-draw
HMC sweep (dH, Δ after).  Regenerate only when the oracle changes."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import dwhmc_oracle as O  # noqa: E402


def main():
    for L, beta in ((4, 8.0), (8, 16.0)):
        p = O.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.05, beta, 0.8, 1.0)
        rng = np.random.default_rng(2024 + L)
        st = O.initialize_state(p, rng)
        Delta = st.Delta + 0.3 * np.stack([np.ones(p.N), -np.ones(p.N)], 1)
        cache, F, Ef = O.evaluate(p, st.disorder_pot, Delta)
        noise = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * math.sqrt(0.5)
        u = float(rng.random())
        Nt = 5
        dt = O.calc_optimal_dt(beta, p.J, p.mass, Nt)
        s2 = O.SimulationState(st.disorder_pot, Delta.copy(), np.zeros_like(Delta))
        acc, dH = O.hmc_sweep(cache, p, s2, Nt, dt, noise, u)
        cache0, _, _ = O.evaluate(p, st.disorder_pot, Delta)
        np.savez_compressed(
            os.path.join(ROOT, "tests", "golden", f"oracle_L{L}.npz"),
            beta=beta, nn=p.nn_table, nnn=p.nnn_table, disorder=st.disorder_pot, Delta=Delta,
            H_upper=cache0.H_base, E=np.sort(cache0.E_n), F=F, Ef=Ef,
            sweep_noise=noise, sweep_uniform=u, sweep_Nt=Nt, sweep_dt=dt,
            sweep_accepted=acc, sweep_dH=dH, sweep_Delta=s2.Delta, sweep_pi=s2.pi)
        print(L, beta, "Ef", Ef, "dH", dH, "acc", acc)


if __name__ == "__main__":
    main()
