#!/usr/bin/env python3
"""First-call cost of the measurement (fresh context: allocation, the
reduction graph's capture and instantiation) against later calls, L = 32,
with and without the reduction graph (DWHMC_Q_GRAPH).  Usage: python tools/q_first_call.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import dwhmc_loader
    from oracle import dwhmc_oracle as O
    m = dwhmc_loader.load_package()
    p = O.ModelParameters(32, 32, 1.0, -0.35, -1.08, 1.0, 0.1, 16.0, 0.8, 1.0)
    rng = np.random.default_rng(32)
    st = O.initialize_state(p, rng)
    D = st.Delta + 0.25 * np.exp(0.3j * rng.standard_normal((p.N, 2)))
    for g in ("1", "0", "1", "0"):
        os.environ["DWHMC_Q_GRAPH"] = g
        ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, st.disorder_pot)
        ctx.set_pairing(D)
        ts = []
        for _ in range(4):
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.measure_transport(p.eta, p.domega, p.omega_max)
            ts.append(1e3 * (time.perf_counter() - t0))
        ctx.close()
        print(f"DWHMC_Q_GRAPH={g}: calls " + " ".join(f"{t:.1f}" for t in ts) + " ms", flush=True)


if __name__ == "__main__":
    main()
