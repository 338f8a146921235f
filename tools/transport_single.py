"""K single-chain transport measurements at L x L (the bench_transport
workload, m = 1) for profiling: python tools/transport_single.py [L] [K] [S].
S > 0: K calls of measure_transport_deltas over S Δ snapshots instead."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    p = m.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.1, 16.0, 0.8, 1.0)
    st = m.initialize_state(p, np.random.default_rng(7))
    D = st.Delta + 0.25 * np.stack([np.ones(p.N), -np.ones(p.N)], 1)
    # DWHMC_LIB: another build of the library (A/B, e.g. an earlier round's)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, st.disorder_pot,
                           lib_path=os.environ.get("DWHMC_LIB"))
    ctx.set_pairing(D)
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if S > 0:
        rng = np.random.default_rng(11)
        Ds = np.stack([D + 0.01 * k * rng.standard_normal((p.N, 2)) for k in range(S)])
        ctx.measure_transport_deltas(Ds, p.eta, p.domega, p.omega_max)
        t0 = time.perf_counter()
        for _ in range(K):
            ctx.measure_transport_deltas(Ds, p.eta, p.domega, p.omega_max)
        dt = (time.perf_counter() - t0) / K
        print(f"L={L} {S} snapshots: {1e3 * dt:.2f} ms per call, {1e3 * dt / S:.2f} ms per measurement", flush=True)
        ctx.close()
        return
    ctx.measure_transport(p.eta, p.domega, p.omega_max)
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.measure_transport(p.eta, p.domega, p.omega_max)
    print(f"L={L} {1e3 * (time.perf_counter() - t0) / K:.2f} ms per measurement ({K} + 1 warmup)", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
