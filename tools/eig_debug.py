"""One own-solver eigendecomposition of a disordered H_BdG at L x L with the
per-phase timing of DWHMC_EIG_DEBUG=1 (stderr), then the eigenvalue symmetry and
orthogonality (numpy).  Usage: python tools/eig_debug.py L [chains]."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    L = int(sys.argv[1])
    os.environ.setdefault("DWHMC_EIG_DEBUG", "1")
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    p = m.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.1, 32.0, 0.8, 1.0)
    st = m.initialize_state(p, np.random.default_rng(L))
    D = st.Delta + 0.25 * np.stack([np.ones(p.N), -np.ones(p.N)], 1)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, st.disorder_pot)
    ctx.set_pairing(D)
    t0 = time.perf_counter()
    E, U = ctx.eigensystem(0)
    print(f"L={L} n={2 * p.N} eigensystem {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    orth = np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N)))
    print(f"L={L} max|E|={np.max(np.abs(E)):.3f} |E+E[::-1]|={np.max(np.abs(E + E[::-1])):.2e} orth={orth:.2e}",
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
