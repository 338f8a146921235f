"""Debug: eig path on the clean d-wave lattice (degenerate spectrum)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dwhmc_loader
from oracle import dwhmc_oracle as O
dw = dwhmc_loader.load_package()
T, TP, MU, J = 1.0, -0.35, -1.08, 0.8
for L, beta in ((8, 16.0), (12, 5000.0)):
    p = O.ModelParameters(L, L, T, TP, MU, 0.0, 0.0, beta, J, 1.0)
    D0 = 0.25
    Delta = np.stack([np.full(p.N, D0), np.full(p.N, -D0)], axis=1).astype(np.complex128)
    _, Px, Fx, Ef = O.clean_dwave_closed_form(D0, L, L, T, TP, MU, beta, J)
    ctx = dw.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                            np.zeros(p.N), algo="eig")
    ctx.set_pairing(Delta)
    E, U = ctx.eigensystem(0)
    print(L, beta, "E nan", np.isnan(E).sum(), "U nan", np.isnan(U).sum(),
          "orth", np.max(np.abs(U.conj().T @ U - np.eye(2 * p.N))) if not np.isnan(U).any() else None, flush=True)
    ctx.factorize()
    P = ctx.pairing()[0]
    print("  P nan", np.isnan(P).sum(), "err", np.nanmax(np.abs(P[:, 0] - Px)), "Ef", ctx.fermion_energy()[0], Ef,
          flush=True)
    ctx.close()
