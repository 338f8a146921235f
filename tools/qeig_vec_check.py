#!/usr/bin/env python3
"""GPU check of the structure-preserving eigensystem (eigen_solve ->
q_heev_enqueue, csrc/dwhmc_qeig.hip + the one-stage back-transform) against
the one-stage solver (DWHMC_EIG_QUAT=0) and LAPACK: eigenvalues, residual
||H U - U E|| / ||H||, orthonormality ||U^H U - I||, and the device time of
eigensystem() with and without vectors.  Usage: python tools/qeig_vec_check.py [L ...]"""
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
    Ls = [int(x) for x in sys.argv[1:]] or [4, 6, 8, 12, 16]
    for L in Ls:
        for clean in (False, True):
            p = O.ModelParameters(L, L, 1.0, -0.35, 0.0 if clean else -1.08, 0.0 if clean else 1.0, 0.1, 16.0, 0.8, 1.0)
            N = p.N
            rng = np.random.default_rng(L)
            st = O.initialize_state(p, rng)
            if clean:
                D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(complex)
                dis = np.zeros(N)
            else:
                D = st.Delta + 0.25 * np.exp(0.3j * rng.standard_normal((N, 2)))
                dis = st.disorder_pot
            cache = O.initialize_cache(p)
            O.init_static_H(cache, p, dis)
            O.update_H_BdG(cache, p, D)
            H = O.hermitian_from_upper(cache.H_base)
            ev = np.linalg.eigvalsh(H)
            hn = np.max(np.abs(ev))
            ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis,
                                   lib_path=os.environ.get("DWHMC_LIB"))
            ctx.set_pairing(D)
            out = []
            for q in ("1", "0"):
                os.environ["DWHMC_EIG_QUAT"] = q
                E, U = ctx.eigensystem(0)
                ctx.synchronize()
                t0 = time.perf_counter()
                E, U = ctx.eigensystem(0)
                t = time.perf_counter() - t0
                res = np.max(np.abs(H @ U - U * E[None, :])) / (1 + hn)
                orth = np.max(np.abs(U.conj().T @ U - np.eye(2 * N)))
                err = np.max(np.abs(E - ev)) / (1 + hn)
                out.append(f"{'quat' if q == '1' else 'one-stage'}: E err {err:.1e} res {res:.1e} orth {orth:.1e} "
                           f"{1e3 * t:7.2f} ms")
            os.environ.pop("DWHMC_EIG_QUAT", None)
            ctx.close()
            print(f"L={L:3d} clean={clean!s:5s} n={2 * N:5d}  " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
