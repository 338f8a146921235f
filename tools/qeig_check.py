#!/usr/bin/env python3
"""GPU check of the structure-preserving eigensolver (dwh_debug_qeig,
csrc/dwhmc_qeig.hip) against LAPACK eigvalsh of the same H_BdG, and the
reduction's device time against the one-stage solver's whole eigensystem
(dwh_eigensystem).  Usage: python tools/qeig_check.py [L ...]"""
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
    from importlib import import_module
    lib = import_module(m.__name__ + "._lib")
    Ls = [int(x) for x in sys.argv[1:]] or [4, 6, 8, 16, 32]
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
            ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis)
            ctx.set_pairing(D)
            E = np.empty(2 * N)
            ms = np.zeros(1)
            for _ in range(2):
                lib.check(ctx._lib.dwh_debug_qeig(ctx._h, 0, lib.ptr(E), lib.ptr(ms)), "qeig")
            err = np.max(np.abs(E - ev)) / (1 + np.max(np.abs(ev)))
            ctx.synchronize()
            t0 = time.perf_counter()
            E1, _ = ctx.eigensystem(0, vectors=True)
            t1 = time.perf_counter() - t0
            ctx.close()
            print(f"L={L:3d} clean={clean!s:5s} n={2 * N:5d}  qeig eig err {err:.2e}  reduction {ms[0]:8.3f} ms  "
                  f"one-stage eigensystem {1e3 * t1:8.2f} ms (err {np.max(np.abs(E1 - ev)) / (1 + np.max(np.abs(ev))):.1e})",
                  flush=True)


if __name__ == "__main__":
    main()
