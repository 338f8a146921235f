#!/usr/bin/env python3
"""GPU check of the structure-preserving eigensolver on clean lattices
(W = 0, uniform d-wave, mu = -1: exactly degenerate shells, k_q_orth):
which solver ran, residual, orthonormality and where its largest error sits
(indices, eigenvalues, whether the pair shares a cluster or is a Theta pair).
Usage: python tools/qeig_cluster_check.py [L ...]"""
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
    mu = float(os.environ.get("QCL_MU", "-1"))   # 0: the nodal zero modes (L % 4 == 0)
    Ls = [int(x) for x in sys.argv[1:]] or [10, 12, 16]
    for L in Ls:
        p = O.ModelParameters(L, L, 1.0, -0.35, mu, 0.0, 0.0, 16.0, 0.8, 1.0)
        N = p.N
        D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(complex)
        dis = np.zeros(N)
        cache = O.initialize_cache(p)
        O.init_static_H(cache, p, dis)
        O.update_H_BdG(cache, p, D)
        H = O.hermitian_from_upper(cache.H_base)
        ev = np.linalg.eigvalsh(H)
        hn = np.max(np.abs(ev))
        ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis)
        ctx.set_pairing(D)
        ctx.timing_enable(["eig_own", "eig_vendor"])
        E, U = ctx.eigensystem(0)
        own, vendor = ctx.timing_read("eig_own")[1], ctx.timing_read("eig_vendor")[1]
        quat = ctx.info["eig_quat"]
        ts = []
        for q in ("1", "0"):   # device time of one eigensystem, structure-preserving vs one-stage
            os.environ["DWHMC_EIG_QUAT"] = q
            ctx.eigensystem(0)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.eigensystem(0)
            ts.append(1e3 * (time.perf_counter() - t0))
        os.environ.pop("DWHMC_EIG_QUAT", None)
        ctx.close()
        res = np.max(np.abs(H @ U - U * E[None, :])) / (1 + hn)
        G = np.abs(U.conj().T @ U - np.eye(2 * N))
        i, j = np.unravel_index(np.argmax(G), G.shape)
        rows = np.max(G, axis=1)
        worst = np.argsort(rows)[::-1][:8]
        print(f"L={L} mu={mu} n={2 * N} own={own} vendor={vendor} quat={quat} res {res:.1e} orth {G.max():.1e} "
              f"at ({i},{j}) E {E[i]:.6f} {E[j]:.6f}; E err {np.max(np.abs(E - ev)) / (1 + hn):.1e}; "
              f"eigensystem {ts[0]:.2f} ms (one-stage {ts[1]:.2f} ms)", flush=True)
        print("  worst columns:", [(int(c), round(float(E[c]), 6), f"{rows[c]:.1e}") for c in worst], flush=True)
        # the largest error per block: upper-upper, upper-lower (Theta), same cluster
        up = slice(N, 2 * N)
        lo = slice(0, N)
        print(f"  upper-upper {G[up, up].max():.1e} upper-lower {G[up, lo].max():.1e} "
              f"lower-lower {G[lo, lo].max():.1e}", flush=True)


if __name__ == "__main__":
    main()
