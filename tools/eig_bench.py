"""Time the eigendecomposition leapfrog step (algo eig) per lattice size:
one dwh_factorize = assemble + zheevd (+ NaN scan) + zgemm + gather + force.
Usage: python tools/eig_bench.py [L ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dwhmc_loader  # noqa: E402

dw = dwhmc_loader.load_package()
Ls = [int(a) for a in sys.argv[1:]] or [8, 16, 32]
for L in Ls:
    p = dw.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.05, 1000.0, 0.8, 1.0)
    rng = np.random.default_rng(L)
    N = L * L
    dis = rng.uniform(-0.5, 0.5, N)
    D = 0.3 * np.stack([np.ones(N), -np.ones(N)], 1) * np.exp(0.2j * rng.standard_normal((N, 1)))
    ctx = dw.FermionContext(L, L, 1.0, -0.35, -1.08, 1000.0, 0.8, p.nn_table, p.nnn_table, dis, algo="eig")
    ctx.set_pairing(D)
    ctx.factorize()
    reps = 5 if L <= 32 else 2
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.factorize()
    dt = (time.perf_counter() - t0) / reps
    print(f"eig L={L} N={N} n2={2 * N}: {dt * 1e3:.2f} ms per step ({1 / dt:.1f} steps/s)", flush=True)
    ctx.close()
