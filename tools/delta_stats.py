#!/usr/bin/env python3
"""Pairing-field extremes along a thermalised chain (GPU): max |Δ_ij| and the
max row sum Σ_j |Δ_ij|/2 of the pairing block, per sweep, for choosing the
spectral guard's default cap.  Usage:
python tools/delta_stats.py --L 32 --beta 16 --sweeps 400"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--beta", type=float, default=16.0)
    ap.add_argument("--sweeps", type=int, default=400)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import bench
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    p = m.ModelParameters(a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    dis, D0 = bench.synthetic_state(m, p, a.seed, 1)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis)
    ctx.set_pairing(D0)
    ctx.factorize()
    Nt, _ = bench.thermalise(m, ctx, p, a.seed, 1, 100, 10)
    dt = m.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
    noise, uni = bench.synthetic_draws(m, p.N, a.seed, 1, a.sweeps, 13)
    ctx.load_draws(noise, uni)
    nn = p.nn_table - 1   # 0-based, N x 4 (+x, +y, -x, -y)
    mx, rs = [], []
    for s in range(a.sweeps):
        ctx.run_sweeps(s, 1, Nt, dt, p.mass)
        D = ctx.get_state()[0][0]          # N x 2: bonds (i, i+x), (i, i+y)
        ab = np.abs(D)
        row = ab[:, 0] + ab[:, 1] + ab[nn[:, 2], 0] + ab[nn[:, 3], 1]   # 4 bonds of site i
        mx.append(ab.max())
        rs.append(0.5 * row.max())
    acc, _ = ctx.sweep_results(0, a.sweeps)
    info = ctx.info
    print(f"L={a.L} beta={a.beta} Nt={Nt} sweeps={a.sweeps} acceptance={acc.mean():.3f} cap={info['delta_cap']:.3f} "
          f"kappa={info['kappa']:.1f} poles={info['npoles']}")
    print(f"max|Delta|: mean {np.mean(mx):.3f} max {np.max(mx):.3f}; max row sum |Delta|/2: mean {np.mean(rs):.3f} "
          f"max {np.max(rs):.3f}; mean |Delta| {np.mean(np.abs(D)):.3f}")


if __name__ == "__main__":
    main()
