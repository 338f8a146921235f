#!/usr/bin/env python3
"""Interleaved in-process A/B of context variants (env knobs read at create):
python tools/ab_bench.py --L 32 --beta 16 --variants "CR_INV0=1" "CR_INV0=0"
KEY=VAL sets the context knob DWHMC_KEY; LIB=path loads another build of the library
(hybrid-monte-carlo-for-d-wave-sc_amd/build.py --out build/var/x.so -D ...) so
kernel variants are compared in one process.  Prints ms per leapfrog step
(median / min over rounds) and the per-kernel event totals of the last round."""
import argparse
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--beta", type=float, default=16.0)
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("--Nt", type=int, default=10)
    ap.add_argument("--sweeps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", nargs="+", default=["CR_INV0=1", "CR_INV0=0"])
    a = ap.parse_args()
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    p = m.ModelParameters(a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    dis, D0 = [], []
    for c in range(a.chains):
        st = m.initialize_state(p, np.random.default_rng(1000 + c))
        dis.append(st.disorder_pot)
        D0.append(st.Delta)
    rng = np.random.default_rng(7)
    shape = (a.sweeps, a.chains, p.N, 2)
    noise = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)) * math.sqrt(0.5)
    uni = rng.random((a.sweeps, a.chains))
    dt = m.calc_optimal_dt(p.beta, p.J, p.mass, a.Nt)
    ctxs = {}
    touched = set()
    for v in a.variants:
        kv = dict(x.split("=") for x in v.split(",") if x)
        for k in touched:                       # knobs of the previous variant do not leak
            os.environ.pop(k, None)
        # any other KEY=VAL of the variant sets the context knob DWHMC_KEY
        for k, val in kv.items():
            if k != "LIB":
                os.environ["DWHMC_" + k] = val
                touched.add("DWHMC_" + k)
        ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                               np.stack(dis), lib_path=kv.get("LIB"))
        ctx.set_pairing(np.stack(D0))
        ctx.factorize()
        ctx.load_draws(noise, uni)
        ctxs[v] = ctx
    res = {v: [] for v in a.variants}
    for r in range(a.rounds + 1):
        for v, ctx in ctxs.items():
            ctx.set_pairing(np.stack(D0))
            ctx.factorize()
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.run_sweeps(0, a.sweeps, a.Nt, dt, p.mass)
            ctx.synchronize()
            el = time.perf_counter() - t0
            if r > 0:
                res[v].append(1000 * el / (a.sweeps * a.Nt))
    print(f"L={a.L} beta={a.beta} chains={a.chains} poles={next(iter(ctxs.values())).info['npoles']}")
    for v, ctx in ctxs.items():
        ctx.timing_enable(True)
        ctx.timing_reset()
        ctx.run_sweeps(0, 1, a.Nt, dt, p.mass)
        ctx.synchronize()
        keys = ("cr_gemm", "cr_inv", "cr_inv_side", "cr_sparse", "step") if ctx.info.get("algorithm", "cr") != "dense" else \
            ("gj_update", "gj_pivot", "assemble", "contract", "step")
        kt = {k: ctx.timing_read(k) for k in keys}
        ctx.timing_enable(False)
        x = np.array(res[v])
        main = kt[keys[0]]
        tf = main[2] / main[0] / 1e9 if main[0] > 0 else float("nan")
        print(f"{v:24s} ms/step median {np.median(x):.4f} min {x.min():.4f}  steps/s {1000*a.chains/np.median(x):.1f}  "
              f"{keys[0]} {tf:.1f} TF  " +
              " ".join(f"{k}={val[0]/a.Nt:.4f}ms/{val[1]//a.Nt}" for k, val in kt.items()), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
