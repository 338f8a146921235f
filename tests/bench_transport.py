"""Time the transport / spectra measurement (measure_transport_and_spectra,
src/Observables.jl:314-526) on the device vs the CPU restatement.

Device: dwh_measure_transport on a BASELINE-size lattice (default C3: 32x32,
β = 16, default η / Δω / ω_max -> 1996 ω points, 4001 DOS points), one warmup
call, then K timed calls (each call is synchronous: eigenpairs, J_mn, all
sums, copies back).  dwh_eigensystem without vectors (eigenvalues only: the
structure-preserving reduction, csrc/dwhmc_qeig.hip) is timed the same way.

CPU: the oracle (numpy + LAPACK, all host threads BLAS uses) on the same
lattice: eigh + J_mn + everything except σ(ω) in full, σ(ω) on a bounded
sample of ω points scaled to the full grid (the sample is stated in the
output).  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU restatement")
    ap.add_argument("--cpu-omega", type=int, default=40, help="ω points of the CPU σ sample")
    ap.add_argument("--chains", type=int, default=4, help="chains of the batched measurement")
    ap.add_argument("--snapshots", default="4,8", help="Δ-snapshot batch sizes (dwh_measure_transport_deltas)")
    a = ap.parse_args()

    import dwhmc_loader
    m = dwhmc_loader.load_package()
    L = a.L
    p = m.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.1, a.beta, 0.8, 1.0)
    rng = np.random.default_rng(7)
    st = m.initialize_state(p, rng)
    N = p.N
    D = st.Delta + 0.25 * np.stack([np.ones(N), -np.ones(N)], 1)
    lib = os.environ.get("DWHMC_LIB")   # another build of the library (A/B)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                           st.disorder_pot, lib_path=lib)
    ctx.set_pairing(D)
    ctx.measure_transport(p.eta, p.domega, p.omega_max)          # warmup (allocations, handle)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = ctx.measure_transport(p.eta, p.domega, p.omega_max)
    t_meas = (time.perf_counter() - t0) / a.steps
    # eigenvalues only: the structure-preserving reduction (dwhmc_qeig.hip)
    ctx.eigensystem(0, vectors=False)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.eigensystem(0, vectors=False)
    t_eig = (time.perf_counter() - t0) / a.steps
    # Δ snapshots of one chain in one call (run_simulation(transport_batch=K))
    snaps = {}
    for K in [int(x) for x in a.snapshots.split(",") if x]:
        Ds = np.stack([D + 0.01 * k * rng.standard_normal((N, 2)) for k in range(K)])
        ctx.measure_transport_deltas(Ds, p.eta, p.domega, p.omega_max)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.measure_transport_deltas(Ds, p.eta, p.domega, p.omega_max)
        t = (time.perf_counter() - t0) / a.steps
        snaps[str(K)] = {"ms_per_call": 1e3 * t, "ms_per_measurement": 1e3 * t / K}
    ctx.close()
    # batched: --chains chains in one context, dwh_measure_transport_batched
    nc = a.chains
    ctxb = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                            np.stack([st.disorder_pot] * nc), lib_path=lib)
    ctxb.set_pairing(np.stack([D] * nc))
    ctxb.measure_transport_all(p.eta, p.domega, p.omega_max)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctxb.measure_transport_all(p.eta, p.domega, p.omega_max)
    t_batch = (time.perf_counter() - t0) / a.steps
    ctxb.close()
    nw, nd = len(r["omega_grid"]), len(r["dos_omega_grid"])
    n2 = 2 * N
    out = {
        "metric": "transport_measurements_per_s", "value": 1.0 / t_meas, "unit": "measurements/s",
        "ms_per_measurement": 1e3 * t_meas, "ms_eigenvalues_only": 1e3 * t_eig,
        "config": {"workload": f"measure_transport_and_spectra {L}x{L} beta={a.beta}", "n2": n2,
                   "n_omega": nw, "n_dos": nd},
        "sigma_pair_terms": n2 * n2 * nw,
        "batched": {"chains": nc, "ms_per_call": 1e3 * t_batch, "ms_per_chain": 1e3 * t_batch / nc},
        "snapshots": snaps,
    }
    if a.cpu:
        from oracle import dwhmc_oracle as O
        po = O.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.1, a.beta, 0.8, 1.0)
        t0 = time.perf_counter()
        cache, _, _ = O.evaluate(po, st.disorder_pot, D)
        t_eig_cpu = time.perf_counter() - t0
        # everything but σ: run with a 1-point ω grid
        po1 = O.ModelParameters(L, L, 1.0, -0.35, -1.08, 1.0, 0.1, a.beta, 0.8, 1.0,
                                omega_max=po.eta)
        t0 = time.perf_counter()
        O.measure_transport_and_spectra(cache, po1)
        t_rest = time.perf_counter() - t0
        # σ sample: a.cpu_omega points
        E, f = cache.E_n, cache.fermi_factors
        Jmn = cache.U.conj().T @ np.vstack([O.current_operator(po) @ cache.U[:N],
                                            O.current_operator(po) @ cache.U[N:]])
        dE = (E[None, :] - E[:, None]).ravel()
        df = (f[:, None] - f[None, :])
        coef = np.where(np.abs(df) >= 1e-12, df * np.abs(Jmn) ** 2, 0.0).ravel()
        om = O.julia_range(po.eta, po.domega, po.omega_max)[:: max(1, nw // a.cpu_omega)][: a.cpu_omega]
        t0 = time.perf_counter()
        for w in om:
            np.sum(coef / w * O.lorentzian(w - dE, po.eta))
        t_sig = (time.perf_counter() - t0) / len(om) * nw
        t_cpu = t_eig_cpu + t_rest + t_sig
        out["cpu_baseline"] = {"value": 1.0 / t_cpu, "unit": "measurements/s", "cores": os.cpu_count(),
                               "kind": "port",
                               "sample": f"eigh + J_mn + stiffness/dc/DOS/A(k) in full ({t_eig_cpu + t_rest:.1f} s); "
                                         f"sigma on {len(om)} of {nw} omega points scaled ({t_sig:.1f} s)"}
        out["cpu_ms_per_measurement"] = 1e3 * t_cpu
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
