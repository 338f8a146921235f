#!/usr/bin/env python3
"""The reference's T scan (scripts/batch_scan_T.jl) on the HIP path, for the
parity pin against the reference's own published outputs
(tests/golden/ref_Tscan_L24.json, extracted from scripts/plot_stiffness.ipynb
by tools/ref_notebook_golden.py).

Model of the published data set (plot_stiffness.ipynb cell 1): L = 24,
J = 0.8, W = 1.0, n_imp = 0.0, μ = -1.4; the rest from batch_scan_T.jl:11-36
(t = 1, t' = -0.35, mass = 1, η = 8/L², Δω = 0.2 η, ω_max = 4, n_therm = 20,
n_measure = 100, Nt_therm_init = 20, Nt_measure = 6, transport every sweep,
bin_size = 10; T grid 10^range(-4, 3, 24)).  Assumption stated, not
recorded by the notebook: the published run used these settings of the
script with only (μ, n_imp) edited.  Its R column is consistent with them:
every 1e8 / R is an integer to display precision, i.e. a mean of 100 values
printed with %.6f (tests/test_ref_tscan.py::test_fixture_consistent_with_100_measurements).

Each T point runs K independent chains (each one a complete run_simulation of
the reference, src/Simulation.jl:34-236, with its own seed), written in the
reference's CSV formats and reduced the way batch_csv_summary_T.jl:23-62 does
(mean, std/sqrt(n) over the measurement rows).  Every chain is an independent
replica of the published single run, so the spread over chains (and each
chain's binned error) sets the statistical tolerance of the comparison.

Usage (GPU box): python tools/ref_tscan.py --rows 15 16 22 --chains 4 --out gpurun_out/tscan
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIXTURE = os.path.join(ROOT, "tests", "golden", "ref_Tscan_L24.json")
SCAN = dict(n_therm=20, n_measure=100, Nt_therm_init=20, Nt_measure=6, measure_transport_freq=1, bin_size=10)


def t_grid():
    """scripts/batch_scan_T.jl:21-24: 24 log-spaced T from 1e-4 to 1e3."""
    return 10.0 ** np.linspace(math.log10(1e-4), math.log10(1000.0), 24)


def row_T(row: int) -> float:
    """Summary row -> simulated T.  The published summary has rows 0..22 =
    grid points 1..23 (the T = 1e-4 point is absent from it)."""
    return float(t_grid()[row + 1])


def sig3(T: float) -> float:
    """round(T, sigdigits=3) of the run directory name (batch_scan_T.jl:64),
    which batch_csv_summary_T.jl:100-104 parses back as the summary's T."""
    return float(f"{T:.3g}")


def read_csv(path):
    """CSV with a header row -> (names, data) (readdlm(path, ',', header=true))."""
    with open(path) as f:
        names = f.readline().strip().split(",")
        data = np.array([[float(x) for x in line.strip().split(",")] for line in f if line.strip()])
    return names, data.reshape(-1, len(names))


def process_csv(path):
    """batch_csv_summary_T.jl:23-68: drop the Sweep column, per column mean and
    std/sqrt(n) (Statistics.std: n - 1 normalisation).  -> {name: (mean, err)}"""
    names, data = read_csv(path)
    keep = [i for i, n in enumerate(names) if n.lower() != "sweep"]
    d = data[:, keep]
    n = d.shape[0]
    mean = d.mean(axis=0)
    err = d.std(axis=0, ddof=1) / math.sqrt(n) if n >= 2 else np.zeros(len(keep))
    return {names[i]: (float(mean[j]), float(err[j])) for j, i in enumerate(keep)}


def binned_se(x, nbins: int = 10) -> float:
    """Standard error of the mean of an autocorrelated series from nbins
    consecutive bins (the sweeps of one chain are Markov-correlated)."""
    x = np.asarray(x, dtype=np.float64)
    m = len(x) // nbins
    b = x[: m * nbins].reshape(nbins, m).mean(axis=1)
    return float(b.std(ddof=1) / math.sqrt(nbins))


def chain_stats(d):
    """Per chain: the summary means (process_csv) and binned errors of the
    columns the notebook uses."""
    obs = process_csv(os.path.join(d, "observables.csv"))
    tr = process_csv(os.path.join(d, "transport.csv"))
    _, od = read_csv(os.path.join(d, "observables.csv"))
    names_o = read_csv(os.path.join(d, "observables.csv"))[0]
    names_t, td = read_csv(os.path.join(d, "transport.csv"))
    col = lambda names, data, n: data[:, names.index(n)]
    return {
        "DC_Conductivity": (tr["DC_Conductivity"][0], binned_se(col(names_t, td, "DC_Conductivity"))),
        "Superfluid_Stiffness": (tr["Superfluid_Stiffness"][0], binned_se(col(names_t, td, "Superfluid_Stiffness"))),
        "Delta_Loc": (obs["Delta_Loc"][0], binned_se(col(names_o, od, "Delta_Loc"))),
        "Delta_LocalPair": (obs["Delta_LocalPair"][0], binned_se(col(names_o, od, "Delta_LocalPair"))),
        "Accepted": (obs["Accepted"][0], binned_se(col(names_o, od, "Accepted"))),
    }


class _ExtraEtaContext:
    """FermionContext wrapper for the investigation runs: every transport
    measurement is repeated at the broadenings eta * mult (the Markov chain
    does not depend on η), the extra DC conductivities collected per chain."""

    base = None
    mults: tuple = ()
    extra: list = []

    def __init__(self, *a, **kw):
        self._ctx = _ExtraEtaContext.base(*a, **kw)

    def __getattr__(self, name):
        return getattr(self._ctx, name)

    def measure_transport_all(self, eta, domega, omega_max):
        out = self._ctx.measure_transport_all(eta, domega, omega_max)
        row = []
        for mlt in _ExtraEtaContext.mults:
            r = self._ctx.measure_transport_all(eta * mlt, domega, omega_max)
            row.append([x["dc_conductivity"] for x in r])
        _ExtraEtaContext.extra.append(row)
        return out


def run_point(m, fixture, row: int, chains: int, out_root: str, seed: int = 2024, device: int = 0, scan=None,
              eta_mults=(), eta_mult: float = 1.0):
    """K chains of the published run at summary row `row`; returns the per-chain
    statistics and the wall time.  eta_mult scales η = 8/L² (batch_scan_T.jl:17
    `* 1.0`); eta_mults: extra broadenings measured on the same chains
    (investigation runs)."""
    scan = dict(SCAN if scan is None else scan)
    md = fixture["model"]
    L = int(md["L"])
    T = row_T(row)
    eta = 8.0 / (L * L) * eta_mult
    p = m.ModelParameters(L, L, 1.0, -0.35, md["mu"], md["W"], md["n_imp"], 1.0 / T, md["J"], 1.0,
                          eta=eta, domega=0.2 * eta, omega_max=4.0)
    dirs = [os.path.join(out_root, f"T_{sig3(T)}", f"chain{k}") for k in range(chains)]
    rngs = [np.random.default_rng([seed, row, k]) for k in range(chains)]
    import importlib
    H = importlib.import_module(m.__name__ + ".hmc")
    saved = H.FermionContext
    if eta_mults:
        _ExtraEtaContext.base, _ExtraEtaContext.mults, _ExtraEtaContext.extra = saved, tuple(eta_mults), []
        H.FermionContext = _ExtraEtaContext
    t0 = time.time()
    try:
        res = m.run_simulation_chains(p, dirs, rngs, device=device, **scan)
    finally:
        H.FermionContext = saved
    el = time.time() - t0
    out = {"row": row, "T": T, "T_summary": sig3(T), "beta": 1.0 / T, "seconds": el, "eta": eta,
           "chains": [chain_stats(d) for d in dirs],
           "Nt_final": [r.Nt_final for r in res],
           "meas_acceptance": [r.meas_acceptance for r in res]}
    if eta_mults:
        # (measurements, mults, chains) -> per mult, per chain: the %.6f values' mean
        # (the transport.csv format) and binned error
        x = np.round(np.array(_ExtraEtaContext.extra), 6)
        out["extra_eta"] = {str(mlt): [(float(x[:, j, k].mean()), binned_se(x[:, j, k])) for k in range(chains)]
                            for j, mlt in enumerate(eta_mults)}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", required=True)
    ap.add_argument("--chains", type=int, default=4)
    ap.add_argument("--out", default="gpurun_out/tscan")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--n-measure", type=int, default=None)
    ap.add_argument("--eta-mult", type=float, default=1.0, help="η = 8/L² x this (batch_scan_T.jl:17)")
    ap.add_argument("--extra-eta-mults", type=float, nargs="*", default=[],
                    help="also measure the DC conductivity at η x these on the same chains")
    a = ap.parse_args(argv)
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    m.load_library(build_if_missing=False)
    with open(FIXTURE) as f:
        fx = json.load(f)
    scan = dict(SCAN)
    if a.n_measure:
        scan["n_measure"] = a.n_measure
    os.makedirs(a.out, exist_ok=True)
    allres = []
    for r in a.rows:
        res = run_point(m, fx, r, a.chains, a.out, a.seed, scan=scan, eta_mults=a.extra_eta_mults,
                        eta_mult=a.eta_mult)
        allres.append(res)
        dc = [c["DC_Conductivity"][0] for c in res["chains"]]
        Rref = fx["R_rows"].get(str(r))
        line = {"row": r, "T": res["T"], "s": round(res["seconds"], 2),
                "R_chains": [1 / x if x else None for x in dc], "R_ref": Rref}
        for k, v in res.get("extra_eta", {}).items():
            line[f"R_eta_x{k}"] = [1 / x[0] if x[0] else None for x in v]
        print(json.dumps(line), flush=True)
        with open(os.path.join(a.out, "summary.json"), "w") as f:
            json.dump(allres, f, indent=1)


if __name__ == "__main__":
    main()
