"""Parity pin against the reference's own published outputs: the T scan of
scripts/plot_stiffness.ipynb (stored outputs of a real run of the Julia
reference; extracted into tests/golden/ref_Tscan_L24.json by
tools/ref_notebook_golden.py, which reads the notebook as data).

CPU: the fixture itself and the reduction restated from
scripts/batch_csv_summary_T.jl:23-62.  GPU: the scan re-run on the HIP path
(tools/ref_tscan.py: run_simulation_chains, i.e. src/Simulation.jl:34-236
per chain) against the published numbers, with tolerances derived from the
runs' own statistical errors (see the GPU test's docstring)."""
import json
import math
import os

import numpy as np
import pytest

from tools import ref_tscan as S

FX = json.load(open(S.FIXTURE))


def test_fixture_rows_are_the_script_grid():
    """The summary's T column = round(T, sigdigits=3) of batch_scan_T.jl:21-24's
    grid (the directory names, :64), rows 0..22 = grid points 1..23; Beta =
    1/T of the rounded value (batch_csv_summary_T.jl:100-104)."""
    for r, T in FX["T_rows"].items():
        assert S.sig3(S.row_T(int(r))) == pytest.approx(T, rel=1e-12), r
    for r, b in FX["beta_rows"].items():
        assert abs(b - 1.0 / FX["T_rows"][r]) <= 6e-7, r      # printed with 6 decimals


def test_fixture_consistent_with_100_measurements():
    """R = 1/mean(DC_Conductivity) over transport.csv, whose values are printed
    with %.6f (src/Simulation.jl:174): with n_measure = 100 and transport every
    sweep (batch_scan_T.jl:31,35) the mean is k·1e-8 for an integer k.  Every
    published R whose 7 displayed digits resolve k satisfies that — the
    measurement count and format the GPU run reproduces."""
    ks = []
    for r, R in FX["R_rows"].items():
        if R is None:
            continue
        k = 1e8 / R
        resolution = k * 5e-7 * 1.01          # 7 significant digits of R
        if resolution >= 0.25:
            continue
        assert abs(k - round(k)) <= resolution, (r, R, k)
        ks.append((k, resolution))
    assert len(ks) >= 6
    # other measurement counts n (mean = integer · 1e-6 / n) do not fit every row
    for n in (50, 80, 90, 99, 101, 110, 120, 150):
        assert not all(abs(k * n / 100 - round(k * n / 100)) <= res * n / 100 for k, res in ks), n


def test_process_csv_restates_summary_reduction(tmp_path):
    """batch_csv_summary_T.jl:23-62: Sweep dropped, mean and std/sqrt(n) with
    Statistics.std's n - 1 normalisation."""
    p = tmp_path / "transport.csv"
    rows = [(1, 0.5, 0.000091), (2, 0.25, 0.000073), (3, 0.0, 0.000119)]
    p.write_text("Sweep,Superfluid_Stiffness,DC_Conductivity\n" +
                 "".join("%d,%.6f,%.6f\n" % r for r in rows))
    out = S.process_csv(str(p))
    assert set(out) == {"Superfluid_Stiffness", "DC_Conductivity"}
    dc = np.array([r[2] for r in rows])
    assert out["DC_Conductivity"][0] == pytest.approx(dc.mean(), rel=1e-15)
    assert out["DC_Conductivity"][1] == pytest.approx(dc.std(ddof=1) / math.sqrt(3), rel=1e-12)


def loglog_fit(T, y):
    """np.polyfit(log T, log y, 1) of plot_stiffness.ipynb cells 3 and 5."""
    slope, icpt = np.polyfit(np.log(T), np.log(y), 1)
    return float(slope), float(icpt)


# ---------------------------------------------------------------------------
# GPU: the published scan re-run on the HIP path
# ---------------------------------------------------------------------------
ROWS_FIT = [16, 17, 18, 19, 20, 21, 22]          # T > 10 (cells 3 and 5)
ROWS_R_LOW = [7, 8, 9, 10, 11, 12, 13, 14, 15]  # 0.027 <= T < 10 (cell 8)
# the low-temperature rows (cell 8): β = 301, 149, 74 — the largest pole sets
# of the scan (κ ≈ 1500, 730, 360: 23, 20, 18 pole pairs) and the worst-conditioned
# no-pivot resolvents of the scan, across the resistive upturn (R = 0.51 ->
# 20.8 -> 182149); 8 chains each (profiles/r04_ref_tscan_lowT.md)
ROWS_R_COLD = [4, 5, 6]
CHAINS = 4
CHAINS_COLD = 8
Z = 4.0
# η of the published run.  The CPU oracle alone fixes it from the reference's
# own T = 1000 point (tests/test_ref_tscan_oracle.py: R = 12368.6 is matched at
# η = 10/L² and excludes the 8/L² that batch_scan_T.jl:17 sets today, where
# σ_DC is ~93 % diagonal (n = m) terms ∝ 1/η).  At that η the HIP path is then
# checked against the whole published curve here — a consistency check of
# the path at the run's broadening, not a fit: the Markov chains do not depend
# on η (measurement only), and with 8/L² the same chains miss the published
# R by 10-19 % at T >= 30 (profiles/r03_ref_tscan_investigation.md; R(T)
# against 8/L² stays parity-unpinned, the published run's η being inferred).
ETA_MULT = 1.25


def _stat_tol(vals, ses, quantum):
    """Statistical tolerance for comparing the published single run with the
    mean of K independent replicas of it: the single-run standard error is
    the larger of the replicas' pooled binned error and their spread; the
    difference of one run and the K-run mean has variance SE²(1 + 1/K).
    `quantum`: the rounding of the published number."""
    vals = np.asarray(vals)
    K = len(vals)
    se_run = max(math.sqrt(float(np.mean(np.square(ses)))), float(np.std(vals, ddof=1)))
    return Z * se_run * math.sqrt(1.0 + 1.0 / K) + quantum


@pytest.fixture(scope="module")
def scan(dwhmc, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("tscan"))
    res = {}
    for r in ROWS_FIT + ROWS_R_LOW + ROWS_R_COLD:
        res[r] = S.run_point(dwhmc, FX, r, CHAINS_COLD if r in ROWS_R_COLD else CHAINS, out, seed=2024,
                             eta_mult=ETA_MULT)
    rec = os.environ.get("DWHMC_TSCAN_RECORD")
    if rec:
        with open(rec, "w") as f:
            json.dump({str(k): v for k, v in res.items()}, f, indent=1)
    return res


@pytest.mark.gpu
def test_published_dc_resistance(scan):
    """R(T) = 1/⟨σ_DC⟩ (plot_stiffness.ipynb cell 8) at T >= 0.0033 (rows 4 ..
    22 of the summary) with η = 10/L² (ETA_MULT), compared as σ_DC with the
    statistical tolerance of _stat_tol (Z = 4, binned errors over 10 bins of
    10 measurements per chain, K = 4 chains; K = 8 at the cold rows 4-6) plus
    the rounding allowance: 5e-7 (the %.6f format of each measurement) at the
    rows of round 3, 1e-8 (the resolution of a mean of 100 such values) at the
    cold rows, where σ_DC is down to 5.5e-6."""
    bad = []
    for r, res in sorted(scan.items()):
        R_ref = FX["R_rows"][str(r)]
        vals = [c["DC_Conductivity"][0] for c in res["chains"]]
        ses = [c["DC_Conductivity"][1] for c in res["chains"]]
        tol = _stat_tol(vals, ses, 1e-8 if r in ROWS_R_COLD else 5e-7)
        diff = float(np.mean(vals)) - 1.0 / R_ref
        if abs(diff) > tol:
            bad.append((r, res["T"], 1.0 / float(np.mean(vals)), R_ref, diff, tol))
    assert not bad, bad


def _fit_check(scan, num, den, published):
    T = np.array([scan[r]["T_summary"] for r in ROWS_FIT])
    fits = []
    for k in range(CHAINS):
        y = np.array([scan[r]["chains"][k][num][0] for r in ROWS_FIT])
        if den:
            y = y / np.array([scan[r]["chains"][k][den][0] for r in ROWS_FIT])
        fits.append(loglog_fit(T, y))
    fits = np.array(fits)
    # the chain-averaged scan (what a single longer run would give)
    ybar = np.array([np.mean([c[num][0] for c in scan[r]["chains"]]) for r in ROWS_FIT])
    if den:
        ybar = ybar / np.array([np.mean([c[den][0] for c in scan[r]["chains"]]) for r in ROWS_FIT])
    s, c = loglog_fit(T, ybar)
    # per-chain fits are independent replicas of the published fit: their
    # spread is the published fit's statistical error
    tol_s = _stat_tol(fits[:, 0], np.zeros(CHAINS), 5e-5)
    tol_c = _stat_tol(fits[:, 1], np.zeros(CHAINS), 5e-5)
    assert abs(s - published["slope"]) <= tol_s, (s, published, tol_s, fits)
    assert abs(c - published["intercept"]) <= tol_c, (c, published, tol_c, fits)


@pytest.mark.gpu
def test_published_delta_loc_fit(scan):
    """Cell 5: log Δ_Loc vs log T over T > 10, slope 0.4994, intercept -0.2286."""
    _fit_check(scan, "Delta_Loc", None, FX["fit_Delta_Loc_T_gt_10"])


@pytest.mark.gpu
def test_published_local_pair_ratio_fit(scan):
    """Cell 3: log(Δ_LocalPair/Δ_Loc) vs log T over T > 10, slope -0.9959,
    intercept -1.6350 (the fermionic pair response P from the pole-expanded
    factorisation against the reference's eigenvector sums)."""
    _fit_check(scan, "Delta_LocalPair", "Delta_Loc", FX["fit_LocalPair_over_Loc_T_gt_10"])
