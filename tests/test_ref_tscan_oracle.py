"""The CPU oracle pinned to a published output of the reference itself:
R(T = 1000) = 12368.6 of scripts/plot_stiffness.ipynb cell 8 (summary row 22,
tests/golden/ref_Tscan_L24.json), and the broadening that run used.

At T = 1000 (β = 0.001) the fermion weight is negligible, so the HMC ensemble
of the reference's run is Gaussian with <|Δ_ij|²> = 2J/β, and σ_DC is the
ensemble mean of the reference's Kubo formula (src/Observables.jl:404-425) —
which the oracle restates — over i.i.d. Gaussian Δ
(tests/ref_tscan_oracle_sigma.py).  No GPU and no free parameter beyond η:
 * at η = 10/L² (batch_scan_T.jl:17's `* 1.0` factor at 1.25) the oracle's
   σ_DC equals the published 1/R within the combined statistical error;
 * at η = 8/L² (the script as committed) it is excluded: σ_DC there is
   ~93 % diagonal (n = m) terms ∝ 1/η.
This makes the η inference behind tests/test_ref_tscan.py a checked claim
(DESIGN.md §5).  Statistical error of the published number: its run's 100
measurements (test_ref_tscan.py::test_fixture_consistent_with_100_measurements)
of σ_DC, each with the per-sample spread measured here, with an allowance of
τ_int = 2 for correlation between sweeps: SE_pub = std · sqrt(2 / 100)."""
import json
import math
import os

import numpy as np
import pytest

import ref_tscan_oracle_sigma as S

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_Tscan_L24.json")
SAMPLES = 60
N_MEASURE = 100
TAU_INT = 2.0


@pytest.fixture(scope="module")
def high_t():
    fx = json.load(open(FIXTURE))
    sig, diag = S.sigma_samples(T=1000.0, ns=SAMPLES, L=int(fx["model"]["L"]), J=fx["model"]["J"],
                                mu=fx["model"]["mu"])
    return fx, sig, diag


def _z(fx, sig, k):
    """(oracle mean - published 1/R) over the combined standard error."""
    pub = 1.0 / fx["R_rows"]["22"]
    col = sig[:, k]
    se_oracle = col.std(ddof=1) / math.sqrt(len(col))
    se_pub = col.std(ddof=1) * math.sqrt(TAU_INT / N_MEASURE)
    return (col.mean() - pub) / math.hypot(se_oracle, se_pub)


@pytest.mark.slow
def test_oracle_matches_published_r_at_eta_10_over_L2(high_t):
    fx, sig, _ = high_t
    k = S.MULTS.index(1.25)
    z = _z(fx, sig, k)
    print(f"eta = 10/L^2: R_oracle {1 / sig[:, k].mean():.1f} vs published {fx['R_rows']['22']}, z = {z:+.2f}")
    assert abs(z) <= 3.0, z


@pytest.mark.slow
def test_oracle_excludes_eta_8_over_L2(high_t):
    fx, sig, diag = high_t
    k = S.MULTS.index(1.0)
    z = _z(fx, sig, k)
    print(f"eta = 8/L^2: R_oracle {1 / sig[:, k].mean():.1f} vs published {fx['R_rows']['22']}, z = {z:+.2f}")
    assert z >= 3.0, z
    # why η matters here: the diagonal (n = m) terms, ∝ 1/η, dominate σ_DC
    assert np.mean(diag) >= 0.85
    # σ_DC decreases monotonically with η on every sample
    assert np.all(np.diff(sig, axis=1) < 0)
