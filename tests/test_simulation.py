"""run_simulation (src/Simulation.jl:34-236) over the hot path.

CPU: the driver logic — adaptive Nt rule, log lines, observables.csv format —
with the oracle behind the FermionContext API (tests/oracle_context.py).
GPU: the same driver on the HIP path against the oracle-backed run with the
same seed; per-sweep records agree within the sweep tolerances of
test_gpu_parity.py (|ΔdH| ≤ 1e-8 (1 + |dH|), observables ≤ 1e-9 abs)."""
import importlib
import os

import numpy as np
import pytest

from oracle_context import OracleContext


@pytest.fixture(scope="module")
def sim(dwhmc):
    return importlib.import_module(dwhmc.__name__ + ".simulation")


@pytest.fixture(scope="module")
def hmc_mod(dwhmc):
    return importlib.import_module(dwhmc.__name__ + ".hmc")


def test_adaptive_nt_rule(sim):
    """src/Simulation.jl:109-129: windows of 5; <0.60 -> +2; >0.95 and Nt>4 -> -1."""
    ctl = sim.AdaptiveNt(10)
    seq = [True, True, False, False, False,      # 0.4 -> 12
           True, True, True, True, False,        # 0.8 -> stable
           True, True, True, True, True]         # 1.0 -> 11
    out = [ctl.record(i + 1, a) for i, a in enumerate(seq)]
    assert [o for o in out if o is not None] == [(0.4, 10, 12), (0.8, 12, 12), (1.0, 12, 11)]
    ctl = sim.AdaptiveNt(4)
    for i in range(1, 6):
        r = ctl.record(i, True)
    assert r == (1.0, 4, 4)                      # Nt > 4 required to shrink


def test_obs_csv_line_format(sim, dwhmc):
    obs = dwhmc.ObservablesResult(-1.25, 0.1, 0.2, 0.3, 0.09, -0.05, 0.5, 0.25, 0.125)
    assert sim.obs_csv_line(7, True, 1.5e-3, obs) == (
        "7,1,1.50000e-03,-1.250000,0.100000,0.200000,0.300000,0.090000,-0.050000,0.500000,0.250000,0.125000\n")


def _run(sim, hmc_mod, dwhmc, out_dir, ctx_cls, seed=11, **kw):
    p = dwhmc.ModelParameters(4, 4, 1.0, -0.35, -1.08, 1.0, 0.25, 8.0, 0.8, 1.0)
    saved = hmc_mod.FermionContext
    if ctx_cls is not None:
        hmc_mod.FermionContext = ctx_cls
    try:
        return sim.run_simulation(p, str(out_dir), rng=np.random.default_rng(seed), verbose=False, **kw)
    finally:
        hmc_mod.FermionContext = saved


def test_run_simulation_driver_on_oracle(sim, hmc_mod, dwhmc, tmp_path):
    res = _run(sim, hmc_mod, dwhmc, tmp_path, OracleContext, n_therm=10, n_measure=10,
               Nt_therm_init=2, Nt_measure=3)
    log = (tmp_path / "simulation.log").read_text()
    for s in ("Starting Simulation...", "System: 4x4, β=8.0", "--- Thermalization Start ---",
              "Init: Nt=2", "Thermalization Done.", "--- Measurement Start ---", "Settings: Nt=3",
              "Meas 10/10.", "Measurement Done."):
        assert s in log, s
    rows = (tmp_path / "observables.csv").read_text().splitlines()
    assert rows[0] == sim.OBS_HEADER and len(rows) == 11
    trows = (tmp_path / "transport.csv").read_text().splitlines()
    assert trows[0] == sim.TRANSPORT_HEADER and len(trows) == 11      # measure_transport_freq = 1
    for k, (i, spec) in enumerate(res.transport):
        assert trows[k + 1] == sim.transport_csv_line(i, spec).rstrip("\n")
    # bins of 5 (src/Simulation.jl:180-220): sweep_5 and sweep_10, the mean of their members
    spec_dir = tmp_path / "spectra_bins"
    assert sorted(os.listdir(spec_dir)) == ["omega_grid.npy", "params.json", "sweep_10.npz", "sweep_5.npz"]
    b = np.load(spec_dir / "sweep_10.npz")
    assert int(b["count"]) == 5
    want = np.mean([s.optical_conductivity for _, s in res.transport[5:]], axis=0)
    assert np.allclose(b["opt_cond"], want, rtol=1e-13, atol=0)
    assert np.allclose(b["A_k0"], np.mean([s.A_k_omega0 for _, s in res.transport[5:]], axis=0))
    assert len(np.load(spec_dir / "omega_grid.npy")) == len(b["opt_cond"])
    for k, (i, acc, dH, obs) in enumerate(res.records):
        assert rows[k + 1] == sim.obs_csv_line(i, acc, dH, obs).rstrip("\n")
        assert np.isfinite(obs.total_energy) and -1.0 <= obs.hole_conc <= 1.0
    # the adaptive rule saw the thermalisation acceptances
    assert res.Nt_final >= 2


@pytest.mark.gpu
def test_run_simulation_device_matches_oracle(sim, hmc_mod, dwhmc, tmp_path):
    kw = dict(n_therm=10, n_measure=10, Nt_therm_init=4, Nt_measure=5)
    ref = _run(sim, hmc_mod, dwhmc, tmp_path / "ref", OracleContext, seed=5, **kw)
    dev = _run(sim, hmc_mod, dwhmc, tmp_path / "dev", None, seed=5, **kw)
    assert dev.Nt_final == ref.Nt_final
    assert len(dev.records) == len(ref.records) == 10
    for (i, a1, dh1, o1), (j, a2, dh2, o2) in zip(dev.records, ref.records):
        assert i == j and a1 == a2
        assert abs(dh1 - dh2) <= 1e-8 * (1 + abs(dh2)), (i, dh1, dh2)
        for f in ("total_energy", "Delta_amp", "Delta_local", "Delta_global", "S_Delta", "hole_conc",
                  "Delta_diff", "Delta_pair", "Delta_localpair"):
            assert abs(getattr(o1, f) - getattr(o2, f)) <= 1e-9, (i, f, getattr(o1, f), getattr(o2, f))
    # transport rows of the same trajectory (device eigenpairs vs LAPACK)
    assert len(dev.transport) == len(ref.transport) == 10
    for (i, s1), (j, s2) in zip(dev.transport, ref.transport):
        assert i == j
        for f in ("superfluid_stiffness", "dc_conductivity"):
            assert abs(getattr(s1, f) - getattr(s2, f)) <= 1e-8 * (1 + abs(getattr(s2, f))), (i, f)
        assert np.max(np.abs(s1.optical_conductivity - s2.optical_conductivity)) <= \
            1e-8 * (1 + np.max(np.abs(s2.optical_conductivity)))


def test_host_sweep_consumes_rng_like_reference(hmc_mod, dwhmc):
    """hmc_sweep with an rng draws the momenta, then rand() only when ΔH >= 0
    (src/HMC.jl:53,128), so a seeded generator runs in the reference's order."""
    p = dwhmc.ModelParameters(3, 3, 1.0, -0.35, -1.08, 1.0, 0.25, 8.0, 0.8, 1.0)
    saved = hmc_mod.FermionContext
    hmc_mod.FermionContext = OracleContext
    try:
        st = dwhmc.initialize_state(p, np.random.default_rng(1))
        cache = dwhmc.initialize_cache(p)
        dwhmc.init_static_H(cache, p, st)
        dwhmc.update_H_BdG(cache, p, st)
        dwhmc.diagonalize_H_BdG(cache, p)
        rng = np.random.default_rng(42)
        replay = np.random.default_rng(42)
        dt = dwhmc.calc_optimal_dt(p.beta, p.J, p.mass, 2)
        signs = set()
        for _ in range(12):
            acc, dH = dwhmc.hmc_sweep(cache, p, st, Nt=4, dt=dt, rng=rng)
            dwhmc.standard_complex_normal(replay, (p.N, 2))
            if dH >= 0:
                u = replay.random()
                assert acc == (u < np.exp(-dH))
            else:
                assert acc
            signs.add(dH >= 0)
        assert signs == {True, False}
        assert rng.random() == replay.random()
    finally:
        hmc_mod.FermionContext = saved


def test_run_simulation_chains_equals_single_runs(sim, hmc_mod, dwhmc, tmp_path):
    """run_simulation_chains (per-chain thermalisation, batched measurement
    phase) writes, for every chain, the files run_simulation writes for the
    same rng: the batching changes how the sweeps are launched, not the
    Markov chains (oracle backend, so the arithmetic is the same bits)."""
    kw = dict(n_therm=10, n_measure=6, Nt_therm_init=2, Nt_measure=3, measure_transport_freq=2, bin_size=2)
    p = dwhmc.ModelParameters(4, 4, 1.0, -0.35, -1.08, 1.0, 0.25, 8.0, 0.8, 1.0)
    saved = hmc_mod.FermionContext
    hmc_mod.FermionContext = OracleContext
    try:
        singles = [sim.run_simulation(p, str(tmp_path / f"single{k}"), rng=np.random.default_rng(100 + k),
                                      verbose=False, **kw) for k in range(2)]
        multi = sim.run_simulation_chains(p, [str(tmp_path / f"chain{k}") for k in range(2)],
                                          [np.random.default_rng(100 + k) for k in range(2)], **kw)
    finally:
        hmc_mod.FermionContext = saved
    for k in range(2):
        for f in ("observables.csv", "transport.csv"):
            assert (tmp_path / f"single{k}" / f).read_text() == (tmp_path / f"chain{k}" / f).read_text(), (k, f)
        assert multi[k].Nt_final == singles[k].Nt_final
        assert sorted(os.listdir(tmp_path / f"chain{k}" / "spectra_bins")) == \
            sorted(os.listdir(tmp_path / f"single{k}" / "spectra_bins"))


def test_transport_batch_writes_the_same_files(sim, hmc_mod, dwhmc, tmp_path):
    """transport_batch > 1 (TransportQueue: Δ snapshots measured in one
    batched call) delays the transport rows, it does not change them: same
    transport.csv and spectra bins as one measurement per sweep, for the
    single-chain driver and the batched-chains driver, a batch size that does
    not divide the measurement count included (the tail is flushed)."""
    kw = dict(n_therm=6, n_measure=7, Nt_therm_init=2, Nt_measure=3, measure_transport_freq=1, bin_size=2)
    p = dwhmc.ModelParameters(4, 4, 1.0, -0.35, -1.08, 1.0, 0.25, 8.0, 0.8, 1.0)
    saved = hmc_mod.FermionContext
    hmc_mod.FermionContext = OracleContext
    try:
        for tb in (1, 3):
            sim.run_simulation(p, str(tmp_path / f"s{tb}"), rng=np.random.default_rng(7), verbose=False,
                               transport_batch=tb, **kw)
            sim.run_simulation_chains(p, [str(tmp_path / f"c{tb}_{k}") for k in range(2)],
                                      [np.random.default_rng(7 + k) for k in range(2)], transport_batch=tb, **kw)
    finally:
        hmc_mod.FermionContext = saved
    for a, b in [("s1", "s3"), ("c1_0", "c3_0"), ("c1_1", "c3_1"), ("s1", "c3_0")]:
        for f in ("observables.csv", "transport.csv"):
            assert (tmp_path / a / f).read_text() == (tmp_path / b / f).read_text(), (a, b, f)
        names = sorted(os.listdir(tmp_path / a / "spectra_bins"))
        assert names == sorted(os.listdir(tmp_path / b / "spectra_bins"))
        assert len((tmp_path / a / "transport.csv").read_text().splitlines()) == 8
        for n in names:
            if n.endswith(".npz"):
                x, y = np.load(tmp_path / a / "spectra_bins" / n), np.load(tmp_path / b / "spectra_bins" / n)
                for key in x.files:
                    assert np.array_equal(x[key], y[key]), (a, b, n, key)
