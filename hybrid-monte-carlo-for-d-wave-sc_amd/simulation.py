"""run_simulation: the reference's driver (src/Simulation.jl:34-236) over the
MI355X hot path.

Same phases, adaptive-Nt rule, log lines and observables.csv format as the
reference; every sweep's fermionic work runs on the GPU through the C ABI
(hmc.py -> FermionContext), and the lightweight measurements come from the
factorisation outputs (P_ij, E_f, Tr ρ_hh; hmc.measure_observables).

Every measure_transport_freq sweeps the heavy measurement
(`measure_transport_and_spectra`, src/Observables.jl:314-526) runs on the
device as well (own eigensolver + HIP kernels) and fills transport.csv;
the JLD2 spectra bins become numpy files (no JLD2 writer in this image).
The reference's RNG is global and unseeded; here the caller
passes `rng` (draw order per sweep: randn(ComplexF64, N, 2), then rand()).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import dataclass, field
from datetime import datetime

import numpy as np

from . import hmc as H
from .context import transport_grid

OBS_HEADER = ("Sweep,Accepted,dH,Energy,Delta_Amp,Delta_Loc,Delta_Glob,S_Delta,Hole_p,Delta_Diff,"
              "Delta_Pair,Delta_LocalPair")
TRANSPORT_HEADER = "Sweep,Superfluid_Stiffness,DC_Conductivity"


def obs_csv_line(sweep: int, acc: bool, dH: float, obs: H.ObservablesResult) -> str:
    """One observables.csv row, src/Simulation.jl:161-166 formats."""
    return "%d,%d,%.5e,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f\n" % (
        sweep, int(acc), dH, obs.total_energy, obs.Delta_amp, obs.Delta_local, obs.Delta_global,
        obs.S_Delta, obs.hole_conc, obs.Delta_diff, obs.Delta_pair, obs.Delta_localpair)


@dataclass
class AdaptiveNt:
    """Thermalisation step-count controller, src/Simulation.jl:103-129: every
    `window` sweeps, acceptance < 0.60 -> Nt += 2; > 0.95 and Nt > 4 -> Nt -= 1."""
    Nt: int
    window: int = 5
    recent: int = 0

    def record(self, i: int, accepted: bool):
        """Sweep i (1-based) finished.  Returns None between windows, else
        (rate, old_Nt, new_Nt)."""
        if accepted:
            self.recent += 1
        if i % self.window != 0:
            return None
        rate = self.recent / self.window
        self.recent = 0
        old = self.Nt
        if rate < 0.60:
            self.Nt += 2
        elif rate > 0.95 and self.Nt > 4:
            self.Nt -= 1
        return rate, old, self.Nt


@dataclass
class SimulationResult:
    Nt_final: int
    therm_acceptance: float
    meas_acceptance: float
    records: list = field(default_factory=list)   # (sweep, accepted, dH, ObservablesResult)
    transport: list = field(default_factory=list)  # (sweep, SpectrumResult)


def transport_csv_line(sweep: int, spec) -> str:
    """src/Simulation.jl:174-177."""
    return "%d,%.6f,%.6f\n" % (sweep, spec.superfluid_stiffness, spec.dc_conductivity)


def write_spectra_header(spec_dir: str, p) -> None:
    """jldsave(params, omega_grid) of src/Simulation.jl:89."""
    os.makedirs(spec_dir, exist_ok=True)
    params = {k: getattr(p, k) for k in ("Lx", "Ly", "t", "tp", "mu", "W", "n_imp", "beta", "J", "mass",
                                         "eta", "domega", "omega_max")}
    with open(os.path.join(spec_dir, "params.json"), "w") as f:
        json.dump(params, f, indent=1)
    n, _ = transport_grid(p.eta, p.domega, p.omega_max)
    np.save(os.path.join(spec_dir, "omega_grid.npy"), p.eta + p.domega * np.arange(n))


class SpectraBins:
    """Bin accumulator of src/Simulation.jl:180-220: sums the spectra of
    bin_size measurements, then writes their mean as group sweep_<i>."""

    def __init__(self):
        self.count = 0
        self.acc = None

    def add(self, spec) -> int:
        arrs = [spec.optical_conductivity, spec.dos, spec.dos_AN, spec.A_k_omega0]
        if self.count == 0:
            self.acc = [np.array(a, dtype=np.float64, copy=True) for a in arrs]
        else:
            for a, b in zip(self.acc, arrs):
                a += b
        self.count += 1
        return self.count

    def flush(self, spec_dir: str, sweep: int) -> None:
        c = self.count
        oc, dos, dos_an, ak = (a / c for a in self.acc)
        np.savez(os.path.join(spec_dir, f"sweep_{sweep}.npz"), opt_cond=oc, dos=dos, dos_AN=dos_an,
                 A_k0=ak, count=c)
        self.count = 0
        self.acc = None


class ChainOutput:
    """The files of one run_simulation (src/Simulation.jl:45-56,69-73):
    simulation.log (appended, timestamped tee), observables.csv and
    transport.csv (truncated, headers written), spectra_bins/."""

    def __init__(self, out_dir: str, verbose: bool):
        os.makedirs(out_dir, exist_ok=True)
        self.verbose = verbose
        self.spec_dir = os.path.join(out_dir, "spectra_bins")
        self.f_log = open(os.path.join(out_dir, "simulation.log"), "a")
        self.f_obs = open(os.path.join(out_dir, "observables.csv"), "w")
        self.f_trans = open(os.path.join(out_dir, "transport.csv"), "w")
        self.f_obs.write(OBS_HEADER + "\n")
        self.f_trans.write(TRANSPORT_HEADER + "\n")
        self.bins = SpectraBins()

    def tee(self, msg: str):
        line = f"[{datetime.now().strftime('%Y-%m-%d %H:%M:%S')}] {msg}"
        print(line, file=self.f_log, flush=True)
        if self.verbose:
            print(line, flush=True)

    def header(self, p, n_therm, n_measure, measure_transport_freq, bin_size):
        self.tee("Starting Simulation...")
        self.tee(f"System: {p.Lx}x{p.Ly}, β={p.beta}, n_imp={p.n_imp}, J={p.J}")
        self.tee(f"Config: Therm={n_therm}, Sweep={n_measure}, TransFreq={measure_transport_freq}, "
                 f"BinSize={bin_size}")
        self.tee("Initializing State...")

    def observables(self, i, acc, dH, obs):
        self.f_obs.write(obs_csv_line(i, acc, dH, obs))
        self.f_obs.flush()

    def transport(self, i, spec, bin_size):
        self.f_trans.write(transport_csv_line(i, spec))
        self.f_trans.flush()
        if self.bins.add(spec) >= bin_size:
            self.bins.flush(self.spec_dir, i)

    def close(self):
        self.f_log.close()
        self.f_obs.close()
        self.f_trans.close()


def thermalize(cache, p, state, out: ChainOutput, n_therm: int, Nt_therm_init: int, rng):
    """The adaptive thermalisation of src/Simulation.jl:92-130 for one chain;
    returns (final Nt, acceptance rate)."""
    ctl = AdaptiveNt(Nt_therm_init)
    dt = H.calc_optimal_dt(p.beta, p.J, p.mass, ctl.Nt)
    out.tee("--- Thermalization Start ---")
    out.tee(f"Init: Nt={ctl.Nt}, dt={round(dt, 5)}")
    t0 = time.time()
    acc_therm = 0
    for i in range(1, n_therm + 1):
        acc, _ = H.hmc_sweep(cache, p, state, Nt=ctl.Nt, dt=dt, rng=rng)
        acc_therm += int(acc)
        r = ctl.record(i, acc)
        if r is None:
            continue
        rate, old, new = r
        if new != old:
            dt = H.calc_optimal_dt(p.beta, p.J, p.mass, new)
            out.tee("Therm %d/%d. Rate=%.2f. Adjust Nt: %d -> %d, dt: %.4f" % (i, n_therm, rate, old, new, dt))
        elif i % 20 == 0:
            out.tee("Therm %d/%d. Rate=%.2f. Nt=%d (Stable)" % (i, n_therm, rate, new))
    out.tee(f"Thermalization Done. Time: {round(time.time() - t0, 2)}s")
    return ctl.Nt, acc_therm / max(n_therm, 1)


class TransportQueue:
    """Transport measurements (src/Simulation.jl:169-220) of one chain taken at
    the Δ of their sweeps and evaluated `batch` at a time: the eigensolves of
    a batch run as one batched call (dwh_measure_transport_deltas), ~3x the
    throughput of one call per sweep at L = 32.  Rows and bins come out in
    sweep order, each when its batch is measured (batch = 1: right away, as
    the reference writes them)."""

    def __init__(self, ctx, p, out: ChainOutput, res: SimulationResult, bin_size: int, batch: int, chain: int = 0):
        self.ctx, self.p, self.out, self.res = ctx, p, out, res
        self.bin_size, self.batch, self.chain = bin_size, max(1, int(batch)), chain
        self.pending = []            # (sweep, Δ snapshot)

    def add(self, sweep: int, Delta):
        self.pending.append((sweep, np.array(Delta, dtype=np.complex128, copy=True)))
        if len(self.pending) >= self.batch:
            self.flush()

    def flush(self):
        if not self.pending:
            return
        p = self.p
        if self.batch == 1:
            specs = [self.ctx.measure_transport(p.eta, p.domega, p.omega_max, chain=self.chain)]
        else:
            specs = self.ctx.measure_transport_deltas(np.stack([d for _, d in self.pending]), p.eta, p.domega,
                                                      p.omega_max, chain=self.chain)
        for (i, _), r in zip(self.pending, specs):
            spec = H.SpectrumResult(**r)
            self.out.transport(i, spec, self.bin_size)
            self.res.transport.append((i, spec))
        self.pending = []


def run_simulation(p: H.ModelParameters, out_dir: str, *, n_therm: int = 100, n_measure: int = 500,
                   Nt_therm_init: int = 10, Nt_measure: int = 5, measure_transport_freq: int = 1,
                   bin_size: int = 5, verbose: bool = True, rng: np.random.Generator | None = None,
                   device: int = 0, delta_cap: float = 0.0, state: H.SimulationState | None = None,
                   cache: H.ComputeCache | None = None, transport_batch: int = 1) -> SimulationResult:
    """src/Simulation.jl:34-236.  Files in out_dir: simulation.log (appended),
    observables.csv, transport.csv (one row per transport measurement, every
    measure_transport_freq sweeps; <= 0 disables), and spectra_bins/ — the
    reference's spectra_bins.jld2 (:52,89,206-214) as numpy files: params.json,
    omega_grid.npy, and one sweep_<i>.npz per completed bin of bin_size
    measurements (opt_cond, dos, dos_AN, A_k0 averaged; count).
    transport_batch > 1 evaluates that many measurement sweeps' transport in
    one batched call (TransportQueue): same rows and bins, written up to
    transport_batch - 1 sweeps later."""
    rng = rng if rng is not None else np.random.default_rng()
    out = ChainOutput(out_dir, verbose)
    try:
        out.header(p, n_therm, n_measure, measure_transport_freq, bin_size)
        if state is None:
            state = H.initialize_state(p, rng)
        if cache is None:
            cache = H.initialize_cache(p, device=device, delta_cap=delta_cap)
        H.init_static_H(cache, p, state)
        H.update_H_BdG(cache, p, state)
        H.diagonalize_H_BdG(cache, p)
        if measure_transport_freq > 0:
            write_spectra_header(out.spec_dir, p)
        Nt_fin, acc_th = thermalize(cache, p, state, out, n_therm, Nt_therm_init, rng)

        dt_meas = H.calc_optimal_dt(p.beta, p.J, p.mass, Nt_measure)
        out.tee("--- Measurement Start ---")
        out.tee(f"Settings: Nt={Nt_measure}, dt={round(dt_meas, 5)}")
        t1 = time.time()
        acc_total = 0
        res = SimulationResult(Nt_fin, acc_th, 0.0)
        tq = TransportQueue(cache.require(), p, out, res, bin_size, transport_batch)
        for i in range(1, n_measure + 1):
            acc, dH = H.hmc_sweep(cache, p, state, Nt=Nt_measure, dt=dt_meas, rng=rng)
            acc_total += int(acc)
            obs = H.measure_observables(cache, p, state)
            out.observables(i, acc, dH, obs)
            res.records.append((i, acc, dH, obs))
            if measure_transport_freq > 0 and i % measure_transport_freq == 0:
                tq.add(i, state.Delta)
            if i % 10 == 0:
                out.tee("Meas %d/%d. Acc=%.2f. E=%.4f" % (i, n_measure, acc_total / i, obs.total_energy))
        tq.flush()
        res.meas_acceptance = acc_total / max(n_measure, 1)
        out.tee(f"Measurement Done. Total Time: {round(time.time() - t1, 2)}s")
        return res
    finally:
        out.close()


def run_simulation_chains(p: H.ModelParameters, out_dirs, rngs, *, n_therm: int = 100, n_measure: int = 500,
                          Nt_therm_init: int = 10, Nt_measure: int = 5, measure_transport_freq: int = 1,
                          bin_size: int = 5, verbose: bool = False, device: int = 0,
                          delta_cap: float = 0.0, transport_batch: int = 1) -> list:
    """len(out_dirs) independent run_simulation's (src/Simulation.jl:34-236),
    chain k writing out_dirs[k] and drawing from rngs[k] in the reference's
    order (initialize_state, then per sweep randn(ComplexF64) and rand() only
    when ΔH >= 0).  Each chain is thermalised on its own single-chain context
    (its own adaptive Nt, :92-130); the measurement phase, whose Nt_measure is
    common to all chains (:133-228), runs every chain in one batched context
    (one factorisation launch sequence per leapfrog step for all chains, and
    one batched eigensolve per transport measurement,
    dwh_measure_transport_batched; with transport_batch > 1, per chain
    transport_batch sweeps at once, TransportQueue).  Returns one
    SimulationResult per chain; each chain runs the same Markov chain as
    run_simulation up to the pole approximation (bit-equal on the oracle
    backend: on the device the batched context selects one pole set for the
    largest spectral bound over the chains, and a guard trip re-selects it
    for every chain, so dH differs at ~1e-12 and a Metropolis decision can
    differ)."""
    K = len(out_dirs)
    if len(rngs) != K or K < 1:
        raise ValueError("one rng per output directory")
    outs = [ChainOutput(d, verbose) for d in out_dirs]
    try:
        states, results = [], []
        for k in range(K):
            outs[k].header(p, n_therm, n_measure, measure_transport_freq, bin_size)
            st = H.initialize_state(p, rngs[k])
            cache = H.initialize_cache(p, device=device, delta_cap=delta_cap)
            H.init_static_H(cache, p, st)
            H.update_H_BdG(cache, p, st)
            H.diagonalize_H_BdG(cache, p)
            if measure_transport_freq > 0:
                write_spectra_header(outs[k].spec_dir, p)
            Nt_fin, acc_th = thermalize(cache, p, st, outs[k], n_therm, Nt_therm_init, rngs[k])
            cache.ctx.close()
            states.append(st)
            results.append(SimulationResult(Nt_fin, acc_th, 0.0))

        dis = np.stack([st.disorder_pot for st in states])
        ctx = H.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis,
                             delta_cap=delta_cap, device=device)
        try:
            ctx.set_pairing(np.stack([st.Delta for st in states]))
            ctx.factorize()
            dt_meas = H.calc_optimal_dt(p.beta, p.J, p.mass, Nt_measure)
            for o in outs:
                o.tee("--- Measurement Start ---")
                o.tee(f"Settings: Nt={Nt_measure}, dt={round(dt_meas, 5)}")
            t1 = time.time()
            acc_total = np.zeros(K, dtype=np.int64)
            tqs = [TransportQueue(ctx, p, outs[k], results[k], bin_size, transport_batch, chain=k)
                   for k in range(K)] if transport_batch > 1 else None
            for i in range(1, n_measure + 1):
                noise = np.stack([H.standard_complex_normal(r, (p.N, 2)) for r in rngs])
                dH = ctx.hmc_trajectory(noise, Nt_measure, dt_meas, p.mass)
                acc = np.array([bool(dH[k] < 0 or rngs[k].random() < math.exp(-dH[k])) for k in range(K)])
                ctx.hmc_finish(acc)
                acc_total += acc
                D, _ = ctx.get_state()
                P, Ef, tr = ctx.pairing(), ctx.fermion_energy(), ctx.hole_trace()
                specs = None
                if measure_transport_freq > 0 and i % measure_transport_freq == 0:
                    if tqs is None:
                        specs = ctx.measure_transport_all(p.eta, p.domega, p.omega_max)
                    else:
                        for k in range(K):
                            tqs[k].add(i, D[k])
                for k in range(K):
                    obs = H.observables_from_outputs(p, D[k], P[k], Ef[k], tr[k])
                    outs[k].observables(i, acc[k], float(dH[k]), obs)
                    results[k].records.append((i, bool(acc[k]), float(dH[k]), obs))
                    if specs is not None:
                        spec = H.SpectrumResult(**specs[k])
                        outs[k].transport(i, spec, bin_size)
                        results[k].transport.append((i, spec))
                    if i % 10 == 0:
                        outs[k].tee("Meas %d/%d. Acc=%.2f. E=%.4f" % (i, n_measure, acc_total[k] / i,
                                                                     obs.total_energy))
            for tq in tqs or []:
                tq.flush()
            for k in range(K):
                results[k].meas_acceptance = acc_total[k] / max(n_measure, 1)
                outs[k].tee(f"Measurement Done. Total Time: {round(time.time() - t1, 2)}s")
        finally:
            ctx.close()
        return results
    finally:
        for o in outs:
            o.close()
