"""Replica parallelism: one process per GPU, independent disorder realisations
and Markov chains, no collective in the data path.

Each rank owns `chains` chains on its own device (one batched context); after
every sweep it records 11 fp64 per chain — accepted, dH and the nine fields of
ObservablesResult (src/Observables.jl:70-80) — and the records are gathered
to rank 0 with torch.distributed (RCCL on MI355X, gloo in CPU tests), which
writes the reference's observables.csv format (src/Simulation.jl:71,161-166).
With transport_freq > 0 every rank also measures transport every
transport_freq sweeps for all its chains at once
(dwh_measure_transport_batched) and the (stiffness, dc) scalars are gathered
the same way into transport.csv (src/Simulation.jl:73,171-177).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

OBS_COLUMNS = ("Accepted", "dH", "Energy", "Delta_Amp", "Delta_Loc", "Delta_Glob", "S_Delta", "Hole_p",
               "Delta_Diff", "Delta_Pair", "Delta_LocalPair")
N_OBS = len(OBS_COLUMNS)


def observables_from_outputs(p, Delta, P, Ef, tr_hh):
    """The nine ObservablesResult fields (src/Observables.jl:88-222) for one
    chain from the factorisation outputs (P_ij, E_f, Tr ρ_hh)."""
    N = p.N
    dx, dy = Delta[:, 0], Delta[:, 1]
    g = np.sum(0.5 * (dx - dy)) / N
    Eb = p.beta / (2 * p.J) * float(np.sum(np.abs(Delta) ** 2))
    Px, Py = P[:, 0], P[:, 1]
    term = p.J * 0.5 * (Px - Py)
    return np.array([
        (Ef + Eb) / N,
        float(np.sum(0.5 * (np.abs(dx) + np.abs(dy)))) / N,
        float(np.sum(0.5 * np.abs(dx - dy))) / N,
        abs(g),
        abs(g) ** 2,
        2.0 * tr_hh / N - 1.0,
        float(np.sum((np.abs(dx - p.J * Px) + np.abs(dy - p.J * Py)) / 2.0)) / N,
        abs(np.sum(term) / N),
        float(np.sum(np.abs(term))) / N,
    ])


@dataclass
class ReplicaConfig:
    chains: int = 1
    n_sweeps: int = 10
    Nt: int = 10
    seed: int = 1000
    transport_freq: int = 0   # measure_transport_and_spectra every k sweeps (0: never)


def replica_seed(cfg: ReplicaConfig, rank: int, chain: int) -> int:
    return cfg.seed + rank * cfg.chains + chain


N_TR = 3   # transport record: sweep, superfluid stiffness, dc conductivity


def run_local(p, cfg: ReplicaConfig, rank: int, device: int, make_context, initialize_state,
              calc_optimal_dt, transport_out: list | None = None):
    """Run cfg.n_sweeps HMC sweeps for this rank's chains; returns
    (n_sweeps, chains, N_OBS).  `make_context(disorder) -> FermionContext`.
    With cfg.transport_freq > 0, one (chains, N_TR) array per transport
    measurement is appended to transport_out."""
    dis, D0, rngs = [], [], []
    for c in range(cfg.chains):
        rng = np.random.default_rng(replica_seed(cfg, rank, c))
        st = initialize_state(p, rng)
        dis.append(st.disorder_pot)
        D0.append(st.Delta)
        rngs.append(rng)
    ctx = make_context(np.stack(dis))
    ctx.set_pairing(np.stack(D0))
    ctx.factorize()                                        # src/Simulation.jl:84-86
    dt = calc_optimal_dt(p.beta, p.J, p.mass, cfg.Nt)
    out = np.zeros((cfg.n_sweeps, cfg.chains, N_OBS))
    for s in range(cfg.n_sweeps):
        noise = np.stack([(r.standard_normal((p.N, 2)) + 1j * r.standard_normal((p.N, 2))) * math.sqrt(0.5)
                          for r in rngs])
        uni = np.array([r.random() for r in rngs])
        acc, dH = ctx.hmc_sweep(noise, uni, cfg.Nt, dt, p.mass)
        D, _ = ctx.get_state()
        P = ctx.pairing()
        Ef = ctx.fermion_energy()
        tr = ctx.hole_trace()
        for c in range(cfg.chains):
            out[s, c, 0] = float(acc[c])
            out[s, c, 1] = dH[c]
            out[s, c, 2:] = observables_from_outputs(p, D[c], P[c], Ef[c], tr[c])
        if cfg.transport_freq > 0 and transport_out is not None and (s + 1) % cfg.transport_freq == 0:
            spec = ctx.measure_transport_all(p.eta, p.domega, p.omega_max)
            transport_out.append(np.array([[s + 1, r["superfluid_stiffness"], r["dc_conductivity"]]
                                           for r in spec]))
    ctx.close()
    return out


def gather_observables(local: np.ndarray, dist=None, device=None):
    """Gather (n_sweeps, chains, N_OBS) records of every rank to rank 0 ->
    (world*chains, n_sweeps, N_OBS) on rank 0, None elsewhere.  Uses the
    process group's backend (RCCL on GPUs with device = the rank's GPU, gloo
    on CPU); an initialised group of one rank still runs the collective."""
    import torch
    rec = np.ascontiguousarray(np.transpose(local, (1, 0, 2)))
    if dist is None or not dist.is_initialized():
        return rec
    t = torch.as_tensor(rec, dtype=torch.float64)
    if device is not None:
        t = t.to(device)
    world = dist.get_world_size()
    rank = dist.get_rank()
    bufs = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, bufs, dst=0)
    if rank != 0:
        return None
    return np.concatenate([b.cpu().numpy() for b in bufs], axis=0)


def write_observables_csv(path: str, records: np.ndarray):
    """observables.csv in the reference's column order and formats
    (src/Simulation.jl:71,161-166), one block of rows per replica chain."""
    with open(path, "w") as f:
        f.write("Replica,Sweep,Accepted,dH,Energy,Delta_Amp,Delta_Loc,Delta_Glob,S_Delta,Hole_p,"
                "Delta_Diff,Delta_Pair,Delta_LocalPair\n")
        for r in range(records.shape[0]):
            for s in range(records.shape[1]):
                x = records[r, s]
                f.write("%d,%d,%d,%.5e,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f,%.6f\n" %
                        (r, s + 1, int(x[0]), x[1], *x[2:]))


def write_transport_csv(path: str, records: np.ndarray):
    """transport.csv (src/Simulation.jl:73,174-177) with a Replica column;
    records: (replica chains, measurements, N_TR)."""
    with open(path, "w") as f:
        f.write("Replica,Sweep,Superfluid_Stiffness,DC_Conductivity\n")
        for r in range(records.shape[0]):
            for m in range(records.shape[1]):
                x = records[r, m]
                f.write("%d,%d,%.6f,%.6f\n" % (r, int(x[0]), x[1], x[2]))


# Launcher: tools/run_replicas.py (python -m torch.distributed.run ... tools/run_replicas.py)
