#!/usr/bin/env python3
"""Headline benchmark: fp64 leapfrog steps/s of DwaveHMC.jl's hot path
(BASELINE.json metric) on MI355X, one process per GPU.

A bench "step" is ONE leapfrog step of hmc_sweep! (src/HMC.jl:98-114) for
every chain the rank owns: drift, pairing update, pole-expanded no-pivot LU of
H_BdG(Δ) - i y_q for all poles, force contraction, kick.  The timed region
runs steps/Nt complete sweeps (momentum refresh, H_old, backup, initial force,
Nt leapfrog steps, H_new, Metropolis, restore), so Metropolis and energies
are inside the timed work.  Workload (BASELINE configs[2] / C3): L=32
(N=1024, BdG n=2048), β=16, one chain per GPU; t=1, t'=-0.35, μ=-1.08, W=1,
n_imp=0.05, J=0.8, m=1, Nt=10, dt = calc_optimal_dt (src/Simulation.jl:11-14);
synthetic disorder/Δ₀/momenta from seed 1000+replica.  N>1: independent
disorder replicas per rank (weak scaling), no collective in the data path;
torch.distributed (RCCL) only for the barrier, the max-time reduction and the
observable gather.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--L 32] [--beta 16]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "fp64 leapfrog steps/sec at L=32, 1→8 MI355X; % fp64 MFMA roofline"
PEAK_F64_TFLOPS = 78.6        # MI355X dense fp64 matrix peak (= fp64 vector peak on CDNA4)
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E peak (MI355X_MICROARCH.md)
TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01_pmc_traffic.json")


def measured_traffic(kernel, L, beta, chains):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md
    gfx950 correction) for this exact workload, else None.  PMC counters cannot
    be read inside the timed run, so they come from their own profiled runs."""
    try:
        with open(TRAFFIC_FILE) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, None
    w = rec.get("workload", {})
    if (w.get("L"), w.get("beta"), w.get("chains")) != (L, beta, chains):
        return None, None
    k = rec.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return k["hbm_bytes_per_launch"], "profiles/" + os.path.basename(TRAFFIC_FILE)


# BASELINE.json configs; the headline line is C3.
PRESETS = {
    "C2": dict(L=16, beta=8.0, chains=1, label="L=16 beta=8 single-chain HMC (BASELINE configs[1], C2)"),
    "C3": dict(L=32, beta=16.0, chains=1, label="L=32 beta=16 single-chain HMC (BASELINE configs[2], C3)"),
    "C4": dict(L=32, beta=16.0, chains=1, label="L=32 beta=16 one disorder replica per GPU (BASELINE configs[3], C4)"),
    "C5": dict(L=48, beta=32.0, chains=4, label="L=48 beta=32 4 chains/GPU batched (BASELINE configs[4], C5)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50, help="leapfrog steps timed (multiple of --Nt)")
    ap.add_argument("--warmup", type=int, default=10, help="untimed leapfrog steps (multiple of --Nt)")
    ap.add_argument("--config", choices=sorted(PRESETS), default=None,
                    help="BASELINE config preset (default: C3, or C4 when launched on >1 GPU)")
    ap.add_argument("--L", type=int, default=None)
    ap.add_argument("--beta", type=float, default=None)
    ap.add_argument("--chains", type=int, default=None, help="chains per GPU")
    ap.add_argument("--Nt", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=0, help="oracle leapfrog steps for the CPU leg (0 = auto)")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--algo", choices=["auto", "dense", "cr"], default="auto",
                    help="factorisation (include/dwhmc.h DWH_ALGO_*); auto = cyclic reduction when 2L <= 96")
    return ap.parse_args()


def synthetic(p, O, replica, nchains, Nt, nsweeps):
    """Disorder, Δ₀ and the sweep draws for `nchains` chains of one replica."""
    dis, D0 = [], []
    for c in range(nchains):
        rng = np.random.default_rng(1000 + replica * nchains + c)
        st = O.initialize_state(p, rng)            # src/Types.jl:118-134
        dis.append(st.disorder_pot)
        D0.append(st.Delta)
    rng = np.random.default_rng(7_000_000 + replica)
    shape = (nsweeps, nchains, p.N, 2)
    noise = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)) * math.sqrt(0.5)
    uni = rng.random((nsweeps, nchains))
    return np.stack(dis), np.stack(D0), noise, uni


def cpu_baseline(O, p, Delta0, disorder, steps):
    """Oracle (numpy/scipy zheevr restatement) leapfrog steps on the host."""
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()
                       if i.get("internal_api") in ("openblas", "mkl", "blis")] or [1])
    except Exception:
        threads = os.cpu_count() or 1
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, disorder)
    Delta = Delta0.copy()
    pi = np.zeros_like(Delta)
    O.update_H_BdG(cache, p, Delta)
    O.diagonalize_H_BdG(cache, p)
    O.compute_forces(cache, p, Delta)
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, 10)
    t0 = time.perf_counter()
    for _ in range(steps):                          # src/HMC.jl:101-113
        Delta += dt / (2 * p.mass) * pi
        O.update_H_BdG(cache, p, Delta)
        O.diagonalize_H_BdG(cache, p)
        O.compute_forces(cache, p, Delta)
        pi += dt * cache.forces
    el = time.perf_counter() - t0
    return steps / el, threads, el


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    preset = PRESETS[a.config or ("C4" if world > 1 else "C3")]
    custom = any(getattr(a, k) not in (None, preset[k]) for k in ("L", "beta", "chains"))
    for k in ("L", "beta", "chains"):
        if getattr(a, k) is None:
            setattr(a, k, preset[k])
    workload = (f"L={a.L} beta={a.beta:g} {a.chains} chain(s)/GPU (custom)" if custom else preset["label"])
    if a.steps % a.Nt or a.warmup % a.Nt:
        raise SystemExit("--steps and --warmup must be multiples of --Nt")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import dwhmc_loader
    from oracle import dwhmc_oracle as O   # synthetic-input generation + CPU leg only
    m = dwhmc_loader.load_package()
    m.load_library(build_if_missing=False)

    p = O.ModelParameters(a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    n_warm, n_time = a.warmup // a.Nt, a.steps // a.Nt
    dis, D0, noise, uni = synthetic(p, O, rank, a.chains, a.Nt, n_warm + n_time)
    dt = m.calc_optimal_dt(p.beta, p.J, p.mass, a.Nt)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis,
                           device=local, algo=a.algo)
    cr = ctx.info["algo"] == 1
    # dominant kernel: block products (cr) / rank-128 GJ update (dense)
    dom = "cr_gemm" if cr else "gj_update"
    ctx.set_pairing(D0)
    ctx.factorize()                                 # src/Simulation.jl:84-86
    ctx.load_draws(noise, uni)                      # inputs resident in HBM before timing
    if n_warm:
        ctx.run_sweeps(0, n_warm, a.Nt, dt, p.mass)
    ctx.synchronize()

    if dist is not None:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.run_sweeps(n_warm, n_time, a.Nt, dt, p.mass)
    ctx.synchronize()
    el = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        dist.barrier()

    acc, dH = ctx.sweep_results(n_warm, n_time)
    info = ctx.info
    kern = {}
    timed_sweeps = 0
    if not a.no_timing:
        # Per-kernel HIP events (on the context's stream) in an instrumented
        # replay of the first timed sweeps right after the timed region: each
        # event record is a barrier packet that costs ~20 % of the step when
        # interleaved with ~30 launches per step, so the timed region itself
        # runs without them.  Same kernels, same sizes; rocprofv3 --stats of the
        # same command (profiles/) agrees on the per-launch averages.
        timed_sweeps = min(n_time, 2)
        ctx.timing_enable([dom, "assemble"] + (["cr_inv"] if cr else []))
        ctx.timing_reset()
        ctx.run_sweeps(n_warm, timed_sweeps, a.Nt, dt, p.mass)
        ctx.synchronize()
        for k in [dom, "assemble"] + (["cr_inv"] if cr else []):
            kern[k] = ctx.timing_read(k)
        ctx.timing_enable(False)
    # observables gather over RCCL (the only collective): acceptance and <dH>
    obs = np.array([acc.mean(), dH.mean(), float(np.mean(np.exp(-dH)))], dtype=np.float64)
    if dist is not None:
        import torch
        t = torch.tensor(obs, device=f"cuda:{local}")
        gl = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, gl, dst=0)
        if rank == 0:
            obs = torch.stack(gl).mean(0).cpu().numpy()

    if rank == 0:
        leap = a.steps * a.chains * world
        value = leap / el
        ms_per_step = 1000.0 * el / a.steps
        N, P = info["N"], info["npoles"]
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "leapfrog steps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": workload,
                       "L": a.L, "N": N, "bdg_dim": 2 * N, "beta": a.beta, "chains_per_gpu": a.chains,
                       "Nt": a.Nt, "dt": dt, "poles": P, "kappa": info["kappa"],
                       "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
            "acceptance": float(obs[0]), "mean_dH": float(obs[1]), "mean_exp_minus_dH": float(obs[2]),
            "algorithm": "block cyclic reduction" if cr else "dense Schur complement + Gauss-Jordan",
            "ref_equiv_tflops": leap * (40.0 / 3.0) * (2 * N) ** 3 / el / 1e12,
            "dense_equiv_tflops": leap * P * 8.0 * N ** 3 / el / 1e12,
        }
        if not cr:
            rec["alg_tflops"] = rec["dense_equiv_tflops"]
        if kern:
            ms, n, w = kern[dom]
            ach = w / n / (ms / n * 1e-3) / 1e12 if n and ms > 0 else None
            if cr:
                kname = f"k_cr_gemm<{info['block']},1,4>"   # 16x16 tiles, 4-way K split (every stage)
                msi, ni, wi = kern["cr_inv"]
                # the CR path's own algorithmic flops: block products + block inversions
                # the CR path's own algorithmic flops per leapfrog step (block
                # products + block inversions) x steps of the timed region
                steps_t = timed_sweeps * a.Nt
                rec["alg_tflops"] = (w + wi) / steps_t * a.steps * world / el / 1e12
                rec["alg_flops_per_step"] = (w + wi) / steps_t / a.chains
                rec["cr_inv"] = {"bound": "latency", "kernel": f"k_cr_inv<{info['block'] // 16}>",
                                 "achieved_tflops": wi / (msi * 1e-3) / 1e12 if msi > 0 else None,
                                 "avg_launch_us": 1000.0 * msi / ni if ni else None,
                                 "ms_per_step": msi / (timed_sweeps * a.Nt)}
            else:
                nb = -(-info["N"] // 64)                 # GJ block steps; odd nb ends with one rank-64 step
                kname = "k_gj_update<2>" if nb % 2 == 0 else "k_gj_update<2>+<0>"
            traffic, tsrc = measured_traffic(kname, a.L, a.beta, a.chains)
            rec["roofline"] = {"bound": "mfma", "kernel": kname, "achieved": ach,
                               "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                               "frac": ach / PEAK_F64_TFLOPS if ach else None, "traffic": traffic,
                               "traffic_unit": "bytes/launch", "traffic_source": tsrc,
                               "avg_launch_us": 1000.0 * ms / n if n else None,
                               "flops_per_launch": w / n if n else None}
            rec[f"{dom}_ms_per_step"] = ms / (timed_sweeps * a.Nt)
            ms, n, w = kern["assemble"]
            if n and ms > 0:
                gbs = w / n / (ms / n * 1e-3) / 1e9
                rec["assembly"] = {"bound": "hbm", "kernel": "k_cr_fill" if cr else "k_assemble",
                                   "achieved": gbs,
                                   "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                                   "bytes_per_launch": w / n, "avg_launch_us": 1000.0 * ms / n}
        if not a.no_cpu_baseline and world == 1:
            steps_cpu = a.cpu_steps or (1 if a.L >= 48 else 3 if a.L >= 32 else 20)
            v, threads, el_cpu = cpu_baseline(O, p, D0[0], dis[0], steps_cpu)
            rec["cpu_baseline"] = {"value": v, "unit": "leapfrog steps/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"{steps_cpu} leapfrog steps at L={a.L}, beta={a.beta:g} "
                                             f"(numpy/scipy zheevr restatement, {el_cpu:.1f} s)"}
        print(json.dumps(rec), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
