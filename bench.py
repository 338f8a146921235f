#!/usr/bin/env python3
"""Headline benchmark: fp64 leapfrog steps/s of DwaveHMC.jl's hot path
(BASELINE.json metric) on MI355X, one process per GPU.

A bench "step" is ONE leapfrog step of hmc_sweep! (src/HMC.jl:98-114) for
every chain the rank owns: drift, pairing update, pole-expanded factorisation
of H_BdG(Δ) - i y_q for all poles, force contraction, kick.  The timed region
runs exactly --steps leapfrog steps as complete trajectories (momentum
refresh, H_old, backup, initial force, Nt leapfrog steps, H_new, Metropolis,
restore), the last one shortened to the remainder when --steps is not a
multiple of Nt, so Metropolis and energies are inside the timed work.

Before anything is timed the chain is thermalised the way the reference's
driver does it (src/Simulation.jl:97-130: n_therm sweeps from Nt_therm_init
= 10, Nt += 2 when a 5-sweep window accepts < 60 %, Nt -= 1 above 95 %,
dt = calc_optimal_dt(β, J, m, Nt)); the timed region runs at the Nt the
thermalisation ends with.  --warmup leapfrog steps are then rounded up to
whole sweeps (untimed).

Workload (BASELINE configs[2] / C3): L=32 (N=1024, BdG n=2048), β=16, one
chain per GPU; t=1, t'=-0.35, μ=-1.08, W=1, n_imp=0.05, J=0.8, m=1;
synthetic disorder/Δ₀/momenta from seed 1000+replica.  N>1: independent
disorder replicas per rank (weak scaling), no collective in the data path;
torch.distributed (RCCL) only for the barrier, the max-time reduction and the
observable gather.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "fp64 leapfrog steps/sec at L=32, 1→8 MI355X; % fp64 MFMA roofline"
PEAK_F64_TFLOPS = 78.6        # MI355X dense fp64 matrix peak (= fp64 vector peak on CDNA4)
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E peak (MI355X_MICROARCH.md)
# newest committed PMC summary first (profiles/README.md)
TRAFFIC_FILES = [os.path.join(ROOT, "profiles", f) for f in ("r06_pmc_traffic.json", "r05_pmc_traffic.json", "r04_pmc_traffic.json", "r03_pmc_traffic.json", "r02_pmc_traffic.json",
                                                                     "r01_pmc_traffic.json")]
# SQ counter passes (tools/pmc_sq.sh -> tools/pmc_mfma.py): executed MFMA work per launch
MFMA_FILES = [os.path.join(ROOT, "profiles", f) for f in ("r06_sq_mfma_L32.json", "r05_sq_mfma_L32.json", "r04_sq_mfma_L32.json")]
# rocprofv3 --kernel-trace --stats summaries of the driver's command (tools/profile_round.sh)
KSTATS_FILES = {(32, 16.0, 1): [os.path.join(ROOT, "profiles", f) for f in ("r06_L32_beta16_kernel_stats.csv", "r05_L32_beta16_kernel_stats.csv")]}
CLOCK_GHZ = 2.4                # the clock PEAK_F64_TFLOPS is quoted at (1024 SIMDs x 32 flop/cycle)
ASSEMBLY_REPS = 200            # warm assembly launches timed for `assembly`


def inv_kernels(bp: int, coarse: bool) -> str:
    """The plan's block-inversion kernels: level 0 from the
    static particle block (k_cr_inv0 at BP = 64, k_cr_inv0_96 at 96,
    k_cr_inv0_32 at 32); coarser levels k_cr_inv<BP/16>, at BP = 32 the
    one-wave Schur complement k_cr_inv32 (the level-0 / coarse stages carrying
    side work are reported under cr_inv_side)."""
    l0 = {32: "k_cr_inv0_32", 64: "k_cr_inv0", 96: "k_cr_inv0_96"}.get(bp, f"k_cr_inv<{bp // 16}>")
    if not coarse:
        return l0
    return l0 + " + " + ("k_cr_inv32" if bp == 32 else f"k_cr_inv<{bp // 16}>")


def survey_poles(P: int, beta: float) -> int:
    """SURVEY.md §8(d)'s P(β): the distinct pole LUs, capped at 8/10/12/15
    for β = 4/8/16/32 (min(actual, cap); no cap for other β)."""
    cap = {4.0: 8, 8.0: 10, 16.0: 12, 32.0: 15}.get(float(beta))
    return min(P, cap) if cap else P


def profiled_kernel_us(kernel, L, beta, chains):
    """Mean duration (µs) and call count of `kernel` in the committed rocprofv3
    --stats summary of this exact workload's bench command, else (None, 0, None)."""
    import csv
    for path in KSTATS_FILES.get((L, float(beta), chains), []):
        try:
            with open(path) as f:
                rows = [r for r in csv.DictReader(f) if kernel + "(" in r["Name"] or r["Name"].endswith(kernel)]
        except (OSError, KeyError):
            continue
        if rows:
            calls = sum(int(r["Calls"]) for r in rows)
            tot = sum(float(r["TotalDurationNs"]) for r in rows)
            return tot / calls / 1000.0, calls, os.path.relpath(path, ROOT)
    return None, 0, None


def measured_traffic(kernel, L, beta, chains):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/pmc_summary.py: FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md
    gfx950 correction) for this exact workload, else None.  PMC counters cannot
    be read inside the timed run, so they come from their own profiled runs."""
    for path in TRAFFIC_FILES:
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        w = rec.get("workload", {})
        if (w.get("L"), w.get("beta"), w.get("chains")) != (L, beta, chains):
            continue
        # a kernel family (the block products at K split 4 and 1): launch-weighted
        names = kernel if isinstance(kernel, (list, tuple)) else [kernel]
        ks = [rec.get("kernels", {}).get(n) for n in names]
        ks = [k for k in ks if k]
        if ks:
            n = sum(k.get("launches_fetch_pass", 1) for k in ks)
            b = sum(k["hbm_bytes_per_launch"] * k.get("launches_fetch_pass", 1) for k in ks)
            return b / n, "profiles/" + os.path.basename(path)
    return None, None


def measured_mfma(kernels, L, beta, chains):
    """Executed MFMA flops and SQ_VALU_MFMA_BUSY_CYCLES per launch of a kernel
    family (launch-weighted) from the committed SQ counter pass of this
    workload, the attainable f64 MFMA rate measured beside it, and the file."""
    for path in MFMA_FILES:
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        w = rec.get("workload", {})
        if (w.get("L"), w.get("beta"), w.get("chains")) != (L, beta, chains):
            continue
        ks = [rec.get("kernels", {}).get(n.replace(" ", "")) for n in kernels]
        ks = [k for k in ks if k]
        if ks:
            n = sum(k["launches_per_step"] for k in ks)
            busy = sum(k["mfma_busy_cycles_per_launch"] * k["launches_per_step"] for k in ks) / n
            flops = sum(k["mfma_exec_flops_per_launch"] * k["launches_per_step"] for k in ks) / n
            return busy, flops, rec.get("attainable_tflops"), "profiles/" + os.path.basename(path)
    return None, None, None, None


def measured_step_mfma(L, beta, chains):
    """Executed MFMA flops per leapfrog step summed over EVERY kernel of the
    committed SQ counter pass of this workload (block products, inversions,
    side work; the sparse and bond kernels contribute zero), and the file."""
    for path in MFMA_FILES:
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        w = rec.get("workload", {})
        if (w.get("L"), w.get("beta"), w.get("chains")) != (L, beta, chains):
            continue
        ks = rec.get("kernels", {})
        if ks:
            # (the sparse level-0 kernels' names come out empty in the counter pass)
            per = {(k or "k_cr_sp_fwd+k_cr_sp_bwd"): v["mfma_exec_flops_per_launch"] * v["launches_per_step"]
                   for k, v in ks.items()}
            return sum(per.values()), per, "profiles/" + os.path.basename(path)
    return None, None, None


# BASELINE.json configs; the headline line is C3.
PRESETS = {
    "C1": dict(L=8, beta=4.0, chains=1, label="L=8 beta=4 single chain (BASELINE configs[0], C1)"),
    "C2": dict(L=16, beta=8.0, chains=1, label="L=16 beta=8 single-chain HMC (BASELINE configs[1], C2)"),
    "C3": dict(L=32, beta=16.0, chains=1, label="L=32 beta=16 single-chain HMC (BASELINE configs[2], C3)"),
    "C4": dict(L=32, beta=16.0, chains=1, label="L=32 beta=16 one disorder replica per GPU (BASELINE configs[3], C4)"),
    "C5": dict(L=48, beta=32.0, chains=4, label="L=48 beta=32 4 chains/GPU batched (BASELINE configs[4], C5)"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50, help="leapfrog steps timed (any positive count)")
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed leapfrog steps after thermalisation (rounded up to whole sweeps)")
    ap.add_argument("--config", choices=sorted(PRESETS), default=None,
                    help="BASELINE config preset (default: C3, or C4 when launched on >1 GPU)")
    ap.add_argument("--L", type=int, default=None)
    ap.add_argument("--beta", type=float, default=None)
    ap.add_argument("--chains", type=int, default=None, help="chains per GPU")
    ap.add_argument("--Nt", type=int, default=10, help="Nt_therm_init (src/Simulation.jl:38)")
    ap.add_argument("--therm", type=int, default=100,
                    help="thermalisation sweeps with the adaptive-Nt rule (src/Simulation.jl:104-130)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=0, help="oracle leapfrog steps for the CPU leg (0 = auto)")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 (L=8, beta=4) side line")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--algo", choices=["auto", "dense", "cr"], default="auto",
                    help="factorisation (include/dwhmc.h DWH_ALGO_*); auto = cyclic reduction when 2L <= 128")
    a = ap.parse_args(argv)
    if a.steps < 1 or a.warmup < 0 or a.therm < 0 or a.Nt < 1:
        ap.error("--steps must be >= 1, --warmup/--therm >= 0, --Nt >= 1")
    return a


def schedule(first: int, steps: int, Nt: int):
    """Exactly `steps` leapfrog steps as (first_draw, n_sweeps, Nt) pieces:
    steps // Nt full trajectories, then one trajectory of steps % Nt."""
    full, rem = divmod(steps, Nt)
    out = []
    if full:
        out.append((first, full, Nt))
    if rem:
        out.append((first + full, 1, rem))
    return out


def n_draws(pieces) -> int:
    return sum(n for _, n, _ in pieces)


def synthetic_state(m, p, replica, nchains):
    """Disorder and Δ₀ of `nchains` chains of one replica (src/Types.jl:118-134,
    seeded per SURVEY.md §8d)."""
    dis, D0 = [], []
    for c in range(nchains):
        st = m.initialize_state(p, np.random.default_rng(1000 + replica * nchains + c))
        dis.append(st.disorder_pot)
        D0.append(st.Delta)
    return np.stack(dis), np.stack(D0)


def synthetic_draws(m, N, replica, nchains, nsweeps, salt):
    rng = np.random.default_rng([salt, replica])
    noise = m.standard_complex_normal(rng, (nsweeps, nchains, N, 2))   # randn(ComplexF64), src/HMC.jl:53
    return noise, rng.random((nsweeps, nchains))


def thermalise(m, ctx, p, replica, nchains, n_therm, Nt0):
    """src/Simulation.jl:97-130 with injected draws; returns (Nt, acceptance
    of the last 20 sweeps).  Chains of one context share Nt (the majority
    vote of their acceptances per window)."""
    ad = m.AdaptiveNt(Nt0)
    if n_therm == 0:
        return ad.Nt, None
    noise, uni = synthetic_draws(m, p.N, replica, nchains, n_therm, 11)
    ctx.load_draws(noise, uni)
    accs = []
    for i in range(0, n_therm, ad.window):
        k = min(ad.window, n_therm - i)
        dt = m.calc_optimal_dt(p.beta, p.J, p.mass, ad.Nt)
        ctx.run_sweeps(i, k, ad.Nt, dt, p.mass)
        acc, _ = ctx.sweep_results(i, k)
        for j in range(k):
            accs.append(float(acc[j].mean()))
            ad.record(i + j + 1, accs[-1] >= 0.5)
    return ad.Nt, float(np.mean(accs[-20:]))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def blas_threads() -> int:
    try:
        from threadpoolctl import threadpool_info
        n = [i.get("num_threads", 1) for i in threadpool_info()
             if i.get("internal_api") in ("openblas", "mkl", "blis")]
        if n:
            return max(n)
    except Exception:
        pass
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def cpu_leapfrog(p_args, disorder, Delta0, steps, Nt=10):
    """The reference CPU path, restated (oracle: numpy/scipy zheevr with
    uplo='U', src/Hamiltonian.jl:96-114, compute_forces!, src/Observables.jl:14-62,
    leapfrog src/HMC.jl:101-113): returns (steps/s, seconds)."""
    from oracle import dwhmc_oracle as O      # CPU baseline leg only
    p = O.ModelParameters(*p_args)
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, disorder)
    Delta = Delta0.copy()
    pi = np.zeros_like(Delta)
    O.update_H_BdG(cache, p, Delta)
    O.diagonalize_H_BdG(cache, p)
    O.compute_forces(cache, p, Delta)
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
    t0 = time.perf_counter()
    for _ in range(steps):
        Delta += dt / (2 * p.mass) * pi
        O.update_H_BdG(cache, p, Delta)
        O.diagonalize_H_BdG(cache, p)
        O.compute_forces(cache, p, Delta)
        pi += dt * cache.forces
    el = time.perf_counter() - t0
    return steps / el, el


def cpu_baseline(p_args, disorder, Delta0, steps_all, steps_one):
    """All BLAS threads, then 1 thread (core count and CPU model stated)."""
    threads = blas_threads()
    v, el = cpu_leapfrog(p_args, disorder, Delta0, steps_all)
    rec = {"value": v, "unit": "leapfrog steps/s", "cores": threads, "kind": "port",
           "cpu": cpu_model(),
           "sample": f"{steps_all} leapfrog steps at L={p_args[0]}, beta={p_args[7]:g}, {threads} BLAS threads "
                     f"(numpy/scipy zheevr restatement of src/Hamiltonian.jl:96-114 + compute_forces!, "
                     f"{el:.1f} s)"}
    if steps_one:
        try:
            from threadpoolctl import threadpool_limits
            with threadpool_limits(limits=1):
                v1, el1 = cpu_leapfrog(p_args, disorder, Delta0, steps_one)
            rec["single_thread"] = {"value": v1, "cores": 1,
                                    "sample": f"{steps_one} leapfrog step(s), 1 thread, {el1:.1f} s"}
        except Exception as e:                  # threadpoolctl missing or BLAS not controllable
            rec["single_thread"] = {"error": repr(e)}
    return rec


def c1_line(m, local):
    """BASELINE configs[0] (C1: L=8, β=4, 10 trajectories x Nt=10 =
    scripts/test_hmc.jl's workload) on the GPU and on the CPU restatement."""
    pr = PRESETS["C1"]
    p_args = (pr["L"], pr["L"], 1.0, -0.35, -1.08, 1.0, 0.05, pr["beta"], 0.8, 1.0)
    p = m.ModelParameters(*p_args)
    dis, D0 = synthetic_state(m, p, 0, 1)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis,
                           device=local)
    ctx.set_pairing(D0)
    ctx.factorize()
    noise, uni = synthetic_draws(m, p.N, 0, 1, 12, 13)
    ctx.load_draws(noise, uni)
    dt = m.calc_optimal_dt(p.beta, p.J, p.mass, 10)
    ctx.run_sweeps(0, 2, 10, dt, p.mass)        # warmup
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.run_sweeps(2, 10, 10, dt, p.mass)
    ctx.synchronize()
    el = time.perf_counter() - t0
    acc, _ = ctx.sweep_results(2, 10)
    ctx.close()
    v_cpu, el_cpu = cpu_leapfrog(p_args, dis[0], D0[0], 100)
    return {"workload": pr["label"], "trajectories": 10, "Nt": 10, "gpu_value": 100 / el,
            "gpu_ms_per_step": 1000.0 * el / 100, "gpu_acceptance": float(acc.mean()),
            "cpu_value": v_cpu, "cpu_cores": blas_threads(), "cpu_kind": "port", "unit": "leapfrog steps/s",
            "cpu_sample": f"100 leapfrog steps (10 x Nt=10), {el_cpu:.2f} s"}


def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torch.distributed.run (the driver's multi-GPU command; also at
    # --nproc-per-node 1): the replica branch with its RCCL collectives runs
    # for any world size, so the N = 1 run exercises the same code as N = 8
    distributed = world > 1 or ("MASTER_ADDR" in os.environ and "WORLD_SIZE" in os.environ)
    preset = PRESETS[a.config or ("C4" if distributed else "C3")]
    custom = any(getattr(a, k) not in (None, preset[k]) for k in ("L", "beta", "chains"))
    for k in ("L", "beta", "chains"):
        if getattr(a, k) is None:
            setattr(a, k, preset[k])
    workload = (f"L={a.L} beta={a.beta:g} {a.chains} chain(s)/GPU (custom)" if custom else preset["label"])
    dist = None
    # DWHMC_BENCH_BACKEND=gloo: rehearsal of the multi-rank logic with ranks
    # sharing fewer GPUs (collectives on host tensors); the driver's runs use
    # the default, RCCL over xGMI with one GPU per rank
    backend = os.environ.get("DWHMC_BENCH_BACKEND", "nccl")
    tdev = "cpu"
    if distributed:
        import torch
        import torch.distributed as dist
        if backend == "gloo":
            local = local % max(1, torch.cuda.device_count())
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            tdev = f"cuda:{local}"

    import dwhmc_loader
    m = dwhmc_loader.load_package()
    m.load_library(build_if_missing=False)

    p_args = (a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    p = m.ModelParameters(*p_args)
    dis, D0 = synthetic_state(m, p, rank, a.chains)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis,
                           device=local, algo=a.algo)
    cr = ctx.info["algo"] == 1
    # dominant kernel: block products (cr) / rank-128 GJ update (dense)
    dom = "cr_gemm" if cr else "gj_update"
    ctx.set_pairing(D0)
    ctx.factorize()                                 # src/Simulation.jl:84-86
    t_th = time.perf_counter()
    Nt, acc_therm = thermalise(m, ctx, p, rank, a.chains, a.therm, a.Nt)
    t_th = time.perf_counter() - t_th
    dt = m.calc_optimal_dt(p.beta, p.J, p.mass, Nt)
    warm = schedule(0, -(-a.warmup // Nt) * Nt, Nt) if a.warmup else []
    w_sw = n_draws(warm)
    timed = schedule(w_sw, a.steps, Nt)
    noise, uni = synthetic_draws(m, p.N, rank, a.chains, w_sw + n_draws(timed), 7)
    ctx.load_draws(noise, uni)                      # inputs resident in HBM before timing
    gc_first = os.environ.get("DWHMC_BENCH_GC_FIRST", "1") != "0"
    if gc_first:
        # host housekeeping before the warmup, so the warmup runs right before
        # the timed region (no idle GPU gap between them)
        gc.collect()
        gc.disable()                                # no collector pause inside the timed region
        if dist is not None:
            dist.barrier()
    for f, n, nt in warm:
        ctx.run_sweeps(f, n, nt, dt, p.mass)
    ctx.synchronize()

    if not gc_first:
        gc.collect()
        gc.disable()
        if dist is not None:
            dist.barrier()
    elif dist is not None:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for f, n, nt in timed:
        ctx.run_sweeps(f, n, nt, dt, p.mass)
    t_enq = time.perf_counter() - t0           # host enqueue time of the timed launches
    ctx.synchronize()
    el = time.perf_counter() - t0
    gc.enable()
    el_local = el
    per_rank = None
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        dist.barrier()
        # each rank's own rate and thermalised Nt next to the max-time
        # aggregate, so a straggler (or a rank whose chain settled at a longer
        # trajectory) shows in the record
        t = torch.tensor([float(rank), a.steps * a.chains / el_local, 1000.0 * el_local / a.steps, float(Nt)],
                         dtype=torch.float64, device=tdev)
        gl = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, gl, dst=0)
        if rank == 0:
            per_rank = [{"rank": int(x[0]), "value": float(x[1]), "ms_per_step": float(x[2]), "Nt_final": int(x[3])}
                        for x in torch.stack(gl).cpu().numpy()]

    acc, dH = ctx.sweep_results(w_sw, n_draws(timed))
    info = ctx.info
    kern = {}
    replay_steps = 0
    if not a.no_timing:
        # Per-kernel HIP events (on the context's stream) in an instrumented
        # replay of the timed schedule's first <= 2 Nt steps right after the
        # timed region: each event record is a barrier packet that costs ~20 %
        # of the step when interleaved with ~30 launches per step, so the
        # timed region itself runs without them.  Same kernels, same sizes;
        # rocprofv3 --stats of the same command (profiles/) agrees on the
        # per-launch averages.
        replay = schedule(w_sw, min(a.steps, 2 * Nt), Nt)
        replay_steps = sum(n * nt for _, n, nt in replay)
        names = [dom, "assemble"] + (["cr_inv", "cr_inv_side", "cr_sparse"] if cr else [])
        ctx.timing_enable(names)
        ctx.timing_reset()
        for f, n, nt in replay:
            ctx.run_sweeps(f, n, nt, dt, p.mass)
        ctx.synchronize()
        for k in names:
            if k != "assemble":
                kern[k] = ctx.timing_read(k)
        # the assembly launch runs once per trajectory (inside one the force
        # kernel scatters the drifted Δ itself): time it over many warm
        # launches so the figure is the kernel's, not one cold launch's
        ctx.timing_enable(["assemble"])
        ctx.timing_reset()
        ctx.bench_assembly(ASSEMBLY_REPS)
        kern["assemble"] = ctx.timing_read("assemble")
        ctx.timing_enable(False)
    # observables gather over RCCL (the only collective): acceptance and <dH>
    obs = np.array([acc.mean(), dH.mean(), float(np.mean(np.exp(-dH)))], dtype=np.float64)
    if dist is not None:
        import torch
        t = torch.tensor(obs, device=tdev)
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
                       "Nt": Nt, "dt": dt, "therm_sweeps": a.therm, "poles": P, "kappa": info["kappa"],
                       "parallelism": f"replicas x{world}" if distributed else "single GPU"},
            "timed_trajectories": [{"sweeps": n, "Nt": nt} for _, n, nt in timed],
            "host_enqueue_ms": 1000.0 * t_enq,
            "warmup_sweeps": w_sw,
            "thermalisation": {"sweeps": a.therm, "Nt_init": a.Nt, "Nt_final": Nt,
                               "acceptance_last20": acc_therm, "seconds": t_th},
            "acceptance": float(obs[0]), "mean_dH": float(obs[1]), "mean_exp_minus_dH": float(obs[2]),
            "algorithm": "block cyclic reduction" if cr else "dense Schur complement + Gauss-Jordan",
            "ref_equiv_tflops": leap * (40.0 / 3.0) * (2 * N) ** 3 / el / 1e12,
            # W = P(β) · 8 n³ per step (zgetrf + zgetri of the
            # n = 2N BdG matrix per distinct pole, P capped at 8/10/12/15 for
            # β = 4/8/16/32) — a dense-LU count the CR path does not execute
            "survey_W_tflops": leap * survey_poles(P, a.beta) * 8.0 * (2 * N) ** 3 / el / 1e12,
            "survey_W_poles": survey_poles(P, a.beta),
            # the N x N Schur complement of the dense path (DWH_ALGO_DENSE), P poles
            "dense_schur_equiv_tflops": leap * P * 8.0 * N ** 3 / el / 1e12,
        }
        if distributed:
            rec["collectives"] = {"backend": dist.get_backend(), "device": tdev,
                                  "ops": ["barrier", "all_reduce(max time)", "gather(per-rank rates)",
                                          "gather(observables)"]}
            rec["per_rank"] = per_rank
        if distributed and backend == "gloo":
            rec["rehearsal"] = f"gloo collectives, {world} ranks on {torch.cuda.device_count()} GPU(s): not a scaling measurement"
        if not cr:
            rec["alg_tflops"] = rec["dense_schur_equiv_tflops"]
        if kern:
            ms, n, w = kern[dom]
            ach = w / n / (ms / n * 1e-3) / 1e12 if n and ms > 0 else None
            if cr:
                # 16x16 tiles, 4-way K split below 2048 tiles per stage, none from there
                # (cr_gemm_config): one timer family, two rocprofv3 rows
                kname = f"k_cr_gemm<{info['block']},1,4|1>"
                kfam = [f"k_cr_gemm<{info['block']},1,4>", f"k_cr_gemm<{info['block']},1,1>"]
                msi, ni, wi = kern["cr_inv"]
                mss, ns, ws = kern["cr_inv_side"]
                msp, nsp, wsp = kern["cr_sparse"]
                # the CR path's own algorithmic flops per leapfrog step (block
                # products, incl. the side work of the inversion stages, the
                # sparse level-0 products, and block inversions at 8 BP^3
                # each) x the timed steps
                wall = w + wi + ws + wsp
                rec["alg_tflops"] = wall / replay_steps * a.steps * world / el / 1e12
                rec["alg_flops_per_step"] = wall / replay_steps / a.chains
                # the whole leapfrog step against the fp64 MFMA peak (north_star: >= 0.30 at L=32)
                rec["alg_frac_of_peak"] = rec["alg_tflops"] / world / PEAK_F64_TFLOPS
                nt = info["block"] // 16
                rec["cr_inv"] = {"bound": "latency", "kernel": inv_kernels(info["block"], ni > replay_steps),
                                 "launches_per_step": ni / replay_steps,
                                 "achieved_tflops": wi / (msi * 1e-3) / 1e12 if msi > 0 else None,
                                 "avg_launch_us": 1000.0 * msi / ni if ni else None,
                                 "ms_per_step": msi / replay_steps}
                if nsp:
                    rec["cr_sparse"] = {"bound": "latency", "kernel": "k_cr_sp_fwd + k_cr_sp_bwd",
                                        "what": "level-0 products with the sparse U / L blocks (VALU)",
                                        "launches_per_step": nsp / replay_steps,
                                        "avg_launch_us": 1000.0 * msp / nsp,
                                        "flops_per_launch": wsp / nsp,
                                        "ms_per_step": msp / replay_steps}
                if ns:
                    rec["cr_inv_side"] = {"bound": "latency", "kernel": f"k_cr_inv_side<{nt}>",
                                          "what": "block inversions + off-critical-path block products "
                                                  "on the CUs the inversions leave idle",
                                          "launches_per_step": ns / replay_steps,
                                          "avg_launch_us": 1000.0 * mss / ns,
                                          "flops_per_launch": ws / ns,
                                          "ms_per_step": mss / replay_steps}
            else:
                nb = -(-info["N"] // 64)                 # GJ block steps; odd nb ends with one rank-64 step
                kname = "k_gj_update<2>" if nb % 2 == 0 else "k_gj_update<2>+<0>"
            traffic, tsrc = measured_traffic(kfam if cr else kname, a.L, a.beta, a.chains)
            rec["roofline"] = {"bound": "mfma", "kernel": kname, "achieved": ach,
                               "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                               "frac": ach / PEAK_F64_TFLOPS if ach else None, "traffic": traffic,
                               "traffic_unit": "bytes/launch", "traffic_source": tsrc,
                               "avg_launch_us": 1000.0 * ms / n if n else None,
                               "flops_per_launch": w / n if n else None,
                               "replayed_steps": replay_steps}
            # hardware view from the SQ counters of the same workload: the
            # MFMA pipe's busy cycles per launch over the launch's duration
            # (this run's HIP events) x 1024 SIMDs at the peak's clock, and the
            # executed MFMA flops (3-multiplication complex MACs: 6 of every 8
            # counted flops) against the peak and the attainable f64 MFMA rate
            busy, xfl, att, msrc = measured_mfma(kfam if cr else [kname], a.L, a.beta, a.chains)
            if busy is not None and n and ms > 0:
                dur = ms / n * 1e-3
                rf = rec["roofline"]
                rf["mfma_busy_frac"] = busy / (dur * CLOCK_GHZ * 1e9 * 1024)
                rf["hw_frac"] = xfl / dur / 1e12 / PEAK_F64_TFLOPS
                rf["hw_flops_per_launch"] = xfl
                rf["hw_over_alg_flops"] = xfl / (w / n) if w else None
                rf["attainable_peak"] = att
                rf["hw_frac_of_attainable"] = xfl / dur / 1e12 / att if att else None
                rf["mfma_source"] = msrc
            if cr:
                # the whole step in executed-MFMA terms: every MFMA kernel's SQ
                # summary (not only the product family) over this run's time per step
                sfl, sper, ssrc = measured_step_mfma(a.L, a.beta, a.chains)
                if sfl is not None:
                    rec["step_hw_frac"] = sfl / (ms_per_step * 1e-3) / 1e12 / PEAK_F64_TFLOPS
                    rec["step_hw"] = {"mfma_exec_flops_per_step": sfl, "per_kernel": sper, "source": ssrc,
                                      "what": "executed MFMA flops per step (SQ_VALU_MFMA_BUSY_CYCLES of every "
                                              "kernel) / ms_per_step / peak"}
            rec[f"{dom}_ms_per_step"] = ms / replay_steps
            ms, n, w = kern["assemble"]
            if n and ms > 0:
                akern = "k_cr_fill" if cr else "k_assemble"
                us = 1000.0 * ms / n
                gbs = w / n / (us * 1e-6) / 1e9
                # this run's HIP-event figure is the rate; the committed rocprofv3
                # mean of the same command (a HIP event pair around a 2-3 µs
                # launch adds its own packet time) is reported beside it, named
                pr_us, pr_calls, pr_src = profiled_kernel_us(akern, a.L, a.beta, a.chains)
                rec["assembly"] = {"bound": "hbm", "kernel": akern,
                                   "achieved": gbs,
                                   "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                                   "bytes_per_launch": w / n, "avg_launch_us": us,
                                   "avg_source": "this run's HIP events per launch",
                                   "launches_timed": n,
                                   "profiled_avg_launch_us": pr_us,
                                   "profiled_source": (f"{pr_src} (rocprofv3 --stats mean over {pr_calls} launches, "
                                                       "committed profile, not this run)" if pr_us else None),
                                   "what": f"{ASSEMBLY_REPS} back-to-back warm launches (dwh_bench_assembly) "
                                           "after the timed region"}
        if world == 1 and not a.no_c1 and a.L != PRESETS["C1"]["L"]:
            rec["c1"] = c1_line(m, local)
        if not a.no_cpu_baseline and world == 1:
            steps_all = a.cpu_steps or (1 if a.L >= 48 else 3 if a.L >= 32 else 20)
            steps_one = 0 if a.L >= 48 else 1 if a.L >= 32 else 5
            rec["cpu_baseline"] = cpu_baseline(p_args, dis[0], D0[0], steps_all, steps_one)
        print(json.dumps(rec), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
