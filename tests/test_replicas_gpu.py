"""Replicas with real device contexts (independent disorder
realisations one per rank, a collective only to gather observables), on the
one-GPU box: two ranks share the GPU and gather over gloo, the same code path
bench.py and replicas.py run one rank per GPU over RCCL (tests/test_replicas_gloo.py
covers the gather on CPU with a fake context).  Not a scaling measurement:
two processes on one GPU."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _local(rank, transport_out=None):
    sys.path.insert(0, ROOT)
    import dwhmc_loader
    from importlib import import_module
    m = dwhmc_loader.load_package()
    rep = import_module(m.__name__ + ".replicas")
    p = m.ModelParameters(6, 6, 1.0, -0.35, -1.08, 1.0, 0.05, 8.0, 0.8, 1.0)
    cfg = rep.ReplicaConfig(chains=2, n_sweeps=3, Nt=4, transport_freq=3)

    def make(dis):
        return m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis, device=0)

    obs = rep.run_local(p, cfg, rank, 0, make, m.initialize_state, m.calc_optimal_dt, transport_out=transport_out)
    return rep, obs


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = []
    rep, local = _local(rank, tr)
    rec = rep.gather_observables(local, dist)
    trec = rep.gather_observables(np.stack(tr), dist)
    if rank == 0:
        np.save(out, rec)
        np.save(out + ".tr.npy", trec)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_replicas_real_contexts(tmp_path):
    """Two ranks, each with its own device context and disorder seeds: the
    rank-0 gather equals each replica run alone in this process, bit for bit
    (the HIP path is deterministic), and the replicas differ."""
    out = str(tmp_path / "rec.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    rec = np.load(out)
    trec = np.load(out + ".tr.npy")
    t0, t1 = [], []
    rep, l0 = _local(0, t0)
    _, l1 = _local(1, t1)
    expect = np.concatenate([np.transpose(l0, (1, 0, 2)), np.transpose(l1, (1, 0, 2))], axis=0)
    assert rec.shape == (4, 3, rep.N_OBS)
    assert np.array_equal(rec, expect)
    assert not np.array_equal(rec[0], rec[2])
    texp = np.concatenate([np.transpose(np.stack(t0), (1, 0, 2)), np.transpose(np.stack(t1), (1, 0, 2))], axis=0)
    assert np.array_equal(trec, texp)


def test_bench_two_ranks_gloo(tmp_path):
    """bench.py under torch.distributed.run with two ranks on the one GPU
    (DWHMC_BENCH_BACKEND=gloo, the driver's launch shape): one JSON line from
    rank 0 with n_gpus = 2, the whole-job rate and the rehearsal note."""
    env = dict(os.environ, DWHMC_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "8", "--warmup", "2", "--L", "8", "--beta", "4", "--therm", "10",
           "--no-cpu-baseline", "--no-c1", "--no-timing"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 8 and rec["value"] > 0
    assert "rehearsal" in rec and 0.0 <= rec["acceptance"] <= 1.0
    assert rec["config"]["parallelism"] == "replicas x2"


def _rccl_worker(rank, world, port, out):
    """One rank, RCCL (backend nccl) bound to the GPU: the replicas' observable
    gather on device tensors, as replicas.py / tools/run_replicas.py run it per GPU."""
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    tr = []
    rep, local = _local(rank, tr)
    rec = rep.gather_observables(local, dist, device=dev)
    trec = rep.gather_observables(np.stack(tr), dist, device=dev)
    t = torch.tensor([1.0 + rank], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    np.save(out, rec)
    np.save(out + ".tr.npy", trec)
    np.save(out + ".max.npy", t.cpu().numpy())
    dist.barrier()
    backend = dist.get_backend()
    dist.destroy_process_group()
    assert backend == "nccl"


def test_rccl_gather_world1(tmp_path):
    """The RCCL branch at world size 1 (the first execution of the collective
    the 8-GPU replica run uses): init_process_group("nccl", device_id=GPU),
    gather_observables on device tensors, the max all_reduce — the gathered
    records equal the replica run alone, bit for bit."""
    out = str(tmp_path / "rec.npy")
    mp.spawn(_rccl_worker, args=(1, _free_port(), out), nprocs=1, join=True)
    rec = np.load(out)
    t0 = []
    rep, l0 = _local(0, t0)
    assert np.array_equal(rec, np.transpose(l0, (1, 0, 2)))
    assert np.array_equal(np.load(out + ".tr.npy"), np.transpose(np.stack(t0), (1, 0, 2)))
    assert float(np.load(out + ".max.npy")[0]) == 1.0


def _bench(args, env_extra=None, torchrun=False):
    env = dict(os.environ, **(env_extra or {}))
    env.pop("DWHMC_BENCH_BACKEND", None)
    cmd = [sys.executable]
    if torchrun:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
                "--master-port", str(_free_port())]
    cmd += [os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_rccl_world1_matches_plain():
    """The driver's multi-GPU command shape at --nproc-per-node 1 with the
    default backend (RCCL over the rank's GPU): the replica branch runs —
    nccl init with device_id, the max-time all_reduce and the observable
    gather on device tensors — on the same workload as the plain run, with the
    per-rank rates gathered next to the max-time aggregate."""
    args = ["--gpus", "1", "--steps", "40", "--warmup", "5", "--no-cpu-baseline", "--no-c1", "--no-timing"]
    plain = _bench(args)
    rec = _bench(args, torchrun=True)
    assert rec["n_gpus"] == 1 and rec["config"]["parallelism"] == "replicas x1"
    assert rec["collectives"]["backend"] == "nccl" and rec["collectives"]["device"] == "cuda:0"
    assert "rehearsal" not in rec
    assert plain["config"]["parallelism"] == "single GPU"
    assert rec["config"]["L"] == plain["config"]["L"] == 32 and rec["config"]["poles"] == plain["config"]["poles"]
    pr = rec["per_rank"]
    assert [r["rank"] for r in pr] == [0] and pr[0]["Nt_final"] == rec["config"]["Nt"]
    # one rank: its own rate is the aggregate (the max time is its time)
    assert abs(pr[0]["value"] / rec["value"] - 1.0) < 1e-9 and pr[0]["ms_per_step"] > 0
    # the throughput itself is logged, not asserted (run-to-run spread on the box)
    print("rccl world-1", rec["value"], "plain", plain["value"])
