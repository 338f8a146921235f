#!/usr/bin/env python3
"""Disorder replicas, one process per GPU (BASELINE config C4):

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29511 tools/run_replicas.py --L 32 --beta 16 --sweeps 20 --out runs/c4

Each rank owns `--chains` chains (seed 1000 + rank*chains + chain, the bench's
convention) on its own device; the hot path has no collective.  After the
sweeps the 11 per-sweep fp64 records of every chain are gathered to rank 0
over the process group (RCCL on MI355X; gloo when no GPU is visible) and
written as observables.csv with a Replica column.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--beta", type=float, default=16.0)
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("--sweeps", type=int, default=10)
    ap.add_argument("--Nt", type=int, default=10)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--transport-freq", type=int, default=0,
                    help="measure transport every k sweeps (0: never) -> transport.csv")
    ap.add_argument("--out", default="runs/replicas")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    import dwhmc_loader
    from importlib import import_module

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    m = dwhmc_loader.load_package()
    rep = import_module(m.__name__ + ".replicas")
    device = None
    # under torch.distributed.run (any world size, also --nproc-per-node 1) the
    # RCCL group runs, so one GPU exercises the collective path of eight
    distributed = world > 1 or "MASTER_ADDR" in os.environ
    if distributed:
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    p = m.ModelParameters(a.L, a.L, 1.0, -0.35, -1.08, 1.0, 0.05, a.beta, 0.8, 1.0)
    cfg = rep.ReplicaConfig(chains=a.chains, n_sweeps=a.sweeps, Nt=a.Nt, seed=a.seed,
                            transport_freq=a.transport_freq)

    def make_context(disorder):
        return m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                                disorder, device=local)

    tr_local = []
    local_rec = rep.run_local(p, cfg, rank, local, make_context, m.initialize_state, m.calc_optimal_dt,
                              transport_out=tr_local)
    allrec = rep.gather_observables(local_rec, dist if distributed else None, device)
    alltr = None
    if tr_local:
        import numpy as np
        alltr = rep.gather_observables(np.stack(tr_local), dist if distributed else None, device)
    if rank == 0:
        os.makedirs(a.out, exist_ok=True)
        path = os.path.join(a.out, "observables.csv")
        rep.write_observables_csv(path, allrec)
        print(f"{allrec.shape[0]} replica chains x {allrec.shape[1]} sweeps -> {path}", flush=True)
        if alltr is not None:
            rep.write_transport_csv(os.path.join(a.out, "transport.csv"), alltr)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
