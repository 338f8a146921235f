"""Replica path on CPU: world_size-2 gloo process group, one fake device
context per rank (the HIP context needs a GPU; the distributed logic under
test — seeding, per-sweep records, the rank-0 gather, the CSV format — does
not).  The same gather runs over RCCL in bench.py on MI355X."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeContext:
    def __init__(self, disorder):
        self.dis = disorder
        self.nchains, self.N = disorder.shape

    def set_pairing(self, D):
        self.D = np.array(D, dtype=complex)

    def factorize(self):
        pass

    def hmc_sweep(self, noise, uni, Nt, dt, mass):
        self.D = self.D + 0.01 * noise + 0.001 * self.dis[:, :, None]
        return uni < 0.5, np.real(noise).sum(axis=(1, 2))

    def get_state(self):
        return self.D, np.zeros_like(self.D)

    def pairing(self):
        return 0.5 * self.D

    def fermion_energy(self):
        return -np.abs(self.D).sum(axis=(1, 2))

    def hole_trace(self):
        return np.full(self.nchains, 0.4 * self.N)

    def measure_transport_all(self, eta, domega, omega_max):
        return [dict(superfluid_stiffness=float(np.abs(self.D[c]).sum()),
                     dc_conductivity=float(self.dis[c].sum() + eta)) for c in range(self.nchains)]

    def close(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _local(rank):
    import dwhmc_loader
    m = dwhmc_loader.load_package()
    from importlib import import_module
    rep = import_module(m.__name__ + ".replicas")
    p = m.ModelParameters(4, 4, 1.0, -0.35, -1.08, 1.0, 0.25, 4.0, 0.8, 1.0)
    cfg = rep.ReplicaConfig(chains=2, n_sweeps=3, Nt=2, transport_freq=2)
    tr = []
    obs = rep.run_local(p, cfg, rank, 0, FakeContext, m.initialize_state, m.calc_optimal_dt, transport_out=tr)
    rep._test_transport = np.stack(tr)
    return rep, obs


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rep, local = _local(rank)
    rec = rep.gather_observables(local, dist)
    trec = rep.gather_observables(rep._test_transport, dist)
    if rank == 0:
        np.save(out, rec)
        np.save(out + ".tr.npy", trec)
        rep.write_observables_csv(out + ".csv", rec)
        rep.write_transport_csv(out + ".tr.csv", trec)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_matches_sequential(tmp_path):
    out = str(tmp_path / "rec.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    rec = np.load(out)
    rep, l0 = _local(0)
    _, l1 = _local(1)
    expect = np.concatenate([np.transpose(l0, (1, 0, 2)), np.transpose(l1, (1, 0, 2))], axis=0)
    assert rec.shape == (4, 3, rep.N_OBS)
    assert np.array_equal(rec, expect)
    # replicas are independent realisations: different seeds -> different records
    assert not np.array_equal(rec[0], rec[2])
    lines = open(out + ".csv").read().splitlines()
    assert lines[0].startswith("Replica,Sweep,Accepted,dH,Energy")
    assert len(lines) == 1 + 4 * 3
    # transport every 2 sweeps of 3 -> one measurement per chain, gathered the same way
    trec = np.load(out + ".tr.npy")
    _local(0)
    t0 = rep._test_transport
    assert trec.shape == (4, 1, rep.N_TR)
    assert np.array_equal(trec[:2], np.transpose(t0, (1, 0, 2)))
    assert np.all(trec[:, 0, 0] == 2)
    tl = open(out + ".tr.csv").read().splitlines()
    assert tl[0] == "Replica,Sweep,Superfluid_Stiffness,DC_Conductivity" and len(tl) == 5


def test_observables_from_outputs_matches_oracle(oracle, dwhmc):
    """The on-device observable formula (P, E_f, Tr ρ_hh) equals the oracle's
    eigenvector-based measure_observables (src/Observables.jl:88-222)."""
    from importlib import import_module
    rep = import_module(dwhmc.__name__ + ".replicas")
    O = oracle
    p = O.ModelParameters(6, 6, 1.0, -0.35, -1.08, 1.0, 0.05, 8.0, 0.8, 1.0)
    st = O.initialize_state(p, np.random.default_rng(3))
    D = st.Delta + 0.2 * np.stack([np.ones(p.N), -np.ones(p.N)], 1)
    cache, F, Ef = O.evaluate(p, st.disorder_pot, D)
    P, f = O.pairing_P(cache.U, cache.E_n, p)
    rho_hh = np.einsum("in,n,in->", cache.U[p.N:], f, cache.U[p.N:].conj()).real
    vals = rep.observables_from_outputs(p, D, P, Ef, rho_hh)
    ref = O.measure_observables(cache, p, D)
    for v, k in zip(vals, O.OBS_FIELDS):
        assert abs(v - ref[k]) < 1e-10 * (1 + abs(ref[k])), k
