"""Test infrastructure: the FermionContext API implemented on the CPU oracle
(oracle/dwhmc_oracle.py, LAPACK zheevr).  Lets the host-side drivers
(hmc.py, simulation.py, replicas.py) run on CPU in `-m "not gpu"` tests and
serves as the reference side of device-vs-oracle driver comparisons.  Never
used by the product path."""
from __future__ import annotations

import dataclasses

import numpy as np

from oracle import dwhmc_oracle as O


class OracleContext:
    def __init__(self, Lx, Ly, t, tp, mu, beta, J, nn_table, nnn_table, disorder,
                 delta_cap: float = 2.0, device: int = 0, lib_path=None):
        self.dis = np.atleast_2d(np.asarray(disorder, dtype=np.float64))
        self.nchains = self.dis.shape[0]
        self.p = O.ModelParameters(int(Lx), int(Ly), t, tp, mu, 0.0, 0.0, beta, J, 1.0)
        assert np.array_equal(self.p.nn_table, np.asarray(nn_table))
        assert np.array_equal(self.p.nnn_table, np.asarray(nnn_table))
        self.N = self.p.N
        self.caches = []
        for c in range(self.nchains):
            cache = O.initialize_cache(self.p)
            O.init_static_H(cache, self.p, self.dis[c])
            self.caches.append(cache)
        self.Delta = np.zeros((self.nchains, self.N, 2), dtype=np.complex128)
        self.pi = np.zeros_like(self.Delta)
        self.info = {"N": self.N, "npoles": 0}

    def _chains(self, a):
        a = np.asarray(a, dtype=np.complex128)
        return a[None] if a.ndim == 2 else a

    def set_pairing(self, Delta):
        self.Delta = self._chains(Delta).copy()
        for c, cache in enumerate(self.caches):
            O.update_H_BdG(cache, self.p, self.Delta[c])

    def factorize(self):
        for cache in self.caches:
            O.diagonalize_H_BdG(cache, self.p)

    def forces(self, Delta=None):
        D = self.Delta if Delta is None else self._chains(Delta)
        out = []
        for c, cache in enumerate(self.caches):
            O.compute_forces(cache, self.p, D[c])
            out.append(cache.forces.copy())
        return np.stack(out)

    def pairing(self):
        return np.stack([O.pairing_P(c.U, c.E_n, self.p)[0] for c in self.caches])

    def fermion_energy(self):
        return np.array([O.fermion_energy(c.E_n, self.p.beta) for c in self.caches])

    def hole_trace(self):
        return np.array([(O.measure_observables(c, self.p, self.Delta[i])["hole_conc"] + 1.0) * self.N / 2
                         for i, c in enumerate(self.caches)])

    def total_energy(self, mass):
        p = dataclasses.replace(self.p, mass=mass)
        return np.array([O.compute_total_energy(c, p, self.Delta[i], self.pi[i])
                         for i, c in enumerate(self.caches)])

    def set_state(self, Delta=None, pi=None):
        if Delta is not None:
            self.Delta = self._chains(Delta).copy()
        if pi is not None:
            self.pi = self._chains(pi).copy()

    def get_state(self):
        return self.Delta.copy(), self.pi.copy()

    def measure_transport(self, eta, domega, omega_max, chain=0):
        p = dataclasses.replace(self.p, eta=eta, domega=domega, omega_max=omega_max)
        cache = self.caches[chain]
        O.update_H_BdG(cache, p, self.Delta[chain])
        O.diagonalize_H_BdG(cache, p)
        O.compute_forces(cache, p, self.Delta[chain])      # fermi_factors
        return O.measure_transport_and_spectra(cache, p)

    def measure_transport_deltas(self, deltas, eta, domega, omega_max, chain=0):
        keep = self.Delta[chain].copy()
        out = []
        for D in np.asarray(deltas):
            self.Delta[chain] = D
            out.append(dict(self.measure_transport(eta, domega, omega_max, chain=chain)))
        self.Delta[chain] = keep
        return out

    def measure_transport_all(self, eta, domega, omega_max):
        out = []
        for c in range(self.nchains):
            out.append(dict(self.measure_transport(eta, domega, omega_max, chain=c)))
        return out

    def hmc_sweep(self, noise, uniform, Nt, dt, mass):
        p = dataclasses.replace(self.p, mass=mass)
        noise = self._chains(noise)
        u = np.atleast_1d(np.asarray(uniform, dtype=np.float64))
        acc = np.zeros(self.nchains, dtype=bool)
        dH = np.zeros(self.nchains)
        for c, cache in enumerate(self.caches):
            st = O.SimulationState(self.dis[c], self.Delta[c].copy(), self.pi[c].copy())
            acc[c], dH[c] = O.hmc_sweep(cache, p, st, Nt, dt, noise[c], float(u[c]))
            self.Delta[c] = st.Delta
            self.pi[c] = st.pi
        return acc, dH

    def hmc_trajectory(self, noise, Nt, dt, mass):
        """dwh_hmc_trajectory: the sweep with the Metropolis decision deferred
        (run accepted, the pre-trajectory state kept for hmc_finish)."""
        self._backup = [(self.Delta[c].copy(), cache.E_n.copy(), cache.U.copy())
                        for c, cache in enumerate(self.caches)]
        _, dH = self.hmc_sweep(noise, np.full(self.nchains, -1.0), Nt, dt, mass)
        return dH

    def hmc_finish(self, accepted):
        acc = np.atleast_1d(np.asarray(accepted)).astype(bool)
        for c, cache in enumerate(self.caches):
            if not acc[c]:                                   # src/HMC.jl:130-141
                D, E, U = self._backup[c]
                self.Delta[c] = D
                cache.E_n[:] = E
                cache.U[:, :] = U
                O.update_H_BdG(cache, self.p, self.Delta[c])
        self._backup = None

    def close(self):
        pass
