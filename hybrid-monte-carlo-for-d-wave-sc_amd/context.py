"""FermionContext: a typed handle on one dwh_ctx (batched over chains).

Array conventions on the Python side follow the reference's Julia indexing:
per chain a bond field is (N, 2) with column 0 = +x, 1 = +y
(src/Types.jl:106-111); batched fields are (nchains, N, 2).  They are
converted to the ABI's column-major layout here and nowhere else.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr


def _to_abi(a: np.ndarray, nc: int, N: int) -> np.ndarray:
    a = np.asarray(a, dtype=np.complex128)
    if a.shape == (N, 2):
        a = a[None]
    if a.shape != (nc, N, 2):
        raise ValueError(f"expected bond field of shape ({nc}, {N}, 2) or ({N}, 2), got {a.shape}")
    return np.ascontiguousarray(np.transpose(a, (0, 2, 1)))


def _from_abi(a: np.ndarray, nc: int, N: int) -> np.ndarray:
    return np.ascontiguousarray(np.transpose(a.reshape(nc, 2, N), (0, 2, 1)))


def table_to_abi(table: np.ndarray) -> np.ndarray:
    """(N, 4) 1-based Int table -> Julia column-major N x 4 Int64 buffer."""
    t = np.asarray(table)
    if t.ndim != 2 or t.shape[1] != 4:
        raise ValueError("neighbour table must be (N, 4)")
    return np.ascontiguousarray(t.T, dtype=np.int64)


# factorisation algorithm (include/dwhmc.h DWH_ALGO_*): "auto" = env DWHMC_ALGO,
# else block cyclic reduction when 2 Lx <= 128, eigendecomposition ("eig") when
# β·E'/2 is beyond the pole table
ALGOS = {"auto": -1, "dense": 0, "cr": 1, "eig": 2}


class FermionContext:
    """Device-resident fermionic action/force evaluator for nchains chains.
    delta_cap <= 0 selects the ABI default for the guard (bond guard on
    max|Δ_ij|: max(2, 6 sqrt(2J/β)); site guard on the mean |Δ| of a site's
    4 bonds, CR path: max(1.25, 4 sqrt(2J/β)))
    on max|Δ_ij|; an uploaded Δ or a trajectory beyond it re-selects the pole
    set (include/dwhmc.h)."""

    def __init__(self, Lx, Ly, t, tp, mu, beta, J, nn_table, nnn_table, disorder,
                 delta_cap: float = 0.0, device: int = 0, lib_path: str | None = None,
                 algo: str = "auto"):
        self._lib = _lib.load() if lib_path is None else _lib.load_path(lib_path)
        dis = np.ascontiguousarray(np.atleast_2d(np.asarray(disorder, dtype=np.float64)))
        self.N = int(Lx) * int(Ly)
        if dis.shape[1] != self.N:
            raise ValueError(f"disorder must have N={self.N} entries per chain")
        self.nchains = dis.shape[0]
        self.beta, self.J = float(beta), float(J)
        h = C.c_void_p()
        nn = table_to_abi(nn_table)
        nnn = table_to_abi(nnn_table)
        if algo not in ALGOS:
            raise ValueError(f"algo must be one of {sorted(ALGOS)}")
        rc = self._lib.dwh_create_ex(C.byref(h), int(Lx), int(Ly), float(t), float(tp),
                                     float(mu), float(beta), float(J), ptr(nn), ptr(nnn),
                                     self.nchains, ptr(dis), float(delta_cap), ALGOS[algo],
                                     int(device))
        check(rc, None)
        self._h = h
        self.info_lattice = (int(Lx), int(Ly))

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.dwh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc):
        check(rc, self._h)

    @property
    def info(self) -> dict:
        """dwh_info: sizes, pole set (kappa, npoles, delta_cap; a guard trip
        re-selects it), algorithm, device bytes."""
        return self._info()

    def _info(self):
        inf = _lib.dwh_info_t()
        self._c(self._lib.dwh_info(self._h, C.byref(inf)))
        return {k: getattr(inf, k) for k, _ in inf._fields_}

    # -- hot path --------------------------------------------------------
    def set_pairing(self, Delta):
        a = _to_abi(Delta, self.nchains, self.N)
        self._c(self._lib.dwh_update_pairing(self._h, ptr(a)))

    def factorize(self):
        self._c(self._lib.dwh_factorize(self._h))

    def forces(self, Delta=None) -> np.ndarray:
        d = None if Delta is None else _to_abi(Delta, self.nchains, self.N)
        out = np.empty((self.nchains, 2, self.N), dtype=np.complex128)
        self._c(self._lib.dwh_forces(self._h, ptr(d), ptr(out)))
        return _from_abi(out, self.nchains, self.N)

    def pairing(self) -> np.ndarray:
        out = np.empty((self.nchains, 2, self.N), dtype=np.complex128)
        self._c(self._lib.dwh_pairing(self._h, ptr(out)))
        return _from_abi(out, self.nchains, self.N)

    def fermion_energy(self) -> np.ndarray:
        out = np.empty(self.nchains)
        self._c(self._lib.dwh_fermion_energy(self._h, ptr(out)))
        return out

    def hole_trace(self) -> np.ndarray:
        out = np.empty(self.nchains)
        self._c(self._lib.dwh_hole_trace(self._h, ptr(out)))
        return out

    def total_energy(self, mass: float) -> np.ndarray:
        out = np.empty(self.nchains)
        self._c(self._lib.dwh_total_energy(self._h, float(mass), ptr(out)))
        return out

    def set_state(self, Delta=None, pi=None):
        d = None if Delta is None else _to_abi(Delta, self.nchains, self.N)
        p = None if pi is None else _to_abi(pi, self.nchains, self.N)
        self._c(self._lib.dwh_set_state(self._h, ptr(d), ptr(p)))

    def get_state(self):
        d = np.empty((self.nchains, 2, self.N), dtype=np.complex128)
        p = np.empty_like(d)
        self._c(self._lib.dwh_get_state(self._h, ptr(d), ptr(p)))
        return _from_abi(d, self.nchains, self.N), _from_abi(p, self.nchains, self.N)

    def hmc_sweep(self, noise, uniform, Nt: int, dt: float, mass: float):
        nz = _to_abi(noise, self.nchains, self.N)
        u = np.ascontiguousarray(np.atleast_1d(np.asarray(uniform, dtype=np.float64)))
        if u.shape != (self.nchains,):
            raise ValueError("one uniform per chain")
        acc = np.zeros(self.nchains, dtype=np.uint8)
        dH = np.zeros(self.nchains)
        self._c(self._lib.dwh_hmc_sweep(self._h, ptr(nz), ptr(u), int(Nt), float(dt), float(mass),
                                        ptr(acc), ptr(dH)))
        return acc.astype(bool), dH

    def hmc_trajectory(self, noise, Nt: int, dt: float, mass: float) -> np.ndarray:
        """hmc_sweep! up to H_new (dwh_hmc_trajectory); returns ΔH per chain.
        Finish with hmc_finish(accepted)."""
        nz = _to_abi(noise, self.nchains, self.N)
        dH = np.zeros(self.nchains)
        self._c(self._lib.dwh_hmc_trajectory(self._h, ptr(nz), int(Nt), float(dt), float(mass), ptr(dH)))
        return dH

    def hmc_finish(self, accepted):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(accepted)).astype(np.uint8))
        if a.shape != (self.nchains,):
            raise ValueError("one accept flag per chain")
        self._c(self._lib.dwh_hmc_finish(self._h, ptr(a)))

    # -- throughput path -------------------------------------------------
    def load_draws(self, noise, uniform):
        noise = np.asarray(noise, dtype=np.complex128)
        ns = noise.shape[0]
        nz = np.ascontiguousarray(np.transpose(noise.reshape(ns, self.nchains, self.N, 2), (0, 1, 3, 2)))
        u = np.ascontiguousarray(np.asarray(uniform, dtype=np.float64).reshape(ns, self.nchains))
        self._c(self._lib.dwh_load_draws(self._h, ns, ptr(nz), ptr(u)))

    def run_sweeps(self, first: int, nsweeps: int, Nt: int, dt: float, mass: float):
        self._c(self._lib.dwh_run_sweeps(self._h, int(first), int(nsweeps), int(Nt), float(dt),
                                         float(mass)))

    def sweep_results(self, first: int, nsweeps: int):
        acc = np.zeros((nsweeps, self.nchains), dtype=np.uint8)
        dH = np.zeros((nsweeps, self.nchains))
        self._c(self._lib.dwh_sweep_results(self._h, int(first), int(nsweeps), ptr(acc), ptr(dH)))
        return acc.astype(bool), dH

    def synchronize(self):
        self._c(self._lib.dwh_synchronize(self._h))

    def stream(self) -> int:
        s = C.c_void_p()
        self._c(self._lib.dwh_stream(self._h, C.byref(s)))
        return s.value or 0

    # -- measurement path (eigenpairs, transport / spectra) ---------------
    def eigensystem(self, chain: int = 0, vectors: bool = True):
        """(E, U) of H_BdG at the device Δ of `chain` (dwh_eigensystem):
        E ascending (2N,), U (2N, 2N) with eigenvectors in columns."""
        n2 = 2 * self.N
        E = np.empty(n2)
        Ucm = np.empty((n2, n2), dtype=np.complex128) if vectors else None   # row c = column c of U
        self._c(self._lib.dwh_eigensystem(self._h, int(chain), ptr(E), ptr(Ucm)))
        return E, (None if Ucm is None else Ucm.T)

    def measure_transport(self, eta: float, domega: float, omega_max: float, chain: int = 0) -> dict:
        """measure_transport_and_spectra (src/Observables.jl:314-526) for one
        chain at the device Δ; keys are the SpectrumResult fields
        (:293-308), A_k_omega0 indexed [kx, ky]."""
        nw, nd = transport_grid(eta, domega, omega_max, self._lib)
        Lx, Ly = self.info_lattice
        st, dc = C.c_double(), C.c_double()
        sigma, dos, dos_an = np.empty(nw), np.empty(nd), np.empty(nd)
        ak = np.empty(Lx * Ly)
        self._c(self._lib.dwh_measure_transport(self._h, int(chain), float(eta), float(domega),
                                                float(omega_max), C.byref(st), C.byref(dc), ptr(sigma),
                                                nw, ptr(dos), ptr(dos_an), nd, ptr(ak)))
        return dict(superfluid_stiffness=st.value, dc_conductivity=dc.value,
                    omega_grid=eta + domega * np.arange(nw), optical_conductivity=sigma,
                    dos_omega_grid=-omega_max + domega * np.arange(nd), dos=dos, dos_AN=dos_an,
                    A_k_omega0=ak.reshape(Ly, Lx).T.copy())

    def measure_transport_all(self, eta: float, domega: float, omega_max: float) -> list:
        """measure_transport for every chain, the eigensolves and J_mn
        products batched (dwh_measure_transport_batched); one dict per chain."""
        nw, nd = transport_grid(eta, domega, omega_max, self._lib)
        Lx, Ly = self.info_lattice
        nc = self.nchains
        st, dc = np.empty(nc), np.empty(nc)
        sigma, dos, dos_an = np.empty((nc, nw)), np.empty((nc, nd)), np.empty((nc, nd))
        ak = np.empty((nc, Lx * Ly))
        self._c(self._lib.dwh_measure_transport_batched(self._h, float(eta), float(domega), float(omega_max),
                                                        ptr(st), ptr(dc), ptr(sigma), nw, ptr(dos),
                                                        ptr(dos_an), nd, ptr(ak)))
        wg, dg = eta + domega * np.arange(nw), -omega_max + domega * np.arange(nd)
        return [dict(superfluid_stiffness=float(st[c]), dc_conductivity=float(dc[c]), omega_grid=wg.copy(),
                     optical_conductivity=sigma[c].copy(), dos_omega_grid=dg.copy(), dos=dos[c].copy(),
                     dos_AN=dos_an[c].copy(), A_k_omega0=ak[c].reshape(Ly, Lx).T.copy())
                for c in range(nc)]

    def measure_transport_deltas(self, deltas, eta: float, domega: float, omega_max: float,
                                 chain: int = 0) -> list:
        """measure_transport at a list of pairing fields (each (N, 2)) on the
        lattice and disorder of `chain`, eigensolves batched over the list
        (dwh_measure_transport_deltas); one dict per field, in order."""
        D = np.asarray(deltas, dtype=np.complex128)
        if D.ndim != 3 or D.shape[1:] != (self.N, 2):
            raise ValueError(f"expected (nstates, {self.N}, 2) pairing fields")
        ns = D.shape[0]
        d = np.ascontiguousarray(np.transpose(D, (0, 2, 1)))
        nw, nd = transport_grid(eta, domega, omega_max, self._lib)
        Lx, Ly = self.info_lattice
        st, dc = np.empty(ns), np.empty(ns)
        sigma, dos, dos_an = np.empty((ns, nw)), np.empty((ns, nd)), np.empty((ns, nd))
        ak = np.empty((ns, Lx * Ly))
        self._c(self._lib.dwh_measure_transport_deltas(self._h, int(chain), ns, ptr(d), float(eta), float(domega),
                                                       float(omega_max), ptr(st), ptr(dc), ptr(sigma), nw,
                                                       ptr(dos), ptr(dos_an), nd, ptr(ak)))
        wg, dg = eta + domega * np.arange(nw), -omega_max + domega * np.arange(nd)
        return [dict(superfluid_stiffness=float(st[k]), dc_conductivity=float(dc[k]), omega_grid=wg.copy(),
                     optical_conductivity=sigma[k].copy(), dos_omega_grid=dg.copy(), dos=dos[k].copy(),
                     dos_AN=dos_an[k].copy(), A_k_omega0=ak[k].reshape(Ly, Lx).T.copy())
                for k in range(ns)]

    # -- assembly read-back (parity tests) --------------------------------
    def debug_dense_H(self, chain: int = 0) -> np.ndarray:
        """H_BdG(Δ) (2N, 2N) as the eigen/transport path assembles it (dwh_debug_dense_H)."""
        n2 = 2 * self.N
        Hcm = np.empty((n2, n2), dtype=np.complex128)          # row c = column c
        self._c(self._lib.dwh_debug_dense_H(self._h, int(chain), ptr(Hcm)))
        return Hcm.T.copy()

    def debug_level0(self, chain: int = 0, pole: int = 0, refill: bool = True):
        """(M, y): H_BdG(Δ) - i y_pole I (2N, 2N) from the CR level-0 blocks the
        factorisation consumes (dwh_debug_level0), and the pole heights y_q."""
        n2 = 2 * self.N
        Mcm = np.empty((n2, n2), dtype=np.complex128)
        y = np.empty(self.info["npoles"])
        self._c(self._lib.dwh_debug_level0(self._h, int(chain), int(pole), int(bool(refill)), ptr(Mcm), ptr(y)))
        return Mcm.T.copy(), y

    # -- timing ----------------------------------------------------------
    TIMERS = ("gj_update", "gj_pivot", "assemble", "contract", "step", "gj_edge", "cr_gemm", "cr_inv",
              "cr_inv_side", "eig_own", "eig_vendor", "cr_sparse")

    def timing_enable(self, on=True):
        """on: True (all timers), False, or an iterable of timer names."""
        if on is True:
            mask = -1
        elif not on:
            mask = 0
        else:
            mask = sum(1 << self.TIMERS.index(n) for n in on)
        self._c(self._lib.dwh_timing_enable(self._h, mask))

    def timing_reset(self):
        self._c(self._lib.dwh_timing_reset(self._h))

    def bench_assembly(self, reps: int):
        """dwh_bench_assembly: reps back-to-back assembly launches (timer "assemble")."""
        self._c(self._lib.dwh_bench_assembly(self._h, int(reps)))

    def timing_read(self, name: str):
        ms = C.c_double()
        n = C.c_int64()
        w = C.c_double()
        self._c(self._lib.dwh_timing_read(self._h, name.encode(), C.byref(ms), C.byref(n), C.byref(w)))
        return ms.value, n.value, w.value


def transport_grid(eta: float, domega: float, omega_max: float, lib=None):
    """(n_omega, n_dos): lengths of η:Δω:ω_max and -ω_max:Δω:ω_max as Julia
    counts them (dwh_transport_grid; host arithmetic, no device)."""
    lib = _lib.load() if lib is None else lib
    nw, nd = C.c_int64(), C.c_int64()
    check(lib.dwh_transport_grid(float(eta), float(domega), float(omega_max), C.byref(nw), C.byref(nd)))
    return nw.value, nd.value


def selftest_mfma(device: int = 0) -> int:
    return int(_lib.load().dwh_selftest_mfma(int(device)))
