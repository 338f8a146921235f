"""CPU ORACLE — test infrastructure only, never the product path.

Plain numpy/scipy restatement of the DwaveHMC.jl hot path
(YinkaiYu/Hybrid-Monte-Carlo-for-d-wave-SC, Julia; the reference cannot run
here because no Julia toolchain exists in this image or on the GPU box, see
DESIGN.md "Oracle").  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.

Every function cites the reference file:line it restates.  The eigen-
decomposition is LAPACK ``zheevr`` with ``uplo='U'`` (scipy ``driver='evr'``,
``lower=False``), i.e. the same driver and triangle Julia 1.11's
``eigen!(Hermitian(U, :U))`` uses at ``src/Hamiltonian.jl:106``.

Pinning (parity anchors, strongest first; exercised in tests/test_oracle.py):
  1. the clean uniform d-wave closed form, which restates the reference's own
     BCS check ``scripts/benchmark_clean.jl:15-43``;
  2. the identities I1-I4 of SURVEY.md §8a (spectrum symmetry, determinant
     form of E_f, force = -dH/dΔ* by finite differences, anomalous-block
     symmetry);
  3. the mean-field fixed point of ``scripts/test_forces.jl:31-55``;
  4. the loop-order invariance of ``scripts/bench_forces.jl:124-129``;
  5. leapfrog reversibility / dt² energy-error scaling of ``src/HMC.jl``.
The reference ships no golden vectors, so parity with the
Julia binary itself is pinned only through these closed forms and identities.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.linalg as sla


# ---------------------------------------------------------------------------
# Types.jl — parameters, lattice tables, state
# ---------------------------------------------------------------------------
def build_tables(Lx: int, Ly: int):
    """Neighbour tables, 1-based, shape (N, 4) — src/Types.jl:53-80.

    nn dirs   1:+x  2:+y  3:-x  4:-y        (src/Types.jl:70-73)
    nnn dirs  1:+x+y 2:-x+y 3:-x-y 4:+x-y   (src/Types.jl:76-79)
    site index i = (y-1)*Lx + x with mod1 PBC (src/Types.jl:60-64).
    """
    N = Lx * Ly

    def get_idx(x, y):
        x = (x - 1) % Lx + 1
        y = (y - 1) % Ly + 1
        return (y - 1) * Lx + x

    nn = np.zeros((N, 4), dtype=np.int64)
    nnn = np.zeros((N, 4), dtype=np.int64)
    for y in range(1, Ly + 1):
        for x in range(1, Lx + 1):
            i = get_idx(x, y) - 1
            nn[i, 0] = get_idx(x + 1, y)
            nn[i, 1] = get_idx(x, y + 1)
            nn[i, 2] = get_idx(x - 1, y)
            nn[i, 3] = get_idx(x, y - 1)
            nnn[i, 0] = get_idx(x + 1, y + 1)
            nnn[i, 1] = get_idx(x - 1, y + 1)
            nnn[i, 2] = get_idx(x - 1, y - 1)
            nnn[i, 3] = get_idx(x + 1, y - 1)
    return nn, nnn


@dataclass
class ModelParameters:
    """src/Types.jl:14-46 (constructor :49-91)."""
    Lx: int
    Ly: int
    t: float
    tp: float
    mu: float
    W: float
    n_imp: float
    beta: float
    J: float
    mass: float
    eta: float = 0.01
    domega: float = 0.002
    omega_max: float = 4.0
    N: int = field(init=False)
    nn_table: np.ndarray = field(init=False, repr=False)
    nnn_table: np.ndarray = field(init=False, repr=False)

    def __post_init__(self):
        self.N = self.Lx * self.Ly
        self.nn_table, self.nnn_table = build_tables(self.Lx, self.Ly)
        self.omega_min = self.eta
        self.n_omega = int(math.floor((self.omega_max - self.omega_min) / self.domega)) + 1


@dataclass
class SimulationState:
    """src/Types.jl:101-116.  Delta, pi: complex (N, 2); column 0 = +x bond,
    column 1 = +y bond (src/Types.jl:106-111)."""
    disorder_pot: np.ndarray
    Delta: np.ndarray
    pi: np.ndarray


def initialize_state(p: ModelParameters, rng: np.random.Generator) -> SimulationState:
    """src/Types.jl:118-134 with an injected RNG (the reference is unseeded,
    SURVEY.md F6): W on round(N*n_imp) sites drawn without replacement
    (:122-124), Delta ~ (U[0,1)+iU[0,1) - (.5+.5i))*0.1 (:128), pi = 0 (:131)."""
    N = p.N
    disorder = np.zeros(N)
    n_sites_imp = int(round_half_even(N * p.n_imp))
    disorder[rng.permutation(N)[:n_sites_imp]] = p.W
    Delta = ((rng.random((N, 2)) + 1j * rng.random((N, 2))) - (0.5 + 0.5j)) * 0.1
    pi = np.zeros((N, 2), dtype=np.complex128)
    return SimulationState(disorder, Delta, pi)


def round_half_even(x: float) -> float:
    """Julia ``round(Int, x)`` rounds half to even (RoundNearest)."""
    return float(np.round(x))


@dataclass
class ComputeCache:
    """src/Types.jl:145-212, hot-path members only (transport/FFT buffers are
    out of scope)."""
    H_base: np.ndarray
    E_n: np.ndarray
    U: np.ndarray
    forces: np.ndarray
    fermi_factors: np.ndarray
    Delta_backup: np.ndarray
    E_n_backup: np.ndarray
    U_backup: np.ndarray


def initialize_cache(p: ModelParameters) -> ComputeCache:
    """src/Types.jl:182-212 (hot-path buffers)."""
    n = 2 * p.N
    return ComputeCache(
        H_base=np.zeros((n, n), dtype=np.complex128),
        E_n=np.zeros(n),
        U=np.zeros((n, n), dtype=np.complex128),
        forces=np.zeros((p.N, 2), dtype=np.complex128),
        fermi_factors=np.zeros(n),
        Delta_backup=np.zeros((p.N, 2), dtype=np.complex128),
        E_n_backup=np.zeros(n),
        U_backup=np.zeros((n, n), dtype=np.complex128),
    )


# ---------------------------------------------------------------------------
# Hamiltonian.jl
# ---------------------------------------------------------------------------
def init_static_H(cache: ComputeCache, p: ModelParameters, disorder: np.ndarray) -> None:
    """src/Hamiltonian.jl:10-47.  Upper triangle only, overwrite semantics,
    reference loop order (diagonal, then per site NN dirs 1..4, NNN dirs 1..4)."""
    N = p.N
    H = cache.H_base
    H.fill(0.0)
    for i in range(N):                                   # :18-22
        term = disorder[i] - p.mu
        H[i, i] = term
        H[i + N, i + N] = -term
    for i in range(N):                                   # :26-44
        for d in range(4):
            j = p.nn_table[i, d] - 1
            if j > i:
                H[i, j] = -p.t
                H[i + N, j + N] = p.t
        for d in range(4):
            j = p.nnn_table[i, d] - 1
            if j > i:
                H[i, j] = -p.tp
                H[i + N, j + N] = p.tp


def update_H_BdG(cache: ComputeCache, p: ModelParameters, Delta: np.ndarray) -> None:
    """src/Hamiltonian.jl:55-86: H[i, jx+N] = H[jx, i+N] = Δ[i,1]/2 then the
    same for +y, overwriting, in site order."""
    N = p.N
    H = cache.H_base
    for i in range(N):
        jx = p.nn_table[i, 0] - 1
        vx = 0.5 * Delta[i, 0]
        H[i, jx + N] = vx
        H[jx, i + N] = vx
        jy = p.nn_table[i, 1] - 1
        vy = 0.5 * Delta[i, 1]
        H[i, jy + N] = vy
        H[jy, i + N] = vy


def hermitian_from_upper(Hu: np.ndarray) -> np.ndarray:
    """The dense Hermitian matrix that ``Hermitian(H, :U)`` denotes."""
    U = np.triu(Hu)
    return U + np.triu(Hu, 1).conj().T


def diagonalize_H_BdG(cache: ComputeCache, p: ModelParameters | None = None) -> None:
    """src/Hamiltonian.jl:96-114: copy, zheevr('V','A','U'), copy back.
    Eigenvalues ascending, eigenvectors in columns."""
    vals, vecs = sla.eigh(cache.H_base, lower=False, driver="evr",
                          check_finite=False)
    cache.E_n[:] = vals
    cache.U[:, :] = vecs


# ---------------------------------------------------------------------------
# Observables.jl — forces
# ---------------------------------------------------------------------------
def logistic(x):
    """LogExpFunctions.logistic (0.3.29): 1/(1+exp(-x)), overflow-safe."""
    x = np.asarray(x, dtype=np.float64)
    out = np.empty_like(x)
    pos = x >= 0
    out[pos] = 1.0 / (1.0 + np.exp(-x[pos]))
    ex = np.exp(x[~pos])
    out[~pos] = ex / (1.0 + ex)
    return out


def log1pexp(x):
    """LogExpFunctions.log1pexp: log(1+exp(x)), overflow-safe."""
    x = np.asarray(x, dtype=np.float64)
    return np.where(x > 0, x + np.log1p(np.exp(-np.abs(x))), np.log1p(np.exp(x)))


def pairing_P(U, E, p: ModelParameters):
    """P_ij = -ρ_{i,j+N} - ρ_{j,i+N}, ρ = U diag(f) U† (src/Observables.jl:32-53),
    vectorised over bonds.  Returns (P (N,2), f)."""
    N = p.N
    f = logistic(-p.beta * E)
    i = np.arange(N)
    P = np.empty((N, 2), dtype=np.complex128)
    Uf = U * f[None, :]
    for d in range(2):
        j = p.nn_table[:, d] - 1
        rho1 = np.einsum("bn,bn->b", Uf[i, :], U[j + N, :].conj())
        rho2 = np.einsum("bn,bn->b", Uf[j, :], U[i + N, :].conj())
        P[:, d] = -rho1 - rho2
    return P, f


def compute_forces(cache: ComputeCache, p: ModelParameters, Delta: np.ndarray) -> None:
    """src/Observables.jl:14-62: F = -β/2J (Δ - J P)."""
    P, f = pairing_P(cache.U, cache.E_n, p)
    cache.fermi_factors[:] = f
    cache.forces[:, :] = -(p.beta / (2 * p.J)) * (Delta - p.J * P)


def compute_forces_loops(U, E, Delta, p: ModelParameters):
    """Literal loop-order restatement of src/Observables.jl:24-59 (small N
    only).  Used to pin the vectorised form, as scripts/bench_forces.jl:124-129
    pins its two loop orders against each other."""
    N = p.N
    f = logistic(-p.beta * E)
    F = np.zeros((N, 2), dtype=np.complex128)
    b2j = p.beta / (2 * p.J)
    for i in range(N):
        for d in range(2):
            j = p.nn_table[i, d] - 1
            r1 = 0j
            r2 = 0j
            for n in range(2 * N):
                r1 += U[i, n] * f[n] * np.conj(U[j + N, n])
                r2 += U[j, n] * f[n] * np.conj(U[i + N, n])
            P = -r1 - r2
            F[i, d] = -b2j * (Delta[i, d] - p.J * P)
    return F


# ---------------------------------------------------------------------------
# HMC.jl
# ---------------------------------------------------------------------------
def fermion_energy(E: np.ndarray, beta: float) -> float:
    """-Σ_{E>0} (βE + 2 log1pexp(-βE))  (src/HMC.jl:21-27)."""
    Ep = E[E > 0]
    x = beta * Ep
    return float(-np.sum(x + 2.0 * log1pexp(-x)))


def compute_total_energy(cache: ComputeCache, p: ModelParameters, Delta, pi) -> float:
    """src/HMC.jl:12-41."""
    E_f = fermion_energy(cache.E_n, p.beta)
    E_b = p.beta / (2 * p.J) * float(np.sum(np.abs(Delta) ** 2))
    E_k = 1.0 / (2 * p.mass) * float(np.sum(np.abs(pi) ** 2))
    return E_k + E_b + E_f


def refresh_momentum(state: SimulationState, p: ModelParameters, noise: np.ndarray) -> None:
    """src/HMC.jl:51-61 with injected noise: ``noise`` is a standard complex
    normal draw (Var Re = Var Im = 1/2, what Julia's randn!(ComplexF64) gives);
    scaled by sqrt(2m)."""
    state.pi[:, :] = noise * math.sqrt(2 * p.mass)


def hmc_sweep(cache: ComputeCache, p: ModelParameters, state: SimulationState,
              Nt: int, dt: float, noise: np.ndarray, uniform: float):
    """src/HMC.jl:71-144 with injected RNG draws."""
    refresh_momentum(state, p, noise)                                 # :77
    H_old = compute_total_energy(cache, p, state.Delta, state.pi)    # :80
    cache.Delta_backup[:, :] = state.Delta                            # :84-86
    cache.E_n_backup[:] = cache.E_n
    cache.U_backup[:, :] = cache.U
    compute_forces(cache, p, state.Delta)                             # :91
    state.pi += (0.5 * dt) * cache.forces                             # :92
    coef_field = dt / (2 * p.mass)                                    # :95
    for step in range(1, Nt + 1):                                     # :98
        state.Delta += coef_field * state.pi                          # :101
        update_H_BdG(cache, p, state.Delta)                           # :105
        diagonalize_H_BdG(cache, p)                                   # :106
        compute_forces(cache, p, state.Delta)                         # :107
        if step < Nt:                                                 # :111
            state.pi += dt * cache.forces
    state.pi += (0.5 * dt) * cache.forces                             # :118
    H_new = compute_total_energy(cache, p, state.Delta, state.pi)    # :122
    dH = H_new - H_old
    accepted = bool(dH < 0 or uniform < math.exp(-dH))               # :128
    if not accepted:                                                  # :130-141
        state.Delta[:, :] = cache.Delta_backup
        cache.E_n[:] = cache.E_n_backup
        cache.U[:, :] = cache.U_backup
        update_H_BdG(cache, p, state.Delta)
    return accepted, dH


def calc_optimal_dt(beta, J, mass, Nt):
    """src/Simulation.jl:11-14."""
    T = 2 * math.pi * math.sqrt(mass * J / beta)
    return T / (2 * Nt)


# ---------------------------------------------------------------------------
# Observables.jl:64-222 — light observables
# ---------------------------------------------------------------------------
OBS_FIELDS = ("total_energy", "Delta_amp", "Delta_local", "Delta_global", "S_Delta",
              "hole_conc", "Delta_diff", "Delta_pair", "Delta_localpair")


def measure_observables(cache: ComputeCache, p: ModelParameters, Delta) -> dict:
    """src/Observables.jl:88-222."""
    N = p.N
    dx, dy = Delta[:, 0], Delta[:, 1]
    val_amp = float(np.sum(0.5 * (np.abs(dx) + np.abs(dy)))) / N
    val_local = float(np.sum(0.5 * np.abs(dx - dy))) / N
    g = np.sum(0.5 * (dx - dy)) / N
    val_global = abs(g)
    val_S = abs(g) ** 2
    U, E = cache.U, cache.E_n
    pos = E > 0
    w = np.sum(np.abs(U[:N, pos]) ** 2 - np.abs(U[N:, pos]) ** 2, axis=0)
    val_hole = float(np.sum(w * np.tanh(0.5 * p.beta * E[pos]))) / N
    E_f = fermion_energy(E, p.beta)
    E_b = p.beta / (2 * p.J) * float(np.sum(np.abs(Delta) ** 2))
    total_energy = (E_f + E_b) / N
    P, _ = pairing_P(U, E, p)
    Px, Py = P[:, 0], P[:, 1]
    diff = (np.abs(dx - p.J * Px) + np.abs(dy - p.J * Py)) / 2.0
    term = p.J * 0.5 * (Px - Py)
    return dict(total_energy=total_energy, Delta_amp=val_amp, Delta_local=val_local,
                Delta_global=val_global, S_Delta=val_S, hole_conc=val_hole,
                Delta_diff=float(np.sum(diff)) / N,
                Delta_pair=abs(np.sum(term) / N),
                Delta_localpair=float(np.sum(np.abs(term))) / N)


# ---------------------------------------------------------------------------
# Observables.jl:225-526 — transport and spectra (needs eigenpairs)
# ---------------------------------------------------------------------------
def julia_range(start: float, step: float, stop: float) -> np.ndarray:
    """collect(start:step:stop) for the float ranges of Observables.jl:395,446
    (Julia rounds the length to the nearest count when (stop-start)/step is
    within rounding of an integer)."""
    r = (stop - start) / step
    n = int(round(r)) if abs(r - round(r)) < 1e-8 * max(1.0, abs(r)) else int(math.floor(r))
    return start + step * np.arange(n + 1)


def current_operator(p: ModelParameters) -> np.ndarray:
    """Particle block of J_x, src/Observables.jl:237-278: i t (c†_i c_{i+x} -
    h.c.) plus the two t' diagonals (+x+y, +x-y); duplicate (row, col) pairs
    are summed (SparseArrays.sparse).  The Nambu operator is diag(Jx, Jx)."""
    N = p.N
    Jx = np.zeros((N, N), dtype=np.complex128)
    for i in range(N):
        for j, val in ((p.nn_table[i, 0] - 1, 1j * p.t), (p.nnn_table[i, 0] - 1, 1j * p.tp),
                       (p.nnn_table[i, 3] - 1, 1j * p.tp)):
            Jx[i, j] += val
            Jx[j, i] += np.conj(val)
    return Jx


def lorentzian(x, eta):
    """src/Observables.jl:399-401."""
    return (1.0 / math.pi) * (eta / (x * x + eta * eta))


def measure_transport_and_spectra(cache: ComputeCache, p: ModelParameters) -> dict:
    """src/Observables.jl:320-526 from the eigenpairs of the cache (and its
    fermi_factors, set by compute_forces!).  Returns the SpectrumResult fields
    (src/Observables.jl:290-305)."""
    N, beta, eta = p.N, p.beta, p.eta
    U, E, f = cache.U, cache.E_n, cache.fermi_factors
    u, v = U[:N], U[N:]
    Jx = current_operator(p)
    Jmn = U.conj().T @ np.vstack([Jx @ u, Jx @ v])        # :334-335, J_mn[n, m]
    # B. superfluid stiffness: diamagnetic term (:345-362)
    i = np.arange(N)
    jx, jxpy, jxmy = p.nn_table[:, 0] - 1, p.nnn_table[:, 0] - 1, p.nnn_table[:, 3] - 1

    def bond(j):
        return 2.0 * np.real(v[i] * np.conj(v[j]) - np.conj(u[i]) * u[j]).sum(axis=0)

    w = p.t * bond(jx) + p.tp * bond(jxpy) + p.tp * bond(jxmy)
    pos = E > 0
    val_dia = float(np.sum(w[pos] * np.tanh(0.5 * beta * E[pos]))) / N
    # paramagnetic term (:366-384): [n, m] with diff_E = E_m - E_n, diff_f = f_n - f_m
    dE = E[None, :] - E[:, None]
    df = f[:, None] - f[None, :]
    J2 = np.abs(Jmn) ** 2
    deg = np.abs(dE) < 1e-8
    ratio = np.where(deg, (beta * f * (1.0 - f))[:, None], df / np.where(deg, 1.0, dE))
    Lambda_xx = float(np.sum(ratio * J2)) / N
    # C. DC and optical conductivity (:395-423)
    omega = julia_range(p.eta, p.domega, p.omega_max)
    dc = math.pi / N * float(np.sum((beta * f * (1.0 - f))[:, None] * J2 * lorentzian(dE, eta)))
    keep = np.abs(df) >= 1e-12
    coef = np.where(keep, df * J2, 0.0).ravel()
    dEr = dE.ravel()
    sigma = np.array([np.sum(coef / om * lorentzian(om - dEr, eta)) for om in omega]) * (math.pi / N)
    # D. DOS, antinodal DOS, A(k, 0) (:430-516)
    dos_grid = julia_range(-p.omega_max, p.domega, p.omega_max)
    Lg = lorentzian(dos_grid[:, None] - E[None, :], eta)          # [w, n]
    Wn = np.sum(np.abs(u) ** 2, axis=0)
    x = i % p.Lx + 1
    y = i // p.Lx + 1
    sx = np.where(x % 2 == 0, 1.0, -1.0)
    sy = np.where(y % 2 == 0, 1.0, -1.0)
    wAN = 0.5 * (np.abs(sx @ u) ** 2 + np.abs(sy @ u) ** 2) / N
    dos = Lg @ Wn / N
    dos_AN = Lg @ wAN
    w0 = lorentzian(-E, eta)
    sel = w0 > 1e-6
    ur = u[:, sel].reshape(p.Ly, p.Lx, -1)                          # [y, x, n]: i = x + Lx y
    uk = np.fft.fft2(ur, axes=(0, 1))
    ak = np.einsum("yxn,n->xy", np.abs(uk) ** 2, w0[sel]) / N       # A_k_ω0[x, y]
    return dict(superfluid_stiffness=val_dia - Lambda_xx, dc_conductivity=dc, omega_grid=omega,
                optical_conductivity=sigma, dos_omega_grid=dos_grid, dos=dos, dos_AN=dos_AN,
                A_k_omega0=ak)


def measure_transport_loops(cache: ComputeCache, p: ModelParameters) -> dict:
    """The same quantities as literal loops over (n, m) and sites in the
    reference's order (src/Observables.jl:345-423), for small lattices: the
    loop-order pin of the vectorised restatement above."""
    N, n2, beta, eta = p.N, 2 * p.N, p.beta, p.eta
    U, E, f = cache.U, cache.E_n, cache.fermi_factors
    Jx = current_operator(p)
    JU = np.vstack([Jx @ U[:N], Jx @ U[N:]])
    Jmn = U.conj().T @ JU
    val_dia = 0.0
    for n in range(n2):
        if E[n] > 0:
            wn = 0.0
            for i in range(N):
                for j, tt in ((p.nn_table[i, 0] - 1, p.t), (p.nnn_table[i, 0] - 1, p.tp),
                              (p.nnn_table[i, 3] - 1, p.tp)):
                    wn += tt * 2.0 * np.real(U[i + N, n] * np.conj(U[j + N, n]) - np.conj(U[i, n]) * U[j, n])
            val_dia += wn * math.tanh(0.5 * beta * E[n]) / N
    lam = 0.0
    dc = 0.0
    omega = julia_range(p.eta, p.domega, p.omega_max)
    sigma = np.zeros(len(omega))
    for n in range(n2):
        for m in range(n2):
            dE = E[m] - E[n]
            J2 = abs(Jmn[n, m]) ** 2
            ratio = beta * f[n] * (1 - f[n]) if abs(dE) < 1e-8 else (f[n] - f[m]) / dE
            lam += ratio * J2
            dc += beta * f[n] * (1 - f[n]) * J2 * lorentzian(dE, eta)
            fnm = f[n] - f[m]
            if abs(fnm) >= 1e-12:
                sigma += fnm / omega * J2 * lorentzian(omega - dE, eta)
    return dict(superfluid_stiffness=val_dia - lam / N, dc_conductivity=dc * math.pi / N,
                optical_conductivity=sigma * math.pi / N)


# ---------------------------------------------------------------------------
# Closed forms (pins)
# ---------------------------------------------------------------------------
def bcs_rhs(Delta_in, Lx, Ly, t, tp, mu, beta, J):
    """scripts/benchmark_clean.jl:15-43, vectorised."""
    nx, ny = np.meshgrid(np.arange(Lx), np.arange(Ly), indexing="xy")
    kx = 2 * np.pi * nx / Lx
    ky = 2 * np.pi * ny / Ly
    eps = -2 * t * (np.cos(kx) + np.cos(ky)) - 4 * tp * np.cos(kx) * np.cos(ky) - mu
    g = np.cos(kx) - np.cos(ky)
    Ek = np.sqrt(eps ** 2 + abs(Delta_in * 1.0) ** 2 * g ** 2)
    val = g ** 2 / (2 * Ek) * np.tanh(0.5 * beta * Ek)
    return J / (Lx * Ly) * float(np.sum(val)) * Delta_in


def clean_dwave_closed_form(Delta0, Lx, Ly, t, tp, mu, beta, J):
    """for W=0, Δx=Δ0, Δy=-Δ0 the BdG problem is 2x2 in k.
    Returns (spectrum sorted, P_x, F_x, E_f)."""
    nx, ny = np.meshgrid(np.arange(Lx), np.arange(Ly), indexing="xy")
    kx = 2 * np.pi * nx / Lx
    ky = 2 * np.pi * ny / Ly
    eps = -2 * t * (np.cos(kx) + np.cos(ky)) - 4 * tp * np.cos(kx) * np.cos(ky) - mu
    g = np.cos(kx) - np.cos(ky)
    Ek = np.sqrt(eps ** 2 + np.abs(Delta0) ** 2 * g ** 2)
    N = Lx * Ly
    Px = np.sum(np.cos(kx) * g * Delta0 / Ek * np.tanh(0.5 * beta * Ek)) / N
    Fx = -(beta / (2 * J)) * (Delta0 - J * Px)
    spec = np.sort(np.concatenate([Ek.ravel(), -Ek.ravel()]))
    Ef = fermion_energy(spec, beta)
    return spec, Px, Fx, Ef


# ---------------------------------------------------------------------------
# Convenience: one full evaluation (H -> E, U -> F) for a given Δ
# ---------------------------------------------------------------------------
def evaluate(p: ModelParameters, disorder, Delta):
    """init_static_H! + update_H_BdG! + diagonalize_H_BdG! + compute_forces!
    (the sequence at src/Simulation.jl:84-86 followed by src/HMC.jl:91).
    Returns (cache, F, E_f)."""
    cache = initialize_cache(p)
    init_static_H(cache, p, disorder)
    update_H_BdG(cache, p, Delta)
    diagonalize_H_BdG(cache, p)
    compute_forces(cache, p, Delta)
    return cache, cache.forces.copy(), fermion_energy(cache.E_n, p.beta)
