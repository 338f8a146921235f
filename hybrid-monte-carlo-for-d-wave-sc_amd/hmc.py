"""Host-side mirror of DwaveHMC.jl's hot-path API, driving the HIP path.

Names follow the reference's exports (src/DwaveHMC.jl:3-9) with Julia's `!`
dropped; argument meaning, mutation and return values are the reference's:

    ModelParameters, SimulationState, ComputeCache, initialize_state,
    initialize_cache, init_static_H, update_H_BdG, diagonalize_H_BdG,
    compute_forces, compute_total_energy, refresh_momentum, hmc_sweep,
    calc_optimal_dt, measure_observables

`diagonalize_H_BdG` no longer produces eigenpairs: it runs the pole-expanded
no-pivot LU on the device and caches what every caller of the eigenpairs in
the hot path consumes (pairing amplitudes P_ij, E_f, Tr ρ_hh).  The reference
RNG is unseeded; every random draw here comes from a caller
supplied numpy Generator or is injected explicitly.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .context import FermionContext


# ---------------------------------------------------------------------------
# Types.jl
# ---------------------------------------------------------------------------
def neighbour_tables(Lx: int, Ly: int):
    """PBC neighbour tables, 1-based (N, 4) Int64 (src/Types.jl:53-80).
    nn dirs 1:+x 2:+y 3:-x 4:-y; nnn dirs 1:+x+y 2:-x+y 3:-x-y 4:+x-y;
    site (x, y) -> (y-1)*Lx + x with mod1 wrap."""
    x = np.arange(1, Lx + 1)
    y = np.arange(1, Ly + 1)
    X, Y = np.meshgrid(x, y, indexing="xy")      # site order: x fastest (i = (y-1)Lx + x)
    X = X.ravel()
    Y = Y.ravel()

    def idx(xx, yy):
        return ((yy - 1) % Ly) * Lx + ((xx - 1) % Lx) + 1

    nn = np.stack([idx(X + 1, Y), idx(X, Y + 1), idx(X - 1, Y), idx(X, Y - 1)], axis=1)
    nnn = np.stack([idx(X + 1, Y + 1), idx(X - 1, Y + 1), idx(X - 1, Y - 1), idx(X + 1, Y - 1)], axis=1)
    return nn.astype(np.int64), nnn.astype(np.int64)


@dataclass
class ModelParameters:
    """src/Types.jl:14-91 (positional order of the constructor at :49)."""
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
        self.Lx, self.Ly = int(self.Lx), int(self.Ly)
        for k in ("t", "tp", "mu", "W", "n_imp", "beta", "J", "mass", "eta", "domega", "omega_max"):
            setattr(self, k, float(getattr(self, k)))
        self.N = self.Lx * self.Ly
        self.nn_table, self.nnn_table = neighbour_tables(self.Lx, self.Ly)
        self.omega_min = self.eta
        self.n_omega = int(math.floor((self.omega_max - self.omega_min) / self.domega)) + 1


@dataclass
class SimulationState:
    """src/Types.jl:101-116: disorder_pot (N,), Delta and pi (N, 2) complex."""
    disorder_pot: np.ndarray
    Delta: np.ndarray
    pi: np.ndarray


def initialize_state(p: ModelParameters, rng: np.random.Generator) -> SimulationState:
    """src/Types.jl:118-134 with an explicit RNG: W on round(N n_imp) sites
    drawn without replacement, Δ = (U + iU - (.5+.5i))·0.1, π = 0."""
    N = p.N
    disorder = np.zeros(N)
    n_imp_sites = int(np.round(N * p.n_imp))
    disorder[rng.permutation(N)[:n_imp_sites]] = p.W
    Delta = ((rng.random((N, 2)) + 1j * rng.random((N, 2))) - (0.5 + 0.5j)) * 0.1
    return SimulationState(disorder, Delta, np.zeros((N, 2), dtype=np.complex128))


class ComputeCache:
    """src/Types.jl:145-212 for the hot path.  The dense H/U/backup matrices
    are replaced by the device context (created by init_static_H, which is
    where the reference first consumes the disorder)."""

    def __init__(self, p: ModelParameters, device: int = 0, delta_cap: float = 0.0):
        self.p = p
        self.device = device
        self.delta_cap = delta_cap
        self.ctx: FermionContext | None = None
        self.forces = np.zeros((p.N, 2), dtype=np.complex128)
        self.E_fermion = 0.0         # cached E_f  (what cache.E_n feeds in src/HMC.jl:21-27)
        self.pairing = np.zeros((p.N, 2), dtype=np.complex128)
        self.Delta_backup = np.zeros((p.N, 2), dtype=np.complex128)

    def require(self) -> FermionContext:
        if self.ctx is None:
            raise RuntimeError("init_static_H must be called before the hot path (src/Simulation.jl:84)")
        return self.ctx


def initialize_cache(p: ModelParameters, device: int = 0, delta_cap: float = 0.0) -> ComputeCache:
    return ComputeCache(p, device=device, delta_cap=delta_cap)


# ---------------------------------------------------------------------------
# Hamiltonian.jl
# ---------------------------------------------------------------------------
def init_static_H(cache: ComputeCache, p: ModelParameters, state: SimulationState) -> None:
    """src/Hamiltonian.jl:10-47: builds the device context (static h, its
    pole resolvents R(z) = (h - z)^-1 and ln|det(h - z)|)."""
    if cache.ctx is not None:
        cache.ctx.close()
    cache.ctx = FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table,
                               state.disorder_pot, delta_cap=cache.delta_cap, device=cache.device)


def update_H_BdG(cache: ComputeCache, p: ModelParameters, state: SimulationState) -> None:
    """src/Hamiltonian.jl:55-86: the pairing block follows state.Δ."""
    cache.require().set_pairing(state.Delta)


def diagonalize_H_BdG(cache: ComputeCache, p: ModelParameters | None = None) -> None:
    """src/Hamiltonian.jl:96-114 replacement: device factorisation of
    H_BdG(Δ) - i y_q for all poles; caches P_ij and E_f."""
    ctx = cache.require()
    ctx.factorize()
    cache.E_fermion = float(ctx.fermion_energy()[0])
    cache.pairing = ctx.pairing()[0]


# ---------------------------------------------------------------------------
# Observables.jl / HMC.jl
# ---------------------------------------------------------------------------
def compute_forces(cache: ComputeCache, p: ModelParameters, state: SimulationState) -> None:
    """src/Observables.jl:14-62: cache.forces = -β/2J (Δ - J P)."""
    cache.forces = cache.require().forces(state.Delta)[0]


def compute_total_energy(cache: ComputeCache, p: ModelParameters, state: SimulationState) -> float:
    """src/HMC.jl:12-41 (kinetic + boson on the device, cached E_f)."""
    ctx = cache.require()
    ctx.set_state(state.Delta, state.pi)
    return float(ctx.total_energy(p.mass)[0])


def refresh_momentum(state: SimulationState, p: ModelParameters, rng: np.random.Generator | None = None,
                     noise: np.ndarray | None = None) -> np.ndarray:
    """src/HMC.jl:51-61: π = sqrt(2m)·randn(ComplexF64) (Var Re = Var Im = 1/2).
    Returns the standard-normal noise used."""
    if noise is None:
        noise = standard_complex_normal(rng, (p.N, 2))
    state.pi = np.asarray(noise, dtype=np.complex128) * math.sqrt(2 * p.mass)
    return noise


def standard_complex_normal(rng: np.random.Generator, shape) -> np.ndarray:
    """Julia randn(ComplexF64): real and imaginary parts N(0, 1/2)."""
    return (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)) * math.sqrt(0.5)


def hmc_sweep(cache: ComputeCache, p: ModelParameters, state: SimulationState, *, Nt: int, dt: float,
              rng: np.random.Generator | None = None, noise: np.ndarray | None = None,
              uniform: float | None = None):
    """src/HMC.jl:71-144.  Draws come from `rng` unless injected.  With `rng`
    and no injected uniform, the Metropolis uniform is drawn only when
    ΔH >= 0 — the short-circuit of src/HMC.jl:128 — so the generator is
    consumed exactly as the reference consumes its own (dwh_hmc_trajectory +
    dwh_hmc_finish).  Returns (accepted, ΔH); mutates state.Δ, state.π and
    the cache."""
    ctx = cache.require()
    if rng is None and (noise is None or uniform is None):
        # checked before any device call: a missing generator must not leave
        # a trajectory pending on the context
        raise ValueError("hmc_sweep needs `rng` unless both noise and uniform are injected")
    if noise is None:
        noise = standard_complex_normal(rng, (p.N, 2))
    ctx.set_state(state.Delta, None)
    if uniform is None:
        dH = float(ctx.hmc_trajectory(noise, Nt, dt, p.mass)[0])
        acc = bool(dH < 0 or rng.random() < math.exp(-dH))
        ctx.hmc_finish([acc])
    else:
        a, d = ctx.hmc_sweep(noise, np.array([uniform]), Nt, dt, p.mass)
        acc, dH = bool(a[0]), float(d[0])
    D, P = ctx.get_state()
    state.Delta = D[0]
    state.pi = P[0]
    cache.E_fermion = float(ctx.fermion_energy()[0])
    cache.pairing = ctx.pairing()[0]
    return acc, dH


def calc_optimal_dt(beta, J, mass, Nt):
    """src/Simulation.jl:11-14."""
    T = 2 * math.pi * math.sqrt(mass * J / beta)
    return T / (2 * Nt)


@dataclass
class ObservablesResult:
    """src/Observables.jl:70-80."""
    total_energy: float
    Delta_amp: float
    Delta_local: float
    Delta_global: float
    S_Delta: float
    hole_conc: float
    Delta_diff: float
    Delta_pair: float
    Delta_localpair: float


@dataclass
class SpectrumResult:
    """src/Observables.jl:293-308 (A_k_omega0 indexed [kx, ky])."""
    superfluid_stiffness: float
    dc_conductivity: float
    omega_grid: np.ndarray
    optical_conductivity: np.ndarray
    dos_omega_grid: np.ndarray
    dos: np.ndarray
    dos_AN: np.ndarray
    A_k_omega0: np.ndarray


def measure_transport_and_spectra(cache: ComputeCache, p: ModelParameters, chain: int = 0) -> SpectrumResult:
    """src/Observables.jl:314-526 on the device: eigenpairs of H_BdG at the Δ
    the cache's context holds (the library's eigensolver), J_mn = U^H J U (the
    library's fp64 MFMA product), stiffness / conductivities / DOS / A(k, 0) in
    HIP kernels."""
    r = cache.require().measure_transport(p.eta, p.domega, p.omega_max, chain=chain)
    return SpectrumResult(**r)


def observables_from_outputs(p: ModelParameters, Delta, P, Ef: float, tr_hh: float) -> ObservablesResult:
    """src/Observables.jl:88-222 for one chain from the factorisation outputs:
    P_ij (the same pole-LU as the force), E_f, and Tr ρ_hh for the hole
    density (hole_conc = 2 Tr ρ_hh / N - 1 by particle-hole symmetry,
    SURVEY.md I4)."""
    N = p.N
    D = np.asarray(Delta)
    dx, dy = D[:, 0], D[:, 1]
    g = np.sum(0.5 * (dx - dy)) / N
    Eb = p.beta / (2 * p.J) * float(np.sum(np.abs(D) ** 2))
    Px, Py = P[:, 0], P[:, 1]
    term = p.J * 0.5 * (Px - Py)
    return ObservablesResult(
        total_energy=(float(Ef) + Eb) / N,
        Delta_amp=float(np.sum(0.5 * (np.abs(dx) + np.abs(dy)))) / N,
        Delta_local=float(np.sum(0.5 * np.abs(dx - dy))) / N,
        Delta_global=abs(g),
        S_Delta=abs(g) ** 2,
        hole_conc=2.0 * float(tr_hh) / N - 1.0,
        Delta_diff=float(np.sum((np.abs(dx - p.J * Px) + np.abs(dy - p.J * Py)) / 2.0)) / N,
        Delta_pair=abs(np.sum(term) / N),
        Delta_localpair=float(np.sum(np.abs(term))) / N,
    )


def measure_observables(cache: ComputeCache, p: ModelParameters, state: SimulationState) -> ObservablesResult:
    """src/Observables.jl:88-222 from the factorisation outputs (see
    observables_from_outputs)."""
    ctx = cache.require()
    return observables_from_outputs(p, state.Delta, ctx.pairing()[0], float(ctx.fermion_energy()[0]),
                                    float(ctx.hole_trace()[0]))
