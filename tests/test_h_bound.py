"""CPU check of the ‖h‖ bound that selects the pole-table entry (no device):
dwh_debug_h_bound runs the host code dwh_create runs — Gershgorin, the
Lanczos estimate and its certification (ρI ∓ h positive definite by band
LDLᵀ in the folded row order).  The bound used must be an upper bound of the
exact spectral radius of every chain's static particle block h
(src/Hamiltonian.jl:10-44 with w_i − μ on the diagonal: numpy eigvalsh),
and no larger than Gershgorin."""
import ctypes as C

import numpy as np
import pytest


def abi_table(t):
    return np.ascontiguousarray(np.asarray(t).T, dtype=np.int64)


def h_bound(lib, p, dis):
    out = np.zeros(5)
    dis = np.ascontiguousarray(np.atleast_2d(dis), dtype=np.float64)
    nn, nnn = abi_table(p.nn_table), abi_table(p.nnn_table)
    rc = lib.dwh_debug_h_bound(p.Lx, p.Ly, p.t, p.tp, p.mu, nn.ctypes.data_as(C.c_void_p),
                               nnn.ctypes.data_as(C.c_void_p), dis.shape[0], dis.ctypes.data_as(C.c_void_p),
                               out.ctypes.data_as(C.c_void_p))
    assert rc == 0, lib.dwh_last_error(None).decode()
    return out


def exact_radius(O, p, dis):
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    h = O.hermitian_from_upper(cache.H_base)[:p.N, :p.N].real
    return np.max(np.abs(np.linalg.eigvalsh(h)))


@pytest.mark.parametrize("Lx,Ly,W,mu", [(4, 4, 1.0, -1.08), (8, 8, 0.0, -1.4), (16, 16, 1.0, -1.08),
                                        (32, 32, 1.0, -1.08), (12, 20, 3.0, 0.3), (5, 7, 1.0, -1.0),
                                        (32, 3, 1.0, -1.08)])
def test_h_bound_is_an_upper_bound(dwhmc, oracle, Lx, Ly, W, mu):
    O = oracle
    lib = dwhmc.load_library()
    p = O.ModelParameters(Lx, Ly, 1.0, -0.35, mu, W, 0.1, 16.0, 0.8, 1.0)
    rng = np.random.default_rng(Lx * 31 + Ly)
    dis = np.stack([O.initialize_state(p, rng).disorder_pot for _ in range(2)])
    g, lz, cert, used, neg = h_bound(lib, p, dis)
    exact = max(exact_radius(O, p, d) for d in dis)
    assert neg == 0.0                       # the LDLᵀ test rejects ρ = 0
    if lz < g:                              # lattice tables: the band test applies
        assert cert == 1.0 and used == lz, (Lx, Ly, g, lz)
    else:                                   # Gershgorin is already tighter (clean lattices)
        assert used == g
    assert used >= exact, (used, exact)
    assert min(lz, g) <= 1.03 * exact + 1e-9   # within Lanczos' 2 % margin of the exact radius


def test_h_bound_uncertified_estimate_falls_back(dwhmc, oracle):
    """A table with a long-range bond (site 0 - the middle site): the folded
    order no longer bounds the band, so the estimate is not certified and
    the bound is Gershgorin (an upper bound whatever Lanczos found)."""
    O = oracle
    lib = dwhmc.load_library()
    p = O.ModelParameters(40, 40, 1.0, -0.35, -1.08, 1.0, 0.1, 16.0, 0.8, 1.0)
    p.nnn_table = p.nnn_table.copy()
    far = p.N // 2 + 20
    p.nnn_table[0, 0] = far + 1
    p.nnn_table[far, 0] = 1
    dis = O.initialize_state(p, np.random.default_rng(3)).disorder_pot
    g, lz, cert, used, _ = h_bound(lib, p, dis)
    assert cert == 0.0 and used == g
    assert used >= exact_radius(O, p, dis)
