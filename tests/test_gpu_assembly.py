"""Bit-exact BdG assembly on the device ("assembled H
entries: bit-exact").

The device never stores the reference's dense H_base: the hot path (block
cyclic reduction) assembles H_BdG(Δ) - i y_q I directly into level-0 lattice-row
blocks (top halves of the particle-hole symmetric M-form), and the
eigen/transport path assembles the dense matrix with k_tr_assemble.  Both are
read back through the C ABI (dwh_debug_level0 / dwh_debug_dense_H) and compared
with `np.array_equal` against the oracle's init_static_H! + update_H_BdG!
(src/Hamiltonian.jl:10-47, 55-86: upper triangle, overwrite order), completed
to the Hermitian matrix that `Hermitian(H, :U)` denotes (src/Hamiltonian.jl:106).

The small lattices are the reference's overwrite cases: on 1- and 2-site rings
the +x and -x (+y and -y) neighbours coincide, so one entry is written twice
(hopping, src/Hamiltonian.jl:28-43, and pairing, :70-82), and an NNN neighbour
can coincide with an NN one (the later NNN write wins).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T, TP, MU, J = 1.0, -0.35, -1.08, 0.8

LATTICES = [(1, 1), (2, 1), (1, 2), (2, 2), (3, 1), (1, 3), (4, 1), (1, 4), (5, 1), (2, 3), (3, 2),
            (2, 4), (4, 2), (3, 3), (4, 4), (5, 7), (6, 6), (8, 8), (16, 8), (16, 16)]


def reference_H(O, p, disorder, Delta):
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, disorder)
    O.update_H_BdG(cache, p, Delta)
    return cache.H_base.copy(), O.hermitian_from_upper(cache.H_base)


def case(O, Lx, Ly, seed):
    p = O.ModelParameters(Lx, Ly, T, TP, MU, 1.0, 0.3, 8.0, J, 1.0)
    rng = np.random.default_rng(seed)
    st = O.initialize_state(p, rng)
    dis = st.disorder_pot + rng.standard_normal(p.N) * 0.1     # arbitrary fp64 diagonals
    Delta = st.Delta + 0.3 * (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2)))
    return p, dis, Delta


def make_ctx(dwhmc, p, dis, algo):
    return dwhmc.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis,
                                algo=algo)


def expected_level0(Hfull, y):
    n2 = Hfull.shape[0]
    return Hfull - 1j * y * np.eye(n2)


@pytest.mark.parametrize("Lx,Ly", LATTICES)
def test_dense_assembly_bit_exact(dwhmc, oracle, Lx, Ly):
    p, dis, Delta = case(oracle, Lx, Ly, 17 * Lx + Ly)
    Hu, Hf = reference_H(oracle, p, dis, Delta)
    ctx = make_ctx(dwhmc, p, dis, "auto")
    ctx.set_pairing(Delta)
    H = ctx.debug_dense_H(0)
    ctx.close()
    assert np.array_equal(np.triu(H), np.triu(Hu)), "upper triangle differs from H_base"
    assert np.array_equal(H, Hf)


@pytest.mark.parametrize("Lx,Ly", LATTICES)
def test_cr_level0_blocks_bit_exact(dwhmc, oracle, Lx, Ly):
    """The matrix the hot-path factorisation consumes, every pole."""
    p, dis, Delta = case(oracle, Lx, Ly, 31 * Lx + Ly)
    _, Hf = reference_H(oracle, p, dis, Delta)
    ctx = make_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    P = ctx.info["npoles"]
    for q in sorted({0, P // 2, P - 1}):
        M, y = ctx.debug_level0(0, q, refill=True)
        assert np.array_equal(M, expected_level0(Hf, y[q])), f"pole {q}"
    ctx.close()


@pytest.mark.parametrize("Lx,Ly,nchains", [(2, 2, 2), (4, 3, 3), (8, 8, 2)])
def test_cr_level0_batched_chains(dwhmc, oracle, Lx, Ly, nchains):
    """Each chain's blocks carry its own disorder and Δ."""
    O = oracle
    cases = [case(O, Lx, Ly, 1000 + c) for c in range(nchains)]
    p = cases[0][0]
    dis = np.stack([c[1] for c in cases])
    Delta = np.stack([c[2] for c in cases])
    ctx = make_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    P = ctx.info["npoles"]
    for c in range(nchains):
        _, Hf = reference_H(O, p, dis[c], Delta[c])
        M, y = ctx.debug_level0(c, P - 1, refill=True)
        assert np.array_equal(M, expected_level0(Hf, y[P - 1])), f"chain {c}"
        assert np.array_equal(ctx.debug_dense_H(c), Hf), f"chain {c}"
    ctx.close()


@pytest.mark.parametrize("Lx,Ly", [(2, 2), (3, 2), (4, 4), (6, 5)])
def test_cr_trajectory_scatter_bit_exact(dwhmc, oracle, Lx, Ly):
    """Inside a trajectory the force kernel scatters the drifted Δ/2 into the
    level-0 blocks itself (no assembly launch): after an accepted Nt=3 sweep
    the pool must hold exactly H_BdG(Δ_final) - i y_q I."""
    O = oracle
    p, dis, Delta = case(O, Lx, Ly, 7 * Lx + Ly)
    ctx = make_ctx(dwhmc, p, dis, "cr")
    ctx.set_pairing(Delta)
    ctx.factorize()
    rng = np.random.default_rng(5)
    noise = (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2))) * np.sqrt(0.5)
    dt = O.calc_optimal_dt(p.beta, p.J, p.mass, 3)
    acc, _ = ctx.hmc_sweep(noise, np.array([0.0]), 3, dt, p.mass)   # u = 0: always accepted
    assert acc[0]
    D_final, _ = ctx.get_state()
    _, Hf = reference_H(O, p, dis, D_final[0])
    P = ctx.info["npoles"]
    for q in (0, P - 1):
        M, y = ctx.debug_level0(0, q, refill=False)
        assert np.array_equal(M, expected_level0(Hf, y[q])), f"pole {q}"
    ctx.close()


@pytest.mark.parametrize("L", [4, 8])
def test_golden_fixture_assembly(dwhmc, L):
    """The committed fixtures' H_upper (tests/golden, tests/make_golden.py)."""
    import dwhmc_loader  # noqa: F401  (package on sys.path)
    g = np.load(os.path.join(ROOT, "tests", "golden", f"oracle_L{L}.npz"))
    Hu = g["H_upper"]
    Hf = np.triu(Hu) + np.triu(Hu, 1).conj().T
    ctx = dwhmc.FermionContext(L, L, T, TP, MU, float(g["beta"]), J, g["nn"], g["nnn"], g["disorder"],
                               algo="cr")
    ctx.set_pairing(g["Delta"])
    assert np.array_equal(ctx.debug_dense_H(0), Hf)
    M, y = ctx.debug_level0(0, 0, refill=True)
    assert np.array_equal(M, Hf - 1j * y[0] * np.eye(2 * L * L))
    ctx.close()
