"""GPU parity of the eigenvalues-only solve (dwh_eigensystem with U = NULL:
the structure-preserving quaternion reduction, csrc/dwhmc_qeig.hip; numpy
restatement tools/qeig_proto.py) against LAPACK eigvalsh of the same H_BdG
(the oracle's assembly, src/Hamiltonian.jl:96-114) and against the
eigenvalues of the full eigensystem (the one-stage solver).  Lattices with
ragged 64-site pass tiles (6x6, 12x12) and several tiles (16x16), disordered
and clean (exactly degenerate levels)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx(m, O, L, clean, seed):
    p = O.ModelParameters(L, L, 1.0, -0.35, 0.0 if clean else -1.08, 0.0 if clean else 1.0, 0.1, 16.0, 0.8, 1.0)
    N = p.N
    rng = np.random.default_rng(seed)
    st = O.initialize_state(p, rng)
    if clean:
        D = np.stack([np.full(N, 0.2), np.full(N, -0.2)], 1).astype(complex)
        dis = np.zeros(N)
    else:
        D = st.Delta + 0.25 * np.exp(0.3j * rng.standard_normal((N, 2)))
        dis = st.disorder_pot
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, D)
    H = O.hermitian_from_upper(cache.H_base)
    ctx = m.FermionContext(p.Lx, p.Ly, p.t, p.tp, p.mu, p.beta, p.J, p.nn_table, p.nnn_table, dis)
    ctx.set_pairing(D)
    return ctx, H


@pytest.mark.parametrize("L", [4, 6, 8, 12, 16])
@pytest.mark.parametrize("clean", [False, True])
def test_eigenvalues_only_matches_lapack(dwhmc, oracle, L, clean):
    ctx, H = _ctx(dwhmc, oracle, L, clean, 100 + L)
    try:
        ev = np.linalg.eigvalsh(H)
        E, U = ctx.eigensystem(0, vectors=False)
        assert U is None
        scale = 1.0 + np.max(np.abs(ev))
        # backward-stable reduction + bisection to the last bit: a few eps ||H|| (n up to 512)
        assert np.max(np.abs(E - ev)) / scale < 2e-13
        assert np.all(np.diff(E) >= 0)
        # the same spectrum as the full (one-stage) eigensystem
        E1, _ = ctx.eigensystem(0, vectors=True)
        assert np.max(np.abs(E - E1)) / scale < 2e-13
        # bit-reproducible (fixed-point integer accumulation of H v)
        E2, _ = ctx.eigensystem(0, vectors=False)
        assert np.array_equal(E, E2)
    finally:
        ctx.close()
