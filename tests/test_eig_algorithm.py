"""The eigensolver's algorithm (csrc/dwhmc_eig.hip) in its numpy prototype
(tools/eig_proto.py: the same operation order — zhetd2 'L' tridiagonalisation
with the rank-2 update deferred into the next hemv sweep, Sturm-count
bisection, inverse iteration with cluster Cholesky QR and one symmetric
orthogonalisation step, blocked compact-WY back-transform) against LAPACK on
random, BdG-structured and exactly degenerate Hermitian matrices.  CPU only;
the device solver itself is checked against the oracle in
tests/test_transport.py (GPU)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import eig_proto as P  # noqa: E402


def _check(A, lam, U, tol=1e-12):
    scale = 1 + np.max(np.abs(np.linalg.eigvalsh(A)))
    assert np.max(np.abs(lam - np.linalg.eigvalsh(A))) <= tol * scale
    assert np.max(np.abs(A @ U - U * lam[None, :])) <= 10 * tol * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(A.shape[0]))) <= tol


@pytest.mark.parametrize("n", [1, 2, 3, 17, 40])
def test_random_hermitian(n):
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    A = X + X.conj().T
    lam, U = P.eigh(A)
    _check(A, lam, U)


def test_degenerate_levels():
    """Exact multiplicities (a clean lattice has them): Cholesky QR turns the
    inverse-iteration vectors of each level into an orthonormal basis."""
    rng = np.random.default_rng(5)
    n = 24
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)))
    ev = np.repeat([-1.0, 0.5, 2.0], 8)
    A = (Q * ev) @ Q.conj().T
    A = 0.5 * (A + A.conj().T)
    lam, U = P.eigh(A)
    _check(A, lam, U)


def test_bdg_matrix(oracle):
    """A small H_BdG(Δ) of the oracle (src/Hamiltonian.jl:10-86): particle-hole
    symmetric spectrum, complex pairing."""
    O = oracle
    p = O.ModelParameters(4, 3, 1.0, -0.35, -1.08, 1.0, 0.1, 8.0, 0.8, 1.0)
    rng = np.random.default_rng(3)
    st = O.initialize_state(p, rng)
    D = st.Delta + 0.25 * np.exp(0.3j * rng.standard_normal((p.N, 2)))
    cache, _, _ = O.evaluate(p, st.disorder_pot, D)
    H = O.hermitian_from_upper(cache.H_base)
    lam, U = P.eigh(H)
    _check(H, lam, U)
    assert np.max(np.abs(lam + lam[::-1])) <= 1e-12 * (1 + np.max(np.abs(lam)))


def test_tridiagonal_is_similar():
    """T = Qᴴ A Q with Q the product of the stored reflectors (real T)."""
    rng = np.random.default_rng(11)
    n = 12
    X = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    A = X + X.conj().T
    d, e, V, tau = P.tridiagonalize(A)
    Q = np.eye(n, dtype=complex)
    for i in range(n - 1):
        Q = Q @ (np.eye(n) - tau[i] * np.outer(V[:, i], V[:, i].conj()))
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    assert np.max(np.abs(Q.conj().T @ A @ Q - T)) <= 1e-12 * np.max(np.abs(A))


def _bdg(O, Lx, Ly, clean=False, mu=-1.08, seed=3):
    if clean:
        p = O.ModelParameters(Lx, Ly, 1.0, -0.35, mu, 0.0, 0.0, 8.0, 0.8, 1.0)
        dis = np.zeros(p.N)
        D = np.stack([np.full(p.N, 0.2), np.full(p.N, -0.2)], 1).astype(np.complex128)
    else:
        p = O.ModelParameters(Lx, Ly, 1.0, -0.35, mu, 1.0, 0.1, 8.0, 0.8, 1.0)
        rng = np.random.default_rng(seed)
        st = O.initialize_state(p, rng)
        dis = st.disorder_pot
        D = st.Delta + 0.25 * np.exp(0.3j * rng.standard_normal((p.N, 2)))
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, dis)
    O.update_H_BdG(cache, p, D)
    return O.hermitian_from_upper(cache.H_base)


@pytest.mark.parametrize("Lx,Ly,clean,mu", [(4, 3, False, -1.08), (2, 4, False, -1.08), (5, 7, False, -1.08),
                                             (6, 6, True, -1.08), (8, 8, True, 0.0), (4, 4, True, 0.0)])
def test_bdg_half_spectrum_vectors(oracle, Lx, Ly, clean, mu):
    """eigh_bdg: eigenvectors of the upper half only (from the start of a
    cluster straddling zero), the lower half as particle-hole partners
    Θ(u; v) = (−v*; u*) — the same eigenpair tolerances as
    the full solve.  Clean lattices at μ = 0 with L % 4 == 0 have exact zero
    modes (the nodes of g_k on the grid): a cluster across zero, computed
    whole."""
    H = _bdg(oracle, Lx, Ly, clean, mu)
    lam, U = P.eigh_bdg(H)
    _check(H, lam, U)
    n = H.shape[0]
    d, e, V, tau = P.tridiagonalize(H)
    lam2, tn = P.bisect_all(d, e)
    c0 = P.zero_cluster_start(lam2, tn)
    if clean and mu == 0.0 and Lx % 4 == 0 and Ly % 4 == 0:
        assert c0 < n // 2          # the zero modes straddle
    else:
        assert c0 == n // 2
    if clean:                       # degenerate levels: eigh_bdg computes every vector
        assert np.any(np.diff(lam2) <= 1e-6 * tn)


@pytest.mark.parametrize("K", [1, 2, 3, 8])
@pytest.mark.parametrize("n", [1, 2, 9, 17, 40])
def test_deferred_pairs_same_reduction(K, n):
    """tridiagonalize_deferred (the device's deferral: the rank-2 pairs reach
    the trailing triangle only every K-th pass; read-only passes' hemv
    corrected by the pending pairs' dots, the next column by the pairs
    themselves) gives the reduction of tridiagonalize to rounding."""
    rng = np.random.default_rng(100 + n)
    X = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    A = X + X.conj().T
    ref = P.tridiagonalize(A)
    got = P.tridiagonalize_deferred(A, K)
    scale = 1 + np.max(np.abs(A))
    for a, b in zip(ref, got):
        if np.size(a):
            assert np.max(np.abs(a - b)) <= 1e-13 * scale * max(n, 1)


def test_fused_step_scalars():
    """The scalars k_eig_pass1f forms from k_eig_reduce's partials equal the
    step's: w = τp − ½τ(τp)ᴴv·v, column c = c0 − v·conj(w_i) − w, and
    ‖c_{i+2:}‖² by the expansion S1 − 2 Re(b̄ S2) + |b|² S3 with c = a − b v,
    a = c0 − τp, b = conj(w_i) + al (al = −½ τ g, g = Σ conj(τp) v)."""
    rng = np.random.default_rng(21)
    n, i = 40, 7
    z = lambda: rng.standard_normal(n) + 1j * rng.standard_normal(n)
    p, c0, v = z(), z(), z()
    v[:i] = 0.0
    v[i] = 1.0
    tp = 1.3 - 0.4j
    r = slice(i, n)
    x = tp * p
    g = np.vdot(x[r], v[r])                    # sum conj(x) v
    al = tp * (-0.5 * g)
    w = x + al * v
    wi = w[i]
    c_step = c0 - v * np.conj(wi) - w
    a = c0 - x
    b = np.conj(wi) + al
    c_fused = a - b * v
    assert np.max(np.abs(c_step[i:] - c_fused[i:])) <= 1e-13 * np.max(np.abs(c_step[i:]))
    q = slice(i + 2, n)
    S1, S2, S3 = np.sum(np.abs(a[q]) ** 2), np.vdot(v[q], a[q]), np.sum(np.abs(v[q]) ** 2)
    xn = S1 - 2.0 * np.real(np.conj(b) * S2) + abs(b) ** 2 * S3
    assert abs(xn - np.sum(np.abs(c_step[q]) ** 2)) <= 1e-12 * (S1 + abs(b) ** 2 * S3)


# --------------------------------------------------------------------------
# Structure-preserving (quaternion) reduction, tools/qeig_proto.py: the
# costed next step for the one-matrix measurement -- half
# the Householder steps of the one-stage reduction, one matrix-vector product
# per site (H Theta v = -Theta H v), the particle rows only.  CPU prototype.
import qeig_proto as QP  # noqa: E402


@pytest.mark.parametrize("M,seed,clean", [(3, 0, False), (7, 1, False), (12, 2, False), (10, 3, True)])
def test_quaternion_reduction_random_bdg(M, seed, clean):
    """Random BdG-form H (h Hermitian, D symmetric): the reduced 2 x 2-block
    tridiagonal T = [[A, C], [conj C, -A]] (A real tridiagonal, C diagonal)
    has H's spectrum, and the whole pipeline (block Sturm bisection, pivoted
    band inverse iteration, site rotations, 2 (M - 1) rank-1 reflectors in
    compact WY) gives eigenpairs at the one-stage solver's tolerances."""
    H = QP.bdg_matrix(M, seed, clean)
    a, d, Y, V, tau = QP.qtridiagonalize_top(H[:M])
    g, a2, d2, b = QP.site_rotations(a, d, Y)
    T = QP.block_tridiag_dense(a2, d2, b)
    ev = np.linalg.eigvalsh(H)
    scale = 1 + np.max(np.abs(ev))
    assert np.max(np.abs(np.linalg.eigvalsh(T) - ev)) <= 1e-12 * scale
    E, U = QP.eigh_quat(H)
    assert np.max(np.abs(E - ev)) <= 1e-12 * scale
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * M))) <= 1e-12


@pytest.mark.parametrize("Lx,Ly,clean,mu", [(6, 6, False, -1.08), (8, 8, True, 0.0), (6, 4, True, -1.0)])
def test_quaternion_reduction_bdg_lattices(oracle, Lx, Ly, clean, mu):
    """The reference's H_BdG (oracle assembly of src/Hamiltonian.jl), disordered
    and clean (exactly degenerate shells, the zero modes of mu = 0)."""
    O = oracle
    p = O.ModelParameters(Lx, Ly, 1.0, -0.35, mu, 0.0 if clean else 1.0, 0.1, 8.0, 0.8, 1.0)
    N = p.N
    rng = np.random.default_rng(Lx + Ly)
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
    E, U = QP.eigh_quat(H)
    ev = np.linalg.eigvalsh(H)
    scale = 1 + np.max(np.abs(ev))
    assert np.max(np.abs(E - ev)) <= 1e-12 * scale
    assert np.max(np.abs(H @ U - U * E[None, :])) <= 1e-11 * scale
    assert np.max(np.abs(U.conj().T @ U - np.eye(2 * N))) <= 1e-12


def _qmul(a1, b1, a2, b2):
    """quat(a1, b1) quat(a2, b2), quat(al, be) = [[al, -conj be], [be, conj al]] (k_q_rot's qmul)."""
    return a1 * a2 - np.conj(b1) * b2, b1 * a2 + np.conj(a1) * b2


@pytest.mark.parametrize("M,seed", [(2, 0), (9, 1), (40, 2)])
def test_site_rotations_prefix_scan(M, seed):
    """k_q_rot (csrc/dwhmc_qeig.hip) forms the site rotations as a prefix
    product instead of the recurrence g_{j+1} = q^_j tau(g_j), tau(quat(al,
    be)) = quat(al, -be) = k g k^-1 (k = i sigma_z): g_j = x_{j-1} .. x_0
    k^-j with x_i = q^_i k and k^-j = quat((-i)^j, 0).  Both equal
    tools/qeig_proto.py site_rotations' g (including q_j = 0, q^ = 1)."""
    rng = np.random.default_rng(seed)
    Y = rng.standard_normal((M - 1, 2)) + 1j * rng.standard_normal((M - 1, 2))
    if M > 3:
        Y[1] = 0.0
    a = rng.standard_normal(M)
    d = rng.standard_normal(M) + 1j * rng.standard_normal(M)
    g_ref, _, _, _ = QP.site_rotations(a, d, Y)
    pa, pb = 1.0 + 0j, 0.0 + 0j   # the prefix product, later factors on the left
    for j in range(M):
        if j > 0:
            nq = np.hypot(abs(Y[j - 1, 0]), abs(Y[j - 1, 1]))
            qa, qb = (Y[j - 1, 0] / nq, Y[j - 1, 1] / nq) if nq > 0 else (1.0 + 0j, 0.0 + 0j)
            pa, pb = _qmul(1j * qa, 1j * qb, pa, pb)   # x = q^ k = quat(i q^a, i q^b)
        c = (-1j) ** j
        np.testing.assert_allclose(QP.quat(pa * c, pb * c), g_ref[j], atol=1e-13)


def test_pass_dot_shares():
    """k_q_pass adds each p entry's share of r = v^H p and c' = sum (v_h p_p -
    v_p p_h) (c = v^H Theta p = conj c') component by component (Re / Im of
    p_p, p_h): the per-component formulas sum to the dots."""
    rng = np.random.default_rng(5)
    m = 7
    vp, vh, pp, ph = (rng.standard_normal(m) + 1j * rng.standard_normal(m) for _ in range(4))
    r = c_re = c_im = 0.0
    for i in range(m):
        for e, val in enumerate((pp[i].real, pp[i].imag, ph[i].real, ph[i].imag)):
            if e == 0:
                r += vp[i].real * val; c_re += vh[i].real * val; c_im += vh[i].imag * val
            elif e == 1:
                r += vp[i].imag * val; c_re -= vh[i].imag * val; c_im += vh[i].real * val
            elif e == 2:
                r += vh[i].real * val; c_re -= vp[i].real * val; c_im -= vp[i].imag * val
            else:
                r += vh[i].imag * val; c_re += vp[i].imag * val; c_im -= vp[i].real * val
    v = np.concatenate([vp, vh])
    p = np.concatenate([pp, ph])
    assert abs(r - np.vdot(v, p).real) < 1e-12
    c = np.vdot(v, QP.theta(p))
    assert abs(complex(c_re, -c_im) - c) < 1e-12


def _theta_interleaved(z):
    """Theta in T's site-interleaved basis (k_q_orth's zin): (Theta z)_2s =
    -conj z_2s+1, (Theta z)_2s+1 = conj z_2s."""
    t = np.empty_like(z)
    t[0::2] = -np.conj(z[1::2])
    t[1::2] = np.conj(z[0::2])
    return t


@pytest.mark.parametrize("n,c,seed", [(16, 1, 0), (24, 3, 1), (64, 8, 2)])
def test_crowd_pair_cholesky_qr(n, c, seed):
    """k_q_orth's crowd at zero: two rounds of Cholesky QR on the columns x0,
    Theta x0, x1, Theta x1, ... (in that order) give orthonormal columns in
    which every odd column is Theta of the even one before it, so writing back
    only the x columns leaves U partner-closed; and the interleaved Theta
    anticommutes with T's block form [[a, d], [conj d, -a]], b diag(1, -1)."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, c)) + 1j * rng.standard_normal((n, c))
    X[:, -1] += 0.999 * X[:, 0]   # a nearly dependent member, as inverse iteration can give
    for _ in range(2):
        Z = np.empty((n, 2 * c), complex)
        Z[:, 0::2] = X
        Z[:, 1::2] = np.stack([_theta_interleaved(X[:, i]) for i in range(c)], 1)
        L = np.linalg.cholesky(Z.conj().T @ Z)
        Q = np.linalg.solve(L, Z.conj().T).conj().T   # Z L^-H
        np.testing.assert_allclose(Q[:, 1::2], np.stack([_theta_interleaved(Q[:, 2 * i]) for i in range(c)], 1),
                                   atol=1e-12)
        X = Q[:, 0::2]
    assert np.max(np.abs(Q.conj().T @ Q - np.eye(2 * c))) <= 1e-13
    M = n // 2
    a = rng.standard_normal(M)
    b = rng.standard_normal(M - 1)
    d = rng.standard_normal(M) + 1j * rng.standard_normal(M)
    T = np.zeros((n, n), complex)
    for s in range(M):
        T[2 * s, 2 * s], T[2 * s + 1, 2 * s + 1] = a[s], -a[s]
        T[2 * s, 2 * s + 1], T[2 * s + 1, 2 * s] = d[s], np.conj(d[s])
        if s + 1 < M:
            T[2 * s, 2 * s + 2] = T[2 * s + 2, 2 * s] = b[s]
            T[2 * s + 1, 2 * s + 3] = T[2 * s + 3, 2 * s + 1] = -b[s]
    z = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    np.testing.assert_allclose(T @ _theta_interleaved(z), -_theta_interleaved(T @ z), atol=1e-12)
