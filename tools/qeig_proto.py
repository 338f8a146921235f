"""numpy prototype of the structure-preserving (quaternion) Hermitian eigensolver
for the BdG matrix of measure_transport_and_spectra (src/Observables.jl:314-526,
the eigen!(Hermitian(H)) of src/Hamiltonian.jl:96-114).  Not imported by the
package; tests/test_eig_algorithm.py checks it against numpy.linalg.eigh.

H_BdG = [[h, D], [conj D, -conj h]] (h Hermitian, D symmetric: singlet
pairing, src/Hamiltonian.jl:26-83) anticommutes with the antiunitary
Theta (u; v) = (-conj v; conj u), Theta^2 = -1.  Every
unitary that commutes with Theta keeps that form, so H is reduced site by
site instead of column by column:

  quaternion Householder  step j (j = 0 .. M-2, M = N sites) reduces column
                          j (particle of site j) below site j+1 to site j+1
                          with U = I - tau (v v^H + w w^H), w = Theta v (v is
                          orthogonal to w and as long, tau = 2 / |v|^2 real):
                          v = x + s x1, s = |x| / |x1| (x1: site j+1's two
                          entries of x), U x = -s x1; U commutes with Theta,
                          so column M+j (the hole of site j) follows.  Since
                          H Theta = -Theta H, H (Theta v) = -Theta (H v): ONE
                          matrix-vector product per site; the update is
                          H <- H - V W^H - W V^H with V = [v, Theta v],
                          W = [w1, -Theta w1], w1 = tau p - tau^2/2 (r v - conj(c) Theta v),
                          p = H v, r = v^H p (real), c = v^H Theta p.
                          Only the particle rows (the top half [h | D]) are
                          stored and updated: M - 1 steps instead of 2M - 1,
                          each over the same number of stored elements.
  site rotations          the reduced matrix is 2 x 2-block tridiagonal with
                          off-diagonal blocks E_j = q_j sigma_z (q_j a
                          quaternion); unit quaternions g_{j+1} = q_j g~_j /
                          |q_j| (g~ = sigma_z g sigma_z, g_0 = 1) make them
                          |q_j| sigma_z:  T = [[A, C], [conj C, -A]],
                          A = tridiag(a; b) real, C = diag(d) complex.
  eigenvalues             bisection on block Sturm counts: S_0 = D_0 - lam,
                          S_{j+1} = D_{j+1} - lam - b_j^2 sigma_z S_j^-1 sigma_z,
                          count = sum of negative eigenvalues of the 2 x 2 S_j
                          (det < 0: 1; det > 0, S_11 < 0: 2).
  eigenvectors            inverse iteration with the band LU of T - lam with
                          partial pivoting (interleaved sites: bandwidth 2;
                          the unpivoted block LDL^H, block_ldl_solve, loses
                          accuracy on clean lattices), Cholesky QR inside
                          clusters, one symmetric orthogonalisation
                          step; U = U_0 U_1 .. U_{M-2} G z (2 (M-1) rank-1
                          reflectors v_0, w_0, v_1, ... with real tau, compact
                          WY as the one-stage back-transform).
"""
from __future__ import annotations

import numpy as np


def theta(x: np.ndarray) -> np.ndarray:
    """Theta (u; v) = (-conj v; conj u) on the last axis split in halves (or rows)."""
    M = x.shape[0] // 2
    return np.concatenate([-np.conj(x[M:]), np.conj(x[:M])], axis=0)


def full_from_top(T: np.ndarray) -> np.ndarray:
    """H from its particle rows [h | D] (M x 2M): rows M + i = [conj D_i | -conj h_i]."""
    M = T.shape[0]
    return np.vstack([T, np.hstack([np.conj(T[:, M:]), -np.conj(T[:, :M])])])


def quat_reflector(x: np.ndarray):
    """For x (2m: particle entries of sites 0..m-1, then hole entries), the
    vector v with (I - tau (v v^H + Theta v (Theta v)^H)) x = -s x1 e1, and
    tau (real).  x1 = (x_p[0], x_h[0])."""
    m = x.shape[0] // 2
    nx = np.linalg.norm(x)
    n1 = np.hypot(abs(x[0]), abs(x[m]))
    v = x.copy()
    if nx == 0.0:
        return v, 0.0, np.zeros(2, complex)
    if n1 == 0.0:               # x1 = 0: map onto the particle unit vector instead
        v[0] += nx
        y = np.array([-nx, 0.0], complex)
    else:
        s = nx / n1
        v[0] += s * x[0]
        v[m] += s * x[m]
        y = np.array([-s * x[0], -s * x[m]])
    tau = 2.0 / np.vdot(v, v).real
    return v, tau, y


def qtridiagonalize_top(T0: np.ndarray):
    """Quaternion Householder reduction on the particle rows only (the device
    layout).  Returns (diag blocks a (real), d (complex), the reduced
    sub-diagonal site blocks y_j (M-1 x 2: particle / hole entries of site
    j+1 in column j), reflectors V (2M x 2M: column 2j = v_j, 2j+1 = Theta v_j,
    zero outside sites j+1..), tau)."""
    T = T0.astype(complex).copy()
    M = T.shape[0]
    a = np.zeros(M)
    d = np.zeros(M, complex)
    Y = np.zeros((max(M - 1, 0), 2), complex)
    V = np.zeros((2 * M, 2 * M), complex)
    tau = np.zeros(max(M - 1, 0))
    for j in range(M - 1):
        S = np.arange(j + 1, M)
        cols = np.concatenate([S, M + S])            # active columns (particle, hole of the sites S)
        a[j] = T[j, j].real
        d[j] = T[j, M + j]
        # column j below site j+1: particle rows = T[S, j], hole rows = conj(D)[S, j] = conj(T[S, M + j])
        x = np.concatenate([T[S, j], np.conj(T[S, M + j])])
        v, t, y = quat_reflector(x)
        Y[j] = y
        tau[j] = t
        m = len(S)
        vf = np.zeros(2 * M, complex)
        vf[cols] = v
        V[:, 2 * j] = vf
        V[:, 2 * j + 1] = theta(vf)
        if t == 0.0:
            continue
        # p = H_S v (both halves) from the stored particle rows
        Hs = full_from_top(T[np.ix_(S, cols)] if True else None)
        p = Hs @ v
        r = np.vdot(v, p).real
        c = np.vdot(v, theta(p))
        tv = theta(v)
        w1 = t * p - 0.5 * t * t * (r * v - np.conj(c) * tv)
        tw = theta(w1)
        # particle rows of H - v w1^H - w1 v^H + Theta v (Theta w1)^H + Theta w1 (Theta v)^H
        upd = (np.outer(v[:m], np.conj(w1)) + np.outer(w1[:m], np.conj(v))
               - np.outer(tv[:m], np.conj(tw)) - np.outer(tw[:m], np.conj(tv)))
        T[np.ix_(S, cols)] -= upd
        # column j / M+j of the particle rows S: y at site j+1, zeros below
        T[S, j] = 0.0
        T[S, M + j] = 0.0
        T[j + 1, j] = y[0]
        T[j + 1, M + j] = np.conj(y[1])           # D[j+1, j] = conj(H[M+j+1, j])
        # (the rows of site j itself are the symmetric images; only diag blocks are read)
    a[M - 1] = T[M - 1, M - 1].real
    d[M - 1] = T[M - 1, 2 * M - 1]
    return a, d, Y, V, tau


def quat(al, be):
    """Unit-quaternion 2 x 2 [[al, -conj be], [be, conj al]] (commutes with Theta per site)."""
    return np.array([[al, -np.conj(be)], [be, np.conj(al)]])


def site_rotations(a, d, Y):
    """g_j with g_{j+1} = q_j g~_j / |q_j|, q_j = [[y_p, -conj y_h], [y_h, conj y_p]],
    g~ = sigma_z g sigma_z; returns (g (M x 2 x 2), a', d' (diag blocks g^H D g),
    b (|q_j|))."""
    M = len(a)
    sz = np.diag([1.0, -1.0])
    g = np.zeros((M, 2, 2), complex)
    g[0] = np.eye(2)
    b = np.zeros(max(M - 1, 0))
    for j in range(M - 1):
        q = quat(Y[j, 0], Y[j, 1])
        nq = np.hypot(abs(Y[j, 0]), abs(Y[j, 1]))
        b[j] = nq
        g[j + 1] = (q @ (sz @ g[j] @ sz)) / nq if nq > 0 else sz @ g[j] @ sz
    a2 = np.zeros(M)
    d2 = np.zeros(M, complex)
    for j in range(M):
        Dj = np.array([[a[j], d[j]], [np.conj(d[j]), -a[j]]])
        Dp = g[j].conj().T @ Dj @ g[j]
        a2[j] = Dp[0, 0].real
        d2[j] = Dp[0, 1]
    return g, a2, d2, b


def block_tridiag_dense(a, d, b):
    """T = [[A, C], [conj C, -A]] (particle / hole ordering) for checks."""
    M = len(a)
    A = np.diag(a) + np.diag(b, 1) + np.diag(b, -1)
    C = np.diag(d)
    return np.block([[A, C], [np.conj(C), -A]])


def block_sturm_count(a, d, b, lam, pivmin):
    """Eigenvalues of T below lam: S_0 = D_0 - lam, S_{j+1} = D_{j+1} - lam -
    b_j^2 sigma_z S_j^-1 sigma_z; negative eigenvalues of each 2 x 2 S_j.
    S = [[p, q], [conj q, r]]; sigma_z S^-1 sigma_z = [[r, q], [conj q, p]] / det."""
    p, q, r = a[0] - lam, d[0], -a[0] - lam
    cnt = 0
    M = len(a)
    for j in range(M):
        det = p * r - (q.real * q.real + q.imag * q.imag)
        if abs(det) < pivmin:
            det = -pivmin
        cnt += 1 if det < 0 else (2 if p < 0 else 0)
        if j + 1 < M:
            f = b[j] * b[j] / det
            p, q, r = a[j + 1] - lam - f * r, d[j + 1] - f * q, -a[j + 1] - lam - f * p
    return cnt


def bisect(a, d, b, idx):
    """Eigenvalues number idx (ascending) of T by bisection on block Sturm counts."""
    M = len(a)
    rad = np.abs(d) + np.concatenate([b, [0.0]]) + np.concatenate([[0.0], b])
    tnorm = float(np.max(np.abs(a) + rad))
    gl, gu = -tnorm * (1 + 1e-14) - 1e-300, tnorm * (1 + 1e-14) + 1e-300
    # a pivot determinant below (eps ||T||)^2 is replaced (the 2 x 2 analogue
    # of dstebz's pivmin; keeps b^2 / det and the next determinant finite)
    pivmin = (np.finfo(float).eps * tnorm) ** 2 + np.finfo(float).tiny
    lam = np.zeros(len(idx))
    for k, i in enumerate(idx):
        lo, hi = gl, gu
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if mid <= lo or mid >= hi:
                break
            if block_sturm_count(a, d, b, mid, pivmin) > i:
                hi = mid
            else:
                lo = mid
        lam[k] = 0.5 * (lo + hi)
    return lam, tnorm


def block_ldl_solve(a, d, b, lam, rhs, small):
    """(T - lam) x = rhs with the unpivoted block LDL^H (sites j: 2-vectors
    (particle j, hole j)); a pivot determinant below `small` is replaced."""
    M = len(a)
    Sinv = np.zeros((M, 2, 2), complex)
    sz = np.diag([1.0, -1.0])
    S = np.array([[a[0] - lam, d[0]], [np.conj(d[0]), -a[0] - lam]])
    for j in range(M):
        det = (S[0, 0] * S[1, 1] - abs(S[0, 1]) ** 2).real
        if abs(det) < small:
            det = small if det >= 0 else -small
        Sinv[j] = np.array([[S[1, 1], -S[0, 1]], [-S[1, 0], S[0, 0]]]) / det
        if j + 1 < M:
            S = (np.array([[a[j + 1] - lam, d[j + 1]], [np.conj(d[j + 1]), -a[j + 1] - lam]])
                 - b[j] * b[j] * (sz @ Sinv[j] @ sz))
    yv = np.stack([rhs[:M], rhs[M:]], 1).astype(complex)
    for j in range(M - 1):          # L y = rhs: y_{j+1} -= E_j S_j^-1 y_j, E_j = b_j sigma_z
        yv[j + 1] -= b[j] * (sz @ (Sinv[j] @ yv[j]))
    x = np.zeros_like(yv)
    x[M - 1] = Sinv[M - 1] @ yv[M - 1]
    for j in range(M - 2, -1, -1):  # L^H x = D^-1 y: x_j = S_j^-1 (y_j - E_j^H x_{j+1})
        x[j] = Sinv[j] @ (yv[j] - b[j] * (sz @ x[j + 1]))
    return np.concatenate([x[:, 0], x[:, 1]])


def band_solve_pivoted(a, d, b, lam, rhs, small):
    """(T - lam) x = rhs with partial pivoting on the interleaved band form
    (site j: rows 2j (particle), 2j+1 (hole); bandwidth 2, as LAPACK gbtrf /
    dstein's dlagtf for the tridiagonal case): the unpivoted block LDL^H
    loses accuracy where a Schur block is near-singular away from the
    eigenvector's support (clean lattices' split blocks)."""
    M = len(a)
    n = 2 * M
    A = np.zeros((n, n), complex)          # dense here: the device keeps the 5-wide band rows
    for j in range(M):
        A[2 * j, 2 * j] = a[j] - lam
        A[2 * j + 1, 2 * j + 1] = -a[j] - lam
        A[2 * j, 2 * j + 1] = d[j]
        A[2 * j + 1, 2 * j] = np.conj(d[j])
        if j + 1 < M:
            A[2 * j, 2 * j + 2] = A[2 * j + 2, 2 * j] = b[j]
            A[2 * j + 1, 2 * j + 3] = A[2 * j + 3, 2 * j + 1] = -b[j]
    y = np.empty(n, complex)
    y[0::2], y[1::2] = rhs[:M], rhs[M:]
    for k in range(n):
        r = k + int(np.argmax(np.abs(A[k:min(k + 3, n), k])))
        if r != k:
            A[[k, r]] = A[[r, k]]
            y[[k, r]] = y[[r, k]]
        if abs(A[k, k]) < small:
            A[k, k] = small
        for i in range(k + 1, min(k + 3, n)):
            f = A[i, k] / A[k, k]
            A[i, k:min(k + 5, n)] -= f * A[k, k:min(k + 5, n)]
            y[i] -= f * y[k]
    x = np.zeros(n, complex)
    for k in range(n - 1, -1, -1):
        e = min(k + 5, n)
        x[k] = (y[k] - A[k, k + 1:e] @ x[k + 1:e]) / A[k, k]
    return np.concatenate([x[0::2], x[1::2]])


def start_vector(m, n):
    rng = np.random.default_rng(1000 + m)
    return rng.standard_normal(n) + 1j * rng.standard_normal(n)


def inverse_iteration(a, d, b, lam, tnorm, cluster_tol=1e-6, iters=3):
    n = 2 * len(a)
    eps = np.finfo(float).eps
    # a pivot determinant (~ pivot eigenvalue x ||T||) below eps ||T||^2 is
    # clamped: the scalar path's clamp of pivots below eps ||T||, so every
    # numerically singular spot amplifies alike (degenerate levels of split
    # blocks then come out as independent combinations)
    small = eps * tnorm * tnorm if tnorm > 0 else eps
    Z = np.zeros((n, len(lam)), complex)
    for k, l in enumerate(lam):
        x = start_vector(k, n)
        for _ in range(iters):
            x = band_solve_pivoted(a, d, b, l, x, eps * tnorm)
            x /= np.linalg.norm(x)
        Z[:, k] = x
    j = 0
    while j < len(lam):
        k = j + 1
        while k < len(lam) and lam[k] - lam[k - 1] <= cluster_tol * tnorm:
            k += 1
        if k - j > 1:
            for _ in range(2):
                C = Z[:, j:k]
                L = np.linalg.cholesky(C.conj().T @ C)
                Z[:, j:k] = np.linalg.solve(L, C.conj().T).conj().T
        j = k
    G = Z.conj().T @ Z
    return Z @ (1.5 * np.eye(len(lam)) - 0.5 * G)


def apply_site_rotations(g, Z):
    """G z: per site j, (z_p[j], z_h[j]) <- g_j (z_p[j], z_h[j])."""
    M = g.shape[0]
    zp, zh = Z[:M], Z[M:]
    return np.concatenate([g[:, 0, 0, None] * zp + g[:, 0, 1, None] * zh,
                           g[:, 1, 0, None] * zp + g[:, 1, 1, None] * zh])


def back_transform(V, tau, Z, nb=8):
    """U = U_0 U_1 .. U_{M-2} Z, U_j = (I - tau_j v_j v_j^H)(I - tau_j w_j w_j^H):
    the 2 (M-1) rank-1 reflectors in blocks of nb as I - V T V^H, last block first."""
    U = Z.astype(complex).copy()
    taus = np.repeat(tau, 2)
    nr = V.shape[1] - 2 if V.shape[1] >= 2 else 0
    nr = len(taus)
    for j0 in reversed(range(0, nr, nb)):
        j1 = min(j0 + nb, nr)
        Vb = V[:, j0:j1]
        k = j1 - j0
        Gm = Vb.conj().T @ Vb
        Tm = np.zeros((k, k), complex)
        for jj in range(k):
            Tm[jj, jj] = taus[j0 + jj]
            if jj:
                Tm[:jj, jj] = -taus[j0 + jj] * (Tm[:jj, :jj] @ Gm[:jj, jj])
        U -= Vb @ (Tm @ (Vb.conj().T @ U))
    return U


def eigh_quat(H: np.ndarray, cluster_tol=1e-6):
    """(E, U) of a BdG-form H through the quaternion reduction (full spectrum)."""
    M = H.shape[0] // 2
    a, d, Y, V, tau = qtridiagonalize_top(H[:M])
    g, a2, d2, b = site_rotations(a, d, Y)
    lam, tnorm = bisect(a2, d2, b, range(2 * M))
    Z = inverse_iteration(a2, d2, b, lam, tnorm, cluster_tol)
    Z = apply_site_rotations(g, Z)
    U = back_transform(V[:, :2 * (M - 1)], tau, Z)
    return lam, U


def bdg_matrix(M, seed=0, clean=False):
    """A random BdG-form H: h Hermitian, D complex symmetric."""
    rng = np.random.default_rng(seed)
    if clean:
        h = np.zeros((M, M))
        for i in range(M):
            h[i, (i + 1) % M] = h[(i + 1) % M, i] = -1.0
        D = 0.3 * (np.eye(M, k=1) + np.eye(M, k=-1)).astype(complex)
        D[0, M - 1] = D[M - 1, 0] = 0.3
    else:
        h = rng.standard_normal((M, M)) + 1j * rng.standard_normal((M, M))
        h = 0.5 * (h + h.conj().T)
        D = rng.standard_normal((M, M)) + 1j * rng.standard_normal((M, M))
        D = 0.5 * (D + D.T)
    return np.block([[h, D], [np.conj(D), -np.conj(h)]])
