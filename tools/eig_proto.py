"""numpy prototype of the hand-written Hermitian eigensolver (csrc/dwhmc_eig.hip):
the exact operation order of the device kernels, at sizes numpy runs in
seconds, checked against numpy.linalg.eigh.  Not imported by the package.

  tridiagonalisation  lower-triangle Householder (LAPACK zhetd2 'L' algebra),
                      the rank-2 update of column i deferred into the pass
                      that forms the next hemv (one read+write sweep of the
                      trailing triangle per column)
  eigenvalues         bisection on Sturm counts, one eigenvalue per thread
  eigenvectors        inverse iteration (T - λI = LU with partial pivoting,
                      three solves), Cholesky QR inside clusters, one
                      symmetric orthogonalisation step over all vectors
  back-transform      U = H_0 H_1 ... H_{n-2} Z, reflectors in blocks of nb
                      as I - V T V^H (forward compact WY), last block first
"""
from __future__ import annotations

import numpy as np


def larfg(alpha: complex, x: np.ndarray):
    """zlarfg: H^H [alpha; x] = [beta; 0], H = I - tau v v^H, v = [1; x/(alpha-beta)], beta real."""
    xn = np.linalg.norm(x)
    ar, ai = alpha.real, alpha.imag
    if xn == 0.0 and ai == 0.0:
        return 0.0 + 0j, ar, np.zeros_like(x)
    beta = -np.copysign(np.sqrt(ar * ar + ai * ai + xn * xn), ar)
    tau = complex((beta - ar) / beta, -ai / beta)
    v = x / (alpha - beta)
    return tau, beta, v


def tridiagonalize(A: np.ndarray):
    """Returns d, e, V (n x n, column i holds v_i at rows i+1.., v_i[i+1] = 1), tau."""
    A = A.copy()
    n = A.shape[0]
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    tau = np.zeros(max(n - 1, 0), complex)
    V = np.zeros((n, n), complex)
    vp = wp = None   # pending rank-2 update (full-length vectors, zero above their support)
    for i in range(n - 1):
        # S_i: pending update applied to column i (rows i..), reflector of column i
        col = A[i:, i].copy()
        if vp is not None:
            col -= vp[i:] * np.conj(wp[i]) + wp[i:] * np.conj(vp[i])
        d[i] = col[0].real
        t, beta, v = larfg(col[1], col[2:])
        e[i] = beta
        tau[i] = t
        vi = np.zeros(n, complex)
        vi[i + 1] = 1.0
        vi[i + 2:] = v
        V[:, i] = vi
        # P_i: pending update on the trailing triangle (rows/cols >= i+1), then p = A v_i
        if vp is not None:
            s = slice(i + 1, n)
            A[s, s] -= np.outer(vp[s], np.conj(wp[s])) + np.outer(wp[s], np.conj(vp[s]))
        s = slice(i + 1, n)
        L = np.tril(A[s, s])
        p = L @ vi[s] + np.conj(np.tril(A[s, s], -1)).T @ vi[s]   # lower triangle only
        # S_{i+1}: w = tau p - 1/2 tau (tau p)^H v  v   (zhetd2: x = tau A v; x += -1/2 tau (x^H v) v)
        x = t * p
        alpha = -0.5 * t * np.vdot(x, vi[s])
        w = np.zeros(n, complex)
        w[s] = x + alpha * vi[s]
        vp, wp = vi, w
    col = A[n - 1:, n - 1].copy()
    if vp is not None:
        col -= vp[n - 1:] * np.conj(wp[n - 1]) + wp[n - 1:] * np.conj(vp[n - 1])
    d[n - 1] = col[0].real
    return d, e, V, tau


def defer_write_pass(i: int, K: int) -> bool:
    """Pass i applies every pending rank-2 pair to the trailing triangle when
    i % K == K - 1 (with K = 1 every pass); the others only read A."""
    return i % K == K - 1


def tridiagonalize_deferred(A: np.ndarray, K: int = 8):
    """tridiagonalize with the rank-2 pairs applied to the trailing triangle
    only every K-th pass (csrc/dwhmc_eig.hip with kEigDefer = K): a read-only
    pass forms A_stale v_i, and the reduction of its partials corrects it with
    the pending pairs j (A v = A_stale v - sum_j v_j (w_j^H v) + w_j (v_j^H v),
    the dots from the pass); the next column gets the pending pairs (all but
    the newest, which the step applies) before the reflector."""
    A = A.copy()
    n = A.shape[0]
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    tau = np.zeros(max(n - 1, 0), complex)
    V = np.zeros((n, n), complex)
    pend = []          # pairs (v_j, w_j) not yet applied to A's trailing triangle
    newest = None      # pair i-1: known once the step has formed w
    for i in range(n - 1):
        col = A[i:, i].copy()
        for (vj, wj) in pend + ([newest] if newest is not None else []):
            col -= vj[i:] * np.conj(wj[i]) + wj[i:] * np.conj(vj[i])
        if newest is not None:
            pend.append(newest)
        d[i] = col[0].real
        t, beta, v = larfg(col[1], col[2:])
        e[i] = beta
        tau[i] = t
        vi = np.zeros(n, complex)
        vi[i + 1] = 1.0
        vi[i + 2:] = v
        V[:, i] = vi
        s = slice(i + 1, n)
        if defer_write_pass(i, K):
            for (vj, wj) in pend:
                A[s, s] -= np.outer(vj[s], np.conj(wj[s])) + np.outer(wj[s], np.conj(vj[s]))
            pend = []
        L = np.tril(A[s, s])
        p = L @ vi[s] + np.conj(np.tril(A[s, s], -1)).T @ vi[s]
        for (vj, wj) in pend:   # read-only pass: the pairs A still lacks
            p -= vj[s] * np.vdot(wj[s], vi[s]) + wj[s] * np.vdot(vj[s], vi[s])
        x = t * p
        alpha = -0.5 * t * np.vdot(x, vi[s])
        w = np.zeros(n, complex)
        w[s] = x + alpha * vi[s]
        newest = (vi, w)
    col = A[n - 1:, n - 1].copy()
    for (vj, wj) in pend + ([newest] if newest is not None else []):
        col -= vj[n - 1:] * np.conj(wj[n - 1]) + wj[n - 1:] * np.conj(vj[n - 1])
    d[n - 1] = col[0].real
    return d, e, V, tau


def sturm_count(d, e2, lam, pivmin):
    """Number of eigenvalues of T below lam (dstebz recurrence)."""
    q = d[0] - lam
    if abs(q) < pivmin:
        q = -pivmin
    c = int(q < 0)
    for k in range(1, len(d)):
        q = d[k] - lam - e2[k - 1] / q
        if abs(q) < pivmin:
            q = -pivmin
        c += int(q < 0)
    return c


def bisect_all(d, e):
    n = len(d)
    e2 = e * e
    r = np.zeros(n)
    r[:-1] += np.abs(e)
    r[1:] += np.abs(e)
    gl, gu = float(np.min(d - r)), float(np.max(d + r))
    tnorm = max(abs(gl), abs(gu))
    gl -= 2 * np.finfo(float).eps * tnorm * n + 1e-300
    gu += 2 * np.finfo(float).eps * tnorm * n + 1e-300
    pivmin = np.finfo(float).tiny * max(1.0, float(np.max(e2)) if n > 1 else 1.0)
    lam = np.zeros(n)
    for j in range(n):
        lo, hi = gl, gu
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if mid <= lo or mid >= hi:
                break
            if sturm_count(d, e2, mid, pivmin) > j:
                hi = mid
            else:
                lo = mid
        lam[j] = 0.5 * (lo + hi)
    return lam, tnorm


def lu_tridiag(d, e, lam, small):
    """dlagtf: (T - lam I) P = L U with row interchanges; U has 3 diagonals u0,u1,u2."""
    n = len(d)
    u0 = d - lam
    u1 = np.concatenate([e.copy(), [0.0]])
    u2 = np.zeros(n)
    lmul = np.zeros(n)
    piv = np.zeros(n, bool)
    sub = np.concatenate([e.copy(), [0.0]])
    for k in range(n - 1):
        a, b = u0[k], sub[k]
        if abs(a) >= abs(b):   # no interchange
            if a == 0.0:
                a = u0[k] = small
            m = b / a
            lmul[k] = m
            u0[k + 1] -= m * u1[k]
            u2[k] = 0.0
        else:                  # interchange rows k, k+1
            m = a / b
            lmul[k] = m
            piv[k] = True
            u0[k] = b
            t = u1[k]
            u1[k] = u0[k + 1]
            u0[k + 1] = t - m * u0[k + 1]
            u2[k] = u1[k + 1] if k + 1 < n - 1 else 0.0
            if k + 1 < n - 1:
                u1[k + 1] = -m * u1[k + 1]
    for k in range(n):
        if abs(u0[k]) < small:
            u0[k] = np.copysign(small, u0[k]) if u0[k] != 0 else small
    return u0, u1, u2, lmul, piv


def lu_solve(u0, u1, u2, lmul, piv, y):
    n = len(y)
    y = y.copy()
    for k in range(n - 1):
        if piv[k]:
            y[k], y[k + 1] = y[k + 1], y[k] - lmul[k] * y[k + 1]
        else:
            y[k + 1] -= lmul[k] * y[k]
    x = np.zeros(n)
    for k in range(n - 1, -1, -1):
        s = y[k]
        if k + 1 < n:
            s -= u1[k] * x[k + 1]
        if k + 2 < n:
            s -= u2[k] * x[k + 2]
        x[k] = s / u0[k]
    return x


def start_vector(m, n):
    """splitmix64 of (m, r) in [-1/2, 1/2), as start_entry in dwhmc_eig.hip."""
    M = (1 << 64) - 1
    out = np.empty(n)
    for r in range(n):
        z = (((m << 32) | r) + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out[r] = (z >> 11) * 2.0 ** -53 - 0.5
    return out


def inverse_iteration(d, e, lam, tnorm, cluster_tol=1e-6, iters=3):
    """Independent inverse iteration per eigenvalue, Cholesky QR (twice) on
    every cluster (consecutive gaps <= cluster_tol ||T||), then one symmetric
    orthogonalisation step Z <- Z (3/2 I - 1/2 Z^T Z) over all vectors."""
    n = len(d)
    eps = np.finfo(float).eps
    small = eps * tnorm if tnorm > 0 else eps
    Z = np.zeros((n, n))
    for m in range(n):
        fac = lu_tridiag(d, e, lam[m], small)
        x = start_vector(m, n)
        for _ in range(iters):
            x = lu_solve(*fac, x)
            x /= np.linalg.norm(x)
        Z[:, m] = x
    j = 0
    while j < n:
        k = j + 1
        while k < n and lam[k] - lam[k - 1] <= cluster_tol * tnorm:
            k += 1
        if k - j > 1:
            for _ in range(2):
                C = Z[:, j:k]
                L = np.linalg.cholesky(C.T @ C)
                Z[:, j:k] = np.linalg.solve(L, C.T).T
        j = k
    G = Z.T @ Z
    return Z @ (1.5 * np.eye(n) - 0.5 * G)


def back_transform(V, tau, Z, nb=8):
    n = Z.shape[0]
    U = Z.astype(complex)
    nr = n - 1
    starts = list(range(0, nr, nb))
    for j0 in reversed(starts):
        j1 = min(j0 + nb, nr)
        Vb = V[:, j0:j1]
        k = j1 - j0
        G = Vb.conj().T @ Vb
        T = np.zeros((k, k), complex)
        for j in range(k):
            T[j, j] = tau[j0 + j]
            if j:
                T[:j, j] = -tau[j0 + j] * (T[:j, :j] @ G[:j, j])
        W = Vb.conj().T @ U
        W = T @ W
        U -= Vb @ W
    return U


def zero_cluster_start(lam, tnorm, zero_tol=2.5e-4):
    """c0 of the particle-hole half solve: the largest index c <= n/2 with
    lam[c] - lam[c-1] > zero_tol ||T|| (0 if none): n/2 unless levels crowd
    around zero (then their vectors are computed, not taken as partners)."""
    h = len(lam) // 2
    c = h
    while c > 0 and not (lam[c] - lam[c - 1] > zero_tol * tnorm):
        c -= 1
    return c


def theta_partner(U, j_src):
    """Theta (u; v) = (-conj v; conj u): the particle-hole partner of an
    eigenvector of a BdG matrix [[h, D], [D^*, -h]] (h real symmetric, D
    symmetric), eigenvalue -E."""
    N = U.shape[0] // 2
    u, v = U[:N, j_src], U[N:, j_src]
    return np.concatenate([-np.conj(v), np.conj(u)])


def inverse_iteration_range(d, e, lam, tnorm, j0, cluster_tol=1e-6, iters=3):
    """inverse_iteration for the eigenvalue indices [j0, n) only (vectors of T
    in Z[:, j0:]); clusters inside the range, then one symmetric
    orthogonalisation step over those columns."""
    n = len(d)
    eps = np.finfo(float).eps
    small = eps * tnorm if tnorm > 0 else eps
    Z = np.zeros((n, n - j0))
    for m in range(j0, n):
        fac = lu_tridiag(d, e, lam[m], small)
        x = start_vector(m, n)
        for _ in range(iters):
            x = lu_solve(*fac, x)
            x /= np.linalg.norm(x)
        Z[:, m - j0] = x
    j = j0
    while j < n:
        k = j + 1
        while k < n and lam[k] - lam[k - 1] <= cluster_tol * tnorm:
            k += 1
        if k - j > 1:
            for _ in range(2):
                C = Z[:, j - j0:k - j0]
                L = np.linalg.cholesky(C.T @ C)
                Z[:, j - j0:k - j0] = np.linalg.solve(L, C.T).T
        j = k
    G = Z.T @ Z
    return Z @ (1.5 * np.eye(n - j0) - 0.5 * G)


def eigh_bdg(A: np.ndarray):
    """eigh for a BdG matrix: every eigenvalue, but eigenvectors only for the
    upper half of the spectrum (from c0, the start of a cluster straddling
    zero, if any); the lower half's vectors are the particle-hole partners of
    the upper half's (index j <-> n-1-j), so inverse iteration, the
    orthogonalisation and the back-transform run on ~half the columns."""
    n = A.shape[0]
    d, e, V, tau = tridiagonalize(A)
    lam, tnorm = bisect_all(d, e)
    c0 = zero_cluster_start(lam, tnorm)
    if n > 1 and np.any(np.diff(lam) <= 1e-6 * tnorm):
        c0 = 0   # degenerate levels: every vector computed (as the device)
    if n % 2 or c0 == 0:
        Z = inverse_iteration(d, e, lam, tnorm)
        return lam, back_transform(V, tau, Z)
    Zr = inverse_iteration_range(d, e, lam, tnorm, c0)
    Uh = back_transform(V, tau, Zr)
    U = np.zeros((n, n), complex)
    U[:, c0:] = Uh
    for j in range(c0):
        U[:, j] = theta_partner(U, n - 1 - j)
    return lam, U


def eigh(A: np.ndarray):
    d, e, V, tau = tridiagonalize(A)
    lam, tnorm = bisect_all(d, e)
    Z = inverse_iteration(d, e, lam, tnorm)
    U = back_transform(V, tau, Z)
    return lam, U


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    for n in (1, 2, 3, 17, 64):
        X = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        A = X + X.conj().T
        lam, U = eigh(A)
        ref = np.linalg.eigvalsh(A)
        print(n, np.max(np.abs(lam - ref)), np.max(np.abs(A @ U - U * lam)), np.max(np.abs(U.conj().T @ U - np.eye(n))))
    # exactly degenerate spectrum
    n = 24
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)))
    ev = np.repeat([-1.0, 0.5, 2.0], 8)
    A = (Q * ev) @ Q.conj().T
    A = 0.5 * (A + A.conj().T)
    lam, U = eigh(A)
    print("degenerate", np.max(np.abs(lam - ev)), np.max(np.abs(A @ U - U * lam)),
          np.max(np.abs(U.conj().T @ U - np.eye(n))))
