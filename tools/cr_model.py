"""Numpy model of the block cyclic-reduction (CR) selected inversion that the
device path `DWHMC_ALGO=cr` implements (design check, not the oracle).

H_BdG - z is block tridiagonal with periodic corners when its rows are
grouped by lattice row y (block y = [particles of row y | holes of row y],
size b = 2 Lx): hopping and pairing couple row y only to rows y-1, y, y+1
(src/Hamiltonian.jl:26-43, 68-83; tables src/Types.jl:60-80).  CR eliminates
every other block per level; the backward pass recovers the block-tridiagonal
part of G = (H - z)^-1, which holds every entry the force, E_f and Tr rho_hh
need.  ln|det| is the sum of ln|det| of the eliminated (Schur-complemented)
diagonal blocks.
"""
from __future__ import annotations

import numpy as np


def blocks_from_dense(A: np.ndarray, Lx: int, Ly: int):
    """Split a 2N x 2N BdG-ordered matrix into (Dg, U, L) per lattice row.
    U[y] = A[y, y+1], L[y] = A[y+1, y]; for Ly == 2 the single off-diagonal
    block goes to U only (U[y] + L[y-1] must equal the true block)."""
    N = Lx * Ly
    b = 2 * Lx

    def idx(y):
        return np.r_[y * Lx:(y + 1) * Lx, N + y * Lx:N + (y + 1) * Lx]

    Dg = np.zeros((Ly, b, b), complex)
    U = np.zeros((Ly, b, b), complex)
    L = np.zeros((Ly, b, b), complex)
    for y in range(Ly):
        Dg[y] = A[np.ix_(idx(y), idx(y))]
        if Ly == 1:
            continue
        yp = (y + 1) % Ly
        U[y] = A[np.ix_(idx(y), idx(yp))]
        if Ly > 2:
            L[y] = A[np.ix_(idx(yp), idx(y))]
    return Dg, U, L


def cr_selected_inverse(Dg, U, L):
    """Returns (logabsdet, GD, GU, GL) with GD[k] = G_kk, GU[k] = G_{k,k+1},
    GL[k] = G_{k+1,k} (indices mod m)."""
    m = len(Dg)
    Dg = [x.copy() for x in Dg]
    U = list(U)
    L = list(L)
    if m == 1:
        Dfin = Dg[0] + U[0] + L[0]
        sign, ld = np.linalg.slogdet(Dfin)
        G = np.linalg.inv(Dfin)
        return ld, [G], [G], [G]
    E = list(range(1, m - (m % 2), 2))          # eliminated positions
    K = [k for k in range(m) if k % 2 == 0]     # kept positions (m odd: m-1 kept)
    ld = 0.0
    Dinv, V1, V2 = {}, {}, {}
    for e in E:
        a, c = e - 1, (e + 1) % m
        s, l_ = np.linalg.slogdet(Dg[e])
        ld += l_
        Dinv[e] = np.linalg.inv(Dg[e])
        V1[e] = U[a] @ Dinv[e]        # A_{a,e} Dinv
        V2[e] = L[e] @ Dinv[e]        # A_{c,e} Dinv
    Dn, Un, Ln = [], [], []
    for kk, k in enumerate(K):
        d = Dg[k].copy()
        if k + 1 in Dinv:
            d -= V1[k + 1] @ L[k]
        if (k - 1) % m in Dinv:
            e = (k - 1) % m
            d -= V2[e] @ U[e]
        Dn.append(d)
        e = k + 1
        if e in Dinv:
            Un.append(-V1[e] @ U[e])
            Ln.append(-V2[e] @ L[k])
        else:                         # odd m: pair (m-1, 0) keeps its coupling
            Un.append(U[k])
            Ln.append(L[k])
    ld2, GDn, GUn, GLn = cr_selected_inverse(Dn, Un, Ln)
    ld += ld2
    mn = len(K)
    GD = [None] * m
    GU = [None] * m
    GL = [None] * m
    for kk, k in enumerate(K):
        GD[k] = GDn[kk]
        if k + 1 not in Dinv:          # kept-kept pair (odd m)
            GU[k] = GUn[kk]
            GL[k] = GLn[kk]
    for e in E:
        a, c = e - 1, (e + 1) % m
        ia, ic = a // 2, (c // 2) % mn
        Gaa, Gcc = GDn[ia], GDn[ic]
        if mn == 1:
            Gac = Gca = GDn[0]
        else:
            Gac, Gca = GUn[ia], GLn[ia]   # G_{a,c}, G_{c,a}: adjacent at the next level
        W1 = Dinv[e] @ L[a]           # Dinv A_{e,a}
        W2 = Dinv[e] @ U[e]           # Dinv A_{e,c}
        Gea = -(W1 @ Gaa + W2 @ Gca)
        Gec = -(W1 @ Gac + W2 @ Gcc)
        Gae = -(Gaa @ V1[e] + Gac @ V2[e])
        Gce = -(Gca @ V1[e] + Gcc @ V2[e])
        Gee = Dinv[e] - W1 @ Gae - W2 @ Gce
        GD[e] = Gee
        GU[a], GL[a] = Gae, Gea
        GU[e], GL[e] = Gec, Gce
    return ld, GD, GU, GL


def check(Lx, Ly, seed=0, y=0.7):
    """Compare against the dense inverse of a random BdG-pattern H - i y."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from oracle import dwhmc_oracle as O
    p = O.ModelParameters(Lx, Ly, 1.0, -0.35, -1.08, 1.0, 0.1, 8.0, 0.8, 1.0)
    rng = np.random.default_rng(seed)
    st = O.initialize_state(p, rng)
    Delta = st.Delta + 0.3 * (rng.standard_normal((p.N, 2)) + 1j * rng.standard_normal((p.N, 2)))
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, st.disorder_pot)
    O.update_H_BdG(cache, p, Delta)
    H = O.hermitian_from_upper(cache.H_base)
    A = H - 1j * y * np.eye(2 * p.N)
    Dg, U, L = blocks_from_dense(A, Lx, Ly)
    # the block split is exact
    ld, GD, GU, GL = cr_selected_inverse(Dg, U, L)
    G = np.linalg.inv(A)
    s, ld_ref = np.linalg.slogdet(A)
    Gd, Gu, Gl = blocks_from_dense(G, Lx, Ly)
    err = max(np.abs(GD[k] - Gd[k]).max() for k in range(Ly))
    if Ly > 1:
        err = max(err, max(np.abs(GU[k] - Gu[k]).max() for k in range(Ly)))
        if Ly > 2:
            err = max(err, max(np.abs(GL[k] - Gl[k]).max() for k in range(Ly)))
    return abs(ld - ld_ref), err


if __name__ == "__main__":
    for Lx, Ly in [(4, 1), (4, 2), (3, 3), (4, 4), (6, 5), (4, 6), (2, 7), (5, 8), (3, 12), (4, 16), (2, 2), (8, 3)]:
        dl, e = check(Lx, Ly)
        print(f"Lx={Lx} Ly={Ly}: |d logdet|={dl:.2e} max|dG|={e:.2e}")
