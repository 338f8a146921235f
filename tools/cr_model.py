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


# ---------------------------------------------------------------------------
# Top-half ("quaternion") representation used by the device path.
#
# Particle-hole symmetry S H* S^-1 = -H (S = [[0, I], [-I, 0]] per site, SURVEY
# I1) makes every block X of the CR (rows/cols = [particles | holes] of one
# lattice row) one of two forms:
#   M-form (s = -1): X = [[A, B], [ conj(B), -conj(A)]]   (H - i y, inverses, G)
#   Q-form (s = +1): X = [[A, B], [-conj(B),  conj(A)]]   (products of two M-forms)
# so only the top half T = [A | B] (n x 2n) is stored.  A product C = X Y has
# form s_X * s_Y and top half  T_C = T_X Y_full  with the bottom rows of Y
# synthesised from T_Y:  Y[n + i, j] = sgn_j * conj(T_Y[i, (j + n) mod 2n]),
# sgn_j = -s_Y (j < n), +s_Y (j >= n).
# ---------------------------------------------------------------------------
def full_from_top(T, s):
    n = T.shape[0]
    A, B = T[:, :n], T[:, n:]
    return np.block([[A, B], [-s * B.conj(), s * A.conj()]])


def top_product(TX, TY, sY):
    n = TX.shape[0]
    Yb = np.empty_like(TY)
    Yb[:, :n] = -sY * TY[:, n:].conj()
    Yb[:, n:] = sY * TY[:, :n].conj()
    return TX @ np.vstack([TY, Yb])


def top_inverse_mform(T):
    """Inverse of an M-form block from its top half by the 2x2 block formula:
    Ainv = A^-1, F = A + B conj(Ainv B), P = F^-1, Q = P B conj(Ainv);
    |det X| = |det A| |det F|.  Returns (top half [P | Q] (M-form), ln|det X|)."""
    n = T.shape[0]
    A, B = T[:, :n], T[:, n:]
    Ainv = np.linalg.inv(A)
    F = A + B @ (Ainv @ B).conj()
    P = np.linalg.inv(F)
    Q = P @ B @ Ainv.conj()
    ld = np.linalg.slogdet(A)[1] + np.linalg.slogdet(F)[1]
    return np.hstack([P, Q]), ld


def check_top_half(n=5, seed=0, y=0.6):
    rng = np.random.default_rng(seed)
    def mform():
        A = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        A = 0.5 * (A + A.conj().T) - 1j * y * np.eye(n)          # h - i y, h Hermitian
        B = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        B = 0.5 * (B + B.T)                                      # pairing: symmetric
        return np.hstack([A, B])
    T1, T2 = mform(), mform()
    X, Y = full_from_top(T1, -1), full_from_top(T2, -1)
    err = 0.0
    # the assembled H - i y is M-form
    H = X
    S = np.block([[np.zeros((n, n)), np.eye(n)], [-np.eye(n), np.zeros((n, n))]])
    err = max(err, np.abs(S @ (H + 1j * y * np.eye(2 * n)).conj() @ np.linalg.inv(S) + (H + 1j * y * np.eye(2 * n))).max())
    P = X @ Y                                                    # M M -> Q-form
    err = max(err, np.abs(full_from_top(top_product(T1, T2, -1), +1) - P).max())
    TP = top_product(T1, T2, -1)
    R = P @ X                                                    # Q M -> M-form
    err = max(err, np.abs(full_from_top(top_product(TP, T1, -1), -1) - R).max())
    R2 = X @ P                                                   # M Q -> M-form
    err = max(err, np.abs(full_from_top(top_product(T1, TP, +1), -1) - R2).max())
    Ti, ld = top_inverse_mform(T1)
    err = max(err, np.abs(full_from_top(Ti, -1) - np.linalg.inv(X)).max())
    err = max(err, abs(ld - np.linalg.slogdet(X)[1]))
    return err


def cr_selected_inverse_top(Dg, U, L, merge=frozenset(), depth=0, _aux=False):
    """cr_selected_inverse on top halves (n x 2n) with the form bookkeeping of
    the device planner: D, U, L, inverses and G blocks are M-form; V, W are
    Q-form.  Inputs/outputs are top halves of M-form blocks.
    merge: the depths f whose first backward stage runs the G_ee stage of the
    level above (u = f + 1) in the device plan (build_cr_plan, round 6): f's
    products then read G_ee(u) at its eliminated positions p through
        W G_ee = (W Dinv) + (W W1) G_ae + (W W2) G_ce,
        G_ee V = (Dinv V) + G_ea (V1 V) + G_ec (V2 V)
    (u's blocks at p), as the device does; the result is the same inverse."""
    M, Q = -1, +1
    m = len(Dg)
    mul = top_product
    if m == 1:
        Dfin = Dg[0] + U[0] + L[0]
        G, ld = top_inverse_mform(Dfin)
        return (ld, [G], [G], [G], {}) if _aux else (ld, [G], [G], [G])
    E = list(range(1, m - (m % 2), 2))
    K = [k for k in range(m) if k % 2 == 0]
    ld = 0.0
    Dinv, V1, V2, W1, W2 = {}, {}, {}, {}, {}
    for e in E:
        a = e - 1
        Dinv[e], l_ = top_inverse_mform(Dg[e])
        ld += l_
        V1[e] = -mul(U[a], Dinv[e], M)
        V2[e] = -mul(L[e], Dinv[e], M)
        W1[e] = -mul(Dinv[e], L[a], M)
        W2[e] = -mul(Dinv[e], U[e], M)
    Dn, Un, Ln = [], [], []
    for k in K:
        if m == 2:
            Dn.append(Dg[0] + mul(V1[1], L[0], M) + mul(V2[1], U[1], M) + mul(V1[1], U[1], M)
                      + mul(V2[1], L[0], M))
            Un.append(np.zeros_like(Dg[0]))
            Ln.append(np.zeros_like(Dg[0]))
            continue
        d = Dg[k].copy()
        if k + 1 in Dinv:
            d += mul(V1[k + 1], L[k], M)
        if (k - 1) % m in Dinv:
            e = (k - 1) % m
            d += mul(V2[e], U[e], M)
        Dn.append(d)
        if k + 1 in Dinv:
            Un.append(mul(V1[k + 1], U[k + 1], M))
            Ln.append(mul(V2[k + 1], L[k], M))
        else:
            Un.append(U[k])
            Ln.append(L[k])
    ld2, GDn, GUn, GLn, up = cr_selected_inverse_top(Dn, Un, Ln, merge, depth + 1, True)
    ld += ld2
    mn = len(K)
    mrg = depth in merge and depth >= 1
    GD, GU, GL = [None] * m, [None] * m, [None] * m
    for kk, k in enumerate(K):
        GD[k] = GDn[kk]
        if k + 1 not in Dinv:
            GU[k], GL[k] = GUn[kk], GLn[kk]
    aux = {}
    for e in E:
        a, c = e - 1, (e + 1) % m
        ia, ic = a // 2, (c // 2) % mn
        Gaa, Gcc = GDn[ia], GDn[ic]
        Gac, Gca = (GDn[0], GDn[0]) if mn == 1 else (GUn[ia], GLn[ia])
        if mrg and ia in up:      # G_aa = G_ee(u)[ia]: its expansion (forward products x)
            x = up[ia]
            Gea = (mul(W1[e], x["Dinv"], M) + mul(mul(W1[e], x["W1"], Q), x["Gae"], M)
                   + mul(mul(W1[e], x["W2"], Q), x["Gce"], M) + mul(W2[e], Gca, M))
            Gae = (mul(x["Dinv"], V1[e], Q) + mul(x["Gea"], mul(x["V1"], V1[e], Q), Q)
                   + mul(x["Gec"], mul(x["V2"], V1[e], Q), Q) + mul(Gac, V2[e], Q))
        else:
            Gea = mul(W1[e], Gaa, M) + mul(W2[e], Gca, M)
            Gae = mul(Gaa, V1[e], Q) + mul(Gac, V2[e], Q)
        if mrg and ic in up:      # G_cc = G_ee(u)[ic]
            x = up[ic]
            Gec = (mul(W2[e], x["Dinv"], M) + mul(mul(W2[e], x["W1"], Q), x["Gae"], M)
                   + mul(mul(W2[e], x["W2"], Q), x["Gce"], M) + mul(W1[e], Gac, M))
            Gce = (mul(x["Dinv"], V2[e], Q) + mul(x["Gea"], mul(x["V1"], V2[e], Q), Q)
                   + mul(x["Gec"], mul(x["V2"], V2[e], Q), Q) + mul(Gca, V1[e], Q))
        else:
            Gec = mul(W1[e], Gac, M) + mul(W2[e], Gcc, M)
            Gce = mul(Gca, V1[e], Q) + mul(Gcc, V2[e], Q)
        GD[e] = Dinv[e] + mul(W1[e], Gae, M) + mul(W2[e], Gce, M)
        GU[a], GL[a], GU[e], GL[e] = Gae, Gea, Gec, Gce
        aux[e] = dict(Dinv=Dinv[e], V1=V1[e], V2=V2[e], W1=W1[e], W2=W2[e], Gea=Gea, Gec=Gec, Gae=Gae, Gce=Gce)
    return (ld, GD, GU, GL, aux) if _aux else (ld, GD, GU, GL)


def check_top_cr(Lx, Ly, seed=0, y=0.7, merge=frozenset()):
    """cr_selected_inverse_top (with the backward merge at the depths in
    `merge`) against the full-block version on a BdG matrix."""
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
    A = O.hermitian_from_upper(cache.H_base) - 1j * y * np.eye(2 * p.N)
    Dg, U, L = blocks_from_dense(A, Lx, Ly)
    ld, GD, GU, GL = cr_selected_inverse(Dg, U, L)
    top = lambda X: [x[:Lx, :] for x in X]
    ldt, GDt, GUt, GLt = cr_selected_inverse_top(top(Dg), top(U), top(L), merge)
    err = abs(ld - ldt)
    for F, T in ((GD, GDt), (GU, GUt), (GL, GLt)):
        for f, t in zip(F, T):
            err = max(err, np.abs(f[:Lx, :] - t).max())
    return err


# ---------------------------------------------------------------------------
# Algorithmic flop count of the recursion above, counted independently of the
# device planner (build_cr_plan): the same levels and terms as
# cr_selected_inverse_top, each product term on a top half (HP x BP output,
# K = BP) at 8 BP HP BP flops, each block inversion at 8 BP^3.  At level 0 the
# backward pass forms only the 16 x 16 output tiles the gathers read: the
# pairing entries G12[i, j] = G[b_i, b_j][p_i, HP + p_j] of every NN bond of
# the periodic Lx x Ly lattice (both orders) and, in G_ee, the diagonal
# (p, p).  rows: lattice rows per block (the device's DWHMC_CR_ROWS); block b
# holds rows rows*b .. rows*b + rows - 1, site (x, y) at p = (y % rows) Lx + x.
# G_ea / G_ec count per tile of their column window [HP, HP + Lxb), G_ee per
# tile of the whole top half.  For a 2-block chain (m = 2) G_ea and G_ec are
# both G[1, 0]; its reads are G_ec's (the planner's G_U[1]).
# Returns (inversion flops, product flops) per batch item.
# ---------------------------------------------------------------------------
def level0_read_tiles(Lx: int, Ly: int, rows: int = 1):
    """{(row block, column block): set of (tile row, tile column)} read by the
    force (pairing entries) and E_f / Tr rho_hh (diagonal of the G_D blocks)."""
    Lxb, m = Lx * rows, Ly // rows
    HP = (Lxb + 15) // 16 * 16
    reads = {}

    def pos(x, y):
        return y // rows, (y % rows) * Lx + x

    for y in range(Ly):
        for x in range(Lx):
            bi, pi = pos(x, y)
            reads.setdefault((bi, bi), set()).add((pi // 16, pi // 16))
            for xj, yj in ((x + 1) % Lx, y), (x, (y + 1) % Ly), ((x - 1) % Lx, y), (x, (y - 1) % Ly):
                bj, pj = pos(xj, yj)
                reads.setdefault((bi, bj), set()).add((pi // 16, (HP + pj) // 16))
    return reads


def level0_nnz_top(Lx: int, Ly: int, rows: int = 1):
    """Top-half nonzeros of the level-0 U[y], L[y] blocks of the CR lattice
    (Lx rows, Ly / rows blocks), counted on a BdG matrix of the reference's
    lattice (t = 1, t' = -0.35) with a nonzero pairing on every bond (the oracle
    assembly, not the device's tables)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from oracle import dwhmc_oracle as O
    p = O.ModelParameters(Lx, Ly, 1.0, -0.35, -1.08, 0.0, 0.0, 8.0, 0.8, 1.0)
    rng = np.random.default_rng(1)
    Delta = 0.5 + rng.random((p.N, 2)) + 1j * (0.5 + rng.random((p.N, 2)))
    cache = O.initialize_cache(p)
    O.init_static_H(cache, p, np.zeros(p.N))
    O.update_H_BdG(cache, p, Delta)
    A = O.hermitian_from_upper(cache.H_base)
    Lxb, Lyb = Lx * rows, Ly // rows
    _, U, L = blocks_from_dense(A, Lxb, Lyb)
    return [int(np.count_nonzero(u[:Lxb])) for u in U], [int(np.count_nonzero(x[:Lxb])) for x in L]


def merge_depths(Lyb: int, BP: int, nbatch: int, side: bool, sp0: bool, ncu: int = 256, merge=True):
    """The depths f whose first backward stage runs the G_ee stage of the
    level above (build_cr_plan's backward merge, round 6): from the level
    below the top downwards, m_f <= 8, not level 0 (sparse or dense), while
    the six forward products per expanded position fit the budget (side work:
    two rounds of 4 wave tiles on the CUs the final inversion leaves idle;
    else 1024 16 x 16 tiles in the top level's D' stage)."""
    HP = BP // 2
    ms = []
    m = Lyb
    while m > 1:
        ms.append(m)
        m = (m + 1) // 2
    out = set()
    # merge: True = the default depth (m_f <= 4 with side work, 8 without), an
    # int = DWHMC_CR_MERGE's m, False / 0 = off
    max_m = (4 if side else 8) if merge is True else int(merge)
    if max_m < 2 or len(ms) < 2:
        return out
    t32 = -(-HP // 32) * -(-BP // 32)
    t16 = (HP // 16) * (BP // 16)
    budget = 8 * (ncu - nbatch) if side else 1024
    used = 0
    for d in range(len(ms) - 2, 0, -1):
        mf, mu = ms[d], ms[d + 1]
        if mf > max_m:
            break
        elim_u = set(range(1, mu - mu % 2, 2))
        nx = 0
        for e in range(1, mf - mf % 2, 2):
            a, c = e - 1, (e + 1) % mf
            nx += (a // 2 in elim_u) + ((c // 2) % mu in elim_u)
        cost = 6 * nx * nbatch * (t32 if side else t16)
        if used + cost > budget:
            break
        used += cost
        out.add(d)
    return out


def cr_flop_count(Lx: int, Ly: int, rows: int = 1, sparse0: bool = True, nbatch: int = 1, side: bool = False,
                  merge=True):
    """sparse0: level 0 by the sparse stages when the device takes them (even
    Ly / rows >= 4, BP <= 96): the sparse products at 8 flops per complex MAC
    of a stored nonzero (cr_selected_inverse_top_sparse0), the dense products
    one term each.  nbatch / side (BP = 64 side work on) / merge: the backward
    merge's extra products (merge_depths): per expanded position six forward
    products and one more term in each of two backward products."""
    Lxb, Lyb = Lx * rows, Ly // rows
    HP = (Lxb + 15) // 16 * 16
    BP = 2 * HP
    sp = sparse0 and Lyb % 2 == 0 and Lyb >= 4 and BP <= 96
    mdepths = merge_depths(Lyb, BP, nbatch, side and BP == 64, sp, merge=merge)
    if sp:
        nU, nL = level0_nnz_top(Lx, Ly, rows)
    full = 8.0 * BP * HP * BP                       # one term, whole top half
    tr = HP // 16                                   # tile rows
    wc = -(-(Lxb) // 16)                            # tile columns of the G_ea / G_ec window
    per_ea = 8.0 * BP * HP * Lxb / (tr * wc)        # one term, one tile of that window
    per_ee = full / (tr * 2 * tr)                   # one term, one tile of the top half
    reads = level0_read_tiles(Lx, Ly, rows)
    inv = 0
    terms = 0.0

    def level(m, depth):
        nonlocal inv, terms
        if m == 1:
            inv += 1
            return
        if depth == 0 and sp:
            E, K = list(range(1, m, 2)), list(range(0, m, 2))
            inv += len(E)
            for k in K:
                er, el = k + 1, (k - 1) % m
                terms += 8.0 * BP * (nU[k] + nL[er] + nL[el]) + 8.0 * HP * 2 * (2 * nL[k] + nU[el] + nU[er])
            level(len(K), 1)
            for e in E:
                a, c = e - 1, (e + 1) % m
                terms += 8.0 * HP * 2 * 2 * (nU[a] + nL[e]) + 8.0 * BP * 3 * (nL[a] + nU[e])
                n_ec = len(reads.get((e, c), ()))
                n_ea = 0 if a == c else len(reads.get((e, a), ()))
                n_ee = len(reads.get((e, e), ()))
                # G_ae = G[a, e], G_ce = G[c, e]: only the gathers read them here
                n_ae = len(reads.get((a, e), ()))
                n_ce = 0 if a == c else len(reads.get((c, e), ()))
                terms += (n_ea + n_ec + n_ae + n_ce) * per_ea + full + n_ee * per_ee
            return
        E = list(range(1, m - (m % 2), 2))
        K = list(range(0, m, 2))
        inv += len(E)
        terms += 4 * len(E) * full                  # V1, V2, W1, W2
        elim = set(E)
        for k in K:
            if m == 2:
                terms += 4 * full                   # D' of the 1-block chain
                continue
            hr, hl = (k + 1) in elim, ((k - 1) % m) in elim
            terms += (int(hr) + int(hl)) * full     # D'
            if hr:
                terms += 2 * full                   # U', L'
        level(len(K), depth + 1)
        for e in E:                                 # backward pass
            if depth == 0:
                a, c = e - 1, (e + 1) % m
                n_ec = len(reads.get((e, c), ()))
                n_ea = 0 if a == c else len(reads.get((e, a), ()))
                n_ee = len(reads.get((e, e), ()))
                terms += 2 * (n_ea + n_ec) * per_ea + 2 * 2 * full + 2 * n_ee * per_ee
            else:
                terms += 5 * 2 * full               # G_ea, G_ec, G_ae, G_ce, G_ee: 2 terms each
                if depth in mdepths:                # expansions of G_ee of the level above
                    mu = len(K)
                    a, c = e - 1, (e + 1) % m
                    for p in (a // 2, (c // 2) % mu):
                        if p % 2 == 1 and p < mu - mu % 2:
                            terms += 8 * full

    level(Lyb, 0)
    return inv * 8.0 * BP ** 3, terms


# ---------------------------------------------------------------------------
# Level 0 with its sparse off-diagonal blocks (round 5, the device's sparse
# level-0 stages, dwhmc_cr.hip k_cr_sp_fwd / k_cr_sp_bwd): U, L of the lattice
# rows are hopping + one pairing entry per row, so at level 0 every product
# with them is a sparse one and V1, V2, W1, W2 are never formed:
#   forward   D'_k = D_k - U_k Dinv_{k+1} L_k - L_{k-1} Dinv_{k-1} U_{k-1}
#             U'_k = -U_k Dinv_{k+1} U_{k+1},  L'_k = -L_{k+1} Dinv_{k+1} L_k
#   backward  Z_a = G_aa U_a + G_ac L_e,  Z_c = G_ca U_a + G_cc L_e      (dense . sparse)
#             Y_a = L_a G_aa + U_e G_ca,  Y_c = L_a G_ac + U_e G_cc      (sparse . dense)
#             M = L_a Z_a + U_e Z_c                                      (sparse . dense)
#             G_ae = -Z_a Dinv, G_ce = -Z_c Dinv, G_ea = -Dinv Y_a, G_ec = -Dinv Y_c,
#             T = -Dinv M, G_ee = Dinv - T Dinv  (= Dinv + Dinv M Dinv)
# (a = e - 1, c = e + 1 mod m; even m >= 4, so every kept block has both
# eliminated neighbours).  The dense products left are one term each.
# ---------------------------------------------------------------------------
def cr_selected_inverse_top_sparse0(Dg, U, L):
    M, Q = -1, +1
    m = len(Dg)
    assert m % 2 == 0 and m >= 4
    mul = top_product
    E = list(range(1, m, 2))
    K = list(range(0, m, 2))
    ld = 0.0
    Dinv = {}
    for e in E:
        Dinv[e], l_ = top_inverse_mform(Dg[e])
        ld += l_
    Dn, Un, Ln = [], [], []
    for k in K:
        er, el = k + 1, (k - 1) % m
        V1r = -mul(U[k], Dinv[er], M)                 # Q-form
        V2r = -mul(L[er], Dinv[er], M)
        V2l = -mul(L[el], Dinv[el], M)
        Dn.append(Dg[k] + mul(V1r, L[k], M) + mul(V2l, U[el], M))
        Un.append(mul(V1r, U[er], M))
        Ln.append(mul(V2r, L[k], M))
    ld2, GDn, GUn, GLn = cr_selected_inverse_top(Dn, Un, Ln)
    ld += ld2
    mn = len(K)
    GD, GU, GL = [None] * m, [None] * m, [None] * m
    for kk, k in enumerate(K):
        GD[k] = GDn[kk]
    for e in E:
        a, c = e - 1, (e + 1) % m
        ia, ic = a // 2, (c // 2) % mn
        Gaa, Gcc = GDn[ia], GDn[ic]
        Gac, Gca = (GDn[0], GDn[0]) if mn == 1 else (GUn[ia], GLn[ia])
        Za = mul(Gaa, U[a], M) + mul(Gac, L[e], M)    # Q-form
        Zc = mul(Gca, U[a], M) + mul(Gcc, L[e], M)
        Ya = mul(L[a], Gaa, M) + mul(U[e], Gca, M)    # Q-form
        Yc = mul(L[a], Gac, M) + mul(U[e], Gcc, M)
        Mx = mul(L[a], Za, Q) + mul(U[e], Zc, Q)      # M-form
        T = -mul(Dinv[e], Mx, M)                      # Q-form
        GU[a] = -mul(Za, Dinv[e], M)                  # G_ae
        GL[e] = -mul(Zc, Dinv[e], M)                  # G_ce
        GL[a] = -mul(Dinv[e], Ya, Q)                  # G_ea
        GU[e] = -mul(Dinv[e], Yc, Q)                  # G_ec
        GD[e] = Dinv[e] - mul(T, Dinv[e], M)          # G_ee
    return ld, GD, GU, GL


def check_top_cr_sparse0(Lx, Ly, seed=0, y=0.7):
    """The sparse level-0 reformulation against the full-block recursion on a
    BdG matrix (every G block the recursion returns, and ln|det|)."""
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
    A = O.hermitian_from_upper(cache.H_base) - 1j * y * np.eye(2 * p.N)
    Dg, U, L = blocks_from_dense(A, Lx, Ly)
    ld, GD, GU, GL = cr_selected_inverse(Dg, U, L)
    top = lambda X: [x[:Lx, :] for x in X]
    ldt, GDt, GUt, GLt = cr_selected_inverse_top_sparse0(top(Dg), top(U), top(L))
    err = abs(ld - ldt)
    for F, T in ((GD, GDt), (GU, GUt), (GL, GLt)):
        for f, t in zip(F, T):
            err = max(err, np.abs(f[:Lx, :] - t).max())
    return err
