#!/usr/bin/env python3
"""Offline generator of the imaginary-axis pole tables used by the HIP path.

What the table approximates
---------------------------
The reference needs f(H) = (1 + e^{βH})^{-1} (src/Observables.jl:24-51) and
E_f = -Σ_n ln(1 + e^{-βE_n}) (src/HMC.jl:21-27).  With x = E' u (E' an upper
bound of the BdG spectrum) and κ = βE'/2:

    tanh(κu) ≈ Σ_q a_q · u / (u² + t_q),     u ∈ [-1, 1],  t_q > 0,  a_q > 0
    ln 2cosh(κu) ≈ C_u + (κ/2) Σ_q a_q ln(u² + t_q)

i.e. a real, odd rational approximant whose poles ±i√t_q lie on the imaginary
axis.  Each pole pair costs ONE complex no-pivot LU per leapfrog step on the
GPU (H - i y_q and H + i y_q = (H - i y_q)† share it), see DESIGN.md §2.

How it is built
---------------
tanh(κ√s)/√s is a Markov (Stieltjes) function of s = u²:
    τ(s) = Σ_{k≥1} (2/κ) / (s + ((2k-1)π/2κ)²).
A multipoint Padé approximant of a Markov function interpolating at 2m real
nodes s_j ∈ [0,1] is the m-point Gauss quadrature of the modified measure
dμ(t)/Π_j(t+s_j) — so its poles are guaranteed real-negative in s (purely
imaginary in u) with positive residues.  The Gauss rule is computed with
mpmath (Lanczos with full re-orthogonalisation); the Matsubara tail k > K is
folded in by an exact Gauss rule on its Hurwitz-zeta moments.  The 2m nodes
are then moved Remez-style (equalising the local error maxima in the
log(s + a) variable) until sup|error| stops improving.

Run: python tools/gen_pole_table.py  (≈10–30 min on 8 cores); writes
hybrid-monte-carlo-for-d-wave-sc_amd/csrc/pole_table.inc and
tests/golden/pole_table.json.  Tests re-verify every entry on a dense grid.
"""
from __future__ import annotations

import json
import math
import os
import sys
import time
from multiprocessing import Pool

import ctypes
import subprocess

import mpmath as mp
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# sup |tanh(κu) - r(u)| target on [-1, 1]; GEN_EPS selects another target
# (the tolerance-budgeted table, written next to the default one with the
# target in its name)
EPS_TANH = float(os.environ.get("GEN_EPS", "2.0e-14"))
TABLE_TAG = "" if "GEN_EPS" not in os.environ else "_eps" + os.environ["GEN_EPS"]
KAPPA_EXPONENTS = range(0, 73)   # κ = 2^(j/4), 1 .. 262144 (β = 10^4 at E' ≈ 50)
DPS = 40
# Above COMPRESS_ABOVE the Matsubara atoms k > GROUP_K0 are compressed: the
# atoms of k ∈ (a, 2a] (a = GROUP_K0·2^i) are equally weighted points of an
# equispaced grid in k, so the GROUP_NODES-point Gauss rule of the discrete
# uniform measure (Gram / discrete Chebyshev polynomials, closed-form
# recurrence) integrates every function the Lanczos process of
# multipoint_pade applies to them (polynomials in t = ((2k-1)π/2κ)² of degree
# <= 2m+1 times 1/Π_j(t + s_j), analytic in k away from Re k = 1/2) to far
# below double precision.  The κ <= 4096 entries keep every atom explicit
# (they are the round-1 entries, unchanged).  The table is verified against
# tanh itself on a dense grid either way, so the compression can only cost
# optimality, never correctness.
COMPRESS_ABOVE = 4096.0
GROUP_K0 = 512
GROUP_NODES = 100


def _gauss_from_moments(M, n):
    H = mp.matrix(n + 1, n + 1)
    for i in range(n + 1):
        for j in range(n + 1):
            H[i, j] = M[i + j]
    R = mp.cholesky(H).T
    a, b = [], []
    for j in range(n):
        aj = R[j, j + 1] / R[j, j] - (R[j - 1, j] / R[j - 1, j - 1] if j > 0 else 0)
        a.append(aj)
        if j < n - 1:
            b.append(R[j + 1, j + 1] / R[j, j])
    Jm = mp.matrix(n, n)
    for i in range(n):
        Jm[i, i] = a[i]
        if i < n - 1:
            Jm[i, i + 1] = Jm[i + 1, i] = b[i]
    E, V = mp.eigsy(Jm)
    return [E[i] for i in range(n)], [M[0] * V[0, i] ** 2 for i in range(n)]


def _hurwitz(s, a):
    """ζ(s, a) through the polygamma function (mpmath's zeta(s, a) loses
    ~50 digits for a ~ 1e3 at s ~ 40; psi stays accurate)."""
    return (-1) ** s * mp.psi(s - 1, a) / mp.factorial(s - 1)


_RULES = {}


def discrete_gauss(M, n):
    """n-point Gauss rule of the uniform measure on {0, 1, ..., M-1}:
    monic recurrence α_j = (M-1)/2, β_j = j²(M²-j²)/(4(4j²-1)) (Gram
    polynomials); nodes x_i, weights summing to M."""
    key = (M, n)
    if key not in _RULES:
        alpha = [mp.mpf(M - 1) / 2] * n
        beta = [mp.sqrt(mp.mpf(j * j * (M * M - j * j)) / (4 * (4 * j * j - 1))) for j in range(1, n)]
        _RULES[key] = gauss_jacobi_q(alpha, beta, M)
    return _RULES[key]


def matsubara_measure(kappa, ntail=10):
    """Atoms (t_k, μ_k) of τ's Stieltjes measure; tail k > K folded into ntail
    Gauss atoms of ρ = Σ_{k>K} (w/t_k) δ(1/t_k) (moments via Hurwitz zeta)."""
    kap = mp.mpf(kappa)
    w = 2 / kap

    def tk(k):
        return ((2 * k - 1) * mp.pi / (2 * kap)) ** 2

    K = int(max(40, math.ceil(kappa)))
    if kappa <= COMPRESS_ABOVE:
        t = [tk(k) for k in range(1, K + 1)]
        mu = [w] * K
    else:
        t = [tk(k) for k in range(1, GROUP_K0 + 1)]
        mu = [w] * GROUP_K0
        a = GROUP_K0
        while a < K:                    # group k = a+1 .. 2a (M = a atoms)
            x, wx = discrete_gauss(a, GROUP_NODES)
            t += [tk(a + 1 + xi) for xi in x]
            mu += [w * wi for wi in wx]
            a *= 2
        K = a
    tK = tk(K)
    with mp.workdps(3 * DPS):
        # moments of ρ in the scaled variable x' = tK / t ∈ (0, 1]
        M = [w * tK ** p * (2 * kap / mp.pi) ** (2 * p + 2) * mp.mpf(2) ** (-2 * p - 2)
             * _hurwitz(2 * p + 2, K + mp.mpf(1) / 2) for p in range(2 * ntail + 1)]
        x, rho = _gauss_from_moments(M, ntail)
    for xi, ri in zip(x, rho):
        ti = tK / xi
        t.append(ti)
        mu.append(ri * ti)
    return t, mu


_QLIB = None


def _qlib():
    """tools/pole_gauss.c (binary128 Lanczos + Golub-Welsch), built on first use."""
    global _QLIB
    if _QLIB is None:
        src = os.path.join(ROOT, "tools", "pole_gauss.c")
        so = os.path.join(ROOT, "tools", "_pole_gauss.so")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", src, "-lquadmath", "-o", so])
        lib = ctypes.CDLL(so)
        P = ctypes.POINTER(ctypes.c_double)
        lib.pg_multipoint_pade.argtypes = [ctypes.c_int, P, P, P, P, ctypes.c_int, ctypes.c_int, P, P, P]
        lib.pg_gauss_jacobi.argtypes = [ctypes.c_int, P, P, P, P, ctypes.c_double, ctypes.c_double, P, P, P, P]
        _QLIB = lib
    return _QLIB


def _dd(xs):
    """mpf list -> double-double (hi, lo) arrays"""
    hi = np.array([float(x) for x in xs])
    lo = np.array([float(x - mp.mpf(h)) for x, h in zip(xs, hi)])
    return hi, lo


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def gauss_jacobi_q(alpha, beta, mu0):
    """Gauss rule of a Jacobi matrix in binary128 (nodes ascending), as mpf."""
    n = len(alpha)
    ah, al = _dd(alpha)
    bh, bl = _dd(list(beta) + [mp.mpf(0)])
    m0 = mp.mpf(mu0)
    xh, xl, wh, wl = (np.zeros(n) for _ in range(4))
    rc = _qlib().pg_gauss_jacobi(n, _ptr(ah), _ptr(al), _ptr(bh), _ptr(bl), float(m0), float(m0 - mp.mpf(float(m0))),
                                 _ptr(xh), _ptr(xl), _ptr(wh), _ptr(wl))
    if rc != 0:
        raise RuntimeError(f"pg_gauss_jacobi failed ({rc})")
    return ([mp.mpf(float(a)) + mp.mpf(float(b)) for a, b in zip(xh, xl)],
            [mp.mpf(float(a)) + mp.mpf(float(b)) for a, b in zip(wh, wl)])


class QAtoms:
    """Atoms of a Stieltjes measure prepared once for the binary128 kernel."""

    def __init__(self, t, mu):
        self.K = len(t)
        self.th, self.tl = _dd(t)
        self.mh, self.ml = _dd(mu)


def multipoint_pade_q(atoms, m, nodes_s):
    """multipoint_pade through tools/pole_gauss.c (same Lanczos / Golub-Welsch
    process in binary128): the κ > 2048 entries, where the 40-digit mpmath
    process takes minutes per Remez iterate."""
    s = np.ascontiguousarray(np.asarray(nodes_s, dtype=np.float64))
    tq, a = np.zeros(m), np.zeros(m)
    rc = _qlib().pg_multipoint_pade(atoms.K, _ptr(atoms.th), _ptr(atoms.tl), _ptr(atoms.mh), _ptr(atoms.ml), m,
                                    len(s), _ptr(s), _ptr(tq), _ptr(a))
    if rc != 0:
        raise RuntimeError(f"pg_multipoint_pade failed ({rc})")
    return tq, a


def multipoint_pade(t, mu, m, nodes_s):
    s = [mp.mpf(float(x)) for x in nodes_s]
    K = len(t)
    nu = []
    for tk, mk in zip(t, mu):
        om = mp.mpf(1)
        for sj in s:
            om *= (tk + sj)
        nu.append(mk / om)
    tot = mp.fsum(nu)
    Q = [[mp.sqrt(x / tot) for x in nu]]
    alpha, beta = [], []
    for j in range(m):
        v = [t[i] * Q[-1][i] for i in range(K)]
        alpha.append(mp.fsum(v[i] * Q[-1][i] for i in range(K)))
        for _ in range(2):
            for qq in Q:
                c = mp.fsum(v[i] * qq[i] for i in range(K))
                v = [v[i] - c * qq[i] for i in range(K)]
        b = mp.sqrt(mp.fsum(x * x for x in v))
        if j < m - 1:
            beta.append(b)
            Q.append([x / b for x in v])
    Jm = mp.matrix(m, m)
    for i in range(m):
        Jm[i, i] = alpha[i]
        if i < m - 1:
            Jm[i, i + 1] = Jm[i + 1, i] = beta[i]
    E, V = mp.eigsy(Jm)
    tq, a = [], []
    for i in range(m):
        om = mp.mpf(1)
        for sj in s:
            om *= (E[i] + sj)
        tq.append(E[i])
        a.append(tot * V[0, i] ** 2 * om)
    order = sorted(range(m), key=lambda i: tq[i])
    return (np.array([float(tq[i]) for i in order]),
            np.array([float(a[i]) for i in order]))


def ugrid(kappa, n):
    return np.unique(np.concatenate([np.linspace(0.0, 1.0, n),
                                     np.geomspace(1e-5 / kappa, 1.0, n)]))


def tanh_error(kappa, tq, a, u):
    return np.sum(a[None, :] * u[:, None] / (u[:, None] ** 2 + tq[None, :]), axis=1) - np.tanh(kappa * u)


def phi_fit(kappa, tq, a, u):
    """C_u and sup error of ln 2cosh(κu) ≈ C_u + (κ/2) Σ a ln(u² + t)."""
    phi = np.logaddexp(kappa * u, -kappa * u)
    apx = 0.5 * kappa * np.sum(a[None, :] * np.log(u[:, None] ** 2 + tq[None, :]), axis=1)
    d = phi - apx
    return 0.5 * (d.max() + d.min()), 0.5 * (d.max() - d.min())


# entries above this κ use the binary128 kernel (tools/pole_gauss.c); the
# committed κ <= 2048 entries came from the 40-digit mpmath process
QUAD_ABOVE = 2048.0


def optimise(kappa, m, t, mu, iters=40):
    a0 = (math.pi / (2 * kappa)) ** 2
    lo, hi = math.log(a0), math.log(1 + a0)
    L = np.full(2 * m + 1, (hi - lo) / (2 * m + 1))
    u = ugrid(kappa, 20001)
    best = (np.inf, None)
    stall = 0
    atoms = QAtoms(t, mu) if kappa > QUAD_ABOVE or os.environ.get("GEN_QUAD") == "1" else None
    for _ in range(iters):
        s = np.exp(lo + np.cumsum(L)[:-1]) - a0
        if atoms is not None:
            tq, a = multipoint_pade_q(atoms, m, s)
        else:
            tq, a = multipoint_pade(t, mu, m, s)
        e = tanh_error(kappa, tq, a, u)
        sup = float(np.max(np.abs(e)))
        if sup < 0.97 * best[0]:
            stall = 0
        else:
            stall += 1
        if sup < best[0]:
            best = (sup, (tq, a))
        if stall >= 6:
            break
        edges = np.concatenate([[0.0], np.sqrt(np.maximum(s, 0.0)), [1.0]])
        E = np.array([np.max(np.abs(e[(u >= edges[i]) & (u <= edges[i + 1])]), initial=0.0) + 1e-300
                      for i in range(2 * m + 1)])
        g = math.exp(float(np.mean(np.log(E))))
        L = L * (E / g) ** (-0.08)
        L *= (hi - lo) / L.sum()
    return best


def entry(j):
    mp.mp.dps = DPS
    kappa = 2.0 ** (j / 4.0)
    t, mu = matsubara_measure(kappa)
    m = max(2, int(math.floor(2.0 + 2.35 * math.log(kappa + 1.0))))
    if kappa > COMPRESS_ABOVE:
        # the table's own trend (m ~ 3.6 ln κ - 1.5 from κ = 512 .. 2048), one
        # below it: the search below moves up or down one pole at a time
        m = max(m, int(round(3.6 * math.log(kappa) - 2.5)))
    tried = {}
    while True:
        sup, (tq, a) = optimise(kappa, m, t, mu)
        tried[m] = (sup, tq, a)
        if sup <= EPS_TANH:
            if m - 1 >= 1 and (m - 1) not in tried:
                m -= 1
                continue
            break
        if (m + 1) in tried:
            m += 1
            break
        m += 1
    sup, tq, a = tried[m]
    uf = ugrid(kappa, 400001)
    err = float(np.max(np.abs(tanh_error(kappa, tq, a, uf))))
    C_u, phierr = phi_fit(kappa, tq, a, uf)
    return dict(j=j, kappa=kappa, m=int(m), t=[float(x) for x in tq], a=[float(x) for x in a],
                C_u=float(C_u), err_tanh=err, err_phi=float(phierr))


def write_outputs(entries):
    entries = sorted(entries, key=lambda e: e["kappa"])
    jpath = os.path.join(ROOT, "tests", "golden", f"pole_table{TABLE_TAG}.json")
    with open(jpath, "w") as f:
        json.dump(dict(eps_tanh=EPS_TANH, generator="tools/gen_pole_table.py", entries=entries), f, indent=1)
    cpath = os.path.join(ROOT, "hybrid-monte-carlo-for-d-wave-sc_amd", "csrc", f"pole_table{TABLE_TAG}.inc")
    with open(cpath, "w") as f:
        f.write("// GENERATED by tools/gen_pole_table.py — do not edit.\n")
        f.write("// tanh(k u) ~ sum_q a_q u/(u^2+t_q) on [-1,1];  ln2cosh(k u) ~ C_u + k/2 sum_q a_q ln(u^2+t_q)\n")
        f.write(f"static const int kPoleTableSize = {len(entries)};\n")
        f.write("struct PoleEntry { double kappa; int m; double C_u; double err_tanh; double err_phi; int off; };\n")
        off = 0
        f.write("static const PoleEntry kPoleEntries[] = {\n")
        for e in entries:
            f.write(f"  {{{e['kappa']!r}, {e['m']}, {e['C_u']!r}, {e['err_tanh']!r}, {e['err_phi']!r}, {off}}},\n")
            off += e["m"]
        f.write("};\n")
        f.write(f"static const double kPoleT[{off}] = {{\n")
        for e in entries:
            f.write("  " + ", ".join(repr(x) for x in e["t"]) + ",\n")
        f.write("};\n")
        f.write(f"static const double kPoleA[{off}] = {{\n")
        for e in entries:
            f.write("  " + ", ".join(repr(x) for x in e["a"]) + ",\n")
        f.write("};\n")
    return jpath, cpath


def main():
    """python tools/gen_pole_table.py [j,j,...|a-b]: regenerate the listed
    entries (default: all) and merge them into the committed table."""
    js = list(KAPPA_EXPONENTS)
    keep = []
    if len(sys.argv) > 1:
        js = []
        for part in sys.argv[1].split(","):
            lo, _, hi = part.partition("-")
            js += list(range(int(lo), int(hi or lo) + 1))
        try:
            with open(os.path.join(ROOT, "tests", "golden", f"pole_table{TABLE_TAG}.json")) as f:
                keep = [e for e in json.load(f)["entries"] if e["j"] not in js]
        except OSError:
            pass
    t0 = time.time()
    procs = int(os.environ.get("GEN_PROCS", "7"))
    out = []
    with Pool(procs) as pool:
        # largest κ first so the slow ones start early
        for e in pool.imap_unordered(entry, sorted(js, reverse=True)):
            out.append(e)
            print(f"kappa={e['kappa']:9.3f} m={e['m']:2d} err_tanh={e['err_tanh']:.2e} "
                  f"err_phi={e['err_phi']:.2e}  [{time.time()-t0:.0f}s]", flush=True)
    print(write_outputs(keep + out))


if __name__ == "__main__":
    main()
