"""The library's own fp64 MFMA product (csrc/dwhmc_gemm.hip: dwh_debug_gemm)
against numpy: complex (3 real MFMAs per complex MAC) and real, every op
combination the measurement path uses (U^H (J U), (U f) U^H, V^H U,
U - V W2, Z Z^T, the Löwdin update), batched, ragged sizes (not multiples of
the 64 x 64 tile or the 16-deep K chunk), alpha / beta.  Tolerance: fp64
rounding of K-term sums, |ΔC| <= 1e-13 sqrt(K) (1 + max|C|) with entries of
O(1)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _op(x, op):
    return x if op == "N" else x.conj().swapaxes(-1, -2)


def run_gemm(lib, opa, opb, M, N, K, alpha, beta, batch, cplx, seed):
    rng = np.random.default_rng(seed)
    dt = np.complex128 if cplx else np.float64

    def rnd(*shape):
        x = rng.uniform(-1, 1, shape)
        if cplx:
            x = x + 1j * rng.uniform(-1, 1, shape)
        return x.astype(dt)

    ar, ac = (M, K) if opa == "N" else (K, M)
    br, bc = (K, N) if opb == "N" else (N, K)
    lda, ldb, ldc = ar + 3, br + 1, M + 2      # padded leading dimensions
    A = rnd(batch, ac, lda)                    # column-major: [batch][col][row]
    B = rnd(batch, bc, ldb)
    Cm = rnd(batch, N, ldc)
    Am = A[:, :, :ar].swapaxes(1, 2)           # (batch, rows, cols)
    Bm = B[:, :, :br].swapaxes(1, 2)
    C0 = Cm[:, :, :M].swapaxes(1, 2).copy()
    ref = alpha * (_op(Am, opa) @ _op(Bm, opb)) + beta * C0
    al = np.array([np.real(alpha), np.imag(alpha)])
    be = np.array([np.real(beta), np.imag(beta)])
    out = np.ascontiguousarray(Cm)
    rc = lib.dwh_debug_gemm(0, int(cplx), opa.encode(), opb.encode(), M, N, K, al.ctypes.data_as(C.c_void_p),
                            np.ascontiguousarray(A).ctypes.data_as(C.c_void_p), lda,
                            np.ascontiguousarray(B).ctypes.data_as(C.c_void_p), ldb,
                            be.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p), ldc, batch)
    assert rc == 0, lib.dwh_last_error(None).decode()
    got = out[:, :, :M].swapaxes(1, 2)
    # the padding rows of C are untouched
    assert np.array_equal(out[:, :, M:], Cm[:, :, M:])
    err = np.max(np.abs(got - ref))
    tol = 1e-13 * np.sqrt(max(K, 1)) * (1 + np.max(np.abs(ref)))
    return err, tol


@pytest.mark.parametrize("cplx", [True, False])
@pytest.mark.parametrize("opa,opb", [("N", "N"), ("C", "N"), ("N", "C"), ("C", "C")])
@pytest.mark.parametrize("M,N,K,batch", [(64, 64, 16, 1), (100, 37, 53, 3), (1, 1, 1, 2), (130, 200, 2, 1),
                                         (17, 300, 257, 2), (256, 128, 512, 1)])
def test_gemm_matches_numpy(dwhmc, cplx, opa, opb, M, N, K, batch):
    lib = dwhmc.load_library()
    alpha = (0.75 - 0.5j) if cplx else -0.5
    beta = (1.5 + 0.25j) if cplx else 1.5
    err, tol = run_gemm(lib, opa, opb, M, N, K, alpha, beta, batch, cplx, seed=M * 7 + N + K)
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("cplx", [True, False])
def test_gemm_beta_zero_ignores_c(dwhmc, cplx):
    """beta = 0 overwrites C; K = 0 gives beta C."""
    lib = dwhmc.load_library()
    err, tol = run_gemm(lib, "C", "N", 70, 90, 33, 1.0, 0.0, 2, cplx, seed=5)
    assert err <= tol
    err, tol = run_gemm(lib, "N", "N", 40, 20, 0, 1.0, 2.0, 1, cplx, seed=6)
    assert err <= tol


def test_gemm_measurement_size(dwhmc):
    """The J_mn product at L = 32 (n = 2048): U^H (J U) for a unitary U."""
    lib = dwhmc.load_library()
    err, tol = run_gemm(lib, "C", "N", 2048, 2048, 2048, 1.0, 0.0, 1, True, seed=9)
    assert err <= tol, (err, tol)
