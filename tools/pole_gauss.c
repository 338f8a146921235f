/* Quad-precision kernels of the pole-table generator (tools/gen_pole_table.py).
 *
 * The multipoint Padé approximant of tanh(κ√s)/√s is the m-point Gauss rule
 * of the modified Matsubara measure ν_k = μ_k / Π_j (t_k + s_j) (see the
 * generator's docstring).  mpmath at 40 digits takes minutes per Remez iterate
 * once κ is large (m ≈ 40 poles over ≈ 1400 atoms); this file does the same
 * Lanczos process (full re-orthogonalisation, two passes) and the Golub-Welsch
 * eigenproblem in IEEE binary128 (113-bit significand, ≈ 34 digits) through
 * gcc's __float128.  Inputs and outputs that must keep more than double
 * precision travel as double-double pairs (hi, lo).
 *
 * Build: gcc -O2 -shared -fPIC tools/pole_gauss.c -lquadmath -o tools/_pole_gauss.so
 * (the generator builds it on first use).  Offline tooling only: nothing in
 * the product path or the GPU runs loads it.
 */
#include <quadmath.h>
#include <stdlib.h>
#include <string.h>

typedef __float128 q;

static q dd(const double* hi, const double* lo, int i) { return (q)hi[i] + (q)lo[i]; }
static void to_dd(q x, double* hi, double* lo, int i) {
  const double h = (double)x;
  hi[i] = h;
  lo[i] = (double)(x - (q)h);
}

/* Symmetric tridiagonal eigenproblem (diagonal d[0..n), off-diagonal e[0..n-1))
 * by implicit QL with Wilkinson shifts; z (n x n, row-major) accumulates the
 * eigenvectors (z[r*n + c] = component r of eigenvector c).  Returns 0 on
 * success. */
static int tql(int n, q* d, q* e, q* z) {
  for (int i = 0; i < n * n; ++i) z[i] = 0;
  for (int i = 0; i < n; ++i) z[i * n + i] = 1;
  if (n == 1) return 0;
  q* ee = (q*)calloc((size_t)n, sizeof(q));
  for (int i = 0; i < n - 1; ++i) ee[i] = e[i];
  ee[n - 1] = 0;
  for (int l = 0; l < n; ++l) {
    int iter = 0, m;
    do {
      for (m = l; m < n - 1; ++m) {
        const q dsum = fabsq(d[m]) + fabsq(d[m + 1]);
        if (fabsq(ee[m]) <= FLT128_EPSILON * dsum) break;
      }
      if (m != l) {
        if (iter++ == 200) {
          free(ee);
          return -1;
        }
        q g = (d[l + 1] - d[l]) / (2 * ee[l]);
        q r = hypotq(g, (q)1);
        g = d[m] - d[l] + ee[l] / (g + (g >= 0 ? fabsq(r) : -fabsq(r)));
        q s = 1, c = 1, p = 0;
        int i;
        for (i = m - 1; i >= l; --i) {
          q f = s * ee[i], b = c * ee[i];
          r = hypotq(f, g);
          ee[i + 1] = r;
          if (r == 0) {
            d[i + 1] -= p;
            ee[m] = 0;
            break;
          }
          s = f / r;
          c = g / r;
          g = d[i + 1] - p;
          r = (d[i] - g) * s + 2 * c * b;
          p = s * r;
          d[i + 1] = g + p;
          g = c * r - b;
          for (int k = 0; k < n; ++k) {
            f = z[k * n + i + 1];
            z[k * n + i + 1] = s * z[k * n + i] + c * f;
            z[k * n + i] = c * z[k * n + i] - s * f;
          }
        }
        if (r == 0 && i >= l) continue;
        d[l] -= p;
        ee[l] = g;
        ee[m] = 0;
      }
    } while (m != l);
  }
  free(ee);
  return 0;
}

/* Gauss weight of node x of the Jacobi matrix (alpha, beta) for a measure of
 * total mass mu0: w = mu0 / Σ_j p_j(x)² with the orthonormal polynomials of the
 * three-term recurrence.  Unlike mu0 · v_0² from the eigenvectors (absolute
 * accuracy only), this keeps the relative accuracy of the tiny weights of far
 * nodes: the sum is dominated by its large terms. */
static q gauss_weight(int n, const q* alpha, const q* beta, q mu0, q x) {
  q pm = 0, p = 1, sum = 1;
  for (int j = 0; j < n - 1; ++j) {
    const q pn = ((x - alpha[j]) * p - (j > 0 ? beta[j - 1] * pm : 0)) / beta[j];
    pm = p;
    p = pn;
    sum += p * p;
  }
  return mu0 / sum;
}

/* Gauss rule from a Jacobi matrix: n nodes (ascending), weights from gauss_weight.
 * alpha[n], beta[n-1] as double-double; outputs double-double. */
int pg_gauss_jacobi(int n, const double* ah, const double* al, const double* bh, const double* bl, double mu0h,
                    double mu0l, double* xh, double* xl, double* wh, double* wl) {
  q* d = (q*)malloc(sizeof(q) * n);
  q* e = (q*)malloc(sizeof(q) * (n > 1 ? n - 1 : 1));
  q* z = (q*)malloc(sizeof(q) * n * n);
  q* a0 = (q*)malloc(sizeof(q) * n);
  q* b0 = (q*)malloc(sizeof(q) * (n > 1 ? n - 1 : 1));
  for (int i = 0; i < n; ++i) a0[i] = d[i] = dd(ah, al, i);
  for (int i = 0; i < n - 1; ++i) b0[i] = e[i] = dd(bh, bl, i);
  const int rc = tql(n, d, e, z);
  const q mu0 = (q)mu0h + (q)mu0l;
  int* ord = (int*)malloc(sizeof(int) * n);
  for (int i = 0; i < n; ++i) ord[i] = i;
  for (int i = 1; i < n; ++i)   /* insertion sort by eigenvalue */
    for (int j = i; j > 0 && d[ord[j]] < d[ord[j - 1]]; --j) {
      const int t = ord[j];
      ord[j] = ord[j - 1];
      ord[j - 1] = t;
    }
  for (int i = 0; i < n; ++i) {
    const int c = ord[i];
    to_dd(d[c], xh, xl, i);
    to_dd(gauss_weight(n, a0, b0, mu0, d[c]), wh, wl, i);
  }
  free(b0);
  free(a0);
  free(ord);
  free(z);
  free(e);
  free(d);
  return rc;
}

/* m-point multipoint Padé of the Stieltjes function with atoms (t_k, μ_k),
 * k < K, interpolating at the ns nodes s_j: Lanczos on diag(t) from the start
 * vector √(ν/Σν), then the Jacobi matrix's eigenvalues (implicit QL) and
 * the Gauss weights from the recurrence (gauss_weight).  Outputs the poles t_q
 * (ascending) and residues a_q = w_q · Π_j (t_q + s_j) as doubles.  Returns 0 on success. */
int pg_multipoint_pade(int K, const double* th, const double* tl, const double* muh, const double* mul, int m,
                       int ns, const double* s, double* tq_out, double* a_out) {
  if (m < 1 || m > K) return -2;
  q* t = (q*)malloc(sizeof(q) * K);
  q* nu = (q*)malloc(sizeof(q) * K);
  q* Q = (q*)malloc(sizeof(q) * (size_t)m * K);
  q* v = (q*)malloc(sizeof(q) * K);
  q* alpha = (q*)malloc(sizeof(q) * m);
  q* beta = (q*)malloc(sizeof(q) * m);
  q* z = (q*)malloc(sizeof(q) * m * m);
  q tot = 0;
  for (int k = 0; k < K; ++k) {
    t[k] = dd(th, tl, k);
    q om = 1;
    for (int j = 0; j < ns; ++j) om *= t[k] + (q)s[j];
    nu[k] = dd(muh, mul, k) / om;
    tot += nu[k];
  }
  for (int k = 0; k < K; ++k) Q[k] = sqrtq(nu[k] / tot);
  int rc = 0;
  for (int j = 0; j < m; ++j) {
    const q* qj = Q + (size_t)j * K;
    q a = 0;
    for (int k = 0; k < K; ++k) {
      v[k] = t[k] * qj[k];
      a += v[k] * qj[k];
    }
    alpha[j] = a;
    for (int pass = 0; pass < 2; ++pass)
      for (int i = 0; i <= j; ++i) {
        const q* qi = Q + (size_t)i * K;
        q c = 0;
        for (int k = 0; k < K; ++k) c += v[k] * qi[k];
        for (int k = 0; k < K; ++k) v[k] -= c * qi[k];
      }
    q b = 0;
    for (int k = 0; k < K; ++k) b += v[k] * v[k];
    b = sqrtq(b);
    if (j < m - 1) {
      if (b == 0) {
        rc = -3;
        break;
      }
      beta[j] = b;
      q* qn = Q + (size_t)(j + 1) * K;
      for (int k = 0; k < K; ++k) qn[k] = v[k] / b;
    }
  }
  q* lam = (q*)malloc(sizeof(q) * m);
  q* ework = (q*)malloc(sizeof(q) * m);
  for (int i = 0; i < m; ++i) lam[i] = alpha[i];
  for (int i = 0; i < m - 1; ++i) ework[i] = beta[i];
  if (rc == 0) rc = tql(m, lam, ework, z);
  if (rc == 0) {
    int* ord = (int*)malloc(sizeof(int) * m);
    for (int i = 0; i < m; ++i) ord[i] = i;
    for (int i = 1; i < m; ++i)
      for (int j = i; j > 0 && lam[ord[j]] < lam[ord[j - 1]]; --j) {
        const int tt = ord[j];
        ord[j] = ord[j - 1];
        ord[j - 1] = tt;
      }
    for (int i = 0; i < m; ++i) {
      const int c = ord[i];
      q om = 1;
      for (int j = 0; j < ns; ++j) om *= lam[c] + (q)s[j];
      tq_out[i] = (double)lam[c];
      a_out[i] = (double)(gauss_weight(m, alpha, beta, tot, lam[c]) * om);
    }
    free(ord);
  }
  free(ework);
  free(lam);
  free(z);
  free(beta);
  free(alpha);
  free(v);
  free(Q);
  free(nu);
  free(t);
  return rc;
}
