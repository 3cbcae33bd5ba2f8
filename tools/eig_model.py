"""numpy model of wide_eig.hip's small SVD (the algorithm, step for step; not the product path).

W (l x l) -> G = W^T W -> Householder tridiagonalisation (tridiag_kernel's per-column recurrence:
p = tau G v, K = tau/2 v.p, w = p - K v, G -= v w^T + w v^T) -> eigenvalues by Sturm-count
multisection on the scaled T with the three-term recurrence and power-of-two rescaling every 8
steps (tridiag_bisect_kernel) -> inverse iteration with partial pivoting, three solves
(tridiag_invit_kernel) -> CGS2 inside tight clusters (cluster_orth_kernel) -> one Newton-Schulz step
Z (3 I - Z^T Z) / 2 -> V = Q_H Z -> X = W V.
Used by tests/test_eig_model.py (CPU) and to size the design.
"""
import numpy as np

EPS = np.finfo(float).eps
CLUSTER_TOL = 1e-12


def tridiag(G):
    A = np.array(G, dtype=float, copy=True)
    n = A.shape[0]
    Y = np.zeros((n, n))
    taus = np.zeros(n)
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    for k in range(n - 2):
        x = A[k + 1:, k].copy()
        xn2 = float(np.dot(x[1:], x[1:]))
        a0 = x[0]
        if xn2 == 0.0:
            tau, beta, v = 0.0, a0, np.eye(n - k - 1)[0]
        else:
            beta = -np.copysign(np.sqrt(a0 * a0 + xn2), a0)
            tau = (beta - a0) / beta
            v = x / (a0 - beta)
            v[0] = 1.0
        p = tau * (A[k + 1:, k + 1:] @ v)
        K = 0.5 * tau * np.dot(v, p)
        w = p - K * v
        A[k + 1:, k + 1:] -= np.outer(v, w) + np.outer(w, v)
        d[k], e[k] = A[k, k], beta
        Y[k + 1:, k] = v
        taus[k] = tau
    if n >= 2:
        d[n - 2], d[n - 1], e[n - 2] = A[n - 2, n - 2], A[n - 1, n - 1], A[n - 1, n - 2]
    elif n == 1:
        d[0] = A[0, 0]
    return d, e, Y, taus


def sturm_count(d, e2, x):
    p0, p1 = 1.0, d[0] - x
    if p1 == 0.0:
        p1 = -1e-300
    c = int(p1 < 0.0)
    for i in range(1, len(d)):
        p2 = (d[i] - x) * p1 - e2[i - 1] * p0
        if p2 == 0.0:
            p2 = 1e-300 if p1 < 0.0 else -1e-300
        c += (p2 < 0.0) != (p1 < 0.0)
        p0, p1 = p1, p2
        if i % 8 == 0:
            ex = np.frexp(max(abs(p0), abs(p1)))[1]
            p0, p1 = np.ldexp(p0, -ex), np.ldexp(p1, -ex)
    return c


def eigvals_desc(d, e):
    n = len(d)
    r = np.abs(np.r_[0.0, e]) + np.abs(np.r_[e, 0.0])
    lo, hi = float((d - r).min()), float((d + r).max())
    nrm = max(abs(lo), abs(hi))
    if nrm == 0.0:
        return np.zeros(n), 0.0
    ds, e2 = d / nrm, (np.r_[e, 0.0] / nrm) ** 2
    lam = np.zeros(n)
    pad = 4.0 * n * EPS
    for jd in range(n):
        rk = n - 1 - jd
        a, b = lo / nrm - pad, hi / nrm + pad
        for _ in range(14):
            xs = a + (b - a) * np.arange(1, 65) / 65.0
            cs = np.array([sturm_count(ds, e2, x) for x in xs])
            hit = np.nonzero(cs > rk)[0]
            ms = int(hit[0]) if len(hit) else 64
            a, b = (xs[ms - 1] if ms > 0 else a), (xs[ms] if ms < 64 else b)
            if b - a <= 2 * EPS * max(abs(a), abs(b)) or b - a <= 1e-3 * EPS:
                break
        lam[jd] = 0.5 * (a + b) * nrm
    return lam, nrm


def invit(d, e, lam, tnorm, seed=0x5EED5EED, solves=2):
    n = len(d)
    tol = EPS * max(tnorm, 1e-300)
    Z = np.zeros((n, n))
    rng = np.random.default_rng(seed)
    for k, lk in enumerate(lam):
        U0 = np.zeros(n); U1 = np.zeros(n); U2 = np.zeros(n); L = np.zeros(n); P = np.zeros(n, bool)
        cd, cu = d[0] - lk, (e[0] if n > 1 else 0.0)
        for i in range(n - 1):
            bi, an, cn = e[i], d[i + 1] - lk, (e[i + 1] if i + 1 < n - 1 else 0.0)
            if abs(bi) > abs(cd):
                m = cd / bi
                U0[i], U1[i], U2[i], L[i], P[i] = bi, an, cn, m, True
                cd, cu = cu - m * an, -m * cn
            else:
                m = bi / cd if cd != 0.0 else 0.0
                U0[i], U1[i], U2[i], L[i] = cd, cu, 0.0, m
                cd, cu = an - m * cu, cn
        U0[n - 1] = cd
        small = np.abs(U0) < tol
        U0[small] = np.where(U0[small] < 0.0, -tol, tol)
        x = rng.uniform(-1.0, 1.0, n)
        for _ in range(solves):
            y = x.copy()
            for i in range(n - 1):
                if P[i]:
                    y[i], y[i + 1] = y[i + 1], y[i] - L[i] * y[i + 1]
                else:
                    y[i + 1] -= L[i] * y[i]
            z = np.zeros(n)
            for i in range(n - 1, -1, -1):
                s = y[i] - (U1[i] * z[i + 1] if i + 1 < n else 0.0) - (U2[i] * z[i + 2] if i + 2 < n else 0.0)
                z[i] = s / U0[i]
            x = z / np.abs(z).max()
        Z[:, k] = x / np.linalg.norm(x)
    return Z


def cluster_cgs2(Z, lam):
    n = len(lam)
    lmax = np.abs(lam).max() if n else 0.0
    c0 = 0
    for a in range(1, n):
        if not (lam[a - 1] - lam[a] <= CLUSTER_TOL * lmax):
            c0 = a
            continue
        for _ in range(2):
            Z[:, a] -= Z[:, c0:a] @ (Z[:, c0:a].T @ Z[:, a])
        Z[:, a] /= np.linalg.norm(Z[:, a])
    return Z


def newton_schulz(Z):
    """One step Z (3 I - Z^T Z) / 2: squares the non-orthogonality of nearly orthonormal columns."""
    return 1.5 * Z - 0.5 * Z @ (Z.T @ Z)


def small_svd(W):
    """X = W V_w (columns orthogonal), V_w orthogonal, lambda (descending) -- what the GPU hands to
    the block Jacobi's check and finish."""
    G = W.T @ W
    d, e, Y, taus = tridiag(G)
    lam, tn = eigvals_desc(d, e)
    Z = newton_schulz(cluster_cgs2(invit(d, e, lam, tn), lam))
    V = Z.copy()
    for k in range(len(d) - 3, -1, -1):
        V -= taus[k] * np.outer(Y[:, k], Y[:, k] @ V)
    return W @ V, V, lam


def max_cos(X, negl=0.0):
    C = X.T @ X
    dd = np.diag(C).copy()
    ok = dd > negl
    Cn = C[np.ix_(ok, ok)] / np.sqrt(np.outer(dd[ok], dd[ok]))
    np.fill_diagonal(Cn, 0.0)
    return float(np.abs(Cn).max()) if Cn.size else 0.0
