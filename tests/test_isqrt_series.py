"""The G^-1/2 series of the deferred second CholeskyQR pass (wide_eig.hip launch_isqrt_near_identity),
restated in numpy: the same coefficients, the same Paterson-Stockmeyer evaluation
M = B0 + E^3 (B1 + E^3 B2), B_i = c_{3i} I + c_{3i+1} E + c_{3i+2} E^2, and the cut-off |E|_F <= 0.1
past which the engine takes the Cholesky factor instead.  The GPU path itself is pinned against the
oracle by tests/test_gpu_switches.py (default and RSVD_ISQRT_CUT=0) and every wide parity test."""
import numpy as np
import pytest
from scipy.special import binom

# kIsqrtC in wide_eig.hip: binom(-1/2, k), k = 0..8
C = [1.0, -0.5, 0.375, -0.3125, 0.2734375, -0.24609375, 0.2255859375, -0.20947265625, 0.196380615234375]
CUT = 0.1


def isqrt_series(G):
    n = G.shape[0]
    I = np.eye(n)
    E = G - I
    E2 = E @ E
    E3 = E2 @ E
    B2 = C[6] * I + C[7] * E + C[8] * E2
    B1T = C[3] * I + C[4] * E + C[5] * E2 + E3 @ B2
    return C[0] * I + C[1] * E + C[2] * E2 + E3 @ B1T


def test_coefficients_are_the_binomial_series():
    assert C == [float(binom(-0.5, k)) for k in range(9)]


@pytest.mark.parametrize("eps", [1e-6, 1e-3, 0.03, CUT])
def test_series_orthonormalises_near_identity_gram(eps):
    rng = np.random.default_rng(7)
    m, l = 2000, 96
    T1 = np.linalg.qr(rng.standard_normal((m, l)))[0]
    # perturb to |T1^T T1 - I|_F = eps (the first pass's departure from orthonormality)
    D = rng.standard_normal((l, l))
    D = (D + D.T) / 2
    D *= eps / 2 / np.linalg.norm(D)
    T1 = T1 @ (np.eye(l) + D)
    G = T1.T @ T1
    e = np.linalg.norm(G - np.eye(l))
    assert e <= 1.2 * eps
    M = isqrt_series(G)
    Q = T1 @ M
    # the degree-8 remainder bound 0.19 |E|^9 plus rounding
    assert np.linalg.norm(Q.T @ Q - np.eye(l)) <= 0.2 * e ** 9 * 4 + 1e-13
    # and it spans span(T1) (M is nonsingular), symmetric like G^-1/2
    assert np.allclose(M, M.T, atol=1e-15)
    w, V = np.linalg.eigh(G)
    assert np.linalg.norm(M - (V / np.sqrt(w)) @ V.T) <= 0.2 * e ** 9 * 4 + 1e-13
