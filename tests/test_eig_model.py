"""CPU: the algorithm of wide_eig.hip (tools/eig_model.py, a numpy restatement step for step) gives
an SVD of W on gapped, clustered and rank-deficient inputs -- the columns of X = W V_w orthogonal to
far below the fp32-result tolerance (1e-6) the GPU path checks, S = |x_k| = LAPACK's to 1e-12."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import eig_model as M  # noqa: E402


def _cases():
    rng = np.random.default_rng(3)
    n = 40
    Q1 = np.linalg.qr(rng.standard_normal((n, n)))[0]
    Q2 = np.linalg.qr(rng.standard_normal((n, n)))[0]
    yield "graded", Q1 @ np.diag(0.8 ** np.arange(n)) @ Q2.T
    yield "random", rng.standard_normal((n, n))
    yield "identity", np.eye(n)
    yield "cluster", Q1 @ np.diag(np.r_[np.full(15, 3.0), np.linspace(1.0, 0.5, n - 15)]) @ Q2.T
    yield "rank3", rng.standard_normal((n, 3)) @ rng.standard_normal((3, n))


@pytest.mark.parametrize("name,W", list(_cases()))
def test_eig_model_is_an_svd(name, W):
    X, V, lam = M.small_svd(W)
    n = W.shape[0]
    # inverse iteration: |v_i . v_j| ~ eps |G| / |lam_i - lam_j| (<= 2e-4 outside the tight clusters,
    # CGS2 inside them); the Newton-Schulz step squares that
    assert np.linalg.norm(V.T @ V - np.eye(n)) < 1e-12
    S = np.linalg.svd(W, compute_uv=False)
    s = np.sort(np.linalg.norm(X, axis=0))[::-1]
    assert np.linalg.norm(s - S) <= 1e-12 * np.linalg.norm(S)
    negl = np.linalg.norm(W) ** 2 * n * n * M.EPS ** 2
    assert M.max_cos(X, negl) < 1e-8, M.max_cos(X, negl)
    assert np.abs(np.sort(lam) - np.sort(S ** 2)).max() <= 1e-13 * S[0] ** 2
