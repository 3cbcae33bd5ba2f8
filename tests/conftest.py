"""Test configuration: the `gpu` marker, repo import path, shared fixtures.

CPU-only tests (`-m "not gpu"`) cover the oracle (against the golden vectors), the host logic
and the C-ABI library's exports.  `-m gpu` tests call the HIP engine through the C ABI and
compare with the oracle (oracle/), which is test infrastructure only.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librsvd_hip.so)")


@pytest.fixture(scope="session")
def engine():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rsvd_kamaneh_raganato_terrana_amd as R

    eng = R.Engine(0)
    yield eng
    eng.close()


def sign_align(X, Xref):
    """Flip columns of X to match Xref (singular vectors are defined up to sign)."""
    s = np.sign(np.sum(X * Xref, axis=0))
    s[s == 0] = 1.0
    return X * s


def rel_fro(X, Xref):
    den = np.linalg.norm(Xref)
    return np.linalg.norm(X - Xref) / (den if den > 0 else 1.0)


def gapped_matrix(m, n, rank, decay=0.9, noise=1e-3, seed=0, dtype=np.float64):
    """A = X diag(sigma) Y^T / sqrt(n) + noise*N : the SURVEY.md §8(d) synthetic family."""
    rng = np.random.default_rng(seed)
    X = np.linalg.qr(rng.standard_normal((m, rank)))[0]
    Y = np.linalg.qr(rng.standard_normal((n, rank)))[0]
    sig = decay ** np.arange(rank)
    A = (X * sig) @ Y.T + noise * rng.standard_normal((m, n)) / np.sqrt(max(m, n))
    return np.asfortranarray(A.astype(dtype))
