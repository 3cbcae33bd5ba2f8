"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the same inputs.

Tolerances (written per test):
* fp64 path: the reference's arithmetic class -> 1e-10 relative Frobenius on S, U, V
  (sign-aligned; gapped spectra), 1e-12 on Omega.
* fp32 path: north_star's 1e-4 relative Frobenius on U, S, V against the fp64 oracle.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import REPO, gapped_matrix, rel_fro, sign_align

pytestmark = pytest.mark.gpu

REF_INPUTS = os.path.join(REPO, "tests", "golden", "inputs.npz")


def test_omega_matches_oracle_twin(engine):
    n, l, seed = 777, 19, 12345
    om = engine.generate_omega_host(n, l, seed)
    ref = oracle.generate_omega(n, l, seed)
    assert np.max(np.abs(om - ref)) < 1e-12
    assert abs(np.mean(om)) < 0.05 and abs(np.std(om) - 1.0) < 0.05


def test_range_finder_spans_oracle_subspace_f64(engine):
    A = gapped_matrix(300, 200, 40, seed=1)
    Om = oracle.generate_omega(200, 16, 7)
    for q in (0, 1, 2):
        Q = engine.range_finder_host(A, Om, q=q)
        Qo = oracle.intermediate_step(A, Om, q=q)
        assert np.linalg.norm(Q.T @ Q - np.eye(16)) < 1e-12
        # same span <=> same orthogonal projector
        assert np.linalg.norm(Q @ Q.T - Qo @ Qo.T) < 1e-10


@pytest.mark.parametrize("m,n,l,q", [(300, 200, 16, 2), (200, 300, 32, 2), (513, 257, 10, 1), (256, 256, 64, 0)])
def test_rsvd_f64_matches_oracle(engine, m, n, l, q):
    A = gapped_matrix(m, n, 3 * l, decay=0.85, seed=m + n + l)
    Om = oracle.generate_omega(n, l, 99)
    U, S, V = engine.rsvd_host(A, l, q=q, omega=Om)
    Uo, So, Vo = oracle.rsvd(A, l, q=q, Omega=Om)
    assert rel_fro(S, So) < 1e-10
    k = l // 2  # leading, well-separated part of the spectrum
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < 1e-8
    assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < 1e-8
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-10
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-10
    # reconstruction error identical to the oracle's
    e = np.linalg.norm(A - (U * S) @ V.T)
    eo = np.linalg.norm(A - (Uo * So) @ Vo.T)
    assert abs(e - eo) <= 1e-10 * np.linalg.norm(A)


def test_identity_known_answer(engine):
    """input/sparse_matrix100.mtx = I_100: S == 1, ||A - U S V^T||_F = sqrt(100 - l)."""
    A = np.eye(100)
    for l in (10, 16):
        U, S, V = engine.rsvd_host(A, l, seed=0x5EED0001)
        assert np.max(np.abs(S - 1.0)) < 1e-12
        assert abs(np.linalg.norm(A - (U * S) @ V.T) - np.sqrt(100 - l)) < 1e-10


def test_rsvd_f32_device_matches_oracle(engine):
    import torch

    m, n, l = 1024, 768, 64
    A64 = gapped_matrix(m, n, 128, decay=0.9, seed=3)
    A32 = A64.astype(np.float32)
    Om = oracle.generate_omega(n, l, 5)
    Uo, So, Vo = oracle.rsvd(A32.astype(np.float64), l, q=2, Omega=Om.astype(np.float32).astype(np.float64))
    At = torch.from_numpy(np.asfortranarray(A32)).cuda()
    At = At.t().contiguous().t()
    U, S, V = engine.rsvd(At, l, q=2, omega=torch.from_numpy(Om.astype(np.float32)))
    torch.cuda.synchronize()
    U, S, V = U.cpu().double().numpy(), S.cpu().double().numpy(), V.cpu().double().numpy()
    assert rel_fro(S, So) < 1e-4
    k = 32
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < 1e-4
    assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < 1e-4


def _ref_rank2(n=100):
    """input/sparse_matrix.mtx (python/matrix_maker.py): A[i][j] = i*n + j + 1, rank 2."""
    return np.asfortranarray(np.arange(1, n * n + 1, dtype=np.float64).reshape(n, n))


@pytest.mark.parametrize("l", [4, 16])
def test_rank_deficient_rank2_known_answer(engine, l):
    """Y = A Omega has rank 2 < l: CholeskyQR breaks down and the robust path must take over."""
    A = _ref_rank2()
    U, S, V = engine.rsvd_host(A, l, seed=0x5EED0001)
    Uo, So, Vo = oracle.rsvd(A, l, q=2, seed=0x5EED0001)
    sv = np.linalg.svd(A, compute_uv=False)
    assert abs(S[0] - sv[0]) < 1e-10 * sv[0] and abs(S[1] - sv[1]) < 1e-8 * sv[0]
    assert np.max(np.abs(S[2:])) < 1e-9 * sv[0]
    assert rel_fro(S, So) < 1e-10
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-10
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-10
    assert np.linalg.norm(A - (U * S) @ V.T) < 1e-9 * np.linalg.norm(A)
    assert engine.info()["cholqr_fallbacks"] > 0


def test_zero_matrix(engine):
    A = np.zeros((64, 48), order="F")
    U, S, V = engine.rsvd_host(A, 8)
    assert np.all(S == 0.0)
    assert np.linalg.norm(U.T @ U - np.eye(8)) < 1e-10
    assert np.linalg.norm(V.T @ V - np.eye(8)) < 1e-10


def test_duplicate_columns_f32_device(engine):
    import torch

    rng = np.random.default_rng(11)
    B = rng.standard_normal((512, 6))
    A = np.asfortranarray(np.repeat(B, 40, axis=1)[:, :200])  # rank 6, l = 32
    At = torch.from_numpy(A.astype(np.float32)).cuda().t().contiguous().t()
    U, S, V = engine.rsvd(At, 32, q=2, seed=3)
    torch.cuda.synchronize()
    U, S, V = U.cpu().double().numpy(), S.cpu().double().numpy(), V.cpu().double().numpy()
    sv = np.linalg.svd(A, compute_uv=False)
    assert rel_fro(S[:6], sv[:6]) < 1e-5
    assert np.max(np.abs(S[6:])) < 1e-4 * sv[0]
    assert np.linalg.norm(U.T @ U - np.eye(32)) < 1e-4
    assert np.linalg.norm(V.T @ V - np.eye(32)) < 1e-4
    assert np.linalg.norm(A - (U * S) @ V.T) < 1e-5 * np.linalg.norm(A)


@pytest.mark.parametrize("mode", [1, 2])  # QRMode.GS2, QRMode.CholQR2
def test_qr_modes_agree_with_oracle(engine, mode):
    import torch

    m, n, l = 400, 300, 24
    A = gapped_matrix(m, n, 3 * l, decay=0.85, seed=17)
    Om = oracle.generate_omega(n, l, 4)
    Uo, So, Vo = oracle.rsvd(A, l, q=2, Omega=Om)
    At = torch.from_numpy(A).cuda().t().contiguous().t()
    U, S, V = engine.rsvd(At, l, q=2, omega=torch.from_numpy(Om), qr_mode=mode)
    torch.cuda.synchronize()
    U, S, V = U.cpu().numpy(), S.cpu().numpy(), V.cpu().numpy()
    assert rel_fro(S, So) < 1e-10
    k = l // 2
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < 1e-8
    assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < 1e-8
