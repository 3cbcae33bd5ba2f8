"""rSVD() past the wide engine's 512 sketch columns (dense_big.cpp big_rsvd_run): the reference's
rSVD (src/rSVD.cpp:72-133) takes any l; here l in (512, 4096] runs the same algorithm on the MFMA
GEMM with block CGS2 + CholeskyQR3 orthonormalisation and the block Jacobi small SVD.

Parity against the fp64 CPU oracle on the same inputs (the caller's Omega, or the engine's own
bf16-rounded Omega for bf16 A).  Tolerances: fp64 A 1e-10 on S, 1e-8 on the sign-aligned leading
half of U, V; bf16 A north_star's 1e-4."""
import numpy as np
import pytest

import oracle
from conftest import gapped_matrix, rel_fro, sign_align

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch


def _dev_colmajor(A_np, dtype):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(A_np.T)).cuda().to(dtype).t()


def _check(U, S, V, Uo, So, Vo, tol_s, tol_uv, orth):
    l = So.shape[0]
    k = l // 2
    assert rel_fro(S, So) < tol_s, rel_fro(S, So)
    eu = rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k])
    ev = rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k])
    assert eu < tol_uv and ev < tol_uv, (eu, ev)
    assert np.linalg.norm(U.T @ U - np.eye(l)) < orth
    assert np.linalg.norm(V.T @ V - np.eye(l)) < orth


def test_big_l_f64_matches_oracle(engine):
    m, n, l = 1400, 1100, 600
    A = gapped_matrix(m, n, 700, decay=0.99, seed=11)
    Om = oracle.generate_omega(n, l, 77)
    U, S, V = engine.rsvd_host(A, l, q=1, omega=Om)
    Uo, So, Vo = oracle.rsvd(A, l, q=1, Omega=Om)
    _check(U, S, V, Uo, So, Vo, 1e-10, 1e-8, 1e-9)


def test_big_l_bf16_matches_oracle(engine):
    torch = _torch()
    m, n, l = 2048, 1536, 640
    A32 = gapped_matrix(m, n, 800, decay=0.985, seed=5).astype(np.float32) * 4
    Ad = _dev_colmajor(A32, torch.bfloat16)
    A_exact = Ad.float().cpu().double().numpy()
    Om = engine.generate_omega(n, l, seed=13, dtype=torch.bfloat16).cpu().double().numpy()
    Uo, So, Vo = oracle.rsvd(A_exact, l, q=1, Omega=Om)
    U, S, V = engine.rsvd(Ad, l, q=1, seed=13)
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    _check(U, S, V, Uo, So, Vo, 1e-4, 1e-4, 1e-3)


def test_big_l_range_finder_and_limits(engine):
    """intermediate_step at l = 520 spans the oracle's Q; Power and l > 4096 are refused."""
    m, n, l = 1200, 900, 520
    A = gapped_matrix(m, n, 600, decay=0.98, seed=3)
    Om = oracle.generate_omega(n, l, 5)
    Q = engine.range_finder_host(A, Om, q=1)
    Qo = oracle.intermediate_step(A, Om, q=1)
    assert np.linalg.norm(Q.T @ Q - np.eye(l)) < 1e-9
    # same subspace: the projectors agree
    assert np.linalg.norm(Q @ (Q.T @ Qo) - Qo) < 1e-8 * np.sqrt(l)
    from rsvd_kamaneh_raganato_terrana_amd._capi import RSVDError
    from rsvd_kamaneh_raganato_terrana_amd.api import SVDMethod

    with pytest.raises(RSVDError):
        engine.rsvd_host(A, l, q=1, omega=Om, method=SVDMethod.Power)
    with pytest.raises(RSVDError):
        engine.rsvd_host(gapped_matrix(5000, 4200, 300, decay=0.9, seed=1), 4100, q=0)
