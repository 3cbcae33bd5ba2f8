"""The small SVD through the symmetric eigensolver (wide_eig.hip; fp32 results, l > 64) against the
fp64 oracle's SVD<Jacobi> (include/SVD_class.hpp:100-180 via oracle/rsvd_oracle.c).

The eigensolver path (G = W^T W, Householder tridiagonalisation, multisection, inverse iteration,
compact-WY back-transformation) ends in the block Jacobi's orthogonality check; `jacobi_sweeps`
(rsvd_get_info) is 0 when the check accepted the eigensolver's X = W V_w as it stands.  Tolerance:
north_star's 1e-4 relative Frobenius on S and on the sign-aligned leading half of U, V (fp32
results), U and V orthonormal to 1e-4.
"""
import os
import sys

import numpy as np
import pytest

import oracle
from conftest import gapped_matrix, rel_fro, sign_align

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torch():
    import torch

    return torch


def _dev_colmajor(A_np, dtype):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(A_np.T)).cuda().to(dtype).t()


def _run_bf16(engine, A32, l, q, seed, dtype=None, scale=1.0):
    torch = _torch()
    dtype = dtype or torch.bfloat16
    Ad = _dev_colmajor(A32 / scale, dtype)
    A_exact = Ad.float().cpu().double().numpy() * scale
    Om = engine.generate_omega(A32.shape[1], l, seed=seed, dtype=dtype)
    torch.cuda.synchronize()
    Uo, So, Vo = oracle.rsvd(A_exact, l, q=q, Omega=Om.cpu().double().numpy())
    U, S, V = engine.rsvd(Ad, l, q=q, seed=seed, a_scale=scale)
    torch.cuda.synchronize()
    info = engine.info()
    return [x.cpu().double().numpy() for x in (U, S, V)], (Uo, So, Vo), A_exact, info


def _check(res, ref, A, frac=0.5, tol=1e-4):
    (U, S, V), (Uo, So, Vo) = res, ref
    l = S.shape[0]
    k = max(1, int(l * frac))
    assert np.linalg.norm(U.T @ U - np.eye(l)) < tol
    assert np.linalg.norm(V.T @ V - np.eye(l)) < tol
    assert rel_fro(S, So) < tol, rel_fro(S, So)
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < tol
    assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < tol
    e = np.linalg.norm(A - (U * S) @ V.T)
    eo = np.linalg.norm(A - (Uo * So) @ Vo.T)
    assert abs(e - eo) <= tol * np.linalg.norm(A) * 10, (e, eo)


@pytest.mark.parametrize("m,n,l,q", [(3000, 2048, 256, 2), (2500, 1800, 130, 1), (2600, 2100, 512, 2),
                                     (2048, 1500, 300, 1)])
def test_eig_small_svd_bf16(engine, m, n, l, q):
    """LP = 256 (four tridiagonalisation workgroups), 256 with l = 130, 512 (sixteen), 512 with
    l = 300: the padded sizes.  The gapped spectrum's X passes the check as computed."""
    A32 = gapped_matrix(m, n, 2 * l, decay=0.97, seed=l + 3).astype(np.float32) * 10
    res, ref, A, info = _run_bf16(engine, A32, l, q, seed=41)
    _check(res, ref, A)
    assert info["jacobi_sweeps"] == 0, info


def test_eig_small_svd_bench_spectrum(engine):
    """The bench's own matrix family (bench.make_A: 128 directions at 0.9^t + 1e-3 noise, so about
    two thirds of the l = 256 Ritz values sit in the noise cluster) at a size the oracle finishes
    in seconds."""
    torch = _torch()
    sys.path.insert(0, REPO)
    import bench

    m, n, l = 4096, 4096, 256
    A, _ = bench.make_A(torch, m, n, 0, "bf16")
    A32 = A.float().cpu().numpy()
    res, ref, Ax, info = _run_bf16(engine, A32, l, 2, seed=0x5EED0002)
    _check(res, ref, Ax, frac=0.25)
    assert info["jacobi_sweeps"] == 0, info


def _hadamard(m):
    H = np.ones((1, 1))
    while H.shape[0] < m:
        H = np.block([[H, H], [H, -H]])
    return H


@pytest.mark.parametrize("blocks", [((8.0, 100), (4.0, 100), (2.0, 100), (1.0, 724)), ((1.0, 1024),)])
def test_eig_small_svd_clusters(engine, blocks):
    """Exactly repeated singular values (orthogonal +-1 Hadamard columns scaled by powers of two,
    exact in bf16): the Gram's eigenvalues come in clusters of 100 (or one cluster of all l),
    where inverse iteration alone returns dependent vectors and the cluster CGS2 must supply an
    orthonormal basis."""
    m, n, l = 2048, 1024, 256
    sig = np.concatenate([np.full(c, v) for v, c in blocks])
    A32 = (_hadamard(m)[:, :n] * sig).astype(np.float32)
    res, ref, A, info = _run_bf16(engine, A32, l, 2, seed=7)
    U, S, V = res
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-4
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-4
    assert rel_fro(S, ref[1]) < 1e-4, rel_fro(S, ref[1])
    e = np.linalg.norm(A - (U * S) @ V.T)
    eo = np.linalg.norm(A - (ref[0] * ref[1]) @ ref[2].T)
    assert abs(e - eo) <= 1e-4 * np.linalg.norm(A), (e, eo)


def test_eig_small_svd_e4m3_l512(engine):
    """C5's kernel instantiation: e4m3 A, l = 512."""
    torch = _torch()
    m, n, l = 4096, 2048, 512
    A32 = gapped_matrix(m, n, 700, decay=0.985, seed=5).astype(np.float32)
    scale = float(np.abs(A32).max()) / 400.0
    res, ref, A, info = _run_bf16(engine, A32, l, 2, seed=19, dtype=torch.float8_e4m3fn, scale=scale)
    _check(res, ref, A, frac=0.25)
