"""GPU parity of the wide engine (l > 64, bf16 / e4m3 A) against the fp64 CPU oracle.

Same inputs on both sides: the oracle runs on the exact values the GPU sees (bf16 / e4m3 A
dequantised to fp64, the Omega the engine draws -- Philox rounded to bf16 / e4m3, obtained
through rsvd_generate_omega).  Tolerances (written per test):
* fp64 A: 1e-10 relative Frobenius on S, 1e-8 on the sign-aligned leading half of U, V.
* fp32 / bf16 / e4m3 A: north_star's 1e-4 relative Frobenius on S and on the leading half of
  U, V (the trailing singular vectors of a 0.9^t spectrum are not determined to 1e-4 by fp32
  panels; the reconstruction error is compared instead).
"""
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
    t = torch.from_numpy(np.ascontiguousarray(A_np.T)).cuda().to(dtype)  # n x m row-major == A col-major
    return t.t()


def _check(U, S, V, Uo, So, Vo, A, tol_s, tol_uv, frac=0.5):
    l = So.shape[0]
    k = max(1, int(l * frac))
    assert rel_fro(S, So) < tol_s, rel_fro(S, So)
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < tol_uv
    assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < tol_uv
    e = np.linalg.norm(A - (U * S) @ V.T)
    eo = np.linalg.norm(A - (Uo * So) @ Vo.T)
    assert abs(e - eo) <= max(tol_s, 1e-12) * np.linalg.norm(A) * 10, (e, eo)


@pytest.mark.parametrize("m,n,l,q", [(600, 400, 80, 2), (512, 700, 128, 1), (800, 640, 200, 2)])
def test_wide_f64_matches_oracle(engine, m, n, l, q):
    A = gapped_matrix(m, n, 2 * l, decay=0.95, seed=m + l)
    Om = oracle.generate_omega(n, l, 31)
    U, S, V = engine.rsvd_host(A, l, q=q, omega=Om)
    Uo, So, Vo = oracle.rsvd(A, l, q=q, Omega=Om)
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-10
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-10
    _check(U, S, V, Uo, So, Vo, A, 1e-10, 1e-8)


def test_wide_f64_l512(engine):
    m, n, l = 1100, 900, 512
    A = gapped_matrix(m, n, 600, decay=0.99, seed=7)
    Om = oracle.generate_omega(n, l, 3)
    U, S, V = engine.rsvd_host(A, l, q=1, omega=Om)
    Uo, So, Vo = oracle.rsvd(A, l, q=1, Omega=Om)
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-9
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-9
    _check(U, S, V, Uo, So, Vo, A, 1e-10, 1e-8, frac=0.25)


def test_wide_f32_device(engine):
    torch = _torch()
    m, n, l = 2048, 1024, 128
    A = gapped_matrix(m, n, 256, decay=0.97, seed=11).astype(np.float32)
    Om = oracle.generate_omega(n, l, 5).astype(np.float32)
    Uo, So, Vo = oracle.rsvd(A.astype(np.float64), l, q=2, Omega=Om.astype(np.float64))
    U, S, V = engine.rsvd(_dev_colmajor(A, torch.float32), l, q=2, omega=torch.from_numpy(Om))
    torch.cuda.synchronize()
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    _check(U, S, V, Uo, So, Vo, A.astype(np.float64), 1e-4, 1e-4)


# (4096, 1024, 128, 1) and (2048, 900, 100, 2) run the two-k-step TN (LP = 128, m % 64 == 0: the
# separate-ring wproj3tn128_kernel);
# (1000, 700, 128, 1) the single-step fallback (m % 64 != 0)
@pytest.mark.parametrize("m,n,l,q", [(4096, 1024, 128, 1), (2048, 3000, 256, 2), (1024, 1536, 64, 2),
                                     (700, 500, 16, 0), (1000, 700, 128, 1), (2048, 900, 100, 2)])
def test_bf16_matches_oracle(engine, m, n, l, q):
    torch = _torch()
    A32 = gapped_matrix(m, n, 2 * l, decay=0.95, seed=l + q).astype(np.float32) * 10
    Ad = _dev_colmajor(A32, torch.bfloat16)
    A_exact = Ad.float().cpu().double().numpy()  # the bf16 values the GPU sees
    Om = engine.generate_omega(n, l, seed=77, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    Om_np = Om.cpu().double().numpy()
    # Omega is bf16: every value has at most 8 significant bits
    assert np.array_equal(Om_np, torch.from_numpy(Om_np).to(torch.bfloat16).double().numpy())
    Uo, So, Vo = oracle.rsvd(A_exact, l, q=q, Omega=Om_np)
    U, S, V = engine.rsvd(Ad, l, q=q, seed=77)
    torch.cuda.synchronize()
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-4
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-4
    _check(U, S, V, Uo, So, Vo, A_exact, 1e-4, 1e-4)


def test_bf16_explicit_omega_equals_seeded(engine):
    torch = _torch()
    m, n, l = 1500, 900, 128
    A = _dev_colmajor(gapped_matrix(m, n, 200, seed=2).astype(np.float32), torch.bfloat16)
    Om = engine.generate_omega(n, l, seed=5, dtype=torch.bfloat16)
    U1, S1, V1 = engine.rsvd(A, l, q=1, seed=5)
    U2, S2, V2 = engine.rsvd(A, l, q=1, omega=Om)
    torch.cuda.synchronize()
    assert torch.equal(S1, S2) and torch.equal(U1, U2) and torch.equal(V1, V2)


def test_fp8_matches_oracle(engine):
    torch = _torch()
    m, n, l = 3000, 2048, 256
    A32 = gapped_matrix(m, n, 512, decay=0.97, seed=9).astype(np.float32)
    scale = float(np.abs(A32).max()) / 400.0
    A8 = _dev_colmajor(A32 / scale, torch.float8_e4m3fn)
    A_exact = A8.float().cpu().double().numpy() * scale
    Om = engine.generate_omega(n, l, seed=123, dtype=torch.float8_e4m3fn)
    torch.cuda.synchronize()
    Om_np = Om.cpu().double().numpy()
    assert np.array_equal(Om_np, torch.from_numpy(Om_np).float().to(torch.float8_e4m3fn).double().numpy())
    Uo, So, Vo = oracle.rsvd(A_exact, l, q=2, Omega=Om_np)
    U, S, V = engine.rsvd(A8, l, q=2, seed=123, a_scale=scale)
    torch.cuda.synchronize()
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    _check(U, S, V, Uo, So, Vo, A_exact, 1e-4, 1e-4)


def test_fp8_decode_all_codes(engine):
    """Every e4m3fn code (NaNs excluded) through the engine's fp8 -> bf16 widening: the rank-1
    matrix a 1^T has the single singular value ||a|| sqrt(n)."""
    torch = _torch()
    codes = torch.arange(256, dtype=torch.uint8)
    vals = codes.view(torch.float8_e4m3fn).float()
    keep = torch.isfinite(vals)
    a = vals[keep]
    m, n = a.numel(), 64
    A8 = a.to(torch.float8_e4m3fn).reshape(m, 1).repeat(1, n).t().contiguous().t().cuda()
    U, S, V = engine.rsvd(A8, 16, q=1, seed=1)
    torch.cuda.synchronize()
    ref = float(torch.linalg.norm(a.double())) * np.sqrt(n)
    assert abs(float(S[0]) - ref) < 1e-5 * ref
    assert float(S[1]) < 1e-4 * ref


@pytest.mark.parametrize("l,rank", [(128, 6), (512, 6), (512, 300), (300, 280)])
def test_wide_rank_deficient_is_orthonormal(engine, l, rank):
    """rank(A) < l: breakdown columns are completed (repair pass), U and V stay orthonormal and A
    is reconstructed exactly, as the reference's Householder Q would.  l = 512 runs the two-level
    LP = 512 factor (wide_qr.hip launch_chol_wide_2level) with breakdowns in its first level
    (rank 6) and only in its second (rank 300)."""
    torch = _torch()
    rng = np.random.default_rng(4)
    m, n = 1200, 800
    # small-integer factors: every entry of A is an integer <= 4 rank in magnitude, exact in bf16
    # (up to 256), so the bf16 matrix the GPU sees has exactly the chosen rank
    A = (rng.integers(-1, 2, (m, rank)) @ rng.integers(-1, 2, (rank, n))).astype(np.float32)
    assert np.abs(A).max() <= 256
    U, S, V = engine.rsvd(_dev_colmajor(A, torch.bfloat16), l, q=1, seed=9)
    torch.cuda.synchronize()
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-3
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-3
    Ab = _dev_colmajor(A, torch.bfloat16).float().cpu().double().numpy()
    assert np.linalg.norm(Ab - (U * S) @ V.T) < 1e-4 * np.linalg.norm(Ab)
    assert np.all(S[rank:] < 1e-4 * S[0])


def test_wide_range_finder_subspace(engine):
    torch = _torch()
    m, n, l = 3000, 1000, 128
    A32 = gapped_matrix(m, n, 300, decay=0.93, seed=21).astype(np.float32)
    Ad = _dev_colmajor(A32, torch.bfloat16)
    A_exact = Ad.float().cpu().double().numpy()
    Om = engine.generate_omega(n, l, seed=8, dtype=torch.bfloat16)
    for q in (0, 1):
        Q = engine.range_finder(Ad, Om, q=q)
        torch.cuda.synchronize()
        Q = Q.cpu().double().numpy()
        Qo = oracle.intermediate_step(A_exact, Om.cpu().double().numpy(), q=q)
        assert np.linalg.norm(Q.T @ Q - np.eye(l)) < 1e-4
        # the leading directions of span(Q) agree with the oracle's span (projectors applied to
        # the top 32 left singular vectors of A); q = 1 also captures them
        Ut = np.linalg.svd(A_exact, full_matrices=False)[0][:, :32]
        assert np.linalg.norm(Q @ (Q.T @ Ut) - Qo @ (Qo.T @ Ut)) < 1e-3
        if q == 1:
            assert np.linalg.norm(Ut - Q @ (Q.T @ Ut)) < 1e-3
