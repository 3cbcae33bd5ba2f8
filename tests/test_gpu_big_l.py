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


def _known_svd_device(m, n, sig, seed):
    """A = X diag(sig) Y^T with orthonormal X (m x k), Y (n x k) drawn on the GPU (torch QR, fp64):
    the exact SVD is known by construction, so sizes the CPU oracle cannot finish (its Householder QR
    and two-sided Jacobi on a 4096-wide B take hours) still get a known answer."""
    torch = _torch()
    g = torch.Generator(device="cuda").manual_seed(seed)
    k = sig.shape[0]
    X = torch.linalg.qr(torch.randn(m, k, generator=g, device="cuda", dtype=torch.float64))[0]
    Y = torch.linalg.qr(torch.randn(n, k, generator=g, device="cuda", dtype=torch.float64))[0]
    A = (X * torch.from_numpy(sig).cuda()) @ Y.t()
    return A, X, Y


def _head_spectrum(n, head=64):
    """64 leading singular values 10 % apart (their vectors are determined far below the fp32 bar),
    then a smooth 0.997^i tail down to ~1e-6 of sigma_1 at i ~ 4300."""
    h = 0.9 ** np.arange(head)
    t = h[-1] * 0.997 ** np.arange(1, n - head + 1)
    return np.concatenate([h, t])


@pytest.mark.parametrize("m,n,l", [(2560, 2304, 2048), (4608, 4352, 4096)])
def test_big_l_2048_4096_known_answer(engine, m, n, l):
    """rSVD() at l = 2048 and l = 4096, the top of the advertised range (VERDICT r04 item 1;
    src/rSVD.cpp:72 has no cap): f32 A with a known SVD (_known_svd_device), q = 1.  The sketch
    captures all but a ~1e-6 tail, so S matches the known sigma to 1e-4 (relative Frobenius), the 64
    well-separated leading singular vectors match X / Y to 1e-4, U and V are orthonormal, and
    |A - U S V^T|_F / |A|_F is at the fp32 floor.  Exercises the l = 4096 block Jacobi small SVD on its
    occupancy-capped cooperative grid (launch_coresident)."""
    torch = _torch()
    sig = _head_spectrum(n)
    A64, X, Y = _known_svd_device(m, n, sig, seed=l)
    A = A64.float().t().contiguous().t()
    U, S, V = engine.rsvd(A, l, q=1, seed=l + 1)
    torch.cuda.synchronize()
    assert U.shape == (m, l) and S.shape == (l,) and V.shape == (n, l)
    S64 = S.double().cpu().numpy()
    assert np.all(np.diff(S64) <= 1e-6 * S64[0])
    assert rel_fro(S64, sig[:l]) < 1e-4, rel_fro(S64, sig[:l])
    Ud, Vd = U.double(), V.double()
    h = 64
    Xh, Yh = X[:, :h].cpu().numpy(), Y[:, :h].cpu().numpy()
    eu = rel_fro(sign_align(Ud[:, :h].cpu().numpy(), Xh), Xh)
    ev = rel_fro(sign_align(Vd[:, :h].cpu().numpy(), Yh), Yh)
    assert eu < 1e-4 and ev < 1e-4, (eu, ev)
    eye = torch.eye(l, dtype=torch.float64, device="cuda")
    # fp32 factors: ~1e-7 per entry over l^2 entries
    assert torch.linalg.norm(Ud.t() @ Ud - eye).item() < 1e-3 * l / 512
    assert torch.linalg.norm(Vd.t() @ Vd - eye).item() < 1e-3 * l / 512
    # the rank-l truncation itself leaves the tail past l (2.0e-5 at l = 2048, ~0 at 4096)
    trunc = np.linalg.norm(sig[l:]) / np.linalg.norm(sig)
    res = torch.linalg.norm(A.double() - (Ud * S.double()) @ Vd.t()) / torch.linalg.norm(A.double())
    assert res.item() < trunc * 1.01 + 1e-5, (res.item(), trunc)


def test_svd_jacobi_4096_columns_known_answer(engine):
    """SVD<Jacobi> at min(m, n) = 4096 (SVD_class.hpp:100-180; INTEGRATION.md's advertised limit): the
    block Jacobi on 128 column blocks, its persistent grid capped by the device's co-resident capacity.
    fp64 A with a known SVD (0.999^i, relative gaps 1e-3): S to 1e-12, the leading 2048 vectors to 1e-8,
    U S V^T = A to 4e-12 (fp64 sums over 4096 terms; 1.9e-12 measured)."""
    torch = _torch()
    m, n = 4200, 4096
    sig = 0.999 ** np.arange(n)
    A, X, Y = _known_svd_device(m, n, sig, seed=4096)
    U, S, V = engine.svd(A.t().contiguous().t(), 0)
    torch.cuda.synchronize()
    assert U.shape == (m, n) and S.shape == (n,) and V.shape == (n, n)
    S64 = S.cpu().numpy()
    assert rel_fro(S64, sig) < 1e-12, rel_fro(S64, sig)
    h = 2048
    Xh, Yh = X[:, :h].cpu().numpy(), Y[:, :h].cpu().numpy()
    assert rel_fro(sign_align(U[:, :h].cpu().numpy(), Xh), Xh) < 1e-8
    assert rel_fro(sign_align(V[:, :h].cpu().numpy(), Yh), Yh) < 1e-8
    res = torch.linalg.norm(A - (U * S) @ V.t()) / torch.linalg.norm(A)
    assert res.item() < 4e-12, res.item()


def test_big_l_range_finder_and_limits(engine):
    """intermediate_step at l = 520 spans the oracle's Q; RSVD_SVD_POWER_IC, l > 4096 and the forced
    n-side shard past 512 are refused."""
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

    with pytest.raises(RSVDError, match="POWER_IC"):  # image_compression's power method: l <= 512
        engine.rsvd_host(A, l, q=1, omega=Om, method=3)
    with pytest.raises(RSVDError):
        engine.rsvd_host(gapped_matrix(5000, 4200, 300, decay=0.9, seed=1), 4100, q=0)
    # the n-side sharded path is built for l <= 512; asking for it past 512 is refused,
    # not silently ignored
    torch = _torch()
    with pytest.raises(RSVDError, match="FORCE_NSHARD"):
        engine.rsvd(_dev_colmajor(A.astype(np.float32), torch.float32), l, q=1, force_nshard=True)
    # l > m on a one-rank handle (m < l is only a valid row shard)
    with pytest.raises(RSVDError, match="min"):
        engine.rsvd(_dev_colmajor(A[:500].astype(np.float32), torch.float32), l, q=1)


PM_KEY = 0x504F574552  # dense.hip power_seed: the power method's start streams are Philox(seed ^ PM_KEY + i)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", [("f64", 560, 0.97, 1e-3), ("f32", 560, 0.97, 1e-3), ("f64", 20, 0.6, 0.0)])
def test_big_l_power_matches_oracle(engine, case):
    """SVDMethod::Power past 512 sketch columns (VERDICT r04 missing 4: src/rSVD.cpp:106-113 has no cap
    on l): dense_big.cpp runs the power method in the coordinates of Q_B on the grid
    (dense.hip launch_power_grid_rsvd) against the oracle's power method on B = Q^T A in the n
    coordinates, the same start vectors (Philox(seed ^ PM_KEY + i)).  Third case: A of exact rank 20
    (singular values 0.6^i -- separated enough for the reference's iteration count to converge --
    then zeros): both stop at sigma_20 < 1e-12 (SVD_class.hpp:198-208), the engine's later triplets
    are zero and info()["power_kept"] is 20.  (A graded or clustered spectrum has no reproducible
    stop: unconverged or sub-sqrt(eps) triplets deflate inexactly, and where an implementation first
    reads sigma < 1e-12 then differs by a few triplets, or never comes.)"""
    torch = _torch()
    import rsvd_kamaneh_raganato_terrana_amd as R

    dt, rank, decay, noise = case
    m, n, l, seed = 800, 600, 520, 2468
    A = gapped_matrix(m, n, rank, decay=decay, noise=noise, seed=21)
    tdt = torch.float64 if dt == "f64" else torch.float32
    At = _dev_colmajor(A, tdt)
    U, S, V = engine.rsvd(At, l, q=1, method=R.SVDMethod.Power, seed=seed)
    kept = engine.info()["power_kept"]
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    Om = engine.generate_omega(n, l, seed=seed, dtype=tdt).cpu().double().numpy()
    Aused = At.cpu().double().numpy()
    oracle.set_threads(16)
    Uo, So, Vf = oracle.rsvd_power(Aused, l, q=1, Omega=Om, pm_seed=seed ^ PM_KEY)
    ko = So.shape[0]
    k = 16
    ts, tv = (1e-10, 1e-8) if dt == "f64" else (1e-4, 1e-4)
    assert rel_fro(S[:k], So[:k]) < ts, rel_fro(S[:k], So[:k])
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < tv
    if noise == 0.0:
        # (on an early stop the reference cuts its n x n V_ -- v_i in rows -- to n x k columns,
        # conservativeResize: the oracle returns that, so V is checked through A v_i = sigma_i u_i)
        assert kept == ko == 20, (kept, ko)
        assert rel_fro(S[:ko], So) < 1e-10
        assert np.all(S[ko:] == 0.0) and np.all(U[:, ko:] == 0.0) and np.all(V[:, ko:] == 0.0)
        r = np.linalg.norm(Aused @ V[:, :k] - U[:, :k] * S[:k]) / np.linalg.norm(S[:k])
        assert r < 1e-8, r
    else:
        assert kept == l and ko == l, (kept, ko)
        Vo = Vf[:l, :].T  # the reference's V_ holds v_i in rows
        assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < tv


@pytest.mark.timeout(600)
def test_big_l_power_2048_known_answer(engine):
    """SVDMethod::Power at l = 2048 (rsvd_c.h advertises Power up to l = 4096 through the
    grid power method, whose u = A v was one serial l-long dot per row): fp64 A with a known SVD,
    48 leading singular values 0.8^i (each power iteration converges: (0.8^2)^s(n) with the reference's
    s(2304) = 149, src/PM.cpp:25-28) over a 0.997^i tail.  The 2048 deflation steps (~3e5 grid
    barriers) must finish in bounded time; S and the 16 leading U / V columns match the known SVD."""
    import time

    torch = _torch()
    import rsvd_kamaneh_raganato_terrana_amd as R

    m, n, l = 2560, 2304, 2048
    h = 0.8 ** np.arange(48)
    sig = np.concatenate([h, h[-1] * 0.997 ** np.arange(1, n - 48 + 1)])
    A, X, Y = _known_svd_device(m, n, sig, seed=77)
    A = A.t().contiguous().t()
    t0 = time.perf_counter()
    U, S, V = engine.rsvd(A, l, q=1, method=R.SVDMethod.Power, seed=5)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"Power rSVD at l = {l}: {dt:.2f} s")
    assert dt < 60.0, dt
    # (the reference's stop at sigma < 1e-12, SVD_class.hpp:198-208, may end the deflation inside the
    # tail, whose later triplets no fixed iteration count resolves; the separated head is always kept)
    assert engine.info()["power_kept"] >= 64
    k = 16
    S64 = S.cpu().numpy()
    assert rel_fro(S64[:k], sig[:k]) < 1e-10, rel_fro(S64[:k], sig[:k])
    Xk, Yk = X[:, :k].cpu().numpy(), Y[:, :k].cpu().numpy()
    assert rel_fro(sign_align(U[:, :k].cpu().numpy(), Xk), Xk) < 1e-8
    assert rel_fro(sign_align(V[:, :k].cpu().numpy(), Yk), Yk) < 1e-8
