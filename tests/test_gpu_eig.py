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


@pytest.mark.parametrize("l", [193, 196])
def test_eig_small_svd_phase_boundary(engine, l):
    """l just past the one-workgroup tridiagonalisation (n <= 192): phase 1 runs
    n - 193 steps (none at l = 193, three at 196) on four workgroups before the single-workgroup
    phase 2 takes the trailing 192 rows -- the hand-off at its boundary."""
    A32 = gapped_matrix(2600, 1800, 2 * l, decay=0.97, seed=l).astype(np.float32) * 10
    res, ref, A, info = _run_bf16(engine, A32, l, 1, seed=l + 1)
    _check(res, ref, A)
    assert info["jacobi_sweeps"] == 0, info


def test_eig_small_svd_f32_A(engine):
    """fp32 A (the narrow projection kernels per 64-column group) into the same eigensolver small SVD:
    its fp32 results take the eigensolver path too (wide.cpp, sizeof(T) == 4, 128 <= LP <= 512)."""
    torch = _torch()
    m, n, l = 2048, 1536, 256
    A = gapped_matrix(m, n, 2 * l, decay=0.97, seed=9)
    A32 = A.astype(np.float32)
    Ad = _dev_colmajor(A32, torch.float32)
    Om = oracle.generate_omega(n, l, 23)
    Uo, So, Vo = oracle.rsvd(A32.astype(np.float64), l, q=2, Omega=Om)
    U, S, V = engine.rsvd(Ad, l, q=2, omega=torch.from_numpy(Om))
    torch.cuda.synchronize()
    info = engine.info()
    _check([x.cpu().double().numpy() for x in (U, S, V)], (Uo, So, Vo), A32.astype(np.float64))
    assert info["jacobi_sweeps"] == 0, info


_POLISH = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "tests"))
import torch, oracle
import rsvd_kamaneh_raganato_terrana_amd as R
from conftest import gapped_matrix, rel_fro, sign_align
eng = R.Engine(0)
m, n, l = 2048, 1500, 256
A32 = gapped_matrix(m, n, 2 * l, decay=0.97, seed=31).astype(np.float32) * 10
Ad = torch.from_numpy(np.ascontiguousarray(A32.T)).cuda().to(torch.bfloat16).t()
Ax = Ad.float().cpu().double().numpy()
Om = eng.generate_omega(n, l, seed=17, dtype=torch.bfloat16).cpu().double().numpy()
Uo, So, Vo = oracle.rsvd(Ax, l, q=1, Omega=Om)
U, S, V = (x.cpu().double().numpy() for x in eng.rsvd(Ad, l, q=1, seed=17))
k = l // 2
out = dict(sweeps=eng.info()["jacobi_sweeps"], s=rel_fro(S, So),
           u=rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]), v=rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]),
           uo=float(np.linalg.norm(U.T @ U - np.eye(l))), vo=float(np.linalg.norm(V.T @ V - np.eye(l))))
eng.close()
print("RESULT " + json.dumps(out))
"""


def test_eig_small_svd_forced_polish():
    """the block-Jacobi polish of the eigensolver's X -- what runs when the orthogonality
    check fails (near-clusters the cluster tolerance does not catch).  RSVD_EIG_FORCE_POLISH=1 skips
    the check (read once per process, so in a child process): the sweeps run on X = W V_w as given,
    jacobi_sweeps > 0, and the results still match the oracle at 1e-4."""
    import json
    import subprocess

    env = dict(os.environ, RSVD_EIG_FORCE_POLISH="1")
    p = subprocess.run([sys.executable, "-c", _POLISH.format(repo=REPO)], env=env, capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
    r = json.loads(line[7:])
    assert r["sweeps"] > 0, r
    assert r["s"] < 1e-4 and r["u"] < 1e-4 and r["v"] < 1e-4, r
    assert r["uo"] < 1e-4 and r["vo"] < 1e-4, r


def test_eig_small_svd_small_sigma(engine):
    """the eigensolver squares the condition number (G = W^T W), so a small
    sigma_i carries an extra absolute error ~ eps_64 |W|^2 / sigma_i from G.  fp32 A with a graded
    spectrum 0.93^i (sigma_255 / sigma_0 ~ 1e-8): every S_i below 1e-4 sigma_1 is checked against the
    oracle with the absolute bound  |S_i - So_i| <= 1e-6 sigma_1 + 1e-13 sigma_1^2 / So_i  (the fp32
    pipeline's noise on R, ~1e-7 sigma_1, plus 1e3 x the eigensolver's eps_64 sigma_1^2 / sigma_i).
    On this spectrum the eigenvectors of the smallest sigma lose orthogonality past the check's 1e-6
    (measured: 4 polish sweeps), so the check hands X to the block-Jacobi polish -- the designed
    route; the bound holds for the result either way."""
    torch = _torch()
    m, n, l = 3000, 2000, 256
    rng = np.random.default_rng(77)
    X = np.linalg.qr(rng.standard_normal((m, 400)))[0]
    Y = np.linalg.qr(rng.standard_normal((n, 400)))[0]
    A32 = ((X * 0.93 ** np.arange(400)) @ Y.T).astype(np.float32)
    Ax = A32.astype(np.float64)
    Om = oracle.generate_omega(n, l, 5)
    Uo, So, Vo = oracle.rsvd(Ax, l, q=2, Omega=Om)
    U, S, V = engine.rsvd(_dev_colmajor(A32, torch.float32), l, q=2, omega=torch.from_numpy(Om))
    torch.cuda.synchronize()
    sweeps = engine.info()["jacobi_sweeps"]
    S = S.cpu().double().numpy()
    s1 = So[0]
    small = So < 1e-4 * s1
    assert small.sum() > 100, small.sum()
    bound = 1e-6 * s1 + 1e-13 * s1 * s1 / np.maximum(So, 1e-300)
    err = np.abs(S - So)
    assert np.all(err[small] <= bound[small]), (err[small].max(), np.argmax(err[small] / bound[small]), sweeps)
    assert rel_fro(S, So) < 1e-4


_ABORT = r"""
import json, sys
sys.path.insert(0, {repo!r})
import numpy as np, torch
import rsvd_kamaneh_raganato_terrana_amd as R
from rsvd_kamaneh_raganato_terrana_amd._capi import RSVDError
rng = np.random.default_rng(3)
m, n, l = 1200, 900, 256
A = np.linalg.qr(rng.standard_normal((m, 400)))[0] * 0.97 ** np.arange(400) @ np.linalg.qr(rng.standard_normal((n, 400)))[0].T
eng = R.Engine(0)
msgs = []
for rep in range(2):
    try:
        eng.rsvd(torch.from_numpy(A.astype(np.float32)).cuda().t().contiguous().t(), l, q=1, seed=9)
        msgs.append(None)
    except RSVDError as e:
        msgs.append((e.status, str(e)))
# the handle and the device are healthy afterwards: an fp64 run (block-Jacobi small SVD) is exact
U, S, V = eng.rsvd(torch.from_numpy(A).cuda().t().contiguous().t(), 64, q=1, seed=9)
torch.cuda.synchronize()
Ud = U.cpu().numpy()
print("RESULT " + json.dumps({{"msgs": msgs, "orth": float(np.linalg.norm(Ud.T @ Ud - np.eye(64))),
                              "s0": float(S[0])}}))
eng.close()
"""


def test_tridiag_abort_path_is_reported():
    """the tridiagonalisation's multi-workgroup hand-off has a bounded spin and
    an abort word that had never executed.  RSVD_TRI_FORCE_ABORT=3 (read once per process, so in a
    child) makes member 0 take the timeout branch at step 3 of phase 1 (l = 256 > 192: four
    workgroups).  The other members must leave at their next spin check (no hang: the child finishes
    inside the timeout), the run must fail with a named status (RSVD_ERR_HIP, "timed out") through
    rsvd_sync -- twice in a row, since the sticky word is cleared when reported -- and the same
    handle must then run an fp64 rSVD (block-Jacobi small SVD, no tridiagonalisation) correctly."""
    import json
    import subprocess

    env = dict(os.environ, RSVD_TRI_FORCE_ABORT="3")
    p = subprocess.run([sys.executable, "-c", _ABORT.format(repo=REPO)], env=env, capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
    r = json.loads(line[7:])
    for msg in r["msgs"]:
        assert msg is not None, r
        status, text = msg
        assert status == 3 and "timed out" in text, r  # RSVD_ERR_HIP
    assert r["orth"] < 1e-10 and abs(r["s0"] - 1.0) < 1e-3, r
