"""CPU: pin the oracle (oracle/, test infrastructure) to the reference's own inputs and golden recipe.

The reference C++ cannot be built here (Eigen is absent), so the oracle is pinned by
* the reference's committed inputs (tests/golden/inputs.npz <- input/*.mtx,
  image_compression/data/input/mat/*.mtx) and the LAPACK goldens its Python scripts produce
  (tests/golden/lapack.npz <- python/test_run_rSVD.py:47, python/test_run_QR.py:31);
* known answers of those inputs (I_n: S == 1 and ||A - U S V^T||_F = sqrt(n - l);
  input/sparse_matrix.mtx has rank 2);
* a pure-Python restatement of the shared Philox Omega stream (tests/golden/philox.npz).
Tolerances are written per assertion (fp64 throughout).
"""
import os
import tempfile

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, gapped_matrix, rel_fro, sign_align

INPUTS = np.load(os.path.join(GOLDEN, "inputs.npz"))
LAPACK = np.load(os.path.join(GOLDEN, "lapack.npz"))
PHILOX = np.load(os.path.join(GOLDEN, "philox.npz"))
NAMES = [k for k in INPUTS.files if k != "sparse_matrix copy"]
DIAG_NAMES = [k for k in NAMES if k.startswith(("sparse_diagonal", "block_diagonal"))]


def _write_mtx(path, A):
    """MatrixMarket coordinate writer (python/matrix_maker.py layout)."""
    r, c = np.nonzero(A)
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{A.shape[0]} {A.shape[1]} {len(r)}\n")
        for i, j in zip(r, c):
            f.write(f"{i + 1} {j + 1} {A[i, j]:.18e}\n")


def test_philox_stream_matches_python_restatement():
    for key in PHILOX.files:
        seed = int(key[4:])
        got = oracle.philox_gaussian(seed, 64)
        assert np.max(np.abs(got - PHILOX[key])) < 1e-14
    om = oracle.generate_omega(8, 8, 1)  # element (i, j) = stream element i + n j
    assert np.max(np.abs(om.ravel(order="F") - PHILOX["seed1"])) < 1e-14


def test_read_matrix_market_roundtrip():
    A = INPUTS["sparse_matrix"]
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "a.mtx")
        _write_mtx(p, A)
        B = oracle.read_matrix_market(p)
    assert np.array_equal(A, B)


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("parallel", [False, True])
def test_jacobi_svd_matches_lapack_golden(name, parallel):
    """SVD<Jacobi> / SVD<ParallelJacobi>::compute (tests/svd_test.cpp) on the committed inputs."""
    A = INPUTS[name]
    U, S, V, sweeps = oracle.jacobi_svd(A, parallel=parallel)
    Sg = LAPACK[f"{name}__S"]
    # SVD<Jacobi> iterates to 2 eps (include/SVD_class.hpp:127); SVD<ParallelJacobi> stops at the
    # absolute 1e-12 'precision' / 'considerAsZero' (:253-254), so its residual is coarser.
    tol = 1e-8 if parallel else 1e-12
    assert np.max(np.abs(S - Sg)) < tol * Sg[0]
    assert np.all(np.diff(S) <= 0)
    assert np.linalg.norm(A - (U * S) @ V.T) < tol * max(1.0, np.linalg.norm(A))
    if f"{name}__U" in LAPACK.files:
        k = LAPACK[f"{name}__U"].shape[1]
        assert rel_fro(sign_align(U[:, :k], LAPACK[f"{name}__U"]), LAPACK[f"{name}__U"]) < 1e-2 * tol ** 0.5
        assert rel_fro(sign_align(V[:, :k], LAPACK[f"{name}__V"]), LAPACK[f"{name}__V"]) < 1e-2 * tol ** 0.5


@pytest.mark.parametrize("name", ["sparse_matrix", "sparse_diagonal_matrix", "sparse_diagonal_matrix_random3"])
def test_householder_and_givens_qr(name):
    """QRTest.cpp: Q R == A, Q^T Q == I, R upper triangular; |diag R| == LAPACK's."""
    A = INPUTS[name]
    n = A.shape[1]
    Q, R = oracle.givens_qr_reduced(A)
    assert np.linalg.norm(Q @ R - A) < 1e-12 * np.linalg.norm(A)
    assert np.linalg.norm(Q.T @ Q - np.eye(n)) < 1e-12
    assert np.allclose(np.tril(R, -1), 0.0)
    dR = np.abs(np.diag(R))
    Rh, tau, W = oracle.householder_qr(A)
    Qh = oracle.thin_q(A)
    assert np.linalg.norm(Qh @ Rh - A) < 1e-12 * np.linalg.norm(A)
    g = LAPACK[f"{name}__absdiagR"]
    well = g > 1e-8 * g[0]  # the rank-deficient tail of sparse_matrix is rounding noise
    assert np.max(np.abs(dR - g)[well]) < 1e-10 * g[0]
    assert np.max(np.abs(np.abs(np.diag(Rh)) - g)[well]) < 1e-10 * g[0]


@pytest.mark.parametrize("name,l", [("sparse_matrix100", 16), ("sparse_matrix110", 16), ("sparse_matrix140", 10),
                                    ("sparse_matrix160", 16), ("sparse_diagonal_matrix_ones", 16)])
def test_rsvd_identity_known_answer(name, l):
    """tests/rSVD_test.cpp (k = 0, p = 16): I_n -> S == 1, ||A - U S V^T||_F = sqrt(n - l)."""
    A = INPUTS[name]
    n = A.shape[0]
    U, S, V = oracle.rsvd(A, l, q=2, seed=0x5EED0001)
    assert np.max(np.abs(S - 1.0)) < 1e-12
    assert abs(np.linalg.norm(A - (U * S) @ V.T) - np.sqrt(n - l)) < 1e-10


@pytest.mark.parametrize("l", [4, 16])
def test_rsvd_rank2_known_answer(l):
    """input/sparse_matrix.mtx (python/matrix_maker.py, A_ij = 100 i + j + 1) has rank 2: rSVD is exact."""
    A = INPUTS["sparse_matrix"]
    U, S, V = oracle.rsvd(A, l, q=2, seed=7)
    Sg = LAPACK["sparse_matrix__S"]
    assert abs(S[0] - Sg[0]) < 1e-12 * Sg[0] and abs(S[1] - Sg[1]) < 1e-10 * Sg[0]
    assert np.max(np.abs(S[2:])) < 1e-9 * Sg[0]
    assert np.linalg.norm(A - (U * S) @ V.T) < 1e-10 * np.linalg.norm(A)
    k = 2
    assert rel_fro(sign_align(U[:, :k], LAPACK["sparse_matrix__U"][:, :k]), LAPACK["sparse_matrix__U"][:, :k]) < 1e-9
    assert rel_fro(sign_align(V[:, :k], LAPACK["sparse_matrix__V"][:, :k]), LAPACK["sparse_matrix__V"][:, :k]) < 1e-9


@pytest.mark.parametrize("name", DIAG_NAMES[:4])
def test_rsvd_diagonal_inputs_bounded_by_truth(name):
    """rSVD singular values never exceed the true ones and the leading ones converge (q = 2)."""
    A = INPUTS[name]
    Sg = LAPACK[f"{name}__S"]
    U, S, V = oracle.rsvd(A, 16, q=2, seed=3)
    assert np.all(S <= Sg[:16] * (1 + 1e-12) + 1e-14)
    assert np.linalg.norm(U.T @ U - np.eye(16)) < 1e-12
    assert np.linalg.norm(V.T @ V - np.eye(16)) < 1e-12


def test_rsvd_converges_to_lapack_on_gapped_spectrum():
    A = gapped_matrix(300, 200, 20, decay=0.5, noise=0.0, seed=4)
    Ug, Sg, VgT = np.linalg.svd(A, full_matrices=False)
    U, S, V = oracle.rsvd(A, 24, q=2, seed=5)
    assert np.max(np.abs(S[:20] - Sg[:20])) < 1e-12
    assert rel_fro(sign_align(U[:, :10], Ug[:, :10]), Ug[:, :10]) < 1e-10
    assert rel_fro(sign_align(V[:, :10], VgT[:10].T), VgT[:10].T) < 1e-10


def test_intermediate_step_is_orthonormal_range_basis():
    A = gapped_matrix(200, 150, 30, seed=6)
    Om = oracle.generate_omega(150, 12, 9)
    for q in (0, 1, 2):
        Q = oracle.intermediate_step(A, Om, q=q)
        assert np.linalg.norm(Q.T @ Q - np.eye(12)) < 1e-13
        # q = 0: span(Q) == span(A Omega)
        if q == 0:
            Y = A @ Om
            assert np.linalg.norm(Y - Q @ (Q.T @ Y)) < 1e-12 * np.linalg.norm(Y)


def test_power_method_svd_matches_lapack():
    """SVD<Power> (src/PM.cpp, tests/PMTest.cpp) on a matrix with a clear spectral gap."""
    A = gapped_matrix(60, 40, 8, decay=0.5, noise=0.0, seed=8)
    U, S, V = oracle.power_svd(A, r=5, seed=1)
    Sg = np.linalg.svd(A, compute_uv=False)
    assert np.max(np.abs(S[:5] - Sg[:5])) < 1e-6


def test_image_compression_power_svd_known_answers():
    """image_compression's SVD (image_compression/src/SVD.cpp:30-55) on its own test inputs
    (image_compression/data/input/mat/*.mtx, tests/golden/inputs.npz).  The diagonal matrices have
    sigma = 100, 99, 98, ...: ratios of 0.99 that the fixed s(n) power iterations
    (PowerMethod.cpp:24-27) resolve only to ~1e-3 -- the reference's own accuracy on them; the
    dim triplets are all returned (no early stop) with unit singular vectors."""
    for name in ("sparse_diagonal_matrix", "block_diagonal_matrix"):
        A = INPUTS[name].astype(np.float64)
        U, S, V = oracle.ic_power_svd(A, 10, seed=5)
        Sg = np.linalg.svd(A, compute_uv=False)
        assert S.shape == (10,) and U.shape == (100, 10) and V.shape == (100, 10)
        assert np.max(np.abs(S - Sg[:10])) < 1e-3 * Sg[0]
        assert np.allclose(np.linalg.norm(U, axis=0), 1.0) and np.allclose(np.linalg.norm(V, axis=0), 1.0)
    # image_compression/tests/SVD_test2.cpp:30-34 style 4 x 4 known matrix against LAPACK
    A = np.asfortranarray(np.array([[4.0, 0, 0, 0], [0, 3, 0, 0], [0, 0, 2, 0], [0, 0, 0, 1]]) +
                          0.1 * np.arange(16).reshape(4, 4))
    U, S, V = oracle.ic_power_svd(A, 4, seed=2)
    Sg = np.linalg.svd(A, compute_uv=False)
    assert np.max(np.abs(S - Sg)) < 1e-9 * Sg[0]


def test_image_compression_svd_recomputes_b():
    """The two power-method SVDs differ only in how B follows the deflation: SVD<Power> updates
    B -= (sigma u v^T)^T (sigma u v^T) (SVD_class.hpp:212), image_compression recomputes A^T A
    (SVD.cpp:48) -- the same matrix when v is an exact eigenvector.  Rank 3: SVD<Power> stops at
    sigma < 1e-12 after three triplets, image_compression's SVD keeps going."""
    rng = np.random.default_rng(3)
    A = np.asfortranarray((rng.standard_normal((40, 3)) * [3.0, 2.0, 1.0]) @ rng.standard_normal((3, 30)))
    U, S, V = oracle.ic_power_svd(A, 6, seed=4)
    Up, Sp, Vp = oracle.power_svd(A, r=6, seed=4)
    assert Sp.shape == (3,) and S.shape == (6,)
    assert np.max(np.abs(S[:3] - Sp)) < 1e-10 * S[0]
    assert np.all(S[3:] < 1e-10 * S[0])
    Om = oracle.generate_omega(30, 8, 9)
    Ui, Si, Vi = oracle.ic_rsvd(A, 8, Om, pm_seed=1)
    assert Si.shape == (8,) and Ui.shape == (40, 8) and Vi.shape == (30, 8)
    assert np.max(np.abs(Si[:3] - np.linalg.svd(A, compute_uv=False)[:3])) < 1e-9 * Si[0]


def test_unsupported_method_raises():
    with pytest.raises(ValueError):
        oracle.rsvd(np.eye(8), 4, method=7)


@pytest.mark.skipif(not os.path.isdir("/root/reference/python"), reason="the reference is mounted only in the build container")
def test_golden_fixtures_regenerate_byte_identical(tmp_path):
    """tests/golden/lapack.npz is the reference's own output: make_golden.py imports
    python/test_run_rSVD.py and python/test_run_QR.py and reads back what their process_matrix()
    writes.  Regenerating all three fixtures must reproduce the committed bytes."""
    import subprocess
    import sys

    subprocess.run([sys.executable, os.path.join(GOLDEN, "make_golden.py"), "/root/reference", str(tmp_path)],
                   check=True, capture_output=True, cwd=str(tmp_path), timeout=600)
    for f in ("inputs.npz", "lapack.npz", "philox.npz"):
        assert (tmp_path / f).read_bytes() == open(os.path.join(GOLDEN, f), "rb").read(), f
