"""CPU parity oracle for the randomized-SVD hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import this package; the product path (``rsvd_kamaneh_raganato_terrana_amd``) never does.

Thin numpy/ctypes front end over ``liboracle.so`` (``rsvd_oracle.c``), a plain-C fp64
restatement of the reference:

* ``generate_omega``     -- src/rSVD.cpp:12-55 (Philox-seeded instead of std::random_device)
* ``intermediate_step``  -- src/rSVD.cpp:57-70
* ``rsvd``               -- src/rSVD.cpp:72-133
* ``thin_q``             -- Eigen::HouseholderQR + householderQ()*Identity, src/rSVD.cpp:60-61
* ``jacobi_svd``         -- include/SVD_class.hpp:100-180 (and ParallelJacobi :223-333)
* ``power_svd``          -- include/SVD_class.hpp:183-219 + src/PM.cpp:4-81
* ``givens_qr_reduced/full`` -- src/QR.cpp:12-80

Pinning: tests/test_oracle.py checks it against the known answers of the reference's committed
inputs and the LAPACK golden vectors in tests/golden/ (see tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SVD_JACOBI, SVD_POWER, SVD_PARALLEL_JACOBI = 0, 1, 2


def build(opt: str = "O3") -> str:
    """Compile the oracle with its Makefile; returns the .so path."""
    target = "liboracle.so" if opt == "O3" else "liboracle_O0.so"
    path = os.path.join(_HERE, target)
    subprocess.run(["make", "-s", "-C", _HERE, path], check=True)
    return path


def lib(opt: str = "O3"):
    global _LIB
    if _LIB is not None and opt == "O3":
        return _LIB
    path = os.path.join(_HERE, "liboracle.so" if opt == "O3" else "liboracle_O0.so")
    src = os.path.join(_HERE, "rsvd_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        build(opt)
    L = ctypes.CDLL(path)
    i64, u64, dp, i32 = ctypes.c_int64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double), ctypes.c_int
    L.orc_set_threads.argtypes = [i32]
    L.orc_set_threads.restype = i32
    L.orc_philox_gaussian.argtypes = [u64, i64, i64, dp]
    L.orc_gemm.argtypes = [ctypes.c_char, ctypes.c_char, i64, i64, i64, dp, i64, dp, i64, ctypes.c_double, dp, i64]
    L.orc_thin_q.argtypes = [i64, i64, dp, i64, dp, i64]
    L.orc_householder_qr.argtypes = [i64, i64, dp, i64, dp]
    L.orc_givens_qr_reduced.argtypes = [i64, i64, dp, i64, dp, dp]
    L.orc_givens_qr_reduced.restype = i32
    L.orc_givens_qr_full.argtypes = [i64, i64, dp, i64, dp, dp]
    L.orc_givens_qr_full.restype = i32
    L.orc_jacobi_svd.argtypes = [i64, i64, dp, i64, i32, dp, dp, dp]
    L.orc_jacobi_svd.restype = i32
    L.orc_power_svd.argtypes = [i64, i64, dp, i64, i64, u64, dp, dp, dp]
    L.orc_power_svd.restype = i64
    L.orc_intermediate_step.argtypes = [i64, i64, dp, i64, dp, i64, i64, i64, dp, i64]
    L.orc_rsvd.argtypes = [i64, i64, dp, i64, i64, i64, dp, i64, i32, dp, dp, dp]
    L.orc_rsvd.restype = i32
    L.orc_rsvd_power.argtypes = [i64, i64, dp, i64, i64, i64, dp, i64, u64, dp, dp, dp]
    L.orc_rsvd_power.restype = i64
    L.orc_ic_power_svd.argtypes = [i64, i64, dp, i64, i64, u64, dp, dp, dp]
    L.orc_ic_power_svd.restype = i64
    L.orc_ic_rsvd.argtypes = [i64, i64, dp, i64, i64, dp, i64, u64, dp, dp, dp]
    L.orc_ic_rsvd.restype = i64
    if opt == "O3":
        _LIB = L
    return L


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _f(a) -> np.ndarray:
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def set_threads(n: int) -> int:
    return lib().orc_set_threads(int(n))


def philox_gaussian(seed: int, count: int, first: int = 0) -> np.ndarray:
    out = np.empty(count, dtype=np.float64)
    lib().orc_philox_gaussian(seed, first, count, _p(out))
    return out


def generate_omega(n: int, l: int, seed: int) -> np.ndarray:
    """n x l i.i.d. N(0,1), element (i, j) = stream element i + n*j (column-major)."""
    return philox_gaussian(seed, n * l).reshape((n, l), order="F")


def gemm(A, B, ta="N", tb="N") -> np.ndarray:
    A, B = _f(A), _f(B)
    m = A.shape[1] if ta == "T" else A.shape[0]
    k = A.shape[0] if ta == "T" else A.shape[1]
    n = B.shape[0] if tb == "T" else B.shape[1]
    C = np.zeros((m, n), order="F")
    lib().orc_gemm(ta.encode(), tb.encode(), m, n, k, _p(A), A.shape[0], _p(B), B.shape[0], 0.0, _p(C), m)
    return C


def thin_q(Y) -> np.ndarray:
    Y = _f(Y)
    m, l = Y.shape
    Q = np.zeros((m, l), order="F")
    lib().orc_thin_q(m, l, _p(Y), m, _p(Q), m)
    return Q


def householder_qr(A):
    """Returns (R, tau, packed) in Eigen's HouseholderQR convention."""
    W = _f(A).copy(order="F")
    m, n = W.shape
    tau = np.zeros(min(m, n))
    lib().orc_householder_qr(m, n, _p(W), m, _p(tau))
    return np.triu(W)[: min(m, n), :], tau, W


def givens_qr_reduced(A):
    A = _f(A)
    m, n = A.shape
    Q = np.zeros((m, n), order="F")
    R = np.zeros((n, n), order="F")
    if lib().orc_givens_qr_reduced(m, n, _p(A), m, _p(Q), _p(R)) != 0:
        raise ValueError("qr_decomposition_reduced requires rows >= cols")
    return Q, R


def givens_qr_full(A):
    A = _f(A)
    m, n = A.shape
    Q = np.zeros((m, m), order="F")
    R = np.zeros((m, n), order="F")
    lib().orc_givens_qr_full(m, n, _p(A), m, _p(Q), _p(R))
    return Q, R


def jacobi_svd(data, parallel: bool = False):
    """SVD<Jacobi>/SVD<ParallelJacobi>::compute(): U (m x d), S (d), V (n x d), d = min(m, n)."""
    D = _f(data)
    m, n = D.shape
    d = min(m, n)
    U = np.zeros((m, d), order="F")
    S = np.zeros(d)
    V = np.zeros((n, d), order="F")
    sweeps = lib().orc_jacobi_svd(m, n, _p(D), m, int(parallel), _p(U), _p(S), _p(V))
    return U, S, V, sweeps


def power_svd(data, r: int = 0, seed: int = 0):
    """SVD<Power>::compute() with the reference's output layouts, trimmed as
    conservativeResize would (include/SVD_class.hpp:198-208)."""
    D = _f(data)
    m, n = D.shape
    U = np.zeros((m, m), order="F")
    S = np.zeros(min(m, n))
    V = np.zeros((n, n), order="F")
    k = lib().orc_power_svd(m, n, _p(D), m, r, seed, _p(U), _p(S), _p(V))
    dim = r if r else min(m, n)
    if k == dim:
        return U, S, V
    if k == 0:
        return np.zeros((m, 1)), np.zeros(1), np.zeros((n, 1))
    return U[:, :k].copy(order="F"), S[:k].copy(), V[:, :k].copy(order="F")


def intermediate_step(A, Omega, q: int = 2) -> np.ndarray:
    A, Om = _f(A), _f(Omega)
    m, n = A.shape
    l = Om.shape[1]
    Q = np.zeros((m, l), order="F")
    lib().orc_intermediate_step(m, n, _p(A), m, _p(Om), n, l, q, _p(Q), m)
    return Q


def rsvd(A, l: int, q: int = 2, Omega=None, seed: int = 0, method: int = SVD_JACOBI):
    """rSVD(A, U, S, V, l, method) with an injected Omega (or Philox stream `seed`)."""
    A = _f(A)
    m, n = A.shape
    Om = _f(Omega) if Omega is not None else generate_omega(n, l, seed)
    d = min(l, n)
    U = np.zeros((m, d), order="F")
    S = np.zeros(d)
    V = np.zeros((n, d), order="F")
    rc = lib().orc_rsvd(m, n, _p(A), m, l, q, _p(Om), n, method, _p(U), _p(S), _p(V))
    if rc != 0:
        raise ValueError("Unsupported SVD method")
    return U, S, V


def rsvd_power(A, l: int, q: int = 2, Omega=None, seed: int = 0, pm_seed: int = 0):
    """rSVD(A, U, S, V, l, SVDMethod::Power) (src/rSVD.cpp:106-113): U (m x l), S (l), V (n x n,
    v_i^T in rows i < l, identity rows beyond -- SVD_class.hpp:82-83, 213-214), cut to the
    triplets kept on an early stop as conservativeResize does (:198-208).  Start vectors of the
    power method: Philox(pm_seed + i)."""
    A = _f(A)
    m, n = A.shape
    Om = _f(Omega) if Omega is not None else generate_omega(n, l, seed)
    U = np.zeros((m, l), order="F")
    S = np.zeros(l)
    V = np.zeros((n, n), order="F")
    k = lib().orc_rsvd_power(m, n, _p(A), m, l, q, _p(Om), n, pm_seed, _p(U), _p(S), _p(V))
    if k == l:
        return U, S, V
    if k == 0:
        return np.zeros((m, 1)), np.zeros(1), np.zeros((n, 1))
    return U[:, :k].copy(order="F"), S[:k].copy(), V[:, :k].copy(order="F")


def ic_power_svd(data, dim: int = 0, seed: int = 0):
    """image_compression's singularValueDecomposition (image_compression/src/SVD.cpp:30-55): U (m x
    dim), S (dim), V (n x dim, v_i in columns); B = A^T A recomputed after every deflation, no early
    stop.  Start vectors Philox(seed + i) (the reference draws std::random_device)."""
    D = _f(data)
    m, n = D.shape
    dim = dim or min(m, n)
    U = np.zeros((m, dim), order="F")
    S = np.zeros(dim)
    V = np.zeros((n, dim), order="F")
    k = lib().orc_ic_power_svd(m, n, _p(D), m, dim, seed, _p(U), _p(S), _p(V))
    return U[:, :k].copy(order="F"), S[:k].copy(), V[:, :k].copy(order="F")


def ic_rsvd(A, l: int, Omega, pm_seed: int = 0):
    """image_compression's 5-argument rSVD(A, U, S, V, l) (image_compression/src/rSVD.cpp:77-118):
    q = 1, the power-method SVD above on B = Q^T A.  U (m x d), S (d), V (n x d), d = min(l, n)."""
    A = _f(A)
    m, n = A.shape
    Om = _f(Omega)
    d = min(l, n)
    U = np.zeros((m, d), order="F")
    S = np.zeros(d)
    V = np.zeros((n, d), order="F")
    k = lib().orc_ic_rsvd(m, n, _p(A), m, l, _p(Om), n, pm_seed, _p(U), _p(S), _p(V))
    return U[:, :k].copy(order="F"), S[:k].copy(), V[:, :k].copy(order="F")


def read_matrix_market(path: str) -> np.ndarray:
    """Dense matrix from a MatrixMarket 'coordinate real general' or 'array' file (what
    Eigen::loadMarket + MatrixXd(sparse) produce in tests/rSVD_test.cpp:54-57)."""
    with open(path) as f:
        header = f.readline()
        line = f.readline()
        while line.startswith("%"):
            line = f.readline()
        dims = [int(x) for x in line.split()]
        body = np.loadtxt(f, ndmin=2)
    if "array" in header:
        return body.reshape(-1)[: dims[0] * dims[1]].reshape((dims[0], dims[1]), order="F")
    A = np.zeros((dims[0], dims[1]))
    for i, j, v in body:
        A[int(i) - 1, int(j) - 1] += v
    return A
