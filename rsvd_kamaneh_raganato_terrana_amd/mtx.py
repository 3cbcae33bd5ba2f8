"""MatrixMarket I/O of the reference's harnesses.

The reference reads its inputs with ``Eigen::loadMarket`` into a sparse matrix and densifies them
(tests/rSVD_test.cpp:54-57, tests/svd_test.cpp:50-52), and writes ``<name>_{U,S,V}.mtx`` with
``Eigen::saveMarket`` (tests/rSVD_test.cpp:108-115).  Format handled here:

* read: ``%%MatrixMarket matrix coordinate real|integer|pattern general|symmetric`` (1-based
  ``i j v`` triplets, duplicates summed as a sparse->dense conversion does) and
  ``%%MatrixMarket matrix array real general`` (column-major values);
* write: ``%%MatrixMarket matrix coordinate real general``, a ``rows cols nnz`` line and every
  entry of the dense matrix as a 1-based ``i j v`` triplet in column-major order, 17 significant
  digits (round-trips fp64 exactly); a vector is written as an n x 1 matrix.

Host-side numpy only: this is file plumbing, not part of the GPU path.
"""
from __future__ import annotations

import numpy as np


def read_market(path: str) -> np.ndarray:
    """Dense float64 (Fortran-order) matrix from a MatrixMarket file."""
    with open(path) as f:
        header = f.readline().strip().lower().split()
        if len(header) < 4 or header[0] != "%%matrixmarket" or header[1] != "matrix":
            raise ValueError(f"{path}: not a MatrixMarket matrix file")
        fmt, field = header[2], header[3]
        sym = header[4] if len(header) > 4 else "general"
        if field == "complex":
            raise ValueError(f"{path}: complex matrices are not supported")
        line = f.readline()
        while line.startswith("%") or not line.strip():
            line = f.readline()
        dims = [int(x) for x in line.split()]
        body = f.read().split()
    m, n = dims[0], dims[1]
    A = np.zeros((m, n), order="F")
    if fmt == "array":
        vals = np.array(body, dtype=np.float64)
        if sym == "general":
            A[:, :] = vals[: m * n].reshape((m, n), order="F")
        else:  # symmetric array: lower triangle by columns
            k = 0
            for j in range(n):
                for i in range(j, m):
                    A[i, j] = A[j, i] = vals[k]
                    k += 1
        return A
    nnz = dims[2]
    per = 2 if field == "pattern" else 3
    t = np.array(body[: nnz * per], dtype=np.float64).reshape(nnz, per)
    ii = t[:, 0].astype(np.int64) - 1
    jj = t[:, 1].astype(np.int64) - 1
    vv = np.ones(nnz) if field == "pattern" else t[:, 2]
    np.add.at(A, (ii, jj), vv)
    if sym in ("symmetric", "skew-symmetric"):
        off = ii != jj
        np.add.at(A, (jj[off], ii[off]), vv[off] if sym == "symmetric" else -vv[off])
    return A


def write_market(path: str, X) -> None:
    """Every entry of the dense matrix (or vector, as n x 1) as a coordinate MatrixMarket file."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X.reshape(-1, 1)
    m, n = X.shape
    jj, ii = np.meshgrid(np.arange(n), np.arange(m), indexing="ij")  # column-major order
    vals = X.T.reshape(-1)
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{m} {n} {m * n}\n")
        rows = np.column_stack([ii.reshape(-1) + 1, jj.reshape(-1) + 1])
        for (i, j), v in zip(rows, vals):
            f.write(f"{i} {j} {v:.17g}\n")
