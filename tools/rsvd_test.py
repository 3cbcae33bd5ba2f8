#!/usr/bin/env python3
"""The reference's test harnesses on the MI355X engine.

``--mode rsvd`` mirrors tests/rSVD_test.cpp: every MatrixMarket file in --input is densified
(:54-57), rSVD(A, U, S, V, l = 0 + 16, SVDMethod::Jacobi) runs (:65-72) and the harness prints
dataset, size, execution time and ||A - U S V^T||_F (:77-96), then writes
<name>_{S,U,V}.mtx to --output (:99-115).  ``--mode svd`` mirrors tests/svd_test.cpp
(SVD<ParallelJacobi>, :58-97).  ``--make-inputs DIR`` writes the reference's five inputs
(input/*.mtx: identities of size 100/110/140/160 and the rank-2 matrix of python/matrix_maker.py)
so the harness runs where the reference tree is absent (the GPU box).

    python tools/rsvd_test.py --make-inputs /tmp/in
    python tools/rsvd_test.py --input /tmp/in --output /tmp/out [--l 16] [--mode rsvd|svd]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rsvd_kamaneh_raganato_terrana_amd import SVD, SVDMethod, rSVD  # noqa: E402
from rsvd_kamaneh_raganato_terrana_amd.mtx import read_market, write_market  # noqa: E402


def make_inputs(d: str) -> None:
    """input/sparse_matrix{100,110,140,160}.mtx (identity, one entry per row) and
    input/sparse_matrix.mtx (A[i, j] = 100 i + j + 1, python/matrix_maker.py:15-25)."""
    os.makedirs(d, exist_ok=True)
    for k in (100, 110, 140, 160):
        with open(os.path.join(d, f"sparse_matrix{k}.mtx"), "w") as f:
            f.write("%%MatrixMarket matrix coordinate real general\n")
            f.write(f"{k} {k} {k}\n")
            for i in range(1, k + 1):
                f.write(f"{i} {i} {1.0:.18e}\n")
    size = 100
    with open(os.path.join(d, "sparse_matrix.mtx"), "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{size} {size} {size * size}\n")
        v = 1
        for i in range(size):
            for j in range(size):
                f.write(f"{i + 1} {j + 1} {float(v):.18e}\n")
                v += 1


def run(inp: str, out: str, mode: str, l: int, seed: int) -> list:
    os.makedirs(out, exist_ok=True)
    results = []
    print("test rSVD reduced" if mode == "rsvd" else "test SVD")
    for name in sorted(os.listdir(inp)):
        path = os.path.join(inp, name)
        if not os.path.isfile(path):
            continue
        A = read_market(path)
        t0 = time.perf_counter()
        if mode == "rsvd":
            U, S, V = rSVD(A, l, SVDMethod.Jacobi, seed=seed)
        else:
            s = SVD(A, method=SVDMethod.ParallelJacobi)
            s.compute()
            U, S, V = s.getU(), s.getS(), s.getV()
        dt = time.perf_counter() - t0
        err = float(np.linalg.norm(A - (U * S) @ V.T))
        print(f"\nDataset: {name}\nSize: {A.shape[0]}, {A.shape[1]}\nNumber of Processors: 1\n"
              f"Execution time: {dt} seconds")
        if mode == "rsvd":
            print(f"norm of diff : {err}")
        print("-------------------------\n")
        stem = name.rsplit(".", 1)[0]
        write_market(os.path.join(out, f"{stem}_S.mtx"), S)
        write_market(os.path.join(out, f"{stem}_U.mtx"), U)
        write_market(os.path.join(out, f"{stem}_V.mtx"), V)
        results.append({"name": name, "shape": A.shape, "seconds": dt, "norm_of_diff": err, "S": S})
    return results


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--make-inputs", metavar="DIR")
    ap.add_argument("--input")
    ap.add_argument("--output")
    ap.add_argument("--mode", choices=("rsvd", "svd"), default="rsvd")
    ap.add_argument("--l", type=int, default=16)  # l = k + p = 0 + 16, tests/rSVD_test.cpp:65-67
    ap.add_argument("--seed", type=int, default=0x5EED0001)
    a = ap.parse_args(argv)
    if a.make_inputs:
        make_inputs(a.make_inputs)
    if a.input:
        run(a.input, a.output or os.path.join(os.getcwd(), "rsvd_out"), a.mode, a.l, a.seed)


if __name__ == "__main__":
    main()
