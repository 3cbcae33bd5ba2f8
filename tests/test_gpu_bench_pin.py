"""The benchmarked workload itself against the oracle.

bench.py times C4 on bench.make_A (128 directions at 0.9^t plus 1e-3 Gaussian noise, bf16).  Here the
same generator builds a 16384 x 16384 A -- a quarter of C4's side, the largest the fp64 CPU oracle
finishes in well under a minute on the box's host cores -- and the engine's rSVD (l = 256, q = 2,
the bench's seed, hence the same bf16 Omega) is compared with the oracle's
(/root/reference/src/rSVD.cpp:72-133 restated in oracle/rsvd_oracle.c) on the bf16-rounded A:
* S: relative Frobenius <= 1e-4 (north_star);
* U, V: sign-aligned relative Frobenius <= 1e-4 over the triplets with s_i >= 10 s_l (the
  noise-cluster triplets below that are not determined by the data to 1e-4 and are not compared).
"""
import os
import sys

import numpy as np
import pytest

import oracle
from conftest import rel_fro, sign_align

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_bench_workload_matches_oracle(engine):
    import torch

    sys.path.insert(0, REPO)
    import bench

    m = n = 16384
    l, q, seed = 256, 2, 0x5EED0002
    A, scale = bench.make_A(torch, m, n, 0, "bf16")
    assert scale == 1.0
    U, S, V = engine.rsvd(A, l, q=q, seed=seed)
    Om = engine.generate_omega(n, l, seed=seed, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    U, S, V = (x.cpu().double().numpy() for x in (U, S, V))
    A_exact = np.asfortranarray(A.float().cpu().double().numpy())
    Om_np = Om.cpu().double().numpy()
    del A
    torch.cuda.empty_cache()
    oracle.set_threads(min(16, os.cpu_count() or 1))
    Uo, So, Vo = oracle.rsvd(A_exact, l, q=q, Omega=Om_np)
    assert rel_fro(S, So) < 1e-4, rel_fro(S, So)
    k = int(np.sum(So >= 10 * So[-1]))
    assert k >= 32, k
    eu = rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k])
    ev = rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k])
    assert eu < 1e-4 and ev < 1e-4, (k, eu, ev)
    assert np.linalg.norm(U.T @ U - np.eye(l)) < 1e-4
    assert np.linalg.norm(V.T @ V - np.eye(l)) < 1e-4
