"""Generate the committed golden fixtures under tests/golden/ (run here, where /root/reference is
mounted; the fixtures travel, the reference does not).

* inputs.npz   -- the reference's own committed test inputs as dense float64 matrices:
                  input/sparse_matrix{,100,110,140,160}.mtx (tests/rSVD_test.cpp, svd_test.cpp)
                  and image_compression/data/input/mat/*.mtx.  Data files, read with
                  scipy.io.mmread exactly as python/test_run_rSVD.py:43-44 does.
* lapack.npz   -- the reference's Python golden recipe (python/test_run_rSVD.py:47 np.linalg.svd,
                  python/test_run_QR.py:31 np.linalg.qr mode="reduced") on those inputs:
                  singular values, the well-determined leading singular vectors, and |diag R|.
* philox.npz   -- the first Gaussian draws of the Philox4x32-10 + Box-Muller stream the engine
                  and the oracle share (generated here by a pure-Python restatement, independent
                  of both C implementations).

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
import math
import os
import sys

import numpy as np
from scipy.io import mmread

HERE = os.path.dirname(os.path.abspath(__file__))


def philox4x32_10(ctr, seed):
    M = 0xFFFFFFFF
    c = [ctr & M, (ctr >> 32) & M, 0x52535644, 0]
    k = [seed & M, (seed >> 32) & M]
    for _ in range(10):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k[0]) & M, p1 & M, ((p0 >> 32) ^ c[3] ^ k[1]) & M, p0 & M]
        k = [(k[0] + 0x9E3779B9) & M, (k[1] + 0xBB67AE85) & M]
    return c


def philox_gaussian_py(seed, count):
    out = []
    for e in range(count):
        x = philox4x32_10(e >> 1, seed)
        u1 = (float(((x[0] >> 5) << 26) | (x[1] >> 6)) + 0.5) * 2.0 ** -53
        u2 = (float(((x[2] >> 5) << 26) | (x[3] >> 6)) + 0.5) * 2.0 ** -53
        r = math.sqrt(-2.0 * math.log(u1))
        th = 2.0 * math.pi * u2
        out.append(r * math.sin(th) if e & 1 else r * math.cos(th))
    return np.array(out)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    files = {}
    for sub in ("input", os.path.join("image_compression", "data", "input", "mat")):
        d = os.path.join(ref, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith(".mtx"):
                key = os.path.splitext(f)[0]
                files[key] = np.asarray(mmread(os.path.join(d, f)).toarray(), dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "inputs.npz"), **files)

    gold = {}
    for key, A in files.items():
        U, S, VT = np.linalg.svd(A)
        gold[f"{key}__S"] = S
        # leading vectors where the spectrum has a gap (sign-free comparison in the tests)
        k = int(np.sum(S > S[0] * 1e-8)) if S[0] > 0 else 0
        k = min(k, 4) if k < len(S) else 0
        gap_ok = k > 0 and all(S[i] - S[i + 1] > 1e-6 * S[0] for i in range(k))
        if gap_ok:
            gold[f"{key}__U"] = U[:, :k]
            gold[f"{key}__V"] = VT[:k, :].T
        Q, R = np.linalg.qr(A, mode="reduced")
        gold[f"{key}__absdiagR"] = np.abs(np.diag(R))
    np.savez_compressed(os.path.join(HERE, "lapack.npz"), **gold)

    ph = {f"seed{s}": philox_gaussian_py(s, 64) for s in (0, 1, 0x5EED0001)}
    np.savez_compressed(os.path.join(HERE, "philox.npz"), **ph)
    print("wrote", sorted(files), "->", HERE)


if __name__ == "__main__":
    main()
