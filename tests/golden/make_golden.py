"""Generate the committed golden fixtures under tests/golden/ (run here, where /root/reference is
mounted; the fixtures travel, the reference does not).

* inputs.npz   -- the reference's own committed test inputs as dense float64 matrices:
                  input/sparse_matrix{,100,110,140,160}.mtx (tests/rSVD_test.cpp, svd_test.cpp)
                  and image_compression/data/input/mat/*.mtx.  Data files, read with
                  scipy.io.mmread exactly as python/test_run_rSVD.py:43-44 does.
* lapack.npz   -- the reference's own Python golden outputs on those inputs: its scripts
                  python/test_run_rSVD.py and python/test_run_QR.py are IMPORTED from a scratch
                  working directory (they create ../data/output/... at import, :11) and their
                  process_matrix() (test_run_rSVD.py:41-57: np.linalg.svd; test_run_QR.py:25-40:
                  np.linalg.qr mode="reduced") writes U, diag(S), V^T and Q, R as MatrixMarket files
                  (%.18e, exact for doubles), which are read back here: singular values, the
                  well-determined leading singular vectors, and |diag R|.  Only in this build
                  container (the reference never travels); nothing of its code is kept.
* philox.npz   -- the first Gaussian draws of the Philox4x32-10 + Box-Muller stream the engine
                  and the oracle share (generated here by a pure-Python restatement, independent
                  of both C implementations).

Usage:  python tests/golden/make_golden.py [/root/reference [out_dir]]
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


def reference_outputs(ref, paths):
    """Run the reference's python/test_run_rSVD.py and test_run_QR.py process_matrix() on every
    input (imported, from a scratch cwd) and read back the .mtx files they write."""
    import importlib.util
    import tempfile

    scratch = tempfile.mkdtemp(prefix="rsvd_golden_")
    work = os.path.join(scratch, "work")
    os.makedirs(work)
    cwd = os.getcwd()
    os.chdir(work)
    try:
        mods = {}
        for name in ("test_run_rSVD", "test_run_QR"):
            spec = importlib.util.spec_from_file_location(f"reference_{name}", os.path.join(ref, "python", f"{name}.py"))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)  # its import side effect: os.makedirs("../data/output/...")
            mods[name] = mod
        out = {}
        for key, path in paths.items():
            mods["test_run_rSVD"].process_matrix(path)
            mods["test_run_QR"].process_matrix(path)
            sv = os.path.join(scratch, "data", "output", "SVD", "py")
            qr = os.path.join(scratch, "data", "output", "QR", "py")
            rd = lambda d, f: np.asarray(mmread(os.path.join(d, f)).toarray(), dtype=np.float64)  # noqa: E731
            out[key] = (rd(sv, f"{key}_U.mtx"), np.diag(rd(sv, f"{key}_S.mtx")).copy(), rd(sv, f"{key}_V.mtx"),
                        rd(qr, f"{key}_Q.mtx"), rd(qr, f"{key}_R.mtx"))
        return out
    finally:
        os.chdir(cwd)
        import shutil

        shutil.rmtree(scratch, ignore_errors=True)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out_dir = sys.argv[2] if len(sys.argv) > 2 else HERE
    files, paths = {}, {}
    for sub in ("input", os.path.join("image_compression", "data", "input", "mat")):
        d = os.path.join(ref, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith(".mtx"):
                key = os.path.splitext(f)[0]
                files[key] = np.asarray(mmread(os.path.join(d, f)).toarray(), dtype=np.float64)
                paths[key] = os.path.join(d, f)
    np.savez_compressed(os.path.join(out_dir, "inputs.npz"), **files)

    refout = reference_outputs(ref, paths)
    gold = {}
    for key, A in files.items():
        U, S, VT, Q, R = refout[key]
        gold[f"{key}__S"] = S
        # leading vectors where the spectrum has a gap (sign-free comparison in the tests)
        k = int(np.sum(S > S[0] * 1e-8)) if S[0] > 0 else 0
        k = min(k, 4) if k < len(S) else 0
        gap_ok = k > 0 and all(S[i] - S[i + 1] > 1e-6 * S[0] for i in range(k))
        if gap_ok:
            gold[f"{key}__U"] = U[:, :k]
            gold[f"{key}__V"] = VT[:k, :].T
        gold[f"{key}__absdiagR"] = np.abs(np.diag(R))
    np.savez_compressed(os.path.join(out_dir, "lapack.npz"), **gold)

    ph = {f"seed{s}": philox_gaussian_py(s, 64) for s in (0, 1, 0x5EED0001)}
    np.savez_compressed(os.path.join(out_dir, "philox.npz"), **ph)
    print("wrote", sorted(files), "->", out_dir)


if __name__ == "__main__":
    main()
