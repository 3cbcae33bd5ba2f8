"""The library's remaining diagnostic environment switches, each pinned against the oracle.

Round 6 retired the settled A/B switches (DESIGN.md §6 lists what is left).
Bit-identity switches back to a replaced kernel are pinned by test_gpu_knob_identity.py; the ones
here select a different (not bit-identical) but supported path, so each runs the same rSVD in a
child process (the switches are read once per process) and must meet the north-star 1e-4 bar
against the fp64 oracle on the same A and Omega:

* RSVD_GRAM_SPLIT=0   every Gram on the fp64 MFMA (no three-piece bf16 split)
* RSVD_SMALL_SVD=jacobi  the block-Jacobi small SVD for fp32 results instead of the eigensolver
* RSVD_DEFER2=0       output panels' CholeskyQR2 with Q and Q_B formed (the pre-round-6 order)
* RSVD_ISQRT=0        the deferred second pass's R2^-1 by the Cholesky factor instead of the G^-1/2 series
* RSVD_ISQRT_CUT=0    the series' cut-off at 0: its predicated Cholesky fallback runs on every second pass
* RSVD_COOP=1         cooperative launches of the persistent kernels (plain is the default since round 6)
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import gapped_matrix, rel_fro, sign_align

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RUN = r"""
import sys, json
sys.path.insert(0, {repo!r})
import numpy as np, torch
import rsvd_kamaneh_raganato_terrana_amd as R
A = np.load({path!r})
eng = R.Engine(0)
Ad = torch.from_numpy(A.astype(np.float32)).cuda().t().contiguous().t().to(torch.bfloat16)
U, S, V = eng.rsvd(Ad, {l}, q=2, seed=31)
torch.cuda.synchronize()
info = eng.info()
Om = eng.generate_omega(A.shape[1], {l}, seed=31, dtype=torch.bfloat16).cpu().double().numpy()
np.savez({out!r}, U=U.cpu().double().numpy(), S=S.cpu().double().numpy(), V=V.cpu().double().numpy(),
         A=Ad.float().cpu().double().numpy(), Om=Om)
print("RESULT " + json.dumps(info))
eng.close()
"""


@pytest.mark.parametrize("env", [{"RSVD_GRAM_SPLIT": "0"}, {"RSVD_SMALL_SVD": "jacobi"}, {"RSVD_DEFER2": "0"},
                                 {"RSVD_ISQRT": "0"}, {"RSVD_ISQRT_CUT": "0"},
                                 {"RSVD_COOP": "1"}, {}])
def test_switch_matches_oracle(env, tmp_path):
    m, n, l = 2048, 1200, 256  # l > 192: the eigensolver's multi-workgroup (persistent) phase runs
    A = gapped_matrix(m, n, 2 * l, decay=0.985, seed=12)
    path, out = str(tmp_path / "A.npy"), str(tmp_path / "out.npz")
    np.save(path, A)
    p = subprocess.run([sys.executable, "-c", _RUN.format(repo=REPO, path=path, out=out, l=l)],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    info = json.loads([x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1][7:])
    if env.get("RSVD_SMALL_SVD") == "jacobi":
        assert info["jacobi_sweeps"] > 0, info  # the block Jacobi ran its sweeps
    else:
        assert info["jacobi_sweeps"] == 0, info  # the eigensolver's check passed
    r = np.load(out)
    Uo, So, Vo = oracle.rsvd(r["A"], l, q=2, Omega=r["Om"])
    k = l // 2
    assert rel_fro(r["S"], So) < 1e-4
    assert rel_fro(sign_align(r["U"][:, :k], Uo[:, :k]), Uo[:, :k]) < 1e-4
    assert rel_fro(sign_align(r["V"][:, :k], Vo[:, :k]), Vo[:, :k]) < 1e-4
    assert np.linalg.norm(r["U"].T @ r["U"] - np.eye(l)) < 1e-3
