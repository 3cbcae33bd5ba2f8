"""Round-5 kernels are drop-in replacements, bit for bit, for the kernels they replaced.

(Round 6 retired RSVD_CHOL_RINV_FUSED, pinned here in round 5: the leaves' fused R^-1 is the only
path at LP = 64 / 128 now; rinv_wide_kernel stays for the LP = 256 / 512 leaves.)

Each optimisation of round 5 kept the summation order of the kernel it replaced, and each left an
environment switch back to the previous kernel (read once per process, so each setting runs in a
child process).  The same rSVDs -- bf16 A at l = 512 / 256 / 128 (LP 512 / 256 / 128), e4m3 A at
l = 512, l < LP at l = 200 / 100 (padding pivots and zero-padded pieces) and a rank-100 A
at l = 128 (breakdown pivots, the repair pass) -- run once with the defaults and once with every switch
at its previous kernel, and the U, S, V bytes must be identical:

* RSVD_NN8=0       the e4m3 NN halves on wproj2_kernel instead of wproj3nn8_kernel (wide_proj.hip)
* RSVD_NN3_128=0   the LP = 128 hi/lo NN on wproj2_kernel instead of wproj3_kernel
* RSVD_TN128=0     the LP = 128 TN on the v2 double-step kernel instead of wproj3tn128_kernel
* RSVD_PANEL_PD=2  the split panel products with In one step ahead (the default is 4 at LP = 512)
* RSVD_TRI_NOSKIP=1  the tridiagonalisation updating the dead row slots too (wide_eig.hip)
* RSVD_TRI_SPLIT2=0  its one-workgroup phase in one launch (no hand-over to the two-slot shape)

The oracle parity of the default path is what test_gpu_wide / test_gpu_eig / test_gpu_bench_pin
check; this test pins that none of these kernels changed a single output bit.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RUN = r"""
import sys, json, hashlib
sys.path.insert(0, {repo!r})
import torch
import rsvd_kamaneh_raganato_terrana_amd as R
out = []
eng = R.Engine(0)
# (the last three: l < LP -- the factors' padding pivots and the zero-padded pieces -- and a rank-100
# A at l = 128, whose breakdown pivots take chol_diag16_v2's careful second pass and the repair)
for (m, n, l, dt, rk) in [(4096, 2048, 512, torch.bfloat16, 0), (4096, 3000, 256, torch.bfloat16, 0),
                          (8192, 1024, 128, torch.bfloat16, 0), (4096, 2048, 512, torch.float8_e4m3fn, 0),
                          (4096, 2048, 200, torch.bfloat16, 0), (8192, 1024, 100, torch.bfloat16, 0),
                          (4096, 2000, 128, torch.bfloat16, 100)]:
    g = torch.Generator().manual_seed(l + 1)
    k = rk if rk else 2 * l
    U0 = torch.linalg.qr(torch.randn(m, k, generator=g, dtype=torch.float64))[0]
    V0 = torch.linalg.qr(torch.randn(n, k, generator=g, dtype=torch.float64))[0]
    s = 0.97 ** torch.arange(k, dtype=torch.float64)
    A = ((U0 * s) @ V0.T).float()
    if dt == torch.float8_e4m3fn:
        A = A * 64.0
    Ad = A.t().contiguous().t().cuda().to(dt)
    U, S, V = eng.rsvd(Ad, l, q=2, seed=5)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for x in (U, S, V):
        h.update(x.cpu().numpy().tobytes())
    out.append(h.hexdigest())
eng.close()
print("RESULT " + json.dumps(out))
"""


def _digests(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-c", _RUN.format(repo=REPO)], env=env, capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
    return json.loads(line[7:])


def test_round5_kernels_bit_identical_to_previous():
    new = _digests({})
    old = _digests({"RSVD_NN8": "0", "RSVD_NN3_128": "0", "RSVD_TN128": "0", "RSVD_PANEL_PD": "2",
                    "RSVD_TRI_NOSKIP": "1", "RSVD_TRI_SPLIT2": "0"})
    assert new == old, (new, old)
    assert len(set(new)) == 7  # seven different problems, seven different digests
