"""Round-5 kernels are drop-in replacements, bit for bit, for the kernels they replaced.

Each optimisation of round 5 kept the summation order of the kernel it replaced, and each left an
environment switch back to the previous kernel (read once per process, so each setting runs in a
child process).  The same rSVDs -- bf16 A at l = 512 / 256 / 128 (LP 512 / 256 / 128) and e4m3 A at
l = 512 -- run once with the defaults and once with every switch at its previous kernel, and the
U, S, V bytes must be identical:

* RSVD_NN8=0       the e4m3 NN halves on wproj2_kernel instead of wproj3nn8_kernel (wide_proj.hip)
* RSVD_NN3_128=0   the LP = 128 hi/lo NN on wproj2_kernel instead of wproj3_kernel
* RSVD_TN128=0     the LP = 128 TN on the v2 double-step kernel instead of wproj3tn128_kernel
* RSVD_PANEL_PD=2  the split panel products with In one step ahead (the default is 4 at LP = 512)
* RSVD_TRI_NOSKIP=1  the tridiagonalisation updating the dead row slots too (wide_eig.hip)
* RSVD_TRI_SPLIT2=0  its one-workgroup phase in one launch (no hand-over to the two-slot shape)
* RSVD_CHOL_RINV_FUSED=0  the leaves' R^-1 on a separate rinv_wide launch (wide_qr.hip)

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
for (m, n, l, dt) in [(4096, 2048, 512, torch.bfloat16), (4096, 3000, 256, torch.bfloat16),
                      (8192, 1024, 128, torch.bfloat16), (4096, 2048, 512, torch.float8_e4m3fn)]:
    g = torch.Generator().manual_seed(l + 1)
    U0 = torch.linalg.qr(torch.randn(m, 2 * l, generator=g, dtype=torch.float64))[0]
    V0 = torch.linalg.qr(torch.randn(n, 2 * l, generator=g, dtype=torch.float64))[0]
    s = 0.97 ** torch.arange(2 * l, dtype=torch.float64)
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
                    "RSVD_TRI_NOSKIP": "1", "RSVD_TRI_SPLIT2": "0",
                    "RSVD_CHOL_RINV_FUSED": "0"})
    assert new == old, (new, old)
    assert len(set(new)) == 4  # four different problems, four different digests
