"""Digest of one wide-engine rSVD's outputs (U, S, V bytes), for bit-identity A/B runs across env
knobs: RSVD_BJ_INNER=0 python tools/digest_run.py; python tools/digest_run.py -- same digest expected."""
import hashlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import rsvd_kamaneh_raganato_terrana_amd as R  # noqa: E402

cases = [(4096, 2048, 512, torch.bfloat16), (4096, 3000, 256, torch.bfloat16), (8192, 1024, 128, torch.bfloat16),
         (4096, 2048, 512, torch.float8_e4m3fn)]  # (the e4m3 case: C5's LP = 512 half kernels)
for (m, n, l, dt) in cases:
    g = torch.Generator().manual_seed(l)
    U0 = torch.linalg.qr(torch.randn(m, 2 * l, generator=g, dtype=torch.float64))[0]
    V0 = torch.linalg.qr(torch.randn(n, 2 * l, generator=g, dtype=torch.float64))[0]
    s = 0.97 ** torch.arange(2 * l, dtype=torch.float64)
    A = ((U0 * s) @ V0.T).float()
    if dt == torch.float8_e4m3fn:
        A = A * 64.0  # into e4m3's normal range
    Ad = A.t().contiguous().t().cuda().to(dt)
    eng = R.Engine()
    U, S, V = eng.rsvd(Ad, l, q=2, seed=11)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for x in (U, S, V):
        h.update(x.cpu().numpy().tobytes())
    print(m, n, l, h.hexdigest()[:16], float(S[0]), float(S[-1]))
