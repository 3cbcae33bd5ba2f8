"""Probe: the l > 512 path's U error against the oracle, by world / row split / dtype (lab only)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import test_gpu_distributed as T
import oracle
from conftest import rel_fro, sign_align


def err(case, world):
    m, n, l, qq, dt = case
    if world == 1:
        import torch
        import rsvd_kamaneh_raganato_terrana_amd as R
        A = T._matrix(case)
        tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
        Ag = torch.from_numpy(np.ascontiguousarray(A.T)).cuda().to(tdt).t()
        eng = R.Engine(0)
        U, S, V = eng.rsvd(Ag, l, q=qq, seed=4242)
        Om = eng.generate_omega(n, l, seed=4242, dtype=tdt).cpu().double().numpy()
        U, S = U.cpu().double().numpy(), S.cpu().double().numpy()
        A = Ag.float().cpu().double().numpy()
        eng.close()
    else:
        res = T._run_world2(case, False, False, world)
        U = np.vstack([r[2] for r in res]); S = res[0][3]
        A = np.vstack([r[5] for r in res])
        import torch
        import rsvd_kamaneh_raganato_terrana_amd as R
        eng = R.Engine(0)
        tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
        Om = eng.generate_omega(n, l, seed=4242, dtype=tdt).cpu().double().numpy()
        eng.close()
    Uo, So, Vo = oracle.rsvd(A, l, q=qq, Omega=Om)
    out = []
    for k in (16, 64, l // 4, l // 2):
        out.append(rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]))
    print(case, "world", world, "S", rel_fro(S, So), "U err at k=16,64,l/4,l/2:", ["%.2e" % e for e in out], flush=True)


if __name__ == "__main__":
    err((2001, 1200, 640, 1, "bf16"), 1)
    err((2000, 1200, 640, 1, "bf16"), 2)
    err((2001, 1200, 640, 1, "f32"), 2)
    err((2001, 1200, 640, 1, "bf16"), 2)
    err((1600, 1000, 768, 1, "f32"), 2)
