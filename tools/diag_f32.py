"""Diagnostic: f32 device path orthogonality over l / rank (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import rsvd_kamaneh_raganato_terrana_amd as R
from conftest import gapped_matrix
eng = R.Engine(0)
def dev(A, dt=torch.float32):
    return torch.from_numpy(np.asarray(A, dtype=np.float64)).to(dt).cuda().t().contiguous().t()
def orth(X):
    return np.linalg.norm(X.T @ X - np.eye(X.shape[1]))
rng = np.random.default_rng(11)
B = rng.standard_normal((512, 6))
Adup = np.asfortranarray(np.repeat(B, 40, axis=1)[:, :200])
for name, A in [("gapped", gapped_matrix(512, 200, 96, seed=1)), ("dup", Adup)]:
    for dt in (torch.float32, torch.float64):
        for l in (8, 16, 24, 32, 48, 64):
            At = dev(A, dt)
            Om = torch.randn(200, l, dtype=dt, device="cuda")
            for q in (0, 2):
                Q = eng.range_finder(At, Om, q=q).cpu().double().numpy()
                U, S, V = eng.rsvd(At, l, q=q, seed=3)
                torch.cuda.synchronize()
                U, S, V = U.cpu().double().numpy(), S.cpu().double().numpy(), V.cpu().double().numpy()
                inf = eng.info()
                print(f"{name:6s} {str(dt)[6:]:8s} l={l:2d} q={q} Q {orth(Q):.1e}  U {orth(U):.1e} V {orth(V):.1e} "
                      f"rec {np.linalg.norm(A - (U*S)@V.T)/np.linalg.norm(A):.1e} fb={inf['cholqr_fallbacks']} sw={inf['jacobi_sweeps']}", flush=True)
