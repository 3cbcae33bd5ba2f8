"""Size-independent properties of the C4 rSVD at its full size (65536^2 bf16, l = 256, q = 2):
orthonormality of U and V, and the Ritz residual A V - U S = (I - Q Q^T) A V chunk-wise in fp32."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    import bench
    import rsvd_kamaneh_raganato_terrana_amd as R

    m = n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    l = 256
    A, _ = bench.make_A(torch, m, n, 0, "bf16")
    eng = R.Engine(0)
    t0 = time.perf_counter()
    U, S, V = eng.rsvd(A, l, q=2, seed=0x5EED0002)
    torch.cuda.synchronize()
    print(f"rsvd {m}x{n}: {(time.perf_counter() - t0) * 1e3:.1f} ms (first call)", flush=True)
    Ud, Vd, Sd = U.double(), V.double(), S.double()
    I = torch.eye(l, dtype=torch.float64, device=U.device)
    ou = float(torch.linalg.norm(Ud.t() @ Ud - I))
    ov = float(torch.linalg.norm(Vd.t() @ Vd - I))
    # residual A V - U S, 4096 rows at a time (A exactly as stored: bf16 -> fp32)
    Vf = V.float()
    res2 = torch.zeros(l, dtype=torch.float64, device=U.device)
    for r0 in range(0, m, 4096):
        blk = A[r0:r0 + 4096].float() @ Vf - U[r0:r0 + 4096].float() * S.float()
        res2 += (blk.double() ** 2).sum(0)
    res = res2.sqrt()
    print(f"|U^T U - I|_F = {ou:.3e}  |V^T V - I|_F = {ov:.3e}", flush=True)
    print(f"S[0] = {float(Sd[0]):.6e}  S[127] = {float(Sd[127]):.6e}  S[255] = {float(Sd[255]):.6e}", flush=True)
    print(f"|A V - U S|_F / |S|_F = {float(res.norm() / Sd.norm()):.3e}", flush=True)
    rel = res / Sd
    print(f"max_i<=64 |A v_i - s_i u_i| / s_i = {float(rel[:64].max()):.3e}; i<=128: {float(rel[:128].max()):.3e}; "
          f"all: {float(rel.max()):.3e}; max residual {float(res.max()):.3e}", flush=True)
    sig = Sd >= 10 * Sd[-1]
    print(f"{int(sig.sum())} triplets with s_i >= 10 s_l: max |A v_i - s_i u_i| / s_i = {float(rel[sig].max()):.3e}",
          flush=True)


if __name__ == "__main__":
    main()
