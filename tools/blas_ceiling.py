"""Library-GEMM ceiling for the C4 projection shapes (hipBLASLt via torch.mm), for comparison
with wproj2_kernel: NN Y = A [hi lo] and TN Z = A^T [hi lo] as one N = 512 bf16 GEMM, and the
single-operand sketch (N = 256).  Timing only; not part of the product."""
import torch, time, json

def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(reps):
        ev[0].record(); fn(); ev[1].record(); torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2] * 1e3

m = n = 65536
A = torch.randn(n, m, device="cuda", dtype=torch.bfloat16).t()  # column-major m x n
out = {}
for N in (256, 512):
    B = torch.randn(n, N, device="cuda", dtype=torch.bfloat16)
    us = t(lambda: torch.mm(A, B))
    out[f"NN N={N}"] = (us, 2.0 * m * n * N / us / 1e6)
    Bt = torch.randn(m, N, device="cuda", dtype=torch.bfloat16)
    us = t(lambda: torch.mm(A.t(), Bt))
    out[f"TN N={N}"] = (us, 2.0 * m * n * N / us / 1e6)
for k, (us, tf) in out.items():
    print(f"{k}: {us:.1f} us  {tf:.0f} TF/s")
