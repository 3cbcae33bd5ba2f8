"""C2 (4096^2 fp32, l=64, q=2): eager rSVD launches vs one captured HIP graph replayed (torch.cuda.CUDAGraph
over the engine's stream).  Timing probe for the launch-gap share of the latency chain."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import rsvd_kamaneh_raganato_terrana_amd as R

m = n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
l = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dt = {"f32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3] if len(sys.argv) > 3 else "f32"]
A = torch.randn(n, m, device="cuda").t().contiguous().t().to(dt)
A = A.t().contiguous().t() if not A.t().is_contiguous() else A
eng = R.Engine(0)
U, S, V = eng.rsvd(A, l, q=2, seed=1)
torch.cuda.synchronize()
def timeit(fn, k=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3
te = timeit(lambda: eng.rsvd(A, l, q=2, seed=1, check_errors=False))
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        eng.rsvd(A, l, q=2, seed=1, check_errors=False)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    Ug, Sg, Vg = eng.rsvd(A, l, q=2, seed=1, check_errors=False)
g.replay()
torch.cuda.synchronize()
print("graph S matches eager:", torch.allclose(Sg, S, rtol=1e-6, atol=0), float((Sg - S).abs().max()))
tg = timeit(lambda: g.replay())
print(f"m=n={m} l={l} {dt}: eager {te:.3f} ms/rSVD, graph replay {tg:.3f} ms/rSVD")
