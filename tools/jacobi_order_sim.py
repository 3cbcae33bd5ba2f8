"""numpy model of the block one-sided Jacobi (16-column blocks, one cyclic inner sweep per pair, as
wide_svd.hip): outer rounds to convergence under the round-robin (cyclic) order vs a dynamic order
(greedy max-weight matching on the block off-diagonal norms).  usage: python tools/jacobi_order_sim.py [l]"""
import numpy as np, sys
rng = np.random.default_rng(0)
l = int(sys.argv[1]) if len(sys.argv) > 1 else 256
b = 16; NB = l // b
def make_W(kind):
    U = np.linalg.qr(rng.standard_normal((l, l)))[0]; V = np.linalg.qr(rng.standard_normal((l, l)))[0]
    t = np.arange(l)
    if kind == "c4": s = np.maximum(255 * 0.9 ** t, 0.0) + 0.44 + 0.02 * rng.standard_normal(l) * 0.01
    elif kind == "flat": s = 0.999 ** t
    else: s = 0.97 ** t
    A = U @ np.diag(s) @ V.T
    R = np.linalg.qr(A)[1]
    return R.T
def inner_sweep(G):
    n = G.shape[0]; J = np.eye(n); G = G.copy(); N = n
    for r in range(N - 1):
        for k in range(N // 2):
            if k == 0: p, q = r, N - 1
            else: p, q = (r + k) % (N - 1), (r - k + N - 1) % (N - 1)
            a, bb, g = G[p, p], G[q, q], G[p, q]
            if g == 0: continue
            d = bb - a
            t = np.sign(d * g) * abs(2 * g) / (abs(d) + np.hypot(d, 2 * g)) if d != 0 else np.sign(g)
            c = 1 / np.sqrt(1 + t * t); s = c * t
            # x_p' = c x_p - s x_q, x_q' = s x_p + c x_q
            gp, gq = G[:, p].copy(), G[:, q].copy()
            G[:, p], G[:, q] = c * gp - s * gq, s * gp + c * gq
            gp, gq = G[p, :].copy(), G[q, :].copy()
            G[p, :], G[q, :] = c * gp - s * gq, s * gp + c * gq
            jp, jq = J[:, p].copy(), J[:, q].copy()
            J[:, p], J[:, q] = c * jp - s * jq, s * jp + c * jq
    return J
def offmax(X):
    G = X.T @ X; d = np.sqrt(np.diag(G)); C = np.abs(G) / np.outer(d, d); np.fill_diagonal(C, 0); return C.max()
def run(W, mode, tol, inner="sweep", maxr=400):
    X = W.copy(); rounds = 0
    while rounds < maxr:
        if offmax(X) < tol: break
        if mode == "cyclic":
            r = rounds % (NB - 1)
            pairs = []
            for k in range(NB // 2):
                if k == 0: P, Q = r, NB - 1
                else: P, Q = (r + k) % (NB - 1), (r - k + NB - 1) % (NB - 1)
                pairs.append((P, Q))
        else:
            G = X.T @ X; d = np.sqrt(np.diag(G)); C = G / np.outer(d, d)
            w = {}
            for P in range(NB):
                for Q in range(P + 1, NB):
                    w[(P, Q)] = np.linalg.norm(C[P*b:(P+1)*b, Q*b:(Q+1)*b])
            used = set(); pairs = []
            for (P, Q), _ in sorted(w.items(), key=lambda kv: -kv[1]):
                if P in used or Q in used: continue
                pairs.append((P, Q)); used |= {P, Q}
        for P, Q in pairs:
            cols = list(range(P*b, (P+1)*b)) + list(range(Q*b, (Q+1)*b))
            Xp = X[:, cols]; Gp = Xp.T @ Xp
            J = inner_sweep(Gp) if inner == "sweep" else np.linalg.eigh(Gp)[1]
            X[:, cols] = Xp @ J
        rounds += 1
    return rounds
for kind in ("c4", "decay", "flat"):
    W = make_W(kind)
    for tol in (1e-8, 1e-12):
        rc = run(W, "cyclic", tol, "sweep"); rd = run(W, "dynamic", tol, "sweep")
        print(f"{kind:6s} tol {tol:.0e}: cyclic {rc} rounds ({rc/(NB-1):.1f} sweeps)  dynamic {rd} rounds  ratio {rd/rc:.2f}", flush=True)
