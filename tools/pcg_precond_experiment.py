import sys, time
import numpy as np, scipy.sparse as sp
sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/slam-robot_simu_amd')
import graph_oracle as go
from slamhip.graph import circle_graph
T = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
init, truth, edges = circle_graph(T, n_landmarks=64, seed=0, odom_noise=0.002)
rows = np.array([[e['time_bfr'], e['pose_bfr'], *e['obs_bfr'], e['time_aft'], e['pose_aft'], *e['obs_aft'], 0] for e in edges], dtype=float)
blocks = go.linearize(rows, init)
# sparse assembly
times = np.unique(np.concatenate([rows[:, 0], rows[:, 5]])).astype(int)
pos = {t: i for i, t in enumerate(times)}
nt = len(times); n = 3 * nt
I, J, V = [], [], []
bb = np.zeros(n)
for e, blk in zip(rows, blocks):
    i, j = pos[int(e[0])], pos[int(e[5])]
    for (r, c, o) in ((i, i, 0), (i, j, 9), (j, i, 18), (j, j, 27)):
        for a in range(3):
            for q in range(3):
                I.append(3 * r + a); J.append(3 * c + q); V.append(blk[o + 3 * a + q])
    bb[3 * i:3 * i + 3] += blk[36:39]; bb[3 * j:3 * j + 3] += blk[39:42]
for a in range(3):
    I.append(a); J.append(a); V.append(1e4)
H = sp.csr_matrix((V, (I, J)), shape=(n, n))
def pcg(H, b, Minv, tol=1e-10, maxit=20000):
    x = np.zeros_like(b); r = -b.copy(); z = Minv(r); p = z.copy(); rz = r @ z; rr0 = r @ r
    for k in range(maxit):
        if r @ r <= tol * tol * rr0: return k
        q = H @ p; al = rz / (p @ q); x += al * p; r -= al * q; z = Minv(r); rz2 = r @ z; p = z + rz2 / rz * p; rz = rz2
    return maxit
for C in (1, 2, 4, 8, 16, 32, 64):
    m = 3 * C
    nb = (n + m - 1) // m
    invs = []
    Hd = H.tolil()
    for k in range(nb):
        a, e = k * m, min(n, (k + 1) * m)
        invs.append(np.linalg.inv(H[a:e, a:e].toarray()))
    def Minv(r):
        out = np.empty_like(r)
        for k in range(nb):
            a, e = k * m, min(n, (k + 1) * m)
            out[a:e] = invs[k] @ r[a:e]
        return out
    print(C, pcg(H, bb, Minv), flush=True)
print("two-level additive: block-Jacobi + coarse aggregates")
D = [np.linalg.inv(H[3*k:3*k+3, 3*k:3*k+3].toarray()) for k in range(nt)]
Dm = sp.block_diag(D).tocsr()
for agg in (8, 16, 32, 64, 128):
    na = (nt + agg - 1) // agg
    Pi, Pj = [], []
    for t in range(nt):
        for a in range(3):
            Pi.append(3 * t + a); Pj.append(3 * (t // agg) + a)
    P = sp.csr_matrix((np.ones(len(Pi)), (Pi, Pj)), shape=(n, 3 * na))
    Ac = (P.T @ H @ P).toarray()
    Aci = np.linalg.inv(Ac)
    Minv = lambda r: Dm @ r + P @ (Aci @ (P.T @ r))
    print(agg, 3 * na, pcg(H, bb, Minv), flush=True)
