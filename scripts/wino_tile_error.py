"""fp32 rounding of Winograd 3-D tiles: F(2,3)/F(4,3) per axis, forward conv, K channels
summed in fp32 (as the point GEMMs do), vs a float64 direct correlation."""
import numpy as np
# F(4,3), points 0, +-1, +-1/2, inf (conv3d.hip ZT<4>)
BT4 = np.array([[0.25, 0, -1.25, 0, 1, 0], [0, -0.25, -0.25, 1, 1, 0], [0, 0.25, -0.25, -1, 1, 0],
                [0, -0.5, -1, 0.5, 1, 0], [0, 0.5, -1, -0.5, 1, 0], [0, 0.25, 0, -1.25, 0, 1]])
G4 = np.array([[4, 0, 0], [2/3, 2/3, 2/3], [2/3, -2/3, 2/3], [-8/3, -4/3, -2/3], [-8/3, 4/3, -2/3], [0, 0, 1]])
AT4 = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 0.5, -0.5, 0], [0, 1, 1, 0.25, 0.25, 0], [0, 1, -1, 0.125, -0.125, 1]])
# F(2,3), points 0, +-1, inf
BT2 = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]])
G2 = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]])
AT2 = np.array([[1, 1, 1, 0], [0, 1, -1, -1]])
F = {2: (BT2, G2, AT2), 4: (BT4, G4, AT4)}
rng = np.random.default_rng(0)
def run(my, mx, mz, K=256, N=32, trials=40):
    errs = []
    for _ in range(trials):
        (By, Gy, Ay), (Bx, Gx, Ax), (Bz, Gz, Az) = F[my], F[mx], F[mz]
        d = rng.standard_normal((my + 2, mx + 2, mz + 2, K))
        w = rng.standard_normal((3, 3, 3, K, N)) / np.sqrt(27 * K)
        # float64 direct
        ref = np.zeros((my, mx, mz, N))
        for a in range(3):
            for b in range(3):
                for c in range(3):
                    ref += np.einsum('yxzk,kn->yxzn', d[a:a + my, b:b + mx, c:c + mz], w[a, b, c])
        d32, w32 = d.astype(np.float32), w.astype(np.float32)
        U = np.einsum('py,qx,rz,yxzk->pqrk', By.astype(np.float32), Bx.astype(np.float32), Bz.astype(np.float32), d32).astype(np.float32)
        V = np.einsum('pa,qb,rc,abckn->pqrkn', Gy.astype(np.float32), Gx.astype(np.float32), Gz.astype(np.float32), w32).astype(np.float32)
        M = np.einsum('pqrk,pqrkn->pqrn', U, V).astype(np.float32)      # fp32 products/sums (approx.)
        Y = np.einsum('yp,xq,zr,pqrn->yxzn', Ay.astype(np.float32), Ax.astype(np.float32), Az.astype(np.float32), M).astype(np.float32)
        # direct fp32 for comparison
        D = np.zeros((my, mx, mz, N), np.float32)
        for a in range(3):
            for b in range(3):
                for c in range(3):
                    D += np.einsum('yxzk,kn->yxzn', d32[a:a + my, b:b + mx, c:c + mz], w32[a, b, c]).astype(np.float32)
        s = np.abs(ref).max()
        errs.append((np.sqrt(np.mean((Y - ref) ** 2)) / s, np.sqrt(np.mean((D - ref) ** 2)) / s))
    e = np.array(errs).mean(0)
    return e
for tile in ((2, 2, 4), (4, 2, 4), (4, 4, 4), (2, 2, 2)):
    e = run(*tile)
    print(f"F{tile}: winograd rms rel err {e[0]:.2e}, direct fp32 {e[1]:.2e}, ratio {e[0] / e[1]:.2f}")
