"""Where the fp32 error of the Winograd weight gradient comes from (host
numpy study for VERDICT r4 item 2).  One 3^3 'same' conv, K -> N channels,
T output tiles of F(my x mx x mz): dW = G^T [sum_t U_t (A dY_t A^T)] G, every
stage either rounded to fp32 (as the GPU does) or kept in float64, against the
float64 direct weight gradient.  The GEMM's sum over tiles is emulated in fp32
as a sequential accumulation of `chunk`-tile partial sums (an MFMA
accumulator fed 16 tiles per instruction: chunk 16), optionally with a second
fp32 level every `outer` chunks (two-level accumulation).

    python scripts/wino_grad_error.py
"""
import numpy as np

BT4 = np.array([[0.25, 0, -1.25, 0, 1, 0], [0, -0.25, -0.25, 1, 1, 0], [0, 0.25, -0.25, -1, 1, 0],
                [0, -0.5, -1, 0.5, 1, 0], [0, 0.5, -1, -0.5, 1, 0], [0, 0.25, 0, -1.25, 0, 1]])
G4 = np.array([[4, 0, 0], [2 / 3, 2 / 3, 2 / 3], [2 / 3, -2 / 3, 2 / 3], [-8 / 3, -4 / 3, -2 / 3],
               [-8 / 3, 4 / 3, -2 / 3], [0, 0, 1]])
AT4 = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 0.5, -0.5, 0], [0, 1, 1, 0.25, 0.25, 0],
                [0, 1, -1, 0.125, -0.125, 1]])
BT2 = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]])
G2 = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]])
AT2 = np.array([[1, 1, 1, 0], [0, 1, -1, -1]])
F = {2: (BT2, G2, AT2), 4: (BT4, G4, AT4)}


def f32(a):
    return a.astype(np.float32).astype(np.float64)


def study(tile, K=32, N=32, tiles=(4, 8, 16), seed=0, chunk=16, outer=0, exact=()):
    rng = np.random.default_rng(seed)
    my, mx, mz = tile
    ty, tx, tz = tiles
    H, W, D = my * ty, mx * tx, mz * tz
    x = np.maximum(rng.standard_normal((H + 2, W + 2, D + 2, K)), 0)      # post-ReLU input, zero-padded ring
    x[0], x[-1], x[:, 0], x[:, -1], x[:, :, 0], x[:, :, -1] = 0, 0, 0, 0, 0, 0
    dy = rng.standard_normal((H, W, D, N)) * (rng.random((H, W, D, N)) < 0.5)
    # float64 direct weight gradient
    ref = np.zeros((3, 3, 3, K, N))
    for a in range(3):
        for b in range(3):
            for c in range(3):
                ref[a, b, c] = np.einsum('yxzk,yxzn->kn', x[a:a + H, b:b + W, c:c + D], dy)
    (By, Gy, Ay), (Bx, Gx, Ax), (Bz, Gz, Az) = F[my], F[mx], F[mz]
    P = (my + 2) * (mx + 2) * (mz + 2)
    Us, Ms = [], []
    for iy in range(ty):
        for ix in range(tx):
            for iz in range(tz):
                d = x[iy * my:iy * my + my + 2, ix * mx:ix * mx + mx + 2, iz * mz:iz * mz + mz + 2]
                g = dy[iy * my:(iy + 1) * my, ix * mx:(ix + 1) * mx, iz * mz:(iz + 1) * mz]
                U = np.einsum('py,qx,rz,yxzk->pqrk', By, Bx, Bz, d)
                M = np.einsum('yp,xq,zr,yxzn->pqrn', Ay, Ax, Az, g)
                Us.append(U.reshape(P, K))
                Ms.append(M.reshape(P, N))
    U = np.stack(Us, 1)          # [P][T][K]
    M = np.stack(Ms, 1)          # [P][T][N]
    if "U" not in exact:
        U = f32(U)
    if "M" not in exact:
        M = f32(M)
    T = U.shape[1]
    if "gemm" in exact:
        dWh = np.einsum('ptk,ptn->pkn', U, M)
    else:
        acc = np.zeros((P, K, N))
        tot = np.zeros((P, K, N))
        for c0 in range(0, T, chunk):
            part = np.einsum('ptk,ptn->pkn', U[:, c0:c0 + chunk], M[:, c0:c0 + chunk])   # one MFMA's 16 products
            acc = f32(acc + f32(part))
            if outer and (c0 // chunk + 1) % outer == 0:
                tot = f32(tot + acc)
                acc = np.zeros_like(acc)
        dWh = f32(tot + acc) if outer else acc
    dWh = dWh.reshape(my + 2, mx + 2, mz + 2, K, N)
    dW = np.einsum('pa,qb,rc,pqrkn->abckn', Gy, Gx, Gz, dWh)
    if "out" not in exact:
        dW = f32(dW)
    return np.abs(dW - ref).max() / np.abs(ref).max()


def direct_f32(K=32, N=32, tiles=(4, 8, 16), tile=(4, 2, 4), seed=0, chunk=16):
    """the direct weight gradient with fp32 MFMA-style chunked accumulation"""
    rng = np.random.default_rng(seed)
    my, mx, mz = tile
    ty, tx, tz = tiles
    H, W, D = my * ty, mx * tx, mz * tz
    x = np.maximum(rng.standard_normal((H + 2, W + 2, D + 2, K)), 0)
    x[0], x[-1], x[:, 0], x[:, -1], x[:, :, 0], x[:, :, -1] = 0, 0, 0, 0, 0, 0
    dy = rng.standard_normal((H, W, D, N)) * (rng.random((H, W, D, N)) < 0.5)
    err = 0.0
    for a in range(3):
        for b in range(3):
            for c in range(3):
                xs = x[a:a + H, b:b + W, c:c + D].reshape(-1, K)
                g = dy.reshape(-1, N)
                ref = xs.T @ g
                acc = np.zeros((K, N))
                for m0 in range(0, xs.shape[0], chunk):
                    acc = f32(acc + f32(xs[m0:m0 + chunk].T @ g[m0:m0 + chunk]))
                err = max(err, np.abs(acc - ref).max())
    return err


if __name__ == "__main__":
    for tile in ((2, 2, 4), (4, 2, 4)):
        base = study(tile)
        print(f"F{tile}: all fp32 {base:.2e}")
        for ex in (("U",), ("M",), ("gemm",), ("out",), ("U", "M"), ("U", "M", "out")):
            print(f"   exact {'+'.join(ex):10s} {study(tile, exact=ex):.2e}")
        for outer in (4, 16):
            print(f"   two-level accumulation every {outer} MFMA chunks: {study(tile, outer=outer):.2e}")
