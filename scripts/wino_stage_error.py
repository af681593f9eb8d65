"""Which stage of a Winograd 3^3 conv (forward or data gradient: the same
algorithm with flipped weights) carries its fp32 error -- host numpy study for
the round-5 gradient-accuracy work.  One output tile F(my x mx x mz), K input
channels, N outputs; every stage is rounded to fp32 as the GPU does, or kept
in float64 ("exact" list), against a float64 direct correlation.  The point
GEMM's sum over K is emulated as the MFMA chain does it: `chunk` products
summed exactly per instruction (32x32x16 bf16: 16) and rounded into a single
fp32 accumulator, or with a second fp32 level every `outer` instructions.
Direct fp32 rows: the same chain over the 27*K taps x channels.

    python scripts/wino_stage_error.py

Modes "x3" / "x3sep" (not exactness switches): the point GEMM on the exact
bf16 split, six roundings per k step into one accumulator (the kernels before
round 5) or the five small-term products into a second accumulator.
"""
import numpy as np

from wino_grad_error import F, f32


def bf16(a):
    """round to bfloat16 (nearest even), as float64"""
    u = a.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).astype(np.float64)


def split3(a):
    h = bf16(a)
    m = bf16(f32(a - h))
    return h, m, bf16(f32(a - h - m))


# the six MFMAs per 16-deep k step of the x3 kernels, in their issue order
# (plane of A, plane of B): smallest terms first, hi x hi last
X3_ORDER = ((2, 0), (1, 1), (0, 2), (1, 0), (0, 1), (0, 0))


def chain_x3(U, V, sep, chunk=16):
    """sum_k U[k] V[k] (U [K][...], V [K][...] broadcastable) on the exact bf16
    split: six MFMAs per k step, each rounding into the fp32 accumulator (sep:
    the five small-term MFMAs into a second accumulator, added at the end)"""
    u, v = split3(U), split3(V)
    acc = small = 0.0
    for c0 in range(0, U.shape[0], chunk):
        for i, j in X3_ORDER:
            p = (u[i][c0:c0 + chunk] * v[j][c0:c0 + chunk]).sum(0)
            if sep and (i, j) != (0, 0):
                small = f32(small + p)
            else:
                acc = f32(acc + p)
    return f32(acc + small) if sep else acc


def chain(prods, chunk, outer=0):
    """sum over axis 0 of prods (float64 products) as the MFMA chain rounds it"""
    acc = np.zeros(prods.shape[1:])
    tot = np.zeros(prods.shape[1:])
    n = prods.shape[0]
    for i, c0 in enumerate(range(0, n, chunk)):
        acc = f32(acc + prods[c0:c0 + chunk].sum(0))
        if outer and (i + 1) % outer == 0:
            tot = f32(tot + acc)
            acc = np.zeros_like(acc)
    return f32(tot + acc) if outer else acc


def study(tile, K=256, N=16, trials=12, chunk=16, outer=0, exact=(), seed=0):
    rng = np.random.default_rng(seed)
    my, mx, mz = tile
    (By, Gy, Ay), (Bx, Gx, Ax), (Bz, Gz, Az) = F[my], F[mx], F[mz]
    ew, ed = [], []
    for _ in range(trials):
        d = rng.standard_normal((my + 2, mx + 2, mz + 2, K)) * (rng.random((my + 2, mx + 2, mz + 2, K)) < 0.5)
        w = f32(rng.standard_normal((3, 3, 3, K, N)) / np.sqrt(27 * K))
        d = f32(d)
        ref = np.zeros((my, mx, mz, N))
        taps = []
        for a in range(3):
            for b in range(3):
                for c in range(3):
                    ref += np.einsum('yxzk,kn->yxzn', d[a:a + my, b:b + mx, c:c + mz], w[a, b, c])
                    taps.append(np.einsum('yxzk,kn->kyxzn', d[a:a + my, b:b + mx, c:c + mz], w[a, b, c]))
        U = np.einsum('py,qx,rz,yxzk->pqrk', By, Bx, Bz, d)
        V = np.einsum('pa,qb,rc,abckn->pqrkn', Gy, Gx, Gz, w)
        if "U" not in exact:
            U = f32(U)
        if "V" not in exact:
            V = f32(V)
        prods = np.einsum('pqrk,pqrkn->kpqrn', U, V)
        if "x3" in exact or "x3sep" in exact:
            M = chain_x3(np.moveaxis(U, -1, 0)[..., None], np.moveaxis(V, 3, 0), "x3sep" in exact)
        else:
            M = prods.sum(0) if "gemm" in exact else chain(prods, chunk, outer)
        Y = np.einsum('yp,xq,zr,pqrn->yxzn', Ay, Ax, Az, M)
        if "out" not in exact:
            Y = f32(Y)
        s = np.abs(ref).max()
        ew.append(np.abs(Y - ref).max() / s)
        dprods = np.concatenate(taps, 0)
        D = chain(dprods, chunk, outer)
        ed.append(np.abs(D - ref).max() / s)
    return float(np.mean(ew)), float(np.mean(ed))


if __name__ == "__main__":
    for tile in ((2, 2, 4), (4, 2, 4)):
        base, direct = study(tile)
        print(f"F{tile}: all fp32 {base:.2e}   (direct fp32 chain {direct:.2e})")
        for ex in (("U",), ("V",), ("gemm",), ("out",), ("U", "V"), ("U", "V", "out"), ("x3",), ("x3sep",)):
            print(f"   exact {'+'.join(ex):10s} {study(tile, exact=ex)[0]:.2e}")
        for outer in (2, 4):
            w, d = study(tile, outer=outer)
            print(f"   two-level every {outer} MFMAs: wino {w:.2e}, direct {d:.2e}")
