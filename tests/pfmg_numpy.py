"""TEST INFRASTRUCTURE: a second statement of the HYPRE StructPFMG set-up
(HYPRE 2.31.0 struct_ls/pfmg_setup.c, pfmg_setup_interp.c, pfmg_setup_rap*,
as afivo calls it: afivo/src/m_coarse_solver.f90:404-439), written apart
from csrc/afh_pfmg.h so that tests/test_pfmg.py can check the set-up the
library and the C oracle share.

Where afh_pfmg.h loops over stencil entries point by point, this works on
whole arrays and on sparse matrices: the coarse operators are the matrix
products R A P (scipy.sparse, R = P^T), not the stencil-walking Galerkin
loop. Only the coarsening decisions -- which compare sums of floating-point
numbers, ties included -- follow HYPRE's own summation order (the grid's
points, i fastest), as HYPRE's serial set-up does.
"""
import math

import numpy as np
import scipy.sparse as sp

OFFS = [(s % 3 - 1, (s // 3) % 3 - 1, s // 9 - 1) for s in range(27)]  # (dx, dy, dz)
A7_OFFS = [(0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)]


def dxyz_of(a7, n, ndim):
    """PFMGComputeDxyz: per direction the mean over the points of
    -sign(a_c) (a_-d + a_+d), relative to the largest; dxyz = mean^-1/2;
    plus the flag for coefficients that vary (squared coefficient of
    variation > 0.1)."""
    n0 = n[0] * n[1] * n[2]
    mean, sq = [0.0] * 3, [0.0] * 3
    for d in range(ndim):
        sgn = np.where(a7[:, 0] < 0.0, -1.0, 1.0)
        t = (-sgn * (a7[:, 1 + 2 * d] + a7[:, 2 + 2 * d])).tolist()
        s = s2 = 0.0
        for v in t:  # HYPRE's box loop order: one running sum
            s += v
            s2 += v * v
        mean[d], sq[d] = s / n0, s2 / n0
    cmax = max(mean)
    cmax = 1.0 if cmax == 0.0 else cmax
    dxyz = [math.sqrt(1.0 / (m / cmax)) if m > 0 else 1.0e123 for m in mean]
    with np.errstate(divide="ignore", invalid="ignore"):
        cv2 = [np.float64(sq[d] - mean[d] * mean[d]) / np.float64(mean[d] * mean[d])
               for d in range(ndim)]
    flag = any(v > 0.1 for v in cv2)
    return dxyz, flag


def coarsening(n, dxyz, flag, ndim):
    """Semicoarsening along the smallest dxyz with more than one point left
    (the first on a tie), doubling it; relaxation where the direction was
    coarsened before since the last relaxed level, on the finest and the
    coarsest; the Jacobi weight 2 / (3 - beta / alpha) (2/3 with varying
    coefficients, 1 on the coarsest). Returns dims, cdir, active, w."""
    max_levels = 1 + sum(int(math.floor(math.log2(n[d]))) + 2 for d in range(ndim))
    dx = list(dxyz)
    dims, cdir, active, w = [list(n)], [], [], []
    seen = {0, 1, 2}  # forces relaxation on the finest level
    while True:
        cur = dims[-1]
        cand = [d for d in range(ndim) if cur[d] > 1]
        cd = min(cand, key=lambda d: (dx[d], d)) if cand else -1
        wl = 1.0
        if cd != -1:
            if flag:
                wl = 2.0 / 3.0
            else:
                alpha = sum(1.0 / (dx[d] * dx[d]) for d in range(ndim))
                beta = sum(1.0 / (dx[d] * dx[d]) for d in range(ndim) if d != cd)
                wl = 2.0 / (3.0 - (0.0 if beta == alpha else beta / alpha))
            if len(dims) == max_levels:
                cd = -1
        if cd == -1:  # the coarsest (its weight as computed, 1 with nothing left)
            cdir.append(-1), active.append(1), w.append(wl)
            return dims, cdir, active, w
        cdir.append(cd)
        w.append(wl)
        if cd in seen:
            active.append(1)
            seen = {cd}
        else:
            active.append(0)
            seen.add(cd)
        dx[cd] *= 2
        nxt = list(cur)
        nxt[cd] //= 2
        dims.append(nxt)


def stencil_matrix(A27, n):
    """The sparse matrix of a 27-point stencil (A27: (points, 27), points in
    the grid's order, i fastest); entries reaching outside the grid dropped."""
    nx, ny, nz = n
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    i, j, k = i.ravel(), j.ravel(), k.ravel()
    rows, cols, vals = [], [], []
    for s, (ox, oy, oz) in enumerate(OFFS):
        ii, jj, kk = i + ox, j + oy, k + oz
        ok = (ii >= 0) & (ii < nx) & (jj >= 0) & (jj < ny) & (kk >= 0) & (kk < nz) & \
            (A27[:, s] != 0.0)
        p = np.nonzero(ok)[0]
        rows.append(p)
        cols.append((kk[p] * ny + jj[p]) * nx + ii[p])
        vals.append(A27[p, s])
    n0 = nx * ny * nz
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                         shape=(n0, n0))


def interpolation(A27, n, cd):
    """Operator-dependent interpolation along cd (PFMGSetupInterpOp): at the
    odd points (1-based) the weights toward the lower / upper coarse
    neighbour are minus the row sums of A's entries at offset -1 / +1 along
    cd over the sum of those at offset 0 (0 when that sum is 0, and 0 where
    A's pure -1 / +1 entry is 0); the even points are injected. Returns the
    sparse P (fine x coarse) and the (points, 2) weights."""
    o = np.array([off[cd] for off in OFFS])
    centre = A27[:, o == 0].sum(axis=1)
    lo = -A27[:, o == -1].sum(axis=1)
    hi = -A27[:, o == 1].sum(axis=1)
    safe = np.where(centre == 0.0, 1.0, centre)
    lo = np.where(centre == 0.0, 0.0, lo / safe)
    hi = np.where(centre == 0.0, 0.0, hi / safe)
    e_lo = [0, 0, 0]
    e_lo[cd] = -1
    e_hi = [0, 0, 0]
    e_hi[cd] = 1
    lo = np.where(A27[:, OFFS.index(tuple(e_lo))] == 0.0, 0.0, lo)
    hi = np.where(A27[:, OFFS.index(tuple(e_hi))] == 0.0, 0.0, hi)
    nx, ny, nz = n
    nc = list(n)
    nc[cd] //= 2
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    q = [i.ravel() + 1, j.ravel() + 1, k.ravel() + 1]  # 1-based
    odd = (q[cd] % 2) == 1
    W = np.zeros((len(odd), 2))
    W[odd, 0], W[odd, 1] = lo[odd], hi[odd]

    def cix(c):
        return ((c[2] - 1) * nc[1] + (c[1] - 1)) * nc[0] + (c[0] - 1)

    rows, cols, vals = [], [], []
    p = np.arange(len(odd))
    ev = ~odd
    c = [x.copy() for x in q]
    c[cd] = q[cd] // 2
    rows.append(p[ev]), cols.append(cix([x[ev] for x in c])), vals.append(np.ones(ev.sum()))
    for side, wcol in ((-1, 0), (1, 1)):
        cc = [x.copy() for x in q]
        cc[cd] = (q[cd] + side) // 2
        ok = odd & (cc[cd] >= 1) & (cc[cd] <= nc[cd])
        if side < 0:
            ok &= q[cd] >= 3
        rows.append(p[ok]), cols.append(cix([x[ok] for x in cc])), vals.append(W[ok, wcol])
    P = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(len(odd), nc[0] * nc[1] * nc[2]))
    return P, W


def setup(a7, n):
    """The hierarchy: dims, cdir, active, w per level; the operators as
    sparse matrices (level 0 from a7), and the interpolation weights."""
    ndim = 3 if n[2] > 1 else 2
    dxyz, flag = dxyz_of(a7, n, ndim)
    dims, cdir, active, w = coarsening(n, dxyz, flag, ndim)
    A27 = np.zeros((len(a7), 27))
    for c, off in enumerate(A7_OFFS):
        if ndim == 2 and off[2] != 0:
            continue
        A27[:, OFFS.index(off)] = a7[:, c]
    mats, weights = [stencil_matrix(A27, dims[0])], []
    for l in range(len(dims) - 1):
        P, W = interpolation(A27, dims[l], cdir[l])
        weights.append(W)
        Ac = (P.T @ mats[-1] @ P).tocsr()
        mats.append(Ac)
        A27 = stencil_of(Ac, dims[l + 1])
    return dict(dims=dims, cdir=cdir, active=active, w=w, mats=mats, weights=weights)


def stencil_of(M, n):
    """(points, 27) stencil of a sparse matrix on grid n (entries beyond the
    27-point neighbourhood are an error)."""
    nx, ny, nz = n
    M = M.tocoo()
    r, c = M.row, M.col
    ri, rj, rk = r % nx, (r // nx) % ny, r // (nx * ny)
    ci, cj, ck = c % nx, (c // nx) % ny, c // (nx * ny)
    ox, oy, oz = ci - ri, cj - rj, ck - rk
    assert np.all(np.abs(ox) <= 1) and np.all(np.abs(oy) <= 1) and np.all(np.abs(oz) <= 1)
    s = (oz + 1) * 9 + (oy + 1) * 3 + (ox + 1)
    out = np.zeros((nx * ny * nz, 27))
    np.add.at(out, (r, s), M.data)
    return out
