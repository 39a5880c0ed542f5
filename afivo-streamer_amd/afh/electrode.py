"""Electrode operators on the host: the level-set function of the streamer's
electrode and the variable multigrid stencils of the boxes it crosses
(afivo/src/m_af_multigrid.f90, restated over numpy arrays).

In the drop-in, afivo's own ``mg_set_operators_tree`` computes these on the
Fortran side and hands them to the library (afh_mg_set_box_stencil /
afh_mg_set_box_lsf). The Python driver (afh.driver) has no Fortran side, so
this module computes the same numbers:

* ``rod_lsf`` / ``sphere_lsf`` (src/m_field.f90:621-630) over GM_dist_line
  (src/m_geometry.f90:23-51), the lsf cell values of set_lsf_box (608-619);
* ``box_operators``: mg_set_box_tag (m_af_multigrid.f90:1100-1131) ->
  store_lsf_distance_matrix (977-1097: get_possible_lsf_root_mask 955-973,
  mg_lsf_dist_gss 1629-1664 with bisection 1667-1689 and gss 1694-1759,
  the search along numerical_gradient 2144-2170) -> mg_box_lsf_stencil
  (1762-1834) and the bc_correction of mg_set_operators_lvl (1156-1160).

Every search runs for all cells at once (numpy masks per iteration), with the
Fortran expressions in the Fortran operand order, so the stencils are those
of the reference's code (tests/test_electrode_ops.py against the rod8
fixture, which holds the reference's own stencils).
"""
import math

import numpy as np

EPS = np.finfo(float).eps
SQRT_EPS = math.sqrt(EPS)
# mg_t defaults (m_af_types.f90:604-616)
LSF_GRADIENT_SAFETY_FACTOR = 1.5
LSF_TOL = 1e-8
LSF_MIN_REL_DISTANCE = 1e-4
MAX_ITER = 100


def norm2(v):
    """NORM2 of the rows of v (..., d) as the Fortran runtime the reference
    is built with computes it (flang's Norm2Accumulator, read from its
    object code): the largest |x| so far m and s = sum (x/m)^2 without the
    term of m itself, element by element in order; m sqrt(s + 1)."""
    v = np.abs(np.asarray(v, float))
    m = np.zeros(v.shape[:-1])
    s = np.zeros(v.shape[:-1])
    for q in range(v.shape[-1]):
        a = v[..., q]
        first = m == 0
        up = ~first & (a > m)
        keep = ~first & ~up
        with np.errstate(divide="ignore", invalid="ignore"):
            t = np.where(up, m / np.where(up, a, 1.0), 0.0)
            t = t * t
            s = np.where(up, s * t + t, s)
            u = np.where(keep, a / np.where(keep, m, 1.0), 0.0)
            s = np.where(keep, s + u * u, s)
        m = np.where(first | up, a, m)
    return m * np.sqrt(s + 1.0)


def _dot3(a, b):
    return a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1] + a[..., 2] * b[..., 2]


def dist_line(r, r0, r1):
    """GM_dist_line (m_geometry.f90:23-51) at points r (..., 3)."""
    r = np.asarray(r, float)
    d = r1 - r0
    line_len2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2]
    frac = _dot3(r - r0, d)
    lo, hi = frac <= 0.0, frac >= line_len2
    mid = r - (r0 + (frac / line_len2)[..., None] * d)
    dv = np.where(lo[..., None], r - r0, np.where(hi[..., None], r - r1, mid))
    return norm2(dv)


class RodLSF:
    """rod_lsf (src/m_field.f90:626-630): distance to the segment r0-r1
    minus the radius; the electrode at the applied voltage
    (field_electrode_grounded = f, m_field.f90:439-443)."""

    def __init__(self, r0, r1, radius):
        self.r0, self.r1 = np.asarray(r0, float), np.asarray(r1, float)
        self.radius = float(radius)
        self.length_scale = self.radius  # mg%lsf_length_scale = rod_radius

    def __call__(self, r):
        return dist_line(r, self.r0, self.r1) - self.radius


class SphereLSF:
    """sphere_lsf (src/m_field.f90:621-624)."""

    def __init__(self, r0, radius):
        self.r0, self.radius = np.asarray(r0, float), float(radius)
        self.length_scale = self.radius

    def __call__(self, r):
        return norm2(np.asarray(r, float) - self.r0) - self.radius


def cell_centers(r_min, dr, nc, lo=1, hi=None):
    """af_r_cc (m_af_types.f90:1035-1040) for cells lo..hi of a box, as an
    array [k][j][i][3]."""
    hi = nc if hi is None else hi
    ix = np.arange(lo, hi + 1) - 0.5
    r = np.empty((len(ix),) * 3 + (3,))
    r[..., 0] = r_min[0] + ix[None, None, :] * dr[0]
    r[..., 1] = r_min[1] + ix[None, :, None] * dr[1]
    r[..., 2] = r_min[2] + ix[:, None, None] * dr[2]
    return r


def numerical_gradient(f, r):
    """numerical_gradient (m_af_multigrid.f90:2144-2170) at points r (n, 3)."""
    step = np.maximum(EPS, SQRT_EPS * np.abs(r))
    g = np.empty_like(r)
    for d in range(3):
        e = r.copy()
        e[:, d] = r[:, d] - step[:, d]
        flo = f(e)
        e[:, d] = r[:, d] + step[:, d]
        fhi = f(e)
        g[:, d] = (fhi - flo) / (2 * step[:, d])
    return g


def bisection(f, a, b, tol=LSF_TOL, max_iter=MAX_ITER):
    """bisection (m_af_multigrid.f90:1667-1689) for rows of a, b (n, 3)."""
    a, b = a.copy(), b.copy()
    c = np.zeros_like(a)
    act = np.ones(len(a), bool)
    for _ in range(max_iter):
        if not act.any():
            break
        ia = np.nonzero(act)[0]
        cc = 0.5 * (a[ia] + b[ia])
        c[ia] = cc
        fc = f(cc)
        stop = (0.5 * norm2(b[ia] - a[ia]) < tol) | (np.abs(fc) <= 0)
        go = ~stop
        left = go & (fc * f(a[ia]) >= 0)
        right = go & ~left
        a[ia[left]] = cc[left]
        b[ia[right]] = cc[right]
        act[ia[stop]] = False
    return c


def gss_bracket(f, a0, b0, minimization, tol=LSF_TOL):
    """gss (m_af_multigrid.f90:1694-1759) with find_bracket for rows of a0,
    b0 (n, 3); minimization (n,) bool. Returns (lo, hi) bracket ends."""
    invphi = (math.sqrt(5.0) - 1) / 2
    invphi2 = (3 - math.sqrt(5.0)) / 2
    a, b = a0.copy(), b0.copy()
    h = b - a
    nh = norm2(h)
    lo, hi = a.copy(), b.copy()
    todo = ~(nh <= tol)
    if not todo.any():
        return lo, hi
    idx = np.nonzero(todo)[0]
    a, b, h, mn = a[idx], b[idx], h[idx], minimization[idx]
    n = np.array([int(math.ceil(math.log(tol / x) / math.log(invphi))) for x in nh[idx]])
    c = a + invphi2 * h
    d = a + invphi * h
    ya, yc, yd = f(a), f(c), f(d)
    act = np.ones(len(idx), bool)
    for k in range(1, int(n.max()) if len(n) else 1):
        act &= k <= n - 1
        if not act.any():
            break
        w = np.nonzero(act)[0]
        sel = (yc[w] < yd[w]) == mn[w]
        s1, s2 = w[sel], w[~sel]
        # branch 1: b = d, d = c, yd = yc, h = invphi h, c = a + invphi2 h
        b[s1] = d[s1]
        d[s1] = c[s1]
        yd[s1] = yc[s1]
        h[s1] = invphi * h[s1]
        c[s1] = a[s1] + invphi2 * h[s1]
        if len(s1):
            yc[s1] = f(c[s1])
        # branch 2: a = c, c = d, yc = yd, h = invphi h, d = a + invphi h
        a[s2] = c[s2]
        c[s2] = d[s2]
        yc[s2] = yd[s2]
        h[s2] = invphi * h[s2]
        d[s2] = a[s2] + invphi * h[s2]
        if len(s2):
            yd[s2] = f(d[s2])
        done = (ya[w] * yc[w] <= 0) & (ya[w] * yd[w] <= 0)
        act[w[done]] = False
    sel = (yc < yd) == mn
    lo[idx] = np.where(sel[:, None], a, c)
    hi[idx] = np.where(sel[:, None], d, b)
    return lo, hi


def lsf_dist_gss(f, a, b):
    """mg_lsf_dist_gss (m_af_multigrid.f90:1629-1664): relative distance in
    [lsf_min_rel_distance, 1] from a to the boundary along a -> b (1: none),
    for rows of a, b (n, 3)."""
    la, lb = f(a), f(b)
    dist = np.ones(len(a))
    root = np.zeros_like(a)
    has = np.zeros(len(a), bool)
    direct = la * lb <= 0
    if direct.any():
        root[direct] = bisection(f, a[direct], b[direct])
        has[direct] = True
    br = ~direct
    if br.any():
        ib = np.nonzero(br)[0]
        lo, hi = gss_bracket(f, a[ib], b[ib], la[ib] >= 0)
        b_new = np.where((f(lo) * la[ib] <= 0)[:, None], lo, hi)
        ok = ~(f(b_new) * la[ib] > 0)
        if ok.any():
            root[ib[ok]] = bisection(f, a[ib[ok]], b_new[ok])
            has[ib[ok]] = True
    if has.any():
        d = norm2(root[has] - a[has]) / norm2(b[has] - a[has])
        dist[has] = np.maximum(d, LSF_MIN_REL_DISTANCE)
    return dist


def box_operators(f, lsf_cells, r_min, dr, nc, boundary_value):
    """mg_set_box_tag + mg_store_operator_stencil for one box (see
    boxes_operators)."""
    return boxes_operators(f, [(lsf_cells, r_min, dr)], nc, boundary_value)[0]


def boxes_operators(f, boxes, nc, boundary_value):
    """mg_set_box_tag + mg_store_operator_stencil for boxes [(lsf_cells,
    r_min, dr)], every search over the cells of all boxes at once.

    lsf_cells: the box's lsf values [k][j][i] over cells 1..nc (set_lsf_box).
    Per box: None when it carries no boundary (store_lsf_distance_matrix
    found no distance < 1: an ordinary box), else (v, f_bc, ix, dd): v
    [k][j][i][7] the variable 7-point stencil, f_bc [k][j][i] the
    bc_correction (f times boundary_value), ix (n, 3) the 1-based cells with
    a boundary neighbour and dd (n, 6) their distances (the
    mg_lsf_distance_key stencil that mg_box_lpllsf_gradient reads)."""
    nb_ = len(boxes)
    n3 = nc * nc * nc
    rmins = np.array([np.asarray(b[1], float) for b in boxes]).reshape(nb_, 3)
    drs = np.array([np.asarray(b[2], float) for b in boxes]).reshape(nb_, 3)
    out = [None] * nb_
    if not nb_:
        return out
    cen = np.concatenate([cell_centers(rmins[q], drs[q], nc).reshape(-1, 3)
                          for q in range(nb_)])  # per box k, j, i order
    lsf = np.concatenate([np.asarray(b[0], float).reshape(-1) for b in boxes])
    box_of = np.repeat(np.arange(nb_), n3)
    # get_possible_lsf_root_mask
    dmax = norm2(drs)[box_of]
    gradnorm = norm2(numerical_gradient(f, cen))
    mask = np.abs(lsf) < dmax * gradnorm * LSF_GRADIENT_SAFETY_FACTOR
    if not mask.any():
        return out
    im = np.nonzero(mask)[0]
    a = cen[im]
    bq = box_of[im]
    cell = im - bq * n3
    kji = np.stack(np.unravel_index(cell, (nc, nc, nc)), axis=1)
    ijk0 = kji[:, ::-1] + 1
    dd = np.ones((len(im), 6))
    for nb in range(6):
        d, sgn = nb // 2, -1 if nb % 2 == 0 else 1
        b = a.copy()
        # af_r_cc of the neighbour cell (its own index, not a + dr)
        b[:, d] = rmins[bq, d] + ((ijk0[:, d] + sgn) - 0.5) * drs[bq, d]
        dd[:, nb] = lsf_dist_gss(f, a, b)
    # the search along the gradient where no boundary was found, in boxes
    # coarser than the electrode's length scale
    min_dr = np.min(drs, axis=1)[bq]
    cand = np.nonzero(np.all(dd >= 1, axis=1) & (min_dr > f.length_scale))[0]
    if len(cand):
        n_steps = np.ceil(min_dr[cand] / f.length_scale).astype(int)
        lc = lsf[im[cand]]
        step = np.where(lc >= 0, abs(f.length_scale), -abs(f.length_scale))
        x = a[cand].copy()
        act = np.ones(len(cand), bool)
        for it in range(int(n_steps.max())):
            act &= it < n_steps
            w = np.nonzero(act)[0]
            if not len(w):
                break
            g = numerical_gradient(f, x[w])
            g = g / np.maximum(norm2(g), 1e-50)[:, None]
            x[w] = x[w] - g * step[w][:, None]
            hit = f(x[w]) * lc[w] <= 0
            act[w[hit]] = False
        dist = lsf_dist_gss(f, a[cand], x)
        near = dist < 1
        if near.any():
            q = cand[near]
            dvec = x[near] - a[q]
            dist = dist[near] * norm2(dvec) / min_dr[q]
            dim = np.argmax(np.abs(dvec), axis=1)
            nbi = 2 * dim + (dvec[np.arange(len(q)), dim] > 0)
            dd[q, nbi] = dist
    keep = np.any(dd < 1.0, axis=1)
    for q in np.unique(bq[keep]):
        sel = keep & (bq == q)
        ix_cells = cell[sel]
        kji = np.stack(np.unravel_index(ix_cells, (nc, nc, nc)), axis=1)
        ix = (kji[:, ::-1] + 1).astype(np.int32)
        dds = dd[sel]
        # mg_box_lsf_stencil
        all_d = np.ones((n3, 6))
        all_d[ix_cells] = dds
        dr2 = drs[q] * drs[q]
        v = np.zeros((n3, 7))
        for idim in range(3):
            lo, hi = all_d[:, 2 * idim], all_d[:, 2 * idim + 1]
            v[:, 1 + 2 * idim] = 1 / (0.5 * dr2[idim] * (lo + hi) * lo)
            v[:, 2 + 2 * idim] = 1 / (0.5 * dr2[idim] * (lo + hi) * hi)
        sm = v[:, 1]
        for c in range(2, 7):  # -sum(v(2:)), left to right
            sm = sm + v[:, c]
        v[:, 0] = -sm
        fb = np.zeros(n3)
        for n in range(6):
            inside = all_d[:, n] < 1.0
            fb = np.where(inside, fb - v[:, n + 1], fb)
            v[inside, n + 1] = 0.0
        shape = (nc, nc, nc)
        out[q] = (v.reshape(shape + (7,)), (fb * boundary_value).reshape(shape), ix, dds)
    return out
