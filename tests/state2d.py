"""Deterministic 2-D species-step states (test infrastructure).

A forward-Euler species step (forward_euler, src/m_fluid.f90:21-99) reads the
densities of its input states, |E| (cell-centred, ghost cells included) and
the face field; it never reaches the field solve. ``build_state`` makes such
a state for a 2-D case without a field solve, so that it can be built the
same way in the build container -- where oracle/make_replay2d.py hands it to
the reference's own forward_euler (oracle/_ref/2d/replay_step) and commits
the reference's output -- and on the GPU box, where tests/test_2d_replay.py
runs libafivo_hip_2d.so's step on it and compares with that output.

The tree is afh.amr.AfTree in 2-D (af_init + af_refine_up_to_lvl, then
boxes near a point refined further, 2:1 balanced by af_adjust_refinement's
own rules), so it has refinement boundaries on several levels. The fields
are smooth closed forms of the cell and face centres (numpy, fixed
parameters, no random numbers): every species a background plus Gaussians,
phi a uniform field plus a Gaussian bump, |E| and the face field its exact
gradient.
"""
import numpy as np

import golden
from afh.amr import AfTree, DO_REF, KEEP_REF
from afh.driver import Case

# (case, uniform level, finest level, refinement centre (relative), radius
# (relative), dt)
SPECS = {
    "s2d": ("case_s2d", 4, 7, (0.5, 0.3), 0.08, 2e-12),
    "test_2d": ("rtest_test_2d", 4, 7, (0.5, 0.3), 0.08, 2e-12),
}
STAGES = (  # (s_deriv, s_prev, w_prev, s_out): the two Heun sub-steps
    (0, [0], [1.0], 1),
    (1, [0, 1], [0.5, 0.5], 0),
)


def build_tree(c, lvl_uniform, lvl_max, centre, radius):
    L = c.ra("domain_len")
    af = AfTree(c.i("box_size"), c.ra("domain_origin") + L, c.ia("coarse_grid_size_value"),
                r_min=c.ra("domain_origin"))
    af.refine_up_to_lvl(lvl_uniform)
    p = np.asarray(centre) * L
    for lvl in range(lvl_uniform, lvl_max):
        def fn(ids, lvl=lvl):
            f = []
            for b in ids:
                mid = af.r_min[b] + 0.5 * af.nc * af.dr[b]
                near = np.linalg.norm(mid - p) < radius * L[0] + af.nc * af.dr[b][0]
                f.append(DO_REF if (af.lvl[b] == lvl and near) else KEEP_REF)
            return np.array(f), np.zeros(len(ids), np.uint32)
        af.adjust_refinement(fn)
    return af


def _cells(af, b, shift=(0.5, 0.5), n=None):
    """Points r_min + (i - shift) dr for i = 0..n-1 (i fastest), as (n^2, 2)."""
    n = af.nc + 2 if n is None else n
    idx = np.arange(n, dtype=float)
    x = af.r_min[b][0] + (idx - shift[0]) * af.dr[b][0]
    y = af.r_min[b][1] + (idx - shift[1]) * af.dr[b][1]
    yy, xx = np.meshgrid(y, x, indexing="ij")
    return xx, yy


def build_state(name):
    """(Case, AfTree, {iv: cc array}, {ivf: fc array}, dt) of SPECS[name]."""
    case_name, lu, lm, centre, radius, dt = SPECS[name]
    c = Case(golden.load(case_name))
    af = build_tree(c, lu, lm, centre, radius)
    L = c.ra("domain_len")
    nb, nc = af.highest_id, af.nc
    ng, nf = nc + 2, nc + 1
    names = list(c.sa("cc_names"))
    n_cc, n_fc = len(names), len(c.sa("fc_names"))
    (i_phi, i_e, i_pos, i_efld, i_rhs, i_tmp, _, f_flux, f_field, _) = c.ia("ivars")
    cc = {iv: np.zeros((nb, ng, ng)) for iv in range(1, n_cc + 1)}
    fc = {iv: np.zeros((nb, 2, nf, nf)) for iv in range(1, n_fc + 1)}
    V = c.r("current_voltage")
    pc = np.asarray(centre) * L
    w = 0.06 * L[0]
    bump = 0.02 * abs(V)

    def phi_of(x, y):
        return V * y / L[1] + bump * np.exp(-((x - pc[0]) ** 2 + (y - pc[1]) ** 2) / w ** 2)

    def grad_of(x, y):
        g = np.exp(-((x - pc[0]) ** 2 + (y - pc[1]) ** 2) / w ** 2)
        gx = bump * g * (-2 * (x - pc[0]) / w ** 2)
        gy = V / L[1] + bump * g * (-2 * (y - pc[1]) / w ** 2)
        return gx, gy

    dens = list(c.ia("all_densities"))
    used = [b for b in range(1, nb + 1) if af.in_use[b]]
    for b in used:
        xx, yy = _cells(af, b)
        for k, iv in enumerate(dens):
            # background + a seed Gaussian + a species-specific offset Gaussian
            q = np.array([0.5 + 0.03 * np.cos(k), 0.3 + 0.03 * np.sin(k)]) * L
            a = 1e15 * (1 + 0.1 * k) + 5e18 / (1 + k) * np.exp(
                -((xx - pc[0]) ** 2 + (yy - pc[1]) ** 2) / (0.5 * w) ** 2)
            a = a + 1e17 * np.exp(-((xx - q[0]) ** 2 + (yy - q[1]) ** 2) / w ** 2)
            cc[iv][b - 1] = a
            # state 1: a perturbed copy (Heun stage 2 reads both)
            cc[iv + 1][b - 1] = a * (1 + 0.01 * np.sin(1e3 * xx + 2e3 * yy + k))
        cc[i_phi][b - 1] = phi_of(xx, yy)
        gx, gy = grad_of(xx, yy)
        cc[i_efld][b - 1] = np.sqrt(gx * gx + gy * gy)
        # face field -dphi/dx on x faces (i = 1..nc+1 at r_min + (i-1) dx),
        # -dphi/dy on y faces, fc(1:nc+1, 1:nc+1, dim)
        fx, fy = _cells(af, b, shift=(1.0, 0.5), n=nf)
        fc[f_field][b - 1, 0] = -grad_of(fx, fy)[0]
        fx, fy = _cells(af, b, shift=(0.5, 1.0), n=nf)
        fc[f_field][b - 1, 1] = -grad_of(fx, fy)[1]
    return c, af, cc, fc, dt


def write_record(path, af, cc, fc, dt, time, stage):
    """oracle/harness/replay_step.f90's record (2-D box shapes)."""
    import struct
    s_deriv, s_prev, w_prev, s_out = stage
    hid = af.highest_id
    used = [b for b in range(1, hid + 1) if af.in_use[b]]
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", hid, len(cc), len(fc), af.nc))
        for b in range(1, hid + 1):
            ix = tuple(af.ix[b]) + (0,) if af.in_use[b] else (0, 0, 0)
            f.write(struct.pack("<6i", af.parent[b], af.lvl[b], *ix, int(af.in_use[b])))
        f.write(struct.pack("<ddii", dt, time, s_deriv, len(s_prev)))
        f.write(struct.pack("<%di" % len(s_prev), *s_prev))
        f.write(struct.pack("<%dd" % len(w_prev), *w_prev))
        f.write(struct.pack("<i", s_out))
        for iv in range(1, len(cc) + 1):
            for b in used:
                f.write(np.ascontiguousarray(cc[iv][b - 1]).tobytes())
        for iv in range(1, len(fc) + 1):
            for b in used:
                f.write(np.ascontiguousarray(fc[iv][b - 1]).tobytes())
    return used
