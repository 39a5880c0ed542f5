"""electrode_species_bc (src/streamer.f90:578-636): species inside the
electrode (lsf < 0) are zeroed; with Neumann-zero species boundary conditions
the cells next to the gas get the mean electron density of their gas
neighbours (copied to the first positive ion).

The streamer module that holds this routine is unbuildable here (it needs
Silo), so no reference-generated vectors cover it: the oracle is pinned by
the numpy restatement below (same summation order, bitwise), and the HIP
library must equal the oracle bitwise."""
import numpy as np
import pytest

from afh import capi
from afh.model import Fluid, Tree
from afh.tree import uniform_tree

NP = 16
X = np.linspace(0.0, 1000.0, NP)
TD = np.stack([1e24 + 0 * X, 1e24 + 0 * X], axis=1)
CHEM = np.stack([1e-16 + 0 * X], axis=1)
L = 2e-3


def make_case(lib, device, seed=5):
    rng = np.random.default_rng(seed)
    topo = uniform_tree(8, (8, 8, 8), (L, L, L), 2)
    t = Tree(lib, topo, 5, 2, device=device)   # e, M+, M-, |E|, lsf
    neu = [(capi.BC_NEUMANN, 0.0)] * 6
    for iv in range(1, 6):
        t.set_cc_methods(iv, neu, capi.RB_GC_INTERP_LIM)
    nb, ng = t.n_boxes, t.nc + 2
    # lsf of a sphere (negative inside) at the cell centres of every box
    lsf = np.zeros(t.cc_shape)
    for q in range(nb):
        r0 = np.asarray(topo["meta_r_min"][q])
        dr = np.asarray(topo["meta_dr"][q])
        c = (np.arange(ng) - 0.5)
        z, y, x = np.meshgrid(r0[2] + c * dr[2], r0[1] + c * dr[1], r0[0] + c * dr[0],
                              indexing="ij")
        lsf[q] = np.sqrt((x - 0.45 * L) ** 2 + (y - 0.5 * L) ** 2 + (z - 0.55 * L) ** 2) - 0.3 * L
    # exact zeros on a few cells: neither inside nor gas
    lsf[np.abs(lsf) < 1e-5] = 0.0
    t.put_cc(5, lsf)
    for iv in (1, 2, 3):
        t.put_cc(iv, 1e15 * (1 + rng.random(t.cc_shape)))
    t.put_cc(4, np.zeros(t.cc_shape))
    for iv in (1, 5):
        t.gc_tree(iv)
    td = {"rows_cols": TD, "x_min": 0.0, "inv_fac": (NP - 1) / 1000.0}
    chem = {"rows_cols": CHEM, "x_min": 0.0, "inv_fac": (NP - 1) / 1000.0}
    f = Fluid(t, [1, 2, 3], [-1, 1, -1], 1, 4, 1, 2, 2.414e25, td, chem, [])
    inside = (lsf[:, 1:-1, 1:-1, 1:-1] < 0).reshape(nb, -1).any(axis=1)
    ids = np.nonzero(inside)[0] + 1
    return t, f, ids


def restated(before, lsf, ids, neumann):
    """src/streamer.f90:586-633 on the arrays before the call."""
    out = {k: v.copy() for k, v in before.items()}
    for b in ids:
        q = b - 1
        ls = lsf[q]
        inner = (slice(1, -1),) * 3
        m = ls[inner] < 0
        for k in out:
            out[k][q][inner][m] = 0.0
        if not neumann:
            continue
        sh = [(0, 0, -1), (0, 0, 1), (0, -1, 0), (0, 1, 0), (-1, 0, 0), (1, 0, 0)]
        s = np.zeros_like(ls[inner])
        cnt = np.zeros(ls[inner].shape, int)
        ne = before["e"][q]
        for dk, dj, di in sh:
            sl = (slice(1 + dk, ls.shape[0] - 1 + dk), slice(1 + dj, ls.shape[1] - 1 + dj),
                  slice(1 + di, ls.shape[2] - 1 + di))
            g = ls[sl] > 0
            s = s + np.where(g, ne[sl], 0.0)
            cnt += g
        upd = m & (cnt > 0)
        v = np.where(upd, s / np.maximum(cnt, 1), 0.0)
        out["e"][q][inner][upd] = v[upd]
        out["M+"][q][inner][upd] = v[upd]
    return out


def run(lib, device, neumann):
    t, f, ids = make_case(lib, device)
    before = {"e": t.get_cc(1), "M+": t.get_cc(2), "M-": t.get_cc(3)}
    lsf = t.get_cc(5)
    f.electrode_species_bc(5, 2, ids, neumann)
    got = {"e": t.get_cc(1), "M+": t.get_cc(2), "M-": t.get_cc(3)}
    t.sync()
    return before, lsf, ids, got


@pytest.mark.parametrize("neumann", [True, False])
def test_oracle_electrode_bc(neumann):
    before, lsf, ids, got = run(capi.oracle_library(), -1, neumann)
    assert len(ids) > 0
    want = restated(before, lsf, ids, neumann)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    # the boundary layer really was averaged (not just zeroed)
    if neumann:
        inner = (slice(None),) + (slice(1, -1),) * 3
        m = (lsf[inner] < 0) & (got["e"][inner] > 0)
        assert m.sum() > 0


def test_bad_arguments_rejected():
    t, f, ids = make_case(capi.oracle_library(), -1)
    with pytest.raises(capi.AfhError):
        f.electrode_species_bc(9, 2, ids)
    with pytest.raises(capi.AfhError):
        f.electrode_species_bc(5, 2, [t.n_boxes + 1])


@pytest.mark.gpu
@pytest.mark.parametrize("neumann", [True, False])
def test_hip_electrode_bc_equals_oracle(neumann):
    _, _, _, gh = run(capi.hip_library(), 0, neumann)
    _, _, _, go = run(capi.oracle_library(), -1, neumann)
    for k in gh:
        assert np.array_equal(gh[k], go[k]), k
