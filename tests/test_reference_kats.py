"""Known-answer tests the reference itself ships (afivo/tests, answers in
afivo/tests/answers/*_3d), restated on this library.

test_ghostcell (afivo/tests/test_ghostcell.f90, answer "Success"): a
tree of one 8^3-cell box (8 m cube, Neumann-zero boundaries)
refined four times around the box with ix = 1 at every level; with a zero
interior, af_gc_tree must give zero in every face ghost cell -- across
refinement boundaries (af_gc_interp) and physical boundaries alike."""
import numpy as np
import pytest

from afh import capi
from afh.model import Tree
from afh.tree import build_tree


def _ghostcell_tree(lib):
    # af_adjust_refinement x 4 with cell_flags = do_ref on boxes with ix == 1
    topo = build_tree(8, (8, 8, 8), (8.0, 8.0, 8.0), 1,
                      refine=lambda lvl, r0, r1: (lvl <= 4 and np.all(r0 == 0.0)))
    t = Tree(lib, topo, 1, 0)
    t.set_cc_methods(1, [(capi.BC_NEUMANN, 0.0)] * 6, capi.RB_GC_INTERP)
    return topo, t


def _check(lib):
    topo, t = _ghostcell_tree(lib)
    assert int(topo["highest_lvl"]) == 5
    rng = np.random.default_rng(3)
    # ghost cells start non-zero; the interior is zero (init in the test)
    cc = rng.standard_normal(t.cc_shape)
    cc[:, 1:-1, 1:-1, 1:-1] = 0.0
    t.put_cc(1, cc)
    t.gc_tree(1)
    out = t.get_cc(1)
    ids = np.concatenate([np.asarray(topo["lvl_ids_%d" % l]) for l in
                          range(1, int(topo["highest_lvl"]) + 1)]) - 1
    a = out[ids]
    faces = [a[:, 1:-1, 1:-1, 0], a[:, 1:-1, 1:-1, -1], a[:, 1:-1, 0, 1:-1],
             a[:, 1:-1, -1, 1:-1], a[:, 0, 1:-1, 1:-1], a[:, -1, 1:-1, 1:-1]]
    for f in faces:
        assert np.all(f == 0.0)


def test_ghostcell_kat_oracle():
    _check(capi.oracle_library())


@pytest.mark.gpu
def test_ghostcell_kat_hip():
    _check(capi.hip_library())
